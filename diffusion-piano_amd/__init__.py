"""MI355X-native batched PianoWithShadowHands environment.

Import with ``importlib.import_module("diffusion-piano_amd")`` (the directory name is the
package name required by the build layout).
"""

from . import abi, music, model, mjcf, evaluation  # noqa: F401
from .envs import (  # noqa: F401
    Array, BatchedPianoEnv, BoundedArray, DEBUG, Environment, PhysicsError, StepType, TaskConfig, TimeStep,
    VectorizedPianoEnv, compile_task, load, obs_layout,
)
from .evaluation import MidiEvaluationWrapper  # noqa: F401,E402
from ._lib import PianosimError  # noqa: F401,E402
