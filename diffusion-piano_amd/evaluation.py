"""Musical-performance metrics of the batched environment.

:class:`MidiEvaluationWrapper` mirrors ``robopianist/wrappers/evaluation.py:37-112`` (same
constructor, ``step`` / ``reset`` / ``get_musical_metrics`` and the deque of the last
``deque_size`` episodes). The per-step work the reference does on the host - appending
``piano.activation`` / ``sustain_activation`` every step and running sklearn's
``precision_recall_fscore_support`` over the episode at LAST (evaluation.py:114-177) -
happens inside the step kernel: each env accumulates its per-step binary precision /
recall / F1 (zero_division = 1) in HBM and publishes the episode means when it finishes
(``ps_musical_metrics``). The wrapper only reads those means after a LAST step.

Wraps a single-env :class:`~envs.Environment` (dm_env ``TimeStep`` API, the reference's
case) or a :class:`~envs.BatchedPianoEnv` / :class:`~envs.VectorizedPianoEnv`; with N envs
every env's finished episode enters the deques.
"""

from __future__ import annotations

from collections import deque
from typing import Deque, Dict, NamedTuple, Sequence

from . import abi

KEYS = ("precision", "recall", "f1", "sustain_precision", "sustain_recall", "sustain_f1")


class EpisodeMetrics(NamedTuple):
    precision: float
    recall: float
    f1: float


class MidiEvaluationWrapper:
    def __init__(self, environment, deque_size: int = 1) -> None:
        self._environment = environment
        self._deques: Dict[str, Deque[float]] = {k: deque(maxlen=deque_size) for k in KEYS}

    def _core(self):
        env = self._environment
        return env.core if hasattr(env, "core") else env

    def _collect(self, finished):
        """Append the episode metrics of the envs flagged in `finished` (device bool [N])."""
        if not bool(finished.any()):
            return
        ep, _ = self._core().musical_metrics()
        for row in ep[finished].double().cpu().numpy():
            for k, v in zip(KEYS, row):
                self._deques[k].append(float(v))

    def step(self, action):
        out = self._environment.step(action)
        core = self._core()
        if hasattr(out, "step_type"):  # single env, dm_env TimeStep
            if out.last():
                self._collect(core.step_type == abi.LAST)
        else:  # batched: (obs, rewards, dones) or (obs, reward, discount, step_type)
            self._collect(core.step_type == abi.LAST)
        return out

    def reset(self):
        return self._environment.reset()

    def get_musical_metrics(self) -> Dict[str, float]:
        """Mean precision / recall / F1 (keys and sustain) over the last ``deque_size``
        finished episodes (evaluation.py:88-105)."""
        if not self._deques["precision"]:
            raise ValueError("No episode metrics available yet.")

        def _mean(seq: Sequence[float]) -> float:
            return sum(seq) / len(seq)

        return {k: _mean(d) for k, d in self._deques.items()}

    def __getattr__(self, name):
        return getattr(self._environment, name)
