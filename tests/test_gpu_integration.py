"""The two bindings shown in INTEGRATION.md, executed verbatim from the document."""
import os
import re

import numpy as np
import pytest

from helpers import ROOT, song

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _blocks():
    text = (ROOT / "INTEGRATION.md").read_text()
    return re.findall(r"```python\n(.*?)```", text, re.S)


def test_dropin_class_snippet(dp):
    ns = {}
    exec(_blocks()[0], ns)
    env = ns["VectorizedPianoEnv"](4, song(dp, "guren"))
    obs = env.reset()
    assert list(obs) == ["goal", "fingering", "piano/state", "piano/sustain_state",
                         "rh_shadow_hand/joints_pos", "lh_shadow_hand/joints_pos"]
    spec = env.envs[0].observation_spec()
    assert sum(int(np.prod(s.shape)) for s in spec.values()) == 329
    obs, rewards, dones = env.step(np.random.uniform(-1, 1, (4, 45)))
    assert isinstance(rewards, np.ndarray) and rewards.dtype == np.float64 and dones.dtype == bool


def test_raw_ctypes_snippet(dp):
    cwd = os.getcwd()
    os.chdir(ROOT)
    try:
        ns = {}
        exec(_blocks()[1], ns)
        assert torch.isfinite(ns["obs"]).all() and torch.isfinite(ns["rew"]).all()
        assert (ns["stype"] == 1).all()
    finally:
        os.chdir(cwd)


def test_ppo_snippets(dp):
    ns = {}
    exec(_blocks()[2], ns)
    assert ns["PPOAgent"].__module__.endswith(".ppo")
    ns = {}
    exec(_blocks()[3], ns)
    log = ns["agent"].last_update_log
    assert log is not None and torch.isfinite(log).all()
    env, ev = ns["env"], ns["evaluator"]
    act = torch.zeros(256, 45, device="cuda:0")
    for _ in range(161):
        ev.step(act)
    m = ev.get_musical_metrics()
    assert 0.0 <= m["f1"] <= 1.0
