"""GPU parity of the in-kernel MidiEvaluationWrapper metrics (ps_musical_metrics) with the
CPU restatement over whole Twinkle episodes, and the wrapper's reference API.

Key presses are driven by qfrc_applied on chosen key subsets (deterministic key dynamics,
no hand contact), sustain by action[44]; per env a different subset. The metrics are
per-step ratios of small integer counts averaged over 161 steps: tolerance 1e-6."""
import importlib

import numpy as np
import pytest

from helpers import song
from test_evaluation import closed_form

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
N = 8


def test_musical_metrics_match_restatement(dp, ref):
    task = dp.TaskConfig()
    seq = song(dp, "twinkle")
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", canonical_actions=False)
    o = ref.OracleEnv(md, st, tc, N)
    rng = np.random.RandomState(0)
    app = np.zeros((N, 140))
    goal_keys = np.flatnonzero(st.goal[:, :88].any(0))
    for i in range(N):  # env 0: nothing; 1: all keys; others: mixes of song keys and others
        if i == 1:
            app[i, :88] = 3.0
        elif i > 1:
            keys = rng.choice(goal_keys, size=min(len(goal_keys), i), replace=False)
            app[i, keys] = 3.0
            app[i, rng.choice(88, size=i - 1, replace=False)] = 3.0
    a = np.zeros((N, 45), np.float32)
    a[::2, 44] = 1.0  # sustain pedal down in even envs
    g.reset(); o.reset()
    g.set_applied(app); o.set_applied(app)
    at = torch.from_numpy(a).cuda()
    for t in range(st.T + 1):
        g.step(at)
        o.step(a)
        if t == st.T - 1:
            ep_g, cnt_g = (x.cpu().numpy() for x in g.musical_metrics())
            ep_o, cnt_o = o.musical_metrics()
            assert (cnt_g == 1).all() and (cnt_o == 1).all()
            np.testing.assert_allclose(ep_g, ep_o, rtol=0, atol=1e-6)
            np.testing.assert_allclose(ep_g[0], closed_form(st.goal, np.zeros(88, bool), True), atol=1e-6)
            np.testing.assert_allclose(ep_g[1], closed_form(st.goal, np.ones(88, bool), False), atol=1e-6)
    ep_g2, cnt_g2 = (x.cpu().numpy() for x in g.musical_metrics())  # after the auto-reset step
    assert (cnt_g2 == 1).all() and np.array_equal(ep_g, ep_g2)
    g.close()


def test_wrapper_reference_api(dp):
    ev = importlib.import_module("diffusion-piano_amd.evaluation")
    env = ev.MidiEvaluationWrapper(dp.load("RoboPianist-debug-TwinkleTwinkleLittleStar-v0"), deque_size=2)
    with pytest.raises(ValueError):
        env.get_musical_metrics()
    ts = env.reset()
    assert ts.first()
    a = np.zeros(45, np.float32)
    a[:] = -1.0  # canonical: every actuator at its lower bound, sustain 0
    n = 0
    while not ts.last():
        ts = env.step(a)
        n += 1
    m = env.get_musical_metrics()
    assert set(m) == {"precision", "recall", "f1", "sustain_precision", "sustain_recall", "sustain_f1"}
    assert n == 161 and all(0.0 <= v <= 1.0 for v in m.values())
    assert m["sustain_precision"] == pytest.approx(1.0) and m["sustain_f1"] == pytest.approx(1.0)
    # a batched env: every env's finished episode enters the deque
    venv = ev.MidiEvaluationWrapper(dp.VectorizedPianoEnv(4, song(dp, "twinkle"), trim_silence=False), deque_size=8)
    venv.reset()
    act = torch.full((4, 45), -1.0, device="cuda:0")
    for _ in range(161):
        venv.step(act)
    m2 = venv.get_musical_metrics()
    assert len(venv._deques["f1"]) == 4 and m2["sustain_f1"] == pytest.approx(1.0)
