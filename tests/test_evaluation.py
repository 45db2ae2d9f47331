"""MidiEvaluationWrapper metrics (robopianist/wrappers/evaluation.py:114-177) in the CPU
restatement, pinned by sklearn's precision_recall_fscore_support (the reference's own
dependency; tests/golden/prf.json from tests/golden/make_eval_golden.py) and by closed
forms over whole episodes."""
import json
from pathlib import Path

import numpy as np
import pytest

from helpers import song

ROOT = Path(__file__).resolve().parents[1]


def closed_form(goal, active_keys, sustain_pred):
    """Episode means when the predicted key set / sustain flag is the same every step."""
    rows = []
    for g in goal:
        yt = g[:88] != 0
        ya = np.asarray(active_keys, bool)
        tp, fp, fn = int((yt & ya).sum()), int((~yt & ya).sum()), int((yt & ~ya).sum())
        st, sp = bool(g[88] != 0), bool(sustain_pred)
        stp, sfp, sfn = int(st and sp), int(not st and sp), int(st and not sp)
        f = lambda t, p, n: [t / (t + p) if t + p else 1.0, t / (t + n) if t + n else 1.0,
                             2 * t / (2 * t + p + n) if 2 * t + p + n else 1.0]
        rows.append(f(tp, fp, fn) + f(stp, sfp, sfn))
    return np.mean(rows, axis=0)


def test_prf_matches_sklearn(ref):
    g = json.loads((ROOT / "tests" / "golden" / "prf.json").read_text())
    assert len(g["cases"]) > 40
    for c in g["cases"]:
        np.testing.assert_allclose(ref.prf(c["y_true"], c["y_pred"]), c["prf"], rtol=0, atol=1e-15)


@pytest.mark.parametrize("pattern", ["zero", "all_keys"])
def test_episode_metrics_closed_form(dp, ref, pattern):
    """Twinkle, one full episode (T = 161). zero: no key ever pressed, no sustain;
    all_keys: qfrc_applied = 3 on every key (piano_with_shadow_hands_test.py:228-242 holds
    them down from the first step) and the sustain pedal down (action[44] = 1)."""
    task = dp.TaskConfig()
    md, st, tc = dp.compile_task(song(dp, "twinkle"), task, canonical_actions=False)
    env = ref.OracleEnv(md, st, tc, 2)
    env.reset()
    a = np.zeros((2, 45), np.float32)
    if pattern == "all_keys":
        app = np.zeros((2, 140))
        app[:, :88] = 3.0
        env.set_applied(app)
        a[:, 44] = 1.0
    for t in range(st.T):
        _, _, _, stype = env.step(a)
    assert (stype == 2).all()
    ep, cnt = env.musical_metrics()
    assert (cnt == 1).all()
    want = closed_form(st.goal, np.full(88, pattern == "all_keys"), pattern == "all_keys")
    np.testing.assert_allclose(ep, np.repeat(want[None], 2, 0), rtol=0, atol=1e-12)
    # the next step auto-resets: the finished episode's metrics stay until the next LAST
    env.step(a)
    ep2, cnt2 = env.musical_metrics()
    assert (cnt2 == 1).all() and np.array_equal(ep, ep2)
