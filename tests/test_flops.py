"""The FLOP-counting build of the oracle (oracle/flops.cpp, tools/count_flops.py ->
profiles/flops.json -> bench.py's valu_roofline): it must compute exactly what the oracle
computes, count deterministically, and the committed profile must cover the bench configs."""
import json
from pathlib import Path

import numpy as np

from helpers import song

ROOT = Path(__file__).resolve().parents[1]


def _rollout(dp, ref, counting, n=4, steps=6):
    md, st, tc = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(), canonical_actions=False)
    env = ref.OracleEnv(md, st, tc, n, counting=counting)
    env.reset()
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(7)
    if counting:
        ref.flops_reset()
    outs = [env.step(rng.uniform(lo, hi, (n, 45)).astype(np.float32)) for _ in range(steps)]
    return outs, env.get_state(), (ref.flops_get() if counting else None)


def test_counting_build_is_bitwise_the_oracle(dp, ref):
    a_out, a_st, _ = _rollout(dp, ref, False)
    b_out, b_st, cnt = _rollout(dp, ref, True)
    for x, y in zip(a_out, b_out):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(u, v)
    for k in a_st:
        np.testing.assert_array_equal(a_st[k], b_st[k])
    assert cnt.sum() > 0


def test_count_is_deterministic_and_plausible(dp, ref):
    c1 = _rollout(dp, ref, True)[2]
    c2 = _rollout(dp, ref, True)[2]
    np.testing.assert_array_equal(c1, c2)
    per = c1.sum() / (4 * 6)
    assert 2e5 < per < 5e6, per   # 10 substeps of a 140-dof contact step


def test_committed_profile_covers_bench_configs():
    d = json.loads((ROOT / "profiles" / "flops.json").read_text())
    for name in ("crossing_field", "twinkle"):
        c = d["configs"][name]
        parts = c["add_sub"] + c["mul"] + c["div"] + c["sqrt_transc_minmax"]
        assert abs(parts - c["flops_per_env_step"]) < 1e-6 * parts
        assert 2e5 < c["flops_per_env_step"] < 5e6
