"""Physics known answers on the GPU: the HIP kernel against MuJoCo's documented formulas on the
exact piano model (tests/analytic.py; the same cases as tests/test_physics_pins.py runs on the
oracle). fp32 tolerances: 1e-6 rad on trajectories of ~0.06 rad, 1e-5 at the upper-limit rest
(~0.11 rad, stiff soft limit); the friction-loss row's qacc within 2e-5 relative."""
import numpy as np
import pytest

from analytic import free_response, key_params, limit_equilibrium
from helpers import song
from test_physics_pins import END_KEYS, free_start, frictionloss_cases, state

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gpu(dp, n=2, **kw):
    task = dp.TaskConfig(**kw)
    g = dp.BatchedPianoEnv(n, song(dp, "twinkle"), task, device="cuda:0", canonical_actions=False)
    return g.model_desc, g


def test_key_free_response_on_gpu(dp):
    md, g = _gpu(dp, control_timestep=0.005)
    q0 = free_start(md)
    g.set_state(state(2, q0))
    steps = 8
    exp = {k: free_response(key_params(md, k), q0[k], 0.0, steps) for k in END_KEYS}
    zero = torch.zeros(2, 45, device="cuda:0")
    for t in range(steps):
        g.step(zero)
        q = g.get_state()["qpos"].cpu().numpy().astype(np.float64)
        for k in END_KEYS:
            assert abs(q[0, k] - exp[k][t]) < 1e-6, (k, t, q[0, k], exp[k][t])


def test_key_lower_limit_rest_on_gpu(dp):
    md, g = _gpu(dp)
    g.set_state(state(2, np.zeros(88)))
    zero = torch.zeros(2, 45, device="cuda:0")
    for _ in range(60):
        g.step(zero)
    q = g.get_state()["qpos"].cpu().numpy().astype(np.float64)
    for k in END_KEYS:
        qs = limit_equilibrium(md, key_params(md, k), side=0)
        assert abs(q[0, k] - qs) < 1e-6, (k, q[0, k], qs)


def test_key_upper_limit_rest_under_applied_force_on_gpu(dp):
    md, g = _gpu(dp)
    g.set_state(state(2, np.array([md.key_range[k][1] for k in range(88)])))
    app = torch.zeros(2, 140, device="cuda:0")
    app[:, END_KEYS] = 3.0
    g.set_applied(app)
    zero = torch.zeros(2, 45, device="cuda:0")
    for _ in range(40):
        g.step(zero)
    q = g.get_state()["qpos"].cpu().numpy().astype(np.float64)
    for k in END_KEYS:
        qs = limit_equilibrium(md, key_params(md, k), side=1, applied=3.0)
        assert abs(q[0, k] - qs) < 1e-5, (k, q[0, k], qs)


def test_frictionloss_single_row_known_answers_on_gpu(dp):
    """The friction-loss row's known answers (regularised creep and slip, at rest and moving;
    tests/test_physics_pins.py) on the kernel's Newton solve."""
    def run(task, s):
        g = dp.BatchedPianoEnv(1, song(dp, "twinkle"), task, device="cuda:0", canonical_actions=False)
        g.set_state(s)
        g.step(torch.zeros(1, 45, device="cuda:0"))
        assert int(g.contact_count()[0]) == 0
        return g.get_state()["qacc_ws"][0].cpu().numpy().astype(np.float64)

    cases = frictionloss_cases(dp, run)
    assert {r for _, _, r in cases} == {"creep", "slip"}
    for got, exp, regime in cases:
        assert abs(got - exp) <= 2e-5 * max(1.0, abs(exp)), (got, exp, regime)
