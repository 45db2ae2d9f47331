"""The step kernel's two register budgets (pianosim_kernel<XG, WPE>): launches of at most one env
per SIMD take the one-wave instantiation (256 VGPRs + ~143 AGPRs; scratch 0 B per lane for the
capsule kernel, ~460 B for the box/hull one), larger ones the two-wave instantiation (256 VGPRs,
scratch ~660 / ~1220 B per lane; round 6, fp64 MPR; tools/resource_usage.sh) - csrc/pianosim.hip
launch(). Both
compile the same source, so
every output must be bitwise equal; PIANOSIM_ONE_WAVE_MAX (read by ps_create) moves the
threshold so one small batch runs through each."""
import numpy as np
import pytest

from helpers import song

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _rollout(dp, task, n, steps, one_wave_max, monkeypatch):
    monkeypatch.setenv("PIANOSIM_ONE_WAVE_MAX", str(one_wave_max))
    g = dp.BatchedPianoEnv(n, song(dp, "crossing_field"), task, device="cuda:0")
    obs0 = g.reset().cpu().numpy()
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    outs = [obs0]
    for _ in range(steps):
        o, r, d, s = g.step(torch.rand(n, g.action_dim, device="cuda:0", generator=gen) * 2 - 1)
        outs += [o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(), s.cpu().numpy()]
    st = {k: v.cpu().numpy() for k, v in g.get_state().items()}
    stats = g.solver_stats().cpu().numpy()
    g.close()
    return outs, st, stats


@pytest.mark.parametrize("hand", [None, False], ids=["capsule", "box_hull"])
def test_one_wave_and_two_wave_instantiations_are_bitwise_equal(dp, hand, monkeypatch):
    task = dp.TaskConfig(trim_silence=True, primitive_fingertip_collisions=hand)
    n, steps = 64, 6
    a_outs, a_st, a_stats = _rollout(dp, task, n, steps, 1 << 30, monkeypatch)  # one-wave
    b_outs, b_st, b_stats = _rollout(dp, task, n, steps, 0, monkeypatch)        # two-wave
    for x, y in zip(a_outs, b_outs):
        np.testing.assert_array_equal(x, y)
    for k in a_st:
        np.testing.assert_array_equal(a_st[k], b_st[k], err_msg=k)
    np.testing.assert_array_equal(a_stats, b_stats)
    assert a_stats[:, 3].max() > 0, "no constraint rows: the solve was not exercised"
