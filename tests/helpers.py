"""Shared test helpers: songs for the benchmark configs and random states."""
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
DATA = ROOT / "tests" / "data"


def song(dp, name):
    m = dp.music
    if name == "twinkle":
        return m.twinkle_twinkle_little_star_one_hand()
    if name == "crossing_field":
        return m.parse_midi(DATA / "Crossing Field Cut 10s.mid")
    if name == "guren":
        return m.add_fingering_from_annotation_file(DATA / "Guren no Yumiya Cut 14s.mid",
                                                    DATA / "Guren no Yumiya Cut 14s_fingering v3.txt")
    if name == "test_task":
        return m.test_midi(0.01)
    raise KeyError(name)


def tool_hand_kwargs():
    """TaskConfig kwargs of the collider set a development tool runs (PIANOSIM_HAND = hull |
    primitive | authored, bench.py --hand; PIANOSIM_HULL=1 = hull; default the all-capsule hand)
    and its Newton refinement (PIANOSIM_REFINE = TaskConfig.solver_refine, default 0)."""
    import os
    h = os.environ.get("PIANOSIM_HAND") or ("hull" if os.environ.get("PIANOSIM_HULL") else "authored")
    kw = {"hull": {"primitive_fingertip_collisions": False}, "primitive": {"primitive_fingertip_collisions": True},
          "authored": {}}[h]
    return dict(kw, solver_refine=int(os.environ.get("PIANOSIM_REFINE", "0")))


def random_states(md, n, rng, vscale=0.5):
    """Random joint configurations inside the ranges (keys slightly beyond, to hit limits)."""
    q = np.zeros((n, 140))
    for k in range(88):
        q[:, k] = rng.uniform(-0.005, md.key_range[k][1] + 0.005, n)
    for h in range(2):
        for j in range(26):
            lo, hi = md.dof_range[h][j]
            q[:, 88 + 26 * h + j] = rng.uniform(lo - 0.02, hi + 0.02, n)
    v = rng.normal(0, vscale, (n, 140))
    v[:, :88] *= 0.2
    return q, v


def capsule_points(radius, halflen, n_ring=8, n_lat=2):
    """Points on a capsule surface along z (mjcf.capsule_points)."""
    import importlib
    return importlib.import_module("diffusion-piano_amd").mjcf.capsule_points(radius, halflen, n_ring, n_lat)


def box_hull_hand(dp):
    """The authored right hand with box and convex-hull colliders (mjcf.box_hull_hand)."""
    return dp.mjcf.box_hull_hand()


_DEFAULT_LIMITS = None


def hand_limits(md=None):
    """(lo, hi, limited, locked) [52] of the hand dofs (rh 26, lh 26) of ``md`` (default: the
    authored hand, whose joint ranges every collider set shares)."""
    global _DEFAULT_LIMITS
    if md is None:
        if _DEFAULT_LIMITS is None:
            import importlib
            _DEFAULT_LIMITS = hand_limits(importlib.import_module("diffusion-piano_amd").model.build_model())
        return _DEFAULT_LIMITS
    rng_ = np.array(md.dof_range, np.float64).reshape(52, 2)
    return (rng_[:, 0], rng_[:, 1], np.array(md.dof_limited, bool).reshape(52),
            np.array(md.dof_locked, bool).reshape(52))


def perturb_joints(q, rng, scale=1e-7, md=None):
    """Hand joints [n, 52] moved by N(0, scale) each WITHOUT changing any joint limit's
    activity: a step that would cross a limit (or leave one: a joint resting exactly ON its
    limit - 22 of the 52 at qpos0 - has an inactive row that any move below the limit would
    activate) is taken in the other direction; locked dofs stay. So the perturbation probes the
    state's sensitivity, not the discontinuity of a limit row switching on."""
    lo, hi, lim, locked = hand_limits(md)
    q = np.array(q, np.float64)
    d = rng.normal(0.0, scale, q.shape)
    d[:, locked] = 0.0

    def zones(x):
        return np.where(lim, (x < lo).astype(int) - (x > hi).astype(int), 0)

    z0 = zones(q)
    flip = zones(q + d) != z0
    d[flip] = -d[flip]
    still = zones(q + d) != z0  # (a range narrower than the step: no move)
    d[still] = 0.0
    return q + d


def perturbed(state, rng, scale=1e-7, md=None):
    """The state with every hand joint moved by N(0, scale) rad, keeping each joint on its side
    of its limits (``perturb_joints``): the checker stepped from it measures the model's own fp64
    sensitivity at that state (parity floor)."""
    s = dict(state)
    q = np.array(state["qpos"], np.float64)
    q[:, 88:] = perturb_joints(q[:, 88:], rng, scale, md)
    s["qpos"] = q
    return s


# absolute ceilings of the all-sample clause (a gate relative to the checker's own
# sensitivity alone is unbounded where that sensitivity is large)
PARITY_P99_CEIL = 2e-4
PARITY_MAX_CEIL = 3e-2


def assert_parity(e, floor, what="", tol=1e-4, well=1e-5, p99_ceil=PARITY_P99_CEIL, max_ceil=PARITY_MAX_CEIL):
    """The parity gate of a teacher-forced comparison (fp32 kernel vs fp64 checker, one control
    step from the same state), per env-step qpos L-inf error `e` and the checker's own
    sensitivity `floor` (the same step from the state moved by ``perturbed``):
      * median < 1e-5;
      * p99 < tol over the well-conditioned env-steps (floor < well; at least half of them);
      * p99 over all env-steps within max(tol, 2x the floor's p99) - the ill-conditioned ones (a
        contact starting or ending at near-zero distance, a stick-slip flip) move the checker
        itself by more than tol under a 1e-7 rad perturbation - and never above the absolute
        ceiling p99_ceil; the largest error at most max_ceil.
    Returns the summary (with the floor's p99, so a loosened gate shows in the logs)."""
    e, floor = np.asarray(e, np.float64), np.asarray(floor, np.float64)
    calm = floor < well
    msg = (f"{what}: n {e.size}, median {np.median(e):.2e}, p99 {np.percentile(e, 99):.2e}, max {e.max():.2e}; "
           f"well-conditioned {int(calm.sum())}: p99 {np.percentile(e[calm], 99) if calm.any() else float('nan'):.2e}; "
           f"floor p99 {np.percentile(floor, 99):.2e}")
    print(msg)
    assert np.median(e) < 1e-5, msg
    assert calm.sum() >= 0.5 * e.size, msg
    assert np.percentile(e[calm], 99) < tol, msg
    assert np.percentile(e, 99) <= min(max(tol, 2.0 * np.percentile(floor, 99)), p99_ceil), msg
    assert e.max() <= max_ceil, msg
    return msg


def assert_flip_rates(e, floor, what="", ts=(1e-3, 1e-2), p99_cap=5e-2, slack=0.01, median=1e-5, tol=1e-4,
                      well=1e-5):
    """The whole-step gate of the box / hull hand, whose MPR contact normals are piecewise
    constant over the hulls' faces (a portal near a face edge switches faces under any tiny
    change of its input, in the fp64 checker too): median below `median`; p99 below `tol` over
    the well-conditioned env-steps (the checker's own move under the perturbation, `floor`, below
    `well`; at least half of them) - the clause of ``assert_parity``, so a systematic error
    confined to the steps the checker resolves cannot hide in the tail; for each threshold t the
    fraction of env-steps the GPU moves by more than t at most 2x the fraction the checker moves
    itself under a 1e-7 rad perturbation + `slack` (the tail is made of such switches: its rate,
    not a single-sample p99, is what the two runs share); p99 below `p99_cap`."""
    e, floor = np.asarray(e, np.float64), np.asarray(floor, np.float64)
    rates = {t: (float(np.mean(e > t)), float(np.mean(floor > t))) for t in ts}
    calm = floor < well
    msg = (f"{what}: n {e.size}, median {np.median(e):.2e}, p99 {np.percentile(e, 99):.2e}, max {e.max():.2e}; "
           f"well-conditioned {int(calm.sum())}: p99 {np.percentile(e[calm], 99) if calm.any() else float('nan'):.2e}; "
           f"floor median {np.median(floor):.2e} p99 {np.percentile(floor, 99):.2e}; flip rates (gpu, floor) " +
           ", ".join(f">{t:.0e}: {a:.3f} {b:.3f}" for t, (a, b) in rates.items()))
    print(msg)
    assert np.median(e) < median, msg
    assert calm.sum() >= 0.5 * e.size, msg
    assert np.percentile(e[calm], 99) < tol, msg
    for t, (a, b) in rates.items():
        assert a <= 2.0 * b + slack, msg
    assert np.percentile(e, 99) <= p99_cap, msg
    return msg
