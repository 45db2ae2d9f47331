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
