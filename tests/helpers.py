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
    """Points on a capsule surface along z (a rounded fingertip shape for hull colliders)."""
    pts = []
    for z0, sgn in ((halflen, 1.0), (-halflen, -1.0)):
        pts.append((0.0, 0.0, z0 + sgn * radius))
        for j in range(n_lat + 1):
            phi = (j / (n_lat + 1)) * np.pi / 2  # 0 at the equator
            for i in range(n_ring):
                t = 2 * np.pi * (i + 0.5 * (j % 2)) / n_ring
                pts.append((radius * np.cos(phi) * np.cos(t), radius * np.cos(phi) * np.sin(t),
                            z0 + sgn * radius * np.sin(phi)))
    return np.asarray(pts)


def box_hull_hand(dp):
    """The authored right hand with box and convex-hull colliders: the two palm capsules and the
    little-finger metacarpal capsule become boxes, every distal capsule a 58-point capsule-shaped
    hull (as the Menagerie hand's palm boxes and distal meshes)."""
    M = dp.model
    mj = dp.mjcf
    hand = M.authored_hand()
    geoms, xgeoms = [], []
    names = [b.name for b in hand.bodies]
    for g in hand.geoms:
        bname = names[g.body]
        if bname == "palm" or bname == "lfmetacarpal":
            q = mj._quat_from_z(g.axis)
            xgeoms.append(M.XGeom(g.body, "box", tuple(g.pos), tuple(q), (g.radius, g.radius * 0.8, g.halflen + g.radius)))
        elif bname.endswith("distal"):
            c, v = mj.convex_hull_collider(capsule_points(g.radius, g.halflen))
            R = M.quat_to_mat(mj._quat_from_z(g.axis))
            pos = np.asarray(g.pos) + R @ c
            xgeoms.append(M.XGeom(g.body, "hull", tuple(pos), tuple(mj._quat_from_z(g.axis)), verts=v))
        else:
            geoms.append(g)
    return hand._replace(geoms=geoms, xgeoms=xgeoms)
