"""Box and convex-hull hand colliders on the CPU checker.

The reference's default hand collides Menagerie's distal meshes (convex hulls) and palm boxes
(shadow_hand.py:95,144-152). MuJoCo collides a mesh pair with libccd's MPR (mjc_Convex, one
contact) and boxes with a box-box routine; the checker restates MPR and a separating-axis +
face-clipping box-box (oracle/pianosim_ref.c). Known answers below are closed-form
geometry; the MPR property tests compare against an independent numpy SAT (exact for
polytopes). MuJoCo itself is absent, so agreement with mjc_Convex's numbers is unpinned.
"""
import math
import struct

import numpy as np
import pytest

from helpers import box_hull_hand, capsule_points, song

CUBE = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], float)


def rot(axis, t):
    a = np.asarray(axis, float)
    a /= np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(t) * K + (1 - math.cos(t)) * K @ K


def sat_depth(ca, Ra, ha, cb, Rb, hb):
    """Exact penetration depth of two boxes (min overlap over the 15 SAT axes; < 0: apart)."""
    axes = [Ra[:, i] for i in range(3)] + [Rb[:, i] for i in range(3)]
    for i in range(3):
        for j in range(3):
            c = np.cross(Ra[:, i], Rb[:, j])
            if np.linalg.norm(c) > 1e-9:
                axes.append(c / np.linalg.norm(c))
    t = np.asarray(cb, float) - np.asarray(ca, float)
    best = np.inf
    for L in axes:
        ra = sum(ha[i] * abs(Ra[:, i] @ L) for i in range(3))
        rb = sum(hb[i] * abs(Rb[:, i] @ L) for i in range(3))
        best = min(best, ra + rb - abs(t @ L))
    return best


def test_box_box_face_contact_known_answer(ref):
    A = ref.shape("box", c=(0, 0, 0), hs=(1, 1, 1))
    B = ref.shape("box", c=(0.2, 0.1, 1.4), hs=(0.5, 0.5, 0.5))  # 0.1 into A's top face
    cons = ref.narrow(A, B)
    assert len(cons) == 4
    corners = sorted((round(p[0], 12), round(p[1], 12)) for p, _, _ in cons)
    assert corners == sorted([(-0.3, -0.4), (-0.3, 0.6), (0.7, -0.4), (0.7, 0.6)])
    for p, n, d in cons:
        np.testing.assert_allclose(n, [0, 0, 1], atol=1e-15)  # geom1 -> geom2
        assert abs(d + 0.1) < 1e-12 and abs(p[2] - 0.95) < 1e-12  # midway between the faces
    # roles swapped: the normal flips, the points stay
    cons2 = ref.narrow(B, A)
    assert len(cons2) == 4 and all(np.allclose(n, [0, 0, -1]) for _, n, _ in cons2)


def test_box_box_clipped_face(ref):
    A = ref.shape("box", c=(0, 0, 0), hs=(1, 1, 1))
    B = ref.shape("box", c=(0.9, 0.1, 1.45), hs=(0.5, 0.5, 0.5))  # overhangs A's x = 1 edge
    cons = ref.narrow(A, B)
    xs = sorted(set(round(p[0], 12) for p, _, _ in cons))
    assert xs == [0.4, 1.0] and len(cons) == 4
    assert all(abs(d + 0.05) < 1e-12 for _, _, d in cons)


def test_box_box_vertex_and_edge_edge(ref):
    h = 0.5
    A = ref.shape("box", c=(0, 0, 0), hs=(1, 1, 1))
    R = rot((1, 0, 0), math.pi / 4) @ rot((0, 0, 1), math.pi / 4)
    ext = h * np.abs(R[2]).sum()  # B's half extent along z
    B = ref.shape("box", c=(0, 0, 1 + ext - 0.03), R=R, hs=(h, h, h))
    (p, n, d), = ref.narrow(A, B)  # one vertex below A's top face
    assert abs(d + 0.03) < 1e-12 and np.allclose(n, [0, 0, 1])
    # edge-edge: A's top edge along y (A turned 45 deg about y), B's bottom edge along x (B
    # turned 45 deg about x): the separating axis is their cross product z
    Ra, Rb = rot((0, 1, 0), math.pi / 4), rot((1, 0, 0), math.pi / 4)
    dz = 2 * h * math.sqrt(2) - 0.02
    A2 = ref.shape("box", c=(0, 0, 0), R=Ra, hs=(h, h, h))
    B2 = ref.shape("box", c=(0.1, -0.05, dz), R=Rb, hs=(h, h, h))
    (p, n, d), = ref.narrow(A2, B2)
    assert abs(d + 0.02) < 1e-12 and np.allclose(n, [0, 0, 1], atol=1e-12)
    # midpoint of the closest points: A's edge at x = 0, B's edge at y = -0.05
    np.testing.assert_allclose(p, [0.0, -0.05, h * math.sqrt(2) - 0.01], atol=1e-12)


def test_mpr_known_answers(ref):
    Ah = ref.shape("hull", c=(0, 0, 0), verts=CUBE)
    Bh = ref.shape("hull", c=(0.2, 0.1, 1.4), verts=CUBE * 0.5)
    (p, n, d), = ref.narrow(Ah, Bh)
    assert abs(d + 0.1) < 1e-9 and np.allclose(n, [0, 0, 1], atol=1e-9)
    assert -1 <= p[0] <= 1 and -1 <= p[1] <= 1 and 0.9 <= p[2] <= 1.0  # inside the overlap slab
    A = ref.shape("box", c=(0, 0, 0), hs=(1, 1, 1))
    R = rot((1, 0, 0), math.pi / 4) @ rot((0, 0, 1), math.pi / 4)
    ext = 0.5 * np.abs(R[2]).sum()
    Bv = ref.shape("hull", c=(0, 0, 1 + ext - 0.03), R=R, verts=CUBE * 0.5)
    (p, n, d), = ref.narrow(A, Bv)
    assert abs(d + 0.03) < 1e-9 and np.allclose(n, [0, 0, 1], atol=1e-9)
    # capsule above a hull cube: depth of the end sphere, normal capsule -> cube
    C = ref.shape("capsule", p0=(0.1, 0.2, 1.05), p1=(0.1, 0.2, 1.5), r=0.1)
    (p, n, d), = ref.narrow(C, Ah)
    assert abs(d + 0.05) < 1e-6 and np.allclose(n, [0, 0, -1], atol=1e-6)  # curved: MPR tolerance
    # apart: no contact
    assert ref.narrow(Ah, ref.shape("hull", c=(0, 0, 2.6), verts=CUBE * 0.5)) == []


def test_mpr_agrees_with_sat_on_random_boxes(ref):
    """Boxes given as 8-vertex hulls: MPR reports a contact iff the shapes overlap (SAT), and
    its depth (the portal plane's distance) is never below the exact penetration."""
    rng = np.random.RandomState(3)
    hits = 0
    for _ in range(400):
        ha, hb = rng.uniform(0.2, 1.0, 3), rng.uniform(0.2, 1.0, 3)
        Ra, Rb = rot(rng.normal(size=3), rng.uniform(0, np.pi)), rot(rng.normal(size=3), rng.uniform(0, np.pi))
        cb = rng.normal(size=3) * 1.2
        exact = sat_depth(np.zeros(3), Ra, ha, cb, Rb, hb)
        if abs(exact) < 1e-6:
            continue
        cons = ref.narrow(ref.shape("hull", c=(0, 0, 0), R=Ra, verts=CUBE * ha),
                          ref.shape("hull", c=cb, R=Rb, verts=CUBE * hb))
        assert (len(cons) == 1) == (exact > 0), (exact, cons)
        if cons:
            hits += 1
            assert -cons[0][2] >= exact - 1e-6, (-cons[0][2], exact)
        # the box-box collider finds the same overlap; its points are no deeper than the chosen
        # axis' overlap, which a face axis keeps up to 1.05 x an edge axis' (the face preference)
        bb = ref.narrow(ref.shape("box", c=(0, 0, 0), R=Ra, hs=ha), ref.shape("box", c=cb, R=Rb, hs=hb))
        assert (len(bb) > 0) == (exact > 0)
        if bb:
            assert max(-d for _, _, d in bb) <= 1.05 * exact + 1e-9
    assert hits > 100


def test_capsule_vs_oriented_box(ref):
    R = rot((0, 0, 1), 0.3)
    B = ref.shape("box", c=(0.5, 0.2, 0.0), R=R, hs=(0.3, 0.2, 0.1))
    C = ref.shape("capsule", p0=(0.5, 0.2, 0.12), p1=(0.5, 0.2, 0.6), r=0.05)
    (p, n, d), = ref.narrow(C, B)  # the box is geom1: normal box -> capsule
    assert abs(d + 0.03) < 1e-12 and np.allclose(n, [0, 0, 1], atol=1e-12)


# ------------------------------------------------------------------ model and loader
def test_box_hull_hand_model(dp):
    M, abi = dp.model, dp.abi
    hand = box_hull_hand(dp)
    md = M.build_model(hand=hand)
    assert [md.xgeom_type[0][i] for i in range(8)] == [1, 1, 2, 2, 2, 1, 2, 2]
    for i, xg in enumerate(hand.xgeoms):
        for h, sgn in ((0, 1.0), (1, -1.0)):  # the left hand mirrors x
            assert md.xgeom_body[h][i] == xg.body
            assert md.xgeom_pos[h][i][0] == sgn * xg.pos[0] and md.xgeom_pos[h][i][1] == xg.pos[1]
        if xg.kind == "hull":
            v0, nv = md.xgeom_vert[1][i]
            v = np.array([list(md.hull_vert[1][v0 + j]) for j in range(nv)])
            np.testing.assert_array_equal(v, xg.verts * [-1, 1, 1])
            assert abs(md.xgeom_rbound[0][i] - np.linalg.norm(xg.verts, axis=1).max()) < 1e-15
    # unused capsule slots, MuJoCo-filtered pairs in global ids
    assert [md.geom_body[0][g] for g in range(12, 20)] == [-1] * 8
    body = lambda g: (hand.geoms[g % 20].body if g < 40 else hand.xgeoms[(g - 40) % 12].body)
    hand_of = lambda g: g // 20 if g < 40 else (g - 40) // 12
    pairs = [tuple(md.xpair[i]) for i in range(md.n_xpairs)]
    same = [p for p in pairs if hand_of(p[0]) == hand_of(p[1])]
    assert pairs == sorted(same) + sorted(p for p in pairs if hand_of(p[0]) != hand_of(p[1]))  # same hand first
    assert all(b >= 40 and a < b for a, b in pairs)
    for a, b in pairs:
        if hand_of(a) == hand_of(b):
            ba, bb = body(a), body(b)
            assert ba != bb and hand.bodies[ba].parent != bb and hand.bodies[bb].parent != ba
    caps = [tuple(md.cappair[i]) for i in range(md.n_cappairs)]
    assert all(a % 20 < 12 and b % 20 < 12 for a, b in caps)
    assert len(M.extra_pairs(hand.bodies, hand.geoms, hand.xgeoms, hand.excludes)) == md.n_xpairs
    assert M.build_model(hand=hand, hand_collisions=False).n_xpairs == 0


def _obj(path, pts):
    path.write_text("".join(f"v {x} {y} {z}\n" for x, y, z in pts) + "f 1 2 3\n")


def _stl(path, pts):
    tris = [pts[i:i + 3] for i in range(0, len(pts) - len(pts) % 3, 3)]
    rest = pts[len(tris) * 3:]
    if len(rest):
        tris.append(np.vstack([rest, pts[:3 - len(rest)]]))
    buf = bytearray(b"\0" * 80) + struct.pack("<I", len(tris))
    for t in tris:
        buf += struct.pack("<3f", 0, 0, 0) + struct.pack("<9f", *np.asarray(t, np.float32).ravel()) + b"\0\0"
    path.write_bytes(bytes(buf))


def test_mjcf_box_and_mesh_colliders(dp, tmp_path):
    mj, M = dp.mjcf, dp.model
    hand = box_hull_hand(dp)
    xml = mj.hand_to_mjcf(hand)
    spec = mj.load_hand(xml)  # inline-vertex meshes
    assert [x.kind for x in spec.xgeoms] == [x.kind for x in hand.xgeoms]
    for a, b in zip(hand.xgeoms, spec.xgeoms):
        assert a.body == b.body
        np.testing.assert_allclose(b.pos, a.pos, atol=1e-15)
        if a.kind == "hull":
            np.testing.assert_allclose(b.verts, a.verts, atol=1e-15)
        else:
            assert b.size == a.size
    # the same hulls from OBJ and binary STL files under meshdir, with a mesh scale
    (tmp_path / "meshes").mkdir()
    pts = capsule_points(0.0085, 0.006) * 2.0
    _obj(tmp_path / "meshes" / "tip.obj", pts)
    _stl(tmp_path / "meshes" / "tip.stl", pts.astype(np.float32).astype(np.float64))
    for fname in ("tip.obj", "tip.stl"):
        text = xml.replace("<compiler ", '<compiler meshdir="meshes" ')
        text = text.replace("<asset>", f'<asset><mesh name="filetip" file="{fname}" scale="0.5 0.5 0.5" />', 1)
        text = text.replace('mesh="hull2"', 'mesh="filetip"', 1)
        (tmp_path / "hand.xml").write_text(text)
        s2 = mj.load_hand(tmp_path / "hand.xml")
        c, v = mj.convex_hull_collider(capsule_points(0.0085, 0.006))
        got = s2.xgeoms[2]
        assert len(got.verts) == len(v)
        tol = 1e-15 if fname.endswith("obj") else 1e-7
        np.testing.assert_allclose(np.sort(got.verts, axis=0), np.sort(v, axis=0), atol=tol)
    with pytest.raises(ValueError, match="fitted to mesh"):
        mj.load_hand(xml.replace('type="mesh" mesh="hull2"', 'type="capsule" mesh="hull2"', 1))
    many = np.random.RandomState(0).normal(size=(400, 3))
    many /= np.linalg.norm(many, axis=1, keepdims=True)  # every point on the hull
    big = xml.replace(f'name="hull2" vertex="', f'name="hull2" vertex="{" ".join(repr(float(x)) for x in (many * 0.01).ravel())} ', 1)
    with pytest.raises(ValueError, match="convex hull has"):
        mj.load_hand(big)


def _contact_phase(kind, g1, g2):
    """the collision phase of a contact in the checker's (and the kernel's) list order: 0
    capsule-piano, 1 capsule-capsule, 2 box / hull-piano, 3 box / hull hand-hand"""
    if kind in (0, 1):
        return 2 if g2 >= 40 else 0
    return 3 if g1 >= 40 or g2 >= 40 else 1


def test_oracle_rollout_with_box_and_hull_colliders(dp, ref):
    """The box / hull hand steps finite in the checker, with key-hull, hull-capsule and
    hull-hull contacts, each env's contact list in the phase order the kernel writes (round 6:
    csrc/kernel_v2.inc collide2 takes the box / hull pairs after every capsule pair, as one list)."""
    hand = box_hull_hand(dp)
    task = dp.TaskConfig(hand_xml=dp.mjcf.hand_to_mjcf(hand))
    md, st, tc = dp.compile_task(song(dp, "twinkle"), task, canonical_actions=False)
    n = 8
    o = ref.OracleEnv(md, st, tc, n)
    o.reset()
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(0)
    kinds, phases = set(), set()
    for _ in range(60):
        o.step(rng.uniform(lo, hi, (n, 45)).astype(np.float32))
        for i in range(n):
            cs = o.contacts(i)
            order = [_contact_phase(kind, g1, g2) for kind, key, g1, g2, dist in cs]
            assert order == sorted(order), cs
            phases.update(order)
            for kind, key, g1, g2, dist in cs:
                assert dist <= 1e-12
                t1 = "key" if kind == 0 else ("base" if kind == 1 else ("x" if g1 >= 40 else "c"))
                kinds.add((t1, "x" if g2 >= 40 else "c"))
    s = o.get_state()
    assert np.isfinite(s["qpos"]).all() and np.isfinite(s["qvel"]).all()
    assert {("key", "x"), ("x", "c"), ("x", "x")} <= kinds, kinds
    assert {0, 2, 3} <= phases, phases


def test_mpr_support_ties_are_stable(ref, dp):
    """Support ties (round 6): a fingertip hull resting on a key box with
    a face exactly parallel to the key's top (and a cube hull face-down on a box) puts MPR's
    portal directions exactly normal to tied faces. The tie-tolerant support must make the
    result a continuous function of the input there: 1e-12 m moves of the hull give the same
    contact to 1e-9 (first-maximal picks by rounding noise and could switch the portal). The
    GPU side of the same rule: tests/test_gpu_colliders.py::test_benched_workload_contact_lists."""
    rng = np.random.RandomState(0)
    _, tip = dp.mjcf.convex_hull_collider(capsule_points(0.0085, 0.006))
    for verts, hs, lift in ((CUBE * 0.01, (0.0117, 0.0235, 0.0113), 0.01), (tip, (0.0117, 0.0235, 0.0113), None)):
        for trial in range(20):
            yaw = rng.uniform(0, 2 * math.pi) if trial % 2 else 0.0
            R = rot((0, 0, 1), yaw)
            if lift is None:  # the tip hull's lowest point just below the key's top
                lift = -np.min(verts[:, 2])
            c = np.array([rng.uniform(-0.005, 0.005), rng.uniform(-0.01, 0.01), 0.0113 + lift - 5e-4])
            A = ref.shape("box", c=(0, 0, 0), hs=hs)
            base = ref.narrow(A, ref.shape("hull", c=c, R=R, verts=verts))
            assert len(base) == 1
            for _ in range(8):
                moved = ref.narrow(A, ref.shape("hull", c=c + rng.normal(0, 1e-12, 3), R=R, verts=verts))
                assert len(moved) == 1
                (p0, n0, d0), (p1, n1, d1) = base[0], moved[0]
                assert np.abs(n1 - n0).max() < 1e-9 and abs(d1 - d0) < 1e-9 and np.abs(p1 - p0).max() < 1e-9
