"""Model compiler: the PianoWithShadowHands scene as a flat ``ps_model_desc``.

This plays the role of MJCF assembly + ``mj_compile`` for the one scene the hot path
simulates (robopianist/suite/tasks/base.py:45-197):

* Piano: generated from the reference constants exactly as ``piano_mjcf.build``
  (robopianist/models/piano/piano_mjcf.py:25-402, piano_constants.py:22-85); keys are
  world-attached hinge bodies sorted by key number; geom solref = (2*dt, 1)
  (tasks/base.py:66); the key inertia is the box inertia about the hinge
  (MuJoCo inertiafromgeom).
* Hands: the Shadow Hand E3M5 of MuJoCo Menagerie is NOT in the container (empty
  submodule). The tree below is an AUTHORED restatement of its
  kinematic/inertial layout (body offsets, joint axes/ranges, masses, position-actuator
  gains, fixed J0 tendons) from the public model, with two documented deviations:
  capsule colliders only (the reference's ``primitive_fingertip_collisions`` option,
  shadow_hand.py:144-152, and the MJX attempt's cylinder->capsule conversion,
  parallelized_base.py:49-64). Joint frictionloss 0.01 on every joint (the Menagerie
  right_hand class; hand_provenance.json). Forearm DOFs, their position
  actuators with critical damping and the forearm_tx range follow shadow_hand.py:41-85,
  272-311 and tasks/base.py:160-194. Left hand = mirror image of the right one through
  the hand's x=0 plane.
* Contact filtering (MuJoCo: no same-body or parent-child pairs, plus <exclude> pairs)
  is resolved here into a static capsule-capsule pair list.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, NamedTuple, Optional, Sequence, Tuple

import numpy as np

from . import abi

# ---------------------------------------------------------------- piano constants
# robopianist/models/piano/piano_constants.py:22-76
NUM_WHITE_KEYS = 52
WHITE_KEY_WIDTH = 0.0225
WHITE_KEY_LENGTH = 0.15
WHITE_KEY_HEIGHT = WHITE_KEY_WIDTH
SPACING_BETWEEN_WHITE_KEYS = 0.001
BLACK_KEY_WIDTH = 0.01
BLACK_KEY_LENGTH = 0.09
BLACK_KEY_HEIGHT = 0.018
PIANO_LENGTH = NUM_WHITE_KEYS * WHITE_KEY_WIDTH + (NUM_WHITE_KEYS - 1) * SPACING_BETWEEN_WHITE_KEYS
WHITE_KEY_Z_OFFSET = WHITE_KEY_HEIGHT / 2
BLACK_KEY_X_OFFSET = -WHITE_KEY_LENGTH / 2 + BLACK_KEY_LENGTH / 2
BLACK_KEY_Z_OFFSET = WHITE_KEY_HEIGHT + 0.0125 - BLACK_KEY_HEIGHT / 2
BASE_SIZE = [0.1 / 2, PIANO_LENGTH / 2, 0.04 / 2]
BASE_POS = [-WHITE_KEY_LENGTH / 2 - 0.5 * 0.1 - 0.002, 0.0, 0.04 / 2]
WHITE_KEY_MAX_ANGLE = math.atan(0.01 / WHITE_KEY_LENGTH)
BLACK_KEY_MAX_ANGLE = math.atan(0.008 / BLACK_KEY_LENGTH)
WHITE_KEY_MASS, BLACK_KEY_MASS = 0.04, 0.02
KEY_SPRINGREF = -1 * math.pi / 180
KEY_STIFFNESS = 2.0
KEY_DAMPING = 0.05
KEY_ARMATURE = 0.001
WHITE_KEY_INDICES = [0, 2, 3, 5, 7, 8, 10, 12, 14, 15, 17, 19, 20, 22, 24, 26, 27, 29, 31, 32, 34,
                     36, 38, 39, 41, 43, 44, 46, 48, 50, 51, 53, 55, 56, 58, 60, 62, 63, 65, 67,
                     68, 70, 72, 74, 75, 77, 79, 80, 82, 84, 86, 87]
BLACK_TWIN_KEY_INDICES = [4, 6, 16, 18, 28, 30, 40, 42, 52, 54, 64, 66, 76, 78]
BLACK_TRIPLET_KEY_INDICES = [1, 9, 11, 13, 21, 23, 25, 33, 35, 37, 45, 47, 49, 57, 59, 61, 69, 71,
                             73, 81, 83, 85]

PHYSICS_TIMESTEP = 0.005  # tasks/base.py:28
CONTROL_TIMESTEP = 0.05   # tasks/base.py:31
HAND_POSITIONS = [(0.4, 0.15, 0.13), (0.4, -0.15, 0.13)]  # right, left (tasks/base.py:34-37)
HAND_QUAT = (-1.0, -1.0, 1.0, 1.0)
ATTACHMENT_YAW = 0.0  # degrees (tasks/base.py:39 _ATTACHMENT_YAW)
# PianoTask(reduced_action_space=True) (shadow_hand.py:51-57,164-183): these joints and their
# actuators are removed, THJ2's range (and its actuator's ctrlrange) narrowed
REDUCED_ACTION_SPACE_EXCLUDED = ("THJ5", "THJ1", "LFJ5")
REDUCED_THUMB_RANGE = (0.0, 0.698132)
# the forearm slides this hand models (shadow_hand.py:59-61 _DEFAULT_FOREARM_DOFS); the
# reference's other forearm dofs (tz, roll, pitch, yaw) would need more dof slots than the
# kernel's 26 per hand
FOREARM_DOFS = ("forearm_tx", "forearm_ty")
FINGERTIP_OFFSET = 0.026  # shadow_hand.py:81-82
THUMBTIP_OFFSET = 0.0275
FOREARM_KP = 300.0  # shadow_hand.py:41-52
FOREARM_TY_RANGE = (0.0, 0.06)


def piano_keys():
    """Key bodies sorted by key number: (pos, half, is_black) (piano_mjcf.py:168-391)."""
    keys = {}
    pitch = WHITE_KEY_WIDTH + SPACING_BETWEEN_WHITE_KEYS
    for i in range(NUM_WHITE_KEYS):
        y = -PIANO_LENGTH * 0.5 + WHITE_KEY_WIDTH * 0.5 + i * pitch
        keys[WHITE_KEY_INDICES[i]] = ([0.0, y, WHITE_KEY_Z_OFFSET], False)
    y = WHITE_KEY_WIDTH + 0.5 * (-PIANO_LENGTH + SPACING_BETWEEN_WHITE_KEYS)
    keys[BLACK_TRIPLET_KEY_INDICES[0]] = ([BLACK_KEY_X_OFFSET, y, BLACK_KEY_Z_OFFSET], True)
    n = 0
    for twin in range(2, NUM_WHITE_KEYS - 1, 7):
        for j in range(2):
            y = -PIANO_LENGTH * 0.5 + (j + 1) * pitch + twin * pitch
            keys[BLACK_TWIN_KEY_INDICES[n]] = ([BLACK_KEY_X_OFFSET, y, BLACK_KEY_Z_OFFSET], True)
            n += 1
    n = 1
    for trip in range(5, NUM_WHITE_KEYS - 1, 7):
        for j in range(3):
            y = -PIANO_LENGTH * 0.5 + (j + 1) * pitch + trip * pitch
            keys[BLACK_TRIPLET_KEY_INDICES[n]] = ([BLACK_KEY_X_OFFSET, y, BLACK_KEY_Z_OFFSET], True)
            n += 1
    assert sorted(keys) == list(range(88))
    out = []
    for k in range(88):
        pos, black = keys[k]
        if black:
            half = [BLACK_KEY_LENGTH / 2, BLACK_KEY_WIDTH / 2, BLACK_KEY_HEIGHT / 2]
        else:
            half = [WHITE_KEY_LENGTH / 2, WHITE_KEY_WIDTH / 2, WHITE_KEY_HEIGHT / 2]
        out.append((pos, half, black))
    return out


# ---------------------------------------------------------------- quaternion helpers
def quat_normalize(q):
    q = np.asarray(q, dtype=np.float64)
    return q / np.linalg.norm(q)


def quat_mul(a, b):
    """Hamilton product a * b (w x y z), as mju_mulQuat."""
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return (aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
            aw * by - ax * bz + ay * bw + az * bx, aw * bz + ax * by - ay * bx + az * bw)


def _quat_axisangle(axis, angle):
    """Unit quaternion of a rotation by ``angle`` about the unit ``axis`` (mju_axisAngle2Quat)."""
    s = math.sin(0.5 * angle)
    return (math.cos(0.5 * angle), axis[0] * s, axis[1] * s, axis[2] * s)


def quat_to_mat(q):
    w, x, y, z = quat_normalize(q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


# ---------------------------------------------------------------- authored hand (right)
@dataclass
class Body:
    name: str
    parent: int
    pos: Tuple[float, float, float]
    quat: Tuple[float, float, float, float]
    mass: float
    ipos: Tuple[float, float, float]
    iquat: Tuple[float, float, float, float]
    diag: Tuple[float, float, float]


@dataclass
class Dof:
    name: str
    body: int
    kind: int  # 0 hinge, 1 slide
    axis: Tuple[float, float, float]
    range: Tuple[float, float]
    damping: float
    armature: float = 2e-4
    frictionloss: float = 0.0   # MuJoCo joint frictionloss (dof_frictionloss)


@dataclass
class Geom:
    body: int
    pos: Tuple[float, float, float]
    axis: Tuple[float, float, float]
    halflen: float
    radius: float


@dataclass
class XGeom:
    """A box or convex-hull collider (MuJoCo geom type box / mesh). ``pos``/``quat``: geom
    frame in the body frame; box: ``size`` = half sizes; hull: ``verts`` in the geom frame,
    whose origin is the hull's centre (MuJoCo re-centres a mesh at its centroid)."""
    body: int
    kind: str                                   # "box" | "hull"
    pos: Tuple[float, float, float]
    quat: Tuple[float, float, float, float] = (1.0, 0.0, 0.0, 0.0)
    size: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    verts: Optional[np.ndarray] = None          # [n, 3], hull only

    def rbound(self) -> float:
        if self.kind == "box":
            return float(np.linalg.norm(self.size))
        return float(np.max(np.linalg.norm(np.asarray(self.verts, dtype=np.float64), axis=1)))


class HandSpec(NamedTuple):
    """One (right) hand as build_model consumes it: the authored tree below, or a user MJCF
    through ``mjcf.load_hand``. Indices are MuJoCo's: bodies in depth-first document order,
    dofs in body order, geoms = the capsule colliders in body order."""

    bodies: List[Body]
    dofs: List[Dof]
    geoms: List[Geom]
    excludes: List[Tuple[int, int]]            # <contact><exclude> body pairs
    sites: List[Tuple[int, Tuple[float, float, float]]]  # fingertip sites (body, pos)
    tendons: List[Tuple[int, int]]             # fixed tendons: (dof, dof)
    acts: List[tuple]                          # (kind 0 joint / 1 tendon, target, kp, ctrlrange, forcerange|None)
    obs_order: List[int]                       # joints_pos observation order (dof indices)
    tendon_coef: Optional[List[Tuple[float, float]]] = None  # None = (1, 1) each
    xgeoms: Optional[List[XGeom]] = None       # box / hull colliders beside the capsules
    contact: Optional[tuple] = None            # collider (solref, solimp, friction); None = HAND_CONTACT


ID = (1.0, 0.0, 0.0, 0.0)
QX90 = (1.0, 0.0, 0.0, 1.0)  # (w, x, y, z) un-normalised as in the MJCF


def _finger(prefix, parent, knuckle_pos):
    """knuckle, proximal, middle, distal bodies of ff/mf/rf (and lf after the metacarpal)."""
    return [
        Body(prefix + "knuckle", parent, knuckle_pos, ID, 0.008, (0, 0, 0), (0.5, 0.5, -0.5, 0.5),
             (3.2e-7, 2.6e-7, 2.6e-7)),
        Body(prefix + "proximal", -1, (0, 0, 0), ID, 0.03, (0, 0, 0.0225), QX90,
             (1e-5, 9.8e-6, 1.8e-6)),
        Body(prefix + "middle", -1, (0, 0, 0.045), ID, 0.017, (0, 0, 0.0125), QX90,
             (2.7e-6, 2.6e-6, 8.7e-7)),
        Body(prefix + "distal", -1, (0, 0, 0.025), ID, 0.013, (0, 0, 0.0130769), QX90,
             (1.28092e-6, 1.12092e-6, 5.3e-7)),
    ]


# Menagerie right_hand collision class: solref / solimp / friction of every hand collider
HAND_CONTACT = ((0.005, 1.0), (0.5, 0.99, 0.0001, 0.5, 2.0), 1.0)
MENAGERIE_FRICTIONLOSS = 0.01  # shadow_hand/right_hand.xml <default class="right_hand"><joint frictionloss>


def _right_hand_tree():
    bodies: List[Body] = [
        Body("forearm", -1, (0, 0, 0), ID, 3.0, (0, 0, 0.09), ID, (0.0138, 0.0138, 0.00744)),
        Body("wrist", 0, (0.01, 0, 0.21301), ID, 0.1, (0, 0, 0.029), (0.5, 0.5, 0.5, 0.5),
             (6.4e-5, 4.38e-5, 3.5e-5)),
        Body("palm", 1, (0, 0, 0.034), ID, 0.3, (0, 0, 0.035), QX90,
             (5.287e-4, 3.581e-4, 1.91e-4)),
    ]
    for prefix, kpos in (("ff", (0.033, 0, 0.095)), ("mf", (0.011, 0, 0.099)),
                         ("rf", (-0.011, 0, 0.095))):
        chain = _finger(prefix, 2, kpos)
        base = len(bodies)
        for i, b in enumerate(chain):
            if i > 0:
                b.parent = base + i - 1
            bodies.append(b)
    bodies.append(Body("lfmetacarpal", 2, (-0.033, 0, 0.02071), ID, 0.03, (0, 0, 0.04), QX90,
                       (1.638e-5, 1.45e-5, 4.272e-6)))
    meta = len(bodies) - 1
    chain = _finger("lf", meta, (0, 0, 0.06579))
    base = len(bodies)
    for i, b in enumerate(chain):
        if i > 0:
            b.parent = base + i - 1
        bodies.append(b)
    th = len(bodies)
    bodies += [
        Body("thbase", 2, (0.034, -0.00858, 0.029), (0.92388, 0, 0.382683, 0), 0.01, (0, 0, 0), ID,
             (1.6e-7, 1.6e-7, 1.6e-7)),
        Body("thproximal", th, (0, 0, 0), ID, 0.04, (0, 0, 0.019), QX90,
             (1.36e-5, 1.36e-5, 3.13e-6)),
        Body("thhub", th + 1, (0, 0, 0.038), ID, 0.005, (0, 0, 0), ID, (1e-6, 1e-6, 3e-7)),
        Body("thmiddle", th + 2, (0, 0, 0), ID, 0.02, (0, 0, 0.016), QX90,
             (5.1e-6, 5.1e-6, 1.21e-6)),
        Body("thdistal", th + 3, (0, 0, 0.032), (1, 0, 0, -1), 0.016, (0, 0, 0.01375), QX90,
             (2.1e-6, 2.2e-6, 1e-6)),
    ]
    assert len(bodies) == abi.HAND_NBODY
    idx = {b.name: i for i, b in enumerate(bodies)}

    knuckle_rng, prox_rng, md_rng = (-0.349066, 0.349066), (-0.261799, 1.5708), (0.0, 1.5708)
    X, NY = (1.0, 0.0, 0.0), (0.0, -1.0, 0.0)
    dofs = [
        Dof("forearm_tx", idx["forearm"], 1, (-1.0, 0.0, 0.0), (-1.0, 1.0), 0.0),
        Dof("forearm_ty", idx["forearm"], 1, (0.0, 0.0, 1.0), FOREARM_TY_RANGE, 0.0),
        Dof("WRJ2", idx["wrist"], 0, (0.0, 1.0, 0.0), (-0.523599, 0.174533), 0.5),
        Dof("WRJ1", idx["palm"], 0, X, (-0.698132, 0.488692), 0.5),
    ]
    for f in ("ff", "mf", "rf"):
        dofs += [Dof(f.upper() + "J4", idx[f + "knuckle"], 0, NY, knuckle_rng, 0.05),
                 Dof(f.upper() + "J3", idx[f + "proximal"], 0, X, prox_rng, 0.05),
                 Dof(f.upper() + "J2", idx[f + "middle"], 0, X, md_rng, 0.05),
                 Dof(f.upper() + "J1", idx[f + "distal"], 0, X, md_rng, 0.05)]
    dofs += [Dof("LFJ5", idx["lfmetacarpal"], 0, (0.573576, 0.0, 0.819152), (0.0, 0.785398), 0.05),
             Dof("LFJ4", idx["lfknuckle"], 0, NY, knuckle_rng, 0.05),
             Dof("LFJ3", idx["lfproximal"], 0, X, prox_rng, 0.05),
             Dof("LFJ2", idx["lfmiddle"], 0, X, md_rng, 0.05),
             Dof("LFJ1", idx["lfdistal"], 0, X, md_rng, 0.05),
             Dof("THJ5", idx["thbase"], 0, (0.0, 0.0, -1.0), (-1.0472, 1.0472), 0.05),
             Dof("THJ4", idx["thproximal"], 0, X, (0.0, 1.22173), 0.05),
             Dof("THJ3", idx["thhub"], 0, X, (-0.20944, 0.20944), 0.05),
             Dof("THJ2", idx["thmiddle"], 0, NY, (-0.698132, 0.698132), 0.05),
             Dof("THJ1", idx["thdistal"], 0, X, (-0.261799, 1.5708), 0.05)]
    assert len(dofs) == abi.HAND_NDOF
    # Menagerie right_hand class: frictionloss on every joint; the forearm slides, added under
    # the root's childclass by _add_dofs (shadow_hand.py:272-311), inherit it
    for dof in dofs:
        dof.frictionloss = MENAGERIE_FRICTIONLOSS
    Z = (0.0, 0.0, 1.0)
    geoms = [Geom(idx["forearm"], (0, 0, 0.11), Z, 0.06, 0.035),
             Geom(idx["wrist"], (0, 0, 0), X, 0.015, 0.0135),
             Geom(idx["palm"], (0, -0.002, 0.028), X, 0.02, 0.011),
             Geom(idx["palm"], (0, -0.002, 0.068), X, 0.026, 0.011)]
    for f in ("ff", "mf", "rf", "lf"):
        if f == "lf":
            geoms.append(Geom(idx["lfmetacarpal"], (0, 0, 0.03), Z, 0.015, 0.011))
        geoms += [Geom(idx[f + "proximal"], (0, 0, 0.025), Z, 0.02, 0.01),
                  Geom(idx[f + "middle"], (0, 0, 0.0125), Z, 0.0125, 0.00805),
                  Geom(idx[f + "distal"], (0, 0, 0.012), Z, 0.006, 0.0085)]
    geoms += [Geom(idx["thproximal"], (0, 0, 0.019), Z, 0.019, 0.013),
              Geom(idx["thmiddle"], (0, 0, 0.016), Z, 0.016, 0.011),
              Geom(idx["thdistal"], (0, 0, 0.013), Z, 0.006, 0.009)]
    assert len(geoms) == abi.HAND_NGEOM
    excludes = [(idx["wrist"], idx["forearm"]), (idx["thproximal"], idx["thmiddle"]),
                (idx["palm"], idx["thproximal"])]
    sites = [(idx["thdistal"], (0, 0, THUMBTIP_OFFSET))] + \
        [(idx[f + "distal"], (0, 0, FINGERTIP_OFFSET)) for f in ("ff", "mf", "rf", "lf")]
    dof_idx = {d.name: i for i, d in enumerate(dofs)}
    tendons = [(dof_idx[f + "J2"], dof_idx[f + "J1"]) for f in ("FF", "MF", "RF", "LF")]
    # Actuators in Menagerie document order, then forearm_tx/ty (shadow_hand.py:303-309).
    # (kind, target, kp, ctrlrange, forcerange)
    acts = [
        (0, "WRJ2", 10.0, (-0.523599, 0.174533), (-10.0, 10.0)),
        (0, "WRJ1", 8.0, (-0.698132, 0.488692), (-5.0, 5.0)),
        (0, "THJ5", 0.4, (-1.0472, 1.0472), (-3.0, 3.0)),
        (0, "THJ4", 1.0, (0.0, 1.22173), (-2.0, 2.0)),
        (0, "THJ3", 0.5, (-0.20944, 0.20944), (-1.0, 1.0)),
        (0, "THJ2", 1.5, (-0.698132, 0.698132), (-1.0, 1.0)),
        (0, "THJ1", 1.0, (-0.261799, 1.5708), (-1.0, 1.0)),
    ]
    for t, f in enumerate(("FF", "MF", "RF")):
        acts += [(0, f + "J4", 1.0, knuckle_rng, (-1.0, 1.0)),
                 (0, f + "J3", 1.0, prox_rng, (-1.0, 1.0)),
                 (1, t, 0.5, (0.0, 3.1415), (-1.0, 1.0))]
    acts += [(0, "LFJ5", 1.0, (0.0, 0.785398), (-1.0, 1.0)),
             (0, "LFJ4", 1.0, knuckle_rng, (-1.0, 1.0)),
             (0, "LFJ3", 1.0, prox_rng, (-1.0, 1.0)),
             (1, 3, 0.5, (0.0, 3.1415), (-1.0, 1.0)),
             (0, "forearm_tx", FOREARM_KP, (-1.0, 1.0), None),
             (0, "forearm_ty", FOREARM_KP, FOREARM_TY_RANGE, None)]
    assert len(acts) == abi.HAND_NACT
    acts = [(k, dof_idx[t] if k == 0 else t, kp, cr, fr) for (k, t, kp, cr, fr) in acts]
    # joints_pos order: Menagerie joints in document order, forearm joints appended last.
    obs_order = list(range(2, abi.HAND_NDOF)) + [0, 1]
    return HandSpec(bodies, dofs, geoms, excludes, sites, tendons, acts, obs_order, contact=HAND_CONTACT)


def authored_hand() -> HandSpec:
    """The authored right hand (the default of build_model)."""
    return _right_hand_tree()


def _mirror_quat(q):
    w, x, y, z = q
    return (w, x, -y, -z)


def _mirror_vec(v):
    return (-v[0], v[1], v[2])


def _mirror_axial(a):
    return (a[0], -a[1], -a[2])


def _inertia6(iquat, diag, mirror=False):
    R = quat_to_mat(iquat)
    I = R @ np.diag(diag) @ R.T
    if mirror:
        S = np.diag([-1.0, 1.0, 1.0])
        I = S @ I @ S
    return [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]


def _subtree_mass(bodies, root):
    total = 0.0
    for i, b in enumerate(bodies):
        j = i
        while j != -1 and j != root:
            j = bodies[j].parent
        if j == root:
            total += b.mass
    return total


def build_model(control_timestep: float = CONTROL_TIMESTEP, physics_timestep: float = PHYSICS_TIMESTEP,
                hand_collisions: bool = True, hand: Optional[HandSpec] = None,
                gravity_compensation: bool = False, attachment_yaw: float = ATTACHMENT_YAW,
                reduced_action_space: bool = False, forearm_dofs=FOREARM_DOFS) -> abi.ModelDesc:
    """Compile the scene into a ``ps_model_desc``.

    ``hand``: the right hand to use (``mjcf.load_hand`` of a user MJCF); default the authored
    one. The left hand is its mirror image, as for the authored hand.

    ``hand_collisions=False`` is ``disable_hand_collisions`` (piano_with_shadow_hands.py:476-489):
    every hand collider gets contype=1, conaffinity=0, so no hand geom pair collides
    (hands still collide with the piano, whose conaffinity is 1).

    ``gravity_compensation`` (tasks/base.py:185-186): gravcomp = 1 on every hand body, a passive
    force cancelling the hands' gravity. ``attachment_yaw`` (degrees, tasks/base.py:174-181): the
    hand roots turned about world z by +yaw (right) / -yaw (left) before their quaternion.

    ``reduced_action_space`` (shadow_hand.py:73-79,164-183) removes THJ5, THJ1 and LFJ5 with
    their actuators and narrows THJ2 to (0, 0.698132); ``forearm_dofs`` (shadow_hand.py:270-311)
    names the forearm slides the hand keeps, a subset of ("forearm_tx", "forearm_ty") in that
    order. A removed joint keeps its dof slot, locked at 0 (``dof_locked``: no force, row or
    Jacobian entry - MuJoCo's body without that joint), and leaves joints_pos and the action row
    (``n_obs_joints``, ``act_column``, ``n_action``).
    """
    forearm_dofs = tuple(forearm_dofs)
    if any(f not in FOREARM_DOFS for f in forearm_dofs) or list(forearm_dofs) != [f for f in FOREARM_DOFS
                                                                                   if f in forearm_dofs]:
        raise ValueError(f"forearm_dofs must be a subset of {FOREARM_DOFS} in that order (this kernel's hand "
                         f"has 26 dof slots: the reference's forearm_tz / roll / pitch / yaw do not fit), "
                         f"got {forearm_dofs!r}")
    m = abi.ModelDesc()
    m.timestep = physics_timestep
    m.n_substeps = int(round(control_timestep / physics_timestep))
    m.gravity[:] = (0.0, 0.0, -9.81)
    m.hand_gravcomp = 1.0 if gravity_compensation else 0.0
    for k, (pos, half, black) in enumerate(piano_keys()):
        m.key_pos[k][:] = pos
        m.key_half[k][:] = half
        m.key_anchor[k][:] = (-half[0], 0.0, 0.0)
        mass = BLACK_KEY_MASS if black else WHITE_KEY_MASS
        m.key_mass[k] = mass
        L, H = 2 * half[0], 2 * half[2]
        m.key_inertia[k] = mass * (L * L + H * H) / 12.0 + mass * half[0] ** 2
        m.key_armature[k] = KEY_ARMATURE
        m.key_damping[k] = KEY_DAMPING
        m.key_stiffness[k] = KEY_STIFFNESS
        m.key_springref[k] = KEY_SPRINGREF
        m.key_range[k][:] = (0.0, BLACK_KEY_MAX_ANGLE if black else WHITE_KEY_MAX_ANGLE)
    m.base_pos[:] = BASE_POS
    m.base_half[:] = BASE_SIZE
    m.piano_contact.solref[:] = (2 * physics_timestep, 1.0)
    m.piano_contact.solimp[:] = (0.9, 0.95, 0.001, 0.5, 2.0)
    m.piano_contact.friction = 1.0
    m.limit_solref[:] = (0.02, 1.0)
    m.limit_solimp[:] = (0.9, 0.95, 0.001, 0.5, 2.0)
    spec = hand if hand is not None else _right_hand_tree()
    sr, si, fr = spec.contact if spec.contact is not None else HAND_CONTACT
    m.hand_contact.solref[:] = sr
    m.hand_contact.solimp[:] = si
    m.hand_contact.friction = fr
    # solreffriction / solimpfriction: MuJoCo's defaults (the reference sets none)
    m.friction_solref[:] = (0.02, 1.0)
    m.friction_solimp[:] = (0.9, 0.95, 0.001, 0.5, 2.0)

    bodies, dofs, geoms, excludes, sites, tendons, acts, obs_order = spec[:8]
    tcoef = spec.tendon_coef or [(1.0, 1.0)] * len(tendons)
    forearm_mass = _subtree_mass(bodies, 0)
    root_quats = [tuple(quat_normalize(quat_mul(_quat_axisangle((0.0, 0.0, 1.0), math.radians(sg * attachment_yaw)),
                                                 HAND_QUAT))) for sg in (1.0, -1.0)]  # right, left
    m.root_geom_count = sum(1 for g in geoms if g.body == 0)
    for h in range(abi.NHAND):
        mir = h == 1
        for i, b in enumerate(bodies):
            m.body_parent[h][i] = b.parent
            if i == 0:
                m.body_pos[h][i][:] = HAND_POSITIONS[h]
                m.body_quat[h][i][:] = root_quats[h]
            else:
                m.body_pos[h][i][:] = _mirror_vec(b.pos) if mir else b.pos
                q = quat_normalize(b.quat)
                m.body_quat[h][i][:] = _mirror_quat(q) if mir else q
            m.body_mass[h][i] = b.mass
            m.body_ipos[h][i][:] = _mirror_vec(b.ipos) if mir else b.ipos
            m.body_inertia[h][i][:] = _inertia6(b.iquat, b.diag, mir)
        y = HAND_POSITIONS[h][1]
        for j, dof in enumerate(dofs):
            m.dof_body[h][j] = dof.body
            m.dof_type[h][j] = dof.kind
            # Forearm slides are added post-hoc with identical axes for both hands.
            axis = dof.axis if (not mir or dof.kind == 1) else _mirror_axial(dof.axis)
            m.dof_axis[h][j][:] = axis
            rng = dof.range
            if dof.name == "forearm_tx":  # tasks/base.py:160-194
                rng = (-PIANO_LENGTH / 2 - y, PIANO_LENGTH / 2 - y)
            m.dof_range[h][j][:] = rng
            m.dof_limited[h][j] = 1
            damping = dof.damping
            if dof.kind == 1:  # critical damping 2*sqrt(m_subtree * kp) (shadow_hand.py:299-301)
                damping = 2.0 * math.sqrt(forearm_mass * FOREARM_KP)
            m.dof_damping[h][j] = damping
            m.dof_armature[h][j] = dof.armature
            m.dof_frictionloss[h][j] = dof.frictionloss
            m.dof_obs_order[h][j] = obs_order[j]
        for g in range(abi.HAND_NGEOM):
            m.geom_body[h][g] = -1  # unused slot
        for g, geom in enumerate(geoms):
            m.geom_body[h][g] = geom.body
            m.geom_pos[h][g][:] = _mirror_vec(geom.pos) if mir else geom.pos
            m.geom_axis[h][g][:] = _mirror_vec(geom.axis) if mir else geom.axis
            m.geom_halflen[h][g] = geom.halflen
            m.geom_radius[h][g] = geom.radius
        for s, (body, pos) in enumerate(sites):
            m.site_body[h][s] = body
            m.site_pos[h][s][:] = _mirror_vec(pos) if mir else pos
        for t, (d2, d1) in enumerate(tendons):
            m.tendon_dof[h][t][:] = (d2, d1)
            m.tendon_coef[h][t][:] = tcoef[t]
        # removed joints (reduced_action_space, forearm_dofs): locked dof slots
        locked = [(reduced_action_space and any(dof.name.endswith(x) for x in REDUCED_ACTION_SPACE_EXCLUDED))
                  or (dof.name in FOREARM_DOFS and dof.name not in forearm_dofs) for dof in dofs]
        for j, dof in enumerate(dofs):
            m.dof_locked[h][j] = int(locked[j])
            if reduced_action_space and dof.name.endswith("THJ2"):
                m.dof_range[h][j][:] = REDUCED_THUMB_RANGE
        if any(locked):
            oo = [j for j in obs_order if not locked[j]]
            m.n_obs_joints[h] = len(oo)
            for i in range(abi.HAND_NDOF):
                m.dof_obs_order[h][i] = oo[i] if i < len(oo) else 0
        for a, (kind, target, kp, cr, fr) in enumerate(acts):
            m.act_kind[h][a] = kind
            m.act_target[h][a] = target
            m.act_kp[h][a] = kp
            if kind == 0 and dofs[target].name == "forearm_tx":
                cr = (-PIANO_LENGTH / 2 - y, PIANO_LENGTH / 2 - y)
            if kind == 0 and reduced_action_space and dofs[target].name.endswith("THJ2"):
                cr = REDUCED_THUMB_RANGE
            m.act_ctrlrange[h][a][:] = cr
            m.act_forcelimited[h][a] = 0 if fr is None else 1
            m.act_forcerange[h][a][:] = (0.0, 0.0) if fr is None else fr
    if any(m.dof_locked[h][j] for h in range(abi.NHAND) for j in range(abi.HAND_NDOF)):
        # the action row: each hand's actuators on kept joints in order, then sustain
        col = 0
        for h in range(abi.NHAND):
            for a, (kind, target, *_) in enumerate(acts):
                present = kind == 1 or not m.dof_locked[h][target]
                m.act_column[h][a] = col if present else -1
                col += present
        m.n_action = col + 1
    xgeoms = spec.xgeoms or []
    if len(geoms) > abi.HAND_NGEOM or len(xgeoms) > abi.HAND_NXGEOM:
        raise ValueError(f"at most {abi.HAND_NGEOM} capsule and {abi.HAND_NXGEOM} box/hull colliders per hand "
                         f"(got {len(geoms)} and {len(xgeoms)})")
    for h in range(abi.NHAND):
        mir = h == 1
        nv = 0
        for i, xg in enumerate(xgeoms):
            m.xgeom_type[h][i] = abi.GEOM_BOX if xg.kind == "box" else abi.GEOM_HULL
            m.xgeom_body[h][i] = xg.body
            m.xgeom_pos[h][i][:] = _mirror_vec(xg.pos) if mir else xg.pos
            q = quat_normalize(xg.quat)
            m.xgeom_quat[h][i][:] = _mirror_quat(q) if mir else q
            m.xgeom_size[h][i][:] = xg.size
            m.xgeom_rbound[h][i] = xg.rbound()
            if xg.kind == "hull":
                v = np.asarray(xg.verts, dtype=np.float64)
                if not 4 <= len(v) <= abi.HULL_MAXVERT:
                    raise ValueError(f"a hull collider needs 4..{abi.HULL_MAXVERT} vertices, got {len(v)}")
                if nv + len(v) > abi.HAND_HULLVERT:
                    raise ValueError(f"more than {abi.HAND_HULLVERT} hull vertices in one hand")
                m.xgeom_vert[h][i][:] = (nv, len(v))
                for j, p in enumerate(v):
                    m.hull_vert[h][nv + j][:] = _mirror_vec(p) if mir else p
                nv += len(v)
    set_const(m)
    pairs = capsule_pairs(bodies, geoms, excludes) if hand_collisions else []
    assert len(pairs) <= abi.MAX_CAPPAIRS
    m.n_cappairs = len(pairs)
    for i, (a, b) in enumerate(pairs):
        m.cappair[i][:] = (a, b)
    xpairs = extra_pairs(bodies, geoms, xgeoms, excludes) if hand_collisions else []
    if len(xpairs) > abi.MAX_XPAIRS:
        raise ValueError(f"{len(xpairs)} collider pairs with a box/hull collider; at most {abi.MAX_XPAIRS}")
    m.n_xpairs = len(xpairs)
    for i, (a, b) in enumerate(xpairs):
        m.xpair[i][:] = (a, b)
    return m


def _axisangle(a, t):
    a = np.asarray(a, dtype=np.float64)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(t) * K + (1 - math.cos(t)) * K @ K


def set_const(m: abi.ModelDesc) -> None:
    """``mj_setConst`` inverse weights at qpos0 (all joint positions zero).

    body: trace(Jp M^-1 Jp^T)/3 for the body COM; dof: diag(M^-1). These set the
    regulariser ``R = (1-imp)/imp * diagApprox`` of every soft constraint, as MuJoCo does
    (diagApprox from invweight0, not from the configuration-dependent J M^-1 J^T).
    """
    for k in range(abi.NKEY):
        mk = m.key_inertia[k] + m.key_armature[k]
        r = np.array([-m.key_anchor[k][0], 0.0, 0.0])  # COM relative to hinge
        jp = np.cross([0.0, 1.0, 0.0], r)
        m.key_body_invweight[k] = float(jp @ jp) / mk / 3.0
        m.key_dof_invweight[k] = 1.0 / mk
    nb, nd = abi.HAND_NBODY, abi.HAND_NDOF
    for h in range(abi.NHAND):
        R = [None] * nb
        o = [None] * nb
        axis = np.zeros((nd, 3))
        for b in range(nb):
            p = m.body_parent[h][b]
            Q = quat_to_mat(list(m.body_quat[h][b]))
            pos = np.array(list(m.body_pos[h][b]))
            if p < 0:
                R[b], o[b] = Q, pos
            else:
                R[b], o[b] = R[p] @ Q, o[p] + R[p] @ pos
            for j in range(nd):
                if m.dof_body[h][j] == b:
                    axis[j] = R[b] @ np.array(list(m.dof_axis[h][j]))
        com = [o[b] + R[b] @ np.array(list(m.body_ipos[h][b])) for b in range(nb)]
        anc = []
        for b in range(nb):
            dofs, bb = [], b
            while bb >= 0:
                dofs += [j for j in range(nd) if m.dof_body[h][j] == bb]
                bb = m.body_parent[h][bb]
            anc.append(dofs)
        Jp = np.zeros((nb, 3, nd))
        Jr = np.zeros((nb, 3, nd))
        for b in range(nb):
            for j in anc[b]:
                jb = m.dof_body[h][j]
                if m.dof_type[h][j] == 0:
                    Jp[b, :, j] = np.cross(axis[j], com[b] - o[jb])
                    Jr[b, :, j] = axis[j]
                else:
                    Jp[b, :, j] = axis[j]
        M = np.diag([m.dof_armature[h][j] for j in range(nd)])
        for b in range(nb):
            I6 = list(m.body_inertia[h][b])
            Il = np.array([[I6[0], I6[3], I6[4]], [I6[3], I6[1], I6[5]], [I6[4], I6[5], I6[2]]])
            Iw = R[b] @ Il @ R[b].T
            M += m.body_mass[h][b] * Jp[b].T @ Jp[b] + Jr[b].T @ Iw @ Jr[b]
        free = [j for j in range(nd) if not m.dof_locked[h][j]]  # a removed joint: not in M
        Minv = np.zeros((nd, nd))
        Minv[np.ix_(free, free)] = np.linalg.inv(M[np.ix_(free, free)])
        for b in range(nb):
            m.body_invweight[h][b] = float(np.trace(Jp[b] @ Minv @ Jp[b].T)) / 3.0
        for j in range(nd):
            m.dof_invweight[h][j] = float(Minv[j, j]) if j in free else 1.0


def capsule_pairs(bodies, geoms, excludes):
    """MuJoCo pair filtering for hand geoms (contype=conaffinity=1 on every collider).

    Same hand: skip same body, parent/child bodies and <exclude> pairs. Across hands:
    every pair. Ordered by (geom1, geom2) global index.
    """
    ex = {frozenset(p) for p in excludes}
    pairs = []
    ng, stride = len(geoms), abi.HAND_NGEOM  # global id h * HAND_NGEOM + g (unused slots past ng)
    for h in range(abi.NHAND):
        for a in range(ng):
            for b in range(a + 1, ng):
                ba, bb = geoms[a].body, geoms[b].body
                if ba == bb or bodies[ba].parent == bb or bodies[bb].parent == ba:
                    continue
                if frozenset((ba, bb)) in ex:
                    continue
                pairs.append((h * stride + a, h * stride + b))
    for a in range(ng):
        for b in range(ng):
            pairs.append((a, stride + b))
    return pairs


def extra_pairs(bodies, geoms, xgeoms, excludes):
    """Hand-hand collider pairs with at least one box/hull collider, MuJoCo-filtered as
    capsule_pairs, in global ids (capsule h*HAND_NGEOM + g, extra 2*HAND_NGEOM +
    h*HAND_NXGEOM + i), a < b: the pairs within one hand first, then the cross-hand ones, each
    ordered by (a, b) (as capsule_pairs: the kernel skips the cross-hand ones wholesale when the
    hands' bounding boxes are apart)."""
    ex = {frozenset(p) for p in excludes}
    ng, nx = abi.HAND_NGEOM, abi.HAND_NXGEOM
    coll = []  # (global id, hand, body, is_extra)
    for h in range(abi.NHAND):
        coll += [(h * ng + g, h, geom.body, False) for g, geom in enumerate(geoms)]
    for h in range(abi.NHAND):
        coll += [(abi.NHAND * ng + h * nx + i, h, xg.body, True) for i, xg in enumerate(xgeoms)]
    coll.sort()
    pairs = []
    for ia, (ga, ha, ba, xa) in enumerate(coll):
        for gb, hb, bb, xb in coll[ia + 1:]:
            if not (xa or xb):
                continue
            if ha == hb:
                if ba == bb or bodies[ba].parent == bb or bodies[bb].parent == ba or frozenset((ba, bb)) in ex:
                    continue
            pairs.append((ga, gb, ha != hb))
    return [(a, b) for a, b, _ in sorted(pairs, key=lambda p: (p[2], p[0], p[1]))]


def action_dim(m: abi.ModelDesc) -> int:
    """The action row width: 45 for the full hands; fewer without some joints (n_action)."""
    return m.n_action if m.n_action > 0 else abi.NACTION


def action_columns(m: abi.ModelDesc):
    """[(hand, actuator, column)] of the actuators in the action row."""
    return [(h, a, m.act_column[h][a] if m.n_action > 0 else h * abi.HAND_NACT + a)
            for h in range(abi.NHAND) for a in range(abi.HAND_NACT)
            if m.n_action <= 0 or m.act_column[h][a] >= 0]


def action_spec(m: abi.ModelDesc):
    """Action bounds [action_dim]: right hand 22, left hand 22, sustain [0, 1]
    (piano_with_shadow_hands.py:226-237); without the removed actuators when the model lacks
    some joints (reduced_action_space, forearm_dofs)."""
    n = action_dim(m)
    lo = np.zeros(n)
    hi = np.zeros(n)
    for h, a, c in action_columns(m):
        lo[c] = m.act_ctrlrange[h][a][0]
        hi[c] = m.act_ctrlrange[h][a][1]
    lo[-1], hi[-1] = 0.0, 1.0
    return lo, hi
