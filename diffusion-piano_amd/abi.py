"""ctypes mirror of include/pianosim.h (descriptor structs and constants)."""

import ctypes as C

NKEY = 88
NHAND = 2
HAND_NBODY = 25
HAND_NDOF = 26
HAND_NGEOM = 20
HAND_NACT = 22
HAND_NTENDON = 4
NFINGER = 5
NV = NKEY + NHAND * HAND_NDOF
NU = NHAND * HAND_NACT
NACTION = NU + 1
MAX_CAPPAIRS = 768
HAND_NXGEOM = 12       # box / convex-hull colliders per hand
HULL_MAXVERT = 64
HAND_HULLVERT = 384
MAX_XPAIRS = 1024
GEOM_NONE, GEOM_BOX, GEOM_HULL = 0, 1, 2
MAX_NOTES = 16
MAX_CONTACTS_LIMIT = 24
NTERMS = 5
NSTATS = 7  # ps_solver_stats slots (PS_STAT_*): Newton iterations, contact-cap substeps, iteration-cap
            # substeps, most contact rows in a substep, hand-coupled substeps, non-positive pivots,
            # most coupled dofs in a substep
STAT_SOLVES, STAT_CONTACT_CAP, STAT_ITER_CAP, STAT_MAX_ROWS, STAT_COUPLED, STAT_BAD_PIVOT, STAT_MAX_CDOFS = range(7)
NWARN = 3  # ps_warnings slots: mj_checkPos / mj_checkVel / mj_checkAcc resets
WARN_BADQPOS, WARN_BADQVEL, WARN_BADQACC = range(3)
NMUSIC = 6  # ps_musical_metrics slots: precision, recall, f1, sustain_precision, sustain_recall, sustain_f1
FIRST, MID, LAST = 0, 1, 2

d = C.c_double
i32 = C.c_int32


def _arr(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


class ContactParam(C.Structure):
    _fields_ = [("solref", _arr(d, 2)), ("solimp", _arr(d, 5)), ("friction", d)]


class ModelDesc(C.Structure):
    _fields_ = [
        ("timestep", d), ("n_substeps", i32), ("gravity", _arr(d, 3)),
        ("key_pos", _arr(d, NKEY, 3)), ("key_half", _arr(d, NKEY, 3)),
        ("key_anchor", _arr(d, NKEY, 3)), ("key_mass", _arr(d, NKEY)),
        ("key_inertia", _arr(d, NKEY)), ("key_armature", _arr(d, NKEY)),
        ("key_damping", _arr(d, NKEY)), ("key_stiffness", _arr(d, NKEY)),
        ("key_springref", _arr(d, NKEY)), ("key_range", _arr(d, NKEY, 2)),
        ("base_pos", _arr(d, 3)), ("base_half", _arr(d, 3)),
        ("piano_contact", ContactParam),
        ("limit_solref", _arr(d, 2)), ("limit_solimp", _arr(d, 5)),
        ("body_parent", _arr(i32, NHAND, HAND_NBODY)),
        ("body_pos", _arr(d, NHAND, HAND_NBODY, 3)), ("body_quat", _arr(d, NHAND, HAND_NBODY, 4)),
        ("body_mass", _arr(d, NHAND, HAND_NBODY)), ("body_ipos", _arr(d, NHAND, HAND_NBODY, 3)),
        ("body_inertia", _arr(d, NHAND, HAND_NBODY, 6)),
        ("dof_body", _arr(i32, NHAND, HAND_NDOF)), ("dof_type", _arr(i32, NHAND, HAND_NDOF)),
        ("dof_axis", _arr(d, NHAND, HAND_NDOF, 3)), ("dof_range", _arr(d, NHAND, HAND_NDOF, 2)),
        ("dof_limited", _arr(i32, NHAND, HAND_NDOF)), ("dof_damping", _arr(d, NHAND, HAND_NDOF)),
        ("dof_armature", _arr(d, NHAND, HAND_NDOF)), ("dof_obs_order", _arr(i32, NHAND, HAND_NDOF)),
        ("geom_body", _arr(i32, NHAND, HAND_NGEOM)), ("geom_pos", _arr(d, NHAND, HAND_NGEOM, 3)),
        ("geom_axis", _arr(d, NHAND, HAND_NGEOM, 3)), ("geom_halflen", _arr(d, NHAND, HAND_NGEOM)),
        ("geom_radius", _arr(d, NHAND, HAND_NGEOM)), ("root_geom_count", i32),
        ("hand_contact", ContactParam),
        ("site_body", _arr(i32, NHAND, NFINGER)), ("site_pos", _arr(d, NHAND, NFINGER, 3)),
        ("tendon_dof", _arr(i32, NHAND, HAND_NTENDON, 2)),
        ("tendon_coef", _arr(d, NHAND, HAND_NTENDON, 2)),
        ("act_kind", _arr(i32, NHAND, HAND_NACT)), ("act_target", _arr(i32, NHAND, HAND_NACT)),
        ("act_kp", _arr(d, NHAND, HAND_NACT)), ("act_ctrlrange", _arr(d, NHAND, HAND_NACT, 2)),
        ("act_forcelimited", _arr(i32, NHAND, HAND_NACT)),
        ("act_forcerange", _arr(d, NHAND, HAND_NACT, 2)),
        ("n_cappairs", i32), ("cappair", _arr(i32, MAX_CAPPAIRS, 2)),
        ("key_body_invweight", _arr(d, NKEY)), ("key_dof_invweight", _arr(d, NKEY)),
        ("body_invweight", _arr(d, NHAND, HAND_NBODY)), ("dof_invweight", _arr(d, NHAND, HAND_NDOF)),
        ("xgeom_type", _arr(i32, NHAND, HAND_NXGEOM)), ("xgeom_body", _arr(i32, NHAND, HAND_NXGEOM)),
        ("xgeom_pos", _arr(d, NHAND, HAND_NXGEOM, 3)), ("xgeom_quat", _arr(d, NHAND, HAND_NXGEOM, 4)),
        ("xgeom_size", _arr(d, NHAND, HAND_NXGEOM, 3)), ("xgeom_rbound", _arr(d, NHAND, HAND_NXGEOM)),
        ("xgeom_vert", _arr(i32, NHAND, HAND_NXGEOM, 2)), ("hull_vert", _arr(d, NHAND, HAND_HULLVERT, 3)),
        ("n_xpairs", i32), ("xpair", _arr(i32, MAX_XPAIRS, 2)),
        ("dof_frictionloss", _arr(d, NHAND, HAND_NDOF)), ("friction_solref", _arr(d, 2)),
        ("friction_solimp", _arr(d, 5)), ("hand_gravcomp", d),
        ("dof_locked", _arr(i32, NHAND, HAND_NDOF)), ("n_obs_joints", _arr(i32, NHAND)),
        ("act_column", _arr(i32, NHAND, HAND_NACT)), ("n_action", i32),
    ]


class SongDesc(C.Structure):
    _fields_ = [("T", i32), ("goal", C.POINTER(C.c_float)), ("count", C.POINTER(i32)),
                ("keys", C.POINTER(i32)), ("fingers", C.POINTER(i32))]

    @classmethod
    def from_tables(cls, song) -> "SongDesc":
        """ps_song_desc over a music.SongTables; the contiguous host copies are kept alive on
        the returned struct (ps_create copies them to the device)."""
        import numpy as np

        sd = cls()
        sd._arrays = (np.ascontiguousarray(song.goal, np.float32), np.ascontiguousarray(song.count, np.int32),
                      np.ascontiguousarray(song.keys, np.int32), np.ascontiguousarray(song.fingers, np.int32))
        goal, count, keys, fingers = sd._arrays
        sd.T = int(song.T)
        sd.goal = goal.ctypes.data_as(C.POINTER(C.c_float))
        sd.count = count.ctypes.data_as(C.POINTER(i32))
        sd.keys = keys.ctypes.data_as(C.POINTER(i32))
        sd.fingers = fingers.ctypes.data_as(C.POINTER(i32))
        return sd


class TaskCfg(C.Structure):
    """ps_task_cfg; struct_size is set to the struct's size (include/pianosim.h: ps_create
    refuses a struct of another layout)."""
    _fields_ = [("struct_size", C.c_uint32), ("n_steps_lookahead", i32), ("fingering_reward", i32), ("forearm_reward", i32),
                ("wrong_press_termination", i32), ("energy_penalty_coef", d),
                ("solver_iterations", i32), ("max_contacts", i32), ("canonical_actions", i32),
                ("solver", i32), ("randomize_hand_positions", i32), ("solver_refine", i32)]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if "struct_size" not in kw:
            self.struct_size = C.sizeof(TaskCfg)


SOLVER_EXACT = SOLVER_NEWTON = 1
HAND_POSITION_OFFSET = 0.05  # piano_with_shadow_hands.py:46


def obs_joints(md: "ModelDesc" = None):
    """joints_pos entries per hand (26 each for the full hand)."""
    if md is None:
        return [HAND_NDOF] * NHAND
    return [md.n_obs_joints[h] or HAND_NDOF for h in range(NHAND)]


def obs_dim(cfg: TaskCfg, md: "ModelDesc" = None) -> int:
    """goal (L+1)*89 + fingering 10 (if enabled) + piano/state 88 + sustain 1 + the joints_pos
    entries of both hands (2*26 for the full hands)."""
    return (cfg.n_steps_lookahead + 1) * (NKEY + 1) + (10 if cfg.fingering_reward else 0) \
        + NKEY + 1 + sum(obs_joints(md))
