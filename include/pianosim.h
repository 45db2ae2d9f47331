/*
 * pianosim.h - C-ABI of the MI355X batched PianoWithShadowHands environment.
 *
 * The reference has no FFI for this path: its boundary is the Python VecEnv
 * `parallelized_base_v2.VectorizedPianoEnv` (parallelized_base_v2.py:21-67), whose
 * per-env work is dm_control `composer.Environment.step/reset` driving MuJoCo
 * `mj_step` on a `PianoWithShadowHands` task (robopianist/suite/tasks/
 * piano_with_shadow_hands.py:49-449). These entry points are what that VecEnv binds
 * (see INTEGRATION.md for the ctypes stub):
 *
 *   ps_create        <- VectorizedPianoEnv.__init__ (parallelized_base_v2.py:22-46):
 *                       builds N tasks + physics (tasks/base.py:45-197,
 *                       piano_with_shadow_hands.py:98-128).
 *   ps_reset         <- VectorizedPianoEnv.reset (parallelized_base_v2.py:48-51) ->
 *                       composer reset: mj_resetData + initialize_episode
 *                       (piano_with_shadow_hands.py:169-174, piano.py:145-152).
 *   ps_step          <- VectorizedPianoEnv.step (parallelized_base_v2.py:53-60) ->
 *                       before_step (:176-186), 10 x mj_step + Piano.after_substep
 *                       (piano.py:154-192), after_step (:188-204), observables
 *                       (:371-449), CompositeReward.compute (composite_reward.py:46-56),
 *                       termination (:213-220), auto-reset after LAST.
 *   ps_get_state /   <- physics.data.qpos/qvel/qacc_warmstart/ctrl + task._t_idx
 *   ps_set_state        (teacher-forced parity; no reference equivalent beyond
 *                       physics.set_state).
 *   ps_set_applied   <- physics.bind(joints).qfrc_applied (piano_with_shadow_hands_test.py:239).
 *   ps_reward_terms  <- CompositeReward.reward_terms (composite_reward.py:62-64).
 *   ps_musical_metrics <- MidiEvaluationWrapper (wrappers/evaluation.py:37-177): per-step
 *                       precision / recall / F1 of the key and sustain activations against
 *                       the notes of the step, averaged over each finished episode.
 *
 * Conventions: all array arguments of ps_reset/ps_step/ps_get_state/ps_set_state are
 * DEVICE pointers (e.g. torch-ROCm tensors' data_ptr()) and the calls are asynchronous
 * on the caller's HIP stream (`stream` = hipStream_t, NULL = default stream). Return
 * value 0 = OK, < 0 = error; ps_last_error() gives a thread-local message. No C++
 * exception crosses the ABI. One handle per device; handles are independent.
 */
#ifndef PIANOSIM_H
#define PIANOSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- fixed topology (robopianist: 88-key piano + 2 Shadow Hand E3M5 + 2 forearm DOFs) */
#define PS_NKEY 88          /* piano_constants.py:22 */
#define PS_NHAND 2          /* right, left (tasks/base.py:116-135) */
#define PS_HAND_NBODY 25    /* forearm + wrist + palm + 4x4 fingers(+lf metacarpal) + 5 thumb */
#define PS_HAND_NDOF 26     /* shadow_hand_constants.py:21 NQ=24, + forearm_tx/ty */
#define PS_HAND_NGEOM 20    /* authored capsule colliders per hand */
#define PS_HAND_NACT 22     /* shadow_hand_constants.py:22 NU=20, + 2 forearm position actuators */
#define PS_HAND_NTENDON 4   /* FFJ0, MFJ0, RFJ0, LFJ0 fixed tendons */
#define PS_NFINGER 5        /* fingertip sites th, ff, mf, rf, lf (shadow_hand_constants.py:33-40) */
#define PS_NV (PS_NKEY + PS_NHAND * PS_HAND_NDOF)     /* 140 */
#define PS_NU (PS_NHAND * PS_HAND_NACT)               /* 44 */
#define PS_NACTION (PS_NU + 1)                        /* 45: hands + sustain */
#define PS_MAX_CAPPAIRS 768 /* capsule-capsule candidate pairs after filtering */
/* Box and convex-hull hand colliders ("extra" geoms, beside the capsule slots): MuJoCo geom
 * types box and mesh (the Menagerie hand's palm boxes and distal meshes, shadow_hand.py:95,
 * 144-152). A mesh collides as the convex hull of its vertices, as in MuJoCo. */
#define PS_HAND_NXGEOM 12      /* extra colliders per hand */
#define PS_HULL_MAXVERT 64     /* vertices of one hull */
#define PS_HAND_HULLVERT 384   /* hull vertices per hand, all hulls */
#define PS_MAX_XPAIRS 1024     /* hand-hand candidate pairs that involve an extra collider */
#define PS_GEOM_NONE 0
#define PS_GEOM_BOX 1
#define PS_GEOM_HULL 2
#define PS_MAX_NOTES 16     /* notes per control step in the song tables */

/* Per-geom contact parameters (MuJoCo geom attributes). */
typedef struct {
  double solref[2];   /* timeconst, dampratio */
  double solimp[5];   /* d0, dwidth, width, midpoint, power */
  double friction;    /* sliding friction (condim 3, pyramidal) */
} ps_contact_param;

/* Compiled model ("mjModel" for this task), produced by the host model compiler
 * (diffusion-piano_amd/model.py). Lengths in metres, angles in radians. */
typedef struct {
  double timestep;          /* tasks/base.py:28 */
  int32_t n_substeps;       /* control 0.05 / physics 0.005 (tasks/base.py:28-31) */
  double gravity[3];
  /* piano keys (piano_mjcf.py:64-400), sorted by key number */
  double key_pos[PS_NKEY][3];      /* body position (world) */
  double key_half[PS_NKEY][3];     /* box half sizes */
  double key_anchor[PS_NKEY][3];   /* hinge position in the key body frame */
  double key_mass[PS_NKEY];
  double key_inertia[PS_NKEY];     /* moment of inertia about the hinge axis (no armature) */
  double key_armature[PS_NKEY];
  double key_damping[PS_NKEY];
  double key_stiffness[PS_NKEY];
  double key_springref[PS_NKEY];
  double key_range[PS_NKEY][2];
  double base_pos[3], base_half[3];  /* static piano base box */
  ps_contact_param piano_contact;
  double limit_solref[2], limit_solimp[5];
  /* hands: [0]=right, [1]=left. Bodies in MuJoCo tree order; parent -1 = world. */
  int32_t body_parent[PS_NHAND][PS_HAND_NBODY];
  double body_pos[PS_NHAND][PS_HAND_NBODY][3];   /* in parent frame */
  double body_quat[PS_NHAND][PS_HAND_NBODY][4];  /* w x y z, in parent frame */
  double body_mass[PS_NHAND][PS_HAND_NBODY];
  double body_ipos[PS_NHAND][PS_HAND_NBODY][3];  /* COM in body frame */
  double body_inertia[PS_NHAND][PS_HAND_NBODY][6]; /* about COM, body frame: xx yy zz xy xz yz */
  /* DOFs in MuJoCo qpos order (each hinge/slide at its body origin). */
  int32_t dof_body[PS_NHAND][PS_HAND_NDOF];
  int32_t dof_type[PS_NHAND][PS_HAND_NDOF];     /* 0 = hinge, 1 = slide */
  double dof_axis[PS_NHAND][PS_HAND_NDOF][3];   /* body frame */
  double dof_range[PS_NHAND][PS_HAND_NDOF][2];
  int32_t dof_limited[PS_NHAND][PS_HAND_NDOF];
  double dof_damping[PS_NHAND][PS_HAND_NDOF];
  double dof_armature[PS_NHAND][PS_HAND_NDOF];
  int32_t dof_obs_order[PS_NHAND][PS_HAND_NDOF]; /* joints_pos[i] = qpos[dof_obs_order[i]] */
  /* capsule colliders (body frame segment centre/axis); geom_body < 0: unused slot */
  int32_t geom_body[PS_NHAND][PS_HAND_NGEOM];
  double geom_pos[PS_NHAND][PS_HAND_NGEOM][3];
  double geom_axis[PS_NHAND][PS_HAND_NGEOM][3];
  double geom_halflen[PS_NHAND][PS_HAND_NGEOM];
  double geom_radius[PS_NHAND][PS_HAND_NGEOM];
  int32_t root_geom_count;   /* capsules [0, root_geom_count) belong to the root (forearm) body
                                (informational: the forearm reward tests the bodies) */
  ps_contact_param hand_contact;
  /* fingertip sites (shadow_hand.py:190-207) */
  int32_t site_body[PS_NHAND][PS_NFINGER];
  double site_pos[PS_NHAND][PS_NFINGER][3];
  /* fixed tendons J0 = J2 + J1 (two dofs each) */
  int32_t tendon_dof[PS_NHAND][PS_HAND_NTENDON][2];
  double tendon_coef[PS_NHAND][PS_HAND_NTENDON][2];
  /* position actuators: target = dof (kind 0) or tendon (kind 1) */
  int32_t act_kind[PS_NHAND][PS_HAND_NACT];
  int32_t act_target[PS_NHAND][PS_HAND_NACT];
  double act_kp[PS_NHAND][PS_HAND_NACT];
  double act_ctrlrange[PS_NHAND][PS_HAND_NACT][2];
  int32_t act_forcelimited[PS_NHAND][PS_HAND_NACT];
  double act_forcerange[PS_NHAND][PS_HAND_NACT][2];
  /* capsule-capsule candidate pairs (global geom index = hand*PS_HAND_NGEOM + g),
   * after MuJoCo's filtering (same body, parent-child, <exclude>) */
  int32_t n_cappairs;
  int32_t cappair[PS_MAX_CAPPAIRS][2];
  /* mj_setConst-style inverse weights at qpos0 (regulariser scale diagApprox of the soft
   * constraints): translational body mobility trace(Jp M^-1 Jp^T)/3 and diag(M^-1). */
  double key_body_invweight[PS_NKEY];
  double key_dof_invweight[PS_NKEY];
  double body_invweight[PS_NHAND][PS_HAND_NBODY];
  double dof_invweight[PS_NHAND][PS_HAND_NDOF];
  /* extra colliders (type PS_GEOM_NONE = unused slot). Frame in the body frame; box: half
   * sizes; hull: vertices [xgeom_vert[0], +xgeom_vert[1]) of hull_vert in the geom frame,
   * whose origin is the hull's centre (MuJoCo's mesh frame). rbound: bounding-sphere radius
   * about the geom origin. Global collider ids: capsule h*PS_HAND_NGEOM + g, extra
   * PS_NHAND*PS_HAND_NGEOM + h*PS_HAND_NXGEOM + i. */
  int32_t xgeom_type[PS_NHAND][PS_HAND_NXGEOM];
  int32_t xgeom_body[PS_NHAND][PS_HAND_NXGEOM];
  double xgeom_pos[PS_NHAND][PS_HAND_NXGEOM][3];
  double xgeom_quat[PS_NHAND][PS_HAND_NXGEOM][4];
  double xgeom_size[PS_NHAND][PS_HAND_NXGEOM][3];
  double xgeom_rbound[PS_NHAND][PS_HAND_NXGEOM];
  int32_t xgeom_vert[PS_NHAND][PS_HAND_NXGEOM][2];
  double hull_vert[PS_NHAND][PS_HAND_HULLVERT][3];
  /* hand-hand candidate pairs with at least one extra collider (a < b, global ids), after
   * MuJoCo's filtering; contacts of these follow the capsule-capsule ones */
  int32_t n_xpairs;
  int32_t xpair[PS_MAX_XPAIRS][2];
  /* joint friction loss (MuJoCo dof_frictionloss; the Menagerie hand's right_hand class sets
   * 0.01 on every joint): each dof with frictionloss > 0 adds one friction-loss constraint row
   * J = e_dof, |f| <= frictionloss, to every substep's constraint solve, with the reference
   * acceleration -b (J v) and regulariser from solreffriction / solimpfriction (MuJoCo's
   * defaults (0.02, 1) and (0.9, 0.95, 0.001, 0.5, 2) unless the XML sets them). */
  double dof_frictionloss[PS_NHAND][PS_HAND_NDOF];
  double friction_solref[2], friction_solimp[5];
  /* MuJoCo body gravcomp of every hand body (PianoTask(gravity_compensation=True),
   * tasks/base.py:185-186: mujoco_utils.physics_utils.compensate_gravity sets 1): a passive force
   * -gravcomp m g at each hand body's COM, i.e. the hands feel (1 - gravcomp) of the gravity */
  double hand_gravcomp;
  /* Joints the reference's hand does not have - PianoTask(reduced_action_space=True) removes
   * THJ5, THJ1 and LFJ5 (shadow_hand.py:73-79,164-183), forearm_dofs without forearm_tx /
   * forearm_ty leaves that slide out (shadow_hand.py:270-311): the dof slot stays in qpos / qvel,
   * held at 0 with no force, no constraint row and no Jacobian entry, so its child body rides its
   * parent rigidly at the joint's zero - MuJoCo's body without that joint. */
  int32_t dof_locked[PS_NHAND][PS_HAND_NDOF];
  int32_t n_obs_joints[PS_NHAND];  /* joints_pos entries: dof_obs_order[h][0 .. n) (0: PS_HAND_NDOF) */
  /* The caller's action row: n_action columns, the last one the sustain pedal; act_column[h][a]
   * = actuator a's column, -1 when the reference has no such actuator (no force). n_action = 0:
   * the full PS_NACTION layout (actuator h * PS_HAND_NACT + a in that column). */
  int32_t act_column[PS_NHAND][PS_HAND_NACT];
  int32_t n_action;
} ps_model_desc;

/* Song tables: NoteTrajectory in dense form (music.py:SongTables). */
typedef struct {
  int32_t T;
  const float* goal;       /* [T][89]: keys + sustain */
  const int32_t* count;    /* [T] */
  const int32_t* keys;     /* [T][PS_MAX_NOTES] */
  const int32_t* fingers;  /* [T][PS_MAX_NOTES], 0-4 right, 5-9 left */
} ps_song_desc;

/* Task options (piano_with_shadow_hands.py:50-66). The first field is the struct's size: a
 * caller sets struct_size = sizeof(ps_task_cfg) (= PS_TASK_CFG_SIZE of the header it was built
 * against) and ps_create / ps_obs_dim refuse any other value - a caller built against an older
 * header (before ps_version 4: no struct_size, no solver_refine) fails with "rebuild against
 * include/pianosim.h" instead of the library reading past the end of its struct. */
typedef struct {
  uint32_t struct_size;             /* sizeof(ps_task_cfg) */
  int32_t n_steps_lookahead;        /* goal rows = lookahead + 1 */
  int32_t fingering_reward;         /* 1: fingering reward + 'fingering' obs; 0: OT reward */
  int32_t forearm_reward;           /* 1: add forearm reward term */
  int32_t wrong_press_termination;
  double energy_penalty_coef;       /* 5e-3 */
  int32_t solver_iterations;        /* Newton iterations per substep at most (0: the default cap, 24);
                                       reaching it is counted (PS_STAT_ITER_CAP) */
  int32_t max_contacts;             /* per env, <= PS_MAX_CONTACTS_LIMIT */
  int32_t canonical_actions;        /* 1: ps_step actions are in [-1,1] and are rescaled to the
                                       spec as dm_env_wrappers.CanonicalSpecWrapper does */
  int32_t solver;                   /* PS_SOLVER_NEWTON (the only value) */
  int32_t randomize_hand_positions; /* piano_with_shadow_hands.py:64,491-499: each episode shifts
                                       both hands by the same U(-0.05, 0.05) m along y */
  int32_t solver_refine;            /* 0: the Newton solve ends when its line search ends in the
                                       Hessian's piece; 1 (TaskConfig's default since round 6): then
                                       one more (refining) Newton step in that piece on the substeps
                                       whose hands are coupled, 2: on every substep - the fp32 solve's
                                       error shrinks (teacher-forced qpos p99 against the fp64 checker
                                       ~1.5e-4 -> ~8e-5 on coupled states) at ~5% of the throughput
                                       (DESIGN.md section 5). A solve that ends in the previous
                                       substep's guessed piece (one checked step) is not refined. */
} ps_task_cfg;
#define PS_TASK_CFG_SIZE ((uint32_t)sizeof(ps_task_cfg))

/* Constraint solver. NEWTON (= EXACT, the only one): the minimiser of MuJoCo's primal
 * constraint problem over the accelerations (mj_solNewton: Newton directions from the
 * Hessian M + sum D J'J of the rows in their quadratic zone, exact line search), to fp32
 * (kernel) / 1e-13 (oracle) precision - the unique solution every MuJoCo solver converges
 * to. The round-1 truncated PGS (value 0) is retired; ps_create rejects it. */
#define PS_SOLVER_EXACT 1
#define PS_SOLVER_NEWTON 1
#define PS_HAND_POSITION_OFFSET 0.05  /* piano_with_shadow_hands.py:46 _POSITION_OFFSET */

#define PS_MAX_CONTACTS_LIMIT 24
/* Constraint rows are not capped: friction loss (one per hand dof with frictionloss), hand and
 * key limits, 4 pyramid edges per contact. */

/* Physics warnings (MuJoCo mjWARN_BADQPOS / BADQVEL / BADQACC): mj_checkPos / mj_checkVel at
 * the start of a substep and mj_checkAcc after its constraint solve find a non-finite value or
 * one beyond 1e10 in qpos / qvel / qacc; the env's physics is reset as mj_resetData does (qpos
 * = qpos0, qvel = qacc_warmstart = ctrl = qfrc_applied = 0; after a bad qacc the forward
 * dynamics is recomputed at the reset state) and the warning is counted (ps_warnings). */
#define PS_WARN_BADQPOS 0
#define PS_WARN_BADQVEL 1
#define PS_WARN_BADQACC 2
#define PS_NWARN 3

/* step_type values (dm_env.StepType) */
#define PS_FIRST 0
#define PS_MID 1
#define PS_LAST 2

/* Reward term slots of ps_reward_terms (CompositeReward insertion order). */
#define PS_TERM_KEY_PRESS 0
#define PS_TERM_SUSTAIN 1
#define PS_TERM_ENERGY 2
#define PS_TERM_FINGERING 3   /* fingering_reward or ot_fingering_reward */
#define PS_TERM_FOREARM 4
#define PS_NTERMS 5

/* Slots of ps_musical_metrics (MidiEvaluationWrapper.get_musical_metrics keys). */
#define PS_MUS_PRECISION 0
#define PS_MUS_RECALL 1
#define PS_MUS_F1 2
#define PS_MUS_SUSTAIN_PRECISION 3
#define PS_MUS_SUSTAIN_RECALL 4
#define PS_MUS_SUSTAIN_F1 5
#define PS_NMUSIC 6

/* Slots of ps_solver_stats: per env, over the substeps of its last step. */
#define PS_STAT_SOLVES 0        /* Newton iterations (Hessian factorizations), summed */
#define PS_STAT_CONTACT_CAP 1   /* substeps whose narrow phase found >= max_contacts contacts */
#define PS_STAT_ITER_CAP 2      /* substeps whose Newton solve stopped at its iteration cap */
#define PS_STAT_MAX_ROWS 3      /* most contact rows (4 pyramid edges per contact) of one
                                   substep; the solve's other rows - one friction-loss row per hand
                                   dof with frictionloss and the violated hand / key limits - are
                                   not counted here */
#define PS_STAT_COUPLED 4       /* substeps whose hands were coupled (hand-hand contact or a key
                                   touched by both hands): the C-block elimination after both
                                   hands' independent pivots */
#define PS_STAT_BAD_PIVOT 5     /* substeps with a non-positive Cholesky pivot (clamped) */
#define PS_STAT_MAX_CDOFS 6     /* most coupled ("C") dofs of both hands in one substep (the dofs
                                   the hand-hand rows act on; > 28 takes the whole-block solve) */
#define PS_NSTATS 7

typedef struct ps_env ps_env;

const char* ps_last_error(void);
int ps_version(void);
int ps_obs_dim(const ps_task_cfg* cfg);  /* the full hand (n_obs_joints = PS_HAND_NDOF) */
/* sizeof(ps_model_desc), for host-side layout checks. */
int ps_model_desc_size(void);

int ps_create(const ps_model_desc* model, const ps_song_desc* song, const ps_task_cfg* cfg,
              int n_envs, int device, uint64_t seed, ps_env** out);
void ps_destroy(ps_env* env);
/* The handle's observation width and action row width (the model's joints_pos entries and
 * actuators: the reference's VecEnv shapes, parallelized_base_v2.py:41-51). */
int ps_env_obs_dim(const ps_env* env);
int ps_env_action_dim(const ps_env* env);

/* Resets envs (all when env_mask == NULL, else where env_mask[i] != 0; device u8[N])
 * and writes their first observation into obs[N][obs_dim]. */
int ps_reset(ps_env* env, const uint8_t* env_mask, float* obs, void* stream);

/* action[N][ps_env_action_dim] (45 for the full hand) in spec units, or canonical [-1,1] units
 * when cfg.canonical_actions. Envs whose
 * previous step was LAST are reset instead and report PS_FIRST (reward 0, discount 1). */
int ps_step(ps_env* env, const float* action, float* obs, float* reward, float* discount,
            uint8_t* step_type, void* stream);

/* qpos/qvel/qacc_warmstart [N][140] (MuJoCo dof order: keys, right hand, left hand),
 * ctrl [N][44], sustain [N], t_idx [N], last [N] (1 if the previous step was LAST). */
int ps_get_state(ps_env* env, float* qpos, float* qvel, float* qacc_ws, float* ctrl,
                 float* sustain, int32_t* t_idx, uint8_t* last, void* stream);
int ps_set_state(ps_env* env, const float* qpos, const float* qvel, const float* qacc_ws,
                 const float* ctrl, const float* sustain, const int32_t* t_idx,
                 const uint8_t* last, void* stream);
/* Generalized applied force [N][140] added every substep until changed (NULL clears). */
int ps_set_applied(ps_env* env, const float* qfrc_applied, void* stream);
/* Per-term rewards of the last step, [N][PS_NTERMS]. */
int ps_reward_terms(ps_env* env, float* terms, void* stream);
/* Fingertip site positions after the last step/reset, [N][2][5][3] (right, left). */
int ps_fingertips(ps_env* env, float* xpos, void* stream);
/* Number of contacts after the last step/reset, [N]. */
int ps_contact_count(ps_env* env, int32_t* ncon, void* stream);

/* One contact of the task layer's final collision pass (physics.data.contact after the step):
 * position (world), frame (normal geom1 -> geom2, two tangents), signed distance (< 0:
 * penetration), kind (0 hand-key, 1 hand-base, 2 hand-hand), key index (kind 0), global
 * collider ids g1 (-1 for a key or the base) and g2. */
typedef struct {
  float pos[3], n[3], t1[3], t2[3], dist;
  int32_t kind, key, g1, g2;
} ps_contact;
/* Contact lists of each env's last step: ps_record_contacts(env, 1) makes the step kernel
 * keep them (off by default: ~70 B per contact of extra HBM writes); ps_contacts copies them
 * to out [N][PS_MAX_CONTACTS_LIMIT] (device; the first ncon of each env are valid), in the
 * order capsule-piano, capsule-capsule, box / hull-piano, box / hull hand-hand (round 6; the
 * checker's, oracle/pianosim_ref.c collide). No reference counterpart beyond
 * physics.data.contact; used for collision parity checks. */
int ps_record_contacts(ps_env* env, int on);
int ps_contacts(ps_env* env, ps_contact* out, void* stream);

/* Musical metrics of each env's LAST finished episode, [N][PS_NMUSIC] (per-step binary
 * precision / recall / F1 with zero_division = 1, as sklearn's precision_recall_fscore_support
 * in evaluation.py:114-177, averaged over the episode's steps), and the number of episodes
 * each env has finished since ps_create, [N]. Device pointers; either may be NULL. */
int ps_musical_metrics(ps_env* env, float* episode, int32_t* episodes, void* stream);

/* Solver / cap counters of each env's last step, [N][PS_NSTATS] int32 (device). No reference
 * counterpart: the evidence that the contact and row caps do not bind. */
int ps_solver_stats(ps_env* env, int32_t* stats, void* stream);

/* Physics warnings of each env since ps_create, [N][PS_NWARN] int32 (device): the counts of
 * mj_checkPos / mj_checkVel / mj_checkAcc resets (see PS_WARN_*). dm_control turns a new
 * warning into PhysicsError (Physics.check_invalid_state); envs.Environment does the same. */
int ps_warnings(ps_env* env, int32_t* warnings, void* stream);

/* Episode-return bookkeeping of a rollout loop in one launch (the reference driver's per-env
 * return sums, parallelized_base_v2.py / ppo_v2.py training loops): after a step with rewards
 * reward[n] and step types step_type[n] (uint8), running[i] (f64) restarts at a FIRST step and
 * accumulates the reward otherwise; at a LAST step last_return[i] (f32) takes it and it is added
 * to *finished_sum (f64) and *finished_count (int64). Device pointers; no env handle. */
int ps_episode_returns(const float* reward, const uint8_t* step_type, int n, double* running, float* last_return,
                       double* finished_sum, int64_t* finished_count, void* stream);

/* randomize_hand_positions (piano_with_shadow_hands.py:491-499): each env's current y shift of
 * both hand roots [N] f32 and its resets so far [N] i32 (device; either may be NULL). The set
 * form overrides the shift until the env's next reset (teacher-forced parity). */
int ps_get_hand_offset(ps_env* env, float* dy, int32_t* episodes, void* stream);
int ps_set_hand_offset(ps_env* env, const float* dy, void* stream);

/* Global id of this handle's env 0 when the envs of one job are sharded over handles/GPUs
 * (default 0). Every per-env random draw (the randomize_hand_positions Philox stream) is keyed
 * by (seed, global env id, episode), so a global env draws the same values at any world size
 * ("Philox streams are keyed by global env id"). */
int ps_set_env_offset(ps_env* env, int64_t global_first_env);

#ifdef __cplusplus
}
#endif
#endif
