/*
 * pianosim_ref.c - CPU fp64 ORACLE for the batched PianoWithShadowHands step.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker / CPU baseline. The product (libpianosim.so, HIP) never
 * links or calls this file.
 *
 * Plain sequential restatement of the reference path, one env at a time:
 *   - task layer: robopianist/suite/tasks/piano_with_shadow_hands.py:176-449,
 *     robopianist/models/piano/piano.py:154-192, composite_reward.py:46-56,
 *     shadow_hand.py:380-416, dm_control composer.Environment.step hook order and
 *     dm_control.utils.rewards.tolerance (gaussian, value_at_margin=0.1);
 *   - physics: MuJoCo's documented mj_step pipeline for hinge/slide trees (the engine
 *     itself is an absent third-party dependency, `mujoco>=3.1.1`, setup.py:62):
 *     kinematics, composite-rigid-body mass matrix + armature, tree LDL (mj_factorI /
 *     mj_solveLD), recursive Newton-Euler bias, passive spring/damper, position
 *     actuators (joint + fixed tendon), collision, soft constraints (solref/solimp,
 *     refsafe), pyramidal friction cones, PGS dual solve (cold start, fixed sweeps),
 *     Euler with implicit joint damping (mj_EulerSkip).
 * Parity status: the task layer is pinned by the reference tests' known answers and the
 * golden song fixtures (tests/golden/); the physics is "parity unpinned" against MuJoCo
 * (no mujoco/dm_control/Menagerie in this container, no reference test records numeric
 * physics state): it is the specification the HIP kernel is checked against.
 * Deviations from MuJoCo defaults are listed in DESIGN.md ("Physics specification").
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include "../include/pianosim.h"

#define NK PS_NKEY
#define NH PS_NHAND
#define NB PS_HAND_NBODY
#define ND PS_HAND_NDOF
#define NG PS_HAND_NGEOM
#define NA PS_HAND_NACT
#define NX PS_HAND_NXGEOM
#define NCAPS (NH * NG)  /* global collider ids: capsules [0, NCAPS), extras NCAPS + h * NX + i */
#define NV PS_NV
#define MAXCON PS_MAX_CONTACTS_LIMIT
#define MINIMP 0.0001
#define MAXIMP 0.9999
#define MINVAL 1e-15
#define KEY_THRESHOLD 0.00872665   /* piano.py:31 */
#define SUSTAIN_THRESHOLD 0.5      /* piano.py:32 */

typedef struct { double v[3]; } v3;

static inline v3 mk(double a, double b, double c) { v3 r = {{a, b, c}}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]); }
static inline v3 sub(v3 a, v3 b) { return mk(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]); }
static inline v3 scl(v3 a, double s) { return mk(a.v[0] * s, a.v[1] * s, a.v[2] * s); }
static inline double dot(v3 a, v3 b) { return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2]; }
static inline v3 crs(v3 a, v3 b) {
  return mk(a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2],
            a.v[0] * b.v[1] - a.v[1] * b.v[0]);
}
static inline double nrm(v3 a) { return sqrt(dot(a, a)); }
static inline double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
/* the model's action row and joints_pos layout (ps_model_desc n_action / act_column /
 * n_obs_joints; 0 = the full hand) */
static inline int n_action(const ps_model_desc* d) { return d->n_action > 0 ? d->n_action : PS_NACTION; }
static inline int act_col(const ps_model_desc* d, int h, int a) {
  return d->n_action > 0 ? d->act_column[h][a] : h * PS_HAND_NACT + a;
}
static inline int act_present(const ps_model_desc* d, int h, int a) { return act_col(d, h, a) >= 0; }
static inline int n_obs_joints(const ps_model_desc* d, int h) {
  return d->n_obs_joints[h] ? d->n_obs_joints[h] : PS_HAND_NDOF;
}

typedef struct { double m[9]; } m3;  /* row-major */
static inline v3 mv(m3 R, v3 a) {
  return mk(R.m[0] * a.v[0] + R.m[1] * a.v[1] + R.m[2] * a.v[2],
            R.m[3] * a.v[0] + R.m[4] * a.v[1] + R.m[5] * a.v[2],
            R.m[6] * a.v[0] + R.m[7] * a.v[1] + R.m[8] * a.v[2]);
}
static inline v3 mtv(m3 R, v3 a) {
  return mk(R.m[0] * a.v[0] + R.m[3] * a.v[1] + R.m[6] * a.v[2],
            R.m[1] * a.v[0] + R.m[4] * a.v[1] + R.m[7] * a.v[2],
            R.m[2] * a.v[0] + R.m[5] * a.v[1] + R.m[8] * a.v[2]);
}
static m3 mm(m3 A, m3 B) {
  m3 C;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
  return C;
}
static m3 quat2mat(const double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  double w = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
  m3 R = {{1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
           2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
           2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)}};
  return R;
}
/* Rotation by angle t about unit axis a (Rodrigues). */
static m3 axisangle(v3 a, double t) {
  double s = sin(t), c = cos(t), C1 = 1 - c;
  double x = a.v[0], y = a.v[1], z = a.v[2];
  m3 R = {{c + x * x * C1, x * y * C1 - z * s, x * z * C1 + y * s,
           y * x * C1 + z * s, c + y * y * C1, y * z * C1 - x * s,
           z * x * C1 - y * s, z * y * C1 + x * s, c + z * z * C1}};
  return R;
}

/* ------------------------------------------------------------------ model (derived) */
typedef struct {
  ps_model_desc d;
  int dof_parent[NH][ND];     /* MuJoCo dof_parentid within the hand */
  int body_dofadr[NH][NB];    /* first dof of the body, -1 if none */
  int body_dofnum[NH][NB];
  double key_y_lo[NK], key_y_hi[NK];
} model;

static void derive(model* m) {
  for (int h = 0; h < NH; h++) {
    for (int b = 0; b < NB; b++) { m->body_dofadr[h][b] = -1; m->body_dofnum[h][b] = 0; }
    for (int j = 0; j < ND; j++) {
      int b = m->d.dof_body[h][j];
      if (m->body_dofadr[h][b] < 0) m->body_dofadr[h][b] = j;
      m->body_dofnum[h][b]++;
    }
    for (int j = 0; j < ND; j++) {
      int b = m->d.dof_body[h][j];
      if (j > m->body_dofadr[h][b]) { m->dof_parent[h][j] = j - 1; continue; }
      int p = m->d.body_parent[h][b], par = -1;
      while (p >= 0) {
        if (m->body_dofnum[h][p] > 0) { par = m->body_dofadr[h][p] + m->body_dofnum[h][p] - 1; break; }
        p = m->d.body_parent[h][p];
      }
      m->dof_parent[h][j] = par;
    }
  }
  for (int k = 0; k < NK; k++) {
    m->key_y_lo[k] = m->d.key_pos[k][1] - m->d.key_half[k][1];
    m->key_y_hi[k] = m->d.key_pos[k][1] + m->d.key_half[k][1];
  }
}

/* ------------------------------------------------------------------ per-env data */
typedef struct {
  int kind;          /* 0 hand-key, 1 hand-base, 2 capsule-capsule */
  int key;           /* key index for kind 0 */
  int h1, b1;        /* side 1: hand/body (kind 2) */
  int h2, b2;        /* side 2: hand/body of the capsule (geom2) */
  int g1, g2;        /* global geom ids (kind 2: both; kind 0/1: g2 only) */
  int sub;           /* capsule-box: 0/1 = endpoint sphere, 2 = segment point; kind 2: 0 */
  v3 pos, n, t1, t2;
  double dist;
} contact;

typedef struct {
  /* state */
  double q[NV], v[NV], qacc_ws[NV], ctrl[PS_NU], sustain, applied[NV];
  int t_idx, last;
  double hand_dy;  /* randomize_hand_positions: this episode's y shift of both hand roots */
  int episode;     /* resets so far (the draw counter of hand_dy) */
  /* MidiEvaluationWrapper (wrappers/evaluation.py): sums of the per-step metrics of the
   * running episode, the last finished episode's means, finished-episode count */
  double mus_acc[PS_NMUSIC], mus_ep[PS_NMUSIC];
  int mus_cnt;
  /* kinematics */
  m3 R[NH][NB];
  v3 o[NH][NB], com[NH][NB], axis[NH][ND];
  double Iw[NH][NB][9];
  v3 cap0[NH][NG], cap1[NH][NG];
  v3 xc[NH][NX];   /* extra colliders: world frame origin and rotation */
  m3 xR[NH][NX];
  m3 keyR[NK];
  v3 keyc[NK], keyanchor[NK];
  /* dynamics */
  double M[NH][ND][ND], Mh[NH][ND][ND], D[NH][ND], Dh[NH][ND];
  double Mfull[NH][ND][ND];  /* the hand mass matrices before factorization (the Newton Hessian) */
  double Mk[NK], Mkh[NK];
  double bias[NV], passive[NV], actfrc[NV], act_force[PS_NU];
  int warnings[PS_NWARN];  /* mj_checkPos / Vel / Acc resets since create (ps_warnings) */
  /* collision */
  int ncon, nfound;
  contact con[MAXCON];
  /* outputs */
  double terms[PS_NTERMS];
  double norm_state[NK];
  int activation[NK];
} envdata;

struct ref_env {
  model m;
  ps_task_cfg cfg;
  int T;
  float* goal;
  int32_t *count, *keys, *fingers;
  int n;
  uint64_t seed;
  int64_t env_offset;  /* global id of env 0 */
  envdata* e;
};
typedef struct ref_env ref_env;

/* Philox4x32-10 (Salmon et al., SC'11), the counter-based generator of the HIP side. */
static uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = mulhi32(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    uint32_t hi1 = mulhi32(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
/* _randomize_initial_hand_positions (piano_with_shadow_hands.py:491-499):
 * offset = random_state.uniform(-_POSITION_OFFSET, _POSITION_OFFSET), the same for both hands
 * (shift_pose (0, offset, 0)). The reference draws from the episode's numpy RandomState; here
 * the draw is counter-based, keyed by (seed, env, episode), in float: u = 24 random bits /
 * 2^24, offset = fma(2 * 0.05, u, -0.05). */
float ref_hand_offset_draw(uint64_t seed, int env, int episode) {
  uint32_t c[4] = {(uint32_t)episode, (uint32_t)env, 0x68616e64u /* "hand" */, 0u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u = (float)(c[0] >> 8) * 0x1p-24f;
  return fmaf((float)(2.0 * PS_HAND_POSITION_OFFSET), u, (float)-PS_HAND_POSITION_OFFSET);
}

/* ------------------------------------------------------------------ kinematics */
static void kinematics(const model* m, envdata* E) {
  const ps_model_desc* d = &m->d;
  for (int h = 0; h < NH; h++) {
    const double* qh = E->q + NK + h * ND;
    for (int b = 0; b < NB; b++) {
      int p = d->body_parent[h][b];
      m3 Q = quat2mat(d->body_quat[h][b]);
      v3 pos = mk(d->body_pos[h][b][0], d->body_pos[h][b][1], d->body_pos[h][b][2]);
      m3 R;
      v3 o;
      if (p < 0) { R = Q; o = pos; o.v[1] += E->hand_dy; }
      else { R = mm(E->R[h][p], Q); o = add(E->o[h][p], mv(E->R[h][p], pos)); }
      for (int j = m->body_dofadr[h][b]; j >= 0 && j < m->body_dofadr[h][b] + m->body_dofnum[h][b]; j++) {
        v3 al = mk(d->dof_axis[h][j][0], d->dof_axis[h][j][1], d->dof_axis[h][j][2]);
        if (d->dof_type[h][j] == 1) {
          v3 aw = mv(R, al);
          E->axis[h][j] = aw;
          o = add(o, scl(aw, qh[j]));
        } else {
          R = mm(R, axisangle(al, qh[j]));
          E->axis[h][j] = mv(R, al);
        }
      }
      E->R[h][b] = R;
      E->o[h][b] = o;
      v3 ip = mk(d->body_ipos[h][b][0], d->body_ipos[h][b][1], d->body_ipos[h][b][2]);
      E->com[h][b] = add(o, mv(R, ip));
      /* world inertia about COM: R I R^T */
      const double* I6 = d->body_inertia[h][b];
      double Il[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
      double tmp[9];
      for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) {
          double s = 0;
          for (int l = 0; l < 3; l++) s += R.m[3 * i + l] * Il[3 * l + k];
          tmp[3 * i + k] = s;
        }
      for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) {
          double s = 0;
          for (int l = 0; l < 3; l++) s += tmp[3 * i + l] * R.m[3 * k + l];
          E->Iw[h][b][3 * i + k] = s;
        }
    }
    for (int g = 0; g < NG; g++) {
      int b = d->geom_body[h][g];
      if (b < 0) continue;  /* unused slot */
      v3 c = add(E->o[h][b], mv(E->R[h][b], mk(d->geom_pos[h][g][0], d->geom_pos[h][g][1], d->geom_pos[h][g][2])));
      v3 a = mv(E->R[h][b], mk(d->geom_axis[h][g][0], d->geom_axis[h][g][1], d->geom_axis[h][g][2]));
      E->cap0[h][g] = sub(c, scl(a, d->geom_halflen[h][g]));
      E->cap1[h][g] = add(c, scl(a, d->geom_halflen[h][g]));
    }
    for (int i = 0; i < NX; i++) {
      if (d->xgeom_type[h][i] == PS_GEOM_NONE) continue;
      int b = d->xgeom_body[h][i];
      E->xc[h][i] = add(E->o[h][b], mv(E->R[h][b], mk(d->xgeom_pos[h][i][0], d->xgeom_pos[h][i][1], d->xgeom_pos[h][i][2])));
      E->xR[h][i] = mm(E->R[h][b], quat2mat(d->xgeom_quat[h][i]));
    }
  }
  for (int k = 0; k < NK; k++) {
    double q = E->q[k], c = cos(q), s = sin(q);
    m3 R = {{c, 0, s, 0, 1, 0, -s, 0, c}};  /* rotation about +y */
    v3 P = mk(d->key_pos[k][0], d->key_pos[k][1], d->key_pos[k][2]);
    v3 al = mk(d->key_anchor[k][0], d->key_anchor[k][1], d->key_anchor[k][2]);
    v3 A = add(P, al);
    E->keyR[k] = R;
    E->keyanchor[k] = A;
    E->keyc[k] = add(A, mv(R, scl(al, -1.0)));
  }
}

static v3 site_pos(const model* m, const envdata* E, int h, int s) {
  const ps_model_desc* d = &m->d;
  int b = d->site_body[h][s];
  return add(E->o[h][b], mv(E->R[h][b], mk(d->site_pos[h][s][0], d->site_pos[h][s][1], d->site_pos[h][s][2])));
}

/* ------------------------------------------------------------------ mass matrix + bias */
static void dynamics(const model* m, const ps_task_cfg* cfg, envdata* E) {
  (void)cfg;
  const ps_model_desc* d = &m->d;
  const double h_t = d->timestep;
  v3 g = mk(d->gravity[0], d->gravity[1], d->gravity[2]);
  for (int h = 0; h < NH; h++) {
    const double* vh = E->v + NK + h * ND;
    /* composite inertia about each body origin */
    double ms[NB];
    v3 hh[NB];
    double Is[NB][9];
    for (int b = 0; b < NB; b++) {
      double mass = d->body_mass[h][b];
      v3 dd = sub(E->com[h][b], E->o[h][b]);
      ms[b] = mass;
      hh[b] = scl(dd, mass);
      double d2 = dot(dd, dd);
      for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++)
          Is[b][3 * i + k] = E->Iw[h][b][3 * i + k] + mass * ((i == k ? d2 : 0.0) - dd.v[i] * dd.v[k]);
    }
    for (int b = NB - 1; b > 0; b--) {
      int p = d->body_parent[h][b];
      v3 r = sub(E->o[h][b], E->o[h][p]);
      double r2 = dot(r, r), rh = dot(r, hh[b]);
      for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++)
          Is[p][3 * i + k] += Is[b][3 * i + k] + ms[b] * ((i == k ? r2 : 0.0) - r.v[i] * r.v[k]) +
                              ((i == k ? 2 * rh : 0.0) - r.v[i] * hh[b].v[k] - hh[b].v[i] * r.v[k]);
      hh[p] = add(hh[p], add(hh[b], scl(r, ms[b])));
      ms[p] += ms[b];
    }
    /* M[i][j] for j ancestor-or-self of i */
    memset(E->M[h], 0, sizeof(E->M[h]));
    for (int i = 0; i < ND; i++) {
      int bi = d->dof_body[h][i];
      v3 ai = E->axis[h][i], flin, fang;
      if (d->dof_type[h][i] == 0) {
        flin = crs(ai, hh[bi]);
        fang = mk(Is[bi][0] * ai.v[0] + Is[bi][1] * ai.v[1] + Is[bi][2] * ai.v[2],
                  Is[bi][3] * ai.v[0] + Is[bi][4] * ai.v[1] + Is[bi][5] * ai.v[2],
                  Is[bi][6] * ai.v[0] + Is[bi][7] * ai.v[1] + Is[bi][8] * ai.v[2]);
      } else {
        flin = scl(ai, ms[bi]);
        fang = crs(hh[bi], ai);
      }
      for (int j = i; j >= 0; j = m->dof_parent[h][j]) {
        int bj = d->dof_body[h][j];
        v3 aj = E->axis[h][j];
        double val;
        if (d->dof_type[h][j] == 0) val = dot(aj, add(fang, crs(sub(E->o[h][bi], E->o[h][bj]), flin)));
        else val = dot(aj, flin);
        E->M[h][i][j] = val;
        E->M[h][j][i] = val;
      }
      E->M[h][i][i] += d->dof_armature[h][i];
    }
    /* a locked dof (a joint the reference's hand lacks): identity row and column */
    for (int i = 0; i < ND; i++)
      if (d->dof_locked[h][i]) {
        for (int j = 0; j < ND; j++) E->M[h][i][j] = E->M[h][j][i] = 0.0;
        E->M[h][i][i] = 1.0;
      }
    /* bias forces: RNE, gravity as base acceleration */
    v3 w[NB], al[NB], vo[NB], ac[NB], F[NB], N[NB];
    for (int b = 0; b < NB; b++) {
      int p = d->body_parent[h][b];
      if (p < 0) {
        w[b] = mk(0, 0, 0);
        al[b] = mk(0, 0, 0);
        vo[b] = mk(0, 0, 0);
        for (int j = m->body_dofadr[h][b]; j >= 0 && j < m->body_dofadr[h][b] + m->body_dofnum[h][b]; j++)
          vo[b] = add(vo[b], scl(E->axis[h][j], vh[j]));
        ac[b] = scl(g, -(1.0 - d->hand_gravcomp));  /* body gravcomp cancels that share (tasks/base.py:185-186) */
      } else {
        v3 r = sub(E->o[h][b], E->o[h][p]);
        w[b] = w[p];
        al[b] = al[p];
        vo[b] = add(vo[p], crs(w[p], r));
        ac[b] = add(ac[p], add(crs(al[p], r), crs(w[p], crs(w[p], r))));
        int j = m->body_dofadr[h][b];  /* one hinge per non-root body */
        v3 a = E->axis[h][j];
        al[b] = add(al[b], scl(crs(w[p], a), vh[j]));
        w[b] = add(w[b], scl(a, vh[j]));
      }
      v3 dd = sub(E->com[h][b], E->o[h][b]);
      v3 acom = add(ac[b], add(crs(al[b], dd), crs(w[b], crs(w[b], dd))));
      F[b] = scl(acom, d->body_mass[h][b]);
      const double* I = E->Iw[h][b];
      v3 Ia = mk(I[0] * al[b].v[0] + I[1] * al[b].v[1] + I[2] * al[b].v[2],
                 I[3] * al[b].v[0] + I[4] * al[b].v[1] + I[5] * al[b].v[2],
                 I[6] * al[b].v[0] + I[7] * al[b].v[1] + I[8] * al[b].v[2]);
      v3 Iw = mk(I[0] * w[b].v[0] + I[1] * w[b].v[1] + I[2] * w[b].v[2],
                 I[3] * w[b].v[0] + I[4] * w[b].v[1] + I[5] * w[b].v[2],
                 I[6] * w[b].v[0] + I[7] * w[b].v[1] + I[8] * w[b].v[2]);
      N[b] = add(add(Ia, crs(w[b], Iw)), crs(dd, F[b]));  /* about body origin */
    }
    for (int b = NB - 1; b > 0; b--) {
      int p = d->body_parent[h][b];
      v3 r = sub(E->o[h][b], E->o[h][p]);
      N[p] = add(N[p], add(N[b], crs(r, F[b])));
      F[p] = add(F[p], F[b]);
    }
    for (int j = 0; j < ND; j++) {
      int b = d->dof_body[h][j];
      E->bias[NK + h * ND + j] = d->dof_type[h][j] == 0 ? dot(E->axis[h][j], N[b]) : dot(E->axis[h][j], F[b]);
      E->passive[NK + h * ND + j] = -d->dof_damping[h][j] * vh[j];
    }
  }
  for (int k = 0; k < NK; k++) {
    v3 r = sub(E->keyc[k], E->keyanchor[k]);
    /* generalized gravity force about +y: (r x m g).y ; bias = -that */
    E->bias[k] = -d->key_mass[k] * (r.v[2] * g.v[0] - r.v[0] * g.v[2]);
    E->passive[k] = -d->key_stiffness[k] * (E->q[k] - d->key_springref[k]) - d->key_damping[k] * E->v[k];
    E->Mk[k] = d->key_inertia[k] + d->key_armature[k];
    E->Mkh[k] = E->Mk[k] + h_t * d->key_damping[k];
  }
  /* actuation (mj_fwdActuation: ctrl clamped to ctrlrange, force clamped to forcerange) */
  memset(E->actfrc, 0, sizeof(E->actfrc));
  for (int h = 0; h < NH; h++) {
    const double* qh = E->q + NK + h * ND;
    for (int a = 0; a < NA; a++) {
      double len;
      int tg = d->act_target[h][a];
      if (d->act_kind[h][a] == 0) len = qh[tg];
      else len = d->tendon_coef[h][tg][0] * qh[d->tendon_dof[h][tg][0]] + d->tendon_coef[h][tg][1] * qh[d->tendon_dof[h][tg][1]];
      double c = clampd(E->ctrl[h * NA + a], d->act_ctrlrange[h][a][0], d->act_ctrlrange[h][a][1]);
      double f = act_present(d, h, a) ? d->act_kp[h][a] * (c - len) : 0.0;
      if (d->act_forcelimited[h][a]) f = clampd(f, d->act_forcerange[h][a][0], d->act_forcerange[h][a][1]);
      E->act_force[h * NA + a] = f;
      if (d->act_kind[h][a] == 0) E->actfrc[NK + h * ND + tg] += f;
      else {
        E->actfrc[NK + h * ND + d->tendon_dof[h][tg][0]] += d->tendon_coef[h][tg][0] * f;
        E->actfrc[NK + h * ND + d->tendon_dof[h][tg][1]] += d->tendon_coef[h][tg][1] * f;
      }
    }
  }
}

/* mj_factorI on the tree-sparse hand matrix (in place: L below diag, D separately) */
static void factor(const model* m, int h, double A[ND][ND], double* D) {
  for (int k = ND - 1; k >= 0; k--) {
    if (A[k][k] < MINVAL) A[k][k] = MINVAL;
    for (int i = m->dof_parent[h][k]; i >= 0; i = m->dof_parent[h][i]) {
      double tmp = A[k][i] / A[k][k];
      for (int j = i; j >= 0; j = m->dof_parent[h][j]) A[i][j] -= tmp * A[k][j];
      A[k][i] = tmp;
    }
  }
  for (int k = 0; k < ND; k++) D[k] = A[k][k];
}

/* x <- L^-T x (first phase of mj_solveLD) */
static void solve_LT(const model* m, int h, double A[ND][ND], double* x) {
  for (int k = ND - 1; k >= 0; k--)
    for (int i = m->dof_parent[h][k]; i >= 0; i = m->dof_parent[h][i]) x[i] -= A[k][i] * x[k];
}
/* x <- L^-1 x (last phase) */
static void solve_L(const model* m, int h, double A[ND][ND], double* x) {
  for (int k = 0; k < ND; k++)
    for (int i = m->dof_parent[h][k]; i >= 0; i = m->dof_parent[h][i]) x[k] -= A[k][i] * x[i];
}
static void solve_full(const model* m, envdata* E, int implicit, const double* b, double* x) {
  memcpy(x, b, sizeof(double) * NV);
  for (int k = 0; k < NK; k++) x[k] /= implicit ? E->Mkh[k] : E->Mk[k];
  for (int h = 0; h < NH; h++) {
    double* xh = x + NK + h * ND;
    double(*A)[ND] = implicit ? E->Mh[h] : E->M[h];
    double* D = implicit ? E->Dh[h] : E->D[h];
    solve_LT(m, h, A, xh);
    for (int k = 0; k < ND; k++) xh[k] /= D[k];
    solve_L(m, h, A, xh);
  }
}

/* ------------------------------------------------------------------ collision */
static void make_frame(v3 n, v3* t1, v3* t2) {
  v3 e = fabs(n.v[2]) < 0.5 ? mk(0, 0, 1) : mk(1, 0, 0);
  v3 a = crs(n, e);
  *t1 = scl(a, 1.0 / nrm(a));
  *t2 = crs(n, *t1);
}

/* point (world) vs box: signed distance, normal box->point, contact midpoint */
static double sphere_box(v3 p, double r, v3 c, m3 R, const double* hs, v3* nout, v3* posout) {
  v3 pl = mtv(R, sub(p, c));
  v3 q;
  int outside = 0;
  for (int i = 0; i < 3; i++) {
    q.v[i] = clampd(pl.v[i], -hs[i], hs[i]);
    if (q.v[i] != pl.v[i]) outside = 1;
  }
  v3 n, mid;
  double dist;
  if (outside) {
    v3 dv = sub(pl, q);
    double dn = nrm(dv);
    n = scl(dv, 1.0 / dn);
    dist = dn - r;
    mid = add(q, scl(n, 0.5 * dist));
  } else {
    int ax = 0;
    double best = hs[0] - fabs(pl.v[0]);
    for (int i = 1; i < 3; i++) {
      double s = hs[i] - fabs(pl.v[i]);
      if (s < best) { best = s; ax = i; }
    }
    n = mk(0, 0, 0);
    n.v[ax] = pl.v[ax] >= 0 ? 1.0 : -1.0;
    dist = -best - r;
    mid = add(pl, scl(n, 0.5 * (best - r)));
  }
  *nout = mv(R, n);
  *posout = add(c, mv(R, mid));
  return dist;
}

/* argmin over t in [0,1] of the outside distance of segment a + t d to the box */
static double seg_box_t(v3 a, v3 dv, const double* hs) {
  double bp[8];
  int nb = 0;
  bp[nb++] = 0.0;
  for (int i = 0; i < 3; i++) {
    if (dv.v[i] == 0.0) continue;
    for (int sgn = -1; sgn <= 1; sgn += 2) {
      double t = (sgn * hs[i] - a.v[i]) / dv.v[i];
      if (t > 0.0 && t < 1.0) bp[nb++] = t;
    }
  }
  bp[nb++] = 1.0;
  for (int i = 1; i < nb; i++)  /* insertion sort */
    for (int j = i; j > 0 && bp[j] < bp[j - 1]; j--) { double t = bp[j]; bp[j] = bp[j - 1]; bp[j - 1] = t; }
  double bestf = INFINITY, bestt = 0.0;
  for (int s = 0; s + 1 < nb; s++) {
    double lo = bp[s], hi = bp[s + 1];
    if (!(hi > lo)) continue;
    double mid = 0.5 * (lo + hi), num = 0.0, den = 0.0;
    for (int i = 0; i < 3; i++) {
      double x = a.v[i] + mid * dv.v[i];
      double tgt = x > hs[i] ? hs[i] : (x < -hs[i] ? -hs[i] : 0.0);
      if (tgt == 0.0 && fabs(x) <= hs[i]) continue;
      num -= (a.v[i] - tgt) * dv.v[i];
      den += dv.v[i] * dv.v[i];
    }
    double t = den > 0.0 ? clampd(num / den, lo, hi) : lo;
    double f = 0.0;
    for (int i = 0; i < 3; i++) {
      double e = fabs(a.v[i] + t * dv.v[i]) - hs[i];
      if (e > 0) f += e * e;
    }
    if (f < bestf) { bestf = f; bestt = t; }
  }
  if (bestf <= 0.0) {  /* intersecting: midpoint of the slab-clipped interval */
    double tin = 0.0, tout = 1.0;
    int empty = 0;
    for (int i = 0; i < 3; i++) {
      if (fabs(dv.v[i]) < 1e-12) {
        if (fabs(a.v[i]) > hs[i]) empty = 1;
        continue;
      }
      double t1 = (-hs[i] - a.v[i]) / dv.v[i], t2 = (hs[i] - a.v[i]) / dv.v[i];
      if (t1 > t2) { double t = t1; t1 = t2; t2 = t; }
      if (t1 > tin) tin = t1;
      if (t2 < tout) tout = t2;
    }
    if (!empty && tin <= tout) bestt = 0.5 * (tin + tout);
  }
  return bestt;
}

static int add_contact(envdata* E, int maxc, const contact* c) {
  E->nfound++;  /* every contact the narrow phase reports, kept or beyond the cap */
  if (E->ncon >= maxc) return 0;
  E->con[E->ncon++] = *c;
  return 1;
}

/* capsule (geom2) vs box (geom1): up to 2 contacts, normal box -> capsule */
static void capsule_box(envdata* E, int maxc, contact proto, v3 p0, v3 p1, double r, v3 c, m3 R, const double* hs) {
  v3 n, pos;
  int found = 0;
  for (int e = 0; e < 2; e++) {
    double dist = sphere_box(e == 0 ? p0 : p1, r, c, R, hs, &n, &pos);
    if (dist <= 0.0) {
      contact cc = proto;
      cc.pos = pos; cc.n = n; cc.dist = dist; cc.sub = e;
      make_frame(n, &cc.t1, &cc.t2);
      add_contact(E, maxc, &cc);
      found = 1;
    }
  }
  if (found) return;
  v3 a = mtv(R, sub(p0, c)), b = mtv(R, sub(p1, c));
  double t = seg_box_t(a, sub(b, a), hs);
  v3 p = add(p0, scl(sub(p1, p0), t));
  double dist = sphere_box(p, r, c, R, hs, &n, &pos);
  if (dist <= 0.0) {
    contact cc = proto;
    cc.pos = pos; cc.n = n; cc.dist = dist; cc.sub = 2;
    make_frame(n, &cc.t1, &cc.t2);
    add_contact(E, maxc, &cc);
  }
}

/* closest points between segments p1-q1 and p2-q2 (Ericson, RTCD 5.1.9) */
static void seg_seg(v3 p1, v3 q1, v3 p2, v3 q2, v3* c1, v3* c2) {
  v3 d1 = sub(q1, p1), d2 = sub(q2, p2), r = sub(p1, p2);
  double a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r), s, t;
  const double eps = 1e-12;
  if (a <= eps && e <= eps) { s = t = 0; }
  else if (a <= eps) { s = 0; t = clampd(f / e, 0, 1); }
  else {
    double c = dot(d1, r);
    if (e <= eps) { t = 0; s = clampd(-c / a, 0, 1); }
    else {
      double b = dot(d1, d2), den = a * e - b * b;
      s = den != 0.0 ? clampd((b * f - c * e) / den, 0, 1) : 0.0;
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = clampd(-c / a, 0, 1); }
      else if (t > 1) { t = 1; s = clampd((b - c) / a, 0, 1); }
    }
  }
  *c1 = add(p1, scl(d1, s));
  *c2 = add(p2, scl(d2, t));
}

/* ---------------------------------------------- box and convex-hull colliders
 * A collider in world coordinates for the narrow phases below: capsule (segment p0-p1,
 * radius r), box (centre c, rotation R, half sizes hs) or convex hull (centre c = the geom
 * origin, rotation R, vertices in the geom frame). */
typedef struct {
  int type;            /* 0 capsule, PS_GEOM_BOX, PS_GEOM_HULL */
  v3 c;
  m3 R;
  v3 p0, p1;
  double r;
  double hs[3];
  const double (*vert)[3];
  int nvert;
  double rb;           /* hull: max vertex norm (xgeom_rbound), the scale of its support ties */
} shape;

static double sgn0(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); }

/* Support ties. MPR's portal directions are often EXACTLY normal to a face of a collider in
 * exact arithmetic - a portal triangle of three vertices of one hull face (or box face) minus
 * one point of the other shape has that face's normal - and then every vertex of the face
 * is a maximal support. libccd's first-maximal rule then picks whichever vertex the rounding
 * of the dots favours: a choice no perturbation of the state moves (the tie moves with the
 * body), that differs between fp64 and fp32 arithmetic, and that changes the portal path and
 * the final normal (by up to ~0.5 here: round 6, tools/contact_diff.py, 3% of the hull
 * contacts of the benched workload). Ties are therefore broken by a tolerance, identically in
 * the kernel (csrc/collide_x.h x_support): a hull vertex replaces the running best only when
 * its projection exceeds it by more than SUP_TIE_HULL x rb x |d| (the earliest vertex wins
 * inside the band; 2e-6 rb: ~10x the fp32 rounding of a projection, below half the support
 * cells' pruning margin of 1e-5 rb, so the pruned candidate lists give the same vertex); a box
 * component |dl_i| <= SUP_TIE_BOX max|dl| counts as 0 (the face centre: a support within 1e-6
 * of the box size); a capsule axis |ax.d| <= SUP_TIE_CAP |ax||d| as perpendicular (the
 * midpoint). Every choice is a support to within 2e-8 m, far inside MPR's 1e-6 m tolerance. */
#define SUP_TIE_HULL 2e-6
#define SUP_TIE_BOX 1e-6
#define SUP_TIE_CAP 1e-6

/* support point of the shape in direction d (MuJoCo's mjccd_support: box corner by the sign
 * of each local component, 0 on a zero component; capsule end by the sign along the axis
 * plus the radius along d; hull: first vertex of maximal projection - each with the tie
 * tolerance above) */
static v3 support(const shape* s, v3 d) {
  if (s->type == 0) {
    v3 ax = sub(s->p1, s->p0);
    double dn = nrm(d), da = dot(ax, d);
    if (fabs(da) <= SUP_TIE_CAP * nrm(ax) * dn) da = 0.0;
    v3 base = da > 0.0 ? s->p1 : (da < 0.0 ? s->p0 : scl(add(s->p0, s->p1), 0.5));
    return dn > 0.0 ? add(base, scl(d, s->r / dn)) : base;
  }
  v3 dl = mtv(s->R, d);
  v3 loc;
  if (s->type == PS_GEOM_BOX) {
    double mx = fmax(fabs(dl.v[0]), fmax(fabs(dl.v[1]), fabs(dl.v[2]))), sg[3];
    for (int k = 0; k < 3; k++) sg[k] = fabs(dl.v[k]) <= SUP_TIE_BOX * mx ? 0.0 : sgn0(dl.v[k]);
    loc = mk(sg[0] * s->hs[0], sg[1] * s->hs[1], sg[2] * s->hs[2]);
  } else {
    int best = 0;
    double bd = -INFINITY, tie = SUP_TIE_HULL * s->rb * nrm(dl);
    for (int i = 0; i < s->nvert; i++) {
      double p = dl.v[0] * s->vert[i][0] + dl.v[1] * s->vert[i][1] + dl.v[2] * s->vert[i][2];
      if (p > bd + tie) { bd = p; best = i; }
    }
    loc = mk(s->vert[best][0], s->vert[best][1], s->vert[best][2]);
  }
  return add(s->c, mv(s->R, loc));
}

static v3 shape_centre(const shape* s) { return s->type == 0 ? scl(add(s->p0, s->p1), 0.5) : s->c; }

/* Minkowski portal refinement (Snethen, GPG7 2.5), the penetration query of libccd's
 * ccdMPRPenetration that MuJoCo's convex collider mjc_Convex runs for mesh geoms (one
 * contact per pair; tolerance 1e-6, at most 50 refinements as MuJoCo's defaults). Portal
 * points are supports of the difference A - B, kept with their A and B witnesses. Returns 1
 * with depth >= 0, the normal A -> B and the contact point (midpoint of the witnesses), or
 * 0 when the shapes are apart. */
#define MPR_TOL 1e-6
#define MPR_MAXIT 50
#define MPR_EPS 2.220446049250313e-16   /* libccd CCD_EPS (double build) */
typedef struct { v3 v, a, b; } mpr_pt;

static int mpr_zero(double x) { return fabs(x) < MPR_EPS; }
static mpr_pt mpr_support(const shape* A, const shape* B, v3 d) {
  mpr_pt p;
  p.a = support(A, d);
  p.b = support(B, scl(d, -1.0));
  p.v = sub(p.a, p.b);
  return p;
}
static v3 nrmz(v3 a) { double n = nrm(a); return n > 0.0 ? scl(a, 1.0 / n) : a; }
static v3 portal_dir(const mpr_pt* P) { return nrmz(crs(sub(P[2].v, P[1].v), sub(P[3].v, P[1].v))); }
static int portal_reach_tol(const mpr_pt* P, const mpr_pt* v4, v3 dir) {
  double d4 = dot(v4->v, dir);
  double m = fmin(d4 - dot(P[1].v, dir), fmin(d4 - dot(P[2].v, dir), d4 - dot(P[3].v, dir)));
  return m <= MPR_TOL;
}
static void expand_portal(mpr_pt* P, const mpr_pt* v4) {
  v3 v4v0 = crs(v4->v, P[0].v);
  if (dot(P[1].v, v4v0) > 0.0) {
    if (dot(P[2].v, v4v0) > 0.0) P[1] = *v4; else P[3] = *v4;
  } else {
    if (dot(P[3].v, v4v0) > 0.0) P[2] = *v4; else P[1] = *v4;
  }
}
/* closest point of triangle (a, b, c) to the origin (Ericson, RTCD 5.1.5) */
static v3 tri_closest_origin(v3 a, v3 b, v3 c) {
  v3 ab = sub(b, a), ac = sub(c, a), ap = scl(a, -1.0);
  double d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.0 && d2 <= 0.0) return a;
  v3 bp = scl(b, -1.0);
  double d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.0 && d4 <= d3) return b;
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) return add(a, scl(ab, d1 / (d1 - d3)));
  v3 cp = scl(c, -1.0);
  double d5 = dot(ab, cp), d6 = dot(ac, cp);
  if (d6 >= 0.0 && d5 <= d6) return c;
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) return add(a, scl(ac, d2 / (d2 - d6)));
  double va = d3 * d6 - d5 * d4;
  if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0)
    return add(b, scl(sub(c, b), (d4 - d3) / ((d4 - d3) + (d5 - d6))));
  double den = 1.0 / (va + vb + vc);
  return add(a, add(scl(ab, vb * den), scl(ac, vc * den)));
}
static v3 mpr_pos(const mpr_pt* P) {
  v3 dir = portal_dir(P);
  double b[4];
  b[0] = dot(crs(P[1].v, P[2].v), P[3].v);
  b[1] = dot(crs(P[3].v, P[2].v), P[0].v);
  b[2] = dot(crs(P[0].v, P[1].v), P[3].v);
  b[3] = dot(crs(P[2].v, P[1].v), P[0].v);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (mpr_zero(sum) || sum < 0.0) {
    b[0] = 0.0;
    b[1] = dot(crs(P[2].v, P[3].v), dir);
    b[2] = dot(crs(P[3].v, P[1].v), dir);
    b[3] = dot(crs(P[1].v, P[2].v), dir);
    sum = b[1] + b[2] + b[3];
  }
  double inv = 1.0 / sum;
  v3 pa = mk(0, 0, 0), pb = mk(0, 0, 0);
  for (int i = 0; i < 4; i++) { pa = add(pa, scl(P[i].a, b[i])); pb = add(pb, scl(P[i].b, b[i])); }
  return scl(add(scl(pa, inv), scl(pb, inv)), 0.5);
}
static int mpr_penetration(const shape* A, const shape* B, double* depth, v3* n, v3* pos) {
  mpr_pt P[4];
  /* discover the portal */
  P[0].a = shape_centre(A); P[0].b = shape_centre(B); P[0].v = sub(P[0].a, P[0].b);
  if (P[0].v.v[0] == 0.0 && P[0].v.v[1] == 0.0 && P[0].v.v[2] == 0.0) P[0].v.v[0] += 10.0 * MPR_EPS;
  v3 dir = nrmz(scl(P[0].v, -1.0));
  P[1] = mpr_support(A, B, dir);
  double dt = dot(P[1].v, dir);
  if (mpr_zero(dt) || dt < 0.0) return 0;
  dir = crs(P[0].v, P[1].v);
  if (mpr_zero(dot(dir, dir))) {
    if (P[1].v.v[0] == 0.0 && P[1].v.v[1] == 0.0 && P[1].v.v[2] == 0.0) {  /* touching at v1 */
      *depth = 0.0; *n = mk(0, 0, 0); *pos = scl(add(P[1].a, P[1].b), 0.5);
    } else {  /* the origin lies on the segment v0-v1 */
      *pos = scl(add(P[1].a, P[1].b), 0.5);
      *depth = nrm(P[1].v); *n = nrmz(P[1].v);
    }
    return 1;
  }
  dir = nrmz(dir);
  P[2] = mpr_support(A, B, dir);
  dt = dot(P[2].v, dir);
  if (mpr_zero(dt) || dt < 0.0) return 0;
  dir = nrmz(crs(sub(P[1].v, P[0].v), sub(P[2].v, P[0].v)));
  if (dot(dir, P[0].v) > 0.0) { mpr_pt t = P[1]; P[1] = P[2]; P[2] = t; dir = scl(dir, -1.0); }
  for (int it = 0;; it++) {
    if (it > 4 * MPR_MAXIT) return 0;  /* guard (libccd has none here) */
    P[3] = mpr_support(A, B, dir);
    dt = dot(P[3].v, dir);
    if (mpr_zero(dt) || dt < 0.0) return 0;
    int cont = 0;
    double t = dot(crs(P[1].v, P[3].v), P[0].v);
    if (t < 0.0 && !mpr_zero(t)) { P[2] = P[3]; cont = 1; }
    if (!cont) {
      t = dot(crs(P[3].v, P[2].v), P[0].v);
      if (t < 0.0 && !mpr_zero(t)) { P[1] = P[3]; cont = 1; }
    }
    if (!cont) break;
    dir = nrmz(crs(sub(P[1].v, P[0].v), sub(P[2].v, P[0].v)));
  }
  /* refine until the portal contains the origin */
  for (int it = 0;; it++) {
    if (it > 4 * MPR_MAXIT) return 0;  /* guard */
    dir = portal_dir(P);
    dt = dot(P[1].v, dir);
    if (mpr_zero(dt) || dt > 0.0) break;  /* portal encapsulates the origin */
    mpr_pt v4 = mpr_support(A, B, dir);
    double d4 = dot(v4.v, dir);
    if (!(mpr_zero(d4) || d4 > 0.0) || portal_reach_tol(P, &v4, dir)) return 0;
    expand_portal(P, &v4);
  }
  /* penetration: refine toward the boundary, then the portal's distance to the origin */
  for (int it = 0;; it++) {
    dir = portal_dir(P);
    mpr_pt v4 = mpr_support(A, B, dir);
    if (portal_reach_tol(P, &v4, dir) || it > MPR_MAXIT) {
      v3 cp = tri_closest_origin(P[1].v, P[2].v, P[3].v);
      *depth = nrm(cp);
      *n = mpr_zero(*depth) ? dir : scl(cp, 1.0 / *depth);
      *pos = mpr_pos(P);
      return 1;
    }
    expand_portal(P, &v4);
  }
}

/* Box-box: separating-axis test over the 15 axes (3 + 3 face normals, 9 edge-edge cross
 * products; an edge axis wins only if 1.05 x its overlap is below the best face overlap),
 * then the contact manifold: face axis -> the incident face of the other box clipped against
 * the reference face's side planes, points below the reference face (at most 4, chosen by
 * deepest-first farthest-point sampling); edge axis -> one contact at the midpoint of the two
 * edges' closest points. Normal A -> B, contact point midway between the surfaces.
 * (MuJoCo's mjc_BoxBox is not available here; this is the standard SAT + clipping
 * restatement, with up to 4 contacts per pair.) Returns the number of contacts. */
#define BB_MAXPT 4
static v3 mcol(m3 R, int i) { return mk(R.m[i], R.m[3 + i], R.m[6 + i]); }
static int box_box(const shape* A, const shape* B, v3* pos, double* dist, v3* nout) {
  v3 a[3], b[3];
  for (int i = 0; i < 3; i++) { a[i] = mcol(A->R, i); b[i] = mcol(B->R, i); }
  v3 t = sub(B->c, A->c);
  double best = INFINITY;
  int bax = -1;
  v3 bn = mk(0, 0, 0);
  for (int k = 0; k < 15; k++) {
    v3 L;
    if (k < 3) L = a[k];
    else if (k < 6) L = b[k - 3];
    else {
      L = crs(a[(k - 6) / 3], b[(k - 6) % 3]);
      double ln = nrm(L);
      if (ln < 1e-6) continue;  /* parallel edges: covered by the face axes */
      L = scl(L, 1.0 / ln);
    }
    double ra = 0, rb = 0;
    for (int i = 0; i < 3; i++) { ra += A->hs[i] * fabs(dot(a[i], L)); rb += B->hs[i] * fabs(dot(b[i], L)); }
    double s = dot(t, L);
    double ov = ra + rb - fabs(s);
    if (ov < 0.0) return 0;
    if (k < 6 ? ov < best : 1.05 * ov < best) { best = ov; bax = k; bn = s >= 0.0 ? L : scl(L, -1.0); }
  }
  if (bax >= 6) {  /* edge-edge */
    int i = (bax - 6) / 3, j = (bax - 6) % 3;
    v3 pa = A->c, pb = B->c;
    for (int k = 0; k < 3; k++) {
      if (k != i) pa = add(pa, scl(a[k], (dot(a[k], bn) >= 0.0 ? 1.0 : -1.0) * A->hs[k]));
      if (k != j) pb = add(pb, scl(b[k], (dot(b[k], bn) >= 0.0 ? -1.0 : 1.0) * B->hs[k]));
    }
    v3 c1, c2;
    seg_seg(sub(pa, scl(a[i], A->hs[i])), add(pa, scl(a[i], A->hs[i])),
            sub(pb, scl(b[j], B->hs[j])), add(pb, scl(b[j], B->hs[j])), &c1, &c2);
    pos[0] = scl(add(c1, c2), 0.5);
    dist[0] = -best;
    *nout = bn;
    return 1;
  }
  /* face axis: reference box Rf (owner of the axis) with outward face normal nf toward the
   * incident box In; contacts keep the normal A -> B */
  const shape *Rf = bax < 3 ? A : B, *In = bax < 3 ? B : A;
  const v3* ra = bax < 3 ? a : b;
  const v3* ia = bax < 3 ? b : a;
  int fi = bax < 3 ? bax : bax - 3;
  v3 nf = bax < 3 ? bn : scl(bn, -1.0);
  /* incident face: the In face most anti-parallel to nf */
  int ij = 0;
  double bd = -1.0;
  for (int k = 0; k < 3; k++) {
    double d = fabs(dot(ia[k], nf));
    if (d > bd) { bd = d; ij = k; }
  }
  double sg = dot(ia[ij], nf) > 0.0 ? -1.0 : 1.0;
  int u = (ij + 1) % 3, w = (ij + 2) % 3;
  v3 fc = add(In->c, scl(ia[ij], sg * In->hs[ij]));
  v3 poly[8], tmp[8];
  const double su[4] = {1, -1, -1, 1}, sw[4] = {1, 1, -1, -1};
  int np = 4;
  for (int k = 0; k < 4; k++)
    poly[k] = add(fc, add(scl(ia[u], su[k] * In->hs[u]), scl(ia[w], sw[k] * In->hs[w])));
  /* Sutherland-Hodgman against the 4 side planes of the reference face */
  for (int e = 0; e < 4; e++) {
    int ax = (fi + 1 + e / 2) % 3;
    double side = (e % 2) ? -1.0 : 1.0;
    v3 pn = scl(ra[ax], side);
    double off = dot(pn, Rf->c) + Rf->hs[ax];
    int nq = 0;
    for (int k = 0; k < np; k++) {
      v3 p = poly[k], q = poly[(k + 1) % np];
      double dp = dot(pn, p) - off, dq = dot(pn, q) - off;
      if (dp <= 0.0) tmp[nq++] = p;
      if ((dp < 0.0 && dq > 0.0) || (dp > 0.0 && dq < 0.0)) tmp[nq++] = add(p, scl(sub(q, p), dp / (dp - dq)));
    }
    np = nq;
    for (int k = 0; k < np; k++) poly[k] = tmp[k];
    if (np == 0) return 0;
  }
  double fo = dot(nf, Rf->c) + Rf->hs[fi];
  v3 cp[8];
  double cd[8];
  int nc = 0;
  for (int k = 0; k < np; k++) {
    double d = fo - dot(nf, poly[k]);
    if (d >= 0.0) { cp[nc] = poly[k]; cd[nc] = d; nc++; }
  }
  int sel[BB_MAXPT], ns = 0;
  if (nc > 0) {
    int i0 = 0;
    for (int k = 1; k < nc; k++) if (cd[k] > cd[i0]) i0 = k;
    sel[ns++] = i0;
    while (ns < BB_MAXPT && ns < nc) {
      int bi = -1;
      double bdist = -1.0;
      for (int k = 0; k < nc; k++) {
        double md = INFINITY;
        int used = 0;
        for (int q = 0; q < ns; q++) {
          if (sel[q] == k) used = 1;
          md = fmin(md, nrm(sub(cp[k], cp[sel[q]])));
        }
        if (!used && md > bdist) { bdist = md; bi = k; }
      }
      sel[ns++] = bi;
    }
  }
  for (int q = 0; q < ns; q++) {
    pos[q] = add(cp[sel[q]], scl(nf, 0.5 * cd[sel[q]]));
    dist[q] = -cd[sel[q]];
  }
  *nout = bn;
  return ns;
}

static shape capsule_shape(const envdata* E, int h, int g, const ps_model_desc* d) {
  shape s;
  memset(&s, 0, sizeof(s));
  s.type = 0; s.p0 = E->cap0[h][g]; s.p1 = E->cap1[h][g]; s.r = d->geom_radius[h][g];
  return s;
}
static shape extra_shape(const envdata* E, int h, int i, const ps_model_desc* d) {
  shape s;
  memset(&s, 0, sizeof(s));
  s.type = d->xgeom_type[h][i]; s.c = E->xc[h][i]; s.R = E->xR[h][i];
  for (int k = 0; k < 3; k++) s.hs[k] = d->xgeom_size[h][i][k];
  s.vert = (const double(*)[3])d->hull_vert[h][d->xgeom_vert[h][i][0]];
  s.nvert = d->xgeom_vert[h][i][1];
  s.rb = d->xgeom_rbound[h][i];
  return s;
}
static shape box_shape(v3 c, m3 R, const double* hs) {
  shape s;
  memset(&s, 0, sizeof(s));
  s.type = PS_GEOM_BOX; s.c = c; s.R = R;
  for (int k = 0; k < 3; k++) s.hs[k] = hs[k];
  return s;
}

/* narrow phase of box/hull A (geom1) and box/hull/capsule B (geom2), contacts into E with the
 * normal A -> B; sub = contact index within the pair */
static void extra_pair(envdata* E, int maxc, contact proto, const shape* A, const shape* B) {
  if (A->type == PS_GEOM_BOX && B->type == PS_GEOM_BOX) {
    v3 pos[BB_MAXPT], n;
    double dist[BB_MAXPT];
    int k = box_box(A, B, pos, dist, &n);
    for (int q = 0; q < k; q++) {
      contact cc = proto;
      cc.pos = pos[q]; cc.n = n; cc.dist = dist[q]; cc.sub = q;
      make_frame(n, &cc.t1, &cc.t2);
      add_contact(E, maxc, &cc);
    }
    return;
  }
  double depth;
  v3 n, pos;
  if (!mpr_penetration(A, B, &depth, &n, &pos)) return;
  if (nrm(n) == 0.0) n = mk(0, 0, 1);  /* touching: no direction (zero depth) */
  contact cc = proto;
  cc.pos = pos; cc.n = n; cc.dist = -depth; cc.sub = 0;
  make_frame(n, &cc.t1, &cc.t2);
  add_contact(E, maxc, &cc);
}

static void collide(const model* m, const ps_task_cfg* cfg, envdata* E) {
  const ps_model_desc* d = &m->d;
  int maxc = cfg->max_contacts;
  E->ncon = 0;
  E->nfound = 0;
  m3 I3 = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
  v3 bc = mk(d->base_pos[0], d->base_pos[1], d->base_pos[2]);
  for (int h = 0; h < NH; h++) {
    for (int g = 0; g < NG; g++) {
      if (d->geom_body[h][g] < 0) continue;  /* unused slot */
      v3 p0 = E->cap0[h][g], p1 = E->cap1[h][g];
      double r = d->geom_radius[h][g];
      double lo[3], hi[3];
      for (int i = 0; i < 3; i++) {
        lo[i] = fmin(p0.v[i], p1.v[i]) - r;
        hi[i] = fmax(p0.v[i], p1.v[i]) + r;
      }
      contact proto;
      memset(&proto, 0, sizeof(proto));
      proto.h2 = h; proto.b2 = d->geom_body[h][g]; proto.g2 = h * NG + g; proto.g1 = -1;
      for (int k = 0; k < NK; k++) {
        /* conservative broadphase: key AABB over its motion */
        if (hi[1] < m->key_y_lo[k] || lo[1] > m->key_y_hi[k]) continue;
        if (lo[2] > d->key_pos[k][2] + d->key_half[k][2] + 0.02) continue;
        if (hi[0] < d->key_pos[k][0] - d->key_half[k][0] - 0.02 || lo[0] > d->key_pos[k][0] + d->key_half[k][0] + 0.02) continue;
        proto.kind = 0; proto.key = k;
        capsule_box(E, maxc, proto, p0, p1, r, E->keyc[k], E->keyR[k], d->key_half[k]);
      }
      proto.kind = 1; proto.key = -1;
      capsule_box(E, maxc, proto, p0, p1, r, bc, I3, d->base_half);
    }
  }
  for (int i = 0; i < d->n_cappairs; i++) {
    int ga = d->cappair[i][0], gb = d->cappair[i][1];
    int ha = ga / NG, la = ga % NG, hb = gb / NG, lb = gb % NG;
    v3 ca = scl(add(E->cap0[ha][la], E->cap1[ha][la]), 0.5), cb = scl(add(E->cap0[hb][lb], E->cap1[hb][lb]), 0.5);
    double ra = d->geom_radius[ha][la], rb = d->geom_radius[hb][lb];
    double bound = d->geom_halflen[ha][la] + d->geom_halflen[hb][lb] + ra + rb;
    if (nrm(sub(ca, cb)) > bound) continue;
    v3 c1, c2;
    seg_seg(E->cap0[ha][la], E->cap1[ha][la], E->cap0[hb][lb], E->cap1[hb][lb], &c1, &c2);
    v3 dv = sub(c2, c1);
    double dn = nrm(dv);
    double dist = dn - ra - rb;
    if (dist > 0.0) continue;
    contact cc;
    memset(&cc, 0, sizeof(cc));
    cc.kind = 2; cc.key = -1;
    cc.h1 = ha; cc.b1 = d->geom_body[ha][la]; cc.g1 = ga;
    cc.h2 = hb; cc.b2 = d->geom_body[hb][lb]; cc.g2 = gb;
    cc.n = dn > 1e-9 ? scl(dv, 1.0 / dn) : mk(0, 0, 1);
    cc.dist = dist;
    cc.pos = add(c1, scl(cc.n, ra + 0.5 * dist));
    make_frame(cc.n, &cc.t1, &cc.t2);
    add_contact(E, maxc, &cc);  /* past the cap: counted in nfound, not kept */
  }
  /* extra colliders (box / hull) against the keys and the base, after every capsule pair (the
   * kernel takes them and the hand-hand pairs below as one list, csrc/kernel_v2.inc collide2) */
  for (int h = 0; h < NH; h++) {
    for (int i = 0; i < NX; i++) {
      if (d->xgeom_type[h][i] == PS_GEOM_NONE) continue;
      shape B = extra_shape(E, h, i, d);
      double rb = d->xgeom_rbound[h][i], lo[3], hi[3];
      for (int k = 0; k < 3; k++) { lo[k] = B.c.v[k] - rb; hi[k] = B.c.v[k] + rb; }
      contact proto;
      memset(&proto, 0, sizeof(proto));
      proto.h2 = h; proto.b2 = d->xgeom_body[h][i]; proto.g2 = NCAPS + h * NX + i; proto.g1 = -1;
      for (int k = 0; k < NK; k++) {
        if (hi[1] < m->key_y_lo[k] || lo[1] > m->key_y_hi[k]) continue;
        if (lo[2] > d->key_pos[k][2] + d->key_half[k][2] + 0.02) continue;
        if (hi[0] < d->key_pos[k][0] - d->key_half[k][0] - 0.02 || lo[0] > d->key_pos[k][0] + d->key_half[k][0] + 0.02) continue;
        proto.kind = 0; proto.key = k;
        shape A = box_shape(E->keyc[k], E->keyR[k], d->key_half[k]);
        extra_pair(E, maxc, proto, &A, &B);
      }
      proto.kind = 1; proto.key = -1;
      shape A = box_shape(bc, I3, d->base_half);
      extra_pair(E, maxc, proto, &A, &B);
    }
  }
  /* hand-hand pairs with an extra collider: bounding spheres, then capsule-box (normal box ->
   * capsule, the box as geom1), box-box or MPR (normal geom a -> geom b) */
  for (int i = 0; i < d->n_xpairs; i++) {
    int ga = d->xpair[i][0], gb = d->xpair[i][1];
    shape S[2];
    int hh[2], bb[2];
    double bound = 0.0;
    v3 cen[2];
    for (int q = 0; q < 2; q++) {
      int g = q ? gb : ga;
      if (g < NCAPS) {
        int h = g / NG, l = g % NG;
        S[q] = capsule_shape(E, h, l, d);
        hh[q] = h; bb[q] = d->geom_body[h][l];
        bound += d->geom_halflen[h][l] + d->geom_radius[h][l];
      } else {
        int h = (g - NCAPS) / NX, l = (g - NCAPS) % NX;
        S[q] = extra_shape(E, h, l, d);
        hh[q] = h; bb[q] = d->xgeom_body[h][l];
        bound += d->xgeom_rbound[h][l];
      }
      cen[q] = shape_centre(&S[q]);
    }
    if (nrm(sub(cen[0], cen[1])) > bound) continue;
    contact proto;
    memset(&proto, 0, sizeof(proto));
    proto.kind = 2; proto.key = -1;
    if (S[0].type == 0 && S[1].type == PS_GEOM_BOX) {
      proto.h1 = hh[1]; proto.b1 = bb[1]; proto.g1 = gb;
      proto.h2 = hh[0]; proto.b2 = bb[0]; proto.g2 = ga;
      capsule_box(E, maxc, proto, S[0].p0, S[0].p1, S[0].r, S[1].c, S[1].R, S[1].hs);
      continue;
    }
    proto.h1 = hh[0]; proto.b1 = bb[0]; proto.g1 = ga;
    proto.h2 = hh[1]; proto.b2 = bb[1]; proto.g2 = gb;
    extra_pair(E, maxc, proto, &S[0], &S[1]);
  }
}

/* ------------------------------------------------------------------ constraints */
/* Constraint rows of one substep (MuJoCo mj_makeConstraint order: friction loss, limits,
 * contacts). Every row is J (dense over the dofs, sparse in practice), its reference
 * acceleration aref, regulariser R (D = 1/R) and type; J x - aref = jar is the row's
 * constraint-space residual at the acceleration x. */
enum { ROW_FRICTION = 0, ROW_LIMIT = 1, ROW_CONTACT = 2 };
typedef struct {
  double J[NV];
  double aref, R, D, floss;  /* floss: friction-loss bound (ROW_FRICTION) */
  int type;
  int closed;                /* free key limit row (solved in closed form) */
} row;

static double impedance(const double* si, double pos) {
  double d0 = clampd(si[0], MINIMP, MAXIMP), dw = clampd(si[1], MINIMP, MAXIMP);
  double width = si[2], mid = si[3], power = si[4];
  double x = fabs(pos) / width, imp;
  if (x >= 1.0 || width <= MINVAL) imp = dw;
  else {
    double y;
    if (power == 1.0) y = x;
    else if (x <= mid) y = pow(x, power) / pow(mid, power - 1.0);
    else y = 1.0 - pow(1.0 - x, power) / pow(1.0 - mid, power - 1.0);
    imp = d0 + y * (dw - d0);
  }
  return clampd(imp, MINIMP, MAXIMP);
}

/* Jacobian row of a point on a hand body along direction u, accumulated with sign */
static void jac_point(const model* m, const envdata* E, int h, int b, v3 p, v3 u, double sgn, double* J) {
  const ps_model_desc* d = &m->d;
  for (int bb = b; bb >= 0; bb = d->body_parent[h][bb]) {
    for (int j = m->body_dofadr[h][bb]; j >= 0 && j < m->body_dofadr[h][bb] + m->body_dofnum[h][bb]; j++) {
      if (d->dof_locked[h][j]) continue;  /* a joint the reference's hand lacks */
      double val = d->dof_type[h][j] == 0 ? dot(u, crs(E->axis[h][j], sub(p, E->o[h][bb]))) : dot(u, E->axis[h][j]);
      J[NK + h * ND + j] += sgn * val;
    }
  }
}

static void contact_jac(const model* m, const envdata* E, const contact* c, v3 u, double* J) {
  memset(J, 0, sizeof(double) * NV);
  jac_point(m, E, c->h2, c->b2, c->pos, u, 1.0, J);
  if (c->kind == 2) jac_point(m, E, c->h1, c->b1, c->pos, u, -1.0, J);
  else if (c->kind == 0) {
    v3 ay = mk(0, 1, 0);
    J[c->key] -= dot(u, crs(ay, sub(c->pos, E->keyanchor[c->key])));
  }
}

static double dotv(const double* a, const double* b) {
  double s = 0;
  for (int i = 0; i < NV; i++) s += a[i] * b[i];
  return s;
}

/* aref and R of a row (mj_makeImpedance / mj_makeKBIP): pos = the row's violation (0 for
 * friction loss), diag_approx = MuJoCo's constant regulariser scale from invweight0 */
static void row_finish(const model* m, envdata* E, row* r, double pos, const double* solref, const double* solimp,
                       double diag_approx) {
  const ps_model_desc* d = &m->d;
  double imp = impedance(solimp, pos);
  double dmax = clampd(solimp[1], MINIMP, MAXIMP);
  double tc = fmax(solref[0], 2.0 * d->timestep), dr = solref[1];
  double K = 1.0 / (dmax * dmax * tc * tc * dr * dr), B = 2.0 / (dmax * tc);
  r->aref = -B * dotv(r->J, E->v) - K * imp * pos;
  r->R = fmax(MINVAL, (1.0 - imp) / imp * diag_approx);
  r->D = 1.0 / r->R;
}

static void mix_param(const ps_contact_param* a, const ps_contact_param* b, double* solref, double* solimp, double* mu) {
  for (int i = 0; i < 2; i++) solref[i] = 0.5 * (a->solref[i] + b->solref[i]);
  for (int i = 0; i < 5; i++) solimp[i] = 0.5 * (a->solimp[i] + b->solimp[i]);
  *mu = fmax(a->friction, b->friction);
}

#define MAXROW (NH * ND + NH * ND + 2 * NK + 4 * MAXCON)  /* friction loss, limits, contacts: no cap */
static _Thread_local row g_rows[MAXROW];
int ref_debug_level = 0;
/* Per-substep study histograms: contacts the narrow phase found (kept or not), constraint
 * rows, contacts kept; substeps where the contact cap dropped a contact. */
#define REF_HIST 256
long ref_rows_hist[REF_HIST];
long ref_con_hist[PS_MAX_CONTACTS_LIMIT + 2];
long ref_found_hist[REF_HIST];
long ref_cap_events[1];
long ref_iter_total, ref_substeps_total;
long ref_newton_hist[64];     /* Newton iterations per substep ([63]: iteration cap) */
long ref_zone_counts[6 + 128];      /* study: rows at the solution by type (friction, limit, contact edge) x (outside, quadratic zone) */
void ref_zone_stats(long* out) { memcpy(out, ref_zone_counts, sizeof(ref_zone_counts)); memset(ref_zone_counts, 0, sizeof(ref_zone_counts)); }
long ref_warnings_total[PS_NWARN];
/* Study override of the constraint solve:
 *   0: the specification (primal Newton, below);
 *   1: projected Gauss-Seidel on the dual, from a cold start until a sweep changes no force by
 *      more than ref_pgs_tol * (1 + max|f|) (at most ref_pgs_maxit sweeps): an independent
 *      method for the same unique solution (the dual of a strictly convex problem). */
int ref_pgs_mode = 0;
int ref_warmstart = 0;
int ref_fullstep = 0;   /* study: full Newton steps when they descend */  /* study: Newton from qacc_warmstart (MuJoCo's rule) instead of qacc_smooth */
double ref_pgs_tol = 1e-12;
int ref_pgs_maxit = 200000;

/* s'(jar) of a row: the negative of its constraint force. Unilateral rows (limits, pyramid
 * edges): D jar while jar < 0, else 0. Friction loss: D jar clamped to [-floss, floss] (the
 * quadratic zone |jar| < R floss, the two linear zones outside) - MuJoCo's
 * mj_constraintUpdate states QUADRATIC / SATISFIED / LINEARNEG / LINEARPOS. */
static double row_dcost(const row* r, double jar) {
  double t = r->D * jar;
  if (r->type == ROW_FRICTION) return clampd(t, -r->floss, r->floss);
  return t < 0.0 ? t : 0.0;
}
static double row_cost(const row* r, double jar) {
  if (r->type == ROW_FRICTION) {
    double z = r->R * r->floss;
    if (jar <= -z) return -r->floss * (jar + 0.5 * z);
    if (jar >= z) return r->floss * (jar - 0.5 * z);
    return 0.5 * r->D * jar * jar;
  }
  return jar < 0.0 ? 0.5 * r->D * jar * jar : 0.0;
}
/* 1: the row is in its quadratic zone (contributes D J'J to the Hessian) */
static int row_quad(const row* r, double jar) {
  if (r->type == ROW_FRICTION) return fabs(jar) < r->R * r->floss;
  return jar < 0.0;
}

/* Primal Newton solve of the constraint forces (MuJoCo's default solver, mj_solNewton):
 *     min_x  1/2 (x - x_s)' M (x - x_s) + sum_r s_r(J_r x - aref_r)
 * over the accelerations x of the coupled dofs (both hands and the keys touched by a
 * contact), x_s = qacc_smooth. The cost is strictly convex and piecewise quadratic, so its
 * minimiser is unique - the one every MuJoCo solver converges to. Iteration: Newton direction
 * from the Hessian M + sum_{quadratic rows} D_r J_r' J_r (dense Cholesky over the coupled
 * dofs), then the EXACT line search along it (the derivative of the piecewise-quadratic cost
 * along the direction is piecewise linear and non-decreasing: its root is found by walking the
 * sorted breakpoints), until the gradient vanishes to 1e-13 relative. Returns the iterations,
 * -1 at the cap. x enters as x_s and leaves as qacc. */
#define NEWTON_MAXIT 100
#define NEWTON_TOL 1e-13
static int newton_solve(const model* m, envdata* E, int nr, const int* dofs, int nd, const double* xs, double* x) {
  static _Thread_local double H[NV][NV], jar[MAXROW], jdir[MAXROW];
  double g[NV], dx[NV], y[NV];
  int ret = -1;
  for (int iter = 1; iter <= NEWTON_MAXIT; iter++) {
    /* residuals, gradient M (x - x_s) + J' s'(jar) */
    for (int i = 0; i < NV; i++) y[i] = x[i] - xs[i];
    double gscale = 0.0;
    for (int a = 0; a < nd; a++) {
      int i = dofs[a];
      double s = 0.0, sa = 0.0;  /* sa: the rounding scale of s, sum |M_ij| (|x_j| + |x_s,j|) */
      if (i < NK) { s = E->Mk[i] * y[i]; sa = E->Mk[i] * (fabs(x[i]) + fabs(xs[i])); }
      else {
        int h = (i - NK) / ND, ii = (i - NK) % ND;
        for (int jj = 0; jj < ND; jj++) {
          s += E->Mfull[h][ii][jj] * y[NK + h * ND + jj];
          sa += fabs(E->Mfull[h][ii][jj]) * (fabs(x[NK + h * ND + jj]) + fabs(xs[NK + h * ND + jj]));
        }
      }
      g[i] = s;
      gscale = fmax(gscale, sa);
    }
    double fscale = 0.0;
    for (int r = 0; r < nr; r++) {
      if (g_rows[r].closed) continue;
      jar[r] = dotv(g_rows[r].J, x) - g_rows[r].aref;
      double ds = row_dcost(&g_rows[r], jar[r]);
      if (ds != 0.0)
        for (int a = 0; a < nd; a++) g[dofs[a]] += g_rows[r].J[dofs[a]] * ds;
      for (int a = 0; a < nd; a++) fscale = fmax(fscale, fabs(g_rows[r].J[dofs[a]] * ds));
    }
    double gmax = 0.0;
    for (int a = 0; a < nd; a++) gmax = fmax(gmax, fabs(g[dofs[a]]));
    if (ref_debug_level == 7 || (ref_debug_level == 8 && iter > 90)) printf("iter %d gmax %.3e scale %.3e %.3e\n", iter, gmax, gscale, fscale);
    if (gmax <= NEWTON_TOL * fmax(fmax(gscale, fscale), 1e-300)) { ret = iter - 1; break; }
    /* Hessian over the coupled dofs */
    for (int a = 0; a < nd; a++)
      for (int b = 0; b < nd; b++) {
        int i = dofs[a], j = dofs[b];
        double v = 0.0;
        if (i < NK || j < NK) v = i == j ? E->Mk[i] : 0.0;
        else if ((i - NK) / ND == (j - NK) / ND) v = E->Mfull[(i - NK) / ND][(i - NK) % ND][(j - NK) % ND];
        H[a][b] = v;
      }
    for (int r = 0; r < nr; r++) {
      if (g_rows[r].closed || !row_quad(&g_rows[r], jar[r])) continue;
      const double* J = g_rows[r].J;
      for (int a = 0; a < nd; a++) {
        double ja = J[dofs[a]];
        if (ja == 0.0) continue;
        for (int b = 0; b < nd; b++) H[a][b] += g_rows[r].D * ja * J[dofs[b]];
      }
    }
    /* Cholesky H = L L' in place (lower), then dx = -H^-1 g */
    for (int k = 0; k < nd; k++) {
      double s = H[k][k];
      for (int c = 0; c < k; c++) s -= H[k][c] * H[k][c];
      H[k][k] = sqrt(fmax(s, MINVAL));
      for (int a = k + 1; a < nd; a++) {
        double t = H[a][k];
        for (int c = 0; c < k; c++) t -= H[a][c] * H[k][c];
        H[a][k] = t / H[k][k];
      }
    }
    double z[NV];
    for (int a = 0; a < nd; a++) {
      double s = -g[dofs[a]];
      for (int c = 0; c < a; c++) s -= H[a][c] * z[c];
      z[a] = s / H[a][a];
    }
    for (int a = nd - 1; a >= 0; a--) {
      double s = z[a];
      for (int c = a + 1; c < nd; c++) s -= H[c][a] * z[c];
      z[a] = s / H[a][a];
    }
    memset(dx, 0, sizeof(dx));
    for (int a = 0; a < nd; a++) dx[dofs[a]] = z[a];
    /* exact line search: phi'(t) = t dx'M dx + dx'M y + sum_r jdir_r s_r'(jar_r + t jdir_r) */
    double q2 = 0.0, q1 = 0.0;
    for (int a = 0; a < nd; a++) {
      int i = dofs[a];
      double s = 0.0;
      if (i < NK) s = E->Mk[i] * dx[i];
      else {
        int h = (i - NK) / ND, ii = (i - NK) % ND;
        for (int jj = 0; jj < ND; jj++) s += E->Mfull[h][ii][jj] * dx[NK + h * ND + jj];
      }
      q2 += dx[i] * s;
      q1 += y[i] * s;
    }
    double bp[2 * MAXROW];
    int nbp = 0;
    for (int r = 0; r < nr; r++) {
      if (g_rows[r].closed) continue;
      jdir[r] = dotv(g_rows[r].J, dx);
      if (jdir[r] == 0.0) continue;
      if (g_rows[r].type == ROW_FRICTION) {
        double z0 = g_rows[r].R * g_rows[r].floss;
        double t1 = (-z0 - jar[r]) / jdir[r], t2 = (z0 - jar[r]) / jdir[r];
        if (t1 > 0.0) bp[nbp++] = t1;
        if (t2 > 0.0) bp[nbp++] = t2;
      } else {
        double t = -jar[r] / jdir[r];
        if (t > 0.0) bp[nbp++] = t;
      }
    }
    for (int i = 1; i < nbp; i++) {  /* insertion sort (breakpoints are few) */
      double v = bp[i];
      int k = i - 1;
      while (k >= 0 && bp[k] > v) { bp[k + 1] = bp[k]; k--; }
      bp[k + 1] = v;
    }
    /* phi' is linear between breakpoints: evaluate it at the left end of each segment and at
     * a point inside it; the root is in the first segment whose right end has phi' >= 0 */
    double t_lo = 0.0, alpha = -1.0;
    for (int s = 0; s <= nbp && alpha < 0.0; s++) {
      double t_hi = s < nbp ? bp[s] : (t_lo > 0.0 ? 2.0 * t_lo + 1.0 : 1.0);
      if (t_hi <= t_lo) continue;
      double tm = 0.5 * (t_lo + t_hi);
      /* within (t_lo, t_hi) every row keeps its zone: phi'(t) = c0 + c1 t */
      double c1 = q2, c0 = q1;
      for (int r = 0; r < nr; r++) {
        if (g_rows[r].closed || jdir[r] == 0.0) continue;
        const row* rr = &g_rows[r];
        double jm = jar[r] + tm * jdir[r];
        if (row_quad(rr, jm)) {
          c1 += rr->D * jdir[r] * jdir[r];
          c0 += rr->D * jdir[r] * jar[r];
        } else {
          c0 += jdir[r] * row_dcost(rr, jm);
        }
      }
      double root = c1 > 0.0 ? -c0 / c1 : (c0 < 0.0 ? 1e300 : t_lo);
      if (s == nbp) alpha = fmax(root, t_lo);  /* last segment is unbounded */
      else if (root <= t_hi) alpha = fmax(root, t_lo);
      t_lo = t_hi;
    }
    if (ref_debug_level == 7 || (ref_debug_level == 8 && iter > 90)) printf("   alpha %.6g nbp %d q2 %.3e q1 %.3e\n", alpha, nbp, q2, q1);
    if (ref_fullstep) {  /* study: the full Newton step whenever it lowers the cost */
      double c0 = 0.5 * 0.0, c1 = 0.5 * q2 + q1;  /* quadratic part: f(t) - f(0) = t^2/2 q2 + t q1 */
      for (int r = 0; r < nr; r++) {
        if (g_rows[r].closed) continue;
        c0 += row_cost(&g_rows[r], jar[r]);
        c1 += row_cost(&g_rows[r], jar[r] + jdir[r]);
      }
      if (c1 < c0) alpha = 1.0;
    }
    double step = 0.0, xmag = 0.0;
    for (int a = 0; a < nd; a++) {
      x[dofs[a]] += alpha * dx[dofs[a]];
      step = fmax(step, fabs(alpha * dx[dofs[a]]));
      xmag = fmax(xmag, fabs(x[dofs[a]]));
    }
    if (step <= 1e-15 * xmag) { ret = iter; break; }  /* at the rounding floor of x */
    (void)row_cost;
  }
  /* study: rows in their quadratic zone at the solution, by type (ref_zone_stats), and a
   * histogram of their number per substep */
  int nq = 0;
  for (int r = 0; r < nr; r++) {
    if (g_rows[r].closed) continue;
    double j = dotv(g_rows[r].J, x) - g_rows[r].aref;
    int q = row_quad(&g_rows[r], j) ? 1 : 0;
    nq += q;
    __atomic_fetch_add(&ref_zone_counts[2 * g_rows[r].type + q], 1, __ATOMIC_RELAXED);
  }
  __atomic_fetch_add(&ref_zone_counts[6 + (nq < 127 ? nq : 127)], 1, __ATOMIC_RELAXED);
  return ret;
}

/* Dual projected Gauss-Seidel run to convergence (study mode 1): rows' Delassus entries
 * J M^-1 J' from the tree factor, boxes [-floss, floss] for friction loss, f >= 0 otherwise. */
static void dual_pgs(const model* m, envdata* E, int nr, const double* xs, double* f) {
  static _Thread_local double Y[MAXROW][NV];  /* M^-1 J' */
  double A[MAXROW], b[MAXROW];
  for (int r = 0; r < nr; r++) {
    solve_full(m, E, 0, g_rows[r].J, Y[r]);
    A[r] = dotv(g_rows[r].J, Y[r]);
    b[r] = dotv(g_rows[r].J, xs) - g_rows[r].aref;
    f[r] = 0.0;
  }
  double acc[NV];  /* M^-1 J' f */
  memset(acc, 0, sizeof(acc));
  for (int it = 0; it < ref_pgs_maxit; it++) {
    double dfmax = 0.0, fmaxabs = 0.0;
    for (int r = 0; r < nr; r++) {
      if (g_rows[r].closed) continue;
      double res = b[r] + g_rows[r].R * f[r] + dotv(g_rows[r].J, acc);
      double fn = f[r] - res / (A[r] + g_rows[r].R);
      fn = g_rows[r].type == ROW_FRICTION ? clampd(fn, -g_rows[r].floss, g_rows[r].floss) : fmax(0.0, fn);
      double df = fn - f[r];
      if (df != 0.0)
        for (int k = 0; k < NV; k++) acc[k] += Y[r][k] * df;
      f[r] = fn;
      dfmax = fmax(dfmax, fabs(df));
      fmaxabs = fmax(fmaxabs, fabs(fn));
    }
    __atomic_fetch_add(&ref_iter_total, 1, __ATOMIC_RELAXED);
    if (dfmax <= ref_pgs_tol * (1.0 + fmaxabs)) break;
  }
}

static void reset_physics(envdata* E, int warning) {
  /* mj_resetData after mj_checkPos / mj_checkVel / mj_checkAcc: qpos = qpos0 (0 here), qvel,
   * qacc_warmstart, ctrl and qfrc_applied = 0; the warning counts survive (dm_control's
   * check_invalid_state compares them around the step) */
  memset(E->q, 0, sizeof(E->q));
  memset(E->v, 0, sizeof(E->v));
  memset(E->qacc_ws, 0, sizeof(E->qacc_ws));
  memset(E->ctrl, 0, sizeof(E->ctrl));
  memset(E->applied, 0, sizeof(E->applied));
  E->warnings[warning]++;
  __atomic_fetch_add(&ref_warnings_total[warning], 1, __ATOMIC_RELAXED);
}
/* mju_isBad: NaN or |x| > mjMAXVAL (1e10) */
static int bad_vec(const double* x, int n) {
  for (int i = 0; i < n; i++)
    if (!(fabs(x[i]) <= 1e10)) return 1;
  return 0;
}

static void step_physics(const model* m, const ps_task_cfg* cfg, envdata* E) {
  const ps_model_desc* d = &m->d;
  const double h_t = d->timestep;
  /* a locked dof stays at its joint zero */
  for (int h = 0; h < NH; h++)
    for (int j = 0; j < ND; j++)
      if (d->dof_locked[h][j]) E->q[NK + h * ND + j] = E->v[NK + h * ND + j] = 0.0;
  /* mj_checkPos, mj_checkVel (mj_step1) */
  if (bad_vec(E->q, NV)) reset_physics(E, PS_WARN_BADQPOS);
  if (bad_vec(E->v, NV)) reset_physics(E, PS_WARN_BADQVEL);
  for (int pass = 0; pass < 2; pass++) {  /* pass 1: after mj_checkAcc reset the state */
    kinematics(m, E);
    dynamics(m, cfg, E);
    collide(m, cfg, E);
    for (int h = 0; h < NH; h++) {
      memcpy(E->Mfull[h], E->M[h], sizeof(E->M[h]));
      memcpy(E->Mh[h], E->M[h], sizeof(E->M[h]));
      for (int j = 0; j < ND; j++)
        if (!d->dof_locked[h][j]) E->Mh[h][j][j] += h_t * d->dof_damping[h][j];
      factor(m, h, E->M[h], E->D[h]);
      factor(m, h, E->Mh[h], E->Dh[h]);
    }
    double fsmooth[NV], qacc_smooth[NV];
    for (int i = 0; i < NV; i++) fsmooth[i] = E->passive[i] + E->actfrc[i] + E->applied[i] - E->bias[i];
    for (int h = 0; h < NH; h++)
      for (int j = 0; j < ND; j++)
        if (d->dof_locked[h][j]) fsmooth[NK + h * ND + j] = 0.0;
    solve_full(m, E, 0, fsmooth, qacc_smooth);

    /* rows: friction loss (hand dofs), hand limits, key limits (keys touched by a contact are
     * coupled; the others are 1-dof problems solved in closed form), contacts (4 pyramid
     * edges each). No row cap. */
    int keyhit[NK];
    memset(keyhit, 0, sizeof(keyhit));
    for (int c = 0; c < E->ncon; c++)
      if (E->con[c].kind == 0) keyhit[E->con[c].key] = 1;
    int nr = 0;
    for (int h = 0; h < NH; h++)
      for (int j = 0; j < ND; j++) {
        if (!(d->dof_frictionloss[h][j] > 0.0) || d->dof_locked[h][j]) continue;
        row* r = &g_rows[nr++];
        memset(r->J, 0, sizeof(r->J));
        r->J[NK + h * ND + j] = 1.0;
        r->type = ROW_FRICTION;
        r->closed = 0;
        r->floss = d->dof_frictionloss[h][j];
        row_finish(m, E, r, 0.0, d->friction_solref, d->friction_solimp, d->dof_invweight[h][j]);
      }
    for (int h = 0; h < NH; h++)
      for (int j = 0; j < ND; j++) {
        if (!d->dof_limited[h][j] || d->dof_locked[h][j]) continue;
        double q = E->q[NK + h * ND + j];
        for (int side = 0; side < 2; side++) {
          double dist = side == 0 ? q - d->dof_range[h][j][0] : d->dof_range[h][j][1] - q;
          if (dist >= 0.0) continue;
          row* r = &g_rows[nr++];
          memset(r->J, 0, sizeof(r->J));
          r->J[NK + h * ND + j] = side == 0 ? 1.0 : -1.0;
          r->type = ROW_LIMIT;
          r->closed = 0;
          row_finish(m, E, r, dist, d->limit_solref, d->limit_solimp, d->dof_invweight[h][j]);
        }
      }
    for (int k = 0; k < NK; k++)
      for (int side = 0; side < 2; side++) {
        double dist = side == 0 ? E->q[k] - d->key_range[k][0] : d->key_range[k][1] - E->q[k];
        if (dist >= 0.0) continue;
        row* r = &g_rows[nr++];
        memset(r->J, 0, sizeof(r->J));
        r->J[k] = side == 0 ? 1.0 : -1.0;
        r->type = ROW_LIMIT;
        r->closed = !keyhit[k];
        row_finish(m, E, r, dist, d->limit_solref, d->limit_solimp, d->key_dof_invweight[k]);
      }
    for (int c = 0; c < E->ncon; c++) {
      contact* cc = &E->con[c];
      double solref[2], solimp[5], mu;
      mix_param(cc->kind == 2 ? &d->hand_contact : &d->piano_contact, &d->hand_contact, solref, solimp, &mu);
      double Jn[NV], Jt1[NV], Jt2[NV];
      contact_jac(m, E, cc, cc->n, Jn);
      contact_jac(m, E, cc, cc->t1, Jt1);
      contact_jac(m, E, cc, cc->t2, Jt2);
      double tran = d->body_invweight[cc->h2][cc->b2];
      if (cc->kind == 0) tran += d->key_body_invweight[cc->key];
      else if (cc->kind == 2) tran += d->body_invweight[cc->h1][cc->b1];
      double diag = (1.0 + mu * mu) * tran;
      for (int e = 0; e < 4; e++) {
        row* r = &g_rows[nr++];
        const double* Jt = e < 2 ? Jt1 : Jt2;
        double s = (e & 1) ? -mu : mu;
        for (int i = 0; i < NV; i++) r->J[i] = Jn[i] + s * Jt[i];
        r->type = ROW_CONTACT;
        r->closed = 0;
        row_finish(m, E, r, cc->dist, solref, solimp, diag);
      }
    }
    __atomic_fetch_add(&ref_rows_hist[nr < REF_HIST ? nr : REF_HIST - 1], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&ref_con_hist[E->ncon], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&ref_found_hist[E->nfound < REF_HIST ? E->nfound : REF_HIST - 1], 1, __ATOMIC_RELAXED);
    if (E->nfound > E->ncon) __atomic_fetch_add(&ref_cap_events[0], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&ref_substeps_total, 1, __ATOMIC_RELAXED);

    /* coupled dofs: both hands, then the keys touched by a contact */
    int dofs[NV], nd = 0;
    for (int i = NK; i < NV; i++) dofs[nd++] = i;
    for (int k = 0; k < NK; k++)
      if (keyhit[k]) dofs[nd++] = k;
    double x[NV], f[MAXROW];
    memcpy(x, qacc_smooth, sizeof(x));
    if (ref_warmstart) {  /* study: MuJoCo's warm start - qacc_warmstart when its cost is lower */
      double cs = 0.0, cw = 0.0, y[NV];
      for (int i = 0; i < NV; i++) y[i] = E->qacc_ws[i] - qacc_smooth[i];
      for (int a = 0; a < nd; a++) {
        int i = dofs[a];
        double s = 0.0;
        if (i < NK) s = E->Mk[i] * y[i];
        else for (int jj = 0; jj < ND; jj++) s += E->Mfull[(i - NK) / ND][(i - NK) % ND][jj] * y[NK + (i - NK) / ND * ND + jj];
        cw += 0.5 * y[i] * s;
      }
      for (int r = 0; r < nr; r++) {
        if (g_rows[r].closed) continue;
        cs += row_cost(&g_rows[r], dotv(g_rows[r].J, qacc_smooth) - g_rows[r].aref);
        cw += row_cost(&g_rows[r], dotv(g_rows[r].J, E->qacc_ws) - g_rows[r].aref);
      }
      if (cw < cs)
        for (int a = 0; a < nd; a++) x[dofs[a]] = E->qacc_ws[dofs[a]];
    }
    if (ref_pgs_mode == 1) {
      dual_pgs(m, E, nr, qacc_smooth, f);
    } else {
      int it = newton_solve(m, E, nr, dofs, nd, qacc_smooth, x);
      __atomic_fetch_add(&ref_newton_hist[it >= 0 && it < 63 ? it : 63], 1, __ATOMIC_RELAXED);
      if (it > 0) __atomic_fetch_add(&ref_iter_total, it, __ATOMIC_RELAXED);
      for (int r = 0; r < nr; r++)
        if (!g_rows[r].closed) f[r] = -row_dcost(&g_rows[r], dotv(g_rows[r].J, x) - g_rows[r].aref);
    }
    /* free key limits: 1-dof problems, f = max(0, -b / (1/Mk + R)) */
    for (int r = 0; r < nr; r++)
      if (g_rows[r].closed) {
        int k = 0;
        while (g_rows[r].J[k] == 0.0) k++;
        double b = g_rows[r].J[k] * qacc_smooth[k] - g_rows[r].aref;
        f[r] = fmax(0.0, -b / (1.0 / E->Mk[k] + g_rows[r].R));
      }
    if (ref_debug_level)
      for (int r = 0; r < nr; r++) printf("row %d type %d R %.4g aref %.4g f %.6g\n", r, g_rows[r].type, g_rows[r].R, g_rows[r].aref, f[r]);
    /* qfrc_constraint = J' f; qacc = M^-1 (qfrc_smooth + qfrc_constraint) */
    double F[NV];
    memcpy(F, fsmooth, sizeof(F));
    for (int r = 0; r < nr; r++)
      if (f[r] != 0.0)
        for (int i = 0; i < NV; i++) F[i] += g_rows[r].J[i] * f[r];
    double qacc[NV], qacc_e[NV];
    solve_full(m, E, 0, F, qacc);
    /* mj_checkAcc: reset and recompute the forward dynamics at the reset state */
    if (pass == 0 && bad_vec(qacc, NV)) {
      reset_physics(E, PS_WARN_BADQACC);
      continue;
    }
    solve_full(m, E, 1, F, qacc_e);
    memcpy(E->qacc_ws, qacc, sizeof(qacc));
    for (int i = 0; i < NV; i++) {
      E->v[i] += h_t * qacc_e[i];
      E->q[i] += h_t * E->v[i];
    }
    break;
  }
}

/* ------------------------------------------------------------------ task layer */
static double tolerance(double x, double lo, double hi, double margin) {
  if (x >= lo && x <= hi) return 1.0;
  double dd = (x < lo ? lo - x : x - hi) / margin;
  double scale = sqrt(-2.0 * log(0.1));
  return exp(-0.5 * (dd * scale) * (dd * scale));
}

/* rectangular assignment, min cost; rows n <= cols mm (e-maxx Hungarian). Returns sum of
 * tol(cost) over the n assigned pairs. */
static double hungarian_tol(int n, int mm, double c[][PS_MAX_NOTES > 10 ? PS_MAX_NOTES : 10]) {
  double u[12], v[PS_MAX_NOTES + 2], minv[PS_MAX_NOTES + 2];
  int p[PS_MAX_NOTES + 2], way[PS_MAX_NOTES + 2], used[PS_MAX_NOTES + 2];
  for (int i = 0; i <= n; i++) u[i] = 0;
  for (int j = 0; j <= mm; j++) { v[j] = 0; p[j] = 0; way[j] = 0; }
  for (int i = 1; i <= n; i++) {
    p[0] = i;
    int j0 = 0;
    for (int j = 0; j <= mm; j++) { minv[j] = INFINITY; used[j] = 0; }
    do {
      used[j0] = 1;
      int i0 = p[j0], j1 = 0;
      double delta = INFINITY;
      for (int j = 1; j <= mm; j++)
        if (!used[j]) {
          double cur = c[i0 - 1][j - 1] - u[i0] - v[j];
          if (cur < minv[j]) { minv[j] = cur; way[j] = j0; }
          if (minv[j] < delta) { delta = minv[j]; j1 = j; }
        }
      for (int j = 0; j <= mm; j++)
        if (used[j]) { u[p[j]] += delta; v[j] -= delta; }
        else minv[j] -= delta;
      j0 = j1;
    } while (p[j0] != 0);
    do { int j1 = way[j0]; p[j0] = p[j1]; j0 = j1; } while (j0);
  }
  double s = 0;
  for (int j = 1; j <= mm; j++)
    if (p[j]) s += tolerance(c[p[j] - 1][j - 1], 0.0, 0.01, 0.1);
  return s;
}

static v3 key_target(const model* m, const envdata* E, int k) {
  /* key geom xpos + [0.35*size_x, 0, 0.5*size_z] (piano_with_shadow_hands.py:310-313) */
  v3 p = E->keyc[k];
  p.v[0] += 0.35 * m->d.key_half[k][0];
  p.v[2] += 0.5 * m->d.key_half[k][2];
  return p;
}

static const float* goal_row(const ref_env* R, int t) { return R->goal + (size_t)t * (NK + 1); }

static void write_obs(ref_env* R, envdata* E, float* obs, int t_obs) {
  const ps_model_desc* d = &R->m.d;
  int L = R->cfg.n_steps_lookahead, o = 0;
  for (int j = 0; j <= L; j++)
    for (int k = 0; k <= NK; k++) {
      int t = t_obs + j;
      obs[o++] = t < R->T ? goal_row(R, t)[k] : 0.0f;
    }
  if (R->cfg.fingering_reward) {
    float fs[10] = {0};
    for (int i = 0; i < R->count[t_obs]; i++) {
      int f = R->fingers[t_obs * PS_MAX_NOTES + i];
      if (f < 5) fs[f < 0 ? f + 5 : f] = 1.0f;
      else fs[5 + f - 5] = 1.0f;
    }
    for (int i = 0; i < 10; i++) obs[o++] = fs[i];
  }
  for (int k = 0; k < NK; k++) obs[o++] = (float)E->norm_state[k];
  obs[o++] = (float)E->sustain;
  for (int h = 0; h < NH; h++)
    for (int j = 0; j < n_obs_joints(d, h); j++) obs[o++] = (float)E->q[NK + h * ND + d->dof_obs_order[h][j]];
}

static void key_state(const model* m, envdata* E) {
  for (int k = 0; k < NK; k++) {
    double lo = m->d.key_range[k][0], hi = m->d.key_range[k][1];
    double s = clampd(E->q[k], lo, hi);
    E->norm_state[k] = s / hi;
    E->activation[k] = fabs(s - hi) <= KEY_THRESHOLD;
  }
}

static void reset_env(ref_env* R, envdata* E, float* obs) {
  E->hand_dy = R->cfg.randomize_hand_positions
                    ? (double)ref_hand_offset_draw(R->seed, (int)((uint32_t)R->env_offset + (uint32_t)(E - R->e)), E->episode)
                    : 0.0;
  E->episode++;
  memset(E->q, 0, sizeof(E->q));
  memset(E->v, 0, sizeof(E->v));
  memset(E->qacc_ws, 0, sizeof(E->qacc_ws));
  memset(E->ctrl, 0, sizeof(E->ctrl));
  E->sustain = 0;
  E->t_idx = 0;
  E->last = 0;
  kinematics(&R->m, E);
  collide(&R->m, &R->cfg, E);
  key_state(&R->m, E);
  memset(E->terms, 0, sizeof(E->terms));
  memset(E->mus_acc, 0, sizeof(E->mus_acc));
  if (obs) write_obs(R, E, obs, 0);
}

/* sklearn.metrics.precision_recall_fscore_support(y_true, y_pred, average="binary",
 * zero_division=1) as the wrapper calls it (evaluation.py:135-140, 162-164): P = tp/(tp+fp),
 * R = tp/(tp+fn), F = 2tp/(2tp+fp+fn) (sklearn >= 1.3 form), each 1 when its denominator is 0 */
static void prf_counts(int tp, int fp, int fn, double* out) {
  out[0] = tp + fp ? (double)tp / (tp + fp) : 1.0;
  out[1] = tp + fn ? (double)tp / (tp + fn) : 1.0;
  out[2] = 2 * tp + fp + fn ? (double)(2 * tp) / (2 * tp + fp + fn) : 1.0;
}

void ref_prf(const uint8_t* y_true, const uint8_t* y_pred, int n, double* out) {
  int tp = 0, fp = 0, fn = 0;
  for (int i = 0; i < n; i++) {
    tp += y_true[i] && y_pred[i];
    fp += !y_true[i] && y_pred[i];
    fn += y_true[i] && !y_pred[i];
  }
  prf_counts(tp, fp, fn, out);
}

static void control_step(ref_env* R, envdata* E, const float* a, float* obs, float* rew, float* disc, uint8_t* st) {
  const model* m = &R->m;
  const ps_model_desc* d = &m->d;
  if (E->last) {
    reset_env(R, E, obs);
    *rew = 0.0f; *disc = 1.0f; *st = PS_FIRST;
    return;
  }
  /* the caller's row: actuator columns (an absent actuator: ctrl 0), then the sustain pedal */
  for (int h = 0; h < NH; h++)
    for (int u = 0; u < NA; u++) {
      const int col = act_col(d, h, u);
      E->ctrl[h * NA + u] = col >= 0 ? a[col] : 0.0;
    }
  E->sustain = a[n_action(d) - 1];
  for (int s = 0; s < d->n_substeps; s++) step_physics(m, &R->cfg, E);
  kinematics(m, E);   /* mj_step1 at the final state (legacy_step) */
  collide(m, &R->cfg, E);
  key_state(m, E);
  int sustain_act = E->sustain >= SUSTAIN_THRESHOLD;
  int t_cur = E->t_idx;  /* goal_current = goal at pre-increment t */
  const float* gc = goal_row(R, t_cur);
  E->t_idx += 1;
  int t_new = E->t_idx;
  int terminal = t_new == R->T;
  int failure = 0;
  for (int k = 0; k < NK; k++) if (gc[k] == 0.0f && E->activation[k]) failure = 1;
  /* MidiEvaluationWrapper.step (evaluation.py:65-86): ground truth = keys of the notes of
   * step t_cur (task._notes, the goal row) and task._sustains[t_cur]; prediction = the
   * piano's activation / sustain_activation after the step */
  {
    int tp = 0, fp = 0, fn = 0;
    for (int k = 0; k < NK; k++) {
      int g = gc[k] != 0.0f, a = E->activation[k] != 0;
      tp += g && a; fp += !g && a; fn += g && !a;
    }
    double m[PS_NMUSIC];
    prf_counts(tp, fp, fn, m);
    int sg = gc[NK] != 0.0f, sa = sustain_act;
    prf_counts(sg && sa, !sg && sa, sg && !sa, m + 3);
    for (int i = 0; i < PS_NMUSIC; i++) E->mus_acc[i] += m[i];
  }
  /* rewards */
  double kp = 0;
  int non = 0;
  double acc = 0;
  for (int k = 0; k < NK; k++)
    if (gc[k] != 0.0f) { acc += tolerance(gc[k] - E->norm_state[k], 0, 0.05, 0.5); non++; }
  if (non > 0) kp += 0.5 * (acc / non);
  kp += 0.5 * (1.0 - (double)failure);
  double sus = tolerance(gc[NK] - (double)sustain_act, 0, 0.05, 0.5);
  double energy = 0;
  for (int h = 0; h < NH; h++)
    for (int a2 = 0; a2 < NA; a2++) {
      int tg = d->act_target[h][a2];
      const double* vh = E->v + NK + h * ND;
      double vel = d->act_kind[h][a2] == 0 ? vh[tg]
                   : d->tendon_coef[h][tg][0] * vh[d->tendon_dof[h][tg][0]] + d->tendon_coef[h][tg][1] * vh[d->tendon_dof[h][tg][1]];
      energy += fabs(E->act_force[h * NA + a2]) * fabs(vel);
    }
  energy *= -R->cfg.energy_penalty_coef;
  double fing = 0;
  if (R->cfg.fingering_reward) {
    double sum = 0;
    int cnt = 0;
    for (int hand = 0; hand < 2; hand++)  /* rh list then lh list */
      for (int i = 0; i < R->count[t_cur]; i++) {
        int f = R->fingers[t_cur * PS_MAX_NOTES + i], k = R->keys[t_cur * PS_MAX_NOTES + i];
        int is_rh = f < 5;
        if (is_rh != (hand == 0)) continue;
        int site = is_rh ? (f < 0 ? f + 5 : f) : f - 5;
        v3 tip = site_pos(m, E, hand, site);
        sum += tolerance(nrm(sub(key_target(m, E, k), tip)), 0, 0.01, 0.1);
        cnt++;
      }
    fing = cnt ? sum / cnt : 0.0;
  } else {
    int keys[NK], K = 0;
    for (int k = 0; k < NK; k++) if (gc[k] != 0.0f) keys[K++] = k;
    if (K == 0) fing = 1.0;
    else {
      v3 tips[10];
      for (int i = 0; i < 5; i++) { tips[i] = site_pos(m, E, 1, i); tips[5 + i] = site_pos(m, E, 0, i); }
      int KK = K > PS_MAX_NOTES ? PS_MAX_NOTES : K;
      double c[PS_MAX_NOTES > 10 ? PS_MAX_NOTES : 10][PS_MAX_NOTES > 10 ? PS_MAX_NOTES : 10];
      double s;
      if (KK <= 10) {
        for (int j = 0; j < KK; j++)
          for (int i = 0; i < 10; i++) c[j][i] = nrm(sub(key_target(m, E, keys[j]), tips[i]));
        s = hungarian_tol(KK, 10, c);
        fing = s / KK;
      } else {
        for (int i = 0; i < 10; i++)
          for (int j = 0; j < KK; j++) c[i][j] = nrm(sub(key_target(m, E, keys[j]), tips[i]));
        s = hungarian_tol(10, KK, c);
        fing = s / 10;
      }
    }
  }
  double fore = 0;
  if (R->cfg.forearm_reward) {
    int hit = 0;
    for (int c = 0; c < E->ncon; c++) {
      const contact* cc = &E->con[c];
      if (cc->kind != 2) continue;
      /* has_collision(rh root-body geoms, lh root-body geoms), piano_with_shadow_hands.py:251-259 */
      if (cc->h1 != cc->h2 && cc->b1 == 0 && cc->b2 == 0) hit = 1;
    }
    fore = hit ? 0.0 : 0.5;
  }
  E->terms[PS_TERM_KEY_PRESS] = kp;
  E->terms[PS_TERM_SUSTAIN] = sus;
  E->terms[PS_TERM_ENERGY] = energy;
  E->terms[PS_TERM_FINGERING] = fing;
  E->terms[PS_TERM_FOREARM] = fore;
  double total = kp + sus + energy + fing + fore;
  double discount = 1.0;
  if (!terminal && R->cfg.wrong_press_termination && failure) { terminal = 1; discount = 0.0; }
  /* observation at t_new; at t_new == T the goal/fingering observables keep their
   * previous value (piano_with_shadow_hands.py:377-378, 392-393) */
  write_obs(R, E, obs, t_new < R->T ? t_new : t_new - 1);
  *rew = (float)total;
  *disc = (float)discount;
  *st = terminal ? PS_LAST : PS_MID;
  E->last = terminal;
  if (terminal) {  /* episode means (np.mean over the episode's steps, evaluation.py:142-144) */
    for (int i = 0; i < PS_NMUSIC; i++) E->mus_ep[i] = E->mus_acc[i] / t_new;
    E->mus_cnt += 1;
  }
}

/* ------------------------------------------------------------------ API */
ref_env* ref_create(const ps_model_desc* md, const ps_song_desc* song, const ps_task_cfg* cfg, int n) {
  ref_env* R = (ref_env*)calloc(1, sizeof(ref_env));
  R->m.d = *md;
  derive(&R->m);
  R->cfg = *cfg;
  if (R->cfg.max_contacts > MAXCON) R->cfg.max_contacts = MAXCON;
  R->T = song->T;
  R->goal = (float*)malloc(sizeof(float) * song->T * (NK + 1));
  memcpy(R->goal, song->goal, sizeof(float) * song->T * (NK + 1));
  R->count = (int32_t*)malloc(sizeof(int32_t) * song->T);
  memcpy(R->count, song->count, sizeof(int32_t) * song->T);
  R->keys = (int32_t*)malloc(sizeof(int32_t) * song->T * PS_MAX_NOTES);
  memcpy(R->keys, song->keys, sizeof(int32_t) * song->T * PS_MAX_NOTES);
  R->fingers = (int32_t*)malloc(sizeof(int32_t) * song->T * PS_MAX_NOTES);
  memcpy(R->fingers, song->fingers, sizeof(int32_t) * song->T * PS_MAX_NOTES);
  R->n = n;
  R->e = (envdata*)calloc((size_t)n, sizeof(envdata));
  for (int i = 0; i < n; i++) {
    reset_env(R, &R->e[i], NULL);
    R->e[i].episode = 0;  /* as a fresh ps_create: the first ps_reset draws episode 0 */
    R->e[i].hand_dy = 0.0;
  }
  return R;
}

void ref_destroy(ref_env* R) {
  if (!R) return;
  free(R->goal); free(R->count); free(R->keys); free(R->fingers); free(R->e); free(R);
}

int ref_obs_dim(const ref_env* R) {
  return (R->cfg.n_steps_lookahead + 1) * (NK + 1) + (R->cfg.fingering_reward ? 10 : 0) + NK + 1 +
         n_obs_joints(&R->m.d, 0) + n_obs_joints(&R->m.d, 1);
}
int ref_action_dim(const ref_env* R) { return n_action(&R->m.d); }

void ref_reset(ref_env* R, const uint8_t* mask, float* obs) {
  int od = ref_obs_dim(R);
  for (int i = 0; i < R->n; i++)
    if (!mask || mask[i]) reset_env(R, &R->e[i], obs + (size_t)i * od);
}

void ref_step(ref_env* R, const float* action, float* obs, float* rew, float* disc, uint8_t* st) {
  int od = ref_obs_dim(R);
  for (int i = 0; i < R->n; i++)
    control_step(R, &R->e[i], action + (size_t)i * n_action(&R->m.d), obs + (size_t)i * od, rew + i, disc + i, st + i);
}

/* The all-cores CPU baseline: the same per-env step, envs spread over
 * OpenMP threads (envs are independent; per-step scratch is thread-local). */
void ref_step_threads(ref_env* R, const float* action, float* obs, float* rew, float* disc, uint8_t* st,
                      int nthreads) {
  int od = ref_obs_dim(R);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
  for (int i = 0; i < R->n; i++)
    control_step(R, &R->e[i], action + (size_t)i * n_action(&R->m.d), obs + (size_t)i * od, rew + i, disc + i, st + i);
}

void ref_get_state(const ref_env* R, double* q, double* v, double* qacc_ws, double* ctrl, double* sustain,
                   int32_t* t_idx, uint8_t* last) {
  for (int i = 0; i < R->n; i++) {
    const envdata* E = &R->e[i];
    if (q) memcpy(q + (size_t)i * NV, E->q, sizeof(E->q));
    if (v) memcpy(v + (size_t)i * NV, E->v, sizeof(E->v));
    if (qacc_ws) memcpy(qacc_ws + (size_t)i * NV, E->qacc_ws, sizeof(E->qacc_ws));
    if (ctrl) memcpy(ctrl + (size_t)i * PS_NU, E->ctrl, sizeof(E->ctrl));
    if (sustain) sustain[i] = E->sustain;
    if (t_idx) t_idx[i] = E->t_idx;
    if (last) last[i] = (uint8_t)E->last;
  }
}

void ref_set_state(ref_env* R, const double* q, const double* v, const double* qacc_ws, const double* ctrl,
                   const double* sustain, const int32_t* t_idx, const uint8_t* last) {
  for (int i = 0; i < R->n; i++) {
    envdata* E = &R->e[i];
    if (q) memcpy(E->q, q + (size_t)i * NV, sizeof(E->q));
    if (v) memcpy(E->v, v + (size_t)i * NV, sizeof(E->v));
    if (qacc_ws) memcpy(E->qacc_ws, qacc_ws + (size_t)i * NV, sizeof(E->qacc_ws));
    if (ctrl) memcpy(E->ctrl, ctrl + (size_t)i * PS_NU, sizeof(E->ctrl));
    if (sustain) E->sustain = sustain[i];
    if (t_idx) E->t_idx = t_idx[i];
    if (last) E->last = last[i];
    kinematics(&R->m, E);
    collide(&R->m, &R->cfg, E);
    key_state(&R->m, E);
  }
}

void ref_set_applied(ref_env* R, const double* qfrc) {
  for (int i = 0; i < R->n; i++) {
    if (qfrc) memcpy(R->e[i].applied, qfrc + (size_t)i * NV, sizeof(R->e[i].applied));
    else memset(R->e[i].applied, 0, sizeof(R->e[i].applied));
  }
}

void ref_reward_terms(const ref_env* R, double* terms) {
  for (int i = 0; i < R->n; i++) memcpy(terms + (size_t)i * PS_NTERMS, R->e[i].terms, sizeof(double) * PS_NTERMS);
}

void ref_fingertips(const ref_env* R, double* xpos) {
  for (int i = 0; i < R->n; i++)
    for (int h = 0; h < NH; h++)
      for (int s = 0; s < PS_NFINGER; s++) {
        v3 p = site_pos(&R->m, &R->e[i], h, s);
        for (int c = 0; c < 3; c++) xpos[(((size_t)i * NH + h) * PS_NFINGER + s) * 3 + c] = p.v[c];
      }
}

void ref_musical_metrics(const ref_env* R, double* episode, int32_t* episodes) {
  for (int i = 0; i < R->n; i++) {
    if (episode) memcpy(episode + (size_t)i * PS_NMUSIC, R->e[i].mus_ep, sizeof(double) * PS_NMUSIC);
    if (episodes) episodes[i] = R->e[i].mus_cnt;
  }
}

void ref_contact_count(const ref_env* R, int32_t* ncon) {
  for (int i = 0; i < R->n; i++) ncon[i] = R->e[i].ncon;
}

void ref_set_seed(ref_env* R, uint64_t seed) { R->seed = seed; }
/* global id of env 0 (ps_set_env_offset): draws keyed by global env id */
void ref_set_env_offset(ref_env* R, int64_t off) { R->env_offset = off; }
void ref_get_hand_offset(const ref_env* R, double* dy, int32_t* episode) {
  for (int i = 0; i < R->n; i++) {
    if (dy) dy[i] = R->e[i].hand_dy;
    if (episode) episode[i] = R->e[i].episode;
  }
}
void ref_set_hand_offset(ref_env* R, const double* dy) {
  for (int i = 0; i < R->n; i++) {
    envdata* E = &R->e[i];
    E->hand_dy = dy[i];
    kinematics(&R->m, E);
    collide(&R->m, &R->cfg, E);
    key_state(&R->m, E);
  }
}

/* Solver study hooks (see ref_pgs_mode above). */
void ref_set_solver(int mode, double tol, int maxit) {
  ref_pgs_mode = mode;
  ref_pgs_tol = tol;
  ref_pgs_maxit = maxit;
}
void ref_stats_reset(void) {
  memset(ref_rows_hist, 0, sizeof(ref_rows_hist));
  memset(ref_con_hist, 0, sizeof(ref_con_hist));
  memset(ref_found_hist, 0, sizeof(ref_found_hist));
  memset(ref_cap_events, 0, sizeof(ref_cap_events));
  memset(ref_newton_hist, 0, sizeof(ref_newton_hist));
  memset(ref_warnings_total, 0, sizeof(ref_warnings_total));
  ref_iter_total = ref_substeps_total = 0;
}
void ref_newton_hist_get(long* out) { memcpy(out, ref_newton_hist, sizeof(ref_newton_hist)); }
/* found [REF_HIST], constraint rows [REF_HIST], kept contacts [MAXCON + 2], misc = {substeps
 * with contacts dropped, solver iterations (Newton) or sweeps (study PGS), substeps, warnings} */
void ref_stats_get(long* found, long* rows, long* cons, long* misc) {
  memcpy(found, ref_found_hist, sizeof(ref_found_hist));
  memcpy(rows, ref_rows_hist, sizeof(ref_rows_hist));
  memcpy(cons, ref_con_hist, sizeof(ref_con_hist));
  misc[0] = ref_cap_events[0];
  misc[1] = ref_iter_total;
  misc[2] = ref_substeps_total;
  misc[3] = ref_warnings_total[0] + ref_warnings_total[1] + ref_warnings_total[2];
}
/* mj_checkPos / Vel / Acc resets of each env since create, [n][PS_NWARN] (ps_warnings) */
void ref_warnings(const ref_env* R, int32_t* out) {
  for (int i = 0; i < R->n; i++)
    for (int w = 0; w < PS_NWARN; w++) out[i * PS_NWARN + w] = R->e[i].warnings[w];
}

/* Single-substep hook for teacher-forced physics parity (no task layer). */
void ref_physics_substep(ref_env* R) {
  for (int i = 0; i < R->n; i++) step_physics(&R->m, &R->cfg, &R->e[i]);
}

/* Exposed helpers for unit tests */
double ref_tolerance(double x, double lo, double hi, double margin) { return tolerance(x, lo, hi, margin); }
double ref_assignment_tol(int n, int mm, const double* cost) {
  double c[PS_MAX_NOTES > 10 ? PS_MAX_NOTES : 10][PS_MAX_NOTES > 10 ? PS_MAX_NOTES : 10];
  for (int i = 0; i < n; i++)
    for (int j = 0; j < mm; j++) c[i][j] = cost[i * mm + j];
  return hungarian_tol(n, mm, c);
}

/* Debug hook for tests: dense mass matrix (before factorization) and bias of env i. */
void ref_debug_dynamics(ref_env* R, int i, double* Mout, double* bias) {
  envdata* E = &R->e[i];
  kinematics(&R->m, E);
  dynamics(&R->m, &R->cfg, E);
  memset(Mout, 0, sizeof(double) * NV * NV);
  for (int k = 0; k < NK; k++) Mout[k * NV + k] = E->Mk[k];
  for (int h = 0; h < NH; h++)
    for (int a = 0; a < ND; a++)
      for (int b = 0; b < ND; b++) Mout[(NK + h * ND + a) * NV + NK + h * ND + b] = E->M[h][a][b];
  memcpy(bias, E->bias, sizeof(double) * NV);
}
/* Body COM positions [2][25][3] of env i (after kinematics). */
void ref_debug_com(ref_env* R, int i, double* com) {
  envdata* E = &R->e[i];
  kinematics(&R->m, E);
  for (int h = 0; h < NH; h++)
    for (int b = 0; b < NB; b++)
      for (int c = 0; c < 3; c++) com[(h * NB + b) * 3 + c] = E->com[h][b].v[c];
}
/* Contacts of env i: info[c] = {kind, key, g1, g2}, data[c] = {dist, pos[3], n[3]} */
int ref_debug_contacts(ref_env* R, int i, int32_t* info, double* data) {
  envdata* E = &R->e[i];
  for (int c = 0; c < E->ncon; c++) {
    info[4 * c] = E->con[c].kind; info[4 * c + 1] = E->con[c].key;
    info[4 * c + 2] = E->con[c].g1; info[4 * c + 3] = E->con[c].g2;
    data[7 * c] = E->con[c].dist;
    for (int k = 0; k < 3; k++) { data[7 * c + 1 + k] = E->con[c].pos.v[k]; data[7 * c + 4 + k] = E->con[c].n.v[k]; }
  }
  return E->ncon;
}

/* The world shape of a collider of env i (test access; tools/contact_diff.py): g < NCAPS a
 * capsule, NCAPS <= g < NCAPS + NH * NX an extra collider, g = -1 - k key k, g = -1000 the
 * base; packed as unpack_shape reads it (23 doubles); *verts / *nv the hull's vertices. */
int ref_debug_shape(ref_env* R, int i, int g, double* out, const double** verts, int* nv) {
  const envdata* E = &R->e[i];
  const ps_model_desc* d = &R->m.d;
  shape s;
  m3 I3 = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
  if (g == -1000) s = box_shape(mk(d->base_pos[0], d->base_pos[1], d->base_pos[2]), I3, d->base_half);
  else if (g < 0) s = box_shape(E->keyc[-1 - g], E->keyR[-1 - g], d->key_half[-1 - g]);
  else if (g < NCAPS) s = capsule_shape(E, g / NG, g % NG, d);
  else s = extra_shape(E, (g - NCAPS) / NX, (g - NCAPS) % NX, d);
  memset(out, 0, 23 * sizeof(double));
  out[0] = s.type;
  for (int k = 0; k < 3; k++) {
    out[1 + k] = s.c.v[k]; out[13 + k] = s.p0.v[k]; out[16 + k] = s.p1.v[k]; out[20 + k] = s.hs[k];
  }
  for (int k = 0; k < 9; k++) out[4 + k] = s.R.m[k];
  out[19] = s.r;
  *verts = s.type == PS_GEOM_HULL ? &s.vert[0][0] : NULL;
  *nv = s.type == PS_GEOM_HULL ? s.nvert : 0;
  return 0;
}

/* Narrow phase of two world colliders (test access). A shape is packed as 23 doubles: type
 * (0 capsule, PS_GEOM_BOX, PS_GEOM_HULL), centre (3), row-major rotation (9), capsule p0 (3),
 * p1 (3), radius, box half sizes (3); hull vertices (geom frame) come separately. A is geom1.
 * Writes up to 4 contacts as pos (3), normal geom1 -> geom2 (3), dist; returns their number.
 * A capsule A with a box B is collided as the kernel's hand-hand pairs do: the box becomes
 * geom1 (the normal then points box -> capsule). */
static shape unpack_shape(const double* p, const double* verts, int nv) {
  shape s;
  memset(&s, 0, sizeof(s));
  s.type = (int)p[0];
  s.c = mk(p[1], p[2], p[3]);
  for (int i = 0; i < 9; i++) s.R.m[i] = p[4 + i];
  s.p0 = mk(p[13], p[14], p[15]);
  s.p1 = mk(p[16], p[17], p[18]);
  s.r = p[19];
  for (int i = 0; i < 3; i++) s.hs[i] = p[20 + i];
  s.vert = (const double(*)[3])verts;
  s.nvert = nv;
  s.rb = 0.0;
  for (int i = 0; i < nv; i++) s.rb = fmax(s.rb, nrm(mk(verts[3 * i], verts[3 * i + 1], verts[3 * i + 2])));
  if (s.type == 0) s.c = scl(add(s.p0, s.p1), 0.5);
  return s;
}
int ref_narrow(const double* pa, const double* va, int nva, const double* pb, const double* vb, int nvb, double* out) {
  static envdata E;
  E.ncon = 0;
  E.nfound = 0;
  shape A = unpack_shape(pa, va, nva), B = unpack_shape(pb, vb, nvb);
  contact proto;
  memset(&proto, 0, sizeof(proto));
  proto.kind = 2;
  if (A.type == 0 && B.type == PS_GEOM_BOX) capsule_box(&E, 4, proto, A.p0, A.p1, A.r, B.c, B.R, B.hs);
  else extra_pair(&E, 4, proto, &A, &B);
  for (int i = 0; i < E.ncon; i++) {
    for (int k = 0; k < 3; k++) { out[7 * i + k] = E.con[i].pos.v[k]; out[7 * i + 3 + k] = E.con[i].n.v[k]; }
    out[7 * i + 6] = E.con[i].dist;
  }
  return E.ncon;
}
