// pianosim.hip - MI355X (gfx950) batched PianoWithShadowHands step/reset + C-ABI.
//
// Device code: prims.h (math, wave primitives, narrow phase) and kernel_v2.inc (the
// step kernel, one wavefront per env, lane-owned registers, LDS for exchange only).
// The algorithm and every result-affecting ordering are stated sequentially in the CPU
// checker; this file adds the host side: descriptor -> device tables,
// buffers, launches, and the extern "C" entry points of include/pianosim.h.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "devmodel.h"
#include "prims.h"
#include "collide_x.h"

using namespace ps;

#include "kernel_v2.inc"

// ------------------------------------------------------------------ host side
static thread_local std::string g_err;
static int fail(const std::string& s) {
  g_err = s;
  return -1;
}
#define HIPCHK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct ps_env {
  int n, device, obs_dim, action_dim;
  int64_t env_offset;       // global id of local env 0 (Philox key of the per-env draws)
  int full_cpl;             // PIANOSIM_DEBUG_FULL_COUPLED: every coupled solve on the 28-column C block
  ps_task_cfg cfg;
  DevModel* d_model;
  int T;
  float* d_goal;
  int *d_count, *d_keys, *d_fingers;
  float *qpos, *qvel, *qws, *ctrl, *sustain, *applied, *terms, *tips;
  int *t_idx, *ncon;
  float *mus_acc, *mus_ep;  // MidiEvaluationWrapper: running sums of this episode, last episode
  int* mus_cnt;             // finished episodes per env
  int* order;               // dispatch order of the step launch (longest-expected first)
  bool ordered;
  uint8_t* last;
  bool applied_on;
  float* hand_dy;           // randomize_hand_positions: this episode's y shift of both hands
  int* episode;             // resets so far per env (the draw counter)
  int* stats;               // [N][PS_NSTATS] solver / cap counters of the last step
  int* warnings;            // [N][PS_NWARN] physics warnings since create
  float* park;              // [N][PARK_WORDS][64] kernel scratch (lane state around the Newton solve)
  uint64_t seed;
  bool has_x;               // box / hull colliders: the pianosim_kernel<true> instantiation
  int wave_slots;           // SIMDs of the device: a step launch of at most this many envs runs one
                            // wave per SIMD and takes the one-wave (no-scratch) instantiation
  Contact* con_out;         // [N][MAXCON] contact lists of the last step (ps_record_contacts)
};

// Every entry point that touches device memory or launches binds the handle's device for its
// duration and restores the caller's afterwards: two handles on two GPUs in one process, or a
// null/default stream, never reach the wrong device ("handles are independent", pianosim.h).
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
#define GUARD(E)                                                                  \
  DeviceGuard guard_((E)->device);                                                \
  if (!guard_.ok) return fail("hipSetDevice(" + std::to_string((E)->device) + ") failed")

static void quat2mat_h(const double* q, float* R) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  double w = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
  double M[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                 2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                 2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
  for (int i = 0; i < 9; i++) R[i] = (float)M[i];
}

// Derive the flattened device model + topology tables from the descriptor.
// An enclosing capsule of a hull's vertices (geom frame), the narrow phase's pre-reject: for
// each frame axis, the segment along it through the centre of the vertices' extent across it,
// radius the largest distance across, ends just long enough to hold every vertex; the axis of
// the smallest capsule is kept. out = p0, p1, radius (padded by 1e-6 relative + 1e-7 m).
static void enclosing_capsule(const double (*v)[3], int n, float* out) {
  double best = INFINITY;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) { lo[k] = fmin(lo[k], v[i][k]); hi[k] = fmax(hi[k], v[i][k]); }
  for (int a = 0; a < 3; a++) {
    const int b = (a + 1) % 3, c = (a + 2) % 3;
    const double cb = 0.5 * (lo[b] + hi[b]), cc = 0.5 * (lo[c] + hi[c]);
    double r = 0.0;
    for (int i = 0; i < n; i++) r = fmax(r, hypot(v[i][b] - cb, v[i][c] - cc));
    double t0 = INFINITY, t1 = -INFINITY;
    for (int i = 0; i < n; i++) {
      const double rho = hypot(v[i][b] - cb, v[i][c] - cc), s = sqrt(fmax(r * r - rho * rho, 0.0));
      t0 = fmin(t0, v[i][a] + s);
      t1 = fmax(t1, v[i][a] - s);
    }
    if (t0 > t1) t0 = t1 = 0.5 * (t0 + t1);  // a sphere holds them all
    const double vol = M_PI * r * r * (t1 - t0) + 4.0 / 3.0 * M_PI * r * r * r;
    if (vol < best) {
      best = vol;
      double p0[3], p1[3];
      p0[a] = t0; p1[a] = t1; p0[b] = p1[b] = cb; p0[c] = p1[c] = cc;
      for (int k = 0; k < 3; k++) { out[k] = (float)p0[k]; out[3 + k] = (float)p1[k]; }
      out[6] = (float)(r * (1.0 + 1e-6) + 1e-7);
      out[7] = 0.f;
    }
  }
}

static int build_dev_model(const ps_model_desc* d, DevModel* m) {
  memset(m, 0, sizeof(*m));
  m->timestep = (float)d->timestep;
  m->nsub = d->n_substeps;
  if (m->nsub < 1) return fail("n_substeps must be >= 1");
  for (int i = 0; i < 3; i++) m->grav[i] = (float)d->gravity[i];
  for (int i = 0; i < 3; i++) m->hgrav[i] = (float)(d->gravity[i] * (1.0 - d->hand_gravcomp));
  for (int k = 0; k < NK; k++) {
    for (int i = 0; i < 3; i++) {
      m->key_pos[k][i] = (float)d->key_pos[k][i];
      m->key_half[k][i] = (float)d->key_half[k][i];
      m->key_anchor[k][i] = (float)d->key_anchor[k][i];
    }
    double M = d->key_inertia[k] + d->key_armature[k];
    m->key_mass[k] = (float)d->key_mass[k];
    m->key_Minv[k] = (float)(1.0 / M);
    m->key_Mhinv[k] = (float)(1.0 / (M + d->timestep * d->key_damping[k]));
    m->key_damp[k] = (float)d->key_damping[k];
    m->key_stiff[k] = (float)d->key_stiffness[k];
    m->key_sref[k] = (float)d->key_springref[k];
    m->key_lo[k] = (float)d->key_range[k][0];
    m->key_hi[k] = (float)d->key_range[k][1];
    m->key_ylo[k] = (float)(d->key_pos[k][1] - d->key_half[k][1]);
    m->key_yhi[k] = (float)(d->key_pos[k][1] + d->key_half[k][1]);
    m->key_binv[k] = (float)d->key_body_invweight[k];
    m->key_dinv[k] = (float)d->key_dof_invweight[k];
    if (k > 0 && (m->key_ylo[k] < m->key_ylo[k - 1] || m->key_yhi[k] < m->key_yhi[k - 1]))
      return fail("keys are not sorted along y");
  }
  for (int i = 0; i < 3; i++) { m->base_pos[i] = (float)d->base_pos[i]; m->base_half[i] = (float)d->base_half[i]; }
  for (int i = 0; i < 2; i++) {
    m->pc_solref[i] = (float)d->piano_contact.solref[i];
    m->hc_solref[i] = (float)d->hand_contact.solref[i];
    m->lim_solref[i] = (float)d->limit_solref[i];
  }
  for (int i = 0; i < 5; i++) {
    m->pc_solimp[i] = (float)d->piano_contact.solimp[i];
    m->hc_solimp[i] = (float)d->hand_contact.solimp[i];
    m->lim_solimp[i] = (float)d->limit_solimp[i];
  }
  m->pc_fric = (float)d->piano_contact.friction;
  for (int i = 0; i < 2; i++) m->fr_solref[i] = (float)d->friction_solref[i];
  for (int i = 0; i < 5; i++) m->fr_solimp[i] = (float)d->friction_solimp[i];
  m->hc_fric = (float)d->hand_contact.friction;
  // bodies
  int depth_b[NBT];
  for (int h = 0; h < NH; h++)
    for (int b = 0; b < NB; b++) {
      int B = h * NB + b, p = d->body_parent[h][b];
      if (p >= b) return fail("bodies must be in tree order");
      m->body_parent[B] = p < 0 ? -1 : h * NB + p;
      depth_b[B] = p < 0 ? 0 : depth_b[h * NB + p] + 1;
      for (int i = 0; i < 3; i++) {
        m->body_pos[B][i] = (float)d->body_pos[h][b][i];
        m->body_ipos[B][i] = (float)d->body_ipos[h][b][i];
      }
      quat2mat_h(d->body_quat[h][b], m->body_Q[B]);
      m->body_mass[B] = (float)d->body_mass[h][b];
      for (int i = 0; i < 6; i++) m->body_I[B][i] = (float)d->body_inertia[h][b][i];
      m->body_binv[B] = (float)d->body_invweight[h][b];
      m->body_dof[B] = -1;
    }
  int maxlev = 0;
  for (int B = 0; B < NBT; B++) maxlev = depth_b[B] > maxlev ? depth_b[B] : maxlev;
  if (maxlev + 1 > MAXLEV) return fail("body tree too deep");
  m->nlev = maxlev + 1;
  int n = 0;
  for (int L = 0; L <= maxlev; L++) {
    m->lev_start[L] = n;
    for (int B = 0; B < NBT; B++)
      if (depth_b[B] == L) m->lev_body[n++] = B;
    if (n - m->lev_start[L] > 64) return fail("too many bodies in one level");
  }
  m->lev_start[maxlev + 1] = n;
  for (int B = 0; B < NBT; B++) {
    int p = m->body_parent[B];
    if (p >= 0) {
      if (m->body_nchild[p] >= MAXCHILD) return fail("too many children");
      m->body_child[p][m->body_nchild[p]++] = B;
    }
  }
  // dofs
  for (int h = 0; h < NH; h++)
    for (int j = 0; j < ND; j++) {
      int g = h * ND + j, B = h * NB + d->dof_body[h][j];
      m->dof_body[g] = B;
      m->dof_type[g] = d->dof_type[h][j];
      m->dof_limited[g] = d->dof_limited[h][j];
      for (int i = 0; i < 3; i++) m->dof_axis[g][i] = (float)d->dof_axis[h][j][i];
      m->dof_lo[g] = (float)d->dof_range[h][j][0];
      m->dof_hi[g] = (float)d->dof_range[h][j][1];
      m->dof_damp[g] = (float)d->dof_damping[h][j];
      m->dof_arm[g] = (float)d->dof_armature[h][j];
      m->dof_dinv[g] = (float)d->dof_invweight[h][j];
      if (!(d->dof_frictionloss[h][j] >= 0.0)) return fail("negative dof_frictionloss");
      m->dof_floss[g] = (float)d->dof_frictionloss[h][j];
      if (m->body_dof[B] < 0) m->body_dof[B] = g;
      else if (m->body_dof[B] + m->body_ndof[B] != g) return fail("dofs of a body must be contiguous");
      m->body_ndof[B]++;
      m->dof_act[g] = -1;
      if (d->dof_locked[h][j]) {  // a joint the reference's hand lacks: held at 0, no force / row
        m->dof_lockmask |= 1ull << g;
        m->dof_limited[g] = 0;
        m->dof_floss[g] = 0.f;
        m->dof_damp[g] = 0.f;
      }
    }
  m->n_obsj = 0;
  for (int h = 0; h < NH; h++) {
    const int nj = d->n_obs_joints[h] ? d->n_obs_joints[h] : ND;
    if (nj < 0 || nj > ND) return fail("n_obs_joints out of range");
    for (int j = 0; j < nj; j++) {
      const int dof = d->dof_obs_order[h][j];
      if (dof < 0 || dof >= ND) return fail("dof_obs_order out of range");
      if (d->dof_locked[h][dof]) return fail("joints_pos lists a locked dof");
      m->obs_dof[m->n_obsj++] = h * ND + dof;
    }
  }
  for (int B = 0; B < NBT; B++) {
    if (m->body_parent[B] >= 0 && m->body_ndof[B] != 1) return fail("non-root bodies need exactly one hinge");
    if (m->body_parent[B] >= 0 && m->dof_type[m->body_dof[B]] != 0) return fail("non-root dofs must be hinges");
    if (m->body_parent[B] < 0)
      for (int j = 0; j < m->body_ndof[B]; j++)
        if (m->dof_type[m->body_dof[B] + j] != 1) return fail("root dofs must be slides");
  }
  // dof parent / ancestors / depth / descendants
  int dpar[NDT];
  for (int g = 0; g < NDT; g++) {
    int B = m->dof_body[g];
    if (g > m->body_dof[B]) { dpar[g] = g - 1; continue; }
    int p = m->body_parent[B], par = -1;
    while (p >= 0) {
      if (m->body_ndof[p] > 0) { par = m->body_dof[p] + m->body_ndof[p] - 1; break; }
      p = m->body_parent[p];
    }
    dpar[g] = par;
    // the kernel's chain-row L^-T (row_LT_chain) relies on ancestors having lower indices
    if (par >= g) return fail("dofs are not in tree order");
  }
  int maxdep = 0;
  for (int g = 0; g < NDT; g++) {
    int a = 0;
    for (int x = g; x >= 0; x = dpar[x]) {
      if (a >= MAXDEP) return fail("dof tree too deep");
      m->dof_anc[g][a++] = x;
      m->dof_ancmask[g] |= 1ull << x;
    }
    for (int r = a; r < MAXDEP; r++) m->dof_anc[g][r] = -1;
    m->dof_depth[g] = a - 1;
    maxdep = a - 1 > maxdep ? a - 1 : maxdep;
  }
  for (int g = 0; g < NDT; g++)
    for (int a = 1; a <= m->dof_depth[g]; a++) {
      int i = m->dof_anc[g][a];
      m->dof_desc[i][m->dof_ndesc[i]++] = g;
      m->dof_descmask[i] |= 1ull << g;
    }
  m->ndepth = maxdep + 1;
  n = 0;
  for (int dd = 0; dd <= maxdep; dd++) {
    m->dep_start[dd] = n;
    for (int g = 0; g < NDT; g++)
      if (m->dof_depth[g] == dd) m->dep_dof[n++] = g;
  }
  m->dep_start[maxdep + 1] = n;
  for (int B = 0; B < NBT; B++) {
    uint64_t mask = 0;
    for (int x = B; x >= 0; x = m->body_parent[x])
      for (int j = 0; j < m->body_ndof[x]; j++) mask |= 1ull << (m->body_dof[x] + j);
    m->body_pathmask[B] = mask & ~m->dof_lockmask;  // no Jacobian entry on a locked dof
  }
  int t = 0;
  for (int a = 1; a < MAXDEP; a++)
    for (int b = a; b < MAXDEP; b++) { m->tri_a[t] = a; m->tri_b[t] = b; t++; }
  // ordering must be: all pairs with b <= dk come first for any dk -> sort by b
  {
    int ta[NTRI], tb[NTRI], c = 0;
    for (int b = 1; b < MAXDEP; b++)
      for (int a = 1; a <= b; a++) { ta[c] = a; tb[c] = b; c++; }
    for (int i = 0; i < NTRI; i++) { m->tri_a[i] = ta[i]; m->tri_b[i] = tb[i]; }
  }
  // actuators + tendons; the caller's action row layout
  m->n_action = d->n_action > 0 ? d->n_action : PS_NACTION;
  if (m->n_action > PS_NACTION) return fail("n_action out of range");
  uint64_t cols = 0;
  for (int h = 0; h < NH; h++)
    for (int a = 0; a < NA; a++) {
      int A = h * NA + a, tg = d->act_target[h][a];
      const int col = d->n_action > 0 ? d->act_column[h][a] : A;
      if (col < -1 || col >= m->n_action - 1) return fail("act_column out of range");
      if (col >= 0 && ((cols >> col) & 1)) return fail("two actuators in one action column");
      if (col >= 0) cols |= 1ull << col;
      m->act_src[A] = col;
      m->act_kind[A] = d->act_kind[h][a];
      if (d->act_kind[h][a] == 0) {
        m->act_dof0[A] = h * ND + tg;
        m->act_c0[A] = 1.f;
        m->act_dof1[A] = h * ND + tg;
        m->act_c1[A] = 0.f;
      } else {
        m->act_dof0[A] = h * ND + d->tendon_dof[h][tg][0];
        m->act_c0[A] = (float)d->tendon_coef[h][tg][0];
        m->act_dof1[A] = h * ND + d->tendon_dof[h][tg][1];
        m->act_c1[A] = (float)d->tendon_coef[h][tg][1];
      }
      m->act_kp[A] = col >= 0 ? (float)d->act_kp[h][a] : 0.f;  // an absent actuator: no force
      m->act_clo[A] = (float)d->act_ctrlrange[h][a][0];
      m->act_chi[A] = (float)d->act_ctrlrange[h][a][1];
      m->act_flim[A] = d->act_forcelimited[h][a];
      m->act_flo[A] = (float)d->act_forcerange[h][a][0];
      m->act_fhi[A] = (float)d->act_forcerange[h][a][1];
      int dofs[2] = {m->act_dof0[A], m->act_dof1[A]};
      float cs[2] = {m->act_c0[A], m->act_c1[A]};
      if (col < 0) continue;  // an absent actuator drives nothing
      for (int i = 0; i < (m->act_kind[A] == 1 ? 2 : 1); i++) {
        if (m->dof_act[dofs[i]] >= 0) return fail("a dof may be driven by at most one actuator");
        m->dof_act[dofs[i]] = A;
        m->dof_act_coef[dofs[i]] = cs[i];
      }
    }
  // every action column before the sustain pedal drives an actuator: a gap would be an input the
  // kernel ignores while ps_env_action_dim reports it
  if (__builtin_popcountll(cols) != m->n_action - 1)
    return fail("act_column must fill columns 0 .. n_action - 2 (" + std::to_string(__builtin_popcountll(cols)) +
                " actuator columns for n_action " + std::to_string(m->n_action) + ")");
  // geoms, sites, pairs
  for (int h = 0; h < NH; h++)
    for (int g = 0; g < NG; g++) {
      int G = h * NG + g;
      if (d->geom_body[h][g] >= NB) return fail("capsule body out of range");
      if (d->geom_body[h][g] < 0) {
        // unused slot: a point at the hand root with radius -1, whose inverted AABB never
        // overlaps a key or the base; no capsule pair may name it
        m->geom_body[G] = h * NB;
        for (int i = 0; i < 3; i++) { m->geom_pos[G][i] = 0.f; m->geom_axis[G][i] = i == 2 ? 1.f : 0.f; }
        m->geom_hl[G] = 0.f;
        m->geom_r[G] = -1.f;
        continue;
      }
      m->geom_body[G] = h * NB + d->geom_body[h][g];
      for (int i = 0; i < 3; i++) {
        m->geom_pos[G][i] = (float)d->geom_pos[h][g][i];
        m->geom_axis[G][i] = (float)d->geom_axis[h][g][i];
      }
      m->geom_hl[G] = (float)d->geom_halflen[h][g];
      m->geom_r[G] = (float)d->geom_radius[h][g];
    }
  m->nx = 0;
  for (int h = 0; h < NH; h++)
    for (int i = 0; i < NX; i++) {
      const int e = h * NX + i, t = d->xgeom_type[h][i];
      m->x_type[e] = t;
      m->geom_body[NGT + e] = h * NB;
      if (t == PS_GEOM_NONE) continue;
      if (t != PS_GEOM_BOX && t != PS_GEOM_HULL) return fail("unknown extra collider type");
      if (d->xgeom_body[h][i] < 0 || d->xgeom_body[h][i] >= NB) return fail("extra collider body out of range");
      m->nx++;
      m->geom_body[NGT + e] = h * NB + d->xgeom_body[h][i];
      double q[4], qn = 0;
      for (int k = 0; k < 4; k++) { q[k] = d->xgeom_quat[h][i][k]; qn += q[k] * q[k]; }
      if (!(qn > 0)) return fail("extra collider quaternion is zero");
      qn = 1.0 / sqrt(qn);
      for (int k = 0; k < 4; k++) q[k] *= qn;
      const double w = q[0], x = q[1], y = q[2], z = q[3];
      const double R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                           2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                           2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
      for (int k = 0; k < 9; k++) m->x_Q[e][k] = (float)R[k];
      for (int k = 0; k < 3; k++) {
        m->x_pos[e][k] = (float)d->xgeom_pos[h][i][k];
        m->x_hs[e][k] = (float)d->xgeom_size[h][i][k];
      }
      m->x_rb[e] = (float)d->xgeom_rbound[h][i];
      m->x_v0[e] = h * PS_HAND_HULLVERT + d->xgeom_vert[h][i][0];
      m->x_nv[e] = d->xgeom_vert[h][i][1];
      if (t == PS_GEOM_HULL && (d->xgeom_vert[h][i][0] < 0 || d->xgeom_vert[h][i][1] < 4 ||
                                d->xgeom_vert[h][i][1] > PS_HULL_MAXVERT ||
                                d->xgeom_vert[h][i][0] + d->xgeom_vert[h][i][1] > PS_HAND_HULLVERT))
        return fail("hull vertex range out of bounds (4 .. PS_HULL_MAXVERT vertices)");
      if (t == PS_GEOM_BOX && !(d->xgeom_size[h][i][0] > 0 && d->xgeom_size[h][i][1] > 0 && d->xgeom_size[h][i][2] > 0))
        return fail("box half sizes must be positive");
      if (t == PS_GEOM_HULL) {
        enclosing_capsule(&d->hull_vert[h][d->xgeom_vert[h][i][0]], d->xgeom_vert[h][i][1], m->x_ec[e]);
        hull_support_cells(&d->hull_vert[h][d->xgeom_vert[h][i][0]], d->xgeom_vert[h][i][1], m->x_cell[e]);
        m->x_cellv_ok[e] = hull_cell_table(&d->hull_vert[h][d->xgeom_vert[h][i][0]], m->x_cell[e], m->x_cellv[e]);
      }
    }
  for (int g = 0; g < NCOLL; g++) {
    m->geom_pathmask[g] = m->body_pathmask[m->geom_body[g]];
    m->geom_binv[g] = m->body_binv[m->geom_body[g]];
  }
  for (int h = 0; h < NH; h++)
    for (int v = 0; v < PS_HAND_HULLVERT; v++) {
      for (int k = 0; k < 3; k++) m->hull_v[h * PS_HAND_HULLVERT + v][k] = (float)d->hull_vert[h][v][k];
      m->hull_v[h * PS_HAND_HULLVERT + v][3] = 0.f;
    }
  if (d->n_xpairs < 0 || d->n_xpairs > PS_MAX_XPAIRS) return fail("bad n_xpairs");
  m->nxpairs = d->n_xpairs;
  for (int i = 0; i < d->n_xpairs; i++) {
    const int a = d->xpair[i][0], b = d->xpair[i][1];
    if (a < 0 || b < 0 || a >= NCOLL || b >= NCOLL || a >= b || b < NGT) return fail("extra pair index out of range");
    if ((a < NGT && m->geom_r[a] < 0.f) || (a >= NGT && m->x_type[a - NGT] == PS_GEOM_NONE) ||
        m->x_type[b - NGT] == PS_GEOM_NONE)
      return fail("extra pair names an unused collider");
    m->xpair[i] = a | (b << 8);
  }
  m->root_geom_count = d->root_geom_count;
  // v2 packed lane topology + conservative piano prefilter bounds
  for (int B = 0; B < NBT; B++) {
    m->body_level[B] = depth_b[B];
    int pk = 0;
    for (int c = 0; c < m->body_nchild[B]; c++) pk |= m->body_child[B][c] << (6 * c);
    m->body_child_pack[B] = pk;
  }
  for (int g = 0; g < NDT; g++) {
    int p[2] = {0, 0};
    for (int a = 1; a < MAXDEP; a++) {
      int v = a <= m->dof_depth[g] ? m->dof_anc[g][a] : g;  // past the root: the dof itself (a valid lane)
      p[(a - 1) / 4] |= v << (8 * ((a - 1) % 4));
    }
    m->dof_anc_pack[g][0] = p[0];
    m->dof_anc_pack[g][1] = p[1];
    m->dof_anc_pack[g][2] = 0;
  }
  {
    float zmax = m->base_pos[2] + m->base_half[2], xmin = m->base_pos[0] - m->base_half[0],
          xmax = m->base_pos[0] + m->base_half[0];
    for (int k = 0; k < NK; k++) {
      zmax = fmaxf(zmax, m->key_pos[k][2] + m->key_half[k][2] + 0.02f);
      xmin = fminf(xmin, m->key_pos[k][0] - m->key_half[k][0] - 0.02f);
      xmax = fmaxf(xmax, m->key_pos[k][0] + m->key_half[k][0] + 0.02f);
    }
    m->key_top_zmax = zmax;
    m->piano_xmin = xmin;
    m->piano_xmax = xmax;
  }
  for (int k = 0; k < NK; k++) {
    float* g = m->key_geo[k];
    for (int i = 0; i < 3; i++) { g[i] = m->key_pos[k][i]; g[3 + i] = m->key_half[k][i]; g[6 + i] = m->key_anchor[k][i]; }
    g[9] = m->key_pos[k][0] - m->key_half[k][0] - 0.02f;
    g[10] = m->key_pos[k][0] + m->key_half[k][0] + 0.02f;
    g[11] = m->key_ylo[k];
    g[12] = m->key_yhi[k];
    g[13] = m->key_pos[k][2] + m->key_half[k][2] + 0.02f;
    g[14] = g[15] = 0.f;
  }
  {
    double y0 = m->key_ylo[0], y1 = m->key_yhi[NK - 1];
    for (int k = 0; k < NK; k++) { y0 = fmin(y0, m->key_ylo[k]); y1 = fmax(y1, m->key_yhi[k]); }
    double bw = (y1 - y0) / NKB;
    m->kb_y0 = (float)y0;
    m->kb_inv = (float)(1.0 / bw);
    for (int b = 0; b < NKB; b++) {
      double blo = y0 + b * bw, bhi = blo + bw;
      int f = 0;
      while (f < NK && m->key_yhi[f] < blo) f++;
      int e = f;
      while (e < NK && m->key_ylo[e] <= bhi) e++;
      m->kb_first[b] = (uint8_t)f;
      m->kb_end[b] = (uint8_t)e;
    }
  }
  for (int h = 0; h < NH; h++)
    for (int s = 0; s < PS_NFINGER; s++) {
      m->site_body[h * PS_NFINGER + s] = h * NB + d->site_body[h][s];
      for (int i = 0; i < 3; i++) m->site_pos[h * PS_NFINGER + s][i] = (float)d->site_pos[h][s][i];
    }
  if (d->n_cappairs < 0 || d->n_cappairs > PS_MAX_CAPPAIRS) return fail("bad n_cappairs");
  m->npairs = d->n_cappairs;
  for (int i = 0; i < d->n_cappairs; i++) {
    m->pair[i][0] = d->cappair[i][0];
    m->pair[i][1] = d->cappair[i][1];
    if (m->pair[i][0] < 0 || m->pair[i][0] >= NGT || m->pair[i][1] < 0 || m->pair[i][1] >= NGT)
      return fail("capsule pair index out of range");
    if (m->geom_r[m->pair[i][0]] < 0.f || m->geom_r[m->pair[i][1]] < 0.f) return fail("capsule pair names an unused slot");
  }
  // the cross-hand pairs can be skipped wholesale when the hands' boxes are apart, if they
  // all come after the same-hand ones (model.capsule_pairs orders them so)
  m->npairs_same = 0;
  while (m->npairs_same < m->npairs && m->pair[m->npairs_same][0] / NG == m->pair[m->npairs_same][1] / NG)
    m->npairs_same++;
  for (int i = m->npairs_same; i < m->npairs; i++)
    if (m->pair[i][0] / NG == m->pair[i][1] / NG) { m->npairs_same = m->npairs; break; }
  // likewise the pairs with an extra collider (model.extra_pairs: same-hand ones first)
  auto xhand = [](int g) { return g < NGT ? g / NG : (g - NGT) / NX; };
  m->nxpairs_same = 0;
  while (m->nxpairs_same < m->nxpairs &&
         xhand(m->xpair[m->nxpairs_same] & 255) == xhand(m->xpair[m->nxpairs_same] >> 8))
    m->nxpairs_same++;
  for (int i = m->nxpairs_same; i < m->nxpairs; i++)
    if (xhand(m->xpair[i] & 255) == xhand(m->xpair[i] >> 8)) { m->nxpairs_same = m->nxpairs; break; }
  return 0;
}

extern "C" {

const char* ps_last_error(void) { return g_err.c_str(); }
int ps_version(void) { return 4; }  // 4: ps_task_cfg.struct_size
int ps_model_desc_size(void) { return (int)sizeof(ps_model_desc); }
int ps_obs_dim(const ps_task_cfg* cfg) {
  if (!cfg || cfg->struct_size != PS_TASK_CFG_SIZE)
    return fail("ps_task_cfg.struct_size != sizeof(ps_task_cfg): rebuild against include/pianosim.h");
  return (cfg->n_steps_lookahead + 1) * (NK + 1) + (cfg->fingering_reward ? 10 : 0) + NK + 1 + NH * ND;
}

int ps_create(const ps_model_desc* model, const ps_song_desc* song, const ps_task_cfg* cfg, int n_envs, int device,
              uint64_t seed, ps_env** out) {
  if (!model || !song || !cfg || !out) return fail("null argument");
  if (cfg->struct_size != PS_TASK_CFG_SIZE)
    return fail("ps_task_cfg.struct_size != sizeof(ps_task_cfg): rebuild against include/pianosim.h");
  if (n_envs <= 0) return fail("n_envs must be positive");
  if (song->T <= 0) return fail("empty song");
  if (cfg->n_steps_lookahead < 0) return fail("negative lookahead");
  if (cfg->max_contacts < 0 || cfg->max_contacts > MAXCON) return fail("max_contacts out of range");
  if (cfg->solver_iterations < 0) return fail("negative solver_iterations");
  if (cfg->solver_refine < 0 || cfg->solver_refine > 2) return fail("solver_refine must be 0, 1 or 2");
  if (cfg->solver != PS_SOLVER_NEWTON) return fail("unknown solver (PS_SOLVER_NEWTON is the only one)");
  for (int t = 0; t < song->T; t++) {
    if (song->count[t] < 0 || song->count[t] > PS_MAX_NOTES) return fail("bad note count");
    // the ot_fingering reward assigns the step's goal keys to fingertips in a table of
    // PS_MAX_NOTES columns (piano_with_shadow_hands.py:340-361 has no cap): more is an error
    int k = 0;
    for (int j = 0; j < NK; j++) k += song->goal[(size_t)t * (NK + 1) + j] != 0.f;
    if (k > PS_MAX_NOTES)
      return fail("step " + std::to_string(t) + " has " + std::to_string(k) + " goal keys; at most " +
                  std::to_string(PS_MAX_NOTES) + " are supported");
  }
  DeviceGuard guard_(device);
  if (!guard_.ok) return fail("hipSetDevice(" + std::to_string(device) + ") failed");
  DevModel* hm = new DevModel;
  if (build_dev_model(model, hm)) { delete hm; return -1; }
  const bool has_x = hm->nx > 0 || hm->nxpairs > 0;
  ps_env* E = new ps_env();
  E->n = n_envs;
  E->device = device;
  E->cfg = *cfg;
  E->obs_dim = ps_obs_dim(cfg) - NH * ND + hm->n_obsj;  // the model's joints_pos entries
  E->action_dim = hm->n_action;
  E->has_x = has_x;
  E->T = song->T;
  size_t N = (size_t)n_envs;
  HIPCHK(hipMalloc(&E->d_model, sizeof(DevModel)));
  HIPCHK(hipMemcpy(E->d_model, hm, sizeof(DevModel), hipMemcpyHostToDevice));
  delete hm;
  HIPCHK(hipMalloc(&E->d_goal, sizeof(float) * song->T * (NK + 1)));
  HIPCHK(hipMemcpy(E->d_goal, song->goal, sizeof(float) * song->T * (NK + 1), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&E->d_count, sizeof(int) * song->T));
  HIPCHK(hipMemcpy(E->d_count, song->count, sizeof(int) * song->T, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&E->d_keys, sizeof(int) * song->T * PS_MAX_NOTES));
  HIPCHK(hipMemcpy(E->d_keys, song->keys, sizeof(int) * song->T * PS_MAX_NOTES, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&E->d_fingers, sizeof(int) * song->T * PS_MAX_NOTES));
  HIPCHK(hipMemcpy(E->d_fingers, song->fingers, sizeof(int) * song->T * PS_MAX_NOTES, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&E->qpos, sizeof(float) * N * NV));
  HIPCHK(hipMalloc(&E->qvel, sizeof(float) * N * NV));
  HIPCHK(hipMalloc(&E->qws, sizeof(float) * N * NV));
  HIPCHK(hipMalloc(&E->applied, sizeof(float) * N * NV));
  HIPCHK(hipMalloc(&E->ctrl, sizeof(float) * N * NU));
  HIPCHK(hipMalloc(&E->sustain, sizeof(float) * N));
  HIPCHK(hipMalloc(&E->terms, sizeof(float) * N * PS_NTERMS));
  HIPCHK(hipMalloc(&E->tips, sizeof(float) * N * 2 * PS_NFINGER * 3));
  HIPCHK(hipMalloc(&E->t_idx, sizeof(int) * N));
  HIPCHK(hipMalloc(&E->ncon, sizeof(int) * N));
  HIPCHK(hipMalloc(&E->mus_acc, sizeof(float) * N * PS_NMUSIC));
  HIPCHK(hipMalloc(&E->mus_ep, sizeof(float) * N * PS_NMUSIC));
  HIPCHK(hipMalloc(&E->mus_cnt, sizeof(int) * N));
  HIPCHK(hipMalloc(&E->order, sizeof(int) * N));
  HIPCHK(hipMalloc(&E->last, N));
  HIPCHK(hipMalloc(&E->hand_dy, sizeof(float) * N));
  HIPCHK(hipMalloc(&E->episode, sizeof(int) * N));
  HIPCHK(hipMalloc(&E->stats, sizeof(int) * N * PS_NSTATS));
  HIPCHK(hipMalloc(&E->warnings, sizeof(int) * N * PS_NWARN));
  HIPCHK(hipMemset(E->warnings, 0, sizeof(int) * N * PS_NWARN));
  HIPCHK(hipMalloc(&E->park, sizeof(float) * N * PARK_WORDS * 64));
  HIPCHK(hipMemset(E->hand_dy, 0, sizeof(float) * N));
  HIPCHK(hipMemset(E->episode, 0, sizeof(int) * N));
  HIPCHK(hipMemset(E->stats, 0, sizeof(int) * N * PS_NSTATS));
  E->seed = seed;
  E->env_offset = 0;
  HIPCHK(hipMemset(E->qpos, 0, sizeof(float) * N * NV));
  HIPCHK(hipMemset(E->qvel, 0, sizeof(float) * N * NV));
  HIPCHK(hipMemset(E->qws, 0, sizeof(float) * N * NV));
  HIPCHK(hipMemset(E->applied, 0, sizeof(float) * N * NV));
  HIPCHK(hipMemset(E->ctrl, 0, sizeof(float) * N * NU));
  HIPCHK(hipMemset(E->sustain, 0, sizeof(float) * N));
  HIPCHK(hipMemset(E->terms, 0, sizeof(float) * N * PS_NTERMS));
  HIPCHK(hipMemset(E->tips, 0, sizeof(float) * N * 2 * PS_NFINGER * 3));
  HIPCHK(hipMemset(E->t_idx, 0, sizeof(int) * N));
  HIPCHK(hipMemset(E->ncon, 0, sizeof(int) * N));
  HIPCHK(hipMemset(E->mus_acc, 0, sizeof(float) * N * PS_NMUSIC));
  HIPCHK(hipMemset(E->mus_ep, 0, sizeof(float) * N * PS_NMUSIC));
  HIPCHK(hipMemset(E->mus_cnt, 0, sizeof(int) * N));
  HIPCHK(hipMemset(E->last, 0, N));
  HIPCHK(hipDeviceSynchronize());
  E->applied_on = false;
  E->ordered = !(getenv("PIANOSIM_NO_ORDER") && atoi(getenv("PIANOSIM_NO_ORDER")));
  E->full_cpl = getenv("PIANOSIM_DEBUG_FULL_COUPLED") && atoi(getenv("PIANOSIM_DEBUG_FULL_COUPLED"));
  {
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    E->wave_slots = 4 * cus;  // 4 SIMDs per CDNA compute unit
    const char* w = getenv("PIANOSIM_ONE_WAVE_MAX");  // (A/B runs: the threshold; 0 never)
    if (w) E->wave_slots = atoi(w);
  }
  *out = E;
  return 0;
}

int ps_env_obs_dim(const ps_env* E) { return E ? E->obs_dim : fail("null env"); }
int ps_env_action_dim(const ps_env* E) { return E ? E->action_dim : fail("null env"); }

void ps_destroy(ps_env* E) {
  if (!E) return;
  DeviceGuard guard_(E->device);
  hipFree(E->d_model); hipFree(E->d_goal); hipFree(E->d_count); hipFree(E->d_keys); hipFree(E->d_fingers);
  hipFree(E->qpos); hipFree(E->qvel); hipFree(E->qws); hipFree(E->applied); hipFree(E->ctrl); hipFree(E->sustain);
  hipFree(E->terms); hipFree(E->tips); hipFree(E->t_idx); hipFree(E->ncon); hipFree(E->last);
  hipFree(E->mus_acc); hipFree(E->mus_ep); hipFree(E->mus_cnt); hipFree(E->order);
  hipFree(E->hand_dy); hipFree(E->episode); hipFree(E->stats); hipFree(E->warnings); hipFree(E->park);
  if (E->con_out) hipFree(E->con_out);
  delete E;
}

// Dispatch order of a step launch: envs by the cost of their previous step, descending -
// the Newton iterations its substeps took (PS_STAT_SOLVES: each is a Hessian assembly,
// factorization and line search) - envs about to auto-reset (no physics this step) last. Workgroups are dispatched in blockIdx order, so the expensive envs start in
// the first wave of workgroups and the cheap ones fill the slots freed late (longest-
// processing-time-first): the launch's tail is shorter. Each env's result is independent of
// the order.
#ifdef PS_DYN_LDS
#define PS_LAUNCH_LDS PS_DYN_LDS
#else
#define PS_LAUNCH_LDS 0
#endif
constexpr int ORDER_THREADS = 1024;
constexpr int ORDER_BUCKETS = 130;  // 0: resets, 1 + min(Newton iterations of the last step, 128)
__global__ void __launch_bounds__(ORDER_THREADS) order_kernel(const int* __restrict__ stats,
                                                              const uint8_t* __restrict__ last,
                                                              int* __restrict__ order, int n) {
  __shared__ int hist[ORDER_BUCKETS], base[ORDER_BUCKETS];
  if (threadIdx.x < ORDER_BUCKETS) hist[threadIdx.x] = 0;
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int b = last[e] ? 0 : 1 + min(max(stats[(size_t)e * PS_NSTATS + PS_STAT_SOLVES], 0), 128);
    atomicAdd(&hist[b], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = ORDER_BUCKETS - 1; b >= 0; b--) {  // most rows first, resets last
      base[b] = acc;
      acc += hist[b];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int b = last[e] ? 0 : 1 + min(max(stats[(size_t)e * PS_NSTATS + PS_STAT_SOLVES], 0), 128);
    order[atomicAdd(&base[b], 1)] = e;
  }
}

static int launch(ps_env* E, int mode, const float* action, const uint8_t* mask, float* obs, float* reward,
                  float* discount, uint8_t* step_type, void* stream) {
  Song song{E->T, E->d_goal, E->d_count, E->d_keys, E->d_fingers};
  Cfg cfg{E->cfg.n_steps_lookahead, E->cfg.fingering_reward, E->cfg.forearm_reward, E->cfg.wrong_press_termination,
          E->cfg.solver_iterations, E->cfg.max_contacts, E->obs_dim, E->cfg.canonical_actions,
          (float)E->cfg.energy_penalty_coef, E->cfg.randomize_hand_positions != 0,
          (uint32_t)E->seed, (uint32_t)(E->seed >> 32), (uint32_t)E->env_offset, E->full_cpl,
          E->cfg.solver_refine};
  Bufs b{E->qpos, E->qvel, E->qws, E->ctrl, E->sustain, E->t_idx, E->last,
         E->applied_on ? E->applied : nullptr, E->terms, E->tips, E->ncon, E->mus_acc, E->mus_ep, E->mus_cnt,
         E->hand_dy, E->episode, E->stats, E->con_out, E->warnings, E->park};
  const int* order = nullptr;
  if (mode == 0 && E->ordered && E->n >= 2048) {  // below one wave of workgroups there is no tail to balance
    hipLaunchKernelGGL(order_kernel, dim3(1), dim3(ORDER_THREADS), 0, (hipStream_t)stream, E->stats, E->last, E->order,
                       E->n);
    HIPCHK(hipGetLastError());
    order = E->order;
  }
  // at most one wave per SIMD: the instantiation built for one resident wave (its spills in
  // AGPRs, no scratch traffic) - the two-wave build's second slot would stay empty anyway
  const bool one = E->n <= E->wave_slots;
#define PS_LAUNCH(XG, WPE)                                                                                    \
  hipLaunchKernelGGL((pianosim_kernel<XG, WPE>), dim3(E->n), dim3(64), PS_LAUNCH_LDS, (hipStream_t)stream, \
                     E->d_model, song, cfg, b, action, mask, obs, reward, discount, step_type, mode, E->n, order)
  if (E->has_x) {
    if (one) PS_LAUNCH(true, 1); else PS_LAUNCH(true, PS_WAVES_PER_EU);
  } else {
    if (one) PS_LAUNCH(false, 1); else PS_LAUNCH(false, PS_WAVES_PER_EU);
  }
#undef PS_LAUNCH
  HIPCHK(hipGetLastError());
  return 0;
}

int ps_reset(ps_env* E, const uint8_t* env_mask, float* obs, void* stream) {
  if (!E || !obs) return fail("null argument");
  GUARD(E);
  return launch(E, 1, nullptr, env_mask, obs, nullptr, nullptr, nullptr, stream);
}

int ps_step(ps_env* E, const float* action, float* obs, float* reward, float* discount, uint8_t* step_type,
            void* stream) {
  if (!E || !action || !obs || !reward || !discount || !step_type) return fail("null argument");
  GUARD(E);
  return launch(E, 0, action, nullptr, obs, reward, discount, step_type, stream);
}

int ps_get_state(ps_env* E, float* qpos, float* qvel, float* qacc_ws, float* ctrl, float* sustain, int32_t* t_idx,
                 uint8_t* last, void* stream) {
  if (!E) return fail("null env");
  GUARD(E);
  hipStream_t s = (hipStream_t)stream;
  size_t N = E->n;
  if (qpos) HIPCHK(hipMemcpyAsync(qpos, E->qpos, sizeof(float) * N * NV, hipMemcpyDeviceToDevice, s));
  if (qvel) HIPCHK(hipMemcpyAsync(qvel, E->qvel, sizeof(float) * N * NV, hipMemcpyDeviceToDevice, s));
  if (qacc_ws) HIPCHK(hipMemcpyAsync(qacc_ws, E->qws, sizeof(float) * N * NV, hipMemcpyDeviceToDevice, s));
  if (ctrl) HIPCHK(hipMemcpyAsync(ctrl, E->ctrl, sizeof(float) * N * NU, hipMemcpyDeviceToDevice, s));
  if (sustain) HIPCHK(hipMemcpyAsync(sustain, E->sustain, sizeof(float) * N, hipMemcpyDeviceToDevice, s));
  if (t_idx) HIPCHK(hipMemcpyAsync(t_idx, E->t_idx, sizeof(int) * N, hipMemcpyDeviceToDevice, s));
  if (last) HIPCHK(hipMemcpyAsync(last, E->last, N, hipMemcpyDeviceToDevice, s));
  return 0;
}

int ps_set_state(ps_env* E, const float* qpos, const float* qvel, const float* qacc_ws, const float* ctrl,
                 const float* sustain, const int32_t* t_idx, const uint8_t* last, void* stream) {
  if (!E) return fail("null env");
  GUARD(E);
  hipStream_t s = (hipStream_t)stream;
  size_t N = E->n;
  if (qpos) HIPCHK(hipMemcpyAsync(E->qpos, qpos, sizeof(float) * N * NV, hipMemcpyDeviceToDevice, s));
  if (qvel) HIPCHK(hipMemcpyAsync(E->qvel, qvel, sizeof(float) * N * NV, hipMemcpyDeviceToDevice, s));
  if (qacc_ws) HIPCHK(hipMemcpyAsync(E->qws, qacc_ws, sizeof(float) * N * NV, hipMemcpyDeviceToDevice, s));
  if (ctrl) HIPCHK(hipMemcpyAsync(E->ctrl, ctrl, sizeof(float) * N * NU, hipMemcpyDeviceToDevice, s));
  if (sustain) HIPCHK(hipMemcpyAsync(E->sustain, sustain, sizeof(float) * N, hipMemcpyDeviceToDevice, s));
  if (t_idx) HIPCHK(hipMemcpyAsync(E->t_idx, t_idx, sizeof(int) * N, hipMemcpyDeviceToDevice, s));
  if (last) HIPCHK(hipMemcpyAsync(E->last, last, N, hipMemcpyDeviceToDevice, s));
  return 0;
}

int ps_set_applied(ps_env* E, const float* qfrc_applied, void* stream) {
  if (!E) return fail("null env");
  GUARD(E);
  if (!qfrc_applied) {
    E->applied_on = false;
    return 0;
  }
  HIPCHK(hipMemcpyAsync(E->applied, qfrc_applied, sizeof(float) * E->n * NV, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  E->applied_on = true;
  return 0;
}

int ps_reward_terms(ps_env* E, float* terms, void* stream) {
  if (!E || !terms) return fail("null argument");
  GUARD(E);
  HIPCHK(hipMemcpyAsync(terms, E->terms, sizeof(float) * E->n * PS_NTERMS, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return 0;
}

int ps_fingertips(ps_env* E, float* xpos, void* stream) {
  if (!E || !xpos) return fail("null argument");
  GUARD(E);
  HIPCHK(hipMemcpyAsync(xpos, E->tips, sizeof(float) * E->n * 2 * PS_NFINGER * 3, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return 0;
}

#ifdef PS_TIMING
// diagnostic: per-env phase cycle sums [n][NPHASE] since the last call (host buffer)
int ps_debug_timing(ps_env* E, uint64_t* out) {
  static uint64_t* d = nullptr;
  static size_t cap = 0;
  size_t bytes = sizeof(uint64_t) * E->n * NPHASE;
  if (cap < bytes) {
    if (d) (void)hipFree(d);
    HIPCHK(hipMalloc(&d, bytes));
    cap = bytes;
    HIPCHK(hipMemset(d, 0, bytes));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_timing), &d, sizeof(d)));
    return 0;
  }
  HIPCHK(hipDeviceSynchronize());
  if (out) HIPCHK(hipMemcpy(out, d, bytes, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(d, 0, bytes));
  return 0;
}
#endif

int ps_musical_metrics(ps_env* E, float* episode, int32_t* episodes, void* stream) {
  if (!E) return fail("null argument");
  GUARD(E);
  if (episode)
    HIPCHK(hipMemcpyAsync(episode, E->mus_ep, sizeof(float) * E->n * PS_NMUSIC, hipMemcpyDeviceToDevice,
                          (hipStream_t)stream));
  if (episodes)
    HIPCHK(hipMemcpyAsync(episodes, E->mus_cnt, sizeof(int) * E->n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

int ps_solver_stats(ps_env* E, int32_t* stats, void* stream) {
  if (!E || !stats) return fail("null argument");
  GUARD(E);
  HIPCHK(hipMemcpyAsync(stats, E->stats, sizeof(int) * E->n * PS_NSTATS, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

int ps_get_hand_offset(ps_env* E, float* dy, int32_t* episodes, void* stream) {
  if (!E) return fail("null argument");
  GUARD(E);
  if (dy) HIPCHK(hipMemcpyAsync(dy, E->hand_dy, sizeof(float) * E->n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  if (episodes)
    HIPCHK(hipMemcpyAsync(episodes, E->episode, sizeof(int) * E->n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

int ps_set_hand_offset(ps_env* E, const float* dy, void* stream) {
  if (!E || !dy) return fail("null argument");
  GUARD(E);
  if (!E->cfg.randomize_hand_positions) return fail("ps_set_hand_offset needs randomize_hand_positions");
  HIPCHK(hipMemcpyAsync(E->hand_dy, dy, sizeof(float) * E->n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

static_assert(sizeof(ps_contact) == sizeof(Contact), "ps_contact mirrors the kernel's contact record");
int ps_record_contacts(ps_env* E, int on) {
  if (!E) return fail("null argument");
  GUARD(E);
  if (on && !E->con_out) {
    HIPCHK(hipMalloc(&E->con_out, sizeof(Contact) * MAXCON * (size_t)E->n));
    HIPCHK(hipMemset(E->con_out, 0, sizeof(Contact) * MAXCON * (size_t)E->n));
  } else if (!on && E->con_out) {
    HIPCHK(hipFree(E->con_out));
    E->con_out = nullptr;
  }
  return 0;
}

int ps_contacts(ps_env* E, ps_contact* out, void* stream) {
  if (!E || !out) return fail("null argument");
  GUARD(E);
  if (!E->con_out) return fail("contact recording is off (ps_record_contacts)");
  HIPCHK(hipMemcpyAsync(out, E->con_out, sizeof(Contact) * MAXCON * (size_t)E->n, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return 0;
}

int ps_warnings(ps_env* E, int32_t* warnings, void* stream) {
  if (!E || !warnings) return fail("null argument");
  GUARD(E);
  HIPCHK(hipMemcpyAsync(warnings, E->warnings, sizeof(int) * E->n * PS_NWARN, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return 0;
}

int ps_set_env_offset(ps_env* E, int64_t global_first_env) {
  if (!E) return fail("null argument");
  if (global_first_env < 0) return fail("negative env offset");
  E->env_offset = global_first_env;
  return 0;
}

// one workgroup: env i by thread i (mod 1024); the finished episodes' sum in a fixed order
// (per-thread partials, then a tree over the 1024 threads): deterministic
__global__ void __launch_bounds__(1024) episode_returns_kernel(const float* __restrict__ reward,
                                                               const uint8_t* __restrict__ step_type, int n,
                                                               double* __restrict__ running, float* __restrict__ last_return,
                                                               double* __restrict__ finished_sum,
                                                               int64_t* __restrict__ finished_count) {
  __shared__ double ssum[1024];
  __shared__ int scnt[1024];
  double fs = 0.0;
  int fc = 0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const int st = step_type[i];
    const double r = st == PS_FIRST ? 0.0 : running[i] + (double)reward[i];
    running[i] = r;
    if (st == PS_LAST) {
      last_return[i] = (float)r;
      fs += r;
      fc++;
    }
  }
  ssum[threadIdx.x] = fs;
  scnt[threadIdx.x] = fc;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      ssum[threadIdx.x] += ssum[threadIdx.x + w];
      scnt[threadIdx.x] += scnt[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *finished_sum += ssum[0];
    *finished_count += scnt[0];
  }
}

int ps_episode_returns(const float* reward, const uint8_t* step_type, int n, double* running, float* last_return,
                       double* finished_sum, int64_t* finished_count, void* stream) {
  if (!reward || !step_type || !running || !last_return || !finished_sum || !finished_count || n <= 0)
    return fail("ps_episode_returns: null argument or n <= 0");
  hipLaunchKernelGGL(episode_returns_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, reward, step_type, n, running,
                     last_return, finished_sum, finished_count);
  HIPCHK(hipGetLastError());
  return 0;
}

int ps_contact_count(ps_env* E, int32_t* ncon, void* stream) {
  if (!E || !ncon) return fail("null argument");
  GUARD(E);
  HIPCHK(hipMemcpyAsync(ncon, E->ncon, sizeof(int) * E->n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

}  // extern "C"
