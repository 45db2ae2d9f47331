// pianosim.hip - MI355X (gfx950) batched PianoWithShadowHands step/reset.
//
// One 64-lane wavefront (= one workgroup) per environment; the whole control step
// (10 physics substeps + task layer) runs in ONE launch with the env's working set
// resident in LDS. HBM traffic per env-step is the state row in/out, the action and the
// observation (see DESIGN.md "Data layout"). Lanes split every phase of the substep:
//   kinematics / composite inertia / RNE      : lanes over bodies of one tree level
//   mass matrix entries                        : lanes over (dof, ancestor) pairs
//   tree LDL (M and M + h*D, mj_factorI)       : lanes over (ancestor, ancestor) updates
//   collision                                  : lanes over capsules / capsule pairs
//   constraint rows                            : lanes over dofs (dense row layout)
//   PGS                                        : lanes over dofs, DPP wave reductions
// The algorithm (and every ordering that affects results) is the one written
// sequentially in oracle/pianosim_ref.c; see that file for the reference citations.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "devmodel.h"

using namespace ps;

#define MINIMP 0.0001f
#define MAXIMP 0.9999f
#define MINVALF 1e-15f
#define KEY_THRESHOLD 0.00872665f
#define SUSTAIN_THRESHOLD 0.5f

// ------------------------------------------------------------------ small vector math
struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk3(float a, float b, float c) { return {a, b, c}; }
__device__ __forceinline__ f3 ld3(const float* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ void st3(float* p, f3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float norm3(f3 a) { return sqrtf(dot3(a, a)); }
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
// row-major 3x3
__device__ __forceinline__ f3 mv3(const float* R, f3 a) {
  return {R[0] * a.x + R[1] * a.y + R[2] * a.z, R[3] * a.x + R[4] * a.y + R[5] * a.z,
          R[6] * a.x + R[7] * a.y + R[8] * a.z};
}
__device__ __forceinline__ f3 mtv3(const float* R, f3 a) {
  return {R[0] * a.x + R[3] * a.y + R[6] * a.z, R[1] * a.x + R[4] * a.y + R[7] * a.z,
          R[2] * a.x + R[5] * a.y + R[8] * a.z};
}
__device__ __forceinline__ void mm3(const float* A, const float* B, float* C) {
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
// symmetric 3x3 stored xx yy zz xy xz yz
__device__ __forceinline__ f3 sym_mv(const float* I, f3 a) {
  return {I[0] * a.x + I[3] * a.y + I[4] * a.z, I[3] * a.x + I[1] * a.y + I[5] * a.z,
          I[4] * a.x + I[5] * a.y + I[2] * a.z};
}

// ------------------------------------------------------------------ wave primitives
// 64-lane sum via DPP row shifts + row broadcasts; result in every lane.
__device__ __forceinline__ float wave_sum(float v) {
  int x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false));  // row_shr:1
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false));  // row_shr:2
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false));  // row_shr:4
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false));  // row_shr:8
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false));  // row_bcast:15
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ int wave_sum_i(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  return __builtin_amdgcn_readlane(v, 63);
}
// exclusive prefix sum over lanes (Hillis-Steele on shuffles; used for compaction only)
__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int t = __shfl_up(incl, off, 64);
    if (lane >= off) incl += t;
  }
  return incl - v;
}
__device__ __forceinline__ int lanes_below(uint64_t mask, int lane) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// ------------------------------------------------------------------ LDS workspace
struct Contact {
  float pos[3], n[3], t1[3], t2[3], dist;
  int kind, key, g1, g2;  // g1: -1 for key/base (kind 0/1)
};

struct Work {
  float q[NV], v[NV], qws[NV], ctrl[NU];
  float sustain;
  float qfs[NV], qas[NV], w[NV], tmp[NV], tmp2[NV];
  float R[NBT][9], o[NBT][3], com[NBT][3], Iw[NBT][6], axis[NDT][3];
  float scr[NBT][15];  // composite (ms,h,Is) or RNE (w,al,ac,F,N)
  float M[NDT][MAXDEP], Mh[NDT][MAXDEP];
  float Dinv[NDT], Dhinv[NDT];
  float kc[NK], ks[NK];
  float cap[NGT][6];
  float actf[NU];
  int ncon;
  Contact con[MAXCON];
  int keyhit[NK];
  int nrow;
  float Y[MAXROW][ROWSTRIDE];
  float r_b[MAXROW], r_R[MAXROW], r_arinv[MAXROW], r_f[MAXROW];
  int r_key[MAXROW];
  uint64_t r_mask[MAXROW];
  float norm_state[NK];
  int act_bits[3];
};

struct Song {
  int T;
  const float* goal;
  const int* count;
  const int* keys;
  const int* fingers;
};

struct Cfg {
  int lookahead, fingering, forearm, wrong_press, pgs_iter, maxcon, obs_dim, canonical;
  float energy_coef;
  int skip;  // development ablation mask (PIANOSIM_SKIP env var); 0 in production
};

struct Bufs {
  float *qpos, *qvel, *qws, *ctrl, *sustain;
  int* t_idx;
  uint8_t* last;
  const float* applied;  // may be null
  float* terms;
  float* tips;
  int* ncon;
};

// ------------------------------------------------------------------ kinematics
__device__ void kinematics(const DevModel* __restrict__ m, Work& W, int lane) {
  for (int L = 0; L < m->nlev; L++) {
    int i0 = m->lev_start[L], cnt = m->lev_start[L + 1] - i0;
    if (lane < cnt) {
      int B = m->lev_body[i0 + lane];
      int p = m->body_parent[B];
      float R[9], T[9];
      f3 pos = ld3(m->body_pos[B]), o;
      if (p < 0) {
#pragma unroll
        for (int k = 0; k < 9; k++) R[k] = m->body_Q[B][k];
        o = pos;
      } else {
        mm3(W.R[p], m->body_Q[B], R);
        o = ld3(W.o[p]) + mv3(W.R[p], pos);
      }
      int d0 = m->body_dof[B], nd = m->body_ndof[B];
      for (int j = d0; j < d0 + nd; j++) {
        f3 al = ld3(m->dof_axis[j]);
        if (m->dof_type[j] == 1) {
          f3 aw = mv3(R, al);
          st3(W.axis[j], aw);
          o = o + aw * W.q[NK + j];
        } else {
          float t = W.q[NK + j], s, c;
          sincosf(t, &s, &c);
          float C1 = 1.f - c, x = al.x, y = al.y, z = al.z;
          float A[9] = {c + x * x * C1,     x * y * C1 - z * s, x * z * C1 + y * s,
                        y * x * C1 + z * s, c + y * y * C1,     y * z * C1 - x * s,
                        z * x * C1 - y * s, z * y * C1 + x * s, c + z * z * C1};
          mm3(R, A, T);
#pragma unroll
          for (int k = 0; k < 9; k++) R[k] = T[k];
          st3(W.axis[j], mv3(R, al));
        }
      }
#pragma unroll
      for (int k = 0; k < 9; k++) W.R[B][k] = R[k];
      st3(W.o[B], o);
      st3(W.com[B], o + mv3(R, ld3(m->body_ipos[B])));
      // world inertia about COM: R I R^T
      const float* I6 = m->body_I[B];
      float Il[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
      mm3(R, Il, T);
      float Iw[9];
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) Iw[3 * i + k] = T[3 * i] * R[3 * k] + T[3 * i + 1] * R[3 * k + 1] + T[3 * i + 2] * R[3 * k + 2];
      W.Iw[B][0] = Iw[0]; W.Iw[B][1] = Iw[4]; W.Iw[B][2] = Iw[8];
      W.Iw[B][3] = Iw[1]; W.Iw[B][4] = Iw[2]; W.Iw[B][5] = Iw[5];
    }
    __syncthreads();
  }
  if (lane < NGT) {
    int B = m->geom_body[lane];
    f3 c = ld3(W.o[B]) + mv3(W.R[B], ld3(m->geom_pos[lane]));
    f3 a = mv3(W.R[B], ld3(m->geom_axis[lane]));
    float hl = m->geom_hl[lane];
    st3(&W.cap[lane][0], c - a * hl);
    st3(&W.cap[lane][3], c + a * hl);
  }
  for (int k = lane; k < NK; k += 64) {
    float s, c;
    sincosf(W.q[k], &s, &c);
    W.kc[k] = c;
    W.ks[k] = s;
  }
  __syncthreads();
}

// key box frame: rotation about +y by q, centre = anchor + R*(-anchor_local)
__device__ __forceinline__ void key_frame(const DevModel* __restrict__ m, const Work& W, int k, float* R, f3* centre,
                                          f3* anchor) {
  float c = W.kc[k], s = W.ks[k];
  R[0] = c; R[1] = 0; R[2] = s; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = -s; R[7] = 0; R[8] = c;
  f3 P = ld3(m->key_pos[k]), al = ld3(m->key_anchor[k]);
  f3 A = P + al;
  *anchor = A;
  *centre = A + mv3(R, al * -1.f);
}

// ------------------------------------------------------------------ dynamics
// mass matrix (ancestor-sparse), bias (RNE), passive, actuation -> qfrc_smooth
__device__ void dynamics(const DevModel* __restrict__ m, Work& W, const float* __restrict__ applied, int lane) {
  // composite inertia about body origins: scr[B] = {ms, h[3], Is[6]}
  if (lane < NBT) {
    int B = lane;
    float mass = m->body_mass[B];
    f3 dd = ld3(W.com[B]) - ld3(W.o[B]);
    float d2 = dot3(dd, dd);
    float* s = W.scr[B];
    s[0] = mass;
    s[1] = dd.x * mass; s[2] = dd.y * mass; s[3] = dd.z * mass;
    s[4] = W.Iw[B][0] + mass * (d2 - dd.x * dd.x);
    s[5] = W.Iw[B][1] + mass * (d2 - dd.y * dd.y);
    s[6] = W.Iw[B][2] + mass * (d2 - dd.z * dd.z);
    s[7] = W.Iw[B][3] - mass * dd.x * dd.y;
    s[8] = W.Iw[B][4] - mass * dd.x * dd.z;
    s[9] = W.Iw[B][5] - mass * dd.y * dd.z;
  }
  __syncthreads();
  for (int L = m->nlev - 2; L >= 0; L--) {  // parents at level L pull their children
    int i0 = m->lev_start[L], cnt = m->lev_start[L + 1] - i0;
    if (lane < cnt) {
      int P = m->lev_body[i0 + lane];
      float* sp = W.scr[P];
      f3 op = ld3(W.o[P]);
      for (int c = 0; c < m->body_nchild[P]; c++) {
        int B = m->body_child[P][c];
        const float* sb = W.scr[B];
        f3 r = ld3(W.o[B]) - op;
        f3 hb = mk3(sb[1], sb[2], sb[3]);
        float msb = sb[0], r2 = dot3(r, r), rh = dot3(r, hb);
        sp[4] += sb[4] + msb * (r2 - r.x * r.x) + (2.f * rh - 2.f * r.x * hb.x);
        sp[5] += sb[5] + msb * (r2 - r.y * r.y) + (2.f * rh - 2.f * r.y * hb.y);
        sp[6] += sb[6] + msb * (r2 - r.z * r.z) + (2.f * rh - 2.f * r.z * hb.z);
        sp[7] += sb[7] - msb * r.x * r.y - (r.x * hb.y + hb.x * r.y);
        sp[8] += sb[8] - msb * r.x * r.z - (r.x * hb.z + hb.x * r.z);
        sp[9] += sb[9] - msb * r.y * r.z - (r.y * hb.z + hb.y * r.z);
        sp[1] += hb.x + r.x * msb; sp[2] += hb.y + r.y * msb; sp[3] += hb.z + r.z * msb;
        sp[0] += msb;
      }
    }
    __syncthreads();
  }
  // M entries: lane over (dof i, ancestor slot a)
  for (int e = lane; e < NDT * MAXDEP; e += 64) {
    int i = e / MAXDEP, a = e - i * MAXDEP;
    int j = m->dof_anc[i][a];
    if (j < 0) continue;
    int bi = m->dof_body[i], bj = m->dof_body[j];
    const float* s = W.scr[bi];
    f3 ai = ld3(W.axis[i]), h = mk3(s[1], s[2], s[3]), flin, fang;
    if (m->dof_type[i] == 0) {
      flin = cross3(ai, h);
      const float Is[6] = {s[4], s[5], s[6], s[7], s[8], s[9]};
      fang = sym_mv(Is, ai);
    } else {
      flin = ai * s[0];
      fang = cross3(h, ai);
    }
    f3 aj = ld3(W.axis[j]);
    float val = m->dof_type[j] == 0 ? dot3(aj, fang + cross3(ld3(W.o[bi]) - ld3(W.o[bj]), flin)) : dot3(aj, flin);
    if (a == 0) val += m->dof_arm[i];
    W.M[i][a] = val;
    W.Mh[i][a] = a == 0 ? val + m->timestep * m->dof_damp[i] : val;
  }
  __syncthreads();
  // RNE forward: scr[B] = {w[3], al[3], ac[3], F[3], N[3]}
  for (int L = 0; L < m->nlev; L++) {
    int i0 = m->lev_start[L], cnt = m->lev_start[L + 1] - i0;
    if (lane < cnt) {
      int B = m->lev_body[i0 + lane];
      int p = m->body_parent[B];
      f3 w, al, ac;
      if (p < 0) {
        w = mk3(0, 0, 0);
        al = mk3(0, 0, 0);
        ac = mk3(-m->grav[0], -m->grav[1], -m->grav[2]);
      } else {
        const float* sp = W.scr[p];
        f3 wp = ld3(sp), alp = ld3(sp + 3), acp = ld3(sp + 6);
        f3 r = ld3(W.o[B]) - ld3(W.o[p]);
        ac = acp + cross3(alp, r) + cross3(wp, cross3(wp, r));
        int j = m->body_dof[B];
        f3 a = ld3(W.axis[j]);
        float qd = W.v[NK + j];
        al = alp + cross3(wp, a) * qd;
        w = wp + a * qd;
      }
      f3 dd = ld3(W.com[B]) - ld3(W.o[B]);
      f3 acom = ac + cross3(al, dd) + cross3(w, cross3(w, dd));
      f3 F = acom * m->body_mass[B];
      f3 N = sym_mv(W.Iw[B], al) + cross3(w, sym_mv(W.Iw[B], w)) + cross3(dd, F);
      float* s = W.scr[B];
      st3(s, w); st3(s + 3, al); st3(s + 6, ac); st3(s + 9, F); st3(s + 12, N);
    }
    __syncthreads();
  }
  for (int L = m->nlev - 2; L >= 0; L--) {
    int i0 = m->lev_start[L], cnt = m->lev_start[L + 1] - i0;
    if (lane < cnt) {
      int P = m->lev_body[i0 + lane];
      float* sp = W.scr[P];
      f3 F = ld3(sp + 9), N = ld3(sp + 12), op = ld3(W.o[P]);
      for (int c = 0; c < m->body_nchild[P]; c++) {
        int B = m->body_child[P][c];
        f3 Fb = ld3(W.scr[B] + 9), Nb = ld3(W.scr[B] + 12);
        N = N + Nb + cross3(ld3(W.o[B]) - op, Fb);
        F = F + Fb;
      }
      st3(sp + 9, F);
      st3(sp + 12, N);
    }
    __syncthreads();
  }
  // actuator forces (mj_fwdActuation)
  if (lane < NU) {
    int a = lane;
    float len = m->act_c0[a] * W.q[NK + m->act_dof0[a]];
    if (m->act_kind[a] == 1) len += m->act_c1[a] * W.q[NK + m->act_dof1[a]];
    float c = clampf(W.ctrl[a], m->act_clo[a], m->act_chi[a]);
    float f = m->act_kp[a] * (c - len);
    if (m->act_flim[a]) f = clampf(f, m->act_flo[a], m->act_fhi[a]);
    W.actf[a] = f;
  }
  __syncthreads();
  // qfrc_smooth = passive + actuator + applied - bias
  if (lane < NDT) {
    int j = lane, B = m->dof_body[j];
    const float* s = W.scr[B];
    float bias = m->dof_type[j] == 0 ? dot3(ld3(W.axis[j]), ld3(s + 12)) : dot3(ld3(W.axis[j]), ld3(s + 9));
    float f = -m->dof_damp[j] * W.v[NK + j] - bias;
    int a = m->dof_act[j];
    if (a >= 0) f += m->dof_act_coef[j] * W.actf[a];
    if (applied) f += applied[NK + j];
    W.qfs[NK + j] = f;
  }
  for (int k = lane; k < NK; k += 64) {
    float c = W.kc[k], s = W.ks[k];
    f3 al = ld3(m->key_anchor[k]) * -1.f;
    f3 r = mk3(c * al.x + s * al.z, al.y, -s * al.x + c * al.z);
    float bias = -m->key_mass[k] * (r.z * m->grav[0] - r.x * m->grav[2]);
    float f = -m->key_stiff[k] * (W.q[k] - m->key_sref[k]) - m->key_damp[k] * W.v[k] - bias;
    if (applied) f += applied[k];
    W.qfs[k] = f;
  }
  __syncthreads();
}

// tree LDL (mj_factorI) of M and Mh simultaneously; lanes [32h, 32h+32) own hand h
__device__ void factor(const DevModel* __restrict__ m, Work& W, int lane) {
  int h = lane >> 5, t = lane & 31;
  for (int kl = ND - 1; kl >= 0; kl--) {
    int k = h * ND + kl;
    int dk = m->dof_depth[k];
    float Dk = fmaxf(W.M[k][0], MINVALF), Dhk = fmaxf(W.Mh[k][0], MINVALF);
    int P = dk * (dk + 1) / 2;
    for (int e = t; e < P; e += 32) {
      int a = m->tri_a[e], b = m->tri_b[e];
      int i = m->dof_anc[k][a];
      W.M[i][b - a] -= (W.M[k][a] / Dk) * W.M[k][b];
      W.Mh[i][b - a] -= (W.Mh[k][a] / Dhk) * W.Mh[k][b];
    }
    __syncthreads();
    if (t == 0) { W.M[k][0] = Dk; W.Mh[k][0] = Dhk; }
    if (t >= 1 && t <= dk) {
      W.M[k][t] = W.M[k][t] / Dk;
      W.Mh[k][t] = W.Mh[k][t] / Dhk;
    }
    __syncthreads();
  }
  if (lane < NDT) {
    W.Dinv[lane] = 1.f / W.M[lane][0];
    W.Dhinv[lane] = 1.f / W.Mh[lane][0];
  }
  __syncthreads();
}

// x <- M^-1 x (hand part, tree LDL by depth levels) ; keys: x *= keyinv
template <bool IMPLICIT>
__device__ void solve(const DevModel* __restrict__ m, Work& W, float* x, int lane) {
  const float(*L)[MAXDEP] = IMPLICIT ? W.Mh : W.M;
  const float* Dinv = IMPLICIT ? W.Dhinv : W.Dinv;
  float* xh = x + NK;
  for (int d = m->ndepth - 1; d >= 0; d--) {  // x <- L^-T x (pull from descendants)
    int i0 = m->dep_start[d], cnt = m->dep_start[d + 1] - i0;
    if (lane < cnt) {
      int i = m->dep_dof[i0 + lane];
      float s = xh[i];
      for (int c = 0; c < m->dof_ndesc[i]; c++) {
        int k = m->dof_desc[i][c];
        s -= L[k][m->dof_depth[k] - d] * xh[k];
      }
      xh[i] = s;
    }
    __syncthreads();
  }
  if (lane < NDT) xh[lane] *= Dinv[lane];
  for (int k = lane; k < NK; k += 64) x[k] *= IMPLICIT ? m->key_Mhinv[k] : m->key_Minv[k];
  __syncthreads();
  for (int d = 1; d < m->ndepth; d++) {  // x <- L^-1 x (pull from ancestors)
    int i0 = m->dep_start[d], cnt = m->dep_start[d + 1] - i0;
    if (lane < cnt) {
      int k = m->dep_dof[i0 + lane];
      float s = xh[k];
      for (int a = 1; a <= d; a++) s -= L[k][a] * xh[m->dof_anc[k][a]];
      xh[k] = s;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ collision
__device__ __forceinline__ void make_frame(f3 n, f3* t1, f3* t2) {
  f3 e = fabsf(n.z) < 0.5f ? mk3(0, 0, 1) : mk3(1, 0, 0);
  f3 a = cross3(n, e);
  *t1 = a * (1.f / norm3(a));
  *t2 = cross3(n, *t1);
}

__device__ float sphere_box(f3 p, float r, f3 c, const float* R, const float* hs, f3* nout, f3* posout) {
  f3 pl = mtv3(R, p - c);
  float plv[3] = {pl.x, pl.y, pl.z}, q[3];
  bool outside = false;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    q[i] = clampf(plv[i], -hs[i], hs[i]);
    if (q[i] != plv[i]) outside = true;
  }
  f3 n, mid;
  float dist;
  if (outside) {
    f3 dv = mk3(plv[0] - q[0], plv[1] - q[1], plv[2] - q[2]);
    float dn = norm3(dv);
    n = dv * (1.f / dn);
    dist = dn - r;
    mid = mk3(q[0], q[1], q[2]) + n * (0.5f * dist);
  } else {
    int ax = 0;
    float best = hs[0] - fabsf(plv[0]);
#pragma unroll
    for (int i = 1; i < 3; i++) {
      float s = hs[i] - fabsf(plv[i]);
      if (s < best) { best = s; ax = i; }
    }
    float nv[3] = {0, 0, 0};
    nv[ax] = plv[ax] >= 0 ? 1.f : -1.f;
    n = mk3(nv[0], nv[1], nv[2]);
    dist = -best - r;
    mid = pl + n * (0.5f * (best - r));
  }
  *nout = mv3(R, n);
  *posout = c + mv3(R, mid);
  return dist;
}

__device__ float seg_box_t(f3 a3, f3 d3, const float* hs) {
  float a[3] = {a3.x, a3.y, a3.z}, dv[3] = {d3.x, d3.y, d3.z};
  float bp[8];
  int nb = 0;
  bp[nb++] = 0.f;
  for (int i = 0; i < 3; i++) {
    if (dv[i] == 0.f) continue;
    for (int sgn = -1; sgn <= 1; sgn += 2) {
      float t = (sgn * hs[i] - a[i]) / dv[i];
      if (t > 0.f && t < 1.f) bp[nb++] = t;
    }
  }
  bp[nb++] = 1.f;
  for (int i = 1; i < nb; i++)
    for (int j = i; j > 0 && bp[j] < bp[j - 1]; j--) { float t = bp[j]; bp[j] = bp[j - 1]; bp[j - 1] = t; }
  float bestf = INFINITY, bestt = 0.f;
  for (int s = 0; s + 1 < nb; s++) {
    float lo = bp[s], hi = bp[s + 1];
    if (!(hi > lo)) continue;
    float mid = 0.5f * (lo + hi), num = 0.f, den = 0.f;
    for (int i = 0; i < 3; i++) {
      float x = a[i] + mid * dv[i];
      float tgt = x > hs[i] ? hs[i] : (x < -hs[i] ? -hs[i] : 0.f);
      if (tgt == 0.f && fabsf(x) <= hs[i]) continue;
      num -= (a[i] - tgt) * dv[i];
      den += dv[i] * dv[i];
    }
    float t = den > 0.f ? clampf(num / den, lo, hi) : lo;
    float f = 0.f;
    for (int i = 0; i < 3; i++) {
      float e = fabsf(a[i] + t * dv[i]) - hs[i];
      if (e > 0) f += e * e;
    }
    if (f < bestf) { bestf = f; bestt = t; }
  }
  if (bestf <= 0.f) {
    float tin = 0.f, tout = 1.f;
    bool empty = false;
    for (int i = 0; i < 3; i++) {
      if (fabsf(dv[i]) < 1e-12f) {
        if (fabsf(a[i]) > hs[i]) empty = true;
        continue;
      }
      float t1 = (-hs[i] - a[i]) / dv[i], t2 = (hs[i] - a[i]) / dv[i];
      if (t1 > t2) { float t = t1; t1 = t2; t2 = t; }
      if (t1 > tin) tin = t1;
      if (t2 < tout) tout = t2;
    }
    if (!empty && tin <= tout) bestt = 0.5f * (tin + tout);
  }
  return bestt;
}

// capsule (geom2) vs box (geom1); writes up to 2 contacts at out (if non-null), returns count
__device__ int capsule_box(f3 p0, f3 p1, float r, f3 c, const float* R, const float* hs, Contact* out, int slot,
                           int maxc, int kind, int key, int g2) {
  int n = 0;
  f3 nrm, pos;
  for (int e = 0; e < 2; e++) {
    float dist = sphere_box(e == 0 ? p0 : p1, r, c, R, hs, &nrm, &pos);
    if (dist <= 0.f) {
      if (out && slot + n < maxc) {
        Contact& cc = out[slot + n];
        st3(cc.pos, pos); st3(cc.n, nrm); cc.dist = dist;
        f3 t1, t2;
        make_frame(nrm, &t1, &t2);
        st3(cc.t1, t1); st3(cc.t2, t2);
        cc.kind = kind; cc.key = key; cc.g1 = -1; cc.g2 = g2;
      }
      n++;
    }
  }
  if (n) return n;
  f3 a = mtv3(R, p0 - c), b = mtv3(R, p1 - c);
  float t = seg_box_t(a, b - a, hs);
  f3 p = p0 + (p1 - p0) * t;
  float dist = sphere_box(p, r, c, R, hs, &nrm, &pos);
  if (dist <= 0.f) {
    if (out && slot < maxc) {
      Contact& cc = out[slot];
      st3(cc.pos, pos); st3(cc.n, nrm); cc.dist = dist;
      f3 t1, t2;
      make_frame(nrm, &t1, &t2);
      st3(cc.t1, t1); st3(cc.t2, t2);
      cc.kind = kind; cc.key = key; cc.g1 = -1; cc.g2 = g2;
    }
    return 1;
  }
  return 0;
}

__device__ void seg_seg(f3 p1, f3 q1, f3 p2, f3 q2, f3* c1, f3* c2) {
  f3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
  float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r), s, t;
  const float eps = 1e-12f;
  if (a <= eps && e <= eps) { s = t = 0.f; }
  else if (a <= eps) { s = 0.f; t = clampf(f / e, 0.f, 1.f); }
  else {
    float c = dot3(d1, r);
    if (e <= eps) { t = 0.f; s = clampf(-c / a, 0.f, 1.f); }
    else {
      float b = dot3(d1, d2), den = a * e - b * b;
      s = den != 0.f ? clampf((b * f - c * e) / den, 0.f, 1.f) : 0.f;
      t = (b * s + f) / e;
      if (t < 0.f) { t = 0.f; s = clampf(-c / a, 0.f, 1.f); }
      else if (t > 1.f) { t = 1.f; s = clampf((b - c) / a, 0.f, 1.f); }
    }
  }
  *c1 = p1 + d1 * s;
  *c2 = p2 + d2 * t;
}

// one capsule against its candidate keys then the piano base (canonical order)
__device__ int capsule_vs_piano(const DevModel* __restrict__ m, const Work& W, int c, Contact* out, int slot, int maxc) {
  f3 p0 = ld3(&W.cap[c][0]), p1 = ld3(&W.cap[c][3]);
  float r = m->geom_r[c];
  float lo[3] = {fminf(p0.x, p1.x) - r, fminf(p0.y, p1.y) - r, fminf(p0.z, p1.z) - r};
  float hi[3] = {fmaxf(p0.x, p1.x) + r, fmaxf(p0.y, p1.y) + r, fmaxf(p0.z, p1.z) + r};
  // first key with yhi >= lo_y ; keys are sorted along y
  int k0 = 0, k1 = NK;
  {
    int L = 0, H = NK;
    while (L < H) { int M = (L + H) >> 1; if (m->key_yhi[M] >= lo[1]) H = M; else L = M + 1; }
    k0 = L;
    L = 0; H = NK;
    while (L < H) { int M = (L + H) >> 1; if (m->key_ylo[M] > hi[1]) H = M; else L = M + 1; }
    k1 = L;  // keys [k0, k1) overlap in y
  }
  int n = 0;
  for (int k = k0; k < k1; k++) {
    if (lo[2] > m->key_pos[k][2] + m->key_half[k][2] + 0.02f) continue;
    if (hi[0] < m->key_pos[k][0] - m->key_half[k][0] - 0.02f || lo[0] > m->key_pos[k][0] + m->key_half[k][0] + 0.02f) continue;
    float R[9];
    f3 centre, anchor;
    key_frame(m, W, k, R, &centre, &anchor);
    n += capsule_box(p0, p1, r, centre, R, m->key_half[k], out, slot + n, maxc, 0, k, c);
  }
  const float I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  n += capsule_box(p0, p1, r, ld3(m->base_pos), I3, m->base_half, out, slot + n, maxc, 1, -1, c);
  return n;
}

__device__ void collide(const DevModel* __restrict__ m, Work& W, int maxc, int lane) {
  // capsules vs piano: count, scan, write
  int cnt = lane < NGT ? capsule_vs_piano(m, W, lane, nullptr, 0, 0) : 0;
  int off = wave_excl_scan(cnt, lane);
  int total = wave_sum_i(cnt);
  if (lane < NGT && cnt) capsule_vs_piano(m, W, lane, W.con, off, maxc);
  int base = total;
  // capsule pairs in chunks of 64
  for (int p0 = 0; p0 < m->npairs && base < maxc; p0 += 64) {
    int p = p0 + lane;
    bool hit = false;
    f3 c1, c2;
    float ra = 0, rb = 0, dn = 0;
    int ga = 0, gb = 0;
    if (p < m->npairs) {
      ga = m->pair[p][0];
      gb = m->pair[p][1];
      f3 a0 = ld3(&W.cap[ga][0]), a1 = ld3(&W.cap[ga][3]), b0 = ld3(&W.cap[gb][0]), b1 = ld3(&W.cap[gb][3]);
      ra = m->geom_r[ga];
      rb = m->geom_r[gb];
      float bound = m->geom_hl[ga] + m->geom_hl[gb] + ra + rb;
      if (norm3((a0 + a1) * 0.5f - (b0 + b1) * 0.5f) <= bound) {
        seg_seg(a0, a1, b0, b1, &c1, &c2);
        dn = norm3(c2 - c1);
        hit = dn - ra - rb <= 0.f;
      }
    }
    uint64_t mask = __ballot(hit);
    int slot = base + lanes_below(mask, lane);
    if (hit && slot < maxc) {
      Contact& cc = W.con[slot];
      f3 dv = c2 - c1;
      f3 n = dn > 1e-9f ? dv * (1.f / dn) : mk3(0, 0, 1);
      float dist = dn - ra - rb;
      st3(cc.n, n);
      cc.dist = dist;
      st3(cc.pos, c1 + n * (ra + 0.5f * dist));
      f3 t1, t2;
      make_frame(n, &t1, &t2);
      st3(cc.t1, t1); st3(cc.t2, t2);
      cc.kind = 2; cc.key = -1; cc.g1 = ga; cc.g2 = gb;
    }
    base += __popcll(mask);
  }
  if (lane == 0) W.ncon = base < maxc ? base : maxc;
  __syncthreads();
}

// ------------------------------------------------------------------ constraints
__device__ __forceinline__ float impedance(const float* si, float pos) {
  float d0 = clampf(si[0], MINIMP, MAXIMP), dw = clampf(si[1], MINIMP, MAXIMP);
  float width = si[2], mid = si[3], power = si[4];
  float x = fabsf(pos) / width, imp;
  if (x >= 1.f || width <= MINVALF) imp = dw;
  else {
    float y;
    if (power == 1.f) y = x;
    else if (x <= mid) y = powf(x, power) / powf(mid, power - 1.f);
    else y = 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
    imp = d0 + y * (dw - d0);
  }
  return clampf(imp, MINIMP, MAXIMP);
}

// Row scalars from the row's (pos, J.v, J.qacc_smooth, J.qacc_ws) and its y (in W.Y[r]).
// Returns via LDS: r_b, r_R, r_arinv, r_f (warm start). All lanes call; lane 0 writes.
__device__ void row_scalars(const DevModel* __restrict__ m, Work& W, int r, float pos, const float* solref,
                            const float* solimp, float diag, float jv, float jqs, float jws, int lane) {
  float y = lane < NDT ? W.Y[r][lane] : 0.f;
  float contrib = lane < NDT ? y * y * W.Dinv[lane] : 0.f;
  int key = W.r_key[r];
  if (lane == KEYLANE && key >= 0) {
    float yk = W.Y[r][KEYLANE];
    contrib = yk * yk * m->key_Minv[key];
  }
  float A = wave_sum(contrib);
  float imp = impedance(solimp, pos);
  float dmax = clampf(solimp[1], MINIMP, MAXIMP);
  float tc = fmaxf(solref[0], 2.f * m->timestep), dr = solref[1];
  float K = 1.f / (dmax * dmax * tc * tc * dr * dr), Bc = 2.f / (dmax * tc);
  float aref = -Bc * jv - K * imp * pos;
  float R = fmaxf(MINVALF, (1.f - imp) / imp * diag);
  if (lane == 0) {
    W.r_b[r] = jqs - aref;
    W.r_R[r] = R;
    W.r_arinv[r] = 1.f / (A + R);
    W.r_f[r] = 0.f;  // cold start: a qacc_warmstart-derived start is unstable for new stiff contacts
  }
}

// y <- L^-T y for rows [r0, r1): lane per row, walking the row's dof support
__device__ void rows_LT(const DevModel* __restrict__ m, Work& W, int r0, int r1, int lane) {
  for (int r = r0 + lane; r < r1; r += 64) {
    uint64_t mask = W.r_mask[r];
    float* y = W.Y[r];
    while (mask) {
      int k = 63 - __clzll(mask);
      mask &= ~(1ull << k);
      float yk = y[k];
      if (yk == 0.f) continue;
      int dk = m->dof_depth[k];
      for (int a = 1; a <= dk; a++) y[m->dof_anc[k][a]] -= W.M[k][a] * yk;
    }
  }
  __syncthreads();
}

__device__ void constraints(const DevModel* __restrict__ m, Work& W, int maxrow, int lane) {
  // keys touched by a contact
  for (int k = lane; k < NK; k += 64) W.keyhit[k] = 0;
  __syncthreads();
  if (lane < W.ncon && W.con[lane].kind == 0) W.keyhit[W.con[lane].key] = 1;
  __syncthreads();
  int nr = 0;
  // 1) hand joint limits, dof order (lane = dof)
  {
    float dist = 0.f;
    int side = 0;
    bool act = false;
    if (lane < NDT && m->dof_limited[lane]) {
      float q = W.q[NK + lane];
      float dlo = q - m->dof_lo[lane], dhi = m->dof_hi[lane] - q;
      if (dlo < 0.f) { act = true; dist = dlo; side = 0; }
      else if (dhi < 0.f) { act = true; dist = dhi; side = 1; }
    }
    uint64_t mask = __ballot(act);
    int slot = nr + lanes_below(mask, lane);
    int tot = __popcll(mask);
    // write the rows (dense y initialised with J = +-e_j)
    for (int r = nr; r < nr + tot && r < maxrow; r++)
      for (int l = lane; l < ROWSTRIDE; l += 64) W.Y[r][l] = 0.f;
    __syncthreads();
    if (act && slot < maxrow) {
      W.Y[slot][lane] = side == 0 ? 1.f : -1.f;
      W.r_key[slot] = -1;
      W.r_mask[slot] = m->dof_ancmask[lane];
    }
    __syncthreads();
    int nlim = tot < maxrow - nr ? tot : maxrow - nr;
    rows_LT(m, W, nr, nr + nlim, lane);
    // scalars per limit row (uniform loop over rows; the row's dof found via ballot order)
    for (int r = nr; r < nr + nlim; r++) {
      int rank = r - nr;
      // the lane that owns this row
      uint64_t mm = mask;
      for (int i = 0; i < rank; i++) mm &= mm - 1;
      int j = __builtin_ctzll(mm);
      float q = W.q[NK + j];
      float dlo = q - m->dof_lo[j];
      float pos = dlo < 0.f ? dlo : m->dof_hi[j] - q;
      float sgn = dlo < 0.f ? 1.f : -1.f;
      row_scalars(m, W, r, pos, m->lim_solref, m->lim_solimp, m->dof_dinv[j], sgn * W.v[NK + j], sgn * W.qas[NK + j],
                  sgn * W.qws[NK + j], lane);
    }
    nr += nlim;
  }
  __syncthreads();
  // 2) limits of keys touched by contacts (key order); 3) free key limits: closed form
  {
    for (int k0 = 0; k0 < NK; k0 += 64) {
      int k = k0 + lane;
      bool act = false, coupled = false;
      float pos = 0.f, sgn = 1.f;
      if (k < NK) {
        float dlo = W.q[k] - m->key_lo[k], dhi = m->key_hi[k] - W.q[k];
        if (dlo < 0.f) { act = true; pos = dlo; sgn = 1.f; }
        else if (dhi < 0.f) { act = true; pos = dhi; sgn = -1.f; }
        coupled = act && W.keyhit[k];
      }
      if (act && !coupled) {  // independent 1-dof row: PGS fixed point in closed form
        float imp = impedance(m->lim_solimp, pos);
        float dmax = clampf(m->lim_solimp[1], MINIMP, MAXIMP);
        float tc = fmaxf(m->lim_solref[0], 2.f * m->timestep), dr = m->lim_solref[1];
        float K = 1.f / (dmax * dmax * tc * tc * dr * dr), Bc = 2.f / (dmax * tc);
        float aref = -Bc * sgn * W.v[k] - K * imp * pos;
        float R = fmaxf(MINVALF, (1.f - imp) / imp * m->key_dinv[k]);
        float b = sgn * W.qas[k] - aref;
        float f = fmaxf(0.f, -b / (m->key_Minv[k] + R));
        W.tmp2[k] = sgn * f;  // contribution to w[k] added after PGS
      } else if (k < NK) {
        W.tmp2[k] = 0.f;
      }
      uint64_t mask = __ballot(coupled);
      int slot = nr + lanes_below(mask, lane);
      int tot = __popcll(mask);
      for (int r = nr; r < nr + tot && r < maxrow; r++)
        for (int l = lane; l < ROWSTRIDE; l += 64) W.Y[r][l] = 0.f;
      __syncthreads();
      if (coupled && slot < maxrow) {
        W.Y[slot][KEYLANE] = sgn;
        W.r_key[slot] = k;
        W.r_mask[slot] = 0;
      }
      __syncthreads();
      int nk = tot < maxrow - nr ? tot : maxrow - nr;
      for (int r = nr; r < nr + nk; r++) {
        int kk = W.r_key[r];
        float s = W.Y[r][KEYLANE];
        float pos2 = s > 0.f ? W.q[kk] - m->key_lo[kk] : m->key_hi[kk] - W.q[kk];
        row_scalars(m, W, r, pos2, m->lim_solref, m->lim_solimp, m->key_dinv[kk], s * W.v[kk], s * W.qas[kk],
                    s * W.qws[kk], lane);
      }
      nr += nk;
      __syncthreads();
    }
  }
  // 4) contacts: 4 pyramid edges each
  int ncon = W.ncon;
  int cfirst = nr;
  int ncr = 0;
  for (int c = 0; c < ncon && nr + 4 * (c + 1) <= maxrow; c++) {  // whole contacts only
    const Contact& cc = W.con[c];
    int g2 = cc.g2, B2 = m->geom_body[g2];
    int B1 = cc.kind == 2 ? m->geom_body[cc.g1] : -1;
    uint64_t m2 = m->body_pathmask[B2], m1 = B1 >= 0 ? m->body_pathmask[B1] : 0ull;
    f3 p = ld3(cc.pos);
    f3 dirs[3] = {ld3(cc.n), ld3(cc.t1), ld3(cc.t2)};
    int rbase = nr + 4 * c;
    float jv[3], jqs[3], jws[3];
    for (int dI = 0; dI < 3; dI++) {
      f3 u = dirs[dI];
      float J = 0.f;
      if (lane < NDT) {
        int j = lane, Bj = m->dof_body[j];
        float val = m->dof_type[j] == 0 ? dot3(u, cross3(ld3(W.axis[j]), p - ld3(W.o[Bj]))) : dot3(u, ld3(W.axis[j]));
        if ((m2 >> j) & 1ull) J += val;
        if ((m1 >> j) & 1ull) J -= val;
      }
      int key = cc.kind == 0 ? cc.key : -1;
      float Jk = 0.f;
      if (key >= 0) {
        float R[9];
        f3 centre, anchor;
        key_frame(m, W, key, R, &centre, &anchor);
        Jk = -dot3(u, cross3(mk3(0, 1, 0), p - anchor));
      }
      float vv = lane < NDT ? W.v[NK + lane] : 0.f, qa = lane < NDT ? W.qas[NK + lane] : 0.f,
            qw = lane < NDT ? W.qws[NK + lane] : 0.f;
      if (lane == KEYLANE) {
        J = Jk;
        vv = key >= 0 ? W.v[key] : 0.f;
        qa = key >= 0 ? W.qas[key] : 0.f;
        qw = key >= 0 ? W.qws[key] : 0.f;
      }
      jv[dI] = wave_sum(J * vv);
      jqs[dI] = wave_sum(J * qa);
      jws[dI] = wave_sum(J * qw);
      if (rbase + dI < maxrow && lane < ROWSTRIDE) W.Y[rbase + dI][lane] = J;
    }
    if (lane == 0) {
      for (int e = 0; e < 4 && rbase + e < maxrow; e++) {
        W.r_key[rbase + e] = cc.kind == 0 ? cc.key : -1;
        W.r_mask[rbase + e] = m1 | m2;
      }
    }
    // stash scalars for the edges in r_b/r_R temporarily (consumed below)
    if (lane == 0 && rbase + 3 < maxrow) {
      W.r_b[rbase + 0] = jv[0]; W.r_b[rbase + 1] = jv[1]; W.r_b[rbase + 2] = jv[2];
      W.r_R[rbase + 0] = jqs[0]; W.r_R[rbase + 1] = jqs[1]; W.r_R[rbase + 2] = jqs[2];
      W.r_f[rbase + 0] = jws[0]; W.r_f[rbase + 1] = jws[1]; W.r_f[rbase + 2] = jws[2];
    } else if (lane == 0) {
      for (int e = 0; e < 3 && rbase + e < maxrow; e++) { W.r_b[rbase + e] = jv[e]; W.r_R[rbase + e] = jqs[e]; W.r_f[rbase + e] = jws[e]; }
    }
    ncr = c + 1;
  }
  __syncthreads();
  // L^-T of the three direction rows of every contact (stored in edge slots 0..2)
  {
    int nrows = 0;
    // lane handles direction row (c, d) -> row index nr + 4c + d
    for (int t = lane; t < 3 * ncr; t += 64) {
      int c = t / 3, dI = t - 3 * c;
      int r = nr + 4 * c + dI;
      if (r >= maxrow) continue;
      uint64_t mask = W.r_mask[r];
      float* y = W.Y[r];
      while (mask) {
        int k = 63 - __clzll(mask);
        mask &= ~(1ull << k);
        float yk = y[k];
        if (yk == 0.f) continue;
        int dk = m->dof_depth[k];
        for (int a = 1; a <= dk; a++) y[m->dof_anc[k][a]] -= W.M[k][a] * yk;
      }
    }
    (void)nrows;
    __syncthreads();
  }
  // expand to edges and finish scalars
  for (int c = 0; c < ncr; c++) {
    const Contact& cc = W.con[c];
    int rbase = nr + 4 * c;
    const float* sr = cc.kind == 2 ? m->hc_solref : m->pc_solref;
    const float* si = cc.kind == 2 ? m->hc_solimp : m->pc_solimp;
    float solref[2], solimp[5];
    for (int i = 0; i < 2; i++) solref[i] = 0.5f * (sr[i] + m->hc_solref[i]);
    for (int i = 0; i < 5; i++) solimp[i] = 0.5f * (si[i] + m->hc_solimp[i]);
    float mu = fmaxf(cc.kind == 2 ? m->hc_fric : m->pc_fric, m->hc_fric);
    int B2 = m->geom_body[cc.g2];
    float tran = m->body_binv[B2];
    if (cc.kind == 0) tran += m->key_binv[cc.key];
    else if (cc.kind == 2) tran += m->body_binv[m->geom_body[cc.g1]];
    float diag = (1.f + mu * mu) * tran;
    float jv[3], jqs[3], jws[3];
    int nd = maxrow - rbase < 3 ? maxrow - rbase : 3;
    for (int e = 0; e < 3; e++) {
      jv[e] = e < nd ? W.r_b[rbase + e] : 0.f;
      jqs[e] = e < nd ? W.r_R[rbase + e] : 0.f;
      jws[e] = e < nd ? W.r_f[rbase + e] : 0.f;
    }
    __syncthreads();
    if (lane < ROWSTRIDE) {
      float yn = W.Y[rbase][lane];
      float y1 = nd > 1 ? W.Y[rbase + 1][lane] : 0.f;
      float y2 = nd > 2 ? W.Y[rbase + 2][lane] : 0.f;
      if (rbase + 0 < maxrow) W.Y[rbase + 0][lane] = yn + mu * y1;
      if (rbase + 1 < maxrow) W.Y[rbase + 1][lane] = yn - mu * y1;
      if (rbase + 2 < maxrow) W.Y[rbase + 2][lane] = yn + mu * y2;
      if (rbase + 3 < maxrow) W.Y[rbase + 3][lane] = yn - mu * y2;
    }
    __syncthreads();
    for (int e = 0; e < 4 && rbase + e < maxrow; e++) {
      int t = e < 2 ? 1 : 2;
      float s = (e & 1) ? -mu : mu;
      row_scalars(m, W, rbase + e, cc.dist, solref, solimp, diag, jv[0] + s * jv[t], jqs[0] + s * jqs[t],
                  jws[0] + s * jws[t], lane);
    }
    __syncthreads();
  }
  int total = nr + 4 * ncr;
  if (lane == 0) W.nrow = total < maxrow ? total : maxrow;
  (void)cfirst;
  __syncthreads();
}

// PGS over the coupled rows (dual), then qfrc_constraint = L^T w, qacc solves, Euler
__device__ void solve_and_integrate(const DevModel* __restrict__ m, Work& W, int iters, int lane) {
  int nrow = W.nrow;
  // w = sum_r y_r f_r ; hand part in a register (lane = dof), keys in LDS
  float wl = 0.f;
  for (int k = lane; k < NK; k += 64) W.w[k] = 0.f;
  __syncthreads();
  for (int r = 0; r < nrow; r++) {
    float f = W.r_f[r];
    if (lane < NDT) wl += W.Y[r][lane] * f;
    if (lane == KEYLANE && W.r_key[r] >= 0) W.w[W.r_key[r]] += W.Y[r][KEYLANE] * f;
  }
  float dinv = lane < NDT ? W.Dinv[lane] : 0.f;
  for (int it = 0; it < iters; it++) {
    for (int r = 0; r < nrow; r++) {
      float y = lane < ROWSTRIDE ? W.Y[r][lane] : 0.f;
      int key = W.r_key[r];
      float p;
      if (lane < NDT) p = y * wl * dinv;
      else if (lane == KEYLANE && key >= 0) p = y * W.w[key] * m->key_Minv[key];
      else p = 0.f;
      float s = wave_sum(p);
      float f = W.r_f[r];
      float res = W.r_b[r] + W.r_R[r] * f + s;
      float fn = fmaxf(0.f, f - res * W.r_arinv[r]);
      float df = fn - f;
      if (lane < NDT) wl += y * df;
      if (lane == KEYLANE && key >= 0) W.w[key] += y * df;
      if (lane == 0) W.r_f[r] = fn;
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane < NDT) W.w[NK + lane] = wl;
  __syncthreads();
  // F = qfrc_smooth + J^T f  (keys: w + closed-form rows; hands: L^T w, pull from descendants)
  for (int k = lane; k < NK; k += 64) W.tmp[k] = W.qfs[k] + W.w[k] + W.tmp2[k];
  if (lane < NDT) {
    int i = lane;
    float s = W.w[NK + i];
    int di = m->dof_depth[i];
    for (int c = 0; c < m->dof_ndesc[i]; c++) {
      int k = m->dof_desc[i][c];
      s += W.M[k][m->dof_depth[k] - di] * W.w[NK + k];
    }
    W.tmp[NK + i] = W.qfs[NK + i] + s;
  }
  __syncthreads();
  for (int i = lane; i < NV; i += 64) { W.qas[i] = W.tmp[i]; W.tmp2[i] = W.tmp[i]; }
  __syncthreads();
  solve<false>(m, W, W.qas, lane);   // qacc (solver output) -> warm start
  solve<true>(m, W, W.tmp2, lane);   // (M + h D)^-1 F  (mj_Euler implicit damping)
  __syncthreads();
  float h = m->timestep;
  for (int i = lane; i < NV; i += 64) {
    W.qws[i] = W.qas[i];
    float vn = W.v[i] + h * W.tmp2[i];
    W.v[i] = vn;
    W.q[i] += h * vn;
  }
  __syncthreads();
}

// ------------------------------------------------------------------ task layer
__device__ __forceinline__ float tolerance(float x, float lo, float hi, float margin) {
  if (x >= lo && x <= hi) return 1.f;
  float dd = (x < lo ? lo - x : x - hi) / margin;
  const float scale2 = 4.605170185988091f;  // -2 ln(0.1)
  return expf(-0.5f * dd * dd * scale2);
}

__device__ f3 site_world(const DevModel* __restrict__ m, const Work& W, int s) {
  int B = m->site_body[s];
  return ld3(W.o[B]) + mv3(W.R[B], ld3(m->site_pos[s]));
}

__device__ f3 key_target(const DevModel* __restrict__ m, const Work& W, int k) {
  float R[9];
  f3 c, a;
  key_frame(m, W, k, R, &c, &a);
  c.x += 0.35f * m->key_half[k][0];
  c.z += 0.5f * m->key_half[k][2];
  return c;
}

// rectangular min-cost assignment (rows n <= cols mm), sum of tol over assigned pairs
__device__ float hungarian_tol(int n, int mm, const float* c /*[n][mm]*/) {
  float u[17], v[17], minv[17];
  int p[17], way[17];
  bool used[17];
  for (int i = 0; i <= n; i++) u[i] = 0.f;
  for (int j = 0; j <= mm; j++) { v[j] = 0.f; p[j] = 0; way[j] = 0; }
  for (int i = 1; i <= n; i++) {
    p[0] = i;
    int j0 = 0;
    for (int j = 0; j <= mm; j++) { minv[j] = INFINITY; used[j] = false; }
    do {
      used[j0] = true;
      int i0 = p[j0], j1 = 0;
      float delta = INFINITY;
      for (int j = 1; j <= mm; j++)
        if (!used[j]) {
          float cur = c[(i0 - 1) * mm + j - 1] - u[i0] - v[j];
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
  float s = 0.f;
  for (int j = 1; j <= mm; j++)
    if (p[j]) s += tolerance(c[(p[j] - 1) * mm + j - 1], 0.f, 0.01f, 0.1f);
  return s;
}

__device__ void write_obs(const DevModel* __restrict__ m, const Song& song, const Cfg& cfg, const Work& W, int t_obs,
                          float* __restrict__ obs, int lane) {
  int G = (cfg.lookahead + 1) * (NK + 1);
  int o_f = G, o_s = G + (cfg.fingering ? 10 : 0);
  for (int i = lane; i < cfg.obs_dim; i += 64) {
    float val;
    if (i < G) {
      int j = i / (NK + 1), k = i - j * (NK + 1);
      int t = t_obs + j;
      val = t < song.T ? song.goal[t * (NK + 1) + k] : 0.f;
    } else if (i < o_s) {
      int slot = i - o_f;  // hand*5 + finger
      val = 0.f;
      for (int n = 0; n < song.count[t_obs]; n++) {
        int f = song.fingers[t_obs * PS_MAX_NOTES + n];
        int idx = f < 5 ? (f < 0 ? f + 5 : f) : f;
        if (idx == slot) val = 1.f;
      }
    } else if (i < o_s + NK) {
      val = W.norm_state[i - o_s];
    } else if (i == o_s + NK) {
      val = W.sustain;
    } else {
      val = W.q[NK + m->obs_dof[i - o_s - NK - 1]];
    }
    obs[i] = val;
  }
}

__device__ void key_state(const DevModel* __restrict__ m, Work& W, int lane) {
  uint64_t b0 = 0, b1 = 0;
  for (int k0 = 0; k0 < NK; k0 += 64) {
    int k = k0 + lane;
    bool act = false;
    if (k < NK) {
      float lo = m->key_lo[k], hi = m->key_hi[k];
      float s = clampf(W.q[k], lo, hi);
      W.norm_state[k] = s / hi;
      act = fabsf(s - hi) <= KEY_THRESHOLD;
    }
    uint64_t mk = __ballot(act);
    if (k0 == 0) b0 = mk; else b1 = mk;
  }
  if (lane == 0) {
    W.act_bits[0] = (int)(b0 & 0xffffffffull);
    W.act_bits[1] = (int)(b0 >> 32);
    W.act_bits[2] = (int)(b1 & 0xffffffull);
  }
  __syncthreads();
}
__device__ __forceinline__ bool key_active(const Work& W, int k) {
  return (W.act_bits[k >> 5] >> (k & 31)) & 1;
}

// ------------------------------------------------------------------ diagnostic phase timing
// Built only with -DPS_TIMING (libpianosim_timing.so): per-phase s_memtime deltas summed
// per env into a debug buffer. The production library contains none of this.
#ifdef PS_TIMING
#define NPHASE 12
#define TSTAMP(slot)                                                      \
  do {                                                                    \
    __syncthreads();                                                      \
    uint64_t t_ = __builtin_amdgcn_s_memtime();                          \
    tacc[slot] += t_ - tlast;                                             \
    tlast = t_;                                                           \
  } while (0)
__device__ uint64_t* g_timing = nullptr;
#else
#define TSTAMP(slot) \
  do {               \
  } while (0)
#endif

// ------------------------------------------------------------------ the kernel
__global__ void __launch_bounds__(64) pianosim_kernel(const DevModel* __restrict__ m, Song song, Cfg cfg, Bufs bufs,
                                                      const float* __restrict__ action, const uint8_t* __restrict__ mask,
                                                      float* __restrict__ obs, float* __restrict__ reward,
                                                      float* __restrict__ discount, uint8_t* __restrict__ step_type,
                                                      int mode, int n_envs) {
  __shared__ Work W;
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  if (e >= n_envs) return;
  float* obs_e = obs + (size_t)e * cfg.obs_dim;
  bool do_reset;
  if (mode == 1) {  // reset mode: only masked envs
    if (mask && !mask[e]) return;
    do_reset = true;
  } else {
    do_reset = bufs.last[e] != 0;
  }
  const float* applied = bufs.applied ? bufs.applied + (size_t)e * NV : nullptr;
  if (do_reset) {
    for (int i = lane; i < NV; i += 64) { W.q[i] = 0.f; W.v[i] = 0.f; W.qws[i] = 0.f; }
    for (int i = lane; i < NU; i += 64) W.ctrl[i] = 0.f;
    if (lane == 0) W.sustain = 0.f;
    __syncthreads();
    kinematics(m, W, lane);
    collide(m, W, cfg.maxcon, lane);
    key_state(m, W, lane);
    write_obs(m, song, cfg, W, 0, obs_e, lane);
    for (int i = lane; i < NV; i += 64) {
      bufs.qpos[(size_t)e * NV + i] = 0.f;
      bufs.qvel[(size_t)e * NV + i] = 0.f;
      bufs.qws[(size_t)e * NV + i] = 0.f;
    }
    for (int i = lane; i < NU; i += 64) bufs.ctrl[(size_t)e * NU + i] = 0.f;
    if (lane < PS_NTERMS) bufs.terms[(size_t)e * PS_NTERMS + lane] = 0.f;
    if (lane < 2 * PS_NFINGER) {
      f3 p = site_world(m, W, lane);
      st3(bufs.tips + ((size_t)e * 2 * PS_NFINGER + lane) * 3, p);
    }
    if (lane == 0) {
      bufs.sustain[e] = 0.f;
      bufs.t_idx[e] = 0;
      bufs.last[e] = 0;
      bufs.ncon[e] = W.ncon;
      if (mode == 0) {
        reward[e] = 0.f;
        discount[e] = 1.f;
        step_type[e] = PS_FIRST;
      }
    }
    return;
  }
  // ---- load state
  for (int i = lane; i < NV; i += 64) {
    W.q[i] = bufs.qpos[(size_t)e * NV + i];
    W.v[i] = bufs.qvel[(size_t)e * NV + i];
    W.qws[i] = bufs.qws[(size_t)e * NV + i];
  }
  const float* a_e = action + (size_t)e * PS_NACTION;
  for (int i = lane; i < NU; i += 64) {
    float a = a_e[i];
    // dm_env_wrappers.CanonicalSpecWrapper: [-1, 1] -> [min, max] of the action spec
    W.ctrl[i] = cfg.canonical ? m->act_clo[i] + (a + 1.f) * 0.5f * (m->act_chi[i] - m->act_clo[i]) : a;
  }
  if (lane == 0) W.sustain = cfg.canonical ? (a_e[NU] + 1.f) * 0.5f : a_e[NU];
  __syncthreads();
  // ---- physics substeps
#ifdef PS_TIMING
  uint64_t tacc[NPHASE] = {0};
  uint64_t tlast = __builtin_amdgcn_s_memtime();
#endif
  for (int s = 0; s < m->nsub; s++) {
    if (!(cfg.skip & 1)) kinematics(m, W, lane);
    TSTAMP(0);
    if (!(cfg.skip & 2)) dynamics(m, W, applied, lane);
    TSTAMP(1);
    if (!(cfg.skip & 4)) collide(m, W, cfg.maxcon, lane);
    else if (lane == 0) W.ncon = 0;
    TSTAMP(2);
    if (!(cfg.skip & 8)) factor(m, W, lane);
    TSTAMP(3);
    for (int i = lane; i < NV; i += 64) W.qas[i] = W.qfs[i];
    __syncthreads();
    if (!(cfg.skip & 16)) solve<false>(m, W, W.qas, lane);
    __syncthreads();
    TSTAMP(4);
    if (!(cfg.skip & 32)) constraints(m, W, MAXROW, lane);
    else if (lane == 0) W.nrow = 0;
    __syncthreads();
    TSTAMP(5);
    solve_and_integrate(m, W, (cfg.skip & 64) ? 0 : cfg.pgs_iter, lane);
    TSTAMP(6);
#ifdef PS_TIMING
    if (lane == 0) { tacc[9] += W.nrow; tacc[10] += W.ncon; }
#endif
  }
  // ---- mj_step1 at the final state + task layer
  kinematics(m, W, lane);
  collide(m, W, cfg.maxcon, lane);
  key_state(m, W, lane);
  const int t_cur = bufs.t_idx[e];
  const int t_new = t_cur + 1;
  const float* gc = song.goal + (size_t)t_cur * (NK + 1);
  // key press + failure
  float on_tol = 0.f, on_cnt = 0.f;
  bool fail_l = false;
  for (int k = lane; k < NK; k += 64) {
    float g = gc[k];
    if (g != 0.f) { on_tol += tolerance(g - W.norm_state[k], 0.f, 0.05f, 0.5f); on_cnt += 1.f; }
    else if (key_active(W, k)) fail_l = true;
  }
  float sum_tol = wave_sum(on_tol), n_on = wave_sum(on_cnt);
  bool failure = __ballot(fail_l) != 0ull;
  float kp = (n_on > 0.f ? 0.5f * (sum_tol / n_on) : 0.f) + 0.5f * (1.f - (failure ? 1.f : 0.f));
  float sus = tolerance(gc[NK] - (W.sustain >= SUSTAIN_THRESHOLD ? 1.f : 0.f), 0.f, 0.05f, 0.5f);
  // energy: |actuator force| * |actuator velocity| at the final state
  float en = 0.f;
  if (lane < NU) {
    float vel = m->act_c0[lane] * W.v[NK + m->act_dof0[lane]];
    if (m->act_kind[lane] == 1) vel += m->act_c1[lane] * W.v[NK + m->act_dof1[lane]];
    en = fabsf(W.actf[lane]) * fabsf(vel);
  }
  float energy = -cfg.energy_coef * wave_sum(en);
  float fing = 0.f;
  if (cfg.fingering) {
    float ds = 0.f, dc = 0.f;
    int cnt = song.count[t_cur];
    if (lane < cnt) {
      int f = song.fingers[t_cur * PS_MAX_NOTES + lane], k = song.keys[t_cur * PS_MAX_NOTES + lane];
      bool rh = f < 5;
      int site = rh ? (f < 0 ? f + 5 : f) : f - 5;
      f3 tip = site_world(m, W, (rh ? 0 : 1) * PS_NFINGER + site);
      ds = tolerance(norm3(key_target(m, W, k) - tip), 0.f, 0.01f, 0.1f);
      dc = 1.f;
    }
    float s = wave_sum(ds), c = wave_sum(dc);
    fing = c > 0.f ? s / c : 0.f;
  } else {
    // OT fingering (RP1M): fingertips lh then rh vs goal keys; Hungarian on lane 0
    float res = 0.f;
    if (lane == 0) {
      int keys[PS_MAX_NOTES], K = 0;
      for (int k = 0; k < NK && K < PS_MAX_NOTES; k++)
        if (gc[k] != 0.f) keys[K++] = k;
      if (K == 0) res = 1.f;
      else {
        f3 tips[10];
        for (int i = 0; i < 5; i++) { tips[i] = site_world(m, W, PS_NFINGER + i); tips[5 + i] = site_world(m, W, i); }
        float c[10 * PS_MAX_NOTES];
        if (K <= 10) {
          for (int j = 0; j < K; j++)
            for (int i = 0; i < 10; i++) c[j * 10 + i] = norm3(key_target(m, W, keys[j]) - tips[i]);
          res = hungarian_tol(K, 10, c) / K;
        } else {
          for (int i = 0; i < 10; i++)
            for (int j = 0; j < K; j++) c[i * K + j] = norm3(key_target(m, W, keys[j]) - tips[i]);
          res = hungarian_tol(10, K, c) / 10.f;
        }
      }
    }
    fing = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(res)));
  }
  float fore = 0.f;
  if (cfg.forearm) {
    bool hit = false;
    if (lane < W.ncon) {
      const Contact& cc = W.con[lane];
      if (cc.kind == 2) {
        int la = cc.g1 % NG, lb = cc.g2 % NG;
        hit = (cc.g1 / NG != cc.g2 / NG) && la < m->root_geom_count && lb < m->root_geom_count;
      }
    }
    fore = __ballot(hit) ? 0.f : 0.5f;
  }
  bool terminal = t_new == song.T;
  float disc = 1.f;
  if (!terminal && cfg.wrong_press && failure) { terminal = true; disc = 0.f; }
  write_obs(m, song, cfg, W, t_new < song.T ? t_new : t_new - 1, obs_e, lane);
  TSTAMP(7);
#ifdef PS_TIMING
  if (lane == 0 && g_timing)
    for (int i = 0; i < NPHASE; i++) g_timing[(size_t)e * NPHASE + i] += tacc[i];
#endif
  // ---- write back
  for (int i = lane; i < NV; i += 64) {
    bufs.qpos[(size_t)e * NV + i] = W.q[i];
    bufs.qvel[(size_t)e * NV + i] = W.v[i];
    bufs.qws[(size_t)e * NV + i] = W.qws[i];
  }
  for (int i = lane; i < NU; i += 64) bufs.ctrl[(size_t)e * NU + i] = W.ctrl[i];
  if (lane < 2 * PS_NFINGER) {
    f3 p = site_world(m, W, lane);
    st3(bufs.tips + ((size_t)e * 2 * PS_NFINGER + lane) * 3, p);
  }
  if (lane == 0) {
    float* tm = bufs.terms + (size_t)e * PS_NTERMS;
    tm[0] = kp; tm[1] = sus; tm[2] = energy; tm[3] = fing; tm[4] = fore;
    reward[e] = kp + sus + energy + fing + fore;
    discount[e] = disc;
    step_type[e] = terminal ? PS_LAST : PS_MID;
    bufs.sustain[e] = W.sustain;
    bufs.t_idx[e] = t_new;
    bufs.last[e] = terminal ? 1 : 0;
    bufs.ncon[e] = W.ncon;
  }
}

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
  int n, device, obs_dim;
  ps_task_cfg cfg;
  DevModel* d_model;
  int T;
  float* d_goal;
  int *d_count, *d_keys, *d_fingers;
  float *qpos, *qvel, *qws, *ctrl, *sustain, *applied, *terms, *tips;
  int *t_idx, *ncon;
  uint8_t* last;
  bool applied_on;
};

static void quat2mat_h(const double* q, float* R) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  double w = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
  double M[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                 2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                 2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
  for (int i = 0; i < 9; i++) R[i] = (float)M[i];
}

// Derive the flattened device model + topology tables from the descriptor.
static int build_dev_model(const ps_model_desc* d, DevModel* m) {
  memset(m, 0, sizeof(*m));
  m->timestep = (float)d->timestep;
  m->nsub = d->n_substeps;
  for (int i = 0; i < 3; i++) m->grav[i] = (float)d->gravity[i];
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
      if (m->body_dof[B] < 0) m->body_dof[B] = g;
      else if (m->body_dof[B] + m->body_ndof[B] != g) return fail("dofs of a body must be contiguous");
      m->body_ndof[B]++;
      m->obs_dof[g] = h * ND + d->dof_obs_order[h][j];
      m->dof_act[g] = -1;
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
    m->body_pathmask[B] = mask;
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
  // actuators + tendons
  for (int h = 0; h < NH; h++)
    for (int a = 0; a < NA; a++) {
      int A = h * NA + a, tg = d->act_target[h][a];
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
      m->act_kp[A] = (float)d->act_kp[h][a];
      m->act_clo[A] = (float)d->act_ctrlrange[h][a][0];
      m->act_chi[A] = (float)d->act_ctrlrange[h][a][1];
      m->act_flim[A] = d->act_forcelimited[h][a];
      m->act_flo[A] = (float)d->act_forcerange[h][a][0];
      m->act_fhi[A] = (float)d->act_forcerange[h][a][1];
      int dofs[2] = {m->act_dof0[A], m->act_dof1[A]};
      float cs[2] = {m->act_c0[A], m->act_c1[A]};
      for (int i = 0; i < (m->act_kind[A] == 1 ? 2 : 1); i++) {
        if (m->dof_act[dofs[i]] >= 0) return fail("a dof may be driven by at most one actuator");
        m->dof_act[dofs[i]] = A;
        m->dof_act_coef[dofs[i]] = cs[i];
      }
    }
  // geoms, sites, pairs
  for (int h = 0; h < NH; h++)
    for (int g = 0; g < NG; g++) {
      int G = h * NG + g;
      m->geom_body[G] = h * NB + d->geom_body[h][g];
      for (int i = 0; i < 3; i++) {
        m->geom_pos[G][i] = (float)d->geom_pos[h][g][i];
        m->geom_axis[G][i] = (float)d->geom_axis[h][g][i];
      }
      m->geom_hl[G] = (float)d->geom_halflen[h][g];
      m->geom_r[G] = (float)d->geom_radius[h][g];
    }
  m->root_geom_count = d->root_geom_count;
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
  }
  return 0;
}

extern "C" {

const char* ps_last_error(void) { return g_err.c_str(); }
int ps_version(void) { return 1; }
int ps_model_desc_size(void) { return (int)sizeof(ps_model_desc); }
int ps_obs_dim(const ps_task_cfg* cfg) {
  return (cfg->n_steps_lookahead + 1) * (NK + 1) + (cfg->fingering_reward ? 10 : 0) + NK + 1 + NH * ND;
}

int ps_create(const ps_model_desc* model, const ps_song_desc* song, const ps_task_cfg* cfg, int n_envs, int device,
              uint64_t seed, ps_env** out) {
  (void)seed;
  if (!model || !song || !cfg || !out) return fail("null argument");
  if (n_envs <= 0) return fail("n_envs must be positive");
  if (song->T <= 0) return fail("empty song");
  if (cfg->n_steps_lookahead < 0) return fail("negative lookahead");
  if (cfg->max_contacts < 0 || cfg->max_contacts > MAXCON) return fail("max_contacts out of range");
  if (cfg->pgs_iterations < 0) return fail("negative pgs_iterations");
  for (int t = 0; t < song->T; t++)
    if (song->count[t] < 0 || song->count[t] > PS_MAX_NOTES) return fail("bad note count");
  HIPCHK(hipSetDevice(device));
  DevModel* hm = new DevModel;
  if (build_dev_model(model, hm)) { delete hm; return -1; }
  ps_env* E = new ps_env();
  E->n = n_envs;
  E->device = device;
  E->cfg = *cfg;
  E->obs_dim = ps_obs_dim(cfg);
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
  HIPCHK(hipMalloc(&E->last, N));
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
  HIPCHK(hipMemset(E->last, 0, N));
  HIPCHK(hipDeviceSynchronize());
  E->applied_on = false;
  *out = E;
  return 0;
}

void ps_destroy(ps_env* E) {
  if (!E) return;
  (void)hipSetDevice(E->device);
  hipFree(E->d_model); hipFree(E->d_goal); hipFree(E->d_count); hipFree(E->d_keys); hipFree(E->d_fingers);
  hipFree(E->qpos); hipFree(E->qvel); hipFree(E->qws); hipFree(E->applied); hipFree(E->ctrl); hipFree(E->sustain);
  hipFree(E->terms); hipFree(E->tips); hipFree(E->t_idx); hipFree(E->ncon); hipFree(E->last);
  delete E;
}

static int launch(ps_env* E, int mode, const float* action, const uint8_t* mask, float* obs, float* reward,
                  float* discount, uint8_t* step_type, void* stream) {
  Song song{E->T, E->d_goal, E->d_count, E->d_keys, E->d_fingers};
  Cfg cfg{E->cfg.n_steps_lookahead, E->cfg.fingering_reward, E->cfg.forearm_reward, E->cfg.wrong_press_termination,
          E->cfg.pgs_iterations, E->cfg.max_contacts, E->obs_dim, E->cfg.canonical_actions,
          (float)E->cfg.energy_penalty_coef, 0};
  if (const char* sk = getenv("PIANOSIM_SKIP")) cfg.skip = atoi(sk);
  Bufs b{E->qpos, E->qvel, E->qws, E->ctrl, E->sustain, E->t_idx, E->last,
         E->applied_on ? E->applied : nullptr, E->terms, E->tips, E->ncon};
  hipLaunchKernelGGL(pianosim_kernel, dim3(E->n), dim3(64), 0, (hipStream_t)stream, E->d_model, song, cfg, b, action,
                     mask, obs, reward, discount, step_type, mode, E->n);
  HIPCHK(hipGetLastError());
  return 0;
}

int ps_reset(ps_env* E, const uint8_t* env_mask, float* obs, void* stream) {
  if (!E || !obs) return fail("null argument");
  return launch(E, 1, nullptr, env_mask, obs, nullptr, nullptr, nullptr, stream);
}

int ps_step(ps_env* E, const float* action, float* obs, float* reward, float* discount, uint8_t* step_type,
            void* stream) {
  if (!E || !action || !obs || !reward || !discount || !step_type) return fail("null argument");
  return launch(E, 0, action, nullptr, obs, reward, discount, step_type, stream);
}

int ps_get_state(ps_env* E, float* qpos, float* qvel, float* qacc_ws, float* ctrl, float* sustain, int32_t* t_idx,
                 uint8_t* last, void* stream) {
  if (!E) return fail("null env");
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
  HIPCHK(hipMemcpyAsync(terms, E->terms, sizeof(float) * E->n * PS_NTERMS, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return 0;
}

int ps_fingertips(ps_env* E, float* xpos, void* stream) {
  if (!E || !xpos) return fail("null argument");
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

int ps_contact_count(ps_env* E, int32_t* ncon, void* stream) {
  if (!E || !ncon) return fail("null argument");
  HIPCHK(hipMemcpyAsync(ncon, E->ncon, sizeof(int) * E->n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

}  // extern "C"
