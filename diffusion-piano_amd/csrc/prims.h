// prims.h - device math, wave primitives and narrow-phase collision shared by the
// pianosim kernels (algorithms stated sequentially in the CPU checker).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "devmodel.h"

namespace ps {

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
// 64-lane min via DPP (same pattern as wave_sum; bound_ctrl off keeps the lane's own value)
__device__ __forceinline__ float wave_min(float v) {
  int x = __float_as_int(v);
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x111, 0xF, 0xF, false)));
  x = __float_as_int(v);
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x112, 0xF, 0xF, false)));
  x = __float_as_int(v);
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x114, 0xF, 0xF, false)));
  x = __float_as_int(v);
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x118, 0xF, 0xF, false)));
  x = __float_as_int(v);
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x142, 0xA, 0xF, false)));
  x = __float_as_int(v);
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x143, 0xC, 0xF, false)));
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
// exclusive prefix sum and total of small non-negative counts (< 2^BITS) by bit-plane
// ballots: BITS ballots + mbcnt, no cross-lane data movement
template <int BITS = 5>
__device__ __forceinline__ int small_excl_scan(int v, int lane, int* total) {
  int ex = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; b++) {
    const uint64_t m = __ballot((v >> b) & 1);
    ex += lanes_below(m, lane) << b;
    tot += __popcll(m) << b;
  }
  *total = tot;
  return ex;
}

// Exchange point of a ONE-WAVE workgroup (every kernel here is launched with 64 threads):
// the wave's LDS operations are performed in issue order, so a value another lane reads
// after this point was written before it without any wait; what must not happen is the
// compiler moving LDS accesses across it or keeping a stale LDS value in a register.
// __syncthreads() would add s_waitcnt lgkmcnt(0), stalling on every LDS / scalar load in
// flight at ~40 exchange points per physics substep.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Philox4x32-10 (Salmon et al., SC'11), 10 rounds
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// randomize_hand_positions draw of (seed, env, episode): U(-0.05, 0.05) from 24 random bits,
// as oracle/pianosim_ref.c ref_hand_offset_draw (bitwise: same bits, same fma)
__device__ __forceinline__ float hand_offset_draw(uint32_t seed_lo, uint32_t seed_hi, int env, int episode) {
  uint32_t c[4] = {(uint32_t)episode, (uint32_t)env, 0x68616e64u /* "hand" */, 0u};
  philox4x32_10(c, seed_lo, seed_hi);
  const float u = (float)(c[0] >> 8) * 0x1p-24f;
  return fmaf((float)(2.0 * PS_HAND_POSITION_OFFSET), u, (float)-PS_HAND_POSITION_OFFSET);
}

struct Contact {
  float pos[3], n[3], t1[3], t2[3], dist;
  int kind, key, g1, g2;  // g1: -1 for key/base (kind 0/1)
};

// ------------------------------------------------------------------ narrow phase
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

// Segment parameter t in [0,1] closest to a box (box frame, half sizes hs): the squared
// distance is convex and piecewise quadratic in t with breakpoints where the segment crosses
// a face plane; minimise each piece in closed form. Register-only: the 8 breakpoints (0, 1
// and the 6 plane crossings, 1 when outside (0,1)) go through a fixed sorting network.
__device__ __forceinline__ void cswap(float& x, float& y) {
  const float lo = fminf(x, y), hi = fmaxf(x, y);
  x = lo;
  y = hi;
}
__device__ __forceinline__ float seg_box_t(f3 a3, f3 d3, const float* hs) {
  const float a[3] = {a3.x, a3.y, a3.z}, dv[3] = {d3.x, d3.y, d3.z};
  float bp[8];
  bp[0] = 0.f;
  bp[7] = 1.f;
#pragma unroll
  for (int i = 0; i < 3; i++) {
#pragma unroll
    for (int sg = 0; sg < 2; sg++) {
      float t = 1.f;
      if (dv[i] != 0.f) {
        const float tt = ((sg ? hs[i] : -hs[i]) - a[i]) / dv[i];
        if (tt > 0.f && tt < 1.f) t = tt;
      }
      bp[1 + 2 * i + sg] = t;
    }
  }
  // Batcher odd-even merge sort network for 8 keys (19 compare-exchanges)
  cswap(bp[0], bp[1]); cswap(bp[2], bp[3]); cswap(bp[4], bp[5]); cswap(bp[6], bp[7]);
  cswap(bp[0], bp[2]); cswap(bp[1], bp[3]); cswap(bp[4], bp[6]); cswap(bp[5], bp[7]);
  cswap(bp[1], bp[2]); cswap(bp[5], bp[6]);
  cswap(bp[0], bp[4]); cswap(bp[1], bp[5]); cswap(bp[2], bp[6]); cswap(bp[3], bp[7]);
  cswap(bp[2], bp[4]); cswap(bp[3], bp[5]);
  cswap(bp[1], bp[2]); cswap(bp[3], bp[4]); cswap(bp[5], bp[6]);
  float bestf = INFINITY, bestt = 0.f;
#pragma unroll
  for (int s = 0; s < 7; s++) {
    const float lo = bp[s], hi = bp[s + 1];
    if (!(hi > lo)) continue;
    float mid = 0.5f * (lo + hi), num = 0.f, den = 0.f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      float x = a[i] + mid * dv[i];
      float tgt = x > hs[i] ? hs[i] : (x < -hs[i] ? -hs[i] : 0.f);
      if (tgt == 0.f && fabsf(x) <= hs[i]) continue;
      num -= (a[i] - tgt) * dv[i];
      den += dv[i] * dv[i];
    }
    float t = den > 0.f ? clampf(num / den, lo, hi) : lo;
    float f = 0.f;
#pragma unroll
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

// capsule (geom2) vs box (geom1); writes up to 2 contacts at out (if non-null), returns count.
// Not inlined: its four call sites (count / write pass, substep / task layer) would each
// carry a copy of the segment-box search, and the kernel is instruction-cache bound enough
// that one shared copy measures ~2% faster (tools/throughput.py A/B on MI355X).
// The box frame is a rotation about +y (keys; the base: cq = 1, sq = 0) and comes in by
// value, like the half sizes: arrays passed by pointer to an out-of-line function live in
// scratch memory, a store/load round trip through the vector memory path per call.
#ifndef PS_CBOX_ATTR
#define PS_CBOX_ATTR __noinline__
#endif
template <int WPE>  // the calling kernel's waves per SIMD (one out-of-line copy per register budget)
__device__ PS_CBOX_ATTR int capsule_box(f3 p0, f3 p1, float r, f3 c, float cq, float sq, f3 hsv, Contact* out, int slot,
                           int maxc, int kind, int key, int g2) {
  const float R[9] = {cq, 0.f, sq, 0.f, 1.f, 0.f, -sq, 0.f, cq};
  const float hs[3] = {hsv.x, hsv.y, hsv.z};
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

// sin/cos for the joint-angle range (|x| << 1e4): Cody-Waite reduction by pi/2 and the
// Cephes minimax polynomials on [-pi/4, pi/4] (~1 ulp); no table loads, no slow path.
__device__ __forceinline__ void fsincos(float x, float* sp, float* cp) {
  const float k = rintf(x * 0.636619772367581343f);
  float r = fmaf(-k, 1.57079637050628662f, x);
  r = fmaf(-k, -4.37113900018624283e-8f, r);
  const float z = r * r;
  const float sn = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
  const float cs = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                        fmaf(-0.5f, z, 1.f));
  const int q = (int)k & 3;
  float s = (q & 1) ? cs : sn, c = (q & 1) ? sn : cs;
  if (q == 1 || q == 2) c = -c;
  if (q & 2) s = -s;
  *sp = s;
  *cp = c;
}

__device__ __forceinline__ float impedance(const float* si, float pos) {
  float d0 = clampf(si[0], MINIMP, MAXIMP), dw = clampf(si[1], MINIMP, MAXIMP);
  float width = si[2], mid = si[3], power = si[4];
  float x = fabsf(pos) / width, imp;
  if (x >= 1.f || width <= MINVALF) imp = dw;
  else {
    float y;
    if (power == 1.f) y = x;
    else if (power == 2.f) y = x <= mid ? x * x / mid : 1.f - (1.f - x) * (1.f - x) / (1.f - mid);
    else if (x <= mid) y = powf(x, power) / powf(mid, power - 1.f);
    else y = 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
    imp = d0 + y * (dw - d0);
  }
  return clampf(imp, MINIMP, MAXIMP);
}

// sklearn precision_recall_fscore_support(average="binary", zero_division=1) from counts:
// P = tp / (tp + fp), R = tp / (tp + fn), F = 2 tp / (2 tp + fp + fn), 1 where 0 / 0
__device__ __forceinline__ void prf(int tp, int fp, int fn, float* out) {
  out[0] = tp + fp ? (float)tp / (float)(tp + fp) : 1.f;
  out[1] = tp + fn ? (float)tp / (float)(tp + fn) : 1.f;
  out[2] = 2 * tp + fp + fn ? (float)(2 * tp) / (float)(2 * tp + fp + fn) : 1.f;
}

__device__ __forceinline__ float tolerance(float x, float lo, float hi, float margin) {
  if (x >= lo && x <= hi) return 1.f;
  float dd = (x < lo ? lo - x : x - hi) / margin;
  const float scale2 = 4.605170185988091f;  // -2 ln(0.1)
  return expf(-0.5f * dd * dd * scale2);
}

// rectangular min-cost assignment (rows n <= cols mm), sum of tol over assigned pairs.
// Runs on one lane; its work arrays (w: 3 * (mm + 1) floats then 3 * (mm + 1) ints) are in
// LDS: as private arrays with data-dependent indices they would sit in scratch memory.
__device__ __forceinline__ float hungarian_tol(int n, int mm, const float* c /*[n][mm]*/, float* w) {
  float* u = w;
  float* v = u + (mm + 1);
  float* minv = v + (mm + 1);
  int* p = reinterpret_cast<int*>(minv + (mm + 1));
  int* way = p + (mm + 1);
  int* used = way + (mm + 1);
  for (int i = 0; i <= n; i++) u[i] = 0.f;
  for (int j = 0; j <= mm; j++) { v[j] = 0.f; p[j] = 0; way[j] = 0; }
  for (int i = 1; i <= n; i++) {
    p[0] = i;
    int j0 = 0;
    for (int j = 0; j <= mm; j++) { minv[j] = INFINITY; used[j] = 0; }
    // every trip marks one more column used, so a finite cost matrix ends this in <= mm + 1
    // trips; the cap (and j1 = 0 when no column qualifies) only stops non-finite costs from
    // looping forever
    int trips = 0;
    do {
      used[j0] = 1;
      int i0 = p[j0], j1 = 0;
      float delta = INFINITY;
      const float ui0 = u[i0];
      for (int j = 1; j <= mm; j++)
        if (!used[j]) {
          float cur = c[(i0 - 1) * mm + j - 1] - ui0 - v[j];
          if (cur < minv[j]) { minv[j] = cur; way[j] = j0; }
          if (minv[j] < delta) { delta = minv[j]; j1 = j; }
        }
      for (int j = 0; j <= mm; j++)
        if (used[j]) { u[p[j]] += delta; v[j] -= delta; }
        else minv[j] -= delta;
      j0 = j1;
    } while (p[j0] != 0 && ++trips <= mm);
    trips = 0;
    do { int j1 = way[j0]; p[j0] = p[j1]; j0 = j1; } while (j0 && ++trips <= mm);
  }
  float s = 0.f;
  for (int j = 1; j <= mm; j++)
    if (p[j]) s += tolerance(c[(p[j] - 1) * mm + j - 1], 0.f, 0.01f, 0.1f);
  return s;
}


}  // namespace ps
