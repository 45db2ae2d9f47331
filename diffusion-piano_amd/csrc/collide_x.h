// collide_x.h - narrow phases of the box and convex-hull hand colliders (MuJoCo geom types
// box and mesh; the Menagerie hand's palm boxes and distal meshes, shadow_hand.py:95,144-152):
// Minkowski portal refinement for every pair with a hull (libccd's ccdMPRPenetration, what
// MuJoCo's mjc_Convex runs for meshes: one contact), separating axes + face clipping for
// box-box (up to 4 contacts), and capsule vs oriented box. Stated sequentially in
// oracle/pianosim_ref.c (support, mpr_penetration, box_box, extra_pair); this is the same
// algorithm in fp32, one pair per lane, registers only (no scratch: every small array is
// indexed by unrolled loops).
#pragma once
#include "prims.h"

namespace ps {

// world collider of a lane's narrow phase
struct XShape {
  int type;        // 0 capsule, PS_GEOM_BOX, PS_GEOM_HULL
  f3 c;            // centre (capsule: segment midpoint)
  float R[9];      // rotation (box / hull), row-major
  f3 p0, p1;       // capsule segment
  float r;         // capsule radius
  f3 hs;           // box half sizes
  int v0, nv;      // hull vertices in DevModel::hull_v (geom frame)
  f3 e0, e1;       // hull: an enclosing capsule (world), radius er
  float er;
  const uint64_t* cells;  // hull: its support cells (DevModel::x_cell), or nullptr: scan all vertices
  const float4* cellv;    // hull: its support-cell vertex table (DevModel::x_cellv), or nullptr
  float tie;              // hull: SUP_TIE_HULL x its max vertex norm (x_support's tie band)
};

// Support ties (oracle/pianosim_ref.c support(), the same rule): MPR's portal directions are
// often exactly normal to a hull or box face in exact arithmetic, where every vertex of that
// face is a maximal support and the first-maximal rule picks by the rounding of the dots - a
// choice that differs between fp32 and fp64 and that no perturbation of the state moves, and
// which steered 3% of the benched workload's hull contacts to another portal and normal (round
// 6, tools/contact_diff.py). A hull vertex replaces the running best only when it exceeds it by
// more than SUP_TIE_HULL x rbound x |d| (~10x the fp32 rounding of a projection; below half the
// support cells' pruning margin, so the pruned candidate lists still give the full scan's
// vertex); a box component |dl_i| <= SUP_TIE_BOX max|dl| counts as 0; a capsule axis |ax.d| <=
// SUP_TIE_CAP |ax||d| as perpendicular.
constexpr float SUP_TIE_HULL = 2e-6f;
constexpr float SUP_TIE_BOX = 1e-6f;
constexpr float SUP_TIE_CAP = 1e-6f;

// a collider moved by -o (its centre, segment and enclosing capsule; rotations, half sizes and
// hull vertices are frame-relative)
__device__ __forceinline__ void x_shift(XShape& s, f3 o) {
  s.c = s.c - o;
  s.p0 = s.p0 - o;
  s.p1 = s.p1 - o;
  s.e0 = s.e0 - o;
  s.e1 = s.e1 - o;
}

__device__ __forceinline__ void quat_to_R(float w, float x, float y, float z, float* R) {
  const float n = rsqrtf(w * w + x * x + y * y + z * z);
  w *= n; x *= n; y *= n; z *= n;
  R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - w * z); R[2] = 2.f * (x * z + w * y);
  R[3] = 2.f * (x * y + w * z); R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - w * x);
  R[6] = 2.f * (x * z - w * y); R[7] = 2.f * (y * z + w * x); R[8] = 1.f - 2.f * (x * x + y * y);
}
// rotation matrix -> unit quaternion (Shepperd's method)
__device__ __forceinline__ void R_to_quat(const float* R, float* q) {
  const float t = R[0] + R[4] + R[8];
  if (t > 0.f) {
    const float s = sqrtf(t + 1.f) * 2.f, i = 1.f / s;
    q[0] = 0.25f * s; q[1] = (R[7] - R[5]) * i; q[2] = (R[2] - R[6]) * i; q[3] = (R[3] - R[1]) * i;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    const float s = sqrtf(1.f + R[0] - R[4] - R[8]) * 2.f, i = 1.f / s;
    q[0] = (R[7] - R[5]) * i; q[1] = 0.25f * s; q[2] = (R[1] + R[3]) * i; q[3] = (R[2] + R[6]) * i;
  } else if (R[4] > R[8]) {
    const float s = sqrtf(1.f + R[4] - R[0] - R[8]) * 2.f, i = 1.f / s;
    q[0] = (R[2] - R[6]) * i; q[1] = (R[1] + R[3]) * i; q[2] = 0.25f * s; q[3] = (R[5] + R[7]) * i;
  } else {
    const float s = sqrtf(1.f + R[8] - R[0] - R[4]) * 2.f, i = 1.f / s;
    q[0] = (R[3] - R[1]) * i; q[1] = (R[2] + R[6]) * i; q[2] = (R[5] + R[7]) * i; q[3] = 0.25f * s;
  }
}

__device__ __forceinline__ float sgn0f(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
__device__ __forceinline__ f3 nrmz3(f3 a) {
  const float n = norm3(a);
  return n > 0.f ? a * (1.f / n) : a;
}

// Support cells of a hull (DevModel::x_cell): for each cube-map cell of the direction sphere
// (face 2 ax + (d_ax < 0), cell (i, j) of the tangent ratios d_(ax+1) / |d_ax|, d_(ax+2) / |d_ax|
// over [-1, 1], as hull_cell in collide_x.h) the cone over the cell grown by 0.02 in the ratios,
// spanned by its 4 corner rays c_k. A vertex v is dropped when one vertex u beats it at every
// corner by more than 1e-5 of the hull's extent: (u - v).c_k > tol for all k holds for every
// direction in the cone (a non-negative combination of the c_k), and the margin is far above
// fp32 rounding of the dots, so v never is the fp32 maximum there either. The fp32 scan over
// the rest returns the first maximal vertex of the full scan.
inline void hull_support_cells(const double (*v)[3], int n, uint64_t* out) {
  double ext = 0.0;
  for (int i = 0; i < n; i++) ext = fmax(ext, sqrt(v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2]));
  const double tol = 1e-5 * ext, grow = 0.02;
  for (int face = 0; face < 6; face++)
    for (int ci = 0; ci < XCG; ci++)
      for (int cj = 0; cj < XCG; cj++) {
        const int ax = face / 2;
        const double sg = face % 2 ? -1.0 : 1.0;
        double c[4][3];
        for (int k = 0; k < 4; k++) {
          const double a = -1.0 + 2.0 * (ci + (k & 1)) / XCG + ((k & 1) ? grow : -grow);
          const double b = -1.0 + 2.0 * (cj + (k >> 1)) / XCG + ((k >> 1) ? grow : -grow);
          c[k][ax] = sg;
          c[k][(ax + 1) % 3] = a;
          c[k][(ax + 2) % 3] = b;
        }
        double P[PS_HULL_MAXVERT][4];
        for (int i = 0; i < n; i++)
          for (int k = 0; k < 4; k++) P[i][k] = v[i][0] * c[k][0] + v[i][1] * c[k][1] + v[i][2] * c[k][2];
        uint64_t mask = 0;
        for (int i = 0; i < n; i++) {
          bool dominated = false;
          for (int u = 0; u < n && !dominated; u++) {
            if (u == i) continue;
            bool all = true;
            for (int k = 0; k < 4 && all; k++) all = P[u][k] - P[i][k] > tol;
            dominated = all;
          }
          if (!dominated) mask |= 1ull << i;
        }
        out[(face * XCG + ci) * XCG + cj] = mask;
      }
}

// The support-cell vertex table of a hull (DevModel::x_cellv) from its cells' masks: per cell the
// candidates' fp32 coordinates in ascending vertex order, padded with the last candidate (a
// repeat never wins the first-maximal search), and cell XNCELL = vertex 0 (the zero direction).
// false when a cell holds more than XCV candidates (or none): the mask scan is used instead.
inline bool hull_cell_table(const double (*v)[3], const uint64_t* cells, float (*out)[XCV][4]) {
  for (int c = 0; c <= XNCELL; c++) {
    uint64_t msk = c < XNCELL ? cells[c] : 1ull;
    const int cnt = __builtin_popcountll(msk);
    if (cnt < 1 || cnt > XCV) return false;
    int k = 0, last = 0;
    while (msk) {
      last = __builtin_ctzll(msk);
      msk &= msk - 1ull;
      for (int j = 0; j < 3; j++) out[c][k][j] = (float)v[last][j];
      out[c][k++][3] = 0.f;
    }
    for (; k < XCV; k++)
      for (int j = 0; j < 4; j++) out[c][k][j] = out[c][k - 1][j];
  }
  return true;
}

// support cell of a (local) direction: the cube-map face of its largest component, the cell of
// its two tangent ratios over [-1, 1] (hull_support_cells above builds the tables with
// the same convention; its cells are grown, so rounding at a cell edge picks a cell that still
// holds the direction). Clamped: any input (NaN included) gives a valid cell.
__device__ __forceinline__ int hull_cell(f3 d) {
  const float ex = fabsf(d.x), ey = fabsf(d.y), ez = fabsf(d.z);
  int ax;
  float mj, a, b;
  if (ex >= ey && ex >= ez) { ax = 0; mj = d.x; a = d.y; b = d.z; }
  else if (ey >= ez) { ax = 1; mj = d.y; a = d.z; b = d.x; }
  else { ax = 2; mj = d.z; a = d.x; b = d.y; }
  const float inv = 1.f / fabsf(mj), hg = 0.5f * XCG;
  const int ia = (int)fminf(fmaxf(fmaf(a, inv, 1.f) * hg, 0.f), XCG - 1.f);
  const int ib = (int)fminf(fmaxf(fmaf(b, inv, 1.f) * hg, 0.f), XCG - 1.f);
  return ((2 * ax + (mj < 0.f ? 1 : 0)) * XCG + ia) * XCG + ib;
}

// support point in direction d (the CPU checker's support(): box corner by sign, 0 on a zero
// component; capsule end by sign along the axis + radius along d; hull: first maximal vertex;
// each with the tie rule above)
__device__ __forceinline__ float sgn_tie(float x, float band) { return fabsf(x) <= band ? 0.f : sgn0f(x); }
// box / hull: the support in the collider's own frame (box corner, hull vertex)
__device__ __forceinline__ f3 x_support_local(const DevModel* __restrict__ m, const XShape& s, f3 d) {
  const f3 dl = mtv3(s.R, d);
  f3 loc;
  if (s.type == PS_GEOM_BOX) {
    const float band = SUP_TIE_BOX * fmaxf(fabsf(dl.x), fmaxf(fabsf(dl.y), fabsf(dl.z)));
    loc = mk3(sgn_tie(dl.x, band) * s.hs.x, sgn_tie(dl.y, band) * s.hs.y, sgn_tie(dl.z, band) * s.hs.z);
  } else if (s.cellv) {
    // the first maximal vertex over the direction's cell's candidates (x_cellv: the same
    // candidates as x_cell's mask, in the same order, padded by repeats): the cell's 128 bytes
    // in one round of reads, then the same compares as the mask scan below - the same vertex
    const bool zero = dl.x == 0.f && dl.y == 0.f && dl.z == 0.f;
    const float4* t = s.cellv + (zero ? XNCELL : hull_cell(dl)) * XCV;
    float4 v[XCV];
#pragma unroll
    for (int u = 0; u < XCV; u++) v[u] = t[u];
    const float tie = s.tie * norm3(dl);
    float bd = -INFINITY;
    loc = mk3(0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < XCV; u++) {
      const float p = fmaf(dl.z, v[u].z, fmaf(dl.y, v[u].y, dl.x * v[u].x));
      if (p > bd + tie) { bd = p; loc = mk3(v[u].x, v[u].y, v[u].z); }
    }
  } else if (s.cells) {
    // the first maximal vertex over the candidates of the direction's support cell (x_cell, its
    // bits in ascending vertex order, four per trip: their reads issued together) - the same
    // vertex as the scan over all of them, ~4 candidates instead of ~50 vertices. A zero
    // direction: every dot is 0, the first vertex.
    const bool zero = dl.x == 0.f && dl.y == 0.f && dl.z == 0.f;
    uint64_t msk = zero ? 1ull : s.cells[hull_cell(dl)];
    const float tie = s.tie * norm3(dl);
    float bd = -INFINITY;
    loc = mk3(0.f, 0.f, 0.f);
    while (msk) {
      bool ok[4];
      f3 v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        ok[u] = msk != 0ull;
        const int id = ok[u] ? __builtin_ctzll(msk) : 0;
        msk &= msk - 1ull;
        const float4 q = *reinterpret_cast<const float4*>(m->hull_v[s.v0 + id]);
        v[u] = mk3(q.x, q.y, q.z);
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const float p = fmaf(dl.z, v[u].z, fmaf(dl.y, v[u].y, dl.x * v[u].x));
        if (ok[u] && p > bd + tie) { bd = p; loc = v[u]; }
      }
    }
  } else {
    // every vertex in order (the harness's reference scan; the step kernel has the cells),
    // eight loads issued together
    const float tie = s.tie * norm3(dl);
    float bd = -INFINITY;
    loc = mk3(0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < s.nv; i0 += 8) {
      float4 v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = *reinterpret_cast<const float4*>(m->hull_v[s.v0 + min(i0 + j, s.nv - 1)]);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const float p = fmaf(dl.z, v[j].z, fmaf(dl.y, v[j].y, dl.x * v[j].x));
        if (i0 + j < s.nv && p > bd + tie) { bd = p; loc = mk3(v[j].x, v[j].y, v[j].z); }
      }
    }
  }
  return loc;
}
__device__ __forceinline__ f3 x_support(const DevModel* __restrict__ m, const XShape& s, f3 d) {
  if (s.type == 0) {
    const f3 ax = s.p1 - s.p0;
    const float dn = norm3(d);
    float da = dot3(ax, d);
    if (fabsf(da) <= SUP_TIE_CAP * norm3(ax) * dn) da = 0.f;
    const f3 base = da > 0.f ? s.p1 : (da < 0.f ? s.p0 : (s.p0 + s.p1) * 0.5f);
    return dn > 0.f ? base + d * (s.r / dn) : base;
  }
  return s.c + mv3(s.R, x_support_local(m, s, d));
}

// ------------------------------------------------------------------ MPR
constexpr float MPR_TOLF = 1e-6f;
constexpr int MPR_MAXITF = 50;
constexpr float MPR_EPSF = 2.220446049250313e-16f;  // the double build's CCD_EPS (MuJoCo's libccd), as the checker
struct MprPt {
  f3 v, a, b;
};
__device__ __forceinline__ bool mpr_zero(float x) { return fabsf(x) < MPR_EPSF; }
__device__ __forceinline__ MprPt mpr_sup(const DevModel* __restrict__ m, const XShape& A, const XShape& B, f3 d) {
  MprPt p;
  p.a = x_support(m, A, d);
  p.b = x_support(m, B, d * -1.f);
  p.v = p.a - p.b;
  return p;
}
// Paired MPR (PAIR = true): the two lanes 2k, 2k + 1 of a wave run the same pair in lockstep -
// every portal step computed by both, identically - and split each step's two support
// searches: lane 2k searches A along d, lane 2k + 1 searches B along -d (O = its own collider,
// role = lane & 1), and the points cross over by DPP. The two searches' dependent L2 reads
// (support cell, then its vertices) overlap instead of running one after the other; the
// points are the same bits as mpr_sup's (same function, same arguments).
__device__ __forceinline__ float xchg1(float v) {  // the value of lane ^ 1 (quad_perm [1, 0, 3, 2])
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
template <bool PAIR>
__device__ __forceinline__ MprPt mpr_sup_t(const DevModel* __restrict__ m, const XShape& A, const XShape& B,
                                           const XShape& O, bool role, f3 d) {
  if (!PAIR) return mpr_sup(m, A, B, d);
  const f3 mine = x_support(m, O, role ? d * -1.f : d);
  const f3 oth = mk3(xchg1(mine.x), xchg1(mine.y), xchg1(mine.z));
  MprPt p;
  p.a = role ? oth : mine;
  p.b = role ? mine : oth;
  p.v = p.a - p.b;
  return p;
}
__device__ __forceinline__ f3 portal_dir(const MprPt& p1, const MprPt& p2, const MprPt& p3) {
  return nrmz3(cross3(p2.v - p1.v, p3.v - p1.v));
}
__device__ __forceinline__ bool portal_reach_tol(const MprPt& p1, const MprPt& p2, const MprPt& p3, const MprPt& v4, f3 dir) {
  const float d4 = dot3(v4.v, dir);
  const float mn = fminf(d4 - dot3(p1.v, dir), fminf(d4 - dot3(p2.v, dir), d4 - dot3(p3.v, dir)));
  return mn <= MPR_TOLF;
}
__device__ __forceinline__ void expand_portal(const MprPt& p0, MprPt& p1, MprPt& p2, MprPt& p3, const MprPt& v4) {
  const f3 v4v0 = cross3(v4.v, p0.v);
  if (dot3(p1.v, v4v0) > 0.f) {
    if (dot3(p2.v, v4v0) > 0.f) p1 = v4; else p3 = v4;
  } else {
    if (dot3(p3.v, v4v0) > 0.f) p2 = v4; else p1 = v4;
  }
}
// closest point of triangle (a, b, c) to the origin (Ericson, RTCD 5.1.5), in fp64: MPR's final
// portal is a small triangle (sub-mm edges) ~1 mm from the origin, and the fp32 form's
// cancellations in the region tests and barycentric weights put the closest point on a wrong
// vertex or edge - its direction, the contact normal, off by up to ~0.4 rad (round 6,
// tools/contact_diff.py); the closest point itself is 1-Lipschitz in the vertices, so from the
// fp32 portal points the fp64 form is accurate to their rounding. Once per MPR call.
__device__ __forceinline__ f3 tri_closest_origin_d(f3 af, f3 bf, f3 cf) {
  const double ax = af.x, ay = af.y, az = af.z, bx = bf.x, by = bf.y, bz = bf.z, cx = cf.x, cy = cf.y, cz = cf.z;
  const double abx = bx - ax, aby = by - ay, abz = bz - az, acx = cx - ax, acy = cy - ay, acz = cz - az;
  const double d1 = -(abx * ax + aby * ay + abz * az), d2 = -(acx * ax + acy * ay + acz * az);
  if (d1 <= 0.0 && d2 <= 0.0) return af;
  const double d3 = -(abx * bx + aby * by + abz * bz), d4 = -(acx * bx + acy * by + acz * bz);
  if (d3 >= 0.0 && d4 <= d3) return bf;
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {
    const double t = d1 / (d1 - d3);
    return mk3((float)(ax + abx * t), (float)(ay + aby * t), (float)(az + abz * t));
  }
  const double d5 = -(abx * cx + aby * cy + abz * cz), d6 = -(acx * cx + acy * cy + acz * cz);
  if (d6 >= 0.0 && d5 <= d6) return cf;
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
    const double t = d2 / (d2 - d6);
    return mk3((float)(ax + acx * t), (float)(ay + acy * t), (float)(az + acz * t));
  }
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
    const double t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    return mk3((float)(bx + (cx - bx) * t), (float)(by + (cy - by) * t), (float)(bz + (cz - bz) * t));
  }
  const double den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;
  return mk3((float)(ax + abx * v + acx * w), (float)(ay + aby * v + acy * w), (float)(az + abz * v + acz * w));
}
__device__ __forceinline__ f3 mpr_pos(const MprPt& p0, const MprPt& p1, const MprPt& p2, const MprPt& p3) {
  const f3 dir = portal_dir(p1, p2, p3);
  float b0 = dot3(cross3(p1.v, p2.v), p3.v), b1 = dot3(cross3(p3.v, p2.v), p0.v);
  float b2 = dot3(cross3(p0.v, p1.v), p3.v), b3 = dot3(cross3(p2.v, p1.v), p0.v);
  float sum = b0 + b1 + b2 + b3;
  if (mpr_zero(sum) || sum < 0.f) {
    b0 = 0.f;
    b1 = dot3(cross3(p2.v, p3.v), dir);
    b2 = dot3(cross3(p3.v, p1.v), dir);
    b3 = dot3(cross3(p1.v, p2.v), dir);
    sum = b1 + b2 + b3;
  }
  const float inv = 1.f / sum;
  const f3 pa = p0.a * b0 + p1.a * b1 + p2.a * b2 + p3.a * b3;
  const f3 pb = p0.b * b0 + p1.b * b1 + p2.b * b2 + p3.b * b3;
  return (pa * inv + pb * inv) * 0.5f;
}
// 1: penetrating (depth >= 0, normal A -> B, contact point); 0: apart. PAIR: paired lanes (O,
// role: see mpr_sup_t)
template <bool PAIR = false>
__device__ __forceinline__ int mpr_penetration(const DevModel* __restrict__ m, const XShape& A, const XShape& B,
                                               float* depth, f3* n, f3* pos, int* its = nullptr,
                                               const XShape* O = nullptr, bool role = false) {
  const XShape& own = PAIR ? *O : A;
  MprPt p0, p1, p2, p3;
  p0.a = A.c; p0.b = B.c; p0.v = A.c - B.c;
  if (p0.v.x == 0.f && p0.v.y == 0.f && p0.v.z == 0.f) p0.v.x += 10.f * MPR_EPSF;
  f3 dir = nrmz3(p0.v * -1.f);
  p1 = mpr_sup_t<PAIR>(m, A, B, own, role, dir);
  float dt = dot3(p1.v, dir);
  if (mpr_zero(dt) || dt < 0.f) return 0;
  dir = cross3(p0.v, p1.v);
  if (mpr_zero(dot3(dir, dir))) {
    *pos = (p1.a + p1.b) * 0.5f;
    if (p1.v.x == 0.f && p1.v.y == 0.f && p1.v.z == 0.f) { *depth = 0.f; *n = mk3(0.f, 0.f, 0.f); }
    else { *depth = norm3(p1.v); *n = nrmz3(p1.v); }
    return 1;
  }
  dir = nrmz3(dir);
  p2 = mpr_sup_t<PAIR>(m, A, B, own, role, dir);
  dt = dot3(p2.v, dir);
  if (mpr_zero(dt) || dt < 0.f) return 0;
  dir = nrmz3(cross3(p1.v - p0.v, p2.v - p0.v));
  if (dot3(dir, p0.v) > 0.f) { const MprPt t = p1; p1 = p2; p2 = t; dir = dir * -1.f; }
  for (int it = 0;; it++) {
    if (its) ++*its;  // (timing build: support calls of the refinement)
    if (it > 4 * MPR_MAXITF) return 0;
    p3 = mpr_sup_t<PAIR>(m, A, B, own, role, dir);
    dt = dot3(p3.v, dir);
    if (mpr_zero(dt) || dt < 0.f) return 0;
    bool cont = false;
    float t = dot3(cross3(p1.v, p3.v), p0.v);
    if (t < 0.f && !mpr_zero(t)) { p2 = p3; cont = true; }
    if (!cont) {
      t = dot3(cross3(p3.v, p2.v), p0.v);
      if (t < 0.f && !mpr_zero(t)) { p1 = p3; cont = true; }
    }
    if (!cont) break;
    dir = nrmz3(cross3(p1.v - p0.v, p2.v - p0.v));
  }
  for (int it = 0;; it++) {
    if (its) ++*its;  // (timing build: support calls of the refinement)
    if (it > 4 * MPR_MAXITF) return 0;
    dir = portal_dir(p1, p2, p3);
    dt = dot3(p1.v, dir);
    if (mpr_zero(dt) || dt > 0.f) break;
    const MprPt v4 = mpr_sup_t<PAIR>(m, A, B, own, role, dir);
    const float d4 = dot3(v4.v, dir);
    if (!(mpr_zero(d4) || d4 > 0.f) || portal_reach_tol(p1, p2, p3, v4, dir)) return 0;
    expand_portal(p0, p1, p2, p3, v4);
  }
  for (int it = 0;; it++) {
    if (its) ++*its;  // (timing build: support calls of the refinement)
    dir = portal_dir(p1, p2, p3);
    const MprPt v4 = mpr_sup_t<PAIR>(m, A, B, own, role, dir);
    if (portal_reach_tol(p1, p2, p3, v4, dir) || it > MPR_MAXITF) {
      const f3 cp = tri_closest_origin_d(p1.v, p2.v, p3.v);
      *depth = norm3(cp);
      *n = mpr_zero(*depth) ? dir : cp * (1.f / *depth);
      *pos = mpr_pos(p0, p1, p2, p3);
      return 1;
    }
    expand_portal(p0, p1, p2, p3, v4);
  }
}

// ------------------------------------------------------------------ MPR in fp64 (PS_MPR_F64)
// The same algorithm with the support points and the portal arithmetic in fp64, from the fp32
// colliders (frames, vertices, radii: a rigid rounding of each collider, which the checker's
// state perturbation models) - the support SELECTION stays fp32 (the tie band above is ~7x its
// rounding). Why: in fp32 the final portal, a sub-mm triangle of support points each rounded
// independently by ~1e-9 m, has a normal with ~1e-5 rad of noise, and the termination test (the
// portal within 1e-6 m) then flips on ~0.5% of the calls where no state perturbation does
// (round 6).
struct d3 {
  double x, y, z;
};
__device__ __forceinline__ d3 mkd3(double a, double b, double c) { return {a, b, c}; }
__device__ __forceinline__ d3 tod3(f3 a) { return {a.x, a.y, a.z}; }
__device__ __forceinline__ f3 tof3(d3 a) { return mk3((float)a.x, (float)a.y, (float)a.z); }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ d3 operator*(d3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ double dotd(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ d3 crossd(d3 a, d3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
#ifndef PS_MPR_FASTN
#define PS_MPR_FASTN 1
#endif
// 1 / sqrt(x) for x > 0: the fp32 estimate and one Newton step (relative error ~1e-14, far below
// anything MPR compares; the correctly rounded fp64 sqrt and division are ~20 instructions each).
// PS_MPR_FASTN: the portal normals and the capsule supports normalised with it, +1% on the box /
// hull hand (725K against 718K env-steps/s, tools/gpu_ab.sh, two interleaved repetitions)
__device__ __forceinline__ double rsqrtd(double x) {
  const double r = (double)__frsqrt_rn((float)x);
  return r * (1.5 - 0.5 * x * r * r);
}
__device__ __forceinline__ d3 nrmzd(d3 a) {
  const double n2 = dotd(a, a);
  if (PS_MPR_FASTN && n2 > 1e-30 && n2 < 1e30) return a * rsqrtd(n2);
  const double n = sqrt(n2);
  return n > 0.0 ? a * (1.0 / n) : a;
}
__device__ __forceinline__ bool mpr_zerod(double x) { return fabs(x) < 2.220446049250313e-16; }
// support in fp64: the capsule analytically, a box / hull at its fp32-selected local point
__device__ __forceinline__ d3 x_support_d(const DevModel* __restrict__ m, const XShape& s, d3 d) {
  if (s.type == 0) {
    const d3 p0 = tod3(s.p0), p1 = tod3(s.p1), ax = p1 - p0;
    const double dd = dotd(d, d);
    double da = dotd(ax, d);
    if (PS_MPR_FASTN && dd > 1e-30 && dd < 1e30) {
      // (the tie band in fp32: a tolerance, not a value)
      if (fabsf((float)da) <= SUP_TIE_CAP * norm3(s.p1 - s.p0) * sqrtf((float)dd)) da = 0.0;
      const d3 base = da > 0.0 ? p1 : (da < 0.0 ? p0 : (p0 + p1) * 0.5);
      return base + d * ((double)s.r * rsqrtd(dd));
    }
    const double dn = sqrt(dd);
    if (fabs(da) <= (double)SUP_TIE_CAP * sqrt(dotd(ax, ax)) * dn) da = 0.0;
    const d3 base = da > 0.0 ? p1 : (da < 0.0 ? p0 : (p0 + p1) * 0.5);
    return dn > 0.0 ? base + d * ((double)s.r / dn) : base;
  }
  const f3 l = x_support_local(m, s, tof3(d));
  const double lx = l.x, ly = l.y, lz = l.z;
  return mkd3(s.c.x + (s.R[0] * lx + s.R[1] * ly + s.R[2] * lz), s.c.y + (s.R[3] * lx + s.R[4] * ly + s.R[5] * lz),
              s.c.z + (s.R[6] * lx + s.R[7] * ly + s.R[8] * lz));
}
// (the witnesses as a and v only, b = a - v: 12 registers per portal point instead of 18 -
// measured slower, 705K against 719K env-steps/s; a, b in fp32: 709K against 718K)
struct MprPtD {
  d3 v, a, b;
};
__device__ __forceinline__ double xchg1d(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffffll), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <bool PAIR>
__device__ __forceinline__ MprPtD mpr_sup_d(const DevModel* __restrict__ m, const XShape& A, const XShape& B,
                                            const XShape& O, bool role, d3 d) {
  MprPtD p;
  if (!PAIR) {
    p.a = x_support_d(m, A, d);
    p.b = x_support_d(m, B, d * -1.0);
  } else {
    const d3 mine = x_support_d(m, O, role ? d * -1.0 : d);
    const d3 oth = mkd3(xchg1d(mine.x), xchg1d(mine.y), xchg1d(mine.z));
    p.a = role ? oth : mine;
    p.b = role ? mine : oth;
  }
  p.v = p.a - p.b;
  return p;
}
__device__ __forceinline__ d3 portal_dir_d(const MprPtD& p1, const MprPtD& p2, const MprPtD& p3) {
  return nrmzd(crossd(p2.v - p1.v, p3.v - p1.v));
}
__device__ __forceinline__ bool portal_reach_tol_d(const MprPtD& p1, const MprPtD& p2, const MprPtD& p3,
                                                   const MprPtD& v4, d3 dir) {
  const double d4 = dotd(v4.v, dir);
  return fmin(d4 - dotd(p1.v, dir), fmin(d4 - dotd(p2.v, dir), d4 - dotd(p3.v, dir))) <= 1e-6;  // (the checker's MPR_TOL)
}
__device__ __forceinline__ void expand_portal_d(const MprPtD& p0, MprPtD& p1, MprPtD& p2, MprPtD& p3, const MprPtD& v4) {
  const d3 v4v0 = crossd(v4.v, p0.v);
  if (dotd(p1.v, v4v0) > 0.0) {
    if (dotd(p2.v, v4v0) > 0.0) p1 = v4; else p3 = v4;
  } else {
    if (dotd(p3.v, v4v0) > 0.0) p2 = v4; else p1 = v4;
  }
}
__device__ __forceinline__ d3 tri_closest_origin_dd(d3 a, d3 b, d3 c) {
  const d3 ab = b - a, ac = c - a;
  const double d1 = -dotd(ab, a), d2 = -dotd(ac, a);
  if (d1 <= 0.0 && d2 <= 0.0) return a;
  const double d3_ = -dotd(ab, b), d4 = -dotd(ac, b);
  if (d3_ >= 0.0 && d4 <= d3_) return b;
  const double vc = d1 * d4 - d3_ * d2;
  if (vc <= 0.0 && d1 >= 0.0 && d3_ <= 0.0) return a + ab * (d1 / (d1 - d3_));
  const double d5 = -dotd(ab, c), d6 = -dotd(ac, c);
  if (d6 >= 0.0 && d5 <= d6) return c;
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) return a + ac * (d2 / (d2 - d6));
  const double va = d3_ * d6 - d5 * d4;
  if (va <= 0.0 && (d4 - d3_) >= 0.0 && (d5 - d6) >= 0.0) return b + (c - b) * ((d4 - d3_) / ((d4 - d3_) + (d5 - d6)));
  const double den = 1.0 / (va + vb + vc);
  return a + ab * (vb * den) + ac * (vc * den);
}
__device__ __forceinline__ d3 mpr_pos_d(const MprPtD& p0, const MprPtD& p1, const MprPtD& p2, const MprPtD& p3) {
  const d3 dir = portal_dir_d(p1, p2, p3);
  double b0 = dotd(crossd(p1.v, p2.v), p3.v), b1 = dotd(crossd(p3.v, p2.v), p0.v);
  double b2 = dotd(crossd(p0.v, p1.v), p3.v), b3 = dotd(crossd(p2.v, p1.v), p0.v);
  double sum = b0 + b1 + b2 + b3;
  if (mpr_zerod(sum) || sum < 0.0) {
    b0 = 0.0;
    b1 = dotd(crossd(p2.v, p3.v), dir);
    b2 = dotd(crossd(p3.v, p1.v), dir);
    b3 = dotd(crossd(p1.v, p2.v), dir);
    sum = b1 + b2 + b3;
  }
  const double inv = 1.0 / sum;
  const d3 pa = p0.a * b0 + p1.a * b1 + p2.a * b2 + p3.a * b3;
  const d3 pb = p0.b * b0 + p1.b * b1 + p2.b * b2 + p3.b * b3;
  return (pa * inv + pb * inv) * 0.5;
}
// mpr_penetration in fp64 (same control flow, the checker's mpr_penetration statement for statement)
template <bool PAIR = false>
__device__ __forceinline__ int mpr_penetration_d(const DevModel* __restrict__ m, const XShape& A, const XShape& B,
                                                 float* depth, f3* n, f3* pos, int* its = nullptr,
                                                 const XShape* O = nullptr, bool role = false) {
  const XShape& own = PAIR ? *O : A;
  MprPtD p0, p1, p2, p3;
  p0.a = tod3(A.c); p0.b = tod3(B.c); p0.v = p0.a - p0.b;
  if (p0.v.x == 0.0 && p0.v.y == 0.0 && p0.v.z == 0.0) p0.v.x += 10.0 * 2.220446049250313e-16;
  d3 dir = nrmzd(p0.v * -1.0);
  p1 = mpr_sup_d<PAIR>(m, A, B, own, role, dir);
  double dt = dotd(p1.v, dir);
  if (mpr_zerod(dt) || dt < 0.0) return 0;
  dir = crossd(p0.v, p1.v);
  if (mpr_zerod(dotd(dir, dir))) {
    *pos = tof3((p1.a + p1.b) * 0.5);
    if (p1.v.x == 0.0 && p1.v.y == 0.0 && p1.v.z == 0.0) { *depth = 0.f; *n = mk3(0.f, 0.f, 0.f); }
    else { *depth = (float)sqrt(dotd(p1.v, p1.v)); *n = tof3(nrmzd(p1.v)); }
    return 1;
  }
  dir = nrmzd(dir);
  p2 = mpr_sup_d<PAIR>(m, A, B, own, role, dir);
  dt = dotd(p2.v, dir);
  if (mpr_zerod(dt) || dt < 0.0) return 0;
  dir = nrmzd(crossd(p1.v - p0.v, p2.v - p0.v));
  if (dotd(dir, p0.v) > 0.0) { const MprPtD t = p1; p1 = p2; p2 = t; dir = dir * -1.0; }
  for (int it = 0;; it++) {
    if (its) ++*its;
    if (it > 4 * MPR_MAXITF) return 0;
    p3 = mpr_sup_d<PAIR>(m, A, B, own, role, dir);
    dt = dotd(p3.v, dir);
    if (mpr_zerod(dt) || dt < 0.0) return 0;
    bool cont = false;
    double t = dotd(crossd(p1.v, p3.v), p0.v);
    if (t < 0.0 && !mpr_zerod(t)) { p2 = p3; cont = true; }
    if (!cont) {
      t = dotd(crossd(p3.v, p2.v), p0.v);
      if (t < 0.0 && !mpr_zerod(t)) { p1 = p3; cont = true; }
    }
    if (!cont) break;
    dir = nrmzd(crossd(p1.v - p0.v, p2.v - p0.v));
  }
  for (int it = 0;; it++) {
    if (its) ++*its;
    if (it > 4 * MPR_MAXITF) return 0;
    dir = portal_dir_d(p1, p2, p3);
    dt = dotd(p1.v, dir);
    if (mpr_zerod(dt) || dt > 0.0) break;
    const MprPtD v4 = mpr_sup_d<PAIR>(m, A, B, own, role, dir);
    const double d4 = dotd(v4.v, dir);
    if (!(mpr_zerod(d4) || d4 > 0.0) || portal_reach_tol_d(p1, p2, p3, v4, dir)) return 0;
    expand_portal_d(p0, p1, p2, p3, v4);
  }
  for (int it = 0;; it++) {
    if (its) ++*its;
    dir = portal_dir_d(p1, p2, p3);
    const MprPtD v4 = mpr_sup_d<PAIR>(m, A, B, own, role, dir);
    if (portal_reach_tol_d(p1, p2, p3, v4, dir) || it > MPR_MAXITF) {
      const d3 cp = tri_closest_origin_dd(p1.v, p2.v, p3.v);
      const double dep = sqrt(dotd(cp, cp));
      *depth = (float)dep;
      *n = tof3(mpr_zerod(dep) ? dir : cp * (1.0 / dep));
      *pos = tof3(mpr_pos_d(p0, p1, p2, p3));
      return 1;
    }
    expand_portal_d(p0, p1, p2, p3, v4);
  }
}

// ------------------------------------------------------------------ box-box
// Small fixed arrays indexed by a run-time count: written through unrolled selects so they
// stay in registers.
template <int N>
__device__ __forceinline__ void put3(f3 (&a)[N], int i, f3 v) {
#pragma unroll
  for (int j = 0; j < N; j++)
    if (j == i) a[j] = v;
}
template <int N>
__device__ __forceinline__ f3 get3(const f3 (&a)[N], int i) {
  f3 r = a[0];
#pragma unroll
  for (int j = 1; j < N; j++)
    if (j == i) r = a[j];
  return r;
}
__device__ __forceinline__ f3 rcol(const float* R, int i) { return mk3(R[i], R[3 + i], R[6 + i]); }
__device__ __forceinline__ float f3c(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

constexpr int BB_MAXPT = 4;
// separating axes + reference-face clipping (the CPU checker's box_box, same rules and order)
__device__ __forceinline__ int box_box(const XShape& A, const XShape& B, f3 (&pos)[BB_MAXPT], float (&dist)[BB_MAXPT],
                                       f3* nout) {
  f3 a[3], b[3];
#pragma unroll
  for (int i = 0; i < 3; i++) { a[i] = rcol(A.R, i); b[i] = rcol(B.R, i); }
  const f3 t = B.c - A.c;
  float best = INFINITY;
  int bax = -1;
  f3 bn = mk3(0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < 15; k++) {
    f3 L;
    if (k < 3) L = a[k];
    else if (k < 6) L = b[k - 3];
    else {
      L = cross3(a[(k - 6) / 3], b[(k - 6) % 3]);
      const float ln = norm3(L);
      if (ln < 1e-6f) continue;
      L = L * (1.f / ln);
    }
    float ra = 0.f, rb = 0.f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      ra += f3c(A.hs, i) * fabsf(dot3(a[i], L));
      rb += f3c(B.hs, i) * fabsf(dot3(b[i], L));
    }
    const float s = dot3(t, L);
    const float ov = ra + rb - fabsf(s);
    if (ov < 0.f) return 0;
    if (k < 6 ? ov < best : 1.05f * ov < best) { best = ov; bax = k; bn = s >= 0.f ? L : L * -1.f; }
  }
  if (bax >= 6) {  // edge-edge
    const int i = (bax - 6) / 3, j = (bax - 6) % 3;
    f3 pa = A.c, pb = B.c, ai = a[0], bj = b[0];
    float hai = A.hs.x, hbj = B.hs.x;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k != i) pa = pa + a[k] * ((dot3(a[k], bn) >= 0.f ? 1.f : -1.f) * f3c(A.hs, k));
      else { ai = a[k]; hai = f3c(A.hs, k); }
      if (k != j) pb = pb + b[k] * ((dot3(b[k], bn) >= 0.f ? -1.f : 1.f) * f3c(B.hs, k));
      else { bj = b[k]; hbj = f3c(B.hs, k); }
    }
    f3 c1, c2;
    seg_seg(pa - ai * hai, pa + ai * hai, pb - bj * hbj, pb + bj * hbj, &c1, &c2);
    pos[0] = (c1 + c2) * 0.5f;
    dist[0] = -best;
    *nout = bn;
    return 1;
  }
  const bool refA = bax < 3;
  const int fi = refA ? bax : bax - 3;
  const XShape& Rf = refA ? A : B;
  const XShape& In = refA ? B : A;
  f3 ra[3], ia[3];
#pragma unroll
  for (int k = 0; k < 3; k++) { ra[k] = refA ? a[k] : b[k]; ia[k] = refA ? b[k] : a[k]; }
  const f3 nf = refA ? bn : bn * -1.f;
  int ij = 0;
  float bd = -1.f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float d = fabsf(dot3(ia[k], nf));
    if (d > bd) { bd = d; ij = k; }
  }
  const f3 iaj = ij == 0 ? ia[0] : (ij == 1 ? ia[1] : ia[2]);
  const float sg = dot3(iaj, nf) > 0.f ? -1.f : 1.f;
  const int u = (ij + 1) % 3, w = (ij + 2) % 3;
  const f3 iau = u == 0 ? ia[0] : (u == 1 ? ia[1] : ia[2]);
  const f3 iaw = w == 0 ? ia[0] : (w == 1 ? ia[1] : ia[2]);
  const float hu = f3c(In.hs, u), hw = f3c(In.hs, w);
  const f3 fc = In.c + iaj * (sg * f3c(In.hs, ij));
  f3 poly[8];
  poly[0] = fc + iau * hu + iaw * hw;
  poly[1] = fc - iau * hu + iaw * hw;
  poly[2] = fc - iau * hu - iaw * hw;
  poly[3] = fc + iau * hu - iaw * hw;
#pragma unroll
  for (int k = 4; k < 8; k++) poly[k] = poly[0];
  int np = 4;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int ax = (fi + 1 + e / 2) % 3;
    const f3 rax = ax == 0 ? ra[0] : (ax == 1 ? ra[1] : ra[2]);
    const f3 pn = (e % 2) ? rax * -1.f : rax;
    const float off = dot3(pn, Rf.c) + f3c(Rf.hs, ax);
    f3 tmp[8];
#pragma unroll
    for (int k = 0; k < 8; k++) tmp[k] = poly[0];
    int nq = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (k < np) {
        const f3 p = poly[k], q = k + 1 < 8 ? (k + 1 < np ? poly[(k + 1) & 7] : poly[0]) : poly[0];
        const float dp = dot3(pn, p) - off, dq = dot3(pn, q) - off;
        if (dp <= 0.f) { put3(tmp, nq, p); nq++; }
        if ((dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f)) { put3(tmp, nq, p + (q - p) * (dp / (dp - dq))); nq++; }
      }
    }
    np = nq;
#pragma unroll
    for (int k = 0; k < 8; k++) poly[k] = tmp[k];
    if (np == 0) return 0;
  }
  const float fo = dot3(nf, Rf.c) + f3c(Rf.hs, fi);
  f3 cp[8];
  float cd[8];
  int nc = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) cp[k] = poly[0];
#pragma unroll
  for (int k = 0; k < 8; k++) cd[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k < np) {
      const float d = fo - dot3(nf, poly[k]);
      if (d >= 0.f) {
        put3(cp, nc, poly[k]);
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (j == nc) cd[j] = d;
        nc++;
      }
    }
  }
  // deepest first, then farthest-point sampling (ties: lowest index)
  int ns = 0;
  uint32_t used = 0;
  float md[8];
#pragma unroll
  for (int k = 0; k < 8; k++) md[k] = INFINITY;
  for (int q = 0; q < BB_MAXPT; q++) {
    if (q >= nc) break;
    int bi = -1;
    float bv = -1.f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (k < nc && !((used >> k) & 1u)) {
        const float v = q == 0 ? cd[k] : md[k];
        if (v > bv) { bv = v; bi = k; }
      }
    }
    used |= 1u << bi;
    const f3 pq = get3(cp, bi);
    float dq = cd[0];
#pragma unroll
    for (int k = 1; k < 8; k++)
      if (k == bi) dq = cd[k];
#pragma unroll
    for (int k = 0; k < 8; k++) md[k] = fminf(md[k], norm3(cp[k] - pq));
#pragma unroll
    for (int j = 0; j < BB_MAXPT; j++)
      if (j == q) { pos[j] = pq + nf * (0.5f * dq); dist[j] = -dq; }
    ns++;
  }
  *nout = bn;
  return ns;
}

// capsule vs oriented box (box = geom1, normal box -> capsule; the checker's capsule_box with
// a general box frame): endpoint spheres, else the segment point closest to the box
__device__ __forceinline__ int capsule_obox(const XShape& C, const XShape& Bx, f3 (&pos)[BB_MAXPT], float (&dist)[BB_MAXPT],
                                            f3 (&nrm)[BB_MAXPT]) {
  const float hs[3] = {Bx.hs.x, Bx.hs.y, Bx.hs.z};
  int n = 0;
#pragma unroll
  for (int e = 0; e < 2; e++) {
    f3 nn, pp;
    const float d = sphere_box(e == 0 ? C.p0 : C.p1, C.r, Bx.c, Bx.R, hs, &nn, &pp);
    if (d <= 0.f) {
#pragma unroll
      for (int j = 0; j < 2; j++)
        if (j == n) { pos[j] = pp; dist[j] = d; nrm[j] = nn; }
      n++;
    }
  }
  if (n) return n;
  const f3 la = mtv3(Bx.R, C.p0 - Bx.c), lb = mtv3(Bx.R, C.p1 - Bx.c);
  const float t = seg_box_t(la, lb - la, hs);
  f3 nn, pp;
  const float d = sphere_box(C.p0 + (C.p1 - C.p0) * t, C.r, Bx.c, Bx.R, hs, &nn, &pp);
  if (d <= 0.f) { pos[0] = pp; dist[0] = d; nrm[0] = nn; return 1; }
  return 0;
}

// A pair with a hull whose enclosing capsule stays clear of the other collider (its enclosing
// capsule, capsule or box) by more than 1e-5 m: the hulls are apart, MPR would find nothing.
__device__ __forceinline__ bool x_apart(const XShape& A, const XShape& B) {
  if (A.type != PS_GEOM_HULL && B.type != PS_GEOM_HULL) return false;
  // (every field selected by value, component by component: a reference to "the other"
  // collider would take both colliders' addresses and put them in scratch memory)
  const bool ha = A.type == PS_GEOM_HULL;
  auto sel = [ha](f3 a, f3 b) { return mk3(ha ? a.x : b.x, ha ? a.y : b.y, ha ? a.z : b.z); };
  const f3 h0 = sel(A.e0, B.e0), h1 = sel(A.e1, B.e1);
  const float hr = ha ? A.er : B.er;
  const int otype = ha ? B.type : A.type;
  float d;
  if (otype == PS_GEOM_BOX) {
    const f3 oc = sel(B.c, A.c), ohs = sel(B.hs, A.hs);
    float oR[9];
#pragma unroll
    for (int i = 0; i < 9; i++) oR[i] = ha ? B.R[i] : A.R[i];
    const float hs[3] = {ohs.x, ohs.y, ohs.z};
    const f3 a = mtv3(oR, h0 - oc), b = mtv3(oR, h1 - oc);
    const float t = seg_box_t(a, b - a, hs);
    f3 n, p;
    d = sphere_box(h0 + (h1 - h0) * t, hr, oc, oR, hs, &n, &p);
  } else {
    const bool oh = otype == PS_GEOM_HULL;
    const f3 e0 = sel(B.e0, A.e0), e1 = sel(B.e1, A.e1), p0 = sel(B.p0, A.p0), p1 = sel(B.p1, A.p1);
    const f3 o0 = oh ? e0 : p0, o1 = oh ? e1 : p1;
    const float orad = oh ? (ha ? B.er : A.er) : (ha ? B.r : A.r);
    f3 c1, c2;
    seg_seg(h0, h1, o0, o1, &c1, &c2);
    d = norm3(c2 - c1) - hr - orad;
  }
  return d > 1e-5f;
}

// Narrow phase of collider A (geom1) with collider B: capsule-box (the box becomes geom1:
// swap = true, normal box -> capsule), box-box, or MPR for every pair with a hull. Returns the
// contact count (<= 4); normals point geom1 -> geom2.
template <bool PAIR = false>
__device__ __forceinline__ int x_narrow(const DevModel* __restrict__ m, const XShape& A, const XShape& B,
                                        f3 (&pos)[BB_MAXPT], float (&dist)[BB_MAXPT], f3 (&nrm)[BB_MAXPT], bool& swap,
                                        int* its = nullptr, const XShape* O = nullptr, bool role = false) {
  swap = false;
  if (A.type == 0 && B.type == PS_GEOM_BOX) {
    swap = true;
    return capsule_obox(A, B, pos, dist, nrm);
  }
  if (A.type == PS_GEOM_BOX && B.type == PS_GEOM_BOX) {
    f3 n;
    const int cnt = box_box(A, B, pos, dist, &n);
#pragma unroll
    for (int j = 0; j < BB_MAXPT; j++) nrm[j] = n;
    return cnt;
  }
  float depth;
  f3 n, p;
#ifndef PS_MPR_F64
#define PS_MPR_F64 1
#endif
  const int cnt = PS_MPR_F64 ? mpr_penetration_d<PAIR>(m, A, B, &depth, &n, &p, its, O, role)
                             : mpr_penetration<PAIR>(m, A, B, &depth, &n, &p, its, O, role);
  if (n.x == 0.f && n.y == 0.f && n.z == 0.f) n = mk3(0.f, 0.f, 1.f);
  pos[0] = p;
  nrm[0] = n;
  dist[0] = -depth;
  return cnt;
}

// x_narrow in a frame at geom2's centre (the step kernel's narrow phase): the support points and
// portal arithmetic at the pair's scale (centimetres) instead of world coordinates (~0.5 m: an
// fp32 ulp of 6e-8 m on every support point, against MPR's 1e-6 m tolerance, steers the portal
// differently from the fp64 checker's); the contact points back in world coordinates
// (PAIR: called by both lanes of a pair with the same A, B; role = lane & 1)
template <bool PAIR = false>
__device__ __forceinline__ int x_narrow_local(const DevModel* __restrict__ m, XShape A, XShape B, f3 (&pos)[BB_MAXPT],
                                              float (&dist)[BB_MAXPT], f3 (&nrm)[BB_MAXPT], bool& swap,
                                              int* its = nullptr, bool role = false) {
  const f3 org = B.c;
  x_shift(A, org);
  x_shift(B, org);
  XShape O;
  if (PAIR) O = role ? B : A;
  const int cnt = x_narrow<PAIR>(m, A, B, pos, dist, nrm, swap, its, &O, role);
#pragma unroll
  for (int j = 0; j < BB_MAXPT; j++) pos[j] = pos[j] + org;
  return cnt;
}

}  // namespace ps
