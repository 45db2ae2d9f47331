// Test harness (not part of the product library): runs the kernel's narrow phase (x_narrow of
// csrc/collide_x.h) on packed collider pairs, one pair per thread, for a parity check against
// the CPU checker's ref_narrow (tests/test_gpu_colliders.py). Build: tools/build_xcheck.sh.
#include <hip/hip_runtime.h>

#include <vector>

#include "../diffusion-piano_amd/csrc/devmodel.h"
#include "../diffusion-piano_amd/csrc/prims.h"
#include "../diffusion-piano_amd/csrc/collide_x.h"

using namespace ps;

// packed collider (as ref_narrow): type, centre 3, row-major R 9, p0 3, p1 3, r, half sizes 3,
// hull first vertex, vertex count (25 floats)
constexpr int PK = 25;
__device__ XShape unpack(const DevModel* m, const float* p, const uint64_t* cells, const float4* table, const int* tok) {
  XShape s;
  s.type = (int)p[0];
  s.c = ld3(p + 1);
  for (int i = 0; i < 9; i++) s.R[i] = p[4 + i];
  s.p0 = ld3(p + 13);
  s.p1 = ld3(p + 16);
  s.r = p[19];
  s.hs = ld3(p + 20);
  s.v0 = (int)p[23];
  s.nv = (int)p[24];
  s.er = 0.f;
  s.cells = cells && s.type == PS_GEOM_HULL ? cells + (size_t)s.v0 * XNCELL : nullptr;
  s.cellv = table && s.type == PS_GEOM_HULL && tok[s.v0] ? table + (size_t)s.v0 * (XNCELL + 1) * XCV : nullptr;
  if (s.type == 0) s.c = (s.p0 + s.p1) * 0.5f;
  s.e0 = s.e1 = s.c;
  float rb = 0.f;  // the hull's max vertex norm (DevModel::x_rb in the step kernel)
  for (int i = 0; s.type == PS_GEOM_HULL && i < s.nv; i++) rb = fmaxf(rb, norm3(ld3(m->hull_v[s.v0 + i])));
  s.tie = SUP_TIE_HULL * rb;
  return s;
}

// paired: the step kernel's paired MPR (x_narrow_local<true>): two threads per pair, lanes 2k
// and 2k + 1 (role = lane & 1), the even one writes; else one thread per pair
template <bool PAIR>
__global__ void xcheck_kernel(const DevModel* m, const uint64_t* cells, const float4* table, const int* tok,
                              const float* a, const float* b, float* out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = PAIR ? t >> 1 : t;
  if (i >= n) return;
  const XShape A = unpack(m, a + PK * i, cells, table, tok), B = unpack(m, b + PK * i, cells, table, tok);
  f3 pos[BB_MAXPT], nrm[BB_MAXPT];
  float dist[BB_MAXPT];
  bool swap;
  const int cnt = x_narrow_local<PAIR>(m, A, B, pos, dist, nrm, swap, nullptr, t & 1);  // the step kernel's
  if (PAIR && (t & 1)) return;
  float* o = out + i * (1 + 7 * BB_MAXPT);
  o[0] = (float)cnt;
  for (int j = 0; j < BB_MAXPT; j++) {
    if (j >= cnt) break;
    st3(o + 1 + 7 * j, pos[j]);
    st3(o + 4 + 7 * j, nrm[j]);
    o[7 + 7 * j] = dist[j];
  }
}

extern "C" {
// host only (CPU tests): the support cells of one hull, vertices [n][3] -> out [XNCELL]
int xcheck_cells(const double* v, int n, uint64_t* out) {
  if (n < 1 || n > PS_HULL_MAXVERT) return -1;
  hull_support_cells(reinterpret_cast<const double(*)[3]>(v), n, out);
  return XNCELL;
}
int xcheck_cell_grid(void) { return XCG; }

// hull vertices [nv][4] (device), pairs a/b [n][25] (device), out [n][29] (device); cells & 1:
// the support search over the hulls' support cells (the step kernel's, DevModel::x_cell, built
// for every hull (v0, nv) the pairs name), else over all vertices; cells & 2: paired MPR (two
// threads per pair, as the step kernel); cells & 4 (with & 1): the support-cell vertex tables
// (DevModel::x_cellv, where no cell overflows them) before the masks
int xcheck_run(const float* hull_v, int nv, const float* a, const float* b, float* out, int n, int cells) {
  const bool paired = cells & 2, tables = cells & 4;
  cells &= 1;
  if (nv > NH * PS_HAND_HULLVERT) return -1;
  DevModel* hm = new DevModel();
  DevModel* dm = nullptr;
  if (hipMalloc(&dm, sizeof(DevModel)) != hipSuccess) return -2;
  if (hipMemcpy(dm, hm, sizeof(DevModel), hipMemcpyHostToDevice) != hipSuccess) return -3;
  delete hm;
  if (nv && hipMemcpy(dm->hull_v, hull_v, sizeof(float) * 4 * nv, hipMemcpyDeviceToDevice) != hipSuccess) return -4;
  uint64_t* dcells = nullptr;
  float4* dtable = nullptr;
  int* dtok = nullptr;
  if (cells && nv) {
    std::vector<float> hv((size_t)4 * nv), ha((size_t)PK * n), hb((size_t)PK * n);
    if (hipMemcpy(hv.data(), hull_v, sizeof(float) * 4 * nv, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(ha.data(), a, sizeof(float) * PK * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hb.data(), b, sizeof(float) * PK * n, hipMemcpyDeviceToHost) != hipSuccess)
      return -6;
    std::vector<uint64_t> hc((size_t)nv * XNCELL, 0ull);
    std::vector<float> ht((size_t)nv * (XNCELL + 1) * XCV * 4, 0.f);
    std::vector<int> hok(nv, 0);
    std::vector<char> done(nv, 0);
    for (const std::vector<float>* src : {&ha, &hb})
      for (int i = 0; i < n; i++) {
        const float* p = src->data() + (size_t)PK * i;
        const int v0 = (int)p[23], cnt = (int)p[24];
        if ((int)p[0] != PS_GEOM_HULL || v0 < 0 || cnt < 1 || cnt > PS_HULL_MAXVERT || v0 + cnt > nv || done[v0]) continue;
        done[v0] = 1;
        std::vector<double> vd((size_t)3 * cnt);
        for (int k = 0; k < cnt; k++)
          for (int c = 0; c < 3; c++) vd[3 * k + c] = hv[4 * (size_t)(v0 + k) + c];
        hull_support_cells(reinterpret_cast<const double(*)[3]>(vd.data()), cnt, hc.data() + (size_t)v0 * XNCELL);
        hok[v0] = hull_cell_table(reinterpret_cast<const double(*)[3]>(vd.data()), hc.data() + (size_t)v0 * XNCELL,
                                  reinterpret_cast<float(*)[XCV][4]>(ht.data() + (size_t)v0 * (XNCELL + 1) * XCV * 4));
      }
    if (hipMalloc(&dcells, sizeof(uint64_t) * hc.size()) != hipSuccess) return -7;
    if (hipMemcpy(dcells, hc.data(), sizeof(uint64_t) * hc.size(), hipMemcpyHostToDevice) != hipSuccess) return -8;
    if (tables) {
      if (hipMalloc(&dtable, sizeof(float) * ht.size()) != hipSuccess || hipMalloc(&dtok, sizeof(int) * nv) != hipSuccess)
        return -9;
      if (hipMemcpy(dtable, ht.data(), sizeof(float) * ht.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(dtok, hok.data(), sizeof(int) * nv, hipMemcpyHostToDevice) != hipSuccess)
        return -10;
    }
  }
  if (paired)
    hipLaunchKernelGGL(xcheck_kernel<true>, dim3((2 * n + 63) / 64), dim3(64), 0, 0, dm, dcells, dtable, dtok, a, b,
                       out, n);
  else
    hipLaunchKernelGGL(xcheck_kernel<false>, dim3((n + 63) / 64), dim3(64), 0, 0, dm, dcells, dtable, dtok, a, b, out,
                       n);
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  hipFree(dm);
  if (dcells) hipFree(dcells);
  if (dtable) hipFree(dtable);
  if (dtok) hipFree(dtok);
  return 0;
}
}
