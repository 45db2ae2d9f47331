// Test harness (not part of the product library): runs the kernel's narrow phase (x_narrow of
// csrc/collide_x.h) on packed collider pairs, one pair per thread, for a parity check against
// the CPU checker's ref_narrow (tests/test_gpu_colliders.py). Build: tools/build_xcheck.sh.
#include <hip/hip_runtime.h>

#include "../diffusion-piano_amd/csrc/devmodel.h"
#include "../diffusion-piano_amd/csrc/prims.h"
#include "../diffusion-piano_amd/csrc/collide_x.h"

using namespace ps;

// packed collider (as ref_narrow): type, centre 3, row-major R 9, p0 3, p1 3, r, half sizes 3,
// hull first vertex, vertex count (25 floats)
constexpr int PK = 25;
__device__ XShape unpack(const float* p) {
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
  s.hx = s.hz = nullptr;
  if (s.type == 0) s.c = (s.p0 + s.p1) * 0.5f;
  return s;
}

__global__ void xcheck_kernel(const DevModel* m, const float* a, const float* b, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const XShape A = unpack(a + PK * i), B = unpack(b + PK * i);
  f3 pos[BB_MAXPT], nrm[BB_MAXPT];
  float dist[BB_MAXPT];
  bool swap;
  const int cnt = x_narrow(m, A, B, pos, dist, nrm, swap);
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
// hull vertices [nv][4] (device), pairs a/b [n][25] (device), out [n][29] (device)
int xcheck_run(const float* hull_v, int nv, const float* a, const float* b, float* out, int n) {
  if (nv > NH * PS_HAND_HULLVERT) return -1;
  DevModel* hm = new DevModel();
  DevModel* dm = nullptr;
  if (hipMalloc(&dm, sizeof(DevModel)) != hipSuccess) return -2;
  if (hipMemcpy(dm, hm, sizeof(DevModel), hipMemcpyHostToDevice) != hipSuccess) return -3;
  delete hm;
  if (nv && hipMemcpy(dm->hull_v, hull_v, sizeof(float) * 4 * nv, hipMemcpyDeviceToDevice) != hipSuccess) return -4;
  hipLaunchKernelGGL(xcheck_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, dm, a, b, out, n);
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  hipFree(dm);
  return 0;
}
}
