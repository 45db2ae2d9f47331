// Measurement harness (not part of the product library): the dense LDL' of the coupled-hands
// Newton Hessian block two ways, one wave per matrix, cycles by s_memtime around the factor
// (DESIGN.md section 5 records the numbers):
//   reg   - the kernel's method (csrc/newton.inc): lane r holds row r in registers, each pivot row
//           broadcast through LDS, a rank-1 update of every row per pivot (n serial steps);
//   mfma  - 16-column panels: the panel's pivots as above on 16-wide rows, then the trailing
//           block A22 -= W21 D^-1 W21' as 16x16 tiles on v_mfma_f32_16x16x4_f32, matrix in LDS.
// Both factor A (n x n SPD, n <= 64, row-major) into unit-lower L (strict lower part) and D, and
// write L D L' back (the caller checks it against A). Built by __graft_entry__.build().
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

constexpr int LS = 68;  // LDS row stride (floats)

// L D L' of the factor held as F[r][c] (c < r: L, c == r: D) in LDS, into out [n][n]
__device__ void reconstruct(const float* F, int n, float* out, int lane) {
  for (int r = lane; r < n; r += 64)
    for (int c = 0; c < n; c++) {
      float s = 0.f;
      const int m = r < c ? r : c;
      for (int k = 0; k <= m; k++) {
        const float lr = k == r ? 1.f : F[r * LS + k], lc = k == c ? 1.f : F[c * LS + k];
        s += lr * F[k * LS + k] * lc;
      }
      out[r * n + c] = s;
    }
}

template <int N>
__global__ void __launch_bounds__(64) ldl_reg_kernel(const float* A, float* out, uint64_t* cyc, int reps) {
  __shared__ __attribute__((aligned(16))) float P[64 + 4];
  __shared__ float F[64 * LS];
  const int lane = threadIdx.x;
  const float* a = A + (size_t)blockIdx.x * N * N;
  float H[N];
  uint64_t t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; rep++) {
#pragma unroll
    for (int c = 0; c < N; c++) H[c] = lane < N ? a[lane * N + c] : (c == lane ? 1.f : 0.f);
    wsync();
    t0 = __builtin_amdgcn_s_memtime();
#pragma clang loop unroll(full)
    for (int k = 0; k < N; k++) {
      if (lane == k) {
        float4* P4 = reinterpret_cast<float4*>(P);
#pragma unroll
        for (int q = 0; q < N / 4; q++)
          if (4 * q + 3 >= k) P4[q] = make_float4(H[4 * q], H[4 * q + 1], H[4 * q + 2], H[4 * q + 3]);
      }
      wsync();
      float pv[N];
      const float4* P4 = reinterpret_cast<const float4*>(P);
#pragma unroll
      for (int q = 0; q < N / 4; q++) {
        if (4 * q + 3 >= k) {
          const float4 v = P4[q];
          pv[4 * q] = v.x; pv[4 * q + 1] = v.y; pv[4 * q + 2] = v.z; pv[4 * q + 3] = v.w;
        } else {
          pv[4 * q] = pv[4 * q + 1] = pv[4 * q + 2] = pv[4 * q + 3] = 0.f;
        }
      }
      const float t = lane > k && lane < N ? H[k] * __builtin_amdgcn_rcpf(pv[k]) : 0.f;
#pragma unroll
      for (int c = k + 1; c < N; c++) H[c] = fmaf(-t, pv[c], H[c]);
      if (lane > k) H[k] = t;  // L(lane, k)
      wsync();
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  if (lane < N)
#pragma unroll
    for (int c = 0; c < N; c++) F[lane * LS + c] = H[c];
  wsync();
  reconstruct(F, N, out + (size_t)blockIdx.x * N * N, lane);
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// n padded to NP = 16 * panels (identity past n)
template <int N>
__global__ void __launch_bounds__(64) ldl_mfma_kernel(const float* A, float* out, uint64_t* cyc, int reps) {
  constexpr int NP = (N + 15) / 16 * 16;
  __shared__ __attribute__((aligned(16))) float M[64 * LS];
  __shared__ __attribute__((aligned(16))) float P[16 + 4];
  __shared__ float dinv[64];
  const int lane = threadIdx.x;
  const float* a = A + (size_t)blockIdx.x * N * N;
  uint64_t t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; rep++) {
    for (int r = 0; r < NP; r++)
      if (lane < NP) M[r * LS + lane] = (r < N && lane < N) ? a[r * N + lane] : (r == lane ? 1.f : 0.f);
    wsync();
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int p0 = 0; p0 < NP; p0 += 16) {
      // panel: lane = row r >= p0 holds M[r][p0 .. p0 + 16)
      float h[16];
      const bool rowon = lane >= p0 && lane < NP;
#pragma unroll
      for (int c = 0; c < 16; c++) h[c] = rowon ? M[lane * LS + p0 + c] : 0.f;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if (lane == p0 + k) {
          float4* P4 = reinterpret_cast<float4*>(P);
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (4 * q + 3 >= k) P4[q] = make_float4(h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
          dinv[p0 + k] = __builtin_amdgcn_rcpf(h[k]);
        }
        wsync();
        float pv[16];
        const float4* P4 = reinterpret_cast<const float4*>(P);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (4 * q + 3 >= k) {
            const float4 v = P4[q];
            pv[4 * q] = v.x; pv[4 * q + 1] = v.y; pv[4 * q + 2] = v.z; pv[4 * q + 3] = v.w;
          } else {
            pv[4 * q] = pv[4 * q + 1] = pv[4 * q + 2] = pv[4 * q + 3] = 0.f;
          }
        }
        const float t = rowon && lane > p0 + k ? h[k] * __builtin_amdgcn_rcpf(pv[k]) : 0.f;
#pragma unroll
        for (int c = k + 1; c < 16; c++) h[c] = fmaf(-t, pv[c], h[c]);
        wsync();
      }
      // the panel back: W (un-divided columns) for rows past the panel, the panel's own rows
      if (rowon)
#pragma unroll
        for (int c = 0; c < 16; c++) M[lane * LS + p0 + c] = h[c];
      wsync();
      // trailing block rows/cols [p0 + 16, NP): C_IJ -= sum_k W[I][k] dinv[k] W[J][k], lower tiles
      // (I >= J) and the diagonal tiles' full 16x16 (the upper part of a diagonal tile is unused)
      const int i = lane & 15, q = lane >> 4;
      for (int I = p0 + 16; I < NP; I += 16)
        for (int J = p0 + 16; J <= I; J += 16) {
          f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kb = 0; kb < 16; kb += 4) {
            // A[i][k] = W[I + i][p0 + kb + q] dinv, B[k][j] = W[J + j][p0 + kb + q] (lane: j = i)
            const int k = p0 + kb + q;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(M[(I + i) * LS + k] * dinv[k], M[(J + i) * LS + k], acc, 0, 0, 0);
          }
#pragma unroll
          for (int rr = 0; rr < 4; rr++) M[(I + 4 * q + rr) * LS + J + i] -= acc[rr];
        }
      wsync();
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  // factor as F: L(r, c) = W[r][c] * dinv[c] below the diagonal, D on it
  __shared__ float F[64 * LS];
  for (int r = 0; r < N; r++)
    if (lane < N) F[r * LS + lane] = lane < r ? M[r * LS + lane] * dinv[lane] : lane == r ? M[r * LS + r] : 0.f;
  wsync();
  reconstruct(F, N, out + (size_t)blockIdx.x * N * N, lane);
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int N>
int run(int method, const float* A, float* out, uint64_t* cyc, int nmat, int reps) {
  if (method == 0)
    hipLaunchKernelGGL(ldl_reg_kernel<N>, dim3(nmat), dim3(64), 0, 0, A, out, cyc, reps);
  else
    hipLaunchKernelGGL(ldl_mfma_kernel<N>, dim3(nmat), dim3(64), 0, 0, A, out, cyc, reps);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
}  // namespace

extern "C" {
// A [nmat][n][n] (device), out [nmat][n][n] (device: L D L'), cyc [nmat] (device: cycles of the
// last repetition's factor); method 0 reg, 1 mfma; n in {16, 28, 40, 52}
int ldl_bench_run(int method, int n, const float* A, float* out, uint64_t* cyc, int nmat, int reps) {
  switch (n) {
    case 16: return run<16>(method, A, out, cyc, nmat, reps);
    case 28: return run<28>(method, A, out, cyc, nmat, reps);
    case 40: return run<40>(method, A, out, cyc, nmat, reps);
    case 52: return run<52>(method, A, out, cyc, nmat, reps);
    default: return -1;
  }
}
}
