// pianorl.hip - MI355X (gfx950) kernels of the on-device PPO loop + the C-ABI of
// include/pianorl.h. The reference computes these on the host (numpy RunningMeanStd,
// a Python GAE loop, torch.distributions sampling behind a host round trip,
// ppo_v2.py:107-131, 211-256); here they run on the rollout tensors where they live.
//
// All of them are HBM/latency-bound reductions and scans over a few MB at most; none is
// GEMM-shaped, so there is no MFMA here: the layout rules are coalesced column access
// (time-major [T, E] arrays, one thread per env column) and single-pass fp64 reductions.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <string>

#include "../../include/pianorl.h"

namespace {

thread_local std::string g_err;
int fail(const std::string& s) {
  g_err = s;
  return -1;
}
#define HIPCHK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int RED_THREADS = 1024;

// ---------------------------------------------------------------- block reductions (fp64)
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;  // valid in lane 0
}

// sum over the block; every thread gets the result
__device__ double block_sum_d(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum_d(v);
  __syncthreads();  // red[] reuse across calls
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; i++) s += red[i];  // fixed order: deterministic
  return s;
}

// mean and sum of squared deviations (two passes over x, fp64 accumulation)
__device__ void mean_m2(const float* __restrict__ x, int n, double* red, double* mean, double* m2) {
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += (double)x[i];
  const double mu = block_sum_d(s, red) / (double)n;
  double q = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double d = (double)x[i] - mu;
    q += d * d;
  }
  *mean = mu;
  *m2 = block_sum_d(q, red);
}

// RunningMeanStd.__call__ (ppo_v2.py:113-131): batch statistics (np.mean / np.var, ddof 0),
// merge into the running statistics, normalise with the merged ones.
__global__ void __launch_bounds__(RED_THREADS) running_norm_kernel(const float* __restrict__ x, int n,
                                                                   double* __restrict__ stats, float* __restrict__ out) {
  __shared__ double red[RED_THREADS / 64];
  __shared__ double nm[2];
  double bm, bm2;
  mean_m2(x, n, red, &bm, &bm2);
  if (threadIdx.x == 0) {
    const double mean = stats[0], var = stats[1], count = stats[2];
    const double bvar = bm2 / (double)n, bc = (double)n;
    const double delta = bm - mean, tot = count + bc;
    const double new_mean = mean + delta * bc / tot;
    const double M2 = var * count + bvar * bc + delta * delta * count * bc / tot;
    const double new_var = M2 / tot;
    stats[0] = new_mean;
    stats[1] = new_var;
    stats[2] = tot;
    nm[0] = new_mean;
    nm[1] = 1.0 / sqrt(new_var + 1e-8);
  }
  __syncthreads();
  const double mu = nm[0], is = nm[1];
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = (float)(((double)x[i] - mu) * is);
}

// advantages = (a - mean) / (std + eps), torch.std's unbiased estimator (ppo_v2.py:256)
__global__ void __launch_bounds__(RED_THREADS) normalize_kernel(float* __restrict__ x, int n, float eps) {
  __shared__ double red[RED_THREADS / 64];
  double mu, m2;
  mean_m2(x, n, red, &mu, &m2);
  const double sd = n > 1 ? sqrt(m2 / (double)(n - 1)) : NAN;  // torch: nan for one sample
  const float muf = (float)mu, den = (float)(sd + (double)eps);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) x[i] = (x[i] - muf) / den;
}

// ---------------------------------------------------------------- GAE (ppo_v2.py:234-253)
struct GaeIn {
  const float *r, *v, *nv, *d;
  float *adv, *ret;
  int T, E;
  float gamma, gl;
  int mode;
};

__device__ __forceinline__ float next_value(const GaeIn& g, int t, int e) {
  return t == g.T - 1 ? g.nv[(size_t)t * g.E + e] : g.v[(size_t)(t + 1) * g.E + e];
}

__device__ __forceinline__ void gae_emit(const GaeIn& g, int t, int e, float gae) {
  const size_t i = (size_t)t * g.E + e;
  g.adv[i] = gae;
  g.ret[i] = g.mode == PRL_RETURNS_TD ? g.r[i] + g.gamma * (g.nv[i] * (1.f - g.d[i])) : gae + g.v[i];
}

// many columns: one thread per env column, serial over time; row t of a warp is one
// coalesced 256-B read per array
__global__ void __launch_bounds__(256) gae_columns_kernel(GaeIn g) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= g.E) return;
  float gae = 0.f;
  for (int t = g.T - 1; t >= 0; t--) {
    const size_t i = (size_t)t * g.E + e;
    const float nd = 1.f - g.d[i];
    const float delta = g.r[i] + g.gamma * next_value(g, t, e) * nd - g.v[i];
    gae = delta + g.gl * nd * gae;
    gae_emit(g, t, e, gae);
  }
}

// few columns, long time axis (the reference's E = 1, T = batch): one block per column, the
// linear recurrence gae_t = delta_t + c_t gae_{t+1} as a chunked scan of affine maps.
constexpr int SCAN_THREADS = 256;
__global__ void __launch_bounds__(SCAN_THREADS) gae_scan_kernel(GaeIn g) {
  __shared__ float sA[SCAN_THREADS], sB[SCAN_THREADS];
  const int e = blockIdx.x, j = threadIdx.x;
  const int chunk = (g.T + SCAN_THREADS - 1) / SCAN_THREADS;
  const int t0 = min(j * chunk, g.T), t1 = min(t0 + chunk, g.T);
  // this chunk as a map g_in (gae at t1) -> gae at t0: A g_in + B
  float A = 1.f, B = 0.f;
  for (int t = t1 - 1; t >= t0; t--) {
    const size_t i = (size_t)t * g.E + e;
    const float nd = 1.f - g.d[i];
    const float delta = g.r[i] + g.gamma * next_value(g, t, e) * nd - g.v[i];
    const float c = g.gl * nd;
    B = delta + c * B;
    A = c * A;
  }
  sA[j] = A;
  sB[j] = B;
  __syncthreads();
  // suffix composition: (A_j, B_j) <- map_j o map_{j+off}
  for (int off = 1; off < SCAN_THREADS; off <<= 1) {
    float a2 = 1.f, b2 = 0.f;
    const bool has = j + off < SCAN_THREADS;
    if (has) { a2 = sA[j + off]; b2 = sB[j + off]; }
    __syncthreads();
    if (has) {
      const float a1 = sA[j], b1 = sB[j];
      sA[j] = a1 * a2;
      sB[j] = a1 * b2 + b1;
    }
    __syncthreads();
  }
  float gae = j + 1 < SCAN_THREADS ? sB[j + 1] : 0.f;  // gae at t1 (0 past the end)
  for (int t = t1 - 1; t >= t0; t--) {
    const size_t i = (size_t)t * g.E + e;
    const float nd = 1.f - g.d[i];
    const float delta = g.r[i] + g.gamma * next_value(g, t, e) * nd - g.v[i];
    gae = delta + g.gl * nd * gae;
    gae_emit(g, t, e, gae);
  }
}

// ---------------------------------------------------------------- Gaussian policy sampling
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
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

// one row per wave, lane = action dimension (a <= 64)
__global__ void __launch_bounds__(256) gauss_sample_kernel(const float* __restrict__ mean, const float* __restrict__ log_std,
                                                           int n, int a, uint64_t seed, uint64_t offset,
                                                           float* __restrict__ action, float* __restrict__ logp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= n) return;  // whole waves exit together
  float lp = 0.f;
  if (lane < a) {
    uint32_t c[4] = {(uint32_t)lane, (uint32_t)row, (uint32_t)offset, (uint32_t)(offset >> 32)};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)c[0] + 1.f) * 2.3283064e-10f;  // (0, 1]
    const float u2 = (float)c[1] * 2.3283064e-10f;
    const float z = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    const float ls = fminf(fmaxf(log_std[lane], -20.f), 2.f);
    const float sd = expf(ls), mu = mean[(size_t)row * a + lane];
    const float x = mu + sd * z;
    action[(size_t)row * a + lane] = x;
    // torch.distributions.Normal.log_prob: -((x - mu)^2) / (2 var) - log(scale) - log(sqrt(2 pi))
    const float dx = x - mu;
    lp = -(dx * dx) / (2.f * sd * sd) - logf(sd) - 0.91893853f;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lp += __shfl_down(lp, off, 64);
  if (lane == 0) logp[row] = lp;
}

// ---------------------------------------------------------------- clip_grad_norm_ + Adam
// Flat fp32 buffers of every parameter (p, g, m, v), split into <= PRL_MAX_SEG contiguous
// segments (one per network: the reference clips and steps actor and critic separately,
// ppo_v2.py:280-293). Two launches replace torch's ~150 per minibatch (per-tensor norms,
// foreach lerp/mul/addcmul/sqrt/div and the capturable bias corrections).
constexpr int ADAM_PARTS = 256;  // partial-sum blocks of the norm pass
constexpr int ADAM_THREADS = 256;

struct Segs {
  int64_t end[PRL_MAX_SEG];
  int n;
};

__device__ __forceinline__ int64_t seg_begin(const Segs& sg, int s) { return s == 0 ? 0 : sg.end[s - 1]; }

// pass 1: per-segment partial sums of g^2 (fp64), one row of partials per block; block 0
// also advances the per-segment step counters (torch's state["step"] += 1)
__global__ void __launch_bounds__(ADAM_THREADS) grad_sumsq_kernel(const float* __restrict__ g, Segs sg,
                                                                  double* __restrict__ part, float* __restrict__ step,
                                                                  const unsigned* __restrict__ guard) {
  __shared__ double red[ADAM_THREADS / 64];
  if (guard && *guard) return;  // a failed minibatch step upstream: apply nothing (block-uniform)
  for (int s = 0; s < sg.n; s++) {
    double acc = 0.0;
#pragma unroll 8
    for (int64_t i = seg_begin(sg, s) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.end[s];
         i += (int64_t)gridDim.x * blockDim.x) {
      const double x = (double)g[i];
      acc += x * x;
    }
    const double tot = block_sum_d(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x * PRL_MAX_SEG + s] = tot;
  }
  if (blockIdx.x == 0 && threadIdx.x < sg.n) step[threadIdx.x] += 1.f;
}

// pass 2: every block folds the partials into the clip coefficient of each segment
// (torch.nn.utils.clip_grad_norm_: coef = min(1, max_norm / (||g|| + 1e-6))), then the Adam
// update (torch.optim.Adam, amsgrad/weight_decay off) over a grid-stride range
#ifndef ADAM_PER_N
#define ADAM_PER_N 4
#endif
constexpr int ADAM_PER = ADAM_PER_N;  // elements per thread and pass (their loads issued before the norm fold)
__global__ void __launch_bounds__(ADAM_THREADS) clip_adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                                 float* __restrict__ m, float* __restrict__ v, Segs sg,
                                                                 const double* __restrict__ part,
                                                                 const float* __restrict__ lr,
                                                                 const float* __restrict__ step, float b1, float b2,
                                                                 float eps, float max_norm, int nparts,
                                                                 const unsigned* __restrict__ guard) {
  __shared__ float coef[PRL_MAX_SEG], ssz[PRL_MAX_SEG], ibc2[PRL_MAX_SEG];
  if (guard && *guard) return;  // a failed minibatch step upstream: apply nothing (block-uniform)
  const int64_t n = sg.end[sg.n - 1];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the first pass's operands in flight while the block folds the norm partials
  float gq[ADAM_PER], mq[ADAM_PER], vq[ADAM_PER], pq[ADAM_PER];
#pragma unroll
  for (int u = 0; u < ADAM_PER; u++) {
    const int64_t i = i0 + u * stride;
    const bool ok = i < n;
    gq[u] = ok ? g[i] : 0.f;
    mq[u] = ok ? m[i] : 0.f;
    vq[u] = ok ? v[i] : 0.f;
    pq[u] = ok ? p[i] : 0.f;
  }
  // every segment's partials in one pass over the rows (each row's PRL_MAX_SEG doubles are one
  // 32-byte read), then one block reduction of the PRL_MAX_SEG sums - per segment the same
  // association order as a per-segment fold (thread stride, wave butterfly, waves in order)
  static_assert(PRL_MAX_SEG == 4, "one double2 pair per partial row");
  double acc[PRL_MAX_SEG] = {0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nparts; b += blockDim.x) {
    const double2 lo = reinterpret_cast<const double2*>(part + (size_t)b * PRL_MAX_SEG)[0];
    const double2 hi = reinterpret_cast<const double2*>(part + (size_t)b * PRL_MAX_SEG)[1];
    acc[0] += lo.x; acc[1] += lo.y; acc[2] += hi.x; acc[3] += hi.y;
  }
  __shared__ double red4[ADAM_THREADS / 64][PRL_MAX_SEG];
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int s = 0; s < PRL_MAX_SEG; s++) {
      const double v = wave_sum_d(acc[s]);
      if (lane == 0) red4[w][s] = v;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < sg.n) {  // thread s: segment s's clip coefficient and Adam step size
    const int s = threadIdx.x;
    double tot = 0.0;
    for (int w = 0; w < ADAM_THREADS / 64; w++) tot += red4[w][s];  // waves in order
    const float norm = (float)sqrt(tot);
    coef[s] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    const double t = (double)step[s];
    const double bc1 = 1.0 - pow((double)b1, t), bc2 = 1.0 - pow((double)b2, t);
    ssz[s] = (float)((double)lr[s] / bc1);
    ibc2[s] = (float)(1.0 / sqrt(bc2));
  }
  __syncthreads();
  auto upd = [&](int64_t i, float gv, float mv, float vv, float pv) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < PRL_MAX_SEG - 1; k++) s += (k + 1 < sg.n && i >= sg.end[k]) ? 1 : 0;
    const float gi = gv * coef[s];
    const float mi = mv + (1.f - b1) * (gi - mv);  // exp_avg.lerp_(grad, 1 - beta1)
    const float vi = b2 * vv + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pv - ssz[s] * mi / (sqrtf(vi) * ibc2[s] + eps);
  };
#pragma unroll
  for (int u = 0; u < ADAM_PER; u++)
    if (i0 + u * stride < n) upd(i0 + u * stride, gq[u], mq[u], vq[u], pq[u]);
  for (int64_t i = i0 + ADAM_PER * stride; i < n; i += stride) upd(i, g[i], m[i], v[i], p[i]);
}


// ---------------------------------------------------------------- fused minibatch step
// The PPO minibatch step of ppo_v2.py:266-293 with the backward pass written out: the GEMMs
// stay library GEMMs (hipBLASLt, issued by ppo.py), everything between them is one kernel
// per layer and direction instead of torch's ~8 elementwise / reduction launches.

// dropout keep decision: Philox4x32-10 keyed by (seed, step counter), counter (col, row, layer)
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t step, int layer, int row, int col, float p) {
  uint32_t c[4] = {(uint32_t)col, (uint32_t)row, (uint32_t)step ^ ((uint32_t)layer << 24), (uint32_t)(step >> 32)};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (float)c[0] * 2.3283064e-10f >= p;
}

// block sum over the row's H <= 1024 threads (fp32), result broadcast
__device__ __forceinline__ float row_sum(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; i++) s += red[i];
  return s;
}

// gather the minibatch rows (DataLoader batch, ppo_v2.py:266-271); thread 0 of block 0 also
// advances the dropout step counter of this minibatch
__global__ void gather_kernel(const float* __restrict__ S, int sdim, const float* __restrict__ A, int adim,
                              const float* __restrict__ lp, const float* __restrict__ adv, const float* __restrict__ ret,
                              const int64_t* __restrict__ idx, int B, float* __restrict__ oS, float* __restrict__ oA,
                              float* __restrict__ olp, float* __restrict__ oadv, float* __restrict__ oret,
                              uint64_t* __restrict__ step) {
  const int r = blockIdx.x;
  if (r == 0 && threadIdx.x == 0 && step) *step += 1;
  if (r >= B) return;
  const int64_t src = idx[r];
  for (int i = threadIdx.x; i < sdim; i += blockDim.x) oS[(size_t)r * sdim + i] = S[(size_t)src * sdim + i];
  for (int i = threadIdx.x; i < adim; i += blockDim.x) oA[(size_t)r * adim + i] = A[(size_t)src * adim + i];
  if (threadIdx.x == 0) {
    olp[r] = lp[src];
    oadv[r] = adv[src];
    oret[r] = ret[src];
  }
}

// y = dropout(LayerNorm(relu(z + b))) of one row per block (nn.ReLU, nn.LayerNorm eps,
// biased variance; nn.Dropout(p) in train mode); keeps xhat and 1/std for the backward
__global__ void lnrelu_fwd_kernel(const float* __restrict__ Z, const float* __restrict__ bias,
                                  const float* __restrict__ gamma, const float* __restrict__ beta, int H, float eps,
                                  float p, uint64_t seed, const uint64_t* __restrict__ step, int layer,
                                  float* __restrict__ Y, float* __restrict__ xhat, float* __restrict__ rstd) {
  __shared__ float red[16];
  const int r = blockIdx.x, c = threadIdx.x;
  const float x = c < H ? fmaxf(Z[(size_t)r * H + c] + bias[c], 0.f) : 0.f;
  const float mean = row_sum(x, red) / (float)H;
  const float d = c < H ? x - mean : 0.f;
  const float var = row_sum(d * d, red) / (float)H;
  const float rs = 1.f / sqrtf(var + eps);
  if (c < H) {
    const float xh = d * rs;
    float y = xh * gamma[c] + beta[c];
    if (p > 0.f) y = keep_elem(seed, *step, layer, r, c, p) ? y / (1.f - p) : 0.f;
    Y[(size_t)r * H + c] = y;
    xhat[(size_t)r * H + c] = xh;
  }
  if (c == 0) rstd[r] = rs;
}

// backward of lnrelu_fwd for one row per block: dZ, and the per-row terms whose column sums
// are the gamma / beta gradients (dye = the gradient reaching the LayerNorm output)
__global__ void lnrelu_bwd_kernel(const float* __restrict__ dY, const float* __restrict__ Z,
                                  const float* __restrict__ bias, const float* __restrict__ xhat,
                                  const float* __restrict__ rstd, const float* __restrict__ gamma, int H, float p,
                                  uint64_t seed, const uint64_t* __restrict__ step, int layer, float* __restrict__ dZ,
                                  float* __restrict__ dyx, float* __restrict__ dye) {
  __shared__ float red[16];
  const int r = blockIdx.x, c = threadIdx.x;
  float g = 0.f, xh = 0.f;
  if (c < H) {
    g = dY[(size_t)r * H + c];
    if (p > 0.f) g = keep_elem(seed, *step, layer, r, c, p) ? g / (1.f - p) : 0.f;
    xh = xhat[(size_t)r * H + c];
  }
  const float dxh = g * (c < H ? gamma[c] : 0.f);
  const float m1 = row_sum(dxh, red) / (float)H;
  const float m2 = row_sum(dxh * xh, red) / (float)H;
  if (c < H) {
    const float dr = rstd[r] * (dxh - m1 - xh * m2);
    dZ[(size_t)r * H + c] = Z[(size_t)r * H + c] + bias[c] > 0.f ? dr : 0.f;
    dyx[(size_t)r * H + c] = g * xh;
    dye[(size_t)r * H + c] = g;
  }
}

// actor head + clipped surrogate (ppo_v2.py:70-74, 272-279), one wave per row (A <= 64):
// mu = tanh(z + b), log-prob of the batch action, ratio, the loss row and its gradients
// dZ (d loss / d z) and the per-row log_std gradient; torch.minimum splits the gradient
// evenly on a tie and clamp passes it at the bounds (derivatives.yaml)
__global__ void actor_head_kernel(const float* __restrict__ Z, const float* __restrict__ bias,
                                  const float* __restrict__ log_std, const float* __restrict__ act,
                                  const float* __restrict__ old_lp, const float* __restrict__ adv, int B, int A,
                                  float clip, float ent_coef, float* __restrict__ dZ, float* __restrict__ dls,
                                  float* __restrict__ stats, float* __restrict__ ent_rows) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= B) return;
  float mu = 0.f, sd = 1.f, ls = 0.f, a = 0.f, lp = 0.f;
  bool inr = false;
  if (lane < A) {
    mu = tanhf(Z[(size_t)r * A + lane] + bias[lane]);
    const float l = log_std[lane];
    inr = l >= -20.f && l <= 2.f;
    ls = fminf(fmaxf(l, -20.f), 2.f);
    sd = expf(ls);
    a = act[(size_t)r * A + lane];
    const float dx = a - mu;
    lp = -(dx * dx) / (2.f * sd * sd) - ls - 0.91893853f;
  }
  // Normal entropy mean over the action dims (dist.entropy().mean(): the same for every row)
  float ent = lane < A ? 0.5f + 0.91893853f + ls : 0.f;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lp += __shfl_xor(lp, off, 64);
    ent += __shfl_xor(ent, off, 64);
  }
  ent /= (float)A;
  const float ratio = expf(lp - old_lp[r]);
  const float A_ = adv[r];
  const float rc = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip);
  const float s1 = ratio * A_, s2 = rc * A_;
  const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
  const float w2 = 1.f - w1;
  const float inclip = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
  // loss = -mean(min(s1, s2)) - ent_coef * entropy: d loss / d ratio for this row
  const float g = -(w1 * A_ + w2 * A_ * inclip) / (float)B;
  const float gl = g * ratio;  // d loss / d log-prob
  if (lane < A) {
    const float dx = a - mu, iv = 1.f / (sd * sd);
    dZ[(size_t)r * A + lane] = gl * dx * iv * (1.f - mu * mu);
    // log-prob term (a - mu)^2 / sd^2 - 1, and the entropy bonus -ent_coef / A spread over rows
    dls[(size_t)r * A + lane] = inr ? gl * (dx * dx * iv - 1.f) - ent_coef / ((float)A * (float)B) : 0.f;
  }
  if (lane == 0) {
    stats[r] = -fminf(s1, s2) - ent_coef * ent;  // row of the actor loss (its mean is the loss)
    ent_rows[r] = ent;
  }
}

// critic head + MSE (ppo_v2.py:283-284): v = z + c, loss row (v - ret)^2, d loss / d z
__global__ void critic_head_kernel(const float* __restrict__ Z, const float* __restrict__ bias,
                                   const float* __restrict__ ret, int B, float* __restrict__ dZ, float* __restrict__ v_out,
                                   float* __restrict__ sq) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  const float v = Z[r] + bias[0];
  const float e = v - ret[r];
  dZ[r] = 2.f * e / (float)B;
  v_out[r] = v;
  sq[r] = e * e;
}

// column sums of several [B, C_i] arrays in one launch (deterministic: one thread per column
// walks the rows in order); out_i[c] = scale_i * sum_r X_i[r][c]
struct ColSums {
  const float* src[PRL_MAX_COLSUMS];
  float* dst[PRL_MAX_COLSUMS];
  int cols[PRL_MAX_COLSUMS];
  int off[PRL_MAX_COLSUMS];  // column offset of entry i in the partials row
  float scale[PRL_MAX_COLSUMS];
  int n, B, chunk, total;
  float* part;  // [nchunks][total] partial sums (nullptr: one pass, straight to dst)
};
constexpr int COLSUM_CHUNK = 128;  // rows per partial sum
// grid (column blocks, entry, row chunk): a thread sums its column over one chunk of rows in
// order; with one chunk the result goes straight to dst, else to the partials row
__global__ void colsums_kernel(ColSums cs) {
  const int i = blockIdx.y;
  if (i >= cs.n) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int C = cs.cols[i];
  if (c >= C) return;
  const float* x = cs.src[i];
  const int r0 = blockIdx.z * cs.chunk, r1 = min(r0 + cs.chunk, cs.B);
  float acc = 0.f;
  for (int r = r0; r < r1; r++) acc += x[(size_t)r * C + c];
  if (cs.part) cs.part[(size_t)blockIdx.z * cs.total + cs.off[i] + c] = acc;
  else cs.dst[i][c] = acc * cs.scale[i];
}
// the partials of each column summed in chunk order (deterministic)
__global__ void colsums_final_kernel(ColSums cs, int nchunks) {
  const int i = blockIdx.y;
  if (i >= cs.n) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cs.cols[i]) return;
  float acc = 0.f;
  for (int k = 0; k < nchunks; k++) acc += cs.part[(size_t)k * cs.total + cs.off[i] + c];
  cs.dst[i][c] = acc * cs.scale[i];
}

#include "mlp_step.inc"
#include "mlp_split.inc"

}  // namespace

// ---------------------------------------------------------------- C-ABI
extern "C" {

const char* prl_last_error(void) { return g_err.c_str(); }
int prl_version(void) { return 2; }  // 2: the guard word of prl_mlp_step* / prl_clip_adam*

int prl_running_norm(const float* x, int n, double* stats, float* out, void* stream) {
  if (!x || !stats || !out || n <= 0) return fail("prl_running_norm: null pointer or n <= 0");
  running_norm_kernel<<<1, RED_THREADS, 0, (hipStream_t)stream>>>(x, n, stats, out);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_gae(const float* rewards, const float* values, const float* next_values, const float* dones, float* adv,
            float* ret, int T, int E, float gamma, float lam, int returns_mode, void* stream) {
  if (!rewards || !values || !next_values || !dones || !adv || !ret) return fail("prl_gae: null pointer");
  if (T <= 0 || E <= 0) return fail("prl_gae: T and E must be positive");
  if (returns_mode != PRL_RETURNS_TD && returns_mode != PRL_RETURNS_GAE) return fail("prl_gae: bad returns_mode");
  GaeIn g{rewards, values, next_values, dones, adv, ret, T, E, gamma, gamma * lam, returns_mode};
  if (E >= 256 || T <= 64)
    gae_columns_kernel<<<(E + 255) / 256, 256, 0, (hipStream_t)stream>>>(g);
  else
    gae_scan_kernel<<<E, SCAN_THREADS, 0, (hipStream_t)stream>>>(g);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_normalize(float* x, int n, float eps, void* stream) {
  if (!x || n <= 0) return fail("prl_normalize: null pointer or n <= 0");
  normalize_kernel<<<1, RED_THREADS, 0, (hipStream_t)stream>>>(x, n, eps);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_gauss_sample(const float* mean, const float* log_std, int n, int a, uint64_t seed, uint64_t offset,
                     float* action, float* logp, void* stream) {
  if (!mean || !log_std || !action || !logp) return fail("prl_gauss_sample: null pointer");
  if (n <= 0 || a <= 0 || a > 64) return fail("prl_gauss_sample: need n > 0 and 0 < a <= 64");
  gauss_sample_kernel<<<(n + 3) / 4, 256, 0, (hipStream_t)stream>>>(mean, log_std, n, a, seed, offset, action, logp);
  HIPCHK(hipGetLastError());
  return 0;
}

}  // extern "C"
namespace {
int clip_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_end, int nseg,
              const float* lr, float* step, float beta1, float beta2, float eps, float max_norm, double* scratch,
              const double* pre_parts, int npre, const unsigned* guard, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !seg_end || !lr || !step || (!scratch && !pre_parts))
    return fail("prl_clip_adam: null pointer");
  if (nseg < 1 || nseg > PRL_MAX_SEG) return fail("prl_clip_adam: need 1 <= nseg <= PRL_MAX_SEG");
  Segs sg{};
  sg.n = nseg;
  for (int s = 0; s < nseg; s++) {
    sg.end[s] = seg_end[s];
    if (sg.end[s] < (s ? sg.end[s - 1] : 0) || sg.end[s] <= 0) return fail("prl_clip_adam: segment ends must increase");
  }
  for (int s = nseg; s < PRL_MAX_SEG; s++) sg.end[s] = sg.end[nseg - 1];
  const int64_t n = sg.end[nseg - 1];
  const int parts = (int)std::min<int64_t>(ADAM_PARTS, (n + ADAM_THREADS - 1) / ADAM_THREADS);
  if (pre_parts) {  // the norm partials (and the step advance) came from prl_mlp_step_norm
    const int blocks = (int)std::min<int64_t>(2048, (n + ADAM_THREADS * ADAM_PER - 1) / (ADAM_THREADS * ADAM_PER));
    clip_adam_kernel<<<blocks, ADAM_THREADS, 0, (hipStream_t)stream>>>(param, grad, exp_avg, exp_avg_sq, sg, pre_parts,
                                                                      lr, step, beta1, beta2, eps, max_norm, npre, guard);
    HIPCHK(hipGetLastError());
    return 0;
  }
  grad_sumsq_kernel<<<parts, ADAM_THREADS, 0, (hipStream_t)stream>>>(grad, sg, scratch, step, guard);
  HIPCHK(hipGetLastError());
  const int blocks = (int)std::min<int64_t>(2048, (n + ADAM_THREADS * ADAM_PER - 1) / (ADAM_THREADS * ADAM_PER));
  clip_adam_kernel<<<blocks, ADAM_THREADS, 0, (hipStream_t)stream>>>(param, grad, exp_avg, exp_avg_sq, sg, scratch, lr,
                                                                    step, beta1, beta2, eps, max_norm, parts, guard);
  HIPCHK(hipGetLastError());
  return 0;
}

}  // namespace
extern "C" {
int prl_clip_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_end,
                  int nseg, const float* lr, float* step, float beta1, float beta2, float eps, float max_norm,
                  double* scratch, const unsigned* guard, void* stream) {
  return clip_adam(param, grad, exp_avg, exp_avg_sq, seg_end, nseg, lr, step, beta1, beta2, eps, max_norm, scratch,
                   nullptr, 0, guard, stream);
}

int prl_clip_adam_parts(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_end,
                        int nseg, const float* lr, const float* step, float beta1, float beta2, float eps,
                        float max_norm, const double* parts, int nparts, const unsigned* guard, void* stream) {
  if (!parts || nparts <= 0) return fail("prl_clip_adam_parts: no partials");
  return clip_adam(param, grad, exp_avg, exp_avg_sq, seg_end, nseg, lr, const_cast<float*>(step), beta1, beta2, eps,
                   max_norm, nullptr, parts, nparts, guard, stream);
}

int prl_gather_minibatch(const float* S, int sdim, const float* A, int adim, const float* lp, const float* adv,
                         const float* ret, const int64_t* idx, int B, float* oS, float* oA, float* olp, float* oadv,
                         float* oret, uint64_t* dropout_step, void* stream) {
  if (!S || !A || !lp || !adv || !ret || !idx || !oS || !oA || !olp || !oadv || !oret) return fail("prl_gather_minibatch: null");
  if (B <= 0 || sdim <= 0 || adim <= 0) return fail("prl_gather_minibatch: bad sizes");
  gather_kernel<<<B, 256, 0, (hipStream_t)stream>>>(S, sdim, A, adim, lp, adv, ret, idx, B, oS, oA, olp, oadv, oret,
                                                    dropout_step);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_lnrelu_fwd(const float* Z, const float* bias, const float* gamma, const float* beta, int B, int H, float eps,
                   float p, uint64_t seed, const uint64_t* dropout_step, int layer, float* Y, float* xhat, float* rstd,
                   void* stream) {
  if (!Z || !bias || !gamma || !beta || !Y || !xhat || !rstd) return fail("prl_lnrelu_fwd: null");
  if (B <= 0 || H <= 0 || H > 1024 || (p > 0.f && !dropout_step)) return fail("prl_lnrelu_fwd: bad arguments");
  const int threads = (H + 63) / 64 * 64;
  lnrelu_fwd_kernel<<<B, threads, 0, (hipStream_t)stream>>>(Z, bias, gamma, beta, H, eps, p, seed, dropout_step, layer,
                                                            Y, xhat, rstd);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_lnrelu_bwd(const float* dY, const float* Z, const float* bias, const float* xhat, const float* rstd,
                   const float* gamma, int B, int H, float p, uint64_t seed, const uint64_t* dropout_step, int layer,
                   float* dZ, float* dyx, float* dye, void* stream) {
  if (!dY || !Z || !bias || !xhat || !rstd || !gamma || !dZ || !dyx || !dye) return fail("prl_lnrelu_bwd: null");
  if (B <= 0 || H <= 0 || H > 1024 || (p > 0.f && !dropout_step)) return fail("prl_lnrelu_bwd: bad arguments");
  const int threads = (H + 63) / 64 * 64;
  lnrelu_bwd_kernel<<<B, threads, 0, (hipStream_t)stream>>>(dY, Z, bias, xhat, rstd, gamma, H, p, seed, dropout_step,
                                                            layer, dZ, dyx, dye);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_actor_head(const float* Z, const float* bias, const float* log_std, const float* act, const float* old_lp,
                   const float* adv, int B, int A, float clip, float ent_coef, float* dZ, float* dls, float* stats,
                   float* ent_rows, void* stream) {
  if (!Z || !bias || !log_std || !act || !old_lp || !adv || !dZ || !dls || !stats || !ent_rows)
    return fail("prl_actor_head: null");
  if (B <= 0 || A <= 0 || A > 64) return fail("prl_actor_head: need 0 < A <= 64");
  actor_head_kernel<<<(B + 3) / 4, 256, 0, (hipStream_t)stream>>>(Z, bias, log_std, act, old_lp, adv, B, A, clip,
                                                                  ent_coef, dZ, dls, stats, ent_rows);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_critic_head(const float* Z, const float* bias, const float* ret, int B, float* dZ, float* v, float* sq,
                    void* stream) {
  if (!Z || !bias || !ret || !dZ || !v || !sq || B <= 0) return fail("prl_critic_head: bad arguments");
  critic_head_kernel<<<(B + 255) / 256, 256, 0, (hipStream_t)stream>>>(Z, bias, ret, B, dZ, v, sq);
  HIPCHK(hipGetLastError());
  return 0;
}

int prl_colsums(int n, const float* const* src, const int* cols, const float* scale, float* const* dst, int B,
                float* scratch, size_t scratch_floats, void* stream) {
  if (n <= 0 || n > PRL_MAX_COLSUMS || !src || !cols || !dst || B <= 0) return fail("prl_colsums: bad arguments");
  ColSums cs{};
  int cmax = 0, total = 0;
  for (int i = 0; i < n; i++) {
    if (!src[i] || !dst[i] || cols[i] <= 0) return fail("prl_colsums: bad entry");
    cs.src[i] = src[i];
    cs.dst[i] = dst[i];
    cs.cols[i] = cols[i];
    cs.off[i] = total;
    cs.scale[i] = scale ? scale[i] : 1.f;
    cmax = cols[i] > cmax ? cols[i] : cmax;
    total += cols[i];
  }
  cs.n = n;
  cs.B = B;
  cs.total = total;
  const int nchunks = (B + COLSUM_CHUNK - 1) / COLSUM_CHUNK;
  cs.chunk = nchunks > 1 ? COLSUM_CHUNK : B;
  if (nchunks > 1) {
    if (!scratch || scratch_floats < (size_t)nchunks * total) return fail("prl_colsums: scratch too small");
    cs.part = scratch;
  }
  colsums_kernel<<<dim3((cmax + 127) / 128, n, nchunks > 1 ? nchunks : 1), 128, 0, (hipStream_t)stream>>>(cs);
  HIPCHK(hipGetLastError());
  if (nchunks > 1) {
    colsums_final_kernel<<<dim3((cmax + 127) / 128, n), 128, 0, (hipStream_t)stream>>>(cs, nchunks);
    HIPCHK(hipGetLastError());
  }
  return 0;
}

// ---------------------------------------------------------------- fused minibatch step on the matrix cores (mlp_step.inc)
namespace {
// the column-split rows kernel's shape conditions: <= 256 rows, state width 32..384, hidden
// widths 128 or 256 (mlp_split.inc)
bool split_shapes(const prl_net* nets, int sdim, int B) {
  if (B > mlp::SPLIT_MAX_ROWS || sdim > mlp::SPLIT_MAX_SDIM || sdim < 32) return false;
  for (int i = 0; i < 2; i++)
    for (int l = 0; l + 1 < nets[i].nlayers; l++)
      if (nets[i].layer[l].out != 128 && nets[i].layer[l].out != 256) return false;
  return true;
}

// work layout of prl_mlp_step: the per-tile partial rows [tiles][total] (bias / LayerNorm /
// log_std column sums and the 6 logged sums), then per network the inputs of layers 1..3
// [B][in] and every layer's dZ [B][out]; the reduction entries and the weight-gradient tiles
int mlp_layout(const prl_net* nets, int sdim, int B, float* work, float* log_row, mlp::Args* a, mlp::GradArgs* g,
               size_t* work_floats) {
  int off = 0, ne = 0;
  auto entry = [&](int n, float* dst, float scale) {
    if (ne >= mlp::MAXRED) return -1;
    g->e[ne] = mlp::RedEntry{off, n, scale, dst, -1};
    ne++;
    const int o = off;
    off += n;
    return o;
  };
  size_t scratch = 0;  // floats of X / dZ scratch, placed after the partial rows below
  for (int i = 0; i < 2; i++) {
    const prl_net& n = nets[i];
    if (n.nlayers != mlp::MAXL) return fail("prl_mlp_step: networks of 3 hidden layers + an output layer");
    if (n.head != i) return fail("prl_mlp_step: nets[0] is the actor (head 0), nets[1] the critic (head 1)");
    mlp::Net& d = a->net[i];
    d.nl = n.nlayers;
    d.head = n.head;
    int in = sdim;
    for (int l = 0; l < n.nlayers; l++) {
      const prl_layer& L = n.layer[l];
      const bool hidden = l + 1 < n.nlayers;
      if (L.in != in) return fail("prl_mlp_step: layer widths do not chain");
      if (hidden && (L.out <= 0 || L.out > mlp::HMAX || L.out % 16))
        return fail("prl_mlp_step: hidden widths must be multiples of 16 up to 256");
      if (!hidden && (L.out <= 0 || L.out > 64)) return fail("prl_mlp_step: output width must be 1..64");
      if (!L.W || !L.b || !L.dW || !L.db || (hidden && (!L.gamma || !L.beta || !L.dgamma || !L.dbeta)))
        return fail("prl_mlp_step: null layer pointer");
      mlp::Layer& o = d.L[l];
      o.in = L.in;
      o.out = L.out;
      o.W = L.W;
      o.b = L.b;
      o.g = L.gamma;
      o.be = L.beta;
      o.p = hidden ? L.dropout : 0.f;
      o.dW = L.dW;
      o.ob = entry(L.out, L.db, 1.f);
      o.og = hidden ? entry(L.out, L.dgamma, 1.f) : 0;
      o.obe = hidden ? entry(L.out, L.dbeta, 1.f) : 0;
      // scratch offsets for now; made pointers once the partial block's size is known
      o.X = l ? reinterpret_cast<float*>(scratch) : nullptr;
      scratch += l ? (size_t)B * L.in : 0;
      o.dZ = reinterpret_cast<float*>(scratch);
      scratch += (size_t)B * L.out;
      in = L.out;
    }
    d.log_std = n.log_std;
    d.ols = 0;
    if (i == 0) {
      if (!n.log_std || !n.dlog_std) return fail("prl_mlp_step: the actor needs log_std and its gradient");
      d.ols = entry(n.layer[n.nlayers - 1].out, n.dlog_std, 1.f);
    } else if (n.layer[n.nlayers - 1].out != 1) {
      return fail("prl_mlp_step: the critic's output width must be 1");
    }
  }
  a->ostat = entry(6, log_row, 1.f / (float)B);
  if (a->ostat < 0) return fail("prl_mlp_step: too many gradient entries");
  a->total = off;
  const int ntiles = (B + mlp::MT - 1) / mlp::MT;
  const size_t npart = (size_t)ntiles * off;
  const size_t sg_off = scratch;  // then the gathered state rows [B][sdim] (prl_mlp_step_idx)
  scratch += (size_t)B * sdim;
  *work_floats = npart + scratch;
  a->Sg = work ? work + npart + sg_off : nullptr;
  // mlp_split_kernel's exchange granules, call counts and error word (the last word), when the
  // shapes allow the split (mlp_split.inc)
  a->hand = nullptr;
  a->cnt = a->err = nullptr;
  if (split_shapes(nets, sdim, B)) {
    const int groups = 2 * ntiles;
    const size_t ho = (*work_floats + 3) & ~(size_t)3;
    const size_t co = ho + mlp::split_hand_floats(groups);
    *work_floats = co + (size_t)groups + 1;
    if (work) {
      a->hand = work + ho;
      a->cnt = reinterpret_cast<unsigned*>(work + co);
      a->err = reinterpret_cast<unsigned*>(work + *work_floats - 1);
    }
  }
  g->ne = ne;
  g->rfirst[0] = 0;
  for (int e = 0; e < ne; e++) g->rfirst[e + 1] = g->rfirst[e] + (g->e[e].n + 63) / 64;
  int qtiles = 0;
  for (int i = 0; i < 2; i++)
    for (int l = 0; l < mlp::MAXL; l++) {
      const mlp::Layer& o = a->net[i].L[l];
      qtiles += ((o.out + 15) / 16) * ((o.in + 15) / 16);
    }
  g->ntw = qtiles;
  if (!work) return 0;  // size query (ne, rfirst, ntw: the gradient kernel's wave count)
  // pointers: partial rows, then the scratch
  g->total = off;
  g->ntiles = ntiles;
  g->part = work;
  int gl = 0, tiles = 0;
  for (int i = 0; i < 2; i++)
    for (int l = 0; l < mlp::MAXL; l++) {
      mlp::Layer& o = a->net[i].L[l];
      o.X = l ? work + npart + reinterpret_cast<size_t>(o.X) : nullptr;
      o.dZ = work + npart + reinterpret_cast<size_t>(o.dZ);
      g->X[gl] = o.X;  // layer 0: the state rows, set by the caller
      g->dZ[gl] = o.dZ;
      g->dW[gl] = o.dW;
      g->N[gl] = o.out;
      g->K[gl] = o.in;
      g->tk[gl] = (o.in + 15) / 16;
      g->first[gl] = tiles;
      tiles += ((o.out + 15) / 16) * g->tk[gl];
      gl++;
    }
  g->first[gl] = tiles;
  g->nl = gl;
  g->ntw = tiles;
  g->B = B;
  return 0;
}
}  // namespace

size_t prl_mlp_step_work(const prl_net* nets, int sdim, int B) {
  mlp::Args a{};
  mlp::GradArgs g{};
  float dummy;
  size_t wf = 0;
  if (!nets || B <= 0 || sdim <= 0 || mlp_layout(nets, sdim, B, nullptr, &dummy, &a, &g, &wf)) return 0;
  return wf;
}

int prl_mlp_step_norm_parts(const prl_net* nets, int sdim, int B) {
  mlp::Args a{};
  mlp::GradArgs g{};
  float dummy;
  size_t wf = 0;
  if (!nets || B <= 0 || sdim <= 0 || mlp_layout(nets, sdim, B, nullptr, &dummy, &a, &g, &wf)) return 0;
  return (g.ntw + g.rfirst[g.ne] + mlp::GWV - 1) / mlp::GWV;  // the gradient kernel's workgroups
}

}  // extern "C"

namespace {
// prl_mlp_step / prl_mlp_step_idx: idx = nullptr takes rows 0..B-1 of S / A / ...; otherwise the
// rows idx[0..B), read in place by the rows kernel, with the dropout step counter advanced once
// (by the gradient kernel, after the rows kernel read it)
struct NormOut {  // prl_mlp_step_idx_norm: the grad-norm partials for prl_clip_adam_parts
  const float* grad_base;
  const int64_t* seg_end;
  int nseg;
  float* adam_step;
  double* part;
  int nparts;
};
int mlp_step(const prl_net* nets, const float* S, int sdim, const float* A, int adim, const float* old_lp,
             const float* adv, const float* ret, const int64_t* idx, int B, float clip, float ent_coef, float ln_eps,
             uint64_t seed, uint64_t* step_inc, const uint64_t* step, float* log_row, float* work, size_t work_floats,
             unsigned* guard, void* stream, const NormOut* no = nullptr) {
  if (!nets || !S || !A || !old_lp || !adv || !ret || !step || !log_row || !work) return fail("prl_mlp_step: null argument");
  if (B <= 0 || sdim <= 0 || sdim > 1024) return fail("prl_mlp_step: B > 0 and 0 < sdim <= 1024 required");
  mlp::Args a{};
  mlp::GradArgs g{};
  size_t need = 0;
  if (mlp_layout(nets, sdim, B, work, log_row, &a, &g, &need)) return -1;
  if (nets[0].layer[3].out != adim) return fail("prl_mlp_step: actor output width != action dim");
  if (work_floats < need) return fail("prl_mlp_step: work space too small (prl_mlp_step_work)");
  const size_t lds = mlp::lds_floats(((sdim + 15) & ~15) + 4) * sizeof(float);
  if (lds > 150 * 1024) return fail("prl_mlp_step: state too wide for the LDS tile");
  a.nnets = 2;
  a.S = S;
  a.A = A;
  a.LP = old_lp;
  a.ADV = adv;
  a.RET = ret;
  a.idx = nullptr;
  a.sdim = sdim;
  a.adim = adim;
  a.B = B;
  a.clip = clip;
  a.ent = ent_coef;
  a.eps = ln_eps;
  a.seed = seed;
  a.step = step;
  a.part = work;
  g.X[0] = S;
  g.X[mlp::MAXL] = S;
  g.step_inc = nullptr;
  if (idx) {  // gathered in the rows kernel; the weight gradient reads its copy Sg
    a.idx = idx;
    g.X[0] = g.X[mlp::MAXL] = a.Sg;
    g.step_inc = step_inc;
  }
  a.Sg = a.idx ? a.Sg : nullptr;
  if (guard && a.hand) a.err = guard;  // the split kernel's error word: the caller's guard
  g.guard = guard ? guard : a.hand ? a.err : nullptr;
  {
    const char* st = getenv("PIANORL_SPLIT_SPIN_TICKS");
    a.spin_ticks = st ? strtoull(st, nullptr, 10) : mlp::SPLIT_SPIN_TICKS;
    const char* ft = getenv("PIANORL_SPLIT_TEST_FAULT");
    a.fault = ft && ft[0] == '1';
  }
  g.npart = nullptr;
  if (no) {  // each gradient write's clip+Adam segment, from its offset in the flat gradient buffer
    if (!no->grad_base || !no->seg_end || no->nseg < 1 || no->nseg > PRL_MAX_SEG || !no->adam_step || !no->part)
      return fail("prl_mlp_step_idx_norm: bad optimiser arguments");
    auto seg_of = [&](const float* p) {
      const int64_t o = p - no->grad_base;
      for (int s = 0; s < no->nseg; s++)
        if (o >= 0 && o < no->seg_end[s]) return s;
      return -1;
    };
    for (int l = 0; l < g.nl; l++) {
      g.seg[l] = seg_of(g.dW[l]);
      if (g.seg[l] < 0) return fail("prl_mlp_step_idx_norm: a weight gradient outside the segments");
    }
    for (int e = 0; e < g.ne; e++) {
      g.e[e].seg = g.e[e].dst == log_row ? -1 : seg_of(g.e[e].dst);
      if (g.e[e].dst != log_row && g.e[e].seg < 0) return fail("prl_mlp_step_idx_norm: a gradient outside the segments");
    }
    const int blocks = (g.ntw + g.rfirst[g.ne] + mlp::GWV - 1) / mlp::GWV;
    if (no->nparts < blocks) return fail("prl_mlp_step_idx_norm: partial buffer too small (prl_mlp_step_norm_parts)");
    g.npart = no->part;
    g.adam_step = no->adam_step;
    g.nseg = no->nseg;
  }
  static bool attr_set = false;
  if (!attr_set) {
    HIPCHK(hipFuncSetAttribute((const void*)mlp::mlp_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               150 * 1024));  // (+ its static LDS)
    HIPCHK(hipFuncSetAttribute((const void*)mlp::mlp_split_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024));
    attr_set = true;
  }
  // the column-split kernel where the shapes allow it (its exchange region is in the work
  // space); PIANORL_MLP_SPLIT=0 selects the one-workgroup-per-tile kernel
  const char* sv = getenv("PIANORL_MLP_SPLIT");
  // its exchanges need every member of a group resident at once: one workgroup per CU (the
  // LDS request), so the groups' workgroups must not outnumber the device's CUs
  int dev = 0, cus = 0;
  HIPCHK(hipGetDevice(&dev));
  HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const bool split_fits = 2 * g.ntiles * mlp::NSPL <= cus;
  if (a.hand && split_fits && !(sv && sv[0] == '0')) {
    const size_t slds = mlp::split_lds_floats(((sdim + 15) & ~15) + 4) * sizeof(float);
    if (slds > 160 * 1024) return fail("prl_mlp_step: split kernel LDS over 160 KB");
    const int groups = 2 * g.ntiles;
    hipLaunchKernelGGL(mlp::mlp_split_kernel, dim3(32 * ((groups + 7) / 8)), dim3(mlp::ST), slds,
                       (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL(mlp::mlp_rows_kernel, dim3(g.ntiles, 2), dim3(mlp::NT), lds, (hipStream_t)stream, a);
  }
  HIPCHK(hipGetLastError());
  const int waves = g.ntw + g.rfirst[g.ne];
  hipLaunchKernelGGL(mlp::mlp_grad_kernel, dim3((waves + mlp::GWV - 1) / mlp::GWV), dim3(mlp::GWV * 64), 0,
                     (hipStream_t)stream, g);
  HIPCHK(hipGetLastError());
  return 0;
}
}  // namespace

extern "C" {
int prl_mlp_step(const prl_net* nets, const float* S, int sdim, const float* A, int adim, const float* old_lp,
                 const float* adv, const float* ret, int B, float clip, float ent_coef, float ln_eps, uint64_t seed,
                 const uint64_t* step, float* log_row, float* work, size_t work_floats, unsigned* guard,
                 void* stream) {
  return mlp_step(nets, S, sdim, A, adim, old_lp, adv, ret, nullptr, B, clip, ent_coef, ln_eps, seed, nullptr, step,
                  log_row, work, work_floats, guard, stream);
}

int prl_mlp_step_idx(const prl_net* nets, const float* S, int sdim, const float* A, int adim, const float* old_lp,
                     const float* adv, const float* ret, const int64_t* idx, int B, float clip, float ent_coef,
                     float ln_eps, uint64_t seed, uint64_t* step, float* log_row, float* work, size_t work_floats,
                     unsigned* guard, void* stream) {
  if (!idx) return fail("prl_mlp_step_idx: null idx");
  return mlp_step(nets, S, sdim, A, adim, old_lp, adv, ret, idx, B, clip, ent_coef, ln_eps, seed, step, step, log_row,
                  work, work_floats, guard, stream);
}

int prl_mlp_step_idx_norm(const prl_net* nets, const float* S, int sdim, const float* A, int adim,
                          const float* old_lp, const float* adv, const float* ret, const int64_t* idx, int B,
                          float clip, float ent_coef, float ln_eps, uint64_t seed, uint64_t* step, float* log_row,
                          float* work, size_t work_floats, const float* grad_base, const int64_t* seg_end, int nseg,
                          float* adam_step, double* norm_part, int nparts, unsigned* guard, void* stream) {
  if (!idx) return fail("prl_mlp_step_idx_norm: null idx");
  const NormOut no{grad_base, seg_end, nseg, adam_step, norm_part, nparts};
  return mlp_step(nets, S, sdim, A, adim, old_lp, adv, ret, idx, B, clip, ent_coef, ln_eps, seed, step, step, log_row,
                  work, work_floats, guard, stream, &no);
}

#ifdef MLP_TIMING
int prl_mlp_timing_get(uint64_t* out /* host [2][32] */) {
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(mlp::g_tstamp), sizeof(uint64_t) * 64));
  return 0;
}
#endif

}  // extern "C"
