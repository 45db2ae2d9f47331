/*
 * pianorl.h - C-ABI of the on-device PPO kernels (the
 * consumer of the hot path, ppo_v2.py's PPOAgent, moved into HBM).
 *
 * The reference has no FFI here either: its agent is Python over torch, with the rollout
 * statistics computed on the host in numpy / Python loops. These entry points replace
 * those host loops; the MLPs stay torch modules (hipBLASLt GEMMs) and are driven by
 * diffusion-piano_amd/ppo.py, which binds this library with ctypes:
 *
 *   prl_running_norm  <- RunningMeanStd.__call__ (ppo_v2.py:113-131): batch mean / population
 *                        variance, running-statistics merge (Chan et al.), normalise with the
 *                        merged statistics. fp64 statistics, as the reference's numpy.
 *   prl_gae           <- the GAE loop of PPOAgent.update (ppo_v2.py:239-253) and the TD
 *                        returns (:234-237). Layout [T, E] (time-major). E = 1, T = batch
 *                        reproduces the reference exactly (it runs the recursion over the
 *                        env batch axis); E = envs gives the time-axis GAE of a rollout.
 *   prl_normalize     <- advantages = (a - a.mean()) / (a.std() + 1e-8) (ppo_v2.py:256),
 *                        unbiased std as torch.std.
 *   prl_clip_adam     <- clip_grad_norm_(max_grad_norm) + optimizer.step() of each network
 *                        (ppo_v2.py:280-293), fused over one flat parameter buffer.
 *   prl_gather_minibatch, prl_lnrelu_fwd / _bwd, prl_actor_head, prl_critic_head,
 *   prl_colsums       <- the minibatch step's forward + autograd backward (ppo_v2.py:266-293)
 *                        between the GEMMs: one launch per layer and direction.
 *   prl_gauss_sample  <- select_actions: Normal(mean, exp(clamp(log_std,-20,2))).sample() and
 *                        log_prob(actions).sum(1) (ppo_v2.py:70-74, 211-218). Counter-based
 *                        Philox4x32-10 keyed by (seed, offset, row, column).
 *
 * Conventions as include/pianosim.h: DEVICE pointers, asynchronous on the caller's HIP
 * stream (NULL = default), 0 = OK / < 0 = error with a thread-local prl_last_error().
 *
 * ABI version 2 (prl_version): prl_mlp_step* and prl_clip_adam* take a trailing `guard`, a
 * device u32 shared by one optimiser's launches (NULL = none). The column-split rows kernel
 * writes its error code there (1 + the exchange whose bounded wait timed out); while it is
 * non-zero the gradient kernel does not advance the Adam step counts and prl_clip_adam* leave
 * parameters, moments and step counts unchanged, so a failed step can never reach the
 * weights. The caller reads it at its next sync point, clears it and the work space, and
 * reports the failure (ppo.py raises PianosimError). Callers built against version 1 must be
 * rebuilt: the argument lists changed.
 */
#ifndef PIANORL_H
#define PIANORL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRL_MAX_SEG 4 /* parameter segments of prl_clip_adam (one per network) */

/* returns_mode of prl_gae */
#define PRL_RETURNS_TD 0  /* ret = r + gamma * next_values * (1 - done)   (ppo_v2.py:234-237) */
#define PRL_RETURNS_GAE 1 /* ret = adv + values                           (standard PPO target) */

const char* prl_last_error(void);
int prl_version(void);

/* x[n] f32 -> out[n] f32; stats[3] f64 = {mean, var, count}, updated in place. */
int prl_running_norm(const float* x, int n, double* stats, float* out, void* stream);

/* rewards/values/next_values/dones [T*E] f32 (dones 0/1) -> adv, ret [T*E] f32.
 * delta_t = r_t + gamma * nv_t * (1 - d_t) - v_t, nv_t = values[t+1] (t < T-1) else
 * next_values[T-1]; gae_t = delta_t + gamma * lam * (1 - d_t) * gae_{t+1}. */
int prl_gae(const float* rewards, const float* values, const float* next_values, const float* dones,
            float* adv, float* ret, int T, int E, float gamma, float lam, int returns_mode, void* stream);

/* x[n] f32, in place: (x - mean) / (std_unbiased + eps). */
int prl_normalize(float* x, int n, float eps, void* stream);

/* mean[n, a] f32, log_std[a] f32 -> action[n, a], logp[n] (sum over a). a <= 64. */
int prl_gauss_sample(const float* mean, const float* log_std, int n, int a, uint64_t seed, uint64_t offset,
                     float* action, float* logp, void* stream);

/* clip_grad_norm_ + Adam over flat fp32 buffers (ppo_v2.py:280-293: clip each network's
 * gradient to max_norm, then its Adam step; torch.nn.utils.clip_grad_norm_ and
 * torch.optim.Adam(betas, eps), amsgrad and weight decay off). param / grad / exp_avg /
 * exp_avg_sq [n], n = seg_end[nseg-1]; segment s = [seg_end[s-1], seg_end[s]) (HOST array)
 * has its own clip, lr[s] (device) and step[s] (device f32, incremented here);
 * scratch: device f64 [256 * PRL_MAX_SEG]. max_norm <= 0 disables clipping. */
int prl_clip_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_end,
                  int nseg, const float* lr, float* step, float beta1, float beta2, float eps, float max_norm,
                  double* scratch, const unsigned* guard, void* stream);
/* prl_clip_adam with the gradient-norm partials already summed per segment (parts [nparts]
 * [PRL_MAX_SEG] f64, prl_mlp_step_idx_norm) and the step counts already advanced: one launch. */
int prl_clip_adam_parts(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_end,
                        int nseg, const float* lr, const float* step, float beta1, float beta2, float eps,
                        float max_norm, const double* parts, int nparts, const unsigned* guard, void* stream);

/* ---- fused minibatch step (ppo_v2.py:266-293 with the backward written out; the GEMMs
 * between these are library GEMMs). All row-major fp32 [rows, cols]. */
#define PRL_MAX_COLSUMS 32

/* gather minibatch rows idx[B] (int64) of S [N, sdim], A [N, adim], lp/adv/ret [N]; also
 * increments *dropout_step (device u64, may be NULL): one dropout draw per minibatch */
int prl_gather_minibatch(const float* S, int sdim, const float* A, int adim, const float* lp, const float* adv,
                         const float* ret, const int64_t* idx, int B, float* oS, float* oA, float* olp, float* oadv,
                         float* oret, uint64_t* dropout_step, void* stream);

/* Y = Dropout_p(LayerNorm(ReLU(Z + bias))) per row (H <= 1024); xhat, rstd kept for the
 * backward. p = 0: no dropout. Keep mask: Philox(seed, *dropout_step, layer, row, col). */
int prl_lnrelu_fwd(const float* Z, const float* bias, const float* gamma, const float* beta, int B, int H, float eps,
                   float p, uint64_t seed, const uint64_t* dropout_step, int layer, float* Y, float* xhat, float* rstd,
                   void* stream);

/* backward: dZ [B, H]; dyx = dY' * xhat and dye = dY' (dY' = dY through the dropout mask),
 * whose column sums are the LayerNorm gamma / beta gradients */
int prl_lnrelu_bwd(const float* dY, const float* Z, const float* bias, const float* xhat, const float* rstd,
                   const float* gamma, int B, int H, float p, uint64_t seed, const uint64_t* dropout_step, int layer,
                   float* dZ, float* dyx, float* dye, void* stream);

/* actor head: mu = tanh(Z + bias) [B, A <= 64], Normal(mu, exp(clamp(log_std))) log-prob of
 * act, PPO clipped surrogate vs old_lp / adv; dZ = d loss / d Z, dls = per-row log_std
 * gradient (entropy bonus included), stats[r] = -min(surr1, surr2) - ent_coef * entropy
 * (its mean is the actor loss), ent_rows[r] = dist.entropy().mean() */
int prl_actor_head(const float* Z, const float* bias, const float* log_std, const float* act, const float* old_lp,
                   const float* adv, int B, int A, float clip, float ent_coef, float* dZ, float* dls, float* stats,
                   float* ent_rows, void* stream);

/* critic head: v = Z + bias [B], dZ = 2 (v - ret) / B, v and (v - ret)^2 out */
int prl_critic_head(const float* Z, const float* bias, const float* ret, int B, float* dZ, float* v, float* sq,
                    void* stream);

/* dst[i][c] = scale[i] * sum_r src[i][r * cols[i] + c] for n <= PRL_MAX_COLSUMS arrays of B rows
 * (pointer / size arrays are HOST arrays of device pointers; scale may be NULL = 1). Above 128
 * rows the sum runs in 128-row chunks through scratch (device, >= ceil(B/128) * sum(cols)
 * floats), summed in chunk order: deterministic for every B. */
int prl_colsums(int n, const float* const* src, const int* cols, const float* scale, float* const* dst, int B,
                float* scratch, size_t scratch_floats, void* stream);

/* One PPO minibatch step (ppo_v2.py:266-293: actor and critic forward, clipped surrogate and
 * MSE heads, the whole backward) on the matrix cores: a workgroup per 16 minibatch rows and
 * network runs every layer in LDS (v_mfma_f32_16x16x4_f32, exact fp32), then one launch adds
 * the per-tile gradient partials in tile order (deterministic). Replaces the ~40 launches of
 * prl_gather_minibatch's followers (GEMMs + lnrelu_fwd/bwd + heads + colsums) for small
 * minibatches. Network i = layers 0..2 (Linear -> ReLU -> LayerNorm (eps ln_eps) -> Dropout
 * p) and the output Linear; nets[0] = actor (tanh mean, Gaussian with log_std, head 0),
 * nets[1] = critic (head 1). Gradients are written (not accumulated) to the d* pointers;
 * log_row [6] = the means of actor loss rows, critic squared errors, entropy, value, return,
 * advantage. Dropout masks are prl_lnrelu_fwd's (seed, *step, layer, row, column). All
 * pointers device; nets is a host array. work: prl_mlp_step_work(nets, sdim, B) floats, ZEROED
 * before its first call and then kept between calls: for B <= 256, state width <= 384 and
 * hidden widths of 128 or 256 its tail holds the column-split rows kernel's tagged exchange
 * slices and per-tile call counts (4 workgroups per 16-row tile and network, six exchanges per
 * step; PIANORL_MLP_SPLIT=0 selects the one-workgroup-per-tile kernel; the host takes it only
 * when its 4 x 2 x ceil(B / 16) workgroups fit the device's CU count), and its last word is
 * that kernel's error word (0, or 1 + the exchange whose bounded wait timed out) unless a
 * guard is given (see the ABI note above). Test hooks, read per call: PIANORL_SPLIT_SPIN_TICKS
 * (the bounded wait, 100 MHz ticks, default 2 s) and PIANORL_SPLIT_TEST_FAULT=1 (one member
 * never publishes its first exchange, so the others time out). */
typedef struct {
  int in, out;
  const float *W, *b, *gamma, *beta;  /* W [out][in]; gamma/beta: NULL on the output layer */
  float dropout;
  float *dW, *db, *dgamma, *dbeta;
} prl_layer;
typedef struct {
  int nlayers, head;  /* 4; 0 actor, 1 critic */
  prl_layer layer[4];
  const float* log_std;
  float* dlog_std;
} prl_net;
size_t prl_mlp_step_work(const prl_net* nets, int sdim, int B);
int prl_mlp_step(const prl_net* nets, const float* S, int sdim, const float* A, int adim, const float* old_lp,
                 const float* adv, const float* ret, int B, float clip, float ent_coef, float ln_eps, uint64_t seed,
                 const uint64_t* step, float* log_row, float* work, size_t work_floats, unsigned* guard,
                 void* stream);
/* prl_gather_minibatch + prl_mlp_step in one: S / A / old_lp / adv / ret are the whole rollout
 * ([N, sdim] ...), the minibatch is rows idx[B] (int64), read in place by the rows kernel; the
 * dropout step counter *step is advanced once (as prl_gather_minibatch does). Same work size. */
int prl_mlp_step_idx(const prl_net* nets, const float* S, int sdim, const float* A, int adim, const float* old_lp,
                     const float* adv, const float* ret, const int64_t* idx, int B, float clip, float ent_coef,
                     float ln_eps, uint64_t seed, uint64_t* step, float* log_row, float* work, size_t work_floats,
                     unsigned* guard, void* stream);
/* prl_mlp_step_idx that also leaves the clip_grad_norm_ partials for prl_clip_adam_parts (one
 * launch less per minibatch): grad_base = the flat gradient buffer the layers' gradients live
 * in, seg_end[nseg] its segments (as prl_clip_adam); the gradient kernel writes each workgroup's sum
 * of squares per segment into norm_part [nparts][PRL_MAX_SEG] f64 (nparts >=
 * prl_mlp_step_norm_parts) and advances adam_step[nseg] (the optimisers' step counts) by one. */
int prl_mlp_step_norm_parts(const prl_net* nets, int sdim, int B);
int prl_mlp_step_idx_norm(const prl_net* nets, const float* S, int sdim, const float* A, int adim,
                          const float* old_lp, const float* adv, const float* ret, const int64_t* idx, int B,
                          float clip, float ent_coef, float ln_eps, uint64_t seed, uint64_t* step, float* log_row,
                          float* work, size_t work_floats, const float* grad_base, const int64_t* seg_end, int nseg,
                          float* adam_step, double* norm_part, int nparts, unsigned* guard, void* stream);

#ifdef __cplusplus
}
#endif
#endif
