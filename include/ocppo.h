/*
 * ocppo.h — C-ABI of libocppo_hip.so, the MI355X (gfx950) kernels behind the OC-CleanRL PPO
 * actor-learner hot path.
 *
 * The reference (BluemlJ/oc_cleanrl) is pure Python; there is no FFI to mirror. Each entry point
 * below replaces one stock-PyTorch op sequence of `cleanrl/ppo_atari_oc.py` (and its DP twin
 * `cleanrl/ppo_atari_multigpu.py`); the replaced lines are cited per function. A caller binds the
 * library with ctypes and passes torch `data_ptr()`s.
 *
 * Conventions (all functions):
 *   - every pointer is a caller-owned DEVICE pointer unless stated otherwise; nothing allocates;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); every launch is asynchronous and
 *     graph-capturable (no host sync, no hipMalloc, no memcpy to host inside);
 *   - the return value is 0 on success, otherwise an OCPPO_E_* code; ocppo_last_error() returns
 *     a thread-local message for the last failure. Nothing throws or aborts across the ABI;
 *   - results are deterministic: fixed-order reductions, no floating-point atomics;
 *   - scalar hyper-parameters are passed as double, exactly as the reference's Python floats,
 *     and rounded to f32 inside the library exactly where PyTorch rounds them.
 *   - all buffers are step-major: element (t, n) of a [T, N] rollout array is at t*N + n
 *     (ppo_atari_oc.py:452-459, flattened at :550-555).
 */
#ifndef OCPPO_H
#define OCPPO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCPPO_ABI_VERSION 28

/* status codes */
#define OCPPO_OK 0
#define OCPPO_E_INVALID 1   /* bad argument (null pointer, size, dtype) */
#define OCPPO_E_LAUNCH 2    /* hipGetLastError() after a launch */
#define OCPPO_E_WORKSPACE 3 /* workspace missing or too small */

/* element types used by the obs storage / frame arguments */
#define OCPPO_F32 0
#define OCPPO_BF16 1
#define OCPPO_U8 2

/* net_flags of the rollout store / reset / channels-last gather */
#define OCPPO_NET_CHANNELS_LAST 1
#define OCPPO_NET_SCALE_255 2

/* layout of the `stats` output of ocppo_ppo_loss_fwd_bwd (all f32) */
#define OCPPO_STAT_LOSS 0          /* loss = pg - ent_coef*entropy + vf_coef*v_loss   :599-602 */
#define OCPPO_STAT_PG_LOSS 1       /* pg_loss                                        :581-583 */
#define OCPPO_STAT_V_LOSS 2        /* v_loss                                         :585-597 */
#define OCPPO_STAT_ENTROPY 3       /* entropy_loss = mean(entropy)                   :599     */
#define OCPPO_STAT_OLD_APPROX_KL 4 /* mean(-logratio)                                :573     */
#define OCPPO_STAT_APPROX_KL 5     /* mean((ratio-1) - logratio)                     :574     */
#define OCPPO_STAT_CLIPFRAC 6      /* mean(|ratio-1| > clip_coef)                    :575     */
#define OCPPO_STAT_ADV_MEAN 7      /* minibatch advantage mean used by the norm      :577-579 */
#define OCPPO_STAT_ADV_STD 8       /* minibatch advantage std (unbiased)             :577-579 */
#define OCPPO_NUM_STATS 9

typedef void* ocppo_stream_t; /* hipStream_t */
/* A deferred finish (ocppo_heads_loss_rows, ocppo_relu_bias_wgrad_rows): a plain host record of
 * device pointers and sizes, run later by ocppo_sum_splits_finish / ocppo_sum_splits_db_finish /
 * ocppo_deferred_finish_run. */
typedef struct ocppo_deferred_finish {
  uint64_t opaque[64];
} ocppo_deferred_finish_t;

#if defined(__GNUC__) || defined(__clang__)
#define OCPPO_API __attribute__((visibility("default")))
#else
#define OCPPO_API
#endif

OCPPO_API int ocppo_abi_version(void);
OCPPO_API const char* ocppo_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * GAE — replaces the reverse Python loop of ppo_atari_oc.py:533-547 (identical in ppo.py:218-231
 * and ppo_atari_multigpu.py:288-301); 9 ATen launches per step → one kernel per rollout.
 *   rewards, values, dones : [T, N] f32;   next_value, next_done : [N] f32
 *   advantages, returns    : [T, N] f32 outputs (returns = advantages + values)
 * f32 arithmetic in the reference's exact op order (no FMA contraction), so the result is
 * bit-identical to the PyTorch loop:  delta = (r + (f32(gamma)*nv)*nnt) - v;
 *                                     A = delta + (f32(gamma*lambda)*nnt)*A'
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_gae(ocppo_stream_t stream, const float* rewards, const float* values, const float* dones,
              const float* next_value, const float* next_done, int64_t T, int64_t N, double gamma,
              double gae_lambda, float* advantages, float* returns);
/* GAE that also writes each sample's record (OcppoSampleRecord: log-prob, advantage, value,
 * action) in batch order for ocppo_minibatch_prepare_records; advantages / returns as ocppo_gae,
 * bit for bit. logprobs [T, N] f32 16-B aligned, actions [T, N] int64 in [0, 2^31), records
 * [T*N] 16-B aligned. */
OCPPO_API int ocppo_gae_records(ocppo_stream_t stream, const float* rewards, const float* values,
                                const float* dones, const float* next_value,
                                const float* next_done, int64_t T, int64_t N, double gamma,
                                double gae_lambda, float* advantages, float* returns,
                                const float* logprobs, const int64_t* actions, void* records);

/* ---------------------------------------------------------------------------------------------
 * Minibatch advantage statistics — the (mean, unbiased std) pair of ppo_atari_oc.py:577-579 for
 * `num_mb` minibatches at once. Minibatch k holds b_advantages[perm[k*M + i]], i < M.
 *   perm : [num_mb*M] int64 (the np.random.shuffle'd b_inds of :561, all epochs concatenated)
 *   out  : [num_mb, 2] f32 = {mean, std}
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_minibatch_adv_stats(ocppo_stream_t stream, const float* b_advantages, const int64_t* perm,
                              int64_t M, int64_t num_mb, float* out);

/* Minibatch prepare: the statistics above AND the per-sample records of every minibatch gathered
 * into minibatch order, mb_*[k*M + i] = b_*[perm[k*M + i]] (SoA), so that each
 * ocppo_ppo_loss_fwd_bwd launch can take the already-gathered arrays (mb_inds = NULL) instead of
 * five scattered loads per element (ppo_atari_oc.py:569-593 index b_* by mb_inds). One launch:
 * gather blocks over all num_mb*M elements on a chip-filling grid beside one statistics block
 * per minibatch (bitwise the figures of ocppo_minibatch_adv_stats).
 * adv_stats : [num_mb, 2] or NULL (statistics skipped). */
OCPPO_API int ocppo_minibatch_prepare(ocppo_stream_t stream, const int64_t* perm, int64_t M,
                                      int64_t num_mb, const int64_t* b_actions,
                                      const float* b_logprobs, const float* b_advantages,
                                      const float* b_returns, const float* b_values,
                                      int64_t* mb_actions, float* mb_logprobs,
                                      float* mb_advantages, float* mb_returns, float* mb_values,
                                      float* adv_stats);

/* ---------------------------------------------------------------------------------------------
 * The same, from 16-B per-sample records (OcppoSampleRecord, written by ocppo_gae_records): one
 * 16-B gather per sample instead of five scattered 4-8 B ones (the batch arrays of
 * ppo_atari_oc.py:550-555 are the records' fields; the return is advantage + value, GAE's own f32
 * add); outputs and statistics bitwise those of ocppo_minibatch_prepare. records: 16-B aligned,
 * [B]; actions in [0, 2^31). From 2^20 samples (num_mb x M) on, the statistics are taken by a
 * second launch from the gathered advantages (contiguous reads; same values, same order). 
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  float logprob, advantage, value;
  int32_t action;
} OcppoSampleRecord;
OCPPO_API int ocppo_minibatch_prepare_records(ocppo_stream_t stream, const int64_t* perm,
                                              int64_t M, int64_t num_mb, const void* records,
                                              int64_t* mb_actions, float* mb_logprobs,
                                              float* mb_advantages, float* mb_returns,
                                              float* mb_values, float* adv_stats);

/* ---------------------------------------------------------------------------------------------
 * Fused PPO minibatch loss, forward AND backward — replaces ppo_atari_oc.py:566-602 from the
 * network's raw outputs onward (Categorical log-softmax / log_prob / entropy of
 * architectures/ppo.py:89-95, ratio, KL stats, clipfrac, advantage norm, clipped surrogate,
 * clipped value loss, entropy bonus) plus the autograd backward of that graph down to the
 * network outputs.
 *   logits    : [M, A] f32 raw actor outputs;  new_value : [M] f32 critic outputs
 *   mb_inds   : [M] int64 indices into the b_* batch arrays, or NULL (inputs already gathered,
 *               b_*[i] is element i)
 *   b_actions : int64 [B]; b_logprobs, b_advantages, b_returns, b_values : f32 [B]
 *   adv_stats : [2] f32 {mean, std} from ocppo_minibatch_adv_stats, or NULL to compute them
 *               here (then workspace must be given); ignored when norm_adv == 0
 *   dlogits   : [M, A] f32 = dLoss/dlogits;  dvalue : [M] f32 = dLoss/dnew_value
 *   stats     : [OCPPO_NUM_STATS] f32 (layout above)
 *   workspace : device scratch of ocppo_ppo_loss_workspace_bytes(M, A) bytes; it must be zeroed
 *               once after allocation and then never touched by the caller (its ticket word is
 *               reset by the kernel itself, so the call can be replayed from a graph).
 * Gradient rules follow autograd exactly: torch.max splits the gradient 1/2-1/2 on ties, clamp
 * passes it at the bounds.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API size_t ocppo_ppo_loss_workspace_bytes(int64_t M, int64_t A);
OCPPO_API int ocppo_ppo_loss_fwd_bwd(ocppo_stream_t stream, const float* logits, const float* new_value,
                           int64_t M, int64_t A, const int64_t* mb_inds, const int64_t* b_actions,
                           const float* b_logprobs, const float* b_advantages,
                           const float* b_returns, const float* b_values, const float* adv_stats,
                           double clip_coef, double ent_coef, double vf_coef, int norm_adv,
                           int clip_vloss, float* dlogits, float* dvalue, float* stats,
                           void* workspace, size_t workspace_bytes);

/* ---------------------------------------------------------------------------------------------
 * Gradient clipping + Adam over ONE flat buffer — replaces
 * `nn.utils.clip_grad_norm_(agent.parameters(), max_grad_norm); optimizer.step()` of
 * ppo_atari_oc.py:608-610 (torch.optim.Adam(lr, eps=1e-5), betas (0.9, 0.999)) and the
 * `grads / world_size` of ppo_atari_multigpu.py:369-374 (grad_scale = 1/world_size).
 *   params, grads, exp_avg, exp_avg_sq : [P] f32, 16-byte aligned; every parameter tensor of the
 *                                        agent is a view into `params` (grads likewise)
 *   lr       : device f32 scalar (annealed in place, graph-replay safe)
 *   scalars  : device f32[OCPPO_OPT_NUM_SCALARS], zero-initialised; the step count lives here and
 *              total_norm (the value clip_grad_norm_ returns) is reported here
 *   max_norm : <= 0 disables clipping
 * Math per element, f32: g = (g*grad_scale)*clip; m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g;
 * p -= (lr/(1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)  (ATen's fused-Adam formula).
 * ------------------------------------------------------------------------------------------- */
#define OCPPO_OPT_STEP 0
#define OCPPO_OPT_TOTAL_NORM 1
#define OCPPO_OPT_CLIP_COEF 2
#define OCPPO_OPT_STEP_SIZE 3
#define OCPPO_OPT_BC2_SQRT 4
#define OCPPO_OPT_NUM_SCALARS 8
OCPPO_API size_t ocppo_clip_adam_workspace_bytes(int64_t P);
/* n_planes (0..8) plane jobs: the new values of the row-major [plane_rows[j], plane_cols[j]]
 * weight at params + plane_offset[j] (offset % 4 == 0, cols % 4 == 0) are also written as the
 * three exact bf16 pieces ocppo_split_planes writes for it (trans as plane_trans[j]), piece p at
 * plane_dst[j] + p * rows * cols: the next update's GEMMs read them without a split launch. */
OCPPO_API int ocppo_clip_adam_step(ocppo_stream_t stream, float* params, const float* grads,
                                   float* exp_avg, float* exp_avg_sq, int64_t P, const float* lr,
                                   double beta1, double beta2, double eps, double grad_scale,
                                   double max_norm, float* scalars, void* workspace,
                                   size_t workspace_bytes, int n_planes,
                                   const int64_t* plane_offset, const int64_t* plane_rows,
                                   const int64_t* plane_cols, const int* plane_trans,
                                   void* const* plane_dst);

/* ---------------------------------------------------------------------------------------------
 * Rollout action head — replaces Categorical(logits).sample() / log_prob / entropy of
 * architectures/ppo.py:91-95 and the storage writes of ppo_atari_oc.py:506-510.
 * torch's sampler (Categorical.sample → multinomial(probs, 1, True)) draws q ~ Exp(1) of shape
 * [N, A] and returns argmax(probs / q); `noise` must be that q (e.g. from
 * torch.empty(N, A).exponential_() on the same generator), so actions are bit-identical.
 *   logits : [N, A] f32; noise : [N, A] f32
 *   action_out : [N] int64 (e.g. &actions[t*N]);  logprob_out : [N] f32 (&logprobs[t*N])
 *   entropy_out : [N] f32 or NULL
 *   value_in / value_out : critic output [N] copied into &values[t*N] (both NULL to skip)
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_categorical_sample(ocppo_stream_t stream, const float* logits, float* noise,
                             const int64_t* philox_state, int64_t philox_offset,
                             int64_t philox_stride, int64_t N, int64_t A, int64_t* action_out,
                             float* logprob_out, float* entropy_out, const float* value_in,
                             float* value_out);

/* The sampling entries' Exp(1) values (ocppo_categorical_sample, ocppo_policy_head_sample,
 * ocppo_policy_head_env_step) come from one of two places:
 *   philox_state == NULL : noise [N, A] is read (any source);
 *   philox_state != NULL : the kernel draws them itself, bit for bit the values
 *     torch.empty(N, A, device=...).exponential_() returns on the CUDA/HIP generator whose
 *     (seed, philox offset) is (philox_state[0], philox_state[1] + philox_offset) -- the stream
 *     Categorical.sample() consumes per step in the reference (architectures/ppo.py:92-94 via
 *     torch.multinomial's Exp(1) path; ppo_atari_oc.py:505-506) -- with philox_stride = torch's
 *     grid stride for N*A elements (ocppo_torch_exponential_geometry); noise, when non-NULL,
 *     receives them. philox_state is device memory [2] (graph-capturable: a replay reads the
 *     generator state of that replay). */

/* torch's launch geometry of exponential_ over `numel` elements (ATen DistributionTemplates.h
 * calc_execution_policy): the grid stride (256 * grid, grid <= cus * max_threads_per_cu / 256) and
 * the generator's philox-offset increment per draw. Host only. */
OCPPO_API int ocppo_torch_exponential_geometry(int64_t numel, int64_t cus, int64_t max_threads_per_cu,
                                               int64_t* stride, int64_t* offset_increment);

/* out[numel] = torch.empty(numel).exponential_() at generator (philox_state[0], philox_state[1] +
 * philox_offset), grid stride philox_stride (the reference stream of the sampling entries,
 * on its own: tests, and callers that need the draws as a tensor). */
OCPPO_API int ocppo_philox_exponential(ocppo_stream_t stream, float* out, int64_t numel,
                                       const int64_t* philox_state, int64_t philox_offset,
                                       int64_t philox_stride);
/* `steps` such draws back to back, as `steps` successive exponential_ calls of one shape make
 * them: out[t * numel + i] = element i of the draw at philox offset philox_offset + t * increment
 * (increment from ocppo_torch_exponential_geometry). One launch for a whole rollout's
 * Categorical.sample draws (the reference's per-step stream, ppo_atari_oc.py:505-506). */
OCPPO_API int ocppo_philox_exponential_steps(ocppo_stream_t stream, float* out, int64_t numel,
                                             int64_t steps, const int64_t* philox_state,
                                             int64_t philox_offset, int64_t increment,
                                             int64_t philox_stride);

/* Fused rollout policy head: logits = hidden @ w_actor^T + b_actor, value = hidden . w_critic +
 * b_critic, then the sampler above — replaces the actor/critic Linear layers AND the sampler of
 * architectures/ppo.py:89-95 for one rollout step (PPObj / PPODefault, shared hidden layer).
 *   hidden : [N, H] f32 (decoder output);  w_actor : [A, H];  b_actor : [A];  w_critic : [H];
 *   b_critic : [1];  noise : [N, A] Exp(1) (or drawn: philox_*, above);  value_out : [N];
 *   entropy_out, logits_out ([N, A]) may be NULL.
 * Logits differ from a GEMM's only by f32 summation order; actions are bit-exact w.r.t. the
 * sampler applied to the logits this kernel computes (returned in logits_out). */
OCPPO_API int ocppo_policy_head_sample(ocppo_stream_t stream, const float* hidden, int64_t N,
                                       int64_t H, const float* w_actor, const float* b_actor,
                                       const float* w_critic, const float* b_critic,
                                       float* noise, const int64_t* philox_state,
                                       int64_t philox_offset, int64_t philox_stride, int64_t A,
                                       int64_t* action_out, float* logprob_out,
                                       float* entropy_out, float* value_out, float* logits_out);

/* log_prob(action) and entropy() of Categorical(logits) for given actions (architectures/ppo.py
 * :92-95 with `action` passed) and the matching backward. */
OCPPO_API int ocppo_categorical_logprob_entropy(ocppo_stream_t stream, const float* logits,
                                      const int64_t* actions, int64_t N, int64_t A,
                                      float* logprob_out, float* entropy_out);
OCPPO_API int ocppo_categorical_logprob_entropy_bwd(ocppo_stream_t stream, const float* logits,
                                          const int64_t* actions, const float* grad_logprob,
                                          const float* grad_entropy, int64_t N, int64_t A,
                                          float* dlogits);

/* ---------------------------------------------------------------------------------------------
 * Rollout store — replaces ppo_atari_oc.py:502-503 and :512-514 (host float32 conversion,
 * pageable H2D copies and `obs[step] = next_obs`) with one device pass per env step that also
 * performs the frame stacking the reference does in N env subprocesses.
 *   frame      : [N, D] newest frame per env, dtype frame_dtype (OCPPO_F32 object vectors of
 *                OCAtari obj mode, D = F; or OCPPO_U8 grayscale 84x84 pixels, D = 7056)
 *   reward     : [N] f32;  done : [N] f32 (0/1)
 *   prev_obs   : [N, W, D] stacked obs of the previous step, dtype obs_dtype (rollout slot t)
 *   obs_out    : [N, W, D] new stacked obs, dtype obs_dtype (rollout slot t+1)
 *   net_obs    : f32 copy of obs_out for the network forward (may be NULL when net_layout = 0)
 *   reward_out : [N] f32 (&rewards[t*N]);  done_out : [N] f32 (&dones[(t+1)*N]); either may be NULL
 *   net_flags  : bit 0 (OCPPO_NET_CHANNELS_LAST): net_obs in channels-last order [N, D, W] (the
 *                NHWC input of a channels_last NatureCNN, 16-B aligned; MIOpen's NHWC
 *                convolutions then need no transpose), else [N, W, D] like obs_out;
 *                bit 1 (OCPPO_NET_SCALE_255): net_obs = value / 255 as ATen computes it
 *                (x * (1.0f / 255.0f)) -- the NatureCNN's NormalizeImg (architectures/common.py:19-22)
 *                folded into the store
 *   reset_prev : [N, W-1, D] frame_dtype or NULL: the older W-1 frames of the observation the env
 *                itself returned on a done (read for done rows only)
 * Stacking: obs_out[n] = prev_obs[n][1:] ++ frame[n]; on done[n] the older W-1 slots are
 * reset_prev[n] when given (a host env whose reset stack holds distinct frames: the reference's
 * NoopResetEnv/FireResetEnv step after reset, EpisodicLifeEnv signals done on a life loss without
 * resetting the stack, ppo_atari_oc.py:278-282), else frame[n] (the gymnasium FrameStack reset
 * fill). Conversion to bf16 is round-to-nearest-even and exact for the integer-valued obs of both
 * modes (|x| <= 256).
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_rollout_store(ocppo_stream_t stream, const void* frame, int frame_dtype,
                        const float* reward, const float* done, int64_t N, int64_t W, int64_t D,
                        const void* prev_obs, void* obs_out, int obs_dtype, float* net_obs,
                        float* reward_out, float* done_out, int net_flags, const void* reset_prev);

/* Fill a whole stacked-obs slot from one frame per env (env reset, ppo_atari_oc.py:464-465);
 * net_flags as in ocppo_rollout_store. */
OCPPO_API int ocppo_obs_reset(ocppo_stream_t stream, const void* frame, int frame_dtype, int64_t N,
                    int64_t W, int64_t D, void* obs_out, int obs_dtype, float* net_obs,
                    int net_flags);

/* ---------------------------------------------------------------------------------------------
 * Frame-encoding cache of the rollout forward (PPObj, architectures/ppo.py:60-84, whose encoder
 * is applied to each stacked frame on its own). `agent.get_action_and_value(next_obs)` at
 * ppo_atari_oc.py:506 re-encodes all W stacked frames every step although W-1 of them were
 * encoded at the previous steps under the same weights; with this entry point the caller encodes
 * only the newest frame and shifts the cache like the frame stack (same reset fill as
 * ocppo_rollout_store):
 *   enc[n, w, :] = done[n] != 0 || w == W-1 ? fresh[n, :] : enc[n, w+1, :]   (in place)
 * enc [N, W, E] f32, fresh [N, E] f32 with row stride ld_fresh (>= E), done [N] f32 or NULL.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_frame_cache_shift(ocppo_stream_t stream, float* enc, const float* fresh,
                            int64_t ld_fresh, const float* done, int64_t N, int64_t W, int64_t E);

/* ---------------------------------------------------------------------------------------------
 * Rollout-batch Linear(+ReLU): y[M, N] = act(x[M, K] @ w[N, K]^T + b[N]) in f32 on the matrix
 * cores (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation; summation order differs
 * from the BLAS library's). Replaces the nn.Linear(+nn.ReLU) layers of architectures/ppo.py:60-84
 * (PPObj) and the NatureCNN head :36-46 in the rollout forward of ppo_atari_oc.py:506, :534
 * (no autograd: the rollout runs under torch.no_grad()), where M is the number of envs (or envs x
 * frames) and the library's large tiles leave the chip idle.
 *   x : row stride ldx (>= K); w : nn.Linear weight, row-major [N, K]; b : [N] or NULL;
 *   y : row stride ldy (>= N); relu : 0 = identity, 1 = max(., 0) after the bias.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_linear_act(ocppo_stream_t stream, const float* x, int64_t ldx, const float* w,
                     const float* b, float* y, int64_t ldy, int64_t M, int64_t N, int64_t K,
                     int relu);

/* ---------------------------------------------------------------------------------------------
 * Linear(+ReLU) backward, elementwise part, in one pass — replaces the threshold_backward + bias
 * `sum(0)` pair autograd runs inside `loss.backward()` (ppo_atari_oc.py:605) for every
 * nn.Linear -> nn.ReLU of architectures/ppo.py:60-84 / :44-46:
 *   gp[r, n] = out[r, n] <= 0 ? 0 : g[r, n]   (out = the layer's ReLU output; out == NULL: no
 *                                             ReLU, gp unused and may be NULL)
 *   db[n]    = sum_r gp[r, n]                 (deterministic fixed-order reduction)
 * g/out/gp [R, N] f32 row-major, 16-B aligned, N % 4 == 0, N <= 16384; workspace 256-B aligned,
 * >= ocppo_relu_bias_grad_workspace_bytes(R, N), ZEROED before its first use (its tickets re-arm).
 * ------------------------------------------------------------------------------------------- */
/* Forward epilogue of a bias-less convolution / GEMM in NHWC / row-major layout, in place:
 *   y[r, n] = act(y[r, n] + b[n])   (act = ReLU when relu != 0; torch's conv + bias then ReLU,
 *                                    one f32 rounding for the add, architectures/ppo.py:20-31)
 * y [R, N] f32, b [N] f32, both 16-B aligned, N % 4 == 0. */
OCPPO_API int ocppo_bias_act(ocppo_stream_t stream, float* y, const float* b, int64_t R, int64_t N,
                   int relu);
/* The same epilogue with the output in NCHW order (the rollout's last NatureCNN convolution, whose
 * nn.Flatten reads NCHW, architectures/ppo.py:20-31): out[b, c, p] = act(y[b, p, c] + bias[c]),
 * y [B, P, C] NHWC f32 (P = H*W), out [B, C, P] f32 (not aliasing y), P * (C + 1) <= 12288. */
OCPPO_API int ocppo_bias_act_nchw(ocppo_stream_t stream, const float* y, const float* b, int64_t B,
                                  int64_t P, int64_t C, int relu, float* out);

/* ---------------------------------------------------------------------------------------------
 * Update-phase f32 GEMM on the bf16 matrix cores — replaces the f32 GEMMs (addmm /
 * _addmm_activation forward, g'W dX, split-K g'^T x dW) of the Linear layers that
 * `agent.get_action_and_value(b_obs[mb])` and `loss.backward()` run (ppo_atari_oc.py:566-606
 * through architectures/ppo.py:60-84):
 *   C_s[m, n] = act( sum_{k in K_s} A(m, k) B(n, k) + bias[n] )     s = 0 .. splits-1
 *   A(m, k) = a[m*sam + k*sak], B(n, k) = b[n*sbn + k*sbk], C_s[m, n] = c[s*split_c + m*ldc + n]
 *   K_s = steps [s*nk/splits, (s+1)*nk/splits) of the nk = K/32 steps of 32 (even partition)
 * Each f32 operand is split exactly into three bf16 pieces (x = x0 + x1 + x2) and the six piece
 * products down to 2^-24 of |a b| are accumulated in f32 (one accumulator per output with tile
 * bit 4 and the mixed tiles, the shipped forms; the small terms in a second one otherwise):
 * f32-level accuracy (tests/test_gemm_gpu.py: error vs f64 at or below
 * hipBLASLt's f32 GEMM) at 6 bf16 MFMAs per f32 multiply-add.
 * One of (sam, sak) and one of (sbn, sbk) must be 1 (the other a multiple of 4, >= the extent it
 * strides over); a, b 16-B aligned; K % 32 == 0, K / 32 >= splits; M, N multiples of the tile (tile 0: 128 x 128,
 * 1: 64 x 128, 2: 128 x 64, 3: 64 x 64 rows x columns); bias (NULL: none) and relu only with
 * splits == 1. Mask epilogue (mask != NULL; the dX product of the layer above a Linear+ReLU,
 * whose input `mask` [M, N] (row stride ldm) is that ReLU's output): C = mask > 0 ? acc : 0
 * (threshold_backward) and dbp[tm, n] = sum of C over row tile tm (tile rows each) — that layer's
 * bias-gradient partials, [M / tile rows, N], for ocppo_sum_splits_db; splits == 1, no bias/relu.
 * ReLU bitmask (mbits: (M / tile rows) x (N / tile columns) x threads per workgroup (256, or 512
 * for the 8-wave shapes) 64-bit words): a forward with relu writes, per tile and thread, one word
 * of !(output <= 0) bits in the MFMA fragment order (mbits_out); the mask
 * epilogue of a later dX over the same [M, N] with the same tile reads them (mbits_in, mask may
 * then be NULL) instead of the f32 mask. tile: bits 0-2 the tile shape (0: 128 x 128, 1: 64 x
 * 128, 2: 128 x 64, 3: 64 x 64 with 4 waves; 4-7: 8-wave forms), bit 3 loads two K steps ahead,
 * bit 4 one accumulator for all six products. tile 56 (bit 5: mixed tiles; splits == 1): rows
 * [0, mbig) in 128 x 128 tiles dispatched first, rows [mbig, M) in 64 x 128 tiles — mbig chosen
 * by the library (one 128 x 128 tile per CU when the output holds 257..384 of them, else all of
 * M) when mbig is -1; mbig >= 0 imposes the split (a multiple of 128, (mbig / 128)(N / 128) a
 * multiple of 8; experiments and tests); mbig must be -1 for every other tile. M, N multiples of
 * 64 x 128, and dbp rows / mbits words counted as for 64 x 128 (a 128-row tile's dbp partial sits in the first of its two rows, the second is written as zeros).
 * Pre-split B (b_planes != NULL; b is then ignored and may be NULL): the three bf16 pieces of
 * B(n, k) at b_planes[p * bp_stride + n * bp_ld + k] (p = 0, 1, 2; ocppo_split_planes wrote them
 * from the f32 B, so the result is bitwise that of the f32 B): staged by copy, no split in the
 * K loop. Needs sak == 1, bp_ld % 8 == 0, 16-B aligned planes, tile 24..27, 56, 57 or 58.
 * relu | OCPPO_X6_MBITS_ROWS (with relu and mbits_out): mbits_out is row-major instead,
 * (M x N / 32) 32-bit words, bit n % 32 of word [m][n / 32] = !(C[m, n] <= 0) — for a consumer
 * that walks the output by rows (ocppo_frames_scatter_relu's mbits).
 * Tiles 57-60 (the pipelined family): 256 x 128, 128 x 256 (8 waves), 128 x 128 (4 waves) and
 * 128 x 128 (8 waves) with two LDS stages and one barrier per K step (the next step's operand
 * split in the MFMAs' shadow); one workgroup per CU.
 * Deterministic (fixed MFMA order, no atomics).
 * ------------------------------------------------------------------------------------------- */
#define OCPPO_X6_MBITS_ROWS 2
OCPPO_API int ocppo_gemm_x6(ocppo_stream_t stream, const float* a, int64_t sam, int64_t sak,
                            const float* b, int64_t sbn, int64_t sbk, float* c, int64_t ldc,
                            int64_t M, int64_t N, int64_t K, int64_t splits, int64_t split_c,
                            const float* bias, int relu, const float* mask, int64_t ldm,
                            float* dbp, uint64_t* mbits_out, const uint64_t* mbits_in,
                            int tile, int mbig, const void* b_planes, int64_t bp_ld,
                            int64_t bp_stride, void* sk_workspace, size_t sk_workspace_bytes);

/* Bytes of the stream-K workspace of a pipelined tile (57, 58; 0 for every other tile). With
 * sk_workspace != NULL ocppo_gemm_x6 runs a pipelined product (tiles 57 / 58: 256 x 128 /
 * 128 x 256, two LDS stages, one workgroup per CU) as a persistent stream-K launch: the tiles are
 * dealt to the 8 XCDs, each XCD's CUs share its tiles' K steps in equal contiguous ranges, and a
 * tile split between two workgroups is finished by the one holding its first K steps, after the
 * later parts' partial accumulators arrive through the workspace (same XCD, so its L2) — every
 * CU busy to the end at any tile count. splits == 1; the workspace must be 256-B aligned and
 * zero before the first launch (its flags return to zero after every launch). Same products in
 * the same order within a part; the parts are added in K order: deterministic. */
OCPPO_API size_t ocppo_gemm_x6_sk_workspace_bytes(int tile);

/* ---------------------------------------------------------------------------------------------
 * ocppo_gemm_x6 with one operand's rows read through a row table (the update's decoder on the
 * Flatten of the stacked frame encodings, architectures/ppo.py:77-80, without materialising the
 * [M, W * E] input of ppo_atari_oc.py:566's b_obs[mb_inds] forward):
 *   mode 1: A(m, k) = a[gidx[m * gw + k / gseg] * sam + k % gseg]   (sak == 1, K == gw * gseg,
 *           every split's K range inside one segment: gseg % (K / splits) == 0)
 *   mode 2: B(n, k) = b[gidx[k * gw + n / gseg] * sbk + n % gseg]   (sbn == 1, N == gw * gseg,
 *           gseg % 128 == 0, K / splits <= 1024; A m-contiguous, as a weight gradient's g'^T)
 * gidx int32 (mode 1: [M, gw], mode 2: [K, gw]; e.g. ocppo_frames_expand_index). The 128 x 128
 * tile (variant 24), M % 128 == N % 128 == 0, (K / 32) % splits == 0; bias / ReLU only with
 * splits == 1; b_planes (mode 1) as ocppo_gemm_x6's. Bitwise ocppo_gemm_x6 on the gathered
 * operand written out.
 * ------------------------------------------------------------------------------------------- */
/* ---------------------------------------------------------------------------------------------
 * The dX product of a layer above a Linear+ReLU whose input needs no gradient, with that lower
 * layer's whole backward in the epilogue (the PPObj encoder's second layer above the first,
 * ppo_atari_oc.py:605 through architectures/ppo.py:60-84): with C = A B as ocppo_gemm_x6 (A = g'
 * [M, K] k-contiguous, B(n, k) = W[k, n] n-contiguous: dX = g' W), gp = mask > 0 ? C : 0 (mask
 * [M, N] = the lower layer's ReLU output, row stride ldm) is never stored; instead
 *   db[n] = sum_m gp[m, n],   dw[n, k1] = sum_m gp[m, n] x[m, k1]   (x [M, K1], K1 <= 16)
 * are formed as per-row-tile records in `records` (>= (M / tile rows) * ceil(N / 256) * 256 *
 * (K1 padded to 4 / 8 / 12 / 16, + 1) floats) and finished later from *finish (as
 * ocppo_relu_bias_wgrad_rows': ocppo_sum_splits_db_finish or ocppo_deferred_finish_run).
 * tile 27 (64 x 64) or 24 (128 x 128); M, N multiples of the tile, K % 32 == 0. Deterministic.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_gemm_x6_wgrad(ocppo_stream_t stream, const float* a, int64_t sam, int64_t sak,
                                  const float* b, int64_t sbn, int64_t sbk, int64_t M, int64_t N,
                                  int64_t K, const float* mask, int64_t ldm, const float* x,
                                  int64_t ldx, int64_t K1, float* dw, float* db, float* records,
                                  int64_t records_floats, int tile,
                                  ocppo_deferred_finish_t* finish);
OCPPO_API int ocppo_gemm_x6_gather(ocppo_stream_t stream, const float* a, int64_t sam, int64_t sak,
                                   const float* b, int64_t sbn, int64_t sbk, float* c, int64_t ldc,
                                   int64_t M, int64_t N, int64_t K, int64_t splits,
                                   int64_t split_c, const float* bias, int relu,
                                   const void* b_planes, const int32_t* gidx, int64_t gw,
                                   int64_t gseg, int mode);

/* ---------------------------------------------------------------------------------------------
 * NHWC convolution (no padding, square stride) as an implicit GEMM on ocppo_gemm_x6's exact
 * three-piece bf16 products (the NatureCNN trunk, cleanrl/architectures/ppo.py:20-31: replaces
 * the convolution forward / backward cuDNN (MIOpen) runs for nn.Conv2d at ppo_atari_oc.py:506
 * and :566-606; deterministic: no atomics, split-K partials summed in split order). No im2col
 * buffer: the convolution rows r = (b, qy, qx) over [B, qh, qw] read element k of their kernel
 * window at x[b sb + qy ys + qx xs + (k / gseg) segs + k % gseg], geom = {qh, qw, sb, ys, xs,
 * segs, gseg} (floats; a segment = one kernel row's KW x C taps, contiguous in NHWC; all strides
 * multiples of 4, x and w 16-B aligned, B qh qw < 2^24).
 *   mode 0 (forward; and each stride class of the data gradient, over the zero-padded output
 *          gradient with the flipped weight): c[row(r) + n] = act(sum_k x(r, k) w[n ldw + k] +
 *          bias[n]) for r < M = B qh qw, n < N, k < K; gseg % 32 == 0; splits > 1 (no bias,
 *          ReLU or out_geom, ldc == N): K-split partials [splits, M, N] in c instead; row(r) =
 *          r ldc, or b sb' + qy ys' + qx xs' + off' with out_geom = {sb', ys', xs', off', cw,
 *          cs, cy, cx}, column n then at row(r) + (c / cs) cy + (c % cs) cx + n % cw, c = n / cw
 *          (all stride classes of a data gradient in one product: they read the same rows).
 *   mode 1 (weight gradient): out[m, n] = sum_r w[r ldw + m] x(r, n) (w = the output gradient
 *          [rows, ldw], m < M = Cout, n < N = KH KW C, r < K = B qh qw); c = split partials
 *          [splits, M, N], then summed in split order (f64, one rounding) into out; qh qw <= 1024.
 * mask (mode 0, or null; needs dbp, no bias / ReLU): the layer below's ReLU backward in the
 * epilogue, c = mask > 0 ? acc : 0 with mask in c's layout, and each row tile's column sums of c
 * in dbp [M / tile rows, N] (that layer's bias-gradient partials).
 * pad (mode 0, or null): {ph, pw, ih, iw, C}: x is the UNPADDED [B, ih, iw, C] tensor that the
 * rows index as if zero-padded by ph rows / pw columns on each side (the data gradient's padded
 * output gradient, never materialised; geom's qh, qw, gseg as for the padded one; tile 2, 3,
 * 5 or 6).
 * tile: 0 = 128 x 32, 2 = 128 x 64, 3 = 64 x 64, 5 = 128 x 128, 6 = 32 x 64 (mode 0); 1 =
 * 32 x 128, 3, 4 =
 * 64 x 128, 5 (mode 1); M, N multiples of it; K % 32 == 0, K / 32 >= splits.
 * tile 7 (mode 0, ABI 27): few rows (the rollout's batch) -- a 32-row tile per workgroup with its
 * K steps split over 8 waves and summed in wave order; N = 32 or 64, 32 | M, splits 1, no
 * out_geom / pad / mask; the same x6 products per K step, grouped differently over K (not the
 * other tiles' bits). w_planes (mode 0, else null; 16-B aligned, K % 8 == 0): w's three bf16
 * pieces [3, N, K] (ocppo_split_planes of w), read instead of splitting w in every workgroup
 * (the same pieces: the same bits). mbits_rows (ABI 28; mode 0 with relu, splits 1, no out_geom /
 * pad / mask, ldc == N, 32 | N, tiles 0, 2, 3, 5, 6; else null): the output's ReLU mask as a
 * row-major bitmask u32 [M, N / 32], bit n % 32 of word m N / 32 + n / 32 = !(c[m, n] <= 0) --
 * read by ocppo_relu_bias_grad_bits instead of the f32 output.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_conv_x6(ocppo_stream_t stream, int mode, const float* x, const int64_t* geom,
                            const float* w, int64_t ldw, float* c, int64_t ldc, int64_t M,
                            int64_t N, int64_t K, int64_t splits, const float* bias, int relu,
                            const int64_t* out_geom, int tile, float* out, const int64_t* pad,
                            const float* mask, float* dbp, const uint16_t* w_planes,
                            uint32_t* mbits_rows);

/* ---------------------------------------------------------------------------------------------
 * The first NatureCNN convolution straight from the rollout's u8 frame stacks (ppo_atari_oc.py:566
 * `b_obs[mb_inds]` -> NormalizeImg -> Conv2d, architectures/ppo.py:17-21), without the f32
 * minibatch copy: sample b's stack is row idx[b] of src u8 [rows, C, H, W] (NCHW); taps k = (c,
 * ky, kx) in nn.Conv2d's weight order (w [N, ldw] row-major, k-contiguous). The bytes are exact
 * bf16 operands; the products are divided by `divisor` (255.0: NormalizeImg's x / 255).
 *   mode 0: c[r, n] = act(sum_k u(r, k) w[n, k] / divisor + bias[n]), r < M = B OH OW (c [M, N])
 *   mode 1: out[m, n] = sum_r w[r ldw + m] u(r, n) / divisor (w = the output gradient [K, ldw],
 *           N = C KH KW taps, K = B OH OW rows); c = split partials [splits, M, N], summed in
 *           split order in f64 and divided once.
 * KW, W, stride multiples of 4; no padding; tile 0 / 2 (mode 0), 1 / 4 (mode 1) as ocppo_conv_x6's.
 * tile 7 (mode 0, ABI 25): each image's stack staged in LDS once, bitwise tile 0's output; needs
 * C = 4, 8 x 8 taps, stride 4, N = 32, 16 | OH OW, src 16-B aligned, 16 | C H W, 2 C H W <= 64 KB
 * (NatureCNN's first layer on 4 x 84 x 84 stacks); M a whole number of images, splits 1.
 * tile 8 (mode 1, ABI 25): the weight gradient with each image's stack staged in LDS once; needs
 * 4 x 84 x 84 stacks, 8 x 8 taps, stride 4, M = 32, K a whole number of images, a 16-B aligned
 * src; runs splits / 4 workgroups, each writing 4 partials into c [splits, M, N] (summed in
 * order in f64 and divided once, as the tile loop's); not the tile loop's summation order.
 * mbits (ABI 26, tiles 7 and 8 only, else null; 16-B aligned u32 [M] / [K]): tile 7 (with relu)
 * writes the output's ReLU mask, bit n of word r = c[r, n] > 0; tile 8 reads it and takes w as
 * the UNMASKED output gradient, zeroing it where the bit is clear (relu_bias_grad's ReLU
 * backward, ppo_atari_oc.py:603's loss.backward through nn.ReLU; the same products as on the
 * masked gradient). dbp / db (tile 8, both or neither): dbp workspace [splits, 32], db [32] the
 * (masked) gradient's per-channel sums = the layer's bias gradient (summed in order in f64).
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_conv_x6_u8(ocppo_stream_t stream, int mode, const uint8_t* src,
                               const int64_t* idx, int64_t C, int64_t H, int64_t W, int64_t KH,
                               int64_t KW, int64_t stride, const float* w, int64_t ldw, float* c,
                               int64_t M, int64_t N, int64_t K, int64_t splits, const float* bias,
                               int relu, float divisor, int tile, float* out, uint32_t* mbits,
                               float* dbp, float* db);

/* ---------------------------------------------------------------------------------------------
 * The exact three-piece bf16 split ocppo_gemm_x6 forms in its K loop, done once per matrix: the
 * update's Linear weights (architectures/ppo.py:60-84) as the B operand of the forward (W [N, K],
 * trans 0) and of dX (W^T, trans 1), after every optimizer step (ppo_atari_oc.py:606) instead of
 * once per row tile and K step. Job i: src[i] f32 [rows, cols] (row stride ld) -> dst[i] three
 * dense bf16 planes [R', C'] (R' x C' = rows x cols, or cols x rows transposed), plane stride
 * R' C' elements; C' % 8 == 0, dst 16-B aligned; 1 <= n <= 8 jobs, one launch.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_split_planes(ocppo_stream_t stream, int n, const float* const* src,
                                 const int64_t* ld, const int64_t* rows, const int64_t* cols,
                                 const int* trans, void* const* dst);

/* ---------------------------------------------------------------------------------------------
 * Split-K combine of a weight gradient — replaces ATen's `sum(0)` after the batched (split-K)
 * weight-gradient GEMM dW = g'^T x the build runs inside `loss.backward()` (ppo_atari_oc.py:605)
 * for the Linear layers of architectures/ppo.py:60-84:
 *   out[i] = part[0*n + i] + part[1*n + i] + ... + part[(S-1)*n + i]   (left fold, split order,
 *            in double, rounded once to float)
 * part [S, n] f32, out [n] f32 (e.g. the parameter's view in the flat grad buffer); both 16-B
 * aligned, n % 4 == 0, S in {1, 2, 4, 8, 16}. Deterministic.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_sum_splits(ocppo_stream_t stream, const float* part, int64_t S, int64_t n,
                     float* out);
/* Split-K combine of a forward product with its epilogue — the decoder forward of the update
 * (architectures/ppo.py:77-80 inside ppo_atari_oc.py:566) as ocppo_gemm_x6 K splits:
 *   out[m, n] = act(sum_s part[s, m, n] + bias[n])   (part [S, M, N], out [M, N] f32 row-major;
 * the splits added in split order in double, rounded once, then + bias, then ReLU if relu —
 * torch._addmm_activation's order). bias [N] or NULL; 16-B aligned; N % 4 == 0. */
OCPPO_API int ocppo_sum_splits_act(ocppo_stream_t stream, const float* part, int64_t S, int64_t M,
                                   int64_t N, const float* bias, int relu, float* out);
OCPPO_API size_t ocppo_relu_bias_grad_workspace_bytes(int64_t R, int64_t N);
OCPPO_API int ocppo_relu_bias_grad(ocppo_stream_t stream, const float* g, const float* out,
                         float* gp, float* db, int64_t R, int64_t N, void* workspace,
                         size_t workspace_bytes);
/* ocppo_relu_bias_grad with the ReLU mask read from a row-major bitmask (ABI 28): gp[r, n] =
 * bit(r, n) ? g[r, n] : 0 with bit(r, n) = bit n % 32 of mbits[r N / 32 + n / 32] (the forward
 * epilogue's ocppo_conv_x6 mbits_rows: the same rule as out <= 0 -> 0), db = sum_r gp[r, n].
 * R >= 1, 32 | N <= 16384; g / gp 16-B aligned; workspace as ocppo_relu_bias_grad's. */
OCPPO_API int ocppo_relu_bias_grad_bits(ocppo_stream_t stream, const float* g,
                                        const uint32_t* mbits, float* gp, float* db, int64_t R,
                                        int64_t N, void* workspace, size_t workspace_bytes);

/* ---------------------------------------------------------------------------------------------
 * First-layer backward in ONE pass — replaces threshold_backward + the split-K weight-gradient
 * GEMM + the bias sum autograd runs inside `loss.backward()` (ppo_atari_oc.py:605) for a
 * Linear(+ReLU) layer whose input needs no gradient and has K <= 16 features (the PPObj
 * encoder's first layer on the object frames, architectures/ppo.py:60-84):
 *   gp[r, n] = out[r, n] <= 0 ? 0 : g[r, n]   (g itself when out == NULL; gp is not written)
 *   db[n]    = sum_r gp[r, n]
 *   dw[n, k] = sum_r gp[r, n] * x[r, k]        (dw [N, K] row-major, nn.Linear.weight layout)
 * g/out [R, N] f32 row-major 16-B aligned, N % 4 == 0, N <= 16384; x [R, K] f32, row stride ldx;
 * 1 <= K <= 16. Workspace 256-B aligned, >= ocppo_relu_bias_wgrad_workspace_bytes(R, N, K),
 * ZEROED before its first use (tickets re-arm). Deterministic (fixed-order sums, f32 fma).
 * ------------------------------------------------------------------------------------------- */
/* Deferred form: gp as above, db left as per-chunk column partials partials[chunks, N]
 * (chunks = ocppo_relu_bias_grad_chunks(R, N)), summed later in chunk order by
 * ocppo_sum_splits_db in the launch that combines the layer's split-K weight gradient: no
 * cross-workgroup hand-off inside this launch. */
OCPPO_API int64_t ocppo_relu_bias_grad_chunks(int64_t R, int64_t N);
OCPPO_API int ocppo_relu_bias_grad_partial(ocppo_stream_t stream, const float* g, const float* out,
                                           float* gp, float* partials, int64_t R, int64_t N);
/* ocppo_sum_splits (out = sum of the S split-K blocks) + db[j] = sum_c db_partials[c, j] (a fixed
 * order) in one launch, both folds in double, rounded once; n, N multiples of 4, all pointers
 * 16-B aligned. */
OCPPO_API int ocppo_sum_splits_db(ocppo_stream_t stream, const float* part, int64_t S, int64_t n,
                                  float* out, const float* db_partials, int64_t chunks, int64_t N,
                                  float* db);
OCPPO_API size_t ocppo_relu_bias_wgrad_workspace_bytes(int64_t R, int64_t N, int64_t K);
OCPPO_API int ocppo_relu_bias_wgrad(ocppo_stream_t stream, const float* g, const float* out,
                          const float* x, int64_t ldx, float* dw, float* db, int64_t R,
                          int64_t N, int64_t K, void* workspace, size_t workspace_bytes);
/* Deferred form: the rows launch only; the finish (the tree over the row-range records that
 * writes dw and db) goes into *finish (R >= 1), to ride in the split-K combine the backward runs
 * next (ocppo_sum_splits_db_finish = ocppo_sum_splits_db, bitwise, plus the finish workgroups in
 * the same launch) or alone (ocppo_deferred_finish_run). Same results as ocppo_relu_bias_wgrad,
 * bitwise; run once, before anything reads dw / db or reuses the workspace. */
OCPPO_API int ocppo_relu_bias_wgrad_rows(ocppo_stream_t stream, const float* g, const float* out,
                                         const float* x, int64_t ldx, float* dw, float* db,
                                         int64_t R, int64_t N, int64_t K, void* workspace,
                                         size_t workspace_bytes, ocppo_deferred_finish_t* finish);
OCPPO_API int ocppo_sum_splits_db_finish(ocppo_stream_t stream, const float* part, int64_t S,
                                         int64_t n, float* out, const float* db_partials,
                                         int64_t chunks, int64_t N, float* db,
                                         const ocppo_deferred_finish_t* finish);

/* ---------------------------------------------------------------------------------------------
 * Policy heads + decoder ReLU backward in ONE pass — replaces, inside `loss.backward()`
 * (ppo_atari_oc.py:605), the actor / critic heads' dX, dW and db (architectures/ppo.py:81-84)
 * and the ReLU-backward + bias grad of the decoder layer feeding them. With
 * c[m] = (dlogits[m, 0..A), dvalue[m]) and W = [wa; wc] ([A+1, H]):
 *   dh[m, j] = sum_k c[m, k] W[k, j];  gp[m, j] = relu && h[m, j] <= 0 ? 0 : dh[m, j]
 *   db_h[j]  = sum_m gp[m, j]   (skipped when db_h == NULL)
 *   dwa[a, j] = sum_m dlogits[m, a] h[m, j];  dwc[j] = sum_m dvalue[m] h[m, j]
 *   dba[a] = sum_m dlogits[m, a];  dbc[0] = sum_m dvalue[m]
 * h / gp [M, H] f32 row-major 16-B aligned, H % 4 == 0, H <= 16384; dlogits [M, A] and dvalue
 * [M] contiguous, 1 <= A <= 7; wa [A, H], wc [H]. wc, dvalue, dwc and dbc may all be NULL: one
 * head only (K = A rows of W; e.g. the DQN Q head of dqn_atari_oc.py:378-392). Workspace 256-B
 * aligned, >=
 * ocppo_heads_bwd_workspace_bytes(M, H, A), ZEROED before first use. Deterministic.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API size_t ocppo_heads_bwd_workspace_bytes(int64_t M, int64_t H, int64_t A);
OCPPO_API int ocppo_heads_bwd(ocppo_stream_t stream, const float* h, const float* dlogits,
                    const float* dvalue, const float* wa, const float* wc, float* gp,
                    float* db_h, float* dwa, float* dwc, float* dba, float* dbc, int64_t M,
                    int64_t H, int64_t A, int relu, void* workspace, size_t workspace_bytes);

/* Two rollout Linear(+ReLU) layers in one launch (the PPObj encoder's first two layers on the
 * newest frame of every env, architectures/ppo.py:60-84, under torch.no_grad()):
 *   y[M, N2] = act2(act1(x[M, K1] @ w1[N1, K1]^T + b1) @ w2[N2, N1]^T + b2)
 * K1 <= 64, N1 % 16 == 0 and N1 <= 512; x row stride ldx (>= K1), y row stride ldy (>= N2);
 * w2 16-B aligned; b1 / b2 may be NULL. Same f32-MFMA arithmetic as ocppo_linear_act per layer. */
OCPPO_API int ocppo_linear2_act(ocppo_stream_t stream, const float* x, int64_t ldx, const float* w1,
                      const float* b1, const float* w2, const float* b2, float* y, int64_t ldy,
                      int64_t M, int64_t N1, int64_t N2, int64_t K1, int relu1, int relu2);

/* ---------------------------------------------------------------------------------------------
 * Frame-deduplicated PPObj minibatch encoder — replaces the per-slot encoder work inside
 * `agent.get_action_and_value(b_obs[mb_inds], ...)` of ppo_atari_oc.py:566 for the PPObj network
 * (architectures/ppo.py:60-84: Linear on the last dim of every stacked frame). Slot k of the
 * stored obs[t, n] ([T+1, N, W, F], step-major) is env n's frame of step max(t-(W-1)+k, r), r the
 * latest reset in (t-(W-1), t] (dones[r, n] = 1); its timeline id is u = (s+W-1)*N + n.
 *   frames_gather : x_out[c, :] = f32(frame uniq[c]) for the C (padded: id -1 -> zeros) distinct
 *                   frames of one minibatch;
 *   frames_expand : h_out[i, k, :] = enc[pos_of[u(perm[i], k)], :]  ([M, W, E], the decoder input);
 *   frames_scatter: denc[c, :] = sum of dh[i, k, :] over the uses of frame uniq[c] by the samples
 *                   of minibatch `mb` (inv[b] = position of sample b in the epoch permutation;
 *                   sample b belongs to minibatch inv[b] / M), fixed order -> deterministic.
 * W <= 16; dones [T+1, N] f32 with row r = "obs[r] starts an episode".
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_frames_gather(ocppo_stream_t stream, const void* obs, int obs_dtype, int64_t T,
                        int64_t N, int64_t W, int64_t F, const int32_t* uniq, int64_t C,
                        float* x_out);
OCPPO_API int ocppo_frames_expand(ocppo_stream_t stream, const float* enc, int64_t C, int64_t E,
                        const int32_t* pos_of, const int64_t* perm, int64_t M, const float* dones,
                        int64_t T, int64_t N, int64_t W, float* h_out);
/* frames_expand's source rows only: idx[i, k] = pos_of[u(perm[i], k)] ([M, W] int32), the row
 * table ocppo_gemm_x6's gathered operands read (the decoder's input never materialised). */
OCPPO_API int ocppo_frames_expand_index(ocppo_stream_t stream, const int32_t* pos_of,
                                        const int64_t* perm, int64_t M, const float* dones,
                                        int64_t T, int64_t N, int64_t W, int32_t* idx);
OCPPO_API int ocppo_frames_scatter(ocppo_stream_t stream, const float* dh, int64_t M, int64_t E,
                         const int32_t* uniq, int64_t C, const int32_t* inv, int64_t mb,
                         const float* dones, int64_t T, int64_t N, int64_t W, float* denc_out);
/* frames_scatter with the encoder's last ReLU backward fused in (the update's `loss.backward()`
 * through architectures/ppo.py:60-84's last Linear->ReLU, ppo_atari_oc.py:605):
 *   gp_out[c, :] = out[c, :] <= 0 ? 0 : denc[c, :]   (out = that layer's ReLU output [C, E];
 *                                                     NULL: no mask, gp_out = denc)
 *   dbp[g, :] = sum of gp_out rows of chunk g (ocppo_frames_scatter_chunks(C) chunks of 16 frames,
 *               summed later in chunk order by ocppo_sum_splits_db); NULL: not written.
 * mbits (NULL: none): the mask as the row-major ReLU bitmask ocppo_gemm_x6 wrote for `out`
 * (relu | OCPPO_X6_MBITS_ROWS, [C][E / 32] words, E % 32 == 0) instead of reading out (then
 * ignored): 1 bit instead of 4 B per element, the same gp_out.
 * E % 4 == 0, dh / out / gp_out / dbp 16-B aligned. Same per-frame sums as frames_scatter. */
OCPPO_API int64_t ocppo_frames_scatter_chunks(int64_t C);
OCPPO_API int ocppo_frames_scatter_relu(ocppo_stream_t stream, const float* dh, int64_t M,
                                        int64_t E, const int32_t* uniq, int64_t C,
                                        const int32_t* inv, int64_t mb, const float* dones,
                                        int64_t T, int64_t N, int64_t W, const float* out,
                                        const uint32_t* mbits, float* gp_out, float* dbp);
/* frames_gather + the encoder's first Linear(+ReLU) in one pass (the update's first encoder layer
 * over the distinct frames, architectures/ppo.py:60-84 on b_obs[mb_inds], ppo_atari_oc.py:566) (F <= 16, N1 % 4 == 0,
 * N1 <= 1024): x_out [C, F] = the gathered frames (as frames_gather),
 * h_out [C, N1] = act(x W^T + b)
 * (w [N1, F], b [N1] or NULL; products summed over f in order, then + b, then ReLU if relu).  idx_out (NULL: none): also ocppo_frames_expand_index(pos_of, perm, M, dones, T, N, W) into
 * idx_out [M, W], made by extra workgroups of the same launch (the row table the update's gathered
 * decoder reads; one launch instead of two). */
OCPPO_API int ocppo_frames_gather_linear(ocppo_stream_t stream, const void* obs, int obs_dtype,
                                         int64_t T, int64_t N, int64_t W, int64_t F,
                                         const int32_t* uniq, int64_t C, const float* w,
                                         const float* b, int64_t N1, int relu, float* x_out,
                                         float* h_out, const int32_t* pos_of,
                                         const int64_t* perm, int64_t M, const float* dones,
                                         int32_t* idx_out);

/* ---------------------------------------------------------------------------------------------
 * Minibatch gather — replaces `b_obs[mb_inds]` of ppo_atari_oc.py:566-567:
 *   dst[i, :] = f32(src[idx[i], :]),  src [B, R] of dtype src_dtype, dst [M, R] f32.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_gather_rows(ocppo_stream_t stream, const void* src, int src_dtype, const int64_t* idx,
                      int64_t M, int64_t R, float* dst);

/* The same gather into channels-last rows (the NHWC input of a channels_last NatureCNN):
 *   dst[i, p, c] = f32(src[idx[i], c, p]) (/ 255 with OCPPO_NET_SCALE_255 in net_flags, as in
 *   ocppo_rollout_store),  src [B, C, P] (C stacked frames of P pixels), dst [M, P, C] f32,
 *   16-B aligned. */
OCPPO_API int ocppo_gather_rows_cl(ocppo_stream_t stream, const void* src, int src_dtype,
                         const int64_t* idx, int64_t M, int64_t C, int64_t P, float* dst,
                         int net_flags);

/* ---------------------------------------------------------------------------------------------
 * Reward normalisation of SB3 VecNormalize(norm_obs=False, norm_reward=True) as wrapped at
 * ppo_atari_oc.py:414 (stable-baselines3 2.0.0, not in the reference tree), on device in f64:
 *   ret = ret*gamma + r;  rms.update(ret) (batch mean/var over N, Chan merge);
 *   r' = clip(r / sqrt(rms.var + epsilon), -clip, clip);  ret[done] = 0
 *   ret_state : [N] f64;  rms_state : [3] f64 = {mean, var, count} (init {0, 1, 1e-4})
 *   reward_out : [N] f32 (may alias nothing; typically &rewards[t*N])
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_vecnorm_reward(ocppo_stream_t stream, const float* reward, const float* done, int64_t N,
                         double gamma, double epsilon, double clip_reward, double* ret_state,
                         double* rms_state, float* reward_out);

/* Rollout store and VecNormalize reward normalisation in ONE launch (one workgroup normalises the
 * N rewards, the others store): ocppo_rollout_store (reward_out unused) + ocppo_vecnorm_reward.
 * reward_out (normalised, typically &rewards[t*N]) must not alias reward. */
OCPPO_API int ocppo_rollout_store_vecnorm(ocppo_stream_t stream, const void* frame, int frame_dtype,
                                          const float* reward, const float* done, int64_t N,
                                          int64_t W, int64_t D, const void* prev_obs, void* obs_out,
                                          int obs_dtype, float* net_obs, float* done_out,
                                          double gamma, double epsilon, double clip_reward,
                                          double* ret_state, double* rms_state, float* reward_out, int net_flags,
                                          const void* reset_prev);

/* ---------------------------------------------------------------------------------------------
 * DQN (config 5, dqn_atari_oc.py) — HBM replay buffer with stable-baselines3 2.0.0
 * ReplayBuffer(optimize_memory_usage=True, handle_timeout_termination=False) semantics
 * (:317-325 add at :369, sample at :377), epsilon-greedy (:345-350) and the fused TD target +
 * MSE loss forward/backward (:378-382). Replay layout: obs [size, E, D] (storage dtype),
 * actions [size, E] i64, rewards/dones [size, E] f32, state = device i64 {pos, full} (zeroed).
 * Sampling law = SB3's (indices in [0, pos) or (randint(1, size) + pos) % size once full, env
 * index uniform); random bits from a counter-based stream (device counter, +1 per call), not numpy.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API size_t ocppo_replay_workspace_bytes(void);
OCPPO_API int ocppo_replay_add(ocppo_stream_t stream, const void* obs, const void* next_obs,
                               int obs_dtype, const int64_t* actions, const float* rewards,
                               const float* dones, int64_t E, int64_t D, int64_t* state,
                               int64_t size, void* rb_obs, int rb_dtype, int64_t* rb_actions,
                               float* rb_rewards, float* rb_dones, void* workspace);
/* obs_out / next_obs_out : [B, D] f32; indices_out : [B, 2] {slot, env} or NULL */
OCPPO_API int ocppo_replay_sample(ocppo_stream_t stream, uint64_t seed, int64_t* counter,
                                  const int64_t* state, int64_t size, int64_t E, int64_t D,
                                  const void* rb_obs, int rb_dtype, const int64_t* rb_actions,
                                  const float* rb_rewards, const float* rb_dones, int64_t B,
                                  float* obs_out, float* next_obs_out, int64_t* actions_out,
                                  float* rewards_out, float* dones_out, int64_t* indices_out);
/* global step t = *step + step_offset (step : device i64, so a captured chunk of env steps
 * reads one counter advanced once per chunk); epsilon_out : device f32 or NULL */
/* the Q head (q = hidden Wq^T + bq, hidden [E, H] H a multiple of 256 <= 1024, wq [A, H], A <= 8)
 * and ocppo_epsilon_greedy on it in one launch (same coin, argmax rule and random action);
 * q_out [E, A] or NULL */
OCPPO_API int ocppo_q_head_epsilon_greedy(ocppo_stream_t stream, const float* hidden, int64_t E,
                                          int64_t H, const float* wq, const float* bq, int64_t A,
                                          uint64_t seed, const int64_t* step, int64_t step_offset,
                                          double start_e, double end_e, double duration,
                                          int64_t* actions, float* epsilon_out, float* q_out);
/* One acting step of the DQN loop (dqn_atari_oc.py:345-372) in ONE launch, for the object-frame
 * synthetic env (ocppo_synth_env_step's, seed env_seed, step id *env_step_base + env_step_offset)
 * and E <= 64 envs: ocppo_q_head_epsilon_greedy's actions (actions, epsilon_out), the env step on
 * them (frame [E, D] f32, env_reward / env_done [E], ep_state [E, 5] or NULL), the frame-stack
 * store of ocppo_rollout_store (prev_obs -> obs_out [E, W, D] in obs_dtype, net_obs f32 or NULL,
 * done_out; reward_out = the reward, or with vecnorm != 0 ocppo_rollout_store_vecnorm's normalised
 * reward and (ret_state, rms_state) update) and ocppo_replay_add of (prev_obs, obs_out, actions,
 * reward_out, done_out) into a replay of obs_dtype (rb_obs [rb_size, E, W * D], rb_state {pos,
 * full}). advance != 0 then adds advance to *step and *env_step_base (both read before: the
 * last env step of a captured chunk moves the chunk's counters, replacing two launches). Every
 * output is bitwise the four launches'. */
OCPPO_API int ocppo_dqn_act_step(
    ocppo_stream_t stream, const float* hidden, int64_t E, int64_t H, const float* wq,
    const float* bq, int64_t A, uint64_t seed, int64_t* step, int64_t step_offset,
    double start_e, double end_e, double duration, int64_t* actions, float* epsilon_out,
    uint64_t env_seed, int64_t* env_step_base, int64_t env_step_offset, int64_t D,
    float* frame, float* env_reward, float* env_done, float* ep_state, int64_t W,
    const void* prev_obs, void* obs_out, int obs_dtype, float* net_obs, float* done_out,
    float* reward_out, int vecnorm, double vn_gamma, double vn_epsilon, double vn_clip,
    double* ret_state, double* rms_state, int64_t* rb_state, int64_t rb_size, void* rb_obs,
    int64_t* rb_actions, float* rb_rewards, float* rb_dones, int64_t advance);
OCPPO_API int ocppo_epsilon_greedy(ocppo_stream_t stream, const float* q, int64_t E, int64_t A,
                                   uint64_t seed, const int64_t* step, int64_t step_offset,
                                   double start_e, double end_e, double duration,
                                   int64_t* actions, float* epsilon_out);
/* q, q_next : [B, A] f32 (q_network(obs), target_network(next_obs)); dq : [B, A] = d loss / d q;
 * stats : [2] = {td_loss, mean(old_val)} (losses/td_loss, losses/q_values of :385-386)
 *   td = r + (f32(gamma) * max_a q_next) * (1 - d);  old = q[b, a_b];  loss = mean((td - old)^2) */
OCPPO_API int ocppo_td_loss_fwd_bwd(ocppo_stream_t stream, const float* q, const float* q_next,
                                    const int64_t* actions, const float* rewards,
                                    const float* dones, int64_t B, int64_t A, double gamma,
                                    float* dq, float* stats);

/* ---------------------------------------------------------------------------------------------
 * Synthetic device-resident env (benchmark / test harness; ALE and OCAtari are not available).
 * Not a reference component. Counter-based hashing of (seed, env, step) gives reproducible
 * frames: object mode x~U{0..159}, y~U{0..209}, w,h~U{1..16} per 4-feature object; pixel mode
 * 84x84 u8 with ~90% zeros; reward = +-1 w.p. 0.005 each; done w.p. 1/3500 (Pong-v5 episode
 * lengths). `actions` shift the first object's y so the env reacts to the policy.
 *   frame_out : [N, D] (f32 for obj, u8 for pixels); reward_out, done_out : [N] f32
 *   step_base : device int64 read at run time (graph replays advance it), the hashed step id is
 *               step_base[0] + step_offset
 *   ep_state  : [N, 5] f32 = {running return, running length, finished-episode return sum,
 *               finished-episode length sum, finished-episode count}, updated in place (may be
 *               NULL); the RecordEpisodeStatistics counters behind ppo_atari_oc.py:516-529
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_synth_env_step(ocppo_stream_t stream, uint64_t seed, const int64_t* step_base,
                         int64_t step_offset, const int64_t* actions, int64_t N, int64_t D, int pixel_mode,
                         void* frame_out, float* reward_out, float* done_out, float* ep_state);

/* The rollout policy head (ocppo_policy_head_sample, one wave per env) with the synthetic env's
 * object-frame step fused behind it: the wave that sampled env n's action writes env n's next
 * frame / reward / done / episode counters exactly as ocppo_synth_env_step(pixel_mode 0) would
 * from action_out -- one launch for architectures/ppo.py:89-95 + the env step of
 * ppo_atari_oc.py:506-511. Entropy and logits are not produced.
 *   N <= 3072 (<= 2048 when H > 512), H in {256, 512, 768, 1024}, A <= 7, D <= 4096; hidden and
 *   the head weights 16-B aligned (else OCPPO_ERR_INVALID: use the two launches). */
OCPPO_API int ocppo_policy_head_env_step(ocppo_stream_t stream, const float* hidden, int64_t N,
                                         int64_t H, const float* w_actor, const float* b_actor,
                                         const float* w_critic, const float* b_critic,
                                         float* noise, const int64_t* philox_state,
                                         int64_t philox_offset, int64_t philox_stride,
                                         int64_t A, int64_t* action_out,
                                         float* logprob_out, float* value_out, uint64_t seed,
                                         const int64_t* step_base, int64_t step_offset, int64_t D,
                                         float* frame_out, float* reward_out, float* done_out,
                                         float* ep_state);

/* ---------------------------------------------------------------------------------------------
 * Policy heads forward + fused PPO loss + heads backward in one pass over the decoder output
 * (ppo_atari_oc.py:566-605 from h = relu(z) on; architectures/ppo.py:81-84):
 *   logits = h Wa^T + ba, value = h Wc^T + bc; the loss of ocppo_ppo_loss_fwd_bwd on the prepared
 *   (minibatch-order, contiguous) records mb_* [M] with adv_stats [2] (required when norm_adv);
 *   c = (d loss / d logits, d loss / d value);  gp [M, H] = (h <= 0 ? 0 : c W), W = [Wa; Wc];
 *   db_h [H] = sum_m gp (the decoder bias grad, may be NULL); dwa [A, H], dwc [H], dba [A],
 *   dbc [1] the heads' grads; stats [9] as ocppo_ppo_loss_fwd_bwd; dlogits [M, A] / dvalue [M]
 *   optional (both NULL or both set).
 * H in {64, 128, 256, 512} (else OCPPO_E_INVALID), 1 <= A <= 7; h, gp, Wa, Wc 16-B aligned. Two
 * launches: a fixed grid of at most 512 workgroups, each owning a contiguous row range and writing
 * ONE partial record, then a fixed-shape tree over the records: deterministic; workspace =
 * ocppo_heads_loss_workspace_bytes(M, H, A), needs no zeroing.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API size_t ocppo_heads_loss_workspace_bytes(int64_t M, int64_t H, int64_t A);
OCPPO_API int ocppo_heads_loss_fwd_bwd(ocppo_stream_t stream, const float* h, int64_t M, int64_t H,
                                       const float* w_actor, const float* b_actor,
                                       const float* w_critic, const float* b_critic, int64_t A,
                                       const int64_t* mb_actions, const float* mb_logprobs,
                                       const float* mb_advantages, const float* mb_returns,
                                       const float* mb_values, const float* adv_stats,
                                       double clip_coef, double ent_coef, double vf_coef,
                                       int norm_adv, int clip_vloss, float* gp, float* db_h,
                                       float* dwa, float* dwc, float* dba, float* dbc,
                                       float* stats, float* dlogits, float* dvalue,
                                       void* workspace, size_t workspace_bytes);
/* Deferred form: ocppo_heads_loss_rows launches the rows kernel only and writes the finish (the
 * tree over the records, which writes db_h, dwa, dwc, dba, dbc and stats) into *finish, a plain
 * host record; the caller runs it later on the same stream, before anything reads those outputs
 * and before the workspace is reused: folded into the split-K combine the backward runs next
 * (ocppo_sum_splits_finish = ocppo_sum_splits, bitwise, plus the finish workgroups in the same
 * launch) or alone (ocppo_deferred_finish_run). Same results as ocppo_heads_loss_fwd_bwd, bitwise.
 * The record holds device pointers only; it may be copied and run once per rows launch. */
OCPPO_API int ocppo_heads_loss_rows(ocppo_stream_t stream, const float* h, int64_t M, int64_t H,
                                    const float* w_actor, const float* b_actor,
                                    const float* w_critic, const float* b_critic, int64_t A,
                                    const int64_t* mb_actions, const float* mb_logprobs,
                                    const float* mb_advantages, const float* mb_returns,
                                    const float* mb_values, const float* adv_stats,
                                    double clip_coef, double ent_coef, double vf_coef,
                                    int norm_adv, int clip_vloss, float* gp, float* db_h,
                                    float* dwa, float* dwc, float* dba, float* dbc, float* stats,
                                    float* dlogits, float* dvalue, void* workspace,
                                    size_t workspace_bytes, ocppo_deferred_finish_t* finish);
OCPPO_API int ocppo_sum_splits_finish(ocppo_stream_t stream, const float* part, int64_t S,
                                      int64_t n, float* out, const ocppo_deferred_finish_t* finish);
OCPPO_API int ocppo_deferred_finish_run(ocppo_stream_t stream,
                                        const ocppo_deferred_finish_t* finish);

/* ---------------------------------------------------------------------------------------------
 * Rollout fusions of the PPObj frame-encoding cache path (ppo_atari_oc.py:502-514 + :506 with
 * architectures/ppo.py:60-95): per env step the launches are [store of step t-1 + the first two
 * encoder layers of the newest frame] -> middle encoder layers -> [last encoder layer + cache
 * shift] -> decoder -> fused policy head.
 *
 * ocppo_linear_cache_shift: fresh = act(x W^T + b) (as ocppo_linear_act, x [M, K], W [N, K]) is
 *   not stored; instead enc [M, W, N] (the frame-encoding cache) is shifted with it:
 *   enc[m, w] = done[m] != 0 || w == W-1 ? fresh[m] : enc[m, w+1]  (ocppo_frame_cache_shift's rule;
 *   done [M] f32 or NULL).
 * ocppo_store_linear2: ocppo_rollout_store (vecnorm = 0; reward_out = the raw reward row) or
 *   ocppo_rollout_store_vecnorm (vecnorm = 1) of frame [N, D] f32 into obs_out / net_obs /
 *   reward_out / done_out, AND y [N, N2] (row stride ldy) = relu(relu(f W1^T + b1) W2^T + b2) of
 *   the newest frames f = frame seen through obs_dtype (OCPPO_F32 or OCPPO_BF16 round trip), as
 *   ocppo_linear2_act (D <= 64, N1 % 16 == 0, N1 <= 512, W2 16-B aligned), in one launch.
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_linear_cache_shift(ocppo_stream_t stream, const float* x, int64_t ldx,
                                       const float* w, const float* b, float* enc,
                                       const float* done, int64_t M, int64_t N, int64_t K,
                                       int64_t W, int relu);
/* Ring form of the frame-encoding cache (no shift): the W physical slots of enc [M, W, N] hold the
 * W logical frames (oldest .. newest) rotated by a per-step offset r, logical slot w at physical
 * (w + r) mod W.
 * ocppo_linear_cache_ring: fresh = act(x W^T + b) overwrites physical slot `slot` only (the
 *   oldest frame's: at rollout step t the newest frame goes to slot (t - 1) mod W), or every
 *   slot of env m when done[m] != 0 (a reset fills the stack with the new frame). No old slot is
 *   read. done [M] f32 or NULL.
 * ocppo_linear_act_ring: ocppo_linear_act whose x rows are W = K / seg segments of seg floats
 *   stored rotated: logical segment s at physical segment (s + rot) mod W (seg a power of two >= 32,
 *   K % seg == 0, x / w 16-B aligned, ldx % 4 == 0). Products and summation order are those of
 *   the logical layout: the decoder (architectures/ppo.py:74-78: Flatten + Linear over the W
 *   frame encodings) on the ring gives bit for bit what it gives on the shifted cache. */
OCPPO_API int ocppo_linear_cache_ring(ocppo_stream_t stream, const float* x, int64_t ldx,
                                      const float* w, const float* b, float* enc,
                                      const float* done, int64_t M, int64_t N, int64_t K,
                                      int64_t W, int64_t slot, int relu);
OCPPO_API int ocppo_linear_act_ring(ocppo_stream_t stream, const float* x, int64_t ldx,
                                    const float* w, const float* b, float* y, int64_t ldy,
                                    int64_t M, int64_t N, int64_t K, int64_t seg, int64_t rot,
                                    int relu);
/* ---------------------------------------------------------------------------------------------
 * NHWC Conv2d (no padding, no dilation, groups 1) + bias + optional ReLU for the rollout
 * forward of the NatureCNN trunk (architectures/ppo.py:20-31 at ppo_atari_oc.py:506):
 *   y[b, oy, ox, co] = act(bias[co] + sum_{ky,kx,ci} x[b, oy*s+ky, ox*s+kx, ci] w[co, ky, kx, ci])
 * x [B, H, W, Cin] f32 (a channels_last NCHW tensor's memory), w [Cout, KH, KW, Cin] (a
 * channels_last conv weight's memory), bias [Cout] or NULL, y [B, OH, OW, Cout] f32, OH =
 * (H - KH) / s + 1. Cin a power of two >= 4, KH*KW*Cin % 16 == 0, x / w 16-B aligned.
 * Implicit GEMM on v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation).
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_conv2d_act(ocppo_stream_t stream, const float* x, int64_t B, int64_t H,
                               int64_t W, int64_t Cin, const float* w, const float* b,
                               int64_t Cout, int64_t KH, int64_t KW, int64_t stride, float* y,
                               int relu);
OCPPO_API int ocppo_store_linear2(ocppo_stream_t stream, const float* frame, const float* reward,
                                  const float* done, int64_t N, int64_t W, int64_t D,
                                  const void* prev_obs, void* obs_out, int obs_dtype,
                                  float* net_obs, float* reward_out, float* done_out, int vecnorm,
                                  double gamma, double epsilon, double clip_reward,
                                  double* ret_state, double* rms_state, const float* w1,
                                  const float* b1, const float* w2, const float* b2, float* y,
                                  int64_t ldy, int64_t N1, int64_t N2);

/* ---------------------------------------------------------------------------------------------
 * CartPole-v1 vector env (config 1: cleanrl/ppo.py:81-91, 162 -- SyncVectorEnv of
 * RecordEpisodeStatistics(gym.make("CartPole-v1"))), device-resident. gymnasium 0.28.1
 * cartpole.py dynamics in f64 (Euler, same constants and op order), reward 1 per step,
 * TimeLimit 500, same-step auto-reset (obs of a done env = its reset obs), obs = f32(state).
 * Reset states ~ U(-0.05, 0.05)^4 from a counter-based stream of (seed, env, episode index).
 *   actions  : [N] i64 (0 = push left, 1 = push right), or NULL = reset every env
 *   state    : [N, 4] f64 (x, x_dot, theta, theta_dot), in/out
 *   counters : [N, 2] i64 = {elapsed steps, episodes started}, in/out (zero-initialised)
 *   obs_out  : [N, 4] f32;  reward_out, done_out : [N] f32 (may be NULL on reset)
 *   ep_state : [N, 5] f32 RecordEpisodeStatistics counters as in ocppo_synth_env_step, or NULL
 * ------------------------------------------------------------------------------------------- */
OCPPO_API int ocppo_cartpole_step(ocppo_stream_t stream, uint64_t seed, const int64_t* actions,
                                  int64_t N, double* state, int64_t* counters, float* obs_out,
                                  float* reward_out, float* done_out, float* ep_state);

#ifdef __cplusplus
}
#endif
#endif /* OCPPO_H */
