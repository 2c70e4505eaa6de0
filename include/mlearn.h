/*
 * mlearn.h — C ABI of the MI355X-native batched-PPO hot path.
 *
 * This is the drop-in boundary beneath the Python plugin surface that
 * madrona-learn exposes for its PPO iteration (rollout collection -> GAE ->
 * minibatch PPO update).  The reference has no native ABI: every entry point
 * below names the reference function (file:line, relative to the
 * shacklettbp/madrona-learn source tree, src/madrona_learn/) whose arithmetic
 * it replaces.  The Python host package (madrona-learn_amd/madrona_learn)
 * calls these through ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Plain pointers to device memory (HBM) + sizes; no torch/framework types.
 *  - The caller owns every buffer.  No entry point allocates or synchronises,
 *    so every call is safe inside HIP-graph capture.  Scratch comes from a
 *    caller-supplied workspace whose size is queried up front.
 *  - Every call takes an explicit hipStream_t (as mlearn_stream_t) and returns
 *    an int status: MLEARN_OK (0), MLEARN_EINVAL (<0: bad argument, nothing
 *    launched) or MLEARN_EHIP (launch failure).  mlearn_last_error() returns a
 *    thread-local message for the last failing call.
 *  - Layouts are row-major.  Rollout arrays are [T][N] (time-major, env-minor)
 *    which is exactly the reference's pre-finalize store [C][T/C][P][B]
 *    (rollouts.py:460-478) viewed flat.
 */
#ifndef MLEARN_H
#define MLEARN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MLEARN_ABI_VERSION 22

#define MLEARN_OK 0
#define MLEARN_EINVAL (-1)
#define MLEARN_EHIP (-2)

#define MLEARN_DTYPE_F32 0
#define MLEARN_DTYPE_BF16 1

#define MLEARN_MAX_LAYERS 4
#define MLEARN_MAX_GROUPS 16
#define MLEARN_HEAD_COLS 32     /* head width of a scalar critic: actor logits + 1, padded */
#define MLEARN_HEAD_COLS_MAX 96 /* head width when actor logits + critic bins exceed 32 */

typedef void* mlearn_stream_t; /* hipStream_t */
typedef void* mlearn_comm_t;   /* RCCL communicator (mlearn_comm_init) */
#define MLEARN_COMM_ID_BYTES 128

const char* mlearn_last_error(void);
int mlearn_abi_version(void);

/* ---------------------------------------------------------------------- */
/* RNG: Philox4x32-10 (replaces jax.random threefry; see DESIGN.md "RNG")  */
/* ---------------------------------------------------------------------- */
/* out[i] = philox4x32(ctr[i], {k0,k1}); ctr/out are [n][4] uint32 in HBM. */
int mlearn_philox4x32(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out,
                      int64_t n, mlearn_stream_t stream);
/* The LSTM cell's gate activations as the fused kernels compute them
 * (v_exp_f32 / v_rcp_f32 sigmoid and tanh, odd series below |x| < 1/8;
 * flax OptimizedLSTMCell gates, rnn.py:30-36): sigmoid_out[i], tanh_out[i]
 * of x[i] (accuracy pin). */
int mlearn_lstm_activations_f32(const float* x, int64_t n, float* sigmoid_out, float* tanh_out,
                                mlearn_stream_t stream);
/* The same on the host (host memory, no GPU): the control-plane draws of the
 * population ops (pbt.py:473-562 explore_param, 565-722 cull / past copy). */
int mlearn_philox4x32_host(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out,
                           int64_t n);

/* Counters.  Every RNG-consuming entry point takes (const uint64_t* ctr,
 * uint64_t add): the effective counter is (ctr ? *ctr : 0) + add, read on the
 * device, so a captured HIP graph replays with fresh randomness once the
 * counters are advanced on the stream with mlearn_counters_add. */
int mlearn_counters_add(uint64_t* ctr, int32_t n, const uint64_t* deltas /* host, n <= 8 */,
                        mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Returns / advantages                                                    */
/* ---------------------------------------------------------------------- */
/* Reverse-time GAE scan over [T][N] (algo_common.py:84-130) fused with
 * returns = advantages + values (rollouts.py:761-769).  dones are bytes
 * (bool, rollouts.py:454-455,933).  bootstrap is [N].  returns may be NULL:
 * only the advantages are written (4 B per element instead of 8) and the
 * consumers form returns = advantages + values themselves, the same f32
 * addition (mlearn_rollout_view.returns = NULL, mlearn_metric_job.x2).
 * gamma_lambda is the product cfg.gamma * cfg.gae_lambda formed by the caller
 * in double precision and rounded to f32 once: algo_common.py:120 evaluates
 * `cfg.gamma * cfg.gae_lambda * next_advantage` left to right with Python
 * floats (rollouts.py:406), so the constant is one f64 product that JAX's
 * weak typing rounds to f32 (f32(gamma) * f32(lambda) differs by an ulp for
 * e.g. 0.998 / 0.95). */
int mlearn_gae_f32(const float* rewards, const float* values, const uint8_t* dones,
                   const float* bootstrap, float* advantages, float* returns, int32_t T,
                   int64_t N, float gamma, float gamma_lambda, mlearn_stream_t stream);

/* mlearn_gae_f32 with a value normaliser (TrainConfig.normalize_values): the
 * stored values and the bootstrap are critic outputs in the normalised space
 * and are inverted first, v * sigma + mu in f32 (EMANormalizer.invert,
 * moving_avg.py:87-95, applied in _finalize_rollouts rollouts.py:726-738);
 * returns = advantages + inverted values (rollouts.py:769).  value_norm holds
 * one 8-float estimate record per policy, {mu, inv_sigma, sigma, mu_biased,
 * sigma_sq_biased, 0, 0, 0} (mlearn_value_norm_chain); column n uses record
 * n / cols_per_norm. */
int mlearn_gae_vnorm_f32(const float* rewards, const float* values, const uint8_t* dones,
                         const float* bootstrap, const float* value_norm, int64_t cols_per_norm,
                         float* advantages, float* returns, int32_t T, int64_t N, float gamma,
                         float gamma_lambda, mlearn_stream_t stream);

/* Discounted returns without advantages (algo_common.py:45-81), used when
 * TrainConfig.compute_advantages is False. */
int mlearn_returns_f32(const float* rewards, const uint8_t* dones, const float* bootstrap,
                       float* returns, int32_t T, int64_t N, float gamma,
                       mlearn_stream_t stream);

/* Whole-array z-score (algo_common.py:133-140): out = (x-mean)*rsqrt(max(var,1e-5)).
 * workspace >= mlearn_zscore_workspace_bytes(n). */
int64_t mlearn_zscore_workspace_bytes(int64_t n);
int mlearn_zscore_f32(const float* x, int64_t n, float* out, void* workspace,
                      mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Discrete action distributions (dists.py:12-77)                          */
/* ---------------------------------------------------------------------- */
typedef struct mlearn_action_layout {
    int32_t num_groups;                        /* K sub-actions */
    int32_t num_logits;                        /* sum of buckets (<= 31) */
    int32_t offsets[MLEARN_MAX_GROUPS + 1];    /* group k = logits[offsets[k], offsets[k+1]) */
} mlearn_action_layout;

/* DiscreteActionDistributions.sample (dists.py:26-44): Gumbel-max per group
 * with noise from Philox(ctr={env_offset+n, j>>2, step}, key={k0,k1}); the
 * log-prob is logit[a] - logsumexp(group); step = *step_ctr + step.
 * sample == 0 gives best()
 * (dists.py:46-52, first-index argmax) and log_probs may be NULL. */
int mlearn_discrete_sample_f32(const float* logits, int64_t ld, mlearn_action_layout layout,
                               int64_t N, uint32_t k0, uint32_t k1, const uint64_t* step_ctr,
                               uint64_t step, uint32_t env_offset, int32_t sample,
                               int32_t* actions, float* log_probs, mlearn_stream_t stream);

/* DiscreteActionDistributions.action_stats (dists.py:54-77). */
int mlearn_action_stats_f32(const float* logits, int64_t ld, mlearn_action_layout layout,
                            int64_t N, const int32_t* actions, float* log_probs,
                            float* entropies, mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* MLP actor-critic (actor_critic.py:38-128 with BackboneShared 202-244,   */
/* BackboneEncoder 131-153, models.py MLP 99-119, LayerNorm 46-56,          */
/* DenseLayerDiscreteActor 122-139, DenseLayerCritic 142-154).             */
/* ---------------------------------------------------------------------- */
/* The compute-dtype weight copies are "fragment-order" images (written by
 * mlearn_policy_sync_weights / mlearn_optim_step): a logical matrix Bt[N][K]
 * stores element (n, k) at
 *   ((n/32 * K/KS + k/KS) * 64 + n%32 + 32*((k%KS)/E)) * E + k%E
 * with (E, KS) = (8, 16) for bf16 and (1, 2) for f32, so that one wave's
 * matrix-core B operand is a single contiguous run. */
typedef struct mlearn_mlp_policy {
    int32_t dtype;       /* compute dtype: MLEARN_DTYPE_F32 / MLEARN_DTYPE_BF16 */
    int32_t obs_dim;     /* multiple of 16, <= 256 */
    int32_t hidden;      /* 64, 128 or 256 */
    int32_t num_layers;  /* 1..MLEARN_MAX_LAYERS */
    int32_t critic_bins; /* 1: DenseLayerCritic (scalar value, models.py:142-154);
                            odd >= 3: DreamerV3Critic two-hot logits (models.py:157-174,
                            SymExpTwoHotDistribution dists.py:119-208; default 63) */
    mlearn_action_layout actions;
    const void* w_t[MLEARN_MAX_LAYERS];  /* hidden*in_l: Bt[n=out][k=in] = W_l[k][n] */
    const void* w[MLEARN_MAX_LAYERS];    /* hidden*in_l: Bt[n=in][k=out] = W_l[n][k];
                                            w[0] is not used */
    const float* ln_scale[MLEARN_MAX_LAYERS];  /* [hidden] f32 */
    const float* ln_bias[MLEARN_MAX_LAYERS];   /* [hidden] f32 */
    /* head columns: 0..A-1 actor logits, A..A+critic_bins-1 critic, zero padding up
     * to HC = mlearn_head_cols(policy) (32, or 96 when A + critic_bins > 32) */
    const void* head_t;      /* HC*hidden: Bt[n=head col][k=unit] */
    const void* head;        /* HC*hidden: Bt[n=unit][k=head col] */
    const float* head_bias;  /* [HC] f32 */
    /* ObservationsEMANormalizer (observations.py:70-132, EMANormalizer
     * moving_avg.py:48-196).  obs_mu == NULL: the preprocess is a cast. */
    const float* obs_mu;         /* [obs_dim] f32: x' = (x - mu) * inv_sigma, then the cast */
    const float* obs_inv_sigma;  /* [obs_dim] f32 */
    float* obs_stats;            /* NULL, or [obs_stats_steps][obs_stats_tiles][obs_dim][2]:
                                    the rollout step `step` writes, per 32-env tile, the
                                    {mean, M2} of its raw observations (update_obs_stats,
                                    rollouts.py:670-676) */
    int64_t obs_stats_tiles;     /* >= ceil(N / 32) */
    int32_t obs_stats_steps;
    int32_t obs_pad;
} mlearn_mlp_policy;

/* Head width HC of a policy descriptor (-1 if invalid). */
int32_t mlearn_head_cols(const mlearn_mlp_policy* policy);

/* Observation statistics of one rollout -> new normaliser estimates
 * (rollouts.py:670-678 + train.py:193-204): per step t the tile partials of
 * obs_stats are merged (Chan) into the batch mean / population variance of
 * the N observations, folded over t = 0..steps-1 by
 * EMANormalizer.update_input_stats (moving_avg.py:107-130, n_a = t), then
 * update_estimates (moving_avg.py:132-180) with decay / eps.
 * est: [5][obs_dim] f32 = mu, inv_sigma, sigma, mu_biased, sigma_sq_biased
 * (in/out); count: the int32 update counter N (in/out, device). */
int mlearn_obs_norm_update(const float* obs_stats, int32_t steps, int64_t tiles, int64_t N,
                           int32_t obs_dim, float decay, float eps, float* est, int32_t* count,
                           mlearn_stream_t stream);

/* EMANormalizer.update_input_stats (moving_avg.py:107-130) of one [rows][dim]
 * f32 batch: batch mean and population variance per column, merged into the
 * running cur_stats = [2][dim] {mean | var} with n_a = num_prev_updates;
 * out_stats [2][dim] (may alias cur_stats).  rows < 2^24. */
int mlearn_ema_input_stats(const float* x, int64_t rows, int32_t dim, const float* cur_stats,
                           int32_t num_prev_updates, float* out_stats, mlearn_stream_t stream);
/* EMANormalizer.update_estimates (moving_avg.py:132-180): est [5][dim] =
 * mu, inv_sigma, sigma, mu_biased, sigma_sq_biased (in/out) from input_stats
 * [2][dim]; count = the int32 update counter N (in/out, device). */
int mlearn_ema_update_estimates(const float* input_stats, int32_t dim, float decay, float eps,
                                float* est, int32_t* count, mlearn_stream_t stream);

/* Post-step bookkeeping of the PREVIOUS env step (rollouts.py:933-973), fused
 * into the next policy launch; same arithmetic as mlearn_rollout_post_step. */
typedef struct mlearn_post_step {
    const float* rewards;       /* [N] env output of step t-1 */
    const uint8_t* dones;       /* [N] */
    float* store_rewards;       /* [N] rollout store, step t-1 */
    uint8_t* store_dones;       /* [N] */
    float* env_returns;         /* [N] running discounted return (in/out) */
    float* env_returns_trace;   /* [N] or NULL */
    float gamma;
} mlearn_post_step;

/* One rollout step of ActorCritic.rollout (actor_critic.py:74-96) fused with
 * the post-inference store (rollouts.py:637-668): preprocess (cast to the
 * compute dtype) -> MLP trunk -> actor logits + critic -> sample -> write
 * obs_store[N][obs_dim] (may be NULL), actions[N][K] i32, log_probs[N][K] f32,
 * values[N] f32 (the scalar critic, or SymExpTwoHotDistribution.mean() of the
 * two-hot critic, rollouts.py:601-605).  actions == NULL computes only the critic
 * (ActorCritic.critic_only, actor_critic.py:65-72, used for the bootstrap
 * values, rollouts.py:607-635).  post (may be NULL) applies the post-step of
 * the previous env step in the same launch. */
int mlearn_policy_rollout_step(const mlearn_mlp_policy* policy, const float* obs, int64_t N,
                               void* obs_store, int32_t* actions, float* log_probs,
                               float* values, uint32_t k0, uint32_t k1,
                               const uint64_t* step_ctr, uint64_t step, uint32_t env_offset,
                               int32_t sample, const mlearn_post_step* post,
                               mlearn_stream_t stream);

/* Post-step bookkeeping of rollout_loop (rollouts.py:933-973, _post_step_cb
 * 682-714): store rewards/dones at step t, env_returns = r + gamma*env_returns,
 * trace it (for the 'Env Returns' metric), then zero it where done. */
int mlearn_rollout_post_step(const float* rewards, const uint8_t* dones, int64_t N,
                             float* store_rewards, uint8_t* store_dones, float* env_returns,
                             float* env_returns_trace, float gamma, mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Metrics (metrics.py:31-48 Metric.init_from_data): mean, m2, min, max,   */
/* count of up to 16 float arrays in one launch.                           */
/* ---------------------------------------------------------------------- */
typedef struct mlearn_metric_job {
    const float* x;
    int64_t n;          /* element count */
    int64_t cols;       /* 0: x is contiguous; else element i is x[(i / cols) * ld + i % cols] */
    int64_t ld;         /*    (a [n/cols][cols] window of a wider array, e.g. one policy's */
                        /*    env columns of the [T][N] store) */
    int32_t abs_value;  /* 1: metric of |x| (ppo.py:358 'Value Errors') */
    int32_t pad;
    const float* x2;    /* NULL, or a second array of the same shape: the metric is of x + x2
                           (the 'Est Returns' = advantages + values of a GAE that did not
                           materialise returns) */
} mlearn_metric_job;

int64_t mlearn_metrics_workspace_bytes(int32_t num_jobs);
/* out[j*5 + {0..4}] = {mean, m2, min, max, count} */
int mlearn_metrics_f32(const mlearn_metric_job* jobs, int32_t num_jobs, float* out,
                       void* workspace, mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* PPO update (ppo.py:109-488)                                             */
/* ---------------------------------------------------------------------- */
/* Epoch permutation of n sequence ids (ppo.py:445-458, random.permutation):
 * perm[i] = cycle-walked 4-round Feistel bijection of i on [0, 2^b), b =
 * ceil(log2 n) rounded up to even, round r function = Philox4x32-10 word 0 of
 * ctr {R + (r << 24), rank, epoch lo, epoch hi}, keys (k0, k1).  n <= 2^30. */
int mlearn_minibatch_perm(uint32_t k0, uint32_t k1, const uint64_t* epoch_ctr, uint64_t epoch,
                          uint32_t rank, int32_t n, int32_t* perm, mlearn_stream_t stream);

typedef struct mlearn_rollout_view {
    const void* obs;          /* [T][N][obs_dim] compute dtype */
    const int32_t* actions;   /* [T][N][K] */
    const float* log_probs;   /* [T][N][K] */
    const float* advantages;  /* [T][N] */
    const float* returns;     /* [T][N]; NULL: returns = advantages + values (GAE without
                                 materialised returns, mlearn_gae_f32) */
    const float* values;      /* [T][N] */
    const uint8_t* dones;     /* [T][N] sequence breaks (recurrent policies; may be NULL) */
    int32_t T;                /* steps per update */
    int32_t bptt_len;         /* T / num_bptt_chunks */
    int64_t N;                /* envs B of the policy this view trains */
    int64_t ld;               /* row stride of the [T][.] arrays in envs (0: = N).  A policy of
                                 a population owns env columns [p*B, (p+1)*B) of a [T][P*B]
                                 store (pbt.py:130-133 self-play split): its view points at
                                 column p*B with N = B, ld = P*B. */
} mlearn_rollout_view;

/* Per-minibatch advantage statistics for zscore_data (algo_common.py:133-140,
 * ppo.py:134-143): for minibatch m of the epoch, double partials of
 * (sum x, sum x^2) over its mb_size sequences x bptt_len steps.  Output
 * partials[m][2] (to be all-reduced across ranks under data parallelism),
 * finished by mlearn_adv_stats_finish into stats[m] = {mean, rsqrt(max(var,1e-5))}.
 * `partials` must hold num_mb * 66 doubles; the first num_mb * 2 are the
 * per-minibatch sums (the rest is scratch). */
int mlearn_adv_stats(const mlearn_rollout_view* ro, const int32_t* perm, int32_t num_mb,
                     int32_t mb_size, double* partials, mlearn_stream_t stream);
int mlearn_adv_stats_finish(const double* partials, int32_t num_mb, double count,
                            float* stats, mlearn_stream_t stream);

/* mlearn_adv_stats over the returns: per-minibatch double (sum x, sum x^2)
 * of the value normaliser's input (ppo.py:209-211), same partials layout. */
int mlearn_return_stats(const mlearn_rollout_view* ro, const int32_t* perm, int32_t num_mb,
                        int32_t mb_size, double* partials, mlearn_stream_t stream);

/* Value normaliser over one epoch's minibatches in order (ppo.py:205-211,
 * 346): minibatch m updates the estimates with its returns'
 * (mean, population variance) = return_sums[m] / count (update_input_stats
 * from zero, then update_estimates, moving_avg.py:103-192; decay =
 * TrainConfig.value_normalizer_decay, eps 1e-5).  est = {mu, inv_sigma,
 * sigma, mu_biased, sigma_sq_biased, ...} (8 floats) and *n_updates are
 * updated in place.  records[m] (8 floats) = {adv mean, adv rstd (from
 * adv_stats[m]), mu and inv_sigma after the update, mu and sigma before it,
 * 0, 0}: the adv_stats argument of mlearn_ppo_minibatch_grad when
 * hp->normalize_values. */
int mlearn_value_norm_chain(const double* return_sums, const float* adv_stats, int32_t num_mb,
                            double count, float decay, float eps, float* est, int32_t* n_updates,
                            float* records, mlearn_stream_t stream);

typedef struct mlearn_ppo_hparams {
    float clip_coef;
    float value_loss_coef;
    float entropy_coef[MLEARN_MAX_GROUPS]; /* per sub-action j (ppo.py:231-239), see obj_weight */
    int32_t normalize_advantages;          /* TrainConfig.normalize_advantages */
    int32_t clip_value_loss;               /* PPOConfig.clip_value_loss */
    int32_t huber_value_loss;              /* PPOConfig.huber_value_loss */
    float loss_scale;                      /* 1/world_size under DP (mean of means) */
    int32_t normalize_values;              /* TrainConfig.normalize_values: adv_stats is a
                                              mlearn_value_norm_chain record */
    float obj_weight[MLEARN_MAX_GROUPS];   /* per sub-action j; 0 means 1.  The loss is
                                              -sum_j obj_weight[j] sum_rows obj_j / (M K)
                                              + c_v mean(vl)
                                              - sum_j entropy_coef[j] sum_rows H_j / (M K)
                                              (K sub-actions, M rows).  The reference's
                                              per-action-group means (ppo.py:221-239) are
                                              obj_weight[j] = K / K_g and entropy_coef[j] =
                                              c_g K / K_g for the group g holding j. */
    double* grad_sumsq_out;                /* may be NULL: per-64-parameter partial sums of
                                              grad^2 (mlearn_grad_sumsq_parts entries),
                                              written by the gradient reduction; the next
                                              mlearn_optim_step may take them as
                                              grad_sumsq_part instead of re-reading grads
                                              (only valid when grads are not all-reduced
                                              in between) */
    int32_t step_kernel;                   /* forward / loss / backward kernel of the MLP
                                              step: 0 = the library's choice (the row-split
                                              kernel where it applies: bf16, hidden 256,
                                              2 layers, scalar critic (head width 32) or
                                              a two-hot critic of <= 64 bins (head width
                                              96, ABI 21), obs_dim 64, at most 7 action
                                              groups,
                                              padded rows of exactly 32768 (one 16-row tile
                                              per wave) or a multiple of 256 and >= 65536;
                                              else the feature-split kernel), 1 = the feature-split
                                              kernel, 2 = the row-split kernel (EINVAL
                                              where it does not apply).  Same inputs and
                                              outputs; results within the compute dtype's
                                              rounding of each other (summation orders) */
    int32_t wgrad_form;                    /* operand staging of the bf16 weight-gradient
                                              launch (ABI 22): 0 = the library's choice
                                              (2), 1 = register-staged (round 5: two
                                              chunks in flight through registers),
                                              2 = LDS-DMA pipeline (global_load_lds,
                                              ML_WG_STAGES stages).  Same fragments in
                                              the same order: bit-identical gradients */
} mlearn_ppo_hparams;

/* Number of partials mlearn_ppo_hparams.grad_sumsq_out receives: one per 64
 * parameters of the flat layout (ceil(param_count / 64)). */
int64_t mlearn_grad_sumsq_parts(int64_t param_count);

/* Size of the minibatch workspace (activations + gradient slabs). */
int64_t mlearn_ppo_workspace_bytes(const mlearn_mlp_policy* policy, int64_t rows);

/* The step kernel mlearn_ppo_minibatch_grad runs for this policy and minibatch
 * row count given mlearn_ppo_hparams.step_kernel = requested: 1 (feature-split)
 * or 2 (row-split); -1 for an invalid policy / request (host-only, no GPU). */
int32_t mlearn_ppo_step_kernel(const mlearn_mlp_policy* policy, int64_t rows, int32_t requested);

/* One PPO minibatch step up to the flat gradient: forward (ActorCritic.update,
 * actor_critic.py:98-128), loss (ppo.py:129-262), backward (jax.value_and_grad,
 * ppo.py:276-281) and the reduction of all per-row-tile partials into
 * grad[param_count] (flat f32, layout of mlearn_param_offsets).
 * mb_seq = the mb_size sequence ids of this minibatch (a slice of perm).
 * adv_stats = {mean, rstd} of this minibatch (with hp->normalize_values the
 * 8-float record of mlearn_value_norm_chain: the value target is the return
 * normalised with the updated estimates, the value error inverts the critic
 * with the previous ones, ppo.py:190-218).  loss_out (may be NULL) receives
 * 5 x {mean, m2, min, max, count}: 'Loss' {loss,0,loss,loss,1}, 'Action Obj',
 * 'Value Loss', 'Value Errors', 'Entropy' (ppo.py:95-106, 351-362).  With
 * critic_bins > 1 the value loss is the two-hot cross entropy of the returns
 * (ppo.py:169-177, dists.py:171-208); clip/huber value losses need the scalar
 * critic (ppo.py:54-57). */
int mlearn_ppo_minibatch_grad(const mlearn_mlp_policy* policy, const mlearn_rollout_view* ro,
                              const int32_t* mb_seq, int32_t mb_size, const float* adv_stats,
                              const mlearn_ppo_hparams* hp, float* grad, float* loss_out,
                              void* workspace, mlearn_stream_t stream);

/* The fused forward / loss / backward stage of mlearn_ppo_minibatch_grad on
 * its own (one launch): fills the workspace with the weight-gradient
 * operands and the per-tile partials, no reduction into a gradient.  Used to
 * time the dominant kernel (bench.py roofline) and by callers that schedule
 * the reduction themselves.  With env MLEARN_A0_RECOMPUTE=1, bf16 policies
 * with >= 2 layers and obs_dim <= 64 keep the first layer's per-row LayerNorm
 * statistics instead of its post-activation rows (the weight-gradient stage
 * recomputes those). */
int mlearn_ppo_minibatch_fwd_bwd(const mlearn_mlp_policy* policy, const mlearn_rollout_view* ro,
                                 const int32_t* mb_seq, int32_t mb_size, const float* adv_stats,
                                 const mlearn_ppo_hparams* hp, void* workspace,
                                 mlearn_stream_t stream);

/* Parameter layout of the flat f32 buffers (params, grads, Adam m/v):
 * per layer l: W_l [in_l][hidden], ln_scale_l [hidden], ln_bias_l [hidden];
 * then head W [hidden][A+C] (logits then the C = critic_bins critic outputs),
 * head bias [A+C]. */
int64_t mlearn_param_count(const mlearn_mlp_policy* policy);

typedef struct mlearn_optim_state {
    float* params;        /* flat f32 master weights */
    const float* grads;   /* flat f32 (already all-reduced / averaged) */
    float* adam_m;
    float* adam_v;
    const float* init_norms;   /* [num_layers] Frobenius norms of W_l at init */
    int32_t* step;        /* device int32 Adam step counter (optax count) */
    float lr, b1, b2, eps, max_grad_norm;
    int32_t normalize_params;      /* ppo.py:303-310 */
    int32_t normalize_layernorms;  /* ppo.py:312-338 */
    const double* grad_sumsq_part; /* may be NULL: partial sums of grads^2 already produced
                                      by the gradient reduction (grad_sumsq_out); the
                                      clip_by_global_norm norm then comes from them */
    int64_t grad_sumsq_nparts;
    int32_t launch_form;           /* 0 = the library's choice (the split launches: measured
                                      no slower than the fused one on MI355X), 1 = the split
                                      launches (norm partials, Adam, projection), 2 = ONE fused
                                      launch (ABI 21: [norm partials] -> clip + Adam ->
                                      projections + images with in-launch grid barriers;
                                      MLEARN_EINVAL where its one-workgroup-per-CU grid does
                                      not fit the device).  Bit-identical results.  The
                                      workspace must be zeroed once before its first use
                                      (the fused launch's barrier counters). */
    int32_t pad_;
} mlearn_optim_state;

int64_t mlearn_optim_workspace_bytes(const mlearn_mlp_policy* policy);
/* optax.chain(clip_by_global_norm, adam) (ppo.py:84-90, 283-286), then the
 * weight-norm re-projection and LayerNorm renorm (ppo.py:303-338), then the
 * compute-dtype weight copies referenced by `policy` are refreshed. */
int mlearn_optim_step(const mlearn_mlp_policy* policy, const mlearn_optim_state* st,
                      void* workspace, mlearn_stream_t stream);

/* The same optimizer step over the flat f32 parameter vector of ANY policy
 * tree (the torch path of init_training for trees the fused kernels do not
 * implement, e.g. BackboneSeparate, actor_critic.py:247-303): clip by the
 * global gradient norm + Adam (ppo.py:84-90, 283-286), then per projection
 * group normalize_params (ppo.py:303-310: a Dense kernel outside the actor
 * and critic back to its initial Frobenius norm, train_state.py:413-423) or
 * normalize_layernorms (ppo.py:312-338: a LayerNorm's scale and bias scaled
 * together so |scale|^2 + |bias|^2 = features).  groups: DEVICE array. */
typedef struct mlearn_flat_group {
    int64_t offset, count;    /* kernel / LayerNorm scale: [offset, offset + count) */
    int64_t offset2, count2;  /* LayerNorm bias (count2 = 0 for a kernel); kind 3: offset2 =
                                 row stride, count2 = rows */
    int32_t kind;             /* 1: kernel, 2: LayerNorm, 3: kernel held as a column block
                                 of a row-major matrix -- elements offset + r * offset2 + c,
                                 r < count2, c < count (one gate's kernel of an LSTM layer's
                                 concatenated [in][4H] weights: flax OptimizedLSTMCell keeps
                                 each gate's Dense kernel as its own leaf, rnn.py:30-36) */
    int32_t features;         /* LayerNorm: F */
    float init_norm;          /* kernel: its Frobenius norm at initialisation */
    int32_t pad;
} mlearn_flat_group;
typedef struct mlearn_flat_optim {
    float* params;            /* [n] f32 */
    const float* grads;       /* [n] f32 (already all-reduced) */
    float* adam_m;
    float* adam_v;
    int32_t* step;            /* device Adam step counter (optax count) */
    int64_t n;
    const mlearn_flat_group* groups;  /* device, num_groups entries */
    int32_t num_groups;
    float lr, b1, b2, eps, max_grad_norm;
    int32_t normalize_params, normalize_layernorms;
    int32_t skip_nonfinite;   /* 1: a step whose gradient holds a NaN / Inf leaves params,
                                 moments and step unchanged (the projections still run):
                                 DynamicScale's where_finite, ppo.py:288-291 (fp16) */
} mlearn_flat_optim;
int64_t mlearn_flat_optim_workspace_bytes(int64_t n, int32_t num_groups);
int mlearn_flat_optim_step(const mlearn_flat_optim* st, void* workspace, mlearn_stream_t stream);

/* Refresh the compute-dtype copies (w_t, w, head_t, head, head_bias) of
 * `policy` from flat f32 params (used at init and after checkpoint loads). */
int mlearn_policy_sync_weights(const mlearn_mlp_policy* policy, const float* params,
                               mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Recurrent policies: BackboneShared(RecurrentBackboneEncoder(MLP, LSTM))  */
/* (actor_critic.py:156-199, rnn.py:10-111; cell = flax 0.8.1              */
/* OptimizedLSTMCell).  One LSTM layer of width = the MLP hidden width.      */
/* ---------------------------------------------------------------------- */
/* Master parameters: the MLP layout of mlearn_param_count padded to a
 * multiple of 64 floats (mlearn_lstm_param_offset), then Wi [H][4H] (input
 * kernels, no bias), Wh [H][4H] (hidden kernels), bias [4H]; gate blocks
 * (i, f, g, o) concatenated along the output axis.  The compute-dtype
 * images (written by mlearn_lstm_sync_weights / mlearn_lstm_optim_step) use
 * the fragment layout of mlearn_mlp_policy with these logical matrices:
 *   wi_perm, wi_nat, wh_nat: [4H gate columns][H] in unit-block order
 *       n' = (u / 32) * 128 + gate * 32 + u % 32 (u = hidden unit), k = input
 *       unit (wi_perm in the permuted k order of accumulator-fed fragments);
 *   w_bwd: [2H][4H], n = input unit of [x ; h], k = gate * H + u;
 *   head_t_nat: the head [32][H] with natural k order. */
typedef struct mlearn_lstm {
    int32_t hidden;          /* == policy hidden (64, 128 or 256) */
    int32_t num_layers;      /* 1 */
    const void* wi_perm;
    const void* wi_nat;
    const void* wh_nat;
    const void* w_bwd;
    const void* head_t_nat;
    const float* bias;       /* [4H] f32 master bias */
} mlearn_lstm;

/* Carry of the rollout: h, c [N][H] in the compute dtype, in the env order.
 * They hold the cell outputs of the last step; the launch clears them where
 * post->dones (the previous env step) is set before using them
 * (rnn_reset_fn, rollouts.py:942).  start_h / start_c (may be NULL) receive
 * the cleared input carry: the rnn_start_states of a BPTT chunk
 * (rollouts.py:528-537).  commit == 0 (bootstrap critic, rollouts.py:607-635)
 * writes back the cleared carry instead of advancing it. */
typedef struct mlearn_lstm_carry {
    void* h;
    void* c;
    void* start_h;
    void* start_c;
    int32_t commit;
    int32_t pad;
    const uint8_t* clear;    /* may be NULL: [N] extra reset mask, cleared like post->dones
                                (the sequence breaks of ActorCritic.update, rnn.py:92-96) */
} mlearn_lstm_carry;

int64_t mlearn_lstm_param_offset(const mlearn_mlp_policy* policy);
int64_t mlearn_lstm_param_count(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm);

/* mlearn_policy_rollout_step with the LSTM between the trunk and the heads
 * (ActorCritic.rollout with RecurrentBackboneEncoder, actor_critic.py:74-96,
 * 173-177). */
int mlearn_lstm_policy_rollout_step(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                    const mlearn_lstm_carry* carry, const float* obs, int64_t N,
                                    void* obs_store, int32_t* actions, float* log_probs,
                                    float* values, uint32_t k0, uint32_t k1,
                                    const uint64_t* step_ctr, uint64_t step,
                                    uint32_t env_offset, int32_t sample,
                                    const mlearn_post_step* post, mlearn_stream_t stream);

/* ActorCritic.update's forward for a feed-forward policy on a flattened
 * batch of N rows (actor_critic.py:98-128 with DiscreteActionDistributions.
 * action_stats, dists.py:54-77): per sub-action the log-prob of the given
 * action (logits - logsumexp) and the entropy -sum softmax * log_softmax,
 * and the critic output (the scalar value, or the two-hot mean()).  obs is
 * [N][obs_dim] f32 (cast to the compute dtype as in the rollout), actions /
 * log_probs / entropies [N][K]. */
int mlearn_policy_evaluate(const mlearn_mlp_policy* policy, const float* obs, int64_t N,
                           const int32_t* actions, float* log_probs, float* entropies,
                           float* values, mlearn_stream_t stream);
/* One time step of the recurrent ActorCritic.update forward: the carry
 * (cleared first where carry->clear is set) is advanced when carry->commit. */
int mlearn_lstm_policy_evaluate(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                const mlearn_lstm_carry* carry, const float* obs, int64_t N,
                                const int32_t* actions, float* log_probs, float* entropies,
                                float* values, mlearn_stream_t stream);

/* Minibatch gradient of the recurrent policy (ActorCritic.update with
 * RecurrentBackboneEncoder.sequence, actor_critic.py:98-128, 179-199;
 * LSTM.sequence rnn.py:81-111; PPO loss ppo.py:129-262 under
 * jax.value_and_grad): trunk forward over the minibatch rows, the LSTM scan
 * from the sequences' start states clearing the carry after done steps
 * (ro->dones), heads + loss, the reverse (BPTT) scan, trunk backward, weight
 * gradients, reduction into grad[mlearn_lstm_param_count].  start_h /
 * start_c are [C][ld][H] compute-dtype rnn_start_states (ld, C from ro).
 * mb_size and mb_size * bptt_len must be multiples of 32 and 64. */
int64_t mlearn_lstm_ppo_workspace_bytes(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                        int64_t rows, int32_t mb_size);
int mlearn_lstm_ppo_minibatch_grad(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                   const mlearn_rollout_view* ro, const void* start_h,
                                   const void* start_c, const int32_t* mb_seq, int32_t mb_size,
                                   const float* adv_stats, const mlearn_ppo_hparams* hp,
                                   float* grad, float* loss_out, void* workspace,
                                   mlearn_stream_t stream);

/* mlearn_optim_step over the whole recurrent parameter vector: global-norm
 * clip and Adam over every parameter, weight-norm projection of the trunk
 * kernels and of each of the 8 LSTM gate kernels (init_norms = [L + 8]:
 * trunk W_l, Wi gates i f g o, Wh gates i f g o; ppo.py:303-310), LayerNorm
 * renorm, then the compute images of policy and lstm are refreshed. */
int64_t mlearn_lstm_optim_workspace_bytes(const mlearn_mlp_policy* policy,
                                          const mlearn_lstm* lstm);
int mlearn_lstm_optim_step(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                           const mlearn_optim_state* st, void* workspace, mlearn_stream_t stream);
int mlearn_lstm_sync_weights(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                             const float* params, mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Synthetic dummy vec-env (test/bench sim plugin, not part of the         */
/* reference: stands in for the Madrona sim_fns['step'] custom call,       */
/* rollouts.py:905-936).                                                   */
/* ---------------------------------------------------------------------- */
/* state is [N][4] int32 per env: {episode step, env step lo, env step hi, 0}.
 * Episode length of env g = env_offset + n is 16 + (g*7 mod 33) (staggered,
 * deterministic dones).  obs[n][f] = Irwin-Hall(4) approximation of N(0,1)
 * from Philox(ctr={g, f, env step}, key={k0, k1^0x5eed}); reward =
 * U[-1,1) + 0.01*action[n][0].  dones are bytes.  Reset puts every env at
 * episode step g mod L_g and env step 0. */
int mlearn_dummy_env_step(int32_t* state, const int32_t* actions, int32_t K, int64_t N,
                          int32_t obs_dim, uint32_t k0, uint32_t k1, uint32_t env_offset,
                          float* obs, float* rewards, uint8_t* dones, mlearn_stream_t stream);
int mlearn_dummy_env_reset(int32_t* state, int64_t N, int32_t obs_dim, uint32_t k0,
                           uint32_t k1, uint32_t env_offset, float* obs,
                           mlearn_stream_t stream);

/* The same env step fused into the rollout policy launch that produced the
 * actions (no separate sim launch, no host round trip): after the sample,
 * each workgroup advances its own envs from their first action, writing the
 * next observations over the launch's obs input (env->obs must equal obs),
 * rewards and dones (which the NEXT launch's post-step reads: post->rewards /
 * post->dones must be env->rewards / env->dones), bit-identical to
 * mlearn_dummy_env_step on the same actions.  Only for this built-in sim:
 * a user sim plugin keeps its own step between the policy launches. */
typedef struct mlearn_dummy_env {
    int32_t* state;     /* [N][4], 16-byte aligned */
    float* obs;         /* [N][obs_dim] */
    float* rewards;     /* [N] */
    uint8_t* dones;     /* [N] */
    uint32_t k0, k1;    /* env keys (not the policy's sampling keys) */
    uint32_t env_offset;
    uint32_t pad;
} mlearn_dummy_env;
int mlearn_policy_rollout_step_env(const mlearn_mlp_policy* policy, const float* obs, int64_t N,
                                   void* obs_store, int32_t* actions, float* log_probs,
                                   float* values, uint32_t k0, uint32_t k1,
                                   const uint64_t* step_ctr, uint64_t step, uint32_t env_offset,
                                   int32_t sample, const mlearn_post_step* post,
                                   const mlearn_dummy_env* env, mlearn_stream_t stream);
/* The whole rollout of the synthetic sim in ONE launch: for t = 0 .. T-1 the
 * rollout step of mlearn_policy_rollout_step_env (post-step of t-1, policy,
 * sample, store row t, env step), then the bootstrap critic at t = T with the
 * post-step of T-1 (and, for a recurrent policy, the carry cleared where
 * that step ended an episode), each workgroup running every step of its own
 * 32 envs back to back.  Store pointers are [T][ld][...] views of this
 * policy's env columns; bit-identical to T + 1 per-step launches. */
typedef struct mlearn_rollout_out {
    void* obs;                  /* [T][ld][obs_dim] compute dtype, or NULL */
    int32_t* actions;           /* [T][ld][K] */
    float* log_probs;           /* [T][ld][K] */
    float* values;              /* [T][ld] */
    float* rewards;             /* [T][ld] store rewards */
    uint8_t* dones;             /* [T][ld] store dones */
    float* env_returns_trace;   /* [T][ld] or NULL */
    float* bootstrap;           /* [N] critic at t = T */
    float* env_returns;         /* [N] running discounted return (in/out) */
    void* start_h;              /* [C][ld][H] rnn_start_states (recurrent policies) */
    void* start_c;
    int32_t T, bptt_len;
    int64_t ld;
    float gamma;
    int32_t max_workgroups;     /* 0: one workgroup per resident slot (every CU busy; with
                                   more 32-env tiles than slots the tiles are dealt
                                   round-robin, 2-3 in series per workgroup at the headline);
                                   > 0: at most this many workgroups (tiles in series);
                                   < 0: T + 1 per-step launches of the same body (same bits
                                   either way) */
    int32_t policy_kernel;      /* 0: the library's choice (the row-split rollout where it
                                   applies: the row-split step's policy shape (incl. the
                                   two-hot critic at head width 96, ABI 21), <= 8 action
                                   groups, no observation normaliser, max_workgroups 0,
                                   N of exactly 32768 or a multiple of 256 and >= 65536;
                                   else the feature-split
                                   kernel), 1: the feature-split kernel (the per-step
                                   launches' body), 2: the row-split kernel (EINVAL where it
                                   does not apply).  The row split accumulates the trunk and
                                   heads in another order: logits within a bf16 ulp of the
                                   feature split's */
    float* advantages;          /* [T][ld] or NULL (ABI 21): when set, the call also runs GAE
                                   (compute_advantages, algo_common.py:84-130) over the rollout
                                   it just stored -- rewards, values, dones, bootstrap -- writing
                                   the advantages only (returns = advantages + values derived by
                                   their consumers, mlearn_gae_f32 with returns = NULL), with
                                   gae_gamma and the caller's single-rounded gae_gamma_lambda:
                                   fused into the row-split kernel's tile epilogue (T <= 32,
                                   each wave reads back the 16 envs' rows it just wrote), else
                                   a trailing mlearn_gae_f32 launch.  Needs ld == N.  Same bits
                                   as mlearn_gae_f32.  No value normaliser applies here (the
                                   caller inverts normalised values with mlearn_gae_vnorm_f32) */
    float gae_gamma, gae_gamma_lambda;
} mlearn_rollout_out;
int mlearn_policy_rollout_env(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                              const mlearn_lstm_carry* carry, const float* obs, int64_t N,
                              const mlearn_rollout_out* out, uint32_t k0, uint32_t k1,
                              const uint64_t* step_ctr, uint32_t env_offset,
                              const mlearn_dummy_env* env, mlearn_stream_t stream);
/* A population's whole rollouts as ONE launch (replaces the P launches of
 * mlearn_policy_rollout_env a PBT population issues, one per policy's env
 * columns, rollouts.py:501-577 run per policy by the reference's
 * rollout_loop over its policy_assignments): policy p's arguments -- exactly
 * those of its own mlearn_policy_rollout_env call, N envs each, every policy
 * of the same shape, max_workgroups 0 -- are written once into a device
 * buffer of mlearn_policy_pop_bytes(P) bytes by mlearn_policy_pop_prepare
 * (a copy on `stream`, ordered after the work already queued there -- e.g. a
 * previous population launch still reading the buffer -- and complete when
 * the call returns; call it outside stream capture, again whenever one of
 * the pointers changes); mlearn_policy_rollout_env_pop then launches the
 * P * ceil(N / 32) env tiles (global tile g = tile g % ceil(N / 32) of
 * policy g / ceil(N / 32)) dealt round-robin over one workgroup per resident
 * slot, or over at most max_workgroups (> 0) workgroups; a workgroup whose
 * next tile belongs to another policy restages that policy's parameters
 * (capture-safe).  Same bits as the P separate launches.  lstms / carries:
 * arrays of P, or both null for feed-forward policies. */
int64_t mlearn_policy_pop_bytes(int32_t num_policies);
int mlearn_policy_pop_prepare(const mlearn_mlp_policy* policies, const mlearn_lstm* lstms,
                              const mlearn_lstm_carry* carries, const float* const* obs,
                              int64_t N, const mlearn_rollout_out* outs,
                              const uint32_t* env_offsets, const mlearn_dummy_env* envs,
                              int32_t num_policies, void* pop, mlearn_stream_t stream);
int mlearn_policy_rollout_env_pop(const mlearn_mlp_policy* policy0, const mlearn_lstm* lstm0,
                                  const void* pop, int32_t num_policies, int64_t N,
                                  uint32_t k0, uint32_t k1, const uint64_t* step_ctr,
                                  int32_t max_workgroups, mlearn_stream_t stream);
/* The kernel mlearn_policy_rollout_env_pop runs for num_policies x N envs
 * under max_workgroups (host-only, v20): 2 = the row-split rollout (the
 * library's choice when uncapped, the row-split rollout's policy shape --
 * see mlearn_rollout_out.policy_kernel -- with no observation normaliser, N a
 * multiple of 128 and >= 2048 16-env tiles in all: 16-env tiles dealt in
 * rounds of 8 per workgroup, W1 / head / LayerNorm images restaged when a
 * workgroup's round belongs to another policy), 1 = the feature-split
 * population kernel (every other case; max_workgroups > 0 selects it); -1 on a
 * bad argument. */
int32_t mlearn_policy_rollout_pop_kernel(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                         int64_t N, int32_t num_policies, int32_t max_workgroups);
/* Workgroups the feature-split population kernel launches for num_policies x
 * N envs under max_workgroups (>= 0); -1 on a bad argument or a failed
 * occupancy query.  P * ceil(N / 32) > the result means tiles run in series. */
int64_t mlearn_policy_rollout_pop_workgroups(const mlearn_mlp_policy* policy,
                                             const mlearn_lstm* lstm, int64_t N,
                                             int32_t num_policies, int32_t max_workgroups);
/* Workgroups mlearn_policy_rollout_env launches for N envs under
 * max_workgroups (0 = the launch it would issue per-step: -1 means per-step
 * launches are used, i.e. the occupancy query failed or max_workgroups < 0);
 * tiles = ceil(N / 32) > the result means tiles run in series. */
int64_t mlearn_policy_rollout_workgroups(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                         int64_t N, int32_t max_workgroups);
/* The rollout kernel mlearn_policy_rollout_env runs for this policy, N and
 * max_workgroups given mlearn_rollout_out.policy_kernel = requested: 1
 * (feature split; its grid is mlearn_policy_rollout_workgroups) or 2 (row
 * split: one 8-wave workgroup per CU, 16-env tiles in series per wave); -1
 * for an invalid request (host-only). */
int32_t mlearn_policy_rollout_kernel(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                     int64_t N, int32_t max_workgroups, int32_t requested);
int mlearn_lstm_policy_rollout_step_env(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                        const mlearn_lstm_carry* carry, const float* obs,
                                        int64_t N, void* obs_store, int32_t* actions,
                                        float* log_probs, float* values, uint32_t k0, uint32_t k1,
                                        const uint64_t* step_ctr, uint64_t step,
                                        uint32_t env_offset, int32_t sample,
                                        const mlearn_post_step* post, const mlearn_dummy_env* env,
                                        mlearn_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Data-parallel collectives on the compute stream  */
/* ---------------------------------------------------------------------- */
/* The reference is single-device; under data parallelism the build sums the
 * per-minibatch gradient (ppo.py:276-286 runs on the union minibatch) and the
 * per-epoch advantage sums (algo_common.py:133-140 over the union) across
 * the ranks.  An RCCL communicator: rank 0 makes the unique id, the caller
 * distributes it (MLEARN_COMM_ID_BYTES bytes), every rank calls
 * mlearn_comm_init.  The all-reduces are in-place sums enqueued on `stream`
 * (capturable into a HIP graph). */
int mlearn_comm_unique_id(uint8_t* id_out);
int mlearn_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, mlearn_comm_t* comm_out);
int mlearn_comm_destroy(mlearn_comm_t comm);
int mlearn_allreduce_f32(mlearn_comm_t comm, float* buf, int64_t n, mlearn_stream_t stream);
int mlearn_allreduce_f64(mlearn_comm_t comm, double* buf, int64_t n, mlearn_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MLEARN_H */
