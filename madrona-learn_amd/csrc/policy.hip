// Fused rollout step: ObservationsCaster -> MLP trunk (Dense no-bias ->
// LayerNorm -> ReLU per layer) -> actor logits + critic -> Gumbel-max sample
// -> rollout store, in ONE launch per step (the reference runs these as
// dozens of XLA fusions per step inside rollout_loop, rollouts.py:867-901).
//
// Reference numerics mirrored (models.py:46-56, 99-154; flax 0.8.1):
//   Dense output rounded to the compute dtype; LayerNorm statistics in f32
//   with fast variance max(E[x^2]-E[x]^2, 0), eps 1e-6, y = (x-mean)*(rstd*g)+b
//   rounded to the compute dtype; heads: rnd(rnd(x.W) + rnd(b)); critic and
//   logits upcast to f32 (dists.py:22, models.py:154).

#include <vector>

#include "common.h"
#include "dists.h"
#include "env.h"
#include "rowtile.h"
#include "r16_common.h"

namespace ml {

PolicyK make_policy_k(const mlearn_mlp_policy& p) {
    PolicyK k;
    k.D = p.obs_dim;
    k.H = p.hidden;
    k.L = p.num_layers;
    k.K = p.actions.num_groups;
    k.A = p.actions.num_logits;
    k.CB = p.critic_bins;
    k.HC = head_cols(p);
    for (int i = 0; i <= MLEARN_MAX_GROUPS; ++i) k.off[i] = p.actions.offsets[i];
    for (int l = 0; l < MLEARN_MAX_LAYERS; ++l) {
        k.wt[l] = p.w_t[l];
        k.w[l] = p.w[l];
        k.lns[l] = p.ln_scale[l];
        k.lnb[l] = p.ln_bias[l];
    }
    k.head_t = p.head_t;
    k.head = p.head;
    k.head_b = p.head_bias;
    k.obs_mu = p.obs_mu;
    k.obs_inv = p.obs_inv_sigma;
    k.obs_stats = p.obs_stats;
    k.obs_tiles = p.obs_stats_tiles;
    k.obs_steps = p.obs_stats_steps;
    return k;
}

int validate_policy(const mlearn_mlp_policy* p) {
    ML_REQUIRE(p, "policy: null descriptor");
    ML_REQUIRE(p->dtype == MLEARN_DTYPE_F32 || p->dtype == MLEARN_DTYPE_BF16, "policy: bad dtype");
    ML_REQUIRE(p->hidden == 64 || p->hidden == 128 || p->hidden == 256,
               "policy: hidden must be 64, 128 or 256 (got %d)", p->hidden);
    ML_REQUIRE(p->obs_dim >= 16 && p->obs_dim <= 256 && p->obs_dim % 16 == 0,
               "policy: obs_dim must be a multiple of 16 in [16, 256] (got %d)", p->obs_dim);
    ML_REQUIRE(p->num_layers >= 1 && p->num_layers <= MLEARN_MAX_LAYERS, "policy: bad num_layers");
    const mlearn_action_layout& l = p->actions;
    ML_REQUIRE(l.num_groups >= 1 && l.num_groups <= MLEARN_MAX_GROUPS, "policy: bad num_groups");
    ML_REQUIRE(p->critic_bins == 1 || (p->critic_bins >= 3 && p->critic_bins % 2 == 1),
               "policy: critic_bins must be 1 (scalar critic) or odd >= 3 (two-hot), got %d",
               p->critic_bins);
    ML_REQUIRE(l.num_logits >= 1 && l.num_logits + p->critic_bins <= MLEARN_HEAD_COLS_MAX,
               "policy: actor logits + critic outputs must be <= %d (got %d + %d)",
               MLEARN_HEAD_COLS_MAX, l.num_logits, p->critic_bins);
    ML_REQUIRE(l.offsets[0] == 0 && l.offsets[l.num_groups] == l.num_logits,
               "policy: bad action offsets");
    for (int k = 0; k < l.num_groups; ++k)
        ML_REQUIRE(l.offsets[k + 1] > l.offsets[k], "policy: empty action group %d", k);
    for (int i = 0; i < p->num_layers; ++i)
        ML_REQUIRE(p->w_t[i] && (i == 0 || p->w[i]) && p->ln_scale[i] && p->ln_bias[i],
                   "policy: null layer %d weights", i);
    ML_REQUIRE(p->head_t && p->head && p->head_bias, "policy: null head weights");
    ML_REQUIRE(!p->obs_mu == !p->obs_inv_sigma, "policy: obs_mu / obs_inv_sigma");
    ML_REQUIRE(!p->obs_stats || (p->obs_stats_steps >= 1 && p->obs_stats_tiles >= 1),
               "policy: obs_stats needs obs_stats_steps and obs_stats_tiles");
    return MLEARN_OK;
}

// Post-step of the previous env step, fused into the next policy launch.
struct PostK {
    const float* rew;
    const uint8_t* done;
    float* srew;
    uint8_t* sdone;
    float* env_ret;
    float* trace;
    float gamma;
};

// rollouts.py:933-973: store reward/done, env_returns = r + gamma * env_returns
// (traced for the 'Env Returns' metric), zeroed where done.
__device__ inline void post_step_row(const PostK& p, int64_t n) {
#pragma clang fp contract(off)
    const float r = p.rew[n];
    const uint8_t d = p.done[n] ? 1 : 0;
    const float er = r + p.gamma * p.env_ret[n];
    if (p.trace) p.trace[n] = er;
    p.srew[n] = r;
    p.sdone[n] = d;
    p.env_ret[n] = d ? 0.f : er;
}

// One workgroup = 32 environments (one per lane pair); its W waves split the
// hidden features (wave w owns blocks w*NBW .. w*NBW+NBW-1 of every layer).
// Per layer: each wave's MFMAs over the full input (B fragments from LDS),
// LayerNorm statistics combined across the waves through LDS, and the
// post-activation fragments written back to LDS for the next layer.  The
// heads split the reduction instead: each wave multiplies its own features,
// partials are summed in wave order.
#ifndef ML_POL_MAXW
#define ML_POL_MAXW 4  // waves per workgroup, feed-forward policy (feature split; 8 measured 54.3 vs 42.4 us)
#endif
#ifndef ML_POL_RNN_MAXW
#define ML_POL_RNN_MAXW 8  // waves per workgroup, recurrent policy (4: 284 VGPRs, one wave per SIMD)
#endif
#ifndef ML_ROLL_MLP_WAVES
#define ML_ROLL_MLP_WAVES 3  // whole-rollout kernel, feed-forward: 3 waves per SIMD (3 workgroups per CU)
#endif
#ifndef ML_ROLL_RNN_WAVES
#define ML_ROLL_RNN_WAVES 3  // whole-rollout kernel, recurrent: 3 waves per SIMD (no spill; 4: 11.71 vs 11.65 ms)
#endif
template <int H, int MAXW = ML_POL_MAXW> struct PolCfg {
    static constexpr int NB = H / 32;
    static constexpr int W = NB < MAXW ? NB : MAXW;
    static constexpr int NBW = NB / W;
};
// The feature split of a policy kernel (the per-step and the whole-rollout
// kernels use the same one, so they compute the same bits).
template <bool RNN> constexpr int pol_maxw() { return RNN ? ML_POL_RNN_MAXW : ML_POL_MAXW; }
template <int H, bool RNN> constexpr int pol_threads() { return 64 * PolCfg<H, pol_maxw<RNN>()>::W; }

// Carry of a recurrent policy (mlearn_lstm_carry).
struct CarryK {
    void* h;
    void* c;
    void* sh;
    void* sc;
    int commit;
    const uint8_t* clear;  // extra reset mask (ActorCritic.update's sequence breaks)
};

// ActorCritic.update forward (evaluate mode): given actions in, per
// sub-action entropies out (log-probs go to logp).
struct EvalK {
    const int32_t* actions;
    float* entropies;
    uint64_t* stamps;  // diagnostic builds only (ML_STAMPS): [blocks][W][16]
};

#ifdef ML_STAMPS
static uint64_t* g_pol_stamp_buf = nullptr;
#define PSTAMP(i)                                                                      \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        if (ev.stamps && actions && lane == 0)                                         \
            ev.stamps[((int64_t)tile * W + w) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
        __builtin_amdgcn_sched_barrier(0);                                             \
    } while (0)
#else
#define PSTAMP(i) \
    do {          \
    } while (0)
#endif

// RNN: the LSTM cell (RecurrentBackboneEncoder, actor_critic.py:173-177)
// sits between the trunk and the heads.  The trunk output fragments (from
// the accumulators, permuted k order) and the carry rows (from HBM, natural k
// order) are staged in LDS; each wave computes the 4 gates of its own 64
// hidden units (8 accumulator blocks, weight images in unit-block gate
// order), so the cell update is register-local and h' lands in exactly the
// layout the heads consume.
template <typename T, int H, bool RNN, int HC, int MAXW, bool STAGED = false>
#ifndef ML_POL_WAVES
#define ML_POL_WAVES 1  // waves per SIMD the recurrent rollout policy kernel is register-budgeted for (1: compiler choice)
#endif
#ifndef ML_POL_MLP_WAVES
#define ML_POL_MLP_WAVES 3  // the feed-forward kernel: 3 waves per SIMD (<= 168 VGPRs, 3 workgroups per CU)
#endif
__device__ __forceinline__ void policy_step_body(
    const PolicyK& P, const float* __restrict__ obs, int64_t N, T* obs_store, int32_t* actions,
    float* logp, float* values, uint32_t k0, uint32_t k1, const uint64_t* step_ctr,
    uint64_t step_add, uint32_t eoff, int sample, const PostK& post, const LstmK& R,
    const CarryK& cy, const EvalK& ev, const EnvK& env, int tile) {
    typedef typename RT<T>::frag frag;
    typedef PolCfg<H, MAXW> C;
    constexpr int NBW = C::NBW, W = C::W, THREADS = 64 * W;
    constexpr int E = RT<T>::E, KS = RT<T>::KS, SPB = RT<T>::SPB, KSH = H / KS;
    constexpr int KSD = 256 / KS;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D, L = P.L;
    // (opaque copy of the lane index: in the rollout kernel's step loop the
    // body's lane-derived addresses are then recomputed per step instead of
    // hoisted out of the loop and held live across it)
    int tid_o = (int)threadIdx.x;
    asm volatile("" : "+v"(tid_o));
    const int tid = tid_o, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR) for the buffer descriptors
    frag* fr = (frag*)smem;                               // [KSH][64] B fragments
    float* gb = (float*)(fr + KSH * 64);                  // [L][2][H]
    constexpr int LGS = HC + 1;                           // LDS row stride of the head outputs
    float* hbias = gb + L * 2 * H;                        // [HC]
    float* red = hbias + HC;                              // [W][32][2]
    float* lgp = red + W * 64;                            // [head_parts][32][LGS] partials
    float* lg = lgp + head_parts<HC, W>() * 32 * LGS;     // [32][LGS]
    float* rbias = lg + 32 * LGS;                         // [4H] LSTM bias (RNN)
    float* bins = rbias + (RNN ? 4 * H : 0);              // [HC] two-hot critic bins
    frag* frh = (frag*)(bins + HC);                       // [KSH][64] carry fragments (RNN)
    // LayerNorm / head-bias parameters: loads issued now, written to LDS after
    // the first product (their latency hides under the observation loads)
    // (STAGED: the whole-rollout kernel staged them once, before its step loop)
    constexpr int NPAR = STAGED ? 1 : (MLEARN_MAX_LAYERS * 2 * H + HC + THREADS - 1) / THREADS;
    float parv[NPAR];
    if constexpr (!STAGED) {
#pragma unroll
        for (int k = 0; k < NPAR; ++k) {
            const int i = tid + k * THREADS;
            float v = 0.f;
            if (i < L * 2 * H) {
                const int l = i / (2 * H), c = i - l * 2 * H;
                v = c < H ? P.lns[l][c] : P.lnb[l][c - H];
            } else if (i < L * 2 * H + HC) {
                v = P.head_b[i - L * 2 * H];
            }
            parv[k] = v;
        }
        if constexpr (RNN)
            for (int i = tid; i < 4 * H; i += THREADS) rbias[i] = R.bias[i];
        if (P.CB > 1)
            for (int i = tid; i < P.CB; i += THREADS) bins[i] = twohot_bin(i, P.CB);
    }
    const int64_t row0 = (int64_t)tile * 32;
    const int64_t row = row0 + r;
    const bool live = row < N;
    if (post.rew && tid < 32 && row0 + tid < N) post_step_row(post, row0 + tid);
    const uint64_t step = (step_ctr ? *step_ctr : 0ull) + step_add;
    const float invH = 1.0f / (float)H;
    PSTAMP(0);

    // layer 0: observation fragments straight from the env output (cast to
    // the compute dtype = ObservationsCaster); wave 0 copies them to the store
    // the second layer's weights (this wave's blocks) are in flight from the start
#ifndef ML_POL_W1_RING
#define ML_POL_W1_RING 8  // k-steps of the second layer's weights in flight from the start (0: all)
#endif
    constexpr int W1R = ML_POL_W1_RING > 0 && ML_POL_W1_RING < KSH ? ML_POL_W1_RING : KSH;
    frag w1[W1R][NBW];
    if (L > 1) {
        if constexpr (W1R == KSH)
            prefetch_img<T, NBW, KSH>(w1, (const T*)P.wt[1] + (int64_t)w * NBW * KSH * 64 * E, lane);
        else
            gemm_lds_issue<T, NBW, KSH, W1R>(w1, (const T*)P.wt[1] + (int64_t)w * NBW * KSH * 64 * E,
                                             lane);
    }
    f32x16 acc[NBW];
    zero_acc<NBW>(acc);
    gemm_first<T, NBW>(acc, obs + (live ? row : 0) * D, live, D / KS,
                       (const T*)P.wt[0] + (int64_t)w * NBW * (D / KS) * 64 * E,
                       (w == 0 && obs_store && live) ? obs_store + row * D : nullptr, lane,
                       P.obs_mu, P.obs_inv);
    PSTAMP(1);
    if constexpr (!STAGED) {
#pragma unroll
        for (int k = 0; k < NPAR; ++k)
            if (tid + k * THREADS < L * 2 * H + HC) gb[tid + k * THREADS] = parv[k];
    }
    // LayerNorm parameters staged: the first LayerNorm's statistics barrier
    // orders them (and the LSTM bias / critic bins) before their first read
    typedef typename Pk<T>::word word;
    word aw[NBW][8];
    for (int l = 0;; ++l) {
        // LayerNorm + ReLU (models.py:46-56); row statistics over all waves
        f2 x2[NBW][8];
        word zw[NBW][8];
        float sum, sq;
        ln_pack_stats<T, NBW>(acc, zw, x2, sum, sq);
        sum = sum_halves(sum);
        sq = sum_halves(sq);
        if (h == 0) {
            red[(w * 32 + r) * 2] = sum;
            red[(w * 32 + r) * 2 + 1] = sq;
        }
        __syncthreads();
        sum = red[r * 2];
        sq = red[r * 2 + 1];
#pragma unroll
        for (int v = 1; v < W; ++v) {
            sum += red[(v * 32 + r) * 2];
            sq += red[(v * 32 + r) * 2 + 1];
        }
        const float mean = sum * invH;
        const float var = fmaxf(sq * invH - mean * mean, 0.f);
        const float rstd = rsqrtf(var + 1e-6f);
        PSTAMP(2 + 2 * (l < 1 ? l : 1));
        ln_apply<T, NBW>(x2, mean, rstd, gb + l * 2 * H, H, w * NBW, h, aw);
        if (l + 1 == L && !RNN) break;
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
            for (int t = 0; t < SPB; ++t)
                fr[((w * NBW + i) * SPB + t) * 64 + lane] = Pk<T>::frag(aw[i], t);
        if (l + 1 == L) break;
        __syncthreads();
        zero_acc<NBW>(acc);
        if (l == 0)
        {
            if constexpr (W1R == KSH)
                gemm_pre_lds<T, NBW, KSH>(acc, w1, fr, lane);
            else
                gemm_lds_run<T, NBW, KSH, W1R>(acc, w1, fr,
                                               (const T*)P.wt[1] + (int64_t)w * NBW * KSH * 64 * E,
                                               lane);
        }
        else
            gemm_lds<T, NBW, KSH, 8>(acc, fr,
                                     (const T*)P.wt[l + 1] + (int64_t)w * NBW * KSH * 64 * E, lane);
        PSTAMP(3);
    }
    PSTAMP(5);

    if constexpr (RNN) {
        // carry rows, cleared where the previous env step was done (rollouts.py:942)
        const bool clr = live && ((post.rew && post.done[row] != 0) ||
                                  (cy.clear && cy.clear[row] != 0));
        const T* hrow = (const T*)cy.h + (live ? row : 0) * H;
        constexpr int SPW = KSH / W;  // k-steps staged per wave
#pragma unroll
        for (int ss = 0; ss < SPW; ++ss) {
            const int s = w * SPW + ss;
            frh[s * 64 + lane] = (live && !clr) ? RT<T>::row(hrow, s, h) : RT<T>::zero();
        }
        __syncthreads();
        constexpr int NG = NBW * 4;
        f32x16 g8[NG];
        zero_acc<NG>(g8);
        gemm_lds<T, NG, KSH, 2>(g8, fr, (const T*)R.wi_perm + (int64_t)w * NG * KSH * 64 * E, lane);
        gemm_lds<T, NG, KSH, 2>(g8, frh, (const T*)R.wh_nat + (int64_t)w * NG * KSH * 64 * E, lane);
        T* hs = (T*)cy.h + row * H;
        T* cs = (T*)cy.c + row * H;
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int u0 = (w * NBW + i) * 32 + 8 * j + 4 * h;  // units of regs 4j .. 4j+3
                float4 hin = make_float4(0.f, 0.f, 0.f, 0.f), cin = hin;
                if (live && !clr) {
                    hin = load4(hs + u0);
                    cin = load4(cs + u0);
                }
                float hn[4], cn[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int q = 4 * j + e, u = u0 + e;
                    const CellOut o = lstm_cell_fwd<T>(
                        g8[i * 4 + 0][q] + rbias[u], g8[i * 4 + 1][q] + rbias[H + u],
                        g8[i * 4 + 2][q] + rbias[2 * H + u], g8[i * 4 + 3][q] + rbias[3 * H + u],
                        f4get(cin, e));
                    hn[e] = o.h;
                    cn[e] = o.c;
                }
                if (live) {
                    if (cy.sh) {
                        store4((T*)cy.sh + row * H + u0, hin.x, hin.y, hin.z, hin.w);
                        store4((T*)cy.sc + row * H + u0, cin.x, cin.y, cin.z, cin.w);
                    }
                    if (cy.commit) {
                        store4(hs + u0, hn[0], hn[1], hn[2], hn[3]);
                        store4(cs + u0, cn[0], cn[1], cn[2], cn[3]);
                    } else if (clr) {
                        store4(hs + u0, 0.f, 0.f, 0.f, 0.f);
                        store4(cs + u0, 0.f, 0.f, 0.f, 0.f);
                    }
                }
                aw[i][2 * j] = Pk<T>::pack(hn[0], hn[1]);
                aw[i][2 * j + 1] = Pk<T>::pack(hn[2], hn[3]);
            }
        }
    }

    // fused env step (mlearn_policy_rollout_step_env): the next observations
    // depend only on the env state, not on the actions, so they are drawn
    // here, behind the trunk, and stored once every wave is past its reads of
    // this launch's observation rows (after the heads' barrier; with the
    // observation statistics, which read the rows last, at the end)
    const bool fenv = env.state && actions;
    const int EQ = D >> 2;  // quads per env (D is a multiple of 16)
    constexpr int kEnvQ = 2;  // quads per thread drawn early (32 * EQ <= kEnvQ * THREADS)
    const bool env_early = fenv && 32 * EQ <= kEnvQ * THREADS;
    float4 enq[kEnvQ];
    if (env_early) {
#pragma unroll
        for (int u = 0; u < kEnvQ; ++u) {
            const int task = tid + u * THREADS, rr = task / EQ, q = task - rr * EQ;
            const int64_t n = row0 + rr;
            if (task < 32 * EQ && n < N) {
                const u32x4 wv = env_obs_words(env.k0, env.k1, env.eoff + (uint32_t)n, q,
                                               env_step_of(env.state[n]));
                enq[u] = make_float4(env_obs_word(wv.x), env_obs_word(wv.y), env_obs_word(wv.z),
                                     env_obs_word(wv.w));
            }
        }
    }
    auto env_store_obs = [&]() {
#pragma unroll
        for (int u = 0; u < kEnvQ; ++u) {
            const int task = tid + u * THREADS, rr = task / EQ, q = task - rr * EQ;
            const int64_t n = row0 + rr;
            if (task < 32 * EQ && n < N) *(float4*)(env.obs + n * D + 4 * q) = enq[u];
        }
    };

    // actor + critic heads (dists.py:22, models.py:154): lg[row][j] =
    // rnd(rnd(a . W) + rnd(b)).  Head width 32: each wave multiplies its own
    // features (B fragments from registers), partials summed in wave order.
    // Head width 96: the features of every wave staged in LDS, wave w computes
    // column block w / KSPLIT over k-slice w % KSPLIT.
    {
        constexpr int HB = HC / 32;
        constexpr int KSPLIT = head_parts<HC, W>();
        constexpr int KPS = KSH / KSPLIT;
        if constexpr (HB == 1) {
            frag hb[NBW * SPB];
#pragma unroll
            for (int i = 0; i < NBW; ++i)
#pragma unroll
                for (int t = 0; t < SPB; ++t) hb[i * SPB + t] = Pk<T>::frag(aw[i], t);
            f32x16 ha[1];
            zero_acc<1>(ha);
            gemm_ring<T, 1, NBW * SPB, NBW * SPB < 8 ? NBW * SPB : 8>(
                ha, hb, NBW * SPB, (const T*)P.head_t + (int64_t)w * NBW * SPB * 64 * E, lane);
#pragma unroll
            for (int q = 0; q < 16; ++q) lgp[(w * 32 + r) * LGS + feat(0, q, h)] = ha[0][q];
        } else {
            if constexpr (RNN) __syncthreads();  // every wave is done reading fr (Wi product)
#pragma unroll
            for (int i = 0; i < NBW; ++i)
#pragma unroll
                for (int t = 0; t < SPB; ++t)
                    fr[((w * NBW + i) * SPB + t) * 64 + lane] = Pk<T>::frag(aw[i], t);
            __syncthreads();
            for (int u = w; u < HB * KSPLIT; u += W) {
                const int nb = u / KSPLIT, part = u % KSPLIT;
                f32x16 ha[1];
                zero_acc<1>(ha);
                gemm_lds<T, 1, KPS, 8>(ha, fr + part * KPS * 64,
                                       (const T*)P.head_t + ((int64_t)nb * KSH + part * KPS) * 64 * E,
                                       lane);
#pragma unroll
                for (int q = 0; q < 16; ++q) lgp[(part * 32 + r) * LGS + feat(nb, q, h)] = ha[0][q];
            }
        }
        __syncthreads();
        for (int i = tid; i < 32 * HC; i += THREADS) {
            const int rr = i / HC, j = i - rr * HC;
            float x = lgp[rr * LGS + j];
#pragma unroll
            for (int v = 1; v < KSPLIT; ++v) x += lgp[(v * 32 + rr) * LGS + j];
            lg[rr * LGS + j] = rnd<T>(rnd<T>(x) + rnd<T>(hbias[j]));
        }
        __syncthreads();
    }
    if (env_early && !P.obs_stats) env_store_obs();
    PSTAMP(6);

    // sample + store.  Gumbel noise first, one Philox block per 4 logits of a
    // row ((env, logit quad) tasks; the head partials' LDS is free now), then
    // one (env, group) task per thread: argmax of the perturbed logits,
    // log-prob from the logits (bit-identical to sample_group, dists.h)
    if (actions) {
        float* nz = lgp;  // [32][LGS] perturbed logits
        if (sample) {
            const int nq = (P.A + 3) >> 2;
            for (int task = tid; task < 32 * nq; task += THREADS) {
                const int rr = task / nq, q = task - rr * nq;
                const int64_t n = row0 + rr;
                if (n >= N) continue;
                const u32x4 u = philox4x32(
                    u32x4{eoff + (uint32_t)n, (uint32_t)q, (uint32_t)step, (uint32_t)(step >> 32)},
                    k0, k1);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = 4 * q + e;
                    if (j < P.A)
                        nz[rr * LGS + j] = lg[rr * LGS + j] + det_gumbel(u32_to_unit(u32x4_get(u, e)));
                }
            }
            __syncthreads();
        }
        PSTAMP(7);
        for (int task = tid; task < 32 * P.K; task += THREADS) {
            const int rr = task / P.K, g = task - rr * P.K;
            const int64_t n = row0 + rr;
            if (n >= N) continue;
            int a;
            float lp;
            pick_group(lg + rr * LGS + P.off[g], sample ? nz + rr * LGS + P.off[g] : nullptr,
                       P.off[g + 1] - P.off[g], &a, &lp);
            actions[n * P.K + g] = a;
            if (logp) logp[n * P.K + g] = lp;
            // fused env: reward, done and state advance of env n from its first
            // action (every lane's state read above is behind the heads' barrier)
            if (fenv && g == 0) {
                const int4 st = env.state[n];
                if (!env_early) {  // the late observation draws read the pre-step counter here
                    ((uint32_t*)red)[2 * rr] = (uint32_t)st.y;
                    ((uint32_t*)red)[2 * rr + 1] = (uint32_t)st.z;
                }
                env_advance_a0(env.state, n, env.eoff + (uint32_t)n, env.k0, env.k1, (float)a,
                               env.rew, env.done, st);
            }
        }
        PSTAMP(8);
    } else if (ev.actions) {
        for (int task = tid; task < 32 * P.K; task += THREADS) {
            const int rr = task / P.K, g = task - rr * P.K;
            const int64_t n = row0 + rr;
            if (n >= N) continue;
            float lp, ent;
            eval_group(lg + rr * LGS + P.off[g], P.off[g + 1] - P.off[g], ev.actions[n * P.K + g],
                       &lp, &ent);
            logp[n * P.K + g] = lp;
            ev.entropies[n * P.K + g] = ent;
        }
    }
    // observation statistics of this step (update_obs_stats, rollouts.py:670-676):
    // the tile's {mean, M2} of the raw observations per feature, 4 lanes per
    // feature (rows q, q + 4, ...), two passes
    if (P.obs_stats && actions && step_add < (uint64_t)P.obs_steps) {
        const int nrow = (int)(N - row0 < 32 ? N - row0 : 32);
        float* out = P.obs_stats + ((int64_t)step_add * P.obs_tiles + tile) * D * 2;
        for (int f0 = 0; f0 < D; f0 += THREADS / 4) {
            const int f = f0 + tid / 4, q = tid % 4;
            const float* col = obs + row0 * D + (f < D ? f : 0);
            float sx = 0.f;
            for (int rr = q; rr < nrow; rr += 4) sx += col[(int64_t)rr * D];
            const float mean = group_sum<4>(sx) / (float)nrow;
            float m2 = 0.f;
            for (int rr = q; rr < nrow; rr += 4) {
                const float d = col[(int64_t)rr * D] - mean;
                m2 += d * d;
            }
            m2 = group_sum<4>(m2);
            if (q == 0 && f < D) {
                out[f * 2] = mean;
                out[f * 2 + 1] = m2;
            }
        }
    }
    if (values) {
        if (P.CB == 1) {
            if (tid < 32 && row0 + tid < N) values[row0 + tid] = lg[tid * LGS + P.A];
        } else {
            // SymExpTwoHotDistribution.mean() (rollouts.py:601-605): 8 lanes per env
            constexpr int G = 8;
            for (int vt = tid; vt < 32 * G; vt += THREADS) {
                const int rr = vt / G, sub = vt % G;
                float mx, se;
                const float v = twohot_mean_g<G>(lg + rr * LGS + P.A, P.CB, bins, sub, &mx, &se);
                if (sub == 0 && row0 + rr < N) values[row0 + rr] = v;
            }
        }
    }
    // fused env, late path: observation statistics read this launch's rows
    // last, or the observation is too wide for the early draws
    if (fenv && (P.obs_stats || !env_early)) {
        __syncthreads();
        if (env_early) {
            env_store_obs();
        } else {
            // pre-step counters from the pick loop (LDS)
            const uint32_t* sc = (const uint32_t*)red;
            for (int task = tid; task < 32 * EQ; task += THREADS) {
                const int rr = task / EQ, q = task - rr * EQ;
                const int64_t n = row0 + rr;
                if (n >= N) continue;
                const uint64_t step = ((uint64_t)sc[2 * rr + 1] << 32) | sc[2 * rr];
                env_obs_quad(env.obs + n * D + 4 * q, D, env.k0, env.k1, env.eoff + (uint32_t)n, q,
                             step, true);
            }
        }
    }
    PSTAMP(9);
}

template <typename T, int H, bool RNN, int HC>
__global__ __launch_bounds__((pol_threads<H, RNN>())) __attribute__((amdgpu_waves_per_eu(RNN ? ML_POL_WAVES : ML_POL_MLP_WAVES, 8))) void policy_step_kernel(
    PolicyK P, const float* __restrict__ obs, int64_t N, T* obs_store, int32_t* actions,
    float* logp, float* values, uint32_t k0, uint32_t k1, const uint64_t* step_ctr,
    uint64_t step_add, uint32_t eoff, int sample, PostK post, LstmK R, CarryK cy, EvalK ev,
    EnvK env) {
    policy_step_body<T, H, RNN, HC, pol_maxw<RNN>()>(P, obs, N, obs_store, actions, logp, values, k0, k1,
                                                 step_ctr, step_add, eoff, sample, post, R, cy, ev,
                                                 env, blockIdx.x);
}

// Whole rollout of the built-in synthetic sim in one launch
// (mlearn_policy_rollout_env): the sim step depends only on its own env, so a
// workgroup runs all T steps of its 32 envs back to back — policy step t
// (with the post-step of t - 1 and the fused env step), then the bootstrap
// critic at t = T — and takes its next env tile after that.  Identical
// per-step arithmetic and counters to T + 1 launches of policy_step_kernel.
struct RollK {
    void* obs;           // [T][ld][D] store rows (compute dtype) or null
    int32_t* actions;    // [T][ld][K]
    float* logp;         // [T][ld][K]
    float* values;       // [T][ld]
    float* rewards;      // [T][ld] store rewards
    uint8_t* dones;      // [T][ld] store dones
    float* trace;        // [T][ld] env-return trace or null
    float* bootstrap;    // [N]
    float* env_returns;  // [N]
    void* start_h;       // [C][ld][H] rnn start states (recurrent)
    void* start_c;
    int T, bptt;
    int64_t ld;
    float gamma;
    int max_wg;          // mlearn_rollout_out.max_workgroups
    float* adv;          // [T][ld] GAE advantages fused into the row-split epilogue, or null
    float gae_gamma, gae_gl;
};

#include "rollout_rows16.h"

// LayerNorm / head-bias parameters, LSTM bias, critic bins of policy P
// staged in LDS for every step of a tile (the body's first statistics
// barrier orders them)
template <typename T, int H, bool RNN, int HC>
__device__ inline void rollout_stage(const PolicyK& P, const LstmK& R) {
    constexpr int THREADS = pol_threads<H, RNN>();
    constexpr int KSH = H / RT<T>::KS;
    constexpr int LGS = HC + 1;
    constexpr int W = THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* gb = (float*)((typename RT<T>::frag*)smem + KSH * 64);
    float* hbias = gb + P.L * 2 * H;
    float* rbias = hbias + HC + W * 64 + head_parts<HC, W>() * 32 * LGS + 32 * LGS;
    float* bins = rbias + (RNN ? 4 * H : 0);
    const int tid = threadIdx.x;
    for (int i = tid; i < P.L * 2 * H + HC; i += THREADS) {
        float v;
        if (i < P.L * 2 * H) {
            const int l = i / (2 * H), c = i - l * 2 * H;
            v = c < H ? P.lns[l][c] : P.lnb[l][c - H];
        } else {
            v = P.head_b[i - P.L * 2 * H];
        }
        gb[i] = v;
    }
    if constexpr (RNN)
        for (int i = tid; i < 4 * H; i += THREADS) rbias[i] = R.bias[i];
    if (P.CB > 1)
        for (int i = tid; i < P.CB; i += THREADS) bins[i] = twohot_bin(i, P.CB);
}

// All T steps + the bootstrap of one 32-env tile (first: the workgroup's
// first tile, whose step 0 needs no leading barrier; RESTAGE: a later tile
// may belong to another policy, whose parameters are staged after that
// barrier).
template <typename T, int H, bool RNN, int HC, bool RESTAGE>
__device__ inline void rollout_tile(const PolicyK& P, const float* __restrict__ obs, int64_t N,
                                    const RollK& rk, uint32_t k0, uint32_t k1,
                                    const uint64_t* step_ctr, uint32_t eoff, const LstmK& R,
                                    const CarryK& cy0, const EnvK& env, int tile, bool first) {
#pragma clang loop unroll(disable)
    for (int t = 0; t <= rk.T; ++t) {
        // the previous step's LDS reads (and its env outputs, read by this
        // step's post-step and first product) are ordered by the barrier
        if (t > 0 || !first) __syncthreads();
        if (RESTAGE && t == 0 && !first) rollout_stage<T, H, RNN, HC>(P, R);
        const bool act = t < rk.T;
        const int64_t so = (int64_t)t * rk.ld;
        PostK post{};
        if (t > 0)
            post = PostK{env.rew, env.done, rk.rewards + so - rk.ld, rk.dones + so - rk.ld,
                         rk.env_returns, rk.trace ? rk.trace + so - rk.ld : nullptr, rk.gamma};
        CarryK cy = cy0;
        if constexpr (RNN) {
            const bool cs = act && t % rk.bptt == 0;
            const int64_t co = (int64_t)(t / rk.bptt) * rk.ld * H;
            cy.sh = cs ? (void*)((T*)rk.start_h + co) : nullptr;
            cy.sc = cs ? (void*)((T*)rk.start_c + co) : nullptr;
            cy.commit = act ? 1 : 0;
        }
        policy_step_body<T, H, RNN, HC, pol_maxw<RNN>(), true>(
            P, obs, N, (act && rk.obs) ? (T*)rk.obs + so * P.D : nullptr,
            act ? rk.actions + so * P.K : nullptr, act ? rk.logp + so * P.K : nullptr,
            act ? rk.values + so : rk.bootstrap, k0, k1, step_ctr, (uint64_t)t, eoff, 1, post,
            R, cy, EvalK{}, act ? env : EnvK{}, tile);
    }
}

template <typename T, int H, bool RNN, int HC>
__global__ __launch_bounds__((pol_threads<H, RNN>())) __attribute__((amdgpu_waves_per_eu(RNN ? ML_ROLL_RNN_WAVES : ML_ROLL_MLP_WAVES, 8))) void policy_rollout_kernel(
    PolicyK P, const float* __restrict__ obs, int64_t N, RollK rk, uint32_t k0, uint32_t k1,
    const uint64_t* step_ctr, uint32_t eoff, LstmK R, CarryK cy0, EnvK env) {
    const int ntiles = (int)((N + 31) / 32);
    rollout_stage<T, H, RNN, HC>(P, R);  // once: every tile has the same policy
    for (int tile = blockIdx.x; tile < ntiles; tile += (int)gridDim.x)
        rollout_tile<T, H, RNN, HC, false>(P, obs, N, rk, k0, k1, step_ctr, eoff, R, cy0, env,
                                           tile, tile == (int)blockIdx.x);
}

// A population's whole rollouts in one launch (mlearn_policy_rollout_env_pop):
// policy p's launch arguments are entry p of a device array written once by
// mlearn_policy_pop_prepare; global tile g is tile g % tpp of policy g / tpp,
// dealt round-robin over one workgroup per resident slot like the
// single-policy launch, so P launches of B / 32 workgroups become one launch
// that fills the chip.  Per tile the same body and arguments as policy p's own
// launch: the same bits.
struct PopEntry {
    PolicyK P;
    const float* obs;
    RollK rk;
    uint32_t eoff;
    LstmK R;
    CarryK cy;
    EnvK env;
};

template <typename T, int H, bool RNN, int HC>
__global__ __launch_bounds__((pol_threads<H, RNN>())) __attribute__((amdgpu_waves_per_eu(RNN ? ML_ROLL_RNN_WAVES : ML_ROLL_MLP_WAVES, 8))) void policy_rollout_pop_kernel(
    const PopEntry* __restrict__ pop, int npol, int64_t N, uint32_t k0, uint32_t k1,
    const uint64_t* step_ctr) {
    const int tpp = (int)((N + 31) / 32);
    const int ntiles = npol * tpp;
    for (int g = blockIdx.x; g < ntiles; g += (int)gridDim.x) {
        const int p = __builtin_amdgcn_readfirstlane(g / tpp);
        const PopEntry& e = pop[p];
        const bool first = g == (int)blockIdx.x;
        if (first) rollout_stage<T, H, RNN, HC>(e.P, e.R);
        rollout_tile<T, H, RNN, HC, true>(e.P, e.obs, N, e.rk, k0, k1, step_ctr, e.eoff, e.R,
                                          e.cy, e.env, g - p * tpp, first);
    }
}

// A population's whole rollouts on the row-split kernel (the library's
// choice where rollout16_pop_eligible): global 16-env tile g is tile g % tpp
// of policy g / tpp (tpp = N / 16, a multiple of 8), dealt in rounds of 8
// consecutive tiles per workgroup, so all 8 waves of a workgroup hold tiles of
// one policy in every round; a workgroup restages that policy's W1 / head /
// LayerNorm images when its round's policy is not the one staged (the
// barriers are workgroup-uniform).  Per tile the body and arguments of the
// policy's own rollout16_kernel launch: the same bits.
__global__ __launch_bounds__(64 * kR16Waves) __attribute__((amdgpu_waves_per_eu(2, 2))) void rollout16_pop_kernel(
    const PopEntry* __restrict__ pop, int npol, int64_t N, uint32_t k0, uint32_t k1,
    const uint64_t* step_ctr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* tab = (int*)(smem + kR16OffTab);
    const uint64_t step0 = step_ctr ? *step_ctr : 0ull;
    const int tpp = (int)(N / 16), ntile = npol * tpp;
    const int TW = (int)gridDim.x * kR16Waves;
    int cur = -1;
#pragma clang loop unroll(disable)
    for (int t0 = (int)blockIdx.x * kR16Waves; t0 < ntile; t0 += TW) {
        const int p = __builtin_amdgcn_readfirstlane(t0 / tpp);
        const PopEntry& e = pop[p];
        if (p != cur) {
            if (cur >= 0) __syncthreads();  // every wave is past its reads of the old images
            r16_stage(e.P, smem, tid);
            if (tid <= MLEARN_MAX_GROUPS) tab[tid] = e.P.off[tid];
            __syncthreads();
            cur = p;
        }
        if (wave >= kR16Waves / 2 && t0 + TW >= ntile) __builtin_amdgcn_s_setprio(1);  // (rollout16_kernel)
        r16_roll_tile(e.P, e.obs, e.rk, k0, k1, step0, e.eoff, e.env, t0 + wave - p * tpp, tid,
                      smem);
    }
}

static int launch_rollout16_pop(const PopEntry* pop, int npol, int64_t N, uint32_t k0, uint32_t k1,
                                const uint64_t* step_ctr, hipStream_t s) {
    // (once per device, kept out of graph capture)
    if (set_lds_attr((const void*)rollout16_pop_kernel, (int)kR16Lds, "rollout16_pop"))
        return MLEARN_EHIP;
    const int cus = device_cus();
    const int64_t rounds_of_8 = (int64_t)npol * (N / 16) / kR16Waves;
    int64_t grid = cus > 0 ? cus : 256;
    if (grid > rounds_of_8) grid = rounds_of_8;
    hipLaunchKernelGGL(rollout16_pop_kernel, dim3((unsigned)grid), dim3(64 * kR16Waves), kR16Lds, s,
                       pop, npol, N, k0, k1, step_ctr);
    return check_launch("policy_rollout_env_pop (row split)");
}

template <typename T, int H, bool RNN, int HC, int MAXW = ML_POL_MAXW>
static size_t policy_step_lds(int L) {
    typedef PolCfg<H, MAXW> C;
    const size_t frags = (size_t)(H / RT<T>::KS) * 64 * sizeof(typename RT<T>::frag);
    return frags * (RNN ? 2 : 1) +
           (size_t)(L * 2 * H + HC + C::W * 64 + (head_parts<HC, C::W>() + 1) * 32 * (HC + 1) +
                    (RNN ? 4 * H : 0) + HC) * 4;
}

template <typename T, int H, bool RNN, int HC>
static int launch_policy_step(const PolicyK& P, const float* obs, int64_t N, void* obs_store,
                              int32_t* actions, float* logp, float* values, uint32_t k0, uint32_t k1,
                              const uint64_t* step_ctr, uint64_t step, uint32_t eoff, int sample,
                              const PostK& post, const LstmK& R, const CarryK& cy, const EvalK& ev,
                              const EnvK& env, hipStream_t s) {
    const size_t lds = policy_step_lds<T, H, RNN, HC, pol_maxw<RNN>()>(P.L);
    auto kern = policy_step_kernel<T, H, RNN, HC>;
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  128 * 1024);
        attr_set = true;
    }
    const int grid = (int)((N + 31) / 32);
#ifdef ML_STAMPS
    EvalK evs = ev;
    evs.stamps = g_pol_stamp_buf;
#else
    const EvalK& evs = ev;
#endif
    hipLaunchKernelGGL(kern, dim3(grid), dim3(pol_threads<H, RNN>()), lds, s, P, obs, N,
                       (T*)obs_store, actions, logp, values, k0, k1, step_ctr, step, eoff, sample,
                       post, R, cy, evs, env);
    return check_launch("policy_rollout_step");
}

// Workgroups of the whole-rollout launch (-1: per-step launches): one per
// resident slot, or at most max_wg (> 0); max_wg < 0 asks for the per-step
// launches.
template <typename T, int H, bool RNN, int HC>
static int64_t rollout_grid(int L, int64_t N, int max_wg) {
    constexpr int NT = pol_threads<H, RNN>();
    const size_t lds = policy_step_lds<T, H, RNN, HC, pol_maxw<RNN>()>(L);
    auto kern = policy_rollout_kernel<T, H, RNN, HC>;
    static bool attr_set = false;
    static int per_cu = 0, cus = 0;
    if (!attr_set) {  // once per instantiation (kept out of graph capture)
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  128 * 1024);
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NT, lds) !=
                hipSuccess)
            per_cu = cus = 0;
        attr_set = true;
    }
    const int64_t tiles = (N + 31) / 32;
    int64_t slots = (int64_t)per_cu * cus;
    if (max_wg < 0 || slots <= 0) return -1;
    if (max_wg > 0 && max_wg < slots) slots = max_wg;
    // one workgroup per resident slot, tiles dealt round-robin (tile =
    // blockIdx + k * grid): at the headline's 2 048 tiles on 768 slots every
    // CU holds workgroups b, b + 256, b + 512 with 3 + 3 + 2 = 8 tiles, the
    // chip's mean.  The earlier grid of ceil(tiles / 3) = 683 workgroups left
    // CUs with 9 or 6 tiles: 1.66 -> 1.45 ms per rollout, 10.01 -> 9.80 ms
    // per update (profiles/r04_rollout_grid_ab.txt).  The W = 8 share (256
    // tiles) keeps one tile per workgroup.
    return tiles < slots ? tiles : slots;
}

// The whole rollout as one launch (every env tile gets a resident workgroup,
// or tiles run in series inside the workgroups), or T + 1 per-step launches
// of the same body when max_wg < 0.
template <typename T, int H, bool RNN, int HC>
static int launch_policy_rollout(const PolicyK& P, const float* obs, int64_t N, const RollK& rk,
                                 uint32_t k0, uint32_t k1, const uint64_t* step_ctr, uint32_t eoff,
                                 const LstmK& R, const CarryK& cy, const EnvK& env, hipStream_t s) {
    constexpr int NT = pol_threads<H, RNN>();
    const size_t lds = policy_step_lds<T, H, RNN, HC, pol_maxw<RNN>()>(P.L);
    const int64_t grid = rollout_grid<T, H, RNN, HC>(P.L, N, rk.max_wg);
    if (grid > 0) {
        hipLaunchKernelGGL((policy_rollout_kernel<T, H, RNN, HC>), dim3((unsigned)grid), dim3(NT),
                           lds, s, P, obs, N, rk, k0, k1, step_ctr, eoff, R, cy, env);
        return check_launch("policy_rollout_env");
    }
    // max_workgroups < 0 (or no occupancy answer): the same body as
    // T + 1 launches of the per-step kernel (same bits)
    for (int t = 0; t <= rk.T; ++t) {
        const bool act = t < rk.T;
        const int64_t so = (int64_t)t * rk.ld;
        PostK post{};
        if (t > 0)
            post = PostK{env.rew, env.done, rk.rewards + so - rk.ld, rk.dones + so - rk.ld,
                         rk.env_returns, rk.trace ? rk.trace + so - rk.ld : nullptr, rk.gamma};
        CarryK c = cy;
        if (RNN) {
            const bool cs = act && t % rk.bptt == 0;
            const int64_t co = (int64_t)(t / rk.bptt) * rk.ld * H;
            c.sh = cs ? (void*)((T*)rk.start_h + co) : nullptr;
            c.sc = cs ? (void*)((T*)rk.start_c + co) : nullptr;
            c.commit = act ? 1 : 0;
        }
        const int rc = launch_policy_step<T, H, RNN, HC>(
            P, obs, N, (act && rk.obs) ? (T*)rk.obs + so * P.D : nullptr,
            act ? rk.actions + so * P.K : nullptr, act ? rk.logp + so * P.K : nullptr,
            act ? rk.values + so : rk.bootstrap, k0, k1, step_ctr, (uint64_t)t, eoff, 1, post, R, c,
            EvalK{}, act ? env : EnvK{}, s);
        if (rc) return rc;
    }
    return MLEARN_OK;
}

// Workgroups of the population launch: one per resident slot of the
// population kernel, at most one per tile.
template <typename T, int H, bool RNN, int HC>
static int64_t rollout_pop_grid(int L, int64_t tiles, int max_wg) {
    constexpr int NT = pol_threads<H, RNN>();
    const size_t lds = policy_step_lds<T, H, RNN, HC, pol_maxw<RNN>()>(L);
    auto kern = policy_rollout_pop_kernel<T, H, RNN, HC>;
    static bool attr_set = false;
    static int per_cu = 0, cus = 0;
    if (!attr_set) {  // once per instantiation (kept out of graph capture)
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  128 * 1024);
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NT, lds) !=
                hipSuccess)
            per_cu = cus = 0;
        attr_set = true;
    }
    int64_t slots = (int64_t)per_cu * cus;
    if (slots <= 0) return -1;
    // max_wg > 0 caps the grid (tiles of several policies in series per
    // workgroup, each move to another policy's tile restaging its parameters)
    if (max_wg > 0 && max_wg < slots) slots = max_wg;
    return tiles < slots ? tiles : slots;
}

template <typename T, int H, bool RNN, int HC>
static int launch_policy_rollout_pop(int L, const PopEntry* pop, int npol, int64_t N, uint32_t k0,
                                     uint32_t k1, const uint64_t* step_ctr, int max_wg,
                                     hipStream_t s) {
    constexpr int NT = pol_threads<H, RNN>();
    const size_t lds = policy_step_lds<T, H, RNN, HC, pol_maxw<RNN>()>(L);
    const int64_t grid =
        rollout_pop_grid<T, H, RNN, HC>(L, (int64_t)npol * ((N + 31) / 32), max_wg);
    ML_REQUIRE(grid > 0, "policy_rollout_env_pop: no occupancy answer for the population kernel");
    hipLaunchKernelGGL((policy_rollout_pop_kernel<T, H, RNN, HC>), dim3((unsigned)grid), dim3(NT),
                       lds, s, pop, npol, N, k0, k1, step_ctr);
    return check_launch("policy_rollout_env_pop");
}

static int rollout_step_entry(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                              const mlearn_lstm_carry* carry, const float* obs, int64_t N,
                              void* obs_store, int32_t* actions, float* log_probs, float* values,
                              uint32_t k0, uint32_t k1, const uint64_t* step_ctr, uint64_t step,
                              uint32_t env_offset, int32_t sample, const mlearn_post_step* post,
                              mlearn_stream_t stream, EvalK ev = EvalK{},
                              const mlearn_dummy_env* denv = nullptr) {
    int rc = lstm ? validate_lstm(policy, lstm) : validate_policy(policy);
    if (rc) return rc;
    ML_REQUIRE(N >= 0, "policy_rollout_step: N < 0");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(obs, "policy_rollout_step: null obs");
    ML_REQUIRE(!actions || log_probs || !sample, "policy_rollout_step: sampling needs log_probs");
    ML_REQUIRE(!ev.actions || (!actions && log_probs && ev.entropies),
               "policy_evaluate: needs log_probs and entropies outputs");
    ML_REQUIRE(actions || values || ev.actions, "policy_rollout_step: nothing to compute");
    ML_REQUIRE(!policy->obs_stats || !actions || policy->obs_stats_tiles >= (N + 31) / 32,
               "policy_rollout_step: obs_stats_tiles %lld < ceil(N / 32)",
               (long long)policy->obs_stats_tiles);
    ML_REQUIRE((uintptr_t)obs % 16 == 0, "policy_rollout_step: obs must be 16-byte aligned");
    ML_REQUIRE(!obs_store || (uintptr_t)obs_store % 16 == 0,
               "policy_rollout_step: obs_store must be 16-byte aligned");
    PostK pk{};
    if (post) {
        ML_REQUIRE(post->rewards && post->dones && post->store_rewards && post->store_dones &&
                       post->env_returns,
                   "policy_rollout_step: null post-step pointer");
        pk = PostK{post->rewards, post->dones, post->store_rewards, post->store_dones,
                   post->env_returns, post->env_returns_trace, post->gamma};
    }
    EnvK ek{};
    if (denv) {
        ML_REQUIRE(actions, "policy_rollout_step_env: the fused env step needs actions");
        ML_REQUIRE(denv->state && denv->obs && denv->rewards && denv->dones,
                   "policy_rollout_step_env: null env pointer");
        ML_REQUIRE(denv->obs == obs,
                   "policy_rollout_step_env: env->obs must be the launch's obs input (the next "
                   "observations overwrite it in place)");
        ML_REQUIRE((uintptr_t)denv->state % 16 == 0, "policy_rollout_step_env: state alignment");
        ML_REQUIRE(!post || (post->rewards == denv->rewards && post->dones == denv->dones),
                   "policy_rollout_step_env: post-step must read the env's rewards / dones");
        ek = EnvK{(int4*)denv->state, denv->obs, denv->rewards, denv->dones, denv->k0, denv->k1,
                  denv->env_offset};
    }
    LstmK R{};
    CarryK cy{};
    if (lstm) {
        ML_REQUIRE(carry && carry->h && carry->c, "lstm rollout step: null carry");
        ML_REQUIRE(!carry->start_h == !carry->start_c, "lstm rollout step: start_h / start_c");
        ML_REQUIRE((uintptr_t)carry->h % 16 == 0 && (uintptr_t)carry->c % 16 == 0,
                   "lstm rollout step: carry must be 16-byte aligned");
        R = make_lstm_k(*lstm);
        cy = CarryK{carry->h, carry->c, carry->start_h, carry->start_c, carry->commit, carry->clear};
    }
    PolicyK P = make_policy_k(*policy);
    hipStream_t s = S(stream);
#define ML_LAUNCH_HC(T, HH, HC)                                                                 \
    (lstm ? launch_policy_step<T, HH, true, HC>(P, obs, N, obs_store, actions, log_probs, values, \
                                                k0, k1, step_ctr, step, env_offset, sample, pk, R, \
                                                cy, ev, ek, s)                                    \
          : launch_policy_step<T, HH, false, HC>(P, obs, N, obs_store, actions, log_probs, values, \
                                                 k0, k1, step_ctr, step, env_offset, sample, pk, R, \
                                                 cy, ev, ek, s))
#define ML_LAUNCH(T, HH) \
    (P.HC == MLEARN_HEAD_COLS ? ML_LAUNCH_HC(T, HH, MLEARN_HEAD_COLS) : ML_LAUNCH_HC(T, HH, MLEARN_HEAD_COLS_MAX))
#define ML_DISPATCH(T)                      \
    switch (policy->hidden) {               \
        case 64: return ML_LAUNCH(T, 64);   \
        case 128: return ML_LAUNCH(T, 128); \
        default: return ML_LAUNCH(T, 256);  \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
#undef ML_LAUNCH
#undef ML_LAUNCH_HC
}

}  // namespace ml

using namespace ml;

extern "C" int mlearn_policy_rollout_step(const mlearn_mlp_policy* policy, const float* obs,
                                          int64_t N, void* obs_store, int32_t* actions,
                                          float* log_probs, float* values, uint32_t k0,
                                          uint32_t k1, const uint64_t* step_ctr, uint64_t step,
                                          uint32_t env_offset, int32_t sample,
                                          const mlearn_post_step* post, mlearn_stream_t stream) {
    return rollout_step_entry(policy, nullptr, nullptr, obs, N, obs_store, actions, log_probs,
                              values, k0, k1, step_ctr, step, env_offset, sample, post, stream);
}

// Validated launch arguments of one policy's whole rollout
// (mlearn_policy_rollout_env / one entry of a population).
static int rollout_env_args(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                            const mlearn_lstm_carry* carry, const float* obs, int64_t N,
                            const mlearn_rollout_out* out, uint32_t env_offset,
                            const mlearn_dummy_env* denv, PopEntry* e) {
    int rc = lstm ? validate_lstm(policy, lstm) : validate_policy(policy);
    if (rc) return rc;
    ML_REQUIRE(N >= 0, "policy_rollout_env: N < 0");
    ML_REQUIRE(obs && out && denv, "policy_rollout_env: null obs / out / env");
    ML_REQUIRE(out->T >= 1 && out->bptt_len >= 1 && out->T % out->bptt_len == 0 && out->ld >= N,
               "policy_rollout_env: bad T / bptt / ld");
    ML_REQUIRE(out->actions && out->log_probs && out->values && out->rewards && out->dones &&
                   out->bootstrap && out->env_returns,
               "policy_rollout_env: null store pointer");
    ML_REQUIRE(denv->state && denv->obs == obs && denv->rewards && denv->dones,
               "policy_rollout_env: env->obs must be the obs input; null env pointer");
    ML_REQUIRE((uintptr_t)obs % 16 == 0 && (uintptr_t)denv->state % 16 == 0 &&
                   (!out->obs || (uintptr_t)out->obs % 16 == 0),
               "policy_rollout_env: obs / state / store alignment");
    ML_REQUIRE(!policy->obs_stats || policy->obs_stats_tiles >= (N + 31) / 32,
               "policy_rollout_env: obs_stats_tiles %lld < ceil(N / 32)",
               (long long)policy->obs_stats_tiles);
    *e = PopEntry{};
    if (lstm) {
        ML_REQUIRE(carry && carry->h && carry->c && out->start_h && out->start_c,
                   "lstm rollout: null carry / start states");
        e->R = make_lstm_k(*lstm);
        e->cy = CarryK{carry->h, carry->c, nullptr, nullptr, 1, nullptr};
    }
    e->rk = RollK{out->obs, out->actions, out->log_probs, out->values, out->rewards, out->dones,
                  out->env_returns_trace, out->bootstrap, out->env_returns, out->start_h,
                  out->start_c, out->T, out->bptt_len, out->ld, out->gamma, out->max_workgroups,
                  nullptr, out->gae_gamma, out->gae_gamma_lambda};
    e->env = EnvK{(int4*)denv->state, denv->obs, denv->rewards, denv->dones, denv->k0, denv->k1,
                  denv->env_offset};
    e->P = make_policy_k(*policy);
    e->obs = obs;
    e->eoff = env_offset;
    return MLEARN_OK;
}

static int feature_split_rollout(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                 const PolicyK& P, const LstmK& R, const CarryK& cy,
                                 const float* obs, int64_t N, const RollK& rk, uint32_t k0,
                                 uint32_t k1, const uint64_t* step_ctr, uint32_t env_offset,
                                 const EnvK& ek, hipStream_t s);

extern "C" int mlearn_policy_rollout_env(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                         const mlearn_lstm_carry* carry, const float* obs,
                                         int64_t N, const mlearn_rollout_out* out, uint32_t k0,
                                         uint32_t k1, const uint64_t* step_ctr,
                                         uint32_t env_offset, const mlearn_dummy_env* denv,
                                         mlearn_stream_t stream) {
    PopEntry e;
    const int rc = rollout_env_args(policy, lstm, carry, obs, N, out, env_offset, denv, &e);
    if (rc) return rc;
    if (N == 0) return MLEARN_OK;
    const PolicyK& P = e.P;
    const LstmK& R = e.R;
    const CarryK& cy = e.cy;
    const RollK& rk = e.rk;
    const EnvK& ek = e.env;
    hipStream_t s = S(stream);
    ML_REQUIRE(out->policy_kernel >= 0 && out->policy_kernel <= 2,
               "policy_rollout_env: policy_kernel %d", out->policy_kernel);
    const bool r16 = rollout16_eligible(P, N, out->max_workgroups,
                                        policy->dtype == MLEARN_DTYPE_BF16, lstm != nullptr);
    ML_REQUIRE(out->policy_kernel != 2 || r16,
               "policy_rollout_env: policy_kernel 2 (row split) needs the row-split step's policy "
               "shape, <= 8 action groups, no observation normaliser, max_workgroups 0 and N of "
               "32768 or a multiple of 256 from 65536");
    ML_REQUIRE(!out->advantages || out->ld == N,
               "policy_rollout_env: advantages need ld == N (ld %lld, N %lld)",
               (long long)out->ld, (long long)N);
    if (r16 && out->policy_kernel != 1) {
        RollK rk2 = rk;
        if (out->advantages && out->T <= 32) rk2.adv = out->advantages;  // fused GAE
        const int rc2 = launch_rollout16(P, obs, N, rk2, k0, k1, step_ctr, env_offset, ek, s);
        if (rc2 || !out->advantages || rk2.adv) return rc2;
        return mlearn_gae_f32(out->rewards, out->values, out->dones, out->bootstrap,
                              out->advantages, nullptr, out->T, N, out->gae_gamma,
                              out->gae_gamma_lambda, stream);
    }
    if (out->advantages) {  // the feature-split rollout, then GAE as its own launch
        const int rc2 = feature_split_rollout(policy, lstm, P, R, cy, obs, N, rk, k0, k1, step_ctr,
                                              env_offset, ek, s);
        if (rc2) return rc2;
        return mlearn_gae_f32(out->rewards, out->values, out->dones, out->bootstrap,
                              out->advantages, nullptr, out->T, N, out->gae_gamma,
                              out->gae_gamma_lambda, stream);
    }
    return feature_split_rollout(policy, lstm, P, R, cy, obs, N, rk, k0, k1, step_ctr, env_offset,
                                 ek, s);
}

// The feature-split whole-rollout launch (policy_rollout_kernel) for the
// policy's dtype / width / head.
static int feature_split_rollout(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                 const PolicyK& P, const LstmK& R, const CarryK& cy,
                                 const float* obs, int64_t N, const RollK& rk, uint32_t k0,
                                 uint32_t k1, const uint64_t* step_ctr, uint32_t env_offset,
                                 const EnvK& ek, hipStream_t s) {
#define ML_LAUNCH_HC(T, HH, HC)                                                                 \
    (lstm ? launch_policy_rollout<T, HH, true, HC>(P, obs, N, rk, k0, k1, step_ctr, env_offset, R, \
                                                   cy, ek, s)                                     \
          : launch_policy_rollout<T, HH, false, HC>(P, obs, N, rk, k0, k1, step_ctr, env_offset, R, \
                                                    cy, ek, s))
#define ML_LAUNCH(T, HH) \
    (P.HC == MLEARN_HEAD_COLS ? ML_LAUNCH_HC(T, HH, MLEARN_HEAD_COLS) : ML_LAUNCH_HC(T, HH, MLEARN_HEAD_COLS_MAX))
#define ML_DISPATCH(T)                      \
    switch (policy->hidden) {               \
        case 64: return ML_LAUNCH(T, 64);   \
        case 128: return ML_LAUNCH(T, 128); \
        default: return ML_LAUNCH(T, 256);  \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
#undef ML_LAUNCH
#undef ML_LAUNCH_HC
}


extern "C" int64_t mlearn_policy_pop_bytes(int32_t num_policies) {
    return num_policies > 0 ? (int64_t)num_policies * (int64_t)sizeof(PopEntry) : 0;
}

extern "C" int mlearn_policy_pop_prepare(const mlearn_mlp_policy* policies,
                                         const mlearn_lstm* lstms,
                                         const mlearn_lstm_carry* carries,
                                         const float* const* obs, int64_t N,
                                         const mlearn_rollout_out* outs,
                                         const uint32_t* env_offsets,
                                         const mlearn_dummy_env* envs, int32_t num_policies,
                                         void* pop, mlearn_stream_t stream) {
    ML_REQUIRE(num_policies >= 1 && policies && obs && outs && env_offsets && envs && pop,
               "policy_pop_prepare: null argument or no policies");
    for (int p = 0; p < num_policies; ++p)
        ML_REQUIRE(!outs[p].advantages,
                   "policy_pop_prepare: advantages (fused GAE) is a single-policy rollout option");
    ML_REQUIRE(N >= 1, "policy_pop_prepare: N < 1");
    std::vector<PopEntry> h((size_t)num_policies);
    for (int p = 0; p < num_policies; ++p) {
        const mlearn_mlp_policy& a = policies[p];
        const mlearn_mlp_policy& b = policies[0];
        ML_REQUIRE(a.dtype == b.dtype && a.hidden == b.hidden && a.num_layers == b.num_layers &&
                       a.obs_dim == b.obs_dim && head_cols(a) == head_cols(b),
                   "policy_pop_prepare: policy %d's shape differs from policy 0's", p);
        ML_REQUIRE(!lstms == !carries, "policy_pop_prepare: lstms and carries go together");
        const int rc = rollout_env_args(&a, lstms ? &lstms[p] : nullptr,
                                        carries ? &carries[p] : nullptr, obs[p], N, &outs[p],
                                        env_offsets[p], &envs[p], &h[(size_t)p]);
        if (rc) return rc;
        ML_REQUIRE(outs[p].max_workgroups == 0,
                   "policy_pop_prepare: the population launch has its own grid (max_workgroups 0)");
        ML_REQUIRE(!a.obs_mu == !b.obs_mu && !a.obs_stats == !b.obs_stats,
                   "policy_pop_prepare: policy %d's observation normaliser differs from policy 0's",
                   p);
    }
    // ordered after the caller's earlier work on its stream (a previous
    // population launch may still read the buffer), and complete on return
    // (the host staging vector dies with this call)
    hipError_t err = hipMemcpyAsync(pop, h.data(), h.size() * sizeof(PopEntry),
                                    hipMemcpyHostToDevice, S(stream));
    if (err == hipSuccess) err = hipStreamSynchronize(S(stream));
    if (err != hipSuccess) {
        set_error("policy_pop_prepare: hipMemcpy: %s", hipGetErrorString(err));
        return MLEARN_EHIP;
    }
    return MLEARN_OK;
}

extern "C" int mlearn_policy_rollout_env_pop(const mlearn_mlp_policy* policy0,
                                             const mlearn_lstm* lstm0, const void* pop,
                                             int32_t num_policies, int64_t N, uint32_t k0,
                                             uint32_t k1, const uint64_t* step_ctr,
                                             int32_t max_workgroups, mlearn_stream_t stream) {
    int rc = lstm0 ? validate_lstm(policy0, lstm0) : validate_policy(policy0);
    if (rc) return rc;
    ML_REQUIRE(pop && num_policies >= 1 && N >= 1 && step_ctr,
               "policy_rollout_env_pop: null pop / step counter, or no work");
    ML_REQUIRE(max_workgroups >= 0, "policy_rollout_env_pop: max_workgroups < 0");
    const int L = policy0->num_layers, HC = head_cols(*policy0);
    const PopEntry* e = (const PopEntry*)pop;
    hipStream_t s = S(stream);
    if (rollout16_pop_eligible(make_policy_k(*policy0), N, num_policies, max_workgroups,
                               policy0->dtype == MLEARN_DTYPE_BF16, lstm0 != nullptr))
        return launch_rollout16_pop(e, num_policies, N, k0, k1, step_ctr, s);
#define ML_POP_HC(T, HH, HCC)                                                                   \
    (lstm0 ? launch_policy_rollout_pop<T, HH, true, HCC>(L, e, num_policies, N, k0, k1, step_ctr, \
                                                       max_workgroups, s)                     \
           : launch_policy_rollout_pop<T, HH, false, HCC>(L, e, num_policies, N, k0, k1, step_ctr, \
                                                        max_workgroups, s))
#define ML_POP(T, HH) \
    (HC == MLEARN_HEAD_COLS ? ML_POP_HC(T, HH, MLEARN_HEAD_COLS) : ML_POP_HC(T, HH, MLEARN_HEAD_COLS_MAX))
#define ML_DISPATCH(T)                   \
    switch (policy0->hidden) {           \
        case 64: return ML_POP(T, 64);   \
        case 128: return ML_POP(T, 128); \
        default: return ML_POP(T, 256);  \
    }
    if (policy0->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
#undef ML_POP
#undef ML_POP_HC
}

extern "C" int32_t mlearn_policy_rollout_pop_kernel(const mlearn_mlp_policy* policy,
                                                    const mlearn_lstm* lstm, int64_t N,
                                                    int32_t num_policies,
                                                    int32_t max_workgroups) {
    if ((lstm ? validate_lstm(policy, lstm) : validate_policy(policy)) || N < 1 ||
        num_policies < 1 || max_workgroups < 0)
        return -1;
    return rollout16_pop_eligible(make_policy_k(*policy), N, num_policies, max_workgroups,
                                  policy->dtype == MLEARN_DTYPE_BF16, lstm != nullptr)
               ? 2
               : 1;
}

extern "C" int64_t mlearn_policy_rollout_pop_workgroups(const mlearn_mlp_policy* policy,
                                                        const mlearn_lstm* lstm, int64_t N,
                                                        int32_t num_policies,
                                                        int32_t max_workgroups) {
    if ((lstm ? validate_lstm(policy, lstm) : validate_policy(policy)) || N < 1 ||
        num_policies < 1 || max_workgroups < 0)
        return -1;
    const int HC = head_cols(*policy), L = policy->num_layers;
    const int64_t tiles = (int64_t)num_policies * ((N + 31) / 32);
#define ML_GRID_HC(T, HH, HCC) \
    (lstm ? rollout_pop_grid<T, HH, true, HCC>(L, tiles, max_workgroups) \
          : rollout_pop_grid<T, HH, false, HCC>(L, tiles, max_workgroups))
#define ML_GRID(T, HH) \
    (HC == MLEARN_HEAD_COLS ? ML_GRID_HC(T, HH, MLEARN_HEAD_COLS) : ML_GRID_HC(T, HH, MLEARN_HEAD_COLS_MAX))
#define ML_DISPATCH(T)                    \
    switch (policy->hidden) {             \
        case 64: return ML_GRID(T, 64);   \
        case 128: return ML_GRID(T, 128); \
        default: return ML_GRID(T, 256);  \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
#undef ML_GRID
#undef ML_GRID_HC
}

extern "C" int64_t mlearn_policy_rollout_workgroups(const mlearn_mlp_policy* policy,
                                                    const mlearn_lstm* lstm, int64_t N,
                                                    int32_t max_workgroups) {
    if ((lstm ? validate_lstm(policy, lstm) : validate_policy(policy)) || N < 1) return -1;
    const int HC = head_cols(*policy), L = policy->num_layers;
#define ML_GRID_HC(T, HH, HCC) \
    (lstm ? rollout_grid<T, HH, true, HCC>(L, N, max_workgroups) \
          : rollout_grid<T, HH, false, HCC>(L, N, max_workgroups))
#define ML_GRID(T, HH) \
    (HC == MLEARN_HEAD_COLS ? ML_GRID_HC(T, HH, MLEARN_HEAD_COLS) : ML_GRID_HC(T, HH, MLEARN_HEAD_COLS_MAX))
#define ML_DISPATCH(T)                    \
    switch (policy->hidden) {             \
        case 64: return ML_GRID(T, 64);   \
        case 128: return ML_GRID(T, 128); \
        default: return ML_GRID(T, 256);  \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
#undef ML_GRID
#undef ML_GRID_HC
}

extern "C" int32_t mlearn_policy_rollout_kernel(const mlearn_mlp_policy* policy,
                                                const mlearn_lstm* lstm, int64_t N,
                                                int32_t max_workgroups, int32_t requested) {
    if ((lstm ? validate_lstm(policy, lstm) : validate_policy(policy)) || N < 1 || requested < 0 ||
        requested > 2)
        return -1;
    const bool r16 = rollout16_eligible(make_policy_k(*policy), N, max_workgroups,
                                        policy->dtype == MLEARN_DTYPE_BF16, lstm != nullptr);
    if (requested == 2 && !r16) return -1;
    return r16 && requested != 1 ? 2 : 1;
}

extern "C" int mlearn_policy_rollout_step_env(const mlearn_mlp_policy* policy, const float* obs,
                                              int64_t N, void* obs_store, int32_t* actions,
                                              float* log_probs, float* values, uint32_t k0,
                                              uint32_t k1, const uint64_t* step_ctr, uint64_t step,
                                              uint32_t env_offset, int32_t sample,
                                              const mlearn_post_step* post,
                                              const mlearn_dummy_env* env, mlearn_stream_t stream) {
    ML_REQUIRE(env, "policy_rollout_step_env: null env descriptor");
    return rollout_step_entry(policy, nullptr, nullptr, obs, N, obs_store, actions, log_probs,
                              values, k0, k1, step_ctr, step, env_offset, sample, post, stream,
                              EvalK{}, env);
}

extern "C" int mlearn_lstm_policy_rollout_step_env(
    const mlearn_mlp_policy* policy, const mlearn_lstm* lstm, const mlearn_lstm_carry* carry,
    const float* obs, int64_t N, void* obs_store, int32_t* actions, float* log_probs,
    float* values, uint32_t k0, uint32_t k1, const uint64_t* step_ctr, uint64_t step,
    uint32_t env_offset, int32_t sample, const mlearn_post_step* post, const mlearn_dummy_env* env,
    mlearn_stream_t stream) {
    ML_REQUIRE(lstm, "lstm rollout step: null lstm descriptor");
    ML_REQUIRE(env, "policy_rollout_step_env: null env descriptor");
    return rollout_step_entry(policy, lstm, carry, obs, N, obs_store, actions, log_probs, values,
                              k0, k1, step_ctr, step, env_offset, sample, post, stream, EvalK{},
                              env);
}

extern "C" int mlearn_lstm_policy_rollout_step(
    const mlearn_mlp_policy* policy, const mlearn_lstm* lstm, const mlearn_lstm_carry* carry,
    const float* obs, int64_t N, void* obs_store, int32_t* actions, float* log_probs,
    float* values, uint32_t k0, uint32_t k1, const uint64_t* step_ctr, uint64_t step,
    uint32_t env_offset, int32_t sample, const mlearn_post_step* post, mlearn_stream_t stream) {
    ML_REQUIRE(lstm, "lstm rollout step: null lstm descriptor");
    return rollout_step_entry(policy, lstm, carry, obs, N, obs_store, actions, log_probs, values,
                              k0, k1, step_ctr, step, env_offset, sample, post, stream);
}

extern "C" int mlearn_policy_evaluate(const mlearn_mlp_policy* policy, const float* obs,
                                      int64_t N, const int32_t* actions, float* log_probs,
                                      float* entropies, float* values, mlearn_stream_t stream) {
    ML_REQUIRE(actions, "policy_evaluate: null actions");
    return rollout_step_entry(policy, nullptr, nullptr, obs, N, nullptr, nullptr, log_probs, values,
                              0, 0, nullptr, 0, 0, 0, nullptr, stream, EvalK{actions, entropies});
}

extern "C" int mlearn_lstm_policy_evaluate(const mlearn_mlp_policy* policy,
                                           const mlearn_lstm* lstm,
                                           const mlearn_lstm_carry* carry, const float* obs,
                                           int64_t N, const int32_t* actions, float* log_probs,
                                           float* entropies, float* values,
                                           mlearn_stream_t stream) {
    ML_REQUIRE(lstm, "lstm policy_evaluate: null lstm descriptor");
    ML_REQUIRE(actions, "lstm policy_evaluate: null actions");
    return rollout_step_entry(policy, lstm, carry, obs, N, nullptr, nullptr, log_probs, values, 0,
                              0, nullptr, 0, 0, 0, nullptr, stream, EvalK{actions, entropies});
}

extern "C" int32_t mlearn_head_cols(const mlearn_mlp_policy* policy) {
    if (validate_policy(policy)) return -1;
    return head_cols(*policy);
}

#ifdef ML_STAMPS
// diagnostic builds only: phase timestamps of the rollout policy kernel
extern "C" void mlearn_debug_set_policy_stamp_buffer(uint64_t* buf) { ml::g_pol_stamp_buf = buf; }
#endif
