// Shared definitions of the PPO minibatch kernels (ppo.hip and the row-split
// step, ppo_rows16.h): rollout / hyperparameter / workspace descriptors, the
// split-K plan, workspace carving, and the PPO loss terms of one (row, action
// group | value) task (ppo.py:129-262).
#pragma once
#include <type_traits>

#include "common.h"
#include "dists.h"
#include "rowtile.h"

namespace ml {

struct RolloutK {
    const void* obs;
    const int32_t* actions;
    const float* logp;
    const float* adv;
    const float* ret;
    const float* values;
    const uint8_t* dones;
    int T, bptt;
    int64_t N, ld;  // envs of this policy, row stride of the store
};

struct HpK {
    float clip, vcoef;
    float ecoef[MLEARN_MAX_GROUPS];
    float objw[MLEARN_MAX_GROUPS];  // per sub-action surrogate weight (K / K_key)
    int norm_adv, clip_vl, huber, norm_vals;
    int metrics;  // reduce the loss metrics (only the minibatch whose metrics are recorded)
    int wg_form;  // mlearn_ppo_hparams.wgrad_form (bf16 weight-gradient staging)
    float loss_scale;
    float inv_sk, inv_s;
};

constexpr int kLossSlots = 20;   // per tile doubles
#ifndef ML_STEP_WAVES
#define ML_STEP_WAVES 4  // waves per SIMD the fused step kernel is register-budgeted for
#endif
constexpr int kColChunks = 32;   // first-level chunks of the per-tile column partials
constexpr int kWgTile = 128;     // weight-gradient output tile (rows and cols)
#ifndef ML_WG_CHUNK
#define ML_WG_CHUNK 32  // weight-gradient K chunk of the bf16 kernel (rows of the minibatch)
#endif
// weight-gradient K chunk (rows of the minibatch staged per LDS stage); f32 keeps 32
template <typename T> constexpr int wg_chunk() { return sizeof(T) == 2 ? ML_WG_CHUNK : 32; }
static inline int wg_chunk_es(size_t es) { return es == 2 ? ML_WG_CHUNK : 32; }
constexpr int kRowAlign = 64;  // Mp granularity of the update (an even number of 32-row tiles)

#ifndef ML_WG_SETS
#define ML_WG_SETS 2  // weight-gradient chunks in flight (register sets of staged rows)
#endif
#ifndef ML_WG_GLDS
#define ML_WG_GLDS 1  // bf16 weight-gradient tiles staged by LDS-DMA (global_load_lds) pipelines
#endif
#ifndef ML_WG_STAGES
#define ML_WG_STAGES 2  // LDS stages of the LDS-DMA pipeline (S - 1 chunks in flight)
#endif
#ifndef ML_WG_SLAB_NT
#define ML_WG_SLAB_NT 1  // LDS-DMA tile: split-K slabs stored nontemporal
#endif
#ifndef ML_WG_WAVES
#define ML_WG_WAVES 3  // waves per SIMD the weight-gradient kernel is register-budgeted for
#endif
constexpr int kMaxJobs = MLEARN_MAX_LAYERS + 3;  // weight-gradient jobs

// LSTM scan buffers of the recurrent update (rows f = t * mb + m, compute
// dtype unless noted).
struct LstmWsK {
    void* hout;   // [Mp][H]  cell outputs h_t (head input)
    void* hin;    // [Mp][H]  carry into step t (cleared after done steps)
    void* cin;    // [Mp][H]
    void* cout;   // [Mp][H]  c_t
    void* gates;  // [Mp][4H] i, f, g, o activations (gate-major columns)
    void* dg;     // [Mp][4H] d loss / d gate pre-activations
    void* dhout;  // [Mp][H]  d loss / d h_t from the heads
    void* dfeat;  // [Mp][H]  d loss / d trunk output
    float* dcc;   // [Mp][H] f32  c cotangent into step t (per-step reverse scan)
};

struct WsK {
    void* x0;                           // [Mp][D]  gathered obs (compute dtype)
    void* a[MLEARN_MAX_LAYERS];         // [Mp][H]  post-ReLU activations
    void* dhead;                        // [Mp][32] d loss / d head outputs
    void* dz[MLEARN_MAX_LAYERS];        // [Mp][H]  d loss / d Dense outputs
    float* colpart;                     // [tiles][CP] per-tile column partials
    float* colpart2;                    // [kColChunks][CP]
    double* loss_part;                  // [2 tiles][kLossSlots]
    float* slab;                        // split-K partial weight gradients
    int64_t slab_off[kMaxJobs];         // jobs: W_0..W_{L-1}, head, (LSTM) Wi, Wh
    int splits[kMaxJobs];
    int64_t rps[kMaxJobs];  // rows per split
    int64_t Mp;
    int ntiles;                         // Mp / 32
    int ncp;                            // colpart rows written: ntiles, 2 ntiles (row-split step)
    int nlp;                            // loss_part rows written: ntiles, 2 ntiles (row-split
                                        // step with one 16-row tile per wave)
    int CP;                             // L*2*H + 32
    uint64_t* stamps;                   // diagnostic builds only (ML_STAMPS): [tiles][16]
};

#ifdef ML_STAMPS
static uint64_t* g_stamp_buf = nullptr;
#define STAMP(i)                                                                  \
    do {                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                        \
        if (ws.stamps && lane == 0)                                               \
            ws.stamps[((int64_t)tile * W + w) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
        __builtin_amdgcn_sched_barrier(0);                                        \
    } while (0)
#else
#define STAMP(i) \
    do {         \
    } while (0)
#endif

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Split-K plan of one weight gradient [I][J] over Mp rows: ~ML_WG_TARGET
// workgroups per weight.
#ifndef ML_WG_TARGET
#define ML_WG_TARGET 128
#endif
#ifndef ML_WG_CPW
#define ML_WG_CPW 32  // > 0: split every weight into splits of this many chunks (balanced per-WG work)
#endif
#ifndef ML_WG_SMALL_CHUNKS
#define ML_WG_SMALL_CHUNKS 512  // slices of at most this many chunks take at most ML_WG_SMALL_SPLITS splits
#endif
#ifndef ML_WG_SMALL_SPLITS
#define ML_WG_SMALL_SPLITS 32
#endif
#ifndef ML_WG_TARGET_LSTM
#define ML_WG_TARGET_LSTM 512  // the LSTM gate weights' (Wi, Wh) workgroup target (config L: 10.94 / 10.60 / 10.47 ms at 128 / 256 / 512); round 5: 10.27 / 10.33 / 10.51 ms at 512 / 768 / 1024
#endif
static void plan_splits(int I, int J, int64_t Mp, int kWgChunk, int* splits, int64_t* rps,
                        int target = ML_WG_TARGET) {
    int tiles = ((I + kWgTile - 1) / kWgTile) * ((J + kWgTile - 1) / kWgTile);
    int64_t chunks = Mp / kWgChunk;
    int64_t s = target / tiles;
    // balanced: splits of at most ML_WG_CPW chunks (never fewer workgroups than
    // the target: small per-rank minibatches under data parallelism keep their
    // parallelism), at most 2 x the target per weight (the MLP trunk / head
    // weights of <= 4 tiles; the LSTM's wide gate weights keep the target)
    if (ML_WG_CPW > 0 && tiles <= 4) {
        int64_t b = (chunks + ML_WG_CPW - 1) / ML_WG_CPW;
        if (b > 8) b = (b + 7) / 8 * 8;  // multiples of 8 keep the XCD-aware tile mapping
        if (b > s) s = b < 2 * s ? b : 2 * s;
    }
    // small minibatch slices (the data-parallel ranks' 8 192 / 16 384 rows
    // = 256 / 512 chunks at W = 8 / 4): at most ML_WG_SMALL_SPLITS splits
    // per weight instead of 64 for W0 and the head, so the f32 slabs
    // (splits x I x J, written here and read by reduce_grads) do not
    // outweigh the operands (emulated rank shares 3.70 -> 3.66 ms at W = 8,
    // 4.35 -> 4.23 ms at W = 4; profiles/r04_wgrad_small_slices_ab.txt)
    if (chunks <= ML_WG_SMALL_CHUNKS && s > ML_WG_SMALL_SPLITS) s = ML_WG_SMALL_SPLITS;
    if (s < 1) s = 1;
    if (s > chunks) s = chunks;
    int64_t per = (chunks + s - 1) / s;
    *rps = per * kWgChunk;
    *splits = (int)((Mp + *rps - 1) / *rps);
}

// Carve the workspace; returns total bytes (base may be null to size only).
// lstm (may be null): recurrent policy; mb = sequences per minibatch.
static size_t carve(const mlearn_mlp_policy& p, int64_t M, char* base, WsK* W,
                    const mlearn_lstm* lstm = nullptr, int64_t mb = 0, LstmWsK* LW = nullptr) {
    const size_t es = p.dtype == MLEARN_DTYPE_BF16 ? 2 : 4;
    const int H = p.hidden, D = p.obs_dim, L = p.num_layers;
    const int64_t Mp = (M + kRowAlign - 1) / kRowAlign * kRowAlign;
    const int64_t tiles = Mp / 32;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* ptr = base ? base + off : nullptr;
        off = align256(off + bytes);
        return (void*)ptr;
    };
    WsK w{};
    w.Mp = Mp;
    w.ntiles = (int)tiles;
    w.ncp = (int)tiles;
    w.nlp = (int)tiles;
    // column partials: LayerNorm [L][2][H], head bias [32], (LSTM) bias [4H]
    const int HC = head_cols(p);
    w.CP = L * 2 * H + HC + (lstm ? 4 * H : 0);
    w.x0 = take(Mp * D * es);
    for (int l = 0; l < L; ++l) {
        w.a[l] = take(Mp * H * es);
        w.dz[l] = take(Mp * H * es);
    }
    w.dhead = take(Mp * HC * es);
    w.colpart = (float*)take(2 * tiles * w.CP * sizeof(float));  // (16-row tiles: row-split)
    w.colpart2 = (float*)take(kColChunks * w.CP * sizeof(float));
    w.loss_part = (double*)take(2 * tiles * kLossSlots * sizeof(double));  // (16-row tiles: row-split)
    int64_t so = 0;
    const int njobs = L + 1 + (lstm ? 2 : 0);
    for (int l = 0; l < njobs; ++l) {
        const int I = l >= L ? H : (l == 0 ? D : H);
        const int J = l == L ? HC : (l > L ? 4 * H : H);
        plan_splits(I, J, Mp, wg_chunk_es(es), &w.splits[l], &w.rps[l],
                    l > L ? ML_WG_TARGET_LSTM : ML_WG_TARGET);
        w.slab_off[l] = so;
        so += (int64_t)w.splits[l] * I * J;
    }
    w.slab = (float*)take(so * sizeof(float));
    if (lstm) {
        LstmWsK lw{};
        lw.hout = take(Mp * H * es);
        lw.hin = take(Mp * H * es);
        lw.cin = take(Mp * H * es);
        lw.cout = take(Mp * H * es);
        lw.gates = take(Mp * 4 * H * es);
        lw.dg = take(Mp * 4 * H * es);
        lw.dhout = take(Mp * H * es);
        lw.dfeat = take(Mp * H * es);
        lw.dcc = (float*)take(Mp * H * sizeof(float));
        if (LW) *LW = lw;
    }
    if (W) *W = w;
    return off;
}

// ---------------------------------------------------------------------------
// PPO loss terms of one (row, action group) / (row, value) task
// (ppo.py:129-262), writing d loss / d logits (or d value) in place of the
// logits.
// ---------------------------------------------------------------------------
struct LossAcc {
    float sobj = 0, qobj = 0, sent = 0, qent = 0, svl = 0, qvl = 0, serr = 0, qerr = 0, sentw = 0;
    float sobjw = 0;  // surrogate sum weighted per action group (reduce_action_objs)
    float mnobj = 3.4e38f, mxobj = -3.4e38f, mnent = 3.4e38f, mxent = -3.4e38f;
    float mnvl = 3.4e38f, mxvl = -3.4e38f, mnerr = 3.4e38f, mxerr = -3.4e38f;
};

// PPO objective terms of one action group given its log-prob of the taken
// action and entropy; returns d loss / d logp[a] and accumulates metrics.
__device__ inline float ppo_obj(const HpK& hp, float lpa, float old_lp, float adv, float ent,
                                float ecoef, float objw, LossAcc& m) {
    const float ratio = __expf(lpa - old_lp);
    const float lo = 1.0f - hp.clip, hi = 1.0f + hp.clip;
    const float s1 = adv * ratio;
    const float y = fmaxf(ratio, lo);
    const float cr = fminf(y, hi);
    const float s2 = adv * cr;
    const float obj = fminf(s1, s2);
    // JAX's balanced min/max derivatives (0.5 on ties)
    const float dmx = ratio > lo ? 1.f : (ratio == lo ? 0.5f : 0.f);
    const float dmn = y < hi ? 1.f : (y == hi ? 0.5f : 0.f);
    const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
    const float dobj = w1 * adv + (1.f - w1) * adv * (dmx * dmn);
    m.sobj += obj;
    m.qobj += obj * obj;
    m.mnobj = fminf(m.mnobj, obj);
    m.mxobj = fmaxf(m.mxobj, obj);
    m.sent += ent;
    m.qent += ent * ent;
    m.mnent = fminf(m.mnent, ent);
    m.mxent = fmaxf(m.mxent, ent);
    m.sentw += ecoef * ent;
    m.sobjw += objw * obj;
    return -hp.inv_sk * objw * dobj * ratio;
}

// Group of at most MAXB logits held in registers (fixed width, masked): no
// dynamically indexed register arrays.
// S: storage of the logits row (f32, or the compute dtype bf16 when every
// consumer of the d logits rounds them to it anyway).
template <int MAXB, typename S>
__device__ inline void loss_group_fixed(const HpK& hp, S* lg, int nb, int a, float old_lp,
                                        float adv, float ecoef, float objw, LossAcc& m) {
    float v[MAXB];
#pragma unroll
    for (int j = 0; j < MAXB; ++j) v[j] = j < nb ? to_f32(lg[j]) : -3.4e38f;
    float mx = v[0];
#pragma unroll
    for (int j = 1; j < MAXB; ++j) mx = fmaxf(mx, v[j]);
    float ex[MAXB], se = 0.f, lpa = 0.f;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
        ex[j] = j < nb ? __expf(v[j] - mx) : 0.f;
        se += ex[j];
    }
    const float inv = 1.0f / se;
    const float lse = mx + __logf(se);
    float ent = 0.f;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
        if (j < nb) ent -= (ex[j] * inv) * (v[j] - lse);  // dists.py:68-69
        lpa = j == a ? v[j] - lse : lpa;
    }
    const float g_lp = ppo_obj(hp, lpa, old_lp, adv, ent, ecoef, objw, m);
    const float ce = ecoef * hp.inv_sk;  // entropy term weight
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
        const float p = ex[j] * inv;
        const float d = g_lp * ((j == a ? 1.f : 0.f) - p) + ce * p * ((v[j] - lse) + ent);
        if (j < nb) lg[j] = cvt<S>(d * hp.loss_scale);
    }
}

// Any group size (<= 31): three passes over the logits in LDS.
template <typename S>
__device__ inline void loss_group(const HpK& hp, S* lg, int nb, int a, float old_lp, float adv,
                                  float ecoef, float objw, LossAcc& m) {
    if (nb <= 8) {
        loss_group_fixed<8>(hp, lg, nb, a, old_lp, adv, ecoef, objw, m);
        return;
    }
    float mx = to_f32(lg[0]);
    for (int j = 1; j < nb; ++j) mx = fmaxf(mx, to_f32(lg[j]));
    float se = 0.f;
    for (int j = 0; j < nb; ++j) se += __expf(to_f32(lg[j]) - mx);
    const float inv = 1.0f / se;
    const float lse = mx + __logf(se);
    float ent = 0.f;
    for (int j = 0; j < nb; ++j) ent -= (__expf(to_f32(lg[j]) - mx) * inv) * (to_f32(lg[j]) - lse);
    const float g_lp = ppo_obj(hp, to_f32(lg[a]) - lse, old_lp, adv, ent, ecoef, objw, m);
    const float ce = ecoef * hp.inv_sk;
    for (int j = 0; j < nb; ++j) {
        const float lj = to_f32(lg[j]);
        const float p = __expf(lj - mx) * inv;
        const float d = g_lp * ((j == a ? 1.f : 0.f) - p) + ce * p * ((lj - lse) + ent);
        lg[j] = cvt<S>(d * hp.loss_scale);
    }
}

// Scalar critic (DenseLayerCritic): lg points at the row, value at column A;
// zeroes columns A+1..HC-1.
// vn (normalize_values, may be null) = {mu', inv_sigma'} after this
// minibatch's update and {mu, sigma} before it (mlearn_value_norm_chain).
// The value normaliser's four values held by the caller (von = vn != null).
struct VnVals {
    bool on;
    float v[4];
};
template <typename S>
__device__ inline void loss_value(const HpK& hp, S* lg, int A, int HC, float R, float ov,
                                  LossAcc& m, const VnVals& vn);
template <typename S>
__device__ inline void loss_value(const HpK& hp, S* lg, int A, int HC, float R, float ov,
                                  LossAcc& m, const float* vn) {
    VnVals w{vn != nullptr, {0.f, 0.f, 0.f, 0.f}};
    if (vn)
        for (int i = 0; i < 4; ++i) w.v[i] = vn[i];
    loss_value(hp, lg, A, HC, R, ov, m, w);
}
template <typename S>
__device__ inline void loss_value(const HpK& hp, S* lg, int A, int HC, float R, float ov,
                                  LossAcc& m, const VnVals& vn) {
    const float V = to_f32(lg[A]);
    // target: the return normalised with the updated estimates (ppo.py:209-211)
    const float tgt = vn.on ? (R - vn.v[0]) * vn.v[1] : R;
    float vpred = V, dvp = 1.f;
    if (hp.clip_vl) {  // ppo.py:197-203
        const float vlo = ov - hp.clip, vhi = ov + hp.clip;
        const float yy = fmaxf(V, vlo);
        vpred = fminf(yy, vhi);
        dvp = (V > vlo ? 1.f : (V == vlo ? 0.5f : 0.f)) * (yy < vhi ? 1.f : (yy == vhi ? 0.5f : 0.f));
    }
    const float e = vpred - tgt;
    float vl, dvl;
    if (hp.huber) {  // optax.huber_loss, delta = 1
        const float ae = fabsf(e);
        const float quad = fminf(ae, 1.f);
        vl = 0.5f * quad * quad + (ae - quad);
        dvl = ae < 1.f ? e : (e > 0.f ? 1.f : -1.f);
    } else {  // optax.l2_loss
        vl = 0.5f * e * e;
        dvl = e;
    }
    lg[A] = cvt<S>(hp.vcoef * hp.inv_s * dvl * dvp * hp.loss_scale);
    for (int j = A + 1; j < HC; ++j) lg[j] = cvt<S>(0.f);
    // value error: the critic inverted with the previous estimates (ppo.py:193-195)
    const float verr = fabsf((vn.on ? V * vn.v[3] + vn.v[2] : V) - R);
    m.svl += vl;
    m.qvl += vl * vl;
    m.mnvl = fminf(m.mnvl, vl);
    m.mxvl = fmaxf(m.mxvl, vl);
    m.serr += verr;
    m.qerr += verr * verr;
    m.mnerr = fminf(m.mnerr, verr);
    m.mxerr = fmaxf(m.mxerr, verr);
}

// DreamerV3Critic (ppo.py:169-177): value loss = two-hot cross entropy of the
// return against the CB bin logits at lg[A..A+CB); value error = mean() - R.
// Run by an aligned group of G lanes (lane sub); writes d loss / d bin
// logits in place, zeroes columns A+CB..HC-1; lane 0 of the group records
// the metrics.
template <int G>
__device__ inline void loss_value_twohot_g(const HpK& hp, float* lg, int A, int CB, int HC,
                                           const float* bins, float R, int sub, LossAcc& m) {
    float mean;
    const float vl =
        twohot_ce_g<G>(lg + A, CB, R, bins, hp.vcoef * hp.inv_s * hp.loss_scale, sub, &mean);
    for (int j = A + CB + sub; j < HC; j += G) lg[j] = 0.f;
    if (sub != 0) return;
    const float verr = fabsf(mean - R);
    m.svl += vl;
    m.qvl += vl * vl;
    m.mnvl = fminf(m.mnvl, vl);
    m.mxvl = fmaxf(m.mxvl, vl);
    m.serr += verr;
    m.qerr += verr * verr;
    m.mnerr = fminf(m.mnerr, verr);
    m.mxerr = fmaxf(m.mxerr, verr);
}


// ReLU' threshold: rnd<T>(y) > 0  <=>  y > THR (bf16 round-to-nearest-even
// sends y <= 2^-134 to zero).
template <typename T> __device__ inline float relu_thr();
template <> __device__ inline float relu_thr<float>() { return 0.f; }
template <> __device__ inline float relu_thr<bf16>() { return __builtin_bit_cast(float, 0x00008000u); }


// Return of store row q: the stored column, or advantages + values when the
// GAE did not materialise it (mlearn_rollout_view.returns = NULL): the same
// f32 addition as gae_kernel's, so the same bits.
__device__ inline float ret_at(const RolloutK& ro, int64_t q) {
    return ro.ret ? ro.ret[q] : ro.adv[q] + ro.values[q];
}

// Store row of minibatch row f (32-bit index math: rows, sequences and N are
// < 2^31, checked on the host).
__device__ inline int64_t store_row(const RolloutK& ro, const int32_t* mb_seq, int mb, int64_t f) {
    const uint32_t fu = (uint32_t)f, mbu = (uint32_t)mb, nu = (uint32_t)ro.N;
    const uint32_t tl = fu / mbu;
    const uint32_t m = fu - tl * mbu;
    const uint32_t seq = (uint32_t)mb_seq[m];
    const uint32_t c = seq / nu, b = seq - c * nu;
    return ((int64_t)c * ro.bptt + tl) * ro.ld + b;
}

}  // namespace ml
