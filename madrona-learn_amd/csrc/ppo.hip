// PPO minibatch step up to the flat gradient (ppo.py:109-364):
//
//   ppo_fwd   per 64-row tile: gather the minibatch rows straight from the
//             [T][N] rollout store (no RolloutData.minibatch copy,
//             rollouts.py:319-329), MLP trunk + heads, PPO loss terms
//             (ppo.py:129-262) and d loss / d {logits, value}.
//   ppo_bwd   per 64-row tile: back through heads, ReLU and LayerNorm of
//             every layer (row-local), writing dZ_l and LayerNorm
//             scale/bias partials.
//   wgrad     dW = X^T dZ over all rows (split-K slabs, MFMA with the
//             rows as the reduction axis staged transposed through LDS).
//   reduce    fixed-order sum of slabs and tile partials into the flat f32
//             gradient + loss/metric outputs.  Deterministic: no atomics.
//
// Minibatch row f (time-major like mb['obs'] of shape [T/C, mb]):
//   tl = f / mb, m = f % mb, seq = mb_seq[m], c = seq / N, b = seq % N,
//   store row = (c * bptt + tl) * N + b.

#include "common.h"
#include "mlp_tile.h"

namespace ml {

struct RolloutK {
    const void* obs;
    const int32_t* actions;
    const float* logp;
    const float* adv;
    const float* ret;
    const float* values;
    int T, bptt;
    int64_t N;
};

struct HpK {
    float clip, vcoef;
    float ecoef[MLEARN_MAX_GROUPS];
    int norm_adv, clip_vl, huber;
    float loss_scale;
    float inv_sk, inv_s;
};

constexpr int kLossSlots = 20;   // per tile doubles
constexpr int kStepRows = 32;    // rows per fused-step tile
#ifndef ML_STEP_WAVES
#define ML_STEP_WAVES 2
#endif
constexpr int kColChunks = 32;   // first-level chunks of the per-tile column partials
constexpr int kWgTile = 128;     // weight-gradient output tile (rows and cols)
constexpr int kWgChunk = 64;     // weight-gradient K chunk (rows of the minibatch)

struct WsK {
    void* x0T;                          // [D][Mp]   gathered obs, transposed
    void* aT[MLEARN_MAX_LAYERS];        // [H][Mp]   post-ReLU activations, transposed
    void* dheadT;                       // [32][Mp]  d loss / d head outputs, transposed
    void* dzT[MLEARN_MAX_LAYERS];       // [H][Mp]   d loss / d Dense outputs, transposed
    float* colpart;                     // [tiles][CP] per-tile column partials
    float* colpart2;                    // [kColChunks][CP]
    double* loss_part;                  // [tiles][kLossSlots]
    float* slab;                        // split-K partial weight gradients
    int64_t slab_off[MLEARN_MAX_LAYERS + 1];
    int splits[MLEARN_MAX_LAYERS + 1];
    int64_t rps[MLEARN_MAX_LAYERS + 1];  // rows per split
    int64_t Mp;
    int ntiles;
    int CP;                             // L*2*H + 32
    uint64_t* stamps;                   // diagnostic builds only (ML_STAMPS): [tiles][16]
};

#ifdef ML_STAMPS
static uint64_t* g_stamp_buf = nullptr;
#define STAMP(i)                                                                   \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        if (ws.stamps && threadIdx.x == 0)                                         \
            ws.stamps[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
#else
#define STAMP(i) \
    do {         \
    } while (0)
#endif

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Split-K plan of one weight gradient [I][J] over Mp rows: ~256 workgroups.
static void plan_splits(int I, int J, int64_t Mp, int* splits, int64_t* rps) {
    int tiles = ((I + kWgTile - 1) / kWgTile) * ((J + kWgTile - 1) / kWgTile);
    int64_t chunks = Mp / kWgChunk;
    int64_t s = 256 / tiles;
    if (s < 1) s = 1;
    if (s > chunks) s = chunks;
    int64_t per = (chunks + s - 1) / s;
    *rps = per * kWgChunk;
    *splits = (int)((Mp + *rps - 1) / *rps);
}

// Carve the workspace; returns total bytes (base may be null to size only).
static size_t carve(const mlearn_mlp_policy& p, int64_t M, char* base, WsK* W) {
    const size_t es = p.dtype == MLEARN_DTYPE_BF16 ? 2 : 4;
    const int H = p.hidden, D = p.obs_dim, L = p.num_layers;
    const int64_t tiles = (M + kStepRows - 1) / kStepRows;
    const int64_t Mp = ((tiles * kStepRows + kWgChunk - 1) / kWgChunk) * kWgChunk;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* ptr = base ? base + off : nullptr;
        off = align256(off + bytes);
        return (void*)ptr;
    };
    WsK w{};
    w.Mp = Mp;
    w.ntiles = (int)tiles;
    w.CP = L * 2 * H + MLEARN_HEAD_COLS;
    w.x0T = take(Mp * D * es);
    for (int l = 0; l < L; ++l) {
        w.aT[l] = take(Mp * H * es);
        w.dzT[l] = take(Mp * H * es);
    }
    w.dheadT = take(Mp * MLEARN_HEAD_COLS * es);
    w.colpart = (float*)take(tiles * w.CP * sizeof(float));
    w.colpart2 = (float*)take(kColChunks * w.CP * sizeof(float));
    w.loss_part = (double*)take(tiles * kLossSlots * sizeof(double));
    int64_t so = 0;
    for (int l = 0; l <= L; ++l) {
        const int I = l == L ? H : (l == 0 ? D : H);
        const int J = l == L ? MLEARN_HEAD_COLS : H;
        plan_splits(I, J, Mp, &w.splits[l], &w.rps[l]);
        w.slab_off[l] = so;
        so += (int64_t)w.splits[l] * I * J;
    }
    w.slab = (float*)take(so * sizeof(float));
    if (W) *W = w;
    return off;
}

// ---------------------------------------------------------------------------
// Fused minibatch step per 64-row tile: gather -> trunk forward -> heads ->
// PPO loss terms and d loss / d head -> backward through heads, ReLU and
// LayerNorm of every layer.  Each layer's Dense output stays in registers
// (packed bf16 pairs in bf16 mode) between the forward and the backward, so
// the only HBM writes are the weight-gradient operands (x0^T, a_l^T, dHead^T,
// dZ_l^T, feature-major) and the per-tile column / loss partials.
// ---------------------------------------------------------------------------
template <typename T, int NB> struct ZStore;
template <int NB> struct ZStore<bf16, NB> {
    uint32_t d[NB][8];
    __device__ void set(int i, int e, float x) {  // x is already bf16-valued
        const uint32_t b = __builtin_bit_cast(uint32_t, x) >> 16;
        d[i][e >> 1] = (e & 1) ? ((d[i][e >> 1] & 0x0000ffffu) | (b << 16))
                               : ((d[i][e >> 1] & 0xffff0000u) | b);
    }
    __device__ float get(int i, int e) const {
        const uint32_t b = (e & 1) ? (d[i][e >> 1] & 0xffff0000u) : (d[i][e >> 1] << 16);
        return __builtin_bit_cast(float, b);
    }
};
template <int NB> struct ZStore<float, NB> {
    float d[NB][16];
    __device__ void set(int i, int e, float x) { d[i][e] = x; }
    __device__ float get(int i, int e) const { return d[i][e]; }
};

// Per-row loss inputs gathered from the store at the start of the tile.
struct LossIn {
    int32_t* act;  // [ROWS][K]
    float* lp;     // [ROWS][K]
    float* adv;    // [ROWS]
    float* ret;    // [ROWS]
    float* val;    // [ROWS]
};

// PPO loss terms of the tile (ppo.py:129-262) and d loss / d {logits, value}
// into dl[ROWS][33]; per-tile loss/metric partials into ws.loss_part.
template <typename T, int ROWS, int THREADS>
__device__ inline void tile_loss(const PolicyK& P, const float* adv_st, const HpK& hp,
                                 const WsK& ws, const float* lgt, float* dl, const LossIn& in,
                                 const int64_t* srow, float* dred, int tid, int lane, int w) {
    const float adv_mean = adv_st[0], adv_rstd = adv_st[1];
    float sobj = 0, qobj = 0, sent = 0, qent = 0, svl = 0, qvl = 0, serr = 0, qerr = 0, sentw = 0;
    float mnobj = 3.4e38f, mxobj = -3.4e38f, mnent = 3.4e38f, mxent = -3.4e38f;
    float mnvl = 3.4e38f, mxvl = -3.4e38f, mnerr = 3.4e38f, mxerr = -3.4e38f;
    const int K = P.K, A = P.A;
    for (int task = tid; task < ROWS * (K + 1); task += THREADS) {
        const int rr = task / (K + 1), g = task - rr * (K + 1);
        if (srow[rr] < 0) {
            if (g == K)
                for (int j = 0; j < 33; ++j) dl[rr * 33 + j] = 0.f;
            continue;
        }
        if (g < K) {
            const float* lg = &lgt[rr * 33 + P.off[g]];
            const int nb = P.off[g + 1] - P.off[g];
            float mx = lg[0];
            for (int j = 1; j < nb; ++j) mx = fmaxf(mx, lg[j]);
            float ex[32];
            float se = 0.f;
            for (int j = 0; j < nb; ++j) {
                ex[j] = __expf(lg[j] - mx);
                se += ex[j];
            }
            const float inv = 1.0f / se;
            const float lse = mx + __logf(se);
            float ent = 0.f;
            for (int j = 0; j < nb; ++j) ent -= (ex[j] * inv) * (lg[j] - lse);  // dists.py:68-69
            const int a = in.act[rr * K + g];
            const float lpa = lg[a] - lse;
            float adv = in.adv[rr];
            if (hp.norm_adv) adv = (adv - adv_mean) * adv_rstd;
            const float ratio = __expf(lpa - in.lp[rr * K + g]);
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
            const float g_lp = -hp.inv_sk * dobj * ratio;  // d loss / d logp[a]
            const float ce = hp.ecoef[g] * hp.inv_sk;       // entropy term weight
            for (int j = 0; j < nb; ++j) {
                const float p = ex[j] * inv;
                const float d = g_lp * ((j == a ? 1.f : 0.f) - p) + ce * p * ((lg[j] - lse) + ent);
                dl[rr * 33 + P.off[g] + j] = d * hp.loss_scale;
            }
            sobj += obj;
            qobj += obj * obj;
            mnobj = fminf(mnobj, obj);
            mxobj = fmaxf(mxobj, obj);
            sent += ent;
            qent += ent * ent;
            mnent = fminf(mnent, ent);
            mxent = fmaxf(mxent, ent);
            sentw += hp.ecoef[g] * ent;
        } else {
            const float V = lgt[rr * 33 + A];
            const float R = in.ret[rr];
            float vpred = V, dvp = 1.f;
            if (hp.clip_vl) {  // ppo.py:197-203
                const float ov = in.val[rr];
                const float vlo = ov - hp.clip, vhi = ov + hp.clip;
                const float yy = fmaxf(V, vlo);
                vpred = fminf(yy, vhi);
                dvp = (V > vlo ? 1.f : (V == vlo ? 0.5f : 0.f)) *
                      (yy < vhi ? 1.f : (yy == vhi ? 0.5f : 0.f));
            }
            const float e = vpred - R;
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
            dl[rr * 33 + A] = hp.vcoef * hp.inv_s * dvl * dvp * hp.loss_scale;
            for (int j = A + 1; j < 33; ++j) dl[rr * 33 + j] = 0.f;
            const float verr = fabsf(V - R);
            svl += vl;
            qvl += vl * vl;
            mnvl = fminf(mnvl, vl);
            mxvl = fmaxf(mxvl, vl);
            serr += verr;
            qerr += verr * verr;
            mnerr = fminf(mnerr, verr);
            mxerr = fmaxf(mxerr, verr);
        }
    }
    // tile loss/metric partials: DPP over each half-wave, then the half-wave
    // partials in fixed order (f32 within the tile, f64 across tiles)
    const float vals[kLossSlots] = {sobj, qobj, mnobj, mxobj, svl, qvl, mnvl, mxvl,
                                    serr, qerr, mnerr, mxerr, sent, qent, mnent, mxent,
                                    sentw, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kLossSlots; ++s) {
        const int kind = (s < 16) ? (s & 3) : 0;
        float v = vals[s];
        v = kind == 2 ? half_reduce<2>(v) : (kind == 3 ? half_reduce<3>(v) : half_reduce<0>(v));
        if ((lane & 31) == 0) dred[(w * 2 + (lane >> 5)) * kLossSlots + s] = v;
    }
    lds_barrier();
    if (tid < kLossSlots) {
        const int kind = (tid < 16) ? (tid & 3) : 0;
        double v = dred[tid];
        for (int q = 1; q < 2 * (THREADS / 64); ++q) {
            double u = dred[q * kLossSlots + tid];
            v = kind == 2 ? fmin(v, u) : (kind == 3 ? fmax(v, u) : v + u);
        }
        ws.loss_part[(int64_t)blockIdx.x * kLossSlots + tid] = v;
    }
}

template <int H> struct StepCfg {
    static constexpr int W = H >= 128 ? 4 : 2;  // waves per workgroup
    static constexpr int CG = W;               // column groups (one row block)
    static constexpr int NB = H / 32 / W;      // column blocks per wave
    static constexpr int ROWS = 32;
    static constexpr int THREADS = 64 * W;
};

template <typename T, int H, int L> static size_t step_lds(int D, int K) {
    typedef StepCfg<H> C;
    const int ld = (D > H ? D : H) + 16 / (int)sizeof(T);
    size_t b = (size_t)C::ROWS * ld * sizeof(T);      // act
    b += (size_t)C::W * C::ROWS * 2 * 4;               // red
    b += 2 * (size_t)C::ROWS * 33 * 4;                 // lgt, dl
    b += (size_t)L * C::ROWS * 2 * 4;                  // stat
    b += 2 * (size_t)C::ROWS * K * 4 + 3 * C::ROWS * 4; // loss inputs
    b += (size_t)2 * C::W * kLossSlots * 4;            // dred
    b += (size_t)C::ROWS * 8;                           // srow
    return b;
}

template <typename T, int H, int L>
__global__ __launch_bounds__(StepCfg<H>::THREADS) __attribute__((amdgpu_waves_per_eu(ML_STEP_WAVES, 8))) void ppo_step_kernel(
    PolicyK P, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, int64_t M,
    const float* __restrict__ adv_st, HpK hp, WsK ws) {
    typedef StepCfg<H> C;
    constexpr int NB = C::NB, CG = C::CG, ROWS = C::ROWS, THREADS = C::THREADS;
    constexpr int PAD = Pad<T>::v;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D, K = P.K;
    const int ld = (D > H ? D : H) + PAD;
    const int ldh = MLEARN_HEAD_COLS + PAD;
    T* act = (T*)smem;                                  // [ROWS][ld]
    float* red = (float*)(act + ROWS * ld);             // [W][ROWS][2]
    float* lgt = red + C::W * ROWS * 2;                 // [ROWS][33]
    float* dl = lgt + ROWS * 33;                        // [ROWS][33]
    float* stat = dl + ROWS * 33;                       // [L][ROWS][2]
    LossIn in;
    in.act = (int32_t*)(stat + L * ROWS * 2);           // [ROWS][K]
    in.lp = (float*)(in.act + ROWS * K);                // [ROWS][K]
    in.adv = in.lp + ROWS * K;
    in.ret = in.adv + ROWS;
    in.val = in.ret + ROWS;
    float* dred = in.val + ROWS;                        // [2W][kLossSlots]
    int64_t* srow = (int64_t*)(((uintptr_t)(dred + 2 * C::W * kLossSlots) + 7) & ~(uintptr_t)7);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cg = w, r = lane & 31;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    STAMP(0);

    if (tid < ROWS) {
        const int64_t f = row0 + tid;
        int64_t sr = -1;
        if (f < M) {
            const int tl = (int)(f / mb);
            const int m = (int)(f - (int64_t)tl * mb);
            const int64_t seq = mb_seq[m];
            const int64_t c = seq / ro.N, b = seq - c * ro.N;
            sr = (c * ro.bptt + tl) * ro.N + b;
        }
        srow[tid] = sr;
    }
    lds_barrier();

    // gather the observation rows (16 B per lane) and the loss inputs
    {
        constexpr int V = 16 / sizeof(T);
        typedef __attribute__((ext_vector_type(4))) uint32_t u4;
        const T* obs = (const T*)ro.obs;
        const int cpr = D / V;
        for (int idx = tid; idx < ROWS * cpr; idx += THREADS) {
            const int rr = idx / cpr, c = (idx - rr * cpr) * V;
            const int64_t sr = srow[rr];
            u4 v = {0u, 0u, 0u, 0u};
            if (sr >= 0) v = *(const u4*)(obs + sr * D + c);
            *(u4*)(act + rr * ld + c) = v;
        }
        for (int idx = tid; idx < ROWS * K; idx += THREADS) {
            const int rr = idx / K, g = idx - rr * K;
            const int64_t sr = srow[rr];
            in.act[idx] = sr >= 0 ? ro.actions[sr * K + g] : 0;
            in.lp[idx] = sr >= 0 ? ro.logp[sr * K + g] : 0.f;
        }
        for (int rr = tid; rr < ROWS; rr += THREADS) {
            const int64_t sr = srow[rr];
            in.adv[rr] = sr >= 0 ? ro.adv[sr] : 0.f;
            in.ret[rr] = sr >= 0 ? ro.ret[sr] : 0.f;
            in.val[rr] = (sr >= 0 && ro.values) ? ro.values[sr] : 0.f;
        }
    }
    lds_barrier();
    store_tile_transposed<T, ROWS, THREADS>(act, ld, D, (T*)ws.x0T, ws.Mp, row0, M, tid);
    STAMP(1);

    // ---- forward ----
    ZStore<T, NB> z[L];
    f32x16 acc[NB];
    const float invH = 1.0f / (float)H;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        const int Kl = l == 0 ? D : H;
        zero_acc<NB>(acc);
        gemm_direct<T, NB, CG>(acc, act, ld, 0, (const T*)P.wt[l], Kl, H, cg, lane);
        STAMP(2 + 2 * l);
        float s[16], q[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const float x = rnd<T>(acc[i][e]);  // Dense output in the compute dtype
                acc[i][e] = x;
                z[l].set(i, e, x);
                a += x;
                b += x * x;
            }
            s[e] = a;
            q[e] = b;
        }
        row_reduce2<1, CG>(s, q, red, w, lane);  // (barrier: every wave is past its GEMM)
        float g[NB], bt[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            g[i] = P.lns[l][(cg + CG * i) * 32 + r];
            bt[i] = P.lnb[l][(cg + CG * i) * 32 + r];
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = acc_row(e, lane);
            const float mean = s[e] * invH;
            const float var = fmaxf(q[e] * invH - mean * mean, 0.f);
            const float rstd = rsqrtf(var + 1e-6f);
            if (cg == 0 && r == 0) {
                stat[(l * ROWS + row) * 2] = mean;
                stat[(l * ROWS + row) * 2 + 1] = rstd;
            }
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int col = (cg + CG * i) * 32 + r;
                const float y = fmaxf(rnd<T>((acc[i][e] - mean) * (rstd * g[i]) + bt[i]), 0.f);
                act[row * ld + col] = cvt<T>(y);
            }
        }
        lds_barrier();
        store_tile_transposed<T, ROWS, THREADS>(act, ld, H, (T*)ws.aT[l], ws.Mp, row0, M, tid);
        STAMP(3 + 2 * l);
    }
    heads_to_lds<T, 1, CG>(act, ld, (const T*)P.head_t, P.head_b, H, lgt, w, lane);
    lds_barrier();
    STAMP(6);

    // ---- loss ----
    tile_loss<T, ROWS, THREADS>(P, adv_st, hp, ws, lgt, dl, in, srow, dred, tid, lane, w);
    lds_barrier();
    STAMP(7);
    for (int idx = tid; idx < MLEARN_HEAD_COLS * (ROWS / 4); idx += THREADS) {
        const int j = idx % MLEARN_HEAD_COLS, gq = idx / MLEARN_HEAD_COLS;
        store4((T*)ws.dheadT + (int64_t)j * ws.Mp + row0 + 4 * gq, dl[(4 * gq) * 33 + j],
               dl[(4 * gq + 1) * 33 + j], dl[(4 * gq + 2) * 33 + j], dl[(4 * gq + 3) * 33 + j]);
    }
    if (tid < MLEARN_HEAD_COLS) {
        float sum = 0.f;
        for (int rr = 0; rr < ROWS; ++rr) sum += rnd<T>(dl[rr * 33 + tid]);
        ws.colpart[(int64_t)blockIdx.x * ws.CP + L * 2 * H + tid] = sum;
    }
    for (int idx = tid; idx < ROWS * MLEARN_HEAD_COLS; idx += THREADS) {
        const int rr = idx / MLEARN_HEAD_COLS, j = idx - rr * MLEARN_HEAD_COLS;
        act[rr * ldh + j] = cvt<T>(dl[rr * 33 + j]);
    }
    lds_barrier();
    STAMP(8);

    // ---- backward ----
    zero_acc<NB>(acc);
    // dA_{L-1} = dHead . Head^T    (B^T = head [H][32])
    gemm_direct<T, NB, CG>(acc, act, ldh, 0, (const T*)P.head, MLEARN_HEAD_COLS, H, cg, lane);
    STAMP(9);
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
        float su[16], sv[16], pg[NB], pb[NB], gm[NB], bt[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            pg[i] = pb[i] = 0.f;
            gm[i] = P.lns[l][(cg + CG * i) * 32 + r];
            bt[i] = P.lnb[l][(cg + CG * i) * 32 + r];
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = acc_row(e, lane);
            const bool live = row0 + row < M;
            const float mean = stat[(l * ROWS + row) * 2];
            const float rstd = stat[(l * ROWS + row) * 2 + 1];
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const float zc = z[l].get(i, e) - mean;
                const float xh = zc * rstd;
                const float y = zc * (rstd * gm[i]) + bt[i];
                const float dy = (live && rnd<T>(y) > 0.f) ? acc[i][e] : 0.f;  // ReLU'
                const float u = dy * gm[i];
                acc[i][e] = u;
                a += u;
                b += u * xh;
                pg[i] += dy * xh;
                pb[i] += dy;
            }
            su[e] = a;
            sv[e] = b;
        }
        // LayerNorm scale/bias partials: fold the two half-waves, one writer per column
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            pg[i] += __shfl_xor(pg[i], 32);
            pb[i] += __shfl_xor(pb[i], 32);
            if (lane < 32) {
                const int col = (cg + CG * i) * 32 + r;
                float* lp = ws.colpart + (int64_t)blockIdx.x * ws.CP + (l * 2) * H;
                lp[col] = pb[i];
                lp[H + col] = pg[i];
            }
        }
        row_reduce2<1, CG>(su, sv, red, w, lane);  // (barrier: every wave is past its GEMM)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = acc_row(e, lane);
            const float mean = stat[(l * ROWS + row) * 2];
            const float rstd = stat[(l * ROWS + row) * 2 + 1];
            const float mu = su[e] * invH, mv = sv[e] * invH;
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int col = (cg + CG * i) * 32 + r;
                const float xh = (z[l].get(i, e) - mean) * rstd;
                act[row * ld + col] = cvt<T>(rstd * (acc[i][e] - mu - xh * mv));
            }
        }
        lds_barrier();
        store_tile_transposed<T, ROWS, THREADS>(act, ld, H, (T*)ws.dzT[l], ws.Mp, row0, M, tid);
        STAMP(10 + 2 * (L - 1 - l));
        if (l > 0) {
            zero_acc<NB>(acc);
            // dA_{l-1} = dZ_l . W_l^T   (B^T = W_l [in][H])
            gemm_direct<T, NB, CG>(acc, act, ld, 0, (const T*)P.w[l], H, H, cg, lane);
            STAMP(11 + 2 * (L - 1 - l));
        }
    }
}

template <typename T, int H, int L>
static void launch_step(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                        int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                        hipStream_t s) {
    auto k = ppo_step_kernel<T, H, L>;
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  128 * 1024);
        attr_set = true;
    }
    const size_t lds = step_lds<T, H, L>(P.D, P.K);
    hipLaunchKernelGGL(k, dim3(ws.ntiles), dim3(StepCfg<H>::THREADS), lds, s, P, R, mb_seq, mb, M,
                       adv_st, hp, ws);
}

// ---------------------------------------------------------------------------
// Weight gradient dW[i][j] = sum_k XT[i][k] * YT[j][k] (NT GEMM, both operands
// feature-major so every lane streams whole 128-B lines along k).
// Tile 128 (i) x 128 (j): 4 waves in 2x2, each 64x64 = 2x2 MFMA blocks.
// Split-K over the minibatch rows; each split writes an f32 slab that the
// reduce kernel sums in split order.  Within a 64-row K chunk, half-wave h
// supplies k in [32h, 32h+32): the same permutation for A and B, so the
// MFMA reduction covers the chunk exactly once.
// ---------------------------------------------------------------------------
template <typename T>
__device__ inline void load_row32(const T* p, typename MT<T>::frag (&f)[32 / MT<T>::E]);

template <>
__device__ inline void load_row32<bf16>(const bf16* p, bf16x8 (&f)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) f[s] = *(const bf16x8*)(p + 8 * s);
}
template <>
__device__ inline void load_row32<float>(const float* p, float (&f)[32]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        float4 v = *(const float4*)(p + 4 * s);
        f[4 * s] = v.x;
        f[4 * s + 1] = v.y;
        f[4 * s + 2] = v.z;
        f[4 * s + 3] = v.w;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void wgrad_nt_kernel(const T* __restrict__ XT,
                                                       const T* __restrict__ YT, int64_t ldk,
                                                       int I, int J, int64_t rps, float* slab) {
    constexpr int E = MT<T>::E, NS = 32 / E;
    typedef typename MT<T>::frag frag;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wi = w & 1, wj = w >> 1;
    const int i0 = blockIdx.x * kWgTile + wi * 64;
    const int j0 = blockIdx.y * kWgTile + wj * 64;
    const bool ai[2] = {i0 < I, i0 + 32 < I};
    const bool bj[2] = {j0 < J, j0 + 32 < J};
    if (!ai[0] || !bj[0]) return;  // whole wave out of range (no barriers below)
    const int64_t k0 = blockIdx.z * rps;
    const int64_t k1 = k0 + rps < ldk ? k0 + rps : ldk;
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    const T* xp[2];
    const T* yp[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        // rows past I / J (I = obs_dim may be a multiple of 16 only) read a valid
        // row; their outputs are dropped below
        const int xi = i0 + 32 * a + r < I ? i0 + 32 * a + r : I - 1;
        const int yj = j0 + 32 * a + r < J ? j0 + 32 * a + r : J - 1;
        xp[a] = XT + (int64_t)xi * ldk + 32 * h;
        yp[a] = YT + (int64_t)yj * ldk + 32 * h;
    }
    for (int64_t k = k0; k < k1; k += kWgChunk) {
        frag fa[2][NS], fb[2][NS];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            load_row32<T>(xp[a] + k, fa[a]);
            load_row32<T>(yp[a] + k, fb[a]);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = MT<T>::mma(fa[a][s], fb[b][s], acc[a][b]);
    }
    float* out = slab + (int64_t)blockIdx.z * I * J;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        if (!ai[a]) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            if (!bj[b]) continue;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                int i = i0 + 32 * a + acc_row(e, lane);
                int j = j0 + 32 * b + r;
                if (i < I && j < J) out[(int64_t)i * J + j] = acc[a][b][e];
            }
        }
    }
}

// First level of the per-tile column partials (LayerNorm scale/bias grads,
// head-bias grad): colpart2[c][col] = sum over tiles t = c, c + 32, ...
__global__ __launch_bounds__(256) void colsum_kernel(WsK ws) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (col >= ws.CP) return;
    float s = 0.f;
    for (int t = c; t < ws.ntiles; t += kColChunks) s += ws.colpart[(int64_t)t * ws.CP + col];
    ws.colpart2[(int64_t)c * ws.CP + col] = s;
}

// ---------------------------------------------------------------------------
// Fixed-order reduction into the flat gradient.
// ---------------------------------------------------------------------------
LayoutK make_layout(const mlearn_mlp_policy& p) {
    LayoutK k{};
    k.L = p.num_layers;
    k.D = p.obs_dim;
    k.H = p.hidden;
    k.A1 = p.actions.num_logits + 1;
    int64_t o = 0;
    for (int l = 0; l < k.L; ++l) {
        k.w_off[l] = o;
        o += (int64_t)(l == 0 ? k.D : k.H) * k.H;
        k.s_off[l] = o;
        o += k.H;
        k.b_off[l] = o;
        o += k.H;
    }
    k.hw_off = o;
    o += (int64_t)k.H * k.A1;
    k.hb_off = o;
    o += k.A1;
    k.total = o;
    return k;
}

__global__ __launch_bounds__(256) void reduce_grads_kernel(LayoutK Lk, WsK ws, float* grad) {
    int64_t p = blockIdx.x * (int64_t)256 + threadIdx.x;
    if (p >= Lk.total) return;
    const int H = Lk.H, L = Lk.L;
    float g = 0.f;
    auto colsum = [&](int col) {
        float t = 0.f;
        for (int c = 0; c < kColChunks; ++c) t += ws.colpart2[(int64_t)c * ws.CP + col];
        return t;
    };
    if (p >= Lk.hb_off) {
        g = colsum(L * 2 * H + (int)(p - Lk.hb_off));
    } else if (p >= Lk.hw_off) {
        int64_t q = p - Lk.hw_off;
        int i = (int)(q / Lk.A1), j = (int)(q % Lk.A1);
        const float* s = ws.slab + ws.slab_off[L] + (int64_t)i * MLEARN_HEAD_COLS + j;
        const int64_t stride = (int64_t)H * MLEARN_HEAD_COLS;
        for (int k = 0; k < ws.splits[L]; ++k) g += s[k * stride];
    } else {
        int l = L - 1;
        while (l > 0 && p < Lk.w_off[l]) --l;
        if (p >= Lk.s_off[l]) {
            const int which = p >= Lk.b_off[l] ? 0 : 1;  // 0: bias (beta), 1: scale (gamma)
            const int col = (int)(p - (which ? Lk.s_off[l] : Lk.b_off[l]));
            g = colsum((l * 2 + which) * H + col);
        } else {
            const int I = l == 0 ? Lk.D : H;
            const float* s = ws.slab + ws.slab_off[l] + (p - Lk.w_off[l]);
            const int64_t stride = (int64_t)I * H;
            for (int k = 0; k < ws.splits[l]; ++k) g += s[k * stride];
        }
    }
    grad[p] = g;
}

// loss_out: five Metric vectors {mean, m2, min, max, count} in the order of
// PPO.add_metrics (ppo.py:95-106): 'Loss' (scalar: {loss, 0, loss, loss, 1}),
// 'Action Obj', 'Value Loss', 'Value Errors', 'Entropy'.
__global__ __launch_bounds__(1024) void reduce_loss_kernel(WsK ws, HpK hp, int64_t M, int K,
                                                            float* out) {
    __shared__ double sh[16][kLossSlots];
    __shared__ double tot[kLossSlots];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double v[kLossSlots];
#pragma unroll
    for (int s = 0; s < kLossSlots; ++s) {
        const int kind = (s < 16) ? (s & 3) : 0;
        v[s] = kind == 2 ? 3.4e38 : (kind == 3 ? -3.4e38 : 0.0);
    }
    for (int t = tid; t < ws.ntiles; t += 1024) {
#pragma unroll
        for (int s = 0; s < kLossSlots; ++s) {
            const int kind = (s < 16) ? (s & 3) : 0;
            double u = ws.loss_part[(int64_t)t * kLossSlots + s];
            v[s] = kind == 2 ? fmin(v[s], u) : (kind == 3 ? fmax(v[s], u) : v[s] + u);
        }
    }
#pragma unroll
    for (int s = 0; s < kLossSlots; ++s) {
        const int kind = (s < 16) ? (s & 3) : 0;
        double x = v[s];
        for (int o = 1; o < 64; o <<= 1) {
            double u = __shfl_xor(x, o);
            x = kind == 2 ? fmin(x, u) : (kind == 3 ? fmax(x, u) : x + u);
        }
        if (lane == 0) sh[w][s] = x;
    }
    __syncthreads();
    if (tid < kLossSlots) {
        const int kind = (tid < 16) ? (tid & 3) : 0;
        double x = sh[0][tid];
        for (int i = 1; i < 16; ++i) {
            double u = sh[i][tid];
            x = kind == 2 ? fmin(x, u) : (kind == 3 ? fmax(x, u) : x + u);
        }
        tot[tid] = x;
    }
    __syncthreads();
    if (tid == 0) {
        const double nk = (double)M * K, n = (double)M;
        const double obj_mean = tot[0] / nk, vl_mean = tot[4] / n;
        // loss = -mean(obj) + c_v * mean(vl) - sum_k c_e[k] * mean(H_k)   (ppo.py:241-252)
        const double loss = -obj_mean + hp.vcoef * vl_mean - tot[16] / nk;
        out[0] = (float)loss;
        out[1] = 0.f;
        out[2] = (float)loss;
        out[3] = (float)loss;
        out[4] = 1.f;
        const double cnt[4] = {nk, n, n, nk};
        for (int m = 0; m < 4; ++m) {
            double mean = tot[4 * m] / cnt[m];
            double m2 = tot[4 * m + 1] - cnt[m] * mean * mean;
            out[5 + 5 * m + 0] = (float)mean;
            out[5 + 5 * m + 1] = (float)(m2 > 0 ? m2 : 0);
            out[5 + 5 * m + 2] = (float)tot[4 * m + 2];
            out[5 + 5 * m + 3] = (float)tot[4 * m + 3];
            out[5 + 5 * m + 4] = (float)cnt[m];
        }
    }
}

template <typename T, int H>
static int launch_minibatch(const mlearn_mlp_policy& p, const mlearn_rollout_view& ro,
                            const int32_t* mb_seq, int mb, const float* adv_st,
                            const mlearn_ppo_hparams& h, float* grad, float* loss_out, void* wsp,
                            hipStream_t s) {
    const int64_t M = (int64_t)mb * ro.bptt_len;
    WsK ws;
    carve(p, M, (char*)wsp, &ws);
#ifdef ML_STAMPS
    ws.stamps = g_stamp_buf;
#endif
    PolicyK P = make_policy_k(p);
    RolloutK R{ro.obs, ro.actions, ro.log_probs, ro.advantages, ro.returns, ro.values,
               ro.T, ro.bptt_len, ro.N};
    HpK hp{};
    hp.clip = h.clip_coef;
    hp.vcoef = h.value_loss_coef;
    for (int i = 0; i < MLEARN_MAX_GROUPS; ++i) hp.ecoef[i] = h.entropy_coef[i];
    hp.norm_adv = h.normalize_advantages;
    hp.clip_vl = h.clip_value_loss;
    hp.huber = h.huber_value_loss;
    hp.loss_scale = h.loss_scale;
    hp.inv_s = (float)(1.0 / (double)M);
    hp.inv_sk = (float)(1.0 / ((double)M * p.actions.num_groups));

    switch (p.num_layers) {
        case 1: launch_step<T, H, 1>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
        case 2: launch_step<T, H, 2>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
        case 3: launch_step<T, H, 3>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
        default: launch_step<T, H, 4>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
    }
    const int L = p.num_layers;
    for (int l = 0; l <= L; ++l) {
        const int I = l == L ? H : (l == 0 ? p.obs_dim : H);
        const int J = l == L ? MLEARN_HEAD_COLS : H;
        const T* X = l == 0 ? (const T*)ws.x0T : (const T*)ws.aT[l - 1];
        const T* Y = l == L ? (const T*)ws.dheadT : (const T*)ws.dzT[l];
        dim3 g((I + kWgTile - 1) / kWgTile, (J + kWgTile - 1) / kWgTile, ws.splits[l]);
        hipLaunchKernelGGL(wgrad_nt_kernel<T>, g, dim3(256), 0, s, X, Y, ws.Mp, I, J, ws.rps[l],
                           ws.slab + ws.slab_off[l]);
    }
    hipLaunchKernelGGL(colsum_kernel, dim3((ws.CP + 255) / 256, kColChunks), dim3(256), 0, s, ws);
    LayoutK Lk = make_layout(p);
    hipLaunchKernelGGL(reduce_grads_kernel, dim3((unsigned)((Lk.total + 255) / 256)), dim3(256), 0,
                       s, Lk, ws, grad);
    if (loss_out)
        hipLaunchKernelGGL(reduce_loss_kernel, dim3(1), dim3(1024), 0, s, ws, hp, M,
                           p.actions.num_groups, loss_out);
    return check_launch("ppo_minibatch_grad");
}

}  // namespace ml

using namespace ml;

extern "C" {

#ifdef ML_STAMPS
// diagnostic builds only: phase timestamps of the fused minibatch kernel
void mlearn_debug_set_stamp_buffer(uint64_t* buf) { g_stamp_buf = buf; }
#endif

int64_t mlearn_param_count(const mlearn_mlp_policy* policy) {
    if (validate_policy(policy)) return -1;
    return make_layout(*policy).total;
}

int64_t mlearn_ppo_workspace_bytes(const mlearn_mlp_policy* policy, int64_t rows) {
    if (validate_policy(policy) || rows < 1) return -1;
    return (int64_t)carve(*policy, rows, nullptr, nullptr);
}

int mlearn_ppo_minibatch_grad(const mlearn_mlp_policy* policy, const mlearn_rollout_view* ro,
                              const int32_t* mb_seq, int32_t mb_size, const float* adv_stats,
                              const mlearn_ppo_hparams* hp, float* grad, float* loss_out,
                              void* workspace, mlearn_stream_t stream) {
    int rc = validate_policy(policy);
    if (rc) return rc;
    ML_REQUIRE(ro && mb_seq && adv_stats && hp && grad && workspace, "ppo: null pointer");
    ML_REQUIRE(mb_size >= 1, "ppo: mb_size must be >= 1");
    ML_REQUIRE(ro->bptt_len >= 1 && ro->T % ro->bptt_len == 0, "ppo: bad bptt_len");
    ML_REQUIRE(ro->obs && ro->actions && ro->log_probs && ro->advantages && ro->returns,
               "ppo: null rollout array");
    ML_REQUIRE(!hp->clip_value_loss || ro->values, "ppo: clip_value_loss needs values");
    hipStream_t s = S(stream);
#define ML_DISPATCH(T)                                                                           \
    switch (policy->hidden) {                                                                   \
        case 64: return launch_minibatch<T, 64>(*policy, *ro, mb_seq, mb_size, adv_stats, *hp,  \
                                                grad, loss_out, workspace, s);                  \
        case 128: return launch_minibatch<T, 128>(*policy, *ro, mb_seq, mb_size, adv_stats, *hp, \
                                                  grad, loss_out, workspace, s);                \
        default: return launch_minibatch<T, 256>(*policy, *ro, mb_seq, mb_size, adv_stats, *hp, \
                                                 grad, loss_out, workspace, s);                 \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
}

}  // extern "C"
