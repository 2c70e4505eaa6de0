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
    int CP;                             // L*4*H + 32
};

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
    const int64_t tiles = (M + kTileRows - 1) / kTileRows;
    const int64_t Mp = tiles * kTileRows;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* ptr = base ? base + off : nullptr;
        off = align256(off + bytes);
        return (void*)ptr;
    };
    WsK w{};
    w.Mp = Mp;
    w.ntiles = (int)tiles;
    w.CP = L * 4 * H + MLEARN_HEAD_COLS;
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

// PPO loss terms of the tile (ppo.py:129-262) and d loss / d {logits, value}
// into dl[64][33]; per-tile loss/metric partials into ws.loss_part.
template <typename T>
__device__ inline void tile_loss(const PolicyK& P, const RolloutK& ro, const float* adv_st,
                                 const HpK& hp, const WsK& ws, const float* lgt, float* dl,
                                 const int64_t* srow, double* dred, int tid, int lane, int w) {
    // loss terms: tasks (row, group) then (row, value)
    const float adv_mean = adv_st[0], adv_rstd = adv_st[1];
    double sobj = 0, qobj = 0, sent = 0, qent = 0, svl = 0, qvl = 0, serr = 0, qerr = 0, sentw = 0;
    float mnobj = 3.4e38f, mxobj = -3.4e38f, mnent = 3.4e38f, mxent = -3.4e38f;
    float mnvl = 3.4e38f, mxvl = -3.4e38f, mnerr = 3.4e38f, mxerr = -3.4e38f;
    const int K = P.K, A = P.A;
    for (int task = tid; task < kTileRows * (K + 1); task += 256) {
        int rr = task / (K + 1), g = task - rr * (K + 1);
        int64_t sr = srow[rr];
        if (sr < 0) {
            if (g == K)
                for (int j = 0; j < 33; ++j) dl[rr * 33 + j] = 0.f;
            continue;
        }
        if (g < K) {
            const float* lg = &lgt[rr * 33 + P.off[g]];
            const int nb = P.off[g + 1] - P.off[g];
            float mx = lg[0];
            for (int j = 1; j < nb; ++j) mx = fmaxf(mx, lg[j]);
            float se = 0.f;
            for (int j = 0; j < nb; ++j) se += __expf(lg[j] - mx);
            const float lse = mx + __logf(se);
            float ent = 0.f;
            for (int j = 0; j < nb; ++j) {
                float lp = lg[j] - lse;
                ent -= (__expf(lg[j] - mx) / se) * lp;  // softmax * log_softmax (dists.py:68-69)
            }
            const int a = ro.actions[sr * K + g];
            const float lpa = lg[a] - lse;
            const float old = ro.logp[sr * K + g];
            float adv = ro.adv[sr];
            if (hp.norm_adv) adv = (adv - adv_mean) * adv_rstd;
            const float ratio = __expf(lpa - old);
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
            const float g_lp = -hp.inv_sk * dobj * ratio;          // d loss / d logp[a]
            const float ce = hp.ecoef[g] * hp.inv_sk;               // entropy term weight
            for (int j = 0; j < nb; ++j) {
                float p = __expf(lg[j] - mx) / se;
                float lp = lg[j] - lse;
                float d = g_lp * ((j == a ? 1.f : 0.f) - p) + ce * p * (lp + ent);
                dl[rr * 33 + P.off[g] + j] = d * hp.loss_scale;
            }
            sobj += obj;
            qobj += (double)obj * obj;
            mnobj = fminf(mnobj, obj);
            mxobj = fmaxf(mxobj, obj);
            sent += ent;
            qent += (double)ent * ent;
            mnent = fminf(mnent, ent);
            mxent = fmaxf(mxent, ent);
            sentw += (double)hp.ecoef[g] * ent;
        } else {
            const float V = lgt[rr * 33 + A];
            const float R = ro.ret[sr];
            float vpred = V, dvp = 1.f;
            if (hp.clip_vl) {  // ppo.py:197-203
                const float ov = ro.values[sr];
                const float vlo = ov - hp.clip, vhi = ov + hp.clip;
                const float yy = fmaxf(V, vlo);
                vpred = fminf(yy, vhi);
                dvp = (V > vlo ? 1.f : (V == vlo ? 0.5f : 0.f)) * (yy < vhi ? 1.f : (yy == vhi ? 0.5f : 0.f));
            }
            const float e = vpred - R;
            float vl, dvl;
            if (hp.huber) {  // optax.huber_loss, delta = 1
                const float ae = fabsf(e);
                const float quad = fminf(ae, 1.f);
                vl = 0.5f * quad * quad + (ae - quad);
                dvl = ae < 1.f ? e : (e > 0.f ? 1.f : -1.f);
            } else {         // optax.l2_loss
                vl = 0.5f * e * e;
                dvl = e;
            }
            dl[rr * 33 + A] = hp.vcoef * hp.inv_s * dvl * dvp * hp.loss_scale;
            for (int j = A + 1; j < 33; ++j) dl[rr * 33 + j] = 0.f;
            const float verr = fabsf(V - R);
            svl += vl;
            qvl += (double)vl * vl;
            mnvl = fminf(mnvl, vl);
            mxvl = fmaxf(mxvl, vl);
            serr += verr;
            qerr += (double)verr * verr;
            mnerr = fminf(mnerr, verr);
            mxerr = fmaxf(mxerr, verr);
        }
    }
    __syncthreads();
    // tile loss/metric partials
    double vals[kLossSlots] = {sobj, qobj, mnobj, mxobj, svl, qvl, mnvl, mxvl,
                               serr, qerr, mnerr, mxerr, sent, qent, mnent, mxent, sentw, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < kLossSlots; ++s) {
        double v = vals[s];
        const int kind = (s < 16) ? (s & 3) : 0;  // 0,1 sum; 2 min; 3 max
        for (int o = 1; o < 64; o <<= 1) {
            double u = __shfl_xor(v, o);
            v = kind == 2 ? fmin(v, u) : (kind == 3 ? fmax(v, u) : v + u);
        }
        if (lane == 0) dred[w * kLossSlots + s] = v;
    }
    __syncthreads();
    if (tid < kLossSlots) {
        const int kind = (tid < 16) ? (tid & 3) : 0;
        double v = dred[tid];
        for (int ww = 1; ww < 4; ++ww) {
            double u = dred[ww * kLossSlots + tid];
            v = kind == 2 ? fmin(v, u) : (kind == 3 ? fmax(v, u) : v + u);
        }
        ws.loss_part[(int64_t)blockIdx.x * kLossSlots + tid] = v;
    }
}

template <typename T, int H, int L>
__global__ __launch_bounds__(256) void ppo_step_kernel(PolicyK P, RolloutK ro,
                                                       const int32_t* __restrict__ mb_seq, int mb,
                                                       int64_t M, const float* __restrict__ adv_st,
                                                       HpK hp, WsK ws) {
    constexpr int NB = H / 64;
    constexpr int PAD = Pad<T>::v;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D;
    const int ld = (D > H ? D : H) + PAD;
    const int ldh = MLEARN_HEAD_COLS + PAD;
    T* act = (T*)smem;
    float* red = (float*)(smem + (size_t)kTileRows * ld * sizeof(T));  // [4][64][2]
    float* lgt = red + 4 * 64 * 2;                                      // [64][33]
    float* dl = lgt + kTileRows * 33;                                   // [64][33]
    float* stat = dl + kTileRows * 33;                                  // [L][64][2]
    int64_t* srow = (int64_t*)(stat + L * kTileRows * 2);               // [64]
    double* dred = (double*)(srow + kTileRows);                         // [4][kLossSlots]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rb = w & 1, r = lane & 31;
    const int64_t row0 = (int64_t)blockIdx.x * kTileRows;

    if (tid < kTileRows) {
        int64_t f = row0 + tid;
        int64_t sr = -1;
        if (f < M) {
            int tl = (int)(f / mb);
            int m = (int)(f - (int64_t)tl * mb);
            int64_t seq = mb_seq[m];
            int64_t c = seq / ro.N, b = seq - c * ro.N;
            sr = (c * ro.bptt + tl) * ro.N + b;
        }
        srow[tid] = sr;
    }
    __syncthreads();

    // gather the observation rows, 16 B per lane
    {
        constexpr int V = 16 / sizeof(T);
        typedef __attribute__((ext_vector_type(4))) uint32_t u32x4v;
        const T* obs = (const T*)ro.obs;
        const int cpr = D / V;  // 16-B chunks per row
        for (int idx = tid; idx < kTileRows * cpr; idx += 256) {
            int rr = idx / cpr, c = (idx - rr * cpr) * V;
            int64_t sr = srow[rr];
            u32x4v v = {0u, 0u, 0u, 0u};
            if (sr >= 0) v = *(const u32x4v*)(obs + sr * D + c);
            *(u32x4v*)(act + rr * ld + c) = v;
        }
    }
    __syncthreads();
    {
        T* x0T = (T*)ws.x0T;
        for (int idx = tid; idx < D * (kTileRows / 4); idx += 256) {
            int c = idx % D, g = idx / D;
            store4(x0T + (int64_t)c * ws.Mp + row0 + 4 * g, to_f32(act[(4 * g) * ld + c]),
                   to_f32(act[(4 * g + 1) * ld + c]), to_f32(act[(4 * g + 2) * ld + c]),
                   to_f32(act[(4 * g + 3) * ld + c]));
        }
    }

    // ---- forward ----
    ZStore<T, NB> z[L];
    f32x16 acc[NB];
    const float invH = 1.0f / (float)H;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        const int K = l == 0 ? D : H;
        zero_acc<NB>(acc);
        tile_gemm<T, NB>(acc, act, ld, rb, (const T*)P.wt[l], K, K, w, lane);
        __syncthreads();
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
        row_reduce2(s, q, red, w, lane);
        const float* gamma = P.lns[l];
        const float* beta = P.lnb[l];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = rb * 32 + acc_row(e, lane);
            const float mean = s[e] * invH;
            const float var = fmaxf(q[e] * invH - mean * mean, 0.f);
            const float rstd = rsqrtf(var + 1e-6f);
            if ((w >> 1) == 0 && r == 0) {
                stat[(l * kTileRows + row) * 2] = mean;
                stat[(l * kTileRows + row) * 2 + 1] = rstd;
            }
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int col = ((w >> 1) + 2 * i) * 32 + r;
                float y = (acc[i][e] - mean) * (rstd * gamma[col]) + beta[col];
                y = fmaxf(rnd<T>(y), 0.f);
                act[row * ld + col] = cvt<T>(y);
                acc[i][e] = y;
            }
        }
        store_transposed<T, NB>(acc, (T*)ws.aT[l], ws.Mp, w, lane, row0, M);
        __syncthreads();
    }
    heads_to_lds<T>(act, ld, (const T*)P.head_t, P.head_b, H, lgt, w, lane);
    __syncthreads();

    // ---- loss ----
    tile_loss<T>(P, ro, adv_st, hp, ws, lgt, dl, srow, dred, tid, lane, w);
    // (tile_loss ends with a barrier: dl is complete)
    {
        T* dhT = (T*)ws.dheadT;
        for (int idx = tid; idx < MLEARN_HEAD_COLS * (kTileRows / 4); idx += 256) {
            int j = idx % MLEARN_HEAD_COLS, g = idx / MLEARN_HEAD_COLS;
            store4(dhT + (int64_t)j * ws.Mp + row0 + 4 * g, dl[(4 * g) * 33 + j],
                   dl[(4 * g + 1) * 33 + j], dl[(4 * g + 2) * 33 + j], dl[(4 * g + 3) * 33 + j]);
        }
    }
    if (tid < MLEARN_HEAD_COLS) {
        float sum = 0.f;
        for (int rr = 0; rr < kTileRows; ++rr) sum += rnd<T>(dl[rr * 33 + tid]);
        ws.colpart[(int64_t)blockIdx.x * ws.CP + L * 4 * H + tid] = sum;
    }
    for (int idx = tid; idx < kTileRows * MLEARN_HEAD_COLS; idx += 256) {
        int rr = idx / MLEARN_HEAD_COLS, j = idx - rr * MLEARN_HEAD_COLS;
        act[rr * ldh + j] = cvt<T>(dl[rr * 33 + j]);
    }
    __syncthreads();

    // ---- backward ----
    zero_acc<NB>(acc);
    // dA_{L-1} = dHead . Head^T    (B^T = head [H][32])
    tile_gemm<T, NB>(acc, act, ldh, rb, (const T*)P.head, MLEARN_HEAD_COLS, MLEARN_HEAD_COLS, w,
                     lane);
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
        __syncthreads();
        const float* gamma = P.lns[l];
        const float* beta = P.lnb[l];
        float su[16], sv[16], pg[NB], pb[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) pg[i] = pb[i] = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = rb * 32 + acc_row(e, lane);
            const bool live = row0 + row < M;
            const float mean = stat[(l * kTileRows + row) * 2];
            const float rstd = stat[(l * kTileRows + row) * 2 + 1];
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int col = ((w >> 1) + 2 * i) * 32 + r;
                const float zz = z[l].get(i, e);
                const float xh = (zz - mean) * rstd;
                const float y = (zz - mean) * (rstd * gamma[col]) + beta[col];
                const float dy = (live && rnd<T>(y) > 0.f) ? acc[i][e] : 0.f;  // ReLU'
                const float u = dy * gamma[col];
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
                const int col = ((w >> 1) + 2 * i) * 32 + r;
                float* lp = ws.colpart + (int64_t)blockIdx.x * ws.CP + ((l * 2 + rb) * 2) * H;
                lp[col] = pb[i];
                lp[H + col] = pg[i];
            }
        }
        row_reduce2(su, sv, red, w, lane);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = rb * 32 + acc_row(e, lane);
            const float mean = stat[(l * kTileRows + row) * 2];
            const float rstd = stat[(l * kTileRows + row) * 2 + 1];
            const float mu = su[e] * invH, mv = sv[e] * invH;
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int col = ((w >> 1) + 2 * i) * 32 + r;
                const float xh = (z[l].get(i, e) - mean) * rstd;
                const float dz = rnd<T>(rstd * (acc[i][e] - mu - xh * mv));
                act[row * ld + col] = cvt<T>(dz);
                acc[i][e] = dz;
            }
        }
        store_transposed<T, NB>(acc, (T*)ws.dzT[l], ws.Mp, w, lane, row0, M);
        if (l > 0) {
            __syncthreads();
            zero_acc<NB>(acc);
            // dA_{l-1} = dZ_l . W_l^T   (B^T = W_l [in][H])
            tile_gemm<T, NB>(acc, act, ld, rb, (const T*)P.w[l], H, H, w, lane);
        }
    }
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
        g = colsum(L * 4 * H + (int)(p - Lk.hb_off));
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
            g = colsum(((l * 2 + 0) * 2 + which) * H + col) + colsum(((l * 2 + 1) * 2 + which) * H + col);
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

static size_t step_lds(int D, int H, int L, int es) {
    int ld = (D > H ? D : H) + 16 / es;
    return (size_t)kTileRows * ld * es + 4 * 64 * 2 * 4 + 2 * kTileRows * 33 * 4 +
           (size_t)L * kTileRows * 2 * 4 + kTileRows * 8 + 4 * kLossSlots * 8;
}

template <typename T, int H, int L>
static void launch_step(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                        int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                        hipStream_t s) {
    auto k = ppo_step_kernel<T, H, L>;
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    size_t lds = step_lds(P.D, H, L, sizeof(T));
    hipLaunchKernelGGL(k, dim3(ws.ntiles), dim3(256), lds, s, P, R, mb_seq, mb, M, adv_st, hp, ws);
}

template <typename T, int H>
static int launch_minibatch(const mlearn_mlp_policy& p, const mlearn_rollout_view& ro,
                            const int32_t* mb_seq, int mb, const float* adv_st,
                            const mlearn_ppo_hparams& h, float* grad, float* loss_out, void* wsp,
                            hipStream_t s) {
    const int64_t M = (int64_t)mb * ro.bptt_len;
    WsK ws;
    carve(p, M, (char*)wsp, &ws);
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
