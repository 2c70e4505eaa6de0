// PPO minibatch step up to the flat gradient (ppo.py:109-364):
//
//   ppo_step  one wave per 32 minibatch rows (row-on-lane orientation,
//             rowtile.h): gather the rows straight from the [T][N] rollout
//             store (no RolloutData.minibatch copy, rollouts.py:319-329), MLP
//             trunk + heads, PPO loss terms (ppo.py:129-262), d loss /
//             d {logits, value}, and back through heads, ReLU and LayerNorm
//             of every layer.  Dense outputs are kept in lane-private LDS,
//             everything else in registers; the wave writes the weight-
//             gradient operands X_l and dZ_l row-major plus LayerNorm
//             scale/bias and head-bias partials.
//   wgrad     dW_l = X_l^T dZ_l over all rows, every weight in one launch
//             (split-K slabs; MFMA operands transposed on the LDS read with
//             ds_read_b64_tr_b16).
//   reduce    fixed-order sum of slabs and tile partials into the flat f32
//             gradient + loss/metric outputs.  Deterministic: no atomics.
//
// Minibatch row f (time-major like mb['obs'] of shape [T/C, mb]):
//   tl = f / mb, m = f % mb, seq = mb_seq[m], c = seq / N, b = seq % N,
//   store row = (c * bptt + tl) * N + b.

#include "ppo_defs.h"
#include "r16_common.h"

namespace ml {

// ---------------------------------------------------------------------------
// Fused minibatch step: one workgroup per 32 rows; its W waves split the
// hidden features (wave w owns blocks w*NBW .. w*NBW+NBW-1 of every layer).
// Per layer the waves run their MFMAs over the full input (B fragments from
// LDS), combine LayerNorm row statistics through LDS, and exchange
// post-activation (forward) or dZ (backward) fragments through LDS.  Each
// wave keeps its own Dense outputs in registers for the backward pass.
// LDS: B fragments [KSH][64], LayerNorm scale/bias [L][2][H], head bias, row
// statistics [W][32][2], head partials [head_parts][32][HC+1], logits /
// d logits [32][HC+1], loss partials [W][kLossSlots], critic bins [HC].
// ---------------------------------------------------------------------------
#ifndef ML_STORE_LATE
// 1: every spill store of the step kernel is issued AFTER the weight loads of
// the product that follows it (vmcnt counts loads and stores in issue order,
// so a store batch issued first delays the product's first load wait)
#define ML_STORE_LATE 1
#endif
#ifndef ML_STEP_RING
#define ML_STEP_RING 8  // k-steps of weight fragments in flight in the step kernel's trunk products
#endif
#ifndef ML_STEP_MAXW
#define ML_STEP_MAXW 8  // waves per workgroup of the fused step kernel (feature split)
#endif
template <int H> struct StepCfg {
    static constexpr int NB = H / 32;
    static constexpr int W = NB < ML_STEP_MAXW ? NB : ML_STEP_MAXW;
    static constexpr int NBW = NB / W;
};

// Per row tile: B fragments [KSH][64], row statistics [W][32][2], head
// partials and outputs, loss partials; shared by the RTW row tiles of a
// workgroup: LayerNorm scale/bias [L][2][H], head bias [HC], critic bins [HC].
template <typename T, int H, int HC> constexpr size_t step_tile_lds() {
    typedef StepCfg<H> C;
    return (size_t)(H / RT<T>::KS) * 64 * sizeof(typename RT<T>::frag) +
           (size_t)(C::W * 64 + (head_parts<HC, C::W>() + 1) * 32 * (HC + 1) + C::W * kLossSlots) * 4;
}
template <typename T, int H, int L, int HC, int RTW = 1> static size_t step_lds() {
    return RTW * step_tile_lds<T, H, HC>() + (size_t)(L * 2 * H + 2 * HC) * 4;
}

// Phases of the step kernel.  kFused: the MLP policy's whole minibatch step.
// Recurrent policies (the LSTM scan runs in between, across time):
//   kTrunkFwd: trunk forward only (writes X_0 and the activations A_l; the
//              last one is the LSTM input);
//   kHeads:    heads + loss + d head from the LSTM outputs (rows of rec.hout,
//              natural k order), writes d loss / d LSTM output rows;
//   kTrunkBwd: trunk forward recomputed, then its backward from the rows of
//              d loss / d trunk output (rec.dfeat).
constexpr int kFused = 0, kTrunkFwd = 1, kHeads = 2, kTrunkBwd = 3;
struct RecK {
    const void* hout;        // [Mp][H] LSTM outputs (kHeads)
    void* dhout;             // [Mp][H] d loss / d LSTM outputs (kHeads)
    const void* dfeat;       // [Mp][H] d loss / d trunk output (kTrunkBwd)
    const void* head_t_nat;  // head image, natural k order (kHeads)
};

// Row-major stores of a wave's NBW 32-feature blocks of its row (bf16), 16
// bytes per lane: lane (r, h) holds features {4h..4h+3, 8+4h..8+4h+3} of
// each 16-feature half s (Pk words 4s .. 4s+3); one v_permlane32_swap per
// word pair trades half h = 0's second quad for half h = 1's first, after
// which lane (r, h) holds the natural features 16s + 8h .. 16s + 8h + 7: two
// 16-byte stores per block instead of four 8-byte row pieces (the A_l / dZ_l
// spill is the step kernel's largest store stream; a tile-native layout with
// 1 KB per store instruction made the step faster and the weight-gradient
// read slower: profiles/r04_spill_layout_ab.txt).  In place (the swap is an
// involution: RESTORE swaps back for a caller that reads the words again; no
// temporaries at the register peak).
template <int NBW, bool RESTORE>
__device__ inline void store_rows16(bf16* rowp, int w, uint32_t (&wd)[NBW][8], int h) {
    typedef __attribute__((ext_vector_type(4))) uint32_t u4;
    auto swap = [&](int i, int s) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const auto v = __builtin_amdgcn_permlane32_swap(wd[i][4 * s + k], wd[i][4 * s + 2 + k],
                                                            false, false);
            wd[i][4 * s + k] = v[0];
            wd[i][4 * s + 2 + k] = v[1];
        }
    };
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            swap(i, s);
            *(u4*)(rowp + (w * NBW + i) * 32 + 16 * s + 8 * h) =
                u4{wd[i][4 * s], wd[i][4 * s + 1], wd[i][4 * s + 2], wd[i][4 * s + 3]};
            if (RESTORE) swap(i, s);
        }
}
template <int NBW, bool RESTORE>
__device__ inline void store_rows16(float*, int, f2 (&)[NBW][8], int) {}

// RTW row tiles of 32 rows per workgroup (kFused): waves w and w + W * rt own
// the same features of different rows, released by the same barriers, so
// their weight-fragment loads of every product meet in the CU's L1.
template <typename T, int H, int L, int MODE = kFused, int HC = MLEARN_HEAD_COLS, int RTW = 1>
__global__ __launch_bounds__(64 * StepCfg<H>::W * RTW) __attribute__((amdgpu_waves_per_eu(ML_STEP_WAVES, 8))) void ppo_step_kernel(
    PolicyK P, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, int64_t M,
    const float* __restrict__ adv_st, HpK hp, WsK ws, RecK rec) {
    constexpr bool kFwd = MODE != kHeads;                     // runs the trunk forward
    constexpr bool kLoss = MODE == kFused || MODE == kHeads;  // heads + loss
    constexpr bool kBwd = MODE == kFused || MODE == kTrunkBwd;  // trunk backward
    typedef typename RT<T>::frag frag;
    typedef StepCfg<H> C;
    constexpr int NBW = C::NBW, W = C::W, THREADS = 64 * W;
    constexpr int E = RT<T>::E, KS = RT<T>::KS, SPB = RT<T>::SPB;
    constexpr int KSH = H / KS, KSHD = HC / KS, KSD = 256 / KS;
    constexpr int LGS = HC + 1;  // LDS row stride of the head outputs
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D, K = P.K;
    // wave-uniform (SGPR) indices for the buffer descriptors: row tile rt of
    // the workgroup, wave w of that tile
    const int wg_wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int rt = wg_wave / W, w = wg_wave - rt * W;
    const int tid = (int)threadIdx.x - rt * THREADS, lane = tid & 63, r = lane & 31, h = lane >> 5;
    char* tsm = smem + (size_t)rt * step_tile_lds<T, H, HC>();
    frag* fr = (frag*)tsm;                     // [KSH][64]
    float* red = (float*)(fr + KSH * 64);      // [W][32][2]
    float* lgp = red + W * 64;                 // [kHeadParts][32][LGS] head partials
    float* lg = lgp + head_parts<HC, W>() * 32 * LGS;  // [32][LGS]
    float* lred = lg + 32 * LGS;               // [W][kLossSlots]
    float* gb = (float*)(smem + (size_t)RTW * step_tile_lds<T, H, HC>());  // [L][2][H] (shared)
    float* hbias = gb + L * 2 * H;             // [HC]
    float* bins = hbias + HC;                  // [HC] two-hot critic bins
    if (kLoss && P.CB > 1)
        for (int i = tid; i < P.CB; i += THREADS) bins[i] = twohot_bin(i, P.CB);
    // LayerNorm / head-bias parameters: loads issued now, written to LDS after
    // the first product (their latency hides under the observation gather)
    constexpr int NPAR = (L * 2 * H + HC + THREADS - 1) / THREADS;
    float parv[NPAR];
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
    const int tile = (int)blockIdx.x * RTW + rt;
    const int64_t row0 = (int64_t)tile * 32;
    const int64_t row = row0 + r;
    const bool live = row < M;
    const int64_t sr = live ? store_row(ro, mb_seq, mb, row) : 0;
    // first loss task of this thread: row tr, task tg (group, or value if tg == K)
    const int tr = tid & 31, tg = tid >> 5;
    const bool tlive = kLoss && row0 + tr < M && tg <= K;
    const int64_t tsr = tlive ? store_row(ro, mb_seq, mb, row0 + tr) : 0;
    int t_act = 0;
    float t_lp = 0.f, t_adv = 0.f, t_ret = 0.f, t_val = 0.f;
    if (tlive) {
        t_adv = ro.adv[tsr];
        if (tg < K) {
            t_act = ro.actions[tsr * K + tg];
            t_lp = ro.logp[tsr * K + tg];
        } else {
            t_ret = ret_at(ro, tsr);
            if (ro.values) t_val = ro.values[tsr];
        }
    }

    STAMP(0);
    // ---- forward ----
    f32x16 acc[NBW];
    zero_acc<NBW>(acc);
    if constexpr (kFwd)
        gemm_first<T, NBW>(acc, (const T*)ro.obs + sr * D, live, D / KS,
                           (const T*)P.wt[0] + (int64_t)w * NBW * (D / KS) * 64 * E,
                           (w == 0 && MODE != kTrunkBwd) ? (T*)ws.x0 + row * D : nullptr, lane);
    STAMP(1);
#pragma unroll
    for (int k = 0; k < NPAR; ++k)
        if (tid + k * THREADS < L * 2 * H + HC) gb[tid + k * THREADS] = parv[k];
    // LayerNorm parameters staged: the first LayerNorm's statistics barrier
    // orders them before their first read (ln_apply)
    if constexpr (!kFwd) __syncthreads();
    typedef typename Pk<T>::word word;
    word zr[L][NBW][8];  // this wave's Dense outputs (exact in the compute dtype)
    word aw[NBW][8];     // post-activation of the current layer
    float mean_r[L], rstd_r[L];
    const float invH = 1.0f / (float)H;
    // post-activation rows A_l (weight-gradient operands), row-major
    // (keep: the caller reads aw again -- the bf16 store permutes it in place)
    auto store_act = [&](int l, auto keep) {
        if (MODE == kTrunkBwd) return;
        T* arow = (T*)ws.a[l] + row * H;
        if constexpr (std::is_same<T, bf16>::value) {
            store_rows16<NBW, decltype(keep)::value>(arow, w, aw, h);
            return;
        }
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                Pk<T>::store4(arow + (w * NBW + i) * 32 + 8 * g + 4 * h, aw[i][2 * g],
                              aw[i][2 * g + 1]);
    };
#pragma unroll
    for (int l = 0; l < (kFwd ? L : 0); ++l) {
        if (l > 0) {
            zero_acc<NBW>(acc);
            const T* img = (const T*)P.wt[l] + (int64_t)w * NBW * KSH * 64 * E;
#if ML_STORE_LATE
            frag ra[ML_STEP_RING][NBW];
            gemm_lds_issue<T, NBW, KSH, ML_STEP_RING>(ra, img, lane);
            store_act(l - 1, std::false_type{});  // A_{l-1}, behind this product's first weight loads
            gemm_lds_run<T, NBW, KSH, ML_STEP_RING>(acc, ra, fr, img, lane);
#else
            gemm_lds<T, NBW, KSH, ML_STEP_RING>(acc, fr, img, lane);
#endif
            STAMP(4);
        }
        f2 x2[NBW][8];
        float sum, sq;
        ln_pack_stats<T, NBW>(acc, zr[l], x2, sum, sq);
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
        mean_r[l] = mean;
        rstd_r[l] = rstd;
        STAMP(2 + 3 * l);
        ln_apply<T, NBW>(x2, mean, rstd, gb + l * 2 * H, H, w * NBW, h, aw);
        // the last layer's rows go out behind the head's weight loads (HC = 32)
        if (!ML_STORE_LATE || (l + 1 == L && (MODE != kFused || HC != 32))) store_act(l, std::true_type{});
        if (l + 1 < L) {
#pragma unroll
            for (int i = 0; i < NBW; ++i)
#pragma unroll
                for (int t = 0; t < SPB; ++t)
                    fr[((w * NBW + i) * SPB + t) * 64 + lane] = Pk<T>::frag(aw[i], t);
            __syncthreads();
        }
    }
    STAMP(6);
    if constexpr (MODE == kTrunkFwd) return;
    if constexpr (kLoss) {
    // heads (dists.py:22, models.py:154): lg[row][j] = rnd(rnd(a . W) + rnd(b)).
    // Head width 32: each wave multiplies its own features (B fragments from
    // its registers), partials summed in wave order.  Head width 96: the
    // backbone output of every wave is staged in LDS and wave w computes
    // column block w / KSPLIT over k-slice w % KSPLIT of the full K.
    {
        constexpr int HB = HC / 32;
        constexpr int KSPLIT = head_parts<HC, W>();
        constexpr int KPS = KSH / KSPLIT;  // k-steps per slice
        if constexpr (HB == 1) {
            frag hb[NBW * SPB];
            if constexpr (MODE == kHeads) {
                // this wave's slice of the LSTM output row (natural k order)
                const T* hrow = (const T*)rec.hout + row * H;
#pragma unroll
                for (int j = 0; j < NBW * SPB; ++j) hb[j] = RT<T>::row(hrow, w * NBW * SPB + j, h);
            } else {
#pragma unroll
                for (int i = 0; i < NBW; ++i)
#pragma unroll
                    for (int t = 0; t < SPB; ++t) hb[i * SPB + t] = Pk<T>::frag(aw[i], t);
            }
            const T* himg = (const T*)(MODE == kHeads ? rec.head_t_nat : P.head_t);
            f32x16 ha[1];
            zero_acc<1>(ha);
#if ML_STORE_LATE
            if constexpr (MODE == kFused) {
                // every head weight fragment of this wave in flight, then the
                // last layer's rows, then the product
                constexpr int HS = NBW * SPB;
                constexpr int FB = 64 * E * (int)sizeof(T);
                const __amdgpu_buffer_rsrc_t hrs = img_rsrc(himg + (int64_t)w * HS * 64 * E);
                frag hA[HS];
#pragma unroll
                for (int s2 = 0; s2 < HS; ++s2) hA[s2] = img_load<T>(hrs, lane * E * (int)sizeof(T), s2 * FB);
                store_act(L - 1, std::false_type{});
#pragma unroll
                for (int s2 = 0; s2 < HS; ++s2) ha[0] = MT<T>::mma(hA[s2], hb[s2], ha[0]);
            } else
#endif
            gemm_ring<T, 1, NBW * SPB, NBW * SPB < 8 ? NBW * SPB : 8>(
                ha, hb, NBW * SPB, himg + (int64_t)w * NBW * SPB * 64 * E, lane);
#pragma unroll
            for (int q = 0; q < 16; ++q) lgp[(w * 32 + r) * LGS + feat(0, q, h)] = ha[0][q];
        } else {
            if constexpr (MODE == kHeads) {
                // LSTM output rows (natural k order), k-steps split over the waves
                const T* hrow = (const T*)rec.hout + row * H;
                for (int s = w; s < KSH; s += W) fr[s * 64 + lane] = RT<T>::row(hrow, s, h);
            } else {
#pragma unroll
                for (int i = 0; i < NBW; ++i)
#pragma unroll
                    for (int t = 0; t < SPB; ++t)
                        fr[((w * NBW + i) * SPB + t) * 64 + lane] = Pk<T>::frag(aw[i], t);
            }
            __syncthreads();
            const T* himg = (const T*)(MODE == kHeads ? rec.head_t_nat : P.head_t);
            for (int u = w; u < HB * KSPLIT; u += W) {
                const int nb = u / KSPLIT, part = u % KSPLIT;
                f32x16 ha[1];
                zero_acc<1>(ha);
                gemm_lds<T, 1, KPS, 8>(ha, fr + part * KPS * 64,
                                       himg + ((int64_t)nb * KSH + part * KPS) * 64 * E, lane);
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

    STAMP(7);
    // ---- loss: one (row, group | value) task per thread (ppo.py:129-262) ----
    {
        LossAcc m;
        bool did = false;  // this lane ran a task (waves without any skip the reductions)
        const float as0 = adv_st[0], as1 = adv_st[1];
        const float* vn = hp.norm_vals ? adv_st + 2 : nullptr;
        // two-hot critic: the value rows run in groups of 8 lanes (below); with
        // 512 threads they take the last 256 while the first ones do the groups
        const bool th = P.CB > 1;
        const bool split = th && THREADS >= 512;
        const int tstride = split ? THREADS - 256 : THREADS;
        const int ntask = 32 * (th ? K : K + 1);
        for (int task = (split && tid >= THREADS - 256) ? ntask : tid; task < ntask;
             task += tstride) {
            const int rr = task & 31, g = task >> 5;
            did = true;
            float* lr = lg + rr * LGS;
            const int64_t f = row0 + rr;
            if (f >= M) {  // padding row: zero its d logits
                if (g < K)
                    for (int j = P.off[g]; j < P.off[g + 1]; ++j) lr[j] = 0.f;
                else
                    for (int j = P.A; j < HC; ++j) lr[j] = 0.f;
                continue;
            }
            int act;
            float olp, adv, ret, oval;
            if (task == tid) {
                act = t_act, olp = t_lp, adv = t_adv, ret = t_ret, oval = t_val;
            } else {
                const int64_t q = store_row(ro, mb_seq, mb, f);
                adv = ro.adv[q];
                act = g < K ? ro.actions[q * K + g] : 0;
                olp = g < K ? ro.logp[q * K + g] : 0.f;
                ret = g < K ? 0.f : ret_at(ro, q);
                oval = (g < K || !ro.values) ? 0.f : ro.values[q];
            }
            if (g < K) {
                if (hp.norm_adv) adv = (adv - as0) * as1;
                loss_group(hp, lr + P.off[g], P.off[g + 1] - P.off[g], act, olp, adv, hp.ecoef[g],
                           hp.objw[g], m);
            } else {
                loss_value(hp, lr, P.A, HC, ret, oval, m, vn);
            }
        }
        if (th) {
            constexpr int G = 8;
            const int vt0 = split ? tid - (THREADS - 256) : tid;
            const int vstride = split ? 256 : THREADS;
            for (int vt = vt0 < 0 ? 32 * G : vt0; vt < 32 * G; vt += vstride) {
                const int rr = vt / G, sub = vt % G;
                did = true;
                float* lr = lg + rr * LGS;
                const int64_t f = row0 + rr;
                if (f >= M) {  // padding row: zero its d critic logits
                    for (int j = P.A + sub; j < HC; j += G) lr[j] = 0.f;
                    continue;
                }
                const float R = ret_at(ro, store_row(ro, mb_seq, mb, f));
                loss_value_twohot_g<G>(hp, lr, P.A, P.CB, HC, bins, R, sub, m);
            }
        }
        const float vals[kLossSlots] = {m.sobj, m.qobj, m.mnobj, m.mxobj, m.svl, m.qvl, m.mnvl,
                                        m.mxvl, m.serr, m.qerr, m.mnerr, m.mxerr, m.sent, m.qent,
                                        m.mnent, m.mxent, m.sentw, m.sobjw, 0.f, 0.f};
        constexpr int kUsed = 18;  // slots 18.. are padding
        if (!hp.metrics) {
        } else if (__any(did)) {
#pragma unroll
            for (int s = 0; s < kUsed; ++s) {
                const int kind = (s < 16) ? (s & 3) : 0;
                float v = vals[s];
                v = kind == 2 ? wave_reduce<2>(v)
                              : (kind == 3 ? wave_reduce<3>(v) : wave_reduce<0>(v));
                if (lane == 0) lred[w * kLossSlots + s] = v;
            }
            if (lane >= kUsed && lane < kLossSlots) lred[w * kLossSlots + lane] = 0.f;
        } else if (lane < kLossSlots) {  // identities of sum / min / max
            const int kind = (lane < 16) ? (lane & 3) : 0;
            lred[w * kLossSlots + lane] = kind == 2 ? 3.4e38f : (kind == 3 ? -3.4e38f : 0.f);
        }
    }
    __syncthreads();
    if (hp.metrics && tid < kLossSlots) {
        const int kind = (tid < 16) ? (tid & 3) : 0;
        double v = lred[tid];
        for (int u = 1; u < W; ++u) {
            const double x = lred[u * kLossSlots + tid];
            v = kind == 2 ? fmin(v, x) : (kind == 3 ? fmax(v, x) : v + x);
        }
        ws.loss_part[(int64_t)tile * kLossSlots + tid] = v;
    }
    STAMP(8);
#if ML_STORE_LATE
    // the backward head product's weight fragments go out before the stores below
    constexpr int kHeadPre = KSHD * NBW <= 16 ? KSHD : 0;
#else
    constexpr int kHeadPre = 0;
#endif
    frag hbw[kHeadPre > 0 ? kHeadPre : 1][NBW];
#if ML_STORE_LATE
    const T* hbimg = (const T*)P.head + (int64_t)w * NBW * KSHD * 64 * E;
    if constexpr (kHeadPre > 0) {
        const __amdgpu_buffer_rsrc_t hrs = img_rsrc(hbimg);
#pragma unroll
        for (int s2 = 0; s2 < kHeadPre; ++s2)
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb)
                hbw[s2][nb] = img_load<T>(hrs, lane * E * (int)sizeof(T), (nb * KSHD + s2) * 64 * E * (int)sizeof(T));
    }
#endif
    // d head: row-major store (wgrad operand) and the head-bias column
    // partials (one 32-column block per wave)
    if (w == 0) {
        const float* lr = lg + r * LGS + (HC / 2) * h;
        T* drow = (T*)ws.dhead + row * HC + (HC / 2) * h;
#pragma unroll
        for (int j = 0; j < HC / 2; j += 4) store4(drow + j, lr[j], lr[j + 1], lr[j + 2], lr[j + 3]);
    }
    for (int cb = w; cb < HC / 32; cb += W) {
        float cs = 0.f;
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) cs += rnd<T>(lg[(16 * h + mm) * LGS + 32 * cb + r]);
        cs = sum_halves(cs);
        if (h == 0) ws.colpart[(int64_t)tile * ws.CP + L * 2 * H + 32 * cb + r] = cs;
    }

    STAMP(9);
    // ---- backward ----
    {
        frag db[KSHD];
#pragma unroll
        for (int s = 0; s < KSHD; ++s) db[s] = RT<T>::row_lds(lg + r * LGS, s, h);
        zero_acc<NBW>(acc);
        // dA_{L-1}^T = Head . dHead^T  (this wave's feature blocks)
        if constexpr (kHeadPre > 0) {
#pragma unroll
            for (int s2 = 0; s2 < kHeadPre; ++s2)
#pragma unroll
                for (int nb = 0; nb < NBW; ++nb) acc[nb] = MT<T>::mma(hbw[s2][nb], db[s2], acc[nb]);
        } else {
            gemm_ring<T, NBW, KSHD, 2>(acc, db, KSHD,
                                       (const T*)P.head + (int64_t)w * NBW * KSHD * 64 * E, lane);
        }
    }
    }  // kLoss
    if constexpr (MODE == kHeads) {
        // d loss / d LSTM output rows, rounded to the compute dtype (the
        // cotangent of a compute-dtype tensor)
        T* drow = (T*)rec.dhout + row * H;
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                Pk<T>::store4(drow + (w * NBW + i) * 32 + 8 * g + 4 * h,
                              Pk<T>::pack(acc[i][4 * g], acc[i][4 * g + 1]),
                              Pk<T>::pack(acc[i][4 * g + 2], acc[i][4 * g + 3]));
        return;
    }
    if constexpr (MODE == kTrunkBwd) {
        // d loss / d trunk output (from the LSTM's reverse scan) into the
        // accumulator layout of this wave's feature blocks
        const T* frow = (const T*)rec.dfeat + row * H;
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 v = live ? load4(frow + (w * NBW + i) * 32 + 8 * g + 4 * h)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
                acc[i][4 * g] = v.x;
                acc[i][4 * g + 1] = v.y;
                acc[i][4 * g + 2] = v.z;
                acc[i][4 * g + 3] = v.w;
            }
    }
    const int qs = col_sum16_index(lane);
    const float thr = relu_thr<T>();
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
        const float mean = mean_r[l], rstd = rstd_r[l];
        const f2 m2 = {mean, mean}, r2 = {rstd, rstd};
        const float* gm = gb + l * 2 * H;
        float* cp = ws.colpart + (int64_t)tile * ws.CP + l * 2 * H;
        f2 su2 = {0.f, 0.f}, sv2 = {0.f, 0.f};
        f2 zc2[NBW][8], u2[NBW][8];
        float cpb[NBW], cpg[NBW];  // this lane's LayerNorm bias / scale column partials
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
            const int nb = w * NBW + i;
            float pg[16], pb[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f0 = nb * 32 + 8 * g + 4 * h;
                const float4 G = *(const float4*)(gm + f0), B = *(const float4*)(gm + H + f0);
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    const int k = 2 * g + p;
                    const f2 gg = p ? f2{G.z, G.w} : f2{G.x, G.y};
                    const f2 bb = p ? f2{B.z, B.w} : f2{B.x, B.y};
                    const f2 zc = Pk<T>::unpack(zr[l][i][k]) - m2;
                    const f2 xh = zc * r2;
                    const f2 y = __builtin_elementwise_fma(zc, r2 * gg, bb);
                    // ReLU' (rnd<T>(y) > 0 <=> y > thr); padding rows carry no gradient
                    const f2 dy = {((y.x > thr) & live) ? acc[i][2 * k] : 0.f,
                                   ((y.y > thr) & live) ? acc[i][2 * k + 1] : 0.f};
                    const f2 u = dy * gg;
                    const f2 pgk = dy * xh;
                    zc2[i][k] = zc;
                    u2[i][k] = u;
                    su2 += u;
                    sv2 = u * xh + sv2;
                    pg[2 * k] = pgk.x;
                    pg[2 * k + 1] = pgk.y;
                    pb[2 * k] = dy.x;
                    pb[2 * k + 1] = dy.y;
                }
            }
            // LayerNorm scale/bias partials: column sums over the tile's rows
            cpg[i] = col_sum16(pg, lane);
            cpb[i] = col_sum16(pb, lane);
        }
        auto store_cp = [&]() {
            if ((lane & 16) == 0)
#pragma unroll
                for (int i = 0; i < NBW; ++i) {
                    const int f = feat(w * NBW + i, qs, h);
                    cp[f] = cpb[i];
                    cp[H + f] = cpg[i];
                }
        };
        if (!ML_STORE_LATE) store_cp();
        STAMP(10 + 3 * (L - 1 - l));
        float su = sum_halves(su2.x + su2.y);
        float sv = sum_halves(sv2.x + sv2.y);
        if (h == 0) {
            red[(w * 32 + r) * 2] = su;
            red[(w * 32 + r) * 2 + 1] = sv;
        }
        __syncthreads();
        su = red[r * 2];
        sv = red[r * 2 + 1];
#pragma unroll
        for (int v = 1; v < W; ++v) {
            su += red[(v * 32 + r) * 2];
            sv += red[(v * 32 + r) * 2 + 1];
        }
        // dZ = rstd (u - mean(u) - xh mean(u xh)) = rstd u + (-rstd^2 mean(u xh)) zc - rstd mean(u)
        const float ca = -(rstd * rstd) * (sv * invH), cb = -rstd * (su * invH);
        const f2 ca2 = {ca, ca}, cb2 = {cb, cb};
        word dzw[NBW][8];
        T* dzrow = (T*)ws.dz[l] + row * H;
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f2 d = r2 * u2[i][k] + (ca2 * zc2[i][k] + cb2);
                dzw[i][k] = Pk<T>::pack(d.x, d.y);
            }
        auto store_dz = [&]() {
            if constexpr (std::is_same<T, bf16>::value) {
                store_rows16<NBW, false>(dzrow, w, dzw, h);
                return;
            }
#pragma unroll
            for (int i = 0; i < NBW; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    Pk<T>::store4(dzrow + (w * NBW + i) * 32 + 8 * g + 4 * h, dzw[i][2 * g],
                                  dzw[i][2 * g + 1]);
        };
        if (!ML_STORE_LATE || l == 0) {
            if (ML_STORE_LATE) store_cp();
            store_dz();
        }
        STAMP(11 + 3 * (L - 1 - l));
        if (l > 0) {
#pragma unroll
            for (int i = 0; i < NBW; ++i)
#pragma unroll
                for (int t = 0; t < SPB; ++t)
                    fr[((w * NBW + i) * SPB + t) * 64 + lane] = Pk<T>::frag(dzw[i], t);
            const T* img = (const T*)P.w[l] + (int64_t)w * NBW * KSH * 64 * E;
#if ML_STORE_LATE
            // dA_{l-1}^T = W_l . dZ_l^T (this wave's feature blocks): weight loads
            // first, then this layer's column partials and dZ rows
            frag ra[ML_STEP_RING][NBW];
            gemm_lds_issue<T, NBW, KSH, ML_STEP_RING>(ra, img, lane);
            store_cp();
            store_dz();
            __syncthreads();
            zero_acc<NBW>(acc);
            gemm_lds_run<T, NBW, KSH, ML_STEP_RING>(acc, ra, fr, img, lane);
#else
            __syncthreads();
            zero_acc<NBW>(acc);
            // dA_{l-1}^T = W_l . dZ_l^T  (this wave's feature blocks)
            gemm_lds<T, NBW, KSH, ML_STEP_RING>(acc, fr, img, lane);
#endif
            STAMP(12 + 3 * (L - 1 - l));
        }
    }
    STAMP(15);
}

#include "ppo_rows16.h"

#ifndef ML_STEP_RTW
#define ML_STEP_RTW 1  // row tiles per workgroup of the fused MLP step (kFused; 2 measured slower)
#endif
template <typename T, int H, int L, int MODE, int HC>
static void launch_step_hc(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                           int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                           hipStream_t s, const RecK& rec) {
    // ntiles = Mp / 32 is even (Mp is a multiple of 64)
    constexpr int RTW = (MODE == kFused && StepCfg<H>::W * ML_STEP_RTW <= 16) ? ML_STEP_RTW : 1;
    auto k = ppo_step_kernel<T, H, L, MODE, HC, RTW>;
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    const size_t lds = step_lds<T, H, L, HC, RTW>();
    const int threads = 64 * StepCfg<H>::W * RTW;
    hipLaunchKernelGGL(k, dim3(ws.ntiles / RTW), dim3(threads), lds, s, P, R, mb_seq, mb, M,
                       adv_st, hp, ws, rec);
}
template <typename T, int H, int L, int MODE = kFused>
static void launch_step(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                        int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                        hipStream_t s, const RecK& rec = RecK{}) {
    if (P.HC == MLEARN_HEAD_COLS)
        launch_step_hc<T, H, L, MODE, MLEARN_HEAD_COLS>(P, R, mb_seq, mb, M, adv_st, hp, ws, s, rec);
    else
        launch_step_hc<T, H, L, MODE, MLEARN_HEAD_COLS_MAX>(P, R, mb_seq, mb, M, adv_st, hp, ws, s,
                                                            rec);
}

// ---------------------------------------------------------------------------
// Weight gradients dW[i][j] = sum_m X[m][i] * Y[m][j] for every weight of the
// policy in one launch (X, Y row-major [Mp][I] / [Mp][J], written by the step
// kernel).  Workgroup tile 128 (i) x 128 (j): 4 waves in 2x2, each 64x64 =
// 2x2 MFMA blocks.  K = minibatch rows in chunks of 32, double-buffered
// through LDS; the MFMA wants both operands k-contiguous, i.e. COLUMNS of the
// row-major tiles: bf16 fragments come from ds_read_b64_tr_b16 (4 rows x 16
// columns per 16-lane group, delivered column-major), f32 from plain reads.
// LDS rows are 160 elements (80 dwords = 16 mod 64): the 32 lanes of a half
// wave cover all 64 banks on the transposed reads.  Split-K over the rows;
// each split writes an f32 slab that reduce_grads sums in split order.
// ---------------------------------------------------------------------------
struct WgJob {
    const void* X;
    const void* Y;
    float* out;
    int64_t rps;
    int I, J, ti, tj, splits, wg0;
};
struct WgJobs {
    WgJob job[kMaxJobs];
    int n;
    int64_t Mp;
    int nwg, ncol, ncolx;  // weight-gradient blocks, column-sum blocks (ncolx per chunk)
};

template <typename T> struct WgCfg {
    static constexpr int LD = sizeof(T) == 2 ? 160 : 132;  // LDS row (elements)
    static constexpr size_t buf = (size_t)wg_chunk<T>() * LD * sizeof(T);  // one operand, one stage
    // register-staged form: 2 stages x 2 operands; LDS-DMA form (bf16): ML_WG_STAGES stages of
    // two 32-row x 256-B operand images
    static constexpr size_t glds = (size_t)ML_WG_STAGES * 2 * 32 * 256;
    static constexpr size_t lds =
        (sizeof(T) == 2 && ML_WG_GLDS && glds > 4 * buf) ? glds : 4 * buf;
};

typedef short short4v __attribute__((ext_vector_type(4)));

template <typename T> struct WgFrag;
template <> struct WgFrag<bf16> {
    typedef bf16x8 frag;
    // lane (r, h): tile[k = 16 ks + 8 h + e][c0 + r], e = 0..7
    __device__ static frag load(const bf16* tile, int ks, int c0, int lane) {
        const int g = lane >> 4, hh = g >> 1, cc = g & 1, q = (lane >> 2) & 3, p = lane & 3;
        const bf16* base = tile + (16 * ks + 8 * hh + q) * WgCfg<bf16>::LD + c0 + 16 * cc + 4 * p;
        typedef __attribute__((address_space(3))) short4v* lp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(base));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(base + 4 * WgCfg<bf16>::LD));
        typedef short short8v __attribute__((ext_vector_type(8)));
        short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(frag, v);
    }
};
template <> struct WgFrag<float> {
    typedef float frag;
    // lane (r, h): tile[k = 2 ks + h][c0 + r]
    __device__ static frag load(const float* tile, int ks, int c0, int lane) {
        return tile[(2 * ks + (lane >> 5)) * WgCfg<float>::LD + c0 + (lane & 31)];
    }
};

__device__ inline void colsum_block(const WsK& ws, int bx, int c);
__device__ inline void loss_block(const WsK& ws, const HpK& hp, int64_t M, int K, float* out);

// Weight-gradient tile (i0, j0) of job J over its split's rows.
template <typename T>
__device__ inline void wgrad_tile(const WgJobs& jobs, const WgJob& J, int local, char* smem) {
    constexpr int kWgChunk = wg_chunk<T>();
    constexpr int VPC = 16 / sizeof(T);                  // elements per 16-B chunk
    constexpr int CPR = kWgTile / VPC;                   // chunks per tile row
    constexpr int PER = kWgChunk * CPR / 256;            // chunks per thread per operand
    constexpr int LD = WgCfg<T>::LD, KSTEPS = kWgChunk / MT<T>::KS;
    typedef __attribute__((ext_vector_type(4))) uint32_t u4;
    T* lds = (T*)smem;  // [stage][operand][kWgChunk][LD]

    const int nt = J.ti * J.tj;
    int split, t;
    if ((J.splits & 7) == 0 && (J.wg0 & 7) == 0) {
        // XCD-aware: blocks are dealt round-robin over the 8 XCDs (b % 8), so
        // the nt tiles of one split (which read the same minibatch rows of X
        // and Y) get block ids 8 apart and share an XCD's L2: the rows come
        // from HBM once instead of once per tile (speed only, never correctness)
        const int x = local & 7, q = local >> 3;
        t = q % nt;
        split = (q / nt) * 8 + x;
    } else {
        split = local / nt;
        t = local - split * nt;
    }
    const int i0 = (t % J.ti) * kWgTile, j0 = (t / J.ti) * kWgTile;
    const int64_t m0 = split * J.rps;
    const int64_t m1 = m0 + J.rps < jobs.Mp ? m0 + J.rps : jobs.Mp;  // whole chunks
    const int nchunks = (int)((m1 - m0) / kWgChunk);
    const T* X = (const T*)J.X;
    const T* Y = (const T*)J.Y;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int iw = (w & 1) * 64, jw = (w >> 1) * 64;
    const bool wi_on = i0 + iw < J.I, wj_on = j0 + jw < J.J;

    // NS register sets of staged rows: chunks c + 1 .. c + NS are in flight
    // while chunk c is multiplied out of LDS (two LDS stages); the chunk loop
    // is unrolled by lcm(NS, 2) so that every set / stage index is static
    constexpr int NS = ML_WG_SETS;
    constexpr int U = NS % 2 ? 2 * NS : NS;
    u4 rx[NS][PER], ry[NS][PER];
    auto gload = [&](int c, int set) {
        const int64_t mb0 = m0 + (int64_t)c * kWgChunk;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = tid + 256 * u;
            const int rr = idx / CPR, cc = (idx - rr * CPR) * VPC;
            const u4 zero = {0u, 0u, 0u, 0u};
            rx[set][u] = i0 + cc < J.I ? *(const u4*)(X + (mb0 + rr) * J.I + i0 + cc) : zero;
            ry[set][u] = j0 + cc < J.J ? *(const u4*)(Y + (mb0 + rr) * J.J + j0 + cc) : zero;
        }
    };
    auto sstore = [&](int stage, int set) {
        T* xs = lds + (size_t)stage * 2 * kWgChunk * LD;
        T* ys = xs + kWgChunk * LD;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = tid + 256 * u;
            const int rr = idx / CPR, cc = (idx - rr * CPR) * VPC;
            *(u4*)(xs + rr * LD + cc) = rx[set][u];
            *(u4*)(ys + rr * LD + cc) = ry[set][u];
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) zero_acc<2>(acc[a]);
    auto compute = [&](int stage) {
        if (!(wi_on && wj_on)) return;
        const T* xs = lds + (size_t)stage * 2 * kWgChunk * LD;
        const T* ys = xs + kWgChunk * LD;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
            typename WgFrag<T>::frag fa[2], fb[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                fa[a] = WgFrag<T>::load(xs, ks, iw + 32 * a, lane);
                fb[a] = WgFrag<T>::load(ys, ks, jw + 32 * a, lane);
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = MT<T>::mma(fa[a], fb[b], acc[a][b]);
        }
    };
#pragma unroll
    for (int k = 0; k < NS; ++k)
        if (k < nchunks) gload(k, k);
    sstore(0, 0);
    if (NS < nchunks) gload(NS, 0);
    __syncthreads();
    for (int c = 0; c < nchunks; c += U) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            // chunk c + k: LDS stage k % 2; chunk c + k + 1 waits in set (k + 1) % NS
            if (c + k >= nchunks) break;
            compute(k % 2);
            if (c + k + 1 < nchunks) {
                sstore((k + 1) % 2, (k + 1) % NS);
                if (c + k + 1 + NS < nchunks) gload(c + k + 1 + NS, (k + 1) % NS);
            }
            __syncthreads();
        }
    }
    if (!wi_on || !wj_on) return;
    float* out = J.out + (int64_t)split * J.I * J.J;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int i = i0 + iw + 32 * a + acc_row(e, lane);
                const int j = j0 + jw + 32 * b + (lane & 31);
                // nontemporal: the slabs are read once, by the next launch
                // (reduce_grads), so they need not sit dirty in L2 at the
                // kernel boundary (headline 9.08 / 9.11 -> 8.97 / 9.00 ms per
                // update, profiles/r06_wgrad_variants_ab.txt)
                if (i < J.I && j < J.J)
                    __builtin_nontemporal_store(acc[a][b][e], out + (int64_t)i * J.J + j);
            }
}

// ---------------------------------------------------------------------------
// The bf16 weight-gradient tile with its operand chunks staged by LDS-DMA
// (global_load_lds_dwordx4: no staging registers, no LDS write pass), S
// stages deep: chunk c + S - 1 is issued right after the barrier that opens
// chunk c.  The launch is not bound by where its operands live (a second
// back-to-back launch on cache-hot operands: 28.9 vs 29.4 us) but by its
// chunk loop; 2 stages measured best (27.6 vs 29.0 us register-staged; 3 / 4
// stages 29.8 / 31.6 us: more bytes in flight only congest,
// profiles/r06_spill_probes.txt).  Same MFMA fragments in the same order as
// wgrad_tile<bf16>, so the slabs are bit-identical.
//
// LDS image of one operand chunk: 32 rows of P bytes (P = 256 for a 128-
// column tile, 128 for a tile of <= 64 columns), no padding; one DMA
// instruction writes 1 KB lane-linearly (lane l -> bytes 16 l), so the XOR
// swizzle that keeps the transposed fragment reads conflict-free is applied
// to each lane's SOURCE address: 16-byte unit u of row r sits at unit
// u ^ swz(r), swz = 4 (r & 3) at P = 256, 4 ((r >> 1) & 1) at P = 128 (the
// four rows of a half-wave's ds_read_b64_tr_b16 land on four 64-byte bank
// groups).  Columns past the operand's width load unit 0 of the tile again:
// they meet only output rows / columns that are never stored.
// ---------------------------------------------------------------------------
template <int P> __device__ inline int wg_swz(int row) {
    return P == 256 ? 4 * (row & 3) : 4 * ((row >> 1) & 1);
}

// one 16-byte-per-lane LDS-DMA piece: LDS bytes [lds_dst + 16 lane, +16) <- gsrc
// (M0 written and restored in the same statement; hipcc does not count these
// loads, the caller's s_waitcnt vmcnt does)
__device__ inline void wg_glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
}
template <int N> __device__ inline void wg_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int PX, int PY, int CH>
__device__ inline void wgrad_tile_glds(const WgJobs& jobs, const WgJob& J, int local, char* smem) {
    constexpr int S = ML_WG_STAGES;
    static_assert(S >= 2, "at least two stages");
    constexpr int XB = CH * PX, YB = CH * PY, SB = XB + YB;  // bytes per operand / stage
    constexpr int NXW = XB / 1024 / 4, NYW = YB / 1024 / 4;  // DMA pieces per wave
    constexpr int G = NXW + NYW;
    const int nt = J.ti * J.tj;
    int split, t;
    if ((J.splits & 7) == 0 && (J.wg0 & 7) == 0) {  // XCD-aware, as wgrad_tile
        const int x = local & 7, q = local >> 3;
        t = q % nt;
        split = (q / nt) * 8 + x;
    } else {
        split = local / nt;
        t = local - split * nt;
    }
    const int i0 = (t % J.ti) * kWgTile, j0 = (t / J.ti) * kWgTile;
    const int64_t m0 = split * J.rps;
    const int64_t m1 = m0 + J.rps < jobs.Mp ? m0 + J.rps : jobs.Mp;
    const int nchunks = (int)((m1 - m0) / CH);
    const bf16* X = (const bf16*)J.X;
    const bf16* Y = (const bf16*)J.Y;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int iw = (w & 1) * 64, jw = (w >> 1) * 64;
    const bool wi_on = i0 + iw < J.I, wj_on = j0 + jw < J.J;

    // per-lane source offsets (elements, relative to the chunk's first row)
    int ox[NXW], oy[NYW];
#pragma unroll
    for (int k = 0; k < NXW; ++k) {
        const int b = (w * NXW + k) * 1024 + lane * 16, r = b / PX;
        const int u = ((b % PX) >> 4) ^ wg_swz<PX>(r);
        const int col = i0 + 8 * u < J.I ? i0 + 8 * u : i0;
        ox[k] = r * J.I + col;
    }
#pragma unroll
    for (int k = 0; k < NYW; ++k) {
        const int b = (w * NYW + k) * 1024 + lane * 16, r = b / PY;
        const int u = ((b % PY) >> 4) ^ wg_swz<PY>(r);
        const int col = j0 + 8 * u < J.J ? j0 + 8 * u : j0;
        oy[k] = r * J.J + col;
    }
    const uint32_t lbase =
        (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)smem;
    auto issue = [&](int c, int st) {
        const bf16* xb = X + (m0 + CH * (int64_t)c) * J.I;
        const bf16* yb = Y + (m0 + CH * (int64_t)c) * J.J;
        const uint32_t sb = lbase + (uint32_t)(st * SB);
#pragma unroll
        for (int k = 0; k < NXW; ++k)
            wg_glds16(xb + ox[k], __builtin_amdgcn_readfirstlane(sb + (uint32_t)((w * NXW + k) * 1024)));
#pragma unroll
        for (int k = 0; k < NYW; ++k)
            wg_glds16(yb + oy[k],
                      __builtin_amdgcn_readfirstlane(sb + (uint32_t)(XB + (w * NYW + k) * 1024)));
    };

    // fragment reads: lane (g = lane >> 4: hh = g >> 1, cc = g & 1; q, p) reads rows
    // 16 ks + 8 hh + q (+ 4) at columns c0 + 16 cc + 4 p .. + 3 (wgrad_tile's WgFrag)
    const int g = lane >> 4, hh = g >> 1, cc = g & 1, q = (lane >> 2) & 3, p = lane & 3;
    auto fofs = [&](int c0, int P, int swz) {
        const int u = (c0 >> 3) + 2 * cc + (p >> 1);
        return (8 * hh + q) * P + ((u ^ swz) << 4) + (p & 1) * 8;
    };
    int fx[2], fy[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        fx[a] = fofs(iw + 32 * a, PX, wg_swz<PX>(q));
        fy[a] = fofs(jw + 32 * a, PY, wg_swz<PY>(q));
    }
    typedef __attribute__((address_space(3))) short4v* lp;
    typedef short short8v __attribute__((ext_vector_type(8)));
    auto frag = [&](const char* base, int ofs, int ks, int P) {
        const char* a = base + ks * 16 * P + ofs;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(a));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(a + 4 * P));
        short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) zero_acc<2>(acc[a]);
    const bool on = wi_on && wj_on;

#pragma unroll
    for (int k = 0; k < S - 1; ++k)
        if (k < nchunks) issue(k, k);
    int st = 0;  // stage of chunk c
    for (int c = 0; c < nchunks; ++c) {
        // chunk c's pieces (this wave's) have landed: S - 2 younger chunks may
        // stay in flight (fewer near the end)
        if (c + S - 2 < nchunks) wg_vmcnt<G * (S - 2)>();
        else wg_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's pieces in; stage (c - 1) % S read out
        __builtin_amdgcn_sched_barrier(0);
        if (c + S - 1 < nchunks) issue(c + S - 1, st == 0 ? S - 1 : st - 1);
        if (on) {
            const char* xs = smem + st * SB;
            const char* ys = xs + XB;
#pragma unroll
            for (int ks = 0; ks < CH / 16; ++ks) {
                bf16x8 fa[2], fb[2];
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    fa[a] = frag(xs, fx[a], ks, PX);
                    fb[a] = frag(ys, fy[a], ks, PY);
                }
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b) acc[a][b] = MT<bf16>::mma(fa[a], fb[b], acc[a][b]);
            }
        }
        st = st + 1 == S ? 0 : st + 1;
    }
    if (!on) return;
    float* out = J.out + (int64_t)split * J.I * J.J;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int i = i0 + iw + 32 * a + acc_row(e, lane);
                const int j = j0 + jw + 32 * b + (lane & 31);
                if (i < J.I && j < J.J) {
#if ML_WG_SLAB_NT
                    __builtin_nontemporal_store(acc[a][b][e], out + (int64_t)i * J.J + j);
#else
                    out[(int64_t)i * J.J + j] = acc[a][b][e];
#endif
                }
            }
}

// Blocks [0, nwg) compute weight gradients; the next ncol blocks the first
// level of the column partials; one more (if loss_out) the loss metrics.
// (The fixed-order reduction into the flat gradient is the next launch,
// reduce_grads_kernel: folding it in as trailing blocks that wait on a
// device-scope counter measured 2.4x slower, profiles/r04_fused_reduce_ab.txt.)
template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ML_WG_WAVES, 8))) void wgrad_kernel(
    WgJobs jobs, WsK ws, HpK hp, int64_t M, int K, float* loss_out) {
    if ((int)blockIdx.x >= jobs.nwg) {
        const int b = blockIdx.x - jobs.nwg;
        if (b < jobs.ncol) colsum_block(ws, b % jobs.ncolx, b / jobs.ncolx);
        else loss_block(ws, hp, M, K, loss_out);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int jb = 0;
    while (jb + 1 < jobs.n && (int)blockIdx.x >= jobs.job[jb + 1].wg0) ++jb;
    const WgJob& J = jobs.job[jb];
#if ML_WG_GLDS
    if constexpr (sizeof(T) == 2) {
        static_assert(kWgTile == 128, "LDS-DMA tile shape");
        if (hp.wg_form != 1) {  // mlearn_ppo_hparams.wgrad_form: 0 / 2 = LDS-DMA
            // operand image rows of 128 B (<= 64 columns) or 256 B
            const int local = blockIdx.x - J.wg0;
            if (J.I <= 64) {
                if (J.J <= 64) wgrad_tile_glds<128, 128, 32>(jobs, J, local, smem);
                else wgrad_tile_glds<128, 256, 32>(jobs, J, local, smem);
            } else {
                if (J.J <= 64) wgrad_tile_glds<256, 128, 32>(jobs, J, local, smem);
                else wgrad_tile_glds<256, 256, 32>(jobs, J, local, smem);
            }
            return;
        }
    }
#endif
    wgrad_tile<T>(jobs, J, blockIdx.x - J.wg0, smem);
}


// First level of the per-tile column partials (LayerNorm scale/bias grads,
// head-bias grad): colpart2[c][col] = sum over tiles t = c, c + kColChunks, ...
// (8 independent accumulators, combined in fixed order).  Runs as extra
// blocks of the weight-gradient launch.
__device__ inline void colsum_block(const WsK& ws, int bx, int c) {
    const int col = bx * 256 + threadIdx.x;
    if (col >= ws.CP) return;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int t = c;
    for (; t + 7 * kColChunks < ws.ncp; t += 8 * kColChunks)
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += ws.colpart[(int64_t)(t + u * kColChunks) * ws.CP + col];
    for (int u = 0; t < ws.ncp; t += kColChunks, ++u) acc[u] += ws.colpart[(int64_t)t * ws.CP + col];
    ws.colpart2[(int64_t)c * ws.CP + col] =
        ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// ---------------------------------------------------------------------------
// Fixed-order reduction into the flat gradient.
// ---------------------------------------------------------------------------
LayoutK make_layout(const mlearn_mlp_policy& p) {
    LayoutK k{};
    k.L = p.num_layers;
    k.D = p.obs_dim;
    k.H = p.hidden;
    k.A1 = p.actions.num_logits + p.critic_bins;
    k.HC = head_cols(p);
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
    k.mlp_total = o;
    k.lstm_off = o;
    k.lstm_H = 0;
    return k;
}

LayoutK make_layout_lstm(const mlearn_mlp_policy& p, const mlearn_lstm& r) {
    LayoutK k = make_layout(p);
    const int64_t H = r.hidden;
    k.lstm_H = (int)H;
    k.lstm_off = (k.mlp_total + 63) / 64 * 64;
    k.total = k.lstm_off + 8 * H * H + 4 * H;
    return k;
}

int validate_lstm(const mlearn_mlp_policy* p, const mlearn_lstm* r) {
    int rc = validate_policy(p);
    if (rc) return rc;
    ML_REQUIRE(r, "lstm: null descriptor");
    ML_REQUIRE(r->num_layers == 1, "lstm: one LSTM layer supported (got %d)", r->num_layers);
    ML_REQUIRE(r->hidden == p->hidden, "lstm: width %d must equal the MLP width %d", r->hidden,
               p->hidden);
    ML_REQUIRE(r->wi_perm && r->wi_nat && r->wh_nat && r->w_bwd && r->head_t_nat && r->bias,
               "lstm: null weight image");
    return MLEARN_OK;
}

// Fixed-order reduction of the split-K slabs and column partials into the
// flat gradient.  A block owns 64 consecutive parameters (every segment of
// the flat layout but the head bias is a multiple of 64 long): 16 column
// threads x 16 split groups; group g sums splits g, g + 16, ... and the
// groups are combined in order through LDS.
constexpr int kRgGroups = 16;
// v += ld(k) for k = g, g + 16, ... < n, in that order, with four loads in
// flight (a plain loop waits for each load before issuing the next)
template <typename F>
__device__ inline void rg_sum4(float (&v)[4], int g, int n, F ld) {
    for (int k0 = g; k0 < n; k0 += 4 * kRgGroups) {
        float4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k0 + u * kRgGroups < n) x[u] = ld(k0 + u * kRgGroups);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k0 + u * kRgGroups < n) {
                v[0] += x[u].x;
                v[1] += x[u].y;
                v[2] += x[u].z;
                v[3] += x[u].w;
            }
    }
}
__global__ __launch_bounds__(256) void reduce_grads_kernel(LayoutK Lk, WsK ws, float* grad,
                                                           double* sumsq) {
    __shared__ float red[kRgGroups][65];
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int64_t p0 = (int64_t)blockIdx.x * 64;
    const int H = Lk.H, L = Lk.L;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (Lk.lstm_H && p0 >= Lk.lstm_off) {  // LSTM segment (64-aligned)
        const int64_t q0 = p0 - Lk.lstm_off, HH = Lk.lstm_H, G = 4 * HH * HH;
        if (q0 >= 2 * G) {  // bias: column partials of d gate pre-activations
            const int col = L * 2 * H + Lk.HC + (int)(q0 - 2 * G) + 4 * c;
            rg_sum4(v, g, kColChunks,
                    [&](int k) { return *(const float4*)(ws.colpart2 + (int64_t)k * ws.CP + col); });
        } else {  // Wi / Wh: split-K slabs [split][H][4H]
            const int which = (int)(q0 / G);
            const float* sp = ws.slab + ws.slab_off[L + 1 + which] + (q0 - which * G) + 4 * c;
            rg_sum4(v, g, ws.splits[L + 1 + which],
                    [&](int k) { return *(const float4*)(sp + (int64_t)k * G); });
        }
    } else if (p0 >= Lk.hw_off) {  // head weight (slab [split][H][32]) and head bias
        // per parameter e: a strided sequence (base, stride, n) summed in
        // order; the four parameters' loads are issued together
        const float* base[4];
        int64_t stride[4];
        int n[4];
        int nmax = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t p = p0 + 4 * c + e;
            base[e] = ws.colpart2;
            stride[e] = 0;
            n[e] = 0;
            if (p >= Lk.mlp_total) continue;  // (recurrent policies: alignment padding)
            if (p >= Lk.hb_off) {
                base[e] = ws.colpart2 + L * 2 * H + (int)(p - Lk.hb_off);
                stride[e] = ws.CP;
                n[e] = kColChunks;
            } else {
                const int64_t q = p - Lk.hw_off;
                const int i = (int)(q / Lk.A1), j = (int)(q % Lk.A1);
                base[e] = ws.slab + ws.slab_off[L] + (int64_t)i * Lk.HC + j;
                stride[e] = (int64_t)H * Lk.HC;
                n[e] = ws.splits[L];
            }
            nmax = n[e] > nmax ? n[e] : nmax;
        }
        for (int k0 = g; k0 < nmax; k0 += 4 * kRgGroups) {
            float x[4][4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + u * kRgGroups;
                    x[e][u] = k < n[e] ? base[e][k * stride[e]] : 0.f;
                }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k0 + u * kRgGroups < n[e]) v[e] += x[e][u];
        }
    } else {
        int l = L - 1;
        while (l > 0 && p0 < Lk.w_off[l]) --l;
        if (p0 >= Lk.s_off[l]) {  // LayerNorm scale / bias: column partials
            const int which = p0 >= Lk.b_off[l] ? 0 : 1;  // 0: bias (beta), 1: scale (gamma)
            const int col = (l * 2 + which) * H + (int)(p0 - (which ? Lk.s_off[l] : Lk.b_off[l])) + 4 * c;
            rg_sum4(v, g, kColChunks,
                    [&](int k) { return *(const float4*)(ws.colpart2 + (int64_t)k * ws.CP + col); });
        } else {  // Dense kernel: split-K slabs
            const int I = l == 0 ? Lk.D : H;
            const float* sp = ws.slab + ws.slab_off[l] + (p0 - Lk.w_off[l]) + 4 * c;
            const int64_t stride = (int64_t)I * H;
            rg_sum4(v, g, ws.splits[l], [&](int k) { return *(const float4*)(sp + k * stride); });
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) red[g][4 * c + e] = v[e];
    __syncthreads();
    if (threadIdx.x < 64) {  // wave 0
        const int64_t p = p0 + threadIdx.x;
        float t = red[0][threadIdx.x];
#pragma unroll
        for (int k = 1; k < kRgGroups; ++k) t += red[k][threadIdx.x];
        if (p < Lk.total) grad[p] = t;
        if (sumsq) {  // this block's partial of the clip_by_global_norm sum (ppo.py:84-90)
            const double q = p < Lk.total ? (double)t * (double)t : 0.0;
            const double w = wave_sum64d(q);
            if (threadIdx.x == 0) sumsq[blockIdx.x] = w;
        }
    }
}

// loss_out: five Metric vectors {mean, m2, min, max, count} in the order of
// PPO.add_metrics (ppo.py:95-106): 'Loss' (scalar: {loss, 0, loss, loss, 1}),
// 'Action Obj', 'Value Loss', 'Value Errors', 'Entropy'.
__device__ inline void loss_block(const WsK& ws, const HpK& hp, int64_t M, int K, float* out) {
    __shared__ double sh[4][kLossSlots];
    __shared__ double tot[kLossSlots];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double v[kLossSlots];
#pragma unroll
    for (int s = 0; s < kLossSlots; ++s) {
        const int kind = (s < 16) ? (s & 3) : 0;
        v[s] = kind == 2 ? 3.4e38 : (kind == 3 ? -3.4e38 : 0.0);
    }
    for (int t = tid; t < ws.nlp; t += 256) {
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
        for (int i = 1; i < 4; ++i) {
            double u = sh[i][tid];
            x = kind == 2 ? fmin(x, u) : (kind == 3 ? fmax(x, u) : x + u);
        }
        tot[tid] = x;
    }
    __syncthreads();
    if (tid == 0) {
        const double nk = (double)M * K, n = (double)M;
        const double vl_mean = tot[4] / n;
        // loss = -sum_key mean(obj_key) + c_v * mean(vl) - sum_key c_e[key] * mean(H_key)
        // (ppo.py:221-252); the per-sub-action weights K / K_key are in slots 16, 17
        const double loss = -tot[17] / nk + hp.vcoef * vl_mean - tot[16] / nk;
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

// The gradient launches: weight-gradient tiles, column partials and loss
// metrics; then the reduction into grad, one 64-parameter chunk per block.
template <typename T>
static void launch_wgrad(const WgJobs& jobs, const WsK& ws, const HpK& hp, int64_t M, int K,
                         float* loss_out, const LayoutK& Lk, float* grad, double* sumsq,
                         hipStream_t s) {
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)wgrad_kernel<T>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)WgCfg<T>::lds);
        attr_set = true;
    }
    const int blocks = jobs.nwg + jobs.ncol + (loss_out ? 1 : 0);
    hipLaunchKernelGGL((wgrad_kernel<T>), dim3(blocks), dim3(256), WgCfg<T>::lds, s, jobs, ws, hp, M,
                       K, loss_out);
#ifdef ML_PROBE_WG_TWICE  // (timing probe: the same launch again, operands now cache-hot)
    hipLaunchKernelGGL((wgrad_kernel<T>), dim3(blocks), dim3(256), WgCfg<T>::lds, s, jobs, ws, hp, M,
                       K, loss_out);
#endif
    hipLaunchKernelGGL(reduce_grads_kernel, dim3((unsigned)((Lk.total + 63) / 64)), dim3(256), 0, s,
                       Lk, ws, grad, sumsq);
}

template <typename T, int H>
static int launch_minibatch(const mlearn_mlp_policy& p, const mlearn_rollout_view& ro,
                            const int32_t* mb_seq, int mb, const float* adv_st,
                            const mlearn_ppo_hparams& h, float* grad, float* loss_out, void* wsp,
                            bool step_only, hipStream_t s) {
    const int64_t M = (int64_t)mb * ro.bptt_len;
    WsK ws;
    carve(p, M, (char*)wsp, &ws);
#ifdef ML_STAMPS
    ws.stamps = g_stamp_buf;
#endif
    PolicyK P = make_policy_k(p);
    RolloutK R{ro.obs, ro.actions, ro.log_probs, ro.advantages, ro.returns, ro.values, ro.dones,
               ro.T, ro.bptt_len, ro.N, ro.ld ? ro.ld : ro.N};
    HpK hp{};
    hp.clip = h.clip_coef;
    hp.vcoef = h.value_loss_coef;
    for (int i = 0; i < MLEARN_MAX_GROUPS; ++i) {
        hp.ecoef[i] = h.entropy_coef[i];
        hp.objw[i] = h.obj_weight[i] != 0.f ? h.obj_weight[i] : 1.f;
    }
    hp.norm_adv = h.normalize_advantages;
    hp.clip_vl = h.clip_value_loss;
    hp.norm_vals = h.normalize_values;
    hp.huber = h.huber_value_loss;
    hp.loss_scale = h.loss_scale;
    hp.metrics = loss_out != nullptr;
    ML_REQUIRE(h.wgrad_form >= 0 && h.wgrad_form <= 2, "ppo: wgrad_form %d", h.wgrad_form);
    hp.wg_form = h.wgrad_form;
    hp.inv_s = (float)(1.0 / (double)M);
    hp.inv_sk = (float)(1.0 / ((double)M * p.actions.num_groups));

    const bool rows16 = rows16_eligible(P, ws.Mp, head_cols(p), p.num_layers, H,
                                        std::is_same<T, bf16>::value);
    ML_REQUIRE(h.step_kernel >= 0 && h.step_kernel <= 2, "ppo: step_kernel %d", h.step_kernel);
    ML_REQUIRE(h.step_kernel != 2 || rows16,
               "ppo: step_kernel 2 (row-split) needs bf16, hidden 256, 2 layers, a scalar critic, "
               "head width 32, obs_dim 64, <= 7 action groups and (padded) rows of 32768 or a "
               "multiple of 256 from 65536");
    if (rows16 && h.step_kernel != 1) {
        ws.ncp = 2 * ws.ntiles;  // one column-partials row per 16-row tile
        if (rows16_cfg(ws.Mp).nt == 1) ws.nlp = 2 * ws.ntiles;  // one loss-partials row per wave
        launch_rows16(P, R, mb_seq, mb, M, adv_st, hp, ws, s);
    } else {
        switch (p.num_layers) {
            case 1: launch_step<T, H, 1>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
            case 2: launch_step<T, H, 2>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
            case 3: launch_step<T, H, 3>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
            default: launch_step<T, H, 4>(P, R, mb_seq, mb, M, adv_st, hp, ws, s); break;
        }
    }
    if (step_only) return check_launch("ppo_minibatch_fwd_bwd");
    const int L = p.num_layers;
    WgJobs jobs{};
    jobs.n = L + 1;
    jobs.Mp = ws.Mp;
    int wg = 0;
    for (int l = 0; l <= L; ++l) {
        WgJob& J = jobs.job[l];
        J.I = l == L ? H : (l == 0 ? p.obs_dim : H);
        J.J = l == L ? head_cols(p) : H;
        J.X = l == 0 ? ws.x0 : ws.a[l - 1];
        J.Y = l == L ? ws.dhead : ws.dz[l];
        J.out = ws.slab + ws.slab_off[l];
        J.rps = ws.rps[l];
        J.ti = (J.I + kWgTile - 1) / kWgTile;
        J.tj = (J.J + kWgTile - 1) / kWgTile;
        J.splits = ws.splits[l];
        J.wg0 = wg;
        wg += J.ti * J.tj * J.splits;
    }
    jobs.nwg = wg;
    jobs.ncolx = (ws.CP + 255) / 256;
    jobs.ncol = jobs.ncolx * kColChunks;
    launch_wgrad<T>(jobs, ws, hp, M, p.actions.num_groups, loss_out, make_layout(p), grad,
                    h.grad_sumsq_out, s);
    return check_launch("ppo_minibatch_grad");
}

// ---------------------------------------------------------------------------
// Recurrent update: the LSTM scan over the minibatch's sequences
// (LSTM.sequence, rnn.py:81-111) and its reverse (BPTT), one launch per
// time step and direction (lstm_scan.h).  Rows f = t * mb + m.
// ---------------------------------------------------------------------------
#include "lstm_scan.h"

template <typename T, int H>
static int launch_minibatch_lstm(const mlearn_mlp_policy& p, const mlearn_lstm& lstm,
                                 const mlearn_rollout_view& ro, const void* start_h,
                                 const void* start_c, const int32_t* mb_seq, int mb,
                                 const float* adv_st, const mlearn_ppo_hparams& h, float* grad,
                                 float* loss_out, void* wsp, hipStream_t s) {
    const int bptt = ro.bptt_len;
    const int64_t M = (int64_t)mb * bptt;
    WsK ws;
    LstmWsK lw;
    carve(p, M, (char*)wsp, &ws, &lstm, mb, &lw);
    PolicyK P = make_policy_k(p);
    LstmK RK = make_lstm_k(lstm);
    RolloutK R{ro.obs, ro.actions, ro.log_probs, ro.advantages, ro.returns, ro.values, ro.dones,
               ro.T, ro.bptt_len, ro.N, ro.ld ? ro.ld : ro.N};
    HpK hp{};
    hp.clip = h.clip_coef;
    hp.vcoef = h.value_loss_coef;
    for (int i = 0; i < MLEARN_MAX_GROUPS; ++i) {
        hp.ecoef[i] = h.entropy_coef[i];
        hp.objw[i] = h.obj_weight[i] != 0.f ? h.obj_weight[i] : 1.f;
    }
    hp.norm_adv = h.normalize_advantages;
    hp.clip_vl = h.clip_value_loss;
    hp.norm_vals = h.normalize_values;
    hp.huber = h.huber_value_loss;
    hp.loss_scale = h.loss_scale;
    hp.metrics = loss_out != nullptr;
    ML_REQUIRE(h.wgrad_form >= 0 && h.wgrad_form <= 2, "ppo: wgrad_form %d", h.wgrad_form);
    hp.wg_form = h.wgrad_form;
    hp.inv_s = (float)(1.0 / (double)M);
    hp.inv_sk = (float)(1.0 / ((double)M * p.actions.num_groups));
    const int L = p.num_layers;
    RecK rec{lw.hout, lw.dhout, lw.dfeat, lstm.head_t_nat};
    auto step = [&](auto mode) {
        constexpr int MODE = decltype(mode)::value;
        switch (L) {
            case 1: launch_step<T, H, 1, MODE>(P, R, mb_seq, mb, M, adv_st, hp, ws, s, rec); break;
            case 2: launch_step<T, H, 2, MODE>(P, R, mb_seq, mb, M, adv_st, hp, ws, s, rec); break;
            case 3: launch_step<T, H, 3, MODE>(P, R, mb_seq, mb, M, adv_st, hp, ws, s, rec); break;
            default: launch_step<T, H, 4, MODE>(P, R, mb_seq, mb, M, adv_st, hp, ws, s, rec); break;
        }
    };
    // trunk forward over every row (the LSTM input F = A_{L-1})
    step(std::integral_constant<int, kTrunkFwd>{});
    const T* feat = (const T*)ws.a[L - 1];
    // forward scan: one launch per step over (mb / 32) x (H / 32) four-wave
    // workgroups (the input product F_t Wi inside each step)
    for (int t = 0; t < bptt; ++t)
        hipLaunchKernelGGL((lstm_fwd_step4_kernel<T, H>), dim3(mb / 32, H / 32), dim3(256), 0, s, RK,
                           R, mb_seq, mb, (const T*)start_h, (const T*)start_c, lw, t, feat);
    // heads + loss from the LSTM outputs
    step(std::integral_constant<int, kHeads>{});
    // reverse scan: dh_t and dF_{t+1} per step, then dF_0 from dG_0
    const int cp0 = L * 2 * H + head_cols(p);
    for (int t = bptt - 1; t >= -1; --t)
        hipLaunchKernelGGL((lstm_bwd_step4_kernel<T, H>), dim3(mb / 32, H / 32), dim3(256), 0, s,
                           RK, R, mb_seq, mb, lw, ws.colpart, ws.CP, cp0, t);
    // trunk backward from d features
    step(std::integral_constant<int, kTrunkBwd>{});
    // weight gradients: trunk, head (from the LSTM outputs), Wi, Wh
    WgJobs jobs{};
    jobs.n = L + 3;
    jobs.Mp = ws.Mp;
    int wg = 0;
    for (int l = 0; l < L + 3; ++l) {
        WgJob& J = jobs.job[l];
        J.I = l >= L ? H : (l == 0 ? p.obs_dim : H);
        J.J = l == L ? head_cols(p) : (l > L ? 4 * H : H);
        J.X = l == 0 ? ws.x0 : (l < L ? ws.a[l - 1] : (l == L ? lw.hout : (l == L + 1 ? (const void*)feat : lw.hin)));
        J.Y = l < L ? ws.dz[l] : (l == L ? ws.dhead : lw.dg);
        J.out = ws.slab + ws.slab_off[l];
        J.rps = ws.rps[l];
        J.ti = (J.I + kWgTile - 1) / kWgTile;
        J.tj = (J.J + kWgTile - 1) / kWgTile;
        J.splits = ws.splits[l];
        J.wg0 = wg;
        wg += J.ti * J.tj * J.splits;
    }
    jobs.nwg = wg;
    jobs.ncolx = (ws.CP + 255) / 256;
    jobs.ncol = jobs.ncolx * kColChunks;
    launch_wgrad<T>(jobs, ws, hp, M, p.actions.num_groups, loss_out, make_layout_lstm(p, lstm),
                    grad, h.grad_sumsq_out, s);
    return check_launch("lstm_ppo_minibatch_grad");
}

}  // namespace ml

using namespace ml;

extern "C" {

#ifdef ML_STAMPS
// diagnostic builds only: phase timestamps of the fused minibatch kernel
void mlearn_debug_set_stamp_buffer(uint64_t* buf) { g_stamp_buf = buf; }
#endif

int64_t mlearn_grad_sumsq_parts(int64_t param_count) {
    return param_count < 1 ? -1 : (param_count + 63) / 64;
}

int64_t mlearn_param_count(const mlearn_mlp_policy* policy) {
    if (validate_policy(policy)) return -1;
    return make_layout(*policy).total;
}

int64_t mlearn_ppo_workspace_bytes(const mlearn_mlp_policy* policy, int64_t rows) {
    if (validate_policy(policy) || rows < 1) return -1;
    return (int64_t)carve(*policy, rows, nullptr, nullptr);
}

int32_t mlearn_ppo_step_kernel(const mlearn_mlp_policy* policy, int64_t rows, int32_t requested) {
    if (validate_policy(policy) || rows < 1 || requested < 0 || requested > 2) return -1;
    const int64_t Mp = (rows + kRowAlign - 1) / kRowAlign * kRowAlign;
    const PolicyK P = make_policy_k(*policy);
    const bool rows16 = rows16_eligible(P, Mp, head_cols(*policy), policy->num_layers,
                                        policy->hidden, policy->dtype == MLEARN_DTYPE_BF16);
    if (requested == 2 && !rows16) return -1;
    return rows16 && requested != 1 ? 2 : 1;
}

static int ppo_entry(const mlearn_mlp_policy* policy, const mlearn_rollout_view* ro,
                     const int32_t* mb_seq, int32_t mb_size, const float* adv_stats,
                     const mlearn_ppo_hparams* hp, float* grad, float* loss_out, void* workspace,
                     bool step_only, mlearn_stream_t stream) {
    int rc = validate_policy(policy);
    if (rc) return rc;
    ML_REQUIRE(ro && mb_seq && adv_stats && hp && workspace, "ppo: null pointer");
    ML_REQUIRE(step_only || grad, "ppo: null grad");
    ML_REQUIRE(mb_size >= 1, "ppo: mb_size must be >= 1");
    ML_REQUIRE(ro->N >= 1 && ro->N < (1ll << 31) && (int64_t)mb_size * ro->bptt_len < (1ll << 31),
               "ppo: N and rows per minibatch must be < 2^31");
    ML_REQUIRE(ro->bptt_len >= 1 && ro->T % ro->bptt_len == 0, "ppo: bad bptt_len");
    ML_REQUIRE(ro->ld == 0 || ro->ld >= ro->N, "ppo: ld %lld < N %lld", (long long)ro->ld,
               (long long)ro->N);
    ML_REQUIRE(ro->obs && ro->actions && ro->log_probs && ro->advantages &&
                   (ro->returns || ro->values),
               "ppo: null rollout array");
    ML_REQUIRE(!hp->clip_value_loss || ro->values, "ppo: clip_value_loss needs values");
    ML_REQUIRE(!hp->normalize_values || policy->critic_bins == 1,
               "ppo: normalize_values needs the scalar critic (ppo.py:54-57)");
    hipStream_t s = S(stream);
#define ML_DISPATCH(T)                                                                           \
    switch (policy->hidden) {                                                                   \
        case 64: return launch_minibatch<T, 64>(*policy, *ro, mb_seq, mb_size, adv_stats, *hp,  \
                                                grad, loss_out, workspace, step_only, s);       \
        case 128: return launch_minibatch<T, 128>(*policy, *ro, mb_seq, mb_size, adv_stats, *hp, \
                                                  grad, loss_out, workspace, step_only, s);     \
        default: return launch_minibatch<T, 256>(*policy, *ro, mb_seq, mb_size, adv_stats, *hp, \
                                                 grad, loss_out, workspace, step_only, s);      \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
}

int mlearn_ppo_minibatch_grad(const mlearn_mlp_policy* policy, const mlearn_rollout_view* ro,
                              const int32_t* mb_seq, int32_t mb_size, const float* adv_stats,
                              const mlearn_ppo_hparams* hp, float* grad, float* loss_out,
                              void* workspace, mlearn_stream_t stream) {
    return ppo_entry(policy, ro, mb_seq, mb_size, adv_stats, hp, grad, loss_out, workspace, false,
                     stream);
}

int64_t mlearn_lstm_ppo_workspace_bytes(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                        int64_t rows, int32_t mb_size) {
    if (validate_lstm(policy, lstm) || rows < 1 || mb_size < 1) return -1;
    return (int64_t)carve(*policy, rows, nullptr, nullptr, lstm, mb_size, nullptr);
}

int mlearn_lstm_ppo_minibatch_grad(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                                   const mlearn_rollout_view* ro, const void* start_h,
                                   const void* start_c, const int32_t* mb_seq, int32_t mb_size,
                                   const float* adv_stats, const mlearn_ppo_hparams* hp,
                                   float* grad, float* loss_out, void* workspace,
                                   mlearn_stream_t stream) {
    int rc = validate_lstm(policy, lstm);
    if (rc) return rc;
    ML_REQUIRE(ro && mb_seq && adv_stats && hp && workspace && grad && start_h && start_c,
               "lstm ppo: null pointer");
    ML_REQUIRE(ro->dones, "lstm ppo: the rollout view needs dones (sequence breaks)");
    ML_REQUIRE(mb_size >= 32 && mb_size % 32 == 0, "lstm ppo: mb_size must be a multiple of 32");
    ML_REQUIRE(((int64_t)mb_size * ro->bptt_len) % 64 == 0,
               "lstm ppo: mb_size * bptt_len must be a multiple of 64");
    ML_REQUIRE(ro->N >= 1 && ro->N < (1ll << 31) && (int64_t)mb_size * ro->bptt_len < (1ll << 31),
               "lstm ppo: N and rows per minibatch must be < 2^31");
    ML_REQUIRE(ro->bptt_len >= 1 && ro->T % ro->bptt_len == 0, "lstm ppo: bad bptt_len");
    ML_REQUIRE(ro->ld == 0 || ro->ld >= ro->N, "lstm ppo: ld < N");
    ML_REQUIRE(ro->obs && ro->actions && ro->log_probs && ro->advantages &&
                   (ro->returns || ro->values),
               "lstm ppo: null rollout array");
    ML_REQUIRE(!hp->clip_value_loss || ro->values, "lstm ppo: clip_value_loss needs values");
    ML_REQUIRE(!hp->normalize_values || policy->critic_bins == 1,
               "lstm ppo: normalize_values needs the scalar critic (ppo.py:54-57)");
    hipStream_t s = S(stream);
#define ML_DISPATCH(T)                                                                            \
    switch (policy->hidden) {                                                                    \
        case 64: return launch_minibatch_lstm<T, 64>(*policy, *lstm, *ro, start_h, start_c,      \
                                                     mb_seq, mb_size, adv_stats, *hp, grad,      \
                                                     loss_out, workspace, s);                    \
        case 128: return launch_minibatch_lstm<T, 128>(*policy, *lstm, *ro, start_h, start_c,    \
                                                       mb_seq, mb_size, adv_stats, *hp, grad,    \
                                                       loss_out, workspace, s);                  \
        default: return launch_minibatch_lstm<T, 256>(*policy, *lstm, *ro, start_h, start_c,     \
                                                      mb_seq, mb_size, adv_stats, *hp, grad,     \
                                                      loss_out, workspace, s);                   \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
}

int mlearn_ppo_minibatch_fwd_bwd(const mlearn_mlp_policy* policy, const mlearn_rollout_view* ro,
                                 const int32_t* mb_seq, int32_t mb_size, const float* adv_stats,
                                 const mlearn_ppo_hparams* hp, void* workspace,
                                 mlearn_stream_t stream) {
    return ppo_entry(policy, ro, mb_seq, mb_size, adv_stats, hp, nullptr, nullptr, workspace, true,
                     stream);
}

}  // extern "C"
