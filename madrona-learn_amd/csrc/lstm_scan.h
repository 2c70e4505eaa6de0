// LSTM kernels of the recurrent PPO update (LSTM.sequence, rnn.py:81-111,
// and its reverse for BPTT).  Textually included by ppo.hip inside namespace
// ml (uses its RolloutK / LstmWsK / store_row).
//
// The products that do not depend on the recurrence run as full-grid
// launches over all minibatch rows, so only the hidden-to-hidden product is
// left inside the sequential scans:
//   lstm_gin_kernel       Gin = F Wi for every row (f32, accumulator order)
//   lstm_fwd_scan_kernel  gates_t = Gin_t + h Wh + bias -> cell, per step
//   lstm_bwd_scan_kernel  dh_t = dG_{t+1} Wh^T -> cell backward, per step
//   lstm_dfeat_kernel     dF = dG Wi^T for every row
// The split keeps the f32 accumulation order of the fused product (the
// F k-steps, then the h k-steps, in one accumulator), so the gates are
// bit-identical to computing both products in the scan.
//
// A scan workgroup owns 32 sequences of the minibatch for the whole chunk
// and has H/32 waves; wave w owns unit block w (units 32w .. 32w+31), i.e.
// the four gate blocks (i, f, g, o) of those units (weight images in
// unit-block gate order), so the cell update is register-local: the c carry
// (forward) and its cotangent (backward) stay in the lanes' registers, the h
// carry / dG_t rows are exchanged between the waves as B fragments in LDS
// (one barrier pair per step).  The Wh image streams from L2 every step.
#pragma once

// Natural-order B fragments in LDS (fr[s * 64 + lane], the layout RT<T>::row
// reads): element k of row r; put4 writes k0 .. k0+3 (k0 % 4 == 0).
template <typename T> struct LdsRow;
template <> struct LdsRow<bf16> {
    __device__ static void put4(bf16x8* fr, int k0, int r, float a, float b, float c, float d) {
        bf16* p = (bf16*)(fr + (k0 >> 4) * 64 + r + 32 * ((k0 >> 3) & 1)) + (k0 & 7);
        store4(p, a, b, c, d);
    }
};
template <> struct LdsRow<float> {
    __device__ static void put4(float* fr, int k0, int r, float a, float b, float c, float d) {
        float* p = fr + (k0 >> 1) * 64 + r;  // k0: step k0/2 half 0; k0+1: half 1; ...
        p[0] = a;
        p[32] = b;
        p[64] = c;
        p[96] = d;
    }
};

// The NKS x 64 B fragments of 32 rows, loaded cooperatively by NT threads
// into registers (load) and written to LDS later (put).
template <typename T, int NKS, int NT> struct RowStage {
    static constexpr int NF = NKS * 64, N = (NF + NT - 1) / NT;
    typename RT<T>::frag v[N];
    template <typename RowF> __device__ void load(RowF rowp, int tid) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int idx = tid + i * NT;
            if (NF % NT == 0 || idx < NF) v[i] = RT<T>::row(rowp(idx & 31), idx >> 6, (idx >> 5) & 1);
        }
    }
    __device__ void put(typename RT<T>::frag* fr, int tid) const {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int idx = tid + i * NT;
            if (NF % NT == 0 || idx < NF) fr[idx] = v[i];
        }
    }
};

template <int H> constexpr int scan_threads() { return 2 * H; }  // H/32 waves

// Gin in accumulator order: for row tile (32 rows) and unit block w, 16
// chunks of 64 float4 (chunk c = 4 * gate + register quad, lane-contiguous),
// i.e. every wave-instruction moves one contiguous KiB.
__device__ inline int64_t gin_base(int64_t tile, int nw, int w) {
    return (tile * nw + w) * 16 * 64;
}

// Gin = F Wi over every row of the minibatch (one 32-row tile per workgroup).
template <typename T, int H>
__global__ __launch_bounds__(scan_threads<H>()) void lstm_gin_kernel(LstmK R,
                                                                    const T* __restrict__ feat,
                                                                    float4* __restrict__ gin) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, KSH = H / KS, NT = scan_threads<H>(), NW = H / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    frag* frf = (frag*)smem;  // [KSH][64]
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t tile = blockIdx.x;
    {
        RowStage<T, KSH, NT> st;
        st.load([&](int i) { return feat + (tile * 32 + i) * H; }, tid);
        st.put(frf, tid);
    }
    __syncthreads();
    f32x16 acc[4];
    zero_acc<4>(acc);
    gemm_lds<T, 4, KSH, 6>(acc, frf, (const T*)R.wi_nat + (int64_t)w * 4 * KSH * 64 * E, lane);
    float4* o = gin + gin_base(tile, NW, w) + lane;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            o[(4 * g + c) * 64] =
                make_float4(acc[g][4 * c], acc[g][4 * c + 1], acc[g][4 * c + 2], acc[g][4 * c + 3]);
}

// Forward scan over the chunk: gates_t = Gin_t + h Wh + bias -> cell ->
// gates / c_t / h_t saved for the backward, carries into t + 1 cleared where
// dones[t] (rnn.py:92-96); the carry-in rows (hin / cin) are written for the
// weight gradient and the backward.  Step 0 starts from the sequences'
// rnn_start_states [C][ld][H] (rollouts.py:533-537).
template <typename T, int H>
__global__ __launch_bounds__(scan_threads<H>()) void lstm_fwd_scan_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb,
    const float4* __restrict__ gin, const T* __restrict__ sh, const T* __restrict__ sc,
    LstmWsK lw) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, KSH = H / KS, NT = scan_threads<H>(), NW = H / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    frag* frh = (frag*)smem;  // [KSH][64] h carry into step t
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0 = blockIdx.x * 32;
    const int bptt = ro.bptt;
    auto start_row = [&](int i) -> int64_t {
        const int64_t seq = mb_seq[m0 + i];
        const int64_t c = seq / ro.N, b = seq - c * ro.N;
        return (c * ro.ld + b) * H;
    };
    float cc[16];  // c carry: register q = 4j + e <-> unit 32w + 8j + 4h + e of row r
    {
        const int64_t src = start_row(r);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int u0 = w * 32 + 8 * j + 4 * h;
            const float4 hv = load4(sh + src + u0), cv = load4(sc + src + u0);
            store4((T*)lw.hin + (int64_t)(m0 + r) * H + u0, hv.x, hv.y, hv.z, hv.w);
            store4((T*)lw.cin + (int64_t)(m0 + r) * H + u0, cv.x, cv.y, cv.z, cv.w);
#pragma unroll
            for (int e = 0; e < 4; ++e) cc[4 * j + e] = f4get(cv, e);
        }
        RowStage<T, KSH, NT> st;
        st.load([&](int i) { return sh + start_row(i); }, tid);
        st.put(frh, tid);
    }
    __syncthreads();
    const T* wh = (const T*)R.wh_nat + (int64_t)w * 4 * KSH * 64 * E;
    for (int t = 0; t < bptt; ++t) {
        const int64_t f = (int64_t)t * mb + m0 + r;
        const bool more = t + 1 < bptt;
        const bool done = more && ro.dones[store_row(ro, mb_seq, mb, f)] != 0;
        f32x16 acc[4];
        {
            const float4* gi = gin + gin_base((int64_t)t * (mb / 32) + blockIdx.x, NW, w) + lane;
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float4 x = gi[(4 * g + c) * 64];
                    acc[g][4 * c] = x.x;
                    acc[g][4 * c + 1] = x.y;
                    acc[g][4 * c + 2] = x.z;
                    acc[g][4 * c + 3] = x.w;
                }
        }
        gemm_lds<T, 4, KSH, 8>(acc, frh, wh, lane);
        T* gts = (T*)lw.gates + f * 4 * H;
        const float keep = done ? 0.f : 1.f;
        float hc[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int u0 = w * 32 + 8 * j + 4 * h;
            float gi[4], gf[4], gg[4], go[4], cn[4], hn[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int q = 4 * j + e, u = u0 + e;
                const CellOut o = lstm_cell_fwd<T>(acc[0][q] + R.bias[u], acc[1][q] + R.bias[H + u],
                                                   acc[2][q] + R.bias[2 * H + u],
                                                   acc[3][q] + R.bias[3 * H + u], cc[q]);
                gi[e] = o.i;
                gf[e] = o.f;
                gg[e] = o.g;
                go[e] = o.o;
                cn[e] = o.c;
                hn[e] = o.h;
                cc[q] = keep * o.c;
                hc[q] = keep * o.h;
            }
            store4(gts + u0, gi[0], gi[1], gi[2], gi[3]);
            store4(gts + H + u0, gf[0], gf[1], gf[2], gf[3]);
            store4(gts + 2 * H + u0, gg[0], gg[1], gg[2], gg[3]);
            store4(gts + 3 * H + u0, go[0], go[1], go[2], go[3]);
            store4((T*)lw.cout + f * H + u0, cn[0], cn[1], cn[2], cn[3]);
            store4((T*)lw.hout + f * H + u0, hn[0], hn[1], hn[2], hn[3]);
            if (more) {
                store4((T*)lw.hin + (f + mb) * H + u0, hc[4 * j], hc[4 * j + 1], hc[4 * j + 2],
                       hc[4 * j + 3]);
                store4((T*)lw.cin + (f + mb) * H + u0, cc[4 * j], cc[4 * j + 1], cc[4 * j + 2],
                       cc[4 * j + 3]);
            }
        }
        if (!more) break;
        __syncthreads();  // every wave's product has read h_t
#pragma unroll
        for (int j = 0; j < 4; ++j)
            LdsRow<T>::put4(frh, w * 32 + 8 * j + 4 * h, r, hc[4 * j], hc[4 * j + 1], hc[4 * j + 2],
                            hc[4 * j + 3]);
        __syncthreads();
    }
}

// Reverse scan.  Step t (from bptt-1 down to 0): dh_t = dG_{t+1} Wh^T (w_bwd
// block H/32 + w, K = 4H from LDS), then the cell backward of step t for unit
// block w: dh = dHout_t + dh_t and the c cotangent, both cut where the carry
// out of step t was cleared (dones[t]) or at the end of the chunk; writes
// dG_t (rounded to the compute dtype) and the per-tile column partials of dG
// (the bias gradient).  dF = dG Wi^T follows as lstm_dfeat_kernel.
template <typename T, int H>
__global__ __launch_bounds__(scan_threads<H>()) void lstm_bwd_scan_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, LstmWsK lw,
    float* colpart, int CP, int cp0) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, NKS = 4 * H / KS, NU = H / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    frag* frg = (frag*)smem;  // [NKS][64] dG_{t+1} of the workgroup's 32 rows
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0 = blockIdx.x * 32, m = m0 + r;
    const int bptt = ro.bptt;
    const T* wdh = (const T*)R.w_bwd + (int64_t)(NU + w) * NKS * 64 * E;  // h-cotangent block w
    float dcc[16];  // c cotangent carried from step t + 1 into t
#pragma unroll
    for (int q = 0; q < 16; ++q) dcc[q] = 0.f;
    for (int t = bptt - 1; t >= 0; --t) {
        const int64_t fs = (int64_t)t * mb + m;
        const bool cut = t + 1 == bptt || ro.dones[store_row(ro, mb_seq, mb, fs)] != 0;
        f32x16 acc[1];
        zero_acc<1>(acc);
        if (t + 1 < bptt) gemm_lds<T, 1, NKS, 8>(acc, frg, wdh, lane);
        const T* gts = (const T*)lw.gates + fs * 4 * H;
        T* dgs = (T*)lw.dg + fs * 4 * H;
        float dpi[16], dpf[16], dpg[16], dpo[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int u0 = w * 32 + 8 * j + 4 * h;
            const float4 dho = load4((const T*)lw.dhout + fs * H + u0);
            const float4 gi = load4(gts + u0), gf = load4(gts + H + u0);
            const float4 gg = load4(gts + 2 * H + u0), go = load4(gts + 3 * H + u0);
            const float4 c4 = load4((const T*)lw.cout + fs * H + u0);
            const float4 ci = load4((const T*)lw.cin + fs * H + u0);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int q = 4 * j + e;
                const float i_ = f4get(gi, e), f_ = f4get(gf, e), g_ = f4get(gg, e), o_ = f4get(go, e);
                const float dh = f4get(dho, e) + (cut ? 0.f : acc[0][q]);
                const float tc = tanh_fast(f4get(c4, e));
                const float dout = dh * tc;
                const float dc = (cut ? 0.f : dcc[q]) + dh * o_ * (1.f - tc * tc);
                dpi[q] = rnd<T>((dc * g_) * i_ * (1.f - i_));
                dpf[q] = rnd<T>((dc * f4get(ci, e)) * f_ * (1.f - f_));
                dpg[q] = rnd<T>((dc * i_) * (1.f - g_ * g_));
                dpo[q] = rnd<T>(dout * o_ * (1.f - o_));
                dcc[q] = dc * f_;
            }
            store4(dgs + u0, dpi[4 * j], dpi[4 * j + 1], dpi[4 * j + 2], dpi[4 * j + 3]);
            store4(dgs + H + u0, dpf[4 * j], dpf[4 * j + 1], dpf[4 * j + 2], dpf[4 * j + 3]);
            store4(dgs + 2 * H + u0, dpg[4 * j], dpg[4 * j + 1], dpg[4 * j + 2], dpg[4 * j + 3]);
            store4(dgs + 3 * H + u0, dpo[4 * j], dpo[4 * j + 1], dpo[4 * j + 2], dpo[4 * j + 3]);
        }
        if (t > 0) {
            __syncthreads();  // every wave's product has read dG_{t+1}
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k0 = w * 32 + 8 * j + 4 * h;
                LdsRow<T>::put4(frg, k0, r, dpi[4 * j], dpi[4 * j + 1], dpi[4 * j + 2],
                                dpi[4 * j + 3]);
                LdsRow<T>::put4(frg, H + k0, r, dpf[4 * j], dpf[4 * j + 1], dpf[4 * j + 2],
                                dpf[4 * j + 3]);
                LdsRow<T>::put4(frg, 2 * H + k0, r, dpg[4 * j], dpg[4 * j + 1], dpg[4 * j + 2],
                                dpg[4 * j + 3]);
                LdsRow<T>::put4(frg, 3 * H + k0, r, dpo[4 * j], dpo[4 * j + 1], dpo[4 * j + 2],
                                dpo[4 * j + 3]);
            }
        }
        // bias gradient: column sums of dG over this tile's 32 rows
        {
            const int qs = col_sum16_index(lane);
            float* cp = colpart + (int64_t)(((int64_t)t * mb + m0) / 32) * CP + cp0;
            const int uq = w * 32 + feat(0, qs, h);
            const float si = col_sum16(dpi, lane), sf = col_sum16(dpf, lane);
            const float sg = col_sum16(dpg, lane), so = col_sum16(dpo, lane);
            if ((lane & 16) == 0) {
                cp[uq] = si;
                cp[H + uq] = sf;
                cp[2 * H + uq] = sg;
                cp[3 * H + uq] = so;
            }
        }
        if (t > 0) __syncthreads();
    }
}

// dF = dG Wi^T over every row of the minibatch (w_bwd blocks 0 .. H/32-1,
// one 32-feature block per wave), rounded to the compute dtype.
template <typename T, int H>
__global__ __launch_bounds__(scan_threads<H>()) void lstm_dfeat_kernel(LstmK R, LstmWsK lw) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, NKS = 4 * H / KS, NT = scan_threads<H>();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    frag* frg = (frag*)smem;  // [NKS][64] dG rows of the tile
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t tile = blockIdx.x;
    {
        RowStage<T, NKS, NT> st;
        st.load([&](int i) { return (const T*)lw.dg + (tile * 32 + i) * 4 * H; }, tid);
        st.put(frg, tid);
    }
    __syncthreads();
    f32x16 acc[1];
    zero_acc<1>(acc);
    gemm_lds<T, 1, NKS, 8>(acc, frg, (const T*)R.w_bwd + (int64_t)w * NKS * 64 * E, lane);
    T* drow = (T*)lw.dfeat + (tile * 32 + (lane & 31)) * H + w * 32;
#pragma unroll
    for (int g = 0; g < 4; ++g)
        store4(drow + 8 * g + 4 * h, acc[0][4 * g], acc[0][4 * g + 1], acc[0][4 * g + 2],
               acc[0][4 * g + 3]);
}

// k-steps of Wh (and, backward, dG) fragments in flight per wave in the
// per-step scans (DEPTH > k-steps: the whole product's loads issued up front)
#ifndef ML_LSTM_FWD_DEPTH
#define ML_LSTM_FWD_DEPTH 8
#endif
#ifndef ML_LSTM_FWD4_DEPTH
#define ML_LSTM_FWD4_DEPTH 8
#endif
#ifndef ML_LSTM_BWD4_DEPTH
#define ML_LSTM_BWD4_DEPTH 8
#endif

// ---------------------------------------------------------------------------
// Per-step scans: one launch per time step with a one-wave workgroup per (32
// sequences, 32-unit block), (mb / 32) x (H / 32) workgroups, so the
// recurrence runs on every CU (the persistent scans above keep H / 32 waves
// on only mb / 32 CUs, each streaming the whole Wh image every step).  The
// carries cross the launch boundary through memory: h and c into step t are
// the rows hin / cin written by step t - 1 (cleared where dones[t - 1]), the
// c cotangent into step t is dcc [Mp][H] f32 written by step t + 1.  B
// fragments are read straight from the natural-order rows (RT<T>::row): no
// LDS, no barrier.  The MFMA sequences and the cell arithmetic are those of
// the persistent scans, so gates, c, h and dG are bit-identical to them.
// ---------------------------------------------------------------------------
template <typename T, int H>
__global__ __launch_bounds__(64) void lstm_fwd_step_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb,
    const float4* __restrict__ gin, const T* __restrict__ sh, const T* __restrict__ sc,
    LstmWsK lw, int t, const T* __restrict__ feat) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, KSH = H / KS, NW = H / 32;
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    const int tile = blockIdx.x, w = blockIdx.y;
    const int m = tile * 32 + r;
    const int64_t f = (int64_t)t * mb + m;
    // carry rows into step t: the sequence's rnn_start_states (rollouts.py:
    // 533-537) at step 0 (also written out as the step's hin / cin rows for
    // the backward and the weight gradient), else the rows step t - 1 wrote
    const T *hrow, *crow;
    if (t == 0) {
        const int64_t seq = mb_seq[m];
        const int64_t c = seq / ro.N, b = seq - c * ro.N;
        hrow = sh + (c * ro.ld + b) * H;
        crow = sc + (c * ro.ld + b) * H;
    } else {
        hrow = (const T*)lw.hin + f * H;
        crow = (const T*)lw.cin + f * H;
    }
    frag hb[KSH];
#pragma unroll
    for (int s = 0; s < KSH; ++s) hb[s] = RT<T>::row(hrow, s, h);
    float cc[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int u0 = w * 32 + 8 * j + 4 * h;
        const float4 cv = load4(crow + u0);
#pragma unroll
        for (int e = 0; e < 4; ++e) cc[4 * j + e] = f4get(cv, e);
        if (t == 0) {
            const float4 hv = load4(hrow + u0);
            store4((T*)lw.hin + f * H + u0, hv.x, hv.y, hv.z, hv.w);
            store4((T*)lw.cin + f * H + u0, cv.x, cv.y, cv.z, cv.w);
        }
    }
    f32x16 acc[4];
    if (feat) {
        // the input product F Wi in this launch (F = the step's trunk output
        // rows): the same k-step sequence into the same zeroed accumulators
        // as lstm_gin_kernel, so the gates are bit-identical to reading Gin
        frag fb[KSH];
#pragma unroll
        for (int s = 0; s < KSH; ++s) fb[s] = RT<T>::row(feat + f * H, s, h);
        zero_acc<4>(acc);
        gemm_ring<T, 4, KSH, ML_LSTM_FWD_DEPTH>(acc, fb, KSH,
                                                (const T*)R.wi_nat + (int64_t)w * 4 * KSH * 64 * E, lane);
    } else {
        const float4* gi = gin + gin_base((int64_t)t * (mb / 32) + tile, NW, w) + lane;
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 x = gi[(4 * g + c) * 64];
                acc[g][4 * c] = x.x;
                acc[g][4 * c + 1] = x.y;
                acc[g][4 * c + 2] = x.z;
                acc[g][4 * c + 3] = x.w;
            }
    }
    // the cell's other operands (done flag: two dependent loads; the biases)
    // in flight under the product: gemm_ring's scheduling fences would
    // otherwise leave their round trips after the last MFMA
    const bool more = t + 1 < ro.bptt;
    const bool done = more && ro.dones[store_row(ro, mb_seq, mb, f)] != 0;
    float bz[4][16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int g = 0; g < 4; ++g) bz[g][4 * j + e] = R.bias[g * H + w * 32 + 8 * j + 4 * h + e];
    gemm_ring<T, 4, KSH, ML_LSTM_FWD_DEPTH>(acc, hb, KSH, (const T*)R.wh_nat + (int64_t)w * 4 * KSH * 64 * E, lane);
    const float keep = done ? 0.f : 1.f;
    T* gts = (T*)lw.gates + f * 4 * H;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int u0 = w * 32 + 8 * j + 4 * h;
        float gi[4], gf[4], gg[4], go[4], cn[4], hn[4], hc[4], ck[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int q = 4 * j + e, u = u0 + e;
            const CellOut o = lstm_cell_fwd<T>(acc[0][q] + bz[0][q], acc[1][q] + bz[1][q],
                                               acc[2][q] + bz[2][q], acc[3][q] + bz[3][q], cc[q]);
            gi[e] = o.i;
            gf[e] = o.f;
            gg[e] = o.g;
            go[e] = o.o;
            cn[e] = o.c;
            hn[e] = o.h;
            ck[e] = keep * o.c;
            hc[e] = keep * o.h;
        }
        store4(gts + u0, gi[0], gi[1], gi[2], gi[3]);
        store4(gts + H + u0, gf[0], gf[1], gf[2], gf[3]);
        store4(gts + 2 * H + u0, gg[0], gg[1], gg[2], gg[3]);
        store4(gts + 3 * H + u0, go[0], go[1], go[2], go[3]);
        store4((T*)lw.cout + f * H + u0, cn[0], cn[1], cn[2], cn[3]);
        store4((T*)lw.hout + f * H + u0, hn[0], hn[1], hn[2], hn[3]);
        if (more) {
            store4((T*)lw.hin + (f + mb) * H + u0, hc[0], hc[1], hc[2], hc[3]);
            store4((T*)lw.cin + (f + mb) * H + u0, ck[0], ck[1], ck[2], ck[3]);
        }
    }
}

template <typename T, int H>
__global__ __launch_bounds__(64) void lstm_bwd_step_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, LstmWsK lw,
    float* colpart, int CP, int cp0, int t) {
    constexpr int KS = RT<T>::KS, E = RT<T>::E, NKS = 4 * H / KS, NU = H / 32;
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    const int tile = blockIdx.x, w = blockIdx.y;
    const int m0 = tile * 32, m = m0 + r;
    const int bptt = ro.bptt;
    const int64_t fs = (int64_t)t * mb + m;
    const bool cut = t + 1 == bptt || ro.dones[store_row(ro, mb_seq, mb, fs)] != 0;
    f32x16 acc[1];
    zero_acc<1>(acc);
    if (t + 1 < bptt)  // dh_t = dG_{t+1} Wh^T (h-cotangent block w of w_bwd)
        gemm_stream<T, 1, NKS, 8>(acc, (const T*)lw.dg + (fs + mb) * 4 * H,
                                  (const T*)R.w_bwd + (int64_t)(NU + w) * NKS * 64 * E, lane);
    const T* gts = (const T*)lw.gates + fs * 4 * H;
    T* dgs = (T*)lw.dg + fs * 4 * H;
    float dpi[16], dpf[16], dpg[16], dpo[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int u0 = w * 32 + 8 * j + 4 * h;
        const float4 dho = load4((const T*)lw.dhout + fs * H + u0);
        const float4 gi = load4(gts + u0), gf = load4(gts + H + u0);
        const float4 gg = load4(gts + 2 * H + u0), go = load4(gts + 3 * H + u0);
        const float4 c4 = load4((const T*)lw.cout + fs * H + u0);
        const float4 ci = load4((const T*)lw.cin + fs * H + u0);
        const float4 dcin = cut ? make_float4(0.f, 0.f, 0.f, 0.f) : *(const float4*)(lw.dcc + fs * H + u0);
        float dco[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int q = 4 * j + e;
            const float i_ = f4get(gi, e), f_ = f4get(gf, e), g_ = f4get(gg, e), o_ = f4get(go, e);
            const float dh = f4get(dho, e) + (cut ? 0.f : acc[0][q]);
            const float tc = tanh_fast(f4get(c4, e));
            const float dout = dh * tc;
            const float dc = f4get(dcin, e) + dh * o_ * (1.f - tc * tc);
            dpi[q] = rnd<T>((dc * g_) * i_ * (1.f - i_));
            dpf[q] = rnd<T>((dc * f4get(ci, e)) * f_ * (1.f - f_));
            dpg[q] = rnd<T>((dc * i_) * (1.f - g_ * g_));
            dpo[q] = rnd<T>(dout * o_ * (1.f - o_));
            dco[e] = dc * f_;
        }
        if (t > 0) *(float4*)(lw.dcc + (fs - mb) * H + u0) = make_float4(dco[0], dco[1], dco[2], dco[3]);
        store4(dgs + u0, dpi[4 * j], dpi[4 * j + 1], dpi[4 * j + 2], dpi[4 * j + 3]);
        store4(dgs + H + u0, dpf[4 * j], dpf[4 * j + 1], dpf[4 * j + 2], dpf[4 * j + 3]);
        store4(dgs + 2 * H + u0, dpg[4 * j], dpg[4 * j + 1], dpg[4 * j + 2], dpg[4 * j + 3]);
        store4(dgs + 3 * H + u0, dpo[4 * j], dpo[4 * j + 1], dpo[4 * j + 2], dpo[4 * j + 3]);
    }
    // bias gradient: column sums of dG over this tile's 32 rows
    const int qs = col_sum16_index(lane);
    float* cp = colpart + (int64_t)(((int64_t)t * mb + m0) / 32) * CP + cp0;
    const int uq = w * 32 + feat(0, qs, h);
    const float si = col_sum16(dpi, lane), sf = col_sum16(dpf, lane);
    const float sg = col_sum16(dpg, lane), so = col_sum16(dpo, lane);
    if ((lane & 16) == 0) {
        cp[uq] = si;
        cp[H + uq] = sf;
        cp[2 * H + uq] = sg;
        cp[3 * H + uq] = so;
    }
}

// ---------------------------------------------------------------------------
// Per-step scans with four waves per (32 sequences, 32-unit block) workgroup
// (ML_LSTM_STEP4, the default): the step's product is split over the waves
// so each wave's serial MFMA chain and weight stream are a quarter of the
// one-wave kernels' above, and 4x as many waves cover the chip.
//   forward:  wave g computes gate block g (Gin_t + h Wh, its 16 KB slice of
//             Wh); the pre-activations meet in LDS; wave j then runs the cell
//             for register quad j (units 8j + 4h .. +3 of the block).  Same
//             MFMA sequence per gate block and same cell arithmetic as
//             lstm_fwd_step_kernel: gates, c, h bit-identical to it.
//   backward: wave g computes dG_{t+1}[:, gate g] Wh_g^T (a quarter of the
//             K = 4H reduction), the four partials are summed in fixed order
//             ((p0 + p1) + p2) + p3 (deterministic; the f32 rounding differs
//             from the single 4H-long chain), then wave j runs the cell
//             backward for register quad j; the bias column partials are
//             32-lane butterfly sums.
// ---------------------------------------------------------------------------
template <typename T, int H>
__global__ __launch_bounds__(256) void lstm_fwd_step4_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb,
    const float4* __restrict__ gin, const T* __restrict__ sh, const T* __restrict__ sc,
    LstmWsK lw, int t) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, KSH = H / KS, NW = H / 32;
    __shared__ float pre[4][16][64];  // gate block g, accumulator register q, lane
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6);  // gate (product) / register quad (cell)
    const int tile = blockIdx.x, w = blockIdx.y;
    const int m = tile * 32 + r;
    const int64_t f = (int64_t)t * mb + m;
    const T *hrow, *crow;
    if (t == 0) {
        const int64_t seq = mb_seq[m];
        const int64_t c = seq / ro.N, b = seq - c * ro.N;
        hrow = sh + (c * ro.ld + b) * H;
        crow = sc + (c * ro.ld + b) * H;
    } else {
        hrow = (const T*)lw.hin + f * H;
        crow = (const T*)lw.cin + f * H;
    }
    frag hb[KSH];
#pragma unroll
    for (int s = 0; s < KSH; ++s) hb[s] = RT<T>::row(hrow, s, h);
    f32x16 acc[1];
    {
        const float4* gi = gin + gin_base((int64_t)t * (mb / 32) + tile, NW, w) + lane;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float4 x = gi[(4 * g + c) * 64];
            acc[0][4 * c] = x.x;
            acc[0][4 * c + 1] = x.y;
            acc[0][4 * c + 2] = x.z;
            acc[0][4 * c + 3] = x.w;
        }
    }
    // cell of register quad j = g: the c carry, the done flag and the biases
    // load under the product
    const int j = g, u0 = w * 32 + 8 * j + 4 * h;
    const float4 cv = load4(crow + u0);
    if (t == 0) {
        const float4 hv = load4(hrow + u0);
        store4((T*)lw.hin + f * H + u0, hv.x, hv.y, hv.z, hv.w);
        store4((T*)lw.cin + f * H + u0, cv.x, cv.y, cv.z, cv.w);
    }
    const bool more = t + 1 < ro.bptt;
    const bool done = more && ro.dones[store_row(ro, mb_seq, mb, f)] != 0;
    float bz[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) bz[gg][e] = R.bias[gg * H + u0 + e];
    gemm_ring<T, 1, KSH, ML_LSTM_FWD4_DEPTH>(acc, hb, KSH, (const T*)R.wh_nat + ((int64_t)w * 4 + g) * KSH * 64 * E,
                            lane);
#pragma unroll
    for (int q = 0; q < 16; ++q) pre[g][q][lane] = acc[0][q];
    const float keep = done ? 0.f : 1.f;
    __syncthreads();
    T* gts = (T*)lw.gates + f * 4 * H;
    float gi[4], gf[4], gg[4], go[4], cn[4], hn[4], hc[4], ck[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int q = 4 * j + e, u = u0 + e;
        const CellOut o = lstm_cell_fwd<T>(pre[0][q][lane] + bz[0][e], pre[1][q][lane] + bz[1][e],
                                           pre[2][q][lane] + bz[2][e], pre[3][q][lane] + bz[3][e],
                                           f4get(cv, e));
        gi[e] = o.i;
        gf[e] = o.f;
        gg[e] = o.g;
        go[e] = o.o;
        cn[e] = o.c;
        hn[e] = o.h;
        ck[e] = keep * o.c;
        hc[e] = keep * o.h;
    }
    store4(gts + u0, gi[0], gi[1], gi[2], gi[3]);
    store4(gts + H + u0, gf[0], gf[1], gf[2], gf[3]);
    store4(gts + 2 * H + u0, gg[0], gg[1], gg[2], gg[3]);
    store4(gts + 3 * H + u0, go[0], go[1], go[2], go[3]);
    store4((T*)lw.cout + f * H + u0, cn[0], cn[1], cn[2], cn[3]);
    store4((T*)lw.hout + f * H + u0, hn[0], hn[1], hn[2], hn[3]);
    if (more) {
        store4((T*)lw.hin + (f + mb) * H + u0, hc[0], hc[1], hc[2], hc[3]);
        store4((T*)lw.cin + (f + mb) * H + u0, ck[0], ck[1], ck[2], ck[3]);
    }
}

// Sum over the 32 lanes of this lane's half wave (fixed butterfly).
__device__ inline float half_sum32(float x) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o);
    return x;
}

template <typename T, int H>
__global__ __launch_bounds__(256) void lstm_bwd_step4_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, LstmWsK lw,
    float* colpart, int CP, int cp0, int t, int dfeat) {
    constexpr int KS = RT<T>::KS, E = RT<T>::E, NKS = 4 * H / KS, NQ = NKS / 4, NU = H / 32;
    __shared__ float part[4][16][64];   // K quarter g, accumulator register q, lane
    __shared__ float partf[4][16][64];  // the same for dF_{t+1} (dfeat)
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6);  // K quarter (product) / register quad (cell)
    const int tile = blockIdx.x, w = blockIdx.y;
    const int m0 = tile * 32, m = m0 + r;
    const int bptt = ro.bptt;
    // t = -1 (dfeat only): the trailing launch that forms dF_0 from dG_0
    const bool cell = t >= 0, prod = t + 1 < bptt;
    const int64_t fs = (int64_t)t * mb + m;  // (not dereferenced at t = -1)
    // cell backward of register quad j = g: its operands load under the
    // product (gemm_stream's scheduling fences would otherwise leave their
    // round trip after the last MFMA)
    const int j = g, u0 = w * 32 + 8 * j + 4 * h;
    bool cut = true;
    float4 dho, gi, gf, gg, go, c4, ci, dcin;
    if (cell) {
        cut = t + 1 == bptt || ro.dones[store_row(ro, mb_seq, mb, fs)] != 0;
        const T* gts = (const T*)lw.gates + fs * 4 * H;
        dho = load4((const T*)lw.dhout + fs * H + u0);
        gi = load4(gts + u0);
        gf = load4(gts + H + u0);
        gg = load4(gts + 2 * H + u0);
        go = load4(gts + 3 * H + u0);
        c4 = load4((const T*)lw.cout + fs * H + u0);
        ci = load4((const T*)lw.cin + fs * H + u0);
        dcin = cut ? make_float4(0.f, 0.f, 0.f, 0.f) : *(const float4*)(lw.dcc + fs * H + u0);
    }
    // quarter g (gate g's H columns of dG_{t+1}) of dh_t = dG_{t+1} Wh^T
    // (acc[1]) and, with dfeat, of dF_{t+1} = dG_{t+1} Wi^T for feature block w
    // (acc[0]): one stream of the dG rows feeds both (w_bwd blocks w and NU + w)
    f32x16 acc[2];
    zero_acc<2>(acc);
    if (prod) {
        const T* brow = (const T*)lw.dg + (fs + mb) * 4 * H + g * H;
        if (dfeat)
            gemm_stream<T, 2, NQ, ML_LSTM_BWD4_DEPTH>(
                acc, brow, (const T*)R.w_bwd + ((int64_t)w * NKS + g * NQ) * 64 * E, lane, NU * NKS);
        else {
            f32x16 a1[1] = {acc[1]};
            gemm_stream<T, 1, NQ, ML_LSTM_BWD4_DEPTH>(
                a1, brow, (const T*)R.w_bwd + ((int64_t)(NU + w) * NKS + g * NQ) * 64 * E, lane);
            acc[1] = a1[0];
        }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) part[g][q][lane] = acc[1][q];
    if (dfeat) {
#pragma unroll
        for (int q = 0; q < 16; ++q) partf[g][q][lane] = acc[0][q];
    }
    __syncthreads();
    if (dfeat && prod) {
        // dF_{t+1} row m, features u0 .. u0 + 3: quarters summed in fixed order
        float d[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int q = 4 * j + e;
            d[e] = ((partf[0][q][lane] + partf[1][q][lane]) + partf[2][q][lane]) + partf[3][q][lane];
        }
        store4((T*)lw.dfeat + (fs + mb) * H + u0, d[0], d[1], d[2], d[3]);
    }
    if (!cell) return;
    float dpi[4], dpf[4], dpg[4], dpo[4], dco[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int q = 4 * j + e;
        const float dhh = ((part[0][q][lane] + part[1][q][lane]) + part[2][q][lane]) + part[3][q][lane];
        const float i_ = f4get(gi, e), f_ = f4get(gf, e), g_ = f4get(gg, e), o_ = f4get(go, e);
        const float dh = f4get(dho, e) + (cut ? 0.f : dhh);
        const float tc = tanh_fast(f4get(c4, e));
        const float dout = dh * tc;
        const float dc = f4get(dcin, e) + dh * o_ * (1.f - tc * tc);
        dpi[e] = rnd<T>((dc * g_) * i_ * (1.f - i_));
        dpf[e] = rnd<T>((dc * f4get(ci, e)) * f_ * (1.f - f_));
        dpg[e] = rnd<T>((dc * i_) * (1.f - g_ * g_));
        dpo[e] = rnd<T>(dout * o_ * (1.f - o_));
        dco[e] = dc * f_;
    }
    if (t > 0) *(float4*)(lw.dcc + (fs - mb) * H + u0) = make_float4(dco[0], dco[1], dco[2], dco[3]);
    T* dgs = (T*)lw.dg + fs * 4 * H;
    store4(dgs + u0, dpi[0], dpi[1], dpi[2], dpi[3]);
    store4(dgs + H + u0, dpf[0], dpf[1], dpf[2], dpf[3]);
    store4(dgs + 2 * H + u0, dpg[0], dpg[1], dpg[2], dpg[3]);
    store4(dgs + 3 * H + u0, dpo[0], dpo[1], dpo[2], dpo[3]);
    // bias gradient: column sums of dG over this tile's 32 rows (units u0 .. u0 + 3)
    float* cp = colpart + (int64_t)(((int64_t)t * mb + m0) / 32) * CP + cp0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float si = half_sum32(dpi[e]), sf = half_sum32(dpf[e]);
        const float sg = half_sum32(dpg[e]), so = half_sum32(dpo[e]);
        if (r == 0) {
            cp[u0 + e] = si;
            cp[H + u0 + e] = sf;
            cp[2 * H + u0 + e] = sg;
            cp[3 * H + u0 + e] = so;
        }
    }
}
