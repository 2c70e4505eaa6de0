// LSTM kernels of the recurrent PPO update (LSTM.sequence, rnn.py:81-111,
// and its reverse for BPTT).  Textually included by ppo.hip inside namespace
// ml (uses its RolloutK / LstmWsK / store_row).
//
// One launch per time step over (mb / 32) x (H / 32) workgroups, one per (32
// sequences, 32-unit block), so the recurrence runs on every CU.  A workgroup
// owns the four gate blocks (i, f, g, o) of its 32 units (weight images in
// unit-block gate order), so the cell update is register-local.  The carries
// cross the launch boundary through memory: h and c into step t are the rows
// hin / cin written by step t - 1 (cleared where dones[t - 1]), the c
// cotangent into step t is dcc [Mp][H] f32 written by step t + 1.  B
// fragments are read straight from the natural-order rows (RT<T>::row).
//   lstm_fwd_step4_kernel  gates_t = F_t Wi + h_{t-1} Wh + bias -> cell
//   lstm_bwd_step4_kernel  dh_t = dG_{t+1} Wh^T and dF_{t+1} = dG_{t+1} Wi^T
//                          from one stream of the dG rows -> cell backward
// (Both scans as one persistent launch per direction -- unit-block slices of
// Wh / Wh^T resident in LDS, carries handed between a tile's workgroups
// through write-through rows and counters -- were bit-identical and slower:
// 13.82 vs 10.40 ms per config-L update, profiles/r04_lstm_scan_ab.txt.)
#pragma once

// k-steps of weight fragments in flight per wave in the per-step scans
// (DEPTH >= k-steps: the whole product's loads issued up front)
#ifndef ML_LSTM_FWD_DEPTH
#define ML_LSTM_FWD_DEPTH 4  // (config L, rocprof us per step: 8 -> 11.0, 4 -> 10.5, 3 -> 10.6, 2 -> 10.9, 6 -> 10.8)
#endif
#ifndef ML_LSTM_BWD_DEPTH
#define ML_LSTM_BWD_DEPTH 8  // (2 -> 14.9, 4 -> 14.7, 6 -> 14.6, 8 -> 14.7, 16 -> 16.3)
#endif
constexpr int kLstmFwdDepth = ML_LSTM_FWD_DEPTH, kLstmBwdDepth = ML_LSTM_BWD_DEPTH;

// Forward step t with four waves per (32 sequences, 32-unit block): wave g
// computes k-half (g & 1) of the input product F_t Wi (g < 2) or of the
// hidden product h_{t-1} Wh (g >= 2) for all four gate blocks; the four
// partials meet in LDS and are summed in fixed order ((p0 + p1) + p2) + p3;
// wave j then runs the cell update for register quad j (as the reverse step).
// The carry rows into step t: the sequence's rnn_start_states (rollouts.py:
// 533-537) at step 0 (also written out as the step's hin / cin rows for the
// backward and the weight gradient), else the rows step t - 1 wrote.
// (One wave per workgroup doing both whole products: 11.13 vs 10.84 us per
// step, 10.26 vs 10.14 ms per config-L update, profiles/r04_lstm_fwd4_ab.txt.)
template <typename T, int H>
__global__ __launch_bounds__(256) void lstm_fwd_step4_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb,
    const T* __restrict__ sh, const T* __restrict__ sc, LstmWsK lw, int t,
    const T* __restrict__ feat) {
    typedef typename RT<T>::frag frag;
    constexpr int KS = RT<T>::KS, E = RT<T>::E, KSH = H / KS, KH = KSH / 2;
    __shared__ float part[4][4][16][64];  // wave g, gate block, accumulator register q, lane
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
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
    const int k0 = (g & 1) * KH;
    const T* brow = g < 2 ? feat + f * H : hrow;
    frag bf[KH];
#pragma unroll
    for (int s = 0; s < KH; ++s) bf[s] = RT<T>::row(brow, k0 + s, h);
    // cell operands of register quad j = g in flight under the product
    const int j = g, u0 = w * 32 + 8 * j + 4 * h;
    const float4 cv = load4(crow + u0);
    const bool more = t + 1 < ro.bptt;
    const bool done = more && ro.dones[store_row(ro, mb_seq, mb, f)] != 0;
    float bz[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) bz[gt][e] = R.bias[gt * H + u0 + e];
    if (t == 0) {
        const float4 hv = load4(hrow + u0);
        store4((T*)lw.hin + f * H + u0, hv.x, hv.y, hv.z, hv.w);
        store4((T*)lw.cin + f * H + u0, cv.x, cv.y, cv.z, cv.w);
    }
    f32x16 acc[4];
    zero_acc<4>(acc);
    const T* img = (const T*)(g < 2 ? R.wi_nat : R.wh_nat) + ((int64_t)w * 4 * KSH + k0) * 64 * E;
    gemm_ring<T, 4, KH, (kLstmFwdDepth < KH ? kLstmFwdDepth : KH)>(acc, bf, KH, img, lane, KSH);
#pragma unroll
    for (int gt = 0; gt < 4; ++gt)
#pragma unroll
        for (int q = 0; q < 16; ++q) part[g][gt][q][lane] = acc[gt][q];
    __syncthreads();
    const float keep = done ? 0.f : 1.f;
    T* gts = (T*)lw.gates + f * 4 * H;
    float gi[4], gf[4], gg[4], go[4], cn[4], hn[4], hc[4], ck[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int q = 4 * j + e;
        float z[4];
#pragma unroll
        for (int gt = 0; gt < 4; ++gt)
            z[gt] = (((part[0][gt][q][lane] + part[1][gt][q][lane]) + part[2][gt][q][lane]) +
                     part[3][gt][q][lane]) + bz[gt][e];
        const CellOut o = lstm_cell_fwd<T>(z[0], z[1], z[2], z[3], f4get(cv, e));
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

// Reverse step t (from bptt-1 down to 0; t = -1: the trailing launch that
// forms dF_0 from dG_0) with four waves per (32 sequences, 32-unit block):
// wave g computes the K quarter g (gate g's H columns of dG_{t+1}) of
// dh_t = dG_{t+1} Wh^T and of dF_{t+1} = dG_{t+1} Wi^T from ONE stream of the
// dG rows; the four partials are summed in fixed order ((p0 + p1) + p2) + p3
// (deterministic); wave j then runs the cell backward for register quad j;
// the bias column partials are 32-lane butterfly sums.
// Sum over the 32 lanes of this lane's half wave (fixed butterfly).
__device__ inline float half_sum32(float x) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o);
    return x;
}

template <typename T, int H>
__global__ __launch_bounds__(256) void lstm_bwd_step4_kernel(
    LstmK R, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, LstmWsK lw,
    float* colpart, int CP, int cp0, int t) {
    constexpr int KS = RT<T>::KS, E = RT<T>::E, NKS = 4 * H / KS, NQ = NKS / 4, NU = H / 32;
    __shared__ float part[4][16][64];   // K quarter g, accumulator register q, lane
    __shared__ float partf[4][16][64];  // the same for dF_{t+1}
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
        gemm_stream<T, 2, NQ, kLstmBwdDepth>(
            acc, brow, (const T*)R.w_bwd + ((int64_t)w * NKS + g * NQ) * 64 * E, lane, NU * NKS);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) part[g][q][lane] = acc[1][q];
#pragma unroll
    for (int q = 0; q < 16; ++q) partf[g][q][lane] = acc[0][q];
    __syncthreads();
    if (prod) {
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

