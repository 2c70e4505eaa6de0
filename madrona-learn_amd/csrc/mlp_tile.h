// Row-tile building blocks of the fused MLP kernels (rollout step, PPO
// forward and backward).  One workgroup = 256 threads = 4 waves owns a tile
// of 64 rows.  Wave w owns row block rb = w & 1 (32 rows) and the column
// blocks cb = (w >> 1) + 2*i, i < NB = H/64, so each output column block of
// a row block is computed by exactly one wave and each wave reuses its A
// fragment across its NB column blocks.
//
// Activations of the tile live in LDS as row-major [64][ld] (ld = K + 16 B of
// padding: rows shift by 4 banks, so the 16 lanes of a ds_read_b128 group hit
// distinct banks).  Weights are read as B fragments straight from L2/HBM in
// the transposed [out][in] layout, 16 B per lane.
#pragma once
#include "common.h"

namespace ml {

constexpr int kTileRows = 64;

template <typename T> struct Pad { static constexpr int v = 16 / sizeof(T); };

// acc[i] += A_lds[rb*32 .. +32][0..K) x WT[cb_i*32 .. +32][0..K)^T
template <typename T, int NB>
__device__ inline void tile_gemm(f32x16 (&acc)[NB], const T* A, int lda, int rb, const T* WT,
                                 int ldw, int K, int w, int lane) {
    constexpr int E = MT<T>::E, KS = MT<T>::KS;
    const int r = lane & 31, h = lane >> 5;
    const T* ap = A + (rb * 32 + r) * lda + h * E;
    const T* bp[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) bp[i] = WT + (int64_t)(((w >> 1) + 2 * i) * 32 + r) * ldw + h * E;
    for (int k0 = 0; k0 < K; k0 += KS) {
        typename MT<T>::frag a = MT<T>::load(ap + k0);
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i] = MT<T>::mma(a, MT<T>::load(bp[i] + k0), acc[i]);
    }
}

template <int NB> __device__ inline void zero_acc(f32x16 (&acc)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
}

// In-place row totals: s[e], q[e] hold this lane's partial sums (over its
// column blocks) for the rows of its 16 accumulator registers; on return they
// hold the totals over all H columns (identical in every lane holding a row).
// red: LDS [4][64][2] floats.  Contains one workgroup barrier.
__device__ inline void row_reduce2(float (&s)[16], float (&q)[16], float* red, int w, int lane) {
    const int rb = w & 1;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        s[e] = wave_sum32(s[e]);
        q[e] = wave_sum32(q[e]);
    }
    if ((lane & 31) == 0) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            int row = rb * 32 + acc_row(e, lane);
            red[(w * 64 + row) * 2 + 0] = s[e];
            red[(w * 64 + row) * 2 + 1] = q[e];
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        int row = rb * 32 + acc_row(e, lane);
        s[e] = red[(rb * 64 + row) * 2 + 0] + red[((rb + 2) * 64 + row) * 2 + 0];
        q[e] = red[(rb * 64 + row) * 2 + 1] + red[((rb + 2) * 64 + row) * 2 + 1];
    }
}

struct PolicyK {
    int D, H, L, K, A;
    int off[MLEARN_MAX_GROUPS + 1];
    const void* wt[MLEARN_MAX_LAYERS];
    const void* w[MLEARN_MAX_LAYERS];
    const float* lns[MLEARN_MAX_LAYERS];
    const float* lnb[MLEARN_MAX_LAYERS];
    const void* head_t;
    const void* head;
    const float* head_b;
};

PolicyK make_policy_k(const mlearn_mlp_policy& p);
int validate_policy(const mlearn_mlp_policy* p);

// Store 4 consecutive elements (one 8-byte bf16 / 16-byte f32 store).
__device__ inline void store4(bf16* p, float a, float b, float c, float d) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
    *(bf16x4*)p = v;
}
__device__ inline void store4(float* p, float a, float b, float c, float d) {
    *(float4*)p = make_float4(a, b, c, d);
}

// Write a wave's accumulator-layout values v[i][e] (rows rb*32.., columns of
// its blocks) transposed into XT[col][row0 + row]: per block 4 stores of 4
// consecutive rows.  Rows >= M are written as zeros (padding of the K axis of
// the weight-gradient GEMMs).
template <typename T, int NB>
__device__ inline void store_transposed(const float (&v)[NB][16], T* XT, int64_t ldT, int w,
                                        int lane, int64_t row0, int64_t M) {
    const int rb = w & 1, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int col = ((w >> 1) + 2 * i) * 32 + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t row = row0 + rb * 32 + 8 * q + 4 * h;
            float x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = row + u < M ? v[i][4 * q + u] : 0.f;
            store4(XT + (int64_t)col * ldT + row, x[0], x[1], x[2], x[3]);
        }
    }
}

template <typename T, int NB>
__device__ inline void store_transposed(const f32x16 (&v)[NB], T* XT, int64_t ldT, int w,
                                        int lane, int64_t row0, int64_t M) {
    const int rb = w & 1, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int col = ((w >> 1) + 2 * i) * 32 + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t row = row0 + rb * 32 + 8 * q + 4 * h;
            float x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = row + u < M ? v[i][4 * q + u] : 0.f;
            store4(XT + (int64_t)col * ldT + row, x[0], x[1], x[2], x[3]);
        }
    }
}

// LayerNorm + ReLU epilogue on a wave's accumulators (rows rb*32.., its
// column blocks).  Writes the compute-dtype activation into act (LDS) and,
// when given, z (Dense output, row-major), stats (mean, rstd) and the
// activation transposed (aT[col][row], for the weight-gradient GEMM).
template <typename T, int NB>
__device__ inline void ln_relu_epilogue(f32x16 (&acc)[NB], const float* __restrict__ gamma,
                                        const float* __restrict__ beta, T* act, int ld,
                                        float* red, int w, int lane, int H) {
    const int rb = w & 1, r = lane & 31;
    float s[16], q[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const float x = rnd<T>(acc[i][e]);  // Dense output in the compute dtype
            acc[i][e] = x;
            a += x;
            b += x * x;
        }
        s[e] = a;
        q[e] = b;
    }
    row_reduce2(s, q, red, w, lane);
    const float invH = 1.0f / (float)H;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int row = rb * 32 + acc_row(e, lane);
        const float mean = s[e] * invH;
        const float var = fmaxf(q[e] * invH - mean * mean, 0.f);
        const float rstd = rsqrtf(var + 1e-6f);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int col = ((w >> 1) + 2 * i) * 32 + r;
            float y = (acc[i][e] - mean) * (rstd * gamma[col]) + beta[col];
            act[row * ld + col] = cvt<T>(fmaxf(rnd<T>(y), 0.f));
        }
    }
}

// Heads: out[64][32] = act[64][H] x head_t^T, waves 0 and 1 (one row block each).
template <typename T>
__device__ inline void heads_to_lds(const T* act, int ld, const T* __restrict__ head_t,
                                    const float* __restrict__ head_b, int H, float* lgt, int w,
                                    int lane) {
    if (w < 2) {
        f32x16 acc[1];
        zero_acc<1>(acc);
        constexpr int E = MT<T>::E, KS = MT<T>::KS;
        const int r = lane & 31, h = lane >> 5;
        const T* ap = act + (w * 32 + r) * ld + h * E;
        const T* bp = head_t + r * H + h * E;
        for (int k0 = 0; k0 < H; k0 += KS)
            acc[0] = MT<T>::mma(MT<T>::load(ap + k0), MT<T>::load(bp + k0), acc[0]);
        const float bias = rnd<T>(head_b[r]);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            int row = w * 32 + acc_row(e, lane);
            lgt[row * 33 + r] = rnd<T>(rnd<T>(acc[0][e]) + bias);
        }
    }
}

// Flat f32 parameter layout (mlearn_param_count): per layer W_l [in][H],
// LN scale [H], LN bias [H]; then head W [H][A+1], head bias [A+1].
struct LayoutK {
    int L, D, H, A1;  // A1 = A + 1 head outputs
    int64_t w_off[MLEARN_MAX_LAYERS], s_off[MLEARN_MAX_LAYERS], b_off[MLEARN_MAX_LAYERS];
    int64_t hw_off, hb_off, total;
};

LayoutK make_layout(const mlearn_mlp_policy& p);

}  // namespace ml
