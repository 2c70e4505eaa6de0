// Row-tile building blocks of the fused MLP kernels (rollout step and PPO
// minibatch step).
//
// A workgroup of W waves owns a tile of ROWS = 32*RB rows.  Wave w owns row
// block rb = w % RB and column group cg = w / RB (CG = W / RB groups); its
// output column blocks are cb = cg + CG*i, i < NB = (N/32) / CG.  Each 32x32
// output block is computed by exactly one wave, the wave's A fragment is
// reused across its NB blocks, and many small waves per CU hide the L2
// latency of the B-fragment loads and the VALU-heavy LayerNorm phases of the
// other tiles resident on the CU.
//
// A operand: the tile's activations in LDS, row-major [ROWS][ld] (ld = K + 16
// B of padding: rows shift by 4 banks, so the 16 lanes of a ds_read_b128
// group hit distinct banks).  B operand: the layer's weights [N][K] (Dense
// kernel transposed), 16 B per lane straight from L2 (the whole weight set is
// <= 180 KB and stays L2-resident).
#pragma once
#include "common.h"

namespace ml {

template <typename T> struct Pad { static constexpr int v = 16 / sizeof(T); };

template <int NB> __device__ inline void zero_acc(f32x16 (&acc)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
}

// LDS-only workgroup barrier: orders LDS traffic between the waves without
// draining outstanding global stores.
__device__ inline void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// acc[i] += act[rb*32 .. +32][0..K) x Bt[cb_i*32 .. +32][0..K)^T,
// cb_i = cg + CG*i, Bt given as a fragment-order image (frag_index); blocks
// with cb_i*32 >= N are skipped.  No barriers.
template <typename T, int NB, int CG>
__device__ inline void gemm_direct(f32x16 (&acc)[NB], const T* act, int lda, int rb,
                                   const T* __restrict__ Bp, int K, int N, int cg, int lane) {
    constexpr int E = MT<T>::E, KS = MT<T>::KS;
    const int r = lane & 31, h = lane >> 5;
    const T* ap = act + (rb * 32 + r) * lda + h * E;
    const T* bp[NB];
    bool on[NB];
    const int nks = K / KS;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int cb = cg + CG * i;
        on[i] = cb * 32 < N;
        bp[i] = Bp + ((int64_t)(on[i] ? cb : 0) * nks * 64 + lane) * E;
    }
#pragma unroll 4
    for (int ks = 0; ks < nks; ++ks) {
        typename MT<T>::frag a = MT<T>::load(ap + ks * KS);
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (on[i]) acc[i] = MT<T>::mma(a, MT<T>::load(bp[i] + ks * 64 * E), acc[i]);
    }
}

// DPP reductions over the 16 lanes of a DPP row (result in every lane), then
// over the 32 lanes of a half-wave (ds_swizzle xor 16: no LDS memory access).
template <int KIND> __device__ inline float red_op(float a, float b) {
    return KIND == 2 ? fminf(a, b) : (KIND == 3 ? fmaxf(a, b) : a + b);
}
template <int KIND> __device__ inline float half_reduce(float v) {
#define ML_DPP(ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xF, 0xF, true))
    v = red_op<KIND>(v, ML_DPP(0xB1));   // quad_perm [1,0,3,2]
    v = red_op<KIND>(v, ML_DPP(0x4E));   // quad_perm [2,3,0,1]
    v = red_op<KIND>(v, ML_DPP(0x124));  // row_ror:4
    v = red_op<KIND>(v, ML_DPP(0x128));  // row_ror:8
#undef ML_DPP
    v = red_op<KIND>(v, __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(
                                                      __builtin_bit_cast(int, v), 0x1F | (0x10 << 10))));
    return v;
}
__device__ inline float half_sum(float v) { return half_reduce<0>(v); }

// Row totals over all output columns of the tile: s[e], q[e] hold this lane's
// partial sums over its column blocks for the rows of its 16 accumulator
// registers; on return the totals.  red: LDS [W][ROWS][2] floats.  Contains
// one LDS barrier.
template <int RB, int CG>
__device__ inline void row_reduce2(float (&s)[16], float (&q)[16], float* red, int w, int lane) {
    constexpr int ROWS = 32 * RB;
    const int rb = w % RB;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        s[e] = half_sum(s[e]);
        q[e] = half_sum(q[e]);
    }
    if ((lane & 31) == 0) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = rb * 32 + acc_row(e, lane);
            red[(w * ROWS + row) * 2 + 0] = s[e];
            red[(w * ROWS + row) * 2 + 1] = q[e];
        }
    }
    lds_barrier();
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int row = rb * 32 + acc_row(e, lane);
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int g = 0; g < CG; ++g) {  // fixed order over column groups
            a += red[((g * RB + rb) * ROWS + row) * 2 + 0];
            b += red[((g * RB + rb) * ROWS + row) * 2 + 1];
        }
        s[e] = a;
        q[e] = b;
    }
}

// Store 4 consecutive elements (one 8-byte bf16 / 16-byte f32 store).
__device__ inline void store4(bf16* p, float a, float b, float c, float d) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
    *(bf16x4*)p = v;
}
__device__ inline void store4(float* p, float a, float b, float c, float d) {
    *(float4*)p = make_float4(a, b, c, d);
}

// Transposed copy of a row-major LDS tile src[ROWS][ld] (ncol columns) into
// the feature-major HBM array XT[col][row0 + row] (ld_t = padded row count),
// 16 B per store: every group of 16/sizeof(T) consecutive rows of a column is
// one store, so a wave writes whole column segments.  Rows >= M are written
// as zeros (padding of the weight-gradient K axis).
template <typename T, int ROWS, int THREADS>
__device__ inline void store_tile_transposed(const T* src, int ld, int ncol, T* XT, int64_t ld_t,
                                             int64_t row0, int64_t M, int tid) {
    constexpr int V = 16 / sizeof(T);
    constexpr int GPC = ROWS / V;  // 16-B groups per column
    typedef __attribute__((ext_vector_type(4))) uint32_t u4;
    for (int idx = tid; idx < ncol * GPC; idx += THREADS) {
        const int col = idx / GPC, g = idx - col * GPC;
        union {
            T v[V];
            u4 q;
        } u;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int row = g * V + j;
            u.v[j] = row0 + row < M ? src[row * ld + col] : cvt<T>(0.f);
        }
        *(u4*)(XT + (int64_t)col * ld_t + row0 + g * V) = u.q;
    }
}

// LayerNorm + ReLU epilogue (models.py:46-56 / flax 0.8.1 LayerNorm, fast
// variance, eps 1e-6) on a wave's accumulators, writing the compute-dtype
// activation into act (LDS).  mean/rstd per accumulator register are
// returned when the pointers are given.
template <typename T, int NB, int RB, int CG>
__device__ inline void ln_relu_epilogue(f32x16 (&acc)[NB], const float* __restrict__ gamma,
                                        const float* __restrict__ beta, T* act, int ld,
                                        float* red, int w, int lane, int H, float* mean_out,
                                        float* rstd_out) {
    const int rb = w % RB, cg = w / RB, r = lane & 31;
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
    row_reduce2<RB, CG>(s, q, red, w, lane);
    const float invH = 1.0f / (float)H;
    float g[NB], bt[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int col = (cg + CG * i) * 32 + r;
        g[i] = gamma[col];
        bt[i] = beta[col];
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int row = rb * 32 + acc_row(e, lane);
        const float mean = s[e] * invH;
        const float var = fmaxf(q[e] * invH - mean * mean, 0.f);
        const float rstd = rsqrtf(var + 1e-6f);
        if (mean_out) {
            mean_out[e] = mean;
            rstd_out[e] = rstd;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int col = (cg + CG * i) * 32 + r;
            const float y = fmaxf(rnd<T>((acc[i][e] - mean) * (rstd * g[i]) + bt[i]), 0.f);
            act[row * ld + col] = cvt<T>(y);
        }
    }
}

// Heads: lgt[ROWS][33] = rnd(rnd(act . head_t^T) + rnd(bias)), f32 (dists.py:22,
// models.py:154).  Waves with cg == 0 hold the single 32-column output block.
template <typename T, int RB, int CG>
__device__ inline void heads_to_lds(const T* act, int ld, const T* __restrict__ head_t,
                                    const float* __restrict__ head_b, int H, float* lgt, int w,
                                    int lane) {
    const int rb = w % RB, cg = w / RB;
    if (cg == 0) {
        f32x16 acc[1];
        zero_acc<1>(acc);
        gemm_direct<T, 1, 1>(acc, act, ld, rb, head_t, H, MLEARN_HEAD_COLS, 0, lane);
        const int r = lane & 31;
        const float bias = rnd<T>(head_b[r]);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = rb * 32 + acc_row(e, lane);
            lgt[row * 33 + r] = rnd<T>(rnd<T>(acc[0][e]) + bias);
        }
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

// Flat f32 parameter layout (mlearn_param_count): per layer W_l [in][H],
// LN scale [H], LN bias [H]; then head W [H][A+1], head bias [A+1].
struct LayoutK {
    int L, D, H, A1;  // A1 = A + 1 head outputs
    int64_t w_off[MLEARN_MAX_LAYERS], s_off[MLEARN_MAX_LAYERS], b_off[MLEARN_MAX_LAYERS];
    int64_t hw_off, hb_off, total;
};

LayoutK make_layout(const mlearn_mlp_policy& p);

}  // namespace ml
