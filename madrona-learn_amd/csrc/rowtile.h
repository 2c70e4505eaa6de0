// Row-on-lane building blocks of the fused MLP kernels (rollout step and PPO
// minibatch step).
//
// Orientation.  Every layer is computed transposed, Z^T = W^T . X^T: the
// weights are the MFMA A operand and the activations the B operand, so the
// 32x32 accumulator of a wave holds 32 output FEATURES (in its 16 registers,
// feature (q&3) + 8(q>>2) + 4h of the block for register q of lane half h)
// for 32 batch ROWS (one per lane, row = lane & 31).  Consequences:
//   - a wave owns whole rows: LayerNorm statistics are per-lane sums over the
//     lane's registers plus one exchange with lane ^ 32; no LDS, no barrier;
//   - the next layer sums over the features, i.e. over the registers, so the
//     post-activation accumulators ARE the next layer's B fragments (no LDS
//     round trip); the weights' A-operand images use the matching permuted k
//     order (img_index perm = true, include/mlearn.h);
//   - only the weights travel: contiguous 1 KiB fragment runs from L2.
// A workgroup is a set of independent waves (one tile of 32 rows each) that
// share the LayerNorm parameters staged once in LDS.
#pragma once
#include <type_traits>

#include "common.h"

namespace ml {

// ---------------------------------------------------------------------------
// A-operand weight images.  Logical Wimg[n][k] (n = output feature of the
// product, k = reduction index); perm selects the k order of B fragments that
// come straight from accumulator registers.
// ---------------------------------------------------------------------------
template <typename T> struct ImgK;
template <> struct ImgK<bf16> {
    __host__ __device__ static inline int64_t index(int n, int k, int K, bool perm) {
        const int kk = k & 15, s = k >> 4;
        const int h = perm ? (kk >> 2) & 1 : kk >> 3;
        const int e = perm ? (((kk >> 3) << 2) | (kk & 3)) : (kk & 7);
        return ((int64_t)((n >> 5) * (K >> 4) + s) * 64 + (n & 31) + 32 * h) * 8 + e;
    }
};
template <> struct ImgK<float> {
    __host__ __device__ static inline int64_t index(int n, int k, int K, bool perm) {
        int s, h;
        if (perm) {
            const int kk = k & 31;
            h = (kk >> 2) & 1;
            s = ((k >> 5) << 4) | ((kk >> 3) << 2) | (kk & 3);
        } else {
            h = k & 1;
            s = k >> 1;
        }
        return (int64_t)((n >> 5) * (K >> 1) + s) * 64 + (n & 31) + 32 * h;
    }
};
template <typename T>
__host__ __device__ inline int64_t img_index(int n, int k, int K, bool perm) {
    return ImgK<T>::index(n, k, K, perm);
}

// ---------------------------------------------------------------------------
// B fragments.
// ---------------------------------------------------------------------------
template <typename T> struct RT;
template <> struct RT<bf16> {
    static constexpr int E = 8, KS = 16, SPB = 2;  // SPB: k-steps per 32-feature block
    typedef bf16x8 frag;
    __device__ static frag zero() {
        frag f;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (bf16)0.f;
        return f;
    }
    // k-step t of a block held in accumulator layout (permuted k order)
    __device__ static frag from_acc(const f32x16& a, int t) {
        frag f;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (bf16)a[8 * t + e];
        return f;
    }
    // natural k order: elements k = 16 s + 8 h + e of a row in memory
    __device__ static frag row(const bf16* p, int s, int h) {
        return *(const bf16x8*)(p + 16 * s + 8 * h);
    }
    __device__ static frag row(const float* p, int s, int h) {
        const float4 a = *(const float4*)(p + 16 * s + 8 * h);
        const float4 b = *(const float4*)(p + 16 * s + 8 * h + 4);
        frag f = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w,
                  (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
        return f;
    }
    __device__ static void put_row(bf16* p, int s, int h, frag f) {
        *(bf16x8*)(p + 16 * s + 8 * h) = f;
    }
    // natural-order fragment from an f32 LDS row with arbitrary alignment
    __device__ static frag row_lds(const float* p, int s, int h) {
        frag f;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (bf16)p[16 * s + 8 * h + e];
        return f;
    }
};
template <> struct RT<float> {
    static constexpr int E = 1, KS = 2, SPB = 16;
    typedef float frag;
    __device__ static frag zero() { return 0.f; }
    __device__ static frag from_acc(const f32x16& a, int t) { return a[t]; }
    __device__ static frag row(const float* p, int s, int h) { return p[2 * s + h]; }
    __device__ static void put_row(float* p, int s, int h, frag f) { p[2 * s + h] = f; }
    __device__ static frag row_lds(const float* p, int s, int h) { return p[2 * s + h]; }
};

template <int NB> __device__ inline void zero_acc(f32x16 (&acc)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
}

// Wave-uniform buffer descriptor over a weight image (raw buffer loads: one
// 32-bit lane offset VGPR for every fragment, block/step offsets in SGPRs).
__device__ inline __amdgpu_buffer_rsrc_t img_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7FFFFFFF, 0x00020000);
}
template <typename T> __device__ inline typename RT<T>::frag img_load(__amdgpu_buffer_rsrc_t rs,
                                                                        int voff, int soff);
template <> __device__ inline bf16x8 img_load<bf16>(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
template <> __device__ inline float img_load<float>(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
}

// acc[nb] += sum_s Img[block nb][step s] x b[s]   (NOUT blocks of 32 outputs).
// A ring of DEPTH k-steps of A fragments is in flight ahead of the MFMAs;
// sched_barrier fences keep the compiler from sinking each load down to its
// MFMA, which would expose a full L2 round trip per MFMA at one wave/SIMD.
// nks (<= NKS) is the wave-uniform number of steps actually taken; bstride
// (default nks) the k-steps between consecutive output blocks of the image.
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_ring(f32x16 (&acc)[NOUT], const typename RT<T>::frag (&b)[NKS],
                                 int nks, const T* __restrict__ img, int lane, int bstride = -1) {
    typedef typename RT<T>::frag frag;
    const int bs = bstride < 0 ? nks : bstride;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);  // bytes per fragment run
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    frag ra[DEPTH][NOUT];
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
        if (s < nks)
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb) ra[s][nb] = img_load<T>(rs, voff, (nb * bs + s) * FB);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        if (s < nks) {
            const int sl = s + DEPTH - 1;
            if (sl < nks) {
#pragma unroll
                for (int nb = 0; nb < NOUT; ++nb)
                    ra[sl % DEPTH][nb] = img_load<T>(rs, voff, (nb * bs + sl) * FB);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb)
                acc[nb] = MT<T>::mma(ra[s % DEPTH][nb], b[s], acc[nb]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_rb(f32x16 (&acc)[NOUT], const typename RT<T>::frag (&b)[NKS],
                               const T* __restrict__ img, int lane) {
    gemm_ring<T, NOUT, NKS, DEPTH>(acc, b, NKS, img, lane);
}

// As gemm_rb, with the B fragments read from LDS (fr[s*64 + lane], written
// by the workgroup's waves) one step ahead instead of held in registers.
// bstride: k-steps between consecutive output blocks of the image (default NKS).
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_lds(f32x16 (&acc)[NOUT], const typename RT<T>::frag* fr,
                                const T* __restrict__ img, int lane, int bstride = NKS) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    frag ra[DEPTH][NOUT];
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) ra[s][nb] = img_load<T>(rs, voff, (nb * bstride + s) * FB);
    frag b = fr[lane];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const int sl = s + DEPTH - 1;
        if (sl < NKS) {
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb)
                ra[sl % DEPTH][nb] = img_load<T>(rs, voff, (nb * bstride + sl) * FB);
        }
        const frag bn = s + 1 < NKS ? fr[(s + 1) * 64 + lane] : b;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) acc[nb] = MT<T>::mma(ra[s % DEPTH][nb], b, acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
        b = bn;
    }
}

// gemm_lds in two halves: the first DEPTH-1 k-steps of A fragments issued
// early (before a barrier or a LayerNorm phase, so the weight stream is
// already flowing when the product starts), then the product itself.
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_lds_issue(typename RT<T>::frag (&ra)[DEPTH][NOUT],
                                      const T* __restrict__ img, int lane, int bstride = NKS) {
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) ra[s][nb] = img_load<T>(rs, voff, (nb * bstride + s) * FB);
}
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_lds_run(f32x16 (&acc)[NOUT], typename RT<T>::frag (&ra)[DEPTH][NOUT],
                                    const typename RT<T>::frag* fr, const T* __restrict__ img,
                                    int lane, int bstride = NKS) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    frag b = fr[lane];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const int sl = s + DEPTH - 1;
        if (sl < NKS) {
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb)
                ra[sl % DEPTH][nb] = img_load<T>(rs, voff, (nb * bstride + sl) * FB);
        }
        const frag bn = s + 1 < NKS ? fr[(s + 1) * 64 + lane] : b;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) acc[nb] = MT<T>::mma(ra[s % DEPTH][nb], b, acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
        b = bn;
    }
}

// acc[nb] += sum_s Img[block nb][step s] x row-fragment(s) with BOTH operands
// streamed: A fragments from the image and B fragments (natural k order) from
// this lane's row in memory, DEPTH k-steps of each in flight.  bstride:
// k-steps between consecutive output blocks of the image (default NKS).
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_stream(f32x16 (&acc)[NOUT], const T* __restrict__ brow,
                                   const T* __restrict__ img, int lane, int bstride = NKS) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    const int h = lane >> 5;
    frag ra[DEPTH][NOUT], rb[DEPTH];
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s) {
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) ra[s][nb] = img_load<T>(rs, voff, (nb * bstride + s) * FB);
        rb[s] = RT<T>::row(brow, s, h);
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const int sl = s + DEPTH - 1;
        if (sl < NKS) {
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb)
                ra[sl % DEPTH][nb] = img_load<T>(rs, voff, (nb * bstride + sl) * FB);
            rb[sl % DEPTH] = RT<T>::row(brow, sl, h);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb)
            acc[nb] = MT<T>::mma(ra[s % DEPTH][nb], rb[s % DEPTH], acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// gemm_lds over two concatenated products acc += Img1 . B1 + Img2 . B2 (each
// NKS k-steps, B fragments from LDS) as ONE ring of 2 NKS steps, so the
// weight prefetch does not drain between them.
template <typename T, int NOUT, int NKS, int DEPTH>
__device__ inline void gemm_lds2(f32x16 (&acc)[NOUT], const typename RT<T>::frag* fr1,
                                 const T* __restrict__ img1, const typename RT<T>::frag* fr2,
                                 const T* __restrict__ img2, int lane) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    constexpr int NS = 2 * NKS;
    const __amdgpu_buffer_rsrc_t rs1 = img_rsrc(img1), rs2 = img_rsrc(img2);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    auto ld = [&](int s, int nb) {
        return s < NKS ? img_load<T>(rs1, voff, (nb * NKS + s) * FB)
                       : img_load<T>(rs2, voff, (nb * NKS + s - NKS) * FB);
    };
    auto bf = [&](int s) { return s < NKS ? fr1[s * 64 + lane] : fr2[(s - NKS) * 64 + lane]; };
    frag ra[DEPTH][NOUT];
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) ra[s][nb] = ld(s, nb);
    frag b = bf(0);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int sl = s + DEPTH - 1;
        if (sl < NS) {
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb) ra[sl % DEPTH][nb] = ld(sl, nb);
        }
        const frag bn = s + 1 < NS ? bf(s + 1) : b;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) acc[nb] = MT<T>::mma(ra[s % DEPTH][nb], b, acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
        b = bn;
    }
}

// Whole-layer A-fragment prefetch: issue every load of a product up front
// (they land while earlier work runs), then multiply with B fragments from LDS.
template <typename T, int NOUT, int NKS>
__device__ inline void prefetch_img(typename RT<T>::frag (&a)[NKS][NOUT], const T* __restrict__ img,
                                    int lane) {
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) a[s][nb] = img_load<T>(rs, voff, (nb * NKS + s) * FB);
}
template <typename T, int NOUT, int NKS>
__device__ inline void gemm_pre_lds(f32x16 (&acc)[NOUT], const typename RT<T>::frag (&a)[NKS][NOUT],
                                    const typename RT<T>::frag* fr, int lane) {
    typedef typename RT<T>::frag frag;
    frag b = fr[lane];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const frag bn = s + 1 < NKS ? fr[(s + 1) * 64 + lane] : b;
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) acc[nb] = MT<T>::mma(a[s][nb], b, acc[nb]);
        b = bn;
    }
}

// acc[nb] += sum_s Img[block nb][step s] x row-fragment(s) for the first layer:
// B fragments (natural k order) read from this lane's row in memory (cast to
// the compute dtype), runtime step count, a plain loop so the accumulators
// stay put; the next step's A fragments and row fragment are in flight while
// the current step's MFMAs run.  copy (may be null) receives the cast row.
// Natural-order fragment s of an f32 observation row normalised as
// ObservationsEMANormalizer.normalize (moving_avg.py:79-88): (x - mu) * inv_sigma
// in f32, then the cast to the compute dtype.
template <typename T> __device__ inline typename RT<T>::frag row_norm(const float* p, const float* mu,
                                                                    const float* inv, int s, int h);
template <> __device__ inline bf16x8 row_norm<bf16>(const float* p, const float* mu, const float* inv,
                                                   int s, int h) {
    const int k = 16 * s + 8 * h;
    bf16x8 f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (bf16)((p[k + e] - mu[k + e]) * inv[k + e]);
    return f;
}
template <> __device__ inline float row_norm<float>(const float* p, const float* mu, const float* inv,
                                                   int s, int h) {
    const int k = 2 * s + h;
    return (p[k] - mu[k]) * inv[k];
}
template <typename T, typename S>
__device__ inline typename RT<T>::frag row_in(const S* p, const float* mu, const float* inv, int s,
                                              int h) {
    if constexpr (std::is_same<S, float>::value)
        if (mu) return row_norm<T>(p, mu, inv, s, h);
    return RT<T>::row(p, s, h);
}

template <typename T, int NOUT, typename S>
__device__ inline void gemm_first(f32x16 (&acc)[NOUT], const S* __restrict__ row, bool live,
                                  int nks, const T* __restrict__ img, T* copy, int lane,
                                  const float* mu = nullptr, const float* inv = nullptr) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    const int h = lane >> 5;
    constexpr int PRE =
        std::is_same<T, bf16>::value && std::is_same<S, T>::value && NOUT <= 2 ? 4 : 0;  // D <= 64
    if (PRE > 0 && nks <= PRE) {
        // short K (the observation width): every A and B fragment of the
        // product is issued before the first MFMA, so the gathered row costs
        // one memory latency instead of one per k-step
        frag ap[PRE > 0 ? PRE : 1][NOUT], bp[PRE > 0 ? PRE : 1];
#pragma unroll
        for (int s = 0; s < PRE; ++s)
            if (s < nks) {
                bp[s] = live ? row_in<T>(row, mu, inv, s, h) : RT<T>::zero();
#pragma unroll
                for (int nb = 0; nb < NOUT; ++nb) ap[s][nb] = img_load<T>(rs, voff, (nb * nks + s) * FB);
            }
#pragma unroll
        for (int s = 0; s < PRE; ++s)
            if (s < nks) {
                if (copy) RT<T>::put_row(copy, s, h, bp[s]);
#pragma unroll
                for (int nb = 0; nb < NOUT; ++nb) acc[nb] = MT<T>::mma(ap[s][nb], bp[s], acc[nb]);
            }
        return;
    }
    frag a[NOUT], an[NOUT];
    frag b = live ? row_in<T>(row, mu, inv, 0, h) : RT<T>::zero(), bn = b;
#pragma unroll
    for (int nb = 0; nb < NOUT; ++nb) a[nb] = img_load<T>(rs, voff, (nb * nks) * FB);
    for (int s = 0; s < nks; ++s) {
        if (s + 1 < nks) {
#pragma unroll
            for (int nb = 0; nb < NOUT; ++nb) an[nb] = img_load<T>(rs, voff, (nb * nks + s + 1) * FB);
            bn = live ? row_in<T>(row, mu, inv, s + 1, h) : RT<T>::zero();
        }
        if (copy) RT<T>::put_row(copy, s, h, b);
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) acc[nb] = MT<T>::mma(a[nb], b, acc[nb]);
#pragma unroll
        for (int nb = 0; nb < NOUT; ++nb) a[nb] = an[nb];
        b = bn;
    }
}

// Feature index of accumulator register q of block nb for lane half h.
__device__ inline int feat(int nb, int q, int h) { return nb * 32 + (q & 3) + 8 * (q >> 2) + 4 * h; }


// ---------------------------------------------------------------------------
// Cross-lane helpers.
// ---------------------------------------------------------------------------
#define ML_DPP(v, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xF, 0xF, true))
#define ML_SWZ(v, pat) \
    __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), pat))

// Reductions over the 32 lanes of each half-wave (result in every lane).
template <int KIND> __device__ inline float red_op(float a, float b) {
    return KIND == 2 ? fminf(a, b) : (KIND == 3 ? fmaxf(a, b) : a + b);
}

template <int D> __device__ inline float xlane(float v) {
    if constexpr (D == 1) return ML_DPP(v, 0xB1);       // quad_perm [1,0,3,2]
    else if constexpr (D == 2) return ML_DPP(v, 0x4E);  // quad_perm [2,3,0,1]
    else if constexpr (D == 8) return ML_DPP(v, 0x128); // row_ror:8 (= xor 8 in a row)
    else if constexpr (D == 4) return ML_SWZ(v, 0x101F);
    else return ML_SWZ(v, 0x401F);                       // xor 16
}
// v + (value of lane ^ 16) / (value of lane ^ 32): one v_permlane16_swap /
// v_permlane32_swap on two copies (VALU only; the builtins' two-result form
// miscompiles when both operands are the same value, so inline asm with the
// hazard padding the compiler would insert).
__device__ inline float add_xor16(float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return a + b;
}
__device__ inline float add_xor32(float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return a + b;
}

template <int KIND> __device__ inline float xor16_op(float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return red_op<KIND>(a, b);
}
template <int KIND> __device__ inline float half_reduce(float v) {
    v = red_op<KIND>(v, xlane<1>(v));
    v = red_op<KIND>(v, xlane<2>(v));
    v = red_op<KIND>(v, ML_DPP(v, 0x124));  // row_ror:4
    v = red_op<KIND>(v, xlane<8>(v));
    return xor16_op<KIND>(v);
}
// Over all 64 lanes (result in every lane).
template <int KIND> __device__ inline float wave_reduce(float v) {
    v = half_reduce<KIND>(v);
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return red_op<KIND>(a, b);
}

// Column sums: the 16 values v[q] of every lane summed over the 32 lanes
// (rows) of its half-wave, by recursive halving (each step sends half the
// values to the partner lane).  Returns the total of value index
// col_sum16_index(lane); lanes r and r ^ 16 return the same total.
template <int D, int N> __device__ inline void bfly(float (&v)[16], int lane) {
    const bool hi = (lane & D) != 0;
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
        const float a = v[i], b = v[i + N / 2];
        const float keep = hi ? b : a, send = hi ? a : b;
        v[i] = keep + xlane<D>(send);
    }
}
__device__ inline float col_sum16(float (&v)[16], int lane) {
    bfly<1, 16>(v, lane);
    bfly<2, 8>(v, lane);
    bfly<8, 4>(v, lane);
    {  // partner lane ^ 4 (same bits 0, 1, 3) within the 16-lane row:
       // row_ror:N delivers lane i - N, so bit-2-clear lanes take ror:12 (i + 4)
        const bool hi = (lane & 4) != 0;
        const float a = v[0], b = v[1];
        const float keep = hi ? b : a, send = hi ? a : b;
        const float r4 = ML_DPP(send, 0x124), r12 = ML_DPP(send, 0x12C);
        v[0] = keep + (hi ? r4 : r12);
    }
    return add_xor16(v[0]);
}
__device__ inline int col_sum16_index(int lane) {
    return ((lane & 1) << 3) | ((lane & 2) << 1) | ((lane >> 2) & 2) | ((lane >> 2) & 1);
}

// Sum of a per-row value over both lane halves (features 4h-interleaved).
__device__ inline float sum_halves(float v) { return add_xor32(v); }

// Order LDS traffic between the lanes of one wave.
__device__ inline void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Store 4 consecutive elements (one 8-byte bf16 / 16-byte f32 store).
__device__ inline void store4(bf16* p, float a, float b, float c, float d) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
    *(bf16x4*)p = v;
}
__device__ inline void store4(float* p, float a, float b, float c, float d) {
    *(float4*)p = make_float4(a, b, c, d);
}
// Load 4 consecutive elements as f32.
__device__ inline float4 load4(const bf16* p) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const bf16x4 v = *(const bf16x4*)p;
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ inline float4 load4(const float* p) { return *(const float4*)p; }
__device__ inline float f4get(const float4& v, int j) {
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// Gate activations on the hardware exp / reciprocal (v_exp_f32, v_rcp_f32,
// ~1 ulp each) instead of IEEE division and libm tanhf: the cell is the
// VALU-heaviest part of the LSTM scans (rocprofv3 PMC: 32 VALU per MFMA in
// the forward scan with libm tanhf).  Both saturate correctly (exp -> inf
// gives rcp -> 0).  tanh uses its odd Taylor series below |x| < 1/8, where
// 1 - 2 / (1 + e^2x) would cancel.
__device__ inline float sigmoidf(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ inline float tanh_fast(float x) {
    const float x2 = x * x;
    const float series = x * (1.0f + x2 * (-1.0f / 3 + x2 * (2.0f / 15 + x2 * (-17.0f / 315))));
    const float big = 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x));
    return fabsf(x) < 0.125f ? series : big;
}

// flax OptimizedLSTMCell step (rnn.py:28-41) on one (row, unit) from the
// f32 gate pre-activations (x.Wi + h.Wh + bias): gate activations, c' and h'
// rounded to the compute dtype (precision contract: oracle/lstm_ref.py).
struct CellOut {
    float i, f, g, o, c, h;
};
template <typename T>
__device__ inline CellOut lstm_cell_fwd(float pi, float pf, float pg, float po, float cin) {
    CellOut r;
    r.i = rnd<T>(sigmoidf(pi));
    r.f = rnd<T>(sigmoidf(pf));
    r.g = rnd<T>(tanh_fast(pg));
    r.o = rnd<T>(sigmoidf(po));
    r.c = rnd<T>(r.f * cin + r.i * r.g);
    r.h = rnd<T>(r.o * tanh_fast(r.c));
    return r;
}

// ---------------------------------------------------------------------------
// Pair-packed blocks: the 16 accumulator values of one 32-feature block as 8
// words of two values in the compute dtype (bf16x2 / float2).  Packing is the
// compute-dtype rounding point; unpacked pairs feed packed f32 math
// (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32); the words are directly the
// next product's B fragments and the 4-feature row-major stores.
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

template <typename T> struct Pk;
template <> struct Pk<bf16> {
    typedef uint32_t word;
    __device__ static word pack(float a, float b) {
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        const bf16x2 v = {(bf16)a, (bf16)b};
        return __builtin_bit_cast(uint32_t, v);
    }
    __device__ static f2 unpack(word w) {
        return f2{__builtin_bit_cast(float, w << 16), __builtin_bit_cast(float, w & 0xffff0000u)};
    }
    // k-step t (0, 1) of the block: elements 8t .. 8t+7 = words 4t .. 4t+3
    __device__ static bf16x8 frag(const word (&w)[8], int t) {
        typedef __attribute__((ext_vector_type(4))) uint32_t u4;
        const u4 v = {w[4 * t], w[4 * t + 1], w[4 * t + 2], w[4 * t + 3]};
        return __builtin_bit_cast(bf16x8, v);
    }
    // features 4g .. 4g+3 of the block (words 2g, 2g+1) -> 8-byte store
    __device__ static void store4(bf16* p, word a, word b) {
        typedef __attribute__((ext_vector_type(2))) uint32_t u2;
        *(u2*)p = u2{a, b};
    }
};
template <> struct Pk<float> {
    typedef f2 word;
    __device__ static word pack(float a, float b) { return f2{a, b}; }
    __device__ static f2 unpack(word w) { return w; }
    // k-step t (0 .. 15) of the block: element t
    __device__ static float frag(const word (&w)[8], int t) { return w[t >> 1][t & 1]; }
    __device__ static void store4(float* p, word a, word b) {
        *(float4*)p = make_float4(a.x, a.y, b.x, b.y);
    }
};

// Dense output -> compute dtype (packed) and the lane's partial row sums.
template <typename T, int NBW>
__device__ inline void ln_pack_stats(const f32x16 (&acc)[NBW], typename Pk<T>::word (&zw)[NBW][8],
                                     f2 (&x2)[NBW][8], float& sum, float& sq) {
    f2 s = {0.f, 0.f}, q = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            zw[i][k] = Pk<T>::pack(acc[i][2 * k], acc[i][2 * k + 1]);
            x2[i][k] = Pk<T>::unpack(zw[i][k]);
            s += x2[i][k];
            q = x2[i][k] * x2[i][k] + q;
        }
    sum = s.x + s.y;
    sq = q.x + q.y;
}

// LayerNorm (x - mean) * (rstd * scale) + bias, ReLU, rounded to the compute
// dtype (models.py:46-56); gm = LDS [2][H] scale | bias of the layer; blocks
// nb0 .. nb0+NBW-1.
template <typename T, int NBW>
__device__ inline void ln_apply(const f2 (&x2)[NBW][8], float mean, float rstd, const float* gm,
                                int H, int nb0, int h, typename Pk<T>::word (&aw)[NBW][8]) {
    const f2 m2 = {mean, mean}, r2 = {rstd, rstd};
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f0 = (nb0 + i) * 32 + 8 * g + 4 * h;
            const float4 G = *(const float4*)(gm + f0), B = *(const float4*)(gm + H + f0);
            // explicit fma: the weight-gradient launch recomputes A_0 from Z_0
            // with the same operations (ln_act), bit for bit
            const f2 y0 = __builtin_elementwise_fma(x2[i][2 * g] - m2, r2 * f2{G.x, G.y}, f2{B.x, B.y});
            const f2 y1 = __builtin_elementwise_fma(x2[i][2 * g + 1] - m2, r2 * f2{G.z, G.w}, f2{B.z, B.w});
            aw[i][2 * g] = Pk<T>::pack(fmaxf(y0.x, 0.f), fmaxf(y0.y, 0.f));
            aw[i][2 * g + 1] = Pk<T>::pack(fmaxf(y1.x, 0.f), fmaxf(y1.y, 0.f));
        }
}

// Scalar form of ln_apply for one element (same operations, same bits).
__device__ inline float ln_act(float x, float mean, float rstd, float g, float b) {
    return fmaxf(__builtin_fmaf(x - mean, rstd * g, b), 0.f);
}

// Lane-private LDS spill of one accumulator block (16 values) in the compute
// dtype: CH 16-byte chunks, chunk-major over the 64 lanes (conflict-free).
template <typename T> struct ZIO {
    static constexpr int VPC = 16 / sizeof(T), CH = 16 / VPC;
    typedef __attribute__((ext_vector_type(4))) uint32_t u4;
    __device__ static void put(u4* base, int lane, const f32x16& a) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            union {
                T v[VPC];
                u4 q;
            } u;
#pragma unroll
            for (int j = 0; j < VPC; ++j) u.v[j] = cvt<T>(a[c * VPC + j]);
            base[c * 64 + lane] = u.q;
        }
    }
    __device__ static void get(const u4* base, int lane, float (&z)[16]) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            union {
                T v[VPC];
                u4 q;
            } u;
            u.q = base[c * 64 + lane];
#pragma unroll
            for (int j = 0; j < VPC; ++j) z[c * VPC + j] = to_f32(u.v[j]);
        }
    }
};

struct PolicyK {
    int D, H, L, K, A;
    int CB, HC;  // critic outputs (1: scalar, else two-hot bins); head width (32 or 96)
    const float* obs_mu;   // ObservationsEMANormalizer estimates (null: plain cast)
    const float* obs_inv;
    float* obs_stats;      // per-step per-tile {mean, M2} of the raw observations
    int64_t obs_tiles;
    int obs_steps;
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

// LSTM weights of a recurrent policy (mlearn_lstm); bias is the f32 master.
struct LstmK {
    const void* wi_perm;
    const void* wi_nat;
    const void* wh_nat;
    const void* w_bwd;
    const void* head_t_nat;
    const float* bias;
};
inline LstmK make_lstm_k(const mlearn_lstm& r) {
    return LstmK{r.wi_perm, r.wi_nat, r.wh_nat, r.w_bwd, r.head_t_nat, r.bias};
}
int validate_policy(const mlearn_mlp_policy* p);

// Partial head sums per output block of the fused kernels: with W waves and
// head width HC, the K of each 32-column block is split over W / (HC/32)
// waves (W for HC = 32).
template <int HC, int W> constexpr int head_parts() {
    return HC == 32 ? W : (W / (HC / 32) > 0 ? W / (HC / 32) : 1);
}

// Head width of a policy: actor logits + critic outputs, padded to 32 or 96.
inline int head_cols(const mlearn_mlp_policy& p) {
    return p.actions.num_logits + p.critic_bins <= MLEARN_HEAD_COLS ? MLEARN_HEAD_COLS
                                                                   : MLEARN_HEAD_COLS_MAX;
}

// Flat f32 parameter layout (mlearn_param_count): per layer W_l [in][H],
// LN scale [H], LN bias [H]; then head W [H][A1], head bias [A1] (A1 = actor
// logits + critic outputs).
// Recurrent policies append, after the MLP layout padded to 64 floats, the
// LSTM segment Wi [H][4H], Wh [H][4H], bias [4H] (lstm_H = 0: no segment).
struct LayoutK {
    int L, D, H, A1;  // A1 = A + critic outputs
    int HC;           // head width (padded)
    int64_t w_off[MLEARN_MAX_LAYERS], s_off[MLEARN_MAX_LAYERS], b_off[MLEARN_MAX_LAYERS];
    int64_t hw_off, hb_off, total;
    int64_t mlp_total, lstm_off;  // end of the MLP parameters, start of the LSTM segment
    int lstm_H;
};

// Projection slots: 2l = trunk kernel W_l, 2l + 1 = LayerNorm l, then (LSTM)
// 2L + 4 * which + gate = gate kernel (which 0: Wi, 1: Wh).
constexpr int kMaxSlots = 2 * MLEARN_MAX_LAYERS + 8;

LayoutK make_layout(const mlearn_mlp_policy& p);
LayoutK make_layout_lstm(const mlearn_mlp_policy& p, const mlearn_lstm& r);
int validate_lstm(const mlearn_mlp_policy* p, const mlearn_lstm* r);

}  // namespace ml
