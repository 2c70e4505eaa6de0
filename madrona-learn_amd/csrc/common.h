// Shared device helpers for the MI355X (gfx950) batched-PPO kernels.
//
// Everything here is written for CDNA4 directly: 64-lane wavefronts,
// 32x32 MFMA tiles (bf16 32x32x16 and exact-f32 32x32x2), no CUDA shims.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mlearn.h"

namespace ml {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// Error reporting (C ABI: every entry point returns an int status and records
// a thread-local message retrievable through mlearn_last_error()).
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// CU count of the current device, queried once per device id (0 when the
// query fails, e.g. without a GPU: callers then assume MI355X's 256)
int device_cus();
// hipFuncAttributeMaxDynamicSharedMemorySize of fn, set once per (function,
// device) outside graph capture; MLEARN_EHIP with a message when refused
int set_lds_attr(const void* fn, int bytes, const char* what);

#define ML_REQUIRE(cond, ...)                                   \
    do {                                                        \
        if (!(cond)) {                                          \
            ::ml::set_error(__VA_ARGS__);                       \
            return MLEARN_EINVAL;                               \
        }                                                       \
    } while (0)

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG.  Identical arithmetic on host and device;
// restated independently in oracle/ (C and numpy) and pinned by the Random123
// known-answer vectors in tests/test_oracle.py (test_philox_random123_kat).
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
#endif
}

__host__ __device__ inline u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // (the full 64-bit products: one v_mad_u64_u32 each instead of a
        // v_mul_hi_u32 + v_mul_lo_u32 pair, both quarter-rate)
        const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
        u32x4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

__host__ __device__ inline uint32_t u32x4_get(const u32x4& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// (x>>8)|1 is an odd integer < 2^24, so the product is exact: u in (0, 1).
__host__ __device__ inline float u32_to_unit(uint32_t x) {
    return (float)((x >> 8) | 1u) * 5.9604644775390625e-08f;  // 2^-24
}

// ---------------------------------------------------------------------------
// Deterministic log2 for Gumbel noise.  Only exact IEEE operations (fmaf,
// exact bit manipulation) so host C, the oracle and the GPU agree bit for bit;
// contraction is explicitly disabled.  Max rel. error ~1.2e-7 on normals.
// ---------------------------------------------------------------------------
__host__ __device__ inline float det_log2(float x) {
#pragma clang fp contract(off)
    uint32_t bits;
    __builtin_memcpy(&bits, &x, 4);
    int e = (int)((bits >> 23) & 0xffu) - 127;
    uint32_t mb = (bits & 0x007fffffu) | 0x3f800000u;
    float m;
    __builtin_memcpy(&m, &mb, 4);
    if (m > 1.41421353816986083984375f) {  // f32(sqrt 2)
        m = m * 0.5f;
        e += 1;
    }
    float f = m - 1.0f;
    float p = -1.102015972e-01f;
    p = __builtin_fmaf(p, f, 1.863120943e-01f);
    p = __builtin_fmaf(p, f, -1.910249740e-01f);
    p = __builtin_fmaf(p, f, 2.045752853e-01f);
    p = __builtin_fmaf(p, f, -2.396190464e-01f);
    p = __builtin_fmaf(p, f, 2.885688841e-01f);
    p = __builtin_fmaf(p, f, -3.606966436e-01f);
    p = __builtin_fmaf(p, f, 4.808982015e-01f);
    p = __builtin_fmaf(p, f, -7.213473320e-01f);
    p = __builtin_fmaf(p, f, 1.442695022e+00f);
    return __builtin_fmaf(f, p, (float)e);
}

// Gumbel(0,1) sample from a uniform in (0,1): -ln(-ln u).
__host__ __device__ inline float det_gumbel(float u) {
#pragma clang fp contract(off)
    const float LN2 = 0.693147182464599609375f;
    float e1 = -(det_log2(u) * LN2);  // -ln u  > 0
    return -(det_log2(e1) * LN2);
}

// Uniform for flattened logit index `j` of environment `env` at rollout step
// `step`: one Philox block yields 4 consecutive indices.
__host__ __device__ inline float sample_uniform(uint32_t k0, uint32_t k1, uint32_t env,
                                                uint64_t step, int j) {
    u32x4 c;
    c.x = (uint32_t)env;
    c.y = (uint32_t)(j >> 2);
    c.z = (uint32_t)step;
    c.w = (uint32_t)(step >> 32);
    u32x4 r = philox4x32(c, k0, k1);
    return u32_to_unit(u32x4_get(r, j & 3));
}

// ---------------------------------------------------------------------------
// bf16 helpers
// ---------------------------------------------------------------------------
__device__ inline float round_to(float x, bf16*) { return (float)(bf16)x; }
__device__ inline float round_to(float x, float*) { return x; }
template <typename T> __device__ inline float rnd(float x) { return round_to(x, (T*)nullptr); }

template <typename T> __device__ inline T cvt(float x);
template <> __device__ inline float cvt<float>(float x) { return x; }
template <> __device__ inline bf16 cvt<bf16>(float x) { return (bf16)x; }

__device__ inline float to_f32(float x) { return x; }
__device__ inline float to_f32(bf16 x) { return (float)x; }

// ---------------------------------------------------------------------------
// MFMA traits.  32x32 output tiles for both dtypes:
//   lane l, r = l & 31, h = l >> 5
//   A fragment = A[row r][k0 + h*E .. + E)      (row-major A, k contiguous)
//   B fragment = BT[col r][k0 + h*E .. + E)     (B stored transposed, k contiguous)
//   C reg i    = C[row (i&3) + 8*(i>>2) + 4*h][col r]
// ---------------------------------------------------------------------------
template <typename T> struct MT;

template <> struct MT<bf16> {
    static constexpr int E = 8;
    static constexpr int KS = 16;
    typedef bf16x8 frag;
    __device__ static frag load(const bf16* p) { return *(const bf16x8*)p; }
    __device__ static f32x16 mma(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};

template <> struct MT<float> {
    static constexpr int E = 1;
    static constexpr int KS = 2;
    typedef float frag;
    __device__ static frag load(const float* p) { return *p; }
    __device__ static f32x16 mma(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
};

__device__ inline int acc_row(int i, int lane) { return (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5); }

__device__ inline float wave_sum32(float v) {
    // reduce across the 32 lanes of a half-wave (lanes sharing lane>>5)
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    return v;
}

__device__ inline float wave_sum64(float v) {
    v = wave_sum32(v);
    v += __shfl_xor(v, 32);
    return v;
}

__device__ inline double wave_sum64d(double v) {
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

inline hipStream_t S(mlearn_stream_t s) { return (hipStream_t)s; }

}  // namespace ml
