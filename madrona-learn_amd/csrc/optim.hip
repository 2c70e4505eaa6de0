// Optimizer step (ppo.py:283-338):
//   optax.chain(clip_by_global_norm(max_grad_norm), adam(lr))  (ppo.py:84-90)
//   -> weight-norm re-projection of every backbone kernel to its initial
//      Frobenius norm (ppo.py:303-310, train_state.py:413-423)
//   -> LayerNorm renorm so that |scale|^2 + |bias|^2 = features (ppo.py:312-338)
//   -> refresh of the compute-dtype weight copies the MLP kernels read
//      (transposed [out][in] and [in][out] images, padded head).
// Three short launches over the flat 90K-float parameter vector; global
// reductions go through fixed-order double partials that every consumer
// block re-reduces identically (deterministic, no finishing launches).

#include "common.h"
#include "rowtile.h"

namespace ml {

constexpr int kNormBlocks = 64;

struct CopiesK {
    void* wt[MLEARN_MAX_LAYERS];
    void* w[MLEARN_MAX_LAYERS];
    void* head_t;
    void* head;
    float* head_b;
    // recurrent policies (null otherwise); see mlearn_lstm in include/mlearn.h
    void* wi_perm;
    void* wi_nat;
    void* wh_nat;
    void* w_bwd;
    void* head_t_nat;
};

static CopiesK make_copies(const mlearn_mlp_policy& p, const mlearn_lstm* r = nullptr) {
    CopiesK c{};
    for (int l = 0; l < MLEARN_MAX_LAYERS; ++l) {
        c.wt[l] = (void*)p.w_t[l];
        c.w[l] = (void*)p.w[l];
    }
    c.head_t = (void*)p.head_t;
    c.head = (void*)p.head;
    c.head_b = (float*)p.head_bias;
    if (r) {
        c.wi_perm = (void*)r->wi_perm;
        c.wi_nat = (void*)r->wi_nat;
        c.wh_nat = (void*)r->wh_nat;
        c.w_bwd = (void*)r->w_bwd;
        c.head_t_nat = (void*)r->head_t_nat;
    }
    return c;
}

__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ g, int64_t n,
                                                            double* part) {
#pragma clang fp contract(off)  // (one rounding per operation: optim_fused_kernel's bits)
    __shared__ double sh[4];
    double s = 0;
    // eight of this thread's strided elements in flight at a time, summed in index order
    const int64_t st = (int64_t)gridDim.x * 256;
    for (int64_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += 8 * st) {
        float x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = i0 + u * st < n ? g[i0 + u * st] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * st < n) {
                const double v = x[u];
                s += v * v;
            }
    }
    s = wave_sum64d(s);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
}


// tensor id of parameter p for the projection partials: 2*l = W_l, 2*l+1 =
// LN_l, 2L + 4*which + gate = LSTM gate kernel, -1 = not projected
__device__ inline int proj_slot(const LayoutK& k, int64_t p) {
    if (k.lstm_H && p >= k.lstm_off) {
        const int64_t q = p - k.lstm_off, H = k.lstm_H;
        if (q >= 8 * H * H) return -1;  // LSTM bias
        const int which = (int)(q / (4 * H * H));
        const int gate = (int)((q % (4 * H)) / H);
        return 2 * k.L + 4 * which + gate;
    }
    if (p >= k.hw_off) return -1;
    int l = k.L - 1;
    while (l > 0 && p < k.w_off[l]) --l;
    return p < k.s_off[l] ? 2 * l : 2 * l + 1;
}

// one parameter per thread up to 512 x 256 parameters (the headline MLP's
// 89 883 take 352 blocks), so each thread's update is one memory latency
// (adam 7.1 -> 6.0 us at the headline config)
#ifndef ML_ADAM_BLOCKS
#define ML_ADAM_BLOCKS 512
#endif
constexpr int kAdamBlocks = ML_ADAM_BLOCKS;

// Global gradient norm from npart partials (every block computes it the same
// way: thread i sums partials i, i + 256, ..., then a fixed butterfly).
__device__ inline float global_norm(const double* gpart, int64_t npart) {
    __shared__ double gn_red[4];
    __shared__ float gn_sh;
    // up to 8 partials per thread loaded together (fixed summation order)
    double t = 0.0;
    for (int64_t i0 = threadIdx.x; i0 < npart; i0 += 8 * 256) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = i0 + (int64_t)u * 256;
            v[u] = i < npart ? gpart[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) t += v[u];
    }
    t = wave_sum64d(t);
    if ((threadIdx.x & 63) == 0) gn_red[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0)
        gn_sh = sqrtf((float)((gn_red[0] + gn_red[1]) + (gn_red[2] + gn_red[3])));  // f32 norm
    __syncthreads();
    return gn_sh;
}

// clip_by_global_norm + one Adam step of one parameter (optax 0.1.9
// scale_by_adam with bias correction).  Contraction off: one rounding per
// operation as written, so every kernel that calls this (adam_kernel,
// optim_fused_kernel) produces the same bits whatever the compiler's
// vectorisation of the caller (an fma's choice of which product to keep
// unrounded otherwise differs between the two kernels' schedules).
__device__ __forceinline__ float adam_param(float g, float m_old, float v_old, float q_old, float gn,
                                            float max_norm, float b1, float b2, float eps, float lr,
                                            int count, float& mm, float& vv) {
#pragma clang fp contract(off)
    if (!(gn < max_norm)) g = (g / gn) * max_norm;  // clip_by_global_norm
    mm = (1.f - b1) * g + b1 * m_old;
    vv = (1.f - b2) * (g * g) + b2 * v_old;
    const float mhat = mm / (1.f - powf(b1, (float)count));
    const float vhat = vv / (1.f - powf(b2, (float)count));
    const float u = mhat / (sqrtf(vhat) + eps);
    return q_old + (-lr) * u;
}

template <int PRE>
__global__ __launch_bounds__(256) void adam_kernel(LayoutK Lk, float* __restrict__ params,
                                                   const float* __restrict__ grads,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   const int32_t* step, const double* gpart,
                                                   int64_t npart, float lr, float b1, float b2, float eps,
                                                   float max_norm, double* proj_part) {
#pragma clang fp contract(off)  // (one rounding per operation: optim_fused_kernel's bits)
    // grid-stride over the parameters with at most kAdamBlocks blocks, so the
    // projection reduces a short, fixed list of per-block partials
    __shared__ float sh[4][kMaxSlots];
    const int nslot = 2 * Lk.L + (Lk.lstm_H ? 8 : 0);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < 4 * kMaxSlots) sh[threadIdx.x / kMaxSlots][threadIdx.x % kMaxSlots] = 0.f;
    // this thread's first PRE parameters (grid-stride) are in flight while
    // the global norm is reduced: the headline MLP has one per thread, the
    // recurrent layouts up to five (one loop that loads as it goes waits a
    // memory latency per parameter); PRE = the launch's count rounded up to
    // a power of two
    constexpr int kAdamPre = PRE;
    const int64_t p0 = blockIdx.x * (int64_t)256 + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * 256;
    float gq[kAdamPre], mq[kAdamPre], vq[kAdamPre], qq[kAdamPre];
#pragma unroll
    for (int u = 0; u < kAdamPre; ++u) {
        const int64_t p = p0 + u * stride;
        gq[u] = mq[u] = vq[u] = qq[u] = 0.f;
        if (p < Lk.total) {
            gq[u] = grads[p];
            mq[u] = m[p];
            vq[u] = v[p];
            qq[u] = params[p];
        }
    }
    const int count = step[0] + 1;
    const float gn = global_norm(gpart, npart);  // (its barriers also order the sh zeroing)
    auto update = [&](int64_t p, float g, float m_old, float v_old, float q_old) {
        float contrib = 0.f;
        int slot = -2;
        // (recurrent layouts: the alignment padding before the LSTM segment is not a parameter)
        const bool pad = Lk.lstm_H && p >= Lk.mlp_total && p < Lk.lstm_off;
        if (p < Lk.total && !pad) {
            float mm, vv;
            const float np = adam_param(g, m_old, v_old, q_old, gn, max_norm, b1, b2, eps, lr,
                                        count, mm, vv);
            m[p] = mm;
            v[p] = vv;
            params[p] = np;
            slot = proj_slot(Lk, p);
            contrib = np * np;
        }
        // per-block partial sums of squares per projection slot (a wave's 64
        // parameters span at most two slots: skip the absent ones)
        for (int s = 0; s < nslot; ++s) {
            if (!__any(slot == s)) continue;
            float x = slot == s ? contrib : 0.f;
            x = wave_sum64(x);
            if (lane == 0) sh[w][s] += x;
        }
    };
#pragma unroll
    for (int u = 0; u < kAdamPre; ++u) {
        const int64_t p = p0 + u * stride;
        if (p - threadIdx.x >= Lk.total) break;  // (block-uniform)
        update(p, gq[u], mq[u], vq[u], qq[u]);
    }
    for (int64_t p = p0 + kAdamPre * stride; p - threadIdx.x < Lk.total; p += stride) {
        const bool in = p < Lk.total;
        update(p, in ? grads[p] : 0.f, in ? m[p] : 0.f, in ? v[p] : 0.f, in ? params[p] : 0.f);
    }
    __syncthreads();
    if (threadIdx.x < nslot) {
        int s = threadIdx.x;
        proj_part[blockIdx.x * (int64_t)nslot + s] =
            ((double)sh[0][s] + sh[1][s]) + ((double)sh[2][s] + sh[3][s]);
    }
}

template <typename T>
__device__ inline void write_copies(const LayoutK& Lk, const CopiesK& C, int64_t p, float val) {
    const int H = Lk.H;
    if (Lk.lstm_H && p >= Lk.mlp_total) {
        if (p < Lk.lstm_off) return;  // alignment padding
        const int64_t q = p - Lk.lstm_off, HH = Lk.lstm_H;
        if (q >= 8 * HH * HH) return;  // bias: read in f32 from the master params
        const int which = (int)(q / (4 * HH * HH));
        const int64_t r = q - which * 4 * HH * HH;
        const int k = (int)(r / (4 * HH)), n = (int)(r % (4 * HH));  // input unit, gate column
        const int gate = n / (int)HH, u = n % (int)HH;
        const int nu = (u >> 5) * 128 + gate * 32 + (u & 31);       // unit-block gate order
        const T v = cvt<T>(val);
        if (which == 0) {
            ((T*)C.wi_perm)[img_index<T>(nu, k, (int)HH, true)] = v;
            ((T*)C.wi_nat)[img_index<T>(nu, k, (int)HH, false)] = v;
        } else {
            ((T*)C.wh_nat)[img_index<T>(nu, k, (int)HH, false)] = v;
        }
        ((T*)C.w_bwd)[img_index<T>(which * (int)HH + k, n, 4 * (int)HH, false)] = v;
        return;
    }
    if (p >= Lk.hb_off) {
        C.head_b[p - Lk.hb_off] = val;
    } else if (p >= Lk.hw_off) {
        int64_t q = p - Lk.hw_off;
        int c = (int)(q / Lk.A1), k = (int)(q % Lk.A1);
        ((T*)C.head_t)[img_index<T>(k, c, H, true)] = cvt<T>(val);
        ((T*)C.head)[img_index<T>(c, k, Lk.HC, false)] = cvt<T>(val);
        if (C.head_t_nat) ((T*)C.head_t_nat)[img_index<T>(k, c, H, false)] = cvt<T>(val);
    } else {
        int l = Lk.L - 1;
        while (l > 0 && p < Lk.w_off[l]) --l;
        if (p < Lk.s_off[l]) {
            const int in = l == 0 ? Lk.D : H;
            int64_t q = p - Lk.w_off[l];
            int i = (int)(q / H), j = (int)(q % H);
            ((T*)C.wt[l])[img_index<T>(j, i, in, l > 0)] = cvt<T>(val);
            if (l > 0) ((T*)C.w[l])[img_index<T>(i, j, H, true)] = cvt<T>(val);
        }
        // LayerNorm scale/bias are read in f32 straight from the master params.
    }
}

template <typename T, int NS>
__global__ __launch_bounds__(256) void project_kernel(LayoutK Lk, CopiesK C, float* params,
                                                      const float* init_norms, const double* ppart,
                                                      int nblk, int norm_params, int norm_ln,
                                                      int32_t* step) {
#pragma clang fp contract(off)  // (one rounding per operation: optim_fused_kernel's bits)
    // per-slot sums of squares of the updated tensors (ppo.py:303-338), the
    // same fixed-order tree in every block
    __shared__ double red[4][kMaxSlots];
    __shared__ float sq[kMaxSlots];
    constexpr int nslot = NS;  // = 2 L (+ 8 recurrent): the launch picks the instantiation
    const int64_t p = blockIdx.x * (int64_t)256 + threadIdx.x;
    const float val0 = p < Lk.total ? params[p] : 0.f;  // in flight under the slot reduction
    // every slot's partials of this thread (blocks tid, tid + 256, ...) loaded
    // together, then summed per slot in block order (one loop per slot would
    // wait for each load before issuing the next)
    double t[NS];
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) t[sl] = 0;
    for (int b0 = threadIdx.x; b0 < nblk; b0 += 512) {
        double x[2][NS];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int sl = 0; sl < NS; ++sl) {
                const int b = b0 + 256 * u;
                x[u][sl] = (b < nblk && sl < nslot) ? ppart[(int64_t)b * nslot + sl] : 0.0;
            }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int sl = 0; sl < NS; ++sl)
                if (b0 + 256 * u < nblk && sl < nslot) t[sl] += x[u][sl];
    }
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
        if (sl >= nslot) break;
        const double tt = wave_sum64d(t[sl]);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][sl] = tt;
    }
    __syncthreads();
    if (threadIdx.x < nslot) {
        const int sl = threadIdx.x;
        sq[sl] = (float)(((red[0][sl] + red[1][sl]) + red[2][sl]) + red[3][sl]);
    }
    __syncthreads();
    if (p == 0 && step) step[0] += 1;
    if (p >= Lk.total) return;
    float val = val0;
    const int slot = proj_slot(Lk, p);
    if (slot >= 2 * Lk.L) {  // LSTM gate kernel (ppo.py:303-310 on each ii..ho kernel)
        if (norm_params) val = (init_norms[Lk.L + slot - 2 * Lk.L] * val) / sqrtf(sq[slot]);
        params[p] = val;
    } else if (slot >= 0) {
        const int l = slot >> 1;
        if ((slot & 1) == 0) {
            if (norm_params) val = (init_norms[l] * val) / sqrtf(sq[slot]);  // ppo.py:307
        } else if (norm_ln) {
            // sqrt(F / (b.b + s.s)) (ppo.py:324-325)
            val = sqrtf((float)Lk.H / sq[slot]) * val;
        }
        params[p] = val;
    }
    write_copies<T>(Lk, C, p, val);
}

// ---------------------------------------------------------------------------
// The optimizer chain as ONE launch (round 6): [global-norm partials] ->
// clip + Adam -> projection + compute images.  The 2-3 launches above each
// cost a kernel boundary plus a dependent load chain; here the seams are an
// in-launch grid barrier whose only payload is the per-block partials (a few
// KB): every workgroup keeps its own parameters in registers from the Adam
// update to the projection, so no parameter crosses a workgroup.
//
// Bit-identical to the split chain: a workgroup of 256 * VB threads runs VB
// "virtual" adam_kernel blocks (virtual block vb = VB * blockIdx + tid / 256,
// the same grid-stride parameter mapping over ablk virtual blocks), writes
// the same per-(virtual block, slot) partials, and its first 256 threads
// replay global_norm / sumsq_partial_kernel / project_kernel's reductions in
// their fixed orders.
//
// Hand-off protocol (MI355X_MICROARCH.md, hand-off table row 1, "one lane of
// each storing workgroup ... agent-scope atomic add"): partials are stored
// with agent-scope (sc1) atomic stores; every wave waits s_waitcnt vmcnt(0);
// a workgroup barrier; ONE lane adds to a counter shard (blockIdx % 8) with an
// agent-scope atomic add; one lane polls the 8 shards with sc1 loads until
// their sum reaches the target, the workgroup barrier releases the other
// waves, and every load of handed-off partials is an sc1 load.  One workgroup
// per CU (the launch requests kFusedLds of LDS), grid <= the device's CUs, so
// every workgroup is resident.  Targets: `base` (arrivals before this launch,
// stored by workgroup 0 after the last barrier of the previous launch) +
// k * grid.  Every poll loop is bounded (kSpinCap); an expired poll sets the
// fail word and proceeds (no hang; results of that step are then invalid).
// ---------------------------------------------------------------------------
constexpr int kBarShards = 8, kBarStride = 16;  // one 128-B line per shard
constexpr int kBarWords = kBarShards * kBarStride + 16;  // shards, base, fail
constexpr uint32_t kSpinCap = 1u << 22;
constexpr int kFusedLds = 96 * 1024;  // > half a CU's LDS: one workgroup per CU

struct GridBarK {
    uint64_t* shard;  // [kBarShards * kBarStride]
    uint64_t* base;
    uint64_t* fail;
};

__device__ inline uint64_t ld_sc1(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double ld_sc1d(const double* p) {
    return __builtin_bit_cast(double, ld_sc1((const uint64_t*)p));
}
__device__ inline void st_sc1d(double* p, double x) {
    __hip_atomic_store((uint64_t*)p, __builtin_bit_cast(uint64_t, x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Arrive and wait until `target` arrivals have been counted.  Every thread
// of the workgroup calls it (its sc1 partial stores issued before).
__device__ inline void grid_sync(const GridBarK& gb, uint64_t target) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(gb.shard + kBarStride * (blockIdx.x % kBarShards), (uint64_t)1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t it = 0;; ++it) {
            uint64_t n = 0;
#pragma unroll
            for (int k = 0; k < kBarShards; ++k) n += ld_sc1(gb.shard + kBarStride * k);
            if (n >= target) break;
            if (it >= kSpinCap) {
                __hip_atomic_store(gb.fail, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

template <typename T, int NS, int PRE, int VB, bool NORM>
__global__ __launch_bounds__(256 * VB) void optim_fused_kernel(
    LayoutK Lk, CopiesK C, float* __restrict__ params, const float* __restrict__ grads,
    float* __restrict__ m, float* __restrict__ v, const float* __restrict__ init_norms,
    int32_t* step, const double* gpart_in, int64_t npart_in, double* gpart, double* ppart, int ablk,
    float lr, float b1, float b2, float eps, float max_norm, int norm_params, int norm_ln,
    GridBarK gb) {
#pragma clang fp contract(off)  // (one rounding per operation: the split kernels' bits)
    extern __shared__ char fused_dyn[];  // (unused: sized so that one workgroup fits per CU)
    __shared__ float sh[VB][4][kMaxSlots];
    __shared__ double red[4][kMaxSlots];
    __shared__ float sq[kMaxSlots];
    __shared__ double gn_red[4];
    __shared__ float gn_sh;
    __shared__ uint64_t base_sh;
    constexpr int nslot = NS;
    const int tid = threadIdx.x, vt = tid & 255, half = tid >> 8, w = vt >> 6, lane = tid & 63;
    const int vb = VB * blockIdx.x + half;
    const uint64_t G = gridDim.x;
    for (int i = tid; i < VB * 4 * kMaxSlots; i += 256 * VB) (&sh[0][0][0])[i] = 0.f;
    if (tid == 0) base_sh = ld_sc1(gb.base);
    (void)fused_dyn;

    // this thread's parameters (adam_kernel's mapping over ablk blocks), in
    // flight while the norm is formed
    const int64_t p0 = vb * (int64_t)256 + vt;
    const int64_t stride = (int64_t)ablk * 256;
    float gq[PRE], mq[PRE], vq[PRE], qq[PRE];
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
        const int64_t p = p0 + u * stride;
        gq[u] = mq[u] = vq[u] = qq[u] = 0.f;
        if (vb < ablk && p < Lk.total) {
            gq[u] = grads[p];
            mq[u] = m[p];
            vq[u] = v[p];
            qq[u] = params[p];
        }
    }
    const int count = step[0] + 1;
    __syncthreads();  // base_sh
    const uint64_t base = base_sh;
    int nbar = 0;

    const double* gp = gpart_in;
    int64_t np = npart_in;
    if (NORM) {
        // sumsq_partial_kernel's kNormBlocks partials of grads^2 (the
        // all-reduced gradient), virtual norm block k on the first 256 threads
        for (int k = blockIdx.x; k < kNormBlocks; k += gridDim.x) {
            double s = 0;
            if (tid < 256) {
                const int64_t st = (int64_t)kNormBlocks * 256;
                for (int64_t i0 = k * 256 + tid; i0 < Lk.total; i0 += 8 * st) {
                    float x[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = i0 + u * st < Lk.total ? grads[i0 + u * st] : 0.f;
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (i0 + u * st < Lk.total) {
                            const double d = x[u];
                            s += d * d;
                        }
                }
                s = wave_sum64d(s);
                if (lane == 0) gn_red[w] = s;
            }
            __syncthreads();
            if (tid == 0) st_sc1d(gpart + k, ((gn_red[0] + gn_red[1]) + gn_red[2]) + gn_red[3]);
            __syncthreads();
        }
        grid_sync(gb, base + (uint64_t)(++nbar) * G);
        gp = gpart;
        np = kNormBlocks;
    }
    // global_norm's fixed order on the first 256 threads (sc1 loads where
    // the partials came from this launch)
    if (tid < 256) {
        double t = 0.0;
        for (int64_t i0 = tid; i0 < np; i0 += 8 * 256) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t i = i0 + (int64_t)u * 256;
                x[u] = i < np ? (NORM ? ld_sc1d(gp + i) : gp[i]) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) t += x[u];
        }
        t = wave_sum64d(t);
        if (lane == 0) gn_red[w] = t;
    }
    __syncthreads();
    if (tid == 0) gn_sh = sqrtf((float)((gn_red[0] + gn_red[1]) + (gn_red[2] + gn_red[3])));
    __syncthreads();
    const float gn = gn_sh;

    // clip + Adam (adam_kernel's arithmetic); the new values and moments stay
    // in registers until after the barrier, so the barrier's vmcnt(0) waits
    // for the partials' stores only
    float nq[PRE];
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
        const int64_t p = p0 + u * stride;
        nq[u] = qq[u];
        if (vb >= ablk || p - vt >= Lk.total) continue;  // (uniform per virtual block)
        float contrib = 0.f;
        int slot = -2;
        const bool pad = Lk.lstm_H && p >= Lk.mlp_total && p < Lk.lstm_off;
        if (p < Lk.total && !pad) {
            nq[u] = adam_param(gq[u], mq[u], vq[u], qq[u], gn, max_norm, b1, b2, eps, lr, count,
                               mq[u], vq[u]);
            slot = proj_slot(Lk, p);
            contrib = nq[u] * nq[u];
        }
        for (int s2 = 0; s2 < nslot; ++s2) {
            if (!__any(slot == s2)) continue;
            float x = slot == s2 ? contrib : 0.f;
            x = wave_sum64(x);
            if (lane == 0) sh[half][w][s2] += x;
        }
    }
    __syncthreads();
    if (vt < nslot && vb < ablk) {
        const int s2 = vt;
        st_sc1d(ppart + vb * (int64_t)nslot + s2,
                ((double)sh[half][0][s2] + sh[half][1][s2]) + ((double)sh[half][2][s2] + sh[half][3][s2]));
    }
    grid_sync(gb, base + (uint64_t)(++nbar) * G);

    // project_kernel's per-slot totals (fixed order, first 256 threads)
    if (tid < 256) {
        double t[NS];
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) t[sl] = 0;
        for (int b0 = tid; b0 < ablk; b0 += 512) {
            double x[2][NS];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int sl = 0; sl < NS; ++sl) {
                    const int b = b0 + 256 * u;
                    x[u][sl] = b < ablk ? ld_sc1d(ppart + (int64_t)b * nslot + sl) : 0.0;
                }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int sl = 0; sl < NS; ++sl)
                    if (b0 + 256 * u < ablk) t[sl] += x[u][sl];
        }
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            const double tt = wave_sum64d(t[sl]);
            if (lane == 0) red[w][sl] = tt;
        }
    }
    __syncthreads();
    if (tid < nslot) sq[tid] = (float)(((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]);
    __syncthreads();
    if (blockIdx.x == 0 && tid == 0) {
        if (step) step[0] += 1;
        // arrivals so far, for the next launch's targets (every workgroup has
        // read base: it arrived at the barriers above after reading it)
        __hip_atomic_store(gb.base, base + (uint64_t)nbar * G, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    // projection (project_kernel's arithmetic) + master params + images
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
        const int64_t p = p0 + u * stride;
        if (vb >= ablk || p >= Lk.total) continue;
        const bool pad = Lk.lstm_H && p >= Lk.mlp_total && p < Lk.lstm_off;
        float val = nq[u];
        const int slot = proj_slot(Lk, p);
        if (slot >= 2 * Lk.L) {
            if (norm_params) val = (init_norms[Lk.L + slot - 2 * Lk.L] * val) / sqrtf(sq[slot]);
        } else if (slot >= 0) {
            const int l = slot >> 1;
            if ((slot & 1) == 0) {
                if (norm_params) val = (init_norms[l] * val) / sqrtf(sq[slot]);
            } else if (norm_ln) {
                val = sqrtf((float)Lk.H / sq[slot]) * val;
            }
        }
        if (!pad) {
            params[p] = val;
            m[p] = mq[u];
            v[p] = vq[u];
        }
        write_copies<T>(Lk, C, p, val);
    }
}

// compute copies from params without any projection; zero the head padding
template <typename T>
__global__ __launch_bounds__(256) void sync_kernel(LayoutK Lk, CopiesK C, const float* params) {
    const int64_t p = blockIdx.x * (int64_t)256 + threadIdx.x;
    const int H = Lk.H;
    // padding: head_t rows A1..31, head cols A1..31, head_b A1..31
    const int64_t pad = (int64_t)(Lk.HC - Lk.A1) * H;
    if (p < pad) {
        int k = Lk.A1 + (int)(p / H), c = (int)(p % H);
        ((T*)C.head_t)[img_index<T>(k, c, H, true)] = cvt<T>(0.f);
        ((T*)C.head)[img_index<T>(c, k, Lk.HC, false)] = cvt<T>(0.f);
        if (C.head_t_nat) ((T*)C.head_t_nat)[img_index<T>(k, c, H, false)] = cvt<T>(0.f);
        if (c == 0) C.head_b[k] = 0.f;
    }
    if (p < Lk.total) write_copies<T>(Lk, C, p, params[p]);
}

// workspace (doubles): norm partials, projection partials, spare, then the
// fused launch's barrier words on 128-B lines (zeroed by the caller once)
static int64_t optim_bar_offset(const LayoutK& k) {
    int64_t nblk = (k.total + 255) / 256;
    return (kNormBlocks + nblk * kMaxSlots + 8 + kMaxSlots + 8 + 15) / 16 * 16;
}
static int64_t optim_ws_doubles(const LayoutK& k) { return optim_bar_offset(k) + kBarWords; }

// Projection slot counts with a project_kernel instantiation: 2 L (trunk
// kernels + LayerNorms, L <= MLEARN_MAX_LAYERS) and 2 L + 8 (the LSTM gate
// kernels); optim_launch checks nslot against it before anything launches.
constexpr int kMaxProjSlots = 16;
static_assert(kMaxSlots <= kMaxProjSlots, "a projection slot count has no project_kernel instantiation");
static bool project_slots_ok(int nslot) { return nslot >= 2 && nslot <= kMaxProjSlots && nslot % 2 == 0; }

template <typename T>
static void launch_project(int nslot, dim3 grid, hipStream_t s, const LayoutK& Lk, const CopiesK& C,
                           const mlearn_optim_state* st, const double* ppart, int ablk) {
#define ML_PROJ(NS)                                                                            \
    case NS:                                                                                   \
        hipLaunchKernelGGL((project_kernel<T, NS>), grid, dim3(256), 0, s, Lk, C, st->params, \
                           st->init_norms, ppart, ablk, st->normalize_params,                  \
                           st->normalize_layernorms, st->step);                                \
        break;
    switch (nslot) {
        ML_PROJ(2)
        ML_PROJ(4)
        ML_PROJ(6)
        ML_PROJ(8)
        ML_PROJ(10)
        ML_PROJ(12)
        ML_PROJ(14)
        ML_PROJ(16)
        default: break;  // unreachable: project_slots_ok(nslot) was required before any launch
    }
#undef ML_PROJ
}

// ---------------------------------------------------------------------------
// Flat optimizer (mlearn_flat_optim_step): any policy tree's f32 parameter
// vector with a table of projection groups.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void flat_adam_kernel(float* __restrict__ params,
                                                        const float* __restrict__ grads,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        const int32_t* step, int64_t n,
                                                        const double* gpart, int64_t npart, float lr,
                                                        float b1, float b2, float eps, float max_norm,
                                                        int skip_nonfinite) {
    const float gn = global_norm(gpart, npart);
    // DynamicScale (ppo.py:288-291): a non-finite gradient keeps params and
    // moments (every block reads the same norm: a uniform exit)
    if (skip_nonfinite && !isfinite(gn)) return;
    const int count = step[0] + 1;
    const float c1 = 1.f - powf(b1, (float)count), c2 = 1.f - powf(b2, (float)count);
    for (int64_t p = blockIdx.x * (int64_t)256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
        float g = grads[p];
        if (!(gn < max_norm)) g = (g / gn) * max_norm;  // clip_by_global_norm
        const float mm = (1.f - b1) * g + b1 * m[p];
        const float vv = (1.f - b2) * (g * g) + b2 * v[p];
        const float u = (mm / c1) / (sqrtf(vv / c2) + eps);
        m[p] = mm;
        v[p] = vv;
        params[p] = params[p] + (-lr) * u;
    }
}

// One block per group: the group's sum of squares (kernel, or LayerNorm
// scale then bias) in a fixed order, then every element rescaled.
__global__ __launch_bounds__(256) void flat_project_kernel(float* __restrict__ params,
                                                           const mlearn_flat_group* groups,
                                                           int ngroups, int norm_params,
                                                           int norm_ln, int32_t* step,
                                                           const double* gpart, int64_t npart,
                                                           int skip_nonfinite) {
    __shared__ double red[4];
    __shared__ float sq;
    if (blockIdx.x == 0) {
        // the step counter advances with the Adam update it counts
        const bool fin = !skip_nonfinite || isfinite(global_norm(gpart, npart));
        if (threadIdx.x == 0 && step && fin) step[0] += 1;
    }
    if ((int)blockIdx.x >= ngroups) return;
    const mlearn_flat_group gr = groups[blockIdx.x];
    const bool on = gr.kind != 2 ? norm_params != 0 : norm_ln != 0;
    if (!on) return;
    // kind 3: a column block (count columns of count2 rows, row stride offset2)
    const bool blk = gr.kind == 3;
    const int64_t nel = blk ? gr.count * gr.count2 : gr.count;
    auto at = [&](int64_t i) -> float& {
        return blk ? params[gr.offset + (i / gr.count) * gr.offset2 + i % gr.count]
                   : params[gr.offset + i];
    };
    double t = 0.0;
    for (int64_t i = threadIdx.x; i < nel; i += 256) {
        const double x = at(i);
        t += x * x;
    }
    for (int64_t i = threadIdx.x; !blk && i < gr.count2; i += 256) {
        const double x = params[gr.offset2 + i];
        t += x * x;
    }
    t = wave_sum64d(t);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) sq = (float)(((red[0] + red[1]) + red[2]) + red[3]);
    __syncthreads();
    if (gr.kind == 1 || blk) {  // ppo.py:307: init_norm * W / |W|
        for (int64_t i = threadIdx.x; i < nel; i += 256) {
            float& q = at(i);
            q = (gr.init_norm * q) / sqrtf(sq);
        }
    } else {  // ppo.py:324-325: sqrt(F / (b.b + s.s)) * (s, b)
        const float f = sqrtf((float)gr.features / sq);
        for (int64_t i = threadIdx.x; i < gr.count; i += 256) params[gr.offset + i] *= f;
        for (int64_t i = threadIdx.x; i < gr.count2; i += 256) params[gr.offset2 + i] *= f;
    }
}

// The fused launch applies when its grid (ablk / kFusedVB workgroups, one per
// CU) fits the device's CUs and every thread's parameters fit PRE = 8.
constexpr int kFusedVB = 4;
static bool fused_ok(int ablk, int64_t nit) {
    const int cus = device_cus();
    const int grid = (ablk + kFusedVB - 1) / kFusedVB;
    return cus > 0 && grid <= cus && nit <= 8;
}

template <typename T, int NS, int PRE, bool NORM>
static int launch_fused_k(const LayoutK& Lk, const CopiesK& C, const mlearn_optim_state* st,
                          const double* gpart_in, int64_t npart_in, double* gpart, double* ppart,
                          int ablk, uint64_t* bar, hipStream_t s) {
    auto kern = optim_fused_kernel<T, NS, PRE, kFusedVB, NORM>;
    int rc = set_lds_attr((const void*)kern, kFusedLds, "optim_fused");
    if (rc) return rc;
    GridBarK gb{bar, bar + kBarShards * kBarStride, bar + kBarShards * kBarStride + 8};
    const int grid = (ablk + kFusedVB - 1) / kFusedVB;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256 * kFusedVB), kFusedLds, s, Lk, C, st->params,
                       st->grads, st->adam_m, st->adam_v, st->init_norms, st->step, gpart_in,
                       npart_in, gpart, ppart, ablk, st->lr, st->b1, st->b2, st->eps,
                       st->max_grad_norm, st->normalize_params, st->normalize_layernorms, gb);
    return check_launch("optim_step (fused)");
}

template <typename T>
static int launch_fused(int nslot, int64_t nit, int norm, const LayoutK& Lk, const CopiesK& C,
                        const mlearn_optim_state* st, const double* gpart_in, int64_t npart_in,
                        double* gpart, double* ppart, int ablk, uint64_t* bar, hipStream_t s) {
#define ML_FUSED(NS)                                                                              \
    case NS:                                                                                      \
        if (nit <= 1)                                                                             \
            return norm ? launch_fused_k<T, NS, 1, true>(Lk, C, st, gpart_in, npart_in, gpart,    \
                                                         ppart, ablk, bar, s)                     \
                        : launch_fused_k<T, NS, 1, false>(Lk, C, st, gpart_in, npart_in, gpart,   \
                                                          ppart, ablk, bar, s);                   \
        return norm ? launch_fused_k<T, NS, 8, true>(Lk, C, st, gpart_in, npart_in, gpart, ppart, \
                                                     ablk, bar, s)                                \
                    : launch_fused_k<T, NS, 8, false>(Lk, C, st, gpart_in, npart_in, gpart,       \
                                                      ppart, ablk, bar, s);
    switch (nslot) {
        ML_FUSED(2)
        ML_FUSED(4)
        ML_FUSED(6)
        ML_FUSED(8)
        ML_FUSED(10)
        ML_FUSED(12)
        ML_FUSED(14)
        ML_FUSED(16)
        default: break;
    }
#undef ML_FUSED
    set_error("optim_step: %d projection slots", nslot);
    return MLEARN_EINVAL;
}

}  // namespace ml

using namespace ml;

extern "C" {

int64_t mlearn_flat_optim_workspace_bytes(int64_t n, int32_t num_groups) {
    if (n < 1 || num_groups < 0) return -1;
    return (int64_t)kNormBlocks * (int64_t)sizeof(double);
}

int mlearn_flat_optim_step(const mlearn_flat_optim* st, void* workspace, mlearn_stream_t stream) {
    ML_REQUIRE(st && st->params && st->grads && st->adam_m && st->adam_v && st->step && workspace,
               "flat_optim_step: null pointer");
    ML_REQUIRE(st->n >= 1 && st->num_groups >= 0 && (st->num_groups == 0 || st->groups),
               "flat_optim_step: bad sizes");
    ML_REQUIRE(st->max_grad_norm > 0 && st->lr >= 0, "flat_optim_step: bad hyperparameters");
    hipStream_t s = S(stream);
    double* gpart = (double*)workspace;
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(kNormBlocks), dim3(256), 0, s, st->grads, st->n,
                       gpart);
    const int64_t nb = (st->n + 255) / 256;
    hipLaunchKernelGGL(flat_adam_kernel, dim3((unsigned)(nb < 1024 ? nb : 1024)), dim3(256), 0, s,
                       st->params, st->grads, st->adam_m, st->adam_v, (const int32_t*)st->step,
                       st->n, (const double*)gpart, (int64_t)kNormBlocks, st->lr, st->b1, st->b2,
                       st->eps, st->max_grad_norm, st->skip_nonfinite);
    // (one block per group; at least one block: it also advances the step counter)
    hipLaunchKernelGGL(flat_project_kernel, dim3((unsigned)(st->num_groups > 0 ? st->num_groups : 1)),
                       dim3(256), 0, s, st->params, st->groups, st->num_groups,
                       st->normalize_params, st->normalize_layernorms, st->step,
                       (const double*)gpart, (int64_t)kNormBlocks, st->skip_nonfinite);
    return check_launch("flat_optim_step");
}


int64_t mlearn_optim_workspace_bytes(const mlearn_mlp_policy* policy) {
    if (validate_policy(policy)) return -1;
    return optim_ws_doubles(make_layout(*policy)) * (int64_t)sizeof(double);
}

static int optim_launch(const LayoutK& Lk, const CopiesK& C, int dtype,
                        const mlearn_optim_state* st, void* workspace, hipStream_t s) {
    ML_REQUIRE(st && st->params && st->grads && st->adam_m && st->adam_v && st->init_norms &&
                   st->step && workspace,
               "optim_step: null pointer");
    ML_REQUIRE(st->max_grad_norm > 0 && st->lr >= 0, "optim_step: bad hyperparameters");
    ML_REQUIRE(project_slots_ok(2 * Lk.L + (Lk.lstm_H ? 8 : 0)),
               "optim_step: %d projection slots (layers %d) have no projection kernel",
               2 * Lk.L + (Lk.lstm_H ? 8 : 0), Lk.L);
    const int64_t nblk = (Lk.total + 255) / 256;
    const int ablk = (int)(nblk < kAdamBlocks ? nblk : kAdamBlocks);
    double* gpart = (double*)workspace;
    double* ppart = gpart + kNormBlocks;
    const double* norm_part = gpart;
    int64_t nparts = kNormBlocks;
    ML_REQUIRE(st->launch_form >= 0 && st->launch_form <= 2, "optim_step: launch_form %d",
               st->launch_form);
    const bool fused_fits =
        fused_ok(ablk, (Lk.total + (int64_t)ablk * 256 - 1) / ((int64_t)ablk * 256));
    ML_REQUIRE(st->launch_form != 2 || fused_fits,
               "optim_step: the fused launch needs %d workgroups (one per CU) on %d CUs",
               (ablk + kFusedVB - 1) / kFusedVB, device_cus());
    // the library's choice is the split launches: the fused launch measured no
    // faster at world 1 (9.32 / 9.25 vs 9.26 / 9.26 ms per headline update)
    // and 2.4 % slower in the emulated world-8 share (3.70 vs 3.61 ms): its
    // grid barrier costs what the kernel boundary it replaces did
    // (profiles/r06_optim_fused_ab.txt)
    const bool fused = fused_fits && st->launch_form == 2;
    if (st->grad_sumsq_part) {  // partials from the gradient reduction (no extra launch)
        ML_REQUIRE(st->grad_sumsq_nparts == (Lk.total + 63) / 64,
                   "optim_step: grad_sumsq_nparts %lld != %lld", (long long)st->grad_sumsq_nparts,
                   (long long)((Lk.total + 63) / 64));
        norm_part = st->grad_sumsq_part;
        nparts = st->grad_sumsq_nparts;
    } else if (!fused) {  // (the fused launch forms the norm partials itself)
        hipLaunchKernelGGL(sumsq_partial_kernel, dim3(kNormBlocks), dim3(256), 0, s, st->grads,
                           Lk.total, gpart);
    }
    const int nslot = 2 * Lk.L + (Lk.lstm_H ? 8 : 0);
    const int64_t nit = (Lk.total + (int64_t)ablk * 256 - 1) / ((int64_t)ablk * 256);
    if (fused) {
        const int norm = st->grad_sumsq_part ? 0 : 1;
        if (dtype == MLEARN_DTYPE_BF16)
            return launch_fused<bf16>(nslot, nit, norm, Lk, C, st, norm_part, nparts, gpart, ppart,
                                      ablk, (uint64_t*)(gpart + optim_bar_offset(Lk)), s);
        return launch_fused<float>(nslot, nit, norm, Lk, C, st, norm_part, nparts, gpart, ppart,
                                   ablk, (uint64_t*)(gpart + optim_bar_offset(Lk)), s);
    }
    auto adam = nit <= 1 ? adam_kernel<1> : nit <= 2 ? adam_kernel<2> : nit <= 4 ? adam_kernel<4> : adam_kernel<8>;
    hipLaunchKernelGGL(adam, dim3((unsigned)ablk), dim3(256), 0, s, Lk, st->params,
                       st->grads, st->adam_m, st->adam_v, (const int32_t*)st->step, norm_part,
                       nparts, st->lr, st->b1, st->b2, st->eps, st->max_grad_norm, ppart);
    if (dtype == MLEARN_DTYPE_BF16)
        launch_project<bf16>(nslot, dim3((unsigned)nblk), s, Lk, C, st, (const double*)ppart, ablk);
    else
        launch_project<float>(nslot, dim3((unsigned)nblk), s, Lk, C, st, (const double*)ppart, ablk);
    return check_launch("optim_step");
}

static int sync_launch(const LayoutK& Lk, const CopiesK& C, int dtype, const float* params,
                       hipStream_t s) {
    ML_REQUIRE(params, "sync_weights: null params");
    int64_t n = Lk.total > (int64_t)Lk.HC * Lk.H ? Lk.total : (int64_t)Lk.HC * Lk.H;
    unsigned g = (unsigned)((n + 255) / 256);
    if (dtype == MLEARN_DTYPE_BF16)
        hipLaunchKernelGGL(sync_kernel<bf16>, dim3(g), dim3(256), 0, s, Lk, C, params);
    else
        hipLaunchKernelGGL(sync_kernel<float>, dim3(g), dim3(256), 0, s, Lk, C, params);
    return check_launch("sync_weights");
}

int mlearn_optim_step(const mlearn_mlp_policy* policy, const mlearn_optim_state* st,
                      void* workspace, mlearn_stream_t stream) {
    int rc = validate_policy(policy);
    if (rc) return rc;
    return optim_launch(make_layout(*policy), make_copies(*policy), policy->dtype, st, workspace,
                        S(stream));
}

int mlearn_policy_sync_weights(const mlearn_mlp_policy* policy, const float* params,
                               mlearn_stream_t stream) {
    int rc = validate_policy(policy);
    if (rc) return rc;
    return sync_launch(make_layout(*policy), make_copies(*policy), policy->dtype, params,
                       S(stream));
}

int64_t mlearn_lstm_param_offset(const mlearn_mlp_policy* policy) {
    if (validate_policy(policy)) return -1;
    return (make_layout(*policy).mlp_total + 63) / 64 * 64;
}

int64_t mlearn_lstm_param_count(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm) {
    if (validate_lstm(policy, lstm)) return -1;
    return make_layout_lstm(*policy, *lstm).total;
}

int64_t mlearn_lstm_optim_workspace_bytes(const mlearn_mlp_policy* policy,
                                          const mlearn_lstm* lstm) {
    if (validate_lstm(policy, lstm)) return -1;
    return optim_ws_doubles(make_layout_lstm(*policy, *lstm)) * (int64_t)sizeof(double);
}

int mlearn_lstm_optim_step(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                           const mlearn_optim_state* st, void* workspace, mlearn_stream_t stream) {
    int rc = validate_lstm(policy, lstm);
    if (rc) return rc;
    return optim_launch(make_layout_lstm(*policy, *lstm), make_copies(*policy, lstm),
                        policy->dtype, st, workspace, S(stream));
}

int mlearn_lstm_sync_weights(const mlearn_mlp_policy* policy, const mlearn_lstm* lstm,
                             const float* params, mlearn_stream_t stream) {
    int rc = validate_lstm(policy, lstm);
    if (rc) return rc;
    return sync_launch(make_layout_lstm(*policy, *lstm), make_copies(*policy, lstm),
                       policy->dtype, params, S(stream));
}

}  // extern "C"
