// Streaming / reduction kernels of the PPO iteration:
//   GAE + returns, discounted returns, z-score, discrete sampling and
//   action stats, metrics, epoch permutation, advantage statistics,
//   rollout post-step bookkeeping, and the synthetic dummy environment.
// All are HBM/latency-bound integer or fp32 streaming work: coalesced
// [T][N] rows, 16-B loads where the layout allows, wave-shuffle reductions,
// deterministic partial slabs instead of float atomics.

#include <stdarg.h>
#include <stdio.h>

#include "common.h"

#include <atomic>
#include <mutex>
#include <set>
#include <utility>
#include "dists.h"
#include "env.h"
#include "rowtile.h"

namespace ml {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

constexpr int kMaxDevices = 64;

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return MLEARN_EHIP;
    }
    return MLEARN_OK;
}

int device_cus() {
    static std::atomic<int> cache[kMaxDevices];  // CU count + 1; 0 = not queried yet
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 0;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (v == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 0;
        v = cus + 1;
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v - 1;
}

int set_lds_attr(const void* fn, int bytes, const char* what) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({fn, dev})) return MLEARN_OK;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        set_error("%s: %d B of LDS refused (%s)", what, bytes, hipGetErrorString(e));
        return MLEARN_EHIP;
    }
    done.insert({fn, dev});
    return MLEARN_OK;
}

static inline int grid_for(int64_t n, int block, int cap = 1 << 20) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// ---------------------------------------------------------------------------
// Philox
// ---------------------------------------------------------------------------
__global__ void philox_kernel(const uint4* __restrict__ ctr, uint32_t k0, uint32_t k1,
                              uint4* __restrict__ out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint4 c = ctr[i];
        u32x4 r = philox4x32(u32x4{c.x, c.y, c.z, c.w}, k0, k1);
        out[i] = make_uint4(r.x, r.y, r.z, r.w);
    }
}

// ---------------------------------------------------------------------------
// GAE (algo_common.py:84-130) + returns = adv + values (rollouts.py:761-769).
// One lane per env column (measured on MI355X at N = 2^22: one column per
// lane streams at 5.6 TB/s, four columns per lane with 16-B loads at 4.6 TB/s,
// fewer waves in flight; tools/gae_sweep.hip).
// The reverse recurrence per column:
//   nv = d_t ? 0 : nv ;  na = d_t ? 0 : na
//   A_t = (r_t + g*nv - v_t) + g*l*na ;  nv = v_t ;  na = A_t
// The recurrence is serial in t, so the loads are what must be parallel:
// time runs in chunks of U steps and every load of chunk c-1 is issued
// before chunk c is computed (register double buffer), so a lane keeps
// 2*U*3 loads in flight instead of 3.  Stores are non-temporal (the
// advantages/returns are read again only by the next kernel, from L2 misses
// anyway).  Operation order mirrors the reference expression tree;
// contraction is off so the fp32 result is reproducible against the
// oracle's fp32 mode.
// ---------------------------------------------------------------------------
template <int VEC>
struct GaeChunk;
template <>
struct GaeChunk<1> {
    float r, v;
    uint32_t d;
    __device__ void load(const float* rw, const float* vl, const uint8_t* dn, int64_t o) {
        r = __builtin_nontemporal_load(rw + o);
        v = __builtin_nontemporal_load(vl + o);
        d = dn[o];
    }
    __device__ float rj(int) const { return r; }
    __device__ float vj(int) const { return v; }
    __device__ uint32_t dj(int) const { return d; }
};

template <int VEC>
__device__ __forceinline__ void gae_store(float* p, const float* x) {
    static_assert(VEC == 1, "one column per lane");
    __builtin_nontemporal_store(x[0], p);
}

template <int VEC, int U>
__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rewards,
                                                  const float* __restrict__ values,
                                                  const uint8_t* __restrict__ dones,
                                                  const float* __restrict__ boot,
                                                  float* __restrict__ adv, float* __restrict__ ret,
                                                  int T, int64_t N, float gamma, float gl,
                                                  const float* __restrict__ vn, int64_t vn_cols) {
#pragma clang fp contract(off)
    int64_t n0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * VEC;
    if (n0 >= N) return;
    // value normaliser (normalize_values): values / bootstrap are inverted,
    // v * sigma + mu (EMANormalizer.invert, moving_avg.py:87-95)
    float vmu = 0.f, vsig = 1.f;
    if (vn) {
        const float* e = vn + (n0 / vn_cols) * 8;
        vmu = e[0];
        vsig = e[2];
    }
    float nv[VEC], na[VEC];
    for (int j = 0; j < VEC; ++j) nv[j] = vn ? boot[n0 + j] * vsig + vmu : boot[n0 + j];
    for (int j = 0; j < VEC; ++j) na[j] = 0.f;

    GaeChunk<VEC> cur[U], nxt[U];
    int t_hi = T - 1;  // chunk = steps (t_hi-U, t_hi]
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (t_hi - u >= 0) cur[u].load(rewards, values, dones, (int64_t)(t_hi - u) * N + n0);
    while (t_hi >= 0) {
        int t_nx = t_hi - U;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t_nx - u >= 0) nxt[u].load(rewards, values, dones, (int64_t)(t_nx - u) * N + n0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int t = t_hi - u;
            if (t < 0) break;
            float a[VEC], rt[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
                uint32_t d = cur[u].dj(j);
                float v = cur[u].vj(j);
                if (vn) v = v * vsig + vmu;
                float nvj = d ? 0.f : nv[j];
                float naj = d ? 0.f : na[j];
                float td = (cur[u].rj(j) + gamma * nvj) - v;
                a[j] = td + gl * naj;
                rt[j] = a[j] + v;
                nv[j] = v;
                na[j] = a[j];
            }
            int64_t o = (int64_t)t * N + n0;
            gae_store<VEC>(adv + o, a);
            if (ret) gae_store<VEC>(ret + o, rt);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        t_hi = t_nx;
    }
}

// compute_returns (algo_common.py:45-81)
__global__ __launch_bounds__(256) void returns_kernel(const float* __restrict__ rewards,
                                                      const uint8_t* __restrict__ dones,
                                                      const float* __restrict__ boot,
                                                      float* __restrict__ ret, int T, int64_t N,
                                                      float gamma) {
#pragma clang fp contract(off)
    int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (n >= N) return;
    float nr = boot[n];
    for (int t = T - 1; t >= 0; --t) {
        int64_t o = (int64_t)t * N + n;
        nr = dones[o] ? 0.f : nr;
        nr = rewards[o] + gamma * nr;
        ret[o] = nr;
    }
}

// ---------------------------------------------------------------------------
// Block-level double reductions with a fixed order (deterministic).
// ---------------------------------------------------------------------------
template <int BLOCK>
__device__ inline double block_sum_d(double v, double* sh) {
    v = wave_sum64d(v);
    int w = threadIdx.x / 64, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double s = 0;
    for (int i = 0; i < BLOCK / 64; ++i) s += sh[i];
    return s;
}

__device__ inline float wave_min(float v) {
    for (int o = 1; o < 64; o <<= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ inline float wave_max(float v) {
    for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// ---------------------------------------------------------------------------
// Metrics: Metric.init_from_data (metrics.py:31-48).  Pass 1: per-block
// (sum, sumsq in double, min, max) partials; pass 2: one block per job sums
// partials in block order: mean = S/n, m2 = SS - n*mean^2 (double).
// ---------------------------------------------------------------------------
struct MetricJobs {
    mlearn_metric_job j[16];
};
constexpr int kMetricBlocks = 256;

// One job's element e (windowed [T][ld] column block when cols != 0).
__device__ inline float metric_x(const mlearn_metric_job& J, int64_t i) {
    const int64_t e = J.cols ? (i / J.cols) * J.ld + i % J.cols : i;
    float x = J.x[e];
    if (J.x2) x = x + J.x2[e];  // (commutative: = advantages + values of the GAE)
    return J.abs_value ? fabsf(x) : x;
}

// Partial {sum, sum of squares, min, max} per (block, job).  Contiguous jobs
// (cols == 0, 16-B aligned, n % 4 == 0) read float4s, four elements per
// thread per iteration in four independent f64 chains (fixed order).
__global__ __launch_bounds__(256) void metrics_partial_kernel(MetricJobs jobs, double* part) {
    __shared__ double sh[4];
    __shared__ float shf[4];
    const mlearn_metric_job& J = jobs.j[blockIdx.y];
    double s4[4] = {0, 0, 0, 0}, q4[4] = {0, 0, 0, 0};
    float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
    const bool vec = J.cols == 0 && (J.n & 3) == 0 && ((uintptr_t)J.x & 15) == 0 &&
                     (!J.x2 || ((uintptr_t)J.x2 & 15) == 0);
    if (vec) {
        const int64_t n4 = J.n >> 2;
        for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
            float4 v = ((const float4*)J.x)[i];
            if (J.x2) {
                const float4 w = ((const float4*)J.x2)[i];
                v = make_float4(v.x + w.x, v.y + w.y, v.z + w.z, v.w + w.w);
            }
            if (J.abs_value) v = make_float4(fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w));
            const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                s4[k] += e[k];
                q4[k] += (double)e[k] * e[k];
                mn = fminf(mn, e[k]);
                mx = fmaxf(mx, e[k]);
            }
        }
    } else {
        for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < J.n; i += (int64_t)gridDim.x * 256) {
            const float x = metric_x(J, i);
            s4[0] += x;
            q4[0] += (double)x * x;
            mn = fminf(mn, x);
            mx = fmaxf(mx, x);
        }
    }
    double s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    double q = (q4[0] + q4[1]) + (q4[2] + q4[3]);
    s = block_sum_d<256>(s, sh);
    q = block_sum_d<256>(q, sh);
    mn = wave_min(mn);
    mx = wave_max(mx);
    int w = threadIdx.x / 64;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) shf[w] = mn;
    __syncthreads();
    float bmn = fminf(fminf(shf[0], shf[1]), fminf(shf[2], shf[3]));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) shf[w] = mx;
    __syncthreads();
    float bmx = fmaxf(fmaxf(shf[0], shf[1]), fmaxf(shf[2], shf[3]));
    if (threadIdx.x == 0) {
        double* p = part + ((int64_t)blockIdx.y * kMetricBlocks + blockIdx.x) * 4;
        p[0] = s;
        p[1] = q;
        p[2] = bmn;
        p[3] = bmx;
    }
}

// One wave per job: lane l takes partials l, l + 64, ... (fixed order), then
// a fixed butterfly.
__global__ __launch_bounds__(64) void metrics_finish_kernel(MetricJobs jobs, const double* part,
                                                            float* out) {
    const mlearn_metric_job& J = jobs.j[blockIdx.x];
    const int l = threadIdx.x;
    double s = 0, q = 0, mn = 3.402823466e+38, mx = -3.402823466e+38;
    for (int b = l; b < kMetricBlocks; b += 64) {
        const double* p = part + ((int64_t)blockIdx.x * kMetricBlocks + b) * 4;
        s += p[0];
        q += p[1];
        mn = fmin(mn, p[2]);
        mx = fmax(mx, p[3]);
    }
    for (int o = 32; o >= 1; o >>= 1) {
        s += __shfl_xor(s, o);
        q += __shfl_xor(q, o);
        mn = fmin(mn, __shfl_xor(mn, o));
        mx = fmax(mx, __shfl_xor(mx, o));
    }
    if (l != 0) return;
    double n = (double)J.n;
    double mean = n > 0 ? s / n : 0.0;
    double m2 = n > 0 ? q - n * mean * mean : 0.0;
    if (m2 < 0) m2 = 0;
    float* o = out + blockIdx.x * 5;
    o[0] = (float)mean;
    o[1] = (float)m2;
    o[2] = (float)mn;
    o[3] = (float)mx;
    o[4] = (float)J.n;
}

// ---------------------------------------------------------------------------
// z-score over a whole array (algo_common.py:133-140).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sum_partial_kernel(const float* x, int64_t n, double* part) {
    __shared__ double sh[4];
    double s = 0, q = 0;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double v = x[i];
        s += v;
        q += v * v;
    }
    s = block_sum_d<256>(s, sh);
    q = block_sum_d<256>(q, sh);
    if (threadIdx.x == 0) {
        part[blockIdx.x * 2] = s;
        part[blockIdx.x * 2 + 1] = q;
    }
}

__global__ __launch_bounds__(256) void zscore_apply_kernel(const float* x, int64_t n,
                                                           const double* part, int nparts,
                                                           float* out) {
    double s = 0, q = 0;
    for (int b = 0; b < nparts; ++b) {
        s += part[2 * b];
        q += part[2 * b + 1];
    }
    double dn = (double)n;
    float mean = (float)(s / dn);
    float var = (float)(q / dn - (s / dn) * (s / dn));
    float rs = rsqrtf(fmaxf(var, 1e-5f));
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = (x[i] - mean) * rs;
}

// ---------------------------------------------------------------------------
// Discrete distributions (dists.py:26-77).  One lane per (row, group).
// ---------------------------------------------------------------------------
struct Layout {
    int K, A;
    int off[MLEARN_MAX_GROUPS + 1];
};

static inline Layout to_layout(const mlearn_action_layout& l) {
    Layout r;
    r.K = l.num_groups;
    r.A = l.num_logits;
    for (int i = 0; i <= MLEARN_MAX_GROUPS; ++i) r.off[i] = l.offsets[i];
    return r;
}

__global__ __launch_bounds__(256) void sample_kernel(const float* __restrict__ logits, int64_t ld,
                                                     Layout lay, int64_t N, uint32_t k0,
                                                     uint32_t k1, const uint64_t* step_ctr,
                                                     uint64_t step_add, uint32_t env_off,
                                                     int sample, int32_t* actions, float* logp) {
    const uint64_t step = (step_ctr ? *step_ctr : 0ull) + step_add;
    int64_t task = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (task >= N * lay.K) return;
    int64_t n = task / lay.K;
    int g = (int)(task % lay.K);
    float lg[32];
    int nb = lay.off[g + 1] - lay.off[g];
    for (int j = 0; j < nb; ++j) lg[j] = logits[n * ld + lay.off[g] + j];
    int a;
    float lp;
    sample_group(lg, nb, lay.off[g], k0, k1, env_off + (uint32_t)n, step, sample, &a, &lp);
    actions[task] = a;
    if (logp) logp[task] = lp;
}

__global__ __launch_bounds__(256) void action_stats_kernel(const float* __restrict__ logits,
                                                           int64_t ld, Layout lay, int64_t N,
                                                           const int32_t* actions, float* logp,
                                                           float* ent) {
    int64_t task = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (task >= N * lay.K) return;
    int64_t n = task / lay.K;
    int g = (int)(task % lay.K);
    const float* lg = logits + n * ld + lay.off[g];
    int nb = lay.off[g + 1] - lay.off[g];
    float mx = lg[0];
    for (int j = 1; j < nb; ++j) mx = fmaxf(mx, lg[j]);
    float se = 0.f;
    for (int j = 0; j < nb; ++j) se += __expf(lg[j] - mx);
    float lse = mx + __logf(se);
    float h = 0.f;
    for (int j = 0; j < nb; ++j) {
        float lp = lg[j] - lse;
        h -= __expf(lg[j] - mx) / se * lp;
    }
    int a = actions[task];
    logp[task] = lg[a] - lse;
    ent[task] = h;
}

// ---------------------------------------------------------------------------
// Epoch permutation (ppo.py:445-458): bitonic sort of (philox key, index)
// pairs in LDS, one workgroup.
// ---------------------------------------------------------------------------

// Epoch permutation as a keyed bijection: a 4-round balanced Feistel network
// on [0, 2^b) (b = ceil(log2 n) rounded up to even, round function = Philox
// word 0 of ctr {R + (round << 24), rank, epoch lo, epoch hi}) restricted to
// [0, n) by cycle walking.  Every element is independent: one thread each.
__device__ inline uint32_t feistel4(uint32_t x, int half, uint32_t mask, uint32_t k0, uint32_t k1,
                                    uint32_t rank, uint64_t epoch) {
    uint32_t L = x >> half, R = x & mask;
#pragma unroll
    for (int rd = 0; rd < 4; ++rd) {
        const u32x4 f = philox4x32(
            u32x4{R + ((uint32_t)rd << 24), rank, (uint32_t)epoch, (uint32_t)(epoch >> 32)}, k0, k1);
        const uint32_t nr = L ^ (f.x & mask);
        L = R;
        R = nr;
    }
    return (L << half) | R;
}

__global__ __launch_bounds__(256) void perm_kernel(uint32_t k0, uint32_t k1,
                                                   const uint64_t* epoch_ctr, uint64_t epoch_add,
                                                   uint32_t rank, int n, int half,
                                                   int32_t* perm) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t epoch = (epoch_ctr ? *epoch_ctr : 0ull) + epoch_add;
    const uint32_t mask = (1u << half) - 1u;
    uint32_t x = (uint32_t)i;
    do {
        x = feistel4(x, half, mask, k0, k1, rank, epoch);
    } while (x >= (uint32_t)n);  // cycle walking: the orbit of i returns below n
    perm[i] = (int32_t)x;
}

// ---------------------------------------------------------------------------
// Advantage statistics per minibatch (zscore_data, algo_common.py:133-140).
// Grid (num_mb, kStatBlocks); sequence s -> (chunk c = s / N, env b = s % N).
// ---------------------------------------------------------------------------
constexpr int kStatBlocks = 32;

__global__ __launch_bounds__(256) void adv_stats_kernel(mlearn_rollout_view ro,
                                                        const float* __restrict__ src,
                                                        const int32_t* __restrict__ perm,
                                                        int mb_size, double* part) {
    __shared__ double sh[4];
    int m = blockIdx.x;
    const int32_t* seqs = perm + (int64_t)m * mb_size;
    int64_t total = (int64_t)mb_size * ro.bptt_len;
    double s = 0, q = 0;
    for (int64_t i = blockIdx.y * 256 + threadIdx.x; i < total; i += (int64_t)kStatBlocks * 256) {
        int tl = (int)(i / mb_size);
        int j = (int)(i % mb_size);
        int64_t seq = seqs[j];
        int64_t c = seq / ro.N, b = seq % ro.N;
        int64_t t = c * ro.bptt_len + tl;
        double x = src[t * ro.ld + b];
        s += x;
        q += x * x;
    }
    s = block_sum_d<256>(s, sh);
    q = block_sum_d<256>(q, sh);
    if (threadIdx.x == 0) {
        double* p = part + ((int64_t)m * kStatBlocks + blockIdx.y) * 2;
        p[0] = s;
        p[1] = q;
    }
}

__global__ void adv_stats_reduce_kernel(const double* part, int num_mb, double* out) {
    int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= num_mb) return;
    double s = 0, q = 0;
    for (int b = 0; b < kStatBlocks; ++b) {
        s += part[((int64_t)m * kStatBlocks + b) * 2];
        q += part[((int64_t)m * kStatBlocks + b) * 2 + 1];
    }
    out[2 * m] = s;
    out[2 * m + 1] = q;
}

__global__ void adv_stats_finish_kernel(const double* sums, int num_mb, double count, float* st) {
    int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= num_mb) return;
    double mean = sums[2 * m] / count;
    double var = sums[2 * m + 1] / count - mean * mean;
    float fm = (float)mean, fv = (float)var;
    st[2 * m] = fm;
    st[2 * m + 1] = rsqrtf(fmaxf(fv, 1e-5f));
}

// Value normaliser chain over an epoch's minibatches (mlearn_value_norm_chain):
// one thread, the estimates carried from minibatch to minibatch as in
// _ppo_update's train_state.value_normalizer_state (ppo.py:205-211, 346).
// f32 arithmetic in the reference's expression order (moving_avg.py:131-181).
__global__ void value_norm_chain_kernel(const double* sums, const float* adv_st, int num_mb,
                                        double count, float decay, float eps, float* est,
                                        int32_t* nupd, float* rec) {
#pragma clang fp contract(off)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float mu = est[0], sig = est[2], mub = est[3], s2b = est[4];
    float inv = est[1];
    int32_t n = *nupd;
    const float oma = decay, alpha = 1.f - oma;
    for (int m = 0; m < num_mb; ++m) {
        // update_input_stats from zero with n_a = 0: the batch's own mean and
        // population variance
        const double mean = sums[2 * m] / count;
        const double var = sums[2 * m + 1] / count - mean * mean;
        const float xm = (float)mean, xv = (float)(var > 0.0 ? var : 0.0);
        const float delta = xm - mu;
        const int32_t nn = n + 1;
        const float mub2 = oma * mub + alpha * xm;
        const float s2b2 = oma * s2b + alpha * xv + ((float)n / (float)nn) * (oma * alpha) * (delta * delta);
        const float bc = -1.f / expm1f((float)nn * logf(oma));
        const float mu2 = mub2 * bc, s22 = s2b2 * bc;
        const float inv2 = 1.f / sqrtf(fmaxf(s22, eps));
        float* r = rec + 8 * (int64_t)m;
        r[0] = adv_st[2 * m];
        r[1] = adv_st[2 * m + 1];
        r[2] = mu2;
        r[3] = inv2;
        r[4] = mu;
        r[5] = sig;
        r[6] = 0.f;
        r[7] = 0.f;
        mu = mu2;
        inv = inv2;
        sig = 1.f / inv2;
        mub = mub2;
        s2b = s2b2;
        n = nn;
    }
    est[0] = mu;
    est[1] = inv;
    est[2] = sig;
    est[3] = mub;
    est[4] = s2b;
    *nupd = n;
}

// ---------------------------------------------------------------------------
// Rollout post-step (rollouts.py:933-973).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void post_step_kernel(const float* __restrict__ rew,
                                                        const uint8_t* __restrict__ done,
                                                        int64_t N, float* srew, uint8_t* sdone,
                                                        float* env_ret, float* trace, float gamma) {
#pragma clang fp contract(off)
    int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (n >= N) return;
    float r = rew[n];
    uint8_t d = done[n] ? 1 : 0;
    float er = r + gamma * env_ret[n];
    if (trace) trace[n] = er;
    srew[n] = r;
    sdone[n] = d;
    env_ret[n] = d ? 0.f : er;
}

// ---------------------------------------------------------------------------
// Synthetic dummy vec-env (bench/test sim plugin).
// ---------------------------------------------------------------------------
// state[n] = {episode step, env step lo, env step hi, 0}.  A workgroup owns
// EB = 256 / Q envs (Q = ceil(D / 4) <= 64): one lane per (env, 4 features)
// for the observations, then the first EB lanes advance the EB envs (reward,
// done, state) after a barrier that orders every lane's state read before the
// writes.  The reward draws run once per workgroup, in wave 0, instead of one
// extra divergent Philox pass in every wave; 32-bit index math.
__global__ __launch_bounds__(256) void env_step_kernel(int4* state, const int32_t* actions,
                                                       int K, int64_t N, int D, uint32_t k0,
                                                       uint32_t k1, uint32_t eoff, float* obs,
                                                       float* rew, uint8_t* done) {
#pragma clang fp contract(off)
    const int Q = (D + 3) >> 2;
    const int EB = 256 / Q;
    const int tid = (int)threadIdx.x;
    const int ln = (int)((uint32_t)tid / (uint32_t)Q), q = tid - ln * Q;
    const int64_t n0 = (int64_t)blockIdx.x * EB;
    const int64_t n = n0 + ln;
    if (ln < EB && n < N) {
        const uint32_t g = eoff + (uint32_t)n;
        const int4 st = state[n];
        env_obs_quad(obs + n * D + 4 * q, D, k0, k1, g, q, env_step_of(st),
                     (D & 3) == 0 && ((uintptr_t)obs & 15) == 0);
    }
    __syncthreads();
    const int64_t m = n0 + tid;
    if (tid < EB && m < N)
        env_advance(state, actions, K, m, eoff + (uint32_t)m, k0, k1, rew, done, state[m]);
}

// Observation dimensions above 256 (Q > 64): one lane per (env, 4 features),
// the first quad's lane also advances the env (all quads of an env read the
// state in the same pass before that lane's write: Q lanes per env, wave-ordered).
__global__ __launch_bounds__(256) void env_step_wide_kernel(int4* state, const int32_t* actions,
                                                            int K, int64_t N, int D, uint32_t k0,
                                                            uint32_t k1, uint32_t eoff, float* obs,
                                                            float* rew, uint8_t* done) {
#pragma clang fp contract(off)
    const int Q = (D + 3) >> 2;
    const int64_t n = (int64_t)blockIdx.x;
    const uint32_t g = eoff + (uint32_t)n;
    const int4 st = state[n];
    const uint64_t step = ((uint64_t)(uint32_t)st.z << 32) | (uint32_t)st.y;
    for (int q = (int)threadIdx.x; q < Q; q += 256) {
        const u32x4 w = env_obs_words(k0, k1, g, q, step);
        for (int j = 0; j < 4 && 4 * q + j < D; ++j) obs[n * D + 4 * q + j] = env_obs_word(u32x4_get(w, j));
    }
    __syncthreads();
    if (threadIdx.x == 0) env_advance(state, actions, K, n, g, k0, k1, rew, done, st);
}

__global__ __launch_bounds__(256) void env_reset_kernel(int4* state, int64_t N, int D,
                                                        uint32_t k0, uint32_t k1, uint32_t eoff,
                                                        float* obs) {
    const int Q = (D + 3) >> 2;
    int64_t task = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (task >= N * Q) return;
    int64_t n = task / Q;
    int q = (int)(task - n * Q);
    uint32_t g = eoff + (uint32_t)n;
    const u32x4 w = env_obs_words(k0, k1, g, q, 0xffffffffffffffffull);
    for (int j = 0; j < 4 && 4 * q + j < D; ++j) obs[n * D + 4 * q + j] = env_obs_word(u32x4_get(w, j));
    if (q == 0) state[n] = make_int4((int)(g % (uint32_t)env_episode_len(g)), 0, 0, 0);
}

struct Deltas {
    uint64_t d[8];
};
__global__ void counters_add_kernel(uint64_t* ctr, int n, Deltas d) {
    int i = threadIdx.x;
    if (i < n) ctr[i] += d.d[i];
}


// ---------------------------------------------------------------------------
// ObservationsEMANormalizer statistics (moving_avg.py:48-196): one block per
// feature.  Per step t the tile partials {mean, M2} are merged (Chan, fixed
// order: thread j of the step's group takes tiles j, j + 8, ..., then a
// butterfly over the 8 threads) into the batch mean and population variance;
// thread 0 folds the steps with update_input_stats (n_a = t) and applies
// update_estimates.  f32 arithmetic like the reference.
// ---------------------------------------------------------------------------
constexpr int kObsGroup = 8;

__device__ inline void chan_merge(float& n, float& m, float& M2, float nb, float mb, float M2b) {
    if (nb == 0.f) return;
    const float nn = n + nb;
    const float d = mb - m;
    m = m + d * (nb / nn);
    M2 = M2 + M2b + d * d * (n * nb / nn);
    n = nn;
}

// EMANormalizer.update_estimates (moving_avg.py:132-180) of column f:
// est = [5][D] mu, inv_sigma, sigma, mu_biased, sigma_sq_biased; Nold = the
// update count before this update.
__device__ inline void ema_update_col(int f, int D, float a_mean, float a_var, float decay,
                                      float eps, float* est, int32_t Nold) {
#pragma clang fp contract(off)
    float* mu = est;
    float* inv_sigma = est + D;
    float* sigma = est + 2 * D;
    float* mu_b = est + 3 * D;
    float* s2_b = est + 4 * D;
    const float oma = decay;
    const float alpha = 1.0f - oma;
    const int32_t Nnew = Nold + 1;
    const float mean_delta = a_mean - mu[f];
    const float nmb = oma * mu_b[f] + alpha * a_mean;
    const float ns2b = oma * s2_b[f] + alpha * a_var +
                       ((float)Nold / (float)Nnew) * (oma * alpha) * (mean_delta * mean_delta);
    const float bc = -1.0f / expm1f((float)Nnew * logf(oma));
    const float nmu = nmb * bc;
    const float ns2 = ns2b * bc;
    const float ninv = rsqrtf(fmaxf(ns2, eps));
    mu[f] = nmu;
    inv_sigma[f] = ninv;
    sigma[f] = 1.0f / ninv;
    mu_b[f] = nmb;
    s2_b[f] = ns2b;
}

// EMANormalizer.update_input_stats (moving_avg.py:107-130) of a [rows][D]
// f32 batch: per column (one block each) the batch mean and population
// variance by Chan merges of the threads' Welford partials in a fixed tree
// order, then the weighted merge with the running (mean, var) at
// num_prev_updates = n_a.  cur and out are [2][D] (mean | var; may alias).
__global__ __launch_bounds__(256) void ema_input_stats_kernel(const float* __restrict__ x,
                                                              int64_t rows, int D,
                                                              const float* cur, int n_prev,
                                                              float* out) {
#pragma clang fp contract(off)
    __shared__ float sn[4], sm[4], sM[4];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float n = 0.f, m = 0.f, M2 = 0.f;
    for (int64_t r = tid; r < rows; r += 256) chan_merge(n, m, M2, 1.f, x[r * D + f], 0.f);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float n2 = __shfl_xor(n, o), m2 = __shfl_xor(m, o), M22 = __shfl_xor(M2, o);
        if ((lane & o) == 0) {
            chan_merge(n, m, M2, n2, m2, M22);
        } else {  // the lower lane is the left operand on both sides
            float nl = n2, ml = m2, Ml = M22;
            chan_merge(nl, ml, Ml, n, m, M2);
            n = nl, m = ml, M2 = Ml;
        }
    }
    if (lane == 0) {
        sn[w] = n;
        sm[w] = m;
        sM[w] = M2;
    }
    __syncthreads();
    if (tid != 0) return;
    n = sn[0], m = sm[0], M2 = sM[0];
    for (int u = 1; u < 4; ++u) chan_merge(n, m, M2, sn[u], sm[u], sM[u]);
    const float b_mean = m, b_var = rows > 0 ? M2 / (float)rows : 0.f;
    const float a_mean = cur[f], a_var = cur[D + f];
    const float delta = b_mean - a_mean;
    const float b_w = 1.0f / (float)(n_prev + 1);
    const float a_w = 1.0f - b_w;
    out[f] = a_mean + delta * b_w;
    out[D + f] = a_w * a_var + b_w * b_var + (delta * delta) * a_w * b_w;
}

__global__ void ema_update_kernel(const float* __restrict__ stats, int D, float decay, float eps,
                                  float* est, const int32_t* count) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < D) ema_update_col(f, D, stats[f], stats[D + f], decay, eps, est, *count);
}

__global__ __launch_bounds__(256) void obs_norm_update_kernel(const float* __restrict__ st,
                                                              int steps, int64_t tiles, int64_t N,
                                                              int D, float decay, float eps,
                                                              float* est, int32_t* count) {
#pragma clang fp contract(off)
    __shared__ float bm[256 / kObsGroup], bv[256 / kObsGroup];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int g = tid / kObsGroup, j = tid % kObsGroup;
    constexpr int SPB = 256 / kObsGroup;  // steps per pass
    float a_mean = 0.f, a_var = 0.f;      // init_input_stats (moving_avg.py:101-105)
    for (int t0 = 0; t0 < steps; t0 += SPB) {
        const int t = t0 + g;
        float n = 0.f, m = 0.f, M2 = 0.f;
        if (t < steps) {
            for (int64_t tile = j; tile < tiles && tile * 32 < N; tile += kObsGroup) {
                const float nb = (float)(N - tile * 32 < 32 ? N - tile * 32 : 32);
                const float* p = st + (((int64_t)t * tiles + tile) * D + f) * 2;
                chan_merge(n, m, M2, nb, p[0], p[1]);
            }
        }
#pragma unroll
        for (int o = 1; o < kObsGroup; o <<= 1) {
            const float n2 = __shfl_xor(n, o), m2 = __shfl_xor(m, o), M22 = __shfl_xor(M2, o);
            // fixed operand order: the lower group index is the left operand
            if ((j & o) == 0) {
                chan_merge(n, m, M2, n2, m2, M22);
            } else {
                float nl = n2, ml = m2, Ml = M22;
                chan_merge(nl, ml, Ml, n, m, M2);
                n = nl, m = ml, M2 = Ml;
            }
        }
        if (j == 0) {
            bm[g] = m;
            bv[g] = M2 / (float)N;
        }
        __syncthreads();
        if (tid == 0) {
            for (int u = 0; u < SPB && t0 + u < steps; ++u) {
                // update_input_stats (moving_avg.py:107-130) with n_a = t
                const float b_mean = bm[u], b_var = bv[u];
                const float delta = b_mean - a_mean;
                const float b_w = 1.0f / (float)(t0 + u + 1);
                const float a_w = 1.0f - b_w;
                a_mean = a_mean + delta * b_w;
                a_var = a_w * a_var + b_w * b_var + (delta * delta) * a_w * b_w;
            }
        }
        __syncthreads();
    }
    if (tid != 0) return;
    // update_estimates (moving_avg.py:132-180)
    ema_update_col(f, D, a_mean, a_var, decay, eps, est, *count);  // count bumped after every block
}

__global__ void obs_count_kernel(int32_t* count) { *count += 1; }

// The LSTM gate activations of the fused kernels (rowtile.h sigmoidf /
// tanh_fast) over an array: the accuracy pin of tests/test_gpu_kernels.py.
__global__ void activations_kernel(const float* x, int64_t n, float* sig, float* th) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    sig[i] = sigmoidf(x[i]);
    th[i] = tanh_fast(x[i]);
}

}  // namespace ml

using namespace ml;

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char* mlearn_last_error(void) { return ml::g_err; }
int mlearn_abi_version(void) { return MLEARN_ABI_VERSION; }

int mlearn_philox4x32(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out, int64_t n,
                      mlearn_stream_t stream) {
    ML_REQUIRE(n >= 0, "philox: n < 0");
    ML_REQUIRE(n == 0 || (ctr && out), "philox: null pointer");
    if (n == 0) return MLEARN_OK;
    hipLaunchKernelGGL(philox_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, S(stream),
                       (const uint4*)ctr, k0, k1, (uint4*)out, n);
    return check_launch("philox");
}

int mlearn_lstm_activations_f32(const float* x, int64_t n, float* sigmoid_out, float* tanh_out,
                                mlearn_stream_t stream) {
    ML_REQUIRE(n >= 0, "lstm_activations: n < 0");
    if (n == 0) return MLEARN_OK;
    ML_REQUIRE(x && sigmoid_out && tanh_out, "lstm_activations: null pointer");
    hipLaunchKernelGGL(ml::activations_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       S(stream), x, n, sigmoid_out, tanh_out);
    return check_launch("lstm_activations");
}

int mlearn_philox4x32_host(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out,
                           int64_t n) {
    ML_REQUIRE(n >= 0, "philox_host: n < 0");
    ML_REQUIRE(n == 0 || (ctr && out), "philox_host: null pointer");
    for (int64_t i = 0; i < n; ++i) {
        const u32x4 r = philox4x32(u32x4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]},
                                   k0, k1);
        out[4 * i] = r.x;
        out[4 * i + 1] = r.y;
        out[4 * i + 2] = r.z;
        out[4 * i + 3] = r.w;
    }
    return MLEARN_OK;
}

int mlearn_gae_f32(const float* rewards, const float* values, const uint8_t* dones,
                   const float* bootstrap, float* advantages, float* returns, int32_t T, int64_t N,
                   float gamma, float gamma_lambda, mlearn_stream_t stream) {
    ML_REQUIRE(T >= 0 && N >= 0, "gae: negative size");
    if (T == 0 || N == 0) return MLEARN_OK;
    ML_REQUIRE(rewards && values && dones && bootstrap && advantages,
               "gae: null pointer");  // (returns may be NULL: not materialised)
    ML_REQUIRE(N <= ((int64_t)1 << 28), "gae: N > 2^28 columns");
    // cfg.gamma * cfg.gae_lambda (algo_common.py:120): one f64 product of the
    // Python floats rounded to f32 once, formed by the caller
    const float gl = gamma_lambda;
    // Blocks of 64 below 2^20 columns so more CUs share the serial T loop (the
    // operating point N = 8192 is latency-bound), 256 above (HBM-bound).
    if (N >= (int64_t)1 << 20) {
        hipLaunchKernelGGL((gae_kernel<1, 8>), dim3(grid_for(N, 256)), dim3(256), 0, S(stream),
                           rewards, values, dones, bootstrap, advantages, returns, T, N, gamma,
                           gl, (const float*)nullptr, (int64_t)1);
    } else {
        hipLaunchKernelGGL((gae_kernel<1, 16>), dim3(grid_for(N, 64)), dim3(64), 0, S(stream),
                           rewards, values, dones, bootstrap, advantages, returns, T, N, gamma,
                           gl, (const float*)nullptr, (int64_t)1);
    }
    return check_launch("gae");
}

int mlearn_gae_vnorm_f32(const float* rewards, const float* values, const uint8_t* dones,
                         const float* bootstrap, const float* value_norm, int64_t cols_per_norm,
                         float* advantages, float* returns, int32_t T, int64_t N, float gamma,
                         float gamma_lambda, mlearn_stream_t stream) {
    ML_REQUIRE(T >= 0 && N >= 0, "gae_vnorm: negative size");
    if (T == 0 || N == 0) return MLEARN_OK;
    ML_REQUIRE(rewards && values && dones && bootstrap && advantages && returns && value_norm,
               "gae_vnorm: null pointer");
    ML_REQUIRE(cols_per_norm >= 1 && N % cols_per_norm == 0,
               "gae_vnorm: N must be a multiple of cols_per_norm");
    ML_REQUIRE(N <= ((int64_t)1 << 28), "gae_vnorm: N > 2^28 columns");
    const float gl = gamma_lambda;  // formed by the caller, as in mlearn_gae_f32
    hipLaunchKernelGGL((gae_kernel<1, 16>), dim3(grid_for(N, 64)), dim3(64), 0, S(stream), rewards,
                       values, dones, bootstrap, advantages, returns, T, N, gamma, gl, value_norm,
                       cols_per_norm);
    return check_launch("gae_vnorm");
}

int mlearn_returns_f32(const float* rewards, const uint8_t* dones, const float* bootstrap,
                       float* returns, int32_t T, int64_t N, float gamma, mlearn_stream_t stream) {
    ML_REQUIRE(T >= 0 && N >= 0, "returns: negative size");
    if (T == 0 || N == 0) return MLEARN_OK;
    ML_REQUIRE(rewards && dones && bootstrap && returns, "returns: null pointer");
    hipLaunchKernelGGL(returns_kernel, dim3(grid_for(N, 256)), dim3(256), 0, S(stream), rewards,
                       dones, bootstrap, returns, T, N, gamma);
    return check_launch("returns");
}

int64_t mlearn_zscore_workspace_bytes(int64_t n) { return 256 * 2 * sizeof(double); }

int mlearn_zscore_f32(const float* x, int64_t n, float* out, void* ws, mlearn_stream_t stream) {
    ML_REQUIRE(n > 0, "zscore: n must be > 0");
    ML_REQUIRE(x && out && ws, "zscore: null pointer");
    int g = grid_for(n, 256, 256);
    hipLaunchKernelGGL(sum_partial_kernel, dim3(g), dim3(256), 0, S(stream), x, n, (double*)ws);
    hipLaunchKernelGGL(zscore_apply_kernel, dim3(grid_for(n, 256, 2048)), dim3(256), 0, S(stream),
                       x, n, (const double*)ws, g, out);
    return check_launch("zscore");
}

static int check_layout(const mlearn_action_layout& l) {
    ML_REQUIRE(l.num_groups >= 1 && l.num_groups <= MLEARN_MAX_GROUPS, "action layout: bad K=%d",
               l.num_groups);
    ML_REQUIRE(l.num_logits >= 1 && l.num_logits < MLEARN_HEAD_COLS, "action layout: bad A=%d",
               l.num_logits);
    ML_REQUIRE(l.offsets[0] == 0 && l.offsets[l.num_groups] == l.num_logits,
               "action layout: offsets do not span the logits");
    for (int k = 0; k < l.num_groups; ++k)
        ML_REQUIRE(l.offsets[k + 1] > l.offsets[k], "action layout: empty group %d", k);
    return MLEARN_OK;
}

int mlearn_counters_add(uint64_t* ctr, int32_t n, const uint64_t* deltas, mlearn_stream_t stream) {
    ML_REQUIRE(ctr && deltas && n >= 1 && n <= 8, "counters_add: bad args");
    Deltas d{};
    for (int i = 0; i < n; ++i) d.d[i] = deltas[i];
    hipLaunchKernelGGL(counters_add_kernel, dim3(1), dim3(64), 0, S(stream), ctr, n, d);
    return check_launch("counters_add");
}

int mlearn_discrete_sample_f32(const float* logits, int64_t ld, mlearn_action_layout layout,
                               int64_t N, uint32_t k0, uint32_t k1, const uint64_t* step_ctr,
                               uint64_t step, uint32_t env_offset, int32_t sample,
                               int32_t* actions, float* log_probs, mlearn_stream_t stream) {
    int rc = check_layout(layout);
    if (rc) return rc;
    ML_REQUIRE(N >= 0 && ld >= layout.num_logits, "sample: bad N/ld");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(logits && actions && (log_probs || !sample), "sample: null pointer");
    int64_t tasks = N * layout.num_groups;
    hipLaunchKernelGGL(sample_kernel, dim3(grid_for(tasks, 256)), dim3(256), 0, S(stream), logits,
                       ld, to_layout(layout), N, k0, k1, step_ctr, step, env_offset, sample,
                       actions, log_probs);
    return check_launch("discrete_sample");
}

int mlearn_action_stats_f32(const float* logits, int64_t ld, mlearn_action_layout layout,
                            int64_t N, const int32_t* actions, float* log_probs, float* entropies,
                            mlearn_stream_t stream) {
    int rc = check_layout(layout);
    if (rc) return rc;
    ML_REQUIRE(N >= 0 && ld >= layout.num_logits, "action_stats: bad N/ld");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(logits && actions && log_probs && entropies, "action_stats: null pointer");
    int64_t tasks = N * layout.num_groups;
    hipLaunchKernelGGL(action_stats_kernel, dim3(grid_for(tasks, 256)), dim3(256), 0, S(stream),
                       logits, ld, to_layout(layout), N, actions, log_probs, entropies);
    return check_launch("action_stats");
}

int64_t mlearn_metrics_workspace_bytes(int32_t num_jobs) {
    return (int64_t)num_jobs * kMetricBlocks * 4 * sizeof(double);
}

int mlearn_metrics_f32(const mlearn_metric_job* jobs, int32_t num_jobs, float* out, void* ws,
                       mlearn_stream_t stream) {
    ML_REQUIRE(num_jobs >= 1 && num_jobs <= 16, "metrics: 1..16 jobs");
    ML_REQUIRE(jobs && out && ws, "metrics: null pointer");
    MetricJobs J;
    for (int i = 0; i < num_jobs; ++i) {
        ML_REQUIRE(jobs[i].n >= 0 && (jobs[i].n == 0 || jobs[i].x), "metrics: bad job %d", i);
        ML_REQUIRE(jobs[i].cols >= 0 && (jobs[i].cols == 0 || (jobs[i].ld >= jobs[i].cols &&
                                                                jobs[i].n % jobs[i].cols == 0)),
                   "metrics: job %d window (cols %lld, ld %lld) does not tile n", i,
                   (long long)jobs[i].cols, (long long)jobs[i].ld);
        J.j[i] = jobs[i];
    }
    hipLaunchKernelGGL(metrics_partial_kernel, dim3(kMetricBlocks, num_jobs), dim3(256), 0,
                       S(stream), J, (double*)ws);
    hipLaunchKernelGGL(metrics_finish_kernel, dim3(num_jobs), dim3(64), 0, S(stream), J,
                       (const double*)ws, out);
    return check_launch("metrics");
}

int mlearn_minibatch_perm(uint32_t k0, uint32_t k1, const uint64_t* epoch_ctr, uint64_t epoch,
                          uint32_t rank, int32_t n, int32_t* perm, mlearn_stream_t stream) {
    ML_REQUIRE(n >= 1 && n <= (1 << 30), "perm: n must be in [1, 2^30], got %d", n);
    ML_REQUIRE(perm, "perm: null pointer");
    int b = 2;
    while ((1ll << b) < n) ++b;
    if (b & 1) ++b;
    hipLaunchKernelGGL(perm_kernel, dim3((n + 255) / 256), dim3(256), 0, S(stream), k0, k1,
                       epoch_ctr, epoch, rank, n, b / 2, perm);
    return check_launch("minibatch_perm");
}

static int minibatch_sums(const mlearn_rollout_view* ro, const float* src, const int32_t* perm,
                          int32_t num_mb, int32_t mb_size, double* partials, hipStream_t stream);

int mlearn_adv_stats(const mlearn_rollout_view* ro, const int32_t* perm, int32_t num_mb,
                     int32_t mb_size, double* partials, mlearn_stream_t stream) {
    ML_REQUIRE(ro && perm && partials, "adv_stats: null pointer");
    return minibatch_sums(ro, ro->advantages, perm, num_mb, mb_size, partials, S(stream));
}

int mlearn_return_stats(const mlearn_rollout_view* ro, const int32_t* perm, int32_t num_mb,
                        int32_t mb_size, double* partials, mlearn_stream_t stream) {
    ML_REQUIRE(ro && perm && partials && ro->returns,
               "return_stats: null pointer (the value normaliser needs materialised returns)");
    return minibatch_sums(ro, ro->returns, perm, num_mb, mb_size, partials, S(stream));
}

int mlearn_value_norm_chain(const double* return_sums, const float* adv_stats, int32_t num_mb,
                            double count, float decay, float eps, float* est, int32_t* n_updates,
                            float* records, mlearn_stream_t stream) {
    ML_REQUIRE(return_sums && adv_stats && est && n_updates && records, "value_norm: null pointer");
    ML_REQUIRE(num_mb >= 1 && count > 0, "value_norm: bad sizes");
    ML_REQUIRE(decay > 0.f && decay < 1.f && eps > 0.f, "value_norm: bad decay / eps");
    hipLaunchKernelGGL(value_norm_chain_kernel, dim3(1), dim3(64), 0, S(stream), return_sums,
                       adv_stats, num_mb, count, decay, eps, est, n_updates, records);
    return check_launch("value_norm_chain");
}

static int minibatch_sums(const mlearn_rollout_view* ro, const float* src, const int32_t* perm,
                          int32_t num_mb, int32_t mb_size, double* partials, hipStream_t stream) {
    ML_REQUIRE(src, "minibatch sums: null source array");
    ML_REQUIRE(num_mb >= 1 && mb_size >= 1, "adv_stats: bad minibatch sizes");
    ML_REQUIRE(ro->bptt_len >= 1 && ro->T % ro->bptt_len == 0, "adv_stats: bad bptt_len");
    ML_REQUIRE((int64_t)num_mb * mb_size <= (ro->T / ro->bptt_len) * ro->N,
               "adv_stats: minibatches exceed the sequences");
    // partials layout: [num_mb][kStatBlocks][2] scratch followed by [num_mb][2] sums
    double* scratch = partials + 2 * num_mb;
    mlearn_rollout_view v = *ro;
    if (v.ld == 0) v.ld = v.N;
    ML_REQUIRE(v.ld >= v.N, "adv_stats: ld %lld < N %lld", (long long)v.ld, (long long)v.N);
    hipLaunchKernelGGL(adv_stats_kernel, dim3(num_mb, kStatBlocks), dim3(256), 0, stream, v, src,
                       perm, mb_size, scratch);
    hipLaunchKernelGGL(adv_stats_reduce_kernel, dim3((num_mb + 63) / 64), dim3(64), 0, stream,
                       (const double*)scratch, num_mb, partials);
    return check_launch("adv_stats");
}

int mlearn_adv_stats_finish(const double* partials, int32_t num_mb, double count, float* stats,
                            mlearn_stream_t stream) {
    ML_REQUIRE(partials && stats && num_mb >= 1 && count > 0, "adv_stats_finish: bad args");
    hipLaunchKernelGGL(adv_stats_finish_kernel, dim3((num_mb + 63) / 64), dim3(64), 0, S(stream),
                       partials, num_mb, count, stats);
    return check_launch("adv_stats_finish");
}

int mlearn_rollout_post_step(const float* rewards, const uint8_t* dones, int64_t N,
                             float* store_rewards, uint8_t* store_dones, float* env_returns,
                             float* env_returns_trace, float gamma, mlearn_stream_t stream) {
    ML_REQUIRE(N >= 0, "post_step: N < 0");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(rewards && dones && store_rewards && store_dones && env_returns,
               "post_step: null pointer");
    hipLaunchKernelGGL(post_step_kernel, dim3(grid_for(N, 256)), dim3(256), 0, S(stream), rewards,
                       dones, N, store_rewards, store_dones, env_returns, env_returns_trace, gamma);
    return check_launch("post_step");
}

int mlearn_dummy_env_step(int32_t* state, const int32_t* actions, int32_t K, int64_t N,
                          int32_t obs_dim, uint32_t k0, uint32_t k1, uint32_t env_offset,
                          float* obs, float* rewards, uint8_t* dones, mlearn_stream_t stream) {
    ML_REQUIRE(N >= 0 && obs_dim >= 1 && K >= 1, "env_step: bad sizes");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(state && obs && rewards && dones, "env_step: null pointer");
    ML_REQUIRE((uintptr_t)state % 16 == 0, "env_step: state must be 16-byte aligned");
    const int Q = (obs_dim + 3) / 4;
    if (Q <= 64) {
        const int EB = 256 / Q;
        hipLaunchKernelGGL(env_step_kernel, dim3((unsigned)((N + EB - 1) / EB)), dim3(256), 0,
                           S(stream), (int4*)state, actions, K, N, obs_dim, k0, k1, env_offset,
                           obs, rewards, dones);
    } else {
        hipLaunchKernelGGL(env_step_wide_kernel, dim3((unsigned)N), dim3(256), 0, S(stream),
                           (int4*)state, actions, K, N, obs_dim, k0, k1, env_offset, obs, rewards,
                           dones);
    }
    return check_launch("env_step");
}

int mlearn_dummy_env_reset(int32_t* state, int64_t N, int32_t obs_dim, uint32_t k0, uint32_t k1,
                           uint32_t env_offset, float* obs, mlearn_stream_t stream) {
    ML_REQUIRE(N >= 0 && obs_dim >= 1, "env_reset: bad sizes");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(state && obs, "env_reset: null pointer");
    ML_REQUIRE((uintptr_t)state % 16 == 0, "env_reset: state must be 16-byte aligned");
    hipLaunchKernelGGL(env_reset_kernel, dim3(grid_for(N * ((obs_dim + 3) / 4), 256)), dim3(256), 0,
                       S(stream), (int4*)state, N, obs_dim, k0, k1, env_offset, obs);
    return check_launch("env_reset");
}

int mlearn_obs_norm_update(const float* obs_stats, int32_t steps, int64_t tiles, int64_t N,
                           int32_t obs_dim, float decay, float eps, float* est, int32_t* count,
                           mlearn_stream_t stream) {
    ML_REQUIRE(obs_stats && est && count, "obs_norm_update: null pointer");
    ML_REQUIRE(steps >= 1 && N >= 1 && tiles >= (N + 31) / 32 && obs_dim >= 1,
               "obs_norm_update: bad sizes");
    ML_REQUIRE(decay > 0.f && decay < 1.f && eps > 0.f, "obs_norm_update: bad decay / eps");
    hipLaunchKernelGGL(obs_norm_update_kernel, dim3((unsigned)obs_dim), dim3(256), 0, S(stream),
                       obs_stats, steps, tiles, N, obs_dim, decay, eps, est, count);
    hipLaunchKernelGGL(obs_count_kernel, dim3(1), dim3(1), 0, S(stream), count);
    return check_launch("obs_norm_update");
}

int mlearn_ema_input_stats(const float* x, int64_t rows, int32_t dim, const float* cur_stats,
                           int32_t num_prev_updates, float* out_stats, mlearn_stream_t stream) {
    ML_REQUIRE(rows >= 0 && dim >= 1 && num_prev_updates >= 0, "ema_input_stats: bad sizes");
    ML_REQUIRE((x || rows == 0) && cur_stats && out_stats, "ema_input_stats: null pointer");
    ML_REQUIRE(rows < ((int64_t)1 << 24), "ema_input_stats: rows >= 2^24 (f32 counts)");
    hipLaunchKernelGGL(ema_input_stats_kernel, dim3((unsigned)dim), dim3(256), 0, S(stream), x,
                       rows, dim, cur_stats, num_prev_updates, out_stats);
    return check_launch("ema_input_stats");
}

int mlearn_ema_update_estimates(const float* input_stats, int32_t dim, float decay, float eps,
                                float* est, int32_t* count, mlearn_stream_t stream) {
    ML_REQUIRE(dim >= 1 && input_stats && est && count, "ema_update_estimates: bad arguments");
    ML_REQUIRE(decay > 0.f && decay < 1.f, "ema_update_estimates: decay must be in (0, 1)");
    hipLaunchKernelGGL(ema_update_kernel, dim3((unsigned)((dim + 255) / 256)), dim3(256), 0,
                       S(stream), input_stats, dim, decay, eps, est, count);
    hipLaunchKernelGGL(obs_count_kernel, dim3(1), dim3(1), 0, S(stream), count);
    return check_launch("ema_update_estimates");
}

}  // extern "C"
