// Fused rollout step: ObservationsCaster -> MLP trunk (Dense no-bias ->
// LayerNorm -> ReLU per layer) -> actor logits + critic -> Gumbel-max sample
// -> rollout store, in ONE launch per step (the reference runs these as
// dozens of XLA fusions per step inside rollout_loop, rollouts.py:867-901).
//
// Reference numerics mirrored (models.py:46-56, 99-154; flax 0.8.1):
//   Dense output rounded to the compute dtype; LayerNorm statistics in f32
//   with fast variance max(E[x^2]-E[x]^2, 0), eps 1e-6, y = (x-mean)*(rstd*g)+b
//   rounded to the compute dtype; heads: rnd(rnd(x.W) + rnd(b)); critic and
//   logits upcast to f32 (dists.py:22, models.py:154).

#include "common.h"
#include "dists.h"
#include "rowtile.h"

namespace ml {

PolicyK make_policy_k(const mlearn_mlp_policy& p) {
    PolicyK k;
    k.D = p.obs_dim;
    k.H = p.hidden;
    k.L = p.num_layers;
    k.K = p.actions.num_groups;
    k.A = p.actions.num_logits;
    for (int i = 0; i <= MLEARN_MAX_GROUPS; ++i) k.off[i] = p.actions.offsets[i];
    for (int l = 0; l < MLEARN_MAX_LAYERS; ++l) {
        k.wt[l] = p.w_t[l];
        k.w[l] = p.w[l];
        k.lns[l] = p.ln_scale[l];
        k.lnb[l] = p.ln_bias[l];
    }
    k.head_t = p.head_t;
    k.head = p.head;
    k.head_b = p.head_bias;
    return k;
}

int validate_policy(const mlearn_mlp_policy* p) {
    ML_REQUIRE(p, "policy: null descriptor");
    ML_REQUIRE(p->dtype == MLEARN_DTYPE_F32 || p->dtype == MLEARN_DTYPE_BF16, "policy: bad dtype");
    ML_REQUIRE(p->hidden == 64 || p->hidden == 128 || p->hidden == 256,
               "policy: hidden must be 64, 128 or 256 (got %d)", p->hidden);
    ML_REQUIRE(p->obs_dim >= 16 && p->obs_dim <= 256 && p->obs_dim % 16 == 0,
               "policy: obs_dim must be a multiple of 16 in [16, 256] (got %d)", p->obs_dim);
    ML_REQUIRE(p->num_layers >= 1 && p->num_layers <= MLEARN_MAX_LAYERS, "policy: bad num_layers");
    const mlearn_action_layout& l = p->actions;
    ML_REQUIRE(l.num_groups >= 1 && l.num_groups <= MLEARN_MAX_GROUPS, "policy: bad num_groups");
    ML_REQUIRE(l.num_logits >= 1 && l.num_logits + 1 <= MLEARN_HEAD_COLS,
               "policy: at most %d logits", MLEARN_HEAD_COLS - 1);
    ML_REQUIRE(l.offsets[0] == 0 && l.offsets[l.num_groups] == l.num_logits,
               "policy: bad action offsets");
    for (int k = 0; k < l.num_groups; ++k)
        ML_REQUIRE(l.offsets[k + 1] > l.offsets[k], "policy: empty action group %d", k);
    for (int i = 0; i < p->num_layers; ++i)
        ML_REQUIRE(p->w_t[i] && (i == 0 || p->w[i]) && p->ln_scale[i] && p->ln_bias[i],
                   "policy: null layer %d weights", i);
    ML_REQUIRE(p->head_t && p->head && p->head_bias, "policy: null head weights");
    return MLEARN_OK;
}

// One wave = 32 environments (one per lane pair), all H features: the trunk,
// heads and sampling of its rows run without any workgroup barrier.  The
// workgroup's waves share the LayerNorm parameters staged once in LDS.
constexpr int kPolicyWaves = 1;  // waves per workgroup (grid = one wave per 32 envs)

template <typename T, int H>
__global__ __launch_bounds__(64 * kPolicyWaves) void policy_step_kernel(
    PolicyK P, const float* __restrict__ obs, int64_t N, T* obs_store, int32_t* actions,
    float* logp, float* values, uint32_t k0, uint32_t k1, const uint64_t* step_ctr,
    uint64_t step_add, uint32_t eoff, int sample) {
    typedef typename RT<T>::frag frag;
    constexpr int NB = H / 32, KS = RT<T>::KS, SPB = RT<T>::SPB, KSH = H / KS;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D, L = P.L;
    float* gb = (float*)smem;            // [L][2][H]
    float* hbias = gb + L * 2 * H;       // [32]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
    for (int i = tid; i < L * 2 * H + MLEARN_HEAD_COLS; i += blockDim.x) {
        float v;
        if (i < L * 2 * H) {
            const int l = i / (2 * H), c = i - l * 2 * H;
            v = c < H ? P.lns[l][c] : P.lnb[l][c - H];
        } else {
            v = P.head_b[i - L * 2 * H];
        }
        gb[i] = v;
    }
    __syncthreads();
    float* lg = hbias + MLEARN_HEAD_COLS + w * (32 * 33);  // [32][33] per wave
    const int64_t row0 = ((int64_t)blockIdx.x * kPolicyWaves + w) * 32;
    if (row0 >= N) return;
    const int64_t row = row0 + r;
    const bool live = row < N;
    const uint64_t step = (step_ctr ? *step_ctr : 0ull) + step_add;
    const float invH = 1.0f / (float)H;

    // layer 0: observation fragments straight from the env output (cast to
    // the compute dtype = ObservationsCaster), copied to the rollout store
    f32x16 acc[NB];
    zero_acc<NB>(acc);
    {
        const float* orow = obs + (live ? row : 0) * D;
        T* srow = obs_store ? obs_store + (live ? row : 0) * D : nullptr;
        const int nks = D / KS;
        const T* img = (const T*)P.wt[0] + lane * RT<T>::E;
        for (int s = 0; s < nks; ++s) {
            const frag b = live ? RT<T>::row(orow, s, h) : RT<T>::zero();
            if (srow && live) RT<T>::put_row(srow, s, h, b);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
                acc[nb] = MT<T>::mma(MT<T>::load(img + (nb * nks + s) * 64 * RT<T>::E), b, acc[nb]);
        }
    }
    frag bf[KSH];
    for (int l = 0;; ++l) {
        // LayerNorm + ReLU (models.py:46-56), statistics per row = per lane
        float sum = 0.f, sq = 0.f;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const float x = rnd<T>(acc[nb][q]);
                acc[nb][q] = x;
                sum += x;
                sq += x * x;
            }
        sum = sum_halves(sum);
        sq = sum_halves(sq);
        const float mean = sum * invH;
        const float var = fmaxf(sq * invH - mean * mean, 0.f);
        const float rstd = rsqrtf(var + 1e-6f);
        const float* gm = gb + l * 2 * H;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f0 = nb * 32 + 8 * g + 4 * h;
                const float4 G = *(const float4*)(gm + f0), B = *(const float4*)(gm + H + f0);
                const float gg[4] = {G.x, G.y, G.z, G.w}, bb[4] = {B.x, B.y, B.z, B.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = 4 * g + j;
                    acc[nb][q] = fmaxf(rnd<T>((acc[nb][q] - mean) * (rstd * gg[j]) + bb[j]), 0.f);
                }
            }
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int t = 0; t < SPB; ++t) bf[nb * SPB + t] = RT<T>::from_acc(acc[nb], t);
        if (l + 1 == L) break;
        zero_acc<NB>(acc);
        gemm_rb<T, NB, KSH, 2>(acc, bf, (const T*)P.wt[l + 1], lane);
    }

    // actor + critic heads: lg[row][j] = rnd(rnd(a . W) + rnd(b)) (dists.py:22)
    {
        f32x16 ha[1];
        zero_acc<1>(ha);
        gemm_rb<T, 1, KSH, 8>(ha, bf, (const T*)P.head_t, lane);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int j = feat(0, q, h);
            lg[r * 33 + j] = rnd<T>(rnd<T>(ha[0][q]) + rnd<T>(hbias[j]));
        }
    }
    wave_lds_sync();

    // sample: lane half h takes the action groups g = h, h + 2, ...
    if (live) {
        const float* lr = lg + r * 33;
        if (actions) {
            for (int g = h; g < P.K; g += 2) {
                int a;
                float lp;
                sample_group(lr + P.off[g], P.off[g + 1] - P.off[g], P.off[g], k0, k1,
                             eoff + (uint32_t)row, step, sample, &a, &lp);
                actions[row * P.K + g] = a;
                if (logp) logp[row * P.K + g] = lp;
            }
        }
        if (values && h == 0) values[row] = lr[P.A];
    }
}

static size_t policy_step_lds(int L, int H) {
    return (size_t)(L * 2 * H + MLEARN_HEAD_COLS) * 4 + (size_t)kPolicyWaves * 32 * 33 * 4;
}

template <typename T, int H>
static int launch_policy_step(const PolicyK& P, const float* obs, int64_t N, void* obs_store,
                              int32_t* actions, float* logp, float* values, uint32_t k0, uint32_t k1,
                              const uint64_t* step_ctr, uint64_t step, uint32_t eoff, int sample,
                              hipStream_t s) {
    const size_t lds = policy_step_lds(P.L, H);
    const int64_t tiles = (N + 31) / 32;
    const int grid = (int)((tiles + kPolicyWaves - 1) / kPolicyWaves);
    hipLaunchKernelGGL((policy_step_kernel<T, H>), dim3(grid), dim3(64 * kPolicyWaves), lds, s, P,
                       obs, N, (T*)obs_store, actions, logp, values, k0, k1, step_ctr, step, eoff,
                       sample);
    return check_launch("policy_rollout_step");
}

}  // namespace ml

using namespace ml;

extern "C" int mlearn_policy_rollout_step(const mlearn_mlp_policy* policy, const float* obs,
                                          int64_t N, void* obs_store, int32_t* actions,
                                          float* log_probs, float* values, uint32_t k0,
                                          uint32_t k1, const uint64_t* step_ctr, uint64_t step,
                                          uint32_t env_offset, int32_t sample,
                                          mlearn_stream_t stream) {
    int rc = validate_policy(policy);
    if (rc) return rc;
    ML_REQUIRE(N >= 0, "policy_rollout_step: N < 0");
    if (N == 0) return MLEARN_OK;
    ML_REQUIRE(obs, "policy_rollout_step: null obs");
    ML_REQUIRE(!actions || log_probs || !sample, "policy_rollout_step: sampling needs log_probs");
    ML_REQUIRE(actions || values, "policy_rollout_step: nothing to compute");
    ML_REQUIRE((uintptr_t)obs % 16 == 0, "policy_rollout_step: obs must be 16-byte aligned");
    ML_REQUIRE(!obs_store || (uintptr_t)obs_store % 16 == 0,
               "policy_rollout_step: obs_store must be 16-byte aligned");
    PolicyK P = make_policy_k(*policy);
    hipStream_t s = S(stream);
#define ML_DISPATCH(T)                                                                              \
    switch (policy->hidden) {                                                                      \
        case 64: return launch_policy_step<T, 64>(P, obs, N, obs_store, actions, log_probs, values, \
                                                  k0, k1, step_ctr, step, env_offset, sample, s);            \
        case 128: return launch_policy_step<T, 128>(P, obs, N, obs_store, actions, log_probs,      \
                                                    values, k0, k1, step_ctr, step, env_offset, sample, s);  \
        default: return launch_policy_step<T, 256>(P, obs, N, obs_store, actions, log_probs,       \
                                                   values, k0, k1, step_ctr, step, env_offset, sample, s);   \
    }
    if (policy->dtype == MLEARN_DTYPE_BF16) {
        ML_DISPATCH(bf16)
    } else {
        ML_DISPATCH(float)
    }
#undef ML_DISPATCH
}
