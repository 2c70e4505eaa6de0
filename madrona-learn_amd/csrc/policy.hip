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
#include "mlp_tile.h"

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

// One workgroup = 32 rows x H/32 waves; wave w computes output column block w
// of every layer (NB = 1), so a 8192-env step runs 256 workgroups x 8 waves.
template <typename T, int H>
__global__ __launch_bounds__(2 * H) void policy_step_kernel(PolicyK P, const float* __restrict__ obs,
                                                            int64_t N, T* obs_store,
                                                            int32_t* actions, float* logp,
                                                            float* values, uint32_t k0,
                                                            uint32_t k1, const uint64_t* step_ctr,
                                                            uint64_t step_add, uint32_t eoff,
                                                            int sample) {
    constexpr int W = H / 32, CG = W, ROWS = 32, THREADS = 64 * W;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D;
    const int ld = (D > H ? D : H) + Pad<T>::v;
    T* act = (T*)smem;
    float* red = (float*)(act + ROWS * ld);  // [W][32][2]
    float* lgt = red + W * ROWS * 2;         // [32][33]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    const uint64_t step = (step_ctr ? *step_ctr : 0ull) + step_add;

    // 1. preprocess (cast) + store the observation tile, 16 B loads
    {
        const int cpr = D / 4;
        for (int idx = tid; idx < ROWS * cpr; idx += THREADS) {
            int rr = idx / cpr, c = (idx - rr * cpr) * 4;
            int64_t n = row0 + rr;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n < N) x = *(const float4*)(obs + n * D + c);
            store4(act + rr * ld + c, x.x, x.y, x.z, x.w);
            if (obs_store && n < N) store4(obs_store + n * D + c, x.x, x.y, x.z, x.w);
        }
    }
    lds_barrier();

    // 2. trunk
    for (int l = 0; l < P.L; ++l) {
        const int K = l == 0 ? D : H;
        f32x16 acc[1];
        zero_acc<1>(acc);
        gemm_direct<T, 1, CG>(acc, act, ld, 0, (const T*)P.wt[l], K, H, w, lane);
        ln_relu_epilogue<T, 1, 1, CG>(acc, P.lns[l], P.lnb[l], act, ld, red, w, lane, H, nullptr,
                                      nullptr);
        lds_barrier();
    }

    // 3. actor + critic heads
    heads_to_lds<T, 1, CG>(act, ld, (const T*)P.head_t, P.head_b, H, lgt, w, lane);
    lds_barrier();

    // 4. sample + store
    if (actions) {
        for (int task = tid; task < ROWS * P.K; task += THREADS) {
            int rr = task / P.K, g = task - rr * P.K;
            int64_t n = row0 + rr;
            if (n >= N) continue;
            int a;
            float lp;
            sample_group(&lgt[rr * 33 + P.off[g]], P.off[g + 1] - P.off[g], P.off[g], k0, k1,
                         eoff + (uint32_t)n, step, sample, &a, &lp);
            actions[n * P.K + g] = a;
            if (logp) logp[n * P.K + g] = lp;
        }
    }
    if (values) {
        for (int rr = tid; rr < ROWS; rr += THREADS) {
            int64_t n = row0 + rr;
            if (n < N) values[n] = lgt[rr * 33 + P.A];
        }
    }
}

size_t policy_step_lds(int D, int H, int esize) {
    int ld = (D > H ? D : H) + 16 / esize;
    return (size_t)32 * ld * esize + (size_t)(H / 32) * 32 * 2 * sizeof(float) +
           32 * 33 * sizeof(float);
}

template <typename T, int H>
static int launch_policy_step(const PolicyK& P, const float* obs, int64_t N, void* obs_store,
                              int32_t* actions, float* logp, float* values, uint32_t k0, uint32_t k1,
                              const uint64_t* step_ctr, uint64_t step, uint32_t eoff, int sample,
                              hipStream_t s) {
    size_t lds = policy_step_lds(P.D, H, sizeof(T));
    auto kern = policy_step_kernel<T, H>;
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  128 * 1024);
        attr_set = true;
    }
    int grid = (int)((N + 31) / 32);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(2 * H), lds, s, P, obs, N, (T*)obs_store, actions,
                       logp, values, k0, k1, step_ctr, step, eoff, sample);
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
