// Synthetic dummy vec-env (the bench / test sim plugin, madrona_learn/envs.py),
// shared by its own launch (misc.hip env_step_kernel) and the rollout policy
// kernel's fused env step (policy.hip, mlearn_policy_rollout_step_env).
// CPU twin: oracle/ref_rng.c.
#pragma once

#include "common.h"

namespace ml {

__host__ __device__ inline int env_episode_len(uint32_t g) { return 16 + (int)((g * 7u) % 33u); }

// One Philox4x32-10 call per 4 features (counter {env, f / 4, step}):
// feature f reads word f % 4 as four bytes b_i, s = sum (b_i + 0.5) / 256
// (Irwin-Hall n = 4 of 8-bit uniforms, exact in f32), obs = (s - 2) sqrt(3):
// mean 0, variance 1.  CPU twin: oracle/ref_rng.c obs_feature.
__device__ inline float env_obs_word(uint32_t w) {
#pragma clang fp contract(off)
    const uint32_t b = (w & 255u) + ((w >> 8) & 255u) + ((w >> 16) & 255u) + (w >> 24) + 2u;
    return ((float)b * 0.00390625f - 2.0f) * 1.73205077648162841796875f;
}
__device__ inline u32x4 env_obs_words(uint32_t k0, uint32_t k1, uint32_t g, int q, uint64_t step) {
    return philox4x32(u32x4{g, (uint32_t)q, (uint32_t)step, (uint32_t)(step >> 32)}, k0,
                      k1 ^ 0x5eedu);
}

// Env step counter of a state word {episode step, env step lo, env step hi, 0}.
__device__ inline uint64_t env_step_of(int4 st) {
    return ((uint64_t)(uint32_t)st.z << 32) | (uint32_t)st.y;
}

// Observation quad q (features 4q .. 4q+3) of env g at the given state.
__device__ inline void env_obs_quad(float* o, int D, uint32_t k0, uint32_t k1, uint32_t g, int q,
                                    uint64_t step, bool vec) {
    const u32x4 w = env_obs_words(k0, k1, g, q, step);
    if (vec) {
        *(float4*)o = make_float4(env_obs_word(w.x), env_obs_word(w.y), env_obs_word(w.z),
                                  env_obs_word(w.w));
    } else {
        for (int j = 0; j < 4 && 4 * q + j < D; ++j) o[j] = env_obs_word(u32x4_get(w, j));
    }
}

// One env's reward / done / state advance (its counter {env, 2^31, step});
// a0 = the env's first action.
// The values of that advance: reward, done, next state word.
__device__ inline int4 env_advance_vals(uint32_t g, uint32_t k0, uint32_t k1, float a0, int4 st,
                                        float& rew, bool& done) {
#pragma clang fp contract(off)
    const uint64_t step = env_step_of(st);
    int s = st.x + 1;
    int L = env_episode_len(g);
    bool d = s >= L;
    u32x4 r = philox4x32(u32x4{g, 0x80000000u, (uint32_t)step, (uint32_t)(step >> 32)}, k0,
                         k1 ^ 0x5eedu);
    float u = u32_to_unit(r.x);
    rew = (u * 2.0f - 1.0f) + 0.01f * a0;
    done = d;
    const uint64_t ns = step + 1;
    return make_int4(d ? 0 : s, (int)(uint32_t)ns, (int)(uint32_t)(ns >> 32), 0);
}
__device__ inline void env_advance_a0(int4* state, int64_t n, uint32_t g, uint32_t k0, uint32_t k1,
                                      float a0, float* rew, uint8_t* done, int4 st) {
    float r;
    bool d;
    const int4 ns = env_advance_vals(g, k0, k1, a0, st, r, d);
    rew[n] = r;
    done[n] = d ? 1 : 0;
    state[n] = ns;
}

__device__ inline void env_advance(int4* state, const int32_t* actions, int K, int64_t n,
                                   uint32_t g, uint32_t k0, uint32_t k1, float* rew,
                                   uint8_t* done, int4 st) {
    const float a0 = actions ? (float)actions[n * K] : 0.f;
    env_advance_a0(state, n, g, k0, k1, a0, rew, done, st);
}

// Fused env step of the rollout policy kernel (mlearn_dummy_env, include/mlearn.h).
struct EnvK {
    int4* state;     // [N] (null: no fused env step)
    float* obs;      // [N][D] next observations (the policy launch's own obs input)
    float* rew;      // [N]
    uint8_t* done;   // [N]
    uint32_t k0, k1, eoff;
};

}  // namespace ml
