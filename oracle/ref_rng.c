/*
 * TEST INFRASTRUCTURE ONLY -- part of the parity oracle (see oracle/__init__.py).
 * Never linked into or called by the product path (madrona-learn_amd/).
 *
 * Plain-C restatement of the integer/byte-exact pieces the HIP kernels must
 * match bit for bit:
 *   - Philox4x32-10 (Salmon et al., SC'11; Random123 reference constants),
 *     pinned by the Random123 known-answer vectors in tests/test_oracle.py;
 *   - the deterministic Gumbel-max sampler that replaces
 *     jax.random.categorical in DiscreteActionDistributions.sample
 *     (src/madrona_learn/dists.py:26-44);
 *   - the synthetic dummy environment (bench/test sim plugin).
 * Built with -ffp-contract=off; every fused multiply-add is an explicit fmaf,
 * every other operation a single IEEE-754 rounding, so the results are the
 * GPU's bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { uint32_t v[4]; } ctr4;

static ctr4 philox(ctr4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)M0 * c.v[0];
        uint64_t p1 = (uint64_t)M1 * c.v[2];
        ctr4 n;
        n.v[0] = (uint32_t)(p1 >> 32) ^ c.v[1] ^ k0;
        n.v[1] = (uint32_t)p1;
        n.v[2] = (uint32_t)(p0 >> 32) ^ c.v[3] ^ k1;
        n.v[3] = (uint32_t)p0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

void oracle_philox(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        ctr4 c;
        memcpy(c.v, ctr + 4 * i, 16);
        ctr4 r = philox(c, k0, k1);
        memcpy(out + 4 * i, r.v, 16);
    }
}

static float unit(uint32_t x) { return (float)((x >> 8) | 1u) * 5.9604644775390625e-08f; }

float oracle_log2(float x) {
    uint32_t bits;
    memcpy(&bits, &x, 4);
    int e = (int)((bits >> 23) & 0xffu) - 127;
    uint32_t mb = (bits & 0x007fffffu) | 0x3f800000u;
    float m;
    memcpy(&m, &mb, 4);
    if (m > 1.41421353816986083984375f) {
        m = m * 0.5f;
        e += 1;
    }
    float f = m - 1.0f;
    /* minimax-fitted log2(1+f)/f on [sqrt(1/2)-1, sqrt(2)-1], Horner with fma */
    float p = -1.102015972e-01f;
    p = fmaf(p, f, 1.863120943e-01f);
    p = fmaf(p, f, -1.910249740e-01f);
    p = fmaf(p, f, 2.045752853e-01f);
    p = fmaf(p, f, -2.396190464e-01f);
    p = fmaf(p, f, 2.885688841e-01f);
    p = fmaf(p, f, -3.606966436e-01f);
    p = fmaf(p, f, 4.808982015e-01f);
    p = fmaf(p, f, -7.213473320e-01f);
    p = fmaf(p, f, 1.442695022e+00f);
    return fmaf(f, p, (float)e);
}

float oracle_gumbel(float u) {
    const float LN2 = 0.693147182464599609375f;
    float e1 = -(oracle_log2(u) * LN2);
    return -(oracle_log2(e1) * LN2);
}

static float sample_uniform(uint32_t k0, uint32_t k1, uint32_t env, uint64_t step, int j) {
    ctr4 c = {{env, (uint32_t)(j >> 2), (uint32_t)step, (uint32_t)(step >> 32)}};
    ctr4 r = philox(c, k0, k1);
    return unit(r.v[j & 3]);
}

/* Gumbel-max sample of every (row, group); logits [N][ld] f32, offsets [K+1].
 * Only the integer action is produced here (the log-prob uses expf/logf and
 * is compared with a tolerance). */
void oracle_sample(const float* logits, int64_t ld, const int32_t* offsets, int32_t K,
                   int64_t N, uint32_t k0, uint32_t k1, uint64_t step, uint32_t env_offset,
                   int32_t sample, int32_t* actions) {
    for (int64_t n = 0; n < N; ++n) {
        for (int g = 0; g < K; ++g) {
            const float* lg = logits + n * ld + offsets[g];
            int nb = offsets[g + 1] - offsets[g];
            int best = 0;
            float bv;
            if (sample) {
                bv = lg[0] + oracle_gumbel(sample_uniform(k0, k1, env_offset + (uint32_t)n, step,
                                                          offsets[g]));
                for (int j = 1; j < nb; ++j) {
                    float v = lg[j] + oracle_gumbel(sample_uniform(
                                          k0, k1, env_offset + (uint32_t)n, step, offsets[g] + j));
                    if (v > bv) {
                        bv = v;
                        best = j;
                    }
                }
            } else {
                bv = lg[0];
                for (int j = 1; j < nb; ++j)
                    if (lg[j] > bv) {
                        bv = lg[j];
                        best = j;
                    }
            }
            actions[n * K + g] = best;
        }
    }
}

/* Gumbel noise table for given (env, step, flattened logit index). */
void oracle_gumbel_table(uint32_t k0, uint32_t k1, uint64_t step, uint32_t env_offset, int64_t N,
                         int32_t A, float* out) {
    for (int64_t n = 0; n < N; ++n)
        for (int j = 0; j < A; ++j)
            out[n * A + j] = oracle_gumbel(sample_uniform(k0, k1, env_offset + (uint32_t)n, step, j));
}

/* ---- synthetic dummy env (misc.hip env_step_kernel restated) ---- */
static int episode_len(uint32_t g) { return 16 + (int)((g * 7u) % 33u); }

/* One Philox4x32-10 call per 4 features (counter {env, f / 4, step}):
 * feature f reads word f % 4 as four bytes b_i, s = sum (b_i + 0.5) / 256
 * (Irwin-Hall n = 4 of 8-bit uniforms, exact in f32), obs = (s - 2) sqrt(3)
 * (mean 0, variance 1). */
static float obs_feature(uint32_t k0, uint32_t k1, uint32_t g, int f, uint64_t step) {
    ctr4 c = {{g, (uint32_t)(f >> 2), (uint32_t)step, (uint32_t)(step >> 32)}};
    ctr4 r = philox(c, k0, k1 ^ 0x5eedu);
    uint32_t w = r.v[f & 3];
    uint32_t b = (w & 255u) + ((w >> 8) & 255u) + ((w >> 16) & 255u) + (w >> 24) + 2u;
    return ((float)b * 0.00390625f - 2.0f) * 1.73205077648162841796875f;
}

void oracle_env_reset(int32_t* state, int64_t N, int32_t D, uint32_t k0, uint32_t k1,
                      uint32_t eoff, float* obs) {
    for (int64_t n = 0; n < N; ++n) {
        uint32_t g = eoff + (uint32_t)n;
        for (int f = 0; f < D; ++f) obs[n * D + f] = obs_feature(k0, k1, g, f, ~0ull);
        state[4 * n + 0] = (int)(g % (uint32_t)episode_len(g));
        state[4 * n + 1] = 0;
        state[4 * n + 2] = 0;
        state[4 * n + 3] = 0;
    }
}

void oracle_env_step(int32_t* state, const int32_t* actions, int32_t K, int64_t N, int32_t D,
                     uint32_t k0, uint32_t k1, uint32_t eoff, float* obs, float* rew,
                     uint8_t* done) {
    for (int64_t n = 0; n < N; ++n) {
        uint32_t g = eoff + (uint32_t)n;
        uint64_t step = ((uint64_t)(uint32_t)state[4 * n + 2] << 32) | (uint32_t)state[4 * n + 1];
        for (int f = 0; f < D; ++f) obs[n * D + f] = obs_feature(k0, k1, g, f, step);
        int s = state[4 * n] + 1;
        int L = episode_len(g);
        int d = s >= L;
        ctr4 c = {{g, 0x80000000u, (uint32_t)step, (uint32_t)(step >> 32)}};
        ctr4 r = philox(c, k0, k1 ^ 0x5eedu);
        float u = unit(r.v[0]);
        float a0 = actions ? (float)actions[n * K] : 0.0f;
        rew[n] = (u * 2.0f - 1.0f) + 0.01f * a0;
        done[n] = (uint8_t)d;
        uint64_t ns = step + 1;
        state[4 * n + 0] = d ? 0 : s;
        state[4 * n + 1] = (int32_t)(uint32_t)ns;
        state[4 * n + 2] = (int32_t)(uint32_t)(ns >> 32);
        state[4 * n + 3] = 0;
    }
}
