// Discrete action distribution math shared by the standalone sampler
// (misc.hip) and the fused rollout kernel (policy.hip).
// DiscreteActionDistributions.sample / best (dists.py:26-52).
#pragma once
#include "common.h"

namespace ml {

// lg: the nb logits of one group (f32, already in the reference's
// post-cast precision).  Gumbel-max with Philox noise for flattened logit
// index jbase + j; first-index argmax on ties (jnp.argmax); log-prob =
// logit[a] - logsumexp (dists.py:36-38).
__device__ inline void sample_group(const float* lg, int nb, int jbase, uint32_t k0, uint32_t k1,
                                    uint32_t env, uint64_t step, int sample, int* action,
                                    float* logp) {
#pragma clang fp contract(off)
    float mx = lg[0];
    for (int j = 1; j < nb; ++j) mx = fmaxf(mx, lg[j]);
    float se = 0.f;
    for (int j = 0; j < nb; ++j) se += __expf(lg[j] - mx);
    float lse = mx + __logf(se);
    int best = 0;
    if (sample) {
        float bv = lg[0] + det_gumbel(sample_uniform(k0, k1, env, step, jbase));
        for (int j = 1; j < nb; ++j) {
            float v = lg[j] + det_gumbel(sample_uniform(k0, k1, env, step, jbase + j));
            if (v > bv) {
                bv = v;
                best = j;
            }
        }
    } else {
        float bv = lg[0];
        for (int j = 1; j < nb; ++j)
            if (lg[j] > bv) {
                bv = lg[j];
                best = j;
            }
    }
    *action = best;
    if (logp) *logp = lg[best] - lse;
}

// DiscreteActionDistributions.action_stats (dists.py:54-77) of one group:
// log_softmax = logits - logsumexp, log-prob of the given action a, entropy
// -sum softmax * log_softmax.
__device__ inline void eval_group(const float* lg, int nb, int a, float* logp, float* ent) {
#pragma clang fp contract(off)
    float mx = lg[0];
    for (int j = 1; j < nb; ++j) mx = fmaxf(mx, lg[j]);
    float se = 0.f;
    for (int j = 0; j < nb; ++j) se += __expf(lg[j] - mx);
    const float lse = mx + __logf(se), inv = 1.0f / se;
    float e = 0.f;
    for (int j = 0; j < nb; ++j) e -= (__expf(lg[j] - mx) * inv) * (lg[j] - lse);
    a = a < 0 ? 0 : (a >= nb ? nb - 1 : a);
    *logp = lg[a] - lse;
    *ent = e;
}

// sample_group with the Gumbel-perturbed logits already computed (nz, the
// same values sample_group forms: lg[j] + det_gumbel(sample_uniform(j))), or
// best() when nz is null.  Bit-identical to sample_group.
__device__ inline void pick_group(const float* lg, const float* nz, int nb, int* action,
                                  float* logp) {
#pragma clang fp contract(off)
    float mx = lg[0];
    for (int j = 1; j < nb; ++j) mx = fmaxf(mx, lg[j]);
    float se = 0.f;
    for (int j = 0; j < nb; ++j) se += __expf(lg[j] - mx);
    const float lse = mx + __logf(se);
    const float* v = nz ? nz : lg;
    int best = 0;
    float bv = v[0];
    for (int j = 1; j < nb; ++j)
        if (v[j] > bv) {
            bv = v[j];
            best = j;
        }
    *action = best;
    if (logp) *logp = lg[best] - lse;
}

// ---------------------------------------------------------------------------
// SymExpTwoHotDistribution (dists.py:119-208) over the nb critic logits of a
// DreamerV3Critic (models.py:157-174), logits already cast to f32.
// ---------------------------------------------------------------------------
// Bin j (dists.py:128-141): half = symexp(linspace(-14, 0, nb/2 + 1)) in f32,
// jnp.linspace's interpolation form start * (1 - i/div) (+ stop * i/div, stop
// = 0); bins = [half, -half[:-1][::-1]]; symexp(x) = sign(x) expm1(|x|)
// (utils.py:39-40).
__device__ inline float twohot_bin(int j, int nb) {
    const int nh = nb / 2;
    const int i = j <= nh ? j : nb - 1 - j;
    if (i == nh) return 0.f;
    const float x = -14.0f * (1.0f - (float)i / (float)nh);
    const float v = -expm1f(-x);  // symexp(x), x < 0
    return j <= nh ? v : -v;
}

// ---------------------------------------------------------------------------
// SymExpTwoHotDistribution statistics computed by an aligned group of G
// lanes of one wave (lane `sub` of the group handles bins sub, sub + G, ...);
// partial results are combined with butterfly shuffles inside the group.
//   twohot_mean_g: mean() (dists.py:143-169): p_mid b_mid plus the mirrored
//     pairs p_{mid-1-i} b_{mid-1-i} + p_{mid+1+i} b_{mid+1+i} (the symmetric
//     sum that makes it exactly 0 at initialisation);
//   twohot_ce_g: two_hot_cross_entropy_loss (dists.py:171-208); the bin
//     weights are the reference's as written: lower = |b_lo - t| / (|b_lo - t|
//     + |b_up - t|), upper = |b_up - t| / (...), 1/2 each when the clipped
//     indices coincide.
// ---------------------------------------------------------------------------
template <int G> __device__ inline float group_max(float v) {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
template <int G> __device__ inline float group_sum(float v) {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

template <int G>
__device__ inline float twohot_mean_g(const float* lg, int nb, const float* bins, int sub,
                                      float* mx_out, float* se_out) {
    float mx = -3.4e38f;
    for (int j = sub; j < nb; j += G) mx = fmaxf(mx, lg[j]);
    mx = group_max<G>(mx);
    float se = 0.f;
    for (int j = sub; j < nb; j += G) se += __expf(lg[j] - mx);
    se = group_sum<G>(se);
    const int mid = (nb - 1) / 2;
    float acc = 0.f;
    for (int i = sub; i < mid; i += G) {
        const int a = mid - 1 - i, b = mid + 1 + i;
        acc += (__expf(lg[a] - mx) / se) * bins[a] + (__expf(lg[b] - mx) / se) * bins[b];
    }
    acc = group_sum<G>(acc);
    *mx_out = mx;
    *se_out = se;
    return (__expf(lg[mid] - mx) / se) * bins[mid] + acc;
}

// Every lane returns the loss and mean(); each lane writes the scaled
// d loss / d logit of its own bins.
template <int G>
__device__ inline float twohot_ce_g(float* lg, int nb, float target, const float* bins, float scale,
                                    int sub, float* mean_out) {
    float cle = 0.f, cgt = 0.f;
    for (int j = sub; j < nb; j += G) {
        cle += bins[j] <= target ? 1.f : 0.f;
        cgt += bins[j] > target ? 1.f : 0.f;
    }
    cle = group_sum<G>(cle);
    cgt = group_sum<G>(cgt);
    const int lo = min(max((int)cle - 1, 0), nb - 1);
    const int up = min(max(nb - (int)cgt, 0), nb - 1);
    const bool same = lo == up;
    const float dl = same ? 1.f : fabsf(bins[lo] - target);
    const float du = same ? 1.f : fabsf(bins[up] - target);
    const float tot = dl + du;
    const float wl = dl / tot, wu = du / tot;
    float mx, se;
    *mean_out = twohot_mean_g<G>(lg, nb, bins, sub, &mx, &se);
    const float lse = mx + __logf(se);
    const float llo = lg[lo], lup = lg[up];  // read before any lane of the group writes
    const float loss = -(wl * (llo - lse) + wu * (lup - lse));
    const float wsum = wl + wu;
    for (int j = sub; j < nb; j += G) {
        const float p = __expf(lg[j] - mx) / se;
        const float w = (j == lo ? wl : 0.f) + (j == up ? wu : 0.f);
        lg[j] = (wsum * p - w) * scale;
    }
    return loss;
}

}  // namespace ml
