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

}  // namespace ml
