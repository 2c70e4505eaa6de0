// Whole rollout of the built-in synthetic sim, row split
// (mlearn_policy_rollout_env, mlearn_rollout_out.policy_kernel = 2, the
// library's choice at the headline shape): rollout_loop rollouts.py:829-978
// -- per step the policy (ObservationsCaster -> MLP trunk -> heads,
// models.py:46-56, 99-154), Gumbel-max sampling (dists.py:26-52), the store
// writes (_post_inference_cb 637-680), the sim step and _post_step_cb
// (682-714, bookkeeping 933-973); then the bootstrap critic (607-635).
// Included by policy.hip inside namespace ml after RollK.
//
// Layout as the row-split minibatch step (r16_common.h): one workgroup of 8
// waves per CU keeps W1 and the head weights in LDS; a wave owns a tile of
// 16 envs (lane & 15 = env row) for all T + 1 steps, then its next tile.  The
// sim is per-env, so the next observations never leave the wave: each lane
// draws exactly the 16 features of its row that its layer-0 B fragment needs
// (4 Philox blocks), carried in registers to the next step; env.obs is
// written once, after the tile's last step.  The step's store writes are
// issued after the next step's first-layer weight loads (vmcnt counts loads
// and stores in issue order: a load behind stores waits for them).
// Same counters and arithmetic order as the feature-split rollout kernel for
// the sim, sampling, post-step and stores; the trunk and heads accumulate in
// another order (16x16x32 MFMAs), so logits can differ by a bf16 ulp and a
// sampled action can differ where two perturbed logits tie that closely.
#pragma once

// Action of one group by Gumbel-max over the bf16 logits of a row in LDS
// (o0: first logit, nb: group size) with the noise of flattened logit j from
// Philox {env, j / 4, step} (one block per quad, cached): the values
// sample_group / pick_group (dists.h) form, bit for bit.
__device__ inline void r16_pick(const bf16* lr, int o0, int nb, uint32_t ge, uint64_t step,
                                uint32_t k0, uint32_t k1, int& act, float& lp) {
#pragma clang fp contract(off)
    float mx = to_f32(lr[o0]);
    for (int j = 1; j < nb; ++j) mx = fmaxf(mx, to_f32(lr[o0 + j]));
    float se = 0.f;
    for (int j = 0; j < nb; ++j) se += __expf(to_f32(lr[o0 + j]) - mx);
    const float lse = mx + __logf(se);
    int best = 0, qc = -1;
    float bv = 0.f;
    u32x4 w{0u, 0u, 0u, 0u};
    for (int j = 0; j < nb; ++j) {
        const int jj = o0 + j;
        if ((jj >> 2) != qc) {
            qc = jj >> 2;
            w = philox4x32(u32x4{ge, (uint32_t)qc, (uint32_t)step, (uint32_t)(step >> 32)}, k0, k1);
        }
        const float v = to_f32(lr[jj]) + det_gumbel(u32_to_unit(u32x4_get(w, jj & 3)));
        if (j == 0 || v > bv) {
            bv = v;
            best = j;
        }
    }
    act = best;
    lp = to_f32(lr[o0 + best]) - lse;
}

// Waves per workgroup of the row-split rollout for N envs (one workgroup per
// CU): 8 from 65 536 envs in multiples of 256 (tiles in series beyond 2 048
// tiles) and at exactly 32 768 (one 16-env tile per wave: a two-rank
// data-parallel shard); 0 otherwise.  (4 and 2 waves at 16 384 / 8 192 envs,
// one wave per SIMD, measured no faster than the feature-split kernel: 363
// vs 361 us per rollout at 8 192, profiles/r05_rank_slices_ab.txt.)
static int rollout16_waves(int64_t N) {
    const int cus = device_cus();
    const int64_t kCUs = cus > 0 ? cus : 256;  // (256: MI355X, when no device answers)
    if (N % 256 == 0 && N >= 65536 && N / 16 <= 0x7fffffff) return 8;
    if (N == 16 * 8 * kCUs) return 8;
    return 0;
}

// The row-split rollout applies on the fused sim to the row-split step's
// policy shape (rows16_eligible), at most 8 action groups (two sampling tasks
// per lane), no observation normaliser, a whole-rollout launch (max_workgroups
// 0) and the env counts rollout16_waves takes.
static bool rollout16_shape(const PolicyK& P, bool bf, bool rnn) {
    // head: the scalar critic at width 32, or (round 6) a two-hot critic at
    // width 96 (R16Lay: the head image streamed from L2)
    const bool head = (P.HC == 32 && P.CB == 1) || (P.HC == 96 && P.CB > 1 && P.CB <= 64);
    return bf && !rnn && P.H == kR16H && P.L == 2 && head && P.D == kR16D && P.K <= 8 &&
           !P.obs_mu && !P.obs_stats;
}
static bool rollout16_eligible(const PolicyK& P, int64_t N, int max_wg, bool bf, bool rnn) {
    return rollout16_shape(P, bf, rnn) && max_wg == 0 && rollout16_waves(N) > 0;
}
// A population's rollouts on the row-split kernel (rollout16_pop_kernel,
// policy.hip): every policy of that shape (mlearn_policy_pop_prepare checks
// they agree), uncapped, N a multiple of 128 (so the 8 waves of a workgroup
// hold tiles of one policy in every round) and every wave of the chip with a
// tile (>= 2 048 16-env tiles in all).
static bool rollout16_pop_eligible(const PolicyK& P0, int64_t N, int npol, int max_wg, bool bf,
                                   bool rnn) {
    const int64_t tiles = (int64_t)npol * (N / 16);
    return rollout16_shape(P0, bf, rnn) && P0.HC == 32 && max_wg == 0 && N % 128 == 0 &&
           tiles >= 2048 && tiles <= 0x7fffffff;
}

// GAE (algo_common.py:84-130, gae_kernel's arithmetic and order, so the same
// bits) of the tile's 16 envs at the end of their rollout: lane (r, g) reads
// back steps 8g .. 8g + 7 of env n that this wave just stored, the four
// chunks run from the last to the first with the carry (next value, next
// advantage) handed between the row's lanes, and the advantages are written
// nontemporal as gae_kernel's (T <= 32).
__device__ __forceinline__ void r16_gae(const RollK& rk, int64_t n, float boot, int g, int lane) {
#pragma clang fp contract(off)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's store rows have landed)
    constexpr int CH = 8;
    const int T = rk.T, t0 = CH * g;
    float v[CH], rw[CH], a[CH];
    uint32_t d[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const int64_t q = (int64_t)(t0 + j < T ? t0 + j : 0) * rk.ld + n;
        v[j] = rk.values[q];
        rw[j] = rk.rewards[q];
        d[j] = rk.dones[q];
    }
    float nv = boot, na = 0.f;
#pragma unroll
    for (int c = 3; c >= 0; --c) {
        if (g == c) {
#pragma unroll
            for (int j = CH - 1; j >= 0; --j) {
                if (t0 + j >= T) continue;
                const float nvj = d[j] ? 0.f : nv;
                const float naj = d[j] ? 0.f : na;
                const float td = (rw[j] + rk.gae_gamma * nvj) - v[j];
                a[j] = td + rk.gae_gl * naj;
                nv = v[j];
                na = a[j];
            }
        }
        if (c > 0) {  // chunk c's carry to the row's lane of chunk c - 1
            nv = __shfl(nv, (lane & 15) + 16 * c);
            na = __shfl(na, (lane & 15) + 16 * c);
        }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j)
        if (t0 + j < T) __builtin_nontemporal_store(a[j], rk.adv + (int64_t)(t0 + j) * rk.ld + n);
}

// One 16-env tile's whole rollout on one wave: T policy steps with the sim
// step and post-step fused, then the bootstrap critic; the policy's W1 /
// head / LayerNorm images and action-group table already staged in smem.
template <int HC = kR16HC>
__device__ __forceinline__ void r16_roll_tile(const PolicyK& P, const float* __restrict__ obs0,
                                              const RollK& rk, uint32_t k0, uint32_t k1,
                                              uint64_t step0, uint32_t eoff, const EnvK& env,
                                              int tile, int tid, char* smem, int prio_t = -1) {
    typedef R16Lay<HC> LY;
    constexpr int LGS = LY::LGS;
    const char* w1img = smem + LY::OffW1;
    const char* whimg = smem + LY::OffWh;
    const float* gb = (const float*)(smem + LY::OffGb);
    const float* hb = (const float*)(smem + LY::OffHb);
    const float* bins = (const float*)(smem + LY::OffBins);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    bf16* lgs = (bf16*)(smem + LY::OffLg) + wave * 16 * LGS;
    const int* t_off = (const int*)(smem + LY::OffTab);
    const int K = P.K, A = P.A;
    constexpr int D = kR16D, DS = D / 32;
    // (the lane through an opaque copy per tile: rows16 kernel, ppo_rows16.h)
    const int lane = r16_late(tid & 63), r = lane & 15, g = lane >> 4;
    const int64_t n = (int64_t)tile * 16 + r;
    const uint32_t ge = eoff + (uint32_t)n;
    // this lane's 16 observation features (32s + 8g + j) and its env's state
    float xo[DS][8];
#pragma unroll
    for (int s = 0; s < DS; ++s) {
        const float4* src = (const float4*)(obs0 + n * D + 32 * s + 8 * g);
        const float4 a = src[0], b = src[1];
        xo[s][0] = a.x; xo[s][1] = a.y; xo[s][2] = a.z; xo[s][3] = a.w;
        xo[s][4] = b.x; xo[s][5] = b.y; xo[s][6] = b.z; xo[s][7] = b.w;
    }
    int4 st = env.state[n];
    float eret = rk.env_returns[n];
    // the previous step's store writes (issued behind this step's weight loads)
    bool pend = false;
    int pa[2] = {0, 0};
    float plp[2] = {0.f, 0.f}, pv = 0.f, prew = 0.f, per = 0.f;
    bool pdone = false;
    int64_t prow = 0;
    float boot = 0.f;  // the bootstrap critic of env n (the fused GAE's first carry)
    auto flush = [&]() {
        if (!pend) return;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int grp = (lane + 64 * u) >> 4;
            if (grp < K) {
                rk.actions[prow * K + grp] = pa[u];
                rk.logp[prow * K + grp] = plp[u];
            }
        }
        if (g == 0) {
            rk.values[prow] = pv;
            rk.rewards[prow] = prew;
            rk.dones[prow] = pdone ? 1 : 0;
            if (rk.trace) rk.trace[prow] = per;
        }
        pend = false;
    };
#pragma clang loop unroll(disable)
    for (int t = 0; t <= rk.T; ++t) {
        const bool act = t < rk.T;
        if (t == prio_t) __builtin_amdgcn_s_setprio(1);
        const uint64_t step = step0 + (uint64_t)t;
        const int64_t srow = (int64_t)t * rk.ld + n;  // store row of step t
        // ObservationsCaster: the compute-dtype cast is layer 0's B operand
        bf16x8 xf[DS];
#pragma unroll
        for (int s = 0; s < DS; ++s) {
            const u4r v = {pk_bf16(xo[s][0], xo[s][1]), pk_bf16(xo[s][2], xo[s][3]),
                           pk_bf16(xo[s][4], xo[s][5]), pk_bf16(xo[s][6], xo[s][7])};
            xf[s] = __builtin_bit_cast(bf16x8, v);
        }
        auto lda0 = [&](int ln) {
            const bf16* w0 = (const bf16*)P.wt[0];
            const int rr = ln & 15, gg = ln >> 4;
            return [=](int b, int s) {
                const int nn = 16 * b + rr;
                const int64_t idx = ((int64_t)(((nn >> 5) * (D >> 4) + 2 * s + (gg >> 1)) * 64 +
                                               (nn & 31) + 32 * (gg & 1))) * 8;
                return *(const bf16x8*)(w0 + idx);
            };
        };
        auto bf0 = [&](int s) { return xf[s]; };
        uint32_t zw[kR16NB][2], aw[kR16NB][2];
        float mean, rstd;
        r16_fwd_layer<DS, kR16Ring0>(lda0(r16_late(lane)), bf0, zw, mean, rstd);
        // the store rows of step t - 1 and this step's observations (behind
        // this step's weight loads)
        flush();
        if (act && rk.obs) {
            bf16* orow = (bf16*)rk.obs + r16_late(srow) * D;
#pragma unroll
            for (int s = 0; s < DS; ++s)
                r16_st16(orow + 32 * s + 8 * g, __builtin_bit_cast(u4r, xf[s]));
        }
        r16_ln_apply(zw, mean, rstd, gb, g, aw);
        r16_fwd_layer<kR16KS, kR16Ring>(
            [&](int b, int s) { return r16_row_frag(w1img, 16 * b + r, s, g); },
            [&](int s) { return r16_bfrag(aw, s); }, zw, mean, rstd);
        r16_ln_apply(zw, mean, rstd, gb + 2 * kR16H, g, aw);
        // heads (models.py:122-154): logits / value = rnd(rnd(A_1 Wh) + rnd(b))
        constexpr int NHB = HC / 16;
        f32x4 ha[NHB];
#pragma unroll
        for (int j = 0; j < NHB; ++j) ha[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (HC == 32) {
            r16_mm<NHB, kR16KS, 4>(ha,
                                   [&](int j, int s) { return r16_row_frag(whimg, 16 * j + r, s, g); },
                                   [&](int s) { return r16_bfrag(aw, s); });
        } else {  // the head image from L2 (R16Lay, r16_head_l2's addressing)
            const bf16* ht = (const bf16*)P.head_t;
            // column 16j + r, k-step s: a uniform part (j, s) plus one lane offset
            const uint32_t lo = r16_late((uint32_t)((r + 32 * (g & 1)) * 8 + 4 * (g >> 1)));
            r16_mm<NHB, kR16KS, kR16RingH>(
                ha,
                [&](int j, int s) {
                    const bf16* p = ht + ((j >> 1) * 8192 + s * 1024 + (j & 1) * 128);
                    const u2r a = *(const u2r*)(p + lo);
                    const u2r b = *(const u2r*)(p + 512 + lo);
                    return __builtin_bit_cast(bf16x8, u4r{a[0], a[1], b[0], b[1]});
                },
                [&](int s) { return r16_bfrag(aw, s); });
        }
        {
            bf16* lr = lgs + r * LGS;
#pragma unroll
            for (int cbk = 0; cbk < NHB; ++cbk) {
                const int c0 = 16 * cbk + 4 * g;
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    v[i] = rnd<bf16>(rnd<bf16>(ha[cbk][i]) + rnd<bf16>(hb[c0 + i]));
                *(u2r*)(lr + c0) = u2r{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])};
            }
        }
        wave_lds_sync();
        // the critic (rollouts.py:601-605): the scalar head column, or
        // SymExpTwoHotDistribution.mean() of the bin columns
        const float value = HC == 32 ? to_f32(lgs[r * LGS + A])
                                     : r16_twohot_mean(lgs + r * LGS + A, P.CB, bins, g);
        if (!act) {  // the bootstrap critic (rollouts.py:607-635)
            if (g == 0) rk.bootstrap[n] = value;
            boot = value;
            break;
        }
        // the sim's next observations: drawn from the state before the
        // advance (env.h), the quads of this lane's B fragment
        const uint64_t es = env_step_of(st);
#pragma unroll
        for (int s = 0; s < DS; ++s)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const u32x4 w = env_obs_words(env.k0, env.k1, ge, 8 * s + 2 * g + hh, es);
                xo[s][4 * hh + 0] = env_obs_word(w.x);
                xo[s][4 * hh + 1] = env_obs_word(w.y);
                xo[s][4 * hh + 2] = env_obs_word(w.z);
                xo[s][4 * hh + 3] = env_obs_word(w.w);
            }
        // sampling: task (row r, group (lane + 64u) >> 4)
        int a0 = 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int grp = (lane + 64 * u) >> 4;
            pa[u] = 0;
            plp[u] = 0.f;
            if (grp < K) {
                const int o0 = t_off[grp];
                r16_pick(lgs + r * LGS, o0, t_off[grp + 1] - o0, ge, step, k0, k1, pa[u],
                         plp[u]);
            }
            if (u == 0) a0 = pa[0];  // lanes 0..15: group 0 of row r
        }
        // the sim step and _post_step_cb of env n (lane g == 0 holds its
        // first action); every lane advances its copy of the env counter
        float rew;
        bool done;
        const int4 ns = env_advance_vals(ge, env.k0, env.k1, (float)a0, st, rew, done);
        float er;
        {
#pragma clang fp contract(off)
            er = rew + rk.gamma * eret;
        }
        eret = done ? 0.f : er;
        st = ns;
        pend = true;
        pv = value;
        prew = rew;
        pdone = done;
        per = er;
        prow = srow;
        wave_lds_sync();  // the logits scratch is rewritten by the next step
    }
    flush();
    if (rk.adv) r16_gae(rk, n, boot, g, lane);
    // the env's state after the rollout: observations, state, running return
    {
        float* orow = env.obs + n * D;
#pragma unroll
        for (int s = 0; s < DS; ++s) {
            float4* dst = (float4*)(orow + 32 * s + 8 * g);
            dst[0] = make_float4(xo[s][0], xo[s][1], xo[s][2], xo[s][3]);
            dst[1] = make_float4(xo[s][4], xo[s][5], xo[s][6], xo[s][7]);
        }
        if (g == 0) {
            env.state[n] = st;
            env.rew[n] = prew;
            env.done[n] = pdone ? 1 : 0;
            rk.env_returns[n] = eret;
        }
    }
}

#ifndef ML_ROLL_PRIO_NUM
#define ML_ROLL_PRIO_NUM 6  // eighths of T: the step the second wave takes priority
#endif

template <int NW, int HC>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu((NW + 3) / 4, (NW + 3) / 4))) void rollout16_kernel(
    PolicyK P, const float* __restrict__ obs0, int64_t N, RollK rk, uint32_t k0, uint32_t k1,
    const uint64_t* step_ctr, uint32_t eoff, EnvK env) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* tab = (int*)(smem + R16Lay<HC>::OffTab);
    static_assert(NW == kR16Waves, "r16_stage stages with kR16Waves waves");
    r16_stage<HC>(P, smem, tid);
    if (tid <= MLEARN_MAX_GROUPS) tab[tid] = P.off[tid];
    __syncthreads();
    const uint64_t step0 = step_ctr ? *step_ctr : 0ull;
    const int ntile = (int)(N / 16);
    const int TW = (int)gridDim.x * NW;
#pragma clang loop unroll(disable)
    for (int tile = (int)blockIdx.x * NW + wave; tile < ntile; tile += TW) {
        // the second wave of each SIMD (waves 4..7) loses issue arbitration
        // throughout; it takes priority for its last tile and from step
        // 6T/8 of the tile before it (rollout 1081-1086 -> 1027-1037 us at the
        // headline on one box; from the last tile's start only: 1058-1083
        // against 1075-1104; from step T/2: 1057-1066; from the start: slower)
        if (NW > 4 && wave >= NW / 2 && tile + TW >= ntile) __builtin_amdgcn_s_setprio(1);
        const int pt = (NW > 4 && wave >= NW / 2 && tile + 2 * TW >= ntile)
                           ? rk.T * ML_ROLL_PRIO_NUM / 8 : -1;
        r16_roll_tile<HC>(P, obs0, rk, k0, k1, step0, eoff, env, tile, tid, smem, pt);
    }
}

template <int NW, int HC>
static void launch_rollout16_nw(const PolicyK& P, const float* obs, int64_t N, const RollK& rk,
                                uint32_t k0, uint32_t k1, const uint64_t* step_ctr, uint32_t eoff,
                                const EnvK& env, int cus, hipStream_t s) {
    constexpr int lds = (int)R16Lay<HC>::Lds;
    const int64_t waves = N / 16;
    int64_t grid = cus > 0 ? cus : 256;
    if (grid * NW > waves) grid = waves / NW;
    hipLaunchKernelGGL((rollout16_kernel<NW, HC>), dim3((unsigned)grid), dim3(64 * NW), lds, s, P,
                       obs, N, rk, k0, k1, step_ctr, eoff, env);
}

static int launch_rollout16(const PolicyK& P, const float* obs, int64_t N, const RollK& rk,
                            uint32_t k0, uint32_t k1, const uint64_t* step_ctr, uint32_t eoff,
                            const EnvK& env, hipStream_t s) {
    // (the LDS attribute once per shape and device, kept out of graph capture)
    if (P.HC == 32) {
        if (set_lds_attr((const void*)rollout16_kernel<8, 32>, (int)R16Lay<32>::Lds, "rollout16"))
            return MLEARN_EHIP;
        launch_rollout16_nw<8, 32>(P, obs, N, rk, k0, k1, step_ctr, eoff, env, device_cus(), s);
    } else {
        if (set_lds_attr((const void*)rollout16_kernel<8, 96>, (int)R16Lay<96>::Lds, "rollout16"))
            return MLEARN_EHIP;
        launch_rollout16_nw<8, 96>(P, obs, N, rk, k0, k1, step_ctr, eoff, env, device_cus(), s);
    }
    return check_launch("policy_rollout_env (row split)");
}
