// Wide-tile fused minibatch step of the feed-forward (MLP) policy: the
// kFused mode of ppo_step_kernel with RB row blocks of 32 minibatch rows per
// workgroup instead of one.  Textually included by ppo.hip inside namespace
// ml (uses its RolloutK / HpK / WsK, store_row, the loss helpers).
//
// Workgroup = H / 32 waves, wave w owns feature block w (32 features) of
// every layer for ALL RB * 32 rows of the tile.  Per layer each k-step's
// weight fragment (the MFMA A operand, streamed from L2 through a ring of
// kWideRing k-steps in flight) feeds RB MFMAs, one per row block, with the
// B fragments (activations) read from the workgroup's LDS exchange buffer:
// the weight stream, the barriers and the LDS row statistics are paid once
// per RB * 32 rows instead of once per 32 (ppo_step_kernel: W_1 streamed
// from L2 twice per 32-row tile, 9 barriers per 32 rows).
//
//   gather   the tile's observation rows (store rows of the [T][N] rollout
//            store, rollouts.py:319-329) -> LDS B fragments + the X_0 spill
//   forward  per layer: Z = X W (MFMA), LayerNorm statistics across the
//            waves (LDS, one barrier), LN + ReLU, next layer's B fragments
//            into LDS (one barrier), A_l rows spilled for the weight gradient
//   heads    logits / critic from the last layer's fragments, K split over
//            the waves when the head has fewer output blocks than waves
//   loss     one (row, action group | value) task per thread (ppo.py:129-262)
//   backward d head -> dA_{L-1} (MFMA), per layer LayerNorm / ReLU backward
//            (row sums across the waves: one barrier), dZ_l spilled + into
//            LDS (one barrier), dA_{l-1} = W_l dZ_l (MFMA)
//
// Column partials (LayerNorm scale / bias, head bias) are summed over the
// tile's rows in registers before the 32-lane butterfly, one row of
// ws.colpart per workgroup (ws.ntiles = workgroups).  Same arithmetic per
// element as ppo_step_kernel; only the f32 summation trees of the column
// partials and of the head's K split differ.
#pragma once

#ifndef ML_WIDE_RING
#define ML_WIDE_RING 6  // k-steps of weight fragments in flight in the wide step kernel's products
#endif

template <typename T, int H, int HC, int RB> struct WideCfg {
    static constexpr int W = H / 32;  // waves = feature blocks
    static constexpr int THREADS = 64 * W;
    static constexpr int ROWS = 32 * RB;
    static constexpr int HB = HC / 32;            // head output blocks
    static constexpr int NTASK = RB * HB;         // head output tiles
    // head K split: every wave gets a tile when the tiles divide the waves
    static constexpr int KSPLIT = (W % NTASK == 0 && W / NTASK > 1) ? W / NTASK : 1;
    static constexpr int LGS = HC + 1;            // LDS row stride of the head outputs
};

// LDS of the wide step kernel: B fragments [FK][RB][64] (FK = k-steps of
// max(D, H)), row statistics [W][ROWS][2], head outputs [KSPLIT][ROWS][LGS],
// loss partials [W][kLossSlots], LayerNorm scale / bias [L][2][H], head bias
// [HC], critic bins [HC].
template <typename T, int H, int L, int HC, int RB> static size_t wide_lds(int D) {
    typedef WideCfg<T, H, HC, RB> C;
    const int FK = (D > H ? D : H) / RT<T>::KS;
    return (size_t)FK * RB * 64 * sizeof(typename RT<T>::frag) +
           (size_t)(C::W * C::ROWS * 2 + C::KSPLIT * C::ROWS * C::LGS + C::W * kLossSlots +
                    L * 2 * H + 2 * HC) * 4;
}

// acc[rb] += sum_s Img[step s] x fr[s][rb] over NKS k-steps (compile time);
// a ring of DEPTH k-steps of A fragments, the RB B fragments of the next
// k-step read from LDS one step ahead.  Issue half (the first DEPTH - 1
// steps' loads, so stores can go out behind them) and run half.
template <typename T, int RB, int DEPTH>
__device__ inline void wide_issue(typename RT<T>::frag (&ra)[DEPTH], const T* __restrict__ img, int lane,
                                  int nks) {
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
        if (s < nks) ra[s] = img_load<T>(rs, voff, s * FB);
}
template <typename T, int RB, int NKS, int DEPTH>
__device__ inline void wide_run(f32x16 (&acc)[RB], typename RT<T>::frag (&ra)[DEPTH],
                                const typename RT<T>::frag* fr, const T* __restrict__ img, int lane) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    frag b[RB], bn[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) b[rb] = fr[rb * 64 + lane];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const int sl = s + DEPTH - 1;
        if (sl < NKS) ra[sl % DEPTH] = img_load<T>(rs, voff, sl * FB);
        if (s + 1 < NKS) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) bn[rb] = fr[((s + 1) * RB + rb) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = MT<T>::mma(ra[s % DEPTH], b[rb], acc[rb]);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < NKS) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) b[rb] = bn[rb];
        }
    }
}

__device__ inline void zero1(f32x16& a) {
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = 0.f;
}

// acc += sum over NKS k-steps of Img[step s] x fr[s][rb] for ONE row block
// (B fragments at stride RB * 64 in the wide exchange buffer).
template <typename T, int RB, int NKS, int DEPTH>
__device__ inline void wide_gemm1(f32x16& acc, const typename RT<T>::frag* fr, int rb,
                                  const T* __restrict__ img, int lane) {
    typedef typename RT<T>::frag frag;
    constexpr int FB = 64 * RT<T>::E * (int)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * RT<T>::E * (int)sizeof(T);
    frag ra[DEPTH];
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
        if (s < NKS) ra[s] = img_load<T>(rs, voff, s * FB);
    frag b = fr[rb * 64 + lane];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const int sl = s + DEPTH - 1;
        if (sl < NKS) ra[sl % DEPTH] = img_load<T>(rs, voff, sl * FB);
        const frag bn = s + 1 < NKS ? fr[((s + 1) * RB + rb) * 64 + lane] : b;
        __builtin_amdgcn_sched_barrier(0);
        acc = MT<T>::mma(ra[s % DEPTH], b, acc);
        __builtin_amdgcn_sched_barrier(0);
        b = bn;
    }
}

// The first layer's product: K = D (runtime, <= NKMAX k-steps fully
// unrolled with guards; every A fragment was issued at kernel start).
template <typename T, int RB, int NKMAX>
__device__ inline void wide_first(f32x16 (&acc)[RB], const typename RT<T>::frag (&a0)[NKMAX],
                                  int nks, const typename RT<T>::frag* fr, int lane) {
#pragma unroll
    for (int s = 0; s < NKMAX; ++s)
        if (s < nks) {
            typename RT<T>::frag b[RB];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) b[rb] = fr[(s * RB + rb) * 64 + lane];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) acc[rb] = MT<T>::mma(a0[s], b[rb], acc[rb]);
        }
}

// Register budget: ~200-256 VGPRs at RB >= 2 (Dense outputs and
// accumulators of every row block held per wave), i.e. 2 waves per SIMD = one
// 8-wave workgroup per CU; RB = 1 runs on ppo_step_kernel instead (tuned for
// 128 VGPRs, two workgroups per CU).
constexpr int kWideWavesPerEU = 2;

template <typename T, int H, int L, int HC, int RB>
__global__ __launch_bounds__(64 * (H / 32)) __attribute__((amdgpu_waves_per_eu(kWideWavesPerEU, 8))) void ppo_wide_kernel(
    PolicyK P, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, int64_t M,
    const float* __restrict__ adv_st, HpK hp, WsK ws) {
    typedef typename RT<T>::frag frag;
    typedef WideCfg<T, H, HC, RB> C;
    constexpr int W = C::W, THREADS = C::THREADS, ROWS = C::ROWS, LGS = C::LGS, HB = C::HB;
    constexpr int KSPLIT = C::KSPLIT;
    constexpr int E = RT<T>::E, KS = RT<T>::KS, SPB = RT<T>::SPB;
    constexpr int KSH = H / KS, KSHD = HC / KS;
    constexpr int ES = (int)sizeof(T), VPC = 16 / ES;  // elements per 16-byte chunk
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int D = P.D, K = P.K;
    const int FK = (D > H ? D : H) / KS;
    frag* fr = (frag*)smem;                            // [FK][RB][64]
    float* red = (float*)(fr + (size_t)FK * RB * 64);  // [W][ROWS][2]
    float* lg = red + W * ROWS * 2;                    // [KSPLIT][ROWS][LGS]; part 0: logits
    float* lred = lg + KSPLIT * ROWS * LGS;            // [W][kLossSlots]
    float* gb = lred + W * kLossSlots;                 // [L][2][H]
    float* hbias = gb + L * 2 * H;                     // [HC]
    float* bins = hbias + HC;                          // [HC]
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int tid = (int)threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int tile = (int)blockIdx.x;
    const int64_t row0 = (int64_t)tile * ROWS;
    STAMP(0);

    // ---- loads issued up front: LayerNorm / head-bias parameters, the first
    // layer's weight fragments, the loss tasks' rollout columns, the tile's
    // observation rows ----
    constexpr int NPAR = (L * 2 * H + HC + THREADS - 1) / THREADS;
    float parv[NPAR];
#pragma unroll
    for (int k = 0; k < NPAR; ++k) {
        const int i = tid + k * THREADS;
        float v = 0.f;
        if (i < L * 2 * H) {
            const int l = i / (2 * H), c = i - l * 2 * H;
            v = c < H ? P.lns[l][c] : P.lnb[l][c - H];
        } else if (i < L * 2 * H + HC) {
            v = P.head_b[i - L * 2 * H];
        }
        parv[k] = v;
    }
    constexpr int NK0 = 64 / KS;  // first-layer k-steps held in registers (D <= 64)
    const int nk0 = D / KS;
    frag a0[NK0];
    {
        const __amdgpu_buffer_rsrc_t rs = img_rsrc((const T*)P.wt[0] + (int64_t)w * nk0 * 64 * E);
#pragma unroll
        for (int s = 0; s < NK0; ++s)
            if (s < nk0) a0[s] = img_load<T>(rs, lane * E * ES, s * 64 * E * ES);
    }
    // loss tasks (row rr, group g; g == K: value) of this thread's first two rounds
    constexpr int NPRE = 2;
    int t_act[NPRE];
    float t_lp[NPRE], t_adv[NPRE], t_ret[NPRE], t_val[NPRE];
#pragma unroll
    for (int u = 0; u < NPRE; ++u) {
        const int task = tid + u * THREADS, rr = task % ROWS, g = task / ROWS;
        t_act[u] = 0;
        t_lp[u] = t_adv[u] = t_ret[u] = t_val[u] = 0.f;
        if (g <= K && row0 + rr < M) {
            const int64_t q = store_row(ro, mb_seq, mb, row0 + rr);
            t_adv[u] = ro.adv[q];
            if (g < K) {
                t_act[u] = ro.actions[q * K + g];
                t_lp[u] = ro.logp[q * K + g];
            } else {
                t_ret[u] = ret_at(ro, q);
                if (ro.values) t_val[u] = ro.values[q];
            }
        }
    }
    typedef __attribute__((ext_vector_type(4))) uint32_t u4;
    const int cpr = D / VPC;  // 16-byte chunks per observation row
    {
        constexpr int NOB = 4;
        for (int c0 = 0; c0 < ROWS * cpr; c0 += NOB * THREADS) {
            u4 v[NOB];
#pragma unroll
            for (int u = 0; u < NOB; ++u) {
                const int c = c0 + tid + u * THREADS;
                const int rr = c / cpr, cc = c - rr * cpr;
                const u4 zero = {0u, 0u, 0u, 0u};
                v[u] = zero;
                if (c < ROWS * cpr && row0 + rr < M)
                    v[u] = *(const u4*)((const T*)ro.obs + store_row(ro, mb_seq, mb, row0 + rr) * D +
                                        cc * VPC);
            }
#pragma unroll
            for (int u = 0; u < NOB; ++u) {
                const int c = c0 + tid + u * THREADS;
                if (c >= ROWS * cpr) continue;
                const int rr = c / cpr, cc = c - rr * cpr, rb = rr >> 5, rl = rr & 31;
                // X_0 spill (weight-gradient operand), row-major; padding rows 0
                *(u4*)((T*)ws.x0 + (row0 + rr) * D + cc * VPC) = v[u];
                if constexpr (std::is_same<T, bf16>::value) {
                    // natural-order fragment (s, hh) of the row: k = 16 s + 8 hh .. + 7
                    fr[((cc >> 1) * RB + rb) * 64 + rl + 32 * (cc & 1)] = __builtin_bit_cast(bf16x8, v[u]);
                } else {
                    // (elements through an f32 vector: a per-element bit_cast of the
                    // u32 vector stored element 0 four times, ROCm 7.2 gfx950)
                    const f32x4 fv = __builtin_bit_cast(f32x4, v[u]);
                    const int k0 = cc * 4;
                    fr[((k0 >> 1) * RB + rb) * 64 + rl] = fv[0];
                    fr[((k0 >> 1) * RB + rb) * 64 + rl + 32] = fv[1];
                    fr[(((k0 >> 1) + 1) * RB + rb) * 64 + rl] = fv[2];
                    fr[(((k0 >> 1) + 1) * RB + rb) * 64 + rl + 32] = fv[3];
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NPAR; ++k)
        if (tid + k * THREADS < L * 2 * H + HC) gb[tid + k * THREADS] = parv[k];
    if (P.CB > 1)
        for (int i = tid; i < P.CB; i += THREADS) bins[i] = twohot_bin(i, P.CB);
    __syncthreads();
    STAMP(1);

    // ---- forward ----
    typedef typename Pk<T>::word word;
    word zr[L][RB][8];  // this wave's Dense outputs (exact in the compute dtype)
    float mean_r[L][RB], rstd_r[L][RB];
    const float invH = 1.0f / (float)H;
    f32x16 acc[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) zero1(acc[rb]);
    if (nk0 <= NK0) {
        wide_first<T, RB, NK0>(acc, a0, nk0, fr, lane);
    } else {  // wide observations: the k-steps streamed through the ring
        frag ra[ML_WIDE_RING];
        const T* img = (const T*)P.wt[0] + (int64_t)w * nk0 * 64 * E;
        const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
        for (int s = 0; s < nk0; ++s) {
            const frag a = img_load<T>(rs, lane * E * ES, s * 64 * E * ES);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) acc[rb] = MT<T>::mma(a, fr[(s * RB + rb) * 64 + lane], acc[rb]);
        }
        (void)ra;
    }
    STAMP(2);
    // post-activation rows A_l (weight-gradient operands), row-major
    word aw[RB][8];
    auto store_act = [&](int l) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            T* arow = (T*)ws.a[l] + (row0 + rb * 32 + r) * H + w * 32;
#pragma unroll
            for (int g = 0; g < 4; ++g) Pk<T>::store4(arow + 8 * g + 4 * h, aw[rb][2 * g], aw[rb][2 * g + 1]);
        }
    };
#pragma unroll
    for (int l = 0; l < L; ++l) {
        if (l > 0) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) zero1(acc[rb]);
            const T* img = (const T*)P.wt[l] + (int64_t)w * KSH * 64 * E;
            frag ra[ML_WIDE_RING];
            wide_issue<T, RB, ML_WIDE_RING>(ra, img, lane, KSH);
            store_act(l - 1);  // A_{l-1}, behind this product's first weight loads
            wide_run<T, RB, KSH, ML_WIDE_RING>(acc, ra, fr, img, lane);
            STAMP(5);
        }
        // Dense output -> compute dtype, per-row partial sums over this wave's features
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            f2 s2 = {0.f, 0.f}, q2 = {0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                zr[l][rb][k] = Pk<T>::pack(acc[rb][2 * k], acc[rb][2 * k + 1]);
                const f2 x = Pk<T>::unpack(zr[l][rb][k]);
                s2 += x;
                q2 = x * x + q2;
            }
            const float sum = sum_halves(s2.x + s2.y), sq = sum_halves(q2.x + q2.y);
            if (h == 0) *(float2*)(red + (w * ROWS + rb * 32 + r) * 2) = make_float2(sum, sq);
        }
        __syncthreads();
        STAMP(3 + 3 * l);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            float2 t = *(const float2*)(red + (rb * 32 + r) * 2);
#pragma unroll
            for (int v = 1; v < W; ++v) {
                const float2 u = *(const float2*)(red + (v * ROWS + rb * 32 + r) * 2);
                t.x += u.x;
                t.y += u.y;
            }
            const float mean = t.x * invH;
            const float var = fmaxf(t.y * invH - mean * mean, 0.f);
            const float rstd = rsqrtf(var + 1e-6f);
            mean_r[l][rb] = mean;
            rstd_r[l][rb] = rstd;
            // LayerNorm (x - mean) * (rstd * scale) + bias, ReLU (models.py:46-56, 110-115)
            const f2 m2 = {mean, mean}, r2 = {rstd, rstd};
            const float* gm = gb + l * 2 * H;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f0 = w * 32 + 8 * g + 4 * h;
                const float4 G = *(const float4*)(gm + f0), B = *(const float4*)(gm + H + f0);
                const f2 y0 = __builtin_elementwise_fma(Pk<T>::unpack(zr[l][rb][2 * g]) - m2,
                                                        r2 * f2{G.x, G.y}, f2{B.x, B.y});
                const f2 y1 = __builtin_elementwise_fma(Pk<T>::unpack(zr[l][rb][2 * g + 1]) - m2,
                                                        r2 * f2{G.z, G.w}, f2{B.z, B.w});
                aw[rb][2 * g] = Pk<T>::pack(fmaxf(y0.x, 0.f), fmaxf(y0.y, 0.f));
                aw[rb][2 * g + 1] = Pk<T>::pack(fmaxf(y1.x, 0.f), fmaxf(y1.y, 0.f));
            }
            // next product's B fragments (permuted k order of accumulator-fed fragments)
#pragma unroll
            for (int t = 0; t < SPB; ++t) fr[((w * SPB + t) * RB + rb) * 64 + lane] = Pk<T>::frag(aw[rb], t);
        }
        __syncthreads();
        STAMP(4 + 3 * l);
    }

    // ---- heads (dists.py:22, models.py:154): lg[row][j] = rnd(rnd(a . W) + rnd(b)) ----
    {
        constexpr int KPS = KSH / KSPLIT;
        const T* himg = (const T*)P.head_t;
        bool first = true;
        for (int u = w; u < C::NTASK * KSPLIT; u += W) {
            const int task = u / KSPLIT, part = u - task * KSPLIT;
            const int rb = task % RB, cb = task / RB;
            f32x16 ha[1];
            zero_acc<1>(ha);
            wide_gemm1<T, RB, KPS, (KPS < 8 ? KPS : 8)>(ha[0], fr + part * KPS * RB * 64, rb,
                                                        himg + ((int64_t)cb * KSH + part * KPS) * 64 * E,
                                                        lane);
            if (first) {
                store_act(L - 1);  // the last layer's rows, behind the head's weight loads
                first = false;
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) lg[(part * ROWS + rb * 32 + r) * LGS + feat(cb, q, h)] = ha[0][q];
        }
        if (first) store_act(L - 1);
    }
    STAMP(8);
    __syncthreads();
    for (int i = tid; i < ROWS * HC; i += THREADS) {
        const int rr = i / HC, j = i - rr * HC;
        float x = lg[rr * LGS + j];
#pragma unroll
        for (int v = 1; v < KSPLIT; ++v) x += lg[(v * ROWS + rr) * LGS + j];
        lg[rr * LGS + j] = rnd<T>(rnd<T>(x) + rnd<T>(hbias[j]));
    }
    __syncthreads();
    STAMP(9);

    // ---- loss: one (row, group | value) task per thread (ppo.py:129-262) ----
    {
        LossAcc m;
        bool did = false;  // this lane ran a task (waves without any skip the reductions)
        const float as0 = adv_st[0], as1 = adv_st[1];
        const float* vn = hp.norm_vals ? adv_st + 2 : nullptr;
        // two-hot critic: the value rows run in groups of 8 lanes (below); with
        // >= 512 threads the last 256 take them while the others do the groups
        const bool th = P.CB > 1;
        const bool split = th && THREADS >= 512;
        const int tstride = split ? THREADS - 256 : THREADS;
        const int ntask = ROWS * (th ? K : K + 1);
        int u = 0;
        for (int task = (split && tid >= THREADS - 256) ? ntask : tid; task < ntask;
             task += tstride, ++u) {
            const int rr = task % ROWS, g = task / ROWS;
            did = true;
            float* lr = lg + rr * LGS;
            const int64_t f = row0 + rr;
            if (f >= M) {  // padding row: zero its d logits
                if (g < K)
                    for (int j = P.off[g]; j < P.off[g + 1]; ++j) lr[j] = 0.f;
                else
                    for (int j = P.A; j < HC; ++j) lr[j] = 0.f;
                continue;
            }
            int act;
            float olp, adv, ret, oval;
            if (!split && u < NPRE) {  // preloaded (task == tid + u * THREADS)
                act = u == 0 ? t_act[0] : t_act[1];
                olp = u == 0 ? t_lp[0] : t_lp[1];
                adv = u == 0 ? t_adv[0] : t_adv[1];
                ret = u == 0 ? t_ret[0] : t_ret[1];
                oval = u == 0 ? t_val[0] : t_val[1];
            } else {
                const int64_t q = store_row(ro, mb_seq, mb, f);
                adv = ro.adv[q];
                act = g < K ? ro.actions[q * K + g] : 0;
                olp = g < K ? ro.logp[q * K + g] : 0.f;
                ret = g < K ? 0.f : ret_at(ro, q);
                oval = (g < K || !ro.values) ? 0.f : ro.values[q];
            }
            if (g < K) {
                if (hp.norm_adv) adv = (adv - as0) * as1;
                loss_group(hp, lr + P.off[g], P.off[g + 1] - P.off[g], act, olp, adv, hp.ecoef[g],
                           hp.objw[g], m);
            } else {
                loss_value(hp, lr, P.A, HC, ret, oval, m, vn);
            }
        }
        if (th) {
            constexpr int G = 8;
            const int vt0 = split ? tid - (THREADS - 256) : tid;
            const int vstride = split ? 256 : THREADS;
            for (int vt = vt0 < 0 ? ROWS * G : vt0; vt < ROWS * G; vt += vstride) {
                const int rr = vt / G, sub = vt % G;
                did = true;
                float* lr = lg + rr * LGS;
                const int64_t f = row0 + rr;
                if (f >= M) {  // padding row: zero its d critic logits
                    for (int j = P.A + sub; j < HC; j += G) lr[j] = 0.f;
                    continue;
                }
                const float R = ret_at(ro, store_row(ro, mb_seq, mb, f));
                loss_value_twohot_g<G>(hp, lr, P.A, P.CB, HC, bins, R, sub, m);
            }
        }
        const float vals[kLossSlots] = {m.sobj, m.qobj, m.mnobj, m.mxobj, m.svl, m.qvl, m.mnvl,
                                        m.mxvl, m.serr, m.qerr, m.mnerr, m.mxerr, m.sent, m.qent,
                                        m.mnent, m.mxent, m.sentw, m.sobjw, 0.f, 0.f};
        constexpr int kUsed = 18;  // slots 18.. are padding
        if (!hp.metrics) {
        } else if (__any(did)) {
#pragma unroll
            for (int s = 0; s < kUsed; ++s) {
                const int kind = (s < 16) ? (s & 3) : 0;
                float v = vals[s];
                v = kind == 2 ? wave_reduce<2>(v) : (kind == 3 ? wave_reduce<3>(v) : wave_reduce<0>(v));
                if (lane == 0) lred[w * kLossSlots + s] = v;
            }
            if (lane >= kUsed && lane < kLossSlots) lred[w * kLossSlots + lane] = 0.f;
        } else if (lane < kLossSlots) {  // identities of sum / min / max
            const int kind = (lane < 16) ? (lane & 3) : 0;
            lred[w * kLossSlots + lane] = kind == 2 ? 3.4e38f : (kind == 3 ? -3.4e38f : 0.f);
        }
    }
    __syncthreads();
    if (hp.metrics && tid < kLossSlots) {
        const int kind = (tid < 16) ? (tid & 3) : 0;
        double v = lred[tid];
        for (int u = 1; u < W; ++u) {
            const double x = lred[u * kLossSlots + tid];
            v = kind == 2 ? fmin(v, x) : (kind == 3 ? fmax(v, x) : v + x);
        }
        ws.loss_part[(int64_t)tile * kLossSlots + tid] = v;
    }
    STAMP(10);

    // ---- backward ----
    // dA_{L-1}^T = Head . dHead^T (this wave's feature block, every row block):
    // the head weight fragments go out before the d head stores
    constexpr int HPRE = KSHD <= 16 ? KSHD : 1;
    frag hbw[HPRE];
    const T* hbimg = (const T*)P.head + (int64_t)w * KSHD * 64 * E;
    const __amdgpu_buffer_rsrc_t hrs = img_rsrc(hbimg);
    if constexpr (KSHD <= 16) {
#pragma unroll
        for (int s2 = 0; s2 < KSHD; ++s2) hbw[s2] = img_load<T>(hrs, lane * E * ES, s2 * 64 * E * ES);
    }
    // d head rows (weight-gradient operand), row-major in the compute dtype
    for (int i = tid; i < ROWS * (HC / 4); i += THREADS) {
        const int rr = i / (HC / 4), c4 = (i - rr * (HC / 4)) * 4;
        const float* lr = lg + rr * LGS + c4;
        store4((T*)ws.dhead + (row0 + rr) * HC + c4, lr[0], lr[1], lr[2], lr[3]);
    }
    // head-bias column partials: wave cb sums column 32 cb + r over the tile's rows
    for (int cb = w; cb < HB; cb += W) {
        float cs = 0.f;
        for (int mm = 0; mm < ROWS / 2; ++mm) cs += rnd<T>(lg[(h * (ROWS / 2) + mm) * LGS + 32 * cb + r]);
        cs = sum_halves(cs);
        if (h == 0) ws.colpart[(int64_t)tile * ws.CP + L * 2 * H + 32 * cb + r] = cs;
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        zero1(acc[rb]);
        const float* lr = lg + (rb * 32 + r) * LGS;
#pragma unroll
        for (int s = 0; s < KSHD; ++s) {
            const frag hw = KSHD <= 16 ? hbw[s < HPRE ? s : 0]
                                       : img_load<T>(hrs, lane * E * ES, s * 64 * E * ES);
            acc[rb] = MT<T>::mma(hw, RT<T>::row_lds(lr, s, h), acc[rb]);
        }
    }

    STAMP(11);
    const int qs = col_sum16_index(lane);
    const float thr = relu_thr<T>();
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
        const float* gm = gb + l * 2 * H;
        float* cp = ws.colpart + (int64_t)tile * ws.CP + l * 2 * H;
        float pg[16], pb[16];  // LayerNorm scale / bias column partials over the tile's rows
#pragma unroll
        for (int q = 0; q < 16; ++q) pg[q] = pb[q] = 0.f;
        f2 u2[RB][8];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const bool live = row0 + rb * 32 + r < M;
            const float mean = mean_r[l][rb], rstd = rstd_r[l][rb];
            const f2 m2 = {mean, mean}, r2 = {rstd, rstd};
            f2 su2 = {0.f, 0.f}, sv2 = {0.f, 0.f};
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f0 = w * 32 + 8 * g + 4 * h;
                const float4 G = *(const float4*)(gm + f0), B = *(const float4*)(gm + H + f0);
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    const int k = 2 * g + p;
                    const f2 gg = p ? f2{G.z, G.w} : f2{G.x, G.y};
                    const f2 bb = p ? f2{B.z, B.w} : f2{B.x, B.y};
                    const f2 zc = Pk<T>::unpack(zr[l][rb][k]) - m2;
                    const f2 xh = zc * r2;
                    const f2 y = __builtin_elementwise_fma(zc, r2 * gg, bb);
                    // ReLU' (rnd<T>(y) > 0 <=> y > thr); padding rows carry no gradient
                    const f2 dy = {((y.x > thr) & live) ? acc[rb][2 * k] : 0.f,
                                   ((y.y > thr) & live) ? acc[rb][2 * k + 1] : 0.f};
                    const f2 u = dy * gg;
                    u2[rb][k] = u;
                    su2 += u;
                    sv2 = u * xh + sv2;
                    pg[2 * k] = __builtin_fmaf(dy.x, xh.x, pg[2 * k]);
                    pg[2 * k + 1] = __builtin_fmaf(dy.y, xh.y, pg[2 * k + 1]);
                    pb[2 * k] += dy.x;
                    pb[2 * k + 1] += dy.y;
                }
            }
            const float su = sum_halves(su2.x + su2.y), sv = sum_halves(sv2.x + sv2.y);
            if (h == 0) *(float2*)(red + (w * ROWS + rb * 32 + r) * 2) = make_float2(su, sv);
        }
        const float cpg = col_sum16(pg, lane), cpb = col_sum16(pb, lane);
        if (l == L - 1) STAMP(12);
        __syncthreads();
        if (l == L - 1) STAMP(13);
        word dzw[RB][8];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            float2 t = *(const float2*)(red + (rb * 32 + r) * 2);
#pragma unroll
            for (int v = 1; v < W; ++v) {
                const float2 u = *(const float2*)(red + (v * ROWS + rb * 32 + r) * 2);
                t.x += u.x;
                t.y += u.y;
            }
            const float mean = mean_r[l][rb], rstd = rstd_r[l][rb];
            // dZ = rstd (u - mean(u) - xh mean(u xh)) = rstd u + (-rstd^2 mean(u xh)) zc - rstd mean(u)
            const float ca = -(rstd * rstd) * (t.y * invH), cbb = -rstd * (t.x * invH);
            const f2 ca2 = {ca, ca}, cb2 = {cbb, cbb}, r2 = {rstd, rstd}, m2 = {mean, mean};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f2 zc = Pk<T>::unpack(zr[l][rb][k]) - m2;
                const f2 d = r2 * u2[rb][k] + (ca2 * zc + cb2);
                dzw[rb][k] = Pk<T>::pack(d.x, d.y);
            }
            if (l > 0) {
#pragma unroll
                for (int t2 = 0; t2 < SPB; ++t2)
                    fr[((w * SPB + t2) * RB + rb) * 64 + lane] = Pk<T>::frag(dzw[rb], t2);
            }
        }
        auto store_dz = [&]() {
            if ((lane & 16) == 0) {
                const int f = feat(w, qs, h);
                cp[f] = cpb;
                cp[H + f] = cpg;
            }
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                T* dzrow = (T*)ws.dz[l] + (row0 + rb * 32 + r) * H + w * 32;
#pragma unroll
                for (int g = 0; g < 4; ++g) Pk<T>::store4(dzrow + 8 * g + 4 * h, dzw[rb][2 * g], dzw[rb][2 * g + 1]);
            }
        };
        if (l > 0) {
            __syncthreads();
            // dA_{l-1}^T = W_l . dZ_l^T (this wave's feature block): weight loads
            // first, then this layer's column partials and dZ rows
            const T* img = (const T*)P.w[l] + (int64_t)w * KSH * 64 * E;
            frag ra[ML_WIDE_RING];
            wide_issue<T, RB, ML_WIDE_RING>(ra, img, lane, KSH);
            store_dz();
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) zero1(acc[rb]);
            wide_run<T, RB, KSH, ML_WIDE_RING>(acc, ra, fr, img, lane);
            if (l == L - 1) STAMP(14);
        } else {
            store_dz();
        }
    }
    STAMP(15);
}

// Row blocks per workgroup of the wide step kernel for M minibatch rows: the
// widest tile that still gives every CU a workgroup (bf16: 4 -> 128 rows;
// f32 keeps 2: its B fragments take twice the LDS); 1 = ppo_step_kernel.
template <typename T> static int wide_rb(int64_t M, int cus) {
    const int rbmax = sizeof(T) == 2 ? 4 : 2;
    for (int rb = rbmax; rb > 1; rb >>= 1)
        if (M / (32 * rb) >= cus) return rb;
    return 1;
}
