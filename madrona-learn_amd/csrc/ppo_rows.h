// Row-split fused PPO minibatch step (ppo.py:109-286 up to the weight
// gradients) for the headline policy shape: bf16 compute, MLP[256, 256]
// (two trunk layers), actor logits + scalar critic in a head of width 32.
//
// Every wave owns one 32-row tile and ALL 256 features of it, so the tile
// runs from the observation gather to the last LayerNorm backward with no
// workgroup barrier: LayerNorm row statistics are lane-local sums (+ one
// v_permlane32_swap), the heads and the loss stay inside the wave, and the
// post-activation / dZ accumulators are the next product's B fragments
// directly (no LDS exchange).  The workgroup shares one copy of W_1 in LDS
// (128 KB, compute dtype), staged once; it serves BOTH products of the
// layer (see the image layout below), so the per-tile weight traffic that
// bounds ppo_step_kernel (W_1 streamed from L2 twice per 32-row tile) is
// gone.  W_0 and the two head images (16-32 KB) stream from L2.
//
// Arithmetic = ppo_step_kernel<bf16, 256, 2, kFused, 32> with its 8 feature
// waves: the same MFMA k-step order per 32-feature block, LayerNorm sums per
// block combined in block order (= that kernel's wave order), head partials
// of k-step pairs summed in block order, the same loss code.  The two
// kernels write identical gradients (tests/test_gpu_rows.py).
//
// Spill for the weight-gradient launch: X_0, Z_0 (the first Dense output,
// in place of A_0: the wave reloads it for its own LayerNorm-0 backward and
// wgrad_kernel recomputes A_0 = relu(LN_0(Z_0)) from it and the per-row
// statistics), A_1, dZ_0, dZ_1, d head, plus the LayerNorm / head-bias
// column partials and the loss-metric partials of ppo_step_kernel.
#pragma once
// (included inside namespace ml by ppo.hip, after the loss helpers)

// ---------------------------------------------------------------------------
// W_1 image in LDS.  Element (i, j) of W_1 [in i][out j]: 8-byte unit u = j/4
// of row i is stored at unit pi(u) ^ Z(i) of a 512-byte row, pi swapping
// bits 0 and 1 of u, Z(i) = ((i & 3) << 3) | (((i >> 2) & 3) << 1).
//   backward A fragment (n = i, k = j, permuted k order): the lane's 8
//     elements are units 4s + h and 4s + 2 + h -> pi-adjacent -> ONE
//     ds_read_b128 at unit (4s + 2h) ^ Z(i); conflict-free (the 16 rows of
//     every b128 lane group have distinct Z / 2).
//   forward A fragment (n = j, k = i): two ds_read_b64_tr_b16 (rows
//     16s + 8hi + 4h + q, columns 32nb + 16jh + 4p ..); conflict-free (the
//     4 rows of a half-wave land in distinct 8-unit groups).
// The staging copy is the backward image mlearn_mlp_policy.w[1] 16 bytes
// at a time: fragment (nb, s) lane (r, h) -> row 32nb + r, unit (4s + 2h) ^ Z.
// ---------------------------------------------------------------------------
__device__ inline int w1z(int i) { return ((i & 3) << 3) | (((i >> 2) & 3) << 1); }
__device__ inline int w1pi(int u) { return (u & ~3) | ((u & 1) << 1) | ((u >> 1) & 1); }

#ifndef ML_ROWS_WPE
#define ML_ROWS_WPE 1  // waves per SIMD the row-split kernel is register-budgeted for (1 or 2)
#endif
constexpr int kRowsH = 256;
constexpr int kRowsCUs = 256;  // MI355X compute units: one row-split workgroup each
constexpr int kRowsLgs = 40;  // bf16 row stride of a wave's logits tile (80 B: 16-B aligned, conflict-free)
constexpr size_t kRowsW1 = (size_t)kRowsH * kRowsH * 2;
constexpr size_t kRowsPar = (size_t)(2 * 2 * kRowsH + 32) * 4;  // LayerNorm scale | bias x 2, head bias
constexpr size_t kRowsLgw = (size_t)32 * kRowsLgs * 2;
constexpr size_t rows_lds(int wpb) { return kRowsW1 + kRowsPar + (size_t)wpb * kRowsLgw; }

typedef short short4v_r __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v_r* lds_s4p;
typedef __attribute__((ext_vector_type(4))) uint32_t u4r;
typedef __attribute__((address_space(3))) u4r* lds_u4p;

// Per-lane base offsets of the fragment reads (everything else is an
// immediate offset):
//   forward  (block nb, step s, half hi): f[hi][nb & 3] + 8192 s + 256 (nb >> 2)
//     with f[hi][m] = 512 (16 s0 + 8 hi + 4 h + q) + 8 (pi(u) ^ Z) at s = 0,
//     u = 8 m + 4 jh + p (lane = 16 (2 h + jh) + 4 q + p);
//   backward (block nb, step s): b[s & 7] + 16384 nb + 256 (s >> 3).
// Offsets past the 16-bit immediate use a second set of bases (+65536).
struct W1Addr {
    uint32_t f[2][4];
    uint32_t b[8];
};
__device__ inline W1Addr w1_addrs(int lane) {
    W1Addr A;
    const int G = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3, hh = G >> 1, jh = G & 1;
#pragma unroll
    for (int hi = 0; hi < 2; ++hi)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int i = 8 * hi + 4 * hh + q, u = 8 * m + 4 * jh + p;
            A.f[hi][m] = (uint32_t)(512 * i + 8 * (w1pi(u) ^ w1z(i)));
        }
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < 8; ++s) A.b[s] = (uint32_t)(512 * i + 8 * ((4 * s + 2 * h) ^ w1z(i)));
    return A;
}
// Forward A fragment: W_1^T block nb (output features j), k-step s (inputs i)
__device__ inline bf16x8 w1_fwd_frag(const char* w1s, const W1Addr& A, int nb, int s) {
    const uint32_t off = 8192u * s + 256u * (nb >> 2);
    const short4v_r lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(w1s + A.f[0][nb & 3] + off));
    const short4v_r hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(w1s + A.f[1][nb & 3] + off));
    typedef short short8v_r __attribute__((ext_vector_type(8)));
    const short8v_r v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}
// Backward A fragment: W_1 block nb (input features i), k-step s (outputs j)
__device__ inline bf16x8 w1_bwd_frag(const char* w1s, const W1Addr& A, int nb, int s) {
    const uint32_t off = 16384u * nb + 256u * (s >> 3);
    return __builtin_bit_cast(bf16x8, *(const lds_u4p)(w1s + A.b[s & 7] + off));
}

// Hide the packed words from common-subexpression elimination: the two
// passes over them (statistics then apply, or the two LayerNorm-backward
// passes) recompute the 2-VALU unpack instead of keeping 128 unpacked floats
// live across the phase.
__device__ inline void rows_opaque(uint32_t (&w)[8][8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(w[i][k]));
}

// Pin values at this point of the instruction stream (the empty asm has side
// effects, so it stays in order with the scheduling fences and the values must
// be computed before it): keeps the per-block phases from being regrouped
// into one phase that holds every block's temporaries at once.
__device__ inline void rows_pin(uint32_t (&w)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(w[k]));
}
__device__ inline void rows_pin(f32x16& a) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(a[k]));
}

// An LDS parameter pointer whose loads the compiler cannot merge with the
// same loads of an earlier phase (it would keep 128 scale / bias values live
// across the whole tile instead of re-reading them from LDS).
__device__ inline const float* rows_fresh(const float* p) {
    int off = 0;
    asm volatile("" : "+s"(off));
    return p + off;
}

// One 32-feature block's LayerNorm row partials of ppo_step_kernel's
// ln_pack_stats<T, 1> + sum_halves (block-order combination by the caller).
__device__ inline void rows_block_stats(const uint32_t (&zw)[8], float& sum, float& sq) {
    f2 s = {0.f, 0.f}, qq = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const f2 x = Pk<bf16>::unpack(zw[k]);
        s += x;
        qq = x * x + qq;
    }
    sum = sum_halves(s.x + s.y);
    sq = sum_halves(qq.x + qq.y);
}

// acc (Dense output, f32) -> packed compute-dtype words, row mean / rstd over
// the 256 features (statistics as ppo_step_kernel: per-block sums in block order)
__device__ inline void rows_ln_stats(const f32x16 (&acc)[8], uint32_t (&zw)[8][8], float& mean,
                                     float& rstd) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) zw[i][k] = Pk<bf16>::pack(acc[i][2 * k], acc[i][2 * k + 1]);
    float sum = 0.f, sq = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float a, b;
        rows_block_stats(zw[i], a, b);
        sum = i == 0 ? a : sum + a;
        sq = i == 0 ? b : sq + b;
    }
    const float invH = 1.0f / (float)kRowsH;
    mean = sum * invH;
    const float var = fmaxf(sq * invH - mean * mean, 0.f);
    rstd = rsqrtf(var + 1e-6f);
    rows_opaque(zw);
}

// LayerNorm + ReLU of every block (ln_apply per block), gm = LDS [2][H]
__device__ inline void rows_ln_apply(const uint32_t (&zw)[8][8], float mean, float rstd,
                                     const float* gm, int h, uint32_t (&aw)[8][8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        f2 x2[1][8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x2[0][k] = Pk<bf16>::unpack(zw[i][k]);
        uint32_t a1[1][8];
        ln_apply<bf16, 1>(x2, mean, rstd, rows_fresh(gm), kRowsH, i, h, a1);
#pragma unroll
        for (int k = 0; k < 8; ++k) aw[i][k] = a1[0][k];
        if (ML_ROWS_WPE > 1) {  // 256 registers: one block's temporaries at a time
            rows_pin(aw[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// Row-major [Mp][256] bf16 spill / reload of this lane's row (features of
// block i, group g: 32 i + 8 g + 4 h .. + 3)
__device__ inline void rows_store(bf16* rowp, int h, const uint32_t (&w)[8][8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) Pk<bf16>::store4(rowp + 32 * i + 8 * g + 4 * h, w[i][2 * g], w[i][2 * g + 1]);
}
__device__ inline void rows_load(const bf16* rowp, int h, uint32_t (&w)[8][8]) {
    typedef __attribute__((ext_vector_type(2))) uint32_t u2;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const u2 v = *(const u2*)(rowp + 32 * i + 8 * g + 4 * h);
            w[i][2 * g] = v.x;
            w[i][2 * g + 1] = v.y;
        }
}

// LayerNorm + ReLU backward of one layer (ppo_step_kernel's trunk backward):
// acc = d loss / d A in, packed dZ out; LayerNorm scale / bias column
// partials of the tile stored to cp.  Two passes so that only the
// accumulators and the packed Dense outputs stay live: pass 1 turns acc
// into u = dy * scale in place and sums su, sv per block; pass 2 recomputes
// the centred input from zw.
__device__ inline void rows_ln_bwd(f32x16 (&acc)[8], uint32_t (&zw)[8][8], float mean,
                                   float rstd, const float* gm, bool live, int lane,
                                   float* cp, uint32_t (&dzw)[8][8]) {
    const int h = lane >> 5;
    rows_opaque(zw);  // no reuse of the forward pass's unpacked values
    const float thr = relu_thr<bf16>();
    const f2 m2 = {mean, mean}, r2 = {rstd, rstd};
    const int qs = col_sum16_index(lane);
    float su = 0.f, sv = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        f2 su2 = {0.f, 0.f}, sv2 = {0.f, 0.f};
        float pg[16], pb[16];
        const float* gmi = rows_fresh(gm);  // this block's parameters loaded here, not hoisted
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f0 = i * 32 + 8 * g + 4 * h;
            const float4 G = *(const float4*)(gmi + f0), B = *(const float4*)(gmi + kRowsH + f0);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int k = 2 * g + p;
                const f2 gg = p ? f2{G.z, G.w} : f2{G.x, G.y};
                const f2 bb = p ? f2{B.z, B.w} : f2{B.x, B.y};
                const f2 zc = Pk<bf16>::unpack(zw[i][k]) - m2;
                const f2 xh = zc * r2;
                const f2 y = __builtin_elementwise_fma(zc, r2 * gg, bb);
                const f2 dy = {((y.x > thr) & live) ? acc[i][2 * k] : 0.f,
                               ((y.y > thr) & live) ? acc[i][2 * k + 1] : 0.f};
                const f2 u = dy * gg;
                const f2 pgk = dy * xh;
                acc[i][2 * k] = u.x;
                acc[i][2 * k + 1] = u.y;
                su2 += u;
                sv2 = u * xh + sv2;
                pg[2 * k] = pgk.x;
                pg[2 * k + 1] = pgk.y;
                pb[2 * k] = dy.x;
                pb[2 * k + 1] = dy.y;
            }
        }
        const float cg = col_sum16(pg, lane);
        const float cb = col_sum16(pb, lane);
        if ((lane & 16) == 0) {
            const int f = feat(i, qs, h);
            cp[f] = cb;
            cp[kRowsH + f] = cg;
        }
        const float a = sum_halves(su2.x + su2.y), b = sum_halves(sv2.x + sv2.y);
        su = i == 0 ? a : su + a;
        sv = i == 0 ? b : sv + b;
        if (ML_ROWS_WPE > 1) {
            rows_pin(acc[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    rows_opaque(zw);
    const float invH = 1.0f / (float)kRowsH;
    const float ca = -(rstd * rstd) * (sv * invH), cb = -rstd * (su * invH);
    const f2 ca2 = {ca, ca}, cb2 = {cb, cb};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const f2 zc = Pk<bf16>::unpack(zw[i][k]) - m2;
            const f2 u = {acc[i][2 * k], acc[i][2 * k + 1]};
            const f2 d = r2 * u + (ca2 * zc + cb2);
            dzw[i][k] = Pk<bf16>::pack(d.x, d.y);
        }
        if (ML_ROWS_WPE > 1) {
            rows_pin(dzw[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

#ifndef ML_ROWS_RING
#define ML_ROWS_RING 4  // A fragments in flight in the LDS products
#endif

// acc[nb] += sum_s W1img(nb, s) x B(s), B(s) = fragment s & 1 of block s >> 1
// of bw (permuted k order); FWD: W_1^T (transposed reads), else W_1.
template <bool FWD>
__device__ inline void rows_w1_product(f32x16 (&acc)[8], const uint32_t (&bw)[8][8],
                                       const char* w1s, const W1Addr& A) {
    constexpr int N = 8 * 16, R = ML_ROWS_RING;
    bf16x8 ring[R];
#pragma unroll
    for (int x = 0; x < R; ++x)
        ring[x] = FWD ? w1_fwd_frag(w1s, A, x >> 4, x & 15) : w1_bwd_frag(w1s, A, x >> 4, x & 15);
#pragma unroll
    for (int x = 0; x < N; ++x) {
        const int nb = x >> 4, s = x & 15;
        const bf16x8 a = ring[x % R];
        if (x + R < N) {
            const int y = x + R;
            ring[x % R] = FWD ? w1_fwd_frag(w1s, A, y >> 4, y & 15)
                              : w1_bwd_frag(w1s, A, y >> 4, y & 15);
        }
        // fences keep the scheduler from hoisting the whole unrolled read
        // stream (128 fragments) above the MFMAs
        __builtin_amdgcn_sched_barrier(0);
        acc[nb] = MT<bf16>::mma(a, Pk<bf16>::frag(bw[s >> 1], s & 1), acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// All 16 fragments (byte offset 1024 x frag_of(x)) of a head image.
template <typename FO>
__device__ inline void rows_img_load16(const void* img, int lane, bf16x8 (&f)[16], FO frag_of) {
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
#pragma unroll
    for (int x = 0; x < 16; ++x) f[x] = img_load<bf16>(rs, lane * 16, frag_of(x) * 1024);
}

// acc[0] (+)= sum over NF image fragments (byte offset 1024 x frag(x)) x B(x),
// a ring of R fragments in flight from L2.
template <int NF, int R, typename FA, typename FB, typename OP>
__device__ inline void rows_l2_ring(const void* img, int lane, FA frag_of, FB b_of, OP op) {
    const __amdgpu_buffer_rsrc_t rs = img_rsrc(img);
    const int voff = lane * 16;
    bf16x8 ring[R];
#pragma unroll
    for (int x = 0; x < R; ++x) ring[x] = img_load<bf16>(rs, voff, frag_of(x) * 1024);
#pragma unroll
    for (int x = 0; x < NF; ++x) {
        const bf16x8 a = ring[x % R];
        if (x + R < NF) ring[x % R] = img_load<bf16>(rs, voff, frag_of(x + R) * 1024);
        __builtin_amdgcn_sched_barrier(0);
        op(x, a, b_of(x));
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Diagnostic builds (ML_STAMPS, tools/stamp_rows.py): per-tile phase stamps.
#ifdef ML_STAMPS
#define RSTAMP(i)                                                                  \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        if (ws.stamps && lane == 0)                                                \
            ws.stamps[(int64_t)tile * 16 + (i)] = __builtin_amdgcn_s_memtime();    \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
#else
#define RSTAMP(i) \
    do {          \
    } while (0)
#endif

// One wave per SIMD (512 registers): Z_0 stays in registers for the
// LayerNorm-0 backward and A_0 is spilled for the weight-gradient launch as
// by ppo_step_kernel.  Two waves per SIMD (256 registers): Z_0 is spilled
// instead, reloaded for the backward, and wgrad_kernel rebuilds A_0 from it.
constexpr bool kRowsKeepZ0 = ML_ROWS_WPE == 1;

template <int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(ML_ROWS_WPE, ML_ROWS_WPE))) void ppo_rows_kernel(
    PolicyK P, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, int64_t M,
    const float* __restrict__ adv_st, HpK hp, WsK ws) {
    typedef bf16 T;
    constexpr int H = kRowsH, HC = 32, THREADS = 64 * WPB;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* w1s = smem;
    float* gb = (float*)(smem + kRowsW1);  // [2][2][H] LayerNorm scale | bias
    float* hbias = gb + 4 * H;             // [32]
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    bf16* lg = (bf16*)(smem + kRowsW1 + kRowsPar + (size_t)w * kRowsLgw);  // [32][kRowsLgs]

    // ---- stage W_1 (16-byte pieces of the backward image), LayerNorm / head-bias parameters ----
    {
        const u4r* src = (const u4r*)P.w[1];
        constexpr int PIECES = H * H * 2 / 16, PER = PIECES / THREADS;
        u4r v[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) v[k] = src[tid + k * THREADS];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int pc = tid + k * THREADS, f = pc >> 6, L = pc & 63;
            const int i = 32 * (f >> 4) + (L & 31), s = f & 15, hh = L >> 5;
            *(lds_u4p)(w1s + 512 * i + 8 * ((4 * s + 2 * hh) ^ w1z(i))) = v[k];
        }
        for (int i = tid; i < 4 * H + HC; i += THREADS) {
            float x;
            if (i < 4 * H) {
                const int l = i / (2 * H), c = i - l * 2 * H;
                x = c < H ? P.lns[l][c] : P.lnb[l][c - H];
            } else {
                x = P.head_b[i - 4 * H];
            }
            gb[i] = x;
        }
    }

    const W1Addr wa = w1_addrs(lane);
    __syncthreads();  // W_1 and the LayerNorm parameters staged (the only workgroup barrier)

    // tiles of 32 rows, one per wave at a time (persistent over the grid)
    for (int tile = (int)blockIdx.x * WPB + w; tile < ws.ntiles; tile += (int)gridDim.x * WPB) {
        const int64_t row0 = (int64_t)tile * 32, row = row0 + r;
        const bool live = row < M;
        const int64_t sr = live ? store_row(ro, mb_seq, mb, row) : 0;
        const int K = P.K, D = P.D;
        // loss tasks (row, group | value) of this lane: task = lane + 64 k; the
        // rollout columns of the first PT are in flight from the tile's start
        const int ntask = 32 * (K + 1);
        constexpr int PT = 4;  // tasks whose rollout columns are prefetched
        int t_act[PT];
        float t_lp[PT], t_adv[PT], t_ret[PT], t_val[PT];
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const int task = lane + 64 * k, rr = task & 31, g = task >> 5;
            t_act[k] = 0;
            t_lp[k] = t_adv[k] = t_ret[k] = t_val[k] = 0.f;
            if (task < ntask && row0 + rr < M) {
                const int64_t q = store_row(ro, mb_seq, mb, row0 + rr);
                t_adv[k] = ro.adv[q];
                if (g < K) {
                    t_act[k] = ro.actions[q * K + g];
                    t_lp[k] = ro.logp[q * K + g];
                } else {
                    t_ret[k] = ret_at(ro, q);
                    if (ro.values) t_val[k] = ro.values[q];
                }
            }
        }

        RSTAMP(0);
        // ---- layer 0: observation gather (X_0 spill), Dense ----
        f32x16 acc[8];
        zero_acc<8>(acc);
        gemm_first<T, 8>(acc, (const T*)ro.obs + sr * D, live, D / 16, (const T*)P.wt[0],
                         (T*)ws.x0 + row * D, lane);
        RSTAMP(1);
        uint32_t zw[8][8], aw[8][8];
        float mean0, rstd0;
        rows_ln_stats(acc, zw, mean0, rstd0);
        rows_ln_apply(zw, mean0, rstd0, gb, h, aw);
        RSTAMP(2);
        uint32_t z0[8][8];  // (unused when Z_0 is spilled)
        if constexpr (kRowsKeepZ0) {
            // Z_0 kept for the LayerNorm-0 backward; A_0 spilled for the weight gradients
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int k = 0; k < 8; ++k) z0[i][k] = zw[i][k];
            rows_store((T*)ws.a[0] + row * H, h, aw);
        } else {
            // Z_0 and its row statistics for the backward and the weight-gradient launch
            rows_store((T*)ws.a[0] + row * H, h, zw);
            if (h == 0) *(float2*)(ws.lnst + 2 * row) = make_float2(mean0, rstd0);
        }

        RSTAMP(3);
        // ---- layer 1 ----
        zero_acc<8>(acc);
        rows_w1_product<true>(acc, aw, w1s, wa);
        // head image fragments in flight under the LayerNorm
        bf16x8 hfr[16];
        rows_img_load16(P.head_t, lane, hfr, [](int x) { return x; });
        RSTAMP(4);
        float mean1, rstd1;
        rows_ln_stats(acc, zw, mean1, rstd1);  // zw: Z_1 from here on
        rows_ln_apply(zw, mean1, rstd1, gb + 2 * H, h, aw);  // aw: A_1
        rows_store((T*)ws.a[1] + row * H, h, aw);

        RSTAMP(5);
        // ---- heads: partial products of k-step pairs summed in block order ----
        {
            f32x16 tot, p;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                if ((x & 1) == 0) {
#pragma unroll
                    for (int q = 0; q < 16; ++q) p[q] = 0.f;
                }
                p = MT<T>::mma(hfr[x], Pk<T>::frag(aw[x >> 1], x & 1), p);
                if (x == 1) {
                    tot = p;
                } else if (x & 1) {
#pragma unroll
                    for (int q = 0; q < 16; ++q) tot[q] += p[q];
                }
            }
            // lg[row][j] = rnd(rnd(x) + rnd(b)) (dists.py:22, models.py:154)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                bf16x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = 8 * g + 4 * h + e;
                    v[e] = (T)(rnd<T>(rnd<T>(tot[4 * g + e]) + rnd<T>(hbias[j])));
                }
                *(bf16x4*)(lg + r * kRowsLgs + 8 * g + 4 * h) = v;
            }
        }
        RSTAMP(6);
        wave_lds_sync();

        // backward head image fragments in flight under the loss
        rows_img_load16(P.head, lane, hfr, [](int x) { return 2 * (x & 7) + (x >> 3); });
        // ---- loss: one (row, group | value) task per lane and step (ppo.py:129-262) ----
        {
            LossAcc m;
            const float as0 = adv_st[0], as1 = adv_st[1];
            const float* vn = hp.norm_vals ? adv_st + 2 : nullptr;
            for (int k = 0, task = lane; task < ntask; ++k, task += 64) {
                const int rr = task & 31, g = task >> 5;
                bf16* lr = lg + rr * kRowsLgs;
                const int64_t f = row0 + rr;
                if (f >= M) {  // padding row: zero its d logits
                    if (g < K)
                        for (int j = P.off[g]; j < P.off[g + 1]; ++j) lr[j] = (T)0.f;
                    else
                        for (int j = P.A; j < HC; ++j) lr[j] = (T)0.f;
                    continue;
                }
                int act;
                float olp, adv, ret, oval;
                if (k < PT) {
                    act = k == 0 ? t_act[0] : (k == 1 ? t_act[1] : (k == 2 ? t_act[2] : t_act[3]));
                    olp = k == 0 ? t_lp[0] : (k == 1 ? t_lp[1] : (k == 2 ? t_lp[2] : t_lp[3]));
                    adv = k == 0 ? t_adv[0] : (k == 1 ? t_adv[1] : (k == 2 ? t_adv[2] : t_adv[3]));
                    ret = k == 0 ? t_ret[0] : (k == 1 ? t_ret[1] : (k == 2 ? t_ret[2] : t_ret[3]));
                    oval = k == 0 ? t_val[0] : (k == 1 ? t_val[1] : (k == 2 ? t_val[2] : t_val[3]));
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
            if (hp.metrics) {
                const float vals[kLossSlots] = {m.sobj, m.qobj, m.mnobj, m.mxobj, m.svl, m.qvl, m.mnvl,
                                                m.mxvl, m.serr, m.qerr, m.mnerr, m.mxerr, m.sent, m.qent,
                                                m.mnent, m.mxent, m.sentw, m.sobjw, 0.f, 0.f};
                double* lp = ws.loss_part + (int64_t)tile * kLossSlots;
#pragma unroll
                for (int s = 0; s < kLossSlots; ++s) {
                    const int kind = (s < 16) ? (s & 3) : 0;
                    float v = vals[s];
                    v = kind == 2 ? wave_reduce<2>(v) : (kind == 3 ? wave_reduce<3>(v) : wave_reduce<0>(v));
                    if (lane == 0) lp[s] = (double)v;
                }
            }
        }
        wave_lds_sync();

        RSTAMP(7);
        // ---- d head: row-major spill, head-bias column partials, backward through the head ----
        {
            const u4r* lr = (const u4r*)(lg + r * kRowsLgs + 16 * h);
            u4r* drow = (u4r*)((T*)ws.dhead + row * HC + 16 * h);
            drow[0] = lr[0];
            drow[1] = lr[1];
            float cs = 0.f;
#pragma unroll
            for (int mm = 0; mm < 16; ++mm) cs += (float)lg[(16 * h + mm) * kRowsLgs + r];
            cs = sum_halves(cs);
            if (h == 0) ws.colpart[(int64_t)tile * ws.CP + 4 * H + r] = cs;
        }
        {
            // dA_1^T = Head . dHead^T: image fragment (nb, s) at 2 nb + s, taken s-major
            bf16x8 db[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) db[s] = *(const bf16x8*)(lg + r * kRowsLgs + 16 * s + 8 * h);
            zero_acc<8>(acc);
#pragma unroll
            for (int x = 0; x < 16; ++x) acc[x & 7] = MT<T>::mma(hfr[x], db[x >> 3], acc[x & 7]);
        }

        RSTAMP(8);
        // ---- layer 1 backward ----
        float* cp = ws.colpart + (int64_t)tile * ws.CP;
        rows_ln_bwd(acc, zw, mean1, rstd1, gb + 2 * H, live, lane, cp + 2 * H, aw);  // aw: dZ_1
        rows_store((T*)ws.dz[1] + row * H, h, aw);
        RSTAMP(9);
        zero_acc<8>(acc);
        rows_w1_product<false>(acc, aw, w1s, wa);
        RSTAMP(10);
        // ---- layer 0 backward ----
        if constexpr (kRowsKeepZ0) {
            rows_ln_bwd(acc, z0, mean0, rstd0, gb, live, lane, cp, aw);  // aw: dZ_0
        } else {
            rows_load((const T*)ws.a[0] + row * H, h, zw);  // the reloaded Z_0
            rows_ln_bwd(acc, zw, mean0, rstd0, gb, live, lane, cp, aw);
        }
        RSTAMP(11);
        rows_store((T*)ws.dz[0] + row * H, h, aw);
        RSTAMP(12);
    }
}

// Opt-in (MLEARN_ROWS=1): measured at the headline minibatch (rocprofv3,
// gpurun_out rows3 / rq1) 111-121 us against ppo_step_kernel's 97 us.  One
// wave per SIMD (the 512-register budget the 32-row tile needs) leaves the
// LayerNorm phases latency-bound: per-tile stamps (tools/stamp_rows.py)
// 117 K cycles, 22 K of them in the layer-1 LayerNorm backward alone.
// Shape check: bf16, H = 256, two trunk layers, head width 32, scalar
// critic, observation width a multiple of 16 up to 256.
static bool rows_ok(const mlearn_mlp_policy& p) {
    const char* e = getenv("MLEARN_ROWS");
    if (!e || e[0] != '1') return false;
    return p.dtype == MLEARN_DTYPE_BF16 && p.hidden == kRowsH && p.num_layers == 2 &&
           head_cols(p) == 32 && p.critic_bins == 1 && p.obs_dim % 16 == 0 && p.obs_dim <= 256;
}

template <int WPB>
static void launch_rows_wpb(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                            int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                            hipStream_t s) {
    auto k = ppo_rows_kernel<WPB>;
    static bool attr_set = false;  // once per instantiation (kept out of graph capture)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)rows_lds(WPB));
        attr_set = true;
    }
    // one workgroup per CU (LDS); waves loop over the tiles
    const int grid = std::min((ws.ntiles + WPB - 1) / WPB, kRowsCUs);
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * WPB), rows_lds(WPB), s, P, R, mb_seq, mb, M,
                       adv_st, hp, ws);
}

// Waves per workgroup: 4 * ML_ROWS_WPE (every SIMD busy) when the tiles fill
// every CU's waves, fewer (more workgroups) for small minibatches.
static void launch_rows(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                        int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                        hipStream_t s) {
    const int nt = ws.ntiles;
    constexpr int WMAX = 4 * ML_ROWS_WPE;
    if (nt >= WMAX * kRowsCUs)
        launch_rows_wpb<WMAX>(P, R, mb_seq, mb, M, adv_st, hp, ws, s);
    else if (WMAX > 4 && nt >= 4 * kRowsCUs)
        launch_rows_wpb<(WMAX > 4 ? 4 : WMAX)>(P, R, mb_seq, mb, M, adv_st, hp, ws, s);
    else if (nt >= 2 * kRowsCUs)
        launch_rows_wpb<2>(P, R, mb_seq, mb, M, adv_st, hp, ws, s);
    else
        launch_rows_wpb<1>(P, R, mb_seq, mb, M, adv_st, hp, ws, s);
}
