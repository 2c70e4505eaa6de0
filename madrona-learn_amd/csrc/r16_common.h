// Shared pieces of the row-split kernels (the minibatch step, ppo_rows16.h,
// and the whole rollout, rollout_rows16.h) for the headline policy shape:
// bf16, H = 256, two trunk layers, scalar critic, head width 32, obs_dim 64.
// One workgroup of 8 waves per CU keeps W1 and the head weights in LDS; a
// wave owns 16-row tiles on v_mfma_f32_16x16x32_bf16 with features on M and
// the tile's rows on N (lane & 15): lane l holds features 16b + 4(l>>4) + i
// (i < 4) of accumulator block b.  k-step s of a product over hidden
// features takes blocks 2s, 2s+1, so its k-slot 8g + j is feature
// 32s + 16(j>>2) + 4g + (j&3) (g = lane >> 4) -- the A operand is read in
// that order.
#pragma once

#include "common.h"
#include "dists.h"
#include "rowtile.h"

namespace ml {

constexpr int kR16Waves = 8;     // waves per workgroup
constexpr int kR16Tiles = 2;     // 16-row tiles per wave: 32 rows = one partials row
constexpr int kR16H = 256;
constexpr int kR16NB = kR16H / 16;   // 16-feature accumulator blocks
constexpr int kR16KS = kR16H / 32;   // k-steps over the hidden features
constexpr int kR16HC = MLEARN_HEAD_COLS;
constexpr int kR16D = 64;            // observation width (the first layer's K)
constexpr int kR16LGS = 40;          // logits scratch row stride (bf16; 80-B rows)
#ifndef ML_R16_RING
#define ML_R16_RING 6
#endif
#ifndef ML_R16_RING0
#define ML_R16_RING0 16
#endif
constexpr int kR16Ring = ML_R16_RING;    // LDS A fragments in flight per product
constexpr int kR16Ring0 = ML_R16_RING0;  // first-layer (L2) A fragments in flight
#ifndef ML_R16_RINGH
#define ML_R16_RINGH 8
#endif
constexpr int kR16RingH = ML_R16_RINGH;  // head (L2, HC = 96) A fragments in flight
// LDS: W1 image [256 rows = out][512 B], head image [32 rows = col][512 B],
// LayerNorm scale/bias [2][2][256] f32, head bias [32] f32, per-wave logits
// scratch [8][16][kR16LGS] bf16, the action groups' logit offsets, entropy
// coefficients and objective weights (read per lane by the loss tasks: from
// the kernel arguments a lane-dependent index would copy the arrays into
// registers)
constexpr size_t kR16OffW1 = 0;
constexpr size_t kR16OffWh = kR16OffW1 + (size_t)kR16H * 512;
constexpr size_t kR16OffGb = kR16OffWh + (size_t)kR16HC * 512;
constexpr size_t kR16OffHb = kR16OffGb + (size_t)2 * 2 * kR16H * 4;
constexpr size_t kR16OffLg = kR16OffHb + (size_t)kR16HC * 4;
constexpr size_t kR16OffTab = kR16OffLg + (size_t)kR16Waves * 16 * kR16LGS * 2;
constexpr int kR16TabN = 3 * (MLEARN_MAX_GROUPS + 1);  // group offsets, entropy coefs, obj weights
constexpr size_t kR16Lds = kR16OffTab + (size_t)kR16TabN * 4;
static_assert(kR16Lds <= 160 * 1024, "row-split step LDS budget");

// The same layout for head width HC (the kR16Off* constants above are HC =
// 32).  At HC = 96 (a DreamerV3 two-hot critic: A logits + up to 63 bins,
// round 6) the 48 KB head image no longer fits beside W1 and a 16-row
// logits scratch of 96 columns, so the head products stream the head image
// from L2 (r16_head_l2) and LDS holds the critic's bin values instead.
template <int HC> struct R16Lay {
    static_assert(HC == 32 || HC == 96, "head width");
    static constexpr int LGS = HC == 32 ? kR16LGS : 104;  // logits scratch row stride (bf16)
    static constexpr size_t OffW1 = 0;
    static constexpr size_t OffWh = OffW1 + (size_t)kR16H * 512;
    static constexpr size_t OffGb = OffWh + (HC == 32 ? (size_t)HC * 512 : 0);
    static constexpr size_t OffHb = OffGb + (size_t)2 * 2 * kR16H * 4;
    static constexpr size_t OffBins = OffHb + (size_t)HC * 4;
    static constexpr size_t OffLg = OffBins + (HC == 32 ? 0 : (size_t)64 * 4);
    static constexpr size_t OffTab = OffLg + (size_t)kR16Waves * 16 * LGS * 2;
    static constexpr size_t Lds = OffTab + (size_t)kR16TabN * 4;
    static_assert(Lds <= 160 * 1024, "row-split LDS budget");
};
static_assert(R16Lay<32>::Lds == kR16Lds && R16Lay<32>::OffLg == kR16OffLg, "layouts agree");

typedef float f2v __attribute__((ext_vector_type(2)));
typedef short short4r __attribute__((ext_vector_type(4)));
typedef __attribute__((ext_vector_type(4))) uint32_t u4r;
typedef __attribute__((ext_vector_type(2))) uint32_t u2r;

// 8-byte unit u (4 consecutive bf16 of a 512-B image row) of row n, XOR-
// swizzled so that the row reads (16 rows x units {8s + g, 8s + 4 + g}) and
// the transposed reads (8 rows x 4 units) of a 32-lane half hit 32 distinct
// bank pairs.
__device__ inline uint32_t r16_off(int n, int u) {
    const int sw = ((n & 7) << 2) | (((n >> 3) & 1) << 1);
    return (uint32_t)(n * 512 + ((u ^ sw) << 3));
}

// An opaque copy of a value (its uses cannot be computed before this point:
// the row-derived store addresses would otherwise be formed at the tile's
// start and held live across it).
template <typename V> __device__ inline V r16_late(V v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ inline f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// A fragment of a forward product from an LDS image: rows n = output feature,
// k-slots 8g + j = input features 32s + 16(j>>2) + 4g + (j&3): units 8s + g
// and 8s + 4 + g of row n.
__device__ inline bf16x8 r16_row_frag(const char* img, int n, int s, int g) {
    const u2r lo = *(const u2r*)(img + r16_off(n, 8 * s + g));
    const u2r hi = *(const u2r*)(img + r16_off(n, 8 * s + 4 + g));
    const u4r v = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8, v);
}

// A fragment of a backward product from the same image read transposed: M =
// image column (input feature 16b + (lane & 15)), k-slots 8g + j = image rows
// r0 + 4g + j (j < 4) and r0 + 16 + 4g + (j - 4) with r0 = 32s (hidden
// operands), or rows 8g + j with `step8` (the head's 32 columns, one k-step).
__device__ inline bf16x8 r16_tr_frag(const char* img, int rlo, int rhi, int b, int lane) {
    // (rlo, rhi split into a multiple of 16 rows, an instruction offset, and
    // a lane part that alone sets the swizzle: one block-dependent address
    // per lane and block)
    const int q = (lane >> 2) & 3, p = lane & 3;
    typedef __attribute__((address_space(3))) short4r* lp;
    const short4r lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lp)(img + (rlo & ~15) * 512 + r16_off((rlo & 15) + q, 4 * b + p)));
    const short4r hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lp)(img + (rhi & ~15) * 512 + r16_off((rhi & 15) + q, 4 * b + p)));
    typedef short short8r __attribute__((ext_vector_type(8)));
    const short8r v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

// 16-byte store of a weight-gradient operand row chunk (plain: nontemporal
// stores made the weight-gradient read miss the Infinity Cache, +9 us there)
__device__ inline void r16_st16(void* p, u4r v) { *(u4r*)p = v; }

__device__ inline uint32_t pk_bf16(float a, float b) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 v = {(bf16)a, (bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ inline f2v up_bf16(uint32_t w) {
    return f2v{__builtin_bit_cast(float, w << 16), __builtin_bit_cast(float, w & 0xffff0000u)};
}
// k-step s B fragment from packed words of blocks 2s, 2s+1 (the acc layout)
__device__ inline bf16x8 r16_bfrag(const uint32_t (&w)[kR16NB][2], int s) {
    const u4r v = {w[2 * s][0], w[2 * s][1], w[2 * s + 1][0], w[2 * s + 1][1]};
    return __builtin_bit_cast(bf16x8, v);
}

// acc[j] += sum_s A(j, s) B(s) over NBO output blocks and NS k-steps, A
// fragments from `lda(j, s)` through a ring of RING fragments in flight
// (sched_barrier fences keep the compiler from hoisting every read of the
// product ahead of its MFMAs, which would hold them all in registers).
template <int NBO, int NS, int RING, typename LDA, typename BF>
__device__ inline void r16_mm(f32x4 (&acc)[NBO], LDA lda, BF bfrag) {
    constexpr int N = NS * NBO;
    constexpr int RG = RING < N ? RING : N;
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 ra[RG];
#pragma unroll
    for (int i = 0; i < RG; ++i) ra[i] = lda(i % NBO, i / NBO);
    bf16x8 bfr = bfrag(0);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bf16x8 a = ra[i % RG];
        if (i + RG < N) ra[i % RG] = lda((i + RG) % NBO, (i + RG) / NBO);
        __builtin_amdgcn_sched_barrier(0);
        acc[i % NBO] = mma16(a, bfr, acc[i % NBO]);
        __builtin_amdgcn_sched_barrier(0);
        if ((i + 1) % NBO == 0 && i + 1 < N) bfr = bfrag((i + 1) / NBO);
    }
}

// As r16_mm, but block-pair-major: blocks 2p, 2p+1 take all NS k-steps
// (alternating, two independent accumulator chains) before the next pair, so
// a fragment address that depends on the block (the transposed reads) is
// formed once per block instead of once per (block, k-step); B fragments
// come from registers.
template <int NBO, int NS, int RING, typename LDA, typename BF>
__device__ inline void r16_mm_bm(f32x4 (&acc)[NBO], LDA lda, BF bfrag) {
    static_assert(NBO % 2 == 0, "block pairs");
    constexpr int N = NS * NBO;
    constexpr int RG = RING < N ? RING : N;
    auto jof = [](int i) { return 2 * (i / (2 * NS)) + (i & 1); };
    auto sof = [](int i) { return (i >> 1) % NS; };
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 ra[RG];
#pragma unroll
    for (int i = 0; i < RG; ++i) ra[i] = lda(jof(i), sof(i));
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bf16x8 a = ra[i % RG];
        if (i + RG < N) ra[i % RG] = lda(jof(i + RG), sof(i + RG));
        __builtin_amdgcn_sched_barrier(0);
        acc[jof(i)] = mma16(a, bfrag(sof(i)), acc[jof(i)]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// A forward layer's product Z^T = W^T X^T in two halves of 8 output blocks
// (32 accumulator registers at a time instead of 64), each half rounded to
// the compute dtype as it completes (flax Dense output dtype) and packed into
// zw; returns the LayerNorm statistics of the rows (f32 sums of the rounded
// values, fast variance, eps 1e-6; models.py:46-56).
template <int NS, int RING, typename LDA, typename BF>
__device__ inline void r16_fwd_layer(LDA lda, BF bfrag, uint32_t (&zw)[kR16NB][2], float& mean_o,
                                     float& rstd_o) {
    f2v s2 = {0.f, 0.f}, q2 = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        f32x4 acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        r16_mm<8, NS, RING>(acc, [&](int j, int s) { return lda(8 * h + j, s); }, bfrag);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                zw[8 * h + j][k] = pk_bf16(acc[j][2 * k], acc[j][2 * k + 1]);
                const f2v x = up_bf16(zw[8 * h + j][k]);
                s2 += x;
                q2 = x * x + q2;
            }
    }
    float sum = s2.x + s2.y, sq = q2.x + q2.y;
    sum = add_xor32(add_xor16(sum));
    sq = add_xor32(add_xor16(sq));
    const float invH = 1.0f / (float)kR16H;
    const float mean = sum * invH;
    const float var = fmaxf(sq * invH - mean * mean, 0.f);
    mean_o = mean;
    rstd_o = rsqrtf(var + 1e-6f);
}

// Row-major store of a [16 rows][256] bf16 operand held as packed words (lane
// (r, g): features 16b + 4g .. 4g+3 of every block b): one v_permlane16_swap
// per word pair leaves lane g with 8 consecutive features of block 2c + (g&1)
// (features 8(g>>1) .. +7), one 16-byte store per block pair.  In place.
__device__ inline void r16_store_rows(bf16* rowp, uint32_t (&w)[kR16NB][2], int g) {
#pragma unroll
    for (int c = 0; c < kR16NB / 2; ++c) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const auto v = __builtin_amdgcn_permlane16_swap(w[2 * c][k], w[2 * c + 1][k], false,
                                                            false);
            w[2 * c][k] = v[0];
            w[2 * c + 1][k] = v[1];
        }
        const int blk = 2 * c + (g & 1);
        r16_st16(rowp + 16 * blk + 8 * (g >> 1),
                 u4r{w[2 * c][0], w[2 * c][1], w[2 * c + 1][0], w[2 * c + 1][1]});
    }
}

// As r16_store_rows, leaving w as it was (the swaps go to temporaries).
__device__ inline void r16_store_rows_keep(bf16* rowp, const uint32_t (&w)[kR16NB][2], int g) {
#pragma unroll
    for (int c = 0; c < kR16NB / 2; ++c) {
        uint32_t t[2][2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const auto v = __builtin_amdgcn_permlane16_swap(w[2 * c][k], w[2 * c + 1][k], false,
                                                            false);
            t[0][k] = v[0];
            t[1][k] = v[1];
        }
        const int blk = 2 * c + (g & 1);
        r16_st16(rowp + 16 * blk + 8 * (g >> 1), u4r{t[0][0], t[0][1], t[1][0], t[1][1]});
    }
}

// A LayerNorm pass's per-block scale / bias reads (features 16b + 4g .. +3,
// f32, LDS) one block ahead: take(following) hands over the values loaded
// last and issues block `following`'s reads (< 0: none), so each read has a
// block's arithmetic to land.  Each take is a scheduling fence and each read
// index opaque: otherwise the compiler issues all 16 blocks' reads up front
// (128 registers).
struct R16GB {
    const float* gm;
    int g;
    float4 G, B;
    __device__ R16GB(const float* gm_, int g_, int first) : gm(gm_), g(g_) { load(first); }
    __device__ void load(int b) {
        const int f0 = r16_late(16 * b + 4 * g);
        G = *(const float4*)(gm + f0);
        B = *(const float4*)(gm + kR16H + f0);
    }
    // block b's values read now (no read ahead)
    __device__ void take_now(int b, float4& Go, float4& Bo) {
        __builtin_amdgcn_sched_barrier(0);
        load(b);
        Go = G;
        Bo = B;
    }
    __device__ void take(int following, float4& Go, float4& Bo) {
        __builtin_amdgcn_sched_barrier(0);
        Go = G;
        Bo = B;
        if (following >= 0) load(following);
    }
};

// LayerNorm apply + ReLU, rounded to the compute dtype: packed Z -> packed
// A (the next product's operand).
__device__ inline void r16_ln_apply(uint32_t (&zw)[kR16NB][2], float mean, float rstd,
                                    const float* gm, int g, uint32_t (&aw)[kR16NB][2]) {
    const f2v m2 = {mean, mean}, r2 = {rstd, rstd};
    R16GB gb(gm, g, 0);
#pragma unroll
    for (int b = 0; b < kR16NB; ++b) {
        float4 G, B;
        gb.take(b + 1 < kR16NB ? b + 1 : -1, G, B);
        // (words made opaque in place: the statistics pass's unpacked values
        // would otherwise be CSE'd into this one and held live, 64 registers
        // across the layer's whole product)
        zw[b][0] = r16_late(zw[b][0]);
        zw[b][1] = r16_late(zw[b][1]);
        const f2v y0 = __builtin_elementwise_fma(up_bf16(zw[b][0]) - m2, r2 * f2v{G.x, G.y},
                                                 f2v{B.x, B.y});
        const f2v y1 = __builtin_elementwise_fma(up_bf16(zw[b][1]) - m2, r2 * f2v{G.z, G.w},
                                                 f2v{B.z, B.w});
        aw[b][0] = pk_bf16(fmaxf(y0.x, 0.f), fmaxf(y0.y, 0.f));
        aw[b][1] = pk_bf16(fmaxf(y1.x, 0.f), fmaxf(y1.y, 0.f));
    }
}

// Division by a launch constant d (rows by the minibatch's sequence count,
// sequence ids by the policy's env count): q = (mulhi(n, mag) + n) >> sh,
// exact for n < 2^31 (magic from r16_magic on the host).
struct R16Div {
    uint32_t mb_mag, n_mag;
    int mb_sh, n_sh;
};
__device__ inline uint32_t r16_udiv(uint32_t n, uint32_t mag, int sh) {
    return (__umulhi(n, mag) + n) >> sh;
}


// Stage the weights every row-split kernel keeps in LDS (the prologue, all
// threads of the 8-wave workgroup; the caller's barrier orders it): W1 and
// head images (P.wt[1], P.head_t: fragment order, permuted k, K = 256)
// re-laid as [out row][512 B] with swizzled 8-byte units, LayerNorm scale /
// bias of both layers, head bias.
template <int HC = kR16HC>
__device__ inline void r16_stage(const PolicyK& P, char* smem, int tid) {
    typedef R16Lay<HC> LY;
    char* w1img = smem + LY::OffW1;
    char* whimg = smem + LY::OffWh;
    float* gb = (float*)(smem + LY::OffGb);
    float* hb = (float*)(smem + LY::OffHb);
    {
        const u4r* src1 = (const u4r*)P.wt[1];
        const u4r* srch = (const u4r*)P.head_t;
        constexpr int N1 = kR16H * kR16H * 2 / 16 / (64 * kR16Waves);  // 16 per thread
        u4r v1[N1], vh[2];
#pragma unroll
        for (int i = 0; i < N1; ++i) v1[i] = src1[tid + i * 64 * kR16Waves];
        if (HC == 32)
#pragma unroll
            for (int i = 0; i < 2; ++i) vh[i] = srch[tid + i * 64 * kR16Waves];
        float pv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int j = tid + i * 64 * kR16Waves, l = j >> 9, c = j & 511;
            pv[i] = c < kR16H ? P.lns[l][c] : P.lnb[l][c - kR16H];
        }
        const float hbv = tid < HC ? P.head_b[tid] : 0.f;
        // 16-byte unit U of a (K = 256, perm) image: n = ((U >> 10) << 5) | (U & 31),
        // h = (U >> 5) & 1, s16 = (U >> 6) & 15; its halves hold inputs
        // 16 s16 + 4h .. +3 and 16 s16 + 8 + 4h .. +3 (units 4 s16 + h, 4 s16 + 2 + h)
        auto put = [&](char* img, int U, u4r v) {
            const int n = ((U >> 10) << 5) | (U & 31), h = (U >> 5) & 1, s16 = (U >> 6) & 15;
            *(u2r*)(img + r16_off(n, 4 * s16 + h)) = u2r{v[0], v[1]};
            *(u2r*)(img + r16_off(n, 4 * s16 + 2 + h)) = u2r{v[2], v[3]};
        };
#pragma unroll
        for (int i = 0; i < N1; ++i) put(w1img, tid + i * 64 * kR16Waves, v1[i]);
        if (HC == 32)
#pragma unroll
            for (int i = 0; i < 2; ++i) put(whimg, tid + i * 64 * kR16Waves, vh[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) gb[tid + i * 64 * kR16Waves] = pv[i];
        if (tid < HC) hb[tid] = hbv;
        if (HC != 32 && tid < P.CB)  // the two-hot critic's bin values (dists.py:128-141)
            ((float*)(smem + LY::OffBins))[tid] = twohot_bin(tid, P.CB);
    }
}

// A fragment of the head's forward product (M = head column n, the k order of
// r16_row_frag) straight from the head's L2 image P.head_t (fragment order,
// permuted k, K = 256; img_index<bf16>(n, k, 256, true)): inputs 32s + 4g ..
// +3 and 32s + 16 + 4g .. +3 of column n are two 8-byte halves 1 KB apart.
__device__ inline bf16x8 r16_head_l2(const bf16* head_t, int n, int s, int g) {
    const int64_t base =
        ((int64_t)(((n >> 5) * 16 + 2 * s) * 64 + (n & 31) + 32 * (g & 1))) * 8 + 4 * (g >> 1);
    const u2r lo = *(const u2r*)(head_t + base);
    const u2r hi = *(const u2r*)(head_t + base + 512);
    const u4r v = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8, v);
}

// two_hot_cross_entropy_loss (dists.py:171-208; twohot_ce_g's arithmetic,
// the reference's bin weights as written) of one row's CB bin logits (bf16,
// LDS) against the return R, by the row's four lanes r + 16 g (bins g, g + 4,
// ...): every lane returns the loss and mean(), and writes scale * d loss /
// d logit of its own bins in place (bf16: every consumer rounds them).
__device__ inline float r16_twohot_ce(bf16* lr, int CB, float R, const float* bins, float scale,
                                      int g, float* mean_out) {
    float cle = 0.f, cgt = 0.f;
    for (int j = g; j < CB; j += 4) {
        cle += bins[j] <= R ? 1.f : 0.f;
        cgt += bins[j] > R ? 1.f : 0.f;
    }
    cle += __shfl_xor(cle, 16);
    cle += __shfl_xor(cle, 32);
    cgt += __shfl_xor(cgt, 16);
    cgt += __shfl_xor(cgt, 32);
    const int lo = min(max((int)cle - 1, 0), CB - 1);
    const int up = min(max(CB - (int)cgt, 0), CB - 1);
    const bool same = lo == up;
    const float dl = same ? 1.f : fabsf(bins[lo] - R);
    const float du = same ? 1.f : fabsf(bins[up] - R);
    const float tot = dl + du;
    const float wl = dl / tot, wu = du / tot;
    float mx = -3.4e38f;
    for (int j = g; j < CB; j += 4) mx = fmaxf(mx, to_f32(lr[j]));
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float se = 0.f;
    for (int j = g; j < CB; j += 4) se += __expf(to_f32(lr[j]) - mx);
    se += __shfl_xor(se, 16);
    se += __shfl_xor(se, 32);
    const int mid = (CB - 1) / 2;
    float acc = 0.f;
    for (int i = g; i < mid; i += 4) {
        const int a = mid - 1 - i, b = mid + 1 + i;
        acc += (__expf(to_f32(lr[a]) - mx) / se) * bins[a] +
               (__expf(to_f32(lr[b]) - mx) / se) * bins[b];
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    *mean_out = (__expf(to_f32(lr[mid]) - mx) / se) * bins[mid] + acc;
    const float lse = mx + __logf(se);
    const float llo = to_f32(lr[lo]), lup = to_f32(lr[up]);  // (read before the row's writes)
    const float loss = -(wl * (llo - lse) + wu * (lup - lse));
    const float wsum = wl + wu;
    for (int j = g; j < CB; j += 4) {
        const float pj = __expf(to_f32(lr[j]) - mx) / se;
        const float w = (j == lo ? wl : 0.f) + (j == up ? wu : 0.f);
        lr[j] = (bf16)((wsum * pj - w) * scale);
    }
    return loss;
}

// SymExpTwoHotDistribution.mean() (dists.py:143-169, twohot_mean_g's sums)
// of the CB bin logits of one row (bf16 in LDS), by the row's four lanes
// r, r + 16, r + 32, r + 48 (g = lane >> 4: bins g, g + 4, ...); every lane of
// the row returns it.
__device__ inline float r16_twohot_mean(const bf16* lr, int CB, const float* bins, int g) {
    float mx = -3.4e38f;
    for (int j = g; j < CB; j += 4) mx = fmaxf(mx, to_f32(lr[j]));
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float se = 0.f;
    for (int j = g; j < CB; j += 4) se += __expf(to_f32(lr[j]) - mx);
    se += __shfl_xor(se, 16);
    se += __shfl_xor(se, 32);
    const int mid = (CB - 1) / 2;
    float acc = 0.f;
    for (int i = g; i < mid; i += 4) {
        const int a = mid - 1 - i, b = mid + 1 + i;
        acc += (__expf(to_f32(lr[a]) - mx) / se) * bins[a] +
               (__expf(to_f32(lr[b]) - mx) / se) * bins[b];
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    return (__expf(to_f32(lr[mid]) - mx) / se) * bins[mid] + acc;
}

// (mulhi(n, mag) + n) >> sh == n / d for n < 2^31: sh = ceil(log2 d),
// mag = floor(2^32 (2^sh - d) / d) + 1 (tests/test_gpu_fullsize.py covers
// d = 4095 and powers of two)
static inline void r16_magic(uint32_t d, uint32_t& mag, int& sh) {
    int l = 0;
    while ((1ull << l) < d) ++l;
    mag = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    sh = l;
}

}  // namespace ml
