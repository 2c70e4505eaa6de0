// Row-split minibatch step (ppo.py:109-364 up to the weight-gradient
// operands) for the headline policy shape: bf16, H = 256, two trunk layers,
// scalar critic, head width 32.  Included by ppo.hip after ppo_step_kernel;
// same inputs, outputs and workspace layout (X_0, A_l, dZ_l, d head rows;
// per-32-row column and loss partials), so wgrad_kernel / reduce_grads_kernel
// consume either kernel's output unchanged.
//
// Why a second kernel.  ppo_step_kernel gives each 32-row tile a workgroup
// whose 8 waves split the 256 features: every layer ends in a LayerNorm whose
// row statistics cross the waves (a barrier) and an LDS exchange of the next
// product's operand (another barrier), and every tile streams its 16 KB-per-
// wave slice of W1 from L2 twice.  The tile's chain of ~12 latency-bound
// phases sets the kernel's time.  Here:
//   * one workgroup of 8 waves per CU stages W1 (128 KB) and the head weights
//     (16 KB) in LDS once, plus the LayerNorm / head-bias parameters;
//   * a wave owns whole rows -- two 16-row tiles, v_mfma_f32_16x16x32_bf16 --
//     so LayerNorm statistics are lane-local sums plus two cross-lane adds,
//     every product's activation operand comes straight from the previous
//     accumulators, and no barrier follows the prologue;
//   * the forward product reads W1 by row (two ds_read_b64 per fragment), the
//     backward product reads the same image transposed (ds_read_b64_tr_b16);
//   * the layer-0 weights (K = obs_dim) stream from L2 per tile.
// Orientation as rowtile.h: Z^T = W^T X^T, features on the MFMA M axis, the
// 16 rows of a tile on N (lane & 15); lane l holds features 16b + 4(l>>4) + i
// (i < 4) of accumulator block b.  k-step s of a product over hidden
// features takes blocks 2s, 2s+1, so its k-slot 8g + j is feature
// 32s + 16(j>>2) + 4g + (j&3) (g = lane >> 4) -- the A operand is read in
// that order.

#pragma once

// (included inside namespace ml by ppo.hip)

// One transpose-reduce level at lane distance D = 8 or 4 within a DPP row:
// lanes with bit D clear return a + (partner's a), the others b + (partner's
// b) -- two bank-masked v_add_f32_dpp writing complementary lane sets (no
// selects).  row_ror:N reads lane i - N of the row, so distance-4 lanes with
// bit 2 clear (banks 0, 2) read through ror:12 (= i + 4).
template <int D> __device__ inline float r16_pair_dpp(float a, float b) {
    float r;
    if constexpr (D == 8)
        asm volatile(
            "s_nop 1\n\t"
            "v_add_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
            "v_add_f32_dpp %0, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xc"
            : "=&v"(r)
            : "v"(a), "v"(b));
    else
        asm volatile(
            "s_nop 1\n\t"
            "v_add_f32_dpp %0, %1, %1 row_ror:12 row_mask:0xf bank_mask:0x5\n\t"
            "v_add_f32_dpp %0, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xa"
            : "=&v"(r)
            : "v"(a), "v"(b));
    return r;
}

// Feature whose column total lane (r, g) holds after r16_rowsum8 of block quad qd.
__device__ inline int r16_colf(int qd, int lane) {
    const int r = lane & 15, g = lane >> 4;
    return 16 * (4 * qd + (r >> 2)) + 4 * g + (r & 3);
}
// Column partials (bias, scale) of one layer's 4 block quads to a colpart row.
__device__ inline void r16_put_cols(float* cpl, const float (&cb)[4], const float (&cg)[4],
                                    int lane) {
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
        const int f = r16_colf(qd, lane);
        cpl[f] = cb[qd];
        cpl[kR16H + f] = cg[qd];
    }
}

// Sum of 16 values v over the 16 lanes of a DPP row (the 16 rows of a tile)
// by recursive halving, partners lane ^ 8 (done by the caller:
// w[i] = r16_pair_dpp<8>(v[i], v[i + 8])), ^ 4 (bank-masked), then ^ 2, ^ 1
// (select + DPP add); lane r returns the total of value index r.
__device__ inline float r16_rowsum8(const float (&w)[8], int lane) {
    float x[4], y[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = r16_pair_dpp<4>(w[i], w[i + 4]);
    const bool h1 = (lane & 2) != 0, h0 = (lane & 1) != 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float keep = h1 ? x[i + 2] : x[i], send = h1 ? x[i] : x[i + 2];
        y[i] = keep + xlane<2>(send);
    }
    const float keep = h0 ? y[1] : y[0], send = h0 ? y[0] : y[1];
    return keep + xlane<1>(send);
}

// LayerNorm + ReLU backward element (models.py:46-56 under jax.value_and_grad,
// f32 inside the LayerNorm): d loss / d A -> dy (ReLU' from the rounded
// output: rnd(y) > 0 <=> y > thr; padding rows carry no gradient), x_hat.
__device__ inline float r16_dy(float z, float mean, float rstd, float gam, float bet, float da,
                               bool live, float& xh) {
    const float zc = z - mean;
    xh = zc * rstd;
    const float y = __builtin_fmaf(zc, rstd * gam, bet);
    return ((y > relu_thr<bf16>()) & live) ? da : 0.f;
}

// dZ = rstd (u - mean(u) - x_hat mean(u x_hat)) of one block from u
__device__ inline void r16_dz_block(const f32x4& u, uint32_t (&zwb)[2], float mean,
                                    float rstd, float ca, float cbc, uint32_t (&dzb)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        zwb[k] = r16_late(zwb[k]);
        const f2v zc = up_bf16(zwb[k]) - f2v{mean, mean};
        const f2v d = f2v{rstd, rstd} * f2v{u[2 * k], u[2 * k + 1]} +
                      (f2v{ca, ca} * zc + f2v{cbc, cbc});
        dzb[k] = pk_bf16(d.x, d.y);
    }
}

// Layer backward (d loss / d A in acc, 64 registers) in two passes.  Pass 1,
// per block: dy (r16_dy), u = dy gamma kept in acc, the row sums su (u) and sv
// (u x_hat), and the column sums of the bias (dy) and scale (dy x_hat)
// gradients over the tile's 16 rows -- blocks of a quad in the order 0, 2, 1,
// 3, so the first transpose-reduce level (value j with j + 8) runs after each
// block pair with 8 values per sum live; lane (r, g) ends with quad qd's total
// of feature r16_colf(qd, lane).  Pass 2: dZ.
__device__ inline void r16_ln_bwd(f32x4 (&acc)[kR16NB], uint32_t (&zw)[kR16NB][2],
                                  float mean, float rstd, const float* gm, int g, int lane,
                                  bool live, uint32_t (&dzw)[kR16NB][2], float (&cb)[4],
                                  float (&cg)[4]) {
    // opaque copies (of the statistics and of every Z word read): the
    // forward's unpacked Z values / (z - mean) pairs are otherwise CSE'd into
    // this pass and held live from the forward LayerNorm
    mean = r16_late(mean);
    rstd = r16_late(rstd);
    float su = 0.f, sv = 0.f;
    constexpr int ord[4] = {0, 2, 1, 3};
    R16GB gb(gm, g, 0);
#pragma unroll
    for (int qd = 0; qd < kR16NB / 4; ++qd) {
        float wb[8], wg[8];
#pragma unroll
        for (int hp = 0; hp < 2; ++hp) {
            float pb[8], pg[8];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int step = 4 * qd + 2 * hp + k;
                const int b = 4 * qd + ord[2 * hp + k];
                float4 G, B;
                gb.take_now(b, G, B);  // (read ahead, one block early: slower)
                const float gv[4] = {G.x, G.y, G.z, G.w}, bv[4] = {B.x, B.y, B.z, B.w};
                zw[b][0] = r16_late(zw[b][0]);
                zw[b][1] = r16_late(zw[b][1]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float xh;
                    const float z = up_bf16(zw[b][i >> 1])[i & 1];
                    const float dy = r16_dy(z, mean, rstd, gv[i], bv[i], acc[b][i], live, xh);
                    const float u = dy * gv[i];
                    su += u;
                    sv = __builtin_fmaf(u, xh, sv);
                    acc[b][i] = u;
                    pb[4 * k + i] = dy;
                    pg[4 * k + i] = dy * xh;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                wb[4 * hp + i] = r16_pair_dpp<8>(pb[i], pb[4 + i]);
                wg[4 * hp + i] = r16_pair_dpp<8>(pg[i], pg[4 + i]);
            }
        }
        cb[qd] = r16_rowsum8(wb, lane);
        cg[qd] = r16_rowsum8(wg, lane);
    }
    su = add_xor32(add_xor16(su));
    sv = add_xor32(add_xor16(sv));
    const float invH = 1.0f / (float)kR16H;
    const float ca = -(rstd * rstd) * (sv * invH), cbc = -rstd * (su * invH);
#pragma unroll
    for (int b = 0; b < kR16NB; ++b) r16_dz_block(acc[b], zw[b], mean, rstd, ca, cbc, dzw[b]);
}

// diagnostic builds only (ML_STAMPS): s_memtime per phase held in SGPRs and
// written once per tile, so the stamps leave the VGPR allocation alone
#ifdef ML_STAMPS
#define R16_STAMP(i) (r16_st[i] = __builtin_amdgcn_s_memtime())
#define R16_STAMPS_OUT()                                                              \
    do {                                                                              \
        if (ws.stamps && (tid & 63) == 0)                                             \
            for (int i_ = 0; i_ < 13; ++i_)                                           \
                ws.stamps[((int64_t)ptile * NT + tt) * 16 + i_] = r16_st[i_];        \
    } while (0)
#else
#define R16_STAMP(i) \
    do {             \
    } while (0)
#define R16_STAMPS_OUT() \
    do {                 \
    } while (0)
#endif

// NW waves per workgroup (8: two per SIMD; 4 or 2: one per SIMD), NT 16-row
// tiles per wave (rows16_cfg).
template <bool METRICS, int NW, int NT, int HC>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu((NW + 3) / 4, (NW + 3) / 4))) void ppo_rows16_kernel(
    PolicyK P, RolloutK ro, const int32_t* __restrict__ mb_seq, int mb, int64_t M,
    const float* __restrict__ adv_st, HpK hp, WsK ws, R16Div dv) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef ML_STAMPS
    const uint64_t r16_t_entry = __builtin_amdgcn_s_memtime();
#endif
    typedef R16Lay<HC> LY;  // (HC = 96: a two-hot critic, the head image from L2)
    constexpr int LGS = LY::LGS, NHB = HC / 16;
    char* w1img = smem + LY::OffW1;
    char* whimg = smem + LY::OffWh;
    float* gb = (float*)(smem + LY::OffGb);
    float* hb = (float*)(smem + LY::OffHb);
    const float* bins = (const float*)(smem + LY::OffBins);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    bf16* lgs = (bf16*)(smem + LY::OffLg) + wave * 16 * LGS;
    const int K = P.K;
    constexpr int D = kR16D, DS = D / 32;  // the first layer's k-steps

    // ---- prologue: W1 and head images (P.wt[1], P.head_t: fragment order,
    // permuted k, K = 256) re-laid as [out row][512 B] with swizzled 8-byte
    // units; LayerNorm scale / bias, head bias, the loss tasks' group tables
    {
        static_assert(NW == kR16Waves, "r16_stage stages with kR16Waves waves");
        r16_stage<HC>(P, smem, tid);
        int* tab = (int*)(smem + LY::OffTab);
        if (tid <= MLEARN_MAX_GROUPS) {
            tab[tid] = P.off[tid];
            ((float*)tab)[MLEARN_MAX_GROUPS + 1 + tid] = tid < MLEARN_MAX_GROUPS ? hp.ecoef[tid] : 0.f;
            ((float*)tab)[2 * (MLEARN_MAX_GROUPS + 1) + tid] =
                tid < MLEARN_MAX_GROUPS ? hp.objw[tid] : 0.f;
        }
    }
    __syncthreads();
#ifdef ML_STAMPS
    const uint64_t r16_t_pro = __builtin_amdgcn_s_memtime();
#endif
    const int* t_off = (const int*)(smem + LY::OffTab);
    const float* t_ec = (const float*)t_off + MLEARN_MAX_GROUPS + 1;
    const float* t_ow = t_ec + MLEARN_MAX_GROUPS + 1;

    // this wave's index: rows [16 NT ptile, 16 NT (ptile + 1)), loss-partials
    // row ptile (32 rows at NT = 2 = a ppo_step tile; 16 rows at NT = 1, WsK::nlp)
    const int ptile = (int)blockIdx.x * NW + wave;
    const float as0 = adv_st[0], as1 = adv_st[1];
    // value normaliser values, loaded once (a load in the loss loop waits on
    // the tile's stores)
    VnVals vn{hp.norm_vals != 0, {0.f, 0.f, 0.f, 0.f}};
    if (hp.norm_vals)
        for (int i = 0; i < 4; ++i) vn.v[i] = adv_st[2 + i];
    LossAcc m;
    bool did = false;
    uint32_t dz0w[kR16NB][2];            // layer-0 dZ of the previous tile (stored late)
    float cb0[4], cg0[4];                // its layer-0 column partials (stored with it)
    float* prev_cp = nullptr;
    int64_t prev_row = -1;
    const int ntask = 16 * (K + 1);
    // minibatch row -> (time step, sequence slot); the slot's sequence id is
    // loaded one tile ahead (issued before, and waited on before, the tile's
    // stores: a load issued behind stores waits for them, vmcnt being in order)
    auto slot_of = [&](int64_t rw, uint32_t& tl) {
        const uint32_t f = (uint32_t)rw;
        tl = r16_udiv(f, dv.mb_mag, dv.mb_sh);
        return f - tl * (uint32_t)mb;
    };
    // store row of minibatch row rw from its slot's sequence id (store_row,
    // ppo_defs.h); padding rows (rw >= M) get row 0 (loaded, never used)
    auto srow_of = [&](int64_t rw, uint32_t seq) -> int64_t {
        uint32_t tl;
        (void)slot_of(rw, tl);
        const uint32_t c = r16_udiv(seq, dv.n_mag, dv.n_sh), b = seq - c * (uint32_t)ro.N;
        return rw < M ? ((int64_t)c * ro.bptt + tl) * ro.ld + b : 0;
    };
    int64_t sr_n;  // store row of this lane's row in the next tile
    {
        uint32_t tl;
        const int64_t rw = (int64_t)ptile * (16 * NT) + (tid & 15);
        sr_n = srow_of(rw, (uint32_t)mb_seq[slot_of(rw, tl)]);
    }

#pragma clang loop unroll(disable)
    for (int tt = 0; tt < NT; ++tt) {
        // the lane index through an opaque copy per tile: otherwise every
        // lane-derived LDS / weight address of the body is hoisted out of the
        // tile loop and held live across it (rollout kernel)
#ifdef ML_STAMPS
        uint64_t r16_st[13];
#endif
        R16_STAMP(0);
        const int lane = r16_late(tid & 63), r = lane & 15, g = lane >> 4;
        const int64_t row0 = (int64_t)ptile * (16 * NT) + 16 * tt;
        const int64_t row = row0 + r;
        const bool live = row < M;
        // (sr_n is VALU-written: reading it here needs no vmcnt wait, which the
        // loop header would otherwise take in full, stores included)
        const int64_t sr = sr_n;
        uint32_t seq_n = 0;
        if (tt + 1 < NT) {
            uint32_t tl;
            seq_n = (uint32_t)mb_seq[slot_of(row + 16, tl)];
        }
        // ---- layer 0: X_0 rows from the store (natural k order), W_0 from its
        // fragment-order image in L2 (P.wt[0], K = D, natural k): element
        // (n, k = 32s + 8g) at ((n/32 * D/16 + 2s + g/2) * 64 + n%32 + 32(g&1)) * 8
        bf16x8 xf[DS];
        const bf16* orow = (const bf16*)ro.obs + sr * D;
#pragma unroll
        for (int s = 0; s < DS; ++s)
            xf[s] = *(const bf16x8*)(orow + 32 * s + 8 * g);  // (padding rows: row 0)
        // (each use of the first layer takes its own opaque copy of the lane: the
        // forward's 16 fragment addresses are otherwise CSE'd into the
        // backward's recompute and held live across the tile)
        auto lda0 = [&](int ln) {
            const bf16* w0 = (const bf16*)P.wt[0];
            const int rr = ln & 15, gg = ln >> 4;
            return [=](int b, int s) {
                const int n = 16 * b + rr;
                const int64_t idx = ((int64_t)(((n >> 5) * (D >> 4) + 2 * s + (gg >> 1)) * 64 +
                                               (n & 31) + 32 * (gg & 1))) * 8;
                return *(const bf16x8*)(w0 + idx);
            };
        };
        // this lane's first two loss tasks (row r, group (lane + 64u) >> 4; group
        // K = the value): raw inputs loaded here, straight-line from valid
        // addresses (sr = 0 on padding rows), and combined after the first
        // layer (a branch or an early use here would wait on the previous
        // tile's stores, vmcnt being in order)
        const bool has_ret = ro.ret != nullptr, has_val = ro.values != nullptr;
        float t_adv = ro.adv[sr];
        float rv = (has_ret ? ro.ret : ro.adv)[sr], vv = (has_val ? ro.values : ro.adv)[sr];
        int ract[2];
        float rlp[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int grp = (lane + 64 * u) >> 4;
            const int ga = grp < K ? grp : K - 1;
            ract[u] = ro.actions[sr * K + ga];
            rlp[u] = ro.logp[sr * K + ga];
        }
        auto bf0 = [&](int s) { return xf[s]; };
        // Z_0 (packed) and its statistics stay live to the layer-0 backward
        uint32_t zw0[kR16NB][2], zw[kR16NB][2], aw[kR16NB][2];
        float mean0, rstd0, mean, rstd;
        r16_fwd_layer<DS, kR16Ring0>(lda0(r16_late(lane)), bf0, zw0, mean0, rstd0);
        // (the tile's loads are consumed here, ahead of its first stores)
        sr_n = srow_of(row + 16, r16_late(seq_n));
        // (action | return bits, old log-prob | old value) per task
        uint32_t t_a[2];
        float t_b[2];
        {
            t_adv = r16_late(t_adv);
            rv = r16_late(rv);
            vv = r16_late(vv);
            const float retv = has_ret ? rv : t_adv + vv;  // ret_at (ppo_defs.h)
            const float ov = has_val ? vv : 0.f;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int grp = (lane + 64 * u) >> 4;
                t_a[u] = grp < K ? (uint32_t)r16_late(ract[u]) : __builtin_bit_cast(uint32_t, retv);
                t_b[u] = grp < K ? r16_late(rlp[u]) : ov;
            }
        }
        R16_STAMP(1);
        // X_0 rows for the weight gradient (16 bytes per lane and k-step)
#ifndef ML_PROBE_NO_X0  // (timing probe only: numerics invalid without the store)
        {
            bf16* xrow = (bf16*)ws.x0 + r16_late(row) * D;
#pragma unroll
            for (int s = 0; s < DS; ++s)
                r16_st16(xrow + 32 * s + 8 * g, __builtin_bit_cast(u4r, xf[s]));
        }
#endif
        // the previous tile's layer-0 dZ rows go out behind this tile's loads
        if (tt > 0) {
            r16_store_rows((bf16*)ws.dz[0] + r16_late(prev_row) * kR16H, dz0w, g);
            r16_put_cols(prev_cp, cb0, cg0, lane);
        }
        r16_ln_apply(zw0, mean0, rstd0, gb, g, aw);
        R16_STAMP(2);
        // ---- layer 1 (W1 from LDS)
        r16_fwd_layer<kR16KS, kR16Ring>(
            [&](int b, int s) { return r16_row_frag(w1img, 16 * b + r, s, g); },
            [&](int s) { return r16_bfrag(aw, s); }, zw, mean, rstd);
        R16_STAMP(3);
        // the second wave of each SIMD (waves 4..7) loses issue arbitration to
        // the first throughout (tile 0 ends ~24 % later); it takes priority from
        // its first tile's layer-1 output on, so the two finish closer together
        // (update 8.43-8.50 -> 8.36-8.38 ms on one box; from the last tile's
        // start: -1..2 % kernel time; from the kernel's start: slower)
        if (NW > 4 && tt == 0 && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
#ifndef ML_PROBE_NO_A0  // (timing probe only)
        r16_store_rows((bf16*)ws.a[0] + r16_late(row) * kR16H, aw, g);  // A_0 rows
#endif
        r16_ln_apply(zw, mean, rstd, gb + 2 * kR16H, g, aw);
        R16_STAMP(4);
        // ---- heads (models.py:122-154): logits / value = rnd(rnd(A_1 Wh) + rnd(b))
        f32x4 ha[NHB];
#pragma unroll
        for (int j = 0; j < NHB; ++j) ha[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (HC == 32) {
            r16_mm<NHB, kR16KS, 4>(
                ha, [&](int j, int s) { return r16_row_frag(whimg, 16 * j + r, s, g); },
                [&](int s) { return r16_bfrag(aw, s); });
        } else {  // the head image from L2 (R16Lay): a uniform part (j, s) + one lane offset
            const bf16* ht = (const bf16*)P.head_t;
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
        r16_store_rows((bf16*)ws.a[1] + r16_late(row) * kR16H, aw, g);  // A_1 rows
        {
            bf16* lr = lgs + r * LGS;
#pragma unroll
            for (int cbk = 0; cbk < NHB; ++cbk) {
                const int c0 = 16 * cbk + 4 * g;
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = rnd<bf16>(rnd<bf16>(ha[cbk][i]) + rnd<bf16>(hb[c0 + i]));
                *(u2r*)(lr + c0) = u2r{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])};
            }
        }
        wave_lds_sync();
        R16_STAMP(5);
        // ---- loss: one (row, group | value) task per lane and pass (ppo.py:129-262),
        // d loss / d logits written over the logits (bf16: every consumer rounds them)
        // one task: padding rows get zero d logits
        auto loss_task = [&](int task, int act, float olp, float adv, float ret, float oval) {
            const int rr = task & 15, grp = task >> 4;
            bf16* lr = lgs + rr * LGS;
            if (row0 + rr >= M) {
                if (grp < K)
                    for (int j = t_off[grp]; j < t_off[grp + 1]; ++j) lr[j] = (bf16)0.f;
                else if (HC == 32)
                    for (int j = P.A; j < HC; ++j) lr[j] = (bf16)0.f;
                return;
            }
            if (grp < K) {
                if (hp.norm_adv) adv = (adv - as0) * as1;
                const int o0 = t_off[grp];
                loss_group(hp, lr + o0, t_off[grp + 1] - o0, act, olp, adv, t_ec[grp], t_ow[grp],
                           m);
            } else if (HC == 32) {
                loss_value(hp, lr, P.A, HC, ret, oval, m, vn);
            }  // (HC = 96: the two-hot value loss runs below, four lanes per row)
        };
        {
            // the tasks' inputs are registers loaded at the tile's start (K + 1 <= 8
            // groups: two tasks per lane; no load in this loop, whose waits
            // would cover the tile's stores)
#pragma clang loop unroll(disable)
            for (int task = lane, u = 0; task < ntask; task += 64, ++u) {
                did = true;
                const uint32_t a = u == 0 ? t_a[0] : t_a[1];
                const float b = u == 0 ? t_b[0] : t_b[1];
                loss_task(task, (int)a, b, t_adv, __builtin_bit_cast(float, a), b);
            }
        }
        if constexpr (HC != 32) {
            // DreamerV3Critic (ppo.py:169-177): two-hot cross entropy of the
            // return against the bin logits, by the row's four lanes; the return
            // is the value task's input (task 16 K + r: lane (16 K + r) % 64 of
            // pass K / 4); padding rows and columns A + CB .. HC - 1 get zero
            wave_lds_sync();  // (the group tasks' writes precede the rows' reads)
            const uint32_t rbits = __shfl(K >= 4 ? t_a[1] : t_a[0], (16 * K + r) & 63);
            bf16* lr = lgs + r * LGS;
            const int CB = P.CB;
            if (row0 + r < M) {
                float mean;
                const float R = __builtin_bit_cast(float, rbits);
                const float vl = r16_twohot_ce(lr + P.A, CB, R, bins,
                                               hp.vcoef * hp.inv_s * hp.loss_scale, g, &mean);
                if (g == 0) {
                    const float verr = fabsf(mean - R);
                    m.svl += vl;
                    m.qvl += vl * vl;
                    m.mnvl = fminf(m.mnvl, vl);
                    m.mxvl = fmaxf(m.mxvl, vl);
                    m.serr += verr;
                    m.qerr += verr * verr;
                    m.mnerr = fminf(m.mnerr, verr);
                    m.mxerr = fmaxf(m.mxerr, verr);
                }
            } else {
                for (int j = P.A + g; j < P.A + CB; j += 4) lr[j] = (bf16)0.f;
            }
            for (int j = P.A + CB + g; j < HC; j += 4) lr[j] = (bf16)0.f;
        }
        wave_lds_sync();
        R16_STAMP(6);
        // ---- d head: B operand of the head backward (cols 8g .. 8g+7 of row r),
        // row-major store, head-bias column sums
        // (k-step s of the head backward: columns 32 s + 8 g .. + 7)
        constexpr int HKS = HC / 32;
        bf16x8 dh[HKS];
#pragma unroll
        for (int s2 = 0; s2 < HKS; ++s2) {
            dh[s2] = *(const bf16x8*)(lgs + r * LGS + 32 * s2 + 8 * g);
            r16_st16((bf16*)ws.dhead + r16_late(row) * HC + 32 * s2 + 8 * g,
                     __builtin_bit_cast(u4r, dh[s2]));
        }
        // column partials of this 16-row tile (colpart row NT ptile + tt, WsK::ncp):
        // head bias here, LayerNorm bias / scale in the layer backwards
        float* cprow = ws.colpart + ((int64_t)ptile * NT + tt) * ws.CP;
#pragma unroll
        for (int c0 = 0; c0 < HC; c0 += 64) {
            if (c0 + lane < HC) {
                float hbs = 0.f;
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) hbs += to_f32(lgs[rr * LGS + c0 + lane]);
                cprow[2 * 2 * kR16H + c0 + lane] = hbs;
            }
        }
        // ---- layer 1 backward: dA_1^T = Wh dHead^T (M = hidden unit = image
        // column, K = head column), recomputed per half in the LayerNorm's
        // second pass
        R16_STAMP(7);
        uint32_t dzw[kR16NB][2];
        {
            f32x4 hacc[kR16NB];
#pragma unroll
            for (int b = 0; b < kR16NB; ++b) hacc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (HC == 32) {
                r16_mm<kR16NB, 1, kR16Ring>(
                    hacc,
                    [&](int b, int) { return r16_tr_frag(whimg, 8 * g, 8 * g + 4, b, lane); },
                    [&](int) { return dh[0]; });
            } else {
                // the head image P.head from L2 (fragment order, natural k,
                // K = HC: img_index<bf16>(n, k, 96, false)): hidden unit n = 16 b + r,
                // columns 32 s + 8 g .. + 7 are 16 contiguous bytes, a uniform part
                // (b, s) plus one lane offset
                const bf16* hd = (const bf16*)P.head;
                const uint32_t lo = r16_late((uint32_t)((g >> 1) * 512 + (r + 32 * (g & 1)) * 8));
                r16_mm<kR16NB, HKS, kR16RingH>(
                    hacc,
                    [&](int b, int s2) {
                        const bf16* p = hd + ((b >> 1) * (HC / 16) * 512 + s2 * 1024 + (b & 1) * 128);
                        return *(const bf16x8*)(p + lo);
                    },
                    [&](int s2) { return dh[s2]; });
            }
            float cb1[4], cg1[4];
            r16_ln_bwd(hacc, zw, mean, rstd, gb + 2 * kR16H, g, lane, live, dzw, cb1, cg1);
            r16_put_cols(cprow + 2 * kR16H, cb1, cg1, lane);
        }
        // dA_0^T = W1 dZ_1^T: M = input feature (image column), K = output feature
        // (image rows 32s + 4g + j, 32s + 16 + 4g + j)
        // dZ_1 rows out now, ahead of the W1^T product and the layer-0
        // backward: the next tile's first loads wait for them (vmcnt in order)
        r16_store_rows_keep((bf16*)ws.dz[1] + r16_late(row) * kR16H, dzw, g);
        R16_STAMP(8);
        f32x4 acc[kR16NB];
#pragma unroll
        for (int b = 0; b < kR16NB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
        r16_mm_bm<kR16NB, kR16KS, kR16Ring>(
            acc,
            [&](int b, int s) {
                return r16_tr_frag(w1img, 32 * s + 4 * g, 32 * s + 16 + 4 * g, b, lane);
            },
            [&](int s) { return r16_bfrag(dzw, s); });
        R16_STAMP(9);
        R16_STAMP(10);
        // ---- layer 0 LayerNorm / ReLU backward
        R16_STAMP(11);
        r16_ln_bwd(acc, zw0, mean0, rstd0, gb, g, lane, live, dz0w, cb0, cg0);
        prev_row = row;
        prev_cp = cprow;
        R16_STAMP(12);
        R16_STAMPS_OUT();
    }
    const int lane = tid & 63, r = lane & 15, g = lane >> 4;
    r16_store_rows((bf16*)ws.dz[0] + prev_row * kR16H, dz0w, g);
    r16_put_cols(prev_cp, cb0, cg0, lane);

#ifdef ML_STAMPS
    {  // entry, after the prologue, end (last stores completed), in tile 0's row
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t t_end = __builtin_amdgcn_s_memtime();
        if (ws.stamps && (tid & 63) == 0) {
            uint64_t* st = ws.stamps + (int64_t)ptile * NT * 16;
            st[13] = r16_t_entry;
            st[14] = r16_t_pro;
            st[15] = t_end;
        }
    }
#endif
    // ---- loss metrics of this wave's rows (only the minibatch whose metrics survive)
    if (METRICS) {
        const float vals[kLossSlots] = {m.sobj, m.qobj, m.mnobj, m.mxobj, m.svl, m.qvl, m.mnvl,
                                        m.mxvl, m.serr, m.qerr, m.mnerr, m.mxerr, m.sent, m.qent,
                                        m.mnent, m.mxent, m.sentw, m.sobjw, 0.f, 0.f};
        constexpr int kUsed = 18;
        double* lp = ws.loss_part + (int64_t)ptile * kLossSlots;
        if (__any(did)) {
#pragma unroll
            for (int s = 0; s < kUsed; ++s) {
                const int kind = (s < 16) ? (s & 3) : 0;
                float v = vals[s];
                v = kind == 2 ? wave_reduce<2>(v) : (kind == 3 ? wave_reduce<3>(v) : wave_reduce<0>(v));
                if (lane == 0) lp[s] = v;
            }
            if (lane >= kUsed && lane < kLossSlots) lp[lane] = 0.0;
        } else if (lane < kLossSlots) {
            const int kind = (lane < 16) ? (lane & 3) : 0;
            lp[lane] = kind == 2 ? 3.4e38 : (kind == 3 ? -3.4e38 : 0.0);
        }
    }
}

// The row-split kernel runs the bf16, H = 256, two-layer, scalar-critic step
// in a shape that gives every CU one 8-wave workgroup: 2 tiles per wave (256
// rows per workgroup) from 65 536 rows, 1 tile per wave at exactly 32 768
// rows (a two-rank data-parallel slice); nw = 0 where it does not apply.
// (Measured and not kept, profiles/r05_rank_slices_ab.txt: 4 x 1 and 2 x 1
// waves x tiles at 16 384 / 8 192 rows, one wave per SIMD: 32.4 / 30.3 us
// against the feature split's 19.6 us at 8 192 rows -- a lone wave exposes
// its whole tile chain.)
struct R16Cfg {
    int nw, nt;
};
static R16Cfg rows16_cfg(int64_t Mp) {
    const int cus = device_cus();
    const int64_t kCUs = cus > 0 ? cus : 256;  // (256: MI355X, when no device answers)
    if (Mp % 256 == 0 && Mp / 256 >= kCUs) return R16Cfg{8, 2};
    if (Mp == 128 * kCUs) return R16Cfg{8, 1};  // exactly one round of workgroups
    return R16Cfg{0, 0};
}
static bool rows16_eligible(const PolicyK& P, int64_t Mp, int HC, int L, int H, bool bf) {
    // head: the scalar critic at width 32, or (round 6) a two-hot critic at
    // width 96 (R16Lay: the head image streamed from L2)
    const bool head = (HC == 32 && P.CB == 1) || (HC == 96 && P.CB > 1 && P.CB <= 64);
    return bf && H == kR16H && L == 2 && head && P.D == kR16D && P.K + 1 <= 8 &&
           rows16_cfg(Mp).nw > 0;
}

template <int NW, int NT, int HC>
static void launch_rows16_cfg(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                              int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                              const R16Div& dv, hipStream_t s) {
    constexpr int lds = (int)R16Lay<HC>::Lds;
    // (once per shape and device, kept out of graph capture)
    if (set_lds_attr((const void*)ppo_rows16_kernel<true, NW, NT, HC>, lds, "ppo_rows16") ||
        set_lds_attr((const void*)ppo_rows16_kernel<false, NW, NT, HC>, lds, "ppo_rows16"))
        return;  // (the caller's check_launch reports a failed launch; the message is set)
    const int grid = (int)(ws.Mp / (16 * NW * NT));
    if (hp.metrics)
        hipLaunchKernelGGL((ppo_rows16_kernel<true, NW, NT, HC>), dim3(grid), dim3(64 * NW), lds,
                           s, P, R, mb_seq, mb, M, adv_st, hp, ws, dv);
    else
        hipLaunchKernelGGL((ppo_rows16_kernel<false, NW, NT, HC>), dim3(grid), dim3(64 * NW), lds,
                           s, P, R, mb_seq, mb, M, adv_st, hp, ws, dv);
}

// (the caller sets ws.ncp / ws.nlp to the row-split partial-row counts)
static void launch_rows16(const PolicyK& P, const RolloutK& R, const int32_t* mb_seq, int mb,
                          int64_t M, const float* adv_st, const HpK& hp, const WsK& ws,
                          hipStream_t s) {
    R16Div dv;
    r16_magic((uint32_t)mb, dv.mb_mag, dv.mb_sh);
    r16_magic((uint32_t)R.N, dv.n_mag, dv.n_sh);
    const R16Cfg c = rows16_cfg(ws.Mp);
    if (P.HC == 32) {
        if (c.nt == 2)
            launch_rows16_cfg<8, 2, 32>(P, R, mb_seq, mb, M, adv_st, hp, ws, dv, s);
        else
            launch_rows16_cfg<8, 1, 32>(P, R, mb_seq, mb, M, adv_st, hp, ws, dv, s);
    } else {
        if (c.nt == 2)
            launch_rows16_cfg<8, 2, 96>(P, R, mb_seq, mb, M, adv_st, hp, ws, dv, s);
        else
            launch_rows16_cfg<8, 1, 96>(P, R, mb_seq, mb, M, adv_st, hp, ws, dv, s);
    }
}
