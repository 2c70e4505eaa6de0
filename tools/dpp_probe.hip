// Diagnostic: lane-exchange primitives used by rowtile.h, checked on the GPU.
//   hipcc --offload-arch=gfx950 -O2 -I madrona-learn_amd/csrc tools/dpp_probe.hip -o /tmp/dpp_probe
#include <cstdio>
#include "rowtile.h"
using namespace ml;

__device__ float x16_copy(float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return a + b;
}
__device__ float x32_copy(float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return a + b;
}

__global__ void probe(float* out) {
    const int lane = threadIdx.x;
    const float v = (float)lane;
    out[5 * 64 + lane] = x16_copy(v) - v;
    out[6 * 64 + lane] = x32_copy(v) - v;
    out[0 * 64 + lane] = ML_DPP(v, 0x124);   // row_ror:4
    out[1 * 64 + lane] = ML_DPP(v, 0x12C);   // row_ror:12
    out[2 * 64 + lane] = add_xor16(v) - v;   // partner ^ 16
    float a[16];
    for (int q = 0; q < 16; ++q) a[q] = (float)(lane * 16 + q);
    out[3 * 64 + lane] = col_sum16(a, lane);
    out[4 * 64 + lane] = (float)col_sum16_index(lane);
}

int main() {
    float* d;
    hipMalloc(&d, 7 * 64 * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    float h[7 * 64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d ror4<-%2.0f ror12<-%2.0f x16<-%2.0f x16c<-%2.0f x32c<-%2.0f", l, h[l], h[64 + l], h[128 + l], h[320 + l], h[384 + l]);
        // expected column sum: sum over lanes of the same half of (lane*16 + q*)
        int q = (int)h[256 + l], half = l >> 5;
        double e = 0;
        for (int m = 0; m < 32; ++m) e += (half * 32 + m) * 16 + q;
        printf("  colsum q*=%2d got %8.0f want %8.0f%s\n", q, h[192 + l], e, h[192 + l] == e ? "" : "  BAD");
        bad += h[192 + l] != e;
    }
    printf("bad %d\n", bad);
    return bad != 0;
}
