// GAE kernel variant sweep (diagnostic tool, not part of the library):
// times gae_kernel<VEC, U> launch shapes at N = 2^22, T = 32 with HIP events.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I madrona-learn_amd/csrc -I include \
//         tools/gae_sweep.hip -o tools/gae_sweep.bin
#include "../madrona-learn_amd/csrc/misc.hip"
#include <vector>

using namespace ml;

template <int VEC, int U, int BS>
static float run(const float* r, const float* v, const uint8_t* d, const float* b, float* a,
                 float* rt, int T, int64_t N) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    dim3 grid((unsigned)((N / VEC + BS - 1) / BS));
    hipLaunchKernelGGL((gae_kernel<VEC, U>), grid, dim3(BS), 0, 0, r, v, d, b, a, rt, T, N, 0.99f,
                       0.95f * 0.99f);
    hipEventRecord(e0, 0);
    const int it = 20;
    for (int i = 0; i < it; ++i)
        hipLaunchKernelGGL((gae_kernel<VEC, U>), grid, dim3(BS), 0, 0, r, v, d, b, a, rt, T, N,
                           0.99f, 0.95f * 0.99f);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / it;
}

int main() {
    const int T = 32;
    const int64_t N = 1 << 22;
    float *r, *v, *b, *a, *rt;
    uint8_t* d;
    hipMalloc(&r, T * N * 4);
    hipMalloc(&v, T * N * 4);
    hipMalloc(&a, T * N * 4);
    hipMalloc(&rt, T * N * 4);
    hipMalloc(&b, N * 4);
    hipMalloc(&d, T * N);
    hipMemset(r, 0, T * N * 4);
    hipMemset(v, 0, T * N * 4);
    hipMemset(b, 0, N * 4);
    hipMemset(d, 0, T * N);
    const double bytes = (double)T * N * 17 + 4.0 * N;
    auto rep = [&](const char* name, float us) {
        printf("%-22s %8.1f us  %7.0f GB/s  %.3f of 8 TB/s\n", name, us, bytes / us * 1e-3,
               bytes / us * 1e-3 / 8000.0);
    };
    rep("VEC1 U16 BS64", run<1, 16, 64>(r, v, d, b, a, rt, T, N));
    rep("VEC1 U8 BS256", run<1, 8, 256>(r, v, d, b, a, rt, T, N));
    rep("VEC1 U4 BS256", run<1, 4, 256>(r, v, d, b, a, rt, T, N));
    // copy reference: hipMemcpy D2D of the same byte count
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int i = 0; i < 20; ++i) hipMemcpyAsync(a, r, T * N * 4, hipMemcpyDeviceToDevice, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const float us = ms * 1e3f / 20;
    printf("%-22s %8.1f us  %7.0f GB/s (read+write)\n", "memcpy D2D 512MB", us,
           2.0 * T * N * 4 / us * 1e-3);
    return 0;
}
