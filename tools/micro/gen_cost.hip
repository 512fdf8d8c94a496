// gen_cost.hip -- microbenchmark: cycles per wave for one Philox4x32-10 call + 4 float Gaussians
// (rng_core.hpp, bitwise glibc Box-Muller), alone and next to f64 MFMA waves on the same SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../randblas_amd/csrc/rng_core.hpp"

typedef double v4d __attribute__((ext_vector_type(4)));

template <int WHAT, bool MF>
__global__ __launch_bounds__(512) void k(int iters, int calls, double *out) {
    __shared__ rb::LogfEntry tab[16];
    if (threadIdx.x < 16) tab[threadIdx.x] = rb::LOGF_TAB[threadIdx.x];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    v4d acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = (v4d){0, 0, 0, 0};
    double s = 0;
    if (wave < 4) {
        if (MF)
            for (int it = 0; it < iters; ++it)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    } else {
        for (int it = 0; it < calls; ++it) {
            const rb::u32x4 w = rb::philox4x32<10>(lane + it, blockIdx.x, 7, 9, 0x1234u, 0x5678u);
            if (WHAT == 0) {
                s += (double)(w.v[0] ^ w.v[1] ^ w.v[2] ^ w.v[3]);
            } else {
                float g[4];
                rb::sample4<rb::GAUSSIAN>(w, g, tab);
                s += (double)g[0] + (double)g[1] + (double)g[2] + (double)g[3];
            }
        }
    }
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int WHAT, bool MF>
static float run(const char *name, int iters, int calls, double *out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<WHAT, MF><<<256, 512>>>(iters, calls, out);
    (void)hipEventRecord(e0);
    k<WHAT, MF><<<256, 512>>>(iters, calls, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-36s %8.3f ms  %.0f cycles/wave-call\n", name, ms, calls ? ms * 1e-3 * 2.4e9 / calls : 0.0);
    return ms;
}

int main() {
    double *out;
    (void)hipMalloc(&out, 256 * 512 * sizeof(double));
    const int calls = 8000, iters = 4000;
    run<0, true>("MFMA only (4 waves)", iters, 0, out);
    run<0, false>("philox only", 0, calls, out);
    run<1, false>("philox + 2 boxmuller only", 0, calls, out);
    run<0, true>("philox + MFMA", iters, calls, out);
    run<1, true>("philox + boxmuller + MFMA", iters, calls, out);
    return 0;
}
