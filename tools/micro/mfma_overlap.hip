// mfma_overlap.hip -- microbenchmark: f64 MFMA throughput on gfx950 alone and next to VALU work.
// Modes (one 512-thread workgroup per CU, waves w and w+4 share a SIMD):
//   0: all 8 waves issue MFMA chains only
//   1: waves 0-3 MFMA only, waves 4-7 VALU only (f64 fma chains)        -> cross-wave overlap
//   2: waves 0-3 MFMA only, waves 4-7 VALU only (u32 mad_u64 like Philox)
//   3: all waves: 1 MFMA then NV independent f64 fma (same wave)         -> intra-wave overlap
//   4: waves 0-3 MFMA only, waves 4-7 idle
// Prints achieved MFMA TF/s (f64 16x16x4 = 2048 flop) per mode.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int MODE, int NV>
__global__ __launch_bounds__(512) void k(int iters, double *out, unsigned *uout) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    v4d acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = (v4d){0, 0, 0, 0};
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = lane + i;
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = lane * 7 + i;
    const bool mf = (MODE == 0 || MODE == 3) ? true : wave < 4;
    if (mf) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
                if (MODE == 3) {
#pragma unroll
                    for (int v = 0; v < NV; ++v) x[v & 7] = __builtin_fma(x[v & 7], 1.0000001, 1e-9);
                }
            }
        }
    } else if (MODE == 1) {
        for (int it = 0; it < iters * 16; ++it) {
#pragma unroll
            for (int v = 0; v < 8; ++v) x[v] = __builtin_fma(x[v], 1.0000001, 1e-9);
        }
    } else if (MODE == 2) {
        for (int it = 0; it < iters * 16; ++it) {
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                unsigned long long p = (unsigned long long)u[v] * 0xD2511F53ull;
                u[v] = (unsigned)(p >> 32) ^ (unsigned)p ^ v;
            }
        }
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < 8; ++i) s += x[i];
    unsigned us = 0;
    for (int i = 0; i < 8; ++i) us ^= u[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
    uout[blockIdx.x * 512 + threadIdx.x] = us;
}

template <int MODE, int NV>
static void run(const char *name, int nblk, int iters, double *out, unsigned *uout) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<MODE, NV><<<nblk, 512>>>(iters, out, uout);   // warm
    hipEventRecord(e0);
    k<MODE, NV><<<nblk, 512>>>(iters, out, uout);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const int mwaves = (MODE == 0 || MODE == 3) ? 8 : 4;
    const double flops = (double)nblk * mwaves * iters * 16 * 2048.0;
    printf("%-44s %8.3f ms  %7.2f TF/s  (%.1f%% of 78.6)\n", name, ms, flops / ms / 1e9, flops / ms / 1e9 / 78.6 * 100);
}

int main() {
    const int nblk = 256, iters = 4000;
    double *out; unsigned *uout;
    hipMalloc(&out, nblk * 512 * sizeof(double));
    hipMalloc(&uout, nblk * 512 * sizeof(unsigned));
    run<0, 0>("mode0 8 MFMA waves", nblk, iters, out, uout);
    run<4, 0>("mode4 4 MFMA waves + 4 idle", nblk, iters, out, uout);
    run<1, 0>("mode1 4 MFMA + 4 f64-FMA VALU waves", nblk, iters, out, uout);
    run<2, 0>("mode2 4 MFMA + 4 u32-mad VALU waves", nblk, iters, out, uout);
    run<3, 2>("mode3 8 waves, 2 f64 fma per MFMA", nblk, iters, out, uout);
    run<3, 4>("mode3 8 waves, 4 f64 fma per MFMA", nblk, iters, out, uout);
    run<3, 8>("mode3 8 waves, 8 f64 fma per MFMA", nblk, iters, out, uout);
    return 0;
}
