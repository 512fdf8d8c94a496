// mfma_coexec.hip -- does VALU work of one wave overlap the MFMAs of its SIMD partner on gfx950?
// One 512-thread workgroup per CU (two waves per SIMD: w and w + 4). The MFMA waves issue
// back-to-back MFMAs of one type (16 independent accumulators); their partners run a VALU loop.
// Each wave stamps s_memtime around its loop; printed: average cycles of the MFMA waves and of the
// VALU waves, run alone and together. Variants: which half is the MFMA half (older waves 0-3 or
// younger 4-7) and the VALU waves' s_setprio.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_coexec mfma_coexec.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

// KIND 0 f32 FMA, 1 f64 FMA, 2 int32, 3 ds_read_b64, 4 ds_write_b128, 5 global_load_dwordx4 (L2-resident
// 64 KiB), 6 global_load_lds_dwordx4 (the same bytes straight into LDS)
template <int KIND>
__device__ __forceinline__ void valu_loop(int n, float &f, double &d, uint32_t &u, double *lds, const double *g) {
    const int lane = threadIdx.x & 63;
    for (int i = 0; i < n; ++i) {
        if (KIND <= 2) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (KIND == 0) f = __builtin_fmaf(f, 1.0000001f, 0.5f);
                if (KIND == 1) d = __builtin_fma(d, 1.0000000001, 0.5);
                if (KIND == 2) u = (u ^ (u >> 3)) + 0x9E3779B9u;
            }
        } else if (KIND == 3) {
#pragma unroll
            for (int j = 0; j < 16; ++j) d += lds[(lane * 2 + j * 128 + (u & 1)) & 4095];
        } else if (KIND == 4) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                typedef double v2d __attribute__((ext_vector_type(2)));
                *reinterpret_cast<v2d *>(lds + ((lane * 2 + j * 128) & 4095)) = (v2d){d, d + j};
            }
        } else if (KIND == 5) {
            typedef double v2d __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const v2d x = *reinterpret_cast<const v2d *>(g + ((i * 16 + j) * 128 + lane * 2) % 8192);
                d += x[0];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(g + ((i * 16 + j) * 128 + lane * 2) % 8192),
                                                 (__attribute__((address_space(3))) void *)(lds + (j & 3) * 128), 16, 0, 0);
        }
        asm volatile("" : "+v"(f), "+v"(d), "+v"(u));
    }
    if (KIND == 6) d += lds[lane];
}

// MT: 0 f64 16x16x4, 1 f32 16x16x4, 2 bf16 32x32x16.  MODE bit 0: MFMA half runs, bit 1: VALU half runs.
template <int MT, int KIND, int MODE, bool MFMA_YOUNG, int PRIO>
__global__ __launch_bounds__(512) void coexec(int n_mfma, int n_valu, unsigned long long *out, const double *g) {
    __shared__ __attribute__((aligned(16))) double lds[4096];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const bool is_mfma = MFMA_YOUNG ? wave >= 4 : wave < 4;
    float f = lane;
    double d = lane;
    uint32_t u = lane;
    v4d accd[16];
    v4f accf[16];
    v16f accb[8];
    for (int i = 0; i < 16; ++i) { accd[i] = (v4d){0, 0, 0, 0}; accf[i] = (v4f){0, 0, 0, 0}; }
    for (int i = 0; i < 8; ++i) for (int j = 0; j < 16; ++j) accb[i][j] = 0;
    const double a = 1.0 + lane * 1e-3, b = 2.0 - lane * 1e-3;
    v8bf ab, bb;
    for (int j = 0; j < 8; ++j) { ab[j] = (__bf16)(1.0f + lane * 1e-2f); bb[j] = (__bf16)(0.5f); }
    __syncthreads();
    if (!is_mfma && PRIO) __builtin_amdgcn_s_setprio(PRIO);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (is_mfma) {
        if (MODE & 1)
            for (int i = 0; i < n_mfma; ++i) {
                if (MT == 0) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) accd[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, accd[j], 0, 0, 0);
                } else if (MT == 1) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) accf[j] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)a, (float)b, accf[j], 0, 0, 0);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) accb[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, accb[j], 0, 0, 0);
                }
            }
    } else {
        if (MODE & 2) valu_loop<KIND>(n_valu, f, d, u, lds + (wave & 3) * 1024 * 0, g);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = f + d + u;
    for (int i = 0; i < 16; ++i) s += accd[i][0] + accf[i][1];
    for (int i = 0; i < 8; ++i) s += accb[i][3];
    if (lane == 0) {
        atomicAdd(&out[is_mfma ? 0 : 1], t1 - t0);
        if (s == 12345.678) out[2] = 1;   // keep the work
    }
}

static const double *g_buf;
template <int MT, int KIND, int MODE, bool MFMA_YOUNG, int PRIO>
static void run(const char *name, int n_mfma, int n_valu, unsigned long long *dout) {
    (void)hipMemset(dout, 0, 3 * sizeof(unsigned long long));
    hipLaunchKernelGGL((coexec<MT, KIND, MODE, MFMA_YOUNG, PRIO>), dim3(256), dim3(512), 0, 0, n_mfma, n_valu, dout, g_buf);
    unsigned long long h[3];
    (void)hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
    printf("%-34s mode %d: mfma waves %9.0f cyc, valu waves %9.0f cyc\n", name, MODE, h[0] / 1024.0, h[1] / 1024.0);
}

#define CASE(MT, KIND, YOUNG, PRIO, NAME)                        \
    run<MT, KIND, 1, YOUNG, PRIO>(NAME, nm, nv, dout);           \
    run<MT, KIND, 2, YOUNG, PRIO>(NAME, nm, nv, dout);           \
    run<MT, KIND, 3, YOUNG, PRIO>(NAME, nm, nv, dout);

int main() {
    unsigned long long *dout;
    (void)hipMalloc(&dout, 3 * sizeof(unsigned long long));
    double *gb;
    (void)hipMalloc(&gb, 8192 * sizeof(double));
    (void)hipMemset(gb, 0, 8192 * sizeof(double));
    g_buf = gb;
    const int nm = 200, nv = 1000;
    run<0, 0, 1, false, 0>("warm-up", nm, nv, dout);
    CASE(0, 0, false, 0, "f64mfma + f32fma");
    CASE(0, 3, false, 0, "f64mfma + ds_read_b64");
    CASE(0, 4, false, 0, "f64mfma + ds_write_b128");
    CASE(0, 5, false, 0, "f64mfma + global_load_dwordx4");
    CASE(0, 6, false, 0, "f64mfma + global_load_lds_dwordx4");
    CASE(1, 3, false, 0, "f32mfma + ds_read_b64");
    CASE(1, 5, false, 0, "f32mfma + global_load_dwordx4");
    CASE(1, 6, false, 0, "f32mfma + global_load_lds_dwordx4");
    (void)hipFree(dout);
    (void)hipFree(gb);
    return 0;
}
