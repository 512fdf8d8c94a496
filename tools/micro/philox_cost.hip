// philox_cost.hip -- microbenchmark: cost of Philox4x32-10 variants next to f64 MFMA waves (gfx950).
// Waves 0-3 issue f64 MFMA chains, waves 4-7 run Philox; reports the MFMA rate and Philox calls/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int IMPL>
__device__ __forceinline__ void mulhilo(uint32_t a, uint32_t m, uint32_t &hi, uint32_t &lo) {
    if (IMPL == 0) {   // 64-bit product (v_mad_u64_u32)
        uint64_t p = (uint64_t)a * m; hi = (uint32_t)(p >> 32); lo = (uint32_t)p;
    } else if (IMPL == 1) {   // separate hi / lo
        hi = __umulhi(a, m); lo = a * m;
    } else {   // 16-bit halves on the 24-bit multiplier
        const uint32_t a0 = a & 0xffff, a1 = a >> 16, m0 = m & 0xffff, m1 = m >> 16;
        uint32_t q00 = a0 * m0, q01 = a0 * m1, q10 = a1 * m0, q11 = a1 * m1;
        uint32_t mid = q01 + q10;                    // may carry out of 32 bits
        uint32_t midc = (mid < q01) ? 0x10000u : 0u;
        lo = q00 + (mid << 16);
        uint32_t c = (lo < q00) ? 1u : 0u;
        hi = q11 + (mid >> 16) + midc + c;
    }
}

template <int IMPL>
__device__ __forceinline__ void philox(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo<IMPL>(c0, 0xD2511F53u, hi0, lo0);
        mulhilo<IMPL>(c2, 0xCD9E8D57u, hi1, lo1);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
}

template <int IMPL, bool MF>
__global__ __launch_bounds__(512) void k(int iters, int calls, double *out, uint32_t *uout) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    v4d acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = (v4d){0, 0, 0, 0};
    uint32_t c0 = lane, c1 = blockIdx.x, c2 = 7, c3 = 9, x = 0;
    if (wave < 4) {
        if (MF)
            for (int it = 0; it < iters; ++it)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    } else {
        for (int it = 0; it < calls; ++it) {
            uint32_t d0 = c0 + it, d1 = c1, d2 = c2, d3 = c3;
            philox<IMPL>(d0, d1, d2, d3, 0x1234u, 0x5678u);
            x ^= d0 ^ d1 ^ d2 ^ d3;
        }
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
    uout[blockIdx.x * 512 + threadIdx.x] = x;
}

template <int IMPL, bool MF>
static void run(const char *name, int iters, int calls, double *out, uint32_t *uout) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<IMPL, MF><<<256, 512>>>(iters, calls, out, uout);
    (void)hipEventRecord(e0);
    k<IMPL, MF><<<256, 512>>>(iters, calls, out, uout);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double cyc_per_call = ms * 1e-3 * 2.4e9 / calls;   // per philox wave-call on one SIMD
    printf("%-40s %8.3f ms   %.0f cycles per philox wave-call (one wave per SIMD)\n", name, ms, cyc_per_call);
}

int main() {
    double *out; uint32_t *uout;
    (void)hipMalloc(&out, 256 * 512 * sizeof(double));
    (void)hipMalloc(&uout, 256 * 512 * sizeof(uint32_t));
    const int calls = 20000;
    run<0, false>("mad_u64 philox alone", 0, calls, out, uout);
    run<1, false>("mul_hi+mul_lo philox alone", 0, calls, out, uout);
    run<2, false>("16-bit split philox alone", 0, calls, out, uout);
    run<0, true>("mad_u64 philox + MFMA waves", 4000, calls, out, uout);
    run<1, true>("mul_hi+lo philox + MFMA waves", 4000, calls, out, uout);
    run<2, true>("16-bit split philox + MFMA waves", 4000, calls, out, uout);
    return 0;
}
