// check_sqrt.hip -- rb::rb_sqrtf_bm (rng_core.hpp, device path) against the correctly rounded sqrt
// (float)sqrt((double)v) for every float v in [0, 64] and for -0. The Box-Muller radius argument
// -2 log(u01(w)) is -0 or lies in [2^-23, 46]; mismatches below 2^-23 are reported separately
// (unreachable). Exit code 0 iff the reachable range matches bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -o check_sqrt check_sqrt.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../randblas_amd/csrc/rng_core.hpp"

__global__ void check(uint32_t lo, uint32_t hi, unsigned long long *bad) {
    unsigned long long nb_reach = 0, nb_tiny = 0;
    for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= hi; b += (uint64_t)gridDim.x * blockDim.x) {
        const float v = rb::f32_from((uint32_t)b);
        const float got = rb::rb_sqrtf_bm(v);
        const float ref = (float)__builtin_sqrt((double)v);
        if (rb::f32_bits(got) != rb::f32_bits(ref)) {
            if (v >= 0x1p-23f) nb_reach++; else nb_tiny++;
        }
    }
    if (nb_reach) atomicAdd(&bad[0], nb_reach);
    if (nb_tiny) atomicAdd(&bad[1], nb_tiny);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const float z = rb::rb_sqrtf_bm(-0.0f);
        if (rb::f32_bits(z) != 0x80000000u) atomicAdd(&bad[0], 1ull);
    }
}

int main() {
    unsigned long long *d, h[2];
    (void)hipMalloc(&d, sizeof h);
    (void)hipMemset(d, 0, sizeof h);
    const uint32_t hi = rb::f32_bits(64.0f);
    hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, 0u, hi, d);
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("check_sqrt: %u floats in [0, 64] and -0: %llu mismatches at v >= 2^-23, %llu below (unreachable)\n",
           hi + 1, h[0], h[1]);
    return h[0] ? 1 : 0;
}
