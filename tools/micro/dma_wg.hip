// LDS-DMA from a full 1024-thread workgroup with 145 KB of LDS: 16 waves x 8 dwordx4 copies
// (2 x 64 KB buffers), as in saso_dma_kernel, then a check of every word.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(1024) void k(const unsigned *g, unsigned *out) {
    __shared__ __attribute__((aligned(16))) unsigned s[148480 / 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < 148480 / 4; i += 1024) s[i] = 0xffffffffu;
    __syncthreads();
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)s);
    for (int b = 0; b < 2; ++b)
        for (int i = 0; i < 4; ++i) {
            const int inst = wave * 4 + i;
            const unsigned *src = g + (b * 64 + inst) * 256 + 4 * lane;
            asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" :: "s"(base + b * 65536 + inst * 1024), "v"(src) : "memory", "m0");
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = tid; i < 32768; i += 1024) out[i] = s[i];
}
int main() {
    std::vector<unsigned> g(32768);
    for (int i = 0; i < 32768; ++i) g[i] = i;
    unsigned *dg, *dout;
    hipMalloc(&dg, 32768 * 4); hipMalloc(&dout, 32768 * 4);
    hipMemcpy(dg, g.data(), 32768 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(64), dim3(1024), 0, 0, dg, dout);
    hipError_t e = hipDeviceSynchronize();
    std::vector<unsigned> out(32768);
    hipMemcpy(out.data(), dout, 32768 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32768; ++i) bad += out[i] != (unsigned)i;
    printf("sync: %s, %d of 32768 words wrong\n", hipGetErrorString(e), bad);
    return 0;
}
