// LDS-DMA layout check for global_load_lds_dwordx4: where does dword c of lane l land?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(64) void k(const unsigned *g, unsigned *out) {
    __shared__ __attribute__((aligned(16))) unsigned s[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) s[i] = 0xffffffffu;
    __syncthreads();
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)s);
    const unsigned *src = g + 4 * threadIdx.x;   // lane l reads dwords 4l .. 4l+3
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" :: "s"(base), "v"(src) : "memory", "m0");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = s[i];
}
int main() {
    std::vector<unsigned> g(256);
    for (int i = 0; i < 256; ++i) g[i] = i;
    unsigned *dg, *dout;
    hipMalloc(&dg, 1024); hipMalloc(&dout, 4096);
    hipMemcpy(dg, g.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dg, dout);
    std::vector<unsigned> out(1024);
    hipMemcpy(out.data(), dout, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += out[i] != (unsigned)i;
    printf("contiguous lane*16 layout: %s (%d words differ)\n", bad ? "NO" : "yes", bad);
    for (int i = 0; i < 24; ++i) printf("%u ", out[i]);
    printf("\n");
    for (int i = 256; i < 264; ++i) printf("%u ", out[i]);
    printf("\n");
    return 0;
}
