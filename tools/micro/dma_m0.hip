// LDS-DMA reach check: global_load_lds_dword to LDS offsets past 64 KB (M0 = byte address).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
template <int CLOBBER>
__global__ __launch_bounds__(64) void k(const unsigned *g, unsigned *out, const unsigned *offs, int noff) {
    __shared__ unsigned s[40960];   // 160 KB
    for (int i = threadIdx.x; i < 40960; i += 64) s[i] = 0xdeadbeefu;
    __syncthreads();
    const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)s;
    for (int o = 0; o < noff; ++o) {
        const unsigned m0 = __builtin_amdgcn_readfirstlane(base + offs[o]);
        const unsigned *src = g + 64 * o + threadIdx.x;
        asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" :: "s"(m0), "v"(src) : "memory", "m0");
        if (CLOBBER == 1) asm volatile("s_mov_b32 m0, 0x2000" ::: "m0");
        if (CLOBBER == 2) asm volatile("s_set_gpr_idx_on %0, gpr_idx(SRC0,DST)\n\ts_set_gpr_idx_off" :: "s"(37) : "m0");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 40960; i += 64) out[i] = s[i];
}
int main() {
    std::vector<unsigned> offs = {0, 4096, 65536, 65536 + 4096, 131072, 147456, 160000};
    int n = offs.size();
    std::vector<unsigned> g(64 * n);
    for (int i = 0; i < 64 * n; ++i) g[i] = 1000000u * (i / 64 + 1) + (i % 64);
    unsigned *dg, *dout, *doff;
    hipMalloc(&dg, g.size() * 4); hipMalloc(&dout, 40960 * 4); hipMalloc(&doff, n * 4);
    hipMemcpy(dg, g.data(), g.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(doff, offs.data(), n * 4, hipMemcpyHostToDevice);
  for (int variant = 0; variant < 3; ++variant) {
    printf("variant %d (0: none, 1: s_mov m0 after issue, 2: s_set_gpr_idx_on after issue)\n", variant);
    hipMemset(dout, 0, 40960 * 4);
    if (variant == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, dg, dout, doff, n);
    if (variant == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, dg, dout, doff, n);
    if (variant == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, dg, dout, doff, n);
    std::vector<unsigned> out(40960);
    if (hipMemcpy(out.data(), dout, 40960 * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
    for (int o = 0; o < n; ++o) {
        unsigned idx = offs[o] / 4;
        bool ok = true;
        for (int l = 0; l < 64; ++l) ok &= out[idx + l] == g[64 * o + l];
        printf("offset %6u: %s (first word %u)\n", offs[o], ok ? "ok" : "WRONG", out[idx]);
    }
    // where did the data land?
    for (int i = 0; i < 40960; ++i)
        if (out[i] != 0xdeadbeefu && (i % 64 == 0)) printf("  word %d (byte %d) = %u\n", i, 4 * i, out[i]);
  }
    return 0;
}
