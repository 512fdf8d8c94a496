// pool_grow.hip -- after a stream-ordered pool trims (release threshold 0), is every byte of the next,
// differently sized block backed? A kernel writes the whole block, a second kernel (blocks in reverse
// order) checks it; the block sizes rise and fall across trims, as the library's workspaces do
// from call to call. No copy engine touches pool memory (an unbacked range read through a kernel
// returns zeros instead of faulting). Prints the bad words and the first bad byte offset per size.
// Build: hipcc --offload-arch=gfx950 -O2 pool_grow.hip -o pool_grow ; run: ./pool_grow [keep]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorName(e_), __LINE__); exit(2); } } while (0)

__global__ void writek(uint32_t *p, size_t n, uint32_t tag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = tag ^ (uint32_t)(i * 2654435761u);
}
__global__ void readk(const uint32_t *p, size_t n, uint32_t tag, unsigned long long *res) {
    const size_t blk = gridDim.x - 1 - blockIdx.x;
    for (size_t i = blk * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != (tag ^ (uint32_t)(i * 2654435761u))) {
            atomicAdd(&res[0], 1ull);
            atomicMin(&res[1], (unsigned long long)i * 4);
        }
}

int main(int argc, char **argv) {
    const uint64_t keep = argc > 1 ? strtoull(argv[1], nullptr, 10) : 0;
    int dev = 0;
    CK(hipGetDevice(&dev));
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool;
    CK(hipMemPoolCreate(&pool, &props));
    uint64_t thr = keep;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
    unsigned long long *res;
    CK(hipMalloc((void **)&res, 16));
    const size_t sizes[] = {1000, 3000, 20000, 4100, 150000, 70000, 2000000, 300000, 9000000, 65536, 5000000, 12000,
                            33554432, 1000, 40000000, 2048};
    long total_bad = 0;
    for (int rep = 0; rep < 3; ++rep)
        for (size_t bytes : sizes) {
            const unsigned long long init[2] = {0ull, ~0ull};
            CK(hipMemcpy(res, init, 16, hipMemcpyHostToDevice));
            void *stg;
            CK(hipMalloc(&stg, 4096 + bytes / 3));   // a staging buffer between trims, as the library has
            uint32_t *p;
            CK(hipMallocFromPoolAsync((void **)&p, bytes, pool, 0));
            const size_t n = bytes / 4;
            hipLaunchKernelGGL(writek, dim3(256), dim3(256), 0, 0, p, n, (uint32_t)bytes);
            hipLaunchKernelGGL(readk, dim3(256), dim3(256), 0, 0, p, n, (uint32_t)bytes, res);
            CK(hipFreeAsync(p, 0));
            CK(hipStreamSynchronize(0));
            CK(hipFree(stg));
            unsigned long long h[2];
            CK(hipMemcpy(h, res, 16, hipMemcpyDeviceToHost));
            if (h[0]) printf("keep=%llu size %zu: %llu bad words, first bad byte %llu\n", (unsigned long long)keep,
                             bytes, h[0], h[1]);
            total_bad += (long)h[0];
        }
    printf("keep=%llu: %ld bad words over %d allocations\n", (unsigned long long)keep, total_bad,
           3 * (int)(sizeof(sizes) / sizeof(sizes[0])));
    return 0;
}
