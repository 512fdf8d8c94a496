// pool_trim.hip -- does a stream-ordered pool that trims at every synchronisation hand back blocks
// whose contents a second kernel cannot see? (Diagnostic for DESIGN.md §7: the sparse apply read a
// kernel-written value back as zero when its workspace came from a pool with release threshold 0.)
//
// Each iteration: allocate from the pool, kernel W writes a pattern over the block, kernel R (a
// grid spread over every XCD) checks it, free, synchronise (the pool trims its memory here when
// the threshold is 0). Interleaved hipMalloc/hipFree of a staging buffer mimics the library's host
// staging. Prints the number of mismatching words per mode.
// Build: hipcc --offload-arch=gfx950 -O2 pool_trim.hip -o pool_trim ; run: ./pool_trim [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorName(e_), __LINE__); exit(2); } } while (0)

__global__ void writek(uint32_t *p, size_t n, uint32_t tag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = tag ^ (uint32_t)(i * 2654435761u);
}
__global__ void readk(const uint32_t *p, size_t n, uint32_t tag, unsigned long long *bad) {
    unsigned long long b = 0;
    // reverse block order, so a word is read by a different XCD than the one that wrote it
    const size_t blk = gridDim.x - 1 - blockIdx.x;
    for (size_t i = blk * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != (tag ^ (uint32_t)(i * 2654435761u));
    if (b) atomicAdd(bad, b);
}

static unsigned long long run(hipMemPool_t pool, bool use_pool, hipStream_t s, int iters, size_t bytes, bool stage,
                              unsigned long long *dbad) {
    CK(hipMemsetAsync(dbad, 0, 8, s));
    const size_t n = bytes / 4;
    for (int it = 0; it < iters; ++it) {
        void *stg = nullptr;
        if (stage) CK(hipMalloc(&stg, bytes / 2 + 4096 * (it % 7)));
        uint32_t *p;
        if (use_pool) CK(hipMallocFromPoolAsync((void **)&p, bytes + 256 * (it % 5), pool, s));
        else CK(hipMallocAsync((void **)&p, bytes + 256 * (it % 5), s));
        hipLaunchKernelGGL(writek, dim3(512), dim3(256), 0, s, p, n, (uint32_t)it * 7919u + 1);
        hipLaunchKernelGGL(readk, dim3(512), dim3(256), 0, s, p, n, (uint32_t)it * 7919u + 1, dbad);
        CK(hipFreeAsync(p, s));
        CK(hipStreamSynchronize(s));
        if (stg) CK(hipFree(stg));
    }
    unsigned long long h = 0;
    CK(hipMemcpy(&h, dbad, 8, hipMemcpyDeviceToHost));
    return h;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    int dev = 0;
    CK(hipGetDevice(&dev));
    unsigned long long *dbad;
    CK(hipMalloc((void **)&dbad, 8));
    hipStream_t own;
    CK(hipStreamCreate(&own));
    for (int stream_kind = 0; stream_kind < 2; ++stream_kind) {
        hipStream_t s = stream_kind ? own : (hipStream_t)0;
        for (uint64_t keep : {(uint64_t)0, (uint64_t)1 << 30}) {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            hipMemPool_t pool;
            CK(hipMemPoolCreate(&pool, &props));
            CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
            for (size_t bytes : {(size_t)64 << 10, (size_t)4 << 20, (size_t)64 << 20}) {
                for (int stage = 0; stage < 2; ++stage) {
                    const unsigned long long bad = run(pool, true, s, iters, bytes, stage, dbad);
                    printf("private pool keep=%llu stream=%s bytes=%zu staging=%d: %llu bad words in %d iterations\n",
                           (unsigned long long)keep, stream_kind ? "own" : "null", bytes, stage, bad, iters);
                }
            }
            CK(hipMemPoolDestroy(pool));
        }
        // the device's default pool at its default threshold (0)
        for (int stage = 0; stage < 2; ++stage) {
            const unsigned long long bad = run(nullptr, false, s, iters, (size_t)4 << 20, stage, dbad);
            printf("default pool stream=%s bytes=4MiB staging=%d: %llu bad words in %d iterations\n",
                   stream_kind ? "own" : "null", stage, bad, iters);
        }
    }
    return 0;
}
