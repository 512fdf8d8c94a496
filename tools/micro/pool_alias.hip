// pool_alias.hip -- after a stream-ordered pool trims (release threshold 0), can a later pool
// allocation overlap memory that hipMalloc handed out in between? The check is on the host (the
// address ranges of live allocations); no kernel touches memory after a trim, so a positive finding
// cannot fault the device.
//
// Per iteration: pool block W (touched by a kernel, freed, synchronised: the pool trims), then six
// hipMalloc staging buffers (as the library stages host A, B, rows, cols, vals), then pool blocks
// of the library's workspace sizes; every live range is compared with every other.
// Build: hipcc --offload-arch=gfx950 -O2 pool_alias.hip -o pool_alias ; run: ./pool_alias [iters] [keep]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorName(e_), __LINE__); exit(2); } } while (0)

__global__ void touch(uint32_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (uint32_t)i;
}

struct Rng { uintptr_t lo, hi; const char *what; };

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    const uint64_t keep = argc > 2 ? strtoull(argv[2], nullptr, 10) : 0;
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
    hipStream_t s = 0;
    long overlaps = 0, checks = 0;
    for (int it = 0; it < iters; ++it) {
        void *w;
        const size_t wb = (size_t)(64 + 64 * (it % 5)) << 10;
        CK(hipMallocFromPoolAsync(&w, wb, pool, s));
        hipLaunchKernelGGL(touch, dim3(64), dim3(256), 0, s, (uint32_t *)w, wb / 4);
        CK(hipFreeAsync(w, s));
        CK(hipStreamSynchronize(s));   // the pool trims here when keep == 0
        std::vector<Rng> live;
        std::vector<void *> stg;
        const size_t sizes[6] = {(size_t)8 * 201 * 6 + 64 * it, (size_t)8 * 17 * 6, 8 * 450, 8 * 450, 8 * 450, 4096};
        for (int q = 0; q < 6; ++q) {
            void *x;
            CK(hipMalloc(&x, sizes[q]));
            stg.push_back(x);
            live.push_back({(uintptr_t)x, (uintptr_t)x + sizes[q], "hipMalloc"});
        }
        std::vector<void *> pb;
        const size_t psizes[3] = {(size_t)16 << 10, (size_t)300 << 10, 1 << 20};
        for (int q = 0; q < 3; ++q) {
            void *y;
            CK(hipMallocFromPoolAsync(&y, psizes[q], pool, s));
            pb.push_back(y);
            live.push_back({(uintptr_t)y, (uintptr_t)y + psizes[q], "pool"});
        }
        for (size_t a = 0; a < live.size(); ++a)
            for (size_t b = a + 1; b < live.size(); ++b) {
                ++checks;
                if (live[a].lo < live[b].hi && live[b].lo < live[a].hi) {
                    if (overlaps < 10)
                        printf("iteration %d: %s [%#lx, %#lx) overlaps %s [%#lx, %#lx)\n", it, live[a].what,
                               (unsigned long)live[a].lo, (unsigned long)live[a].hi, live[b].what,
                               (unsigned long)live[b].lo, (unsigned long)live[b].hi);
                    ++overlaps;
                }
            }
        for (void *y : pb) CK(hipFreeAsync(y, s));
        CK(hipStreamSynchronize(s));
        for (void *x : stg) CK(hipFree(x));
    }
    printf("keep=%llu: %ld overlapping pairs of live allocations in %ld checks over %d iterations\n",
           (unsigned long long)keep, overlaps, checks, iters);
    CK(hipMemPoolDestroy(pool));
    return overlaps ? 1 : 0;
}
