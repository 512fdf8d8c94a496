// pool_live.hip -- does trimming a stream-ordered pool (release threshold 0: trim at every
// synchronisation) disturb a block that is still allocated, when a neighbouring block of the same
// pool was freed before the trim? (with threshold 0 and no workspace arena,
// the C++ client's sparse cases read B back as zeros -- their calls hold two or three workspaces
// at once, freed in between, and synchronise after each allocation.)
//
// Per iteration: A = alloc (live throughout), kernel writes A; B = alloc, C = alloc; free B;
// D = alloc + synchronise (the trim); kernel checks A; free A, C, D. Sizes are not page multiples
// so blocks share pages. Prints mismatching words of A per (threshold, size) case.
// Build: hipcc --offload-arch=gfx950 -O2 pool_live.hip -o pool_live ; run: ./pool_live [iters]
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
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != (tag ^ (uint32_t)(i * 2654435761u));
    if (b) atomicAdd(bad, b);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 100;
    int dev = 0;
    CK(hipGetDevice(&dev));
    unsigned long long *dbad;
    CK(hipMalloc((void **)&dbad, 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (uint64_t keep : {(uint64_t)0, (uint64_t)1 << 30}) {
        for (size_t abytes : {(size_t)100000, (size_t)3000000, (size_t)40000000}) {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            hipMemPool_t pool;
            CK(hipMemPoolCreate(&pool, &props));
            CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
            CK(hipMemsetAsync(dbad, 0, 8, s));
            for (int it = 0; it < iters; ++it) {
                const size_t a = abytes + 4 * (size_t)(it % 13), n = a / 4;
                uint32_t *A, *B, *C, *D;
                CK(hipMallocFromPoolAsync((void **)&A, a, pool, s));
                CK(hipStreamSynchronize(s));
                hipLaunchKernelGGL(writek, dim3(256), dim3(256), 0, s, A, n, (uint32_t)it * 7919u + 1);
                CK(hipMallocFromPoolAsync((void **)&B, a / 3 + 1000, pool, s));
                CK(hipStreamSynchronize(s));
                CK(hipMallocFromPoolAsync((void **)&C, a / 7 + 300, pool, s));
                CK(hipStreamSynchronize(s));
                CK(hipMemsetAsync(B, 0x5a, a / 3 + 1000, s));
                CK(hipFreeAsync(B, s));
                CK(hipMallocFromPoolAsync((void **)&D, a / 5 + 77, pool, s));
                CK(hipStreamSynchronize(s));   // threshold 0: the pool trims here
                CK(hipMemsetAsync(D, 0x33, a / 5 + 77, s));
                hipLaunchKernelGGL(readk, dim3(256), dim3(256), 0, s, A, n, (uint32_t)it * 7919u + 1, dbad);
                CK(hipFreeAsync(A, s));
                CK(hipFreeAsync(C, s));
                CK(hipFreeAsync(D, s));
                CK(hipStreamSynchronize(s));
            }
            // the library's no-arena sync mode: allocate + synchronise (trim), write, check, free
            // asynchronously, synchronise (trim) -- each allocation reuses the previous one's address
            for (int it = 0; it < iters; ++it) {
                const size_t a = abytes + 8 * (size_t)(it % 3), n = a / 4;
                uint32_t *P;
                CK(hipMallocFromPoolAsync((void **)&P, a, pool, s));
                CK(hipStreamSynchronize(s));
                hipLaunchKernelGGL(writek, dim3(256), dim3(256), 0, s, P, n, (uint32_t)it * 31u + 5);
                hipLaunchKernelGGL(readk, dim3(256), dim3(256), 0, s, P, n, (uint32_t)it * 31u + 5, dbad);
                CK(hipFreeAsync(P, s));
                CK(hipStreamSynchronize(s));
            }
            unsigned long long h = 0;
            CK(hipMemcpy(&h, dbad, 8, hipMemcpyDeviceToHost));
            // control: the same loop on hipMalloc / hipFree
            CK(hipMemsetAsync(dbad, 0, 8, s));
            for (int it = 0; it < iters; ++it) {
                const size_t a = abytes + 8 * (size_t)(it % 3), n = a / 4;
                uint32_t *P;
                CK(hipMalloc((void **)&P, a));
                hipLaunchKernelGGL(writek, dim3(256), dim3(256), 0, s, P, n, (uint32_t)it * 31u + 5);
                hipLaunchKernelGGL(readk, dim3(256), dim3(256), 0, s, P, n, (uint32_t)it * 31u + 5, dbad);
                CK(hipStreamSynchronize(s));
                CK(hipFree(P));
            }
            unsigned long long hc = 0;
            CK(hipMemcpy(&hc, dbad, 8, hipMemcpyDeviceToHost));
            printf("keep=%llu bytes=%zu: pool %llu bad words, hipMalloc control %llu, in %d iterations each\n",
                   (unsigned long long)keep, abytes, h, hc, iters);
            CK(hipMemPoolDestroy(pool));
        }
    }
    return 0;
}
