// sksy.hip -- util::require_symmetric on the device (RandBLAS/util.hh:165-188), the O(n^2) serial
// check that sketch_symmetric runs before sketch_general (sksy.hh:165-537).
//
// One workgroup compares a 64 x 64 tile of the strict upper block triangle with its mirror: the
// mirror tile is read coalesced and transposed through LDS, so A is read once at streaming rate.
// The predicate is the reference's, in the operand precision T:
//   viol = |A(i,j) - A(j,i)| > (|A(i,j)| + |A(j,i)| + 1) * tol.
#include "saso.hpp"

namespace rbh {

template <typename T>
__global__ __launch_bounds__(256) void symcheck_kernel(int64_t n, const T *A, int64_t irs, int64_t ics, T tol,
                                                       int *flag) {
    __shared__ T mir[64][65];
    // blockIdx.x enumerates tile pairs (bi <= bj) row by row of the upper block triangle
    const int64_t nt = (n + 63) / 64;
    int64_t b = blockIdx.x, bi = 0;
    while (b >= nt - bi) { b -= nt - bi; ++bi; }
    const int64_t bj = bi + b;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
    // mirror tile: A(bj*64 + r, bi*64 + c), stored transposed as mir[c][r]
    for (int rr = ty; rr < 64; rr += 4) {
        // coalesce along whichever index is contiguous
        int64_t gi, gj;
        int lr, lc;
        if (irs == 1) { gi = bj * 64 + tx; gj = bi * 64 + rr; lr = tx; lc = rr; }
        else { gi = bj * 64 + rr; gj = bi * 64 + tx; lr = rr; lc = tx; }
        mir[lc][lr] = (gi < n && gj < n) ? A[gi * irs + gj * ics] : (T)0;
    }
    __syncthreads();
    bool bad = false;
    for (int rr = ty; rr < 64; rr += 4) {
        int64_t gi, gj;
        int lr, lc;
        if (irs == 1) { gi = bi * 64 + tx; gj = bj * 64 + rr; lr = tx; lc = rr; }
        else { gi = bi * 64 + rr; gj = bj * 64 + tx; lr = rr; lc = tx; }
        if (gi < n && gj < n && gi < gj) {
            const T aij = A[gi * irs + gj * ics];
            const T aji = mir[lr][lc];   // A(gj, gi)
            const T d = aij - aji;
            const T viol = d < (T)0 ? -d : d;
            const T rel = ((aij < (T)0 ? -aij : aij) + (aji < (T)0 ? -aji : aji) + (T)1) * tol;
            if (viol > rel) bad = true;
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

template <typename T>
static hipError_t launch_sym(char layout, const T *A, int64_t n, int64_t lda, T tol, int *flag, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const int64_t nt = (n + 63) / 64;
    const int64_t pairs = nt * (nt + 1) / 2;
    const int64_t irs = layout == 'C' ? 1 : lda, ics = layout == 'C' ? lda : 1;
    hipLaunchKernelGGL(symcheck_kernel<T>, dim3((unsigned)pairs), dim3(256), 0, s, n, A, irs, ics, tol, flag);
    return hipGetLastError();
}

hipError_t launch_symcheck_f64(char layout, const double *A, int64_t n, int64_t lda, double tol, int *flag,
                               hipStream_t s) {
    return launch_sym<double>(layout, A, n, lda, tol, flag, s);
}
hipError_t launch_symcheck_f32(char layout, const float *A, int64_t n, int64_t lda, float tol, int *flag,
                               hipStream_t s) {
    return launch_sym<float>(layout, A, n, lda, tol, flag, s);
}

}  // namespace rbh
