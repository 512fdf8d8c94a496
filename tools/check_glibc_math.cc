// check_glibc_math.cc -- host equivalence check of rb::rb_sincosf / rb::rb_logf / rb::boxmuller
// (randblas_amd/csrc/rng_core.hpp) against the host libm that the reference calls
// (RandBLAS/random_gen.hh:62-65 -> sincosf; Random123 boxmuller -> logf, sqrtf).
//
// Usage: check_glibc_math <stride> [start]
//   Visits every stride-th 32-bit word w (from start) and compares, bit for bit,
//     sincosf(pi_f * uneg11(w))  and  logf(u01(w))  and  the Box-Muller pair of (w, w*2654435761).
// Prints "checked N mismatches_sin K mismatches_cos K mismatches_log K mismatches_bm K".
// stride 1 is the exhaustive run (about a minute on 8 cores).
#define _GNU_SOURCE 1
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "../randblas_amd/csrc/rng_core.hpp"

int main(int argc, char **argv) {
    uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4099;
    uint64_t start = argc > 2 ? strtoull(argv[2], nullptr, 10) : 0;
    if (stride == 0) stride = 1;
    unsigned long long n_checked = 0, bad_s = 0, bad_c = 0, bad_l = 0, bad_bm = 0;
    long long first_bad = -1;
    const float PIf = 3.1415926535897932f;
#pragma omp parallel for schedule(static) reduction(+ : n_checked, bad_s, bad_c, bad_l, bad_bm)
    for (int64_t w = (int64_t)start; w < (int64_t)1 << 32; w += (int64_t)stride) {
        uint32_t u = (uint32_t)w;
        float y = PIf * rb::uneg11f(u);
        float s_ref, c_ref;
        sincosf(y, &s_ref, &c_ref);
        float s, c;
        rb::rb_sincosf(y, s, c);
        float x = rb::u01f(u);
        float l_ref = logf(x);
        float l = rb::rb_logf(x);
        uint32_t u1 = u * 2654435761u;
        float g0, g1;
        rb::boxmuller(u, u1, g0, g1);
        float ss, cc;
        sincosf(PIf * rb::uneg11f(u), &ss, &cc);
        float rr = sqrtf(-2.0f * logf(rb::u01f(u1)));
        float h0 = ss * rr, h1 = cc * rr;
        n_checked += 1;
        if (rb::f32_bits(s) != rb::f32_bits(s_ref)) bad_s += 1;
        if (rb::f32_bits(c) != rb::f32_bits(c_ref)) bad_c += 1;
        if (rb::f32_bits(l) != rb::f32_bits(l_ref)) bad_l += 1;
        if (rb::f32_bits(g0) != rb::f32_bits(h0) || rb::f32_bits(g1) != rb::f32_bits(h1)) bad_bm += 1;
        if ((rb::f32_bits(s) != rb::f32_bits(s_ref) || rb::f32_bits(c) != rb::f32_bits(c_ref) ||
             rb::f32_bits(l) != rb::f32_bits(l_ref)) && first_bad < 0) {
#pragma omp critical
            { if (first_bad < 0) { first_bad = w;
                fprintf(stderr, "first mismatch w=%08x y=%a sin %a vs %a cos %a vs %a | x=%a log %a vs %a\n",
                        u, y, s, s_ref, c, c_ref, x, l, l_ref); } }
        }
    }
    printf("checked %llu mismatches_sin %llu mismatches_cos %llu mismatches_log %llu mismatches_bm %llu\n",
           n_checked, bad_s, bad_c, bad_l, bad_bm);
    return (bad_s || bad_c || bad_l || bad_bm) ? 1 : 0;
}
