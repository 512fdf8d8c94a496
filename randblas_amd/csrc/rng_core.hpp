// rng_core.hpp -- counter-based RNG arithmetic shared by the HIP kernels and host checks.
//
// This header is compiled twice: by hipcc for gfx950 device code (RB_HD = __host__ __device__)
// and by g++ for the host-side equivalence checks in tests/ (RB_HD empty). Everything here is
// integer or IEEE-754 arithmetic with explicitly placed fma() calls, so both builds produce the
// same bits.
//
// What is restated, and where it comes from:
//   * Philox4x32-10 (Random123, DEShawResearch; external dependency of RandBLAS, not vendored,
//     unpinned HEAD in the reference CI: .github/workflows/core-linux.yaml:34-39). Called by the
//     reference at RandBLAS/dense_skops.hh:142,155,161 and RandBLAS/sparse_skops.hh:78.
//     Pinned by the philox4x32 rows of test/test_basic_rng/r123_kat_vectors.txt:16-21.
//   * ctr_type::incr(u64): 128-bit little-endian add with carry (pinned by
//     test/test_basic_rng/test_r123.cc:679-766).
//   * r123::u01<float>, r123::uneg11<float> (Random123 uniform.hpp) and r123::boxmuller
//     (Random123 boxmuller.hpp) as composed by r123ext::boxmul / boxmulall
//     (RandBLAS/random_gen.hh:96-145) and r123ext::uneg11 (random_gen.hh:148-173).
//   * The reference evaluates boxmuller's sincosf/logf through the host libm (glibc 2.35 on this
//     image, random_gen.hh:62-65). glibc >= 2.28 implements both with the double-precision
//     table+polynomial algorithms of ARM's optimized-routines (sysdeps/ieee754/flt-32/s_sincosf.c,
//     e_logf.c), and on x86-64 CPUs with FMA dispatches to builds compiled with -mfma where the
//     compiler contracts a*b+c into fma. rb_sincosf/rb_logf below restate that arithmetic with
//     the fma placement of the -mfma build, so the device reproduces the reference's float
//     Gaussians bit for bit. tests/test_glibc_math.py checks this against the host libm.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RB_HD __host__ __device__ __forceinline__
#else
#define RB_HD static inline
#include <math.h>
#endif

namespace rb {

// ------------------------------------------------------------------------------------------
// Philox4x32-10
// ------------------------------------------------------------------------------------------
struct u32x4 { uint32_t v[4]; };

constexpr uint32_t PHILOX_M0 = 0xD2511F53u;
constexpr uint32_t PHILOX_M1 = 0xCD9E8D57u;
constexpr uint32_t PHILOX_W0 = 0x9E3779B9u;
constexpr uint32_t PHILOX_W1 = 0xBB67AE85u;

RB_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t &hi, uint32_t &lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
}

// R rounds of Philox4x32 on counter (c0..c3) with key (k0,k1). Random123's round function:
// (hi0,lo0) = M0*c0, (hi1,lo1) = M1*c2, c' = {hi1^c1^k0, lo1, hi0^c3^k1, lo0}; the key is
// bumped by the Weyl constants between rounds.
template <int R = 10>
RB_HD u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r > 0) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo32(PHILOX_M0, c0, hi0, lo0);
        mulhilo32(PHILOX_M1, c2, hi1, lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    u32x4 out = {{c0, c1, c2, c3}};
    return out;
}

#if defined(__HIPCC__)
// a ^ b ^ k in one v_bitop3_b32 (gfx950 has no v_xor3) with the key word k in an SGPR. For
// wave-uniform k only: every Philox key of the library comes from a kernel argument.
__device__ __forceinline__ uint32_t xor3_uk(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
#endif

// philox4x32 with a wave-uniform key: the same words, the round's two three-way xors as one
// instruction each on the device (the dense draws, where every Philox call is on the critical
// issue path beside the MFMAs).
template <int R = 10>
RB_HD u32x4 philox4x32_uk(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r > 0) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo32(PHILOX_M0, c0, hi0, lo0);
        mulhilo32(PHILOX_M1, c2, hi1, lo1);
        const uint32_t n0 = xor3_uk(hi1, c1, k0);
        const uint32_t n2 = xor3_uk(hi0, c3, k1);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    u32x4 out = {{c0, c1, c2, c3}};
    return out;
#else
    return philox4x32<R>(c0, c1, c2, c3, k0, k1);
#endif
}

// Random123 Threefry4x32-R (threefry.h), RandBLAS's other counter-based generator
// (RNGState<r123::Threefry4x32>, base.hh:159; Random123's default R = 20): key schedule
// ks[4] = 0x1BD11BDA ^ k0 ^ k1 ^ k2 ^ k3, the key added before round 0 and after every 4th round
// (injection s: x_i += ks[(s + i) % 5], x3 += s); even rounds mix (x0, x1), (x2, x3), odd rounds
// (x0, x3), (x2, x1), with the rotations R_32x4[r % 8]. Pinned by the reference's KAT rows
// (tests/golden/threefry4x32_kat.txt).
RB_HD uint32_t rotl32(uint32_t x, unsigned r) { return (x << r) | (x >> (32u - r)); }
template <int R = 20>
RB_HD u32x4 threefry4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t k2,
                         uint32_t k3) {
    const uint32_t ks[5] = {k0, k1, k2, k3, 0x1BD11BDAu ^ k0 ^ k1 ^ k2 ^ k3};
    uint32_t x0 = c0 + k0, x1 = c1 + k1, x2 = c2 + k2, x3 = c3 + k3;
    constexpr unsigned ROT[8][2] = {{10, 26}, {11, 21}, {13, 27}, {23, 5}, {6, 20}, {17, 11}, {25, 10}, {18, 20}};
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int r = 0; r < R; ++r) {
        if (r % 2 == 0) {
            x0 += x1; x1 = rotl32(x1, ROT[r % 8][0]) ^ x0;
            x2 += x3; x3 = rotl32(x3, ROT[r % 8][1]) ^ x2;
        } else {
            x0 += x3; x3 = rotl32(x3, ROT[r % 8][0]) ^ x0;
            x2 += x1; x1 = rotl32(x1, ROT[r % 8][1]) ^ x2;
        }
        if (r % 4 == 3) {
            const uint32_t s = (uint32_t)((r + 1) / 4);
            x0 += ks[s % 5]; x1 += ks[(s + 1) % 5]; x2 += ks[(s + 2) % 5]; x3 += ks[(s + 3) % 5] + s;
        }
    }
    u32x4 out = {{x0, x1, x2, x3}};
    return out;
}

// The operators' generator (RNGState<RNG>): rng 0 Philox4x32-10 (key[0..1]), 1 Threefry4x32-20
// (key[0..3]). The streamed / tiled GEMM kernels call Philox directly; a Threefry operator reaches
// them only as a window drawn by this one (fill_dense) into a workspace.
constexpr int RNG_PHILOX = 0, RNG_THREEFRY = 1;
struct CbKey { uint32_t k[4]; int rng; };   // a generator's key and kind, as one kernel argument
RB_HD u32x4 cbrng(int rng, const uint32_t c[4], const uint32_t k[4]) {
    if (rng == RNG_THREEFRY) return threefry4x32<20>(c[0], c[1], c[2], c[3], k[0], k[1], k[2], k[3]);
    return philox4x32_uk<10>(c[0], c[1], c[2], c[3], k[0], k[1]);
}

// 128-bit counter = base (4 x u32, little-endian words) + off (u64), carries across words.
RB_HD void ctr_add(const uint32_t base[4], uint64_t off, uint32_t out[4]) {
    uint64_t lo = (uint64_t)base[0] + (uint32_t)off;
    out[0] = (uint32_t)lo;
    uint64_t mid = (uint64_t)base[1] + (uint32_t)(off >> 32) + (lo >> 32);
    out[1] = (uint32_t)mid;
    uint64_t w2 = (uint64_t)base[2] + (mid >> 32);
    out[2] = (uint32_t)w2;
    out[3] = base[3] + (uint32_t)(w2 >> 32);
}

// ------------------------------------------------------------------------------------------
// Random123 uniform transforms (float flavour).
//   u01<float>(u)    = float(u) * 2^-32 + 2^-33    (u as uint32)
//   uneg11<float>(u) = float(int32(u)) * 2^-31 + 2^-32
// The products are exact (power-of-two scaling), so fma contraction cannot change them.
// ------------------------------------------------------------------------------------------
RB_HD float u01f(uint32_t u) {
    const float factor = 2.3283064365386963e-10f;       // 2^-32
    const float half   = 1.1641532182693481e-10f;       // 2^-33
    return (float)u * factor + half;
}
RB_HD float uneg11f(uint32_t u) {
    const float factor = 4.6566128730773926e-10f;       // 2^-31
    const float half   = 2.3283064365386963e-10f;       // 2^-32
    return (float)(int32_t)u * factor + half;
}

// ------------------------------------------------------------------------------------------
// glibc-equivalent sincosf / logf (double-precision evaluation, fma placement of the -mfma build)
// ------------------------------------------------------------------------------------------
RB_HD uint32_t f32_bits(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
RB_HD float f32_from(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }
// x with its sign bit xor-ed by `sign` (0 or 0x80000000): x * -1.0 exactly when sign is set
RB_HD double f64_xor_sign(double x, uint32_t sign) {
    union { double d; uint64_t u; } c;
    c.d = x;
    c.u ^= (uint64_t)sign << 32;
    return c.d;
}

#if defined(__HIPCC__)
#define RB_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#define RB_FMA(a, b, c) fma((a), (b), (c))
#endif

// Polynomial coefficients of the sincosf kernel (glibc __sincosf_table[0]). Table [1], used for
// quadrants with n & 2, negates c0..c4; every cosine-polynomial step is an fma whose operands all
// flip sign with them, so that result is exactly the negation of the table-[0] result.
constexpr double SC_HPI_INV = 0x1.45F306DC9C883p+23;   // 2/pi * 2^24
constexpr double SC_HPI     = 0x1.921FB54442D18p0;     // pi/2
constexpr double SC_C0 = 0x1p0;
constexpr double SC_C1 = -0x1.ffffffd0c621cp-2;
constexpr double SC_C2 = 0x1.55553e1068f19p-5;
constexpr double SC_C3 = -0x1.6c087e89a359dp-10;
constexpr double SC_C4 = 0x1.99343027bf8c3p-16;
constexpr double SC_S1 = -0x1.555545995a603p-3;
constexpr double SC_S2 =  0x1.1107605230bc4p-7;
constexpr double SC_S3 = -0x1.994eb3774cf24p-13;

// sin(y), cos(y) for the Box-Muller arguments y = pi_f * uneg11(w), |y| < pi. The small-argument
// branch of glibc (|y| < pi/4, no reduction) is the n == 0 case of the reduced path bit for bit
// (n == 0 makes the reduction x - 0*hpi == x and the sign factor 1), so one branch-free path
// serves both. glibc's tiny branch (|y| < 2^-12: sin = y, cos = 1) needs no select either: there the
// polynomial rounds to y and to 1 (x^2 / 6 and x^2 / 2 are below a quarter ulp). Both facts are
// checked against glibc for all 2^32 words w (tools/check_glibc_math.cc).
RB_HD void rb_sincosf(float y, float &sin_out, float &cos_out) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const double xd = (double)y;
    const double r = xd * SC_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double x = RB_FMA(-(double)n, SC_HPI, xd);
    // xs = x * sign[n & 3], sign = {1, -1, -1, 1}; the signs below are applied as bit operations
    // (the same values: multiplying by -1 only flips the sign bit), which keeps the draw free of
    // compare-and-select pairs
    const double xs = f64_xor_sign(x, ((uint32_t)(n + 1) & 2u) << 30);
    const double x2 = x * x;
    // sincosf_poly(xs, x2, ...)
    const double x4 = x2 * x2;
    const double x3 = x2 * xs;
    const double cc2 = RB_FMA(x2, SC_C4, SC_C3);
    const double ss1 = RB_FMA(x2, SC_S3, SC_S2);
    const double cc1 = RB_FMA(x2, SC_C1, SC_C0);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = RB_FMA(x3, SC_S1, xs);
    const double c = RB_FMA(x4, SC_C2, cc1);
    const float ps = (float)RB_FMA(x5, ss1, s);
    const float pc0 = (float)RB_FMA(x6, cc2, c);
    const uint32_t pcb = f32_bits(pc0) ^ (((uint32_t)n & 2u) << 30);   // (n & 2) ? -pc0 : pc0
    const uint32_t psb = f32_bits(ps);
    const uint32_t odd = 0u - ((uint32_t)n & 1u);                       // all ones for odd n
    sin_out = f32_from((pcb & odd) | (psb & ~odd));
    cos_out = f32_from((psb & odd) | (pcb & ~odd));
}

// logf for normal positive finite x (the Box-Muller radius argument is u01 in [2^-33, 1]; all 2^32
// of them are checked against glibc by tools/check_glibc_math.cc).
constexpr double LOGF_LN2 = 0x1.62e42fefa39efp-1;
constexpr double LOGF_A0 = -0x1.00ea348b88334p-2;
constexpr double LOGF_A1 =  0x1.5575b0be00b6ap-2;
constexpr double LOGF_A2 = -0x1.ffffef20a4123p-2;

// 16 subintervals of [OFF, 2*OFF); c near the centre of each, invc = 1/c, logc = log(c).
// A constexpr table: device code indexes it from the read-only global segment (one 16-B load per
// lane), which keeps the 32 constants out of the register file.
struct LogfEntry { double invc, logc; };
constexpr LogfEntry LOGF_TAB[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};

// tab: LOGF_TAB or a copy of it (the fused GEMM keeps one in LDS, away from the vector-memory
// counter its operand prefetch waits on).
RB_HD float rb_logf_tab(float xf, const LogfEntry *tab) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const uint32_t ix = f32_bits(xf);
    const uint32_t OFF = 0x3f330000u;
    const uint32_t tmp = ix - OFF;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double invc = tab[i].invc;
    const double logc = tab[i].logc;
    const double z = (double)f32_from(iz);
    const double r = RB_FMA(z, invc, -1.0);
    const double y0 = RB_FMA((double)k, LOGF_LN2, logc);
    const double r2 = r * r;
    double y = RB_FMA(LOGF_A1, r, LOGF_A2);
    y = RB_FMA(LOGF_A0, r2, y);
    y = RB_FMA(y, r2, y0 + r);
    return (float)y;   // (x = 1 needs no special case: table entry 9 is {1, 0}, so r = 0 and y = 0)
}
RB_HD float rb_logf(float xf) { return rb_logf_tab(xf, LOGF_TAB); }

// Correctly rounded float sqrt. Host: via double (double rounding is innocuous for sqrt at
// p = 53). Device: the compiler's correctly rounded f32 sqrt (HIP's default
// -fhip-fp32-correctly-rounded-divide-sqrt: v_sqrt_f32 and an fma residual fix-up, about half the
// issue cycles of the f64 sequence) -- the same bits, as any two correctly rounded results are.
RB_HD float rb_sqrtf(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_sqrtf(v);
#else
    return (float)sqrt((double)v);
#endif
}

// The Box-Muller radius sqrt(-2 log u) for u = u01(w): its argument is -0 (u = 1) or in
// [2^-23, 46]. On the device: v_sqrt_f32 (within 1 ulp) and the residual fix-up of the compiler's
// correctly rounded sqrtf, without that sequence's scaling for tiny inputs and its special-value
// cases, none of which the argument reaches (-0 passes through the fix-up unchanged: its lower
// neighbour is a NaN, its upper one gives a zero residual). tools/micro/check_sqrt.hip checks it
// against the correctly rounded sqrt for every float in [0, 64] and -0.
RB_HD float rb_sqrtf_bm(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float s = __builtin_amdgcn_sqrtf(v);
    const float sd = f32_from(f32_bits(s) - 1u), su = f32_from(f32_bits(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, v), ru = __builtin_fmaf(-su, s, v);
    const float t = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : t;
#else
    return (float)sqrt((double)v);
#endif
}

// r123::boxmuller(u0, u1) -> {r*sin(pi*x), r*cos(pi*x)}, x = uneg11(u0), r = sqrt(-2 log u01(u1)).
RB_HD void boxmuller(uint32_t u0, uint32_t u1, float &g0, float &g1, const LogfEntry *tab = LOGF_TAB) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const float PIf = 3.1415926535897932f;
    float s, c;
    rb_sincosf(PIf * uneg11f(u0), s, c);
    const float r = rb_sqrtf_bm(-2.0f * rb_logf_tab(u01f(u1), tab));
    g0 = s * r;
    g1 = c * r;
}

// Distribution families (DenseDistName, RandBLAS/dense_skops.hh:204-218)
enum Family : int { GAUSSIAN = 0, UNIFORM = 1 };

// The four float samples of one Philox call (r123ext::boxmul / r123ext::uneg11 generate()).
template <int FAMILY>
RB_HD void sample4(const u32x4 &w, float out[4], const LogfEntry *tab = LOGF_TAB) {
    if (FAMILY == GAUSSIAN) {
        boxmuller(w.v[0], w.v[1], out[0], out[1], tab);
        boxmuller(w.v[2], w.v[3], out[2], out[3], tab);
    } else {
        out[0] = uneg11f(w.v[0]); out[1] = uneg11f(w.v[1]);
        out[2] = uneg11f(w.v[2]); out[3] = uneg11f(w.v[3]);
    }
}

} // namespace rb
