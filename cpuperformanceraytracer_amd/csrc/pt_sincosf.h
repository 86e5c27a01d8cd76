// pt_sincosf.h -- sinf/cosf on the GPU, bit-identical to the host libm the reference calls.
//
// RandomUnitVector (demofox_path_tracing_scalar.cpp:42-50) evaluates cos(a) and sin(a) on an f32
// a in [0, 2*pi].  Under MSVC -- the reference's platform -- those unqualified calls resolve to
// the float overloads (cosf/sinf); with the image's glibc 2.35 they are glibc's sinf/cosf, whose
// algorithm evaluates in double: a Cody-Waite-free "fast" reduction by pi/2 (exact enough below
// 120) and two short double polynomials, rounded once to f32.  Every double op below is IEEE
// (mul/fma) on both x86-64 and gfx950, so reproducing the same ops with the same constants and
// the same fused multiply-adds gives the same f32, bit for bit.  This replaces OCML's sinf/cosf,
// whose results differ by an ulp on a fraction of inputs and would flip hit/miss decisions.
//
// Verified exhaustively on every f32 in [0, 2*pi*1.0001] against the host libm in
// tests/test_sincosf.py (tests/native/check_sincosf.cpp compiles THIS header for the host).
// Domain: |y| < 120, y != -0 (the reference's argument never leaves [+0, 2*pi]; larger |y| is
// excluded by the caller's construction, not handled here, and for -0 glibc's sinf returns -0,
// the straight-line form below +0).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PT_HD __host__ __device__ __forceinline__
#else
#define PT_HD static inline
#include <math.h>
#endif

namespace pt {

// glibc 2.35 __sincosf_table[0] (sysdeps/ieee754/flt-32), read from the image's libm.so.6:
//   hpi_inv = 2/pi * 2^24, hpi = pi/2, cosine c0..c4, sine s1..s3.  Table [1] differs only in the
//   sign of c0..c4, i.e. cos_poly_T1 == -cos_poly_T0 exactly (round-to-nearest is sign-symmetric).
constexpr double kHpiInv = 0x1.45f306dc9c883p+23;
constexpr double kHpi = 0x1.921fb54442d18p+0;
constexpr double kC0 = 0x1p0;
constexpr double kC1 = -0x1.ffffffd0c621cp-2;
constexpr double kC2 = 0x1.55553e1068f19p-5;
constexpr double kC3 = -0x1.6c087e89a359dp-10;
constexpr double kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3;
constexpr double kS2 = 0x1.1107605230bc4p-7;
constexpr double kS3 = -0x1.994eb3774cf24p-13;

PT_HD uint32_t f32_bits(float f)
{
#if defined(__HIPCC__)
    return __builtin_bit_cast(uint32_t, f);
#else
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
#endif
}

// Both results of one argument (the reduction is shared; each output equals the separate call).
// Straight-line form of glibc's sincosf for |y| < 120 (same results, no branches):
//  * |y| < 2^-12 (glibc: sinf = y, cosf = 1) and 2^-12 <= |y| < 0.75 (glibc: no reduction) run
//    the reduction and polynomials too: below 0.75 the reduction yields n = 0 and x = y exactly,
//    and below 2^-12 the polynomials round to y and 1 (|y^3/6| and y^2/2 stay below half an ulp);
//  * the sine polynomial of glibc's x * sign[n & 3] is evaluated on x and its f32 result negated:
//    every term of the odd polynomial changes sign exactly (round-to-nearest is sign-symmetric).
// Checked exhaustively against the host libm (tests/test_sincosf.py).
PT_HD void sincosf_glibc(float y, float* s_out, float* c_out)
{
    double x = (double)y;
    const double r = x * kHpiInv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = __builtin_fma(-(double)n, kHpi, x);
    // The two polynomial constants that end up as fma addends must sit in VGPRs; writing them with
    // inline v_mov makes the device code materialise them here (two v_mov each) instead of
    // hoisting them out of the caller's loop, where the register allocator spilled them to scratch.
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t s2lo, s2hi, c3lo, c3hi;
    asm volatile("v_mov_b32 %0, %1" : "=v"(s2lo) : "n"((uint32_t)(__builtin_bit_cast(uint64_t, kS2) & 0xffffffffu)));
    asm volatile("v_mov_b32 %0, %1" : "=v"(s2hi) : "n"((uint32_t)(__builtin_bit_cast(uint64_t, kS2) >> 32)));
    asm volatile("v_mov_b32 %0, %1" : "=v"(c3lo) : "n"((uint32_t)(__builtin_bit_cast(uint64_t, kC3) & 0xffffffffu)));
    asm volatile("v_mov_b32 %0, %1" : "=v"(c3hi) : "n"((uint32_t)(__builtin_bit_cast(uint64_t, kC3) >> 32)));
    const double s2 = __builtin_bit_cast(double, (uint64_t)s2hi << 32 | s2lo);
    const double c3 = __builtin_bit_cast(double, (uint64_t)c3hi << 32 | c3lo);
#else
    const double s2 = kS2, c3 = kC3;
#endif
    const double x2 = x * x;
    // sine polynomial (sinf_poly, even n), on x; its sign sign[n & 3] = {1,-1,-1,1} applied below
    const double x3 = x * x2;
    const double s1 = __builtin_fma(x2, kS3, s2);
    const double x7 = x3 * x2;
    const double ss = __builtin_fma(x3, kS1, x);
    const float sp = (float)__builtin_fma(x7, s1, ss);
    // cosine polynomial (sinf_poly, odd n), table selected by n & 2 (negated)
    const double x4 = x2 * x2;
    const double c2 = __builtin_fma(x2, kC4, c3);
    const double c1 = __builtin_fma(x2, kC1, kC0);
    const double x6 = x4 * x2;
    const double cc = __builtin_fma(x4, kC2, c1);
    const float cp = (float)__builtin_fma(x6, c2, cc);
    const uint32_t sps = f32_bits(sp) ^ ((uint32_t)((n + 1) & 2) << 30);
    const uint32_t cps = f32_bits(cp) ^ ((uint32_t)(n & 2) << 30);
    // sinf uses poly(n), cosf uses poly(n ^ 1)
    const uint32_t sb = (n & 1) ? cps : sps, cb = (n & 1) ? sps : cps;
#if defined(__HIPCC__)
    *s_out = __builtin_bit_cast(float, sb);
    *c_out = __builtin_bit_cast(float, cb);
#else
    __builtin_memcpy(s_out, &sb, 4);
    __builtin_memcpy(c_out, &cb, 4);
#endif
}

}  // namespace pt
