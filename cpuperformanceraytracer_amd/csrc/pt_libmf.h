// pt_libmf.h -- expf and powf on the GPU, bit-identical to the host libm (glibc 2.35, x86-64 FMA
// variant) the oracle calls where the reference calls SVML.
//
// The reference's non-default global_preprocessor_flags branches (global_preprocessor_flags.h:62,64)
// call SVML: USE_FAST_APPROXIMATE_EXP 0 -> exp_ps (Beer absorption, v4 :786, :974) and
// USE_FAST_APPROXIMATE_GAMMA 0 -> pow_ps (LinearToSRGB, v4 :184-185).  SVML's results have no
// published bit pattern, so -- as for its atan2/asin/sincos -- the oracle substitutes
// the host libm (expf, powf) and this header reproduces glibc's algorithms: they evaluate in double
// with a 32-entry 2^(i/32) table (expf; exp2 part of powf) and a 16-entry (1/c, log2 c) table
// (log2 part of powf), short polynomials, fused multiply-adds exactly where the x86-64 FMA ifunc
// variants (__expf_fma / __powf_fma, selected on AVX2+FMA hosts) fuse, and one rounding to f32.
// Every double op is IEEE on both x86-64 and gfx950, so the same ops on the same constants give the
// same f32.  The constants below were read from the image's libm.so.6 (the FMA variants' code and
// the shared __exp2f_data / __powf_log2_data tables).
//
// Verified on the host against libm (tests/native/check_libmf.cpp compiles THIS header):
//   expf on every f32 (all 2^32 bit patterns), powf(x, 1/2.4f) on every f32 x in [2^-9, 1] (the
//   tonemap's domain [0.0031308, 1]) and on random (x, y) with |y log2 x| < 126.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PT_LM_HD __host__ __device__ __forceinline__
#else
#define PT_LM_HD static inline
#endif

namespace pt {
namespace lm {

// __exp2f_data.tab: asuint64(2^(i/32)) - (i << 47)
constexpr uint64_t kExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
// expf (__exp2f_data: shift_scaled, invln2_scaled, poly_scaled)
constexpr double kExpShift = 0x1.8p+52;
constexpr double kExpInvLn2N = 0x1.71547652b82fep+5;
constexpr double kExpC0 = 0x1.c6af84b912394p-20, kExpC1 = 0x1.ebfce50fac4f3p-13, kExpC2 = 0x1.62e42ff0c52d6p-6;
// exp2 (powf's exp2_inline: shift, poly)
constexpr double kExp2Shift = 0x1.8p+47;
constexpr double kExp2C0 = 0x1.c6af84b912394p-5, kExp2C1 = 0x1.ebfce50fac4f3p-3, kExp2C2 = 0x1.62e42ff0c52d6p-1;
// __powf_log2_data: (invc, logc) per interval, poly A[0..4]
constexpr double kLog2Tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
};
constexpr double kLog2A0 = 0x1.27616c9496e0bp-2, kLog2A1 = -0x1.71969a075c67ap-2, kLog2A2 = 0x1.ec70a6ca7baddp-2,
                 kLog2A3 = -0x1.7154748bef6c8p-1, kLog2A4 = 0x1.71547652ab82bp+0;

PT_LM_HD uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
PT_LM_HD float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }
PT_LM_HD uint64_t dbits(double d) { return __builtin_bit_cast(uint64_t, d); }
PT_LM_HD double bitsd(uint64_t u) { return __builtin_bit_cast(double, u); }

// glibc expf (sysdeps/ieee754/flt-32/e_expf.c, FMA build).
PT_LM_HD float expf_glibc(float x)
{
    const uint32_t ux = fbits(x);
    const uint32_t abstop = (ux >> 20) & 0x7ffu;
    if (abstop > 0x42au) {                                   // |x| >= 88 or not finite
        if (ux == 0xff800000u) return 0.0f;                  // -inf
        if (abstop >= 0x7f8u) return x + x;                  // +inf, nan
        if (x > 0x1.62e42ep6f) return bitsf(0x7f800000u);    // __math_oflowf: +inf
        if (x < -0x1.9fe368p6f) return 0.0f;                 // __math_uflowf: 0x1p-95f * 0x1p-95f
        if (x < -0x1.9d1d9ep6f) return bitsf(1u);            // __math_may_uflowf: 0x1.4p-75f^2 -> 2^-149
    }
    const double xd = (double)x;
    double kd = __builtin_fma(kExpInvLn2N, xd, kExpShift);   // z + shift, fused
    const uint64_t ki = dbits(kd);
    kd -= kExpShift;
    const double r = __builtin_fma(kExpInvLn2N, xd, -kd);    // z - kd, fused
    const uint64_t t = kExp2Tab[ki % 32u] + (ki << 47);
    const double s = bitsd(t);
    const double z = __builtin_fma(kExpC0, r, kExpC1);
    const double r2 = r * r;
    double y = __builtin_fma(kExpC2, r, 1.0);
    y = __builtin_fma(z, r2, y);
    y = y * s;
    return (float)y;
}

// glibc powf (sysdeps/ieee754/flt-32/e_powf.c, FMA build), main path only: x a positive normal
// f32, y finite and non-zero, |y * log2(x)| < 126 (no overflow / underflow handling -- the caller's
// domain, LinearToSRGB's x in [0.0031308, 1] and y = 1/2.4f, never reaches it).
PT_LM_HD float powf_glibc_main(float x, float y)
{
    const uint32_t ix = fbits(x);
    // log2_inline
    const uint32_t tmp = ix - 0x3f330000u;
    const uint32_t i = (tmp >> 19) & 15u;
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int32_t k = (int32_t)top >> 23;
    const double invc = kLog2Tab[i][0], logc = kLog2Tab[i][1];
    const double zz = (double)bitsf(iz);
    const double r = __builtin_fma(zz, invc, -1.0);
    const double y0 = (double)k + logc;
    const double r2 = r * r;
    double yy = __builtin_fma(r, kLog2A0, kLog2A1);
    const double p = __builtin_fma(r, kLog2A2, kLog2A3);
    const double r4 = r2 * r2;
    double q = __builtin_fma(r, kLog2A4, y0);
    q = __builtin_fma(r2, p, q);
    yy = __builtin_fma(yy, r4, q);
    const double ylogx = (double)y * yy;
    // exp2_inline(ylogx, sign_bias = 0)
    double kd = ylogx + kExp2Shift;
    const uint64_t ki = dbits(kd);
    kd -= kExp2Shift;
    const double rr = ylogx - kd;
    const uint64_t t = kExp2Tab[ki % 32u] + (ki << 47);
    const double s = bitsd(t);
    const double z = __builtin_fma(rr, kExp2C0, kExp2C1);
    const double rr2 = rr * rr;
    double e = __builtin_fma(rr, kExp2C2, 1.0);
    e = __builtin_fma(z, rr2, e);
    e = e * s;
    return (float)e;
}

}  // namespace lm
}  // namespace pt
