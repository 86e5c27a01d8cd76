// pt_invtrig.h -- atan2f / asinf on the GPU, bit-identical to the host libm the reference calls.
//
// EquirectangularTextureSample (texture.cpp:101-139) maps a direction to texture coordinates with
// atan2(Direction.z, Direction.x) and asin(Direction.y) on f32 -- the float overloads under MSVC,
// i.e. atan2f/asinf (see oracle/build_ref.sh).  The image's glibc 2.35 implements both with the
// classic fdlibm single-precision algorithms (e_atan2f.c + s_atanf.c, and e_asinf.c with a
// degree-5 polynomial): pure f32 arithmetic with correctly rounded '/' and sqrt.  The functions
// below restate those algorithms operation for operation; compiled without contraction
// (-ffp-contract=off) and with IEEE '/' and sqrt they give the host's bit patterns on any IEEE
// binary32 unit.  Checked on the host against glibc: asinf on every f32 in [-1, 1], atanf on every
// non-negative f32, atan2f on 1e8 random pairs (tests/test_invtrig.py).
#pragma once
#include <stdint.h>

#ifndef PT_IT_HD
#if defined(__HIPCC__)
#define PT_IT_HD __host__ __device__ __forceinline__
#else
#define PT_IT_HD static inline
#endif
#endif
// correctly rounded '/' and sqrt; a GPU includer may substitute cheaper exact forms
// (pt_exactmath.h div_guarded / sqrt_guarded, bit-identical for every input)
#ifndef PT_IT_DIV
#define PT_IT_DIV(a, b) ((a) / (b))
#endif
#ifndef PT_IT_SQRT
#define PT_IT_SQRT(x) it_sqrt(x)
#endif

namespace pt {

PT_IT_HD uint32_t it_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
PT_IT_HD float it_float(uint32_t u) { return __builtin_bit_cast(float, u); }
PT_IT_HD float it_fabs(float x) { return it_float(it_bits(x) & 0x7fffffffu); }
PT_IT_HD float it_sqrt(float x) { return __builtin_sqrtf(x); }   // IEEE (parity build flags)
// table lookup as a select chain (a dynamically indexed local array would go to GPU scratch)
PT_IT_HD float it_pick4(int i, float a, float b, float c, float d) { return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d)); }

// s_atanf.c (fdlibm single precision).  Written as selects: the four argument reductions are the
// same operations, chosen per lane, feeding ONE division (no reduction: x / 1 == x exactly), and
// the out-of-range results are selected at the end -- one straight-line sequence per wave
// whatever mix of ranges its lanes hold.
PT_IT_HD float atanf_glibc(float x)
{
    const float hi0 = 4.6364760399e-01f, hi1 = 7.8539812565e-01f, hi2 = 9.8279368877e-01f, hi3 = 1.5707962513e+00f;
    const float lo0 = 5.0121582440e-09f, lo1 = 3.7748947079e-08f, lo2 = 3.4473217170e-08f, lo3 = 7.5497894159e-08f;
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = (int32_t)it_bits(x);
    const int32_t ix = hx & 0x7fffffff;
    const float ax = it_fabs(x);
    const bool no_red = ix < 0x3ee00000;          // |x| < 0.4375
    const bool r0 = ix < 0x3f300000;              // 7/16 <= |x| < 11/16
    const bool r1 = ix < 0x3f980000;              // 11/16 <= |x| < 19/16
    const bool r2 = ix < 0x401c0000;              // 19/16 <= |x| < 2.4375 (else: up to 2^25)
    const float n0 = 2.0f * ax - 1.0f, d0 = 2.0f + ax;
    const float n1 = ax - 1.0f, d1 = ax + 1.0f;
    const float n2 = ax - 1.5f, d2 = 1.0f + 1.5f * ax;
    float num = r2 ? n2 : -1.0f, den = r2 ? d2 : ax;
    num = r1 ? n1 : num;
    den = r1 ? d1 : den;
    num = r0 ? n0 : num;
    den = r0 ? d0 : den;
    num = no_red ? x : num;
    den = no_red ? 1.0f : den;
    const int id = no_red ? -1 : (r0 ? 0 : (r1 ? 1 : (r2 ? 2 : 3)));
    const float xr = PT_IT_DIV(num, den);
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const float r_small = xr - xr * (s1 + s2);
    const float r = it_pick4(id, hi0, hi1, hi2, hi3) - ((xr * (s1 + s2) - it_pick4(id, lo0, lo1, lo2, lo3)) - xr);
    float res = no_red ? r_small : (hx < 0 ? -r : r);
    res = ix < 0x31000000 ? x : res;              // |x| < 2^-29
    if (ix >= 0x4c000000)                         // |x| >= 2^25, NaN
        res = ix > 0x7f800000 ? x + x : (hx > 0 ? hi3 + lo3 : -hi3 - lo3);
    return res;
}

// e_atan2f.c (fdlibm single precision).  The special operands (NaN, zero, infinite, x == 1) are
// tested together and handled off the main path, so a wave of ordinary directions runs one
// branch-free sequence.
PT_IT_HD float atan2f_special(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f;
    const int32_t hx = (int32_t)it_bits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)it_bits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;   // NaN
    if (hx == 0x3f800000) return atanf_glibc(y);            // x == 1.0
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      // 2*sign(x) + sign(y)
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;          // iy == 0x7f800000
}

PT_IT_HD float atan2f_glibc(float y, float x)
{
    const float pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)it_bits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)it_bits(y), iy = hy & 0x7fffffff;
    if ((uint32_t)(ix - 1) >= 0x7f7fffffu || (uint32_t)(iy - 1) >= 0x7f7fffffu || hx == 0x3f800000)   // 0, inf, NaN; x == 1
        return atan2f_special(y, x);
    const int32_t k = (iy - ix) >> 23;
    const float zq = atanf_glibc(it_fabs(PT_IT_DIV(y, x)));
    float z = (hx < 0 && k < -60) ? 0.0f : zq;              // |y|/x < -2^60
    z = k > 60 ? pi_o_2 + 0.5f * pi_lo : z;                  // |y/x| > 2^60
    const float zn = it_float(it_bits(z) ^ 0x80000000u);
    const float zl = z - pi_lo;
    const float r_neg_x = hy < 0 ? zl - pi : pi - zl;       // m == 3 : m == 2
    return hx < 0 ? r_neg_x : (hy < 0 ? zn : z);             // m == 0, 1
}

// e_asinf.c (glibc single precision, degree-5 polynomial).  Both ranges share the polynomial
// (its argument selected per lane); both |x| >= 0.5 tails run for every lane and are selected.
PT_IT_HD float asinf_glibc(float x)
{
    const float pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
                pio4_hi = 0.785398185253143310546875f, p0 = 1.666675248e-01f, p1 = 7.495297643e-02f,
                p2 = 4.547037598e-02f, p3 = 2.417951451e-02f, p4 = 4.216630880e-02f;
    const int32_t hx = (int32_t)it_bits(x), ix = hx & 0x7fffffff;
    if ((uint32_t)(ix - 0x32000000) >= (uint32_t)(0x3f800000 - 0x32000000)) {   // rare operands, one test
        if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;   // |x| == 1
        if (ix > 0x3f800000) return (x - x) / (x - x);             // |x| > 1: NaN
        return x;                                                  // |x| < 2^-27
    }
    const bool small = ix < 0x3f000000;                            // |x| < 0.5
    const float t = small ? x * x : (1.0f - it_fabs(x)) * 0.5f;
    const float p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    const float r_small = x + x * p;
    const float s = PT_IT_SQRT(t);
    const float r_far = pio2_hi - (2.0f * (s + s * p) - pio2_lo);  // |x| > 0.975
    const float w = it_float(it_bits(s) & 0xfffff000u);              // else
    const float c = PT_IT_DIV(t - w * w, s + w);
    const float pp = 2.0f * s * p - (pio2_lo - 2.0f * c);
    const float q = pio4_hi - 2.0f * w;
    const float r_mid = pio4_hi - (pp - q);
    const float r_big = ix >= 0x3F79999A ? r_far : r_mid;
    return small ? r_small : (hx > 0 ? r_big : -r_big);
}

}  // namespace pt
