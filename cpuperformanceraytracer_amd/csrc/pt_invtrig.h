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
// non-negative f32, atan2f on 4e8 random pairs (tests/test_invtrig.py).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PT_IT_HD __host__ __device__ __forceinline__
#else
#define PT_IT_HD static inline
#endif

namespace pt {

PT_IT_HD uint32_t it_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
PT_IT_HD float it_float(uint32_t u) { return __builtin_bit_cast(float, u); }
PT_IT_HD float it_fabs(float x) { return it_float(it_bits(x) & 0x7fffffffu); }
PT_IT_HD float it_sqrt(float x) { return __builtin_sqrtf(x); }   // IEEE (parity build flags)

// s_atanf.c (fdlibm single precision)
PT_IT_HD float atanf_glibc(float x)
{
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = (int32_t)it_bits(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {                       // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;        // NaN
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {                        // |x| < 0.4375
        if (ix < 0x31000000) return x;            // |x| < 2^-29
        id = -1;
    } else {
        x = it_fabs(x);
        if (ix < 0x3f980000) {                    // |x| < 1.1875
            if (ix < 0x3f300000) {                // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {                              // 11/16 <= |x| < 19/16
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000) {             // |x| < 2.4375
            id = 2;
            x = (x - 1.5f) / (1.0f + 1.5f * x);
        } else {                                  // 2.4375 <= |x| < 2^25
            id = 3;
            x = -1.0f / x;
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

// e_atan2f.c (fdlibm single precision)
PT_IT_HD float atan2f_glibc(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
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
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;                  // |y/x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0f;                    // |y|/x < -2^60
    else z = atanf_glibc(it_fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return it_float(it_bits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// e_asinf.c (glibc single precision, degree-5 polynomial)
PT_IT_HD float asinf_glibc(float x)
{
    const float pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
                pio4_hi = 0.785398185253143310546875f, p0 = 1.666675248e-01f, p1 = 7.495297643e-02f,
                p2 = 4.547037598e-02f, p3 = 2.417951451e-02f, p4 = 4.216630880e-02f;
    const int32_t hx = (int32_t)it_bits(x), ix = hx & 0x7fffffff;
    float t, w, p, q, c, r, s;
    if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;       // |x| == 1
    if (ix > 0x3f800000) return (x - x) / (x - x);                 // |x| > 1: NaN
    if (ix < 0x3f000000) {                                         // |x| < 0.5
        if (ix < 0x32000000) return x;                             // |x| < 2^-27
        t = x * x;
        w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
        return x + x * w;
    }
    w = 1.0f - it_fabs(x);                                         // 0.5 <= |x| < 1
    t = w * 0.5f;
    p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    s = it_sqrt(t);
    if (ix >= 0x3F79999A) {                                        // |x| > 0.975
        t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
    } else {
        w = it_float(it_bits(s) & 0xfffff000u);
        c = (t - w * w) / (s + w);
        r = p;
        p = 2.0f * s * r - (pio2_lo - 2.0f * c);
        q = pio4_hi - 2.0f * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

}  // namespace pt
