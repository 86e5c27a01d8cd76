// pt_envcert.h -- certified fast texel cells of EquirectangularTextureSample* (texture.cpp:101-139,
// :186-203): the texel a miss reads, bit-identical to the reference's, with most of the glibc-exact
// atan2f / asinf arithmetic (pt_invtrig.h) replaced by short polynomials.
//
// What the reference computes from the direction is only an integer pair: the texel row and column,
// each a monotone non-decreasing step function of one angle --
//   at = atan2f(d.z, d.x) -> u = 0.1591 at + 0.5 -> column;   as = asinf(d.y) -> v = 0.3183 as + 0.5 -> row
// (fma / mul / add / floor / truncation of f32 values, each monotone; the fract-wrap u - floor(u) is
// the identity because |at| <= pi and |as| <= pi / 2 keep u, v inside (1.7e-5, 0.99983)).  So if the
// exact glibc angle is known to lie in [lo, hi] and the reference's own f32 operations map lo and hi
// to the same integer, that integer is the reference's.  This header gives such intervals:
//   * atan2f: glibc (e_atan2f.c) computes z = atanf(q), q = RN(|y| / |x|), then the sign of y and, for
//     x < 0, pi - (z - pi_lo) -- the same operations here, applied to the interval ends of z (both
//     maps are monotone in z).  ec_atan(q) is within kEcAtanE of atanf_glibc(q) for EVERY f32 q of the
//     domain (2^-40, 2^40): checked exhaustively on the host (tests/native/check_envcert.cpp);
//   * asinf: odd in glibc exactly (e_asinf.c), ec_asin(a) within kEcAsinE of asinf_glibc(a) for every
//     f32 a in [0, 1 - 2^-20] (exhaustive, the same check).
// The containment is checked with the interval ends as computed here (fl(z -+ E)), so the rounding of
// the ends is covered too.  The operations are f32 add / mul / fma and the correctly rounded 1/x, a/b
// and sqrt (pt_exactmath.h on the GPU, bit-identical to IEEE inside the ranges used here), so host and
// GPU compute the same bits and the host's exhaustive check is a check of the GPU's values.
// Directions outside the domain (a component below 2^-20 or above 2^20 in magnitude, |d.y| > 1 -
// 2^-20, NaN) and cells whose ends disagree take the exact path (the caller's fallback).
#pragma once
#include <stdint.h>

#ifndef PT_EC_HD
#if defined(__HIPCC__)
#define PT_EC_HD __host__ __device__ __forceinline__
#else
#define PT_EC_HD static inline
#endif
#endif
// correctly rounded 1/x, a/b and sqrt for the operand ranges below (a GPU includer substitutes the
// fast sequences of pt_exactmath.h)
#ifndef PT_EC_RCP
#define PT_EC_RCP(x) (1.0f / (x))
#endif
#ifndef PT_EC_DIV
#define PT_EC_DIV(a, b) ((a) / (b))
#endif
#ifndef PT_EC_SQRT
#define PT_EC_SQRT(x) __builtin_sqrtf(x)
#endif

#ifndef PT_EC_FORCE_EXACT
#define PT_EC_FORCE_EXACT 0   // test builds: no cell is certified, every lookup takes the exact fallback
#endif

namespace pt {

// Interval half-widths (radians): the exhaustive host check measures max |ec_atan - atanf_glibc| =
// 1.19e-7 and max |ec_asin - asinf_glibc| = 1.19e-7 and asserts containment with these values.  The
// cells of uniformly distributed directions are then uncertified (exact fallback) for 1.6e-4 of them.
constexpr float kEcAtanE = 1.5e-7f;
constexpr float kEcAsinE = 1.5e-7f;

PT_EC_HD uint32_t ec_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

// atan(q) for q in (2^-40, 2^40): atan(s), s = min(q, 1/q), as s + s z P(z), z = s^2 (a degree-8
// weighted least-squares fit on [0, 1], 1.2e-8 in real arithmetic); pi/2 - atan(1/q) above 1.
PT_EC_HD float ec_atan(float q)
{
    const bool big = q > 1.0f;
    const float s = big ? PT_EC_RCP(q) : q;
    const float z = s * s;
    float p = -0x1.48d92ep-9f;
    p = __builtin_fmaf(p, z, 0x1.caaef6p-7f);
    p = __builtin_fmaf(p, z, -0x1.2c6c58p-5f);
    p = __builtin_fmaf(p, z, 0x1.02cdbap-4f);
    p = __builtin_fmaf(p, z, -0x1.63e87cp-4f);
    p = __builtin_fmaf(p, z, 0x1.c4488p-4f);
    p = __builtin_fmaf(p, z, -0x1.247258p-3f);
    p = __builtin_fmaf(p, z, 0x1.99988p-3f);
    p = __builtin_fmaf(p, z, -0x1.555554p-2f);
    const float r = __builtin_fmaf(s * z, p, s);
    return big ? 1.57079637f - r : r;
}

// asin(a) for a in [0, 1 - 2^-20]: asin(s) = s + s t Q(t) on t in [0, 1/4] (degree 4, 8e-9), with
// s = a, t = a^2 below 1/2 and pi/2 - 2 asin(sqrt((1 - a) / 2)) above (1 - a and the halving exact).
PT_EC_HD float ec_asin(float a)
{
    const bool small = a < 0.5f;
    const float t = small ? a * a : (1.0f - a) * 0.5f;
    const float s = small ? a : PT_EC_SQRT(t);   // t >= 2^-21 where it is used
    float p = 0x1.39fa5ap-5f;
    p = __builtin_fmaf(p, t, 0x1.b117bap-6f);
    p = __builtin_fmaf(p, t, 0x1.70ce08p-5f);
    p = __builtin_fmaf(p, t, 0x1.332638p-4f);
    p = __builtin_fmaf(p, t, 0x1.55555ep-3f);
    const float r = __builtin_fmaf(s * t, p, s);
    return small ? r : 1.57079637f - 2.0f * r;
}

// The domain: |x|, |y| in [2^-20, 2^20) (so q is in (2^-40, 2^40), normal, and glibc's |k| > 60
// branches and special operands cannot occur); |s| <= 1 - 2^-20.  Integer range tests on the bits
// (NaN fails them).
PT_EC_HD bool ec_in_domain(float y, float x, float s)
{
    const uint32_t ix = ec_bits(x) & 0x7fffffffu, iy = ec_bits(y) & 0x7fffffffu, is = ec_bits(s) & 0x7fffffffu;
    return !PT_EC_FORCE_EXACT && (ix - 0x35800000u) < (0x49800000u - 0x35800000u) && (iy - 0x35800000u) < (0x49800000u - 0x35800000u) &&
           is <= 0x3f7ffff0u;   // 1 - 2^-20
}

// [lo, hi] holding atan2f_glibc(y, x), for (y, x) in the domain
PT_EC_HD void ec_atan2_bounds(float y, float x, float& lo, float& hi)
{
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;   // e_atan2f.c
    const float z = ec_atan(PT_EC_DIV(__builtin_fabsf(y), __builtin_fabsf(x)));
    const float zlo = z - kEcAtanE, zhi = z + kEcAtanE;
    // x < 0: pi - (z - pi_lo), non-increasing in z; then y < 0 negates ((z - pi_lo) - pi ==
    // -(pi - (z - pi_lo)) exactly: RN is symmetric)
    const bool nx = ec_bits(x) >> 31, ny = ec_bits(y) >> 31;
    const float wa = nx ? pi - (zhi - pi_lo) : zlo;
    const float wb = nx ? pi - (zlo - pi_lo) : zhi;
    lo = ny ? -wb : wa;
    hi = ny ? -wa : wb;
}

// [lo, hi] holding asinf_glibc(s), for s in the domain (asinf is odd)
PT_EC_HD void ec_asin_bounds(float s, float& lo, float& hi)
{
    const float r = ec_asin(__builtin_fabsf(s));
    const float rlo = r - kEcAsinE, rhi = r + kEcAsinE;
    const bool ns = ec_bits(s) >> 31;
    lo = ns ? -rhi : rlo;
    hi = ns ? -rlo : rhi;
}

// The reference's f32 maps from the angles to the texel cell, on the interval ends (each monotone
// non-decreasing in its angle; the fract-wrap and the [0, 1) range test they follow are the identity
// and always true on these angles: |at| <= pi + 1.6e-7 gives u in (1.7e-4, 0.99983), |as| <= pi/2 +
// 1.6e-7 gives v in (1.7e-5, 0.99999)).

// EquirectangularTextureSampleRandom (texture.cpp:186-203) + TexelSampleRandom (:78-86), the v4
// default: floor(v (h - 1) + r1), floor(u (w - 1) + r2) with the sampler's two draws r1, r2 (Row's
// first).  true = certified: (row, col) are the reference's.
PT_EC_HD bool ec_cell_random(float y, float x, float s, float w, float h, float r1, float r2, float& row, float& col)
{
    if (!ec_in_domain(y, x, s)) return false;
    float alo, ahi, slo, shi;
    ec_atan2_bounds(y, x, alo, ahi);
    ec_asin_bounds(s, slo, shi);
    const float ulo = __builtin_fmaf(0.1591f, alo, 0.5f), uhi = __builtin_fmaf(0.1591f, ahi, 0.5f);
    const float vlo = __builtin_fmaf(0.3183f, slo, 0.5f), vhi = __builtin_fmaf(0.3183f, shi, 0.5f);
    const float rlo = __builtin_floorf(__builtin_fmaf(vlo, h, -vlo) + r1), rhi = __builtin_floorf(__builtin_fmaf(vhi, h, -vhi) + r1);
    const float clo = __builtin_floorf(__builtin_fmaf(ulo, w, -ulo) + r2), chi = __builtin_floorf(__builtin_fmaf(uhi, w, -uhi) + r2);
    row = rlo;
    col = clo;
    return rlo == rhi && clo == chi;
}

// EquirectangularTextureSample (texture.cpp:101-139) nearest texel, the config-4 env term:
// trunc(v (H - 1)), trunc(u (W - 1)) with u = at 0.1591 + 0.5, v = as 0.3183 + 0.5.
PT_EC_HD bool ec_cell_nearest(float y, float x, float s, float wm1, float hm1, int32_t& row, int32_t& col)
{
    if (!ec_in_domain(y, x, s)) return false;
    float alo, ahi, slo, shi;
    ec_atan2_bounds(y, x, alo, ahi);
    ec_asin_bounds(s, slo, shi);
    const int32_t rlo = (int32_t)((slo * 0.3183f + 0.5f) * hm1), rhi = (int32_t)((shi * 0.3183f + 0.5f) * hm1);
    const int32_t clo = (int32_t)((alo * 0.1591f + 0.5f) * wm1), chi = (int32_t)((ahi * 0.1591f + 0.5f) * wm1);
    row = rlo;
    col = clo;
    return rlo == rhi && clo == chi;
}

}  // namespace pt
