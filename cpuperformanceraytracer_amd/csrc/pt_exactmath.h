// pt_exactmath.h -- correctly rounded f32 reciprocal / division / square root in fewer VALU
// instructions than the compiler's general IEEE expansions, for the operand ranges the path
// tracer produces.  Bit-identical to IEEE '/' and sqrtf wherever they are used (proofs and
// exhaustive GPU checks: tests/native/exactmath_probe.hip, tests/test_gpu_exactmath.py).
//
// Why: on gfx950 the compiler's correctly rounded f32 division costs ~17 v_add-equivalents of
// issue time and sqrtf ~23 (scripts/valu_microbench.hip), because they handle every
// input class (denormals via scaling, inf/nan fix-ups).  The path tracer's divisors and radicands
// are normal numbers in a known range, and outside it only the SIGN or ORDER of the result
// matters to the reference (it is compared against 0.01 / the running best and discarded), so a
// guarded fast path keeps bit-exactness where the value is used.
#pragma once
#include <stdint.h>

namespace pt {

__device__ __forceinline__ float rcp_approx(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sqrt_approx(float x) { return __builtin_amdgcn_sqrtf(x); }

// RN(1/x) for |x| in [2^-125, 2^125]: hardware reciprocal (<= 1 ulp) + one Newton-Raphson step
// with exact-residual FMA.  Outside that range callers must not rely on the value.
__device__ __forceinline__ float rcp_rn(float x)
{
    float r = rcp_approx(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    return r;
}

// RN(1/x) for |x| < 2^-125 (zero, denormals, the lowest normals) and NaN: 1/+-0 = +-inf, else x 2^24 is
// exact and inside rcp_rn's range, and scaling its correctly rounded reciprocal back by 2^24 is exact
// (the same relative rounding; a result that rounds to 2^128 overflows to inf, as RN(1/x) does).
// The slow path of a range guard: a few VALU instead of the compiler's IEEE division sequence
// (tests/native/exactmath_probe.hip checks every such x).
__device__ __forceinline__ float rcp_tiny_rn(float x)
{
    const float r = rcp_rn(x * 0x1p24f) * 0x1p24f;
    return x == 0.0f ? __builtin_copysignf(__builtin_huge_valf(), x) : r;
}

// RN(a/b) given y = RN(1/b) (Markstein: with y the correctly rounded reciprocal and a faithful
// first quotient, the exact-remainder correction yields the correctly rounded quotient).  Two
// corrections: the first makes the quotient faithful, the second rounds it correctly.  Valid when
// b, a and a/b are normal and no intermediate overflows.
__device__ __forceinline__ float div_rn(float a, float b, float y)
{
    float q = a * y;
    float r = __builtin_fmaf(-q, b, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, y, q);
}

// RN(sqrt(x)) for x in [2^-100, FLT_MAX]: Markstein's sequence on the hardware reciprocal square
// root -- s = x y and h = y / 2 from y ~ 1/sqrt(x), the exact FMA residual r = x - s^2, then
// s + r h rounded once.  Correctly rounded for EVERY f32 in that range on gfx950 (exhaustive,
// tests/native/exactmath_probe.hip: 1 912 602 624 inputs, 0 mismatches; v_sqrt_f32 alone misses
// 15 % of them).  Five VALU operations, none a compare or select: the previous neighbour check
// around v_sqrt_f32 needed two compares and two selects.
__device__ __forceinline__ float sqrt_rn(float x)
{
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y, h = 0.5f * y;
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, h, s);
}

// General-purpose guarded forms: the fast path where its preconditions provably hold, IEEE
// otherwise (bit-identical to '/' and sqrtf for every input).
__device__ __forceinline__ float sqrt_guarded(float x)
{
    float s = sqrt_rn(x);
    if (__builtin_expect(!(x >= 0x1p-100f), 0)) s = __builtin_sqrtf(x);   // 0, tiny, NaN
    return s;
}

// a / b: div_rn is correctly rounded when b is in [2^-125, 2^125], |a| < 2^124 and the quotient
// is normal; the result is accepted only with a margin of one binade on both ends of the normal
// range (so a rounded quotient cannot hide a subnormal or overflowing true quotient).
__device__ __forceinline__ float div_guarded(float a, float b)
{
    const float ab = __builtin_fabsf(b);
    float q = div_rn(a, b, rcp_rn(b));
    const float aq = __builtin_fabsf(q);
    const bool ok = ab >= 0x1p-125f && ab <= 0x1p125f && __builtin_fabsf(a) < 0x1p124f && aq >= 0x1p-125f &&
                    aq <= 0x1p126f;
    if (__builtin_expect(!ok, 0)) q = a / b;
    return q;
}

}  // namespace pt
