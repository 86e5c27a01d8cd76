// pt_tonemap.h -- the output stage's per-channel conversion (linear HDR -> 8-bit), shared by the
// standalone pass (pt_output.hip pt_tonemap_kernel) and the render kernels' fused presentation
// (pt_kernel.hip render_body_ct: a pixel's packed value written at its last fold).
//
// Reference (CPUPerformanceRayTracer/demofox_path_tracing_optimization_v4.cpp; both branches of
// global_preprocessor_flags.h:62-63, USE_FAST_APPROXIMATE_GAMMA / USE_FAST_APPROXIMATE_ACES_TONEMAP):
//   OutputToScreen :1260-1295 / OutputToFile :1297-1331: ACESFilm :165-175 -> LinearToSRGB :177-186
//   (fast_pow_gamma :144-155) -> saturate * 255 -> cvtps_epi32 -> packed u32.
// Numerics: the reference's operations in its order, fmadd/fmsub fused (__builtin_fmaf), sqrt
// correctly rounded (guarded fast path), MAXPS/MINPS NaN rules, round-to-nearest-even conversion.
// `rcp` is _mm256_rcp_ps in the reference, whose table is CPU-model specific; here it is the
// correctly rounded 1/x (as in the oracle, oracle/pt_oracle_output.c): at most 1 LSB from any x86 run.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pt_exactmath.h"
#include "pt_libmf.h"

namespace pt_tone {

__device__ __forceinline__ float max_ps(float a, float b) { return a > b ? a : b; }   // b on NaN / equal
__device__ __forceinline__ float min_ps(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float saturate(float x) { return min_ps(max_ps(x, 0.0f), 1.0f); }
// correctly rounded 1/x and sqrt through the guarded fast paths (bit-identical to IEEE '/' and
// sqrtf for every input, pt_exactmath.h): ~3x fewer instructions than the general sequences
__device__ __forceinline__ float rcp(float x) { return pt::div_guarded(1.0f, x); }
__device__ __forceinline__ float sqrt_(float x) { return pt::sqrt_guarded(x); }

__device__ __forceinline__ float fast_pow_gamma(float x)   // :144-155
{
    const float sqrtx = sqrt_(x);
    const float onethird = 1.f / 3.f, twothirds = 2.f / 3.f;
    const float nit1 = __builtin_fmaf(sqrtx, twothirds, onethird);
    const float nit2 = __builtin_fmaf(nit1, twothirds, (x * rcp(nit1 * nit1)) * onethird);
    const float nit3 = __builtin_fmaf(nit2, twothirds, (x * rcp(nit2 * nit2)) * onethird);
    return sqrt_(sqrtx * nit3);
}

template <bool FAST>
__device__ __forceinline__ float aces(float X)   // ACESFilm :165-175
{
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    if (FAST) {   // USE_FAST_APPROXIMATE_ACES_TONEMAP 1 (:168-171): rcp of the fused denominator
        const float rcp_denom = rcp(__builtin_fmaf(X, __builtin_fmaf(c, X, d), e));
        return saturate((X * __builtin_fmaf(a, X, b)) * rcp_denom);
    }
    // 0 (:172-174): f32 scalar * m256x3 operators, unfused (mul, add), then the IEEE division
    const float num = X * (a * X + b);
    const float den = X * (c * X + d) + e;
    return saturate(pt::div_guarded(num, den));
}

template <bool FAST>
__device__ __forceinline__ float linear_to_srgb(float x)   // :177-186
{
    x = saturate(x);
    if (x < 0.0031308f) return x * 12.92f;
    if (FAST) return __builtin_fmaf(1.055f, fast_pow_gamma(x), -0.055f);   // :182-183 (fmsub)
    // USE_FAST_APPROXIMATE_GAMMA 0 (:184-185): 1.055f * pow_ps(rgb, 1 / 2.4f) - 0.055f, SVML pow_ps ->
    // glibc-exact powf (pt_libmf.h; x in [0.0031308, 1] is inside its main path)
    return 1.055f * pt::lm::powf_glibc_main(x, 1.0f / 2.4f) - 0.055f;
}

template <bool FAST_ACES, bool FAST_GAMMA>
__device__ __forceinline__ uint32_t channel(float linear)
{
    const float c_exposure = 1.0f;
    const float v = saturate(linear_to_srgb<FAST_GAMMA>(aces<FAST_ACES>(linear * c_exposure))) * 255.f;
    return (uint32_t)(int32_t)__builtin_rintf(v) & 0xFFu;   // cvtps_epi32 (nearest even) & ByteMask
}

// One pixel: OutputToScreen's 0x00RRGGBB (xrgb) or OutputToFile's 0xFFBBGGRR
template <bool FAST_ACES, bool FAST_GAMMA>
__device__ __forceinline__ uint32_t pack(float r_lin, float g_lin, float b_lin, bool xrgb)
{
    const uint32_t r = channel<FAST_ACES, FAST_GAMMA>(r_lin), g = channel<FAST_ACES, FAST_GAMMA>(g_lin),
                   b = channel<FAST_ACES, FAST_GAMMA>(b_lin);
    return xrgb ? ((r << 16) | (g << 8) | b)           // OutputToScreen :1282-1285
                : (0xFF000000u | (b << 16) | (g << 8) | r);   // OutputToFile :1319-1323
}

}  // namespace pt_tone
