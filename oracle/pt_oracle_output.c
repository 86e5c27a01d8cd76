/* oracle/pt_oracle_output.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's
 * output stage, the checker for the GPU tonemap kernel (csrc/pt_output.hip).  Never linked into
 * the product.
 *
 * Reference (CPUPerformanceRayTracer/demofox_path_tracing_optimization_v4.cpp; the defaults of
 * global_preprocessor_flags.h:62-63, USE_FAST_APPROXIMATE_GAMMA = USE_FAST_APPROXIMATE_ACES_TONEMAP = 1,
 * and (pto_tonemap_ex) their 0 branches: ACESFilm :172-174 with '/', LinearToSRGB :184-185 with
 * SVML pow_ps, for which the host libm's powf stands in -- as for the other SVML calls, parity with
 * SVML itself is unpinned):
 *   fast_pow_gamma        :144-155   x^(1/2.4) = sqrt(sqrt(x) * cbrt(x)), 3 Newton steps for cbrt
 *   ACESFilm              :165-175   saturate(X (a X + b) * rcp(X (c X + d) + e))
 *   LinearToSRGB          :177-186   x < 0.0031308 ? 12.92 x : 1.055 pow - 0.055 (fmsub)
 *   OutputToScreen        :1260-1295 saturate(.) * 255 -> cvtps_epi32 -> 0x00RRGGBB
 *   OutputToFile          :1297-1331 ... -> 0xFFBBGGRR (bytes R, G, B, A = 255)
 * fmadd/fmsub are fused (mathlib.h:149,212: _mm256_fmadd_ps); sroot is IEEE sqrt (:439);
 * saturate = min_ps(max_ps(x, 0), 1) (:405,410), whose NaN rule returns the second operand;
 * cvtps_epi32 rounds to nearest even.  rcp is _mm256_rcp_ps (:417), an approximation whose exact
 * table differs between CPU models -- it has no portable bit pattern -- so this restatement (and
 * the GPU kernel) use the correctly rounded 1/x.  Against the reference on a given x86 CPU a
 * channel can then differ by at most 1 (the 12-bit RCPPS error is < 0.1 LSB after x255):
 * parity with that substitution is pinned bit-exactly, against RCPPS it is unpinned.
 * Compiled with -ffp-contract=off: only the explicit fmaf calls fuse.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include "pt_oracle.h"

static float max_ps(float a, float b) { return a > b ? a : b; }   /* MAXPS: b on NaN / equal */
static float min_ps(float a, float b) { return a < b ? a : b; }
static float saturate(float x) { return min_ps(max_ps(x, 0.0f), 1.0f); }
static float rcp(float x) { return 1.0f / x; }                    /* see header: RCPPS substitute */

static float fast_pow_gamma(float x)   /* v4 :144-155 */
{
    const float sqrtx = sqrtf(x);
    const float onethird = 1.f / 3.f, twothirds = 2.f / 3.f;
    const float nit1 = fmaf(sqrtx, twothirds, onethird);
    const float nit2 = fmaf(nit1, twothirds, (x * rcp(nit1 * nit1)) * onethird);
    const float nit3 = fmaf(nit2, twothirds, (x * rcp(nit2 * nit2)) * onethird);
    return sqrtf(sqrtx * nit3);
}

static float aces(float X)   /* v4 :165-175 (fast path) */
{
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    const float rcp_denom = rcp(fmaf(X, fmaf(c, X, d), e));
    return saturate((X * fmaf(a, X, b)) * rcp_denom);
}

static float aces_exact(float X)   /* v4 :172-174 (USE_FAST_APPROXIMATE_ACES_TONEMAP 0) */
{
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    /* f32 scalar x m256x3 operators: unfused mul / add, then _mm256_div_ps (IEEE) */
    return saturate((X * (a * X + b)) / (X * (c * X + d) + e));
}

static float linear_to_srgb(float x, int exact_gamma)   /* v4 :177-186 */
{
    x = saturate(x);
    if (x < 0.0031308f) return x * 12.92f;
    if (exact_gamma)   /* :184-185: 1.055f * pow_ps(rgb, 1 / 2.4f) - 0.055f; SVML pow_ps -> libm powf */
        return 1.055f * powf(x, 1.0f / 2.4f) - 0.055f;
    return fmaf(1.055f, fast_pow_gamma(x), -0.055f);   /* :182-183 fmsub */
}

uint32_t pto_tonemap_channel_ex(float linear, int32_t exact_aces, int32_t exact_gamma)
{
    const float c_exposure = 1.0f;
    const float t = exact_aces ? aces_exact(linear * c_exposure) : aces(linear * c_exposure);
    const float v = saturate(linear_to_srgb(t, exact_gamma)) * 255.f;
    const float r = rintf(v);   /* cvtps_epi32, round to nearest even (default MXCSR) */
    return (uint32_t)(int32_t)r & 0xFFu;
}

uint32_t pto_tonemap_channel(float linear) { return pto_tonemap_channel_ex(linear, 0, 0); }

static uint32_t pixel_ex(const float rgb[3], int32_t format, int32_t exact_aces, int32_t exact_gamma)
{
    const uint32_t r = pto_tonemap_channel_ex(rgb[0], exact_aces, exact_gamma);
    const uint32_t g = pto_tonemap_channel_ex(rgb[1], exact_aces, exact_gamma);
    const uint32_t b = pto_tonemap_channel_ex(rgb[2], exact_aces, exact_gamma);
    if (format == PTO_PIXEL_XRGB8) return (r << 16) | (g << 8) | b;               /* :1282-1285 */
    return 0xFF000000u | (b << 16) | (g << 8) | r;                               /* :1319-1323 */
}

uint32_t pto_tonemap_pixel(const float rgb[3], int32_t format) { return pixel_ex(rgb, format, 0, 0); }

/* The whole accumulator, interleaved RGB rows (row 0 = top), to packed pixels. */
void pto_tonemap_ex(const float* rgb, int32_t w, int32_t h, int32_t format, int32_t exact_aces, int32_t exact_gamma,
                    uint32_t* out)
{
    for (int64_t i = 0; i < (int64_t)w * h; ++i) out[i] = pixel_ex(rgb + 3 * i, format, exact_aces, exact_gamma);
}

void pto_tonemap(const float* rgb, int32_t w, int32_t h, int32_t format, uint32_t* out)
{
    pto_tonemap_ex(rgb, w, h, format, 0, 0, out);
}
