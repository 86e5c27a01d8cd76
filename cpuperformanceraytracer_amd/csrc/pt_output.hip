// pt_output.hip -- the output stage: linear HDR accumulator -> 8-bit display / file pixels.
//
// Reference (CPUPerformanceRayTracer/demofox_path_tracing_optimization_v4.cpp; both branches of
// global_preprocessor_flags.h:62-63, USE_FAST_APPROXIMATE_GAMMA / USE_FAST_APPROXIMATE_ACES_TONEMAP):
//   OutputToScreen :1260-1295 / OutputToFile :1297-1331, called per tile by CopyOutputToFile
//   :1729-1760 and the frame loop: ACESFilm :165-175 -> LinearToSRGB :177-186 (fast_pow_gamma
//   :144-155) -> saturate * 255 -> cvtps_epi32 -> packed u32.
// One thread per pixel, any accumulator layout; 12 B read + 4 B written per pixel: HBM-bound
// (fused into no other pass: it runs once per presented frame, not per rendered frame).
// Numerics: the reference's operations in its order, fmadd/fmsub fused (__builtin_fmaf), sqrt
// correctly rounded (guarded fast path), MAXPS/MINPS NaN rules, round-to-nearest-even conversion.  `rcp` is
// _mm256_rcp_ps in the reference, whose table is CPU-model specific; here it is the correctly
// rounded 1/x (as in the oracle, oracle/pt_oracle_output.c): at most 1 LSB from any x86 run.
#include "pt_output.h"
#include "pt_exactmath.h"
#include "pt_libmf.h"
#include <algorithm>

namespace {

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

template <int LAYOUT, bool FAST_ACES, bool FAST_GAMMA>
__global__ __launch_bounds__(256) void pt_tonemap_kernel(PtToneJob j)
{
    const uint32_t npix = (uint32_t)j.width * (uint32_t)j.height;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += gridDim.x * blockDim.x) {
        const uint32_t y = p / (uint32_t)j.width, x = p - y * (uint32_t)j.width;
        size_t base;
        size_t cs = 8;   // channel stride
        if (LAYOUT == PT_LAYOUT_INTERLEAVED) {
            base = (size_t)p * 3u;
            cs = 1;
        } else if (LAYOUT == PT_LAYOUT_PLANAR8) {
            base = ((size_t)y * j.width + (x & ~7u)) * 3u + (x & 7u);
        } else {   // tiled planar8 (RenderTile, simd_tiled.cpp:499-531; v4 :1266-1290)
            const uint32_t tx = x / (uint32_t)j.tile_w, ty = y / (uint32_t)j.tile_h;
            const uint32_t lx = x - tx * j.tile_w, ly = y - ty * j.tile_h;
            base = (size_t)ty * j.tile_h * j.width * 3u + (size_t)tx * j.tile_w * j.tile_h * 3u +
                   ((size_t)ly * j.tile_w + (lx & ~7u)) * 3u + (lx & 7u);
        }
        const uint32_t r = channel<FAST_ACES, FAST_GAMMA>(j.accum[base]), g = channel<FAST_ACES, FAST_GAMMA>(j.accum[base + cs]),
                       b = channel<FAST_ACES, FAST_GAMMA>(j.accum[base + 2 * cs]);
        j.out[p] = j.format == PT_PIXEL_XRGB8 ? ((r << 16) | (g << 8) | b)        // OutputToScreen :1282-1285
                                              : (0xFF000000u | (b << 16) | (g << 8) | r);   // OutputToFile :1319-1323
    }
}

template <int LAYOUT>
hipError_t launch_layout(const PtToneJob& j, unsigned blocks, hipStream_t st)
{
    if (j.fast_aces && j.fast_gamma) hipLaunchKernelGGL((pt_tonemap_kernel<LAYOUT, true, true>), dim3(blocks), dim3(256), 0, st, j);
    else if (j.fast_aces) hipLaunchKernelGGL((pt_tonemap_kernel<LAYOUT, true, false>), dim3(blocks), dim3(256), 0, st, j);
    else if (j.fast_gamma) hipLaunchKernelGGL((pt_tonemap_kernel<LAYOUT, false, true>), dim3(blocks), dim3(256), 0, st, j);
    else hipLaunchKernelGGL((pt_tonemap_kernel<LAYOUT, false, false>), dim3(blocks), dim3(256), 0, st, j);
    return hipGetLastError();
}

}  // namespace

hipError_t pt_launch_tonemap(const PtToneJob& j, hipStream_t st)
{
    if (j.width <= 0 || j.height <= 0) return hipSuccess;
    if (!j.accum || !j.out) return hipErrorInvalidValue;
    const long npix = (long)j.width * j.height;
    const unsigned blocks = (unsigned)std::min<long>((npix + 255) / 256, 256L * 16);
    switch (j.layout) {
        case PT_LAYOUT_INTERLEAVED: return launch_layout<PT_LAYOUT_INTERLEAVED>(j, blocks, st);
        case PT_LAYOUT_PLANAR8: return launch_layout<PT_LAYOUT_PLANAR8>(j, blocks, st);
        case PT_LAYOUT_TILED_PLANAR8:
            if (j.tile_w <= 0 || j.tile_h <= 0) return hipErrorInvalidValue;
            return launch_layout<PT_LAYOUT_TILED_PLANAR8>(j, blocks, st);
        default: return hipErrorInvalidValue;
    }
}

// ---- PT_FLAG_GATHER_ROOT: a device's rows into the root's accumulator (pt_output.h) ----------------
namespace {

template <bool TILED>
__global__ __launch_bounds__(256) void pt_scatter_rows_kernel(PtScatterJob j)
{
    const int32_t rowf = j.width * 3;   // floats of one image row in every layout
    for (int32_t k = blockIdx.x; k < j.nrows; k += gridDim.x) {
        const int32_t Y = j.dev + k * j.ndev;
        if constexpr (!TILED) {
            const float* s = j.src + (size_t)k * rowf;
            float* d = j.dst + (size_t)Y * rowf;
            for (int32_t i = threadIdx.x; i < rowf; i += blockDim.x) d[i] = s[i];
        } else {   // simd_tiled.cpp:499-502 offsets: the row's segment in each tile of its tile row
            const int32_t ty = Y / j.tile_h, ly = Y - ty * j.tile_h, segf = j.tile_w * 3;
            const size_t base = (size_t)ty * j.tile_h * rowf + (size_t)ly * segf;
            const size_t tilef = (size_t)j.tile_w * j.tile_h * 3;
            for (int32_t i = threadIdx.x; i < rowf; i += blockDim.x) {
                const int32_t tx = i / segf, r = i - tx * segf;
                const size_t off = base + (size_t)tx * tilef + r;
                j.dst[off] = j.src[off];
            }
        }
    }
}

}  // namespace

hipError_t pt_launch_scatter_rows(const PtScatterJob& j, hipStream_t st)
{
    if (j.nrows <= 0 || j.width <= 0) return hipSuccess;
    if (!j.src || !j.dst || j.ndev < 1 || j.dev < 0 || j.dev >= j.ndev) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)std::min<int32_t>(j.nrows, 2048);
    if (j.layout == PT_LAYOUT_TILED_PLANAR8) {
        if (j.tile_w <= 0 || j.tile_h <= 0) return hipErrorInvalidValue;
        hipLaunchKernelGGL((pt_scatter_rows_kernel<true>), dim3(blocks), dim3(256), 0, st, j);
    } else {
        hipLaunchKernelGGL((pt_scatter_rows_kernel<false>), dim3(blocks), dim3(256), 0, st, j);
    }
    return hipGetLastError();
}
