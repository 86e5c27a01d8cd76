// pt_output.hip -- the output stage: linear HDR accumulator -> 8-bit display / file pixels.
//
// Reference (CPUPerformanceRayTracer/demofox_path_tracing_optimization_v4.cpp): OutputToScreen
// :1260-1295 / OutputToFile :1297-1331, called per tile by CopyOutputToFile :1729-1760 and the frame
// loop; the per-channel conversion (ACESFilm :165-175 -> LinearToSRGB :177-186 -> 8 bits) and its
// numerics are in pt_tonemap.h, shared with the render kernels' fused presentation
// (pt_render_device_present: a pixel's value written at its last fold, no second pass).
// One thread per pixel, any accumulator layout; 12 B read + 4 B written per pixel: HBM-bound.
#include "pt_output.h"
#include "pt_tonemap.h"
#include <algorithm>

namespace {

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
        j.out[p] = pt_tone::pack<FAST_ACES, FAST_GAMMA>(j.accum[base], j.accum[base + cs], j.accum[base + 2 * cs],
                                                        j.format == PT_PIXEL_XRGB8);
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
