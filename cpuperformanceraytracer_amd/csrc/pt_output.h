// pt_output.h -- internal interface of the output-stage kernel (pt_output.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pt_kernel.h"

#include "../../include/pt_mi355.h"   // PT_PIXEL_RGBA8 / PT_PIXEL_XRGB8

struct PtToneJob {
    const float* accum;       // device accumulator (PtLayout)
    int32_t width, height;
    int32_t layout;
    int32_t tile_w, tile_h;   // PT_LAYOUT_TILED_PLANAR8
    uint32_t* out;            // device, width * height packed pixels, row 0 = top
    int32_t format;           // PT_PIXEL_*
    int32_t fast_aces;        // USE_FAST_APPROXIMATE_ACES_TONEMAP (else the unfused fit with '/')
    int32_t fast_gamma;       // USE_FAST_APPROXIMATE_GAMMA (else 1.055 powf(x, 1/2.4) - 0.055)
};

hipError_t pt_launch_tonemap(const PtToneJob& job, hipStream_t stream);

// Several devices, PT_FLAG_GATHER_ROOT: device `dev` of `ndev` writes the global rows it owns
// (Y = dev + k * ndev) from its mirror into the root device's full-size accumulator -- remote stores
// over xGMI (peer access), each device over its own link.  Row layouts: the mirror holds the rows
// compactly; tiled layout: the mirror is full-size (same offsets as the root's).
struct PtScatterJob {
    const float* src;         // this device's mirror
    float* dst;               // the root's W x H x 3 buffer
    int32_t width, height;
    int32_t layout;
    int32_t tile_w, tile_h;   // PT_LAYOUT_TILED_PLANAR8
    int32_t dev, ndev, nrows; // owned rows
};

hipError_t pt_launch_scatter_rows(const PtScatterJob& job, hipStream_t stream);
