// include/demofox_path_tracing_mi355.h -- reference-shaped C++ surface of libpt_mi355.so.
//
// Same names, signatures and C++ linkage as the reference's renderer headers, so a reference host
// (Application.cpp:474 style) links against libpt_mi355.so instead of compiling the CPU renderer:
//   demofox_path_tracing_scalar.h:7      void DemofoxRenderScalar(f32*, i32, i32, i32)
//   demofox_path_tracing_simd.h:7        void DemofoxRenderSimd(f32*, i32, i32, i32)
//   demofox_path_tracing_simd_tiled.h:7  void DemofoxRenderSimdTiled(f32*, i32, i32, i32, i32, i32, i32, i32)
//   demofox_path_tracing_simd_tiled.cpp:473-489  RenderBufferInfo, RenderTileInfo, RenderTile(&, &)
//   texture.h:6-12, asset_loading.h:6       struct texture, texture LoadTexture(char*)
//   demofox_path_tracing_simt_textured.h:8  void DemofoxRenderSimtTextured(f32*, i32 x7, texture)
//   demofox_path_tracing_optimization_v4.h:21  void CopyOutputToFile(f32*, i32 x7, texture, void*)
//   asset_loading.h:8                          void WriteImage(char*, i32, i32, i32, void*)
// Like the reference (which __debugbreak()s on bad settings), these have no error return: on
// failure they print pt_last_error() to stderr and abort().
#pragma once
#include <stdint.h>
#include "pt_mi355.h"

typedef float f32;
typedef int32_t i32;

struct RenderBufferInfo {
    f32* BufferDataPtr;
    i32 BufferWidth;
    i32 BufferHeight;
    i32 NumChannels;
};

struct RenderTileInfo {
    i32 TileX, TileY;
    i32 TileWidth, TileHeight;
    i32 TileMinX, TileMaxX;
    i32 TileMinY, TileMaxY;
};

void DemofoxRenderScalar(f32* BufferOut, i32 Width, i32 Height, i32 NumChannels);
void DemofoxRenderSimd(f32* BufferOut, i32 Width, i32 Height, i32 NumChannels);
void DemofoxRenderSimdTiled(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY,
                            i32 TileWidth, i32 TileHeight, i32 NumChannels);
void RenderTile(RenderBufferInfo& BufferInfo, RenderTileInfo& TileInfo);

struct texture {
    f32* Data = 0;
    i32 Width = 0;
    i32 Height = 0;
    i32 Components = 3;
};

// Like stbi_loadf: Data == 0 when the file cannot be read (the reference does not check either).
texture LoadTexture(char* filename);
void DemofoxRenderSimtTextured(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY,
                               i32 TileWidth, i32 TileHeight, i32 NumChannels, texture Texture);

// asset_loading.h:7: six faces (px nx py ny pz nz) stacked vertically; Data == 0 on failure.
texture LoadCubemapTexture(char* filename[6]);

// demofox_path_tracing_optimization_v4.h:14-26 -- the shipping renderer (Application.cpp:474).
// DemofoxRenderOptV4 advances v4's iFrame, renders every tile into the tiled accumulator and, with
// OUTPUT_TO_SCREEN (pt_v4_config.output_to_screen, default 1) and ScreenBufferData != 0, writes the
// BufferWidth x BufferHeight XRGB8 screen pixels (OutputToScreen v4 :1260-1295).  The env-map mode
// and sampling switches of global_preprocessor_flags.h are pt_v4_set_config() (default: equirect,
// random-jitter texel sampling, rejection-sampled unit vectors).
void DemofoxRenderOptV4(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY,
                        i32 TileWidth, i32 TileHeight, i32 NumChannels, texture Texture, void* ScreenBufferData);
void InitializeGlobalRenderResources();
void ReinitializeRenderTileData();

// The post-process of the tiled accumulator into 32-bit file pixels (bytes R, G, B, A = 255):
// ACES + sRGB + 8-bit, v4 :1297-1331, after advancing v4's iFrame (:1738).  (Through its pool's
// callback mix-up (v4 :1588 vs :1756) the reference's function may also re-render tiles; only the
// documented post-process is performed here.)  Texture is unused, as in the reference.
void CopyOutputToFile(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY, i32 TileWidth,
                      i32 TileHeight, i32 NumChannels, texture Texture, void* ScreenBufferData);
// stbi_write_bmp: a 24-bit BMP (asset_loading.cpp:48-54).  Prints pt_last_error() on failure.
void WriteImage(char* filename, i32 width, i32 height, i32 components, void* data);
