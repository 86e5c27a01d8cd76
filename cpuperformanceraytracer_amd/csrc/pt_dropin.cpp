// pt_dropin.cpp -- the reference's renderer entry points (C++ linkage, same signatures) forwarding
// to the C ABI.  See include/demofox_path_tracing_mi355.h.
#include "../../include/demofox_path_tracing_mi355.h"
#include <stdio.h>
#include <stdlib.h>

static void pt_check(int rc, const char* what)
{
    if (rc == PT_OK) return;
    fprintf(stderr, "%s: %s (rc=%d)\n", what, pt_last_error(), rc);
    abort();   // the reference __debugbreak()s on invalid settings (Application.cpp:59,69,79,89)
}

void DemofoxRenderScalar(f32* BufferOut, i32 Width, i32 Height, i32 NumChannels)
{
    pt_check(pt_render_scalar(BufferOut, Width, Height, NumChannels), "DemofoxRenderScalar");
}

void DemofoxRenderSimd(f32* BufferOut, i32 Width, i32 Height, i32 NumChannels)
{
    pt_check(pt_render_simd(BufferOut, Width, Height, NumChannels), "DemofoxRenderSimd");
}

void DemofoxRenderSimdTiled(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY,
                            i32 TileWidth, i32 TileHeight, i32 NumChannels)
{
    pt_check(pt_render_simd_tiled(BufferOut, BufferWidth, BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight,
                                  NumChannels),
             "DemofoxRenderSimdTiled");
}

void RenderTile(RenderBufferInfo& BufferInfo, RenderTileInfo& TileInfo)
{
    const pt_buffer_info b = {BufferInfo.BufferDataPtr, BufferInfo.BufferWidth, BufferInfo.BufferHeight,
                              BufferInfo.NumChannels};
    const pt_tile_info t = {TileInfo.TileX,    TileInfo.TileY,    TileInfo.TileWidth, TileInfo.TileHeight,
                            TileInfo.TileMinX, TileInfo.TileMaxX, TileInfo.TileMinY,  TileInfo.TileMaxY};
    pt_check(pt_render_tile(&b, &t), "RenderTile");
}

texture LoadTexture(char* filename)
{
    texture t;
    pt_texture p;
    if (pt_load_texture(filename, &p) != PT_OK) {
        fprintf(stderr, "LoadTexture: %s\n", pt_last_error());
        return t;
    }
    t.Data = p.data;
    t.Width = p.width;
    t.Height = p.height;
    t.Components = p.components;
    return t;
}

void DemofoxRenderSimtTextured(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY,
                               i32 TileWidth, i32 TileHeight, i32 NumChannels, texture Texture)
{
    const pt_texture p = {Texture.Data, Texture.Width, Texture.Height, Texture.Components};
    pt_check(pt_render_simt_textured(BufferOut, BufferWidth, BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight,
                                     NumChannels, &p),
             "DemofoxRenderSimtTextured");
}

texture LoadCubemapTexture(char* filename[6])
{
    texture t;
    pt_texture p;
    if (pt_load_cubemap_texture(filename, &p) != PT_OK) {
        fprintf(stderr, "LoadCubemapTexture: %s\n", pt_last_error());
        return t;
    }
    t.Data = p.data;
    t.Width = p.width;
    t.Height = p.height;
    t.Components = p.components;
    return t;
}

void DemofoxRenderOptV4(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY, i32 TileWidth,
                        i32 TileHeight, i32 NumChannels, texture Texture, void* ScreenBufferData)
{
    const pt_texture p = {Texture.Data, Texture.Width, Texture.Height, Texture.Components};
    pt_check(pt_render_opt_v4(BufferOut, BufferWidth, BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight,
                              NumChannels, Texture.Data ? &p : nullptr, ScreenBufferData),
             "DemofoxRenderOptV4");
}

void InitializeGlobalRenderResources() { pt_check(pt_v4_initialize_global_render_resources(), "InitializeGlobalRenderResources"); }

void ReinitializeRenderTileData() { pt_check(pt_v4_reinitialize_render_tile_data(), "ReinitializeRenderTileData"); }

void CopyOutputToFile(f32* BufferOut, i32 BufferWidth, i32 BufferHeight, i32 NumTilesX, i32 NumTilesY, i32 TileWidth,
                      i32 TileHeight, i32 NumChannels, texture Texture, void* ScreenBufferData)
{
    (void)Texture;
    pt_check(pt_copy_output_to_file(BufferOut, BufferWidth, BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight,
                                    NumChannels, ScreenBufferData),
             "CopyOutputToFile");
}

void WriteImage(char* filename, i32 width, i32 height, i32 components, void* data)
{
    if (pt_write_bmp(filename, width, height, components, data) != PT_OK)   // stbi_write_bmp: no abort
        fprintf(stderr, "WriteImage: %s\n", pt_last_error());
}
