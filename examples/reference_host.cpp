// examples/reference_host.cpp -- a reference-shaped C++ host linked against libpt_mi355.so.
//
// Mirrors ApplicationState::RenderOffline / Render (CPUPerformanceRayTracer/Application.cpp:400-477)
// using ONLY the reference's function names and types, from include/demofox_path_tracing_mi355.h:
// InitializeGlobalRenderResources, DemofoxRenderOptV4 / DemofoxRenderSimdTiled / DemofoxRenderScalar,
// CopyOutputToFile and WriteImage, plus the flags bridge (pt_flags.h) for -D overrides of the
// reference's global_preprocessor_flags.h switches.  The env map is generated in memory (deterministic hash pattern) so
// the program needs no texture file; tests/test_gpu_host.py renders the same with the oracle.
//
//   reference_host <renderer: scalar|tiled|v4> <width> <height> <frames> <out.f32> [out.bmp]
#include "demofox_path_tracing_mi355.h"
// The reference's compile-time switches (global_preprocessor_flags.h) -- given with -D here -- are
// applied to the backend by the bridge header (include/pt_flags.h).
#include "pt_flags.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

static texture MakeTexture(i32 w, i32 h)   // T[i] = (u32)(i * 2654435761) / 2^32 * 4 (+ 0.01)
{
    texture t;
    t.Width = w;
    t.Height = h;
    t.Components = 3;
    t.Data = (f32*)malloc(sizeof(f32) * (size_t)w * h * 3);
    for (uint32_t i = 0; i < (uint32_t)(w * h * 3); ++i)
        t.Data[i] = (f32)(i * 2654435761u) * (4.0f / 4294967296.0f) + 0.01f;
    return t;
}

int main(int argc, char** argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s scalar|tiled|v4 W H frames out.f32 [out.bmp]\n", argv[0]);
        return 2;
    }
    const char* renderer = argv[1];
    const i32 W = atoi(argv[2]), H = atoi(argv[3]), frames = atoi(argv[4]);
    const i32 NumTilesX = 10, NumTilesY = 15;   // global_preprocessor_flags.h:85-86
    const i32 TileWidth = W / NumTilesX, TileHeight = H / NumTilesY;
    std::vector<f32> RenderTarget((size_t)W * H * 3, 0.0f);   // BackBuffer.Resize (Application.cpp:142-151)
    std::vector<uint32_t> Screen((size_t)W * H, 0);
    texture Texture = MakeTexture(128, 64);

    if (pt_apply_global_preprocessor_flags() != PT_OK) {   // the host's global_preprocessor_flags.h
        fprintf(stderr, "flags: %s\n", pt_last_error());
        return 1;
    }
    InitializeGlobalRenderResources();   // Application.cpp:413
    for (i32 f = 0; f < frames; ++f) {   // Render() per frame (Application.cpp:460-477)
        if (!strcmp(renderer, "v4"))
            DemofoxRenderOptV4(RenderTarget.data(), W, H, NumTilesX, NumTilesY, TileWidth, TileHeight, 3, Texture,
                               Screen.data());
        else if (!strcmp(renderer, "tiled"))
            DemofoxRenderSimdTiled(RenderTarget.data(), W, H, NumTilesX, NumTilesY, TileWidth, TileHeight, 3);
        else
            DemofoxRenderScalar(RenderTarget.data(), W, H, 3);
    }
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(RenderTarget.data(), sizeof(f32), RenderTarget.size(), f) != RenderTarget.size()) {
        fprintf(stderr, "cannot write %s\n", argv[5]);
        return 1;
    }
    fclose(f);
    if (argc > 6 && strcmp(renderer, "scalar")) {   // Application.cpp:390-396: CopyOutputToFile + WriteImage
        std::vector<uint32_t> FilePixels((size_t)W * H);
        CopyOutputToFile(RenderTarget.data(), W, H, NumTilesX, NumTilesY, TileWidth, TileHeight, 3, Texture,
                         FilePixels.data());
        WriteImage(argv[6], W, H, 4, FilePixels.data());
    }
    free(Texture.Data);
    printf("rendered %d frames of %dx%d with %s\n", frames, W, H, renderer);
    return 0;
}
