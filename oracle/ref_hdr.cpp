// ref_hdr.cpp -- oracle-side driver around the reference's vendored stb_image v2.26
// (CPUPerformanceRayTracer/stb_image.h, compiled where it lies by oracle/build_ref.sh).
// Decodes an .hdr exactly as LoadTexture does (asset_loading.cpp:9-16: flip on load, stbi_loadf,
// req_comp 0) and writes int32 {width, height, components} followed by the f32 texels.
// Test infrastructure only (tests/test_texture.py): the product decoder is csrc/pt_texture.cpp.
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"
#include <stdio.h>

int main(int argc, char** argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: ref_hdr IN.hdr OUT.bin\n");
        return 2;
    }
    stbi_set_flip_vertically_on_load(1);
    int w = 0, h = 0, c = 0;
    float* d = stbi_loadf(argv[1], &w, &h, &c, 0);
    if (!d) {
        fprintf(stderr, "stbi_loadf: %s\n", stbi_failure_reason());
        return 1;
    }
    FILE* f = fopen(argv[2], "wb");
    if (!f) return 1;
    const int hdr[3] = {w, h, c};
    fwrite(hdr, sizeof(int), 3, f);
    fwrite(d, sizeof(float), (size_t)w * h * c, f);
    fclose(f);
    stbi_image_free(d);
    return 0;
}
