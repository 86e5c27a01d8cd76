// ref_bmp.cpp -- oracle-side driver around the reference's vendored stb_image_write v1.15
// (CPUPerformanceRayTracer/stb_image_write.h, compiled where it lies by oracle/build_ref.sh).
// Writes `raw` (w*h*comp bytes) as BMP exactly as WriteImage does (asset_loading.cpp:48-54).
// Test infrastructure only (tests/test_bmp.py): the product writer is csrc/pt_texture.cpp.
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

int main(int argc, char** argv)
{
    if (argc != 6) {
        fprintf(stderr, "usage: ref_bmp IN.raw W H COMP OUT.bmp\n");
        return 2;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]), comp = atoi(argv[4]);
    std::vector<unsigned char> px((size_t)(w > 0 ? w : 0) * (h > 0 ? h : 0) * comp + 1);
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    const size_t n = fread(px.data(), 1, px.size() - 1, f);
    fclose(f);
    if (n != px.size() - 1) return 1;
    return stbi_write_bmp(argv[5], w, h, comp, px.data()) ? 0 : 1;
}
