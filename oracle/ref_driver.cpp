// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
//
// Thin driver around the reference's own, unmodified scalar path tracer
// (demofox_path_tracing_scalar.cpp:785-820, DemofoxRenderScalar), compiled in place from
// /root/reference by oracle/build_ref.sh.  This file is ours; no reference source is copied.
//
// Two products are built from it:
//   oracle/_ref/ref_scalar        : CLI  `ref_scalar W H FRAMES OUT.f32` -> raw interleaved RGB f32
//                                   (fresh process => the reference's `static f32 iFrame` starts at 0,
//                                   exactly like one run of the reference host).
//   oracle/_ref/libref_scalar.so  : C ABI `ref_render_scalar(buf, W, H, frames)` used as the
//                                   "reference" CPU baseline timing in bench.py.  NOTE the static
//                                   frame counter inside the reference keeps counting across calls.
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef float f32;
typedef int32_t i32;

// demofox_path_tracing_scalar.h:7 (C++ linkage, as declared by the reference)
void DemofoxRenderScalar(f32* BufferOut, i32 Width, i32 Height, i32 NumChannels);

extern "C" int ref_render_scalar(float* buf, int w, int h, int frames)
{
    for (int f = 0; f < frames; ++f) DemofoxRenderScalar(buf, w, h, 3);
    return 0;
}

#ifdef REF_DRIVER_MAIN
int main(int argc, char** argv)
{
    if (argc != 5) {
        std::fprintf(stderr, "usage: %s W H FRAMES OUT.f32\n", argv[0]);
        return 2;
    }
    const int w = std::atoi(argv[1]), h = std::atoi(argv[2]), frames = std::atoi(argv[3]);
    if (w <= 0 || h <= 0 || frames <= 0) return 2;
    std::vector<float> buf((size_t)w * h * 3, 0.0f);   // zeroed like Application.cpp:142-151
    ref_render_scalar(buf.data(), w, h, frames);
    FILE* f = std::fopen(argv[4], "wb");
    if (!f) return 3;
    std::fwrite(buf.data(), sizeof(float), buf.size(), f);
    std::fclose(f);
    return 0;
}
#endif
