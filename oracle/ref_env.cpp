// oracle/ref_env.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
//
// Runs the reference's own per-lane body of EquirectangularTextureSample (texture.cpp:111-135,
// config 4's miss term, called from demofox_path_tracing_simt_textured.cpp:408) on a list of
// directions.  oracle/build_ref.sh extracts, into a temporary directory:
//   ref_texture_fetch.inc : the mathlib.h scalar subset + struct texture (texture.h:6-12) +
//                           TexelFetch (texture.cpp:6-14)
//   ref_env_lane_body.inc : texture.cpp:111-135 verbatim (the body of `for (lane ...)`)
// and compiles this wrapper against them.  The wrapper only supplies what the loop header of
// texture.cpp:104-110 supplies to the body -- `lane`, `Direction` (one lane's f32x3) and the
// `Result` whose `.x/.y/.z.m256_f32[lane]` the body writes -- so no arithmetic is ours.
//
//   ref_env TEX.f32 W H DIRS.f32 OUT.f32
//     TEX.f32 : H x W x 3 f32 (row 0 = the first row in memory, as LoadTexture leaves it)
//     DIRS.f32: N x 3 f32 directions;  OUT.f32: N x 3 f32 texels (0 outside [0,1) uv)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ref_texture_fetch.inc"

namespace {
struct lane_channel { f32 m256_f32[8]; };
struct lane_result { lane_channel x, y, z; };

void sample_one(texture texture, f32x3 Direction, f32* out)
{
    lane_result Result;
    u32 lane = 0;
#include "ref_env_lane_body.inc"
    out[0] = Result.x.m256_f32[lane];
    out[1] = Result.y.m256_f32[lane];
    out[2] = Result.z.m256_f32[lane];
}

std::vector<f32> read_f32(const char* path)
{
    std::vector<f32> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    f32 x;
    while (std::fread(&x, sizeof x, 1, f) == 1) v.push_back(x);
    std::fclose(f);
    return v;
}
}  // namespace

int main(int argc, char** argv)
{
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s TEX.f32 W H DIRS.f32 OUT.f32\n", argv[0]);
        return 2;
    }
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
    std::vector<f32> tex = read_f32(argv[1]);
    std::vector<f32> dirs = read_f32(argv[4]);
    if (w <= 0 || h <= 0 || tex.size() != (size_t)w * h * 3 || dirs.size() % 3) return 3;
    texture t;
    t.Data = tex.data();
    t.Width = w;
    t.Height = h;
    t.Components = 3;
    const size_t n = dirs.size() / 3;
    std::vector<f32> out(n * 3);
    for (size_t i = 0; i < n; ++i)
        sample_one(t, f32x3{dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]}, &out[3 * i]);
    FILE* f = std::fopen(argv[5], "wb");
    if (!f) return 4;
    std::fwrite(out.data(), sizeof(f32), out.size(), f);
    std::fclose(f);
    return 0;
}
