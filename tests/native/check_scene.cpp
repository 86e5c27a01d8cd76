// tests/native/check_scene.cpp -- the kernel's compile-time scene table (DemofoxScene, pt_scene.h)
// must equal, bit for bit, the scene the host derives with the reference's own f32 operations
// (pt_build_demofox_scene: translation adds, normalize(cross(c-a, c-b)), r*r).
#include "../../cpuperformanceraytracer_amd/csrc/pt_scene.h"
#include <cstdio>
#include <cstring>

static int bad = 0;
static void eq(float a, float b, const char* what, int i, int j)
{
    if (std::memcmp(&a, &b, 4)) {
        std::printf("mismatch %s[%d][%d]: table %a host %a\n", what, i, j, a, b);
        ++bad;
    }
}

int main()
{
    PtScene s;
    const float amb[3] = {0.1f, 0.1f, 0.1f};
    pt_build_demofox_scene(&s, amb);
    for (int q = 0; q < PT_NQUADS; ++q) {
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 3; ++j) eq(DemofoxScene::qv[q][k][j], s.qv[q][k][j], "qv", q, k * 3 + j);
        for (int j = 0; j < 3; ++j) eq(DemofoxScene::qn[q][j], s.qn[q][j], "qn", q, j);
    }
    for (int k = 0; k < PT_NSPHERES; ++k) {
        for (int j = 0; j < 4; ++j) eq(DemofoxScene::sph[k][j], s.sph[k][j], "sph", k, j);
        eq(DemofoxScene::sph_r2[k], s.sph_r2[k], "sph_r2", k, 0);
    }
    std::printf("scene table %s\n", bad ? "MISMATCH" : "ok");
    return bad ? 1 : 0;
}
