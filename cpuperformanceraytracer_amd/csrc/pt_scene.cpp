// pt_scene.cpp -- host construction of the device scene table (see pt_scene.h).
// Compiled with -ffp-contract=off: every f32 op below rounds once, exactly like the reference's
// per-call evaluation of the same expressions in TestSceneTrace (demofox_path_tracing_scalar.cpp).
#include "pt_scene.h"
#include <math.h>
#include <string.h>

namespace {
// TestSceneTrace, scalar.cpp:194-262 (vertices before sceneTranslation)
const float kQuad[PT_NQUADS][4][3] = {
    {{-12.6f, -12.6f, 25.0f}, {12.6f, -12.6f, 25.0f}, {12.6f, 12.6f, 25.0f}, {-12.6f, 12.6f, 25.0f}},        // back wall
    {{-12.6f, -12.45f, 25.0f}, {12.6f, -12.45f, 25.0f}, {12.6f, -12.45f, 15.0f}, {-12.6f, -12.45f, 15.0f}},  // floor
    {{-12.6f, 12.5f, 25.0f}, {12.6f, 12.5f, 25.0f}, {12.6f, 12.5f, 15.0f}, {-12.6f, 12.5f, 15.0f}},          // ceiling
    {{-12.5f, -12.6f, 25.0f}, {-12.5f, -12.6f, 15.0f}, {-12.5f, 12.6f, 15.0f}, {-12.5f, 12.6f, 25.0f}},      // left
    {{12.5f, -12.6f, 25.0f}, {12.5f, -12.6f, 15.0f}, {12.5f, 12.6f, 15.0f}, {12.5f, 12.6f, 25.0f}},          // right
    {{-5.0f, 12.4f, 22.5f}, {5.0f, 12.4f, 22.5f}, {5.0f, 12.4f, 17.5f}, {-5.0f, 12.4f, 17.5f}},              // light
};
// scalar.cpp:270, 276, 282
const float kSphere[PT_NSPHERES][4] = {{-9.0f, -9.5f, 20.0f, 3.0f}, {0.0f, -9.5f, 20.0f, 3.0f}, {9.0f, -9.5f, 20.0f, 3.0f}};
// scalar.cpp:200-285 (light albedo 0; sphere 3 = (0.75, 0.9, 0.9) in the scalar file, :284)
const float kAlbedo[PT_NPRIMS][3] = {{0.7f, 0.7f, 0.7f}, {0.7f, 0.7f, 0.7f}, {0.7f, 0.7f, 0.7f},
                                     {0.7f, 0.1f, 0.1f}, {0.1f, 0.7f, 0.1f}, {0.0f, 0.0f, 0.0f},
                                     {0.9f, 0.9f, 0.75f}, {0.9f, 0.75f, 0.9f}, {0.75f, 0.9f, 0.9f}};
}  // namespace

void pt_build_demofox_scene(PtScene* s, const float ambient[3])
{
    memset(s, 0, sizeof(*s));
    const float tr[3] = {0.0f, 0.0f, 10.0f};   // sceneTranslation, scalar.cpp:189
    for (int q = 0; q < PT_NQUADS; ++q) {
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 3; ++j) s->qv[q][k][j] = kQuad[q][k][j] + tr[j];
        const float* a = s->qv[q][0];
        const float* b = s->qv[q][1];
        const float* c = s->qv[q][2];
        const float e1[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
        const float e2[3] = {c[0] - b[0], c[1] - b[1], c[2] - b[2]};
        const float cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const float inv = 1.0f / sqrtf((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
        for (int j = 0; j < 3; ++j) s->qn[q][j] = cr[j] * inv;
    }
    for (int k = 0; k < PT_NSPHERES; ++k) {
        for (int j = 0; j < 3; ++j) s->sph[k][j] = kSphere[k][j] + tr[j];
        s->sph[k][3] = kSphere[k][3] + 0.0f;                 // sceneTranslation4.w = 0
        s->sph_r2[k] = s->sph[k][3] * s->sph[k][3];
    }
    for (int p = 0; p < PT_NPRIMS; ++p)
        for (int j = 0; j < 3; ++j) s->albedo[p][j] = kAlbedo[p][j];
    s->emissive[5][0] = 1.0f * 20.0f;                        // mul(f32x3{1.0f, 0.9f, 0.7f}, 20.0f), :266
    s->emissive[5][1] = 0.9f * 20.0f;
    s->emissive[5][2] = 0.7f * 20.0f;
    for (int j = 0; j < 3; ++j) s->ambient[j] = ambient[j];
    s->cam_dist = 1.0f / tanf(PT_FOV_DEG * 0.5f * PT_PI / 180.0f);
}
