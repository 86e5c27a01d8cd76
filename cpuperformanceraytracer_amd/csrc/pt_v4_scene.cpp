// pt_v4_scene.cpp -- host side of the v4 scene: InitializeScene (v4 :1403-1496), PrecomputeQuadData
// (:269-320) and AddMaterialToScene (:1368-1388), evaluated once per scene with the reference's f32
// operations (fused where it wrote fmadd/fmsub: cross mathlib.h:770-778, dot :145).  The kernel reads
// the resulting tables; nothing per pixel is precomputed beyond what the reference precomputes.
#include "pt_v4.h"
#include "pt_v4_default_scene.h"
#include <cmath>
#include <cstring>

namespace {

struct F3 {
    float x, y, z;
};
F3 f3(const float* p) { return {p[0], p[1], p[2]}; }
F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
F3 neg(F3 a) { return {-a.x, -a.y, -a.z}; }
float dot(F3 u, F3 v) { return std::fma(u.x, v.x, std::fma(u.y, v.y, u.z * v.z)); }
F3 cross(F3 u, F3 v)
{
    return {std::fma(u.y, v.z, -(u.z * v.y)), std::fma(u.z, v.x, -(u.x * v.z)), std::fma(u.x, v.y, -(u.y * v.x))};
}
F3 div(F3 a, float d) { return {a.x / d, a.y / d, a.z / d}; }
void put(float* o, F3 a)
{
    o[0] = a.x;
    o[1] = a.y;
    o[2] = a.z;
}

}  // namespace

void pt_v4_default_scene_desc(PtV4SceneDesc* d)
{
    std::memset(d, 0, sizeof(*d));
    const float T[3] = {0.0f, 0.0f, 10.0f};   // sceneTranslation :1407
    static const float quads[4][4][3] = {
        {{-25.0f, -12.5f, 5.0f}, {25.0f, -12.5f, 5.0f}, {25.0f, -12.5f, -5.0f}, {-25.0f, -12.5f, -5.0f}},  // floor :1415
        {{-25.0f, -1.5f, 5.0f}, {25.0f, -1.5f, 5.0f}, {25.0f, -10.5f, 5.0f}, {-25.0f, -10.5f, 5.0f}},    // stripes :1428 (not translated)
        {{-7.5f, 12.5f, 5.0f}, {7.5f, 12.5f, 5.0f}, {7.5f, 12.5f, -5.0f}, {-7.5f, 12.5f, -5.0f}},        // ceiling :1446
        {{-5.0f, 12.4f, 2.5f}, {5.0f, 12.4f, 2.5f}, {5.0f, 12.4f, -2.5f}, {-5.0f, 12.4f, -2.5f}},        // light :1461
    };
    static const float albedo[4] = {0.7f, 0.35f, 0.7f, 0.0f};
    for (int i = 0; i < 4; ++i) {
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 3; ++j) d->quad[i][k][j] = quads[i][k][j] + (i == 1 ? 0.0f : T[j]);
        PtV4Mat& m = d->mat[d->nmat++];   // SceneMaterial NewMaterial{ 0 }: IOR 0
        m.albedo[0] = m.albedo[1] = m.albedo[2] = albedo[i];
        if (i == 3) {   // (1.0, 0.9, 0.7) * 20 (:1469)
            m.emissive[0] = 1.0f * 20.0f;
            m.emissive[1] = 0.9f * 20.0f;
            m.emissive[2] = 0.7f * 20.0f;
        }
    }
    d->nquads = 4;
    for (int i = 0; i < 7; ++i) {   // c_numSpheres (:1474-1495), translated by sceneTranslation4
        float* p = d->sphere[d->nspheres++];
        p[0] = (-18.0f + 6.0f * (float)i) + 0.0f;
        p[1] = -8.0f + 0.0f;
        p[2] = 0.0f + 10.0f;
        p[3] = 2.8f + 0.0f;
        const float r = (((float)i) / (float)(7 - 1)) * 0.5f;
        PtV4Mat& m = d->mat[d->nmat++];
        m.spec_chance = 0.02f;
        m.ior = 1.1f;
        m.refr_chance = 1.0f;
        m.albedo[0] = 0.9f;
        m.albedo[1] = 0.25f;
        m.albedo[2] = 0.25f;
        m.refr_color[0] = 0.0f;
        m.refr_color[1] = 0.5f;
        m.refr_color[2] = 1.0f;
        m.spec_color[0] = m.spec_color[1] = m.spec_color[2] = 1.0f * 0.8f;
        m.spec_rough = r;
        m.refr_rough = r;
    }
}

int pt_v4_build_scene(const PtV4SceneDesc* d, PtV4Scene* s)
{
    if (d->nquads < 0 || d->nspheres < 0 || d->nmat < 0 || d->nquads + d->nspheres > PT_V4_MAX_OBJECTS ||
        d->nmat > PT_V4_MAX_OBJECTS)
        return -1;
    std::memset(s, 0, sizeof(*s));
    s->nquads = d->nquads;
    s->nspheres = d->nspheres;
    for (int i = 0; i < d->nquads; ++i) {   // PrecomputeQuadData :269-320
        const F3 V0 = f3(d->quad[i][0]), V1 = f3(d->quad[i][1]), V2 = f3(d->quad[i][2]), V3 = f3(d->quad[i][3]);
        const F3 V01 = sub(V1, V0), V02 = sub(V2, V0), V30 = sub(V0, V3), V20 = neg(V02);
        const F3 V01xV02 = cross(V01, V02), V02xV03 = cross(V30, V01);
        const float inv = 1.0f / std::sqrt(dot(V01xV02, V01xV02));   // normalize, mathlib.h:759
        const F3 N = {V01xV02.x * inv, V01xV02.y * inv, V01xV02.z * inv};
        const float DetTop = dot(V02xV03, N), DetBot = dot(V01xV02, N);
        PtV4Quad& q = s->quad[i];
        put(q.v0, V0);
        put(q.n, N);
        put(q.a0, div(cross(N, V01), DetBot));
        put(q.a1, div(cross(N, V20), DetBot));
        put(q.b0, div(cross(N, V30), DetTop));
        put(q.b1, div(cross(N, V02), DetTop));
    }
    for (int i = 0; i < d->nspheres; ++i) std::memcpy(s->sph[i], d->sphere[i], sizeof(s->sph[i]));
    for (int i = 0; i < d->nmat; ++i) {   // AddMaterialToScene :1370-1372: albedoR/G/B all = albedo.x
        s->mat[i] = d->mat[i];
        s->mat[i].albedo[1] = s->mat[i].albedo[2] = d->mat[i].albedo[0];
    }
    return 0;
}

bool pt_v4_is_default_geometry(const PtV4Scene& s)
{
    namespace D = pt_v4_default;
    if (s.nquads != D::kQuads || s.nspheres != D::kSpheres) return false;
    for (int i = 0; i < D::kQuads; ++i)
        if (std::memcmp(&s.quad[i], D::kQuad[i], sizeof(D::kQuad[i]))) return false;   // bit patterns (signed zeros)
    for (int i = 0; i < D::kSpheres; ++i)
        if (std::memcmp(s.sph[i], D::kSphere[i], sizeof(D::kSphere[i]))) return false;
    return true;
}
