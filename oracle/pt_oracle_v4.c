/* oracle/pt_oracle_v4.c -- TEST INFRASTRUCTURE ONLY: CPU parity checker for the v4 renderer.
 *
 * From-scratch scalar C restatement of the reference's shipping renderer,
 * demofox_path_tracing_optimization_v4.cpp (paths relative to
 * /root/reference/CPUPerformanceRayTracer/; "v4 :N" = that file's line N), which is 8-wide AVX2
 * code: every __m256 lane is one pixel with its own RNG state (seed from its own fragCoord,
 * v4 :1096-1102), so one lane == one scalar pixel here.  Lane masking is reproduced where it is
 * observable: a lane's RNG advances for every loop iteration the 8-wide group runs, but a lane's
 * own draws happen in a fixed order per iteration (env sample 2, ray roll 1, diffuse 3,
 * refraction 3, roulette 1), so a pixel's result depends only on its own iterations.
 *
 * Numerics (every operation in the reference's order; fused ops as fmaf):
 *   dot(m256x3)   = fma(x,x', fma(y,y', z*z'))            mathlib.h:145
 *   cross(m256x3) = (fma(uy,vz,-(uz*vy)), ...)            mathlib.h:770-778
 *   normalize     = v * (1 / sqrt(dot(v,v)))              mathlib.h:759
 *   lerp          = u + x*(v-u)                           mathlib.h:763
 *   max_ps/min_ps = a > b ? a : b / a < b ? a : b         (MAXPS/MINPS: second operand on NaN)
 *   to_epi32      = round-to-nearest-even conversion      mathlib.h:863
 * Substitutions (no portable bit pattern exists for the reference's instruction):
 *   rcp(x)    _mm256_rcp_ps (~12-bit table, CPU-model specific)  -> 1.f / x   (mathlib.h:415, scalar rcp)
 *   rsroot(x) _mm256_rsqrt_ps (same)                              -> 1.f / sqrtf(x) (mathlib.h:437)
 *   atan2_ps / asin_ps / sincos_ps (SVML, MSVC-only)              -> glibc atan2f / asinf / sinf+cosf
 * so against a run of the reference on a particular x86 CPU a pixel may differ in low bits
 * ("parity unpinned" for those terms); the HIP kernel must match THIS restatement bit
 * for bit.  The reference file itself is Win32 code (work queue, Interlocked*, SVML) and is not
 * built here.
 *
 * Reference quirks reproduced on purpose:
 *   - AddMaterialToScene stores albedo.x in all three albedo channels (v4 :1370-1372);
 *   - TestQuadTrace writes the hit normal only when the ray hits the quad's back side
 *     (v4 :630, blend with cond && dot(normal, rayDir) > 0); otherwise the normal of the previous
 *     closest hit (or zero) stays;
 *   - quads get a zero-initialised material (IOR 0, v4 :1418 `SceneMaterial NewMaterial{ 0 }`);
 *   - "Russian roulette" only chooses whether to boost the throughput; it never ends a path
 *     (v4 :891-899);
 *   - the striped background quad is not translated (v4 :1425-1429);
 *   - the env term is weighted by the throughput (v4 :787) and, with random-jitter sampling,
 *     draws two random numbers every loop iteration (hit or miss).
 */
#include "pt_oracle.h"
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define V4_MIN_HIT 0.01f       /* c_minimumRayHitTime  v4 :10 */
#define V4_NUDGE 0.01f         /* c_rayPosNormalNudge  v4 :14 */
#define V4_SUPER_FAR 10000.0f  /* c_superFar           v4 :17 */
#define V4_PI 3.14159265359f   /* c_pi                 mathutils.h:5 */

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add3(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 neg3(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 sel3(int c, v3 a, v3 b) { return c ? a : b; }
static inline float dot3(v3 u, v3 v) { return fmaf(u.x, v.x, fmaf(u.y, v.y, u.z * v.z)); }      /* mathlib.h:145 */
static inline v3 cross3(v3 u, v3 v)                                                              /* mathlib.h:770-778 */
{
    return mk(fmaf(u.y, v.z, -(u.z * v.y)), fmaf(u.z, v.x, -(u.x * v.z)), fmaf(u.x, v.y, -(u.y * v.x)));
}
static inline v3 normalize3(v3 v) { return muls(v, 1.0f / sqrtf(dot3(v, v))); }                  /* mathlib.h:759 */
static inline v3 fast_normalize3(v3 v) { return muls(v, 1.0f / sqrtf(dot3(v, v))); }             /* :755, rsroot -> :437 */
static inline float rcpf_(float x) { return 1.0f / x; }                                           /* rcp -> mathlib.h:415 */
static inline float max_ps(float a, float b) { return a > b ? a : b; }
static inline float min_ps(float a, float b) { return a < b ? a : b; }
static inline float saturate(float x) { return min_ps(max_ps(x, 0.0f), 1.0f); }                  /* mathlib.h:404 */
static inline int32_t cvt_rne(float x)   /* _mm256_cvtps_epi32: nearest-even, INT_MIN when out of range */
{
    if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
    return (int32_t)nearbyintf(x);
}

/* ---- scene (InitializeScene v4 :1403-1496, PrecomputeQuadData :269-320, AddMaterialToScene :1368-1388) */

typedef struct {
    v3 v0, n, a0, a1, b0, b1;   /* V0, normal, NxV01, NxV20 (bottom tri), NxV30, NxV02 (top tri) */
} q4;

typedef struct {
    float albedo[3], emissive[3], spec_chance, spec_rough, spec_color[3], ior, refr_chance, refr_rough, refr_color[3];
} m4;

typedef struct {
    int nq, ns;
    q4 quad[PTO4_MAX_OBJECTS];
    float sph[PTO4_MAX_OBJECTS][4];
    m4 mat[PTO4_MAX_OBJECTS];   /* indexed by object index (quads first); zero rows = zero material */
} s4;

static void precompute_quad(const float v[4][3], q4* q)   /* v4 :269-320 */
{
    const v3 V0 = mk(v[0][0], v[0][1], v[0][2]), V1 = mk(v[1][0], v[1][1], v[1][2]);
    const v3 V2 = mk(v[2][0], v[2][1], v[2][2]), V3 = mk(v[3][0], v[3][1], v[3][2]);
    const v3 V01 = sub3(V1, V0), V02 = sub3(V2, V0), V30 = sub3(V0, V3);
    const v3 V20 = neg3(V02), V23 = sub3(V3, V2), V12 = sub3(V2, V1);
    const v3 V01xV02 = cross3(V01, V02);
    const v3 V02xV03 = cross3(V30, V01);
    const v3 N = normalize3(V01xV02);
    const float DetTop = dot3(V02xV03, N);
    const float DetBot = dot3(V01xV02, N);
    v3 t;
    q->v0 = V0;
    q->n = N;
    t = cross3(N, V01); q->a0 = mk(t.x / DetBot, t.y / DetBot, t.z / DetBot);   /* NxV01 */
    (void)V12;                                                                    /* NxV12: unused by the test */
    t = cross3(N, V20); q->a1 = mk(t.x / DetBot, t.y / DetBot, t.z / DetBot);   /* NxV20 */
    t = cross3(N, V02); q->b1 = mk(t.x / DetTop, t.y / DetTop, t.z / DetTop);   /* NxV02 */
    (void)V23;                                                                    /* NxV23: unused */
    t = cross3(N, V30); q->b0 = mk(t.x / DetTop, t.y / DetTop, t.z / DetTop);   /* NxV30 */
}

void pto4_default_scene(pto4_scene* s)   /* InitializeScene, v4 :1403-1496 (SCENE == 1) */
{
    memset(s, 0, sizeof(*s));
    const float T[3] = {0.0f, 0.0f, 10.0f};   /* sceneTranslation :1407 */
    static const float quads[4][4][3] = {
        {{-25.0f, -12.5f, 5.0f}, {25.0f, -12.5f, 5.0f}, {25.0f, -12.5f, -5.0f}, {-25.0f, -12.5f, -5.0f}},  /* floor :1415-1418 */
        {{-25.0f, -1.5f, 5.0f}, {25.0f, -1.5f, 5.0f}, {25.0f, -10.5f, 5.0f}, {-25.0f, -10.5f, 5.0f}},    /* background :1428-1431 (untranslated) */
        {{-7.5f, 12.5f, 5.0f}, {7.5f, 12.5f, 5.0f}, {7.5f, 12.5f, -5.0f}, {-7.5f, 12.5f, -5.0f}},        /* ceiling :1446-1449 */
        {{-5.0f, 12.4f, 2.5f}, {5.0f, 12.4f, 2.5f}, {5.0f, 12.4f, -2.5f}, {-5.0f, 12.4f, -2.5f}},        /* light :1461-1464 */
    };
    static const float albedo[4] = {0.7f, 0.35f, 0.7f, 0.0f};
    for (int i = 0; i < 4; ++i) {
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 3; ++j) s->quad[i][k][j] = quads[i][k][j] + (i == 1 ? 0.0f : T[j]);
        pto4_material* m = &s->mat[s->nmat++];
        m->albedo[0] = m->albedo[1] = m->albedo[2] = albedo[i];
        if (i == 3) {   /* light: emissive (1, .9, .7) * 20 (:1469) */
            m->emissive[0] = 1.0f * 20.0f; m->emissive[1] = 0.9f * 20.0f; m->emissive[2] = 0.7f * 20.0f;
        }
    }
    s->nquads = 4;
    for (int i = 0; i < 7; ++i) {   /* :1474-1495 */
        float* p = s->sphere[s->nspheres++];
        p[0] = (-18.0f + 6.0f * (float)i) + 0.0f;
        p[1] = -8.0f + 0.0f;
        p[2] = 0.0f + 10.0f;
        p[3] = 2.8f + 0.0f;
        const float r = (((float)i) / (float)(7 - 1)) * 0.5f;
        pto4_material* m = &s->mat[s->nmat++];
        m->spec_chance = 0.02f;
        m->ior = 1.1f;
        m->refr_chance = 1.0f;
        m->albedo[0] = 0.9f; m->albedo[1] = 0.25f; m->albedo[2] = 0.25f;
        m->refr_color[0] = 0.0f; m->refr_color[1] = 0.5f; m->refr_color[2] = 1.0f;
        m->spec_color[0] = m->spec_color[1] = m->spec_color[2] = 1.0f * 0.8f;
        m->spec_rough = r;
        m->refr_rough = r;
    }
}

static int build_scene(const pto4_scene* src, s4* s)
{
    if (src->nquads < 0 || src->nspheres < 0 || src->nmat < 0 || src->nquads + src->nspheres > PTO4_MAX_OBJECTS ||
        src->nmat > PTO4_MAX_OBJECTS)
        return -1;
    memset(s, 0, sizeof(*s));
    s->nq = src->nquads;
    s->ns = src->nspheres;
    for (int i = 0; i < s->nq; ++i) precompute_quad(src->quad[i], &s->quad[i]);
    for (int i = 0; i < s->ns; ++i) memcpy(s->sph[i], src->sphere[i], sizeof(s->sph[i]));
    for (int i = 0; i < src->nmat; ++i) {   /* AddMaterialToScene :1370-1386 -- note albedo.x x3 */
        const pto4_material* a = &src->mat[i];
        m4* m = &s->mat[i];
        m->albedo[0] = m->albedo[1] = m->albedo[2] = a->albedo[0];
        memcpy(m->emissive, a->emissive, 12);
        m->spec_chance = a->spec_chance;
        m->spec_rough = a->spec_rough;
        memcpy(m->spec_color, a->spec_color, 12);
        m->ior = a->ior;
        m->refr_chance = a->refr_chance;
        m->refr_rough = a->refr_rough;
        memcpy(m->refr_color, a->refr_color, 12);
    }
    return 0;
}

/* ---- RNG (mathutils.h:8-26, v4 :109-130, mathutils.h:33-46) ---------------------------------- */

static inline uint32_t wang(uint32_t* s)
{
    uint32_t x = *s;
    x = (x ^ 61u) ^ (x >> 16);
    x *= 9u;
    x = x ^ (x >> 4);
    x *= 0x27d4eb2du;
    x = x ^ (x >> 15);
    *s = x;
    return x;
}

static inline float randf(uint32_t* s) { return (float)(int32_t)(wang(s) & 0x7FFFFFFFu) / 2147483648.0f; }

float pto4_randomf(uint32_t* s) { return randf(s); }

static inline v3 ruv_rejection(uint32_t* s)   /* RandomUnitVectorRejectionSample_ps, v4 :109-130 */
{
    const float u = fmaf(2.0f, randf(s), -1.0f);
    const float v = fmaf(2.0f, randf(s), -1.0f);
    const float w = fmaf(2.0f, randf(s), -1.0f);
    const float uv_d2 = fmaf(u, u, v * v);
    const float uvw_d2 = fmaf(w, w, uv_d2);
    return muls(mk(u, v, w), 1.0f / sqrtf(uvw_d2));
}

static inline v3 ruv_angle(uint32_t* s)   /* RandomUnitVector_ps, mathutils.h:33-46 */
{
    const float wide_z = randf(s);
    const float wide_a = randf(s);
    const float z = wide_z * 2.0f - 1.0f;
    const float a = wide_a * (2.0f * V4_PI);
    const float r = sqrtf(1.0f - z * z);
    return mk(r * cosf(a), r * sinf(a), z);
}

void pto4_random_unit_vector(uint32_t* s, int rejection, float out[3])
{
    const v3 r = rejection ? ruv_rejection(s) : ruv_angle(s);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ---- env lookups (texture.cpp) ----------------------------------------------------------------- */

/* GatherRGB (:16-26) at element index e.  Out of the texture the reference reads out of bounds
 * (UB): clamped to [0, last texel's first element] (INT32_MIN from cvtps_epi32 -> 0). */
static inline v3 texel_e(const pto_env* t, int64_t e)
{
    const int64_t last = 3 * ((int64_t)t->width * t->height - 1);
    if (e < 0) e = 0;
    if (e > last) e = last;
    const float* p = t->data + e;
    return mk(p[0], p[1], p[2]);
}

static v3 texel_sample_random(const pto_env* t, float u, float v, uint32_t* s)   /* :78-86 */
{
    const float Row = fmaf(v, (float)t->height, -v);
    const float Col = fmaf(u, (float)t->width, -u);
    const float RandRow = floorf(Row + randf(s));
    const float RandCol = floorf(Col + randf(s));
    int64_t lin = cvt_rne(fmaf(RandRow, (float)t->width, RandCol));
    const int64_t n = (int64_t)t->width * t->height;
    if (lin < 0) lin = 0;          /* incl. INT32_MIN */
    if (lin >= n) lin = n - 1;
    return texel_e(t, 3 * lin);    /* Rand_Idx = 3 * to_epi32(...) (:84) */
}

static v3 texel_sample_bilinear(const pto_env* t, float u, float v)   /* :38-76 */
{
    const float Row = v * (float)(t->height - 1);
    const float Col = u * (float)(t->width - 1);
    float Row0 = floorf(Row), Row1 = ceilf(Row), Col0 = floorf(Col), Col1 = ceilf(Col);
    const float dV = Row - Row0, dU = Col - Col0;
    const float texWidth = 3.0f * (float)t->width;
    Row0 = Row0 * texWidth; Row1 = Row1 * texWidth;
    Col0 = Col0 * 3.0f; Col1 = Col1 * 3.0f;
    const int32_t I00 = cvt_rne(Col0 + Row0), I10 = cvt_rne(Col1 + Row0);
    const int32_t I01 = cvt_rne(Col0 + Row1), I11 = cvt_rne(Col1 + Row1);
    const v3 C00 = texel_e(t, I00), C10 = texel_e(t, I10);   /* element indices (:63-66) */
    const v3 C01 = texel_e(t, I01), C11 = texel_e(t, I11);
    const v3 C0 = add3(C00, muls(sub3(C10, C00), dU));   /* lerp: u + x*(v-u), mathlib.h:763 */
    const v3 C1 = add3(C01, muls(sub3(C11, C01), dU));
    return add3(C0, muls(sub3(C1, C0), dV));
}

static inline float fract_(float a) { return a - floorf(a); }   /* mathlib.h:395 */

static v3 equirect_random(const pto_env* t, v3 d, uint32_t* s)   /* EquirectangularTextureSampleRandom :186-203 */
{
    float u = atan2f(d.z, d.x), v = asinf(d.y);
    u = saturate(fract_(fmaf(0.1591f, u, 0.5f)));
    v = saturate(fract_(fmaf(0.3183f, v, 0.5f)));
    return texel_sample_random(t, u, v, s);
}

static v3 equirect_bilinear(const pto_env* t, v3 d)   /* EquirectangularTextureSampleBilinear :164-184 */
{
    float u = atan2f(d.z, d.x) * 0.1591f, v = asinf(d.y) * 0.3183f;
    u = u + 0.5f; v = v + 0.5f;
    u = u - floorf(u); v = v - floorf(v);
    return texel_sample_bilinear(t, saturate(u), saturate(v));
}

/* face selection shared by both cubemap samplers (texture.cpp:283-331 / :345-392); the offsets of
 * the two functions are different f32 constants, passed in */
static void cube_face(v3 d, const float off[6], float* fu, float* fv, float* voff, float* maxabs)
{
    const v3 a = mk(fabsf(d.x), fabsf(d.y), fabsf(d.z));
    const int cx = d.x >= 0.0f;
    *fu = cx ? -d.z : d.z;
    *fv = d.y;
    *voff = cx ? off[0] : off[1];
    const int cy = d.y >= 0.0f;
    if (a.y >= a.x) {
        *voff = cy ? off[2] : off[3];
        *fu = d.x;
        *fv = cy ? -d.z : d.z;
    }
    const int cz = d.z >= 0.0f;
    if (a.z >= a.x && a.z >= a.y) {
        *voff = cz ? off[4] : off[5];
        *fu = cz ? d.x : -d.x;
        *fv = d.y;
    }
    *maxabs = max_ps(a.x, max_ps(a.y, a.z));
}

static v3 cubemap_random(const pto_env* t, v3 d, uint32_t* s)   /* CubemapTextureSampleRandom :339-404 */
{
    const float k = 0.166666666666667f;
    const float off[6] = {0.0f, k, 2.0f * k, 3.0f * k, 4.0f * k, 5.0f * k};
    float fu, fv, voff, m;
    cube_face(d, off, &fu, &fv, &voff, &m);
    const float r = rcpf_(m);
    const float u = saturate(fmaf(fu * r, 0.5f, 0.5f));
    float v = saturate(fmaf(fv * r, 0.5f, 0.5f));
    v = saturate(fmaf(v, 0.166666666666667f, voff));
    return texel_sample_random(t, u, v, s);
}

static v3 cubemap_bilinear(const pto_env* t, v3 d)   /* CubemapTextureSampleBilinear :275-337 */
{
    const float off[6] = {0.0f, 1.0f / 6.0f, 2.0f / 6.0f, 3.0f / 6.0f, 4.0f / 6.0f, 5.0f / 6.0f};
    float fu, fv, voff, m;
    cube_face(d, off, &fu, &fv, &voff, &m);
    const float u = saturate((fu / m) * 0.5f + 0.5f);
    float v = saturate((fv / m) * 0.5f + 0.5f);
    v = saturate(fmaf(v, 1.0f / 6.0f, voff));
    return texel_sample_bilinear(t, u, v);
}

void pto4_env_sample(const pto_env* env, int32_t env_mode, int32_t random_jitter, const float dir[3], uint32_t* s,
                     float out[3])
{
    const v3 d = mk(dir[0], dir[1], dir[2]);
    v3 r = mk(0.11f, 0.1f, 0.15f);
    if (env_mode == PTO4_ENV_EQUIRECT) {
        const v3 sd = mk(-d.x, d.y, -d.z);   /* v4 :775-776 */
        r = random_jitter ? equirect_random(env, sd, s) : equirect_bilinear(env, sd);
    } else if (env_mode == PTO4_ENV_CUBEMAP) {
        r = random_jitter ? cubemap_random(env, d, s) : cubemap_bilinear(env, d);
    }
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ---- intersection (v4 :556-718) -------------------------------------------------------------- */

typedef struct { int from_inside; float dist; v3 normal; int mat; } hit4;

static inline int quad_trace(v3 pos, v3 dir, hit4* h, const q4* q)   /* TestQuadTrace :556-637 */
{
    const v3 off = sub3(q->v0, pos);
    const float rdn = dot3(dir, q->n);
    const float ron = dot3(off, q->n);
    const float dist = ron * rcpf_(rdn);
    const v3 hp = mk(fmaf(dist, dir.x, -off.x), fmaf(dist, dir.y, -off.y), fmaf(dist, dir.z, -off.z));
    const float A0 = dot3(hp, q->a0), A1 = dot3(hp, q->a1), A2 = 1.0f - A0 - A1;
    const float B0 = dot3(hp, q->b0), B1 = dot3(hp, q->b1), B2 = 1.0f - B0 - B1;
    const int tri1 = A0 >= 0.0f && A1 >= 0.0f && A2 >= 0.0f;
    const int tri2 = B0 >= 0.0f && B1 >= 0.0f && B2 >= 0.0f;
    const int cond = (tri1 || tri2) && (dist > V4_MIN_HIT && dist < h->dist);
    if (cond) {
        h->from_inside = 0;
        h->dist = dist;
        if (dot3(q->n, dir) > 0.0f) h->normal = neg3(q->n);
    }
    return cond;
}

static inline int sphere_trace(v3 pos, v3 dir, hit4* h, const float* sp)   /* TestSphereTrace :641-695 */
{
    const v3 m = sub3(pos, mk(sp[0], sp[1], sp[2]));
    const float b = dot3(m, dir);
    const float c = fmaf(-sp[3], sp[3], dot3(m, m));
    const int cond = c > 0.0f && b > 0.0f;
    const float discr = fmaf(b, b, -c);
    const int early = discr < 0.0f || cond;
    const float s = sqrtf(discr);
    const int inside = -b < s;
    const float dist = (inside ? s : -s) - b;
    const int check = !early && (dist > V4_MIN_HIT && dist < h->dist);
    if (check) {
        h->from_inside = inside;
        h->dist = dist;
        const v3 p = mk(fmaf(dir.x, dist, m.x), fmaf(dir.y, dist, m.y), fmaf(dir.z, dist, m.z));
        h->normal = muls(normalize3(p), inside ? -1.0f : 1.0f);
    }
    return check;
}

static inline uint64_t scene_trace(const s4* s, v3 pos, v3 dir, hit4* h)   /* TestSceneTrace :700-718 */
{
    int obj = 0;
    uint64_t flops = 53u * (uint64_t)s->nq + 25u * (uint64_t)s->ns;
    for (int i = 0; i < s->nq; ++i, ++obj)
        if (quad_trace(pos, dir, h, &s->quad[i])) {
            h->mat = obj;
            flops += 6;
        }
    for (int i = 0; i < s->ns; ++i, ++obj)
        if (sphere_trace(pos, dir, h, s->sph[i])) {
            h->mat = obj;
            flops += 19;
        }
    return flops;
}

static inline float fresnel(float n1, float n2, v3 normal, v3 incident, float f0, float f90)   /* :429-453 */
{
    float r0 = (n1 - n2) * rcpf_(n1 + n2);
    r0 = r0 * r0;
    float cosX = -dot3(normal, incident);
    const int cond = n1 > n2;
    const float n = n1 * rcpf_(n2);
    const float sinT2Compl = fmaf(-(n * n), fmaf(-cosX, cosX, 1.0f), 1.0f);
    const float newCosX = sqrtf(sinT2Compl);
    const int tir = 0.0f > sinT2Compl;
    if (cond && !tir) cosX = newCosX;
    const float x = 1.0f - cosX;
    const float x2 = x * x;
    float ret = fmaf(((1.0f - r0) * x2) * x2, x, r0);
    if (cond && tir) ret = 1.0f;
    return fmaf(ret, f90 - f0, f0);
}

static inline v3 refract3(v3 v, v3 n, float ior)   /* rfrct, mathlib.h:781-789 */
{
    const float vdotn = dot3(v, n);
    const float k = fmaf(-ior, ior * fmaf(-vdotn, vdotn, 1.0f), 1.0f);
    const float s = fmaf(ior, vdotn, sqrtf(k));
    v3 r = mk(fmaf(ior, v.x, -(s * n.x)), fmaf(ior, v.y, -(s * n.y)), fmaf(ior, v.z, -(s * n.z)));
    if (k < 0.0f) r = mk(0.0f, 0.0f, 0.0f);
    return r;
}

static inline float approx_exp(float a)   /* approx_exp_ps, mathlib.h:501-516 */
{
    const float b = fmaf(a, 0.05995203836930455f, 1.0f);
    const float b2 = b * b, b4 = b2 * b2, b8 = b4 * b4;
    return b8 * b8;
}

typedef struct {
    const s4* scene;
    const pto4_params* p;
    pto4_counts* cnt;
} ctx4;

/* FLOP accounting (SURVEY.md §8d convention: 1 per f32 add/sub/mul/div/sqrt/compare/min/max the
 * reference executes, an fmadd/fmsub/fnmadd = 2, negation/abs/select/floor/conversions 0; scene-
 * and frame-constant work (PrecomputeQuadData, rcp of the resolution, 1/(iFrame+1)) excluded;
 * atan2/asin/sin/cos counted as transcendentals).  Per-function totals, counted by hand from the
 * code above and below:
 *   TestQuadTrace   53 (+6 on a hit: the facing dot + compare)            v4 :556-637
 *   TestSphereTrace 25 (+19 on a hit: hit point, normalize, sign)        v4 :641-695
 *   miss            6 (throughput-weighted ambient) + env lookup: equirect 10 + 2T, cubemap 23
 *                   (bilinear 22), then the texel sampler: random 8, bilinear 39
 *   hit shading     absorption 24 (inside only); last bounce 6 (emissive); otherwise 199
 *                   (Fresnel 31, chances 15, nudge 13, diffuse 29, specular 22, refraction 63,
 *                   normalize 10, emissive + throughput + roulette 16..20 (+4 on a boost))
 *   per sample      camera 23, c_numRendersPerFrame scale 6, accumulate 9 = 38 */
#define CNT(c, n) do { if ((c)->cnt) (c)->cnt->flops += (uint64_t)(n); } while (0)

/* GetColorForRay, v4 :722-911 (USE_FAST_APPROXIMATE_EXP: p->exact_exp) */
static v3 color_for_ray(const ctx4* c, v3 pos, v3 dir, uint32_t* rng)
{
    const pto4_params* p = c->p;
    const s4* s = c->scene;
    v3 ret = mk(0.0f, 0.0f, 0.0f), T = mk(1.0f, 1.0f, 1.0f);
    for (int bounce = 0; bounce <= p->num_bounces; ++bounce) {
        hit4 h = {0, V4_SUPER_FAR, {0.0f, 0.0f, 0.0f}, 0};
        const uint64_t trace_flops = scene_trace(s, pos, dir, &h);
        CNT(c, trace_flops);
        if (c->cnt) c->cnt->segments++;
        const int miss = h.dist == V4_SUPER_FAR;
        /* the ambient / env term is evaluated every iteration (:769-784): its RNG draws happen on
         * hits too */
        float amb[3];
        const float dv[3] = {dir.x, dir.y, dir.z};
        pto4_env_sample(p->env, p->env ? p->env_mode : PTO4_ENV_NONE, p->random_jitter, dv, rng, amb);
        if (miss) {
            ret = mk(fmaf(amb[0], T.x, ret.x), fmaf(amb[1], T.y, ret.y), fmaf(amb[2], T.z, ret.z));   /* :787 */
            if (c->cnt) {
                c->cnt->escaped++;
                const int mode = p->env ? p->env_mode : PTO4_ENV_NONE;
                uint64_t f = 6;
                if (mode == PTO4_ENV_EQUIRECT) f += 10, c->cnt->transcendentals += 2;
                if (mode == PTO4_ENV_CUBEMAP) f += p->random_jitter ? 23 : 22;
                if (mode != PTO4_ENV_NONE) f += p->random_jitter ? 8 : 39;
                c->cnt->flops += f;
            }
            break;
        }
        const m4* M = &s->mat[h.mat];   /* GatherMaterials :389-427 */
        const v3 rc = mk(M->refr_color[0], M->refr_color[1], M->refr_color[2]);
        if (h.from_inside) {   /* :797 (Beer's law) */
            if (p->exact_exp)      /* USE_FAST_APPROXIMATE_EXP 0 (:785-787): exp_ps -> libm expf */
                T = mul3(T, mk(expf(-rc.x * h.dist), expf(-rc.y * h.dist), expf(-rc.z * h.dist)));
            else                   /* :783-784: approx_exp_ps */
                T = mul3(T, mk(approx_exp(-rc.x * h.dist), approx_exp(-rc.y * h.dist), approx_exp(-rc.z * h.dist)));
            CNT(c, 24);
        }

        if (bounce == p->num_bounces) {   /* last iteration: only the emissive term below is used */
            ret = mk(fmaf(M->emissive[0], T.x, ret.x), fmaf(M->emissive[1], T.y, ret.y), fmaf(M->emissive[2], T.z, ret.z));
            CNT(c, 6);
            break;
        }
        CNT(c, 199);
        if (c->cnt && !p->rejection) c->cnt->transcendentals += 4;
        float spec = M->spec_chance, refr = M->refr_chance;
        {   /* :807-829 */
            const int has_spec = spec > 0.0f;
            const float n1 = h.from_inside ? M->ior : 1.0f;
            const float n2 = h.from_inside ? 1.0f : M->ior;
            const float new_spec = fresnel(n1, n2, h.normal, dir, M->spec_chance, 1.0f);
            const float rscc = rcpf_(1.0f - M->spec_chance);
            const float mult = fmaf(-new_spec, rscc, rscc);
            if (has_spec) {
                spec = new_spec;
                refr = refr * mult;
            }
        }
        const float roll = randf(rng);   /* :831 */
        const int do_spec = spec > 0.0f && roll < spec;
        const int do_refr = !do_spec && refr > 0.0f && roll < spec + refr;
        const int do_diff = !do_spec && !do_refr;
        const float diff_chance = max_ps(1.0f - (spec + refr), 0.0f);
        float prob = 1.0f;
        if (do_spec) prob = spec;
        if (do_refr) prob = refr;
        if (do_diff) prob = diff_chance;
        prob = max_ps(prob, 0.001f);

        const float nudge = V4_NUDGE * (do_refr ? -1.0f : 1.0f);   /* :848-849 */
        const v3 npos = mk(fmaf(nudge, h.normal.x, fmaf(dir.x, h.dist, pos.x)),
                           fmaf(nudge, h.normal.y, fmaf(dir.y, h.dist, pos.y)),
                           fmaf(nudge, h.normal.z, fmaf(dir.z, h.dist, pos.z)));
        v3 ndir;
        {   /* :852-888 */
            const v3 diffuse = p->rejection ? fast_normalize3(add3(h.normal, ruv_rejection(rng)))
                                            : normalize3(add3(h.normal, ruv_angle(rng)));
            const float d2 = 2.0f * dot3(dir, h.normal);
            v3 specd = mk(fmaf(-d2, h.normal.x, dir.x), fmaf(-d2, h.normal.y, dir.y), fmaf(-d2, h.normal.z, dir.z));
            const float srsq = M->spec_rough * M->spec_rough;
            specd = mk(fmaf(srsq, diffuse.x - specd.x, specd.x), fmaf(srsq, diffuse.y - specd.y, specd.y),
                       fmaf(srsq, diffuse.z - specd.z, specd.z));
            const float ior = h.from_inside ? M->ior : rcpf_(M->ior);
            const float rrsq = M->refr_rough * M->refr_rough;
            v3 refd = refract3(dir, h.normal, ior);
            if (p->rejection) {
                const v3 nrd = fast_normalize3(sub3(ruv_rejection(rng), h.normal));
                refd = mk(fmaf(rrsq, nrd.x - refd.x, refd.x), fmaf(rrsq, nrd.y - refd.y, refd.y),
                          fmaf(rrsq, nrd.z - refd.z, refd.z));
            } else {
                const v3 nrd = normalize3(sub3(ruv_angle(rng), h.normal));
                refd = normalize3(add3(refd, muls(sub3(nrd, refd), rrsq)));
            }
            ndir = sel3(do_spec, specd, diffuse);
            ndir = sel3(do_refr, refd, ndir);
            ndir = normalize3(ndir);
        }
        ret = mk(fmaf(M->emissive[0], T.x, ret.x), fmaf(M->emissive[1], T.y, ret.y), fmaf(M->emissive[2], T.z, ret.z));
        const v3 cf = do_spec ? mk(M->spec_color[0], M->spec_color[1], M->spec_color[2])
                              : mk(M->albedo[0], M->albedo[1], M->albedo[2]);
        if (!do_refr) T = mul3(T, cf);
        T = muls(T, rcpf_(prob));
        {   /* :891-899 */
            const float pm = max_ps(T.x, max_ps(T.y, T.z));
            const int term = randf(rng) > pm;
            if (!term) {
                T = muls(T, rcpf_(pm));
                CNT(c, 4);
            }
        }
        pos = npos;
        dir = ndir;
    }
    return ret;
}

/* mainImage, v4 :1092-1130 (c_numRendersPerFrame = NUM_SAMPLES_PER_FRAME = 1) */
static v3 main_image(const ctx4* c, int32_t X, int32_t Y, uint32_t frame)
{
    const pto4_params* p = c->p;
    const float fx = (float)X, fy = (float)(p->height - 1 - Y);   /* RenderTile :1207-1226 */
    uint32_t rng = 1u | ((uint32_t)cvt_rne(fx) * 1973u + (uint32_t)cvt_rne(fy) * 9277u + frame * 26699u);
    const float W = (float)p->width, H = (float)p->height;
    const float rW = rcpf_(W), rH = rcpf_(H);
    const float jx = randf(&rng) - 0.5f;
    const float jy = randf(&rng) - 0.5f;
    const float tx = fmaf((fx + jx) * rW, 2.0f, -1.0f);
    float ty = fmaf((fy + jy) * rH, 2.0f, -1.0f);
    ty = ty * (rW * H);
    const float cam_dist = 1.0f / tanf(90.0f * 0.5f * V4_PI / 180.0f);   /* InitializeCamera :1500 */
    const v3 dir = normalize3(sub3(mk(tx, ty, -cam_dist), mk(0.0f, 0.0f, 0.0f)));
    if (c->cnt) c->cnt->samples++;
    CNT(c, 38);
    const v3 col = color_for_ray(c, mk(0.0f, 0.0f, 1.0f * 40.0f), dir, &rng);
    return mk(fmaf(col.x, 1.0f, 0.0f), fmaf(col.y, 1.0f, 0.0f), fmaf(col.z, 1.0f, 0.0f));   /* :1127 */
}

static void row4(const ctx4* c, float* out, int32_t Y)
{
    const pto4_params* p = c->p;
    for (int32_t X = 0; X < p->width; ++X) {
        float* px = out + 3 * (size_t)X;
        for (int32_t f = 0; f < p->nframes; ++f) {
            const uint32_t frame = p->frame_first + (uint32_t)f;
            const v3 col = main_image(c, X, Y, frame);
            if (p->no_accumulate) {   /* ACCUMULATE_FRAMES 0: the colour is stored (:1245-1250) */
                px[0] = col.x;
                px[1] = col.y;
                px[2] = col.z;
                continue;
            }
            const float bf = 1.0f / ((float)frame + 1.0f);   /* :1200, ACCUMULATE_FRAMES */
            px[0] = fmaf(bf, col.x - px[0], px[0]);         /* :1243 */
            px[1] = fmaf(bf, col.y - px[1], px[1]);
            px[2] = fmaf(bf, col.z - px[2], px[2]);
        }
    }
}

typedef struct { float* buf; const ctx4* c; int tid, nt; } job4;

static void* worker4(void* arg)
{
    job4* j = (job4*)arg;
    const pto4_params* p = j->c->p;
    for (int32_t r = j->tid; r < p->nrows; r += j->nt)
        row4(j->c, j->buf + (size_t)r * 3 * (size_t)p->width, p->row_start + r * p->row_stride);
    return NULL;
}

static int check4(const float* buf, const pto4_params* p)
{
    if (!buf || !p) return -1;
    if (p->width <= 0 || p->height <= 0 || p->nrows < 0 || p->nframes < 0 || p->row_stride <= 0 || p->row_start < 0)
        return -1;
    if (p->nrows > 0 && p->row_start + (int64_t)(p->nrows - 1) * p->row_stride >= p->height) return -1;
    if (p->num_bounces < 0 || p->frame_first < 1 || (uint64_t)p->frame_first + (uint64_t)p->nframes > (1u << 24))
        return -1;
    if (p->env && (!p->env->data || p->env->width < 1 || p->env->height < 1)) return -1;
    return 0;
}

int pto4_render(float* buf, const pto4_params* p, const pto4_scene* scene, pto4_counts* counts)
{
    if (check4(buf, p)) return -1;
    pto4_scene def;
    if (!scene) {
        pto4_default_scene(&def);
        scene = &def;
    }
    s4* s = (s4*)malloc(sizeof(s4));
    if (!s) return -1;
    if (build_scene(scene, s)) {
        free(s);
        return -1;
    }
    ctx4 c = {s, p, counts};
    if (counts) memset(counts, 0, sizeof(*counts));
    int nt = (p->nthreads > 1 && !counts) ? p->nthreads : 1;
    if (nt > 256) nt = 256;
    if (nt == 1) {
        job4 j = {buf, &c, 0, 1};
        worker4(&j);
    } else {
        pthread_t th[256];
        job4 jobs[256];
        int started = 0;
        for (int t = 0; t < nt; ++t) {
            jobs[t].buf = buf; jobs[t].c = &c; jobs[t].tid = t; jobs[t].nt = nt;
            if (pthread_create(&th[t], NULL, worker4, &jobs[t])) break;
            ++started;
        }
        if (started < nt) {   /* run the missing workers' rows here */
            for (int t = started; t < nt; ++t) worker4(&jobs[t]);
        }
        for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    }
    free(s);
    return 0;
}

/* TestSceneTrace (v4 :700-718) of one ray against `scene` (NULL: InitializeScene): the hit distance
 * (c_superFar on a miss), *mat = the hit object (-1 none).  Checker entry point for the kernel's
 * sky test (tests/native/check_sky.cpp). */
static s4 g_def_scene;
static pthread_once_t g_def_once = PTHREAD_ONCE_INIT;
static void build_default_scene(void)
{
    pto4_scene def;
    pto4_default_scene(&def);
    (void)build_scene(&def, &g_def_scene);
}
float pto4_trace_scene_flops(const pto4_scene* scene, const float P[3], const float D[3], int* mat, uint64_t* flops);
float pto4_trace_scene(const pto4_scene* scene, const float P[3], const float D[3], int* mat)
{
    return pto4_trace_scene_flops(scene, P, D, mat, NULL);
}
/* ... and the reference's f32 FLOP count of that TestSceneTrace (the instrumented accounting) */
float pto4_trace_scene_flops(const pto4_scene* scene, const float P[3], const float D[3], int* mat, uint64_t* flops)
{
    s4 own;
    const s4* s = &own;
    if (!scene) {
        pthread_once(&g_def_once, build_default_scene);
        s = &g_def_scene;
    } else if (build_scene(scene, &own)) {
        return -1.0f;
    }
    hit4 h = {0, V4_SUPER_FAR, {0.0f, 0.0f, 0.0f}, -1};
    const uint64_t fl = scene_trace(s, mk(P[0], P[1], P[2]), mk(D[0], D[1], D[2]), &h);
    if (flops) *flops = fl;
    if (mat) *mat = h.dist == V4_SUPER_FAR ? -1 : h.mat;
    return h.dist;
}

int pto4_scene_tables(const pto4_scene* scene, float* out, int32_t n)
{
    /* precomputed quad rows (v0, n, NxV01, NxV20, NxV30, NxV02: 18 f32 per quad) then the material
     * rows after AddMaterialToScene (17 f32 per object) -- for checking the product's host tables */
    pto4_scene def;
    if (!scene) {
        pto4_default_scene(&def);
        scene = &def;
    }
    s4 s;
    if (build_scene(scene, &s)) return -1;
    const int need = 18 * s.nq + 17 * PTO4_MAX_OBJECTS;
    if (n < need) return -1;
    float* o = out;
    for (int i = 0; i < s.nq; ++i) {
        const v3* r[6] = {&s.quad[i].v0, &s.quad[i].n, &s.quad[i].a0, &s.quad[i].a1, &s.quad[i].b0, &s.quad[i].b1};
        for (int k = 0; k < 6; ++k) { *o++ = r[k]->x; *o++ = r[k]->y; *o++ = r[k]->z; }
    }
    for (int i = 0; i < PTO4_MAX_OBJECTS; ++i) {
        memcpy(o, &s.mat[i], 17 * sizeof(float));
        o += 17;
    }
    return need;
}
