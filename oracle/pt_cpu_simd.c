/* oracle/pt_cpu_simd.c -- TEST / BASELINE INFRASTRUCTURE ONLY: the CPU baseline of bench.py.
 *
 * An AVX2 + FMA port, written from scratch in C, of the reference's fastest CPU renderer of the
 * diffuse+emissive path: demofox_path_tracing_simt_pooled.cpp (paths relative to
 * /root/reference/CPUPerformanceRayTracer/) -- 8 pixels per __m256, one Wang-hash state PER LANE
 * (wang_hash_ps :36-44, seeded from each lane's fragCoord :435-445), RandomUnitVector_ps with
 * vector sin/cos (:86-100), TestQuadTrace / TestSphereTrace / TestSceneTrace with masked blends
 * (:104-383, same structure as demofox_path_tracing_simd.cpp:109-380), GetColorForRay running all
 * c_numBounces + 1 iterations with masks (:386-428), RenderTile over 8-pixel groups of a tile
 * (:500-545) and a pool of worker threads taking tiles (:551-660; here a fixed pthread pool pulling
 * tiles from an atomic counter instead of one condition-variable thread per tile).
 *
 * Why a port: the reference's SIMD files need MSVC (operator overloads on __m256 and SVML
 * _mm256_sin_ps / _mm256_cos_ps) and cannot be built here without writing stand-ins for them
 * (SURVEY.md §8c A2), which this repo does not do.  This port is what bench.py times as the
 * reference's CPU SIMD path on the GPU box's host cores ("kind": "port").  It is NOT a parity
 * checker (the SIMD files are not bitwise comparable to the scalar path); its image
 * is checked statistically against the scalar oracle (tests/test_cpu_simd.py).
 *
 * Port choices (timing-neutral): the scalar file's scene constants (ambient 0.1, sphere albedos of
 * scalar.cpp:270-284) so the statistical check against the oracle applies; vector sin/cos from
 * glibc's libmvec (_ZGVdN8v_sinf/_ZGVdN8v_cosf) where the reference calls SVML; c_numBounces a
 * parameter (4 in the reference file, 8 in the benchmark configs); the tile-major planar8 layout of
 * RenderTile (simd_tiled.cpp:499-531).
 */
#include "pt_oracle.h"
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

__m256 _ZGVdN8v_sinf(__m256);   /* glibc libmvec, AVX2 variants */
__m256 _ZGVdN8v_cosf(__m256);

typedef struct { __m256 x, y, z; } v8;

#define SET1(a) _mm256_set1_ps(a)
static inline v8 mk8(__m256 x, __m256 y, __m256 z) { v8 r = {x, y, z}; return r; }
static inline v8 set8(float x, float y, float z) { return mk8(SET1(x), SET1(y), SET1(z)); }
static inline v8 add8(v8 a, v8 b) { return mk8(_mm256_add_ps(a.x, b.x), _mm256_add_ps(a.y, b.y), _mm256_add_ps(a.z, b.z)); }
static inline v8 sub8(v8 a, v8 b) { return mk8(_mm256_sub_ps(a.x, b.x), _mm256_sub_ps(a.y, b.y), _mm256_sub_ps(a.z, b.z)); }
static inline v8 mul8(v8 a, v8 b) { return mk8(_mm256_mul_ps(a.x, b.x), _mm256_mul_ps(a.y, b.y), _mm256_mul_ps(a.z, b.z)); }
static inline v8 muls8(v8 a, __m256 s) { return mk8(_mm256_mul_ps(a.x, s), _mm256_mul_ps(a.y, s), _mm256_mul_ps(a.z, s)); }
static inline v8 blend8(v8 a, v8 b, __m256 m)
{
    return mk8(_mm256_blendv_ps(a.x, b.x, m), _mm256_blendv_ps(a.y, b.y, m), _mm256_blendv_ps(a.z, b.z, m));
}
static inline __m256 dot8(v8 u, v8 v)   /* mathlib.h:145 */
{
    return _mm256_fmadd_ps(u.x, v.x, _mm256_fmadd_ps(u.y, v.y, _mm256_mul_ps(u.z, v.z)));
}
static inline v8 cross8(v8 u, v8 v)   /* mathlib.h:770-778 */
{
    return mk8(_mm256_fmsub_ps(u.y, v.z, _mm256_mul_ps(u.z, v.y)), _mm256_fmsub_ps(u.z, v.x, _mm256_mul_ps(u.x, v.z)),
               _mm256_fmsub_ps(u.x, v.y, _mm256_mul_ps(u.y, v.x)));
}
static inline v8 normalize8(v8 v) { return muls8(v, _mm256_div_ps(SET1(1.0f), _mm256_sqrt_ps(dot8(v, v)))); }
static inline __m256 gt(__m256 a, __m256 b) { return _mm256_cmp_ps(a, b, _CMP_GT_OQ); }
static inline __m256 lt(__m256 a, __m256 b) { return _mm256_cmp_ps(a, b, _CMP_LT_OQ); }
static inline __m256 ge(__m256 a, __m256 b) { return _mm256_cmp_ps(a, b, _CMP_GE_OQ); }
static inline __m256 and8(__m256 a, __m256 b) { return _mm256_and_ps(a, b); }
static inline __m256 or8(__m256 a, __m256 b) { return _mm256_or_ps(a, b); }
static inline __m256 not8(__m256 a) { return _mm256_xor_ps(a, _mm256_castsi256_ps(_mm256_set1_epi32(-1))); }

typedef struct { __m256 dist; v8 normal, albedo, emissive; } hit8;

static inline __m256i wang8(__m256i* s)   /* wang_hash_ps, simt_pooled.cpp:36-44 */
{
    __m256i x = *s;
    x = _mm256_xor_si256(_mm256_xor_si256(x, _mm256_set1_epi32(61)), _mm256_srli_epi32(x, 16));
    x = _mm256_mullo_epi32(x, _mm256_set1_epi32(9));
    x = _mm256_xor_si256(x, _mm256_srli_epi32(x, 4));
    x = _mm256_mullo_epi32(x, _mm256_set1_epi32(0x27d4eb2d));
    x = _mm256_xor_si256(x, _mm256_srli_epi32(x, 15));
    *s = x;
    return x;
}

static inline __m256 randf8(__m256i* s)   /* Randomf3201_ps: u32 -> f32 (:46-60) / 2^32 */
{
    const __m256i v = wang8(s);
    const __m256 v2f = _mm256_cvtepi32_ps(_mm256_srli_epi32(v, 1));
    const __m256 v1f = _mm256_cvtepi32_ps(_mm256_and_si256(v, _mm256_set1_epi32(1)));
    return _mm256_div_ps(_mm256_add_ps(_mm256_add_ps(v2f, v2f), v1f), SET1(4294967296.0f));
}

static inline v8 ruv8(__m256i* s)   /* RandomUnitVector_ps :86-100 */
{
    const __m256 z = _mm256_sub_ps(_mm256_mul_ps(randf8(s), SET1(2.0f)), SET1(1.0f));
    const __m256 a = _mm256_mul_ps(randf8(s), SET1(2.0f * 3.14159265359f));
    const __m256 r = _mm256_sqrt_ps(_mm256_sub_ps(SET1(1.0f), _mm256_mul_ps(z, z)));
    return mk8(_mm256_mul_ps(r, _ZGVdN8v_cosf(a)), _mm256_mul_ps(r, _ZGVdN8v_sinf(a)), z);
}

/* TestQuadTrace (simd.cpp:109-227) */
static inline __m256 quad8(v8 p, v8 dir, hit8* info, v8 a, v8 b, v8 c, v8 d)
{
    __m256 early = _mm256_setzero_ps();
    v8 normal = normalize8(cross8(sub8(c, a), sub8(c, b)));
    {
        const __m256 cond = gt(dot8(normal, dir), _mm256_setzero_ps());
        normal = blend8(normal, muls8(normal, SET1(-1.0f)), cond);
        const v8 t = d;
        d = blend8(d, a, cond);
        a = blend8(a, t, cond);
        const v8 t2 = b;
        b = blend8(b, c, cond);
        c = blend8(c, t2, cond);
    }
    const v8 q = add8(p, dir);
    const v8 pq = sub8(q, p), pa = sub8(a, p), pb = sub8(b, p), pc = sub8(c, p);
    v8 ip;
    const v8 m = cross8(pc, pq);
    __m256 v = dot8(pa, m);
    const __m256 vnn = ge(v, _mm256_setzero_ps());
    {
        __m256 u = _mm256_sub_ps(_mm256_setzero_ps(), dot8(pb, m));
        early = or8(early, and8(vnn, lt(u, _mm256_setzero_ps())));
        __m256 w = dot8(cross8(pq, pb), pa);
        early = or8(early, and8(vnn, lt(w, _mm256_setzero_ps())));
        const __m256 den = _mm256_div_ps(SET1(1.0f), _mm256_add_ps(_mm256_add_ps(u, v), w));
        u = _mm256_mul_ps(u, den);
        v = _mm256_blendv_ps(v, _mm256_mul_ps(v, den), vnn);
        w = _mm256_mul_ps(w, den);
        ip = add8(add8(muls8(a, u), muls8(b, v)), muls8(c, w));
    }
    {
        const v8 pd = sub8(d, p);
        __m256 u = dot8(pd, m);
        early = or8(early, and8(not8(vnn), lt(u, _mm256_setzero_ps())));
        __m256 w = dot8(cross8(pq, pa), pd);
        early = or8(early, and8(not8(vnn), lt(w, _mm256_setzero_ps())));
        v = _mm256_sub_ps(_mm256_setzero_ps(), v);
        const __m256 den = _mm256_div_ps(SET1(1.0f), _mm256_add_ps(_mm256_add_ps(u, v), w));
        u = _mm256_mul_ps(u, den);
        v = _mm256_mul_ps(v, den);
        w = _mm256_mul_ps(w, den);
        ip = blend8(ip, add8(add8(muls8(a, u), muls8(d, v)), muls8(c, w)), not8(vnn));
    }
    const __m256 absmask = _mm256_castsi256_ps(_mm256_set1_epi32(0x7fffffff));
    const __m256 c1 = gt(_mm256_and_ps(dir.x, absmask), _mm256_setzero_ps());
    const __m256 c2 = gt(_mm256_and_ps(dir.y, absmask), _mm256_setzero_ps());
    __m256 dist = _mm256_div_ps(_mm256_sub_ps(ip.z, p.z), dir.z);
    dist = _mm256_blendv_ps(dist, _mm256_div_ps(_mm256_sub_ps(ip.y, p.y), dir.y), c2);
    dist = _mm256_blendv_ps(dist, _mm256_div_ps(_mm256_sub_ps(ip.x, p.x), dir.x), c1);
    const __m256 cond = and8(not8(early), and8(gt(dist, SET1(0.01f)), lt(dist, info->dist)));
    info->dist = _mm256_blendv_ps(info->dist, dist, cond);
    info->normal = blend8(info->normal, normal, cond);
    return cond;
}

/* TestSphereTrace (simd.cpp:229-290) */
static inline __m256 sphere8(v8 p, v8 dir, hit8* info, float cx, float cy, float cz, float r)
{
    const v8 ctr = set8(cx, cy, cz);
    const v8 m = sub8(p, ctr);
    const __m256 b = dot8(m, dir);
    const __m256 c = _mm256_sub_ps(dot8(m, m), SET1(r * r));
    __m256 early = and8(gt(c, _mm256_setzero_ps()), gt(b, _mm256_setzero_ps()));
    const __m256 discr = _mm256_sub_ps(_mm256_mul_ps(b, b), c);
    early = or8(early, lt(discr, _mm256_setzero_ps()));
    const __m256 sq = _mm256_sqrt_ps(discr);
    __m256 dist = _mm256_sub_ps(_mm256_sub_ps(_mm256_setzero_ps(), b), sq);
    const __m256 inside = lt(dist, _mm256_setzero_ps());
    dist = _mm256_blendv_ps(dist, _mm256_add_ps(_mm256_sub_ps(_mm256_setzero_ps(), b), sq), inside);
    const __m256 check = and8(not8(early), and8(gt(dist, SET1(0.01f)), lt(dist, info->dist)));
    info->dist = _mm256_blendv_ps(info->dist, dist, check);
    const v8 n = muls8(normalize8(sub8(add8(p, muls8(dir, dist)), ctr)), _mm256_blendv_ps(SET1(1.0f), SET1(-1.0f), inside));
    info->normal = blend8(info->normal, n, check);
    return check;
}

typedef struct { float v[4][3]; float albedo[3]; float emissive[3]; } quad_desc;

/* the scalar file's scene (scalar.cpp:186-287; translation (0,0,10) folded in) */
static const quad_desc k_quads[6] = {
    {{{-12.6f, -12.6f, 35.0f}, {12.6f, -12.6f, 35.0f}, {12.6f, 12.6f, 35.0f}, {-12.6f, 12.6f, 35.0f}}, {0.7f, 0.7f, 0.7f}, {0, 0, 0}},
    {{{-12.6f, -12.45f, 35.0f}, {12.6f, -12.45f, 35.0f}, {12.6f, -12.45f, 25.0f}, {-12.6f, -12.45f, 25.0f}}, {0.7f, 0.7f, 0.7f}, {0, 0, 0}},
    {{{-12.6f, 12.5f, 35.0f}, {12.6f, 12.5f, 35.0f}, {12.6f, 12.5f, 25.0f}, {-12.6f, 12.5f, 25.0f}}, {0.7f, 0.7f, 0.7f}, {0, 0, 0}},
    {{{-12.5f, -12.6f, 35.0f}, {-12.5f, -12.6f, 25.0f}, {-12.5f, 12.6f, 25.0f}, {-12.5f, 12.6f, 35.0f}}, {0.7f, 0.1f, 0.1f}, {0, 0, 0}},
    {{{12.5f, -12.6f, 35.0f}, {12.5f, -12.6f, 25.0f}, {12.5f, 12.6f, 25.0f}, {12.5f, 12.6f, 35.0f}}, {0.1f, 0.7f, 0.1f}, {0, 0, 0}},
    {{{-5.0f, 12.4f, 32.5f}, {5.0f, 12.4f, 32.5f}, {5.0f, 12.4f, 27.5f}, {-5.0f, 12.4f, 27.5f}}, {0.0f, 0.0f, 0.0f}, {20.0f, 18.0f, 14.0f}},
};
static const float k_spheres[3][4] = {{-9.0f, -9.5f, 30.0f, 3.0f}, {0.0f, -9.5f, 30.0f, 3.0f}, {9.0f, -9.5f, 30.0f, 3.0f}};
static const float k_sphere_albedo[3][3] = {{0.9f, 0.9f, 0.75f}, {0.9f, 0.75f, 0.9f}, {0.75f, 0.9f, 0.9f}};

static inline void scene8(v8 p, v8 dir, hit8* h, __m256 terminated)   /* TestSceneTrace :292-383 */
{
    const __m256 live = not8(terminated);
    for (int i = 0; i < 6; ++i) {
        const quad_desc* q = &k_quads[i];
        const __m256 cond = and8(live, quad8(p, dir, h, set8(q->v[0][0], q->v[0][1], q->v[0][2]),
                                             set8(q->v[1][0], q->v[1][1], q->v[1][2]),
                                             set8(q->v[2][0], q->v[2][1], q->v[2][2]),
                                             set8(q->v[3][0], q->v[3][1], q->v[3][2])));
        h->albedo = blend8(h->albedo, set8(q->albedo[0], q->albedo[1], q->albedo[2]), cond);
        h->emissive = blend8(h->emissive, set8(q->emissive[0], q->emissive[1], q->emissive[2]), cond);
    }
    for (int i = 0; i < 3; ++i) {
        const __m256 cond =
            and8(live, sphere8(p, dir, h, k_spheres[i][0], k_spheres[i][1], k_spheres[i][2], k_spheres[i][3]));
        h->albedo = blend8(h->albedo, set8(k_sphere_albedo[i][0], k_sphere_albedo[i][1], k_sphere_albedo[i][2]), cond);
        h->emissive = blend8(h->emissive, set8(0, 0, 0), cond);
    }
}

static inline v8 color8(v8 pos, v8 dir, __m256i* rng, int bounces)   /* GetColorForRay :386-428 */
{
    v8 ret = set8(0, 0, 0), T = set8(1, 1, 1);
    __m256 brk = _mm256_setzero_ps();
    for (int b = 0; b <= bounces; ++b) {
        hit8 h;
        memset(&h, 0, sizeof(h));
        h.dist = SET1(10000.0f);
        scene8(pos, dir, &h, brk);
        const __m256 prev = brk;
        brk = _mm256_cmp_ps(h.dist, SET1(10000.0f), _CMP_EQ_OQ);
        ret = blend8(ret, add8(ret, set8(0.1f, 0.1f, 0.1f)), and8(not8(prev), brk));
        pos = blend8(add8(add8(pos, muls8(dir, h.dist)), muls8(h.normal, SET1(0.01f))), pos, brk);
        dir = blend8(normalize8(add8(h.normal, ruv8(rng))), dir, brk);
        ret = blend8(add8(ret, mul8(h.emissive, T)), ret, brk);
        T = blend8(mul8(T, h.albedo), T, brk);
    }
    return ret;
}

typedef struct {
    float* buf;
    int32_t w, h, ntx, nty, tw, th, bounces;
    uint32_t frame;
    atomic_int next;
} job8;

static void tile8(job8* j, int tx, int ty)   /* RenderTile :500-545 */
{
    const __m256 W = SET1((float)j->w), H = SET1((float)j->h);
    const __m256 lanes = _mm256_set_ps(7.f, 6.f, 5.f, 4.f, 3.f, 2.f, 1.f, 0.f);
    float* pos = j->buf + (size_t)ty * j->th * j->w * 3 + (size_t)tx * j->tw * j->th * 3;
    const float cam = 1.0f / tanf(90.0f * 0.5f * 3.14159265359f / 180.0f);
    const __m256 t = SET1(1.0f / ((float)j->frame + 1.0f));
    for (int Y = ty * j->th; Y < (ty + 1) * j->th; ++Y) {
        const __m256 fy = SET1((float)(j->h - 1 - Y));
        for (int X = tx * j->tw; X < (tx + 1) * j->tw; X += 8) {
            const __m256 fx = _mm256_add_ps(SET1((float)X), lanes);
            __m256i rng = _mm256_or_si256(   /* :435-445 */
                _mm256_add_epi32(_mm256_add_epi32(_mm256_mullo_epi32(_mm256_cvtps_epi32(fx), _mm256_set1_epi32(1973)),
                                                  _mm256_mullo_epi32(_mm256_cvtps_epi32(fy), _mm256_set1_epi32(9277))),
                                 _mm256_set1_epi32((int)(j->frame * 26699u))),
                _mm256_set1_epi32(1));
            const __m256 tx2 = _mm256_sub_ps(_mm256_mul_ps(_mm256_div_ps(fx, W), SET1(2.0f)), SET1(1.0f));
            __m256 ty2 = _mm256_sub_ps(_mm256_mul_ps(_mm256_div_ps(fy, H), SET1(2.0f)), SET1(1.0f));
            ty2 = _mm256_div_ps(ty2, _mm256_div_ps(W, H));
            const v8 dir = normalize8(mk8(tx2, ty2, SET1(cam)));
            const v8 c = color8(set8(0, 0, 0), dir, &rng, j->bounces);
            float* R = pos;
            const v8 last = mk8(_mm256_loadu_ps(R), _mm256_loadu_ps(R + 8), _mm256_loadu_ps(R + 16));
            const v8 out = add8(last, muls8(sub8(c, last), t));   /* lerp (mathlib.h:763) */
            _mm256_storeu_ps(R, out.x);
            _mm256_storeu_ps(R + 8, out.y);
            _mm256_storeu_ps(R + 16, out.z);
            pos += 24;
        }
    }
}

static void* worker8(void* arg)
{
    job8* j = (job8*)arg;
    const int n = j->ntx * j->nty;
    for (;;) {
        const int k = atomic_fetch_add(&j->next, 1);
        if (k >= n) break;
        tile8(j, k % j->ntx, k / j->ntx);
    }
    return NULL;
}

int ptc_simd_supported(void) { return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma"); }

/* Accumulate frames [frame_first, frame_first + nframes) into buf (tile-major planar8, like
 * DemofoxRenderSimtPooled), with nthreads workers.  0 on success. */
int ptc_render_simd_tiled(float* buf, int32_t w, int32_t h, int32_t ntx, int32_t nty, uint32_t frame_first,
                          int32_t nframes, int32_t bounces, int32_t nthreads)
{
    if (!ptc_simd_supported()) return -2;
    if (!buf || w <= 0 || h <= 0 || ntx <= 0 || nty <= 0 || w % ntx || h % nty || (w / ntx) % 8 || bounces < 0)
        return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int32_t f = 0; f < nframes; ++f) {
        job8 j = {buf, w, h, ntx, nty, w / ntx, h / nty, bounces, frame_first + (uint32_t)f, 0};
        atomic_init(&j.next, 0);
        int started = 0;
        for (int t = 0; t < nthreads - 1; ++t) {
            if (pthread_create(&th[t], NULL, worker8, &j)) break;
            ++started;
        }
        worker8(&j);
        for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    }
    return 0;
}
