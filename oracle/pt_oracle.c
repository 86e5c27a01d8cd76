/* oracle/pt_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU parity checker (see pt_oracle.h).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math; x86-64 SSE float, so every
 * f32 op rounds once, like the reference's MSVC /fp:precise build).
 */
#include "pt_oracle.h"
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define PTO_MIN_HIT 0.01f         /* c_minimumRayHitTime  scalar.cpp:6  */
#define PTO_NUDGE 0.01f           /* c_rayPosNormalNudge  scalar.cpp:10 */
#define PTO_SUPER_FAR 10000.0f    /* c_superFar           scalar.cpp:13 */
#define PTO_FOV_DEG 90.0f         /* c_FOVDegrees         scalar.cpp:16 */
#define PTO_PI 3.14159265359f     /* c_pi                 scalar.cpp:24 */
#define PTO_TWOPI (2.0f * PTO_PI) /* c_twopi              scalar.cpp:25 */
#define PTO_NQUADS 6
#define PTO_NSPHERES 3

typedef struct { float v[4][3]; float n[3]; } pto_quad;
typedef struct { float albedo[3]; float emissive[3]; } pto_mat;

/* Scene of TestSceneTrace (scalar.cpp:186-287) with sceneTranslation (0,0,10) folded in using the
 * same f32 adds; quad normals = normalize(cross(c-a, c-b)) with the same ops as :68. */
static pto_quad g_quads[PTO_NQUADS];
static float g_spheres[PTO_NSPHERES][4];
static pto_mat g_mats[PTO_NQUADS + PTO_NSPHERES];
static float g_cam_dist;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static const float k_quad_src[PTO_NQUADS][4][3] = {
    {{-12.6f, -12.6f, 25.0f}, {12.6f, -12.6f, 25.0f}, {12.6f, 12.6f, 25.0f}, {-12.6f, 12.6f, 25.0f}},     /* back wall :194-197 */
    {{-12.6f, -12.45f, 25.0f}, {12.6f, -12.45f, 25.0f}, {12.6f, -12.45f, 15.0f}, {-12.6f, -12.45f, 15.0f}}, /* floor :207-210 */
    {{-12.6f, 12.5f, 25.0f}, {12.6f, 12.5f, 25.0f}, {12.6f, 12.5f, 15.0f}, {-12.6f, 12.5f, 15.0f}},     /* ceiling :220-223 */
    {{-12.5f, -12.6f, 25.0f}, {-12.5f, -12.6f, 15.0f}, {-12.5f, 12.6f, 15.0f}, {-12.5f, 12.6f, 25.0f}}, /* left :233-236 */
    {{12.5f, -12.6f, 25.0f}, {12.5f, -12.6f, 15.0f}, {12.5f, 12.6f, 15.0f}, {12.5f, 12.6f, 25.0f}},     /* right :246-249 */
    {{-5.0f, 12.4f, 22.5f}, {5.0f, 12.4f, 22.5f}, {5.0f, 12.4f, 17.5f}, {-5.0f, 12.4f, 17.5f}},         /* light :259-262 */
};
static const float k_sphere_src[PTO_NSPHERES][4] = {
    {-9.0f, -9.5f, 20.0f, 3.0f}, {0.0f, -9.5f, 20.0f, 3.0f}, {9.0f, -9.5f, 20.0f, 3.0f}};  /* :270,276,282 */
static const float k_albedo[PTO_NQUADS + PTO_NSPHERES][3] = {
    {0.7f, 0.7f, 0.7f}, {0.7f, 0.7f, 0.7f}, {0.7f, 0.7f, 0.7f}, {0.7f, 0.1f, 0.1f}, {0.1f, 0.7f, 0.1f},
    {0.0f, 0.0f, 0.0f}, {0.9f, 0.9f, 0.75f}, {0.9f, 0.75f, 0.9f}, {0.75f, 0.9f, 0.9f}};
/* light emissive = mul(f32x3{1.0f, 0.9f, 0.7f}, 20.0f) (:266) -- computed below with the same mul. */

static void pto_init_scene(void)
{
    const float tr[3] = {0.0f, 0.0f, 10.0f};
    for (int i = 0; i < PTO_NQUADS; ++i) {
        pto_quad* q = &g_quads[i];
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 3; ++j) q->v[k][j] = k_quad_src[i][k][j] + tr[j];
        const float* a = q->v[0]; const float* b = q->v[1]; const float* c = q->v[2];
        float e1[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
        float e2[3] = {c[0] - b[0], c[1] - b[1], c[2] - b[2]};
        float cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        float inv = 1.0f / sqrtf((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
        q->n[0] = cr[0] * inv; q->n[1] = cr[1] * inv; q->n[2] = cr[2] * inv;
    }
    for (int i = 0; i < PTO_NSPHERES; ++i) {
        for (int j = 0; j < 3; ++j) g_spheres[i][j] = k_sphere_src[i][j] + tr[j];
        g_spheres[i][3] = k_sphere_src[i][3] + 0.0f;
    }
    for (int i = 0; i < PTO_NQUADS + PTO_NSPHERES; ++i) {
        memcpy(g_mats[i].albedo, k_albedo[i], 12);
        memset(g_mats[i].emissive, 0, 12);
    }
    g_mats[5].emissive[0] = 1.0f * 20.0f; g_mats[5].emissive[1] = 0.9f * 20.0f; g_mats[5].emissive[2] = 0.7f * 20.0f;
    g_cam_dist = 1.0f / tanf(PTO_FOV_DEG * 0.5f * PTO_PI / 180.0f);   /* scalar.cpp:338 */
}

uint32_t pto_wang_hash(uint32_t* s)
{
    uint32_t x = *s;
    x = (uint32_t)(x ^ 61u) ^ (uint32_t)(x >> 16);
    x *= 9u;
    x = x ^ (x >> 4);
    x *= 0x27d4eb2du;
    x = x ^ (x >> 15);
    *s = x;
    return x;
}

float pto_randomf(uint32_t* s) { return (float)pto_wang_hash(s) / 4294967296.0f; }

uint32_t pto_seed(uint32_t x, uint32_t y, uint32_t frame)
{
    return (uint32_t)(x * 1973u + y * 9277u + frame * 26699u) | 1u;
}

/* texture.cpp:101-139, one lane (TexelFetch :6-14).  atan2/asin on f32 resolve to the float
 * overloads under MSVC (see build_ref.sh), i.e. atan2f/asinf here. */
void pto_env_sample(const pto_env* env, const float d[3], float o[3])
{
    float u = atan2f(d[2], d[0]);
    float v = asinf(d[1]);
    u = u * 0.1591f; v = v * 0.3183f;
    u = u + 0.5f; v = v + 0.5f;
    u -= (float)(int32_t)u;
    v -= (float)(int32_t)v;
    if (u >= 0.0f && u < 1.0f && v >= 0.0f && v < 1.0f) {
        int32_t row = (int32_t)(v * (float)(env->height - 1));
        int32_t col = (int32_t)(u * (float)(env->width - 1));
        const float* t = env->data + 3 * ((size_t)row * (size_t)env->width + (size_t)col);
        o[0] = t[0]; o[1] = t[1]; o[2] = t[2];
    } else {
        o[0] = o[1] = o[2] = 0.0f;
    }
}

/* ---- instantiation 1: plain (timed CPU baseline / checker) ---- */
#define SFX(n) n##_plain
#define CNT(n) ((void)0)
#define CNTS(n) ((void)0)
#define CNT_T(n) ((void)0)
#define CNT_SEG() ((void)0)
#define CNT_ESC() ((void)0)
#define CNT_SAMP() ((void)0)
#define CNT_MARK() ((void)0)
#define CNT_PRIM() ((void)0)
#define CNT_SHARED(n) ((void)0)
#define CNT_SHARED_PRIM(d) ((void)0)
#include "pt_oracle_core.inc"
#undef SFX
#undef CNT
#undef CNTS
#undef CNT_T
#undef CNT_SEG
#undef CNT_ESC
#undef CNT_SAMP
#undef CNT_MARK
#undef CNT_PRIM
#undef CNT_SHARED
#undef CNT_SHARED_PRIM

/* ---- instantiation 2: counted (single thread) ---- */
static pto_counts* g_cnt;
static uint64_t g_mark;
#define SFX(n) n##_counted
#define CNT(n) (g_cnt->flops_segment += (uint64_t)(n))
#define CNTS(n) (g_cnt->flops_sample += (uint64_t)(n))
#define CNT_T(n) (g_cnt->transcendentals += (uint64_t)(n))
#define CNT_SEG() (g_cnt->segments++)
#define CNT_ESC() (g_cnt->escaped++)
#define CNT_SAMP() (g_cnt->samples++)
#define CNT_MARK() (g_mark = g_cnt->flops_segment)
#define CNT_PRIM() (g_cnt->flops_segment_primary += g_cnt->flops_segment - g_mark, g_cnt->segments_primary++)
#define CNT_SHARED(n) (g_cnt->flops_shared += (uint64_t)(n))
#define CNT_SHARED_PRIM(d) (g_cnt->flops_shared += g_cnt->flops_segment - g_mark - (uint64_t)(d))
#include "pt_oracle_core.inc"

static void ruv_unused_guard(void) { (void)ruv_counted; (void)ruv_plain; }

void pto_random_unit_vector(uint32_t* s, float o[3])
{
    pthread_once(&g_once, pto_init_scene);
    ruv_plain(s, o);
}

/* The quad stage of TestSceneTrace alone (scalar.cpp:192-261): the six TestQuadTrace calls in
 * order from info.dist = c_superFar.  *id = the last quad that updated (-1 none), *flipped = its
 * normal was flipped (:69-80).  Returns the resulting info.dist. */
float pto_trace_quads(const float P[3], const float D[3], int* id, int* flipped)
{
    pthread_once(&g_once, pto_init_scene);
    hit_t_plain h;
    h.dist = PTO_SUPER_FAR;
    *id = -1;
    *flipped = 0;
    for (int i = 0; i < PTO_NQUADS; ++i)
        if (quad_plain(P, D, &h, &g_quads[i])) {
            *id = i;
            *flipped = h.n[0] != g_quads[i].n[0] || h.n[1] != g_quads[i].n[1] || h.n[2] != g_quads[i].n[2];
        }
    return h.dist;
}

/* The whole TestSceneTrace (scalar.cpp:186-287): dist, hit normal, material id (-1 on a miss). */
float pto_trace_scene(const float P[3], const float D[3], float n_out[3], int* id)
{
    pthread_once(&g_once, pto_init_scene);
    hit_t_plain h;
    h.dist = PTO_SUPER_FAR;
    *id = -1;
    for (int i = 0; i < PTO_NQUADS; ++i)
        if (quad_plain(P, D, &h, &g_quads[i])) *id = i;
    for (int i = 0; i < PTO_NSPHERES; ++i)
        if (sphere_plain(P, D, &h, g_spheres[i])) *id = PTO_NQUADS + i;
    n_out[0] = h.n[0]; n_out[1] = h.n[1]; n_out[2] = h.n[2];
    return h.dist;
}

/* The sky tiles of the diffuse kernel (csrc/pt_kernel.hip sky_ray): 8x8 tiles of the p->nrows x
 * p->width buffer (rows p->row_start + r * p->row_stride) whose camera rays all have |D.x| or |D.y|
 * > slope * D.z skip those rays' TestSceneTrace.  Returns how many camera rays that is and, in
 * *flops, what their TestSceneTrace costs the reference (the counted instantiation's accounting) --
 * the work the kernel does not execute, for the bench's roofline (roofline.py). */
uint64_t pto_sky_skipped(const pto_params* p, float slope, uint64_t* flops)
{
    pthread_once(&g_once, pto_init_scene);
    const float W = (float)p->width, H = (float)p->height, aspect = W / H;
    uint64_t n = 0, fl = 0;
    pto_counts c;
    pto_counts* const saved = g_cnt;
    for (int32_t ty = 0; ty < (p->nrows + 7) / 8; ++ty)
        for (int32_t tx = 0; tx < (p->width + 7) / 8; ++tx) {
            float D[64][3];
            int m = 0, sky = 1;
            for (int k = 0; k < 64 && sky; ++k) {
                const int32_t x = tx * 8 + (k & 7), r = ty * 8 + (k >> 3);
                if (x >= p->width || r >= p->nrows) continue;
                const float fx = (float)x, fy = (float)(p->height - 1 - (p->row_start + r * p->row_stride));
                float t[3] = {(fx / W) * 2.0f - 1.0f, ((fy / H) * 2.0f - 1.0f) / aspect, g_cam_dist - 0.0f};
                const float inv = 1.0f / sqrtf((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
                D[m][0] = t[0] * inv; D[m][1] = t[1] * inv; D[m][2] = t[2] * inv;
                sky = fabsf(D[m][0]) > slope * D[m][2] || fabsf(D[m][1]) > slope * D[m][2];
                ++m;
            }
            if (!sky || m == 0) continue;
            for (int k = 0; k < m; ++k) {
                memset(&c, 0, sizeof c);
                g_cnt = &c;
                hit_t_counted h;
                h.dist = PTO_SUPER_FAR;
                const float P[3] = {0.0f, 0.0f, 0.0f};
                scene_counted(P, D[k], &h);
                fl += c.flops_segment;
            }
            n += (uint64_t)m;
        }
    g_cnt = saved;
    if (flops) *flops = fl;
    return n;
}

static int pto_check(const float* buf, const pto_params* p)
{
    (void)ruv_unused_guard;
    if (!buf || !p) return -1;
    if (p->width <= 0 || p->height <= 0 || p->nrows < 0 || p->nframes < 0) return -1;
    if (p->row_stride <= 0 || p->row_start < 0) return -1;
    if (p->nrows > 0 && p->row_start + (int64_t)(p->nrows - 1) * p->row_stride >= p->height) return -1;
    if (p->num_bounces < 0 || p->frame_first < 1) return -1;
    if ((uint64_t)p->frame_first + (uint64_t)p->nframes > (1u << 24)) return -1;  /* f32 iFrame exact */
    if (p->env && (!p->env->data || p->env->width < 1 || p->env->height < 1)) return -1;
    return 0;
}

typedef struct { float* buf; const pto_params* p; int tid, nt; } pto_job;

static void* pto_worker(void* arg)
{
    pto_job* j = (pto_job*)arg;
    for (int32_t r = j->tid; r < j->p->nrows; r += j->nt)
        row_plain(j->buf + (size_t)r * 3 * (size_t)j->p->width, j->p->row_start + r * j->p->row_stride, j->p);
    return NULL;
}

int pto_render(float* buf, const pto_params* p)
{
    if (pto_check(buf, p)) return -1;
    pthread_once(&g_once, pto_init_scene);
    int nt = p->nthreads > 1 ? p->nthreads : 1;
    if (nt > 256) nt = 256;
    if (nt == 1) {
        pto_job j = {buf, p, 0, 1};
        pto_worker(&j);
        return 0;
    }
    pthread_t th[256];
    pto_job jobs[256];
    for (int t = 0; t < nt; ++t) {
        jobs[t].buf = buf; jobs[t].p = p; jobs[t].tid = t; jobs[t].nt = nt;
        if (pthread_create(&th[t], NULL, pto_worker, &jobs[t])) { nt = t; break; }
    }
    for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
    return 0;
}

int pto_render_counted(float* buf, const pto_params* p, pto_counts* c)
{
    if (pto_check(buf, p) || !c) return -1;
    pthread_once(&g_once, pto_init_scene);
    memset(c, 0, sizeof(*c));
    g_cnt = c;
    for (int32_t r = 0; r < p->nrows; ++r)
        row_counted(buf + (size_t)r * 3 * (size_t)p->width, p->row_start + r * p->row_stride, p);
    g_cnt = NULL;
    return 0;
}
