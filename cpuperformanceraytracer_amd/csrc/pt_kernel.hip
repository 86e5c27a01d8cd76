// pt_kernel.hip -- MI355X (gfx950) path-tracing kernel for the demofox diffuse+emissive hot path.
//
// Reference hot path (paths relative to /root/reference/CPUPerformanceRayTracer/):
//   DemofoxRenderScalar  demofox_path_tracing_scalar.cpp:785-820   (parity semantics)
//   mainImage            :329-360   camera ray + per-(pixel, frame) Wang-hash seed
//   GetColorForRay       :289-327   bounce loop, ambient on miss, emissive*throughput
//   TestSceneTrace       :186-287   6 quads + 3 spheres, fixed order, strict '<' closest hit
//   TestQuadTrace        :65-143    TestSphereTrace :145-184   RandomUnitVector :42-50
//   DemofoxRenderSimd    demofox_path_tracing_simd.cpp:468-514    (north-star structure/layout)
//   RenderTile           demofox_path_tracing_simd_tiled.cpp:489-535 (tile surface/layout)
//
// Design (DESIGN.md has the numbers):
//   * a lane renders a pixel's nframes samples IN FRAME ORDER and applies the reference's
//     progressive lerp after each, so a launch of S frames is bit-identical to S calls of
//     DemofoxRenderScalar.  The accumulator is read once and written once per launch.
//   * the camera ray and its first TestSceneTrace + bounce-0 shading are the same for every frame
//     of a pixel (no jitter; the RNG is first drawn after them), so they run once per pixel and
//     every sample starts at bounce 1 from the saved state (PixelHit, LDS).
//   * persistent waves + path regeneration: the bounce, sample and pixel loops are flattened into
//     one loop of "segments" (one TestSceneTrace each).  A lane whose sample ends starts its next
//     sample, and a lane whose pixel ends takes the next pixel of the wave's 8x8 tile (ballot +
//     mbcnt), tiles coming from a per-launch atomic queue.  All 64 lanes trace every iteration
//     until the queue drains; the loop exits when __any(has_pixel) is false.
//   * scene geometry is compile-time constant, as in the reference's TestSceneTrace: vertex
//     coordinates are instruction literals (no loads, no registers, nothing to spill);
//     per-lane closest-hit material / normal lookups and the per-axis vertex components (indexed
//     by each lane's own ray) -> LDS tables.
//   * TestQuadTrace's vertex re-ordering (flip) and triangle choice become VGPR selects of the
//     ray-relative vertex vectors; only the intersection component the distance divides by is
//     evaluated (the reference computes all three and uses one).
//   * every f32 op is the reference's op, in its order, single-rounded: built with
//     -ffp-contract=off, denormals kept; '/' and sqrt are correctly rounded (pt_exactmath.h fast
//     paths, IEEE fallback outside their verified ranges); sin/cos via the glibc-exact double
//     evaluation (pt_sincosf.h).  Result: bit-identical to the CPU path.
#include "pt_kernel.h"
#include "pt_exactmath.h"
#include "pt_sincosf.h"
// the env-map lookup's atan2f/asinf with the guarded fast '/' and sqrt (bit-identical)
#define PT_IT_HD __device__ __forceinline__
#define PT_IT_DIV(a, b) pt::div_guarded((a), (b))
#define PT_IT_SQRT(x) pt::sqrt_guarded(x)
#include "pt_invtrig.h"
// certified texel cells (the exact atan2f/asinf above only where a cell is not certified)
#define PT_EC_HD __device__ __forceinline__
#define PT_EC_RCP(x) pt::rcp_rn(x)                       // q in (1, 2^40)
#define PT_EC_DIV(a, b) pt::div_rn((a), (b), pt::rcp_rn(b))   // |x|, |y| in [2^-20, 2^20)
#define PT_EC_SQRT(x) pt::sqrt_rn(x)                     // t >= 2^-21 where the value is used
#include "pt_envcert.h"
#include "pt_tile_queue.h"
#include "pt_guard.h"
#include "pt_tonemap.h"
#include "pt_output.h"
#include "pt_wave.h"
#include "pt_chain.h"
#include <math.h>
#include <algorithm>

namespace {

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 sel(bool c, V3 a, V3 b) { return v3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
// mathlib.h:64   dot = (x*x' + y*y') + z*z'
__device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// mathlib.h:768
__device__ __forceinline__ V3 cross(V3 u, V3 v)
{
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}

// ---- correctly rounded '/' and sqrt (pt_exactmath.h), an exact slow path outside the fast range ----
// Every reciprocal of the kernel has a proven operand range: unguarded rcp_rn where it is inside
// [2^-125, 2^125] (1/dD, the sphere normal, the lerp weights), rcp_x_nonneg where only the lower
// end can fail.
__device__ __forceinline__ float sqrt_x(float x) { return pt::sqrt_guarded(x); }
// RN(1/x) for an x that is >= 0 (or NaN) and provably <= 2^125: only the lower end of rcp_rn's range
// can fail (0, denormals), so one compare guards it.
__device__ __forceinline__ float rcp_x_nonneg(float x)
{
    float r = pt::rcp_rn(x);
    if (__builtin_expect(!(x >= 0x1p-125f), 0)) r = pt::rcp_tiny_rn(x);   // 0, denormals, NaN
    return r;
}
// a / b with y = RN(1/b) and b normal in [2^-125, 2^125]: exact whenever a/b is normal and
// |a| < 2^124; callers only use it where any other quotient is discarded by the reference's
// comparisons (see quad_test) or cannot occur (camera: 0 <= a <= 2^24).
__device__ __forceinline__ float div_x(float a, float b, float y) { return pt::div_rn(a, b, y); }

}  // namespace
#define PTQC_HD __device__ __forceinline__
#define PTQC_RCP_APPROX(x) pt::rcp_approx(x)
#define PTQC_RCP_EXACT(x) rcp_x_nonneg(x)   // quad_exact's weight sum: >= 0 and <= 3 x 9.2e3 (pt_quadcull.h)
#define PTQC_DIV_EXACT(a, b, y) div_x((a), (b), (y))
#define PTQC_FMA(a, b, c) __builtin_fmaf((a), (b), (c))
#include "pt_quadcull.h"
namespace {

// mathlib.h:750   normalize = v * (1 / sqrt(dot(v, v))).  Its arguments here are n + u (unit normal +
// unit vector: |v| <= 2) and the camera's (tx, ty, cam_dist): sqrt(dot) <= 2^125, and >= 0.
__device__ __forceinline__ V3 normalize(V3 v) { return mul(v, rcp_x_nonneg(sqrt_x(dot(v, v)))); }

// scalar.cpp:27-35 (logical shifts, wrapping u32)
__device__ __forceinline__ uint32_t wang_hash(uint32_t& s)
{
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
// scalar.cpp:37-40: f32(h) / 2^32 -- dividing by a power of two is an exact scaling
__device__ __forceinline__ float randomf(uint32_t& s) { return (float)wang_hash(s) * 0x1p-32f; }

// scalar.cpp:42-50 ; cosf/sinf == glibc's, see pt_sincosf.h
__device__ __forceinline__ V3 random_unit_vector(uint32_t& s)
{
    const float z = randomf(s) * 2.0f - 1.0f;
    const float a = randomf(s) * PT_TWOPI;
    const float r = sqrt_x(1.0f - z * z);
    float sa, ca;
    pt::sincosf_glibc(a, &sa, &ca);
    return v3(r * ca, r * sa, z);
}

// dot(n, D) > 0 (scalar.cpp:69) for the compile-time normal n.  For a signed unit axis n and finite
// D this is exactly the sign test of that component: the products with n's zero components are
// signed zeros, which neither change a non-zero sum nor make a zero sum positive.
__device__ __forceinline__ bool facing(V3 n, V3 D)
{
    if (n.x == 0.0f && n.z == 0.0f && n.y == 1.0f) return D.y > 0.0f;
    if (n.x == 0.0f && n.z == 0.0f && n.y == -1.0f) return D.y < 0.0f;
    if (n.y == 0.0f && n.z == 0.0f && n.x == 1.0f) return D.x > 0.0f;
    if (n.y == 0.0f && n.z == 0.0f && n.x == -1.0f) return D.x < 0.0f;
    if (n.x == 0.0f && n.y == 0.0f && n.z == 1.0f) return D.z > 0.0f;
    if (n.x == 0.0f && n.y == 0.0f && n.z == -1.0f) return D.z < 0.0f;
    return dot(n, D) > 0.0f;
}

// Per-quad, per-axis vertex components (A_k, B_k, C_k, D_k): indexed by the lane's axis.
struct alignas(16) AxisRow {   // (16-byte aligned: one ds_read_b128 per row)
    float a, b, c, d;
};
// The per-axis rows of a quad, s_axis[(q * 2 + fl) * 3 + k], for both vertex orders: row (q, fl, k)
// holds the components in the order after the facing flip, so the culled stage reads its quad's
// rows without selects (the six exact tests of the fallback read the unflipped ones, fl = 0).
template <bool QV>
constexpr int kAxisRowsPerQuad = 6;

// TestQuadTrace, scalar.cpp:65-143.  `pq` = (rayPos + rayDir) - rayPos (ray-constant, hoisted),
// `axis`/`dP`/`dD`/`yD` = the component :121-133 divides by, its ray origin, direction, RN(1/dir),
// `ax` = the quad's vertex components on that axis (its LDS row, read one quad ahead by quads_exact).
// On a closer hit: best = dist, id = q, flag = flipped.
template <class SC>
__device__ __forceinline__ void quad_test(int q, V3 P, V3 D, V3 pq, float dP, float dD, float yD, float& best, int& id,
                                          int& flag, AxisRow ax)
{
    const V3 n = v3(SC::qn[q][0], SC::qn[q][1], SC::qn[q][2]);
    const bool flip = facing(n, D);                           // :69-80 (flipped order d,c,b,a)
    const V3 PA = sub(v3(SC::qv[q][0][0], SC::qv[q][0][1], SC::qv[q][0][2]), P);
    const V3 PB = sub(v3(SC::qv[q][1][0], SC::qv[q][1][1], SC::qv[q][1][2]), P);
    const V3 PC = sub(v3(SC::qv[q][2][0], SC::qv[q][2][1], SC::qv[q][2][2]), P);
    const V3 PD = sub(v3(SC::qv[q][3][0], SC::qv[q][3][1], SC::qv[q][3][2]), P);
    const V3 pa = sel(flip, PD, PA), pb = sel(flip, PC, PB), pc = sel(flip, PB, PC), pd = sel(flip, PA, PD);
    const V3 m = cross(pc, pq);                               // :90
    float v = dot(pa, m);                                     // :91
    const bool t1 = v >= 0.0f;                                // :93 triangle a,b,c (else a,c,d)
    // :96 u = -dot(pb, m)  |  :109 u = dot(pd, m)
    const float tu = dot(sel(t1, pb, pd), m);
    float u = t1 ? -tu : tu;
    // :98 w = ScalarTriple(pq, pb, pa)  |  :111 w = ScalarTriple(pq, pa, pd)
    float w = dot(cross(pq, sel(t1, pb, pa)), sel(t1, pa, pd));
    v = t1 ? v : -v;                                          // :113
    // :104 / :118 intersectPos = u*a + v*e + w*c (e = b or d), component `axis` only; selected for
    // every lane BEFORE the divergent exit (inside the branch the LDS row's latency is exposed)
    const float ak = flip ? ax.d : ax.a;
    const float ck = flip ? ax.b : ax.c;
    const float ek = t1 ? (flip ? ax.c : ax.b) : (flip ? ax.a : ax.d);
    if (u < 0.0f || w < 0.0f) return;                         // :97,99,110,112
    // :100-103 / :114-117 (u, w >= 0 here and v >= 0 by the triangle choice: a sum >= 0, <= 3 x 9.2e3)
    const float denom = rcp_x_nonneg((u + v) + w);
    u *= denom;
    v *= denom;
    w *= denom;
    const float ip = (u * ak + v * ek) + w * ck;
    // :124/128/132 dist = (ip - rayPos_k) / rayDir_k.  A result that is not a normal number with
    // |dist| < 2^124 fails the test below under either division, so the fast quotient is exact
    // wherever the reference can keep it.
    const float dist = div_x(ip - dP, dD, yD);
    if (dist > PT_MIN_HIT && dist < best) {                   // :135-140
        best = dist;
        id = q;
        flag = flip ? 1 : 0;
    }
}

// TestSphereTrace, scalar.cpp:145-184 (the normal is produced later, only for the winner).
template <class SC>
__device__ __forceinline__ void sphere_test(int s, V3 P, V3 D, float& best, int& id, int& flag)
{
    const V3 m = sub(P, v3(SC::sph[s][0], SC::sph[s][1], SC::sph[s][2]));
    const float b = dot(m, D);
    const float c = dot(m, m) - SC::sph_r2[s];
    if (c > 0.0f && b > 0.0f) return;                         // :157
    const float discr = b * b - c;
    if (discr < 0.0f) return;                                 // :164
    const float sq = sqrt_x(discr);
    float dist = -b - sq;                                     // :169
    bool inside = false;
    if (dist < 0.0f) {                                        // :170-174
        inside = true;
        dist = -b + sq;
    }
    if (dist > PT_MIN_HIT && dist < best) {                   // :176-181
        best = dist;
        id = PT_NQUADS + s;
        flag = inside ? 1 : 0;
    }
}

// The three TestSphereTrace calls (scalar.cpp:274-285) with one root.  The spheres are pairwise
// disjoint balls (static_assert: 3 apart), so along a ray the chords of two balls it meets are
// disjoint, at least that far apart, and ordered like the centres' projections -b (see pt_v4.hip's
// closest-sphere stage for the argument).  Of the spheres the reference does not reject early --
// its exact operations -- only the one with the largest b can hold the smallest distance: its root
// and distance are evaluated as TestSphereTrace does and accepted against the running best.  A
// distance that fails c_minimumRayHitTime (origin within 0.01 of that surface) sends the ray to the
// sequential tests (rare; a sphere farther along could still be accepted).
constexpr bool scene_spheres_disjoint()
{
    for (int i = 0; i < PT_NSPHERES; ++i)
        for (int j = i + 1; j < PT_NSPHERES; ++j) {
            const float dx = DemofoxScene::sph[i][0] - DemofoxScene::sph[j][0];
            const float dy = DemofoxScene::sph[i][1] - DemofoxScene::sph[j][1];
            const float dz = DemofoxScene::sph[i][2] - DemofoxScene::sph[j][2];
            const float rr = DemofoxScene::sph[i][3] + DemofoxScene::sph[j][3] + 0.1f;
            if (!(dx * dx + dy * dy + dz * dz > rr * rr)) return false;
        }
    return true;
}
static_assert(scene_spheres_disjoint(), "the closest-sphere stage needs pairwise disjoint spheres");
#ifndef PT_SPHERE_FORCE_SEQ
#define PT_SPHERE_FORCE_SEQ 0   // test builds: every candidate ray takes the sequential fallback
#endif

// Which candidate has the largest b, without comparing b's: the spheres' centres lie on one line
// parallel to x in ascending x (static_assert below), so for two candidates i < j the exact
// b_i - b_j = (C_j - C_i).D = (x_j - x_i) D.x, and the chords (or the closest approaches, for a
// candidate the rounded discriminant admits at a tangent) are >= 3 - 1e-4 apart along the ray,
// far beyond the ~1e-5 rounding of the computed b's: for D.x > 0 the first candidate in index
// order has the largest b, for D.x < 0 the last one; D.x == 0 admits at most one candidate.
constexpr bool scene_spheres_on_x_line()
{
    for (int i = 1; i < PT_NSPHERES; ++i)
        if (!(DemofoxScene::sph[i][1] == DemofoxScene::sph[0][1] && DemofoxScene::sph[i][2] == DemofoxScene::sph[0][2] &&
              DemofoxScene::sph[i][0] > DemofoxScene::sph[i - 1][0]))
            return false;
    return true;
}
static_assert(scene_spheres_on_x_line(), "the closest-sphere order rule needs collinear spheres in ascending x");

template <class SC>
__device__ __forceinline__ void spheres_closest(V3 P, V3 D, float& best, int& id, int& flag)
{
    float bsel = 0.0f, dsel = 0.0f;
    int ksel = -1;
    const bool first = D.x > 0.0f;   // take the first candidate (else the last)
    bool found = false;
#pragma unroll
    for (int s = 0; s < PT_NSPHERES; ++s) {   // :150-164 exactly
        const V3 m = sub(P, v3(SC::sph[s][0], SC::sph[s][1], SC::sph[s][2]));
        const float b = dot(m, D);
        const float c = dot(m, m) - SC::sph_r2[s];
        const float discr = b * b - c;
        const bool cand = !((c > 0.0f && b > 0.0f) || discr < 0.0f);
        const bool take = cand && !(found && first);
        found = found || cand;
        bsel = take ? b : bsel;
        dsel = take ? discr : dsel;
        ksel = take ? s : ksel;
    }
    const float bmax = bsel;
    bool seq = false;
    if (ksel >= 0) {
        const float sq = sqrt_x(dsel);
        float dist = -bmax - sq;                                  // :169
        const bool inside = dist < 0.0f;                          // :170-174
        dist = inside ? -bmax + sq : dist;
        if (dist > PT_MIN_HIT && !PT_SPHERE_FORCE_SEQ) {
            if (dist < best) {                                    // :176-181
                best = dist;
                id = PT_NQUADS + ksel;
                flag = inside ? 1 : 0;
            }
        } else {
            seq = true;
        }
    }
    // (a divergent branch: s_cbranch_execz skips it for the whole wave when no lane needs it, with
    // no VALU vote)
    if (__builtin_expect(seq, 0)) {
#pragma unroll
        for (int k = 0; k < PT_NSPHERES; ++k) sphere_test<SC>(k, P, D, best, id, flag);
    }
}

template <int LAYOUT>
__device__ __forceinline__ size_t out_index(const PtJob& j, int lc, int lr)
{
    if (LAYOUT == PT_LAYOUT_INTERLEAVED) {
        return ((size_t)lr * (size_t)j.width + (size_t)(j.col0 + lc)) * 3u;
    } else if (LAYOUT == PT_LAYOUT_PLANAR8) {
        const int x = j.col0 + lc;
        return ((size_t)lr * (size_t)j.width + (size_t)(x & ~7)) * 3u + (size_t)(x & 7);
    } else {  // tiled: demofox_path_tracing_simd_tiled.cpp:499-504, 512-531 (global X, Y)
        const int x = j.col0 + lc;
        const int y = j.row_start + lr * j.row_stride;
        const int tx = x / j.tile_w, ty = y / j.tile_h;
        const int lx = x - tx * j.tile_w, ly = y - ty * j.tile_h;
        return (size_t)ty * j.tile_h * j.width * 3u + (size_t)tx * j.tile_w * j.tile_h * 3u +
               ((size_t)ly * j.tile_w + (size_t)(lx & ~7)) * 3u + (size_t)(lx & 7);
    }
}

// The elements of the job's buffer (the checked build's pixel guard, pt_guard.h): the job's rows for
// the row layouts; the whole image in whole tile rows for the tiled layout, whose index is global.
template <int LAYOUT>
__device__ __forceinline__ size_t pixel_extent(const PtJob& j)
{
    if (LAYOUT != PT_LAYOUT_TILED_PLANAR8) return (size_t)j.nrows * (size_t)j.width * 3u;
    const int rows = j.height > j.nrows ? j.height : j.nrows;
    return (size_t)((rows + j.tile_h - 1) / j.tile_h) * (size_t)j.tile_h * (size_t)j.width * 3u;
}

// Frame-constant camera terms (mainImage, scalar.cpp:338-351).
struct Camera {
    float W, H, yW, yH, aspect, yAspect, cam_dist;
};

// mainImage, scalar.cpp:338-351: the camera ray of pixel (fx, fy).  It does not depend on the
// frame (no jitter in the reference), so it is computed once per pixel.
// A wave-uniform divisor copied into a VGPR here, at the use: the division's fmas read it beside
// another scalar operand (one SGPR per VALU instruction), and a copy the compiler hoists out of
// the tile loop stays live across the pool and is spilled.
__device__ __forceinline__ float vgpr_here(float x)
{
    float v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}
__device__ __forceinline__ V3 camera_dir(const Camera& cam, float fx, float fy)
{
    const float tx = div_x(fx, vgpr_here(cam.W), cam.yW) * 2.0f - 1.0f;                       // :342
    float ty = div_x(fy, vgpr_here(cam.H), cam.yH) * 2.0f - 1.0f;
    ty = div_x(ty, vgpr_here(cam.aspect), cam.yAspect);                                         // :347
    return normalize(v3(tx - 0.0f, ty - 0.0f, cam.cam_dist - 0.0f));                            // :351
}

// A camera ray (origin 0, D.z > 0) with |D.x| > 0.51 D.z or |D.y| > 0.51 D.z misses every primitive
// of TestSceneTrace (scalar.cpp:186-287, translated scene):
//   back wall z = 35, |x|,|y| <= 12.6 needs |D.x|,|D.y| <= 0.36 D.z;
//   side walls x = +-12.5 (z in [25, 35]) need |D.x| / D.z = 12.5 / z <= 0.5, and |y| <= 12.6 at
//   z >= 25 then needs |D.y| / D.z <= 0.504;
//   floor y = -12.45 and ceiling y = 12.5 (z in [25, 35], |x| <= 12.6) need |D.y| / D.z <= 0.5 and
//   |D.x| / D.z <= 12.6 / 25 = 0.504;  the light (y = 12.4, |x| <= 5, z in [27.5, 32.5]) less;
//   the spheres (centres (-9 | 0 | 9, -9.5, 30), r = 3) subtend slopes below 0.41 (x) and 0.43 (y).
// The 0.51 threshold leaves >= 0.006 of slope (0.15 units at z = 25) to every boundary: the
// reference's rounding moves its triple products / discriminants by ~1e-3 of that scale, far
// inside it (the culled quad stage's bounds, pt_quadcull.h).  tests/native/check_sky.cpp checks it
// against the oracle's TestSceneTrace on dense direction grids around the thresholds.
constexpr float kSkySlope = 0.51f;
__device__ __forceinline__ bool sky_ray(V3 D)
{
    return __builtin_fabsf(D.x) > kSkySlope * D.z || __builtin_fabsf(D.y) > kSkySlope * D.z;
}
static_assert(DemofoxScene::qv[0][0][2] == 35.0f && DemofoxScene::qv[3][0][0] == -12.5f && DemofoxScene::qv[4][0][0] == 12.5f &&
                  DemofoxScene::qv[1][0][1] == -12.45f && DemofoxScene::qv[2][0][1] == 12.5f && DemofoxScene::qv[5][0][1] == 12.4f &&
                  DemofoxScene::sph[0][0] == -9.0f && DemofoxScene::sph[2][0] == 9.0f && DemofoxScene::sph[0][3] == 3.0f,
              "sky_ray's bounds are derived for the demofox scene");

// scalar.cpp:332: (uint32_t)(float)x * 1973 + (uint32_t)(float)y * 9277 + (uint32_t)iFrame * 26699, | 1.
// The pixel coordinates and the frame index are integers below 2^24 (the C ABI rejects larger
// images and frame counters), so every float round trip is the identity, and each wrapping u32
// product is the low word of the 24 x 24-bit product (v_mul_u32_u24, not the quarter-rate
// v_mul_lo_u32).
__device__ __forceinline__ uint32_t seed_int(uint32_t x, uint32_t y, uint32_t frame)
{
    return (__umul24(x, 1973u) + __umul24(y, 9277u) + __umul24(frame, 26699u)) | 1u;
}

// Closest hit of one ray against the scene (TestSceneTrace, scalar.cpp:186-287).
struct Hit {
    float best;   // c_superFar (10000) on a miss
    int id;       // primitive 0..8 (quads then spheres)
    int flag;     // quad: normal flipped; sphere: hit from inside
    int fb;       // the culled quad stage fell back to the six exact tests (counted by COUNT builds)
};

// The six exact quad tests in the reference's order (TestSceneTrace :192-261) into h.  Plain LDS
// loads of the per-quad rows: the compiler's waitcnt insertion places each wait before the row's
// first use.  (Until round 5 this was a software pipeline of inline-asm ds_read_b128 with its
// s_waitcnt in a separate asm statement: the compiler treats an asm output as defined when the
// load's statement ends and may copy or spill it before the data returns -- a hazard that depends on
// each template instance's register allocation.  The plain loads also spill less: the 6-wave
// presenting instance 2 VGPRs instead of 3, the counting instances 18-31 instead of 25-31, and four
// env per-tile instances reach 4 waves instead of 3.  tests/test_isa_lgkm.py checks every kernel of
// the built library for LDS return hazards.)
template <class SC, bool QV>
__device__ __forceinline__ void quads_exact(const AxisRow* s_axis, V3 P, V3 D, V3 pq, int axis, float dP, float dD,
                                            float yD, Hit& h)
{
    const AxisRow* rows = s_axis + axis;
#pragma unroll
    for (int q = 0; q < PT_NQUADS; ++q)
        quad_test<SC>(q, P, D, pq, dP, dD, yD, h.best, h.id, h.flag, rows[q * kAxisRowsPerQuad<QV>]);
}

// Per (quad, flip): the vertices in the reference's order after its facing flip (a, b, c, d or
// d, c, b, a), 12 floats in 3 float4 -- the exact test of the culling's chosen quad reads them.
constexpr int kQuadVecs = PT_NQUADS * 2 * 3;

// TestSceneTrace (scalar.cpp:186-287).  CAMERA: P is the camera origin (0, 0, 0).  QV: the culled
// quad's vertices come from the flip-ordered table s_qv (else from its three per-axis rows of
// s_axis, flipped by selects -- the env kernel, whose LDS has no room for the 576-B table at 4
// blocks per CU).  SPH_CLOSEST: the closest-sphere stage (else the three sequential tests).
template <class SC, bool CAMERA, bool QV = true, bool SPH_CLOSEST = true>
__device__ __forceinline__ Hit trace(const AxisRow* s_axis, const float4* s_qv, V3 P, V3 D)
{
    const V3 pq = sub(add(P, D), P);
    // :122-133 axis used for the hit distance (ray-constant)
    const int axis = fabsf(D.x) > 0.1f ? 0 : (fabsf(D.y) > 0.1f ? 1 : 2);
    const float dP = axis == 0 ? P.x : (axis == 1 ? P.y : P.z);
    const float dD = axis == 0 ? D.x : (axis == 1 ? D.y : D.z);
    // |dD| is in [0.1, 1.0001] (or NaN), so RN(1/dD) needs no range guard: D is normalize(v) of a
    // non-zero v (a unit vector within 1e-6; v = 0 gives NaN, and every test of a NaN ray fails as
    // in the reference), and axis 2 is taken only when |D.x|, |D.y| <= 0.1, i.e. |D.z| > 0.98
    const float yD = pt::rcp_rn(dD);
    Hit h{PT_SUPER_FAR, -1, 0, 0};
    // classify the six quads cheaply, test the one candidate W exactly (pt_quadcull.h); a ray whose
    // result is not certified runs the six exact tests (wave-uniform branch, rare).  Then the
    // spheres' updates in the reference's order (a sphere's distance does not depend on the
    // running best).
    const ptqc::F3 Pf{P.x, P.y, P.z}, pqf{pq.x, pq.y, pq.z};
    const ptqc::Cull cl = ptqc::cull<CAMERA>(Pf, pqf, dP, yD);
    const bool hasW = cl.k1 < ptqc::kNoKey;
    const int W = cl.k1 & 7;   // (any quad when there is no candidate: its result is then discarded)
    const uint32_t jW = (ptqc::kAxisBits >> (2u * (uint32_t)W)) & 3u;
    const float DjW = jW == 0 ? D.x : (jW == 1 ? D.y : D.z);
    const bool fl = DjW > 0.0f;                                          // :69 (unit normal +e_j)
    float4 r0, r1, r2;
    AxisRow ar;
    if (QV) {
        const float4* rec = s_qv + (W * 2 + (fl ? 1 : 0)) * 3;
        r0 = rec[0], r1 = rec[1], r2 = rec[2];
        ar = s_axis[(W * 2 + (fl ? 1 : 0)) * 3 + axis];   // flip-ordered: (ak, bk, ck, dk)
    } else {
        // the flip-ordered rows x, y, z of quad W: vertex v of the reference's order is (rx[v], ry[v], rz[v])
        const AxisRow* rr = s_axis + (W * 2 + (fl ? 1 : 0)) * 3;
        const AxisRow rx = rr[0], ry = rr[1], rz = rr[2];
        ar = rr[axis];
        r0 = make_float4(rx.a, ry.a, rz.a, rx.b);
        r1 = make_float4(ry.b, rz.b, rx.c, ry.c);
        r2 = make_float4(rz.c, rx.d, ry.d, rz.d);
    }
    const float ak = ar.a, bk = ar.b, ck = ar.c, dk = ar.d;
    float dist;
    const int code = ptqc::quad_exact<false>(Pf, pqf, ptqc::F3{r0.x, r0.y, r0.z}, ptqc::F3{r0.w, r1.x, r1.y},
                                      ptqc::F3{r1.z, r1.w, r2.x}, ptqc::F3{r2.y, r2.z, r2.w}, ak, bk, ck, dk, dP, dD,
                                      yD, PT_SUPER_FAR, dist);
    const bool ok = code == ptqc::kAccepted && ptqc::cull_beyond(cl, dist);
    bool unc = cl.unc || (hasW && !ok);
    if (hasW && ok) {
        h.best = dist;
        h.id = W;
        h.flag = fl ? 1 : 0;
    }
    if (__builtin_expect(unc, 0)) {   // (divergent: skipped by s_cbranch_execz when no lane needs it)
        h = Hit{PT_SUPER_FAR, -1, 0, 1};
        quads_exact<SC, QV>(s_axis, P, D, pq, axis, dP, dD, yD, h);
    }
    if (SPH_CLOSEST) {
        spheres_closest<SC>(P, D, h.best, h.id, h.flag);
    } else {
#pragma unroll
        for (int k = 0; k < PT_NSPHERES; ++k) sphere_test<SC>(k, P, D, h.best, h.id, h.flag);
    }
    return h;
}

// The hit normal the reference's TestQuadTrace/TestSphereTrace stored for the winning primitive.
__device__ __forceinline__ V3 hit_normal(const PtLdsPrim& pr, const Hit& h, V3 P, V3 D)
{
    if (h.id < PT_NQUADS) {
        const V3 n = v3(pr.nx, pr.ny, pr.nz);
        return h.flag ? mul(n, -1.0f) : n;                              // :71
    }
    const V3 c = sub(add(P, mul(D, h.best)), v3(pr.nx, pr.ny, pr.nz));  // :179
    // normalize(c) * (inside ? -1 : 1): (c_i * g) * -1 == c_i * -g exactly, so the sign goes on g.
    // c is the hit point minus the centre, |c| = the radius (3) up to rounding: the radicand and the
    // divisor are far inside the fast paths' ranges, no guard
    static_assert(DemofoxScene::sph[0][3] == 3.0f && DemofoxScene::sph[1][3] == 3.0f && DemofoxScene::sph[2][3] == 3.0f,
                  "the unguarded sphere normal assumes radius 3");
    const float g = pt::rcp_rn(pt::sqrt_rn(dot(c, c)));
    return mul(c, h.flag ? -g : g);
}

// s_prim[id] (id < PT_NPRIMS): the byte offset as a 24-bit multiply (v_mul_u32_u24, full rate)
// instead of the quarter-rate v_mul_lo_u32 the compiler emits for a 32-bit index times 48
__device__ __forceinline__ PtLdsPrim prim_at(const PtLdsPrim* s_prim, int id)
{
    return *(const PtLdsPrim*)((const char*)s_prim + __umul24((uint32_t)id, (uint32_t)sizeof(PtLdsPrim)));
}

// ret after bounce 0 (scalar.cpp:319): 0 + emissive * (1, 1, 1).  e * 1 == e, and 0 + e == e for
// every e but -0; the scene's emissive values are +0 or positive (pt_build_demofox_scene: memset, then
// the light's 20 x (1, 0.9, 0.7)), so the sum is the emissive value itself
__device__ __forceinline__ V3 emissive0(const PtLdsPrim& pr) { return v3(pr.er, pr.eg, pr.eb); }

// Miss radiance of the textured variant: EquirectangularTextureSample (texture.cpp:101-139), the
// per-lane nearest lookup demofox_path_tracing_simt_textured.cpp:408 adds (unweighted) on a miss.
// atan2f/asinf are the glibc algorithms (pt_invtrig.h); the texture is H x W x 3 f32, row 0 the
// bottom row (stbi flip-on-load, asset_loading.cpp:12), L2/MALL-resident.
// The texel cell is certified from short atan/asin polynomials (pt_envcert.h: the same row and column
// whenever it certifies); the glibc-exact angles run only for the rare uncertified cells (a divergent
// branch that s_cbranch_execz skips when no lane needs it).
__device__ __forceinline__ V3 env_sample(const float* __restrict__ env, int W, int H, V3 d)
{
    int32_t row, col;
    if (__builtin_expect(!pt::ec_cell_nearest(d.z, d.x, d.y, (float)(W - 1), (float)(H - 1), row, col), 0)) {
        float u = pt::atan2f_glibc(d.z, d.x);
        float v = pt::asinf_glibc(d.y);
        u = u * 0.1591f;                                        // uv *= invAtan
        v = v * 0.3183f;
        u = u + 0.5f;
        v = v + 0.5f;
        u -= (float)(int32_t)u;                                 // :115-116
        v -= (float)(int32_t)v;
        const bool in = u >= 0.0f && u < 1.0f && v >= 0.0f && v < 1.0f;   // :121
        row = in ? (int32_t)(v * (float)(H - 1)) : -1;
        col = (int32_t)(u * (float)(W - 1));
    }
    if (row >= 0) {
        const float* t = env + 3u * (uint32_t)(row * W + col);   // TexelFetch :6-14 (< 2^28 texels)
        return v3(t[0], t[1], t[2]);
    }
    return v3(0.0f, 0.0f, 0.0f);
}

template <bool ENV>
__device__ __forceinline__ V3 miss_radiance(const PtJob& job, V3 amb, V3 d)
{
    if (ENV) return env_sample(job.env, job.env_w, job.env_h, d);
    return amb;
}

#ifndef PT_DIAG_NOATOMIC
#define PT_DIAG_NOATOMIC 0
#endif
#ifndef PT_DIAG_WAVES_ONLY
#define PT_DIAG_WAVES_ONLY 0   // diagnostic build: per-wave birth/death only (no per-tile timeline)
#endif
#ifndef PT_DIAG
#define PT_DIAG 0   // diagnostic build: per-phase shader-clock cycles in counters[5..] (COUNT launches)
#endif
#if PT_DIAG >= 2   // per-phase cycle counters (heavier: perturbs register allocation)
#define DIAG_MARK(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define DIAG_ADD(k, t0) \
    dg[k] += __builtin_amdgcn_s_memtime() - (t0)
#else
#define DIAG_MARK(var)
#define DIAG_ADD(k, t0)
#endif

constexpr int kMaxWeights = 64;    // LDS table of the lerp weights 1/(iFrame+1) of a launch
constexpr int kChunk = 8;   // frames per phase-B/C chunk (LDS colour slots per pixel)
static_assert(kChunk >= 1 && kChunk < 32, "the pool's k / npf multiply is exact for npf < 32");

// Waves (8x8 tiles in flight) per workgroup.  LDS is allocated per workgroup in 1280-B granules
// on gfx950 (measured, scripts/lds_probe.hip; hipOccupancyMaxActiveBlocksPerMultiprocessor does not
// model it and over-reports 5 blocks for 32001..32768 B): the ambient kernel's 4-wave workgroup
// fits 5 per CU only with its LDS at <= 32 000 B (OWN_LAST below).  5-wave workgroups were placed
// only 3 per CU (15 waves), 10-wave ones 1 per CU: slower.
template <bool ENV>
constexpr int waves_per_block() { return 4; }

// Env variant: a phase-B miss adds EquirectangularTextureSample(dir) to the sample's radiance
// (simt_textured.cpp:408), two glibc inverse-trig calls and a texel gather.  Evaluated where the
// miss happens it runs in almost every pool iteration for the few lanes that escaped.  Deferred,
// the miss writes its radiance-so-far to its colour slot and queues (dir, slot) in LDS; once 64
// are queued all lanes evaluate one each and add it to the slot (ret + env == env + ret in f32,
// so the sum is the reference's bit for bit).  The queue is drained before phase C.  Measured at
// 1920x1080 x 8 spp, 8 bounces: 0.625 -> 0.541 ms per launch (LDS 32.7 -> 40.9 KiB per block,
// still 4 blocks per CU, the VGPR-bound occupancy of this kernel).

// One 8x8 tile of pixels per wave at a time, in three phases:
//   A  every lane traces its pixel's camera ray (coherent, once per pixel: the camera ray, its
//      TestSceneTrace and the bounce-0 shading are identical for every frame -- no jitter, the
//      RNG is first drawn after them, scalar.cpp:316);
//   B  the (pixel, frame) samples that continue past bounce 0 form a pool of items; lanes take
//      items in lane order as they free up (ballot + mbcnt) and trace them to completion, one
//      segment per iteration, writing each sample's radiance to LDS -- no lane waits for a
//      longer path of "its" pixel;
//   C  every lane runs the reference's progressive lerp over its pixel's frames IN FRAME ORDER
//      (:812), reading the radiance of each frame from LDS (or the constant radiance of a pixel
//      whose camera ray missed / of c_numBounces = 0).
// Tiles come from a per-launch atomic queue (persistent waves, next tile prefetched).
template <int LAYOUT, bool ENV, bool COUNT, bool MULTI, bool RING>
__device__ __forceinline__ void render_body(const PtJob& job)
{
    const PtScene* __restrict__ sc = job.scene;
    constexpr int kWavesPerBlock = waves_per_block<ENV>();
    __shared__ PtLdsPrim s_prim[PT_NPRIMS];
    __shared__ AxisRow s_axis[PT_NQUADS * kAxisRowsPerQuad<!ENV>];
    // the culled quad stage (pt_quadcull.h); the env kernel's LDS (4 blocks per CU: <= 40 960 B) has
    // no room for the 576-B flip-ordered vertex table, so it assembles W's vertices from the three
    // flip-ordered per-axis rows (QV false), and computes the lerp weights instead of tabling them
    constexpr bool QV = !ENV;
    __shared__ float4 s_qv[QV ? kQuadVecs : 1];
    constexpr bool WTAB = !ENV;
    // the closest-sphere stage, in both kernels (the env kernel kept the sequential tests while its
    // miss term was the exact inverse trig: 0.6024 vs 0.6001 ms at 1080p 16 spp, profiles/r03n_ab.jsonl;
    // with the certified texel cells 0.5459 vs 0.5524 ms, profiles/r03t_ab_c4.jsonl)
    constexpr bool SPHC = true;
    __shared__ float s_w[WTAB ? kMaxWeights : 1];
    constexpr int CH = kChunk;
    // The last frame of a chunk is traced by the pixel's own lane (OWN_LAST): its radiance stays in
    // that lane's registers, and the LDS holds CH - 1 frames per pixel -- 3 KiB less per block,
    // which brings the ambient kernel to 29 648 B = 24 LDS granules and 5 blocks per CU (5 waves
    // per SIMD, what its 96 VGPRs allow).  The env kernel (4 waves per SIMD by VGPRs) keeps CH.
    constexpr bool OWN_LAST = !ENV && CH > 1;
    constexpr int CHS = OWN_LAST ? CH - 1 : CH;   // LDS colour slots per pixel
    // RING (MULTI launches of the ambient kernel with >= kRingMinFrames frames): one continuous pool
    // over all frames, the colour slots a ring
    static_assert(!RING || (MULTI && !ENV), "the ring pool is the ambient kernel's MULTI mode");
    __shared__ float s_col[kWavesPerBlock][64 * CHS * 3];   // phase-B radiance per (pixel, frame)
    // per item pixel: P1.xyz + (id | lane << 8) and n1 (planar), 28 B
    __shared__ float4 s_rec[kWavesPerBlock][64];
    __shared__ float s_nrm[kWavesPerBlock][3][64];
    // env variant: the misses of phase B queue their direction (+ colour slot) here, and the queue
    // is drained 64 at a time by the whole wave (see kEnvDefer); 8 KiB, 40 KiB per block in all
    constexpr bool DEFER = ENV;
    __shared__ float4 s_envq[DEFER ? kWavesPerBlock : 1][DEFER ? 128 : 1];
    {
        const int t = threadIdx.x;
        if (t < PT_NPRIMS) {
            PtLdsPrim e;
            if (t < PT_NQUADS) {
                e.nx = sc->qn[t][0]; e.ny = sc->qn[t][1]; e.nz = sc->qn[t][2];
            } else {
                e.nx = sc->sph[t - PT_NQUADS][0]; e.ny = sc->sph[t - PT_NQUADS][1]; e.nz = sc->sph[t - PT_NQUADS][2];
            }
            e.ar = sc->albedo[t][0]; e.ag = sc->albedo[t][1]; e.ab = sc->albedo[t][2];
            e.er = sc->emissive[t][0]; e.eg = sc->emissive[t][1]; e.eb = sc->emissive[t][2];
            e.pad0 = e.pad1 = e.pad2 = 0.0f;
            s_prim[t] = e;
        } else if (t >= 64 && t < 64 + PT_NQUADS * kAxisRowsPerQuad<!ENV>) {
            constexpr int F = kAxisRowsPerQuad<!ENV> / 3;
            const int r = (t - 64) / 3, k = (t - 64) % 3, q = r / F, fl = r % F;
            const auto vk = [&](int v) { return sc->qv[q][fl ? 3 - v : v][k]; };
            s_axis[t - 64] = AxisRow{vk(0), vk(1), vk(2), vk(3)};
        } else if (QV && t >= 128 && t < 128 + kQuadVecs) {
            const int r = (t - 128) / 3, part = (t - 128) % 3, q = r >> 1, fl = r & 1;
            float e[4];
            for (int i = 0; i < 4; ++i) {
                const int f = part * 4 + i, v = f / 3, k = f % 3;   // vertex v of the flipped order
                e[i] = sc->qv[q][fl ? 3 - v : v][k];
            }
            s_qv[t - 128] = make_float4(e[0], e[1], e[2], e[3]);
        }
        if (WTAB && t < kMaxWeights && t < job.nframes)   // :812 1/(iFrame + 1), iFrame exact below 2^24
            s_w[t] = pt::rcp_rn((float)(job.frame_first + (uint32_t)t) + 1.0f);   // in [1, 2^24 + 1]: no guard
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar addressing
    // this wave's colour slots through a 32-bit LDS pointer (a generic one is 64-bit: its base was
    // hoisted out of the pool loop and spilled)
    typedef __attribute__((address_space(3))) float lds_f32;
    lds_f32* const col_lds = (lds_f32*)&s_col[0][0] + wv * (64 * CHS * 3);
    const int tiles_x = (job.ncols + 7) >> 3;
    const uint32_t total_tiles = (uint32_t)tiles_x * (uint32_t)((job.nrows + 7) >> 3);
    const int S = job.nframes, B = job.num_bounces;
    const size_t cs = (LAYOUT == PT_LAYOUT_INTERLEAVED) ? 1u : 8u;   // channel stride

    Camera cam;   // frame constants from the kernel arguments (pt_launch_render, host)
    cam.W = job.cam_W;
    cam.H = job.cam_H;
    cam.yW = job.cam_yW;
    cam.yH = job.cam_yH;
    cam.aspect = job.cam_aspect;                                                // :346
    cam.yAspect = job.cam_yAspect;
    cam.cam_dist = sc->cam_dist;
    const V3 amb = v3(sc->ambient[0], sc->ambient[1], sc->ambient[2]);
    const V3 zero = v3(0.0f, 0.0f, 0.0f), one = v3(1.0f, 1.0f, 1.0f);

    unsigned long long n_seg = 0, n_iter = 0, n_samp = 0, n_esc = 0, n_prim = 0, n_fb = 0, n_sky = 0;
#if PT_DIAG
#if PT_DIAG >= 2
    unsigned long long dg[7] = {0, 0, 0, 0, 0, 0, 0};   // A, take, dir, trace, shade, C, tile-total
#endif
    const unsigned long long t_birth = __builtin_amdgcn_s_memtime();
    const unsigned long long r_birth = __builtin_amdgcn_s_memrealtime();
    unsigned long long n_tiles_diag = 0;
#endif

    // the next launch's queue counters start at zero: this launch clears them (pt_capi.cpp use_sched;
    // it saves the stream a 1-KiB fill before every launch)
    pt_queue_zero_next(job.queue_next);   // (pt_tile_queue.h)
    // tiles from the launch's queue (pt_tile_queue.h)
    constexpr uint32_t kNone = PtTileQueue<kWavesPerBlock>::kNone;
    PtTileQueue<kWavesPerBlock> tq(job.queue, job.order, job.units, job.nunits, total_tiles, wv);
    uint32_t tile = kNone, next_tile = kNone;
    tile = tq.first(job.err);   // (the whole wave: uniform, scalar registers)
    tile = __builtin_amdgcn_readfirstlane(tile);
    while (tile != kNone) {
        // a queue entry is a tile or one half of it (pt_tile_queue.h): the pixels of the other half
        // are treated as outside the image
        const uint32_t part = pt_entry_part(tile);
        const int tyi = (int)(pt_entry_tile(tile) / (uint32_t)tiles_x), txi = (int)(pt_entry_tile(tile) % (uint32_t)tiles_x);
        DIAG_MARK(t_tile);
#if PT_DIAG && !PT_DIAG_WAVES_ONLY
        const unsigned long long r_tile0 = __builtin_amdgcn_s_memrealtime();
        const uint32_t diag_tile_id = tile;
#endif
#if PT_DIAG
        ++n_tiles_diag;
#endif
        // ---------------- phase A: camera ray, once per pixel ----------------
        const int lc = txi * 8 + (lane & 7), lr = tyi * 8 + (lane >> 3);
        const bool valid = lc < job.ncols && lr < job.nrows && pt_part_has_lane(part, lane);
        const float fx = (float)(job.col0 + lc);                                            // :806
        const float fy = (float)(job.height - 1 - (job.row_start + lr * job.row_stride));   // :803
        // Registers live across the pool loop are kept to a minimum (the 96-VGPR budget of 5 waves per
        // SIMD): the accumulator is loaded in phase C when one chunk covers the launch's frames
        // (!MULTI) -- its address recomputed there --, the pixel's bounce-0 record is re-read from
        // LDS when the own-lane sample starts, whether the pixel has pool items is bit `lane` of
        // the wave-uniform hitmask, and one register triple (c_keep) holds the constant radiance
        // of a pixel without items or the own-lane radiance of one with items.
        V3 acc = zero;
        V3 c_keep = zero;         // no items: the radiance of every frame; items: the own-lane frame's
        V3 P1 = zero, N1 = zero;
        int id1 = 0;
        bool items = false;       // the camera ray hit and c_numBounces > 0: the pixel's frames are pool items
        const V3 D0 = camera_dir(cam, fx, fy);   // (lanes outside the image: unused values)
        // A tile whose camera rays all leave the box's silhouette skips their TestSceneTrace: the
        // result is the reference's miss (sky_ray below), and the trace is the whole cost of such
        // a tile's phase A -- about half of all 1080p tiles are sky.
        const bool all_sky = pt_ballot(valid && !sky_ray(D0)) == 0;
        if (valid) {
            if (MULTI) {
                const float* px = job.buf + out_index<LAYOUT>(job, lc, lr);
                acc = v3(px[0], px[cs], px[2 * cs]);
            }
            const Hit h = all_sky ? Hit{PT_SUPER_FAR, -1, 0, 0}
                                  : trace<DemofoxScene, true, QV, SPHC>(s_axis, s_qv, zero, D0);   // :335 rayPos = origin
            if (COUNT) ++n_seg, ++n_prim, n_fb += (unsigned long long)h.fb, n_sky += all_sky ? 1ull : 0ull;
            if (h.best == PT_SUPER_FAR) {                                 // :305-310
                c_keep = add(zero, miss_radiance<ENV>(job, amb, D0));
                if (COUNT) n_esc += (unsigned long long)S;
            } else {
                const PtLdsPrim pr = prim_at(s_prim, h.id);
                const V3 n1 = hit_normal(pr, h, zero, D0);
                P1 = add(add(zero, mul(D0, h.best)), mul(n1, PT_NUDGE));  // :313
                N1 = n1;
                id1 = h.id;
                items = B != 0;
                c_keep = add(zero, mulv(v3(pr.er, pr.eg, pr.eb), one));  // :319 (ret after bounce 0)
            }
            if (COUNT) n_samp += (unsigned long long)S;
        }
        const uint64_t hitmask = pt_ballot(items);
        const int nh = __popcll(hitmask);
        // compacted record slot of this lane's pixel: its rank among the pixels with items
        const int my_slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(hitmask >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)hitmask, 0u));
        if (items) {
            const int slot = my_slot;
            s_rec[wv][slot] = make_float4(P1.x, P1.y, P1.z, __builtin_bit_cast(float, id1 | (lane << 8)));
            s_nrm[wv][0][slot] = N1.x;
            s_nrm[wv][1][slot] = N1.y;
            s_nrm[wv][2][slot] = N1.z;
        }
        // advance the queue now (this tile's coordinates are already taken): the prefetched slot
        // becomes the next tile and the following slot is requested, hidden behind phases B/C
        const uint32_t this_tile = tile;
        uint32_t tile_work = 1;   // trace iterations of this tile (the schedule's cost)

        if constexpr (RING) {
            // ------- phases B + C for a launch of several chunks' frames (MULTI): one continuous pool -------
            // The chunked pool below drains its items at the end of every chunk (the pool tail: 18 % of
            // the lane slots idle at 4K 64 spp, against 11 % at 8 spp with one chunk).  Here the items
            // (pixel with items, frame) of ALL the launch's frames form one pool, frame-major, and the
            // LDS colour slots are a ring: frame f of pixel p lives in slot (p, f mod R).  Each lane folds
            // its pixel's frames IN FRAME ORDER as their radiance arrives (the reference's lerp, :812),
            // which frees the slot for frame f + R; an item is handed out only when its slot is free, in
            // item order.  slot.x < 0 marks a slot free (-1) or reserved by an item in flight (-2); a
            // sample's radiance is >= +0 or NaN (never negative), i.e. "ready".  Same values, same order:
            // bit-identical to the chunked path.
            constexpr int R = CHS;
            const bool mine = (hitmask >> lane) & 1u;   // this lane's pixel has pool items
            if (valid && !mine) {   // no items: every frame's radiance is c_keep, folded now in frame order
                for (int f = 0; f < S; ++f) {
                    const float t = WTAB && f < kMaxWeights ? s_w[f] : pt::rcp_rn((float)(job.frame_first + (uint32_t)f) + 1.0f);
                    acc = add(acc, mul(sub(c_keep, acc), t));
                }
            }
            for (int i = lane; i < 64 * R; i += 64) col_lds[i * 3] = -1.0f;   // every slot free
            const int total = nh * S;                                         // pool items
            // i / nh as umulhi(i, ceil(2^32 / nh)) for nh >= 2: exact for i < 2^32 / 63 (here i < nh + 64);
            // nh = 1 (ceil(2^32 / 1) does not fit 32 bits) divides by itself
            const uint32_t div_nh = nh > 1 ? (uint32_t)((0x100000000ull + (uint64_t)nh - 1u) / (uint64_t)nh) : 0u;
            int f_next = 0, i_next = 0;   // wave-uniform: (frame, compacted pixel) of the next item
            int issued = 0, folded = 0;   // wave-uniform
            int nfold = 0;                // this lane's pixel: frames folded so far
            int fold_addr = lane * R * 3;  // its slot of frame nfold
            const bool wtab = WTAB && S <= kMaxWeights;
            V3 P = zero, D = zero, T = zero, ret = zero, n = zero;
            uint32_t rng = 0;
            int bounce = 0;   // 0: no item
            int it_addr = 0;  // the item's colour slot (floats from col_lds)
            const uint64_t live = pt_ballot(true);
            // iteration guard: every item ends after <= B + 1 segments and a pool of `total` items
            // drains in < total (B + 2) + S iterations.  The bound is formed in 64 bits (total can be
            // 2^30 and B 1024) and clamped to what the 32-bit iteration count can reach, so it never
            // fires early; if it fires (a scheduling fault) the tile is abandoned mid-pool, which the
            // job's error words record (the host returns PT_EKERNEL naming the tile) instead of
            // hanging the GPU.
            // (job.guard_cap: ~0u, or a low test value -- PT_MI355_RING_GUARD_CAP -- that makes it fire)
            const uint64_t guard64 = (uint64_t)total * (uint64_t)(B + 2) + (uint64_t)S + 64u;
            const uint32_t guard_lim = guard64 < (uint64_t)job.guard_cap ? (uint32_t)guard64 : job.guard_cap;
            while (true) {
                const bool had = bounce != 0;
                const uint64_t idle = pt_ballot(!had);
                bool took = false;
                int ntaken = 0;
                if (idle != 0 && issued < total) {
                    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    const int ii = i_next + rank;
                    const int q = nh == 1 ? ii : (int)__umulhi((uint32_t)ii, div_nh);
                    const int f = f_next + q, slot = ii - (int)__umul24((uint32_t)q, (uint32_t)nh);
                    const bool cand = !had && issued + rank < total;
                    bool free = false;
                    int addr = 0;
                    float4 a0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    if (cand) {
                        a0 = s_rec[wv][slot];
                        const int src = __builtin_bit_cast(int, a0.w) >> 8;
                        addr = (int)__umul24((uint32_t)(src * R + f % R), 3u);
                        // free, and not the slot of an earlier item of this hand-out (frames < f_next + R)
                        free = col_lds[addr] == -1.0f && q < R;
                    }
                    const uint64_t cm = pt_ballot(cand), fm = pt_ballot(cand && free);
                    const uint64_t blocked = cm & ~fm;   // items in order: stop at the first blocked one
                    const uint64_t tm = blocked ? (cm & ((1ull << __builtin_ctzll(blocked)) - 1ull)) : cm;
                    took = (tm >> lane) & 1u;
                    if (took) {
                        col_lds[addr] = -2.0f;   // reserved
                        const int packed = __builtin_bit_cast(int, a0.w);
                        const int sId = packed & 0xff;
                        const int src = packed >> 8;                  // lane owning the pixel
                        const int slc = txi * 8 + (src & 7), slr = tyi * 8 + (src >> 3);
                        const PtLdsPrim pr = prim_at(s_prim, sId);
                        rng = seed_int((uint32_t)(job.col0 + slc),
                                       (uint32_t)(job.height - 1 - (job.row_start + (int)__umul24((uint32_t)slr, (uint32_t)job.row_stride))),
                                       job.frame_first + (uint32_t)f);                            // :332
                        P = v3(a0.x, a0.y, a0.z);                                            // :313 (bounce 0)
                        n = v3(s_nrm[wv][0][slot], s_nrm[wv][1][slot], s_nrm[wv][2][slot]);
                        ret = emissive0(pr);                                                 // :319
                        T = mulv(one, v3(pr.ar, pr.ag, pr.ab));                              // :322
                        bounce = 1;
                        it_addr = addr;
                    }
                    ntaken = __popcll(tm);
                    issued += ntaken;
                    i_next += ntaken;
                    while (i_next >= nh) {   // (SALU)
                        i_next -= nh;
                        ++f_next;
                    }
                }
                if ((live & ~idle) == 0 && ntaken == 0 && folded >= total) break;
                if (__builtin_expect(tile_work > guard_lim, 0)) {   // (never reached, see guard_lim)
                    if (lane == 0 && job.err) {
                        atomicAdd(&job.err[0], 1u);           // abandoned tiles
                        atomicMin(&job.err[1], pt_entry_tile(this_tile));   // the first of them
                    }
                    break;
                }
                ++tile_work;
                if (COUNT) ++n_iter;
                if (had || took) {
                    D = normalize(add(n, random_unit_vector(rng)));                          // :316
                    const Hit h = trace<DemofoxScene, false, QV, SPHC>(s_axis, s_qv, P, D);
                    if (COUNT) ++n_seg, n_fb += (unsigned long long)h.fb;
                    bool done;
                    if (h.best == PT_SUPER_FAR) {                                     // :305-310
                        ret = add(ret, miss_radiance<ENV>(job, amb, D));
                        done = true;
                        if (COUNT) ++n_esc;
                    } else {
                        const PtLdsPrim pr = prim_at(s_prim, h.id);
                        n = hit_normal(pr, h, P, D);
                        P = add(add(P, mul(D, h.best)), mul(n, PT_NUDGE));            // :313
                        ret = add(ret, mulv(v3(pr.er, pr.eg, pr.eb), T));             // :319
                        T = mulv(T, v3(pr.ar, pr.ag, pr.ab));                         // :322
                        bounce += 1;
                        done = bounce > B;
                    }
                    if (done) {
                        lds_f32* c = col_lds + it_addr;
                        c[1] = ret.y;
                        c[2] = ret.z;
                        c[0] = ret.x;   // (x last: it marks the slot ready)
                        bounce = 0;
                    }
                }
                // fold this pixel's next frame if its radiance is in (one frame per iteration)
                bool fnow = false;
                if (mine && nfold < S) {
                    lds_f32* c = col_lds + fold_addr;
                    const float cx = c[0];
                    if (!(cx < 0.0f)) {
                        const V3 colr = v3(cx, c[1], c[2]);   // color = c (see the chunked phase C)
                        const float t = wtab ? s_w[nfold] : pt::rcp_rn((float)(job.frame_first + (uint32_t)nfold) + 1.0f);
                        acc = add(acc, mul(sub(colr, acc), t));
                        c[0] = -1.0f;   // free
                        ++nfold;
                        fold_addr = fold_addr + 3 == (lane + 1) * R * 3 ? lane * R * 3 : fold_addr + 3;
                        fnow = true;
                    }
                }
                folded += __popcll(pt_ballot(fnow));
            }
            next_tile = tq.next(job.err);   // the pool is done
        } else {
        // one chunk covers the launch's frames unless MULTI (then the loop carries acc and c_keep)
        for (int f0 = 0; f0 < (MULTI ? S : 1); f0 += CH) {
            const int nf = S - f0 < CH ? S - f0 : CH;
            DIAG_ADD(0, t_tile);
            // ---------------- phase B: the pool of (pixel, frame) items ----------------
            const bool own = OWN_LAST && nf > 1;   // last frame traced by the pixel's lane
            const int npf = own ? nf - 1 : nf;            // pooled frames per pixel
            const int nitems = nh * npf;                  // pooled items
            const uint32_t div_m = (65536u + (uint32_t)npf - 1u) / (uint32_t)npf;   // see the take
            int next_item = 0;
            int it_lane = 0, it_f = 0;
            V3 P = zero, D = zero, T = zero, ret = zero, n = zero;
            uint32_t rng = 0;
            int bounce = 0;   // 0: no item (a lane holds an item iff bounce != 0)
            const bool mine = (hitmask >> lane) & 1u;   // this lane's pixel has pool items
            if (own && mine) {   // start with this pixel's own last-frame sample (bounce 0 done)
                // its bounce-0 record from LDS (P1 / N1 / id1 are not kept across the pool)
                const float4 a0 = s_rec[wv][my_slot];
                const int sId = __builtin_bit_cast(int, a0.w) & 0xff;
                const PtLdsPrim pr = prim_at(s_prim, sId);
                const int olc = txi * 8 + (lane & 7), olr = tyi * 8 + (lane >> 3);
                rng = seed_int((uint32_t)(job.col0 + olc), (uint32_t)(job.height - 1 - (job.row_start + olr * job.row_stride)),
                               job.frame_first + (uint32_t)(f0 + nf - 1));   // :332
                P = v3(a0.x, a0.y, a0.z);
                n = v3(s_nrm[wv][0][my_slot], s_nrm[wv][1][my_slot], s_nrm[wv][2][my_slot]);
                ret = emissive0(pr);                                             // :319
                T = mulv(one, v3(pr.ar, pr.ag, pr.ab));                          // :322
                bounce = 1;
                it_lane = lane;
                it_f = nf - 1;
            }
            int qn = 0;   // queued misses (DEFER), wave-uniform
            float4* const envq = s_envq[DEFER ? wv : 0];
            // evaluate the queued misses [q0, q0 + m) (m <= 64), one per lane, into their slots
            auto drain = [&](int q0, int m) {
                if (lane < m) {
                    const float4 e = envq[q0 + lane];
                    const V3 c = env_sample(job.env, job.env_w, job.env_h, v3(e.x, e.y, e.z));
                    lds_f32* cp = col_lds + __builtin_bit_cast(int, e.w);
                    cp[0] = cp[0] + c.x;
                    cp[1] = cp[1] + c.y;
                    cp[2] = cp[2] + c.z;
                }
            };
            const uint64_t live = pt_ballot(true);   // the wave's lanes (exec)
            while (true) {
                DIAG_MARK(t_it);
                const bool had = bounce != 0;   // this lane holds an item (lane mask, before the refill)
                const uint64_t idle = pt_ballot(!had);
                bool took = false;              // this lane takes an item now (lane mask)
                int ntaken = 0;   // items handed out by this refill (wave-uniform)
                if (idle != 0 && next_item < nitems) {
                    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    const int k = next_item + rank;
                    const bool take = !had && k < nitems;
                    took = take;
                    // pixel-major: consecutive items are the frames of one pixel (shared ray
                    // origin; 1-1.3 % faster than frame-major).  k / npf as (k * ceil(2^16 / npf)) >>
                    // 16: exact for k < 64 npf, npf < 32 (the error k (M - 2^16 / npf) / 2^16 <
                    // npf / 1024 stays below the 1/npf gap)
                    const int slot_pm = take ? (int)(__umul24((uint32_t)k, div_m) >> 16) : 0;   // k * div_m < 2^25
                    const int fi = take ? k - (int)__umul24((uint32_t)slot_pm, (uint32_t)npf) : 0;
                    if (take) {
                        const int slot = slot_pm;                     // the item's pixel record
                        const float4 a0 = s_rec[wv][slot];
                        const int packed = __builtin_bit_cast(int, a0.w);
                        const int sId = packed & 0xff;
                        const int src = packed >> 8;                  // lane owning the pixel
                        const int slc = txi * 8 + (src & 7), slr = tyi * 8 + (src >> 3);
                        const PtLdsPrim pr = prim_at(s_prim, sId);
                        rng = seed_int((uint32_t)(job.col0 + slc),
                                       (uint32_t)(job.height - 1 - (job.row_start + (int)__umul24((uint32_t)slr, (uint32_t)job.row_stride))),
                                       job.frame_first + (uint32_t)(f0 + fi));                    // :332
                        P = v3(a0.x, a0.y, a0.z);                                            // :313 (bounce 0)
                        n = v3(s_nrm[wv][0][slot], s_nrm[wv][1][slot], s_nrm[wv][2][slot]);
                        ret = emissive0(pr);                                                 // :319
                        T = mulv(one, v3(pr.ar, pr.ag, pr.ab));                              // :322
                        bounce = 1;
                        it_lane = src;
                        it_f = fi;
                    }
                    const int npop = __popcll(idle);
                    ntaken = npop < nitems - next_item ? npop : nitems - next_item;
                    next_item += ntaken;
                }
                // __any(a lane holds an item), from the masks alone (SALU): the lanes that held an item before the
                // refill, or any lane that took one
                if ((live & ~idle) == 0 && ntaken == 0) break;
                ++tile_work;
                DIAG_ADD(1, t_it);
                DIAG_MARK(t_dir);
                if (COUNT) ++n_iter;
                bool queued = false;   // DEFER: this lane's item missed, (D, slot) to be queued
                if (had || took) {   // (bounce != 0, from the two lane masks: no compare)
                    // :316.  Every lane that holds an item at the start of an iteration needs a new
                    // direction: a taken item starts at bounce 1, a hit that does not end the path
                    // continues, and the direction after the last bounce is never drawn (the path
                    // ends there; its RNG draws are unused)
                    D = normalize(add(n, random_unit_vector(rng)));
                    DIAG_ADD(2, t_dir);
                    DIAG_MARK(t_tr);
                    const Hit h = trace<DemofoxScene, false, QV, SPHC>(s_axis, s_qv, P, D);
                    DIAG_ADD(3, t_tr);
                    DIAG_MARK(t_sh);
                    if (COUNT) ++n_seg, n_fb += (unsigned long long)h.fb;
                    bool done;
                    if (h.best == PT_SUPER_FAR) {                                     // :305-310
                        if (DEFER) queued = true;                                     // env added at the drain
                        else ret = add(ret, miss_radiance<ENV>(job, amb, D));         // ambient or env (:408)
                        done = true;
                        if (COUNT) ++n_esc;
                    } else {
                        const PtLdsPrim pr = prim_at(s_prim, h.id);
                        n = hit_normal(pr, h, P, D);
                        P = add(add(P, mul(D, h.best)), mul(n, PT_NUDGE));            // :313
                        ret = add(ret, mulv(v3(pr.er, pr.eg, pr.eb), T));             // :319
                        T = mulv(T, v3(pr.ar, pr.ag, pr.ab));                         // :322
                        bounce += 1;
                        done = bounce > B;
                    }
                    if (done) {
                        if (own && it_f == nf - 1) {   // own item: it_lane == lane
                            c_keep = ret;
                        } else {
                            lds_f32* c = col_lds + (it_lane * CHS + it_f) * 3;
                            c[0] = ret.x;
                            c[1] = ret.y;
                            c[2] = ret.z;
                        }
                        bounce = 0;   // no item
                    }
                    DIAG_ADD(4, t_sh);
                }
                if (DEFER) {
                    const uint64_t qm = pt_ballot(queued);
                    if (queued) {
                        const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
                        envq[qn + r] = make_float4(D.x, D.y, D.z, __builtin_bit_cast(float, (it_lane * CHS + it_f) * 3));
                    }
                    qn += __popcll(qm);
                    if (qn >= 64) {   // a full wave of misses: evaluate the last 64
                        qn -= 64;
                        drain(qn, 64);
                    }
                }
            }
            if (DEFER && qn > 0) drain(0, qn);
            if (f0 + CH >= S) next_tile = tq.next(job.err);   // the last chunk's pool is done
            // ---------------- phase C: progressive lerp in frame order ----------------
            DIAG_MARK(t_c);
            const int clc = txi * 8 + (lane & 7), clr = tyi * 8 + (lane >> 3);
            const bool cvalid = clc < job.ncols && clr < job.nrows && pt_part_has_lane(part, lane);
            if (cvalid) {
                if (!MULTI) {   // the accumulator, read once (24 B per pixel per launch with the store)
                    const float* px = job.buf + out_index<LAYOUT>(job, clc, clr);
                    acc = v3(px[0], px[cs], px[2 * cs]);
                }
                for (int fi = 0; fi < nf; ++fi) {
                    V3 c = c_keep;   // a pixel without items: the same radiance every frame
                    if (mine) {
                        if (own && fi == nf - 1) {
                            c = c_keep;
                        } else {
                            const lds_f32* cp = col_lds + (lane * CHS + fi) * 3;
                            c = v3(cp[0], cp[1], cp[2]);
                        }
                    }
                    // color = 0 + c * (1/1) (:355-356); lerp(last, color, 1/(iFrame+1)) (:812).  c * 1 == c
                    // and 0 + c == c for every c but -0, and a sample's radiance is never -0: it is
                    // 0 + (the miss radiance) for a missed camera ray, else the emissive value (+0 or
                    // positive) plus products and sums of non-negative terms and, in the env kernel, the
                    // texel added to that (x + (-0) == x) -- so color is c itself
                    const V3 colr = c;
                    const int f = f0 + fi;
                    const float t = WTAB && f < kMaxWeights ? s_w[f] : pt::rcp_rn((float)(job.frame_first + (uint32_t)f) + 1.0f);
                    acc = add(acc, mul(sub(colr, acc), t));
                }
            }
            DIAG_ADD(5, t_c);
        }
        }
        if (txi * 8 + (lane & 7) < job.ncols && tyi * 8 + (lane >> 3) < job.nrows && pt_part_has_lane(part, lane)) {
            float* px = job.buf + out_index<LAYOUT>(job, txi * 8 + (lane & 7), tyi * 8 + (lane >> 3));
            px[0] = acc.x;
            px[cs] = acc.y;
            px[2 * cs] = acc.z;
        }
        if (job.cost && lane == 0) pt_record_cost(job.cost, this_tile, total_tiles, tile_work);
        if (S <= 0) next_tile = tq.next(job.err);   // no chunk ran (nframes 0)
        tile = __builtin_amdgcn_readfirstlane(next_tile);
#if PT_DIAG && !PT_DIAG_WAVES_ONLY
        if (job.counters && lane == 0 && n_tiles_diag <= 32) {
            unsigned long long* tl = job.counters + 32 + 4 * 65536 + 96 * (size_t)(blockIdx.x * kWavesPerBlock + wv);
            tl[3 * (n_tiles_diag - 1) + 0] = r_tile0;
            tl[3 * (n_tiles_diag - 1) + 1] = __builtin_amdgcn_s_memrealtime();
            tl[3 * (n_tiles_diag - 1) + 2] = ((unsigned long long)diag_tile_id << 32) | tile_work;
        }
#endif
        DIAG_ADD(6, t_tile);
    }
    tq.report(job.err);   // (a schedule entry outside the launch, pt_tile_queue.h)
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            n_seg += __shfl_xor(n_seg, off, 64);
            n_samp += __shfl_xor(n_samp, off, 64);
            n_esc += __shfl_xor(n_esc, off, 64);
            n_prim += __shfl_xor(n_prim, off, 64);
            n_fb += __shfl_xor(n_fb, off, 64);
            n_sky += __shfl_xor(n_sky, off, 64);
        }
        if (lane == 0) {
            atomicAdd(&job.counters[PT_CNT_SEGMENTS], n_seg);
            atomicAdd(&job.counters[PT_CNT_LANE_SLOTS], 64ull * n_iter);
            atomicAdd(&job.counters[PT_CNT_SAMPLES], n_samp);
            atomicAdd(&job.counters[PT_CNT_ESCAPED], n_esc);
            atomicAdd(&job.counters[PT_CNT_PRIMARY], n_prim);
            atomicAdd(&job.counters[PT_CNT_FALLBACK], n_fb);
            atomicAdd(&job.counters[PT_CNT_SKY], n_sky);
        }
    }
#if PT_DIAG
    if (job.counters && lane == 0) {
#if PT_DIAG >= 2
            for (int k = 0; k < 7; ++k) atomicAdd(&job.counters[PT_CNT_N + k], dg[k]);
#endif
            const unsigned long long r_death = __builtin_amdgcn_s_memrealtime();
#if !PT_DIAG_NOATOMIC   // (same-address atomics from every wave; the per-wave records suffice)
            const unsigned long long t_death = __builtin_amdgcn_s_memtime();
            atomicAdd(&job.counters[PT_CNT_N + 7], t_death - t_birth);      // wave lifetimes
            atomicAdd(&job.counters[PT_CNT_N + 10], r_death - r_birth);      // 100 MHz ticks
            atomicMax(&job.counters[PT_CNT_N + 8], r_birth);                 // last wave start
            atomicMin(&job.counters[PT_CNT_N + 9], r_death);                 // first wave end
            atomicMax(&job.counters[PT_CNT_N + 11], r_death);                // last wave end
            atomicMin(&job.counters[PT_CNT_N + 12], r_birth);                // first wave start
#endif
            unsigned long long* rec = job.counters + 32 + 4 * (size_t)(blockIdx.x * kWavesPerBlock + wv);
            rec[0] = r_birth;
            rec[1] = r_death;
            rec[2] = n_tiles_diag;
            rec[3] = n_iter;
    }
#endif
}

// ---- continuous tiles (CT): the ambient kernel's pool without per-tile tails ----------------------
// render_body's item pool drains at the end of every tile (and, for MULTI launches, of every 8-frame
// chunk): its last items run while the other lanes idle -- the pool runs at 81 % of its lane slots at
// 1080p and 4K, 8 spp, 8 bounces.  Here the work of a wave is a stream of CHUNKS -- (tile, kChunk
// frames), a tile's chunks in frame order -- and the wave keeps TWO chunk contexts: A, whose items
// are being handed out, and D, whose items are all handed out and still in flight.  When A's last item
// is handed out and D is folded, A becomes D and the next chunk starts at once, so the lanes that
// free up take the next chunk's items instead of idling while the slowest paths end.  A new tile's
// camera rays are traced coherently by all 64 lanes (render_body's phase A) while lanes keep D's
// items in their registers; the next chunk of a tile needs no camera rays (the bounce-0 records are
// the same for every frame).  A chunk is folded -- the reference's progressive lerp of its frames, in
// frame order, :812 -- as soon as its last item ends, and chunks fold in stream order, so every pixel
// sees its frames in order.  Storage: one set of bounce-0 records per wave (a tile's records are only
// read when its items are handed out, which ends before the next tile starts), the pixels' running
// accumulators between a tile's chunks (LDS), and the per-(pixel, frame) radiance of the two
// contexts in a global slot area (ct_slots: per wave 2 x 64 pixels x kChunk frames x RGB, 12 KiB;
// an item's write is one 12-B store, a pixel's fold reads its frames with 16-B loads).  A pixel
// without pool items (camera ray missed, or 0 bounces) folds its constant radiance for all the
// launch's frames when its tile starts.  Same operations on the same operands, frames in the same
// order: bit-identical to render_body (every -m gpu parity test).
constexpr uint32_t kCtWaveFloats = 2u * 64u * (uint32_t)kChunk * 3u;   // per wave: 12 KiB of f32
// render_body_ct's per-wave LDS words: the tile being chunked (queue entry, pixel terms of the seed,
// item-pixel mask, item pixels, next chunk's first frame), A's first frame, D (entry, first frame,
// frames, item-pixel mask), the tile's folded segments, flags (1 claimed, 2 queue done), chunks
enum : int {
    kWsTcur, kWsHm, kWsHm1, kWsNh, kWsF0next, kWsF0A, kWsTD, kWsF0D, kWsNfD, kWsHmD, kWsHmD1,
    kWsTileSeg, kWsSegA, kWsSegD, kWsFlags, kWsChunks, kWsWords
};

// The env CT kernel runs 6 waves per SIMD: its pool loop fits 80 VGPRs (the spills of that build
// are in the event code), and a block's LDS fits 6 per CU with a 96-entry miss queue per wave
// (128 entries: 30 KiB per block, 5 per CU).  PT_ENV_WAVES / PT_ENV_Q: A/B builds.
#ifndef PT_ENV_WAVES
#define PT_ENV_WAVES 6
#endif
#ifndef PT_ENV_Q
#define PT_ENV_Q 96
#endif
static_assert(PT_ENV_Q >= 64 && PT_ENV_Q <= 128, "the env miss queue holds 64 .. 128 entries per wave");
// ENV (config 4, the env-map miss term): a missed segment's item is queued with its direction and
// radiance so far (s_envq, 32 B), and the queue is drained 64 at a time by the whole wave -- the
// coherent texel gathers of render_body's env kernel; a drain writes the items' radiance + texel
// (render_body's `cp + c`) to their slots.  D's fold drains the whole queue first.
// PRESENT: the fused output stage (job.pix_out; pt_render_device_present) -- its own instances, so
// the plain kernels' register allocation is untouched.
template <int LAYOUT, bool ENV, bool COUNT, bool PRESENT>
__device__ __forceinline__ void render_body_ct(const PtJob& job)
{
    // chained launches: this block has started (the next launch's stream waits for every block of
    // this one: hipStreamWaitValue64 in pt_capi.cpp launch_chain)
    pt_chain_started(job.started);
#if PT_CHAIN_DIAG
    if (job.tile_epoch && blockIdx.x == 0 && threadIdx.x == 0) job.queue[kPtDiagWaves] = gridDim.x * (blockDim.x / 64u);
#endif
    const PtScene* __restrict__ sc = job.scene;
    constexpr int kWavesPerBlock = waves_per_block<ENV>();
    constexpr bool QV = true;
    __shared__ PtLdsPrim s_prim[PT_NPRIMS];
    __shared__ AxisRow s_axis[PT_NQUADS * kAxisRowsPerQuad<true>];
    __shared__ float4 s_qv[kQuadVecs];
    __shared__ float s_w[kMaxWeights];
    // the current tile's item pixels: bounce-0 records P1.xyz + (id | lane << 8), n1 (planar), as
    // render_body's; and the item pixels' running accumulators between the tile's chunks
    __shared__ float4 s_rec[kWavesPerBlock][64];
    __shared__ float s_nrm[kWavesPerBlock][3][64];
    __shared__ float s_acc[kWavesPerBlock][3][64];
    __shared__ uint32_t s_seed[kWavesPerBlock][64];   // the item pixels' seed terms (x, y) of :332
    __shared__ uint32_t s_ws[kWavesPerBlock][kWsWords];   // the events' wave-uniform state (below)
    __shared__ uint32_t s_tq[kWavesPerBlock][PtTileQueue<kWavesPerBlock>::kWords];   // the wave's tile queue
    constexpr int kQ = ENV ? PT_ENV_Q : 1;   // queued misses: direction + slot, radiance so far
    __shared__ float4 s_envq[ENV ? kWavesPerBlock : 1][kQ][2];
    {
        const int t = threadIdx.x;
        if (t < PT_NPRIMS) {
            PtLdsPrim e;
            if (t < PT_NQUADS) {
                e.nx = sc->qn[t][0]; e.ny = sc->qn[t][1]; e.nz = sc->qn[t][2];
            } else {
                e.nx = sc->sph[t - PT_NQUADS][0]; e.ny = sc->sph[t - PT_NQUADS][1]; e.nz = sc->sph[t - PT_NQUADS][2];
            }
            e.ar = sc->albedo[t][0]; e.ag = sc->albedo[t][1]; e.ab = sc->albedo[t][2];
            e.er = sc->emissive[t][0]; e.eg = sc->emissive[t][1]; e.eb = sc->emissive[t][2];
            e.pad0 = e.pad1 = e.pad2 = 0.0f;
            s_prim[t] = e;
        } else if (t >= 64 && t < 64 + PT_NQUADS * kAxisRowsPerQuad<true>) {
            constexpr int F = kAxisRowsPerQuad<true> / 3;
            const int r = (t - 64) / 3, k = (t - 64) % 3, q = r / F, fl = r % F;
            const auto vk = [&](int v) { return sc->qv[q][fl ? 3 - v : v][k]; };
            s_axis[t - 64] = AxisRow{vk(0), vk(1), vk(2), vk(3)};
        } else if (t >= 128 && t < 128 + kQuadVecs) {
            const int r = (t - 128) / 3, part = (t - 128) % 3, q = r >> 1, fl = r & 1;
            float e[4];
            for (int i = 0; i < 4; ++i) {
                const int f = part * 4 + i, v = f / 3, k = f % 3;
                e[i] = sc->qv[q][fl ? 3 - v : v][k];
            }
            s_qv[t - 128] = make_float4(e[0], e[1], e[2], e[3]);
        }
        if (t < kMaxWeights && t < job.nframes)   // :812 1/(iFrame + 1), iFrame exact below 2^24
            s_w[t] = pt::rcp_rn((float)(job.frame_first + (uint32_t)t) + 1.0f);
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tiles_x = (job.ncols + 7) >> 3;
    const uint32_t total_tiles = (uint32_t)tiles_x * (uint32_t)((job.nrows + 7) >> 3);
    const int S = job.nframes, B = job.num_bounces;
    const size_t cs = (LAYOUT == PT_LAYOUT_INTERLEAVED) ? 1u : 8u;   // channel stride
    float* const slots = job.ct_slots + (size_t)(blockIdx.x * kWavesPerBlock + wv) * kCtWaveFloats;
    // (the host launches at most ct_waves waves: launch_ct)
    if (!PT_GUARD(job.err, blockIdx.x * (uint32_t)kWavesPerBlock + (uint32_t)wv < job.ct_waves, PT_G_SLOT_BASE,
                  blockIdx.x * (uint32_t)kWavesPerBlock + (uint32_t)wv))
        return;
    const size_t px_extent = pixel_extent<LAYOUT>(job);   // (guards; the accumulator's buffer resource)
    const uint32_t pxb = pt_px_nbytes(px_extent);          // (pt_chain.h pt_px_ld3 / pt_px_st3)
    // lerp weight of frame f of the launch: the table, or its correctly rounded reciprocal (:812)
    auto weight = [&](int f) {
        return f < kMaxWeights ? s_w[f] : pt::rcp_rn((float)(job.frame_first + (uint32_t)f) + 1.0f);
    };
    // the fused output stage: a pixel's final accumulator value -> its 8-bit pixel (OutputToScreen /
    // OutputToFile, v4 :1260-1331; pt_tonemap.h), at the point the launch writes that value
    auto present = [&](int lc, int lr, const V3& acc) {
        if constexpr (PRESENT) {
            const size_t o = (size_t)lr * (uint32_t)job.ncols + (uint32_t)lc;
            if (PT_GUARD(job.err, o < (size_t)job.nrows * (uint32_t)job.ncols, PT_G_PIXOUT, o))
                job.pix_out[o] = pt_tone::pack<true, true>(acc.x, acc.y, acc.z, job.pix_xrgb != 0);
        }
    };

    Camera cam;
    cam.W = job.cam_W;
    cam.H = job.cam_H;
    cam.yW = job.cam_yW;
    cam.yH = job.cam_yH;
    cam.aspect = job.cam_aspect;
    cam.yAspect = job.cam_yAspect;
    cam.cam_dist = sc->cam_dist;
    const V3 amb = v3(sc->ambient[0], sc->ambient[1], sc->ambient[2]);
    const V3 zero = v3(0.0f, 0.0f, 0.0f), one = v3(1.0f, 1.0f, 1.0f);
    unsigned long long n_seg = 0, n_iter = 0, n_samp = 0, n_esc = 0, n_prim = 0, n_fb = 0, n_sky = 0;
#if PT_DIAG   // diagnostic build: render_body's per-wave records; tile records from claim to last fold
    const unsigned long long r_birth = __builtin_amdgcn_s_memrealtime();
    unsigned long long n_tiles_diag = 0;
    uint32_t didx_cur = 0, didxA = 0, didxD = 0;   // tile record index of tcur / A / D
    unsigned long long* const dtl =
        job.counters ? job.counters + 32 + 4 * 65536 + 96 * (size_t)(blockIdx.x * kWavesPerBlock + wv) : nullptr;
#endif

    pt_queue_zero_next(job.queue_next);   // (pt_tile_queue.h)
    constexpr uint32_t kNone = PtTileQueue<kWavesPerBlock>::kNone;
    {
        PtTileQueue<kWavesPerBlock> q(job.queue, job.order, job.units, job.nunits, total_tiles, wv);
        q.back = (uint64_t)blockIdx.x * 100u >= (uint64_t)gridDim.x * (100u - (job.ct_back_pct < 100u ? job.ct_back_pct : 100u)) &&
                 job.ct_back_pct != 0;
        q.save(s_tq[wv], lane);
    }

    // Wave-uniform state.  What only the events (chunk start, retire, fold) use lives in LDS (s_ws),
    // not in scalar registers: the pool loop then keeps its constants in SGPRs instead of
    // rematerialising them every iteration (the scalar register file is the pool's tight budget:
    // 102 per wave).  ws_ld / ws_st: a uniform load (readfirstlane) / lane 0's store.
    uint32_t* const ws = s_ws[wv];
    auto ws_ld = [&](int k) -> uint32_t { return __builtin_amdgcn_readfirstlane(ws[k]); };
    auto ws_st = [&](int k, uint32_t v) {
        if (lane == 0) ws[k] = v;
    };
    // chained launches (pt_chain.h): before touching entry e's pixels, wait for the previous launch's
    // epoch; after e's last pixel store, publish this launch's
    auto chain_wait_tile = [&](uint32_t e) {
        if (job.chain_wait != 0u) pt_chain_wait(job.tile_epoch, e, job.chain_wait, job.err, lane, PT_CHAIN_DIAG ? job.queue : nullptr);
    };
    auto chain_publish = [&](uint32_t e) {
        if (job.tile_epoch) pt_chain_publish(job.tile_epoch, e, job.chain_seq, job.chain_delay, lane);
    };

    if (lane == 0) {
        ws[kWsTcur] = kNone;   // the tile being chunked (A's tile whenever A is set)
        ws[kWsFlags] = 0u;
        ws[kWsChunks] = 0u;
        ws[kWsTileSeg] = 0u;
    }
    // In the pool loop (scalar registers): the chunk contexts -- A hands out items; D has handed out
    // all of its items
    int cA = 0;                            // A's slot context (D's is 1 - cA)
    int nfA = 0;
    uint32_t fterm = 0;                    // the seed's frame term of A's first frame (:332)
    int issA = 0, nitA = 0;                // A's items handed out / all (nitA 0: no A)
    // D's items are the ones in flight when A retired (every earlier chunk was folded then): the lanes
    // that still hold one.  A lane whose D item ends takes A's items from then on.
    bool hasD = false;
    uint64_t dmask = 0;
    // k / nfA as (k * divA) >> 16 (exact for k < 64 nfA, nfA < 32; __umul24 reads bits 0-23); bit 31:
    // this launch records the schedule's costs (segments traced, counted in s_ws)
    uint32_t divA = 0;
    const uint32_t rec_cost = (job.cost || PT_DIAG) ? 0x80000000u : 0u;
    // per lane: the item (bounce 0: none) and the float index of its radiance slot in `slots`
    V3 P = zero, D = zero, T = zero, ret = zero, n = zero;
    uint32_t rng = 0;
    int bounce = 0;
    int it_addr = 0;

    // Start chunks until A is set or the queue is empty: the current tile's next chunk, or a new tile
    // (render_body's phase A, run by the whole wave while lanes may hold D's items -- item registers
    // untouched).  A new tile starts only when the previous tile's last chunk has handed out every
    // item, so its records are free.
    auto start_chunk = [&]() {
        while (nitA == 0) {
            const int f0next = (int)ws_ld(kWsF0next);
            if (ws_ld(kWsTcur) != kNone && f0next < S) {   // the current tile's next chunk
                // frame < 2^24 (C ABI): umul24(frame_first + f0A + fi) = fterm + fi * 26699 (mod 2^32)
                fterm = __umul24(job.frame_first + (uint32_t)f0next, 26699u);
                nfA = S - f0next < kChunk ? S - f0next : kChunk;
                ws_st(kWsF0A, (uint32_t)f0next);
                ws_st(kWsF0next, (uint32_t)(f0next + nfA));
                divA = ((65536u + (uint32_t)nfA - 1u) / (uint32_t)nfA) | rec_cost;
                issA = 0;
                nitA = (int)ws_ld(kWsNh) * nfA;   // >= 1
                ws_st(kWsSegA, 0u);
#if PT_DIAG
                didxA = didx_cur;
#endif
                break;
            }
            ws_st(kWsTcur, kNone);
            const uint32_t flags = ws_ld(kWsFlags);
            if (flags & 2u) break;   // the queue is done
            PtTileQueue<kWavesPerBlock> tq = PtTileQueue<kWavesPerBlock>::restore(s_tq[wv]);
            uint32_t tile = (flags & 1u) ? tq.next(job.err) : tq.first(job.err);
            tile = __builtin_amdgcn_readfirstlane(tile);
            tq.save(s_tq[wv], lane);
            ws_st(kWsFlags, tile == kNone ? 3u : 1u);   // claimed (and done)
            if (tile == kNone) break;
            chain_wait_tile(tile);
#if PT_DIAG && !PT_DIAG_WAVES_ONLY
            didx_cur = (uint32_t)n_tiles_diag;
            if (dtl && lane == 0 && n_tiles_diag < 32) {
                dtl[3 * n_tiles_diag + 0] = __builtin_amdgcn_s_memrealtime();
                dtl[3 * n_tiles_diag + 2] = (unsigned long long)tile << 32;
                dtl[3 * n_tiles_diag + 1] = n_iter;   // (until the last fold: the pool iteration of the claim)
            }
#endif
#if PT_DIAG
            ++n_tiles_diag;
#endif
            // (a queue entry is a tile or one half of it, pt_tile_queue.h)
            const uint32_t part = pt_entry_part(tile);
            const int tyi = (int)(pt_entry_tile(tile) / (uint32_t)tiles_x), txi = (int)(pt_entry_tile(tile) % (uint32_t)tiles_x);
            const int lc = txi * 8 + (lane & 7), lr = tyi * 8 + (lane >> 3);
            const bool valid = lc < job.ncols && lr < job.nrows && pt_part_has_lane(part, lane);
            const float fx = (float)(job.col0 + lc);                                            // :806
            const float fy = (float)(job.height - 1 - (job.row_start + lr * job.row_stride));   // :803
            const V3 D0 = camera_dir(cam, fx, fy);
            const bool all_sky = pt_ballot(valid && !sky_ray(D0)) == 0;   // (render_body's sky tiles)
            bool items = false;
            V3 P1 = zero, N1 = zero;
            int id1 = 0;
            if (valid) {
                const Hit h = all_sky ? Hit{PT_SUPER_FAR, -1, 0, 0}
                                      : trace<DemofoxScene, true, QV, true>(s_axis, s_qv, zero, D0);   // :335
                if (COUNT) ++n_seg, ++n_prim, n_fb += (unsigned long long)h.fb, n_sky += all_sky ? 1ull : 0ull;
                if (COUNT) n_samp += (unsigned long long)S;
                V3 c_keep;
                if (h.best == PT_SUPER_FAR) {                                 // :305-310
                    c_keep = add(zero, miss_radiance<ENV>(job, amb, D0));         // (:408 env kernel)
                    if (COUNT) n_esc += (unsigned long long)S;
                } else {
                    const PtLdsPrim pr = prim_at(s_prim, h.id);
                    const V3 n1 = hit_normal(pr, h, zero, D0);
                    P1 = add(add(zero, mul(D0, h.best)), mul(n1, PT_NUDGE));    // :313
                    N1 = n1;
                    id1 = h.id;
                    items = B != 0;
                    c_keep = add(zero, mulv(v3(pr.er, pr.eg, pr.eb), one));    // :319 (ret after bounce 0)
                }
                const size_t pi = out_index<LAYOUT>(job, lc, lr);
                if (!items && PT_GUARD(job.err, pi + 2 * cs < px_extent, PT_G_PIXEL, pi)) {
                    // the same radiance in every frame: fold all of the launch's frames now
                    V3 acc;
                    pt_px_ld3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);
                    for (int f = 0; f < S; ++f) acc = add(acc, mul(sub(c_keep, acc), weight(f)));
                    pt_px_st3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);
                    present(lc, lr, acc);
                }
            }
            const uint64_t hm = pt_ballot(items);
            const int nh = __popcll(hm);
            if (nh == 0) {
                if (job.cost && lane == 0) pt_record_cost(job.cost, tile, total_tiles, 1u);
                chain_publish(tile);   // (every pixel of the tile was stored above)
#if PT_DIAG && !PT_DIAG_WAVES_ONLY
                if (dtl && lane == 0 && didx_cur < 32) {
                    dtl[3 * didx_cur + 1] = __builtin_amdgcn_s_memrealtime();
                    dtl[3 * didx_cur + 2] = ((unsigned long long)tile << 32) | 1u;
                }
#endif
                continue;
            }
            if (items) {   // compacted record slot: the pixel's rank among the tile's item pixels
                const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
                s_rec[wv][slot] = make_float4(P1.x, P1.y, P1.z, __builtin_bit_cast(float, id1 | (lane << 8)));
                s_nrm[wv][0][slot] = N1.x;
                s_nrm[wv][1][slot] = N1.y;
                s_nrm[wv][2][slot] = N1.z;
                // the seed's pixel terms (:332; x, y < 2^24)
                s_seed[wv][slot] = __umul24((uint32_t)(job.col0 + lc), 1973u) +
                                   __umul24((uint32_t)(job.height - 1 - (job.row_start + lr * job.row_stride)), 9277u);
            }
            ws_st(kWsTcur, tile);
            ws_st(kWsHm, (uint32_t)hm);
            ws_st(kWsHm + 1, (uint32_t)(hm >> 32));
            ws_st(kWsNh, (uint32_t)nh);
            ws_st(kWsF0next, 0u);
        }
    };
    // ENV: the queued misses [q0, q0 + m) (m <= 64), one per lane: radiance + the texel into the slot
    int qn = 0;   // queued misses (wave-uniform)
    auto drain = [&](int q0, int m) {
        if (ENV && lane < m) {
            const float4 e = s_envq[ENV ? wv : 0][q0 + lane][0], r = s_envq[ENV ? wv : 0][q0 + lane][1];
            const V3 c = env_sample(job.env, job.env_w, job.env_h, v3(e.x, e.y, e.z));
            const uint32_t a = __builtin_bit_cast(uint32_t, e.w);
            if (PT_GUARD(job.err, a + 3u <= kCtWaveFloats, PT_G_ITEM_SLOT, a)) {
                float* const o = slots + a;
                o[0] = r.x + c.x;
                o[1] = r.y + c.y;
                o[2] = r.z + c.z;
            }
        }
    };
    // Fold D: every item of it has ended, its radiance is in the slots of context 1 - cA
    auto fold_D = [&]() {
        if (ENV && qn > 0) {   // (D's misses among them)
            drain(0, qn);
            qn = 0;
        }
        const int c = cA ^ 1;
        // the slots were written by this wave's lanes (global stores): complete them before reading
        // (workgroup scope: the same CU's L1 -- LLVM AMDGPU memory model)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int f0D = (int)ws_ld(kWsF0D), nfD = (int)ws_ld(kWsNfD);
        const uint32_t tD = ws_ld(kWsTD);
        const uint64_t hmD = (uint64_t)ws_ld(kWsHmD) | ((uint64_t)ws_ld(kWsHmD + 1) << 32);
        const bool first = f0D == 0, last = f0D + nfD == S;
        if ((hmD >> lane) & 1u) {   // (an item pixel is a valid pixel)
            const float4* sp = (const float4*)(slots + (c * 64 + lane) * (kChunk * 3));   // 96 B, 16-B aligned
            float4 v[kChunk * 3 / 4];
#pragma unroll
            for (int i = 0; i < kChunk * 3 / 4; ++i)
                if (i * 4 < nfD * 3) v[i] = sp[i];
            const float* fr = (const float*)v;
            const uint32_t tdi = pt_entry_tile(tD);
            const int lc = (int)(tdi % (uint32_t)tiles_x) * 8 + (lane & 7), lr = (int)(tdi / (uint32_t)tiles_x) * 8 + (lane >> 3);
            size_t pi = out_index<LAYOUT>(job, lc, lr);
            if (!PT_GUARD(job.err, pi + 2 * cs < px_extent, PT_G_PIXEL, pi)) pi = 0;   // (checked build: reported)
            V3 acc;
            if (first) pt_px_ld3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);
            else acc = v3(s_acc[wv][0][lane], s_acc[wv][1][lane], s_acc[wv][2][lane]);
#pragma unroll
            for (int f = 0; f < kChunk; ++f) {
                if (f < nfD) {
                    // color = the sample's radiance (0 + c * 1 == c, render_body's phase C)
                    const V3 colr = v3(fr[3 * f], fr[3 * f + 1], fr[3 * f + 2]);
                    acc = add(acc, mul(sub(colr, acc), weight(f0D + f)));        // :812
                }
            }
            if (last) {
                pt_px_st3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);
                present(lc, lr, acc);
            } else {
                s_acc[wv][0][lane] = acc.x;
                s_acc[wv][1][lane] = acc.y;
                s_acc[wv][2][lane] = acc.z;
            }
        }
        const uint32_t tile_seg = ws_ld(kWsTileSeg) + ws_ld(kWsSegD);   // segments of the tile's folded chunks
        ws_st(kWsTileSeg, last ? 0u : tile_seg);
        // the schedule's cost: segments / 64 -- about the tile's pool iterations.  (Lane-time measured
        // with s_memrealtime instead ordered the tiles worse: 1080p 8 spp 0.2605 vs 0.2535 ms, 1 spp
        // 0.130 vs 0.112 -- an iteration's time is set more by what shares the SIMD than by the tile.)
        const uint32_t tile_cost = 1u + (tile_seg + 63u) / 64u;
        if (last) {
            if (job.cost && lane == 0) pt_record_cost(job.cost, tD, total_tiles, tile_cost);
            chain_publish(tD);   // (the item-less pixels were stored when the tile started)
#if PT_DIAG && !PT_DIAG_WAVES_ONLY
            if (dtl && lane == 0 && didxD < 32) {
                const unsigned long long it0 = dtl[3 * didxD + 1];
                dtl[3 * didxD + 1] = __builtin_amdgcn_s_memrealtime();
                // low word: the tile's cost | the pool iterations from its claim to its last fold << 16
                dtl[3 * didxD + 2] = ((unsigned long long)tD << 32) | tile_cost |
                                     ((n_iter - it0) << 16);
            }
#endif
        }
        hasD = false;
    };

    start_chunk();
    uint32_t idle_events = 0;                         // outer iterations in a row without progress
    bool fault = false;
    // outer loop: the events (D is folded; A becomes D and the next chunk starts); inner loop: pool
    // iterations until an event is due -- the hot loop holds no start / fold code
    while (!fault) {
        bool event = false;
        if (hasD && dmask == 0) {   // D's last item ended: fold it
            fold_D();
            event = true;
        }
        if (nitA > 0 && issA >= nitA && !hasD) {   // A has handed out every item and D is folded
            ws_st(kWsTD, ws_ld(kWsTcur));
            ws_st(kWsHmD, ws_ld(kWsHm));
            ws_st(kWsHmD + 1, ws_ld(kWsHm + 1));
            ws_st(kWsF0D, ws_ld(kWsF0A));
            ws_st(kWsNfD, (uint32_t)nfA);
            hasD = true;
            dmask = pt_ballot(bounce != 0);
            ws_st(kWsSegD, ws_ld(kWsSegA));
#if PT_DIAG
            didxD = didxA;
#endif
            nitA = 0;   // no A
            issA = 0;
            cA ^= 1;
            // (job.guard_cap: ~0u, or a low test value -- PT_MI355_RING_GUARD_CAP -- that ends the
            // wave after that many chunks, so that the fault path runs on a correct launch)
            const uint32_t n_chunks = ws_ld(kWsChunks) + 1u;   // chunks retired
            ws_st(kWsChunks, n_chunks);
            if (__builtin_expect(n_chunks > job.guard_cap, 0)) {
                fault = true;
                break;
            }
            start_chunk();
            event = true;
            if (dmask == 0) continue;   // (D's items had all ended: fold it first)
        }
        if (nitA == 0 && !hasD) break;   // every chunk of every tile of the queue is folded
        // (guard, never reached: with a chunk left, an outer iteration folds, retires or runs the pool)
        idle_events = event ? 0u : idle_events + 1u;
        if (__builtin_expect(idle_events > 2u, 0)) {
            fault = true;
            break;
        }
        while (true) {
            const bool had = bounce != 0;
            const uint64_t idle = pt_ballot(!had);
            bool took = false;
            int ntaken = 0;
            if (idle != 0 && issA < nitA) {
                const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const int k = issA + rank;
                const bool take = !had && k < nitA;
                took = take;
                // pixel-major: consecutive items are the frames of one pixel (render_body's order)
                const int slot_pm = take ? (int)(__umul24((uint32_t)k, divA) >> 16) : 0;
                const int fi = take ? k - (int)__umul24((uint32_t)slot_pm, (uint32_t)nfA) : 0;
                if (take) {
                    const float4 a0 = s_rec[wv][slot_pm];
                    const int packed = __builtin_bit_cast(int, a0.w);
                    const int sId = packed & 0xff;
                    const int src = packed >> 8;                  // lane owning the pixel
                    const PtLdsPrim pr = prim_at(s_prim, sId);
                    // seed_int of the pixel and frame f0A + fi (:332)
                    rng = (s_seed[wv][slot_pm] + fterm + __umul24((uint32_t)fi, 26699u)) | 1u;
                    P = v3(a0.x, a0.y, a0.z);                                            // :313 (bounce 0)
                    n = v3(s_nrm[wv][0][slot_pm], s_nrm[wv][1][slot_pm], s_nrm[wv][2][slot_pm]);
                    ret = emissive0(pr);                                                 // :319
                    T = mulv(one, v3(pr.ar, pr.ag, pr.ab));                              // :322
                    bounce = 1;
                    it_addr = (int)__umul24((uint32_t)(cA * 64 + src), (uint32_t)(kChunk * 3)) + fi * 3;
                }
                const int npop = __popcll(idle);
                ntaken = npop < nitA - issA ? npop : nitA - issA;
                issA += ntaken;
            }
            // no lane holds an item: an event is due (or the wave is done).  (Every lane of the wave
            // is live: full blocks, no lane has returned.)
            if (idle == ~0ull && ntaken == 0) break;
            idle_events = 0;
            if (COUNT || PT_DIAG) ++n_iter;
            bool done = false, queued = false;
            if (had || took) {
                D = normalize(add(n, random_unit_vector(rng)));                          // :316
                const Hit h = trace<DemofoxScene, false, QV, true>(s_axis, s_qv, P, D);
                if (COUNT) ++n_seg, n_fb += (unsigned long long)h.fb;
                if (h.best == PT_SUPER_FAR) {                                     // :305-310
                    if (ENV) queued = true;   // the env term is added at the drain (:408)
                    else ret = add(ret, amb);
                    done = true;
                    if (COUNT) ++n_esc;
                } else {
                    const PtLdsPrim pr = prim_at(s_prim, h.id);
                    n = hit_normal(pr, h, P, D);
                    P = add(add(P, mul(D, h.best)), mul(n, PT_NUDGE));            // :313
                    ret = add(ret, mulv(v3(pr.er, pr.eg, pr.eb), T));             // :319
                    T = mulv(T, v3(pr.ar, pr.ag, pr.ab));                         // :322
                    bounce += 1;
                    done = bounce > B;
                }
                if (done) {
                    if (!queued && PT_GUARD(job.err, (uint32_t)it_addr + 3u <= kCtWaveFloats, PT_G_ITEM_SLOT, it_addr)) {
                        float* c = slots + it_addr;
                        c[0] = ret.x;
                        c[1] = ret.y;
                        c[2] = ret.z;
                    }
                    bounce = 0;
                }
            }
            if (ENV) {
                const uint64_t qm = pt_ballot(queued);
                const int nq = __popcll(qm);
                // room for this iteration's misses (<= 64): the queue holds kQ; after the drain below
                // qn < 64, so with kQ < 128 a queue of more than kQ - 64 entries is evaluated first
                // (all of them: < 64 lanes busy, rare -- most iterations queue a few misses)
                if (kQ < 128 && qn + nq > kQ) {
                    drain(0, qn);
                    qn = 0;
                }
                if (queued && PT_GUARD(job.err, qn + nq <= kQ, PT_G_ENVQ, qn + nq)) {
                    const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
                    s_envq[ENV ? wv : 0][qn + r][0] = make_float4(D.x, D.y, D.z, __builtin_bit_cast(float, it_addr));
                    s_envq[ENV ? wv : 0][qn + r][1] = make_float4(ret.x, ret.y, ret.z, 0.0f);
                }
                qn += nq;
                if (qn >= 64) {   // a full wave of misses: evaluate the last 64
                    qn -= 64;
                    drain(qn, 64);
                }
            }
            const uint64_t ended = pt_ballot(done);
            if ((int)divA < 0) {   // (only launches whose tile costs feed the next schedule): segments traced
                const int inD = __popcll(dmask), in_all = __popcll(pt_ballot(had || took));
                if (lane == 0) {
                    ws[kWsSegA] += (uint32_t)(in_all - inD);
                    ws[kWsSegD] += (uint32_t)inD;
                }
            }
            dmask &= ~ended;
            // (no stall guard here: every lane that holds an item advances it by one segment per
            // iteration and ends it after at most B + 1, hand-outs are bounded by nitA, and an iteration
            // without an item in flight or a hand-out leaves the loop -- so the loop ends; the outer
            // loop's guard covers the event logic)
            if (hasD && dmask == 0) break;                       // fold due
            if (nitA > 0 && issA >= nitA && !hasD) break;        // retire due
        }
    }
    // a fault ends the wave with its chunks unfinished: recorded in the job's error words (the host
    // returns PT_EKERNEL), instead of a hung GPU
    if (__builtin_expect(fault, 0) && lane == 0 && job.err) {
        atomicAdd(&job.err[0], 1u);
        atomicMin(&job.err[1], pt_entry_tile(nitA > 0 ? ws_ld(kWsTcur) : (hasD ? ws_ld(kWsTD) : 0u)));
    }
    PtTileQueue<kWavesPerBlock>::restore(s_tq[wv]).report(job.err);   // (a schedule entry outside the launch)
#if PT_CHAIN_DIAG
    if (job.tile_epoch && lane == 0) atomicAdd(job.queue + kPtDiagEnded, 1u);
#endif
#if PT_DIAG
    if (job.counters && lane == 0) {
        unsigned long long* rec = job.counters + 32 + 4 * (size_t)(blockIdx.x * kWavesPerBlock + wv);
        rec[0] = r_birth;
        rec[1] = __builtin_amdgcn_s_memrealtime();
        rec[2] = n_tiles_diag;
        rec[3] = n_iter;
    }
#endif
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            n_seg += __shfl_xor(n_seg, off, 64);
            n_samp += __shfl_xor(n_samp, off, 64);
            n_esc += __shfl_xor(n_esc, off, 64);
            n_prim += __shfl_xor(n_prim, off, 64);
            n_fb += __shfl_xor(n_fb, off, 64);
            n_sky += __shfl_xor(n_sky, off, 64);
        }
        if (lane == 0) {
            atomicAdd(&job.counters[PT_CNT_SEGMENTS], n_seg);
            atomicAdd(&job.counters[PT_CNT_LANE_SLOTS], 64ull * n_iter);
            atomicAdd(&job.counters[PT_CNT_SAMPLES], n_samp);
            atomicAdd(&job.counters[PT_CNT_ESCAPED], n_esc);
            atomicAdd(&job.counters[PT_CNT_PRIMARY], n_prim);
            atomicAdd(&job.counters[PT_CNT_FALLBACK], n_fb);
            atomicAdd(&job.counters[PT_CNT_SKY], n_sky);
        }
    }
}

// Kernel entry points.  The ambient kernel is held to 96 VGPRs (the 5-waves-per-SIMD budget; 10
// spilled); the env-map kernel needs ~117 and runs at 4.
#ifndef PT_AMBIENT_WAVES
#define PT_AMBIENT_WAVES 5
#endif
// MULTI: the launch accumulates more frames than one LDS chunk holds (nframes > kChunk).
template <int LAYOUT, bool COUNT, bool MULTI, bool RING>
__global__ __launch_bounds__(64 * waves_per_block<false>()) __attribute__((amdgpu_waves_per_eu(PT_AMBIENT_WAVES, PT_AMBIENT_WAVES))) void
pt_render_kernel(PtJob job)
{
    render_body<LAYOUT, false, COUNT, MULTI, RING>(job);
}

template <int LAYOUT, bool COUNT, bool MULTI>
__global__ __launch_bounds__(64 * waves_per_block<true>()) void pt_render_env_kernel(PtJob job)
{
    render_body<LAYOUT, true, COUNT, MULTI, false>(job);
}

// WAVES per SIMD: 5 (96 VGPRs) or 6 (80 VGPRs, 29 SGPRs spilled to VGPR lanes); which one is faster
// depends on the launch geometry (pt_capi.cpp launch(): timed on a geometry's first launches)
template <int LAYOUT, bool COUNT, int WAVES, bool PRESENT = false>
__global__ __launch_bounds__(64 * waves_per_block<false>()) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void
pt_render_ct_kernel(PtJob job)
{
    render_body_ct<LAYOUT, false, COUNT, PRESENT>(job);
}

template <int LAYOUT, bool COUNT, bool PRESENT = false>
__global__ __launch_bounds__(64 * waves_per_block<true>()) __attribute__((amdgpu_waves_per_eu(PT_ENV_WAVES, PT_ENV_WAVES))) void pt_render_ct_env_kernel(PtJob job)
{
    render_body_ct<LAYOUT, true, COUNT, PRESENT>(job);
}

template <int LAYOUT, bool ENV, bool COUNT, bool MULTI, bool RING>
constexpr auto kernel_of()
{
    if constexpr (ENV) return pt_render_env_kernel<LAYOUT, COUNT, MULTI>;
    else return pt_render_kernel<LAYOUT, COUNT, MULTI, RING>;
}

template <int LAYOUT, bool ENV, bool COUNT, bool MULTI, bool RING = false>
void launch_k(const PtJob& job, hipStream_t st, unsigned tiles)
{
    constexpr int wpb = waves_per_block<ENV>();
    auto k = kernel_of<LAYOUT, ENV, COUNT, MULTI, RING>();
    const unsigned blocks = (unsigned)std::min<long>(pt_resident_blocks(k, 64 * wpb), (tiles + wpb - 1) / wpb);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * wpb), 0, st, job);
}

// Launches of at least kRingMinFrames frames run the ambient kernel's continuous ring pool (one pool
// tail per tile instead of one per 8-frame chunk); fewer frames keep the chunked pool, whose own-lane
// frame and lighter iteration win while there are only a few chunks.  Ring vs chunked at 1080p
// (profiles/r03y_ab_*.jsonl): 16 spp 0.484 vs 0.462 ms, 32 spp 0.898 vs 0.890, 48 spp 1.307 vs
// 1.316; 4K 64 spp 6.33 vs 6.74 ms; 8K 256 spp 97.9 vs 106.4 ms.
#ifndef PT_RING_MIN
#define PT_RING_MIN 48
#endif
constexpr int kRingMinFrames = PT_RING_MIN;

// One-chunk ambient launches on the continuous-tiles pool (render_body_ct) when the caller provides
// its slots for the whole grid; false: not launched (render_body then).
template <int LAYOUT, bool ENV, bool COUNT, bool WIDE, bool PRESENT = false>
constexpr auto ct_kernel_of()
{
    if constexpr (ENV) return pt_render_ct_env_kernel<LAYOUT, COUNT, PRESENT>;
    else return pt_render_ct_kernel<LAYOUT, COUNT, WIDE ? 6 : 5, PRESENT>;
}

// *presented: the kernel wrote job.pix_out (the presenting instances: row layouts, uncounted launches)
template <int LAYOUT, bool ENV, bool COUNT>
bool launch_ct(const PtJob& job, hipStream_t st, unsigned tiles, bool* presented, uint32_t* ct_blocks)
{
    constexpr int wpb = waves_per_block<ENV>();
    *presented = false;
    auto k = job.ct_wide ? ct_kernel_of<LAYOUT, ENV, COUNT, true>() : ct_kernel_of<LAYOUT, ENV, COUNT, false>();
    bool pres = false;
    if constexpr (!COUNT && LAYOUT != PT_LAYOUT_TILED_PLANAR8) {
        if (job.pix_out) {
            k = job.ct_wide ? ct_kernel_of<LAYOUT, ENV, false, true, true>() : ct_kernel_of<LAYOUT, ENV, false, false, true>();
            pres = true;
        }
    }
    const unsigned blocks = (unsigned)std::min<long>(pt_resident_blocks(k, 64 * wpb), (tiles + wpb - 1) / wpb);
    if (!job.ct_slots || (uint64_t)blocks * wpb > job.ct_waves) return false;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * wpb), 0, st, job);
    *presented = pres;
    if (ct_blocks) *ct_blocks = blocks;
    return true;
}

template <int LAYOUT, bool ENV>
hipError_t launch_pools(const PtJob& job, hipStream_t st, bool count, unsigned tiles);

template <int LAYOUT, bool ENV>
hipError_t launch_t(const PtJob& job, hipStream_t st, bool count, uint32_t* ct_blocks)
{
    const unsigned tiles = (unsigned)((job.ncols + 7) / 8) * (unsigned)((job.nrows + 7) / 8);
    // the continuous-tiles pool when its slots are provided (its presenting instances write
    // job.pix_out themselves)
    bool presented = false;
    hipError_t e;
    // counted launches are device jobs (pt_capi.cpp pt_count_device: the row layouts only), so the
    // tiled layout has no counting instances
    constexpr bool kCountable = LAYOUT != PT_LAYOUT_TILED_PLANAR8;
    if (!kCountable && count) return hipErrorInvalidValue;
    bool ct;
    if constexpr (kCountable)
        ct = count ? launch_ct<LAYOUT, ENV, true>(job, st, tiles, &presented, ct_blocks)
                   : launch_ct<LAYOUT, ENV, false>(job, st, tiles, &presented, ct_blocks);
    else
        ct = launch_ct<LAYOUT, ENV, false>(job, st, tiles, &presented, ct_blocks);
    if (ct)
        e = hipGetLastError();
    else
        e = launch_pools<LAYOUT, ENV>(job, st, count, tiles);
    if (e != hipSuccess || !job.pix_out || presented) return e;
    // the other pools do not present: the standalone output pass over the job's rows
    PtToneJob tj{job.buf, job.ncols, job.nrows, LAYOUT, 0, 0, job.pix_out, job.pix_xrgb ? PT_PIXEL_XRGB8 : PT_PIXEL_RGBA8, 1, 1};
    return pt_launch_tonemap(tj, st);
}

template <int LAYOUT, bool ENV>
hipError_t launch_pools(const PtJob& job, hipStream_t st, bool count, unsigned tiles)
{
    const bool multi = job.nframes > kChunk;
    const bool ring = !ENV && job.nframes >= kRingMinFrames && job.nframes > kChunk;
    if constexpr (LAYOUT == PT_LAYOUT_TILED_PLANAR8) {   // (no counting instances: launch_t)
        if (ring) launch_k<LAYOUT, ENV, false, true, !ENV>(job, st, tiles);
        else if (multi) launch_k<LAYOUT, ENV, false, true>(job, st, tiles);
        else launch_k<LAYOUT, ENV, false, false>(job, st, tiles);
    } else if (count) {
        if (ring) launch_k<LAYOUT, ENV, true, true, !ENV>(job, st, tiles);
        else if (multi) launch_k<LAYOUT, ENV, true, true>(job, st, tiles);
        else launch_k<LAYOUT, ENV, true, false>(job, st, tiles);
    } else {
        if (ring) launch_k<LAYOUT, ENV, false, true, !ENV>(job, st, tiles);
        else if (multi) launch_k<LAYOUT, ENV, false, true>(job, st, tiles);
        else launch_k<LAYOUT, ENV, false, false>(job, st, tiles);
    }
    return hipGetLastError();
}

// The schedule of the next launch from this launch's per-tile costs (trace iterations + 1), one
// workgroup, O(tiles) with coalesced loads:
//   (1) counting sort of the tiles by descending cost (costs capped at kCostBins - 1);
//   (2) units: inside the run of tiles of equal cost c, consecutive groups of max(1, kUnitCost / c)
//       tiles -- expensive tiles are units of their own, cheap ones are dequeued in runs.  Built
//       from the histogram alone (no per-tile prefix pass).
constexpr int kCostBins = 1024;
// The unit size adapts to the launch: the cheapest tiles (camera rays that miss: cost 1, ~4-6 us
// each) come last, and at the end of a 1080p launch units of 12 of them left ~3600 of the 5120
// waves idle while ~1500 ran 60-us units (per-tile timeline, scripts/diag_timeline.py).  Units
// of ~tiles / (1.5 x waves) iterations, clamped to [2, 12]: 1080p 4 (c2 360 -> 353 us), 4K 12
// (its 4x more cheap tiles keep every wave busy; 4 measured 1-2 % slower there).
constexpr uint32_t kUnitCostMax = 12, kUnitCostMin = 2;
static_assert(kCostBins == 1024, "the schedule kernel scans one histogram bin per thread");

// In-place exclusive scan of a[0..1023] by a 1024-thread workgroup (one entry per thread);
// returns the total.  Wave-level shuffles, then the 16 wave totals.
__device__ uint32_t block_exclusive_scan_1024(uint32_t* a, uint32_t* wave_tot)
{
    const uint32_t t = threadIdx.x, ln = t & 63, w = t >> 6;
    const uint32_t v = a[t];
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (ln >= (uint32_t)d) x += y;
    }
    if (ln == 63) wave_tot[w] = x;
    __syncthreads();
    if (t == 0) {
        uint32_t run = 0;
        for (int k = 0; k < 16; ++k) {
            const uint32_t c = wave_tot[k];
            wave_tot[k] = run;
            run += c;
        }
        wave_tot[16] = run;
    }
    __syncthreads();
    a[t] = wave_tot[w] + x - v;
    const uint32_t total = wave_tot[16];
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(1024) void pt_schedule_kernel(const uint32_t* __restrict__ cost, uint32_t* __restrict__ order,
                                                           uint32_t* __restrict__ units, uint32_t* __restrict__ nunits,
                                                           uint32_t n, uint32_t kUnitCost, uint32_t split_div,
                                                           uint32_t* err)
{
    __shared__ uint32_t hist[kCostBins];    // entries per bin, then the bin's first schedule position
    __shared__ uint32_t ucnt[kCostBins];    // units per bin, then the bin's first unit index
    __shared__ uint32_t wave_tot[17];
    __shared__ unsigned long long s_total;
    const uint32_t t = threadIdx.x;
    constexpr uint32_t nt = 1024, kBatch = 8;
    constexpr uint32_t kNoTile = 0xffffffffu;
    hist[t] = 0;
    if (t == 0) s_total = 0;
    __syncthreads();
    // a tile's cost: its two words (a whole tile's second is 0, a split tile's halves are one each)
    auto cost_at = [&](uint32_t i) { return i < n ? cost[i] + cost[n + i] : kNoTile; };
    // descending cost: the most expensive entries get bin 0
    auto bin_of = [&](uint32_t c) {
        return (uint32_t)(kCostBins - 1) - (c < (uint32_t)(kCostBins - 1) ? c : (uint32_t)(kCostBins - 1));
    };
    // (0) the split threshold: tiles costing more than total / split_div become two entries
    uint32_t thr = 0xffffffffu;
    if (split_div) {
        unsigned long long part = 0;
        for (uint32_t i = t; i < n; i += nt) part += cost[i] + cost[n + i];
        atomicAdd(&s_total, part);
        __syncthreads();
        const unsigned long long th = s_total / split_div;
        thr = th < 0xffffffffull ? (uint32_t)th : 0xffffffffu;
    }
    auto split = [&](uint32_t c) { return c > thr && c >= 2u; };
    for (uint32_t base = 0; base < n; base += nt * kBatch) {
        uint32_t c[kBatch];
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) c[k] = cost_at(base + k * nt + t);   // loads in flight together
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            if (c[k] == kNoTile) continue;
            if (split(c[k])) atomicAdd(&hist[bin_of((c[k] + 1u) >> 1)], 2u);
            else atomicAdd(&hist[bin_of(c[k])], 1u);
        }
    }
    __syncthreads();
    const uint32_t count = hist[t];   // bin t
    const uint32_t npos = block_exclusive_scan_1024(hist, wave_tot);   // hist[b]: the bin's first schedule position
    // units of bin t: cost c = kCostBins - 1 - t, k = max(1, U / c) entries each
    const uint32_t c = (uint32_t)(kCostBins - 1) - t;
    const uint32_t per = c >= kUnitCost || c == 0 ? 1u : kUnitCost / c;
    ucnt[t] = (count + per - 1) / per;
    __syncthreads();
    const uint32_t total_units = block_exclusive_scan_1024(ucnt, wave_tot);
    // unit u of bin b starts at schedule position hist[b] + (u - ucnt[b]) * per(b): every thread
    // writes every 1024th unit, its bin found by binary search over the bins' first units (one
    // thread per bin would write a whole large bin serially)
    for (uint32_t u = t; u < total_units; u += nt) {
        uint32_t lo = 0, hi = kCostBins - 1;   // the last bin whose first unit is <= u
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (ucnt[mid] <= u) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t cb = (uint32_t)(kCostBins - 1) - lo;
        const uint32_t pb = cb >= kUnitCost || cb == 0 ? 1u : kUnitCost / cb;
        if (PT_GUARD(err, u < 2u * n, PT_G_SCHED_UNIT, u)) units[u] = hist[lo] + (u - ucnt[lo]) * pb;
    }
    __syncthreads();   // hist is advanced by the scatter below
    if (t == 0 && PT_GUARD(err, total_units <= 2u * n && npos <= 2u * n, PT_G_SCHED_UNIT, total_units)) {
        *nunits = total_units;
        units[total_units] = npos;
    }
    // scatter: order[position] = entry (positions inside a bin in arbitrary order; a split tile's
    // two halves land next to each other only by chance)
    for (uint32_t base = 0; base < n; base += nt * kBatch) {
        uint32_t cc[kBatch];
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) cc[k] = cost_at(base + k * nt + t);
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            if (cc[k] == kNoTile) continue;
            const uint32_t tile = base + k * nt + t;
            // (the checked build: every position inside order's 2 n entries)
            auto put = [&](uint32_t pos, uint32_t e) {
                if (PT_GUARD(err, pos < 2u * n, PT_G_SCHED_ORDER, pos)) order[pos] = e;
            };
            if (split(cc[k])) {
                const uint32_t b = bin_of((cc[k] + 1u) >> 1);
                put(atomicAdd(&hist[b], 1u), tile | (1u << PT_TILE_PART_SHIFT));
                put(atomicAdd(&hist[b], 1u), tile | (2u << PT_TILE_PART_SHIFT));
            } else {
                put(atomicAdd(&hist[bin_of(cc[k])], 1u), tile);
            }
        }
    }
}

}  // namespace

hipError_t pt_launch_schedule(const uint32_t* cost, uint32_t* order, uint32_t* units, uint32_t* nunits,
                              uint32_t ntiles, uint32_t split, uint32_t unit_mult, hipStream_t st, uint32_t* err)
{
    if (ntiles == 0) return hipSuccess;
    if (!cost || !order || !units || !nunits) return hipErrorInvalidValue;
    uint32_t unit_cost;
    {   // adaptive: ~tiles / (1.5 x resident waves), 20 waves per CU
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        const uint32_t waves = (uint32_t)cus * 20u;
        unit_cost = (uint32_t)((2ull * ntiles) / (3ull * waves));
        unit_cost = std::min(kUnitCostMax, std::max(kUnitCostMin, unit_cost)) * (unit_mult ? unit_mult : 1u);
    }
    uint32_t split_div = 0;
    {   // tiles costing more than 1/split of a wave's share are split (pt_tile_queue.h)
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        split_div = split ? (uint32_t)cus * 20u * split : 0u;
    }
    hipLaunchKernelGGL(pt_schedule_kernel, dim3(1), dim3(1024), 0, st, cost, order, units, nunits, ntiles, unit_cost,
                       split_div, err);
    return hipGetLastError();
}

hipError_t pt_set_chain_polls(uint32_t polls)
{
    const uint32_t v = polls ? polls : kPtChainPolls;
    return hipMemcpyToSymbol(HIP_SYMBOL(pt_chain_polls_dev), &v, sizeof(v));
}

uint32_t pt_ct_wave_floats() { return kCtWaveFloats; }

int32_t pt_ct_env_waves() { return PT_ENV_WAVES; }

uint32_t pt_ct_resident_waves()
{
    static_assert(waves_per_block<false>() == waves_per_block<true>(), "one block shape for the CT kernels");
    constexpr int wpb = waves_per_block<false>();
    // (every continuous-tiles instance launch_ct can pick; the presenting ones have the plain ones'
    // occupancy attributes and LDS, and launch_ct checks the grid against ct_waves anyway)
    const int r[] = {pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_INTERLEAVED, false, 5>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_INTERLEAVED, true, 5>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_PLANAR8, false, 5>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_PLANAR8, true, 5>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_TILED_PLANAR8, false, 5>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_INTERLEAVED, false, 6>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_INTERLEAVED, true, 6>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_PLANAR8, false, 6>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_PLANAR8, true, 6>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_kernel<PT_LAYOUT_TILED_PLANAR8, false, 6>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_env_kernel<PT_LAYOUT_INTERLEAVED, false>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_env_kernel<PT_LAYOUT_INTERLEAVED, true>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_env_kernel<PT_LAYOUT_PLANAR8, false>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_env_kernel<PT_LAYOUT_PLANAR8, true>, 64 * wpb),
                     pt_resident_blocks(pt_render_ct_env_kernel<PT_LAYOUT_TILED_PLANAR8, false>, 64 * wpb)};
    return (uint32_t)*std::max_element(std::begin(r), std::end(r)) * (uint32_t)wpb;
}

hipError_t pt_launch_render(const PtJob& job_in, hipStream_t st, bool count, uint32_t* ct_blocks)
{
    if (ct_blocks) *ct_blocks = 0;
    if (job_in.ncols <= 0 || job_in.nrows <= 0) return hipSuccess;
    if (job_in.nframes <= 0) {   // nothing to render; a presenting job still converts the accumulator
        if (!job_in.pix_out) return hipSuccess;
        const PtToneJob tj{job_in.buf, job_in.ncols, job_in.nrows, job_in.layout, 0, 0, job_in.pix_out,
                           job_in.pix_xrgb ? PT_PIXEL_XRGB8 : PT_PIXEL_RGBA8, 1, 1};
        return pt_launch_tonemap(tj, st);
    }
    if (!job_in.scene || !job_in.buf || !job_in.queue) return hipErrorInvalidValue;
    // mainImage's frame constants (scalar.cpp:338-347): IEEE f32 '/' here (host, -ffp-contract=off)
    // == the kernel's correctly rounded div_x / rcp_rn
    PtJob job = job_in;
    job.cam_W = (float)job.width;
    job.cam_H = (float)job.height;
    job.cam_yW = 1.0f / job.cam_W;
    job.cam_yH = 1.0f / job.cam_H;
    job.cam_aspect = job.cam_W / job.cam_H;
    job.cam_yAspect = 1.0f / job.cam_aspect;
    if (job.env) {
        if (job.env_w <= 0 || job.env_h <= 0) return hipErrorInvalidValue;
        switch (job.layout) {
            case PT_LAYOUT_INTERLEAVED: return launch_t<PT_LAYOUT_INTERLEAVED, true>(job, st, count, ct_blocks);
            case PT_LAYOUT_PLANAR8: return launch_t<PT_LAYOUT_PLANAR8, true>(job, st, count, ct_blocks);
            case PT_LAYOUT_TILED_PLANAR8: return launch_t<PT_LAYOUT_TILED_PLANAR8, true>(job, st, count, ct_blocks);
            default: return hipErrorInvalidValue;
        }
    }
    switch (job.layout) {
        case PT_LAYOUT_INTERLEAVED: return launch_t<PT_LAYOUT_INTERLEAVED, false>(job, st, count, ct_blocks);
        case PT_LAYOUT_PLANAR8: return launch_t<PT_LAYOUT_PLANAR8, false>(job, st, count, ct_blocks);
        case PT_LAYOUT_TILED_PLANAR8: return launch_t<PT_LAYOUT_TILED_PLANAR8, false>(job, st, count, ct_blocks);
        default: return hipErrorInvalidValue;
    }
}
