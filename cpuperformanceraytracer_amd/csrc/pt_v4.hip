// pt_v4.hip -- the reference's shipping renderer (demofox_path_tracing_optimization_v4.cpp,
// DemofoxRenderOptV4 :1696-1721 -> RenderTile :1179-1258 -> mainImage :1092-1130 ->
// GetColorForRay :722-911) as one HIP kernel for gfx950.
//
// Materials: diffuse / specular (roughness-lerped reflection) / refraction (Fresnel-Schlick,
// Beer absorption with approx_exp), Russian-roulette throughput boost, jittered camera, env map
// (equirect or cubemap, random-jitter or bilinear texel sampling) weighted by the throughput.
//
// Mapping: the reference runs 8 pixels per AVX2 register, each with its own RNG state, looping
// until all 8 paths end.  Here one wave owns an 8x8 tile and the (pixel, frame) samples of the
// tile form a pool of items: a lane that finishes a path takes the next item (ballot + mbcnt), so
// no lane idles while paths of the tile remain.  Each sample's radiance goes to LDS; at the end
// the lane of each pixel accumulates its frames in frame order with the reference's fused lerp
// (:1243) -- read once, written once per launch.
//
// Numerics: the reference's f32 operations in its order, fmadd/fmsub/fnmadd fused, '/' and sqrt
// correctly rounded; rcp / rsroot are the exact 1/x and 1/sqrtf(x) (mathlib.h:415,437 -- the
// x86 approximations have no portable bit pattern); atan2/asin/sin/cos are glibc's
// (pt_invtrig.h, pt_sincosf.h).  Bit-identical to oracle/pt_oracle_v4.c.
#include "pt_v4.h"
#include "pt_kernel.h"
#include "pt_exactmath.h"
#include "pt_sincosf.h"
#include "pt_libmf.h"
// atan2f/asinf with the guarded fast '/' and sqrt (bit-identical to IEEE, pt_exactmath.h)
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
#include "pt_v4_default_scene.h"
#include "pt_tile_queue.h"
#include "pt_guard.h"
#include "pt_chain.h"
#include "pt_wave.h"
#include "pt_tonemap.h"
#include <algorithm>

namespace {

constexpr float kMinHit = 0.01f;      // c_minimumRayHitTime  v4 :10
constexpr float kNudge = 0.01f;       // c_rayPosNormalNudge  v4 :14
constexpr float kSuperFar = 10000.0f; // c_superFar           v4 :17
constexpr float kPi = 3.14159265359f; // c_pi                 mathutils.h:5
constexpr int kWaves = 4;    // waves (tiles) per workgroup
constexpr int kChunk = 8;    // frames per LDS chunk
// Env modes: a miss adds fma(env(dir), throughput, ret) (:787), two glibc inverse-trig calls (or a
// cube-face pick) and texel gathers.  Evaluated where the miss happens it runs in most pool
// iterations for a fraction of the lanes.  Deferred, the miss stores ret in its colour slot and
// queues (env dir, rng, throughput, slot) in LDS; when the queue would overflow, all lanes
// evaluate one queued miss each (the same fma on the same operands, bit for bit) -- or, when the
// new misses outnumber the queue, those are evaluated at once.  The queue is drained before
// phase C.  kEnvQ entries of 32 B per wave keep the block at 31 536 B of LDS, 25 of the 1280-B
// granules, so 5 blocks per CU stay resident (the VGPR-bound occupancy; at 56 entries the block
// needed 26 granules and dropped to 4 per CU, and the queue then measured slower).  1920x1080 x
// 8 spp, 8 bounces: equirect 0.615 -> 0.561 ms, cubemap 0.525 -> 0.510 ms.
constexpr int kEnvQ = 48;

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 sel(bool c, V3 a, V3 b) { return v3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ float dot(V3 u, V3 v) { return fma_(u.x, v.x, fma_(u.y, v.y, u.z * v.z)); }   // mathlib.h:145
__device__ __forceinline__ V3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }
__device__ __forceinline__ float max_ps(float a, float b) { return a > b ? a : b; }   // MAXPS: b on NaN
__device__ __forceinline__ float min_ps(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float saturate(float x) { return min_ps(max_ps(x, 0.0f), 1.0f); }
// correctly rounded 1/x and sqrt: the fast sequences of pt_exactmath.h inside their verified
// ranges, IEEE outside (bit-identical to '1.0f / x' and sqrtf for every input)
__device__ __forceinline__ float rcp(float x)   // rcp -> 1.f / x (mathlib.h:415)
{
    float r = pt::rcp_rn(x);
    const float ax = __builtin_fabsf(x);
    if (__builtin_expect(!(ax >= 0x1p-125f && ax <= 0x1p125f), 0)) r = 1.0f / x;
    return r;
}
// 1.f / x for an x >= 0 (or NaN) that is provably <= 2^125: only the lower end of rcp_rn's range can
// fail (0, denormals), one compare guards it
__device__ __forceinline__ float rcp_nonneg(float x)
{
    float r = pt::rcp_rn(x);
    if (__builtin_expect(!(x >= 0x1p-125f), 0)) r = pt::rcp_tiny_rn(x);   // 0, denormals, NaN
    return r;
}
__device__ __forceinline__ float sqrt_(float x) { return pt::sqrt_guarded(x); }
__device__ __forceinline__ V3 normalize(V3 v) { return v * rcp(sqrt_(dot(v, v))); }  // mathlib.h:759
// normalize of a vector no longer than ~2 (unit vectors, their sums and lerps): sqrt(dot) <= 2^125
__device__ __forceinline__ V3 normalize_small(V3 v) { return v * rcp_nonneg(sqrt_(dot(v, v))); }

__device__ __forceinline__ uint32_t wang(uint32_t& s)   // mathutils.h:8-16 (logical shifts)
{
    uint32_t x = s;
    x = (x ^ 61u) ^ (x >> 16);
    x *= 9u;
    x = x ^ (x >> 4);
    x *= 0x27d4eb2du;
    x = x ^ (x >> 15);
    s = x;
    return x;
}
__device__ __forceinline__ void rng_skip(uint32_t& s, int n)   // draws whose values are not used
{
    for (int i = 0; i < n; ++i) wang(s);
}
// Randomf3201_ps (mathutils.h:18-26): cvtepi32_ps(h & 0x7FFFFFFF) / 2^31 (an exact scaling)
__device__ __forceinline__ float randf(uint32_t& s) { return (float)(int32_t)(wang(s) & 0x7FFFFFFFu) * 0x1p-31f; }

__device__ __forceinline__ V3 ruv_rejection(uint32_t& s)   // v4 :109-130
{
    const float u = fma_(2.0f, randf(s), -1.0f);
    const float v = fma_(2.0f, randf(s), -1.0f);
    const float w = fma_(2.0f, randf(s), -1.0f);
    const float d2 = fma_(w, w, fma_(u, u, v * v));
    return v3(u, v, w) * rcp(sqrt_(d2));   // rsroot -> 1/sqrtf (mathlib.h:437)
}

// the same unit vector from three draws already taken (h0, h1, h2 = wang's outputs in draw order)
__device__ __forceinline__ float randf_of(uint32_t h) { return (float)(int32_t)(h & 0x7FFFFFFFu) * 0x1p-31f; }
__device__ __forceinline__ V3 ruv_rejection_of(uint32_t h0, uint32_t h1, uint32_t h2)
{
    const float u = fma_(2.0f, randf_of(h0), -1.0f);
    const float v = fma_(2.0f, randf_of(h1), -1.0f);
    const float w = fma_(2.0f, randf_of(h2), -1.0f);
    const float d2 = fma_(w, w, fma_(u, u, v * v));
    return v3(u, v, w) * rcp(sqrt_(d2));
}

__device__ __forceinline__ V3 ruv_angle(uint32_t& s)   // mathutils.h:33-46 (sincos -> glibc sinf/cosf)
{
    const float wz = randf(s);
    const float wa = randf(s);
    const float z = wz * 2.0f - 1.0f;
    const float a = wa * (2.0f * kPi);
    const float r = sqrt_(1.0f - z * z);
    float sa, ca;
    pt::sincosf_glibc(a, &sa, &ca);
    return v3(r * ca, r * sa, z);
}

// ---- env lookups (texture.cpp) -----------------------------------------------------------------

struct Tex {
    const float* data;
    int32_t w, h;
};

// GatherRGB (:16-26) at f32 element index `f` after cvtps_epi32 (nearest even; INT_MIN when out of
// range).  Outside the texture the reference reads out of bounds (UB); clamped here exactly like the
// oracle: negative / INT_MIN -> element 0, past the end -> the last texel.
__device__ __forceinline__ V3 texel_at(const Tex& t, float f)
{
    f = __builtin_rintf(f);
    const int32_t last = 3 * (t.w * t.h - 1);
    int32_t e = 0;
    if (f >= 0.0f && f < 2147483648.0f) {
        e = (int32_t)f;
        e = e > last ? last : e;
    }
    const float* p = t.data + (uint32_t)e;
    return v3(p[0], p[1], p[2]);
}

// TexelSampleRandom's index 3 * cvtps_epi32(texel) (:84): texel clamped to [0, n-1] before the multiply
__device__ __forceinline__ V3 texel_rn(const Tex& t, float f)
{
    f = __builtin_rintf(f);
    const int32_t nn = t.w * t.h;
    int32_t i = 0;
    if (f >= 0.0f && f < 2147483648.0f) {
        i = (int32_t)f;
        i = i >= nn ? nn - 1 : i;
    }
    const float* p = t.data + 3u * (uint32_t)i;
    return v3(p[0], p[1], p[2]);
}

__device__ __forceinline__ V3 sample_random(const Tex& t, float u, float v, uint32_t& s)   // :78-86
{
    const float Row = fma_(v, (float)t.h, -v);
    const float Col = fma_(u, (float)t.w, -u);
    const float rr = __builtin_floorf(Row + randf(s));
    const float rc = __builtin_floorf(Col + randf(s));
    return texel_rn(t, fma_(rr, (float)t.w, rc));
}

__device__ __forceinline__ V3 sample_bilinear(const Tex& t, float u, float v)   // :38-76
{
    const float Row = v * (float)(t.h - 1);
    const float Col = u * (float)(t.w - 1);
    float Row0 = __builtin_floorf(Row), Row1 = __builtin_ceilf(Row);
    float Col0 = __builtin_floorf(Col), Col1 = __builtin_ceilf(Col);
    const float dV = Row - Row0, dU = Col - Col0;
    const float tw = 3.0f * (float)t.w;
    Row0 = Row0 * tw;
    Row1 = Row1 * tw;
    Col0 = Col0 * 3.0f;
    Col1 = Col1 * 3.0f;
    const V3 C00 = texel_at(t, Col0 + Row0), C10 = texel_at(t, Col1 + Row0);
    const V3 C01 = texel_at(t, Col0 + Row1), C11 = texel_at(t, Col1 + Row1);
    const V3 C0 = C00 + (C10 - C00) * dU;   // lerp mathlib.h:763
    const V3 C1 = C01 + (C11 - C01) * dU;
    return C0 + (C1 - C0) * dV;
}

__device__ __forceinline__ V3 equirect(const Tex& t, V3 d, bool random, uint32_t& s)
{
    if (random) {   // EquirectangularTextureSampleRandom :186-203 + TexelSampleRandom :78-86
        // the texel cell certified from short atan/asin polynomials (pt_envcert.h); the glibc-exact
        // angles only for the rare uncertified cells (a divergent branch, skipped when no lane needs it)
        const float r1 = randf(s), r2 = randf(s);   // the sampler's draws, Row's first
        const float fw = (float)t.w, fh = (float)t.h;
        float rr, rc;
        if (__builtin_expect(!pt::ec_cell_random(d.z, d.x, d.y, fw, fh, r1, r2, rr, rc), 0)) {
            const float at = pt::atan2f_glibc(d.z, d.x), as = pt::asinf_glibc(d.y);
            float u = fma_(0.1591f, at, 0.5f), v = fma_(0.3183f, as, 0.5f);
            u = saturate(u - __builtin_floorf(u));
            v = saturate(v - __builtin_floorf(v));
            rr = __builtin_floorf(fma_(v, fh, -v) + r1);
            rc = __builtin_floorf(fma_(u, fw, -u) + r2);
        }
        return texel_rn(t, fma_(rr, fw, rc));
    }
    const float at = pt::atan2f_glibc(d.z, d.x), as = pt::asinf_glibc(d.y);
    float u = at * 0.1591f + 0.5f, v = as * 0.3183f + 0.5f;   // Bilinear :164-184
    u = u - __builtin_floorf(u);
    v = v - __builtin_floorf(v);
    return sample_bilinear(t, saturate(u), saturate(v));
}

__device__ __forceinline__ V3 cubemap(const Tex& t, V3 d, bool random, uint32_t& s)   // :275-404
{
    const float ax = __builtin_fabsf(d.x), ay = __builtin_fabsf(d.y), az = __builtin_fabsf(d.z);
    const float k = 0.166666666666667f;
    // face offsets: Random uses multiples of 0.166666666666667f, Bilinear i/6.f
    const float o1 = random ? k : 1.0f / 6.0f, o2 = random ? 2.0f * k : 2.0f / 6.0f, o3 = random ? 3.0f * k : 3.0f / 6.0f;
    const float o4 = random ? 4.0f * k : 4.0f / 6.0f, o5 = random ? 5.0f * k : 5.0f / 6.0f;
    const bool cx = d.x >= 0.0f;
    float fu = cx ? -d.z : d.z, fv = d.y, voff = cx ? 0.0f : o1;
    if (ay >= ax) {
        const bool cy = d.y >= 0.0f;
        voff = cy ? o2 : o3;
        fu = d.x;
        fv = cy ? -d.z : d.z;
    }
    if (az >= ax && az >= ay) {
        const bool cz = d.z >= 0.0f;
        voff = cz ? o4 : o5;
        fu = cz ? d.x : -d.x;
        fv = d.y;
    }
    const float m = max_ps(ax, max_ps(ay, az));
    if (random) {
        const float r = rcp(m);
        const float u = saturate(fma_(fu * r, 0.5f, 0.5f));
        float v = saturate(fma_(fv * r, 0.5f, 0.5f));
        v = saturate(fma_(v, 0.166666666666667f, voff));
        return sample_random(t, u, v, s);
    }
    const float u = saturate(pt::div_guarded(fu, m) * 0.5f + 0.5f);
    float v = saturate(pt::div_guarded(fv, m) * 0.5f + 0.5f);
    v = saturate(fma_(v, 1.0f / 6.0f, voff));
    return sample_bilinear(t, u, v);
}

// ---- intersection and shading -------------------------------------------------------------------

// Per-material constants of fresnel() and the refraction ratio, evaluated once per block with the
// very operations the per-hit code used (so the same bits): r0 = (n1 - n2) * rcp(n1 + n2) squared
// is the same for (n1, n2) = (1, ior) and (ior, 1) (1 + ior == ior + 1, 1 - ior == -(ior - 1));
// n1 * rcp(n2) is rcp(ior) outside (1 * x == x) and ior inside (rcp(1) == 1).
struct MatX {
    float r0sq, omr0, rior, nnout, rscc;
};
__device__ __forceinline__ MatX mat_consts(const PtV4Mat& M)
{
    MatX x;
    float r0 = (1.0f - M.ior) * rcp(1.0f + M.ior);
    x.r0sq = r0 * r0;
    x.omr0 = 1.0f - x.r0sq;
    x.rior = rcp(M.ior);
    x.nnout = x.rior * x.rior;
    x.rscc = rcp(1.0f - M.spec_chance);
    return x;
}

// Fresnel-Schlick (v4 :429-453) for (n1, n2) = inside ? (ior, 1) : (1, ior), with the constants of MatX
__device__ __forceinline__ float fresnel_m(bool inside, float ior, const MatX& X, V3 normal, V3 incident, float f0)
{
    const float r0 = X.r0sq;
    float cosX = -dot(normal, incident);
    const bool cond = inside ? ior > 1.0f : 1.0f > ior;
    const float nn = inside ? ior * ior : X.nnout;
    const float stc = fma_(-nn, fma_(-cosX, cosX, 1.0f), 1.0f);
    const float ncos = sqrt_(stc);
    const bool tir = 0.0f > stc;
    cosX = (cond && !tir) ? ncos : cosX;
    const float x = 1.0f - cosX;
    const float x2 = x * x;
    float ret = fma_((X.omr0 * x2) * x2, x, r0);
    ret = (cond && tir) ? 1.0f : ret;
    return fma_(ret, 1.0f - f0, f0);
}

__device__ __forceinline__ V3 refract(V3 v, V3 n, float ior)   // rfrct, mathlib.h:781-789
{
    const float vdn = dot(v, n);
    const float k = fma_(-ior, ior * fma_(-vdn, vdn, 1.0f), 1.0f);
    const float s = fma_(ior, vdn, sqrt_(k));
    const V3 r = v3(fma_(ior, v.x, -(s * n.x)), fma_(ior, v.y, -(s * n.y)), fma_(ior, v.z, -(s * n.z)));
    return k < 0.0f ? v3(0.0f, 0.0f, 0.0f) : r;
}

__device__ __forceinline__ float approx_exp(float a)   // mathlib.h:501-516
{
    const float b = fma_(a, 0.05995203836930455f, 1.0f);
    const float b2 = b * b, b4 = b2 * b2, b8 = b4 * b4;
    return b8 * b8;
}

struct Hit {
    float dist;
    V3 n;
    bool inside;
    int mat;
};

// TestQuadTrace :556-637 for one quad (the reference's operations; `dk` evaluates its fused dots)
// DEF (InitializeScene's quads): 1/rdn without the range guard.  Their normals are axis vectors and
// their v0 components have magnitudes >= 1.5, so ron = dot(v0 - pos, n) = +-(v0_j - pos_j) is 0 or
// >= 6e-8 in magnitude (Sterbenz, or >= |v0_j| / 2).  The reference keeps dist = ron / rdn only inside
// (0.01, best <= 1e4), which needs |rdn| >= 6e-12 -- inside rcp_rn's range, where the values agree.
// Outside it (|rdn| < 2^-125, 0, NaN) both quotients are 0, huge, +-inf or NaN: rejected either way.
template <bool DEF, class DOT>
__device__ __forceinline__ void quad_test(V3 pos, V3 dir, Hit& h, int obj, V3 v0, V3 n, const DOT& dk, int q)
{
    const V3 off = v0 - pos;
    const float rdn = dk(dir, q, 1);   // dot(dir, normal)
    const float dist = dk(off, q, 1) * (DEF ? pt::rcp_rn(rdn) : rcp(rdn));
    // the hit needs (tri1 || tri2) && 0.01 < dist < best: the barycentric tests only run for
    // distances in range (a wave whose lanes all fail skips them)
    if (dist > kMinHit && dist < h.dist) {
        const V3 hp = v3(fma_(dist, dir.x, -off.x), fma_(dist, dir.y, -off.y), fma_(dist, dir.z, -off.z));
        const float A0 = dk(hp, q, 2), A1 = dk(hp, q, 3), A2 = 1.0f - A0 - A1;
        const float B0 = dk(hp, q, 4), B1 = dk(hp, q, 5), B2 = 1.0f - B0 - B1;
        const bool tri1 = A0 >= 0.0f && A1 >= 0.0f && A2 >= 0.0f;
        const bool tri2 = B0 >= 0.0f && B1 >= 0.0f && B2 >= 0.0f;
        if (tri1 || tri2) {
            h.inside = false;
            h.dist = dist;
            if (rdn > 0.0f) h.n = neg(n);   // only back-side hits write the normal (:630)
            h.mat = obj;
        }
    }
}

// TestSphereTrace :641-695
__device__ __forceinline__ void sphere_test(V3 pos, V3 dir, Hit& h, int obj, V3 c, float r)
{
    const V3 m = pos - c;
    const float b = dot(m, dir);
    const float cc = fma_(-r, r, dot(m, m));
    const float discr = fma_(b, b, -cc);
    const bool early = discr < 0.0f || (cc > 0.0f && b > 0.0f);
    if (!early) {   // the root and the distance only for candidates (most rays miss most spheres)
        const float s = sqrt_(discr);
        const bool inside = -b < s;
        const float dist = (inside ? s : -s) - b;
        if (dist > kMinHit && dist < h.dist) {
            h.inside = inside;
            h.dist = dist;
            const V3 p = v3(fma_(dir.x, dist, m.x), fma_(dir.y, dist, m.y), fma_(dir.z, dist, m.z));
            h.n = normalize(p) * (inside ? -1.0f : 1.0f);
            h.mat = obj;
        }
    }
}

// the reference's dot fma(x,x', fma(y,y', z*z')) against a COMPILE-TIME vector with its zero
// components dropped.  Exact for every use in quad_test: dropping a term v*0 can only change the
// sign of a zero result, or a NaN from inf*0; the dots feed `>= 0` / `> 0` tests and 1 - A0 - A1
// (where +0 and -0 behave alike), and dist = ron * rcp(rdn), where a signed-zero rdn or ron gives
// +-inf or +-0 and a non-finite hit point needs a non-finite dist -- all of which fail the
// reference's 0.01 < dist < best test either way.
__device__ __forceinline__ float dot_k(V3 v, float cx, float cy, float cz)
{
    if (cz != 0.0f) {
        float t = v.z * cz;
        if (cy != 0.0f) t = fma_(v.y, cy, t);
        if (cx != 0.0f) t = fma_(v.x, cx, t);
        return t;
    }
    if (cy != 0.0f) {
        float t = v.y * cy;
        if (cx != 0.0f) t = fma_(v.x, cx, t);
        return t;
    }
    return cx != 0.0f ? v.x * cx : 0.0f;
}

// Closest sphere only (default scene).  TestSphereTrace's result for the whole sphere list is the
// accepted sphere with the smallest distance.  The default scene's spheres are pairwise disjoint
// balls, at least kSphereGap apart (static_assert below), so along any ray the chords of two balls
// the ray meets are disjoint and kSphereGap apart, and they come in the order of the centres'
// projections -b.  (Both balls within r of the line => their projections differ by
// sqrt(|c_i - c_j|^2 - (r_i + r_j)^2) > 0; a ball holding the origin has the chord around t = 0, and
// every ball behind the origin is rejected by the reference's own early test.)  So of the spheres
// the reference does not reject early -- computed with its exact operations -- the one with the
// largest b is the only one whose distance can be the smallest: its root, distance and normal are
// evaluated once, exactly as TestSphereTrace does.  When its distance fails c_minimumRayHitTime
// (the origin within 0.01 of its surface) a later sphere could still be accepted, so that ray runs
// the reference's sequential tests (`fallback`, rare).  Rounding moves a distance by ~1e-5, far
// inside the gap (0.4 in the default scene; asserted >= kSphereGap).
constexpr float kSphereGap = 0.1f;
constexpr bool default_spheres_disjoint()
{
    namespace D = pt_v4_default;
    for (int i = 0; i < D::kSpheres; ++i)
        for (int j = i + 1; j < D::kSpheres; ++j) {
            const float dx = D::kSphere[i][0] - D::kSphere[j][0], dy = D::kSphere[i][1] - D::kSphere[j][1],
                        dz = D::kSphere[i][2] - D::kSphere[j][2];
            const float rr = D::kSphere[i][3] + D::kSphere[j][3] + kSphereGap;
            if (!(dx * dx + dy * dy + dz * dz > rr * rr)) return false;
        }
    return true;
}
static_assert(default_spheres_disjoint(), "the closest-sphere trace needs pairwise disjoint spheres");
// The candidate with the largest b without tracking it (the sphere-order rule).  InitializeScene's
// spheres lie on one line parallel to x, in ascending x, `spacing` apart, radius r, 2r < spacing
// (asserted below).  Then b_i = (pos - c_i).dir = b_0 - i spacing dir.x exactly, so the largest b of
// the candidates is the lowest candidate index when dir.x > 0 and the highest when dir.x < 0 --
// provided the computed b's keep that order.  They do: two candidates i < j mean the line passes
// within r (+ the discriminant's rounding, ~1e-4) of both centres, so its closest approaches are
// >= (j - i) spacing - 2r >= 0.4 apart along the line, |dir.x| >= 0.4 / ((j - i) spacing) and the
// exact b's differ by >= 0.4 -- against rounding errors of ~1e-5 in b.  (dir.x == 0 admits at most
// one candidate.)  A NaN ray makes every b NaN: the reference's b > bmax never takes one, and the
// recomputed b of the chosen index is NaN too, which drops it.  The kernel keeps the per-sphere
// early tests (exactly) and replaces the per-sphere compare + three selects by a candidate bit mask.
constexpr bool default_spheres_on_x_line()
{
    namespace D = pt_v4_default;
    for (int i = 1; i < D::kSpheres; ++i) {
        if (D::kSphere[i][1] != D::kSphere[0][1] || D::kSphere[i][2] != D::kSphere[0][2] ||
            D::kSphere[i][3] != D::kSphere[0][3])
            return false;
        if (!(D::kSphere[i][0] - D::kSphere[i - 1][0] >= 2.0f * D::kSphere[0][3] + 0.4f)) return false;
    }
    return D::kSpheres <= 32;
}
static_assert(default_spheres_on_x_line(),
              "the sphere-order rule needs InitializeScene's spheres on one x line, >= 0.4 apart");
static_assert(pt_v4_default::kSphere[0][3] > 1.0f && pt_v4_default::kSphere[0][3] < 4.0f,
              "the unguarded closest-sphere normal assumes radii of order 1 (all equal, above)");
#ifndef PT_V4_SPHERE_FORCE_SEQ
#define PT_V4_SPHERE_FORCE_SEQ 0   // test builds: every candidate ray takes the sequential fallback
#endif

// A camera ray of the default scene (origin (0, 0, 40), D.z < 0) that misses every primitive: with
// slopes sx = |D.x| / -D.z, sy = D.y / -D.z, InitializeScene's objects cover only
//   sy in [-0.5, -0.043], sx <= 1.0   (floor y = -12.5 at z 5..15, x +-25; stripes z = 5, y -10.5..-1.5,
//                                      x +-25; the sphere row y = -8, z = 10, x +-18, r 2.8)
//   sy in [0.357, 0.5],   sx <= 0.3   (ceiling y = 12.5, x +-7.5, z 5..15; the light inside it)
// (derived from the geometry; the oracle's TestSceneTrace on a 2400 x 1400 slope grid finds exactly
// these extents).  The thresholds below keep >= 0.0135 of slope (>= 0.3 units at the objects'
// distances) from every boundary -- far beyond the reference's rounding.  Checked against the v4
// oracle by tests/native/check_sky.cpp.
__device__ __forceinline__ bool sky_ray_v4(V3 D)
{
    const float nz = -D.z, ax = __builtin_fabsf(D.x);
    const bool band_hi = D.y > 0.34f * nz && D.y < 0.52f * nz && ax < 0.32f * nz;
    return nz > 0.0f && (D.y < -0.52f * nz || ax > 1.02f * nz || (D.y > -0.03f * nz && !band_hi));
}
static_assert(pt_v4_default::kQuads == 4 && pt_v4_default::kSpheres == 7, "sky_ray_v4 is derived for InitializeScene");

// TestSceneTrace :700-718: quads in order, then spheres (object index = material index).
// DEF: the reference's InitializeScene, geometry as instruction literals (pt_v4_default_scene.h,
// generated from pt_v4_build_scene and checked by tests/test_oracle_v4.py); otherwise the scene
// table of the kernel arguments (scalar loads per primitive).  s_sc: the default scene's sphere
// centres in LDS (DEF); fb: set when the closest-sphere stage fell back to the sequential tests.
template <bool DEF>
__device__ __forceinline__ Hit trace(const PtV4Scene& sc, V3 pos, V3 dir, const float4* s_sc, int& fb)
{
    Hit h{kSuperFar, v3(0.0f, 0.0f, 0.0f), false, 0};
    if constexpr (DEF) {
        namespace D = pt_v4_default;
        const auto dk = [](V3 v, int q, int k) {
            return dot_k(v, D::kQuad[q][3 * k], D::kQuad[q][3 * k + 1], D::kQuad[q][3 * k + 2]);
        };
#pragma unroll
        for (int i = 0; i < D::kQuads; ++i)
            quad_test<true>(pos, dir, h, i, v3(D::kQuad[i][0], D::kQuad[i][1], D::kQuad[i][2]),
                      v3(D::kQuad[i][3], D::kQuad[i][4], D::kQuad[i][5]), dk, i);
        {   // closest-sphere stage
            float bmax = -__builtin_huge_valf(), dsel = 0.0f;
            int ksel = -1;
            uint32_t cand = 0;   // spheres that pass the early test
#pragma unroll
            for (int i = 0; i < D::kSpheres; ++i) {   // :645-657, the early test exactly
                const V3 m = pos - v3(D::kSphere[i][0], D::kSphere[i][1], D::kSphere[i][2]);
                const float b = dot(m, dir);
                const float cc = fma_(-D::kSphere[i][3], D::kSphere[i][3], dot(m, m));
                const float discr = fma_(b, b, -cc);
                const bool early = discr < 0.0f || (cc > 0.0f && b > 0.0f);
                cand |= early ? 0u : 1u << i;
            }
            if (cand) {   // the largest b: by the sign of dir.x (the sphere-order rule above)
                ksel = dir.x > 0.0f ? __builtin_ctz(cand) : 31 - __builtin_clz(cand);
                const float4 c = s_sc[ksel];
                const V3 m = pos - v3(c.x, c.y, c.z);
                bmax = dot(m, dir);
                dsel = fma_(bmax, bmax, -fma_(-c.w, c.w, dot(m, m)));
                if (!(bmax == bmax)) ksel = -1;
            }
            bool seq = false;
            if (ksel >= 0) {
                const float4 c = s_sc[ksel];
                const V3 m = pos - v3(c.x, c.y, c.z);
                const float s = sqrt_(dsel);
                const bool inside = -bmax < s;
                const float dist = (inside ? s : -s) - bmax;
                if (dist > kMinHit && !PT_V4_SPHERE_FORCE_SEQ) {
                    if (dist < h.dist) {
                        h.inside = inside;
                        h.dist = dist;
                        const V3 p = v3(fma_(dir.x, dist, m.x), fma_(dir.y, dist, m.y), fma_(dir.z, dist, m.z));
                        // p = hit point - centre, |p| = the radius (2.8, asserted) up to rounding: the
                        // radicand and the divisor are far inside the fast paths' ranges, no guards
                        h.n = (p * pt::rcp_rn(pt::sqrt_rn(dot(p, p)))) * (inside ? -1.0f : 1.0f);
                        h.mat = D::kQuads + ksel;
                    }
                } else {
                    seq = true;
                }
            }
            if (__builtin_expect(seq, 0)) {   // rare; s_cbranch_execz skips it when no lane needs it
                fb = 1;
#pragma unroll 1
                for (int i = 0; i < D::kSpheres; ++i) {
                    const float4 c = s_sc[i];
                    sphere_test(pos, dir, h, D::kQuads + i, v3(c.x, c.y, c.z), c.w);
                }
            }
        }
    } else {
        int obj = 0;
        for (int i = 0; i < sc.nquads; ++i, ++obj) {
            const PtV4Quad& q = sc.quad[i];
            const float* t = &q.v0[0];
            const auto dk = [t](V3 v, int, int k) { return dot(v, ld3(t + 3 * k)); };
            quad_test<false>(pos, dir, h, obj, ld3(q.v0), ld3(q.n), dk, i);
        }
        for (int i = 0; i < sc.nspheres; ++i, ++obj) sphere_test(pos, dir, h, obj, ld3(sc.sph[i]), sc.sph[i][3]);
    }
    return h;
}

template <int LAYOUT>
__device__ __forceinline__ size_t out_index(const PtV4Job& j, int x, int r)   // r = buffer row
{
    if (LAYOUT == PT_LAYOUT_INTERLEAVED) return ((size_t)r * j.width + x) * 3u;
    if (LAYOUT == PT_LAYOUT_PLANAR8) return ((size_t)r * j.width + (size_t)(x & ~7)) * 3u + (size_t)(x & 7);
    const int tx = x / j.tile_w, ty = r / j.tile_h;   // RenderTile :1186-1191 (tiles of the full image)
    const int lx = x - tx * j.tile_w, ly = r - ty * j.tile_h;
    return (size_t)ty * j.tile_h * j.width * 3u + (size_t)tx * j.tile_w * j.tile_h * 3u +
           ((size_t)ly * j.tile_w + (size_t)(lx & ~7)) * 3u + (size_t)(lx & 7);
}

// The elements of the job's buffer (the checked build's pixel guard, pt_guard.h): the job's rows for
// the row layouts; the whole image in whole tile rows for the tiled layout, whose row index is global.
template <int LAYOUT>
__device__ __forceinline__ size_t pixel_extent(const PtV4Job& j)
{
    if (LAYOUT != PT_LAYOUT_TILED_PLANAR8) return (size_t)j.nrows * (size_t)j.width * 3u;
    const int rows = j.height > j.nrows ? j.height : j.nrows;
    return (size_t)((rows + j.tile_h - 1) / j.tile_h) * (size_t)j.tile_h * (size_t)j.width * 3u;
}

// One iteration of an item's path: GetColorForRay's bounce loop, :733-909 (the pool kernels' shared
// body).  done: the path ended (queued: DEFER, the miss's env term is deferred to the queue's drain).
template <int ENV, bool COUNT, bool DEF, int FEXP, bool DFL>
__device__ __forceinline__ void v4_segment(const PtV4Job& job, const PtV4Scene& sc, const PtV4Mat* s_mat,
                                           const MatX* s_mx, const float4* s_sc, const Tex& tex, bool random,
                                           bool rejection, int B, bool all_sky, V3& pos, V3& dir, V3& T, V3& ret,
                                           uint32_t& rng, int& bounce, bool& done, bool& queued,
                                           unsigned long long& n_seg, unsigned long long& n_esc,
                                           unsigned long long& n_fb, unsigned long long& n_sky)
{
    constexpr bool DEFER = ENV != PT_V4_ENV_NONE_;
    // one iteration of GetColorForRay's bounce loop (:733-909)
    int fb = 0;
    const Hit h = all_sky ? Hit{kSuperFar, v3(0.0f, 0.0f, 0.0f), false, 0} : trace<DEF>(sc, pos, dir, s_sc, fb);
    if (COUNT) ++n_seg, n_fb += (unsigned long long)fb, n_sky += all_sky ? 1ull : 0ull;
    const bool miss = h.dist == kSuperFar;
    done = false;
    if (miss) {
        if (DEFER) {
            queued = true;
        } else {
            V3 amb = v3(0.11f, 0.1f, 0.15f);   // :782
            if (ENV == PT_V4_ENV_EQUIRECT_) amb = equirect(tex, v3(-dir.x, dir.y, -dir.z), random, rng);
            if (ENV == PT_V4_ENV_CUBEMAP_) amb = cubemap(tex, dir, random, rng);
            ret = v3(fma_(amb.x, T.x, ret.x), fma_(amb.y, T.y, ret.y), fma_(amb.z, T.z, ret.z));   // :787
        }
        done = true;
        if (COUNT) ++n_esc;
    } else {
        if (ENV != PT_V4_ENV_NONE_ && random) {   // the env sample's two draws happen on hits too
            wang(rng);
            wang(rng);
        }
        const PtV4Mat& M = s_mat[h.mat];
        if (h.inside) {   // :797, Beer's law
            if (FEXP == 2 ? job.fast_exp != 0 : FEXP == 1)   // USE_FAST_APPROXIMATE_EXP 1 (:783-784)
                T = mul(T, v3(approx_exp(-M.refr_color[0] * h.dist), approx_exp(-M.refr_color[1] * h.dist),
                              approx_exp(-M.refr_color[2] * h.dist)));
            else                // 0 (:785-787): exp_ps -> glibc-exact expf (pt_libmf.h)
                T = mul(T, v3(pt::lm::expf_glibc(-M.refr_color[0] * h.dist),
                              pt::lm::expf_glibc(-M.refr_color[1] * h.dist),
                              pt::lm::expf_glibc(-M.refr_color[2] * h.dist)));
        }
        const V3 em = ld3(M.emissive);
        if (bounce == B) {   // last iteration: only its emissive term is used
            ret = v3(fma_(em.x, T.x, ret.x), fma_(em.y, T.y, ret.y), fma_(em.z, T.z, ret.z));
            done = true;
        } else {
            float spec = M.spec_chance, refr = M.refr_chance;
            if (spec > 0.0f) {   // :807-829 (the Fresnel result is used only with a specular chance)
                const MatX& X = s_mx[h.mat];
                const float nspec = fresnel_m(h.inside, M.ior, X, h.n, dir, M.spec_chance);
                const float rscc = X.rscc;
                spec = nspec;
                refr = refr * fma_(-nspec, rscc, rscc);
            }
            const float roll = randf(rng);   // :831
            const bool do_spec = spec > 0.0f && roll < spec;
            const bool do_refr = !do_spec && refr > 0.0f && roll < spec + refr;
            const float diff_chance = max_ps(1.0f - (spec + refr), 0.0f);
            float prob = do_spec ? spec : (do_refr ? refr : diff_chance);
            prob = max_ps(prob, 0.001f);
            const float nudge = kNudge * (do_refr ? -1.0f : 1.0f);   // :848-849
            const V3 npos = v3(fma_(nudge, h.n.x, fma_(dir.x, h.dist, pos.x)),
                               fma_(nudge, h.n.y, fma_(dir.y, h.dist, pos.y)),
                               fma_(nudge, h.n.z, fma_(dir.z, h.dist, pos.z)));
            // :852-888.  The reference evaluates the diffuse, specular and refraction
            // directions and selects one; only the selected one (and the diffuse direction
            // the specular one lerps towards) is evaluated here.  Both random unit vectors
            // are still drawn, in the reference's order (diffuse first).
            const bool unified = rejection;   // one straight-line direction for all three outcomes
            uint32_t s_diff = rng, s_refr = rng;
            uint32_t h0 = 0, h1 = 0, h2 = 0;   // unified: the chosen stream's three draws
            if (unified) {
                // both streams' draws once (6 hashes, not 6 skipped + 3 redrawn), then the
                // chosen stream's three selected -- the same values in the same order
                const uint32_t d0 = wang(rng), d1 = wang(rng), d2 = wang(rng);
                const uint32_t r0 = wang(rng), r1 = wang(rng), r2 = wang(rng);
                h0 = do_refr ? r0 : d0;
                h1 = do_refr ? r1 : d1;
                h2 = do_refr ? r2 : d2;
            } else {
                rng_skip(rng, rejection ? 3 : 2);
                s_refr = rng;
                rng_skip(rng, rejection ? 3 : 2);
            }
            V3 ndir;
            if (unified) {
                // The three outcomes share one shape: a unit vector u drawn from the chosen
                // stream, nb = (u +- n) * rcp(sqrt(|u +- n|^2)) (diffuse: n + u; refraction:
                // u - n == u + (-n) exactly), and -- for specular and refraction -- the
                // reference's fma lerp from a mirror direction R (reflect or refract) towards
                // nb.  Evaluated once per lane with per-lane operands instead of as two
                // divergent branches; every value is the branch's own, bit for bit.
                const V3 u = ruv_rejection_of(h0, h1, h2);
                const V3 sn = do_refr ? neg(h.n) : h.n;
                const V3 a = u + sn;
                const V3 nb = a * rcp_nonneg(sqrt_(dot(a, a)));   // |a| <= 2
                const float vdn = dot(dir, h.n);
                // reflect (:861-862): dir - 2 dot(dir, n) n as fma
                const float d2 = 2.0f * vdn;
                const V3 sd = v3(fma_(-d2, h.n.x, dir.x), fma_(-d2, h.n.y, dir.y), fma_(-d2, h.n.z, dir.z));
                // refract (rfrct, mathlib.h:781-789); k of the lanes that do not refract is
                // replaced by 1 so that no lane takes sqrt's slow path for a discarded value
                const float ior = h.inside ? M.ior : s_mx[h.mat].rior;
                const float k = fma_(-ior, ior * fma_(-vdn, vdn, 1.0f), 1.0f);
                const float sk = fma_(ior, vdn, sqrt_(do_refr ? k : 1.0f));
                V3 rd = v3(fma_(ior, dir.x, -(sk * h.n.x)), fma_(ior, dir.y, -(sk * h.n.y)),
                           fma_(ior, dir.z, -(sk * h.n.z)));
                rd = k < 0.0f ? v3(0.0f, 0.0f, 0.0f) : rd;
                const V3 R = do_refr ? rd : sd;
                const float rough = do_refr ? M.refr_rough : M.spec_rough;
                const float rsq = rough * rough;
                const V3 lr = v3(fma_(rsq, nb.x - R.x, R.x), fma_(rsq, nb.y - R.y, R.y), fma_(rsq, nb.z - R.z, R.z));
                ndir = (do_spec || do_refr) ? lr : nb;
            } else if (!do_refr) {
                uint32_t r = s_diff;
                V3 diffuse;
                if (rejection) {
                    const V3 a = h.n + ruv_rejection(r);
                    diffuse = a * rcp(sqrt_(dot(a, a)));   // fast_approx_normalize, rsroot -> 1/sqrtf
                } else {
                    diffuse = normalize(h.n + ruv_angle(r));
                }
                ndir = diffuse;
                if (do_spec) {
                    const float d2 = 2.0f * dot(dir, h.n);
                    const V3 sd = v3(fma_(-d2, h.n.x, dir.x), fma_(-d2, h.n.y, dir.y), fma_(-d2, h.n.z, dir.z));
                    const float srsq = M.spec_rough * M.spec_rough;
                    ndir = v3(fma_(srsq, diffuse.x - sd.x, sd.x), fma_(srsq, diffuse.y - sd.y, sd.y),
                              fma_(srsq, diffuse.z - sd.z, sd.z));
                }
            } else {
                uint32_t r = s_refr;
                const float ior = h.inside ? M.ior : s_mx[h.mat].rior;
                const float rrsq = M.refr_rough * M.refr_rough;
                V3 rd = refract(dir, h.n, ior);
                if (rejection) {
                    const V3 a = ruv_rejection(r) - h.n;
                    const V3 nrd = a * rcp(sqrt_(dot(a, a)));
                    rd = v3(fma_(rrsq, nrd.x - rd.x, rd.x), fma_(rrsq, nrd.y - rd.y, rd.y),
                            fma_(rrsq, nrd.z - rd.z, rd.z));
                } else {
                    const V3 nrd = normalize(ruv_angle(r) - h.n);
                    rd = normalize(rd + (nrd - rd) * rrsq);
                }
                ndir = rd;
            }
            ndir = normalize_small(ndir);   // a unit vector or a lerp of two
            ret = v3(fma_(em.x, T.x, ret.x), fma_(em.y, T.y, ret.y), fma_(em.z, T.z, ret.z));
            const V3 cf = do_spec ? ld3(M.spec_color) : ld3(M.albedo);
            if (!do_refr) T = mul(T, cf);
            T = T * rcp(prob);   // (prob >= 0.001; materials may set any chance)
            {   // :891-899 (boost only; the path continues either way)
                const float pm = max_ps(T.x, max_ps(T.y, T.z));
                const bool term = randf(rng) > pm;
                if (!term) T = T * rcp(pm);
            }
            pos = npos;
            dir = ndir;
            ++bounce;
        }
    }
}

#ifdef PT_V4_WAVES   // A/B builds: force the occupancy (waves per SIMD)
#define PT_V4_OCC __attribute__((amdgpu_waves_per_eu(PT_V4_WAVES, PT_V4_WAVES)))
#define PT_V4_CT_OCC PT_V4_OCC
#else
// render instances: at least 5 waves per SIMD (<= 96 VGPRs; the exact-exp instance needs 97
// otherwise and compiles spill-free at 96); the diagnostic COUNT instances are left unconstrained
#define PT_V4_OCC __attribute__((amdgpu_waves_per_eu(COUNT ? 1 : 5)))
// the continuous-tiles kernel at 6 waves per SIMD (80 VGPRs -- its pool loop needs no more, the one
// spilled register is in the event code; 16 KiB of LDS per block: 6 blocks per CU).  Against 5
// waves (interleaved A/B, profiles/r05/r05g_v4_ab.jsonl): 1080p 8 spp 0.3591 vs 0.3652 ms, 1080p
// 32 spp 1.247 vs 1.261, 4K 8 spp 1.272 vs 1.296 -- and ahead of the per-tile kernel (0.3602,
// 1.260, 1.298) at all three.  The instance with the reference's default flags (DFL) only: the
// others spill in their pool loops at 80 VGPRs and keep 5 waves.
#define PT_V4_CT_OCC __attribute__((amdgpu_waves_per_eu(COUNT ? 1 : (DFL ? 6 : 5))))
#endif
// FEXP: USE_FAST_APPROXIMATE_EXP as a compile-time switch (1 fast, 0 exact) for the render
// instances -- the exact expf's registers in the Beer branch would otherwise raise the kernel from
// 93 to 97 VGPRs, i.e. from 5 to 4 waves per SIMD (0.410 -> 0.451 ms at 1080p equirect) -- and as
// the runtime flag (2) for the diagnostic COUNT instances.
// DFL: the reference's default sampling flags (USE_RANDOM_JITTER_TEXTURE_SAMPLING 1,
// USE_UNIT_VECTOR_REJECTION_SAMPLING 1) compiled in -- the default scene's render instance only
// (0.3950 -> 0.3924 ms at 1080p equirect, profiles/r03r_ab_v4_flags.txt).
// PRESENT: the fused OutputToScreen (v4 :1562-1564 calls it right after RenderTile, per tile): each
// pixel's 8-bit value (pt_tonemap.h, the default fast ACES / gamma) is written with its final
// accumulator value at job.pix_out[Y * width + X] -- the presenting instances (pt_launch_v4: the
// drop-in's one-frame calls in the tiled layout, default scene and flags), so the plain kernels'
// register allocation is untouched.
template <bool PRESENT>
__device__ __forceinline__ void v4_present(const PtV4Job& job, int X, int Y, V3 acc)
{
    if constexpr (PRESENT)
        job.pix_out[(size_t)(uint32_t)Y * (uint32_t)job.width + (uint32_t)X] =
            pt_tone::pack<true, true>(acc.x, acc.y, acc.z, job.pix_xrgb != 0);
}

template <int ENV, int LAYOUT, bool COUNT, bool DEF, int FEXP, bool DFL = false, bool PRESENT = false>
__global__ __launch_bounds__(64 * kWaves) PT_V4_OCC void pt_v4_kernel(PtV4Job job, PtV4Scene sc)
{
    __shared__ float s_col[kWaves][kChunk * 64 * 3];
    __shared__ PtV4Mat s_mat[PT_V4_MAX_OBJECTS];
    __shared__ float4 s_sc[DEF ? pt_v4_default::kSpheres : 1];   // default scene: sphere centre, radius
    __shared__ MatX s_mx[PT_V4_MAX_OBJECTS];                        // per-material constants (mat_consts)
    constexpr bool DEFER = ENV != PT_V4_ENV_NONE_;
    __shared__ float4 s_qd[DEFER ? kWaves : 1][DEFER ? kEnvQ : 1];   // env dir, rng
    __shared__ float4 s_qt[DEFER ? kWaves : 1][DEFER ? kEnvQ : 1];   // throughput, colour slot
    for (int t = threadIdx.x; t < PT_V4_MAX_OBJECTS * 17; t += 64 * kWaves)
        reinterpret_cast<float*>(s_mat)[t] = reinterpret_cast<const float*>(sc.mat)[t];
    __syncthreads();
    if (threadIdx.x < PT_V4_MAX_OBJECTS) s_mx[threadIdx.x] = mat_consts(s_mat[threadIdx.x]);
    if (DEF && threadIdx.x < pt_v4_default::kSpheres) {
        const float* c = pt_v4_default::kSphere[threadIdx.x];
        s_sc[threadIdx.x] = make_float4(c[0], c[1], c[2], c[3]);
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    pt_queue_zero_next(job.queue_next);   // (pt_tile_queue.h)
    const int tiles_x = (job.ncols + 7) >> 3;
    const int ntiles = tiles_x * ((job.nrows + 7) >> 3);
    float* const col = s_col[wv];
    const size_t cs = (LAYOUT == PT_LAYOUT_INTERLEAVED) ? 1u : 8u;
    const Tex tex{job.env, job.env_w, job.env_h};
    const bool random = DFL || job.random_jitter != 0, rejection = DFL || job.rejection != 0;
    const int B = job.num_bounces;
    const float W = (float)job.width, H = (float)job.height;
    const float rW = rcp(W), rH = rcp(H);
    const float cam_dist = 1.0f;   // 1 / tanf(c_FOVDegrees * 0.5f * c_pi / 180.0f) == 1.0f exactly (InitializeCamera :1500)
    unsigned long long n_seg = 0, n_esc = 0, n_slots = 0, n_fb = 0, n_sky = 0;

    // persistent waves: 8x8 tiles from the launch's queue (pt_tile_queue.h), longest first when the
    // geometry has a schedule
    constexpr uint32_t kNone = PtTileQueue<kWaves>::kNone;
    PtTileQueue<kWaves> tq(job.queue, job.order, job.units, job.nunits, (uint32_t)ntiles, wv);
    uint32_t tile = kNone, next_tile = kNone;
    tile = tq.first(job.err);   // (the whole wave: uniform, scalar registers)
    tile = __builtin_amdgcn_readfirstlane(tile);
    while (tile != kNone) {
    // (this kernel's schedules hold whole tiles: pt_capi.cpp v4_launch)
    const int tcol = ((int)pt_entry_tile(tile) % tiles_x) * 8, trow = ((int)pt_entry_tile(tile) / tiles_x) * 8;
    uint32_t tile_work = 1;   // pool iterations of this tile (the schedule's cost)

    // this lane's pixel (phase C) and its accumulator
    const int px = job.col0 + tcol + (lane & 7), pr = trow + (lane >> 3);
    const bool pvalid = (tcol + (lane & 7)) < job.ncols && pr < job.nrows;
    float* acc_p = nullptr;
    V3 acc = v3(0.0f, 0.0f, 0.0f);
    if (pvalid) {
        // compact layouts index the buffer row; the tiled layout indexes the full image (global row)
        const int orow = LAYOUT == PT_LAYOUT_TILED_PLANAR8 ? job.row_start + pr * job.row_stride : pr;
        acc_p = job.buf + out_index<LAYOUT>(job, px, orow);
        if (job.accumulate) acc = v3(acc_p[0], acc_p[cs], acc_p[2 * cs]);   // (:1233: only to blend)
    }

    for (int c0 = 0; c0 < job.nframes; c0 += kChunk) {
        const int nf = std::min(kChunk, job.nframes - c0);
        const int total = 64 * nf;
        int next = 0;      // wave-uniform
        int item = -1;     // this lane's (pixel, frame) sample, -1 = none
        V3 pos, dir, T, ret;
        uint32_t rng = 0;
        int bounce = 0;
        int qn = 0;   // queued misses (DEFER), wave-uniform
        // a deferred miss: env(d) with the rng state r, fma'd with throughput t into colour slot k
        auto resolve = [&](V3 d, uint32_t r, V3 t, int k) {
            V3 amb = v3(0.0f, 0.0f, 0.0f);
            if (ENV == PT_V4_ENV_EQUIRECT_) amb = equirect(tex, d, random, r);
            if (ENV == PT_V4_ENV_CUBEMAP_) amb = cubemap(tex, d, random, r);
            float* o = col + k;
            const V3 rt = v3(fma_(amb.x, t.x, o[0]), fma_(amb.y, t.y, o[1]), fma_(amb.z, t.z, o[2]));   // :787
            o[0] = fma_(rt.x, 1.0f, 0.0f);   // :1127
            o[1] = fma_(rt.y, 1.0f, 0.0f);
            o[2] = fma_(rt.z, 1.0f, 0.0f);
        };
        // evaluate the queued misses [0, m), one per lane
        auto drain = [&](int m) {
            if (lane < m) {
                const float4 a = s_qd[DEFER ? wv : 0][lane], b = s_qt[DEFER ? wv : 0][lane];
                resolve(v3(a.x, a.y, a.z), __builtin_bit_cast(uint32_t, a.w), v3(b.x, b.y, b.z),
                        __builtin_bit_cast(int, b.w));
            }
        };
        for (;;) {
            // hand out items to idle lanes, in lane order
            const bool need = item < 0;
            const unsigned long long m = pt_ballot(need);
            if (need) {
                const int it = next + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (it < total) {
                    // frame-major (pixel-major, a pixel's frames on neighbouring lanes, measured
                    // 1-2.5 % slower here: the jittered camera rays share no bounce-0 origin)
                    const int p = it & 63, f = it >> 6;
                    const int X = job.col0 + tcol + (p & 7), rb = trow + (p >> 3);
                    if ((tcol + (p & 7)) < job.ncols && rb < job.nrows) {
                        item = f * 64 + p;   // colour slot order (phase C)
                        // mainImage :1092-1130
                        const int Y = job.row_start + rb * job.row_stride;
                        const uint32_t frame = job.frame_first + (uint32_t)(c0 + f);
                        const int fyi = job.height - 1 - Y;
                        // 24 x 24-bit products: X, fyi, frame < 2^24 (C ABI), low words = the u32 products
                        rng = 1u | (__umul24((uint32_t)X, 1973u) + __umul24((uint32_t)fyi, 9277u) + __umul24(frame, 26699u));
                        const float jx = randf(rng) - 0.5f;
                        const float jy = randf(rng) - 0.5f;
                        const float tx = fma_(((float)X + jx) * rW, 2.0f, -1.0f);
                        float ty = fma_(((float)fyi + jy) * rH, 2.0f, -1.0f);
                        ty = ty * (rW * H);
                        // |(tx, ty, -1)| >= 1 and tx, ty are O(1): no range guards
                        const V3 cv = v3(tx, ty, -cam_dist) - v3(0.0f, 0.0f, 0.0f);
                        dir = cv * pt::rcp_rn(pt::sqrt_rn(dot(cv, cv)));
                        pos = v3(0.0f, 0.0f, 1.0f * 40.0f);   // camera.Position :1501
                        T = v3(1.0f, 1.0f, 1.0f);
                        ret = v3(0.0f, 0.0f, 0.0f);
                        bounce = 0;
                    }
                }
            }
            next += __builtin_popcountll(m);
            if (pt_ballot(item >= 0) == 0ull) break;
            ++tile_work;
            if (COUNT) n_slots += 64;
            bool queued = false;   // DEFER: this lane's item missed and goes to the queue
            int qslot = 0;
            // default scene: when every busy lane traces a camera ray that leaves the scene's
            // silhouette (sky_ray_v4), the wave skips TestSceneTrace -- the reference's miss
            // (the slope test runs only in iterations where every busy lane is at bounce 0: a wave-
            // uniform branch, instead of the test on every lane in every iteration)
            bool all_sky = false;
            if (DEF && pt_ballot(item >= 0 && bounce != 0) == 0)
                all_sky = pt_ballot(item >= 0 && !sky_ray_v4(dir)) == 0;
            if (item >= 0) {
                bool done = false;
                v4_segment<ENV, COUNT, DEF, FEXP, DFL>(job, sc, s_mat, s_mx, s_sc, tex, random, rejection, B, all_sky, pos,
                                                       dir, T, ret, rng, bounce, done, queued, n_seg, n_esc, n_fb, n_sky);
                if (done) {
                    const int p = item & 63, f = item >> 6;
                    qslot = (f * 64 + p) * 3;
                    float* o = col + qslot;
                    if (DEFER && queued) {   // ret so far; the drain adds the env term
                        o[0] = ret.x;
                        o[1] = ret.y;
                        o[2] = ret.z;
                    } else {
                        // mainImage :1127: fmadd(color, 1/c_numRendersPerFrame, 0)
                        o[0] = fma_(ret.x, 1.0f, 0.0f);
                        o[1] = fma_(ret.y, 1.0f, 0.0f);
                        o[2] = fma_(ret.z, 1.0f, 0.0f);
                    }
                    item = -1;
                }
            }
            if (DEFER) {
                const unsigned long long qm = pt_ballot(queued);
                const int nq = __builtin_popcountll(qm);
                const V3 ed = ENV == PT_V4_ENV_EQUIRECT_ ? v3(-dir.x, dir.y, -dir.z) : dir;
                if (qn + nq > kEnvQ) {
                    // overflow: one env pass over the whole wave -- the new misses in their own lanes,
                    // the other lanes each take one queued miss (the top `take` entries, so the rest
                    // stay in place).  At least kEnvQ + 1 lanes busy (min(qn + nq, 64)); the drain-or-
                    // new-batch choice this replaces ran 24-48 of the 64.
                    const int take = std::min(qn, 64 - nq);
                    const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(~qm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)~qm, 0u));
                    V3 d = ed, t = T;
                    uint32_t rr = rng;
                    int k = qslot;
                    bool act = queued;
                    if (!queued && r < take) {
                        const int e = qn - take + r;
                        const float4 a = s_qd[DEFER ? wv : 0][DEFER ? e : 0], b = s_qt[DEFER ? wv : 0][DEFER ? e : 0];
                        d = v3(a.x, a.y, a.z);
                        rr = __builtin_bit_cast(uint32_t, a.w);
                        t = v3(b.x, b.y, b.z);
                        k = __builtin_bit_cast(int, b.w);
                        act = true;
                    }
                    if (act) resolve(d, rr, t, k);
                    qn -= take;
                } else {
                    if (queued) {
                    const int k = qn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
                        s_qd[DEFER ? wv : 0][k] = make_float4(ed.x, ed.y, ed.z, __builtin_bit_cast(float, rng));
                        s_qt[DEFER ? wv : 0][k] = make_float4(T.x, T.y, T.z, __builtin_bit_cast(float, qslot));
                    }
                    qn += nq;
                }
            }
        }
        if (DEFER && qn > 0) drain(qn);
        if (c0 + kChunk >= job.nframes) next_tile = tq.next(job.err);   // the last pool is done
        // all radiance of this chunk is in LDS (written by lanes of this wave)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (pvalid) {
            for (int f = 0; f < nf; ++f) {
                const float* c = col + (f * 64 + lane) * 3;
                if (job.accumulate) {   // ACCUMULATE_FRAMES 1: fmadd(blend_factor, color - last, last) :1233-1241
                    const float bf = rcp((float)(job.frame_first + (uint32_t)(c0 + f)) + 1.0f);   // :1200
                    acc = v3(fma_(bf, c[0] - acc.x, acc.x), fma_(bf, c[1] - acc.y, acc.y), fma_(bf, c[2] - acc.z, acc.z));
                } else {                // ACCUMULATE_FRAMES 0: the frame's colour is stored (:1245-1250)
                    acc = v3(c[0], c[1], c[2]);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (job.nframes <= 0) next_tile = tq.next(job.err);   // no chunk ran
    if (pvalid) {
        acc_p[0] = acc.x;
        acc_p[cs] = acc.y;
        acc_p[2 * cs] = acc.z;
        v4_present<PRESENT>(job, px, job.row_start + pr * job.row_stride, acc);
    }
    if (job.cost && lane == 0) pt_record_cost(job.cost, tile, (uint32_t)ntiles, tile_work);
    tile = __builtin_amdgcn_readfirstlane(next_tile);
    }
    tq.report(job.err);   // (a schedule entry outside the launch, pt_tile_queue.h)
    if (COUNT) {
        // per-lane counts summed over the wave by lane 0's atomics
        for (int off = 32; off > 0; off >>= 1) {
            n_seg += __shfl_down(n_seg, off);
            n_esc += __shfl_down(n_esc, off);
            n_fb += __shfl_down(n_fb, off);
            n_sky += __shfl_down(n_sky, off);
        }
        if (lane == 0) {
            atomicAdd(&job.counters[0], n_seg);
            atomicAdd(&job.counters[2], n_esc);
            atomicAdd(&job.counters[3], n_slots);
            atomicAdd(&job.counters[4], n_fb);
            atomicAdd(&job.counters[5], n_sky);
        }
    }
}

// ---- continuous tiles (CT): the v4 pool without per-tile tails ----------------------------------
// pt_v4_kernel's pool drains at the end of every tile chunk (lane efficiency 0.898 at 1080p: the
// last paths of a chunk run while the other lanes idle).  Here, as in pt_kernel.hip's
// render_body_ct, a wave's items form one stream over its tiles' chunks: two chunk contexts, A
// (handing out items) and D (all handed out, in flight), the per-(pixel, frame) radiance in the
// global slot area (ct_slots, 12 KiB per wave), D folded -- the progressive lerp of its frames in
// frame order, :1233-1250 -- when its last item ends, the next chunk started as soon as A's last
// item is handed out and D is folded.  v4 items need no records: each generates its own jittered
// camera ray from (pixel, frame); a tile's valid pixels are listed in LDS (compacted, with their
// seed terms).  The deferred env misses keep the wave-wide drains of pt_v4_kernel; a queue entry
// also carries the radiance so far (48 B), and D's fold drains the whole queue first.  The same
// operations on the same operands: bit-identical to pt_v4_kernel (the -m gpu v4 parity tests).
constexpr uint32_t kV4CtWaveFloats = 2u * 64u * (uint32_t)kChunk * 3u;
static_assert(kV4CtWaveFloats == 2u * 64u * 8u * 3u, "the slot area is the diffuse pool's (pt_ct_wave_floats)");
enum : int {   // per-wave LDS words of the events (pt_kernel.hip kWs*)
    kVwTcur, kVwNh, kVwF0next, kVwF0A, kVwTD, kVwF0D, kVwNfD, kVwHmD, kVwHmD1, kVwHm, kVwHm1, kVwTileSeg,
    kVwSegA, kVwSegD, kVwFlags, kVwSky, kVwSkyD, kVwWords
};

template <int ENV, int LAYOUT, bool COUNT, bool DEF, int FEXP, bool DFL = false>
__global__ __launch_bounds__(64 * kWaves) PT_V4_CT_OCC void pt_v4_ct_kernel(PtV4Job job, PtV4Scene sc)
{
    __shared__ PtV4Mat s_mat[PT_V4_MAX_OBJECTS];
    __shared__ float4 s_sc[DEF ? pt_v4_default::kSpheres : 1];   // default scene: sphere centre, radius
    __shared__ MatX s_mx[PT_V4_MAX_OBJECTS];                        // per-material constants (mat_consts)
    constexpr bool DEFER = ENV != PT_V4_ENV_NONE_;
    __shared__ float4 s_qd[DEFER ? kWaves : 1][DEFER ? kEnvQ : 1];   // env dir, rng
    __shared__ float4 s_qt[DEFER ? kWaves : 1][DEFER ? kEnvQ : 1];   // throughput, slot
    __shared__ float4 s_qr[DEFER ? kWaves : 1][DEFER ? kEnvQ : 1];   // radiance so far
    __shared__ float s_acc[kWaves][3][64];    // the pixels' accumulators between a tile's chunks
    __shared__ uint32_t s_pl[kWaves][64];     // the current tile's valid pixels: lane | X << 8
    __shared__ uint32_t s_py[kWaves][64];     // and their y term (height - 1 - Y) of the seed
    __shared__ uint32_t s_ws[kWaves][kVwWords];
    __shared__ uint32_t s_tq[kWaves][PtTileQueue<kWaves>::kWords];
    for (int t = threadIdx.x; t < PT_V4_MAX_OBJECTS * 17; t += 64 * kWaves)
        reinterpret_cast<float*>(s_mat)[t] = reinterpret_cast<const float*>(sc.mat)[t];
    __syncthreads();
    if (threadIdx.x < PT_V4_MAX_OBJECTS) s_mx[threadIdx.x] = mat_consts(s_mat[threadIdx.x]);
    if (DEF && threadIdx.x < pt_v4_default::kSpheres) {
        const float* c = pt_v4_default::kSphere[threadIdx.x];
        s_sc[threadIdx.x] = make_float4(c[0], c[1], c[2], c[3]);
    }
    __syncthreads();

    pt_chain_started(job.started);   // (chained launches, pt_chain.h)
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    pt_queue_zero_next(job.queue_next);   // (pt_tile_queue.h)
    const int tiles_x = (job.ncols + 7) >> 3;
    const uint32_t ntiles = (uint32_t)tiles_x * (uint32_t)((job.nrows + 7) >> 3);
    const int S = job.nframes;
    float* const slots = job.ct_slots + (size_t)(blockIdx.x * kWaves + wv) * kV4CtWaveFloats;
    // (the host launches at most ct_waves waves: pt_launch_v4)
    if (!PT_GUARD(job.err, blockIdx.x * (uint32_t)kWaves + (uint32_t)wv < job.ct_waves, PT_G_SLOT_BASE,
                  blockIdx.x * (uint32_t)kWaves + (uint32_t)wv))
        return;
    const size_t px_extent = pixel_extent<LAYOUT>(job);   // (guards; the accumulator's buffer resource)
    const uint32_t pxb = pt_px_nbytes(px_extent);          // (pt_chain.h pt_px_ld3 / pt_px_st3)
    const size_t cs = (LAYOUT == PT_LAYOUT_INTERLEAVED) ? 1u : 8u;
    const Tex tex{job.env, job.env_w, job.env_h};
    const bool random = DFL || job.random_jitter != 0, rejection = DFL || job.rejection != 0;
    const int B = job.num_bounces;
    const float W = (float)job.width, H = (float)job.height;
    const float rW = rcp(W), rH = rcp(H);
    const float cam_dist = 1.0f;   // (as pt_v4_kernel, InitializeCamera :1500)
    unsigned long long n_seg = 0, n_esc = 0, n_slots = 0, n_fb = 0, n_sky = 0;

    constexpr uint32_t kNone = PtTileQueue<kWaves>::kNone;
    {
        PtTileQueue<kWaves> q(job.queue, job.order, job.units, job.nunits, ntiles, wv);
        q.back = job.ct_back_pct != 0 &&
                 (uint64_t)blockIdx.x * 100u >= (uint64_t)gridDim.x * (100u - (job.ct_back_pct < 100u ? job.ct_back_pct : 100u));
        q.save(s_tq[wv], lane);
    }
    // the events' wave-uniform state in LDS (as render_body_ct: the pool loop's SGPRs stay free)
    uint32_t* const ws = s_ws[wv];
    auto ws_ld = [&](int k) -> uint32_t { return __builtin_amdgcn_readfirstlane(ws[k]); };
    auto ws_st = [&](int k, uint32_t v) {
        if (lane == 0) ws[k] = v;
    };
    if (lane == 0) {
        ws[kVwTcur] = kNone;
        ws[kVwFlags] = 0u;
        ws[kVwTileSeg] = 0u;
    }
    // pool state (scalar registers): A's slot context, frames, items handed out / all (nitA 0: no A),
    // its pixels and the item -> (frame, pixel) divisor, its first frame; D
    int cA = 0, nfA = 0, issA = 0, nitA = 0, nhA = 1;
    uint32_t div_nh = 0;   // frame-major items: fi = k / nhA as umulhi(k, ceil(2^32 / nhA)) (nhA >= 2)
    uint32_t fA = 0;
    bool hasD = false;
    uint64_t dmask = 0;    // lanes holding D's items
    const bool rec_cost = job.cost != nullptr;
    // per lane: the item (slot < 0: none)
    V3 pos = v3(0.0f, 0.0f, 0.0f), dir = pos, T = pos, ret = pos;
    uint32_t rng = 0;
    int bounce = 0;
    int slot = -1;         // float index of the item's radiance slot in `slots`
    int qn = 0;            // queued misses (DEFER), wave-uniform

    // a deferred miss: env(d) with the rng state r, fma'd with throughput t onto the radiance so far,
    // into slot k (pt_v4_kernel's resolve, its slot read replaced by the entry's radiance)
    // (always_inline: without it the non-default-flag equirect instances called it out of line)
    auto resolve = [&](V3 d, uint32_t r, V3 t, V3 rs, int k) __attribute__((always_inline)) {
        V3 amb = v3(0.0f, 0.0f, 0.0f);
        if (ENV == PT_V4_ENV_EQUIRECT_) amb = equirect(tex, d, random, r);
        if (ENV == PT_V4_ENV_CUBEMAP_) amb = cubemap(tex, d, random, r);
        const V3 rt = v3(fma_(amb.x, t.x, rs.x), fma_(amb.y, t.y, rs.y), fma_(amb.z, t.z, rs.z));   // :787
        if (!PT_GUARD(job.err, k >= 0 && (uint32_t)k + 3u <= kV4CtWaveFloats, PT_G_ITEM_SLOT, k)) return;
        float* const o = slots + k;
        o[0] = fma_(rt.x, 1.0f, 0.0f);   // :1127
        o[1] = fma_(rt.y, 1.0f, 0.0f);
        o[2] = fma_(rt.z, 1.0f, 0.0f);
    };
    auto drain = [&](int m) {   // the queued misses [0, m), one per lane
        if (DEFER && lane < m) {
            const float4 a = s_qd[DEFER ? wv : 0][lane], b = s_qt[DEFER ? wv : 0][lane], c = s_qr[DEFER ? wv : 0][lane];
            resolve(v3(a.x, a.y, a.z), __builtin_bit_cast(uint32_t, a.w), v3(b.x, b.y, b.z), v3(c.x, c.y, c.z),
                    __builtin_bit_cast(int, b.w));
        }
    };

    // an item's camera ray: mainImage :1092-1130 (as pt_v4_kernel) for pixel column X, flipped row
    // fyi (height - 1 - Y) and frame
    const auto camera = [&](int X, int fyi, uint32_t frame, uint32_t& r, V3& d) {
        // 24 x 24-bit products: X, fyi, frame < 2^24 (C ABI), low words = the u32 products
        r = 1u | (__umul24((uint32_t)X, 1973u) + __umul24((uint32_t)fyi, 9277u) + __umul24(frame, 26699u));
        const float jx = randf(r) - 0.5f;
        const float jy = randf(r) - 0.5f;
        const float tx = fma_(((float)X + jx) * rW, 2.0f, -1.0f);
        float ty = fma_(((float)fyi + jy) * rH, 2.0f, -1.0f);
        ty = ty * (rW * H);
        const V3 cv = v3(tx, ty, -cam_dist) - v3(0.0f, 0.0f, 0.0f);
        d = cv * pt::rcp_rn(pt::sqrt_rn(dot(cv, cv)));
    };
    // Start chunks until A is set or the queue is done: the current tile's next chunk, or a new tile
    // (its valid pixels listed; a new tile starts only when the previous tile's last chunk has handed
    // out every item, so its list is free)
    auto start_chunk = [&]() {
        while (nitA == 0) {
            const int f0next = (int)ws_ld(kVwF0next);
            if (ws_ld(kVwTcur) != kNone && f0next < S) {
                nfA = S - f0next < kChunk ? S - f0next : kChunk;
                fA = job.frame_first + (uint32_t)f0next;
                ws_st(kVwF0A, (uint32_t)f0next);
                ws_st(kVwF0next, (uint32_t)(f0next + nfA));
                nhA = (int)ws_ld(kVwNh);
                div_nh = nhA > 1 ? (uint32_t)((0x100000000ull + (uint64_t)nhA - 1u) / (uint64_t)nhA) : 0u;
                issA = 0;
                nitA = nhA * nfA;   // >= 1
                if (rec_cost) ws_st(kVwSegA, 0u);
                break;
            }
            ws_st(kVwTcur, kNone);
            const uint32_t flags = ws_ld(kVwFlags);
            if (flags & 2u) break;   // the queue is done
            PtTileQueue<kWaves> tq = PtTileQueue<kWaves>::restore(s_tq[wv]);
            uint32_t tile = (flags & 1u) ? tq.next(job.err) : tq.first(job.err);
            tile = __builtin_amdgcn_readfirstlane(tile);
            tq.save(s_tq[wv], lane);
            ws_st(kVwFlags, tile == kNone ? 3u : 1u);
            if (tile == kNone) break;
            if (job.chain_wait != 0u) pt_chain_wait(job.tile_epoch, tile, job.chain_wait, job.err, lane);   // (pt_chain.h)
            // (a queue entry is a tile or one half of it, pt_tile_queue.h)
            const int tcol = ((int)pt_entry_tile(tile) % tiles_x) * 8, trow = ((int)pt_entry_tile(tile) / tiles_x) * 8;
            const bool valid = (tcol + (lane & 7)) < job.ncols && trow + (lane >> 3) < job.nrows &&
                               pt_part_has_lane(pt_entry_part(tile), lane);
            const uint64_t hm = pt_ballot(valid);
            const int X = job.col0 + tcol + (lane & 7), pr = trow + (lane >> 3);
            const int fyi = job.height - 1 - (job.row_start + pr * job.row_stride);
            if (valid) {
                const int k = __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
                s_pl[wv][k] = (uint32_t)lane | ((uint32_t)X << 8);   // X < 2^24 (C ABI)
                s_py[wv][k] = (uint32_t)fyi;
            }
            // DEF: the tile's leading frames whose camera rays ALL leave the scene's silhouette
            // (sky_ray_v4, exact per ray) are rendered here, by the whole wave: pt_v4_kernel skips
            // their trace when every busy lane holds such a ray, which the pool's mix of tiles
            // rarely allows -- half of the 1080p tiles are sky.  Each is the pool's miss at bounce 0
            // (T = 1, ret = 0: v4_segment, resolve) and the fold's lerp, with the same operations.
            int fsky = 0;
            if (DEF) {
                const int orow = LAYOUT == PT_LAYOUT_TILED_PLANAR8 ? job.row_start + pr * job.row_stride : pr;
                size_t pi = valid ? out_index<LAYOUT>(job, X, orow) : 0;
                if (valid && !PT_GUARD(job.err, pi + 2 * cs < px_extent, PT_G_PIXEL, pi)) pi = 0;   // (checked build: reported)
                V3 acc = v3(0.0f, 0.0f, 0.0f);
                if (valid && job.accumulate) pt_px_ld3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);
                for (; fsky < S; ++fsky) {
                    uint32_t r;
                    V3 d;
                    camera(X, fyi, job.frame_first + (uint32_t)fsky, r, d);
                    if (pt_ballot(valid && !sky_ray_v4(d)) != 0) break;
                    if (COUNT) n_slots += 64;
                    if (valid) {
                        V3 amb = v3(0.11f, 0.1f, 0.15f);   // :782
                        if (ENV == PT_V4_ENV_EQUIRECT_) amb = equirect(tex, v3(-d.x, d.y, -d.z), random, r);
                        if (ENV == PT_V4_ENV_CUBEMAP_) amb = cubemap(tex, d, random, r);
                        const V3 rt = v3(fma_(amb.x, 1.0f, 0.0f), fma_(amb.y, 1.0f, 0.0f), fma_(amb.z, 1.0f, 0.0f));   // :787
                        const V3 c = v3(fma_(rt.x, 1.0f, 0.0f), fma_(rt.y, 1.0f, 0.0f), fma_(rt.z, 1.0f, 0.0f));     // :1127
                        if (job.accumulate) {   // :1233-1241
                            const float bf = rcp((float)(job.frame_first + (uint32_t)fsky) + 1.0f);   // :1200
                            acc = v3(fma_(bf, c.x - acc.x, acc.x), fma_(bf, c.y - acc.y, acc.y), fma_(bf, c.z - acc.z, acc.z));
                        } else {                // :1245-1250
                            acc = c;
                        }
                        if (COUNT) ++n_seg, ++n_sky, ++n_esc;
                    }
                }
                if (fsky > 0 && valid) pt_px_st3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);   // (the pool's first chunk reads it back)
                if (fsky == S) {   // the whole tile: ~one pool iteration per frame (the schedule's cost)
                    if (rec_cost && lane == 0) pt_record_cost(job.cost, tile, ntiles, 1u + (uint32_t)fsky);
                    if (job.tile_epoch) pt_chain_publish(job.tile_epoch, tile, job.chain_seq, job.chain_delay, lane);
                    continue;
                }
            }
            ws_st(kVwTcur, tile);
            ws_st(kVwHm, (uint32_t)hm);
            ws_st(kVwHm1, (uint32_t)(hm >> 32));
            ws_st(kVwNh, (uint32_t)__popcll(hm));   // >= 1 (a tile of the launch has a pixel)
            ws_st(kVwF0next, (uint32_t)fsky);
            ws_st(kVwSky, (uint32_t)fsky);
        }
    };
    // Fold D: its misses drained, every item of it ended; the radiance is in slot context 1 - cA
    auto fold_D = [&]() {
        if (DEFER && qn > 0) {
            drain(qn);
            qn = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // (the lanes' slot stores, then reads)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int c = cA ^ 1;
        const int f0D = (int)ws_ld(kVwF0D), nfD = (int)ws_ld(kVwNfD);
        const uint32_t tD = ws_ld(kVwTD);
        const uint64_t hmD = (uint64_t)ws_ld(kVwHmD) | ((uint64_t)ws_ld(kVwHmD1) << 32);
        // first: the tile's first pool chunk (after its sky frames, if any): the accumulator from buf
        const bool first = f0D == (int)ws_ld(kVwSkyD), last = f0D + nfD == S;
        if ((hmD >> lane) & 1u) {   // this lane's pixel of D's tile
            const int tcol = ((int)pt_entry_tile(tD) % tiles_x) * 8, trow = ((int)pt_entry_tile(tD) / tiles_x) * 8;
            const int px = job.col0 + tcol + (lane & 7), pr = trow + (lane >> 3);
            const int orow = LAYOUT == PT_LAYOUT_TILED_PLANAR8 ? job.row_start + pr * job.row_stride : pr;
            size_t pi = out_index<LAYOUT>(job, px, orow);
            if (!PT_GUARD(job.err, pi + 2 * cs < px_extent, PT_G_PIXEL, pi)) pi = 0;   // (checked build: reported)
            V3 acc = v3(0.0f, 0.0f, 0.0f);
            if (first) {
                if (job.accumulate) pt_px_ld3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);   // (:1233: only to blend)
            } else {
                acc = v3(s_acc[wv][0][lane], s_acc[wv][1][lane], s_acc[wv][2][lane]);
            }
            const float4* sp = (const float4*)(slots + (c * 64 + lane) * (kChunk * 3));   // 96 B, 16-B aligned
            float4 v[kChunk * 3 / 4];
#pragma unroll
            for (int i = 0; i < kChunk * 3 / 4; ++i)
                if (i * 4 < nfD * 3) v[i] = sp[i];
            const float* fr = (const float*)v;
#pragma unroll
            for (int f = 0; f < kChunk; ++f) {
                if (f < nfD) {
                    const V3 cc = v3(fr[3 * f], fr[3 * f + 1], fr[3 * f + 2]);
                    if (job.accumulate) {   // ACCUMULATE_FRAMES 1: fmadd(blend_factor, color - last, last) :1233-1241
                        const float bf = rcp((float)(job.frame_first + (uint32_t)(f0D + f)) + 1.0f);   // :1200
                        acc = v3(fma_(bf, cc.x - acc.x, acc.x), fma_(bf, cc.y - acc.y, acc.y), fma_(bf, cc.z - acc.z, acc.z));
                    } else {                // ACCUMULATE_FRAMES 0: the frame's colour is stored (:1245-1250)
                        acc = cc;
                    }
                }
            }
            if (last) {
                pt_px_st3(job.buf, pxb, cs, pi, acc.x, acc.y, acc.z);
            } else {
                s_acc[wv][0][lane] = acc.x;
                s_acc[wv][1][lane] = acc.y;
                s_acc[wv][2][lane] = acc.z;
            }
        }
        if (last && job.tile_epoch) pt_chain_publish(job.tile_epoch, tD, job.chain_seq, job.chain_delay, lane);
        if (rec_cost) {   // the schedule's cost: about the tile's pool iterations (its sky frames: one each)
            const uint32_t tile_seg = ws_ld(kVwTileSeg) + ws_ld(kVwSegD) + (first ? 64u * ws_ld(kVwSkyD) : 0u);
            ws_st(kVwTileSeg, last ? 0u : tile_seg);
            if (last && lane == 0) pt_record_cost(job.cost, tD, ntiles, 1u + (tile_seg + 63u) / 64u);
        }
        hasD = false;
    };

    start_chunk();
    uint32_t idle_events = 0;   // outer iterations in a row without progress (guard)
    bool fault = false;
    while (!fault) {
        bool event = false;
        if (hasD && dmask == 0) {   // D's last item ended: fold it
            fold_D();
            event = true;
        }
        if (nitA > 0 && issA >= nitA && !hasD) {   // A has handed out every item and D is folded
            ws_st(kVwTD, ws_ld(kVwTcur));
            ws_st(kVwHmD, ws_ld(kVwHm));
            ws_st(kVwHmD1, ws_ld(kVwHm1));
            ws_st(kVwF0D, ws_ld(kVwF0A));
            ws_st(kVwNfD, (uint32_t)nfA);
            ws_st(kVwSkyD, ws_ld(kVwSky));
            if (rec_cost) ws_st(kVwSegD, ws_ld(kVwSegA));
            hasD = true;
            dmask = pt_ballot(slot >= 0);   // every earlier chunk is folded: the items in flight are A's
            nitA = 0;
            issA = 0;
            cA ^= 1;
            start_chunk();
            event = true;
            if (dmask == 0) continue;   // (D's items had all ended: fold it first)
        }
        if (nitA == 0 && !hasD) break;   // every chunk of every tile of the queue is folded
        idle_events = event ? 0u : idle_events + 1u;
        if (__builtin_expect(idle_events > 2u, 0)) {   // (guard, never reached)
            fault = true;
            break;
        }
        while (true) {
            const bool had = slot >= 0;
            const uint64_t idle = pt_ballot(!had);
            bool took = false;
            int ntaken = 0;
            if (idle != 0 && issA < nitA) {
                const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const int k = issA + rank;
                const bool take = !had && k < nitA;
                took = take;
                if (take) {
                    // frame-major (pt_v4_kernel's order): item k is frame k / nhA of listed pixel k % nhA
                    const int fi = nhA == 1 ? k : (int)__umulhi((uint32_t)k, div_nh);
                    const int sl = k - (int)__umul24((uint32_t)fi, (uint32_t)nhA);
                    const uint32_t pl = s_pl[wv][sl];
                    const int p = (int)(pl & 63u), X = (int)(pl >> 8);
                    const int fyi = (int)s_py[wv][sl];
                    camera(X, fyi, fA + (uint32_t)fi, rng, dir);
                    pos = v3(0.0f, 0.0f, 1.0f * 40.0f);   // camera.Position :1501
                    T = v3(1.0f, 1.0f, 1.0f);
                    ret = v3(0.0f, 0.0f, 0.0f);
                    bounce = 0;
                    slot = (int)__umul24((uint32_t)(cA * 64 + p), (uint32_t)(kChunk * 3)) + fi * 3;
                }
                const int npop = __popcll(idle);
                ntaken = npop < nitA - issA ? npop : nitA - issA;
                issA += ntaken;
            }
            if (idle == ~0ull && ntaken == 0) break;   // no item in flight: an event is due
            idle_events = 0;
            if (COUNT) n_slots += 64;
            const bool busy = had || took;
            bool all_sky = false;   // (as pt_v4_kernel)
            if (DEF && pt_ballot(busy && bounce != 0) == 0) all_sky = pt_ballot(busy && !sky_ray_v4(dir)) == 0;
            bool done = false, queued = false;
            int qslot = 0;
            if (busy) {
                v4_segment<ENV, COUNT, DEF, FEXP, DFL>(job, sc, s_mat, s_mx, s_sc, tex, random, rejection, B, all_sky, pos,
                                                       dir, T, ret, rng, bounce, done, queued, n_seg, n_esc, n_fb, n_sky);
                if (done) {
                    qslot = slot;
                    if (!(DEFER && queued) &&
                        PT_GUARD(job.err, slot >= 0 && (uint32_t)slot + 3u <= kV4CtWaveFloats, PT_G_ITEM_SLOT, slot)) {
                        // mainImage :1127: fmadd(color, 1/c_numRendersPerFrame, 0)
                        float* const o = slots + slot;
                        o[0] = fma_(ret.x, 1.0f, 0.0f);
                        o[1] = fma_(ret.y, 1.0f, 0.0f);
                        o[2] = fma_(ret.z, 1.0f, 0.0f);
                    }
                    slot = -1;
                }
            }
            if (DEFER) {   // (pt_v4_kernel's queue, each entry with its radiance)
                const uint64_t qm = pt_ballot(queued);
                const int nq = __popcll(qm);
                const V3 ed = ENV == PT_V4_ENV_EQUIRECT_ ? v3(-dir.x, dir.y, -dir.z) : dir;
                if (qn + nq > kEnvQ) {
                    const int take = std::min(qn, 64 - nq);
                    const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(~qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)~qm, 0u));
                    V3 d = ed, t = T, rs = ret;
                    uint32_t rr = rng;
                    int k = qslot;
                    bool act = queued;
                    if (!queued && r < take) {
                        const int e = qn - take + r;
                        const float4 a = s_qd[DEFER ? wv : 0][DEFER ? e : 0], b = s_qt[DEFER ? wv : 0][DEFER ? e : 0];
                        const float4 c = s_qr[DEFER ? wv : 0][DEFER ? e : 0];
                        d = v3(a.x, a.y, a.z);
                        rr = __builtin_bit_cast(uint32_t, a.w);
                        t = v3(b.x, b.y, b.z);
                        k = __builtin_bit_cast(int, b.w);
                        rs = v3(c.x, c.y, c.z);
                        act = true;
                    }
                    if (act) resolve(d, rr, t, rs, k);
                    qn -= take;
                } else {
                    if (queued) {
                        const int k = qn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
                        s_qd[DEFER ? wv : 0][k] = make_float4(ed.x, ed.y, ed.z, __builtin_bit_cast(float, rng));
                        s_qt[DEFER ? wv : 0][k] = make_float4(T.x, T.y, T.z, __builtin_bit_cast(float, qslot));
                        s_qr[DEFER ? wv : 0][k] = make_float4(ret.x, ret.y, ret.z, 0.0f);
                    }
                    qn += nq;
                }
            }
            const uint64_t ended = pt_ballot(done);
            if (rec_cost) {   // segments traced per context (the schedule's cost)
                const int inD = __popcll(dmask), in_all = __popcll(pt_ballot(busy));
                if (lane == 0) {
                    ws[kVwSegA] += (uint32_t)(in_all - inD);
                    ws[kVwSegD] += (uint32_t)inD;
                }
            }
            dmask &= ~ended;
            if (hasD && dmask == 0) break;                    // fold due
            if (nitA > 0 && issA >= nitA && !hasD) break;     // retire due
        }
    }
    if (__builtin_expect(fault, 0) && DEFER && qn > 0) drain(qn);
    // a fault ends the wave with its chunks unfinished: recorded in the job's error words (the host
    // returns PT_EKERNEL), as the diffuse pool's
    if (__builtin_expect(fault, 0) && lane == 0 && job.err) {
        atomicAdd(&job.err[0], 1u);
        atomicMin(&job.err[1], pt_entry_tile(ws_ld(kVwTcur)));
    }
    PtTileQueue<kWaves>::restore(s_tq[wv]).report(job.err);   // (a schedule entry outside the launch)
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            n_seg += __shfl_down(n_seg, off);
            n_esc += __shfl_down(n_esc, off);
            n_fb += __shfl_down(n_fb, off);
            n_sky += __shfl_down(n_sky, off);
        }
        if (lane == 0) {
            atomicAdd(&job.counters[0], n_seg);
            atomicAdd(&job.counters[2], n_esc);
            atomicAdd(&job.counters[3], n_slots);
            atomicAdd(&job.counters[4], n_fb);
            atomicAdd(&job.counters[5], n_sky);
        }
    }
}

template <int ENV, int LAYOUT>
hipError_t launch_t(const PtV4Job& j, const PtV4Scene& sc, hipStream_t st, bool count, uint32_t* ct_blocks_out)
{
    const int tiles = ((j.ncols + 7) / 8) * ((j.nrows + 7) / 8);
    const dim3 block(64 * kWaves);
    // persistent grid: the resident blocks, at most one tile per wave.  The continuous-tiles kernel
    // when the caller provides its slots for the whole grid and the launch holds >= 4 full chunks
    // (8 frames x tile) per wave, else the per-tile pool kernel.  Measured (round 4, 5-wave CT vs
    // per-tile): 1080p 32 spp 1.257 vs 1.320 ms (51 chunks per wave), 4K 8 spp 1.308 vs 1.328 (25),
    // 1080p 8 spp 0.3602 vs 0.3589 (6), 1 spp 0.133 vs 0.115 (one item per pixel and chunk: the
    // chunk events, claim and fold, dominate); round 5, the 6-wave CT kernel: 1080p 8 spp (5.3 chunks
    // per wave) 0.3591 vs 0.3602.
    const auto go = [&](auto kern, auto ct_kern) {
        const long ct_blocks = std::min<long>(pt_resident_blocks(ct_kern, 64 * kWaves), (tiles + kWaves - 1) / kWaves);
        const uint64_t ct_waves = (uint64_t)ct_blocks * kWaves;
        if (j.ct_slots && ct_waves <= j.ct_waves && j.nframes >= kChunk &&
            (j.ct_force || (uint64_t)j.nframes * (uint64_t)tiles >= 4ull * kChunk * ct_waves)) {
            hipLaunchKernelGGL(ct_kern, dim3((unsigned)ct_blocks), block, 0, st, j, sc);
            if (ct_blocks_out) *ct_blocks_out = (uint32_t)ct_blocks;
            return;
        }
        const long blocks = std::min<long>(pt_resident_blocks(kern, 64 * kWaves), (tiles + kWaves - 1) / kWaves);
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), block, 0, st, j, sc);
    };
    if constexpr (LAYOUT == PT_LAYOUT_TILED_PLANAR8) {   // the presenting instances (pt_launch_v4: one frame)
        if (j.pix_out && !count) {
            auto k = pt_v4_kernel<ENV, LAYOUT, false, true, 1, true, true>;
            const long blocks = std::min<long>(pt_resident_blocks(k, 64 * kWaves), (tiles + kWaves - 1) / kWaves);
            hipLaunchKernelGGL(k, dim3((unsigned)blocks), block, 0, st, j, sc);
            return hipGetLastError();
        }
    }
    // The tiled layout is the drop-in's (pt_capi.cpp pt_render_opt_v4 and its work-queue entries): one
    // frame per call (NUM_SAMPLES_PER_FRAME = 1), never counted (counted launches are device jobs, the
    // row layouts only) -- so only the per-tile pool's uncounted instances exist for it.
    if constexpr (LAYOUT == PT_LAYOUT_TILED_PLANAR8) {
        if (count || j.nframes >= kChunk) return hipErrorInvalidValue;
        const auto tile_go = [&](auto kern) {
            const long blocks = std::min<long>(pt_resident_blocks(kern, 64 * kWaves), (tiles + kWaves - 1) / kWaves);
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), block, 0, st, j, sc);
        };
        if (j.default_scene) {
            if (j.fast_exp && j.random_jitter && j.rejection) tile_go(pt_v4_kernel<ENV, LAYOUT, false, true, 1, true>);
            else if (j.fast_exp) tile_go(pt_v4_kernel<ENV, LAYOUT, false, true, 1>);
            else tile_go(pt_v4_kernel<ENV, LAYOUT, false, true, 0>);
        } else {
            if (j.fast_exp) tile_go(pt_v4_kernel<ENV, LAYOUT, false, false, 1>);
            else tile_go(pt_v4_kernel<ENV, LAYOUT, false, false, 0>);
        }
    } else if (j.default_scene) {
        if (count) go(pt_v4_kernel<ENV, LAYOUT, true, true, 2>, pt_v4_ct_kernel<ENV, LAYOUT, true, true, 2>);
        else if (j.fast_exp && j.random_jitter && j.rejection)
            go(pt_v4_kernel<ENV, LAYOUT, false, true, 1, true>, pt_v4_ct_kernel<ENV, LAYOUT, false, true, 1, true>);
        else if (j.fast_exp) go(pt_v4_kernel<ENV, LAYOUT, false, true, 1>, pt_v4_ct_kernel<ENV, LAYOUT, false, true, 1>);
        else go(pt_v4_kernel<ENV, LAYOUT, false, true, 0>, pt_v4_ct_kernel<ENV, LAYOUT, false, true, 0>);
    } else {
        if (count) go(pt_v4_kernel<ENV, LAYOUT, true, false, 2>, pt_v4_ct_kernel<ENV, LAYOUT, true, false, 2>);
        else if (j.fast_exp) go(pt_v4_kernel<ENV, LAYOUT, false, false, 1>, pt_v4_ct_kernel<ENV, LAYOUT, false, false, 1>);
        else go(pt_v4_kernel<ENV, LAYOUT, false, false, 0>, pt_v4_ct_kernel<ENV, LAYOUT, false, false, 0>);
    }
    return hipGetLastError();
}

template <int ENV>
hipError_t launch_env(const PtV4Job& j, const PtV4Scene& sc, hipStream_t st, bool count, uint32_t* ct_blocks)
{
    switch (j.layout) {
        case PT_LAYOUT_INTERLEAVED: return launch_t<ENV, PT_LAYOUT_INTERLEAVED>(j, sc, st, count, ct_blocks);
        case PT_LAYOUT_PLANAR8: return launch_t<ENV, PT_LAYOUT_PLANAR8>(j, sc, st, count, ct_blocks);
        case PT_LAYOUT_TILED_PLANAR8: return launch_t<ENV, PT_LAYOUT_TILED_PLANAR8>(j, sc, st, count, ct_blocks);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t pt_v4_set_chain_polls(uint32_t polls)
{
    const uint32_t v = polls ? polls : kPtChainPolls;
    return hipMemcpyToSymbol(HIP_SYMBOL(pt_chain_polls_dev), &v, sizeof(v));
}

hipError_t pt_launch_v4(const PtV4Job& j_in, const PtV4Scene& sc, hipStream_t st, bool count, bool* presented,
                        uint32_t* ct_blocks)
{
    if (presented) *presented = false;
    if (ct_blocks) *ct_blocks = 0;
    if (j_in.ncols <= 0 || j_in.nrows <= 0 || j_in.nframes <= 0) return hipSuccess;
    // the fused output stage (j.pix_out) runs in the presenting instances only: the drop-in's calls
    // (DemofoxRenderOptV4: the tiled layout, one frame -- the per-tile pool kernel), the default scene
    // and sampling flags, fast exp, and the default fast ACES / gamma
    PtV4Job j = j_in;
    if (j.pix_out && !(j.layout == PT_LAYOUT_TILED_PLANAR8 && j.nframes < kChunk && j.default_scene && j.fast_exp &&
                       j.random_jitter && j.rejection && j.pix_fast_tone && !count))
        j.pix_out = nullptr;
    if (presented) *presented = j.pix_out != nullptr;
    if (sc.nquads < 0 || sc.nspheres < 0 || sc.nquads + sc.nspheres > PT_V4_MAX_OBJECTS) return hipErrorInvalidValue;
    if (j.env_mode != PT_V4_ENV_NONE_ && (!j.env || j.env_w <= 0 || j.env_h <= 0)) return hipErrorInvalidValue;
    if (count && !j.counters) return hipErrorInvalidValue;
    if (!j.queue || (j.order && (!j.units || !j.nunits))) return hipErrorInvalidValue;
    switch (j.env_mode) {
        case PT_V4_ENV_NONE_: return launch_env<PT_V4_ENV_NONE_>(j, sc, st, count, ct_blocks);
        case PT_V4_ENV_EQUIRECT_: return launch_env<PT_V4_ENV_EQUIRECT_>(j, sc, st, count, ct_blocks);
        case PT_V4_ENV_CUBEMAP_: return launch_env<PT_V4_ENV_CUBEMAP_>(j, sc, st, count, ct_blocks);
        default: return hipErrorInvalidValue;
    }
}
