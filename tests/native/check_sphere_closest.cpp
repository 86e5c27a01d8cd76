// tests/native/check_sphere_closest.cpp -- host check of the closest-sphere argument both kernels
// rely on (pt_kernel.hip spheres_closest, pt_v4.hip trace<DEF>): for pairwise-disjoint spheres, of
// the spheres that pass the reference's early tests the one with the largest b is the only one
// whose distance can be the accepted minimum, so evaluating its root alone -- and running the
// sequential tests when its distance fails c_minimumRayHitTime -- gives TestSphereTrace's result.
//
// Both arithmetic flavours are modelled with the reference's f32 operations (-ffp-contract=off):
//   diffuse (demofox_path_tracing_scalar.cpp:145-184): b = dot(m, d), c = dot(m, m) - r^2,
//            discr = b*b - c, plain (x*x' + y*y') + z*z' dots, the DemofoxScene spheres;
//   v4      (demofox_path_tracing_optimization_v4.cpp:641-695): fused dots fma(x,x', fma(y,y', z*z')),
//            cc = fma(-r, r, dot(m, m)), discr = fma(b, b, -cc), the v4 InitializeScene spheres.
// For every ray the sequential tests (in order, strict '<' against a running best that starts at a
// random "quad" distance) and the closest-sphere stage must agree on (distance bits, sphere,
// inside) whenever the stage does not fall back, and the candidate with the largest b must be the
// first (D.x > 0) or last (else) candidate in index order -- the rule both kernels use instead of
// comparing b's (the spheres of both scenes lie on one x line).  Ray families: random origins and directions,
// rays aimed between two neighbouring spheres (grazing both), origins just off a sphere surface
// (either side), origins inside a sphere.
//
// usage: check_sphere_closest [n_per_family] [seed]     exit 0 iff no disagreement
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../cpuperformanceraytracer_amd/csrc/pt_scene.h"
#include "../../cpuperformanceraytracer_amd/csrc/pt_v4_default_scene.h"

namespace {

constexpr float kMinHit = 0.01f;   // c_minimumRayHitTime (both files)

struct F3 {
    float x, y, z;
};
F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
float dot_plain(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
float dot_fma(F3 a, F3 b) { return std::fmaf(a.x, b.x, std::fmaf(a.y, b.y, a.z * b.z)); }

struct Res {
    float dist;
    int id;
    bool inside;
};

// one sphere up to the distance (the reference's operations); returns false on the early reject
template <bool V4>
bool sphere_pre(F3 P, F3 D, const float* s, float& b, float& discr)
{
    const F3 m = sub(P, F3{s[0], s[1], s[2]});
    if (V4) {
        b = dot_fma(m, D);
        const float cc = std::fmaf(-s[3], s[3], dot_fma(m, m));
        discr = std::fmaf(b, b, -cc);
        return !(discr < 0.0f || (cc > 0.0f && b > 0.0f));
    }
    b = dot_plain(m, D);
    const float c = dot_plain(m, m) - s[3] * s[3];
    discr = b * b - c;
    return !((c > 0.0f && b > 0.0f) || discr < 0.0f);
}
template <bool V4>
float sphere_dist(float b, float discr, bool& inside)
{
    const float sq = std::sqrt(discr);
    if (V4) {
        inside = -b < sq;
        return (inside ? sq : -sq) - b;
    }
    float dist = -b - sq;
    inside = dist < 0.0f;
    return inside ? -b + sq : dist;
}

template <bool V4>
Res sequential(F3 P, F3 D, const float (*sph)[4], int n, float best0)
{
    Res r{best0, -1, false};
    for (int k = 0; k < n; ++k) {
        float b, discr;
        if (!sphere_pre<V4>(P, D, sph[k], b, discr)) continue;
        bool inside;
        const float dist = sphere_dist<V4>(b, discr, inside);
        if (dist > kMinHit && dist < r.dist) r = Res{dist, k, inside};
    }
    return r;
}

// the kernels' stage: argmax b over the early-test survivors, one root; fb = fell back
template <bool V4>
Res closest(F3 P, F3 D, const float (*sph)[4], int n, float best0, bool& fb)
{
    float bmax = -INFINITY, dsel = 0.0f;
    int ksel = -1;
    for (int k = 0; k < n; ++k) {
        float b, discr;
        const bool hit = sphere_pre<V4>(P, D, sph[k], b, discr);
        if (hit && b > bmax) bmax = b, dsel = discr, ksel = k;
    }
    fb = false;
    Res r{best0, -1, false};
    if (ksel < 0) return r;
    bool inside;
    const float dist = sphere_dist<V4>(bmax, dsel, inside);
    if (dist > kMinHit) {
        if (dist < r.dist) r = Res{dist, ksel, inside};
        return r;
    }
    fb = true;
    return sequential<V4>(P, D, sph, n, best0);
}

uint64_t g_rng = 0x2545F4914F6CDD1Dull;
double urand()
{
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (double)(g_rng >> 11) * 0x1p-53;
}
F3 normalize_ref(F3 v)   // mathlib.h:750
{
    const float inv = 1.0f / std::sqrt(dot_plain(v, v));
    return F3{v.x * inv, v.y * inv, v.z * inv};
}
F3 rand_dir()
{
    for (;;) {
        const F3 v{(float)(2 * urand() - 1), (float)(2 * urand() - 1), (float)(2 * urand() - 1)};
        const float l = dot_plain(v, v);
        if (l > 1e-4f && l <= 1.0f) return normalize_ref(v);
    }
}

long long n_rays = 0, n_fb = 0, n_bad = 0, n_hit = 0, n_multi = 0;

template <bool V4>
void check(F3 P, F3 D, const float (*sph)[4], int n)
{
    ++n_rays;
    const float best0 = urand() < 0.5 ? 10000.0f : (float)(0.005 + 60.0 * urand());
    bool fb;
    const Res a = sequential<V4>(P, D, sph, n, best0), c = closest<V4>(P, D, sph, n, best0, fb);
    n_fb += fb;
    n_hit += a.id >= 0;
    int cands = 0;
    for (int k = 0; k < n; ++k) {
        float b, discr;
        cands += sphere_pre<V4>(P, D, sph[k], b, discr);
    }
    n_multi += cands > 1;
    {   // both kernels: the argmax of b is the first / last candidate by sign(D.x) (collinear spheres)
        float bmax = -INFINITY;
        int karg = -1;
        uint32_t cand = 0;
        for (int k = 0; k < n; ++k) {
            float b, discr;
            const bool c = sphere_pre<V4>(P, D, sph[k], b, discr);
            if (c) cand |= 1u << k;
            if (c && b > bmax) bmax = b, karg = k;
        }
        int kord = -1;
        if (cand) {
            kord = D.x > 0.0f ? __builtin_ctz(cand) : 31 - __builtin_clz(cand);
            float b, discr;
            sphere_pre<V4>(P, D, sph[kord], b, discr);
            if (!(b == b)) kord = -1;
        }
        if (kord != karg && ++n_bad <= 20)
            std::printf("ORDER MISMATCH P=(%a,%a,%a) D=(%a,%a,%a) argmax=%d order=%d\n", P.x, P.y, P.z, D.x, D.y, D.z,
                        karg, kord);
    }
    if (std::memcmp(&a.dist, &c.dist, 4) || a.id != c.id || (a.id >= 0 && a.inside != c.inside)) {
        if (++n_bad <= 20)
            std::printf("MISMATCH %s P=(%a,%a,%a) D=(%a,%a,%a) seq=(%a,%d,%d) closest=(%a,%d,%d)\n", V4 ? "v4" : "diffuse",
                        P.x, P.y, P.z, D.x, D.y, D.z, a.dist, a.id, a.inside, c.dist, c.id, c.inside);
    }
}

template <bool V4>
void families(const float (*sph)[4], int n, long N, F3 lo, F3 hi, const char* name)
{
    const long long r0 = n_rays, f0 = n_fb, h0 = n_hit, m0 = n_multi;
    auto rand_in = [&]() {
        return F3{(float)(lo.x + (hi.x - lo.x) * urand()), (float)(lo.y + (hi.y - lo.y) * urand()),
                  (float)(lo.z + (hi.z - lo.z) * urand())};
    };
    for (long i = 0; i < N; ++i) check<V4>(rand_in(), rand_dir(), sph, n);   // uniform
    for (long i = 0; i < N; ++i) {   // between two neighbouring spheres, grazing both
        const int k = (int)(urand() * (n - 1));
        const float* a = sph[k];
        const float* b = sph[k + 1];
        const double t = 0.3 + 0.4 * urand();
        F3 target{(float)(a[0] + t * (b[0] - a[0])), (float)(a[1] + t * (b[1] - a[1]) + (urand() - 0.5) * 2.0 * a[3]),
                  (float)(a[2] + t * (b[2] - a[2]) + (urand() - 0.5) * 2.0 * a[3])};
        const F3 P = rand_in();
        check<V4>(P, normalize_ref(sub(target, P)), sph, n);
    }
    for (long i = 0; i < N; ++i) {   // origin just off a surface, either side, any direction
        const int k = (int)(urand() * n);
        const F3 u = rand_dir();
        const double r = sph[k][3] + std::pow(10.0, -5.0 + 4.0 * urand()) * (urand() < 0.5 ? -1 : 1);
        const F3 P{(float)(sph[k][0] + r * u.x), (float)(sph[k][1] + r * u.y), (float)(sph[k][2] + r * u.z)};
        check<V4>(P, rand_dir(), sph, n);
    }
    for (long i = 0; i < N; ++i) {   // origin inside a sphere
        const int k = (int)(urand() * n);
        const F3 u = rand_dir();
        const double r = sph[k][3] * urand();
        const F3 P{(float)(sph[k][0] + r * u.x), (float)(sph[k][1] + r * u.y), (float)(sph[k][2] + r * u.z)};
        check<V4>(P, rand_dir(), sph, n);
    }
    std::printf("%-8s rays %9lld  sphere hits %8lld  >1 candidate %8lld  fallbacks %6lld\n", name, n_rays - r0,
                n_hit - h0, n_multi - m0, n_fb - f0);
}

}  // namespace

int main(int argc, char** argv)
{
    const long N = argc > 1 ? std::atol(argv[1]) : 200000;
    if (argc > 2) g_rng = std::strtoull(argv[2], nullptr, 0) | 1;
    float dsph[PT_NSPHERES][4];
    for (int k = 0; k < PT_NSPHERES; ++k)
        for (int j = 0; j < 4; ++j) dsph[k][j] = DemofoxScene::sph[k][j];
    // diffuse: origins over the box and in front of it (the camera side)
    families<false>(dsph, PT_NSPHERES, N, F3{-12.5f, -12.45f, 0.0f}, F3{12.5f, 12.5f, 35.0f}, "diffuse");
    families<true>(pt_v4_default::kSphere, pt_v4_default::kSpheres, N, F3{-25.0f, -12.0f, -5.0f},
                   F3{25.0f, 15.0f, 45.0f}, "v4");
    std::printf("rays %lld  disagreements %lld\n", n_rays, n_bad);
    return n_bad ? 1 : 0;
}
