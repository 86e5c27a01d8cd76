// tests/native/check_quadcull.cpp -- host check of the product's quad culling (csrc/pt_quadcull.h)
// against the oracle's exact quad stage (oracle/pt_oracle.c: pto_trace_quads, the six
// TestQuadTrace calls of demofox_path_tracing_scalar.cpp:192-261).
//
// For every ray it checks, per quad:
//   * a quad classified OUT fails the reference's inside test;
//   * a non-candidate that passes the inside test has dist <= 0.01;
//   * a quad passing the inside test has |dist - s| <= delta (max ratio reported);
//   * the reference's triple products are within E_T of their exact values (max ratio reported);
// and per ray: the certified fast result (quad, distance bits, flip) equals the oracle's, and the
// per-quad exact tests composed in order equal the oracle (validates quad_exact).
//
// usage: check_quadcull [n_random_per_family] [seed]     exit 0 iff no violation
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define PTQC_HD static inline
// v_rcp_f32 is accurate to 1 ulp: model it as the correctly rounded 1/x moved by one ulp for a
// pseudo-random half of the inputs (the bounds assume <= 2 eps relative error).
static inline float rcp_1ulp(float x)
{
    float r = 1.0f / x;
    uint32_t b;
    std::memcpy(&b, &x, 4);
    if (std::isfinite(r) && r != 0.0f && ((b * 2654435761u) >> 31)) r = std::nextafter(r, (b & 1) ? INFINITY : -INFINITY);
    return r;
}
#define PTQC_RCP_APPROX(x) rcp_1ulp(x)
#define PTQC_RCP_EXACT(x) (1.0f / (x))
#define PTQC_DIV_EXACT(a, b, y) ((a) / (b))
#define PTQC_FMA(a, b, c) std::fmaf((a), (b), (c))
#include "../../cpuperformanceraytracer_amd/csrc/pt_quadcull.h"
#include "../../oracle/pt_oracle.h"

using ptqc::F3;
using ptqc::f3;

static long long n_rays = 0, n_unc = 0, n_fail = 0, n_nocand = 0;
static long long n_r_flag = 0, n_r_wrej = 0, n_r_block = 0, n_r_block_own = 0, n_r_wrej_own = 0;
static double max_dist_ratio = 0.0, max_T_ratio = 0.0;
static const double kETtheory = 9.6e-4;

static void fail(const char* what, F3 P, F3 D, int q)
{
    if (++n_fail <= 20)
        std::printf("VIOLATION %s q=%d P=(%a,%a,%a) D=(%a,%a,%a)\n", what, q, P.x, P.y, P.z, D.x, D.y, D.z);
}

// exact triple (b-P).((c-P) x pq) in long double from the f32 inputs
static long double triple_exact(const float* b, const float* c, F3 P, F3 pq)
{
    long double bx = (long double)b[0] - P.x, by = (long double)b[1] - P.y, bz = (long double)b[2] - P.z;
    long double cx = (long double)c[0] - P.x, cy = (long double)c[1] - P.y, cz = (long double)c[2] - P.z;
    long double mx = cy * pq.z - cz * pq.y, my = cz * pq.x - cx * pq.z, mz = cx * pq.y - cy * pq.x;
    return bx * mx + by * my + bz * mz;
}
static float triple_ref(const float* b, const float* c, F3 P, F3 pq)   // f32, the reference's order
{
    const F3 pb = f3(b[0] - P.x, b[1] - P.y, b[2] - P.z), pc = f3(c[0] - P.x, c[1] - P.y, c[2] - P.z);
    return ptqc::dot(pb, ptqc::cross(pc, pq));
}

static void check_ray(F3 P, F3 D, bool camera)
{
    ++n_rays;
    const F3 Q = f3(P.x + D.x, P.y + D.y, P.z + D.z);
    const F3 pq = f3(Q.x - P.x, Q.y - P.y, Q.z - P.z);
    const int axis = std::fabs(D.x) > 0.1f ? 0 : (std::fabs(D.y) > 0.1f ? 1 : 2);   // scalar.cpp:121-133
    const float dP = ptqc::comp(P, axis), dD = ptqc::comp(D, axis);
    const float yD = 1.0f / dD;
    ptqc::CullTrace tr;
    const ptqc::Cull c = camera ? ptqc::cull<true>(P, pq, dP, yD, &tr) : ptqc::cull<false>(P, pq, dP, yD, &tr);

    // per-quad exact tests (reference order a,b,c,d after the facing flip)
    float best = PT_SUPER_FAR;
    int best_id = -1, best_flip = 0;
    float qdist[PT_NQUADS];
    int qcode[PT_NQUADS], qflip[PT_NQUADS];
    for (int q = 0; q < PT_NQUADS; ++q) {
        const ptqc::Rect R = ptqc::kRect[q];
        const bool flip = ptqc::comp(D, R.j) > 0.0f;
        const float* v[4];
        for (int i = 0; i < 4; ++i) v[i] = DemofoxScene::qv[q][flip ? 3 - i : i];
        auto V = [&](int i) { return f3(v[i][0], v[i][1], v[i][2]); };
        qcode[q] = ptqc::quad_exact(P, pq, V(0), V(1), V(2), V(3), v[0][axis], v[1][axis], v[2][axis], v[3][axis], dP,
                                    dD, yD, PT_SUPER_FAR, qdist[q]);
        qflip[q] = flip;
        if (qcode[q] == ptqc::kAccepted && qdist[q] < best) best = qdist[q], best_id = q, best_flip = flip;
        // triple-product error vs exact (the three the reference evaluates, both triangles)
        const F3 Pv = P;
        const float *a = v[0], *b = v[1], *cc = v[2], *d = v[3];
        const float Tf[4] = {triple_ref(b, cc, Pv, pq), triple_ref(a, cc, Pv, pq), triple_ref(d, cc, Pv, pq),
                             triple_ref(a, b, Pv, pq)};
        const long double Te[4] = {triple_exact(b, cc, Pv, pq), triple_exact(a, cc, Pv, pq), triple_exact(d, cc, Pv, pq),
                                   triple_exact(a, b, Pv, pq)};
        for (int i = 0; i < 4; ++i) {
            const double r = (double)fabsl((long double)Tf[i] - Te[i]) / kETtheory;
            if (r > max_T_ratio) max_T_ratio = r;
        }
        // per-quad invariants of the classification
        if (tr.out[q] && qcode[q] != ptqc::kOutside) fail("OUT quad passes the inside test", P, D, q);
        if (!tr.out[q] && !tr.cand[q] && qcode[q] != ptqc::kOutside && qdist[q] > PT_MIN_HIT)
            fail("non-candidate with dist > 0.01", P, D, q);
        if (!tr.out[q] && qcode[q] != ptqc::kOutside && !c.unc) {
            const double r = std::fabs((double)qdist[q] - (double)tr.s[q]) / (double)tr.dl[q];
            if (r > max_dist_ratio) max_dist_ratio = r;
            if (r > 1.0) fail("|dist - s| > delta", P, D, q);
        }
    }
    int oid, oflip;
    const float odist = pto_trace_quads(&P.x, &D.x, &oid, &oflip);
    if (std::memcmp(&odist, &best, 4) || oid != best_id || (oid >= 0 && oflip != best_flip))
        fail("per-quad exact tests disagree with the oracle", P, D, oid);

    // the certified fast result
    bool unc = c.unc;
    float fd = PT_SUPER_FAR;
    int fid = -1, fflip = 0;
    const int cW = ptqc::cull_W(c);
    if (cW >= 0) {
        fid = cW;
        fd = qdist[cW];
        fflip = qflip[cW];
        auto own = [&](int q) { return std::fabs(ptqc::comp(P, ptqc::kRect[q].j) - ptqc::kRect[q].c) < 0.02f; };
        if (!c.unc && qcode[cW] != ptqc::kAccepted) ++n_r_wrej, n_r_wrej_own += own(cW);
        else if (!c.unc && !ptqc::cull_beyond(c, fd)) {
            ++n_r_block;
            for (int q = 0; q < PT_NQUADS; ++q)
                if (q != cW && tr.cand[q] && own(q)) { ++n_r_block_own; break; }
        }
        if (qcode[cW] != ptqc::kAccepted || !ptqc::cull_beyond(c, fd)) unc = true;
    } else {
        ++n_nocand;
    }
    if (c.unc) ++n_r_flag;
    if (unc) {
        ++n_unc;
        return;
    }
    if (std::memcmp(&fd, &odist, 4) || fid != oid || (oid >= 0 && fflip != oflip))
        fail("certified result differs from the oracle", P, D, oid);
}

// ---- ray families ----
static uint64_t g_rng = 88172645463325252ull;
static double urand()
{
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (double)(g_rng >> 11) * 0x1p-53;
}
static F3 normalize_f(F3 v)   // the reference's normalize (mathlib.h:750)
{
    const float inv = 1.0f / std::sqrt(ptqc::dot(v, v));
    return f3(v.x * inv, v.y * inv, v.z * inv);
}
static F3 rand_dir()
{
    for (;;) {
        const F3 v = f3((float)(2 * urand() - 1), (float)(2 * urand() - 1), (float)(2 * urand() - 1));
        const float l = ptqc::dot(v, v);
        if (l > 1e-4f && l <= 1.0f) return normalize_f(v);
    }
}
static F3 rand_in_box()
{
    return f3((float)(-12.49 + 24.98 * urand()), (float)(-12.44 + 24.93 * urand()), (float)(25.01 + 9.98 * urand()));
}
static F3 rand_on_quad(int q)
{
    const ptqc::Rect R = ptqc::kRect[q];
    float p[3];
    p[R.j] = R.c;
    p[R.k1] = (float)(R.c1 + R.h1 * (2 * urand() - 1));
    p[R.k2] = (float)(R.c2 + R.h2 * (2 * urand() - 1));
    return f3(p[0], p[1], p[2]);
}

// realistic paths: camera rays of a w x h image, frames 1..nf, bounces through the whole scene
static void family_paths(int w, int h, int nf, int bounces)
{
    const float W = (float)w, H = (float)h, aspect = W / H;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            for (int f = 1; f <= nf; ++f) {
                const float fx = (float)x, fy = (float)(h - 1 - y);
                F3 D = normalize_f(f3((fx / W) * 2.0f - 1.0f, ((fy / H) * 2.0f - 1.0f) / aspect, 1.0f));
                F3 P = f3(0, 0, 0);
                uint32_t rng = pto_seed((uint32_t)fx, (uint32_t)fy, (uint32_t)f);
                for (int b = 0; b <= bounces; ++b) {
                    check_ray(P, D, b == 0);
                    float n[3];
                    int id;
                    const float dist = pto_trace_scene(&P.x, &D.x, n, &id);
                    if (dist == PT_SUPER_FAR) break;
                    P = f3((P.x + D.x * dist) + n[0] * 0.01f, (P.y + D.y * dist) + n[1] * 0.01f,
                           (P.z + D.z * dist) + n[2] * 0.01f);
                    float r[3];
                    pto_random_unit_vector(&rng, r);
                    D = normalize_f(f3(n[0] + r[0], n[1] + r[1], n[2] + r[2]));
                }
            }
}

int main(int argc, char** argv)
{
    const long n = argc > 1 ? std::atol(argv[1]) : 200000;
    if (argc > 2) g_rng = std::strtoull(argv[2], nullptr, 0) | 1;
    long long base;
    auto report = [&](const char* fam) {
        std::printf("%-28s rays %9lld  uncertain %8lld (%.4f%%)  flag %lld  W-rejected %lld (own %lld)  blocked %lld (own %lld)\n", fam, n_rays - base, n_unc,
                    100.0 * (double)n_unc / (double)(n_rays - base), n_r_flag, n_r_wrej, n_r_wrej_own, n_r_block, n_r_block_own);
        n_unc = n_r_flag = n_r_wrej = n_r_block = n_r_block_own = n_r_wrej_own = 0;
        base = n_rays;
    };
    base = 0;
    // 1. realistic: 240x135 (1080p aspect), 4 frames, 8 bounces; and 64x64 (square)
    family_paths(240, 135, 4, 8);
    report("paths 240x135 x4f x8b");
    family_paths(64, 64, 2, 8);
    report("paths 64x64 x2f x8b");
    // 2. uniform origins in the box, uniform directions
    for (long i = 0; i < n; ++i) check_ray(rand_in_box(), rand_dir(), false);
    report("uniform box");
    // 3. aimed at quad edges and corners, offsets 1e-9 .. 1e-1 in and out of the rectangle
    for (long i = 0; i < n; ++i) {
        const int q = (int)(urand() * PT_NQUADS);
        const ptqc::Rect R = ptqc::kRect[q];
        F3 t = rand_on_quad(q);
        float p[3] = {t.x, t.y, t.z};
        const double off = std::pow(10.0, -9.0 + 8.0 * urand()) * (urand() < 0.5 ? -1 : 1);
        const int which = (int)(urand() * 3);   // edge along k1, k2, or a corner
        if (which != 1) p[R.k1] = (float)(R.c1 + (urand() < 0.5 ? -1 : 1) * (R.h1 + off));
        if (which != 0) p[R.k2] = (float)(R.c2 + (urand() < 0.5 ? -1 : 1) * (R.h2 + off));
        const F3 P = rand_in_box();
        check_ray(P, normalize_f(f3(p[0] - P.x, p[1] - P.y, p[2] - P.z)), false);
    }
    report("edges/corners");
    // 4. grazing directions (one component 1e-8 .. 1e-2)
    for (long i = 0; i < n; ++i) {
        F3 d = rand_dir();
        float c[3] = {d.x, d.y, d.z};
        c[(int)(urand() * 3)] *= (float)std::pow(10.0, -8.0 + 6.0 * urand());
        check_ray(rand_in_box(), normalize_f(f3(c[0], c[1], c[2])), false);
    }
    report("grazing");
    // 5. origins just off a quad (1e-4 .. 0.1 along its normal, either side), any direction
    for (long i = 0; i < n; ++i) {
        const int q = (int)(urand() * PT_NQUADS);
        const ptqc::Rect R = ptqc::kRect[q];
        F3 t = rand_on_quad(q);
        float p[3] = {t.x, t.y, t.z};
        p[R.j] += (float)(std::pow(10.0, -4.0 + 3.0 * urand()) * (urand() < 0.5 ? -1 : 1));
        check_ray(f3(p[0], p[1], p[2]), rand_dir(), false);
    }
    report("near a quad");
    // 6. camera rays in every direction of the front hemisphere
    for (long i = 0; i < n; ++i) {
        F3 d = rand_dir();
        check_ray(f3(0, 0, 0), f3(d.x, d.y, std::fabs(d.z)), true);
    }
    report("camera");
    std::printf("rays %lld  no-candidate %lld  max |dist-s|/delta %.3g  max |T'-T|/E_T(theory 9.6e-4) %.3g\n", n_rays,
                n_nocand, max_dist_ratio, max_T_ratio);
    std::printf("violations %lld\n", n_fail);
    return n_fail ? 1 : 0;
}
