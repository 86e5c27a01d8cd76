// pt_quadcull.h -- the six quad tests of TestSceneTrace (demofox_path_tracing_scalar.cpp:186-261,
// TestQuadTrace :65-143) with ONE exact quad test per ray instead of six, bit-identical results.
//
// Why.  The exact quad test costs ~48 VALU instructions for the three scalar triples that decide
// "inside" plus ~24 for the barycentric hit point and its distance; a wave's 64 rays point in all
// directions, so every quad's tail runs in every iteration: 6 x 72 = 435 of the ~765 instructions
// of a path-tracing iteration (pt_kernel.hip, ISA of the round-1 kernel).  What the reference
// needs from the six tests is only (closest accepted quad, its distance, flipped or not).
//
// How.  Per ray, every quad is classified with a few cheap f32 operations on the line's
// intersection X with the quad's plane (all quads are axis-aligned rectangles, checked below):
//   OUT   -- X is outside the rectangle by more than a margin: the reference's test certainly
//            rejects the quad (its u or w is certainly negative, whichever triangle it picks);
//   else  -- a *candidate* if its distance could exceed c_minimumRayHitTime; its distance, if the
//            reference accepts it, lies in [s - delta, s + delta] (s = our plane distance).
// The candidate with the smallest lower bound, W, is tested exactly (the reference's arithmetic,
// quad_exact below).  The result is certified when W is accepted and every other candidate's lower
// bound exceeds W's exact distance (so none can be accepted closer, nor tie).  Otherwise the ray is
// flagged uncertain and the caller runs the six exact tests for it (pt_kernel.hip: rare, decided
// per wave).  A ray with no candidate certainly misses every quad.
//
// Error bounds (eps = 2^-24; P the ray origin, D its direction, pq = fl(fl(P + D) - P) the
// reference's line direction; all arithmetic the reference's f32, round to nearest):
// (1) Scalar triples.  Each of the reference's u, v, w is a triple product T' = pb.(pc x pq) of
//     the f32 vectors pX = fl(X - P).  Against the exact T = (b - P).((c - P) x pq):
//       |T' - T| <= (5.0002 sqrt2 eps + 2 eps) |b-P| |c-P| |pq| <= 9.1 eps R^2 |pq|
//     (cross: eps(2+eps) per component of M = |pc|x|pq| "abs-cross", |M| <= sqrt2 |pc||pq|; dot:
//     gamma3; inputs: |fl(b - P) - (b - P)| <= eps |b - P|).  With R = max |vertex - P| <= 42 for
//     every origin the path tracer produces (the camera at 0; points inside the box, checked per
//     ray: |x|,|y| <= 13, |z - 30| <= 6) and |pq| <= 1.0001: |T' - T| <= 9.6e-4; every bound below
//     uses E_T = kET = 1.2e-3 (x 1.25).
// (2) Geometry.  With X = P + sigma pq on the quad's plane (axis j), T = pq . ((e1-X) x (e2-X)) =
//     +-pq_j L_e dist(X, edge e) for the edge (e1, e2) the triple tests (u: bc or cd, w: ab or da,
//     v: the diagonal ac).  So T' has the sign of the geometry when dist > E_T / (L_e |pq_j|).
// (3) OUT.  If X is beyond an edge of length L by more than 2 E_T / (L |pq_j|), the reference
//     rejects whichever triangle its v picks: the picked triangle owns that edge (rejected by (2)),
//     or v put X within E_T/(|ac| |pq_j|) of the other side of the diagonal, and then X is beyond
//     the picked triangle's other outer edge by more than E_T/(L' |pq_j|) (rectangle geometry:
//     beyond bc by d and across ac => beyond cd by (H d - E_T/|pq_j|) / W).  In the rectangle's
//     centred coordinates Y = X - centre: OUT if h2 |Y1| - h1 h2 > K g_j or h1 |Y2| - h1 h2 > K g_j
//     with g_j = |1/pq_j| and K = kET + 3.6e-4 (covers our own rounding of s, Y: 4.1 eps |s| +
//     eps |P| + eps |Y|, |s| <= 35 g_j, and of the fma).
// (4) Distance.  If the reference accepts a quad (u', v', w' >= 0), its weights beta' = T'/sum T'
//     differ from X's barycentrics beta (sum beta = sum beta' = 1) by
//       sum|dbeta| <= (3 E_T + 3 E_T sum|beta|) / S' <= 7.11 E_T / S
//     where S = sum T = |pq_j| x rect area and S' = sum T' >= S - 3 E_T >= 0.9 S (requires S >= 30 E_T,
//     i.e. |pq_j| >= kTiny for the smallest quad), beta_i >= -E_T/S (T'_i >= 0), so
//     sum|beta| <= 1.14.  In centred coordinates (sum dbeta = 0) the reference's ip_k is within
//     h_k sum|dbeta| + 7 eps max|V_k| of X_k, and with |pq_k/D_k - 1| <= eps (|P_k|/|D_k| + 2), our
//     s within 4 eps of sigma and the rounding of dist and of s +- delta:
//       |dist - s| <= |s| 1.25 eps (|P_k| |1/D_k| + 10.7) + (A_j g_j + B) |1/D_k|
//     A_j = max over the quads on axis j of 7.11 kET h_k,max / area, B = 3e-5.
// (5) Parallel camera rays.  A camera ray through the image's centre column or row has pq_j = 0
//     exactly: the line is parallel to the planes on axis j at height h = |c - P_j|.  Then
//     u + v + w = 0 for either triangle, so the reference can pass only with all three |T| <=
//     2 E_T; but the triples of two perpendicular edges are h L |sin phi| and h L' |cos phi|, one
//     of which is >= h 5 / sqrt2 > 2 kET for h > 1e-3: OUT.  (Pool rays: pq_j = 0 flags.)
// tests/native/check_quadcull.cpp verifies the certified results against the oracle's exact quad
// stage on realistic path segments and on adversarial rays (edges, corners, grazing, near the
// 0.01 threshold), and that the observed triple-product and distance errors stay far inside
// E_T and delta.
//
// Host + device header.  The includer defines, before including:
//   PTQC_HD                      function qualifiers
//   PTQC_RCP_APPROX(x)           1/x within 1 ulp (v_rcp_f32)
//   PTQC_RCP_EXACT(x)            the reference's correctly rounded 1.0f / x
//   PTQC_DIV_EXACT(a, b, y)      the reference's correctly rounded a / b (y = RN(1/b)), as used by
//                                the product's exact quad test
//   PTQC_FMA(a, b, c)            fused multiply-add
#pragma once
#include <stdint.h>
#include "pt_scene.h"

namespace ptqc {

struct F3 {
    float x, y, z;
};
PTQC_HD F3 f3(float x, float y, float z) { return F3{x, y, z}; }
PTQC_HD float comp(F3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
PTQC_HD F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
PTQC_HD float dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }   // mathlib.h:64
PTQC_HD F3 cross(F3 u, F3 v) { return f3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x); }
PTQC_HD F3 sel(bool c, F3 a, F3 b) { return f3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }

// A quad as an axis-aligned rectangle: plane x_j = c; in-plane axes k1, k2 with centres c1, c2
// (0 on x and y, 30 on z) and half-sizes h1, h2.
struct Rect {
    int j;
    float c;
    int k1;
    float c1, h1;
    int k2;
    float c2, h2;
};
constexpr Rect kRect[PT_NQUADS] = {
    {2, 35.0f, 0, 0.0f, 12.6f, 1, 0.0f, 12.6f},      // back wall
    {1, -12.45f, 0, 0.0f, 12.6f, 2, 30.0f, 5.0f},    // floor
    {1, 12.5f, 0, 0.0f, 12.6f, 2, 30.0f, 5.0f},      // ceiling
    {0, -12.5f, 1, 0.0f, 12.6f, 2, 30.0f, 5.0f},     // left wall
    {0, 12.5f, 1, 0.0f, 12.6f, 2, 30.0f, 5.0f},      // right wall
    {1, 12.4f, 0, 0.0f, 5.0f, 2, 30.0f, 2.5f},   // light
};
constexpr float kDemofoxZCentre = 30.0f;

// Every vertex of DemofoxScene lies on its Rect's plane and on a corner of its rectangle.
constexpr float cabs(float x) { return x < 0.0f ? -x : x; }
constexpr float ccomp(const float* v, int k) { return v[k]; }
constexpr bool rect_matches(int q)
{
    const Rect r = kRect[q];
    bool ok = r.j != r.k1 && r.j != r.k2 && r.k1 != r.k2;
    ok = ok && (r.k1 == 2 ? r.c1 == kDemofoxZCentre : r.c1 == 0.0f) && (r.k2 == 2 ? r.c2 == kDemofoxZCentre : r.c2 == 0.0f);
    bool lo1 = false, hi1 = false, lo2 = false, hi2 = false;
    for (int v = 0; v < 4; ++v) {
        const float* p = DemofoxScene::qv[q][v];
        ok = ok && ccomp(p, r.j) == r.c && cabs(ccomp(p, r.k1) - r.c1) == r.h1 && cabs(ccomp(p, r.k2) - r.c2) == r.h2;
        lo1 = lo1 || ccomp(p, r.k1) < r.c1;
        hi1 = hi1 || ccomp(p, r.k1) > r.c1;
        lo2 = lo2 || ccomp(p, r.k2) < r.c2;
        hi2 = hi2 || ccomp(p, r.k2) > r.c2;
        // the unit normal (pt_scene.h) is +e_j: the reference's facing test is D_j > 0
        ok = ok && DemofoxScene::qn[q][r.j] == 1.0f && DemofoxScene::qn[q][r.k1] == 0.0f && DemofoxScene::qn[q][r.k2] == 0.0f;
    }
    return ok && lo1 && hi1 && lo2 && hi2;
}
static_assert(rect_matches(0) && rect_matches(1) && rect_matches(2) && rect_matches(3) && rect_matches(4) &&
                  rect_matches(5),
              "DemofoxScene quads must be the axis-aligned rectangles of kRect");

constexpr float kET = 1.2e-3f;              // (1)
constexpr float kK = kET + 3.6e-4f;         // (3)
constexpr float kTiny = 1e-3f;              // (4): below, a non-OUT quad on axis j is tested exactly
// (4): A_j for axes x (side walls 25.2 x 10), y (floor, ceiling 25.2 x 10; light 10 x 5), z (back
// wall 25.2 x 25.2): 7.11 kET h_k,max / area
constexpr float kA[3] = {7.11f * kET * 12.6f / 252.0f * 1.001f, 7.11f * kET * 5.0f / 50.0f * 1.001f,
                         7.11f * kET * 12.6f / 635.04f * 1.001f};
constexpr float kB = 3e-5f;
constexpr float kRho = 1.25f * 0x1p-24f;
constexpr float kMinHitLo = 0.0099999f;     // below c_minimumRayHitTime (0.01f) by > 1 ulp
constexpr float kInf = __builtin_huge_valf();
constexpr float kDomXY = 13.0f, kDomZ = 6.0f;   // origin domain of (1) (camera origin = 0 also ok)

// Quad index -> normal axis j (2 bits each): back 2, floor 1, ceiling 1, left 0, right 0, light 1.
constexpr uint32_t kAxisBits = (2u << 0) | (1u << 2) | (1u << 4) | (0u << 6) | (0u << 8) | (1u << 10);
static_assert(((kAxisBits >> 0) & 3) == (uint32_t)kRect[0].j && ((kAxisBits >> 2) & 3) == (uint32_t)kRect[1].j &&
                  ((kAxisBits >> 4) & 3) == (uint32_t)kRect[2].j && ((kAxisBits >> 6) & 3) == (uint32_t)kRect[3].j &&
                  ((kAxisBits >> 8) & 3) == (uint32_t)kRect[4].j && ((kAxisBits >> 10) & 3) == (uint32_t)kRect[5].j,
              "kAxisBits");

// median of three (never NaN here: the lower bounds are finite or +-inf)
PTQC_HD float med3(float a, float b, float c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_fmed3f(a, b, c);
#else
    const float lo = a < b ? a : b, hi = a < b ? b : a;
    const float m = c < hi ? c : hi;
    return m > lo ? m : lo;
#endif
}

// Outcome of the classification.  Each candidate's lower bound lb is kept as a signed-integer key
// (bits(lb) & ~7) | q: its float bits with the quad index in the low three bits.  For lb >= 0 the
// integer order is the float order, and clearing the three low bits only lowers the bound; every
// negative lb orders below every non-negative one (the order among negatives is irrelevant: any
// accepted distance exceeds 0.01, so a negative bound never certifies, whichever quad is W).  Ties
// go to the lower index.  So one min and one median per quad track the smallest key k1 (W = its
// low bits) and the second smallest k2, with no compare / select for W.  Non-candidates have the
// key of +inf (>= kNoKey).  unc = a quad's status could not be decided.
struct Cull {
    int32_t k1, k2;
    bool unc;
};
constexpr int32_t kNoKey = 0x7f800000;   // bits(+inf): the keys of non-candidates are >= it
PTQC_HD int32_t fbits(float x) { return __builtin_bit_cast(int32_t, x); }
PTQC_HD int32_t imin(int32_t a, int32_t b) { return a < b ? a : b; }
PTQC_HD int32_t imax(int32_t a, int32_t b) { return a < b ? b : a; }
PTQC_HD int32_t imed3(int32_t a, int32_t b, int32_t c) { return imax(imin(a, b), imin(imax(a, b), c)); }
// W: the quad to test exactly (-1: no candidate)
PTQC_HD int cull_W(const Cull& c) { return c.k1 < kNoKey ? (c.k1 & 7) : -1; }
// W's exact distance dist (> 0.01) is certified closest: every other candidate's bound exceeds it
PTQC_HD bool cull_beyond(const Cull& c, float dist) { return (c.k2 & ~7) > fbits(dist); }

// Per-quad classification, recorded only by the host check (tests/native/check_quadcull.cpp).
struct CullTrace {
    bool out[PT_NQUADS], cand[PT_NQUADS];
    float s[PT_NQUADS], dl[PT_NQUADS];
};

// Opposite walls (left / right on x, floor / ceiling on y) are congruent rectangles on parallel
// planes (static_asserts below).  Of such a pair only the wall the line runs towards -- the plane
// c = +-12.5 in the direction of pq_j -- can be met ahead of the origin when the origin lies between
// the planes; the other one is classified by its distance test alone: it is no candidate when
// s + delta <= c_minimumRayHitTime (exactly the rule below, whatever its OUT status), and when that
// test does not hold (an origin outside the slab, a loose bound) the ray is flagged uncertain and
// takes the six exact tests.  A ray nearly parallel to the pair (|pq_j| < kTiny: (4) does not hold,
// ~0.1% of the rays per axis) classifies the far wall as a rectangle too, in a branch.  So the
// classification computes four rectangles and two distance tests instead of six rectangles; every
// certified result is certified by the same rules.
struct Pair {
    int q_lo, q_hi;   // the quads at the lower / higher plane
};
constexpr Pair kPairX{3, 4}, kPairY{1, 2};
constexpr bool pair_ok(Pair p)
{
    const Rect a = kRect[p.q_lo], b = kRect[p.q_hi];
    return a.j == b.j && a.k1 == b.k1 && a.k2 == b.k2 && a.c1 == b.c1 && a.c2 == b.c2 && a.h1 == b.h1 && a.h2 == b.h2 &&
           a.c < b.c;
}
static_assert(pair_ok(kPairX) && pair_ok(kPairY), "opposite walls must be congruent rectangles on parallel planes");

// The rectangle classification of quad q with plane constant c (q's or its pair partner's; the
// other Rect fields are q's) into the running keys (k1, k2).
template <bool CAMERA>
PTQC_HD void classify(Cull& o, int q, Rect R, float c, int qi, F3 P, F3 pq, F3 Pc, const float* r, const float* mu,
                      const bool* tiny, float rho, const float* d0, CullTrace* tr)
{
    const float s = (c - comp(P, R.j)) * r[R.j];                     // plane distance along pq
    const float Y1 = PTQC_FMA(s, comp(pq, R.k1), comp(Pc, R.k1));    // centred in-plane coords
    const float Y2 = PTQC_FMA(s, comp(pq, R.k2), comp(Pc, R.k2));
    const float h1h2 = R.h1 * R.h2;
    bool out = PTQC_FMA(R.h2, __builtin_fabsf(Y1), -h1h2) > mu[R.j] || PTQC_FMA(R.h1, __builtin_fabsf(Y2), -h1h2) > mu[R.j];
    if (CAMERA) out = out || (comp(pq, R.j) == 0.0f && __builtin_fabsf(c - comp(P, R.j)) > 1e-3f);   // (5)
    const float dl = PTQC_FMA(__builtin_fabsf(s), rho, d0[R.j]);
    // a non-OUT quad whose distance bound (4) does not hold (tiny |pq_j|) gets the lower bound
    // -inf: it becomes W and is tested exactly, and a second such quad fails the certification
    const bool cand = !out && (tiny[R.j] || s + dl > kMinHitLo);
    if (tr) tr->out[q] = out, tr->cand[q] = cand, tr->s[q] = s, tr->dl[q] = tiny[R.j] ? kInf : dl;
    const float lb = cand ? (tiny[R.j] ? -kInf : s - dl) : kInf;
    const int32_t key = (fbits(lb) & ~7) | qi;
    o.k2 = imed3(o.k1, o.k2, key);   // second smallest (k1 <= k2 holds throughout)
    o.k1 = imin(o.k1, key);
}

// The distance test alone of quad q at plane c: true when q is certainly no candidate.
PTQC_HD bool behind(int q, Rect R, float c, F3 P, const float* r, float rho, const float* d0, CullTrace* tr)
{
    const float s = (c - comp(P, R.j)) * r[R.j];
    const float dl = PTQC_FMA(__builtin_fabsf(s), rho, d0[R.j]);
    const bool ok = !(s + dl > kMinHitLo);
    if (tr) tr->out[q] = false, tr->cand[q] = !ok, tr->s[q] = s, tr->dl[q] = dl;
    return ok;
}

// Classify the six quads for the ray (P, D) with the reference's line direction pq; k = the lane's
// distance axis (:121-133), dP = P_k, yD = RN(1/D_k).  CAMERA: P is the camera origin (0, 0, 0).
template <bool CAMERA>
PTQC_HD Cull cull(F3 P, F3 pq, float dP, float yD, CullTrace* tr = nullptr)
{
    const float r0 = PTQC_RCP_APPROX(pq.x), r1 = PTQC_RCP_APPROX(pq.y), r2 = PTQC_RCP_APPROX(pq.z);
    const float g[3] = {__builtin_fabsf(r0), __builtin_fabsf(r1), __builtin_fabsf(r2)};
    const float r[3] = {r0, r1, r2};
    const float mu[3] = {kK * g[0], kK * g[1], kK * g[2]};
    const bool tiny[3] = {!(__builtin_fabsf(pq.x) >= kTiny), !(__builtin_fabsf(pq.y) >= kTiny),
                          !(__builtin_fabsf(pq.z) >= kTiny)};
    const float ayD = __builtin_fabsf(yD);
    const float rho = PTQC_FMA(__builtin_fabsf(dP), ayD, 10.7f) * kRho;
    const float d0[3] = {PTQC_FMA(kA[0], g[0], kB) * ayD, PTQC_FMA(kA[1], g[1], kB) * ayD,
                         PTQC_FMA(kA[2], g[2], kB) * ayD};
    const F3 Pc = f3(P.x, P.y, P.z - kDemofoxZCentre);   // centred origin (centres 0, 0, 30)
    bool unc = false;   // the origin is outside the domain of (1)
    if (!CAMERA)
        unc = !(__builtin_fabsf(P.x) <= kDomXY && __builtin_fabsf(P.y) <= kDomXY && __builtin_fabsf(Pc.z) <= kDomZ);
    Cull o{0x7fffffff, 0x7fffffff, false};
    // the reference's order: back (0), floor (1), ceiling (2), left (3), right (4), light (5); the
    // classification's result does not depend on the order (ties in lb: W = the lower index)
    classify<CAMERA>(o, 0, kRect[0], kRect[0].c, 0, P, pq, Pc, r, mu, tiny, rho, d0, tr);
    {   // floor / ceiling: the one pq.y runs towards, the other by its distance
        static_assert(kPairY.q_hi == kPairY.q_lo + 1, "y pair");
        const uint32_t neg = (uint32_t)fbits(r1) >> 31;   // pq.y < 0
        const bool up = neg == 0;
        const int qa = kPairY.q_hi - (int)neg, qb = kPairY.q_lo + (int)neg;
        const float ca = up ? kRect[kPairY.q_hi].c : kRect[kPairY.q_lo].c, cb = up ? kRect[kPairY.q_lo].c : kRect[kPairY.q_hi].c;
        if (tr) {   // (host check: record under the real quad indices)
            classify<CAMERA>(o, qa, kRect[qa], ca, qa, P, pq, Pc, r, mu, tiny, rho, d0, tr);
            if (tiny[1]) classify<CAMERA>(o, qb, kRect[qb], cb, qb, P, pq, Pc, r, mu, tiny, rho, d0, tr);
            else unc = !behind(qb, kRect[qb], cb, P, r, rho, d0, tr) || unc;
        } else {
            classify<CAMERA>(o, kPairY.q_lo, kRect[kPairY.q_lo], ca, qa, P, pq, Pc, r, mu, tiny, rho, d0, nullptr);
            if (tiny[1]) classify<CAMERA>(o, kPairY.q_lo, kRect[kPairY.q_lo], cb, qb, P, pq, Pc, r, mu, tiny, rho, d0, nullptr);
            else unc = !behind(kPairY.q_lo, kRect[kPairY.q_lo], cb, P, r, rho, d0, nullptr) || unc;
        }
    }
    {   // left / right walls (planes x = -+12.5: the forward one is copysign(12.5, pq.x), by bits)
        static_assert(kRect[kPairX.q_lo].c == -kRect[kPairX.q_hi].c && kPairX.q_hi == kPairX.q_lo + 1, "x pair");
        const uint32_t neg = (uint32_t)fbits(r0) >> 31;   // pq.x < 0 (r0 = +-inf for pq.x = +-0)
        const int qa = kPairX.q_hi - (int)neg, qb = kPairX.q_lo + (int)neg;
        const float ca = __builtin_bit_cast(float, fbits(kRect[kPairX.q_hi].c) | (int32_t)(neg << 31)), cb = -ca;
        if (tr) {
            classify<CAMERA>(o, qa, kRect[qa], ca, qa, P, pq, Pc, r, mu, tiny, rho, d0, tr);
            if (tiny[0]) classify<CAMERA>(o, qb, kRect[qb], cb, qb, P, pq, Pc, r, mu, tiny, rho, d0, tr);
            else unc = !behind(qb, kRect[qb], cb, P, r, rho, d0, tr) || unc;
        } else {
            classify<CAMERA>(o, kPairX.q_lo, kRect[kPairX.q_lo], ca, qa, P, pq, Pc, r, mu, tiny, rho, d0, nullptr);
            if (tiny[0]) classify<CAMERA>(o, kPairX.q_lo, kRect[kPairX.q_lo], cb, qb, P, pq, Pc, r, mu, tiny, rho, d0, nullptr);
            else unc = !behind(kPairX.q_lo, kRect[kPairX.q_lo], cb, P, r, rho, d0, nullptr) || unc;
        }
    }
    classify<CAMERA>(o, 5, kRect[5], kRect[5].c, 5, P, pq, Pc, r, mu, tiny, rho, d0, tr);
    o.unc = unc;
    return o;
}

// TestQuadTrace (scalar.cpp:65-143) of one quad whose vertices a, b, c, d are already in the
// reference's order after its facing flip, with (ak, bk, ck, dk) their components on the lane's
// distance axis.  Returns kAccepted when the reference accepts (u, w >= 0 and 0.01 < dist < limit),
// kOutside when its inside test fails, kRejected when the distance test does.
// LIMIT = false: the caller's limit is c_superFar and the ray's |dD| >= 0.1 (pt_kernel.hip's axis
// rule on a unit direction), so an accepted distance is finite and < 10^4 anyway: |ip_k - dP| <= 70
// (ip_k a weighted mean of the vertices' k components, |.| <= 35; |dP| <= 36 for the camera origin
// and every origin of cull()'s domain -- others take the exact fallback), dist <= 700.
enum QuadExact : int { kOutside = 0, kRejected = 1, kAccepted = 2 };
template <bool LIMIT = true>
PTQC_HD int quad_exact(F3 P, F3 pq, F3 a, F3 b, F3 c, F3 d, float ak, float bk, float ck, float dk, float dP,
                       float dD, float yD, float limit, float& dist)
{
    // straight-line: every lane evaluates every step (a rejected lane's later values are unused;
    // its weight sum is replaced by 1 so the reciprocal stays on its fast path)
    const F3 pa = sub(a, P), pc = sub(c, P);
    const F3 m = cross(pc, pq);                        // :90
    float v = dot(pa, m);                              // :91
    const bool t1 = v >= 0.0f;                         // :93 triangle a,b,c (else a,c,d)
    const F3 pe = sub(sel(t1, b, d), P);               // pb | pd (the same subtraction)
    const float tu = dot(pe, m);                       // :96 -dot(pb, m) | :109 dot(pd, m)
    const float u = t1 ? -tu : tu;
    const float w = dot(cross(pq, sel(t1, pe, pa)), sel(t1, pa, pe));   // :98 | :111 ScalarTriple
    v = t1 ? v : -v;                                   // :113
    const bool inside = !(u < 0.0f || w < 0.0f);       // :97,99,110,112
    const float denom = PTQC_RCP_EXACT(inside ? (u + v) + w : 1.0f);   // :100 / :114
    const float un = u * denom, vn = v * denom, wn = w * denom;
    const float ek = t1 ? bk : dk;
    const float ip = (un * ak + vn * ek) + wn * ck;    // :104 / :118, component k
    dist = PTQC_DIV_EXACT(ip - dP, dD, yD);            // :124 / :128 / :132
    if (!inside) return kOutside;
    return dist > PT_MIN_HIT && (!LIMIT || dist < limit) ? kAccepted : kRejected;   // :135
}

}  // namespace ptqc
