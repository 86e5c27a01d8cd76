// tests/native/check_envcert.cpp -- host check of the certified env-texel cells (csrc/pt_envcert.h)
// against the exact glibc restatements the kernels fall back to (csrc/pt_invtrig.h):
//   1. every f32 q in [2^-40, 2^40]: atanf_glibc(q) lies in [fl(ec_atan(q) - E), fl(ec_atan(q) + E)];
//   2. every f32 a in [0, 1 - 2^-20]: asinf_glibc(a) lies in [fl(ec_asin(a) - E), fl(ec_asin(a) + E)];
//   3. N pseudo-random (y, x) pairs of the domain, every sign combination: atan2f_glibc(y, x) lies in
//      ec_atan2_bounds (the sign / x < 0 glue of e_atan2f.c), and asinf_glibc(s) in ec_asin_bounds;
//   4. N pseudo-random unit directions (normalised like the kernels' rays): every certified cell of
//      the v4 random-jitter sampler (2048 x 1024 map, random draws) and of the config-4 nearest
//      sampler equals the cell of the exact pipeline; prints the fallback (uncertified) rates.
// 1 and 2 make the containment a proof for every input of the domain (the GPU computes the same
// bits: f32 add/mul/fma and correctly rounded 1/x, a/b, sqrt); 3 and 4 exercise the glue and the
// monotone maps.  Exit status 1 on any violation.
#include "../../cpuperformanceraytracer_amd/csrc/pt_invtrig.h"
#include "../../cpuperformanceraytracer_amd/csrc/pt_envcert.h"
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

// the kernels' exact pipelines (pt_v4.hip equirect/sample_random, pt_kernel.hip env_sample)
static float saturate(float x) { return std::fmin(std::fmax(x, 0.0f), 1.0f); }
static void exact_random(float y, float x, float s, float w, float h, float r1, float r2, float& row, float& col)
{
    const float at = pt::atan2f_glibc(y, x), as = pt::asinf_glibc(s);
    float u = std::fmaf(0.1591f, at, 0.5f), v = std::fmaf(0.3183f, as, 0.5f);
    u = saturate(u - std::floor(u));
    v = saturate(v - std::floor(v));
    row = std::floor(std::fmaf(v, h, -v) + r1);
    col = std::floor(std::fmaf(u, w, -u) + r2);
}
static bool exact_nearest(float y, float x, float s, int W, int H, int32_t& row, int32_t& col)
{
    float u = pt::atan2f_glibc(y, x), v = pt::asinf_glibc(s);
    u = u * 0.1591f;
    v = v * 0.3183f;
    u = u + 0.5f;
    v = v + 0.5f;
    u -= (float)(int32_t)u;
    v -= (float)(int32_t)v;
    if (!(u >= 0.0f && u < 1.0f && v >= 0.0f && v < 1.0f)) return false;
    row = (int32_t)(v * (float)(H - 1));
    col = (int32_t)(u * (float)(W - 1));
    return true;
}

int main(int argc, char** argv)
{
    const long n = argc > 1 ? std::atol(argv[1]) : 100000000L;
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0 || nt > 16) nt = 8;
    std::atomic<long> bad_atan{0}, bad_asin{0}, bad_glue{0}, bad_rand{0}, bad_near{0}, fb_rand{0}, fb_near{0}, fb_nat{0}, n_nat{0},
        n_atan{0}, n_asin{0}, n_dir{0};
    std::vector<double> e_atan(nt, 0.0), e_asin(nt, 0.0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            long ba = 0, bs = 0, bg = 0, br = 0, bn = 0, fr = 0, fn = 0, na = 0, ns = 0, nd = 0, fnat = 0, nnat = 0;
            for (uint64_t u = 0x2b800000u + t; u <= 0x53800000u; u += nt) {   // 2^-40 .. 2^40
                const float q = pt::it_float((uint32_t)u);
                const float zg = pt::atanf_glibc(q), z = pt::ec_atan(q);
                ++na;
                e_atan[t] = std::fmax(e_atan[t], std::fabs((double)z - (double)zg));
                if (!(z - pt::kEcAtanE <= zg && zg <= z + pt::kEcAtanE)) {
                    if (ba < 3) std::printf("atan %a: %a vs %a\n", q, z, zg);
                    ++ba;
                }
            }
            for (uint64_t u = t; u <= 0x3f7ffff0u; u += nt) {   // 0 .. 1 - 2^-20
                const float a = pt::it_float((uint32_t)u);
                const float sg = pt::asinf_glibc(a), s = pt::ec_asin(a);
                ++ns;
                e_asin[t] = std::fmax(e_asin[t], std::fabs((double)s - (double)sg));
                if (!(s - pt::kEcAsinE <= sg && sg <= s + pt::kEcAsinE)) {
                    if (bs < 3) std::printf("asin %a: %a vs %a\n", a, s, sg);
                    ++bs;
                }
            }
            uint64_t st = 0x9E3779B97F4A7C15ull * (t + 1);
            auto next = [&] {
                st ^= st << 13; st ^= st >> 7; st ^= st << 17;
                return st;
            };
            for (long i = 0; i < n / (long)nt; ++i) {
                // a unit direction, normalised as the kernels do (v * RN(1 / RN(sqrt(dot))))
                const uint64_t a = next(), b = next(), c = next();
                float dx = (float)((int32_t)(a & 0xffffffffu)) * 0x1p-31f, dy = (float)((int32_t)(b & 0xffffffffu)) * 0x1p-31f,
                      dz = (float)((int32_t)(c & 0xffffffffu)) * 0x1p-31f;
                if (i % 7 == 0) dy *= 0x1p-12f;   // grazing directions
                if (i % 11 == 0) dx *= 0x1p-14f;
                const float dd = std::fmaf(dx, dx, std::fmaf(dy, dy, dz * dz));
                if (!(dd > 1e-6f)) continue;
                const float g = 1.0f / std::sqrt(dd);
                dx *= g, dy *= g, dz *= g;
                ++nd;
                // 3: the glue (every sign combination of the domain's pairs)
                if (pt::ec_in_domain(dz, dx, dy)) {
                    float lo, hi;
                    pt::ec_atan2_bounds(dz, dx, lo, hi);
                    const float ag = pt::atan2f_glibc(dz, dx);
                    if (!(lo <= ag && ag <= hi)) {
                        if (bg < 3) std::printf("atan2 %a %a: %a not in [%a, %a]\n", dz, dx, ag, lo, hi);
                        ++bg;
                    }
                    pt::ec_asin_bounds(dy, lo, hi);
                    const float sg = pt::asinf_glibc(dy);
                    if (!(lo <= sg && sg <= hi)) ++bg;
                }
                // 4: the cells (v4 equirect takes (-D.x, D.y, -D.z); the sign is irrelevant here)
                const float r1 = (float)(int32_t)(next() & 0x7fffffffu) * 0x1p-31f, r2 = (float)(int32_t)(next() & 0x7fffffffu) * 0x1p-31f;
                float er, ec, cr, cc;
                exact_random(dz, dx, dy, 2048.0f, 1024.0f, r1, r2, er, ec);
                if (pt::ec_cell_random(dz, dx, dy, 2048.0f, 1024.0f, r1, r2, cr, cc)) {
                    if (cr != er || cc != ec) {
                        if (br < 3) std::printf("random cell %a %a %a: (%g %g) vs (%g %g)\n", dz, dx, dy, cr, cc, er, ec);
                        ++br;
                    }
                } else {
                    ++fr;
                    fnat += (i % 7 != 0 && i % 11 != 0);
                }
                nnat += (i % 7 != 0 && i % 11 != 0);
                int32_t nr, nc, xr, xc;
                const bool inr = exact_nearest(dz, dx, dy, 2048, 1024, xr, xc);
                if (pt::ec_cell_nearest(dz, dx, dy, 2047.0f, 1023.0f, nr, nc)) {
                    if (!inr || nr != xr || nc != xc) {
                        if (bn < 3) std::printf("nearest cell %a %a %a: (%d %d) vs (%d %d)\n", dz, dx, dy, nr, nc, xr, xc);
                        ++bn;
                    }
                } else {
                    ++fn;
                }
            }
            bad_atan += ba; bad_asin += bs; bad_glue += bg; bad_rand += br; bad_near += bn; fb_rand += fr; fb_near += fn;
            n_atan += na; n_asin += ns; n_dir += nd; fb_nat += fnat; n_nat += nnat;
        });
    for (auto& x : th) x.join();
    double ea = 0, es = 0;
    for (unsigned t = 0; t < nt; ++t) ea = std::fmax(ea, e_atan[t]), es = std::fmax(es, e_asin[t]);
    std::printf("atan checked %ld violations %ld max_err %.3g\n", n_atan.load(), bad_atan.load(), ea);
    std::printf("asin checked %ld violations %ld max_err %.3g\n", n_asin.load(), bad_asin.load(), es);
    std::printf("glue checked %ld violations %ld\n", n_dir.load(), bad_glue.load());
    std::printf("random cells checked %ld violations %ld fallback_rate %.3g\n", n_dir.load(), bad_rand.load(),
                (double)fb_rand.load() / (double)n_dir.load());
    std::printf("random cells, uniform directions only: fallback_rate %.3g\n", (double)fb_nat.load() / (double)n_nat.load());
    std::printf("nearest cells checked %ld violations %ld fallback_rate %.3g\n", n_dir.load(), bad_near.load(),
                (double)fb_near.load() / (double)n_dir.load());
    return (bad_atan || bad_asin || bad_glue || bad_rand || bad_near) ? 1 : 0;
}
