// tests/native/check_invtrig.cpp -- host check of the product's atan2f/asinf restatements
// (cpuperformanceraytracer_amd/csrc/pt_invtrig.h compiled for the host) against the host libm:
//   asinf  every f32 in [-1, 1]          atanf  every non-negative f32 (and its negation)
//   atan2f N pseudo-random pairs: half unit-vector components (the env sampler's inputs), half
//          arbitrary bit patterns.
// Prints per-function counts; exit status 1 on any mismatch.
#include "../../cpuperformanceraytracer_amd/csrc/pt_invtrig.h"
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static bool same(float a, float b) { return pt::it_bits(a) == pt::it_bits(b) || (std::isnan(a) && std::isnan(b)); }

int main(int argc, char** argv)
{
    const long npairs = argc > 1 ? std::atol(argv[1]) : 200000000L;
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0 || nt > 16) nt = 8;
    std::atomic<long> bad_asin{0}, bad_atan{0}, bad_atan2{0}, n_asin{0}, n_atan{0}, n_atan2{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            long ba = 0, bt = 0, b2 = 0, na = 0, ntn = 0, n2 = 0;
            for (uint64_t u = t; u <= 0x3f800000u; u += nt)
                for (int sg = 0; sg < 2; ++sg) {
                    const float x = pt::it_float((uint32_t)u | (sg ? 0x80000000u : 0u));
                    ++na;
                    if (!same(pt::asinf_glibc(x), asinf(x))) ++ba;
                }
            for (uint64_t u = t; u < 0x7f800000u; u += nt)
                for (int sg = 0; sg < 2; ++sg) {
                    const float x = pt::it_float((uint32_t)u | (sg ? 0x80000000u : 0u));
                    ++ntn;
                    if (!same(pt::atanf_glibc(x), atanf(x))) {
                        if (bt < 3) std::printf("atanf %a: %a vs %a\n", x, pt::atanf_glibc(x), atanf(x));
                        ++bt;
                    }
                }
            uint64_t s = 0x9E3779B97F4A7C15ull * (t + 1);
            for (long i = 0; i < npairs / (long)nt; ++i) {
                s ^= s << 13; s ^= s >> 7; s ^= s << 17;
                float x, y;
                if (i & 1) {
                    const float a = (float)((s & 0xffffffffu) * (6.283185307179586 / 4294967296.0));
                    const float zz = ((float)((s >> 32) & 0xffffff) / 16777216.0f) * 2.0f - 1.0f;
                    const float rr = std::sqrt(1.0f - zz * zz);
                    x = rr * std::cos(a);
                    y = rr * std::sin(a);
                } else {
                    x = pt::it_float((uint32_t)s);
                    y = pt::it_float((uint32_t)(s >> 32));
                }
                ++n2;
                if (!same(pt::atan2f_glibc(y, x), atan2f(y, x))) {
                    if (b2 < 3) std::printf("atan2f %a %a\n", y, x);
                    ++b2;
                }
            }
            bad_asin += ba; bad_atan += bt; bad_atan2 += b2; n_asin += na; n_atan += ntn; n_atan2 += n2;
        });
    for (auto& x : th) x.join();
    std::printf("asinf checked %ld mismatches %ld\natanf checked %ld mismatches %ld\natan2f checked %ld mismatches %ld\n",
                n_asin.load(), bad_asin.load(), n_atan.load(), bad_atan.load(), n_atan2.load(), bad_atan2.load());
    return (bad_asin || bad_atan || bad_atan2) ? 1 : 0;
}
