// tests/native/check_libmf.cpp -- host check of the product's glibc restatements
// (cpuperformanceraytracer_amd/csrc/pt_libmf.h, compiled here for the host) against the host libm
// expf / powf the oracle calls (where the reference calls SVML exp_ps / pow_ps).
//   check_libmf exp             every f32 bit pattern
//   check_libmf pow_gamma       powf(x, 1/2.4f) for every f32 x in [2^-9, 1] (LinearToSRGB's domain)
//   check_libmf pow_random N    N pseudo-random (x, y), x positive normal, |y log2 x| < 126
// Prints "checked N mismatches M"; exits non-zero on any mismatch.
#include "../../cpuperformanceraytracer_amd/csrc/pt_libmf.h"
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

static bool same(float a, float b) { return std::memcmp(&a, &b, 4) == 0 || (a != a && b != b); }

static int run(uint64_t n, const std::function<bool(uint64_t, float*, float*, float*)>& one)
{
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0 || nt > 16) nt = 8;
    std::atomic<uint64_t> bad{0}, cnt{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            uint64_t b = 0, c = 0;
            for (uint64_t i = t; i < n; i += nt) {
                float arg, got, want;
                if (!one(i, &arg, &got, &want)) continue;
                if (!same(got, want)) {
                    if (b < 4) std::printf("mismatch at %a: %a vs libm %a\n", arg, got, want);
                    ++b;
                }
                ++c;
            }
            bad += b;
            cnt += c;
        });
    for (auto& x : th) x.join();
    std::printf("checked %llu mismatches %llu\n", (unsigned long long)cnt.load(), (unsigned long long)bad.load());
    return bad.load() ? 1 : 0;
}

int main(int argc, char** argv)
{
    const char* what = argc > 1 ? argv[1] : "exp";
    if (!std::strcmp(what, "exp")) {
        return run(1ull << 32, [](uint64_t i, float* a, float* got, float* want) {
            const uint32_t u = (uint32_t)i;
            std::memcpy(a, &u, 4);
            *got = pt::lm::expf_glibc(*a);
            *want = expf(*a);
            return true;
        });
    }
    if (!std::strcmp(what, "pow_gamma")) {
        const float y = 1.0f / 2.4f;   // set1x3_ps(1.f) / 2.4f (v4 :184)
        const uint32_t lo = 0x3b000000u /* 2^-9 */, hi = 0x3f800000u /* 1 */;
        return run(hi - lo + 1, [=](uint64_t i, float* a, float* got, float* want) {
            const uint32_t u = lo + (uint32_t)i;
            std::memcpy(a, &u, 4);
            *got = pt::lm::powf_glibc_main(*a, y);
            *want = powf(*a, y);
            return true;
        });
    }
    if (!std::strcmp(what, "pow_random")) {
        const uint64_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 100000000ull;
        return run(n, [](uint64_t i, float* a, float* got, float* want) {
            uint64_t s = i * 0x9E3779B97F4A7C15ull + 12345;
            s ^= s >> 29; s *= 0xBF58476D1CE4E5B9ull; s ^= s >> 32;
            const uint32_t ux = 0x00800000u + (uint32_t)(s % (0x7f800000u - 0x00800000u));   // positive normal
            const uint32_t uy = (uint32_t)(s >> 32);
            float x, y;
            std::memcpy(&x, &ux, 4);
            std::memcpy(&y, &uy, 4);
            if (!(std::fabs(y) < 1e30f) || y == 0.0f) return false;
            if (!(std::fabs((double)y * std::log2((double)x)) < 125.0)) return false;
            *a = x;
            *got = pt::lm::powf_glibc_main(x, y);
            *want = powf(x, y);
            return true;
        });
    }
    std::fprintf(stderr, "unknown check %s\n", what);
    return 2;
}
