// tests/native/check_sky.cpp -- the diffuse kernel's sky test (pt_kernel.hip sky_ray): a camera ray
// (origin 0) with |D.x| > 0.51 D.z or |D.y| > 0.51 D.z misses every primitive, so a tile whose
// camera rays all satisfy it skips their TestSceneTrace.  Checked against the oracle's
// TestSceneTrace (oracle/pt_oracle.c pto_trace_scene, the reference's f32 operations):
//   1. every camera ray of several images (mainImage's camera, scalar.cpp:338-351) that the
//      predicate classifies as sky;
//   2. dense direction grids across and along the thresholds (slopes 0.4 .. 1.6 on one axis, the
//      whole field on the other, both signs) -- every sky direction must miss.
// It also reports the largest slope max(|D.x|, |D.y|) / D.z of any direction that hits.
//
// usage: check_sky    exit 0 iff no sky direction hits
#include <cmath>
#include <cstdint>
#include <cstdio>

#include "../../oracle/pt_oracle.h"

namespace {

constexpr float kSkySlope = 0.51f;   // pt_kernel.hip
bool sky_ray(const float D[3])
{
    return std::fabs(D[0]) > kSkySlope * D[2] || std::fabs(D[1]) > kSkySlope * D[2];
}
void normalize_ref(float v[3])   // mathlib.h:750
{
    const float inv = 1.0f / std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    v[0] *= inv, v[1] *= inv, v[2] *= inv;
}

long long n_sky = 0, n_bad = 0, n_dirs = 0;
double max_hit_slope = 0.0;   // the largest max(|D.x|, |D.y|) / D.z of a direction that hits

void check(const float D[3])
{
    ++n_dirs;
    const float P[3] = {0.0f, 0.0f, 0.0f};
    float n[3];
    int id;
    const float dist = pto_trace_scene(P, D, n, &id);
    const bool hit = dist != 10000.0f;
    if (hit)
        max_hit_slope = std::fmax(max_hit_slope, std::fmax(std::fabs((double)D[0]), std::fabs((double)D[1])) / (double)D[2]);
    if (!sky_ray(D)) return;
    ++n_sky;
    if (hit && ++n_bad <= 20) std::printf("SKY RAY HITS id=%d D=(%a, %a, %a) dist=%g\n", id, D[0], D[1], D[2], dist);
}

void image(int w, int h)
{
    const float W = (float)w, H = (float)h, aspect = W / H;
    const float cam_dist = 1.0f / std::tan(90.0f * 0.5f * 3.14159265359f / 180.0f);   // :338
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float fx = (float)x, fy = (float)(h - 1 - y);
            float D[3] = {(fx / W) * 2.0f - 1.0f, ((fy / H) * 2.0f - 1.0f) / aspect, cam_dist};
            normalize_ref(D);
            check(D);
        }
}

void grid(int axis, double lo, double hi, int n1, int n2)
{
    for (int i = 0; i < n1; ++i)
        for (int j = 0; j < n2; ++j)
            for (int sgn = -1; sgn <= 1; sgn += 2) {
                const double a = sgn * (lo + (hi - lo) * (i + 0.5) / n1);
                const double b = -1.6 + 3.2 * (j + 0.5) / n2;
                float D[3];
                D[axis] = (float)a;
                D[1 - axis] = (float)b;
                D[2] = 1.0f;
                normalize_ref(D);
                check(D);
            }
}

}  // namespace

int main()
{
    image(256, 256);
    image(1920, 1080);
    image(3840, 2160);
    image(1000, 2000);   // a portrait aspect: the y slopes reach 2
    grid(0, 0.40, 0.60, 1500, 1200);   // across the x threshold
    grid(1, 0.40, 0.60, 1500, 1200);   // across the y threshold
    grid(0, 0.60, 1.60, 300, 600);
    grid(1, 0.60, 1.60, 300, 600);
    std::printf("directions %lld  classified sky %lld  sky rays that hit %lld  largest hitting slope %.4f "
                "(threshold %.2f)\n", n_dirs, n_sky, n_bad, max_hit_slope, kSkySlope);
    return n_bad || max_hit_slope >= kSkySlope ? 1 : 0;
}
