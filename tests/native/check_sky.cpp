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
// The same for the v4 kernel's sky test (pt_v4.hip sky_ray_v4) against the v4 oracle's TestSceneTrace
// (pto4_trace_scene, InitializeScene, camera at (0, 0, 40)): v4 camera rays with the jitter at its
// extremes, and slope grids around every threshold.
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

// ---- v4 (demofox_path_tracing_optimization_v4.cpp InitializeScene, camera at (0, 0, 40)) ----
bool sky_ray_v4(const float D[3])   // pt_v4.hip
{
    const float nz = -D[2], ax = std::fabs(D[0]);
    const bool band_hi = D[1] > 0.34f * nz && D[1] < 0.52f * nz && ax < 0.32f * nz;
    return nz > 0.0f && (D[1] < -0.52f * nz || ax > 1.02f * nz || (D[1] > -0.03f * nz && !band_hi));
}
long long n4_dirs = 0, n4_sky = 0, n4_bad = 0;
void check4(const float D[3])
{
    ++n4_dirs;
    if (!sky_ray_v4(D)) return;
    ++n4_sky;
    const float P[3] = {0.0f, 0.0f, 40.0f};
    int mat;
    const float dist = pto4_trace_scene(nullptr, P, D, &mat);
    if (dist != 10000.0f && ++n4_bad <= 20)
        std::printf("V4 SKY RAY HITS mat=%d D=(%a, %a, %a) dist=%g\n", mat, D[0], D[1], D[2], dist);
}
void normalize_fma(float v[3])   // v4's normalize: v * rcp(sqrt(dot)), dot = fma(x,x', fma(y,y', z*z'))
{
    const float inv = 1.0f / std::sqrt(std::fmaf(v[0], v[0], std::fmaf(v[1], v[1], v[2] * v[2])));
    v[0] *= inv, v[1] *= inv, v[2] *= inv;
}
void image4(int w, int h)   // mainImage v4 :1092-1130, jitter at its extremes and the centre
{
    const float rW = 1.0f / (float)w, rH = 1.0f / (float)h, H = (float)h;
    const float jit[3] = {-0.5f, 0.0f, 0.49999997f};
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            for (int jx = 0; jx < 3; ++jx)
                for (int jy = 0; jy < 3; jy += 2) {
                    const float tx = std::fmaf(((float)x + jit[jx]) * rW, 2.0f, -1.0f);
                    float ty = std::fmaf(((float)(h - 1 - y) + jit[jy]) * rH, 2.0f, -1.0f);
                    ty = ty * (rW * H);
                    float D[3] = {tx, ty, -1.0f};
                    normalize_fma(D);
                    check4(D);
                }
}
void grid4(double sx0, double sx1, double sy0, double sy1, int n1, int n2)
{
    for (int i = 0; i < n1; ++i)
        for (int j = 0; j < n2; ++j)
            for (int sgn = -1; sgn <= 1; sgn += 2) {
                float D[3] = {(float)(sgn * (sx0 + (sx1 - sx0) * (i + 0.5) / n1)), (float)(sy0 + (sy1 - sy0) * (j + 0.5) / n2),
                              -1.0f};
                normalize_fma(D);
                check4(D);
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
    image4(480, 270);
    image4(1920, 1080);
    grid4(0.0, 1.3, -0.7, 0.7, 1300, 1400);      // the whole field
    grid4(0.0, 1.1, -0.06, -0.02, 1100, 400);     // around sy = -0.043 / -0.03
    grid4(0.2, 0.4, 0.30, 0.56, 800, 800);        // around the ceiling band's corners
    grid4(0.95, 1.05, -0.6, 0.1, 400, 700);       // around sx = 1.0 / 1.02
    grid4(0.0, 1.1, -0.56, -0.48, 1100, 400);     // around sy = -0.5 / -0.52
    std::printf("v4 directions %lld  classified sky %lld  sky rays that hit %lld\n", n4_dirs, n4_sky, n4_bad);
    return n_bad || n4_bad || max_hit_slope >= kSkySlope ? 1 : 0;
}
