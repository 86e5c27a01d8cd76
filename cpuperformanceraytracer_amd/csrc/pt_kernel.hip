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
//   * one lane = one pixel; the lane renders the launch's nframes samples of that pixel IN FRAME
//     ORDER and applies the reference's progressive lerp after each, so a launch of S frames is
//     bit-identical to S calls of DemofoxRenderScalar.  The accumulator is read once and written
//     once per launch.
//   * path regeneration: the bounce loop and the sample loop are flattened into one loop of
//     "segments" (one TestSceneTrace each).  A lane whose path ends (miss, or bounce budget spent)
//     finishes that sample and starts its next one in the same iteration, so a wave keeps all 64
//     lanes tracing until its lanes run out of samples; the loop exits when no lane has work
//     (exec mask empty == wave-wide __any() false; the COUNT build makes the ballot explicit).
//   * scene geometry is wave-uniform -> scalar loads (SGPR operands) from a device scene table,
//     re-read every segment rather than pinned in SGPRs (no SGPR spilling); per-lane closest-hit
//     material / normal lookups and the per-axis vertex components -> LDS tables.
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
#include <math.h>

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

// ---- correctly rounded '/' and sqrt (pt_exactmath.h), IEEE fallback outside the fast range ----
__device__ __forceinline__ float sqrt_x(float x)
{
    float s = pt::sqrt_rn(x);
    if (__builtin_expect(!(x >= 0x1p-100f), 0)) s = __builtin_sqrtf(x);   // 0, tiny, NaN
    return s;
}
__device__ __forceinline__ float rcp_x(float x)
{
    float r = pt::rcp_rn(x);
    const float ax = __builtin_fabsf(x);
    if (__builtin_expect(!(ax >= 0x1p-125f && ax <= 0x1p125f), 0)) r = 1.0f / x;
    return r;
}
// a / b with y = rcp_x(b) and b normal in [2^-125, 2^125]: exact whenever a/b is normal and
// |a| < 2^124; callers only use it where any other quotient is discarded by the reference's
// comparisons (see quad_test) or cannot occur (camera: 0 <= a <= 2^24).
__device__ __forceinline__ float div_x(float a, float b, float y) { return pt::div_rn(a, b, y); }

// mathlib.h:750   normalize = v * (1 / sqrt(dot(v, v)))
__device__ __forceinline__ V3 normalize(V3 v) { return mul(v, rcp_x(sqrt_x(dot(v, v)))); }

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

// Per-quad, per-axis vertex components (A_k, B_k, C_k, D_k): indexed by the lane's axis.
struct AxisRow {
    float a, b, c, d;
};

// TestQuadTrace, scalar.cpp:65-143.  `pq` = (rayPos + rayDir) - rayPos (ray-constant, hoisted),
// `axis`/`dP`/`dD`/`yD` = the component :121-133 divides by, its ray origin, direction, RN(1/dir).
// On a closer hit: best = dist, id = q, flag = flipped.
__device__ __forceinline__ void quad_test(const PtScene* __restrict__ sc, const AxisRow* s_axis, int q, V3 P, V3 D,
                                          V3 pq, int axis, float dP, float dD, float yD, float& best, int& id,
                                          int& flag)
{
    const AxisRow ax = s_axis[q * 3 + axis];                  // LDS, issued early
    const V3 n = v3(sc->qn[q][0], sc->qn[q][1], sc->qn[q][2]);
    const bool flip = dot(n, D) > 0.0f;                       // :69-80 (flipped order d,c,b,a)
    const V3 PA = sub(v3(sc->qv[q][0][0], sc->qv[q][0][1], sc->qv[q][0][2]), P);
    const V3 PB = sub(v3(sc->qv[q][1][0], sc->qv[q][1][1], sc->qv[q][1][2]), P);
    const V3 PC = sub(v3(sc->qv[q][2][0], sc->qv[q][2][1], sc->qv[q][2][2]), P);
    const V3 PD = sub(v3(sc->qv[q][3][0], sc->qv[q][3][1], sc->qv[q][3][2]), P);
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
    if (u < 0.0f || w < 0.0f) return;                         // :97,99,110,112
    // :100-103 / :114-117
    const float denom = rcp_x((u + v) + w);
    u *= denom;
    v *= denom;
    w *= denom;
    // :104 / :118 intersectPos = u*a + v*e + w*c (e = b or d), component `axis` only
    const float ak = flip ? ax.d : ax.a;
    const float ck = flip ? ax.b : ax.c;
    const float ek = t1 ? (flip ? ax.c : ax.b) : (flip ? ax.a : ax.d);
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
__device__ __forceinline__ void sphere_test(const PtScene* __restrict__ sc, int s, V3 P, V3 D, float& best, int& id,
                                            int& flag)
{
    const V3 m = sub(P, v3(sc->sph[s][0], sc->sph[s][1], sc->sph[s][2]));
    const float b = dot(m, D);
    const float c = dot(m, m) - sc->sph_r2[s];
    if (c > 0.0f && b > 0.0f) return;
    const float discr = b * b - c;
    if (discr < 0.0f) return;
    const float sq = sqrt_x(discr);
    float dist = -b - sq;
    bool inside = false;
    if (dist < 0.0f) {
        inside = true;
        dist = -b + sq;
    }
    if (dist > PT_MIN_HIT && dist < best) {
        best = dist;
        id = PT_NQUADS + s;
        flag = inside ? 1 : 0;
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

struct Sample {
    V3 P, D, T, ret;
    uint32_t rng;
    int bounce;
};

// Frame-constant camera terms (mainImage, scalar.cpp:338-351).
struct Camera {
    float W, H, yW, yH, aspect, yAspect, cam_dist;
};

// mainImage, scalar.cpp:329-360: seed + camera ray for (x, fy, iFrame).
__device__ __forceinline__ void start_sample(Sample& s, const Camera& cam, float fx, float fy, float iFrame)
{
    s.rng = ((uint32_t)fx * 1973u + (uint32_t)fy * 9277u + (uint32_t)iFrame * 26699u) | 1u;   // :332
    const float tx = div_x(fx, cam.W, cam.yW) * 2.0f - 1.0f;                                   // :342
    float ty = div_x(fy, cam.H, cam.yH) * 2.0f - 1.0f;
    ty = div_x(ty, cam.aspect, cam.yAspect);                                                    // :347
    s.D = normalize(v3(tx - 0.0f, ty - 0.0f, cam.cam_dist - 0.0f));                             // :351
    s.P = v3(0.0f, 0.0f, 0.0f);
    s.T = v3(1.0f, 1.0f, 1.0f);
    s.ret = v3(0.0f, 0.0f, 0.0f);
    s.bounce = 0;
}

template <int LAYOUT, bool ENV, bool COUNT>
__global__ __launch_bounds__(256) void pt_render_kernel(PtJob job)
{
    const PtScene* __restrict__ sc = job.scene;
    __shared__ PtLdsPrim s_prim[PT_NPRIMS];
    __shared__ AxisRow s_axis[PT_NQUADS * 3];
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
        } else if (t >= 64 && t < 64 + PT_NQUADS * 3) {
            const int q = (t - 64) / 3, k = (t - 64) % 3;
            s_axis[t - 64] = AxisRow{sc->qv[q][0][k], sc->qv[q][1][k], sc->qv[q][2][k], sc->qv[q][3][k]};
        }
    }
    __syncthreads();

    // 16x16 pixels per 256-thread block, one 8x8 pixel square per wave (coherent rays per wave).
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lc = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool valid = lc < job.ncols && lr < job.nrows;

    unsigned long long n_seg = 0, n_iter = 0, n_samp = 0, n_esc = 0;
    if (valid) {
        const size_t o = out_index<LAYOUT>(job, lc, lr);
        const size_t cs = (LAYOUT == PT_LAYOUT_INTERLEAVED) ? 1u : 8u;     // channel stride
        float* px = job.buf + o;
        V3 acc = v3(px[0], px[cs], px[2 * cs]);

        Camera cam;
        cam.W = (float)job.width;
        cam.H = (float)job.height;
        cam.yW = rcp_x(cam.W);
        cam.yH = rcp_x(cam.H);
        cam.aspect = div_x(cam.W, cam.H, cam.yH);                               // :346
        cam.yAspect = rcp_x(cam.aspect);
        cam.cam_dist = sc->cam_dist;
        const float fx = (float)(job.col0 + lc);                                 // :806
        const float fy = (float)(job.height - 1 - (job.row_start + lr * job.row_stride));  // :803
        int sidx = 0;
        float iFrame = (float)job.frame_first;
        Sample s;
        start_sample(s, cam, fx, fy, iFrame);

        for (;;) {
            if (COUNT) {
                n_iter += 64;
                ++n_seg;
            }
            // scene tables are re-read (scalar loads) each segment instead of living in SGPRs
            asm volatile("" ::: "memory");
            // ---- TestSceneTrace (:186-287) ----
            const V3 P = s.P, D = s.D;
            const V3 pq = sub(add(P, D), P);
            // :122-133 axis used for the hit distance (ray-constant)
            const int axis = fabsf(D.x) > 0.1f ? 0 : (fabsf(D.y) > 0.1f ? 1 : 2);
            const float dP = axis == 0 ? P.x : (axis == 1 ? P.y : P.z);
            const float dD = axis == 0 ? D.x : (axis == 1 ? D.y : D.z);
            const float yD = rcp_x(dD);
            float best = PT_SUPER_FAR;
            int id = -1, flag = 0;
#pragma unroll
            for (int q = 0; q < PT_NQUADS; ++q) quad_test(sc, s_axis, q, P, D, pq, axis, dP, dD, yD, best, id, flag);
#pragma unroll
            for (int k = 0; k < PT_NSPHERES; ++k) sphere_test(sc, k, P, D, best, id, flag);

            bool done;
            if (best == PT_SUPER_FAR) {                          // :305-310 miss
                V3 amb = v3(sc->ambient[0], sc->ambient[1], sc->ambient[2]);
                (void)ENV;
                s.ret = add(s.ret, amb);
                done = true;
                if (COUNT) ++n_esc;
            } else {
                const PtLdsPrim pr = s_prim[id];
                V3 n;
                if (id < PT_NQUADS) {
                    n = v3(pr.nx, pr.ny, pr.nz);
                    if (flag) n = mul(n, -1.0f);                  // :71
                } else {                                          // :179 sphere normal
                    const V3 h = sub(add(P, mul(D, best)), v3(pr.nx, pr.ny, pr.nz));
                    n = mul(normalize(h), flag ? -1.0f : 1.0f);
                }
                s.P = add(add(P, mul(D, best)), mul(n, PT_NUDGE));   // :313
                if (s.bounce < job.num_bounces)                    // the last direction is never used
                    s.D = normalize(add(n, random_unit_vector(s.rng)));   // :316
                s.ret = add(s.ret, mulv(v3(pr.er, pr.eg, pr.eb), s.T));   // :319
                s.T = mulv(s.T, v3(pr.ar, pr.ag, pr.ab));                // :322
                s.bounce += 1;
                done = s.bounce > job.num_bounces;
            }
            if (done) {
                // :355-356 color = 0 + c * (1/1);  :812 lerp(last, color, 1/(iFrame+1))
                const V3 col = v3(0.0f + s.ret.x * 1.0f, 0.0f + s.ret.y * 1.0f, 0.0f + s.ret.z * 1.0f);
                const float t = rcp_x(iFrame + 1.0f);
                acc = add(acc, mul(sub(col, acc), t));
                if (COUNT) ++n_samp;
                if (++sidx == job.nframes) break;
                iFrame = (float)(job.frame_first + (uint32_t)sidx);
                start_sample(s, cam, fx, fy, iFrame);
            }
        }
        px[0] = acc.x;
        px[cs] = acc.y;
        px[2 * cs] = acc.z;
    }
    if (COUNT) {
        // n_iter per lane counts this lane's iterations; the wave issued max over lanes.
        unsigned long long wave_iters = n_iter;
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(wave_iters, off, 64);
            wave_iters = o > wave_iters ? o : wave_iters;
        }
        for (int off = 32; off > 0; off >>= 1) {
            n_seg += __shfl_xor(n_seg, off, 64);
            n_samp += __shfl_xor(n_samp, off, 64);
            n_esc += __shfl_xor(n_esc, off, 64);
        }
        if (lane == 0) {
            atomicAdd(&job.counters[PT_CNT_SEGMENTS], n_seg);
            atomicAdd(&job.counters[PT_CNT_LANE_SLOTS], wave_iters);
            atomicAdd(&job.counters[PT_CNT_SAMPLES], n_samp);
            atomicAdd(&job.counters[PT_CNT_ESCAPED], n_esc);
        }
    }
}

template <int LAYOUT, bool ENV>
hipError_t launch_t(const PtJob& job, hipStream_t st, bool count)
{
    const dim3 grid((unsigned)((job.ncols + 15) / 16), (unsigned)((job.nrows + 15) / 16));
    if (count)
        hipLaunchKernelGGL((pt_render_kernel<LAYOUT, ENV, true>), grid, dim3(256), 0, st, job);
    else
        hipLaunchKernelGGL((pt_render_kernel<LAYOUT, ENV, false>), grid, dim3(256), 0, st, job);
    return hipGetLastError();
}

}  // namespace

hipError_t pt_launch_render(const PtJob& job, hipStream_t st, bool count)
{
    if (job.ncols <= 0 || job.nrows <= 0 || job.nframes <= 0) return hipSuccess;
    if (!job.scene || !job.buf) return hipErrorInvalidValue;
    switch (job.layout) {
        case PT_LAYOUT_INTERLEAVED: return launch_t<PT_LAYOUT_INTERLEAVED, false>(job, st, count);
        case PT_LAYOUT_PLANAR8: return launch_t<PT_LAYOUT_PLANAR8, false>(job, st, count);
        case PT_LAYOUT_TILED_PLANAR8: return launch_t<PT_LAYOUT_TILED_PLANAR8, false>(job, st, count);
        default: return hipErrorInvalidValue;
    }
}
