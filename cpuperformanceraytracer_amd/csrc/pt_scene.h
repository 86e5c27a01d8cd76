// pt_scene.h -- the demofox scene table as it lives on the device (kernel argument + LDS).
//
// TestSceneTrace (demofox_path_tracing_scalar.cpp:186-287) hard-codes 6 quads, 3 spheres and 9
// materials, adding sceneTranslation (0,0,10) and recomputing every quad normal on every call.
// Those are scene constants: the host evaluates them ONCE with the very same f32 operations
// (translation adds, normalize(cross(c-a, c-b)), r*r) and the kernel reads the results, so the
// per-segment arithmetic the GPU performs is exactly the reference's per-segment arithmetic.
//
// Device placement: geometry is wave-uniform (every lane tests the same primitive at the same
// time) -> kernel argument, read with scalar loads into SGPRs.  Per-hit material / normal data
// is indexed by each lane's own closest-hit id -> staged into LDS (PtLdsPrim) at kernel start.
#pragma once
#include <stdint.h>

#define PT_NQUADS 6
#define PT_NSPHERES 3
#define PT_NPRIMS (PT_NQUADS + PT_NSPHERES)

// constants of demofox_path_tracing_scalar.cpp:6-25
#define PT_MIN_HIT 0.01f       // c_minimumRayHitTime
#define PT_NUDGE 0.01f         // c_rayPosNormalNudge
#define PT_SUPER_FAR 10000.0f  // c_superFar
#define PT_FOV_DEG 90.0f       // c_FOVDegrees
#define PT_PI 3.14159265359f   // c_pi
#define PT_TWOPI (2.0f * PT_PI)

struct PtScene {
    float qv[PT_NQUADS][4][3];     // translated quad vertices a, b, c, d
    float qn[PT_NQUADS][3];        // normalize(cross(c - a, c - b))           (scalar.cpp:68)
    float sph[PT_NSPHERES][4];     // translated centre xyz, radius w
    float sph_r2[PT_NSPHERES];     // sphere.w * sphere.w                      (scalar.cpp:154)
    float albedo[PT_NPRIMS][3];
    float emissive[PT_NPRIMS][3];
    float ambient[3];              // miss radiance (scalar.cpp:307)
    float cam_dist;                // 1 / tan(c_FOVDegrees * 0.5 * c_pi / 180) (scalar.cpp:338)
};

// What a lane needs after its closest hit is known, by primitive id.
struct PtLdsPrim {
    float nx, ny, nz, pad0;        // quad: unflipped normal;  sphere: centre
    float ar, ag, ab, pad1;        // albedo
    float er, eg, eb, pad2;        // emissive
};

// The same scene as compile-time constants for the kernel's hot loop: TestSceneTrace hard-codes
// its geometry in code, and so does the device trace -- vertex coordinates become instruction
// literals / inline constants (no loads, no registers).  Translated vertices are constexpr f32
// adds (round-to-nearest, like the reference's per-call adds); the quad normals need sqrtf and
// '/', so they are written out here as the exact f32 results of normalize(cross(c-a, c-b))
// (scalar.cpp:68) -- tests/test_scene.py recomputes them with pt_build_demofox_scene and checks
// every constant of this table bit for bit.
struct DemofoxScene {
    static constexpr float T = 10.0f;   // sceneTranslation.z (scalar.cpp:189)
    static constexpr float qv[PT_NQUADS][4][3] = {
        {{-12.6f, -12.6f, 25.0f + T}, {12.6f, -12.6f, 25.0f + T}, {12.6f, 12.6f, 25.0f + T}, {-12.6f, 12.6f, 25.0f + T}},
        {{-12.6f, -12.45f, 25.0f + T}, {12.6f, -12.45f, 25.0f + T}, {12.6f, -12.45f, 15.0f + T}, {-12.6f, -12.45f, 15.0f + T}},
        {{-12.6f, 12.5f, 25.0f + T}, {12.6f, 12.5f, 25.0f + T}, {12.6f, 12.5f, 15.0f + T}, {-12.6f, 12.5f, 15.0f + T}},
        {{-12.5f, -12.6f, 25.0f + T}, {-12.5f, -12.6f, 15.0f + T}, {-12.5f, 12.6f, 15.0f + T}, {-12.5f, 12.6f, 25.0f + T}},
        {{12.5f, -12.6f, 25.0f + T}, {12.5f, -12.6f, 15.0f + T}, {12.5f, 12.6f, 15.0f + T}, {12.5f, 12.6f, 25.0f + T}},
        {{-5.0f, 12.4f, 22.5f + T}, {5.0f, 12.4f, 22.5f + T}, {5.0f, 12.4f, 17.5f + T}, {-5.0f, 12.4f, 17.5f + T}},
    };
    // x + 0.0f (the translation's x/y) is x for every finite x, so those adds are folded above.
    static constexpr float qn[PT_NQUADS][3] = {
        {0.0f, 0.0f, 1.0f}, {0.0f, 1.0f, 0.0f}, {0.0f, 1.0f, 0.0f},
        {1.0f, -0.0f, 0.0f}, {1.0f, -0.0f, 0.0f}, {0.0f, 1.0f, 0.0f},
    };
    static constexpr float sph[PT_NSPHERES][4] = {
        {-9.0f, -9.5f, 20.0f + T, 3.0f}, {0.0f, -9.5f, 20.0f + T, 3.0f}, {9.0f, -9.5f, 20.0f + T, 3.0f}};
    static constexpr float sph_r2[PT_NSPHERES] = {3.0f * 3.0f, 3.0f * 3.0f, 3.0f * 3.0f};
};

#ifndef __HIPCC_DEVICE_ONLY__
// Host-side construction (compiled with -ffp-contract=off: one rounding per op, like the
// reference).  tanf is the host libm's, like the reference's (MSVC float overload of tan()).
void pt_build_demofox_scene(PtScene* s, const float ambient[3]);
#endif
