// pt_v4.h -- the v4 renderer (demofox_path_tracing_optimization_v4.cpp, the reference's shipping
// path, Application.cpp:474): scene tables, launch interface, host scene builder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_V4_MAX_OBJECTS 12   // MAX_OBJECTS / MAX_MATERIALS, v4 :351-352

// env modes (global_preprocessor_flags.h:58-59)
#define PT_V4_ENV_NONE_ 0       // USE_ENV_MAP 0: ambient (0.11, 0.1, 0.15), v4 :782
#define PT_V4_ENV_EQUIRECT_ 1   // USE_ENV_MAP 1, USE_ENV_CUBEMAP 0 (default)
#define PT_V4_ENV_CUBEMAP_ 2    // USE_ENV_CUBEMAP 1 (six faces stacked, LoadCubemapTexture)

// QuadSceneObject after PrecomputeQuadData (v4 :256-320): only what TestQuadTrace (:556-637) reads.
struct PtV4Quad {
    float v0[3];
    float n[3];    // normalize(cross(V01, V02))
    float a0[3];   // NxV01 / DetBot   (bottom triangle 0,1,2)
    float a1[3];   // NxV20 / DetBot
    float b0[3];   // NxV30 / DetTop   (top triangle 0,2,3)
    float b1[3];   // NxV02 / DetTop
};

// One row of SceneMaterialSOA (v4 :354-373) as GatherMaterials (:389-427) reads it: 17 f32.
struct PtV4Mat {
    float albedo[3], emissive[3];
    float spec_chance, spec_rough, spec_color[3];
    float ior, refr_chance, refr_rough, refr_color[3];
};
static_assert(sizeof(PtV4Mat) == 17 * sizeof(float), "material row");

struct PtV4Scene {
    int32_t nquads, nspheres;
    PtV4Quad quad[PT_V4_MAX_OBJECTS];
    float sph[PT_V4_MAX_OBJECTS][4];     // PositionAndRadius
    PtV4Mat mat[PT_V4_MAX_OBJECTS];      // by object index (quads first); unused rows zero
};

struct PtV4Job {
    float* buf;                 // device accumulator
    int32_t width, height;      // iResolution
    int32_t col0, ncols;        // pixel columns [col0, col0 + ncols)
    int32_t row_start, row_stride, nrows;
    int32_t layout;             // PtLayout (pt_kernel.h)
    int32_t tile_w, tile_h;     // PT_LAYOUT_TILED_PLANAR8
    uint32_t frame_first;       // iFrame of the first frame (>= 1)
    int32_t nframes;
    int32_t num_bounces;        // c_numBounces (8)
    int32_t env_mode;           // PT_V4_ENV_*_
    int32_t random_jitter;      // USE_RANDOM_JITTER_TEXTURE_SAMPLING
    int32_t rejection;          // USE_UNIT_VECTOR_REJECTION_SAMPLING
    int32_t accumulate;         // ACCUMULATE_FRAMES: fused lerp into the accumulator (else store)
    int32_t fast_exp;           // USE_FAST_APPROXIMATE_EXP: approx_exp_ps (else glibc-exact expf)
    const float* env;           // device texture (H x W x 3), nullptr with PT_V4_ENV_NONE_
    int32_t env_w, env_h;
    unsigned long long* counters;   // COUNT launches: [0] segments, [1] samples, [2] escaped, [3] lane slots
    int32_t default_scene;          // the scene is InitializeScene's: literal-geometry instantiation
    // persistent-grid tile queue and schedule (pt_tile_queue.h; as PtJob, pt_kernel.h)
    unsigned int* queue;            // PT_QUEUE_WORDS words, zero at the launch's start
    unsigned int* queue_next;       // the next launch's words, zeroed by this launch (nullptr: none)
    const uint32_t* order;          // tile schedule (longest first) or nullptr
    const uint32_t* units;
    const uint32_t* nunits;
    uint32_t* cost;                 // per-tile cost written by this launch, or nullptr
    uint32_t* err;                  // PT_ERR_WORDS error words (pt_kernel.h), nullptr = not recorded
    // continuous-tiles pool (pt_v4.hip pt_v4_ct_kernel): pt_ct_wave_floats() f32 per wave for ct_waves
    // waves (the diffuse kernels' slot area, pt_kernel.h); nullptr: the per-tile pool kernel
    float* ct_slots;
    uint32_t ct_waves;
    int32_t ct_force;               // 1: the continuous-tiles kernel for every launch of >= 8 frames (tests)
    uint32_t ct_back_pct;           // the CT kernel: the last-dispatched ct_back_pct % of the grid claims
                                    // its units from the back of its queue group (pt_tile_queue.h)
    // fused output stage (OutputToScreen / OutputToFile after RenderTile, v4 :1562-1564): each
    // pixel's 8-bit value at pix_out[Y * width + X] (full-image rows, the screen's layout), written
    // with its final accumulator value; nullptr: none.  pix_fast_tone: the tonemap flags are the
    // default fast ACES / gamma (the only ones the presenting kernels carry)
    uint32_t* pix_out;
    int32_t pix_xrgb;               // PT_PIXEL_XRGB8 (OutputToScreen) else RGBA8 (OutputToFile)
    int32_t pix_fast_tone;
    // chained launches (pt_v4_render_device_chain): as PtJob's (pt_kernel.h) -- the continuous-tiles
    // kernel only
    uint32_t* tile_epoch;
    uint32_t chain_seq;
    uint32_t chain_wait;
    unsigned long long* started;
    uint32_t chain_delay;
};

// Scene description in AddQuad/Sphere/MaterialToScene order (v4 :1368-1401).
struct PtV4SceneDesc {
    int32_t nquads, nspheres, nmat;
    float quad[PT_V4_MAX_OBJECTS][4][3];
    float sphere[PT_V4_MAX_OBJECTS][4];
    PtV4Mat mat[PT_V4_MAX_OBJECTS];   // as passed to AddMaterialToScene (before its albedo.x copy)
};

void pt_v4_default_scene_desc(PtV4SceneDesc* d);                   // InitializeScene, v4 :1403-1496
int pt_v4_build_scene(const PtV4SceneDesc* d, PtV4Scene* out);     // PrecomputeQuadData + AddMaterialToScene
bool pt_v4_is_default_geometry(const PtV4Scene& s);                // geometry == pt_v4_default_scene.h
// *presented (optional): the launch also wrote job.pix_out (the fused output stage; only for the
// presenting configuration, pt_v4.hip pt_launch_v4 -- otherwise the caller converts separately)
// *ct_blocks (optional): the grid of the continuous-tiles kernel it launched (0: the per-tile pool, or
// nothing launched) -- a chained launch's gate waits for that many started blocks.
// (as pt_set_chain_polls, for the v4 kernels)
hipError_t pt_v4_set_chain_polls(uint32_t polls);
hipError_t pt_launch_v4(const PtV4Job& job, const PtV4Scene& scene, hipStream_t stream, bool count,
                        bool* presented = nullptr, uint32_t* ct_blocks = nullptr);
