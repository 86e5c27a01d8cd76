/* oracle/pt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, written from scratch) of the reference's scalar diffuse+emissive
 * path tracer, demofox_path_tracing_scalar.cpp (paths relative to
 * /root/reference/CPUPerformanceRayTracer/).  It is the parity checker for the HIP product path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Pinning: bit-identical to the reference's own scalar code (compiled unmodified by
 * oracle/build_ref.sh) on the committed golden fixtures in tests/golden/ (f32, xz)
 * (256x256, 1 and 8 frames, 4 bounces) -- see tests/test_oracle.py.
 *
 * Generalisations beyond the reference's compile-time constants (each is a loop bound or a
 * constant the reference hard-codes, the arithmetic is unchanged):
 *   - num_bounces           (c_numBounces, scalar.cpp:19; 4 in the reference, 8 in configs 2-5)
 *   - frame_first, nframes  (the static iFrame, scalar.cpp:798-799; nframes calls in a row)
 *   - row_start/row_stride  (render a row-interleaved shard of the image with GLOBAL pixel
 *                            coordinates, so every shard is bit-identical to the full image)
 *   - env                   (miss radiance = equirectangular env sample, the textured variant
 *                            demofox_path_tracing_simt_textured.cpp:408 -> texture.cpp:101-139;
 *                            NOT pinned by a reference run: that file needs SVML)
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct pto_env {
    const float* data;   /* Height x Width x 3 f32, row 0 = bottom (stbi flip-on-load, asset_loading.cpp:12) */
    int32_t width;
    int32_t height;
} pto_env;

typedef struct pto_params {
    int32_t width, height;        /* iResolution                                            */
    int32_t row_start;            /* first global row (Y, row 0 = top)                     */
    int32_t row_stride;           /* global row step between consecutive buffer rows       */
    int32_t nrows;                /* rows in the buffer                                     */
    uint32_t frame_first;         /* iFrame of the first accumulated frame (>= 1)           */
    int32_t nframes;              /* frames accumulated in order                            */
    int32_t num_bounces;          /* c_numBounces                                           */
    float ambient[3];             /* miss radiance when env == NULL (scalar.cpp:307: 0.1)   */
    const pto_env* env;           /* NULL => constant ambient                                */
    int32_t nthreads;             /* host threads (row-cyclic); <= 1 => single thread        */
} pto_params;

/* Flop accounting (SURVEY.md §8d convention: 1 per fp32 add/sub/mul/div/sqrt/compare executed by
 * the scalar reference; negation/abs/moves 0; frame- or scene-constant work excluded;
 * sin/cos/atan2/asin counted separately as transcendentals). */
typedef struct pto_counts {
    uint64_t samples;        /* primary samples (pixels x frames)                 */
    uint64_t segments;       /* TestSceneTrace calls                              */
    uint64_t flops_sample;   /* camera ray + accumulate, per sample               */
    uint64_t flops_segment;  /* scene trace + shading, per segment                */
    uint64_t transcendentals;
    uint64_t escaped;        /* paths that ended on a miss                        */
    uint64_t segments_primary;       /* bounce-0 (camera ray) segments            */
    uint64_t flops_segment_primary;  /* their flops (trace + bounce-0 shading)    */
    uint64_t flops_shared;   /* flops that are identical for every frame of a pixel: the camera
                                ray, its trace and its shading except the new direction (RUV +
                                normalize); a renderer may evaluate them once per pixel          */
} pto_counts;

/* Render into buf (nrows x width x 3 f32, interleaved RGB, accumulating in place).  0 on success. */
int pto_render(float* buf, const pto_params* p);
/* Same, single-threaded, counting work (slower; for deriving the roofline constants). */
int pto_render_counted(float* buf, const pto_params* p, pto_counts* counts);

/* Known-answer hooks. */
uint32_t pto_wang_hash(uint32_t* state);                  /* scalar.cpp:27-35  */
float pto_randomf(uint32_t* state);                        /* scalar.cpp:37-40  */
void pto_random_unit_vector(uint32_t* state, float out3[3]);/* scalar.cpp:42-50 */
uint32_t pto_seed(uint32_t x, uint32_t y, uint32_t frame); /* scalar.cpp:332    */
/* TestSceneTrace pieces (scalar.cpp:186-287) for the product's quad-culling check. */
float pto_trace_quads(const float P[3], const float D[3], int* id, int* flipped);
float pto_trace_scene(const float P[3], const float D[3], float n_out[3], int* id);
uint64_t pto_sky_skipped(const pto_params* p, float slope, uint64_t* flops);   /* sky tiles (pt_kernel.hip) */
void pto_env_sample(const pto_env* env, const float dir[3], float out3[3]); /* texture.cpp:101-139 */

/* Output stage (pt_oracle_output.c): ACES + fast sRGB + 8-bit pack, v4 :144-187, :1260-1331. */
#define PTO_PIXEL_RGBA8 0   /* OutputToFile:   bytes R, G, B, A = 255 (u32 0xFFBBGGRR) */
#define PTO_PIXEL_XRGB8 1   /* OutputToScreen: u32 0x00RRGGBB                          */
uint32_t pto_tonemap_channel(float linear);
uint32_t pto_tonemap_pixel(const float rgb[3], int32_t format);
void pto_tonemap(const float* rgb, int32_t w, int32_t h, int32_t format, uint32_t* out);
/* the non-default branches: exact_aces = USE_FAST_APPROXIMATE_ACES_TONEMAP 0, exact_gamma =
 * USE_FAST_APPROXIMATE_GAMMA 0 (global_preprocessor_flags.h:62-63) */
uint32_t pto_tonemap_channel_ex(float linear, int32_t exact_aces, int32_t exact_gamma);
void pto_tonemap_ex(const float* rgb, int32_t w, int32_t h, int32_t format, int32_t exact_aces, int32_t exact_gamma,
                    uint32_t* out);

/* ---- v4 renderer (pt_oracle_v4.c): demofox_path_tracing_optimization_v4.cpp restated ---------- */
#define PTO4_MAX_OBJECTS 12      /* MAX_OBJECTS / MAX_MATERIALS, v4 :351-352 (quads + spheres <= 12) */
#define PTO4_ENV_NONE 0          /* USE_ENV_MAP 0: ambient (0.11, 0.1, 0.15), v4 :782            */
#define PTO4_ENV_EQUIRECT 1      /* USE_ENV_MAP 1, USE_ENV_CUBEMAP 0 (flags.h:58-59, default)     */
#define PTO4_ENV_CUBEMAP 2       /* USE_ENV_CUBEMAP 1: six faces stacked (LoadCubemapTexture)     */

typedef struct pto4_material {   /* SceneMaterial, v4 :367-378 */
    float albedo[3], emissive[3];
    float spec_chance, spec_rough, spec_color[3];
    float ior, refr_chance, refr_rough, refr_color[3];
} pto4_material;

typedef struct pto4_scene {      /* the arguments of AddQuad/Sphere/MaterialToScene, in call order */
    int32_t nquads, nspheres, nmat;
    float quad[PTO4_MAX_OBJECTS][4][3];   /* V0..V3, already translated (v4 :1415-1418)          */
    float sphere[PTO4_MAX_OBJECTS][4];    /* PositionAndRadius                                   */
    pto4_material mat[PTO4_MAX_OBJECTS];  /* object index order: quads first, then spheres       */
} pto4_scene;

typedef struct pto4_params {
    int32_t width, height, row_start, row_stride, nrows;
    uint32_t frame_first;         /* the static iFrame of the first frame (>= 1)                 */
    int32_t nframes;
    int32_t num_bounces;          /* c_numBounces, v4 :23 (8)                                    */
    int32_t env_mode;             /* PTO4_ENV_*                                                  */
    int32_t random_jitter;        /* USE_RANDOM_JITTER_TEXTURE_SAMPLING (1) else bilinear         */
    int32_t rejection;            /* USE_UNIT_VECTOR_REJECTION_SAMPLING (1) else sin/cos          */
    const pto_env* env;           /* equirect map or stacked cubemap; NULL => ambient             */
    int32_t nthreads;
    int32_t no_accumulate;        /* ACCUMULATE_FRAMES 0 (flags.h:60): store each frame's colour   */
    int32_t exact_exp;            /* USE_FAST_APPROXIMATE_EXP 0 (flags.h:64): expf for exp_ps      */
} pto4_params;

typedef struct pto4_counts {
    uint64_t samples, segments, escaped;
    uint64_t flops;             /* executed f32 FLOP (convention in pt_oracle_v4.c)          */
    uint64_t transcendentals;   /* atan2f/asinf/sinf/cosf calls                              */
} pto4_counts;

void pto4_default_scene(pto4_scene* s);   /* InitializeScene, v4 :1403-1496 */
/* Render into buf (nrows x width x 3 f32, interleaved, accumulating in place); scene NULL =>
 * the default scene; counts (optional) forces one thread.  0 on success. */
int pto4_render(float* buf, const pto4_params* p, const pto4_scene* scene, pto4_counts* counts);
int pto4_scene_tables(const pto4_scene* scene, float* out, int32_t n);
float pto4_trace_scene(const pto4_scene* scene, const float P[3], const float D[3], int* mat);   /* v4 :700-718 */
float pto4_trace_scene_flops(const pto4_scene* scene, const float P[3], const float D[3], int* mat, uint64_t* flops);
float pto4_randomf(uint32_t* state);                                          /* mathutils.h:18-26 */
void pto4_random_unit_vector(uint32_t* state, int rejection, float out[3]);   /* v4 :109 / mathutils.h:33 */
void pto4_env_sample(const pto_env* env, int32_t env_mode, int32_t random_jitter, const float dir[3],
                     uint32_t* state, float out[3]);                          /* v4 :769-784 */

#ifdef __cplusplus
}
#endif
#endif
