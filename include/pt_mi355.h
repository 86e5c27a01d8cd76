/* include/pt_mi355.h -- C ABI of the MI355X (gfx950) path-tracing backend, libpt_mi355.so.
 *
 * Drop-in boundary for the reference's per-pixel path-tracing hot path
 * (torgeiba/CPUPerformanceRayTracer; file:line below are relative to CPUPerformanceRayTracer/).
 * Plain C types only: pointers, sizes, POD structs.  Every function returns PT_OK (0) or a
 * negative PT_E* code; pt_last_error() then describes the failure (the reference has no error
 * returns -- it __debugbreak()s, Application.cpp:59,69,79,89 -- see the C++ wrappers in
 * demofox_path_tracing_mi355.h for the reference-shaped, abort-on-error surface).
 *
 * Semantics: results are bit-identical to the reference's scalar path
 * (demofox_path_tracing_scalar.cpp) for the same (pixel, frame): same Wang-hash seed, same f32
 * operations in the same order, glibc-identical sinf/cosf.  Frame state mirrors the reference's
 * `static f32 iFrame` (scalar.cpp:798-799): each frame call first increments it, then renders
 * with it; the first call renders frame 1.
 *
 * Threading: like the reference (static state, not re-entrant) -- call from one host thread.
 * Devices: one or several GPUs per process (pt_config.device_count / PT_MI355_DEVICES); entry points
 * restore the caller's current HIP device before they return.
 */
#ifndef PT_MI355_H
#define PT_MI355_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_EINVAL (-1)   /* invalid argument / settings (CheckValidSettings, Application.cpp:36-94) */
#define PT_EHIP (-2)     /* HIP runtime error (no device, launch failure, ...)                     */
#define PT_ENOMEM (-3)   /* device allocation failed                                               */
#define PT_ESTATE (-4)   /* call out of order (e.g. readback without a deferred buffer)            */
#define PT_EKERNEL (-5)  /* a kernel abandoned work (the ring pool's iteration guard fired on a    */
                         /* tile): the accumulator it wrote is invalid; pt_last_error names the tile */

/* Buffer layouts written by the reference's three frame functions. */
#define PT_LAYOUT_INTERLEAVED 0    /* DemofoxRenderScalar: RGB of pixel (X,Y) at 3*(Y*W+X)+c          */
#define PT_LAYOUT_PLANAR8 1        /* DemofoxRenderSimd (simd.cpp:496-511): per row, per 8 pixels    */
                                   /*   [R0..R7][G0..G7][B0..B7]                                      */
#define PT_LAYOUT_TILED_PLANAR8 2  /* RenderTile (simd_tiled.cpp:499-531): tile-major, planar8 rows   */

#define PT_FLAG_DEFER_READBACK 1u  /* keep the accumulator in HBM between frame calls: no H2D/D2H;    */
                                   /* the host buffer is refreshed by pt_readback(), or written back */
                                   /* automatically when a call names a different buffer (the device */
                                   /* mirror holds one buffer at a time).  pt_shutdown discards it.  */
                                   /* Call pt_release_buffer(buf) before freeing or reallocating a   */
                                   /* deferred buffer (its device copy is dropped, never written to  */
                                   /* freed memory); ReinitializeRenderTileData does it for Resize.  */
#define PT_FLAG_PIN_HOST 2u        /* page-lock the caller's frame buffer (hipHostRegister; kept until */
                                   /* pt_unpin_host, pt_shutdown, ReinitializeRenderTileData or      */
                                   /* another buffer is passed) and overlap its PCIe transfers with  */
                                   /* rendering, in row bands (same results) -- frame calls, and work */
                                   /* queues whose entries are a whole frame of tiles of one buffer. */
                                   /* Free a pinned buffer only after pt_unpin_host(buf) or          */
                                   /* pt_release_buffer(buf) (a Resize that reallocates it): the     */
                                   /* registration of a freed buffer cannot be detected reliably.    */
                                   /* One device only (several devices: the plain path).             */
#define PT_FLAG_GATHER_ROOT 4u     /* several devices + PT_FLAG_DEFER_READBACK: the output stage    */
                                   /* (pt_tonemap, v4 screen pixels, CopyOutputToFile) and            */
                                   /* pt_readback first assemble the whole accumulator on the root    */
                                   /* device (devices[0]): every device stores its rows there over     */
                                   /* xGMI (peer access), the root converts / copies it once.  Off:   */
                                   /* each device converts and copies its own rows over its own PCIe  */
                                   /* link (faster for a host consumer).         */

#define PT_MAX_DEVICES 16

/* Runtime form of the reference's compile-time configuration (global_preprocessor_flags.h and the
 * file-scope constants of demofox_path_tracing_scalar.cpp:6-25). */
typedef struct pt_config {
    int32_t device;              /* HIP device ordinal (device_count <= 1)                         */
    int32_t num_bounces;         /* c_numBounces (scalar.cpp:19); reference default 4              */
    int32_t samples_per_frame;   /* NUM_SAMPLES_PER_FRAME (flags.h:30): frames accumulated per call */
    uint32_t flags;              /* PT_FLAG_*                                                      */
    float ambient[3];            /* miss radiance (scalar.cpp:307), reference default 0.1          */
    /* Several GPUs in one process (the reference fans a frame's tiles out over NUM_THREADS CPU
     * threads, simd_tiled.cpp:549-571, v4 :1696-1721): with device_count > 1 every host-buffer entry
     * point deals the frame's rows to devices[0..device_count) -- row Y to devices[Y % device_count]
     * -- and each device mirrors its own rows; results are bit-identical to one device.  An ordinal
     * may repeat (logical shards of one GPU).  pt_default_config fills these from the environment
     * variable PT_MI355_DEVICES ("all" or "0,1,2,3"; unset: device 0), so a reference host that
     * never calls pt_init drives several GPUs unchanged.  Device jobs run on the device holding
     * their buffer. */
    int32_t device_count;        /* 0 or 1: `device` alone                                         */
    int32_t devices[PT_MAX_DEVICES];
} pt_config;

/* Mirrors of RenderBufferInfo / RenderTileInfo (demofox_path_tracing_simd_tiled.cpp:473-487). */
typedef struct pt_buffer_info {
    float* data;                 /* BufferDataPtr (host memory, W*H*NumChannels f32)               */
    int32_t width, height, num_channels;
} pt_buffer_info;

typedef struct pt_tile_info {
    int32_t tile_x, tile_y;
    int32_t tile_width, tile_height;
    int32_t tile_min_x, tile_max_x;
    int32_t tile_min_y, tile_max_y;
} pt_tile_info;

/* Mirror of `texture` (texture.h:6-12): height x width x components f32, row 0 = the image's
 * bottom row (LoadTexture flips on load, asset_loading.cpp:12).  The env map of config 4. */
typedef struct pt_texture {
    float* data;
    int32_t width, height;
    int32_t components;          /* 3 (stbi_loadf of an .hdr always yields RGB)                    */
} pt_texture;

/* Device-resident job: the buffer already lives in HBM (bench, multi-GPU shards).  Renders the
 * global rows Y = row_start + k*row_stride, k in [0, nrows), of a width x height image into a
 * compact buffer of nrows rows, accumulating frames frame_first .. frame_first+nframes-1. */
typedef struct pt_device_job {
    float* buf;                  /* device pointer                                                  */
    int32_t width, height;
    int32_t row_start, row_stride, nrows;
    int32_t layout;              /* PT_LAYOUT_INTERLEAVED or PT_LAYOUT_PLANAR8                      */
    uint32_t frame_first;        /* >= 1                                                            */
    int32_t nframes;
    int32_t num_bounces;
    int32_t use_env;             /* 0: ambient miss term; 1: the env map set by pt_set_env_map      */
} pt_device_job;

/* Work counters of pt_count_device(). */
typedef struct pt_work_counts {
    uint64_t segments;           /* TestSceneTrace calls traced (camera rays once per pixel)        */
    uint64_t lane_slots;         /* 64 x loop iterations issued per wave, summed over waves        */
    uint64_t samples;            /* primary samples (pixels x frames)                              */
    uint64_t escaped;            /* paths that ended on a miss                                     */
    uint64_t primary;            /* camera-ray segments traced (= pixels rendered)                 */
    uint64_t quad_fallbacks;     /* segments whose culled quad stage was not certified, so the six */
                                 /* exact quad tests ran (diffuse kernel; pt_quadcull.h)           */
    uint64_t sphere_fallbacks;   /* segments whose closest-sphere stage fell back to the sequential */
                                 /* sphere tests (v4 kernel, default scene)                        */
    uint64_t sky_skipped;        /* camera-ray segments (counted in `segments`) whose TestSceneTrace */
                                 /* was skipped because the whole tile/iteration was sky           */
} pt_work_counts;

/* --- lifecycle -------------------------------------------------------------------------------- */
int pt_init(const pt_config* cfg);            /* NULL => defaults; (re)initialises the backend      */
void pt_shutdown(void);
const char* pt_last_error(void);
void pt_default_config(pt_config* cfg);
int pt_set_frame(uint32_t frame);             /* set the static iFrame value (next call: frame+1)  */
uint32_t pt_get_frame(void);

/* --- drop-in frame entry points (host buffers; synchronous: the buffer is updated on return) --- */
/* replaces DemofoxRenderScalar, demofox_path_tracing_scalar.h:7 / .cpp:785-820 */
int pt_render_scalar(float* buf, int32_t width, int32_t height, int32_t num_channels);
/* replaces DemofoxRenderSimd, demofox_path_tracing_simd.h:7 / .cpp:468-514 (planar8 layout) */
int pt_render_simd(float* buf, int32_t width, int32_t height, int32_t num_channels);
/* replaces DemofoxRenderSimdTiled, demofox_path_tracing_simd_tiled.h:7 / .cpp:537-574 */
int pt_render_simd_tiled(float* buf, int32_t width, int32_t height, int32_t num_tiles_x, int32_t num_tiles_y,
                         int32_t tile_width, int32_t tile_height, int32_t num_channels);
/* replaces RenderTile, demofox_path_tracing_simd_tiled.cpp:489-535 (renders at the current frame,
 * does not advance it; only the tile's contiguous slice of the buffer is transferred) */
int pt_render_tile(const pt_buffer_info* buffer, const pt_tile_info* tile);
/* advance the frame counter once (DemofoxRenderSimdTiled :547) without rendering -- for hosts that
 * fan RenderTile calls out themselves (the v4 / simt_pooled pattern) */
int pt_begin_frame(void);
/* PT_FLAG_DEFER_READBACK: copy the device accumulator of `buf` back into it */
int pt_readback(float* buf);
/* PT_FLAG_DEFER_READBACK: the accumulator of `buf` assembled in the root device's HBM (devices[0];
 * several devices: gathered over xGMI as for PT_FLAG_GATHER_ROOT).  *device_accum = a library-owned
 * W x H x 3 f32 buffer in buf's layout, valid until the next call; synchronous. */
int pt_gather_root(const float* buf, const float** device_accum);
/* PT_FLAG_PIN_HOST: drop the page-lock of `buf` (NULL: of whichever buffer is pinned) before the
 * caller frees or reallocates it (Application.cpp:142-151 Resize).  No-op if it is not pinned. */
int pt_unpin_host(const void* buf);
/* The caller is about to free or reallocate `buf` (NULL: whichever buffer): forget every device-side
 * association -- the PT_FLAG_DEFER_READBACK device copy (dropped, NOT written back) and the
 * PT_FLAG_PIN_HOST page-lock.  Mandatory before freeing a deferred or pinned buffer. */
int pt_release_buffer(const void* buf);
/* the (first) HIP device the library state lives on, or -1 before pt_init (a device job on a device
 * the library was not initialised with is an error, not a re-initialisation) */
int32_t pt_initialized_device(void);
/* Device-resident jobs (pt_render_device, ...) return when launched.  After synchronising the streams
 * they ran on, this reports PT_EKERNEL if any launch since the last check abandoned a tile (every
 * host-buffer entry point makes the same check before it returns). */
int pt_check_device_errors(void);
/* 1 if this library is the bounds-checked diagnostic build (-DPT_CHECKED=1: every global index of the
 * continuous-tiles pools and the schedule builder is tested and reported as PT_EKERNEL), else 0 */
int32_t pt_build_checked(void);
int32_t pt_device_count(void);               /* logical devices (0 before pt_init)             */
int32_t pt_device_ordinal(int32_t index);    /* HIP ordinal of logical device `index`, or -1    */

/* --- env map (config 4: miss radiance = EquirectangularTextureSample, texture.cpp:101-139) ----- */
/* replaces LoadTexture, asset_loading.cpp:9-16 (Radiance RGBE .hdr, flipped vertically) */
int pt_load_texture(const char* path, pt_texture* out);
int pt_decode_hdr(const void* bytes, size_t nbytes, pt_texture* out);   /* same, from memory */
void pt_free_texture(pt_texture* tex);
/* replaces LoadCubemapTexture (asset_loading.h:7, .cpp:18-44): six .hdr faces (px nx py ny pz nz)
 * stacked vertically into one width x 6*height texture (the layout the cubemap samplers index) */
int pt_load_cubemap_texture(const char* const paths[6], pt_texture* out);
/* copy `tex` into HBM as the env map of device jobs with use_env (NULL: release it) */
int pt_set_env_map(const pt_texture* tex);
/* replaces DemofoxRenderSimtTextured, demofox_path_tracing_simt_textured.h:8 / .cpp:560-620:
 * the tiled frame call with the env-map miss term (tile layout of RenderTile :491-533).  The
 * texture is uploaded when its (data, width, height) differ from the previous call's. */
int pt_render_simt_textured(float* buf, int32_t width, int32_t height, int32_t num_tiles_x, int32_t num_tiles_y,
                            int32_t tile_width, int32_t tile_height, int32_t num_channels, const pt_texture* tex);

/* --- output stage: ACES + sRGB + 8-bit pack, BMP ---------------------------- */
#define PT_PIXEL_RGBA8 0   /* OutputToFile   (v4 :1297-1331): bytes R, G, B, A = 255 (u32 0xFFBBGGRR) */
#define PT_PIXEL_XRGB8 1   /* OutputToScreen (v4 :1260-1295): u32 0x00RRGGBB                          */
/* replaces the post-process of OutputToScreen / OutputToFile (demofox_path_tracing_optimization_v4.cpp
 * :1260-1331, ACESFilm :165-175, LinearToSRGB :177-186): accumulator (host buffer in `layout`,
 * tile sizes for PT_LAYOUT_TILED_PLANAR8) -> width*height packed pixels, row 0 = top.  The
 * HBM-resident accumulator is used directly when `accum` is the PT_FLAG_DEFER_READBACK buffer. */
int pt_tonemap(const float* accum, int32_t width, int32_t height, int32_t layout, int32_t tile_width,
               int32_t tile_height, uint32_t* out, int32_t format);
int pt_tonemap_device(const float* accum, int32_t width, int32_t height, int32_t layout, int32_t tile_width,
                      int32_t tile_height, uint32_t* out, int32_t format, void* hip_stream);   /* async */
/* replaces WriteImage (asset_loading.h:8, .cpp:48-54: stbi_write_bmp, 24-bit BMP) */
int pt_write_bmp(const char* path, int32_t width, int32_t height, int32_t components, const void* data);

/* --- v4 renderer: the reference's shipping path -------------------------------
 * demofox_path_tracing_optimization_v4.cpp, called by ApplicationState::Render (Application.cpp:474):
 * diffuse / specular / refraction materials (Fresnel-Schlick, Beer absorption, roughness), Russian-
 * roulette throughput boost, jittered camera, throughput-weighted env map.  Its own frame counter
 * (the file's `static f32 iFrame`, v4 :34) and scene (v4 :1403-1496, editable through the Add*
 * functions).  Results are bit-identical to oracle/pt_oracle_v4.c, which restates v4 with the exact
 * 1/x and 1/sqrtf(x) for the x86 rcp/rsqrt approximations and glibc atan2f/asinf/sinf/cosf for SVML. */
#define PT_V4_ENV_NONE 0        /* USE_ENV_MAP 0: ambient (0.11, 0.1, 0.15), v4 :782             */
#define PT_V4_ENV_EQUIRECT 1    /* USE_ENV_MAP 1, USE_ENV_CUBEMAP 0 (global_preprocessor_flags.h:58-59) */
#define PT_V4_ENV_CUBEMAP 2     /* USE_ENV_CUBEMAP 1: six faces stacked vertically (LoadCubemapTexture,  */
                                /*   asset_loading.cpp:18-44, order px nx py ny pz nz)                  */
#define PT_V4_MAX_OBJECTS 12    /* MAX_OBJECTS / MAX_MATERIALS (v4 :351-352): quads + spheres <= 12     */

/* Runtime form of the v4 compile-time switches (global_preprocessor_flags.h, v4 :23). */
typedef struct pt_v4_config {
    int32_t env_mode;            /* PT_V4_ENV_*; default PT_V4_ENV_EQUIRECT                               */
    int32_t random_jitter;       /* USE_RANDOM_JITTER_TEXTURE_SAMPLING (1) else bilinear texel sampling     */
    int32_t rejection;           /* USE_UNIT_VECTOR_REJECTION_SAMPLING (1) else RandomUnitVector_ps (sin/cos) */
    int32_t num_bounces;         /* c_numBounces (v4 :23): 8                                                */
    int32_t output_to_screen;    /* OUTPUT_TO_SCREEN (flags.h:60, 1): DemofoxRenderOptV4 also writes the    */
                                 /*   ScreenBufferData pixels (OutputToScreen v4 :1260-1295) when non-NULL  */
    int32_t accumulate_frames;   /* ACCUMULATE_FRAMES (flags.h:60, 1): the progressive fused lerp into the  */
                                 /*   accumulator (RenderTile v4 :1199-1241); 0 stores each frame's colour  */
    int32_t fast_aces;           /* USE_FAST_APPROXIMATE_ACES_TONEMAP (flags.h:63, 1): ACESFilm by rcp of   */
                                 /*   the fused denominator (v4 :168-171); 0: unfused ops and '/' (:172-174) */
    int32_t fast_gamma;          /* USE_FAST_APPROXIMATE_GAMMA (flags.h:62, 1): fast_pow_gamma (v4 :144-155, */
                                 /*   :182-183); 0: pow(x, 1/2.4) (:184-185, SVML pow_ps -> glibc powf)      */
    int32_t fast_exp;            /* USE_FAST_APPROXIMATE_EXP (flags.h:64, 1): Beer absorption by           */
                                 /*   approx_exp_ps (v4 :783-784, :971-972); 0: exp_ps (SVML -> glibc expf) */
} pt_v4_config;

/* SceneMaterial (v4 :367-378), the argument of AddMaterialToScene. */
typedef struct pt_v4_material {
    float albedo[3], emissive[3];
    float specular_chance, specular_roughness, specular_color[3];
    float ior, refraction_chance, refraction_roughness, refraction_color[3];
} pt_v4_material;

void pt_v4_default_config(pt_v4_config* cfg);
int pt_v4_set_config(const pt_v4_config* cfg);
int pt_v4_get_config(pt_v4_config* cfg);
/* InitializeGlobalRenderResources (v4 :1640-1661): camera + InitializeScene on first use */
int pt_v4_initialize_global_render_resources(void);
/* ReinitializeRenderTileData (v4 :1723-1726), called by the host's Resize (Application.cpp:154)
 * after it reallocated the render target: drops the PT_FLAG_PIN_HOST page-lock of the old buffer
 * (every pt_render_opt_v4 call uses its own arguments) */
int pt_v4_reinitialize_render_tile_data(void);
/* scene editing: the reference's InitializeScene / AddMaterialToScene / AddQuadObjectToScene /
 * AddSphereObjectToScene (v4 :1403, :1368, :1390, :1397) plus an explicit clear.  Material i shades
 * object i (quads first, then spheres: TestSceneTrace v4 :700-718). */
int pt_v4_initialize_scene(void);                     /* the default scene (replaces the current one)   */
int pt_v4_clear_scene(void);
int pt_v4_add_material(const pt_v4_material* m);      /* returns its index (>= 0) or PT_E*              */
int pt_v4_add_quad(const float vertices[12]);         /* V0..V3 xyz; returns the quad count or PT_E*    */
int pt_v4_add_sphere(const float position_radius[4]); /* returns the quad count (as v4 :1400) or PT_E*  */
int pt_v4_set_frame(uint32_t frame);
uint32_t pt_v4_get_frame(void);
/* introspection: the current scene's precomputed tables (PrecomputeQuadData v4 :269-320 +
 * AddMaterialToScene :1368-1388): per quad V0, normal, NxV01/DetBot, NxV20/DetBot, NxV30/DetTop,
 * NxV02/DetTop (18 f32), per sphere x y z r (4 f32), then PT_V4_MAX_OBJECTS material rows (17 f32,
 * pt_v4_material order).  Returns the number of floats written (or needed, when n is too small),
 * with *nquads / *nspheres set; PT_E* on error. */
int pt_v4_get_scene_tables(float* out, int32_t n, int32_t* nquads, int32_t* nspheres);
/* replaces DemofoxRenderOptV4 (v4 .h:14, .cpp:1696-1721): advance iFrame, render every tile into the
 * tiled accumulator (RenderTile v4 :1179-1258 layout), then (output_to_screen, screen != NULL) write
 * width*height XRGB8 pixels into `screen`.  tex may be NULL with PT_V4_ENV_NONE. */
int pt_render_opt_v4(float* buf, int32_t width, int32_t height, int32_t num_tiles_x, int32_t num_tiles_y,
                     int32_t tile_width, int32_t tile_height, int32_t num_channels, const pt_texture* tex,
                     void* screen);
/* replaces CopyOutputToFile (v4 .h:19, .cpp:1729-1760): iFrame += 1 (:1738), then the tiled
 * accumulator -> width*height RGBA8 file pixels (OutputToFile :1297-1331) */
int pt_copy_output_to_file(const float* buf, int32_t width, int32_t height, int32_t num_tiles_x,
                           int32_t num_tiles_y, int32_t tile_width, int32_t tile_height, int32_t num_channels,
                           void* file_pixels);
/* advance v4's iFrame once without rendering (the `iFrame += 1.0f` of DemofoxRenderOptV4 :1703) -- for
 * hosts that queue the frame's tiles themselves (pt_make_work_queue(PT_RENDERER_V4)) */
int pt_v4_begin_frame(void);
/* HBM-resident v4 job (bench / shards): the interleaved or planar8 layout; use_env selects the
 * config's env mode with the map of pt_set_env_map (else the ambient); num_bounces from the job */
int pt_v4_render_device(const pt_device_job* job, void* hip_stream);
/* pt_v4_render_device for consecutive launches of one geometry: may overlap the previous chained launch
 * of that geometry on this stream, same result (the contract of pt_render_device_chain) */
int pt_v4_render_device_chain(const pt_device_job* job, void* hip_stream);
int pt_v4_count_device(const pt_device_job* job, void* hip_stream, pt_work_counts* out);   /* sync */

/* --- tile work queue: the host tile scheduler, on the GPU ------------------------
 * Replaces work_queue.cpp (MakeWorkQueue :84-108, AddWorkQueueEntry :37-56, CompleteAllWork :63-71) for
 * its one use by the renderers: a frame's RenderTile entries (simd_tiled.cpp:549-571, simt_pooled,
 * v4 :1696-1721, DoWorkerThreadWork :1350-1358).  Entries only record (buffer, tile); completion renders
 * them all at the renderer's CURRENT frame (pt_begin_frame / pt_v4_begin_frame advance it): a queue
 * holding every tile of a buffer becomes ONE launch over the frame with one upload and one download,
 * otherwise one launch per tile, back to back on one stream.  Results equal one RenderTile call per
 * entry.  Not thread-safe (one host thread, like the rest of the library). */
#define PT_RENDERER_SIMD_TILED 0      /* RenderTile of demofox_path_tracing_simd_tiled.cpp:489-535      */
#define PT_RENDERER_SIMT_TEXTURED 1   /* its env-map variant (simt_textured.cpp:491-533; pt_set_env_map)  */
#define PT_RENDERER_V4 2              /* RenderTile of optimization_v4.cpp:1179-1258 (pt_v4_set_config)   */
typedef struct pt_work_queue pt_work_queue;
pt_work_queue* pt_make_work_queue(int32_t renderer);          /* NULL on error (pt_last_error)          */
int pt_add_work_queue_entry(pt_work_queue* q, const pt_buffer_info* buffer, const pt_tile_info* tile);
int pt_complete_all_work(pt_work_queue* q);                    /* render every entry, wait, empty queue  */
/* enqueue the same work and return: the host buffers are updated once pt_wait_work returns (keep them
 * alive and untouched meanwhile) -- a progressive host presents frame k while frame k+1 renders */
int pt_complete_all_work_async(pt_work_queue* q);
int pt_wait_work(pt_work_queue* q);
int32_t pt_work_queue_size(const pt_work_queue* q);
void pt_free_work_queue(pt_work_queue* q);

/* --- device-resident entry points -------------------------------------------------------------- */
int pt_render_device(const pt_device_job* job, void* hip_stream);      /* async on hip_stream     */
/* pt_render_device for a progressive renderer's consecutive launches of one geometry: the launch may
 * run overlapped with the previous pt_render_device_chain launch of that geometry on this stream (on
 * two streams of the library's; the next launch's waves fill the CUs where the previous launch's last
 * waves end), with every pixel's frames still accumulated in order -- bit for bit the result of
 * pt_render_device.  The launch does not wait for work enqueued on hip_stream since the previous
 * chained call: such work must not read or write the buffer unless it has completed before this call
 * (the caller synchronised), else make this call a plain pt_render_device.  Anything the caller
 * enqueues on hip_stream after this call is ordered after the launch, as with pt_render_device.
 * Any other launch on the device (another geometry, pt_render_device, counting, v4, host-buffer
 * calls) ends the overlap: the next chained call then waits for hip_stream as pt_render_device does.
 * Async on hip_stream. */
int pt_render_device_chain(const pt_device_job* job, void* hip_stream);
/* pt_render_device_chain launches since pt_init that restarted the overlap (waited for hip_stream as
 * pt_render_device does) and that continued it (overlapped with their predecessor).  Host state. */
int pt_chain_counts(uint64_t* restarts, uint64_t* continued);
int pt_count_device(const pt_device_job* job, void* hip_stream, pt_work_counts* out); /* sync;    */
                                  /* renders like pt_render_device AND counts the work it did     */
/* pt_render_device with the output stage fused into the render (the
 * per-frame OutputToScreen / OutputToFile of demofox_path_tracing_optimization_v4.cpp :1260-1331 with
 * the reference's default USE_FAST_APPROXIMATE_ACES_TONEMAP / _GAMMA 1): besides accumulating, every
 * pixel of the job's rows is converted to its packed 8-bit value (PT_PIXEL_*) in `pixels` (device
 * memory on the job's device, nrows x width u32, row k = the job's row k) by the render kernel itself,
 * where the pixel's final accumulator value is -- no second pass over the accumulator.  Equal bit for
 * bit to pt_render_device followed by pt_tonemap_device on the job's rows.  Async on hip_stream. */
int pt_render_device_present(const pt_device_job* job, uint32_t* pixels, int32_t format, void* hip_stream);
/* The launch variant the continuous-tiles pool runs for `job`'s geometry (its buffer's device): waves
 * per SIMD (5 or 6) and the share of the grid that claims units from the back (percent; 0 for
 * launches of more than 16 frames).  Fixed by PT_MI355_CT_WAVES / PT_MI355_BACK, else the pick of the
 * geometry's timed launches; *waves = 0 while it is undecided (no scheduled launch timed yet), or for a
 * job that does not run the continuous-tiles pool.  Host state only, no GPU work. */
int pt_launch_variant(const pt_device_job* job, int32_t* waves, int32_t* back_pct);

#ifdef __cplusplus
}
#endif
#endif
