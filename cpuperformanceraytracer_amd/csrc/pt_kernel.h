// pt_kernel.h -- launch interface between the C-ABI layer (pt_capi.cpp) and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pt_scene.h"

// Output layouts of the reference's frame functions (include/pt_mi355.h documents each).
enum PtLayout : int32_t {
    PT_LAYOUT_INTERLEAVED = 0,    // DemofoxRenderScalar: [(row*W + x)*3 + ch]
    PT_LAYOUT_PLANAR8 = 1,        // DemofoxRenderSimd:   per 8-px group [R x8][G x8][B x8]
    PT_LAYOUT_TILED_PLANAR8 = 2,  // RenderTile:          tile-major, planar8 inside each tile row
};

// Work counters written by the COUNT build (one atomic per wave at exit).
enum PtCounter : int {
    PT_CNT_SEGMENTS = 0,     // TestSceneTrace calls over all lanes (useful work)
    PT_CNT_LANE_SLOTS = 1,   // 64 x trace-loop iterations over all waves (issued lane-slots)
    PT_CNT_SAMPLES = 2,      // primary samples finished
    PT_CNT_ESCAPED = 3,      // paths that ended on a miss
    PT_CNT_PRIMARY = 4,      // camera-ray segments traced (one per pixel)
    PT_CNT_FALLBACK = 5,     // segments whose culled quad stage ran the six exact tests
    PT_CNT_SKY = 6,          // camera rays whose TestSceneTrace a sky tile skipped (counted in SEGMENTS)
    PT_CNT_N = 7,
};

struct PtJob {
    float* buf;                 // device accumulator (layout below)
    const PtScene* scene;       // device scene table (pt_scene.h)
    int32_t width, height;      // iResolution (full image)
    int32_t col0, ncols;        // pixel columns [col0, col0 + ncols)
    int32_t row_start;          // first global row Y (row 0 = top of image)
    int32_t row_stride;         // global-row step between consecutive buffer rows
    int32_t nrows;              // buffer rows rendered
    int32_t layout;             // PtLayout
    int32_t tile_w, tile_h;     // PT_LAYOUT_TILED_PLANAR8 only
    uint32_t frame_first;       // iFrame of the first accumulated frame (>= 1)
    int32_t nframes;            // frames accumulated in order (spp of this launch)
    int32_t num_bounces;        // c_numBounces
    const float* env;           // device env map (H x W x 3), nullptr => ambient
    int32_t env_w, env_h;
    unsigned long long* counters;  // PT_CNT_N u64, COUNT build only
    unsigned int* queue;           // PT_QUEUE_WORDS tile-queue words, zero at the launch's start
    unsigned int* queue_next;      // the next launch's words, zeroed by this launch (nullptr: none)
    const uint32_t* order;         // tile schedule: position -> tile (a permutation), nullptr = identity
    const uint32_t* units;         // schedule runs: unit k = positions [units[k], units[k+1]), nullptr = one tile each
    const uint32_t* nunits;        // device word: number of units (with units)
    uint32_t* cost;                // per-tile work of this launch (trace iterations), nullptr = not recorded
    uint32_t* err;                 // PT_ERR_WORDS error words (below); nullptr = not recorded
    uint32_t guard_cap;            // upper limit of the ring pool's iteration guard: ~0u (tests lower it)
    float* ct_slots;               // continuous-tiles pool (pt_kernel.hip render_body_ct): pt_ct_wave_floats()
    uint32_t ct_waves;             // f32 per wave for ct_waves waves; nullptr: one-chunk launches use render_body
    uint32_t ct_back_pct;          // the continuous-tiles pool: the last-dispatched ct_back_pct % of the grid
                                   // claims its units from the back of its queue group (pt_tile_queue.h)
    uint32_t ct_wide;              // the diffuse continuous-tiles kernel at 6 waves per SIMD (0: 5)
    // fused output stage (pt_render_device_present): each pixel's 8-bit value (pt_tonemap.h, the
    // reference's default fast ACES / gamma) at pix_out[row * ncols + col] of the job's rows, written
    // where its final accumulator value is (the continuous-tiles kernels; nullptr: none)
    uint32_t* pix_out;
    int32_t pix_xrgb;              // PT_PIXEL_XRGB8 (OutputToScreen) else RGBA8 (OutputToFile)
    // mainImage's frame constants (scalar.cpp:338-347), set by pt_launch_render on the host with the
    // same correctly rounded f32 operations: W, H, 1/W, 1/H, W/H, 1/(W/H).  Kernel arguments are
    // scalar registers; computed in the kernel they were VGPRs that the tile loop spilled.
    float cam_W, cam_H, cam_yW, cam_yH, cam_aspect, cam_yAspect;
    // chained launches (pt_render_device_chain; pt_capi.cpp launch_chain): consecutive launches of one
    // geometry run overlapped on two streams, so the next launch's waves fill the CUs the finishing
    // ones free.  The only data one launch needs from the one before is a tile's accumulator values
    // (the lerp chain of :812): a launch touches a tile's pixels only after the previous launch has
    // stored them -- per half-tile epochs, stored after the tile's last pixel stores (`sc1` stores,
    // vmcnt(0), an `sc1` epoch store; MI355X_MICROARCH.md hand-off row 1) and polled with `sc1`
    // loads.  The continuous-tiles kernels only (render_body_ct).
    uint32_t* tile_epoch;          // 2 x tiles words (halves: rows 0-3, 4-7); nullptr: not chained
    uint32_t chain_seq;            // stored into a tile's epochs once its pixels are final
    uint32_t chain_wait;           // touch a tile's pixels only once its epochs are >= chain_wait (0: none)
    unsigned long long* started;   // + 1 per block at its start: the next launch's stream gate (nullptr: none)
    uint32_t chain_delay;          // test hook (PT_MI355_TEST_CHAIN_DELAY): ~us a wave sleeps before publishing
};

// Kernel error words (PtJob::err, PtV4Job::err; reset by the host after it reports them, pt_capi.cpp
// sync_all): [0] tiles abandoned by a pool guard (the ring pool's iteration guard, the
// continuous-tiles pools' chunk / event guards), [1] the smallest such tile index (~0u: none),
// [2] failed bounds guards (pt_guard.h), [3] 0, [4..5] the smallest (guard id << 32 | detail) of
// them (~0: none).
#define PT_ERR_WORDS 6
#define PT_ERR_GUARD_COUNT 2
#define PT_ERR_GUARD_FIRST 4
enum PtGuardId : uint32_t {
    PT_G_QUEUE_ENTRY = 1,   // a schedule entry outside the launch's tiles (tile_at; every build)
    PT_G_NUNITS = 2,        // the schedule's unit count beyond its order (2 x tiles entries)
    PT_G_UNIT_RANGE = 3,    // a unit's schedule positions outside order[]
    PT_G_SLOT_BASE = 4,     // a wave's continuous-tiles slot area beyond ct_waves
    PT_G_ITEM_SLOT = 5,     // an item's radiance slot outside its wave's area
    PT_G_PIXEL = 6,         // an accumulator element outside the job's buffer
    PT_G_PIXOUT = 7,        // a presented pixel outside the job's pixel buffer
    PT_G_ENVQ = 8,          // an env miss-queue entry outside the wave's queue
    PT_G_SCHED_ORDER = 9,   // the schedule builder: an order position >= 2 x tiles
    PT_G_SCHED_UNIT = 10,   // the schedule builder: a unit index > 2 x tiles
    PT_G_RECORD = 11,       // a tile's item record slot >= 64
    PT_G_QUEUE_GROUP = 12,  // a queue group counter beyond PT_NQUEUES
    PT_G_CHAIN_WAIT = 13,   // a chained launch polled 2^21 times (>= 2 s) for the previous launch's tile (every build)
};

// Tile queues: one counter per XCD group, 128 B apart (PT_QUEUE_WORDS u32 per launch).
#ifndef PT_NQUEUES
#define PT_NQUEUES 8
#endif
#define PT_QUEUE_WORDS (PT_NQUEUES * 32)
// Tile queue entries (pt_tile_queue.h): the tile index in the low 30 bits, its part in the top 2 (0 the
// whole 8x8 tile, 1 rows 0-3, 2 rows 4-7)
#define PT_TILE_MASK 0x3fffffffu
#define PT_TILE_PART_SHIFT 30

// Enqueue one render launch on `stream`.  Returns hipSuccess or the launch error.  With job.pix_out
// the pixels are written by the render kernel itself when it is a continuous-tiles one, else by the
// standalone output pass enqueued after it (pt_output.hip).
// *ct_blocks (optional): the grid of the continuous-tiles kernel it launched (0: another pool, or
// nothing launched) -- a chained launch's gate waits for that many started blocks.
hipError_t pt_launch_render(const PtJob& job, hipStream_t stream, bool count, uint32_t* ct_blocks = nullptr);

// The continuous-tiles pool's scratch: f32 per wave, and the waves of its resident grid on the
// current device (the most a launch uses).
uint32_t pt_ct_wave_floats();
uint32_t pt_ct_resident_waves();
int32_t pt_ct_env_waves();   // the env continuous-tiles kernel's waves per SIMD (PT_ENV_WAVES)

// Tiles of a job (8x8 pixel tiles over ncols x nrows).
inline uint32_t pt_job_tiles(const PtJob& j)
{
    return (uint32_t)((j.ncols + 7) / 8) * (uint32_t)((j.nrows + 7) / 8);
}

// Enqueue the schedule builder: order = the queue entries sorted by descending cost (every tile
// once, or as its two halves when it costs more than 1/split of a resident wave's share of the
// launch; split 0: never), units = runs of about equal cost over it, *nunits = their number.
// cost: 2 x ntiles words (pt_record_cost), order: up to 2 x ntiles entries, units: 2 x ntiles + 1.
// unit_mult: a multiple of the adaptive unit cost (the continuous-tiles pools: 2).
// err: the device's error words (the checked build's guards; nullptr: none).
// The chained-launch wait bound of this library's diffuse kernels on the current device (test hook:
// pt_chain.h pt_chain_polls_dev; 0: the default)
hipError_t pt_set_chain_polls(uint32_t polls);
hipError_t pt_launch_schedule(const uint32_t* cost, uint32_t* order, uint32_t* units, uint32_t* nunits,
                              uint32_t ntiles, uint32_t split, uint32_t unit_mult, hipStream_t stream,
                              uint32_t* err = nullptr);
