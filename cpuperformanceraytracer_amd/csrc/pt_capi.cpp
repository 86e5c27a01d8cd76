// pt_capi.cpp -- the C ABI of libpt_mi355.so (include/pt_mi355.h): validation, frame state,
// host<->device buffer mirroring, dispatch to the HIP kernels (pt_kernel.hip, pt_v4.hip,
// pt_output.hip), and the fan-out of every host-buffer entry point over one or several GPUs.
//
// Reference behaviour mirrored here (paths relative to CPUPerformanceRayTracer/):
//   - frame counter: `static f32 iFrame; iFrame += 1` before rendering (scalar.cpp:798-799,
//     simd.cpp:483-484, simd_tiled.cpp:547);
//   - settings checks of ApplicationState::CheckValidSettings (Application.cpp:36-94), returned
//     as PT_EINVAL instead of __debugbreak();
//   - the caller owns the host buffer, the call returns after it is updated (Application.cpp:474).
//
// Several devices (pt_config.device_count > 1, or PT_MI355_DEVICES): the reference fans a frame's
// tiles out over its CPU threads (simd_tiled.cpp:549-571, v4 :1696-1721); here a frame's ROWS are
// dealt to the devices, row Y to device Y mod N (neighbouring rows cost alike, so every device gets
// the same mix of cheap sky rows and expensive rows into the box).  Every pixel's value depends only
// on its global (x, y) and the frame, so any split renders bit-identical pixels.  Each device keeps
// its own mirror of its rows: a compact sub-image for the row layouts (interleaved, planar8) and a
// full-size buffer of which it owns the rows for the tiled layout (whose rows are not contiguous in
// the host buffer); transfers move only the owned rows (pitched 2D copies).
#include "pt_kernel.h"
#include "pt_guard.h"
#include "pt_output.h"
#include "pt_v4.h"
#include "../../include/pt_mi355.h"
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <new>
#include <vector>

namespace {

// Tile schedule of a recurring job geometry: the previous launch's per-tile costs, and the order
// built from them (longest tiles first) for the next launch on the same stream.  Per-pixel work
// varies ~10x across the image (rays inside the box bounce, sky rays stop), and with the tiles
// taken in raster order the last-dequeued expensive tiles left most of the chip idle at the end.
// The geometry a schedule belongs to (which renderer, which pixels, how many bounces, which env).
struct SchedKey {
    int32_t kind = 0;   // 0: the diffuse kernels; 1 + env mode: v4
    int32_t width = 0, height = 0, col0 = 0, ncols = 0, row_start = 0, row_stride = 0, nrows = 0, bounces = 0;
    const float* env = nullptr;
    uint32_t ntiles = 0;
    uint32_t split = 0;   // the schedule builder's split factor (launch(): one-chunk launches only)
    bool operator==(const SchedKey& o) const
    {
        return kind == o.kind && width == o.width && height == o.height && col0 == o.col0 && ncols == o.ncols &&
               row_start == o.row_start && row_stride == o.row_stride && nrows == o.nrows && bounces == o.bounces &&
               env == o.env && ntiles == o.ntiles && split == o.split;
    }
};
struct Sched {
    bool used = false;
    hipStream_t stream = nullptr;
    SchedKey key;
    uint32_t* cost = nullptr;
    uint32_t* order = nullptr;
    uint32_t* units = nullptr;    // 2 ntiles + 2 words: run starts, then the run count (cost: 2 ntiles words,
                                  // order: up to 2 ntiles entries -- split tiles, pt_tile_queue.h)
    bool have_cost = false;
    bool built = false;           // order/units hold a schedule
    unsigned long long launches = 0;
    unsigned long long last_use = 0;
    // launch variant of the diffuse continuous-tiles kernel (PT_MI355_CT_WAVES=0, the default): the
    // first scheduled launches time the arms (ct_occupancy) between event pairs, the fastest is kept
    hipEvent_t tune_ev[2 * 18] = {};
    uint32_t tuned = 0;           // timed launches enqueued
    uint32_t narms = 0;           // arms timed (2 or 3; 0: not started)
    int32_t tune_nframes = 0;     // the frames of the first timed launch: only launches of that length are timed
    int8_t wide = -1;             // the pick: arm index (-1: not yet)
    // chained launches (launch_chain): per half-tile, the chain sequence number of the last launch
    // that stored its pixels (2 ntiles words), and that number of the geometry's last chained launch
    uint32_t* epoch = nullptr;
    uint32_t chain_seq = 0;
};
constexpr uint32_t kTuneRounds = 3;   // rounds of the palindromic arm order timed; the first is discarded
constexpr int kSchedSlots = 16;
constexpr int kBands = 4;   // PT_FLAG_PIN_HOST: row bands of a pipelined frame
constexpr uint32_t kSchedMinTiles = 512;   // smaller jobs (e.g. one RenderTile) are not scheduled
constexpr unsigned kQueueRing = 256;       // tile-queue ring slots (reuse across streams is event-ordered)
// launches per schedule build (g.sched_rebuild; PT_MI355_SCHED_REBUILD): 256 -- a build restarts the
// chained overlap and costs a one-workgroup kernel (~57 us at 1080p); 3-round A/B of chained steps vs 64
// (profiles/r06/r06zl_*): c2 0.2160 vs 0.2189 ms, c4 0.4582 vs 0.4633, v4 0.3286 vs 0.3313
constexpr unsigned long long kSchedRebuildDefault = 256;

// One (logical) device: its streams, scene, tile queues, schedules, env map and the mirror of its
// share of the caller's host accumulator.  Several logical devices may name the same HIP device
// (tests shard a frame over N logical devices on one GPU).
struct Dev {
    int32_t ordinal = 0;
    hipStream_t stream = nullptr;
    PtScene* dscene = nullptr;          // device copy of State::scene
    float* dbuf = nullptr;              // mirror of this device's rows of the host accumulator
    size_t dbuf_cap = 0;
    unsigned long long* dcounters = nullptr;
    uint32_t* derr = nullptr;           // PT_ERR_WORDS kernel error words (PtJob::err)
    float* dct = nullptr;               // continuous-tiles pool slots (PtJob::ct_slots), for dct_waves waves
    uint32_t dct_waves = 0;
    int ct_slot = -1;                   // tile-queue ring slot of the last launch that used dct (its event
                                        // orders the next such launch on another stream: one set of slots)
    uint32_t* herr = nullptr;           // their page-locked host copy (read at every synchronisation)
    unsigned int* dqueue = nullptr;     // ring of kQueueRing tile-queue blocks (PT_QUEUE_WORDS each)
    unsigned queue_next = 0;
    bool queue_pre_zeroed = false;      // the last launch's kernel zeroes ring slot queue_next % kQueueRing
    hipStream_t last_stream = nullptr;  // the stream of the last launch
    // per ring slot: the stream of the last launch that used it and an event recorded after that
    // launch; a launch on another stream waits for it before re-zeroing the slot
    hipStream_t queue_stream[kQueueRing] = {};   // (compared for equality only, never used: it may be
    hipEvent_t queue_event[kQueueRing] = {};     //  a caller's stream that no longer exists)
    // a slot skipped by a change of stream is ordered by the event of the slot before it (recorded
    // after the launch whose kernel zeroes the skipped slot): its index, or -1
    int16_t queue_alias[kQueueRing];
    float* denv = nullptr;              // env map in HBM (pt_set_env_map / textured / v4)
    Sched sched[kSchedSlots];
    unsigned long long sched_clock = 0;
    float* dtone_in = nullptr;          // output stage scratch
    size_t dtone_in_cap = 0;
    uint32_t* dtone_out = nullptr;
    size_t dtone_out_cap = 0;
    // PT_FLAG_GATHER_ROOT: the root (device 0) assembles the whole accumulator from every device's
    // rows -- each device stores its rows into dgather of the root over xGMI (peer access)
    float* dgather = nullptr;           // root only: W x H x 3
    size_t dgather_cap = 0;
    hipEvent_t ev_gather = nullptr;     // recorded after this device's rows were stored
    bool peer_root = false;             // this device may store into the root's memory
    // chained launches (pt_render_device_chain, launch_chain): consecutive launches of one geometry
    // alternate on two streams of the library's and overlap on the GPU
    struct Chain {
        hipStream_t st[2] = {};            // the two streams (non-blocking)
        hipEvent_t done[2] = {};           // recorded after each stream's last launch
        bool pending[2] = {};              // done[i] has been recorded
        hipEvent_t ev_caller = nullptr;    // the caller's stream at a chain (re)start
        float* area1 = nullptr;            // a second continuous-tiles slot area (the first: dct)
        unsigned int* qblk = nullptr;      // 4 tile-queue blocks of the continuing launches
        // blocks started by every chained launch so far (monotonic: a stream gate that is evaluated
        // before a restart's launch has started -- its stream waits only for the gate -- must not pass
        // on a count from before the restart), and the blocks those launches have
        unsigned long long* started = nullptr;
        unsigned long long cum = 0;
        Sched* sched = nullptr;            // the live chain's geometry (nullptr: the next chained launch restarts)
        int area = 0;                      // slot area of the live chain's last launch (0: dct, 1: area1)
        int par = 0;                       // stream of the live chain's last launch
        unsigned long long restarts = 0, continued = 0;   // chained launches of each kind (pt_chain_counts)
        // a chained launch's wait ran out on this device (guard PT_G_CHAIN_WAIT, reported by sync_all):
        // chained calls are plain launches from then on ("Residency")
        bool off = false;
    } chain;
};

// The host buffer the device mirrors currently represent, and the geometry they were split by.
struct Mirror {
    const float* host = nullptr;
    size_t bytes = 0;
    int32_t width = 0, height = 0;
    bool tiled = false;
    int32_t tile_w = 0, tile_h = 0;
    bool valid = false;                 // deferred mode: the device copies are authoritative
};

struct State {
    bool inited = false;
    pt_config cfg{};
    int ndev = 0;
    Dev dev[PT_MAX_DEVICES];
    PtScene scene{};
    uint32_t frame = 0;                 // value of the reference's static iFrame
    Mirror m;
    // env map (the same texture on every device)
    const float* env_src = nullptr;     // host data the device copies were made from
    int32_t env_w = 0, env_h = 0;
    bool have_env = false;
    // PT_FLAG_PIN_HOST (one device): the registered host buffer, copy streams and band events
    const float* pinned = nullptr;
    size_t pinned_bytes = 0;
    hipStream_t s_in = nullptr, s_out = nullptr;
    hipEvent_t ev_in[kBands] = {}, ev_done[kBands] = {};
    hipEvent_t ev_q = nullptr;          // work queues: orders banded copies against the stream
    hipEvent_t ev_root_free = nullptr;  // PT_FLAG_GATHER_ROOT: the root's earlier reads of dgather are done
    // v4 renderer (demofox_path_tracing_optimization_v4.cpp): its own iFrame (v4 :34) and scene
    pt_v4_config v4cfg{PT_V4_ENV_EQUIRECT, 1, 1, 8, 1, 1, 1, 1, 1};
    bool v4_scene_ready = false;
    PtV4SceneDesc v4desc{};
    PtV4Scene v4scene{};
    uint32_t v4_frame = 0;
    // test hook: PT_MI355_RING_GUARD_CAP (read by pt_init) caps the pools' iteration guards so
    // that it fires -- the error path's own GPU test (tests/test_gpu_state.py)
    uint32_t ring_guard_cap = ~0u;
    int32_t v4_ct_force = 0;   // PT_MI355_V4_CT=1 (read by pt_init): PtV4Job::ct_force (tests)
    uint32_t ct_back_pct = 20;   // PT_MI355_BACK (read by pt_init): PtJob::ct_back_pct (0: none)
    bool back_set = false;       // PT_MI355_BACK given: the occupancy timing keeps it
    uint32_t ct_waves = 0;       // PT_MI355_CT_WAVES (read by pt_init): 5 or 6 waves per SIMD; 0 (default):
                                 // the faster of the two, timed on each geometry's first launches
    // test hook: PT_MI355_CT_WAVES_SEQ (read by pt_init), a string of '5' / '6' cycled over the
    // diffuse continuous-tiles launches -- forced changes of the grid between the launches of one
    // accumulation (tests/test_gpu_configs.py); empty: off
    char ct_seq[64] = {};
    uint32_t ct_seq_len = 0, ct_seq_pos = 0;
    uint32_t split = 1;   // PT_MI355_SPLIT (read by pt_init): tile split factor of the schedule (0: none)
    int64_t test_bad_entry = -1;   // PT_MI355_TEST_BAD_ENTRY (test hook, pt_init)
    bool no_ct = false;   // PT_MI355_NO_CT=1 (read by pt_init): one-chunk launches on render_body (A/B)
    uint32_t test_chain_delay = 0;   // PT_MI355_TEST_CHAIN_DELAY=<us> (pt_init): chained launches publish late
    uint32_t unit_mult = 2;          // PT_MI355_UNIT_MULT (pt_init, A/B): the diffuse CT schedule's unit multiple
    unsigned long long sched_rebuild = kSchedRebuildDefault;   // PT_MI355_SCHED_REBUILD (pt_init): launches per schedule build
};

State g;
char g_err[512] = "no error";

int vfail(int code, const char* fmt, va_list ap)
{
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    return code;
}

int fail(int code, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return fail(PT_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

constexpr uint32_t kMaxFrame = 1u << 24;   // iFrame is an f32 counter: exact below 2^24
constexpr int32_t kMaxDim = 1 << 24;        // pixel coordinates are f32 in mainImage: exact up to 2^24
#if PT_DIAG
constexpr int kCounterSlots = 32 + 4 * 65536 + 96 * 65536;   // + per-wave records, per-tile log
#else
constexpr int kCounterSlots = 32;
#endif

// The caller's current HIP device is restored when an entry point returns (the library switches to
// each device it drives).
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int use_dev(const Dev& d)
{
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != d.ordinal) HIP_TRY(hipSetDevice(d.ordinal));
    return PT_OK;
}

int ensure_init()
{
    if (g.inited) return PT_OK;
    return pt_init(nullptr);
}

// ---- shards -----------------------------------------------------------------------------------
// Device d of n owns the global rows d, d + n, ...
int32_t shard_rows(int32_t h, int n, int d) { return d < h ? (h - 1 - d) / n + 1 : 0; }

// Geometry of a host accumulator: size and whether it is tile-major (RenderTile layout).
struct Geo {
    int32_t w = 0, h = 0;
    bool tiled = false;
    int32_t tw = 0, th = 0;
};

// Bytes of device d's mirror: the whole buffer with one device or the tiled layout, else the
// compact rows.
size_t dev_bytes(const Geo& geo, int d)
{
    if (g.ndev == 1 || geo.tiled) return (size_t)geo.w * geo.h * 3 * sizeof(float);
    return (size_t)shard_rows(geo.h, g.ndev, d) * geo.w * 3 * sizeof(float);
}

// A region of the host buffer: the whole frame, or one RenderTile slice (tile index k).
struct Region {
    bool whole = true;
    int32_t tile_x = 0, tile_y = 0;
};

// Copy device d's part of `rg` between the host buffer and its mirror (async on its stream).
int xfer(int d, const Geo& geo, float* host, bool to_device, const Region& rg)
{
    Dev& dv = g.dev[d];
    const hipMemcpyKind kind = to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
    const int n = g.ndev;
    if (n == 1) {
        size_t off = 0, len = (size_t)geo.w * geo.h * 3 * sizeof(float);
        if (!rg.whole) {   // simd_tiled.cpp:499-502: the tile is one contiguous slice
            off = ((size_t)rg.tile_y * geo.th * geo.w * 3 + (size_t)rg.tile_x * geo.tw * geo.th * 3) * sizeof(float);
            len = (size_t)geo.tw * geo.th * 3 * sizeof(float);
        }
        char* hp = (char*)host + off;
        char* dp = (char*)dv.dbuf + off;
        HIP_TRY(hipMemcpyAsync(to_device ? (void*)dp : (void*)hp, to_device ? (void*)hp : (void*)dp, len, kind, dv.stream));
        return PT_OK;
    }
    if (!geo.tiled) {   // compact rows: one pitched copy
        const int32_t nr = shard_rows(geo.h, n, d);
        if (nr == 0) return PT_OK;
        const size_t row = (size_t)geo.w * 3 * sizeof(float);
        char* hp = (char*)host + (size_t)d * row;
        if (to_device) HIP_TRY(hipMemcpy2DAsync(dv.dbuf, row, hp, row * n, row, nr, kind, dv.stream));
        else HIP_TRY(hipMemcpy2DAsync(hp, row * n, dv.dbuf, row, row, nr, kind, dv.stream));
        return PT_OK;
    }
    // tiled: every tile is contiguous (TW x TH x 3 floats, raster tile order); the device's rows of a
    // tile are every n-th of its tile rows -- one pitched copy per tile, same offsets on both sides
    const int32_t ntx = geo.w / geo.tw, nty = geo.h / geo.th;
    const size_t tile_f = (size_t)geo.tw * geo.th * 3, trow = (size_t)geo.tw * 3 * sizeof(float);
    const int32_t k0 = rg.whole ? 0 : rg.tile_y * ntx + rg.tile_x, k1 = rg.whole ? ntx * nty : k0 + 1;
    for (int32_t k = k0; k < k1; ++k) {
        const int32_t ty = k / ntx;
        const int32_t ly0 = (int32_t)((((int64_t)d - (int64_t)ty * geo.th) % n + n) % n);
        if (ly0 >= geo.th) continue;
        const int32_t cnt = (geo.th - 1 - ly0) / n + 1;
        const size_t off = (k * tile_f + (size_t)ly0 * geo.tw * 3) * sizeof(float);
        char* hp = (char*)host + off;
        char* dp = (char*)dv.dbuf + off;
        HIP_TRY(hipMemcpy2DAsync(to_device ? (void*)dp : (void*)hp, trow * n, to_device ? (void*)hp : (void*)dp,
                                 trow * n, trow, cnt, kind, dv.stream));
    }
    return PT_OK;
}

// Synchronise every device stream and report what the kernels recorded in their error words since
// the last synchronisation: a tile that a pool's guard abandoned (the ring pool's iteration guard or
// the continuous-tiles pool's chunk / event guards, pt_kernel.hip, pt_v4.hip) leaves a wrong
// accumulator, so no call that waited for such a launch returns PT_OK.  The words are reset when
// reported.  Device jobs on callers' streams are covered once those streams have been synchronised
// (pt_check_device_errors): a launch still running when the words are read and reset may record its
// fault after the reset, and that fault is then reported by the next check.
const char* guard_name(uint32_t id)
{
    switch (id) {
        case PT_G_QUEUE_ENTRY: return "schedule entry outside the launch's tiles";
        case PT_G_NUNITS: return "schedule unit count beyond its entries";
        case PT_G_UNIT_RANGE: return "unit positions outside the schedule";
        case PT_G_SLOT_BASE: return "wave slot area beyond the allocation";
        case PT_G_ITEM_SLOT: return "item radiance slot outside its wave's area";
        case PT_G_PIXEL: return "accumulator element outside the buffer";
        case PT_G_PIXOUT: return "presented pixel outside the pixel buffer";
        case PT_G_ENVQ: return "env miss-queue entry outside the queue";
        case PT_G_SCHED_ORDER: return "schedule builder: order position out of range";
        case PT_G_SCHED_UNIT: return "schedule builder: unit index out of range";
        case PT_G_RECORD: return "item record slot >= 64";
        case PT_G_QUEUE_GROUP: return "queue group out of range";
        case PT_G_CHAIN_WAIT: return "chained launch: the previous launch's tile never became ready; value: the tile | its epoch's lag "
                                     "<< 24 | bit 31 when an atomic read also lags (pt_chain.h)";
        default: return "unknown";
    }
}

int sync_all()
{
    int rc;
    for (int d = 0; d < g.ndev; ++d) {
        Dev& dv = g.dev[d];
        if ((rc = use_dev(dv))) return rc;
        HIP_TRY(hipMemcpyAsync(dv.herr, dv.derr, PT_ERR_WORDS * sizeof(uint32_t), hipMemcpyDeviceToHost, dv.stream));
    }
    for (int d = 0; d < g.ndev; ++d) {
        if ((rc = use_dev(g.dev[d]))) return rc;
        HIP_TRY(hipStreamSynchronize(g.dev[d].stream));
    }
    for (int d = 0; d < g.ndev; ++d) {
        Dev& dv = g.dev[d];
        const uint32_t guards = dv.herr[PT_ERR_GUARD_COUNT];
        if (dv.herr[0] == 0 && guards == 0) continue;
        const uint32_t n = dv.herr[0], tile = dv.herr[1];
        const unsigned long long first =
            (unsigned long long)dv.herr[PT_ERR_GUARD_FIRST] | ((unsigned long long)dv.herr[PT_ERR_GUARD_FIRST + 1] << 32);
        if ((rc = use_dev(dv))) return rc;
        const uint32_t init[PT_ERR_WORDS] = {0u, ~0u, 0u, 0u, ~0u, ~0u};
        memcpy(dv.herr, init, sizeof(init));
        HIP_TRY(hipMemcpyAsync(dv.derr, dv.herr, sizeof(init), hipMemcpyHostToDevice, dv.stream));
        HIP_TRY(hipStreamSynchronize(dv.stream));
        if (guards && (uint32_t)(first >> 32) == PT_G_CHAIN_WAIT) dv.chain.off = true;
        if (guards)
            return fail(PT_EKERNEL, "device %d: %u kernel bounds guard failure(s), the first: guard %u (%s), value %u; "
                        "pool guards: %u (first tile %u); the accumulator is invalid", dv.ordinal, guards,
                        (uint32_t)(first >> 32), guard_name((uint32_t)(first >> 32)), (uint32_t)first, n, n ? tile : 0u);
        return fail(PT_EKERNEL, "device %d: a pool guard (ring iterations or continuous-tiles chunks) abandoned %u "
                    "tile(s) (first: tile %u of its launch); the accumulator is invalid", dv.ordinal, n, tile);
    }
    return PT_OK;
}

int ensure_dbuf(int d, size_t bytes)
{
    Dev& dv = g.dev[d];
    if (bytes <= dv.dbuf_cap) return PT_OK;
    if (dv.dbuf) {
        HIP_TRY(hipStreamSynchronize(dv.stream));
        HIP_TRY(hipFree(dv.dbuf));
        dv.dbuf = nullptr;
        dv.dbuf_cap = 0;
    }
    if (hipMalloc(&dv.dbuf, bytes) != hipSuccess) {
        dv.dbuf = nullptr;
        return fail(PT_ENOMEM, "hipMalloc(%zu) failed on device %d", bytes, dv.ordinal);
    }
    dv.dbuf_cap = bytes;
    g.m.valid = false;
    return PT_OK;
}

Geo mirror_geo()
{
    Geo geo;
    geo.w = g.m.width;
    geo.h = g.m.height;
    geo.tiled = g.m.tiled;
    geo.tw = g.m.tile_w;
    geo.th = g.m.tile_h;
    return geo;
}

// Deferred mode: a valid mirror is the only up-to-date copy of its host buffer's accumulation.
// Before the mirror is given to another buffer it is written back to its own host buffer (as if
// pt_readback had been called), so alternating buffers loses nothing.  The caller must release a
// deferred buffer (pt_release_buffer) before freeing it.
int flush_mirror()
{
    int rc;
    if (!g.m.valid || !g.m.host) {
        g.m.valid = false;
        return PT_OK;
    }
    const Geo geo = mirror_geo();
    for (int d = 0; d < g.ndev; ++d) {
        if ((rc = use_dev(g.dev[d])) || (rc = xfer(d, geo, (float*)g.m.host, false, Region{}))) return rc;
    }
    if ((rc = sync_all())) return rc;
    g.m.valid = false;
    return PT_OK;
}

void drop_mirror()
{
    g.m = Mirror{};
}

bool same_split(const Geo& geo)
{
    if (g.m.width != geo.w || g.m.height != geo.h) return false;
    if (g.ndev == 1) return true;   // one device mirrors the whole buffer in any layout
    return g.m.tiled == geo.tiled && (!geo.tiled || (g.m.tile_w == geo.tw && g.m.tile_h == geo.th));
}

// Make the device mirrors hold region `rg` of the host buffer `host` (geometry `geo`).  In
// deferred mode an already valid mirror of the same buffer is authoritative and nothing is copied.
int stage_in(float* host, const Geo& geo, const Region& rg)
{
    const bool deferred = (g.cfg.flags & PT_FLAG_DEFER_READBACK) != 0;
    const size_t bytes = (size_t)geo.w * geo.h * 3 * sizeof(float);
    int rc;
    if (g.m.valid) {
        if (g.m.host == host && g.m.bytes != bytes) drop_mirror();   // reallocated in place: never write back
        else if (g.m.host != host || !same_split(geo))
            if ((rc = flush_mirror())) return rc;
    }
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = use_dev(g.dev[d])) || (rc = ensure_dbuf(d, dev_bytes(geo, d)))) return rc;
    if (deferred && g.m.valid) return PT_OK;
    const Region r = deferred ? Region{} : rg;   // first deferred touch: the whole buffer becomes device-resident
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = use_dev(g.dev[d])) || (rc = xfer(d, geo, host, true, r))) return rc;
    g.m.host = host;
    g.m.bytes = bytes;
    g.m.width = geo.w;
    g.m.height = geo.h;
    g.m.tiled = geo.tiled;
    g.m.tile_w = geo.tw;
    g.m.tile_h = geo.th;
    g.m.valid = deferred;
    return PT_OK;
}

int stage_out(float* host, const Geo& geo, const Region& rg)
{
    int rc;
    if (!(g.cfg.flags & PT_FLAG_DEFER_READBACK))
        for (int d = 0; d < g.ndev; ++d)
            if ((rc = use_dev(g.dev[d])) || (rc = xfer(d, geo, host, false, rg))) return rc;
    return sync_all();
}

int check_frame_budget(uint32_t add)
{
    if ((uint64_t)g.frame + add >= kMaxFrame)
        return fail(PT_EINVAL, "frame counter %u + %u exceeds the exact f32 range 2^24", g.frame, add);
    return PT_OK;
}

PtJob base_job(float* buf, int32_t w, int32_t h)
{
    PtJob j{};
    j.buf = buf;
    j.width = w;
    j.height = h;
    j.col0 = 0;
    j.ncols = w;
    j.row_start = 0;
    j.row_stride = 1;
    j.nrows = h;
    j.layout = PT_LAYOUT_INTERLEAVED;
    j.tile_w = j.tile_h = 0;
    j.frame_first = g.frame + 1;
    j.nframes = g.cfg.samples_per_frame;
    j.num_bounces = g.cfg.num_bounces;
    j.env = nullptr;
    j.env_w = j.env_h = 0;
    j.counters = nullptr;
    j.order = nullptr;
    j.units = nullptr;
    j.nunits = nullptr;
    j.cost = nullptr;
    j.err = nullptr;
    j.guard_cap = g.ring_guard_cap;
    j.ct_slots = nullptr;
    j.ct_waves = 0;
    j.ct_back_pct = 0;   // (launch(): launches of <= 16 frames)
    j.ct_wide = 0;
    j.scene = nullptr;
    j.tile_epoch = nullptr;
    j.chain_seq = 0;
    j.chain_wait = 0;
    j.started = nullptr;
    return j;
}

void free_sched(Sched& s)
{
    if (s.cost) (void)hipFree(s.cost);
    if (s.order) (void)hipFree(s.order);
    if (s.units) (void)hipFree(s.units);
    if (s.epoch) (void)hipFree(s.epoch);
    for (hipEvent_t e : s.tune_ev)
        if (e) (void)hipEventDestroy(e);
    s = Sched{};
}

SchedKey sched_key(const PtJob& j)
{
    SchedKey k;
    k.kind = 0;
    k.width = j.width;
    k.height = j.height;
    k.col0 = j.col0;
    k.ncols = j.ncols;
    k.row_start = j.row_start;
    k.row_stride = j.row_stride;
    k.nrows = j.nrows;
    k.bounces = j.num_bounces;
    k.env = j.env;
    k.ntiles = pt_job_tiles(j);
    return k;
}

SchedKey sched_key(const PtV4Job& j)
{
    SchedKey k;
    k.kind = 1 + j.env_mode;
    k.width = j.width;
    k.height = j.height;
    k.col0 = j.col0;
    k.ncols = j.ncols;
    k.row_start = j.row_start;
    k.row_stride = j.row_stride;
    k.nrows = j.nrows;
    k.bounces = j.num_bounces;
    k.env = j.env;
    k.ntiles = (uint32_t)((j.ncols + 7) / 8) * (uint32_t)((j.nrows + 7) / 8);
    return k;
}

Sched* find_sched(Dev& dv, const SchedKey& key, hipStream_t st)
{
    const uint32_t n = key.ntiles;
    if (n < kSchedMinTiles) return nullptr;
    Sched* lru = &dv.sched[0];
    for (Sched& s : dv.sched) {
        if (s.used && s.stream == st && s.key == key) {
            s.last_use = ++dv.sched_clock;
            return &s;
        }
        if (!s.used || (lru->used && s.last_use < lru->last_use)) lru = &s;
    }
    if (lru->used) {   // evict: its buffers may still be read by a launch (its stream may be gone)
        (void)hipDeviceSynchronize();
        if (dv.chain.sched == lru) dv.chain.sched = nullptr;   // (its chain ends: the next chained launch restarts)
        free_sched(*lru);
    }
    Sched s;
    if (hipMalloc(&s.cost, 2 * (size_t)n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&s.order, 2 * (size_t)n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&s.units, (2 * (size_t)n + 2) * sizeof(uint32_t)) != hipSuccess) {
        free_sched(s);
        return nullptr;   // unscheduled launch (raster order): correct, only slower
    }
    s.used = true;
    s.stream = st;
    s.key = key;
    s.last_use = ++dv.sched_clock;
    *lru = s;
    return lru;
}

int slot_event(Dev& dv, unsigned slot)
{
    if (!dv.queue_event[slot]) HIP_TRY(hipEventCreateWithFlags(&dv.queue_event[slot], hipEventDisableTiming));
    return PT_OK;
}

// The event ordering the last use of ring slot `slot` (nullptr: never used).
hipEvent_t slot_order(const Dev& dv, unsigned slot)
{
    const int a = dv.queue_alias[slot];
    return a >= 0 ? dv.queue_event[a] : dv.queue_event[slot];
}

// The schedule and queue fields of a launch of geometry `key` on stream `st`.
struct LaunchSched {
    unsigned slot = 0;   // tile-queue ring slot (queue_done after the launch)
    unsigned int* queue = nullptr;
    unsigned int* queue_next = nullptr;   // the next ring slot, zeroed by this launch's kernel
    const uint32_t* order = nullptr;
    const uint32_t* units = nullptr;
    const uint32_t* nunits = nullptr;
    uint32_t* cost = nullptr;
    Sched* sched = nullptr;
};
// Order `st` after every chained launch of the device and end the live chain (launch_chain): a
// launch that is not a continuing chained one may use what the chained launches use -- the slot
// areas, the geometry's schedule, the accumulator.
int chain_join(Dev& dv, hipStream_t st)
{
    for (int i = 0; i < 2; ++i) {
        if (!dv.chain.pending[i]) continue;
        if (hipEventQuery(dv.chain.done[i]) == hipSuccess) {
            dv.chain.pending[i] = false;
        } else {
            (void)hipGetLastError();   // (hipErrorNotReady)
            HIP_TRY(hipStreamWaitEvent(st, dv.chain.done[i], 0));
        }
    }
    dv.chain.sched = nullptr;
    return PT_OK;
}

// split: the schedule builder's tile split factor (pt_launch_schedule; 0: whole tiles).  *sched_st: the
// stream that identifies the geometry's schedule (launch_chain: the caller's stream, which may be the
// null stream; nullptr: st).
int use_sched(Dev& dv, const SchedKey& key, hipStream_t st, LaunchSched* ls, uint32_t split,
              const hipStream_t* sched_st = nullptr)
{
    *ls = LaunchSched{};
    int rc;
    if ((rc = chain_join(dv, st))) return rc;
    if (Sched* s = find_sched(dv, key, sched_st ? *sched_st : st)) {
        // (re)build the schedule from the last launch's costs on the 2nd launch of a geometry and
        // then every g.sched_rebuild launches (the costs of a fixed view barely change; the builder
        // is a one-workgroup kernel of ~57 us at 1080p)
        if (s->have_cost && (!s->built || s->launches % g.sched_rebuild == 0)) {
            // units of twice the adaptive cost for the diffuse kernels' continuous-tiles pool, whose
            // lanes no longer idle in a unit's tail while the dequeues still cost (A/B, 60 launches:
            // 1080p 8 spp 0.2497 vs 0.2525 ms, env 16 spp 0.4911 vs 0.4961, 4K 8 spp 0.8185 vs 0.8202;
            // 3x: 0.2513 / 0.4965 / 0.8356)
            const uint32_t unit_mult = key.kind == 0 && !g.no_ct ? g.unit_mult : 1u;
            hipError_t e = pt_launch_schedule(s->cost, s->order, s->units, s->units + 2 * s->key.ntiles + 1, s->key.ntiles,
                                              split, unit_mult, st, dv.derr);
            if (e != hipSuccess) return fail(PT_EHIP, "schedule launch failed: %s", hipGetErrorString(e));
            s->built = true;
            if (g.test_bad_entry >= 0 && (uint32_t)g.test_bad_entry < 2u * s->key.ntiles)   // (test hook, below)
                HIP_TRY(hipMemsetAsync(s->order + g.test_bad_entry, 0xff, sizeof(uint32_t), st));
        }
        if (s->built) {
            ls->sched = s;
            ls->order = s->order;
            ls->units = s->units;
            ls->nunits = s->units + 2 * s->key.ntiles + 1;
        }
        // the kernel records the tiles' costs only when the next launch builds from them (one 4-B
        // store per tile is a 32-B HBM write: ~1 MB per 1080p launch otherwise)
        if (!s->built || (s->launches + 1) % g.sched_rebuild == 0) {
            ls->cost = s->cost;
            s->have_cost = true;
        }
        ++s->launches;
    }
    // Ring slots are used in order.  Each render kernel zeroes the NEXT slot's counters at its start,
    // so a launch after a launched kernel on the same stream finds its slot zero.  After a launch on
    // another stream that slot may still be being zeroed: it is skipped (its next user waits for that
    // kernel) and this launch zeroes the slot after it with a memset on its own stream, so launches on
    // different streams overlap.  A slot whose previous user ran on another stream is waited for
    // before it is zeroed or used.
    // Nothing is ever enqueued on a stream other than `st` (a previous launch's stream may be a
    // caller's stream that has been destroyed since): the skipped slot takes the previous slot's
    // event, recorded by queue_done right after the launch whose kernel zeroes it.
    unsigned slot = dv.queue_next++ % kQueueRing;
    bool pre = dv.queue_pre_zeroed;
    if (pre && dv.last_stream != st) {
        const unsigned prev = (slot + kQueueRing - 1) % kQueueRing;
        dv.queue_alias[slot] = (int16_t)prev;
        dv.queue_stream[slot] = dv.queue_stream[prev];
        slot = dv.queue_next++ % kQueueRing;
        pre = false;
    }
    ls->slot = slot;
    if (hipEvent_t ev = slot_order(dv, slot); ev && dv.queue_stream[slot] != st) HIP_TRY(hipStreamWaitEvent(st, ev, 0));
    ls->queue = dv.dqueue + (size_t)slot * PT_QUEUE_WORDS;
    if (!pre) HIP_TRY(hipMemsetAsync(ls->queue, 0, PT_QUEUE_WORDS * sizeof(unsigned), st));
    dv.queue_pre_zeroed = false;   // (set by queue_done once this launch's kernel is enqueued)
    const unsigned next = (slot + 1) % kQueueRing;
    if (hipEvent_t ev = slot_order(dv, next); ev && dv.queue_stream[next] != st) HIP_TRY(hipStreamWaitEvent(st, ev, 0));
    ls->queue_next = dv.dqueue + (size_t)next * PT_QUEUE_WORDS;
    return PT_OK;
}

// After the launch that used ring slot `slot` was enqueued on `st`; `zeroed_next`: its kernel ran
// (a launch with nothing to render returns without one) and zeroes the next slot.
int queue_done(Dev& dv, unsigned slot, hipStream_t st, bool zeroed_next)
{
    int rc;
    if ((rc = slot_event(dv, slot))) return rc;
    HIP_TRY(hipEventRecord(dv.queue_event[slot], st));
    dv.queue_stream[slot] = st;
    dv.queue_alias[slot] = -1;
    dv.queue_pre_zeroed = zeroed_next;
    dv.last_stream = st;
    return PT_OK;
}

// The continuous-tiles pools' slot area (pt_kernel.hip render_body_ct, pt_v4.hip pt_v4_ct_kernel) for
// a launch in ring slot ls.slot on `st`: nullptr (the per-tile pool kernels) with PT_MI355_NO_CT=1.
// The device's slot area (Dev::dct), allocated on first use: 12 KiB per wave of the resident grid
// (~75 MB).  Left null when the allocation fails (the per-tile pools then: correct, slower).
void ct_area_alloc(Dev& dv)
{
    if (dv.dct) return;
    const uint32_t w = pt_ct_resident_waves();
    if (hipMalloc(&dv.dct, (size_t)w * pt_ct_wave_floats() * sizeof(float)) == hipSuccess) dv.dct_waves = w;
    else dv.dct = nullptr, (void)hipGetLastError();
}

int use_ct_slots(Dev& dv, const LaunchSched& ls, hipStream_t st, float** slots, uint32_t* waves)
{
    *slots = nullptr;
    *waves = 0;
    if (g.no_ct) return PT_OK;
    ct_area_alloc(dv);
    *slots = dv.dct;
    *waves = dv.dct_waves;
    if (dv.dct) {   // launches on several streams share the slots: one after the other
        if (dv.ct_slot >= 0 && dv.queue_stream[dv.ct_slot] != st)
            if (hipEvent_t ev = slot_order(dv, (unsigned)dv.ct_slot)) HIP_TRY(hipStreamWaitEvent(st, ev, 0));
        dv.ct_slot = (int)ls.slot;
    }
    return PT_OK;
}

// The launch variant of a continuous-tiles launch (diffuse and env kernels): PtJob::ct_wide (5 or 6 waves per SIMD) and
// PtJob::ct_back_pct.  PT_MI355_CT_WAVES=5|6 fixes the occupancy (and the env share); by default (0) the geometry's first
// scheduled launches time the ARMS and the fastest is kept (per stream: a geometry's Sched):
//   arm 0: 5 waves, arm 1: 6 waves -- each with the default back-claim share (20 %) -- and, for
//   launches that take back claims (<= 16 frames) unless PT_MI355_BACK is given, arm 2: 6 waves with
//   kBackWide % of the grid claiming from the back.  Measured (profiles/r05/r05i_back_sweep_ab.jsonl,
//   r05h_back_ab.jsonl): at 6 waves 45 % gave 1080p 8 spp 0.2392 vs 0.2440 ms and 4K 8 spp 0.8015 vs
//   0.8395 (55-90 %: 0.249 / 0.80), but 720p 0.1490 vs 0.1462 and, at 5 waves, 1080p 0.2526 vs 0.2488 --
//   so it is one more timed arm, not a new default.
// The env kernel has one occupancy (PT_ENV_WAVES); its arms, for launches that take back claims unless
//   PT_MI355_BACK is given, are the back-claim shares 20 (default), 33 and 45 %: measured
//   (profiles/r05/r05k_env_back_ab.jsonl) 1080p 8 frames 0.2786 / 0.2809 / 0.2738 ms, 16 frames
//   0.4821 / 0.4770 / 0.4885 -- the best share depends on the launch, as for the diffuse kernel.
// The arms are timed in a palindromic order (ABBA, ABCCBA), three rounds of which the first is not
// counted: the clocks of a fresh process ramp up over its first launches -- a plain
// alternation favoured the later arm, and one round of ABCCBA still picked 5 waves for 4K 8 spp in
// one of two runs (0.8242 vs 0.8023 ms, profiles/r05/r05j_timing3_ab.jsonl).  Until the pick: 6
// waves for launches of several chunks (ahead at 16 and 64 spp), 5 for one-chunk launches.  No pixel
// depends on the variant (tests/test_gpu_regime.py forces grid changes).
// *tev: the event pair to record around this launch while it is timed.
constexpr uint32_t kBackWide = 45;
constexpr uint32_t kEnvBack[3] = {0, 33, 45};   // env arms 1, 2 (arm 0: the default share)
int ct_occupancy(const LaunchSched& ls, PtJob& j, hipEvent_t** tev, bool count)
{
    *tev = nullptr;
    j.ct_wide = g.ct_waves == 6 ? 1u : 0u;
    if (g.ct_seq_len && j.ct_slots && !j.env) {   // (test hook: the forced sequence)
        j.ct_wide = g.ct_seq[g.ct_seq_pos++ % g.ct_seq_len] == '6' ? 1u : 0u;
        return PT_OK;
    }
    Sched* s = ls.sched;
    const bool env_arms = j.env && j.ct_back_pct != 0 && !g.back_set;
    if (g.ct_waves || !j.ct_slots || !s || (j.env && !env_arms)) return PT_OK;
    const auto apply = [&](int arm) {
        if (j.env) {   // (one occupancy: the arms are back-claim shares)
            if (arm) j.ct_back_pct = kEnvBack[arm];
            return;
        }
        j.ct_wide = arm != 0 ? 1u : 0u;
        if (arm == 2 && j.ct_back_pct != 0) j.ct_back_pct = kBackWide;   // (launches that take back claims)
    };
    // only uncounted launches of the first timed launch's length are timed: a counted launch (the
    // bench's work-count pass) or one of another length sharing the geometry's schedule would bias the
    // arms' sums; they run the interim choice below.  The first timed launch fixes the
    // arms (and the length).
    const bool timeable = !count && (s->tune_nframes == 0 || s->tune_nframes == j.nframes);
    if (!s->narms && timeable) s->narms = (j.env || (j.ct_back_pct != 0 && !g.back_set)) ? 3u : 2u;
    const uint32_t per_round = s->narms == 3 ? 6u : 4u, nt = s->narms ? kTuneRounds * per_round : 0u;
    static constexpr int kOrder3[6] = {0, 1, 2, 2, 1, 0};
    const auto arm_of = [&](uint32_t t) { return s->narms == 3 ? kOrder3[t % 6] : (int)((t ^ (t >> 1)) & 1u); };
    if (s->wide >= 0) {
        apply(s->wide);
    } else if (s->tuned < nt && timeable) {
        s->tune_nframes = j.nframes;
        hipEvent_t* ev = &s->tune_ev[2 * s->tuned];
        for (int i = 0; i < 2; ++i)
            if (!ev[i]) HIP_TRY(hipEventCreate(&ev[i]));
        apply(arm_of(s->tuned++));
        *tev = ev;
    } else if (nt && s->tuned >= nt && hipEventQuery(s->tune_ev[2 * nt - 1]) == hipSuccess) {
        float t[3] = {0.f, 0.f, 0.f};
        for (uint32_t i = per_round; i < nt; ++i) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, s->tune_ev[2 * i], s->tune_ev[2 * i + 1]));
            t[arm_of(i)] += ms;
        }
        int best = 0;
        for (int a = 1; a < (int)s->narms; ++a)
            if (t[a] < t[best]) best = a;
        s->wide = (int8_t)best;
        apply(best);
    } else {
        (void)hipGetLastError();   // (hipErrorNotReady: the timed launches are still running)
        apply(j.env || j.nframes <= 8 ? 0 : 1);
    }
    return PT_OK;
}

// *ct_blocks (optional): the continuous-tiles grid launched (0: none); sched_st: see use_sched.
int launch(Dev& dv, PtJob j, hipStream_t st, bool count, uint32_t* ct_blocks = nullptr, const hipStream_t* sched_st = nullptr)
{
    LaunchSched ls;
    int rc;
    // split tiles: launches of one 8-frame chunk (a tile's half of several chunks is a short chunk
    // each, and the pool's two chunk contexts then wait on each other: 1080p 16 spp 0.452 vs 0.437 ms)
    SchedKey key = sched_key(j);
    key.split = j.nframes <= 8 ? g.split : 0u;
    if ((rc = use_dev(dv)) || (rc = use_sched(dv, key, st, &ls, key.split, sched_st))) return rc;
    j.scene = dv.dscene;
    j.queue = ls.queue;
    j.queue_next = ls.queue_next;
    j.order = ls.order;
    j.units = ls.units;
    j.nunits = ls.nunits;
    j.cost = ls.cost;
    j.err = dv.derr;
    if ((rc = use_ct_slots(dv, ls, st, &j.ct_slots, &j.ct_waves))) return rc;
    // the last-dispatched fifth of the grid (each CU's 5th block, the slowest under the SQ's
    // oldest-first issue) claims the cheapest units, for launches of <= 16 frames, whose end is a
    // large part of them (A/B, scripts/gpu_ab.sh, 20 % vs none: 1080p 8 spp 0.2533 vs 0.2561 ms,
    // env 16 spp 0.4967 vs 0.5030, 4K 8 spp 0.8217 vs 0.8309; 4K 64 spp 5.913 vs 5.763: not there)
    j.ct_back_pct = j.nframes <= 16 ? g.ct_back_pct : 0u;
    hipEvent_t* tev = nullptr;
    if ((rc = ct_occupancy(ls, j, &tev, count))) return rc;
    if (tev) HIP_TRY(hipEventRecord(tev[0], st));
    hipError_t e = pt_launch_render(j, st, count, ct_blocks);
    if (e != hipSuccess) return fail(PT_EHIP, "render launch failed: %s", hipGetErrorString(e));
    if (tev) HIP_TRY(hipEventRecord(tev[1], st));
    return queue_done(dv, ls.slot, st, j.ncols > 0 && j.nrows > 0 && j.nframes > 0);   // (pt_launch_render's early return)
}

// Chained launches (pt_render_device_chain).  A progressive renderer launches the same geometry again
// and again; back to back on one stream, each launch's end leaves the chip partly idle (c2: the queue
// runs dry ~170 us into a ~234 us launch and the last waves finish their chunks while the others have
// exited).  Consecutive chained launches alternate between two streams, so the next
// launch's blocks take the CUs the finishing waves free.  Each pixel's frames still fold in order:
// the kernel touches a tile's pixels only after the previous launch has stored them (the tile epochs,
// render_body_ct), and nothing else passes between the two launches -- each has its own tile-queue
// block, slot area and started counter, and the schedule they share is read-only while they overlap.
// Deadlock freedom: a launch waits only for its predecessor's tiles, and its stream starts it only
// after every block of the predecessor has started (hipStreamWaitValue64 on the chain's started
// counter), so the oldest running launch never waits and all of its waves are resident: it completes,
// then the next oldest, and so on (the kernel's bounded wait is a report, not a mechanism).
// A chained launch RESTARTS the chain -- its stream waits for the caller's stream and every chained
// launch before it, as a plain launch would -- when another launch came between (any launch on the
// device ends the live chain: chain_join), on the geometry's first launches (schedule not built, launch
// variant being timed), when it builds the schedule or records the costs it is built from, or when it
// is not a continuous-tiles launch.  Otherwise it CONTINUES: it does not wait for the caller's stream
// (the caller promises that nothing enqueued there since its previous chained call is needed by this
// one, include/pt_mi355.h) -- only for its predecessor's blocks to have started.  Every chained launch
// is joined back into the caller's stream (it waits for the launch's event), so work the caller
// enqueues afterwards sees it complete.
int chain_setup(Dev& dv, Sched& sc)
{
    Dev::Chain& c = dv.chain;
    for (int i = 0; i < 2; ++i) {
        if (!c.st[i]) HIP_TRY(hipStreamCreateWithFlags(&c.st[i], hipStreamNonBlocking));
        if (!c.done[i]) HIP_TRY(hipEventCreateWithFlags(&c.done[i], hipEventDisableTiming));
    }
    if (!c.ev_caller) HIP_TRY(hipEventCreateWithFlags(&c.ev_caller, hipEventDisableTiming));
    if (!c.qblk && hipMalloc(&c.qblk, 4 * PT_QUEUE_WORDS * sizeof(unsigned)) != hipSuccess)
        return fail(PT_ENOMEM, "hipMalloc(chain queue blocks) failed");
    if (!c.started) {   // (never reset: a gate evaluated early must not see a count from before a restart)
        if (hipMalloc(&c.started, sizeof(unsigned long long)) != hipSuccess)
            return fail(PT_ENOMEM, "hipMalloc(chain counter) failed");
        HIP_TRY(hipMemset(c.started, 0, sizeof(unsigned long long)));
        c.cum = 0;
    }
    if (!c.area1 && dv.dct &&
        hipMalloc(&c.area1, (size_t)dv.dct_waves * pt_ct_wave_floats() * sizeof(float)) != hipSuccess)
        return fail(PT_ENOMEM, "hipMalloc(second slot area) failed");
    if (!sc.epoch) {
        if (hipMalloc(&sc.epoch, 2 * (size_t)sc.key.ntiles * sizeof(uint32_t)) != hipSuccess)
            return fail(PT_ENOMEM, "hipMalloc(tile epochs) failed");
        HIP_TRY(hipMemset(sc.epoch, 0, 2 * (size_t)sc.key.ntiles * sizeof(uint32_t)));
        sc.chain_seq = 0;
    }
    return PT_OK;
}

int v4_launch(Dev& dv, PtV4Job j, hipStream_t st, bool count, bool* presented = nullptr, uint32_t* ct_blocks = nullptr,
              const hipStream_t* sched_st = nullptr);

// What differs between the diffuse and the v4 renderer in launch_chain: the schedule's key, whether
// the launch variant is settled (the diffuse kernels time their arms on a geometry's first launches;
// v4 has one variant), the restarting launch (launch / v4_launch) and the continuing one.
SchedKey chain_key(const PtJob& j)
{
    SchedKey k = sched_key(j);
    k.split = j.nframes <= 8 ? g.split : 0u;   // (as launch())
    return k;
}
SchedKey chain_key(const PtV4Job& j) { return sched_key(j); }   // (v4 takes whole tiles: v4_launch)
bool chain_variant_fixed(const PtJob& j, const Sched& sc)
{
    const bool env_arms = j.env && j.nframes <= 16 && g.ct_back_pct != 0 && !g.back_set;   // (ct_occupancy)
    return g.ct_waves || g.ct_seq_len || sc.wide >= 0 || (j.env && !env_arms);
}
bool chain_variant_fixed(const PtV4Job&, const Sched&) { return true; }
int chain_restart(Dev& dv, const PtJob& j, hipStream_t X, uint32_t* blocks, const hipStream_t* s)
{
    return launch(dv, j, X, false, blocks, s);
}
int chain_restart(Dev& dv, const PtV4Job& j, hipStream_t X, uint32_t* blocks, const hipStream_t* s)
{
    return v4_launch(dv, j, X, false, nullptr, blocks, s);
}
// A continuing chained launch that takes back claims (<= 16 frames) takes ALL its dynamic units from
// the back (cheapest first, after each wave's static first unit): its tail overlaps the next launch,
// so the launch-end balancing of the timed share no longer pays, and the reversed order measured faster
// (3 interleaved rounds, profiles/r06/r06u_*: c2 0.2180 vs 0.2207 ms at the timed 45 %, v4 0.3302 vs
// 0.3468 at its 20 %; the env kernel showed no difference, r06v: it keeps its timed share).  Launches of
// more frames keep claiming from the front (4K 64 spp 5.55 vs 5.62 ms with back claims, r06x).
constexpr uint32_t kChainBack = 100;
int chain_continue(Dev& dv, PtJob& j, Sched* sc, hipStream_t X, uint32_t* blocks)
{
    int rc;
    j.scene = dv.dscene;
    j.ct_back_pct = j.nframes <= 16 ? g.ct_back_pct : 0u;   // (as launch())
    LaunchSched ls;
    ls.sched = sc;
    hipEvent_t* tev = nullptr;   // (none: the variant is settled)
    if ((rc = ct_occupancy(ls, j, &tev, false))) return rc;
    if (j.ct_back_pct != 0 && !j.env && !g.back_set) j.ct_back_pct = kChainBack;
    hipError_t e = pt_launch_render(j, X, false, blocks);
    if (e != hipSuccess) return fail(PT_EHIP, "render launch failed: %s", hipGetErrorString(e));
    return PT_OK;
}
int chain_continue(Dev& dv, PtV4Job& j, Sched*, hipStream_t X, uint32_t* blocks)
{
    if (j.env_mode != PT_V4_ENV_NONE) j.env = dv.denv;   // (as v4_launch())
    j.ct_force = g.v4_ct_force;
    j.ct_back_pct = j.nframes <= 16 ? (g.back_set ? g.ct_back_pct : kChainBack) : 0u;   // (kChainBack: above)
    hipError_t e = pt_launch_v4(j, g.v4scene, X, false, nullptr, blocks);
    if (e != hipSuccess) return fail(PT_EHIP, "v4 render launch failed: %s", hipGetErrorString(e));
    return PT_OK;
}

template <typename Job>
int launch_chain(Dev& dv, Job j, hipStream_t s)
{
    int rc;
    if ((rc = use_dev(dv))) return rc;
    if (dv.chain.off) return chain_restart(dv, j, s, nullptr, nullptr);   // (a plain launch: use_sched joins the chain)
    const SchedKey key = chain_key(j);
    // (the continuous-tiles pool and a scheduled geometry: the tile epochs live in its schedule)
    Sched* sc = g.no_ct || j.ncols <= 0 || j.nrows <= 0 || j.nframes <= 0 ? nullptr : find_sched(dv, key, s);
    if (!sc) return chain_restart(dv, j, s, nullptr, nullptr);   // (a plain launch: use_sched joins the chain)
    ct_area_alloc(dv);
    if ((rc = chain_setup(dv, *sc))) return rc;
    Dev::Chain& c = dv.chain;
    if (!dv.dct || !c.area1) return chain_restart(dv, j, s, nullptr, nullptr);
    // what the plain launch's use_sched would do for this launch: build the schedule (restart), record
    // the costs it is built from (a launch that records them may continue: the overlapped launches
    // before it do not write them, and the next launch, which builds from them, restarts)
    const bool builds = sc->have_cost && (!sc->built || sc->launches % g.sched_rebuild == 0);
    const bool records = !sc->built || (sc->launches + 1) % g.sched_rebuild == 0;
    const bool cont = c.sched == sc && sc->built && !builds && chain_variant_fixed(j, *sc);
    const uint32_t seq = sc->chain_seq + 1;
    const int par = cont ? c.par ^ 1 : 0;
    hipStream_t X = c.st[par];
    j.tile_epoch = sc->epoch;
    j.chain_seq = seq;
    j.started = c.started;
    j.chain_delay = g.test_chain_delay;
    uint32_t blocks = 0;
    if (!cont) {
        // restart: after the caller's stream and every chained launch (the plain launch's use_sched joins them)
        HIP_TRY(hipEventRecord(c.ev_caller, s));
        HIP_TRY(hipStreamWaitEvent(X, c.ev_caller, 0));
        if ((rc = chain_join(dv, X))) return rc;
        HIP_TRY(hipMemsetAsync(c.qblk, 0, 4 * PT_QUEUE_WORDS * sizeof(unsigned), X));
        j.chain_wait = 0;
        if ((rc = chain_restart(dv, j, X, &blocks, &s))) return rc;   // (slot area dct)
        c.area = 0;
    } else {
        // continue: once every block of the previous launch has started
        HIP_TRY(hipStreamWaitValue64(X, c.started, c.cum, hipStreamWaitValueGte, ~0ull));
        j.chain_wait = seq - 1;
        j.queue = c.qblk + (size_t)(seq % 4u) * PT_QUEUE_WORDS;
        j.queue_next = c.qblk + (size_t)((seq + 2u) % 4u) * PT_QUEUE_WORDS;   // (the launch after next: this stream's)
        j.order = sc->order;
        j.units = sc->units;
        j.nunits = sc->units + 2 * sc->key.ntiles + 1;
        j.cost = records ? sc->cost : nullptr;
        if (records) sc->have_cost = true;
        j.err = dv.derr;
        c.area ^= 1;
        j.ct_slots = c.area ? c.area1 : dv.dct;
        j.ct_waves = dv.dct_waves;
        ++sc->launches;
        if ((rc = chain_continue(dv, j, sc, X, &blocks))) return rc;
    }
    c.cum += blocks;
    sc->chain_seq = seq;
    ++(cont ? c.continued : c.restarts);
    HIP_TRY(hipEventRecord(c.done[par], X));
    c.pending[par] = true;
    HIP_TRY(hipStreamWaitEvent(s, c.done[par], 0));
    // a launch that did not run a continuous-tiles pool published no epochs and counted no blocks:
    // the next chained launch restarts
    c.sched = blocks ? sc : nullptr;
    c.par = par;
    return PT_OK;
}

void unpin()
{
    if (g.pinned) {
        (void)hipDeviceSynchronize();
        (void)hipHostUnregister((void*)g.pinned);
    }
    g.pinned = nullptr;
    g.pinned_bytes = 0;
}

bool pin(const float* p, size_t bytes)
{
    if (g.pinned == p && g.pinned_bytes == bytes) return true;
    unpin();
    if (hipHostRegister((void*)p, bytes, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        return false;   // e.g. already page-locked by the caller: unpipelined path
    }
    g.pinned = p;
    g.pinned_bytes = bytes;
    return true;
}

// PT_FLAG_PIN_HOST (one device, without deferred readback) and `buf` page-locked: the frame job `j`
// (whole image, either renderer) is split into kBands row bands (multiples of row_align rows:
// contiguous in every layout) whose upload, render (`run(band_job)` on the device stream) and
// download overlap on three streams.  Returns with the downloads queued on g.s_out; *used = false if
// the path does not apply.
template <typename Job, typename Run>
int render_bands(float* buf, const Job& j, int32_t row_align, Run&& run, bool* used)
{
    int rc;
    const size_t bytes = (size_t)j.width * j.height * 3 * sizeof(float);
    *used = false;
    if (g.ndev != 1 || !(g.cfg.flags & PT_FLAG_PIN_HOST) || (g.cfg.flags & PT_FLAG_DEFER_READBACK)) return PT_OK;
    Dev& dv = g.dev[0];
    if ((rc = use_dev(dv))) return rc;
    if (!pin(buf, bytes)) return PT_OK;
    *used = true;
    if ((rc = ensure_dbuf(0, bytes))) return rc;
    drop_mirror();
    const int32_t w = j.width, h = j.height;
    int32_t rows = (h + kBands - 1) / kBands;
    rows = (rows + row_align - 1) / row_align * row_align;
    int k = 0;
    for (int32_t r0 = 0; r0 < h && k < kBands; r0 += rows, ++k) {
        const int32_t r1 = r0 + rows < h ? r0 + rows : h;
        const size_t off = (size_t)r0 * w * 3, len = (size_t)(r1 - r0) * w * 3 * sizeof(float);
        HIP_TRY(hipMemcpyAsync(dv.dbuf + off, buf + off, len, hipMemcpyHostToDevice, g.s_in));
        HIP_TRY(hipEventRecord(g.ev_in[k], g.s_in));
        HIP_TRY(hipStreamWaitEvent(dv.stream, g.ev_in[k], 0));
        Job b = j;
        b.row_start = r0;
        b.nrows = r1 - r0;
        b.buf = j.layout == PT_LAYOUT_TILED_PLANAR8 ? dv.dbuf : dv.dbuf + off;   // tiled: global offsets
        if ((rc = run(b))) return rc;
        HIP_TRY(hipEventRecord(g.ev_done[k], dv.stream));
        HIP_TRY(hipStreamWaitEvent(g.s_out, g.ev_done[k], 0));
        HIP_TRY(hipMemcpyAsync(buf + off, dv.dbuf + off, len, hipMemcpyDeviceToHost, g.s_out));
    }
    return PT_OK;
}

// Device d's share of a whole-frame job `j` (global geometry): its rows d::n, into its mirror.
template <typename Job>
Job shard_job(const Job& j, int d)
{
    Job b = j;
    b.buf = g.dev[d].dbuf;
    if (g.ndev > 1) {
        b.row_start = j.row_start + d;
        b.row_stride = g.ndev;
        b.nrows = shard_rows(j.nrows, g.ndev, d);
    }
    return b;
}

// Device d's rows of one tile job (tiled layout: rows are global, the buffer is full-size).
template <typename Job>
Job tile_shard_job(const Job& j, int d)
{
    Job b = j;
    b.buf = g.dev[d].dbuf;
    if (g.ndev > 1) {
        const int32_t ly0 = (int32_t)((((int64_t)d - j.row_start) % g.ndev + g.ndev) % g.ndev);
        b.row_start = j.row_start + ly0;
        b.row_stride = g.ndev;
        b.nrows = ly0 < j.nrows ? (j.nrows - 1 - ly0) / g.ndev + 1 : 0;
    }
    return b;
}

Geo geo_of(int32_t w, int32_t h, int32_t layout, int32_t tw, int32_t th)
{
    Geo geo;
    geo.w = w;
    geo.h = h;
    geo.tiled = layout == PT_LAYOUT_TILED_PLANAR8;
    geo.tw = tw;
    geo.th = th;
    return geo;
}

// One frame call on a host buffer: the job `j` (whole image) is rendered into the device mirrors
// of `buf` -- pipelined in row bands with PT_FLAG_PIN_HOST on one device, otherwise upload, render,
// download in turn (every device's share enqueued before any is waited for).
int render_frame(float* buf, PtJob j, int32_t row_align)
{
    int rc;
    const uint32_t spf = (uint32_t)g.cfg.samples_per_frame;
    bool banded = false;
    if ((rc = render_bands(buf, j, row_align, [](const PtJob& b) { return launch(g.dev[0], b, g.dev[0].stream, false); },
                           &banded)))
        return rc;
    if (banded) {
        g.frame += spf;
        HIP_TRY(hipStreamSynchronize(g.s_out));
        return sync_all();
    }
    const Geo geo = geo_of(j.width, j.height, j.layout, j.tile_w, j.tile_h);
    if ((rc = stage_in(buf, geo, Region{}))) return rc;
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = launch(g.dev[d], shard_job(j, d), g.dev[d].stream, false))) return rc;
    g.frame += spf;
    return stage_out(buf, geo, Region{});
}

int grow(Dev& dv, void** p, size_t* cap, size_t bytes)
{
    if (bytes <= *cap) return PT_OK;
    if (*p) {
        HIP_TRY(hipStreamSynchronize(dv.stream));
        (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
    }
    if (hipMalloc(p, bytes) != hipSuccess) {
        *p = nullptr;
        return fail(PT_ENOMEM, "hipMalloc(%zu) failed", bytes);
    }
    *cap = bytes;
    return PT_OK;
}

// the accumulator geometry the output stage accepts (the layouts' own constraints)
int check_tone_args(const void* accum, const void* out, int32_t w, int32_t h, int32_t layout, int32_t tw, int32_t th,
                    int32_t format)
{
    if (!accum || !out) return fail(PT_EINVAL, "null accumulator/output");
    if (w <= 0 || h <= 0 || (int64_t)w * h > (int64_t)1 << 30) return fail(PT_EINVAL, "invalid size %dx%d", w, h);
    if (format != PT_PIXEL_RGBA8 && format != PT_PIXEL_XRGB8) return fail(PT_EINVAL, "unknown pixel format %d", format);
    if (layout == PT_LAYOUT_INTERLEAVED) return PT_OK;
    if (w % 8) return fail(PT_EINVAL, "planar layouts need width %% 8 == 0 (got %d)", w);
    if (layout == PT_LAYOUT_PLANAR8) return PT_OK;
    if (layout != PT_LAYOUT_TILED_PLANAR8) return fail(PT_EINVAL, "unknown layout %d", layout);
    if (tw <= 0 || th <= 0 || tw % 8 || w % tw || h % th)
        return fail(PT_EINVAL, "tiles %dx%d do not divide %dx%d (tile width multiple of 8)", tw, th, w, h);
    return PT_OK;
}

PtToneJob tone_job(const float* accum, int32_t w, int32_t h, int32_t layout, int32_t tw, int32_t th, uint32_t* out,
                   int32_t format)
{
    PtToneJob j{};
    j.accum = accum;
    j.width = w;
    j.height = h;
    j.layout = layout;
    j.tile_w = tw;
    j.tile_h = th;
    j.out = out;
    j.format = format;
    j.fast_aces = g.v4cfg.fast_aces;     // USE_FAST_APPROXIMATE_ACES_TONEMAP (flags.h:63)
    j.fast_gamma = g.v4cfg.fast_gamma;   // USE_FAST_APPROXIMATE_GAMMA (flags.h:62)
    return j;
}

// The output stage of the mirrored accumulator, per device on its own rows: every device converts
// its mirror (its compact rows, or the full-size tiled buffer of which it owns rows d::n) and copies
// its rows of the w x h pixel image into `out` (host).  Enqueued only; the caller synchronises.
int tone_mirror(int32_t layout, int32_t tw, int32_t th, uint32_t* out, int32_t format)
{
    int rc;
    const int32_t w = g.m.width, h = g.m.height;
    const int n = g.ndev;
    for (int d = 0; d < n; ++d) {
        Dev& dv = g.dev[d];
        if ((rc = use_dev(dv))) return rc;
        const bool compact = n > 1 && layout != PT_LAYOUT_TILED_PLANAR8;
        const int32_t nr = n > 1 ? shard_rows(h, n, d) : h;
        if (nr == 0) continue;
        const int32_t rows = compact ? nr : h;   // rows of the image this device converts
        if ((rc = grow(dv, (void**)&dv.dtone_out, &dv.dtone_out_cap, (size_t)w * rows * sizeof(uint32_t)))) return rc;
        const PtToneJob j = tone_job(dv.dbuf, w, rows, layout, tw, th, dv.dtone_out, format);
        hipError_t e = pt_launch_tonemap(j, dv.stream);
        if (e != hipSuccess) return fail(PT_EHIP, "tonemap launch failed: %s", hipGetErrorString(e));
        const size_t row = (size_t)w * sizeof(uint32_t);
        if (n == 1) {
            HIP_TRY(hipMemcpyAsync(out, dv.dtone_out, row * h, hipMemcpyDeviceToHost, dv.stream));
        } else {
            const uint32_t* src = compact ? dv.dtone_out : dv.dtone_out + (size_t)d * w;
            HIP_TRY(hipMemcpy2DAsync(out + (size_t)d * w, row * n, src, compact ? row : row * n, row, nr,
                                     hipMemcpyDeviceToHost, dv.stream));
        }
    }
    return PT_OK;
}

// PT_FLAG_GATHER_ROOT (several devices, deferred accumulator): assemble the whole accumulator of the
// mirrored buffer in the root's dgather.  Every device stores its own rows there (a kernel on its own
// stream, after its renders; remote stores over its xGMI link), then the root stream waits for all of
// them.  *out = the assembled W x H x 3 buffer (mirror layout) on the root, ordered on its stream.
int gather_root(float** out)
{
    int rc;
    const Geo geo = mirror_geo();
    const int n = g.ndev;
    Dev& r = g.dev[0];
    if ((rc = use_dev(r))) return rc;
    if (n == 1) {
        *out = r.dbuf;
        return PT_OK;
    }
    for (int d = 1; d < n; ++d)
        if (!g.dev[d].peer_root)
            return fail(PT_ESTATE, "PT_FLAG_GATHER_ROOT: device %d has no peer access to device %d", g.dev[d].ordinal,
                        r.ordinal);
    const size_t bytes = (size_t)geo.w * geo.h * 3 * sizeof(float);
    if ((rc = grow(r, (void**)&r.dgather, &r.dgather_cap, bytes))) return rc;
    HIP_TRY(hipEventRecord(g.ev_root_free, r.stream));   // (the root's earlier tonemap / copy of dgather)
    for (int d = 0; d < n; ++d) {
        Dev& dv = g.dev[d];
        if ((rc = use_dev(dv))) return rc;
        if (d > 0) HIP_TRY(hipStreamWaitEvent(dv.stream, g.ev_root_free, 0));
        PtScatterJob j{};
        j.src = dv.dbuf;
        j.dst = r.dgather;
        j.width = geo.w;
        j.height = geo.h;
        j.layout = geo.tiled ? PT_LAYOUT_TILED_PLANAR8 : PT_LAYOUT_INTERLEAVED;   // (planar8 rows: same bytes)
        j.tile_w = geo.tw;
        j.tile_h = geo.th;
        j.dev = d;
        j.ndev = n;
        j.nrows = shard_rows(geo.h, n, d);
        hipError_t e = pt_launch_scatter_rows(j, dv.stream);
        if (e != hipSuccess) return fail(PT_EHIP, "gather launch failed: %s", hipGetErrorString(e));
        if (d > 0) HIP_TRY(hipEventRecord(dv.ev_gather, dv.stream));
    }
    if ((rc = use_dev(r))) return rc;
    for (int d = 1; d < n; ++d) HIP_TRY(hipStreamWaitEvent(r.stream, g.dev[d].ev_gather, 0));
    *out = r.dgather;
    return PT_OK;
}

// The output stage of the deferred accumulator into host pixels: per device on its own rows, or
// (PT_FLAG_GATHER_ROOT) gathered on the root and converted there.  Enqueued; the caller synchronises.
int tone_output(int32_t layout, int32_t tw, int32_t th, uint32_t* out, int32_t format)
{
    int rc;
    if (g.ndev == 1 || !(g.cfg.flags & PT_FLAG_GATHER_ROOT)) return tone_mirror(layout, tw, th, out, format);
    float* acc = nullptr;
    if ((rc = gather_root(&acc))) return rc;
    Dev& r = g.dev[0];
    const int32_t w = g.m.width, h = g.m.height;
    if ((rc = grow(r, (void**)&r.dtone_out, &r.dtone_out_cap, (size_t)w * h * sizeof(uint32_t)))) return rc;
    const PtToneJob j = tone_job(acc, w, h, layout, tw, th, r.dtone_out, format);
    hipError_t e = pt_launch_tonemap(j, r.stream);
    if (e != hipSuccess) return fail(PT_EHIP, "tonemap launch failed: %s", hipGetErrorString(e));
    HIP_TRY(hipMemcpyAsync(out, r.dtone_out, (size_t)w * h * sizeof(uint32_t), hipMemcpyDeviceToHost, r.stream));
    return PT_OK;
}

int check_frame_args(const float* buf, int32_t w, int32_t h, int32_t nc)
{
    if (!buf) return fail(PT_EINVAL, "null buffer");
    if (w <= 0 || h <= 0) return fail(PT_EINVAL, "invalid size %dx%d", w, h);
    if (nc != 3) return fail(PT_EINVAL, "NumChannels must be 3 (RGB f32), got %d", nc);
    if ((int64_t)w * h > (int64_t)1 << 30) return fail(PT_EINVAL, "image too large");
    if (w > kMaxDim || h > kMaxDim) return fail(PT_EINVAL, "image side > 2^24 (f32 pixel coordinates inexact)");
    return PT_OK;
}

int tiled_settings(int32_t w, int32_t h, int32_t ntx, int32_t nty, int32_t tw, int32_t th)
{
    // CheckValidSettings (Application.cpp:36-94) + the tile cover DemofoxRenderSimdTiled assumes
    if (ntx <= 0 || nty <= 0 || tw <= 0 || th <= 0) return fail(PT_EINVAL, "invalid tiling");
    if (tw % 8) return fail(PT_EINVAL, "tile width %d must be a multiple of 8 (SIMD lane width)", tw);
    if (w % 8) return fail(PT_EINVAL, "image width %d must be a multiple of 8", w);
    if (w % ntx || h % nty) return fail(PT_EINVAL, "image %dx%d not divisible into %dx%d tiles", w, h, ntx, nty);
    if (ntx * tw != w || nty * th != h) return fail(PT_EINVAL, "tiles %dx(%d) x %dx(%d) do not cover %dx%d", ntx, tw, nty, th, w, h);
    return PT_OK;
}

int check_texture(const pt_texture* t)
{
    if (!t->data) return fail(PT_EINVAL, "texture has no data");
    if (t->width <= 0 || t->height <= 0) return fail(PT_EINVAL, "invalid texture size %dx%d", t->width, t->height);
    if (t->components != 3) return fail(PT_EINVAL, "texture must have 3 components (RGB f32), got %d", t->components);
    if ((int64_t)t->width * t->height > (int64_t)1 << 28) return fail(PT_EINVAL, "texture too large");
    return PT_OK;
}

void release_env()
{
    for (int d = 0; d < g.ndev; ++d) {
        Dev& dv = g.dev[d];
        if (dv.denv) {
            (void)use_dev(dv);
            (void)hipStreamSynchronize(dv.stream);
            (void)hipFree(dv.denv);
        }
        dv.denv = nullptr;
    }
    g.env_w = g.env_h = 0;
    g.env_src = nullptr;
    g.have_env = false;
}

int upload_env(const pt_texture* t)
{
    int rc;
    if ((rc = check_texture(t))) return rc;
    const size_t bytes = (size_t)t->width * t->height * 3 * sizeof(float);
    release_env();
    for (int d = 0; d < g.ndev; ++d) {
        Dev& dv = g.dev[d];
        if ((rc = use_dev(dv))) return rc;
        if (hipMalloc(&dv.denv, bytes) != hipSuccess) {
            dv.denv = nullptr;
            release_env();
            return fail(PT_ENOMEM, "hipMalloc(env %zu) failed on device %d", bytes, dv.ordinal);
        }
        HIP_TRY(hipMemcpyAsync(dv.denv, t->data, bytes, hipMemcpyHostToDevice, dv.stream));
    }
    if ((rc = sync_all())) return rc;
    g.env_w = t->width;
    g.env_h = t->height;
    g.env_src = t->data;
    g.have_env = true;
    return PT_OK;
}

// RenderTile argument checks (simd_tiled.cpp:489-535 assumptions; Application.cpp:36-94)
int check_tile(const pt_buffer_info* b, const pt_tile_info* t)
{
    int rc;
    if (!b || !t) return fail(PT_EINVAL, "null tile/buffer info");
    if ((rc = check_frame_args(b->data, b->width, b->height, b->num_channels))) return rc;
    const int32_t tw = t->tile_width, th = t->tile_height;
    if (tw <= 0 || th <= 0 || tw % 8) return fail(PT_EINVAL, "tile width %d must be a positive multiple of 8", tw);
    if (t->tile_x < 0 || t->tile_y < 0) return fail(PT_EINVAL, "negative tile index");
    if (t->tile_min_x != t->tile_x * tw || t->tile_max_x != t->tile_min_x + tw - 1 ||
        t->tile_min_y != t->tile_y * th || t->tile_max_y != t->tile_min_y + th - 1)
        return fail(PT_EINVAL, "tile bounds inconsistent with (TileX, TileY, TileWidth, TileHeight)");
    if (t->tile_max_x >= b->width || t->tile_max_y >= b->height) return fail(PT_EINVAL, "tile outside the buffer");
    if (b->width % tw) return fail(PT_EINVAL, "buffer width %d not a multiple of tile width %d", b->width, tw);
    if (g.ndev > 1 && b->height % th)
        return fail(PT_EINVAL, "several devices: buffer height %d must be a multiple of the tile height %d", b->height, th);
    return PT_OK;
}

// the diffuse-path job of one tile at the current frame (env: the config-4 miss term)
PtJob tile_job(const pt_buffer_info* b, const pt_tile_info* t, bool env)
{
    PtJob j = base_job(nullptr, b->width, b->height);
    j.layout = PT_LAYOUT_TILED_PLANAR8;
    j.tile_w = t->tile_width;
    j.tile_h = t->tile_height;
    j.col0 = t->tile_min_x;
    j.ncols = t->tile_width;
    j.row_start = t->tile_min_y;
    j.nrows = t->tile_height;
    j.frame_first = g.frame - (uint32_t)g.cfg.samples_per_frame + 1;
    if (env) {
        j.env_w = g.env_w;
        j.env_h = g.env_h;
    }
    return j;
}

PtJob with_env(PtJob j, const Dev& dv, bool env)
{
    if (env) j.env = dv.denv;
    return j;
}

// ---- v4 helpers ----------------------------------------------------------------------------------

int v4_rebuild()
{
    if (pt_v4_build_scene(&g.v4desc, &g.v4scene))
        return fail(PT_EINVAL, "v4 scene exceeds MAX_OBJECTS (%d quads + %d spheres, %d materials; limit %d)",
                    g.v4desc.nquads, g.v4desc.nspheres, g.v4desc.nmat, PT_V4_MAX_OBJECTS);
    g.v4_scene_ready = true;
    return PT_OK;
}

int v4_ensure_scene()
{
    if (g.v4_scene_ready) return PT_OK;
    pt_v4_default_scene_desc(&g.v4desc);   // InitializeGlobalRenderResources -> InitializeScene (v4 :1650-1654)
    return v4_rebuild();
}

PtV4Job v4_job(float* buf, int32_t w, int32_t h)
{
    PtV4Job j{};
    j.buf = buf;
    j.width = w;
    j.height = h;
    j.col0 = 0;
    j.ncols = w;
    j.row_start = 0;
    j.row_stride = 1;
    j.nrows = h;
    j.layout = PT_LAYOUT_INTERLEAVED;
    j.frame_first = g.v4_frame + 1;
    j.nframes = 1;   // NUM_SAMPLES_PER_FRAME = 1: one frame per DemofoxRenderOptV4 call
    j.num_bounces = g.v4cfg.num_bounces;
    j.env_mode = PT_V4_ENV_NONE;
    j.random_jitter = g.v4cfg.random_jitter;
    j.rejection = g.v4cfg.rejection;
    j.accumulate = g.v4cfg.accumulate_frames;   // ACCUMULATE_FRAMES (flags.h:60)
    j.fast_exp = g.v4cfg.fast_exp;              // USE_FAST_APPROXIMATE_EXP (flags.h:64)
    j.default_scene = pt_v4_is_default_geometry(g.v4scene) ? 1 : 0;
    return j;
}

int v4_use_env(PtV4Job& j)
{
    if (g.v4cfg.env_mode == PT_V4_ENV_NONE) return PT_OK;
    if (!g.have_env) return fail(PT_ESTATE, "v4 env mode %d without an env map", g.v4cfg.env_mode);
    j.env_mode = g.v4cfg.env_mode;
    j.env_w = g.env_w;
    j.env_h = g.env_h;
    return PT_OK;
}

// *ct_blocks, sched_st: as launch()
int v4_launch(Dev& dv, PtV4Job j, hipStream_t st, bool count, bool* presented, uint32_t* ct_blocks, const hipStream_t* sched_st)
{
    LaunchSched ls;
    int rc;
    // v4 takes whole tiles: its per-tile kernel runs launches of < 8 frames (and PT_MI355_NO_CT=1), and
    // split tiles measured slower on the continuous-tiles one (0.3666 vs 0.3633 ms at 1080p 8 spp)
    if ((rc = use_dev(dv)) || (rc = use_sched(dv, sched_key(j), st, &ls, 0u, sched_st))) return rc;
    if (j.env_mode != PT_V4_ENV_NONE) j.env = dv.denv;
    j.queue = ls.queue;
    j.queue_next = ls.queue_next;
    j.order = ls.order;
    j.units = ls.units;
    j.nunits = ls.nunits;
    j.cost = ls.cost;
    j.err = dv.derr;
    // (the v4 pool's slots per wave: pt_v4_ct_wave_floats() <= pt_ct_wave_floats(), pt_v4.hip)
    if ((rc = use_ct_slots(dv, ls, st, &j.ct_slots, &j.ct_waves))) return rc;
    j.ct_force = g.v4_ct_force;
    j.ct_back_pct = j.nframes <= 16 ? g.ct_back_pct : 0u;   // (as launch())
    hipError_t e = pt_launch_v4(j, g.v4scene, st, count, presented, ct_blocks);
    if (e != hipSuccess) return fail(PT_EHIP, "v4 render launch failed: %s", hipGetErrorString(e));
    return queue_done(dv, ls.slot, st, j.ncols > 0 && j.nrows > 0 && j.nframes > 0);   // (pt_launch_v4's early return)
}

// The logical device a device-resident job runs on: the device holding its buffer.
int dev_of(const void* p, Dev** out)
{
    if (g.ndev == 1) {
        *out = &g.dev[0];
        return PT_OK;
    }
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return fail(PT_EINVAL, "device job buffer is not device memory");
    }
    for (int d = 0; d < g.ndev; ++d)
        if (g.dev[d].ordinal == a.device) {
            *out = &g.dev[d];
            return PT_OK;
        }
    return fail(PT_ESTATE, "device job on device %d, which the library was not initialised with", a.device);
}

int parse_device_list(const char* s, pt_config* c)
{
    if (!s || !*s) return 0;
    int n = 0;
    if (!strcmp(s, "all")) {
        int cnt = 0;
        if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0) return 0;
        for (int i = 0; i < cnt && i < PT_MAX_DEVICES; ++i) c->devices[n++] = i;
    } else {
        const char* p = s;
        while (*p && n < PT_MAX_DEVICES) {
            char* end = nullptr;
            const long v = strtol(p, &end, 10);
            if (end == p || v < 0) return 0;
            c->devices[n++] = (int32_t)v;
            p = end;
            while (*p == ',' || *p == ' ') ++p;
        }
    }
    if (n == 0) return 0;
    c->device = c->devices[0];
    c->device_count = n;
    return n;
}

void free_dev(Dev& dv)
{
    if (use_dev(dv)) return;
    if (dv.stream) (void)hipStreamSynchronize(dv.stream);
    if (dv.dbuf) (void)hipFree(dv.dbuf);
    if (dv.dcounters) (void)hipFree(dv.dcounters);
    if (dv.derr) (void)hipFree(dv.derr);
    if (dv.dct) (void)hipFree(dv.dct);
    if (dv.herr) (void)hipHostFree(dv.herr);
    if (dv.dscene) (void)hipFree(dv.dscene);
    if (dv.dqueue) (void)hipFree(dv.dqueue);
    if (dv.denv) (void)hipFree(dv.denv);
    if (dv.dtone_in) (void)hipFree(dv.dtone_in);
    if (dv.dtone_out) (void)hipFree(dv.dtone_out);
    if (dv.dgather) (void)hipFree(dv.dgather);
    if (dv.ev_gather) (void)hipEventDestroy(dv.ev_gather);
    for (Sched& sc : dv.sched)
        if (sc.used) free_sched(sc);
    for (hipEvent_t& e : dv.queue_event)
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (dv.chain.st[i]) (void)hipStreamSynchronize(dv.chain.st[i]), (void)hipStreamDestroy(dv.chain.st[i]);
        if (dv.chain.done[i]) (void)hipEventDestroy(dv.chain.done[i]);
    }
    if (dv.chain.ev_caller) (void)hipEventDestroy(dv.chain.ev_caller);
    if (dv.chain.area1) (void)hipFree(dv.chain.area1);
    if (dv.chain.qblk) (void)hipFree(dv.chain.qblk);
    if (dv.chain.started) (void)hipFree(dv.chain.started);
    if (dv.stream) (void)hipStreamDestroy(dv.stream);
    dv = Dev{};
}

int init_dev(Dev& dv, int32_t ordinal)
{
    dv = Dev{};
    dv.ordinal = ordinal;
    for (int16_t& a : dv.queue_alias) a = -1;
    HIP_TRY(hipSetDevice(ordinal));
    HIP_TRY(hipStreamCreateWithFlags(&dv.stream, hipStreamNonBlocking));
    if (hipMalloc(&dv.dcounters, kCounterSlots * sizeof(unsigned long long)) != hipSuccess)
        return fail(PT_ENOMEM, "hipMalloc(counters) failed");
    if (hipMalloc(&dv.derr, PT_ERR_WORDS * sizeof(uint32_t)) != hipSuccess) return fail(PT_ENOMEM, "hipMalloc(err) failed");
    if (hipHostMalloc(&dv.herr, PT_ERR_WORDS * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
        return fail(PT_ENOMEM, "hipHostMalloc(err) failed");
    {
        const uint32_t init[PT_ERR_WORDS] = {0u, ~0u, 0u, 0u, ~0u, ~0u};   // (pt_kernel.h: the words' meaning)
        HIP_TRY(hipMemcpy(dv.derr, init, sizeof(init), hipMemcpyHostToDevice));
        memcpy(dv.herr, init, sizeof(init));
    }
    if (hipMalloc(&dv.dqueue, (size_t)kQueueRing * PT_QUEUE_WORDS * sizeof(unsigned)) != hipSuccess)
        return fail(PT_ENOMEM, "hipMalloc(queue) failed");
    if (hipMalloc(&dv.dscene, sizeof(PtScene)) != hipSuccess) return fail(PT_ENOMEM, "hipMalloc(scene) failed");
    HIP_TRY(hipEventCreateWithFlags(&dv.ev_gather, hipEventDisableTiming));
    HIP_TRY(hipMemcpy(dv.dscene, &g.scene, sizeof(PtScene), hipMemcpyHostToDevice));
    {   // the chained-launch wait bound (pt_chain.h; test hook PT_MI355_TEST_CHAIN_POLLS, else the default --
        // set on every init: the device symbols outlive pt_shutdown)
        const char* tp = getenv("PT_MI355_TEST_CHAIN_POLLS");
        const uint32_t polls = tp ? (uint32_t)strtoul(tp, nullptr, 10) : 0u;
        HIP_TRY(pt_set_chain_polls(polls));
        HIP_TRY(pt_v4_set_chain_polls(polls));
    }
    return PT_OK;
}

}  // namespace

int pt_internal_fail(int code, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

extern "C" {

void pt_default_config(pt_config* c)
{
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->device = 0;
    c->num_bounces = 4;          // c_numBounces, scalar.cpp:19
    c->samples_per_frame = 1;    // NUM_SAMPLES_PER_FRAME, global_preprocessor_flags.h:30
    c->flags = 0;
    c->ambient[0] = c->ambient[1] = c->ambient[2] = 0.1f;   // scalar.cpp:307
    c->device_count = 1;
    c->devices[0] = 0;
    // the devices of a host that never calls pt_init (the reference-shaped drop-in): PT_MI355_DEVICES
    // = "all" or a list of HIP ordinals ("0,1,2,3"; repeats make logical shards of one GPU)
    parse_device_list(getenv("PT_MI355_DEVICES"), c);
}

int pt_init(const pt_config* cfg)
{
    pt_config c;
    if (cfg) c = *cfg;
    else pt_default_config(&c);
    if (c.num_bounces < 0 || c.num_bounces > 1024) return fail(PT_EINVAL, "num_bounces %d out of range", c.num_bounces);
    if (c.samples_per_frame < 1 || c.samples_per_frame > 65536)
        return fail(PT_EINVAL, "samples_per_frame %d out of range", c.samples_per_frame);
    if (c.device_count < 0 || c.device_count > PT_MAX_DEVICES)
        return fail(PT_EINVAL, "device_count %d out of range [0, %d]", c.device_count, PT_MAX_DEVICES);
    if (c.device_count <= 1) {   // one device: `device` (devices[] ignored)
        c.device_count = 1;
        c.devices[0] = c.device;
    }
    if (const char* cw = getenv("PT_MI355_CT_WAVES"); cw && strcmp(cw, "5") && strcmp(cw, "6") && strcmp(cw, "0"))
        return fail(PT_EINVAL, "PT_MI355_CT_WAVES=%s: 5, 6 or 0 (timed per geometry)", cw);
    if (g.inited) pt_shutdown();
    DeviceGuard guard;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    for (int d = 0; d < c.device_count; ++d)
        if (c.devices[d] < 0 || c.devices[d] >= ndev)
            return fail(PT_EHIP, "device %d not available (%d devices)", c.devices[d], ndev);
    c.device = c.devices[0];
    g.cfg = c;
    pt_build_demofox_scene(&g.scene, c.ambient);
    int rc;
    g.ndev = c.device_count;
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = init_dev(g.dev[d], c.devices[d]))) {
            g.inited = true;   // release what was created
            pt_shutdown();
            return rc;
        }
    // peer access to the root for PT_FLAG_GATHER_ROOT (MI355X nodes: every GPU pair over xGMI)
    for (int d = 0; d < g.ndev; ++d) {
        Dev& dv = g.dev[d];
        if (dv.ordinal == g.dev[0].ordinal) {
            dv.peer_root = true;
            continue;
        }
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, dv.ordinal, g.dev[0].ordinal) != hipSuccess || !can) continue;
        HIP_TRY(hipSetDevice(dv.ordinal));
        const hipError_t e = hipDeviceEnablePeerAccess(g.dev[0].ordinal, 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) dv.peer_root = true;
        (void)hipGetLastError();
    }
    HIP_TRY(hipSetDevice(g.dev[0].ordinal));
    HIP_TRY(hipEventCreateWithFlags(&g.ev_root_free, hipEventDisableTiming));
    HIP_TRY(hipStreamCreateWithFlags(&g.s_in, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&g.s_out, hipStreamNonBlocking));
    for (int k = 0; k < kBands; ++k) {
        HIP_TRY(hipEventCreateWithFlags(&g.ev_in[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&g.ev_done[k], hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&g.ev_q, hipEventDisableTiming));
    g.frame = 0;
    g.ring_guard_cap = ~0u;
    g.no_ct = getenv("PT_MI355_NO_CT") && !strcmp(getenv("PT_MI355_NO_CT"), "1");
    g.test_chain_delay = getenv("PT_MI355_TEST_CHAIN_DELAY") ? (uint32_t)strtoul(getenv("PT_MI355_TEST_CHAIN_DELAY"), nullptr, 10) : 0u;
    g.sched_rebuild = getenv("PT_MI355_SCHED_REBUILD") ? std::max<unsigned long long>(2ull, strtoull(getenv("PT_MI355_SCHED_REBUILD"), nullptr, 10))
                                                        : kSchedRebuildDefault;
    g.unit_mult = getenv("PT_MI355_UNIT_MULT") ? std::max<uint32_t>(1u, (uint32_t)strtoul(getenv("PT_MI355_UNIT_MULT"), nullptr, 10)) : 2u;
    g.v4_ct_force = getenv("PT_MI355_V4_CT") && !strcmp(getenv("PT_MI355_V4_CT"), "1");
    g.ct_back_pct = 20;
    g.back_set = false;
    if (const char* bk = getenv("PT_MI355_BACK")) g.ct_back_pct = (uint32_t)strtoul(bk, nullptr, 10), g.back_set = true;
    g.ct_waves = 0;
    if (const char* cw = getenv("PT_MI355_CT_WAVES")) g.ct_waves = (uint32_t)strtoul(cw, nullptr, 10);
    g.ct_seq_len = g.ct_seq_pos = 0;
    if (const char* sq = getenv("PT_MI355_CT_WAVES_SEQ")) {
        for (const char* c = sq; *c && g.ct_seq_len < sizeof(g.ct_seq); ++c)
            if (*c == '5' || *c == '6') g.ct_seq[g.ct_seq_len++] = *c;
    }
    // test hook: PT_MI355_TEST_BAD_ENTRY=<position> overwrites that entry of every schedule built with
    // ~0u (a tile outside the launch) -- the queue's entry guard must report it (tests/test_gpu_guards.py)
    g.test_bad_entry = -1;
    if (const char* be = getenv("PT_MI355_TEST_BAD_ENTRY")) g.test_bad_entry = (int64_t)strtoll(be, nullptr, 10);
    g.split = 1;
    if (const char* sp = getenv("PT_MI355_SPLIT")) g.split = (uint32_t)strtoul(sp, nullptr, 10);
    if (const char* cap = getenv("PT_MI355_RING_GUARD_CAP")) {
        const unsigned long v = strtoul(cap, nullptr, 10);
        if (v > 0 && v < 0xfffffffful) g.ring_guard_cap = (uint32_t)v;
    }
    g.inited = true;
    return PT_OK;
}

void pt_shutdown(void)
{
    if (!g.inited) return;
    DeviceGuard guard;
    for (int d = 0; d < g.ndev; ++d) free_dev(g.dev[d]);
    if (g.ndev > 0) (void)hipSetDevice(g.cfg.devices[0]);
    unpin();
    for (int k = 0; k < kBands; ++k) {
        if (g.ev_in[k]) (void)hipEventDestroy(g.ev_in[k]);
        if (g.ev_done[k]) (void)hipEventDestroy(g.ev_done[k]);
    }
    if (g.ev_q) (void)hipEventDestroy(g.ev_q);
    if (g.ev_root_free) (void)hipEventDestroy(g.ev_root_free);
    if (g.s_in) (void)hipStreamDestroy(g.s_in);
    if (g.s_out) (void)hipStreamDestroy(g.s_out);
    g = State{};
}

const char* pt_last_error(void) { return g_err; }

int pt_set_frame(uint32_t frame)
{
    if (frame >= kMaxFrame) return fail(PT_EINVAL, "frame %u >= 2^24", frame);
    g.frame = frame;
    return PT_OK;
}

uint32_t pt_get_frame(void) { return g.frame; }

int pt_render_scalar(float* buf, int32_t w, int32_t h, int32_t nc)
{
    int rc;
    if ((rc = check_frame_args(buf, w, h, nc)) || (rc = ensure_init())) return rc;
    if ((rc = check_frame_budget((uint32_t)g.cfg.samples_per_frame))) return rc;
    DeviceGuard guard;
    return render_frame(buf, base_job(nullptr, w, h), 8);
}

int pt_render_simd(float* buf, int32_t w, int32_t h, int32_t nc)
{
    int rc;
    if ((rc = check_frame_args(buf, w, h, nc)) || (rc = ensure_init())) return rc;
    if (w % 8) return fail(PT_EINVAL, "image width %d must be a multiple of 8 (SIMD lane width)", w);
    if ((rc = check_frame_budget((uint32_t)g.cfg.samples_per_frame))) return rc;
    DeviceGuard guard;
    PtJob j = base_job(nullptr, w, h);
    j.layout = PT_LAYOUT_PLANAR8;
    return render_frame(buf, j, 8);
}

int pt_render_simd_tiled(float* buf, int32_t w, int32_t h, int32_t ntx, int32_t nty, int32_t tw, int32_t th, int32_t nc)
{
    int rc;
    if ((rc = check_frame_args(buf, w, h, nc)) || (rc = ensure_init())) return rc;
    if ((rc = tiled_settings(w, h, ntx, nty, tw, th))) return rc;
    if ((rc = check_frame_budget((uint32_t)g.cfg.samples_per_frame))) return rc;
    DeviceGuard guard;
    PtJob j = base_job(nullptr, w, h);
    j.layout = PT_LAYOUT_TILED_PLANAR8;
    j.tile_w = tw;
    j.tile_h = th;
    return render_frame(buf, j, th);
}

int pt_set_env_map(const pt_texture* tex)
{
    int rc;
    if ((rc = ensure_init())) return rc;
    DeviceGuard guard;
    if (!tex) {
        release_env();
        return PT_OK;
    }
    return upload_env(tex);
}

static int ensure_env(const pt_texture* tex)
{
    int rc;
    if ((rc = check_texture(tex))) return rc;
    if (!g.have_env || g.env_src != tex->data || g.env_w != tex->width || g.env_h != tex->height)
        return upload_env(tex);
    return PT_OK;
}

int pt_render_simt_textured(float* buf, int32_t w, int32_t h, int32_t ntx, int32_t nty, int32_t tw, int32_t th,
                            int32_t nc, const pt_texture* tex)
{
    int rc;
    if (!tex) return fail(PT_EINVAL, "null texture");
    if ((rc = check_frame_args(buf, w, h, nc)) || (rc = ensure_init())) return rc;
    if ((rc = tiled_settings(w, h, ntx, nty, tw, th)) || (rc = check_texture(tex))) return rc;
    if ((rc = check_frame_budget((uint32_t)g.cfg.samples_per_frame))) return rc;
    DeviceGuard guard;
    if ((rc = ensure_env(tex))) return rc;
    PtJob j = base_job(nullptr, w, h);
    j.layout = PT_LAYOUT_TILED_PLANAR8;   // RenderTile, simt_textured.cpp:491-533
    j.tile_w = tw;
    j.tile_h = th;
    j.env_w = g.env_w;
    j.env_h = g.env_h;
    const uint32_t spf = (uint32_t)g.cfg.samples_per_frame;
    bool banded = false;
    if ((rc = render_bands(buf, j, th, [](const PtJob& b) {
             return launch(g.dev[0], with_env(b, g.dev[0], true), g.dev[0].stream, false);
         }, &banded)))
        return rc;
    if (banded) {
        g.frame += spf;
        HIP_TRY(hipStreamSynchronize(g.s_out));
        return sync_all();
    }
    const Geo geo = geo_of(w, h, j.layout, tw, th);
    if ((rc = stage_in(buf, geo, Region{}))) return rc;
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = launch(g.dev[d], with_env(shard_job(j, d), g.dev[d], true), g.dev[d].stream, false))) return rc;
    g.frame += spf;
    return stage_out(buf, geo, Region{});
}

int pt_begin_frame(void)
{
    int rc;
    if ((rc = ensure_init())) return rc;
    if ((rc = check_frame_budget((uint32_t)g.cfg.samples_per_frame))) return rc;
    g.frame += (uint32_t)g.cfg.samples_per_frame;
    return PT_OK;
}

int pt_render_tile(const pt_buffer_info* b, const pt_tile_info* t)
{
    int rc;
    if ((rc = ensure_init()) || (rc = check_tile(b, t))) return rc;
    if (g.frame < (uint32_t)g.cfg.samples_per_frame)
        return fail(PT_ESTATE, "RenderTile before the first frame was started (pt_begin_frame)");
    DeviceGuard guard;
    const Geo geo = geo_of(b->width, b->height, PT_LAYOUT_TILED_PLANAR8, t->tile_width, t->tile_height);
    Region rg;
    rg.whole = false;
    rg.tile_x = t->tile_x;
    rg.tile_y = t->tile_y;
    if ((rc = stage_in(b->data, geo, rg))) return rc;
    const PtJob j = tile_job(b, t, false);
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = launch(g.dev[d], tile_shard_job(j, d), g.dev[d].stream, false))) return rc;
    return stage_out(b->data, geo, rg);
}

int pt_readback(float* buf)
{
    if (!g.inited || !g.m.valid || buf != g.m.host)
        return fail(PT_ESTATE, "no deferred device accumulator for this buffer");
    DeviceGuard guard;
    int rc;
    const Geo geo = mirror_geo();
    if (g.ndev > 1 && (g.cfg.flags & PT_FLAG_GATHER_ROOT)) {   // assembled on the root: one copy
        float* acc = nullptr;
        if ((rc = gather_root(&acc))) return rc;
        HIP_TRY(hipMemcpyAsync(buf, acc, g.m.bytes, hipMemcpyDeviceToHost, g.dev[0].stream));
        return sync_all();
    }
    for (int d = 0; d < g.ndev; ++d)
        if ((rc = use_dev(g.dev[d])) || (rc = xfer(d, geo, buf, false, Region{}))) return rc;
    return sync_all();
}

int pt_gather_root(const float* buf, const float** device_accum)
{
    if (!device_accum) return fail(PT_EINVAL, "null output pointer");
    if (!g.inited || !g.m.valid || buf != g.m.host)
        return fail(PT_ESTATE, "no deferred device accumulator for this buffer");
    DeviceGuard guard;
    int rc;
    float* acc = nullptr;
    if ((rc = gather_root(&acc)) || (rc = sync_all())) return rc;
    *device_accum = acc;
    return PT_OK;
}

int pt_release_buffer(const void* buf)
{
    if (!g.inited) return PT_OK;
    DeviceGuard guard;
    if (!buf || buf == (const void*)g.m.host) {
        (void)sync_all();   // nothing in flight may still copy into it
        drop_mirror();
    }
    if (g.pinned && (!buf || buf == (const void*)g.pinned)) unpin();
    return PT_OK;
}

static int device_job(const pt_device_job* dj, PtJob* j)
{
    if (!dj || !dj->buf) return fail(PT_EINVAL, "null device job/buffer");
    if (dj->width <= 0 || dj->height <= 0 || dj->nrows < 0 || dj->row_stride <= 0 || dj->row_start < 0)
        return fail(PT_EINVAL, "invalid device job geometry");
    if (dj->width > kMaxDim || dj->height > kMaxDim)
        return fail(PT_EINVAL, "image side > 2^24 (f32 pixel coordinates inexact)");
    if (dj->nrows > 0 && dj->row_start + (int64_t)(dj->nrows - 1) * dj->row_stride >= dj->height)
        return fail(PT_EINVAL, "row shard exceeds the image height");
    if (dj->layout != PT_LAYOUT_INTERLEAVED && dj->layout != PT_LAYOUT_PLANAR8)
        return fail(PT_EINVAL, "device jobs support the interleaved and planar8 layouts");
    if (dj->layout == PT_LAYOUT_PLANAR8 && dj->width % 8) return fail(PT_EINVAL, "planar8 needs width % 8 == 0");
    if (dj->frame_first < 1 || dj->nframes < 0 || (uint64_t)dj->frame_first + (uint64_t)dj->nframes > kMaxFrame)
        return fail(PT_EINVAL, "frame range [%u, +%d) invalid", dj->frame_first, dj->nframes);
    if (dj->num_bounces < 0 || dj->num_bounces > 1024) return fail(PT_EINVAL, "num_bounces out of range");
    *j = base_job(dj->buf, dj->width, dj->height);
    j->row_start = dj->row_start;
    j->row_stride = dj->row_stride;
    j->nrows = dj->nrows;
    j->layout = dj->layout;
    j->frame_first = dj->frame_first;
    j->nframes = dj->nframes;
    j->num_bounces = dj->num_bounces;
    if (dj->use_env) {
        if (!g.have_env) return fail(PT_ESTATE, "use_env without an env map (pt_set_env_map)");
        j->env_w = g.env_w;
        j->env_h = g.env_h;
    }
    return PT_OK;
}

#if PT_DIAG
static void diag_dump(const unsigned long long* h)
{
    fprintf(stderr, "PT_DIAG cycles: A %llu take %llu dir %llu trace %llu shade %llu C %llu tile %llu\n",
            h[PT_CNT_N + 0], h[PT_CNT_N + 1], h[PT_CNT_N + 2], h[PT_CNT_N + 3], h[PT_CNT_N + 4], h[PT_CNT_N + 5],
            h[PT_CNT_N + 6]);
    fprintf(stderr, "PT_DIAG wave lifetimes %llu memtime ticks, %llu realtime (100 MHz) ticks\n", h[PT_CNT_N + 7],
            h[PT_CNT_N + 10]);
    const unsigned long long r0 = h[PT_CNT_N + 12];
    fprintf(stderr, "PT_DIAG realtime (us from first start): last start %.1f, first end %.1f, last end %.1f\n",
            (h[PT_CNT_N + 8] - r0) * 0.01, (h[PT_CNT_N + 9] - r0) * 0.01, (h[PT_CNT_N + 11] - r0) * 0.01);
    if (const char* path = getenv("PT_DIAG_OUT")) {
        FILE* f = fopen(path, "wb");
        if (f) {
            fwrite(h + 32, sizeof(unsigned long long), 4 * 65536 + 96 * 65536, f);
            fclose(f);
        }
    }
}
#endif

int pt_tonemap_device(const float* accum, int32_t w, int32_t h, int32_t layout, int32_t tw, int32_t th, uint32_t* out,
                      int32_t format, void* stream)
{
    int rc;
    if ((rc = ensure_init()) || (rc = check_tone_args(accum, out, w, h, layout, tw, th, format))) return rc;
    DeviceGuard guard;
    Dev* dv = nullptr;
    if ((rc = dev_of(accum, &dv)) || (rc = use_dev(*dv))) return rc;
    const PtToneJob j = tone_job(accum, w, h, layout, tw, th, out, format);
    hipError_t e = pt_launch_tonemap(j, (hipStream_t)stream);
    if (e != hipSuccess) return fail(PT_EHIP, "tonemap launch failed: %s", hipGetErrorString(e));
    return PT_OK;
}

int pt_tonemap(const float* accum, int32_t w, int32_t h, int32_t layout, int32_t tw, int32_t th, uint32_t* out,
               int32_t format)
{
    int rc;
    if ((rc = ensure_init()) || (rc = check_tone_args(accum, out, w, h, layout, tw, th, format))) return rc;
    DeviceGuard guard;
    const size_t in_bytes = (size_t)w * h * 3 * sizeof(float), out_bytes = (size_t)w * h * sizeof(uint32_t);
    const bool tiled = layout == PT_LAYOUT_TILED_PLANAR8;
    if (g.m.valid && accum == g.m.host && g.m.bytes == in_bytes && g.m.width == w && g.m.height == h &&
        (g.ndev == 1 || (g.m.tiled == tiled && (!tiled || (g.m.tile_w == tw && g.m.tile_h == th))))) {
        // the deferred accumulator is already in HBM: each device converts its own rows (or the root
        // converts the gathered image, PT_FLAG_GATHER_ROOT)
        if ((rc = tone_output(layout, tw, th, out, format))) return rc;
        return sync_all();
    }
    Dev& dv = g.dev[0];
    if ((rc = use_dev(dv))) return rc;
    if ((rc = grow(dv, (void**)&dv.dtone_in, &dv.dtone_in_cap, in_bytes))) return rc;
    HIP_TRY(hipMemcpyAsync(dv.dtone_in, accum, in_bytes, hipMemcpyHostToDevice, dv.stream));
    if ((rc = grow(dv, (void**)&dv.dtone_out, &dv.dtone_out_cap, out_bytes))) return rc;
    const PtToneJob j = tone_job(dv.dtone_in, w, h, layout, tw, th, dv.dtone_out, format);
    hipError_t e = pt_launch_tonemap(j, dv.stream);
    if (e != hipSuccess) return fail(PT_EHIP, "tonemap launch failed: %s", hipGetErrorString(e));
    HIP_TRY(hipMemcpyAsync(out, dv.dtone_out, out_bytes, hipMemcpyDeviceToHost, dv.stream));
    HIP_TRY(hipStreamSynchronize(dv.stream));
    return PT_OK;
}

int pt_render_device(const pt_device_job* dj, void* stream)
{
    int rc;
    PtJob j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if ((rc = ensure_init()) || (rc = device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv))) return rc;
    if (dj->use_env) j.env = dv->denv;
#if PT_DIAG   // diagnostic build: with PT_DIAG_OUT set, a device launch records and dumps its
              // timeline (synchronous); without it launches run as usual (warm-up at full clocks)
    if (!getenv("PT_DIAG_OUT")) return launch(*dv, j, (hipStream_t)stream, false);
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(dv->dcounters, 0, kCounterSlots * sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(dv->dcounters + PT_CNT_N + 9, 0xff, sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(dv->dcounters + PT_CNT_N + 12, 0xff, sizeof(unsigned long long), st));
    j.counters = dv->dcounters;
    if ((rc = launch(*dv, j, st, false))) return rc;
    static unsigned long long h[kCounterSlots];
    HIP_TRY(hipMemcpyAsync(h, dv->dcounters, sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    diag_dump(h);
    return PT_OK;
#else
    return launch(*dv, j, (hipStream_t)stream, false);
#endif
}

int pt_render_device_chain(const pt_device_job* dj, void* stream)
{
    int rc;
    PtJob j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if ((rc = ensure_init()) || (rc = device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv))) return rc;
    if (dj->use_env) j.env = dv->denv;
#if PT_DIAG
    if (getenv("PT_DIAG_OUT")) return pt_render_device(dj, stream);   // (the diagnostic timeline: one launch)
#endif
    return launch_chain(*dv, j, (hipStream_t)stream);
}

int pt_chain_counts(uint64_t* restarts, uint64_t* continued)
{
    if (!restarts || !continued) return fail(PT_EINVAL, "null output");
    *restarts = *continued = 0;
    for (int d = 0; d < (g.inited ? g.ndev : 0); ++d) {
        *restarts += g.dev[d].chain.restarts;
        *continued += g.dev[d].chain.continued;
    }
    return PT_OK;
}

int pt_render_device_present(const pt_device_job* dj, uint32_t* pixels, int32_t format, void* stream)
{
    int rc;
    PtJob j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if (!pixels) return fail(PT_EINVAL, "null pixel buffer");
    if (format != PT_PIXEL_RGBA8 && format != PT_PIXEL_XRGB8) return fail(PT_EINVAL, "unknown pixel format %d", format);
    if ((rc = ensure_init()) || (rc = device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv))) return rc;
    if (dj->use_env) j.env = dv->denv;
    j.pix_out = pixels;
    j.pix_xrgb = format == PT_PIXEL_XRGB8;
    return launch(*dv, j, (hipStream_t)stream, false);
}

int pt_launch_variant(const pt_device_job* dj, int32_t* waves, int32_t* back_pct)
{
    int rc;
    PtJob j;
    Dev* dv = nullptr;
    if (!waves || !back_pct) return fail(PT_EINVAL, "null output");
    *waves = 0;
    *back_pct = 0;
    if ((rc = ensure_init()) || (rc = device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv))) return rc;
    if (dj->use_env) j.env = dv->denv;
    if (g.no_ct) return PT_OK;   // (the per-tile pools)
    const bool back = j.nframes <= 16;
    const uint32_t dflt = back ? g.ct_back_pct : 0u;
    if (g.ct_waves) {   // fixed (launch(), ct_occupancy)
        *waves = j.env ? pt_ct_env_waves() : (int32_t)g.ct_waves;
        *back_pct = (int32_t)dflt;
        return PT_OK;
    }
    SchedKey key = sched_key(j);
    key.split = j.nframes <= 8 ? g.split : 0u;
    if (key.ntiles < kSchedMinTiles) {   // never scheduled, never timed: the fixed fallback (ct_occupancy)
        *waves = j.env ? pt_ct_env_waves() : 5;
        *back_pct = (int32_t)dflt;
        return PT_OK;
    }
    for (const Sched& s : dv->sched) {
        if (!s.used || !(s.key == key) || s.wide < 0) continue;
        if (j.env) {
            *waves = pt_ct_env_waves();
            *back_pct = (int32_t)(s.wide && back && !g.back_set ? kEnvBack[s.wide] : dflt);
        } else {
            *waves = s.wide ? 6 : 5;
            *back_pct = (int32_t)(s.wide == 2 && back ? kBackWide : dflt);
        }
        return PT_OK;
    }
    return PT_OK;   // (undecided)
}

int pt_count_device(const pt_device_job* dj, void* stream, pt_work_counts* out)
{
    int rc;
    PtJob j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if (!out) return fail(PT_EINVAL, "null counts");
    if ((rc = ensure_init()) || (rc = device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv)) || (rc = use_dev(*dv))) return rc;
    if (dj->use_env) j.env = dv->denv;
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(dv->dcounters, 0, kCounterSlots * sizeof(unsigned long long), st));
#if PT_DIAG
    HIP_TRY(hipMemsetAsync(dv->dcounters + PT_CNT_N + 9, 0xff, sizeof(unsigned long long), st));    // min
    HIP_TRY(hipMemsetAsync(dv->dcounters + PT_CNT_N + 12, 0xff, sizeof(unsigned long long), st));   // min
#endif
    j.counters = dv->dcounters;
    if ((rc = launch(*dv, j, st, true))) return rc;
    static unsigned long long h[kCounterSlots];
    HIP_TRY(hipMemcpyAsync(h, dv->dcounters, sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
#if PT_DIAG
    diag_dump(h);
#endif
    if ((rc = sync_all())) return rc;   // the launch's error words
    out->segments = h[PT_CNT_SEGMENTS];
    out->lane_slots = h[PT_CNT_LANE_SLOTS];
    out->samples = h[PT_CNT_SAMPLES];
    out->escaped = h[PT_CNT_ESCAPED];
    out->primary = h[PT_CNT_PRIMARY];
    out->quad_fallbacks = h[PT_CNT_FALLBACK];
    out->sphere_fallbacks = 0;
    out->sky_skipped = h[PT_CNT_SKY];
    return PT_OK;
}

int pt_check_device_errors(void)
{
    if (!g.inited) return PT_OK;
    DeviceGuard guard;
    return sync_all();
}

int32_t pt_initialized_device(void) { return g.inited ? g.dev[0].ordinal : -1; }

int32_t pt_build_checked(void) { return PT_CHECKED ? 1 : 0; }

int32_t pt_device_count(void) { return g.inited ? g.ndev : 0; }

int32_t pt_device_ordinal(int32_t i) { return g.inited && i >= 0 && i < g.ndev ? g.dev[i].ordinal : -1; }

int pt_unpin_host(const void* buf)
{
    if (!g.inited || !g.pinned) return PT_OK;
    if (buf && buf != (const void*)g.pinned) return PT_OK;
    DeviceGuard guard;
    unpin();
    return PT_OK;
}

// ---- v4 renderer -------------------------------------------------------------------------------

void pt_v4_default_config(pt_v4_config* c)
{
    if (!c) return;
    c->env_mode = PT_V4_ENV_EQUIRECT;   // USE_ENV_MAP 1, USE_ENV_CUBEMAP 0
    c->random_jitter = 1;               // USE_RANDOM_JITTER_TEXTURE_SAMPLING 1
    c->rejection = 1;                   // USE_UNIT_VECTOR_REJECTION_SAMPLING 1
    c->num_bounces = 8;                 // c_numBounces, v4 :23
    c->output_to_screen = 1;            // OUTPUT_TO_SCREEN = !RENDER_OFFLINE
    c->accumulate_frames = 1;           // ACCUMULATE_FRAMES 1
    c->fast_aces = 1;                   // USE_FAST_APPROXIMATE_ACES_TONEMAP 1
    c->fast_gamma = 1;                  // USE_FAST_APPROXIMATE_GAMMA 1
    c->fast_exp = 1;                    // USE_FAST_APPROXIMATE_EXP 1
}

int pt_v4_set_config(const pt_v4_config* c)
{
    if (!c) return fail(PT_EINVAL, "null v4 config");
    if (c->env_mode < PT_V4_ENV_NONE || c->env_mode > PT_V4_ENV_CUBEMAP) return fail(PT_EINVAL, "unknown env mode %d", c->env_mode);
    if (c->num_bounces < 0 || c->num_bounces > 1024) return fail(PT_EINVAL, "num_bounces %d out of range", c->num_bounces);
    g.v4cfg = *c;
    g.v4cfg.random_jitter = c->random_jitter != 0;
    g.v4cfg.rejection = c->rejection != 0;
    g.v4cfg.output_to_screen = c->output_to_screen != 0;
    g.v4cfg.accumulate_frames = c->accumulate_frames != 0;
    g.v4cfg.fast_aces = c->fast_aces != 0;
    g.v4cfg.fast_gamma = c->fast_gamma != 0;
    g.v4cfg.fast_exp = c->fast_exp != 0;
    return PT_OK;
}

int pt_v4_get_config(pt_v4_config* c)
{
    if (!c) return fail(PT_EINVAL, "null v4 config");
    *c = g.v4cfg;
    return PT_OK;
}

int pt_v4_initialize_global_render_resources(void)
{
    int rc;
    if ((rc = ensure_init())) return rc;
    return v4_ensure_scene();
}

int pt_v4_reinitialize_render_tile_data(void)
{
    // Resize reallocated the render target (Application.cpp:142-154): the old buffer is gone, so
    // neither its page-lock nor its deferred device copy may outlive it (dropped, not written back)
    return pt_release_buffer(nullptr);
}

int pt_v4_initialize_scene(void)
{
    pt_v4_default_scene_desc(&g.v4desc);
    return v4_rebuild();
}

int pt_v4_clear_scene(void)
{
    memset(&g.v4desc, 0, sizeof(g.v4desc));
    return v4_rebuild();
}

int pt_v4_add_material(const pt_v4_material* m)
{
    int rc;
    if (!m) return fail(PT_EINVAL, "null material");
    if ((rc = v4_ensure_scene())) return rc;
    if (g.v4desc.nmat >= PT_V4_MAX_OBJECTS) return fail(PT_EINVAL, "more than MAX_MATERIALS (%d) materials", PT_V4_MAX_OBJECTS);
    static_assert(sizeof(pt_v4_material) == sizeof(PtV4Mat), "material layout");
    memcpy(&g.v4desc.mat[g.v4desc.nmat], m, sizeof(PtV4Mat));
    const int idx = g.v4desc.nmat++;
    if ((rc = v4_rebuild())) return rc;
    return idx;   // AddMaterialToScene returns scene.NumMaterials++ (v4 :1387)
}

int pt_v4_add_quad(const float v[12])
{
    int rc;
    if (!v) return fail(PT_EINVAL, "null quad");
    if ((rc = v4_ensure_scene())) return rc;
    if (g.v4desc.nquads + g.v4desc.nspheres >= PT_V4_MAX_OBJECTS)
        return fail(PT_EINVAL, "more than MAX_OBJECTS (%d) objects", PT_V4_MAX_OBJECTS);
    memcpy(g.v4desc.quad[g.v4desc.nquads++], v, 12 * sizeof(float));
    if ((rc = v4_rebuild())) return rc;
    return g.v4desc.nquads;   // v4 :1394
}

int pt_v4_add_sphere(const float pr[4])
{
    int rc;
    if (!pr) return fail(PT_EINVAL, "null sphere");
    if ((rc = v4_ensure_scene())) return rc;
    if (g.v4desc.nquads + g.v4desc.nspheres >= PT_V4_MAX_OBJECTS)
        return fail(PT_EINVAL, "more than MAX_OBJECTS (%d) objects", PT_V4_MAX_OBJECTS);
    memcpy(g.v4desc.sphere[g.v4desc.nspheres++], pr, 4 * sizeof(float));
    if ((rc = v4_rebuild())) return rc;
    return g.v4desc.nquads;   // v4 :1400 returns NumQuadObjects
}

int pt_v4_set_frame(uint32_t frame)
{
    if (frame >= kMaxFrame) return fail(PT_EINVAL, "frame %u >= 2^24", frame);
    g.v4_frame = frame;
    return PT_OK;
}

uint32_t pt_v4_get_frame(void) { return g.v4_frame; }

int pt_v4_get_scene_tables(float* out, int32_t n, int32_t* nq, int32_t* ns)
{
    int rc;
    if ((rc = v4_ensure_scene())) return rc;
    const PtV4Scene& s = g.v4scene;
    const int32_t need = 18 * s.nquads + 4 * s.nspheres + 17 * PT_V4_MAX_OBJECTS;
    if (nq) *nq = s.nquads;
    if (ns) *ns = s.nspheres;
    if (!out || n < need) return need;
    float* o = out;
    for (int i = 0; i < s.nquads; ++i) {
        memcpy(o, &s.quad[i], sizeof(PtV4Quad));
        o += 18;
    }
    for (int i = 0; i < s.nspheres; ++i) {
        memcpy(o, s.sph[i], 4 * sizeof(float));
        o += 4;
    }
    memcpy(o, s.mat, sizeof(s.mat));
    return need;
}

int pt_render_opt_v4(float* buf, int32_t w, int32_t h, int32_t ntx, int32_t nty, int32_t tw, int32_t th, int32_t nc,
                     const pt_texture* tex, void* screen)
{
    int rc;
    if ((rc = check_frame_args(buf, w, h, nc)) || (rc = ensure_init())) return rc;
    if ((rc = tiled_settings(w, h, ntx, nty, tw, th))) return rc;
    if ((int64_t)ntx * nty > 1024) return fail(PT_EINVAL, "%d x %d tiles exceed NumMaxThreads (1024, v4 :1341)", ntx, nty);
    if ((rc = v4_ensure_scene())) return rc;
    if (g.v4_frame + 1u >= kMaxFrame) return fail(PT_EINVAL, "v4 frame counter exceeds the exact f32 range 2^24");
    DeviceGuard guard;
    if (g.v4cfg.env_mode != PT_V4_ENV_NONE) {
        if (!tex) return fail(PT_EINVAL, "env mode %d needs a texture", g.v4cfg.env_mode);
        if ((rc = ensure_env(tex))) return rc;
    }
    PtV4Job j = v4_job(nullptr, w, h);
    j.layout = PT_LAYOUT_TILED_PLANAR8;   // RenderTile v4 :1186-1191
    j.tile_w = tw;
    j.tile_h = th;
    if ((rc = v4_use_env(j))) return rc;
    bool banded = false;   // PT_FLAG_PIN_HOST: bands of whole tile rows
    if ((rc = render_bands(buf, j, th, [](const PtV4Job& b) { return v4_launch(g.dev[0], b, g.dev[0].stream, false); },
                           &banded)))
        return rc;
    const Geo geo = geo_of(w, h, PT_LAYOUT_TILED_PLANAR8, tw, th);
    bool presented = false;   // the render launch wrote the screen pixels (fused OutputToScreen)
    if (!banded) {
        if ((rc = stage_in(buf, geo, Region{}))) return rc;
        for (int d = 0; d < g.ndev; ++d) {
            PtV4Job jd = shard_job(j, d);
            // RenderTile + OutputToScreen in one pass, as the reference's worker does per tile (v4
            // :1562-1564): one device, the presenting configuration (pt_launch_v4 decides)
            if (screen && g.v4cfg.output_to_screen && g.ndev == 1) {
                Dev& dv = g.dev[d];
                if ((rc = grow(dv, (void**)&dv.dtone_out, &dv.dtone_out_cap, (size_t)w * h * sizeof(uint32_t)))) return rc;
                jd.pix_out = dv.dtone_out;
                jd.pix_xrgb = 1;
                jd.pix_fast_tone = g.v4cfg.fast_aces && g.v4cfg.fast_gamma ? 1 : 0;
            }
            if ((rc = v4_launch(g.dev[d], jd, g.dev[d].stream, false, &presented))) return rc;
        }
    }
    g.v4_frame += 1;   // iFrame += 1.0f (v4 :1703), before rendering
    if (screen && g.v4cfg.output_to_screen) {   // OutputToScreen per tile (v4 :1562-1564)
        if (presented) {
            Dev& dv = g.dev[0];
            HIP_TRY(hipMemcpyAsync(screen, dv.dtone_out, (size_t)w * h * sizeof(uint32_t), hipMemcpyDeviceToHost, dv.stream));
        } else if (banded) {
            Dev& dv = g.dev[0];
            const size_t out_bytes = (size_t)w * h * sizeof(uint32_t);
            if ((rc = grow(dv, (void**)&dv.dtone_out, &dv.dtone_out_cap, out_bytes))) return rc;
            const PtToneJob tj = tone_job(dv.dbuf, w, h, PT_LAYOUT_TILED_PLANAR8, tw, th, dv.dtone_out, PT_PIXEL_XRGB8);
            hipError_t e = pt_launch_tonemap(tj, dv.stream);
            if (e != hipSuccess) return fail(PT_EHIP, "tonemap launch failed: %s", hipGetErrorString(e));
            HIP_TRY(hipMemcpyAsync(screen, dv.dtone_out, out_bytes, hipMemcpyDeviceToHost, dv.stream));
        } else if ((rc = tone_output(PT_LAYOUT_TILED_PLANAR8, tw, th, (uint32_t*)screen, PT_PIXEL_XRGB8))) {
            return rc;
        }
    }
    if (banded) {
        HIP_TRY(hipStreamSynchronize(g.s_out));
        return sync_all();
    }
    return stage_out(buf, geo, Region{});
}

int pt_copy_output_to_file(const float* buf, int32_t w, int32_t h, int32_t ntx, int32_t nty, int32_t tw, int32_t th,
                           int32_t nc, void* file_pixels)
{
    int rc;
    if ((rc = check_frame_args(buf, w, h, nc)) || (rc = ensure_init())) return rc;
    if ((rc = tiled_settings(w, h, ntx, nty, tw, th))) return rc;
    if (g.v4_frame + 1u >= kMaxFrame) return fail(PT_EINVAL, "v4 frame counter exceeds the exact f32 range 2^24");
    if ((rc = pt_tonemap(buf, w, h, PT_LAYOUT_TILED_PLANAR8, tw, th, (uint32_t*)file_pixels, PT_PIXEL_RGBA8))) return rc;
    g.v4_frame += 1;   // v4 :1738
    return PT_OK;
}

static int v4_device_job(const pt_device_job* dj, PtV4Job* j4)
{
    int rc;
    if (!dj) return fail(PT_EINVAL, "null device job");
    pt_device_job geo = *dj;   // geometry / frame checks of the scalar-path jobs
    geo.use_env = 0;
    PtJob j;
    if ((rc = device_job(&geo, &j)) || (rc = v4_ensure_scene())) return rc;
    *j4 = v4_job(dj->buf, dj->width, dj->height);
    j4->row_start = dj->row_start;
    j4->row_stride = dj->row_stride;
    j4->nrows = dj->nrows;
    j4->layout = dj->layout;
    j4->frame_first = dj->frame_first;
    j4->nframes = dj->nframes;
    j4->num_bounces = dj->num_bounces;
    if (dj->use_env) {
        if (g.v4cfg.env_mode == PT_V4_ENV_NONE) return fail(PT_ESTATE, "use_env with v4 env mode NONE");
        if ((rc = v4_use_env(*j4))) return rc;
    }
    return PT_OK;
}

int pt_v4_render_device(const pt_device_job* dj, void* stream)
{
    int rc;
    PtV4Job j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if ((rc = ensure_init()) || (rc = v4_device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv))) return rc;
    return v4_launch(*dv, j, (hipStream_t)stream, false);
}

int pt_v4_render_device_chain(const pt_device_job* dj, void* stream)
{
    int rc;
    PtV4Job j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if ((rc = ensure_init()) || (rc = v4_device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv))) return rc;
    return launch_chain(*dv, j, (hipStream_t)stream);
}

int pt_v4_count_device(const pt_device_job* dj, void* stream, pt_work_counts* out)
{
    int rc;
    PtV4Job j;
    Dev* dv = nullptr;
    DeviceGuard guard;
    if (!out) return fail(PT_EINVAL, "null counts");
    if ((rc = ensure_init()) || (rc = v4_device_job(dj, &j)) || (rc = dev_of(dj->buf, &dv)) || (rc = use_dev(*dv))) return rc;
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(dv->dcounters, 0, kCounterSlots * sizeof(unsigned long long), st));
    j.counters = dv->dcounters;
    if ((rc = v4_launch(*dv, j, st, true))) return rc;
    unsigned long long h[6];
    HIP_TRY(hipMemcpyAsync(h, dv->dcounters, sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    out->segments = h[0];
    out->lane_slots = h[3];
    out->samples = (uint64_t)dj->width * (uint64_t)dj->nrows * (uint64_t)dj->nframes;
    out->escaped = h[2];
    out->primary = out->samples;   // one camera ray per sample (jittered)
    out->quad_fallbacks = 0;
    out->sphere_fallbacks = h[4];
    out->sky_skipped = h[5];
    return PT_OK;
}

int pt_v4_begin_frame(void)
{
    if (g.v4_frame + 1u >= kMaxFrame) return fail(PT_EINVAL, "v4 frame counter exceeds the exact f32 range 2^24");
    g.v4_frame += 1;
    return PT_OK;
}

// ---- tile work queue ------------------------------------------------------------------------------

}  // extern "C"

struct pt_work_queue {
    int32_t renderer = PT_RENDERER_SIMD_TILED;
    std::vector<std::pair<pt_buffer_info, pt_tile_info>> entries;
    bool pending = false;   // an async completion not yet waited for
};

namespace {

// Render the queued entries: per buffer (in first-use order) either one full-frame launch per device
// (the entries are exactly the buffer's NTX x NTY tiles) or per tile one launch per device; uploads /
// downloads of only what is rendered.  Everything is enqueued on the device streams; `wait`
// synchronises at the end.
int run_queue(pt_work_queue* q, bool wait)
{
    int rc;
    if ((rc = ensure_init())) return rc;
    const bool v4 = q->renderer == PT_RENDERER_V4;
    if (v4) {
        if (g.v4_frame < 1) return fail(PT_ESTATE, "v4 work queue before the first frame (pt_v4_begin_frame)");
        if ((rc = v4_ensure_scene())) return rc;
    } else if (g.frame < (uint32_t)g.cfg.samples_per_frame) {
        return fail(PT_ESTATE, "work queue before the first frame was started (pt_begin_frame)");
    }
    const bool env = q->renderer == PT_RENDERER_SIMT_TEXTURED;
    if (env && !g.have_env) return fail(PT_ESTATE, "textured work queue without an env map (pt_set_env_map)");
    DeviceGuard guard;
    Dev& d0 = g.dev[0];
    std::vector<bool> done(q->entries.size(), false);
    for (size_t i = 0; i < q->entries.size(); ++i) {
        if (done[i]) continue;
        const pt_buffer_info& b = q->entries[i].first;
        std::vector<size_t> mine;
        for (size_t k = i; k < q->entries.size(); ++k)
            if (!done[k] && q->entries[k].first.data == b.data) {
                const pt_buffer_info& bk = q->entries[k].first;
                if (bk.width != b.width || bk.height != b.height)
                    return fail(PT_EINVAL, "entries of one buffer disagree on its size");
                mine.push_back(k);
                done[k] = true;
            }
        const pt_tile_info& t0 = q->entries[mine[0]].second;
        const int32_t tw = t0.tile_width, th = t0.tile_height;
        for (size_t k : mine) {
            const pt_tile_info& t = q->entries[k].second;
            if (t.tile_width != tw || t.tile_height != th)
                return fail(PT_EINVAL, "entries of one buffer disagree on the tile size");
        }
        bool full = b.width % tw == 0 && b.height % th == 0 &&
                    mine.size() == (size_t)(b.width / tw) * (size_t)(b.height / th);
        if (full) {   // exactly every tile once?
            std::vector<char> seen((size_t)(b.width / tw) * (b.height / th), 0);
            for (size_t k : mine) {
                const pt_tile_info& t = q->entries[k].second;
                const size_t id = (size_t)t.tile_y * (b.width / tw) + t.tile_x;
                if (seen[id]) {
                    full = false;
                    break;
                }
                seen[id] = 1;
            }
        }
        const Geo geo = geo_of(b.width, b.height, PT_LAYOUT_TILED_PLANAR8, tw, th);
        if (full && g.ndev == 1 && (g.cfg.flags & PT_FLAG_PIN_HOST) && !(g.cfg.flags & PT_FLAG_DEFER_READBACK)) {
            // A whole frame of tiles with PT_FLAG_PIN_HOST: the frame calls' band pipeline (bands of
            // whole tile rows, upload / render / download overlapped on three streams).  The bands'
            // copies run on s_in / s_out, so they are ordered after the work already queued on
            // the device stream (an earlier buffer's download from the mirror), and that stream --
            // which the completion calls synchronise -- after the last download.
            if ((rc = use_dev(d0))) return rc;
            HIP_TRY(hipEventRecord(g.ev_q, d0.stream));
            HIP_TRY(hipStreamWaitEvent(g.s_in, g.ev_q, 0));
            bool banded = false;
            if (v4) {
                PtV4Job j = v4_job(nullptr, b.width, b.height);
                j.layout = PT_LAYOUT_TILED_PLANAR8;
                j.tile_w = tw;
                j.tile_h = th;
                j.frame_first = g.v4_frame;
                if ((rc = v4_use_env(j))) return rc;
                rc = render_bands(b.data, j, th, [](const PtV4Job& bj) { return v4_launch(g.dev[0], bj, g.dev[0].stream, false); },
                                  &banded);
            } else {
                pt_tile_info t = t0;
                t.tile_min_x = 0;
                t.tile_min_y = 0;
                PtJob j = tile_job(&b, &t, env);
                j.ncols = b.width;
                j.nrows = b.height;
                if (env)
                    rc = render_bands(b.data, j, th, [](const PtJob& bj) {
                        return launch(g.dev[0], with_env(bj, g.dev[0], true), g.dev[0].stream, false);
                    }, &banded);
                else
                    rc = render_bands(b.data, j, th, [](const PtJob& bj) { return launch(g.dev[0], bj, g.dev[0].stream, false); },
                                      &banded);
            }
            if (rc) return rc;
            if (banded) {
                HIP_TRY(hipEventRecord(g.ev_q, g.s_out));
                HIP_TRY(hipStreamWaitEvent(d0.stream, g.ev_q, 0));
                continue;
            }
        }
        // one job per device for the whole frame, or per tile
        std::vector<Region> regions;
        if (full) {
            regions.push_back(Region{});
        } else {
            for (size_t k : mine) {
                Region rg;
                rg.whole = false;
                rg.tile_x = q->entries[k].second.tile_x;
                rg.tile_y = q->entries[k].second.tile_y;
                regions.push_back(rg);
            }
        }
        for (const Region& rg : regions)
            if ((rc = stage_in(b.data, geo, rg))) return rc;
        for (const Region& rg : regions) {
            // the frame as one "tile" region in the tiled layout, or the entry's tile
            const int32_t col0 = rg.whole ? 0 : rg.tile_x * tw, row0 = rg.whole ? 0 : rg.tile_y * th;
            const int32_t ncols = rg.whole ? b.width : tw, nrows = rg.whole ? b.height : th;
            for (int d = 0; d < g.ndev; ++d) {
                Dev& dv = g.dev[d];
                if (v4) {
                    PtV4Job j = v4_job(nullptr, b.width, b.height);
                    j.layout = PT_LAYOUT_TILED_PLANAR8;
                    j.tile_w = tw;
                    j.tile_h = th;
                    j.col0 = col0;
                    j.ncols = ncols;
                    j.row_start = row0;
                    j.nrows = nrows;
                    j.frame_first = g.v4_frame;   // the frame pt_v4_begin_frame started
                    if ((rc = v4_use_env(j)) || (rc = v4_launch(dv, tile_shard_job(j, d), dv.stream, false))) return rc;
                } else {
                    pt_tile_info t{};
                    t.tile_width = tw;
                    t.tile_height = th;
                    t.tile_min_x = col0;
                    t.tile_min_y = row0;
                    PtJob j = tile_job(&b, &t, env);
                    j.ncols = ncols;
                    j.nrows = nrows;
                    if ((rc = launch(dv, with_env(tile_shard_job(j, d), dv, env), dv.stream, false))) return rc;
                }
            }
        }
        if (!(g.cfg.flags & PT_FLAG_DEFER_READBACK))
            for (const Region& rg : regions)
                for (int d = 0; d < g.ndev; ++d)
                    if ((rc = use_dev(g.dev[d])) || (rc = xfer(d, geo, b.data, false, rg))) return rc;
        // the mirror holds one buffer at a time: another buffer of the queue must not start
        // overwriting it before this one's downloads are done (stream order guarantees that)
    }
    q->entries.clear();
    if (wait) {
        if ((rc = sync_all())) return rc;
        q->pending = false;
    } else {
        q->pending = true;
    }
    return PT_OK;
}

}  // namespace

extern "C" {

pt_work_queue* pt_make_work_queue(int32_t renderer)
{
    if (renderer < PT_RENDERER_SIMD_TILED || renderer > PT_RENDERER_V4) {
        fail(PT_EINVAL, "unknown renderer %d", renderer);
        return nullptr;
    }
    pt_work_queue* q = new (std::nothrow) pt_work_queue;
    if (!q) {
        fail(PT_ENOMEM, "out of host memory");
        return nullptr;
    }
    q->renderer = renderer;
    q->entries.reserve(1024);   // WORK_QUEUE_MAX_ENTRIES (work_queue.h:16)
    return q;
}

int pt_add_work_queue_entry(pt_work_queue* q, const pt_buffer_info* b, const pt_tile_info* t)
{
    int rc;
    if (!q) return fail(PT_EINVAL, "null queue");
    if ((rc = check_tile(b, t))) return rc;
    if (q->entries.size() >= 1023)   // the ring holds MaxEntryCount - 1 (work_queue.cpp:42 assert)
        return fail(PT_EINVAL, "work queue full (WORK_QUEUE_MAX_ENTRIES 1024)");
    q->entries.emplace_back(*b, *t);
    return PT_OK;
}

int pt_complete_all_work(pt_work_queue* q)
{
    if (!q) return fail(PT_EINVAL, "null queue");
    return run_queue(q, true);
}

int pt_complete_all_work_async(pt_work_queue* q)
{
    if (!q) return fail(PT_EINVAL, "null queue");
    return run_queue(q, false);
}

int pt_wait_work(pt_work_queue* q)
{
    if (!q) return fail(PT_EINVAL, "null queue");
    if (q->pending && g.inited) {
        DeviceGuard guard;
        int rc;
        if ((rc = sync_all())) return rc;
    }
    q->pending = false;
    return PT_OK;
}

int32_t pt_work_queue_size(const pt_work_queue* q) { return q ? (int32_t)q->entries.size() : 0; }

void pt_free_work_queue(pt_work_queue* q)
{
    if (!q) return;
    if (q->pending && g.inited) {
        DeviceGuard guard;
        (void)sync_all();
    }
    delete q;
}

}  // extern "C"
