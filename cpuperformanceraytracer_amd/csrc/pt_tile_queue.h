// pt_tile_queue.h -- the tile queue of the persistent render kernels (pt_kernel.hip: the diffuse
// renderers, pt_v4.hip: DemofoxRenderOptV4), and the resident-grid size they are launched with.
//
// The launch's work is a list of UNITS -- runs of 8x8 tiles in schedule order (order: the previous
// launch's tiles sorted by descending cost, so the long tiles start first and the tail is made of
// short ones; units: run boundaries, each run worth about a unit cost of pool iterations (2-12, adaptive), so a run of
// cheap sky tiles costs one dequeue, not dozens; pt_kernel.hip's pt_schedule_kernel builds both).
// Without a schedule every tile is a unit, in raster order.
//
// Units are dealt to PT_NQUEUES groups of blocks (block b -> group b % 8, the XCD it is dispatched
// to): group x owns unit slots x, x+8, ...  Each wave's first unit is static (its index in the
// group); later ones come from the group's own counter, one returning atomic per unit, claimed
// only when the current unit is used up -- the kernels call next() once the pool of the unit's last
// tile has drained, so the atomic and the schedule loads overlap that tile's epilogue.  A claim
// made earlier reserves a long tile for a wave that is still busy, and the longest-first order
// comes apart at the end of the launch (claiming one and two units ahead, tiles of 23-26
// iterations started 500 us into a launch while other waves ran sky tiles).  One counter for the
// whole chip saturated (~90 dequeues/us, MI355X_MICROARCH.md "dequeue").
//
// A group whose units are used up takes the others'.  That happens only at the end of the launch,
// when thousands of waves run out at once and atomics on the counters queue up: a group found
// exhausted is remembered per wave, and a plain load of a counter screens it first (a counter
// only grows, so a load that shows it used up is right; without the screening the tail's atomics
// tripled the launch time).  Victims are visited in a per-wave rotation.
//
// A queue entry is a tile or one half of it: the schedule splits the few tiles that cost more than
// a wave's share of the launch (pt_capi.cpp: split factor 1, PT_MI355_SPLIT), so that a launch of
// about one such tile per wave does not end on the waves that drew two.  Part 1 is the tile's rows 0-3 (lanes 0-31), part 2 its rows 4-7 (lanes 32-63); the
// other half's pixels are treated as outside the image.
//
// The whole wave runs the queue code (uniform control flow): every value is wave-uniform and lives
// in scalar registers -- held by lane 0 alone they took vector registers across the whole pool
// loop, which the 96-VGPR budget of the ambient kernel spilled.  Only the counter atomics are
// issued by one lane (the first active one) and broadcast with readfirstlane; the kernels are
// built with the atomic optimizer off, so that single-lane atomic needs no wave reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "pt_kernel.h"   // PT_NQUEUES
#include "pt_guard.h"

__device__ __forceinline__ uint32_t pt_entry_tile(uint32_t e) { return e & PT_TILE_MASK; }
__device__ __forceinline__ uint32_t pt_entry_part(uint32_t e) { return e >> PT_TILE_PART_SHIFT; }
__device__ __forceinline__ bool pt_part_has_lane(uint32_t part, int lane)
{
    return part == 0u || (uint32_t)(lane >> 5) + 1u == part;
}
// The schedule's cost record of entry e (cost: 2 x ntiles words; a tile's cost is the sum of its
// two words -- a whole tile writes 0 into its second)
__device__ __forceinline__ void pt_record_cost(uint32_t* cost, uint32_t e, uint32_t ntiles, uint32_t w)
{
    const uint32_t tile = pt_entry_tile(e), part = pt_entry_part(e);
    cost[part == 2u ? ntiles + tile : tile] = w;
    if (part == 0u) cost[ntiles + tile] = 0u;
}

// The next launch's queue counters, zeroed by the launch's block 0 (pt_capi.cpp use_sched)
__device__ __forceinline__ void pt_queue_zero_next(unsigned int* queue_next)
{
    if (queue_next && blockIdx.x == 0 && threadIdx.x < PT_NQUEUES)
        *reinterpret_cast<unsigned long long*>(queue_next + threadIdx.x * 32u) = 0ull;
#if PT_CHAIN_DIAG   // (pt_chain.h's diagnostic words 34-36)
    if (queue_next && blockIdx.x == 0 && threadIdx.x >= 64 && threadIdx.x < 67) queue_next[34 + threadIdx.x - 64] = 0u;
#endif
}

// A group's counter is 64 bits: dynamic units taken from the front (low word: longest first) and
// from the back (high word: the cheapest units).  A wave set to `back` (the continuous-tiles
// kernels' last-dispatched blocks, which the SQ's oldest-first issue leaves the slowest) takes its
// group's cheapest units, so the launch's last expensive units go to fast waves; a claim is valid
// while front + back stays below the group's dynamic unit count.
static_assert(PT_NQUEUES <= 31, "the queue's dead-group mask keeps bit 31 for tile_at's flag");
template <int WAVES_PER_BLOCK>
struct PtTileQueue {
    static constexpr uint32_t kNone = 0xffffffffu;
    static constexpr uint32_t kBadSeen = 0x80000000u;   // dead's flag: tile_at met a bad entry (groups: bits 0-7)
    unsigned int* base;       // PT_NQUEUES 64-bit counters, 128 B apart (zeroed before the launch)
    const uint32_t* order;    // schedule position -> tile, or nullptr (raster order)
    const uint32_t* units;    // unit -> first schedule position (units[u + 1] its end), or nullptr
                              // (order: entries -- tile | part << PT_TILE_PART_SHIFT)
    uint32_t nunits, ntiles, ngroups, qg, wave;
    uint32_t dead = 0;        // groups known to be exhausted
    uint32_t bad = 0;         // a schedule entry outside the launch's tiles (tile_at: valid when dead's bit 31 is set)
    uint32_t c_pos = kNone, c_end = kNone;   // the current unit's remaining schedule positions
    uint32_t back = 0;        // 1: claim from the back of the own group

    __device__ PtTileQueue(unsigned int* queue, const uint32_t* order_, const uint32_t* units_,
                           const uint32_t* nunits_, uint32_t total_tiles, int wv)
        : base(queue), order(order_), units(units_)
    {
        nunits = units ? __builtin_amdgcn_readfirstlane(*nunits_) : total_tiles;
        ntiles = total_tiles;
        ngroups = gridDim.x < PT_NQUEUES ? gridDim.x : PT_NQUEUES;   // small grids: fewer groups
        qg = blockIdx.x % ngroups;
        wave = (blockIdx.x / ngroups) * WAVES_PER_BLOCK + (uint32_t)wv;   // index inside the group
    }
    // The queue's state as kWords words (a wave's LDS copy: a kernel whose pool loop must not hold
    // the queue in scalar registers keeps it there between dequeues -- render_body_ct).  save: lane 0
    // stores; restore: uniform loads.
    static constexpr int kWords = 16;
    __device__ PtTileQueue() = default;
    __device__ void save(uint32_t* w, int lane) const
    {
        if (lane != 0) return;
        const uint64_t p[3] = {(uint64_t)base, (uint64_t)order, (uint64_t)units};
        for (int i = 0; i < 3; ++i) {
            w[2 * i] = (uint32_t)p[i];
            w[2 * i + 1] = (uint32_t)(p[i] >> 32);
        }
        w[6] = nunits;
        w[7] = ntiles;
        w[8] = ngroups;
        w[9] = qg;
        w[10] = wave;
        w[11] = dead;
        w[12] = c_pos;
        w[13] = c_end;
        w[14] = back;
        w[15] = bad;
    }
    __device__ static PtTileQueue restore(const uint32_t* w)
    {
        auto u = [&](int i) { return (uint32_t)__builtin_amdgcn_readfirstlane(w[i]); };
        auto ptr = [&](int i) { return (uint64_t)u(2 * i) | ((uint64_t)u(2 * i + 1) << 32); };
        PtTileQueue q;
        q.base = (unsigned int*)ptr(0);
        q.order = (const uint32_t*)ptr(1);
        q.units = (const uint32_t*)ptr(2);
        q.nunits = u(6);
        q.ntiles = u(7);
        q.ngroups = u(8);
        q.qg = u(9);
        q.wave = u(10);
        q.dead = u(11);
        q.c_pos = u(12);
        q.c_end = u(13);
        q.back = u(14);
        q.bad = u(15);
        return q;
    }
    __device__ uint32_t group_waves(uint32_t g) const
    {
        return ((gridDim.x - g + ngroups - 1) / ngroups) * WAVES_PER_BLOCK;
    }
    __device__ uint32_t slot_of(uint32_t g, uint32_t c) const   // unit slot of dynamic position c of group g
    {
        const uint32_t slot = g + ngroups * (group_waves(g) + c);
        return slot < nunits ? slot : kNone;
    }
    __device__ uint32_t dyn_units(uint32_t g) const   // dynamic positions of group g
    {
        const uint32_t all = g < nunits ? (nunits - g + ngroups - 1) / ngroups : 0u, w = group_waves(g);
        return all > w ? all - w : 0u;
    }
    // the slot of a claim whose counter read `old` (front or back), kNone past the group's units
    __device__ uint32_t claimed(uint32_t g, unsigned long long old, bool from_back) const
    {
        const uint32_t f = (uint32_t)old, b = (uint32_t)(old >> 32), n = dyn_units(g);
        if ((unsigned long long)f + b >= n) return kNone;
        return slot_of(g, from_back ? n - 1u - b : f);
    }
    __device__ uint32_t unit_lo(uint32_t u) const { return units ? __builtin_amdgcn_readfirstlane(units[u]) : u; }
    __device__ uint32_t unit_hi(uint32_t u) const { return units ? __builtin_amdgcn_readfirstlane(units[u + 1]) : u + 1; }
    // A schedule entry outside the launch's tiles ends the wave instead of faulting, and is kept in
    // `bad`, which the kernel records in the job's error words when the wave ends, in every build
    // (report(): guard PT_G_QUEUE_ENTRY, the host returns PT_EKERNEL -- a corrupt entry must not drop
    // tiles silently; recorded at the end, off the claim path, whose registers the pool loop shares).
    __device__ uint32_t tile_at(uint32_t i)
    {
        const uint32_t e = order ? __builtin_amdgcn_readfirstlane(order[i]) : i;
        if (pt_entry_tile(e) < ntiles && pt_entry_part(e) < 3u) return e;
        bad = e;
        dead |= kBadSeen;
        return kNone;
    }
    // the wave's end: a bad entry seen by tile_at into the job's error words (the first active lane)
    __device__ void report(uint32_t* err) const
    {
        if ((dead & kBadSeen) && err &&
            __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) ==
                (uint32_t)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))))
            pt_guard_report(err, PT_G_QUEUE_ENTRY, bad);
    }
    // the checked build: a unit's schedule positions [c_pos, c_end) inside order[] (2 x ntiles
    // entries with a schedule, ntiles without); err: the job's error words
    __device__ bool unit_ok(uint32_t* err) const
    {
        return PT_GUARD(err, c_pos <= c_end && c_end <= (units ? 2u * ntiles : ntiles), PT_G_UNIT_RANGE, c_end);
    }

    __device__ unsigned long long* counter(uint32_t g) const
    {
        return reinterpret_cast<unsigned long long*>(base + g * 32u);
    }
    // one returning atomic for the wave (its first active lane), the result broadcast
    __device__ static unsigned long long wave_atomic_add(unsigned long long* c, unsigned long long inc)
    {
        const uint32_t me = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        unsigned long long r = 0;
        if (me == (uint32_t)__builtin_amdgcn_readfirstlane(me)) r = atomicAdd(c, inc);
        return ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32) |
               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r);
    }
    __device__ static unsigned long long wave_load(const unsigned long long* c)
    {
        const unsigned long long v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    }
    __device__ uint32_t steal()
    {
        for (uint32_t k = 1; k < ngroups; ++k) {
            const uint32_t g = (qg + 1 + (wave + k - 1) % (ngroups - 1)) % ngroups;
            if ((dead >> g) & 1u) continue;
            unsigned long long* const c = counter(g);
            if (claimed(g, wave_load(c), false) == kNone) {
                dead |= 1u << g;
                continue;
            }
            const uint32_t slot = claimed(g, wave_atomic_add(c, 1ull), false);
            if (slot != kNone) return slot;
            dead |= 1u << g;
        }
        return kNone;
    }
    // the first tile of this wave's static unit, kNone if the launch has fewer units than waves
    __device__ uint32_t first(uint32_t* err = nullptr)
    {
        // (the checked build: a unit count beyond the schedule's 2 x ntiles entries ends every wave)
        if (!PT_GUARD(err, !units || nunits <= 2u * ntiles, PT_G_NUNITS, nunits)) nunits = 0;
        const uint32_t u0 = qg + ngroups * wave;
        if (u0 >= nunits) return kNone;
        c_pos = unit_lo(u0);
        c_end = unit_hi(u0);
        if (!unit_ok(err)) return kNone;
        return next(err);
    }
    // the next tile: the current unit's, or the first of a newly claimed unit; kNone when every
    // unit of every group has been taken
    __device__ uint32_t next(uint32_t* err = nullptr)
    {
        if (c_pos >= c_end) {
            uint32_t u = ((dead >> qg) & 1u) ? kNone
                                             : claimed(qg, wave_atomic_add(counter(qg), back ? 1ull << 32 : 1ull), back != 0);
            if (u == kNone) {
                dead |= 1u << qg;
                u = steal();
            }
            if (u == kNone) return kNone;
            c_pos = unit_lo(u);
            c_end = unit_hi(u);
            if (!unit_ok(err)) return kNone;
        }
        return tile_at(c_pos++);
    }
};

// Blocks of `threads` threads of `kern` the device keeps resident: the grid of a persistent
// launch.  It must be exact -- a block beyond residency starts only when a resident one ends, and
// its waves' static first units (the most expensive tiles of the schedule) then run last
// (measured: 1024 of 5120 waves born 270-460 us into a 470 us launch).
// hipOccupancyMaxActiveBlocksPerMultiprocessor is capped by the LDS rule measured on gfx950
// (scripts/lds_probe.hip): LDS is allocated in 1280-B granules of the CU's 160 KiB, which the API
// does not model (it reports 5 blocks for 32001..32768 B, where 4 fit).
constexpr int kPtLdsGranule = 1280;
template <typename K>
int pt_resident_blocks(K kern, int threads)
{
    struct Entry {
        const void* kern;
        int dev, blocks;
    };
    static Entry cache[64];   // (kernel, device) -> resident blocks; one entry per instantiation
    static int used = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024;
    for (int i = 0; i < used; ++i)
        if (cache[i].kern == (const void*)kern && cache[i].dev == dev) return cache[i].blocks;
    int nb = 0, cus = 0, lds_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, 0) != hipSuccess || nb <= 0) nb = 4;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
        lds_cu <= 0)
        lds_cu = 160 * 1024;
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, (const void*)kern) == hipSuccess && fa.sharedSizeBytes > 0) {
        const int granules = (int)((fa.sharedSizeBytes + kPtLdsGranule - 1) / kPtLdsGranule);
        nb = std::min(nb, std::max(1, lds_cu / (granules * kPtLdsGranule)));
    }
    if (used < 64) cache[used++] = Entry{(const void*)kern, dev, nb * cus};
    return nb * cus;
}
