// pt_chain.h -- the device side of chained launches (pt_capi.cpp launch_chain), shared by
// the continuous-tiles pools of pt_kernel.hip (render_body_ct) and pt_v4.hip (pt_v4_ct_kernel).
//
// Consecutive launches of one geometry overlap on two streams.  The only data a launch needs from the
// one before is a tile's accumulator values: the progressive lerp of demofox_path_tracing_scalar.cpp:812
// (v4: the fused lerp of demofox_path_tracing_optimization_v4.cpp:1233-1241) folds each pixel's frames
// in order.  So a launch touches a tile's pixels only after the previous launch has stored them:
//   * the accumulator's loads and stores are `sc1` (agent-scope relaxed atomics: global_load /
//     global_store ... sc1, past the L1) -- in every continuous-tiles launch, one code path (a pixel is
//     loaded and stored once per launch; A/B: no measurable cost, profiles/r06/r06l_ab_chain_code.txt);
//   * after a queue entry's (tile or half tile) last pixel store the wave waits for its stores
//     (s_waitcnt vmcnt(0)) and one lane stores the launch's sequence number into the entry's half-tile
//     epoch words (`sc1`);
//   * a chained launch polls the epochs of an entry it claims (`sc1` loads) until they reach its
//     predecessor's number, before it touches the entry's pixels.
// This is the hand-off of MI355X_MICROARCH.md's inter-workgroup table, row 1 (sc1 stores, the storing
// wave's vmcnt(0), an sc1 flag store; sc1 polls and loads).  Every block adds 1 to the chain's started
// counter at its start: the next launch's stream waits for all of them (hipStreamWaitValue64), which
// makes the chain deadlock-free (tests/test_chain_protocol.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_kernel.h"        // PT_G_CHAIN_WAIT
#include "pt_guard.h"         // pt_guard_report
#include "pt_tile_queue.h"    // pt_entry_tile / pt_entry_part

__device__ __forceinline__ float pt_px_ld(const float* p)
{
    return __builtin_bit_cast(float, __hip_atomic_load(reinterpret_cast<uint32_t*>(const_cast<float*>(p)), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void pt_px_st(float* p, float v)
{
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A pixel's three channels at element pi of the accumulator `buf` (channel stride cs).  The interleaved
// layout (cs = 1) keeps one 12-byte access per pixel: a raw buffer load / store of 96 bits with the
// sc1 cache policy (buffer_load/store_dwordx3 ... sc1) over the job's buffer (nbytes: its size, < 2^31;
// 0: the per-channel accesses above), so a tile row's eight pixels stay one 96-byte write -- three
// dword sc1 stores per pixel wrote each dword through on its own (c2: 217 vs 177 MB of WRITE_SIZE).
typedef unsigned pt_v3u __attribute__((ext_vector_type(3)));
typedef float pt_v3f __attribute__((ext_vector_type(3)));
constexpr int kPtCpolSc1 = 16;               // CPol::SC1 (gfx940+ cache-policy bits of the buffer intrinsics)
constexpr int kPtBufRsrcWord3 = 0x00020000;  // raw (untyped) buffer resource, the gfx9 data-format word
__device__ __forceinline__ void pt_px_ld3(const float* buf, uint32_t nbytes, size_t cs, size_t pi, float& x, float& y, float& z)
{
    if (cs == 1 && nbytes) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(buf), 0, (int)nbytes, kPtBufRsrcWord3);
        // (the whole vector is bit-cast: element-wise bit casts of the u32 vector made this compiler
        // shrink the load to its first dword -- tests/test_isa_lgkm.py checks the built loads)
        const pt_v3f v = __builtin_bit_cast(pt_v3f, __builtin_amdgcn_raw_buffer_load_b96(r, (int)(pi * 4u), 0, kPtCpolSc1));
        x = v.x, y = v.y, z = v.z;
        return;
    }
    x = pt_px_ld(buf + pi), y = pt_px_ld(buf + pi + cs), z = pt_px_ld(buf + pi + 2 * cs);
}
__device__ __forceinline__ void pt_px_st3(float* buf, uint32_t nbytes, size_t cs, size_t pi, float x, float y, float z)
{
    if (cs == 1 && nbytes) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, (int)nbytes, kPtBufRsrcWord3);
        const pt_v3f v = {x, y, z};
        __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(pt_v3u, v), r, (int)(pi * 4u), 0, kPtCpolSc1);
        return;
    }
    pt_px_st(buf + pi, x), pt_px_st(buf + pi + cs, y), pt_px_st(buf + pi + 2 * cs, z);
}
// the accumulator's size in bytes for pt_px_ld3 / pt_px_st3 (0: too large for a buffer resource)
__device__ __forceinline__ uint32_t pt_px_nbytes(size_t floats)
{
    return floats * 4u < (1ull << 31) ? (uint32_t)(floats * 4u) : 0u;
}

// the block has started (the next chained launch's stream gate); started: nullptr when not chained
__device__ __forceinline__ void pt_chain_started(unsigned long long* started)
{
    if (started && threadIdx.x == 0) __hip_atomic_fetch_add(started, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// entry e's half-tile epochs are >= w (every lane loads the same words; the value is made wave-uniform)
__device__ __forceinline__ bool pt_chain_ready(const uint32_t* ep, uint32_t e, uint32_t w)
{
    const uint32_t t = pt_entry_tile(e), part = pt_entry_part(e);
    uint32_t m = ~0u;
    if (part != 2u) {
        const uint32_t a = __hip_atomic_load(const_cast<uint32_t*>(ep + 2u * t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = a < m ? a : m;
    }
    if (part != 1u) {
        const uint32_t b = __hip_atomic_load(const_cast<uint32_t*>(ep + 2u * t + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = b < m ? b : m;
    }
    return __builtin_amdgcn_readfirstlane(m) >= w;
}

// (the whole wave) before touching entry e's pixels: wait until the previous launch has published it.
// Rare -- both launches take the tiles longest first, so a launch reaches a tile long after its
// predecessor folded it.  Bounded: after 2^21 polls (>= 2 s of the wave's own running time) the wait is
// reported (guard PT_G_CHAIN_WAIT, every build) instead of hanging the GPU; the host's stream gate makes
// that unreachable.  The bound counts polls, not wall-clock time: while the process's queues are
// preempted the waves do not run, and a wall-clock bound (round 6's first form, 1.3 s of
// s_memrealtime) would end every wait in progress when they resume.
//
// PT_CHAIN_DIAG=1 (a diagnostic build, scripts/build_variant.sh): words 34-36 of a continuing launch's
// tile-queue block count its waves, the ones that ended and the ones waiting; a wait that runs out
// (after 2^16 polls there) prints them for the launch and its predecessor.
#ifndef PT_CHAIN_DIAG
#define PT_CHAIN_DIAG 0
#endif
constexpr uint32_t kPtChainPolls = PT_CHAIN_DIAG ? 1u << 16 : 1u << 21;
// the bound, per translation unit and device (test hook PT_MI355_TEST_CHAIN_POLLS: pt_set_chain_polls /
// pt_v4_set_chain_polls), read only once a wait has begun
static __device__ uint32_t pt_chain_polls_dev = kPtChainPolls;
constexpr uint32_t kPtDiagWaves = 34, kPtDiagEnded = 35, kPtDiagWaiting = 36;
// (diag) the tile-queue block of the chained launch before the one whose block is q (seq: its number)
__device__ __forceinline__ unsigned* pt_chain_diag_prev(unsigned* q, uint32_t seq)
{
    return q - (size_t)(seq % 4u) * PT_QUEUE_WORDS + (size_t)((seq + 3u) % 4u) * PT_QUEUE_WORDS;
}
__device__ __forceinline__ void pt_chain_wait(const uint32_t* ep, uint32_t e, uint32_t w, uint32_t* err, int lane,
                                              unsigned* qdiag = nullptr)
{
    if (pt_chain_ready(ep, e, w)) return;
    bool ok = false;
    uint32_t polls = 0;
    if (PT_CHAIN_DIAG && qdiag && lane == 0) atomicAdd(qdiag + kPtDiagWaiting, 1u);
    do {
        __builtin_amdgcn_s_sleep(8);   // (~0.2 us; a poll's sc1 loads take ~1-2 us more)
        ok = pt_chain_ready(ep, e, w);
    } while (!ok && ++polls < pt_chain_polls_dev);
    if (PT_CHAIN_DIAG && qdiag && lane == 0) atomicSub(qdiag + kPtDiagWaiting, 1u);
#if PT_CHAIN_DIAG
    if (!ok && lane == 0 && qdiag) {
        unsigned* const qp = pt_chain_diag_prev(qdiag, w + 1u);
        auto rd = [](unsigned* p) { return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        const uint32_t t = pt_entry_tile(e);
        printf("chain wait ran out: launch %u entry %u (tile %u) epochs %u %u | this launch: waves %u ended %u waiting %u "
               "| previous: waves %u ended %u waiting %u | block %u wave %u\n",
               w + 1u, e, t, rd(const_cast<uint32_t*>(ep + 2u * t)), rd(const_cast<uint32_t*>(ep + 2u * t + 1u)),
               rd(qdiag + kPtDiagWaves), rd(qdiag + kPtDiagEnded), rd(qdiag + kPtDiagWaiting), rd(qp + kPtDiagWaves),
               rd(qp + kPtDiagEnded), rd(qp + kPtDiagWaiting), blockIdx.x, threadIdx.x >> 6);
    }
#endif
    if (!ok && lane == 0) {
        // detail: the tile (bits 0-23); bits 24-30: how far the epoch is behind (an agent-scope atomic's
        // read, capped at 127); bit 31: that read is behind too (clear: only the polls saw a stale value)
        const uint32_t t = pt_entry_tile(e), part = pt_entry_part(e);
        uint32_t m = ~0u;
        if (part != 2u) m = __hip_atomic_fetch_add(const_cast<uint32_t*>(ep + 2u * t), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (part != 1u) {
            const uint32_t b = __hip_atomic_fetch_add(const_cast<uint32_t*>(ep + 2u * t + 1u), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            m = b < m ? b : m;
        }
        const uint32_t behind = m >= w ? 0u : (w - m < 127u ? w - m : 127u);
        pt_guard_report(err, PT_G_CHAIN_WAIT, (t & 0xffffffu) | (behind << 24) | (m < w ? 0x80000000u : 0u));
    }
}

// (the whole wave) after entry e's last pixel store: publish sequence number seq for it.  delay: the
// test hook PT_MI355_TEST_CHAIN_DELAY (~us slept first, so that the next launch meets unready tiles)
__device__ __forceinline__ void pt_chain_publish(uint32_t* ep, uint32_t e, uint32_t seq, uint32_t delay, int lane)
{
    if (__builtin_expect(delay != 0u, 0)) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * delay) __builtin_amdgcn_s_sleep(8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every lane's sc1 pixel stores have completed
    if (lane == 0) {
        const uint32_t t = pt_entry_tile(e), part = pt_entry_part(e);
        if (part != 2u) __hip_atomic_store(ep + 2u * t, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (part != 1u) __hip_atomic_store(ep + 2u * t + 1u, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
