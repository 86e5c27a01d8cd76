// pt_wave.h -- wave-level votes on a bool lane predicate, for gfx950 wave64.
//
// HIP's __ballot(int) / __any(int) take the predicate as an int: the compiler materialises it in a
// VGPR (v_cndmask 0/1) and compares it back to a lane mask (v_cmp_ne) before the ballot -- two
// 4-cycle VALU instructions per vote in a loop whose predicates already live in SGPR lane masks.
// The builtin on the bool itself is the lane mask ANDed with exec: SALU only.
#pragma once
#include <stdint.h>

__device__ __forceinline__ uint64_t pt_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool pt_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
