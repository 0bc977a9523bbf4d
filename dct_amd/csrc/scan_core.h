// dct_amd/csrc/scan_core.h -- wave- and workgroup-level scans for the RLE
// symbol offsets ("prefix-sum compaction").
//
// Why no single-pass (decoupled look-back) scan: it needs tiles claimed in
// order from one atomic word, and one word saturates near 88 claims/us on
// MI355X (MI355X_MICROARCH.md "dequeue"), while the count pass streams ~700
// 64-block tiles/us.  A static grid-stride assignment (no claim word, the grid
// co-resident) fails the other way: the batches of one sweep are all in flight
// together, so a wave's predecessors have only their aggregates, and its
// look-back walks back through up to one sweep (~4 096 batches, 64 per flag
// read at ~1 us each) per batch, against ~6 us of work per batch.  The counts
// therefore go reduce-then-scan: per-tile totals, one workgroup scan of the
// totals, a fix-up.
#pragma once
#include "dctq_internal.h"

namespace dctq {

// Inclusive wave scan (DPP row shifts + row broadcasts: VALU only, no LDS).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t e) {
    e += __builtin_amdgcn_update_dpp(0u, e, 0x111, 0xF, 0xF, false);  // row_shr:1
    e += __builtin_amdgcn_update_dpp(0u, e, 0x112, 0xF, 0xF, false);  // row_shr:2
    e += __builtin_amdgcn_update_dpp(0u, e, 0x114, 0xF, 0xF, false);  // row_shr:4
    e += __builtin_amdgcn_update_dpp(0u, e, 0x118, 0xF, 0xF, false);  // row_shr:8
    e += __builtin_amdgcn_update_dpp(0u, e, 0x142, 0xA, 0xF, false);  // row_bcast:15
    e += __builtin_amdgcn_update_dpp(0u, e, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return e;
}

}  // namespace dctq
