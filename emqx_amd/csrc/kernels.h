// kernels.h — host-side declarations of the HIP launchers in kernels.hip.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>
#include "image.h"

namespace tmx {

constexpr uint32_t WREG = 16;        // topic levels kept in VGPRs / LDS path slots; longer
                                     // topics keep their path in global scratch
constexpr size_t QWS_BYTES = 1024;   // queue heads: 8 ranges x 128 B
constexpr size_t STATS_BYTES = 512;  // 8 totals + per-level diagnostic histogram

// per-batch device workspace of the queue pipeline
struct QueueBufs {
    uint32_t* twords;     // n x WREG word ids (levels < WREG)
    uint32_t* words;      // levels >= WREG of long topics, at (byte offset + topic index)
    uint32_t* meta;       // n: levels | long << 30 | dollar << 31
    uint32_t* path;       // global path of long topics, at (byte offset + 2 x topic index)
    uint32_t* stage;      // n x K: first K ids of each topic (written from the row's end)
    uint64_t* scan_tmp;   // scan_tmp_elems(n)
    unsigned long long* ws;   // QWS_BYTES of queue heads
};

// tokenize -> NFA walk -> scan -> copy-out, all on st.  marks: 8 events,
// [2i] before / [2i+1] after stage i, or null.  out_cap == 0: counts and
// offsets only.  stats (6 x u64, zeroed by the caller) is filled when
// stats_mode: levels, visits, edge reads, matches, leaf visits, probe loads.
hipError_t launch_queue(bool stats_mode, bool xcdq, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, const QueueBufs& qb, uint32_t K, uint32_t* counts, uint64_t* out_off,
                        uint32_t* out, uint64_t out_cap, uint64_t* total, unsigned long long* stats,
                        hipStream_t st, hipEvent_t* marks, uint32_t walk_blocks_per_cu = 0, bool hist = false);
size_t scan_tmp_elems(uint32_t n);

}  // namespace tmx
