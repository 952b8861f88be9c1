// kernels.h — host-side declarations of the HIP launchers in kernels.hip.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>
#include "image.h"

#define TM_MODE_COUNT 0
#define TM_MODE_EMIT 1
#define TM_MODE_STATS 2

// fused-kernel variants (A/B; TM_WALK env in the engine)
#define TM_VARIANT_LANE 0
#define TM_VARIANT_TILE256 1
#define TM_VARIANT_TILE512 2
#define TM_VARIANT_TILE1024 3
#define TM_VARIANT_QUEUE 5

namespace tmx {

// marks: 8 events, [2i] before / [2i+1] after stage i (tokenize, walk, scan, copy-out), or null
hipError_t launch_queue(bool stats_mode, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, uint32_t* words, uint32_t* meta, uint32_t* path_scratch, uint32_t* stage,
                        uint32_t K, uint32_t* counts, uint64_t* out_off, uint32_t* out, uint64_t out_cap,
                        uint64_t* total, uint64_t* scan_tmp, unsigned long long* ws, unsigned long long* stats,
                        hipStream_t st, hipEvent_t* marks);
hipError_t launch_tokenize(const ImageView& im, const uint8_t* bytes, const uint64_t* off, uint32_t n,
                           uint32_t* words, uint32_t* meta, hipStream_t st);
hipError_t launch_match(int mode, bool long_topics, const ImageView& im, const uint64_t* off, uint32_t n,
                        const uint32_t* words, const uint32_t* meta, uint32_t* counts,
                        const uint64_t* out_off, uint32_t* out, uint64_t out_cap,
                        uint32_t* path_scratch, unsigned long long* stats, hipStream_t st);
size_t scan_tmp_elems(uint32_t n);
size_t fused_ws_words(uint32_t n);
size_t fused_stage_elems(uint32_t n, uint32_t K);
hipError_t launch_fused(int variant, bool stats_mode, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, uint32_t* words, uint32_t* path_scratch, uint32_t* stage, uint32_t K,
                        uint32_t* counts, uint64_t* out_off, uint32_t* out, uint64_t out_cap, uint64_t* total,
                        unsigned long long* ws, unsigned long long* stats, hipStream_t st);
hipError_t launch_scan(const uint32_t* counts, uint32_t n, uint64_t* out_off, uint64_t* total,
                       uint64_t* tmp, hipStream_t st);

}  // namespace tmx
