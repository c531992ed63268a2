// Kernel-side batch descriptor and launch entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuinspect.h"
#include "gi_program.h"

namespace gi {

// Per-request scratch layout (computed by the host from request lengths when
// the batch is staged; see runtime.cpp gi_stage_batch).  Region =
// [256 B ReqHdr][cap_f fields][TX slots][cap_b bytes][2 x cap_t][2 x cap_mt].
struct ReqLayout {
  uint64_t base;   // byte offset of the request's region in DBatch.scratch
  uint32_t cap_f;  // field records
  uint32_t cap_b;  // decoded-bytes arena
  uint32_t cap_t;  // each of the two transformation buffers
  uint32_t cap_mt; // macro expansion scratch == TX string arena size
};

struct DBatch {
  const uint8_t* data;
  const gi_request* reqs;
  const gi_header* headers;
  uint32_t n_req;
  uint32_t mcap;
  uint8_t* scratch;
  const ReqLayout* layout;
  gi_verdict* verdicts;
  uint32_t* matched;
  unsigned long long* tally;  // gi_tally as 6 counters
  uint32_t* hits;             // phase-A hit words [ceil(n_hit_slots/32)][n_req]
  uint8_t* tscratch;          // k_match transformation buffers (2 x tcap per resident thread)
  uint32_t tcap;
};

// Resident thread count of k_match with lds_bytes of dynamic LDS per block.
uint32_t scan_resident_threads(uint32_t lds_bytes);

// k_collect -> k_scan -> k_eval on `stream`; ev (optional) = 2 events recorded
// after k_collect and after k_match.
void launch_pipeline(const DProgram& P, const DBatch& B, uint32_t scan_threads, hipStream_t stream,
                     hipEvent_t* ev);

}  // namespace gi
