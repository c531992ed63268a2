// Kernel-side batch descriptor and launch entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuinspect.h"
#include "gi_program.h"

namespace gi {

// Per-request scratch layout (computed by the host from request lengths when
// the batch is staged; see runtime.cpp stage()).
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
};

void launch_inspect(const DProgram& P, const DBatch& B, hipStream_t stream);

}  // namespace gi
