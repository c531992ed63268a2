// Test harness: csrc/libinj.h (the device restatement of libinjection)
// compiled for the host, so the CPU suite can compare the very code the
// kernels run with oracle/libinjection.py on large corpora.  Test-only.
#define __device__
#define __constant__
#define __noinline__ __attribute__((noinline))
#define __forceinline__ inline
#define GI_HD             // gi_program.h's markers, host build
#define GI_TABLE static const
#include "../../coraza-kubernetes-operator_amd/csrc/libinj.h"

extern "C" int li_host_sqli(const uint8_t* s, uint32_t n) {
  gi::LiSqli st;
  return gi::li_detect_sqli(s, n, &st, gi::li_tables_const()) ? 1 : 0;
}
extern "C" int li_host_candidate(int sqli, const uint8_t* s, uint32_t n) { return gi::li_candidate(sqli != 0, s, n) ? 1 : 0; }
extern "C" int li_host_xss(const uint8_t* s, uint32_t n) { return gi::li_detect_xss(s, n) ? 1 : 0; }
extern "C" int li_host_fp_black(const uint8_t* f, uint32_t n) { return gi::li_fp_black(f, n) ? 1 : 0; }
