// kg_interp.hip -- rewrite interpreter for queries whose reachable region holds subject-set
// rewrites (internal/check/rewrites.go, binop.go).  First milestone: not yet implemented on the
// device; such queries return KG_ERROR / KG_ERR_NOT_IMPLEMENTED (never a silent CPU fallback).
#include <hip/hip_runtime.h>

#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

__global__ void k_general_stub(const uint32_t* gen_list, const uint32_t* gen_count, uint8_t* out, uint32_t* err) {
  uint32_t n = *gen_count;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t qi = gen_list[i];
    out[qi] = KG_ERROR;
    if (err) err[qi] = KG_ERR_NOT_IMPLEMENTED;
  }
}

int launch_general(Snapshot* s, const RQuery* rq, const uint32_t* gen_list, const uint32_t* gen_count,
                   uint32_t* gen_head, uint8_t* out, uint32_t* err, unsigned long long* st_general,
                   unsigned long long* st_rows, unsigned long long* st_edges, unsigned long long* st_probes,
                   hipStream_t stream) {
  (void)rq;
  (void)gen_head;
  (void)st_general;
  (void)st_rows;
  (void)st_edges;
  (void)st_probes;
  hipLaunchKernelGGL(k_general_stub, dim3(64), dim3(256), 0, stream, gen_list, gen_count, out, err);
  HIPC(hipGetLastError());
  (void)s;
  return 0;
}

}  // namespace kg
