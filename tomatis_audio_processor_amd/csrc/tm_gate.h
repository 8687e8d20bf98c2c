// tm_gate.h -- the standard gate automaton on exact level predicates, shared
// by the gate kernels (tm_kernels.hip) and the fused transform's in-kernel gate
// (tm_transform.hip).  Reference: src/process_tomatis.py:373-385.
// state id: 0 = C1 idle, 1..D = C1 pending for (id-1) frames, D+1 = C2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tomatis_hip.h"

namespace tgate {

// (n <= 4, TomatisStream's arrays; constant indices keep a register copy of
// the stream struct out of scratch)
__device__ __forceinline__ bool in_exc(uint32_t b, const uint32_t* e, int n) {
  bool hit = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) hit |= (i < n) && (b == e[i]);
  return hit;
}
// bit 0: level >= Ton, bit 1: level <= Toff -- decided on r's float32 bit
// pattern (dsp.gate_bits: integer threshold + the exception list where numpy's
// log10 is not monotone), so no level is computed on the device
__device__ __forceinline__ uint8_t gate_pred(float r, const TomatisStream& S) {
  const uint32_t b = __float_as_uint(r);
  if (r != r) return 0;
  const bool on = (b >= S.on_bits) != in_exc(b, S.on_exc, S.n_on_exc);
  const bool off = (b <= S.off_bits) != in_exc(b, S.off_exc, S.n_off_exc);
  return (uint8_t)((on ? 1 : 0) | (off ? 2 : 0));
}
__device__ __forceinline__ int gate_step(int id, uint8_t pr, int D) {
  if (id == D + 1) return (pr & 2) ? 0 : id;
  if (pr & 1) {
    const int age = (id == 0) ? 0 : id;  // frames since pending was set, after this frame
    return (age >= D) ? D + 1 : age + 1;
  }
  return 0;
}

}  // namespace tgate
