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

// cross-fade alpha (process_tomatis_xfade.py:251-274), float64 exactly as the
// reference: +-step toward the target (0 in C1, 1 in C2), snapped once within
// a step (callers: a = xf > 0 ? alpha_step(a, tgt, 1.0 / xf) : tgt)
__device__ __forceinline__ double alpha_step(double a, double tgt, double step) {
  const double d = tgt - a;
  if (fabs(d) <= step) return tgt;
  return a + step * (d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0));
}
// gain row of an alpha: the pure rows 0 (C1) / 1 (C2), else lattice row 2 + m
__device__ __forceinline__ uint16_t xfade_row(double a, int xf) {
  if (xf > 0 && a > 0.0 && a < 1.0) return (uint16_t)(2 + (int)rint(a * xf));
  return (a < 0.5) ? 0 : 1;
}

}  // namespace tgate
