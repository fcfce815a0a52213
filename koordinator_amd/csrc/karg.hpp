// karg.hpp -- wave-uniform kernel arguments re-read from the kernarg segment.
//
// The evaluation kernels take DevCfg and DevNodes by value: ~50 column
// pointers and the plugin configuration, more wave-uniform values than a
// wave's 102 SGPRs.  The compiler then parks them in VGPR lanes and spends one
// v_readlane per use (42 % of k_eval_topk<3>'s loop VALU instructions before
// this helper).  kernarg_fresh returns the argument at byte `off` of the
// kernarg segment through a pointer the compiler cannot follow across the
// asm, so each evaluation re-reads what it needs with scalar loads (the
// scalar cache holds the segment) instead of keeping it live.  Offsets follow
// the kernel's explicit argument order (each argument at its natural
// alignment; DevCfg first and DevNodes right after it, asserted below).
// Call it in wave-uniform control flow only: inside a divergent branch (a
// per-lane node guard) the multi-slot Reservation builds read wrong values
// (test_reservation_slots' streams), outside it they are bit-exact.  The
// pod record stays in SGPRs: re-reading it per evaluation put its scalar
// loads on every evaluation's critical path (config 5 230k -> 168k pods/s).
#pragma once
#include <hip/hip_runtime.h>

#include "eval.hpp"

namespace kh {

template <class T>
__device__ __forceinline__ const T &kernarg_fresh(size_t off) {
  const __attribute__((address_space(4))) char *k =
      (const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(k));
  return *(const T *)(k + off);
}
static_assert(sizeof(DevCfg) % alignof(DevNodes) == 0, "DevNodes follows DevCfg in the kernarg segment");
constexpr size_t KARG_NODES = sizeof(DevCfg);  // (DevCfg c, DevNodes d, ...) kernels

}  // namespace kh
