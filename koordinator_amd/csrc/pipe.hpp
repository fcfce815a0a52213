// pipe.hpp -- the device flags of the round pipeline, shared by kernels.hip
// (k_select_split, k_eval_topk, k_resolve) and cls.hip (the class lists).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kh {

static __device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// Device-side handshake between the evaluation stream and the persistent
// resolve kernel (one per koordhip_place_staged call):
//   sel[b]     pods of the rounds with parity b whose final lists are ready
//              (cumulative; rounds alternate between two evaluation streams, so
//              a later round may finish first) (k_select_split's
//              merging workgroups add 1 each; k_signal_lists stores the count
//              after a separate merge)
//   res_round  rounds resolved + written back (k_resolve, release store)
//   err        a side gave up waiting (watchdog): the call fails, nothing hangs
//   ext_req    device pods placed inside the pipeline (k_ext_final, seq.hip):
//              the resolve stores pod index + 1 once every earlier commit is
//              written back (write-through, drained)
//   ext_done   k_ext_final stores pod index + 1 once that pod's placement is
//              published (out_node write-through); its DeviceShare Reserve
//              follows, published in the ext flags (cdone)
// Every flag many waves poll has a 128-B line of its own: relaxed agent-scope
// polls of one line from a few hundred workgroups serialise at its home and
// delay every other waiter on it (round 5's persistent device-pod worker's
// idle workgroups made a step 5x slower before ext_req / ext_done moved off
// sel / res_round).
struct PipeSync {
  int32_t sel[2], res_round, err;
  int32_t pad0[28];
  int32_t ext_req;
  int32_t pad1[31];
  int32_t ext_done;
  int32_t pad2[31];
};
static_assert(sizeof(PipeSync) == 384, "PipeSync lines");
// After the struct: the resolve's X set at a device-pod hand-off, {count,
// nodes[kPipeXMax]} (M' and this round's M so far), stored write-through
// before ext_req.
constexpr int kPipeXMax = 128;
static __device__ __forceinline__ int32_t *pipe_xlist(PipeSync *sy) { return reinterpret_cast<int32_t *>(sy + 1); }

constexpr uint64_t PIPE_WATCHDOG = 8ull << 30;  // s_memtime ticks (~seconds) before a waiter gives up

static __device__ __forceinline__ int32_t load_acquire(const int32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
static __device__ __forceinline__ int32_t load_relaxed(const int32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Publish a flag after this wave's global stores (MI355X_MICROARCH.md
// cross-XCD hand-off: wait for the stores, write the XCD L2 back, wait for
// the write-back -- spelled out in asm because ROCm 7.2 can drop the wait
// after buffer_wbl2 -- then a relaxed agent-scope flag store).
static __device__ __forceinline__ void store_release(int32_t *p, int32_t v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One pod's final list is stored write-through (st_wt: every byte sc1, every
// storing wave drained vmcnt and met at a barrier): count it into sel[par]
// with a relaxed agent add, no release fence (Guideline 16 R1; the resolve's
// wave acquires after its poll).
static __device__ void pipe_count_pod(PipeSync *sy, int32_t par) {
  __hip_atomic_fetch_add(&sy->sel[par], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Spin (one thread) until *p >= v; false when the watchdog fires or the other
// side reported an error.  Relaxed polls, ONE agent acquire after the match
// (an acquire per poll costs 2-3x per hop, Guideline 16 Pitfall 5).
static __device__ bool wait_at_least(const int32_t *p, int32_t v, PipeSync *sy) {
  const uint64_t t0 = stamp();
  while (load_relaxed(p) < v) {
    if (load_relaxed(&sy->err)) return false;
    if (stamp() - t0 > PIPE_WATCHDOG) {
      store_release(&sy->err, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}
// The same for waiters off the critical path (idle
// workgroups): longer sleeps, the error word read every 16th poll.
static __device__ bool wait_at_least_idle(const int32_t *p, int32_t v, PipeSync *sy) {
  const uint64_t t0 = stamp();
  for (uint32_t k = 0; load_relaxed(p) < v; k++) {
    if ((k & 15u) == 15u && load_relaxed(&sy->err)) return false;
    if (stamp() - t0 > PIPE_WATCHDOG) {
      store_release(&sy->err, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(32);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}

}  // namespace kh
