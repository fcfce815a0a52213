// rows.hpp -- the node rows the pipelined greedy's kernels share (kernels.hip:
// k_scan / k_resolve; cls.hip: the class lists): the side row of each plugin
// set (NM), its loads / stores, and one (pod, node) evaluation on a row.
#pragma once
#include <type_traits>

#include "eval.hpp"

namespace kh {

// NM: 0 = no NodeNUMAResource, 1 = NodeNUMAResource, 2 = ... with
// topology-policy nodes (the zone code is compiled only here), 3 = with the
// Reservation plugin (NUMA side rows carry the node's reservation), 4 = ...
// with several reservations per node (KOORDHIP_RESV_SLOTS slots per row), 5 =
// ... with reservations holding CPUs (the Score's preferred-CPU Allocate runs
// the accumulator: its registers cap these kernels at 2 waves per SIMD)
template <int NM>
using side_row_t = typename std::conditional<NM >= 4, NumaRowR4,
                                             typename std::conditional<NM == 3, NumaRowR, NumaRow>::type>::type;

template <int NM>
__device__ __forceinline__ void load_side_row(side_row_t<NM> &r, const DevNodes &d, int32_t i) {
  load_numa_row<NM == 2>(r, d, i);
  if constexpr (NM >= 3) load_resv(r, d.rv, i);
}
template <int NM>
__device__ __forceinline__ void store_side_row(const side_row_t<NM> &r, const DevNodes &d, int32_t i) {
  store_numa_row<NM == 2>(r, d, i);
  if constexpr (NM >= 3) store_resv(r, d.rv, i);
}
template <int NM>
__device__ __forceinline__ void store_side_row_wt(const side_row_t<NM> &r, const DevNodes &d, int32_t i) {
  store_numa_row_wt<NM == 2>(r, d, i);
  if constexpr (NM >= 3) store_resv_wt(r, d.rv, i);
}

template <int NM>
__device__ __forceinline__ int32_t eval_row(const DevPod &p, const NV &v, const side_row_t<NM> &nr,
                                            const DevNumaClass *cls, const DevCfg &c) {
  if constexpr (NM >= 3) {
    return eval_total_resv<side_row_t<NM>::kSlots, NM == 5>(p, v, nr, cls, c);
  } else if constexpr (NM != 0) {
    return eval_total_numa<NM == 2>(p, v, nr, cls, c);
  } else {
    (void)nr;
    (void)cls;
    return eval_total(p, v, c);
  }
}

}  // namespace kh
