// kernels.h -- launch wrappers of kernels.hip (host side).
#pragma once
#include <hip/hip_runtime.h>

#include "eval.hpp"

namespace kh {

// LoadAware Filter inputs (device copies of koordhip_node_soa.laf_* / la_flags).
struct PrepIn {
  const int64_t *used_m[2];
  const int64_t *total_m[2];
  const int64_t *prod_used_m[2];
  const int64_t *thr[2];
  const int64_t *prod_thr[2];
  const uint8_t *la_flags;
};

hipError_t launch_prep_flags(const PrepIn &in, const DevNodes &d, const int32_t *rows, int32_t m, hipStream_t s);
hipError_t launch_eval_full(const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods,
                            uint8_t *status, int32_t *scores, hipStream_t s);
// k_topk_partial: one wave evaluates 64 x R nodes (R in {1, 2, 4, 8})
hipError_t launch_topk_partial(int R, const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods,
                               int32_t lo, int32_t hi, int32_t nchunks, int32_t k, int32_t score_bits,
                               uint64_t *out, hipStream_t s);
// lists: ranges ascending with l, equal-score keys in ascending node order
hipError_t launch_topk_merge(const uint64_t *in, int64_t pod_stride, int64_t list_stride, int32_t n_pods, int32_t L,
                             int32_t k, int32_t score_bits, uint64_t *out, hipStream_t s);
template <typename T>
hipError_t launch_scatter(T *dst, const T *src, const int32_t *idx, int32_t m, hipStream_t s);
hipError_t launch_resolve(const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods, int32_t k,
                          const uint64_t *lists, int32_t monotone, int32_t *out_node, uint64_t *out_cpus,
                          uint64_t *dbg, hipStream_t s);
// single Reserve (sign +1, cpus <- allocated CPUs, *rc = KOORDHIP_ERESERVE on failure) / Unreserve (cpus given)
hipError_t launch_commit(const DevCfg &c, const DevNodes &d, const DevPod *pod, int32_t node, int32_t sign,
                         uint64_t *cpus, int32_t *rc, hipStream_t s);

}  // namespace kh
