// pod.hpp -- the device pod record and the exact-f64 quantity range shared by
// every kernel of libkoordhip.so.
#pragma once
#include <stdint.h>

#include "../../include/koordhip.h"

namespace kh {

// Largest quantity magnitude the engine accepts (validated by the host side
// of api.hip): every quantity is then an exact f64 (see eval.hpp).
constexpr double KH_EXACT_LIMIT = 35184372088832.0;  // 2^45

// Device copy of one koordhip_pod (same fields, quantities as exact f64).
struct DevPod {
  double req[KOORDHIP_NRES];
  double nz_cpu_m, nz_mem;
  double est_cpu, est_mem;
  uint32_t flags;
  int32_t numa_cpus;
  uint32_t numa_policy;
  int32_t sclass;  // static class (KOORDHIP_PLUGIN_NODE_STATIC), 0 .. 31
  uint64_t resv_match;
};
static_assert(sizeof(DevPod) == 96, "DevPod is 96 bytes");

// Engine-internal flag bit (never from the host API: to_dev_pods rejects it):
// a pod whose koordhip_pod_ext record requests devices / extended scalars,
// placed inside the pipelined greedy by k_ext_pre / k_ext_final (seq.hip) -- the resolve
// hands it the exact state and takes its node back.
constexpr uint32_t KH_POD_EXT = 1u << 30;

// Engine-internal flag bit (set by the host from the pod's koordhip_pod_ext;
// to_dev_pods rejects it from callers): DeviceShare is in the profile and the
// pod requests devices, so DeviceShare's FilterReservation takes part in the
// reservation nomination (deviceshare/plugin.go:325-356) -- it fails every
// reservation holding no devices, and none does in the engine's envelope, so
// such a pod is nominated into no reservation (resv_nominate, resv.hpp).
constexpr uint32_t KH_POD_DEVSHARE = 1u << 29;

}  // namespace kh
