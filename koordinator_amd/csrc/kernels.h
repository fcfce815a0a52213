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
// k_scan / k_scan_nm: score matrix S[p][i - lo] = total score + 1 (0 =
// infeasible) over the shard [lo, hi), XCD-aware grid; Mx[p][chunk] = the
// best value of chunk (64 x R nodes).  ppw > 0 and R <= 2: node-major, one
// wave per (chunk, group of ppw pods) with the node columns loaded once into
// VGPRs; ppw == 0: pod-major, one wave per (pod, chunk), R in {1, 2, 4, 8}
// (NUMA: {1, 2, 4}).  scan_ppw: the default group size (~2 waves per SIMD).
int32_t scan_chunks(int R, int32_t lo, int32_t hi);
int32_t scan_ppw(int R, int32_t lo, int32_t hi, int32_t n_pods);
hipError_t launch_scan(int R, const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods, int32_t lo,
                       int32_t hi, uint16_t *S, int64_t s_stride, uint16_t *Mx, int32_t m_stride, int32_t ppw,
                       hipStream_t s);
// k_select: per pod the exact top-k keys of its S row (best first, 0-padded);
// nbins = max total score + 2
hipError_t launch_select(const uint16_t *S, int64_t s_stride, int32_t lo, int32_t m, int32_t n_pods, int32_t k,
                         int32_t nbins, const uint16_t *Mx, int32_t m_stride, int32_t nchunks, uint64_t *out,
                         uint64_t *dbg, hipStream_t s);
// k_select_split: the same top-k with G workgroups per pod (row slices) and an
// in-launch merge by each pod's last workgroup.  part: [n_pods][G][k] slice
// lists (kSelPartKeys keys); cnt: kSelMaxPods arrival counters, zero before
// the first launch (the kernel leaves them zero); sync: optional, sel[sel_par]
// += 1 per pod once its final list in `out` is published, and with res_wait >
// 0 the launch does not end before res_round >= res_wait.
struct PipeSync;
constexpr int kSelGMax = 16;
constexpr int kSelMaxPods = 64;
constexpr size_t kSelPartKeys = (size_t)kSelMaxPods * kSelGMax * 128;
int32_t select_split_groups(int32_t m, int32_t G);
hipError_t launch_select_split(const uint16_t *S, int64_t s_stride, int32_t lo, int32_t m, int32_t n_pods, int32_t k,
                               int32_t nbins, const uint16_t *Mx, int32_t m_stride, int32_t nchunks, int32_t G,
                               uint64_t *part, uint32_t *cnt, uint64_t *out, PipeSync *sync, int32_t sel_par,
                               int32_t res_wait, hipStream_t s);
// k_eval_topk: evaluation + exact per-pod top-k in one launch, no score
// matrix: one workgroup per (pod, slice of 256 x VT nodes); each slice hands
// on its own top-k keys, the pod's last slice merges them into out[p][k]
// (best first, 0-padded) and, with `sync`, counts the pod into sel[sel_par]
// (like k_select_split).  part: [n_pods][slices][k] keys, pcnt:
// [n_pods][slices], arrive: [n_pods] words that are zero before a launch and
// left zero by it.  eval_topk_vt: the slice width for k-key lists.
int32_t eval_topk_slices(int VT, int32_t lo, int32_t hi);
int eval_topk_vt(int nm, int32_t n_cu, int32_t n_pods, int32_t lo, int32_t hi, int32_t k);
hipError_t launch_eval_topk(const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods, int32_t lo,
                            int32_t hi, int32_t k, int VT, uint64_t *part, int32_t *pcnt, uint32_t *arrive,
                            uint64_t *out, PipeSync *sync, int32_t sel_par, int32_t res_wait, uint64_t *dbg,
                            hipStream_t s);
// lists: ranges ascending with l, equal-score keys in ascending node order
// sync: optional, sel[sel_par] += 1 per pod once its merged list is published
hipError_t launch_topk_merge(const uint64_t *in, int64_t pod_stride, int64_t list_stride, int32_t n_pods, int32_t L,
                             int32_t k, int32_t score_bits, uint64_t *out, PipeSync *sync, int32_t sel_par,
                             hipStream_t s);
template <typename T>
hipError_t launch_scatter(T *dst, const T *src, const int32_t *idx, int32_t m, hipStream_t s);
// whole rows of `bytes` (a multiple of 4) per node
hipError_t launch_scatter_rows(void *dst, const void *src, const int32_t *idx, int32_t m, int32_t bytes, hipStream_t s);
// The round pipeline (kernels.hip): k_resolve resolves rounds [r_begin, r_end)
// of the staged stream (P pods per round, k keys per list).  Round r's lists
// are evaluated on the state after round r - 1 - lag (lag 1: k >= 2P, lists
// double buffered at lists0 + (r & 1) * list_buf; lag 2: one persistent
// launch, k >= 3P, four buffers at (r & 3)); it waits for sel[r & 1] (the
// cumulative pods of the rounds of r's parity) and publishes res_round in
// `sync`; M' is handed between launches in mbuf ({count, nodes}, lag 1).  The
// evaluation stream(s) bracket each round with k_wait_resolved (before k_scan)
// and k_signal_lists (after the lists).
constexpr int32_t kResolveMaxK = 128;  // longest list the resolve takes (RES_MAXP)
// nm: the kernels' node-row mode, 0 none, 1 NodeNUMAResource, 2 + topology-policy zones, 3 + Reservation
int side_mode(const DevCfg &c);
// the last evaluation / resolve kernel instantiation launched by this host
// thread, as rocprofv3 names it ("kh::k_scan<4, 0>")
const char *last_eval_kernel();
const char *last_resolve_kernel();

int32_t resolve_lds_bytes(int32_t n_pods_max, int32_t k, int32_t n_nodes, int nm, int32_t lag);
hipError_t launch_resolve(const DevCfg &c, const DevNodes &d, const DevNodes *d_desc, const DevPod *pods, int32_t total, int32_t P, int32_t k,
                          int32_t r_begin, int32_t r_end, const uint64_t *lists0, int64_t list_buf, int32_t monotone,
                          int32_t lag, PipeSync *sync, int32_t *mbuf, int32_t *out_node, uint64_t *out_cpus, uint64_t *dbg,
                          int32_t trace, hipStream_t s);
hipError_t launch_wait_resolved(PipeSync *sync, int32_t rounds, hipStream_t s);
hipError_t launch_signal_lists(PipeSync *sync, int32_t par, int32_t pods, hipStream_t s);
constexpr size_t kPipeSyncBytes = 384 + 4 * (1 + 128);  // PipeSync (three 128-B lines) + the X list (pipe.hpp kPipeXMax)
constexpr int kPipeSyncErrWord = 3;  // PipeSync {sel[2], res_round, err, ...}: err's int32 index
constexpr int kPipeSyncExtReqWord = 32, kPipeSyncExtDoneWord = 64;
// single Reserve (sign +1, cpus <- allocated CPUs, *rc = KOORDHIP_ERESERVE on failure) / Unreserve (cpus given)
hipError_t launch_commit(const DevCfg &c, const DevNodes &d, const DevPod *pod, int32_t node, int32_t sign,
                         uint64_t *cpus, int32_t *rc, hipStream_t s);

}  // namespace kh
