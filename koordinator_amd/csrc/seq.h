// seq.h -- launch wrappers of seq.hip (host side; api.hip and seq.hip only,
// so DeviceShare changes do not rebuild kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "dev.hpp"
#include "kernels.h"
#include "ipa.hpp"
#include "pts.hpp"

namespace kh {

// Granules: phases A, B, 0 (PodTopologySpread hostname minimum), P (its raw
// Score min / max), each [2 parities][grid][SEQ_GRAN] u64, then the commit
// result ring (2 words), then the spin timeout word on its own 64 B.  Phase A
// uses words 0..5 (feasible count, raw maxima, best key), 6..14
// (PodTopologySpread's soft pairs) and 15..16 (InterPodAffinity's raw min / max).
constexpr int SEQ_GRAN = 32;
constexpr int SEQ_WORK_PLANES = 6;  // koordhip_eval_ext's work rows: total, 3 raw, PodTopologySpread raw,
                                    // InterPodAffinity raw
constexpr size_t seq_granule_words(int grid) { return (size_t)8 * grid * SEQ_GRAN + 8; }
constexpr size_t seq_tmo_offset(int grid) { return seq_granule_words(grid) * sizeof(uint64_t); }
constexpr size_t seq_granule_bytes(int grid) { return seq_tmo_offset(grid) + 64; }

// The exact sequential cycle (normalized-score profiles).  grid = resident
// blocks (one per CU); granules: 2 phases x 2 parities x grid x 8 u64 (zeroed
// before the first launch of a call), tmo: one u32 (zeroed).  rs: the
// Reservation plugin scores.  dbg: KOORDHIP_STAMPS counters (NULL: off).
// The host structs c and d must stay unchanged until the launch's copies of
// them ran (they are the context's own).
hipError_t launch_seq(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t n_pods,
                      int32_t grid, uint64_t *granules, uint32_t *tmo, int32_t *out_node, uint64_t *out_cpus,
                      uint32_t *out_dev, int32_t rs, uint64_t *dbg, void *desc, const PtsArgs &pts,
                      const IpaArgs &ipa, hipStream_t s);
// desc: a device buffer of seq_desc_bytes() the launch copies the config and
// the column descriptors into (the commit reads them from there)
constexpr size_t seq_desc_cfg_bytes() { return (sizeof(DevCfg) + 15) & ~(size_t)15; }
constexpr size_t seq_desc_bytes() { return seq_desc_cfg_bytes() + sizeof(DevNodes); }
// parity: status bits (ORed into status: k_eval_full writes them first;
// InterPodAffinity's into ipa_status [np][n], 1 = its Filter fails), the
// normalized plugins' raw planes of scores ([np][NPLUGINS + NEXT][n]), and
// the top-k of the normalized totals per pod; work: [np][SEQ_WORK_PLANES][n] int32
hipError_t launch_seq_eval(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t n_pods,
                           int32_t rs, uint8_t *status, uint8_t *ipa_status, int32_t *scores, int32_t *work, int32_t k,
                           uint64_t *topk, const PtsArgs &pts, const IpaArgs &ipa, hipStream_t s);
// Reserve (sign > 0) / Unreserve (sign < 0) of one pod with its ext record on
// `node` (koordhip_commit_ext / koordhip_uncommit_ext); one device thread.  cpus
// [NW], dev [DT]: Reserve's outputs, Unreserve's inputs; rc: 0 / KOORDHIP_ERESERVE
// / KOORDHIP_EINVAL.  rs: the Reservation plugin scores (PreScore nominated).
hipError_t launch_commit_ext(const DevCfg &c, const DevNodes &d, const DevPod *pod, const DevPodX *px, int32_t node,
                             int32_t sign, int32_t rs, uint64_t *cpus, uint32_t *dev, int32_t *rc, const PtsArgs &pts,
                             const IpaArgs &ipa, hipStream_t s);
// Device pods inside the pipelined greedy (plain build, seq_mode 0): per place
// call launch_ext_begin once, then per device pod e (staged index gp, round u)
// launch_ext_pre (a wait for the resolve's rounds < `rounds` = u - lead, the
// device commits of the first `needc` device pods and the final of e - ext_ring(),
// whose ring buffer it reuses; then the pre-evaluation of every node) and
// launch_ext_final (a wait for sync->ext_req = gp + 1 and pre-evaluation e, then
// the exact placement over the pre-evaluated values with the X nodes and the
// commit-log rounds [xlo, xhi) evaluated again; out_node, sync->ext_done,
// DeviceShare's Reserve without the Fit / LoadAware row, out_dev).  Every wait
// is one workgroup on device flags; submitted in an order whose waits the
// launches before them satisfy (api.hip), they stay deadlock-free on one stream
// or two.  scratch: ext_scratch_bytes(n_ext, n).
size_t ext_scratch_bytes(int32_t n_ext, int32_t n);
int32_t ext_ring();
hipError_t launch_ext_begin(const DevNodes &d, int32_t n_ext, void *scratch, hipStream_t s);
// the device word counting the finals' re-evaluated nodes of the call (zeroed by launch_ext_begin)
const uint32_t *ext_reevals(const void *scratch, int32_t n_ext, int32_t n);
hipError_t launch_ext_pre(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t e,
                          int32_t gp, int32_t rounds, int32_t needc, int32_t n_ext, void *scratch, PipeSync *sync,
                          hipStream_t s);
// (ext_idx: the device pods' staged indices on the device; dlo: the `needc`
// pre-evaluation e waited for -- the device pods [dlo, e) may have committed
// after it read their nodes, which the final then evaluates in full)
hipError_t launch_ext_final(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t e,
                            int32_t gp, int32_t xlo, int32_t xhi, int32_t n_ext, void *scratch, int32_t *out_node,
                            uint32_t *out_dev, PipeSync *sync, uint64_t *dbg, const int32_t *ext_idx, int32_t dlo,
                            hipStream_t s);
hipError_t launch_mark_ext(DevPod *pods, const int32_t *idx, int32_t n, hipStream_t s);
// the k_seq instantiation launch_seq runs for this config, as rocprofv3 names it
const char *seq_kernel_name(const DevCfg &c, const DevNodes &d);

}  // namespace kh
