// api.hip -- the C-ABI of libkoordhip.so (include/koordhip.h): context,
// HBM-resident columnar snapshot, the round loop of the greedy stream and the
// RCCL all-gather of per-shard top-k for node-sharded multi-GPU runs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/koordhip.h"
#include "cls.h"
#include "kernels.h"
#include "seq.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail(KOORDHIP_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));       \
  } while (0)

#define NCCL_TRY(expr)                                                                        \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) return fail(KOORDHIP_ECOMM, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

constexpr int kDefaultBatch = 24;  // config-4 round-size sweep: 24 best (970k pods/s vs 911k at 32)
constexpr int kDefaultBatchNuma = 16;
constexpr int kDefaultBatchResv = 32;  // config 5 (evaluation-bound): 143k pods/s vs 135k at 16
constexpr int32_t kMaxNodes = 400000;  // the resolve keeps a per-node bit in LDS (next to 2 x 64 x 128 list keys)
constexpr int kMaxBatch = 64;
// plugin_weight[p] / koordhip_eval's score plane p belong to these plugins
constexpr uint32_t kScorePluginBit[KOORDHIP_NPLUGINS] = {KOORDHIP_PLUGIN_FIT, KOORDHIP_PLUGIN_LOADAWARE,
                                                          KOORDHIP_PLUGIN_NUMA, KOORDHIP_PLUGIN_BALANCED};
constexpr int kRing = 4;               // per-round events in flight (lag-1 pipeline needs 3)

// Contexts of one process sharing node shards without RCCL
// (koordhip_comm_init_local): a generation barrier per exchange step; a
// failing member aborts the group so its peers return instead of waiting.
struct LocalGroup {
  int32_t world = 0;
  std::vector<koordhip_ctx *> ctx;
  std::vector<int64_t> keys;
  std::mutex mu;
  std::condition_variable cv;
  int32_t arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;

  bool barrier() {
    std::unique_lock<std::mutex> l(mu);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return true;
    }
    cv.wait(l, [&] { return gen != g || aborted; });
    return gen != g;
  }
  void abort() {
    std::lock_guard<std::mutex> l(mu);
    aborted = true;
    cv.notify_all();
  }
};

}  // namespace

struct koordhip_ctx {
  koordhip_config cfg{};
  kh::DevCfg dc{};
  int device = 0;
  hipStream_t stream = nullptr;
  int32_t n = 0;
  bool loaded = false;
  int32_t batch = kDefaultBatch;
  int32_t last_P = 1;  // pods per round of the last place call (batch, LDS-clamped)
  int32_t last_lag = 1;  // its pipeline depth
  int32_t monotone = 1;
  int32_t score_bits = 16;  // bits of (max total score + 1)
  int32_t nbins = 2;        // score histogram bins of k_select: max total score + 2
  int32_t partial_r = 2;    // nodes per lane of k_scan (tuning knob KOORDHIP_TOPK_R)
  int32_t scan_ppw = 0;     // pods per node-major scan wave: 0 = pod-major k_scan, -1 auto (KOORDHIP_SCAN_PPW)

  std::vector<void *> cols;  // every device column allocation
  kh::DevNodes d{};
  kh::PrepIn prep{};

  // stream buffers
  kh::DevPod *d_pods = nullptr;
  int32_t pods_cap = 0, n_staged = 0;
  int32_t *d_out = nullptr;
  uint64_t *d_cpus = nullptr;  // [pods_cap][KOORDHIP_NUMA_WORDS] cpusets of the last place call (NUMA)
  int32_t out_cap = 0;
  bool numa = false;           // NodeNUMAResource enabled (Filter or Score)
  bool resv = false;           // Reservation enabled (Filter or Score)
  bool side = false;           // the kernels keep NUMA side rows (NodeNUMAResource or Reservation)
  int32_t n_classes = 0;
  kh::DevNumaClass *d_classes = nullptr;
  int32_t *d_rc = nullptr;     // k_commit status
  // per evaluation stream (rounds alternate between two): score matrix of
  // k_scan (u16 [pods][stride]), k_select_split slice lists ([pods][G][k]) and
  // arrival counters (zero between launches)
  uint64_t *d_partial[2] = {nullptr, nullptr};
  uint64_t *d_selpart[2] = {nullptr, nullptr};
  uint32_t *d_selcnt[2] = {nullptr, nullptr};
  int32_t sel_g = kh::kSelGMax;   // workgroups per pod of k_select_split (KOORDHIP_SEL_G)
  int32_t n_cu = 256;             // device CU count
  uint32_t cu_reserve = 0;        // KOORDHIP_CU_RESERVE: CUs (mask word 0) of the resolve alone, 0 = shared
  bool sel_split = true;          // the list producer counts pods into the pipeline (k_eval_topk / k_select_split);
                                  // false (KOORDHIP_SELECT_ONEWG): k_select + signal kernel
  bool eval_fused = true;         // k_eval_topk (no score matrix); false (KOORDHIP_EVAL_SPLIT): k_scan + select
  // k_eval_topk per evaluation stream: slice lists, their counts, and the
  // per-pod bound / arrival words ([2][kSelMaxPods], zero between launches)
  uint64_t *d_etk_part[2] = {nullptr, nullptr};
  int32_t *d_etk_pcnt[2] = {nullptr, nullptr};
  uint32_t *d_etk_sync[2] = {nullptr, nullptr};
  size_t etk_cap[2] = {0, 0}, etk_ccap[2] = {0, 0};
  int etk_vt[2] = {0, 0};
  size_t partial_cap[2] = {0, 0};
  hipStream_t stream2 = nullptr;  // second evaluation stream (odd rounds) of a single-GPU place call
  hipEvent_t ev_eval2 = nullptr;
  uint64_t *d_lists = nullptr;   // [2][batch][k] (rank-local lists; double buffer: round parity)
  uint64_t *d_gather = nullptr;  // [2 streams][world][batch][k]
  int32_t gather_world = 1;
  uint64_t *d_final = nullptr;   // [4][batch][k] (merged lists, multi-rank; indexed like d_lists)
  int32_t *d_mod = nullptr;      // {count, nodes} M' between resolve launches, then PipeSync
  kh::DevNodes *d_desc = nullptr;  // device copy of d (column pointers) for k_resolve
  kh::DevNodes desc_host{};        // its host source (stable while the copy is in flight)
  const uint64_t *d_cur_lists = nullptr;  // this round's rank-local lists (local-group exchange)
  hipStream_t rstream = nullptr;  // resolve stream (the eval kernels use `stream`)
  hipEvent_t ev_res[kRing] = {}, ev_start = nullptr;
  bool pipe_check = false;       // a place call ran: check PipeSync.err when it completes
  bool pipe_err = false;         // ... and it had stalled (sticky until the next place call)
  int32_t pipe_errc = 0;         // ... PipeSync.err's code (0: the sequential cycle's timeout)
  kh::DevPod *d_tmp_pod = nullptr;
  kh::DevPodX *d_tmp_podx = nullptr;  // koordhip_commit_ext's record
  void *d_upd = nullptr;           // koordhip_update_nodes staging (grown, kept)
  size_t upd_cap = 0;
  std::vector<uint8_t> upd_host;   // its host image
  uint64_t *d_dbg = nullptr;  // KOORDHIP_STAMPS diagnostic counters (resolve segments)

  // checkpoint of the mutable columns
  std::vector<void *> ckpt;
  std::vector<kh::DevNumaClass> host_classes;  // the loaded topology classes (host copy)

  // sharding
  ncclComm_t comm = nullptr;
  ncclComm_t comm2 = nullptr;              // split of `comm` for the second evaluation stream's rounds
  std::shared_ptr<LocalGroup> group;       // koordhip_comm_init_local
  hipEvent_t ev_part = nullptr, ev_copy = nullptr;
  int32_t world = 1, rank = 0;

  // stats
  std::vector<hipEvent_t> ev;  // pairs around stream launches (profile_kernels)
  std::vector<int8_t> ev_kind; // per pair: TK_SCAN / TK_SELECT / TK_RESOLVE
  hipEvent_t t0 = nullptr, t1 = nullptr;
  int32_t ev_used = 0;
  double last_eval_ms = 0, last_total_ms = 0;
  std::string eval_kernel, resolve_kernel;  // template instantiations of the last place call's launches
  // the exact sequential cycle (normalized-score plugins: seq.hip)
  bool seq = false;                // the sequential cycle runs the placements (seq_profile, or a Reservation
                                   // snapshot with NUMA topology-policy nodes)
  bool seq_profile = false;        // the profile enables DeviceShare or a normalized upstream Score
  bool seq_ext_only = false;       // ... and its such plugins read only koordhip_pod_ext (DeviceShare,
                                   // PodTopologySpread, InterPodAffinity): a batch whose records are all empty
                                   // (no device / extended-scalar request, no spread constraint or counted
                                   // match, no affinity term or count entry) couples no nodes and runs pipelined
  bool resv_x = false;             // a device-holding reservation lists extended scalars (ABI 14 resv_xalloc)
  bool seq_snap = false;           // the snapshot needs the sequential cycle (Reservation + topology-policy
                                   // nodes, or more than KOORDHIP_RESV_SLOTS reservations on a node)
  bool last_seq = false;           // the last place call ran the sequential cycle
  kh::DevPodX *d_podx = nullptr;   // staged koordhip_pod_ext records (NULL: none staged)
  int32_t podx_cap = 0;
  bool podx_staged = false;
  bool staged_qos_nonbind = false;  // a staged pod KOORDHIP_POD_CPUSET_QOS rejects on some snapshots
  bool staged_dsr = false;          // the staged device pods carry kh::KH_POD_DEVSHARE (reservations were loaded)
  bool staged_reserve = false;     // the staged batch holds a reserve pod (KOORDHIP_POD_RESERVE): the sequential cycle
  bool staged_ext = false;         // the staged batch's koordhip_pod_ext records carry requests / constraints
  // device pods inside the pipelined greedy (k_ext_pre / k_ext_final, seq.hip): the
  // staged pods whose records carry content, when that content is device /
  // extended-scalar requests only (no spread constraint or count, no affinity
  // entry); their DevPods carry KH_POD_EXT
  bool staged_ext_dev = false;
  std::vector<int32_t> ext_idx;
  int32_t *d_ext_idx = nullptr;
  int32_t ext_idx_cap = 0;
  void *d_ext_scr = nullptr;        // the device-pod launches' table, arrival counters, pre-evaluation ring
  size_t ext_scr_cap = 0;
  hipStream_t xstream = nullptr;    // their streams (pooled: transient launches, one-workgroup waits):
  hipStream_t xstream2 = nullptr, xstream3 = nullptr;  // the pre-evaluations, the finals (alternating)
  hipEvent_t ev_ext = nullptr, ev_ext2 = nullptr, ev_ext3 = nullptr;
  bool last_ext_pipe = false;       // the last place call placed device pods inside the pipeline
  bool last_local = false;          // ... ran a node-sharded rank on the full table (class lists, no exchange)
  // class-incremental lists (cls.hip): the staged pods' classes (byte-identical
  // device records), the class buffers and the plan of the staged batch
  std::vector<int32_t> pod_cls;    // class of each staged pod
  std::vector<kh::DevPod> cls_rep; // each class's record
  int32_t *d_pod_cls = nullptr;    // [pods_cap]
  kh::DevPod *d_cls_pod = nullptr; // [cls_cap]
  uint64_t *d_cls_buf = nullptr;   // [cls_cap][2][kClsCap]
  kh::ClsMeta *d_cls_meta = nullptr;  // [cls_cap][2]
  int32_t cls_cap = 0, cls_pod_cap = 0, pod_cls_cap = 0;
  void *d_cls_S = nullptr;         // a build's score rows [kClsBuildRows][stride] and chunk maxima
  size_t cls_S_cap = 0;
  bool plan_ok = false;            // the plan below is the staged batch's for (plan_P, plan_lag)
  int32_t plan_P = 0, plan_lag = 0;
  struct ClsBuild {
    int32_t u, er, tb, e0, ne;  // first use round, enqueue round, base round, entries [e0, e0 + ne)
  };
  std::vector<ClsBuild> plan_builds;
  // per class its schedule (the rounds it appears in, bit 31: switch first to
  // build plan_csm[] of the class), concatenated; per build entry the class /
  // slot, the build number and the workgroup switches to wait for
  std::vector<int32_t> plan_coff, plan_csched, plan_csm, plan_ent, plan_bm, plan_bw;
  std::vector<kh::DevPod> plan_bpods;
  int32_t *d_plan = nullptr;        // coff | csched | csm | ent | bm | bw | done[cls] | sw[cls]
  kh::DevPod *d_plan_pods = nullptr;
  size_t plan_cap = 0, plan_pods_cap = 0;
  size_t plan_off[8] = {};          // element offsets of the arrays in d_plan
  uint32_t *d_devout = nullptr;    // [pods][DEV_TYPES] device slots of the last place call
  uint64_t *d_seqg = nullptr;
  void *d_seqdesc = nullptr;  // the sequential cycle's device copies of dc / d
  kh::PtsArgs pts{};          // PodTopologySpread columns (device pointers) and tables' shape
  kh::IpaArgs ipa{};          // InterPodAffinity count entries (device pointers) and their keys
  int64_t ipa_pods_bound = 0; // pods the snapshot's entries can count (for the raw Score's int32 bound)
  int32_t seq_grid = 0;
  int64_t last_launches = 0, last_evals = 0;
  // executed evaluations of the last call: the host-known part (builds, device
  // pods' pre-evaluations) plus the device counters read by kernel_stats
  int64_t last_exec = 0, last_ext_exec = 0;
  const uint32_t *last_evc = nullptr, *last_reev = nullptr;
  int32_t last_plan_us = 0;  // the class-list plan of the staged batch (0: none made)
};

namespace {

template <typename T>
int dev_alloc(koordhip_ctx *c, T **p, size_t count) {
  void *q = nullptr;
  HIP_TRY(hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
  c->cols.push_back(q);
  *p = static_cast<T *>(q);
  return 0;
}

void free_cols(koordhip_ctx *c) {
  for (void *p : c->cols) (void)hipFree(p);
  c->cols.clear();
  c->d = kh::DevNodes{};
  c->prep = kh::PrepIn{};
  c->loaded = false;
  c->n = 0;
}

template <typename T>
int upload(koordhip_ctx *c, T *dst, const T *src, size_t count) {
  if (count == 0) return 0;
  if (src) {
    HIP_TRY(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, c->stream));
  } else {
    HIP_TRY(hipMemsetAsync(dst, 0, count * sizeof(T), c->stream));
  }
  return 0;
}

// Resource quantities live on device as exact f64 (eval.hpp): |v| < 2^45.
constexpr int64_t kExact = 1ll << 45;

bool exact_ok(int64_t v) { return v < kExact && v > -kExact; }

// int64 quantity column -> f64 device column (NULL src -> zeros)
int upload_q(koordhip_ctx *c, double *dst, const int64_t *src, size_t count, const char *what) {
  if (count == 0) return 0;
  if (!src) {
    HIP_TRY(hipMemsetAsync(dst, 0, count * sizeof(double), c->stream));
    return 0;
  }
  std::vector<double> tmp(count);
  for (size_t i = 0; i < count; i++) {
    if (!exact_ok(src[i]))
      return fail(KOORDHIP_EINVAL, std::string(what) + ": quantity magnitude >= 2^45 is outside the engine's exact range");
    tmp[i] = (double)src[i];
  }
  HIP_TRY(hipMemcpyAsync(dst, tmp.data(), count * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

// f64 device column -> int64 host array
int download_q(double *src, int64_t *dst, size_t count) {
  if (count == 0) return 0;
  std::vector<double> tmp(count);
  HIP_TRY(hipMemcpy(tmp.data(), src, count * sizeof(double), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < count; i++) dst[i] = (int64_t)tmp[i];
  return 0;
}

// koordhip_pod (ABI) -> DevPod (device record).  ext (optional, the pods'
// koordhip_pod_ext records) with `devshare` (DeviceShare in the profile): the
// device pods get kh::KH_POD_DEVSHARE.
int to_dev_pods(const koordhip_pod *src, int32_t n, std::vector<kh::DevPod> &out,
                const koordhip_pod_ext *ext = nullptr, bool devshare = false) {
  out.resize(std::max(n, 0));
  for (int32_t j = 0; j < n; j++) {
    const koordhip_pod &p = src[j];
    kh::DevPod &o = out[j];
    std::memset(&o, 0, sizeof(o));
    const int64_t q[] = {p.req[0], p.req[1], p.req[2], p.req[3], p.req[4], p.nz_cpu_m, p.nz_mem, p.est_cpu, p.est_mem};
    for (int64_t v : q)
      if (!exact_ok(v)) return fail(KOORDHIP_EINVAL, "pod quantity magnitude >= 2^45 is outside the engine's exact range");
    for (int r = 0; r < KOORDHIP_NRES; r++) o.req[r] = (double)p.req[r];
    o.nz_cpu_m = (double)p.nz_cpu_m;
    o.nz_mem = (double)p.nz_mem;
    o.est_cpu = (double)p.est_cpu;
    o.est_mem = (double)p.est_mem;
    if (p.flags & (kh::KH_POD_EXT | kh::KH_POD_DEVSHARE))
      return fail(KOORDHIP_EINVAL, "koordhip_pod.flags bits 29-30 are reserved");
    o.flags = p.flags;
    if (devshare && ext && (ext[j].flags & KOORDHIP_PODX_DEVICE)) o.flags |= kh::KH_POD_DEVSHARE;
    o.numa_cpus = p.numa_cpus;
    o.numa_policy = p.numa_policy;
    if (p.static_class < 0 || p.static_class >= KOORDHIP_MAX_STATIC_CLASSES)
      return fail(KOORDHIP_EINVAL, "pod static_class out of range");
    o.sclass = p.static_class;
    o.resv_match = p.resv_match;
  }
  return 0;
}

int validate_soa(const koordhip_node_soa *s) {
  if (!s) return fail(KOORDHIP_EINVAL, "soa is NULL");
  for (int r = 0; r < KOORDHIP_NRES; r++)
    if (!s->alloc[r] || !s->requested[r]) return fail(KOORDHIP_EINVAL, "alloc/requested column missing");
  if (!s->alloc_pods || !s->npods || !s->nz_cpu_m || !s->nz_mem || !s->la_alloc_cpu_m || !s->la_alloc_mem ||
      !s->la_used_cpu_m || !s->la_used_mem || !s->la_flags)
    return fail(KOORDHIP_EINVAL, "required column missing");
  for (int r = 0; r < 2; r++)
    if (!s->laf_used_m[r] || !s->laf_total_m[r] || !s->laf_prod_used_m[r] || !s->laf_thr[r] || !s->laf_prod_thr[r])
      return fail(KOORDHIP_EINVAL, "LoadAware filter column missing");
  return 0;
}

int ensure(koordhip_ctx *c, void **p, size_t *cap, size_t bytes) {
  if (*cap >= bytes && *p) return 0;
  if (*p) HIP_TRY(hipFree(*p));
  *p = nullptr;
  HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 64)));
  *cap = bytes;
  return 0;
}

// profile_kernels: HIP event pairs around the stream's launches, by kernel
enum { TK_SCAN = 0, TK_SELECT = 1, TK_RESOLVE = 2, TK_KINDS = 3 };

int timed_begin(koordhip_ctx *c, int kind, hipStream_t s, int32_t *idx) {
  *idx = -1;
  if (!c->cfg.profile_kernels) return 0;
  if (c->ev_used + 2 > (int32_t)c->ev.size()) {
    for (int i = 0; i < 1024; i++) {
      hipEvent_t e;
      HIP_TRY(hipEventCreate(&e));
      c->ev.push_back(e);
    }
    c->ev_kind.resize(c->ev.size() / 2);
  }
  *idx = c->ev_used;
  c->ev_kind[c->ev_used / 2] = (int8_t)kind;
  c->ev_used += 2;
  HIP_TRY(hipEventRecord(c->ev[*idx], s));
  return 0;
}
int timed_end(koordhip_ctx *c, int32_t idx, hipStream_t s) {
  if (idx >= 0) HIP_TRY(hipEventRecord(c->ev[idx + 1], s));
  return 0;
}

// The evaluation buffers of one stream slot, sized for np pods over [lo, hi):
// the score matrix + chunk maxima, the split select's slice lists and arrival
// counters.  place_staged sizes them before it launches the persistent
// resolve: an allocation (or a free) inside the round loop could wait for a
// device that is busy with that resolve.
int eval_buffers(koordhip_ctx *c, int32_t np, int32_t lo, int32_t hi, int slot, hipStream_t es,
                 int32_t kmax = kh::kResolveMaxK) {
  if (c->eval_fused) {
    // the slice width is fixed here for every launch until the next call (a
    // shorter last round must not pick narrower slices: more of them than the
    // buffers hold)
    const int vt = kh::eval_topk_vt(kh::side_mode(c->dc), c->n_cu, np, lo, hi, kmax);
    c->etk_vt[slot] = vt;
    const size_t ns = (size_t)std::max(1, kh::eval_topk_slices(vt, lo, hi));
    const size_t pods = (size_t)std::max(np, 1);
    if (int e = ensure(c, reinterpret_cast<void **>(&c->d_etk_part[slot]), &c->etk_cap[slot],
                       pods * ns * kh::kResolveMaxK * sizeof(uint64_t)))
      return e;
    if (int e = ensure(c, reinterpret_cast<void **>(&c->d_etk_pcnt[slot]), &c->etk_ccap[slot], pods * ns * sizeof(int32_t)))
      return e;
    if (!c->d_etk_sync[slot]) {
      HIP_TRY(hipMalloc(&c->d_etk_sync[slot], 2 * kh::kSelMaxPods * sizeof(uint32_t)));
      HIP_TRY(hipMemsetAsync(c->d_etk_sync[slot], 0, 2 * kh::kSelMaxPods * sizeof(uint32_t), es));
    }
    return 0;
  }
  const int64_t stride = ((int64_t)(hi - lo) + 63) & ~63ll;
  const int32_t nchunks = kh::scan_chunks(c->partial_r, lo, hi);
  const int32_t mstride = (nchunks + 63) & ~63;
  const size_t need = (size_t)np * stride * sizeof(uint16_t) + (size_t)np * mstride * sizeof(uint16_t) + 64;
  if (int e = ensure(c, reinterpret_cast<void **>(&c->d_partial[slot]), &c->partial_cap[slot], need)) return e;
  if (c->sel_split && !c->d_selcnt[slot]) {
    HIP_TRY(hipMalloc(&c->d_selpart[slot], kh::kSelPartKeys * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&c->d_selcnt[slot], kh::kSelMaxPods * sizeof(uint32_t)));
    HIP_TRY(hipMemsetAsync(c->d_selcnt[slot], 0, kh::kSelMaxPods * sizeof(uint32_t), es));
  }
  return 0;
}

// Exact per-pod top-k over node range [lo, hi) of np pods: k_scan fills the
// score matrix, k_select reduces each row (best first, 0-padded).
int topk_batch(koordhip_ctx *c, const kh::DevPod *d_pods, int32_t np, int32_t k, int32_t lo, int32_t hi,
               uint64_t *out, bool timed, kh::PipeSync *sync, int32_t sel_par, int32_t res_wait, hipStream_t es,
               int slot) {
  if (c->eval_fused) {
    // buffers sized by eval_buffers before the call's first launch
    const int vt = c->etk_vt[slot];
    if (!vt || kh::eval_topk_slices(vt, lo, hi) * (size_t)np * kh::kResolveMaxK * sizeof(uint64_t) > c->etk_cap[slot])
      return fail(KOORDHIP_EINVAL, "k_eval_topk buffers not sized for this launch");
    int32_t tm = -1;
    if (timed)
      if (int e = timed_begin(c, TK_SCAN, es, &tm)) return e;
    uint32_t *w = c->d_etk_sync[slot];
    HIP_TRY(kh::launch_eval_topk(c->dc, c->d, d_pods, np, lo, hi, k, vt, c->d_etk_part[slot], c->d_etk_pcnt[slot],
                                 w + kh::kSelMaxPods, out, sync, sel_par, res_wait, c->d_dbg, es));
    c->eval_kernel = kh::last_eval_kernel();
    if (int e = timed_end(c, tm, es)) return e;
    c->last_launches++;
    c->last_evals += (int64_t)np * (hi - lo);
    return 0;
  }
  const int R = c->partial_r;
  const int64_t stride = ((int64_t)(hi - lo) + 63) & ~63ll;
  const int32_t nchunks = kh::scan_chunks(R, lo, hi);
  const int32_t mstride = (nchunks + 63) & ~63;
  const size_t sbytes = (size_t)np * stride * sizeof(uint16_t);
  if (int e = eval_buffers(c, np, lo, hi, slot, es)) return e;
  uint16_t *S = reinterpret_cast<uint16_t *>(c->d_partial[slot]);
  uint16_t *Mx = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(c->d_partial[slot]) + sbytes);
  int32_t tm = -1;
  if (timed)
    if (int e = timed_begin(c, TK_SCAN, es, &tm)) return e;
  const int32_t ppw = c->scan_ppw < 0 ? kh::scan_ppw(R, lo, hi, np) : c->scan_ppw;
  HIP_TRY(kh::launch_scan(R, c->dc, c->d, d_pods, np, lo, hi, S, stride, Mx, mstride, ppw, es));
  c->eval_kernel = kh::last_eval_kernel();
  if (int e = timed_end(c, tm, es)) return e;
  c->last_launches++;
  c->last_evals += (int64_t)np * (hi - lo);
  if (!c->sel_split) {
    HIP_TRY(kh::launch_select(S, stride, lo, hi - lo, np, k, c->nbins, Mx, mstride, nchunks, out, c->d_dbg, es));
    return 0;
  }
  if (timed)
    if (int e = timed_begin(c, TK_SELECT, es, &tm)) return e;
  HIP_TRY(kh::launch_select_split(S, stride, lo, hi - lo, np, k, c->nbins, Mx, mstride, nchunks, c->sel_g,
                                  c->d_selpart[slot], c->d_selcnt[slot], out, sync, sel_par, res_wait, es));
  if (int e = timed_end(c, tm, es)) return e;
  return 0;
}

// NodeNUMAResource topology classes -> device tables (numa.hpp DevNumaClass).
int build_numa_class(const koordhip_numa_class &t, kh::DevNumaClass &o) {
  std::memset(&o, 0, sizeof(o));
  if (t.num_cpus <= 0 || t.num_cpus > KOORDHIP_NUMA_MAX_CPUS || t.num_cores <= 0 || t.num_nodes <= 0 ||
      t.num_sockets <= 0)
    return fail(KOORDHIP_EINVAL, "invalid NUMA topology class");
  const int cpc = t.num_cpus / t.num_cores;
  if (cpc != t.cpus_per_core || (cpc != 1 && cpc != 2) || cpc * t.num_cores != t.num_cpus)
    return fail(KOORDHIP_EINVAL, "NUMA topology class: cpus_per_core must be 1 or 2 with uniform cores");
  o.ncpu = t.num_cpus;
  o.cpc = cpc;
  o.cpn = t.num_cpus / t.num_nodes;
  o.cps = t.num_cpus / t.num_sockets;
  int nn = 0, ns = 0;
  for (int p = 0; p < t.num_cpus; p++) {
    const int k = t.node_of[p], sck = t.socket_of[p];
    if (k >= KOORDHIP_NUMA_MAX_NODES || sck >= KOORDHIP_NUMA_MAX_NODES)
      return fail(KOORDHIP_EINVAL, "NUMA topology class: more than 8 NUMA nodes / sockets");
    if (p % cpc != 0 && (t.node_of[p - 1] != k || t.socket_of[p - 1] != sck))
      return fail(KOORDHIP_EINVAL, "NUMA topology class: a core spans NUMA nodes");
    // the resolve's lane-parallel spread take relies on it (numa.hpp acc_take_spread_by_id)
    if (p % cpc != 0 && t.cpu_id[p - 1] >= t.cpu_id[p])
      return fail(KOORDHIP_EINVAL, "NUMA topology class: positions inside a core must ascend by CPU id");
    nn = std::max(nn, k + 1);
    ns = std::max(ns, sck + 1);
    o.nm[k][p >> 6] |= 1ull << (p & 63);
    o.sm[sck][p >> 6] |= 1ull << (p & 63);
    o.sock_of_node[k] = (uint8_t)sck;
  }
  o.nnuma = nn;
  o.nsock = ns;
  std::vector<int> order(t.num_cpus);
  for (int p = 0; p < t.num_cpus; p++) order[p] = p;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return t.cpu_id[a] < t.cpu_id[b]; });
  for (int i = 0; i < t.num_cpus; i++) o.pos_by_id[i] = (uint8_t)order[i];
  return 0;
}

// CPU amplification ratios: finite, >= 0; > 1 is supported only on nodes
// without a NUMA topology policy (zone amplification is not modelled)
int check_amp(const double *amp, const uint8_t *flags, int32_t m, bool *any) {
  for (int32_t i = 0; i < m; i++) {
    const double v = amp[i];
    if (!std::isfinite(v) || v < 0.0) return fail(KOORDHIP_EINVAL, "numa_amp_cpu: ratio must be finite and >= 0");
    if (v > 1.0) {
      *any = true;
      if (flags && KOORDHIP_NODE_NUMA_POLICY(flags[i]))
        return fail(KOORDHIP_EINVAL, "CPU amplification on a node with a NUMA topology policy is not supported");
    }
  }
  return 0;
}

// NUMA zone rows [m][2][KOORDHIP_NUMA_MAX_NODES] int64 -> the device's
// [m][2][KOORDHIP_NUMA_MAX_ZONES] f64; rows of topology-policy nodes are
// checked (<= KOORDHIP_NUMA_MAX_ZONES NUMA nodes, exact quantities)
int zone_rows(const int64_t *src, const int32_t *cls_of, const uint8_t *flags, const kh::DevNumaClass *cls, int32_t m,
              std::vector<double> &out, bool *any_policy) {
  constexpr int Z = KOORDHIP_NUMA_MAX_ZONES, NM = KOORDHIP_NUMA_MAX_NODES;
  out.assign((size_t)m * 2 * Z, 0.0);
  for (int32_t i = 0; i < m; i++) {
    if (!KOORDHIP_NODE_NUMA_POLICY(flags[i])) continue;
    *any_policy = true;
    if (!src) return fail(KOORDHIP_EINVAL, "a node has a NUMA topology policy but numa_zone_alloc / numa_zone_used are NULL");
    if (cls_of[i] >= 0 && cls[cls_of[i]].nnuma > Z)
      return fail(KOORDHIP_EINVAL, "a node with a NUMA topology policy has more NUMA nodes than KOORDHIP_NUMA_MAX_ZONES");
    for (int q = 0; q < 2; q++)
      for (int k = 0; k < NM; k++) {
        const int64_t v = src[((size_t)i * 2 + q) * NM + k];
        if (!exact_ok(v)) return fail(KOORDHIP_EINVAL, "numa zone: quantity magnitude >= 2^45 is outside the engine's exact range");
        if (k >= Z) {
          if (v != 0) return fail(KOORDHIP_EINVAL, "numa zone: values past the node's NUMA nodes must be 0");
          continue;
        }
        out[((size_t)i * 2 + q) * Z + k] = (double)v;
      }
  }
  return 0;
}

int load_numa_columns(koordhip_ctx *c, const koordhip_node_soa *s, int32_t n) {
  kh::DevNuma &nu = c->d.nu;
  nu = kh::DevNuma{};
  if (c->d_classes) {
    (void)hipFree(c->d_classes);
    c->d_classes = nullptr;
  }
  if (!c->side) return 0;
  const bool have = s->numa_class != nullptr;
  if (have && s->n_numa_classes > 0 && !s->numa_classes) return fail(KOORDHIP_EINVAL, "numa_classes is NULL");
  if (have)
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
      if (!s->numa_free[w] || !s->numa_excl_pcpu[w] || !s->numa_excl_numa[w])
        return fail(KOORDHIP_EINVAL, "NUMA mask column missing");
  if (have && (!s->numa_alloc_cnt || !s->numa_flags)) return fail(KOORDHIP_EINVAL, "NUMA column missing");
  std::vector<kh::DevNumaClass> cls(std::max(1, have ? s->n_numa_classes : 0));
  for (int q = 0; have && q < s->n_numa_classes; q++)
    if (int e = build_numa_class(s->numa_classes[q], cls[q])) return e;
  if (have)
    for (int32_t i = 0; i < n; i++)
      if (s->numa_class[i] >= s->n_numa_classes) return fail(KOORDHIP_EINVAL, "numa_class index out of range");
  c->n_classes = have ? s->n_numa_classes : 0;
  HIP_TRY(hipMalloc(&c->d_classes, cls.size() * sizeof(kh::DevNumaClass)));
  HIP_TRY(hipMemcpyAsync(c->d_classes, cls.data(), cls.size() * sizeof(kh::DevNumaClass), hipMemcpyHostToDevice,
                         c->stream));
  nu.cls = c->d_classes;
  nu.ncls = c->n_classes;
  int e = 0;
  int32_t *nc = nullptr, *cnt = nullptr;
  uint8_t *nf = nullptr;
  e = dev_alloc(c, &nc, n);
  if (!e) {
    if (have) {
      e = upload(c, nc, s->numa_class, n);
    } else if (n) {
      std::vector<int32_t> none(n, -1);  // no NodeResourceTopology anywhere
      HIP_TRY(hipMemcpyAsync(nc, none.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
    }
  }
  if (!e) e = dev_alloc(c, &cnt, n);
  if (!e) e = upload(c, cnt, have ? s->numa_alloc_cnt : nullptr, n);
  if (!e) e = dev_alloc(c, &nf, n);
  if (!e) e = upload(c, nf, have ? s->numa_flags : nullptr, n);
  for (int w = 0; w < KOORDHIP_NUMA_WORDS && !e; w++) {
    uint64_t *a = nullptr, *b = nullptr, *d = nullptr;
    e = dev_alloc(c, &a, n);
    if (!e) e = upload(c, a, have ? s->numa_free[w] : nullptr, n);
    if (!e) e = dev_alloc(c, &b, n);
    if (!e) e = upload(c, b, have ? s->numa_excl_pcpu[w] : nullptr, n);
    if (!e) e = dev_alloc(c, &d, n);
    if (!e) e = upload(c, d, have ? s->numa_excl_numa[w] : nullptr, n);
    nu.fr[w] = a;
    nu.ep[w] = b;
    nu.en[w] = d;
  }
  nu.node_cls = nc;
  nu.cnt = cnt;
  nu.nflags = nf;
  // NUMA zones: kept when the snapshot carries the columns (a later
  // update_nodes may give a node a topology policy); zones mode once any
  // node has a policy
  bool any = false;
  c->dc.zones = 0;
  if (!e && have) {
    std::vector<double> za, zu;
    e = zone_rows(s->numa_zone_alloc, s->numa_class, s->numa_flags, cls.data(), n, za, &any);
    if (!e) e = zone_rows(s->numa_zone_used, s->numa_class, s->numa_flags, cls.data(), n, zu, &any);
    if (!e && s->numa_zone_alloc && s->numa_zone_used) {
      // rows of nodes without a policy are never read: converted as zeros
      double *a = nullptr, *u = nullptr;
      e = dev_alloc(c, &a, (size_t)n * 2 * KOORDHIP_NUMA_MAX_ZONES);
      if (!e) e = dev_alloc(c, &u, (size_t)n * 2 * KOORDHIP_NUMA_MAX_ZONES);
      if (!e) e = upload(c, a, za.data(), za.size());
      if (!e) e = upload(c, u, zu.data(), zu.size());
      if (!e) HIP_TRY(hipStreamSynchronize(c->stream));
      nu.za = a;
      nu.zu = u;
    }
    c->dc.zones = any ? 1 : 0;
  }
  // CPU amplification ratios (kept whenever the snapshot carries the column)
  c->dc.amp = 0;
  if (!e && have && s->numa_amp_cpu) {
    bool any_amp = false;
    e = check_amp(s->numa_amp_cpu, s->numa_flags, n, &any_amp);
    double *a = nullptr;
    if (!e) e = dev_alloc(c, &a, (size_t)n);
    if (!e) e = upload(c, a, s->numa_amp_cpu, (size_t)n);
    if (!e) HIP_TRY(hipStreamSynchronize(c->stream));
    nu.amp = a;
    c->dc.amp = any_amp ? 1 : 0;
  }
  c->host_classes = cls;
  return e;
}

// Reservation columns (resv_slots Available reservations per node, slot-major):
// validated, then uploaded; without them (or with the plugin off) the device
// sees none.  m: the column length (slots x rows).
int check_resv_rows(const koordhip_node_soa *s, int32_t m) {
  for (int k = 0; k < 2; k++)
    if (!s->resv_alloc[k] || !s->resv_nz[k] || !s->resv_allocated[k]) return fail(KOORDHIP_EINVAL, "reservation column missing");
  if (!s->resv_order_rank || !s->resv_assigned) return fail(KOORDHIP_EINVAL, "reservation column missing");
  for (int32_t i = 0; i < m; i++) {
    const uint32_t f = s->resv_flags[i];
    if (!(f & KOORDHIP_RESV_PRESENT)) continue;
    if (KOORDHIP_RESV_POLICY(f) > 2) return fail(KOORDHIP_EINVAL, "resv_flags: unknown allocate policy");
    if ((f & KOORDHIP_RESV_ORDERED) && (s->resv_order_rank[i] < 0 || s->resv_order_rank[i] >= KOORDHIP_RESV_MAX_ORDERS))
      return fail(KOORDHIP_EINVAL, "resv_order_rank out of [0, KOORDHIP_RESV_MAX_ORDERS)");
    if (s->resv_assigned[i] < 0) return fail(KOORDHIP_EINVAL, "resv_assigned < 0");
    for (int k = 0; k < 2; k++)
      if (s->resv_alloc[k][i] < 0 || s->resv_allocated[k][i] < 0 || s->resv_nz[k][i] < 0 || !exact_ok(s->resv_alloc[k][i]) ||
          !exact_ok(s->resv_allocated[k][i]) || !exact_ok(s->resv_nz[k][i]))
        return fail(KOORDHIP_EINVAL, "reservation quantity out of range");
  }
  return 0;
}

// reserved CPUs: only on present slots of nodes with a CPU topology and no
// NUMA topology policy, inside the topology's positions, and allocated (not
// free: the reservation's own allocation holds them)
int check_resv_cpus(const koordhip_node_soa *s, int32_t m, int32_t slots, const std::vector<int32_t> &class_cpus) {
  const int32_t nclasses = (int32_t)class_cpus.size();
  for (int32_t q = 0; q < slots; q++)
    for (int32_t i = 0; i < m; i++) {
      const size_t at = (size_t)q * (size_t)m + (size_t)i;
      uint64_t any = 0;
      for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) any |= s->resv_cpus[w][at];
      if (!any) continue;
      if (!(s->resv_flags[at] & KOORDHIP_RESV_PRESENT))
        return fail(KOORDHIP_EINVAL, "resv_cpus on an empty reservation slot");
      const int32_t cls = s->numa_class ? s->numa_class[i] : -1;
      if (cls < 0 || cls >= nclasses) return fail(KOORDHIP_EINVAL, "resv_cpus on a node without a CPU topology");
      const int32_t ncpu = class_cpus[cls];
      for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
        const uint64_t x = s->resv_cpus[w][at];
        const int32_t lo = 64 * w;
        const uint64_t valid = ncpu >= lo + 64 ? ~0ull : (ncpu <= lo ? 0ull : ((1ull << (ncpu - lo)) - 1));
        if (x & ~valid) return fail(KOORDHIP_EINVAL, "resv_cpus outside the node's CPU positions");
        if (s->numa_free[w] && (x & s->numa_free[w][i]))
          return fail(KOORDHIP_EINVAL, "resv_cpus must be allocated CPUs (the reservation holds them), not free ones");
      }
    }
  return 0;
}

int load_resv_columns(koordhip_ctx *c, const koordhip_node_soa *s, int32_t n) {
  c->d.rv = kh::DevResv{};
  c->dc.resv = 0;
  c->dc.resv_slots = 1;
  if (!c->resv) return 0;
  if (s->resv_slots < 0 || s->resv_slots > KOORDHIP_RESV_SLOTS_MAX)
    return fail(KOORDHIP_EINVAL, "resv_slots out of [0, KOORDHIP_RESV_SLOTS_MAX]");
  // a snapshot without reservation columns gets zero columns: the Reservation
  // build (NM 3) still runs the plugin, e.g. a pod with a required reservation
  // affinity fails its Filter on every node (plugin.go:378-381)
  std::vector<uint32_t> zf;
  std::vector<int32_t> zi;
  std::vector<int64_t> zq;
  koordhip_node_soa zs;
  if (!s->resv_flags) {
    zf.assign(std::max(n, 1), 0u);
    zi.assign(std::max(n, 1), 0);
    zq.assign(std::max(n, 1), 0);
    zs = *s;
    zs.resv_flags = zf.data();
    zs.resv_order_rank = zi.data();
    zs.resv_assigned = zi.data();
    for (int k = 0; k < 2; k++) zs.resv_alloc[k] = zs.resv_nz[k] = zs.resv_allocated[k] = zq.data();
    s = &zs;
  }
  const int32_t slots = std::max(1, s->resv_slots);
  const int32_t sn = slots * n;  // slot-major columns
  if (int e = check_resv_rows(s, sn)) return e;
  kh::DevResv &rv = c->d.rv;
  uint32_t *f = nullptr;
  int32_t *rk = nullptr, *rn = nullptr;
  int e = dev_alloc(c, &f, sn);
  if (!e) e = upload(c, f, s->resv_flags, sn);
  if (!e) e = dev_alloc(c, &rk, sn);
  if (!e) e = upload(c, rk, s->resv_order_rank, sn);
  if (!e) e = dev_alloc(c, &rn, sn);
  if (!e) e = upload(c, rn, s->resv_assigned, sn);
  for (int k = 0; k < 2 && !e; k++) {
    double *a = nullptr, *z = nullptr, *d = nullptr;
    e = dev_alloc(c, &a, sn);
    if (!e) e = upload_q(c, a, s->resv_alloc[k], sn, "resv_alloc");
    if (!e) e = dev_alloc(c, &z, sn);
    if (!e) e = upload_q(c, z, s->resv_nz[k], sn, "resv_nz");
    if (!e) e = dev_alloc(c, &d, sn);
    if (!e) e = upload_q(c, d, s->resv_allocated[k], sn, "resv_allocated");
    rv.ra[k] = a;
    rv.rz[k] = z;
    rv.rd[k] = d;
  }
  // the reserved CPUs left per slot (NodeNUMAResource RestoreReservation)
  c->dc.resv_cpus = 0;
  if (!e && s->resv_cpus[0] && c->numa) {  // (without NodeNUMAResource nothing reads them)
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
      if (!s->resv_cpus[w]) e = fail(KOORDHIP_EINVAL, "resv_cpus: every word column or none");
    std::vector<int32_t> ncpu;
    for (int32_t k = 0; k < s->n_numa_classes && s->numa_classes; k++) ncpu.push_back(s->numa_classes[k].num_cpus);
    if (!e) e = check_resv_cpus(s, n, slots, ncpu);
    for (int w = 0; w < KOORDHIP_NUMA_WORDS && !e; w++) {
      uint64_t *m = nullptr;
      e = dev_alloc(c, &m, sn);
      if (!e) e = upload(c, m, s->resv_cpus[w], sn);
      rv.rc[w] = m;
    }
    if (!e) c->dc.resv_cpus = 1;
  }
  rv.flags = f;
  rv.rank = rk;
  rv.rn = rn;
  rv.slots = slots;
  rv.stride = n;
  if (!e) {
    c->dc.resv = 1;
    c->dc.resv_slots = slots;
  }
  return e;
}

// The device-holding reservation columns of a snapshot or of update rows (m
// rows, slot-major reservation columns of stride m): each node's one such
// reservation names an Available slot, holds devices only on the node's minors,
// its allocated only on its own minors; values in [0, 2^45).
int check_resv_dev(const koordhip_node_soa *s, int32_t n) {
  const int32_t S = s->resv_slots > 1 ? s->resv_slots : 1;
  if (!s->resv_flags) return fail(KOORDHIP_EINVAL, "resv_dev without reservation columns");
  const size_t per = (size_t)KOORDHIP_DEV_TYPES * s->dev_slots * KOORDHIP_DEV_RES;
  for (int32_t i = 0; i < n; i++) {
    const int32_t h = s->resv_dev_slot[i];
    if (h < -1 || h >= S) return fail(KOORDHIP_EINVAL, "resv_dev_slot out of [-1, resv_slots)");
    const int64_t *row = s->resv_dev + (size_t)i * 2 * per;
    bool any = false;
    for (size_t a = 0; a < 2 * per; a++) {
      if (row[a] < 0 || row[a] >= (1ll << 45)) return fail(KOORDHIP_EINVAL, "resv_dev out of [0, 2^45)");
      any = any || (a < per && row[a] != 0);
    }
    if (h < 0) {
      for (size_t a = 0; a < 2 * per; a++)
        if (row[a]) return fail(KOORDHIP_EINVAL, "resv_dev values on a node without a device-holding reservation");
      continue;
    }
    if (!(s->resv_flags[(size_t)h * n + i] & KOORDHIP_RESV_PRESENT))
      return fail(KOORDHIP_EINVAL, "resv_dev_slot names an empty reservation slot");
    if (!any) return fail(KOORDHIP_EINVAL, "a device-holding reservation with no devices (use resv_dev_slot -1)");
    // its minors are the node's; its allocated lies on them
    for (int t = 0; t < KOORDHIP_DEV_TYPES; t++)
      for (int32_t q = 0; q < s->dev_slots; q++) {
        const int64_t *A = row + ((size_t)t * s->dev_slots + q) * KOORDHIP_DEV_RES;
        const int64_t *D = A + per;
        const bool a = A[0] || A[1] || A[2], d = D[0] || D[1] || D[2];
        if ((a || d) && s->dev_minor[((size_t)i * KOORDHIP_DEV_TYPES + t) * s->dev_slots + q] < 0)
          return fail(KOORDHIP_EINVAL, "resv_dev on an empty device slot");
        if (d && !a) return fail(KOORDHIP_EINVAL, "resv_dev allocated outside the reservation's minors");
      }
  }
  return 0;
}

// ABI 14: the extended scalars of the device-holding reservations, [NXRES][m]
// rows of a snapshot or of update rows: values in [0, 2^45) (the scorer's
// 100 x quotient stays exact), none on a node without such a reservation.
int check_resv_scalars(const int64_t *xa, const int64_t *xd, const int32_t *slot, int32_t m) {
  for (int j = 0; j < KOORDHIP_NXRES; j++)
    for (int32_t i = 0; i < m; i++) {
      const int64_t a = xa[(size_t)j * m + i], d = xd ? xd[(size_t)j * m + i] : 0;
      if (a < 0 || a >= (1ll << 45) || d < 0 || d >= (1ll << 45))
        return fail(KOORDHIP_EINVAL, "resv_xalloc / resv_xallocated out of [0, 2^45)");
      if ((a || d) && (!slot || slot[i] < 0))
        return fail(KOORDHIP_EINVAL, "resv_xalloc / resv_xallocated on a node without a device-holding reservation");
    }
  return 0;
}

// ABI 9 columns of the sequential cycle: DeviceShare devices, extended
// scalars, static Scores (int64 on device: the device code is integer).
int load_ext_columns(koordhip_ctx *c, const koordhip_node_soa *s, int32_t n) {
  kh::DevDev &dv = c->d.dv;
  dv = kh::DevDev{};
  const bool dev = ((c->cfg.filter_plugins | c->cfg.score_plugins) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  c->resv_x = false;
  if (!c->seq_profile) {
    if (s->dev_slots > 0 || s->xalloc || s->static_score[0] || s->static_score[1] || s->pts_keys > 0 || s->ipa_ents > 0)
      return fail(KOORDHIP_EINVAL, "device / extended-scalar / static-score / topology-spread columns need DeviceShare, "
                                   "PodTopologySpread or a normalized Score plugin in the profile (the sequential cycle)");
    return 0;
  }
  int e = 0;
  if (dev && s->dev_slots > 0) {
    if (s->dev_slots > KOORDHIP_DEV_SLOTS || !s->dev_present || !s->dev_minor || !s->dev_total)
      return fail(KOORDHIP_EINVAL, "dev_slots > KOORDHIP_DEV_SLOTS or a device column missing");
    const size_t ns = (size_t)n * KOORDHIP_DEV_TYPES * s->dev_slots;
    // the scorer's percent quotients (dev.hpp dev_pct_div: an f64 reciprocal and
    // one exact fix-up) equal Go's int64 division only for operands below 2^45
    for (size_t a = 0; a < ns * KOORDHIP_DEV_RES; a++)
      if (s->dev_total[a] < 0 || s->dev_total[a] >= (1ll << 45) ||
          (s->dev_used && (s->dev_used[a] < 0 || s->dev_used[a] >= (1ll << 45))))
        return fail(KOORDHIP_EINVAL, "dev_total / dev_used out of [0, 2^45)");
    // a node holds one GPU model: every GPU with resources has the same memory
    // (fillGPUTotalMem reads the first one, utils.go:211-233)
    for (int32_t i = 0; i < n; i++) {
      int64_t mem = -1;
      for (int32_t q = 0; q < s->dev_slots; q++) {
        const size_t a = ((size_t)i * KOORDHIP_DEV_TYPES + KOORDHIP_DEV_GPU) * s->dev_slots + q;
        if (s->dev_minor[a] < 0) continue;
        const int64_t *t = s->dev_total + a * KOORDHIP_DEV_RES;
        if (t[0] == 0 && t[1] == 0 && t[2] == 0) continue;
        if (t[2] <= 0) return fail(KOORDHIP_EINVAL, "a GPU with resources but no gpu-memory");
        if (mem >= 0 && t[2] != mem) return fail(KOORDHIP_EINVAL, "GPUs of different memory sizes on one node");
        mem = t[2];
      }
    }
    uint8_t *pr = nullptr;
    int32_t *mi = nullptr;
    int64_t *tt = nullptr, *us = nullptr;
    e = dev_alloc(c, &pr, n);
    if (!e) e = upload(c, pr, s->dev_present, n);
    if (!e) e = dev_alloc(c, &mi, ns);
    if (!e) e = upload(c, mi, s->dev_minor, ns);
    if (!e) e = dev_alloc(c, &tt, ns * KOORDHIP_DEV_RES);
    if (!e) e = upload(c, tt, s->dev_total, ns * KOORDHIP_DEV_RES);
    if (!e) e = dev_alloc(c, &us, ns * KOORDHIP_DEV_RES);
    if (!e) e = upload(c, us, s->dev_used, ns * KOORDHIP_DEV_RES);  // NULL: zeros
    dv.slots = s->dev_slots;
    dv.present = pr;
    dv.minor = mi;
    dv.total = tt;
    dv.used = us;
    // DeviceShare's reservation restore (deviceshare/reservation.go:119-170):
    // each node's one reservation holding devices
    if (!e && s->resv_dev_slot && s->resv_dev) {
      if (int ce = check_resv_dev(s, n)) return ce;
      const size_t per = (size_t)KOORDHIP_DEV_TYPES * s->dev_slots * KOORDHIP_DEV_RES;
      int32_t *rs = nullptr;
      int64_t *rd = nullptr;
      e = dev_alloc(c, &rs, n);
      if (!e) e = upload(c, rs, s->resv_dev_slot, n);
      if (!e) e = dev_alloc(c, &rd, (size_t)n * 2 * per);
      if (!e) e = upload(c, rd, s->resv_dev, (size_t)n * 2 * per);
      dv.rslot = rs;
      dv.rdev = rd;
      // ABI 14: that reservation's extended scalars (Allocatable, Allocated)
      if (!e && s->resv_xalloc) {
        if (int xe = check_resv_scalars(s->resv_xalloc, s->resv_xallocated, s->resv_dev_slot, n)) return xe;
        int64_t *xa = nullptr, *xd = nullptr;
        e = dev_alloc(c, &xa, (size_t)n * KOORDHIP_NXRES);
        if (!e) e = upload(c, xa, s->resv_xalloc, (size_t)n * KOORDHIP_NXRES);
        if (!e) e = dev_alloc(c, &xd, (size_t)n * KOORDHIP_NXRES);
        if (!e) e = upload(c, xd, s->resv_xallocated, (size_t)n * KOORDHIP_NXRES);  // NULL: zeros
        dv.rxa = xa;
        dv.rxd = xd;
        for (size_t a = 0; a < (size_t)n * KOORDHIP_NXRES && !c->resv_x; a++) c->resv_x = s->resv_xalloc[a] != 0;
      }
    }
  }
  if (!e && s->resv_xalloc && !dv.rxa)
    return fail(KOORDHIP_EINVAL, "resv_xalloc needs DeviceShare and the device-holding reservation columns "
                                 "(resv_dev_slot, resv_dev)");
  int64_t *xa = nullptr, *xr = nullptr;
  if (!e && s->xalloc) {
    e = dev_alloc(c, &xa, (size_t)n * KOORDHIP_NXRES);
    if (!e) e = upload(c, xa, s->xalloc, (size_t)n * KOORDHIP_NXRES);
  }
  if (!e) e = dev_alloc(c, &xr, (size_t)n * KOORDHIP_NXRES);
  if (!e) e = upload(c, xr, s->xrequested, (size_t)n * KOORDHIP_NXRES);
  dv.xalloc = xa;
  dv.xreq = xr;
  for (int w = 0; w < 2 && !e; w++) {
    const uint32_t bit = w == 0 ? KOORDHIP_PLUGIN_AFFINITY_SCORE : KOORDHIP_PLUGIN_TAINT_SCORE;
    if (!(c->cfg.score_plugins & bit) || !s->static_score[w]) continue;
    uint16_t *ss = nullptr;
    e = dev_alloc(c, &ss, (size_t)n * KOORDHIP_MAX_STATIC_CLASSES);
    if (!e) e = upload(c, ss, s->static_score[w], (size_t)n * KOORDHIP_MAX_STATIC_CLASSES);
    dv.sscore[w] = ss;
  }
  // PodTopologySpread: the keys' domains, the constraint table's counts, the classes' eligibility
  c->pts = kh::PtsArgs{};
  c->ipa = kh::IpaArgs{};
  c->ipa_pods_bound = 0;
  const bool pts = ((c->cfg.filter_plugins | c->cfg.score_plugins) & KOORDHIP_PLUGIN_PTS) != 0;
  const bool ipa = ((c->cfg.filter_plugins | c->cfg.score_plugins) & KOORDHIP_PLUGIN_IPA) != 0;
  // (the topology keys serve both plugins: loaded when either runs)
  if (!e && (pts || ipa) && s->pts_keys > 0) {
    if (s->pts_keys > KOORDHIP_PTS_KEYS || s->pts_cons < 0 || s->pts_cons > KOORDHIP_PTS_CONS || s->pts_classes < 0 ||
        s->pts_classes > KOORDHIP_PTS_CLASSES || !s->pts_dom || !s->pts_elig || (s->pts_cons > 0 && !s->pts_cnt))
      return fail(KOORDHIP_EINVAL, "PodTopologySpread tables outside KOORDHIP_PTS_* or a column missing");
    for (int k = 0; k < s->pts_keys; k++)
      if (!((s->pts_hostname >> k) & 1u) && (s->pts_ndom[k] < 1 || s->pts_ndom[k] > KOORDHIP_PTS_DOMAINS))
        return fail(KOORDHIP_EINVAL, "PodTopologySpread: a non-hostname key needs 1..KOORDHIP_PTS_DOMAINS domains");
    for (int cc = 0; cc < s->pts_cons; cc++)
      if (s->pts_cons_key[cc] < 0 || s->pts_cons_key[cc] >= s->pts_keys)
        return fail(KOORDHIP_EINVAL, "PodTopologySpread: a constraint's key is out of range");
    for (int k = 0; k < s->pts_keys; k++)
      for (int32_t i = 0; i < n; i++) {
        const int32_t v = s->pts_dom[(size_t)k * n + i];
        const int32_t hi = ((s->pts_hostname >> k) & 1u) ? n : s->pts_ndom[k];
        if (v < -1 || v >= hi || (((s->pts_hostname >> k) & 1u) && v >= 0 && v != i))
          return fail(KOORDHIP_EINVAL, "PodTopologySpread: pts_dom out of range (a hostname domain is the node)");
      }
    int32_t *pd = nullptr, *pc = nullptr;
    uint16_t *pe = nullptr;
    e = dev_alloc(c, &pd, (size_t)n * s->pts_keys);
    if (!e) e = upload(c, pd, s->pts_dom, (size_t)n * s->pts_keys);
    if (!e) e = dev_alloc(c, &pc, (size_t)n * std::max(1, s->pts_cons));
    if (!e) e = upload(c, pc, s->pts_cons > 0 ? s->pts_cnt : nullptr, (size_t)n * std::max(1, s->pts_cons));
    if (!e) e = dev_alloc(c, &pe, (size_t)n);
    if (!e) e = upload(c, pe, s->pts_elig, (size_t)n);
    kh::PtsArgs &pa = c->pts;
    pa.dom = pd;
    pa.cnt = pc;
    pa.elig = pe;
    pa.keys = s->pts_keys;
    pa.cons = s->pts_cons;
    pa.classes = s->pts_classes;
    pa.host = s->pts_hostname;
    pa.filt = (c->cfg.filter_plugins & KOORDHIP_PLUGIN_PTS) ? 1 : 0;
    pa.score = (c->cfg.score_plugins & KOORDHIP_PLUGIN_PTS) ? 1 : 0;
    for (int cc = 0; cc < KOORDHIP_PTS_CONS; cc++) pa.cons_key[cc] = cc < s->pts_cons ? s->pts_cons_key[cc] : 0;
  }
  // InterPodAffinity: the count entries over those keys
  if (!e && ipa && s->ipa_ents > 0) {
    if (s->ipa_ents > KOORDHIP_IPA_ENTRIES || !s->ipa_cnt || !c->pts.dom)
      return fail(KOORDHIP_EINVAL, "InterPodAffinity: more than KOORDHIP_IPA_ENTRIES entries, ipa_cnt missing, or no "
                                   "topology keys (pts_keys / pts_dom)");
    for (int q = 0; q < s->ipa_ents; q++)
      if (s->ipa_ent_key[q] < 0 || s->ipa_ent_key[q] >= s->pts_keys)
        return fail(KOORDHIP_EINVAL, "InterPodAffinity: an entry's key is out of range");
    int64_t most = 0;  // the largest entry total: what a count can reach before the stream adds its pods
    for (int q = 0; q < s->ipa_ents; q++) {
      int64_t tot = 0;
      for (int32_t i = 0; i < n; i++) {
        const int32_t v = s->ipa_cnt[(size_t)q * n + i];
        if (v < 0) return fail(KOORDHIP_EINVAL, "InterPodAffinity: a negative ipa_cnt");
        tot += v;
      }
      most = std::max(most, tot);
    }
    c->ipa_pods_bound = most;
    int32_t *ic = nullptr, *sums = nullptr;
    e = dev_alloc(c, &ic, (size_t)n * s->ipa_ents);
    if (!e) e = upload(c, ic, s->ipa_cnt, (size_t)n * s->ipa_ents);
    if (!e) e = dev_alloc(c, &sums, (size_t)kh::IPA_SUMS);
    kh::IpaArgs &ia = c->ipa;
    ia.dom = c->pts.dom;
    ia.cnt = ic;
    ia.sums = sums;
    ia.ents = s->ipa_ents;
    ia.host = s->pts_hostname;
    ia.filt = (c->cfg.filter_plugins & KOORDHIP_PLUGIN_IPA) ? 1 : 0;
    ia.score = (c->cfg.score_plugins & KOORDHIP_PLUGIN_IPA) ? 1 : 0;
    for (int q = 0; q < KOORDHIP_IPA_ENTRIES; q++) ia.ent_key[q] = q < s->ipa_ents ? s->ipa_ent_key[q] : 0;
  }
  c->ipa.w = (c->cfg.score_plugins & KOORDHIP_PLUGIN_IPA) ? c->cfg.ext_weight[4] : 0;
  c->pts.w = (c->cfg.score_plugins & KOORDHIP_PLUGIN_PTS) ? c->cfg.ext_weight[3] : 0;
  // (a profile scoring PodTopologySpread on a snapshot without tables: every
  // node scores 100, as for pods without constraints)
  if (pts && !c->pts.dom) c->pts.score = (c->cfg.score_plugins & KOORDHIP_PLUGIN_PTS) ? 1 : 0;
  return e;
}

int pipe_status(koordhip_ctx *c);

void shard(const koordhip_ctx *c, int32_t *lo, int32_t *hi) {
  *lo = (int32_t)((int64_t)c->n * c->rank / c->world);
  *hi = (int32_t)((int64_t)c->n * (c->rank + 1) / c->world);
  // KOORDHIP_SHARD_SIM=W (timing diagnostics for the multi-GPU estimate, a
  // one-rank communicator only): evaluate shard 0 of W, as rank 0 of a
  // W-GPU job would; the placements then differ from the full table's
  if (c->comm && c->world == 1)
    if (const char *w = std::getenv("KOORDHIP_SHARD_SIM")) {
      static bool warned = false;  // a diagnostic: say so, placements are not the full table's
      if (!warned) {
        std::fprintf(stderr, "[koordhip] KOORDHIP_SHARD_SIM=%s: evaluating shard 0 only (timing diagnostic; "
                             "placements differ from the full table's)\n", w);
        warned = true;
      }
      *hi = (int32_t)((int64_t)c->n / std::max(1, std::atoi(w)));
    }
}

}  // namespace

extern "C" {

const char *koordhip_last_error(void) { return g_err.c_str(); }
int koordhip_abi_version(void) { return KOORDHIP_ABI_VERSION; }

int koordhip_create(const koordhip_config *cfg, koordhip_ctx **out) {
  if (!cfg || !out) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (cfg->abi_version != KOORDHIP_ABI_VERSION) return fail(KOORDHIP_EINVAL, "abi_version mismatch");
  const uint32_t known = KOORDHIP_PLUGIN_FIT | KOORDHIP_PLUGIN_LOADAWARE | KOORDHIP_PLUGIN_NUMA |
                         KOORDHIP_PLUGIN_RESERVATION | KOORDHIP_PLUGIN_NODE_STATIC | KOORDHIP_PLUGIN_BALANCED |
                         KOORDHIP_PLUGIN_DEVICESHARE | KOORDHIP_PLUGIN_AFFINITY_SCORE | KOORDHIP_PLUGIN_TAINT_SCORE |
                         KOORDHIP_PLUGIN_PTS | KOORDHIP_PLUGIN_IPA;
  if ((cfg->filter_plugins | cfg->score_plugins) & ~known) return fail(KOORDHIP_EINVAL, "unknown plugin bit");
  if (cfg->filter_plugins & (KOORDHIP_PLUGIN_AFFINITY_SCORE | KOORDHIP_PLUGIN_TAINT_SCORE))
    return fail(KOORDHIP_EINVAL, "the NodeAffinity / TaintToleration Score bits are Score plugins");
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) {
    static const uint32_t xb[KOORDHIP_NEXT_PLUGINS] = {KOORDHIP_PLUGIN_DEVICESHARE, KOORDHIP_PLUGIN_AFFINITY_SCORE,
                                                       KOORDHIP_PLUGIN_TAINT_SCORE, KOORDHIP_PLUGIN_PTS,
                                                       KOORDHIP_PLUGIN_IPA};
    if ((cfg->score_plugins & xb[e]) && (cfg->ext_weight[e] < 1 || cfg->ext_weight[e] > 100))
      return fail(KOORDHIP_EINVAL, "DeviceShare / NodeAffinity / TaintToleration / PodTopologySpread / "
                                   "InterPodAffinity score weight must be in [1, 100]");
  }
  for (int k = 0; k < 5; k++)
    if (cfg->dev_res_weight[k] < 0 || cfg->dev_res_weight[k] > 100)
      return fail(KOORDHIP_EINVAL, "DeviceShare scoring resource weights must be in [0, 100]");
  if (cfg->score_plugins & KOORDHIP_PLUGIN_NODE_STATIC) return fail(KOORDHIP_EINVAL, "the static node filters have no Score");
  if (cfg->filter_plugins & KOORDHIP_PLUGIN_BALANCED) return fail(KOORDHIP_EINVAL, "BalancedAllocation has no Filter");
  if (cfg->score_plugins & KOORDHIP_PLUGIN_NUMA) {
    if (cfg->numa_weight_cpu < 0 || cfg->numa_weight_cpu > 100 || cfg->numa_weight_mem < 0 || cfg->numa_weight_mem > 100)
      return fail(KOORDHIP_EINVAL, "NodeNUMAResource resource weights must be in [0, 100]");
  }
  for (int p = 0; p < KOORDHIP_NPLUGINS; p++) {
    const uint32_t bit = kScorePluginBit[p];
    if ((cfg->score_plugins & bit) && (cfg->plugin_weight[p] < 1 || cfg->plugin_weight[p] > 100))
      return fail(KOORDHIP_EINVAL, "plugin score weight must be in [1, 100]");
  }
  for (int r = 0; r < KOORDHIP_NRES; r++)
    if (cfg->fit_weight[r] < 0 || cfg->fit_weight[r] > 100) return fail(KOORDHIP_EINVAL, "fit weight out of range");
  if (cfg->score_plugins & KOORDHIP_PLUGIN_LOADAWARE) {
    if (cfg->la_weight_cpu < 0 || cfg->la_weight_cpu > 100 || cfg->la_weight_mem < 0 || cfg->la_weight_mem > 100 ||
        cfg->la_weight_cpu + cfg->la_weight_mem == 0)
      return fail(KOORDHIP_EINVAL, "LoadAware resource weights must be in [1, 100]");
  }
  if (cfg->batch_pods < 0 || cfg->batch_pods > kMaxBatch) return fail(KOORDHIP_EINVAL, "batch_pods must be in [0, 64]");
  auto *c = new koordhip_ctx();
  c->cfg = *cfg;
  // evaluation path: k_eval_topk (fused, no score matrix) for the NUMA /
  // Reservation plugin sets, whose heavier rows make the split path's matrix
  // round trip the longer chain (config 5: 177k -> 207k pods/s); k_scan +
  // k_select_split for the plain Fit + LoadAware set, where the fused
  // launch's 24x column re-reads from L2 cost more than the u16 matrix
  // (config 4: 43 vs 39.5 us per round).  KOORDHIP_EVAL=fused|split forces one.
  {
    const uint32_t pl = cfg->filter_plugins | cfg->score_plugins;
    c->eval_fused = (pl & (KOORDHIP_PLUGIN_NUMA | KOORDHIP_PLUGIN_RESERVATION)) != 0;
    if (const char *ev = std::getenv("KOORDHIP_EVAL")) c->eval_fused = std::strcmp(ev, "split") != 0;
    if (std::getenv("KOORDHIP_EVAL_SPLIT") || std::getenv("KOORDHIP_SELECT_ONEWG")) c->eval_fused = false;
  }
  // NodeNUMAResource streams are bound by the resolve's cpuset Reserve: shorter
  // rounds re-evaluate fewer stale list entries (config 3: 16 pods 106k, 32 pods 98k pods/s)
  const uint32_t plugins = cfg->filter_plugins | cfg->score_plugins;
  c->batch = cfg->batch_pods ? cfg->batch_pods
                             : ((plugins & KOORDHIP_PLUGIN_RESERVATION) ? kDefaultBatchResv
                                : (plugins & KOORDHIP_PLUGIN_NUMA)     ? kDefaultBatchNuma
                                                                       : kDefaultBatch);
  c->dc.filt = cfg->filter_plugins;
  c->dc.score = cfg->score_plugins;
  c->dc.w_fit = (int32_t)cfg->plugin_weight[0];
  c->dc.w_la = (int32_t)cfg->plugin_weight[1];
  c->dc.w_numa = (int32_t)cfg->plugin_weight[2];
  c->dc.w_bal = (int32_t)cfg->plugin_weight[3];
  for (int r = 0; r < KOORDHIP_NRES; r++) c->dc.fit_w[r] = (int32_t)cfg->fit_weight[r];
  c->dc.la_w_cpu = (int32_t)cfg->la_weight_cpu;
  c->dc.la_w_mem = (int32_t)cfg->la_weight_mem;
  c->dc.according = cfg->la_score_according_prod_usage ? 1 : 0;
  c->dc.numa_w_cpu = cfg->numa_weight_cpu;
  c->dc.numa_w_mem = cfg->numa_weight_mem;
  c->dc.numa_most = cfg->numa_most_allocated ? 1 : 0;
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) c->dc.w_ext[e] = cfg->ext_weight[e];
  c->dc.dev_most = cfg->dev_most_allocated ? 1 : 0;
  for (int k = 0; k < 5; k++) c->dc.dev_w[k] = cfg->dev_res_weight[k];
  // normalized scores couple a pod's nodes: the exact sequential cycle
  c->seq = ((cfg->filter_plugins | cfg->score_plugins) &
            (KOORDHIP_PLUGIN_DEVICESHARE | KOORDHIP_PLUGIN_PTS | KOORDHIP_PLUGIN_IPA)) ||
           (cfg->score_plugins & (KOORDHIP_PLUGIN_AFFINITY_SCORE | KOORDHIP_PLUGIN_TAINT_SCORE));
  c->seq_profile = c->seq;
  c->seq_ext_only = c->seq_profile && !(cfg->score_plugins & (KOORDHIP_PLUGIN_AFFINITY_SCORE | KOORDHIP_PLUGIN_TAINT_SCORE));
  c->numa = ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_NUMA) != 0;
  c->resv = ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_RESERVATION) != 0;
  c->side = c->numa || c->resv;
  // 4 nodes per lane: Reservation builds (config 5 scan 195 -> 170 us per launch, 143k -> 150k pods/s) and,
  // since round 3's resolve, the plain set too (config 4 with 6 select workgroups per pod: 1.117M -> 1.157M
  // pods/s, profiles/r03_ab/sweep4.txt); the NUMA-only scan stays at 2
  c->partial_r = (c->resv || !c->numa) ? 4 : 2;
  if (const char *r = std::getenv("KOORDHIP_TOPK_R")) {
    const int v = std::atoi(r);
    if (v == 1 || v == 2 || v == 4 || v == 8) c->partial_r = v;
  }
  if (c->side && c->partial_r > 4) c->partial_r = 4;  // the NUMA / Reservation scan kernels are built for R <= 4
  // node-major scan (k_scan_nm) group size, "auto" = ~2 waves per SIMD; the
  // pod-major k_scan stays the default (node-major measured equal on config 4
  // and slower on config 5: DESIGN.md §5)
  if (const char *q = std::getenv("KOORDHIP_SCAN_PPW"))
    c->scan_ppw = std::strcmp(q, "auto") == 0 ? -1 : std::max(0, std::min(kMaxBatch, std::atoi(q)));
  // the split select shortens the evaluation stream (and drops the signal
  // kernel); KOORDHIP_SELECT_ONEWG restores one workgroup per pod for A/B runs
  c->sel_split = std::getenv("KOORDHIP_SELECT_ONEWG") == nullptr;
  // Fit LeastAllocated + LoadAware least-used (+ NodeNUMAResource LeastAllocated):
  // a commit never raises a key.  A MostAllocated NUMA score rises with every
  // commit, so the resolve re-evaluates its modified nodes for every pod.
  // BalancedAllocation rewards the balance of cpu and memory, which a commit
  // can improve: not monotone either.
  c->monotone = (((cfg->score_plugins & KOORDHIP_PLUGIN_NUMA) && cfg->numa_most_allocated) ||
                 (cfg->score_plugins & KOORDHIP_PLUGIN_BALANCED))
                    ? 0
                    : 1;
  {
    int64_t max_total = 0;  // every plugin score is in [0, 100]
    for (int p = 0; p < KOORDHIP_NPLUGINS; p++)
      if (cfg->score_plugins & kScorePluginBit[p]) max_total += 100 * cfg->plugin_weight[p];
    if (cfg->score_plugins & KOORDHIP_PLUGIN_DEVICESHARE) max_total += 100 * (int64_t)cfg->ext_weight[0];
    if (cfg->score_plugins & KOORDHIP_PLUGIN_AFFINITY_SCORE) max_total += 100 * (int64_t)cfg->ext_weight[1];
    if (cfg->score_plugins & KOORDHIP_PLUGIN_TAINT_SCORE) max_total += 100 * (int64_t)cfg->ext_weight[2];
    if (cfg->score_plugins & KOORDHIP_PLUGIN_PTS) max_total += 100 * (int64_t)cfg->ext_weight[3];
    if (cfg->score_plugins & KOORDHIP_PLUGIN_IPA) max_total += 100 * (int64_t)cfg->ext_weight[4];
    c->dc.resv_b1 = (int32_t)max_total + 1;
    if (cfg->score_plugins & KOORDHIP_PLUGIN_RESERVATION) {
      // the ranking totals of resv.hpp: one normalised Reservation unit must
      // outweigh every other total, and they must fit the u16 score matrix /
      // the selection histogram
      if ((int64_t)cfg->reservation_weight <= max_total) {
        delete c;
        return fail(KOORDHIP_EINVAL, "reservation_weight must exceed 100 x the other score weights");
      }
      max_total = 101 * (max_total + 1) + KOORDHIP_RESV_MAX_ORDERS - 1;
    }
    // ranking totals travel as 32-bit key halves (total + 1); the split
    // evaluation (k_scan's u16 score matrix) only takes totals below 2^15
    if (max_total + 2 > (1ll << 30)) {
      delete c;
      return fail(KOORDHIP_EINVAL, "score weights too large: the ranking total must stay below 2^30");
    }
    // totals the split path's u16 score matrix cannot hold run the fused path,
    // whose 32-bit keys take them (also when KOORDHIP_EVAL=split asked for the split one)
    if (!c->eval_fused && max_total + 2 > 32768) c->eval_fused = true;
    int bits = 1;
    while ((1ll << bits) <= max_total + 1) bits++;
    c->score_bits = bits;
    c->nbins = (int32_t)std::min<int64_t>(max_total + 2, 32768);
    c->dc.wide_keys = max_total + 1 >= 65536 ? 1 : 0;
  }
  int dev = cfg->device;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  c->device = dev;
  hipError_t e = hipSetDevice(dev);
  {
    // split select: one workgroup per CU over a round (G x batch ~ CUs).  More
    // groups queue behind the persistent resolve workgroup's CU and lengthen
    // the evaluation stream (config 4 sweep: G=8 748k, G=16 718k pods/s at 32 pods)
    int cus = 256;
    if (e == hipSuccess && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0))
      cus = 256;
    c->n_cu = cus;
    // (5/8 of a CU per pod and round: config 4 measured 6 per pod above 10)
    c->sel_g = std::max(1, std::min(kh::kSelGMax, (cus * 5) / (8 * c->batch)));
    if (const char *g = std::getenv("KOORDHIP_SEL_G")) c->sel_g = std::max(1, std::min(kh::kSelGMax, std::atoi(g)));
  }
  // KOORDHIP_CU_RESERVE=<mask>: the persistent resolve gets the CUs of bit
  // mask <mask> (word 0 of the stream CU mask; "1" = CU 0) to itself, the
  // evaluation streams run on every other CU
  if (const char *r = std::getenv("KOORDHIP_CU_RESERVE")) c->cu_reserve = (uint32_t)std::strtoul(r, nullptr, 0);
  if (c->cu_reserve && e == hipSuccess) {
    std::vector<uint32_t> m((size_t)(c->n_cu + 31) / 32, 0xffffffffu);
    m[0] &= ~c->cu_reserve;
    if (c->n_cu % 32) m.back() &= (1u << (c->n_cu % 32)) - 1u;
    e = hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)m.size(), m.data());
  } else if (e == hipSuccess && !std::getenv("KOORDHIP_POOLED_STREAM")) {
    // the main evaluation stream on a hardware queue of its own: a CU-masked
    // stream is never pooled.  A pooled stream shares its queue with other
    // streams of the process (the null stream, RCCL's internal streams), and
    // with a communicator attached the one-rank exchange path measured 468k
    // pods/s on config 4 there against 1.00M on a dedicated queue (its small
    // per-round kernels waited ~40 us behind the queue's other work).
    std::vector<uint32_t> m((size_t)(c->n_cu + 31) / 32, 0xffffffffu);
    if (c->n_cu % 32) m.back() &= (1u << (c->n_cu % 32)) - 1u;
    e = hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)m.size(), m.data());
  } else if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  }
  if (e == hipSuccess) e = hipEventCreate(&c->t0);
  if (e == hipSuccess) e = hipEventCreate(&c->t1);
  if (e == hipSuccess) e = hipMalloc(&c->d_tmp_pod, sizeof(kh::DevPod));
  if (e == hipSuccess) e = hipMalloc(&c->d_rc, 64);  // int32 status + (at byte 8) the commit cpuset
  if (e != hipSuccess) {
    std::string m = std::string("device init: ") + hipGetErrorString(e);
    delete c;
    return fail(KOORDHIP_EDEVICE, m);
  }
  *out = c;
  return 0;
}

int koordhip_destroy(koordhip_ctx *c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_cols(c);
  for (void *p : c->ckpt) (void)hipFree(p);
  for (void *p : {(void *)c->d_pods, (void *)c->d_out, (void *)c->d_partial[0], (void *)c->d_partial[1], (void *)c->d_lists,
                  (void *)c->d_gather, (void *)c->d_final, (void *)c->d_tmp_pod, (void *)c->d_tmp_podx, (void *)c->d_dbg,
                  (void *)c->d_cpus, (void *)c->d_classes, (void *)c->d_rc, (void *)c->d_mod, (void *)c->d_desc,
                  (void *)c->d_selpart[0], (void *)c->d_selcnt[0], (void *)c->d_selpart[1], (void *)c->d_selcnt[1],
                  (void *)c->d_etk_part[0], (void *)c->d_etk_part[1], (void *)c->d_etk_pcnt[0],
                  (void *)c->d_etk_pcnt[1], (void *)c->d_etk_sync[0], (void *)c->d_etk_sync[1], c->d_upd,
                  (void *)c->d_podx, (void *)c->d_devout, (void *)c->d_seqg, c->d_seqdesc, (void *)c->d_pod_cls,
                  (void *)c->d_cls_pod, (void *)c->d_cls_buf, (void *)c->d_cls_meta, c->d_cls_S,
                  (void *)c->d_plan, (void *)c->d_plan_pods, (void *)c->d_ext_idx, c->d_ext_scr})
    if (p) (void)hipFree(p);
  for (int i = 0; i < kRing; i++)
    if (c->ev_res[i]) (void)hipEventDestroy(c->ev_res[i]);
  if (c->ev_start) (void)hipEventDestroy(c->ev_start);
  if (c->rstream) {
    (void)hipStreamSynchronize(c->rstream);
    (void)hipStreamDestroy(c->rstream);
  }
  if (c->stream2) {
    (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamDestroy(c->stream2);
  }
  if (c->ev_eval2) (void)hipEventDestroy(c->ev_eval2);
  for (hipStream_t xs : {c->xstream, c->xstream2, c->xstream3})
    if (xs) {
      (void)hipStreamSynchronize(xs);
      (void)hipStreamDestroy(xs);
    }
  if (c->ev_ext) (void)hipEventDestroy(c->ev_ext);
  if (c->ev_ext2) (void)hipEventDestroy(c->ev_ext2);
  if (c->ev_ext3) (void)hipEventDestroy(c->ev_ext3);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->t0) (void)hipEventDestroy(c->t0);
  if (c->t1) (void)hipEventDestroy(c->t1);
  if (c->comm2) (void)ncclCommDestroy(c->comm2);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->group) c->group->abort();
  for (hipEvent_t e : {c->ev_part, c->ev_copy})
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int koordhip_load_snapshot(koordhip_ctx *c, const koordhip_node_soa *s, int32_t n) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (n < 0) return fail(KOORDHIP_EINVAL, "n < 0");
  if (n > kMaxNodes) return fail(KOORDHIP_EINVAL, "more than 400000 nodes in one snapshot");
  if (int e = validate_soa(s)) return e;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  free_cols(c);
  for (void *p : c->ckpt) (void)hipFree(p);
  c->ckpt.clear();
  kh::DevNodes &d = c->d;
  d.n = n;
  int e = 0;
  for (int r = 0; r < KOORDHIP_NRES && !e; r++) {
    double *a = nullptr, *q = nullptr;
    e = dev_alloc(c, &a, n);
    if (!e) e = dev_alloc(c, &q, n);
    if (!e) e = upload_q(c, a, s->alloc[r], n, "alloc");
    if (!e) e = upload_q(c, q, s->requested[r], n, "requested");
    d.alloc[r] = a;
    d.requested[r] = q;
  }
  auto col64 = [&](int64_t **dst, const int64_t *src) {
    if (!e) e = dev_alloc(c, dst, n);
    if (!e) e = upload(c, *dst, src, n);
  };
  auto colq = [&](double **dst, const int64_t *src, const char *what) {
    if (!e) e = dev_alloc(c, dst, n);
    if (!e) e = upload_q(c, *dst, src, n, what);
  };
  int32_t *ap = nullptr, *np = nullptr;
  if (!e) e = dev_alloc(c, &ap, n);
  if (!e) e = upload(c, ap, s->alloc_pods, n);
  if (!e) e = dev_alloc(c, &np, n);
  if (!e) e = upload(c, np, s->npods, n);
  d.alloc_pods = ap;
  d.npods = np;
  colq(&d.nz_cpu, s->nz_cpu_m, "nz_cpu_m");
  colq(&d.nz_mem, s->nz_mem, "nz_mem");
  double *lac = nullptr, *lam = nullptr;
  colq(&lac, s->la_alloc_cpu_m, "la_alloc_cpu_m");
  colq(&lam, s->la_alloc_mem, "la_alloc_mem");
  d.la_alloc_cpu = lac;
  d.la_alloc_mem = lam;
  colq(&d.la_used_cpu, s->la_used_cpu_m, "la_used_cpu_m");
  colq(&d.la_used_mem, s->la_used_mem, "la_used_mem");
  colq(&d.la_used_prod_cpu, s->la_used_prod_cpu_m, "la_used_prod_cpu_m");  // NULL -> zeros
  colq(&d.la_used_prod_mem, s->la_used_prod_mem, "la_used_prod_mem");
  if (!e) e = dev_alloc(c, &d.flags, n);
  // LoadAware Filter inputs
  kh::PrepIn &pi = c->prep;
  for (int r = 0; r < 2 && !e; r++) {
    int64_t *a = nullptr, *b = nullptr, *cc = nullptr, *t = nullptr, *pt = nullptr;
    col64(&a, s->laf_used_m[r]);
    col64(&b, s->laf_total_m[r]);
    col64(&cc, s->laf_prod_used_m[r]);
    col64(&t, s->laf_thr[r]);
    col64(&pt, s->laf_prod_thr[r]);
    pi.used_m[r] = a;
    pi.total_m[r] = b;
    pi.prod_used_m[r] = cc;
    pi.thr[r] = t;
    pi.prod_thr[r] = pt;
  }
  uint8_t *lf = nullptr;
  if (!e) e = dev_alloc(c, &lf, n);
  if (!e) e = upload(c, lf, s->la_flags, n);
  pi.la_flags = lf;
  // static node filters: the allow mask per node (no column = every class)
  d.sallow = nullptr;
  if (!e && (c->dc.filt & KOORDHIP_PLUGIN_NODE_STATIC) && s->static_allow) {
    uint32_t *sa = nullptr;
    e = dev_alloc(c, &sa, n);
    if (!e) e = upload(c, sa, s->static_allow, n);
    d.sallow = sa;
  }
  if (!e) e = load_numa_columns(c, s, n);
  if (!e) e = load_resv_columns(c, s, n);
  if (!e) e = load_ext_columns(c, s, n);
  // the Reservation plugin on NUMA topology-policy nodes: the pipelined greedy's
  // rows keep either the zones or the reserved CPUs, so such a snapshot runs in
  // the sequential cycle (seq.hip: eval_total_resv<.., Z>)
  // (and more than KOORDHIP_RESV_SLOTS reservations per node: the pipelined
  // rows hold at most that many)
  // (and device-holding reservations listing extended scalars: their
  // scoreReservation / FilterReservation / fitsNode terms live only in the
  // sequential cycle's rules, resv.hpp ResvXS)
  c->seq_snap = c->dc.resv && (c->dc.zones || c->dc.resv_slots > KOORDHIP_RESV_SLOTS || c->resv_x);
  c->seq = c->seq_profile || c->seq_snap;
  if (e) {
    free_cols(c);
    return e;
  }
  // la_alloc == alloc for cpu and memory? then the eval kernels read them once
  c->dc.la_alias = (n == 0) || (std::memcmp(s->la_alloc_cpu_m, s->alloc[KOORDHIP_RES_CPU], n * sizeof(int64_t)) == 0 &&
                                std::memcmp(s->la_alloc_mem, s->alloc[KOORDHIP_RES_MEM], n * sizeof(int64_t)) == 0);
  HIP_TRY(kh::launch_prep_flags(pi, d, nullptr, n, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->n = n;
  c->loaded = true;
  return 0;
}

int koordhip_update_nodes(koordhip_ctx *c, const int32_t *idx, const koordhip_node_soa *rows, int32_t m) {
  if (!c || !idx) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (m <= 0) return 0;
  if (int e = validate_soa(rows)) return e;
  // ---- validate everything before the first device write: a rejected call
  //      leaves the snapshot untouched
  {
    std::vector<int32_t> sorted(idx, idx + m);
    std::sort(sorted.begin(), sorted.end());
    if (sorted.front() < 0 || sorted.back() >= c->n) return fail(KOORDHIP_EINVAL, "row index out of range");
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
      return fail(KOORDHIP_EINVAL, "duplicate row index (a row would mix fields of two updates)");
  }
  // device-holding reservations (ABI 13 / 14): a row carrying the reservation
  // columns replaces ALL of the node's reservation state, its device-holding
  // reservation included -- rows without resv_dev_slot / resv_dev (and
  // resv_xalloc) hold none, so the node's slot, device allocation and scalars
  // are cleared (a different reservation moving into the slot cannot inherit
  // them).  Rows without reservation columns leave all of it alone.
  const bool rdev_rows = rows->resv_dev_slot || rows->resv_dev || rows->resv_xalloc || rows->resv_xallocated;
  if (rdev_rows) {
    if (!c->d.dv.rslot)
      return fail(KOORDHIP_EINVAL, "update rows: device-holding reservations need the resv_dev columns at load_snapshot");
    if (!rows->resv_flags) return fail(KOORDHIP_EINVAL, "update rows: resv_dev columns come with the reservation columns");
    if (!rows->resv_dev_slot || !rows->resv_dev || (rows->resv_xallocated && !rows->resv_xalloc))
      return fail(KOORDHIP_EINVAL, "update rows: resv_dev_slot and resv_dev together (resv_xallocated with resv_xalloc)");
    if (rows->dev_slots != c->d.dv.slots || !rows->dev_minor)
      return fail(KOORDHIP_EINVAL, "update rows: a device-holding reservation row needs the node's device columns");
    if (std::max(1, rows->resv_slots) != c->d.rv.slots)
      return fail(KOORDHIP_EINVAL, "update rows: resv_slots differs from the loaded snapshot's");
    if (int e = check_resv_dev(rows, m)) return e;
    if (rows->resv_xalloc) {
      if (int e = check_resv_scalars(rows->resv_xalloc, rows->resv_xallocated, rows->resv_dev_slot, m)) return e;
      bool anyx = false;
      for (size_t a = 0; a < (size_t)m * KOORDHIP_NXRES && !anyx; a++) anyx = rows->resv_xalloc[a] != 0;
      if (anyx && !c->d.dv.rxa)
        return fail(KOORDHIP_EINVAL, "update rows: reservations listing extended scalars need the resv_xalloc column at "
                                     "load_snapshot");
    }
  }
  const bool numa_rows = c->numa && rows->numa_class;
  if (numa_rows) {
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
      if (!rows->numa_free[w] || !rows->numa_excl_pcpu[w] || !rows->numa_excl_numa[w])
        return fail(KOORDHIP_EINVAL, "NUMA mask column missing");
    if (!rows->numa_alloc_cnt || !rows->numa_flags) return fail(KOORDHIP_EINVAL, "NUMA column missing");
    for (int32_t j = 0; j < m; j++)
      if (rows->numa_class[j] >= c->n_classes)
        return fail(KOORDHIP_EINVAL, "numa_class index out of range (classes are fixed at load_snapshot)");
  }
  std::vector<double> zrow_a, zrow_u;
  bool zrows = false, zpolicy = false;
  if (numa_rows) {
    if (int e = zone_rows(rows->numa_zone_alloc, rows->numa_class, rows->numa_flags, c->host_classes.data(), m, zrow_a,
                          &zpolicy))
      return e;
    if (int e = zone_rows(rows->numa_zone_used, rows->numa_class, rows->numa_flags, c->host_classes.data(), m, zrow_u,
                          &zpolicy))
      return e;
    zrows = rows->numa_zone_alloc && rows->numa_zone_used;
    if (zpolicy && !c->d.nu.za)
      return fail(KOORDHIP_EINVAL, "a NUMA topology policy needs the zone columns at load_snapshot");
    if (zpolicy && c->dc.resv && !c->seq)
      return fail(KOORDHIP_EINVAL, "a NUMA topology policy on a Reservation snapshot without one: load the snapshot "
                                   "again (such snapshots run in the sequential cycle)");
    zrows = zrows && c->d.nu.za;
  }
  bool amp_rows = false, amp_any = false;
  if (numa_rows && rows->numa_amp_cpu) {
    if (int e = check_amp(rows->numa_amp_cpu, rows->numa_flags, m, &amp_any)) return e;
    if (!c->d.nu.amp) {
      bool any = amp_any;
      if (any) return fail(KOORDHIP_EINVAL, "a CPU amplification ratio needs the numa_amp_cpu column at load_snapshot");
    }
    amp_rows = c->d.nu.amp != nullptr;
  }
  if ((c->dc.filt & KOORDHIP_PLUGIN_NODE_STATIC) && rows->static_allow && !c->d.sallow)
    for (int32_t j = 0; j < m; j++)
      if (rows->static_allow[j] != 0xFFFFFFFFu)
        return fail(KOORDHIP_EINVAL, "a static node filter needs the static_allow column at load_snapshot");
  const bool resv_rows = c->dc.resv && rows->resv_flags;
  const int32_t rslots = std::max(1, rows->resv_slots);
  if (c->resv && rows->resv_flags && !c->dc.resv) {
    for (int32_t j = 0; j < rslots * m; j++)
      if (rows->resv_flags[j] & KOORDHIP_RESV_PRESENT)
        return fail(KOORDHIP_EINVAL, "a reservation needs the reservation columns at load_snapshot");
  }
  if (resv_rows && rslots != c->d.rv.slots)
    return fail(KOORDHIP_EINVAL, "update rows: resv_slots differs from the loaded snapshot's");
  if (resv_rows)
    if (int e = check_resv_rows(rows, rslots * m)) return e;
  // reserved CPUs of the rows (NULL: none), only into a snapshot loaded with them
  std::vector<uint64_t> zero_rc;
  const uint64_t *rc_rows[KOORDHIP_NUMA_WORDS] = {};
  if (resv_rows && c->numa && rows->resv_cpus[0]) {
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
      if (!rows->resv_cpus[w]) return fail(KOORDHIP_EINVAL, "resv_cpus: every word column or none");
    if (!numa_rows) return fail(KOORDHIP_EINVAL, "update rows with resv_cpus need the NUMA columns");
    std::vector<int32_t> ncpu;
    for (const auto &k : c->host_classes) ncpu.push_back(k.ncpu);
    if (int e = check_resv_cpus(rows, m, rslots, ncpu)) return e;
    if (!c->dc.resv_cpus) {
      for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
        for (int32_t j = 0; j < rslots * m; j++)
          if (rows->resv_cpus[w][j]) return fail(KOORDHIP_EINVAL, "reserved CPUs need the resv_cpus columns at load_snapshot");
    } else {
      for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) rc_rows[w] = rows->resv_cpus[w];
    }
  } else if (resv_rows && c->dc.resv_cpus) {
    zero_rc.assign((size_t)rslots * (size_t)m, 0ull);
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) rc_rows[w] = zero_rc.data();
  }
  // ---- one host staging image: [idx][column 0][column 1]..., 8-B aligned
  //      segments, quantities converted to the device's exact f64
  struct Col {
    void *dst;
    const void *src;
    int32_t esize;  // 8, 4 or 1 (or a whole ZoneRow)
    bool q;         // int64 quantity -> f64
    const char *what;
  };
  kh::DevNodes &d = c->d;
  kh::PrepIn &pi = c->prep;
  std::vector<Col> cols;
  for (int r = 0; r < KOORDHIP_NRES; r++) {
    cols.push_back({const_cast<double *>(d.alloc[r]), rows->alloc[r], 8, true, "alloc"});
    cols.push_back({d.requested[r], rows->requested[r], 8, true, "requested"});
  }
  cols.push_back({const_cast<int32_t *>(d.alloc_pods), rows->alloc_pods, 4, false, "alloc_pods"});
  cols.push_back({d.npods, rows->npods, 4, false, "npods"});
  cols.push_back({d.nz_cpu, rows->nz_cpu_m, 8, true, "nz_cpu_m"});
  cols.push_back({d.nz_mem, rows->nz_mem, 8, true, "nz_mem"});
  cols.push_back({const_cast<double *>(d.la_alloc_cpu), rows->la_alloc_cpu_m, 8, true, "la_alloc_cpu_m"});
  cols.push_back({const_cast<double *>(d.la_alloc_mem), rows->la_alloc_mem, 8, true, "la_alloc_mem"});
  cols.push_back({d.la_used_cpu, rows->la_used_cpu_m, 8, true, "la_used_cpu_m"});
  cols.push_back({d.la_used_mem, rows->la_used_mem, 8, true, "la_used_mem"});
  cols.push_back({d.la_used_prod_cpu, rows->la_used_prod_cpu_m, 8, true, "la_used_prod_cpu_m"});
  cols.push_back({d.la_used_prod_mem, rows->la_used_prod_mem, 8, true, "la_used_prod_mem"});
  for (int r = 0; r < 2; r++) {
    cols.push_back({const_cast<int64_t *>(pi.used_m[r]), rows->laf_used_m[r], 8, false, "laf_used_m"});
    cols.push_back({const_cast<int64_t *>(pi.total_m[r]), rows->laf_total_m[r], 8, false, "laf_total_m"});
    cols.push_back({const_cast<int64_t *>(pi.prod_used_m[r]), rows->laf_prod_used_m[r], 8, false, "laf_prod_used_m"});
    cols.push_back({const_cast<int64_t *>(pi.thr[r]), rows->laf_thr[r], 8, false, "laf_thr"});
    cols.push_back({const_cast<int64_t *>(pi.prod_thr[r]), rows->laf_prod_thr[r], 8, false, "laf_prod_thr"});
  }
  cols.push_back({const_cast<uint8_t *>(pi.la_flags), rows->la_flags, 1, false, "la_flags"});
  if (numa_rows) {
    kh::DevNuma &nu = c->d.nu;
    cols.push_back({const_cast<int32_t *>(nu.node_cls), rows->numa_class, 4, false, "numa_class"});
    cols.push_back({nu.cnt, rows->numa_alloc_cnt, 4, false, "numa_alloc_cnt"});
    cols.push_back({const_cast<uint8_t *>(nu.nflags), rows->numa_flags, 1, false, "numa_flags"});
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
      cols.push_back({nu.fr[w], rows->numa_free[w], 8, false, "numa_free"});
      cols.push_back({nu.ep[w], rows->numa_excl_pcpu[w], 8, false, "numa_excl_pcpu"});
      cols.push_back({nu.en[w], rows->numa_excl_numa[w], 8, false, "numa_excl_numa"});
    }
  }
  if (amp_rows)
    cols.push_back({const_cast<double *>(c->d.nu.amp), rows->numa_amp_cpu, 8, false, "numa_amp_cpu"});
  if (c->d.sallow && rows->static_allow)
    cols.push_back({const_cast<uint32_t *>(c->d.sallow), rows->static_allow, 4, false, "static_allow"});
  if (resv_rows) {  // slot q of the rows -> slot q of the nodes (the same indices)
    kh::DevResv &rv = c->d.rv;
    const size_t dn = (size_t)rv.stride, sm = (size_t)m;
    for (int32_t q = 0; q < rslots; q++) {
      cols.push_back({const_cast<uint32_t *>(rv.flags) + q * dn, rows->resv_flags + q * sm, 4, false, "resv_flags"});
      cols.push_back({const_cast<int32_t *>(rv.rank) + q * dn, rows->resv_order_rank + q * sm, 4, false, "resv_order_rank"});
      cols.push_back({rv.rn + q * dn, rows->resv_assigned + q * sm, 4, false, "resv_assigned"});
      for (int k = 0; k < 2; k++) {
        cols.push_back({const_cast<double *>(rv.ra[k]) + q * dn, rows->resv_alloc[k] + q * sm, 8, true, "resv_alloc"});
        cols.push_back({const_cast<double *>(rv.rz[k]) + q * dn, rows->resv_nz[k] + q * sm, 8, true, "resv_nz"});
        cols.push_back({rv.rd[k] + q * dn, rows->resv_allocated[k] + q * sm, 8, true, "resv_allocated"});
      }
      if (rc_rows[0])
        for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
          cols.push_back({rv.rc[w] + q * dn, rc_rows[w] + q * sm, 8, false, "resv_cpus"});
    }
  }
  // the device-holding reservation of every row with reservation columns (none: cleared)
  std::vector<int32_t> no_rslot;
  std::vector<int64_t> no_rdev, no_rx;
  bool rows_x = false;
  if (resv_rows && c->d.dv.rslot) {
    kh::DevDev &dv = c->d.dv;
    const int32_t rb = 2 * KOORDHIP_DEV_TYPES * dv.slots * KOORDHIP_DEV_RES;
    if (!rdev_rows) {
      no_rslot.assign((size_t)m, -1);
      no_rdev.assign((size_t)m * rb, 0);
    }
    cols.push_back({const_cast<int32_t *>(dv.rslot), rdev_rows ? rows->resv_dev_slot : no_rslot.data(), 4, false,
                    "resv_dev_slot"});
    cols.push_back({dv.rdev, rdev_rows ? rows->resv_dev : no_rdev.data(), rb * 8, false, "resv_dev"});
    if (dv.rxa) {
      const bool given = rdev_rows && rows->resv_xalloc;
      if (!given || !rows->resv_xallocated) no_rx.assign((size_t)m * KOORDHIP_NXRES, 0);
      for (int j = 0; j < KOORDHIP_NXRES; j++) {
        cols.push_back({const_cast<int64_t *>(dv.rxa) + (size_t)j * c->n,
                        (given ? rows->resv_xalloc : no_rx.data()) + (size_t)j * m, 8, false, "resv_xalloc"});
        cols.push_back({dv.rxd + (size_t)j * c->n,
                        ((given && rows->resv_xallocated) ? rows->resv_xallocated : no_rx.data()) + (size_t)j * m, 8,
                        false, "resv_xallocated"});
      }
      for (size_t a = 0; given && a < (size_t)m * KOORDHIP_NXRES && !rows_x; a++) rows_x = rows->resv_xalloc[a] != 0;
    }
  }
  // ABI 9: DeviceShare device rows, extended scalars, static Scores (the
  // sequential cycle's columns; element = a node's whole device row)
  if (c->seq_profile) {
    kh::DevDev &dv = c->d.dv;
    if (rows->dev_slots > 0) {
      if (!dv.used || rows->dev_slots != dv.slots || !rows->dev_present || !rows->dev_minor || !rows->dev_total)
        return fail(KOORDHIP_EINVAL, "update rows: device columns must match the loaded snapshot's dev_slots");
      const int32_t S = dv.slots;
      for (size_t a = 0; a < (size_t)m * KOORDHIP_DEV_TYPES * S * KOORDHIP_DEV_RES; a++)
        if (rows->dev_total[a] < 0 || rows->dev_total[a] >= (1ll << 45) ||
            (rows->dev_used && (rows->dev_used[a] < 0 || rows->dev_used[a] >= (1ll << 45))))
          return fail(KOORDHIP_EINVAL, "update rows: dev_total / dev_used out of [0, 2^45)");
      for (int32_t j = 0; j < m; j++) {
        int64_t mem = -1;
        for (int32_t q = 0; q < S; q++) {
          const size_t a = ((size_t)j * KOORDHIP_DEV_TYPES + KOORDHIP_DEV_GPU) * S + q;
          const int64_t *t = rows->dev_total + a * KOORDHIP_DEV_RES;
          if (rows->dev_minor[a] < 0 || (t[0] == 0 && t[1] == 0 && t[2] == 0)) continue;
          if (t[2] <= 0 || (mem >= 0 && t[2] != mem)) return fail(KOORDHIP_EINVAL, "update rows: GPU memory sizes differ");
          mem = t[2];
        }
      }
      const int32_t rb = KOORDHIP_DEV_TYPES * S;
      cols.push_back({const_cast<uint8_t *>(dv.present), rows->dev_present, 1, false, "dev_present"});
      cols.push_back({const_cast<int32_t *>(dv.minor), rows->dev_minor, rb * 4, false, "dev_minor"});
      cols.push_back({const_cast<int64_t *>(dv.total), rows->dev_total, rb * KOORDHIP_DEV_RES * 8, false, "dev_total"});
      if (rows->dev_used) cols.push_back({dv.used, rows->dev_used, rb * KOORDHIP_DEV_RES * 8, false, "dev_used"});
    }
    if (rows->xalloc && !dv.xalloc) return fail(KOORDHIP_EINVAL, "extended scalars need the xalloc column at load_snapshot");
    for (int j = 0; j < KOORDHIP_NXRES; j++) {
      if (rows->xalloc)
        cols.push_back({const_cast<int64_t *>(dv.xalloc) + (size_t)j * c->n, rows->xalloc + (size_t)j * m, 8, false, "xalloc"});
      if (rows->xrequested)
        cols.push_back({dv.xreq + (size_t)j * c->n, rows->xrequested + (size_t)j * m, 8, false, "xrequested"});
    }
    for (int w = 0; w < 2; w++) {
      if (!rows->static_score[w]) continue;
      if (!dv.sscore[w]) return fail(KOORDHIP_EINVAL, "static scores need their column at load_snapshot");
      for (int q = 0; q < KOORDHIP_MAX_STATIC_CLASSES; q++)
        cols.push_back({const_cast<uint16_t *>(dv.sscore[w]) + (size_t)q * c->n, rows->static_score[w] + (size_t)q * m, 2,
                        false, "static_score"});
    }
    // PodTopologySpread rows: the same keys / constraint table as the loaded snapshot
    if (rows->pts_keys > 0) {
      const kh::PtsArgs &pa = c->pts;
      if (!pa.dom || rows->pts_keys != pa.keys || rows->pts_cons != pa.cons || !rows->pts_dom || !rows->pts_elig ||
          (pa.cons > 0 && !rows->pts_cnt))
        return fail(KOORDHIP_EINVAL, "update rows: PodTopologySpread columns must match the loaded snapshot's tables");
      for (int k = 0; k < pa.keys; k++) {
        for (int32_t j = 0; j < m; j++) {
          const int32_t v = rows->pts_dom[(size_t)k * m + j];
          if (v < -1 || v >= (((pa.host >> k) & 1u) ? c->n : KOORDHIP_PTS_DOMAINS) ||
              (((pa.host >> k) & 1u) && v >= 0 && v != idx[j]))
            return fail(KOORDHIP_EINVAL, "update rows: pts_dom out of range");
        }
        cols.push_back({const_cast<int32_t *>(pa.dom) + (size_t)k * c->n, rows->pts_dom + (size_t)k * m, 4, false,
                        "pts_dom"});
      }
      for (int cc = 0; cc < pa.cons; cc++)
        cols.push_back({pa.cnt + (size_t)cc * c->n, rows->pts_cnt + (size_t)cc * m, 4, false, "pts_cnt"});
      cols.push_back({const_cast<uint16_t *>(pa.elig), rows->pts_elig, 2, false, "pts_elig"});
    }
    // InterPodAffinity rows: the loaded snapshot's entries
    if (rows->ipa_ents > 0) {
      const kh::IpaArgs &ia = c->ipa;
      if (!ia.cnt || rows->ipa_ents != ia.ents || !rows->ipa_cnt)
        return fail(KOORDHIP_EINVAL, "update rows: InterPodAffinity columns must match the loaded snapshot's entries");
      for (int q = 0; q < ia.ents; q++)
        cols.push_back({ia.cnt + (size_t)q * c->n, rows->ipa_cnt + (size_t)q * m, 4, false, "ipa_cnt"});
    }
  } else if (rows->dev_slots > 0 || rows->xalloc || rows->static_score[0] || rows->static_score[1] ||
             rows->pts_keys > 0 || rows->ipa_ents > 0) {
    return fail(KOORDHIP_EINVAL, "device / extended-scalar / static-score rows need DeviceShare or a normalized Score "
                                 "plugin in the profile");
  }
  if (zrows) {  // [m][2][ZMAX] f64 rows, scattered as one ZoneRow element per row
    kh::DevNuma &nu = c->d.nu;
    cols.push_back({const_cast<double *>(nu.za), zrow_a.data(), (int32_t)sizeof(kh::ZoneRow), false, "numa_zone_alloc"});
    cols.push_back({nu.zu, zrow_u.data(), (int32_t)sizeof(kh::ZoneRow), false, "numa_zone_used"});
  }
  const size_t seg_idx = ((size_t)m * 4 + 7) & ~(size_t)7;
  size_t bytes = seg_idx;
  std::vector<size_t> off(cols.size());
  for (size_t q = 0; q < cols.size(); q++) {
    off[q] = bytes;
    bytes += ((size_t)m * cols[q].esize + 7) & ~(size_t)7;
  }
  std::vector<uint8_t> &img = c->upd_host;
  img.assign(bytes, 0);
  std::memcpy(img.data(), idx, (size_t)m * 4);
  for (size_t q = 0; q < cols.size(); q++) {
    const Col &k = cols[q];
    if (k.q) {
      const int64_t *src = static_cast<const int64_t *>(k.src);
      double *o = reinterpret_cast<double *>(img.data() + off[q]);
      for (int32_t j = 0; j < m; j++) {
        if (!exact_ok(src[j]))
          return fail(KOORDHIP_EINVAL, std::string(k.what) + ": quantity magnitude >= 2^45 is outside the engine's exact range");
        o[j] = (double)src[j];
      }
    } else {
      std::memcpy(img.data() + off[q], k.src, (size_t)m * k.esize);
    }
  }
  bool alias = c->dc.la_alias;
  for (int32_t j = 0; j < m && alias; j++)
    if (rows->la_alloc_cpu_m[j] != rows->alloc[KOORDHIP_RES_CPU][j] || rows->la_alloc_mem[j] != rows->alloc[KOORDHIP_RES_MEM][j])
      alias = false;
  // ---- device: one upload into the persistent staging buffer, the scatters,
  //      the flag recompute, one synchronisation
  HIP_TRY(hipSetDevice(c->device));
  if (int e = ensure(c, &c->d_upd, &c->upd_cap, bytes)) return e;
  uint8_t *dev = static_cast<uint8_t *>(c->d_upd);
  const int32_t *d_idx = reinterpret_cast<const int32_t *>(dev);
  HIP_TRY(hipMemcpyAsync(dev, img.data(), bytes, hipMemcpyHostToDevice, c->stream));
  for (size_t q = 0; q < cols.size(); q++) {
    const Col &k = cols[q];
    const void *src = dev + off[q];
    if (k.esize > 8)  // whole rows (NUMA zone rows, device rows)
      HIP_TRY(kh::launch_scatter_rows(k.dst, src, d_idx, m, k.esize, c->stream));
    else if (k.esize == 2)
      HIP_TRY(kh::launch_scatter<uint16_t>(static_cast<uint16_t *>(k.dst), static_cast<const uint16_t *>(src), d_idx, m,
                                           c->stream));
    else if (k.esize == 8)
      HIP_TRY(kh::launch_scatter<int64_t>(static_cast<int64_t *>(k.dst), static_cast<const int64_t *>(src), d_idx, m, c->stream));
    else if (k.esize == 4)
      HIP_TRY(kh::launch_scatter<int32_t>(static_cast<int32_t *>(k.dst), static_cast<const int32_t *>(src), d_idx, m, c->stream));
    else
      HIP_TRY(kh::launch_scatter<uint8_t>(static_cast<uint8_t *>(k.dst), static_cast<const uint8_t *>(src), d_idx, m, c->stream));
  }
  c->dc.la_alias = alias ? 1 : 0;
  if (zpolicy) c->dc.zones = 1;
  if (zpolicy && c->dc.resv) c->seq_snap = true;
  if (rows_x && !c->resv_x) {  // reservations listing extended scalars from now on: the sequential cycle places
    c->resv_x = true;
    c->seq_snap = true;
    c->seq = true;
  }
  if (amp_any) c->dc.amp = 1;
  HIP_TRY(kh::launch_prep_flags(pi, d, d_idx, m, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));  // the host image may be reused by the next call
  return 0;
}

int koordhip_read_nodes(koordhip_ctx *c, int64_t *requested, int64_t *nz, int32_t *npods, int64_t *la_used,
                        int64_t *la_used_prod) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t n = c->n, b = n * sizeof(int64_t);
  if (n == 0) return 0;
  (void)b;
  int e = 0;
  if (requested)
    for (int r = 0; r < KOORDHIP_NRES && !e; r++) e = download_q(c->d.requested[r], requested + r * n, n);
  if (nz && !e) e = download_q(c->d.nz_cpu, nz, n);
  if (nz && !e) e = download_q(c->d.nz_mem, nz + n, n);
  if (e) return e;
  if (npods) HIP_TRY(hipMemcpy(npods, c->d.npods, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (la_used && !e) e = download_q(c->d.la_used_cpu, la_used, n);
  if (la_used && !e) e = download_q(c->d.la_used_mem, la_used + n, n);
  if (la_used_prod && !e) e = download_q(c->d.la_used_prod_cpu, la_used_prod, n);
  if (la_used_prod && !e) e = download_q(c->d.la_used_prod_mem, la_used_prod + n, n);
  return e;
}

int koordhip_read_numa(koordhip_ctx *c, uint64_t *free_mask, uint64_t *excl_pcpu, uint64_t *excl_numa,
                       int32_t *alloc_cnt) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (!c->numa) return fail(KOORDHIP_ESTATE, "NodeNUMAResource is not enabled");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t n = c->n, b = n * sizeof(uint64_t);
  if (n == 0) return 0;
  const kh::DevNuma &nu = c->d.nu;
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    if (free_mask) HIP_TRY(hipMemcpy(free_mask + w * n, nu.fr[w], b, hipMemcpyDeviceToHost));
    if (excl_pcpu) HIP_TRY(hipMemcpy(excl_pcpu + w * n, nu.ep[w], b, hipMemcpyDeviceToHost));
    if (excl_numa) HIP_TRY(hipMemcpy(excl_numa + w * n, nu.en[w], b, hipMemcpyDeviceToHost));
  }
  if (alloc_cnt) HIP_TRY(hipMemcpy(alloc_cnt, nu.cnt, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_read_numa_zones(koordhip_ctx *c, int64_t *zone_used) {
  if (!c || !zone_used) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (!c->numa) return fail(KOORDHIP_ESTATE, "NodeNUMAResource is not enabled");
  constexpr int Z = KOORDHIP_NUMA_MAX_ZONES, NM = KOORDHIP_NUMA_MAX_NODES;
  const size_t n = c->n;
  std::memset(zone_used, 0, n * 2 * NM * sizeof(int64_t));
  if (n == 0 || !c->d.nu.zu) return 0;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::vector<double> zu(n * 2 * Z);
  HIP_TRY(hipMemcpy(zu.data(), c->d.nu.zu, zu.size() * sizeof(double), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; i++)
    for (int q = 0; q < 2; q++)
      for (int k = 0; k < Z; k++) zone_used[(i * 2 + q) * NM + k] = (int64_t)zu[(i * 2 + q) * Z + k];
  return 0;
}

int koordhip_read_reservations(koordhip_ctx *c, int64_t *allocated, int32_t *assigned) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (!c->resv) return fail(KOORDHIP_ESTATE, "Reservation is not enabled");
  const size_t n = (size_t)c->n * (size_t)(c->dc.resv ? c->d.rv.slots : 1);
  if (n == 0) return 0;
  if (!c->dc.resv) {  // no reservation columns: nothing is reserved anywhere
    if (allocated) std::memset(allocated, 0, 2 * n * sizeof(int64_t));
    if (assigned) std::memset(assigned, 0, n * sizeof(int32_t));
    return 0;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  int e = 0;
  if (allocated) e = download_q(c->d.rv.rd[0], allocated, n);
  if (allocated && !e) e = download_q(c->d.rv.rd[1], allocated + n, n);
  if (e) return e;
  if (assigned) HIP_TRY(hipMemcpy(assigned, c->d.rv.rn, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_read_resv_cpus(koordhip_ctx *c, uint64_t *cpus) {
  if (!c || !cpus) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (!c->resv) return fail(KOORDHIP_ESTATE, "Reservation is not enabled");
  const size_t n = (size_t)c->n * (size_t)(c->dc.resv ? c->d.rv.slots : 1);
  if (n == 0) return 0;
  if (!c->dc.resv_cpus) {
    std::memset(cpus, 0, KOORDHIP_NUMA_WORDS * n * sizeof(uint64_t));
    return 0;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++)
    HIP_TRY(hipMemcpy(cpus + (size_t)w * n, c->d.rv.rc[w], n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_read_resv_devices(koordhip_ctx *c, int64_t *resv_dev) {
  if (!c || !resv_dev) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  const size_t nd = (size_t)c->n * 2 * KOORDHIP_DEV_TYPES * (size_t)std::max(c->d.dv.slots, 0) * KOORDHIP_DEV_RES;
  if (nd == 0) return 0;
  if (!c->d.dv.rdev) {
    std::memset(resv_dev, 0, nd * sizeof(int64_t));
    return 0;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(resv_dev, c->d.dv.rdev, nd * sizeof(int64_t), hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_read_resv_scalars(koordhip_ctx *c, int64_t *resv_xallocated) {
  if (!c || !resv_xallocated) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  const size_t nx = (size_t)c->n * KOORDHIP_NXRES;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (!c->d.dv.rxd) {
    std::memset(resv_xallocated, 0, nx * sizeof(int64_t));
    return 0;
  }
  HIP_TRY(hipMemcpy(resv_xallocated, c->d.dv.rxd, nx * sizeof(int64_t), hipMemcpyDeviceToHost));
  return 0;
}

static int check_reserve_pods(const koordhip_ctx *c, const koordhip_pod *pods, int32_t n, bool *any);

int koordhip_eval(koordhip_ctx *c, const koordhip_pod *pods, int32_t n_pods, uint8_t *status, int32_t *scores,
                  koordhip_topk *topk, int32_t k) {
  if (!c || (!pods && n_pods > 0)) return fail(KOORDHIP_EINVAL, "NULL argument");
  bool reserve = false;
  if (pods)
    if (int e = check_reserve_pods(c, pods, n_pods, &reserve)) return e;
  if ((c->seq || reserve) && n_pods > 0) {  // the sequential cycle's evaluator (its first planes)
    if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
    const size_t n = (size_t)c->n, NPX = KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS;
    std::vector<int32_t> sc(scores ? (size_t)n_pods * NPX * n : 0);
    std::vector<uint16_t> st16(status ? (size_t)n_pods * n : 0);
    if (int e = koordhip_eval_ext(c, pods, nullptr, n_pods, status ? st16.data() : nullptr,
                                  scores ? sc.data() : nullptr, topk, k))
      return e;
    for (size_t q = 0; q < st16.size(); q++) status[q] = (uint8_t)st16[q];  // (no ext: no InterPodAffinity bit)
    if (scores)
      for (int32_t p = 0; p < n_pods; p++)
        std::memcpy(scores + (size_t)p * KOORDHIP_NPLUGINS * n, sc.data() + (size_t)p * NPX * n,
                    (size_t)KOORDHIP_NPLUGINS * n * sizeof(int32_t));
    return 0;
  }
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (n_pods < 0) return fail(KOORDHIP_EINVAL, "n_pods < 0");
  if (topk && (k < 1 || k > kMaxBatch)) return fail(KOORDHIP_EINVAL, "k must be in [1, 64]");
  if (n_pods == 0) return 0;
  HIP_TRY(hipSetDevice(c->device));
  const int32_t n = c->n;
  // parity mode works in slices of pods so the status/score buffers stay bounded
  const int32_t per = std::max<int32_t>(1, std::min<int32_t>(kMaxBatch, (int32_t)((256ll << 20) / (16ll * std::max(n, 1)))));
  kh::DevPod *dp = nullptr;
  uint8_t *dst = nullptr;
  int32_t *dsc = nullptr;
  uint64_t *dk = nullptr;
  int e = 0;
  auto cleanup = [&]() {
    for (void *p : {(void *)dp, (void *)dst, (void *)dsc, (void *)dk})
      if (p) (void)hipFree(p);
  };
  std::vector<kh::DevPod> hp;
  if (int ce = to_dev_pods(pods, n_pods, hp)) return ce;
  if (hipMalloc(&dp, (size_t)per * sizeof(kh::DevPod)) != hipSuccess ||
      (status && hipMalloc(&dst, (size_t)per * n) != hipSuccess) ||
      (scores && hipMalloc(&dsc, (size_t)per * KOORDHIP_NPLUGINS * n * sizeof(int32_t)) != hipSuccess) ||
      (topk && hipMalloc(&dk, (size_t)per * k * sizeof(uint64_t)) != hipSuccess)) {
    cleanup();
    return fail(KOORDHIP_ENOMEM, "eval buffers");
  }
  std::vector<uint64_t> hk(topk ? (size_t)per * k : 0);
  if (topk) e = eval_buffers(c, std::min(per, n_pods), 0, n, 0, c->stream, k);
  for (int32_t p0 = 0; p0 < n_pods && !e; p0 += per) {
    const int32_t np = std::min(per, n_pods - p0);
    if (hipMemcpyAsync(dp, hp.data() + p0, np * sizeof(kh::DevPod), hipMemcpyHostToDevice, c->stream) != hipSuccess) {
      e = fail(KOORDHIP_EDEVICE, "copy pods");
      break;
    }
    if ((status || scores) && kh::launch_eval_full(c->dc, c->d, dp, np, dst, dsc, c->stream) != hipSuccess) {
      e = fail(KOORDHIP_EDEVICE, "eval_full launch");
      break;
    }
    if (topk) e = topk_batch(c, dp, np, k, 0, n, dk, false, nullptr, 0, 0, c->stream, 0);
    if (e) break;
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
      e = fail(KOORDHIP_EDEVICE, "eval sync");
      break;
    }
    if (status && hipMemcpy(status + (size_t)p0 * n, dst, (size_t)np * n, hipMemcpyDeviceToHost) != hipSuccess)
      e = fail(KOORDHIP_EDEVICE, "copy status");
    if (!e && scores &&
        hipMemcpy(scores + (size_t)p0 * KOORDHIP_NPLUGINS * n, dsc, (size_t)np * KOORDHIP_NPLUGINS * n * sizeof(int32_t),
                  hipMemcpyDeviceToHost) != hipSuccess)
      e = fail(KOORDHIP_EDEVICE, "copy scores");
    if (!e && topk) {
      if (hipMemcpy(hk.data(), dk, (size_t)np * k * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) {
        e = fail(KOORDHIP_EDEVICE, "copy topk");
        break;
      }
      for (size_t j = 0; j < (size_t)np * k; j++) {
        koordhip_topk &o = topk[(size_t)p0 * k + j];
        const uint64_t x = hk[j];
        o.node = x ? (int32_t)(0xFFFFFFFFu - (uint32_t)x) : -1;
        o.score = x ? (int32_t)(x >> 32) - 1 : 0;
      }
    }
  }
  cleanup();
  return e;
}

// reserve pods (KOORDHIP_POD_RESERVE) in a batch: validated; true when the
// Reservation plugin handles one (the batch then runs in the sequential cycle)
static int check_reserve_pods(const koordhip_ctx *c, const koordhip_pod *pods, int32_t n, bool *any) {
  *any = false;
  for (int32_t j = 0; j < n; j++) {
    const uint32_t f = pods[j].flags;
    if (!(f & (KOORDHIP_POD_RESERVE | KOORDHIP_POD_RESV_OPERATING))) continue;
    if ((f & KOORDHIP_POD_RESERVE) && (f & KOORDHIP_POD_RESV_OPERATING))
      return fail(KOORDHIP_EINVAL, "a pod is either a reserve pod or in the reservation operating mode");
    if ((f & KOORDHIP_POD_RESERVE) && (pods[j].resv_match != 0 || (f & KOORDHIP_POD_RESV_AFFINITY)))
      return fail(KOORDHIP_EINVAL, "a reserve pod matches no reservation (resv_match 0, no reservation affinity)");
    if ((f & KOORDHIP_POD_RESV_OPERATING) && KOORDHIP_POD_RESERVE_POLICY(f) != 1u)
      return fail(KOORDHIP_EINVAL, "a reservation-operating-mode pod checks AllocatePolicy Aligned (bits 12-13 = 1)");
    if (KOORDHIP_POD_RESERVE_POLICY(f) > 2) return fail(KOORDHIP_EINVAL, "reserve pod: unknown allocate policy");
    *any = *any || c->dc.resv;
  }
  return 0;
}

// The staged pods' classes for the class-incremental lists (cls.hip): pods
// whose device records are byte-identical share a class.  More than
// kClsMaxClasses classes: none (the pipelined greedy evaluates every pod).
constexpr int32_t kClsMaxClasses = 1024;
struct PodBytesHash {
  size_t operator()(const std::array<uint64_t, 12> &a) const {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (uint64_t x : a) h = (h ^ x) * 0x100000001b3ull + (h >> 29);
    return (size_t)h;
  }
};

static int stage_classes(koordhip_ctx *c, const std::vector<kh::DevPod> &hp) {
  static_assert(sizeof(kh::DevPod) == 12 * sizeof(uint64_t), "DevPod as 12 words");
  const int32_t n = (int32_t)hp.size();
  c->pod_cls.assign(n, 0);
  c->cls_rep.clear();
  c->plan_ok = false;
  c->last_plan_us = 0;
  std::unordered_map<std::array<uint64_t, 12>, int32_t, PodBytesHash> m;
  for (int32_t j = 0; j < n; j++) {
    std::array<uint64_t, 12> k;
    std::memcpy(k.data(), &hp[j], sizeof(kh::DevPod));
    auto it = m.find(k);
    if (it == m.end()) {
      if ((int32_t)c->cls_rep.size() >= kClsMaxClasses) {
        c->cls_rep.clear();  // too many classes for the class lists
        return 0;
      }
      it = m.emplace(k, (int32_t)c->cls_rep.size()).first;
      c->cls_rep.push_back(hp[j]);
    }
    c->pod_cls[j] = it->second;
  }
  if (n == 0) return 0;
  const int32_t nc = (int32_t)c->cls_rep.size();
  if (nc > c->cls_pod_cap) {
    if (c->d_cls_pod) HIP_TRY(hipFree(c->d_cls_pod));
    c->d_cls_pod = nullptr;
    HIP_TRY(hipMalloc(&c->d_cls_pod, (size_t)nc * sizeof(kh::DevPod)));
    c->cls_pod_cap = nc;
  }
  if (n > c->pod_cls_cap) {
    if (c->d_pod_cls) HIP_TRY(hipFree(c->d_pod_cls));
    c->d_pod_cls = nullptr;
    HIP_TRY(hipMalloc(&c->d_pod_cls, (size_t)n * sizeof(int32_t)));
    c->pod_cls_cap = n;
  }
  HIP_TRY(hipMemcpyAsync(c->d_cls_pod, c->cls_rep.data(), (size_t)nc * sizeof(kh::DevPod), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_pod_cls, c->pod_cls.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  return 0;
}

static bool devshare_on(const koordhip_ctx *c) {
  return ((c->cfg.filter_plugins | c->cfg.score_plugins) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
}
// kh::KH_POD_DEVSHARE only matters to the reservation nomination: without
// reservations it stays off, so device pods keep sharing pod classes with
// byte-identical plain pods (the class lists of the pipelined greedy)
static bool devshare_resv_on(const koordhip_ctx *c) { return devshare_on(c) && c->dc.resv; }

// ext (optional): the pods' records, for kh::KH_POD_DEVSHARE (staged by stage_ext)
static int stage_pods_impl(koordhip_ctx *c, const koordhip_pod *pods, int32_t n_pods, const koordhip_pod_ext *ext) {
  if (!c || (!pods && n_pods > 0)) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (n_pods < 0) return fail(KOORDHIP_EINVAL, "n_pods < 0");
  bool reserve = false;
  if (int e = check_reserve_pods(c, pods, n_pods, &reserve)) return e;
  std::vector<kh::DevPod> hp;
  if (int e = to_dev_pods(pods, n_pods, hp, ext, devshare_resv_on(c))) return e;
  HIP_TRY(hipSetDevice(c->device));
  if (n_pods > c->pods_cap) {
    if (c->d_pods) HIP_TRY(hipFree(c->d_pods));
    if (c->d_out) HIP_TRY(hipFree(c->d_out));
    if (c->d_cpus) HIP_TRY(hipFree(c->d_cpus));
    if (c->d_devout) HIP_TRY(hipFree(c->d_devout));
    c->d_pods = nullptr;
    c->d_out = nullptr;
    c->d_cpus = nullptr;
    c->d_devout = nullptr;
    // +16 records of padding: the resolve kernel DMA-copies pod records in 1 KiB pieces
    HIP_TRY(hipMalloc(&c->d_pods, (size_t)(n_pods + 16) * sizeof(kh::DevPod)));
    HIP_TRY(hipMalloc(&c->d_out, (size_t)n_pods * sizeof(int32_t)));
    if (c->numa) HIP_TRY(hipMalloc(&c->d_cpus, (size_t)std::max(n_pods, 1) * KOORDHIP_NUMA_WORDS * sizeof(uint64_t)));
    c->pods_cap = n_pods;
  }
  if (n_pods) HIP_TRY(hipMemcpyAsync(c->d_pods, hp.data(), (size_t)n_pods * sizeof(kh::DevPod), hipMemcpyHostToDevice, c->stream));
  if (int e = stage_classes(c, hp)) return e;
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->n_staged = n_pods;
  c->staged_dsr = devshare_resv_on(c);
  c->podx_staged = false;
  c->staged_ext = false;
  c->staged_ext_dev = false;
  c->ext_idx.clear();
  c->staged_reserve = reserve;
  // prod LSE / LSR pods that bind no CPUs but some reservation may match (see
  // KOORDHIP_POD_CPUSET_QOS): checked against the snapshot at place time
  c->staged_qos_nonbind = false;
  for (int32_t j = 0; j < n_pods && !c->staged_qos_nonbind; j++)
    c->staged_qos_nonbind = (pods[j].flags & KOORDHIP_POD_CPUSET_QOS) && pods[j].resv_match != 0 &&
                            !(pods[j].flags & (KOORDHIP_POD_CPUSET | KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
  return 0;
}

int koordhip_stage_pods(koordhip_ctx *c, const koordhip_pod *pods, int32_t n_pods) {
  return stage_pods_impl(c, pods, n_pods, nullptr);
}

// DeviceShare PreFilter products (PreparePod, deviceshare/plugin.go:162-182) validated
static int check_pod_ext(const koordhip_pod_ext *x, int32_t n, bool *any) {
  *any = false;
  for (int32_t j = 0; j < n; j++) {
    const koordhip_pod_ext &e = x[j];
    if (e.flags & ~(uint32_t)KOORDHIP_PODX_DEVICE) return fail(KOORDHIP_EINVAL, "unknown koordhip_pod_ext flag");
    if (e.xmask >> KOORDHIP_NXRES) return fail(KOORDHIP_EINVAL, "koordhip_pod_ext.xmask beyond KOORDHIP_NXRES");
    for (int t = 0; t < KOORDHIP_DEV_TYPES; t++)
      for (int r = 0; r < KOORDHIP_DEV_RES; r++)
        if (e.dev_req[t][r] < -1 || e.dev_req[t][r] >= (1ll << 45))
          return fail(KOORDHIP_EINVAL, "koordhip_pod_ext device request out of range");
    if ((e.flags & KOORDHIP_PODX_DEVICE) && e.dev_req[KOORDHIP_DEV_GPU][1] < 0 && e.dev_req[KOORDHIP_DEV_GPU][2] < 0 &&
        e.dev_req[KOORDHIP_DEV_GPU][0] > 0)
      return fail(KOORDHIP_EINVAL, "a GPU request needs gpu-memory-ratio or gpu-memory (ValidDeviceResourceCombinations)");
    if (e.pts_n > KOORDHIP_PTS_POD || e.pts_class >= KOORDHIP_PTS_CLASSES)
      return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: more than KOORDHIP_PTS_POD constraints or a spread class out of range");
    for (int j = 0; j < e.pts_n; j++)
      if (e.pts_c[j] >= KOORDHIP_PTS_CONS || e.pts_skew[j] < 1 || (e.pts_fl[j] & ~(KOORDHIP_PTS_HARD | KOORDHIP_PTS_SELF)))
        return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: a topology spread constraint out of range");
    if (e.ipa_flags & ~(uint32_t)KOORDHIP_IPA_SELF) return fail(KOORDHIP_EINVAL, "unknown koordhip_pod_ext.ipa_flags bit");
    for (int q = 0; q < KOORDHIP_IPA_ENTRIES; q++)
      if (((e.ipa_score >> q) & 1u) != (e.ipa_w[q] != 0 ? 1u : 0u))
        return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: ipa_score must be exactly the entries with a nonzero ipa_w");
    *any = *any || e.flags != 0 || e.xmask != 0 || e.pts_n != 0 || e.pts_match != 0 ||
           (e.ipa_inc | e.ipa_aff | e.ipa_anti | e.ipa_score) != 0;
  }
  return 0;
}

// the pods' InterPodAffinity entries against the loaded snapshot's; the raw
// Score must stay in int32 (sum of |w| x the most pods an entry can count)
static int check_pod_ipa(const koordhip_ctx *c, const koordhip_pod_ext *x, int32_t n) {
  const uint32_t valid = c->ipa.ents >= 32 ? ~0u : ((1u << std::max(0, c->ipa.ents)) - 1u);
  for (int32_t j = 0; j < n; j++) {
    if ((x[j].ipa_inc | x[j].ipa_aff | x[j].ipa_anti | x[j].ipa_score) & ~valid)
      return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: an InterPodAffinity entry beyond the snapshot's ipa_ents");
    int64_t wsum = 0;
    for (int q = 0; q < KOORDHIP_IPA_ENTRIES; q++) wsum += std::abs((int64_t)x[j].ipa_w[q]);
    if (wsum * (c->ipa_pods_bound + n) >= (1ll << 31))
      return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: InterPodAffinity weights x counts could overflow int32");
  }
  return 0;
}

// the pods' topology spread constraints against the loaded snapshot's tables
static int check_pod_pts(const koordhip_ctx *c, const koordhip_pod_ext *x, int32_t n) {
  if (int e = check_pod_ipa(c, x, n)) return e;
  if (c->pts.keys <= 0) return 0;
  for (int32_t j = 0; j < n; j++) {
    if (x[j].pts_n && x[j].pts_class >= c->pts.classes)
      return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: spread class beyond the snapshot's pts_classes");
    for (int q = 0; q < x[j].pts_n; q++)
      if (x[j].pts_c[q] >= c->pts.cons)
        return fail(KOORDHIP_EINVAL, "koordhip_pod_ext: constraint beyond the snapshot's pts_cons");
  }
  return 0;
}

static int stage_ext(koordhip_ctx *c, const koordhip_pod_ext *ext, int32_t n_pods) {
  c->podx_staged = false;
  if (!ext || n_pods <= 0) return 0;
  bool any = false, rn = false;
  if (int e = check_pod_ext(ext, n_pods, &any)) return e;
  if (int e = check_pod_pts(c, ext, n_pods)) return e;
  for (int32_t j = 0; j < n_pods; j++) {
    if (ext[j].reserve_node < 0 || ext[j].reserve_node > c->n)
      return fail(KOORDHIP_EINVAL, "koordhip_pod_ext.reserve_node out of [0, n]");
    rn = rn || ext[j].reserve_node != 0;
  }
  if (any && !c->seq_profile)
    return fail(KOORDHIP_EINVAL, "device / extended-scalar pod requests need DeviceShare in the profile");
  c->staged_ext = any;
  // the pods with content; device / extended-scalar content only: they can be
  // placed inside the pipelined greedy (KH_POD_EXT marks them)
  bool devonly = any;
  for (int32_t j = 0; j < n_pods && any; j++) {
    const koordhip_pod_ext &e = ext[j];
    const bool spread = e.pts_n != 0 || e.pts_match != 0 || (e.ipa_inc | e.ipa_aff | e.ipa_anti | e.ipa_score) != 0;
    if (e.flags != 0 || e.xmask != 0 || spread) c->ext_idx.push_back(j);
    devonly = devonly && !spread;
  }
  if (!any && !rn) return 0;
  if (n_pods > c->podx_cap) {
    if (c->d_podx) HIP_TRY(hipFree(c->d_podx));
    c->d_podx = nullptr;
    HIP_TRY(hipMalloc(&c->d_podx, (size_t)n_pods * sizeof(kh::DevPodX)));
    c->podx_cap = n_pods;
  }
  HIP_TRY(hipMemcpyAsync(c->d_podx, ext, (size_t)n_pods * sizeof(kh::DevPodX), hipMemcpyHostToDevice, c->stream));
  if (devonly && !c->ext_idx.empty()) {
    const int32_t ne = (int32_t)c->ext_idx.size();
    if (ne > c->ext_idx_cap) {  // [ext_idx | needc] (needc: per place call, for its P / lag)
      if (c->d_ext_idx) HIP_TRY(hipFree(c->d_ext_idx));
      c->d_ext_idx = nullptr;
      HIP_TRY(hipMalloc(&c->d_ext_idx, (size_t)2 * ne * sizeof(int32_t)));
      c->ext_idx_cap = ne;
    }
    HIP_TRY(hipMemcpyAsync(c->d_ext_idx, c->ext_idx.data(), (size_t)ne * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(kh::launch_mark_ext(c->d_pods, c->d_ext_idx, ne, c->stream));
    c->staged_ext_dev = true;
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->podx_staged = true;
  return 0;
}

int koordhip_stage_pods_ext(koordhip_ctx *c, const koordhip_pod *pods, const koordhip_pod_ext *ext, int32_t n_pods) {
  // the nodeName pin (reserve_node) belongs to reserve pods only: elsewhere it
  // would be silently ignored
  if (pods && ext)
    for (int32_t j = 0; j < n_pods; j++)
      if (ext[j].reserve_node != 0 && !(pods[j].flags & KOORDHIP_POD_RESERVE))
        return fail(KOORDHIP_EINVAL, "koordhip_pod_ext.reserve_node set on a pod without KOORDHIP_POD_RESERVE");
  if (int e = stage_pods_impl(c, pods, n_pods, ext)) return e;
  return stage_ext(c, ext, n_pods);
}

int koordhip_place_stream_ext(koordhip_ctx *c, const koordhip_pod *pods, const koordhip_pod_ext *ext, int32_t n_pods,
                              int32_t *out_node) {
  if (int e = koordhip_stage_pods_ext(c, pods, ext, n_pods)) return e;
  if (int e = koordhip_place_staged(c)) return e;
  return koordhip_fetch_placements(c, out_node, n_pods);
}

int koordhip_fetch_devices(koordhip_ctx *c, uint32_t *slots, int32_t n_pods) {
  if (!c || (!slots && n_pods > 0)) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (n_pods > c->n_staged) return fail(KOORDHIP_EINVAL, "n_pods exceeds the staged stream");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (int e = pipe_status(c)) return e;
  const size_t b = (size_t)n_pods * KOORDHIP_DEV_TYPES * sizeof(uint32_t);
  if (!c->d_devout) {
    if (b) std::memset(slots, 0, b);
    return 0;
  }
  if (b) HIP_TRY(hipMemcpy(slots, c->d_devout, b, hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_read_devices(koordhip_ctx *c, int64_t *dev_used, int64_t *xrequested) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t nd = (size_t)c->n * KOORDHIP_DEV_TYPES * c->d.dv.slots * KOORDHIP_DEV_RES;
  if (dev_used && nd) {
    if (c->d.dv.used) {
      HIP_TRY(hipMemcpy(dev_used, c->d.dv.used, nd * sizeof(int64_t), hipMemcpyDeviceToHost));
    } else {
      std::memset(dev_used, 0, nd * sizeof(int64_t));
    }
  }
  const size_t nx = (size_t)c->n * KOORDHIP_NXRES;
  if (xrequested) {
    if (c->d.dv.xreq) {
      HIP_TRY(hipMemcpy(xrequested, c->d.dv.xreq, nx * sizeof(int64_t), hipMemcpyDeviceToHost));
    } else {
      std::memset(xrequested, 0, nx * sizeof(int64_t));
    }
  }
  return 0;
}

int koordhip_read_ipa(koordhip_ctx *c, int32_t *cnt) {
  if (!c || !cnt) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t nb = (size_t)c->n * std::max(0, c->ipa.ents) * sizeof(int32_t);
  if (!c->ipa.cnt || !nb) return 0;
  HIP_TRY(hipMemcpy(cnt, c->ipa.cnt, nb, hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_read_pts(koordhip_ctx *c, int32_t *cnt) {
  if (!c || !cnt) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t nb = (size_t)c->n * std::max(0, c->pts.cons) * sizeof(int32_t);
  if (!c->pts.cnt || !nb) return 0;
  HIP_TRY(hipMemcpy(cnt, c->pts.cnt, nb, hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_eval_ext(koordhip_ctx *c, const koordhip_pod *pods, const koordhip_pod_ext *ext, int32_t n_pods,
                      uint16_t *status, int32_t *scores, koordhip_topk *topk, int32_t k) {
  if (!c || (!pods && n_pods > 0)) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (n_pods < 0) return fail(KOORDHIP_EINVAL, "n_pods < 0");
  if (topk && (k < 1 || k > kMaxBatch)) return fail(KOORDHIP_EINVAL, "k must be in [1, 64]");
  if (n_pods == 0) return 0;
  bool any = false;
  if (ext) {
    if (int e = check_pod_ext(ext, n_pods, &any)) return e;
    if (int e = check_pod_pts(c, ext, n_pods)) return e;
  }
  if (any && !c->seq_profile)
    return fail(KOORDHIP_EINVAL, "device / extended-scalar pod requests need DeviceShare in the profile");
  bool reserve = false;
  if (int e = check_reserve_pods(c, pods, n_pods, &reserve)) return e;
  if (!c->seq && !reserve) {
    // the per-node plugins only: koordhip_eval, its planes widened
    const int32_t n = c->n;
    const int NPX = KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS;
    std::vector<int32_t> sc(scores ? (size_t)n_pods * KOORDHIP_NPLUGINS * n : 0);
    std::vector<uint8_t> st8(status ? (size_t)n_pods * n : 0);
    if (int e = koordhip_eval(c, pods, n_pods, status ? st8.data() : nullptr, scores ? sc.data() : nullptr, topk, k))
      return e;
    for (size_t q = 0; q < st8.size(); q++) status[q] = st8[q];
    if (scores)
      for (int32_t p = 0; p < n_pods; p++) {
        std::memcpy(scores + (size_t)p * NPX * n, sc.data() + (size_t)p * KOORDHIP_NPLUGINS * n,
                    (size_t)KOORDHIP_NPLUGINS * n * sizeof(int32_t));
        std::memset(scores + ((size_t)p * NPX + KOORDHIP_NPLUGINS) * n, 0, (size_t)KOORDHIP_NEXT_PLUGINS * n * sizeof(int32_t));
      }
    return 0;
  }
  HIP_TRY(hipSetDevice(c->device));
  const int32_t n = c->n;
  const int NPX = KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS;
  const int32_t per = std::max<int32_t>(1, std::min<int32_t>(kMaxBatch, (int32_t)((256ll << 20) / (48ll * std::max(n, 1)))));
  kh::DevPod *dp = nullptr;
  kh::DevPodX *dx = nullptr;
  uint8_t *dst = nullptr, *dist = nullptr;
  int32_t *dsc4 = nullptr, *dsc = nullptr, *work = nullptr;
  uint64_t *dk = nullptr;
  auto cleanup = [&]() {
    for (void *p : {(void *)dp, (void *)dx, (void *)dst, (void *)dist, (void *)dsc4, (void *)dsc, (void *)work, (void *)dk})
      if (p) (void)hipFree(p);
  };
  std::vector<kh::DevPod> hp;
  if (int ce = to_dev_pods(pods, n_pods, hp, ext, devshare_resv_on(c))) return ce;
  if (hipMalloc(&dp, (size_t)per * sizeof(kh::DevPod)) != hipSuccess ||
      (ext && hipMalloc(&dx, (size_t)per * sizeof(kh::DevPodX)) != hipSuccess) ||
      hipMalloc(&dst, (size_t)per * std::max(n, 1)) != hipSuccess ||
      hipMalloc(&dist, (size_t)per * std::max(n, 1)) != hipSuccess ||
      hipMalloc(&dsc4, (size_t)per * KOORDHIP_NPLUGINS * std::max(n, 1) * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&dsc, (size_t)per * NPX * std::max(n, 1) * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&work, (size_t)per * kh::SEQ_WORK_PLANES * std::max(n, 1) * sizeof(int32_t)) != hipSuccess ||
      (topk && hipMalloc(&dk, (size_t)per * k * sizeof(uint64_t)) != hipSuccess)) {
    cleanup();
    return fail(KOORDHIP_ENOMEM, "eval buffers");
  }
  const int32_t rs = (c->dc.resv && (c->cfg.score_plugins & KOORDHIP_PLUGIN_RESERVATION)) ? 1 : 0;
  std::vector<uint64_t> hk(topk ? (size_t)per * k : 0);
  std::vector<uint8_t> h8(status ? (size_t)per * n : 0), hi8(status ? (size_t)per * n : 0);
  int e = 0;
  for (int32_t p0 = 0; p0 < n_pods && !e; p0 += per) {
    const int32_t np = std::min(per, n_pods - p0);
    if (hipMemcpyAsync(dp, hp.data() + p0, np * sizeof(kh::DevPod), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        (dx && hipMemcpyAsync(dx, ext + p0, np * sizeof(kh::DevPodX), hipMemcpyHostToDevice, c->stream) != hipSuccess)) {
      e = fail(KOORDHIP_EDEVICE, "copy pods");
      break;
    }
    if (hipMemsetAsync(dist, 0, (size_t)np * n, c->stream) != hipSuccess ||
        kh::launch_eval_full(c->dc, c->d, dp, np, dst, dsc4, c->stream) != hipSuccess ||
        hipMemcpy2DAsync(dsc, (size_t)NPX * n * sizeof(int32_t), dsc4, (size_t)KOORDHIP_NPLUGINS * n * sizeof(int32_t),
                         (size_t)KOORDHIP_NPLUGINS * n * sizeof(int32_t), np, hipMemcpyDeviceToDevice, c->stream) != hipSuccess ||
        kh::launch_seq_eval(c->dc, c->d, dp, dx, np, rs, dst, dist, dsc, work, topk ? k : 0, dk, c->pts, c->ipa,
                            c->stream) != hipSuccess) {
      e = fail(KOORDHIP_EDEVICE, "eval_ext launch");
      break;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
      e = fail(KOORDHIP_EDEVICE, "eval sync");
      break;
    }
    if (status) {
      if (hipMemcpy(h8.data(), dst, (size_t)np * n, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(hi8.data(), dist, (size_t)np * n, hipMemcpyDeviceToHost) != hipSuccess) {
        e = fail(KOORDHIP_EDEVICE, "copy status");
      } else {
        for (size_t q = 0; q < (size_t)np * n; q++)
          status[(size_t)p0 * n + q] = (uint16_t)(h8[q] | (hi8[q] ? KOORDHIP_ST_IPA_FAIL : 0u));
      }
    }
    if (!e && scores &&
        hipMemcpy(scores + (size_t)p0 * NPX * n, dsc, (size_t)np * NPX * n * sizeof(int32_t), hipMemcpyDeviceToHost) !=
            hipSuccess)
      e = fail(KOORDHIP_EDEVICE, "copy scores");
    if (!e && topk) {
      if (hipMemcpy(hk.data(), dk, (size_t)np * k * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) {
        e = fail(KOORDHIP_EDEVICE, "copy topk");
        break;
      }
      for (size_t j = 0; j < (size_t)np * k; j++) {
        koordhip_topk &o = topk[(size_t)p0 * k + j];
        const uint64_t x = hk[j];
        o.node = x ? (int32_t)(0xFFFFFFFFu - (uint32_t)x) : -1;
        o.score = x ? (int32_t)(x >> 32) - 1 : 0;
      }
    }
  }
  cleanup();
  return e;
}

}  // extern "C"

namespace {

// the gather buffer of evaluation stream `slot` ([world][batch][k] each)
uint64_t *gather_buf(koordhip_ctx *c, int slot) {
  return c->d_gather + (size_t)slot * c->gather_world * ((size_t)kMaxBatch * 2 * kMaxBatch);
}

// All-gather of the per-shard lists of one round: RCCL, or for a local group
// a device-to-device pull of every member's list after its eval finished
// (events + host barrier), then a second barrier so no member overwrites its
// list before every peer has copied it.
// With two evaluation streams, the rounds of stream `slot` exchange on their
// own communicator (comm / comm2: every rank issues each communicator's
// all-gathers in the same round order) into their own gather buffer.
int exchange(koordhip_ctx *c, const uint64_t *lists, size_t count, int slot, hipStream_t es) {
  if (c->comm) {
    if (c->world == 1 && std::getenv("KOORDHIP_EXCH_MEMCPY")) {  // diagnostics: RCCL's one-rank all-gather as a plain copy
      HIP_TRY(hipMemcpyAsync(gather_buf(c, slot), lists, count * sizeof(uint64_t), hipMemcpyDeviceToDevice, es));
      return 0;
    }
    NCCL_TRY(ncclAllGather(lists, gather_buf(c, slot), count, ncclUint64, slot ? c->comm2 : c->comm, es));
    return 0;
  }
  LocalGroup &g = *c->group;
  c->d_cur_lists = lists;
  HIP_TRY(hipEventRecord(c->ev_part, c->stream));
  if (!g.barrier()) return fail(KOORDHIP_ECOMM, "local group aborted by a peer");
  for (int32_t j = 0; j < g.world; j++) {
    koordhip_ctx *p = g.ctx[j];
    if (p != c) HIP_TRY(hipStreamWaitEvent(c->stream, p->ev_part, 0));
    HIP_TRY(hipMemcpyAsync(c->d_gather + (size_t)j * count, p->d_cur_lists, count * sizeof(uint64_t),
                           hipMemcpyDefault, c->stream));
  }
  HIP_TRY(hipEventRecord(c->ev_copy, c->stream));
  if (!g.barrier()) return fail(KOORDHIP_ECOMM, "local group aborted by a peer");
  for (int32_t j = 0; j < g.world; j++)
    if (g.ctx[j] != c) HIP_TRY(hipStreamWaitEvent(c->stream, g.ctx[j]->ev_copy, 0));
  return 0;
}

// Members of a local group must agree on the stream before the first round,
// or the per-round barriers would never match up.
int group_agree(koordhip_ctx *c) {
  LocalGroup &g = *c->group;
  const int64_t key = ((int64_t)c->n << 40) ^ ((int64_t)c->n_staged << 8) ^ c->batch;
  g.keys[c->rank] = key;
  if (!g.barrier()) return fail(KOORDHIP_ECOMM, "local group aborted by a peer");
  for (int32_t j = 0; j < g.world; j++)
    if (g.keys[j] != key) return fail(KOORDHIP_EINVAL, "local group members disagree on snapshot size, stream or batch");
  return 0;
}

int place_staged_impl(koordhip_ctx *c);
int pmc_replay(koordhip_ctx *c);

// every CU of the device as a hipExtStreamCreateWithCUMask mask
std::vector<uint32_t> full_cu_mask(const koordhip_ctx *c) {
  std::vector<uint32_t> m((size_t)(c->n_cu + 31) / 32, 0xffffffffu);
  if (c->n_cu % 32) m.back() &= (1u << (c->n_cu % 32)) - 1u;
  return m;
}

}  // namespace

extern "C" {

int koordhip_place_staged(koordhip_ctx *c) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (c->n_staged > 0 && c->staged_dsr != devshare_resv_on(c))
    return fail(KOORDHIP_ESTATE, "the pods were staged under a snapshot with(out) reservations; stage them again");
  int e = place_staged_impl(c);
  if (e && c->group) c->group->abort();
  if (!e && std::getenv("KOORDHIP_PMC_REPLAY") && std::getenv("KOORDHIP_SERIAL")) e = pmc_replay(c);
  return e;
}

}  // extern "C"

namespace {

// The exact sequential cycle (seq.hip): one persistent cooperative launch,
// one block per CU, pod by pod.  The granules restart at epoch 1 every call.
int seq_place(koordhip_ctx *c) {
  const int32_t np = c->n_staged;
  if (c->world > 1 || c->comm || c->group)
    return fail(KOORDHIP_EINVAL, "the sequential cycle (DeviceShare / normalized Scores) runs on one GPU only");
  const int32_t G = c->n_cu;
  if ((int64_t)G * 256 * 8 < c->n) return fail(KOORDHIP_EINVAL, "too many nodes for the sequential cycle's grid");
  const size_t gbytes = kh::seq_granule_bytes(G);
  if (!c->d_seqg) {
    HIP_TRY(hipMalloc(&c->d_seqg, gbytes));
    c->seq_grid = G;
  }
  const bool dev = ((c->cfg.filter_plugins | c->cfg.score_plugins) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  if (dev && !c->d_devout && c->pods_cap > 0)
    HIP_TRY(hipMalloc(&c->d_devout, (size_t)c->pods_cap * KOORDHIP_DEV_TYPES * sizeof(uint32_t)));
  uint32_t *tmo = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(c->d_seqg) + kh::seq_tmo_offset(G));
  HIP_TRY(hipMemsetAsync(c->d_seqg, 0, gbytes, c->stream));
  const int32_t rs = (c->dc.resv && (c->cfg.score_plugins & KOORDHIP_PLUGIN_RESERVATION)) ? 1 : 0;
  const bool stamps = std::getenv("KOORDHIP_STAMPS") != nullptr;
  if (stamps) {
    if (!c->d_dbg) HIP_TRY(hipMalloc(&c->d_dbg, 128 * sizeof(uint64_t)));
    HIP_TRY(hipMemsetAsync(c->d_dbg, 0, 64 * sizeof(uint64_t), c->stream));
  }
  HIP_TRY(hipEventRecord(c->t0, c->stream));
  if (!c->d_seqdesc) HIP_TRY(hipMalloc(&c->d_seqdesc, kh::seq_desc_bytes()));
  HIP_TRY(kh::launch_seq(c->dc, c->d, c->d_pods, c->podx_staged ? c->d_podx : nullptr, np, G, c->d_seqg, tmo,
                         c->d_out, c->d_cpus, dev ? c->d_devout : nullptr, rs, stamps ? c->d_dbg : nullptr,
                         c->d_seqdesc, c->pts, c->ipa, c->stream));
  HIP_TRY(hipEventRecord(c->t1, c->stream));
  if (stamps) {
    uint64_t h[9];
    HIP_TRY(hipMemcpyAsync(h, c->d_dbg, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const double q = 1.0 / std::max(np, 1);
    std::fprintf(stderr, "[koordhip stamps] k_seq block 0 cycles per pod: evaluate %.0f  wait A %.0f  normalize+publish %.0f  "
                 "wait B %.0f  commit barrier %.0f | owner commits %.0f | evaluate split: pod prep %.0f  node "
                 "evaluation %.0f  reduce + publish %.0f\n", h[0] * q, h[1] * q, h[2] * q, h[3] * q,
                 h[4] * q, h[5] * q, h[6] * q, h[7] * q, h[8] * q);
  }
  c->last_P = 1;
  c->last_lag = 0;
  c->last_evals = (int64_t)np * c->n;
  c->last_launches = 1;
  c->ev_used = 0;
  c->eval_kernel = kh::seq_kernel_name(c->dc, c->d);
  c->resolve_kernel = c->eval_kernel;
  c->pipe_check = true;
  return 0;
}

// The class-incremental lists' plan of the staged batch for (P, lag): the
// builds (batches by round) and each class's schedule.  A class is (re)built
// when a round needs it and its current build is too old: lists of round u
// apply the log rounds [tb, u - lag) of a build on the state after round
// tb - 1, each round can move at most P of its keys out of the valid range, so
// a build stays valid for amax = (kClsTarget - K) / P log rounds (at least K
// valid keys remain).  A round that needs a build rebuilds, in the same batch,
// every class whose build would expire within the next amax / 2 rounds (few
// large batches: a build launch costs the same for 1 or 64 classes).  A
// build for round u is enqueued kClsLead rounds ahead, on the state the lists
// of round u - kClsLead see.  Class c's workgroup switches to the newest
// build of c whose batch round is <= the round it is at (skipping builds it
// never needed); a build overwrites the buffer slot of the class's build two
// before it, so it waits until the workgroup copied the last build of that
// slot it loads (bw, in switches; builds of a class alternate slots).
constexpr int32_t kClsLead = 12;

static int cls_plan(koordhip_ctx *c, int32_t P, int32_t lag, int32_t K) {
  if (c->plan_ok && c->plan_P == P && c->plan_lag == lag) return 0;
  const auto tp0 = std::chrono::steady_clock::now();
  const int32_t total = c->n_staged, rounds = (total + P - 1) / P, nc = (int32_t)c->cls_rep.size();
  const int32_t amax = (kh::kClsTarget - K) / P, horizon = amax / 2;
  c->plan_ok = false;
  c->plan_builds.clear();
  c->plan_ent.clear();
  c->plan_bm.clear();
  c->plan_bw.clear();
  c->plan_bpods.clear();
  std::vector<int32_t> valid(nc, -1), nb(nc, 0), seen(nc, -1);
  std::vector<std::vector<std::pair<int32_t, int32_t>>> builds(nc);  // per class (batch round, entry index)
  std::vector<std::vector<int32_t>> apps(nc);                         // per class the rounds it appears in
  for (int32_t u = 0; u < rounds; u++) {
    const int32_t p0 = u * P, np = std::min(P, total - p0);
    koordhip_ctx::ClsBuild b{u, std::max(0, u - kClsLead), 0, (int32_t)c->plan_ent.size(), 0};
    b.tb = std::max(0, b.er - lag);
    bool need = false;
    for (int32_t j = 0; j < np && !need; j++) need = valid[c->pod_cls[p0 + j]] < u;
    if (need)
      for (int32_t cl = 0; cl < nc; cl++)
        if (valid[cl] < u + horizon) {
          valid[cl] = b.tb + lag + amax;
          nb[cl]++;
          builds[cl].push_back({u, (int32_t)c->plan_ent.size()});
          c->plan_ent.push_back((cl << 1) | ((nb[cl] - 1) & 1));
          c->plan_bm.push_back(nb[cl]);
          c->plan_bw.push_back(0);
          c->plan_bpods.push_back(c->cls_rep[cl]);
          b.ne++;
        }
    if (b.ne) c->plan_builds.push_back(b);
    for (int32_t j = 0; j < np; j++) {
      const int32_t cl = c->pod_cls[p0 + j];
      if (seen[cl] == u) continue;
      seen[cl] = u;
      apps[cl].push_back(u);
    }
  }
  // schedules: switch at an appearance when a newer build's batch round has
  // come; the switch count at which each loaded build was copied
  c->plan_coff.assign(nc + 1, 0);
  c->plan_csched.clear();
  c->plan_csm.clear();
  for (int32_t cl = 0; cl < nc; cl++) {
    c->plan_coff[cl] = (int32_t)c->plan_csched.size();
    const auto &bl = builds[cl];
    std::vector<int32_t> loaded_at(bl.size() + 1, 0);  // build m -> the switch that copied it (0: never)
    int32_t cur = 0, nsw = 0;
    size_t bi = 0;
    for (int32_t u : apps[cl]) {
      while (bi < bl.size() && bl[bi].first <= u) bi++;
      const int32_t latest = (int32_t)bi;  // builds 1 .. bi have batch rounds <= u
      if (latest != cur) {
        cur = latest;
        loaded_at[cur] = ++nsw;
        c->plan_csched.push_back(u | (int32_t)0x80000000);
        c->plan_csm.push_back(cur);
      } else {
        c->plan_csched.push_back(u);
        c->plan_csm.push_back(0);
      }
    }
    for (size_t q = 0; q < bl.size(); q++) {
      const int32_t m = (int32_t)q + 1;
      int32_t w = 0;  // the newest loaded build of the same slot before m
      for (int32_t x = m - 2; x >= 1 && !w; x -= 2) w = loaded_at[x];
      c->plan_bw[bl[q].second] = w;
    }
  }
  c->plan_coff[nc] = (int32_t)c->plan_csched.size();
  // one device array for the schedule tables, the build tables and the sync words
  const size_t sz[8] = {c->plan_coff.size(), c->plan_csched.size(), c->plan_csm.size(), c->plan_ent.size(),
                        c->plan_bm.size(), c->plan_bw.size(), (size_t)nc, (((size_t)nc + 15) & ~(size_t)15) + kh::kClsRoundRing + 1 + (size_t)nc + 1};  // sw | rcnt ring, started, states, evc
  size_t tot = 0;
  for (int q = 0; q < 8; q++) {
    c->plan_off[q] = tot;
    tot += (sz[q] + 15) & ~(size_t)15;
  }
  if (tot > c->plan_cap) {
    if (c->d_plan) HIP_TRY(hipFree(c->d_plan));
    c->d_plan = nullptr;
    HIP_TRY(hipMalloc(&c->d_plan, tot * sizeof(int32_t)));
    c->plan_cap = tot;
  }
  const size_t np2 = std::max<size_t>(1, c->plan_bpods.size()) + 16;
  if (np2 > c->plan_pods_cap) {
    if (c->d_plan_pods) HIP_TRY(hipFree(c->d_plan_pods));
    c->d_plan_pods = nullptr;
    HIP_TRY(hipMalloc(&c->d_plan_pods, np2 * sizeof(kh::DevPod)));
    c->plan_pods_cap = np2;
  }
  const std::vector<int32_t> *src[6] = {&c->plan_coff, &c->plan_csched, &c->plan_csm, &c->plan_ent, &c->plan_bm,
                                        &c->plan_bw};
  for (int q = 0; q < 6; q++)
    if (!src[q]->empty())
      HIP_TRY(hipMemcpyAsync(c->d_plan + c->plan_off[q], src[q]->data(), src[q]->size() * sizeof(int32_t),
                             hipMemcpyHostToDevice, c->stream));
  if (!c->plan_bpods.empty())
    HIP_TRY(hipMemcpyAsync(c->d_plan_pods, c->plan_bpods.data(), c->plan_bpods.size() * sizeof(kh::DevPod),
                           hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->plan_ok = true;
  c->plan_P = P;
  c->plan_lag = lag;
  // (kernel stats: the host time of the staged batch's plan, made by its first place call)
  c->last_plan_us = (int32_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - tp0).count();
  return 0;
}

// buffers and build scratch of the class lists (before the persistent
// resolve is launched: an allocation later could wait behind it)
static int cls_alloc(koordhip_ctx *c, int32_t n) {
  const int32_t nc = (int32_t)c->cls_rep.size();
  if (nc > c->cls_cap) {
    if (c->d_cls_buf) HIP_TRY(hipFree(c->d_cls_buf));
    if (c->d_cls_meta) HIP_TRY(hipFree(c->d_cls_meta));
    c->d_cls_buf = nullptr;
    c->d_cls_meta = nullptr;
    HIP_TRY(hipMalloc(&c->d_cls_buf, (size_t)nc * 2 * kh::kClsCap * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&c->d_cls_meta, (size_t)nc * 2 * sizeof(kh::ClsMeta)));
    c->cls_cap = nc;
  }
  const int64_t stride = ((int64_t)n + 63) & ~63ll;
  const int32_t mstride = (kh::scan_chunks(c->partial_r, 0, n) + 63) & ~63;
  const size_t sb = (size_t)kh::kClsBuildRows * (stride + mstride) * sizeof(uint16_t) + 64;
  return ensure(c, &c->d_cls_S, &c->cls_S_cap, sb);
}

static kh::ClsSync cls_sync(koordhip_ctx *c, kh::PipeSync *sync) {
  kh::ClsSync cs;
  cs.sy = sync;
  cs.done = c->d_plan + c->plan_off[6];
  cs.sw = c->d_plan + c->plan_off[7];
  cs.rcnt = cs.sw + ((c->cls_rep.size() + 15) & ~(size_t)15);
  cs.evc = reinterpret_cast<uint32_t *>(cs.rcnt + kh::kClsRoundRing + 1 + c->cls_rep.size());
  return cs;
}

// One build batch on the build stream: every class of the batch evaluated on
// every node (k_scan), its buffer collected (k_cls_collect).
static int cls_build(koordhip_ctx *c, const koordhip_ctx::ClsBuild &b, kh::PipeSync *sync, hipStream_t bs, bool timed) {
  const int32_t n = c->n;
  if (b.tb > 0) HIP_TRY(kh::launch_wait_resolved(sync, b.tb, bs));
  const int64_t stride = ((int64_t)n + 63) & ~63ll;
  const int32_t mstride = (kh::scan_chunks(c->partial_r, 0, n) + 63) & ~63;
  uint16_t *S = reinterpret_cast<uint16_t *>(c->d_cls_S);
  uint16_t *Mx = S + (size_t)kh::kClsBuildRows * stride;
  const kh::ClsSync cs = cls_sync(c, sync);
  for (int32_t j = 0; j < b.ne; j += kh::kClsBuildRows) {
    const int32_t nb = std::min(kh::kClsBuildRows, b.ne - j);
    int32_t tm = -1;
    if (timed)
      if (int e = timed_begin(c, TK_SELECT, bs, &tm)) return e;
    HIP_TRY(kh::launch_scan(c->partial_r, c->dc, c->d, c->d_plan_pods + b.e0 + j, nb, 0, n, S, stride, Mx, mstride, 0, bs));
    HIP_TRY(kh::launch_cls_collect(S, stride, n, c->d_plan + c->plan_off[3] + b.e0 + j,
                                   c->d_plan + c->plan_off[4] + b.e0 + j, c->d_plan + c->plan_off[5] + b.e0 + j, nb,
                                   b.tb, c->d_cls_buf, c->d_cls_meta, cs, c->d_dbg ? c->d_dbg + 64 : nullptr, bs));
    if (int e = timed_end(c, tm, bs)) return e;
  }
  return 0;
}

// KOORDHIP_PMC_REPLAY (with KOORDHIP_SERIAL; for rocprofv3 --pmc, which
// serialises every dispatch, so the pipeline's persistent kernels cannot run
// beside each other): after a completed call, the class lists' builds
// (k_scan + k_cls_collect) and class workgroups (k_cls_run), and the device
// pods' pre-evaluations and finals, launched again one after another on the
// checkpointed snapshot state over the call's own commit log, with every wait
// satisfied in advance -- the pipeline's launches and grids, for their HBM
// counters (the state is the snapshot's, not each round's: the evaluations
// read the same columns, the class buffers change less).  The call's
// placements are kept; the node state is the checkpoint's plus the replayed
// device commits (the caller restores).  Diagnostics only.
int pmc_replay(koordhip_ctx *c) {
  if (c->last_seq && !(c->seq_profile && c->seq_ext_only && c->staged_ext_dev)) return 0;
  if (c->n_staged <= 0) return 0;
  HIP_TRY(hipStreamSynchronize(c->stream));
  // (a context that has only run the sequential cycle has no pipeline buffers: temporary ones)
  const size_t lbytes = (size_t)kMaxBatch * 2 * kMaxBatch * sizeof(uint64_t);
  int32_t *mod = c->d_mod;
  uint64_t *lists = c->d_lists;
  if (!mod) HIP_TRY(hipMalloc(&mod, (1 + kMaxBatch) * sizeof(int32_t) + kh::kPipeSyncBytes));
  if (!lists) HIP_TRY(hipMalloc(&lists, 4 * lbytes));
  if (int e = koordhip_restore(c)) return e;
  const int32_t total = c->n_staged;
  int32_t P = c->batch;
  int32_t lag = ((!c->side || c->resv) && !std::getenv("KOORDHIP_LAG1")) ? 2 : 1;
  if (lag == 2 && (3 * P > kh::kResolveMaxK || 2 * P > kMaxBatch)) lag = 1;
  const int nm = kh::side_mode(c->dc);
  while (P > 1 && kh::resolve_lds_bytes(P, (lag + 1) * P, c->n, nm, lag) > 157 * 1024) P--;
  const int32_t K = (lag + 1) * P, rounds = (total + P - 1) / P;
  const bool ext = c->seq_profile && c->seq_ext_only && c->staged_ext && c->staged_ext_dev && c->podx_staged &&
                   !c->staged_reserve && !c->seq_snap && !c->d.dv.rslot && nm == 0 && c->world == 1 &&
                   !c->ext_idx.empty();
  const bool cls = (!c->last_seq || ext) && !c->cls_rep.empty() && c->nbins <= 32768 && c->world == 1 &&
                   (int64_t)c->cls_rep.size() <= c->n_cu / 2 && kh::cls_run_lds(c->n, c->monotone) <= 150 * 1024 &&
                   (kh::kClsTarget - K) / P >= 4 * kClsLead + 2;
  int32_t *saved = nullptr;
  HIP_TRY(hipMalloc(&saved, (size_t)total * sizeof(int32_t)));
  HIP_TRY(hipMemcpyAsync(saved, c->d_out, (size_t)total * sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
  kh::PipeSync *sync = reinterpret_cast<kh::PipeSync *>(mod + 1 + kMaxBatch);
  HIP_TRY(hipMemsetAsync(sync, 0, kh::kPipeSyncBytes, c->stream));
  const int32_t big = 0x3fffffff;
  const int32_t head[3] = {big, big, rounds};  // sel[0], sel[1], res_round: every round published and resolved
  HIP_TRY(hipMemcpyAsync(sync, head, sizeof(head), hipMemcpyHostToDevice, c->stream));
  int32_t nscan = 0;
  if (cls) {
    if (int e = cls_plan(c, P, lag, K)) return e;
    if (int e = cls_alloc(c, c->n)) return e;
    const kh::ClsSync cs = cls_sync(c, sync);
    const size_t nc = c->cls_rep.size();
    HIP_TRY(hipMemsetAsync(c->d_plan + c->plan_off[6], 0,
                           (2 * ((nc + 15) & ~(size_t)15) + kh::kClsRoundRing + 1 + nc + 1) * sizeof(int32_t), c->stream));
    // every build's slot free and every build published before anything waits
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(cs.done), big, nc, c->stream));
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(cs.sw), big, nc, c->stream));
    for (const koordhip_ctx::ClsBuild &b : c->plan_builds) {
      if (int e = cls_build(c, b, sync, c->stream, false)) return e;
      nscan += (b.ne + kh::kClsBuildRows - 1) / kh::kClsBuildRows;
    }
    HIP_TRY(kh::launch_cls_run(c->dc, c->d, c->d_cls_pod, (int32_t)nc, c->d_plan + c->plan_off[0],
                               c->d_plan + c->plan_off[1], c->d_plan + c->plan_off[2], c->d_pod_cls, c->d_out, lag, P,
                               total, c->d_cls_buf, c->d_cls_meta, K, c->monotone, lists,
                               (int64_t)((size_t)kMaxBatch * 2 * kMaxBatch), cs, nullptr, c->stream));
  }
  const int32_t ne = (int32_t)c->ext_idx.size();
  if (ext) {
    if (!c->d_devout && c->pods_cap > 0)
      HIP_TRY(hipMalloc(&c->d_devout, (size_t)c->pods_cap * KOORDHIP_DEV_TYPES * sizeof(uint32_t)));
    const size_t xb = kh::ext_scratch_bytes(ne, c->n);
    if (xb > c->ext_scr_cap) {
      if (c->d_ext_scr) HIP_TRY(hipFree(c->d_ext_scr));
      c->d_ext_scr = nullptr;
      HIP_TRY(hipMalloc(&c->d_ext_scr, xb));
      c->ext_scr_cap = xb;
    }
    const char *ld = std::getenv("KOORDHIP_EXT_LEAD");
    const int32_t lead = std::max(lag, ld ? std::atoi(ld) : lag);
    HIP_TRY(kh::launch_ext_begin(c->d, ne, c->d_ext_scr, c->stream));
    for (int32_t e = 0; e < ne; e++) {
      const int32_t gp = c->ext_idx[e], u = gp / P;
      HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(reinterpret_cast<int32_t *>(sync) +
                                                                  kh::kPipeSyncExtReqWord),
                                gp + 1, 1, c->stream));
      HIP_TRY(kh::launch_ext_pre(c->dc, c->d, c->d_pods, c->d_podx, e, gp, u - lead, e, ne, c->d_ext_scr, sync,
                                 c->stream));
      HIP_TRY(kh::launch_ext_final(c->dc, c->d, c->d_pods, c->d_podx, e, gp, std::max(0, u - lead) * P,
                                   std::max(0, u - lag) * P, ne, c->d_ext_scr, c->d_out, c->d_devout, sync, nullptr,
                                   c->d_ext_idx, e, c->stream));
    }
  }
  HIP_TRY(hipMemcpyAsync(c->d_out, saved, (size_t)total * sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipFree(saved));
  int32_t err = 0;
  HIP_TRY(hipMemcpy(&err, reinterpret_cast<int32_t *>(sync) + kh::kPipeSyncErrWord, sizeof(err), hipMemcpyDeviceToHost));
  if (mod != c->d_mod) HIP_TRY(hipFree(mod));
  if (lists != c->d_lists) HIP_TRY(hipFree(lists));
  std::fprintf(stderr, "[koordhip pmc replay] P %d lag %d: class lists %s (%zu builds, %d k_scan + k_cls_collect "
               "launches, %d k_cls_run of %zu workgroups), device pods %d (k_ext_pre + k_ext_final each)%s\n", P, lag,
               cls ? "replayed" : "not used", cls ? c->plan_builds.size() : (size_t)0, nscan, cls ? 1 : 0,
               cls ? c->cls_rep.size() : (size_t)0, ext ? ne : 0, err ? ": ERROR (a replayed kernel gave up)" : "");
  if (err) return fail(KOORDHIP_EDEVICE, "PMC replay: a replayed kernel reported an error");
  return 0;
}

int place_staged_impl(koordhip_ctx *c) {
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  c->pipe_err = false;
  c->pipe_errc = 0;
  c->pipe_check = false;
  HIP_TRY(hipSetDevice(c->device));
  // the sequential cycle: a snapshot or profile that needs it, a reserve pod in
  // the batch, or an ext-record profile whose batch carries ext content.  An
  // empty record: DeviceShare's PreFilter skips the pod (Filter passes, Score 0,
  // no Reserve: deviceshare/plugin.go:162-182, scoring.go:33-40);
  // PodTopologySpread has no constraint (Filter passes; every Score 0, which
  // NormalizeScore turns into the same 100 on every node) and the pod counts
  // for none; InterPodAffinity has no term, no existing pod's term matches it
  // (Filter passes, Score 0 everywhere, normalised to 0) and it counts for no
  // entry -- nothing couples its nodes or changes the cycle's state.
  // Upstream restores the nominated reservation's reserved CPUs for every
  // AllowUseCPUSet pod (nodenumaresource/reservation.go:68-74), and on a
  // topology-policy or CPU-amplified node they enter the zone / amplified
  // Score and Reserve of a pod that binds none (plugin.go:465-479,
  // scoring.go:95-120): not modelled for such pods -- refused, not diverged
  if (c->staged_qos_nonbind && c->dc.resv_cpus && (c->dc.zones || c->dc.amp) &&
      (c->cfg.score_plugins & KOORDHIP_PLUGIN_RESERVATION))
    return fail(KOORDHIP_EINVAL, "a prod LSE/LSR pod binding no CPUs that a reservation may match, on a snapshot with "
                                 "reservations holding CPUs and topology-policy or CPU-amplified nodes: the reserved "
                                 "CPUs' restore for such pods is not modelled (KOORDHIP_POD_CPUSET_QOS)");
  // Device pods among pods without ext content (DeviceShare as the only
  // coupling plugin the records use, the plain plugin build, one GPU, the
  // persistent pipeline): placed inside the pipelined greedy -- the resolve
  // hands each one the exact state and k_ext_pre / k_ext_final run its reference cycle
  // (seq.hip) -- instead of the whole batch in the sequential cycle.
  // KOORDHIP_EXT_SEQ: the sequential cycle for such batches too (A/B).
  const bool ext_pipe = c->seq_profile && c->seq_ext_only && c->staged_ext && c->staged_ext_dev && c->podx_staged &&
                        !c->staged_reserve && !c->seq_snap && !c->d.dv.rslot && kh::side_mode(c->dc) == 0 && c->world == 1 &&
                        !c->comm && !c->group && !std::getenv("KOORDHIP_SERIAL") && !std::getenv("KOORDHIP_ROUND_LAUNCH") &&
                        !std::getenv("KOORDHIP_EXT_SEQ");
  c->last_ext_pipe = ext_pipe;
  c->last_seq = c->staged_reserve || c->seq_snap || (c->seq_profile && (!c->seq_ext_only || c->staged_ext) && !ext_pipe);
  if (c->last_seq) return seq_place(c);
  if (ext_pipe) {  // (allocations before the persistent launches: one later could wait behind them)
    if (!c->d_devout && c->pods_cap > 0)
      HIP_TRY(hipMalloc(&c->d_devout, (size_t)c->pods_cap * KOORDHIP_DEV_TYPES * sizeof(uint32_t)));
    const size_t xb = kh::ext_scratch_bytes((int32_t)c->ext_idx.size(), c->n);
    if (xb > c->ext_scr_cap) {
      if (c->d_ext_scr) HIP_TRY(hipFree(c->d_ext_scr));
      c->d_ext_scr = nullptr;
      HIP_TRY(hipMalloc(&c->d_ext_scr, xb));
      c->ext_scr_cap = xb;
    }
    if (!c->xstream) {
      // The device pods' streams: transient launches only (the pre-evaluations
      // behind one-workgroup waits on xstream, the finals spinning in their
      // own small grid between the previous final and their hand-off on
      // xstream2), two pooled streams created back to back (HIP deals pooled
      // streams over its queues in turn, so they get two).  Measured on
      // config4dsmix at lead 2: 114.2 ms per step; one stream for both
      // (KOORDHIP_EXT_ONE, A/B) 130.2 -- a pre-evaluation enqueued ahead of a
      // final keeps it from being resident before its hand-off (1,067 of 1,957
      // finals late); two CU-masked streams (KOORDHIP_EXT_DEDICATED, A/B) 114.2
      // but they add two hardware queues to the pipeline's three, and a lead-5
      // run stalled into the watchdog.
      if (std::getenv("KOORDHIP_EXT_DEDICATED")) {
        const std::vector<uint32_t> all = full_cu_mask(c);
        HIP_TRY(hipExtStreamCreateWithCUMask(&c->xstream, (uint32_t)all.size(), all.data()));
        HIP_TRY(hipExtStreamCreateWithCUMask(&c->xstream2, (uint32_t)all.size(), all.data()));
      } else {
        HIP_TRY(hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking));
        if (!std::getenv("KOORDHIP_EXT_ONE")) HIP_TRY(hipStreamCreateWithFlags(&c->xstream2, hipStreamNonBlocking));
      }
      if (std::getenv("KOORDHIP_EXT_ALT")) {
        HIP_TRY(hipStreamCreateWithFlags(&c->xstream3, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_ext3, hipEventDisableTiming));
      }
      HIP_TRY(hipEventCreateWithFlags(&c->ev_ext, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&c->ev_ext2, hipEventDisableTiming));
    }
  }
  // the pipelined greedy allocates no device but the device pods' (k_ext_final):
  // clear the slots a previous sequential batch left (koordhip_fetch_devices
  // reads this buffer)
  if (c->d_devout && c->n_staged > 0)
    HIP_TRY(hipMemsetAsync(c->d_devout, 0, (size_t)c->n_staged * KOORDHIP_DEV_TYPES * sizeof(uint32_t), c->stream));
  if (c->podx_staged && c->staged_ext && !ext_pipe)
    return fail(KOORDHIP_EINVAL, "device / extended-scalar pod requests need DeviceShare in the profile");
  // KOORDHIP_SERIAL (profiling under rocprofv3 --pmc, which serialises
  // dispatches): every launch on one stream in dependency order, one resolve
  // per round; the lists are then fresher than in the pipeline, which the
  // resolve treats exactly like refreshed entries.
  const bool serial = std::getenv("KOORDHIP_SERIAL") != nullptr;
  // KOORDHIP_FOLD_WAIT: the split select's merging workgroups hold the stream
  // until the resolve is far enough instead of a k_wait_resolved launch
  // (measured 2-3 % slower: their spinning delays the launch's end)
  const bool wait_kernel = std::getenv("KOORDHIP_FOLD_WAIT") == nullptr;
  const bool persistent = !serial && !c->group && !std::getenv("KOORDHIP_ROUND_LAUNCH");
  // A lone single-GPU context alternates the rounds between two evaluation
  // streams (each with its own score matrix and select buffers; the resolve
  // counts finished lists per round parity).
  // exchanged: node-sharded, or a one-rank RCCL communicator (the exchange
  // path end to end on one GPU: all-gather, merge, per-round signal)
  // A node-sharded rank (world > 1) whose batch the class-incremental lists
  // cover evaluates the full table itself: every rank holds the full replica
  // and resolves every pod anyway, and sharding divides only the evaluation,
  // which the class lists already took off the critical path -- through the
  // per-round all-gather world > 1 would run slower than one GPU (DESIGN.md
  // section 6).  KOORDHIP_SHARD_FORCE keeps the exchange (A/B).
  const bool cls_fit = !c->cls_rep.empty() && c->nbins <= 32768 && !std::getenv("KOORDHIP_CLS_OFF") && !c->cu_reserve &&
                       (int64_t)c->cls_rep.size() <= c->n_cu / 2 && kh::cls_run_lds(c->n, c->monotone) <= 150 * 1024;
  // (KOORDHIP_SHARD_LOCAL_SIM: a lone one-GPU context takes that decision as
  // if it were a rank of a sharded job -- the path's one-GPU test)
  const bool local_sim = c->world == 1 && !c->comm && std::getenv("KOORDHIP_SHARD_LOCAL_SIM") != nullptr;
  const bool local = (c->world > 1 || local_sim) && !c->group && persistent && c->sel_split && wait_kernel && cls_fit &&
                     !std::getenv("KOORDHIP_SHARD_FORCE");
  c->last_local = local;
  const bool exch = (c->world > 1 || c->comm != nullptr) && !local;
  // (node-sharded: the rounds of the second stream exchange on comm2)
  const bool two = persistent && (!exch || c->comm2) && c->sel_split && wait_kernel &&
                   !std::getenv("KOORDHIP_ONE_EVAL_STREAM");
  // class-incremental lists (cls.hip): the staged pods fall into few classes
  // (byte-identical records); the second stream then runs the class builds
  // (one persistent workgroup per class: every one resident, one per CU with
  // half the CUs to spare for the resolve and the builds; not beside the
  // KOORDHIP_CU_RESERVE A/B knob, whose masks were measured to stall 202
  // class workgroups)
  bool cls = two && !exch && !c->cls_rep.empty() && c->nbins <= 32768 && !std::getenv("KOORDHIP_CLS_OFF") &&
             !c->cu_reserve && (int64_t)c->cls_rep.size() <= c->n_cu / 2 &&
             kh::cls_run_lds(c->n, c->monotone) <= 150 * 1024;
  // Pipeline depth: round r's lists are evaluated on the state after round
  // r - 1 - lag.  Lag 2 (the default with the two evaluation streams) lets an
  // evaluation overlap two resolve rounds; the resolve then re-evaluates the
  // nodes of the last two rounds (k >= 3P).  Lag 1: k >= 2P.
  // pods per round: batch_pods, lowered until the resolve kernel's LDS holds
  // the round (NodeNUMAResource rows are large)
  int32_t P = c->batch;
  // (NodeNUMAResource streams are bound by the resolve's cpuset Reserve: the
  // longer re-evaluated set of lag 2 measured slower there, 87k vs 93k pods/s
  // (round 2), 149k vs 154k (round 3, config 3); the Reservation streams are
  // bound by the evaluation -- the period of a round is (eval + resolve) / 2 at
  // lag 1, / 3 at lag 2 -- and run lag 2: config 5 170k -> 182k pods/s in
  // spite of the shorter rounds the resolve's LDS then allows (24 -> 15 pods).
  // KOORDHIP_LAG2: lag 2 with NodeNUMAResource alone too.)
  int32_t lag = (two && (!c->side || c->resv || std::getenv("KOORDHIP_LAG2")) && !std::getenv("KOORDHIP_LAG1")) ? 2 : 1;
  if (lag == 2 && (3 * P > kh::kResolveMaxK || 2 * P > kMaxBatch)) lag = 1;  // M' spans 2 rounds <= 64 slots
  const int nm = kh::side_mode(c->dc);
  while (P > 1 && kh::resolve_lds_bytes(P, (lag + 1) * P, c->n, nm, lag) > 157 * 1024) P--;
  const int32_t K = (lag + 1) * P;
  if (cls && (kh::kClsTarget - K) / P < 4 * kClsLead + 2) cls = false;
  c->last_P = P;
  c->last_lag = lag;
  const size_t lbytes = (size_t)kMaxBatch * 2 * kMaxBatch * sizeof(uint64_t);
  if (!c->d_lists) {
    HIP_TRY(hipMalloc(&c->d_lists, 4 * lbytes));
    HIP_TRY(hipMalloc(&c->d_final, 4 * lbytes));
    HIP_TRY(hipMalloc(&c->d_mod, (1 + kMaxBatch) * sizeof(int32_t) + kh::kPipeSyncBytes));
    HIP_TRY(hipMalloc(&c->d_desc, sizeof(kh::DevNodes)));
    // The persistent resolve occupies its hardware queue for the whole call:
    // a CU-masked stream gets a dedicated queue (HIP pools plain streams over
    // GPU_MAX_HW_QUEUES queues, and an evaluation stream sharing the resolve's
    // queue would wait behind it forever).  KOORDHIP_CU_RESERVE: CU 0 only.
    if (c->cu_reserve) {
      const uint32_t m0 = c->cu_reserve;
      HIP_TRY(hipExtStreamCreateWithCUMask(&c->rstream, 1, &m0));
    } else {
      const std::vector<uint32_t> all = full_cu_mask(c);
      HIP_TRY(hipExtStreamCreateWithCUMask(&c->rstream, (uint32_t)all.size(), all.data()));
    }
    for (int i = 0; i < kRing; i++) HIP_TRY(hipEventCreateWithFlags(&c->ev_res[i], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
  }
  if (exch && (c->world > c->gather_world || !c->d_gather)) {
    if (c->d_gather) HIP_TRY(hipFree(c->d_gather));
    c->d_gather = nullptr;
    HIP_TRY(hipMalloc(&c->d_gather, 2 * (size_t)c->world * lbytes));
    c->gather_world = c->world;
  }
  if (kh::resolve_lds_bytes(P, K, c->n, nm, lag) > 157 * 1024)
    return fail(KOORDHIP_EINVAL, "snapshot too large for the resolve kernel's LDS");
  if (c->group)
    if (int e = group_agree(c)) return e;
  // profile_kernels: event pairs around the evaluation launches of at most
  // ~256 evenly spaced rounds (the per-kernel averages need no more; every
  // outstanding timed event holds a runtime signal, and a host thread that
  // runs out of them waits for the oldest -- possibly behind the persistent
  // resolve, which waits for rounds that thread has not enqueued yet)
  const int32_t tstride = std::max<int32_t>(1, (((c->n_staged + P - 1) / P) + 255) / 256);
  if (c->cfg.profile_kernels) {
    // every event pair of this call created now: hipEventCreate inside the
    // round loop could wait on a device that is busy with the persistent
    // resolve, which itself waits for rounds not yet enqueued
    const size_t nr = ((size_t)c->n_staged + P - 1) / P;  // rounds; per-round resolve launches are all timed
    const size_t want = (size_t)6 * ((persistent ? nr / tstride : nr) + 2) + 8;
    while (c->ev.size() < want) {
      hipEvent_t e;
      HIP_TRY(hipEventCreate(&e));
      c->ev.push_back(e);
    }
    c->ev_kind.resize(c->ev.size() / 2);
  }
  int32_t lo = 0, hi = c->n;
  if (!local) shard(c, &lo, &hi);
  c->ev_used = 0;
  c->last_launches = 0;
  c->last_evals = 0;
  c->last_exec = -1;  // -1: equal to last_evals (every pair evaluated once)
  c->last_ext_exec = 0;
  c->last_evc = c->last_reev = nullptr;
  if (std::getenv("KOORDHIP_STAMPS")) {
    if (!c->d_dbg) HIP_TRY(hipMalloc(&c->d_dbg, 128 * sizeof(uint64_t)));
    HIP_TRY(hipMemsetAsync(c->d_dbg, 0, 128 * sizeof(uint64_t), c->stream));
  }
  int32_t *mbuf = c->d_mod;  // M' handed between resolve launches
  kh::PipeSync *sync = reinterpret_cast<kh::PipeSync *>(c->d_mod + 1 + kMaxBatch);
  HIP_TRY(hipEventRecord(c->t0, c->stream));
  c->desc_host = c->d;  // the resolve kernel reads the column pointers from this device copy
  HIP_TRY(hipMemcpyAsync(c->d_desc, &c->desc_host, sizeof(kh::DevNodes), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemsetAsync(sync, 0, kh::kPipeSyncBytes, c->stream));
  HIP_TRY(hipEventRecord(c->ev_start, c->stream));
  HIP_TRY(hipStreamWaitEvent(c->rstream, c->ev_start, 0));
  // Round pipeline: round r's lists are evaluated (stream) while rounds
  // r-lag.. are resolved (rstream); round r's evaluation waits only for round
  // r-1-lag's commits.  Both sides synchronise through device flags (PipeSync).  A lone
  // context runs ONE persistent resolve launch for the whole stream (no
  // per-round launch or event latency on the sequential path); contexts of a
  // local group share hardware queues with their peers, so they launch one
  // resolve per round, enqueued after that round's lists (deadlock-free
  // whatever the stream -> queue mapping).
  const int32_t total = c->n_staged;
  const int32_t rounds = (total + P - 1) / P;
  hipStream_t rs = serial ? c->stream : c->rstream;
  const char *trace_env = std::getenv("KOORDHIP_TRACE_POD");  // diagnostics: printf one pod's resolve step
  const int32_t trace = trace_env ? std::atoi(trace_env) : -1;
  const int64_t list_buf = (int64_t)(lbytes / sizeof(uint64_t));
  uint64_t *lists0 = exch ? c->d_final : c->d_lists;
  uint64_t *cpus = c->d_cpus;
  if (two && !c->stream2) {
    std::vector<uint32_t> m = full_cu_mask(c);  // its own queue too (see rstream)
    if (c->cu_reserve) m[0] &= ~c->cu_reserve;
    HIP_TRY(hipExtStreamCreateWithCUMask(&c->stream2, (uint32_t)m.size(), m.data()));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_eval2, hipEventDisableTiming));
  }
  if (two) HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev_start, 0));
  if (cls && rounds > 0) {
    if (int e = cls_plan(c, P, lag, K)) return e;
    if (int e = cls_alloc(c, c->n)) return e;
    // the build / switch counters start every call at zero; the build stream sees them
    HIP_TRY(hipMemsetAsync(c->d_plan + c->plan_off[6], 0,
                           (2 * ((c->cls_rep.size() + 15) & ~(size_t)15) + kh::kClsRoundRing + 1 + c->cls_rep.size() + 1) *
                               sizeof(int32_t), c->stream));
    HIP_TRY(hipEventRecord(c->ev_start, c->stream));
    HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev_start, 0));
  }
  for (int slot = 0; slot < (two ? 2 : 1) && rounds > 0 && !cls; slot++) {
    hipStream_t es = slot ? c->stream2 : c->stream;
    if (int e = eval_buffers(c, std::min(P, total), lo, hi, slot, es, K)) return e;
    // the per-pod hand-off words start every call at zero (Guideline 16: a
    // call the watchdog stopped can leave them set); in-kernel resets keep
    // them zero between the rounds of a call
    if (c->eval_fused) HIP_TRY(hipMemsetAsync(c->d_etk_sync[slot], 0, 2 * kh::kSelMaxPods * sizeof(uint32_t), es));
  }
  int32_t res_tm = -1;
  if (persistent && rounds > 0) {
    int32_t tm = -1;
    if (int e = timed_begin(c, TK_RESOLVE, c->rstream, &tm)) return e;
    // (monotone bit 1: the chained decisions, wave 0 at the start of each
    // round's loop: they take the staged-conflict pods off the general path --
    // config 4: 16.0k -> 0.4k general-path pods, 75.0 -> 62.5 ms per step,
    // profiles/r05n_chain_ab.txt; KOORDHIP_CHAIN_OFF for A/B)
    // (bits 2-3: chain passes, 1 by default -- 1 / 2 / 3 passes measured 60.1 /
    // 60.5 / 61.0 ms per step on config 4, r05o; KOORDHIP_CHAIN_PASSES for A/B)
    const char *cp = std::getenv("KOORDHIP_CHAIN_PASSES");
    const int32_t mono = c->monotone | ((c->monotone && !std::getenv("KOORDHIP_CHAIN_OFF")) ? 2 : 0) |
                         (c->monotone ? (((cp ? std::atoi(cp) : 1) & 3) << 2) : 0);
    HIP_TRY(kh::launch_resolve(c->dc, c->d, c->d_desc, c->d_pods, total, P, K, 0, rounds, lists0, list_buf, mono, lag, sync,
                               mbuf, c->d_out, cpus, c->d_dbg, trace, c->rstream));
    c->resolve_kernel = kh::last_resolve_kernel();
    res_tm = tm;  // its end event is recorded after the round loop (nothing else runs on rstream)
  }

  if (cls && rounds > 0) {
    // ONE persistent workgroup per class for the whole stream (c->stream), the
    // builds on the second stream, all enqueued now (each build waits for its
    // state's round on the device)
    hipStream_t cs = c->stream;
    int32_t tm = -1;
    if (int e = timed_begin(c, TK_SCAN, cs, &tm)) return e;
    HIP_TRY(kh::launch_cls_run(c->dc, c->d, c->d_cls_pod, (int32_t)c->cls_rep.size(), c->d_plan + c->plan_off[0],
                               c->d_plan + c->plan_off[1], c->d_plan + c->plan_off[2], c->d_pod_cls, c->d_out, lag, P,
                               total, c->d_cls_buf, c->d_cls_meta, K, c->monotone, c->d_lists, list_buf,
                               cls_sync(c, sync), c->d_dbg ? c->d_dbg + 64 : nullptr, cs));
    if (int e = timed_end(c, tm, cs)) return e;
    for (const koordhip_ctx::ClsBuild &b : c->plan_builds)
      if (int e = cls_build(c, b, sync, c->stream2, b.u % tstride == 0)) return e;
    c->eval_kernel = kh::cls_run_kernel_name(c->dc);
    c->last_launches = 1;
    c->last_evals = (int64_t)total * c->n;  // every (pod, node) pair decided exactly (the lists' equivalent work)
    // executed: each build evaluates its classes over every node, the class
    // workgroups count their incremental re-evaluations on the device
    c->last_exec = 0;
    for (const koordhip_ctx::ClsBuild &b : c->plan_builds) c->last_exec += (int64_t)b.ne * c->n;
    c->last_evc = cls_sync(c, sync).evc;
  }
  if (ext_pipe && rounds > 0) {
    // The device pods: per pod e (round u) a pre-evaluation once the resolve
    // finished round u - lead (and the device commits of the device pods of
    // the rounds before that are published), and the exact placement at its
    // hand-off -- transient launches (streams: see their creation): the
    // pre-evaluations behind a one-workgroup wait on device flags on xstream,
    // the finals (with the device Reserve) on xstream2, spinning in their own grid
    // (seq.hip ext_spin: resident before the hand-off unless two device pods
    // come close together), after the call's PipeSync / device-slot resets
    // (ev_start).  They are submitted in an order whose every wait the
    // launches before it satisfy, so they cannot deadlock even where the two
    // streams share one in-order queue:
    // final(e) waits for the hand-off of e (round u: the lists of rounds <= u
    // and the finals of the device pods before e, all earlier), pre(e) and the
    // previous pod's Reserve; pre(e) waits for rounds < u - lead (the finals of
    // the device pods of those rounds come before it: a final of round u'
    // precedes a pre whose wait round exceeds u') and follows final(e - RING),
    // whose ring buffer it reuses.  lead: the rounds between lag and lead add
    // their commits, from the commit log, to the final's re-evaluated set.
    HIP_TRY(hipStreamWaitEvent(c->xstream, c->ev_start, 0));
    hipStream_t xs2 = c->xstream2 ? c->xstream2 : c->xstream;  // the finals' stream
    if (c->xstream2) HIP_TRY(hipStreamWaitEvent(c->xstream2, c->ev_start, 0));
    if (c->xstream3) HIP_TRY(hipStreamWaitEvent(c->xstream3, c->ev_start, 0));
    const char *ld = std::getenv("KOORDHIP_EXT_LEAD");
    const int32_t lead = std::max(lag, ld ? std::atoi(ld) : lag);
    const int32_t ne = (int32_t)c->ext_idx.size(), R = kh::ext_ring();
    const bool alt = c->xstream3 != nullptr;  // (KOORDHIP_EXT_ALT at the streams' creation)
    HIP_TRY(kh::launch_ext_begin(c->d, ne, c->d_ext_scr, c->xstream));
    c->last_ext_exec = (int64_t)ne * c->n;  // the pre-evaluations; the finals' re-evaluations on the device
    c->last_reev = kh::ext_reevals(c->d_ext_scr, ne, c->n);
    HIP_TRY(hipEventRecord(c->ev_ext, c->xstream));
    if (c->xstream2) HIP_TRY(hipStreamWaitEvent(c->xstream2, c->ev_ext, 0));  // (the zeroed flags)
    if (c->xstream3) HIP_TRY(hipStreamWaitEvent(c->xstream3, c->ev_ext, 0));
    auto u_of = [&](int32_t e) { return c->ext_idx[e] / P; };
    std::vector<int32_t> pre_needc(ne, 0);  // per device pod the device commits its pre-evaluation waited for
    for (int32_t ip = 0, ifn = 0, needc = 0; ifn < ne;) {
      const bool can_pre = ip < ne && ifn >= ip - R + 1;
      if (can_pre && (ip <= ifn || u_of(ip) - lead < u_of(ifn))) {
        while (needc < ip && u_of(needc) < u_of(ip) - lead) needc++;  // device pods of the rounds < u - lead
        pre_needc[ip] = needc;
        HIP_TRY(kh::launch_ext_pre(c->dc, c->d, c->d_pods, c->d_podx, ip, c->ext_idx[ip], u_of(ip) - lead, needc, ne,
                                   c->d_ext_scr, sync, c->xstream));
        ip++;
      } else {
        const int32_t u = u_of(ifn);
        HIP_TRY(kh::launch_ext_final(c->dc, c->d, c->d_pods, c->d_podx, ifn, c->ext_idx[ifn], std::max(0, u - lead) * P,
                                     std::max(0, u - lag) * P, ne, c->d_ext_scr, c->d_out, c->d_devout, sync, c->d_dbg,
                                     c->d_ext_idx, pre_needc[ifn], (alt && (ifn & 1)) ? c->xstream3 : xs2));
        ifn++;
      }
    }
    HIP_TRY(hipEventRecord(c->ev_ext, c->xstream));
    if (c->xstream2) HIP_TRY(hipEventRecord(c->ev_ext2, c->xstream2));
    if (c->xstream3) HIP_TRY(hipEventRecord(c->ev_ext3, c->xstream3));
  }
  for (int32_t r = 0; r < rounds && !cls; r++) {
    const int32_t p0 = r * P, np = std::min(P, total - p0);
    const int par = r & 1;
    const int32_t cum = P * (r >> 1) + np;  // pods of the rounds of parity `par` up to r
    hipStream_t es = (two && par) ? c->stream2 : c->stream;
    const int slot = two ? par : 0;
    const kh::DevPod *pods = c->d_pods + p0;
    uint64_t *lists = c->d_lists + (size_t)(r & (2 * lag - 1)) * list_buf;
    const bool select_waits = c->sel_split && !exch && !wait_kernel;  // the previous select held the stream
    if (r > lag && !serial && !select_waits) HIP_TRY(kh::launch_wait_resolved(sync, r - lag, es));
    if (exch) {
      if (np < P) HIP_TRY(hipMemsetAsync(lists, 0, (size_t)P * K * sizeof(uint64_t), es));
      if (int e = topk_batch(c, pods, np, K, lo, hi, lists, r % tstride == 0, nullptr, 0, 0, es, slot)) return e;
      if (int e = exchange(c, lists, (size_t)P * K, slot, es)) return e;
      // the merge counts each pod's list into the pipeline itself (no signal kernel on the chain)
      HIP_TRY(kh::launch_topk_merge(gather_buf(c, slot), K, (int64_t)P * K, np, c->world, K, c->score_bits,
                                    c->d_final + (size_t)(r & (2 * lag - 1)) * list_buf, sync, par, es));
    } else {
      // the split select's merging workgroups count the round's pods into sync->sel[par] themselves
      // (KOORDHIP_FOLD_WAIT: and hold the stream until round r - 1 is resolved, what the next scan needs)
      if (int e = topk_batch(c, pods, np, K, lo, hi, lists, r % tstride == 0, c->sel_split ? sync : nullptr, par,
                             wait_kernel ? 0 : r, es, slot))
        return e;
    }
    if (!exch && !c->sel_split) HIP_TRY(kh::launch_signal_lists(sync, par, cum, es));
    if (!persistent) {
      if (!serial) {
        HIP_TRY(hipEventRecord(c->ev_res[r % kRing], c->stream));
        HIP_TRY(hipStreamWaitEvent(rs, c->ev_res[r % kRing], 0));
      }
      int32_t tm = -1;
      if (int e = timed_begin(c, TK_RESOLVE, rs, &tm)) return e;
      HIP_TRY(kh::launch_resolve(c->dc, c->d, c->d_desc, c->d_pods, total, P, K, r, r + 1, lists0, list_buf, c->monotone, 1, sync,
                                 mbuf, c->d_out, cpus, c->d_dbg, trace, rs));
      c->resolve_kernel = kh::last_resolve_kernel();
      if (int e = timed_end(c, tm, rs)) return e;
    }
  }
  if (int e = timed_end(c, res_tm, c->rstream)) return e;
  if (two) {
    HIP_TRY(hipEventRecord(c->ev_eval2, c->stream2));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_eval2, 0));
  }
  if (ext_pipe && rounds > 0) {
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_ext, 0));
    if (c->xstream2) HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_ext2, 0));
    if (c->xstream3) HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_ext3, 0));
  }
  if (!serial) {
    HIP_TRY(hipEventRecord(c->ev_res[0], c->rstream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_res[0], 0));
  }
  HIP_TRY(hipEventRecord(c->t1, c->stream));
  c->pipe_check = true;
  if (c->d_dbg) {
    uint64_t h[64];
    HIP_TRY(hipMemcpyAsync(h, c->d_dbg, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::fprintf(stderr,
                 "[koordhip stamps] select blocks %llu cycles: bound %llu  pass1 %llu  kth %llu  pass2 %llu  out %llu\n",
                 (unsigned long long)h[8], (unsigned long long)h[9], (unsigned long long)h[10],
                 (unsigned long long)h[11], (unsigned long long)h[12], (unsigned long long)h[13]);
    if (c->eval_fused && h[40])
      std::fprintf(stderr,
                   "[koordhip stamps] k_eval_topk: %llu workgroups, cycles per workgroup: evaluate %.0f  select+emit %.0f  "
                   "publish %.0f | %llu merges, cycles per merge %.0f, candidates per merge %.1f\n",
                   (unsigned long long)h[40], (double)h[41] / h[40], (double)h[42] / h[40], (double)h[43] / h[40],
                   (unsigned long long)h[45], h[45] ? (double)h[44] / h[45] : 0.0, h[45] ? (double)h[46] / h[45] : 0.0);
    std::fprintf(stderr,
                 "[koordhip stamps] resolve cycles: prologue walk %llu  hash %llu  waiting for lists %llu  loop %llu  "
                 "release %llu | pods %llu  bulk commits %llu  staged pods %llu  general-path pods %llu  HBM row loads %llu\n",
                 (unsigned long long)h[0], (unsigned long long)h[2], (unsigned long long)h[1], (unsigned long long)h[4],
                 (unsigned long long)h[14], (unsigned long long)h[7], (unsigned long long)h[20],
                 (unsigned long long)h[21], (unsigned long long)h[5], (unsigned long long)h[6]);
    std::fprintf(stderr, "[koordhip stamps] resolve loop cycles: conflict detection %llu  bulk commits %llu | "
                 "general path: candidate+keys %llu  commit %llu | write-back %llu | kernel total %llu\n",
                 (unsigned long long)h[16], (unsigned long long)h[17], (unsigned long long)h[18],
                 (unsigned long long)h[19], (unsigned long long)h[25], (unsigned long long)h[26]);
    std::fprintf(stderr, "[koordhip stamps] round overlap: wave-0 end-of-round barrier %llu | wave 1: waiting for the "
                 "next lists %llu  loading them %llu\n",
                 (unsigned long long)h[29], (unsigned long long)h[27], (unsigned long long)h[28]);
    if (c->numa)
      std::fprintf(stderr, "[koordhip stamps] NUMA: accumulator replays full %llu cycles / %llu, spread %llu / %llu | "
                   "row passes of required-spread pods %llu / %llu, of other pods %llu / %llu\n",
                   (unsigned long long)h[32], (unsigned long long)h[33], (unsigned long long)h[34],
                   (unsigned long long)h[35], (unsigned long long)h[36], (unsigned long long)h[37],
                   (unsigned long long)h[38], (unsigned long long)h[39]);
    std::fprintf(stderr, "[koordhip stamps] general path detail: candidate + table keys %llu  row evaluations %llu | "
                 "pods served by the key tables %llu\n",
                 (unsigned long long)h[22], (unsigned long long)h[23], (unsigned long long)h[24]);
    std::fprintf(stderr, "[koordhip stamps] prologue phases: walk %llu  winner rows %llu (HBM loads %llu)  conflicts %llu | "
                 "general-path causes: staged conflict %llu  slow %llu  voided by a general commit %llu\n",
                 (unsigned long long)h[48], (unsigned long long)h[49], (unsigned long long)h[51],
                 (unsigned long long)h[50], (unsigned long long)h[52], (unsigned long long)h[53],
                 (unsigned long long)h[54]);
    std::fprintf(stderr, "[koordhip stamps] general path split: list + X + c %llu cycles | pods with ready key tables %llu | "
                 "evaluation passes %llu\n",
                 (unsigned long long)h[55], (unsigned long long)h[56], (unsigned long long)h[57]);
    if (cls) {
      uint64_t q[32];
      HIP_TRY(hipMemcpy(q, c->d_dbg + 64, sizeof(q), hipMemcpyDeviceToHost));
      const double nl = (double)std::max<uint64_t>(q[7], 1), nc = (double)std::max<uint64_t>(q[15], 1);
      std::fprintf(stderr, "[koordhip stamps] class lists, cycles per launch (workgroup 0, %llu launches): buffer %.0f  log %.0f  "
                   "touched keys %.0f  compaction %.0f  sort %.0f  merge %.0f  outputs %.0f | builds (%llu): histogram %.0f  "
                   "fine %.0f  emit %.0f  sort %.0f  write %.0f\n", (unsigned long long)q[7], q[0] / nl, q[1] / nl, q[2] / nl,
                   q[3] / nl, q[4] / nl, q[5] / nl, q[6] / nl, (unsigned long long)q[15], q[8] / nc, q[9] / nc, q[10] / nc,
                   q[11] / nc, q[12] / nc);
    }
    {
      uint64_t q[4] = {0, 0, 0, 0}, rw[7] = {0, 0, 0, 0, 0, 0, 0};
      HIP_TRY(hipMemcpy(q, c->d_dbg + 90, sizeof(q), hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(rw, c->d_dbg + 107, sizeof(rw), hipMemcpyDeviceToHost));
      std::fprintf(stderr, "[koordhip stamps] chain re-walks: walk + keys %llu (entries + claims %llu, row + evaluation "
                   "%llu)  winners' rows %llu cycles | winner rows loaded from HBM %llu\n", (unsigned long long)rw[0],
                   (unsigned long long)rw[5], (unsigned long long)rw[6], (unsigned long long)rw[1],
                   (unsigned long long)rw[2]);
      std::fprintf(stderr, "[koordhip stamps] chained decisions: %llu cycles, %llu pods resolved | claim tables %llu  "
                   "re-walks %llu  re-check + closure %llu  final table %llu\n", (unsigned long long)h[62],
                   (unsigned long long)h[63], (unsigned long long)q[0], (unsigned long long)q[1],
                   (unsigned long long)q[2], (unsigned long long)q[3]);
    }
    if (ext_pipe) {
      uint64_t q[8];
      HIP_TRY(hipMemcpy(q, c->d_dbg + 80, sizeof(q), hipMemcpyDeviceToHost));
      const double np = (double)std::max<uint64_t>(q[6], 1);
      std::fprintf(stderr, "[koordhip stamps] device pods (k_ext_pre / k_ext_final): %llu, resolve cycles from the "
                   "hand-off to the answer %llu (%.0f per pod) | final launch per pod: workgroup 0 evaluate + fold "
                   "%.0f | last workgroup: decide + publish %.0f  device commit %.0f\n",
                   (unsigned long long)h[31], (unsigned long long)h[30], h[31] ? (double)h[30] / h[31] : 0.0,
                   q[0] / np, q[3] / np, q[4] / np);
      uint64_t r[16];
      HIP_TRY(hipMemcpy(r, c->d_dbg + 96, sizeof(r), hipMemcpyDeviceToHost));
      std::fprintf(stderr, "[koordhip stamps] device-pod finals: workgroups with a full (device) re-evaluation %llu, "
                   "their re-evaluation %.2f us each\n", (unsigned long long)r[14], r[14] ? r[15] * 0.01 / r[14] : 0.0);
      const double nb = (double)std::max<uint64_t>(r[10], 1);
      std::fprintf(stderr, "[koordhip stamps] device-pod finals, us: request seen -> last workgroup arrived %.2f per pod | "
                   "per workgroup: -> gate seen %.2f  X marked %.2f  re-evaluated %.2f  folded + arrived %.2f\n",
                   r[5] * 0.01 / np, r[6] * 0.01 / nb, r[7] * 0.01 / nb, r[8] * 0.01 / nb, r[9] * 0.01 / nb);
      // (s_memrealtime: 100 MHz, one clock for every CU)
      std::fprintf(stderr, "[koordhip stamps] device-pod hand-offs, us per pod: the request seen -> published %.2f | "
                   "requests already set when the final's first workgroup started: %llu of %llu | pre-evaluation "
                   "published after the request: %llu pods, waited %.2f us each\n",
                   r[2] * 0.01 / np, (unsigned long long)r[0], (unsigned long long)q[6], (unsigned long long)r[1],
                   r[1] ? r[3] * 0.01 / r[1] : 0.0);
    }
    std::fprintf(stderr, "[koordhip stamps] general commit split: row source %llu  Reserve delta %llu  voiding + "
                 "outputs %llu cycles | winners already in M %llu\n",
                 (unsigned long long)h[58], (unsigned long long)h[59], (unsigned long long)h[60],
                 (unsigned long long)h[61]);
  }
  return 0;
}

// After a place call: did either side of the pipeline give up waiting?  The
// error is sticky until the next place call: every later fetch / stats call
// of this stream reports it.
static const char *pipe_msg(int32_t err) {
  switch (err) {
    case 2: return "class lists underflowed (fewer than k keys above a build's boundary): placements are incomplete";
    case 4: return "a device pod's DeviceShare Reserve failed where its Filter passed (k_ext_final): placements are "
                   "incomplete";
    default: return "round pipeline stalled (watchdog): placements are incomplete";
  }
}

int pipe_status(koordhip_ctx *c) {
  static const char *kStall = "round pipeline stalled (watchdog): placements are incomplete";
  if (c->pipe_err) return fail(KOORDHIP_EDEVICE, c->pipe_errc ? pipe_msg(c->pipe_errc) : kStall);
  if (c->last_seq && c->pipe_check && c->d_seqg) {  // the sequential cycle's spin timeout word
    c->pipe_check = false;
    uint32_t tmo = 0;
    HIP_TRY(hipMemcpy(&tmo, reinterpret_cast<char *>(c->d_seqg) + kh::seq_tmo_offset(c->seq_grid), sizeof(tmo),
                      hipMemcpyDeviceToHost));
    if (tmo) {
      c->pipe_err = true;
      return fail(KOORDHIP_EDEVICE, "sequential cycle stalled (watchdog): placements are incomplete");
    }
    return 0;
  }
  if (!c->pipe_check || !c->d_mod) return 0;
  c->pipe_check = false;
  kh::PipeSync *sync = reinterpret_cast<kh::PipeSync *>(c->d_mod + 1 + kMaxBatch);
  int32_t err = 0;
  HIP_TRY(hipMemcpy(&err, reinterpret_cast<int32_t *>(sync) + kh::kPipeSyncErrWord, sizeof(err), hipMemcpyDeviceToHost));
  if (err) {
    c->pipe_err = true;
    c->pipe_errc = err;
    if (c->last_ext_pipe || (c->d_plan && !c->cls_rep.empty())) {  // where the pipeline stood
      int32_t sy[96], cstarted = -1;
      HIP_TRY(hipMemcpy(sy, sync, sizeof(sy), hipMemcpyDeviceToHost));
      const int32_t sw[6] = {sy[0], sy[1], sy[2], sy[3], sy[kh::kPipeSyncExtReqWord], sy[kh::kPipeSyncExtDoneWord]};
      if (c->d_plan && !c->cls_rep.empty()) {
        const kh::ClsSync cs = cls_sync(c, sync);
        HIP_TRY(hipMemcpy(&cstarted, cs.rcnt + kh::kClsRoundRing, sizeof(int32_t), hipMemcpyDeviceToHost));
        std::vector<int32_t> st(c->cls_rep.size()), dn(c->cls_rep.size()), swv(c->cls_rep.size());
        HIP_TRY(hipMemcpy(st.data(), cs.rcnt + kh::kClsRoundRing + 1, st.size() * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(dn.data(), cs.done, dn.size() * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(swv.data(), cs.sw, swv.size() * 4, hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[koordhip] class workgroups (round << 4 | 1 build wait, 2 commit wait, 3 publish wait, 4 "
                     "published; done; switches):");
        for (size_t q = 0; q < st.size(); q++) std::fprintf(stderr, " %zu:%d/%d/%d", q, st[q], dn[q], swv[q]);
        std::fprintf(stderr, "\n");
      }
      std::fprintf(stderr, "[koordhip] pipeline error %d: sel %d/%d res_round %d ext_req %d ext_done %d | class-list "
                   "workgroups started %d of %zu\n", err, sw[0], sw[1], sw[2], sw[4], sw[5], cstarted, c->cls_rep.size());
    }
    return fail(KOORDHIP_EDEVICE, pipe_msg(err));
  }
  return 0;
}

}  // namespace

extern "C" {

int koordhip_synchronize(koordhip_ctx *c) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return pipe_status(c);
}

int koordhip_fetch_placements(koordhip_ctx *c, int32_t *out_node, int32_t n_pods) {
  if (!c || (!out_node && n_pods > 0)) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (n_pods > c->n_staged) return fail(KOORDHIP_EINVAL, "n_pods exceeds the staged stream");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (int e = pipe_status(c)) return e;
  if (n_pods) HIP_TRY(hipMemcpy(out_node, c->d_out, (size_t)n_pods * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_fetch_cpusets(koordhip_ctx *c, uint64_t *cpus, int32_t n_pods) {
  if (!c || (!cpus && n_pods > 0)) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (n_pods > c->n_staged) return fail(KOORDHIP_EINVAL, "n_pods exceeds the staged stream");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (int e = pipe_status(c)) return e;
  const size_t b = (size_t)n_pods * KOORDHIP_NUMA_WORDS * sizeof(uint64_t);
  if (!c->d_cpus) {
    if (b) std::memset(cpus, 0, b);
    return 0;
  }
  if (b) HIP_TRY(hipMemcpy(cpus, c->d_cpus, b, hipMemcpyDeviceToHost));
  return 0;
}

int koordhip_place_stream(koordhip_ctx *c, const koordhip_pod *pods, int32_t n_pods, int32_t *out_node) {
  if (int e = koordhip_stage_pods(c, pods, n_pods)) return e;
  if (int e = koordhip_place_staged(c)) return e;
  return koordhip_fetch_placements(c, out_node, n_pods);
}

// mutable columns: (device pointer, bytes)
static std::vector<std::pair<void *, size_t>> mutable_cols(koordhip_ctx *c) {
  const size_t n = c->n, b = n * sizeof(int64_t);
  std::vector<std::pair<void *, size_t>> v;
  for (int r = 0; r < KOORDHIP_NRES; r++) v.push_back({c->d.requested[r], b});
  v.push_back({c->d.nz_cpu, b});
  v.push_back({c->d.nz_mem, b});
  v.push_back({c->d.npods, n * sizeof(int32_t)});
  v.push_back({c->d.la_used_cpu, b});
  v.push_back({c->d.la_used_mem, b});
  v.push_back({c->d.la_used_prod_cpu, b});
  v.push_back({c->d.la_used_prod_mem, b});
  v.push_back({c->d.flags, n});
  if (c->numa) {
    const kh::DevNuma &nu = c->d.nu;
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
      v.push_back({nu.fr[w], n * sizeof(uint64_t)});
      v.push_back({nu.ep[w], n * sizeof(uint64_t)});
      v.push_back({nu.en[w], n * sizeof(uint64_t)});
    }
    v.push_back({nu.cnt, n * sizeof(int32_t)});
    if (nu.zu) v.push_back({nu.zu, n * 2 * KOORDHIP_NUMA_MAX_ZONES * sizeof(double)});
  }
  if (c->d.dv.used)
    v.push_back({c->d.dv.used, n * KOORDHIP_DEV_TYPES * (size_t)c->d.dv.slots * KOORDHIP_DEV_RES * sizeof(int64_t)});
  if (c->d.dv.xreq) v.push_back({c->d.dv.xreq, n * KOORDHIP_NXRES * sizeof(int64_t)});
  if (c->d.dv.rxd) v.push_back({c->d.dv.rxd, n * KOORDHIP_NXRES * sizeof(int64_t)});
  if (c->d.dv.rdev)
    v.push_back({c->d.dv.rdev, n * 2 * KOORDHIP_DEV_TYPES * (size_t)c->d.dv.slots * KOORDHIP_DEV_RES * sizeof(int64_t)});
  if (c->pts.cnt) v.push_back({c->pts.cnt, n * (size_t)std::max(1, c->pts.cons) * sizeof(int32_t)});
  if (c->ipa.cnt) v.push_back({c->ipa.cnt, n * (size_t)c->ipa.ents * sizeof(int32_t)});
  if (c->dc.resv) {
    const size_t sl = (size_t)c->d.rv.slots;
    v.push_back({c->d.rv.rd[0], b * sl});
    v.push_back({c->d.rv.rd[1], b * sl});
    v.push_back({c->d.rv.rn, n * sl * sizeof(int32_t)});
    if (c->dc.resv_cpus)
      for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) v.push_back({c->d.rv.rc[w], n * sl * sizeof(uint64_t)});
  }
  return v;
}

int koordhip_checkpoint(koordhip_ctx *c) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  HIP_TRY(hipSetDevice(c->device));
  auto cols = mutable_cols(c);
  if (c->ckpt.size() != cols.size()) {
    for (void *p : c->ckpt) (void)hipFree(p);
    c->ckpt.assign(cols.size(), nullptr);
    for (size_t i = 0; i < cols.size(); i++) HIP_TRY(hipMalloc(&c->ckpt[i], std::max<size_t>(cols[i].second, 1)));
  }
  for (size_t i = 0; i < cols.size(); i++)
    if (cols[i].second) HIP_TRY(hipMemcpyAsync(c->ckpt[i], cols[i].first, cols[i].second, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int koordhip_restore(koordhip_ctx *c) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  auto cols = mutable_cols(c);
  if (c->ckpt.size() != cols.size()) return fail(KOORDHIP_ESTATE, "no checkpoint");
  HIP_TRY(hipSetDevice(c->device));
  for (size_t i = 0; i < cols.size(); i++)
    if (cols[i].second) HIP_TRY(hipMemcpyAsync(cols[i].first, c->ckpt[i], cols[i].second, hipMemcpyDeviceToDevice, c->stream));
  return 0;
}

static int commit_ext_impl(koordhip_ctx *c, const koordhip_pod *pod, const koordhip_pod_ext *ext, int32_t node, int sign,
                           uint64_t *cpus_io, uint32_t *dev_io);

static int commit_impl(koordhip_ctx *c, const koordhip_pod *pod, int32_t node, int sign, uint64_t *cpus_io) {
  if (!c || !pod) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (c->resv_x) {
    // reservations listing extended scalars: the nomination's scoreReservation
    // counts them (resv.hpp ResvXS) -- the sequential cycle's Reserve, with an
    // empty koordhip_pod_ext record (no device request: gpu keys absent)
    koordhip_pod_ext none;
    std::memset(&none, 0, sizeof(none));
    for (int r = 0; r < KOORDHIP_DEV_RES; r++) none.dev_req[KOORDHIP_DEV_GPU][r] = -1;
    return commit_ext_impl(c, pod, &none, node, sign, cpus_io, nullptr);
  }
  if (node < 0 || node >= c->n) return fail(KOORDHIP_EINVAL, "node index out of range");
  const bool cpuset = c->numa && (pod->flags & KOORDHIP_POD_CPUSET) &&
                      !(pod->flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
  if (sign < 0 && cpuset && !cpus_io) return fail(KOORDHIP_EINVAL, "Unreserve of a cpuset pod needs its cpus");
  HIP_TRY(hipSetDevice(c->device));
  uint64_t *d_cpus = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(c->d_rc) + sizeof(uint64_t));
  std::vector<kh::DevPod> hp;
  if (int e = to_dev_pods(pod, 1, hp)) return e;
  HIP_TRY(hipMemcpyAsync(c->d_tmp_pod, hp.data(), sizeof(kh::DevPod), hipMemcpyHostToDevice, c->stream));
  if (sign < 0 && cpus_io)
    HIP_TRY(hipMemcpyAsync(d_cpus, cpus_io, KOORDHIP_NUMA_WORDS * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(kh::launch_commit(c->dc, c->d, c->d_tmp_pod, node, sign, d_cpus, c->d_rc, c->stream));
  int32_t rc = 0;
  uint64_t got[KOORDHIP_NUMA_WORDS];
  HIP_TRY(hipMemcpyAsync(&rc, c->d_rc, sizeof(rc), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(got, d_cpus, sizeof(got), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (rc == KOORDHIP_EINVAL)
    return fail(rc, "Unreserve not supported here: a NodeNUMAResource pod on a NUMA topology-policy node (its zone amounts "
                    "are not passed back) or a pod its node's reservation matches (whether the Reserve took the "
                    "reservation is not passed back)");
  if (rc) return fail(rc, "Reserve failed: NodeNUMAResource could not allocate the cpuset");
  if (sign > 0 && cpus_io) std::memcpy(cpus_io, got, sizeof(got));
  return 0;
}

int koordhip_commit(koordhip_ctx *c, const koordhip_pod *pod, int32_t node, uint64_t *cpus_out) {
  return commit_impl(c, pod, node, +1, cpus_out);
}

static int commit_ext_impl(koordhip_ctx *c, const koordhip_pod *pod, const koordhip_pod_ext *ext, int32_t node, int sign,
                           uint64_t *cpus_io, uint32_t *dev_io) {
  if (!c || !pod || !ext) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (!c->loaded) return fail(KOORDHIP_ESTATE, "no snapshot loaded");
  if (node < 0 || node >= c->n) return fail(KOORDHIP_EINVAL, "node index out of range");
  bool any = false;
  if (int e = check_pod_ext(ext, 1, &any)) return e;
  if (int e = check_pod_pts(c, ext, 1)) return e;
  if (any && !c->seq_profile)
    return fail(KOORDHIP_EINVAL, "device / extended-scalar pod requests need DeviceShare in the profile");
  if (ext->reserve_node != 0 || (pod->flags & KOORDHIP_POD_RESERVE))
    return fail(KOORDHIP_EINVAL, "a reserve pod's Reserve assumes its reservation: not on this entry point");
  const bool cpuset = c->numa && (pod->flags & KOORDHIP_POD_CPUSET) &&
                      !(pod->flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
  if (sign < 0 && cpuset && !cpus_io) return fail(KOORDHIP_EINVAL, "Unreserve of a cpuset pod needs its cpus");
  const bool dev = (ext->flags & KOORDHIP_PODX_DEVICE) &&
                   ((c->cfg.filter_plugins | c->cfg.score_plugins) & KOORDHIP_PLUGIN_DEVICESHARE);
  if (sign < 0 && dev && !dev_io) return fail(KOORDHIP_EINVAL, "Unreserve of a device pod needs its device slots");
  HIP_TRY(hipSetDevice(c->device));
  if (!c->d_tmp_podx) HIP_TRY(hipMalloc(&c->d_tmp_podx, sizeof(kh::DevPodX)));
  // d_rc: status (byte 0), cpus (bytes 8..39), device slots (bytes 40..51)
  uint64_t *d_cpus = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(c->d_rc) + sizeof(uint64_t));
  uint32_t *d_dev = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(c->d_rc) + 40);
  std::vector<kh::DevPod> hp;
  if (int e = to_dev_pods(pod, 1, hp, ext, devshare_resv_on(c))) return e;
  HIP_TRY(hipMemcpyAsync(c->d_tmp_pod, hp.data(), sizeof(kh::DevPod), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_tmp_podx, ext, sizeof(kh::DevPodX), hipMemcpyHostToDevice, c->stream));
  uint64_t cz[KOORDHIP_NUMA_WORDS] = {0, 0, 0, 0};
  uint32_t dz[KOORDHIP_DEV_TYPES] = {0u, 0u, 0u};
  HIP_TRY(hipMemcpyAsync(d_cpus, (sign < 0 && cpus_io) ? cpus_io : cz, sizeof(cz), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_dev, (sign < 0 && dev_io) ? dev_io : dz, sizeof(dz), hipMemcpyHostToDevice, c->stream));
  const int32_t rs = (c->dc.resv && (c->cfg.score_plugins & KOORDHIP_PLUGIN_RESERVATION)) ? 1 : 0;
  HIP_TRY(kh::launch_commit_ext(c->dc, c->d, c->d_tmp_pod, c->d_tmp_podx, node, sign, rs, d_cpus, d_dev, c->d_rc,
                                c->pts, c->ipa, c->stream));
  int32_t rc = 0;
  uint64_t got[KOORDHIP_NUMA_WORDS];
  uint32_t gdev[KOORDHIP_DEV_TYPES];
  HIP_TRY(hipMemcpyAsync(&rc, c->d_rc, sizeof(rc), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(got, d_cpus, sizeof(got), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(gdev, d_dev, sizeof(gdev), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (rc == KOORDHIP_EINVAL)
    return fail(rc, "Unreserve not supported here: a NodeNUMAResource pod on a NUMA topology-policy node (its zone amounts "
                    "are not passed back) or a pod its node's reservation matches (whether the Reserve took the "
                    "reservation is not passed back)");
  if (rc) return fail(rc, "Reserve failed: DeviceShare or NodeNUMAResource could not allocate");
  if (sign > 0) {
    if (cpus_io) std::memcpy(cpus_io, got, sizeof(got));
    if (dev_io) std::memcpy(dev_io, gdev, sizeof(gdev));
  }
  return 0;
}

int koordhip_commit_ext(koordhip_ctx *c, const koordhip_pod *pod, const koordhip_pod_ext *ext, int32_t node,
                        uint64_t *cpus_out, uint32_t *dev_slots_out) {
  return commit_ext_impl(c, pod, ext, node, +1, cpus_out, dev_slots_out);
}
int koordhip_uncommit_ext(koordhip_ctx *c, const koordhip_pod *pod, const koordhip_pod_ext *ext, int32_t node,
                          const uint64_t *cpus, const uint32_t *dev_slots) {
  return commit_ext_impl(c, pod, ext, node, -1, const_cast<uint64_t *>(cpus), const_cast<uint32_t *>(dev_slots));
}
int koordhip_uncommit(koordhip_ctx *c, const koordhip_pod *pod, int32_t node, const uint64_t *cpus) {
  return commit_impl(c, pod, node, -1, const_cast<uint64_t *>(cpus));
}

int koordhip_last_stats(koordhip_ctx *c, double *eval_ms, int64_t *eval_launches, int64_t *evals, double *total_ms) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (int e = pipe_status(c)) return e;
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, c->t0, c->t1));
  double em = 0;
  for (int32_t i = 0; i + 1 < c->ev_used; i += 2) {
    if (c->ev_kind[i / 2] != TK_SCAN) continue;
    float x = 0;
    HIP_TRY(hipEventElapsedTime(&x, c->ev[i], c->ev[i + 1]));
    em += x;
  }
  if (eval_ms) *eval_ms = em;
  if (eval_launches) *eval_launches = c->last_launches;
  if (evals) *evals = c->last_evals;
  if (total_ms) *total_ms = ms;
  return 0;
}

int koordhip_last_kernel_stats(koordhip_ctx *c, koordhip_kernel_stats *out) {
  if (!c || !out) return fail(KOORDHIP_EINVAL, "NULL argument");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (int e = pipe_status(c)) return e;
  std::memset(out, 0, sizeof(*out));
  double ms[TK_KINDS] = {0, 0, 0};
  int64_t n[TK_KINDS] = {0, 0, 0};
  for (int32_t i = 0; i + 1 < c->ev_used; i += 2) {
    float x = 0;
    HIP_TRY(hipEventElapsedTime(&x, c->ev[i], c->ev[i + 1]));
    ms[c->ev_kind[i / 2]] += x;
    n[c->ev_kind[i / 2]]++;
  }
  float tot = 0;
  HIP_TRY(hipEventElapsedTime(&tot, c->t0, c->t1));
  out->scan_ms = ms[TK_SCAN];
  out->scan_launches = n[TK_SCAN];
  out->select_ms = ms[TK_SELECT];
  out->select_launches = n[TK_SELECT];
  out->resolve_ms = ms[TK_RESOLVE];
  out->resolve_launches = n[TK_RESOLVE];
  out->total_ms = tot;
  out->evals = c->last_evals;
  out->pods = c->n_staged;
  out->rounds = (c->n_staged + c->last_P - 1) / std::max(c->last_P, 1);
  out->round_pods = c->last_P;
  out->lag = c->last_lag;
  int64_t ex = (c->last_exec < 0 ? c->last_evals : c->last_exec) + c->last_ext_exec;
  for (const uint32_t *p : {c->last_evc, c->last_reev})
    if (p) {
      uint32_t v = 0;
      HIP_TRY(hipMemcpy(&v, p, sizeof(v), hipMemcpyDeviceToHost));
      ex += v;
    }
  out->executed_evals = ex;
  out->plan_us = c->last_plan_us;
  out->flags = c->last_local ? KOORDHIP_KSTAT_LOCAL : 0;
  return 0;
}

int koordhip_set_profile_kernels(koordhip_ctx *c, int32_t on) {
  if (!c) return fail(KOORDHIP_EINVAL, "ctx is NULL");
  c->cfg.profile_kernels = on ? 1 : 0;
  return 0;
}

int koordhip_last_kernel_names(koordhip_ctx *c, char *eval_out, char *resolve_out, int32_t cap) {
  if (!c || !eval_out || !resolve_out || cap < 1) return fail(KOORDHIP_EINVAL, "NULL argument");
  std::snprintf(eval_out, (size_t)cap, "%s", c->eval_kernel.c_str());
  std::snprintf(resolve_out, (size_t)cap, "%s", c->resolve_kernel.c_str());
  return 0;
}

int koordhip_comm_unique_id(uint8_t *id_out) {
  if (!id_out) return fail(KOORDHIP_EINVAL, "NULL argument");
  static_assert(sizeof(ncclUniqueId) <= KOORDHIP_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memset(id_out, 0, KOORDHIP_UNIQUE_ID_BYTES);
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}

int koordhip_comm_init(koordhip_ctx *c, const uint8_t *id, int32_t world, int32_t rank) {
  if (!c || !id) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (world < 1 || rank < 0 || rank >= world) return fail(KOORDHIP_EINVAL, "bad world/rank");
  HIP_TRY(hipSetDevice(c->device));
  if (c->comm2) {
    (void)ncclCommDestroy(c->comm2);
    c->comm2 = nullptr;
  }
  if (c->comm) {
    (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  c->group.reset();
  // world 1 creates a one-rank communicator too: the same exchange path as a
  // sharded group (RCCL all-gather of the lists + k_topk_merge), on one GPU
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCL_TRY(ncclCommInitRank(&c->comm, world, uid, rank));
  // a second communicator over the same ranks for the second evaluation
  // stream (collective: every rank splits here, in the same order)
  NCCL_TRY(ncclCommSplit(c->comm, 0, rank, &c->comm2, nullptr));
  c->world = world;
  c->rank = rank;
  return 0;
}

int koordhip_comm_init_local(koordhip_ctx **ctxs, int32_t world) {
  if (!ctxs) return fail(KOORDHIP_EINVAL, "NULL argument");
  if (world < 1 || world > 64) return fail(KOORDHIP_EINVAL, "world must be in [1, 64]");
  for (int32_t r = 0; r < world; r++) {
    if (!ctxs[r]) return fail(KOORDHIP_EINVAL, "NULL context in group");
    for (int32_t q = 0; q < r; q++)
      if (ctxs[q] == ctxs[r]) return fail(KOORDHIP_EINVAL, "context listed twice in group");
  }
  auto g = std::make_shared<LocalGroup>();
  g->world = world;
  g->ctx.assign(ctxs, ctxs + world);
  g->keys.assign(world, 0);
  for (int32_t r = 0; r < world; r++) {
    koordhip_ctx *c = ctxs[r];
    HIP_TRY(hipSetDevice(c->device));
    if (c->comm2) {
      (void)ncclCommDestroy(c->comm2);
      c->comm2 = nullptr;
    }
    if (c->comm) {
      (void)ncclCommDestroy(c->comm);
      c->comm = nullptr;
    }
    for (hipEvent_t *e : {&c->ev_part, &c->ev_copy})
      if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    c->group = world > 1 ? g : nullptr;
    c->world = world;
    c->rank = r;
  }
  return 0;
}

}  // extern "C"
