// cls.h -- launch wrappers of cls.hip: class-incremental candidate lists for
// the pipelined greedy (host side; api.hip and cls.hip only).
#pragma once
#include <hip/hip_runtime.h>

#include "eval.hpp"
#include "kernels.h"

namespace kh {

// A pod class = the pods whose device records (DevPod) are byte-identical:
// they rank every node the same way.  Per class, a buffer of candidate keys
// (make_key of the class's total on a node), sorted descending, and its meta:
// every node OUTSIDE the buffer has a current key <= boundary (0: the buffer
// holds every feasible node), the buffer's keys are exact on the state after
// the log rounds < base (later commits are in the resolve's out_node log).
struct ClsMeta {
  uint64_t boundary;
  int32_t cnt;
  int32_t base;
};
static_assert(sizeof(ClsMeta) == 16, "ClsMeta");

constexpr int32_t kClsCap = 4096;   // keys a buffer holds (a build fills kClsTarget, log insertions the rest)
constexpr int32_t kClsTarget = 2048;  // keys a build takes (the best ones, ties by lowest index)
constexpr int32_t kClsBuildRows = 64;  // class rows one build launch evaluates

// Device words of the class pipeline: the round pipeline's flags, and per
// class the builds completed (done[c] = the newest build number m, published by
// k_cls_collect after its buffer and meta) and the builds its workgroup
// switched to (sw[c]: a slot is rebuilt only after the workgroup copied the
// previous build of that slot).  done / sw are zero at the start of a call.
struct ClsSync {
  PipeSync *sy;
  int32_t *done;
  int32_t *sw;
  int32_t *rcnt;  // [kClsRoundRing]: the listed pods of round u at u % kClsRoundRing (zero between rounds)
  uint32_t *evc;  // (pod class, node) evaluations the lists re-ran from the commit log (per call; bench accounting)
};
constexpr int32_t kClsRoundRing = 16;  // rounds in flight between the class lists and the resolve (<= lag + 2)

// k_cls_collect: build bm[b] of class ent[b] >> 1 from its k_scan score row S[b]
// (total + 1, 0 = infeasible): the best min(target, feasible) keys sorted
// descending into buffer slot ent[b] ((class << 1) | slot), meta {boundary,
// cnt, base = tb}, once the class's workgroup has made bw[b] switches (0: no
// wait); then done[class] = bm[b].
hipError_t launch_cls_collect(const uint16_t *S, int64_t s_stride, int32_t n, const int32_t *ent, const int32_t *bm,
                              const int32_t *bw, int32_t nb, int32_t tb, uint64_t *bufs, ClsMeta *metas,
                              const ClsSync &cs, uint64_t *dbg, hipStream_t s);
// k_cls_run: ONE persistent workgroup per class, for the whole stream.  Class
// c's workgroup walks its schedule csched[coff[c], coff[c + 1]) (the rounds
// the class appears in; bit 31: switch first to build csm[] of the class,
// copying it from its buffer slot into LDS when k_cls_collect has published
// it).  Per round u: wait for the commits of the rounds < u - lag
// (res_round), apply the log rounds [base, u - lag) of out_node to its
// LDS-resident buffer (re-evaluate the class on the current rows of the nodes
// committed there; insert a node whose key now exceeds the boundary), keep it
// sorted, and write its best k keys as the list of every pod of the round in
// the class (pod_cls), stored write-through and counted into sync->sel[u & 1].
// An underflow (fewer than k keys above a nonzero boundary) sets sync->err = 2.
// Every workgroup of the grid must be resident (the host checks the LDS
// budget against the device's CUs).
size_t cls_run_lds(int32_t n, int32_t monotone);
hipError_t launch_cls_run(const DevCfg &c, const DevNodes &d, const DevPod *cls_pod, int32_t n_cls, const int32_t *coff,
                          const int32_t *csched, const int32_t *csm, const int32_t *pod_cls, const int32_t *out_node,
                          int32_t lag, int32_t P, int32_t total, const uint64_t *bufs, const ClsMeta *metas, int32_t k,
                          int32_t monotone, uint64_t *lists0, int64_t list_buf, const ClsSync &cs, uint64_t *dbg,
                          hipStream_t s);
// dbg (KOORDHIP_STAMPS, else NULL): class 0's phase cycles -- per appearance
// [0..6] (wait + setup, log, touched keys, compaction, sort, merge, outputs),
// appearances [7]; collect's workgroup 0 [8..12] (max / count, threshold, emit,
// sort, write), builds [15]
const char *cls_run_kernel_name(const DevCfg &c);

}  // namespace kh
