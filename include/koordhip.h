/*
 * koordhip.h -- C-ABI of libkoordhip.so, the MI355X batched placement engine
 * for koord-scheduler's Filter/Score hot path (NodeResourcesFit,
 * LoadAwareScheduling, NodeNUMAResource) plus argmax and the Reserve delta.
 *
 * Plain C, no torch / HIP types in any signature: a Go host binds it with cgo
 * (see INTEGRATION.md), Python with ctypes.  Every function returns 0 on
 * success and a negative KOORDHIP_E* code on error; the message of the last
 * error on the calling thread is returned by koordhip_last_error().
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * koordinator tree, "(upstream)" = k8s.io/kubernetes v1.24.15):
 *   koordhip_create         <- loadaware.New            pkg/scheduler/plugins/loadaware/load_aware.go:76-110
 *                              nodenumaresource.New     pkg/scheduler/plugins/nodenumaresource/plugin.go:101-151
 *                              (upstream) noderesources.NewFit + args from config/manager/scheduler-config.yaml:17-46
 *   koordhip_load_snapshot  <- the per-cycle NodeInfo snapshot + NodeMetric lister reads
 *                              load_aware.go:133,270-278; (upstream) Snapshot.NodeInfos()
 *   koordhip_update_nodes   <- informer deltas: podAssignCache.OnAdd/OnUpdate/OnDelete pod_assign_cache.go:82-117,
 *                              NodeMetric informer (load_aware.go:114-121)
 *   koordhip_eval           <- Filter  load_aware.go:123-171, (upstream) fit.go Filter/fitsRequest,
 *                              Score   load_aware.go:269-335, (upstream) resource_allocation.go score,
 *                              called per (pod,node) by frameworkext/framework_extender.go:192-238
 *   koordhip_place_stream   <- (upstream) schedule_one.go scheduleOne: findNodesThatFitPod ->
 *                              prioritizeNodes -> selectHost (tie -> lowest node index) -> Reserve
 *   koordhip_commit         <- Reserve  load_aware.go:260-263 (podAssignCache.assign, pod_assign_cache.go:53-68),
 *                              (upstream) cache.AssumePod -> NodeInfo.AddPod
 *   koordhip_uncommit       <- Unreserve load_aware.go:265-267 (pod_assign_cache.go:70-80)
 *   koordhip_commit_ext / koordhip_uncommit_ext
 *                           <- the same plus DeviceShare Reserve / Unreserve deviceshare/plugin.go:368-426 and the
 *                              (upstream) PodTopologySpread / InterPodAffinity AddPod / RemovePod of the pod
 *   reservation columns     <- Reservation BeforePreFilter restore reservation/transformer.go:48-293,
 *                              filterWithReservations plugin.go:373-494, PreScore/Score scoring.go:42-200,
 *                              NominateReservation nominator.go:32-85, Reserve -> reservationCache.assumePod
 *                              plugin.go:537-575 / cache.go:170-191
 *   resv_cpus columns       <- NodeNUMAResource RestoreReservation nodenumaresource/reservation.go:68-122 and the
 *                              reservation-preferred CPUs of getResourceOptions plugin.go:455-524 (Score / Reserve)
 *   dev_* columns, koordhip_pod_ext
 *                           <- DeviceShare PreFilter plugin.go:146-182, Filter :284-323, Score scoring.go:33-80,
 *                              Reserve plugin.go:368-405 over nodeDevice (device_cache.go:44-482) and the
 *                              default allocator (allocator.go:91-122)
 *   static_score columns    <- (upstream) NodeAffinity / TaintToleration Score + NormalizeScore
 *   koordhip_place_stream_ext / koordhip_eval_ext
 *                           <- the exact sequential cycle for profiles with plugins whose scores are normalized
 *                              over the feasible nodes (DefaultNormalizeScore, upstream helper/normalize_score.go)
 */
#ifndef KOORDHIP_H
#define KOORDHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KOORDHIP_ABI_VERSION 14

/* ---- error codes ------------------------------------------------------- */
#define KOORDHIP_OK 0
#define KOORDHIP_EINVAL (-1)   /* bad argument / config (validation_pluginargs.go:31-95 analogue) */
#define KOORDHIP_EDEVICE (-2)  /* HIP runtime error */
#define KOORDHIP_ESTATE (-3)   /* call out of order (e.g. eval before load_snapshot) */
#define KOORDHIP_ENOMEM (-4)
#define KOORDHIP_ECOMM (-5)    /* RCCL error */
#define KOORDHIP_ERESERVE (-6) /* a Reserve plugin failed (NodeNUMAResource Allocate, plugin.go:398-401) */

/* ---- plugins ------------------------------------------------------------ */
#define KOORDHIP_PLUGIN_FIT 1u        /* NodeResourcesFit (upstream) */
#define KOORDHIP_PLUGIN_LOADAWARE 2u  /* LoadAwareScheduling */
#define KOORDHIP_PLUGIN_NUMA 4u       /* NodeNUMAResource */
#define KOORDHIP_PLUGIN_RESERVATION 8u /* Reservation (restore + filterWithReservations + Score, weight
                                          koordhip_config.reservation_weight) */
/* Upstream default-profile plugins (k8s v1.24.15, un-vendored: SURVEY.md
 * section 8(f)#4; restated in DESIGN.md, parity unpinned by reference tests): */
#define KOORDHIP_PLUGIN_NODE_STATIC 16u /* Filter: NodeUnschedulable + NodeAffinity (nodeSelector +
                                           requiredDuringScheduling) + TaintToleration (NoSchedule /
                                           NoExecute), resolved per (pod static class, node) by the host
                                           into koordhip_node_soa.static_allow */
#define KOORDHIP_PLUGIN_BALANCED 32u    /* Score: NodeResourcesBalancedAllocation (cpu + memory,
                                           Requested + the pod request, 1 - |f_cpu - f_mem| / 2) */
#define KOORDHIP_NPLUGINS 4             /* plugins with a per-node score in koordhip_eval's scores:
                                           Fit, LoadAware, NUMA, BalancedAllocation */
/* Plugins whose Score is normalized over the pod's feasible nodes
 * (DefaultNormalizeScore(100, reverse)): a profile enabling any of them places
 * through the exact sequential cycle (koordhip_place_stream_ext).
 * Their raw scores are planes KOORDHIP_NPLUGINS.. of koordhip_eval_ext. */
#define KOORDHIP_PLUGIN_DEVICESHARE 64u      /* DeviceShare Filter / Score / Reserve (koordhip_pod_ext, dev_* columns) */
#define KOORDHIP_PLUGIN_AFFINITY_SCORE 128u  /* NodeAffinity Score: preferred terms (static_score[0]) */
#define KOORDHIP_PLUGIN_TAINT_SCORE 256u     /* TaintToleration Score: intolerable PreferNoSchedule taints
                                                (static_score[1], normalized reversed) */
#define KOORDHIP_PLUGIN_PTS 512u             /* PodTopologySpread Filter (DoNotSchedule constraints) and Score
                                                (ScheduleAnyway constraints, weight ext_weight[3]; its own
                                                min-max NormalizeScore); pts_* columns, koordhip_pod_ext.pts_* */
#define KOORDHIP_PLUGIN_IPA 1024u            /* InterPodAffinity Filter (required affinity / anti-affinity, the
                                                existing pods' required anti-affinity) and Score (preferred terms,
                                                the existing pods' terms; weight ext_weight[4]; its own min-max
                                                NormalizeScore); ipa_* columns, koordhip_pod_ext.ipa_* */
#define KOORDHIP_NEXT_PLUGINS 5              /* DeviceShare, NodeAffinity, TaintToleration, PodTopologySpread,
                                                InterPodAffinity */
/* PodTopologySpread envelope (k8s v1.24 podtopologyspread, not vendored): */
#define KOORDHIP_PTS_KEYS 4      /* distinct topology keys of the snapshot's constraints */
#define KOORDHIP_PTS_DOMAINS 64  /* values of a non-hostname key */
#define KOORDHIP_PTS_CONS 8      /* distinct (label selector, namespace) of the snapshot's constraints */
#define KOORDHIP_PTS_CLASSES 8   /* spread classes: (required node affinity, hard keys, soft keys) */
#define KOORDHIP_PTS_POD 4       /* constraints per pod */
/* InterPodAffinity envelope (k8s v1.24 interpodaffinity, not vendored): the
 * topology keys are the pts_* keys (shared with PodTopologySpread) */
#define KOORDHIP_IPA_ENTRIES 32  /* count entries of the snapshot (ipa_cnt rows) */
/* NodeResourcesFit's extended scalar resources of device pods (koordinator.sh/
 * gpu-core, gpu-memory-ratio, gpu-memory, nvidia.com/gpu, ...): fitsRequest
 * checks each one the pod requests against Allocatable - Requested (upstream
 * fit.go); koordhip_pod_ext.xreq / koordhip_node_soa.xalloc, xrequested */
#define KOORDHIP_NXRES 8
#define KOORDHIP_MAX_STATIC_CLASSES 32  /* distinct pod static classes (koordhip_pod.static_class) */

/* Fit resource slots (ResourceSpec names in scheduler-config.yaml:21-31). */
#define KOORDHIP_RES_CPU 0   /* "cpu", milli-CPU */
#define KOORDHIP_RES_MEM 1   /* "memory", bytes */
#define KOORDHIP_RES_EPH 2   /* "ephemeral-storage", bytes */
#define KOORDHIP_RES_BCPU 3  /* "kubernetes.io/batch-cpu", Value() */
#define KOORDHIP_RES_BMEM 4  /* "kubernetes.io/batch-memory", bytes */
#define KOORDHIP_NRES 5

/* Per-node LoadAware snapshot flags (koordhip_node_soa.la_flags), resolved by the
 * marshaller at snapshot time T0 (wall-clock predicates are never re-read). */
#define KOORDHIP_LA_HAS_METRIC 1u        /* nodeMetricLister.Get found (load_aware.go:133-142,278-286) */
#define KOORDHIP_LA_FILTER_SKIP 2u       /* FilterExpiredNodeMetrics && expired (load_aware.go:144-147) */
#define KOORDHIP_LA_SCORE_EXPIRED 4u     /* isNodeMetricExpired(NodeMetricExpirationSeconds) (load_aware.go:287-289) */
#define KOORDHIP_LA_FILTER_USAGE 8u      /* Status.NodeMetric != nil and the filter's usage source non-nil (load_aware.go:174-211) */
#define KOORDHIP_LA_PROD_MODE 16u        /* len(ProdUsageThresholds) > 0 (load_aware.go:150) */
#define KOORDHIP_LA_HAS_PODS_METRIC 32u  /* len(Status.PodsMetric) > 0 (load_aware.go:227-229) */
#define KOORDHIP_LA_AGGREGATED 64u       /* filter uses aggregated usage (status reason only) */

/* Per-pod flags (koordhip_pod.flags), computed once per pod by the host
 * (PreFilter analogue). */
#define KOORDHIP_POD_PROD 1u          /* GetPodPriorityClassWithDefault == koord-prod (priority_utils.go:26-34) */
#define KOORDHIP_POD_DAEMONSET 2u     /* isDaemonSetPod (helper.go:188-196) */
#define KOORDHIP_POD_HAS_REQ 4u       /* request not all-zero / scalar map non-empty (upstream fitsRequest) */
#define KOORDHIP_POD_REQ_BCPU 8u      /* batch-cpu key present in the pod request map */
#define KOORDHIP_POD_REQ_BMEM 16u     /* batch-memory key present in the pod request map */
#define KOORDHIP_POD_CPUSET 32u       /* NUMA: requestCPUBind (plugin.go:230-245) */
#define KOORDHIP_POD_NUMA_SKIP 64u    /* NUMA: PreFilter skip (zero request) (plugin.go:218-226) */
#define KOORDHIP_POD_NUMA_ERROR 128u  /* NUMA: PreFilter error (non-integral cpuset request, plugin.go:242-245) */
#define KOORDHIP_POD_KEY_CPU 256u     /* "cpu" key present in PodRequestsAndLimits (Reservation nominate / score / Restricted) */
#define KOORDHIP_POD_KEY_MEM 512u     /* "memory" key present */
#define KOORDHIP_POD_RESERVE 2048u    /* a reserve pod (IsReservePod, util/reservation): the Reservation Filter checks
                                         its reservation's nodeName (koordhip_pod_ext.reserve_node) and AllocatePolicy
                                         against the node's Available reservations (plugin.go:326-362), no reservation
                                         matches it (transformer.go:60,96; resv_match must be 0), its Reservation
                                         Score is 0 (scoring.go:127-130) and its Reserve assumes a reservation that is
                                         not Available yet (no slot, plugin.go:538-548).  A batch holding one runs in
                                         the sequential cycle (ABI 11) */
#define KOORDHIP_POD_RESERVE_POLICY_SHIFT 12  /* bits 12-13: the reserve pod's AllocatePolicy (KOORDHIP_RESV_POLICY codes) */
#define KOORDHIP_POD_RESV_OPERATING 16384u /* a pod in the reservation operating mode (IsReservationOperatingMode,
                                              apis/extension/operating_pod.go:51-53): the Reservation Filter checks
                                              AllocatePolicy Aligned (bits 12-13 = 1) against the node's Available
                                              reservations (plugin.go:332-357), then filterWithReservations as for
                                              any pod; a batch holding one runs in the sequential cycle (ABI 11) */
#define KOORDHIP_POD_RESERVE_POLICY(f) (((f) >> KOORDHIP_POD_RESERVE_POLICY_SHIFT) & 3u)
#define KOORDHIP_POD_CPUSET_QOS 32768u /* ABI 12: AllowUseCPUSet (nodenumaresource/util.go:42-49: koord-prod and
                                          QoS LSE / LSR) -- such a pod gets the nominated reservation's reserved
                                          CPUs restored (reservation.go:68-74) even when it binds none; on
                                          topology-policy or CPU-amplified nodes that changes its zone / amplified
                                          Score and Reserve (plugin.go:465-479), which the engine does not model
                                          for non-binding pods: such a batch is refused (KOORDHIP_EINVAL) on a
                                          snapshot with reservations holding CPUs on such nodes */
#define KOORDHIP_POD_RESV_AFFINITY 1024u /* a required reservation affinity (util/reservation/reservation.go:444-487): a node
                                            without a matched reservation fails the Reservation Filter (plugin.go:378-381) */

/* koordhip_node_soa.resv_flags: a node's Available reservations, one per slot
 * (koordhip_node_soa.resv_slots).  The reference keeps them in a map
 * (cache.go:236-252: forEachAvailableReservationOnNode iterates in Go map
 * order) and its nomination ties (findMostPreferredReservationByOrder's first
 * smallest order, nominator.go:60; sort.Slice by score, nominator.go:69-71)
 * follow that order: here they go to the lowest slot.  0 = empty slot. */
#define KOORDHIP_RESV_PRESENT 1u       /* IsAvailable && ParseError == nil (transformer.go:87-89) */
#define KOORDHIP_RESV_ALLOCATE_ONCE 2u /* IsReservationAllocateOnce (apis/extension/reservation.go:98-100) */
#define KOORDHIP_RESV_UNSCHEDULABLE 4u /* IsUnschedulable: spec.unschedulable or terminating (reservation_info.go:248-255) */
#define KOORDHIP_RESV_ORDERED 8u       /* label scheduling.koordinator.sh/reservation-order parses to != 0 (scoring.go:156-175) */
#define KOORDHIP_RESV_KEY_CPU 16u      /* "cpu" in ResourceNames (the Allocatable keys, reservation_info.go:80-81) */
#define KOORDHIP_RESV_KEY_MEM 32u      /* "memory" in ResourceNames */
#define KOORDHIP_RESV_POLICY_SHIFT 6   /* bits 6-7 AllocatePolicy: 0 Default, 1 Aligned, 2 Restricted */
#define KOORDHIP_RESV_POLICY(f) (((f) >> KOORDHIP_RESV_POLICY_SHIFT) & 3u)
#define KOORDHIP_RESV_GROUP_SHIFT 8    /* bits 8-13: owner group g, the pod matches iff bit g of koordhip_pod.resv_match */
#define KOORDHIP_RESV_GROUP(f) (((f) >> KOORDHIP_RESV_GROUP_SHIFT) & 63u)
#define KOORDHIP_RESV_MAX_ORDERS 1024  /* distinct reservation-order values (resv_order_rank < this) */
#define KOORDHIP_RESV_SLOTS 4          /* Available reservations per node on the pipelined greedy */
#define KOORDHIP_RESV_SLOTS_MAX 8      /* ... in a snapshot (koordhip_node_soa.resv_slots <= this); a snapshot with
                                          more than KOORDHIP_RESV_SLOTS runs in the sequential cycle (ABI 11) */

/* koordhip_pod.numa_policy, the NUMA PreFilter state (plugin.go:227-255):
 * bits 0-1 requiredCPUBindPolicy, 2-3 preferredCPUBindPolicy (= required when
 * set), 4-5 preferredCPUExclusivePolicy. */
#define KOORDHIP_CPUBIND_NONE 0u
#define KOORDHIP_CPUBIND_FULL_PCPUS 1u
#define KOORDHIP_CPUBIND_SPREAD_BY_PCPUS 2u
#define KOORDHIP_CPUEXCL_NONE 0u
#define KOORDHIP_CPUEXCL_PCPU 1u
#define KOORDHIP_CPUEXCL_NUMA 2u
#define KOORDHIP_NUMA_REQUIRED(p) ((p) & 3u)
#define KOORDHIP_NUMA_PREFERRED(p) (((p) >> 2) & 3u)
#define KOORDHIP_NUMA_EXCLUSIVE(p) (((p) >> 4) & 3u)

/* koordhip_node_soa.numa_flags: node CPU bind policy (GetNodeCPUBindPolicy,
 * apis/extension/numa_aware.go:314-325) and NUMA allocate strategy
 * (GetNUMAAllocateStrategy, nodenumaresource/util.go:34-40). */
#define KOORDHIP_NODE_CPUBIND_MASK 3u   /* 0 None, 1 FullPCPUsOnly, 2 SpreadByPCPUs */
#define KOORDHIP_NODE_NUMA_MOST_ALLOCATED 4u
/* bits 3-4: the node's NUMA topology policy (getNUMATopologyPolicy: label
 * node.koordinator.sh/numa-topology-policy over the NRT's policy,
 * nodenumaresource/util.go; apis/extension/numa_aware.go:56-64) */
#define KOORDHIP_NODE_NUMA_POLICY_SHIFT 3
#define KOORDHIP_NODE_NUMA_POLICY(f) (((f) >> KOORDHIP_NODE_NUMA_POLICY_SHIFT) & 3u)
#define KOORDHIP_NUMA_TOPO_NONE 0u
#define KOORDHIP_NUMA_TOPO_BEST_EFFORT 1u
#define KOORDHIP_NUMA_TOPO_RESTRICTED 2u
#define KOORDHIP_NUMA_TOPO_SINGLE_NUMA_NODE 3u
/* NUMA zones (NRT zones "node-<k>", zone k = NUMA node rank k) of a node with
 * a topology policy: up to this many (hint merge over <= 255 masks per
 * (pod, node), e.g. a 2-socket host in NPS4 mode). */
#define KOORDHIP_NUMA_MAX_ZONES 8

/* CPU topology of a node (cpu_topology.go:25-103), shared by every node of
 * the same shape.  CPU "positions" are core-major: pos = core_rank *
 * cpus_per_core + t, cores in ascending CoreID, t in ascending CPU id, so one
 * bit per position in a 4 x 64-bit mask.  NUMA nodes and sockets are ranked
 * by ascending id.  Every core must hold exactly cpus_per_core CPUs. */
#define KOORDHIP_NUMA_MAX_CPUS 256
#define KOORDHIP_NUMA_MAX_NODES 8
#define KOORDHIP_NUMA_WORDS 4
typedef struct koordhip_numa_class {
  int32_t num_cpus, num_cores, num_nodes, num_sockets; /* CPUTopology counters (builder semantics) */
  int32_t cpus_per_core;
  int32_t reserved0;
  int32_t cpu_id[KOORDHIP_NUMA_MAX_CPUS];       /* pos -> logical CPU id */
  uint8_t node_of[KOORDHIP_NUMA_MAX_CPUS];      /* pos -> NUMA node rank */
  uint8_t socket_of[KOORDHIP_NUMA_MAX_CPUS];    /* pos -> socket rank */
} koordhip_numa_class;

/* Per-(pod,node) status bits written by koordhip_eval (no short-circuit, one
 * bit per plugin that returned non-Success from Filter). */
#define KOORDHIP_ST_FIT_FAIL 1u
#define KOORDHIP_ST_LA_FAIL 2u
#define KOORDHIP_ST_NUMA_FAIL 4u
#define KOORDHIP_ST_RESV_FAIL 8u  /* filterWithReservations (reservation/plugin.go:373-440) */
#define KOORDHIP_ST_STATIC_FAIL 16u /* NodeUnschedulable / NodeAffinity / TaintToleration */
#define KOORDHIP_ST_DEVICE_FAIL 32u /* DeviceShare Filter (plugin.go:284-323) */
#define KOORDHIP_ST_XFIT_FAIL 64u   /* NodeResourcesFit on an extended scalar resource (koordhip_pod_ext.xreq) */
#define KOORDHIP_ST_PTS_FAIL 128u   /* PodTopologySpread Filter (a missing topology key, or the skew) */
#define KOORDHIP_ST_IPA_FAIL 256u   /* InterPodAffinity Filter (koordhip_eval_ext's 16-bit status only) */

/* DeviceShare's device model (nodeDevice, device_cache.go:44-50): per node
 * and device type up to KOORDHIP_DEV_SLOTS minors, each with the Device CR's
 * resources (deviceTotal) and what pods hold (deviceUsed); free = total - used
 * clamped at 0 per resource (resetDeviceFree, :185-202). */
#define KOORDHIP_DEV_TYPES 3  /* 0 gpu, 1 rdma, 2 fpga (DeviceResourceNames, device_resources.go:42-53) */
#define KOORDHIP_DEV_GPU 0
#define KOORDHIP_DEV_RDMA 1
#define KOORDHIP_DEV_FPGA 2
#define KOORDHIP_DEV_SLOTS 8  /* minors per type per node */
#define KOORDHIP_DEV_RES 3    /* gpu: [0] koordinator.sh/gpu-core, [1] gpu-memory-ratio, [2] gpu-memory (bytes);
                                 rdma / fpga: [0] koordinator.sh/rdma | fpga */

/* place_stream out_node values */
#define KOORDHIP_UNSCHEDULABLE (-1)
#define KOORDHIP_RESERVE_FAILED (-2)

typedef struct koordhip_ctx koordhip_ctx;

/* Plugin arguments (pkg/scheduler/apis/config/types.go:29-108, defaults
 * v1beta2/defaults.go:32-121, weights scheduler-config.yaml:82-91). */
typedef struct koordhip_config {
  int32_t abi_version;      /* must be KOORDHIP_ABI_VERSION */
  uint32_t filter_plugins;  /* KOORDHIP_PLUGIN_* bits enabled at Filter */
  uint32_t score_plugins;   /* KOORDHIP_PLUGIN_* bits enabled at Score */
  int32_t device;           /* HIP device ordinal; -1 = current device */
  int64_t plugin_weight[KOORDHIP_NPLUGINS]; /* score weight: Fit, LoadAware, NUMA, BalancedAllocation (1..100) */
  int64_t fit_weight[KOORDHIP_NRES];        /* NodeResourcesFitArgs LeastAllocated weights, 0 = resource not listed */
  int64_t la_weight_cpu;                    /* LoadAwareSchedulingArgs.ResourceWeights[cpu] (1..100) */
  int64_t la_weight_mem;                    /* LoadAwareSchedulingArgs.ResourceWeights[memory] (1..100) */
  int32_t la_score_according_prod_usage;    /* LoadAwareSchedulingArgs.ScoreAccordingProdUsage */
  int32_t batch_pods;       /* pods per pipelined round of place_stream (0 = default: 32, 16 with NodeNUMAResource; max 64) */
  int32_t numa_weight_cpu;  /* NodeNUMAResourceArgs.ScoringStrategy LeastAllocated weights */
  int32_t numa_weight_mem;
  int32_t profile_kernels;  /* 1 = time every stream eval launch with HIP events (koordhip_last_stats) */
  int32_t numa_most_allocated; /* NodeNUMAResourceArgs.ScoringStrategy.Type == MostAllocated
                                  (nodenumaresource/most_allocated.go:30-62); 0 = LeastAllocated */
  int32_t reservation_weight;  /* Reservation score weight (scheduler-config.yaml:90-91: 5000); must exceed
                                  100 x the sum of the other score weights (Reservation key) */
  int32_t reserved[5];
  /* ABI 9: the normalized-score plugins */
  int32_t ext_weight[KOORDHIP_NEXT_PLUGINS]; /* score weights: DeviceShare (scheduler-config.yaml:88-89: 1),
                                               NodeAffinity, TaintToleration, PodTopologySpread,
                                               InterPodAffinity (1..100) */
  int32_t dev_most_allocated;  /* DeviceShareArgs.ScoringStrategy.Type == MostAllocated (scoring.go:125-132) */
  int32_t dev_res_weight[5];   /* DeviceShareArgs.ScoringStrategy.Resources weights (0 = not listed): gpu-core,
                                  gpu-memory-ratio, gpu-memory, rdma, fpga (defaults v1beta2/defaults.go:168-189:
                                  gpu-memory-ratio, rdma, fpga at 1) */
  int32_t reserved2[1];
} koordhip_config;

/* Columnar node snapshot, all arrays of length n, little-endian, caller-owned
 * and copied by koordhip_load_snapshot.  Units: CPU in milli-cores, memory /
 * ephemeral storage in bytes, batch-cpu as Quantity.Value().  Mutable columns
 * (requested / nz / npods / la_used*) are advanced on device by commits. */
typedef struct koordhip_node_soa {
  /* NodeResourcesFit: NodeInfo.Allocatable (upstream framework/types.go) */
  const int64_t *alloc[KOORDHIP_NRES];
  const int32_t *alloc_pods;               /* Allocatable.AllowedPodNumber */
  /* NodeResourcesFit: NodeInfo.Requested, .NonZeroRequested, len(.Pods) */
  const int64_t *requested[KOORDHIP_NRES];
  const int64_t *nz_cpu_m;
  const int64_t *nz_mem;
  const int32_t *npods;
  /* LoadAwareScheduling Score (load_aware.go:269-335) */
  const int64_t *la_alloc_cpu_m;           /* EstimateNode(node)[cpu].MilliValue() (default_estimator.go:110-129) */
  const int64_t *la_alloc_mem;             /* EstimateNode(node)[memory].Value() */
  const int64_t *la_used_cpu_m;            /* assigned-pod estimates + nodeUsage (cond. minus estimated pods' actual) */
  const int64_t *la_used_mem;
  const int64_t *la_used_prod_cpu_m;       /* prod-pod variant (ScoreAccordingProdUsage); may be NULL otherwise */
  const int64_t *la_used_prod_mem;
  /* LoadAwareScheduling Filter inputs (load_aware.go:173-254), milli values */
  const int64_t *laf_used_m[2];            /* nodeUsage (or target aggregated usage) cpu, memory: MilliValue() */
  const int64_t *laf_total_m[2];           /* EstimateNode allocatable cpu, memory: MilliValue() */
  const int64_t *laf_prod_used_m[2];       /* sum of prod pods' usage (buildPodMetricMap+sumPodUsages) */
  const int64_t *laf_thr[2];               /* resolved usage thresholds cpu, memory (0 = disabled) */
  const int64_t *laf_prod_thr[2];          /* resolved prod usage thresholds (0 = disabled) */
  const uint8_t *la_flags;                 /* KOORDHIP_LA_* */
  /* NodeNUMAResource (TopologyOptions + NodeAllocation, topology_options.go:40-48,
   * node_allocation.go:32-38); all NULL / n_numa_classes = 0 when unused */
  const koordhip_numa_class *numa_classes;
  int32_t n_numa_classes;
  int32_t reserved0;
  const int32_t *numa_class;               /* class index, -1 = no (valid) CPU topology */
  const uint64_t *numa_free[KOORDHIP_NUMA_WORDS];      /* available CPUs: all - refcount>=1 - ReservedCPUs (node_allocation.go:133-153) */
  const uint64_t *numa_excl_pcpu[KOORDHIP_NUMA_WORDS]; /* allocated CPUs whose ExclusivePolicy is PCPULevel */
  const uint64_t *numa_excl_numa[KOORDHIP_NUMA_WORDS]; /* allocated CPUs whose ExclusivePolicy is NUMANodeLevel */
  const int32_t *numa_alloc_cnt;           /* |allocatedCPUs| (scoring.go:161-166) */
  const uint8_t *numa_flags;               /* KOORDHIP_NODE_* */
  /* NUMA zone resources, [n][2][KOORDHIP_NUMA_MAX_NODES] row-major, [.][0][k] cpu
   * (milli), [.][1][k] memory (bytes) of zone k: NRT zone allocatable
   * (TopologyOptions.NUMANodeResources, topology_options.go:181-211) and the
   * amounts allocated by pods (NodeAllocation.allocatedResources,
   * node_allocation.go:76-103).  Read only for nodes with a topology policy;
   * NULL when no node has one. */
  const int64_t *numa_zone_alloc;
  const int64_t *numa_zone_used;
  /* CPU amplification ratio of the node (annotation node.koordinator.sh/
   * resource-amplification-ratio, apis/extension/node_resource_amplification.go:
   * 56-76; the same ratio the NodeResourceTopology carries): NodeNUMAResource's
   * filterAmplifiedCPUs / scoreWithAmplifiedCPUs / amplified cpuset requests
   * (plugin.go:326-363, scoring.go:95-168).  NULL or <= 1: not amplified. */
  const double *numa_amp_cpu;
  /* Reservation (KOORDHIP_PLUGIN_RESERVATION): the node's Available reservation,
   * KOORDHIP_RESV_* flags (NULL = no reservations), the rank of its order label
   * among the snapshot's distinct orders (ascending, smaller order = preferred),
   * ReservationInfo.Allocatable / .Allocated (cpu milli, memory bytes; masked to
   * ResourceNames) and len(AssignedPods).  Allocated / assigned are advanced by
   * commits of pods the reservation is nominated for.  resv_nz: the reserve
   * pod's non-zero cpu / memory request (calculateResource, transformer.go:
   * 302-333; Requested of the reserve pod is resv_alloc). */
  const uint32_t *resv_flags;
  const int32_t *resv_order_rank;
  const int64_t *resv_alloc[2];
  const int64_t *resv_nz[2];
  const int64_t *resv_allocated[2];
  const int32_t *resv_assigned;
  /* KOORDHIP_PLUGIN_NODE_STATIC: bit c set = pods of static class c pass
   * NodeUnschedulable, NodeAffinity and TaintToleration's Filter on this node
   * (the node's labels, taints and spec.unschedulable against the class's
   * nodeSelector, required affinity and tolerations); NULL = every class. */
  const uint32_t *static_allow;
  /* Reservation slots per node held by the resv_* columns: 0 or 1 = one
   * reservation per node (columns of n values); S in [2, KOORDHIP_RESV_SLOTS_MAX]
   * = up to S per node (S > KOORDHIP_RESV_SLOTS: the sequential cycle places), every resv_* column then holds S x n values,
   * slot-major (slot s of node i at [s * n + i]); a node's reservations fill
   * its slots from 0, unused slots have resv_flags 0.  koordhip_update_nodes
   * rows use the loaded snapshot's slot count. */
  int32_t resv_slots;
  int32_t reserved1;
  /* NodeNUMAResource's reservation restore (RestoreReservation,
   * nodenumaresource/reservation.go:76-113): per reservation slot, the CPUs of
   * the reservation's cpuset allocation not held by its AssignedPods (core-major
   * positions of the node's topology class, slot-major like the resv_* columns).
   * These CPUs are allocated in the node's NodeAllocation (not in numa_free).  A
   * cpuset pod nominated into the reservation (PreScore) takes them first
   * (takePreferredCPUs, cpu_accumulator.go:29-85) at Score and Reserve; a
   * Reserve removes the pod's CPUs.  NULL = no reservation holds CPUs (also
   * the update_nodes default). */
  const uint64_t *resv_cpus[KOORDHIP_NUMA_WORDS];
  /* ---- ABI 9 (read only by the sequential cycle, koordhip_place_stream_ext) */
  /* DeviceShare: minors per type per node held by the dev_* columns (0 = no
   * devices anywhere: the columns may be NULL); dev_minor [n][TYPES][dev_slots]
   * in ascending minor order, -1 = empty slot; dev_total / dev_used
   * [n][TYPES][dev_slots][RES]: the minor's Device CR resources (all 0 for an
   * unhealthy device, buildDeviceResources device_cache.go:550-568) and the
   * amounts pods hold (advanced by Reserve) */
  int32_t dev_slots;
  int32_t reserved2;
  const uint8_t *dev_present;  /* [n] 1 = the node has a nodeDevice entry (a Device CR); without one DeviceShare's
                                  Filter passes, its Score is 0 and its Reserve allocates nothing (plugin.go:298-301,
                                  scoring.go:42-45, :377-380) */
  const int32_t *dev_minor;
  const int64_t *dev_total;
  const int64_t *dev_used;
  /* NodeResourcesFit extended scalars [KOORDHIP_NXRES][n]: Allocatable and
   * Requested (advanced by Reserve); NULL = 0 */
  const int64_t *xalloc;
  const int64_t *xrequested;
  /* raw NodeAffinity (sum of the weights of the class's preferred terms that
   * match) and TaintToleration (count of PreferNoSchedule taints the class does
   * not tolerate) scores per (pod static class, node), [MAX_STATIC_CLASSES][n];
   * NULL = 0 */
  const uint16_t *static_score[2];
  /* PodTopologySpread (KOORDHIP_PLUGIN_PTS): the topology keys of the
   * snapshot's constraints (pts_keys <= KOORDHIP_PTS_KEYS; bit k of
   * pts_hostname: key k is kubernetes.io/hostname, whose domain is the node
   * itself), pts_dom [keys][n] = the node's domain for key k (0 ..
   * pts_ndom[k] - 1 < KOORDHIP_PTS_DOMAINS; the node index for a hostname key;
   * -1 = the node has no such label); the constraint table (pts_cons <=
   * KOORDHIP_PTS_CONS distinct (label selector, namespace), pts_cons_key[c] =
   * its key) with pts_cnt [cons][n] = the node's pods in that namespace the
   * selector matches (countPodsMatchSelector; advanced by Reserve); pts_elig [n]
   * bit 2s = the node matches spread class s's required node affinity and holds
   * every DoNotSchedule key of the class, bit 2s + 1 = ... every ScheduleAnyway
   * key (pts_classes <= KOORDHIP_PTS_CLASSES).  pts_keys 0: no columns. */
  int32_t pts_keys;
  uint32_t pts_hostname;
  int32_t pts_ndom[KOORDHIP_PTS_KEYS];
  int32_t pts_cons;
  int32_t pts_classes;
  int32_t pts_cons_key[KOORDHIP_PTS_CONS];
  const int32_t *pts_dom;
  const int32_t *pts_cnt;
  const uint16_t *pts_elig;
  /* InterPodAffinity (KOORDHIP_PLUGIN_IPA): count entries over the pts_* topology
   * keys (ipa_ents <= KOORDHIP_IPA_ENTRIES, entry e on key ipa_ent_key[e]); ipa_cnt
   * [ents][n] = the node's pods entry e counts (advanced by Reserve): a "match"
   * entry counts the pods a term (or, for a pod's required affinity, all of its
   * terms) matches, a "carry" entry the pods that carry an affinity term.  The
   * pod-side masks and weights (koordhip_pod_ext.ipa_*) say which entries a pod
   * reads and how; the domain sums over the nodes of a (key, value) pair are the
   * reference's topologyPair counts.  ipa_ents 0: no columns. */
  int32_t ipa_ents;
  int32_t ipa_reserved;
  int32_t ipa_ent_key[KOORDHIP_IPA_ENTRIES];
  const int32_t *ipa_cnt;
  /* ABI 13: DeviceShare with a reservation holding devices (the reservation
   * restore, deviceshare/reservation.go:119-170; Filter / FilterReservation /
   * Score / ScoreReservation / Reserve through tryAllocateFromReservation
   * :181-283 and the nominated reservation :365-443).  resv_dev_slot [n]: the
   * reservation slot (0 .. max(resv_slots, 1) - 1) of node i's one reservation
   * holding devices, -1 = none (at most one per node: the host rejects more).
   * resv_dev [n][2][TYPES][dev_slots][RES]: [0] that reservation's allocatable
   * (its reserve pod's device allocation, nd.getUsed(reservePod)) and [1] its
   * allocated (its AssignedPods' allocations on those minors,
   * appendAllocatedByHints :145-151; advanced by Reserve).  Both allocations
   * are also in dev_used, as in the reference's deviceUsed.  NULL = none.  The
   * sequential cycle places batches on such snapshots. */
  const int32_t *resv_dev_slot;
  const int64_t *resv_dev;
  /* ABI 14: the NodeResourcesFit extended scalars of that reservation
   * (koordinator.sh/gpu-core, nvidia.com/gpu, ...; the KOORDHIP_NXRES slots of
   * xalloc): resv_xalloc [NXRES][n] = its Allocatable's scalars (the reserve
   * pod's scalar requests; a scalar it lists must be > 0: the host rejects a
   * zero-valued key), resv_xallocated [NXRES][n] = its Allocated's (its
   * AssignedPods' scalar requests masked to those keys, reservation_info.go:
   * 297-306; advanced by Reserve).  0 on nodes whose resv_dev_slot is -1.  They
   * enter every rule the reference applies to a reservation's ResourceList:
   * the restore of NodeInfo.Requested's scalars (RemovePod of the reserve pod
   * for a matched reservation, -Allocatable + SubtractWithNonNegativeResult(
   * Allocatable, Allocated) for an unmatched one with assigned pods,
   * transformer.go:227-293), filterWithReservations' fitsNode over the pod's
   * scalars (plugin.go:445-494), Restricted's LessThanOrEqual (:420-432),
   * FilterReservation's intersection (:504-535), scoreReservation's
   * MostAllocated over RemoveZeros(Allocatable) (scoring.go:177-200) and the
   * Reserve's AddAssignedPod.  NULL = none.  A snapshot with a non-zero value
   * places every batch in the sequential cycle (koordhip_eval refuses it: use
   * koordhip_eval_ext). */
  const int64_t *resv_xalloc;
  const int64_t *resv_xallocated;
} koordhip_node_soa;

/* One pod of the stream, the host-side PreFilter product (96 bytes). */
typedef struct koordhip_pod {
  int64_t req[KOORDHIP_NRES]; /* computePodResourceRequest (upstream fit.go): max(sum containers, init) + overhead */
  int64_t nz_cpu_m;           /* non-zero request: GetNonzeroRequests defaults 100m / 200Mi (upstream) */
  int64_t nz_mem;
  int64_t est_cpu;            /* EstimatePod(pod)[cpu]    (default_estimator.go:57-108) */
  int64_t est_mem;            /* EstimatePod(pod)[memory] */
  uint32_t flags;             /* KOORDHIP_POD_* */
  int32_t numa_cpus;          /* NUMA numCPUsNeeded (plugin.go:252) */
  uint32_t numa_policy;       /* KOORDHIP_NUMA_* packed policies */
  int32_t static_class;       /* KOORDHIP_PLUGIN_NODE_STATIC: the pod's class (0 .. MAX_STATIC_CLASSES-1): pods
                                 of one class share nodeSelector, required node affinity and tolerations */
  uint64_t resv_match;        /* bit g: MatchReservationOwners(pod, owner group g) (util/reservation/reservation.go:389-410) */
} koordhip_pod;

/* Per-pod inputs of the normalized-score plugins (the host's DeviceShare
 * PreFilter: PreparePod, plugin.go:162-182), beside koordhip_pod. */
typedef struct koordhip_pod_ext {
  /* ConvertDeviceRequest of each type's request (utils.go:86-181): gpu [0]
   * core, [1] memory-ratio, [2] memory bytes, -1 = key absent (memory and
   * ratio are completed per node from its GPU memory, fillGPUTotalMem
   * utils.go:211-233); rdma / fpga [t][0], 0 = none */
  int64_t dev_req[KOORDHIP_DEV_TYPES][KOORDHIP_DEV_RES];
  int64_t xreq[KOORDHIP_NXRES];  /* NodeResourcesFit extended scalar requests */
  uint32_t flags;                /* KOORDHIP_PODX_* */
  uint32_t xmask;                /* bit j: the pod's request map holds extended scalar j (xreq[j], even 0) */
  /* PodTopologySpread: the pod's spec.topologySpreadConstraints in order
   * (pts_n <= KOORDHIP_PTS_POD): pts_c[j] = its constraint table index,
   * pts_fl[j] KOORDHIP_PTS_HARD (DoNotSchedule) / KOORDHIP_PTS_SELF (its
   * selector matches the pod's own labels), pts_skew[j] = maxSkew; pts_class =
   * the pod's spread class; pts_match bit c = table constraint c counts this
   * pod once it is placed (its namespace and selector match). */
  uint8_t pts_n;
  uint8_t pts_class;
  uint8_t pts_match;
  uint8_t pts_pad;
  uint8_t pts_c[KOORDHIP_PTS_POD];
  uint8_t pts_fl[KOORDHIP_PTS_POD];
  int32_t pts_skew[KOORDHIP_PTS_POD];
  int32_t reserve_node;  /* KOORDHIP_POD_RESERVE: 1 + the node index its reservation names
                            (GetReservePodNodeName, plugin.go:335-339), 0 = any node */
  /* InterPodAffinity, bit e = count entry e of the snapshot:
   *   ipa_inc   entries that count this pod once it is placed (NodeInfo.AddPod)
   *   ipa_aff   its required affinity terms' entry per topology key: a node
   *             passes when it has every key and each pair counts > 0, or when
   *             no pair counts anywhere and KOORDHIP_IPA_SELF (satisfyPodAffinity)
   *   ipa_anti  its required anti-affinity terms' entries and the existing
   *             pods' required anti-affinity terms that match it: a node fails
   *             when one of them counts > 0 in the node's pair
   *   ipa_score entries with a nonzero ipa_w: raw Score = sum of ipa_w[e] x the
   *             pair count of e at the node (the reference's topologyScore) */
  uint32_t ipa_inc;
  uint32_t ipa_aff;
  uint32_t ipa_anti;
  uint32_t ipa_score;
  uint32_t ipa_flags;
  int32_t ipa_reserved;
  int32_t ipa_w[KOORDHIP_IPA_ENTRIES];
} koordhip_pod_ext;
#define KOORDHIP_PODX_DEVICE 1u  /* some device request (DeviceShare state.skip == false) */
#define KOORDHIP_PTS_HARD 1u
#define KOORDHIP_PTS_SELF 2u
#define KOORDHIP_IPA_SELF 1u     /* the pod matches all of its own required affinity terms */

/* One top-k record of koordhip_eval. */
typedef struct koordhip_topk {
  int32_t node;   /* node index, -1 = none */
  int32_t score;  /* total weighted score */
} koordhip_topk;

/* ---- lifecycle ---------------------------------------------------------- */
const char *koordhip_last_error(void);
int koordhip_abi_version(void);
int koordhip_create(const koordhip_config *cfg, koordhip_ctx **out);
int koordhip_destroy(koordhip_ctx *ctx);

/* Copy a full snapshot of n nodes to device (replaces any previous one) and
 * run the on-device LoadAware threshold-mask kernel. */
int koordhip_load_snapshot(koordhip_ctx *ctx, const koordhip_node_soa *soa, int32_t n);

/* Replace rows idx[0..m) with rows 0..m of `rows` (informer deltas) and
 * recompute their masks. */
int koordhip_update_nodes(koordhip_ctx *ctx, const int32_t *idx, const koordhip_node_soa *rows, int32_t m);

/* Copy the current (committed) mutable columns back to host arrays; any
 * pointer may be NULL.  Used by tests and the Go shim's debug service. */
int koordhip_read_nodes(koordhip_ctx *ctx, int64_t *requested /* [NRES][n] */, int64_t *nz /* [2][n] */,
                        int32_t *npods, int64_t *la_used /* [2][n] */, int64_t *la_used_prod /* [2][n] */);
/* NodeNUMAResource mutable state: free / exclusive masks [WORDS][n], allocated CPU counts [n]. */
int koordhip_read_numa(koordhip_ctx *ctx, uint64_t *free_mask, uint64_t *excl_pcpu, uint64_t *excl_numa,
                       int32_t *alloc_cnt);
/* ... and the NUMA zone allocations, [n][2][KOORDHIP_NUMA_MAX_NODES] like numa_zone_used
 * (rows of nodes without a topology policy read as 0: the engine does not keep them). */
int koordhip_read_numa_zones(koordhip_ctx *ctx, int64_t *zone_used);
/* Reservation mutable state: Allocated [2][S n] (cpu milli, memory), len(AssignedPods) [S n],
 * S = the loaded snapshot's reservation slots (1 when resv_slots <= 1), slot-major like the columns. */
int koordhip_read_reservations(koordhip_ctx *ctx, int64_t *allocated, int32_t *assigned);
/* ... and the reservations' remaining reserved CPUs [WORDS][S n] (zeros when no loaded reservation holds CPUs). */
int koordhip_read_resv_cpus(koordhip_ctx *ctx, uint64_t *cpus);
/* ABI 13: the loaded resv_dev column [n][2][TYPES][dev_slots][RES] (its
 * allocated half advanced by Reserve); zeros without one. */
int koordhip_read_resv_devices(koordhip_ctx *ctx, int64_t *resv_dev);
/* ABI 14: the loaded resv_xallocated column [NXRES][n] (advanced by Reserve);
 * zeros without one. */
int koordhip_read_resv_scalars(koordhip_ctx *ctx, int64_t *resv_xallocated);

/* Parity/debug mode, no commit: for n_pods pods against the current state.
 *   status : optional, [n_pods][n] KOORDHIP_ST_* bits (every plugin evaluated)
 *   scores : optional, [n_pods][KOORDHIP_NPLUGINS][n] per-plugin scores (0 where the plugin is disabled;
 *            the NodeNUMAResource score of a pair failing the NUMA Filter is unspecified, as the
 *            framework never scores such a node)
 *   topk   : optional, [n_pods][k] best feasible nodes by (total desc, index asc), node = -1 past the end
 *            (with the Reservation plugin, `score` is the ranking total of DESIGN.md's Reservation key:
 *            its order equals the order of the normalized weighted sums for the pod) */
int koordhip_eval(koordhip_ctx *ctx, const koordhip_pod *pods, int32_t n_pods, uint8_t *status, int32_t *scores,
                  koordhip_topk *topk, int32_t k);

/* ABI 9: the same with koordhip_pod_ext records (ext may be NULL: no device
 * requests), for every profile, including the normalized-score plugins.
 * status: [n_pods][n] 16-bit KOORDHIP_ST_* bits (incl. KOORDHIP_ST_IPA_FAIL).
 * scores: [n_pods][KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS][n], planes
 * NPLUGINS.. the raw (un-normalized) DeviceShare / NodeAffinity /
 * TaintToleration / PodTopologySpread (feasible nodes) / InterPodAffinity
 * (every node) scores; topk ranks the normalized weighted sums. */
int koordhip_eval_ext(koordhip_ctx *ctx, const koordhip_pod *pods, const koordhip_pod_ext *ext, int32_t n_pods,
                      uint16_t *status, int32_t *scores, koordhip_topk *topk, int32_t k);

/* Greedy stream: pods attempted once, in order, each against the state left
 * by all earlier commits; winner = lowest-index max total score; the Reserve
 * delta is applied on device.  out_node[i] = node, -1 unschedulable, -2 the
 * winner's Reserve failed (NodeNUMAResource Allocate; nothing committed, no
 * retry). */
int koordhip_place_stream(koordhip_ctx *ctx, const koordhip_pod *pods, int32_t n_pods, int32_t *out_node);
/* ABI 9: the greedy stream with koordhip_pod_ext records (ext may be NULL).
 * A profile enabling a normalized-score plugin (DeviceShare, NodeAffinity /
 * TaintToleration Score) runs the exact sequential cycle: per pod, every node
 * is filtered and scored on the state all earlier commits left, the
 * normalized plugins' maxima are reduced over the feasible nodes, then the
 * lowest-index argmax commits -- one persistent launch over every CU. */
int koordhip_place_stream_ext(koordhip_ctx *ctx, const koordhip_pod *pods, const koordhip_pod_ext *ext,
                              int32_t n_pods, int32_t *out_node);
/* Devices each pod of the last place call got: [n_pods][KOORDHIP_DEV_TYPES]
 * bit s = dev slot s of its node (the DeviceAllocations PreBind writes,
 * plugin.go:465-478: every allocated minor holds the pod's per-card request). */
int koordhip_fetch_devices(koordhip_ctx *ctx, uint32_t *slots, int32_t n_pods);
/* DeviceShare and extended-scalar mutable state: dev_used [n][TYPES][dev_slots][RES],
 * xrequested [NXRES][n] (either may be NULL). */
int koordhip_read_devices(koordhip_ctx *ctx, int64_t *dev_used, int64_t *xrequested);
/* PodTopologySpread: each table constraint's matching pods per node after the
 * last place call, [pts_cons][n] (NodeInfo.AddPod of the placed pods). */
int koordhip_read_pts(koordhip_ctx *ctx, int32_t *cnt);
/* InterPodAffinity: each count entry's pods per node after the last place
 * call, [ipa_ents][n]. */
int koordhip_read_ipa(koordhip_ctx *ctx, int32_t *cnt);

/* The same split in two so a caller can time the device part alone: stage
 * (host -> HBM copy) then place (HBM-resident pods, result kept on device
 * until koordhip_fetch_placements). */
int koordhip_stage_pods(koordhip_ctx *ctx, const koordhip_pod *pods, int32_t n_pods);
/* ABI 9: stage pods with their koordhip_pod_ext records (ext may be NULL),
 * for koordhip_place_staged on a sequential-cycle profile. */
int koordhip_stage_pods_ext(koordhip_ctx *ctx, const koordhip_pod *pods, const koordhip_pod_ext *ext,
                            int32_t n_pods);
int koordhip_place_staged(koordhip_ctx *ctx);
int koordhip_fetch_placements(koordhip_ctx *ctx, int32_t *out_node, int32_t n_pods);
int koordhip_synchronize(koordhip_ctx *ctx);

/* Device-side checkpoint of the mutable columns (requested / nz / npods /
 * la_used* / flags) and its restore: rolls a whole speculative cycle back
 * (bulk Unreserve) without re-uploading the snapshot. */
int koordhip_checkpoint(koordhip_ctx *ctx);
int koordhip_restore(koordhip_ctx *ctx);

/* Reserve / Unreserve of one pod on one node (state delta only).  For a
 * cpuset pod the NodeNUMAResource Reserve allocates CPUs (the exact
 * cpuAccumulator choice, cpu_accumulator.go:87-232); cpus_out (optional,
 * KOORDHIP_NUMA_WORDS words, core-major positions) receives them, and
 * KOORDHIP_ERESERVE means Allocate failed and nothing was committed.
 * Unreserve of a cpuset pod takes the CPUs it was given. */
int koordhip_commit(koordhip_ctx *ctx, const koordhip_pod *pod, int32_t node, uint64_t *cpus_out);
int koordhip_uncommit(koordhip_ctx *ctx, const koordhip_pod *pod, int32_t node, const uint64_t *cpus);

/* ABI 12: Reserve / Unreserve of one pod WITH its koordhip_pod_ext record on
 * one node -- the same Reserve the sequential cycle runs on its winner:
 *   DeviceShare Reserve   <- deviceshare/plugin.go:368-405 (allocator.go:91-122: the
 *                            device choice; deviceUsed += the per-device request)
 *   DeviceShare Unreserve <- deviceshare/plugin.go:407-426 (deviceUsed -= it)
 *   NodeResourcesFit      <- the extended scalars' Requested (xrequested) +/- xreq
 *   PodTopologySpread / InterPodAffinity <- upstream AddPod / RemovePod of the
 *                            placed pod: pts_cnt / ipa_cnt of the constraints and
 *                            entries it counts for (pts_match, ipa_inc) +/- 1
 * plus everything koordhip_commit does (Fit / LoadAware, NodeNUMAResource,
 * Reservation).  Reserve assumes the cycle ran PreScore (more than one
 * feasible node: a matched reservation is nominated).  dev_slots_out /
 * dev_slots ([KOORDHIP_DEV_TYPES], bit s = device slot s of the type, as
 * koordhip_fetch_devices): what Reserve took, what Unreserve returns.
 * KOORDHIP_ERESERVE: Reserve failed and nothing was applied.  Unreserve is
 * refused (KOORDHIP_EINVAL) where koordhip_uncommit is. */
int koordhip_commit_ext(koordhip_ctx *ctx, const koordhip_pod *pod, const koordhip_pod_ext *ext, int32_t node,
                        uint64_t *cpus_out, uint32_t *dev_slots_out);
int koordhip_uncommit_ext(koordhip_ctx *ctx, const koordhip_pod *pod, const koordhip_pod_ext *ext, int32_t node,
                          const uint64_t *cpus, const uint32_t *dev_slots);

/* CPUs allocated to each pod of the last place call ([n_pods][KOORDHIP_NUMA_WORDS],
 * zero for non-cpuset pods): what PreBind writes into the resource-status
 * annotation (plugin.go:425-453). */
int koordhip_fetch_cpusets(koordhip_ctx *ctx, uint64_t *cpus, int32_t n_pods);

/* Device-time of the last place call's eval kernels, split for roofline
 * accounting: total ms of eval kernels, launches, evals processed. */
int koordhip_last_stats(koordhip_ctx *ctx, double *eval_ms, int64_t *eval_launches, int64_t *evals,
                        double *total_ms);

/* Per-kernel device time of the last place call (profile_kernels = 1: HIP
 * event pairs on the stream each kernel is launched on): the evaluation
 * (k_scan), the top-k selection (k_select_split / k_select) and the
 * sequential resolve (k_resolve; one persistent launch per call unless the
 * context is in a local group).  Roofline accounting in bench.py. */
typedef struct koordhip_kernel_stats {
  /* *_ms / *_launches: the timed launches only -- a persistent pipeline times
   * the evaluation launches of ~256 evenly spaced rounds (their averages are
   * what the sample is for); `rounds` counts every round */
  double scan_ms;
  int64_t scan_launches;
  double select_ms;
  int64_t select_launches;
  double resolve_ms;
  int64_t resolve_launches;
  double total_ms;   /* the place call, first to last event on the engine stream */
  int64_t evals;     /* (pod, node) pairs evaluated by this rank */
  int64_t pods;      /* pods of the staged stream */
  int64_t rounds;    /* pipelined rounds */
  int64_t round_pods; /* pods per round (batch_pods, LDS-clamped) */
  int64_t lag;        /* pipeline depth: round r's lists see the state after round r - 1 - lag */
  int64_t executed_evals; /* (pod, node) evaluations actually run: class-list builds + incremental
                            * re-evaluations + device pods' pre-evaluations and final re-evaluations
                            * (evals is the equivalent work: every pair decided exactly) */
  int32_t plan_us;        /* host time of the class-list plan of the call */
  int32_t flags;          /* KOORDHIP_KSTAT_LOCAL: a sharded rank ran the full table (no exchange) */
} koordhip_kernel_stats;
#define KOORDHIP_KSTAT_LOCAL 1
int koordhip_last_kernel_stats(koordhip_ctx *ctx, koordhip_kernel_stats *out);
/* Turn the per-launch event timing on / off for later place calls (the
 * events cost a few microseconds per round: bench.py times its steps with it
 * off and takes the per-kernel split from one extra step). */
int koordhip_set_profile_kernels(koordhip_ctx *ctx, int32_t on);
/* The template instantiations the last place call launched for its evaluation
 * (k_scan / k_eval_topk) and its resolve, spelled as rocprofv3 names them
 * ("kh::k_scan<4, 0>"), NUL-terminated in buffers of `cap` bytes -- so a
 * profile can be matched to the exact kernel a timed run used. */
int koordhip_last_kernel_names(koordhip_ctx *ctx, char *eval_out, char *resolve_out, int32_t cap);

/* ---- multi-GPU (node-index sharding, RCCL all-gather of per-shard top-k) -- */
#define KOORDHIP_UNIQUE_ID_BYTES 128
int koordhip_comm_unique_id(uint8_t *id_out /* KOORDHIP_UNIQUE_ID_BYTES */);
/* Attach an RCCL communicator: this context then evaluates only node shard
 * [rank*n/world, (rank+1)*n/world) and merges per-shard top-k over xGMI.
 * world == 1 attaches a one-rank communicator: the whole table, through the
 * same per-round all-gather + merge path (lag 1, one evaluation stream). */
int koordhip_comm_init(koordhip_ctx *ctx, const uint8_t *id, int32_t world, int32_t rank);
/* The same sharding for `world` contexts driven by ONE process (one host
 * thread per context, e.g. one scheduler process owning several GPUs, or
 * several contexts on one GPU): ctxs[r] becomes rank r and the per-round
 * exchange is a device-to-device copy instead of RCCL.  The contexts'
 * place_staged / place_stream calls must then run concurrently with the same
 * pod stream, as collective calls. */
int koordhip_comm_init_local(koordhip_ctx **ctxs, int32_t world);

#ifdef __cplusplus
}
#endif

#endif /* KOORDHIP_H */
