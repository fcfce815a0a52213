"""Headline benchmark: greedy placement of the BASELINE config-4 stream
(50k nodes x 100k pods, 70% LS / 30% BE, Fit + LoadAware with the shipped
scheduler profile) through libkoordhip.so, on N GPUs of one node.

  python bench.py --gpus N --steps K --warmup W
  (N > 1: torch.distributed.run, one rank per GPU, RCCL over xGMI)

A step = one full greedy pass of the pod stream over the node table, starting
from the same snapshot (device-side restore of the mutable columns, ~5 MB of
D2D copies, inside the timed region).  Inputs are HBM-resident before timing.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "pods placed/sec + (pod,node) Filter+Score evals/sec at 50k nodes, 1-8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def bytes_per_eval(pods: np.ndarray, cfg) -> np.ndarray:
    """Algorithmic node-column bytes one (pod, node) evaluation reads under the
    koordhip_node_soa schema, per pod (SURVEY.md §8(d) accounting, exact per pod
    class: the kernel reads only what that pod's Filter/Score consult)."""
    from koordinator_amd import abi
    req = pods["req"]
    flags = pods["flags"]
    b = np.full(len(pods), 1, np.int64)              # flags byte
    b += 8                                           # alloc_pods + npods (i32 x2)
    hr = (flags & abi.POD_HAS_REQ) != 0
    rcpu = hr & (req[:, 0] != 0)
    rmem = hr & (req[:, 1] != 0)
    b += 8 * rcpu + 8 * rmem                         # requested cpu/mem
    b += 16                                          # alloc cpu/mem (Fit score + LoadAware, aliased)
    b += 16                                          # nz cpu/mem
    b += 16                                          # la_used cpu/mem
    bc = (flags & abi.POD_REQ_BCPU) != 0
    bm = (flags & abi.POD_REQ_BMEM) != 0
    b += 16 * bc + 16 * bm                           # batch alloc + requested
    if cfg.score_plugins & abi.PLUGIN_NUMA or cfg.filter_plugins & abi.PLUGIN_NUMA:
        cs = (flags & abi.POD_CPUSET) != 0
        b += 4                                       # NUMA topology class (i32)
        b += (8 * ~rcpu) * ((flags & abi.POD_NUMA_SKIP) == 0)   # Score reads Requested cpu (non-cpuset pods)
        b += cs * (3 * abi.NUMA_WORDS * 8 + 4 + 1)   # cpuset pods: free / exclusive masks, allocated count, flags
    if (cfg.score_plugins | cfg.filter_plugins) & abi.PLUGIN_RESERVATION:
        # reservation flags (u32) on every node; on a reservation node (10%) the
        # restore reads Allocatable / Allocated / NonZero / assigned (6 f64 + i32 + rank)
        b += 4 + (6 * 8 + 8) // 10
        b += 8 * ~rcpu + 8 * ~rmem                   # the restore rewrites Requested: always read
    return b


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """CPUs this process may use: the cgroup CPU quota when there is one (the
    GPU box shows every host CPU but grants a share), else the affinity mask."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), open(
                            "/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()])):
        try:
            quota, period = parse(open(path).read())[:2]
            if quota not in ("max", "-1"):
                n = min(n, max(1, int(int(quota) // int(period))))
            break
        except (OSError, ValueError, IndexError):
            continue
    return n


def cpu_baseline(table, pods, cfg, budget_s=12.0, ext=None):
    """The oracle (C port of the reference loop: parallelize.Until over nodes,
    sqrt-n chunks, serial selectHost + Reserve) on this host, on a bounded
    prefix of the same stream, at the reference's parallelism (16 workers,
    pkg/util/parallelize/parallelism.go:28), at every CPU this process may use,
    and on one thread (the three legs).  `value` is the
    16-worker leg, the reference's own configuration (its per-node atomic
    append of feasible nodes, findNodesThatPassFilters, is kept: that
    contention is why the one-worker leg can be faster)."""
    import oracle
    ncpu = cpu_share()
    legs = {}
    for name, threads in (("ref16", min(16, ncpu)), ("nproc", ncpu), ("single", 1)):
        per = budget_s / 3
        probe = 32
        run = ((lambda o, m: o.place_stream(pods[:m], threads=threads)) if ext is None else
               (lambda o, m: o.place_stream_ext(pods[:m], ext[:m], threads=threads)))
        t = time.perf_counter()
        run(oracle.Oracle(cfg, table), probe)
        dt = time.perf_counter() - t
        n = int(min(len(pods), max(probe, per / max(dt / probe, 1e-9))))
        o = oracle.Oracle(cfg, table)
        t = time.perf_counter()
        run(o, n)
        dt = time.perf_counter() - t
        legs[name] = {"threads": threads, "pods": n, "pods_per_s": round(n / dt, 2),
                      "evals_per_s": round(n * table.n / dt, 1)}
    ref = legs["ref16"]
    best = max(legs, key=lambda k: legs[k]["pods_per_s"])
    return {"value": ref["pods_per_s"], "unit": "pods/s", "cores": ref["threads"], "kind": "port",
            "evals_per_s": ref["evals_per_s"], "legs": legs,
            "best_leg": {"name": best, **legs[best]}, "cpu_model": _cpu_model(), "nproc": ncpu,
            "sample": f"first {ref['pods']} pods of the same stream on the same {table.n}-node snapshot, "
                      f"oracle/koord_oracle.c {'orc_place_stream' if ext is None else 'orc_place_stream_ext'} "
                      f"with {ref['threads']} workers "
                      f"(legs: {ncpu} workers, 1 worker); the Go reference itself cannot run here (no Go toolchain)"}


def pmc_traffic(workload="config4"):
    """HBM bytes per eval launch from the committed rocprofv3 PMC summary of
    this workload (profiles/pmc_summary_<workload>.json; config 4's is also
    profiles/pmc_summary.json), if any."""
    p = os.path.join(ROOT, "profiles", f"pmc_summary_{workload}.json")
    if not os.path.exists(p) and workload == "config4":
        p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None, None, None, {}
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch"), d.get("source"), d.get("kernel"), d.get("kernels", {})
    except (OSError, ValueError):
        return None, None, None, {}


def latency_leg(eng, pods, ext=None, reps=200):
    """The per-cycle drop-in path (the shim's
    PreFilter calls koordhip_eval for the one pod of a scheduling cycle and
    reads the per-node status / per-plugin score arrays; batch admission calls
    koordhip_place_stream): host-to-host wall time per call on the loaded
    snapshot, median and p99 of `reps` calls after 10 warm-up calls -- the
    pod upload, the launches, the synchronisation and the result copies
    included.  place_stream commits its pods (the state is restored after)."""
    import numpy as _np

    def timed(fn):
        for _ in range(10):
            fn()
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t) * 1e6)
        ts = _np.sort(_np.array(ts))
        return {"median_us": round(float(_np.median(ts)), 1), "p99_us": round(float(ts[int(len(ts) * 0.99) - 1]), 1),
                "calls": reps}

    one, many = pods[:1], pods[:64]
    out = {"nodes": int(eng.n), "method": "time.perf_counter around each C-ABI call (host to host), after 10 warm-up calls",
           "eval_1pod_status_scores": timed(lambda: eng.eval(one, status=True, scores=True)),
           "eval_1pod_status_only": timed(lambda: eng.eval(one, status=True, scores=False))}
    if ext is None:
        out["place_stream_1pod"] = timed(lambda: eng.place_stream(one))
        out["place_stream_64pods"] = timed(lambda: eng.place_stream(many))
    else:
        out["place_stream_1pod"] = timed(lambda: eng.place_stream_ext(one, ext[:1]))
        out["place_stream_64pods"] = timed(lambda: eng.place_stream_ext(many, ext[:64]))
    eng.restore()
    return out


def launch_ranks(n: int) -> int:
    """`--gpus N > 1` without a torch.distributed launcher: start one as a CHILD
    process (nothing here has touched the GPU yet) with this command line, and
    return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["config4", "config3", "config5", "deviceshare", "spread", "affinity",
                                                   "resvpolicy", "config4ds", "config4dsmix"], default="config4",
                    help="config4: the headline (50k x 100k, Fit + LoadAware); config3: NodeNUMAResource "
                         "cpuset/NUMA-fit scoring (5k 2-socket nodes x 10k pods, 50%% LSR/LSE cpuset pods); "
                         "config5: 200k nodes, 10%% holding a Reservation matched by 20%% of the pods, "
                         "+ LoadAware + NodeNUMAResource; deviceshare: config 4's cluster with GPU / RDMA "
                         "devices and 20%% device pods, + DeviceShare (weight 1): the exact sequential cycle, "
                         "one GPU; spread: config 4's cluster with zone / rack / hostname topology and 60%% of "
                         "the pods in five PodTopologySpread classes, + PodTopologySpread (filter, weight 2): "
                         "the exact sequential cycle, one GPU; affinity: config 4's cluster with zone / hostname "
                         "topology, four apps' running pods and 60%% of the pods carrying pod affinity / "
                         "anti-affinity terms, + InterPodAffinity (filter, weight 1): the exact sequential cycle; "
                         "resvpolicy: config 5's profile and cluster with 30%% NUMA topology-policy nodes, up to 4 "
                         "reservations per node (70%% holding cpusets, on policy nodes too) and 30%% cpuset pods: "
                         "the exact sequential cycle; config4ds: config 4 under the shipped profile with DeviceShare "
                         "(weight 1) on a cluster with devices, no pod requesting one: the pipelined greedy")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--be-frac", type=float, default=None)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--dev-frac", type=float, default=None,
                    help="deviceshare / config4dsmix workloads: share of pods requesting GPUs (default 0.2 / 0.02)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--check", action="store_true", help="verify placements vs the oracle (slow)")
    ap.add_argument("--one-rank-comm", action="store_true",
                    help="N=1 only: attach a one-rank RCCL communicator, so every round takes the multi-GPU "
                         "exchange path (all-gather + merge) -- measures that pipeline on one GPU")
    ap.add_argument("--mode", choices=["replicas", "shard"], default="shard",
                    help="N > 1: 'shard' (default, north_star's partition: ONE cluster's schedule) -- the node "
                         "table sharded across the ranks with the per-round top-k all-gathered over RCCL, or, "
                         "where the class-incremental lists cover the batch, every rank on the full replica "
                         "without an exchange (the library's fallback: never slower than one GPU; DESIGN.md "
                         "section 6); 'replicas' (opt-in) -- independent replicas, not one cluster: every rank "
                         "places its own copy of the stream on its own copy of the cluster")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the per-cycle latency leg (koordhip_eval of 1 pod, koordhip_place_stream of 1 / "
                         "64 pods on the loaded snapshot)")
    ap.add_argument("--probe-ranks", action="store_true",
                    help="print this rank's RANK / WORLD_SIZE and exit before any GPU work (launcher test)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.probe_ranks:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank}), flush=True)
        return

    import torch
    from koordinator_amd import synth
    from koordinator_amd.config import (shipped_profile, to_c_config, with_deviceshare, with_interpod_affinity,
                                        with_topology_spread)
    from koordinator_amd.engine import PlacementEngine

    if args.workload in ("deviceshare", "spread", "affinity", "resvpolicy"):
        if world > 1:
            raise SystemExit(f"--workload {args.workload} runs on one GPU (the sequential cycle is not node-sharded)")
        prof = {"deviceshare": lambda: with_deviceshare(shipped_profile()),
                "spread": lambda: with_topology_spread(shipped_profile()),
                "affinity": lambda: with_interpod_affinity(shipped_profile()),
                "resvpolicy": lambda: shipped_profile(numa=True, reservation=True)}[args.workload]()
        return run_sequential(args, torch, synth, prof, PlacementEngine)

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    resv = args.workload == "config5"
    numa = args.workload == "config3" or resv
    c = synth.CONFIGS[{"config3": 3, "config4": 4, "config5": 5, "config4ds": 4, "config4dsmix": 4}[args.workload]]
    dsmix = args.workload == "config4dsmix"
    args.nodes = args.nodes or c["nodes"]
    args.pods = args.pods or c["pods"]
    args.be_frac = c["be_frac"] if args.be_frac is None else args.be_frac
    prof = shipped_profile(numa=numa, reservation=resv)
    if args.workload in ("config4ds", "config4dsmix"):
        prof = with_deviceshare(prof)
    prof.batch_pods = args.batch
    table = synth.make_cluster(synth.ClusterSpec(args.nodes), prof)
    if args.workload in ("config4ds", "config4dsmix"):
        synth.add_devices(table, synth.DevSpec())
    if numa:
        synth.add_numa(table, synth.NumaSpec(), prof)
    if resv:
        synth.add_reservations(table, synth.ResvSpec())
    pods = synth.make_pods(synth.StreamSpec(args.pods, be_frac=args.be_frac, cpuset_frac=c.get("cpuset_frac", 0.0),
                                            resv_match_frac=c.get("resv_match_frac", 0.0)), prof)
    # config4dsmix: a few pods request GPUs (the reference's request forms,
    # synth.make_device_ext); the rest carry empty records
    ext = synth.make_device_ext(args.pods, synth.DevStreamSpec(frac=0.02 if args.dev_frac is None else args.dev_frac)) \
        if dsmix else None
    cfg = to_c_config(prof)

    eng = PlacementEngine(prof, device=local_rank, profile_kernels=False)
    shard = world > 1 and args.mode == "shard"
    if shard:
        uid = PlacementEngine.comm_unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device="cuda")
        dist.broadcast(t, 0)
        eng.comm_init(bytes(t.cpu().tolist()), world, rank)
    elif args.one_rank_comm:
        eng.comm_init(PlacementEngine.comm_unique_id(), 1, 0)
    eng.load_snapshot(table)
    eng.checkpoint()
    t_st = time.perf_counter()
    if ext is None:
        eng.stage_pods(pods)
    else:
        eng.stage_pods_ext(pods, ext)
    stage_pods_ms = (time.perf_counter() - t_st) * 1e3

    def step():
        eng.restore()
        eng.place_staged()

    for _ in range(args.warmup):
        step()
    eng.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        eng.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    # per-kernel split for the roofline: one more (untimed) step with HIP
    # events around every launch (they cost a few us per round, so the timed
    # steps run without them)
    eng.set_profile_kernels(True)
    step()
    ks = eng.kernel_stats()
    kn = eng.kernel_names()
    eng.set_profile_kernels(False)
    executed = float(ks["executed_evals"])   # this rank's, per step
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        te = torch.tensor([executed], dtype=torch.float64, device="cuda")
        dist.all_reduce(te, op=dist.ReduceOp.SUM)   # every rank's evaluations (a local rank runs the full table)
        executed = float(te.item())
    placements = eng.fetch_placements(len(pods))
    lat = latency_leg(eng, pods, ext) if (world == 1 and not args.no_latency) else None

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    pods_total = args.pods * args.steps * (world if world > 1 and not shard else 1)  # replicas: every rank's stream
    pods_profiled = args.pods
    # equivalent evaluations: every (pod, node) pair of the schedule decided
    # exactly (what a full Filter + Score pass per pod computes); executed: the
    # (pod, node) evaluations the kernels actually ran (class-list builds +
    # commit-log re-evaluations + the device pods' evaluations), all ranks
    evals_total = pods_total * args.nodes
    executed_total = executed * args.steps * (world if world > 1 and not shard else 1)
    local = shard and world > 1 and (int(ks["flags"]) & 1) != 0
    value = pods_total / elapsed
    batch = int(ks["round_pods"]) or eng.cfg.batch_pods or (16 if numa else 32)
    lag = int(ks["lag"]) or 1
    k = (lag + 1) * batch   # list length: the resolve re-checks the nodes of the last `lag` rounds
    # ---- the dominant kernel: k_resolve, the sequential greedy (one persistent
    #      launch per step spanning the round pipeline).  Algorithmic bytes per
    #      pod: its list (k x 8 B) + pod record (96 B) + the
    #      prefetched list-head rows (128 / batch rows x 160 B) + one row
    #      write-back (13 mutable columns, 100 B).
    heads = max(1, 128 // batch)
    b_pod = k * 8 + 96 + heads * 160 + 100
    persistent = ks["resolve_launches"] <= 1
    # a persistent resolve spans the whole step: its launch time is the timed
    # step itself (an upper bound), never the separately instrumented step
    res_s = (elapsed / args.steps) if persistent else ks["resolve_ms"] * 1e-3 / max(ks["resolve_launches"], 1)
    pods_per_launch = pods_profiled / max(ks["resolve_launches"], 1)
    res_gbs = pods_per_launch * b_pod / res_s / 1e9 if res_s > 0 else None
    # ---- the evaluation kernel k_scan: physical bytes per launch = the node
    #      columns the round's pods consult, read once (VGPR-resident across the
    #      pod loop), + the u16 score-matrix row per (pod, node) + chunk maxima
    b_eval = bytes_per_eval(pods, cfg)
    scan_us = ks["scan_ms"] * 1e3 / max(ks["scan_launches"], 1)
    evals_per_launch = ks["evals"] / max(ks["rounds"], 1)   # one scan launch per round (the timed ones are a sample)
    pods_per_round = evals_per_launch / max(args.nodes, 1)
    col_bytes = float(b_eval.max()) * args.nodes
    # the fused k_eval_topk (no select launches) keeps the scores in LDS: its
    # physical bytes are the node columns once (+ the small slice lists); the
    # split k_scan also writes the u16 score matrix and the chunk maxima
    fused = ks["select_launches"] == 0
    phys = col_bytes if fused else col_bytes + pods_per_round * args.nodes * 2 + pods_per_round * args.nodes / 64 * 2
    scan_gbs = phys / (scan_us * 1e-6) / 1e9 if scan_us > 0 else None
    traffic, traffic_src, traffic_kernel, pmc_kernels = pmc_traffic(args.workload)
    if traffic_src is not None and traffic_kernel != kn["eval"]:
        traffic, traffic_src = None, (f"none for {kn['eval']} (the committed PMC summary is of "
                                      f"{traffic_kernel or 'an unnamed kernel'})")
    cls = kn["eval"].startswith("kh::k_cls_run")
    if cls:
        # class-incremental lists (cls.hip): one persistent workgroup per pod
        # class for the whole step, builds (k_scan over the class records +
        # k_cls_collect) in batches on the second stream
        raw = np.ascontiguousarray(pods).view(np.uint8).reshape(len(pods), -1)
        ncls = int(len(np.unique(raw, axis=0)))
        bld_us = ks["select_ms"] * 1e3 / max(ks["select_launches"], 1)
        eval_obj = {"bound": "latency", "kernel": kn["eval"],
                    "mode": "class-incremental lists: one persistent workgroup per pod class keeps its best "
                            f"{2048} keys in LDS and re-evaluates only the nodes the resolve committed since its "
                            "last round (the commit log); the lists are exact top-k keys like k_scan + select's",
                    "classes": ncls, "avg_launch_ms": round(ks["scan_ms"] / max(ks["scan_launches"], 1), 3),
                    "timing": "HIP events around the persistent launch (the whole step)",
                    "builds": {"kernels": "k_scan over the class records + k_cls_collect",
                               "timed_batches": int(ks["select_launches"]), "avg_batch_us": round(bld_us, 3),
                               "traffic": {k: v["hbm_bytes_per_launch"] for k, v in pmc_kernels.items()
                                           if "class build" in k or "k_cls_collect" in k} or None},
                    "executed_evals_per_step": int(ks["executed_evals"]),
                    "traffic": traffic, "traffic_source": traffic_src,
                    "traffic_note": "HBM bytes of one k_cls_run launch (the whole stream's class workgroups) "
                                    "from the PMC replay (scripts/pmc_summary.py), of the stream size it was "
                                    "collected on"}
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "pods/s",
        "equivalent_evals_per_s": round(evals_total / elapsed, 1),
        "executed_evals_per_s": round(executed_total / elapsed, 1),
        "evals_note": "equivalent: every (pod, node) pair decided exactly; executed: the evaluations the kernels ran",
        "stage_ms": round(stage_pods_ms + ks["plan_us"] / 1e3, 3),
        "stage_split_ms": {"stage_pods": round(stage_pods_ms, 3), "cls_plan": round(ks["plan_us"] / 1e3, 3)},
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if world == 1 or shard else "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded splitmix64 cluster + pod stream, SURVEY.md §8(d))",
        "config": {"workload": (f"config5: {args.nodes} nodes (10% holding an Available Reservation) x "
                                f"{args.pods} pods, {int(args.be_frac * 100)}% BE, "
                                f"{int(c.get('resv_match_frac', 0) * 100)}% matching a reservation owner, "
                                "NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource + Reservation (weight 5000)"
                                if resv else
                                f"config3: {args.nodes} 2-socket nodes x {args.pods} pods, "
                                f"{int(args.be_frac * 100)}% BE, {int(c.get('cpuset_frac', 0) * 100)}% of LS pods "
                                "LSR/LSE cpuset, NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource"
                                if numa else
                                f"config4: {args.nodes} nodes x {args.pods} pods, {int(args.be_frac * 100)}% BE, "
                                "NodeResourcesFit + LoadAwareScheduling, shipped scheduler-config.yaml profile"
                                + (" + DeviceShare (weight 1; 30% of the nodes with GPUs, no pod requesting one: "
                                   "the pipelined greedy)" if args.workload == "config4ds" else "")
                                + (f" + DeviceShare (weight 1; 30% of the nodes with GPUs; "
                                   f"{int((ext['flags'] != 0).sum())} pods ({(ext['flags'] != 0).mean() * 100:.1f}%) "
                                   "requesting GPUs in the reference's four request forms, placed inside the pipelined "
                                   "greedy by k_ext_pre / k_ext_final)" if dsmix else "")),
                   "nodes": args.nodes, "pods": args.pods, "batch_pods": batch, "pipeline_lag": lag,
                   "parallelism": (f"independent replicas x{world}, not one cluster (every rank: its own cluster "
                                   "copy and stream)" if world > 1 and not shard
                                   else f"node-shard x{world}: every rank on the full replica, no exchange (class "
                                   "lists; the library's fallback, one cluster's schedule)" if local
                                   else f"node-shard x{world}" + (" (one-rank RCCL exchange path)" if args.one_rank_comm and world == 1 else ""))},
        "unschedulable": int((placements < 0).sum()),
        "latency": lat,
        "roofline": {"bound": "latency", "kernel": kn["resolve"],
                     "limiter": "latency: one workgroup's sequential greedy (not bandwidth); priced against HBM peak",
                     "timing": "the timed step (persistent launch)" if persistent else "HIP events per launch",
                     "achieved": round(res_gbs, 3) if res_gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(res_gbs / HBM_PEAK_GBS, 6) if res_gbs else None, "traffic": None,
                     "bytes_per_pod": b_pod, "avg_launch_ms": round(res_s * 1e3, 3),
                     "pods_per_launch": pods_per_launch,
                     "us_per_pod": round(res_s * 1e6 / max(pods_per_launch, 1), 4)},
        "eval_roofline": eval_obj if cls else {"bound": "hbm", "kernel": kn["eval"],
                          "achieved": round(scan_gbs, 1) if scan_gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(scan_gbs / HBM_PEAK_GBS, 4) if scan_gbs else None,
                          "traffic": traffic, "traffic_source": traffic_src,
                          "bytes_per_launch": round(phys), "avg_launch_us": round(scan_us, 3),
                          "evals_per_launch": evals_per_launch,
                          "algorithmic_bytes_per_eval": round(float(b_eval.mean()), 2),
                          "algorithmic_GBps": round(evals_per_launch * float(b_eval.mean()) / (scan_us * 1e-6) / 1e9, 1)
                          if scan_us > 0 else None},
    }
    if not cls:
        out["select"] = {"kernel": "(in k_eval_topk)" if fused else "k_select_split",
                         "avg_launch_us": round(ks["select_ms"] * 1e3 / max(ks["select_launches"], 1), 3)}
    if dsmix:
        out["device_pods_traffic"] = {k: v["hbm_bytes_per_launch"] for k, v in pmc_kernels.items() if "k_ext_" in k} or None
        out["device_pods"] = {"pods": int((ext["flags"] != 0).sum()), "kernels": "k_ext_pre<0> + k_ext_final<0>",
                              "route": "pipelined (resolve hand-off)" if kn["resolve"].startswith("kh::k_resolve")
                              else "sequential cycle"}
    if args.check:
        import oracle
        orc = oracle.Oracle(cfg, table)
        ref = orc.place_stream(pods, threads=min(16, os.cpu_count() or 1)) if ext is None else \
            orc.place_stream_ext(pods, ext, threads=min(16, os.cpu_count() or 1))
        out["check"] = bool(np.array_equal(ref, placements))
    if world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(table, pods, cfg, args.cpu_budget, ext=ext)
        out["cpu_baseline"] = cb
        out["speedup_vs_best_cpu_leg"] = round(value / cb["best_leg"]["pods_per_s"], 1)
    print(json.dumps(out), flush=True)
    eng.close()                      # before interpreter teardown (the HIP runtime's own exit handlers)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def seq_bytes_per_eval(pods: np.ndarray, ext: np.ndarray, cfg, dev_slots: int) -> np.ndarray:
    """Algorithmic node-column bytes per (pod, node) of the sequential cycle's
    evaluation: the Fit / LoadAware columns (bytes_per_eval), the extended
    scalars a pod requests (xalloc + xrequested, 16 B per requested name), and
    for a device pod the node's nodeDevice entry (dev_present 1 B) and its GPU
    and RDMA slots (minor i32, total + used of the requested resources i64)."""
    from koordinator_amd import abi
    b = bytes_per_eval(pods, cfg).copy()
    if ext is None:
        return b
    xm = ext["xmask"].astype(np.int64)
    b += 16 * np.array([bin(int(x)).count("1") for x in xm], np.int64)
    dev = (ext["flags"] & abi.PODX_DEVICE) != 0
    g = ext["dev_req"][:, abi.DEV_GPU]
    gres = (g > 0).sum(axis=1)
    rd = ext["dev_req"][:, abi.DEV_RDMA, 0] > 0
    per = 1 + dev_slots * (4 + 16 * gres) + rd * dev_slots * (4 + 16)
    b = b + np.where(dev, per, 0)
    # PodTopologySpread: pts_elig (2 B), the domain of each key the pod's
    # constraints name and the node's count of each of its constraints (4 B each)
    pn = ext["pts_n"].astype(np.int64)
    nkeys = np.array([len(set(int(c) for c in x["pts_c"][:int(x["pts_n"])])) for x in ext], np.int64)
    b = b + np.where(pn > 0, 2 + 4 * nkeys + 4 * pn, 0)
    # InterPodAffinity: per entry the pod's Filter / Score reads, the node's
    # domain for the entry's key and (hostname entries) its own count: 8 B
    m = (ext["ipa_aff"] | ext["ipa_anti"] | ext["ipa_score"]).astype(np.uint64)
    ne = np.array([bin(int(v)).count("1") for v in m], np.int64)
    return b + 8 * ne


def run_sequential(args, torch, synth, prof, PlacementEngine):
    """The DeviceShare / spread workloads: one persistent cooperative k_seq
    launch per step (every node filtered and scored per pod, normalized over
    the feasible nodes, the argmax committed before the next pod)."""
    resvpol = args.workload == "resvpolicy"
    c = synth.CONFIGS[5 if resvpol else 4]
    args.nodes = args.nodes or c["nodes"]
    args.pods = args.pods or 20000
    args.be_frac = c["be_frac"] if args.be_frac is None else args.be_frac
    spread = args.workload == "spread"
    affinity = args.workload == "affinity"
    table = synth.make_cluster(synth.ClusterSpec(args.nodes), prof)
    pods = synth.make_pods(synth.StreamSpec(args.pods, be_frac=args.be_frac, cpuset_frac=0.3 if resvpol else 0.0,
                                            resv_match_frac=c.get("resv_match_frac", 0.0)), prof)
    if resvpol:
        # the Reservation plugin on NUMA topology-policy nodes: such snapshots run in the sequential cycle
        synth.add_numa(table, synth.NumaSpec(policy_frac=0.3), prof)
        synth.add_reservations(table, synth.ResvSpec(slots=4, multi_frac=0.3))
        synth.add_reserved_cpus(table, frac=0.7, policy_nodes=True)
        ext = None
    elif spread or affinity:
        from koordinator_amd import abi
        table.enable_ext(0)
        ext = abi.pod_ext_array(args.pods)
        if spread:
            synth.add_spread(table, ext, synth.SpreadSpec())
        else:
            synth.add_ipa(table, ext, synth.IpaSpec())
    else:
        synth.add_devices(table, synth.DevSpec())
        ext = synth.make_device_ext(args.pods, synth.DevStreamSpec(frac=0.2 if args.dev_frac is None else args.dev_frac))
    from koordinator_amd.config import to_c_config
    cfg = to_c_config(prof)
    eng = PlacementEngine(prof, device=0, profile_kernels=False)
    eng.load_snapshot(table)
    eng.checkpoint()
    t_st = time.perf_counter()
    if ext is None:
        eng.stage_pods(pods)
    else:
        eng.stage_pods_ext(pods, ext)
    stage_pods_ms = (time.perf_counter() - t_st) * 1e3

    def step():
        eng.restore()
        eng.place_staged()

    for _ in range(args.warmup):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ks = eng.kernel_stats()          # the last step's k_seq launch, HIP events on the engine's stream
    kn = eng.kernel_names()
    placements = eng.fetch_placements(len(pods))
    seq_s = ks["total_ms"] * 1e-3
    # a DeviceShare batch of device pods among plain ones runs on the pipelined
    # greedy (k_resolve + k_ext_pre / k_ext_final); everything else here in k_seq
    pipelined = kn["resolve"].startswith("kh::k_resolve")
    b = seq_bytes_per_eval(pods, ext, cfg, table.dev_slots)
    alg = float(b.sum()) * args.nodes
    gbs = alg / seq_s / 1e9 if seq_s > 0 else None
    value = args.pods * args.steps / elapsed
    if ext is None:
        from koordinator_amd import abi
        ext = abi.pod_ext_array(args.pods)   # (the counters below: no device / spread / affinity pods)
    dev = (ext["flags"] & 1) != 0
    if resvpol:
        pol = ((table["numa_flags"].astype(np.int64) >> 3) & 3) != 0
        wl = (f"resvpolicy: {args.nodes} nodes ({int(pol.mean() * 100)}% with a NUMA topology policy; "
              f"reservations on {int((table['resv_flags'] != 0).mean() * 100)}% of the nodes, up to 4 per node, "
              f"70% holding cpusets) x {args.pods} pods (30% cpuset, {int(c['resv_match_frac'] * 100)}% matching "
              "a reservation), NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource + Reservation, "
              "the exact sequential cycle")
    elif affinity:
        wl = (f"affinity: {args.nodes} nodes (6 zones, hostname; 4 apps' running pods) x {args.pods} pods "
              f"({int(((ext['ipa_inc'] | ext['ipa_aff'] | ext['ipa_anti'] | ext['ipa_score']) != 0).mean() * 100)}% "
              "carrying pod affinity / anti-affinity terms), NodeResourcesFit + LoadAwareScheduling + "
              "InterPodAffinity (filter, weight 1), the exact sequential cycle")
    elif spread:
        wl = (f"spread: {args.nodes} nodes (6 zones, 24 racks, hostname; 3 apps' running pods) x {args.pods} pods "
              f"({int((ext['pts_n'] > 0).mean() * 100)}% in five PodTopologySpread classes), NodeResourcesFit + "
              "LoadAwareScheduling + PodTopologySpread (filter, weight 2), the exact sequential cycle")
    else:
        wl = (f"deviceshare: {args.nodes} nodes (30% with 4/8 GPUs, half of those 2 RDMA NICs) x "
              f"{args.pods} pods ({int(dev.mean() * 100)}% requesting GPUs), "
              "NodeResourcesFit + LoadAwareScheduling + DeviceShare (weight 1, LeastAllocated), "
              + ("the pipelined greedy with the device pods placed exactly by k_ext_pre / k_ext_final"
                 if pipelined else "the exact sequential cycle"))
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "pods/s",
        "equivalent_evals_per_s": round(args.pods * args.nodes * args.steps / elapsed, 1),
        "executed_evals_per_s": round(float(ks["executed_evals"]) * args.steps / elapsed, 1),
        "evals_note": "equivalent: every (pod, node) pair decided exactly; executed: the evaluations the kernels ran",
        "stage_ms": round(stage_pods_ms, 3),
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic (seeded splitmix64 cluster + pod stream)",
        "config": {"workload": wl, "nodes": args.nodes, "pods": args.pods,
                   "parallelism": "single GPU" + (" (pipelined greedy + device-pod kernels)" if pipelined
                                                  else " (cooperative grid)")},
        "unschedulable": int((placements < 0).sum()),
        "device_pods_placed": int(((placements >= 0) & dev).sum()),
        "spread_pods_placed": int(((placements >= 0) & (ext["pts_n"] > 0)).sum()),
        "affinity_pods_placed": int(((placements >= 0) & ((ext["ipa_aff"] | ext["ipa_anti"] | ext["ipa_score"]) != 0)).sum()),
        "roofline": {"bound": "latency", "kernel": kn["resolve"],
                     "limiter": ("latency: the persistent resolve's sequential greedy, and per device pod one hand-off to k_ext_final (write-back, re-evaluation of the nodes changed since the pre-evaluation, last-arriver winner + device Reserve) and back (not bandwidth); priced against HBM peak" if pipelined else "latency: per pod one grid-wide hand-off (two for device pods) after the owner's commit and one evaluation chain (not bandwidth); priced against HBM peak" if not (spread or affinity) else "latency: per pod the spread pre-pass (hostname minimum), one or two grid-wide hand-offs (soft scoring adds the raw min / max) and one evaluation chain (not bandwidth); priced against HBM peak"),
                     "timing": "HIP events around the place call of the last timed step",
                     "achieved": round(gbs, 2) if gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs / HBM_PEAK_GBS, 5) if gbs else None, "traffic": None,
                     "algorithmic_bytes_per_eval": round(float(b.mean()), 2),
                     "avg_launch_ms": round(seq_s * 1e3, 3),
                     "us_per_pod": round(seq_s * 1e6 / args.pods, 3)},
    }
    if not args.no_cpu_baseline:
        cb = cpu_baseline(table, pods, cfg, args.cpu_budget, ext=None if resvpol else ext)
        out["cpu_baseline"] = cb
        out["speedup_vs_best_cpu_leg"] = round(value / cb["best_leg"]["pods_per_s"], 1)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
