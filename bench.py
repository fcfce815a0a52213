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
    return b


def cpu_baseline(table, pods, cfg, budget_s=12.0):
    """The oracle (C port of the reference loop: parallelize.Until over nodes,
    16 workers, sqrt-n chunks) on this host, on a bounded prefix of the stream."""
    import oracle
    threads = min(16, os.cpu_count() or 1)
    probe = 64
    t = time.perf_counter()
    oracle.Oracle(cfg, table).place_stream(pods[:probe], threads=threads)
    dt = time.perf_counter() - t
    n = int(min(len(pods), max(probe, budget_s / max(dt / probe, 1e-9))))
    o = oracle.Oracle(cfg, table)
    t = time.perf_counter()
    o.place_stream(pods[:n], threads=threads)
    dt = time.perf_counter() - t
    return {"value": round(n / dt, 2), "unit": "pods/s", "cores": threads, "kind": "port",
            "evals_per_s": round(n * table.n / dt, 1),
            "sample": f"first {n} pods of the same stream on the same {table.n}-node snapshot, "
                      f"oracle/koord_oracle.c orc_place_stream, {threads} threads, host {os.cpu_count()} cpus"}


def pmc_traffic():
    """HBM bytes per eval launch from the committed rocprofv3 PMC summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch"), d.get("source")
    except Exception:
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["config4", "config3"], default="config4",
                    help="config4: the headline (50k x 100k, Fit + LoadAware); config3: NodeNUMAResource "
                         "cpuset/NUMA-fit scoring (5k 2-socket nodes x 10k pods, 50%% LSR/LSE cpuset pods)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--be-frac", type=float, default=None)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--check", action="store_true", help="verify placements vs the oracle (slow)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    from koordinator_amd import synth
    from koordinator_amd.config import shipped_profile, to_c_config
    from koordinator_amd.engine import PlacementEngine

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    numa = args.workload == "config3"
    c = synth.CONFIGS[3 if numa else 4]
    args.nodes = args.nodes or c["nodes"]
    args.pods = args.pods or c["pods"]
    args.be_frac = c["be_frac"] if args.be_frac is None else args.be_frac
    prof = shipped_profile(numa=numa)
    prof.batch_pods = args.batch
    table = synth.make_cluster(synth.ClusterSpec(args.nodes), prof)
    if numa:
        synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(args.pods, be_frac=args.be_frac,
                                            cpuset_frac=c.get("cpuset_frac", 0.0)), prof)
    cfg = to_c_config(prof)

    eng = PlacementEngine(prof, device=local_rank, profile_kernels=True)
    if world > 1:
        uid = PlacementEngine.comm_unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device="cuda")
        dist.broadcast(t, 0)
        eng.comm_init(bytes(t.cpu().tolist()), world, rank)
    eng.load_snapshot(table)
    eng.checkpoint()
    eng.stage_pods(pods)

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
    eval_ms = 0.0
    launches = 0
    evals = 0
    for _ in range(args.steps):
        step()
        st = eng.last_stats()   # synchronizes the engine stream after each step
        eval_ms += st["eval_ms"]
        launches += st["eval_launches"]
        evals += st["evals"]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    placements = eng.fetch_placements(len(pods))

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    pods_total = args.pods * args.steps
    evals_total = args.pods * args.nodes * args.steps   # every pod is evaluated against every node
    value = pods_total / elapsed
    # roofline of the evaluation kernel (k_scan), this rank's launches
    b_eval = bytes_per_eval(pods, cfg)
    b_per_pod = float(b_eval.mean())
    avg_launch_ms = eval_ms / max(launches, 1)
    evals_per_launch = evals / max(launches, 1)
    achieved = evals_per_launch * b_per_pod / (avg_launch_ms * 1e-3) / 1e9 if eval_ms > 0 else None
    traffic, traffic_src = pmc_traffic() if not numa else (None, None)   # the committed PMC pass is config 4's
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "pods/s",
        "evals_per_s": round(evals_total / elapsed, 1),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded splitmix64 cluster + pod stream, SURVEY.md §8(d))",
        "config": {"workload": (f"config3: {args.nodes} 2-socket nodes x {args.pods} pods, "
                                f"{int(args.be_frac * 100)}% BE, {int(c.get('cpuset_frac', 0) * 100)}% of LS pods "
                                "LSR/LSE cpuset, NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource"
                                if numa else
                                f"config4: {args.nodes} nodes x {args.pods} pods, {int(args.be_frac * 100)}% BE, "
                                "NodeResourcesFit + LoadAwareScheduling, shipped scheduler-config.yaml profile"),
                   "nodes": args.nodes, "pods": args.pods, "batch_pods": eng.cfg.batch_pods or (16 if args.workload == "config3" else 32),
                   "parallelism": f"node-shard x{world}"},
        "unschedulable": int((placements < 0).sum()),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 3) if achieved else None,
                     "traffic": traffic, "kernel": "k_scan",
                     "avg_launch_us": round(avg_launch_ms * 1e3, 3), "evals_per_launch": evals_per_launch,
                     "bytes_per_eval": round(b_per_pod, 2), "traffic_source": traffic_src},
    }
    if args.check:
        import oracle
        ref = oracle.Oracle(cfg, table).place_stream(pods, threads=min(16, os.cpu_count() or 1))
        out["check"] = bool(np.array_equal(ref, placements))
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(table, pods, cfg, args.cpu_budget)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
