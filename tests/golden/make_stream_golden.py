"""TEST INFRASTRUCTURE: golden placements for the headline stream.

Runs the CPU oracle (oracle/koord_oracle.c orc_place_stream: the reference
loop -- load_aware.go:123-335, upstream fitsRequest / LeastAllocated, the
lowest-index selectHost, Reserve after every pod) over the exact BASELINE
config-4 workload bench.py times (synth.config_workload(4): 50k nodes x 100k
pods, 30% BE, shipped profile) and writes

  tests/golden/stream_config4.npz   placements (int32 [100000]), and sha256
                                     digests of the generated inputs and of
                                     every final mutable node column
  tests/golden/stream_config5.npz   the same for config 5 (200k nodes with
                                     reservations + NUMA): also the digests of
                                     the final NUMA / reservation columns and
                                     of the pods' cpusets

so the GPU tests (tests/test_gpu_fullsize.py) can compare libkoordhip.so's
full-size stream bit for bit without re-running a ~6-minute oracle on the box.

  python tests/golden/make_stream_golden.py [--config 4] [--threads 1]

Single-threaded by default: on this 8-CPU container the oracle's per-pod
parallelize.Until fan-out costs more than it saves at 50k nodes.
"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def input_digests(table, pods) -> dict:
    d = {c: digest(table[c]) for c in sorted(table.cols)}
    d["__pods__"] = digest(pods)
    return d


def state_digests(state: dict) -> dict:
    return {k: digest(v) for k, v in sorted(state.items())}


def main():
    import oracle
    from koordinator_amd import synth
    from koordinator_amd.config import shipped_profile, to_c_config

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--threads", type=int, default=1)
    args = ap.parse_args()
    cc = synth.CONFIGS[args.config]
    prof = shipped_profile(numa=bool(cc.get("numa")), reservation=bool(cc.get("reservation")))
    table, pods = synth.config_workload(args.config, prof)
    cfg = to_c_config(prof)
    o = oracle.Oracle(cfg, table)
    t = time.time()
    numa = bool(cc.get("numa"))
    cpus = None
    if numa:
        out, cpus = o.place_stream(pods, threads=args.threads, cpusets=True)
    else:
        out = o.place_stream(pods, threads=args.threads)
    dt = time.time() - t
    st = o.state()
    if numa:
        st.update({"numa." + k: v for k, v in o.numa_state().items()})
        st["__cpusets__"] = cpus
    if cc.get("reservation"):
        st.update({"resv." + k: v for k, v in o.resv_state().items()})
    ind = input_digests(table, pods)
    sd = state_digests(st)
    path = os.path.join(HERE, f"stream_config{args.config}.npz")
    np.savez_compressed(
        path, placements=out,
        input_keys=np.array(list(ind.keys())), input_sha=np.array(list(ind.values())),
        state_keys=np.array(list(sd.keys())), state_sha=np.array(list(sd.values())),
        meta=np.array([f"config{args.config}: {table.n} nodes x {len(pods)} pods, oracle orc_place_stream "
                       f"threads={args.threads}, {dt:.1f} s"]))
    print(f"wrote {path}: {len(out)} placements, {int((out < 0).sum())} unschedulable, {dt:.1f} s")


if __name__ == "__main__":
    main()
