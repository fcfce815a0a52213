import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import oracle
from koordinator_amd import synth, abi
from koordinator_amd.config import shipped_profile, to_c_config
from koordinator_amd.engine import PlacementEngine
prof = shipped_profile(numa=True)
table = synth.make_cluster(synth.ClusterSpec(600), prof)
synth.add_numa(table, synth.NumaSpec(), prof)
pods = synth.make_pods(synth.StreamSpec(1000, be_frac=0.2, cpuset_frac=0.5), prof)
cfg = to_c_config(prof)
o = oracle.Oracle(cfg, table)
ref = o.place_stream(pods)
o2 = oracle.Oracle(cfg, table)
with PlacementEngine(prof, device=0) as e:
    e.load_snapshot(table)
    for i in range(299):
        if ref[i] >= 0:
            o2.commit(pods[i], int(ref[i])); e.commit(pods[i], int(ref[i]))
    g = e.eval(pods[299:300], k=8)
    r = o2.eval(pods[299:300], k=8)
    ds = np.flatnonzero(g["status"][0] != r["status"][0])
    print("status diffs", len(ds), ds[:10], g["status"][0][ds[:10]], r["status"][0][ds[:10]])
    dsc = np.flatnonzero((g["scores"][0] != r["scores"][0]).any(0) & (r["status"][0] == 0))
    print("score diffs", len(dsc), dsc[:10])
    print("gpu topk", g["topk"][0], "\nref topk", r["topk"][0])
    # first-999: full stream via place_stream for reference on the fresh engine
    st = e.read_numa()
    ns = o2.numa_state()
    for kk in ("free", "excl_pcpu", "excl_numa", "alloc_cnt"):
        print(kk, "state diff nodes", np.flatnonzero((np.atleast_2d(st[kk]) != np.atleast_2d(ns[kk])).any(0))[:10])
