import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import oracle
from koordinator_amd import synth, abi
from koordinator_amd.config import shipped_profile, to_c_config
from koordinator_amd.engine import PlacementEngine
j = int(sys.argv[1])
prof = shipped_profile(numa=True)
table = synth.make_cluster(synth.ClusterSpec(600), prof)
synth.add_numa(table, synth.NumaSpec(), prof)
pods = synth.make_pods(synth.StreamSpec(64, be_frac=0.2, cpuset_frac=0.5), prof)
cfg = to_c_config(prof)
o = oracle.Oracle(cfg, table)
ref, rcs = o.place_stream(pods, cpusets=True)
with PlacementEngine(prof, device=0) as e:
    e.load_snapshot(table)
    got = e.place_stream(pods)
    cs = e.fetch_cpusets(64)
print("pod", j, "node", ref[j], got[j], "oracle cpus", [hex(int(x)) for x in rcs[j]], "gpu", [hex(int(x)) for x in cs[j]])
print("pod fields", pods[j])
o2 = oracle.Oracle(cfg, table)
for i in range(j):
    if ref[i] >= 0: o2.commit(pods[i], int(ref[i]))
ns = o2.numa_state(); w = int(ref[j])
print("oracle row", w, [hex(int(ns['free'][q][w])) for q in range(4)], hex(int(ns['excl_pcpu'][0][w])), hex(int(ns['excl_numa'][0][w])), ns['alloc_cnt'][w])
