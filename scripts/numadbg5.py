import sys
import numpy as np
sys.path.insert(0, '/root/repo')
import oracle
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile, to_c_config
from koordinator_amd.engine import PlacementEngine

j = int(sys.argv[1])
prof = shipped_profile(numa=True)
table = synth.make_cluster(synth.ClusterSpec(600), prof)
synth.add_numa(table, synth.NumaSpec(), prof)
pods = synth.make_pods(synth.StreamSpec(64, be_frac=0.2, cpuset_frac=0.5), prof)
cfg = to_c_config(prof)
ref, rcs = oracle.Oracle(cfg, table).place_stream(pods, cpusets=True)
o2 = oracle.Oracle(cfg, table)
with PlacementEngine(prof, device=0) as e:
    e.load_snapshot(table)
    for i in range(j):
        if ref[i] >= 0:
            e.commit(pods[i], int(ref[i]))
            o2.commit(pods[i], int(ref[i]))
    c = e.commit(pods[j], int(ref[j]))
    rc, oc = o2.commit(pods[j], int(ref[j]))
print("k_commit cpus", [hex(int(x)) for x in c], "oracle commit", [hex(int(x)) for x in oc],
      "oracle stream", [hex(int(x)) for x in rcs[j]])
