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
for npods in (64, 128, 192, 256):
    o = oracle.Oracle(cfg, table)
    ref, rcs = o.place_stream(pods[:npods], cpusets=True)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods[:npods])
        cs = e.fetch_cpusets(npods)
        st = e.read_numa(); s2 = e.read_nodes()
    ns = o.numa_state(); rs = o.state()
    print(npods, "placement diffs", np.flatnonzero(got != ref)[:5], "cpuset diffs", np.flatnonzero((cs != rcs).any(1))[:8])
    for kk in ("free", "excl_pcpu", "excl_numa", "alloc_cnt"):
        d = np.flatnonzero((np.atleast_2d(st[kk]) != np.atleast_2d(ns[kk])).any(0))
        print("  ", kk, "diff nodes", d[:10])
    for kk in ("requested", "npods", "la_used"):
        d = np.flatnonzero((np.atleast_2d(s2[kk]) != np.atleast_2d(rs[kk])).any(0))
        print("  ", kk, "diff nodes", d[:10])
    w = np.flatnonzero(ref == 511)
    print("   pods on 511:", w, [(int(pods[i]['flags']), int(pods[i]['numa_policy']), int(pods[i]['numa_cpus'])) for i in w])
