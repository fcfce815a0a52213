import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import oracle
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile, to_c_config
from koordinator_amd.engine import PlacementEngine
cases = [tuple(float(x) if '.' in x else int(x) for x in a.split(',')) for a in sys.argv[1:]]
for (n, np_, batch, cf) in cases:
    prof = shipped_profile(numa=True); prof.batch_pods = batch
    table = synth.make_cluster(synth.ClusterSpec(n), prof)
    synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(np_, be_frac=0.2, cpuset_frac=cf), prof)
    cfg = to_c_config(prof)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
    ref = oracle.Oracle(cfg, table).place_stream(pods)
    bad = np.flatnonzero(got != ref)
    print(n, np_, batch, cf, "mismatch", len(bad), bad[:6], got[bad[:6]], ref[bad[:6]], flush=True)
