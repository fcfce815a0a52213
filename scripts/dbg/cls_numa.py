import os, sys, numpy as np
sys.path.insert(0, "/root/repo")
import oracle
from koordinator_amd import synth, abi
from koordinator_amd.config import shipped_profile, to_c_config
from koordinator_amd.engine import PlacementEngine
import torch
for mode in sys.argv[1:]:
    for k in ("KOORDHIP_CU_RESERVE", "KOORDHIP_LAG2", "KOORDHIP_CLS_OFF"):
        os.environ.pop(k, None)
    if mode != "default":
        os.environ[mode] = "1"
    prof = shipped_profile(numa=True)
    prof.batch_pods = 16
    table = synth.make_cluster(synth.ClusterSpec(400), prof)
    synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(700, be_frac=0.3, cpuset_frac=0.4), prof)
    raw = pods.view(np.uint8).reshape(len(pods), -1)
    print(mode, "classes", len(np.unique(raw, axis=0)), flush=True)
    ref = oracle.Oracle(to_c_config(prof), table).place_stream(pods)
    try:
        with PlacementEngine(prof, device=0) as e:
            e.load_snapshot(table)
            got = e.place_stream(pods)
            print(mode, "kernels", e.kernel_names(), "match", bool(np.array_equal(got, ref)), flush=True)
    except Exception as ex:
        print(mode, "ERR", ex, flush=True)
