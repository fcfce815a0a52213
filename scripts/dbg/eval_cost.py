"""Diagnostic: per-round k_eval_topk time on the config-5 cluster (200k nodes)
for plugin subsets -- which plugin's evaluation costs the most."""
import copy
import os
import sys
sys.path.insert(0, ".")
from koordinator_amd import synth
from koordinator_amd.config import PLUGIN_NUMA, PLUGIN_RESERVATION, shipped_profile
from koordinator_amd.engine import PlacementEngine

os.environ["KOORDHIP_EVAL"] = "fused"
full = shipped_profile(numa=True, reservation=True)
t = synth.make_cluster(synth.ClusterSpec(200000), full)
synth.add_numa(t, synth.NumaSpec(), full)
synth.add_reservations(t, synth.ResvSpec())
c = synth.CONFIGS[5]
pods = synth.make_pods(synth.StreamSpec(2400, be_frac=c["be_frac"], resv_match_frac=c["resv_match_frac"]), full)


def variant(name, drop):
    p = copy.deepcopy(full)
    p.filters = tuple(f for f in p.filters if f not in drop)
    p.scores = {k: v for k, v in p.scores.items() if k not in drop}
    return name, p


for name, prof in [variant("full", ()), variant("no-NUMA", (PLUGIN_NUMA,)), variant("no-Reservation", (PLUGIN_RESERVATION,)),
                   variant("Fit+LoadAware", (PLUGIN_NUMA, PLUGIN_RESERVATION))]:
    with PlacementEngine(prof, device=0, profile_kernels=True) as e:
        e.load_snapshot(t)
        e.place_stream(pods)
        e.load_snapshot(t)
        e.place_stream(pods)
        ks = e.kernel_stats()
    print(f"{name:16s} eval us/launch {ks['scan_ms'] * 1e3 / max(ks['scan_launches'], 1):8.1f}  pods/round {ks['round_pods']}"
          f"  lag {ks['lag']}  total ms {ks['total_ms']:.1f}", flush=True)
