"""Host enqueue time of one place_staged call vs its device completion
(config 4), with and without a one-rank RCCL communicator."""
import sys
import time

sys.path.insert(0, ".")
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile
from koordinator_amd.engine import PlacementEngine

comm = len(sys.argv) > 1 and sys.argv[1] == "comm"
prof = shipped_profile()
table, pods = synth.config_workload(4, prof)
eng = PlacementEngine(prof, device=0)
if comm:
    eng.comm_init(PlacementEngine.comm_unique_id(), 1, 0)
eng.load_snapshot(table)
eng.checkpoint()
eng.stage_pods(pods)
for it in range(3):
    eng.restore()
    eng.synchronize()
    t0 = time.perf_counter()
    eng.place_staged()
    t1 = time.perf_counter()
    eng.synchronize()
    t2 = time.perf_counter()
    print(f"comm={comm} enqueue {1e3 * (t1 - t0):.1f} ms, total {1e3 * (t2 - t0):.1f} ms", flush=True)
