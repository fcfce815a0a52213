"""Debug: eval_ext of the first pods of the device-holding reservation stream, GPU vs oracle."""
import sys
sys.path[:0] = [".", "tests"]
import numpy as np
import torch  # noqa: F401
import oracle
from test_deviceshare_reservation import _dev_resv_cluster, _dev_resv_pods
from koordinator_amd.config import to_c_config
from koordinator_amd.engine import PlacementEngine

prof, t = _dev_resv_cluster(400, seed=42)
pods, ext = _dev_resv_pods(800, prof, seed=42)
o = oracle.Oracle(to_c_config(prof), t)
r = o.eval_ext(pods[:4], ext[:4], k=5)
with PlacementEngine(prof, device=0) as e:
    e.load_snapshot(t)
    g = e.eval_ext(pods[:4], ext[:4], k=5)
for k in ("status", "scores", "topk"):
    bad = np.argwhere(g[k] != r[k])
    print(k, "mismatches", len(bad), bad[:10].tolist())
print("gpu topk", g["topk"][0].tolist())
print("orc topk", r["topk"][0].tolist())
for i in (129, 287):
    print(i, "gpu", g["status"][0, i], g["scores"][0, :, i].tolist(), "orc", r["status"][0, i], r["scores"][0, :, i].tolist())
