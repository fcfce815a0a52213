"""Summarise the rocprofv3 --pmc passes of scripts/pmc.sh into
profiles/pmc_summary_<WORKLOAD>.json (config 4's also profiles/pmc_summary.json):
HBM bytes per launch of every kernel of the run, the evaluation kernel's at
the top level (bench.py reads it as eval_roofline.traffic).

Usage: python scripts/pmc_summary.py NAME [OUT_PREFIX [WORKLOAD]]

Under KOORDHIP_PMC_REPLAY (api.hip pmc_replay) the class lists' launches are
replayed after each serial call: the k_scan dispatches followed by a
k_cls_collect are the class-list builds ("k_scan (class build)"), told apart
from the serial path's own k_scan launches by dispatch order."""
import collections
import csv
import json
import os
import sys

name = sys.argv[1]
prefix = sys.argv[2] if len(sys.argv) > 2 else None
workload = sys.argv[3] if len(sys.argv) > 3 else "config4"
root = os.path.join("gpurun_out", name)


def short(k: str) -> str:
    return k.split("(")[0].replace("void ", "")


per = collections.defaultdict(lambda: collections.defaultdict(list))
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    path = None
    for dp, _, fs in os.walk(os.path.join(root, ctr)):
        for f in fs:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(dp, f)
    if path is None:
        sys.exit(f"no counter file for {ctr}")
    acc = collections.defaultdict(float)   # dispatch id -> value
    kern = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        acc[d] += float(r["Counter_Value"])
        kern[d] = short(r["Kernel_Name"])
    order = sorted(acc)
    for i, d in enumerate(order):
        k = kern[d]
        if "k_scan" in k and i + 1 < len(order) and "k_cls_collect" in kern[order[i + 1]]:
            k = k + " (class build)"
        per[k][ctr].append(acc[d])


def row(v):
    f = sum(v["FETCH_SIZE"]) / max(len(v["FETCH_SIZE"]), 1)
    w = sum(v["WRITE_SIZE"]) / max(len(v["WRITE_SIZE"]), 1)
    return {"launches": len(v["FETCH_SIZE"]), "fetch_bytes_per_launch": int(f * 1024 * 2),
            "write_bytes_per_launch": int(w * 1024), "hbm_bytes_per_launch": int(f * 1024 * 2 + w * 1024),
            "FETCH_SIZE_KB_avg": round(f, 1), "WRITE_SIZE_KB_avg": round(w, 1)}


table = {k: row(v) for k, v in per.items()}
# the evaluation kernel: the class workgroups where the replay ran them, else
# the fused k_eval_topk, else the serial path's k_scan
ev = (next((k for k in table if "k_cls_run" in k), None) or next((k for k in table if "k_eval_topk" in k), None)
      or next((k for k in table if "k_scan" in k and "build" not in k), None))
summary = {
    "source": f"profiles/{prefix or name}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
    "workload": workload,
    "kernel": ev,
    "hbm_bytes_per_launch": table[ev]["hbm_bytes_per_launch"] if ev else None,
    "fetch_bytes_per_launch": table[ev]["fetch_bytes_per_launch"] if ev else None,
    "write_bytes_per_launch": table[ev]["write_bytes_per_launch"] if ev else None,
    "launches": table[ev]["launches"] if ev else None,
    "kernels": table,
    "correction": "FETCH_SIZE x1024 x2 (MI355X_MICROARCH.md: gfx950 reports half of a coalesced read stream; "
                  "the 8-B/lane column loads are uncalibrated, so x2 is an upper estimate); WRITE_SIZE x1024",
    "replay": "k_cls_run / k_cls_collect / class-build k_scan / k_ext_pre / k_ext_final: KOORDHIP_PMC_REPLAY "
              "(api.hip pmc_replay) -- the pipeline's launches replayed one after another on the snapshot state "
              "over the serial call's commit log (rocprofv3 --pmc serialises dispatches, so the persistent "
              "pipeline cannot run under it)",
}
if prefix:
    json.dump(table, open(f"profiles/{prefix}_pmc.json", "w"), indent=1)
    json.dump(summary, open(f"profiles/pmc_summary_{workload}.json", "w"), indent=1)
    if workload == "config4":
        json.dump(summary, open("profiles/pmc_summary.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
