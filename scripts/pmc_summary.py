"""Summarise the rocprofv3 --pmc passes of scripts/pmc.sh into
profiles/pmc_summary.json (HBM bytes per launch of the evaluation kernel) and
a per-kernel table.  Usage: python scripts/pmc_summary.py NAME [OUT_PREFIX [WORKLOAD]]
(WORKLOAD other than config4 writes profiles/pmc_summary_<WORKLOAD>.json)"""
import csv
import collections
import json
import os
import sys

name = sys.argv[1]
prefix = sys.argv[2] if len(sys.argv) > 2 else None
workload = sys.argv[3] if len(sys.argv) > 3 else "config4"
root = os.path.join("gpurun_out", name)
per = collections.defaultdict(lambda: collections.defaultdict(list))
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    path = None
    for dp, _, fs in os.walk(os.path.join(root, ctr)):
        for f in fs:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(dp, f)
    if path is None:
        sys.exit(f"no counter file for {ctr}")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        per[k][ctr + "_KB_avg"] = sum(d.values()) / len(d)
        per[k]["launches"] = len(d)
table = {k: dict(v) for k, v in per.items()}
# the evaluation kernel: the fused k_eval_topk where it ran, else k_scan
scan = next((k for k in table if "k_eval_topk" in k), None) or next(k for k in table if "k_scan" in k)
f_kb, w_kb = table[scan]["FETCH_SIZE_KB_avg"], table[scan]["WRITE_SIZE_KB_avg"]
summary = {
    "source": f"profiles/{prefix or name}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
    "kernel": scan,
    "hbm_bytes_per_launch": int(f_kb * 1024 * 2 + w_kb * 1024),
    "fetch_bytes_per_launch": int(f_kb * 1024 * 2),
    "write_bytes_per_launch": int(w_kb * 1024),
    "workload": workload,
    "launches": table[scan]["launches"],
    "correction": "FETCH_SIZE x1024 x2 (MI355X_MICROARCH.md: gfx950 reports half of a coalesced read stream; "
                  "the 8-B/lane column loads are uncalibrated, so x2 is an upper estimate); WRITE_SIZE x1024",
}
if prefix:
    json.dump(table, open(f"profiles/{prefix}_pmc.json", "w"), indent=1)
    json.dump(summary, open(f"profiles/pmc_summary_{workload}.json", "w"), indent=1)
    if workload == "config4":
        json.dump(summary, open("profiles/pmc_summary.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
