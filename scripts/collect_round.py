"""Copy one GPU pass's evidence (scripts/gpu_round.sh, ROUND=R) from the
scratch gpurun_out/ into the tracked profiles/:
  profiles/R_<w>_bench.json           the bench line
  profiles/R_<w>_kernel_stats.csv     rocprofv3 --kernel-trace --stats summary
  profiles/R_<w>_resolve_stamps.txt   KOORDHIP_STAMPS lines
  profiles/R_<w>_pmc.json + pmc_summary_<w>.json   FETCH_SIZE / WRITE_SIZE passes
  profiles/R_gpu_pytest_tail.txt      the pytest summary
Usage: python scripts/collect_round.py R [workloads...]"""
import glob
import json
import os
import shutil
import subprocess
import sys

R = sys.argv[1]
W = sys.argv[2:] or ["config4", "config3", "config5"]
G, P = "gpurun_out", "profiles"
for w in W:
    b = f"{G}/bench_{R}_{w}.json"
    if os.path.exists(b):
        line = open(b).read().strip().splitlines()[-1]
        json.loads(line)
        open(f"{P}/{R}_{w}_bench.json", "w").write(line + "\n")
        print("bench", w)
    st = glob.glob(f"{G}/{R}_{w}/**/*kernel_stats.csv", recursive=True)
    if st:
        shutil.copy(st[0], f"{P}/{R}_{w}_kernel_stats.csv")
        print("kernel stats", w)
    s = f"{G}/stamps_{R}_{w}.err"
    if os.path.exists(s):
        lines = [x for x in open(s) if "[koordhip stamps]" in x]
        open(f"{P}/{R}_{w}_resolve_stamps.txt", "w").writelines(lines)
        print("stamps", w, len(lines))
    if os.path.isdir(f"{G}/pmc_{R}_{w}"):
        subprocess.run([sys.executable, "scripts/pmc_summary.py", f"pmc_{R}_{w}", f"{R}_{w}", w], check=True,
                       stdout=subprocess.DEVNULL)
        print("pmc", w)
t = f"{G}/{R}_pytest.log"
if os.path.exists(t):
    lines = open(t).read().splitlines()
    open(f"{P}/{R}_gpu_pytest_tail.txt", "w").write("\n".join(lines[-6:]) + "\n")
    print("pytest tail")
