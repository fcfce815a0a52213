"""Debug: where the device's eval scores differ from the oracle's on the
reserved-CPU workload (tests/test_resv_cpus.py)."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import oracle
from koordinator_amd import abi
from koordinator_amd.config import to_c_config
from koordinator_amd.engine import PlacementEngine
from test_resv_cpus import _workload, _resv_cpu_masks

prof, t, pods = _workload(1500, 48)
o = oracle.Oracle(to_c_config(prof), t)
ref = o.eval(pods, k=16)
with PlacementEngine(prof, device=0) as e:
    e.load_snapshot(t)
    got = e.eval(pods, k=16)
d = np.argwhere(ref["scores"] != got["scores"])
print("mismatches", len(d), "planes", np.unique(d[:, 1], return_counts=True))
m = _resv_cpu_masks(t)
n = t.n
for p, pl, i in d[:25]:
    P = [m[w, q * n + i] for q in range(t.resv_slots) for w in range(4)]
    pc = sum(bin(int(x)).count("1") for x in P)
    fr = sum(bin(int(t[f"numa_free{w}"][i])).count("1") for w in range(4))
    print(f"pod {p} plane {pl} node {i}: ref {ref['scores'][p, pl, i]} got {got['scores'][p, pl, i]} "
          f"st {ref['status'][p, i]} flags {pods['flags'][p]:#x} need {pods['numa_cpus'][p]} pol {pods['numa_policy'][p]:#x} "
          f"match {pods['resv_match'][p]:#x} cnt {t['numa_alloc_cnt'][i]} free {fr} resv_cpus(all slots) {pc} "
          f"rflags {[int(t['resv_flags' + (f'@{q}' if q else '')][i]) for q in range(t.resv_slots)]}")
