"""Writes fit_cases.json: the reference-held vectors of the fitsRequest
arithmetic (data only) -- the non-reservation rows of Test_filterWithReservations
(reservation/plugin_test.go:725-807), where fitsNode (reservation/plugin.go:445-494)
with rInfo = nil is NodeResourcesFit's fitsRequest on
Requested' = podRequested - preemptible:

  podRequest.X > Allocatable.X - (podRequested.X - preemptible.X)  -> does not fit

The test node: allocatable cpu 32, memory 32Gi, pods 100 (:528-539); the pod
requests cpu 4.  A row without any preemptible resources skips the check (:383)
and is left out.  preemptibleInRRs without a node entry leaves preemptible 0 (:763-786).
"""
import json
import os

S = "reservation/plugin_test.go:"
CASES = [
    {"name": "filter non-reservations with preemption", "source": S + "725-745",
     "alloc_cpu_m": 32000, "pod_requested_cpu_m": 32000, "preemptible_cpu_m": 4000, "req_cpu_m": 4000, "fits": True},
    {"name": "filter non-reservations with preemption but no preemptible resources and have preemptibleInRR",
     "source": S + "763-786", "alloc_cpu_m": 32000, "pod_requested_cpu_m": 32000, "preemptible_cpu_m": 0,
     "req_cpu_m": 4000, "fits": False},
    {"name": "filter non-reservations with preemption (2 preemptible)", "source": S + "787-807",
     "alloc_cpu_m": 32000, "pod_requested_cpu_m": 32000, "preemptible_cpu_m": 2000, "req_cpu_m": 4000, "fits": False},
]


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fit_cases.json")
    with open(path, "w") as f:
        json.dump({"fits_request": CASES, "alloc_mem": 32 * 2**30, "alloc_pods": 100}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
