"""Writes reservation_cases.json: Reservation plugin known-answer tests
transcribed from the reference's table tests (data only).

  plugins/reservation/scoring_test.go:39-243    TestScore (single-reservation rows)
  plugins/reservation/scoring_test.go:245-379   TestScoreWithOrder (raw and normalized scores)
  plugins/reservation/plugin_test.go:545-724    Test_filterWithReservations, the matched
                                                Aligned / Restricted rows without preemption
  plugins/reservation/plugin_test.go:1485-1666  TestFilterReservation (nomination)
  plugins/reservation/transformer_test.go:40-345  TestRestoreReservation, per reservation:
                                                the unmatched and the matched restore deltas
  plugins/reservation/transformer_test.go:347-441 Test_matchReservation (owner row)

Quantities: cpu as Kubernetes quantity strings, memory likewise.  Rows with
two reservations on one node are left out (one reservation per node on the
device; the reference orders several by Go map iteration), as are the
preemption rows (no preemption state in a placement stream).
"""
import json
import os

GI = "Gi"


def res(cpu=None, mem=None):
    r = {}
    if cpu is not None:
        r["cpu"] = cpu
    if mem is not None:
        r["memory"] = mem
    return r


S = "scoring_test.go:"
SCORE = [
    {"name": "reservation matched but zero-request pod", "source": S + "124-132",
     "reservation": {"allocatable": res("2", "4Gi")}, "pod": {}, "want_raw": 0},
    {"name": "reservation matched and pod has part empty resource requests", "source": S + "133-153",
     "reservation": {"allocatable": res("4", "8Gi")}, "pod": res("2", "4Gi"), "want_raw": 50},
    {"name": "allocated reservation matched and pod has part empty resource requests", "source": S + "154-180",
     "reservation": {"allocatable": res("2", "4Gi"), "allocated": res("2", "3Gi")}, "pod": res("2", "4Gi"),
     "want_raw": 0},
]

ORDER = {"name": "TestScoreWithOrder", "source": S + "245-379",
         "reservations": [{"node": f"test-node-{i}", "allocatable": res("4", "8Gi")} for i in (1, 2, 3)]
         + [{"node": "test-node-4", "allocatable": res("4", "8Gi"), "order": "123456"}],
         "pod": res("4", "8Gi"), "want_raw": [100, 100, 100, 1000], "want_normalized": [10, 10, 10, 100],
         "want_preferred": "test-node-4"}

P = "plugin_test.go:"
# node allocatable 32 cpu / 32Gi / 100 pods (:528-539); podRequested as the state holds it
FILTER = [
    {"name": "filter aligned reservation with nodeInfo", "source": P + "546-589", "policy": "Aligned",
     "pod": res("8", "8Gi"), "pod_requested": res("30", "24Gi"), "reservation": {"allocatable": res("6")},
     "want": True},
    {"name": "failed to filter aligned reservation with nodeInfo", "source": P + "590-634", "policy": "Aligned",
     "pod": res("8", "8Gi"), "pod_requested": res("32", "24Gi"), "reservation": {"allocatable": res("6")},
     "want": False},
    {"name": "filter restricted reservation with nodeInfo", "source": P + "635-679", "policy": "Restricted",
     "pod": res("6", "8Gi"), "pod_requested": res("30", "24Gi"), "reservation": {"allocatable": res("6")},
     "want": True},
    {"name": "failed to filter restricted reservation with nodeInfo", "source": P + "680-724", "policy": "Restricted",
     "pod": res("8", "8Gi"), "pod_requested": res("30", "24Gi"), "reservation": {"allocatable": res("6")},
     "want": False},
]

NOMINATE = [
    {"name": "satisfied reservation", "source": P + "1567-1579", "pod": res("2", "4Gi"),
     "reservation": {"allocatable": res("2", "4Gi")}, "want": True},
    {"name": "intersection resource names", "source": P + "1580-1591", "pod": res("2"),
     "reservation": {"allocatable": res("2", "4Gi")}, "want": True},
    {"name": "no intersection resource names", "source": P + "1592-1603", "pod": {"ephemeral-storage": "2Gi"},
     "reservation": {"allocatable": res("2", "4Gi")}, "want": False},
]

T = "transformer_test.go:"
# node 32 cpu / 64Gi; normal pods 4C8Gi + 8C16Gi; Requested before the restore 36C/72Gi (:285-289)
RESTORE = {
    "source": T + "40-345", "node": res("32", "64Gi"), "pods": [res("4", "8Gi"), res("8", "16Gi")],
    "requested_before": res("36", "72Gi"),
    "unmatched": {"allocatable": res("12", "24Gi"), "allocate_once": False,
                  "assigned": [res("4", "8Gi")], "want_delta": res("-4", "-8Gi")},
    "matched": {"allocatable": res("8", "16Gi"), "owner_labels": {"test-reservation": "true"},
                "want_delta": res("-8", "-16Gi"), "want_pods_delta": -1},
    "pod_labels": {"test-reservation": "true"},
    # podRequested = Requested after the unmatched restore (:317-320); the node's Requested after both
    "want_pod_requested": res("32", "64Gi"), "want_requested_after": res("24", "48Gi"),
}

MATCH = [
    {"name": "only match reservation owners", "source": T + "355-378", "pod_labels": {"app": "test"},
     "owner_labels": {"app": "test"}, "want": True},
]

if __name__ == "__main__":
    out = {"score": SCORE, "order": ORDER, "filter": FILTER, "nominate": NOMINATE, "restore": RESTORE,
           "match": MATCH}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reservation_cases.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)
