"""Pins the CPU oracle (and the host marshaller feeding it) against the
known-answer tables of the reference's own tests, transcribed in
tests/golden/*.json with their file:line provenance."""
import pytest

import oracle
from koordinator_amd import abi, k8s, marshal
from koordinator_amd.config import to_c_config

import golden_cases as G


@pytest.mark.parametrize("name,case,node", G.score_cases(), ids=[c[0] for c in G.score_cases()])
def test_loadaware_score_kat(name, case, node):
    profile, table, rec = G.build_case(case, node)
    o = oracle.Oracle(to_c_config(profile), table)
    out = o.eval(rec, status=True, scores=True)
    assert out["scores"][0, 1, 0] == case["want"], case["source"]


@pytest.mark.parametrize("name,case,node", G.filter_cases(), ids=[c[0] for c in G.filter_cases()])
def test_loadaware_filter_kat(name, case, node):
    profile, table, rec = G.build_case(case, node, test_pod_key="test_pod")
    o = oracle.Oracle(to_c_config(profile), table)
    out = o.eval(rec, status=True, scores=False)
    ok = (out["status"][0, 0] & abi.ST_LA_FAIL) == 0
    assert ok == case["want_ok"], case["source"]


def test_estimator_kat():
    d = G.load("estimator.json")
    for c in d["estimate_pod"]:
        args = G.make_args({"estimated_scaling_factors": c["factors"]} if c["factors"] else {}).with_defaults()
        got = marshal.estimate_pod(G.make_pod(c["pod"]), args)
        assert got == c["want"], c["source"]
    for c in d["estimate_node"]:
        node = k8s.Node("n", allocatable=G.rlist(c["allocatable"]), annotations=c["annotations"])
        got = marshal.estimate_node(node)
        assert got == G.rlist(c["want"]), c["source"]


def test_usage_percent_rounding():
    # load_aware_test.go filter table: 60/96 = 62.5% -> 63 (< 65 passes), 70/96 -> 73
    assert oracle.usage_percent(60000, 96000) == 63
    assert oracle.usage_percent(70000, 96000) == 73
    assert oracle.usage_percent(63000, 96000) == 66
    # exact half rounds away from zero (math.Round), unlike rint
    assert oracle.usage_percent(1, 200) == 1
    assert oracle.usage_percent(5, 1000) == 1
    assert oracle.usage_percent(0, 1) == 0


def test_least_requested():
    assert oracle.least_requested(0, 0) == 0
    assert oracle.least_requested(11, 10) == 0
    assert oracle.least_requested(45600, 96000) == 52   # SURVEY §4 hand check, "load node"
    assert oracle.least_requested(10, 10) == 0
    assert oracle.least_requested(0, 10) == 100
