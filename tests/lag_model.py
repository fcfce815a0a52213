"""CPU model of the lag-1 round pipeline of koordhip_place_staged (test
infrastructure, built on the oracle): round r's per-pod top-k lists come from
the state at the END of round r-2 (what k_scan may see while round r-1 is
being resolved), then k_resolve's rules are replayed exactly -- refresh of the
list entries on round r-1's nodes, re-sort, first entry outside this round's
committed set M, re-evaluation of M when it ranks above that entry, of M and
M' for non-monotone pods.  It must reproduce the oracle's sequential greedy
bit for bit; tests/test_lag_model.py checks that on CPU, independently of the
kernels."""
import numpy as np

import oracle
from koordinator_amd import abi


def _totals(o: oracle.Oracle, cfg, pod) -> np.ndarray:
    """Total score + 1 of one pod on every node of o's current state (0 = infeasible)."""
    r = o.eval(np.atleast_1d(pod), status=True, scores=True)
    st, sc = r["status"][0], r["scores"][0].astype(np.int64)
    tot = np.zeros(o.n, np.int64)
    for p in range(abi.NPLUGINS):
        if cfg.score_plugins & (1 << p):
            tot += cfg.plugin_weight[p] * sc[p]
    return np.where(st == 0, tot + 1, 0)


def _key(v: int, node: int) -> int:
    return 0 if v <= 0 else (int(v) << 32) | (0xFFFFFFFF - node)


def _node(key: int) -> int:
    return 0xFFFFFFFF - (key & 0xFFFFFFFF)


def _nonmono(pod) -> bool:
    f = int(pod["flags"])
    cpuset = (f & abi.POD_CPUSET) and not (f & (abi.POD_NUMA_SKIP | abi.POD_NUMA_ERROR))
    return bool(cpuset and (int(pod["numa_policy"]) & 3) != 0)


def place_lagged(cfg, table, pods, batch: int) -> np.ndarray:
    k = 2 * batch
    # a MostAllocated NodeNUMAResource score rises with commits: every pod re-evaluates M and M'
    monotone = not ((cfg.score_plugins & abi.PLUGIN_NUMA) and cfg.numa_most_allocated)
    cur = oracle.Oracle(cfg, table)   # the live state
    lag = oracle.Oracle(cfg, table)   # state at the end of round r - 2
    out = np.full(len(pods), abi.UNSCHEDULABLE, np.int32)
    commits = []                      # per round: [(pod, node)]
    prev = []                         # M' = nodes committed in round r - 1
    for r, p0 in enumerate(range(0, len(pods), batch)):
        if r >= 2:
            for pod, node in commits[r - 2]:
                lag.commit(pod, node)
        rp = pods[p0:p0 + batch]
        lists = []
        for pod in rp:
            v = _totals(lag, cfg, pod)
            keys = sorted((_key(v[i], i) for i in np.flatnonzero(v)), reverse=True)[:k]
            lists.append(keys)
        # prologue: refresh entries on M' against the state at round start, re-sort
        if prev:
            pset = set(prev)
            for j, pod in enumerate(rp):
                v = _totals(cur, cfg, pod)
                lists[j] = sorted((_key(v[_node(e)], _node(e)) if _node(e) in pset else e for e in lists[j]),
                                  reverse=True)
        M, done = [], []
        for j, pod in enumerate(rp):
            L = [e for e in lists[j] if e]
            first = next((q for q, e in enumerate(L) if _node(e) not in M), None)
            cand = L[first] if first is not None else 0
            prefix_mod = any(_node(e) in M for e in L[:first if first is not None else len(L)])
            best = cand
            nonmono = _nonmono(pod) or not monotone
            if M and (prefix_mod or nonmono):
                v = _totals(cur, cfg, pod)
                best = max([best] + [_key(v[i], i) for i in M])
            if nonmono and prev:
                v = _totals(cur, cfg, pod)
                best = max([best] + [_key(v[i], i) for i in prev if i not in M])
            if best == 0:
                continue
            w = _node(best)
            rc, _ = cur.commit(pod, w)
            if rc == abi.E_RESERVE:
                out[p0 + j] = abi.RESERVE_FAILED
                continue
            out[p0 + j] = w
            done.append((pod, w))
            if w not in M:
                M.append(w)
        commits.append(done)
        prev = M
    return out
