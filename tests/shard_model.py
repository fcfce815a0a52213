"""Executable model of the node-sharded placement round, for
CPU tests over torch.distributed `gloo`.  Test infrastructure: it composes the
oracle (per-(pod,node) Filter/Score, Reserve) the same way libkoordhip.so
composes its kernels, so the N>1 algorithm -- contiguous node shards, exact
per-shard top-k, all-gather, list merge, replicated greedy resolve with
re-evaluation of the nodes committed earlier in the round -- can be checked
against the reference's one-pod-at-a-time loop without a GPU.

Keys follow the device encoding: (score + 1) << 32 | (0xFFFFFFFF - node),
0 = infeasible, larger is better, equal score -> lower node index.
"""
import numpy as np

from koordinator_amd import abi


def keys_of(cfg, out, lo, hi):
    """Per-pod keys of nodes [lo, hi) from an oracle eval result."""
    fmask = 0
    if cfg.filter_plugins & 1:
        fmask |= abi.ST_FIT_FAIL
    if cfg.filter_plugins & 2:
        fmask |= abi.ST_LA_FAIL
    st = out["status"][:, lo:hi]
    sc = out["scores"][:, :, lo:hi].astype(np.int64)
    total = np.zeros(st.shape, np.int64)
    for p in range(abi.NPLUGINS):
        if cfg.score_plugins & (1 << p):
            total += int(cfg.plugin_weight[p]) * sc[:, p, :]
    node = np.arange(lo, hi, dtype=np.int64)
    key = ((total + 1) << 32) | (0xFFFFFFFF - node)
    key[(st & fmask) != 0] = 0
    return key.astype(np.uint64)


def shard_topk(cfg, orc, pods, k, lo, hi):
    """Exact top-k keys of node shard [lo, hi) for every pod: [P][k], 0-padded."""
    out = orc.eval(pods, status=True, scores=True)
    key = keys_of(cfg, out, lo, hi)
    res = np.zeros((len(pods), k), np.uint64)
    if hi > lo:
        srt = np.sort(key, axis=1)[:, ::-1]
        m = min(k, hi - lo)
        res[:, :m] = srt[:, :m]
    return res


def merge_lists(gathered, k):
    """[world][P][k] -> [P][k]: exact top-k of the union (keys are unique)."""
    allk = np.concatenate(list(gathered), axis=1)
    return np.sort(allk, axis=1)[:, ::-1][:, :k].copy()


def resolve_round(cfg, orc, pods, lists):
    """Greedy replay of one round against the exact lists: pod j takes the best
    of (first list entry not committed to this round) and the current keys of
    the nodes committed this round (re-evaluated), then commits."""
    modified = []
    out = np.full(len(pods), -1, np.int32)
    for j in range(len(pods)):
        best = np.uint64(0)
        for x in lists[j]:
            if x == 0:
                break
            node = 0xFFFFFFFF - int(x & np.uint64(0xFFFFFFFF))
            if node not in modified:
                best = x
                break
        if modified:
            ev = orc.eval(pods[j:j + 1], status=True, scores=True)
            kk = keys_of(cfg, ev, 0, orc.n)[0]
            for node in modified:
                if kk[node] > best:
                    best = kk[node]
        if best:
            node = 0xFFFFFFFF - int(best & np.uint64(0xFFFFFFFF))
            orc.commit(pods[j], node)
            if node not in modified:
                modified.append(node)
            out[j] = node
    return out


def place_sharded(cfg, orc, pods, world, rank, batch, all_gather):
    """The rank's view of the sharded stream; `all_gather(arr) -> [world] arrays`."""
    n = orc.n
    lo, hi = n * rank // world, n * (rank + 1) // world
    k = batch
    out = np.full(len(pods), -1, np.int32)
    for p0 in range(0, len(pods), batch):
        pr = pods[p0:p0 + batch]
        mine = shard_topk(cfg, orc, pr, k, lo, hi)
        lists = merge_lists(all_gather(mine), k)
        out[p0:p0 + len(pr)] = resolve_round(cfg, orc, pr, lists)
    return out
