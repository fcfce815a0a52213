"""N>1 path on CPU: node-index shards, exact per-shard top-k,
all-gather over torch.distributed `gloo` (world_size 2, two processes), merge
and the replicated greedy resolve must reproduce the reference's one-pod-at-a-
time placements on every rank.  The GPU version of the same composition is
tests/test_gpu_parity.py::test_sharded_group_bit_exact."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import shard_model as SM
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile, to_c_config


def _workload(n_nodes, n_pods, be, batch):
    prof = shipped_profile()
    prof.batch_pods = batch
    table = synth.make_cluster(synth.ClusterSpec(n_nodes), prof)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=be), prof)
    return to_c_config(prof), table, pods


def test_keys_match_oracle_topk():
    cfg, table, pods = _workload(300, 20, 0.3, 8)
    o = oracle.Oracle(cfg, table)
    got = SM.shard_topk(cfg, o, pods, 8, 0, table.n)
    ref = o.eval(pods, k=8)["topk"]
    node = np.where(got != 0, 0xFFFFFFFF - (got & np.uint64(0xFFFFFFFF)).astype(np.int64), -1)
    assert np.array_equal(node, ref["node"])


@pytest.mark.parametrize("world,n_nodes,n_pods,be,batch", [(3, 400, 300, 0.3, 16), (4, 37, 150, 0.5, 8),
                                                            (5, 4, 30, 0.3, 4)])
def test_sharded_model_in_process(world, n_nodes, n_pods, be, batch):
    """All ranks simulated in one process (lock-step rounds)."""
    cfg, table, pods = _workload(n_nodes, n_pods, be, batch)
    ref = oracle.Oracle(cfg, table).place_stream(pods)
    orcs = [oracle.Oracle(cfg, table) for _ in range(world)]
    n = table.n
    outs = [np.full(len(pods), -1, np.int32) for _ in range(world)]
    for p0 in range(0, len(pods), batch):
        pr = pods[p0:p0 + batch]
        mine = [SM.shard_topk(cfg, orcs[r], pr, batch, n * r // world, n * (r + 1) // world) for r in range(world)]
        for r in range(world):
            outs[r][p0:p0 + len(pr)] = SM.resolve_round(cfg, orcs[r], pr, SM.merge_lists(mine, batch))
    for r in range(world):
        assert np.array_equal(outs[r], ref), r


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, case, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, table, pods = _workload(*case)
        o = oracle.Oracle(cfg, table)

        def all_gather(arr):
            t = torch.from_numpy(arr.view(np.int64).copy())
            bufs = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(bufs, t)
            return [b.numpy().view(np.uint64) for b in bufs]

        out = SM.place_sharded(cfg, o, pods, world, rank, case[3], all_gather)
        np.save(os.path.join(result_dir, f"rank{rank}.npy"), out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", [(500, 400, 0.3, 32), (61, 200, 0.5, 16)])
def test_sharded_gloo_world2(tmp_path, case):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True)
    cfg, table, pods = _workload(*case)
    ref = oracle.Oracle(cfg, table).place_stream(pods)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert np.array_equal(got, ref), (r, int(np.flatnonzero(got != ref)[0]))
