"""CPU tests of the N>1 path: world_size 2 and 3 over gloo (127.0.0.1).

Covers the pair sharding (weak scaling, global seeds), the pose all-gather
(rank order), the sequence sharding with its 1-frame halo, and rank 0's
ordered trajectory composition — the same helpers bench.py uses over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import youth_dist
import youth_synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 3
        first, cnt = youth_dist.pair_shard(rank, n)
        src, dst, T_gt = youth_synth.pairs(first, cnt, 64, 48)
        local = torch.from_numpy(T_gt.reshape(cnt, 16).astype(np.float32))
        allp = youth_dist.gather_poses(local, world)
        out = torch.zeros((world * cnt, 16), dtype=torch.float32)
        h = youth_dist.gather_poses_async(local, out, world)   # bench.py's double-buffered form
        if h is not None:
            h.wait()
        assert torch.equal(out, allp)
        # sequence: 9 frames -> 8 pairs over 2 ranks with a 1-frame halo
        f0, f1 = youth_dist.sequence_shard(9, world, rank)
        frames, Twc = youth_synth.sequence(f0, f1 - f0, 64, 48)
        rel = np.stack([np.linalg.inv(Twc[k]) @ Twc[k + 1] for k in range(f1 - f0 - 1)])
        rows = youth_dist.gather_ragged(torch.from_numpy(rel.reshape(-1, 16)), world, 8)
        counts = [max(0, (lambda f: f[1] - f[0] - 1)(youth_dist.sequence_shard(9, world, r)))
                  for r in range(world)]
        rows_k = youth_dist.gather_ragged(torch.from_numpy(rel.reshape(-1, 16)), world, 8, counts)
        assert torch.equal(rows, rows_k)
        # bench.py's N > 1 self-report: the group's size and every rank's times
        rep = youth_dist.rank_report({"k_icp_ms": 1.0 + rank, "k_prep_ms": 0.1 * rank,
                                      "gather_ms": 0.01}, world,
                                     {"pose_max_abs_err_vs_cpu": 1e-9 * rank,
                                      "pairs_checked": 4})
        q.put((rank, allp.numpy(), (f0, f1), rows.numpy(), rep))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_world2_gloo_shards_and_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, allp, rng, rows, rep = q.get(timeout=240)
        res[rank] = (allp, rng, rows)
        assert rep["rccl_world_size"] == world and rep["backend"] == "gloo"
        assert rep["per_rank_ms"]["k_icp_ms"] == [1.0 + r for r in range(world)]
        assert np.allclose(rep["per_rank_ms"]["k_prep_ms"], [0.1 * r for r in range(world)])
        assert rep["per_rank_ms"]["gather_ms"] == [0.01] * world
        # non-time figures (bench.py: each rank's pose check against the oracle)
        assert rep["per_rank"]["pairs_checked"] == [4.0] * world
        assert rep["per_rank"]["pose_max_abs_err_vs_cpu"] == [1e-9 * r for r in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank sees the same rank-ordered gather == the global pair list
    _, _, T_all = youth_synth.pairs(0, 3 * world, 64, 48)
    for r in range(world):
        assert np.array_equal(res[r][0], T_all.reshape(3 * world, 16).astype(np.float32))
    # sequence shards tile the 8 pairs with a shared halo frame
    if world == 2:
        assert res[0][1] == (0, 5) and res[1][1] == (4, 9)
    for r in range(1, world):
        assert res[r][1][0] == res[r - 1][1][1] - 1          # one-frame halo
    assert res[0][1][0] == 0 and res[world - 1][1][1] == 9
    rows = res[0][2]
    assert rows.shape == (8, 16)
    for r in range(1, world):
        assert np.array_equal(rows, res[r][2])
    _, Twc = youth_synth.sequence(0, 9, 64, 48)
    traj = youth_dist.compose_trajectory(rows.reshape(8, 4, 4))
    assert np.allclose(traj, np.linalg.inv(Twc[0]) @ Twc, atol=1e-12)


def test_rank_report_without_group():
    rep = youth_dist.rank_report({"k_icp_ms": 2.5}, 1)
    assert rep == {"rccl_world_size": 1, "backend": None, "per_rank_ms": {"k_icp_ms": [2.5]}}
    rep = youth_dist.rank_report({"k_icp_ms": 2.5}, 1, {"pose_max_abs_err_vs_cpu": 3e-14})
    assert rep["per_rank"] == {"pose_max_abs_err_vs_cpu": [3e-14]}


def test_sequence_shard_edge_cases():
    for F in (2, 3, 10, 1000):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                f0, f1 = youth_dist.sequence_shard(F, world, r)
                covered += list(range(f0, max(f0, f1 - 1)))
            assert covered == list(range(F - 1)), (F, world)


def test_pair_shard_weak_scaling():
    assert [youth_dist.pair_shard(r, 64) for r in range(8)][-1] == (448, 64)
