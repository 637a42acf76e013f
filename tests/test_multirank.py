"""World-size-2 gloo run of the multi-GPU bench path's host logic (CPU): pair / gallery sharding
covers every pair exactly once, per-rank host Hungarian on its shard equals the single-process
result, and the max-over-ranks timing reduction.  (The device path is covered by the GPU shard
test: a shard computed alone equals its slice of the full batch bit for bit.)"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mats(n_pairs, n):
    g = torch.Generator().manual_seed(3)
    s = torch.rand(n_pairs, n, n, generator=g)
    s[:, :, :3] = 0.5                              # ties
    return s


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fpm import ops
    res = {}
    for cfg, batch, gallery in (("c3", 6, 0), ("c4", 0, 13)):
        first, cnt = bench.shard(cfg, rank, world, batch, gallery)
        total = batch * world if cfg == "c3" else gallery
        s = _mats(total, 12)[first:first + cnt]
        n = torch.full((cnt,), 12, dtype=torch.int32)
        a = ops.lsa_batch_host(s, n, n, 2) if cnt else torch.empty(0, 12, dtype=torch.int32)
        parts = [None] * world
        dist.all_gather_object(parts, (first, cnt, a.tolist()))
        res[cfg] = parts
    t = bench.reduce_max([float(rank + 1), 10.0 - rank], world)
    if rank == 0:
        with open(os.path.join(out_dir, "res.json"), "w") as f:
            json.dump({"res": res, "t": t}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_rank_sharding(tmp_path, world):
    """World size 2 and 8 (the 8-GPU node's rank count): shard bounds cover every pair once in
    rank order, the gathered per-rank Hungarian results equal the single-process ones, and the
    max-over-ranks timing reduction."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    with open(os.path.join(tmp_path, "res.json")) as f:
        d = json.load(f)
    res, t = d["res"], d["t"]
    assert t == [float(world), 10.0]
    from fpm import ops
    for cfg, total in (("c3", 6 * world), ("c4", 13)):
        parts = sorted(res[cfg], key=lambda p: p[0])
        assert parts[0][0] == 0 and sum(p[1] for p in parts) == total
        assert all(a[0] + a[1] == b[0] for a, b in zip(parts, parts[1:]))
        got = np.concatenate([np.array(p[2], dtype=np.int32) for p in parts if p[1]])
        n = torch.full((total,), 12, dtype=torch.int32)
        ref = ops.lsa_batch_host(_mats(total, 12), n, n, 1).numpy()
        np.testing.assert_array_equal(got, ref)


def test_host_cpu_share_under_torchrun(monkeypatch):
    """torch.distributed.run's OMP_NUM_THREADS=1 default must not shrink the Hungarian pool to
    2 threads per rank: the affinity mask is split over the node's ranks instead."""
    monkeypatch.delenv("FPM_CPU_SHARE", raising=False)
    from fpm.model import host_cpu_share
    n_aff = len(os.sched_getaffinity(0))
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    assert host_cpu_share() == min(16, n_aff)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert host_cpu_share() == 1                      # an explicit single-thread request outside torchrun
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert host_cpu_share() == max(1, min(16, n_aff // 2))
    monkeypatch.setenv("FPM_CPU_SHARE", "1")          # explicit limit honoured under torchrun too
    assert host_cpu_share() == 1
    monkeypatch.setenv("FPM_CPU_SHARE", "3")
    assert host_cpu_share() == min(3, n_aff)


def _cpu_worker(rank, world, port, out_dir):
    """One torchrun-like rank: LOCAL_RANK / LOCAL_WORLD_SIZE set, OMP_NUM_THREADS=1 (the launcher's
    default), pins itself (bench.py's pin_rank_cpus) and reports its CPU set and pool share."""
    os.environ.update(LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    for k in ("FPM_CPU_SHARE", "FPM_RANK_PINNED", "FPM_PIN_RANKS"):
        os.environ.pop(k, None)
    from fpm.model import host_cpu_share, pin_rank_cpus
    before = host_cpu_share()
    cpus = pin_rank_cpus()
    after = host_cpu_share()
    with open(os.path.join(out_dir, "cpu%d.json" % rank), "w") as f:
        json.dump({"cpus": cpus, "mask": sorted(os.sched_getaffinity(0)), "before": before, "after": after}, f)


def test_eight_rank_cpu_split(tmp_path):
    """8 ranks on one node: every rank's host Hungarian pool gets its own non-empty slice of the
    affinity mask (disjoint when the mask has >= 8 CPUs), and its pool share equals the slice (at
    most 16 CPUs) before and after pinning."""
    world = 8
    mp.spawn(_cpu_worker, args=(world, 0, str(tmp_path)), nprocs=world, join=True)
    n_aff = len(os.sched_getaffinity(0))
    sets = []
    for r in range(world):
        with open(os.path.join(tmp_path, "cpu%d.json" % r)) as f:
            d = json.load(f)
        assert d["cpus"] and d["mask"] == sorted(d["cpus"])
        assert d["before"] == d["after"] == min(16, len(d["cpus"])) >= 1
        sets.append(set(d["cpus"]))
    if n_aff >= world:
        assert all(not (a & b) for i, a in enumerate(sets) for b in sets[i + 1:])
        assert all(len(s) == n_aff // world for s in sets)
