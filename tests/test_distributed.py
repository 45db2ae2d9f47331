"""world_size-2 gloo tests of the sharding and logging collectives (CPU)."""
import importlib
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_envs_cover_and_balance():
    sh = importlib.import_module("diffusion-piano_amd.sharding")
    for total, world in ((32768, 8), (4096, 1), (10, 3), (7, 7)):
        parts = [sh.shard_envs(total, r, world) for r in range(world)]
        assert parts[0].start == 0 and parts[-1].stop == total
        assert all(a.stop == b.start for a, b in zip(parts, parts[1:]))
        assert max(p.count for p in parts) - min(p.count for p in parts) <= 1
    with pytest.raises(ValueError):
        sh.shard_envs(3, 0, 4)
    with pytest.raises(ValueError):
        sh.shard_envs(8, 2, 2)


def test_episode_returns_single_process():
    sh = importlib.import_module("diffusion-piano_amd.sharding")
    er = sh.EpisodeReturns(3, "cpu")
    # env 0: 2-step episode (MID, LAST) then auto-reset FIRST; env 1 never ends
    for st, r in (([1, 1, 1], [1.0, 2.0, 3.0]), ([2, 1, 1], [1.0, 2.0, 3.0]), ([0, 1, 2], [0.0, 1.0, 1.0])):
        er.update(torch.tensor(r), torch.tensor(st, dtype=torch.uint8))
    s, n, rs, ne = er.gather()
    assert n == 2 and s == pytest.approx(2.0 + 7.0)
    assert rs == pytest.approx(0.0 + 5.0 + 7.0) and ne == 3


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = importlib.import_module("diffusion-piano_amd.sharding")
        shard = sh.shard_envs(8, rank, world)
        er = sh.EpisodeReturns(shard.count, "cpu")
        # every env gets reward = its global id, episode of one step ending with LAST
        ids = torch.arange(shard.start, shard.stop, dtype=torch.float32)
        er.update(ids, torch.full((shard.count,), 2, dtype=torch.uint8))
        s, n, _, ne = er.gather()
        t = sh.max_over_ranks(1.0 + rank)
        q.put((rank, s, n, ne, t))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gather_and_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, s, n, ne, t in res:
        assert s == pytest.approx(sum(range(8))) and n == 8 and ne == 8 and t == 2.0
