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
        # per-env float32 returns, uneven shards: 7 envs over 2 ranks (4 + 3)
        odd = sh.shard_envs(7, rank, world)
        er2 = sh.EpisodeReturns(odd.count, "cpu")
        er2.update(torch.arange(odd.start, odd.stop, dtype=torch.float32) * 0.5,
                   torch.full((odd.count,), 1, dtype=torch.uint8))
        er2.update(torch.ones(odd.count), torch.tensor([2 if (odd.start + i) % 2 == 0 else 1
                                                      for i in range(odd.count)], dtype=torch.uint8))
        per_env = sh.gather_episode_returns(er2, odd, 7)
        q.put((rank, s, n, ne, t, per_env.dtype == torch.float32, per_env.tolist()))
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
    import math
    for rank, s, n, ne, t, is_f32, per_env in res:
        assert s == pytest.approx(sum(range(8))) and n == 8 and ne == 8 and t == 2.0
        # every rank holds all 7 envs in global order: even ids finished with 0.5 g + 1, odd ones
        # have not finished an episode (NaN)
        assert is_f32 and len(per_env) == 7
        for g, v in enumerate(per_env):
            assert (v == pytest.approx(0.5 * g + 1.0)) if g % 2 == 0 else math.isnan(v)


# ------------------------------------------------------------------ bench.py rank logic
class StubEnv:
    """bench.py's view of an env on CPU: step() returns (obs, reward, discount, step_type) with
    an episode of T steps per env (LAST at t_idx == T - 1, FIRST after it), reward 1 per MID."""

    def __init__(self, n, T):
        self.num_envs, self.T = n, T
        self.t = torch.zeros(n, dtype=torch.int64)
        self.last = torch.zeros(n, dtype=torch.bool)
        self.steps = 0

    def set_state(self, s):
        self.t = torch.as_tensor(s["t_idx"]).to(torch.int64)

    def step(self, a):
        self.steps += 1
        first = self.last.clone()
        self.t = torch.where(first, torch.zeros_like(self.t), self.t + 1)
        self.last = ~first & (self.t == self.T)
        st = torch.where(first, torch.zeros_like(self.t), torch.where(self.last, 2, 1)).to(torch.uint8)
        rew = torch.where(first, torch.zeros(self.num_envs), torch.ones(self.num_envs))
        return None, rew, None, st


def _bench_worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    world_, rank_, local, dev = bench.setup_distributed("gloo")
    try:
        sh = importlib.import_module("diffusion-piano_amd.sharding")
        shard = sh.shard_envs(10 * world_, rank_, world_)
        env = StubEnv(shard.count, T=4)
        bench.stagger_episodes(env, shard.start, env.T)
        staggered = env.t.tolist()
        er = sh.EpisodeReturns(shard.count, dev)
        elapsed, kms = bench.timed_rollout(env, [None], steps=6, warmup=2, dev=dev, returns=er, sharding=sh)
        s, n, _, ne = er.gather()
        q.put((rank_, world_, str(dev), staggered, env.steps, elapsed, kms, n, ne))
    finally:
        dist.destroy_process_group()


def test_bench_rank_logic_gloo_world2():
    """bench.py's rank path on CPU: device before the process group, staggered episode phase
    keyed by global env id, W + K steps, wall time max over ranks, returns gathered."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert [r[0] for r in res] == [0, 1] and all(r[1] == 2 and r[2] == "cpu" for r in res)
    assert res[0][3] == [g % 4 for g in range(10)] and res[1][3] == [g % 4 for g in range(10, 20)]
    assert all(r[4] == 8 for r in res)  # warmup + timed steps
    assert res[0][5] == res[1][5]  # the max over ranks, the same on both
    assert all(r[6] is None for r in res)  # no device events on CPU
    # 20 envs, 8 steps from staggered phases of a 4-step episode: episodes end on every rank
    assert res[0][7] == res[1][7] and res[0][7] > 0 and res[0][8] == 20
