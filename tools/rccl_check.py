"""RCCL on the hardware (development aid): the job's collectives - the episode-return
all-gathers and the max-over-ranks all-reduce of bench.py / sharding.py, and a GradBucket-sized
SUM all-reduce as PPO's data-parallel step issues - over an nccl (RCCL) process group, checked
against the local values. Any world size; on the one-GPU pool it runs at world size 1 (RCCL
initialises, binds the device and runs every collective; the data movement is the identity).

usage: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
       --master-port P tools/rccl_check.py"""
import importlib
import json
import math
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
sh = importlib.import_module("diffusion-piano_amd.sharding")
from helpers import song  # noqa: E402

rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
torch.cuda.set_device(local)
dev = torch.device(f"cuda:{local}")
dist.init_process_group("nccl", device_id=dev)
try:
    total = 512 * world
    shard = sh.shard_envs(total, rank, world)
    env = dp.BatchedPianoEnv(shard.count, song(dp, "twinkle"), dp.TaskConfig(), device=dev, env_offset=shard.start)
    env.reset()
    er = sh.EpisodeReturns(shard.count, dev)
    gen = torch.Generator(device=dev).manual_seed(3 + rank)
    for _ in range(200):  # Twinkle: T = 161 control steps, so every env finishes an episode
        _, r, _, st = env.step(torch.rand(shard.count, env.action_dim, device=dev, generator=gen) * 2 - 1)
        er.update(r, st)
    fin_sum, fin_n, run_sum, n_all = er.gather()
    per_env = sh.gather_episode_returns(er, shard, total)
    mx = sh.max_over_ranks(float(rank + 1), device=dev)
    flat = torch.full((1 << 20,), float(rank + 1), device=dev)  # PPO GradBucket: SUM, then / world
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat.div_(world)
    torch.cuda.synchronize()
    mine = per_env[shard.start:shard.start + shard.count].cpu()
    ok = {
        "envs_gathered": n_all == total and per_env.numel() == total,
        "own_slice_matches": bool(torch.equal(torch.nan_to_num(mine, nan=-1.0),
                                              torch.nan_to_num(er.last_return.cpu(), nan=-1.0))),
        "every_env_finished": bool(torch.isfinite(per_env).all()),
        "episodes_counted": fin_n >= total,
        "max_over_ranks": mx == float(world),
        "grad_allreduce": bool(torch.allclose(flat, torch.full_like(flat, (world + 1) / 2.0))),
    }
    if rank == 0:
        print(json.dumps({"backend": dist.get_backend(), "world_size": world, "device": torch.cuda.get_device_name(dev),
                          "rccl_version": ".".join(map(str, torch.cuda.nccl.version())),
                          "finished_episodes": fin_n, "mean_finished_return": fin_sum / max(fin_n, 1),
                          "checks": ok, "all_ok": all(ok.values())}), flush=True)
    assert all(ok.values()), ok
    assert not math.isnan(fin_sum)
finally:
    dist.destroy_process_group()
