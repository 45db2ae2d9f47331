"""BASELINE.json config 5: the full PPO loop (ppo_v2.py driven as parallelized_base_v2.py
does) on the batched environment - rollout + GAE + MLP policy update - in env-steps/s.

Two loops (diffusion-piano_amd/ppo.py RolloutTrainer):

* ``--mode reference``: the reference driver's schedule (parallelized_base_v2.py:116-166):
  after EVERY env step, ``agent.update`` on that step's N transitions - reward
  normalisation, batch-axis GAE, ``--epochs`` epochs of minibatches of ``--batch``.
* ``--mode rollout``: ``--horizon`` env steps into time-major HBM buffers, then one update
  with time-axis GAE over [horizon, N].

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node G tools/ppo_bench.py ...``;
each rank owns ``--envs`` envs (weak scaling) and one replica of the networks; the
gradient bucket is all-reduced over RCCL once per minibatch. ``--eager`` disables the HIP
graph of the minibatch step (the same math launched op by op, as the reference does).

Prints one JSON line on rank 0 with the phase split (env step, action sampling, update).
"""

from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    p.add_argument("--song", default="twinkle", choices=["twinkle", "crossing_field", "guren"])
    p.add_argument("--mode", default="reference", choices=["reference", "rollout"])
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--horizon", type=int, default=16)
    p.add_argument("--eager", action="store_true")
    p.add_argument("--blas", default="default", choices=["default", "rocblas", "hipblaslt"])
    p.add_argument("--no-tune", action="store_true", help="no TunableOp GEMM selection")
    p.add_argument("--autograd", action="store_true", help="torch autograd minibatch step instead of FusedStep")
    p.add_argument("--hand", default="hull", choices=["hull", "primitive", "authored"],
                   help="collider set (bench.py HANDS; default: the reference's default colliders)")
    args = p.parse_args()

    import torch
    if args.blas != "default":
        torch.backends.cuda.preferred_blas_library("cublas" if args.blas == "rocblas" else "cublaslt")
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)  # the device first, then the process group bound to it
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        dist.init_process_group(os.environ.get("PIANOSIM_DIST_BACKEND", "nccl"), device_id=dev)
    dp = importlib.import_module("diffusion-piano_amd")
    ppo = importlib.import_module("diffusion-piano_amd.ppo")
    sharding = importlib.import_module("diffusion-piano_amd.sharding")
    import dataclasses

    from bench import HANDS, load_song

    seq, task = load_song(dp, args.song)
    task = dataclasses.replace(task, primitive_fingertip_collisions=HANDS[args.hand][0])
    shard = sharding.shard_envs(args.envs * world, rank, world)
    env = dp.BatchedPianoEnv(shard.count, seq, task, device=dev, seed=12345,
                             env_offset=shard.start)
    torch.manual_seed(0)
    agent = ppo.PPOAgent(env.obs_dim, env.action_dim, lr=1e-4, gamma=0.99, epsilon=0.2, batch_size=args.batch,
                         ppo_epochs=args.epochs, checkpoint_dir="/tmp/ppo_bench_ckpt", use_wandb=False,
                         graphs=not args.eager, sample_seed=1000 + rank, tune_gemms=not args.no_tune,
                         fused=not args.autograd)
    tr = ppo.RolloutTrainer(env, agent, horizon=args.horizon, reference_semantics=args.mode == "reference")
    for _ in range(args.warmup):
        tr.iterate()
    # phase timing with events on the launch stream (everything runs on the current stream)
    ev = {k: [] for k in ("total",)}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 0
    upd = 0.0
    for _ in range(args.iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        steps += tr.iterate()
        e.record()
        ev["total"].append((s, e))
        upd += agent.timing.get("update_s", 0.0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = sharding.max_over_ranks(time.perf_counter() - t0, device=dev)
    # env-only and sampling-only timing of the same shapes (separate short runs)
    obs = env.obs.clone()
    torch.cuda.synchronize()
    te = time.perf_counter()
    for _ in range(10):
        a, _ = agent.select_actions(obs)
    torch.cuda.synchronize()
    t_sel = (time.perf_counter() - te) / 10
    te = time.perf_counter()
    for _ in range(10):
        env.step(a)
    torch.cuda.synchronize()
    t_env = (time.perf_counter() - te) / 10
    total = steps * world
    if rank == 0:
        nmb = -(-(args.envs if args.mode == "reference" else args.envs * args.horizon) // args.batch)
        line = {
            "metric": "PPO loop env-steps/s (rollout + GAE + policy update)",
            "value": total / elapsed, "unit": "env-steps/s", "n_gpus": world, "iters": args.iters,
            "warmup": args.warmup, "ms_per_iter": elapsed / args.iters * 1e3, "higher_is_better": True,
            "scaling": "weak", "dtype": "f32", "data": "synthetic: env rollouts of the policy, random init",
            "config": {"workload": f"ppo_v2 {args.mode} loop, {args.envs} envs/GPU {args.song}",
                       "hand": f"{args.hand}: {HANDS[args.hand][2]}",
                       "mode": args.mode, "envs_per_gpu": args.envs, "batch": args.batch, "epochs": args.epochs,
                       "horizon": args.horizon if args.mode == "rollout" else 1,
                       "minibatch_steps_per_update": nmb * args.epochs, "graphs": not args.eager,
                       "blas": args.blas, "tunableop": not args.no_tune, "fused_step": not args.autograd,
                       "parallelism": f"dp{world}"},
            "phases_ms": {"env_step": t_env * 1e3, "select_actions": t_sel * 1e3,
                          "update_host_wall": upd / args.iters * 1e3},
            "minibatch_step_ms": upd / args.iters * 1e3 / max(1, nmb * args.epochs),
        }
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
