"""Data-parallel PPOAgent on the GPU: two ranks (gloo, both on cuda:0 - the pool's boxes
have one GPU; on a node the same code runs one rank per GPU over RCCL) with DIFFERENT local
batches must stay bitwise identical replicas: rank 0's initial weights are broadcast, the
flat gradient bucket is all-reduced between the captured backward and optimiser graphs, and
the plateau-scheduler inputs are averaged. Two update() calls, graphs on."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import importlib
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        ppo = importlib.import_module("diffusion-piano_amd.ppo")
        torch.manual_seed(100 + rank)  # different local init: the broadcast must fix it
        agent = ppo.PPOAgent(64, 45, batch_size=32, ppo_epochs=2, use_wandb=False,
                             checkpoint_dir=f"/tmp/ppo_dp_{rank}", graphs=True)
        init = agent.flat.param.detach().cpu().clone()
        rng = np.random.RandomState(rank)
        for _ in range(2):
            s = rng.rand(96, 64).astype(np.float32)
            a = rng.uniform(-1, 1, (96, 45)).astype(np.float32)
            lp = rng.uniform(-60, -40, 96).astype(np.float32)
            agent.update(s, a, rng.rand(96), lp, rng.rand(96, 64).astype(np.float32),
                         (rng.rand(96) < 0.1).astype(np.float32))
        torch.cuda.synchronize()
        q.put((rank, init.numpy(), agent.flat.param.detach().cpu().numpy(),
               float(agent.actor_optimizer.param_groups[0]["lr"])))
    finally:
        dist.destroy_process_group()


def test_two_rank_replicas_stay_identical():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(2)), key=lambda t: t[0])
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    (_, init0, fin0, lr0), (_, init1, fin1, lr1) = res
    np.testing.assert_array_equal(init0, init1)  # broadcast from rank 0
    np.testing.assert_array_equal(fin0, fin1)    # same averaged gradients, same steps
    assert lr0 == lr1
    assert np.abs(fin0 - init0).max() > 0        # it trained
