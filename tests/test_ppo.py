"""CPU tests of the on-device PPO counterpart of ppo_v2.py (no GPU calls):

* the CPU restatement (oracle/rl_ref.py) against tests/golden/ppo_v2.npz, which was made
  by running the reference's own PPOAgent (tests/golden/make_ppo_golden.py): GAE
  advantages, TD returns and the RunningMeanStd statistics;
* the networks: same state_dict keys and, under the same seed, the same initial weights
  as the reference's Actor / Critic;
* the DataLoader minibatch order reproduced by ``loader_permutation``;
* libpianorl.so loads and exports every symbol include/pianorl.h declares;
* the gradient bucket's all-reduce with world_size-2 gloo.
"""
import importlib
import os
import re
import socket
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden" / "ppo_v2.npz"


def ppo_mod():
    return importlib.import_module("diffusion-piano_amd.ppo")


def golden():
    return np.load(GOLD, allow_pickle=False)


def golden_batch(z, call):
    """Regenerate the update() inputs of golden call `call` (make_ppo_golden.batch)."""
    S, A, N = (int(x) for x in z["meta"][:3])
    rng = np.random.RandomState(int(z["meta"][-1]))
    for c in range(call + 1):
        s = rng.uniform(0, 1, (N, S)).astype(np.float32)
        ns = rng.uniform(0, 1, (N, S)).astype(np.float32)
        r = rng.uniform(0, 2, N).astype(np.float64)
        d = rng.uniform(0, 1, N) < 0.1
    assert s.astype(np.float64).sum() + ns.astype(np.float64).sum() == pytest.approx(float(z[f"u{call}/states_sum"]))
    assert np.array_equal(d, z[f"u{call}/dones"]) and np.allclose(r, z[f"u{call}/rewards"])
    return s, z[f"u{call}/actions"], r, z[f"u{call}/log_probs"], ns, d.astype(np.float32)


def sample_index(n):
    return np.linspace(0, n - 1, min(n, 64)).astype(np.int64)


def critic_state(critic):
    """The portable critic start state both the golden run and the tests load
    (make_ppo_golden.critic_state; the script only reads /root/reference inside main())."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_ppo_golden", ROOT / "tests" / "golden" / "make_ppo_golden.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.critic_state(critic)


def load_critic_state(critic):
    with torch.no_grad():
        for k, v in critic_state(critic).items():
            critic.state_dict()[k].copy_(v.to(critic.state_dict()[k].device))


def networks(seed=0):
    m = ppo_mod()
    torch.manual_seed(seed)
    actor = m.Actor(319, 45)
    critic = m.Critic(319)
    return actor, critic


def test_networks_match_reference_init():
    z = golden()
    actor, critic = networks(int(z["meta"][5]))
    params = {"actor." + k: v for k, v in actor.state_dict().items()}
    params.update({"critic." + k: v for k, v in critic.state_dict().items()})
    assert sorted(params) == list(z["param_names"])
    for k, v in params.items():
        flat = v.reshape(-1).numpy()
        if k.startswith("actor."):
            np.testing.assert_array_equal(flat[sample_index(flat.size)], z["init/" + k], err_msg=k)
        else:  # orthogonal init: LAPACK QR, last bits vary between host CPUs
            np.testing.assert_allclose(flat[sample_index(flat.size)], z["init/" + k], rtol=1e-3, atol=1e-8, err_msg=k)


def test_oracle_gae_and_normalizer_pinned_by_reference():
    rl = importlib.import_module("rl_ref")
    z = golden()
    _, critic = networks(int(z["meta"][5]))
    load_critic_state(critic)
    critic.eval()
    stats = (0.0, 1.0, 1e-4)
    for call in (0, 1):
        s, a, r, lp, ns, d = golden_batch(z, call)
        stats, rn = rl.running_norm(stats, r)
        np.testing.assert_allclose(stats, (z[f"u{call}/rn_mean"], z[f"u{call}/rn_var"], z[f"u{call}/rn_count"]),
                                   rtol=1e-12)
        if call == 0:  # values need the initial critic (call 1 runs after the reference's update)
            with torch.no_grad():
                v = critic(torch.from_numpy(s)).squeeze(-1).double().numpy()
                nv = critic(torch.from_numpy(ns)).squeeze(-1).double().numpy()
            adv, ret = rl.gae(rn.astype(np.float32), v, nv, d, 0.99, 0.95, returns_mode=0)
            np.testing.assert_allclose(ret, z["u0/returns"], atol=2e-6)
            np.testing.assert_allclose(rl.normalize(adv), z["u0/advantages"], atol=2e-5)


def test_oracle_gae_time_axis_equals_columns():
    rl = importlib.import_module("rl_ref")
    rng = np.random.RandomState(3)
    T, E = 17, 5
    r, v, nv = rng.randn(T, E), rng.randn(T, E), rng.randn(T, E)
    d = (rng.rand(T, E) < 0.2).astype(np.float64)
    adv, ret = rl.gae(r, v, nv, d, returns_mode=1)
    for e in range(E):
        a1, r1 = rl.gae(r[:, e], v[:, e], nv[:, e], d[:, e], returns_mode=1)
        np.testing.assert_allclose(adv[:, e], a1)
        np.testing.assert_allclose(ret[:, e], a1 + v[:, e])


def test_loader_permutation_matches_dataloader():
    from torch.utils.data import DataLoader, TensorDataset
    m = ppo_mod()
    for n, bs in ((96, 32), (10, 4), (4096, 128)):
        torch.manual_seed(11)
        ds = TensorDataset(torch.arange(n))
        want = [torch.cat([b[0] for b in DataLoader(ds, batch_size=bs, shuffle=True)]) for _ in range(3)]
        tail = torch.rand(1)
        torch.manual_seed(11)
        got = [m.loader_permutation(n) for _ in range(3)]
        for w, g in zip(want, got):
            assert torch.equal(w, g)
        assert torch.equal(tail, torch.rand(1))  # same number of generator draws


def test_rl_library_exports_header_symbols():
    lib = importlib.import_module("diffusion-piano_amd._lib")
    L = lib.load_rl()
    header = (ROOT / "include" / "pianorl.h").read_text()
    declared = set(re.findall(r"\b(prl_[a-z_]+)\s*\(", header))
    assert declared == set(lib.RL_EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    assert L.prl_version() >= 1
    # argument validation happens before any device call
    assert L.prl_gae(None, None, None, None, None, None, 4, 1, 0.99, 0.95, 0, None) < 0
    assert b"null" in L.prl_last_error()
    assert L.prl_gauss_sample(1, 1, 4, 65, 0, 0, 1, 1, None) < 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = ppo_mod()
        torch.manual_seed(0)  # same replica on both ranks
        net = torch.nn.Sequential(torch.nn.Linear(5, 3), torch.nn.ReLU(), torch.nn.Linear(3, 2))
        b = m.GradBucket(list(net.parameters()))
        x = torch.full((4, 5), float(rank + 1))
        net(x).pow(2).sum().backward()  # accumulates into the bucket views
        local = b.flat.clone()
        b.allreduce_()
        views_ok = all(p.grad.data_ptr() >= b.flat.data_ptr() for p in net.parameters())
        q.put((rank, local.numpy(), b.flat.numpy(), views_ok))
    finally:
        dist.destroy_process_group()


def _guard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = ppo_mod()
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(5, 3), torch.nn.ReLU(), torch.nn.Linear(3, 2))
        b = m.GradBucket(list(net.parameters()))
        b.guard = torch.tensor([3 if rank == 1 else 0], dtype=torch.int32)
        net(torch.full((4, 5), float(rank + 1))).pow(2).sum().backward()
        b.allreduce_()
        first = int(b.guard.item())
        b.guard.zero_()
        b.allreduce_()  # a clean step after the reset: no rank flagged
        q.put((rank, first, int(b.guard.item())))
    finally:
        dist.destroy_process_group()


def test_grad_bucket_carries_the_guard_word_gloo_world2():
    """The guard word (include/pianorl.h: a failed split-kernel step) rides the gradient
    all-reduce, so one rank's failure stops every rank's optimiser step: rank 1 flags 3, both
    ranks come out flagged (rank 1 keeps its code); after clearing, nothing is flagged."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted((q.get(timeout=5) for _ in range(2)), key=lambda t: t[0])
    assert res == [(0, 1, 0), (1, 3, 0)]


def test_grad_bucket_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted((q.get(timeout=5) for _ in range(2)), key=lambda t: t[0])
    mean = (res[0][1] + res[1][1]) / 2
    for _, _, red, views_ok in res:
        assert views_ok
        np.testing.assert_allclose(red, mean, rtol=1e-6)
