"""GPU parity of the on-device PPO path (libpianorl.so + diffusion-piano_amd/ppo.py).

* prl_gae / prl_running_norm / prl_normalize / prl_gauss_sample against the CPU
  restatement (oracle/rl_ref.py) on seeded inputs, every launch shape the wrapper picks
  (column kernel, chunked-scan kernel, T = 1, the reference's E = 1 / T = batch case).
  Tolerances: GAE 2e-5 relative to the largest |advantage| (fp32 scan vs fp64 loop, the
  chunked scan reassociates the recursion), statistics 1e-12 relative (fp64 on both sides),
  log-probs 1e-5 relative.
* PPOAgent.update against tests/golden/ppo_v2.npz, the reference's own agent run on CPU:
  per-minibatch losses / entropy / value / return / advantage means, the normaliser
  statistics and sampled weights after two update() calls (first call: two eager
  warm-up minibatches, then the HIP-graph replay; second call: all graph replays).
  Tolerance: 2e-4 relative on the logged scalars (5e-4 absolute on the actor loss, whose
  importance ratio exponentiates log-prob differences; fp32
  GPU GEMMs vs fp32 CPU GEMMs), parameter deltas within 2% of each tensor's largest delta.
"""
import importlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from test_ppo import golden, golden_batch, load_critic_state, sample_index  # noqa: E402


@pytest.fixture(scope="module")
def ppo():
    return importlib.import_module("diffusion-piano_amd.ppo")


@pytest.fixture(scope="module")
def rl():
    return importlib.import_module("rl_ref")


def dev(x):
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float32, device="cuda:0")


@pytest.mark.parametrize("T,E", [(96, 1), (4096, 1), (1000, 3), (166, 4096), (7, 5), (1, 9), (300, 300), (257, 2)])
@pytest.mark.parametrize("mode", [0, 1])
def test_gae_matches_restatement(ppo, rl, T, E, mode):
    rng = np.random.RandomState(T * 31 + E)
    r, v, nv = rng.randn(T, E), rng.randn(T, E), rng.randn(T, E)
    d = (rng.rand(T, E) < 0.05).astype(np.float64)
    adv, ret = ppo.gae(dev(r), dev(v), dev(nv), dev(d), 0.99, 0.95, returns_mode=mode)
    a_ref, r_ref = rl.gae(r.astype(np.float32), v.astype(np.float32), nv.astype(np.float32), d, 0.99, 0.95, mode)
    scale = max(1.0, np.abs(a_ref).max())
    np.testing.assert_allclose(adv.cpu().numpy(), a_ref, atol=2e-5 * scale, rtol=0)
    np.testing.assert_allclose(ret.cpu().numpy(), r_ref, atol=2e-5 * scale, rtol=0)


@pytest.mark.parametrize("n", [1, 96, 4096, 680000])
def test_running_norm_and_normalize(ppo, rl, n):
    rng = np.random.RandomState(n)
    rms = ppo.RunningMeanStd(device="cuda:0")
    stats = (0.0, 1.0, 1e-4)
    for k in range(3):
        x = (rng.randn(n) * (k + 1) + k).astype(np.float32)
        out = rms(dev(x))
        stats, want = rl.running_norm(stats, x)
        np.testing.assert_allclose(rms.stats.cpu().numpy(), stats, rtol=1e-12)
        np.testing.assert_allclose(out.cpu().numpy(), want, rtol=1e-5, atol=1e-6)
    if n > 1:
        x = (rng.randn(n) * 3 + 1).astype(np.float32)
        y = ppo.normalize_(dev(x))
        np.testing.assert_allclose(y.cpu().numpy(), rl.normalize(x), rtol=1e-5, atol=1e-5)


def test_gauss_sample(ppo, rl):
    n, a = 20000, 45
    rng = np.random.RandomState(5)
    mean = dev(rng.uniform(-1, 1, (n, a)))
    log_std = dev(np.linspace(-2.0, 0.5, a))
    act, lp = ppo.gauss_sample(mean, log_std, seed=1234, offset=7)
    act2, lp2 = ppo.gauss_sample(mean, log_std, seed=1234, offset=7)
    act3, _ = ppo.gauss_sample(mean, log_std, seed=1234, offset=8)
    assert torch.equal(act, act2) and torch.equal(lp, lp2)  # counter-based: reproducible
    assert not torch.equal(act, act3)
    want = rl.gauss_logp(mean.cpu().numpy(), log_std.cpu().numpy(), act.cpu().numpy())
    np.testing.assert_allclose(lp.cpu().numpy(), want, rtol=1e-5, atol=1e-4)
    z = ((act - mean) / torch.exp(log_std)).cpu().numpy().astype(np.float64)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 0.03  # lanes are independent streams
    # torch's Normal.log_prob on the same actions
    d = torch.distributions.Normal(mean, torch.exp(torch.clamp(log_std, -20, 2)))
    torch.testing.assert_close(lp, d.log_prob(act).sum(1), rtol=1e-5, atol=1e-4)


def _agent(ppo, z, tmp_path, graphs=True):
    torch.manual_seed(int(z["meta"][5]))
    S, A, N, B, EP = (int(x) for x in z["meta"][:5])
    agent = ppo.PPOAgent(S, A, lr=1e-4, gamma=0.99, epsilon=0.2, batch_size=B, ppo_epochs=EP, device="cuda",
                         checkpoint_dir=str(tmp_path), use_wandb=False, graphs=graphs)
    agent.critic.eval()  # dropout off, as the golden run (make_ppo_golden.py)
    load_critic_state(agent.critic)  # the golden run's portable critic start state
    return agent


def _params(agent):
    p = {"actor." + k: v for k, v in agent.actor.state_dict().items()}
    p.update({"critic." + k: v for k, v in agent.critic.state_dict().items()})
    return p


@pytest.mark.parametrize("graphs", [True, False])
def test_update_matches_reference_agent(ppo, tmp_path, graphs):
    z = golden()
    agent = _agent(ppo, z, tmp_path, graphs)
    for k, v in _params(agent).items():
        if k.startswith("actor."):
            flat = v.reshape(-1).cpu().numpy()
            np.testing.assert_array_equal(flat[sample_index(flat.size)], z["init/" + k], err_msg=k)
    for call, seed in enumerate(int(x) for x in z["meta"][6:8]):
        s, a, r, lp, ns, d = golden_batch(z, call)
        torch.manual_seed(seed)
        agent.update(s, a, r, lp, ns, d)
        log = agent.last_update_log.cpu().numpy()
        want = z[f"u{call}/log"]
        assert log.shape == want.shape
        # actor loss: mean of min(ratio * A, clip(ratio) * A), ratio = exp(new - old log-prob)
        # over 45 dims - the most rounding-sensitive scalar, 5e-4 absolute (values ~0.1-0.5)
        np.testing.assert_allclose(log[:, 0], want[:, 0], rtol=0, atol=5e-4, err_msg=f"update {call} actor loss")
        np.testing.assert_allclose(log[:, 1:], want[:, 1:], rtol=2e-4, atol=2e-5, err_msg=f"update {call} log")
        np.testing.assert_allclose(agent.reward_normalizer.stats.cpu().numpy(),
                                   [z[f"u{call}/rn_mean"], z[f"u{call}/rn_var"], z[f"u{call}/rn_count"]], rtol=1e-7)
        assert float(agent.actor_optimizer.param_groups[0]["lr"]) == pytest.approx(float(z[f"u{call}/actor_lr"]))
    # parameter deltas of the 12 Adam steps: Adam normalises each gradient element, so an
    # element whose gradient is near zero moves by a rounding-dependent amount; bound the
    # delta error by 2% of the tensor's largest delta
    init = {k: v.reshape(-1).cpu().numpy() for k, v in _params(_agent(ppo, z, tmp_path, graphs)).items()}
    for k, v in _params(agent).items():
        idx = sample_index(init[k].size)
        d_ours = v.reshape(-1).cpu().numpy()[idx] - init[k][idx]
        d_ref = z["final/" + k] - init[k][idx]
        assert np.abs(d_ours - d_ref).max() <= 0.02 * np.abs(d_ref).max() + 1e-7, k


def test_select_actions_numpy_and_tensor(ppo, tmp_path):
    z = golden()
    agent = _agent(ppo, z, tmp_path)
    s, *_ = golden_batch(z, 0)
    a_np, lp_np = agent.select_actions(s)
    assert isinstance(a_np, np.ndarray) and a_np.shape == (s.shape[0], 45) and lp_np.shape == (s.shape[0],)
    a_t, lp_t = agent.select_actions(dev(s))
    assert a_t.is_cuda and lp_t.is_cuda
    with torch.no_grad():
        want = agent.actor(dev(s)).log_prob(a_t).sum(1)
    torch.testing.assert_close(lp_t, want, rtol=1e-5, atol=1e-4)


def test_checkpoint_round_trip(ppo, tmp_path):
    z = golden()
    a1 = _agent(ppo, z, tmp_path)
    s, a, r, lp, ns, d = golden_batch(z, 0)
    torch.manual_seed(1)
    a1.update(s, a, r, lp, ns, d)
    path = a1.save_checkpoint(5, {"episode_rewards": [[1.0]], "mean_rewards": [1.0]})
    a2 = _agent(ppo, z, tmp_path)
    a2.load_checkpoint(path)
    for (k, v), (_, w) in zip(_params(a1).items(), _params(a2).items()):
        assert torch.equal(v, w), k
    assert torch.equal(a1.reward_normalizer.stats, a2.reward_normalizer.stats)
    s, a, r, lp, ns, d = golden_batch(z, 1)
    for ag in (a1, a2):
        torch.manual_seed(2)
        ag.update(s, a, r, lp, ns, d)
    for (k, v), (_, w) in zip(_params(a1).items(), _params(a2).items()):
        torch.testing.assert_close(v, w, rtol=0, atol=1e-6, msg=k)


@pytest.mark.parametrize("reference_semantics", [True, False])
def test_rollout_trainer_on_env(ppo, reference_semantics, tmp_path):
    dp = importlib.import_module("diffusion-piano_amd")
    env = dp.BatchedPianoEnv(64, dp.music.twinkle_twinkle_little_star_one_hand(), dp.TaskConfig(), device="cuda:0")
    torch.manual_seed(0)
    agent = ppo.PPOAgent(env.obs_dim, 45, batch_size=128, ppo_epochs=2, checkpoint_dir=str(tmp_path), use_wandb=False)
    tr = ppo.RolloutTrainer(env, agent, horizon=4, reference_semantics=reference_semantics)
    steps = sum(tr.iterate() for _ in range(3))
    assert steps == 64 * (3 if reference_semantics else 12)
    log = agent.last_update_log
    assert torch.isfinite(log).all()
    assert torch.isfinite(tr.ep_return).all()
    env.close()


@pytest.mark.parametrize("reference_semantics", [True, False])
def test_rollout_trainer_reduced_action_space(ppo, reference_semantics, tmp_path):
    """The loop on a model whose action row is not 45 wide: reduced_action_space
    gives 2 x 19 actuators + sustain = 39 columns (shadow_hand_test.py:89-99); the agent and the
    trainer's action buffer take env.action_dim."""
    dp = importlib.import_module("diffusion-piano_amd")
    env = dp.BatchedPianoEnv(64, dp.music.twinkle_twinkle_little_star_one_hand(),
                             dp.TaskConfig(reduced_action_space=True), device="cuda:0")
    assert env.action_dim == 39
    torch.manual_seed(0)
    agent = ppo.PPOAgent(env.obs_dim, env.action_dim, batch_size=128, ppo_epochs=2, checkpoint_dir=str(tmp_path),
                         use_wandb=False)
    tr = ppo.RolloutTrainer(env, agent, horizon=4, reference_semantics=reference_semantics)
    assert tr.act.shape[-1] == 39
    steps = sum(tr.iterate() for _ in range(2))
    assert steps == 64 * (2 if reference_semantics else 8)
    assert torch.isfinite(agent.last_update_log).all()
    assert torch.isfinite(tr.ep_return).all()
    env.close()


def _fused_agent(ppo, z, tmp_path, mfma, train_critic, batch):
    ag = _agent(ppo, z, tmp_path, graphs=False)
    ag.fused = True
    if train_critic:
        ag.critic.train()
    ag._prepare(*batch)
    ag._fused = ppo.FusedStep(ag)
    ag._fused.mfma = mfma  # False: the hipBLASLt GEMMs + prl_lnrelu / head kernels (B > 512 path)
    return ag


@pytest.mark.parametrize("mfma", [True, False])
@pytest.mark.parametrize("train_critic", [False, True])
def test_fused_step_matches_autograd(ppo, tmp_path, train_critic, mfma):
    """FusedStep against the torch autograd step on the same weights and minibatch: logged
    losses and every gradient, for both FusedStep paths (mfma: the one-kernel prl_mlp_step;
    not: hipBLASLt GEMMs with libpianorl kernels between them). With the critic in train mode
    dropout is active on both sides with different masks, so there only the actor side (no
    dropout) is compared (test_fused_paths_agree_with_dropout compares the two fused paths)."""
    z = golden()
    batch = golden_batch(z, 0)
    agents = [_fused_agent(ppo, z, tmp_path, mfma, train_critic, batch)]
    ag = _agent(ppo, z, tmp_path, graphs=False)
    ag.fused = False
    if train_critic:
        ag.critic.train()
    ag._prepare(*batch)
    agents.append(ag)
    idx = torch.randperm(96, generator=torch.Generator().manual_seed(3))[:32].cuda()
    rows = []
    for ag in agents:
        ag._forward_backward(idx, ag._log_row)
        torch.cuda.synchronize()
        rows.append(ag._log_row.cpu().numpy().copy())
    cols = [0, 2, 4, 5] if train_critic else list(range(6))
    np.testing.assert_allclose(rows[0][cols], rows[1][cols], rtol=2e-5, atol=2e-6)
    nets = ("actor",) if train_critic else ("actor", "critic")
    for net in nets:
        for (k, p0), (_, p1) in zip(getattr(agents[0], net).named_parameters(), getattr(agents[1], net).named_parameters()):
            g0, g1 = p0.grad.cpu().numpy(), p1.grad.cpu().numpy()
            scale = max(np.abs(g1).max(), 1e-6)
            np.testing.assert_allclose(g0, g1, rtol=0, atol=2e-4 * scale, err_msg=f"{net}.{k}")


def test_fused_paths_agree_with_dropout(ppo, tmp_path):
    """The two FusedStep paths with the critic in train mode (dropout active): the matrix-core
    kernel's dropout masks are prl_lnrelu_fwd's (same Philox keys: seed, minibatch counter,
    layer, row, column), so the logged losses and every gradient agree tightly."""
    z = golden()
    batch = golden_batch(z, 0)
    agents = [_fused_agent(ppo, z, tmp_path, m, True, batch) for m in (True, False)]
    idx = torch.randperm(96, generator=torch.Generator().manual_seed(5))[:32].cuda()
    rows = []
    for ag in agents:
        ag._forward_backward(idx, ag._log_row)
        torch.cuda.synchronize()
        rows.append(ag._log_row.cpu().numpy().copy())
    np.testing.assert_allclose(rows[0], rows[1], rtol=2e-5, atol=2e-6)
    for net in ("actor", "critic"):
        for (k, p0), (_, p1) in zip(getattr(agents[0], net).named_parameters(), getattr(agents[1], net).named_parameters()):
            g0, g1 = p0.grad.cpu().numpy(), p1.grad.cpu().numpy()
            np.testing.assert_allclose(g0, g1, rtol=0, atol=2e-4 * max(np.abs(g1).max(), 1e-6), err_msg=f"{net}.{k}")


@pytest.mark.parametrize("mfma", [True, False])
def test_fused_step_large_minibatch(ppo, tmp_path, mfma):
    """B = 512 rows against autograd, on both FusedStep paths: the matrix-core kernel at its
    row limit, and the hipBLASLt path whose column sums run in 128-row chunks (partials +
    ordered final sum)."""
    rng = np.random.RandomState(9)
    n, S = 1024, 64
    s = rng.rand(n, S).astype(np.float32)
    a = rng.uniform(-1, 1, (n, 45)).astype(np.float32)
    lp = rng.uniform(-60, -40, n).astype(np.float32)
    r, d = rng.rand(n), (rng.rand(n) < 0.1).astype(np.float32)
    ns = rng.rand(n, S).astype(np.float32)
    agents = []
    for fused in (True, False):
        torch.manual_seed(0)
        ag = ppo.PPOAgent(S, 45, batch_size=512, ppo_epochs=1, use_wandb=False, checkpoint_dir=str(tmp_path),
                          graphs=False, fused=fused)
        ag.critic.eval()
        ag._prepare(s, a, r, lp, ns, d)
        if fused:
            ag._fused = ppo.FusedStep(ag)
            ag._fused.mfma = mfma
        agents.append(ag)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(1))[:512].cuda()
    for ag in agents:
        ag._forward_backward(idx, ag._log_row)
    torch.cuda.synchronize()
    np.testing.assert_allclose(agents[0]._log_row.cpu().numpy(), agents[1]._log_row.cpu().numpy(), rtol=2e-5, atol=2e-6)
    for net in ("actor", "critic"):
        for (k, p0), (_, p1) in zip(getattr(agents[0], net).named_parameters(), getattr(agents[1], net).named_parameters()):
            g0, g1 = p0.grad.cpu().numpy(), p1.grad.cpu().numpy()
            np.testing.assert_allclose(g0, g1, rtol=0, atol=2e-4 * max(np.abs(g1).max(), 1e-6), err_msg=f"{net}.{k}")


def _split_agent(ppo, tmp_path, S, B, train_critic):
    rng = np.random.RandomState(11)
    n = 2 * B
    args = (rng.rand(n, S).astype(np.float32), rng.uniform(-1, 1, (n, 45)).astype(np.float32), rng.rand(n),
            rng.uniform(-60, -40, n).astype(np.float32), rng.rand(n, S).astype(np.float32),
            (rng.rand(n) < 0.1).astype(np.float32))
    torch.manual_seed(0)
    ag = ppo.PPOAgent(S, 45, batch_size=B, ppo_epochs=1, use_wandb=False, checkpoint_dir=str(tmp_path), graphs=False,
                      fused=True)
    ag.critic.train() if train_critic else ag.critic.eval()
    ag._prepare(*args)
    ag._fused = ppo.FusedStep(ag)
    return ag, torch.randperm(n, generator=torch.Generator().manual_seed(2))[:B].cuda()


def _grads(ag):
    return {f"{net}.{k}": p.grad.detach().cpu().numpy().copy()
            for net in ("actor", "critic") for k, p in getattr(ag, net).named_parameters()}


@pytest.mark.parametrize("B,train_critic", [(128, False), (128, True), (40, True), (256, False)])
def test_split_rows_kernel_matches_tile_kernel(ppo, tmp_path, monkeypatch, B, train_critic):
    """The column-split rows kernel (4 workgroups per 16-row tile and network, six exchanges per
    step; csrc/mlp_split.inc) against the one-workgroup-per-tile kernel (PIANORL_MLP_SPLIT=0) on
    the same weights, minibatch and dropout masks: the GEMMs run in the same k order, only the
    LayerNorm row sums and column sums are added in another order, so the logged sums agree to
    1e-5 relative and every gradient to 1e-4 of its tensor's largest entry (measured: <= 5.5e-5,
    a LayerNorm beta gradient summed over 256 rows with cancellation). The state width 329
    is the piano observation's (unaligned weight rows), B = 40 a ragged last tile, B = 256 the
    split's row limit (128 workgroups). Three split steps in a row are bitwise equal (the
    monotonic exchange counters carry over calls) and the error word stays 0."""
    ag, idx = _split_agent(ppo, tmp_path, 329, B, train_critic)
    out = {}
    for mode in ("0", "1", "1", "1"):
        monkeypatch.setenv("PIANORL_MLP_SPLIT", mode)
        step0 = ag._fused.step.clone()
        ag._forward_backward(idx, ag._log_row)
        torch.cuda.synchronize()
        ag._fused.step.copy_(step0)  # the same dropout draw for every run
        out.setdefault(mode, []).append((ag._log_row.cpu().numpy().copy(), _grads(ag)))
    assert ag._fused.mlp_error(B) == 0
    (row0, g0), = out["0"]
    for row1, g1 in out["1"][1:]:
        np.testing.assert_array_equal(row1, out["1"][0][0])
        for k in g1:
            np.testing.assert_array_equal(g1[k], out["1"][0][1][k], err_msg=k)
    row1, g1 = out["1"][0]
    np.testing.assert_allclose(row1, row0, rtol=1e-5, atol=1e-7)
    for k in g0:
        np.testing.assert_allclose(g1[k], g0[k], rtol=0, atol=1e-4 * max(np.abs(g0[k]).max(), 1e-6), err_msg=k)


@pytest.mark.parametrize("graphs", [False, True])
def test_split_exchange_timeout_raises_and_applies_nothing(ppo, tmp_path, monkeypatch, graphs):
    """A timed-out exchange of the column-split rows kernel can no longer reach the weights
    (ADVICE r5): with the test hook PIANORL_SPLIT_TEST_FAULT=1 member 1 of
    every group never publishes exchange 0, so the other members' bounded waits (shortened to
    10 ms by PIANORL_SPLIT_SPIN_TICKS) time out and write the guard word. Then the gradient
    kernel does not advance the Adam step counts, clip+Adam applies nothing (parameters, moments,
    step counts bitwise unchanged over the whole update: every minibatch step fails here), and
    update() raises PianosimError. The guard and the exchange region are re-zeroed, so the next
    update (hook off) runs and changes the weights."""
    lib = importlib.import_module("diffusion-piano_amd._lib")
    rng = np.random.RandomState(5)
    n, S, B = 512, 329, 128
    args = (rng.rand(n, S).astype(np.float32), rng.uniform(-1, 1, (n, 45)).astype(np.float32), rng.rand(n),
            rng.uniform(-60, -40, n).astype(np.float32), rng.rand(n, S).astype(np.float32),
            (rng.rand(n) < 0.1).astype(np.float32))
    torch.manual_seed(0)
    ag = ppo.PPOAgent(S, 45, batch_size=B, ppo_epochs=2, use_wandb=False, checkpoint_dir=str(tmp_path),
                      graphs=graphs, fused=True)
    fl = ag.flat
    before = [t.detach().clone() for t in (fl.param, fl.exp_avg, fl.exp_avg_sq, fl.step_count)]
    monkeypatch.setenv("PIANORL_SPLIT_SPIN_TICKS", "1000000")
    monkeypatch.setenv("PIANORL_SPLIT_TEST_FAULT", "1")
    with pytest.raises(lib.PianosimError, match="timed out"):
        ag.update(*args)
    torch.cuda.synchronize()
    for a, b in zip(before, (fl.param, fl.exp_avg, fl.exp_avg_sq, fl.step_count)):
        assert torch.equal(a, b)
    assert int(ag._guard.item()) == 0
    monkeypatch.delenv("PIANORL_SPLIT_TEST_FAULT")
    ag._graph = ag._chunk_graph = None  # (a captured graph keeps the hook's launch arguments)
    ag._graph_eager_left = 2
    ag.update(*args)
    torch.cuda.synchronize()
    assert int(ag._guard.item()) == 0
    assert not torch.equal(before[0], fl.param)
    assert torch.isfinite(fl.param).all()


def test_rollout_trainer_masks_auto_reset_steps(ppo, tmp_path):
    """An auto-reset step (FIRST: the kernel ignored the action and reset the env) is not a
    transition: the horizon rollout marks it invalid and _prepare drops it after GAE (it enters
    neither the advantage normalisation nor a minibatch); the LAST step before it does not
    bootstrap (done = 1). The reference-semantics loop skips an all-FIRST step's update, as
    the reference (which resets after all(dones)) never trains on one."""
    dp = importlib.import_module("diffusion-piano_amd")
    N = 16
    env = dp.BatchedPianoEnv(N, dp.music.test_midi(0.05), dp.TaskConfig(), device="cuda:0")
    assert env.song.T == 4
    torch.manual_seed(0)
    agent = ppo.PPOAgent(env.obs_dim, 45, batch_size=16, ppo_epochs=1, checkpoint_dir=str(tmp_path), use_wandb=False)
    tr = ppo.RolloutTrainer(env, agent, horizon=8)
    tr.iterate()
    valid, done = tr.valid.cpu().numpy(), tr.done.cpu().numpy()
    assert (valid[4] == 0).all() and valid.sum() == 7 * N  # steps 0-3 episode 1, 4 FIRST, 5-7 episode 2
    assert (done[3] == 1).all() and done.sum() == N
    r, n = agent._prepare(tr.obs, tr.act, tr.rew, tr.logp, tr._cur.unsqueeze(0), tr.done, tr.valid)
    assert n == 7 * N
    kept = torch.cat([tr.obs[:4], tr.obs[5:]]).reshape(7 * N, -1)
    assert torch.equal(agent._S[:n], kept)
    # GAE at the boundary: the LAST step's advantage is its own TD error (no bootstrap)
    with torch.no_grad():
        v = agent.critic(tr.obs.reshape(8 * N, -1)).reshape(8, N)
        nv = agent.critic(tr._cur).reshape(1, N).expand(8, N).contiguous()
    rn = r.reshape(8, N)
    adv, ret = ppo.gae(rn, v, nv, tr.done, agent.gamma, agent.gae_lambda, returns_mode=1)
    torch.testing.assert_close(adv[3], rn[3] - v[3], rtol=1e-5, atol=1e-5)
    # reference semantics: 4 steps of one episode, then an all-FIRST step with no update
    calls = []
    agent2 = ppo.PPOAgent(env.obs_dim, 45, batch_size=16, ppo_epochs=1, checkpoint_dir=str(tmp_path), use_wandb=False)
    orig = agent2.update
    agent2.update = lambda *a, **k: (calls.append(k.get("valid") is None), orig(*a, **k))
    tr2 = ppo.RolloutTrainer(env, agent2, horizon=1, reference_semantics=True)
    for _ in range(5):
        tr2.iterate()
    assert calls == [True] * 4
    env.close()


def test_chunked_graph_update_equals_eager(ppo, tmp_path):
    """update() with graphs replays CHUNK full-size minibatch steps per graph once the
    single-step graph exists (20 minibatches: 2 eager warm-ups, 1 single-step capture, then
    chunks of 8, and single replays / the short tail eagerly). The same launches in the same
    order as the eager fused step: logs and parameters bitwise equal (critic in eval mode)."""
    rng = np.random.RandomState(11)
    n, S, B = 20 * 16 - 5, 64, 16  # 19 full minibatches + a 11-row tail per epoch
    s = rng.rand(n, S).astype(np.float32)
    a = rng.uniform(-1, 1, (n, 45)).astype(np.float32)
    lp = rng.uniform(-60, -40, n).astype(np.float32)
    r, d = rng.rand(n), (rng.rand(n) < 0.1).astype(np.float32)
    ns = rng.rand(n, S).astype(np.float32)
    agents = []
    for graphs in (True, False):
        torch.manual_seed(0)
        ag = ppo.PPOAgent(S, 45, batch_size=B, ppo_epochs=2, use_wandb=False, checkpoint_dir=str(tmp_path),
                          graphs=graphs)
        ag.critic.eval()
        for call in range(2):
            torch.manual_seed(100 + call)
            ag.update(s, a, r, lp, ns, d)
        agents.append(ag)
    assert agents[0]._chunk_graph is not None  # the chunk path ran
    np.testing.assert_array_equal(agents[0].last_update_log.cpu().numpy(), agents[1].last_update_log.cpu().numpy())
    for (k, p0), (_, p1) in zip(_params(agents[0]).items(), _params(agents[1]).items()):
        np.testing.assert_array_equal(p0.cpu().numpy(), p1.cpu().numpy(), err_msg=k)


def test_fused_norm_partials_equal_norm_pass(ppo, tmp_path, monkeypatch):
    """clip_grad_norm_ from the gradient kernel's per-workgroup partials (one clip+Adam launch,
    the default) against the separate grad_sumsq pass (PIANORL_SUMSQ=1): the same f64 norm up to
    summation order, so parameters and logs agree to fp32 rounding after two update() calls."""
    rng = np.random.RandomState(12)
    n, S, B = 200, 64, 32
    s = rng.rand(n, S).astype(np.float32)
    a = rng.uniform(-1, 1, (n, 45)).astype(np.float32)
    lp = rng.uniform(-60, -40, n).astype(np.float32)
    r, d = rng.rand(n), (rng.rand(n) < 0.1).astype(np.float32)
    ns = rng.rand(n, S).astype(np.float32)
    agents = []
    for sumsq in (False, True):
        if sumsq:
            monkeypatch.setenv("PIANORL_SUMSQ", "1")
        else:
            monkeypatch.delenv("PIANORL_SUMSQ", raising=False)
        torch.manual_seed(0)
        ag = ppo.PPOAgent(S, 45, batch_size=B, ppo_epochs=2, use_wandb=False, checkpoint_dir=str(tmp_path),
                          graphs=False)
        ag.critic.eval()
        for call in range(2):
            torch.manual_seed(200 + call)
            ag.update(s, a, r, lp, ns, d)
        assert ag._fused is not None and ag._fused.fused_norm == (not sumsq)
        agents.append(ag)
    np.testing.assert_allclose(agents[0].last_update_log.cpu().numpy(), agents[1].last_update_log.cpu().numpy(),
                               rtol=1e-5, atol=1e-6)
    for (k, p0), (_, p1) in zip(_params(agents[0]).items(), _params(agents[1]).items()):
        q0, q1 = p0.cpu().numpy(), p1.cpu().numpy()
        np.testing.assert_allclose(q0, q1, rtol=0, atol=1e-6 * max(np.abs(q1).max(), 1e-6), err_msg=k)


def test_fused_norm_partials_per_segment(ppo, tmp_path):
    """The gradient kernel's clip-norm partials themselves (Adam barely moves under a
    constant gradient scale, so parameters alone would not catch a dropped segment): summed over
    the partial rows, each optimiser segment's partial equals the f64 sum of squares of that
    segment of the flat gradient the same launch wrote, to 1e-12 relative."""
    rng = np.random.RandomState(13)
    n, S, B = 96, 64, 32
    batch = (rng.rand(n, S).astype(np.float32), rng.uniform(-1, 1, (n, 45)).astype(np.float32), rng.rand(n),
             rng.uniform(-60, -40, n).astype(np.float32), rng.rand(n, S).astype(np.float32),
             (rng.rand(n) < 0.1).astype(np.float32))
    torch.manual_seed(0)
    ag = ppo.PPOAgent(S, 45, batch_size=B, ppo_epochs=1, use_wandb=False, checkpoint_dir=str(tmp_path), graphs=False)
    ag.critic.train()
    ag._prepare(*batch)
    ag._fused = ppo.FusedStep(ag)
    assert ag._fused.fused_norm and ag._fused._mlp_ok(B)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(3))[:B].cuda()
    ag._fused(idx)
    torch.cuda.synchronize()
    parts = ag._fused.bufs[B]["_norm_part"].sum(0).cpu().numpy()
    fl = ag.flat
    ends = [int(x) for x in fl.seg_end]
    g = fl.flat.double().cpu().numpy()
    for s, (a, b) in enumerate(zip([0] + ends[:-1], ends)):
        ref = float(np.sum(g[a:b] ** 2))
        assert ref > 0.0, s
        assert abs(parts[s] - ref) <= 1e-12 * ref, (s, parts[s], ref)
    assert np.all(parts[fl.nseg:] == 0.0)
