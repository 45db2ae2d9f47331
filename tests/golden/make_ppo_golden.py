"""Generate tests/golden/ppo_v2.npz from the reference's own PPO agent (ppo_v2.py).

Runs only in the build container (it reads /root/reference, absent on the GPU box). The
reference module is loaded by path and executed unmodified, with two stand-ins the image
forces on it (SURVEY.md section 7 "ppo_v2 drop-in"):

* ``wandb`` is not installed: a stub module records ``wandb.log`` calls (the reference logs
  actor_loss / critic_loss / entropy / value_predictions / returns / advantages once per
  minibatch, ppo_v2.py:295-303), which become golden per-minibatch values;
* ``ReduceLROnPlateau(verbose=True)`` raises TypeError on the installed torch 2.10 (the
  keyword was removed): the scheduler class is wrapped to drop ``verbose``.

A spy on ``torch.utils.data.TensorDataset`` records the tensors ``update`` builds
(ppo_v2.py:262-264): the GAE advantages after normalisation and the TD returns.

Determinism: the agent runs on CPU; ``torch.manual_seed`` is set before construction
(initial weights) and again before every ``update`` call (the DataLoader's RandomSampler
draws its permutation seed from the global CPU generator). The critic's Dropout layers
are put in eval mode because their masks come from a device-specific RNG stream; that is
the only behavioural change, and the parity test applies the same setting.

Usage: python tests/golden/make_ppo_golden.py   (writes tests/golden/ppo_v2.npz)
"""

from __future__ import annotations

import importlib.util
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "ppo_v2.npz"

STATE_DIM, ACTION_DIM = 319, 45
N, BATCH, EPOCHS = 96, 32, 2
INIT_SEED, UPDATE_SEEDS, DATA_SEED = 0, (1234, 4321), 7
NSAMPLE = 64  # sampled elements per parameter tensor


def _stub_wandb():
    logs = []
    w = types.ModuleType("wandb")
    w.init = lambda *a, **k: None
    w.log = lambda d, *a, **k: logs.append(dict(d))
    w.save = lambda *a, **k: None
    sys.modules["wandb"] = w
    return logs


def _load_reference():
    base = torch.optim.lr_scheduler.ReduceLROnPlateau

    class _NoVerbose(base):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)

    torch.optim.lr_scheduler.ReduceLROnPlateau = _NoVerbose
    spec = importlib.util.spec_from_file_location("ref_ppo_v2", REF / "ppo_v2.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod  # the wrapper stays installed: the reference looks the class up at call time


def critic_state(critic):
    """Portable critic start state: Linear weights U(-1, 1) * 0.01 * sqrt(3 / fan_in) from
    RandomState(99) in module order, biases 0 (the orthogonal gain-0.01 scale)."""
    rng = np.random.RandomState(99)
    out = {}
    for k, v in critic.state_dict().items():
        if k.endswith("weight") and v.dim() == 2:
            w = rng.uniform(-1, 1, tuple(v.shape)) * 0.01 * np.sqrt(3.0 / v.shape[1])
            out[k] = torch.from_numpy(w.astype(np.float32))
        elif k.endswith("bias") and k.replace("bias", "weight") in out:
            out[k] = torch.zeros_like(v)
    return out


def sample_index(n):
    return np.linspace(0, n - 1, min(n, NSAMPLE)).astype(np.int64)


def batch(rng):
    """States / rewards / dones of one update() batch (parallelized_base_v2.py:133-160).
    numpy's legacy RandomState stream is stable, so the test regenerates these."""
    states = rng.uniform(0, 1, (N, STATE_DIM)).astype(np.float32)
    next_states = rng.uniform(0, 1, (N, STATE_DIM)).astype(np.float32)
    rewards = rng.uniform(0, 2, N).astype(np.float64)
    dones = (rng.uniform(0, 1, N) < 0.1)
    return states, rewards, next_states, dones


def main():
    logs = _stub_wandb()
    ref = _load_reference()
    torch.manual_seed(INIT_SEED)
    agent = ref.PPOAgent(STATE_DIM, ACTION_DIM, lr=1e-4, gamma=0.99, epsilon=0.2, batch_size=BATCH,
                         ppo_epochs=EPOCHS, device="cpu", checkpoint_dir="/tmp/ppo_golden_ckpt", use_wandb=True)
    agent.critic.eval()  # dropout off (see module docstring)
    out = {}
    # the orthogonal critic init goes through LAPACK QR, whose last bits differ between
    # host CPUs: the orthogonal weights are recorded (init/), then every critic Linear is
    # set to a portable seeded state that both sides load (critic_state)
    init_critic = {k: v.clone() for k, v in agent.critic.state_dict().items()}
    with torch.no_grad():
        for k, v in critic_state(agent.critic).items():
            agent.critic.state_dict()[k].copy_(v)
    params = dict(("actor." + k, v) for k, v in agent.actor.state_dict().items())
    params.update(("critic." + k, v) for k, v in init_critic.items())
    out["param_names"] = np.array(sorted(params))
    for k in sorted(params):
        flat = params[k].detach().reshape(-1).numpy().copy()
        out["init/" + k] = flat[sample_index(flat.size)]

    spy = []
    real_td = torch.utils.data.TensorDataset

    class _Spy(real_td):
        def __init__(self, *tensors):
            spy.append([t.detach().clone() for t in tensors])  # once per epoch, same tensors
            super().__init__(*tensors)

    torch.utils.data.TensorDataset = _Spy
    rng = np.random.RandomState(DATA_SEED)
    for call, seed in enumerate(UPDATE_SEEDS):
        s, r, ns, d = batch(rng)
        # actions and old log-probs from the reference's own sampler (ppo_v2.py:211-218)
        torch.manual_seed(seed + 1)
        a, lp = agent.select_actions(s)
        with torch.no_grad():
            ent = agent.actor(torch.from_numpy(s)).entropy().mean().item()
        out[f"u{call}/states_sum"] = np.float64(s.astype(np.float64).sum() + ns.astype(np.float64).sum())
        out[f"u{call}/actions"], out[f"u{call}/rewards"], out[f"u{call}/dones"] = a, r, d
        out[f"u{call}/log_probs"] = lp.astype(np.float32)
        out[f"u{call}/entropy"] = np.float64(ent)
        nlog = len(logs)
        torch.manual_seed(seed)
        agent.update(s, a, r, lp, ns, d.astype(np.float32))
        rec = spy[-1]
        out[f"u{call}/advantages"] = rec[3].numpy()
        out[f"u{call}/returns"] = rec[4].numpy()
        keys = ("actor_loss", "critic_loss", "entropy", "value_predictions", "returns", "advantages")
        out[f"u{call}/log"] = np.array([[L[k] for k in keys] for L in logs[nlog:]], np.float64)
        out[f"u{call}/rn_mean"] = np.float64(agent.reward_normalizer.mean)
        out[f"u{call}/rn_var"] = np.float64(agent.reward_normalizer.var)
        out[f"u{call}/rn_count"] = np.float64(agent.reward_normalizer.count)
        out[f"u{call}/actor_lr"] = np.float64(agent.actor_optimizer.param_groups[0]["lr"])
        out[f"u{call}/critic_lr"] = np.float64(agent.critic_optimizer.param_groups[0]["lr"])
    torch.utils.data.TensorDataset = real_td
    params = dict(("actor." + k, v) for k, v in agent.actor.state_dict().items())
    params.update(("critic." + k, v) for k, v in agent.critic.state_dict().items())
    for k in sorted(params):
        flat = params[k].detach().reshape(-1).numpy().copy()
        out["final/" + k] = flat[sample_index(flat.size)]
    out["meta"] = np.array([STATE_DIM, ACTION_DIM, N, BATCH, EPOCHS, INIT_SEED, *UPDATE_SEEDS, DATA_SEED])
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({OUT.stat().st_size} B), {len(logs)} minibatch log records")


if __name__ == "__main__":
    main()
