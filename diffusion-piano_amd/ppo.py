"""On-device PPO agent: the consumer of the hot path.

Mirrors ``ppo_v2.py`` (AlmondGod/diffusion-piano) so the reference driver
(``parallelized_base_v2.py:70-189``) runs against it unchanged - same class and method
names, constructor arguments, network layouts (``state_dict`` keys load both ways),
optimiser / scheduler settings, update math and checkpoint format - while every tensor of
the loop stays in HBM:

* :class:`Actor` / :class:`Critic` - ``ppo_v2.py:51-105`` (torch modules; the GEMMs run on
  hipBLASLt).
* :class:`RunningMeanStd` - ``ppo_v2.py:107-131``; statistics live on the device and are
  merged by ``prl_running_norm`` (libpianorl.so) in fp64, as the reference's numpy.
* :class:`PPOAgent` - ``ppo_v2.py:133-336``. ``select_actions`` samples with the fused
  ``prl_gauss_sample`` kernel; ``update`` runs the reward normaliser, the GAE scan
  (``prl_gae``) and the advantage normalisation (``prl_normalize``) on the device, then the
  10 epochs of shuffled minibatches with the minibatch step captured once in a HIP graph
  and replayed (the reference launches ~150 kernels and 6 host syncs per minibatch).

Semantics kept from the reference, on purpose:

* ``update(states[N], ...)`` runs the GAE recursion over the BATCH axis, exactly as
  ``ppo_v2.py:245-253`` does (a reference bug); the returns are the
  TD targets ``r + gamma V(s') (1 - d)`` (``:234-237``). Passing time-major rollouts
  ``[T, E, ...]`` instead runs the proper time-axis GAE with ``adv + V`` returns
  (:class:`RolloutTrainer`).
* The minibatch order is the one ``DataLoader(shuffle=True)`` draws: per epoch two draws
  of the global CPU generator (the loader's base seed, then the sampler's seed) and
  ``randperm`` on a CPU generator seeded with the second (verified against torch's own
  DataLoader in tests/test_ppo.py).
* The critic stays in train mode (its Dropout is active in ``update``, as in the
  reference); the actor loss and the critic loss are independent, so both backward passes
  run before both optimiser steps (same result as the reference's critic-then-actor order).

Data parallel: with ``process_group`` set, the gradients of both
networks live in one flat bucket that is all-reduced (RCCL over xGMI) once per minibatch,
between the captured backward graph and the captured optimiser graph.

There is no CPU fallback: the agent needs a ROCm GPU and libpianorl.so.
"""

from __future__ import annotations

import ctypes as C
import os
import math
import time
import warnings
from pathlib import Path
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

from . import _lib, abi

_LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
LOG_KEYS = ("actor_loss", "critic_loss", "entropy", "value_predictions", "returns", "advantages")


# ---------------------------------------------------------------- networks (ppo_v2.py:51-105)
class Actor(nn.Module):
    def __init__(self, state_dim, action_dim, hidden_dim=256):
        super().__init__()
        self.network = nn.Sequential(
            nn.Linear(state_dim, hidden_dim), nn.ReLU(), nn.LayerNorm(hidden_dim),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.LayerNorm(hidden_dim),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.LayerNorm(hidden_dim),
            nn.Linear(hidden_dim, action_dim), nn.Tanh(),
        )
        self.log_std = nn.Parameter(torch.ones(action_dim) * -1.0)

    def forward(self, state):
        mean = self.network(state)
        std = torch.exp(torch.clamp(self.log_std, -20, 2))
        return Normal(mean, std)


class Critic(nn.Module):
    def __init__(self, state_dim, hidden_dim=256):
        super().__init__()
        self.network = nn.Sequential(
            nn.Linear(state_dim, hidden_dim), nn.ReLU(), nn.LayerNorm(hidden_dim), nn.Dropout(0.1),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.LayerNorm(hidden_dim), nn.Dropout(0.1),
            nn.Linear(hidden_dim, hidden_dim // 2), nn.ReLU(), nn.LayerNorm(hidden_dim // 2),
            nn.Linear(hidden_dim // 2, 1),
        )
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=0.01)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def forward(self, state):
        return self.network(state)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _f32(x, device):
    return torch.as_tensor(x, device=device, dtype=torch.float32).contiguous()


# ---------------------------------------------------------------- kernels (include/pianorl.h)
def gae(rewards, values, next_values, dones, gamma=0.99, lam=0.95, returns_mode=0):
    """Time-major ``[T, E]`` (or ``[T]``) device tensors -> (advantages, returns). ``prl_gae``."""
    r = rewards.contiguous()
    T = r.shape[0]
    E = r.numel() // T
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    _lib.check_rl(_lib.load_rl().prl_gae(r.data_ptr(), values.contiguous().data_ptr(), next_values.contiguous().data_ptr(),
                                         dones.contiguous().data_ptr(), adv.data_ptr(), ret.data_ptr(), T, E,
                                         float(gamma), float(lam), int(returns_mode), _stream()))
    return adv, ret


def normalize_(x, eps=1e-8):
    """In place ``(x - mean) / (std + eps)`` (unbiased std). ``prl_normalize``."""
    assert x.is_contiguous() and x.dtype == torch.float32
    _lib.check_rl(_lib.load_rl().prl_normalize(x.data_ptr(), x.numel(), float(eps), _stream()))
    return x


def gauss_sample(mean, log_std, seed, offset):
    """-> (actions [N, A], log_prob sums [N]). ``prl_gauss_sample``."""
    mean = mean.contiguous()
    n, a = mean.shape
    act = torch.empty_like(mean)
    lp = torch.empty(n, device=mean.device, dtype=torch.float32)
    _lib.check_rl(_lib.load_rl().prl_gauss_sample(mean.data_ptr(), log_std.detach().contiguous().data_ptr(), n, a,
                                                  int(seed) & (2**64 - 1), int(offset), act.data_ptr(), lp.data_ptr(),
                                                  _stream()))
    return act, lp


# ---------------------------------------------------------------- RunningMeanStd (ppo_v2.py:107-131)
class RunningMeanStd:
    """Scalar running statistics in HBM (``shape=()``, the only one the agent uses)."""

    def __init__(self, epsilon=1e-4, shape=(), device=None):
        if tuple(shape) != ():
            raise ValueError("RunningMeanStd: only shape=() is implemented (what PPOAgent uses)")
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.stats = torch.tensor([0.0, 1.0, epsilon], dtype=torch.float64, device=self.device)

    # host views (synchronising; for inspection and checkpoints)
    @property
    def mean(self):
        return float(self.stats[0])

    @property
    def var(self):
        return float(self.stats[1])

    @property
    def count(self):
        return float(self.stats[2])

    def normalize_(self, x):
        """Device tensor -> fp32 device tensor normalised with the merged statistics."""
        x = _f32(x, self.device).reshape(-1)
        out = torch.empty_like(x)
        _lib.check_rl(_lib.load_rl().prl_running_norm(x.data_ptr(), x.numel(), self.stats.data_ptr(), out.data_ptr(),
                                                      _stream()))
        return out

    def __call__(self, x):
        if isinstance(x, torch.Tensor):
            return self.normalize_(x).reshape(x.shape)
        arr = np.asarray(x, np.float64)
        return self.normalize_(torch.from_numpy(arr.astype(np.float32))).cpu().numpy().astype(np.float64).reshape(arr.shape)


class RolloutBuffer:
    """``ppo_v2.py:13-49`` (kept for API parity; the drivers do not use it)."""

    def __init__(self, batch_size=64):
        self.batch_size = batch_size
        self.clear()

    def push(self, state, action, reward, log_prob, next_state, done):
        for k, v in zip(("states", "actions", "rewards", "log_probs", "next_states", "dones"),
                        (state, action, reward, log_prob, next_state, done)):
            getattr(self, k).append(v)

    def get(self):
        return tuple(torch.FloatTensor(np.array(getattr(self, k))) for k in
                     ("states", "actions", "rewards", "log_probs", "next_states", "dones"))

    def clear(self):
        self.states, self.actions, self.rewards = [], [], []
        self.log_probs, self.next_states, self.dones = [], [], []


# ---------------------------------------------------------------- DataLoader order
def loader_permutation(n: int) -> torch.Tensor:
    """The index order ``DataLoader(dataset, shuffle=True)`` yields for one epoch: the
    iterator draws its base seed, then ``RandomSampler`` draws a seed for a fresh CPU
    generator and returns ``randperm`` from it (torch/utils/data/{dataloader,sampler}.py)."""
    torch.empty((), dtype=torch.int64).random_()
    seed = int(torch.empty((), dtype=torch.int64).random_().item())
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g)


# ---------------------------------------------------------------- flat parameter state
FLAT_ALIGN = 16  # floats: every tensor of the flat buffers starts on a 64-byte boundary, so the
                 # minibatch kernels read weight rows with 16-byte loads (the gaps stay zero)


def flat_offsets(params):
    """Offsets of ``params`` in a flat buffer (each rounded up to FLAT_ALIGN) and its length."""
    offs, o = [], 0
    for p in params:
        offs.append(o)
        o += -(-p.numel() // FLAT_ALIGN) * FLAT_ALIGN
    return offs, o


class GradBucket:
    """One flat fp32 buffer holding the gradients of ``params`` (``p.grad`` are views), so
    data-parallel training does one all-reduce per minibatch instead of one per tensor. One
    slot past the gradients carries the ``guard`` word (a device int32 [1], optional) through
    the same all-reduce: a rank whose minibatch step failed stops every rank's optimiser step,
    not only its own (include/pianorl.h, the guard)."""

    guard = None

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        offs, n = flat_offsets(self.params)
        self.n = n
        self.flat = torch.zeros(n + FLAT_ALIGN, dtype=torch.float32, device=self.params[0].device)
        for p, o in zip(self.params, offs):
            p.grad = self.flat[o:o + p.numel()].view_as(p)

    def allreduce_(self, group=None):
        import torch.distributed as dist
        ws = dist.get_world_size(group)
        if ws > 1:
            st = self.flat[self.n:self.n + 1]
            if self.guard is not None:
                st.copy_(self.guard)
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
            self.flat.div_(ws)
            if self.guard is not None:  # any rank's failure: every rank's guard set
                self.guard.bitwise_or_((st != 0).to(torch.int32))


class FlatAdam(GradBucket):
    """Parameters, gradients and Adam moments of several networks in four flat HBM buffers;
    ``step()`` is ``clip_grad_norm_`` + ``Adam.step`` of every network in two launches
    (``prl_clip_adam``). The torch optimisers given are kept for their ``param_groups``
    (ReduceLROnPlateau writes their lr tensors, which are views of ``self.lr``) and
    ``state_dict`` (their state tensors are views of the flat moments)."""

    def __init__(self, optimizers, lrs, max_norm, betas=(0.9, 0.999), eps=1e-5):
        if len(optimizers) > 4:
            raise ValueError("FlatAdam: at most PRL_MAX_SEG = 4 networks")
        self.optimizers = optimizers
        segs = [[p for g in opt.param_groups for p in g["params"]] for opt in optimizers]
        params = [p for seg in segs for p in seg]
        dev = params[0].device
        offs, n = flat_offsets(params)
        self.param = torch.zeros(n, dtype=torch.float32, device=dev)
        for p, o in zip(params, offs):  # parameters become views of the flat buffer
            self.param[o:o + p.numel()].copy_(p.data.reshape(-1))
            p.data = self.param[o:o + p.numel()].view_as(p)
        super().__init__(params)
        self.exp_avg = torch.zeros_like(self.param)
        self.exp_avg_sq = torch.zeros_like(self.param)
        self._offs = offs
        ends, k = [], 0
        for seg in segs:  # a segment ends where the next one's first tensor starts
            k += len(seg)
            ends.append(offs[k] if k < len(offs) else n)
        self.seg_end = (C.c_int64 * len(segs))(*ends)
        self.nseg = len(segs)
        self.lr = torch.tensor([float(x) for x in lrs], dtype=torch.float32, device=dev)
        self.step_count = torch.zeros(self.nseg, dtype=torch.float32, device=dev)
        self.scratch = torch.zeros(256 * 4, dtype=torch.float64, device=dev)
        self.betas, self.eps, self.max_norm = betas, eps, max_norm
        for s, opt in enumerate(optimizers):
            for g in opt.param_groups:
                g["lr"] = self.lr[s]
        self._bind_state()

    def _views(self):
        offs = iter(self._offs)
        for s, opt in enumerate(self.optimizers):
            for g in opt.param_groups:
                for p in g["params"]:
                    o = next(offs)
                    yield s, p, slice(o, o + p.numel())

    def _bind_state(self):
        for s, p, sl in self._views():
            st = self.optimizers[s].state[p]
            st["step"] = self.step_count[s]
            st["exp_avg"] = self.exp_avg[sl].view_as(p)
            st["exp_avg_sq"] = self.exp_avg_sq[sl].view_as(p)

    def load_optimizer_states(self, state_dicts):
        """``Adam.load_state_dict`` for each network, then re-point the loaded state into the
        flat buffers (load_state_dict replaces the tensors)."""
        for s, (opt, sd) in enumerate(zip(self.optimizers, state_dicts)):
            opt.load_state_dict(sd)
            for g in opt.param_groups:
                self.lr[s].fill_(float(g["lr"]))
                g["lr"] = self.lr[s]
        for s, p, sl in self._views():
            st = self.optimizers[s].state[p]
            self.exp_avg[sl].copy_(st["exp_avg"].reshape(-1))
            self.exp_avg_sq[sl].copy_(st["exp_avg_sq"].reshape(-1))
            self.step_count[s].fill_(float(st["step"]))
        self._bind_state()

    # (ptr, n): gradient-norm partials a fused minibatch step left for the next step() (and the
    # step counts it advanced), prl_mlp_step_idx_norm
    pre_parts = None
    # GradBucket.guard: the guard word (include/pianorl.h, ABI version 2) - while it is non-zero
    # step() applies nothing (PPOAgent sets it; the split rows kernel writes it)
    def _guard_ptr(self):
        return None if self.guard is None else self.guard.data_ptr()

    def step(self):
        b1, b2 = self.betas
        if self.pre_parts is not None:
            ptr, n = self.pre_parts
            self.pre_parts = None
            _lib.check_rl(_lib.load_rl().prl_clip_adam_parts(
                self.param.data_ptr(), self.flat.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                self.seg_end, self.nseg, self.lr.data_ptr(), self.step_count.data_ptr(), float(b1), float(b2),
                float(self.eps), float(self.max_norm), ptr, n, self._guard_ptr(), _stream()))
            return
        _lib.check_rl(_lib.load_rl().prl_clip_adam(
            self.param.data_ptr(), self.flat.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
            self.seg_end, self.nseg, self.lr.data_ptr(), self.step_count.data_ptr(), float(b1), float(b2),
            float(self.eps), float(self.max_norm), self.scratch.data_ptr(), self._guard_ptr(), _stream()))


# ---------------------------------------------------------------- fused minibatch step
class FusedStep:
    """The minibatch step of ppo_v2.py:266-293 (actor and critic forward, losses, backward)
    without autograd: the 8 + 8 GEMMs per network go to hipBLASLt through ``torch.mm``
    (gradient GEMMs written straight into the flat gradient bucket), every op between them
    is ONE libpianorl kernel per layer and direction (bias + ReLU + LayerNorm (+ Dropout)
    forward / backward, the Gaussian-policy surrogate head, the MSE head), and all bias /
    LayerNorm / log_std gradients and the logged means come out of one column-sum launch:
    ~40 launches instead of the ~150 of torch autograd. Numerically the same math as the
    autograd path (tests/test_gpu_ppo.py compares them)."""

    # minibatches up to this many rows run as ONE matrix-core kernel (prl_mlp_step: every layer
    # of both networks in LDS, a workgroup per 16 rows) + one gradient reduction; larger ones
    # keep the hipBLASLt GEMMs, which fill the GPU on their own
    MFMA_MAX_ROWS = 512

    def __init__(self, agent: "PPOAgent"):
        self.agent = agent
        self.mfma = os.environ.get("PIANORL_NO_MFMA") is None
        # the rows kernel gathers the minibatch itself (prl_mlp_step_idx); PIANORL_GATHER=1 keeps
        # the separate gather launch (A/B)
        self.fused_gather = os.environ.get("PIANORL_GATHER") is None
        # and the gradient kernel leaves the clip norm's partials for FlatAdam (prl_clip_adam_parts);
        # PIANORL_SUMSQ=1 keeps the separate norm pass (A/B)
        self.fused_norm = os.environ.get("PIANORL_SUMSQ") is None
        self.nets = {}
        a, c = agent.actor.network, agent.critic.network
        # (linear, layernorm, dropout p) per hidden layer, then the output linear
        self.actor = [(a[0], a[2], 0.0), (a[3], a[5], 0.0), (a[6], a[8], 0.0)], a[9]
        self.critic = [(c[0], c[2], 0.1), (c[4], c[6], 0.1), (c[8], c[10], 0.0)], c[11]
        self.step = torch.zeros(1, dtype=torch.int64, device=agent.device)  # dropout draw counter
        self.seed = agent._seed ^ 0x2545F4914F6CDD1D
        self.bufs = {}

    def _buffers(self, B):
        if B in self.bufs:
            return self.bufs[B]
        ag = self.agent
        # keep the full-minibatch entry and ONE tail entry: with valid masks the tail size
        # n % B changes every update, and each size's buffers would otherwise stay allocated
        for k in [k for k in self.bufs if k != ag.batch_size]:
            del self.bufs[k]
        f32 = dict(device=ag.device, dtype=torch.float32)
        sdim, adim = ag._S.shape[1], ag._A.shape[1]
        b = dict(S=torch.empty(B, sdim, **f32), A=torch.empty(B, adim, **f32), LP=torch.empty(B, **f32),
                 ADV=torch.empty(B, **f32), RET=torch.empty(B, **f32))
        for net, (hidden, out) in (("a", self.actor), ("c", self.critic)):
            for i, (lin, ln, p) in enumerate(hidden):
                H = lin.out_features
                for k in ("Z", "Y", "XH", "dY", "dZ", "dyx", "dye"):
                    b[f"{net}{k}{i}"] = torch.empty(B, H, **f32)
                b[f"{net}rs{i}"] = torch.empty(B, **f32)
            b[f"{net}Zo"] = torch.empty(B, out.out_features, **f32)
            b[f"{net}dZo"] = torch.empty(B, out.out_features, **f32)
        b["dls"] = torch.empty(B, adim, **f32)
        for k in ("arow", "ent", "v", "sq"):
            b[k] = torch.empty(B, **f32)
        # one column-sum launch: every bias / LayerNorm / log_std gradient + the logged means
        # (actor loss, critic loss, entropy, value, return, advantage -> agent._log_row)
        L = ag._log_row
        entries = []
        for net, (hidden, out) in (("a", self.actor), ("c", self.critic)):
            for i, (lin, ln, p) in enumerate(hidden):
                H = lin.out_features
                entries += [(b[f"{net}dZ{i}"], H, 1.0, lin.bias.grad), (b[f"{net}dyx{i}"], H, 1.0, ln.weight.grad),
                            (b[f"{net}dye{i}"], H, 1.0, ln.bias.grad)]
            entries.append((b[f"{net}dZo"], out.out_features, 1.0, out.bias.grad))
        entries.append((b["dls"], adim, 1.0, ag.actor.log_std.grad))
        for j, k in enumerate(("arow", "sq", "ent", "v", "RET", "ADV")):
            entries.append((b[k], 1, 1.0 / B, L[j:j + 1]))
        n = len(entries)
        b["_cs"] = ((C.c_void_p * n)(*[e[0].data_ptr() for e in entries]), (C.c_int * n)(*[e[1] for e in entries]),
                    (C.c_float * n)(*[e[2] for e in entries]), (C.c_void_p * n)(*[e[3].data_ptr() for e in entries]), n)
        b["_scratch"] = torch.empty(((B + 127) // 128) * sum(e[1] for e in entries), **f32)
        self.bufs[B] = b
        return b

    def __call__(self, idx, log_row=None):
        """One minibatch step; the logged means go to ``log_row`` where the matrix-core step
        runs (returns True), else to the agent's ``_log_row``."""
        with torch.no_grad():  # the backward is written out: no autograd graph
            return self._step(idx, log_row)

    def _mlp_nets(self, train):
        """prl_net descriptors of (actor, critic) for prl_mlp_step (cached per dropout mode)."""
        if train in self.nets:
            return self.nets[train]
        nets = (_lib.PrlNet * 2)()
        for i, (hidden, out) in enumerate((self.actor, self.critic)):
            nets[i].nlayers, nets[i].head = 4, i
            for l, (lin, ln, p) in enumerate(hidden):
                L = nets[i].layer[l]
                L.in_, L.out = lin.in_features, lin.out_features
                L.W, L.b, L.gamma, L.beta = (lin.weight.data_ptr(), lin.bias.data_ptr(), ln.weight.data_ptr(),
                                             ln.bias.data_ptr())
                L.dropout = float(p) if (i == 0 or train) else 0.0
                L.dW, L.db, L.dgamma, L.dbeta = (lin.weight.grad.data_ptr(), lin.bias.grad.data_ptr(),
                                                 ln.weight.grad.data_ptr(), ln.bias.grad.data_ptr())
            L = nets[i].layer[3]
            L.in_, L.out = out.in_features, out.out_features
            L.W, L.b, L.dW, L.db = out.weight.data_ptr(), out.bias.data_ptr(), out.weight.grad.data_ptr(), \
                out.bias.grad.data_ptr()
        nets[0].log_std = self.agent.actor.log_std.data_ptr()
        nets[0].dlog_std = self.agent.actor.log_std.grad.data_ptr()
        self.nets[train] = nets
        return nets

    def mlp_error(self, B=None):
        """The column-split rows kernel's error word (0: every exchange completed; 1 + e: a wait on
        exchange e timed out, that step's outputs were garbage and nothing from it on was
        applied). It is the agent's guard word (``PPOAgent._guard``) for every minibatch size."""
        return int(self.agent._guard.item())

    def reset_exchanges(self):
        """After a timed-out exchange: zero every work space (the split kernel's granule tags and
        call counts restart at 0, so no stale tag of the failed call can match a later wait)."""
        for b in self.bufs.values():
            if "_mlp_work" in b:
                b["_mlp_work"].zero_()

    def _mlp_ok(self, B):
        if not self.mfma or B > self.MFMA_MAX_ROWS:
            return False
        hidden_ok = all(lin.out_features % 16 == 0 and lin.out_features <= 256
                        for lin, _, _ in self.actor[0] + self.critic[0])
        return hidden_ok and self.actor[1].out_features <= 64 and self.agent._S.shape[1] <= 384

    def _step(self, idx, log_row=None):
        ag, R, st = self.agent, _lib.load_rl(), _stream()
        B = idx.numel()
        b = self._buffers(B)
        sdim, adim = ag._S.shape[1], ag._A.shape[1]
        chk = _lib.check_rl
        train = ag.critic.training
        if self._mlp_ok(B) and self.fused_gather:  # the rows kernel reads the minibatch rows in place
            nets = self._mlp_nets(train)
            if "_mlp_work" not in b:
                n = R.prl_mlp_step_work(nets, sdim, B)
                # zeroed once: the column-split kernel's exchange counters start at 0 (include/pianorl.h)
                b["_mlp_work"] = torch.zeros(max(int(n), 1), device=ag.device, dtype=torch.float32)
            w = b["_mlp_work"]
            lr_ptr = (ag._log_row if log_row is None else log_row).data_ptr()
            fl = getattr(ag, "flat", None)
            if self.fused_norm and isinstance(fl, FlatAdam) and not ag.distributed:
                # the gradient kernel also leaves clip_grad_norm_'s partials: FlatAdam.step then
                # runs one launch (no grad_sumsq pass); single process only (no all-reduce between)
                if "_norm_part" not in b:
                    b["_norm_part"] = torch.zeros(max(1, R.prl_mlp_step_norm_parts(nets, sdim, B)), 4,
                                                  device=ag.device, dtype=torch.float64)
                npart = b["_norm_part"]
                chk(R.prl_mlp_step_idx_norm(nets, ag._S.data_ptr(), sdim, ag._A.data_ptr(), adim, ag._LP.data_ptr(),
                                            ag._ADV.data_ptr(), ag._RET.data_ptr(), idx.data_ptr(), B,
                                            float(ag.epsilon), float(ag.entropy_coef), float(self.actor[0][0][1].eps),
                                            self.seed, self.step.data_ptr(), lr_ptr, w.data_ptr(), w.numel(),
                                            fl.flat.data_ptr(), fl.seg_end, fl.nseg, fl.step_count.data_ptr(),
                                            npart.data_ptr(), npart.shape[0], ag._guard.data_ptr(), st))
                fl.pre_parts = (npart.data_ptr(), npart.shape[0])
                return log_row is not None
            chk(R.prl_mlp_step_idx(nets, ag._S.data_ptr(), sdim, ag._A.data_ptr(), adim, ag._LP.data_ptr(),
                                   ag._ADV.data_ptr(), ag._RET.data_ptr(), idx.data_ptr(), B, float(ag.epsilon),
                                   float(ag.entropy_coef), float(self.actor[0][0][1].eps), self.seed,
                                   self.step.data_ptr(), lr_ptr, w.data_ptr(), w.numel(), ag._guard.data_ptr(), st))
            return log_row is not None
        chk(R.prl_gather_minibatch(ag._S.data_ptr(), sdim, ag._A.data_ptr(), adim, ag._LP.data_ptr(), ag._ADV.data_ptr(),
                                   ag._RET.data_ptr(), idx.data_ptr(), B, b["S"].data_ptr(), b["A"].data_ptr(),
                                   b["LP"].data_ptr(), b["ADV"].data_ptr(), b["RET"].data_ptr(), self.step.data_ptr(), st))
        if self._mlp_ok(B):
            nets = self._mlp_nets(train)
            if "_mlp_work" not in b:
                n = R.prl_mlp_step_work(nets, sdim, B)
                # zeroed once: the column-split kernel's exchange counters start at 0 (include/pianorl.h)
                b["_mlp_work"] = torch.zeros(max(int(n), 1), device=ag.device, dtype=torch.float32)
            w = b["_mlp_work"]
            chk(R.prl_mlp_step(nets, b["S"].data_ptr(), sdim, b["A"].data_ptr(), adim, b["LP"].data_ptr(),
                               b["ADV"].data_ptr(), b["RET"].data_ptr(), B, float(ag.epsilon), float(ag.entropy_coef),
                               float(self.actor[0][0][1].eps), self.seed, self.step.data_ptr(),
                               (ag._log_row if log_row is None else log_row).data_ptr(),
                               w.data_ptr(), w.numel(), ag._guard.data_ptr(), st))
            return log_row is not None
        for net, (hidden, out) in (("a", self.actor), ("c", self.critic)):
            x = b["S"]
            for i, (lin, ln, p) in enumerate(hidden):  # forward
                p = p if (net == "a" or train) else 0.0
                Z = b[f"{net}Z{i}"]
                torch.mm(x, lin.weight.t(), out=Z)
                chk(R.prl_lnrelu_fwd(Z.data_ptr(), lin.bias.data_ptr(), ln.weight.data_ptr(), ln.bias.data_ptr(), B,
                                     lin.out_features, float(ln.eps), float(p), self.seed, self.step.data_ptr(), i,
                                     b[f"{net}Y{i}"].data_ptr(), b[f"{net}XH{i}"].data_ptr(),
                                     b[f"{net}rs{i}"].data_ptr(), st))
                x = b[f"{net}Y{i}"]
            torch.mm(x, out.weight.t(), out=b[f"{net}Zo"])
            if net == "a":
                chk(R.prl_actor_head(b["aZo"].data_ptr(), out.bias.data_ptr(), ag.actor.log_std.data_ptr(),
                                     b["A"].data_ptr(), b["LP"].data_ptr(), b["ADV"].data_ptr(), B, adim,
                                     float(ag.epsilon), float(ag.entropy_coef), b["adZo"].data_ptr(), b["dls"].data_ptr(),
                                     b["arow"].data_ptr(), b["ent"].data_ptr(), st))
            else:
                chk(R.prl_critic_head(b["cZo"].data_ptr(), out.bias.data_ptr(), b["RET"].data_ptr(), B,
                                      b["cdZo"].data_ptr(), b["v"].data_ptr(), b["sq"].data_ptr(), st))
            dz = b[f"{net}dZo"]  # backward
            torch.mm(dz.t(), x, out=out.weight.grad)
            dy = torch.mm(dz, out.weight, out=b[f"{net}dY{len(hidden) - 1}"])
            for i in reversed(range(len(hidden))):
                lin, ln, p = hidden[i]
                p = p if (net == "a" or train) else 0.0
                chk(R.prl_lnrelu_bwd(dy.data_ptr(), b[f"{net}Z{i}"].data_ptr(), lin.bias.data_ptr(),
                                     b[f"{net}XH{i}"].data_ptr(), b[f"{net}rs{i}"].data_ptr(), ln.weight.data_ptr(), B,
                                     lin.out_features, float(p), self.seed, self.step.data_ptr(), i,
                                     b[f"{net}dZ{i}"].data_ptr(), b[f"{net}dyx{i}"].data_ptr(),
                                     b[f"{net}dye{i}"].data_ptr(), st))
                dz = b[f"{net}dZ{i}"]
                xin = b["S"] if i == 0 else b[f"{net}Y{i - 1}"]
                torch.mm(dz.t(), xin, out=lin.weight.grad)
                if i > 0:
                    dy = torch.mm(dz, lin.weight, out=b[f"{net}dY{i - 1}"])
        src, cols, scale, dst, n = b["_cs"]
        chk(R.prl_colsums(n, src, cols, scale, dst, B, b["_scratch"].data_ptr(), b["_scratch"].numel(), st))


# ---------------------------------------------------------------- the agent (ppo_v2.py:133-336)
class PPOAgent:
    def __init__(self, state_dim, action_dim, lr=1e-4, gamma=0.99, epsilon=0.2, entropy_coef=0.01, value_coef=1.0,
                 max_grad_norm=0.5, ppo_epochs=10, batch_size=64, device="cuda", checkpoint_dir="checkpoints",
                 use_wandb=True, *, gae_lambda=0.95, process_group=None, graphs=True, sample_seed=None,
                 tune_gemms=False, fused=True):
        if not torch.cuda.is_available():
            raise _lib.PianosimError("PPOAgent needs a ROCm GPU (torch.cuda.is_available() is False)")
        _lib.load_rl()  # fail loudly if the kernels are missing
        if tune_gemms:
            # TunableOp: the first call of each GEMM shape times the rocBLAS and hipBLASLt
            # solutions and keeps the fastest (the minibatch GEMMs are M = 128 problems the
            # default heuristics serve with 256-wide macro tiles). Every shape of the captured
            # step is first met in the eager warm-up steps, so no tuning runs during capture.
            import torch.cuda.tunable as tunable
            tunable.enable(True)
            tunable.tuning_enable(True)
            tunable.set_max_tuning_duration(30)
        self.device = torch.device(device if str(device).startswith("cuda") else "cuda")
        self.actor = Actor(state_dim, action_dim).to(self.device)
        self.critic = Critic(state_dim).to(self.device)
        self.process_group = process_group
        self.distributed = process_group is not None or (
            torch.distributed.is_available() and torch.distributed.is_initialized()
            and torch.distributed.get_world_size() > 1)
        # the torch optimisers carry the reference's settings, param_groups and state_dict
        # format; their step is FlatAdam's fused kernel (critic segment first, then actor)
        adam = dict(betas=(0.9, 0.999), eps=1e-5, capturable=True)
        self.actor_optimizer = torch.optim.Adam(self.actor.parameters(), lr=torch.tensor(float(lr)), **adam)
        self.critic_optimizer = torch.optim.Adam(self.critic.parameters(), lr=torch.tensor(float(lr) * 2), **adam)
        self.flat = FlatAdam([self.critic_optimizer, self.actor_optimizer], [float(lr) * 2, float(lr)],
                             max_norm=max_grad_norm, betas=(0.9, 0.999), eps=1e-5)
        self.bucket = self.flat
        # the guard word (include/pianorl.h): the split rows kernel's timeout code; while set, no
        # optimiser launch applies anything; update() reads it with its statistics and raises
        self._guard = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.flat.guard = self._guard
        if self.distributed:  # identical replicas: rank 0's initial weights everywhere
            torch.distributed.broadcast(self.flat.param, src=0, group=process_group)
        self.actor_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.actor_optimizer, mode="max", factor=0.5,
                                                                          patience=100)
        self.critic_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.critic_optimizer, mode="min",
                                                                           factor=0.5, patience=100)
        self.reward_normalizer = RunningMeanStd(device=self.device)
        self.max_grad_norm = max_grad_norm
        self.gamma = gamma
        self.gae_lambda = gae_lambda
        self.epsilon = epsilon
        self.entropy_coef = entropy_coef
        self.value_coef = value_coef  # stored, unused in the loss: as the reference (ppo_v2.py:287)
        self.ppo_epochs = ppo_epochs
        self.batch_size = batch_size
        self.rollout_buffer = RolloutBuffer(batch_size)
        self.checkpoint_dir = Path(checkpoint_dir)
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        self.use_wandb = use_wandb
        self._wandb = None
        if use_wandb:
            try:
                import wandb
                self._wandb = wandb
                wandb.init(project="robopianist-ppo", config=dict(lr=lr, gamma=gamma, epsilon=epsilon,
                                                                   entropy_coef=entropy_coef, value_coef=value_coef,
                                                                   ppo_epochs=ppo_epochs, batch_size=batch_size))
            except ImportError:
                warnings.warn("wandb is not installed: PPOAgent logs stay in agent.last_update_log")
        self.graphs = graphs
        self._seed = (torch.initial_seed() if sample_seed is None else int(sample_seed)) ^ 0x5DEECE66D
        self._offset = 0
        self._cap = 0
        self._graph = None
        self._chunk_graph = None
        self._graph_eager_left = 2
        self._cap_stream = torch.cuda.Stream(self.device)
        self.last_update_log = None
        self.timing = {}
        self.fused = fused
        self._fused = None

    # -- acting (ppo_v2.py:211-218)
    def select_actions(self, states):
        as_numpy = not isinstance(states, torch.Tensor)
        s = _f32(states, self.device)
        with torch.no_grad():
            mean = self.actor.network(s)
        actions, log_probs = gauss_sample(mean, self.actor.log_std, self._seed, self._offset)
        self._offset += 1
        if as_numpy:
            return actions.cpu().numpy(), log_probs.cpu().numpy()
        return actions, log_probs

    # -- minibatch step (ppo_v2.py:266-293): forward + both backwards | all-reduce | clip + steps
    def _forward_backward(self, idx, log_row):
        if self.fused:
            if self._fused is None:
                self._fused = FusedStep(self)
            # the matrix-core step writes the log row in place (no copy node per minibatch in
            # the chunk graph); the per-layer path writes self._log_row
            if not self._fused(idx, log_row) and log_row.data_ptr() != self._log_row.data_ptr():
                log_row.copy_(self._log_row)
            return
        b_s = self._S.index_select(0, idx)
        b_a = self._A.index_select(0, idx)
        b_lp = self._LP.index_select(0, idx)
        b_adv = self._ADV.index_select(0, idx)
        b_ret = self._RET.index_select(0, idx)
        # Normal(mean, std).log_prob / .entropy written out with torch.distributions' own
        # formulas: the distribution object validates its arguments with a host sync, which
        # cannot sit inside a captured graph
        mean = self.actor.network(b_s)
        log_scale = torch.log(torch.exp(torch.clamp(self.actor.log_std, -20, 2)))
        var = torch.exp(torch.clamp(self.actor.log_std, -20, 2)) ** 2
        new_lp = (-((b_a - mean) ** 2) / (2 * var) - log_scale - _LOG_SQRT_2PI).sum(1)
        entropy = (0.5 + 0.5 * math.log(2 * math.pi) + log_scale).expand_as(mean).mean()
        ratio = torch.exp(new_lp - b_lp)
        surr1 = ratio * b_adv
        surr2 = torch.clamp(ratio, 1 - self.epsilon, 1 + self.epsilon) * b_adv
        actor_loss = -torch.min(surr1, surr2).mean() - self.entropy_coef * entropy
        value_pred = self.critic(b_s).squeeze(-1)
        critic_loss = F.mse_loss(value_pred, b_ret)
        self.flat.flat.zero_()
        critic_loss.backward()
        actor_loss.backward()
        log_row.copy_(torch.stack([actor_loss, critic_loss, entropy, value_pred.mean(), b_ret.mean(),
                                   b_adv.mean()]).detach())

    def _clip_step(self):
        self.flat.step()  # clip_grad_norm_ + Adam.step of the critic, then of the actor

    def _eager_step(self, idx, log_row):
        self._forward_backward(idx, log_row)
        if self.distributed:
            self.bucket.allreduce_(self.process_group)
        self._clip_step()

    def _warmup_step(self):
        """A real minibatch step, run eagerly on the capture stream before capturing (BLAS
        handles / workspaces and the optimiser state then exist outside the capture)."""
        s = self._cap_stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._eager_step(self._idx, self._log_row)
        torch.cuda.current_stream().wait_stream(s)

    def _capture(self):
        """Capture the full-size minibatch step as HIP graph(s): one graph on a single GPU;
        [forward+backward] and [clip+step] around the eager all-reduce when distributed."""
        pool = torch.cuda.graph_pool_handle()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, pool=pool, stream=self._cap_stream):
            self._forward_backward(self._idx, self._log_row)
            if not self.distributed:
                self._clip_step()
        g2 = None
        if self.distributed:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool, stream=self._cap_stream):
                self._clip_step()
        self._graph = (g1, g2)

    # full-size minibatch steps per captured graph once the single-step graph exists (single
    # GPU): one index upload, one replay and one log copy per CHUNK steps instead of per step
    CHUNK = 8

    def _capture_chunk(self):
        """CHUNK consecutive minibatch steps as ONE graph: step j reads its indices from
        ``_idx_chunk[j B:(j + 1) B]`` and logs into ``_log_chunk[j]``; the same launches in the
        same order as CHUNK single-step replays (bitwise the same update)."""
        B = self.batch_size
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle(), stream=self._cap_stream):
            for j in range(self.CHUNK):
                self._forward_backward(self._idx_chunk[j * B:(j + 1) * B], self._log_chunk[j])
                self._clip_step()
        self._chunk_graph = g

    def _replay(self):
        g1, g2 = self._graph
        g1.replay()
        if g2 is not None:
            self.bucket.allreduce_(self.process_group)
            g2.replay()

    def _ensure_capacity(self, n, sdim, adim):
        if n <= self._cap and self._S.shape[1] == sdim and self._A.shape[1] == adim:
            return
        f32 = dict(device=self.device, dtype=torch.float32)
        self._cap = n
        self._S = torch.empty(n, sdim, **f32)
        self._A = torch.empty(n, adim, **f32)
        self._LP = torch.empty(n, **f32)
        self._ADV = torch.empty(n, **f32)
        self._RET = torch.empty(n, **f32)
        self._idx = torch.zeros(self.batch_size, device=self.device, dtype=torch.int64)
        self._idx_chunk = torch.zeros(self.CHUNK * self.batch_size, device=self.device, dtype=torch.int64)
        self._log_row = torch.zeros(len(LOG_KEYS), **f32)
        self._log_chunk = torch.zeros(self.CHUNK, len(LOG_KEYS), **f32)
        self._graph = None  # buffers moved: re-capture
        self._chunk_graph = None
        self._fused = None
        self._graph_eager_left = 2

    def _prepare(self, states, actions, rewards, log_probs, next_states, dones, valid=None):
        """Reward normalisation, critic values, GAE, advantage normalisation (ppo_v2.py:221-256).
        ``valid`` (same shape as ``rewards``, optional): samples to train on; the others (an
        auto-reset's FIRST step: its action had no effect, its "next state" is a new episode)
        are dropped after GAE, so they enter neither the advantage normalisation nor a
        minibatch. Returns (normalised rewards, number of samples)."""
        dev = self.device
        s = _f32(states, dev)
        a = _f32(actions, dev)
        lp = _f32(log_probs, dev).reshape(-1)
        ns = _f32(next_states, dev)
        d = _f32(dones, dev)
        raw = _f32(rewards, dev)
        keep = None
        if valid is None:
            r = self.reward_normalizer(raw)
        else:  # the running statistics see only the samples trained on
            keep = _f32(valid, dev).reshape(-1) != 0
            r = torch.zeros_like(raw).reshape(-1)
            r[keep] = self.reward_normalizer(raw.reshape(-1)[keep]).reshape(-1)
            r = r.reshape(raw.shape)
        time_major = s.dim() == 3
        with torch.no_grad():
            if time_major:  # [T, E, D]: values of every step, bootstrap from the last next state
                T, E = s.shape[:2]
                values = self.critic(s.reshape(T * E, -1)).reshape(T, E)
                next_values = self.critic(ns[-1] if ns.dim() == 3 else ns).reshape(1, E).expand(T, E).contiguous()
                adv, ret = gae(r.reshape(T, E), values, next_values, d.reshape(T, E), self.gamma, self.gae_lambda,
                               returns_mode=1)
            else:  # the reference's batch-axis recursion and TD returns
                values = self.critic(s).squeeze(-1)
                next_values = self.critic(ns).squeeze(-1)
                adv, ret = gae(r, values, next_values, d, self.gamma, self.gae_lambda, returns_mode=0)
        sdim, adim = s.shape[-1], a.shape[-1]
        s, a, adv, ret = s.reshape(-1, sdim), a.reshape(-1, adim), adv.reshape(-1), ret.reshape(-1)
        if keep is not None:
            s, a, lp, adv, ret = s[keep], a[keep], lp[keep], adv[keep].contiguous(), ret[keep]
        n = adv.numel()
        adv = normalize_(adv)
        self._ensure_capacity(n, sdim, adim)
        self._S[:n].copy_(s)
        self._A[:n].copy_(a)
        self._LP[:n].copy_(lp)
        self._ADV[:n].copy_(adv)
        self._RET[:n].copy_(ret)
        return r, n

    # -- update (ppo_v2.py:220-309)
    def update(self, states, actions, rewards, log_probs, next_states, dones, valid=None):
        """ppo_v2.PPOAgent.update; ``valid`` (optional, this implementation): see _prepare."""
        t0 = time.perf_counter()
        r, n = self._prepare(states, actions, rewards, log_probs, next_states, dones, valid)
        B = self.batch_size
        nmb = (n + B - 1) // B
        log = torch.empty(self.ppo_epochs * nmb, len(LOG_KEYS), device=self.device)
        row = 0
        nfull = n // B  # the full-size minibatches come first; only the last may be short
        CH = self.CHUNK
        for _ in range(self.ppo_epochs):
            perm = loader_permutation(n).to(self.device, non_blocking=True)
            i = 0
            while i < nmb:
                if self.graphs and not self.distributed and self._graph is not None and i + CH <= nfull:
                    if self._chunk_graph is None:
                        self._capture_chunk()
                    self._idx_chunk.copy_(perm[i * B:(i + CH) * B])
                    self._chunk_graph.replay()
                    log[row:row + CH].copy_(self._log_chunk)
                    i += CH
                    row += CH
                    continue
                idx = perm[i * B:(i + 1) * B]
                i += 1
                if idx.numel() == B and self.graphs:
                    self._idx.copy_(idx)
                    if self._graph is None and self._graph_eager_left > 0:
                        self._warmup_step()
                        self._graph_eager_left -= 1
                    else:
                        if self._graph is None:
                            self._capture()
                        self._replay()
                    log[row].copy_(self._log_row)
                else:
                    self._eager_step(idx, log[row])
                row += 1
        self.last_update_log = log
        if self._wandb is not None:
            for rec in log.cpu().numpy():
                self._wandb.log(dict(zip(LOG_KEYS, map(float, rec))))
        # the plateau signal: the mean normalised reward of the samples trained on (r holds 0
        # at the dropped auto-reset rows)
        r_mean = r.mean() if valid is None else r.reshape(-1)[_f32(valid, self.device).reshape(-1) != 0].mean()
        # (the guard word rides along: one host read per update, no extra sync)
        stats = torch.stack([r_mean, log[-1, 1], self._guard[0].to(r_mean.dtype)])
        if self.distributed:  # one plateau decision for all replicas (else their lrs drift apart)
            torch.distributed.all_reduce(stats, group=self.process_group)
            stats /= torch.distributed.get_world_size(self.process_group)
        mean_reward, mean_critic_loss, failed = (float(x) for x in stats.cpu())
        if failed != 0.0:
            code = int(self._guard.item())
            self._guard.zero_()
            if self._fused is not None:
                self._fused.reset_exchanges()
            raise _lib.PianosimError(
                "PPOAgent.update: a column-split rows kernel exchange timed out "
                f"(error word {code}: 1 + exchange index; on another rank if 0); the minibatch steps "
                "from the failed one on were not applied (parameters, Adam moments and step counts "
                "unchanged). Another kernel occupying CUs can cause this; PIANORL_MLP_SPLIT=0 selects "
                "the one-workgroup-per-tile rows kernel.")
        self.actor_scheduler.step(mean_reward)
        self.critic_scheduler.step(mean_critic_loss)
        self.timing["update_s"] = time.perf_counter() - t0

    # -- checkpoints (ppo_v2.py:311-336, ppo_base.py:150-155)
    def _state(self):
        return {
            "actor_state_dict": self.actor.state_dict(),
            "critic_state_dict": self.critic.state_dict(),
            "actor_optimizer_state_dict": self.actor_optimizer.state_dict(),
            "critic_optimizer_state_dict": self.critic_optimizer.state_dict(),
            "actor_scheduler_state_dict": self.actor_scheduler.state_dict(),
            "critic_scheduler_state_dict": self.critic_scheduler.state_dict(),
        }

    def save_checkpoint(self, episode, rewards):
        ck = dict(episode=episode, rewards=rewards, reward_normalizer=self.reward_normalizer.stats.cpu(), **self._state())
        path = self.checkpoint_dir / f"checkpoint_episode_{episode}.pt"
        torch.save(ck, path)
        if self._wandb is not None:
            self._wandb.save(str(path))
        print(f"Saved checkpoint to {path}")
        return path

    def load_checkpoint(self, path):
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.actor.load_state_dict(ck["actor_state_dict"])
        self.critic.load_state_dict(ck["critic_state_dict"])
        self.flat.load_optimizer_states([ck["critic_optimizer_state_dict"], ck["actor_optimizer_state_dict"]])
        self.actor_scheduler.load_state_dict(ck["actor_scheduler_state_dict"])
        self.critic_scheduler.load_state_dict(ck["critic_scheduler_state_dict"])
        if "reward_normalizer" in ck:
            self.reward_normalizer.stats.copy_(ck["reward_normalizer"])
        self._graph = None  # optimiser state tensors were replaced: re-capture
        self._chunk_graph = None
        self._graph_eager_left = 2

    def save_model(self, path):
        torch.save({"actor_state_dict": self.actor.state_dict(), "critic_state_dict": self.critic.state_dict()}, path)


# ---------------------------------------------------------------- time-axis rollouts
class RolloutTrainer:
    """The MI355X-first loop: ``horizon`` control steps of all envs are collected into
    time-major HBM buffers (observations never leave the device), then one PPO update runs
    with time-axis GAE over ``[horizon, N]``. ``reference_semantics=True`` instead calls
    ``agent.update`` after every env step with that step's batch, as
    ``parallelized_base_v2.py:116-166`` does."""

    def __init__(self, env, agent: PPOAgent, horizon: int = 16, reference_semantics: bool = False):
        self.env, self.agent = env, agent
        self.horizon = horizon
        self.reference_semantics = reference_semantics
        N, D = env.num_envs, env.obs_dim
        f32 = dict(device=env.device, dtype=torch.float32)
        H = 1 if reference_semantics else horizon
        self.obs = torch.empty(H, N, D, **f32)
        self.act = torch.empty(H, N, env.action_dim, **f32)  # the model's action row (39 / 41 / 43 / 45)
        self.logp = torch.empty(H, N, **f32)
        self.rew = torch.empty(H, N, **f32)
        self.done = torch.empty(H, N, **f32)
        self.valid = torch.empty(H, N, **f32)  # 0 at an auto-reset's FIRST step (action ignored)
        self.ep_return = torch.zeros(N, **f32)
        self.return_sum = torch.zeros((), **f32)  # over finished episodes (device; read when logging)
        self.episodes = torch.zeros((), **f32)
        self._cur = env.reset().clone()

    def _act_step(self, t):
        env = self.env
        self.obs[t].copy_(self._cur)
        a, lp = self.agent.select_actions(self._cur)
        self.act[t].copy_(a)
        self.logp[t].copy_(lp)
        obs, rew, _, st = env.step(a)
        self.rew[t].copy_(rew)
        done = self.done[t]
        done.copy_(st == abi.LAST)
        self.valid[t].copy_(st != abi.FIRST)
        self.ep_return += rew
        self.return_sum += (self.ep_return * done).sum()
        self.episodes += done.sum()
        self.ep_return.mul_(1.0 - done)
        self._cur.copy_(obs)

    def iterate(self):
        """One outer iteration; returns the number of env-steps taken."""
        N = self.env.num_envs
        if self.reference_semantics:
            # the reference loop (parallelized_base_v2.py:116-166) steps until all(dones), then
            # resets: it never updates on a reset transition. Here the envs auto-reset, so a
            # step whose batch is all FIRST is not trained on, and FIRST rows of a mixed
            # batch are dropped.
            self._act_step(0)
            nv = int(self.valid[0].sum().item())
            if nv == N:
                self.agent.update(self.obs[0], self.act[0], self.rew[0], self.logp[0], self._cur, self.done[0])
            elif nv > 0:
                self.agent.update(self.obs[0], self.act[0], self.rew[0], self.logp[0], self._cur, self.done[0],
                                  valid=self.valid[0])
            return N
        for t in range(self.horizon):
            self._act_step(t)
        nxt = self._cur.unsqueeze(0)
        self.agent.update(self.obs, self.act, self.rew, self.logp, nxt, self.done, valid=self.valid)
        return self.horizon * N
