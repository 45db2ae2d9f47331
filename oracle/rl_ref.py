"""CPU restatement of the PPO statistics of ppo_v2.py (TEST INFRASTRUCTURE ONLY).

Checker for libpianorl.so (include/pianorl.h): imported by tests/ only, never by the
product package. Plain numpy loops in fp64, following the reference line by line:

* running_norm  <- RunningMeanStd.__call__          ppo_v2.py:107-131
* gae           <- PPOAgent.update, returns + GAE   ppo_v2.py:234-253
* normalize     <- advantage normalisation          ppo_v2.py:256
* gauss_logp    <- Actor.forward + Normal.log_prob  ppo_v2.py:70-74, 216

Pinned by tests/golden/ppo_v2.npz, produced by running the reference's own PPOAgent
(tests/golden/make_ppo_golden.py): the GAE advantages / TD returns it built and the
RunningMeanStd statistics after two update() calls.
"""

from __future__ import annotations

import numpy as np


def running_norm(stats, x):
    """stats = (mean, var, count) -> (new_stats, normalised x). ppo_v2.py:113-131."""
    mean, var, count = stats
    x = np.asarray(x, np.float64)
    batch_mean = np.mean(x, axis=0)
    batch_var = np.var(x, axis=0)
    batch_count = x.shape[0]
    delta = batch_mean - mean
    tot_count = count + batch_count
    new_mean = mean + delta * batch_count / tot_count
    m_a = var * count
    m_b = batch_var * batch_count
    M2 = m_a + m_b + np.square(delta) * count * batch_count / tot_count
    new_var = M2 / tot_count
    return (new_mean, new_var, tot_count), (x - new_mean) / np.sqrt(new_var + 1e-8)


def gae(rewards, values, next_values, dones, gamma=0.99, lam=0.95, returns_mode=0):
    """Arrays [T, E] (or [T]): the reference's recursion over axis 0 (ppo_v2.py:245-253).
    returns_mode 0: TD returns r + gamma * next_values * (1 - d) (:234-237); 1: adv + values."""
    r = np.asarray(rewards, np.float64)
    squeeze = r.ndim == 1
    r = r.reshape(r.shape[0], -1)
    v = np.asarray(values, np.float64).reshape(r.shape)
    nv = np.asarray(next_values, np.float64).reshape(r.shape)
    d = np.asarray(dones, np.float64).reshape(r.shape)
    T = r.shape[0]
    adv = np.zeros_like(r)
    g = np.zeros(r.shape[1])
    for t in reversed(range(T)):
        next_value = nv[t] if t == T - 1 else v[t + 1]
        delta = r[t] + gamma * next_value * (1 - d[t]) - v[t]
        g = delta + gamma * lam * (1 - d[t]) * g
        adv[t] = g
    ret = r + gamma * nv * (1 - d) if returns_mode == 0 else adv + v
    if squeeze:
        return adv[:, 0], ret[:, 0]
    return adv, ret


def normalize(x, eps=1e-8):
    """(x - mean) / (std + eps) with torch.std's unbiased estimator (ppo_v2.py:256)."""
    x = np.asarray(x, np.float64)
    return (x - x.mean()) / (x.std(ddof=1) + eps)


def gauss_logp(mean, log_std, action):
    """Normal(mean, exp(clamp(log_std, -20, 2))).log_prob(action).sum(1) (ppo_v2.py:70-74, 216)."""
    mean = np.asarray(mean, np.float64)
    ls = np.clip(np.asarray(log_std, np.float64), -20, 2)
    sd = np.exp(ls)
    a = np.asarray(action, np.float64)
    return (-((a - mean) ** 2) / (2 * sd * sd) - np.log(sd) - 0.5 * np.log(2 * np.pi)).sum(-1)
