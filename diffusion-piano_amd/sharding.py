"""Env sharding across GPUs (one process per GPU) and the logging-only collectives.

Envs are independent units: global env ``g`` lives on rank
``g // envs_per_rank`` at local index ``g % envs_per_rank``; ``step()`` has no exchange
step. The only collectives are off the data path, for logging: the max of a wall time over
ranks (benchmark) and an all-gather of finished-episode returns - RCCL over xGMI on the GPU
node (backend "nccl"), gloo in the CPU tests. The reference's serial VecEnv
(parallelized_base_v2.py:53-60) has no counterpart of either.
"""

from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class EnvShard:
    rank: int
    world: int
    start: int   # first global env id on this rank
    count: int   # envs on this rank

    @property
    def stop(self) -> int:
        return self.start + self.count


def shard_envs(total: int, rank: int, world: int) -> EnvShard:
    """Contiguous, balanced split of ``total`` envs over ``world`` ranks (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if total < world:
        raise ValueError(f"{total} envs cannot be spread over {world} ranks")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return EnvShard(rank, world, start, base + (1 if rank < extra else 0))


class EpisodeReturns:
    """Per-env running returns on the env's device; finished episodes (step_type LAST)
    are appended to a device-side log without a host sync per step."""

    def __init__(self, num_envs: int, device):
        import torch

        self._torch = torch
        self.running = torch.zeros(num_envs, device=device, dtype=torch.float64)
        # per env: the return of its most recently finished episode (NaN before the first one)
        self.last_return = torch.full((num_envs,), float("nan"), device=device, dtype=torch.float32)
        self.finished_sum = torch.zeros((), device=device, dtype=torch.float64)
        self.finished_count = torch.zeros((), device=device, dtype=torch.int64)

    def update(self, reward, step_type) -> None:
        """Call after every step: FIRST steps (reward 0 after auto-reset) start a new
        episode, LAST steps close one."""
        torch = self._torch
        if self.running.is_cuda:  # one launch (libpianosim ps_episode_returns) instead of ~12
            from . import _lib
            L = _lib.load()
            if hasattr(L, "ps_episode_returns"):
                dev = self.running.device
                st = step_type.to(device=dev, dtype=torch.uint8).contiguous()
                rew = reward.to(device=dev, dtype=torch.float32).contiguous()
                # launched on the buffers' device and its current stream, whatever the caller's
                # current device is (several GPUs in one process)
                with torch.cuda.device(dev):
                    _lib.check(L.ps_episode_returns(rew.data_ptr(), st.data_ptr(), self.running.numel(),
                                                    self.running.data_ptr(), self.last_return.data_ptr(),
                                                    self.finished_sum.data_ptr(), self.finished_count.data_ptr(),
                                                    torch.cuda.current_stream(dev).cuda_stream))
                return
        first = step_type == 0
        self.running = torch.where(first, torch.zeros_like(self.running), self.running + reward.to(torch.float64))
        last = step_type == 2
        self.last_return = torch.where(last, self.running.to(torch.float32), self.last_return)
        self.finished_sum += torch.where(last, self.running, torch.zeros_like(self.running)).sum()
        self.finished_count += last.sum()

    def gather(self, group=None):
        """All ranks: (sum of finished returns, number of finished episodes, sum of the
        running returns, number of envs) over the whole job."""
        import torch
        import torch.distributed as dist

        local = torch.stack([self.finished_sum, self.finished_count.to(torch.float64),
                             self.running.sum(), torch.tensor(float(self.running.numel()),
                                                              device=self.running.device, dtype=torch.float64)])
        if dist.is_available() and dist.is_initialized():
            parts = [torch.empty_like(local) for _ in range(dist.get_world_size(group))]
            dist.all_gather(parts, local, group=group)
            local = torch.stack(parts).sum(0)
        s, n, rs, ne = (float(x) for x in local.cpu())
        return s, int(n), rs, int(ne)


def gather_episode_returns(returns: EpisodeReturns, shard: EnvShard, total: int, group=None):
    """All ranks: the per-env float32 returns of each env's last finished episode for the whole
    job, [total] in global env order (``ncclAllGather(float32
    episode_return[N/8])`` over xGMI; the reference driver keeps per-env returns,
    parallelized_base_v2.py:151,172). Shards differ in size by at most one env, so every rank
    sends a buffer padded to the largest shard and the padding is dropped after the gather."""
    import torch
    import torch.distributed as dist

    local = returns.last_return
    if not (dist.is_available() and dist.is_initialized()):
        return local.clone()
    world = dist.get_world_size(group)
    width = -(-total // world)
    buf = torch.full((width,), float("nan"), device=local.device, dtype=torch.float32)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = [parts[r][: shard_envs(total, r, world).count] for r in range(world)]
    return torch.cat(out)


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a host scalar over ranks (identity when not distributed)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
