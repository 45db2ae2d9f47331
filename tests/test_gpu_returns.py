"""sharding.EpisodeReturns on the GPU goes through one libpianosim launch (ps_episode_returns);
it must keep the torch formulation's bookkeeping (the CPU path, same inputs): running returns
restart at FIRST and accumulate otherwise, LAST closes an episode into last_return and the
finished sum / count."""
import importlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_episode_returns_kernel_matches_torch_path():
    sh = importlib.import_module("diffusion-piano_amd.sharding")
    rng = np.random.RandomState(5)
    n = 3001
    gpu, cpu = sh.EpisodeReturns(n, "cuda:0"), sh.EpisodeReturns(n, "cpu")
    for _ in range(40):
        rew = rng.normal(size=n).astype(np.float32)
        st = rng.choice([0, 1, 1, 1, 2], size=n).astype(np.uint8)
        gpu.update(torch.from_numpy(rew).cuda(), torch.from_numpy(st).cuda())
        cpu.update(torch.from_numpy(rew), torch.from_numpy(st))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gpu.running.cpu().numpy(), cpu.running.numpy())
    np.testing.assert_array_equal(gpu.last_return.cpu().numpy(), cpu.last_return.numpy())
    assert int(gpu.finished_count) == int(cpu.finished_count) > 0
    assert abs(float(gpu.finished_sum) - float(cpu.finished_sum)) <= 1e-9 * max(1.0, abs(float(cpu.finished_sum)))
