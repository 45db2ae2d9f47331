"""Benchmark: env-steps/s of the batched PianoWithShadowHands step on MI355X.

One "step" = one control step (0.05 s of simulated time = 10 physics substeps + task
layer) of every env on every GPU, random uniform canonical actions (pre-generated on
device with torch's Philox generator, seed 12345 + rank). Inputs and state are resident in
HBM when the timed region starts. The timed hand is the reference's default PianoTask collider
set (--hand hull: primitive_fingertip_collisions=False, palm boxes + convex-hull distal
colliders); the same workload with the reference's primitive option (palm boxes + capsule distal
colliders) and with the all-capsule authored hand follows as the line's "primitive_fingertips"
and "capsule_hand" legs. Multi-GPU: one process per GPU, 4096 envs per GPU
(weak scaling, envs shard with no data-path collective); episode returns are gathered
over RCCL after the timed region for logging.

Prints ONE JSON line (rank 0); see DESIGN.md "Measurement".
"""

from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

ENVS_PER_GPU = 4096
METRIC = "env steps/sec at 4096 parallel envs; qpos L\u221e drift vs CPU MuJoCo"


def bytes_per_env_step(obs_dim):
    """compulsory HBM bytes per env-step, the roofline's algorithmic basis:
    action 45x4 + (qpos, qvel, qacc_warmstart) 140x4 read+write + sustain/t_idx 16
    + obs write + reward/discount/step_type 12 = 4884 B (obs 329) / 4844 B (obs 319)."""
    return 45 * 4 + 3 * 140 * 4 * 2 + 16 + obs_dim * 4 + 12

# collider sets: TaskConfig.primitive_fingertip_collisions value, kernel instantiation, description
HANDS = {
    "hull": (False, "pianosim_kernel<true, 2>", "palm boxes + convex-hull distal colliders: the reference's default "
                                             "PianoTask(primitive_fingertip_collisions=False)"),
    "primitive": (True, "pianosim_kernel<true, 2>", "palm boxes + capsule distal colliders: the reference's "
                                                 "PianoTask(primitive_fingertip_collisions=True)"),
    "authored": (None, "pianosim_kernel<false, 2>", "all-capsule authored hand (no reference counterpart)"),
}

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector), spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    p.add_argument("--song", default="crossing_field", choices=["twinkle", "crossing_field", "guren"])
    p.add_argument("--hand", default="hull", choices=list(HANDS),
                   help="collider set of the timed workload: hull = the reference's default "
                        "(PianoTask(primitive_fingertip_collisions=False): palm boxes + convex-hull distal "
                        "colliders, shadow_hand.py:95,144-152, tasks/base.py:101); primitive = the reference's "
                        "primitive_fingertip_collisions=True (palm boxes + capsule distal colliders); authored = "
                        "the all-capsule hand (no reference counterpart)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-legs", "--no-hull-leg", dest="no_legs", action="store_true",
                   help="skip timing the same workload with the other two collider sets after the main line")
    p.add_argument("--cpu-sample-envs", type=int, default=16)
    p.add_argument("--cpu-sample-steps", type=int, default=500)
    return p.parse_args()


def load_song(dp, name):
    data = ROOT / "tests" / "data"
    if name == "twinkle":
        return dp.music.twinkle_twinkle_little_star_one_hand(), dp.TaskConfig()
    if name == "crossing_field":
        return dp.music.parse_midi(data / "Crossing Field Cut 10s.mid"), dp.TaskConfig(trim_silence=True)
    seq = dp.music.add_fingering_from_annotation_file(data / "Guren no Yumiya Cut 14s.mid",
                                                      data / "Guren no Yumiya Cut 14s_fingering v3.txt")
    return seq, dp.TaskConfig(trim_silence=True)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """The host cores this process may use (the box's CPU share: OMP_NUM_THREADS there)."""
    n = len(os.sched_getaffinity(0))
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_baseline(dp, seq, task, n_envs, steps):
    """The fp64 oracle (oracle/pianosim_ref.c), one thread (the reference's serial VecEnv),
    same song/task, random actions; plus the all-cores variant (OpenMP over envs)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import ref  # CPU checker/baseline only
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    lo, hi = dp.model.action_spec(md)

    def run(n, k, threads):
        env = ref.OracleEnv(md, st, tc, n)
        env.reset()
        rng = np.random.RandomState(12345)
        acts = [rng.uniform(lo, hi, (n, 45)).astype(np.float32) for _ in range(k)]
        t0 = time.perf_counter()
        for a in acts:
            env.step(a, threads=threads)
        dt = time.perf_counter() - t0
        return n * k / dt, dt

    v1, dt1 = run(n_envs, steps, 1)
    out = {"value": v1, "unit": "env-steps/s", "cores": 1, "kind": "port",
           "sample": f"{n_envs} envs x {steps} random-action control steps, {dt1:.1f} s, 1 thread "
                     f"(fp64 oracle restatement; MuJoCo/dm_control absent)", "cpu": _cpu_model()}
    nt = _cpu_threads()
    if nt > 1:
        n_all, k_all = 16 * nt, max(50, steps // 5)
        va, dta = run(n_all, k_all, nt)
        out["all_cores"] = {"value": va, "unit": "env-steps/s", "cores": nt, "kind": "port",
                            "sample": f"{n_all} envs x {k_all} steps, {dta:.1f} s, OpenMP over envs"}
    return out


def oracle_sha() -> str:
    """sha256 (16 hex) of the physics a CPU-side profile was measured on: the checker's source
    text and the compiled default model (ps_model_desc bytes); tools/chaos_floor.py records the
    same. Reads the checker's file text only."""
    import ctypes
    import hashlib

    sys.path.insert(0, str(ROOT))
    model = importlib.import_module("diffusion-piano_amd.model")
    h = hashlib.sha256()
    try:
        h.update((ROOT / "oracle" / "pianosim_ref.c").read_bytes())
    except OSError:
        return "missing"
    h.update(ctypes.string_at(ctypes.addressof(md := model.build_model()), ctypes.sizeof(md)))
    return h.hexdigest()[:16]


def lib_sha(path=None) -> str:
    """sha256 (16 hex) of the step kernel's library: profiles record it, and the bench only
    quotes a profile measured on the very binary it runs."""
    import hashlib

    if path is None:  # the library the loader actually binds (PIANOSIM_LIB can point elsewhere)
        sys.path.insert(0, str(ROOT))
        path = importlib.import_module("diffusion-piano_amd._lib").LIB_PATH
    p = Path(path)
    try:
        return hashlib.sha256(p.read_bytes()).hexdigest()[:16]
    except OSError:
        return "missing"


def _profile(name, sha=None):
    """A committed profile; with ``sha``, only if it was measured on that library build."""
    f = ROOT / "profiles" / name
    try:
        d = json.loads(f.read_text()) if f.exists() else None
    except ValueError:
        return None
    if d is not None and sha is not None and d.get("lib_sha") != sha:
        return None
    return d


def _pmc_match(d, n_envs, song, hand):
    return d and d.get("envs") == n_envs and d.get("song", song) == song and d.get("hand", "authored") == hand


def pmc_traffic(n_envs, song, sha, hand="authored"):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary of THIS build, else None."""
    d = _profile("pmc_latest.json", sha)
    if _pmc_match(d, n_envs, song, hand):
        return d.get("hbm_bytes_per_launch")
    return None


def issue_summary(n_envs, song, sha, hand="authored"):
    """Where the wave time goes (the binding limit: latency, not HBM), from the committed SQ
    counter pass of THIS build (tools/collect_pmc.py): fractions of the waves' lifetime
    issuing / waiting."""
    d = _profile("pmc_latest.json", sha)
    if _pmc_match(d, n_envs, song, hand) and "wave_issue_frac" in d:
        return {k: d[k] for k in ("wave_issue_frac", "wave_wait_frac", "wave_issue_stall_frac", "valu_insts_per_env_step")}
    return None


def valu_roofline(song, n_envs, kernel_ms):
    """The compute-side roofline: algorithmic FLOPs per env-step from the
    oracle's counting build (tools/count_flops.py -> profiles/flops.json) over the FP32 vector
    peak. Like the HBM one it is far from 1: the bound is dependent-op latency per wave."""
    d = _profile("flops.json")
    c = d and d.get("configs", {}).get(song)
    if not c:
        return None
    achieved = c["flops_per_env_step"] * n_envs / (kernel_ms * 1e-3) / 1e12
    return {"bound": "valu", "achieved": achieved, "peak": FP32_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP32_VECTOR_PEAK_TFLOPS, "flops_per_env_step": c["flops_per_env_step"],
            "source": "profiles/flops.json (tools/count_flops.py)"}


def drift_summary(sha):
    """qpos L-inf drift vs the fp64 CPU step, from the drift report tests/test_gpu_drift.py
    wrote for THIS build (PIANOSIM_REPORT=profiles/drift_latest.json; it records the library
    hash), else None."""
    d = _profile("drift_latest.json", sha)
    if not d or "bench" not in d:
        return None
    # the workload the headline times (Crossing Field, the reference's default box / hull
    # colliders); the all-capsule Twinkle report beside it
    out = {"reference": "fp64 CPU restatement (MuJoCo absent)", "envs": d.get("envs"),
           "workload": (d.get("workloads") or {}).get("bench"),
           "source": "profiles/drift_latest.json (tests/test_gpu_drift.py, same library build)"}
    chaos = _profile("chaos_floor.json") or {}
    if chaos.get("oracle_sha") != oracle_sha():  # measured on other physics: not this floor
        chaos = {}
    for w in ("bench", "twinkle"):
        dw, cw, ow = d.get(w, {}), chaos.get(w, {}), {}
        for k in ("zero_action", "trace_actions", "random_actions"):
            if k in dw:
                tf = dw[k]["teacher_forced_qpos_linf"]
                ow[k] = {"teacher_forced_p99": tf["p99"], "teacher_forced_p99_well_conditioned":
                         tf.get("p99_well_conditioned"), "free_running_1000_steps_max": dw[k]["free_running_max_over_1000"]}
                # the same metric for the fp64 checker against itself, 1e-12 limit-preserving
                # perturbation per episode (tools/chaos_floor.py)
                c = cw.get(f"{k.split('_')[0]}/delta=1e-12")
                if c:
                    ow[k]["fp64_self_1e-12_free_running_max"] = c["max_over_1000"]
        out[w if w != "bench" else "bench_workload"] = ow
    return out


def setup_distributed(backend=None):
    """One process per GPU (torch.distributed.run env vars). The device is selected BEFORE the
    process group is created and handed to it (device_id), so RCCL binds this rank's GPU
    instead of guessing; ``backend`` defaults to nccl (RCCL) with a GPU, gloo without."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
    else:
        dev = torch.device("cpu")
    backend = backend or os.environ.get("PIANOSIM_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
    if world > 1:
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return world, rank, local, dev


def stagger_episodes(env, global_start, T):
    """Spread the envs over the episode: env g starts at t_idx = g mod T, so every timed step
    auto-resets ~N/T envs (reset time included as the episodes roll over)."""
    t = ((np.arange(env.num_envs) + global_start) % T).astype(np.int32)
    env.set_state({"t_idx": t})


def timed_rollout(env, actions, steps, warmup, dev, returns, sharding):
    """W untimed steps, then exactly K steps between barrier + device sync on both sides;
    the wall time is the max over ranks. Also the mean per-step device time of env.step from
    events on the launch stream (None on CPU)."""
    import torch
    import torch.distributed as dist

    dist_on = dist.is_available() and dist.is_initialized()
    cuda = dev.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    pool = len(actions)
    for i in range(warmup):
        _, rew, _, st = env.step(actions[i % pool])
        returns.update(rew, st)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(steps)] if cuda else None
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(steps)] if cuda else None
    if dist_on:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        if cuda:
            starts[i].record()
        _, rew, _, st = env.step(actions[(warmup + i) % pool])
        if cuda:
            ends[i].record()
        returns.update(rew, st)
    sync()
    if dist_on:
        dist.barrier()
    elapsed = sharding.max_over_ranks(time.perf_counter() - t0, device=dev)
    kernel_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)])) if cuda else None
    return elapsed, kernel_ms


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world, rank, local, dev = setup_distributed()
    dp = importlib.import_module("diffusion-piano_amd")
    sharding = importlib.import_module("diffusion-piano_amd.sharding")
    seq, task = load_song(dp, args.song)
    import dataclasses

    def hand_task(hand):  # TaskConfig of a collider set (HANDS)
        return dataclasses.replace(task, primitive_fingertip_collisions=HANDS[hand][0])

    shard = sharding.shard_envs(args.envs * world, rank, world)  # weak scaling: envs per GPU fixed
    env = dp.BatchedPianoEnv(shard.count, seq, hand_task(args.hand), device=dev, seed=12345,
                             env_offset=shard.start)
    N = shard.count
    gen = torch.Generator(device=dev).manual_seed(12345 + rank)
    pool = max(1, min(args.steps + args.warmup, 64))
    actions = [torch.rand(N, 45, device=dev, generator=gen) * 2 - 1 for _ in range(pool)]
    env.reset()
    stagger_episodes(env, shard.start, env.song.T)
    returns = sharding.EpisodeReturns(N, dev)
    elapsed, kernel_ms = timed_rollout(env, actions, args.steps, args.warmup, dev, returns, sharding)
    # logging only: RCCL all-gather of the episode returns over xGMI, after the timed region
    fin_sum, fin_n, run_sum, n_all = returns.gather()
    mean_ret = run_sum / n_all
    # per-env float32 returns of each env's last finished episode, all ranks
    per_env = sharding.gather_episode_returns(returns, shard, args.envs * world)
    per_env_done = per_env[~torch.isnan(per_env)]
    stats = env.solver_stats().cpu().numpy()
    obs_dim = env.obs_dim
    total_steps = args.envs * world * args.steps
    value = total_steps / elapsed
    env.close()
    env = None
    legs = {}
    if not args.no_legs:
        # the same workload (envs, actions, K, W) with the other collider sets, after the main
        # timed region; top-level keys of the line (the driver's parsed record keeps them)
        # and the timed hand without the refining Newton step on coupled substeps (solver_refine=0;
        # TaskConfig's default, timed above, is 1 since round 6: the price of the 1e-4 parity target)
        runs = [(h, h, hand_task(h)) for h in HANDS if h != args.hand]
        runs.append(("unrefined", args.hand, dataclasses.replace(hand_task(args.hand), solver_refine=0)))
        for key, hand, ltask in runs:
            lenv = dp.BatchedPianoEnv(shard.count, seq, ltask, device=dev, seed=12345, env_offset=shard.start)
            lenv.reset()
            stagger_episodes(lenv, shard.start, lenv.song.T)
            l_elapsed, l_kernel_ms = timed_rollout(lenv, actions, args.steps, args.warmup, dev,
                                                   sharding.EpisodeReturns(N, dev), sharding)
            legs[key] = {"value": total_steps / l_elapsed, "ms_per_step": l_elapsed / args.steps * 1e3,
                         "kernel_ms_avg": l_kernel_ms, "unit": "env-steps/s", "hand": HANDS[hand][2],
                         "kernel": HANDS[hand][1]}
            if key == "unrefined":
                legs[key]["solver_refine"] = 0
            lenv.close()
    if rank == 0:
        sha = lib_sha()
        bpe = bytes_per_env_step(obs_dim)
        achieved = bpe * N / (kernel_ms * 1e-3) / 1e9
        traffic = pmc_traffic(N, args.song, sha, args.hand)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform random canonical actions (torch Philox, seed 12345+rank); episodes "
                    "staggered (env g starts at t_idx = g mod T) so every step auto-resets ~N/T envs",
            "config": {"workload": f"{N} envs/GPU {args.song} random-action rollout, 10 physics substeps "
                                   f"per env-step, constraint forces by the primal Newton solve (friction loss, "
                                   f"uncapped rows)",
                       "envs_per_gpu": N, "song": args.song, "parallelism": f"dp{world}",
                       "hand": f"{args.hand}: {HANDS[args.hand][2]}",
                       "mean_return_logged": mean_ret, "episodes_finished": fin_n,
                       "per_env_returns_gathered": int(per_env.numel()),
                       "mean_last_episode_return": float(per_env_done.mean()) if per_env_done.numel() else None,
                       "lib_sha": sha,
                       "solver_last_step": {"newton_iterations_per_substep": float(stats[:, 0].mean() / 10.0),
                                            "contact_cap_substeps": int(stats[:, 1].sum()),
                                            "newton_cap_substeps": int(stats[:, 2].sum()),
                                            "max_contact_rows": int(stats[:, 3].max()),
                                            "coupled_substep_frac": float(stats[:, 4].sum() / (10.0 * stats.shape[0])),
                                            "bad_pivot_substeps": int(stats[:, 5].sum()),
                                            "max_coupled_dofs": int(stats[:, 6].max())}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": HANDS[args.hand][1], "kernel_ms_avg": kernel_ms,
                         "kernel_ms_note": "HIP events around ps_step on the launch stream: order_kernel "
                                           "(counting sort, ~5 us) + pianosim_kernel",
                         "bytes_per_env_step": bpe, "wave_time": issue_summary(N, args.song, sha, args.hand),
                         "profile_note": "traffic / wave_time: rocprofv3 PMC passes of this library build "
                                         "(profiles/pmc_latest.json lib_sha), null when none exists"},
            "valu_roofline": valu_roofline(args.song, N, kernel_ms),
            "qpos_drift": drift_summary(sha),
        }
        # the other collider sets on the same workload (reference primitive option; all-capsule hand)
        if "primitive" in legs:
            line["primitive_fingertips"] = legs["primitive"]
        if "authored" in legs:
            line["capsule_hand"] = legs["authored"]
        if "hull" in legs:
            line["reference_default_hand"] = legs["hull"]
        if "unrefined" in legs:  # TaskConfig(solver_refine=0): no refining step
            line["unrefined_solve"] = legs["unrefined"]
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N=1 figure
            line["cpu_baseline"] = cpu_baseline(dp, seq, hand_task(args.hand), args.cpu_sample_envs, args.cpu_sample_steps)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
