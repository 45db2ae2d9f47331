"""Batched PianoWithShadowHands environments on the MI355X kernel.

Host-side mirror of the reference's interface for the hot path:

* :class:`VectorizedPianoEnv` - the VecEnv surface of ``parallelized_base_v2.py:21-67``
  (``reset() -> obs dict``, ``step(actions) -> (obs dict, rewards, dones)``,
  ``envs[i].observation_spec()/action_spec()``) plus the ``observation_spec`` /
  ``action_spec`` attributes of ``parallelized_base.py:87-89``.
* :class:`BatchedPianoEnv` - the torch-native core: flat ``[N, obs_dim]`` observations,
  rewards, discounts and dm_env step types as torch-ROCm tensors; no host round trip.
* :func:`load` - ``robopianist.suite.load`` (suite/__init__.py:50-93) for one env,
  returning dm_env ``TimeStep`` objects.

Task options follow ``PianoWithShadowHands.__init__`` (piano_with_shadow_hands.py:50-66).
Every compute call goes through libpianosim.so; there is no CPU fallback.
"""

from __future__ import annotations

import ctypes as C
import enum
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, NamedTuple, Optional, Tuple, Union

import numpy as np

from . import _lib, abi, model as model_lib, music


# ---------------------------------------------------------------- dm_env (not installed)
class StepType(enum.IntEnum):
    FIRST = abi.FIRST
    MID = abi.MID
    LAST = abi.LAST

    def first(self) -> bool:
        return self is StepType.FIRST

    def mid(self) -> bool:
        return self is StepType.MID

    def last(self) -> bool:
        return self is StepType.LAST


class TimeStep(NamedTuple):
    """dm_env.TimeStep: FIRST carries reward/discount None."""

    step_type: Any
    reward: Any
    discount: Any
    observation: Any

    def first(self) -> bool:
        return self.step_type == StepType.FIRST

    def mid(self) -> bool:
        return self.step_type == StepType.MID

    def last(self) -> bool:
        return self.step_type == StepType.LAST


class Array(NamedTuple):
    shape: tuple
    dtype: Any
    name: str = ""


class BoundedArray(NamedTuple):
    shape: tuple
    dtype: Any
    minimum: np.ndarray
    maximum: np.ndarray
    name: str = ""


# ---------------------------------------------------------------- task configuration
@dataclass
class TaskConfig:
    """``PianoWithShadowHands`` keyword arguments (piano_with_shadow_hands.py:50-66) plus the
    solver settings of this implementation."""

    n_steps_lookahead: int = 1
    n_seconds_lookahead: Optional[float] = None
    trim_silence: bool = False
    wrong_press_termination: bool = False
    initial_buffer_time: float = 0.0
    disable_fingering_reward: bool = False
    disable_forearm_reward: bool = False
    disable_colorization: bool = False  # rendering only: no effect here
    disable_hand_collisions: bool = False
    energy_penalty_coef: float = 5e-3
    randomize_hand_positions: bool = False  # piano_with_shadow_hands.py:64,491-499
    control_timestep: float = model_lib.CONTROL_TIMESTEP
    physics_timestep: float = model_lib.PHYSICS_TIMESTEP
    # Constraint solve: "newton" (alias "exact") = MuJoCo's primal problem minimised by Newton
    # iterations with exact line search (mj_solNewton), to convergence - the unique solution
    # every MuJoCo solver converges to. `solver_iterations` caps the Newton iterations per
    # substep (None: the library default, 24). The round-1 truncated "pgs" is retired.
    constraint_solver: str = "newton"
    solver_iterations: Optional[int] = None
    # 0: the solve ends when its line search ends in the Hessian's piece (the exact minimiser, to
    # the fp32 factor's error); 1 (the default since round 6): one more Newton step in that piece
    # on coupled-hand substeps - the fp32 parity target of 1e-4 over all env-steps of the coupled /
    # heavy-contact / Guren cases needs it, ~5% of the throughput; 2: on
    # every substep. Solves that end in the previous substep's guessed piece are not refined
    # (ps_task_cfg.solver_refine)
    solver_refine: int = 1
    max_contacts: int = 20
    hand_xml: Optional[str] = None  # a user hand MJCF (path or text, mjcf.load_hand); None = authored hand
    # PianoTask keyword arguments (tasks/base.py:96-107, forwarded by PianoWithShadowHands'
    # **kwargs, piano_with_shadow_hands.py:65):
    gravity_compensation: bool = False  # gravcomp 1 on every hand body (tasks/base.py:185-186)
    attachment_yaw: float = model_lib.ATTACHMENT_YAW  # degrees, hand roots about z (tasks/base.py:174-181)
    # Fingertip colliders (shadow_hand.py:95,144-152). None: the authored hand (capsules
    # everywhere, this implementation's default); True: Menagerie-style palm boxes with capsule
    # distal colliders; False (the reference's default): palm boxes with convex-hull (mesh)
    # distal colliders, the step kernel's hull instantiation. Exclusive with hand_xml.
    primitive_fingertip_collisions: Optional[bool] = None
    # THJ5, THJ1, LFJ5 and their actuators removed, THJ2 narrowed (shadow_hand.py:73-79,164-183):
    # action 39, joints_pos 23 per hand
    reduced_action_space: bool = False
    # the forearm slides kept: a subset of ("forearm_tx", "forearm_ty") (shadow_hand.py:270-311)
    forearm_dofs: Tuple[str, ...] = model_lib.FOREARM_DOFS

    def lookahead(self) -> int:
        if self.n_seconds_lookahead is not None:
            return int(math.ceil(self.n_seconds_lookahead / self.control_timestep))
        return self.n_steps_lookahead


def _to_sequence(midi) -> music.NoteSequence:
    if isinstance(midi, music.NoteSequence):
        return midi
    if isinstance(midi, (str, Path)):
        return music.parse_midi(midi)
    raise TypeError(f"unsupported midi input {type(midi)!r}")


def compile_task(midi, cfg: TaskConfig, canonical_actions: bool = True):
    """-> (ps_model_desc, SongTables, ps_task_cfg) for a song and task options."""
    if isinstance(midi, music.SongTables):
        song = midi
    else:
        seq = _to_sequence(midi)
        if cfg.trim_silence:
            seq = music.trim_silence(seq)
        song = music.song_tables(seq, cfg.control_timestep, cfg.initial_buffer_time)
    hand = None
    if cfg.hand_xml is not None and cfg.primitive_fingertip_collisions is not None:
        raise ValueError("hand_xml and primitive_fingertip_collisions are exclusive: the MJCF names its colliders")
    if cfg.hand_xml is not None:
        from . import mjcf
        hand = mjcf.load_hand(cfg.hand_xml)
    elif cfg.primitive_fingertip_collisions is not None:
        from . import mjcf
        hand = mjcf.box_hull_hand(hull_fingertips=not cfg.primitive_fingertip_collisions)
    md = model_lib.build_model(control_timestep=cfg.control_timestep,
                               physics_timestep=cfg.physics_timestep,
                               hand_collisions=not cfg.disable_hand_collisions, hand=hand,
                               gravity_compensation=cfg.gravity_compensation,
                               attachment_yaw=cfg.attachment_yaw,
                               reduced_action_space=cfg.reduced_action_space,
                               forearm_dofs=cfg.forearm_dofs)
    tc = abi.TaskCfg()
    tc.n_steps_lookahead = cfg.lookahead()
    tc.fingering_reward = int(not cfg.disable_fingering_reward and song.has_fingering)
    tc.forearm_reward = int(not cfg.disable_forearm_reward)
    tc.wrong_press_termination = int(cfg.wrong_press_termination)
    tc.energy_penalty_coef = cfg.energy_penalty_coef
    if cfg.constraint_solver not in ("newton", "exact"):
        raise ValueError(f"constraint_solver must be 'newton' (or its alias 'exact'), got {cfg.constraint_solver!r}"
                         " (the round-1 truncated 'pgs' solver is retired)")
    tc.solver = abi.SOLVER_NEWTON
    tc.solver_iterations = 0 if cfg.solver_iterations is None else int(cfg.solver_iterations)
    if cfg.solver_refine not in (0, 1, 2):
        raise ValueError(f"solver_refine must be 0, 1 or 2, got {cfg.solver_refine!r}")
    tc.solver_refine = int(cfg.solver_refine)
    tc.randomize_hand_positions = int(cfg.randomize_hand_positions)
    tc.max_contacts = min(cfg.max_contacts, abi.MAX_CONTACTS_LIMIT)
    tc.canonical_actions = int(canonical_actions)
    return md, song, tc


def obs_layout(tc: abi.TaskCfg, md: Optional[abi.ModelDesc] = None) -> Dict[str, slice]:
    """Observation keys in the order the reference driver concatenates them
    (parallelized_base_v2.py:122-131); joints_pos as wide as the model's hands (``md``)."""
    out, o = {}, 0
    g = (tc.n_steps_lookahead + 1) * (abi.NKEY + 1)
    out["goal"] = slice(o, o + g); o += g
    if tc.fingering_reward:
        out["fingering"] = slice(o, o + 10); o += 10
    out["piano/state"] = slice(o, o + abi.NKEY); o += abi.NKEY
    out["piano/sustain_state"] = slice(o, o + 1); o += 1
    nj = abi.obs_joints(md)
    out["rh_shadow_hand/joints_pos"] = slice(o, o + nj[0]); o += nj[0]
    out["lh_shadow_hand/joints_pos"] = slice(o, o + nj[1]); o += nj[1]
    return out


# ---------------------------------------------------------------- batched core
class BatchedPianoEnv:
    """N envs on one GPU; all tensors live in HBM (torch-ROCm)."""

    def __init__(self, num_envs: int, midi, task: Optional[TaskConfig] = None, device=None,
                 canonical_actions: bool = True, seed: int = 0, env_offset: int = 0):
        """``seed`` keys the per-env random draws (randomize_hand_positions); ``env_offset`` is the
        global id of env 0 when one job's envs are sharded over GPUs (sharding.EnvShard.start), so
        global env g draws the same values at any world size."""
        import torch

        self._torch = torch
        if not torch.cuda.is_available():
            raise _lib.PianosimError("BatchedPianoEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.task = task or TaskConfig()
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.num_envs = int(num_envs)
        self.model_desc, self.song, self.task_cfg = compile_task(midi, self.task, canonical_actions)
        self.canonical_actions = canonical_actions
        self.obs_dim = abi.obs_dim(self.task_cfg, self.model_desc)
        self.obs_slices = obs_layout(self.task_cfg, self.model_desc)
        self.action_dim = model_lib.action_dim(self.model_desc)
        self.action_lo, self.action_hi = model_lib.action_spec(self.model_desc)
        L = _lib.load()
        sd = abi.SongDesc.from_tables(self.song)
        if L.ps_model_desc_size() != C.sizeof(abi.ModelDesc):
            raise _lib.PianosimError("ps_model_desc layout mismatch between abi.py and the library")
        h = C.c_void_p()
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _lib.check(L.ps_create(C.addressof(self.model_desc), C.addressof(sd), C.addressof(self.task_cfg),
                               self.num_envs, dev_index, seed, C.byref(h)))
        self._h = h
        if hasattr(L, "ps_env_obs_dim") and (L.ps_env_obs_dim(h) != self.obs_dim or
                                             L.ps_env_action_dim(h) != self.action_dim):
            raise _lib.PianosimError("observation / action layout mismatch between the host and the library")
        if env_offset:
            _lib.check(L.ps_set_env_offset(h, int(env_offset)))
        N = self.num_envs
        f32 = dict(device=self.device, dtype=torch.float32)
        self.obs = torch.zeros(N, self.obs_dim, **f32)
        self.reward = torch.zeros(N, **f32)
        self.discount = torch.ones(N, **f32)
        self.step_type = torch.zeros(N, device=self.device, dtype=torch.uint8)

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().ps_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return self._torch.cuda.current_stream(self.device).cuda_stream

    # -- core API (device tensors, asynchronous on the current stream)
    def reset(self, mask=None):
        torch = self._torch
        mptr = None
        if mask is not None:
            self._mask = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
            mptr = self._mask.data_ptr()
        _lib.check(_lib.load().ps_reset(self._h, mptr, self.obs.data_ptr(), self.stream))
        if mask is None:
            self.step_type.fill_(abi.FIRST)
        return self.obs

    def step(self, action):
        torch = self._torch
        a = torch.as_tensor(action, device=self.device, dtype=torch.float32)
        if a.shape != (self.num_envs, self.action_dim):
            raise ValueError(f"action must be [{self.num_envs}, {self.action_dim}], got {tuple(a.shape)}")
        a = a.contiguous()
        self._action = a  # keep alive until the kernel ran
        _lib.check(_lib.load().ps_step(self._h, a.data_ptr(), self.obs.data_ptr(), self.reward.data_ptr(),
                                       self.discount.data_ptr(), self.step_type.data_ptr(), self.stream))
        return self.obs, self.reward, self.discount, self.step_type

    def get_state(self) -> Dict[str, Any]:
        torch = self._torch
        N = self.num_envs
        out = dict(qpos=torch.empty(N, abi.NV, device=self.device), qvel=torch.empty(N, abi.NV, device=self.device),
                   qacc_ws=torch.empty(N, abi.NV, device=self.device), ctrl=torch.empty(N, abi.NU, device=self.device),
                   sustain=torch.empty(N, device=self.device),
                   t_idx=torch.empty(N, device=self.device, dtype=torch.int32),
                   last=torch.empty(N, device=self.device, dtype=torch.uint8))
        _lib.check(_lib.load().ps_get_state(self._h, *(out[k].data_ptr() for k in
                                                      ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")),
                                            self.stream))
        return out

    def set_state(self, state: Dict[str, Any]):
        torch = self._torch
        kinds = dict(qpos=torch.float32, qvel=torch.float32, qacc_ws=torch.float32, ctrl=torch.float32,
                     sustain=torch.float32, t_idx=torch.int32, last=torch.uint8)
        keep = {}
        for k, dt in kinds.items():
            if k in state and state[k] is not None:
                keep[k] = torch.as_tensor(state[k], device=self.device).to(dt).contiguous()
        ptr = lambda k: keep[k].data_ptr() if k in keep else None
        _lib.check(_lib.load().ps_set_state(self._h, *(ptr(k) for k in kinds), self.stream))
        self._keep = keep

    def set_applied(self, qfrc):
        torch = self._torch
        if qfrc is None:
            _lib.check(_lib.load().ps_set_applied(self._h, None, self.stream))
            return
        t = torch.as_tensor(qfrc, device=self.device, dtype=torch.float32).contiguous()
        _lib.check(_lib.load().ps_set_applied(self._h, t.data_ptr(), self.stream))
        self._applied = t

    def reward_terms(self):
        t = self._torch.empty(self.num_envs, abi.NTERMS, device=self.device)
        _lib.check(_lib.load().ps_reward_terms(self._h, t.data_ptr(), self.stream))
        return t

    def fingertips(self):
        t = self._torch.empty(self.num_envs, 2, 5, 3, device=self.device)
        _lib.check(_lib.load().ps_fingertips(self._h, t.data_ptr(), self.stream))
        return t

    def contact_count(self):
        t = self._torch.empty(self.num_envs, device=self.device, dtype=self._torch.int32)
        _lib.check(_lib.load().ps_contact_count(self._h, t.data_ptr(), self.stream))
        return t

    def record_contacts(self, on: bool = True) -> None:
        """Keep each step's contact list for contacts() (ps_record_contacts; off by default)."""
        _lib.check(_lib.load().ps_record_contacts(self._h, 1 if on else 0))

    def contacts(self):
        """-> list per env of (kind, key, g1, g2, dist, pos[3], normal[3]) of the last step's
        task-layer collision pass (physics.data.contact); needs record_contacts()."""
        raw = self._torch.empty(self.num_envs, abi.MAX_CONTACTS_LIMIT, 17, device=self.device, dtype=self._torch.float32)
        _lib.check(_lib.load().ps_contacts(self._h, raw.data_ptr(), self.stream))
        self._torch.cuda.synchronize(self.device)
        f = raw.cpu().numpy()
        ints = f.view(np.int32)
        n = self.contact_count().cpu().numpy()
        out = []
        for e in range(self.num_envs):
            out.append([(int(ints[e, c, 13]), int(ints[e, c, 14]), int(ints[e, c, 15]), int(ints[e, c, 16]),
                         float(f[e, c, 12]), f[e, c, 0:3].copy(), f[e, c, 3:6].copy()) for c in range(n[e])])
        return out

    def musical_metrics(self):
        """-> (episode [N, 6] f32, episodes [N] i32): each env's last finished episode's mean
        precision / recall / F1 / sustain_precision / sustain_recall / sustain_f1
        (MidiEvaluationWrapper, wrappers/evaluation.py:114-177) and its finished-episode count."""
        torch = self._torch
        ep = torch.empty(self.num_envs, abi.NMUSIC, device=self.device)
        cnt = torch.empty(self.num_envs, device=self.device, dtype=torch.int32)
        _lib.check(_lib.load().ps_musical_metrics(self._h, ep.data_ptr(), cnt.data_ptr(), self.stream))
        return ep, cnt

    def warnings(self):
        """[N, 3] int32: each env's mj_checkPos / mj_checkVel / mj_checkAcc resets since create
        (ps_warnings). MuJoCo resets the data of a diverged env and raises the warning that
        dm_control turns into ``PhysicsError``; the kernel does the reset per env and counts."""
        t = self._torch.empty(self.num_envs, abi.NWARN, device=self.device, dtype=self._torch.int32)
        _lib.check(_lib.load().ps_warnings(self._h, t.data_ptr(), self.stream))
        return t

    def solver_stats(self):
        """[N, 7] int32 counters of each env's last step (PS_STAT_*): Newton iterations, substeps
        at the contact cap, substeps at the Newton iteration cap, most contact rows, substeps with
        the hands coupled, substeps with a non-positive Hessian pivot, most coupled dofs of both
        hands in a substep."""
        t = self._torch.empty(self.num_envs, abi.NSTATS, device=self.device, dtype=self._torch.int32)
        _lib.check(_lib.load().ps_solver_stats(self._h, t.data_ptr(), self.stream))
        return t

    def hand_offset(self):
        """-> (dy [N] f32, episodes [N] i32): randomize_hand_positions' y shift of both hands this
        episode (piano_with_shadow_hands.py:491-499) and each env's resets so far."""
        torch = self._torch
        dy = torch.empty(self.num_envs, device=self.device)
        ep = torch.empty(self.num_envs, device=self.device, dtype=torch.int32)
        _lib.check(_lib.load().ps_get_hand_offset(self._h, dy.data_ptr(), ep.data_ptr(), self.stream))
        return dy, ep

    def set_hand_offset(self, dy):
        t = self._torch.as_tensor(dy, device=self.device, dtype=self._torch.float32).contiguous()
        _lib.check(_lib.load().ps_set_hand_offset(self._h, t.data_ptr(), self.stream))
        self._dy = t

    def obs_dict(self, obs=None) -> Dict[str, Any]:
        obs = self.obs if obs is None else obs
        return {k: obs[:, s] for k, s in self.obs_slices.items()}

    # -- specs (dm_env)
    def observation_spec(self) -> Dict[str, Array]:
        return {k: Array((s.stop - s.start,), np.float64, k) for k, s in self.obs_slices.items()}

    def action_spec(self) -> BoundedArray:
        n = self.action_dim
        if self.canonical_actions:
            return BoundedArray((n,), np.float32, -np.ones(n, np.float32), np.ones(n, np.float32), "action")
        return BoundedArray((n,), np.float32, self.action_lo.astype(np.float32),
                            self.action_hi.astype(np.float32), "action")


# ---------------------------------------------------------------- reference surfaces
class _EnvView:
    """``vec_env.envs[i]``: per-env dm_env views (specs; reset/step of that slot)."""

    def __init__(self, parent: "VectorizedPianoEnv", i: int):
        self._p, self._i = parent, i

    def observation_spec(self):
        return self._p._core.observation_spec()

    def action_spec(self):
        return self._p._core.action_spec()


class VectorizedPianoEnv:
    """Drop-in for ``parallelized_base_v2.VectorizedPianoEnv`` (parallelized_base_v2.py:21-67).

    ``reset()`` returns ``{key: [N, d]}``; ``step(actions[N, 45])`` (canonical [-1, 1], as
    after the reference's per-env ``CanonicalSpecWrapper``) returns ``(obs, rewards, dones)``.
    With ``return_numpy=True`` the outputs are numpy arrays like the reference's; otherwise
    they are torch-ROCm tensors that never leave HBM. The task kwargs default to the ones
    the reference hard-codes (parallelized_base_v2.py:28-39).
    """

    def __init__(self, num_envs: int, midi_sequence, return_numpy: bool = False, device=None, seed: int = 0,
                 **task_kwargs):
        kw = dict(n_steps_lookahead=1, trim_silence=True, wrong_press_termination=False,
                  initial_buffer_time=0.0, disable_fingering_reward=False, disable_forearm_reward=False,
                  disable_colorization=False, disable_hand_collisions=False)
        kw.update(task_kwargs)
        self.num_envs = num_envs
        self._core = BatchedPianoEnv(num_envs, midi_sequence, TaskConfig(**kw), device=device, seed=seed)
        self.return_numpy = return_numpy
        self.envs = [_EnvView(self, i) for i in range(num_envs)]
        self.observation_spec = self._core.observation_spec()
        self.action_spec = self._core.action_spec()

    @property
    def core(self) -> BatchedPianoEnv:
        return self._core

    def _obs(self, obs):
        # The reference returns fresh arrays each call (parallelized_base_v2.py:60-67); the
        # core's obs / reward buffers are reused by the next step, so the torch mode returns a
        # copy (one [N, obs_dim] device copy per step) that a driver may keep across steps.
        if self.return_numpy:
            flat = obs.detach().cpu().numpy().astype(np.float64)
        else:
            flat = obs.clone()
        return {k: flat[:, s] for k, s in self._core.obs_slices.items()}

    def reset(self):
        return self._obs(self._core.reset())

    def step(self, actions):
        obs, rew, disc, st = self._core.step(actions)
        obs_d = self._obs(obs)
        dones = st == abi.LAST
        if self.return_numpy:
            return obs_d, rew.detach().cpu().numpy().astype(np.float64), dones.cpu().numpy()
        return obs_d, rew.clone(), dones


class PhysicsError(RuntimeError):
    """dm_control's ``control.PhysicsError``: the simulation diverged (MuJoCo's mj_checkPos /
    mj_checkVel / mj_checkAcc warning: a NaN or |x| > 1e10 qpos, qvel or qacc)."""


_WARN_NAMES = ("mjWARN_BADQPOS", "mjWARN_BADQVEL", "mjWARN_BADQACC")


class Environment:
    """Single-env dm_env facade (``composer_utils.Environment`` + ``CanonicalSpecWrapper``).

    Physics errors follow ``composer.Environment.step``: the kernel resets a diverged env's
    physics and counts the warning (ps_warnings); with ``raise_exception_on_physics_error``
    (composer's default, True) the step raises ``PhysicsError``, otherwise it logs the warning
    and ends the episode with reward 0 and discount 0, and the next step resets."""

    def __init__(self, midi, task: Optional[TaskConfig] = None, device=None, seed: int = 0,
                 raise_exception_on_physics_error: bool = True):
        self._core = BatchedPianoEnv(1, midi, task, device=device, seed=seed)
        self._raise = raise_exception_on_physics_error
        self._warn = np.zeros(abi.NWARN, np.int64)
        self._reset_next = False

    def _obs(self, obs):
        return {k: v[0].detach().cpu().numpy() for k, v in self._core.obs_dict(obs).items()}

    def reset(self) -> TimeStep:
        self._reset_next = False
        obs = self._core.reset()
        self._warn = self._core.warnings()[0].cpu().numpy().astype(np.int64)
        return TimeStep(StepType.FIRST, None, None, self._obs(obs))

    def step(self, action) -> TimeStep:
        if self._reset_next:
            return self.reset()
        a = self._core._torch.as_tensor(np.asarray(action, np.float32).reshape(1, -1), device=self._core.device)
        obs, rew, disc, st = self._core.step(a)
        o = self._obs(obs)
        w = self._core.warnings()[0].cpu().numpy().astype(np.int64)
        new = w - self._warn
        self._warn = w
        if new.any():
            msg = "Physics state is invalid. Warning(s) raised: " + ", ".join(
                n for n, c in zip(_WARN_NAMES, new) if c > 0)
            if self._raise:
                raise PhysicsError(msg)
            import logging
            logging.warning(msg)
            self._reset_next = True
            return TimeStep(StepType.LAST, 0.0, 0.0, o)
        t = StepType(int(st[0]))
        if t == StepType.FIRST:
            return TimeStep(t, None, None, o)
        return TimeStep(t, float(rew[0]), float(disc[0]), o)

    def observation_spec(self):
        return self._core.observation_spec()

    def action_spec(self):
        return self._core.action_spec()

    @property
    def core(self):
        return self._core


DEBUG = ["RoboPianist-debug-TwinkleTwinkleLittleStar-v0"]
_DEBUG_SONGS = {"RoboPianist-debug-TwinkleTwinkleLittleStar-v0": music.twinkle_twinkle_little_star_one_hand}


def song_for(environment_name: str, midi_file=None) -> music.NoteSequence:
    if midi_file is not None:
        return music.parse_midi(midi_file)
    if environment_name not in _DEBUG_SONGS:
        raise ValueError(f"Unknown environment {environment_name}. Available environments: {DEBUG}")
    return _DEBUG_SONGS[environment_name]()


def load(environment_name: str, midi_file=None, seed=None, task_kwargs=None, device=None) -> Environment:
    """``robopianist.suite.load`` (suite/__init__.py:50-93) for the debug songs / MIDI files."""
    return Environment(song_for(environment_name, midi_file), TaskConfig(**(task_kwargs or {})), device=device,
                       seed=0 if seed is None else int(seed))
