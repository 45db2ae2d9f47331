"""ctypes binding of libpianosim.so (the HIP product). No CPU fallback: if the library or
a GPU is missing, the calls that need them raise."""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("PIANOSIM_LIB", HERE / "libpianosim.so"))
RL_LIB_PATH = Path(os.environ.get("PIANORL_LIB", HERE / "libpianorl.so"))

# Every entry point declared in include/pianosim.h.
EXPORTS = (
    "ps_last_error", "ps_version", "ps_obs_dim", "ps_model_desc_size", "ps_create", "ps_destroy",
    "ps_reset", "ps_step", "ps_get_state", "ps_set_state", "ps_set_applied", "ps_reward_terms",
    "ps_fingertips", "ps_contact_count", "ps_musical_metrics", "ps_solver_stats", "ps_get_hand_offset",
    "ps_set_hand_offset", "ps_record_contacts", "ps_contacts", "ps_set_env_offset", "ps_warnings",
    "ps_env_obs_dim", "ps_env_action_dim", "ps_episode_returns",
)

# Every entry point declared in include/pianorl.h.
RL_EXPORTS = ("prl_last_error", "prl_version", "prl_running_norm", "prl_gae", "prl_normalize", "prl_gauss_sample",
              "prl_clip_adam", "prl_gather_minibatch", "prl_lnrelu_fwd", "prl_lnrelu_bwd", "prl_actor_head",
              "prl_critic_head", "prl_colsums", "prl_mlp_step_work", "prl_mlp_step", "prl_mlp_step_idx",
              "prl_mlp_step_norm_parts", "prl_mlp_step_idx_norm", "prl_clip_adam_parts")


class PrlLayer(C.Structure):  # prl_layer of include/pianorl.h
    _fields_ = [("in_", C.c_int), ("out", C.c_int), ("W", C.c_void_p), ("b", C.c_void_p), ("gamma", C.c_void_p),
                ("beta", C.c_void_p), ("dropout", C.c_float), ("dW", C.c_void_p), ("db", C.c_void_p),
                ("dgamma", C.c_void_p), ("dbeta", C.c_void_p)]


class PrlNet(C.Structure):  # prl_net
    _fields_ = [("nlayers", C.c_int), ("head", C.c_int), ("layer", PrlLayer * 4), ("log_std", C.c_void_p),
                ("dlog_std", C.c_void_p)]

_lib = None
_rl = None


class PianosimError(RuntimeError):
    pass


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise PianosimError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    vp, i32, u64 = C.c_void_p, C.c_int, C.c_uint64
    L.ps_last_error.restype = C.c_char_p
    L.ps_version.restype = i32
    L.ps_obs_dim.argtypes = [vp]
    L.ps_model_desc_size.restype = i32
    L.ps_create.argtypes = [vp, vp, vp, i32, i32, u64, C.POINTER(vp)]
    L.ps_destroy.argtypes = [vp]
    L.ps_reset.argtypes = [vp, vp, vp, vp]
    L.ps_step.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.ps_get_state.argtypes = [vp] * 9
    L.ps_set_state.argtypes = [vp] * 9
    L.ps_set_applied.argtypes = [vp, vp, vp]
    L.ps_reward_terms.argtypes = [vp, vp, vp]
    L.ps_fingertips.argtypes = [vp, vp, vp]
    L.ps_contact_count.argtypes = [vp, vp, vp]
    L.ps_musical_metrics.argtypes = [vp, vp, vp, vp]
    if hasattr(L, "ps_record_contacts"):
        L.ps_record_contacts.argtypes = [vp, i32]
    if hasattr(L, "ps_episode_returns"):
        L.ps_episode_returns.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
    if hasattr(L, "ps_set_env_offset"):
        L.ps_set_env_offset.argtypes = [vp, C.c_int64]
    for name, argc in (("ps_solver_stats", 3), ("ps_get_hand_offset", 4), ("ps_set_hand_offset", 3),
                       ("ps_contacts", 3), ("ps_warnings", 3), ("ps_env_obs_dim", 1), ("ps_env_action_dim", 1)):
        if hasattr(L, name):  # (absent from older builds loaded for A/B runs via PIANOSIM_LIB)
            getattr(L, name).argtypes = [vp] * argc
    for name in EXPORTS:
        if name not in ("ps_last_error", "ps_version", "ps_model_desc_size", "ps_destroy") and hasattr(L, name):
            getattr(L, name).restype = i32
    L.ps_destroy.restype = None
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = load().ps_last_error()
        raise PianosimError(msg.decode() if msg else f"pianosim error {rc}")


def load_rl() -> C.CDLL:
    """libpianorl.so: the on-device PPO kernels (include/pianorl.h)."""
    global _rl
    if _rl is not None:
        return _rl
    if not RL_LIB_PATH.exists():
        raise PianosimError(
            f"{RL_LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(str(RL_LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    vp, i32, u64, f32 = C.c_void_p, C.c_int, C.c_uint64, C.c_float
    L.prl_last_error.restype = C.c_char_p
    L.prl_version.restype = i32
    L.prl_running_norm.argtypes = [vp, i32, vp, vp, vp]
    L.prl_gae.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, i32, vp]
    L.prl_normalize.argtypes = [vp, i32, f32, vp]
    L.prl_gauss_sample.argtypes = [vp, vp, i32, i32, u64, u64, vp, vp, vp]
    L.prl_clip_adam.argtypes = [vp, vp, vp, vp, C.POINTER(C.c_int64), i32, vp, vp, f32, f32, f32, f32, vp, vp, vp]
    L.prl_gather_minibatch.argtypes = [vp, i32, vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
    L.prl_lnrelu_fwd.argtypes = [vp, vp, vp, vp, i32, i32, f32, f32, u64, vp, i32, vp, vp, vp, vp]
    L.prl_lnrelu_bwd.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, f32, u64, vp, i32, vp, vp, vp, vp]
    L.prl_actor_head.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, vp, vp, vp, vp, vp]
    L.prl_critic_head.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp]
    L.prl_colsums.argtypes = [i32, C.POINTER(vp), C.POINTER(i32), C.POINTER(f32), C.POINTER(vp), i32, vp, C.c_size_t,
                              vp]
    if hasattr(L, "prl_mlp_step"):
        L.prl_mlp_step_work.argtypes = [C.POINTER(PrlNet), i32, i32]
        L.prl_mlp_step.argtypes = [C.POINTER(PrlNet), vp, i32, vp, i32, vp, vp, vp, i32, f32, f32, f32, u64, vp, vp, vp,
                                   C.c_size_t, vp, vp]
        L.prl_mlp_step_idx.argtypes = [C.POINTER(PrlNet), vp, i32, vp, i32, vp, vp, vp, vp, i32, f32, f32, f32, u64, vp,
                                       vp, vp, C.c_size_t, vp, vp]
        L.prl_mlp_step_norm_parts.argtypes = [C.POINTER(PrlNet), i32, i32]
        L.prl_mlp_step_idx_norm.argtypes = [C.POINTER(PrlNet), vp, i32, vp, i32, vp, vp, vp, vp, i32, f32, f32, f32, u64,
                                            vp, vp, vp, C.c_size_t, vp, C.POINTER(C.c_int64), i32, vp, vp, i32, vp, vp]
        L.prl_clip_adam_parts.argtypes = [vp, vp, vp, vp, C.POINTER(C.c_int64), i32, vp, vp, f32, f32, f32, f32, vp, i32,
                                          vp, vp]
    for name in RL_EXPORTS[2:]:
        getattr(L, name).restype = i32
    if hasattr(L, "prl_mlp_step_work"):
        L.prl_mlp_step_work.restype = C.c_size_t
    _rl = L
    return L


SONG_LIB_PATH = Path(os.environ.get("PIANOSONG_LIB", HERE / "libpianosong.so"))
# Every entry point declared in include/pianosong.h.
SONG_EXPORTS = ("pss_last_error", "pss_version", "pss_parse_midi", "pss_from_notes", "pss_free", "pss_info",
                "pss_get", "pss_add_fingering", "pss_trim_silence", "pss_song_tables")
_song = None


def load_song() -> C.CDLL:
    """libpianosong.so: native MIDI / fingering ingestion (include/pianosong.h, host only)."""
    global _song
    if _song is not None:
        return _song
    if not SONG_LIB_PATH.exists():
        raise PianosimError(
            f"{SONG_LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(str(SONG_LIB_PATH))
    vp, i32, f64 = C.c_void_p, C.c_int, C.c_double
    L.pss_last_error.restype = C.c_char_p
    L.pss_version.restype = i32
    L.pss_parse_midi.argtypes = [vp, C.c_size_t, C.POINTER(vp)]
    L.pss_from_notes.argtypes = [vp, i32, vp, i32, f64, C.POINTER(vp)]
    L.pss_free.argtypes = [vp]
    L.pss_free.restype = None
    L.pss_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(f64), C.POINTER(i32)]
    L.pss_get.argtypes = [vp, vp, vp]
    L.pss_add_fingering.argtypes = [vp, C.c_char_p]
    L.pss_trim_silence.argtypes = [vp]
    L.pss_song_tables.argtypes = [vp, f64, f64, i32, i32, vp, vp, vp, vp, C.POINTER(i32)]
    for name in SONG_EXPORTS[2:]:
        if name != "pss_free":
            getattr(L, name).restype = i32
    _song = L
    return L


def check_rl(rc: int) -> None:
    if rc != 0:
        msg = load_rl().prl_last_error()
        raise PianosimError(msg.decode() if msg else f"pianorl error {rc}")
