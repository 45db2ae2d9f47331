"""The C-ABI library loads and exports every symbol include/pianosim.h declares (no GPU
calls), and the ctypes descriptor layout matches the C one."""
import ctypes as C
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_header_symbols_exported(dp):
    lib = __import__("importlib").import_module("diffusion-piano_amd._lib")
    L = lib.load()
    header = (ROOT / "include" / "pianosim.h").read_text()
    declared = set(re.findall(r"\b(ps_[a-z_]+)\s*\(", header))
    assert declared == set(lib.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_descriptor_layout(dp):
    L = __import__("importlib").import_module("diffusion-piano_amd._lib").load()
    assert L.ps_model_desc_size() == C.sizeof(dp.abi.ModelDesc)
    assert L.ps_version() >= 1
    for fing in (0, 1):
        for la in (0, 1, 3):
            cfg = dp.abi.TaskCfg(n_steps_lookahead=la, fingering_reward=fing)
            assert L.ps_obs_dim(C.byref(cfg)) == dp.abi.obs_dim(cfg)


def test_task_cfg_struct_size_is_checked(dp):
    """ps_task_cfg starts with its own size: a caller built against another layout
    of the header is refused by ps_obs_dim and by ps_create (before any device call) instead of
    the library reading past the end of its struct."""
    lib = __import__("importlib").import_module("diffusion-piano_amd._lib")
    L = lib.load()
    assert L.ps_version() >= 4
    good = dp.abi.TaskCfg(n_steps_lookahead=1)
    assert good.struct_size == C.sizeof(dp.abi.TaskCfg)
    for size in (0, C.sizeof(dp.abi.TaskCfg) - 4, 1):  # 1: an old caller's n_steps_lookahead there
        bad = dp.abi.TaskCfg(n_steps_lookahead=1, struct_size=size)
        assert L.ps_obs_dim(C.byref(bad)) < 0
        assert b"rebuild" in L.ps_last_error()
        out = C.c_void_p()
        rc = L.ps_create(None, None, C.byref(bad), 4, 0, 0, C.byref(out))
        assert rc < 0
    md, st, tc = dp.compile_task(dp.music.test_midi(0.05), dp.TaskConfig())
    sd = dp.abi.SongDesc.from_tables(st)
    tc.struct_size = 8
    out = C.c_void_p()
    assert L.ps_create(C.addressof(md), C.addressof(sd), C.addressof(tc), 4, 0, 0, C.byref(out)) < 0
    assert b"rebuild" in L.ps_last_error()


def test_product_has_no_oracle_dependency():
    """The product package never references the oracle."""
    for p in (ROOT / "diffusion-piano_amd").rglob("*"):
        if p.suffix in (".py", ".hip", ".h", ".cpp"):
            txt = p.read_text()
            assert "oracle" not in txt.replace("oracle/pianosim_ref.c", ""), p
