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


def test_product_has_no_oracle_dependency():
    """The product package never references the oracle."""
    for p in (ROOT / "diffusion-piano_amd").rglob("*"):
        if p.suffix in (".py", ".hip", ".h", ".cpp"):
            txt = p.read_text()
            assert "oracle" not in txt.replace("oracle/pianosim_ref.c", ""), p
