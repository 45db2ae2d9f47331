import importlib
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libpianosim.so")


@pytest.fixture(scope="session")
def dp():
    return importlib.import_module("diffusion-piano_amd")


@pytest.fixture(scope="session")
def ref():
    import ref as _ref  # oracle/ref.py (test infrastructure)
    _ref.build()
    return _ref


@pytest.fixture(scope="session")
def golden():
    import json
    d = ROOT / "tests" / "golden"
    return {p.stem: json.loads(p.read_text()) for p in d.glob("*.json")}
