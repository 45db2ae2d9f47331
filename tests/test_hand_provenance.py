"""The authored hand against its provenance table.

diffusion-piano_amd/hand_provenance.json lists every quantity of model.authored_hand() with its
public source (Menagerie right_hand.xml element, the reference's shadow_hand.py / tasks/base.py
line, or a documented deviation). These tests fail when the hand drifts from the table, and pin
the rows whose source is in the reference against the reference's constants."""
import importlib.util
import json
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
TABLE = ROOT / "diffusion-piano_amd" / "hand_provenance.json"


@pytest.fixture(scope="module")
def table():
    return json.loads(TABLE.read_text())


@pytest.fixture(scope="module")
def fresh():
    spec = importlib.util.spec_from_file_location("mkprov", ROOT / "tools" / "make_hand_provenance.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.table()


def _close(a, b):
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_close(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)) and a and isinstance(a[0], str):
        return list(a) == list(b)
    if a is None or isinstance(a, str):
        return a == b
    return np.allclose(np.asarray(a, float), np.asarray(b, float), rtol=0, atol=1e-12)


def test_authored_hand_matches_the_table(table, fresh):
    assert fresh["counts"] == table["counts"]
    assert [r["quantity"] for r in fresh["rows"]] == [r["quantity"] for r in table["rows"]]
    bad = [r["quantity"] for r, t in zip(fresh["rows"], table["rows"]) if not _close(r["value"], t["value"])]
    assert not bad, bad[:10]


def test_every_row_has_a_source(table):
    for r in table["rows"]:
        assert r["status"] in ("transcribed", "verifiable", "deviation", "assumed"), r
        assert r["source"], r
        assert (r["status"] == "deviation") == r["source"].startswith("DEV"), r
        assert (r["status"] == "assumed") == r["source"].startswith("ASSUMED"), r
    assert table["counts"] == {"bodies": 25, "dofs": 26, "actuators": 22, "tendons": 4,
                               "colliders": 20, "sites": 5}


def _row(table, q):
    (r,) = [r for r in table["rows"] if r["quantity"] == q]
    return r["value"]


def test_reference_side_rows(table):
    """Rows whose source is the reference itself, against its constants."""
    # shadow_hand.py:81-82 fingertip / thumb-tip site offsets along the distal z
    tips = [r["value"] for r in table["rows"] if r["quantity"].startswith("fingertip site")]
    assert len(tips) == 5  # shadow_hand_constants FINGERTIP_BODIES: th, ff, mf, rf, lf
    np.testing.assert_allclose(tips[0], [0, 0, 0.0275], atol=1e-12)
    for p in tips[1:]:
        np.testing.assert_allclose(p, [0, 0, 0.026], atol=1e-12)
    # shadow_hand.py:41-52 _FOREARM_DOFS: forearm_tx slides along -x, forearm_ty along +z, 0..0.06
    np.testing.assert_allclose(_row(table, "joint forearm_tx axis"), [-1, 0, 0])
    np.testing.assert_allclose(_row(table, "joint forearm_ty axis"), [0, 0, 1])
    np.testing.assert_allclose(_row(table, "joint forearm_ty range"), [0.0, 0.06])
    # shadow_hand.py:303-309 forearm position actuators: kp = stiffness 300, ctrlrange = range
    acts = [r for r in table["rows"] if r["quantity"].startswith("actuator") and "forearm" in r["quantity"]]
    kps = [r["value"] for r in acts if r["quantity"].endswith(" kp")]
    assert kps == [300.0, 300.0]
    # 20 Menagerie actuators + 2 forearm actuators (shadow_hand_constants NU = 20)
    assert table["counts"]["actuators"] - 2 == 20
    # NQ = 24 hand joints + 2 forearm slides
    assert table["counts"]["dofs"] - 2 == 24


def test_deviations_are_the_documented_ones(table):
    dev = [r for r in table["rows"] if r["status"] == "deviation"]
    kinds = {r["quantity"].split()[0] for r in dev}
    assert kinds == {"collider"}  # the capsule colliders (frictionloss is modelled since round 3)
    design = (ROOT / "DESIGN.md").read_text()
    assert "hand_provenance.json" in design


def test_frictionloss_is_modelled(table):
    """the 26 joint frictionloss rows are transcribed (modelled), no longer
    deviations; the only deviations left are the capsule colliders."""
    fl = [r for r in table["rows"] if r["quantity"].endswith(" frictionloss")]
    assert len(fl) == 26 and all(r["status"] == "transcribed" and r["value"] == 0.01 for r in fl)
    dev = [r for r in table["rows"] if r["status"] == "deviation"]
    assert len(dev) == 20 and all(r["quantity"].startswith("collider ") for r in dev)
