"""The CPU oracle reproduces the committed golden fixtures exactly (regression pin).

GPU parity against the same fixtures is in tests/test_gpu_parity.py.
"""
import os

import numpy as np
import pytest

import oracle
from golden_cases import boxes_of, chain_files, contour_cases, load_chain, origins_of


def test_fixtures_present():
    names = {os.path.basename(p) for p in chain_files()}
    assert len(names) >= 5, names


@pytest.mark.parametrize("path", chain_files(), ids=lambda p: os.path.basename(p))
def test_oracle_reproduces_chain_fixture(path):
    c = load_chain(path)
    cfg = oracle.OracleConfig(H=c["H"], W=c["W"], box=c["box"], ksize=c["ksize"], thresh=c["thresh"], alpha=c["alpha"])
    st = oracle.OracleStream(cfg, c["keep"] if c["has_keep"] else None)
    for t in range(c["T"]):
        r = st.step(c["frames"][t])
        for plane in ("gray", "blur", "delta", "mask"):
            np.testing.assert_array_equal(r[plane], c[plane][t], err_msg=f"{plane} frame {t}")
        assert r["count"] == c["count"][t]
        assert r["boxes"] == boxes_of(c, t)
        assert r["origins"] == origins_of(c, t)
    np.testing.assert_array_equal(st.bg, c["bg"])


def test_chain_fixtures_exercise_motion():
    total = sum(int(load_chain(p)["count"].sum()) for p in chain_files())
    assert total > 10  # the fixtures are not all-quiet


@pytest.mark.parametrize("name", sorted(contour_cases()))
def test_oracle_reproduces_contour_fixture(name):
    case = contour_cases()[name]
    cs = oracle.find_contours_ext(case["mask"])
    assert [c["bbox"] for c in cs] == case["boxes"]
    assert [c["origin"] for c in cs] == case["origins"]
    np.testing.assert_array_equal(np.array([c["area"] for c in cs]), case["areas"])
