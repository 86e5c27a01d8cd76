"""Config 4's env miss term is pinned to the reference's OWN code.

tests/golden/env_kat.npz holds texels that texture.cpp:111-135 (the per-lane body of
EquirectangularTextureSample, with TexelFetch :6-14) returned when compiled from the reference's
line ranges (oracle/build_ref.sh -> oracle/_ref/ref_env; generator tests/golden/make_env_kat.py),
for index-coded textures of 7 shapes and ~9000 directions (poles, the +-x seam, quadrant edges,
asin's NaN above |y| = 1, denormals, both sides of column and row boundaries, random unit vectors).
The oracle's restatement (pto_env_sample) must return the same bits; the GPU env kernels are
checked bit-exact against that restatement (tests/test_gpu_env.py, tests/test_gpu_v4.py), so they
are pinned transitively.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

from oracle import pyoracle

GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLDEN))
from make_env_kat import index_texture  # noqa: E402


@pytest.fixture(scope="module")
def kat():
    return dict(np.load(GOLDEN / "env_kat.npz"))


def test_kat_covers_the_edges(kat):
    d = kat["dirs"]
    assert len(d) > 8000
    assert (np.abs(d[:, 1]) > 1).any()                               # asin NaN branch
    assert ((d[:, 0] == -1) & (d[:, 1] == 0) & (d[:, 2] == 0) & np.signbit(d[:, 2])).any()   # seam, -0
    e = kat["texels_2048x1024"]
    assert (~(e != 0).any(1)).sum() >= 2                             # the zero (out-of-range) branch
    cols = set(e[(e != 0).any(1), 1].astype(int).tolist())
    assert len(cols) > 1000 and 0 in cols and 2046 in cols


@pytest.mark.parametrize("shape", [(2048, 1024), (512, 256), (1, 1), (1, 9), (9, 1), (3, 5), (2, 2)])
def test_oracle_env_sample_matches_reference_kat(kat, shape):
    w, h = shape
    exp = kat[f"texels_{w}x{h}"]
    got = pyoracle.env_sample(index_texture(w, h), kat["dirs"])
    bad = np.nonzero((got.view(np.uint32) != exp.view(np.uint32)).any(1))[0]
    assert len(bad) == 0, (len(bad), kat["dirs"][bad[:5]].tolist(), got[bad[:5]].tolist(), exp[bad[:5]].tolist())


@pytest.mark.skipif(not pyoracle.ref_env_available(), reason="reference env build (oracle/_ref) not present")
def test_oracle_env_sample_matches_live_reference(tmp_path):
    """Random directions on a random (non-index) texture against a live run of the reference's lines."""
    rng = np.random.default_rng(7)
    tex = rng.lognormal(size=(37, 61, 3)).astype(np.float32)
    dirs = rng.normal(size=(20000, 3)).astype(np.float32)
    dirs[:100] *= np.float32(1e-38)                                   # denormal-range components
    ref = pyoracle.ref_env_sample(tex, dirs, tmp_path)
    got = pyoracle.env_sample(tex, dirs)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
