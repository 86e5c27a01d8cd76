"""The oracle (oracle/pt_oracle.c) is pinned to the reference before it is trusted as a checker.

  * bit-identical to the golden fixtures, which the reference's own scalar code produced
    (tests/golden/make_golden.py via oracle/build_ref.sh);
  * the reference's Wang-hash known answers;
  * when the reference is present (this container), bit-identical to a live run of it;
  * its generalisations (row shards, frame offsets, multi-frame batches, bounce count) reduce to
    the reference's call pattern.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN_B4, GOLDEN_B8, bits_equal, load_golden, mismatch_report
from oracle import pyoracle


@pytest.mark.parametrize("name", GOLDEN_B4 + GOLDEN_B8)
def test_oracle_matches_reference_golden(manifest, name):
    """Every golden: B = 4 (the reference as shipped) and B = 8 (the reference with only
    c_numBounces = 8, its own `//8`; configs[1]-[4]'s bounce count), incl. the 1080p row sample."""
    c = manifest["cases"][name]
    rows = c.get("rows")
    kw = {}
    if rows:
        kw = dict(row_start=rows["start"], row_stride=rows["stride"], nrows=rows["count"])
    img = pyoracle.render(c["width"], c["height"], frame_first=c["frame_first"], nframes=c["frames"],
                          num_bounces=c["num_bounces"], **kw)
    g = load_golden(name)
    assert bits_equal(img, g), mismatch_report(img, g)


def test_b8_goldens_come_from_a_one_line_change(manifest):
    """The B = 8 fixtures' generator differs from the reference file in line 19 only."""
    p = manifest["b8_patch"]
    assert p["line"] == 19 and p["file"] == "demofox_path_tracing_scalar.cpp"
    assert p["diff"].splitlines() == ["19c19", "< const int c_numBounces = 4; //8", "---",
                                      "> const int c_numBounces = 8; //8"]
    for n in GOLDEN_B8:
        assert manifest["cases"][n]["num_bounces"] == 8
    # and B = 8 is not B = 4: the fixtures differ from the 4-bounce image of the same size
    g5 = load_golden("g5_256x256_f8_b8")
    assert not bits_equal(g5, load_golden("g2_256x256_f8"))


def test_golden_integrity(manifest):
    import hashlib
    for name, c in manifest["cases"].items():
        g = load_golden(name)
        assert hashlib.sha256(g.astype("<f4").tobytes()).hexdigest() == c["sha256"], name
        assert np.isfinite(g).all()


def test_golden_known_pixels():
    """SURVEY.md §8c sample pixels of G1 (row, col): (0,0) is the 1/2-weighted ambient 0.05."""
    g = load_golden("g1_256x256_f1")
    assert np.all(g[0, 0] == np.float32(0.05))
    assert g.max() <= 10.05 + 1e-6


def test_wang_hash_kats(manifest):
    for seed, seq in manifest["kat_wang_hash"].items():
        assert pyoracle.wang_hash_sequence(int(seed), len(seq)) == seq


def test_seed_formula(manifest):
    k = manifest["kat_seed"]
    assert pyoracle.seed(k["x"], k["y"], k["frame"]) == k["seed"]
    # wrapping u32 arithmetic at large coordinates / frames
    assert pyoracle.seed(7679, 4319, 16_000_000) == ((7679 * 1973 + 4319 * 9277 + 16_000_000 * 26699) & 0xFFFFFFFF) | 1


def test_random_unit_vectors_are_unit():
    v = pyoracle.random_unit_vector(12345, 1000).astype(np.float64)
    assert np.allclose(np.linalg.norm(v, axis=1), 1.0, atol=1e-6)


@pytest.mark.skipif(not pyoracle.ref_available(), reason="reference build (oracle/_ref) not present")
@pytest.mark.parametrize("w,h,frames", [(96, 64, 2), (17, 33, 3)])
def test_oracle_matches_live_reference(tmp_path, w, h, frames):
    ref = pyoracle.ref_render(w, h, frames, tmp_path)
    img = pyoracle.render(w, h, nframes=frames, num_bounces=4)
    assert bits_equal(img, ref), mismatch_report(img, ref)


@pytest.mark.skipif(not pyoracle.ref_available(8), reason="reference B=8 build (oracle/_ref) not present")
@pytest.mark.parametrize("w,h,frames", [(96, 64, 2), (17, 33, 3), (40, 24, 49)])
def test_oracle_matches_live_reference_b8(tmp_path, w, h, frames):
    ref = pyoracle.ref_render(w, h, frames, tmp_path, num_bounces=8)
    img = pyoracle.render(w, h, nframes=frames, num_bounces=8)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_row_shards_are_bit_identical_to_full_image():
    w, h, f, b = 120, 77, 2, 8
    full = pyoracle.render(w, h, nframes=f, num_bounces=b)
    for G in (2, 3, 8):
        for r in range(G):
            n = len(range(r, h, G))
            part = pyoracle.render(w, h, nframes=f, num_bounces=b, row_start=r, row_stride=G, nrows=n)
            assert bits_equal(part, full[r::G])


def test_frame_batches_compose():
    """frames 1..5 in one call == 1..2 then 3..5 on the same buffer (the lerp chain)."""
    w, h = 64, 40
    one = pyoracle.render(w, h, frame_first=1, nframes=5, num_bounces=8)
    two = pyoracle.render(w, h, frame_first=1, nframes=2, num_bounces=8)
    two = pyoracle.render(w, h, frame_first=3, nframes=3, num_bounces=8, buf=two)
    assert bits_equal(one, two)


def test_thread_count_does_not_change_result():
    a = pyoracle.render(100, 60, nframes=2, num_bounces=8, nthreads=1)
    b = pyoracle.render(100, 60, nframes=2, num_bounces=8, nthreads=7)
    assert bits_equal(a, b)


def test_zero_bounces_and_empty():
    img = pyoracle.render(32, 16, nframes=1, num_bounces=0)
    assert np.isfinite(img).all()
    empty = pyoracle.render(32, 16, nframes=0, num_bounces=4)
    assert not empty.any()
    with pytest.raises(ValueError):
        pyoracle.render(32, 16, frame_first=0)


def test_tonemap_oracle_properties():
    """The output-stage restatement (oracle/pt_oracle_output.c, v4 :144-187, :1260-1331): 0 -> 0,
    monotone over the displayable range, saturating at 255, 8-bit packing of both formats."""
    from oracle import pyoracle as po
    xs = np.concatenate([[0.0], np.geomspace(1e-6, 20.0, 4000)]).astype(np.float32)
    v = np.array([po.tonemap_channel(x) for x in xs])
    assert v[0] == 0 and v[-1] == 255
    assert (np.diff(v) >= 0).all()
    assert po.tonemap_channel(1.0) == 232 and po.tonemap_channel(0.1) == 99   # KATs of this restatement
    rgb = np.array([[[1.0, 0.1, 0.0]]], np.float32)
    assert po.tonemap(rgb, po.PIXEL_RGBA8)[0, 0] == 0xFF000000 | (0 << 16) | (99 << 8) | 232
    assert po.tonemap(rgb, po.PIXEL_XRGB8)[0, 0] == (232 << 16) | (99 << 8) | 0
