"""The oracle restatements and the host-side checkers under AddressSanitizer + UBSan (SURVEY.md
section 5: the reference's own tooling is none; the CPU restatement is the place sanitizers apply --
GPU sanitizers are not available on this pool).

* tests/native/sanitize_driver.c + oracle/pt_oracle.c, pt_oracle_output.c, pt_oracle_v4.c built with
  -fsanitize=address,undefined -fno-sanitize-recover=all: the scalar path (threads, row shards, env
  term), the counted path, the output stage and the v4 renderer (equirect and cubemap, counted) run
  clean, and every result is byte-identical to the normal build's (pyoracle).
* the product's host code that parses untrusted input -- the Radiance RGBE decoder of
  csrc/pt_texture.cpp (LoadTexture, asset_loading.cpp:9-16) -- under the same sanitizers on valid
  files of every encoding and on truncated / corrupt ones.
* the host checkers of the kernels' certified stages (check_quadcull, check_sky, check_scene) built
  with the sanitizers, on reduced workloads.
"""
from __future__ import annotations

import shutil
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from oracle import pyoracle

ROOT = Path(__file__).resolve().parents[1]
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=86", "UBSAN_OPTIONS": "print_stacktrace=1"}


def _cc(name):
    exe = shutil.which(name)
    if not exe:
        pytest.skip(f"no {name}")
    return exe


def _run(cmd, timeout=600):
    import os
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env={**os.environ, **ENV})
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    return r


def test_oracle_under_asan_ubsan(tmp_path):
    gcc = _cc("gcc")
    exe = tmp_path / "sanitize_driver"
    o = ROOT / "oracle"
    subprocess.run([gcc, "-std=c11", *SAN, "-ffp-contract=off", "-fno-fast-math", f"-I{o}",
                    str(ROOT / "tests/native/sanitize_driver.c"), str(o / "pt_oracle.c"), str(o / "pt_oracle_output.c"),
                    str(o / "pt_oracle_v4.c"), "-lm", "-lpthread", "-o", str(exe)], check=True)
    out = tmp_path / "out.bin"
    _run([str(exe), str(out)])
    got = out.read_bytes()
    # the same results from the normal build
    W, H = 48, 32
    tex = np.empty(24 * 12 * 3, np.float32)
    lcg = 12345
    for i in range(tex.size):
        lcg = (lcg * 1664525 + 1013904223) & 0xFFFFFFFF
        tex[i] = np.float32(0.01) + np.float32(lcg >> 8) * np.float32(3.0 / 16777216.0)
    env = tex.reshape(12, 24, 3)
    parts = [pyoracle.render(W, H, frame_first=5, nframes=3, num_bounces=8, nthreads=4).tobytes(),
             pyoracle.render(W, H, frame_first=1, nframes=2, num_bounces=4, row_start=1, row_stride=2, nrows=H // 2,
                             env=env, nthreads=3).tobytes()]
    img, c = pyoracle.render_counted(W, H, frame_first=1, nframes=2, num_bounces=8)
    parts.append(img.tobytes())
    cut = sum(len(p) for p in parts)
    assert got[:cut] == b"".join(parts)
    counts = struct.unpack("<9Q", got[cut:cut + 72])
    assert counts[0] == c["samples"] and counts[1] == c["segments"] and counts[5] == c["escaped"]
    cut += 72
    rgba = pyoracle.tonemap(img, pyoracle.PIXEL_RGBA8)
    assert got[cut:cut + W * H * 4] == np.ascontiguousarray(rgba, np.uint32).tobytes()
    cut += 2 * W * H * 4
    v4 = pyoracle.render4(W, H, frame_first=1, nframes=2, num_bounces=8, env=env, nthreads=2)
    assert got[cut:cut + W * H * 12] == v4.tobytes()
    cut += W * H * 12
    cube = tex[: 2 * 12 * 3].copy().reshape(12, 2, 3)
    v4c = pyoracle.render4(W, H, frame_first=3, nframes=2, num_bounces=4, env=cube, env_mode=pyoracle.ENV_CUBEMAP,
                           random_jitter=False, rejection=False, nthreads=1, fast_exp=False)
    assert got[cut:cut + W * H * 12] == v4c.tobytes()


def _hdr_files(tmp_path):
    """Radiance files: flat, new-RLE, truncated, corrupt header, absurd size."""
    w, h = 20, 6
    rng = np.random.default_rng(3)
    px = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    px[..., 3] = rng.integers(120, 140, (h, w))
    hdr = f"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y {h} +X {w}\n".encode()
    flat = hdr + px.tobytes()
    rle_rows = b""
    for y in range(h):   # new RLE: 2, 2, w>>8, w&255, then each channel as literal runs of <= 128
        rle_rows += bytes([2, 2, w >> 8, w & 255])
        for ch in range(4):
            rle_rows += bytes([w]) + px[y, :, ch].tobytes()
    rle = hdr + rle_rows
    files = {"flat": flat, "rle": rle, "trunc_flat": flat[:-7], "trunc_rle": rle[: len(rle) // 2],
             "bad_header": b"#?RADIANCE\nFORMAT=garbage\n\n-Y 4 +X 4\n" + bytes(64),
             "huge": b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 99999999 +X 99999999\n" + bytes(16),
             "bad_run": hdr + bytes([2, 2, 0, w, 200, 1]) + bytes(32)}
    paths = []
    for k, v in files.items():
        p = tmp_path / f"{k}.hdr"
        p.write_bytes(v)
        paths.append(p)
    return paths


def test_rgbe_decoder_under_asan_ubsan(tmp_path):
    """csrc/pt_texture.cpp (the product's RGBE decoder, host code) on valid and malformed files."""
    gxx = _cc("g++")
    drv = tmp_path / "hdr_driver.cpp"
    drv.write_text(r'''
#include <cstdio>
#include "pt_mi355.h"
int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        pt_texture t{};
        int rc = pt_load_texture(argv[i], &t);
        double s = 0;
        if (rc == 0) for (long k = 0; k < (long)t.width * t.height * 3; ++k) s += t.data[k];
        std::printf("%s %d %d %d %.9g\n", argv[i], rc, t.width, t.height, s);
        pt_free_texture(&t);
    }
    return 0;
}
// the decoder's only dependency on the rest of the library (pt_capi.cpp): the error message
#include <cstdarg>
int pt_internal_fail(int code, const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); std::vfprintf(stderr, fmt, ap); va_end(ap); std::fputc('\n', stderr);
    return code;
}
''')
    exe = tmp_path / "hdr_driver"
    csrc = ROOT / "cpuperformanceraytracer_amd" / "csrc"
    r = subprocess.run([gxx, "-std=c++17", *SAN, f"-I{ROOT / 'include'}", f"-I{csrc}",
                        str(drv), str(csrc / "pt_texture.cpp"), "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("pt_texture.cpp does not build standalone: " + r.stderr[-2000:])
    files = _hdr_files(tmp_path)
    out = _run([str(exe), *map(str, files)]).stdout.splitlines()
    res = {Path(ln.split()[0]).stem: ln.split()[1:] for ln in out}
    assert res["flat"][0] == "0" and res["rle"][0] == "0" and res["flat"][1:3] == ["20", "6"]
    assert res["flat"][3] == res["rle"][3]                     # both encodings decode to the same texels
    for bad in ("trunc_flat", "trunc_rle", "bad_header", "huge", "bad_run"):
        assert res[bad][0] != "0", bad                            # rejected, without a sanitizer report


@pytest.mark.parametrize("checker,args", [("check_scene", []), ("check_sky", []),
                                          ("check_quadcull", ["3000", "11"])])
def test_host_checkers_under_asan_ubsan(tmp_path, checker, args):
    gxx = _cc("g++")
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s", "liboracle.so"], check=True)
    exe = tmp_path / checker
    o = ROOT / "oracle"
    srcs = [str(ROOT / "tests/native" / f"{checker}.cpp")]
    if checker == "check_scene":   # the product's host scene builder (csrc/pt_scene.cpp)
        srcs.append(str(ROOT / "cpuperformanceraytracer_amd" / "csrc" / "pt_scene.cpp"))
    link = []
    if checker != "check_scene":
        link = [str(o / "pt_oracle.c"), str(o / "pt_oracle_output.c"), str(o / "pt_oracle_v4.c")]
    cmd = [gxx, "-std=c++17", *SAN, "-ffp-contract=off", "-Wno-unknown-pragmas", f"-I{ROOT / 'include'}",
           f"-I{ROOT / 'cpuperformanceraytracer_amd' / 'csrc'}", f"-I{o}", *srcs]
    objs = []
    for c in link:   # C sources of the oracle, compiled as C
        obj = tmp_path / (Path(c).stem + ".o")
        subprocess.run(["gcc", "-std=c11", *SAN, "-ffp-contract=off", "-fno-fast-math", f"-I{o}", "-c", c, "-o",
                        str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run(cmd + objs + ["-lm", "-lpthread", "-o", str(exe)], check=True)
    _run([str(exe), *args], timeout=900)
