"""The diffuse kernel's culled quad stage (csrc/pt_quadcull.h) against the oracle's exact quad
stage (the six TestQuadTrace calls, demofox_path_tracing_scalar.cpp:192-261), on the host: the
header is compiled for the CPU with the same f32 operations (-ffp-contract=off) and checked by
tests/native/check_quadcull.cpp on realistic path segments (the oracle's own paths) and on
adversarial rays -- quad edges and corners, grazing directions, origins next to a quad, camera
rays.  Every certified result must equal the oracle's (quad, distance bits, flip); every per-quad
classification must be consistent with the exact test; and on realistic paths the uncertain
fraction (rays that fall back to the six exact tests) must stay negligible.  The GPU parity tests
check the kernel that uses it, bit for bit, on whole images."""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    lib = ROOT / "oracle" / "liboracle.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s", "liboracle.so"], check=True)
    exe = tmp_path_factory.mktemp("quadcull") / "check_quadcull"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", "-Wno-unknown-pragmas",
                    str(ROOT / "tests/native/check_quadcull.cpp"), "-o", str(exe), f"-L{ROOT / 'oracle'}",
                    "-loracle", f"-Wl,-rpath,{ROOT / 'oracle'}", "-lm"], check=True)
    return exe


def test_quadcull_certified_results_equal_oracle(checker):
    out = subprocess.run([str(checker), "150000", "0x9e3779b97f4a7c15"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "violations 0" in out.stdout
    # realistic paths: the six exact tests run for well under 0.1 % of the segments
    m = re.search(r"paths 240x135 x4f x8b\s+rays\s+(\d+)\s+uncertain\s+(\d+)", out.stdout)
    assert m, out.stdout
    rays, unc = int(m.group(1)), int(m.group(2))
    assert rays > 250_000 and unc / rays < 1e-3, out.stdout
    # the observed errors stay far inside the bounds the classification assumes
    m = re.search(r"max \|dist-s\|/delta ([0-9.e+-]+)\s+max \|T'-T\|/E_T\(theory 9.6e-4\) ([0-9.e+-]+)", out.stdout)
    assert m and float(m.group(1)) < 0.5 and float(m.group(2)) < 0.5, out.stdout


def test_quadcull_second_seed(checker):
    out = subprocess.run([str(checker), "150000", "7"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0 and "violations 0" in out.stdout, out.stdout[-3000:]
