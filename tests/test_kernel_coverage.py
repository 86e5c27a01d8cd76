"""Every kernel the library's code objects hold is launched by the -m gpu suite.

The compiled set comes from libpt_mi355.so's .hip_fatbin (kernel descriptors `*.kd`, demangled); the
launched set from the suite run under rocprofv3 --kernel-trace (scripts/gpu_coverage.sh), committed
as profiles/r06/*_kernels_launched.txt (the newest file).  tests/test_gpu_instances.py is the matrix
that reaches the instances no other test does.  CPU only: it reads the committed trace."""
from __future__ import annotations

import re
import subprocess
import tempfile
from pathlib import Path

import pytest

import isa_lgkm as I

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "cpuperformanceraytracer_amd" / "libpt_mi355.so"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def compiled_kernels(lib: Path) -> set[str]:
    names = set()
    for _name, co in I.code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            out = subprocess.run([READELF, "-s", "-W", f.name], check=True, capture_output=True, text=True).stdout
        for line in out.splitlines():
            parts = line.split()
            if parts and parts[-1].endswith(".kd"):
                names.add(parts[-1][:-3])
    dem = subprocess.run(["c++filt"], input="\n".join(sorted(names)), check=True, capture_output=True,
                         text=True).stdout.splitlines()
    return {d.strip() for d in dem if d.strip()}


def launched_kernels() -> tuple[Path, set[str]]:
    files = sorted((ROOT / "profiles" / "r06").glob("*_kernels_launched.txt"))
    if not files:
        pytest.skip("no committed kernel trace of the -m gpu suite")
    f = files[-1]
    return f, {ln.strip() for ln in f.read_text().splitlines() if ln.strip()}


@pytest.mark.skipif(not Path(READELF).exists(), reason="ROCm llvm-readelf not available")
def test_every_compiled_kernel_is_launched_by_the_gpu_suite():
    if not LIB.exists():
        pytest.skip("libpt_mi355.so not built")
    compiled = compiled_kernels(LIB)
    assert len(compiled) >= 50
    f, launched = launched_kernels()
    missing = sorted(compiled - launched)
    assert not missing, f"{len(missing)} of {len(compiled)} kernels never launched in {f.name}: {missing[:10]}"
