"""LDS return hazards in the built gfx950 code (no GPU needed): every kernel of libpt_mi355.so is
checked by the CFG data-flow of tests/isa_lgkm.py -- no instruction reads or overwrites a VGPR an
LDS read will still write.  VERDICT r05 "What's weak" 1: quads_exact's inline-asm ds_read_b128
with its s_waitcnt in a separate asm statement (removed this round; pt_kernel.hip quads_exact).
The checker itself is validated on a fixture kernel with exactly that shape."""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

import isa_lgkm as I

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "cpuperformanceraytracer_amd" / "csrc"
LIB = ROOT / "cpuperformanceraytracer_amd" / "libpt_mi355.so"

needs_rocm = pytest.mark.skipif(not Path(I.OBJDUMP).exists() or not (shutil.which("hipcc") or
                                                                    Path("/opt/rocm/bin/hipcc").exists()),
                                reason="ROCm llvm tools / hipcc not available")


@needs_rocm
def test_checker_flags_the_split_asm_wait(tmp_path):
    out = tmp_path / "fx.co"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output",
                    "-O3", "-c", str(ROOT / "tests" / "native" / "lds_hazard_fixture.hip"), "-o", str(out)],
                   check=True, capture_output=True, timeout=300)
    bad = I.hazards(out.read_bytes())["hazards"]
    assert any("split_wait" in k for k in bad), bad
    assert not any("fused_wait" in k for k in bad), bad
    h = next(v for k, v in bad.items() if "split_wait" in k)[0]
    assert h["lds_op_at"] < h["at"]


@needs_rocm
def test_library_kernels_have_no_lds_return_hazard():
    if not LIB.exists():
        pytest.skip("libpt_mi355.so not built")
    cos = I.code_objects(LIB)
    assert len(cos) >= 3                       # pt_kernel.hip, pt_output.hip, pt_v4.hip
    total_f = total_r = 0
    for name, co in cos:
        r = I.hazards(co)
        bad = {k: v[:3] for k, v in r["hazards"].items()}
        assert not bad, (name, bad)
        total_f += r["functions"]
        total_r += r["lds_reads"]
    assert total_f >= 100 and total_r >= 5000   # (the checker saw the kernels: ~160 functions, ~9000 LDS reads)


def test_no_inline_asm_touches_lds_or_waits():
    """The product's remaining inline asm is single self-contained VALU moves (pt_kernel.hip
    vgpr_here, pt_sincosf.h's f64 constants): no LDS/memory access and no register-carrying
    s_waitcnt in any asm.  One exception, by form: pt_chain.h's publish waits for the wave's own
    pixel stores with a standalone `asm volatile("s_waitcnt vmcnt(0)" ::: "memory")` -- no operands
    (so no value can be read early), a memory clobber (the compiler keeps the stores before it and
    the epoch store after it) -- the form MI355X_MICROARCH.md prescribes between stores and a flag."""
    seen = 0
    for f in list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + list(CSRC.glob("*.cpp")):
        text = f.read_text()
        for m in re.finditer(r"asm\s+volatile\s*\(\s*\"([^\"]*)\"([^;]*);", text):
            seen += 1
            body, rest = m.group(1), m.group(2)
            if body == "s_waitcnt vmcnt(0)":
                assert f.name == "pt_chain.h" and re.fullmatch(r"\s*:::\s*\"memory\"\s*\)\s*", rest), (f.name, rest)
                continue
            assert not re.search(r"\b(ds_|s_waitcnt|buffer_|global_|flat_|scratch_|s_load|s_store)", body), (f.name, body)
            assert body.startswith("v_mov_b32"), (f.name, body)
    assert seen >= 1


def test_accumulator_buffer_accesses_are_whole_pixels():
    """pt_chain.h's 96-bit sc1 buffer accesses of the accumulator: every buffer load / store in the
    built library is a dwordx3 of the continuous-tiles pools (one 12-byte pixel).  An element-wise
    bit cast of the intrinsic's u32 vector once made the compiler shrink the load to its first dword
    (the other two channels then undefined) -- this catches that form."""
    if not LIB.exists():
        pytest.skip("libpt_mi355.so not built")
    n = 0
    for name, co in I.code_objects(LIB):
        for f, ins in I.parse_functions(I.disassemble(co)).items():
            for _, mn, ops, _ in ins:
                if mn.startswith("buffer_"):
                    n += 1
                    assert mn in ("buffer_load_dwordx3", "buffer_store_dwordx3") and "sc1" in ops and "_ct_" in f, (f, mn, ops)
    assert n >= 20
