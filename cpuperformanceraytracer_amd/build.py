"""Build the native libraries in-tree (they travel to the GPU box with the repo snapshot).

  libpt_mi355.so  -- the product: HIP kernels for gfx950 + the C ABI (include/pt_mi355.h) + the
                     reference-named C++ entry points (include/demofox_path_tracing_mi355.h).

Compile flags that carry the parity contract (DESIGN.md "Numerics"):
  -ffp-contract=off                           no a*b+c fusion (the reference's MSVC /fp:precise)
  -fhip-fp32-correctly-rounded-divide-sqrt    IEEE f32 '/' and sqrtf, like x86 SSE
  -fno-gpu-flush-denormals-to-zero            keep f32 denormals, like x86 SSE
  no -ffast-math                              NaN/inf/ordering semantics of the C++ source
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libpt_mi355.so"
ARCH = os.environ.get("PT_OFFLOAD_ARCH", "gfx950")

SOURCES = ["pt_kernel.hip", "pt_output.hip", "pt_v4.hip", "pt_scene.cpp", "pt_v4_scene.cpp", "pt_capi.cpp",
           "pt_dropin.cpp", "pt_texture.cpp"]
HEADERS = ["pt_kernel.h", "pt_output.h", "pt_v4.h", "pt_v4_default_scene.h", "pt_scene.h", "pt_sincosf.h", "pt_exactmath.h",
           "pt_invtrig.h", "pt_envcert.h", "pt_tile_queue.h", "pt_quadcull.h", "pt_libmf.h", "pt_wave.h", "pt_guard.h",
           "pt_chain.h"]
CHECKED_LIB = ROOT / "build" / "libpt_checked.so"
PARITY_FLAGS = [
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero",
]
# Performance-only flags (no effect on results): the tile-queue atomic is issued by one lane, so the
# wave-reduction rewrite of the atomic optimizer only adds an immediate wait on its return value.
# -fno-slp-vectorize: the SLP vectorizer pairs independent f32 ops into v_pk_* (no faster than two
# plain ops on gfx950) and then needs v_mov copies to build the register pairs: off, the hot loop
# has 100 fewer VALU instructions and needs 96 instead of 122 VGPRs (5 waves per SIMD).
PERF_FLAGS = ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-fno-slp-vectorize"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libpt_mi355.so)")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _compile_link(out: Path, flags, tag: str, verbose: bool = False) -> None:
    """Compile SOURCES to objects in parallel (one hipcc per file: the same translation units as one
    hipcc call over all of them) under build/obj/<tag>/, then link the shared library `out`."""
    from concurrent.futures import ThreadPoolExecutor
    objdir = ROOT / "build" / "obj" / tag
    objdir.mkdir(parents=True, exist_ok=True)
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *flags, f"-I{ROOT / 'include'}",
            f"-I{CSRC}", "-Wno-unused-function"]

    deps = [CSRC / h for h in HEADERS] + [ROOT / "include" / "pt_mi355.h", ROOT / "include" / "demofox_path_tracing_mi355.h"]

    def one(src):
        obj = objdir / (src + ".o")
        cmd = [*base, "-c", str(CSRC / src), "-o", str(obj)]
        stamp = obj.with_suffix(".cmd")
        # (an object is reused when it is newer than its source and every header, and was built by the same command)
        if obj.exists() and stamp.exists() and stamp.read_text() == " ".join(cmd) and not _stale(obj, [CSRC / src, *deps]):
            return obj
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        stamp.write_text(" ".join(cmd))
        return obj

    # the largest translation units first
    order = sorted(SOURCES, key=lambda f: -(CSRC / f).stat().st_size)
    with ThreadPoolExecutor(max_workers=min(len(order), os.cpu_count() or 4)) as ex:
        objs = list(ex.map(one, order))
    tmp = str(out) + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)


def build_lib(force: bool = False, verbose: bool = False) -> Path:
    deps = [CSRC / s for s in SOURCES + HEADERS] + [ROOT / "include" / "pt_mi355.h",
                                                     ROOT / "include" / "demofox_path_tracing_mi355.h",
                                                     Path(__file__)]
    if not force and not _stale(LIB, deps):
        return LIB
    _compile_link(LIB, [*PARITY_FLAGS, *PERF_FLAGS, "-Wall"], "lib", verbose)
    return LIB


def build_variant(name: str, defines=(), extra=()) -> Path:
    """Dev tool: the library with extra -D defines into build/libpt_<name>.so (select it with
    PT_MI355_LIB=...); used for kernel A/B experiments."""
    out = ROOT / "build" / f"libpt_{name}.so"
    out.parent.mkdir(exist_ok=True)
    _compile_link(out, [*PARITY_FLAGS, *PERF_FLAGS, *[f"-D{d}" for d in defines], *extra], f"v_{name}")
    return out


def build_checked(force: bool = False, verbose: bool = False) -> Path:
    """The checked build (-DPT_CHECKED=1, pt_guard.h): every global index the continuous-tiles pools and
    the schedule builder compute is bounds-tested and a failure is reported as PT_EKERNEL naming the
    guard.  build/libpt_checked.so, selected with PT_MI355_LIB (a diagnostic library, not the product)."""
    deps = [CSRC / s for s in SOURCES + HEADERS] + [ROOT / "include" / "pt_mi355.h", Path(__file__)]
    if not force and not _stale(CHECKED_LIB, deps):
        return CHECKED_LIB
    CHECKED_LIB.parent.mkdir(exist_ok=True)
    _compile_link(CHECKED_LIB, [*PARITY_FLAGS, *PERF_FLAGS, "-DPT_CHECKED=1", "-Wall"], "checked", verbose)
    return CHECKED_LIB


def build_examples(verbose: bool = False) -> Path:
    """examples/reference_host: a reference-shaped C++ host linked against libpt_mi355.so through
    the reference-named header only (the drop-in boundary exercised as a real link)."""
    src = ROOT / "examples" / "reference_host.cpp"
    out = ROOT / "examples" / "reference_host"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", f"-I{ROOT / 'include'}", str(src), f"-L{PKG}", "-lpt_mi355",
           "-Wl,-rpath,$ORIGIN/../cpuperformanceraytracer_amd", "-o", str(out)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return out


def build_oracle(verbose: bool = False) -> None:
    """Test infrastructure: the C restatement (oracle/liboracle.so) and, when the reference is
    present in this container, its own scalar build (oracle/_ref/).  Building the checker is not
    using it: the product never loads either."""
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    ref = Path("/root/reference/CPUPerformanceRayTracer")
    if ref.exists():
        subprocess.run([str(ROOT / "oracle" / "build_ref.sh")], check=True,
                       stdout=None if verbose else subprocess.DEVNULL)


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv, verbose=True)
    if "--checked" in sys.argv:
        build_checked(verbose=True)
    build_examples(verbose=True)
    build_oracle(verbose=True)
    print(LIB)
