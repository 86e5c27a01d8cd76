#!/usr/bin/env python3
"""Per-phase instruction budget of the diffuse kernel's pool iteration, from the gfx950 ISA.

  python scripts/valu_budget.py [--kernel MANGLED] [--defines X=1 ...]

Compiles csrc/pt_kernel.hip for gfx950 (device code with debug info: every instruction keeps its
chain of inlined functions), disassembles the kernel, finds the pool loop of phase B (the innermost
loop holding the non-camera trace) and attributes each instruction of its body to a phase: the
function render_body calls that the instruction was inlined from (one level deeper inside
trace() and random_unit_vector()), or the render_body source line for its own bookkeeping.
Counts per issue class: VALU 2-cycle (f32 add/mul/fma, moves, logic, 24-bit mul), VALU 4-cycle
(compares, cndmask, min/max/med3, bfi, mul_lo_u32, f64, conversions), VALU transcendental
(rcp/rsq/sqrt/...), SALU, LDS, VMEM, scratch (spill traffic), branches.  Static counts: each
instruction of the loop body once; phases behind rarely taken branches are marked "(fallback)".
Debug info does not change the code (same instruction count as the release build).
"""
from __future__ import annotations

import argparse
import collections
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "cpuperformanceraytracer_amd" / "csrc"
LLVM = Path("/opt/rocm/lib/llvm/bin")

FOUR = re.compile(r"^v_(cmp|cmpx|cndmask|max|min|med3|bfi|mul_lo_u32|mul_hi|cvt|\w*_f64|frexp|ldexp|div_|trig|fract|readlane|writelane|readfirstlane)")
TRANS = re.compile(r"^v_(rcp|rsq|sqrt|sin|cos|exp|log)")


def build(defines, src="pt_kernel.hip", csrc=None) -> Path:
    csrc = Path(csrc) if csrc else CSRC
    obj, co = Path("/tmp/_vb.o"), Path("/tmp/_vb.co")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero", "-mllvm",
           "-amdgpu-atomic-optimizer-strategy=None", "-fno-slp-vectorize", f"-I{csrc.parents[1] / 'include'}", f"-I{csrc}",
           "--cuda-device-only", "-c", "-g", *[f"-D{d}" for d in defines], str(csrc / src), "-o", str(obj)]
    subprocess.run(cmd, check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={obj}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def classify(op: str) -> str:
    if op.startswith("v_"):
        if TRANS.match(op):
            return "valu_trans"
        if FOUR.match(op):
            return "valu_4cyc"
        return "valu_2cyc"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def short(fn: str) -> str:
    return re.sub(r"<.*", "", fn.split("(")[0]).split("::")[-1]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="_ZN12_GLOBAL__N_116pt_render_kernelILi0ELb0ELb0ELb0EEEv5PtJob")
    ap.add_argument("--defines", nargs="*", default=[])
    ap.add_argument("--src", default="pt_kernel.hip")
    ap.add_argument("--csrc", default=None, help="another tree's csrc/ (e.g. a git worktree of an earlier round)")
    ap.add_argument("--body", default="render_body", help="the function whose callees are the phases")
    ap.add_argument("--need", nargs="*", default=["trace<*, false,", "random_unit_vector"],
                    help="function-name prefixes the pool loop must hold ('*' = anything)")
    ap.add_argument("--groups", action="store_true", help="also print the grouped markdown table (DESIGN.md §3)")
    ap.add_argument("--dump", default=None, help="print the instructions of the phases starting with this")
    ap.add_argument("--by-line", action="store_true",
                    help="attribute instructions to the body function's source line (its call sites)")
    a = ap.parse_args()
    co = build(a.defines, a.src, a.csrc)
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co), f"--disassemble-symbols={a.kernel}"],
                         capture_output=True, text=True, check=True).stdout
    ins = []   # (addr, op, text, branch target)
    for line in dis.splitlines():
        m = re.match(r"\s+(\w+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if not m:
            continue
        op, addr = m.group(1), int(m.group(3), 16)
        tgt = None
        t = re.search(r"<\S+\+0x([0-9a-f]+)>", line)
        if t and (op.startswith("s_cbranch") or op == "s_branch"):
            tgt = t.group(1)
        ins.append([addr, op, line.strip(), tgt])
    base = ins[0][0]
    for x in ins:
        if x[3] is not None:
            x[3] = base + int(x[3], 16)
    addrs = "\n".join(hex(x[0]) for x in ins) + "\n"
    sym = subprocess.run([str(LLVM / "llvm-symbolizer"), f"--obj={co}", "--inlining", "--functions=short"],
                         input=addrs, capture_output=True, text=True, check=True).stdout
    chains = [blk.strip().splitlines() for blk in sym.strip().split("\n\n")]
    assert len(chains) == len(ins), (len(chains), len(ins))
    frames = []   # per instruction: [(function, file:line), ...] innermost first
    for c in chains:
        frames.append([(c[i], c[i + 1]) for i in range(0, len(c) - 1, 2)])
    idx = {x[0]: i for i, x in enumerate(ins)}
    loops = [(idx[x[3]], i) for i, x in enumerate(ins) if x[3] is not None and x[3] <= x[0] and x[3] in idx]

    def holds(lo, hi, pred):
        return any(any(pred(f) for f, _ in frames[j]) for j in range(lo, hi + 1))

    # the pool iteration: the smallest loop holding phase B's trace AND the new direction
    pats = [re.compile(re.escape(n).replace(r"\*", ".*")) for n in a.need]
    pool = min((l for l in loops if all(holds(*l, lambda f, r=r: r.match(f) is not None) for r in pats)),
               key=lambda l: l[1] - l[0])
    # rarely taken sub-paths, marked "(fallback)": the sequential sphere tests, the six exact quad
    # tests, and the cull's far-wall rectangle for rays nearly parallel to a wall pair
    qcp = (Path(a.csrc) if a.csrc else CSRC) / "pt_quadcull.h"
    qc = qcp.read_text().splitlines() if qcp.exists() else []
    tiny_lines = {str(i + 1) for i, l in enumerate(qc) if "if (tiny[" in l and "classify" in l}
    counts = collections.defaultdict(collections.Counter)
    cross = collections.defaultdict(collections.Counter)   # cross-cutting: exact-math sequences, f64
    for j in range(pool[0], pool[1] + 1):
        fr = frames[j]
        names = [f for f, _ in fr]
        k = next((i for i, f in enumerate(names) if f.startswith(a.body)), len(names))
        if a.by_line and k < len(names):
            ph = a.body + ":" + fr[k][1].rsplit(":", 2)[-2]   # the body's line (own code or call site)
        elif k == 0:
            ph = a.body + ":" + fr[0][1].rsplit(":", 2)[-2]   # its own line
        else:
            ph = short(names[k - 1])
            if ph in ("trace", "random_unit_vector") and k >= 2:
                ph += "/" + short(names[k - 2])
            if ph == "trace/quads_exact" or ph == "trace/sphere_test" or "sphere_test" in names[:k]:
                ph = ph + " (fallback)" if ph.endswith("sphere_test") or ph.endswith("quads_exact") else "trace/sphere_test (fallback)"
            if ph == "trace/cull" and any(f.startswith("cull") and ln.rsplit(":", 2)[-2] in tiny_lines for f, ln in fr):
                ph = "trace/cull (tiny-pq branch)"
        counts[ph][classify(ins[j][1])] += 1
        if "(fallback)" not in ph and "branch)" not in ph:
            if any(short(f) in ("rcp_x", "sqrt_x", "div_x", "rcp_rn", "sqrt_rn", "div_rn", "sqrt_guarded", "rcp_guarded",
                                "div_guarded") for f in names):
                cross["exact rcp / sqrt / div sequences (pt_exactmath.h)"][classify(ins[j][1])] += 1
            if "_f64" in ins[j][1] or ins[j][1].startswith("v_cvt_f32_f64") or ins[j][1].startswith("v_cvt_f64"):
                cross["f64 instructions (all in sincosf_glibc)"][classify(ins[j][1])] += 1
        if a.dump is not None and ph.startswith(a.dump):
            print(f"{ph[:28]:28s} {ins[j][2].split('//')[0]}")
    # fold render_body's own lines into one bucket per source line range
    cols = ["valu_2cyc", "valu_4cyc", "valu_trans", "salu", "lds", "vmem", "scratch", "branch", "other"]
    print(f"pool loop of {a.kernel}: instructions {pool[0]}..{pool[1]} ({pool[1] - pool[0] + 1}) of {len(ins)}")
    print(f"{'phase':34s}" + "".join(f"{c[:9]:>10s}" for c in cols) + f"{'VALU':>7s}{'cyc':>7s}")
    tot = collections.Counter()

    def valu(c):
        return c["valu_2cyc"] + c["valu_4cyc"] + c["valu_trans"]

    def cyc(c):
        return 2 * c["valu_2cyc"] + 4 * c["valu_4cyc"] + 8 * c["valu_trans"]

    for ph in sorted(counts, key=lambda p: -cyc(counts[p])):
        c = counts[ph]
        tot.update(c)
        print(f"{ph[:34]:34s}" + "".join(f"{c[k]:10d}" for k in cols) + f"{valu(c):7d}{cyc(c):7d}")
    print(f"{'total':34s}" + "".join(f"{tot[k]:10d}" for k in cols) + f"{valu(tot):7d}{cyc(tot):7d}")
    if not a.groups:
        return
    groups = [
        ("cull classification (pt_quadcull.h)", lambda p: p == "trace/cull"),
        ("exact TestQuadTrace of the cull's W", lambda p: p == "trace/quad_exact"),
        ("closest-sphere stage", lambda p: p == "trace/spheres_closest"),
        ("trace glue (distance axis, W's vertex rows, result)", lambda p: p.startswith("trace") and "(" not in p
         and p not in ("trace/cull", "trace/quad_exact", "trace/spheres_closest")),
        ("glibc-exact sincosf (f64)", lambda p: p == "random_unit_vector/sincosf_glibc"),
        ("RNG (wang_hash, Randomf3201, seed)", lambda p: p in ("random_unit_vector/randomf", "seed_int")),
        ("unit vector + new direction (sqrt, normalize)", lambda p: p in ("random_unit_vector", "random_unit_vector/sqrt_x",
                                                                          "normalize", "add")),
        ("shading (hit normal, emissive, albedo, origin)", lambda p: p in ("hit_normal", "mulv", "mul")),
        ("pool bookkeeping (refill, slots, ballots)", lambda p: p.startswith(a.body) or p.startswith("__")),
    ]
    main = collections.Counter()
    print("\n| phase | VALU | of which 4-cycle | transcendental | issue cycles |\n|---|---|---|---|---|")
    seen = set()
    for name, pred in groups:
        c = collections.Counter()
        for ph in counts:
            if pred(ph) and "(fallback)" not in ph and "branch)" not in ph:
                c.update(counts[ph]); seen.add(ph)
        main.update(c)
        print(f"| {name} | {valu(c)} | {c['valu_4cyc']} | {c['valu_trans']} | {cyc(c)} |")
    rest = collections.Counter()
    for ph in counts:
        if ph not in seen and "(fallback)" not in ph and "branch)" not in ph:
            rest.update(counts[ph])
    if valu(rest):
        print(f"| other | {valu(rest)} | {rest['valu_4cyc']} | {rest['valu_trans']} | {cyc(rest)} |")
    main.update(rest)
    print(f"| **main path per iteration** | **{valu(main)}** | **{main['valu_4cyc']}** | **{main['valu_trans']}** | **{cyc(main)}** |")
    for ph in sorted(p for p in counts if "(fallback)" in p or "branch)" in p):
        c = counts[ph]
        print(f"| rare: {ph} | {valu(c)} | {c['valu_4cyc']} | {c['valu_trans']} | {cyc(c)} |")
    for name, c in cross.items():
        print(f"| cross-cut: {name} | {valu(c)} | {c['valu_4cyc']} | {c['valu_trans']} | {cyc(c)} |")


if __name__ == "__main__":
    sys.exit(main())
