#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the reference's OWN scalar code.

Requires /root/reference (this container only) -- the reference never travels; these fixtures
(data: inputs + expected outputs) do.  Steps:
  1. oracle/build_ref.sh compiles demofox_path_tracing_scalar.cpp unmodified (see that script), and
     a temporary copy whose only change is c_numBounces = 8 (line 19's own `//8`).
  2. oracle/_ref/ref_scalar[_b8] W H F out.f32 runs DemofoxRenderScalar F times on a zeroed buffer
     in a fresh process (static iFrame starts at 0), exactly one run of the reference host.
     A case with "rows" stores only rows start::stride of the image (the reference renders all).
  3. Each result is stored xz-compressed raw little-endian f32 (H x W x 3, interleaved RGB), with
     its SHA-256 in manifest.json.

The wang-hash KATs in manifest.json are the survey's values for the reference's wang_hash
(demofox_path_tracing_scalar.cpp:27-35), SURVEY.md §8c.
"""
from __future__ import annotations

import hashlib
import json
import lzma
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

CASES = [
    # name, width, height, frames, num_bounces, stored rows (start, stride) or None = all
    # num_bounces 4: the reference's c_numBounces as shipped (scalar.cpp:19)
    ("g1_256x256_f1", 256, 256, 1, 4, None),    # configs[0]: 256x256, 1 spp, 4 bounces
    ("g2_256x256_f8", 256, 256, 8, 4, None),    # 8 accumulated frames
    ("g3_200x120_f3", 200, 120, 3, 4, None),    # non-square, not a multiple of the 16x16 block
    ("g4_64x64_f32", 64, 64, 32, 4, None),      # long accumulation chain (lerp weights 1/2 .. 1/33)
    # num_bounces 8: the build whose ONLY change is line 19's `= 4; //8` -> `= 8; //8`
    # (oracle/build_ref.sh; the diff and both sha256s are recorded under "b8_patch")
    ("g5_256x256_f8_b8", 256, 256, 8, 8, None),       # configs[1]'s bounce count, 8 frames
    ("g6_1920x1080_f2_b8", 1920, 1080, 2, 8, (0, 54)),  # configs[1]'s image, rows 0::54 (20 rows)
    ("g7_96x64_f53_b8", 96, 64, 53, 8, None),         # >= 48 frames: the ring pool in one launch
]


def main() -> None:
    subprocess.run([str(ROOT / "oracle" / "build_ref.sh")], check=True)
    from oracle import pyoracle
    manifest = {"generator": "tests/golden/make_golden.py (oracle/_ref/ref_scalar = reference scalar code)",
                "layout": "H x W x 3 float32 little-endian, interleaved RGB, row 0 = top", "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        for name, w, h, f, b, rows in CASES:
            img = pyoracle.ref_render(w, h, f, Path(td), num_bounces=b)
            if rows is not None:
                img = np.ascontiguousarray(img[rows[0]::rows[1]])
            raw = img.astype("<f4").tobytes()
            (HERE / f"{name}.f32.xz").write_bytes(lzma.compress(raw, preset=9))
            manifest["cases"][name] = {
                "width": w, "height": h, "frames": f, "num_bounces": b, "frame_first": 1,
                "sha256": hashlib.sha256(raw).hexdigest(),
                "mean_rgb": [float(x) for x in img.reshape(-1, 3).astype(np.float64).mean(0)],
            }
            if rows is not None:
                manifest["cases"][name]["rows"] = {"start": rows[0], "stride": rows[1],
                                                   "count": int(img.shape[0])}
    manifest["b8_patch"] = json.loads((ROOT / "oracle" / "_ref" / "b8_patch.json").read_text())
    manifest["kat_wang_hash"] = {
        "1": [663891101, 1738326990, 801461103, 3205955024],
        "2392335": [2263930673, 3823003730, 2449867500, 723927079],
    }
    manifest["kat_seed"] = {"comment": "pixel (0, row 0 => fragCoord.y = 255), frame 1, 256x256",
                            "x": 0, "y": 255, "frame": 1, "seed": 2392335}
    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
