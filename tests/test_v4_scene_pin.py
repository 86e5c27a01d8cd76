"""Pins the v4 oracle's default scene to the reference's own InitializeScene (v4 :1403-1496).

The v4 renderer cannot be built here (Win32 / MSVC / SVML), so its outputs are "parity unpinned"
(DESIGN.md §2b).  Its scene, though, is literal data in the reference source: this test reads that
source as text (CPU suite only, skipped where /root/reference is absent -- it never travels to the
GPU box) and checks every number of the oracle's scene description against it: the quad vertices
with the scene translation (0, 0, 10) of SCENE 1 (v4 :697, :1406-1408) added where the reference
adds it (not to the striped background, :1431-1434), the seven spheres of the loop (:1469-1494) and
every material field.  The oracle description feeds pt_v4_build_scene and the generated literal
header, which tests/test_oracle_v4.py already checks against each other.
"""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np
import pytest

from oracle import pyoracle as po

V4 = Path("/root/reference/CPUPerformanceRayTracer/demofox_path_tracing_optimization_v4.cpp")
pytestmark = pytest.mark.skipif(not V4.exists(), reason="reference source not present (GPU box)")

F = r"(-?\d+(?:\.\d*)?|-?\.\d+)f?"   # a float literal as the reference writes it


def _f32(x: str) -> np.float32:
    return np.float32(float(x))


def _body() -> str:
    src = V4.read_text(errors="replace")
    start = src.index("void InitializeScene()")
    end = src.index("void InitializeCamera()", start)
    return src[start:end]


def _translation(src_all: str) -> np.ndarray:
    assert re.search(r"#define SCENE 1\b", src_all)
    m = re.search(r"scene\.sceneTranslation = set1x3_ps\(" + F + r", " + F + r", " + F + r"\)", src_all)
    return np.array([_f32(m.group(k)) for k in (1, 2, 3)], np.float32)


def test_quads_match_reference_literals():
    body = _body()
    t = _translation(V4.read_text(errors="replace"))
    pat = re.compile(r"NewQuadObject\.V(\d) = set1x3_ps\(" + F + r", " + F + r", " + F + r"\)(\s*\+\s*scene\.sceneTranslation)?;")
    verts = [(int(m.group(1)), np.array([_f32(m.group(k)) for k in (2, 3, 4)], np.float32), bool(m.group(5)))
             for m in pat.finditer(body)]
    assert len(verts) == 16 and [v[0] for v in verts] == [0, 1, 2, 3] * 4
    sc = po.default_scene4()
    assert sc.nquads == 4
    got = np.array(sc.quad, np.float32)[:4]
    for i, (_, v, translated) in enumerate(verts):
        want = (v + t).astype(np.float32) if translated else v   # f32 adds, as set1x3_ps + m256x3
        assert np.array_equal(got[i // 4, i % 4], want), (i, got[i // 4, i % 4], want, translated)
    # the striped background (second quad) is the one the reference leaves untranslated
    assert [v[2] for v in verts[4:8]] == [False] * 4 and all(v[2] for v in verts[:4] + verts[8:])


def test_quad_materials_match_reference_literals():
    body = _body()
    blocks = re.findall(r"QuadSceneObject NewQuadObject\{ 0 \};(.*?)AddMaterialToScene", body, re.S)
    assert len(blocks) == 4
    sc = po.default_scene4()
    for q, blk in enumerate(blocks):
        mat = sc.mat[q]
        a = re.search(r"^\s*NewMaterial\.albedo = f32x3\{\s*" + F + r",\s*" + F + r",\s*" + F + r"\s*\};", blk, re.M)
        want_alb = [_f32(a.group(k)) for k in (1, 2, 3)] if a else [np.float32(0)] * 3
        assert list(np.array(mat.albedo, np.float32)) == want_alb, (q, list(mat.albedo), want_alb)
        e = re.search(r"^\s*NewMaterial\.emissive = \(f32x3\{\s*" + F + r",\s*" + F + r",\s*" + F + r"\s*\}\s*\*\s*" + F + r"\);",
                      blk, re.M)
        want_em = [np.float32(_f32(e.group(k)) * _f32(e.group(4))) for k in (1, 2, 3)] if e else [np.float32(0)] * 3
        assert list(np.array(mat.emissive, np.float32)) == want_em, (q, list(mat.emissive), want_em)
        for field in ("spec_chance", "spec_rough", "ior", "refr_chance", "refr_rough"):
            assert getattr(mat, field) == 0.0, (q, field)
        assert list(mat.spec_color) == [0.0] * 3 and list(mat.refr_color) == [0.0] * 3


def test_spheres_and_their_materials_match_reference_literals():
    body = _body()
    body = body[body.index("const i32 c_numSpheres"):]   # the sphere loop
    n = int(re.search(r"const i32 c_numSpheres = (\d+);", body).group(1))
    m = re.search(r"set1x4_ps\(" + F + r" \+ " + F + r" \* \(f32\)\(sphereIndex\), " + F + r", " + F + r", " + F + r"\)"
                  r" \+ scene\.sceneTranslation4", body)
    x0, dx, y, z, r = (_f32(m.group(k)) for k in (1, 2, 3, 4, 5))
    t = _translation(V4.read_text(errors="replace"))
    sc = po.default_scene4()
    assert sc.nspheres == n == 7
    lit = {}
    for name in ("specularChance", "IOR", "refractionChance"):
        lit[name] = _f32(re.search(r"NewMaterial\." + name + r" = " + F + ";", body).group(1))
    vec = {}
    for name in ("albedo", "emissive", "refractionColor"):
        mm = re.search(r"NewMaterial\." + name + r" = f32x3\{ " + F + ", " + F + ", " + F + r" \};", body)
        vec[name] = [_f32(mm.group(k)) for k in (1, 2, 3)]
    sm = re.search(r"NewMaterial\.specularColor = f32x3\{ " + F + ", " + F + ", " + F + r" \} \*" + F + ";", body)
    spec_color = [np.float32(_f32(sm.group(k)) * _f32(sm.group(4))) for k in (1, 2, 3)]
    for i in range(n):
        # (-18 + 6 * i) in f32, then + sceneTranslation4 (w + 0)
        cx = np.float32(x0 + np.float32(dx * np.float32(i)))
        want = np.array([cx + t[0], y + t[1], z + t[2], r], np.float32)
        assert np.array_equal(np.array(sc.sphere[i], np.float32), want), (i, list(sc.sphere[i]), want)
        mat = sc.mat[4 + i]
        rough = np.float32(np.float32(np.float32(i) / np.float32(n - 1)) * np.float32(0.5))   # :1478
        assert mat.spec_chance == lit["specularChance"] and mat.ior == lit["IOR"]
        assert mat.refr_chance == lit["refractionChance"]
        assert list(np.array(mat.albedo, np.float32)) == vec["albedo"]
        assert list(np.array(mat.emissive, np.float32)) == vec["emissive"]
        assert list(np.array(mat.refr_color, np.float32)) == vec["refractionColor"]
        assert list(np.array(mat.spec_color, np.float32)) == spec_color
        assert np.float32(mat.spec_rough) == rough and np.float32(mat.refr_rough) == rough, (i, mat.spec_rough, rough)
