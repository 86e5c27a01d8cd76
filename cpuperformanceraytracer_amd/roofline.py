"""Roofline constants for the path-tracing kernel (DESIGN.md "Roofline").

Algorithmic work is counted the way SURVEY.md §8d defines it: 1 FLOP per fp32 add, sub, mul,
div, sqrt or compare that the reference's SCALAR path executes (demofox_path_tracing_scalar.cpp),
negation/abs/moves 0, scene- and frame-constant work excluded (vertex translation, quad normals,
camera distance, aspect ratio, 1/(iFrame+1)), sin/cos counted separately as transcendentals.

The per-segment figure depends on which early exits of TestQuadTrace/TestSphereTrace a ray takes,
so it is an average measured by the instrumented CPU restatement over a sample of the benchmark
workload (tests/test_flops.py re-derives it and checks these constants).  The traced segments
themselves are counted exactly on the device for every benchmarked launch (pt_count_device).

Two figures per launch:
  algorithmic           SURVEY.md §8d's formula, FLOP = samples * F_SAMPLE + segments * F_SEGMENT
                        with `segments` the TestSceneTrace calls the output depends on, counted on
                        the device: the camera ray of a pixel (and its trace) is identical for
                        every frame -- no jitter, scalar.cpp:338-351 -- so it is ONE segment per
                        pixel, not one per sample.  Every counted segment is priced at the
                        reference's per-segment cost however the kernel decides it: the culled
                        quad stage, the closest-sphere stage and the sky-tile test
                        (pt_kernel.hip) compute the same closest hit with fewer instructions --
                        an implementation's economy, not less algorithmic work.  This is the
                        roofline's `achieved` numerator.
  reference-equivalent  the reference's own schedule of the same pixels: every frame traces its
                        own camera ray, segments_ref = traced - camera rays + samples and
                        FLOP_ref = segments_ref * F_SEGMENT + samples * F_SAMPLE (reported beside
                        it, never used for the fraction).
How much of the chip the kernel keeps busy is measured separately, from the PMC VALU instruction
counts (profiles/pmc_summary*.json, bench.py `valu_issue`).
"""

# Mean fp32 FLOP per traced segment (one TestSceneTrace + shading), 1920x1080, 8 bounces,
# rows 0::8 and 3::8, frames 1-2 (426.85 / 426.64); 3840x2160 rows 5::16 gives 426.68.
F_SEGMENT = 426.8
# FLOP per primary sample: camera ray (20) + the c_numRendersPerFrame=1 scale/add (6) +
# the progressive lerp (9) = 35, exact (no data dependence).
F_SAMPLE = 35.0
# Transcendentals (cosf + sinf) per traced segment: 2 per bounce that continues.
T_SEGMENT = 1.14
# FLOP per sample that are identical for every frame of its pixel (camera ray 20 + camera-ray
# trace + bounce-0 shading without RUV/normalize), 1920x1080 8 bounces rows 0::8 / 3::8 (402.47 /
# 402.52), 3840x2160 rows 5::16 (402.37).
F_SHARED = 402.45

# Mean reference FLOP of the TestSceneTrace of a camera ray in a sky tile (what the sky-tile test
# replaces with a slope comparison), the oracle's accounting (pto_sky_skipped) over the bench
# geometries: 1920x1080 347.09, 3840x2160 347.09, the weak-scaling shards 346.96-347.11
# (tests/test_flops.py).  Documents the economy of the sky test; not subtracted from the
# algorithmic work.
F_SKY_TRACE = 347.1

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters").
PEAK_FP32_TFLOPS = 157.3   # FP32 vector (= FP32 MFMA) peak, FMA counted as 2
PEAK_HBM_GBPS = 8000.0     # HBM3E spec peak (6.29 TB/s measured copy)

# Algorithmic HBM bytes: the accumulator is read once and written once per launch.
BYTES_PER_PIXEL_PER_LAUNCH = 24
# Config 4: one RGB f32 texel gathered per escaping path (texture.cpp:8-13).
BYTES_PER_ENV_GATHER = 12
# Config 4: the env miss term's f32 arithmetic per escaping path (EquirectangularTextureSample's
# per-lane body, texture.cpp:111-124): uv *= invAtan 2, + 0.5 2, fract 2, the four range compares,
# the (H-1) / (W-1) scaling 2 = 12 FLOP, plus atan2f and asinf counted as 2 transcendentals like
# sin/cos -- counted by the instrumented oracle (tests/test_flops.py).
F_ENV_ESCAPE = 12.0


def ref_segments(traced: int, camera_rays: int, samples: int) -> int:
    """Segments the reference traces for the same output (one camera ray per frame)."""
    return traced - camera_rays + samples


def launch_flops_ref(traced: int, camera_rays: int, samples: int, env_escapes: int = 0) -> float:
    return ref_segments(traced, camera_rays, samples) * F_SEGMENT + samples * F_SAMPLE + env_escapes * F_ENV_ESCAPE


def launch_flops_alg(traced: int, samples: int, env_escapes: int = 0) -> float:
    """samples * F_SAMPLE + device-counted segments * F_SEGMENT (+ config 4's env
    arithmetic per escaping path, F_ENV_ESCAPE; the device counts escapes per sample, as the
    reference evaluates them)."""
    return traced * F_SEGMENT + samples * F_SAMPLE + env_escapes * F_ENV_ESCAPE


# ---- v4 renderer (demofox_path_tracing_optimization_v4.cpp) ------------------------------------
# Mean executed f32 FLOP per traced segment (TestSceneTrace over 4 quads + 7 spheres, then either
# the env miss term or the material shading), counted by the instrumented oracle
# (oracle/pt_oracle_v4.c, per-function totals documented there) over 1920x1080, 8 bounces,
# default scene + 2k synthetic env, rows 0::8 / 3::8, frames 1-2: 496.01 / 495.84.  Every frame
# traces its own jittered camera ray, so executed == reference work (nothing is shared).
V4_F_SEGMENT = 495.9
# Per sample: camera ray 23 + c_numRendersPerFrame scale 6 + fused accumulate 9 (exact).
V4_F_SAMPLE = 38.0
# A camera ray that misses everything costs the reference 4 x 53 (quads) + 7 x 25 (spheres) FLOP in
# TestSceneTrace (the v4 oracle's accounting, tests/test_flops.py): what the sky-iteration test
# (pt_v4.hip sky_ray_v4) replaces.  Documented, not subtracted.
V4_F_SKY_TRACE = 387.0


def v4_launch_flops(segments: int, samples: int) -> float:
    """Algorithmic (= reference) work: every frame traces its own jittered camera ray, so nothing
    is shared; the sky-iteration test (pt_v4.hip sky_ray_v4) is priced like the trace it replaces."""
    return segments * V4_F_SEGMENT + samples * V4_F_SAMPLE
