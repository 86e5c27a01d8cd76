"""Runtime mirror of the reference's compile-time configuration.

global_preprocessor_flags.h (CPUPerformanceRayTracer/) and the file-scope constants of
demofox_path_tracing_scalar.cpp:6-25, plus ApplicationState::CheckValidSettings
(Application.cpp:36-94).  The reference bakes these in with #define / const; here they are
values handed to the backend at init time (pt_config) or per call.
"""
from __future__ import annotations

from dataclasses import dataclass

# global_preprocessor_flags.h
NUM_SAMPLES_PER_FRAME = 1            # :30 / :33
NUM_FRAMES_TO_RENDER_OFFLINE = 600   # :31
RENDER_BUFFER_PIXEL_WIDTH = 1280     # :40
RENDER_BUFFER_PIXEL_HEIGHT = 720     # :39
ACCUMULATE_FRAMES = 1                # :60
NUM_THREADS = 8                      # :69 (CPU threads; the GPU grid replaces them)
NUM_TILES_X = 10                     # :85
NUM_TILES_Y = 15                     # :86
LANE_COUNT = 8                       # mathlib.h:10 (the tile-width / buffer-width granule)

# demofox_path_tracing_scalar.cpp
C_MINIMUM_RAY_HIT_TIME = 0.01        # :6
C_RAY_POS_NORMAL_NUDGE = 0.01        # :10
C_SUPER_FAR = 10000.0                # :13
C_FOV_DEGREES = 90.0                 # :16
C_NUM_BOUNCES = 4                    # :19
C_AMBIENT = (0.1, 0.1, 0.1)          # :307


@dataclass(frozen=True)
class Workload:
    """One benchmark/parity configuration (BASELINE.json `configs`)."""
    name: str
    width: int
    height: int
    spp: int
    num_bounces: int
    env: bool = False   # miss radiance = env-map sample (config 4) instead of the ambient
    renderer: str = "scalar"   # "scalar": the diffuse+emissive path (configs 1-5); "v4": optimization_v4
    scaling: str = "weak"      # N-rank bench: "weak" grows the image with N, "strong" keeps it fixed

    @property
    def primary_samples(self) -> int:
        return self.width * self.height * self.spp

    @property
    def ray_samples(self) -> int:
        """BASELINE.json metric unit: pixels x spp x bounces."""
        return self.width * self.height * self.spp * self.num_bounces


CONFIGS = {
    "c1_golden": Workload("c1_golden", 256, 256, 1, 4),          # configs[0] (CPU golden)
    "c2_1080p": Workload("c2_1080p", 1920, 1080, 8, 8),          # configs[1] (headline)
    "c3_4k": Workload("c3_4k", 3840, 2160, 64, 8),               # configs[2]
    "c4_env_1080p": Workload("c4_env_1080p", 1920, 1080, 16, 8, env=True),  # configs[3] (env map)
    "c5_8k": Workload("c5_8k", 7680, 4320, 256, 8, scaling="strong"),   # configs[4] (8 GPUs, fixed image)
    # the shipping v4 renderer (Application.cpp:474) at the headline size, its
    # default flags (equirect env map, random-jitter texel sampling, rejection-sampled directions)
    "v4_1080p": Workload("v4_1080p", 1920, 1080, 8, 8, env=True, renderer="v4"),
}


# Config 4 names chinese_garden_2k.hdr, which is missing from the reference checkout
# (.MISSING_LARGE_BLOBS); the stand-in is a synthetic 2k equirectangular map of the same shape.
SYNTHETIC_ENV_SHAPE = (1024, 2048)   # rows (height) x columns (width)
SYNTHETIC_ENV_SEED = 0xC0FFEE


def synthetic_env(height: int = SYNTHETIC_ENV_SHAPE[0], width: int = SYNTHETIC_ENV_SHAPE[1],
                  seed: int = SYNTHETIC_ENV_SEED):
    """H x W x 3 f32 radiance, log-normal (median 0.37, sigma 1): HDR-like dynamic range, as a
    texture LoadTexture would return (row 0 = bottom)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    return rng.lognormal(mean=-1.0, sigma=1.0, size=(height, width, 3)).astype(np.float32)


def check_valid_settings(width: int, height: int, num_tiles_x: int = NUM_TILES_X,
                         num_tiles_y: int = NUM_TILES_Y) -> list[str]:
    """Application.cpp:36-94.  Returns the list of violated rules (empty == valid)."""
    errs = []
    if num_tiles_x <= 0 or num_tiles_y <= 0:
        return ["number of tiles must be positive"]
    tile_w = width // num_tiles_x
    if tile_w % LANE_COUNT:
        errs.append("Invalid tile width detected. Must be multiple of 8 wide because of SIMD lane width")
    if height % num_tiles_y:
        errs.append("Invalid number of tile rows detected.")
    if width % num_tiles_x:
        errs.append("Invalid number of tile columns detected.")
    if width % LANE_COUNT:
        errs.append("Invalid image width detected. Must be multiple of 8 because of SIMD")
    return errs
