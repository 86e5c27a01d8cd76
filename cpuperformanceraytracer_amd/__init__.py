"""MI355X (gfx950) backend for the per-pixel diffuse+emissive path-tracing hot path of
torgeiba/CPUPerformanceRayTracer (demofox_path_tracing_scalar.cpp / _simd.cpp / _simd_tiled.cpp).

  renderer  -- the reference's frame/tile interface on host buffers (drop-in)
  device    -- device-resident rendering on torch tensors (bench, shards)
  shard     -- row-interleaved multi-GPU sharding + RCCL gather of sub-images
  config    -- global_preprocessor_flags.h / CheckValidSettings mirror, benchmark workloads
  build     -- compiles libpt_mi355.so (HIP, gfx950) in-tree
"""
from .config import CONFIGS, Workload, check_valid_settings  # noqa: F401
from .renderer import (  # noqa: F401
    BeginFrame,
    CopyOutputToFile,
    DemofoxRenderScalar,
    DemofoxRenderSimd,
    DemofoxRenderSimdTiled,
    DemofoxRenderSimtTextured,
    LoadTexture,
    RenderBufferInfo,
    RenderTile,
    RenderTileInfo,
    get_frame,
    init,
    make_tiles,
    readback,
    set_env_map,
    set_frame,
    shutdown,
    texture,
    tonemap,
    WriteImage,
)

__all__ = [
    "CONFIGS", "Workload", "check_valid_settings", "BeginFrame", "CopyOutputToFile", "DemofoxRenderScalar", "DemofoxRenderSimd",
    "DemofoxRenderSimdTiled", "DemofoxRenderSimtTextured", "LoadTexture", "RenderBufferInfo", "RenderTile", "RenderTileInfo", "get_frame", "init",
    "make_tiles", "readback", "set_env_map", "set_frame", "shutdown", "texture", "tonemap", "WriteImage",
]
