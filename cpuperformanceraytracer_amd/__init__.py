"""MI355X (gfx950) backend for the per-pixel path-tracing hot path of torgeiba/CPUPerformanceRayTracer:
the diffuse+emissive tracer (demofox_path_tracing_scalar.cpp / _simd.cpp / _simd_tiled.cpp /
_simt_textured.cpp) and the shipping v4 renderer (demofox_path_tracing_optimization_v4.cpp).

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
    DemofoxRenderOptV4,
    InitializeGlobalRenderResources,
    ReinitializeRenderTileData,
    InitializeScene,
    ClearScene,
    AddMaterialToScene,
    AddQuadObjectToScene,
    AddSphereObjectToScene,
    LoadCubemapTexture,
    v4_config,
    v4_begin_frame,
    v4_get_frame,
    MakeWorkQueue,
    AddWorkQueueEntry,
    CompleteAllWork,
    WorkQueue,
    v4_set_frame,
    LoadTexture,
    RenderBufferInfo,
    RenderTile,
    RenderTileInfo,
    get_frame,
    init,
    initialized_device,
    initialized_devices,
    make_tiles,
    readback,
    gather_root,
    set_env_map,
    set_frame,
    shutdown,
    texture,
    tonemap,
    unpin_host,
    release_buffer,
    v4_get_config,
    WriteImage,
)

__all__ = [
    "CONFIGS", "Workload", "check_valid_settings", "BeginFrame", "CopyOutputToFile", "DemofoxRenderScalar", "DemofoxRenderSimd",
    "DemofoxRenderSimdTiled", "DemofoxRenderSimtTextured", "LoadTexture", "RenderBufferInfo", "RenderTile", "RenderTileInfo", "get_frame", "init",
    "make_tiles", "readback", "gather_root", "set_env_map", "set_frame", "shutdown", "texture", "tonemap", "WriteImage",
    "DemofoxRenderOptV4", "InitializeGlobalRenderResources", "ReinitializeRenderTileData", "InitializeScene",
    "ClearScene", "AddMaterialToScene", "AddQuadObjectToScene", "AddSphereObjectToScene", "LoadCubemapTexture",
    "v4_config", "v4_begin_frame", "v4_get_frame", "v4_set_frame", "MakeWorkQueue", "AddWorkQueueEntry",
    "CompleteAllWork", "WorkQueue", "initialized_device", "initialized_devices", "unpin_host", "release_buffer",
    "v4_get_config",
]
