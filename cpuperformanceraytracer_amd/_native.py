"""ctypes binding of libpt_mi355.so (include/pt_mi355.h).

The product path is the HIP library only: if it cannot be loaded, or no GPU is present, every
render call raises -- there is no CPU fallback (the CPU restatement under oracle/ is a test
checker and is never imported here).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

from .build import LIB as _LIB_PATH

PT_OK = 0
PT_EINVAL = -1
PT_EHIP = -2
PT_ENOMEM = -3
PT_ESTATE = -4
PT_EKERNEL = -5

PT_LAYOUT_INTERLEAVED = 0
PT_LAYOUT_PLANAR8 = 1
PT_LAYOUT_TILED_PLANAR8 = 2

PT_FLAG_DEFER_READBACK = 1
PT_FLAG_PIN_HOST = 2
PT_FLAG_GATHER_ROOT = 4

PT_MAX_DEVICES = 16

PT_PIXEL_RGBA8 = 0
PT_PIXEL_XRGB8 = 1

# Every symbol include/pt_mi355.h declares (tests/test_abi.py checks they are all exported).
EXPORTED_SYMBOLS = (
    "pt_init", "pt_shutdown", "pt_last_error", "pt_default_config", "pt_set_frame", "pt_get_frame",
    "pt_render_scalar", "pt_render_simd", "pt_render_simd_tiled", "pt_render_tile", "pt_begin_frame",
    "pt_readback", "pt_gather_root", "pt_unpin_host", "pt_release_buffer", "pt_initialized_device", "pt_check_device_errors", "pt_build_checked", "pt_device_count",
    "pt_device_ordinal", "pt_render_device", "pt_render_device_chain", "pt_chain_counts", "pt_count_device", "pt_render_device_present", "pt_launch_variant",
    "pt_load_texture", "pt_decode_hdr", "pt_free_texture", "pt_set_env_map", "pt_render_simt_textured",
    "pt_tonemap", "pt_tonemap_device", "pt_write_bmp", "pt_load_cubemap_texture",
    "pt_v4_default_config", "pt_v4_set_config", "pt_v4_get_config", "pt_v4_initialize_global_render_resources",
    "pt_v4_reinitialize_render_tile_data", "pt_v4_initialize_scene", "pt_v4_clear_scene", "pt_v4_add_material",
    "pt_v4_add_quad", "pt_v4_add_sphere", "pt_v4_set_frame", "pt_v4_get_frame", "pt_v4_get_scene_tables", "pt_render_opt_v4",
    "pt_copy_output_to_file", "pt_v4_render_device", "pt_v4_render_device_chain", "pt_v4_count_device", "pt_v4_begin_frame",
    "pt_make_work_queue", "pt_add_work_queue_entry", "pt_complete_all_work", "pt_complete_all_work_async",
    "pt_wait_work", "pt_work_queue_size", "pt_free_work_queue",
)

PT_RENDERER_SIMD_TILED = 0
PT_RENDERER_SIMT_TEXTURED = 1
PT_RENDERER_V4 = 2

PT_V4_ENV_NONE = 0
PT_V4_ENV_EQUIRECT = 1
PT_V4_ENV_CUBEMAP = 2
PT_V4_MAX_OBJECTS = 12


class PtConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("num_bounces", ctypes.c_int32),
                ("samples_per_frame", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("ambient", ctypes.c_float * 3), ("device_count", ctypes.c_int32),
                ("devices", ctypes.c_int32 * PT_MAX_DEVICES)]


class PtBufferInfo(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("num_channels", ctypes.c_int32)]


class PtTileInfo(ctypes.Structure):
    _fields_ = [("tile_x", ctypes.c_int32), ("tile_y", ctypes.c_int32),
                ("tile_width", ctypes.c_int32), ("tile_height", ctypes.c_int32),
                ("tile_min_x", ctypes.c_int32), ("tile_max_x", ctypes.c_int32),
                ("tile_min_y", ctypes.c_int32), ("tile_max_y", ctypes.c_int32)]


class PtDeviceJob(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("row_start", ctypes.c_int32), ("row_stride", ctypes.c_int32), ("nrows", ctypes.c_int32),
                ("layout", ctypes.c_int32), ("frame_first", ctypes.c_uint32), ("nframes", ctypes.c_int32),
                ("num_bounces", ctypes.c_int32), ("use_env", ctypes.c_int32)]


class PtTexture(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_float)), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("components", ctypes.c_int32)]


class PtWorkCounts(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("lane_slots", ctypes.c_uint64),
                ("samples", ctypes.c_uint64), ("escaped", ctypes.c_uint64), ("primary", ctypes.c_uint64),
                ("quad_fallbacks", ctypes.c_uint64), ("sphere_fallbacks", ctypes.c_uint64),
                ("sky_skipped", ctypes.c_uint64)]


class PtV4Config(ctypes.Structure):
    _fields_ = [("env_mode", ctypes.c_int32), ("random_jitter", ctypes.c_int32), ("rejection", ctypes.c_int32),
                ("num_bounces", ctypes.c_int32), ("output_to_screen", ctypes.c_int32),
                ("accumulate_frames", ctypes.c_int32), ("fast_aces", ctypes.c_int32), ("fast_gamma", ctypes.c_int32),
                ("fast_exp", ctypes.c_int32)]


class PtV4Material(ctypes.Structure):
    _fields_ = [("albedo", ctypes.c_float * 3), ("emissive", ctypes.c_float * 3),
                ("specular_chance", ctypes.c_float), ("specular_roughness", ctypes.c_float),
                ("specular_color", ctypes.c_float * 3), ("ior", ctypes.c_float),
                ("refraction_chance", ctypes.c_float), ("refraction_roughness", ctypes.c_float),
                ("refraction_color", ctypes.c_float * 3)]


class PtError(RuntimeError):
    def __init__(self, code: int, what: str, detail: str):
        super().__init__(f"{what} failed (rc={code}): {detail}")
        self.code = code


_lib = None


def lib_path() -> Path:
    return Path(os.environ.get("PT_MI355_LIB", str(_LIB_PATH)))


def load() -> ctypes.CDLL:
    """Load libpt_mi355.so (build it first with cpuperformanceraytracer_amd.build)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not path.exists():
        raise FileNotFoundError(f"{path} not built: run `python -m cpuperformanceraytracer_amd.build`")
    # One HIP runtime per process: the ROCm PyTorch wheel bundles its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Loaded first, torch's copy is the one this library binds to; loaded
    # after /opt/rocm's, torch finds no GPU.  So torch (when installed) is imported before dlopen.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(str(path))
    i32, u32, vp = ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p
    sig = {
        "pt_init": (i32, [ctypes.POINTER(PtConfig)]),
        "pt_shutdown": (None, []),
        "pt_last_error": (ctypes.c_char_p, []),
        "pt_default_config": (None, [ctypes.POINTER(PtConfig)]),
        "pt_set_frame": (i32, [u32]),
        "pt_get_frame": (u32, []),
        "pt_render_scalar": (i32, [vp, i32, i32, i32]),
        "pt_render_simd": (i32, [vp, i32, i32, i32]),
        "pt_render_simd_tiled": (i32, [vp, i32, i32, i32, i32, i32, i32, i32]),
        "pt_render_tile": (i32, [ctypes.POINTER(PtBufferInfo), ctypes.POINTER(PtTileInfo)]),
        "pt_begin_frame": (i32, []),
        "pt_readback": (i32, [vp]),
        "pt_gather_root": (i32, [vp, ctypes.POINTER(vp)]),
        "pt_unpin_host": (i32, [vp]),
        "pt_release_buffer": (i32, [vp]),
        "pt_initialized_device": (i32, []),
        "pt_check_device_errors": (i32, []),
        "pt_build_checked": (i32, []),
        "pt_device_count": (i32, []),
        "pt_device_ordinal": (i32, [i32]),
        "pt_render_device": (i32, [ctypes.POINTER(PtDeviceJob), vp]),
        "pt_count_device": (i32, [ctypes.POINTER(PtDeviceJob), vp, ctypes.POINTER(PtWorkCounts)]),
        "pt_render_device_present": (i32, [ctypes.POINTER(PtDeviceJob), vp, i32, vp]),
        "pt_render_device_chain": (i32, [ctypes.POINTER(PtDeviceJob), vp]),
        "pt_chain_counts": (i32, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "pt_launch_variant": (i32, [ctypes.POINTER(PtDeviceJob), ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pt_load_texture": (i32, [ctypes.c_char_p, ctypes.POINTER(PtTexture)]),
        "pt_decode_hdr": (i32, [vp, ctypes.c_size_t, ctypes.POINTER(PtTexture)]),
        "pt_free_texture": (None, [ctypes.POINTER(PtTexture)]),
        "pt_set_env_map": (i32, [ctypes.POINTER(PtTexture)]),
        "pt_render_simt_textured": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, ctypes.POINTER(PtTexture)]),
        "pt_tonemap": (i32, [vp, i32, i32, i32, i32, i32, vp, i32]),
        "pt_tonemap_device": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, vp]),
        "pt_write_bmp": (i32, [ctypes.c_char_p, i32, i32, i32, vp]),
        "pt_load_cubemap_texture": (i32, [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(PtTexture)]),
        "pt_v4_default_config": (None, [ctypes.POINTER(PtV4Config)]),
        "pt_v4_set_config": (i32, [ctypes.POINTER(PtV4Config)]),
        "pt_v4_get_config": (i32, [ctypes.POINTER(PtV4Config)]),
        "pt_v4_initialize_global_render_resources": (i32, []),
        "pt_v4_reinitialize_render_tile_data": (i32, []),
        "pt_v4_initialize_scene": (i32, []),
        "pt_v4_clear_scene": (i32, []),
        "pt_v4_add_material": (i32, [ctypes.POINTER(PtV4Material)]),
        "pt_v4_add_quad": (i32, [ctypes.POINTER(ctypes.c_float)]),
        "pt_v4_add_sphere": (i32, [ctypes.POINTER(ctypes.c_float)]),
        "pt_v4_set_frame": (i32, [u32]),
        "pt_v4_get_frame": (u32, []),
        "pt_v4_get_scene_tables": (i32, [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pt_render_opt_v4": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, ctypes.POINTER(PtTexture), vp]),
        "pt_copy_output_to_file": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp]),
        "pt_v4_render_device": (i32, [ctypes.POINTER(PtDeviceJob), vp]),
        "pt_v4_render_device_chain": (i32, [ctypes.POINTER(PtDeviceJob), vp]),
        "pt_v4_count_device": (i32, [ctypes.POINTER(PtDeviceJob), vp, ctypes.POINTER(PtWorkCounts)]),
        "pt_v4_begin_frame": (i32, []),
        "pt_make_work_queue": (vp, [i32]),
        "pt_add_work_queue_entry": (i32, [vp, ctypes.POINTER(PtBufferInfo), ctypes.POINTER(PtTileInfo)]),
        "pt_complete_all_work": (i32, [vp]),
        "pt_complete_all_work_async": (i32, [vp]),
        "pt_wait_work": (i32, [vp]),
        "pt_work_queue_size": (i32, [vp]),
        "pt_free_work_queue": (None, [vp]),
    }
    dev_lib = bool(os.environ.get("PT_MI355_LIB"))
    for name, (res, args) in sig.items():
        fn = getattr(L, name, None)
        if fn is None and dev_lib:   # (an A/B library of an earlier revision: entry points added since are absent)
            continue
        if fn is None:
            raise AttributeError(f"{path}: missing symbol {name}")
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != PT_OK:
        detail = load().pt_last_error().decode(errors="replace")
        raise PtError(rc, what, detail)
