"""Host-side mirror of the reference renderer interface, backed by libpt_mi355.so.

Same names, argument meaning and error behaviour as the reference's frame functions
(paths relative to /root/reference/CPUPerformanceRayTracer/):

  DemofoxRenderScalar(BufferOut, Width, Height, NumChannels)      demofox_path_tracing_scalar.h:7
  DemofoxRenderSimd(BufferOut, Width, Height, NumChannels)        demofox_path_tracing_simd.h:7
  DemofoxRenderSimdTiled(BufferOut, W, H, NTX, NTY, TW, TH, NC)   demofox_path_tracing_simd_tiled.h:7
  RenderBufferInfo / RenderTileInfo / RenderTile(info, tile)      demofox_path_tracing_simd_tiled.cpp:473-535
  texture / LoadTexture(filename)                                 texture.h:6-12, asset_loading.cpp:9-16
  DemofoxRenderSimtTextured(BufferOut, W, H, NTX, NTY, TW, TH, NC, Texture)
                                                                  demofox_path_tracing_simt_textured.h:8
  CopyOutputToFile(BufferOut, W, H, NTX, NTY, TW, TH, NC, Texture, ScreenBufferData)
                                                                  demofox_path_tracing_optimization_v4.h:21
  WriteImage(filename, width, height, components, data)           asset_loading.h:8

`BufferOut` is a float32 numpy array (the host render target of Application.cpp:142-151).  Each
frame call advances the frame counter first (the reference's `static f32 iFrame`) and returns after
the buffer holds the running average -- bit-identical to the reference's scalar path.  Invalid
settings raise PtError (the reference __debugbreak()s, Application.cpp:36-94).
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass

import numpy as np

from . import _native as N

_watch_buffers = False  # the library keeps a host buffer associated (PT_FLAG_PIN_HOST / DEFER_READBACK)
_buf_watch = {}        # (id(owner), ptr) -> weakref.finalize releasing ptr


def _release_ptr(ptr: int) -> None:
    try:
        N.load().pt_release_buffer(ctypes.c_void_p(ptr))
    except Exception:   # interpreter shutdown
        pass


def _watch(a: np.ndarray) -> None:
    """PT_FLAG_PIN_HOST / PT_FLAG_DEFER_READBACK: the library keeps the frame buffer page-locked or
    mirrored in HBM across calls.  When the array that owns the memory is released (a Resize
    reallocating the render target, Application.cpp:142-151), drop that association
    (pt_release_buffer: no write-back into freed memory) before numpy can hand the address out again."""
    owner = a
    while isinstance(owner.base, np.ndarray):
        owner = owner.base
    ptr = a.ctypes.data
    key = (id(owner), ptr)
    f = _buf_watch.get(key)
    if f is not None and f.alive:
        return
    for k in [k for k, v in _buf_watch.items() if not v.alive]:
        del _buf_watch[k]
    try:
        _buf_watch[key] = weakref.finalize(owner, _release_ptr, ptr)
    except TypeError:   # memory owned by an object without weakref support: released at shutdown
        pass


def _buf(a: np.ndarray, width: int, height: int, num_channels: int) -> int:
    if not isinstance(a, np.ndarray) or a.dtype != np.float32 or not a.flags["C_CONTIGUOUS"]:
        raise N.PtError(N.PT_EINVAL, "buffer", "BufferOut must be a C-contiguous float32 numpy array")
    if not a.flags["WRITEABLE"]:
        raise N.PtError(N.PT_EINVAL, "buffer", "BufferOut must be writeable")
    if width > 0 and height > 0 and num_channels > 0 and a.size < width * height * num_channels:
        raise N.PtError(N.PT_EINVAL, "buffer", f"BufferOut holds {a.size} floats < {width}x{height}x{num_channels}")
    if _watch_buffers:
        _watch(a)
    return a.ctypes.data


def init(num_bounces: int = 4, samples_per_frame: int = 1, ambient=(0.1, 0.1, 0.1), device: int | None = None,
         defer_readback: bool = False, pin_host: bool = False, devices=None, gather_root: bool = False) -> None:
    """(Re)initialise the backend: the runtime form of the reference's compile-time settings
    (c_numBounces scalar.cpp:19, NUM_SAMPLES_PER_FRAME global_preprocessor_flags.h:30).
    Resets the frame counter to 0, like a fresh process of the reference.
    pin_host: page-lock the frame buffer and overlap its transfers with rendering (row bands).
    devices: several HIP devices (ordinals may repeat: logical shards of one GPU) that every frame
    call deals its rows to (row Y -> devices[Y % len]).  device: that one HIP device alone -- an
    explicit device overrides PT_MI355_DEVICES (a rank of bench.py / shard.py initialises only its
    own GPU).  Neither: PT_MI355_DEVICES, else device 0.
    gather_root (several devices, deferred): the output stage and readback assemble the accumulator on
    devices[0] over xGMI first (PT_FLAG_GATHER_ROOT)."""
    if device is not None and devices is not None:
        raise N.PtError(N.PT_EINVAL, "init", "pass device or devices, not both")
    L = N.load()
    c = N.PtConfig()
    L.pt_default_config(ctypes.byref(c))
    if device is not None:
        c.device = device
        c.device_count = 1
        c.devices[0] = device
    if devices is not None:
        devices = list(devices)
        if not 1 <= len(devices) <= N.PT_MAX_DEVICES:
            raise N.PtError(N.PT_EINVAL, "init", f"1..{N.PT_MAX_DEVICES} devices expected")
        c.device = devices[0]
        c.device_count = len(devices)
        for i, d in enumerate(devices):
            c.devices[i] = d
    c.num_bounces = num_bounces
    c.samples_per_frame = samples_per_frame
    c.flags = ((N.PT_FLAG_DEFER_READBACK if defer_readback else 0) | (N.PT_FLAG_PIN_HOST if pin_host else 0) |
               (N.PT_FLAG_GATHER_ROOT if gather_root else 0))
    for i in range(3):
        c.ambient[i] = float(ambient[i])
    global _watch_buffers
    _watch_buffers = False
    N.check(L.pt_init(ctypes.byref(c)), "pt_init")
    _watch_buffers = bool(pin_host or defer_readback)


def shutdown() -> None:
    global _watch_buffers
    N.load().pt_shutdown()
    _watch_buffers = False


def initialized_device() -> int | None:
    """The (first) HIP device the library state lives on (None before init)."""
    d = int(N.load().pt_initialized_device())
    return None if d < 0 else d


def initialized_devices() -> list[int]:
    """The HIP ordinals of the library's logical devices ([] before init)."""
    L = N.load()
    return [int(L.pt_device_ordinal(i)) for i in range(int(L.pt_device_count()))]


def unpin_host(BufferOut: np.ndarray | None = None) -> None:
    """pin_host mode: drop the page-lock of BufferOut (None: of any pinned buffer) before freeing it."""
    ptr = None if BufferOut is None else ctypes.c_void_p(BufferOut.ctypes.data)
    N.check(N.load().pt_unpin_host(ptr), "pt_unpin_host")


def release_buffer(BufferOut: np.ndarray | None = None) -> None:
    """Before freeing / reallocating BufferOut (None: whichever buffer): drop its deferred device copy
    (not written back) and its page-lock (pt_release_buffer)."""
    ptr = None if BufferOut is None else ctypes.c_void_p(BufferOut.ctypes.data)
    N.check(N.load().pt_release_buffer(ptr), "pt_release_buffer")


def set_frame(frame: int) -> None:
    """Set the value of the reference's static iFrame (the next frame call renders frame+1)."""
    N.check(N.load().pt_set_frame(frame), "pt_set_frame")


def get_frame() -> int:
    return int(N.load().pt_get_frame())


def readback(BufferOut: np.ndarray) -> None:
    """defer_readback mode: copy the HBM-resident accumulator into BufferOut."""
    N.check(N.load().pt_readback(_buf(BufferOut, 0, 0, 0)), "pt_readback")


def gather_root(BufferOut: np.ndarray) -> int:
    """defer_readback mode: the accumulator of BufferOut assembled in the root device's HBM
    (pt_gather_root); returns its device address (library-owned, valid until the next call)."""
    p = ctypes.c_void_p()
    N.check(N.load().pt_gather_root(_buf(BufferOut, 0, 0, 0), ctypes.byref(p)), "pt_gather_root")
    return int(p.value)


def DemofoxRenderScalar(BufferOut: np.ndarray, Width: int, Height: int, NumChannels: int) -> None:
    N.check(N.load().pt_render_scalar(_buf(BufferOut, Width, Height, NumChannels), Width, Height, NumChannels),
            "DemofoxRenderScalar")


def DemofoxRenderSimd(BufferOut: np.ndarray, Width: int, Height: int, NumChannels: int) -> None:
    N.check(N.load().pt_render_simd(_buf(BufferOut, Width, Height, NumChannels), Width, Height, NumChannels),
            "DemofoxRenderSimd")


def DemofoxRenderSimdTiled(BufferOut: np.ndarray, BufferWidth: int, BufferHeight: int, NumTilesX: int,
                           NumTilesY: int, TileWidth: int, TileHeight: int, NumChannels: int) -> None:
    N.check(N.load().pt_render_simd_tiled(_buf(BufferOut, BufferWidth, BufferHeight, NumChannels), BufferWidth,
                                          BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight, NumChannels),
            "DemofoxRenderSimdTiled")


@dataclass
class RenderBufferInfo:
    """demofox_path_tracing_simd_tiled.cpp:473-479"""
    BufferDataPtr: np.ndarray
    BufferWidth: int
    BufferHeight: int
    NumChannels: int


@dataclass
class RenderTileInfo:
    """demofox_path_tracing_simd_tiled.cpp:481-487"""
    TileX: int
    TileY: int
    TileWidth: int
    TileHeight: int
    TileMinX: int
    TileMaxX: int
    TileMinY: int
    TileMaxY: int


def BeginFrame() -> None:
    """Advance the frame counter once without rendering (what DemofoxRenderSimdTiled does before
    fanning out RenderTile calls, simd_tiled.cpp:547)."""
    N.check(N.load().pt_begin_frame(), "pt_begin_frame")


def _tile_args(BufferInfo: RenderBufferInfo, TileInfo: RenderTileInfo):
    b = N.PtBufferInfo(_buf(BufferInfo.BufferDataPtr, BufferInfo.BufferWidth, BufferInfo.BufferHeight,
                            BufferInfo.NumChannels),
                       BufferInfo.BufferWidth, BufferInfo.BufferHeight, BufferInfo.NumChannels)
    t = N.PtTileInfo(TileInfo.TileX, TileInfo.TileY, TileInfo.TileWidth, TileInfo.TileHeight,
                     TileInfo.TileMinX, TileInfo.TileMaxX, TileInfo.TileMinY, TileInfo.TileMaxY)
    return b, t


def RenderTile(BufferInfo: RenderBufferInfo, TileInfo: RenderTileInfo) -> None:
    """Render one tile at the current frame into its tile-major slice (simd_tiled.cpp:489-535)."""
    b, t = _tile_args(BufferInfo, TileInfo)
    N.check(N.load().pt_render_tile(ctypes.byref(b), ctypes.byref(t)), "RenderTile")


class WorkQueue:
    """work_queue.cpp (MakeWorkQueue / AddWorkQueueEntry / CompleteAllWork) for the renderers' one
    use of it: a frame's RenderTile entries, rendered on the GPU at completion -- one launch for a
    whole frame of tiles.  renderer: N.PT_RENDERER_SIMD_TILED / _SIMT_TEXTURED / _V4."""

    def __init__(self, renderer: int = N.PT_RENDERER_SIMD_TILED):
        L = N.load()
        self._q = L.pt_make_work_queue(renderer)
        if not self._q:
            raise N.PtError(N.PT_EINVAL, "MakeWorkQueue", L.pt_last_error().decode(errors="replace"))
        self._keep = []   # host buffers referenced by queued entries

    def add(self, BufferInfo: RenderBufferInfo, TileInfo: RenderTileInfo) -> None:
        b, t = _tile_args(BufferInfo, TileInfo)
        N.check(N.load().pt_add_work_queue_entry(self._q, ctypes.byref(b), ctypes.byref(t)), "AddWorkQueueEntry")
        self._keep.append(BufferInfo.BufferDataPtr)

    def complete(self, wait: bool = True) -> None:
        L = N.load()
        if wait:
            N.check(L.pt_complete_all_work(self._q), "CompleteAllWork")
            self._keep = []
        else:
            N.check(L.pt_complete_all_work_async(self._q), "pt_complete_all_work_async")

    def wait(self) -> None:
        N.check(N.load().pt_wait_work(self._q), "pt_wait_work")
        self._keep = []

    def __len__(self) -> int:
        return int(N.load().pt_work_queue_size(self._q))

    def close(self) -> None:
        if self._q:
            N.load().pt_free_work_queue(self._q)
            self._q = None
            self._keep = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def MakeWorkQueue(renderer: int = N.PT_RENDERER_SIMD_TILED) -> WorkQueue:
    """work_queue.cpp:84-108 (the GPU takes the place of the NUM_THREADS workers)."""
    return WorkQueue(renderer)


def AddWorkQueueEntry(Queue: WorkQueue, BufferInfo: RenderBufferInfo, TileInfo: RenderTileInfo) -> None:
    """work_queue.cpp:37-56 with the RenderTile callback (DoWorkerThreadWork, v4 :1350-1358)."""
    Queue.add(BufferInfo, TileInfo)


def CompleteAllWork(Queue: WorkQueue) -> None:
    """work_queue.cpp:63-71: every queued tile rendered, buffers updated on return."""
    Queue.complete(wait=True)


def make_tiles(width: int, height: int, num_tiles_x: int, num_tiles_y: int):
    """The tile list DemofoxRenderSimdTiled walks (simd_tiled.cpp:549-571)."""
    tw, th = width // num_tiles_x, height // num_tiles_y
    tiles = []
    for tx in range(num_tiles_x):
        for ty in range(num_tiles_y):
            tiles.append(RenderTileInfo(tx, ty, tw, th, tx * tw, tx * tw + tw - 1, ty * th, ty * th + th - 1))
    return tiles


@dataclass
class texture:
    """texture.h:6-12 -- Data is Height x Width x Components f32, row 0 = bottom row."""
    Data: np.ndarray
    Width: int
    Height: int
    Components: int = 3


def _pt_texture(t) -> tuple[N.PtTexture, np.ndarray]:
    data = t.Data if isinstance(t, texture) else t
    data = np.ascontiguousarray(data, dtype=np.float32)
    if data.ndim != 3:
        raise N.PtError(N.PT_EINVAL, "texture", "texture data must be Height x Width x Components")
    h, w, c = data.shape
    if isinstance(t, texture) and (t.Width != w or t.Height != h or t.Components != c):
        raise N.PtError(N.PT_EINVAL, "texture", "texture Width/Height/Components disagree with Data.shape")
    return N.PtTexture(data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), w, h, c), data


def _from_pt_texture(pt: N.PtTexture) -> texture:
    L = N.load()
    try:
        n = pt.width * pt.height * pt.components
        data = np.ctypeslib.as_array(pt.data, shape=(n,)).copy().reshape(pt.height, pt.width, pt.components)
    finally:
        L.pt_free_texture(ctypes.byref(pt))
    return texture(data, data.shape[1], data.shape[0], data.shape[2])


def LoadTexture(filename) -> texture:
    """asset_loading.cpp:9-16: an RGBE .hdr file, flipped vertically (row 0 = bottom)."""
    pt = N.PtTexture()
    N.check(N.load().pt_load_texture(str(filename).encode(), ctypes.byref(pt)), "LoadTexture")
    return _from_pt_texture(pt)


def DecodeHdr(data: bytes) -> texture:
    """LoadTexture on an in-memory .hdr file."""
    pt = N.PtTexture()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    N.check(N.load().pt_decode_hdr(buf, len(data), ctypes.byref(pt)), "pt_decode_hdr")
    return _from_pt_texture(pt)


def set_env_map(tex) -> None:
    """Upload an env map (texture, or an H x W x 3 float32 array) to HBM for device jobs with
    use_env; None releases it."""
    L = N.load()
    if tex is None:
        N.check(L.pt_set_env_map(None), "pt_set_env_map")
        return
    pt, keep = _pt_texture(tex)
    N.check(L.pt_set_env_map(ctypes.byref(pt)), "pt_set_env_map")
    del keep


def DemofoxRenderSimtTextured(BufferOut: np.ndarray, BufferWidth: int, BufferHeight: int, NumTilesX: int,
                              NumTilesY: int, TileWidth: int, TileHeight: int, NumChannels: int, Texture) -> None:
    """demofox_path_tracing_simt_textured.cpp:560-620: the tiled frame with miss radiance =
    EquirectangularTextureSample(Texture, rayDir) (:408, texture.cpp:101-139)."""
    pt, keep = _pt_texture(Texture)
    N.check(N.load().pt_render_simt_textured(_buf(BufferOut, BufferWidth, BufferHeight, NumChannels), BufferWidth,
                                             BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight, NumChannels,
                                             ctypes.byref(pt)), "DemofoxRenderSimtTextured")
    del keep


def tonemap(accum: np.ndarray, width: int, height: int, layout: int = N.PT_LAYOUT_INTERLEAVED,
            tile_width: int = 0, tile_height: int = 0, fmt: int = N.PT_PIXEL_RGBA8) -> np.ndarray:
    """The output stage (v4 :1260-1331): accumulator -> height x width packed u32 pixels
    (PT_PIXEL_RGBA8: bytes R, G, B, 255; PT_PIXEL_XRGB8: 0x00RRGGBB)."""
    a = np.ascontiguousarray(accum, dtype=np.float32)
    if a.size < width * height * 3:
        raise N.PtError(N.PT_EINVAL, "tonemap", "accumulator smaller than width x height x 3")
    out = np.empty((height, width), np.uint32)
    N.check(N.load().pt_tonemap(a.ctypes.data, width, height, layout, tile_width, tile_height, out.ctypes.data, fmt),
            "pt_tonemap")
    return out


def _pixels(a, width: int, height: int, what: str) -> int:
    if (not isinstance(a, np.ndarray) or a.dtype != np.uint32 or not a.flags["C_CONTIGUOUS"]
            or not a.flags["WRITEABLE"] or a.size < width * height):
        raise N.PtError(N.PT_EINVAL, what, "pixel buffer must be a writeable contiguous uint32 array of W*H")
    return a.ctypes.data


def CopyOutputToFile(BufferOut: np.ndarray, BufferWidth: int, BufferHeight: int, NumTilesX: int, NumTilesY: int,
                     TileWidth: int, TileHeight: int, NumChannels: int, Texture, ScreenBufferData: np.ndarray) -> None:
    """v4 :1729-1760 (the post-process it documents): advances v4's iFrame (:1738), then the tiled
    accumulator -> ScreenBufferData, BufferWidth x BufferHeight u32 file pixels (bytes R, G, B, A = 255)."""
    px = _pixels(ScreenBufferData, BufferWidth, BufferHeight, "CopyOutputToFile")
    a = _buf(BufferOut, BufferWidth, BufferHeight, NumChannels)
    N.check(N.load().pt_copy_output_to_file(a, BufferWidth, BufferHeight, NumTilesX, NumTilesY, TileWidth, TileHeight,
                                            NumChannels, px), "CopyOutputToFile")


# ---- v4 renderer (demofox_path_tracing_optimization_v4.cpp) -------------------------------------------

def LoadCubemapTexture(filenames) -> texture:
    """asset_loading.cpp:18-44: six .hdr faces (px nx py ny pz nz) stacked into W x 6H."""
    if len(filenames) != 6:
        raise N.PtError(N.PT_EINVAL, "LoadCubemapTexture", "six face files expected")
    arr = (ctypes.c_char_p * 6)(*[str(f).encode() for f in filenames])
    pt = N.PtTexture()
    N.check(N.load().pt_load_cubemap_texture(arr, ctypes.byref(pt)), "LoadCubemapTexture")
    return _from_pt_texture(pt)


def v4_config(env_mode: int = N.PT_V4_ENV_EQUIRECT, random_jitter: bool = True, rejection: bool = True,
              num_bounces: int = 8, output_to_screen: bool = True, accumulate_frames: bool = True,
              fast_aces: bool = True, fast_gamma: bool = True, fast_exp: bool = True) -> None:
    """The v4 switches of global_preprocessor_flags.h (USE_ENV_MAP / USE_ENV_CUBEMAP,
    USE_RANDOM_JITTER_TEXTURE_SAMPLING, USE_UNIT_VECTOR_REJECTION_SAMPLING, OUTPUT_TO_SCREEN,
    ACCUMULATE_FRAMES, USE_FAST_APPROXIMATE_ACES_TONEMAP / _GAMMA / _EXP) and c_numBounces (v4 :23)."""
    c = N.PtV4Config(env_mode, int(random_jitter), int(rejection), num_bounces, int(output_to_screen),
                     int(accumulate_frames), int(fast_aces), int(fast_gamma), int(fast_exp))
    N.check(N.load().pt_v4_set_config(ctypes.byref(c)), "pt_v4_set_config")


def v4_get_config() -> dict:
    c = N.PtV4Config()
    N.check(N.load().pt_v4_get_config(ctypes.byref(c)), "pt_v4_get_config")
    return {k: int(getattr(c, k)) for k, _ in N.PtV4Config._fields_}


def InitializeGlobalRenderResources() -> None:
    """v4 :1640-1661: camera and InitializeScene on first use."""
    N.check(N.load().pt_v4_initialize_global_render_resources(), "InitializeGlobalRenderResources")


def ReinitializeRenderTileData() -> None:
    """v4 :1723-1726, called by the host's Resize (Application.cpp:154) after reallocating the render
    target: drops the pin_host page-lock of the old buffer (every call uses its own arguments)."""
    N.check(N.load().pt_v4_reinitialize_render_tile_data(), "ReinitializeRenderTileData")


def InitializeScene() -> None:
    """v4 :1403-1496: replace the scene by the reference's default (4 quads, 7 glass spheres)."""
    N.check(N.load().pt_v4_initialize_scene(), "InitializeScene")


def ClearScene() -> None:
    N.check(N.load().pt_v4_clear_scene(), "pt_v4_clear_scene")


def AddMaterialToScene(albedo=(0, 0, 0), emissive=(0, 0, 0), specular_chance=0.0, specular_roughness=0.0,
                       specular_color=(0, 0, 0), ior=0.0, refraction_chance=0.0, refraction_roughness=0.0,
                       refraction_color=(0, 0, 0)) -> int:
    """v4 :1368-1388 (SceneMaterial fields; zero defaults like `SceneMaterial{ 0 }`).  Returns its index."""
    m = N.PtV4Material((ctypes.c_float * 3)(*albedo), (ctypes.c_float * 3)(*emissive), specular_chance,
                       specular_roughness, (ctypes.c_float * 3)(*specular_color), ior, refraction_chance,
                       refraction_roughness, (ctypes.c_float * 3)(*refraction_color))
    rc = N.load().pt_v4_add_material(ctypes.byref(m))
    if rc < 0:
        N.check(rc, "AddMaterialToScene")
    return rc


def AddQuadObjectToScene(vertices) -> int:
    """v4 :1390-1395: four vertices (V0..V3, xyz).  Returns the quad count."""
    v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(12)
    rc = N.load().pt_v4_add_quad(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    if rc < 0:
        N.check(rc, "AddQuadObjectToScene")
    return rc


def AddSphereObjectToScene(position_radius) -> int:
    """v4 :1397-1401: (x, y, z, r).  Returns the quad count, like the reference."""
    v = np.ascontiguousarray(position_radius, dtype=np.float32).reshape(4)
    rc = N.load().pt_v4_add_sphere(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    if rc < 0:
        N.check(rc, "AddSphereObjectToScene")
    return rc


def v4_scene_tables() -> tuple[np.ndarray, int, int]:
    """The current v4 scene's precomputed tables (pt_v4_get_scene_tables): (floats, nquads, nspheres)."""
    L = N.load()
    nq, ns = ctypes.c_int32(), ctypes.c_int32()
    need = L.pt_v4_get_scene_tables(None, 0, ctypes.byref(nq), ctypes.byref(ns))
    if need < 0:
        N.check(need, "pt_v4_get_scene_tables")
    out = np.zeros(need, np.float32)
    N.check(0 if L.pt_v4_get_scene_tables(out.ctypes.data, need, ctypes.byref(nq), ctypes.byref(ns)) == need else -1,
            "pt_v4_get_scene_tables")
    return out, nq.value, ns.value


def v4_begin_frame() -> None:
    """iFrame += 1 of DemofoxRenderOptV4 (v4 :1703) without rendering (hosts that queue tiles)."""
    N.check(N.load().pt_v4_begin_frame(), "pt_v4_begin_frame")


def v4_set_frame(frame: int) -> None:
    N.check(N.load().pt_v4_set_frame(frame), "pt_v4_set_frame")


def v4_get_frame() -> int:
    return int(N.load().pt_v4_get_frame())


def DemofoxRenderOptV4(BufferOut: np.ndarray, BufferWidth: int, BufferHeight: int, NumTilesX: int, NumTilesY: int,
                       TileWidth: int, TileHeight: int, NumChannels: int, Texture=None,
                       ScreenBufferData: np.ndarray | None = None) -> None:
    """v4 :1696-1721: advance iFrame, render every tile (tiled planar8 accumulator) and, when
    ScreenBufferData is given (OUTPUT_TO_SCREEN), write its XRGB8 pixels."""
    L = N.load()
    keep = None
    tp = None
    if Texture is not None:
        pt, keep = _pt_texture(Texture)
        tp = ctypes.byref(pt)
    scr = None if ScreenBufferData is None else _pixels(ScreenBufferData, BufferWidth, BufferHeight, "DemofoxRenderOptV4")
    N.check(L.pt_render_opt_v4(_buf(BufferOut, BufferWidth, BufferHeight, NumChannels), BufferWidth, BufferHeight,
                               NumTilesX, NumTilesY, TileWidth, TileHeight, NumChannels, tp, scr),
            "DemofoxRenderOptV4")
    del keep


def WriteImage(filename, width: int, height: int, components: int, data: np.ndarray) -> None:
    """asset_loading.cpp:48-54 (stbi_write_bmp): a 24-bit BMP of width x height pixels of
    `components` bytes each."""
    d = np.ascontiguousarray(data)
    if d.nbytes < width * height * components:
        raise N.PtError(N.PT_EINVAL, "WriteImage", "data smaller than width x height x components bytes")
    N.check(N.load().pt_write_bmp(str(filename).encode(), width, height, components, d.ctypes.data), "WriteImage")
