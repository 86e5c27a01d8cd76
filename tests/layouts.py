"""Test helpers: convert the reference's planar8 / tiled-planar8 buffers to the interleaved layout.

Index maps (CPUPerformanceRayTracer/):
  planar8  demofox_path_tracing_simd.cpp:496-511   per row, per 8 pixels: [R x8][G x8][B x8]
  tiled    demofox_path_tracing_simd_tiled.cpp:499-531   tile (tx,ty) occupies the contiguous slice
           starting at ty*TH*W*3 + tx*TW*TH*3; inside it rows of TW pixels in planar8 groups.
"""
from __future__ import annotations

import numpy as np


def planar8_to_interleaved(buf: np.ndarray, width: int, height: int) -> np.ndarray:
    g = buf.reshape(height, width // 8, 3, 8)          # row, group, channel, lane
    return np.ascontiguousarray(g.transpose(0, 1, 3, 2).reshape(height, width, 3))


def interleaved_to_planar8(img: np.ndarray) -> np.ndarray:
    h, w, _ = img.shape
    return np.ascontiguousarray(img.reshape(h, w // 8, 8, 3).transpose(0, 1, 3, 2).reshape(-1))


def tiled_to_interleaved(buf: np.ndarray, width: int, height: int, tw: int, th: int) -> np.ndarray:
    ntx, nty = width // tw, height // th
    # element order: ty, tx, ly, group, channel, lane
    t = buf.reshape(nty, ntx, th, tw // 8, 3, 8)
    return np.ascontiguousarray(t.transpose(0, 2, 1, 3, 5, 4).reshape(height, width, 3))


def interleaved_to_tiled(img: np.ndarray, tw: int, th: int) -> np.ndarray:
    h, w, _ = img.shape
    ntx, nty = w // tw, h // th
    t = img.reshape(nty, th, ntx, tw // 8, 8, 3)      # ty, ly, tx, group, lane, ch
    return np.ascontiguousarray(t.transpose(0, 2, 1, 3, 5, 4).reshape(-1))
