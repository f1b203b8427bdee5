"""Minimal image writers for the RGBA framebuffer surface (PNG via zlib, PFM for RGBA32F).

The reference shows the framebuffer in a GL window (screenQuadFrag.c); the headless build
writes it to disk instead.  Row 0 of the framebuffer is the BOTTOM row (GL texture
convention, ogl_path_trace.h:228-231), so writers flip vertically.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def write_png(path, rgba8):
    """rgba8: (H, W, 4) uint8 with row 0 = bottom."""
    img = np.ascontiguousarray(np.flipud(rgba8), np.uint8)
    h, w = img.shape[:2]
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(png)


def write_pfm(path, rgba32f):
    """Portable float map (RGB, little endian); PFM rows are stored bottom-to-top already."""
    img = np.ascontiguousarray(rgba32f[..., :3], np.float32)
    h, w = img.shape[:2]
    with open(path, "wb") as fh:
        fh.write(b"PF\n%d %d\n-1.0\n" % (w, h))
        fh.write(img.astype("<f4").tobytes())


def read_pfm(path):
    with open(path, "rb") as fh:
        assert fh.readline().strip() == b"PF"
        w, h = map(int, fh.readline().split())
        scale = float(fh.readline())
        data = np.frombuffer(fh.read(), "<f4" if scale < 0 else ">f4").reshape(h, w, 3)
    return data.astype(np.float32)
