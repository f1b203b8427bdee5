"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product path.  Builds the library on first use if it is missing (needs g++).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None
F = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
I = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
U64 = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
U8 = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


def build():
    src = os.path.join(ORACLE_DIR, "pt_oracle.cpp")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.oracle_logf.restype = C.c_float
        L.oracle_logf.argtypes = [C.c_float]
        L.oracle_cosf.restype = C.c_float
        L.oracle_cosf.argtypes = [C.c_float]
        L.oracle_logf_n.argtypes = [F, F, C.c_longlong]
        L.oracle_cosf_n.argtypes = [F, F, C.c_longlong]
        L.oracle_random_seq.argtypes = [C.c_uint, C.c_int, F, np.ctypeslib.ndpointer(np.uint32)]
        L.oracle_seed.restype = C.c_uint
        L.oracle_seed.argtypes = [C.c_int, C.c_int, C.c_int]
        L.oracle_load_obj.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p, C.c_int,
                                      C.POINTER(C.c_int), C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.oracle_build_bvh.argtypes = [F, C.c_int, F, C.c_int, C.POINTER(C.c_int)]
        L.oracle_builtins.argtypes = [C.c_int, F, F]
        scene = [F, C.c_int, F, C.c_int, F, C.c_int, F, C.c_int, F]
        L.oracle_render.argtypes = scene + [C.c_int] * 9 + [F, C.c_int, C.c_void_p]
        L.oracle_render_pixels.argtypes = scene + [C.c_int] * 9 + [I, I, C.c_int, F, C.c_int,
                                                                   C.c_void_p]
        L.oracle_aces_rgba8.argtypes = [F, C.c_int, U8]
        D = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        L.oracle_viewer_replay.restype = C.c_int
        L.oracle_viewer_replay.argtypes = [C.c_int, I, D, D, I, I, C.c_void_p, C.c_int, C.c_float, C.c_float,
                                           C.c_int, C.c_int, F, I]
        for fn in (L.oracle_mt_triangle, L.oracle_hit_triangle):
            fn.restype = C.c_float
            fn.argtypes = [F, F, F, F]
        _lib = L
    return _lib


def load_obj(obj_path, mtl_path):
    L = lib()
    nt, nm = C.c_int(), C.c_int()
    rc = L.oracle_load_obj(obj_path.encode(), mtl_path.encode(), None, 0, C.byref(nt), None, 0,
                           C.byref(nm))
    if rc:
        raise RuntimeError("oracle_load_obj failed: %d" % rc)
    tris = np.zeros((max(nt.value, 1), 16), np.float32)
    mats = np.zeros((max(nm.value, 1), 16), np.float32)
    rc = L.oracle_load_obj(obj_path.encode(), mtl_path.encode(), tris.ctypes.data, nt.value,
                           C.byref(nt), mats.ctypes.data, nm.value, C.byref(nm))
    assert rc == 0
    return tris[: nt.value].copy(), mats[: nm.value].copy()


def build_bvh(tris):
    tris = np.ascontiguousarray(tris, np.float32)
    n = len(tris)
    out = np.zeros((max(2 * n, 1), 12), np.float32)
    nn = C.c_int()
    rc = lib().oracle_build_bvh(tris, n, out, len(out), C.byref(nn))
    if rc:
        raise RuntimeError("oracle_build_bvh failed")
    return out[: nn.value].copy()


def builtins(n_loaded):
    m = np.zeros((5, 16), np.float32)
    s = np.zeros((1, 8), np.float32)
    lib().oracle_builtins(n_loaded, m, s)
    return m, s


def setup_buffers(obj_path, mtl_path):
    """Restates setupBuffers(): returns dict of the five std140 buffers."""
    tris, mats = load_obj(obj_path, mtl_path)
    nodes = build_bvh(tris)
    bm, sph = builtins(len(mats))
    cam = np.array([0, -6, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0], np.float32)
    return dict(tris=tris, nodes=nodes, mats=np.concatenate([mats, bm]), spheres=sph, cam=cam,
                n_loaded_mats=len(mats))


def _scene_args(sc):
    t = np.ascontiguousarray(sc["tris"], np.float32)
    n = np.ascontiguousarray(sc["nodes"], np.float32)
    m = np.ascontiguousarray(sc["mats"], np.float32)
    s = np.ascontiguousarray(sc["spheres"], np.float32).reshape(-1, 8)
    return [t.reshape(-1) if t.size else np.zeros(16, np.float32), len(t),
            n.reshape(-1) if n.size else np.zeros(12, np.float32), len(n),
            m.reshape(-1), len(m), s.reshape(-1) if s.size else np.zeros(8, np.float32), len(s)]


def render(sc, W, H, max_bounce=5, mode=1, frame_first=1, n_frames=1, acc_first=0, accum=None,
           threads=None, counters=False, flags=0, rpp=1):
    if accum is None:
        accum = np.zeros((H, W, 4), np.float32)
    accum = np.ascontiguousarray(accum, np.float32)
    cnt = np.zeros(5, np.uint64)
    threads = threads or os.cpu_count() or 1
    lib().oracle_render(*_scene_args(sc), np.ascontiguousarray(sc["cam"], np.float32), W, H,
                        max_bounce, mode, flags, rpp, frame_first, n_frames, acc_first,
                        accum.reshape(-1),
                        threads, cnt.ctypes.data if counters else None)
    return (accum, cnt) if counters else accum


def render_pixels(sc, W, H, xs, ys, max_bounce=5, mode=1, frame_first=1, n_frames=1,
                  acc_first=0, prior=None, threads=None, counters=False, flags=0, rpp=1):
    xs = np.ascontiguousarray(xs, np.int32)
    ys = np.ascontiguousarray(ys, np.int32)
    out = np.zeros((len(xs), 4), np.float32) if prior is None else np.array(prior, np.float32)
    cnt = np.zeros(5, np.uint64)
    threads = threads or os.cpu_count() or 1
    lib().oracle_render_pixels(*_scene_args(sc), np.ascontiguousarray(sc["cam"], np.float32), W,
                               H, max_bounce, mode, flags, rpp, frame_first, n_frames, acc_first,
                               xs, ys,
                               len(xs), out.reshape(-1), threads,
                               cnt.ctypes.data if counters else None)
    return (out, cnt) if counters else out


def aces_rgba8(img):
    img = np.ascontiguousarray(img, np.float32)
    out = np.zeros(img.shape[:-1] + (4,), np.uint8)
    lib().oracle_aces_rgba8(img.reshape(-1), img.size // 4, out.reshape(-1))
    return out


def triangle_test(o, d, tri, mt=False):
    """One triangle test (hit_triangle :274-307, or RayIntersectsTriangle :228-272 when mt)
    -> (t, normal)."""
    n = np.zeros(3, np.float32)
    fn = lib().oracle_mt_triangle if mt else lib().oracle_hit_triangle
    t = fn(np.asarray(o, np.float32), np.asarray(d, np.float32), np.ascontiguousarray(tri, np.float32), n)
    return np.float32(t), n


def viewer_replay(events, camera=None, display_mode=1, move_speed=10.0, rot_speed=0.1, accumulate=1):
    """Restated interactive loop (ogl_path_trace.h:160-204, 258-364) over an event list of
    ("frame", t) / ("key", code, action) / ("cursor", x, y) -> list of per-frame dicts
    {camera[12], frame, accumulate, display_mode}."""
    n = len(events)
    kind = np.zeros(max(n, 1), np.int32)
    a = np.zeros(max(n, 1), np.float64)
    b = np.zeros(max(n, 1), np.float64)
    key = np.zeros(max(n, 1), np.int32)
    act = np.zeros(max(n, 1), np.int32)
    for i, e in enumerate(events):
        if e[0] == "frame":
            a[i] = e[1]
        elif e[0] == "key":
            kind[i], key[i], act[i] = 1, e[1], e[2]
        else:
            kind[i], a[i], b[i] = 2, e[1], e[2]
    nf = max(1, sum(1 for e in events if e[0] == "frame"))
    cam_out = np.zeros(12 * nf, np.float32)
    fia = np.zeros(3 * nf, np.int32)
    cam = None if camera is None else np.ascontiguousarray(camera, np.float32).reshape(12)
    got = lib().oracle_viewer_replay(n, kind, a, b, key, act, None if cam is None else cam.ctypes.data,
                                     display_mode, move_speed, rot_speed, accumulate, nf, cam_out, fia)
    return [dict(camera=cam_out[12 * i: 12 * i + 12].copy(), frame=int(fia[3 * i]), accumulate=int(fia[3 * i + 1]),
                 display_mode=int(fia[3 * i + 2])) for i in range(got)]
