"""Python mirror of the reference's host interface for the hot path, over the pt_api.h /
pt_scene.h C ABI (ctypes; build/libptrace.so).

Names follow the reference so that its call sequence reads the same:
  load_vertex_data(obj, mtl)  geometry_loader.h:15-142   -> (tris[N,16], mats[M,16])
  buildSAHTree(tris)          bvh.h:255-268              -> nodes[K,12]
  setupBuffers(obj, mtl)      ogl_path_trace.h:367-530   -> SceneBuffers (5 std140 buffers)
  ComputeShader / PathTracer  shader_c.h + glDispatchCompute(ogl_path_trace.h:174-186)
    .dispatch(frame, accumulate)        one reference dispatch (uniforms frame/accumulate)
    .render(frame_first, n, acc_first)  n dispatches fused in one launch (bit-identical)
Errors raise PTError carrying the library's code and message (the reference prints and
continues; the drop-in fails loudly instead -- DESIGN.md §1).

There is no CPU fallback: if the HIP library is missing or no device is present, the
calls raise.  The CPU oracle lives in oracle/ and is only used by tests and the bench's
cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# PT_LIB selects another in-tree build of the same library (tools/ab.py A/B timing only).
LIB_PATH = os.environ.get("PT_LIB") or os.path.join(PKG_DIR, "build", "libptrace.so")
INCLUDE_DIR = os.path.join(os.path.dirname(PKG_DIR), "include")

PT_FLAG_NO_AA, PT_FLAG_NO_SKY, PT_FLAG_NO_SPHERES, PT_FLAG_NO_TRIANGLES, PT_FLAG_REF_DISPATCH = 1, 2, 4, 8, 16
PT_FLAG_MOLLER_TRUMBORE = 32   # opt-in fast triangle test (not the reference image; see pt_api.h)
DEFAULT_CAMERA = np.array([0, -6, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0], np.float32)  # ogl_path_trace.h:53-54

_ERR = {-1: "PT_E_ARG", -2: "PT_E_IO", -3: "PT_E_PARSE", -4: "PT_E_SCENE", -5: "PT_E_HIP", -6: "PT_E_STATE",
        -7: "PT_E_RCCL"}


class PTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (_ERR.get(code, "PT_E?"), code, msg))
        self.code = code


class _Config(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("width", "height", "max_bounce", "display_mode", "flags",
                                       "rays_per_pixel", "device", "rank", "world")]


class ViewerFrame(C.Structure):
    """pt_viewer_frame_info (include/pt_viewer.h)."""
    _fields_ = [("camera", C.c_float * 12), ("frame", C.c_int), ("accumulate", C.c_int),
                ("display_mode", C.c_int), ("should_close", C.c_int)]


_lib = None
_F = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_I = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def build(force=False):
    """Compile build/libptrace.so (hipcc, gfx950) in-tree."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", PKG_DIR, "all"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PTError(-5, "native library %s is missing; run `make -C %s`" % (LIB_PATH, PKG_DIR))
        L = C.CDLL(LIB_PATH)
        vp, ip, fp = C.c_void_p, C.c_int, C.c_float
        sig = {
            "pt_scene_load_obj": (ip, [C.c_char_p, C.c_char_p, C.POINTER(vp)]),
            "pt_scene_load_obj_ex": (ip, [C.c_char_p, C.c_char_p, ip, C.POINTER(vp)]),
            "pt_scene_from_arrays": (ip, [_F, ip, _F, ip, C.POINTER(vp)]),
            "pt_scene_add_builtins": (ip, [vp]),
            "pt_scene_build_bvh": (ip, [vp]),
            "pt_scene_counts": (ip, [vp, np.ctypeslib.ndpointer(np.int32)]),
            "pt_scene_get_tris": (ip, [vp, _F, ip]),
            "pt_scene_get_mats": (ip, [vp, _F, ip]),
            "pt_scene_get_spheres": (ip, [vp, _F, ip]),
            "pt_scene_get_nodes": (ip, [vp, _F, ip]),
            "pt_scene_last_error": (C.c_char_p, [vp]),
            "pt_scene_free": (None, [vp]),
            "pt_bvh_build": (ip, [_F, ip, _F, ip, C.POINTER(ip)]),
            "pt_bvh_build_gpu": (ip, [_F, ip, _F, ip, C.POINTER(ip), ip]),
            "pt_scene_build_bvh_gpu": (ip, [vp, ip]),
            "pt_bvh_last_error": (C.c_char_p, []),
            "pt_bvh_culling_ok": (ip, [_F, ip]),
            "pt_aces_rgba8_host": (None, [_F, C.c_longlong, np.ctypeslib.ndpointer(np.uint8)]),
            "pt_create": (ip, [C.POINTER(_Config), C.POINTER(vp)]),
            "pt_destroy": (None, [vp]),
            "pt_last_error": (C.c_char_p, [vp]),
            "pt_upload_scene": (ip, [vp, _F, ip, _F, ip, _F, ip, _F, ip]),
            "pt_set_camera": (ip, [vp, _F]),
            "pt_render": (ip, [vp, ip, ip, ip]),
            "pt_render_async": (ip, [vp, ip, ip, ip]),
            "pt_sync": (ip, [vp]),
            "pt_rows": (ip, [vp, C.POINTER(ip), C.POINTER(ip), C.POINTER(ip)]),
            "pt_read_rgba32f": (ip, [vp, vp, C.c_size_t]),
            "pt_read_rgba8_aces": (ip, [vp, vp, C.c_size_t]),
            "pt_write_rgba32f": (ip, [vp, vp, C.c_size_t]),
            "pt_present_begin": (ip, [vp, ip]),
            "pt_present_end": (ip, [vp, ip, C.POINTER(C.POINTER(C.c_ubyte))]),
            "pt_accum_device": (ip, [vp, C.POINTER(vp), C.POINTER(C.c_size_t)]),
            "pt_stream": (ip, [vp, C.POINTER(vp)]),
            "pt_set_counting": (ip, [vp, ip]),
            "pt_stats": (ip, [vp, C.POINTER(C.c_double), np.ctypeslib.ndpointer(np.uint64)]),
            "pt_set_kernel": (ip, [vp, ip]),
            "pt_copy_rows_device": (ip, [vp, vp, C.c_size_t]),
            "pt_timing": (ip, [vp, C.POINTER(C.c_double), C.POINTER(ip), ip]),
            "pt_stats_ex": (ip, [vp, np.ctypeslib.ndpointer(np.uint64)]),
            "pt_set_tuning": (ip, [vp, ip, ip]),
            "pt_progressive_setup": (ip, [vp, ip, ip]),
            "pt_progressive_reset": (ip, [vp, ip]),
            "pt_progressive_run": (ip, [vp, ip]),
            "pt_set_display_mode": (ip, [vp, ip]),
            "pt_get_config": (ip, [vp, C.POINTER(_Config)]),
            "pt_group_create": (ip, [C.POINTER(vp), ip, C.POINTER(vp)]),
            "pt_group_destroy": (None, [vp]),
            "pt_group_last_error": (C.c_char_p, [vp]),
            "pt_group_upload_scene": (ip, [vp, _F, ip, _F, ip, _F, ip, _F, ip]),
            "pt_group_gather_rgba32f": (ip, [vp, vp, C.c_size_t, ip]),
            "pt_group_stats": (ip, [vp, C.POINTER(C.c_double), C.POINTER(C.c_size_t)]),
            "pt_group_gather_rgba8_aces": (ip, [vp, vp, C.c_size_t, ip]),
            "pt_group_present_begin": (ip, [vp, ip]),
            "pt_group_present_end": (ip, [vp, ip, C.POINTER(C.POINTER(C.c_ubyte))]),
            "pt_gather_rgba32f": (ip, [C.POINTER(vp), ip, vp, C.c_size_t, ip]),
            "pt_group_plan": (ip, [_I, _I, ip, _I, C.POINTER(ip), _I, _I, C.POINTER(ip), _I]),
            "pt_group_interleave_host": (ip, [_F, C.c_size_t, _I, ip, ip, ip, _F]),
            "pt_viewer_create": (ip, [vp, ip, C.POINTER(vp)]),
            "pt_viewer_destroy": (None, [vp]),
            "pt_viewer_set_params": (ip, [vp, fp, fp, ip]),
            "pt_viewer_key": (ip, [vp, ip, ip]),
            "pt_viewer_cursor": (ip, [vp, C.c_double, C.c_double]),
            "pt_viewer_should_close": (ip, [vp]),
            "pt_viewer_next": (ip, [vp, C.c_double, C.POINTER(ViewerFrame)]),
            "pt_viewer_frame": (ip, [vp, vp, C.c_double, C.POINTER(ViewerFrame)]),
        }
        for name, (res, args) in sig.items():
            # tools/ab_inproc.py loads older builds beside this one: PT_LIB_PARTIAL=1 lets a
            # build without the newer entry points load (the product always binds all of them)
            if os.environ.get("PT_LIB_PARTIAL") == "1" and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def header_symbols():
    """Function names declared in include/*.h (for the ABI export test)."""
    import re
    names = []
    for h in ("pt_api.h", "pt_scene.h", "pt_viewer.h", "pt_group.h"):
        txt = open(os.path.join(INCLUDE_DIR, h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names += re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", txt)
    return sorted(set(names))


# ----------------------------------------------------------------------------- scene ingest
def _f32(a, cols):
    a = np.ascontiguousarray(a, np.float32)
    return a.reshape(-1, cols) if a.size else np.zeros((0, cols), np.float32)


class _Scene:
    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        if getattr(self, "h", None):
            lib().pt_scene_free(self.h)
            self.h = None

    def check(self, rc):
        if rc:
            raise PTError(rc, lib().pt_scene_last_error(self.h).decode())

    def counts(self):
        c = np.zeros(5, np.int32)
        self.check(lib().pt_scene_counts(self.h, c))
        return dict(n_tris=int(c[0]), n_mats=int(c[1]), n_spheres=int(c[2]), n_nodes=int(c[3]), n_loaded_mats=int(c[4]))

    def arrays(self):
        c = self.counts()
        out = {}
        for key, n, cols, fn in (("tris", c["n_tris"], 16, lib().pt_scene_get_tris),
                                 ("mats", c["n_mats"], 16, lib().pt_scene_get_mats),
                                 ("spheres", c["n_spheres"], 8, lib().pt_scene_get_spheres),
                                 ("nodes", c["n_nodes"], 12, lib().pt_scene_get_nodes)):
            a = np.zeros((max(n, 1), cols), np.float32)
            self.check(fn(self.h, a, max(n, 1)))
            out[key] = a[:n].copy()
        out["n_loaded_mats"] = c["n_loaded_mats"]
        return out


def load_vertex_data(obj_path, mtl_path):
    """geometry_loader.h:15 -> (tris[N,16], mats[M,16]) float32 std140 records."""
    h = C.c_void_p()
    rc = lib().pt_scene_load_obj(str(obj_path).encode(), str(mtl_path).encode(), C.byref(h))
    s = _Scene(h)
    s.check(rc)
    a = s.arrays()
    return a["tris"], a["mats"]


def load_obj_robust(obj_path, mtl_path=None):
    """General Wavefront ingest (pt_scene_load_obj_ex, PT_LOAD_ROBUST) -> (tris, mats);
    mtl_path None = the OBJ's `mtllib`."""
    h = C.c_void_p()
    rc = lib().pt_scene_load_obj_ex(str(obj_path).encode(), None if mtl_path is None else str(mtl_path).encode(),
                                    1, C.byref(h))
    if not h.value:
        raise PTError(rc, "pt_scene_load_obj_ex failed")
    s = _Scene(h)
    s.check(rc)
    a = s.arrays()
    return a["tris"], a["mats"]


def buildSAHTree(tris, device=None):
    """bvh.h:255 -> nodes[K,12] {min, max, {tri0, tri1, hit, miss}} (preorder-pair layout).
    device: None = the host builder (pt_bvh_build), else the GPU builder on that device
    (pt_bvh_build_gpu; the same output)."""
    tris = _f32(tris, 16)
    n = len(tris)
    out = np.zeros((max(2 * n, 1), 12), np.float32)
    nn = C.c_int()
    src = tris.reshape(-1) if n else np.zeros(16, np.float32)
    if device is None:
        rc = lib().pt_bvh_build(src, n, out.reshape(-1), len(out), C.byref(nn))
    else:
        rc = lib().pt_bvh_build_gpu(src, n, out.reshape(-1), len(out), C.byref(nn), int(device))
    if rc:
        raise PTError(rc, lib().pt_bvh_last_error().decode())
    return out[: nn.value].copy()


class SceneBuffers(dict):
    """The five SSBO contents of setupBuffers(): tris, nodes, mats, spheres, cam."""


def setupBuffers(obj_path, mtl_path, camera=None):
    """ogl_path_trace.h:367-530: load, build the BVH, append built-ins + metal sphere."""
    h = C.c_void_p()
    rc = lib().pt_scene_load_obj(str(obj_path).encode(), str(mtl_path).encode(), C.byref(h))
    s = _Scene(h)
    s.check(rc)
    s.check(lib().pt_scene_add_builtins(s.h))
    s.check(lib().pt_scene_build_bvh(s.h))
    a = s.arrays()
    a["cam"] = DEFAULT_CAMERA.copy() if camera is None else np.asarray(camera, np.float32).reshape(12)
    return SceneBuffers(a)


def scene_from_arrays(tris, mats, builtins=True, camera=None):
    tris, mats = _f32(tris, 16), _f32(mats, 16)
    h = C.c_void_p()
    rc = lib().pt_scene_from_arrays(tris.reshape(-1) if len(tris) else np.zeros(16, np.float32), len(tris),
                                    mats.reshape(-1) if len(mats) else np.zeros(16, np.float32), len(mats), C.byref(h))
    s = _Scene(h)
    s.check(rc)
    if builtins:
        s.check(lib().pt_scene_add_builtins(s.h))
    if len(tris):
        s.check(lib().pt_scene_build_bvh(s.h))
    a = s.arrays()
    a["cam"] = DEFAULT_CAMERA.copy() if camera is None else np.asarray(camera, np.float32).reshape(12)
    return SceneBuffers(a)


def bvh_culling_ok(nodes):
    """pt_bvh_culling_ok: does the threaded tree qualify for the culling walk?"""
    n = _f32(nodes, 12)
    return bool(lib().pt_bvh_culling_ok(n.reshape(-1) if len(n) else np.zeros(12, np.float32), len(n)))


def aces_rgba8_host(img):
    img = np.ascontiguousarray(img, np.float32)
    out = np.zeros(img.shape[:-1] + (4,), np.uint8)
    lib().pt_aces_rgba8_host(img.reshape(-1), img.size // 4, out.reshape(-1))
    return out


# ----------------------------------------------------------------------------- renderer
class PathTracer:
    """The compute program + its image: pt_create / pt_upload_scene / pt_render."""

    def __init__(self, width, height, max_bounce=5, display_mode=1, flags=0, rays_per_pixel=1,
                 device=0, rank=0, world=1):
        cfg = _Config(width, height, max_bounce, display_mode, flags, rays_per_pixel, device, rank, world)
        h = C.c_void_p()
        rc = lib().pt_create(C.byref(cfg), C.byref(h))
        self.h = h
        self.width, self.height = width, height
        self._check(rc)
        rl, r0, rs = C.c_int(), C.c_int(), C.c_int()
        self._check(lib().pt_rows(self.h, C.byref(rl), C.byref(r0), C.byref(rs)))
        self.rows_local, self.row0, self.row_stride = rl.value, r0.value, rs.value

    def _check(self, rc):
        if rc:
            raise PTError(rc, lib().pt_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            lib().pt_destroy(self.h)
            self.h = None

    __del__ = close

    def upload(self, sb):
        t, n, m, s = _f32(sb["tris"], 16), _f32(sb["nodes"], 12), _f32(sb["mats"], 16), _f32(sb["spheres"], 8)
        z = lambda a, c: a.reshape(-1) if a.size else np.zeros(c, np.float32)
        self._check(lib().pt_upload_scene(self.h, z(t, 16), len(t), z(n, 12), len(n), z(m, 16), len(m), z(s, 8), len(s)))
        if "cam" in sb:
            self.set_camera(sb["cam"])

    def set_camera(self, cam):
        self._check(lib().pt_set_camera(self.h, np.ascontiguousarray(cam, np.float32).reshape(12)))

    def set_display_mode(self, mode):
        """Uniform displayMode (ogl_path_trace.h:182)."""
        self._check(lib().pt_set_display_mode(self.h, int(mode)))

    def set_counting(self, on=True):
        self._check(lib().pt_set_counting(self.h, int(bool(on))))

    def set_kernel(self, variant):
        self._check(lib().pt_set_kernel(self.h, int(variant)))

    def set_tuning(self, leaf_thresh=None, shade_thresh=None, adaptive=None, waves_per_simd=None, group=None,
                   trav_floor=None, compact_max=None, scratch_mib=None):
        if leaf_thresh is not None:
            self._check(lib().pt_set_tuning(self.h, 0, int(leaf_thresh)))
        if shade_thresh is not None:
            self._check(lib().pt_set_tuning(self.h, 1, int(shade_thresh)))
        if adaptive is not None:
            self._check(lib().pt_set_tuning(self.h, 2, int(bool(adaptive))))
        if waves_per_simd is not None:
            self._check(lib().pt_set_tuning(self.h, 3, int(waves_per_simd)))
        if group is not None:
            self._check(lib().pt_set_tuning(self.h, 5, int(group)))
        if trav_floor is not None:
            self._check(lib().pt_set_tuning(self.h, 6, int(trav_floor)))
        if compact_max is not None:
            self._check(lib().pt_set_tuning(self.h, 7, int(compact_max)))
        if scratch_mib is not None:
            self._check(lib().pt_set_tuning(self.h, 8, int(scratch_mib)))

    def set_culling(self, enable):
        """Tuning key 15: the LDS walk's conservative culling (on by default where the tree
        qualifies).  Never changes the image."""
        self._check(lib().pt_set_tuning(self.h, 15, 0 if enable else 1))

    def set_key(self, key, value):
        """Raw pt_set_tuning(key, value) (experiments)."""
        self._check(lib().pt_set_tuning(self.h, int(key), int(value)))

    def dispatch(self, frame, accumulate):
        """One glDispatchCompute with uniforms frame/accumulate (ogl_path_trace.h:176-183)."""
        self._check(lib().pt_render(self.h, frame, 1, accumulate))

    def render(self, frame_first, n_frames, accumulate_first):
        self._check(lib().pt_render(self.h, frame_first, n_frames, accumulate_first))

    def render_async(self, frame_first, n_frames, accumulate_first):
        self._check(lib().pt_render_async(self.h, frame_first, n_frames, accumulate_first))

    def sync(self):
        self._check(lib().pt_sync(self.h))

    def read_rgba32f(self):
        out = np.zeros((self.rows_local, self.width, 4), np.float32)
        self._check(lib().pt_read_rgba32f(self.h, out.ctypes.data, out.nbytes))
        return out

    def write_rgba32f(self, img):
        img = np.ascontiguousarray(img, np.float32)
        self._check(lib().pt_write_rgba32f(self.h, img.ctypes.data, img.nbytes))

    def read_rgba8(self):
        out = np.zeros((self.rows_local, self.width, 4), np.uint8)
        self._check(lib().pt_read_rgba8_aces(self.h, out.ctypes.data, out.nbytes))
        return out

    def present_begin(self, buf):
        """Enqueue the ACES RGBA8 image of the renders issued so far into pinned buffer buf
        (0..3) without waiting (pt_present_begin)."""
        self._check(lib().pt_present_begin(self.h, int(buf)))

    def present_end(self, buf, copy=True):
        """Wait for buffer buf and return its (rows_local, W, 4) uint8 pixels: a copy, or with
        copy=False a view of the pinned buffer, valid until the next present_begin(buf)."""
        ptr = C.POINTER(C.c_ubyte)()
        self._check(lib().pt_present_end(self.h, int(buf), C.byref(ptr)))
        view = np.ctypeslib.as_array(ptr, shape=(self.rows_local, self.width, 4))
        return view.copy() if copy else view

    def accum_device(self):
        p, n = C.c_void_p(), C.c_size_t()
        self._check(lib().pt_accum_device(self.h, C.byref(p), C.byref(n)))
        return p.value, n.value

    def progressive_setup(self, frames_per_launch, launches_per_replay):
        """Capture the progressive sample loop as a hipGraph (see pt_api.h)."""
        self._check(lib().pt_progressive_setup(self.h, int(frames_per_launch), int(launches_per_replay)))

    def progressive_reset(self, next_frame=1):
        self._check(lib().pt_progressive_reset(self.h, int(next_frame)))

    def progressive_run(self, replays=1, sync=True):
        self._check(lib().pt_progressive_run(self.h, int(replays)))
        if sync:
            self.sync()

    def diag(self):
        """Lane utilisation per kernel phase from the last counting render."""
        v = np.zeros(16, np.uint64)
        self._check(lib().pt_stats_ex(self.h, v))
        util = lambda w, l: float(v[l]) / max(1.0, 64.0 * float(v[w]))
        return dict(trav_iters=int(v[5]), trav_util=util(5, 6), leaf_iters=int(v[7]), leaf_util=util(7, 8),
                    seg_iters=int(v[9]), seg_util=util(9, 10), slow_segments=int(v[11]), nan_segments=int(v[12]),
                    lds_bytes=int(v[13]), lds_bytes_sinks=int(v[14]), culling_walk=bool(v[15]))

    def copy_rows_device(self, dst_ptr, nbytes):
        self._check(lib().pt_copy_rows_device(self.h, C.c_void_p(dst_ptr), nbytes))

    def timing(self, reset=False):
        ms, n = C.c_double(), C.c_int()
        self._check(lib().pt_timing(self.h, C.byref(ms), C.byref(n), int(bool(reset))))
        return ms.value, n.value

    def stream(self):
        s = C.c_void_p()
        self._check(lib().pt_stream(self.h, C.byref(s)))
        return s.value

    def stats(self):
        ms = C.c_double()
        cnt = np.zeros(5, np.uint64)
        self._check(lib().pt_stats(self.h, C.byref(ms), cnt))
        return ms.value, dict(segments=int(cnt[0]), node_visits=int(cnt[1]), tri_tests=int(cnt[2]),
                              sphere_tests=int(cnt[3]), hits=int(cnt[4]))


# ----------------------------------------------------------------------------- interactive loop
# GLFW key codes / actions the reference's key callback tests (ogl_path_trace.h:258-299)
KEY_SPACE, KEY_1, KEY_2, KEY_3, KEY_4 = 32, 49, 50, 51, 52
KEY_A, KEY_D, KEY_S, KEY_W, KEY_ESCAPE, KEY_LEFT_SHIFT = 65, 68, 83, 87, 256, 340
RELEASE, PRESS, REPEAT = 0, 1, 2


class Viewer:
    """The reference's render loop without its window (include/pt_viewer.h): GLFW
    callbacks handleMovementInput / cursorPosCallback, then one frame per frame() call."""

    def __init__(self, camera=None, display_mode=1, move_speed=10.0, rot_speed=0.1, accumulate=1):
        h = C.c_void_p()
        cam = None if camera is None else np.ascontiguousarray(camera, np.float32).reshape(12)
        rc = lib().pt_viewer_create(None if cam is None else cam.ctypes.data, int(display_mode), C.byref(h))
        if rc:
            raise PTError(rc, "pt_viewer_create")
        self.h = h
        self._cam = cam
        self._check(lib().pt_viewer_set_params(self.h, move_speed, rot_speed, int(accumulate)))

    def _check(self, rc):
        if rc:
            raise PTError(rc, "pt_viewer")

    def close(self):
        if getattr(self, "h", None):
            lib().pt_viewer_destroy(self.h)
            self.h = None

    __del__ = close

    def key(self, key, action):
        self._check(lib().pt_viewer_key(self.h, int(key), int(action)))

    def cursor(self, x, y):
        self._check(lib().pt_viewer_cursor(self.h, float(x), float(y)))

    @property
    def should_close(self):
        return bool(lib().pt_viewer_should_close(self.h))

    @staticmethod
    def _info(fi):
        return dict(camera=np.array(fi.camera[:], np.float32), frame=fi.frame, accumulate=fi.accumulate,
                    display_mode=fi.display_mode, should_close=bool(fi.should_close))

    def next(self, now):
        """Host side of one loop iteration -> its dispatch parameters."""
        fi = ViewerFrame()
        self._check(lib().pt_viewer_next(self.h, float(now), C.byref(fi)))
        return self._info(fi)

    def frame(self, pt, now):
        """One loop iteration rendered on PathTracer pt."""
        fi = ViewerFrame()
        rc = lib().pt_viewer_frame(self.h, pt.h, float(now), C.byref(fi))
        if rc:
            raise PTError(rc, lib().pt_last_error(pt.h).decode())
        return self._info(fi)


class Group:
    """pt_group.h: one process, several row-split contexts of one image -- the scene
    validated once and broadcast over RCCL, the frame gathered over RCCL and interleaved on the
    first context's device."""

    def __init__(self, tracers):
        self.tracers = list(tracers)
        arr = (C.c_void_p * len(self.tracers))(*[t.h for t in self.tracers])
        h = C.c_void_p()
        rc = lib().pt_group_create(arr, len(self.tracers), C.byref(h))
        self.h = h
        if rc:
            msg = lib().pt_group_last_error(h).decode() if h.value else ""
            self.close()
            raise PTError(rc, msg)
        t0 = self.tracers[0]
        self.W, self.H = t0.width, t0.height

    def _check(self, rc):
        if rc:
            raise PTError(rc, lib().pt_group_last_error(self.h).decode())

    def upload(self, sb):
        t, n, m, s = (_f32(sb["tris"], 16), _f32(sb["nodes"], 12), _f32(sb["mats"], 16), _f32(sb["spheres"], 8))
        flat = lambda a, c: a.reshape(-1) if len(a) else np.zeros(c, np.float32)
        self._check(lib().pt_group_upload_scene(self.h, flat(t, 16), len(t), flat(n, 12), len(n), flat(m, 16), len(m),
                                                flat(s, 8), len(s)))
        if "cam" in sb:
            for tr in self.tracers:
                tr.set_camera(sb["cam"])

    def gather(self, device_ptr=None):
        """The full (H, W, 4) frame: to host (numpy), or into device memory at device_ptr on the
        first context's device (returns None)."""
        nbytes = self.W * self.H * 16
        if device_ptr is not None:
            self._check(lib().pt_group_gather_rgba32f(self.h, C.c_void_p(device_ptr), nbytes, 1))
            return None
        out = np.zeros((self.H, self.W, 4), np.float32)
        self._check(lib().pt_group_gather_rgba32f(self.h, out.ctypes.data, nbytes, 0))
        return out

    def gather_rgba8(self, device_ptr=None):
        """The gathered frame through the ACES view (H, W, 4) uint8: to host, or into root-device
        memory at device_ptr (returns None)."""
        nbytes = self.W * self.H * 4
        if device_ptr is not None:
            self._check(lib().pt_group_gather_rgba8_aces(self.h, C.c_void_p(device_ptr), nbytes, 1))
            return None
        out = np.zeros((self.H, self.W, 4), np.uint8)
        self._check(lib().pt_group_gather_rgba8_aces(self.h, out.ctypes.data, nbytes, 0))
        return out

    def present_begin(self, buf):
        self._check(lib().pt_group_present_begin(self.h, int(buf)))

    def present_end(self, buf, copy=True):
        p = C.POINTER(C.c_ubyte)()
        self._check(lib().pt_group_present_end(self.h, int(buf), C.byref(p)))
        arr = np.ctypeslib.as_array(p, shape=(self.H, self.W, 4))
        return arr.copy() if copy else arr

    def stats(self):
        ms, b = C.c_double(), C.c_size_t()
        self._check(lib().pt_group_stats(self.h, C.byref(ms), C.byref(b)))
        return ms.value, b.value

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().pt_group_destroy(self.h)
        self.h = C.c_void_p()


def group_plan(devices, ranks):
    """pt_group_plan (host arithmetic, no device): -> dict(devices, dev_idx, slot, max_slots,
    table) for contexts on `devices` with image `ranks`."""
    n = len(devices)
    dev = np.ascontiguousarray(devices, np.int32)
    rk = np.ascontiguousarray(ranks, np.int32)
    devs, dev_idx, slot, table = (np.zeros(n, np.int32) for _ in range(4))
    nd, ms = C.c_int(0), C.c_int(0)
    rc = lib().pt_group_plan(dev, rk, n, devs, C.byref(nd), dev_idx, slot, C.byref(ms), table)
    if rc:
        raise PTError(rc, "pt_group_plan: ranks must be 0..n-1, each once")
    return dict(devices=devs[:nd.value].tolist(), dev_idx=dev_idx, slot=slot, max_slots=ms.value, table=table)


def group_interleave_host(blocks, table, world, width, height):
    """pt_group_interleave_host: the root's interleave of gathered row blocks on the host."""
    b = np.ascontiguousarray(blocks, np.float32)
    n_blocks = b.size // (max(1, -(-height // world)) * width * 4) if width and height else 0
    out = np.zeros((height, width, 4), np.float32)
    rc = lib().pt_group_interleave_host(b.reshape(-1), n_blocks, np.ascontiguousarray(table, np.int32), world,
                                        width, height, out.reshape(-1))
    if rc:
        raise PTError(rc, "pt_group_interleave_host: table entry outside the blocks")
    return out


def gather_rgba32f(tracers, device_ptr=None):
    """pt_gather_rgba32f: one-shot group + gather."""
    t0 = tracers[0]
    arr = (C.c_void_p * len(tracers))(*[t.h for t in tracers])
    nbytes = t0.width * t0.height * 16
    if device_ptr is not None:
        rc = lib().pt_gather_rgba32f(arr, len(tracers), C.c_void_p(device_ptr), nbytes, 1)
        if rc:
            raise PTError(rc, "pt_gather_rgba32f")
        return None
    out = np.zeros((t0.height, t0.width, 4), np.float32)
    rc = lib().pt_gather_rgba32f(arr, len(tracers), out.ctypes.data, nbytes, 0)
    if rc:
        raise PTError(rc, "pt_gather_rgba32f")
    return out


def assemble_rows(parts, height):
    """Interleave per-rank local rows (rank r owns rows r, r+G, ...) into a full image."""
    G = len(parts)
    W = parts[0].shape[1]
    img = np.zeros((height, W, 4), np.float32)
    for r, p in enumerate(parts):
        img[r::G][: len(p)] = p
    return img
