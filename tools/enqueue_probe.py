"""Host-side cost of enqueuing one-frame renders (pt_render_async) against the GPU time: if the
enqueue loop takes as long as the whole run, the loop is host-bound or a call blocks.
python tools/enqueue_probe.py [--frames 200]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host as H  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
a = ap.parse_args()
sb = H.setupBuffers(*pt_scenes.write_scene("cornell", os.path.join(REPO, "scenes")))
pt = H.PathTracer(a.width, a.height, max_bounce=8)
pt.upload(sb)
out = {}
cam = sb["cam"]
v = H.Viewer()
for mode in ("raw", "viewer"):
  for overlap in (3, 2, 4, 1):
    pt.set_key(9, overlap)
    for i in range(70):
        pt.render_async(1 + i, 1, 0 if i == 0 else 1)
    pt.sync()
    calls = []
    t0 = time.perf_counter()
    for i in range(a.frames):
        t1 = time.perf_counter()
        if mode == "viewer":
            v.frame(pt, 1.0 + 0.001 * i)
        else:
            if mode == "camera":
                pt.set_camera(cam)
            pt.render_async(71 + i, 1, 1)
        calls.append(time.perf_counter() - t1)
    t_enq = time.perf_counter() - t0
    pt.sync()
    t_all = time.perf_counter() - t0
    calls.sort()
    out["%s_overlap%d" % (mode, overlap)] = {"enqueue_ms_per_frame": round(t_enq * 1e3 / a.frames, 4),
                                  "total_ms_per_frame": round(t_all * 1e3 / a.frames, 4),
                                  "call_us_median": round(calls[len(calls) // 2] * 1e6, 1),
                                  "call_us_max": round(calls[-1] * 1e6, 1)}
pt.close()
print(json.dumps(out))
