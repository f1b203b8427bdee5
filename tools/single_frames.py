"""One frame per dispatch, the reference's render-loop pattern (profiling helper):
python tools/single_frames.py [--frames 100] [--width 1920 --height 1080] [--scene cornell]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host as H  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=100)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--scene", default="cornell")
ap.add_argument("--keys", default="", help="tuning key=value list, comma separated")
a = ap.parse_args()
sb = H.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
pt = H.PathTracer(a.width, a.height, max_bounce=8)
pt.upload(sb)
for kv in filter(None, a.keys.split(",")):
    k, v = kv.split("=")
    pt.set_key(int(k), int(v))
for i in range(5):
    pt.render(1 + i, 1, 0 if i == 0 else 1)
pt.timing(reset=True)
t0 = time.perf_counter()
for i in range(a.frames):
    pt.render(1 + i, 1, 0 if i == 0 else 1)
dt = time.perf_counter() - t0
kms, n = pt.timing(reset=True)
print("%d single-frame dispatches: wall %.3f ms/frame, render kernels %.3f ms/frame" % (a.frames, dt * 1e3 / a.frames, kms / n))
pt.close()
