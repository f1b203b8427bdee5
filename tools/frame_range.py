"""Per-launch timing over consecutive frame ranges (diagnoses frame-dependent cost).
python tools/frame_range.py --scene bunny --chunk 32 --launches 4"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell")
ap.add_argument("--chunk", type=int, default=32)
ap.add_argument("--launches", type=int, default=4)
ap.add_argument("--group", type=int, default=0)
ap.add_argument("--adaptive", type=int, default=1)
ap.add_argument("--no-count", action="store_true")
ap.add_argument("--starts", default="", help="explicit comma list of first frames")
a = ap.parse_args()
sb = pt_host.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
pt = pt_host.PathTracer(1920, 1080, max_bounce=8)
pt.upload(sb)
pt.set_tuning(group=a.group, adaptive=a.adaptive)
for rnd in range(2):
    starts = [int(x) for x in a.starts.split(",")] if a.starts else [1 + i * a.chunk for i in range(a.launches)]
    for f0 in starts:
        seg = 0
        if not a.no_count:
            pt.set_counting(True)
            pt.render(f0, a.chunk, 0 if f0 == 1 else 1)
            stt = pt.stats()[1]
            seg = stt["segments"]
            print("   counts", stt, pt.diag(), flush=True)
            pt.set_counting(False)
        t0 = time.perf_counter()
        pt.render(f0, a.chunk, 0 if f0 == 1 else 1)
        dt = time.perf_counter() - t0
        print("round %d frames %d..%d: %.1f ms, %d segments, %.1f Mrays/s" % (
            rnd, f0, f0 + a.chunk - 1, dt * 1e3, seg, seg / dt / 1e6), flush=True)
pt.close()
