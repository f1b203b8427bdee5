"""Wavefront-kernel (variant 4) diagnostics from a -DPT_WF_DIAG build:
PT_LIB=.../libptrace_wfdiag.so python tools/wfdiag.py [--spp 64] [--keys 11=40,12=64]"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--scene", default="cornell")
ap.add_argument("--keys", default="")
ap.add_argument("--variant", type=int, default=4)
a = ap.parse_args()
sb = pt_host.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
pt = pt_host.PathTracer(1920, 1080, max_bounce=8)
pt.upload(sb)
pt.set_counting(True)
pt.render(1, a.spp, 0)
seg = pt.stats()[1]["segments"]
pt.set_counting(False)
pt.set_kernel(a.variant)
for kv in filter(None, a.keys.split(",")):
    k, v = kv.split("=")
    pt.set_key(int(k), int(v))
fn = pt_host.lib().pt_debug_wf_diag
out = (ctypes.c_ulonglong * 16)()
for rnd in range(2):
    fn(out, 1)
    t0 = time.perf_counter()
    pt.render(1, a.spp, 0)
    dt = time.perf_counter() - t0
    fn(out, 1)
    v = list(out)
    clk = sum(v[7:11]) or 1
    print("round %d: %.1f Mrays/s" % (rnd, seg / dt / 1e6))
    print("  walk: wave-steps/seg %.3f lane util %.3f | leaf: batches/seg %.4f lanes/batch %.1f | shade: batches/seg %.4f"
          " lanes/batch %.1f | sleeps/seg %.4f refill lanes/seg %.2f pop waits %d" % (
              v[0] / seg, v[1] / max(1, 64 * v[0]), v[2] / seg, v[3] / max(1, v[2]), v[4] / seg, v[5] / max(1, v[4]),
              v[6] / seg, v[11] / seg, v[12]))
    print("  clock share: walk %.3f leaf %.3f shade %.3f idle %.3f | clk per seg %.1f" % (
        v[7] / clk, v[8] / clk, v[9] / clk, v[10] / clk, clk / seg))
pt.close()
