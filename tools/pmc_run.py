"""Workload for PMC passes: the bench configuration's render kernel, one warm-up launch and
`--launches` measured launches of `--chunk` frames (C2: Cornell 1920x1080, 8 bounces).
Run under rocprofv3 --pmc ... -- python3 tools/pmc_run.py; tools/pmc_traffic.py reduces."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))

import pt_host  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chunk", type=int, default=128)
ap.add_argument("--launches", type=int, default=2)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--scene", default="cornell")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--key", action="append", default=[], help="pt_set_tuning key=value (repeatable)")
a = ap.parse_args()
sb = pt_host.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
pt = pt_host.PathTracer(a.width, a.height, max_bounce=8)
pt.set_kernel(a.variant)
for kv in a.key:
    k, v = (int(x) for x in kv.split("="))
    pt.set_key(k, v)
pt.upload(sb)
if os.environ.get("PMC_SEGMENTS"):   # the workload's segment count (counting build, same frames)
    pt.set_counting(True)
    pt.render(1, a.chunk, 0)
    print("segments %d" % pt.stats()[1]["segments"], flush=True)
    pt.set_counting(False)
# the bench's step: frames 1..chunk from accumulate = 0, re-rendered (warm-up launch first)
for i in range(a.launches + 1):
    pt.render(1, a.chunk, 0)
pt.close()
print("pmc workload done")
