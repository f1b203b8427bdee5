"""Workload for PMC passes: the render launches of one bench.py configuration on this GPU --
one warm-up launch and `--launches` measured launches of the config's frames per launch.  At
--world N it is rank 0's share of the row split with N times the frames per launch, exactly
what bench.py's rank 0 launches at N GPUs.  Run under rocprofv3 --pmc ... -- python3
tools/pmc_run.py --config C3; tools/pmc_traffic.py reduces."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (CONFIGS only; bench imports torch lazily)
import pt_host  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2", choices=sorted(bench.CONFIGS))
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--chunk", type=int, default=None, help="frames per launch (default: the bench's)")
ap.add_argument("--launches", type=int, default=2)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--scene", default=None)
ap.add_argument("--width", type=int, default=None)
ap.add_argument("--height", type=int, default=None)
ap.add_argument("--key", action="append", default=[], help="pt_set_tuning key=value (repeatable)")
a = ap.parse_args()
scene, W, H, spp, bounces, chunk0, graph = bench.CONFIGS[a.config]
scene = a.scene or scene
W, H = a.width or W, a.height or H
chunk = min(a.chunk or (chunk0 * a.world if graph == 0 else chunk0), spp)
sb = pt_host.setupBuffers(*pt_scenes.write_scene(scene, os.path.join(REPO, "scenes")))
pt = pt_host.PathTracer(W, H, max_bounce=bounces, rank=0, world=a.world)
pt.set_kernel(a.variant)
for kv in a.key:
    k, v = (int(x) for x in kv.split("="))
    pt.set_key(k, v)
pt.upload(sb)
if os.environ.get("PMC_SEGMENTS"):   # the workload's segment count (counting build, same frames)
    pt.set_counting(True)
    pt.render(1, chunk, 0)
    print("segments %d" % pt.stats()[1]["segments"], flush=True)
    pt.set_counting(False)
# the bench's launch: frames 1..chunk from accumulate = 0, re-rendered (warm-up launch first)
for i in range(a.launches + 1):
    pt.render(1, chunk, 0)
pt.close()
print("pmc workload done: %s %s %dx%d world %d, %d frames per launch" % (a.config, scene, W, H, a.world, chunk))
