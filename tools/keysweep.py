"""Same-process A/B of pt_set_tuning settings on one scene (interleaved rounds).

python tools/keysweep.py --scene bunny --spp 64 --configs "9=256;9=768" --rounds 3
Each config is a ';'-separated entry of comma-separated key=value pairs (pt_api.h keys).
"""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host  # noqa: E402
import pt_scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--tris", type=int, default=0, help="generator target_tris (bunny / sponza)")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--configs", default="")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    chunk = a.chunk or a.spp
    cfgs = [[tuple(int(x) for x in kv.split("=")) for kv in c.split(",") if kv] for c in a.configs.split(";")]
    kw = {"target_tris": a.tris} if a.tris else {}
    sdir = os.path.join(REPO, "scenes", "%s_%d" % (a.scene, a.tris)) if a.tris else os.path.join(REPO, "scenes")
    sb = pt_host.setupBuffers(*pt_scenes.write_scene(a.scene, sdir, **kw))
    pt = pt_host.PathTracer(a.width, a.height, max_bounce=a.bounces, world=a.world)
    pt.set_kernel(a.variant)
    pt.upload(sb)
    pt.set_counting(True)
    seg = 0
    for f0 in range(1, a.spp + 1, chunk):
        pt.render(f0, min(chunk, a.spp - f0 + 1), 0 if f0 == 1 else 1)
        seg += pt.stats()[1]["segments"]
    pt.set_counting(False)
    ref = pt.read_rgba32f()
    res = [[] for _ in cfgs]
    for rnd in range(a.rounds + 1):
        for i, cfg in enumerate(cfgs):
            for k, v in cfg:
                pt.set_key(k, v)
            t0 = time.perf_counter()
            for f0 in range(1, a.spp + 1, chunk):
                pt.render_async(f0, min(chunk, a.spp - f0 + 1), 0 if f0 == 1 else 1)
            pt.sync()
            dt = time.perf_counter() - t0
            img = pt.read_rgba32f()
            same = bool((img.view("u4") == ref.view("u4")).all())
            for k, v in cfg:            # back to the defaults
                pt.set_key(k, 0 if k not in (2, 7) else (1 if k == 2 else 63))
            if rnd:
                res[i].append(seg / dt / 1e6)
                print("round %d cfg %-16s %9.1f Mrays/s  %.3f ms/frame  image %s" % (
                    rnd, a.configs.split(";")[i] or "default", res[i][-1], dt * 1e3 / a.spp,
                    "identical" if same else "DIFFERS"), flush=True)
    base = statistics.median(res[0])
    for i, r in enumerate(res):
        m = statistics.median(r)
        print("cfg %-16s median %9.1f Mrays/s (%+.2f%%)" % (a.configs.split(";")[i] or "default", m, 100 * (m / base - 1)))
    pt.close()


if __name__ == "__main__":
    main()
