"""Same-process A/B timing of library builds: every build is loaded into ONE process (its own
ctypes handle through its own copy of pt_host), and their renders are interleaved round by
round, so clock and thermal drift between processes does not enter the comparison.

python tools/ab_inproc.py --libs base,cur --rounds 4 --spp 128 --chunk 128 [--scene bunny [--tris 300]]
('cur' = build/libptrace.so, other names = build/libptrace_<name>.so from tools/ab_build.sh;
 an entry name:k=v[:k=v] adds pt_set_tuning keys for that entry only, e.g. --libs cur,p37:3=8)

The build order rotates every round (each build is timed first equally often): a fixed order
favoured the later entries by about 0.25% (ABBA runs, profiles/ab/r06n_*).

Launches of at most 16 frames run overlapped on extra streams (tuning key 9), and the contexts
of every build after the first then share the process's hardware queues (GPU_MAX_HW_QUEUES=4)
with the first's: measured 15-25% slower whichever build comes second.  Compare such launch
shapes one build per process (or with --key 9=1 for all).
"""
import argparse
import importlib.util
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "opengl-path-tracing_amd")
sys.path.insert(0, PKG)
import pt_scenes  # noqa: E402


def load_host(name):
    path = os.path.join(PKG, "build", "libptrace.so" if name == "cur" else "libptrace_%s.so" % name)
    os.environ["PT_LIB"] = path
    os.environ["PT_LIB_PARTIAL"] = "1" if name != "cur" else "0"
    spec = importlib.util.spec_from_file_location("pt_host_" + name, os.path.join(PKG, "pt_host.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.LIB_PATH == path
    mod.lib()   # bind now, while PT_LIB_PARTIAL describes this build
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="base,cur")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--chunk", type=int, default=128)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--tris", type=int, default=0, help="generator target_tris (bunny / sponza)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--world", type=int, default=1, help="render rank 0 of a WORLD-way row split (per-GPU share)")
    ap.add_argument("--rank", type=int, default=0, help="... or this rank of it")
    ap.add_argument("--key", action="append", default=[], help="pt_set_tuning key=value for every build (repeatable)")
    a = ap.parse_args()
    libs = a.libs.split(",")
    if len(libs) > 1 and min(a.chunk, a.spp) <= 16 and not any(k.startswith("9=") for k in a.key):
        print("warning: overlapped short launches of several builds share hardware queues; the order "
              "biases the result (run one build per process, or --key 9=1)", flush=True)
    mods = {}
    for l in libs:
        name = l.split(":")[0]
        if name not in mods:
            mods[name] = load_host(name)
    hosts = {l: mods[l.split(":")[0]] for l in libs}
    own_keys = {l: l.split(":")[1:] for l in libs}
    kw = {"target_tris": a.tris} if a.tris else {}
    obj, mtl = pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes", "%s_%d" % (a.scene, a.tris)) if a.tris
                                     else os.path.join(REPO, "scenes"), **kw)
    pts, seg = {}, {}
    for l in libs:
        H = hosts[l]
        pt = H.PathTracer(a.width, a.height, max_bounce=8, rank=a.rank, world=a.world)
        pt.upload(H.setupBuffers(obj, mtl))
        for kv in a.key + own_keys[l]:
            k, v = (int(x) for x in kv.split("="))
            pt.set_key(k, v)
        pt.set_counting(True)
        total = 0
        for f0 in range(1, a.spp + 1, a.chunk):
            pt.render(f0, min(a.chunk, a.spp - f0 + 1), 0 if f0 == 1 else 1)
            total += pt.stats()[1]["segments"]
        pt.set_counting(False)
        pts[l], seg[l] = pt, total
    if len(set(seg.values())) != 1:   # builds that change the image (timing experiments)
        print("segment counts differ between builds (each build's own count is used): %s" % seg)
    res = {l: [] for l in libs}
    # the order rotates every round: the build timed first in a round measured about 0.25% slow
    # (ABBA runs of identical settings, profiles/ab/r06n_*), so a fixed order biased every A/B
    # by up to that much in favour of the later entries
    for rnd in range(a.rounds + 1):             # round 0 warms every build up
        k = rnd % len(libs)
        for l in libs[k:] + libs[:k]:
            pt = pts[l]
            t0 = time.perf_counter()
            for f0 in range(1, a.spp + 1, a.chunk):
                pt.render_async(f0, min(a.chunk, a.spp - f0 + 1), 0 if f0 == 1 else 1)
            pt.sync()
            dt = time.perf_counter() - t0
            if rnd:
                res[l].append(seg[l] / dt / 1e6)
                print("round %d %-8s %9.1f Mrays/s" % (rnd, l, res[l][-1]), flush=True)
    base = statistics.median(res[libs[0]])
    for l in libs:
        m = statistics.median(res[l])
        print("%-8s median %9.1f  best %9.1f  (%+.2f%% vs %s)" % (l, m, max(res[l]), 100.0 * (m / base - 1.0), libs[0]))
    for pt in pts.values():
        pt.close()


if __name__ == "__main__":
    main()
