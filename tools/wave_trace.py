"""Per-wave timeline of one render launch (experiment build with -DPT_WAVE_TRACE):
PT_LIB=.../libptrace_wt.so python tools/wave_trace.py [--frames 1] [--reps 20]
Reports, relative to the first wave's entry: when waves entered (the ramp), how long the LDS
staging took, when they exited (the tail), and the idle share of resident wave-time."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host as H  # noqa: E402
import pt_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=1)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--scene", default="cornell")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--world", type=int, default=1, help="rank 0 of a WORLD-way row split")
a = ap.parse_args()
sb = H.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
pt = H.PathTracer(a.width, a.height, max_bounce=8, rank=0, world=a.world)
pt.upload(sb)
pt.set_key(9, 1)
fn = H.lib().pt_debug_wave_trace
fn.restype = C.c_int
fn.argtypes = [np.ctypeslib.ndpointer(np.uint64), C.c_int, C.c_int]
N = 16384
buf = np.zeros(4 * N, np.uint64)
f = 1
res = []
warm = 5 if a.frames <= 64 else 1
for r in range(a.reps + warm):
    fn(buf, N, 1)
    pt.render(f, a.frames, 0 if f == 1 else 1)
    f += a.frames
    fn(buf, N, 0)
    t = buf.reshape(N, 4).astype(np.int64)
    t = t[t[:, 0] > 0]
    if r < warm:
        continue
    t0 = t[:, 0].min()
    entry, staged, end, items = (t[:, 0] - t0) * 10.0, (t[:, 1] - t0) * 10.0, (t[:, 2] - t0) * 10.0, t[:, 3]
    dur = end.max()
    busy = items > 0
    res.append(dict(waves=int(len(t)), busy_waves=int(busy.sum()), launch_us=float(dur),
                    entry_p50=float(np.percentile(entry, 50)), entry_p99=float(np.percentile(entry, 99)),
                    entry_busy_max=float(entry[busy].max()),
                    staging_us_p50=float(np.percentile((staged - entry)[busy], 50)),
                    end_busy_p10=float(np.percentile(end[busy], 10)), end_busy_p50=float(np.percentile(end[busy], 50)),
                    end_busy_p90=float(np.percentile(end[busy], 90)),
                    idle_frac=float(((dur - end[busy]) + entry[busy]).sum() / (busy.sum() * dur))))
keys = res[0].keys()
print(json.dumps({k: round(float(np.median([r[k] for r in res])), 2) for k in keys}))
pt.close()
