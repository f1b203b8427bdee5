"""Interactive-loop rate: the reference's render loop -- one dispatch per
displayed frame, ogl_path_trace.h:160-204 -- through pt_viewer_frame (pt_render_async, like
glDispatchCompute), with and without the per-frame readback a window would upload (the ACES
RGBA8 view or the raw RGBA32F accumulation; a readback waits for its frame; rgba8_present_L
is the pipelined ACES view through pt_present_begin / _end, the host showing frame f-L while
the later frames render and frame f-L+1's image crosses PCIe into pinned memory, L+1
buffers in rotation).  Each row is run
with the overlapped short launches on (default) and off (tuning key 9).  Scene and accumulator
stay in HBM.  One GPU.

python tools/interactive_fps.py [--width 1920 --height 1080 --frames 300]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host as H  # noqa: E402
import pt_scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--rows", default="none,rgba8_aces,rgba8_present_1,rgba8_present_2,rgba32f")
    ap.add_argument("--combos", default="9=0;9=1",
                    help="tuning settings to run, ';'-separated, each a ','-list of key=value (pt_set_tuning); "
                         "row suffix: '' for 9=0 (automatic overlap), '_no_overlap' for 9=1, else the settings")
    a = ap.parse_args()
    sb = H.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
    pt = H.PathTracer(a.width, a.height, max_bounce=a.bounces)
    t0 = time.perf_counter()
    pt.upload(sb)
    upload_s = time.perf_counter() - t0
    # segments per frame from an untimed counting pass over frames 1..8
    pt.set_counting(True)
    pt.render(1, 8, 0)
    seg_per_frame = pt.stats()[1]["segments"] / 8.0
    pt.set_counting(False)
    out = {"width": a.width, "height": a.height, "bounces": a.bounces, "scene": a.scene, "frames": a.frames,
           "scene_upload_ms": round(upload_s * 1e3, 3), "segments_per_frame": seg_per_frame}
    touched = set()
    for combo in a.combos.split(";"):
        kv = [tuple(int(x) for x in item.split("=")) for item in combo.split(",") if item]
        for k in touched:                                     # back to automatic
            pt.set_key(k, 0)
        for k, v in kv:
            pt.set_key(k, v)
            touched.add(k)
        suffix = {"9=0": "", "9=1": "_no_overlap"}.get(combo, "_" + combo.replace("=", "_").replace(",", "_"))
        for readback in a.rows.split(","):
            v = H.Viewer()
            for i in range(70):                               # warm-up (and the first tile sorts)
                v.frame(pt, 0.001 * i)
            pt.sync()
            t0 = time.perf_counter()
            for i in range(a.frames):
                v.frame(pt, 1.0 + 0.001 * i)                  # enqueued, like glDispatchCompute
                if readback == "rgba8_aces":
                    pt.read_rgba8()
                elif readback.startswith("rgba8_present_"):
                    lag = int(readback.rsplit("_", 1)[1])
                    pt.present_begin(i % (lag + 1))
                    if i >= lag:                                  # frame i-lag, shown while later ones render
                        pt.present_end((i - lag) % (lag + 1), copy=False)
                elif readback == "rgba32f":
                    pt.read_rgba32f()
            if readback.startswith("rgba8_present_"):
                lag = int(readback.rsplit("_", 1)[1])
                for j in range(max(0, a.frames - lag), a.frames):
                    pt.present_end(j % (lag + 1), copy=False)
            pt.sync()
            dt = time.perf_counter() - t0
            v.close()
            name = readback + suffix
            while name in out:                                # a repeated setting: keep every row
                name += "+"
            out[name] = {
                "ms_per_frame": round(dt * 1e3 / a.frames, 4), "fps": round(a.frames / dt, 1),
                "mrays_per_s": round(seg_per_frame * a.frames / dt / 1e6, 1)}
    pt.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
