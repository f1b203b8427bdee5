"""Quick A/B of kernel variants / launch shapes on one GPU (interleaved, one process).

python tools/probe.py --spp 64 --variants 0,3 --chunks 16,64 --rounds 2
Prints Mrays/s and kernel ms per configuration; segment counts come from a counting pass.
"""
import argparse
import os
import sys
import ctypes
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))

import pt_host  # noqa: E402
import pt_scenes  # noqa: E402


def phase_clock(segments):
    """Experiment builds with -DPT_PHASE_CLOCK: wave-clock share per state-machine phase."""
    fn = getattr(pt_host.lib(), "pt_debug_phase_clock", None)
    if fn is None:
        return
    out = (ctypes.c_ulonglong * 8)()
    fn(out, 1)
    tot = float(sum(out[:3])) or 1.0
    print("  phase clock: shade %.3f leaf %.3f trav %.3f | wave-iters/segment shade %.4f leaf %.4f trav %.4f"
          " | clk per wave-iter %.0f %.0f %.0f" % (
              out[0] / tot, out[1] / tot, out[2] / tot, out[3] / segments, out[4] / segments, out[5] / segments,
              out[0] / max(out[3], 1), out[1] / max(out[4], 1), out[2] / max(out[5], 1)), flush=True)
    print("  walk: wave-steps %d lane-steps %d (util %.3f, lane-steps/segment %.2f)" % (
        out[6], out[7], out[7] / max(64.0 * out[6], 1.0), out[7] / segments), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--chunks", default="64")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--tunings", default="0:0", help="leaf:shade[:adaptive[:waves[:group[:floor[:compact]]]]] for variants 0/3, comma list")
    ap.add_argument("--world", type=int, default=1, help="render rank 0 of a WORLD-way row split (per-GPU share)")
    ap.add_argument("--flags", type=int, default=0, help="PT_FLAG_* bits (32 = Moller-Trumbore mode)")
    ap.add_argument("--key", action="append", default=[], help="pt_set_tuning key=value after each tuning (repeatable)")
    a = ap.parse_args()
    sb = pt_host.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
    pt = pt_host.PathTracer(a.width, a.height, max_bounce=a.bounces, rank=0, world=a.world, flags=a.flags)
    pt.upload(sb)
    seg = {}
    configs = [(int(v), int(c), tu) for v in a.variants.split(",") for c in a.chunks.split(",")
               for tu in (a.tunings.split(",") if int(v) in (0, 3) else ["-"])]
    def apply(v, tu):
        pt.set_kernel(v)
        if tu != "-":
            parts = [int(x) for x in tu.split(":")]
            pt.set_tuning(parts[0], parts[1], parts[2] if len(parts) > 2 else 1,
                          parts[3] if len(parts) > 3 else 0, parts[4] if len(parts) > 4 else None,
                          parts[5] if len(parts) > 5 else None, parts[6] if len(parts) > 6 else None)
        for kv in a.key:
            k, val = (int(x) for x in kv.split("="))
            pt.set_key(k, val)

    for v, c, tu in configs:
        apply(v, tu)
        pt.set_counting(True)
        total = 0
        for f0 in range(1, a.spp + 1, c):
            pt.render(f0, min(c, a.spp - f0 + 1), 0 if f0 == 1 else 1)
            st = pt.stats()[1]
            total += st["segments"]
        pt.set_counting(False)
        seg[(v, c, tu)] = total
        dg = pt.diag()
        print("variant %d chunk %d tune %s (last launch): %s  nodes/seg %.2f tri/seg %.2f" % (
            v, c, tu, {k: (round(x, 3) if isinstance(x, float) else x) for k, x in dg.items()},
            st["node_visits"] / st["segments"], st["tri_tests"] / st["segments"]), flush=True)
    for rnd in range(a.rounds):
        for v, c, tu in configs:
            apply(v, tu)
            pt.timing(reset=True)
            t0 = time.perf_counter()
            for f0 in range(1, a.spp + 1, c):
                pt.render_async(f0, min(c, a.spp - f0 + 1), 0 if f0 == 1 else 1)
            pt.sync()
            dt = time.perf_counter() - t0
            kms, n = pt.timing(reset=True)
            print("round %d variant %d chunk %4d tune %-6s: %8.1f Mrays/s  wall %.1f ms  kernel %.1f ms (%d launches)  %.3f ms/frame"
                  % (rnd, v, c, tu, seg[(v, c, tu)] / dt / 1e6, dt * 1e3, kms, n, dt * 1e3 / a.spp), flush=True)
            phase_clock(seg[(v, c, tu)])
    pt.close()


if __name__ == "__main__":
    main()
