"""Screen-space locality probe for the global-memory walk: does a GPU that renders one
contiguous band of the image (the rays of 1/8 of the vertical field of view) run faster per
segment than one that renders the whole image, or every 8th row (the row split's share)?
A band is rendered as its own 1920 x H/8 image whose camera spans that band's rays
(fwd' = fwd + up * (k/8 + 1/16 - 1/2), up' = up / 8: the same ray directions up to rounding).
If bands are markedly faster, an XCD-aware work queue that keeps each XCD's L2 on one screen
region is worth building.  Timing only; one GPU.

python tools/band_locality.py --scene sponza --spp 64 [--bands 8 --rounds 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
import pt_host as H  # noqa: E402
import pt_scenes  # noqa: E402


def run(pt, spp, chunk, rounds):
    pt.set_counting(True)
    seg = 0
    for f0 in range(1, spp + 1, chunk):
        pt.render(f0, min(chunk, spp - f0 + 1), 0 if f0 == 1 else 1)
        seg += pt.stats()[1]["segments"]
    pt.set_counting(False)
    times = []
    for rnd in range(rounds + 1):
        t0 = time.perf_counter()
        for f0 in range(1, spp + 1, chunk):
            pt.render_async(f0, min(chunk, spp - f0 + 1), 0 if f0 == 1 else 1)
        pt.sync()
        if rnd:
            times.append(time.perf_counter() - t0)
    return seg, min(times)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bands", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    sb = H.setupBuffers(*pt_scenes.write_scene(a.scene, os.path.join(REPO, "scenes")))
    cam = np.asarray(sb["cam"], np.float32).copy()
    fwd, up = cam[3:6].astype(np.float64), cam[9:12].astype(np.float64)
    out = {"scene": a.scene, "width": a.width, "height": a.height, "spp": a.spp, "bands": a.bands}

    pt = H.PathTracer(a.width, a.height, max_bounce=8)
    pt.upload(sb)
    seg, dt = run(pt, a.spp, a.spp, a.rounds)
    pt.close()
    out["full"] = {"segments": seg, "s": round(dt, 5), "mrays_s": round(seg / dt / 1e6, 1)}

    pt = H.PathTracer(a.width, a.height, max_bounce=8, rank=0, world=a.bands)
    pt.upload(sb)
    seg, dt = run(pt, a.spp, a.spp, a.rounds)
    pt.close()
    out["row_share"] = {"segments": seg, "s": round(dt, 5), "mrays_s": round(seg / dt / 1e6, 1)}

    hb = a.height // a.bands
    tot_seg, tot_s, per = 0, 0.0, []
    for k in range(a.bands):
        c = cam.copy()
        c[3:6] = (fwd + up * (k / a.bands + 0.5 / a.bands - 0.5)).astype(np.float32)
        c[9:12] = (up / a.bands).astype(np.float32)
        sbk = dict(sb)
        sbk["cam"] = c
        pt = H.PathTracer(a.width, hb, max_bounce=8)
        pt.upload(sbk)
        seg, dt = run(pt, a.spp, a.spp, a.rounds)
        pt.close()
        tot_seg += seg
        tot_s += dt
        per.append(round(seg / dt / 1e6, 1))
    out["bands_mrays_s"] = per
    out["bands_total"] = {"segments": tot_seg, "s": round(tot_s, 5), "mrays_s": round(tot_seg / tot_s / 1e6, 1)}
    out["bands_over_row_share"] = round(out["bands_total"]["mrays_s"] / out["row_share"]["mrays_s"], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
