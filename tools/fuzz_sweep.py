"""Long seeded random-scene sweep, HIP path vs oracle (the GPU fuzz test's cases at larger
images and more frames).  Prints one line per failing case and a summary; exit 1 on any
mismatch.
  python tools/fuzz_sweep.py --cases 1000 --first 100000 --scale 2
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "opengl-path-tracing_amd")]

import fuzz_scenes as F  # noqa: E402
import oracle_lib as O  # noqa: E402
import pt_host as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--first", type=int, default=100000)
    ap.add_argument("--scale", type=int, default=2, help="image size multiplier")
    ap.add_argument("--frames", type=int, default=4)
    a = ap.parse_args()
    bad = 0
    t0 = time.time()
    for i in range(a.cases):
        seed = a.first + i
        sc, kw = F.random_case(seed)
        W, Hh = kw["W"] * a.scale, kw["H"] * a.scale
        nf = 1 + seed % a.frames
        want = O.render(sc, W, Hh, max_bounce=kw["max_bounce"], mode=kw["mode"], frame_first=kw["frame_first"],
                        n_frames=nf, flags=kw["flags"])
        for variant in (0, 3):
            pt = H.PathTracer(W, Hh, max_bounce=kw["max_bounce"], display_mode=kw["mode"], flags=kw["flags"])
            pt.set_kernel(variant)
            pt.upload(sc)
            pt.render(kw["frame_first"], nf, 0)
            got = pt.read_rgba32f()
            pt.close()
            diff = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
            if diff.size:
                bad += 1
                print("MISMATCH seed %d variant %d %dx%d frames %d tris %d %s: %d words, first %s got %r want %r"
                      % (seed, variant, W, Hh, nf, len(sc["tris"]), kw, len(diff), diff[0].tolist(),
                         got[tuple(diff[0])], want[tuple(diff[0])]), flush=True)
        if (i + 1) % 50 == 0:
            print("%d cases, %d mismatches, %.0f s" % (i + 1, bad, time.time() - t0), flush=True)
    print("done: %d cases x 2 variants, %d mismatches" % (a.cases, bad))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
