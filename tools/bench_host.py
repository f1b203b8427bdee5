"""Host ingest timing: the product's exact BVH builder and loaders
against the oracle's literal restatement of the reference builder (bvh.h:173-268, with its
O(N^2) first-equal std::find per leaf), on the benchmark scenes.  CPU only.

python tools/bench_host.py [--out profiles/host_ingest.json]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
import pt_host as H  # noqa: E402
import pt_scenes  # noqa: E402


def timed(fn, *a):
    t0 = time.perf_counter()
    r = fn(*a)
    return r, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "host_ingest.json"))
    ap.add_argument("--scenes", default="cornell,bunny,sponza")
    a = ap.parse_args()
    rows = []
    for name in a.scenes.split(","):
        obj, mtl = pt_scenes.write_scene(name, os.path.join(REPO, "scenes"))
        mb = (os.path.getsize(obj) + os.path.getsize(mtl)) / 1e6
        (tris, mats), t_load = timed(H.load_vertex_data, obj, mtl)
        _, t_rob = timed(H.load_obj_robust, obj, mtl)
        nodes, t_build = timed(H.buildSAHTree, tris)
        onodes, t_oracle = timed(O.build_bvh, tris)
        same = bool(np.array_equal(np.ascontiguousarray(nodes).view(np.uint32), np.ascontiguousarray(onodes).view(np.uint32)))
        row = dict(scene=name, triangles=int(len(tris)), nodes=int(len(nodes)), file_mb=round(mb, 2),
                   load_s=round(t_load, 4), load_robust_s=round(t_rob, 4), build_s=round(t_build, 4),
                   oracle_literal_build_s=round(t_oracle, 3), build_speedup=round(t_oracle / max(t_build, 1e-9), 1),
                   identical_nodes=same)
        rows.append(row)
        print(json.dumps(row), flush=True)
    with open(a.out, "w") as fh:
        json.dump({"host": os.uname().nodename, "cpu_count": os.cpu_count(), "rows": rows}, fh, indent=1)


if __name__ == "__main__":
    main()
