"""Reduces tools/pmc_ab.sh output: per build, render-launch counters averaged over launches
(warm-up dropped), side by side."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import load  # noqa: E402


def main():
    d = sys.argv[1]
    res = {}
    for name in sorted(os.listdir(d)):
        p = os.path.join(d, name)
        if not os.path.exists(os.path.join(p, "run_counter_collection.csv")):
            continue
        lib = name.rsplit("_g", 1)[0]
        launches = load(p)[1:] or load(p)
        for ctr, ms in launches:
            for k, v in ctr.items():
                res.setdefault(lib, {}).setdefault(k, []).append(v)
            res.setdefault(lib, {}).setdefault("ms_" + name[-2:], []).append(sum(ms.values()))
    libs = sorted(res)
    keys = sorted(set(k for l in libs for k in res[l]))
    print("%-26s" % "counter" + "".join("%16s" % l for l in libs))
    for k in keys:
        print("%-26s" % k + "".join("%16.4g" % (sum(res[l].get(k, [0])) / max(len(res[l].get(k, [1])), 1)) for l in libs))


if __name__ == "__main__":
    main()
