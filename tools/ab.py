"""Same-box A/B timing of library builds: runs tools/probe.py once per build per round,
interleaved, each in its own process (PT_LIB selects the build).

python tools/ab.py --libs base,cur --rounds 3 -- --spp 64 --variants 0 --chunks 64 --rounds 1
('cur' = build/libptrace.so, other names = build/libptrace_<name>.so from tools/ab_build.sh)
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "opengl-path-tracing_amd", "build")


def main():
    argv = sys.argv[1:]
    probe_args = []
    if "--" in argv:
        i = argv.index("--")
        argv, probe_args = argv[:i], argv[i + 1:]
    libs, rounds = ["cur"], 3
    for k in range(0, len(argv), 2):
        if argv[k] == "--libs":
            libs = argv[k + 1].split(",")
        elif argv[k] == "--rounds":
            rounds = int(argv[k + 1])
    res = {l: [] for l in libs}
    for r in range(rounds):
        for l in libs:
            path = os.path.join(BUILD, "libptrace.so" if l == "cur" else "libptrace_%s.so" % l)
            env = dict(os.environ, PT_LIB=path)
            out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "probe.py")] + probe_args,
                                 env=env, capture_output=True, text=True, timeout=900)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-2000:])
                sys.exit(out.returncode)
            vals = [float(m) for m in re.findall(r"([0-9.]+) Mrays/s", out.stdout)]
            res[l].append(vals)
            print("round %d %-6s %s" % (r, l, " ".join("%.1f" % v for v in vals)), flush=True)
    for l in libs:
        cols = list(zip(*res[l]))
        print("%-6s best %s" % (l, " ".join("%.1f" % max(c) for c in cols)))


if __name__ == "__main__":
    main()
