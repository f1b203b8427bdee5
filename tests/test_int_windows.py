"""The unsigned-window forms of the walk guard, the normalize range test and the hit windows
(pt_math.h range_abs_u / guard_u / fast_range_u / win_open_u / win_closed_u) agree with their
float-compare forms on every input class: zeros, window edges and their neighbours, inf, NaN
and denormals of both signs, and random bit patterns (tests/math/int_windows.cpp).  The kernel's
guards use the unsigned forms; its hit windows may (PT_INT_WINDOWS), with the same image."""
import json
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integer_windows_match_float_compares(tmp_path):
    exe = str(tmp_path / "int_windows")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", "-o", exe,
                           os.path.join(REPO, "tests", "math", "int_windows.cpp")])
    r = subprocess.run([exe, "3000000", "5"], capture_output=True, text=True)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["mismatches"] == 0, r.stderr[:2000]
    assert out["checks"] > 40000000
