"""Exhaustive GPU check of pt_math.h (tools/verify_fastmath.hip): the guarded fast
reciprocal / square root (rcp_fast, sqrt_fast) are bit-identical to the correctly rounded
1.0f/x and sqrtf(x) for every binary32 in the guarded range [2^-100, 2^100] (both signs for
the reciprocal) on this GPU's v_rcp_f32 / v_rsq_f32; and the pinned Box-Muller log / cos
compute on the device the same bits as on the host over their whole domains (checksums), which
tests/test_exact_div.py ties to the oracle.  The kernels use these forms only inside those
ranges."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fast_rcp_sqrt_exhaustive(tmp_path):
    exe = str(tmp_path / "verify_fastmath")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                           "-fhip-fp32-correctly-rounded-divide-sqrt",
                           os.path.join(REPO, "tools", "verify_fastmath.hip"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    print(out.stdout)
    lines = [l for l in out.stdout.splitlines() if "tested=" in l]
    assert len(lines) == 5, out.stdout + out.stderr
    for l in lines:
        assert " bad=0 " in l, l
    assert out.returncode == 0
