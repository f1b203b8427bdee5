"""The exact-reciprocal slab quotient: under the kernel's guard,
q0 = a*rd; r = fma(-q0, d, a); q = fma(r, rd, q0) with rd = RN(1/d) equals RN(a/d) bit for
bit (Markstein's theorem).  Checked here on the host with IEEE fmaf over 2e7 random pairs
spanning the guarded ranges plus structured near-tie cases; the GPU kernels use the same
v_fma_f32 sequence and are checked image-wise by tests/test_gpu_parity.py."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static float bf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
int main(int argc, char** argv) {
    long long n = atoll(argv[1]), bad = 0;
    for (long long i = 0; i < n; i++) {
        uint64_t r = rnd(), r2 = rnd();
        /* |d| in [2^-20, 2): the ray half of the guard */
        float d = bf(((127u - 20u + (uint32_t)(r % 21)) << 23) | (uint32_t)((r >> 8) & 0x7fffff) | (uint32_t)((r >> 40) & 1u) << 31);
        /* a = b - o with b, o each 0 or in [2^-40, 2^60]: |a| in {0} U [2^-63, 2^61] */
        uint32_t ea = 127u - 63u + (uint32_t)(r2 % 125);
        if (ea > 127u + 60u) ea = 127u + 60u;
        float a = bf((ea << 23) | (uint32_t)((r2 >> 8) & 0x7fffff) | (uint32_t)((r2 >> 40) & 1u) << 31);
        switch ((r2 >> 50) & 15) {
            case 0: a = d * (float)((r2 >> 20) % 4096); break;             /* exact multiples */
            case 1: a = 0.0f; break;
            case 2: a = bf(fb(d * 3.0f) + (uint32_t)((r2 >> 20) % 3) - 1u); break;   /* near ties */
            default: break;
        }
        float rd = 1.0f / d;
        float q0 = a * rd;
        float rem = fmaf(-q0, d, a);
        float q = fmaf(rem, rd, q0);
        float ex = a / d;
        if (fb(q) != fb(ex) && !(q == 0.0f && ex == 0.0f)) {
            if (bad < 5) printf("a=%a d=%a got %a want %a\n", a, d, q, ex);
            bad++;
        }
    }
    printf("n=%lld bad=%lld\n", n, bad);
    return bad != 0;
}
"""


PROG_CAM = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 0x2545F4914F6CDD1Dull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
int main(void) {
    long long bad = 0, n = 0;
    for (int W = 1; W <= 65536; W++) {
        float w = (float)W, rw = 1.0f / w;
        for (int k = 0; k < 400; k++) {
            uint64_t r = rnd();
            int x = (int)(r % (uint64_t)(W + 1));
            float j = (float)(uint32_t)(r >> 32) * (1.0f / 4294967296.0f);   /* random() in [0,1] */
            if (k == 0) j = 0.0f;
            if (k == 1) j = 1.0f;
            float a = (float)x + j;
            float q0 = a * rw, rem = fmaf(-q0, w, a), q = fmaf(rem, rw, q0), ex = a / w;
            n++;
            if (fb(q) != fb(ex)) { if (bad < 5) printf("a=%a W=%d got %a want %a\n", a, W, q, ex); bad++; }
        }
    }
    printf("n=%lld bad=%lld\n", n, bad);
    return bad != 0;
}
"""


def test_camera_quotient_is_correctly_rounded(tmp_path):
    """The kernel's camera ray divides (x + jitter) by W with RN(1/W) and a Markstein
    correction (pt_render.hip): every W in [1, 2^16] with 400 numerators each, including
    jitter 0 and 1, against IEEE division."""
    src = tmp_path / "cam.c"
    src.write_text(PROG_CAM)
    exe = tmp_path / "cam"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-march=x86-64-v3", str(src), "-o", str(exe), "-lm"])
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "bad=0" in out.stdout


def test_markstein_quotient_is_correctly_rounded(tmp_path):
    src = tmp_path / "mk.c"
    src.write_text(PROG)
    exe = tmp_path / "mk"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-march=x86-64-v3", str(src), "-o", str(exe), "-lm"])
    out = subprocess.run([str(exe), "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "bad=0" in out.stdout


def test_pinned_log_cos_match_the_oracle(tmp_path):
    """The kernels' pinned log / cos (pt_math.h logf_pinned / cosf_pinned, compiled here for
    the host) return the oracle's bits (oracle/pt_oracle.cpp, a separate restatement): every
    7th binary32 of the hot-path domains (tools/verify_bf.cpp; stride 1 runs the exhaustive
    check in ~10 s on 8 threads, and tools/verify_fastmath.hip checks on the GPU that the
    device computes the host's bits on the whole domains)."""
    exe = tmp_path / "verify_bf"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", "-pthread",
                           os.path.join(REPO, "tools", "verify_bf.cpp"), os.path.join(REPO, "oracle", "pt_oracle.cpp"),
                           "-o", str(exe)])
    out = subprocess.run([str(exe), "7"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    lines = [l for l in out.stdout.splitlines() if "tested=" in l]
    assert len(lines) == 2 and all(" bad=0" in l for l in lines), out.stdout


PROG_DIVG = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 0x853C49E6748FEA9Bull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static float bf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
int main(int argc, char** argv) {
    long long n = atoll(argv[1]), bad = 0;
    for (long long i = 0; i < n; i++) {
        uint64_t r = rnd(), r2 = rnd();
        /* both magnitudes in [2^-60, 2^60]: div_g's fast range (pt_math.h) */
        float den = bf(((127u - 60u + (uint32_t)(r % 121)) << 23) | (uint32_t)((r >> 8) & 0x7fffff) | (uint32_t)((r >> 40) & 1u) << 31);
        float num = bf(((127u - 60u + (uint32_t)(r2 % 121)) << 23) | (uint32_t)((r2 >> 8) & 0x7fffff) | (uint32_t)((r2 >> 40) & 1u) << 31);
        switch ((r2 >> 50) & 7) {
            case 0: num = den * (float)((r2 >> 20) % 4096 + 1); break;      /* exact multiples */
            case 1: num = bf(fb(den * 3.0f) + (uint32_t)((r2 >> 20) % 3) - 1u); break;   /* near ties */
            case 2: den = bf(fb(den) | 0x7fffffu); break;                  /* all-ones mantissa */
            default: break;
        }
        float an = fabsf(num), ad = fabsf(den);
        if (!(an >= 0x1p-60f && an <= 0x1p60f && ad >= 0x1p-60f && ad <= 0x1p60f)) continue;
        float rd = 1.0f / den, q0 = num * rd, rem = fmaf(-q0, den, num), q = fmaf(rem, rd, q0);
        float ex = num / den;
        if (fb(q) != fb(ex)) { if (bad < 5) printf("num=%a den=%a got %a want %a\n", num, den, q, ex); bad++; }
    }
    printf("n=%lld bad=%lld\n", n, bad);
    return bad != 0;
}
"""


def test_guarded_division_is_correctly_rounded(tmp_path):
    """pt_math.h div_g (the guarded quotient; the kernel's sphere root uses the IEEE sequence
    since round 5, DESIGN.md §6, and the camera ray div_mk under a static guard): the exact
    reciprocal + Markstein correction over its guard (both magnitudes in [2^-60, 2^60]),
    2e7 random pairs incl. exact multiples, near ties and all-ones divisor mantissas."""
    src = tmp_path / "dg.c"
    src.write_text(PROG_DIVG)
    exe = tmp_path / "dg"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-march=x86-64-v3", str(src), "-o", str(exe), "-lm"])
    out = subprocess.run([str(exe), "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "bad=0" in out.stdout


def test_length_threshold_without_root():
    """pt_math.h length_gt_001: dot(c,c) >= 0x38d1b719 <=> RN(sqrt(dot(c,c))) > 0.01f, for
    every non-negative binary32 (and NaN), against the IEEE root."""
    import numpy as np
    thr = np.uint32(0x38d1b719)
    step = 1 << 26
    for base in range(0, 0x7f800001 + step, step):
        u = np.arange(base, min(base + step, 0x7fc00001), dtype=np.uint32)
        if u.size == 0:
            break
        q = u.view(np.float32)
        with np.errstate(invalid="ignore"):
            want = np.sqrt(q) > np.float32(0.01)
        got = q >= thr.view(np.float32)
        assert np.array_equal(want, got), hex(int(u[np.argmax(want != got)]))
