"""The drop-in boundary: libptrace.so loads on a CPU-only host, exports every symbol that
include/*.h declares, and the headers are plain C (a C program links against it)."""
import ctypes
import os
import subprocess

import pytest

import pt_host as H

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(H.LIB_PATH)
    names = H.header_symbols()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    H.lib()
    L = H.lib()
    for n in H.header_symbols():
        assert getattr(L, n).argtypes is not None or getattr(L, n).restype is None, n


def test_oracle_is_not_linked_into_product():
    out = subprocess.run(["nm", "-D", "--defined-only", H.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in out
    ldd = subprocess.run(["ldd", H.LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in ldd


C_PROG = r"""
#include "pt_api.h"
#include "pt_scene.h"
#include <stdio.h>
int main(int argc, char** argv) {
    pt_scene* s = 0;
    int rc = pt_scene_load_obj(argv[1], argv[2], &s);
    if (!rc) rc = pt_scene_add_builtins(s);
    if (!rc) rc = pt_scene_build_bvh(s);
    int c[5];
    pt_scene_counts(s, c);
    printf("%d %d %d %d %d %d\n", rc, c[0], c[1], c[2], c[3], c[4]);
    pt_scene_free(s);
    pt_config cfg = {64, 64, 5, 1, 0, 1, 0, 0, 1};
    (void)cfg;
    return rc;
}
"""


def test_headers_are_c_and_link(tmp_path, cornell_paths):
    src = tmp_path / "abi.c"
    src.write_text(C_PROG)
    exe = tmp_path / "abi"
    build = os.path.dirname(H.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"), str(src),
                           "-o", str(exe), "-L", build, "-lptrace", "-Wl,-rpath," + build])
    out = subprocess.run([str(exe), *cornell_paths], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["0", "36", "11", "1", "35", "6"]


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(H.PTError) as e:
        H.PathTracer(32, 32)
    assert e.value.code == -5


def test_bench_roofline_needs_the_profiled_build(tmp_path):
    """bench.py's VALU roofline uses a PMC pass only for the exact library it profiled
    (sha256) and the same workload; otherwise frac is null with the reason."""
    import hashlib
    import json
    import bench
    lib = tmp_path / "libptrace.so"
    lib.write_bytes(b"build A")
    tj = tmp_path / "traffic.json"
    meta = dict(scene="cornell", width=1920, height=1080, chunk=1024, valu_instr_per_launch=1.0)
    tj.write_text(json.dumps(dict(meta, lib_sha256=hashlib.sha256(b"build A").hexdigest())))
    pmc, stale, sha = bench.pmc_for(str(tj), str(lib), 1920, 1080, 1024, "cornell", 1)
    assert pmc is not None and stale is None and sha == hashlib.sha256(b"build A").hexdigest()
    lib.write_bytes(b"build B")                  # rebuilt kernel, no fresh PMC pass
    pmc, stale, _ = bench.pmc_for(str(tj), str(lib), 1920, 1080, 1024, "cornell", 1)
    assert pmc is None and "another build" in stale
    lib.write_bytes(b"build A")
    pmc, stale, _ = bench.pmc_for(str(tj), str(lib), 1920, 1080, 128, "cornell", 1)   # other launch shape
    assert pmc is None and "another workload" in stale
    pmc, stale, _ = bench.pmc_for(str(tmp_path / "missing.json"), str(lib), 1920, 1080, 1024, "cornell", 1)
    assert pmc is None and "no PMC pass" in stale


def test_bench_roofline_per_rank_share_and_bounds(tmp_path):
    """At N > 1 rank 0's line may carry the roofline of its own share when the PMC pass was of
    that share (world recorded in the summary); the bound is the unit with the larger
    utilisation, with occupancy from SQ_WAVE_CYCLES (quad-cycles) against 8 wave slots."""
    import hashlib
    import json
    import bench
    lib = tmp_path / "libptrace.so"
    lib.write_bytes(b"build A")
    sha = hashlib.sha256(b"build A").hexdigest()
    tj = tmp_path / "C2_w2.json"
    clk, t_ms = 2.4, 100.0
    cyc = clk * 1e9 * t_ms * 1e-3            # cycles of the launch
    ctr = {"SQ_INSTS_VALU": 0.5 * 512 * cyc,   # VALU busy 0.5 of 1024 SIMDs x clk / 2
           "TD_TD_BUSY_sum": 0.9 * 256 * cyc,  # TD busy 0.9
           "SQ_WAVE_CYCLES": 6.0 * 1024 * cyc / 4.0, "GRBM_GUI_ACTIVE": 8 * cyc,
           "SQ_THREAD_CYCLES_VALU": 40.0 * 1e9, "SQ_ACTIVE_INST_VALU": 1e9,
           "TCC_HIT_sum": 90.0, "TCC_MISS_sum": 10.0}
    tj.write_text(json.dumps(dict(scene="cornell", width=1920, height=1080, chunk=2048, world=2, lib_sha256=sha,
                                  counters_per_launch=ctr, clock_ghz=clk)))
    pmc, stale, _ = bench.pmc_for(str(tj), str(lib), 1920, 1080, 2048, "cornell", 2)
    assert pmc is not None and stale is None
    pmc1, stale1, _ = bench.pmc_for(str(tj), str(lib), 1920, 1080, 2048, "cornell", 1)
    assert pmc1 is None and "another workload" in stale1
    r = bench.roofline_from(pmc, None, sha, t_ms, 1, 1e9, 1e12)
    assert r["bound"] == "texture" and abs(r["frac"] - 0.9) < 1e-3
    assert abs(r["bounds"]["valu"]["frac"] - 0.5) < 1e-3
    assert abs(r["occupancy"]["waves_per_simd"] - 6.0) < 1e-6 and r["occupancy"]["peak"] == 8
    assert r["active_lanes_per_valu"] == 40.0 and r["memory_pipe"]["l2_hit_rate"] == 0.9
    none = bench.roofline_from(None, "no PMC pass", sha, t_ms, 1, 1e9, 1e12)
    assert none["frac"] is None and none["pmc_stale"] == "no PMC pass"


def test_bench_texture_bound_ranked_unstalled():
    """The texture unit's busy figure includes cycles stalled on L1 (TD_TC_STALL): the line
    reports stall_frac and unstalled_frac, and the bound is chosen on the unstalled share, so
    a walk whose TD is 95% busy but 61% stalled reports its VALU bound instead."""
    import bench
    clk, t_ms = 2.4, 100.0
    cyc = clk * 1e9 * t_ms * 1e-3
    ctr = {"SQ_INSTS_VALU": 0.73 * 512 * cyc, "TD_TD_BUSY_sum": 0.95 * 256 * cyc,
           "TD_TC_STALL_sum": 0.61 * 0.95 * 256 * cyc}
    r = bench.roofline_from({"counters_per_launch": ctr, "clock_ghz": clk}, None, "0" * 64, t_ms, 1, 1e9, 1e12)
    tx = r["bounds"]["texture"]
    assert abs(tx["stall_frac"] - 0.61) < 1e-3 and abs(tx["unstalled_frac"] - 0.95 * 0.39) < 1e-3
    assert r["bound"] == "valu" and abs(r["frac"] - 0.73) < 1e-3


def test_bench_roofline_partial_counters():
    """A PMC summary holding only some counter groups (a hand-made or partial one) must not
    stop the line: fields whose counters are missing are left out."""
    import bench
    ctr = {"SQ_INSTS_VALU": 1e9, "SQ_ACTIVE_INST_VALU": 1e8, "TCP_TOTAL_CACHE_ACCESSES_sum": 5e9}
    r = bench.roofline_from({"counters_per_launch": ctr, "clock_ghz": 2.4}, None, "0" * 64, 100.0, 1, 1e9, 1e12)
    assert r["bound"] == "valu" and "active_lanes_per_valu" not in r
    assert r["memory_pipe"] == {"l1_accesses_per_segment": 5.0}


def test_bench_timed_image_parity_check(cornell_scene):
    """bench.check_timed_image: sampled pixels of a timed image against the oracle, for a full
    frame and for a row-split share (global row y = row0 + k * stride); one flipped bit in a
    sampled pixel is one mismatching word."""
    import numpy as np
    import bench
    import oracle_lib as O
    W, Hh, spp = 40, 24, 3
    img = O.render(cornell_scene, W, Hh, max_bounce=4, n_frames=spp)
    r = bench.check_timed_image(img, cornell_scene, W, Hh, spp, 4, 0, 1, 200, 7, 4)
    assert r["pixels"] == 200 and r["words"] == 800 and r["mismatches"] == 0 and r["frames"] == "1..3"
    share = img[1::3]                                   # rank 1 of 3
    assert bench.check_timed_image(share, cornell_scene, W, Hh, spp, 4, 1, 3, 100, 7, 4)["mismatches"] == 0
    bad = img.copy()
    bad.view(np.uint32)[...] ^= 1                       # every word off by one ulp
    r = bench.check_timed_image(bad, cornell_scene, W, Hh, spp, 4, 0, 1, 50, 7, 4)
    assert r["mismatches"] == 200
    assert bench.parity_pixels_for(1024, None) == 16384 and bench.parity_pixels_for(4096, None) == 4096
    assert bench.parity_pixels_for(256, 0) == 0
