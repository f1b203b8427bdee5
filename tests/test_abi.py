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
