"""ASan + UBSan run of the host-side ingest.

tests/sanitize/host_fuzz.cpp links csrc/pt_scene.cpp and csrc/pt_viewer.cpp with
-fsanitize=address,undefined -fno-sanitize-recover=all and drives:
  * both loaders (reference semantics, geometry_loader.h:15-142, and the robust reader) on the
    generated Cornell scene, the reference's shipped scenes when mounted, and a few thousand
    mutated OBJ/MTL texts (byte flips, truncation, long lines, huge / negative indices, NaN);
  * the SAH builder (bvh.h:173-268) on every accepted scene, twice (scene object and raw
    arrays, which must agree), and an undersized node buffer, which must be refused;
  * pt_bvh_culling_ok on random node arrays (NaN / huge link floats);
  * the headless viewer (ogl_path_trace.h:258-364) on random key / cursor / clock events.
Any sanitizer report aborts the process.  No GPU needed.
"""
import os
import subprocess

import pytest

from conftest import REF_SCENES

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tests", "sanitize")


@pytest.fixture(scope="module")
def host_fuzz(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("sanbuild"))
    r = subprocess.run(["make", "-s", "-C", SAN, "OUT=" + out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(out, "host_fuzz")


def test_host_ingest_under_asan_ubsan(host_fuzz, cornell_paths, tmp_path):
    import pt_scenes
    args = list(cornell_paths)
    args += list(pt_scenes.write_scene("bunny", str(tmp_path), target_tris=2000))
    for name in ("ship", "p", "drift"):
        obj, mtl = os.path.join(REF_SCENES, name + "obj.txt"), os.path.join(REF_SCENES, name + "mtl.txt")
        if os.path.exists(obj) and os.path.exists(mtl):
            args += [obj, mtl]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([host_fuzz, str(tmp_path), "3000"] + args, capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-4000:])
    assert "host_fuzz ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
