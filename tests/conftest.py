import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "opengl-path-tracing_amd")
for p in (os.path.join(REPO, "tests"), PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

REF_SCENES = "/root/reference/LearnOpenGL/scene_data"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


@pytest.fixture(scope="session")
def cornell_paths():
    import pt_scenes
    return pt_scenes.write_scene("cornell", os.path.join(REPO, "scenes"))


@pytest.fixture(scope="session")
def cornell_scene(cornell_paths):
    """setupBuffers() output for the Cornell box, via the product host library."""
    import pt_host
    return pt_host.setupBuffers(*cornell_paths)


@pytest.fixture(scope="session")
def ship_scene():
    """The reference's ship scene (scene_data/ship*.txt) as loaded by the product loader
    (tests/golden/ship_scene.npz; loader parity vs the oracle is tested on CPU)."""
    import numpy as np
    import pt_host
    z = np.load(os.path.join(REPO, "tests", "golden", "ship_scene.npz"))
    return pt_host.scene_from_arrays(z["tris"], z["mats"])
