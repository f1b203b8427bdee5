"""Seeded random scenes for the fuzz parity tests (tests/test_gpu_fuzz.py on the GPU,
tests/test_oracle_pinning.py's twin check on the CPU).

Each case is a triangle soup in the reference's std140 records (triangle.h, material.h,
sphere.h), run through the product's own setupBuffers path (pt_scene_from_arrays +
built-ins + the SAH builder restated from bvh.h:173-268), with the geometry the hot path's
special cases hinge on mixed in:
  * random triangles over four decades of size (deep, uneven trees);
  * axis-aligned quads (flat leaf boxes: the culling walk's exact leaf re-test, §5.6);
  * degenerate triangles (repeated vertices, collinear) and exact duplicates with another
    material (ties in the leaf's 2-way choice, computeShader.c:411-428);
  * large floor triangles, spheres inside and around the soup (:209-226, :372-385);
  * emissive / specular / smooth materials in any mix (:454-501);
  * optionally the whole scene and camera moved far from the origin (the exact-reciprocal
    guard and the culling margins).
The camera, image size, bounce count, frame numbers, toggles and display mode are drawn too.
"""
import numpy as np

import pt_host as H

# image / triangle sizes of the cases: LDS scenes (<= ~400 triangles), wide-workgroup LDS
# scenes and global-memory scenes (the walk from a top tree in LDS)
SIZES = [1, 2, 7, 24, 90, 300, 700, 2500, 9000]


def _tri(v0, v1, v2, m):
    t = np.zeros(16, np.float32)
    t[0:3], t[4:7], t[8:11], t[12] = v0, v1, v2, m
    return t


def random_case(seed, n_tris=None, far=None):
    """-> (scene buffers, render kwargs) for seed; n_tris / far override the drawn values."""
    rng = np.random.default_rng(seed)
    if n_tris is None:
        n_tris = int(SIZES[seed % len(SIZES)])
    if far is None:
        far = rng.random() < 0.2
    off = rng.uniform(-3000, 3000, 3) if far else np.zeros(3)

    n_m = int(rng.integers(1, 9))
    mats = np.zeros((n_m, 16), np.float32)
    mats[:, 0:3] = rng.random((n_m, 3))                                   # color
    emit = rng.random(n_m) < 0.35
    mats[:, 4:7] = rng.random((n_m, 3)) * emit[:, None]                     # emissionColor
    mats[:, 8:11] = rng.random((n_m, 3))                                  # specularColor
    mats[:, 12] = rng.uniform(0.5, 6.0, n_m) * emit                       # emissionStrength
    mats[:, 13] = rng.random(n_m) * (rng.random(n_m) < 0.6)               # smoothness
    mats[:, 14] = rng.random(n_m) * (rng.random(n_m) < 0.6)               # specularProbability

    tris = []
    kinds = rng.choice(5, size=n_tris, p=[0.55, 0.2, 0.08, 0.07, 0.1])
    for k in kinds:
        m = int(rng.integers(0, n_m))
        if k == 0 or not tris and k == 3:          # random triangle, size over four decades
            c = rng.uniform(-3, 3, 3)
            s = 10.0 ** rng.uniform(-3, 0.3)
            v = c + s * rng.standard_normal((3, 3))
            tris.append(_tri(v[0], v[1], v[2], m))
        elif k == 1:                               # axis-aligned quad: two triangles, flat box
            ax = int(rng.integers(0, 3))
            lo = rng.uniform(-3, 3, 3)
            hi = lo + 10.0 ** rng.uniform(-2, 0.5, 3)
            hi[ax] = lo[ax]
            a, b = [i for i in range(3) if i != ax]
            p00, p11 = lo.copy(), hi.copy()
            p10, p01 = lo.copy(), lo.copy()
            p10[a], p01[b] = hi[a], hi[b]
            tris.append(_tri(p00, p10, p11, m))
            tris.append(_tri(p00, p11, p01, m))
        elif k == 2:                               # degenerate: repeated vertex or collinear
            v0 = rng.uniform(-3, 3, 3)
            v1 = v0 + rng.standard_normal(3)
            v2 = v0 if rng.random() < 0.5 else v0 + 2.0 * (v1 - v0)
            tris.append(_tri(v0, v1, v2, m))
        elif k == 3:                               # exact duplicate with its own material
            t = tris[int(rng.integers(0, len(tris)))].copy()
            t[12] = m
            tris.append(t)
        else:                                      # large floor / wall triangle
            z = rng.uniform(-4, -1)
            tris.append(_tri((-40, -40, z), (40, -40, z), (0, 40, z), m))
    tris = np.stack(tris)[: max(n_tris, 1)]
    tris[:, 0:3] += off
    tris[:, 4:7] += off
    tris[:, 8:11] += off

    sc = H.scene_from_arrays(tris, mats)
    # extra spheres (reference layout: center, radius | material) beside the built-ins
    n_s = int(rng.integers(0, 4))
    if n_s:
        sph = np.zeros((n_s, 8), np.float32)
        sph[:, 0:3] = rng.uniform(-3, 3, (n_s, 3)) + off
        sph[:, 3] = 10.0 ** rng.uniform(-1.5, 0.3, n_s)
        sph[:, 4] = rng.integers(0, len(sc["mats"]), n_s)
        sc["spheres"] = np.concatenate([sc["spheres"], sph]).astype(np.float32)

    pos = rng.uniform(-7, 7, 3)
    if rng.random() < 0.5:
        pos[1] = rng.uniform(-9, -5)               # outside the soup, looking in
    look = rng.uniform(-1, 1, 3) - pos
    look[:2] += rng.uniform(0.05, 0.3, 2)          # never parallel to +z (the camera basis)
    cam = np.zeros(12, np.float32)
    cam[0:3] = pos + off
    cam[4:7] = look
    sc["cam"] = cam

    flags = 0
    for f in (H.PT_FLAG_NO_AA, H.PT_FLAG_NO_SKY, H.PT_FLAG_NO_SPHERES):
        if rng.random() < 0.2:
            flags |= f
    kw = dict(W=int(rng.integers(5, 41)), H=int(rng.integers(3, 33)), max_bounce=int(rng.integers(0, 9)),
              mode=int(rng.choice([1, 1, 1, 2, 3, 4])), frame_first=int(rng.integers(1, 4000)),
              n_frames=int(rng.integers(1, 4)), flags=flags)
    return sc, kw
