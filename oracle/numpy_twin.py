"""TEST INFRASTRUCTURE ONLY -- an independent numpy-float32 restatement of the hot path.

A second, separately written reading of computeShader.c (Trace :434-501,
calculateRayCollision :367-432, bvh_intersect :309-365, hit_triangle :274-307,
hit_sphere :209-226, RNG :87-129, main :505-554), vectorised over pixels.  It shares no
code with oracle/pt_oracle.cpp; tests require the two to agree bit for bit, which pins the
C++ oracle against transcription slips.  Small images only (pure numpy, masked loops).

Arithmetic: numpy binary32 array ops are IEEE round-to-nearest (no FMA), np.sqrt and '/'
are correctly rounded -- the same pinning as DESIGN.md §3.2.  log/cos are the build's pinned
polynomials, re-implemented here with uint32/float32 array arithmetic and an exactly rounded
binary32 fma emulation (numpy has no fma).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
u32 = np.uint32
i32 = np.int32


def _bits(x):
    return np.asarray(x, f32).view(i32)


def _float(b):
    return np.asarray(b, i32).view(f32)


# ------------------------------------------------------------------ transcendentals
def fma(a, b, c):
    """Correctly rounded binary32 fused multiply-add, vectorised: a*b is exact in binary64,
    TwoSum gives the exact a*b + c as s + e, and the binary64 -> binary32 rounding of s is
    corrected when s sits exactly on a binary32 rounding midpoint (the only case where the
    double rounding can differ: midpoints are binary64 numbers, so RN64 never crosses one)."""
    a, b, c = (np.asarray(v, f32).astype(np.float64) for v in (a, b, c))
    p = a * b
    s = p + c
    bb = s - p
    e = (p - (s - bb)) + (c - bb)
    r = s.astype(f32)
    rr = r.astype(np.float64)
    d = s - rr
    nb = np.nextafter(r, np.where(d > 0, f32(np.inf), f32(-np.inf)).astype(f32))
    mid = (d != 0) & (np.abs(nb.astype(np.float64) - rr) == 2 * np.abs(d))
    fix = mid & (e != 0) & (np.sign(e) == np.sign(d))
    return np.where(fix, nb, r).astype(f32)


_LOGP = [float.fromhex(h) for h in ("0x1.87c9c0p-4", "-0x1.2bf636p-3", "0x1.2f3194p-3", "-0x1.52694ep-3",
                                     "0x1.98eb62p-3", "-0x1.000924p-2", "0x1.5556ccp-2", "-0x1.fffff0p-2")]


def logf(x):
    """The build's pinned log (pt_math.h logf_pinned), for x in {0} U [2^-32, 1]:
    x = 2^k z split at the exponent boundary 0x3f330000, f = z - 1, f + f^2 P(f) by Horner in
    fma, then + k ln2_lo and + k ln2_hi."""
    x = np.asarray(x, f32)
    ix = x.view(u32)
    split = (ix - u32(0x3F330000)).astype(u32)
    k = split.view(i32) >> 23
    z = (ix - (split & u32(0xFF800000))).astype(u32).view(f32)
    f = z - f32(1.0)
    P = np.full(x.shape, f32(_LOGP[0]), f32)
    for c in _LOGP[1:]:
        P = fma(f, P, f32(c))
    kf = k.astype(f32)
    y = fma(f * f, P, f)
    y = fma(kf, f32(float.fromhex("0x1.2fefa2p-17")), y)
    y = fma(kf, f32(float.fromhex("0x1.62e300p-1")), y)
    return np.where(x == 0, f32(-np.inf), y).astype(f32)


def cosf(t):
    """The build's pinned cos (pt_math.h cosf_pinned) for t in [0, 2 pi]: quadrant q =
    rint(t 2/pi), r = t - q pi/2 (two-part pi/2 by fma), cos r or sin r polynomial."""
    t = np.asarray(t, f32)
    q = np.rint(t * f32(float.fromhex("0x1.45f306p-1"))).astype(f32)
    r = fma(-q, f32(float.fromhex("0x1.921fb6p+0")), t)
    r = fma(-q, f32(float.fromhex("-0x1.777a5cp-25")), r)
    r2 = r * r
    cp = fma(r2, f32(float.fromhex("-0x1.64756cp-10")), f32(float.fromhex("0x1.553f94p-5")))
    cp = fma(r2, cp, f32(float.fromhex("-0x1.ffffbap-2")))
    c = fma(r2, cp, f32(1.0))
    sp = fma(r2, f32(float.fromhex("-0x1.98da64p-13")), f32(float.fromhex("0x1.1105b4p-7")))
    sp = fma(r2, sp, f32(float.fromhex("-0x1.555540p-3")))
    sn = fma(r * r2, sp, r)
    quad = q.astype(i32) & 3
    v = np.where((quad & 1) == 1, sn, c)
    return np.where((quad == 1) | (quad == 2), -v, v).astype(f32)


# ------------------------------------------------------------------ RNG
def next_random(state):
    state = (state * u32(747796405) + u32(2891336453)).astype(u32)
    r = (((state >> ((state >> u32(28)) + u32(4))) ^ state) * u32(277803737)).astype(u32)
    return state, ((r >> u32(22)) ^ r).astype(u32)


def random01(state):
    state, r = next_random(state)
    return state, r.astype(f32) * f32(2.0 ** -32)


# ------------------------------------------------------------------ vector helpers (tuples of arrays)
def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1])


def add(a, b):
    return tuple(x + y for x, y in zip(a, b))


def sub(a, b):
    return tuple(x - y for x, y in zip(a, b))


def scale(a, s):
    return tuple(x * s for x in a)


def normalize(a):
    r = f32(1.0) / np.sqrt(dot(a, a))
    return scale(a, r)


def pick(mask, a, b):
    return tuple(np.where(mask, x, y) for x, y in zip(a, b))


# ------------------------------------------------------------------ hot path
def render(sc, W, H, max_bounce=5, mode=1, frame_first=1, n_frames=1, acc_first=0, accum=None):
    tris = np.asarray(sc["tris"], f32).reshape(-1, 16)
    nodes = np.asarray(sc["nodes"], f32).reshape(-1, 12)
    mats = np.asarray(sc["mats"], f32).reshape(-1, 16)
    sph = np.asarray(sc["spheres"], f32).reshape(-1, 8)
    cam = np.asarray(sc["cam"], f32).reshape(12)
    ys, xs = np.meshgrid(np.arange(H, dtype=np.int64), np.arange(W, dtype=np.int64), indexing="ij")
    xs, ys = xs.reshape(-1), ys.reshape(-1)
    P = xs.size
    fwd = normalize(tuple(np.full(1, cam[4 + i], f32) for i in range(3)))
    right = normalize(cross(fwd, (f32(0), f32(0), f32(1))))
    up = scale(normalize(cross(right, fwd)), f32(H))
    up = tuple(c / f32(W) for c in up)
    pos = tuple(np.full(P, cam[i], f32) for i in range(3))
    acc = np.zeros((P, 4), f32) if accum is None else np.asarray(accum, f32).reshape(P, 4).copy()
    for k in range(n_frames):
        frame = frame_first + k
        st = ((ys.astype(np.uint64) * 831266 + xs.astype(np.uint64) * 923766 + np.uint64(frame) * 719393)
              & 0xFFFFFFFF).astype(u32)
        st, ax = random01(st)
        st, ay = random01(st)
        u = (xs.astype(f32) + ax) / f32(W) - f32(0.5)
        v = (ys.astype(f32) + ay) / f32(H) - f32(0.5)
        d = normalize(add(add(tuple(np.broadcast_to(c, (P,)) for c in fwd), scale(right, u)), scale(up, v)))
        rgb = _trace(tris, nodes, mats, sph, pos, d, st, max_bounce, mode)
        rgb = tuple(f32(0.0) + c for c in rgb)
        rgb = tuple(c / f32(1.0) for c in rgb)
        if k == 0 and acc_first != 1:
            acc = np.stack([rgb[0], rgb[1], rgb[2], np.ones(P, f32)], 1)
        else:
            ff = f32(frame)
            w = (ff - f32(1.0)) / ff
            acc = np.stack([acc[:, 0] * w + rgb[0] / ff, acc[:, 1] * w + rgb[1] / ff,
                            acc[:, 2] * w + rgb[2] / ff, acc[:, 3] * w + f32(1.0) / ff], 1)
    return acc.reshape(H, W, 4)


def _tri(tris, idx, o, d):
    t = tris[idx]
    v0, v1, v2 = (t[:, 0], t[:, 1], t[:, 2]), (t[:, 4], t[:, 5], t[:, 6]), (t[:, 8], t[:, 9], t[:, 10])
    n = normalize(cross(sub(v1, v0), sub(v2, v0)))
    dd = -dot(n, v0)
    tt = -(dot(n, o) + dd) / dot(n, d)
    p = add(o, scale(d, tt))
    inside = (dot(n, cross(sub(v1, v0), sub(p, v0))) > 0) & (dot(n, cross(sub(v2, v1), sub(p, v1))) > 0) & \
             (dot(n, cross(sub(v0, v2), sub(p, v2))) > 0)
    res = np.where((tt < 0) | ~inside, f32(-1.0), tt)
    return res, n


def _collide(tris, nodes, sph, o, d):
    P = o[0].size
    t = np.full(P, np.inf, f32)
    hit = np.zeros(P, bool)
    normal = (np.zeros(P, f32),) * 3
    hp = (np.zeros(P, f32),) * 3
    mat = np.zeros(P, np.int64)
    for s in sph:
        c = (s[0], s[1], s[2])
        oc = sub(o, c)
        a = dot(d, d)
        hb = dot(oc, d)
        cc = dot(oc, oc) - s[3] * s[3]
        disc = hb * hb - a * cc
        with np.errstate(invalid="ignore"):
            ht = np.where(disc < 0, f32(-1.0), (-hb - np.sqrt(disc)) / a)
        ok = (ht > f32(0.0001)) & (ht < t)
        pn = normalize(sub(add(o, scale(d, ht)), c))
        flip = dot(pn, d) > 0
        pn = pick(flip, scale(pn, f32(-1.0)), pn)
        hit |= ok
        t = np.where(ok, ht, t)
        normal = pick(ok, pn, normal)
        hp = pick(ok, add(o, scale(d, ht)), hp)
        mat = np.where(ok, int(s[4]), mat)
    if len(nodes) == 0:
        return hit, normal, hp, mat
    bi = np.zeros(P, np.int64)
    while True:
        act = np.nonzero(bi > -1)[0]
        if act.size == 0:
            break
        nd = nodes[bi[act]]
        oo = tuple(c[act] for c in o)
        dd = tuple(c[act] for c in d)
        tc = t[act]
        tmin = (nd[:, 0] - oo[0]) / dd[0]
        tmax = (nd[:, 4] - oo[0]) / dd[0]
        sw = tmin > tmax
        tmin, tmax = np.where(sw, tmax, tmin), np.where(sw, tmin, tmax)
        tymin = (nd[:, 1] - oo[1]) / dd[1]
        tymax = (nd[:, 5] - oo[1]) / dd[1]
        sw = tymin > tymax
        tymin, tymax = np.where(sw, tymax, tymin), np.where(sw, tymin, tymax)
        ok = ~((tmin > tymax) | (tymin > tmax))
        tmin = np.where(tymin > tmin, tymin, tmin)
        tmax = np.where(tymax < tmax, tymax, tmax)
        tzmin = (nd[:, 2] - oo[2]) / dd[2]
        tzmax = (nd[:, 6] - oo[2]) / dd[2]
        sw = tzmin > tzmax
        tzmin, tzmax = np.where(sw, tzmax, tzmin), np.where(sw, tzmin, tzmax)
        ok &= ~((tmin > tzmax) | (tzmin > tmax))
        tmin = np.where(tzmin > tmin, tzmin, tmin)
        ok &= ~(tmin > tc)
        nxt = np.where(ok, nd[:, 10], nd[:, 11]).astype(np.int64)
        leaf = ok & (nd[:, 8] > -1)
        li = np.nonzero(leaf)[0]
        if li.size:
            g = act[li]
            o2 = tuple(c[g] for c in o)
            d2 = tuple(c[g] for c in d)
            i0 = nd[li, 8].astype(np.int64)
            i1 = nd[li, 9].astype(np.int64)
            h1, n1 = _tri(tris, i0, o2, d2)
            h2, n2 = _tri(tris, i1, o2, d2)
            tg = t[g]
            c1 = (h1 > f32(0.0001)) & (h1 < tg) & ((h1 < h2) | (h2 < f32(0.0001)))
            c2 = ~c1 & (h2 > f32(0.0001)) & (h2 < tg)
            n1 = pick(dot(n1, d2) > 0, scale(n1, f32(-1.0)), n1)
            n2 = pick(dot(n2, d2) > 0, scale(n2, f32(-1.0)), n2)
            th = np.where(c1, h1, h2)
            nn = pick(c1, n1, n2)
            sel = c1 | c2
            gs = g[sel]
            hit[gs] = True
            t[gs] = th[sel]
            for q in range(3):
                normal[q][gs] = nn[q][sel]
            hpn = add(o2, scale(d2, th))
            for q in range(3):
                hp[q][gs] = hpn[q][sel]
            mat[gs] = np.where(c1, tris[i0, 12], tris[i1, 12]).astype(np.int64)[sel]
        bi[act] = nxt
    return hit, normal, hp, mat


def _trace(tris, nodes, mats, sph, o, d, st, max_bounce, mode):
    P = o[0].size
    inc = (np.zeros(P, f32),) * 3
    col = (np.ones(P, f32),) * 3
    out = [None, None, None]
    alive = np.ones(P, bool)
    result = [np.zeros(P, f32) for _ in range(3)]
    o = tuple(c.copy() for c in o)
    d = tuple(np.asarray(c, f32).copy() for c in d)
    for _ in range(max_bounce + 1):
        idx = np.nonzero(alive)[0]
        if idx.size == 0:
            break
        oo = tuple(c[idx] for c in o)
        dd = tuple(c[idx] for c in d)
        normal0 = (np.zeros(idx.size, f32),) * 3
        hit, normal, hp, mat = _collide(tris, nodes, sph, oo, dd)
        cc = tuple(c[idx] for c in col)
        shade = hit & (np.sqrt(dot(cc, cc)) > f32(0.01))
        # misses / dark: add sky and finish
        miss = ~shade
        if miss.any():
            dn = normalize(dd)
            tt = f32(0.5) * (dn[2] + f32(1.0))
            omt = f32(1.0) - tt
            env = (omt * f32(1.0) + tt * f32(0.5), omt * f32(1.0) + tt * f32(0.7), omt * f32(1.0) + tt * f32(1.0))
            for q in range(3):
                val = inc[q][idx] + env[q] * cc[q]
                result[q][idx[miss]] = val[miss]
            alive[idx[miss]] = False
        sidx = idx[shade]
        if sidx.size == 0:
            continue
        n = tuple(c[shade] for c in normal)
        h = tuple(c[shade] for c in hp)
        o_s = tuple(c[shade] for c in oo)
        d_s = tuple(c[shade] for c in dd)
        m = mats[mat[shade]]
        if mode == 2:
            for q in range(3):
                result[q][sidx] = (n[q] + f32(1.0)) * f32(0.5)
            alive[sidx] = False
            continue
        if mode == 4:
            s = np.sqrt(dot(sub(h, o_s), sub(h, o_s)))
            dist = f32(1.0) - np.sqrt(s + f32(1.0)) / (s + f32(1.0))
            for q in range(3):
                result[q][sidx] = dist * dist
            alive[sidx] = False
            continue
        s_ = st[sidx]
        g = []
        for _q in range(3):
            s_, r1 = random01(s_)
            theta = (f32(2.0) * f32(3.1415926)) * r1
            s_, r2 = random01(s_)
            with np.errstate(divide="ignore", invalid="ignore"):
                rho = np.sqrt(f32(-2.0) * logf(r2))
            g.append(rho * cosf(theta))
        with np.errstate(divide="ignore", invalid="ignore"):
            diffuse = normalize(add(n, normalize(tuple(g))))
        kk = f32(2.0) * dot(n, d_s)
        spec = normalize(sub(d_s, scale(n, kk)))
        if mode == 3:
            for q in range(3):
                result[q][sidx] = m[:, q]
            st[sidx] = s_
            alive[sidx] = False
            continue
        s_, coin = random01(s_)
        st[sidx] = s_
        is_spec = np.where(m[:, 14] > coin, f32(1.0), f32(0.0))
        a = m[:, 13] * is_spec
        oma = f32(1.0) - a
        nd_ = tuple(diffuse[q] * oma + spec[q] * a for q in range(3))
        for q in range(3):
            o[q][sidx] = h[q]
            d[q][sidx] = nd_[q]
        emis = tuple(m[:, 4 + q] * m[:, 12] for q in range(3))
        ie = f32(1.0) - is_spec
        for q in range(3):
            inc_q = inc[q].copy()
            inc_q[sidx] = inc[q][sidx] + emis[q] * cc[q][shade]
            col_q = col[q].copy()
            col_q[sidx] = cc[q][shade] * (m[:, q] * ie + m[:, 8 + q] * is_spec)
            inc = inc[:q] + (inc_q,) + inc[q + 1:]
            col = col[:q] + (col_q,) + col[q + 1:]
    # paths that exhausted the bounce budget return the accumulated light
    for q in range(3):
        result[q][alive] = inc[q][alive]
    return tuple(result)
