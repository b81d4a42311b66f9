"""TEST INFRASTRUCTURE ONLY: an independent restatement of the marching-cubes case table that the
product (neus2_amd/csrc/mc.hip, `mc_build_table`) generates, used by the parity tests to check the GPU
mesh face-for-face.

Neither side copies a published triangle table. For each of the 256 corner masks the crossing edges are
joined face by face into segments — on a face with four crossings, each set corner is cut off by its own
segment (the rule is symmetric, so the two cubes sharing a face agree and the mesh is watertight) — the
segments are oriented with the set corners on their left seen from outside the cube, chained into loops,
and each loop is fanned into triangles from its lowest-numbered edge. Corner / edge numbering is the
reference's (marching_cubes.cu:255-275, 377-420): corner bit k of the mask is set iff density > thresh.
"""
from __future__ import annotations

import numpy as np

# corner k -> (x, y, z) offset
CORNERS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
# edge e -> (corner a, corner b)
EDGES = [(0, 1), (1, 2), (3, 2), (0, 3), (4, 5), (5, 6), (7, 6), (4, 7), (0, 4), (1, 5), (2, 6), (3, 7)]
# edge e -> (grid point offset, axis) of the vertex it owns (gen_faces local_edges order)
EDGE_OWNER = [((0, 0, 0), 0), ((1, 0, 0), 1), ((0, 1, 0), 0), ((0, 0, 0), 1),
              ((0, 0, 1), 0), ((1, 0, 1), 1), ((0, 1, 1), 0), ((0, 0, 1), 1),
              ((0, 0, 0), 2), ((1, 0, 0), 2), ((1, 1, 0), 2), ((0, 1, 0), 2)]
# faces: corners in cyclic order and outward normal
FACES = [((0, 3, 7, 4), (-1, 0, 0)), ((1, 2, 6, 5), (1, 0, 0)), ((0, 1, 5, 4), (0, -1, 0)),
         ((3, 2, 6, 7), (0, 1, 0)), ((0, 1, 2, 3), (0, 0, -1)), ((4, 5, 6, 7), (0, 0, 1))]
MAX_TRIS = 6


def _edge_of(a, b):
    for e, (p, q) in enumerate(EDGES):
        if {p, q} == {a, b}:
            return e
    raise KeyError((a, b))


def _mid(e):
    a, b = EDGES[e]
    return (np.array(CORNERS[a], float) + np.array(CORNERS[b], float)) * 0.5


def case_triangles(mask):
    if mask == 0 or mask == 255:
        return []
    inside = [(mask >> k) & 1 for k in range(8)]
    nxt = {}
    for corners, normal in FACES:
        n = np.array(normal, float)
        cyc = list(corners)
        segs = []
        set_corners = [c for c in cyc if inside[c]]
        if len(set_corners) in (0, 4):
            continue
        if len(set_corners) == 2 and not any(inside[cyc[i]] and inside[cyc[(i + 1) % 4]] for i in range(4)):
            # ambiguous face (diagonal set corners): cut off each set corner separately
            for c in set_corners:
                i = cyc.index(c)
                segs.append((_edge_of(c, cyc[(i - 1) % 4]), _edge_of(c, cyc[(i + 1) % 4]), c))
        else:
            xs = [_edge_of(cyc[i], cyc[(i + 1) % 4]) for i in range(4) if inside[cyc[i]] != inside[cyc[(i + 1) % 4]]]
            assert len(xs) == 2
            segs.append((xs[0], xs[1], set_corners[0]))
        for a, b, c in segs:
            A, B, P = _mid(a), _mid(b), np.array(CORNERS[c], float)
            # orient A->B with the set corner on the left seen from outside: cross(n, B - A) . (P - A) > 0
            if np.dot(np.cross(n, B - A), P - A) < 0:
                a, b = b, a
            assert a not in nxt
            nxt[a] = b
    tris = []
    seen = set()
    for start in sorted(nxt):
        if start in seen:
            continue
        loop = [start]
        seen.add(start)
        v = nxt[start]
        while v != start:
            loop.append(v)
            seen.add(v)
            v = nxt[v]
        # fan from the smallest edge id of the loop
        k = loop.index(min(loop))
        loop = loop[k:] + loop[:k]
        for i in range(1, len(loop) - 1):
            tris.append((loop[0], loop[i], loop[i + 1]))
    return tris


def build_table():
    """int8 [256][3 * MAX_TRIS + 1]: edge triples, -1 terminated."""
    t = np.full((256, 3 * MAX_TRIS + 1), -1, np.int8)
    for m in range(256):
        tr = case_triangles(m)
        assert len(tr) <= MAX_TRIS, (m, len(tr))
        for i, tri in enumerate(tr):
            t[m, 3 * i:3 * i + 3] = tri
    return t


def marching_cubes(density, thresh, aabb_min=(0, 0, 0), aabb_max=(1, 1, 1)):
    """Reference gen_vertices / gen_faces (marching_cubes.cu:276-420) over density [rz][ry][rx] in the
    canonical deterministic order: vertices by (grid point linear index, axis x < y < z), triangles by
    (cube linear index, table order). Returns V float32 [n, 3], F uint32 [m, 3]."""
    d = np.asarray(density, np.float32)
    rz, ry, rx = d.shape
    thresh = np.float32(thresh)
    amin, amax = np.asarray(aabb_min, np.float32), np.asarray(aabb_max, np.float32)
    res = np.array([rx, ry, rz], np.float32)
    scale = (amax - amin) / res
    ins = d > thresh
    # crossing flags per grid point and axis
    cx = np.zeros_like(ins); cy = np.zeros_like(ins); cz = np.zeros_like(ins)
    cx[:, :, :-1] = ins[:, :, :-1] != ins[:, :, 1:]
    cy[:, :-1, :] = ins[:, :-1, :] != ins[:, 1:, :]
    cz[:-1, :, :] = ins[:-1, :, :] != ins[1:, :, :]
    flags = np.stack([cx, cy, cz], -1).reshape(-1, 3)  # point-major, axis-minor
    nv = flags.sum(1)
    vbase = np.concatenate([[0], np.cumsum(nv)[:-1]]).astype(np.int64)
    pts, axes = np.nonzero(flags)
    z, rem = np.divmod(pts, rx * ry)
    y, x = np.divmod(rem, rx)
    f0 = d.reshape(-1)[pts]
    step = np.array([1, rx, rx * ry])[axes]
    f1 = d.reshape(-1)[pts + step]
    dt = ((thresh - f0) / (f1 - f0)).astype(np.float32)
    g = np.stack([x, y, z], 1).astype(np.float32)
    g[np.arange(len(axes)), axes] = g[np.arange(len(axes)), axes] + dt
    V = (g * scale + amin).astype(np.float32)
    # faces
    table = build_table()
    c = np.zeros((rz - 1, ry - 1, rx - 1), np.int32)
    for k, (ox, oy, oz) in enumerate(CORNERS):
        c |= ins[oz:oz + rz - 1, oy:oy + ry - 1, ox:ox + rx - 1].astype(np.int32) << k
    F = []
    cz_, cy_, cx_ = np.nonzero((c != 0) & (c != 255))
    for zz, yy, xx in zip(cz_, cy_, cx_):
        m = c[zz, yy, xx]
        row = table[m]
        for i in range(MAX_TRIS):
            if row[3 * i] < 0:
                break
            tri = []
            for e in row[3 * i:3 * i + 3]:
                (ox, oy, oz), ax = EDGE_OWNER[e]
                p = (xx + ox) + (yy + oy) * rx + (zz + oz) * rx * ry
                tri.append(vbase[p] + int(flags[p, :ax].sum()))
            F.append(tri)
    return V, np.asarray(F, np.uint32).reshape(-1, 3)
