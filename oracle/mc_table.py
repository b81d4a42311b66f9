"""TEST INFRASTRUCTURE ONLY: the marching-cubes case table for the parity tests and the numpy mesh restatement.

The table is the reference's constant `triangle_table` (src/marching_cubes.cu:401-658, the classic Lorensen /
Bourke table via PyMCubes, BSD-3), stored as data in oracle/mc_triangle_table.npy (tools/extract_mc_table.py).
Corner / edge numbering is the reference's (marching_cubes.cu:255-275, 377-420): corner bit k of the mask is set
iff density > thresh.
"""
from __future__ import annotations

import os

import numpy as np

# corner k -> (x, y, z) offset
CORNERS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
# edge e -> (corner a, corner b)
EDGES = [(0, 1), (1, 2), (3, 2), (0, 3), (4, 5), (5, 6), (7, 6), (4, 7), (0, 4), (1, 5), (2, 6), (3, 7)]
# edge e -> (grid point offset, axis) of the vertex it owns (gen_faces local_edges order)
EDGE_OWNER = [((0, 0, 0), 0), ((1, 0, 0), 1), ((0, 1, 0), 0), ((0, 0, 0), 1),
              ((0, 0, 1), 0), ((1, 0, 1), 1), ((0, 1, 1), 0), ((0, 0, 1), 1),
              ((0, 0, 0), 2), ((1, 0, 0), 2), ((1, 1, 0), 2), ((0, 1, 0), 2)]
MAX_TRIS = 6
_TABLE = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mc_triangle_table.npy"))


def case_triangles(mask):
    row = [int(v) for v in _TABLE[mask] if v >= 0]
    return [tuple(row[i:i + 3]) for i in range(0, len(row), 3)]


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
