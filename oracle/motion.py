"""TEST INFRASTRUCTURE ONLY: CPU restatement of the dynamic-scene movement in float32
numpy with the reference's operation order and fp16 rounding points, the checker for neus2_amd/csrc/motion.hip.

  rot6d_to_matrix       rotation_6d_to_matrix               common_operation.cuh:37-60
  delta_apply           add_global_movement_with_rotation_6d common_operation.cuh:416-492
  grad_rot6d            gradient_rotation_matrix_to_6d      common_operation.cuh:62-157 (d_b1/d_b2 are T = half)
  delta_grad            add_loss_to_rotation_6d_each + reduce_sum   common_operation.cuh:788-845,
                                                            transform_network.h:206-245
  accumulate_movement   accumulate_global_movement_rotation_6d_kernel   common_operation.cuh:551-585

Parameters follow the DeltaNetwork layout: transition[4] | rotation 6D[8] (transform_network.h:313-333); the
forward reads them as fp16. All arithmetic is scalar float32 without FMA contraction (each numpy float32 op
rounds), matching the kernels compiled with -ffp-contract=off.
"""
from __future__ import annotations

import numpy as np

f = np.float32


def rh(x):
    return f(np.float16(f(x)))


def _norm(v):
    return f(np.sqrt(f(f(f(v[0] * v[0]) + f(v[1] * v[1])) + f(v[2] * v[2]))))


def rot6d_to_matrix(r6):
    a1, a2 = [f(v) for v in r6[:3]], [f(v) for v in r6[3:6]]
    n1 = _norm(a1)
    b1 = [f(a / n1) for a in a1]
    d = f(f(f(b1[0] * a2[0]) + f(b1[1] * a2[1])) + f(b1[2] * a2[2]))
    u = [f(a2[k] - f(d * b1[k])) for k in range(3)]
    n2 = _norm(u)
    b2 = [f(x / n2) for x in u]
    b3 = [f(f(b1[1] * b2[2]) - f(b1[2] * b2[1])), f(f(b1[2] * b2[0]) - f(b1[0] * b2[2])), f(f(b1[0] * b2[1]) - f(b1[1] * b2[0]))]
    R = np.zeros(9, np.float32)
    for k in range(3):
        R[3 * k], R[3 * k + 1], R[3 * k + 2] = b1[k], b2[k], b3[k]
    return R


def matvec3(R, v):
    return [f(f(f(R[3 * k] * v[0]) + f(R[3 * k + 1] * v[1])) + f(R[3 * k + 2] * v[2])) for k in range(3)]


def inverse3(m):
    m = [f(x) for x in m]
    c00 = f(f(m[4] * m[8]) - f(m[5] * m[7]))
    c01 = f(f(m[5] * m[6]) - f(m[3] * m[8]))
    c02 = f(f(m[3] * m[7]) - f(m[4] * m[6]))
    det = f(f(f(m[0] * c00) + f(m[1] * c01)) + f(m[2] * c02))
    i = f(f(1.0) / det)
    return np.array([f(c00 * i), f(f(f(m[2] * m[7]) - f(m[1] * m[8])) * i), f(f(f(m[1] * m[5]) - f(m[2] * m[4])) * i),
                     f(c01 * i), f(f(f(m[0] * m[8]) - f(m[2] * m[6])) * i), f(f(f(m[2] * m[3]) - f(m[0] * m[5])) * i),
                     f(c02 * i), f(f(f(m[1] * m[6]) - f(m[0] * m[7])) * i), f(f(f(m[0] * m[4]) - f(m[1] * m[3])) * i)], np.float32)


def params_half(p):
    r6 = [rh(p[4 + k]) for k in range(6)]
    t = [rh(p[k]) for k in range(3)]
    return r6, t


def delta_apply(p, coords):
    """coords [n, 3] or [n, 7] float32 -> moved records (pos' = R (pos + t); dir' = (R (2 dir - 1) + 1) / 2)."""
    r6, t = params_half(p)
    R = rot6d_to_matrix(r6)
    c = np.asarray(coords, np.float32)
    out = c.copy()
    for i in range(c.shape[0]):
        q = matvec3(R, [f(c[i, k] + t[k]) for k in range(3)])
        out[i, :3] = q
        if c.shape[1] == 7:
            d = [f(f(c[i, 4 + k] * f(2.0)) - f(1.0)) for k in range(3)]
            e = matvec3(R, d)
            out[i, 4:7] = [f(f(e[k] + f(1.0)) * f(0.5)) for k in range(3)]
    return out


def _gnorm(v, g):
    nn = f(np.sqrt(f(f(f(v[0] * v[0]) + f(v[1] * v[1])) + f(v[2] * v[2]))))
    n3 = f(f(nn * nn) * nn)
    jxx, jyx, jzx = f(f(f(v[1] * v[1]) + f(v[2] * v[2])) / n3), f(f(-v[0] * v[1]) / n3), f(f(-v[0] * v[2]) / n3)
    o0 = f(f(f(g[0] * jxx) + f(g[1] * jyx)) + f(g[2] * jzx))
    jxy, jyy, jzy = f(f(-v[0] * v[1]) / n3), f(f(f(v[0] * v[0]) + f(v[2] * v[2])) / n3), f(f(-v[1] * v[2]) / n3)
    o1 = f(f(f(g[0] * jxy) + f(g[1] * jyy)) + f(g[2] * jzy))
    jxz, jyz, jzz = f(f(-v[0] * v[2]) / n3), f(f(-v[1] * v[2]) / n3), f(f(f(v[0] * v[0]) + f(v[1] * v[1])) / n3)
    o2 = f(f(f(g[0] * jxz) + f(g[1] * jyz)) + f(g[2] * jzz))
    return [o0, o1, o2]


def grad_rot6d(r6, G):
    a1, a2 = [f(v) for v in r6[:3]], [f(v) for v in r6[3:6]]
    n1 = _norm(a1)
    b1 = [f(a / n1) for a in a1]
    dd = f(f(f(b1[0] * a2[0]) + f(b1[1] * a2[1])) + f(b1[2] * a2[2]))
    u = [f(a2[k] - f(dd * b1[k])) for k in range(3)]
    n2 = _norm(u)
    b2 = [f(x / n2) for x in u]
    G = [f(x) for x in G]
    db1 = [rh(G[0]), rh(G[3]), rh(G[6])]
    db2 = [rh(G[1]), rh(G[4]), rh(G[7])]
    db1[0] = rh(f(db1[0] + f(f(b2[1] * G[8]) - f(b2[2] * G[5]))))
    db1[1] = rh(f(db1[1] + f(f(b2[2] * G[2]) - f(b2[0] * G[8]))))
    db1[2] = rh(f(db1[2] + f(f(b2[0] * G[5]) - f(b2[1] * G[2]))))
    db2[0] = rh(f(db2[0] + f(f(b1[2] * G[5]) - f(b1[1] * G[8]))))
    db2[1] = rh(f(db2[1] + f(f(b1[0] * G[8]) - f(b1[2] * G[2]))))
    db2[2] = rh(f(db2[2] + f(f(b1[1] * G[2]) - f(b1[0] * G[5]))))
    r = _gnorm(u, db2)
    da2 = list(r)
    da2[0] = f(da2[0] + f(f(f(-r[0] * b1[0]) * b1[0]) - f(f(r[1] * b1[0]) * b1[1])) - f(f(r[2] * b1[0]) * b1[2]))
    da2[1] = f(da2[1] + f(f(f(-r[0] * b1[0]) * b1[1]) - f(f(r[1] * b1[1]) * b1[1])) - f(f(r[2] * b1[2]) * b1[1]))
    da2[2] = f(da2[2] + f(f(f(-r[0] * b1[0]) * b1[2]) - f(f(r[1] * b1[1]) * b1[2])) - f(f(r[2] * b1[2]) * b1[2]))
    d1 = list(db1)
    s0 = f(f(f(f(2.0) * b1[0]) * a2[0]) + f(b1[1] * a2[1])) + f(b1[2] * a2[2])
    d1[0] = f(d1[0] + f(f(f(-r[0] * f(s0)) - f(f(r[1] * b1[1]) * a2[0])) - f(f(r[2] * b1[2]) * a2[0])))
    s1 = f(f(f(f(2.0) * b1[1]) * a2[1]) + f(b1[0] * a2[0])) + f(b1[2] * a2[2])
    d1[1] = f(d1[1] + f(f(f(-r[1] * f(s1)) - f(f(r[0] * b1[0]) * a2[1])) - f(f(r[2] * b1[2]) * a2[1])))
    s2 = f(f(f(f(2.0) * b1[2]) * a2[2]) + f(b1[0] * a2[0])) + f(b1[1] * a2[1])
    d1[2] = f(d1[2] + f(f(f(-r[2] * f(s2)) - f(f(r[0] * b1[0]) * a2[2])) - f(f(r[1] * b1[1]) * a2[2])))
    da1 = _gnorm(a1, d1)
    return [da1[0], da1[1], da1[2], da2[0], da2[1], da2[2]]


def delta_grad(p, coords, dpos):
    """Loss-scaled DeltaNetwork gradients (12 floats, fp16 values) from dL/d(moved position) dpos [n, >=3] and the
    undeformed positions coords [n, >=3]: per sample R^-1 g and d6D(g (x + t)^T), fp16-rounded, summed (float64
    here; the device sums fp32 in a fixed tree), rounded to fp16."""
    r6, t = params_half(p)
    R = rot6d_to_matrix(r6)
    Ri = inverse3(R)
    acc = np.zeros(9, np.float64)
    c = np.asarray(coords, np.float32)
    g_all = np.asarray(dpos, np.float32)
    for i in range(c.shape[0]):
        g = [f(v) for v in g_all[i, :3]]
        x = [f(c[i, k] + t[k]) for k in range(3)]
        gt = matvec3(Ri, g)
        G = [f(g[a] * x[b]) for a in range(3) for b in range(3)]
        g6 = grad_rot6d(r6, G)
        acc[:3] += [float(rh(v)) for v in gt]
        acc[3:] += [float(rh(v)) for v in g6]
    out = np.zeros(12, np.float32)
    out[:3] = [rh(v) for v in acc[:3]]
    out[4:10] = [rh(v) for v in acc[3:]]
    return out


def accumulate_movement(p, Rt):
    """R_acc <- R_local R_acc, t_acc <- R_local (t_acc + t_local), fp16-rounded; Rt is the 3x4 [R | t]."""
    r6 = [rh(p[4 + k]) for k in range(6)]
    R = rot6d_to_matrix(r6)
    A = np.asarray(Rt, np.float32)[:, :3].reshape(-1)
    t = np.asarray(Rt, np.float32)[:, 3]
    nR = np.zeros(9, np.float32)
    for i in range(3):
        for j in range(3):
            nR[3 * i + j] = f(f(f(R[3 * i] * A[j]) + f(R[3 * i + 1] * A[3 + j])) + f(R[3 * i + 2] * A[6 + j]))
    v = [f(t[k] + rh(p[k])) for k in range(3)]
    nt = matvec3(R, v)
    out = np.zeros((3, 4), np.float32)
    out[:, :3] = np.array([rh(x) for x in nR], np.float32).reshape(3, 3)
    out[:, 3] = [rh(x) for x in nt]
    return out
