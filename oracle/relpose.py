"""ORACLE (test infrastructure only): relative pose of two robots, ``dgl/utils.py:54-77``.

Restated from the math rather than the code: q_rel = conj(q1) (x) q2 (Hamilton product,
quaternions stored (x, y, z, w)), R = rotation matrix of q_rel, and the edge feature is
``[t2 - t1, R[:, 0], R[:, 1]]`` (the first six entries of R flattened column-major, the order
``quat_to_so3`` returns them in).  Computed in float64; checked against the reference's own
self-check pose pair and float32 dataset-path fixtures to a tolerance.
"""
import numpy as np


def hamilton(a, b):
    """Quaternion product a (x) b for (x, y, z, w) quaternions."""
    av, aw = np.asarray(a[:3], np.float64), float(a[3])
    bv, bw = np.asarray(b[:3], np.float64), float(b[3])
    v = aw * bv + bw * av + np.cross(av, bv)
    return np.array([v[0], v[1], v[2], aw * bw - av @ bv])


def quat_to_so3(q):
    """Rotation matrix of an (x, y, z, w) quaternion (unit or not: the reference uses the
    un-normalised form 1 - 2(y^2 + z^2) ...), returned flattened column-major (9,)."""
    x, y, z, w = (float(t) for t in q)
    R = np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])
    return R.T.reshape(-1)  # column-major


def cal_relative_pose(p1, p2):
    p1 = np.asarray(p1, np.float64)
    p2 = np.asarray(p2, np.float64)
    conj_q1 = np.array([-p1[3], -p1[4], -p1[5], p1[6]])
    q_rel = hamilton(conj_q1, p2[3:7])
    return np.concatenate([p2[:3] - p1[:3], quat_to_so3(q_rel)[:6]])
