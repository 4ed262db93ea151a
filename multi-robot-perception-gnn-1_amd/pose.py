"""Relative pose between robots: the 9-d edge feature of the per-frame graph.

Restates ``dgl/utils.py:54-77`` (``quat_to_so3``, ``cal_relative_pose``) with a batched
form used by the graph builders.  The edge u->v carries
``[t_v - t_u (3), first two columns of R(q_v * q_u^-1) flattened column-major (6)]``;
quaternions are ``(x, y, z, w)`` as in the pose files (``flight_record.py:75``).
Arithmetic keeps the input precision and the reference's operation order: the dataset
path feeds float32 arrays (``torch.tensor(list_of_floats).numpy()``,
``dgl/dataloader_utils.py:114-116`` -> ``dgl/dataloader.py:119-120``) and so computes in
float32, while the self-check at ``dgl/utils.py:80-85`` runs float64.
"""
from __future__ import annotations

import numpy as np


def _as_float(a) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype not in (np.float32, np.float64):
        a = a.astype(np.float64)
    return a


def quat_to_so3(q) -> np.ndarray:
    """Rotation matrix of quaternion ``q = (x, y, z, w)`` as 9 entries, column-major
    (``a00, a10, a20, a01, ...``), exactly the ordering of ``dgl/utils.py:54-66``."""
    return quat_to_so3_batch(_as_float(q)[None])[0]


def quat_to_so3_batch(q: np.ndarray) -> np.ndarray:
    """Batched ``quat_to_so3``: (M, 4) -> (M, 9), same dtype as ``q``."""
    q = _as_float(q)
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    cols = [
        1 - 2 * y ** 2 - 2 * z ** 2,  # a00
        2 * x * y + 2 * z * w,  # a10
        2 * x * z - 2 * y * w,  # a20
        2 * x * y - 2 * z * w,  # a01
        1 - 2 * x ** 2 - 2 * z ** 2,  # a11
        2 * y * z + 2 * x * w,  # a21
        2 * x * z + 2 * y * w,  # a02
        2 * y * z - 2 * x * w,  # a12
        1 - 2 * x ** 2 - 2 * y ** 2,  # a22
    ]
    return np.stack(cols, axis=1)


def relative_pose_batch(p_src: np.ndarray, p_dst: np.ndarray) -> np.ndarray:
    """Batched ``cal_relative_pose(p1=p_src, p2=p_dst)`` (``dgl/utils.py:69-77``).

    p_src, p_dst: (M, 7) rows ``(tx, ty, tz, qx, qy, qz, qw)``.  Returns (M, 9) in the
    inputs' floating dtype.
    """
    p1 = _as_float(p_src)
    p2 = _as_float(p_dst)
    if p1.dtype != p2.dtype:
        p1 = p1.astype(np.float64)
        p2 = p2.astype(np.float64)
    x1, y1, z1, w1 = -p1[:, 3], -p1[:, 4], -p1[:, 5], p1[:, 6]  # conjugate of q1
    x2, y2, z2, w2 = p2[:, 3], p2[:, 4], p2[:, 5], p2[:, 6]
    # Hamilton product (q1^-1 on the left, in the reference's expansion)
    qx = w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2
    qy = w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2
    qz = w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2
    qw = w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2
    rot = quat_to_so3_batch(np.stack([qx, qy, qz, qw], axis=1))[:, :6]
    return np.concatenate([p2[:, :3] - p1[:, :3], rot], axis=1)


def cal_relative_pose(p1, p2) -> np.ndarray:
    """Single-pair form with the reference's signature (``dgl/utils.py:69``)."""
    return relative_pose_batch(np.asarray(p1)[None], np.asarray(p2)[None])[0]
