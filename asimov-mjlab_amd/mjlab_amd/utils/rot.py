"""Float64 numpy rotation helpers for the model compiler (host side only).

Quaternions are (w, x, y, z), as in MuJoCo and mjlab.
"""

from __future__ import annotations

import numpy as np

MINVAL = 1e-15


def quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
  aw, ax, ay, az = a
  bw, bx, by, bz = b
  return np.array(
    [
      aw * bw - ax * bx - ay * by - az * bz,
      aw * bx + ax * bw + ay * bz - az * by,
      aw * by - ax * bz + ay * bw + az * bx,
      aw * bz + ax * by - ay * bx + az * bw,
    ]
  )


def quat_to_mat(q: np.ndarray) -> np.ndarray:
  w, x, y, z = q
  return np.array(
    [
      [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ]
  )


def rotate(q: np.ndarray, v: np.ndarray) -> np.ndarray:
  return quat_to_mat(q) @ v


def axis_angle_to_quat(axis: np.ndarray, angle: float) -> np.ndarray:
  n = np.linalg.norm(axis)
  if n < MINVAL:
    return np.array([1.0, 0.0, 0.0, 0.0])
  axis = axis / n
  s = np.sin(angle / 2)
  return np.array([np.cos(angle / 2), *(axis * s)])


def mat_to_quat(R: np.ndarray) -> np.ndarray:
  """Rotation matrix (columns = frame axes) to unit quaternion."""
  t = np.trace(R)
  if t > 0:
    s = np.sqrt(t + 1.0) * 2
    q = np.array(
      [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    )
  elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
    s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
    q = np.array(
      [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    )
  elif R[1, 1] > R[2, 2]:
    s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
    q = np.array(
      [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    )
  else:
    s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
    q = np.array(
      [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    )
  if q[0] < 0:
    q = -q
  return q / np.linalg.norm(q)


def quat_z2vec(vec: np.ndarray) -> np.ndarray:
  """Minimal rotation taking +z onto ``vec`` (MuJoCo's ``mju_quatZ2Vec``)."""
  v = np.asarray(vec, dtype=np.float64)
  n = np.linalg.norm(v)
  if n < MINVAL:
    return np.array([1.0, 0.0, 0.0, 0.0])
  v = v / n
  z = np.array([0.0, 0.0, 1.0])
  c = np.cross(z, v)
  s = np.linalg.norm(c)
  if s < 1e-10:
    return np.array([1.0, 0.0, 0.0, 0.0]) if v[2] > 0 else np.array([0.0, 1.0, 0.0, 0.0])
  ang = np.arctan2(s, v[2])
  return axis_angle_to_quat(c / s, ang)
