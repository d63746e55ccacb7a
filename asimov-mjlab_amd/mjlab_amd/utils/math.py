"""Torch quaternion / sampling helpers used by the env layer.

Conventions and results match the Isaac Lab math mjlab vendors
(``src/mjlab/third_party/isaaclab/isaaclab/utils/math.py``): quaternions are
(w, x, y, z); ``quat_apply_inverse`` rotates by the conjugate (line 651),
``quat_from_euler_xyz`` composes yaw·pitch·roll (line 275),
``sample_uniform`` is ``(upper - lower) * rand + lower`` (line 1360).
All functions are pure torch and capture-safe (no host syncs).
"""

from __future__ import annotations

import torch


def quat_mul(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  shape = q1.shape
  q1 = q1.reshape(-1, 4)
  q2 = q2.reshape(-1, 4)
  w1, x1, y1, z1 = q1[:, 0], q1[:, 1], q1[:, 2], q1[:, 3]
  w2, x2, y2, z2 = q2[:, 0], q2[:, 1], q2[:, 2], q2[:, 3]
  ww = (z1 + x1) * (x2 + y2)
  yy = (w1 - y1) * (w2 + z2)
  zz = (w1 + y1) * (w2 - z2)
  xx = ww + yy + zz
  qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
  w = qq - ww + (z1 - y1) * (y2 - z2)
  x = qq - xx + (x1 + w1) * (x2 + w2)
  y = qq - yy + (w1 - x1) * (y2 + z2)
  z = qq - zz + (z1 + y1) * (w2 - x2)
  return torch.stack([w, x, y, z], dim=-1).view(shape)


def quat_conjugate(q: torch.Tensor) -> torch.Tensor:
  return torch.cat((q[..., 0:1], -q[..., 1:]), dim=-1)


def quat_apply(quat: torch.Tensor, vec: torch.Tensor) -> torch.Tensor:
  shape = vec.shape
  quat = quat.reshape(-1, 4)
  vec = vec.reshape(-1, 3)
  xyz = quat[:, 1:]
  t = xyz.cross(vec, dim=-1) * 2
  return (vec + quat[:, 0:1] * t + xyz.cross(t, dim=-1)).view(shape)


def quat_apply_inverse(quat: torch.Tensor, vec: torch.Tensor) -> torch.Tensor:
  shape = vec.shape
  quat = quat.reshape(-1, 4)
  vec = vec.reshape(-1, 3)
  xyz = quat[:, 1:]
  t = xyz.cross(vec, dim=-1) * 2
  return (vec - quat[:, 0:1] * t + xyz.cross(t, dim=-1)).view(shape)


def quat_from_euler_xyz(roll: torch.Tensor, pitch: torch.Tensor, yaw: torch.Tensor) -> torch.Tensor:
  cy = torch.cos(yaw * 0.5)
  sy = torch.sin(yaw * 0.5)
  cr = torch.cos(roll * 0.5)
  sr = torch.sin(roll * 0.5)
  cp = torch.cos(pitch * 0.5)
  sp = torch.sin(pitch * 0.5)
  qw = cy * cr * cp + sy * sr * sp
  qx = cy * sr * cp - sy * cr * sp
  qy = cy * cr * sp + sy * sr * cp
  qz = sy * cr * cp - cy * sr * sp
  return torch.stack([qw, qx, qy, qz], dim=-1)


def quat_from_matrix(matrix: torch.Tensor) -> torch.Tensor:
  """Rotation matrix (..., 3, 3) or flattened (..., 9) to quaternion, w >= 0."""
  if matrix.shape[-1] == 9:
    matrix = matrix.reshape(*matrix.shape[:-1], 3, 3)
  m00, m01, m02 = matrix[..., 0, 0], matrix[..., 0, 1], matrix[..., 0, 2]
  m10, m11, m12 = matrix[..., 1, 0], matrix[..., 1, 1], matrix[..., 1, 2]
  m20, m21, m22 = matrix[..., 2, 0], matrix[..., 2, 1], matrix[..., 2, 2]
  q_abs = torch.sqrt(
    torch.clamp(
      torch.stack(
        [1 + m00 + m11 + m22, 1 + m00 - m11 - m22, 1 - m00 + m11 - m22, 1 - m00 - m11 + m22],
        dim=-1,
      ),
      min=0.0,
    )
  )
  quat_by = torch.stack(
    [
      torch.stack([q_abs[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], dim=-1),
      torch.stack([m21 - m12, q_abs[..., 1] ** 2, m10 + m01, m02 + m20], dim=-1),
      torch.stack([m02 - m20, m10 + m01, q_abs[..., 2] ** 2, m12 + m21], dim=-1),
      torch.stack([m10 - m01, m20 + m02, m21 + m12, q_abs[..., 3] ** 2], dim=-1),
    ],
    dim=-2,
  )
  # floor 0.1 as a scalar clamp (a host-made tensor here would be an H2D copy
  # inside the captured env step); best-conditioned candidate, no sign fix-up
  cand = quat_by / (2.0 * q_abs[..., None].clamp(min=0.1))
  idx = q_abs.argmax(dim=-1, keepdim=True)
  return torch.gather(cand, -2, idx[..., None].expand(*idx.shape, 4)).squeeze(-2)


def yaw_quat(quat: torch.Tensor) -> torch.Tensor:
  shape = quat.shape
  q = quat.reshape(-1, 4)
  qw, qx, qy, qz = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
  yaw = torch.atan2(2 * (qw * qz + qx * qy), 1 - 2 * (qy * qy + qz * qz))
  out = torch.zeros_like(q)
  out[:, 0] = torch.cos(yaw / 2)
  out[:, 3] = torch.sin(yaw / 2)
  return (out / out.norm(dim=-1, keepdim=True)).view(shape)


def wrap_to_pi(angles: torch.Tensor) -> torch.Tensor:
  wrapped = torch.remainder(angles, 2 * torch.pi)
  return torch.where((wrapped > torch.pi), wrapped - 2 * torch.pi, wrapped)


def sample_uniform(lower, upper, size, device, generator: torch.Generator | None = None) -> torch.Tensor:
  if isinstance(size, int):
    size = (size,)
  return torch.rand(*size, device=device, generator=generator) * (upper - lower) + lower


def matrix_from_quat(q: torch.Tensor) -> torch.Tensor:
  w, x, y, z = torch.unbind(q, -1)
  two_s = 2.0 / (q * q).sum(-1)
  o = torch.stack(
    (
      1 - two_s * (y * y + z * z),
      two_s * (x * y - z * w),
      two_s * (x * z + y * w),
      two_s * (x * y + z * w),
      1 - two_s * (x * x + z * z),
      two_s * (y * z - x * w),
      two_s * (x * z - y * w),
      two_s * (y * z + x * w),
      1 - two_s * (x * x + y * y),
    ),
    -1,
  )
  return o.reshape(q.shape[:-1] + (3, 3))


def quat_inv(q: torch.Tensor, eps: float = 1e-9) -> torch.Tensor:
  """conj(q) / |q|^2 (isaaclab math.py:261-271)."""
  return quat_conjugate(q) / q.pow(2).sum(dim=-1, keepdim=True).clamp(min=eps)


def axis_angle_from_quat(quat: torch.Tensor, eps: float = 1.0e-6) -> torch.Tensor:
  """Rotation vector of a (w, x, y, z) quaternion (math.py:478-505)."""
  quat = quat * (1.0 - 2.0 * (quat[..., 0:1] < 0.0))
  mag = torch.linalg.norm(quat[..., 1:], dim=-1)
  half_angle = torch.atan2(mag, quat[..., 0])
  angle = 2.0 * half_angle
  s = torch.where(angle.abs() > eps, torch.sin(half_angle) / angle, 0.5 - angle * angle / 48)
  return quat[..., 1:4] / s.unsqueeze(-1)


def quat_error_magnitude(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  """|log(q1 q2^*)| (quat_box_minus, math.py:596-604,688-699)."""
  shape = q1.shape
  d = quat_mul(q1.reshape(-1, 4), quat_conjugate(q2).reshape(-1, 4)).view(shape)
  return torch.norm(axis_angle_from_quat(d), dim=-1)


def subtract_frame_transforms(t01, q01, t02=None, q02=None):
  """T12 = T01^-1 T02 (math.py:832-864)."""
  q10 = quat_inv(q01)
  q12 = quat_mul(q10, q02) if q02 is not None else q10
  t12 = quat_apply(q10, t02 - t01) if t02 is not None else quat_apply(q10, -t01)
  return t12, q12
