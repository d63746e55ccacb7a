"""Fused env-layer kernels (csrc/mjh_envops.hip) with the torch formulas as the
semantics: on HIP tensors of the supported 2-D row layouts the fused kernel runs
(one launch instead of 5-25 small torch ops, also inside the captured env
step); other shapes — and CPU tensors, which only the CPU test harness uses —
take the torch expression of utils/math.py. Results agree to float32 rounding
(tests/test_gpu_envops.py)."""

from __future__ import annotations

import ctypes

import torch

from mjlab_amd.sim import native
from mjlab_amd.utils import math as M


def _rows(t: torch.Tensor, width: int) -> bool:
  return t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == width and t.stride(1) == 1


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
  return ctypes.c_void_p(t.data_ptr())


def _stream() -> ctypes.c_void_p:
  return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _rotate(q: torch.Tensor, v: torch.Tensor, inverse: bool) -> torch.Tensor:
  n = q.shape[0]
  out = torch.empty((n, 3), dtype=torch.float32, device=q.device)
  native.check(
    native.lib().mjh_quat_rotate(_ptr(q), q.stride(0), _ptr(v), v.stride(0), _ptr(out), n, int(inverse), _stream()),
    "mjh_quat_rotate",
  )
  return out


def quat_apply_inverse(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
  if _rows(q, 4) and _rows(v, 3) and q.shape[0] == v.shape[0]:
    return _rotate(q, v, True)
  return M.quat_apply_inverse(q, v)


def quat_apply(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
  if _rows(q, 4) and _rows(v, 3) and q.shape[0] == v.shape[0]:
    return _rotate(q, v, False)
  return M.quat_apply(q, v)


def quat_mul(p: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
  if _rows(p, 4) and _rows(q, 4) and p.shape[0] == q.shape[0]:
    n = p.shape[0]
    out = torch.empty((n, 4), dtype=torch.float32, device=p.device)
    native.check(native.lib().mjh_quat_mul(_ptr(p), p.stride(0), _ptr(q), q.stride(0), _ptr(out), n, _stream()), "mjh_quat_mul")
    return out
  return M.quat_mul(p, q)


def velocity_from_cvel(pos: torch.Tensor, com: torch.Tensor, cvel: torch.Tensor, reference) -> torch.Tensor:
  """``reference`` is the torch implementation (entity/data.py) for other layouts."""
  if _rows(pos, 3) and _rows(com, 3) and _rows(cvel, 6) and pos.shape[0] == com.shape[0] == cvel.shape[0]:
    n = pos.shape[0]
    out = torch.empty((n, 6), dtype=torch.float32, device=pos.device)
    native.check(
      native.lib().mjh_velocity_from_cvel(
        _ptr(pos), pos.stride(0), _ptr(com), com.stride(0), _ptr(cvel), cvel.stride(0), _ptr(out), n, _stream()
      ),
      "mjh_velocity_from_cvel",
    )
    return out
  return reference(pos, com, cvel)


def air_time_update(sensordata, cols, time, last_time, cur_air, last_air, cur_con, last_con) -> bool:
  """Fused contact-sensor timer update; returns False if the layout is unsupported."""
  if not (sensordata.is_cuda and sensordata.stride(1) == 1 and cols.is_cuda and cols.dtype == torch.int32):
    return False
  if not all(t.is_contiguous() for t in (time, last_time, cur_air, last_air, cur_con, last_con)):
    return False
  n, k = cur_air.shape
  native.check(
    native.lib().mjh_air_time_update(
      _ptr(sensordata), sensordata.stride(0), _ptr(cols), k, _ptr(time), _ptr(last_time), _ptr(cur_air),
      _ptr(last_air), _ptr(cur_con), _ptr(last_con), n, _stream(),
    ),
    "mjh_air_time_update",
  )
  return True


def obs_term(x: torch.Tensor, out: torch.Tensor, u: torch.Tensor | None, lo: float, hi: float, clip, scale: float) -> bool:
  """out[:] = clip(x + U(lo, hi), clip) * scale in one launch; False if unsupported."""
  if not (x.is_cuda and out.is_cuda and x.dtype == torch.float32):
    return False
  if x.dim() == 1:
    x2 = x.view(-1, 1)
  elif x.dim() == 2:
    x2 = x
  else:
    return False
  n, w = x2.shape
  if out.shape != (n, w) or out.stride(1) != 1 or x2.stride(1) != 1 or (u is not None and u.stride(1) != 1):
    return False
  cmin, cmax = (float(clip[0]), float(clip[1])) if clip else (1.0, -1.0)
  native.check(
    native.lib().mjh_obs_term(
      _ptr(x2), x2.stride(0), _ptr(u) if u is not None else None, u.stride(0) if u is not None else 0, float(lo), float(hi),
      cmin, cmax, float(scale), _ptr(out), out.stride(0), w, n, _stream(),
    ),
    "mjh_obs_term",
  )
  return True
