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


# ---- job batches (csrc/mjh_batch.h) ---------------------------------------------
_OPEN_BATCH = None


class JobBatch:
  """Context for a pass of independent per-env fused kernels (the reward terms):
  inside it the batchable entry points record their job (mjh_batch_begin) and
  the exit launches them all at once (mjh_batch_end: one dispatch per kernel
  source file instead of one per term). The jobs' outputs must not be read
  before the exit. The inputs they were recorded with are kept alive until the
  batch has been launched (a temporary freed earlier could be reused by a
  later allocation on the stream before the batch reads it). CPU tensors: no-op."""

  def __init__(self, like: torch.Tensor, sequential: bool = False) -> None:
    self.on = bool(like.is_cuda)
    self.sequential = sequential
    self.keep: list = []

  def __enter__(self) -> "JobBatch":
    global _OPEN_BATCH
    if self.on and _OPEN_BATCH is None:
      native.check(native.lib().mjh_batch_begin(int(self.sequential)), "mjh_batch_begin")
      _OPEN_BATCH = self
    return self

  def __exit__(self, *exc) -> bool:
    global _OPEN_BATCH
    if _OPEN_BATCH is self:
      _OPEN_BATCH = None
      native.check(native.lib().mjh_batch_end(_stream()), "mjh_batch_end")
      self.keep.clear()
    return False


def refuse_fallback_in_batch(name: str) -> None:
  """A torch fallback inside an open sequential batch would read outputs of jobs
  recorded before it, which have not run yet: refuse it loudly (the env enables
  such batches only for term sets whose kernels all fuse)."""
  if _OPEN_BATCH is not None and _OPEN_BATCH.sequential:
    raise RuntimeError(f"{name}: torch fallback inside an open sequential job batch (its inputs are recorded, "
                       "not yet launched jobs' outputs)")


def _keep(*ts) -> None:
  """Inputs of a job recorded into the open batch stay referenced until it launches."""
  if _OPEN_BATCH is not None:
    _OPEN_BATCH.keep.extend(t for t in ts if isinstance(t, torch.Tensor))


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
  """``reference`` is the torch implementation (entity/data.py) for other layouts.
  2-D: (N, 3) rows; 3-D: (N, k, 3) contiguous rows sharing a (N, 1, 3) com."""
  if _rows(pos, 3) and _rows(com, 3) and _rows(cvel, 6) and pos.shape[0] == com.shape[0] == cvel.shape[0]:
    n, k, rows = pos.shape[0], 1, (pos, com, cvel)
  elif (
    pos.is_cuda and pos.dim() == 3 and cvel.dim() == 3 and com.dim() == 3 and pos.is_contiguous() and cvel.is_contiguous()
    and com.shape[1] == 1 and com.stride(2) == 1 and pos.shape[:2] == cvel.shape[:2] and pos.shape[0] == com.shape[0]
    and pos.shape[2] == 3 and cvel.shape[2] == 6 and pos.dtype == cvel.dtype == com.dtype == torch.float32
  ):
    n, k = pos.shape[0] * pos.shape[1], pos.shape[1]
    rows = (pos.view(-1, 3), com[:, 0, :], cvel.view(-1, 6))
  else:
    return reference(pos, com, cvel)
  p2, c2, v2 = rows
  out = torch.empty((n, 6), dtype=torch.float32, device=pos.device)
  native.check(
    native.lib().mjh_velocity_from_cvel(
      _ptr(p2), p2.stride(0), _ptr(c2), c2.stride(0), _ptr(v2), v2.stride(0), _ptr(out), n, k, _stream()
    ),
    "mjh_velocity_from_cvel",
  )
  return out.view(*pos.shape[:-1], 6)


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
    x2 = x.unsqueeze(1)  # (n, 1) with strides (s, 1)
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


# ---- fused reward terms (csrc/mjh_mdp.hip) -------------------------------------
def _vec_out(n: int, device) -> torch.Tensor:
  return torch.empty(n, dtype=torch.float32, device=device)


def rew_track(cmd: torch.Tensor, v: torch.Tensor, std: float, angular: bool):
  if not (_rows(cmd, 3) and _rows(v, 3) and cmd.shape[0] == v.shape[0]):
    return None
  out = _vec_out(cmd.shape[0], cmd.device)
  _keep(cmd, v)
  native.check(native.lib().mjh_rew_track(_ptr(cmd), cmd.stride(0), _ptr(v), v.stride(0), 1.0 / (std * std), int(angular),
                                          _ptr(out), cmd.shape[0], _stream()), "mjh_rew_track")
  return out


def rew_flat_orientation(q: torch.Tensor, g: torch.Tensor, std: float):
  if not (_rows(q, 4) and _rows(g, 3) and q.shape[0] == g.shape[0]):
    return None
  out = _vec_out(q.shape[0], q.device)
  _keep(q, g)
  native.check(native.lib().mjh_rew_flat_orientation(_ptr(q), q.stride(0), _ptr(g), g.stride(0), 1.0 / (std * std), _ptr(out),
                                                     q.shape[0], _stream()), "mjh_rew_flat_orientation")
  return out


def rew_sqsum(x: torch.Tensor, k: int):
  if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1 and x.shape[1] >= k):
    return None
  out = _vec_out(x.shape[0], x.device)
  _keep(x)
  native.check(native.lib().mjh_rew_sqsum(_ptr(x), x.stride(0), k, _ptr(out), x.shape[0], _stream()), "mjh_rew_sqsum")
  return out


def rew_diffsq(a: torch.Tensor, b: torch.Tensor):
  ok = all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 for t in (a, b))
  if not ok or a.shape != b.shape:
    return None
  out = _vec_out(a.shape[0], a.device)
  _keep(a, b)
  native.check(native.lib().mjh_rew_diffsq(_ptr(a), a.stride(0), _ptr(b), b.stride(0), a.shape[1], _ptr(out), a.shape[0],
                                           _stream()), "mjh_rew_diffsq")
  return out


def rew_pos_limits(q: torch.Tensor, lim: torch.Tensor):
  if not (q.is_cuda and q.dim() == 2 and q.stride(1) == 1 and lim.dim() == 3 and lim.shape[:2] == q.shape
          and lim.stride(2) == 1 and lim.stride(1) == 2 and q.dtype == lim.dtype == torch.float32):
    return None
  out = _vec_out(q.shape[0], q.device)
  _keep(q, lim)
  native.check(native.lib().mjh_rew_pos_limits(_ptr(q), q.stride(0), _ptr(lim), lim.stride(0), q.shape[1], _ptr(out),
                                               q.shape[0], _stream()), "mjh_rew_pos_limits")
  return out


def rew_posture(q, q0, std_stand, std_walk, std_run, cmd, walk_thr, run_thr):
  ok = all(t.is_cuda and t.dtype == torch.float32 and t.stride(-1) == 1 for t in (q, q0, std_stand, std_walk, std_run, cmd))
  if not ok or q.dim() != 2 or q0.shape != q.shape or not _rows(cmd, 3):
    return None
  if not all(t.is_contiguous() and t.numel() == q.shape[1] for t in (std_stand, std_walk, std_run)):
    return None
  out = _vec_out(q.shape[0], q.device)
  _keep(q, q0, std_stand, std_walk, std_run, cmd)
  native.check(native.lib().mjh_rew_posture(
    _ptr(q), q.stride(0), _ptr(q0), q0.stride(0), _ptr(std_stand), _ptr(std_walk), _ptr(std_run), _ptr(cmd), cmd.stride(0),
    float(walk_thr), float(run_thr), q.shape[1], _ptr(out), q.shape[0], _stream()), "mjh_rew_posture")
  return out


def rew_feet(pos: torch.Tensor, vel: torch.Tensor, found, cmd: torch.Tensor, target: float, thr_clear: float,
             thr_slip: float, want: str):
  """want = "clearance" -> (N,) cost; "slip" -> (cost, sum |v_xy|*found, sum found)."""
  if not (pos.is_cuda and pos.dim() == 3 and vel.dim() == 3 and pos.stride(2) == 1 and vel.stride(2) == 1
          and pos.stride(1) >= 3 and vel.stride(1) >= 3 and pos.shape[:2] == vel.shape[:2] and _rows(cmd, 3)):
    return None
  n, k = pos.shape[0], pos.shape[1]
  # strided views are read in place (velocity rows of 6, sensor-slot columns)
  if found is not None and not (found.dim() == 2 and found.shape == (n, k) and found.dtype == torch.float32
                                and found.is_cuda):
    return None
  if want == "slip" and found is None:  # the slip reward needs the contact flags: torch path
    return None
  z = pos[:, :, 2]
  cl = _vec_out(n, pos.device) if want == "clearance" else None
  outs = [_vec_out(n, pos.device) for _ in range(3)] if want == "slip" else [None, None, None]
  _keep(pos, vel, found, cmd)
  native.check(native.lib().mjh_rew_feet(
    ctypes.c_void_p(pos.data_ptr() + 8), pos.stride(0), pos.stride(1), _ptr(vel), vel.stride(0), vel.stride(1),
    _ptr(found) if want == "slip" else None, found.stride(0) if want == "slip" else 0,
    found.stride(1) if want == "slip" else 0, _ptr(cmd), cmd.stride(0),
    float(target), float(thr_clear), float(thr_slip), k, _ptr(cl) if cl is not None else None,
    *[_ptr(t) if t is not None else None for t in outs], n, _stream()), "mjh_rew_feet")
  del z
  return cl if want == "clearance" else tuple(outs)


# ---- rotations for resets and motion tracking --------------------------------
def _rowsN(t: torch.Tensor, width: int) -> bool:
  """(n, width) float32 rows on the GPU with unit last-dim stride (any row stride)."""
  return t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == width and t.stride(1) == 1


def _flat_rows(t: torch.Tensor, width: int):
  """(..., width) -> (n, width) rows without a copy when possible, else None."""
  if not (t.is_cuda and t.dtype == torch.float32 and t.shape[-1] == width and t.stride(-1) == 1):
    return None
  if t.dim() == 2:
    return t
  try:
    return t.view(-1, width)
  except RuntimeError:
    return None


def quat_from_euler_xyz(rpy: torch.Tensor) -> torch.Tensor:
  """quat_from_euler_xyz(rpy[:, 0], rpy[:, 1], rpy[:, 2]) for (n, 3) rows."""
  if not _rowsN(rpy, 3):
    return M.quat_from_euler_xyz(rpy[:, 0], rpy[:, 1], rpy[:, 2])
  n = rpy.shape[0]
  out = torch.empty((n, 4), dtype=torch.float32, device=rpy.device)
  native.check(native.lib().mjh_quat_from_euler(_ptr(rpy), rpy.stride(0), _ptr(out), n, _stream()), "mjh_quat_from_euler")
  return out


def quat_error_magnitude(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  a, b = _flat_rows(q1, 4), _flat_rows(q2, 4)
  if a is None or b is None or q1.shape != q2.shape:
    return M.quat_error_magnitude(q1, q2)
  out = torch.empty(q1.shape[:-1], dtype=torch.float32, device=q1.device)
  native.check(native.lib().mjh_quat_error(_ptr(a), a.stride(0), _ptr(b), b.stride(0), _ptr(out), a.shape[0], _stream()),
               "mjh_quat_error")
  return out


def _env_rows(t: torch.Tensor, width: int):
  """(N, width) or (N, k, width) float32 GPU tensor with unit last stride ->
  (k, env stride, row stride), else None."""
  if not (t.is_cuda and t.dtype == torch.float32 and t.shape[-1] == width and t.stride(-1) == 1):
    return None
  if t.dim() == 2:
    return 1, t.stride(0), 0
  if t.dim() == 3:
    return t.shape[1], t.stride(0), t.stride(1)
  return None


def frame_subtract(t01, q01, t02, q02, want_t: bool = True, want_q: bool = True, qcols: int = 0):
  """subtract_frame_transforms with (N, 3)/(N, 4) frames and (N, k, 3)/(N, k, 4)
  or (N, 3)/(N, 4) targets. Returns (t12, q12), q12 optionally as the first
  `qcols` columns of its rotation matrix, flattened per target row."""
  et, eq = _env_rows(t02, 3), _env_rows(q02, 4)
  ok = _rowsN(t01, 3) and _rowsN(q01, 4) and et is not None and eq is not None and et[0] == eq[0]
  if not ok or t02.shape[:-1] != q02.shape[:-1] or t01.shape[0] != t02.shape[0]:
    k = t02.shape[1] if t02.dim() == 3 else 1
    if t02.dim() == 3:
      t01, q01 = t01[:, None, :].expand(-1, k, -1), q01[:, None, :].expand(-1, k, -1)
    t12, q12 = M.subtract_frame_transforms(t01, q01, t02, q02)
    if qcols:
      q12 = M.matrix_from_quat(q12)[..., :qcols].reshape(*q12.shape[:-1], 3 * qcols)
    return (t12 if want_t else None), (q12 if want_q else None)
  k = et[0]
  n = t02.shape[0] * k
  t12 = torch.empty((*t02.shape[:-1], 3), dtype=torch.float32, device=t02.device) if want_t else None
  qw = 3 * qcols if qcols else 4
  q12 = torch.empty((*q02.shape[:-1], qw), dtype=torch.float32, device=q02.device) if want_q else None
  native.check(native.lib().mjh_frame_subtract(
    _ptr(t01), t01.stride(0), _ptr(q01), q01.stride(0), _ptr(t02), et[1], et[2], _ptr(q02), eq[1], eq[2], k,
    _ptr(t12) if t12 is not None else None, _ptr(q12) if q12 is not None else None, qcols, n, _stream()),
    "mjh_frame_subtract")
  return t12, q12


def motion_relative(anchor_pos, anchor_quat, robot_anchor_pos, robot_anchor_quat, body_pos, body_quat, out_pos, out_quat) -> bool:
  """MotionCommand's anchor-relative targets into out_pos (N, k, 3) / out_quat (N, k, 4);
  False when the layout is not supported (caller runs the torch formulas)."""
  ep, eq = _env_rows(body_pos, 3), _env_rows(body_quat, 4)
  if ep is None or eq is None or ep[0] != eq[0] or body_pos.dim() != 3:
    return False
  if not all(_rowsN(t, w) for t, w in ((anchor_pos, 3), (anchor_quat, 4), (robot_anchor_pos, 3), (robot_anchor_quat, 4))):
    return False
  if not (out_pos.is_contiguous() and out_quat.is_contiguous() and out_pos.shape == body_pos.shape):
    return False
  k = ep[0]
  native.check(native.lib().mjh_motion_relative(
    _ptr(anchor_pos), anchor_pos.stride(0), _ptr(anchor_quat), anchor_quat.stride(0), _ptr(robot_anchor_pos),
    robot_anchor_pos.stride(0), _ptr(robot_anchor_quat), robot_anchor_quat.stride(0), _ptr(body_pos), ep[1], ep[2],
    _ptr(body_quat), eq[1], eq[2], k, _ptr(out_pos), _ptr(out_quat), body_pos.shape[0] * k, _stream()),
    "mjh_motion_relative")
  return True


# ---- manager-level fusion (csrc/mjh_mgr.hip) -------------------------------------
MAX_TERMS = 32


class ObsTermDesc(ctypes.Structure):
  """mjh_obs_term_desc (include/mjh_abi.h)."""
  _fields_ = [("x", ctypes.c_void_p), ("xs", ctypes.c_longlong), ("w", ctypes.c_int), ("off", ctypes.c_int),
              ("lo", ctypes.c_float), ("hi", ctypes.c_float), ("cmin", ctypes.c_float), ("cmax", ctypes.c_float),
              ("scale", ctypes.c_float), ("noise", ctypes.c_int), ("y", ctypes.c_void_p), ("ys", ctypes.c_longlong),
              ("xcs", ctypes.c_longlong), ("op", ctypes.c_int), ("xd", ctypes.c_int)]


OBS_COPY, OBS_SUB, OBS_POSITIVE, OBS_SIGNED_LOG1P = 0, 1, 2, 3


class ObsSrc:
  """An observation term as an elementwise op on strided device inputs, which
  the group kernel evaluates while assembling the group (no per-term launch):
  x (n, w) any strides, or (n, k, d) rows of d contiguous floats (columns
  flattened row-major); OBS_SUB subtracts y (n, w) (unit column stride)."""

  __slots__ = ("x", "op", "y")

  def __init__(self, x: torch.Tensor, op: int = OBS_COPY, y: torch.Tensor | None = None) -> None:
    self.x, self.op, self.y = x, op, y

  def evaluate(self) -> torch.Tensor:
    """The torch formula of the op (reference for the fused evaluation)."""
    x = self.x if self.x.dim() < 3 else self.x.reshape(self.x.shape[0], -1)
    if self.op == OBS_SUB:
      return x - self.y
    if self.op == OBS_POSITIVE:
      return (x > 0).float()
    if self.op == OBS_SIGNED_LOG1P:
      return torch.sign(x) * torch.log1p(torch.abs(x))
    return x


def _term_rows(x: torch.Tensor):
  """(n,) or (n, w) float32 GPU tensor (any strides) -> (2-D view, w), else None."""
  if not (x.is_cuda and x.dtype == torch.float32):
    return None
  if x.dim() == 1:
    x = x.unsqueeze(1)  # (n, 1)
  if x.dim() != 2:
    return None
  return x, x.shape[1]


def obs_group(xs: list, plan: list, u: torch.Tensor | None, out: torch.Tensor, rng=None) -> bool:
  """All terms of a concatenated observation group in one launch.
  xs[i]: the term's tensor or an ObsSrc; plan[i] = (tcfg, off, w, noise (lo, hi) |
  None, clip | None, scale); noise draws from u (n, width) or, when u is None,
  the device stream rng = (seed, key, counter ptr) of envops.rng_args."""
  if len(xs) > MAX_TERMS or not out.is_cuda or out.stride(1) != 1 or (u is not None and u.stride(1) != 1):
    return False
  if u is None and rng is None and any(p[3] is not None for p in plan):
    return False
  n = out.shape[0]
  descs = (ObsTermDesc * len(xs))()
  for i, (x, (_, off, w, noise, clip, scale)) in enumerate(zip(xs, plan)):
    op, y, xd = OBS_COPY, None, 1
    if isinstance(x, ObsSrc):
      op, y, x = x.op, x.y, x.x
      if y is not None and not (y.is_cuda and y.dtype == torch.float32 and y.dim() == 2 and y.stride(1) == 1
                                and y.shape == (n, w)):
        return False
      if x.dim() == 3:  # rows of d contiguous floats at a row stride
        if not (x.is_cuda and x.dtype == torch.float32 and x.stride(2) == 1 and x.shape[1] * x.shape[2] == w):
          return False
        xd = x.shape[2]
        x = x.as_strided((x.shape[0], x.shape[1]), (x.stride(0), x.stride(1)))
        r = (x, w)
      else:
        r = _term_rows(x)
    else:
      r = _term_rows(x)
    if r is None or r[1] != w or r[0].shape[0] != n:
      return False
    x2 = r[0]
    cmin, cmax = (float(clip[0]), float(clip[1])) if clip else (1.0, -1.0)
    lo, hi = noise if noise is not None else (0.0, 0.0)
    descs[i] = ObsTermDesc(x2.data_ptr(), x2.stride(0), w, off, float(lo), float(hi), cmin, cmax, float(scale),
                           int(noise is not None), y.data_ptr() if y is not None else None, y.stride(0) if y is not None else 0,
                           x2.stride(1), op, xd)
  seed, key, ctr = rng if rng is not None else (ctypes.c_ulonglong(0), ctypes.c_ulonglong(0), None)
  native.check(native.lib().mjh_obs_group(descs, len(xs), _ptr(u) if u is not None else None,
                                          u.stride(0) if u is not None else 0, _ptr(out), out.stride(0), n, seed, key, ctr,
                                          _stream()), "mjh_obs_group")
  return True


def reward_combine(vals: list, weights: torch.Tensor, dt: float, reward: torch.Tensor, step_reward: torch.Tensor,
                   sums: torch.Tensor) -> bool:
  """RewardManager's weight/accumulate/sum over term vectors (None = weight-0 term) in one launch."""
  T = len(vals)
  if T > MAX_TERMS or not (reward.is_cuda and reward.is_contiguous() and step_reward.is_contiguous() and sums.is_contiguous()):
    return False
  n = reward.shape[0]
  ptrs = (ctypes.c_void_p * max(T, 1))()
  strides = (ctypes.c_longlong * max(T, 1))()
  for i, v in enumerate(vals):
    if v is None:
      continue
    if not (v.is_cuda and v.dtype == torch.float32 and v.dim() == 1 and v.shape[0] == n):
      return False
    ptrs[i] = v.data_ptr()
    strides[i] = v.stride(0)
  native.check(native.lib().mjh_reward_combine(ptrs, strides, T, _ptr(weights), float(dt), _ptr(reward),
                                               _ptr(step_reward), _ptr(sums), n, _stream()), "mjh_reward_combine")
  return True


# ---- reset path, events and commands (csrc/mjh_fuse.hip) -----------------------
def _bool_mask(m) -> bool:
  return m is None or (isinstance(m, torch.Tensor) and m.is_cuda and m.dtype == torch.bool and m.dim() == 1
                       and m.is_contiguous())


def _mptr(m):
  return _ptr(m) if m is not None else None


def _site_hash(site: str) -> int:
  h = 1469598103934665603
  for ch in site.encode():
    h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
  return h


def rng_args(env, site: str):
  """(seed, key, step-counter pointer) of the device random stream for one call
  site: draws differ per site, per env step (the counter is a device tensor the
  env step increments, so graph replays draw anew) and per host call."""
  salt = env.__dict__.get("_rng_calls", 0) + 1
  env.__dict__["_rng_calls"] = salt
  key = (_site_hash(site) ^ (salt * 0x9E3779B97F4A7C15)) & 0xFFFFFFFFFFFFFFFF
  return ctypes.c_ulonglong(env._rng_seed), ctypes.c_ulonglong(key), _ptr(env._rng_ctr)


def uniform_draws(seed, key, ctr: torch.Tensor | None, n: int, device) -> torch.Tensor:
  """The U[0,1) stream the fused kernels draw from (tests reconstruct them with it)."""
  out = torch.empty(n, dtype=torch.float32, device=device)
  native.check(native.lib().mjh_uniform_draws(_ptr(out), n, ctypes.c_ulonglong(seed), ctypes.c_ulonglong(key),
                                              _ptr(ctr) if ctr is not None else None, _stream()), "mjh_uniform_draws")
  return out


def masked_means(cols: list, mask, scale: float, zero_rows: bool, out: torch.Tensor) -> bool:
  """out[t] = scale * mean over masked rows of cols[t] (and clear them) in one launch."""
  T = len(cols)
  if T == 0 or T > MAX_TERMS or not _bool_mask(mask) or not out.is_cuda or out.numel() < T:
    return False
  n = cols[0].shape[0]
  ptrs = (ctypes.c_void_p * T)()
  strides = (ctypes.c_longlong * T)()
  for i, c in enumerate(cols):
    if not (c.is_cuda and c.dtype == torch.float32 and c.dim() == 1 and c.shape[0] == n):
      return False
    ptrs[i], strides[i] = c.data_ptr(), c.stride(0)
  if mask is not None and mask.shape[0] != n:
    return False
  native.check(native.lib().mjh_masked_means(ptrs, strides, T, _mptr(mask), float(scale), int(zero_rows), _ptr(out), n,
                                             _stream()), "mjh_masked_means")
  return True


def masked_counts(flags: list, mask, out: torch.Tensor) -> bool:
  """out[t] = count(flags[t] & mask) (int64) in one launch."""
  T = len(flags)
  if T == 0 or T > MAX_TERMS or not _bool_mask(mask) or out.dtype != torch.int64 or not out.is_cuda:
    return False
  if not all(_bool_mask(f) and f is not None for f in flags):
    return False
  ptrs = (ctypes.c_void_p * T)(*[f.data_ptr() for f in flags])
  native.check(native.lib().mjh_masked_counts(ptrs, T, _mptr(mask), _ptr(out), flags[0].shape[0], _stream()),
               "mjh_masked_counts")
  return True


def uniform_where(env, site: str, t: torch.Tensor, mask, lo: float, hi: float) -> bool:
  """t[mask] = U[lo, hi) in one launch (draws from the device stream)."""
  if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 1 and t.is_contiguous() and _bool_mask(mask)):
    return False
  seed, key, ctr = rng_args(env, site)
  _keep(t, mask)
  native.check(native.lib().mjh_uniform_where(_ptr(t), _mptr(mask), float(lo), float(hi), seed, key, ctr, t.shape[0],
                                              _stream()), "mjh_uniform_where")
  return True


def interval_tick(env, site: str, t: torch.Tensor, dt: float, lo: float, hi: float, due: torch.Tensor) -> bool:
  if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 1 and t.is_contiguous() and _bool_mask(due)):
    return False
  seed, key, ctr = rng_args(env, site)
  _keep(t, due)
  native.check(native.lib().mjh_interval_tick(_ptr(t), float(dt), float(lo), float(hi), _ptr(due), seed, key, ctr,
                                              t.shape[0], _stream()), "mjh_interval_tick")
  return True


def _f6(v) -> ctypes.Array:
  return (ctypes.c_float * 6)(*[float(x) for x in v])


def reset_root_uniform(env, site: str, qpos, qadr: int, qvel, vadr: int, mask, root_state, origins, lo6, hi6, vlo6, vhi6,
                       pose_rand: bool, vel_rand: bool) -> bool:
  ok = all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 for t in (qpos, qvel, root_state, origins))
  if not ok or not _bool_mask(mask) or root_state.shape[1] != 13 or origins.shape[1] != 3:
    return False
  n = qpos.shape[0]
  if root_state.shape[0] != n or origins.shape[0] != n:
    return False
  seed, key, ctr = rng_args(env, site)
  _keep(qpos, qvel, mask, root_state, origins)
  native.check(native.lib().mjh_reset_root_uniform(
    _ptr(qpos), qpos.stride(0), int(qadr), _ptr(qvel), qvel.stride(0), int(vadr), _mptr(mask), _ptr(root_state),
    root_state.stride(0), _ptr(origins), origins.stride(0), _f6(lo6), _f6(hi6), _f6(vlo6), _f6(vhi6), int(pose_rand),
    int(vel_rand), seed, key, ctr, n, _stream()), "mjh_reset_root_uniform")
  return True


def reset_joints_offset(env, site: str, qpos, qadr: int, qvel, vadr: int, mask, def_pos, def_vel, lim, prange, vrange) -> bool:
  ok = all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 for t in (qpos, qvel, def_pos, def_vel))
  if not ok or not _bool_mask(mask) or lim.dim() != 3 or lim.stride(2) != 1 or lim.stride(1) != 2:
    return False
  n, k = def_pos.shape
  if def_vel.shape != (n, k) or lim.shape[:2] != (n, k) or qpos.shape[0] != n or lim.dtype != torch.float32:
    return False
  seed, key, ctr = rng_args(env, site)
  pr, vr = tuple(prange) != (0.0, 0.0), tuple(vrange) != (0.0, 0.0)
  _keep(qpos, qvel, mask, def_pos, def_vel, lim)
  native.check(native.lib().mjh_reset_joints_offset(
    _ptr(qpos), qpos.stride(0), int(qadr), _ptr(qvel), qvel.stride(0), int(vadr), k, _mptr(mask), _ptr(def_pos),
    def_pos.stride(0), _ptr(def_vel), def_vel.stride(0), _ptr(lim), lim.stride(0), float(prange[0]), float(prange[1]),
    float(vrange[0]), float(vrange[1]), int(pr), int(vr), seed, key, ctr, n, _stream()), "mjh_reset_joints_offset")
  return True


def push_velocity(env, site: str, qpos, qadr: int, qvel, vadr: int, mask, vel_w, lo6, hi6) -> bool:
  ok = all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 for t in (qpos, qvel, vel_w))
  if not ok or not _bool_mask(mask) or vel_w.shape != (qpos.shape[0], 6):
    return False
  seed, key, ctr = rng_args(env, site)
  _keep(qpos, qvel, mask, vel_w)
  native.check(native.lib().mjh_push_velocity(
    _ptr(qpos), qpos.stride(0), int(qadr), _ptr(qvel), qvel.stride(0), int(vadr), _mptr(mask), _ptr(vel_w), vel_w.stride(0),
    _f6(lo6), _f6(hi6), seed, key, ctr, qpos.shape[0], _stream()), "mjh_push_velocity")
  return True


def event_mark(last: torch.Tensor, once: torch.Tensor, mask, step: torch.Tensor) -> bool:
  if not (last.is_cuda and last.dtype == torch.int32 and once.dtype == torch.bool and _bool_mask(mask)
          and isinstance(step, torch.Tensor) and step.is_cuda and step.dtype == torch.int64 and step.numel() == 1):
    return False
  _keep(last, once, mask, step)
  native.check(native.lib().mjh_event_mark(_ptr(last), _ptr(once), _mptr(mask), _ptr(step), last.shape[0], _stream()),
               "mjh_event_mark")
  return True


def gz_above(gz: torch.Tensor, thr: float) -> torch.Tensor | None:
  """(thr < gz) & (gz <= 1) as a bool vector in one launch (bad_orientation), or
  None on CPU / an unsupported layout."""
  if not (gz.is_cuda and gz.dtype == torch.float32 and gz.dim() == 1):
    return None
  n = gz.shape[0]
  out = torch.empty(n, dtype=torch.bool, device=gz.device)
  _keep(gz, out)
  native.check(native.lib().mjh_gz_above(_ptr(gz), gz.stride(0), float(thr), _ptr(out), n, _stream()), "mjh_gz_above")
  return out


def time_out(episode_length: torch.Tensor, max_len: int) -> torch.Tensor | None:
  """episode_length >= max_len as a bool vector in one launch (batchable), or None."""
  if not (episode_length.is_cuda and episode_length.dtype == torch.int64 and episode_length.dim() == 1
          and episode_length.is_contiguous()):
    return None
  n = episode_length.shape[0]
  out = torch.empty(n, dtype=torch.bool, device=episode_length.device)
  _keep(episode_length, out)
  native.check(native.lib().mjh_time_out(_ptr(episode_length), int(max_len), _ptr(out), n, _stream()), "mjh_time_out")
  return out


def term_combine(values: list, term_dones: list, time_out: list, truncated, terminated, dones) -> bool:
  """TerminationManager's copy / OR / dones chain over bool term vectors in one launch."""
  T = len(values)
  if T == 0:
    return False
  if T > MAX_TERMS:
    refuse_fallback_in_batch("term_combine")
    return False
  n = dones.shape[0]
  for v in values + term_dones + [truncated, terminated, dones]:
    if not (isinstance(v, torch.Tensor) and v.is_cuda and v.dtype == torch.bool and v.dim() == 1 and v.shape[0] == n
            and v.stride(0) == 1):
      refuse_fallback_in_batch("term_combine")
      return False
  vp = (ctypes.c_void_p * T)(*[v.data_ptr() for v in values])
  dp = (ctypes.c_void_p * T)(*[d.data_ptr() for d in term_dones])
  to = (ctypes.c_int * T)(*[int(bool(x)) for x in time_out])
  _keep(*values, *term_dones, truncated, terminated, dones)
  native.check(native.lib().mjh_term_combine(vp, dp, to, T, _ptr(truncated), _ptr(terminated), _ptr(dones), n, _stream()),
               "mjh_term_combine")
  return True


def velocity_rows(pos: torch.Tensor, com: torch.Tensor, cvel: torch.Tensor, body: torch.Tensor) -> torch.Tensor | None:
  """compute_velocity_from_cvel(pos (N, k, 3) strided view, com (N, 3), cvel[:, body] of
  cvel (N, nbody, 6)) without the gathers, or None if the layout is unsupported."""
  ok = all(t.is_cuda and t.dtype == torch.float32 for t in (pos, com, cvel)) and body.is_cuda and body.dtype == torch.int32
  if not ok or pos.dim() != 3 or pos.stride(2) != 1 or com.dim() != 2 or com.stride(1) != 1 or cvel.dim() != 3:
    return None
  if cvel.stride(2) != 1 or cvel.stride(1) != 6 or body.numel() != pos.shape[1] or not body.is_contiguous():
    return None
  n, k = pos.shape[0], pos.shape[1]
  out = torch.empty((n, k, 6), dtype=torch.float32, device=pos.device)
  native.check(native.lib().mjh_velocity_rows(_ptr(pos), pos.stride(0), pos.stride(1), _ptr(com), com.stride(0), _ptr(cvel),
                                              cvel.stride(0), _ptr(body), _ptr(out), k, n, _stream()), "mjh_velocity_rows")
  return out


def masked_copy(dst: torch.Tensor, src: torch.Tensor, mask) -> bool:
  """dst[mask] = src[mask] for contiguous float vectors in one launch (batchable)."""
  if not (_bool_mask(mask) and mask is not None and all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 1
                                                        and t.is_contiguous() and t.shape == mask.shape for t in (dst, src))):
    return False
  _keep(dst, src, mask)
  native.check(native.lib().mjh_masked_copy(_ptr(dst), _ptr(src), _ptr(mask), dst.shape[0], _stream()), "mjh_masked_copy")
  return True


def masked_zero_i64(dst: torch.Tensor, mask) -> bool:
  """dst[mask] = 0 for a contiguous int64 vector in one launch (batchable)."""
  if not (_bool_mask(mask) and mask is not None and dst.is_cuda and dst.dtype == torch.int64 and dst.dim() == 1
          and dst.is_contiguous() and dst.shape == mask.shape):
    return False
  _keep(dst, mask)
  native.check(native.lib().mjh_masked_zero_i64(_ptr(dst), _ptr(mask), dst.shape[0], _stream()), "mjh_masked_zero_i64")
  return True


def masked_zero(tensors: list, mask) -> bool:
  """t[mask] = 0 for several float tensors (rows of unit column stride) in one launch."""
  T = len(tensors)
  if T == 0 or T > MAX_TERMS or not _bool_mask(mask) or mask is None:
    return False
  n = mask.shape[0]
  ptrs = (ctypes.c_void_p * T)()
  rs = (ctypes.c_longlong * T)()
  ws = (ctypes.c_int * T)()
  for i, t in enumerate(tensors):
    t2 = t.unsqueeze(1) if t.dim() == 1 else (t.reshape(t.shape[0], -1) if t.dim() > 2 and t.is_contiguous() else t)
    if not (t2.is_cuda and t2.dtype == torch.float32 and t2.dim() == 2 and t2.shape[0] == n and (t2.shape[1] == 1 or t2.stride(1) == 1)):
      return False
    ptrs[i], rs[i], ws[i] = t2.data_ptr(), t2.stride(0), t2.shape[1]
  _keep(*tensors, mask)
  native.check(native.lib().mjh_masked_zero(ptrs, rs, ws, T, _ptr(mask), n, _stream()), "mjh_masked_zero")
  return True


def sum_ratios(pairs: list, out: torch.Tensor) -> bool:
  """out[t] = sum(num_t) / max(sum(den_t), 1) for (num_t, den_t) (N,) float vectors
  (den_t None: mean(sqrt(num_t))), one launch."""
  T = len(pairs)
  if T == 0 or T > MAX_TERMS or not out.is_cuda or out.numel() < T:
    return False
  for a, b in pairs:
    if not all(x.is_cuda and x.dtype == torch.float32 and x.dim() == 1 and x.is_contiguous() for x in (a, b) if x is not None):
      return False
  num = (ctypes.c_void_p * T)(*[a.data_ptr() for a, _ in pairs])
  den = (ctypes.c_void_p * T)(*[b.data_ptr() if b is not None else None for _, b in pairs])
  native.check(native.lib().mjh_sum_ratios(num, den, T, _ptr(out), pairs[0][0].shape[0], _stream()), "mjh_sum_ratios")
  return True


def _col_strides(t: torch.Tensor, n: int, k: int):
  """(env stride, column stride) of a float32 (n, k) GPU view, else None."""
  if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape == (n, k)):
    return None
  return t.stride(0), t.stride(1)


def _cmd_args(cmd):
  if cmd is None:
    return None, 0
  return _ptr(cmd), cmd.stride(0)


def rew_air_time(t, cmd, tmin: float, tmax: float, cmd_thr: float):
  """feet_air_time in one launch -> (reward, log num, log den), or None."""
  n, k = t.shape
  st = _col_strides(t, n, k)
  if st is None or st[1] != 1 or (cmd is not None and not _rows(cmd, 3)):
    return None
  out, num, den = (_vec_out(n, t.device) for _ in range(3))
  cp, cs = _cmd_args(cmd)
  _keep(t, cmd)
  native.check(native.lib().mjh_rew_air_time(_ptr(t), st[0], cp, cs, float(tmin), float(tmax), float(cmd_thr), _ptr(out),
                                             _ptr(num), _ptr(den), k, n, _stream()), "mjh_rew_air_time")
  return out, num, den


def rew_swing_height(peak, h, found, cct, cmd, first_lim: float, target: float, cmd_thr: float):
  """feet_swing_height (peak-height state updated in place) in one launch -> (cost, num, den), or None."""
  n, k = peak.shape
  sh, sf, sc = _col_strides(h, n, k), _col_strides(found, n, k), _col_strides(cct, n, k)
  if None in (sh, sf, sc) or not peak.is_contiguous() or sc[1] != 1 or (cmd is not None and not _rows(cmd, 3)):
    return None
  out, num, den = (_vec_out(n, peak.device) for _ in range(3))
  cp, cs = _cmd_args(cmd)
  _keep(peak, h, found, cct, cmd)
  native.check(native.lib().mjh_rew_swing_height(
    _ptr(peak), _ptr(h), sh[0], sh[1], _ptr(found), sf[0], sf[1], _ptr(cct), sc[0], cp, cs, float(first_lim), float(target),
    float(cmd_thr), _ptr(out), _ptr(num), _ptr(den), k, n, _stream()), "mjh_rew_swing_height")
  return out, num, den


def rew_soft_landing(force, cct, cmd, first_lim: float, cmd_thr: float):
  """soft_landing in one launch -> (cost, num, den), or None."""
  if not (force.is_cuda and force.dtype == torch.float32 and force.dim() == 3 and force.shape[2] == 3 and force.stride(2) == 1):
    return None
  n, k = force.shape[:2]
  sc = _col_strides(cct, n, k)
  if sc is None or sc[1] != 1 or (cmd is not None and not _rows(cmd, 3)):
    return None
  out, num, den = (_vec_out(n, force.device) for _ in range(3))
  cp, cs = _cmd_args(cmd)
  _keep(force, cct, cmd)
  native.check(native.lib().mjh_rew_soft_landing(
    _ptr(force), force.stride(0), force.stride(1), _ptr(cct), sc[0], cp, cs, float(first_lim), float(cmd_thr), _ptr(out),
    _ptr(num), _ptr(den), k, n, _stream()), "mjh_rew_soft_landing")
  return out, num, den


def log_ratio(env, key: str, num: torch.Tensor, den: torch.Tensor | None) -> None:
  """extras['log'][key] = sum(num) / max(sum(den), 1), or mean(sqrt(num)) when
  den is None. Inside a reward pass the reward manager evaluates every such log
  of the pass in one launch."""
  pending = env.__dict__.get("_reward_log_ratios")
  if pending is not None:
    pending.append((key, num, den))
    return
  env.extras["log"][key] = ratio_value(num, den)


def ratio_value(num: torch.Tensor, den: torch.Tensor | None) -> torch.Tensor:
  if den is None:
    return torch.mean(torch.sqrt(num))
  return torch.sum(num) / torch.clamp(torch.sum(den), min=1)


def root_frame(xpos, xquat, com, cvel, grav, fwd) -> torch.Tensor | None:
  """(N, 16) [root_link_vel_w | lin_vel_b | ang_vel_b | projected_gravity_b | heading_w]
  of the root body in one launch, or None when the layout is unsupported (CPU)."""
  ts = (xpos, xquat, com, cvel, grav, fwd)
  widths = (3, 4, 3, 6, 3, 3)
  if not all(_rowsN(t, w) for t, w in zip(ts, widths)):
    return None
  n = xpos.shape[0]
  if not all(t.shape[0] == n for t in ts):
    return None
  out = torch.empty((n, 16), dtype=torch.float32, device=xpos.device)
  _keep(xpos, xquat, com, cvel, grav, fwd, out)
  native.check(native.lib().mjh_root_frame(_ptr(xpos), xpos.stride(0), _ptr(xquat), xquat.stride(0), _ptr(com), com.stride(0),
                                           _ptr(cvel), cvel.stride(0), _ptr(grav), grav.stride(0), _ptr(fwd), fwd.stride(0),
                                           _ptr(out), n, _stream()), "mjh_root_frame")
  return out


def joint_action(inp, action, prev, raw, processed, scale, offset) -> bool:
  """ActionManager.process_action for one JointAction term in one launch."""
  n, d = action.shape
  bufs = (action, prev, raw, processed)
  if not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.shape == (n, d) for t in bufs):
    return False
  if not (_rowsN(inp, d) and inp.shape[0] == n):
    return False
  def arg(x):
    if isinstance(x, torch.Tensor):
      if not (_rowsN(x, d) and x.shape[0] == n):
        return None
      return _ptr(x), x.stride(0), 0.0
    return None, 0, float(x)
  sa, oa = arg(scale), arg(offset)
  if sa is None or oa is None:
    return False
  native.check(native.lib().mjh_joint_action(_ptr(inp), inp.stride(0), _ptr(action), _ptr(prev), _ptr(raw), _ptr(processed),
                                             *sa, *oa, d, n, _stream()), "mjh_joint_action")
  return True


def _row_view(t: torch.Tensor, d: int):
  """(N, d) or (N, k, d) float32 GPU view with unit last stride -> (ptr, env stride, row stride, k), else None."""
  if not (t.is_cuda and t.dtype == torch.float32 and t.shape[-1] == d and t.stride(-1) == 1):
    return None
  if t.dim() == 2:
    return t.data_ptr(), t.stride(0), 0, 1
  if t.dim() == 3:
    return t.data_ptr(), t.stride(0), t.stride(1), t.shape[1]
  return None


def rew_exp_err(a: torch.Tensor, b: torch.Tensor, std: float, quat: bool = False, rows_a=None, rows_b=None):
  """exp(-mean_j err_j / std^2) of rows of a and b (rows_*: int32 row indices or None) in one launch, or None."""
  d = 4 if quat else a.shape[-1]
  va, vb = _row_view(a, d), _row_view(b, d)
  if va is None or vb is None or a.shape[0] != b.shape[0]:
    return None
  k = rows_a.numel() if rows_a is not None else va[3]
  kb = rows_b.numel() if rows_b is not None else vb[3]
  if k != kb or k == 0:
    return None
  for r in (rows_a, rows_b):
    if r is not None and not (r.is_cuda and r.dtype == torch.int32 and r.is_contiguous()):
      return None
  n = a.shape[0]
  out = _vec_out(n, a.device)
  native.check(native.lib().mjh_rew_exp_err(
    ctypes.c_void_p(va[0]), va[1], va[2], _ptr(rows_a) if rows_a is not None else None, ctypes.c_void_p(vb[0]), vb[1], vb[2],
    _ptr(rows_b) if rows_b is not None else None, k, d, int(quat), 1.0 / (std * std), _ptr(out), n, _stream()),
    "mjh_rew_exp_err")
  return out


def step_counters(episode_length: torch.Tensor, step: torch.Tensor) -> None:
  """episode_length += 1; step += 1 (int64 device tensors) in one launch."""
  _keep(episode_length, step)
  native.check(native.lib().mjh_step_counters(_ptr(episode_length), _ptr(step), episode_length.shape[0], _stream()),
               "mjh_step_counters")


def reset_stats(reset: torch.Tensor, any_reset: torch.Tensor, stats: torch.Tensor) -> None:
  """any_reset = any(reset); stats += [count, any] in one launch."""
  native.check(native.lib().mjh_reset_stats(_ptr(reset), _ptr(any_reset), _ptr(stats), reset.shape[0], _stream()),
               "mjh_reset_stats")
