"""Motion-tracking command (``src/mjlab/tasks/tracking/mdp/commands.py:32-502``).

Same observable semantics as the reference ``MotionCommand`` — reference frame
indexed by a per-env ``time_steps`` counter, start/uniform/adaptive sampling of
the start frame, root pose/velocity and joint perturbations on resample, the
anchor-relative body targets and the failure-weighted adaptive bins — laid out
for a captured env step:

* all motion arrays of one frame are packed into one ``(T, F)`` table at load,
  so fetching the current frame for every env is a single ``index_select`` into
  a persistent ``(N, F)`` buffer (refreshed whenever ``time_steps`` changes);
  the reference's properties re-gather ``motion[time_steps]`` on every read;
* resampling is mask-based: draws for all envs, selected with the mask, no
  ``nonzero``/``len(env_ids)``;
* adaptive sampling draws bins by inverse-CDF (``searchsorted`` on the
  cumulative, capture-safe) instead of ``torch.multinomial`` — same categorical
  distribution; the non-causal smoothing kernel is a gather-and-weight instead
  of ``conv1d`` with replicate padding — same sums; the failed-bin histogram is
  a ``scatter_add`` instead of ``bincount`` (whose output size is data-dependent);
* robot-side body reads are cached per sim epoch, like ``EntityData``.

The RNG stream differs from the reference (draws are taken for all envs).
"""

from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Literal

import torch

from mjlab_amd import envops
from mjlab_amd.managers.command_manager import CommandTerm
from mjlab_amd.managers.manager_term_config import CommandTermCfg
from mjlab_amd.motion import load_motion
from mjlab_amd.sim import native
from mjlab_amd.envops import quat_error_magnitude
from mjlab_amd.utils.math import quat_inv, yaw_quat

_AXES6 = ("x", "y", "z", "roll", "pitch", "yaw")


def _qmul(p: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
  """quat_mul over any leading dims (flattened to rows for the fused kernel)."""
  shape = torch.broadcast_shapes(p.shape, q.shape)
  out = envops.quat_mul(p.expand(shape).reshape(-1, 4), q.expand(shape).reshape(-1, 4))
  return out.view(shape)


def _qapply(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
  shape = torch.broadcast_shapes(q.shape[:-1], v.shape[:-1])
  out = envops.quat_apply(q.expand(*shape, 4).reshape(-1, 4), v.expand(*shape, 3).reshape(-1, 3))
  return out.view(*shape, 3)


class MotionLoader:
  """``commands.py:32-68``. Arrays of the npz written by ``mjlab_amd.motion``
  (format of ``scripts/csv_to_npz.py``), loaded with ``allow_pickle=False``.

  ``frame_table`` packs, per frame, [joint_pos | joint_vel | body_pos_w |
  body_quat_w | body_lin_vel_w | body_ang_vel_w] of the selected bodies."""

  def __init__(self, motion_file: str, body_indexes: torch.Tensor, device: str = "cpu") -> None:
    if not motion_file:
      raise ValueError("MotionCommandCfg.motion_file is empty: set it to a motion .npz (mjlab_amd.motion)")
    data = load_motion(motion_file)
    t = {k: torch.tensor(v, dtype=torch.float32, device=device) for k, v in data.items() if k != "fps"}
    self.fps = float(data["fps"][0])
    self.joint_pos = t["joint_pos"]
    self.joint_vel = t["joint_vel"]
    self._body_pos_w = t["body_pos_w"]
    self._body_quat_w = t["body_quat_w"]
    self._body_lin_vel_w = t["body_lin_vel_w"]
    self._body_ang_vel_w = t["body_ang_vel_w"]
    self._body_indexes = body_indexes
    self.time_step_total = self.joint_pos.shape[0]
    nb_all = self._body_pos_w.shape[1]
    if body_indexes.numel() and int(body_indexes.max()) >= nb_all:
      raise ValueError(f"motion has {nb_all} bodies, body index {int(body_indexes.max())} requested")
    T = self.time_step_total
    sel = [self.body_pos_w, self.body_quat_w, self.body_lin_vel_w, self.body_ang_vel_w]
    self.frame_table = torch.cat([self.joint_pos, self.joint_vel] + [s.reshape(T, -1) for s in sel], dim=1).contiguous()

  @property
  def body_pos_w(self) -> torch.Tensor:
    return self._body_pos_w[:, self._body_indexes]

  @property
  def body_quat_w(self) -> torch.Tensor:
    return self._body_quat_w[:, self._body_indexes]

  @property
  def body_lin_vel_w(self) -> torch.Tensor:
    return self._body_lin_vel_w[:, self._body_indexes]

  @property
  def body_ang_vel_w(self) -> torch.Tensor:
    return self._body_ang_vel_w[:, self._body_indexes]


class MotionCommand(CommandTerm):
  def __init__(self, cfg: "MotionCommandCfg", env) -> None:
    super().__init__(cfg, env)
    self.robot = env.scene[cfg.asset_name]
    self.robot_anchor_body_index = self.robot.body_names.index(cfg.anchor_body_name)
    self.motion_anchor_body_index = cfg.body_names.index(cfg.anchor_body_name)
    ids = self.robot.find_bodies(cfg.body_names, preserve_order=True)[0]
    self.body_indexes = torch.tensor(ids, dtype=torch.long, device=self.device)
    self.motion = MotionLoader(cfg.motion_file, self.body_indexes, device=self.device)
    n, nb, nj = self.num_envs, len(cfg.body_names), self.motion.joint_pos.shape[1]
    self._nb, self._nj = nb, nj
    self.time_steps = torch.zeros(n, dtype=torch.long, device=self.device)
    self.body_pos_relative_w = torch.zeros(n, nb, 3, device=self.device)
    self.body_quat_relative_w = torch.zeros(n, nb, 4, device=self.device)
    self.body_quat_relative_w[:, :, 0] = 1.0

    # current reference frame for every env: views into one (N, F) buffer
    self._frame = torch.zeros(n, self.motion.frame_table.shape[1], device=self.device)
    o = 0
    views = {}
    for name, w in (("joint_pos", nj), ("joint_vel", nj), ("body_pos", nb * 3), ("body_quat", nb * 4),
                    ("body_lin_vel", nb * 3), ("body_ang_vel", nb * 3)):
      views[name] = self._frame[:, o:o + w]
      o += w
    self._f_joint_pos, self._f_joint_vel = views["joint_pos"], views["joint_vel"]
    self._f_body_pos = views["body_pos"].view(n, nb, 3)  # motion frame, before env origins
    self._f_body_quat = views["body_quat"].view(n, nb, 4)
    self._f_body_lin_vel = views["body_lin_vel"].view(n, nb, 3)
    self._f_body_ang_vel = views["body_ang_vel"].view(n, nb, 3)
    self._body_pos_w = torch.zeros(n, nb, 3, device=self.device)  # + env origins
    self._origins = env.scene.env_origins
    self._refresh_frame()

    T = self.motion.time_step_total
    self.bin_count = int(T // (1 / env.step_dt)) + 1
    self.bin_failed_count = torch.zeros(self.bin_count, device=self.device)
    self._current_bin_failed = torch.zeros(self.bin_count, device=self.device)
    k = torch.tensor([cfg.adaptive_lambda**i for i in range(cfg.adaptive_kernel_size)], device=self.device)
    self.kernel = k / k.sum()
    # non-causal smoothing with replicate padding on the right: p_s[i] = sum_k w_k p[min(i+k, B-1)]
    ar = torch.arange(self.bin_count, device=self.device)
    self._smooth_idx = torch.clamp(ar[:, None] + torch.arange(cfg.adaptive_kernel_size, device=self.device)[None],
                                   max=self.bin_count - 1)

    def rng6(r):
      t = torch.tensor([r.get(a, (0.0, 0.0)) for a in _AXES6], dtype=torch.float32, device=self.device)
      return t[:, 0].clone(), t[:, 1].clone(), any(tuple(r.get(a, (0.0, 0.0))) != (0.0, 0.0) for a in _AXES6)

    self._pose_lo, self._pose_hi, self._pose_any = rng6(cfg.pose_range)
    self._vel_lo, self._vel_hi, self._vel_any = rng6(cfg.velocity_range)
    self._ranges_host = [[float(r.get(a, (0.0, 0.0))[i]) for a in _AXES6] for r in (cfg.pose_range, cfg.velocity_range)
                         for i in (0, 1)]

    for name in ("error_anchor_pos", "error_anchor_rot", "error_anchor_lin_vel", "error_anchor_ang_vel",
                 "error_body_pos", "error_body_rot", "error_body_lin_vel", "error_body_ang_vel",
                 "error_joint_pos", "error_joint_vel",
                 "sampling_entropy", "sampling_top1_prob", "sampling_top1_bin"):
      self.metrics[name] = torch.zeros(n, device=self.device)
    self._robot_cache_ep = None
    self._robot_cache: dict[str, torch.Tensor] = {}

  # ---- reference-frame reads (commands.py:134-181) ----
  @property
  def command(self) -> torch.Tensor:
    return self._frame[:, : 2 * self._nj]  # == cat([joint_pos, joint_vel], 1)

  joint_pos = property(lambda s: s._f_joint_pos)
  joint_vel = property(lambda s: s._f_joint_vel)
  body_pos_w = property(lambda s: s._body_pos_w)
  body_quat_w = property(lambda s: s._f_body_quat)
  body_lin_vel_w = property(lambda s: s._f_body_lin_vel)
  body_ang_vel_w = property(lambda s: s._f_body_ang_vel)
  anchor_pos_w = property(lambda s: s._body_pos_w[:, s.motion_anchor_body_index])
  anchor_quat_w = property(lambda s: s._f_body_quat[:, s.motion_anchor_body_index])
  anchor_lin_vel_w = property(lambda s: s._f_body_lin_vel[:, s.motion_anchor_body_index])
  anchor_ang_vel_w = property(lambda s: s._f_body_ang_vel[:, s.motion_anchor_body_index])

  def _refresh_frame(self) -> None:
    if self._frame.is_cuda and self._origins.stride(1) == 1:  # one launch (csrc/mjh_fuse.hip)
      P = envops._ptr
      native.check(native.lib().mjh_motion_frame(
        P(self.motion.frame_table), P(self.time_steps), P(self._frame), self._frame.shape[1], 2 * self._nj, self._nb,
        P(self._body_pos_w), P(self._origins), self._origins.stride(0), self.num_envs, envops._stream()), "mjh_motion_frame")
      return
    torch.index_select(self.motion.frame_table, 0, self.time_steps, out=self._frame)
    torch.add(self._f_body_pos, self._origins[:, None, :], out=self._body_pos_w)

  # ---- robot reads (commands.py:183-221), cached per sim epoch ----
  def _robot(self, key: str) -> torch.Tensor:
    ep = self._env.sim.epoch.v
    if ep != self._robot_cache_ep:
      self._robot_cache = {}
      self._robot_cache_ep = ep
    v = self._robot_cache.get(key)
    if v is None:
      d = self.robot.data
      if key == "pos":
        v = d.body_link_pos_w[:, self.body_indexes]
      elif key == "quat":
        v = d.body_link_quat_w[:, self.body_indexes]
      elif key == "lin":
        v = d.body_link_lin_vel_w[:, self.body_indexes]
      else:
        v = d.body_link_ang_vel_w[:, self.body_indexes]
      self._robot_cache[key] = v
    return v

  robot_joint_pos = property(lambda s: s.robot.data.joint_pos)
  robot_joint_vel = property(lambda s: s.robot.data.joint_vel)
  robot_body_pos_w = property(lambda s: s._robot("pos"))
  robot_body_quat_w = property(lambda s: s._robot("quat"))
  robot_body_lin_vel_w = property(lambda s: s._robot("lin"))
  robot_body_ang_vel_w = property(lambda s: s._robot("ang"))
  robot_anchor_pos_w = property(lambda s: s.robot.data.body_link_pos_w[:, s.robot_anchor_body_index])
  robot_anchor_quat_w = property(lambda s: s.robot.data.body_link_quat_w[:, s.robot_anchor_body_index])
  robot_anchor_lin_vel_w = property(lambda s: s.robot.data.body_link_lin_vel_w[:, s.robot_anchor_body_index])
  robot_anchor_ang_vel_w = property(lambda s: s.robot.data.body_link_ang_vel_w[:, s.robot_anchor_body_index])

  # ---- metrics (commands.py:223-256) ----
  def _update_metrics(self) -> None:
    m = self.metrics
    torch.norm(self.anchor_pos_w - self.robot_anchor_pos_w, dim=-1, out=m["error_anchor_pos"])
    m["error_anchor_rot"].copy_(quat_error_magnitude(self.anchor_quat_w, self.robot_anchor_quat_w))
    torch.norm(self.anchor_lin_vel_w - self.robot_anchor_lin_vel_w, dim=-1, out=m["error_anchor_lin_vel"])
    torch.norm(self.anchor_ang_vel_w - self.robot_anchor_ang_vel_w, dim=-1, out=m["error_anchor_ang_vel"])
    m["error_body_pos"].copy_(torch.norm(self.body_pos_relative_w - self.robot_body_pos_w, dim=-1).mean(dim=-1))
    m["error_body_rot"].copy_(quat_error_magnitude(self.body_quat_relative_w, self.robot_body_quat_w).mean(dim=-1))
    # the reference adds these two keys on the first update (commands.py:244-249);
    # here they are registered up front so every metric is a persistent buffer
    m["error_body_lin_vel"].copy_(torch.norm(self.body_lin_vel_w - self.robot_body_lin_vel_w, dim=-1).mean(dim=-1))
    m["error_body_ang_vel"].copy_(torch.norm(self.body_ang_vel_w - self.robot_body_ang_vel_w, dim=-1).mean(dim=-1))
    torch.norm(self.joint_pos - self.robot_joint_pos, dim=-1, out=m["error_joint_pos"])
    torch.norm(self.joint_vel - self.robot_joint_vel, dim=-1, out=m["error_joint_vel"])

  # ---- sampling (commands.py:258-307) ----
  def sampling_probabilities(self) -> torch.Tensor:
    p = self.bin_failed_count + self.cfg.adaptive_uniform_ratio / float(self.bin_count)
    p = (p[self._smooth_idx] * self.kernel[None]).sum(-1)
    return p / p.sum()

  def _adaptive_sampling_fused(self, mask: torch.Tensor) -> bool:
    if not (mask.is_cuda and mask.dtype == torch.bool and self.bin_count <= 4096):
      return False
    term = self._env.termination_manager.terminated
    P = envops._ptr
    seed, key, ctr = envops.rng_args(self._env, "motion_command.adaptive_sampling")
    m = self.metrics
    native.check(native.lib().mjh_motion_adaptive(
      P(mask), P(term), P(self.time_steps), P(self.bin_failed_count), P(self._current_bin_failed), P(self.kernel),
      self.bin_count, self.kernel.numel(), self.motion.time_step_total, float(self.cfg.adaptive_uniform_ratio),
      P(m["sampling_entropy"]), P(m["sampling_top1_prob"]), P(m["sampling_top1_bin"]), seed, key, ctr, self.num_envs,
      envops._stream()), "mjh_motion_adaptive")
    return True

  def _adaptive_sampling(self, mask: torch.Tensor) -> None:
    if self._adaptive_sampling_fused(mask):
      return
    T = self.motion.time_step_total
    failed = mask & self._env.termination_manager.terminated
    cur_bin = torch.clamp((self.time_steps * self.bin_count) // max(T, 1), 0, self.bin_count - 1)
    counts = torch.zeros_like(self._current_bin_failed).scatter_add_(0, cur_bin, failed.float())
    # reference overwrites the histogram only when some resampled env failed
    torch.where(failed.any(), counts, self._current_bin_failed, out=self._current_bin_failed)

    p = self.sampling_probabilities()
    cdf = torch.cumsum(p, 0)
    u = torch.rand(2, self.num_envs, device=self.device)
    bins = torch.searchsorted(cdf, (u[0] * cdf[-1]).contiguous(), right=True).clamp_(max=self.bin_count - 1)
    new = ((bins + u[1]) / self.bin_count * (T - 1)).long()
    torch.where(mask, new, self.time_steps, out=self.time_steps)

    # the reference updates the sampling metrics only when some env resampled
    H = -(p * (p + 1e-12).log()).sum()
    pmax, imax = p.max(dim=0)
    any_r = mask.any()
    for key, val in (("sampling_entropy", H / math.log(self.bin_count)), ("sampling_top1_prob", pmax),
                     ("sampling_top1_bin", imax.float() / self.bin_count)):
      mt = self.metrics[key]
      torch.where(any_r, val.expand(self.num_envs), mt, out=mt)

  def _uniform_sampling(self, mask: torch.Tensor) -> None:
    new = torch.randint(0, self.motion.time_step_total, (self.num_envs,), device=self.device)
    torch.where(mask, new, self.time_steps, out=self.time_steps)
    any_r = mask.any()
    for key, val in (("sampling_entropy", 1.0), ("sampling_top1_prob", 1.0 / self.bin_count), ("sampling_top1_bin", 0.5)):
      mt = self.metrics[key]
      torch.where(any_r, torch.full_like(mt, val), mt, out=mt)

  def _resample_command(self, mask: torch.Tensor) -> None:
    """commands.py:309-375 for the envs selected by ``mask``."""
    mode = self.cfg.sampling_mode
    if mode == "start":
      self.time_steps.masked_fill_(mask, 0)
    elif mode == "uniform":
      self._uniform_sampling(mask)
    elif mode == "adaptive":
      self._adaptive_sampling(mask)
    else:
      raise ValueError(f"unknown sampling_mode '{mode}'")
    self._refresh_frame()
    if self._write_state_fused(mask):
      return

    n = self.num_envs
    root_pos = self.body_pos_w[:, 0]
    root_ori = self.body_quat_w[:, 0]
    root_lin_vel = self.body_lin_vel_w[:, 0]
    root_ang_vel = self.body_ang_vel_w[:, 0]
    if self._pose_any:
      r = torch.rand(n, 6, device=self.device) * (self._pose_hi - self._pose_lo) + self._pose_lo
      root_pos = root_pos + r[:, 0:3]
      root_ori = envops.quat_mul(envops.quat_from_euler_xyz(r[:, 3:6]), root_ori)
    if self._vel_any:
      r = torch.rand(n, 6, device=self.device) * (self._vel_hi - self._vel_lo) + self._vel_lo
      root_lin_vel = root_lin_vel + r[:, 0:3]
      root_ang_vel = root_ang_vel + r[:, 3:6]

    lo, hi = self.cfg.joint_position_range
    joint_pos = self.joint_pos + (torch.rand(n, self._nj, device=self.device) * (hi - lo) + lo)
    lim = self.robot.data.soft_joint_pos_limits
    joint_pos = torch.clip(joint_pos, lim[:, :, 0], lim[:, :, 1])
    self.robot.write_joint_state_to_sim(joint_pos, self.joint_vel, env_ids=mask)
    self.robot.write_root_state_to_sim(torch.cat([root_pos, root_ori, root_lin_vel, root_ang_vel], dim=-1), env_ids=mask)
    self.robot.clear_state(env_ids=mask)

  def _write_state_fused(self, mask: torch.Tensor) -> bool:
    """The resampled envs' robot state (reference root +- pose/velocity offsets,
    joints + offsets clipped) written in one launch, plus clear_state."""
    d = self.robot.data
    c = d._cols
    keys = ("free_joint_q_adr", "free_joint_v_adr", "joint_q_adr", "joint_v_adr")
    if not (mask.is_cuda and mask.dtype == torch.bool and all(isinstance(c[k], slice) for k in keys)):
      return False
    lim = d.soft_joint_pos_limits
    qpos, qvel = d.data.qpos, d.data.qvel
    if not (lim.is_contiguous() and lim.shape[1] == self._nj and qpos.stride(1) == 1 and qvel.stride(1) == 1):
      return False
    nj, nb = self._nj, self._nb
    pos_off = 2 * nj
    F6 = ctypes.c_float * 6
    plo, phi, vlo, vhi = (F6(*r) for r in self._ranges_host)
    lo, hi = self.cfg.joint_position_range
    seed, key, ctr = envops.rng_args(self._env, "motion_command.resample_state")
    P = envops._ptr
    native.check(native.lib().mjh_motion_reset(
      P(self._frame), self._frame.stride(0), nj, pos_off, pos_off + 3 * nb, pos_off + 7 * nb, pos_off + 10 * nb,
      P(self._body_pos_w), self._body_pos_w.stride(0), P(mask), plo, phi, vlo, vhi, int(self._pose_any), int(self._vel_any),
      float(lo), float(hi), P(lim), lim.stride(0), P(qpos), qpos.stride(0), c["free_joint_q_adr"].start, c["joint_q_adr"].start,
      P(qvel), qvel.stride(0), c["free_joint_v_adr"].start, c["joint_v_adr"].start, seed, key, ctr, self.num_envs,
      envops._stream()), "mjh_motion_reset")
    self.robot.clear_state(env_ids=mask)
    return True

  # ---- per-step update (commands.py:377-412) ----
  def _update_command(self) -> None:
    self.time_steps += 1
    self._resample_command(self.time_steps >= self.motion.time_step_total)  # refreshes the frame

    anchor_pos = self.anchor_pos_w
    robot_anchor_pos = self.robot_anchor_pos_w
    if envops.motion_relative(anchor_pos, self.anchor_quat_w, robot_anchor_pos, self.robot_anchor_quat_w, self.body_pos_w,
                              self.body_quat_w, self.body_pos_relative_w, self.body_quat_relative_w):
      self._adaptive_update()
      return
    delta_pos = torch.cat([robot_anchor_pos[:, 0:2], anchor_pos[:, 2:3]], dim=-1)
    delta_ori = yaw_quat(envops.quat_mul(self.robot_anchor_quat_w, quat_inv(self.anchor_quat_w)))
    self.body_quat_relative_w.copy_(_qmul(delta_ori[:, None, :], self.body_quat_w))
    self.body_pos_relative_w.copy_(delta_pos[:, None, :] + _qapply(delta_ori[:, None, :], self.body_pos_w - anchor_pos[:, None, :]))

    self._adaptive_update()

  def _adaptive_update(self) -> None:
    if self.cfg.sampling_mode == "adaptive":
      a = self.cfg.adaptive_alpha
      self.bin_failed_count.mul_(1 - a).add_(a * self._current_bin_failed)
      self._current_bin_failed.zero_()


@dataclass(kw_only=True)
class MotionCommandCfg(CommandTermCfg):
  motion_file: str
  anchor_body_name: str
  body_names: tuple[str, ...]
  asset_name: str
  class_type: type = MotionCommand
  pose_range: dict[str, tuple[float, float]] = field(default_factory=dict)
  velocity_range: dict[str, tuple[float, float]] = field(default_factory=dict)
  joint_position_range: tuple[float, float] = (-0.52, 0.52)
  adaptive_kernel_size: int = 1
  adaptive_lambda: float = 0.8
  adaptive_uniform_ratio: float = 0.1
  adaptive_alpha: float = 0.001
  sampling_mode: Literal["adaptive", "uniform", "start"] = "adaptive"
