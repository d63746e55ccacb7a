"""Uniform velocity command (``src/mjlab/tasks/velocity/mdp/velocity_command.py:22-123``).

Mask-based and capturable: resampling draws for all envs and selects with the
mask; ``ranges`` are mirrored into a device tensor (``sync_ranges``, called by
the env on the host before each step) so curricula that edit
``cfg.ranges`` take effect without re-capturing the step graph.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import torch

from mjlab_amd.managers.command_manager import CommandTerm
from mjlab_amd.managers.manager_term_config import CommandTermCfg
from mjlab_amd.envops import quat_apply
from mjlab_amd.utils.math import wrap_to_pi


class UniformVelocityCommand(CommandTerm):
  def __init__(self, cfg: "UniformVelocityCommandCfg", env) -> None:
    super().__init__(cfg, env)
    if cfg.heading_command and cfg.ranges.heading is None:
      raise ValueError("heading_command=True but ranges.heading is set to None.")
    if cfg.ranges.heading and not cfg.heading_command:
      raise ValueError("ranges.heading is set but heading_command=False.")
    self.robot = env.scene[cfg.asset_name]
    n = self.num_envs
    self.vel_command_b = torch.zeros(n, 3, device=self.device)
    self.heading_target = torch.zeros(n, device=self.device)
    self.heading_error = torch.zeros(n, device=self.device)
    self.is_heading_env = torch.zeros(n, dtype=torch.bool, device=self.device)
    self.is_standing_env = torch.zeros_like(self.is_heading_env)
    self.metrics["error_vel_xy"] = torch.zeros(n, device=self.device)
    self.metrics["error_vel_yaw"] = torch.zeros(n, device=self.device)
    self._ranges_t = torch.zeros(4, 2, device=self.device)
    self._ranges_host = None
    self.sync_ranges()

  @property
  def command(self) -> torch.Tensor:
    return self.vel_command_b

  def sync_ranges(self) -> None:
    r = self.cfg.ranges
    host = (tuple(r.lin_vel_x), tuple(r.lin_vel_y), tuple(r.ang_vel_z), tuple(r.heading) if r.heading else (0.0, 0.0))
    if host != self._ranges_host:
      self._ranges_t.copy_(torch.tensor(host, dtype=torch.float32))
      self._ranges_host = host

  def _draw(self) -> torch.Tensor:
    """(N, 4) uniform draws over [lin_vel_x, lin_vel_y, ang_vel_z, heading] ranges."""
    lo, hi = self._ranges_t[:, 0], self._ranges_t[:, 1]
    return torch.rand(self.num_envs, 4, device=self.device) * (hi - lo) + lo

  def compute(self, dt: float) -> None:
    """CommandTerm.compute (command_manager.py:53-67) with one (N, 8) uniform
    draw per step: [timer, lin_x, lin_y, ang_z, heading, heading-env,
    standing-env, init-velocity]. On the GPU the whole update is one fused
    kernel (csrc/mjh_mdp.hip); the torch path below is its reference."""
    if self.cfg.init_velocity_prob == 0.0 and self._compute_fused(dt, None):
      return  # draws from the env's device stream inside the kernel
    u = torch.rand(self.num_envs, 8, device=self.device)
    self._compute_torch(dt, u)

  def _compute_fused(self, dt: float, u: torch.Tensor | None) -> bool:
    if not self.vel_command_b.is_cuda:
      return False
    import ctypes

    from mjlab_amd.sim import native

    d = self.robot.data
    lin, ang, q = d.root_link_lin_vel_b, d.root_link_ang_vel_b, d.root_link_quat_w
    if not all(t.dim() == 2 and t.stride(1) == 1 for t in (lin, ang, q)):
      return False
    from mjlab_amd import envops

    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    lo, hi = self.cfg.resampling_time_range
    max_step = self.cfg.resampling_time_range[1] / self._env.step_dt
    seed, key, ctr = envops.rng_args(self._env, "velocity_command.compute") if u is None else (
      ctypes.c_ulonglong(0), ctypes.c_ulonglong(0), None)
    envops._keep(lin, ang, q, u)
    native.check(native.lib().mjh_velocity_command(
      P(lin), lin.stride(0), P(ang), ang.stride(0), P(q), q.stride(0), P(u) if u is not None else None,
      u.stride(0) if u is not None else 0, P(self._ranges_t),
      float(dt), 1.0 / max_step, float(lo), float(hi), float(self.cfg.rel_heading_envs), float(self.cfg.rel_standing_envs),
      float(self.cfg.heading_control_stiffness), int(self.cfg.heading_command), P(self.vel_command_b),
      P(self.heading_target), P(self.heading_error), P(self.is_heading_env), P(self.is_standing_env), P(self.time_left),
      P(self.command_counter), P(self.metrics["error_vel_xy"]), P(self.metrics["error_vel_yaw"]), seed, key, ctr, self.num_envs,
      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "mjh_velocity_command")
    return True

  def _compute_torch(self, dt: float, u: torch.Tensor) -> None:
    self._update_metrics()
    self.time_left -= dt
    mask = self.time_left <= 0.0
    lo, hi = self.cfg.resampling_time_range
    torch.where(mask, u[:, 0] * (hi - lo) + lo, self.time_left, out=self.time_left)
    r = self._ranges_t
    new = u[:, 1:5] * (r[:, 1] - r[:, 0]) + r[:, 0]
    torch.where(mask[:, None], new[:, :3], self.vel_command_b, out=self.vel_command_b)
    if self.cfg.heading_command:
      torch.where(mask, new[:, 3], self.heading_target, out=self.heading_target)
      torch.where(mask, u[:, 5] <= self.cfg.rel_heading_envs, self.is_heading_env, out=self.is_heading_env)
    torch.where(mask, u[:, 6] <= self.cfg.rel_standing_envs, self.is_standing_env, out=self.is_standing_env)
    if self.cfg.init_velocity_prob > 0.0:
      self._init_velocity(mask & (u[:, 7] < self.cfg.init_velocity_prob))
    self.command_counter += mask.long()
    self._update_command()

  def _resample_fused(self, mask: torch.Tensor, reset: bool) -> bool:
    """CommandTerm._resample (+ the counter restart of reset) in one launch
    (csrc/mjh_fuse.hip), draws from the env's device stream."""
    if self.cfg.init_velocity_prob != 0.0 or not self.vel_command_b.is_cuda or mask.dtype != torch.bool:
      return False
    import ctypes

    from mjlab_amd import envops
    from mjlab_amd.sim import native

    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    lo, hi = self.cfg.resampling_time_range
    seed, key, ctr = envops.rng_args(self._env, "velocity_command.resample")
    envops._keep(mask)
    native.check(native.lib().mjh_velocity_resample(
      P(mask), P(self._ranges_t), float(lo), float(hi), float(self.cfg.rel_heading_envs), float(self.cfg.rel_standing_envs),
      int(self.cfg.heading_command), int(reset), P(self.vel_command_b), P(self.heading_target), P(self.is_heading_env),
      P(self.is_standing_env), P(self.time_left), P(self.command_counter), seed, key, ctr, self.num_envs,
      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "mjh_velocity_resample")
    return True

  def _reset_resample(self, mask: torch.Tensor) -> bool:
    return self._resample_fused(mask, reset=True)

  def _update_metrics(self) -> None:
    max_command_step = self.cfg.resampling_time_range[1] / self._env.step_dt
    d = self.robot.data
    self.metrics["error_vel_xy"] += torch.norm(self.vel_command_b[:, :2] - d.root_link_lin_vel_b[:, :2], dim=-1) / max_command_step
    self.metrics["error_vel_yaw"] += torch.abs(self.vel_command_b[:, 2] - d.root_link_ang_vel_b[:, 2]) / max_command_step

  def _resample_command(self, mask: torch.Tensor) -> None:
    new = self._draw()
    torch.where(mask[:, None], new[:, :3], self.vel_command_b, out=self.vel_command_b)
    u = torch.rand(self.num_envs, 2, device=self.device)
    if self.cfg.heading_command:
      torch.where(mask, new[:, 3], self.heading_target, out=self.heading_target)
      torch.where(mask, u[:, 0] <= self.cfg.rel_heading_envs, self.is_heading_env, out=self.is_heading_env)
    torch.where(mask, u[:, 1] <= self.cfg.rel_standing_envs, self.is_standing_env, out=self.is_standing_env)
    if self.cfg.init_velocity_prob > 0.0:
      self._init_velocity(mask & (torch.rand(self.num_envs, device=self.device) < self.cfg.init_velocity_prob))

  def _init_velocity(self, iv: torch.Tensor) -> None:
    """Start the selected envs moving at their command (velocity_command.py:80-89)."""
    d = self.robot.data
    lin_b = d.root_link_lin_vel_b.clone()
    lin_b[:, :2] = self.vel_command_b[:, :2]
    ang_b = d.root_link_ang_vel_b.clone()
    ang_b[:, 2] = self.vel_command_b[:, 2]
    state = torch.cat([d.root_link_pos_w, d.root_link_quat_w, quat_apply(d.root_link_quat_w, lin_b), ang_b], dim=-1)
    self.robot.write_root_state_to_sim(state, iv)

  def _update_command(self) -> None:
    if self.cfg.heading_command:
      self.heading_error.copy_(wrap_to_pi(self.heading_target - self.robot.data.heading_w))
      yaw = torch.clamp(self.cfg.heading_control_stiffness * self.heading_error, self._ranges_t[2, 0], self._ranges_t[2, 1])
      self.vel_command_b[:, 2] = torch.where(self.is_heading_env, yaw, self.vel_command_b[:, 2])
    self.vel_command_b.masked_fill_(self.is_standing_env[:, None], 0.0)


@dataclass(kw_only=True)
class UniformVelocityCommandCfg(CommandTermCfg):
  asset_name: str
  heading_command: bool = False
  heading_control_stiffness: float = 1.0
  rel_standing_envs: float = 0.0
  rel_heading_envs: float = 1.0
  init_velocity_prob: float = 0.0
  class_type: type = UniformVelocityCommand

  @dataclass
  class Ranges:
    lin_vel_x: tuple[float, float]
    lin_vel_y: tuple[float, float]
    ang_vel_z: tuple[float, float]
    heading: tuple[float, float] | None = None

  ranges: Ranges

  @dataclass
  class VizCfg:
    z_offset: float = 0.2
    scale: float = 0.5

  viz: VizCfg = field(default_factory=VizCfg)

  def __post_init__(self):
    if self.heading_command and self.ranges.heading is None:
      raise ValueError(
        "The velocity command has heading commands active (heading_command=True) but "
        "the `ranges.heading` parameter is set to None."
      )
