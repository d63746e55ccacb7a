"""Reset/event/command golden vectors from the reference's own functions (run HERE only).

The reference's reset, push and resampling functions are executed unmodified
(stub recipe of tools/make_golden.py) with their random draws INJECTED: the
draws are exactly the U[0, 1) elements the fused HIP kernels consume from the
env's device stream (tests/rng_np.py restates csrc/mjh_rng.h; the element
layout of each kernel is cited below). The GPU test
(tests/test_gpu_golden_events.py) builds the mjlab_amd env, loads the fixture's
inputs into it, calls the same term through the product path (which launches
the mjh_fuse.hip kernel) with the fixture's (seed, step, call counter), and
compares with the reference's outputs.

Covered (reference file:line -> kernel):
  reset_root_state_uniform   envs/mdp/events.py:45-132      reset_root_uniform_kernel (u[e*12 + j])
  reset_joints_by_offset     envs/mdp/events.py:135-170     reset_joints_offset_kernel (u[e*2k + j])
  push_by_setting_velocity   envs/mdp/events.py:173-187     push_velocity_kernel (u[e*6 + j])
  randomize_field            envs/mdp/events.py:256-309     (host torch; draws injected via torch.rand)
  CommandTerm._resample +    managers/command_manager.py:63-69,
  UniformVelocityCommand._resample_command  velocity_command.py:65-89   velocity_resample_kernel (u[e*8 + j])
  MotionCommand._adaptive_sampling / _resample_command
                             tracking/mdp/commands.py:258-375  motion_adaptive_kernel (u[2e], u[2e+1]),
                                                               motion_reset_kernel (u[e*(12+nj) + j])
Writes go through the reference's EntityData (entity/data.py:75-198) over
stand-in state tensors. ``torch.multinomial`` (adaptive sampling) is replaced
by inverse-CDF sampling of the same probabilities with the injected draw
(the kernel's sampler); every deterministic quantity around it (failed-bin
histogram, smoothed probabilities, entropy/top-1 metrics, the time-step
formula) is the reference's.
Output: tests/golden/events_g1.npz (data only). Re-running reproduces it byte for byte.
"""

from __future__ import annotations

import io
import json
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT))

import make_golden  # noqa: E402
from tests import rng_np  # noqa: E402

OUT = ROOT / "tests" / "golden" / "events_g1.npz"
N = 16
NJ = 29
SEED = 0x5EED1234
STEP = 7
MOTION_T = 300


def _draws(site: str, salt: int, idx) -> torch.Tensor:
  return torch.from_numpy(rng_np.u01(SEED, rng_np.site_key(site, salt), STEP, idx))


def _ref_entity_data(qpos, qvel, default_root_state, default_joint_pos, default_joint_vel, soft_limits):
  """The reference EntityData over stand-in state tensors (G1 layout: free joint
  q 0..6 / v 0..5, then the NJ hinge joints)."""
  from mjlab.entity.data import EntityData

  idx = SimpleNamespace(free_joint_q_adr=torch.arange(7), free_joint_v_adr=torch.arange(6),
                        joint_q_adr=torch.arange(7, 7 + NJ), joint_v_adr=torch.arange(6, 6 + NJ),
                        body_ids=torch.arange(1, 2), ctrl_ids=torch.arange(NJ), root_body_id=1, mocap_id=None)
  data = SimpleNamespace(qpos=qpos, qvel=qvel, ctrl=torch.zeros(N, NJ), qfrc_applied=torch.zeros(N, 6 + NJ),
                         xfrc_applied=torch.zeros(N, 2, 6))
  ed = EntityData(indexing=idx, data=data, model=None, device="cpu", default_root_state=default_root_state,
                  default_joint_pos=default_joint_pos, default_joint_vel=default_joint_vel,
                  default_joint_stiffness=torch.zeros(N, NJ), default_joint_damping=torch.zeros(N, NJ),
                  default_joint_pos_limits=soft_limits.clone(), joint_pos_limits=soft_limits.clone(),
                  soft_joint_pos_limits=soft_limits, gravity_vec_w=torch.tensor([0.0, 0.0, -1.0]).repeat(N, 1),
                  forward_vec_b=torch.tensor([1.0, 0.0, 0.0]).repeat(N, 1), is_fixed_base=False, is_articulated=True,
                  is_actuated=True)
  return ed


class _Asset:
  """Entity write API (entity.py:428-599 delegate to EntityData)."""

  is_fixed_base = False
  is_mocap = False

  def __init__(self, ed, vel_w=None):
    self.data = ed
    self._vel_w = vel_w

  def write_root_state_to_sim(self, s, env_ids=None):
    self.data.write_root_state(s, env_ids)

  def write_root_link_pose_to_sim(self, p, env_ids=None):
    self.data.write_root_pose(p, env_ids)

  def write_root_link_velocity_to_sim(self, v, env_ids=None):
    self.data.write_root_velocity(v, env_ids)

  def write_joint_state_to_sim(self, p, v, joint_ids=None, env_ids=None):
    self.data.write_joint_state(p, v, joint_ids, env_ids)

  def clear_state(self, env_ids=None):
    self.data.clear_state(env_ids)


def _state(g: torch.Generator):
  q = torch.randn(N, 4, generator=g)
  q = q / q.norm(dim=-1, keepdim=True)
  qpos = torch.cat([torch.randn(N, 3, generator=g), q, 0.3 * torch.randn(N, NJ, generator=g)], 1)
  qvel = torch.randn(N, 6 + NJ, generator=g)
  rq = torch.randn(N, 4, generator=g)
  rq = rq / rq.norm(dim=-1, keepdim=True)
  drs = torch.cat([0.2 * torch.randn(N, 2, generator=g), 0.76 + 0.01 * torch.randn(N, 1, generator=g), rq,
                   0.1 * torch.randn(N, 6, generator=g)], 1)
  djp = 0.4 * torch.randn(N, NJ, generator=g)
  djv = 0.1 * torch.randn(N, NJ, generator=g)
  mid = djp + 0.1 * torch.randn(N, NJ, generator=g)
  half = 0.2 + torch.rand(N, NJ, generator=g)
  lim = torch.stack([mid - half, mid + half], -1)
  org = 2.0 * torch.randn(N, 3, generator=g)
  org[:, 2] = 0.0
  mask = torch.rand(N, generator=g) < 0.5
  mask[0], mask[1] = True, False
  return qpos, qvel, drs, djp, djv, lim, org, mask


def gen_events(out: dict, g: torch.Generator) -> None:
  from mjlab.envs.mdp import events as ref_events
  from mjlab.managers.scene_entity_config import SceneEntityCfg
  from mjlab.tasks.velocity.config.g1.env_cfgs import UNITREE_G1_FLAT_ENV_CFG as CFG

  qpos, qvel, drs, djp, djv, lim, org, mask = _state(g)
  ids = mask.nonzero().flatten()
  out.update(in_qpos=qpos, in_qvel=qvel, in_default_root_state=drs, in_default_joint_pos=djp, in_default_joint_vel=djv,
             in_soft_joint_pos_limits=lim, in_env_origins=org, in_mask=mask)
  queue: list[torch.Tensor] = []

  def sample_uniform(lower, upper, size, device=None):  # isaaclab math.py:1360-1378 with the draws injected
    u = queue.pop(0)
    assert tuple(u.shape) == tuple(size if not isinstance(size, int) else (size,)), (u.shape, size)
    return u * (upper - lower) + lower

  ref_events.sample_uniform = sample_uniform
  cases = {
    "root_cfg": ("reset_root_state_uniform.robot", CFG.events["reset_base"].params["pose_range"],
                 CFG.events["reset_base"].params["velocity_range"]),
    "root_all": ("reset_root_state_uniform.robot",
                 {"x": (-0.5, 0.5), "y": (-0.4, 0.6), "z": (-0.05, 0.1), "roll": (-0.3, 0.2), "pitch": (-0.25, 0.3),
                  "yaw": (-3.14, 3.14)},
                 {"x": (-0.5, 0.5), "y": (-0.5, 0.4), "z": (-0.2, 0.2), "roll": (-0.6, 0.5), "pitch": (-0.4, 0.7),
                  "yaw": (-1.0, 1.2)}),
  }
  for name, (site, pr, vr) in cases.items():
    ed = _ref_entity_data(qpos.clone(), qvel.clone(), drs, djp, djv, lim)
    env = SimpleNamespace(num_envs=N, device="cpu", scene=_Scene(robot=_Asset(ed), env_origins=org))
    e = ids.numpy()
    j = np.arange(6)
    queue[:] = [_draws(site, 1, e[:, None] * 12 + j), _draws(site, 1, e[:, None] * 12 + 6 + j)]
    ref_events.reset_root_state_uniform(env, ids, pr, vr, SceneEntityCfg("robot"))
    assert not queue
    out[f"{name}_pose_range"] = np.array([pr.get(k, (0.0, 0.0)) for k in ("x", "y", "z", "roll", "pitch", "yaw")])
    out[f"{name}_velocity_range"] = np.array([(vr or {}).get(k, (0.0, 0.0)) for k in ("x", "y", "z", "roll", "pitch", "yaw")])
    out[f"{name}_qpos"], out[f"{name}_qvel"] = ed.data.qpos, ed.data.qvel

  jcases = {"joints_cfg": (CFG.events["reset_robot_joints"].params["position_range"],
                           CFG.events["reset_robot_joints"].params["velocity_range"]),
            "joints_all": ((-0.35, 0.45), (-0.6, 0.5))}
  site = "reset_joints_by_offset.robot"
  for name, (prange, vrange) in jcases.items():
    ed = _ref_entity_data(qpos.clone(), qvel.clone(), drs, djp, djv, lim)
    env = SimpleNamespace(num_envs=N, device="cpu", scene=_Scene(robot=_Asset(ed), env_origins=org))
    e = ids.numpy()[:, None]
    j = np.arange(NJ)
    queue[:] = [_draws(site, 1, e * 2 * NJ + j), _draws(site, 1, e * 2 * NJ + NJ + j)]
    ref_events.reset_joints_by_offset(env, ids, prange, vrange, SceneEntityCfg("robot", joint_ids=slice(None)))
    assert not queue
    out[f"{name}_ranges"] = np.array([prange, vrange], dtype=np.float64)
    out[f"{name}_qpos"], out[f"{name}_qvel"] = ed.data.qpos, ed.data.qvel

  # push: root_link_vel_w is an input (the GPU test makes it the env's read)
  vel_w = torch.randn(N, 6, generator=g)
  out["in_root_link_vel_w"] = vel_w
  site = "push_by_setting_velocity.robot"
  for name, vr in (("push_cfg", CFG.events["push_robot"].params["velocity_range"]),
                   ("push_all", {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "z": (-0.3, 0.1), "roll": (-0.4, 0.4),
                                 "pitch": (-0.2, 0.5), "yaw": (-0.7, 0.6)})):
    ed = _ref_entity_data(qpos.clone(), qvel.clone(), drs, djp, djv, lim)
    ed.__class__ = type("EDv", (ed.__class__,), {"root_link_vel_w": property(lambda s: vel_w.clone())})
    env = SimpleNamespace(num_envs=N, device="cpu", scene=_Scene(robot=_Asset(ed), env_origins=org))
    e = ids.numpy()[:, None]
    queue[:] = [_draws(site, 1, e * 6 + np.arange(6))]
    ref_events.push_by_setting_velocity(env, ids, vr, SceneEntityCfg("robot"))
    assert not queue
    out[f"{name}_velocity_range"] = np.array([vr.get(k, (0.0, 0.0)) for k in ("x", "y", "z", "roll", "pitch", "yaw")])
    out[f"{name}_qvel"] = ed.data.qvel


class _Scene(dict):
  def __init__(self, env_origins, **kw):
    super().__init__(**kw)
    self.env_origins = env_origins


RF_CASES = (  # (field, per-world shape, ranges, operation, axes, entity ids kind, ids)
  ("geom_friction", (12, 3), (0.3, 1.2), "abs", [0], "geom_ids", [2, 5, 7, 11]),
  ("body_mass", (9,), (0.8, 1.2), "scale", None, "body_ids", [1, 2, 3, 4, 5, 6, 7, 8]),
  ("dof_damping", (10,), (0.1, 0.5), "add", None, "joint_ids", [0, 2, 3]),
  ("body_ipos", (9, 3), {0: (-0.01, 0.01), 2: (-0.02, 0.03)}, "add", None, "body_ids", [3, 4]),
)


def gen_randomize_field(out: dict, g: torch.Generator) -> None:
  """randomize_field (events.py:256-309) on per-world fields; draws injected."""
  from mjlab.envs.mdp import events as ref_events
  from mjlab.managers.scene_entity_config import SceneEntityCfg

  mask = torch.rand(N, generator=g) < 0.6
  ids = mask.nonzero().flatten().int()
  out["rf_mask"] = mask
  I = lambda *a: torch.arange(*a, dtype=torch.int)  # noqa: E731  (EntityIndexing holds int32, entity.py:632-660)
  indexing = SimpleNamespace(geom_ids=I(12), body_ids=I(1, 9), joint_v_adr=I(6, 10), joint_q_adr=I(7, 11), joint_ids=I(1, 5))
  queue: list[torch.Tensor] = []

  def sample_uniform(lower, upper, size, device=None):
    u = torch.rand(size, generator=g)
    queue.append(u)
    return u * (upper - lower) + lower

  ref_events.sample_uniform = sample_uniform
  for i, (field, shp, ranges, op, axes, kind, sel) in enumerate(RF_CASES):
    fld = torch.rand(N, *shp, generator=g) + 0.5
    out[f"rf{i}_in"] = fld.clone()
    asset = SimpleNamespace(indexing=indexing)
    model = SimpleNamespace(**{field: fld})
    env = SimpleNamespace(num_envs=N, device="cpu", scene={"robot": asset}, sim=SimpleNamespace(model=model))
    key = {"geom_ids": "geom_ids", "body_ids": "body_ids", "joint_ids": "joint_ids"}[kind]
    sel_local = [int(x) for x in sel] if kind != "body_ids" else [int(x) - 1 for x in sel]
    queue.clear()
    ref_events.randomize_field(env, ids, field, ranges, "uniform", op, SceneEntityCfg("robot", **{key: sel_local}), axes)
    out[f"rf{i}_draws"] = torch.cat([u.reshape(-1) for u in queue])
    out[f"rf{i}_out"] = fld
    out[f"rf{i}_meta"] = np.array(json.dumps({"field": field, "ranges": ranges if isinstance(ranges, tuple) else
                                              {str(k): v for k, v in ranges.items()}, "operation": op, "axes": axes,
                                              "kind": kind, "ids": sel_local}))
  out["rf_indexing"] = np.array(json.dumps({k: getattr(indexing, k).tolist() for k in vars(indexing)}))


def gen_velocity_command(out: dict, g: torch.Generator) -> None:
  from mjlab.tasks.velocity.config.g1.env_cfgs import UNITREE_G1_FLAT_ENV_CFG as CFG
  from mjlab.tasks.velocity.mdp.velocity_command import UniformVelocityCommand

  cfg = CFG.commands["twist"]
  assert cfg.init_velocity_prob == 0.0
  mask = torch.rand(N, generator=g) < 0.6
  ids = mask.nonzero().flatten()
  cmd = UniformVelocityCommand.__new__(UniformVelocityCommand)
  cmd.cfg = cfg
  cmd._env = SimpleNamespace(num_envs=N, device="cpu")
  cmd.vel_command_b = torch.randn(N, 3, generator=g)
  cmd.heading_target = torch.randn(N, generator=g)
  cmd.is_heading_env = torch.rand(N, generator=g) < 0.5
  cmd.is_standing_env = torch.rand(N, generator=g) < 0.5
  cmd.time_left = torch.rand(N, generator=g) * 5
  cmd.command_counter = torch.randint(0, 9, (N,), generator=g)
  out.update({"vc_in_" + k: getattr(cmd, k).clone() for k in ("vel_command_b", "heading_target", "is_heading_env",
                                                                 "is_standing_env", "time_left", "command_counter")})
  out["vc_mask"] = mask
  out["vc_cfg"] = np.array([*cfg.resampling_time_range, cfg.rel_heading_envs, cfg.rel_standing_envs,
                            *cfg.ranges.lin_vel_x, *cfg.ranges.lin_vel_y, *cfg.ranges.ang_vel_z, *cfg.ranges.heading])
  site = "velocity_command.resample"
  e = ids.numpy()
  draws = [_draws(site, 1, e * 8 + j) for j in range(8)]  # time, lin x/y, ang z, heading, is_heading, is_standing, init_vel
  real = torch.Tensor.uniform_

  def uniform_(self, a=0.0, b=1.0):
    return self.copy_(draws.pop(0) * (b - a) + a)

  torch.Tensor.uniform_ = uniform_
  try:
    cmd._resample(ids)  # command_manager.py:63-69 -> velocity_command.py:65-89
  finally:
    torch.Tensor.uniform_ = real
  assert not draws
  out.update({"vc_out_" + k: getattr(cmd, k).clone() for k in ("vel_command_b", "heading_target", "is_heading_env",
                                                                  "is_standing_env", "time_left", "command_counter")})


def gen_motion(out: dict, g: torch.Generator) -> None:
  import mjlab.tasks.tracking.mdp.commands as ref_cmds
  from mjlab.tasks.tracking.config.g1.env_cfgs import G1_FLAT_TRACKING_ENV_CFG as CFG

  sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
  from mjlab_amd.asset_zoo.g1 import get_g1_robot_cfg
  from mjlab_amd.entity import Entity

  body_names = list(Entity(get_g1_robot_cfg()).body_names)  # G1 body order (data, from the MJCF)
  nb = len(body_names)
  cfg = CFG.commands["motion"]
  # synthetic clip in the csv_to_npz.py format (inputs)
  T = MOTION_T
  quat = torch.randn(T, nb, 4, generator=g)
  quat = quat / quat.norm(dim=-1, keepdim=True)
  clip = {"fps": np.array([50.0]), "joint_pos": 0.5 * torch.randn(T, NJ, generator=g), "joint_vel": torch.randn(T, NJ, generator=g),
          "body_pos_w": torch.randn(T, nb, 3, generator=g), "body_quat_w": quat,
          "body_lin_vel_w": torch.randn(T, nb, 3, generator=g), "body_ang_vel_w": torch.randn(T, nb, 3, generator=g)}
  buf = io.BytesIO()
  np.savez(buf, **{k: np.asarray(v, dtype=np.float32) if k != "fps" else v for k, v in clip.items()})
  buf.seek(0)
  body_indexes = torch.tensor([body_names.index(b) for b in cfg.body_names], dtype=torch.long)
  motion = ref_cmds.MotionLoader(buf, body_indexes)
  step_dt = 0.02
  qpos, qvel, drs, djp, djv, lim, org, _ = _state(g)
  mask = torch.rand(N, generator=g) < 0.5
  mask[0] = True
  terminated = torch.rand(N, generator=g) < 0.5
  terminated[0] = True
  ids = mask.nonzero().flatten()
  ed = _ref_entity_data(qpos.clone(), qvel.clone(), drs, djp, djv, lim)

  cmd = ref_cmds.MotionCommand.__new__(ref_cmds.MotionCommand)
  cmd.cfg = cfg
  cmd._env = SimpleNamespace(termination_manager=SimpleNamespace(terminated=terminated),
                             scene=_Scene(robot=_Asset(ed), env_origins=org), step_dt=step_dt, num_envs=N,
                             device="cpu")
  cmd.robot = _Asset(ed)
  cmd.motion = motion
  cmd.time_steps = torch.randint(0, T, (N,), generator=g)
  cmd.bin_count = int(motion.time_step_total // (1 / step_dt)) + 1  # commands.py:100
  cmd.bin_failed_count = torch.rand(cmd.bin_count, generator=g) * 0.3
  cmd._current_bin_failed = torch.rand(cmd.bin_count, generator=g)
  k = torch.tensor([cfg.adaptive_lambda**i for i in range(cfg.adaptive_kernel_size)])
  cmd.kernel = k / k.sum()
  cmd.metrics = {m: torch.zeros(N) for m in ("sampling_entropy", "sampling_top1_prob", "sampling_top1_bin")}
  out.update(mo_in_time_steps=cmd.time_steps.clone(), mo_in_bin_failed_count=cmd.bin_failed_count.clone(),
             mo_in_current_bin_failed=cmd._current_bin_failed.clone(), mo_mask=mask, mo_terminated=terminated,
             mo_in_qpos=qpos, mo_in_qvel=qvel, mo_in_soft_joint_pos_limits=lim, mo_in_env_origins=org,
             mo_body_names=np.array(body_names))
  out.update({"mo_clip_" + k: np.asarray(v) for k, v in clip.items()})
  out["mo_cfg"] = np.array([cfg.adaptive_kernel_size, cfg.adaptive_lambda, cfg.adaptive_uniform_ratio, *cfg.joint_position_range])

  e = ids.numpy()
  s1, s2 = "motion_command.adaptive_sampling", "motion_command.resample_state"
  u_bin, u_frac = _draws(s1, 1, 2 * e), _draws(s1, 1, 2 * e + 1)
  S = 12 + NJ
  queue = [u_frac, _draws(s2, 2, e[:, None] * S + np.arange(6)), _draws(s2, 2, e[:, None] * S + 6 + np.arange(6)),
           _draws(s2, 2, np.arange(N)[:, None] * S + 12 + np.arange(NJ))]

  def sample_uniform(lower, upper, size, device=None):
    u = queue.pop(0)
    assert tuple(u.shape) == tuple(size if not isinstance(size, int) else (size,)), (u.shape, size)
    return u * (upper - lower) + lower

  def multinomial(p, num, replacement=False):  # inverse CDF with the injected draw (the kernel's sampler)
    cdf = torch.cumsum(p, 0)
    return torch.searchsorted(cdf, (u_bin * cdf[-1]).contiguous(), right=True).clamp_(max=p.numel() - 1)

  real_su, real_mn = ref_cmds.sample_uniform, torch.multinomial
  ref_cmds.sample_uniform, torch.multinomial = sample_uniform, multinomial
  try:
    cmd._resample_command(ids)  # commands.py:309-375 (adaptive sampling, commands.py:258-301)
  finally:
    ref_cmds.sample_uniform, torch.multinomial = real_su, real_mn
  assert not queue
  out.update(mo_out_time_steps=cmd.time_steps, mo_out_current_bin_failed=cmd._current_bin_failed,
             mo_out_qpos=ed.data.qpos, mo_out_qvel=ed.data.qvel, mo_bin_count=np.array(cmd.bin_count))
  out.update({"mo_out_" + m: v for m, v in cmd.metrics.items()})


def main() -> None:
  make_golden.setup()
  torch.manual_seed(0)
  g = torch.Generator().manual_seed(20261017)
  out: dict = {"seed": np.array(SEED, dtype=np.uint64), "step": np.array(STEP), "n": np.array(N)}
  gen_events(out, g)
  gen_randomize_field(out, g)
  gen_velocity_command(out, g)
  gen_motion(out, g)
  arrs = {k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in out.items()}
  OUT.parent.mkdir(parents=True, exist_ok=True)
  with open(OUT, "wb") as f:  # fixed member timestamps: byte-reproducible
    import zipfile

    with zipfile.ZipFile(f, "w", zipfile.ZIP_DEFLATED) as z:
      for k in sorted(arrs):
        b = io.BytesIO()
        np.save(b, arrs[k], allow_pickle=False)
        zi = zipfile.ZipInfo(k + ".npy", date_time=(2026, 1, 1, 0, 0, 0))
        zi.compress_type = zipfile.ZIP_DEFLATED
        z.writestr(zi, b.getvalue())
  print("wrote", OUT, len(arrs), "arrays")


if __name__ == "__main__":
  main()
