"""Env-layer golden vectors from the reference's own managers (run HERE only).

The reference's managers, MDP terms, EntityData, ContactSensor/BuiltinSensor and
UniformVelocityCommand are executed unmodified on a stand-in env whose
simulation data are plain torch tensors (the physics modules are inert stubs,
tools/make_golden.py recipe). The sim-data frames fed to them are INPUTS only:
seeded numpy initial states and actions, stepped by the float64 oracle
(tests/oracle_sim.py) through mjlab_amd's action manager (capture(); no use of
mjlab_amd's RNG, so a rerun writes byte-identical fixtures). Every output in
the fixture comes from reference code:

  - EntityData.initialize-derived defaults (default_joint_pos from the G1
    keyframe regexes, soft joint limits)                  entity/entity.py:326-400
  - ActionManager.process_action/apply_action + JointPositionAction
    (per-actuator scale from G1_ACTION_SCALE, offset = default pose) -> ctrl
                                                          joint_actions.py:90-108
  - ContactSensor air-time tracking                       contact_sensor.py:327-367
  - TerminationManager.compute (time_out, fell_over)      termination_manager.py:86-96
  - RewardManager.compute (14 G1 terms, weights, dt)      reward_manager.py:76-88
  - CommandManager.compute (UniformVelocityCommand, heading control, metrics)
                                                          velocity_command.py:51-101
  - ObservationManager.compute (policy with uniform noise, critic)
                                                          observation_manager.py:147-195

Uniform noise draws are fixed: torch.rand_like is replaced by a supplier of
pre-drawn U[0,1) tensors (stored in the fixture), consumed in term order.
Tracking (G1): the reference MotionCommand (MotionLoader over a synthetic
clip in the csv_to_npz.py format, relative body targets, metrics) with the
tracking rewards/observations/terminations (tracking/mdp/*.py).
Output: tests/golden/{velocity_g1,velocity_go1,tracking_g1}_env.npz (data only; no reference source).
"""

from __future__ import annotations

import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))

import make_golden  # noqa: E402

OUT = ROOT / "tests" / "golden"
SIM_FIELDS = ("xpos", "xquat", "xmat", "xipos", "subtree_com", "cvel", "geom_xpos", "geom_xmat", "site_xpos", "site_xmat",
              "qpos", "qvel", "qacc", "actuator_force", "qfrc_applied", "xfrc_applied", "sensordata", "time")
MODEL_FIELDS = ("body_iquat", "geom_bodyid", "site_bodyid", "actuator_gainprm", "actuator_biasprm", "jnt_range")
TASKS = {
  # task id: (reference env-cfg module, cfg value, robot-cfg module, robot-cfg fn, fixture)
  "Mjlab-Velocity-Flat-Unitree-G1": ("mjlab.tasks.velocity.config.g1.env_cfgs", "UNITREE_G1_FLAT_ENV_CFG",
                                     "mjlab.asset_zoo.robots.unitree_g1.g1_constants", "get_g1_robot_cfg",
                                     "velocity_g1_env.npz"),
  "Mjlab-Velocity-Flat-Unitree-Go1": ("mjlab.tasks.velocity.config.go1.env_cfgs", "UNITREE_GO1_FLAT_ENV_CFG",
                                      "mjlab.asset_zoo.robots.unitree_go1.go1_constants", "get_go1_robot_cfg",
                                      "velocity_go1_env.npz"),
  "Mjlab-Tracking-Flat-Unitree-G1": ("mjlab.tasks.tracking.config.g1.env_cfgs", "G1_FLAT_TRACKING_ENV_CFG",
                                     "mjlab.asset_zoo.robots.unitree_g1.g1_constants", "get_g1_robot_cfg",
                                     "tracking_g1_env.npz"),
}
MOTION_FRAMES = 40


def save_npz(path: Path, arrs: dict) -> None:
  """np.savez_compressed with fixed member timestamps and order: byte-reproducible."""
  import io
  import zipfile

  with open(path, "wb") as f, zipfile.ZipFile(f, "w", zipfile.ZIP_DEFLATED) as z:
    for k in sorted(arrs):
      b = io.BytesIO()
      np.save(b, arrs[k], allow_pickle=False)
      zi = zipfile.ZipInfo(k + ".npy", date_time=(2026, 1, 1, 0, 0, 0))
      zi.compress_type = zipfile.ZIP_DEFLATED
      z.writestr(zi, b.getvalue())


def synthetic_motion_file(path: Path) -> dict:
  """INPUT motion clip (mjlab_amd's synthetic clip, csv_to_npz.py format)."""
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.motion import KEYS, save_motion, synthetic_motion
  from mjlab_amd.tasks import load_env_cfg
  from tests import oracle_sim

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = MOTION_FRAMES
  env = ManagerBasedRlEnv(cfg, device="cpu")
  oracle_sim.attach(env.sim)
  mot = synthetic_motion(env.sim, env.scene["robot"], num_frames=MOTION_FRAMES, fps=50.0)
  save_motion(path, 50.0, **{k: mot[k] for k in KEYS})
  return dict(np.load(path))


def capture(task: str, n: int, frames: int, warm: int, seed: int, motion_file: str | None = None):
  """INPUT frames, independent of mjlab_amd's own randomness: the
  initial states, actions and manager states are drawn from a seeded numpy
  Generator, and the physics is the float64 oracle (tests/oracle_sim.py)
  stepped through mjlab_amd's action manager (process/apply, decimation) —
  no env.reset/env.step, so no event, command-resampling or reset draws. The
  same seed gives byte-identical fixtures on every run."""
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg
  from mjlab_amd.utils.math import quat_mul
  from tests import oracle_sim

  cfg = load_env_cfg(task)
  cfg.scene.num_envs = n
  cfg.seed = seed
  if motion_file is not None:
    cfg.commands["motion"].motion_file = motion_file
  env = ManagerBasedRlEnv(cfg, device="cpu")
  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
  rng = np.random.default_rng(seed)
  f32 = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32))  # noqa: E731
  robot = env.scene["robot"]
  ed = robot.data
  adim = env.action_manager.total_action_dim
  # initial state: default pose at the env origin, random planar offset / yaw /
  # joint offsets (within the soft limits), small random velocities
  root = ed.default_root_state.clone()
  root[:, :3] += env.scene.env_origins
  root[:, :2] += f32(rng.uniform(-0.3, 0.3, (n, 2)))
  yaw = rng.uniform(-np.pi, np.pi, n)
  qz = f32(np.stack([np.cos(yaw / 2), np.zeros(n), np.zeros(n), np.sin(yaw / 2)], 1))
  root[:, 3:7] = quat_mul(qz, root[:, 3:7])
  root[:, 7:13] = f32(rng.uniform(-0.2, 0.2, (n, 6)))
  lim = ed.soft_joint_pos_limits
  jp = torch.clamp(ed.default_joint_pos + f32(rng.uniform(-0.2, 0.2, ed.default_joint_pos.shape)), lim[..., 0], lim[..., 1])
  jv = f32(rng.uniform(-0.5, 0.5, jp.shape))
  robot.write_root_state_to_sim(root)
  robot.write_joint_state_to_sim(jp, jv)
  env.sim.forward()

  def physics_step(a: torch.Tensor) -> None:
    env.action_manager.process_action(a)
    for _ in range(env.cfg.decimation):
      env.action_manager.apply_action()
      env.sim.step()

  for _ in range(warm):
    physics_step(f32(rng.uniform(-1, 1, (n, adim))))
  init = {
    "action": env.action_manager.action.clone(), "prev_action": env.action_manager.prev_action.clone(),
    "episode_length": torch.as_tensor(rng.integers(0, env.max_episode_length - 10, n)),
    "env_origins": env.scene.env_origins.clone(),
  }
  if "feet_ground_contact" in env.scene.sensors:
    k = env.scene["feet_ground_contact"]._air_time_state.current_air_time.shape[1]
    cur = rng.uniform(0.0, 0.6, (n, k))
    in_air = rng.random((n, k)) < 0.5
    init.update({"air_cur": f32(np.where(in_air, cur, 0.0)), "air_last": f32(rng.uniform(0.0, 0.6, (n, k))),
                 "con_cur": f32(np.where(in_air, 0.0, cur)), "con_last": f32(rng.uniform(0.0, 0.6, (n, k))),
                 "air_last_time": f32(np.full(n, float(env.sim.data.time[0])))})
  if "twist" in env.command_manager.active_terms:
    init.update({"cmd_vel": f32(rng.uniform(-1.0, 1.0, (n, 3))),
                 "cmd_heading_target": f32(rng.uniform(-np.pi, np.pi, n)),
                 "cmd_is_heading": torch.as_tensor(rng.random(n) < 0.5),
                 "cmd_is_standing": torch.as_tensor(rng.random(n) < 0.2)})
  if "motion" in env.command_manager.active_terms:
    # motion phase per env, kept clear of the clip end inside the window
    init["time_steps"] = torch.as_tensor(rng.integers(0, MOTION_FRAMES - frames - 2, n))
  # a few envs start one step short of the time limit, so time_out fires
  init["episode_length"][:3] = env.max_episode_length - 1
  seq = []
  for t in range(frames):
    a = f32(rng.uniform(-1, 1, (n, adim)))
    physics_step(a)
    fr = {f: getattr(env.sim.data, f).detach().clone() for f in SIM_FIELDS}
    if t == 0:  # tilt a few roots past the fell_over limit (input perturbation)
      tilt = torch.tensor([np.cos(0.7), np.sin(0.7), 0.0, 0.0], dtype=torch.float32)
      rb = robot.indexing.root_body_id
      fr["xquat"][4:7, rb] = quat_mul(fr["xquat"][4:7, rb], tilt.expand(3, 4))
      if motion_file is not None:  # and lift a few robots off the motion (anchor/ee height terms)
        fr["xpos"][8:11, :, 2] += 0.5
    fr["action"] = a
    seq.append(fr)
  model = {f: getattr(env.sim.model, f).detach().clone() for f in MODEL_FIELDS}
  names = {k: list(getattr(robot, k)) for k in ("joint_names", "body_names", "geom_names", "site_names", "actuator_names")}
  ix = robot.indexing
  indexing = {k: getattr(ix, k) for k in ("body_ids", "geom_ids", "site_ids", "ctrl_ids", "joint_ids", "joint_q_adr",
                                          "joint_v_adr", "free_joint_q_adr", "free_joint_v_adr")}
  indexing["root_body_id"] = ix.root_body_id
  sensors = {}
  for name, s in env.scene.sensors.items():
    if hasattr(s, "_slots"):
      sensors[name] = [(sl.field_name, sl.data_view.storage_offset() - env.sim.data.sensordata.storage_offset(),
                        sl.data_view.shape[1]) for sl in s._slots]
    else:
      v = s.data
      sensors[name] = (v.storage_offset() - env.sim.data.sensordata.storage_offset(), v.shape[1])
  meta = dict(step_dt=env.step_dt, max_episode_length=env.max_episode_length, max_episode_length_s=env.max_episode_length_s)
  return init, seq, model, names, indexing, sensors, meta


def gen(task: str, n: int = 24, frames: int = 4) -> None:
  import importlib
  import tempfile

  motion_file, motion = None, {}
  if "Tracking" in task:
    motion_file = str(Path(tempfile.mkdtemp()) / "clip.npz")
    motion = synthetic_motion_file(Path(motion_file))
  init, seq, model, names, indexing, sensors, meta = capture(task, n, frames, warm=6, seed=11, motion_file=motion_file)
  cfg_mod, cfg_name, robot_mod, robot_fn, fixture = TASKS[task]
  from mjlab.entity.data import EntityData
  from mjlab.entity.entity import Entity
  from mjlab.managers.action_manager import ActionManager
  from mjlab.managers.command_manager import CommandManager
  from mjlab.managers.observation_manager import ObservationManager
  from mjlab.managers.reward_manager import RewardManager
  from mjlab.managers.termination_manager import TerminationManager
  from mjlab.sensor.builtin_sensor import BuiltinSensor
  from mjlab.sensor.contact_sensor import ContactSensor
  CFG = getattr(importlib.import_module(cfg_mod), cfg_name)
  if motion_file is not None:
    CFG.commands["motion"].motion_file = motion_file
  get_robot_cfg = getattr(importlib.import_module(robot_mod), robot_fn)

  dev = "cpu"
  data = SimpleNamespace(nworld=n, ctrl=torch.zeros(n, len(names["actuator_names"])),
                         **{f: seq[0][f].clone() for f in SIM_FIELDS})
  mdl = SimpleNamespace(**{f: model[f] for f in MODEL_FIELDS})

  # ---- the robot: reference Entity/EntityData over the stand-in data ----
  class Robot(Entity):
    joint_names = property(lambda self: tuple(names["joint_names"]))
    body_names = property(lambda self: tuple(names["body_names"]))
    geom_names = property(lambda self: tuple(names["geom_names"]))
    site_names = property(lambda self: tuple(names["site_names"]))
    actuator_names = property(lambda self: tuple(names["actuator_names"]))
    num_joints = property(lambda self: len(names["joint_names"]))
    num_bodies = property(lambda self: len(names["body_names"]))
    num_geoms = property(lambda self: len(names["geom_names"]))
    num_sites = property(lambda self: len(names["site_names"]))
    num_actuators = property(lambda self: len(names["actuator_names"]))
    is_fixed_base = property(lambda self: False)
    is_articulated = property(lambda self: True)
    is_actuated = property(lambda self: True)

    def _compute_indexing(self, mj_model, device):
      return SimpleNamespace(**indexing, bodies=None)

  robot = Robot.__new__(Robot)
  robot.cfg = get_robot_cfg()
  jid = indexing["joint_ids"].tolist()
  robot._non_free_joints = [SimpleNamespace(id=j) for j in jid]
  robot.initialize(None, mdl, data, dev)
  ed: EntityData = robot.data
  assert isinstance(ed, EntityData)

  # ---- sensors ----
  sd = data.sensordata
  class Scene(dict):
    env_origins = init["env_origins"]

  scene = Scene(robot=robot)
  for sname, spec in sensors.items():
    if isinstance(spec, tuple):
      s = BuiltinSensor.__new__(BuiltinSensor)
      s._data_view = sd[:, spec[0] : spec[0] + spec[1]]
      scene[sname] = s
  for scfg in CFG.scene.sensors:
    s = ContactSensor.__new__(ContactSensor)
    s.cfg = scfg
    s._slots = [SimpleNamespace(field_name=f, data_view=sd[:, a : a + w]) for f, a, w in sensors[scfg.name]]
    s._data = data
    s._air_time_state = None
    scene[scfg.name] = s
  feet = scene.get("feet_ground_contact")
  if feet is not None:
    feet._air_time_state = SimpleNamespace(
      current_air_time=init["air_cur"].clone(), last_air_time=init["air_last"].clone(),
      current_contact_time=init["con_cur"].clone(), last_contact_time=init["con_last"].clone(),
      last_time=init["air_last_time"].clone())

  env = SimpleNamespace(num_envs=n, device=dev, scene=scene, step_dt=meta["step_dt"],
                        max_episode_length=meta["max_episode_length"], max_episode_length_s=meta["max_episode_length_s"],
                        episode_length_buf=init["episode_length"].clone(), extras={"log": {}}, common_step_counter=0)
  env.action_manager = ActionManager(CFG.actions, env)
  env.action_manager._action[:] = init["action"]
  env.action_manager._prev_action[:] = init["prev_action"]
  env.command_manager = CommandManager(CFG.commands, env)
  env.termination_manager = TerminationManager(CFG.terminations, env)
  cname = env.command_manager.active_terms[0]
  cmd = env.command_manager.get_term(cname)
  cmd.time_left[:] = 100.0  # no resampling inside the fixture window (RNG streams differ by design)
  if cname == "twist":
    cmd.vel_command_b[:] = init["cmd_vel"]
    cmd.heading_target[:] = init["cmd_heading_target"]
    cmd.is_heading_env[:] = init["cmd_is_heading"]
    cmd.is_standing_env[:] = init["cmd_is_standing"]
  else:
    cmd.time_steps[:] = init["time_steps"]
    cmd._update_command()  # relative targets for the initial phase (as after a reset)
  env.reward_manager = RewardManager(CFG.rewards, env)

  g = torch.Generator().manual_seed(5)
  pending: list[torch.Tensor] = []
  real_rand_like = torch.rand_like

  def rand_like(x, *a, **k):
    u = torch.rand(x.shape, generator=g)
    pending.append(u)
    return u

  torch.rand_like = rand_like
  # velocity_env_cfg.py builds critic_terms = {**policy_terms, ...}: the two
  # groups share term-cfg objects, and ObservationManager._prepare_terms sets
  # noise=None on every critic term, which would also strip the policy noise
  # when the cfg object is used directly (the CLI scripts rebuild the cfg).
  # mjlab_amd keeps the groups separate, so the fixture does too.
  from copy import deepcopy

  crit = CFG.observations["critic"]
  crit.terms = {k: deepcopy(v) for k, v in crit.terms.items()}
  pol = CFG.observations["policy"]
  pol.terms = {k: deepcopy(v) for k, v in pol.terms.items()}
  env.observation_manager = ObservationManager(CFG.observations, env)
  pending.clear()

  out = {
    "init_" + k: v for k, v in init.items()
  }
  out.update({"motion_" + k: torch.as_tensor(v) for k, v in motion.items()})
  out["default_joint_pos"] = ed.default_joint_pos
  out["soft_joint_pos_limits"] = ed.soft_joint_pos_limits
  out["action_scale"] = env.action_manager.get_term("joint_pos").scale
  out["action_offset"] = env.action_manager.get_term("joint_pos").offset
  for t, fr in enumerate(seq):
    env.action_manager.process_action(fr["action"])
    env.action_manager.apply_action()
    out[f"f{t}_ctrl"] = data.ctrl.clone()
    for f in SIM_FIELDS:
      getattr(data, f).copy_(fr[f])
    if feet is not None:
      feet.update(env.step_dt)
    env.episode_length_buf += 1
    env.termination_manager.compute()
    rew = env.reward_manager.compute(env.step_dt)
    env.command_manager.compute(env.step_dt)
    pending.clear()
    obs = env.observation_manager.compute()
    u_policy = torch.cat(pending, dim=1)
    rec = {
        "action": fr["action"], "u_policy": u_policy, "obs_policy": obs["policy"], "obs_critic": obs["critic"],
        "reward": rew, "terminated": env.termination_manager.terminated, "time_outs": env.termination_manager.time_outs,
        "cmd": cmd.command, "heading_w": ed.heading_w,
        "root_lin_vel_b": ed.root_link_lin_vel_b, "root_ang_vel_b": ed.root_link_ang_vel_b,
        "projected_gravity_b": ed.projected_gravity_b, "body_link_ang_vel_w": ed.body_link_ang_vel_w,
        "site_lin_vel_w": ed.site_lin_vel_w, "site_quat_w": ed.site_quat_w, "geom_quat_w": ed.geom_quat_w,
        "root_com_vel_w": ed.root_com_vel_w,
    }
    for name in env.termination_manager.active_terms:
      rec["term_" + name] = env.termination_manager.get_term(name)
    rec.update({"metric_" + k: v for k, v in cmd.metrics.items()})
    if feet is not None:
      st = feet._air_time_state
      rec.update({"air_cur": st.current_air_time, "air_last": st.last_air_time, "con_cur": st.current_contact_time,
                  "con_last": st.last_contact_time})
    if cname == "motion":
      rec.update({"body_pos_relative_w": cmd.body_pos_relative_w, "body_quat_relative_w": cmd.body_quat_relative_w,
                  "time_steps": cmd.time_steps})
    out.update({f"f{t}_{k}": v.clone() for k, v in rec.items()})
    for name in env.reward_manager.active_terms:
      i = env.reward_manager._term_names.index(name)
      out[f"f{t}_rew_{name}"] = env.reward_manager._step_reward[:, i].clone()
    out.update({f"f{t}_sim_{f}": fr[f] for f in SIM_FIELDS})
  torch.rand_like = real_rand_like
  out["n_frames"] = torch.tensor(len(seq))
  OUT.mkdir(parents=True, exist_ok=True)
  arrs = {k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in out.items()}
  save_npz(OUT / fixture, arrs)
  print("wrote", fixture, len(arrs), "arrays;", "terminated", [int(out[f"f{t}_terminated"].sum()) for t in range(frames)],
        "time_outs", [int(out[f"f{t}_time_outs"].sum()) for t in range(frames)])


def main() -> None:
  make_golden.setup()
  for task in TASKS:
    gen(task)


if __name__ == "__main__":
  main()
