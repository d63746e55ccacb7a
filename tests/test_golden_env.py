"""G1 / Go1 velocity and G1 tracking env layers vs the reference's own managers (golden vectors from
tools/make_golden_env.py: the reference's EntityData, ActionManager,
ContactSensor air-time tracking, TerminationManager, RewardManager,
UniformVelocityCommand and ObservationManager run over recorded sim-data
frames).

The same frames are written into mjlab_amd's env and the same manager calls
are made; on CPU the torch paths run, on the GPU (``-m gpu``) the HIP paths
(fused reward/observation/command/air-time kernels, entity-read kernels).
Tolerances: float32 formulas evaluated in a different order -> rtol 1e-5 /
atol 1e-5 (rewards scaled by weight*dt), booleans exact.
"""

from pathlib import Path

import numpy as np
import pytest
import torch

G = Path(__file__).resolve().parent / "golden"
TASKS = {"Mjlab-Velocity-Flat-Unitree-G1": "velocity_g1_env.npz", "Mjlab-Velocity-Flat-Unitree-Go1": "velocity_go1_env.npz",
         "Mjlab-Tracking-Flat-Unitree-G1": "tracking_g1_env.npz"}
SIM_FIELDS = ("xpos", "xquat", "xmat", "xipos", "subtree_com", "cvel", "geom_xpos", "geom_xmat", "site_xpos", "site_xmat",
              "qpos", "qvel", "qacc", "actuator_force", "qfrc_applied", "xfrc_applied", "sensordata", "time")


def _close(got, want, name, rtol=1e-5, atol=1e-5):
  got = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
  if want.ndim == got.ndim and want.shape[0] == 1:  # unexpanded model field (dim0 = 1) vs per-world copy
    want = np.broadcast_to(want, got.shape)
  np.testing.assert_allclose(got.astype(np.float64), want.astype(np.float64), rtol=rtol, atol=atol, err_msg=name)


def _make_env(task: str, device: str, n: int, motion_file=None):
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg(task)
  cfg.scene.num_envs = n
  cfg.seed = 3
  if motion_file is not None:
    cfg.commands["motion"].motion_file = str(motion_file)
  env = ManagerBasedRlEnv(cfg, device=device, use_graph=False)
  if device == "cpu":
    from tests import oracle_sim

    oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
  env.reset()
  return env


def _policy_u(env, u_terms: np.ndarray, device) -> torch.Tensor:
  """Group-width U[0,1) draw whose noisy-term columns hold the reference's
  per-term draws (consumed in term order)."""
  plan, width = env.observation_manager._fused["policy"]
  u = torch.zeros(u_terms.shape[0], width, device=device)
  k = 0
  for tcfg, off, w, noise, clip, scale in plan:
    if noise is not None:
      u[:, off : off + w] = torch.as_tensor(u_terms[:, k : k + w], device=device)
      k += w
  assert k == u_terms.shape[1]
  return u


def run_golden(task: str, device: str, tmp_path) -> None:
  z = dict(np.load(G / TASKS[task]))
  n = z["init_action"].shape[0]
  motion_file = None
  if "motion_joint_pos" in z:  # the clip the reference's MotionLoader read
    motion_file = tmp_path / "clip.npz"
    np.savez(motion_file, **{k[7:]: v for k, v in z.items() if k.startswith("motion_")})
  env = _make_env(task, device, n, motion_file)
  T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
  robot = env.scene["robot"]
  # ---- defaults derived by the reference's Entity.initialize / JointAction ----
  _close(robot.data.default_joint_pos, z["default_joint_pos"], "default_joint_pos", atol=1e-7)
  _close(robot.data.soft_joint_pos_limits, z["soft_joint_pos_limits"], "soft_joint_pos_limits", atol=1e-7)
  term = env.action_manager.get_term("joint_pos")
  _close(term.scale, z["action_scale"], "action_scale", rtol=1e-6, atol=1e-7)
  _close(term.offset, z["action_offset"], "action_offset", atol=1e-7)

  # ---- initial manager state ----
  env.action_manager._action.copy_(T(z["init_action"]))
  env.action_manager._prev_action.copy_(T(z["init_prev_action"]))
  feet = env.scene.sensors.get("feet_ground_contact")
  st = feet._air_time_state if feet is not None else None
  if st is not None:
    for dst, key in ((st.current_air_time, "air_cur"), (st.last_air_time, "air_last"), (st.current_contact_time, "con_cur"),
                     (st.last_contact_time, "con_last"), (st.last_time, "air_last_time")):
      dst.copy_(T(z["init_" + key]))
  _close(env.scene.env_origins, z["init_env_origins"], "env_origins", atol=1e-6)
  cname = env.command_manager.active_terms[0]
  cmd = env.command_manager.get_term(cname)
  cmd.time_left.fill_(100.0)
  for k in cmd.metrics:
    cmd.metrics[k].zero_()
  if cname == "twist":
    cmd.vel_command_b.copy_(T(z["init_cmd_vel"]))
    cmd.heading_target.copy_(T(z["init_cmd_heading_target"]))
    cmd.is_heading_env.copy_(T(z["init_cmd_is_heading"]))
    cmd.is_standing_env.copy_(T(z["init_cmd_is_standing"]))
  else:
    cmd.time_steps.copy_(T(z["init_time_steps"]))
  env.episode_length_buf.copy_(T(z["init_episode_length"]))

  from mjlab_amd.sim import native

  native.CALLS.clear()
  real_rand_like = torch.rand_like
  try:
    for t in range(int(z["n_frames"])):
      f = lambda k: z[f"f{t}_{k}"]  # noqa: E731
      env.action_manager.process_action(T(f("action")))
      env.action_manager.apply_action()
      _close(env.sim.data.ctrl, f("ctrl"), f"f{t} ctrl", atol=1e-6)
      for name in SIM_FIELDS:
        dst = getattr(env.sim.data, name)
        if name.startswith("site_"):  # the fixture holds the robot's sites; ours follow the env-origin sites
          dst = dst[:, env.sim.mj_model.nsite_origin:]
        dst.copy_(T(f("sim_" + name)).view_as(dst))
      env.sim.epoch.bump()
      if t == 0 and cname == "motion":  # relative targets of the initial phase (generator did the same)
        cmd._update_command()
      # entity reads (EntityData properties)
      d = robot.data
      for key, got in (("heading_w", d.heading_w), ("root_lin_vel_b", d.root_link_lin_vel_b),
                       ("root_ang_vel_b", d.root_link_ang_vel_b), ("projected_gravity_b", d.projected_gravity_b),
                       ("body_link_ang_vel_w", d.body_link_ang_vel_w), ("site_lin_vel_w", d.site_lin_vel_w),
                       ("root_com_vel_w", d.root_com_vel_w)):
        _close(got, f(key), f"f{t} {key}")
      # quaternions from rotation matrices: sign-canonical per the reference
      _close(d.site_quat_w, f("site_quat_w"), f"f{t} site_quat_w", atol=2e-5)
      _close(d.geom_quat_w, f("geom_quat_w"), f"f{t} geom_quat_w", atol=2e-5)
      if st is not None:
        feet.update(env.step_dt)
        for key, got in (("air_cur", st.current_air_time), ("air_last", st.last_air_time),
                         ("con_cur", st.current_contact_time), ("con_last", st.last_contact_time)):
          _close(got, f(key), f"f{t} {key}", atol=1e-6)
      env.episode_length_buf += 1
      env.termination_manager.compute()
      np.testing.assert_array_equal(env.termination_manager.terminated.cpu().numpy(), f("terminated"), err_msg=f"f{t} terminated")
      np.testing.assert_array_equal(env.termination_manager.time_outs.cpu().numpy(), f("time_outs"), err_msg=f"f{t} time_outs")
      for name in env.termination_manager.active_terms:
        np.testing.assert_array_equal(env.termination_manager.get_term(name).cpu().numpy(), f("term_" + name),
                                      err_msg=f"f{t} termination {name}")
      rew = env.reward_manager.compute(dt=env.step_dt)
      for name in env.reward_manager.active_terms:
        if f"f{t}_rew_{name}" in z:
          i = env.reward_manager._term_names.index(name)
          _close(env.reward_manager._step_reward[:, i], f("rew_" + name), f"f{t} reward {name}")
      _close(rew, f("reward"), f"f{t} reward")
      env.command_manager.compute(dt=env.step_dt)
      _close(cmd.command, f("cmd"), f"f{t} command")
      for k, v in cmd.metrics.items():
        if f"f{t}_metric_{k}" in z:
          _close(v, f("metric_" + k), f"f{t} metric {k}", atol=2e-5)
      if cname == "motion":
        np.testing.assert_array_equal(cmd.time_steps.cpu().numpy(), f("time_steps"), err_msg=f"f{t} time_steps")
        _close(cmd.body_pos_relative_w, f("body_pos_relative_w"), f"f{t} body_pos_relative_w")
        _close(cmd.body_quat_relative_w, f("body_quat_relative_w"), f"f{t} body_quat_relative_w")
      # observations with the reference's noise draws
      u = f("u_policy")
      env.observation_manager.noise_override["policy"] = _policy_u(env, u, device)
      k = [0]

      def rand_like(x, *a, **kw):  # CPU torch path: per-term draws in term order
        w = x.shape[-1]
        out = torch.as_tensor(u[:, k[0] : k[0] + w], device=x.device, dtype=x.dtype)
        k[0] += w
        return out

      torch.rand_like = rand_like
      obs = env.observation_manager.compute()
      torch.rand_like = real_rand_like
      _close(obs["policy"], f("obs_policy"), f"f{t} obs policy")
      _close(obs["critic"], f("obs_critic"), f"f{t} obs critic")
  finally:
    torch.rand_like = real_rand_like
    env.observation_manager.noise_override.clear()
  if device != "cpu":  # the HIP entry points of this env layer actually ran
    want = ["mjh_obs_group", "mjh_reward_combine"]
    want += ["mjh_velocity_command", "mjh_air_time_update", "mjh_rew_track"] if cname == "twist" else ["mjh_motion_relative"]
    for name in want:
      assert native.CALLS[name] > 0, f"HIP entry point {name} never ran"


@pytest.mark.parametrize("task", list(TASKS))
def test_env_layer_matches_reference_cpu(task, tmp_path):
  run_golden(task, "cpu", tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize("task", list(TASKS))
def test_env_layer_matches_reference_gpu(task, tmp_path):
  run_golden(task, "cuda:0", tmp_path)
