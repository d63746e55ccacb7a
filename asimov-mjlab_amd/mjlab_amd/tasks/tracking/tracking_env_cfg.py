"""Motion-tracking task cfg (``src/mjlab/tasks/tracking/tracking_env_cfg.py:36-332``).

Term-for-term the reference's ``create_tracking_env_cfg`` (BeyondMimic-style
whole-body tracking); the viewer config is out of scope.
"""

from __future__ import annotations

from copy import deepcopy

from mjlab_amd.entity import EntityCfg
from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnvCfg
from mjlab_amd.envs.mdp.actions import JointPositionActionCfg
from mjlab_amd.managers.manager_term_config import (
  EventTermCfg,
  ObservationGroupCfg,
  ObservationTermCfg,
  RewardTermCfg,
  TerminationTermCfg,
)
from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd.scene import SceneCfg
from mjlab_amd.scene.scene import TerrainImporterCfg
from mjlab_amd.sensor import ContactSensorCfg
from mjlab_amd.sim.sim import MujocoCfg, SimulationCfg
from mjlab_amd.tasks.tracking import mdp
from mjlab_amd.tasks.tracking.mdp.commands import MotionCommandCfg
from mjlab_amd.utils.noise import UniformNoiseCfg as Unoise

VELOCITY_RANGE = {
  "x": (-0.5, 0.5), "y": (-0.5, 0.5), "z": (-0.2, 0.2),
  "roll": (-0.52, 0.52), "pitch": (-0.52, 0.52), "yaw": (-0.78, 0.78),
}

SCENE_CFG = SceneCfg(terrain=TerrainImporterCfg(terrain_type="plane"), num_envs=1)

SIM_CFG = SimulationCfg(
  nconmax=35,
  njmax=250,
  mujoco=MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20),
)


def create_tracking_env_cfg(
  robot_cfg: EntityCfg,
  action_scale: float | dict[str, float],
  viewer_body_name: str,
  motion_file: str,
  anchor_body_name: str,
  body_names: tuple[str, ...],
  foot_friction_geom_names: tuple[str, ...],
  ee_body_names: tuple[str, ...],
  base_com_body_name: str,
  sensors: tuple[ContactSensorCfg, ...],
  pose_range: dict[str, tuple[float, float]],
  velocity_range: dict[str, tuple[float, float]],
  joint_position_range: tuple[float, float],
) -> ManagerBasedRlEnvCfg:
  del viewer_body_name  # viewer is out of scope
  scene = deepcopy(SCENE_CFG)
  scene.entities = {"robot": robot_cfg}
  scene.sensors = sensors

  actions = {"joint_pos": JointPositionActionCfg(asset_name="robot", actuator_names=(".*",), scale=action_scale, use_default_offset=True)}

  commands = {
    "motion": MotionCommandCfg(
      asset_name="robot",
      resampling_time_range=(1.0e9, 1.0e9),
      debug_vis=True,
      pose_range=pose_range,
      velocity_range=velocity_range,
      joint_position_range=joint_position_range,
      motion_file=motion_file,
      anchor_body_name=anchor_body_name,
      body_names=body_names,
    )
  }

  cmd = {"command_name": "motion"}
  policy_terms = {
    "command": ObservationTermCfg(func=mdp.generated_commands, params=dict(cmd)),
    "motion_anchor_pos_b": ObservationTermCfg(func=mdp.motion_anchor_pos_b, params=dict(cmd), noise=Unoise(n_min=-0.25, n_max=0.25)),
    "motion_anchor_ori_b": ObservationTermCfg(func=mdp.motion_anchor_ori_b, params=dict(cmd), noise=Unoise(n_min=-0.05, n_max=0.05)),
    "base_lin_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_lin_vel"}, noise=Unoise(n_min=-0.5, n_max=0.5)),
    "base_ang_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_ang_vel"}, noise=Unoise(n_min=-0.2, n_max=0.2)),
    "joint_pos": ObservationTermCfg(func=mdp.joint_pos_rel, noise=Unoise(n_min=-0.01, n_max=0.01)),
    "joint_vel": ObservationTermCfg(func=mdp.joint_vel_rel, noise=Unoise(n_min=-0.5, n_max=0.5)),
    "actions": ObservationTermCfg(func=mdp.last_action),
  }
  critic_terms = {
    "command": ObservationTermCfg(func=mdp.generated_commands, params=dict(cmd)),
    "motion_anchor_pos_b": ObservationTermCfg(func=mdp.motion_anchor_pos_b, params=dict(cmd)),
    "motion_anchor_ori_b": ObservationTermCfg(func=mdp.motion_anchor_ori_b, params=dict(cmd)),
    "body_pos": ObservationTermCfg(func=mdp.robot_body_pos_b, params=dict(cmd)),
    "body_ori": ObservationTermCfg(func=mdp.robot_body_ori_b, params=dict(cmd)),
    "base_lin_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_lin_vel"}),
    "base_ang_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_ang_vel"}),
    "joint_pos": ObservationTermCfg(func=mdp.joint_pos_rel),
    "joint_vel": ObservationTermCfg(func=mdp.joint_vel_rel),
    "actions": ObservationTermCfg(func=mdp.last_action),
  }
  observations = {
    "policy": ObservationGroupCfg(terms=policy_terms, concatenate_terms=True, enable_corruption=True),
    "critic": ObservationGroupCfg(terms=critic_terms, concatenate_terms=True, enable_corruption=False),
  }

  events = {
    "push_robot": EventTermCfg(
      func=mdp.push_by_setting_velocity, mode="interval", interval_range_s=(1.0, 3.0),
      params={"velocity_range": velocity_range},
    ),
    "base_com": EventTermCfg(
      mode="startup", func=mdp.randomize_field, domain_randomization=True,
      params={
        "asset_cfg": SceneEntityCfg("robot", body_names=(base_com_body_name,)),
        "operation": "add",
        "field": "body_ipos",
        "ranges": {0: (-0.025, 0.025), 1: (-0.05, 0.05), 2: (-0.05, 0.05)},
      },
    ),
    "add_joint_default_pos": EventTermCfg(
      mode="startup", func=mdp.randomize_field, domain_randomization=True,
      params={"asset_cfg": SceneEntityCfg("robot"), "operation": "add", "field": "qpos0", "ranges": (-0.01, 0.01)},
    ),
    "foot_friction": EventTermCfg(
      mode="startup", func=mdp.randomize_field, domain_randomization=True,
      params={
        "asset_cfg": SceneEntityCfg("robot", geom_names=foot_friction_geom_names),
        "operation": "abs",
        "field": "geom_friction",
        "ranges": (0.3, 1.2),
      },
    ),
  }

  rewards = {
    "motion_global_root_pos": RewardTermCfg(func=mdp.motion_global_anchor_position_error_exp, weight=0.5, params={**cmd, "std": 0.3}),
    "motion_global_root_ori": RewardTermCfg(func=mdp.motion_global_anchor_orientation_error_exp, weight=0.5, params={**cmd, "std": 0.4}),
    "motion_body_pos": RewardTermCfg(func=mdp.motion_relative_body_position_error_exp, weight=1.0, params={**cmd, "std": 0.3}),
    "motion_body_ori": RewardTermCfg(func=mdp.motion_relative_body_orientation_error_exp, weight=1.0, params={**cmd, "std": 0.4}),
    "motion_body_lin_vel": RewardTermCfg(func=mdp.motion_global_body_linear_velocity_error_exp, weight=1.0, params={**cmd, "std": 1.0}),
    "motion_body_ang_vel": RewardTermCfg(func=mdp.motion_global_body_angular_velocity_error_exp, weight=1.0, params={**cmd, "std": 3.14}),
    "action_rate_l2": RewardTermCfg(func=mdp.action_rate_l2, weight=-1e-1),
    "joint_limit": RewardTermCfg(func=mdp.joint_pos_limits, weight=-10.0, params={"asset_cfg": SceneEntityCfg("robot", joint_names=(".*",))}),
    "self_collisions": RewardTermCfg(func=mdp.self_collision_cost, weight=-10.0, params={"sensor_name": "self_collision"}),
  }

  terminations = {
    "time_out": TerminationTermCfg(func=mdp.time_out, time_out=True),
    "anchor_pos": TerminationTermCfg(func=mdp.bad_anchor_pos_z_only, params={**cmd, "threshold": 0.25}),
    "anchor_ori": TerminationTermCfg(
      func=mdp.bad_anchor_ori, params={"asset_cfg": SceneEntityCfg("robot"), **cmd, "threshold": 0.8},
    ),
    "ee_body_pos": TerminationTermCfg(
      func=mdp.bad_motion_body_pos_z_only, params={**cmd, "threshold": 0.25, "body_names": ee_body_names},
    ),
  }

  return ManagerBasedRlEnvCfg(
    scene=scene,
    observations=observations,
    actions=actions,
    commands=commands,
    rewards=rewards,
    terminations=terminations,
    events=events,
    sim=deepcopy(SIM_CFG),
    decimation=4,
    episode_length_s=10.0,
  )
