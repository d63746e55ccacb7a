"""Unitree G1 flat velocity task (``src/mjlab/tasks/velocity/config/g1/env_cfgs.py:15-113``)."""

from __future__ import annotations

from mjlab_amd.asset_zoo.g1 import G1_ACTION_SCALE, get_g1_robot_cfg
from mjlab_amd.sensor import ContactMatch, ContactSensorCfg
from mjlab_amd.tasks.velocity.velocity_env_cfg import create_velocity_env_cfg

_STD_WALKING = {
  r".*hip_pitch.*": 0.3, r".*hip_roll.*": 0.15, r".*hip_yaw.*": 0.15, r".*knee.*": 0.35,
  r".*ankle_pitch.*": 0.25, r".*ankle_roll.*": 0.1, r".*waist_yaw.*": 0.2, r".*waist_roll.*": 0.08,
  r".*waist_pitch.*": 0.1, r".*shoulder_pitch.*": 0.15, r".*shoulder_roll.*": 0.15,
  r".*shoulder_yaw.*": 0.1, r".*elbow.*": 0.15, r".*wrist.*": 0.3,
}
_STD_RUNNING = {
  r".*hip_pitch.*": 0.5, r".*hip_roll.*": 0.2, r".*hip_yaw.*": 0.2, r".*knee.*": 0.6,
  r".*ankle_pitch.*": 0.35, r".*ankle_roll.*": 0.15, r".*waist_yaw.*": 0.3, r".*waist_roll.*": 0.08,
  r".*waist_pitch.*": 0.2, r".*shoulder_pitch.*": 0.5, r".*shoulder_roll.*": 0.2,
  r".*shoulder_yaw.*": 0.15, r".*elbow.*": 0.35, r".*wrist.*": 0.3,
}


def feet_ground_cfg() -> ContactSensorCfg:
  return ContactSensorCfg(
    name="feet_ground_contact",
    primary=ContactMatch(mode="subtree", pattern=r"^(left_ankle_roll_link|right_ankle_roll_link)$", entity="robot"),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found", "force"),
    reduce="netforce",
    num_slots=1,
    track_air_time=True,
  )


def self_collision_cfg() -> ContactSensorCfg:
  return ContactSensorCfg(
    name="self_collision",
    primary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    secondary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    fields=("found",),
    reduce="none",
    num_slots=1,
  )


def unitree_g1_flat_env_cfg():
  site_names = ("left_foot", "right_foot")
  geom_names = tuple(f"{side}_foot{i}_collision" for side in ("left", "right") for i in range(1, 8))
  cfg = create_velocity_env_cfg(
    robot_cfg=get_g1_robot_cfg(),
    action_scale=G1_ACTION_SCALE,
    viewer_body_name="torso_link",
    site_names=site_names,
    feet_sensor_cfg=feet_ground_cfg(),
    self_collision_sensor_cfg=self_collision_cfg(),
    foot_friction_geom_names=geom_names,
    posture_std_standing={".*": 0.05},
    posture_std_walking=dict(_STD_WALKING),
    posture_std_running=dict(_STD_RUNNING),
    body_ang_vel_weight=-0.05,
    angular_momentum_weight=-0.02,
    self_collision_weight=-1.0,
    air_time_weight=0.0,
  )
  cfg.commands["twist"].viz.z_offset = 1.15
  return cfg
