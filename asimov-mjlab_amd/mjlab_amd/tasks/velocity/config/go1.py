"""Unitree Go1 flat velocity task (``src/mjlab/tasks/velocity/config/go1/env_cfgs.py:15-102``)."""

from __future__ import annotations

from mjlab_amd.asset_zoo.go1 import GO1_ACTION_SCALE, get_go1_robot_cfg
from mjlab_amd.managers.manager_term_config import TerminationTermCfg
from mjlab_amd.sensor import ContactMatch, ContactSensorCfg
from mjlab_amd.tasks.velocity import mdp
from mjlab_amd.tasks.velocity.velocity_env_cfg import create_velocity_env_cfg


def unitree_go1_flat_env_cfg():
  feet = ("FR", "FL", "RR", "RL")
  geom_names = tuple(f"{n}_foot_collision" for n in feet)
  feet_ground = ContactSensorCfg(
    name="feet_ground_contact",
    primary=ContactMatch(mode="geom", pattern=geom_names, entity="robot"),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found", "force"),
    reduce="netforce",
    num_slots=1,
    track_air_time=True,
  )
  nonfoot = ContactSensorCfg(
    name="nonfoot_ground_touch",
    primary=ContactMatch(mode="geom", entity="robot", pattern=r".*_collision\d*$", exclude=tuple(geom_names)),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found",),
    reduce="none",
    num_slots=1,
  )
  hipthigh, calf = r".*(FR|FL|RR|RL)_(hip|thigh)_joint.*", r".*(FR|FL|RR|RL)_calf_joint.*"
  cfg = create_velocity_env_cfg(
    robot_cfg=get_go1_robot_cfg(),
    action_scale=GO1_ACTION_SCALE,
    viewer_body_name="trunk",
    site_names=feet,
    feet_sensor_cfg=feet_ground,
    self_collision_sensor_cfg=nonfoot,
    foot_friction_geom_names=geom_names,
    posture_std_standing={hipthigh: 0.05, calf: 0.1},
    posture_std_walking={hipthigh: 0.3, calf: 0.6},
    posture_std_running={hipthigh: 0.3, calf: 0.6},
    body_ang_vel_weight=0.0,
    angular_momentum_weight=0.0,
    self_collision_weight=0.0,
    air_time_weight=0.0,
  )
  cfg.terminations["illegal_contact"] = TerminationTermCfg(func=mdp.illegal_contact, params={"sensor_name": "nonfoot_ground_touch"})
  return cfg
