"""Unitree G1 constants (restated from src/mjlab/asset_zoo/robots/unitree_g1/g1_constants.py).

Actuator groups, reflected inertias, PD gains (10 Hz natural frequency,
damping ratio 2), keyframes, collision configs and action scales follow
g1_constants.py:39-297.
"""

from __future__ import annotations

import math

from mjlab_amd.asset_zoo import load_spec
from mjlab_amd.entity.entity import EntityArticulationInfoCfg, EntityCfg
from mjlab_amd.utils.spec_config import ActuatorCfg, CollisionCfg


def reflected_inertia_from_two_stage_planetary(rotor, gear):
  """utils/actuator.py:26-37."""
  assert gear[0] == 1
  return rotor[0] * (gear[1] * gear[2]) ** 2 + rotor[1] * gear[2] ** 2 + rotor[2]


ARMATURE_5020 = reflected_inertia_from_two_stage_planetary(
  (0.139e-4, 0.017e-4, 0.169e-4), (1, 1 + 46 / 18, 1 + 56 / 16)
)
ARMATURE_7520_14 = reflected_inertia_from_two_stage_planetary(
  (0.489e-4, 0.098e-4, 0.533e-4), (1, 4.5, 1 + 48 / 22)
)
ARMATURE_7520_22 = reflected_inertia_from_two_stage_planetary(
  (0.489e-4, 0.109e-4, 0.738e-4), (1, 4.5, 5)
)
ARMATURE_4010 = reflected_inertia_from_two_stage_planetary((0.068e-4, 0.0, 0.0), (1, 5, 5))

NATURAL_FREQ = 10 * 2.0 * 3.1415926535
DAMPING_RATIO = 2.0


def _kp(a):
  return a * NATURAL_FREQ**2


def _kd(a):
  return 2.0 * DAMPING_RATIO * a * NATURAL_FREQ


G1_ACTUATOR_5020 = ActuatorCfg(
  joint_names_expr=(
    ".*_elbow_joint",
    ".*_shoulder_pitch_joint",
    ".*_shoulder_roll_joint",
    ".*_shoulder_yaw_joint",
    ".*_wrist_roll_joint",
  ),
  effort_limit=25.0,
  armature=ARMATURE_5020,
  stiffness=_kp(ARMATURE_5020),
  damping=_kd(ARMATURE_5020),
)
G1_ACTUATOR_7520_14 = ActuatorCfg(
  joint_names_expr=(".*_hip_pitch_joint", ".*_hip_yaw_joint", "waist_yaw_joint"),
  effort_limit=88.0,
  armature=ARMATURE_7520_14,
  stiffness=_kp(ARMATURE_7520_14),
  damping=_kd(ARMATURE_7520_14),
)
G1_ACTUATOR_7520_22 = ActuatorCfg(
  joint_names_expr=(".*_hip_roll_joint", ".*_knee_joint"),
  effort_limit=139.0,
  armature=ARMATURE_7520_22,
  stiffness=_kp(ARMATURE_7520_22),
  damping=_kd(ARMATURE_7520_22),
)
G1_ACTUATOR_4010 = ActuatorCfg(
  joint_names_expr=(".*_wrist_pitch_joint", ".*_wrist_yaw_joint"),
  effort_limit=5.0,
  armature=ARMATURE_4010,
  stiffness=_kp(ARMATURE_4010),
  damping=_kd(ARMATURE_4010),
)
G1_ACTUATOR_WAIST = ActuatorCfg(
  joint_names_expr=("waist_pitch_joint", "waist_roll_joint"),
  effort_limit=25.0 * 2,
  armature=ARMATURE_5020 * 2,
  stiffness=_kp(ARMATURE_5020) * 2,
  damping=_kd(ARMATURE_5020) * 2,
)
G1_ACTUATOR_ANKLE = ActuatorCfg(
  joint_names_expr=(".*_ankle_pitch_joint", ".*_ankle_roll_joint"),
  effort_limit=25.0 * 2,
  armature=ARMATURE_5020 * 2,
  stiffness=_kp(ARMATURE_5020) * 2,
  damping=_kd(ARMATURE_5020) * 2,
)

HOME_KEYFRAME = EntityCfg.InitialStateCfg(
  pos=(0, 0, 0.783675),
  joint_pos={
    ".*_hip_pitch_joint": -0.1,
    ".*_knee_joint": 0.3,
    ".*_ankle_pitch_joint": -0.2,
    ".*_shoulder_pitch_joint": 0.2,
    ".*_elbow_joint": 1.28,
    "left_shoulder_roll_joint": 0.2,
    "right_shoulder_roll_joint": -0.2,
  },
  joint_vel={".*": 0.0},
)

KNEES_BENT_KEYFRAME = EntityCfg.InitialStateCfg(
  pos=(0, 0, 0.76),
  joint_pos={
    ".*_hip_pitch_joint": -0.312,
    ".*_knee_joint": 0.669,
    ".*_ankle_pitch_joint": -0.363,
    ".*_elbow_joint": 0.6,
    "left_shoulder_roll_joint": 0.2,
    "left_shoulder_pitch_joint": 0.2,
    "right_shoulder_roll_joint": -0.2,
    "right_shoulder_pitch_joint": 0.2,
  },
  joint_vel={".*": 0.0},
)

_FEET = r"^(left|right)_foot[1-7]_collision$"

FULL_COLLISION = CollisionCfg(
  geom_names_expr=(".*_collision",),
  condim={_FEET: 3, ".*_collision": 1},
  priority={_FEET: 1},
  friction={_FEET: (0.6,)},
)

FULL_COLLISION_WITHOUT_SELF = CollisionCfg(
  geom_names_expr=(".*_collision",),
  contype=0,
  conaffinity=1,
  condim={_FEET: 3, ".*_collision": 1},
  priority={_FEET: 1},
  friction={_FEET: (0.6,)},
)

FEET_ONLY_COLLISION = CollisionCfg(
  geom_names_expr=(_FEET,),
  contype=0,
  conaffinity=1,
  condim=3,
  priority=1,
  friction=(0.6,),
)

G1_ARTICULATION = EntityArticulationInfoCfg(
  actuators=(
    G1_ACTUATOR_5020,
    G1_ACTUATOR_7520_14,
    G1_ACTUATOR_7520_22,
    G1_ACTUATOR_4010,
    G1_ACTUATOR_WAIST,
    G1_ACTUATOR_ANKLE,
  ),
  soft_joint_pos_limit_factor=0.9,
)


def get_spec():
  return load_spec("unitree_g1")


def get_g1_robot_cfg() -> EntityCfg:
  return EntityCfg(
    init_state=KNEES_BENT_KEYFRAME,
    collisions=(FULL_COLLISION,),
    spec_fn=get_spec,
    articulation=G1_ARTICULATION,
  )


G1_ACTION_SCALE: dict[str, float] = {}
for _a in G1_ARTICULATION.actuators:
  for _n in _a.joint_names_expr:
    if _a.stiffness:
      G1_ACTION_SCALE[_n] = 0.25 * _a.effort_limit / _a.stiffness

assert math.isfinite(sum(G1_ACTION_SCALE.values()))
