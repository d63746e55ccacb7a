"""Unitree Go1 constants (restated from src/mjlab/asset_zoo/robots/unitree_go1/go1_constants.py)."""

from __future__ import annotations

from mjlab_amd.asset_zoo import load_spec
from mjlab_amd.entity.entity import EntityArticulationInfoCfg, EntityCfg
from mjlab_amd.utils.spec_config import ActuatorCfg, CollisionCfg

ROTOR_INERTIA = 0.000111842
HIP_GEAR_RATIO = 6
KNEE_GEAR_RATIO = HIP_GEAR_RATIO * 1.5
HIP_ARMATURE = ROTOR_INERTIA * HIP_GEAR_RATIO**2
KNEE_ARMATURE = ROTOR_INERTIA * KNEE_GEAR_RATIO**2

NATURAL_FREQ = 10 * 2.0 * 3.1415926535
DAMPING_RATIO = 2.0

GO1_HIP_ACTUATOR_CFG = ActuatorCfg(
  joint_names_expr=(".*_hip_joint", ".*_thigh_joint"),
  effort_limit=23.7,
  stiffness=HIP_ARMATURE * NATURAL_FREQ**2,
  damping=2 * DAMPING_RATIO * HIP_ARMATURE * NATURAL_FREQ,
  armature=HIP_ARMATURE,
)
GO1_KNEE_ACTUATOR_CFG = ActuatorCfg(
  joint_names_expr=(".*_calf_joint",),
  effort_limit=35.55,
  stiffness=KNEE_ARMATURE * NATURAL_FREQ**2,
  damping=2 * DAMPING_RATIO * KNEE_ARMATURE * NATURAL_FREQ,
  armature=KNEE_ARMATURE,
)

INIT_STATE = EntityCfg.InitialStateCfg(
  pos=(0.0, 0.0, 0.278),
  joint_pos={
    ".*thigh_joint": 0.9,
    ".*calf_joint": -1.8,
    ".*R_hip_joint": 0.1,
    ".*L_hip_joint": -0.1,
  },
  joint_vel={".*": 0.0},
)

_FOOT = "^[FR][LR]_foot_collision$"

FEET_ONLY_COLLISION = CollisionCfg(
  geom_names_expr=(_FOOT,),
  contype=0,
  conaffinity=1,
  condim=3,
  priority=1,
  friction=(0.6,),
  solimp=(0.9, 0.95, 0.023),
)

FULL_COLLISION = CollisionCfg(
  geom_names_expr=(".*_collision",),
  condim={_FOOT: 3, ".*_collision": 1},
  priority={_FOOT: 1},
  friction={_FOOT: (0.6,)},
  solimp={_FOOT: (0.9, 0.95, 0.023)},
  contype=1,
  conaffinity=0,
)

GO1_ARTICULATION = EntityArticulationInfoCfg(
  actuators=(GO1_HIP_ACTUATOR_CFG, GO1_KNEE_ACTUATOR_CFG),
  soft_joint_pos_limit_factor=0.9,
)


def get_spec():
  return load_spec("unitree_go1")


def get_go1_robot_cfg() -> EntityCfg:
  return EntityCfg(
    init_state=INIT_STATE,
    collisions=(FULL_COLLISION,),
    spec_fn=get_spec,
    articulation=GO1_ARTICULATION,
  )


GO1_ACTION_SCALE: dict[str, float] = {}
for _a in GO1_ARTICULATION.actuators:
  for _n in _a.joint_names_expr:
    if _a.stiffness:
      GO1_ACTION_SCALE[_n] = 0.25 * _a.effort_limit / _a.stiffness
