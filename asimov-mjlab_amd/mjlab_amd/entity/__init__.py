from mjlab_amd.entity.data import EntityData, compute_velocity_from_cvel
from mjlab_amd.entity.entity import Entity, EntityArticulationInfoCfg, EntityCfg, EntityIndexing

__all__ = [
  "Entity",
  "EntityArticulationInfoCfg",
  "EntityCfg",
  "EntityData",
  "EntityIndexing",
  "compute_velocity_from_cvel",
]
