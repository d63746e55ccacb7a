"""Scene composition: terrain + entities (prefix ``name/``) + sensors.

Restates ``src/mjlab/scene/scene.py`` and the plane path of
``src/mjlab/terrains/terrain_importer.py``:

* the terrain is a static body ``terrain`` with one plane geom
  (``terrain_importer.py:154-163``), added before the entities so that body 1
  is ``terrain`` and geom 0 is the plane, as in the reference;
* env origins follow the reference grid (``terrain_importer.py:225-240``);
* one visual site per env origin, ``env_origin_{i}``, on the world body
  (``terrain_importer.py:95-120``), so ``nsite = num_envs + (robot sites)``
  and the robot's site ids start at num_envs, as in the reference model. The
  compiled model records them as ``Model.nsite_origin``: static world sites
  whose poses the Simulation writes once, so the step kernel sees only the
  sites that move.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

import numpy as np
import torch

from mjlab_amd.entity import Entity, EntityCfg
from mjlab_amd.entity.entity import merge_keyframes
from mjlab_amd.sensor import BuiltinSensor, SensorCfg
from mjlab_amd.spec.compiler import Model, compile_spec
from mjlab_amd.spec.spec import BodySpec, GeomSpec, SiteSpec, Spec


@dataclass
class TerrainImporterCfg:
  terrain_type: str = "plane"
  terrain_generator: Any = None
  env_spacing: float | None = 2.0
  max_init_terrain_level: int | None = None
  num_envs: int = 1


class TerrainImporter:
  def __init__(self, cfg: TerrainImporterCfg, device: str) -> None:
    if cfg.terrain_type != "plane":
      raise NotImplementedError("only plane terrain is supported by mjlab_amd")
    self.cfg = cfg
    self.device = device
    self.spec = Spec()
    body = BodySpec(name="terrain")
    body.geoms.append(GeomSpec(name="terrain", type="plane", size=[0.0, 0.0, 0.01]))
    self.spec.worldbody.children.append(body)
    self.terrain_origins = None
    self.env_origins = self._grid(cfg.num_envs, cfg.env_spacing)
    self._add_env_origin_sites()

  def _add_env_origin_sites(self) -> None:
    """terrain_importer.py:95-120: a transparent sphere site per env origin."""
    for i, o in enumerate(self.env_origins.cpu().numpy()):
      self.spec.worldbody.sites.append(SiteSpec(name=f"env_origin_{i}", type="sphere", pos=[float(x) for x in o],
                                                size=[0.3, 0.3, 0.3], group=4, rgba=[0.2, 0.6, 0.2, 0.3]))

  def _grid(self, num_envs: int, spacing: float) -> torch.Tensor:
    origins = torch.zeros(num_envs, 3, device=self.device)
    num_rows = np.ceil(num_envs / int(np.sqrt(num_envs)))
    num_cols = np.ceil(num_envs / num_rows)
    ii, jj = torch.meshgrid(
      torch.arange(num_rows, device=self.device), torch.arange(num_cols, device=self.device), indexing="ij"
    )
    origins[:, 0] = -(ii.flatten()[:num_envs] - (num_rows - 1) / 2) * spacing
    origins[:, 1] = (jj.flatten()[:num_envs] - (num_cols - 1) / 2) * spacing
    return origins

  def update_env_origins(self, env_ids, move_up, move_down) -> None:
    return


@dataclass(kw_only=True)
class SceneCfg:
  num_envs: int = 1
  env_spacing: float = 2.0
  terrain: TerrainImporterCfg | None = None
  entities: dict[str, EntityCfg] = field(default_factory=dict)
  sensors: tuple[SensorCfg, ...] = field(default_factory=tuple)
  extent: float | None = None


class Scene:
  def __init__(self, scene_cfg: SceneCfg, device: str) -> None:
    self._cfg = scene_cfg
    self._device = device
    self._entities: dict[str, Entity] = {}
    self._sensors: dict[str, Any] = {}
    self._terrain: TerrainImporter | None = None
    self._default_env_origins: torch.Tensor | None = None
    self._spec = Spec(model="mjlab scene")
    self._add_terrain()
    self._add_entities()
    self._add_sensors()

  def compile(self, nconmax: int | None = None, njmax: int | None = None) -> Model:
    m = compile_spec(self._spec, nconmax or 0, njmax or 0)
    merge_keyframes(m, self._entities.values())
    # the env-origin sites lead the site list (the terrain's world sites are attached first)
    n0 = self._cfg.num_envs if self._terrain is not None else 0
    names = m.names["site"][:n0]
    assert all(nm == f"env_origin_{i}" for i, nm in enumerate(names)) and (m.site_bodyid[:n0] == 0).all()
    m.nsite_origin = n0
    return m

  @property
  def spec(self) -> Spec:
    return self._spec

  @property
  def env_origins(self) -> torch.Tensor:
    if self._terrain is not None:
      return self._terrain.env_origins
    assert self._default_env_origins is not None
    return self._default_env_origins

  @property
  def env_spacing(self) -> float:
    return self._cfg.env_spacing

  @property
  def entities(self) -> dict[str, Entity]:
    return self._entities

  @property
  def sensors(self) -> dict[str, Any]:
    return self._sensors

  @property
  def terrain(self) -> TerrainImporter | None:
    return self._terrain

  @property
  def num_envs(self) -> int:
    return self._cfg.num_envs

  @property
  def device(self) -> str:
    return self._device

  def __getitem__(self, key: str) -> Any:
    if key == "terrain":
      if self._terrain is None:
        raise KeyError("No terrain configured in this scene.")
      return self._terrain
    if key in self._sensors:
      return self._sensors[key]
    if key in self._entities:
      return self._entities[key]
    raise KeyError(f"Scene element '{key}' not found. Available: {list(self._entities) + list(self._sensors)}")

  def initialize(self, model: Model, sim_model, data) -> None:
    self._default_env_origins = torch.zeros((self._cfg.num_envs, 3), device=self._device)
    for ent in self._entities.values():
      ent.initialize(model, sim_model, data, self._device)
    for s in self._sensors.values():
      s.initialize(model, sim_model, data, self._device)

  def reset(self, env_ids=None) -> None:
    for ent in self._entities.values():
      ent.reset(env_ids)
    for s in self._sensors.values():
      s.reset(env_ids)

  def update(self, dt: float, skip=None) -> None:
    """skip: a sensor whose update the physics step already made (the env's
    fused contact-sensor timers, ContactSensor.attach_air_time_to)."""
    for ent in self._entities.values():
      ent.update(dt)
    for s in self._sensors.values():
      if s is not skip:
        s.update(dt)

  def write_data_to_sim(self) -> None:
    for ent in self._entities.values():
      ent.write_data_to_sim()

  def _add_entities(self) -> None:
    for name, cfg in self._cfg.entities.items():
      ent = Entity(cfg)
      ent.prefix = f"{name}/"
      self._entities[name] = ent
      self._spec.attach(ent.spec, prefix=f"{name}/")

  def _add_terrain(self) -> None:
    if self._cfg.terrain is None:
      return
    self._cfg.terrain.num_envs = self._cfg.num_envs
    self._cfg.terrain.env_spacing = self._cfg.env_spacing
    self._terrain = TerrainImporter(self._cfg.terrain, self._device)
    self._spec.attach(self._terrain.spec)

  def _add_sensors(self) -> None:
    for scfg in self._cfg.sensors:
      s = scfg.build()
      s.edit_spec(self._spec, self._entities)
      self._sensors[scfg.name] = s
    for s in self._spec.sensors:
      if s.name not in self._sensors and s.type != "contact":
        self._sensors[s.name] = BuiltinSensor.from_existing(s.name)
