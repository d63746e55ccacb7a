"""SceneEntityCfg: names -> ids resolution (``src/mjlab/managers/scene_entity_config.py``).

Fully-selected, in-order name lists collapse to ``slice(None)``, as in the reference.
"""

from __future__ import annotations

from dataclasses import dataclass, field

_FIELDS = [
  ("joint_names", "joint_ids", "find_joints", "num_joints"),
  ("body_names", "body_ids", "find_bodies", "num_bodies"),
  ("geom_names", "geom_ids", "find_geoms", "num_geoms"),
  ("site_names", "site_ids", "find_sites", "num_sites"),
]


@dataclass
class SceneEntityCfg:
  name: str
  joint_names: str | tuple[str, ...] | None = None
  joint_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  body_names: str | tuple[str, ...] | None = None
  body_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  geom_names: str | tuple[str, ...] | None = None
  geom_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  site_names: str | tuple[str, ...] | None = None
  site_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  preserve_order: bool = False
  # device-side copies of the resolved ids (slice(None) when all are selected):
  # indexing a device tensor with a host list issues an H2D copy, which is
  # illegal inside the captured env-step graph, so hot-path terms use these.
  joint_idx: object = field(default_factory=lambda: slice(None), repr=False, compare=False)
  body_idx: object = field(default_factory=lambda: slice(None), repr=False, compare=False)
  geom_idx: object = field(default_factory=lambda: slice(None), repr=False, compare=False)
  site_idx: object = field(default_factory=lambda: slice(None), repr=False, compare=False)

  def resolve(self, scene) -> None:
    ent = scene[self.name]
    for names_attr, ids_attr, find, num in _FIELDS:
      names = getattr(self, names_attr)
      ids = getattr(self, ids_attr)
      if names is None and not isinstance(ids, list):
        continue
      if isinstance(names, str):
        names = [names]
      elif isinstance(names, tuple):
        names = list(names)
      if names is not None:
        setattr(self, names_attr, names)
        found, _ = getattr(ent, find)(names, preserve_order=self.preserve_order)
        if len(found) == getattr(ent, num) and found == list(range(len(found))) and not isinstance(ids, list):
          setattr(self, ids_attr, slice(None))
        else:
          setattr(self, ids_attr, found)
      elif isinstance(ids, list):
        all_names = getattr(ent, names_attr)
        setattr(self, names_attr, [all_names[i] for i in ids])
    import torch

    for _, ids_attr, _, _ in _FIELDS:
      ids = getattr(self, ids_attr)
      if isinstance(ids, slice):
        idx = slice(None)
      elif len(ids) > 0 and list(ids) == list(range(ids[0], ids[0] + len(ids))):
        idx = slice(ids[0], ids[0] + len(ids))  # a contiguous range: reads are views, no gather launch
      elif len(ids) > 1 and ids[1] > ids[0] and list(ids) == list(range(ids[0], ids[-1] + 1, ids[1] - ids[0])):
        # an increasing arithmetic progression (e.g. two feet): a strided view, no gather launch
        idx = slice(ids[0], ids[-1] + 1, ids[1] - ids[0])
      else:
        idx = torch.tensor(ids, dtype=torch.long, device=scene.device)
      setattr(self, ids_attr.replace("_ids", "_idx"), idx)
