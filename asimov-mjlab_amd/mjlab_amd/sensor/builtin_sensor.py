"""Builtin sensors: views into ``sensordata`` (``src/mjlab/sensor/builtin_sensor.py:264-340``)."""

from __future__ import annotations

import torch


class BuiltinSensor:
  def __init__(self, cfg=None, name: str | None = None) -> None:
    self.cfg = cfg
    self._name = cfg.name if cfg is not None else name
    self._data = None
    self._data_view: torch.Tensor | None = None

  @classmethod
  def from_existing(cls, name: str) -> "BuiltinSensor":
    return cls(cfg=None, name=name)

  def edit_spec(self, scene_spec, entities) -> None:
    del scene_spec, entities

  def initialize(self, model, sim_model, data, device: str) -> None:
    del sim_model, device
    self._data = data
    s = model.sensor(self._name)
    a, d = int(s.adr[0]), int(s.dim[0])
    self._data_view = data.sensordata[:, a : a + d]

  @property
  def data(self) -> torch.Tensor:
    assert self._data_view is not None
    return self._data_view

  def reset(self, env_ids=None) -> None:
    del env_ids

  def update(self, dt: float) -> None:
    del dt
