"""Torch views of the batched model/data buffers (the WarpBridge analogue).

Restates the contract of ``src/mjlab/sim/sim_data.py``: attribute access
returns torch tensors that alias the device buffers the kernels read/write
(zero-copy, in-place writable), and rebinding an attribute is forbidden
because captured graphs hold the raw pointers (``sim_data.py:217-223``).
Shapes follow MuJoCo Warp's arrays: world-outermost, vectors/matrices
unflattened (``xpos (N, nbody, 3)``, ``xmat (N, nbody, 3, 3)``).
"""

from __future__ import annotations

from types import SimpleNamespace

import torch

# per-world view shapes (size names resolved at bind time)
DATA_SHAPES: dict[str, tuple] = {
  "qpos": ("nq",),
  "qvel": ("nv",),
  "act": ("na",),
  "qacc_warmstart": ("nv",),
  "ctrl": ("nu",),
  "qfrc_applied": ("nv",),
  "xfrc_applied": ("nbody", 6),
  "mocap_pos": ("nmocap", 3),
  "mocap_quat": ("nmocap", 4),
  "time": (),
  "qacc": ("nv",),
  "qacc_smooth": ("nv",),
  "xpos": ("nbody", 3),
  "xquat": ("nbody", 4),
  "xmat": ("nbody", 3, 3),
  "xipos": ("nbody", 3),
  "ximat": ("nbody", 3, 3),
  "xanchor": ("njnt", 3),
  "xaxis": ("njnt", 3),
  "geom_xpos": ("ngeom", 3),
  "geom_xmat": ("ngeom", 3, 3),
  "site_xpos": ("nsite", 3),
  "site_xmat": ("nsite", 3, 3),
  "subtree_com": ("nbody", 3),
  "cvel": ("nbody", 6),
  "cacc": ("nbody", 6),
  "actuator_force": ("nu",),
  "actuator_length": ("nu",),
  "actuator_velocity": ("nu",),
  "qfrc_bias": ("nv",),
  "qfrc_passive": ("nv",),
  "qfrc_actuator": ("nv",),
  "qfrc_smooth": ("nv",),
  "qfrc_constraint": ("nv",),
  "sensordata": ("nsensordata",),
  "ncon": (),
  "contact_dist": ("nconmax",),
  "contact_pos": ("nconmax", 3),
  "contact_frame": ("nconmax", 3, 3),
  "contact_friction": ("nconmax", 5),
  "contact_includemargin": ("nconmax",),
  "contact_dim": ("nconmax",),
  "contact_geom": ("nconmax", 2),
  "contact_efc_address": ("nconmax",),
  "nefc": (),
  "efc_type": ("njmax",),
  "efc_id": ("njmax",),
  "efc_pos": ("njmax",),
  "efc_D": ("njmax",),
  "efc_aref": ("njmax",),
  "efc_force": ("njmax",),
  "solver_niter": (),
  "flags": (),
  "flags_acc": (),
  "solver_lstrace": (3,),
}

MODEL_SHAPES: dict[str, tuple] = {
  "body_pos": ("nbody", 3),
  "body_quat": ("nbody", 4),
  "body_ipos": ("nbody", 3),
  "body_iquat": ("nbody", 4),
  "body_mass": ("nbody",),
  "body_inertia": ("nbody", 3),
  "body_invweight0": ("nbody", 2),
  "jnt_range": ("njnt", 2),
  "jnt_stiffness": ("njnt",),
  "jnt_pos": ("njnt", 3),
  "jnt_axis": ("njnt", 3),
  "jnt_solref": ("njnt", 2),
  "jnt_solimp": ("njnt", 5),
  "dof_solref": ("nv", 2),
  "dof_solimp": ("nv", 5),
  "dof_armature": ("nv",),
  "dof_damping": ("nv",),
  "dof_frictionloss": ("nv",),
  "geom_pos": ("ngeom", 3),
  "geom_quat": ("ngeom", 4),
  "geom_friction": ("ngeom", 3),
  "geom_rgba": ("ngeom", 4),
  "geom_size": ("ngeom", 3),
  "geom_solref": ("ngeom", 2),
  "geom_solimp": ("ngeom", 5),
  "site_pos": ("nsite", 3),
  "site_quat": ("nsite", 4),
  "qpos0": ("nq",),
  "actuator_gainprm": ("nu", 10),
  "actuator_biasprm": ("nu", 10),
  "actuator_ctrlrange": ("nu", 2),
  "actuator_forcerange": ("nu", 2),
}
# static fields exposed with a leading world dim of 1 (batched in MuJoCo Warp)
BATCHED_STATIC = {"actuator_gainprm", "actuator_biasprm", "actuator_ctrlrange", "actuator_forcerange"}


def shape_of(spec: tuple, sizes: dict[str, int]) -> tuple[int, ...]:
  return tuple(sizes[s] if isinstance(s, str) else s for s in spec)


class Epoch:
  """Monotonic counter bumped whenever the sim data changes (step, forward,
  state writes). Derived-quantity caches (EntityData, ContactSensor) key on
  it; it is host state, so a captured graph replays the same cache hits."""

  __slots__ = ("v",)

  def __init__(self) -> None:
    self.v = 0

  def bump(self) -> None:
    self.v += 1


class Bridge:
  """Read-only attribute namespace over torch tensors (pointer-stable)."""

  def __init__(self, views: dict[str, torch.Tensor], extra: dict | None = None, nworld: int | None = None) -> None:
    object.__setattr__(self, "_views", views)
    object.__setattr__(self, "_extra", extra or {})
    object.__setattr__(self, "nworld", nworld)

  def __getattr__(self, name: str):
    views = object.__getattribute__(self, "_views")
    if name in views:
      return views[name]
    extra = object.__getattribute__(self, "_extra")
    if name in extra:
      return extra[name]
    raise AttributeError(f"'{name}' is not available on this bridge")

  def __setattr__(self, name: str, value) -> None:
    raise AttributeError(
      f"Cannot set attribute '{name}': buffers are pointer-stable (captured graphs hold them). "
      f"Write in place instead, e.g. sim.data.{name}[:] = value"
    )

  def _rebind(self, name: str, t: torch.Tensor) -> None:
    object.__getattribute__(self, "_views")[name] = t

  def fields(self) -> list[str]:
    return list(object.__getattribute__(self, "_views"))


def make_opt(model, cfg) -> SimpleNamespace:
  return SimpleNamespace(
    timestep=torch.tensor([model.timestep], dtype=torch.float32),
    gravity=torch.tensor([list(model.gravity)], dtype=torch.float32),
    impratio=torch.tensor([model.impratio], dtype=torch.float32),
    tolerance=torch.tensor([model.tolerance], dtype=torch.float32),
    ls_tolerance=torch.tensor([model.ls_tolerance], dtype=torch.float32),
    iterations=model.iterations,
    ls_iterations=model.ls_iterations,
    integrator=model.integrator,
    cone=model.cone,
    solver=model.solver,
    ls_parallel=cfg.ls_parallel,
    contact_sensor_maxmatch=cfg.contact_sensor_maxmatch,
  )
