"""Backends for the restated reference tests (TEST INFRASTRUCTURE ONLY).

The reference's boundary tests (``tests/test_entity_data.py``,
``test_entity.py``, ``test_contact_sensor.py``, ``test_builtin_sensor.py``,
``test_sim.py``, ``test_domain_randomization.py``) run against a real
``Simulation``. They are restated here to run on two backends:

* ``hip``: the product path — ``Simulation`` on ``cuda:0`` calling the HIP
  step library. Every ``step()`` / ``forward()`` is *shadowed* by the float64
  oracle from the same pre-state and compared with ``tests.scenes.compare_step``
  (the tolerances written there), so each qualitative reference assertion is
  backed by a per-step numeric check of the HIP path;
* ``oracle``: a CPU ``Simulation`` whose step/forward run the oracle
  (``tests/oracle_sim.py``), so the host logic of the same tests runs in the
  CPU suite.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from mjlab_amd.sim import Simulation
from oracle.oracle import INPUTS, Oracle
from tests import oracle_sim
from tests.scenes import compare_step

BACKENDS = [pytest.param("oracle", id="oracle"), pytest.param("hip", id="hip", marks=pytest.mark.gpu)]


def device_of(backend: str) -> str:
  return "cuda:0" if backend == "hip" else "cpu"


class Shadow:
  """Wrap sim.step/forward: run the oracle from the same pre-state and compare."""

  def __init__(self, sim: Simulation, skip: tuple[str, ...] = ()) -> None:
    self.sim = sim
    self.skip = skip
    self.nsteps = 0
    self.maxerr: dict[str, float] = {}
    self.int_mismatch_worlds = 0
    self._step, self._forward = sim.step, sim.forward
    sim.step = lambda keep_image=False: self._run(True)  # (eager: every step packs the image anyway)
    sim.forward = lambda: self._run(False)

  def _snapshot(self) -> dict:
    n = self.sim.num_envs
    return {f: self.sim._data_flat[f].detach().cpu().numpy().reshape(n, -1).copy() for f in INPUTS if f in self.sim._data_flat}

  def _run(self, integrate: bool) -> None:
    sim = self.sim
    n = sim.num_envs
    st = self._snapshot()
    (self._step if integrate else self._forward)()
    torch.cuda.synchronize()
    got = {k: v.detach().cpu().numpy().reshape(n, -1) for k, v in sim._data_flat.items()}
    ov = {f: sim._model_flat[f].detach().cpu().numpy() for f, s in sim._wstride.items() if s}
    ref = Oracle(sim.mj_model, "f64", overrides=ov).run(n, st, integrate=integrate, follow=got)
    rep = compare_step(got, ref, dt=float(sim.mj_model.timestep), skip=self.skip)
    self.nsteps += 1
    self.int_mismatch_worlds += len(rep["int_mismatch_worlds"])
    for k, v in rep["maxerr"].items():
      self.maxerr[k] = max(self.maxerr.get(k, 0.0), v)
    fails = [f for f in rep["failures"] if f.split(":")[0] not in self.skip]
    assert not fails, f"HIP vs oracle, call {self.nsteps} ({'step' if integrate else 'forward'}): {fails}"


def make_sim(num_envs: int, cfg, model, backend: str, shadow: bool = True, skip: tuple[str, ...] = ()) -> Simulation:
  """``Simulation(num_envs, cfg, model, device)`` on the requested backend.

  The reference's constructor runs ``mj_forward`` on the CPU data it uploads
  (``src/mjlab/sim/sim.py:111-112``); the HIP constructor launches a forward
  too, and the oracle backend runs one here, so derived fields are current."""
  sim = Simulation(num_envs=num_envs, cfg=cfg, model=model, device=device_of(backend))
  if backend == "oracle":
    oracle_sim.attach(sim, overrides_fields=())
    sim.forward()
  elif shadow:
    sim.shadow = Shadow(sim, skip)
  return sim


def expanded_fields_attach(sim) -> None:
  """Re-attach the oracle so per-world (expanded) model fields are honoured."""
  if not sim.use_cuda_graph:
    oracle_sim.attach(sim, overrides_fields=tuple(f for f, s in sim._wstride.items() if s))


def as_np(t: torch.Tensor) -> np.ndarray:
  return t.detach().cpu().numpy()
