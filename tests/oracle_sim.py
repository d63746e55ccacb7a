"""CPU stand-in physics for env-layer tests (TEST INFRASTRUCTURE ONLY).

Replaces ``Simulation.step/forward/forward_gated`` of a CPU-device env with the
float64 oracle so the manager/env logic (masks, resets, rewards, graph-free
control flow) can be exercised without a GPU. Never used by the product path.
"""

from __future__ import annotations

import numpy as np
import torch

from oracle.oracle import INPUTS, Oracle


def attach(sim, overrides_fields=()) -> None:
  n = sim.num_envs
  state_fields = [f for f in INPUTS]

  def run(integrate: bool) -> None:
    sim.epoch.bump()
    ov = {f: getattr(sim.model, f).detach().cpu().numpy() for f in overrides_fields}
    orc = Oracle(sim.mj_model, "f64", overrides=ov)
    st = {}
    for f in state_fields:
      try:
        st[f] = getattr(sim.data, f).detach().cpu().numpy().reshape(n, -1)
      except AttributeError:
        pass
    out = orc.run(n, st, integrate=integrate)
    for f in sim.data.fields():
      if f in out:
        t = getattr(sim.data, f)
        if t.numel() == 0:
          continue
        t.copy_(torch.as_tensor(out[f].reshape(n, -1)[:, : t[0].numel()]).view_as(t).to(t.dtype))

  sim._require_gpu = lambda: None
  sim.step = lambda: run(True)
  sim.forward = lambda: run(False)

  def gated(gate):
    if bool(gate.any()):
      run(False)

  sim.forward_gated = gated
