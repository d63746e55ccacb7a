"""NaN guard (``src/mjlab/utils/nan_guard.py``): the guard lives next to the
Simulation it watches (mjlab_amd/sim/sim.py); this module keeps the
reference's import path and adds the dump reader."""

from __future__ import annotations

from pathlib import Path

import numpy as np

from mjlab_amd.sim.sim import NanGuard, NanGuardCfg

__all__ = ["NanGuard", "NanGuardCfg", "load_nan_dump"]


def load_nan_dump(path: str | Path) -> tuple[dict, dict[int, np.ndarray], Path]:
  """Read a NaN dump the way ``scripts/nan_viz.py:29-45`` does: the metadata
  dict (``_metadata.item()``), the buffered mjSTATE_PHYSICS states by step, and
  the model file next to it (MJCF here: ``MjModel.from_xml_path`` loads it).
  The dump is this build's own file (its metadata is a pickled dict, as the
  reference writes it)."""
  path = Path(path)
  z = np.load(path, allow_pickle=True)
  meta = z["_metadata"].item()
  keys = sorted((k for k in z.files if k.startswith("states_step_")), key=lambda k: int(k.split("_")[-1]))
  states = {int(k.split("_")[-1]): z[k] for k in keys}
  return meta, states, path.parent / meta["model_file"]
