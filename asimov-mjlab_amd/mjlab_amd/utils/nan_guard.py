"""NaN guard (``src/mjlab/utils/nan_guard.py``); implemented next to the
Simulation it watches (mjlab_amd/sim/sim.py)."""

from mjlab_amd.sim.sim import NanGuard, NanGuardCfg

__all__ = ["NanGuard", "NanGuardCfg"]
