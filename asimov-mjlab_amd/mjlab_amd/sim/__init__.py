from mjlab_amd.sim.sim import MujocoCfg, NanGuardCfg, Simulation, SimulationCfg, detect_nans

__all__ = ["MujocoCfg", "NanGuardCfg", "Simulation", "SimulationCfg", "detect_nans"]
