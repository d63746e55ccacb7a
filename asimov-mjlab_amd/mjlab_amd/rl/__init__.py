from mjlab_amd.rl.vecenv_wrapper import ObsDict, RslRlVecEnvWrapper

__all__ = ["ObsDict", "RslRlVecEnvWrapper"]
