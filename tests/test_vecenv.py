"""RSL-RL VecEnv contract (restates src/mjlab/rl/vecenv_wrapper.py:68-95) on CPU with oracle physics."""

import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.rl import RslRlVecEnvWrapper
from mjlab_amd.tasks import load_env_cfg
from tests import oracle_sim


def test_wrapper_contract():
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 4
  env = ManagerBasedRlEnv(cfg, device="cpu")
  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
  w = RslRlVecEnvWrapper(env, clip_actions=1.0)
  assert w.num_envs == 4 and w.num_actions == 29 and w.max_episode_length == 1000
  obs = w.get_observations()
  assert set(obs) == {"policy", "critic"} and obs.batch_size == [4]
  o, r, d, ex = w.step(torch.full((4, 29), 5.0))
  assert d.dtype == torch.long and r.shape == (4,) and "time_outs" in ex
  assert torch.allclose(env.action_manager.action, torch.ones(4, 29))  # clipped
  assert w.action_space.high == 1.0
