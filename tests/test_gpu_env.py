"""The full env step on the GPU: graph capture, replay, resets, finiteness."""

import pytest
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.sim import native
from mjlab_amd.tasks import load_env_cfg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("task,adim", [("Mjlab-Velocity-Flat-Unitree-G1", 29), ("Mjlab-Velocity-Flat-Unitree-Go1", 12)])
def test_env_graph_rollout(task, adim):
  cfg = load_env_cfg(task)
  cfg.scene.num_envs = 256
  cfg.seed = 0
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  assert env.use_graph
  env.reset()
  g = torch.Generator(device="cuda:0").manual_seed(1)
  dones = 0
  for i in range(60):
    a = 2 * torch.rand(256, adim, device="cuda:0", generator=g) - 1
    obs, rew, term, trunc, extras = env.step(a)
    dones += int((term | trunc).sum())
  assert env._graph is not None
  assert torch.isfinite(obs["policy"]).all() and torch.isfinite(obs["critic"]).all() and torch.isfinite(rew).all()
  assert ((env.sim.data.flags & 4) == 0).all()
  assert (env.episode_length_buf <= 60).all()
  assert native.LIB_PATH.name.startswith("libmjh")
