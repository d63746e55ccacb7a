"""Kernel census of one captured env step (run under rocprofv3 --kernel-trace --stats).

Steady state: random actions, episode lengths start uniform (resets and the
gated forward fire as in the bench). Setup steps are eager; then exactly K
graph replays, so per-step counts = calls / K for kernels that only run inside
the graph. usage: python tools/env_kernel_census.py [task] [N] [K]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
K = int(sys.argv[3]) if len(sys.argv) > 3 else 50
cfg = load_env_cfg(task)
cfg.scene.num_envs = N
env = ManagerBasedRlEnv(cfg, device="cuda:0")
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(0)
env.episode_length_buf.random_(0, int(env.max_episode_length), generator=g)
adim = env.action_manager.total_action_dim
acts = [2 * torch.rand(N, adim, device="cuda:0", generator=g) - 1 for _ in range(4)]
for i in range(3):
  env.step(acts[i % 4])
torch.cuda.synchronize()
for i in range(K):
  env.step(acts[i % 4])
torch.cuda.synchronize()
print("done", K)
