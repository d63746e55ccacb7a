"""Kernel census of one captured env step (run under rocprofv3 --kernel-trace --stats).
Setup steps are eager; then exactly K graph replays, so per-step counts = calls / K
for kernels that only run inside the graph."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

K = 50
cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
cfg.scene.num_envs = 4096
env = ManagerBasedRlEnv(cfg, device="cuda:0")
env.reset()
a = torch.zeros(4096, 29, device="cuda:0")
for _ in range(3):
  env.step(a)
torch.cuda.synchronize()
for _ in range(K):
  env.step(a)
torch.cuda.synchronize()
print("done")
