"""Distribution of constraint-row counts (nefc) per world in the steady-state bench
workload (diagnostic, GPU box): sizes the LDS-resident row capacity of the step
kernel. usage: python tools/nefc_hist.py [task] [N] [steps]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import numpy as np
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 300
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
env = ManagerBasedRlEnv(cfg, device="cuda:0")
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(1234)
env.episode_length_buf.copy_(torch.randint(0, int(env.max_episode_length), (n,), device="cuda:0", generator=g))
adim = env.action_manager.total_action_dim
hist = torch.zeros(512, dtype=torch.long, device="cuda:0")
for k in range(steps):
  env.step(2 * torch.rand(n, adim, device="cuda:0", generator=g) - 1)
  if k >= 50:
    hist += torch.bincount(env.sim.data.nefc.view(-1).long().clamp(max=511), minlength=512)
h = hist.cpu().numpy()
c = np.cumsum(h) / h.sum()
pct = {p: int(np.searchsorted(c, p)) for p in (0.5, 0.9, 0.99, 0.999, 0.9999)}
print(f"{task} N={n} world-steps={h.sum()} mean={np.dot(np.arange(512), h) / h.sum():.1f} percentiles {pct} max={int(np.nonzero(h)[0].max())}")
for t in (48, 64, 80, 96, 112, 128, 160):
  print(f"  > {t}: {h[t + 1:].sum() / h.sum():.2e}")
