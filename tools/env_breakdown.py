"""Split one env step's time into physics launches and the env layer (diagnostic tool)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
cfg.seed = 42
env = ManagerBasedRlEnv(cfg, device="cuda:0")
env.reset()
adim = env.action_manager.total_action_dim
g = torch.Generator(device="cuda:0").manual_seed(1)
act = torch.empty(n, adim, device="cuda:0")


def timeit(fn, k):
  torch.cuda.synchronize()
  t = time.perf_counter()
  for _ in range(k):
    fn()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / k * 1e3


def env_step():
  act.uniform_(-1, 1, generator=g)
  env.step(act)


for _ in range(30):
  env_step()
t_env = timeit(env_step, 100)
t_step = timeit(env.sim.step, 100)
gate = torch.ones(1, dtype=torch.bool, device="cuda:0")
t_fwd = timeit(lambda: env.sim.forward_gated(gate), 50)
dec = env.cfg.decimation
print(f"{task} N={n}: env step {t_env:.3f} ms = {dec} x physics {t_step:.3f} + forward {t_fwd:.3f} + env layer "
      f"{t_env - dec * t_step - t_fwd:.3f} ms  -> {n / t_env * 1e3:,.0f} env-steps/s "
      f"(nefc {env.sim.data.nefc.float().mean().item():.1f}, iters {env.sim.data.solver_niter.float().mean().item():.2f})")
