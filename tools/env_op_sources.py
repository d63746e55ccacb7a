"""Aten ops of given kinds in one env-step body with their mjlab_amd call stacks (diagnostic tool).
usage: python tools/env_op_sources.py <task> <op,op,...> [device]"""
import sys, traceback
from collections import Counter
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd")); sys.path.insert(0, str(ROOT))
import torch
from torch.utils._python_dispatch import TorchDispatchMode
from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg
from tests import oracle_sim
task = sys.argv[1]
dev = sys.argv[3] if len(sys.argv) > 3 else "cpu"
cfg = load_env_cfg(task); cfg.scene.num_envs = 64
if "Tracking" in task:
  import bench
  cfg.commands["motion"].motion_file = bench.synthetic_motion_file(dev)
env = ManagerBasedRlEnv(cfg, device=dev)
env.use_graph = False
if dev == "cpu":
  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
env.reset()
a = 2 * torch.rand(64, env.action_manager.total_action_dim, device=dev) - 1
for _ in range(2): env.step(a)
env.sim.step = lambda: None; env.sim.forward_gated = lambda g: None
env._action_in.copy_(a)
want = set(sys.argv[2].split(','))
c = Counter()
class M(TorchDispatchMode):
  def __torch_dispatch__(self, func, types, args=(), kwargs=None):
    n = func.__name__.split('.')[0]
    if n in want:
      st = [f"{fr.filename.split('mjlab_amd/')[-1]}:{fr.lineno}" for fr in traceback.extract_stack()[:-1] if "mjlab_amd" in fr.filename][-3:]
      c[(n, " <- ".join(reversed(st)))] += 1
    return func(*args, **(kwargs or {}))
with M():
  env._step_body()
print(sum(c.values()), "ops")
for k, v in c.most_common(60): print(v, k)
