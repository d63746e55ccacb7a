"""Aten-op census of one eager env-step body by source line (diagnostic tool).

Counts the aten ops (≈ kernel launches; views excluded) that one env-step body
issues, attributed to the first mjlab_amd frame outside the generic helpers.
Physics is excluded. On cpu the oracle stands in for the physics (tests/oracle_sim.py).
usage: python tools/env_aten_census.py [task] [device] [N]
"""
import sys
import traceback
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import torch
from torch.utils._python_dispatch import TorchDispatchMode

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
dev = sys.argv[2] if len(sys.argv) > 2 else "cpu"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 64
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
if "Tracking" in task:
  import bench

  cfg.commands["motion"].motion_file = bench.synthetic_motion_file(dev)
env = ManagerBasedRlEnv(cfg, device=dev)
if dev == "cpu":
  from tests import oracle_sim

  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
env.use_graph = False
env.reset()
env.episode_length_buf.random_(0, int(env.max_episode_length))
a = 2 * torch.rand(n, env.action_manager.total_action_dim, device=dev) - 1
for _ in range(3):
  env.step(a)
sim = env.sim
sim.step = lambda: None
sim.forward_gated = lambda g: None
env._action_in.copy_(a)
VIEW = {"view", "_unsafe_view", "expand", "select", "slice", "unsqueeze", "squeeze", "t", "transpose", "permute",
        "alias", "as_strided", "detach", "_reshape_alias", "unbind", "split", "lift_fresh", "reshape", "empty", "empty_like",
        "empty_strided", "_local_scalar_dense"}
SKIP = ("utils/math.py", "envops.py", "manager_base.py")
counts, names = defaultdict(int), defaultdict(int)


class Census(TorchDispatchMode):
  def __torch_dispatch__(self, func, types, args=(), kwargs=None):
    nm = func.__name__.split(".")[0]
    if nm not in VIEW:
      loc = "?"
      for fr in reversed(traceback.extract_stack()[:-1]):
        if "mjlab_amd" in fr.filename and not any(s in fr.filename for s in SKIP):
          loc = f"{fr.filename.split('mjlab_amd/')[-1]}:{fr.lineno} {fr.name}"
          break
      counts[loc] += 1
      names[nm] += 1
    return func(*args, **(kwargs or {}))


with Census():
  env._step_body()
print(f"{task} {dev} N={n}: {sum(counts.values())} aten ops in one env-step body (physics excluded)")
for k, v in sorted(counts.items(), key=lambda x: -x[1])[:80]:
  print(f"{v:4d} {k}")
print(sorted(names.items(), key=lambda x: -x[1])[:40])
