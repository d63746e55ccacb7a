"""Call sites of the torch ops one eager env step runs on GPU tensors
(diagnostic, GPU box): a TorchDispatchMode records each aten op that is not a
view / metadata op, with the innermost mjlab_amd frame that issued it."""
import sys
import traceback
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import collections

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

SKIP = ("view", "select", "slice", "unsqueeze", "squeeze", "expand", "as_strided", "alias", "detach", "t.default",
        "transpose", "permute", "_to_copy", "empty", "lift_fresh", "reshape", "unbind", "split", "is_nonzero", "item",
        "_local_scalar_dense", "result_type", "set_")


class Sites(TorchDispatchMode):
  def __init__(self):
    super().__init__()
    self.c = collections.Counter()

  def __torch_dispatch__(self, func, types, args=(), kwargs=None):
    name = str(func)
    if not any(k in name for k in SKIP):
      fr = [f for f in traceback.extract_stack() if "mjlab_amd" in f.filename and "_python_dispatch" not in f.filename]
      site = f"{Path(fr[-1].filename).name}:{fr[-1].lineno} {fr[-1].name}" if fr else "?"
      self.c[(name, site)] += 1
    return func(*args, **(kwargs or {}))


task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
cfg = load_env_cfg(task)
cfg.scene.num_envs = 4096
env = ManagerBasedRlEnv(cfg, device="cuda:0")
env.reset()
act = torch.zeros(4096, env.action_manager.total_action_dim, device="cuda:0")
for _ in range(3):
  env._action_in.copy_(act)
  env._step_body()
torch.cuda.synchronize()
m = Sites()
with m:
  env._action_in.copy_(act)
  env._step_body()
torch.cuda.synchronize()
for (name, site), n in sorted(m.c.items(), key=lambda x: x[1], reverse=True):
  print(f"{n:3d}  {name:40s} {site}")
