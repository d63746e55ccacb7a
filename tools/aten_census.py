"""Which torch (aten) kernels one eager env step launches besides the fused HIP
kernels (diagnostic, GPU box): the env step body under torch.profiler, CUDA
kernels grouped by name with the Python call site that issued them."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import collections

import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

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
from torch.profiler import ProfilerActivity, profile

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
  env._action_in.copy_(act)
  env._step_body()
  torch.cuda.synchronize()
cnt = collections.Counter()
sites = collections.defaultdict(collections.Counter)
for e in prof.events():
  if e.device_type == torch.autograd.DeviceType.CPU and e.name.startswith("aten::") and e.stack:
    frames = [f for f in e.stack if "mjlab_amd" in f and "torch/" not in f]
    site = frames[0] if frames else (e.stack[0] if e.stack else "?")
    sites[e.name][site] += 1
kern = collections.Counter()
for e in prof.events():
  if e.device_type == torch.autograd.DeviceType.CUDA:
    kern[e.name[:80]] += 1
print("device kernels in one eager env step:", sum(kern.values()))
for k, v in kern.most_common(80):
  print(f"{v:4d}  {k}")
print("\naten ops by call site (those that may launch kernels):")
for name, c in sorted(sites.items(), key=lambda x: -sum(x[1].values())):
  if name in ("aten::empty", "aten::empty_strided", "aten::view", "aten::as_strided", "aten::reshape", "aten::select",
              "aten::slice", "aten::unsqueeze", "aten::squeeze", "aten::expand", "aten::t", "aten::transpose",
              "aten::detach", "aten::alias", "aten::lift_fresh", "aten::resolve_conj", "aten::resolve_neg", "aten::item",
              "aten::_local_scalar_dense", "aten::result_type", "aten::is_nonzero", "aten::to", "aten::_to_copy"):
    continue
  for site, n in c.most_common(4):
    print(f"{n:3d} {name:28s} {site}")
