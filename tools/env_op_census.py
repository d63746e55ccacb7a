"""Where the env layer's kernels come from (diagnostic tool, GPU box).

Profiles eager env-step bodies with torch.profiler (CPU+GPU, Python stacks) and
attributes GPU kernel time and launch counts to the first frame inside
mjlab_amd that is not a generic helper, so the next fusion targets are visible.
usage: python tools/env_op_census.py [task] [N]
"""
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import torch
from torch.profiler import ProfilerActivity, profile

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
if "Tracking" in task:
  sys.path.insert(0, str(ROOT))
  import bench

  cfg.commands["motion"].motion_file = bench.synthetic_motion_file("cuda:0")
env = ManagerBasedRlEnv(cfg, device="cuda:0")
env.use_graph = False
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(0)
env.episode_length_buf.random_(0, int(env.max_episode_length), generator=g)  # steady state: resets every step
a = 2 * torch.rand(n, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
for _ in range(3):
  env.step(a)
env._action_in.copy_(a)
sim = env.sim
phys = (sim.step, sim.forward_gated)
sim.step = lambda: None  # physics excluded: the env layer only
sim.forward_gated = lambda g: None
torch.cuda.synchronize()
K = 5
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
  for _ in range(K):
    env._step_body()
  torch.cuda.synchronize()
sim.step, sim.forward_gated = phys

SKIP = ("envops.py", "utils/math.py", "manager_base.py", "functional.py", "_tensor.py")
print(f"{task} N={n}: " + ", ".join(
  f"{k.name if hasattr(k, 'name') else k}" for k in []))
tot_k = 0
for ev in prof.events():
  if ev.device_type == torch.autograd.DeviceType.CPU and ev.kernels:
    tot_k += len(ev.kernels)
tot_t = sum(k.duration for ev in prof.events() if ev.device_type == torch.autograd.DeviceType.CPU for k in ev.kernels)
print(f"  env layer: {tot_k / K:.0f} kernels/step, {tot_t / K / 1e3:.3f} ms GPU time/step (eager, physics excluded)")

# attribution: torch calls per source line (a torch op launches ~1 kernel; fused
# envops kernels are ctypes calls and appear through their output allocation)
import traceback
from torch.overrides import TorchFunctionMode

counts = defaultdict(int)


class Census(TorchFunctionMode):
  def __torch_function__(self, func, types, args=(), kwargs=None):
    name = getattr(func, "__name__", str(func))
    if name not in ("__get__", "size", "dim", "stride", "data_ptr", "is_contiguous", "numel", "__len__", "view", "reshape",
                    "__getitem__", "expand", "unsqueeze", "squeeze", "t", "transpose", "permute", "contiguous"):
      loc = "?"
      for fr in reversed(traceback.extract_stack()[:-1]):
        f = fr.filename
        if "mjlab_amd" in f and not any(x in f for x in SKIP):
          loc = f"{f.split('mjlab_amd/')[-1]}:{fr.lineno} {fr.name}"
          break
      counts[loc] += 1
    return func(*args, **(kwargs or {}))


sim.step = lambda: None
sim.forward_gated = lambda g: None
with Census():
  env._step_body()
sim.step, sim.forward_gated = phys
print(f"  torch calls in one step body: {sum(counts.values())}")
for loc, c in sorted(counts.items(), key=lambda kv: -kv[1])[:90]:
  print(f"  {c:5d}  {loc}")
