"""Kernel launches and GPU time per env-step phase (eager, steady state, GPU box).

Each manager call of ManagerBasedRlEnv._step_body runs inside a
torch.profiler.record_function range; kernels are attributed to the innermost
range. usage: python tools/env_phase_census.py [task] [N]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import torch
from torch.profiler import ProfilerActivity, profile, record_function

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.tasks import load_env_cfg

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
if "Tracking" in task:
  import bench

  cfg.commands["motion"].motion_file = bench.synthetic_motion_file("cuda:0")
env = ManagerBasedRlEnv(cfg, device="cuda:0", use_graph=False)
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(0)
env.episode_length_buf.random_(0, int(env.max_episode_length), generator=g)
a = 2 * torch.rand(n, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
for _ in range(5):
  env.step(a)
torch.cuda.synchronize()


def wrap(obj, name, label):
  f = getattr(obj, name)

  def w(*args, **kw):
    with record_function(label):
      return f(*args, **kw)

  setattr(obj, name, w)


wrap(env.action_manager, "process_action", "1 action.process")
wrap(env.action_manager, "apply_action", "2 action.apply")
wrap(env.scene, "write_data_to_sim", "3 scene.write")
wrap(env.sim, "step", "4 sim.step")
wrap(env.scene, "update", "5 scene.update")
wrap(env.termination_manager, "compute", "6 terminations")
wrap(env.reward_manager, "compute", "7 rewards")
wrap(env, "_reset_idx", "8 reset_idx")
wrap(env.sim, "forward_gated", "9 forward")
wrap(env.command_manager, "compute", "A commands")
wrap(env.event_manager, "apply", "B events")
wrap(env.observation_manager, "compute", "C observations")
env._action_in.copy_(a)
K = 5
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
  for _ in range(K):
    with record_function("0 step_body"):
      env._step_body()
  torch.cuda.synchronize()
stats = {}
for ev in prof.events():
  if ev.device_type == torch.autograd.DeviceType.CPU and ev.kernels:
    # innermost enclosing labelled range
    p, lab = ev, "0 step_body"
    while p is not None:
      if p.name[:2] in {f"{c} " for c in "0123456789ABC"}:
        lab = p.name
        break
      p = p.cpu_parent
    s = stats.setdefault(lab, [0, 0.0])
    s[0] += len(ev.kernels)
    s[1] += sum(k.duration for k in ev.kernels)
tk = sum(v[0] for v in stats.values()) / K
tt = sum(v[1] for v in stats.values()) / K
print(f"{task} N={n}: {tk:.0f} kernels/step, {tt / 1e3:.3f} ms GPU time/step (eager)")
for lab in sorted(stats):
  c, t = stats[lab]
  print(f"  {lab:22s} {c / K:6.1f} kernels  {t / K / 1e3:7.3f} ms")
