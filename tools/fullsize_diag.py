"""Diagnostics: the full-size G1 env sample of tests/test_gpu_fullsize.py, with
per-world solver agreement (follow-mode excess, iterations, warm-start choice,
qacc/qvel errors) for the worst worlds."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv  # noqa: E402
from mjlab_amd.tasks import load_env_cfg  # noqa: E402
from oracle.oracle import INPUTS, Oracle  # noqa: E402
from tests.scenes import compare_step  # noqa: E402

DEV = "cuda:0"
task, n = "Mjlab-Velocity-Flat-Unitree-G1", 4096
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
cfg.seed = 42
env = ManagerBasedRlEnv(cfg, device=DEV)
env.reset()
adim = env.action_manager.total_action_dim
g = torch.Generator(device=DEV).manual_seed(1234)
env.episode_length_buf.random_(0, int(env.max_episode_length), generator=g)
for _ in range(30):
  env.step(2 * torch.rand(n, adim, device=DEV, generator=g) - 1)
torch.cuda.synchronize()
sim = env.sim
idx = torch.randperm(n, generator=torch.Generator().manual_seed(0))[:64].sort().values.numpy()
state = {f: getattr(sim.data, f).detach().cpu().numpy().reshape(n, -1)[idx] for f in INPUTS if getattr(sim.data, f).numel()}
ov = {f: getattr(sim.model, f).detach().cpu().numpy()[idx] for f in env.event_manager.domain_randomization_fields
      if getattr(sim.model, f).shape[0] == n}
sim.step()
torch.cuda.synchronize()
got = {k: getattr(sim.data, k).detach().cpu().numpy().reshape(n, -1)[idx] for k in sim.data.fields()}
orc = Oracle(sim.mj_model, overrides=ov)
fol = orc.run(len(idx), state, integrate=True, follow=got)
free = orc.run(len(idx), state, integrate=True)
rep = compare_step(got, fol)
print("failures", rep["failures"])
print("capped", rep["capped_worlds"])


def rel(a, b):
  return np.abs(a - b).max(1) / (1 + np.abs(b).max(1))


dq = rel(got["qacc"], fol["qacc"])
dv = np.abs(got["qvel"] - fol["qvel"]).max(1)
for w in np.argsort(-dv)[:8]:
  print(f"w{w}: qvel d {dv[w]:.2e} qacc rel {dq[w]:.2e} excess {fol['ls_excess'][w, 0]:.2e} niter gpu {got['solver_niter'][w, 0]} "
        f"free {free['solver_niter'][w, 0]} warm gpu {(got['solver_lstrace'][w, 0] >> 30) & 1} free {(free['solver_lstrace'][w, 0] >> 30) & 1} "
        f"nefc {got['nefc'][w, 0]} capped {fol['solver_capped'][w, 0]} free-vs-gpu qacc rel {rel(got['qacc'], free['qacc'])[w]:.2e}")
ex = fol["ls_excess"][:, 0]
print("excess quantiles", np.quantile(ex, [0.5, 0.9, 0.99, 1.0]))
# the sample's inputs and the device outputs, for offline analysis with the oracle
np.savez_compressed(ROOT / "gpurun_out" / "r03m" / "fs_sample.npz",
                    **{"in_" + k: v for k, v in state.items()}, **{"ov_" + k: v for k, v in ov.items()},
                    **{"got_" + k: got[k] for k in ("qacc", "qvel", "qpos", "actuator_force", "qfrc_constraint",
                                                    "qfrc_smooth", "solver_niter", "solver_lstrace", "nefc")})
