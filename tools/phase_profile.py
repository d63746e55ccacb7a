"""Per-phase cycle breakdown of the step kernel (diagnostic build libmjh_prof.so).

Run: MJH_LIB=asimov-mjlab_amd/mjlab_amd/libmjh_prof.so python tools/phase_profile.py [N]
Stamps are s_memtime (shader clock) at phase boundaries, lane 0 of each world.
"""

import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("MJH_LIB", str(ROOT / "asimov-mjlab_amd/mjlab_amd/libmjh_prof.so"))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT / "tools"))

import numpy as np
import torch

sys.path.insert(0, str(ROOT))
from tests.scenes import g1_scene, random_states
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg, native

NAMES = ["kinematics", "com/crb/M/factor", "collision", "constraints", "rne/smooth/qacc_smooth", "solver",
         "cacc+sensors", "outputs", "integration"]
PHASES = [(0, 1), (1, 2), (2, 4), (4, 5), (5, 3), (3, 6), (6, 7), (7, 8), (8, 9)]

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sc = g1_scene(N)
m = sc.compile(50, 300)
cfg = SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20),
                    ls_parallel=os.environ.get("MJH_LS_PARALLEL", "1") == "1")
buf = torch.zeros(N * 32, dtype=torch.int64, device="cuda:0")
L = native.lib()
L.mjh_set_profile_buffer.argtypes = [ctypes.c_void_p]
assert L.mjh_set_profile_buffer(ctypes.c_void_p(buf.data_ptr())) == 0  # before any launch
torch.cuda.synchronize()
sim = Simulation(N, cfg, m, "cuda:0")
rng = np.random.default_rng(0)
st = random_states(m, N, rng, drop=0.03)
for k, v in st.items():
  getattr(sim.data, k)[:] = torch.as_tensor(v, dtype=torch.float32, device="cuda:0").view_as(getattr(sim.data, k))
for _ in range(int(os.environ.get("SETTLE", "20"))):
  sim.step()
torch.cuda.synchronize()
p = buf.view(N, 32).cpu().numpy().astype(np.int64)
tot = p[:, 9] - p[:, 0]
print(f"N={N} ls_parallel={int(cfg.ls_parallel)} mean total cycles/world-step: {tot.mean():.0f} (max {tot.max()})")
# the launch as a whole: span from the first world's start to the last world's
# end (shader clock), and when worlds start (late starts = a second round)
st0 = p[:, 0] - p[:, 0].min()
print(f"  launch span {(p[:, 9].max() - p[:, 0].min()):.0f} cycles; world start p50 {np.percentile(st0, 50):.0f} "
      f"p90 {np.percentile(st0, 90):.0f} max {st0.max():.0f}; world cycles p50 {np.percentile(tot, 50):.0f} "
      f"p90 {np.percentile(tot, 90):.0f} p99 {np.percentile(tot, 99):.0f} max {tot.max():.0f}")
# phase stamps in execution order: the position stage (kinematics .. constraint
# rows) runs before the velocity stage (rne / smooth forces / qacc_smooth)
for n, (a, b) in zip(NAMES, PHASES):
  v = (p[:, b] - p[:, a]).mean()
  print(f"  {n:26s} {v:10.0f}  ({100*v/tot.mean():5.1f}%)")
print(f"  solver: linesearch {p[:,12].mean():.0f}  update {p[:,13].mean():.0f}  newton_dir {p[:,14].mean():.0f}")
print(f"    newton_dir parts: hessian {p[:,15].mean():.0f}  factor {p[:,16].mean():.0f}  solve {p[:,17].mean():.0f}")
print(f"  M factor alone: {(p[:,2]-p[:,10]).mean():.0f}  (com/crb/M before it: {(p[:,10]-p[:,1]).mean():.0f})")
def seg(a, b):
  return (p[:, b] - p[:, a]).mean()
print(f"  kinematics: bodies {seg(0,27):.0f} geoms {seg(27,28):.0f} sites {seg(28,1):.0f}")
print(f"  com: subtree+cinert {seg(1,18):.0f} cdof {seg(18,19):.0f} crb {seg(19,20):.0f} M-fill {seg(20,10):.0f} factor {seg(10,2):.0f}")
print(f"  cacc {seg(6,26):.0f}  contact/subtree/ft sensors {seg(26,11):.0f}  lane sensors {seg(11,7):.0f}")
print(f"  rne: cvel {seg(5,21):.0f} cdof_dot {seg(21,22):.0f} rne {seg(22,23):.0f} cfrc-sum+bias {seg(23,24):.0f} "
      f"passive/act/smooth {seg(24,25):.0f} qacc_smooth solve {seg(25,3):.0f}")
niter = sim.data.solver_niter.cpu().numpy()
nefc = sim.data.nefc.cpu().numpy()
wg = tot[: (N // 8) * 8].reshape(-1, 8)
print(f"  hessian+factor recomputations per world-step: {p[:, 29].mean():.2f}")
print(f"  workgroup (8 worlds) max/mean: {wg.max(1).mean():.0f} / {tot.mean():.0f}; "
      f"p50 {np.percentile(tot, 50):.0f} p90 {np.percentile(tot, 90):.0f} p99 {np.percentile(tot, 99):.0f}")
for nm, x in (("nefc", nefc), ("niter", niter)):
  print(f"  corr(total, {nm}) = {np.corrcoef(tot, x.reshape(-1).astype(np.float64))[0, 1]:.2f}")
srt = np.sort(tot)[: (N // 8) * 8].reshape(-1, 8)
print(f"  if sorted by true cost: workgroup max mean {srt.max(1).mean():.0f}")
print(f"  niter mean {niter.mean():.2f}  nefc mean {nefc.mean():.1f}  ncon mean {sim.data.ncon.float().mean().item():.1f}")

# cost predictability for load balancing: one more step, per-world cycles of
# step t+1 against predictors from step t
tot1 = tot.copy()
key1 = ((niter.reshape(-1).astype(np.int64) + 2) * nefc.reshape(-1).astype(np.int64))
sim.step()
torch.cuda.synchronize()
p2 = buf.view(N, 32).cpu().numpy().astype(np.int64)
tot2 = p2[:, 9] - p2[:, 0]
M8 = (N // 8) * 8


def wg_max(order):
  return tot2[order][:M8].reshape(-1, 8).max(1).mean()


print(f"  next step: corr(cycles_t, cycles_t+1) = {np.corrcoef(tot1, tot2)[0, 1]:.2f}; "
      f"workgroup max mean: identity {wg_max(np.arange(N)):.0f}, by prev cycles {wg_max(np.argsort(-tot1)):.0f}, "
      f"by prev (niter+2)*nefc {wg_max(np.argsort(-key1, kind='stable')):.0f}, by true cost {wg_max(np.argsort(-tot2)):.0f}")

# per-world data of the two steps for offline predictor studies
if os.environ.get("DUMP"):
  np.savez_compressed(os.environ["DUMP"], tot1=tot1, tot2=tot2, niter=niter.reshape(-1), nefc=nefc.reshape(-1),
                      ncon=sim.data.ncon.cpu().numpy().reshape(-1), niter2=sim.data.solver_niter.cpu().numpy().reshape(-1),
                      nefc2=sim.data.nefc.cpu().numpy().reshape(-1))
