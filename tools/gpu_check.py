"""Quick GPU-vs-oracle comparison on the G1 velocity scene (diagnostic tool)."""

import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

from mjlab_amd.asset_zoo.g1 import get_g1_robot_cfg
from mjlab_amd.scene.scene import Scene, SceneCfg, TerrainImporterCfg
from mjlab_amd.sensor import ContactMatch, ContactSensorCfg
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
from oracle.oracle import Oracle


def g1_scene(num_envs):
  feet = ContactSensorCfg(
    name="feet_ground_contact",
    primary=ContactMatch(mode="subtree", pattern=r"^(left_ankle_roll_link|right_ankle_roll_link)$", entity="robot"),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found", "force"), reduce="netforce", num_slots=1, track_air_time=True)
  selfc = ContactSensorCfg(
    name="self_collision", primary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    secondary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"), fields=("found",), reduce="none", num_slots=1)
  return Scene(SceneCfg(num_envs=num_envs, terrain=TerrainImporterCfg(), entities={"robot": get_g1_robot_cfg()}, sensors=(feet, selfc)), "cpu")


def random_states(m, n, rng):
  qpos = np.tile(m.key_qpos, (n, 1))
  qpos[:, 2] += rng.uniform(-0.06, 0.02, n)
  yaw = rng.uniform(-np.pi, np.pi, n)
  qpos[:, 3] = np.cos(yaw / 2)
  qpos[:, 6] = np.sin(yaw / 2)
  qpos[:, 7:] += rng.uniform(-0.15, 0.15, (n, m.nq - 7))
  qvel = rng.normal(0, 0.3, (n, m.nv))
  ctrl = np.tile(m.key_ctrl, (n, 1)) + rng.uniform(-0.3, 0.3, (n, m.nu))
  return {"qpos": qpos, "qvel": qvel, "ctrl": ctrl}


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
  sc = g1_scene(N)
  m = sc.compile(50, 300)
  cfg = SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20))
  sim = Simulation(N, cfg, m, "cuda:0")
  rng = np.random.default_rng(0)
  st = random_states(m, N, rng)
  for k, v in st.items():
    getattr(sim.data, k)[:] = torch.as_tensor(v, dtype=torch.float32, device="cuda:0").view_as(getattr(sim.data, k))
  torch.cuda.synchronize()
  sim.step()
  torch.cuda.synchronize()
  out = {k: getattr(sim.data, k).detach().cpu().numpy().reshape(N, -1) for k in sim.data.fields()}
  orc = Oracle(m)
  ref = orc.run(N, st, integrate=True)
  print("ncon gpu", out["ncon"][:8].ravel(), "ref", ref["ncon"][:8].ravel())
  print("nefc gpu", out["nefc"][:8].ravel(), "ref", ref["nefc"][:8].ravel())
  print("niter gpu", out["solver_niter"][:8].ravel(), "ref", ref["solver_niter"][:8].ravel())
  print("flags gpu", np.unique(out["flags"]), "ref", np.unique(ref["flags"]))
  for k in ["xpos", "xquat", "xmat", "subtree_com", "cvel", "geom_xpos", "site_xpos", "qfrc_bias", "qfrc_actuator",
            "qfrc_smooth", "qacc_smooth", "qacc", "qfrc_constraint", "qvel", "qpos", "sensordata", "cacc", "actuator_force"]:
    a, b = out[k], ref[k]
    err = np.abs(a - b)
    scale = np.abs(b).max() + 1e-9
    print(f"{k:16s} maxabs {err.max():.3e}  rel-to-max {err.max()/scale:.3e}  median {np.median(err):.2e}")
  # per-world worst cases
  e = np.abs(out["qvel"] - ref["qvel"]).max(axis=1)
  worst = np.argsort(-e)[:6]
  print("worst qvel worlds:", [(int(w), float(e[w]), int(out["solver_niter"][w, 0]), int(ref["solver_niter"][w, 0]), int(ref["nefc"][w, 0])) for w in worst])
  conv = (ref["solver_niter"][:, 0] < 10) & (out["solver_niter"][:, 0] < 10)
  print(f"converged worlds: {conv.sum()}/{N}; max qvel err on converged {e[conv].max():.3e}, unconverged {e[~conv].max() if (~conv).any() else 0:.3e}")
  # timing
  for n2 in (N,):
    torch.cuda.synchronize()
    t = time.time()
    K = 50
    for _ in range(K):
      sim.step()
    torch.cuda.synchronize()
    dt = (time.time() - t) / K
    print(f"N={n2}: {dt*1e3:.3f} ms/step  {n2/dt:.0f} world-steps/s")


if __name__ == "__main__":
  main()
