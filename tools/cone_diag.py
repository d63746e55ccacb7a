"""Elliptic-cone block slide, HIP step vs oracle step by step (diagnostic, GPU
box): per step the device's and the oracle's (own choices) forces, solver
iterations and tangential speed, from the same state."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np
import torch

from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from oracle.oracle import Oracle

mu, g = 0.65, 9.81
th = np.arctan(0.8)
gt = g * np.sin(th) / np.sqrt(2)
xml = f"""<mujoco><option timestep="0.002" gravity="{gt} {gt} {-g * np.cos(th)}"/><worldbody>
<geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>
<body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>
</worldbody></mujoco>"""
for lsp in (True, False):
  m = compile_spec(read_mjcf_string(xml), 8, 64)
  sim = Simulation(2, SimulationCfg(nconmax=8, njmax=64, ls_parallel=lsp,
                                    mujoco=MujocoCfg(timestep=0.002, iterations=20, cone="elliptic", gravity=(gt, gt, -g * np.cos(th)))), m, "cuda:0")
  orc = Oracle(m)
  keys = ("qpos", "qvel", "qacc_warmstart", "time")
  for step in range(60):
    st = {k: getattr(sim.data, k).detach().cpu().numpy().reshape(2, -1).astype(np.float64) for k in keys}
    sim.step()
    torch.cuda.synchronize()
    got = {k: getattr(sim.data, k).detach().cpu().numpy().reshape(2, -1) for k in sim.data.fields()}
    ref = orc.run(2, st, integrate=True)
    if step % 5 == 0 or step < 6:
      ne = int(got["nefc"][0, 0])
      print(f"ls_parallel={lsp} step {step} nefc {ne}/{int(ref['nefc'][0, 0])} niter {int(got['solver_niter'][0, 0])}/{int(ref['solver_niter'][0, 0])} "
            f"v {np.hypot(*got['qvel'][0, :2]):.5f}/{np.hypot(*ref['qvel'][0, :2]):.5f}")
      print("   dev f", np.round(got["efc_force"][0, :ne], 4))
      print("   ora f", np.round(ref["efc_force"][0, :ne], 4))
      print("   dev qacc", np.round(got["qacc"][0], 4), "ora", np.round(ref["qacc"][0], 4))
