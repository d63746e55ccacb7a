"""Box-pair contacts, HIP step vs oracle (diagnostic, GPU box): per pair type,
the contacts whose position or normal differ, with both sides' values."""
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
import tests.test_gpu_parity as t

n = 512
m = compile_spec(read_mjcf_string(t.BOX_SCENE), 50, 300)
st = t._box_states(m, n, np.random.default_rng(51))
sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.002, iterations=20, ls_iterations=20)), m, "cuda:0")
t.put(sim, st)
sim.forward()
got = t.get(sim, n)
ref = Oracle(m).run(n, st, integrate=False)
types = np.asarray(m.geom_type)
shown = 0
for w in range(n):
  ng, nr = int(got["ncon"][w, 0]), int(ref["ncon"][w, 0])
  gg = got["contact_geom"][w].reshape(-1, 2)[:ng]
  rg = ref["contact_geom"][w].reshape(-1, 2)[:nr]
  gp = got["contact_pos"][w].reshape(-1, 3)[:ng]
  rp = ref["contact_pos"][w].reshape(-1, 3)[:nr]
  gf = got["contact_frame"][w].reshape(-1, 9)[:ng, :3]
  rf = ref["contact_frame"][w].reshape(-1, 9)[:nr, :3]
  gd = got["contact_dist"][w][:ng]
  rd = ref["contact_dist"][w][:nr]
  for i in range(ng):
    j = [k for k in range(nr) if tuple(rg[k]) == tuple(gg[i]) and np.abs(rp[k] - gp[i]).max() < 1e-3]
    if j:
      continue
    if shown < 12:
      print(f"w{w} pair types {types[gg[i][0]]}-{types[gg[i][1]]} dev dist {gd[i]:.6f} pos {gp[i]} n {gf[i]}")
      for k in range(nr):
        if tuple(rg[k]) == tuple(gg[i]):
          print(f"     oracle dist {rd[k]:.6f} pos {rp[k]} n {rf[k]}")
      print("     qpos", st["qpos"][w])
    shown += 1
print("unmatched device contacts:", shown, "ncon equal", float((got["ncon"] == ref["ncon"]).mean()))
