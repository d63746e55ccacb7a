"""NaN guard (utils/nan_guard.py semantics): rolling mjSTATE_PHYSICS buffer,
detection over qpos/qvel/qacc/qacc_warmstart, npz dump of the first
max_envs_to_dump non-finite worlds with the reference's metadata dict, and the
model as MJCF that compiles back to the same model."""

import json
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from mjlab_amd.utils.nan_guard import NanGuard, NanGuardCfg
from tests.scenes import g1_scene_model


def _data(n, m, g):
  return SimpleNamespace(qpos=torch.randn(n, m.nq, generator=g), qvel=torch.randn(n, m.nv, generator=g),
                         act=torch.zeros(n, 0), qacc=torch.randn(n, m.nv, generator=g),
                         qacc_warmstart=torch.randn(n, m.nv, generator=g))


def test_disabled_guard_is_inert(tmp_path):
  m = g1_scene_model(1)
  guard = NanGuard(NanGuardCfg(enabled=False, output_dir=str(tmp_path)), 4, m)
  d = _data(4, m, torch.Generator().manual_seed(0))
  d.qpos[1, 3] = float("nan")
  with guard.watch(d):
    pass
  assert not list(tmp_path.iterdir())


def test_dump_on_nan_injection(tmp_path):
  m = g1_scene_model(1)
  n = 8
  guard = NanGuard(NanGuardCfg(enabled=True, buffer_size=3, output_dir=str(tmp_path), max_envs_to_dump=2), n, m)
  g = torch.Generator().manual_seed(1)
  hist = []
  for k in range(5):
    d = _data(n, m, g)
    if k == 4:
      d.qvel[5, 0] = float("inf")
      d.qacc_warmstart[2, 1] = float("nan")  # qacc_warmstart is checked too
      d.qacc_warmstart[7, 1] = float("nan")
    hist.append(torch.cat([d.qpos, d.qvel], 1).double().numpy())
    with guard.watch(d):
      pass
    assert guard.check_and_dump(d) is False  # dumps once
  np.testing.assert_array_equal(NanGuard.detect_nans(d).numpy(), [0, 0, 1, 0, 0, 1, 0, 1])
  from mjlab_amd.utils.nan_guard import load_nan_dump

  meta, states, model_file = load_nan_dump(tmp_path / "nan_dump_latest.npz")
  z = np.load(tmp_path / "nan_dump_latest.npz", allow_pickle=True)
  assert isinstance(z["_metadata"].item(), dict)  # scripts/nan_viz.py:31 reads it with .item()
  assert meta["nan_env_ids"] == [2, 5, 7] and meta["dumped_env_ids"] == [2, 5]
  assert meta["state_size"] == m.nq + m.nv and meta["buffer_size"] == 3 and meta["detection_step"] == 5
  steps = sorted(k for k in z.files if k.startswith("states_step_"))
  assert steps == ["states_step_000002", "states_step_000003", "states_step_000004"]
  for s in steps:
    k = int(s[-6:])
    np.testing.assert_array_equal(z[s], hist[k][[2, 5]])
  assert model_file.exists() and model_file.suffix == ".xml"
  assert sorted(states) == [2, 3, 4]
  assert guard.tripped.tolist() == [2, 5, 7]


@pytest.mark.gpu
def test_simulation_step_dumps_on_nan(tmp_path):
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg

  n = 8
  m = g1_scene_model(n)
  cfg = SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.005),
                      nan_guard=NanGuardCfg(enabled=True, buffer_size=4, output_dir=str(tmp_path)))
  sim = Simulation(n, cfg, m, "cuda:0")
  sim.data.qpos[:] = torch.as_tensor(m.key_qpos, dtype=torch.float32, device="cuda:0")
  for _ in range(3):
    sim.step()
  assert not (tmp_path / "nan_dump_latest.npz").exists()
  sim.data.qvel[3, 10] = float("nan")
  sim.step()
  meta = np.load(tmp_path / "nan_dump_latest.npz", allow_pickle=True)["_metadata"].item()
  assert 3 in meta["nan_env_ids"] and meta["num_envs_total"] == n
