"""The built library's model-specialised step kernels (tools/gen_spec.py ->
csrc/mjh_spec_table.h) match the benchmark tasks' launch plans at any world
count, so the benchmark runs a specialised instance, not the generic one
(host-side plan comparison, mjh_spec_index: no GPU call)."""

import ctypes

import pytest

from mjlab_amd.scene.scene import Scene
from mjlab_amd.sim import Simulation, native
from mjlab_amd.tasks import load_env_cfg

TASKS = ("Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Velocity-Flat-Unitree-Go1", "Mjlab-Tracking-Flat-Unitree-G1")


@pytest.mark.parametrize("task", TASKS)
@pytest.mark.parametrize("num_envs", [2, 64])
def test_benchmark_tasks_select_a_specialised_kernel(task, num_envs):
  cfg = load_env_cfg(task)
  cfg.scene.num_envs = num_envs
  sim = Simulation(num_envs, cfg.sim, Scene(cfg.scene, device="cpu").compile(), "cpu")
  assert native.lib().mjh_spec_index(ctypes.addressof(sim._mstruct)) >= 0


def test_a_sensor_outside_the_benchmark_set_selects_the_generic_kernel():
  """Model.nsensor_ext is a model size, so part of the plan: the G1 task with
  one extra framepos sensor no longer matches the specialised instance, whose
  code has no framepos evaluation, and runs the generic one."""
  from mjlab_amd.sensor.builtin_sensor import BuiltinSensorCfg, ObjRef

  cfg = load_env_cfg(TASKS[0])
  cfg.scene.num_envs = 2
  assert Scene(cfg.scene, device="cpu").compile().nsensor_ext == 0
  cfg.scene.sensors = tuple(cfg.scene.sensors) + (
    BuiltinSensorCfg(name="pelvis_pos", sensor_type="framepos", obj=ObjRef(type="xbody", name="pelvis", entity="robot")),)
  m = Scene(cfg.scene, device="cpu").compile()
  assert m.nsensor_ext == 1
  sim = Simulation(2, cfg.sim, m, "cpu")
  assert native.lib().mjh_spec_index(ctypes.addressof(sim._mstruct)) == -1
