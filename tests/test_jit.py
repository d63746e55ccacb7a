"""Launch plugins, host side (mjlab_amd/sim/jit.py; no GPU call): the one-plan table a
plugin is compiled from, the cache key, and registration with the main library.
GPU parity and speed of a plugin: tests/test_gpu_jit.py."""

import ctypes
import re
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
from jit_build import task_model  # noqa: E402

from mjlab_amd.sim import Simulation, jit, native  # noqa: E402
from mjlab_amd.sim.spec_table import layout_ints, plan_of, render, size_ints  # noqa: E402

G1 = "Mjlab-Velocity-Flat-Unitree-G1"


def _plan(framepos=("pelvis",)):
  cfg, m = task_model(G1, framepos)
  cfg.sim.specialize = "off"
  sim = Simulation(2, cfg.sim, m, "cpu")
  return sim, m, plan_of(native.lib(), ctypes.addressof(sim._mstruct))


def test_one_plan_table_renders_the_plan():
  _, _, plan = _plan()
  text = render([plan], ["g1+framepos"], layout_ints(native.lib()), origin="test")
  assert "#define MJH_NSPEC 1" in text
  row = re.search(r"kSpecPlan\[MJH_NSPEC\]\[kPlanInts\] = \{\n  \{([^}]*)\}", text).group(1)
  assert [int(x) for x in row.split(",")] == plan
  sizes = re.search(r"return Sizes\{([^}]*)\}", text).group(1)
  assert [int(x) for x in sizes.split(",")] == plan[1:1 + size_ints()]


def test_plugin_key_depends_on_the_plan():
  _, _, p1 = _plan()
  _, _, p0 = _plan(framepos=())
  assert p1 != p0
  assert jit.plugin_path(p1) != jit.plugin_path(p0)
  assert jit.plugin_path(p1) == jit.plugin_path(list(p1))


def test_the_benchmark_model_needs_no_plugin():
  sim, m, _ = _plan(framepos=())
  assert jit.ensure(ctypes.addressof(sim._mstruct), m, compile_missing=False)["kind"] == "builtin"


def test_elliptic_or_pgs_models_keep_the_generic_instance():
  cfg, m = task_model(G1, ("pelvis",))
  cfg.sim.mujoco.cone = "elliptic"
  cfg.sim.specialize = "off"
  sim = Simulation(2, cfg.sim, m, "cpu")
  r = jit.ensure(ctypes.addressof(sim._mstruct), m, compile_missing=False)
  assert r["kind"] == "generic" and "elliptic" in r["reason"]


def test_prebuilt_plugin_registers_for_its_plan():
  """build() prebuilds the plugin of G1 + pelvis framepos (tools/jit_build.py)."""
  sim, m, plan = _plan()
  path = jit.plugin_path(plan)
  if not path.exists():
    pytest.skip(f"{path.name} not built (run __graft_entry__.build())")
  r = jit.ensure(ctypes.addressof(sim._mstruct), m, compile_missing=False)
  assert r["kind"] == "plugin"
  assert native.lib().mjh_plugin_index(ctypes.addressof(sim._mstruct)) == r["index"]
  lib = ctypes.CDLL(str(path))
  assert lib.mjh_plugin_abi() == native.ABI_VERSION
  # the model without the extra sensor still takes the built-in instance, not the plugin
  base, _, _ = _plan(framepos=())
  assert native.lib().mjh_plugin_index(ctypes.addressof(base._mstruct)) == -1
  assert native.lib().mjh_spec_index(ctypes.addressof(base._mstruct)) >= 0
