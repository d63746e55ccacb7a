"""The C-ABI library loads and exports every symbol include/mjh_abi.h declares
(no compute calls: these run without a GPU)."""

import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

from mjlab_amd.sim import abi, native
from tests.scenes import g1_scene_model, go1_scene_model

ROOT = Path(__file__).resolve().parents[1]


def declared_functions() -> list[str]:
  txt = (ROOT / "include" / "mjh_abi.h").read_text()
  return re.findall(r"^\s*(?:int|size_t|long long|const char\*)\s+(mjh_\w+)\s*\(", txt, flags=re.M)


def test_header_declarations_match_exports():
  decl = declared_functions()
  assert len(decl) >= 12
  assert set(decl) == set(native.EXPORTS)


def test_library_exports_every_symbol():
  L = native.lib()
  for name in declared_functions():
    assert hasattr(L, name), name


def test_struct_layouts_and_version():
  L = native.lib()
  assert L.mjh_abi_version() == native.ABI_VERSION
  assert L.mjh_sizeof_model() == ctypes.sizeof(abi.model_struct())
  assert L.mjh_sizeof_data() == ctypes.sizeof(abi.data_struct())


def _model_struct(m):
  ms = abi.model_struct()()
  for k, v in abi.model_sizes(m).items():
    setattr(ms, k, v)
  for k, v in abi.model_options(m).items():
    setattr(ms, k, v)
  return ms


@pytest.mark.parametrize("make", [g1_scene_model, go1_scene_model])
def test_host_side_plan(make):
  """Host-only entry points: image size, LDS plan and capacity checks."""
  m = make(4)
  L = native.lib()
  ms = _model_struct(m)
  words = L.mjh_image_words(ctypes.byref(ms))
  assert words > 0
  buf = np.zeros(words, np.float32)  # host buffer: only the pointer/size are checked
  ms.image = buf.ctypes.data
  ms.image_words = words
  assert L.mjh_model_check(ctypes.byref(ms)) == 0, L.mjh_last_error()
  assert 0 < L.mjh_scratch_bytes(ctypes.byref(ms)) <= 160 * 1024
  cap = L.mjh_efc_capacity(ctypes.byref(ms))
  assert 64 <= cap <= m.njmax
  ms.image_words = words - 4
  assert L.mjh_model_check(ctypes.byref(ms)) != 0
  assert b"image" in L.mjh_last_error()


def test_model_check_rejects_oversize():
  m = g1_scene_model(1)
  L = native.lib()
  ms = _model_struct(m)
  ms.nv = 80
  assert L.mjh_model_check(ctypes.byref(ms)) != 0
  assert b"nv" in L.mjh_last_error()


def test_simulation_without_gpu_fails_loudly():
  """No CPU fallback: stepping on a non-GPU device raises."""
  from mjlab_amd.sim import Simulation, SimulationCfg

  m = g1_scene_model(2)
  sim = Simulation(2, SimulationCfg(nconmax=50, njmax=300), m, "cpu")
  with pytest.raises(native.NativeLibraryError):
    sim.step()
  with pytest.raises(native.NativeLibraryError):
    sim.forward()
