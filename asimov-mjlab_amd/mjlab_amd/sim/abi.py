"""ctypes view of the C ABI descriptors, generated from ``include/mjh_fields.h``.

The header's X-macro lists are the single source of truth for the layout of
``mjh_model`` / ``mjh_data``. This module parses those lines and builds
matching ``ctypes.Structure`` classes, so the Python host and the HIP library
can never disagree on field order. The same parser serves the CPU oracle
(tests only), whose structs use the same lists with float64 reals.
"""

from __future__ import annotations

import ctypes
import re
from dataclasses import dataclass
from functools import lru_cache
from pathlib import Path

REPO = Path(__file__).resolve().parents[3]
HEADER = REPO / "include" / "mjh_fields.h"


@dataclass(frozen=True)
class Field:
  kind: str  # MS | MO | MA | MW | DA
  ctype: str  # float | int | mjh_i64 (MS: int)
  name: str
  count: str  # expression in size names ("" for MS/MO)


def _macro_body(text: str, macro: str) -> str:
  m = re.search(rf"#define {macro}\((\w+)\)(.*?)(?:\n\s*\n|\n/\*|\Z)", text, re.S)
  if not m:
    raise RuntimeError(f"macro {macro} not found in {HEADER}")
  return m.group(2).replace("\\\n", " ")


@lru_cache(maxsize=None)
def fields() -> tuple[Field, ...]:
  text = HEADER.read_text()
  out: list[Field] = []
  for name in re.findall(r"MS\((\w+)\)", _macro_body(text, "MJH_MODEL_SIZES")):
    out.append(Field("MS", "int", name, ""))
  for t, name in re.findall(r"MO\((\w+),\s*(\w+)\)", _macro_body(text, "MJH_MODEL_OPTIONS")):
    out.append(Field("MO", t, name, ""))
  for kind, macro in (("MA", "MJH_MODEL_ARRAYS"), ("MW", "MJH_MODEL_WARRAYS"), ("DA", "MJH_DATA_ARRAYS")):
    for t, name, count in re.findall(rf"{kind}\((\w+),\s*(\w+),\s*([^)]+)\)", _macro_body(text, macro)):
      out.append(Field(kind, t, name, count.strip()))
  return tuple(out)


def count(field: Field, sizes: dict[str, int]) -> int:
  return int(eval(field.count, {"__builtins__": {}}, dict(sizes)))  # noqa: S307 (header-controlled)


_SCALAR = {"int": ctypes.c_int, "mjh_i64": ctypes.c_longlong}


def _ct(t: str, real):
  return real if t == "float" else _SCALAR[t]


@lru_cache(maxsize=None)
def model_struct(real=ctypes.c_float, device: bool = True):
  """ctypes mirror of ``mjh_model`` (device=True, float reals) or of the
  oracle's ``or_model`` (device=False; float64 or float32 reals)."""
  members = []
  for f in fields():
    if f.kind == "MS":
      members.append((f.name, ctypes.c_int))
    elif f.kind == "MO":
      members.append((f.name, _ct(f.ctype, real)))
  for f in fields():
    if f.kind == "MA":
      members.append((f.name, ctypes.c_void_p))
    elif f.kind == "MW":
      members.append((f.name, ctypes.c_void_p))
      members.append((f.name + "_wstride", ctypes.c_longlong))
  # MA and MW are interleaved in declaration order in C: MA list first, then MW list.
  if device:  # device descriptor: packed model-image scratch
    members += [("image", ctypes.c_void_p), ("image_words", ctypes.c_int), ("_pad_image", ctypes.c_int)]
  return type("mjh_model" if device else "or_model", (ctypes.Structure,), {"_fields_": members})


@lru_cache(maxsize=None)
def data_struct(real=ctypes.c_float, device: bool = True):
  members = [("nworld", ctypes.c_int), ("_pad", ctypes.c_int)]
  for f in fields():
    if f.kind == "DA":
      members.append((f.name, ctypes.c_void_p))
  if device:  # device descriptor: per-world global scratch
    members += [("scratch", ctypes.c_void_p), ("scratch_words", ctypes.c_longlong), ("world_order", ctypes.c_void_p)]
    # optional fused contact-sensor timers (mjh_data.at_*)
    members += [(f"at_{n}", ctypes.c_void_p) for n in ("last_time", "cur_air", "last_air", "cur_con", "last_con")]
    members += [("at_k", ctypes.c_int), ("at_cols", ctypes.c_int * 7)]
    # optional site-output layout inside a wider per-world site array (env-origin sites)
    members += [("site_wstride", ctypes.c_longlong), ("site_off", ctypes.c_int), ("_pad_site", ctypes.c_int)]
  return type("mjh_data" if device else "or_data", (ctypes.Structure,), {"_fields_": members})


def size_names() -> list[str]:
  return [f.name for f in fields() if f.kind == "MS"]


def option_fields() -> list[Field]:
  return [f for f in fields() if f.kind == "MO"]


def model_array_fields() -> list[Field]:
  return [f for f in fields() if f.kind in ("MA", "MW")]


def data_array_fields() -> list[Field]:
  return [f for f in fields() if f.kind == "DA"]


def model_sizes(model) -> dict[str, int]:
  return {n: int(getattr(model, n)) for n in size_names()}


def model_options(model) -> dict[str, float]:
  out = {}
  for f in option_fields():
    if f.name.startswith("gravity_"):
      out[f.name] = float(model.gravity["xyz".index(f.name[-1])])
    elif f.name.startswith("magnetic_"):
      out[f.name] = float(model.magnetic["xyz".index(f.name[-1])])
    else:
      out[f.name] = getattr(model, f.name)
  return out


def model_host_arrays(model) -> dict:
  """Flat numpy arrays for every MA/MW field, float64 for reals."""
  import numpy as np

  sizes = model_sizes(model)
  out = {}
  for f in model_array_fields():
    n = count(f, sizes)
    a = np.asarray(getattr(model, f.name))
    dt = {"float": np.float64, "int": np.int32, "mjh_i64": np.int64}[f.ctype]
    a = np.ascontiguousarray(a, dtype=dt).reshape(-1)
    if a.size != n:
      if n == 0 and a.size <= 1:
        a = np.zeros(1, dtype=dt)
      else:
        raise ValueError(f"model field {f.name}: {a.size} elements, header says {n}")
    out[f.name] = a
  return out
