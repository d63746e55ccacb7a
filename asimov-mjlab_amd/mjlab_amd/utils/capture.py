"""Capture-safe HIP graph ownership.

A HIP graph capture forbids synchronising API calls while the stream is
capturing. Destroying a ``torch.cuda.CUDAGraph`` is one (its destructor
destroys the executable graph and releases the graph's private memory pool);
when the destructor throws inside a capture, the process aborts
(``gpurun_out/r04m/gputests.log:34``: a capture in
``test_fused_velocity_command_matches_torch`` while the cyclic collector ran,
with the previous tests' envs and Simulations, each holding captured graphs,
waiting in reference cycles).

Graphs are therefore never owned by the objects that use them:

* ``GraphSlot`` is the attribute type for a graph (``Simulation.step_graph``,
  ``ManagerBasedRlEnv._graph``). The graph itself lives in a module-level table;
  the owner holds only a handle. When the owner dies (collected anywhere, a
  capture included) or the slot is overwritten, the graph moves to a retired
  list instead of being destroyed.
* ``release_retired()`` destroys the retired graphs, and only when no capture
  is running. ``no_gc()`` (entered around every capture) calls it first, after
  a collection, so retired graphs go before the next capture starts.
* ``no_gc()`` still pauses the collector during the capture: other
  finalisers (a user's objects) may hold device resources too.
"""

from __future__ import annotations

import contextlib
import gc
import itertools
import weakref

_graphs: dict[int, object] = {}  # handle -> live graph
_retired: list = []  # graphs whose owner died or replaced them
_ids = itertools.count(1)


def _retire(h: int) -> None:
  g = _graphs.pop(h, None)
  if g is not None:
    _retired.append(g)


def _capturing() -> bool:
  import torch

  return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def release_retired() -> int:
  """Destroy retired graphs unless a capture is running; returns how many."""
  if _capturing():
    return 0
  n = len(_retired)
  _retired.clear()
  return n


def retired_count() -> int:
  return len(_retired)


class GraphSlot:
  """Descriptor for an attribute that holds a captured graph (or None)."""

  def __set_name__(self, owner, name: str) -> None:
    self.key = "_graphslot_" + name

  def __get__(self, obj, objtype=None):
    if obj is None:
      return self
    ent = obj.__dict__.get(self.key)
    return None if ent is None else _graphs.get(ent[0])

  def __set__(self, obj, g) -> None:
    ent = obj.__dict__.pop(self.key, None)
    if ent is not None:
      ent[1].detach()
      _retire(ent[0])
    if g is not None:
      h = next(_ids)
      _graphs[h] = g
      obj.__dict__[self.key] = (h, weakref.finalize(obj, _retire, h))


@contextlib.contextmanager
def no_gc():
  enabled = gc.isenabled()
  gc.collect()
  release_retired()
  gc.disable()
  try:
    yield
  finally:
    if enabled:
      gc.enable()
