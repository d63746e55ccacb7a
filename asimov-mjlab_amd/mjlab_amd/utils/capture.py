"""Graph capture without the garbage collector.

A HIP graph capture forbids synchronising API calls on the capturing stream.
Python's cyclic garbage collector may run at any allocation inside the capture
and finalise an unrelated object whose destructor calls such an API (a
previous env's graph, a Simulation's buffers), which aborts the process. The
capture therefore collects first and runs with the collector paused."""

from __future__ import annotations

import contextlib
import gc


@contextlib.contextmanager
def no_gc():
  enabled = gc.isenabled()
  gc.collect()
  gc.disable()
  try:
    yield
  finally:
    if enabled:
      gc.enable()
