"""Observation history and delay buffers (``src/mjlab/utils/buffers``), device-resident
and capturable: every piece of state a step reads or advances (the write pointer, push
counts, lags, step counts, phase offsets) is a device tensor updated in place, so the
buffers run inside the captured env step (a Python-side pointer would be baked into the
graph at capture time and every replay would write the same slot)."""

from mjlab_amd.utils.buffers.circular_buffer import CircularBuffer
from mjlab_amd.utils.buffers.delay_buffer import DelayBuffer

__all__ = ["CircularBuffer", "DelayBuffer"]
