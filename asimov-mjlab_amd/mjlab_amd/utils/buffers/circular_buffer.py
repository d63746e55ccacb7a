"""Per-env history ring (``src/mjlab/utils/buffers/circular_buffer.py``).

Semantics of the reference (``circular_buffer.py:107-215``): storage (max_len, batch, ...)
written at a pointer shared by all rows; ``buffer`` returns (batch, max_len, ...) oldest to
newest; a row's first append after construction or ``reset`` back-fills every slot of that
row with the appended frame (``:190-215``); ``reset`` zeroes the rows and their push counts;
``buffer[lags]`` returns each row's frame ``lag`` appends back, clamped to the frames it has.

What differs is where the state lives. The reference keeps the pointer as a Python int
and tests ``torch.any(first_push)`` on the host; here the pointer is a 0-d device tensor
advanced in place and the back-fill is a select over the ring, so an append is a fixed
sequence of device ops with no host sync (capturable into the env-step graph; the
values are identical: the same frames land in the same slots).
"""

from __future__ import annotations

from collections.abc import Sequence

import torch


def _rows_mask(batch_ids, batch_size: int, device) -> torch.Tensor | None:
  """None (every row) or a bool mask (batch,) from None / a bool mask / indices."""
  if batch_ids is None or (isinstance(batch_ids, slice) and batch_ids == slice(None)):
    return None
  if isinstance(batch_ids, torch.Tensor) and batch_ids.dtype == torch.bool:
    return batch_ids.to(device)
  m = torch.zeros(batch_size, dtype=torch.bool, device=device)
  if isinstance(batch_ids, slice):
    m[batch_ids] = True
  else:
    m[torch.as_tensor(batch_ids, dtype=torch.long, device=device)] = True
  return m


class CircularBuffer:
  """Fixed-length ring of batched frames; (batch, max_len, ...) view oldest -> newest."""

  def __init__(self, max_len: int, batch_size: int, device: str) -> None:
    if max_len < 1:
      raise ValueError(f"Buffer size must be >= 1, got {max_len}")
    self._max_len = max_len
    self._batch_size = batch_size
    self._device = device
    self._pointer = torch.full((), -1, dtype=torch.long, device=device)
    self._buffer: torch.Tensor | None = None
    self._all_indices = torch.arange(batch_size, device=device)
    self._num_pushes = torch.zeros(batch_size, dtype=torch.long, device=device)
    self._max_len_tensor = torch.full((batch_size,), max_len, dtype=torch.long, device=device)
    self._ring = torch.arange(max_len, device=device)

  @property
  def batch_size(self) -> int:
    return self._batch_size

  @property
  def device(self) -> str:
    return self._device

  @property
  def max_length(self) -> int:
    return self._max_len

  @property
  def current_length(self) -> torch.Tensor:
    """Valid frames per row, min(pushes, max_len). Shape (batch,)."""
    return torch.minimum(self._num_pushes, self._max_len_tensor)

  @property
  def is_initialized(self) -> bool:
    return self._buffer is not None

  @property
  def buffer(self) -> torch.Tensor:
    """(batch, max_len, ...), index 0 oldest, -1 newest."""
    if self._buffer is None:
      raise RuntimeError("Buffer not initialized. Call append() first.")
    idx = torch.remainder(self._ring + (self._pointer + 1), self._max_len)
    return self._buffer.index_select(0, idx).transpose(0, 1)

  def reset(self, batch_ids: Sequence[int] | torch.Tensor | None = None) -> None:
    """Zero the rows' frames and push counts (None: every row)."""
    m = _rows_mask(batch_ids, self._batch_size, self._device)
    if m is None:
      self._num_pushes.zero_()
      if self._buffer is not None:
        self._buffer.zero_()
      return
    self._num_pushes.masked_fill_(m, 0)
    if self._buffer is not None:
      self._buffer.masked_fill_(m.view(1, -1, *([1] * (self._buffer.dim() - 2))), 0.0)

  def append(self, data: torch.Tensor) -> None:
    """Write a (batch, ...) frame at the next slot; first pushes back-fill their row."""
    if data.shape[0] != self._batch_size:
      raise ValueError(f"Expected batch size {self._batch_size}, got {data.shape[0]}")
    data = data.to(self._device)
    if self._buffer is None:
      self._pointer.fill_(-1)
      self._buffer = torch.zeros((self._max_len, *data.shape), dtype=data.dtype, device=self._device)
    self._pointer.add_(1).remainder_(self._max_len)
    self._buffer.index_copy_(0, self._pointer.view(1), data.unsqueeze(0))
    first = (self._num_pushes == 0).view(1, -1, *([1] * (data.dim() - 1)))
    self._buffer.copy_(torch.where(first, data.unsqueeze(0), self._buffer))
    self._num_pushes.add_(1)

  def __getitem__(self, key: torch.Tensor | int) -> torch.Tensor:
    """Each row's frame `key` appends back (LIFO), clamped to the frames it holds."""
    if self._buffer is None:
      raise RuntimeError("Buffer not initialized. Call append() first.")
    if isinstance(key, int):
      key = torch.full((self._batch_size,), key, dtype=torch.long, device=self._device)
    else:
      if key.ndim == 0:
        key = key.expand(self._batch_size)
      key = key.to(device=self._device, dtype=torch.long)
    if key.numel() != self._batch_size:
      raise ValueError(f"Expected {self._batch_size} lags, got {key.numel()}")
    valid = torch.minimum(key, self._num_pushes.clamp_min(1) - 1).clamp_min(0)
    idx = torch.remainder(self._pointer - valid, self._max_len)
    return self._buffer[idx, self._all_indices]
