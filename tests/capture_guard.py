"""Detects host syncs / host->device copies in code meant to be graph-captured.

Runs on CPU (no GPU needed): under ``CaptureGuard`` any op that would, on the
GPU, synchronise with the host or copy host data to the device — the ops a
HIP stream capture rejects (``hipErrorStreamCaptureUnsupported``) — raises.
TEST INFRASTRUCTURE ONLY.
"""

from __future__ import annotations

import torch
from torch.overrides import TorchFunctionMode

_SYNC = {
  torch.Tensor.item, torch.Tensor.tolist, torch.Tensor.nonzero, torch.nonzero, torch.Tensor.__bool__,
  torch.Tensor.cpu, torch.Tensor.numpy, torch.tensor, torch.as_tensor, torch.from_numpy,
  torch.Tensor.__int__, torch.Tensor.__float__, torch.masked_select, torch.Tensor.masked_select,
  torch.unique, torch.Tensor.unique, torch.argwhere,
}


def _has_host_index(idx) -> bool:
  if isinstance(idx, (list, range)):
    return True
  if isinstance(idx, torch.Tensor) and idx.dtype == torch.bool:
    return True  # boolean-mask indexing runs nonzero() on the host
  if isinstance(idx, tuple):
    return any(_has_host_index(i) for i in idx)
  return False


class CaptureHazard(RuntimeError):
  pass


class CaptureGuard(TorchFunctionMode):
  def __torch_function__(self, func, types, args=(), kwargs=None):
    kwargs = kwargs or {}
    if func in _SYNC:
      raise CaptureHazard(f"{getattr(func, '__name__', func)} is a host sync / H2D copy")
    if func in (torch.Tensor.masked_fill_, torch.Tensor.masked_fill, torch.masked_fill) and len(args) > 2 and isinstance(args[2], torch.Tensor):
      raise CaptureHazard("masked_fill with a tensor value reads it on the host (.item())")
    if func in (torch.Tensor.__getitem__, torch.Tensor.__setitem__) and len(args) > 1 and _has_host_index(args[1]):
      raise CaptureHazard("indexing with a host list (H2D copy) or a bool mask (nonzero sync)")
    return func(*args, **kwargs)
