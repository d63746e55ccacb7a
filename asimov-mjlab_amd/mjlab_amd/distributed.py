"""Multi-GPU env sharding: one process per GPU, each owning an
independent shard of worlds; the only exchange is an all-gather of the
learner-facing step outputs (RCCL over xGMI on the GPU box, gloo in tests)."""

from __future__ import annotations

import torch
import torch.distributed as dist


def shard_seed(base_seed: int, rank: int) -> int:
  """Per-rank env seed (rank r of a 42-seeded job uses 42 + r)."""
  return base_seed + rank


def packed_width(obs_dims: dict) -> int:
  """Columns of the packed step outputs for observation groups of these widths."""
  return sum(int(obs_dims[k]) for k in sorted(obs_dims)) + 3


def pack_step_outputs(obs: dict, reward: torch.Tensor, terminated: torch.Tensor, truncated: torch.Tensor,
                      out: torch.Tensor | None = None) -> torch.Tensor:
  """(num_envs, D) float32: [obs groups in key order | reward | terminated | truncated].
  With ``out`` (preallocated, e.g. the env's graph-resident pack buffer) the
  result is written in place: no allocation, capturable."""
  parts = [obs[k].reshape(obs[k].shape[0], -1).float() for k in sorted(obs)]
  parts += [reward[:, None].float(), terminated[:, None].float(), truncated[:, None].float()]
  if out is None:
    return torch.cat(parts, dim=1)
  return torch.cat(parts, dim=1, out=out)


class StepGather:
  """Collects each rank's packed step outputs into one (world * num_envs, D)
  buffer (rank-major) — one collective per env step, no other data-path traffic.

  ``dst=None``: all-gather (every rank holds the full batch, the north star's
  RCCL all-gather). ``dst=r``: gather to the learner rank ``r`` only (RCCL
  gather: each rank sends its shard once; other ranks get ``None``)."""

  def __init__(self, group=None, dst: int | None = None) -> None:
    self.group = group
    self.dst = dst  # rank within `group`
    self.world = dist.get_world_size(group) if dist.is_initialized() else 1
    self.rank = dist.get_rank(group) if dist.is_initialized() else 0
    # the collective takes a global rank (a subgroup's ranks need not be 0..k-1)
    self._dst_global = (dist.get_global_rank(group, dst) if (group is not None and dst is not None) else dst)
    self.buf: torch.Tensor | None = None

  def __call__(self, obs, reward, terminated, truncated) -> torch.Tensor:
    return self.gather_packed(pack_step_outputs(obs, reward, terminated, truncated))

  def gather_packed(self, packed: torch.Tensor) -> torch.Tensor | None:
    """Exchange an already packed (num_envs, D) buffer — the env's graph-resident
    pack buffer (ManagerBasedRlEnv.enable_step_pack) — stream-ordered after the
    step, no host sync."""
    if self.world == 1:
      return packed
    if self.buf is None or self.buf.shape != (self.world * packed.shape[0], packed.shape[1]):
      self.buf = torch.empty((self.world * packed.shape[0], packed.shape[1]), dtype=packed.dtype, device=packed.device)
    if self.dst is None:
      dist.all_gather_into_tensor(self.buf, packed.contiguous(), group=self.group)
      return self.buf
    if self.rank == self.dst:
      dist.gather(packed.contiguous(), list(self.buf.chunk(self.world, dim=0)), dst=self._dst_global, group=self.group)
      return self.buf
    dist.gather(packed.contiguous(), None, dst=self._dst_global, group=self.group)
    return None
