"""World-size-2 gloo test of the sharded step-output exchange (CPU)."""

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mjlab_amd.distributed import StepGather, pack_step_outputs, shard_seed


def _free_port() -> int:
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _worker(rank, world, port, q):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  n = 5
  g = torch.Generator().manual_seed(shard_seed(42, rank))
  obs = {"policy": torch.randn(n, 3, generator=g), "critic": torch.randn(n, 4, generator=g)}
  rew = torch.randn(n, generator=g)
  term = torch.rand(n, generator=g) > 0.5
  trunc = torch.zeros(n, dtype=torch.bool)
  out = StepGather()(obs, rew, term, trunc)
  q.put((rank, out.clone(), pack_step_outputs(obs, rew, term, trunc)))
  dist.destroy_process_group()


def test_step_gather_world2():
  world = 2
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
  for p in ps:
    p.start()
  res = [q.get(timeout=120) for _ in range(world)]
  for p in ps:
    p.join(timeout=60)
    assert p.exitcode == 0
  res.sort(key=lambda x: x[0])
  full = torch.cat([r[2] for r in res], dim=0)
  for _, gathered, _ in res:
    assert gathered.shape == (10, 3 + 4 + 3)
    assert torch.equal(gathered, full)  # rank-major, identical on every rank


def test_shard_seeds_distinct():
  assert len({shard_seed(42, r) for r in range(8)}) == 8


def test_pack_layout():
  obs = {"policy": torch.ones(2, 3), "critic": torch.zeros(2, 1)}
  p = pack_step_outputs(obs, torch.tensor([5.0, 6.0]), torch.tensor([True, False]), torch.tensor([False, True]))
  assert p.shape == (2, 7)
  assert p[0].tolist() == [0.0, 1.0, 1.0, 1.0, 5.0, 1.0, 0.0]
