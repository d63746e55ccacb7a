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
  to0 = StepGather(dst=0)(obs, rew, term, trunc)
  assert (to0 is None) == (rank != 0)
  if rank == 0:
    assert torch.equal(to0, out)  # gather to the learner rank == all-gather there
  # numpy payloads: torch tensors travel as shared-memory handles that die with
  # the child process (ConnectionResetError if it exits before the parent reads)
  q.put((rank, out.numpy().copy(), pack_step_outputs(obs, rew, term, trunc).numpy().copy()))
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
  res = [(r, torch.from_numpy(a), torch.from_numpy(b)) for r, a, b in res]
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


def _env_worker(rank, world, port, q):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  torch.set_num_threads(1)
  outs = _run_shard(rank, gather=True)
  q.put((rank, [(o.numpy().copy(), g.numpy().copy()) for o, g in outs]))
  dist.destroy_process_group()


def _run_shard(rank, gather, n=3, steps=3):
  """One rank's env shard (G1 velocity, seed 42 + rank, CPU oracle physics)."""
  import sys
  from pathlib import Path

  sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg
  from tests import oracle_sim

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = n
  cfg.seed = shard_seed(42, rank)
  env = ManagerBasedRlEnv(cfg, device="cpu")
  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
  env.reset()
  packed = env.enable_step_pack()  # written by the env step itself (inside the graph on the GPU)
  g = torch.Generator().manual_seed(1234 + rank)
  sg = StepGather() if gather else None
  outs = []
  for _ in range(steps):
    a = 2 * torch.rand(n, env.action_manager.total_action_dim, generator=g) - 1
    obs, rew, term, trunc, _ = env.step(a)
    own = pack_step_outputs(obs, rew, term, trunc).clone()
    assert torch.equal(own, packed)
    outs.append((own, sg.gather_packed(packed).clone() if sg else None))
  return outs


def test_env_shards_world2_match_single_process():
  """each rank's shard is bit-identical to a single-process run
  with seed 42 + rank, and the all-gather returns the shards rank-major."""
  world = 2
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_env_worker, args=(r, world, port, q)) for r in range(world)]
  for p in ps:
    p.start()
  res = {r: [(torch.from_numpy(o), torch.from_numpy(g)) for o, g in v] for r, v in (q.get(timeout=300) for _ in range(world))}
  for p in ps:
    p.join(timeout=60)
    assert p.exitcode == 0
  for r in range(world):
    single = _run_shard(r, gather=False)
    for t, (own, gathered) in enumerate(res[r]):
      assert torch.equal(own, single[t][0]), (r, t)
      full = torch.cat([res[k][t][0] for k in range(world)], dim=0)
      assert torch.equal(gathered, full)


def _subgroup_worker(rank, world, port, q):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  sub = dist.new_group([1, 2])  # group ranks 0, 1 = global ranks 1, 2
  res = None
  if rank in (1, 2):
    n = 2
    obs = {"policy": torch.full((n, 2), float(rank))}
    rew = torch.full((n,), 10.0 * rank)
    z = torch.zeros(n, dtype=torch.bool)
    sg = StepGather(group=sub, dst=0)
    out = sg(obs, rew, z, z)
    res = None if out is None else out.numpy().copy()
  q.put((rank, res))
  dist.destroy_process_group()


def test_step_gather_to_learner_in_a_subgroup():
  """dst is a group rank; the collective needs its global rank."""
  world = 3
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_subgroup_worker, args=(r, world, port, q)) for r in range(world)]
  for p in ps:
    p.start()
  res = dict(q.get(timeout=120) for _ in range(world))
  for p in ps:
    p.join(timeout=60)
    assert p.exitcode == 0
  assert res[0] is None and res[2] is None
  got = torch.from_numpy(res[1])
  assert got.shape == (4, 2 + 3)
  assert got[:2, 0].tolist() == [1.0, 1.0] and got[2:, 0].tolist() == [2.0, 2.0]
  assert got[:2, 2].tolist() == [10.0, 10.0] and got[2:, 2].tolist() == [20.0, 20.0]


def _bench_cpu(args: list[str], env_extra: dict | None = None):
  import subprocess
  import sys
  from pathlib import Path

  root = Path(__file__).resolve().parents[1]
  env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
  for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
    if not env_extra or k not in env_extra:
      env.pop(k, None)
  return subprocess.run([sys.executable, str(root / "tests" / "bench_cpu_ranks.py"), *args], capture_output=True,
                        text=True, timeout=600, env=env)


def test_bench_multirank_path_world2_cpu():
  """bench.py's N > 1 path end to end: `--gpus 2` without
  torchrun spawns 2 ranks through torch.distributed.run (bench.spawn_ranks),
  each asserts WORLD_SIZE == --gpus, runs its own env shard (seed 42+rank,
  oracle physics on CPU standing in for the HIP step), barriers around the
  timed window, all-reduces its time with MAX, all-gathers the packed
  learner outputs every step; rank 0 alone prints one JSON line."""
  import json

  out = _bench_cpu(["--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1", "--settle", "1", "--num-envs", "4",
                    "--kernel-launches", "1", "--no-cpu-baseline"])
  assert out.returncode == 0, out.stderr[-4000:]
  lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
  assert len(lines) == 1, out.stdout[-2000:]
  j = json.loads(lines[0])
  assert j["n_gpus"] == 2 and j["config"]["world_size"] == 2 and j["scaling"] == "weak"
  assert "all-gather" in j["config"]["parallelism"]
  assert j["config"]["gather_ms_per_step"] is not None and j["config"]["gather_ms_per_step"] > 0
  # value = all ranks' env steps / the slowest rank's window
  assert abs(j["value"] - 2 * 4 * 2 / (j["ms_per_step"] * 2 / 1e3)) < 1e-6 * j["value"]
  assert j["cpu_baseline"] is None  # rank 0 at N = 1 only


def test_bench_rejects_world_size_mismatch():
  out = _bench_cpu(["--gpus", "1", "--device", "cpu", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
  assert out.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in out.stderr
