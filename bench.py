#!/usr/bin/env python3
"""Benchmark: env steps/s on Mjlab-Velocity-Flat-Unitree-G1 @ 4096 envs/GPU.

Contract ("Measurement"):
  python bench.py [--gpus N] [--steps K] [--warmup W] [--task T] [--num-envs E]
One process per GPU. When started as a plain `python bench.py --gpus N` (N > 1),
the script re-launches itself under `torch.distributed.run` with N ranks before
touching the GPU (a child process, not an exec); when the driver launches it
under torchrun it reads RANK / LOCAL_RANK / WORLD_SIZE and asserts
WORLD_SIZE == --gpus. Each rank owns its own env shard (seed 42 + rank) —
worlds are independent, so the work shards with weak scaling; after every env
step the ranks all-gather the learner-facing outputs (policy obs, critic obs,
reward, terminated, truncated) over RCCL, the one exchange the north star names.

A "step" is one full env step of the manager-based RL env: action processing,
4 physics sub-steps (the HIP step kernel), terminations, rewards, masked
resets + gated forward, commands, push events and observations — captured in
one HIP graph. Actions come from the random agent of the reference's
`play --agent random` (2*U[0,1)-1, torch.Generator seeded 1234 + rank).

Steady state. Episode lengths start uniformly random (rsl_rl's
`init_at_random_ep_len=True`, which the reference's train.py:121 passes), but
every env starts standing, so the random agent's falls come in waves that take
many episodes of fall time to dephase. The settle (untimed, before the W warmup
steps) therefore runs at least one episode (--settle-min 1000 env steps,
velocity_env_cfg.py:383) and then continues in 100-step blocks until the last
two 250-step reset rates agree within 5 % (--settle-max 4000). The timed window
then sees the stationary reset rate (and with it the forward pass that the
reference runs over all worlds whenever any env resets,
manager_based_rl_env.py:133-137) whatever --steps and --warmup the caller picks.
The line reports the window's resets per step next to the settle tail's, and
the fraction of timed steps that ran that forward.

Rank 0 prints ONE JSON line with, in addition to the contract fields:
  roofline      — the dominant kernel (the fused physics step) measured live
                  with HIP events on its stream: algorithmic bytes per launch
                  (5,384 B per world per physics step) / average
                  launch duration, against the 8 TB/s HBM peak. `traffic` is the
                  PMC-measured HBM bytes per launch from profiles/ (or null).
  roofline_valu — the same launch against the VALU issue peak: SQ_INSTS_VALU
                  per launch from the committed counter summary
                  (profiles/step_kernel_sq.json) / live launch time, 2 cycles
                  per wave64 instruction on 1024 SIMD-32 at 2.4 GHz.
  cpu_baseline  — the CPU restatement (oracle/, float64 and float32, OpenMP
                  over worlds) of the same physics step on this host's cores,
                  bounded sample of the live state.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path


def _native():
  from mjlab_amd.sim import native

  return native.lib()


REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "asimov-mjlab_amd"))

TASK = "Mjlab-Velocity-Flat-Unitree-G1"
METRIC = "env steps/sec (whole node), Unitree G1 flat velocity task @ 4096 envs/GPU"
# per-task envs per GPU (BASELINE.json configs 2-4)
DEFAULT_ENVS = {TASK: 4096, "Mjlab-Velocity-Flat-Unitree-Go1": 8192, "Mjlab-Tracking-Flat-Unitree-G1": 4096}
# algorithmic bytes per world per physics step: G1 5,384 B, Go1 3,040 B
B_PHYS = {"Unitree-Go1": 3040}
B_PHYS_G1 = 5384
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
# VALU issue peak: 256 CUs x 4 SIMD-32, a wave64 VALU instruction issues over 2
# cycles, 2.4 GHz max clock (MI355X_MICROARCH.md:34, :53-54)
N_SIMD, CLK_HZ, VALU_CYC = 1024, 2.4e9, 2
VALU_PEAK_GIPS = N_SIMD * CLK_HZ / VALU_CYC / 1e9


def parse() -> argparse.Namespace:
  p = argparse.ArgumentParser()
  p.add_argument("--gpus", type=int, default=1)
  p.add_argument("--steps", type=int, default=300)
  p.add_argument("--warmup", type=int, default=30)
  p.add_argument("--settle", type=int, default=-1,
                 help="untimed env steps before warmup; -1 (default): adaptive, until the reset rate is stationary")
  p.add_argument("--settle-min", type=int, default=1000, help="adaptive settle: at least this many env steps (one episode)")
  p.add_argument("--settle-max", type=int, default=4000, help="adaptive settle: at most this many env steps")
  p.add_argument("--num-envs", type=int, default=0, help="envs per GPU (default: the task's BASELINE config)")
  p.add_argument("--task", default=TASK)
  p.add_argument("--no-gather", action="store_true", help="skip the per-step RCCL all-gather (N > 1)")
  p.add_argument("--no-cpu-baseline", action="store_true")
  p.add_argument("--cpu-sample-worlds", type=int, default=0, help="0: all of the workload's worlds")
  p.add_argument("--cpu-seconds", type=float, default=8.0, help="per precision")
  p.add_argument("--kernel-launches", type=int, default=50)
  p.add_argument("--motion-file", default="", help="tracking tasks: motion npz (default: synthetic 500-frame clip)")
  # test harness only (tests/bench_cpu_ranks.py): the multi-rank path on CPU
  # tensors over gloo, with the test's stand-in physics attached by env_hook
  p.add_argument("--device", default="cuda", choices=("cuda", "cpu"), help=argparse.SUPPRESS)
  return p.parse_args()


def spawn_ranks(args) -> None:
  """`python bench.py --gpus N` with no torchrun around it: run N ranks as a
  child `torch.distributed.run` (before any GPU call) and exit with its code.
  The child runs the script that was started (bench.py, or a test harness that
  calls bench.main)."""
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
         "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(sys.argv[0]).resolve()), *sys.argv[1:]]
  env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
  sys.exit(subprocess.call(cmd, env=env))


def synthetic_motion_file(dev: str, frames: int = 500) -> str:
  """Config 4's input: a smooth sinusoidal G1 joint trajectory
  around the default pose, evaluated by one batched forward pass on the GPU
  (mjlab_amd.motion), written in the csv_to_npz format."""
  import tempfile

  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.motion import KEYS, save_motion, synthetic_motion
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg(TASK)
  cfg.scene.num_envs = frames
  env = ManagerBasedRlEnv(cfg, device=dev)
  mot = synthetic_motion(env.sim, env.scene["robot"], num_frames=frames, fps=50.0)
  path = Path(tempfile.mkdtemp()) / "g1_synthetic_motion.npz"
  save_motion(path, 50.0, **{k: mot[k] for k in KEYS})
  del env
  return str(path)


def _host_threads() -> tuple[int, int]:
  """(threads used, host cores in this process's affinity). The threads are the
  affinity's cores unless OMP_NUM_THREADS says otherwise (on the GPU box it is
  set to the box's CPU share: the machine's other cores belong to other jobs)."""
  try:
    host = len(os.sched_getaffinity(0))
  except AttributeError:
    host = os.cpu_count() or 1
  omp = os.environ.get("OMP_NUM_THREADS")
  return (max(1, min(host, int(omp))) if omp else host), host


def cpu_baseline(env, args) -> dict:
  """Time the oracle (CPU restatement of the same physics step, OpenMP over
  worlds) on the workload's worlds (all N of them, from the bench's live
  state), float64 then float32, for a bounded time each."""
  sys.path.insert(0, str(REPO))
  from oracle.oracle import Oracle

  cores, host = _host_threads()
  n = min(args.cpu_sample_worlds, env.num_envs) if args.cpu_sample_worlds > 0 else env.num_envs
  d = env.sim.data
  state0 = {k: getattr(d, k)[:n].detach().cpu().numpy() for k in ("qpos", "qvel", "act", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied", "time")}
  overrides = {}
  m = env.sim.model
  for name in env.event_manager.domain_randomization_fields:
    overrides[name] = getattr(m, name)[:n].detach().cpu().numpy()
  dec = env.cfg.decimation
  res = {}
  for prec in ("f64", "f32"):
    state = {k: v.copy() for k, v in state0.items()}
    orc = Oracle(env.sim.mj_model, prec, overrides=overrides)
    orc.run(n, state, integrate=True, nthreads=cores)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
      out = orc.run(n, state, integrate=True, nthreads=cores)
      for k in ("qpos", "qvel", "qacc_warmstart", "time"):
        state[k] = out[k]
      reps += 1
      el = time.perf_counter() - t0
      if el > args.cpu_seconds or reps >= 20000:
        break
    res[prec] = (n * reps / el / dec, reps, el)
  v64, r64, e64 = res["f64"]
  v32, r32, e32 = res["f32"]
  return {
    "value": v64,
    "unit": "env steps/sec (physics only: decimation x mj_step per env step)",
    "cores": cores,
    "host_cores": host,
    "kind": "port",
    "value_f32": v32,
    "sample": f"all {n} {env.sim.mj_model.nv}-dof worlds of the workload from the bench's live state, oracle/oracle.c "
    f"with OpenMP {cores} threads ({host} cores in the affinity, OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}): "
    f"float64 {r64} physics steps ({e64:.1f} s) -> value; float32 {r32} steps ({e32:.1f} s) -> value_f32; "
    "env-layer cost excluded; MuJoCo C is not available",
  }


def cpu_config1(args) -> dict:
  """BASELINE.json config 1: Mjlab-Velocity-Flat-Unitree-G1, num_envs=1, zero
  agent (scripts/play.py:212-215), the whole env step on the CPU: mjlab_amd's
  env layer on CPU tensors with the oracle's float64 physics standing in for
  MuJoCo C's mj_step (absent). One thread. Timed for --cpu-seconds."""
  import torch

  sys.path.insert(0, str(REPO))
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg
  from oracle.oracle import INPUTS, Oracle

  nthr = torch.get_num_threads()
  torch.set_num_threads(1)
  try:
    cfg = load_env_cfg(TASK)
    cfg.scene.num_envs = 1
    cfg.seed = 42
    env = ManagerBasedRlEnv(cfg, device="cpu")
    sim = env.sim
    ov = {f: getattr(sim.model, f).numpy() for f in env.event_manager.domain_randomization_fields}
    orc = Oracle(sim.mj_model, "f64", overrides=ov)
    fields = [f for f in INPUTS if f in sim._data_flat]

    def run(integrate: bool) -> None:
      sim.epoch.bump()
      out = orc.run(1, {f: sim._data_flat[f].numpy() for f in fields}, integrate=integrate)
      for f, t in sim._data_flat.items():
        if f in out and t.numel():
          t.copy_(torch.as_tensor(out[f].reshape(1, -1)[:, : t.shape[1]]).to(t.dtype))

    sim._require_gpu = lambda: None
    sim.step = lambda: run(True)
    sim.forward = lambda: run(False)
    sim.forward_gated = lambda gate: run(False) if bool(gate.any()) else None
    env.reset()
    zero = torch.zeros(1, env.action_manager.total_action_dim)
    for _ in range(10):
      env.step(zero)
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
      env.step(zero)
      k += 1
    el = time.perf_counter() - t0
  finally:
    torch.set_num_threads(nthr)
  return {"value": k / el, "unit": "env steps/s", "cores": 1, "kind": "port", "steps": k,
          "sample": f"config 1: {TASK}, num_envs=1, zero agent, {k} full env steps in {el:.1f} s on one host thread "
          "(env layer on CPU tensors + oracle float64 physics; MuJoCo C is not available)"}


def main(env_hook=None) -> None:
  """env_hook(env): called on each rank's env before its first reset (the CPU
  test harness attaches its stand-in physics there; None on the GPU)."""
  args = parse()
  if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
    spawn_ranks(args)
  import torch
  import torch.distributed as dist

  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if world != args.gpus:
    raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
  on_gpu = args.device == "cuda"
  if on_gpu:
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"
  else:
    dev = "cpu"
  if world > 1:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if on_gpu:
      dist.init_process_group("nccl", device_id=torch.device(dev))
    else:
      dist.init_process_group("gloo")

  def sync() -> None:
    if on_gpu:
      torch.cuda.synchronize()

  num_envs = args.num_envs or DEFAULT_ENVS.get(args.task, 4096)

  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg(args.task)
  cfg.scene.num_envs = num_envs
  motion = getattr(cfg, "commands", {}).get("motion") if isinstance(getattr(cfg, "commands", None), dict) else None
  if motion is not None and not motion.motion_file:
    motion.motion_file = args.motion_file or synthetic_motion_file(dev)
  from mjlab_amd.distributed import StepGather, shard_seed

  cfg.seed = shard_seed(42, rank)
  env = ManagerBasedRlEnv(cfg, device=dev)
  if env_hook is not None:
    env_hook(env)
  env.reset()
  # rsl_rl OnPolicyRunner.learn(init_at_random_ep_len=True) (reference train.py:121)
  g_ep = torch.Generator(device=dev)
  g_ep.manual_seed(4321 + rank)
  env.episode_length_buf.copy_(torch.randint(0, int(env.max_episode_length), (num_envs,), device=dev, generator=g_ep))
  gen = torch.Generator(device=dev)
  gen.manual_seed(1234 + rank)
  act = torch.empty(num_envs, env.action_manager.total_action_dim, device=dev)

  def agent():
    # 2 U[0,1) - 1 as one launch: uniform_(-1, 1) draws u * 2 + (-1) from the
    # same generator state (2u is exact, so the values equal the three-op form)
    return act.uniform_(-1.0, 1.0, generator=gen)

  gather = StepGather()
  use_gather = world > 1 and not args.no_gather
  # learner-facing outputs packed by the env step itself (inside its graph),
  # then all-gathered over RCCL, stream-ordered after the replay (no host sync)
  packed = env.enable_step_pack() if use_gather else None

  def exchange(obs, rew, term, trunc):
    if use_gather:
      gather.gather_packed(packed)

  # graph capture happens on the 2nd step; settle + warmup steps are untimed
  def run(k: int) -> None:
    for _ in range(k):
      o, r, te, tr, _ = env.step(agent())
      exchange(o, r, te, tr)

  run(2)
  settle_log, tail_rate = [], None
  if args.settle >= 0:
    run(args.settle)
    settled = args.settle
  else:
    # adaptive: per-block reset counts (one host read per 50-step block, untimed)
    blk, win = 50, 5  # two windows of 5 blocks = 250 steps each
    counts, settled = [], 0
    last = int(env.step_stats()[0].item())
    while settled < args.settle_max:
      run(blk)
      settled += blk
      cur = int(env.step_stats()[0].item())
      counts.append(cur - last)
      last = cur
      if settled >= args.settle_min and len(counts) >= 2 * win and settled % 100 == 0:
        a, b = sum(counts[-2 * win:-win]) / (win * blk), sum(counts[-win:]) / (win * blk)
        done = int(abs(a - b) <= 0.05 * max(a, b, 1e-9))
        if world > 1:  # every rank stops at the same step (the per-step gather is collective)
          t = torch.tensor([done], device=dev, dtype=torch.long)
          dist.all_reduce(t, op=dist.ReduceOp.MIN)
          done = int(t.item())
        if done:
          break
    settle_log = [c / blk for c in counts[-20:]]
    tail_rate = sum(counts[-2 * win:]) / (2 * win * blk)
  run(args.warmup)
  sync()
  stats0 = env.step_stats().clone()
  flags0 = env.sim.flag_stats()[3:].clone()  # running totals of worlds that overflowed / went non-finite
  if world > 1:
    dist.barrier()
  sync()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    o, r, te, tr, _ = env.step(agent())
    exchange(o, r, te, tr)
  if world > 1:
    dist.barrier()
  sync()
  el = time.perf_counter() - t0
  if world > 1:
    t = torch.tensor([el], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
  stats = (env.step_stats() - stats0).double().cpu()
  flags = (env.sim.flag_stats()[3:] - flags0).cpu().tolist()  # world-passes in the timed window
  resets_per_step = float(stats[0]) / args.steps
  gate_rate = float(stats[1]) / args.steps
  n_total = num_envs * world
  value = n_total * args.steps / el

  # the per-step RCCL all-gather alone (same buffers), timed separately
  gather_ms = None
  if use_gather:
    sync()
    dist.barrier()
    tg = time.perf_counter()
    for _ in range(args.steps):
      exchange(o, r, te, tr)
    sync()
    gather_ms = (time.perf_counter() - tg) / args.steps * 1e3

  # ---- dominant kernel: the fused physics step, HIP events on its stream ----
  sim = env.sim
  nefc = sim.data.nefc.float().mean().item()
  niter = sim.data.solver_niter.float().mean().item()
  L = args.kernel_launches
  sim.step()
  if on_gpu:
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(L):
      sim.step()
    e1.record(stream)
    torch.cuda.synchronize()
    t_launch = e0.elapsed_time(e1) / 1e3 / L  # s per physics step (pack + step kernels)
  else:  # CPU test harness: host time of its stand-in physics (not a measurement)
    tl = time.perf_counter()
    for _ in range(L):
      sim.step()
    t_launch = (time.perf_counter() - tl) / L
  b_phys = next((v for k, v in B_PHYS.items() if k in args.task), B_PHYS_G1)
  bytes_per_launch = b_phys * num_envs
  achieved = bytes_per_launch / t_launch / 1e9
  traffic = None
  tf = REPO / "profiles" / "step_kernel_traffic.json"
  if tf.exists():
    try:
      tj = json.loads(tf.read_text())
      if int(tj.get("num_envs", -1)) == num_envs and tj.get("task", TASK) == args.task:
        traffic = tj.get("bytes_per_launch")
    except (ValueError, OSError):
      traffic = None
  # VALU roofline: SQ_INSTS_VALU of the step kernel(s) of one physics step, from
  # the committed counter summary of the same workload (tools/gpu_pmc_sq.sh ->
  # profiles/step_kernel_sq.json), over the live launch time: issue cycles
  # (2 per wave64 instruction) / SIMD-cycles available
  valu = None
  sqf = REPO / "profiles" / "step_kernel_sq.json"
  if sqf.exists():
    try:
      sj = json.loads(sqf.read_text())
      if int(sj.get("num_envs", -1)) == num_envs and sj.get("task", TASK) == args.task:
        ins = float(sj["valu_insts_per_launch"])
        gips = ins / t_launch / 1e9
        valu = {"bound": "valu", "achieved": gips, "peak": VALU_PEAK_GIPS, "unit": "G wave64-VALU-instr/s",
                "frac": gips / VALU_PEAK_GIPS, "insts_per_launch": ins, "source": sj.get("source", sqf.name),
                "model": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x launch time)"}
    except (ValueError, OSError, KeyError):
      valu = None
  nv = sim.mj_model.nv
  b_solve = niter * 4 * (nefc * nv + nv * nv + 6 * nefc + 4 * nv) + 4 * (nefc + 2 * nv)
  # what limits the step launch, from the committed SQ counters of the same workload
  # (profiles/step_kernel_sq.json): the share of wave-cycles spent waiting (SQ_WAIT_ANY)
  limiter = None
  if sqf.exists():
    try:
      sj = json.loads(sqf.read_text())
      if "wait_any_frac" in sj:
        limiter = {"kind": "latency", "sq_wait_any_frac": sj["wait_any_frac"], "source": sj.get("source", sqf.name),
                   "note": "per-world dependent chains (LDS/L2 round trips, readlane-serial factor sweeps): "
                           "SQ_WAIT_ANY / SQ_WAVE_CYCLES of the step kernel"}
    except (ValueError, OSError):
      limiter = None
  # the north-star solver figure (BASELINE.json: >= 40% of HBM roofline in the
  # constraint-solver kernel), measured on the split build's solver launch by
  # tools/gpu_solver_pmc.sh -> profiles/solver_roofline.json (same task, 4096 envs)
  solver_rl = None
  srf = REPO / "profiles" / "solver_roofline.json"
  if srf.exists():
    try:
      sr = json.loads(srf.read_text())
      if int(sr.get("num_envs", -1)) == num_envs and sr.get("task", TASK) == args.task:
        solver_rl = {"bound": "hbm", "kernel": sr.get("kernel"), "launch_us": sr.get("launch_us"),
                     "algorithmic_frac": sr.get("algorithmic_frac"), "counter_frac": sr.get("counter_frac"),
                     "achieved_algorithmic_gbs": sr.get("algorithmic_gbs"), "achieved_counter_gbs": sr.get("counter_gbs"),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "target_frac": 0.40, "head": sr.get("head"),
                     "gap": sr.get("gap"), "source": "profiles/solver_roofline.json (" + sr.get("source", "") + ")"}
    except (ValueError, OSError):
      solver_rl = None

  # algorithmic FLOPs per env step (SURVEY §8d / BASELINE.md): smooth dynamics,
  # collision over the pair table, and per Newton iteration the Hessian
  # (nefc nv(nv+1)), the factor (nv^3/3), gradient/J products (4 nefc nv) and
  # the line search (6 ls nefc, ls ~ 3 evaluations), with this run's mean nefc
  # and iterations; x decimation physics steps (+ the gated forward's pass)
  npair = int(sim.mj_model.npair)
  f_phys = 60e3 + 150 * npair + niter * (nefc * nv * (nv + 1) + nv ** 3 / 3 + 4 * nefc * nv + 6 * 3 * nefc)
  f_env = f_phys * (env.cfg.decimation + gate_rate)
  flops = {"per_env_step": f_env, "achieved_tflops": f_env * value / 1e12, "fp32_vector_peak_tflops": 157.3,
           "model": "60k + 150 npair + iters (nefc nv(nv+1) + nv^3/3 + 4 nefc nv + 18 nefc) per physics pass, "
                    "x (decimation + forward_gate_rate); mean nefc/iters of this run"}

  cpu = None
  if rank == 0 and world == 1 and not args.no_cpu_baseline:
    try:
      cpu = cpu_baseline(env, args)
    except Exception as e:  # noqa: BLE001 - a missing oracle build must not void the GPU line
      cpu = {"value": None, "unit": "env steps/sec", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}
    if args.task == TASK:
      try:
        cpu["config1"] = cpu_config1(args)
      except Exception as e:  # noqa: BLE001
        cpu["config1"] = {"value": None, "sample": f"unavailable: {e}"}

  if rank == 0:
    line = {
      "metric": METRIC if (args.task == TASK and num_envs == 4096) else f"env steps/sec (whole node), {args.task} @ {num_envs} envs/GPU",
      "value": value,
      "unit": "env steps/s",
      "n_gpus": world,
      "steps": args.steps,
      "warmup": args.warmup,
      "ms_per_step": el / args.steps * 1e3,
      "higher_is_better": True,
      "scaling": "weak",
      "vs_baseline": None,
      "dtype": "f32",
      "data": "synthetic: random agent 2*U[0,1)-1 (seed 1234+rank), env seed 42+rank, episode lengths start uniform "
      "(init_at_random_ep_len), DR/pushes/resets/commands on"
      + ("; synthetic 500-frame motion clip (mjlab_amd.motion)" if motion is not None and not args.motion_file else ""),
      "config": {
        "workload": f"{args.task}, num_envs={num_envs}/GPU, random agent",
        "num_envs_per_gpu": num_envs,
        "decimation": env.cfg.decimation,
        "physics_steps_per_s": value * env.cfg.decimation,
        "parallelism": f"env-sharded x{world}" + ("" if not use_gather else " + RCCL all-gather of obs/reward/dones"),
        "world_size": world,
        "settle_steps": settled,
        "resets_per_step": resets_per_step,
        "settle_tail_resets_per_step": tail_rate,
        "settle_block_resets_per_step": settle_log,
        "forward_gate_rate": gate_rate,
        "gather_ms_per_step": gather_ms,
        "mean_nefc": nefc,
        "mean_solver_iters": niter,
        "efc_capacity": sim.efc_capacity(),
        "njmax": int(sim.mj_model.njmax),
        "nconmax": int(sim.mj_model.nconmax),
        "nconmax_share": int(getattr(sim.mj_model, "ncon_share", sim.mj_model.nconmax)),
        # the step kernel instance: >= 0 a model-specialised one (csrc/mjh_spec_table.h), -1 the generic
        "spec_instance": int(_native().mjh_spec_index(ctypes.addressof(sim._mstruct))),
        # which instance ran: "builtin" (the table above), "plugin" (compiled for this
        # model's plan, mjlab_amd/sim/jit.py) or "generic"
        "kernel_instance": sim.kernel_instance()["kind"],
        "contact_overflow_worlds": int(flags[0]),
        "efc_overflow_worlds": int(flags[1]),
        "nonfinite_worlds": int(flags[2]),
        "overflow_window": f"world-physics-passes flagged over the {args.steps} timed env steps (5 passes each)",
      },
      "flops": flops,
      "roofline": {
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "kernel": "step_kernel (+pack_kernel), one launch per physics step",
        "launch_us": t_launch * 1e6,
        "bytes_per_launch": bytes_per_launch,
        "solver_streamed_model_gbs": b_solve * num_envs / t_launch / 1e9,
        "limiter": limiter,
      },
      "roofline_solver": solver_rl,
      "roofline_valu": valu,
      "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
  if world > 1:
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
