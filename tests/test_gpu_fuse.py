"""Fused reset-path / event / command kernels (csrc/mjh_fuse.hip) vs the torch
formulas they replace (managers/*.py, envs/mdp/events.py, velocity_command.py),
fed the same U[0,1) draws (reconstructed from the device stream with
envops.uniform_draws)."""

import ctypes

import pytest
import torch

from mjlab_amd import envops
from mjlab_amd.sim import native
from mjlab_amd.utils import math as M

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SEED, KEY = 1234567, 987654321


def _ctr(v: int) -> torch.Tensor:
  return torch.full((), v, dtype=torch.long, device=DEV)


def _args(ctr):
  return ctypes.c_ulonglong(SEED), ctypes.c_ulonglong(KEY), envops._ptr(ctr)


def _s():
  return envops._stream()


def test_draws_are_uniform_and_keyed():
  c0, c1 = _ctr(5), _ctr(6)
  a = envops.uniform_draws(SEED, KEY, c0, 1 << 20, DEV)
  b = envops.uniform_draws(SEED, KEY, c1, 1 << 20, DEV)
  c = envops.uniform_draws(SEED, KEY + 1, c0, 1 << 20, DEV)
  assert 0.0 <= a.min().item() and a.max().item() < 1.0
  assert abs(a.mean().item() - 0.5) < 2e-3 and abs(a.var().item() - 1 / 12) < 2e-3
  # different step counter / key: a different stream
  assert (a == b).float().mean().item() < 1e-3 and (a == c).float().mean().item() < 1e-3
  assert torch.equal(a, envops.uniform_draws(SEED, KEY, c0, 1 << 20, DEV))
  # consecutive draws uncorrelated
  x = a.view(-1, 2)
  assert abs(torch.corrcoef(x.T)[0, 1].item()) < 5e-3


def test_masked_means_and_counts_match_torch():
  g = torch.Generator(device=DEV).manual_seed(0)
  n, t = 4096, 12
  sums = torch.randn(n, t, device=DEV, generator=g)
  m = torch.rand(n, device=DEV, generator=g) < 0.1
  ref_means = (sums * m.float()[:, None]).sum(0) / (m.float().sum().clamp(min=1.0) * 20.0)
  ref_sums = sums.masked_fill(m[:, None], 0.0)
  out = torch.zeros(t, device=DEV)
  assert envops.masked_means([sums[:, i] for i in range(t)], m, 1 / 20.0, True, out)
  torch.testing.assert_close(out, ref_means, rtol=1e-5, atol=1e-6)
  assert torch.equal(sums, ref_sums)
  # empty mask: the outputs keep their last values (the reference logs episode
  # statistics only from _reset_idx, i.e. only when some env resets), nothing cleared
  z = torch.zeros(n, dtype=torch.bool, device=DEV)
  v = torch.randn(n, device=DEV, generator=g)
  v0 = v.clone()
  held = out.clone()
  assert envops.masked_means([v], z, 1.0, True, out)
  assert torch.equal(out, held) and torch.equal(v, v0)
  flags = [torch.rand(n, device=DEV, generator=g) < p for p in (0.01, 0.5, 0.0, 1.0)]
  cnt = torch.zeros(4, dtype=torch.long, device=DEV)
  assert envops.masked_counts(flags, m, cnt)
  assert cnt.tolist() == [int((f & m).sum()) for f in flags]
  held = cnt.clone()
  assert envops.masked_counts(flags, z, cnt)
  assert torch.equal(cnt, held)


def test_uniform_where_and_interval_tick():
  n = 4096
  g = torch.Generator(device=DEV).manual_seed(1)
  ctr = _ctr(3)
  u = envops.uniform_draws(SEED, KEY, ctr, n, DEV)
  t = torch.rand(n, device=DEV, generator=g)
  m = torch.rand(n, device=DEV, generator=g) < 0.3
  ref = torch.where(m, u * (5.0 - 2.0) + 2.0, t)
  native.check(native.lib().mjh_uniform_where(envops._ptr(t), envops._ptr(m), 2.0, 5.0, *_args(ctr), n, _s()), "uw")
  torch.testing.assert_close(t, ref, rtol=0, atol=1e-6)
  # interval events: t -= dt; due = t < 1e-6; redraw (event_manager.py:120-145)
  t = torch.rand(n, device=DEV, generator=g) * 0.05
  due = torch.zeros(n, dtype=torch.bool, device=DEV)
  tt = t - 0.02
  ref_due = tt < 1e-6
  ref = torch.where(ref_due, u * (15.0 - 10.0) + 10.0, tt)
  native.check(native.lib().mjh_interval_tick(envops._ptr(t), 0.02, 10.0, 15.0, envops._ptr(due), *_args(ctr), n, _s()), "it")
  assert torch.equal(due, ref_due)
  torch.testing.assert_close(t, ref, rtol=0, atol=1e-6)


def _rows(n, k, g):
  return torch.randn(n, k, device=DEV, generator=g)


def test_reset_root_uniform_matches_events_formula():
  n = 2048
  g = torch.Generator(device=DEV).manual_seed(2)
  ctr = _ctr(7)
  nq, nv, qa, va = 40, 38, 2, 1
  qpos, qvel = _rows(n, nq, g), _rows(n, nv, g)
  q0 = qpos.clone()
  v0 = qvel.clone()
  rs = _rows(n, 13, g)
  rs[:, 3:7] = rs[:, 3:7] / rs[:, 3:7].norm(dim=1, keepdim=True)
  org = _rows(n, 3, g)
  m = torch.rand(n, device=DEV, generator=g) < 0.4
  plo, phi = [-0.5, -0.5, 0.0, -0.1, -0.2, -3.14], [0.5, 0.5, 0.0, 0.1, 0.2, 3.14]
  vlo, vhi = [-0.5] * 6, [0.5] * 6
  u = envops.uniform_draws(SEED, KEY, ctr, n * 12, DEV).view(n, 12)
  pose = u[:, :6] * (torch.tensor(phi, device=DEV) - torch.tensor(plo, device=DEV)) + torch.tensor(plo, device=DEV)
  dv = u[:, 6:] * (torch.tensor(vhi, device=DEV) - torch.tensor(vlo, device=DEV)) + torch.tensor(vlo, device=DEV)
  pos = rs[:, 0:3] + pose[:, 0:3] + org
  quat = M.quat_mul(rs[:, 3:7], M.quat_from_euler_xyz(pose[:, 3], pose[:, 4], pose[:, 5]))
  vel = rs[:, 7:13] + dv
  ref_q, ref_v = q0.clone(), v0.clone()
  ref_q[:, qa:qa + 7] = torch.where(m[:, None], torch.cat([pos, quat], 1), q0[:, qa:qa + 7])
  qv = torch.cat([vel[:, :3], M.quat_apply_inverse(quat, vel[:, 3:])], 1)
  ref_v[:, va:va + 6] = torch.where(m[:, None], qv, v0[:, va:va + 6])
  F = (ctypes.c_float * 6)
  native.check(native.lib().mjh_reset_root_uniform(
    envops._ptr(qpos), nq, qa, envops._ptr(qvel), nv, va, envops._ptr(m), envops._ptr(rs), 13, envops._ptr(org), 3,
    F(*plo), F(*phi), F(*vlo), F(*vhi), 1, 1, *_args(ctr), n, _s()), "rr")
  torch.testing.assert_close(qpos, ref_q, rtol=1e-5, atol=2e-6)
  torch.testing.assert_close(qvel, ref_v, rtol=1e-5, atol=2e-6)


def test_reset_joints_offset_matches_events_formula():
  n, k = 2048, 29
  g = torch.Generator(device=DEV).manual_seed(3)
  ctr = _ctr(9)
  qpos, qvel = _rows(n, 36, g), _rows(n, 35, g)
  q0, v0 = qpos.clone(), qvel.clone()
  dp, dv = _rows(n, k, g), _rows(n, k, g)
  lo = _rows(n, k, g) - 1.0
  lim = torch.stack([lo, lo + 1.5], dim=-1)
  m = torch.rand(n, device=DEV, generator=g) < 0.5
  u = envops.uniform_draws(SEED, KEY, ctr, n * 2 * k, DEV).view(n, 2 * k)
  jp = (dp + u[:, :k] * (0.3 + 0.2) - 0.2).clamp(lim[..., 0], lim[..., 1])
  jv = dv + u[:, k:] * (0.1 + 0.1) - 0.1
  ref_q, ref_v = q0.clone(), v0.clone()
  ref_q[:, 7:] = torch.where(m[:, None], jp, q0[:, 7:])
  ref_v[:, 6:] = torch.where(m[:, None], jv, v0[:, 6:])
  native.check(native.lib().mjh_reset_joints_offset(
    envops._ptr(qpos), 36, 7, envops._ptr(qvel), 35, 6, k, envops._ptr(m), envops._ptr(dp), k, envops._ptr(dv), k,
    envops._ptr(lim), 2 * k, -0.2, 0.3, -0.1, 0.1, 1, 1, *_args(ctr), n, _s()), "rj")
  torch.testing.assert_close(qpos, ref_q, rtol=1e-6, atol=1e-6)
  torch.testing.assert_close(qvel, ref_v, rtol=1e-6, atol=1e-6)


def test_push_velocity_matches_events_formula():
  n = 2048
  g = torch.Generator(device=DEV).manual_seed(4)
  ctr = _ctr(11)
  qpos, qvel = _rows(n, 36, g), _rows(n, 35, g)
  qpos[:, 3:7] = qpos[:, 3:7] / qpos[:, 3:7].norm(dim=1, keepdim=True)
  v0 = qvel.clone()
  vw = _rows(n, 6, g)
  m = torch.rand(n, device=DEV, generator=g) < 0.2
  lo, hi = [-0.5, -0.5, 0.0, 0.0, 0.0, 0.0], [0.5, 0.5, 0.0, 0.0, 0.0, 0.0]
  u = envops.uniform_draws(SEED, KEY, ctr, n * 6, DEV).view(n, 6)
  vel = vw + u * (torch.tensor(hi, device=DEV) - torch.tensor(lo, device=DEV)) + torch.tensor(lo, device=DEV)
  qv = torch.cat([vel[:, :3], M.quat_apply_inverse(qpos[:, 3:7], vel[:, 3:])], 1)
  ref_v = v0.clone()
  ref_v[:, 0:6] = torch.where(m[:, None], qv, v0[:, 0:6])
  F = (ctypes.c_float * 6)
  native.check(native.lib().mjh_push_velocity(envops._ptr(qpos), 36, 0, envops._ptr(qvel), 35, 0, envops._ptr(m),
                                              envops._ptr(vw), 6, F(*lo), F(*hi), *_args(ctr), n, _s()), "pv")
  torch.testing.assert_close(qvel, ref_v, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("reset", [0, 1])
def test_velocity_resample_matches_command_formula(reset):
  n = 4096
  g = torch.Generator(device=DEV).manual_seed(5)
  ctr = _ctr(13)
  ranges = torch.tensor([[-1.0, 1.0], [-0.5, 0.5], [-1.0, 1.0], [-3.14, 3.14]], device=DEV)
  cmd, ht = _rows(n, 3, g), _rows(n, 1, g)[:, 0].contiguous()
  ih = torch.rand(n, device=DEV, generator=g) < 0.5
  isd = torch.rand(n, device=DEV, generator=g) < 0.5
  tl = torch.rand(n, device=DEV, generator=g)
  cnt = torch.randint(0, 5, (n,), device=DEV, generator=g)
  m = torch.rand(n, device=DEV, generator=g) < 0.3
  u = envops.uniform_draws(SEED, KEY, ctr, n * 8, DEV).view(n, 8)
  r_tl = torch.where(m, u[:, 0] * (10.0 - 3.0) + 3.0, tl)
  new = u[:, 1:5] * (ranges[:, 1] - ranges[:, 0]) + ranges[:, 0]
  r_cmd = torch.where(m[:, None], new[:, :3], cmd)
  r_ht = torch.where(m, new[:, 3], ht)
  r_ih = torch.where(m, u[:, 5] <= 1.0, ih)
  r_isd = torch.where(m, u[:, 6] <= 0.1, isd)
  r_cnt = torch.where(m, torch.ones_like(cnt) if reset else cnt + 1, cnt)
  P = envops._ptr
  native.check(native.lib().mjh_velocity_resample(P(m), P(ranges), 3.0, 10.0, 1.0, 0.1, 1, reset, P(cmd), P(ht), P(ih),
                                                  P(isd), P(tl), P(cnt), *_args(ctr), n, _s()), "vr")
  torch.testing.assert_close(tl, r_tl, rtol=0, atol=1e-6)
  torch.testing.assert_close(cmd, r_cmd, rtol=0, atol=1e-6)
  torch.testing.assert_close(ht, r_ht, rtol=0, atol=1e-6)
  assert torch.equal(ih, r_ih) and torch.equal(isd, r_isd) and torch.equal(cnt, r_cnt)


def test_event_mark():
  n = 1000
  g = torch.Generator(device=DEV).manual_seed(6)
  last = torch.randint(0, 50, (n,), dtype=torch.int32, device=DEV, generator=g)
  once = torch.rand(n, device=DEV, generator=g) < 0.5
  m = torch.rand(n, device=DEV, generator=g) < 0.5
  step = _ctr(77)
  r_last = torch.where(m, torch.full_like(last, 77), last)
  r_once = once | m
  assert envops.event_mark(last, once, m, step)
  assert torch.equal(last, r_last) and torch.equal(once, r_once)


def test_term_combine_matches_manager_formula():
  n = 4096
  g = torch.Generator(device=DEV).manual_seed(7)
  vals = [torch.rand(n, device=DEV, generator=g) < p for p in (0.02, 0.3, 0.0, 0.5)]
  time_out = [True, False, False, True]
  dones = [torch.zeros(n, dtype=torch.bool, device=DEV) for _ in vals]
  tr, te, dn = (torch.ones(n, dtype=torch.bool, device=DEV) for _ in range(3))
  assert envops.term_combine(vals, dones, time_out, tr, te, dn)
  r_tr = vals[0] | vals[3]
  r_te = vals[1] | vals[2]
  assert torch.equal(tr, r_tr) and torch.equal(te, r_te) and torch.equal(dn, r_tr | r_te)
  assert all(torch.equal(d, v) for d, v in zip(dones, vals))


@pytest.mark.parametrize("n", [1, 1000, 5000])
def test_step_counters_and_reset_stats(n):
  g = torch.Generator(device=DEV).manual_seed(8)
  ep = torch.randint(0, 900, (n,), dtype=torch.long, device=DEV, generator=g)
  r_ep = ep + 1
  step = _ctr(41)
  envops.step_counters(ep, step)
  assert torch.equal(ep, r_ep) and int(step) == 42
  for p in (0.0, 0.01, 1.0):
    reset = torch.rand(n, device=DEV, generator=g) < p
    anyr = torch.ones(1, dtype=torch.bool, device=DEV)
    stats = torch.tensor([5, 3], dtype=torch.long, device=DEV)
    envops.reset_stats(reset, anyr, stats)
    c = int(reset.sum())
    assert bool(anyr) == (c > 0)
    assert stats.tolist() == [5 + c, 3 + (1 if c > 0 else 0)]


def test_env_reset_path_uses_fused_kernels():
  """A captured velocity-task env step runs the fused reset path (C-ABI tally)
  and keeps its invariants: reset envs restart at step 0 with fresh commands."""
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 256
  env = ManagerBasedRlEnv(cfg, device=DEV)
  env.reset()
  native.CALLS.clear()
  a = torch.zeros(256, env.action_manager.total_action_dim, device=DEV)
  env.step(a)  # eager
  for name in ("mjh_masked_means", "mjh_masked_counts", "mjh_reset_root_uniform", "mjh_reset_joints_offset",
               "mjh_velocity_resample", "mjh_event_mark", "mjh_interval_tick", "mjh_term_combine"):
    assert native.CALLS[name] >= 1, name
  env.episode_length_buf.fill_(int(env.max_episode_length) - 1)  # every env times out at the next step
  cmd_before = env.command_manager.get_command("twist").clone()
  _, _, _, trunc, _ = env.step(a)
  torch.cuda.synchronize()
  assert trunc.all() and (env.episode_length_buf == 0).all()
  assert not torch.equal(env.command_manager.get_command("twist"), cmd_before)
  t = env.command_manager.get_term("twist")
  assert (t.command_counter == 1).all()
  lo, hi = t.cfg.resampling_time_range
  assert ((t.time_left >= lo - env.step_dt) & (t.time_left <= hi)).all()
  q = env.sim.data.qpos
  assert torch.isfinite(q).all() and torch.allclose(q[:, 3:7].norm(dim=1), torch.ones(256, device=DEV), atol=1e-5)


@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_obs_group_ops_and_strides(op):
  """Observation terms given as ObsSrc (strided inputs + elementwise op) are
  evaluated inside the group kernel exactly as ObsSrc.evaluate's torch formula."""
  from mjlab_amd.managers.manager_term_config import ObservationTermCfg

  n = 4096
  g = torch.Generator(device=DEV).manual_seed(10 + op)
  base = torch.randn(n, 40, device=DEV, generator=g) * 3
  x = base[:, 2:30:4]  # (n, 7) with column stride 4
  y = torch.randn(n, 7, device=DEV, generator=g)
  src = envops.ObsSrc(x, op, y if op == envops.OBS_SUB else None)
  other = torch.randn(n, 3, device=DEV, generator=g)
  tc = ObservationTermCfg(func=lambda env: None)
  plan = [(tc, 0, 3, (-0.1, 0.1), None, 1.0), (tc, 3, 7, (-0.5, 0.5), (-2.0, 2.0), 0.25)]
  u = torch.rand(n, 10, device=DEV, generator=g)
  out = torch.empty(n, 10, device=DEV)
  assert envops.obs_group([other, src], plan, u, out)
  ref1 = other + (u[:, :3] * 0.2 - 0.1)
  ref2 = (src.evaluate() + (u[:, 3:] * 1.0 - 0.5)).clamp(-2.0, 2.0) * 0.25
  torch.testing.assert_close(out[:, :3], ref1, rtol=1e-6, atol=1e-6)
  torch.testing.assert_close(out[:, 3:], ref2, rtol=1e-5, atol=1e-6)
  # noise from the device stream: element e * width + column
  ctr = _ctr(21)
  out2 = torch.empty(n, 10, device=DEV)
  assert envops.obs_group([other, src], plan, None, out2, _args(ctr))
  uu = envops.uniform_draws(SEED, KEY, ctr, n * 10, DEV).view(n, 10)
  torch.testing.assert_close(out2[:, :3], other + (uu[:, :3] * 0.2 - 0.1), rtol=1e-6, atol=1e-6)


def test_velocity_rows_masked_zero_sum_ratios():
  from mjlab_amd.entity.data import compute_velocity_from_cvel

  n, nb = 2048, 30
  g = torch.Generator(device=DEV).manual_seed(30)
  xpos = torch.randn(n, nb, 3, device=DEV, generator=g)
  cvel = torch.randn(n, nb, 6, device=DEV, generator=g)
  com = torch.randn(n, nb, 3, device=DEV, generator=g)
  rows = slice(1, 8)
  body = torch.tensor([1, 4, 4, 9, 2, 29, 0], dtype=torch.int32, device=DEV)
  got = envops.velocity_rows(xpos[:, rows], com[:, 0], cvel, body)
  ref = compute_velocity_from_cvel(xpos[:, rows], com[:, 0].unsqueeze(1), cvel[:, body.long()])
  torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
  a, b = torch.randn(n, 5, device=DEV, generator=g), torch.randn(n, device=DEV, generator=g)
  big = torch.randn(n, 20, device=DEV, generator=g)
  c = big[:, 4:10]  # column slice of a wider tensor
  m = torch.rand(n, device=DEV, generator=g) < 0.3
  ra, rb, rbig = a.masked_fill(m[:, None], 0.0), b.masked_fill(m, 0.0), big.clone()
  rbig[:, 4:10] = rbig[:, 4:10].masked_fill(m[:, None], 0.0)
  assert envops.masked_zero([a, b, c], m)
  assert torch.equal(a, ra) and torch.equal(b, rb) and torch.equal(big, rbig)
  nums = [torch.rand(n, device=DEV, generator=g) for _ in range(3)]
  dens = [torch.rand(n, device=DEV, generator=g) > 0.5, torch.zeros(n, device=DEV), torch.rand(n, device=DEV, generator=g)]
  dens = [d.float() for d in dens]
  out = torch.zeros(3, device=DEV)
  assert envops.sum_ratios(list(zip(nums, dens)), out)
  ref = torch.stack([x.sum() / torch.clamp(y.sum(), min=1) for x, y in zip(nums, dens)])
  torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-6)


def test_contact_timing_rewards_match_formulas():
  """feet_air_time / feet_swing_height / soft_landing kernels vs the torch
  formulas of tasks/velocity/mdp/rewards.py (sensor slots as strided views)."""
  n, k = 4096, 2
  g = torch.Generator(device=DEV).manual_seed(31)
  cmd = torch.randn(n, 3, device=DEV, generator=g) * 0.3
  t = torch.rand(n, k, device=DEV, generator=g) * 0.6 * (torch.rand(n, k, device=DEV, generator=g) > 0.3)
  total = torch.norm(cmd[:, :2], dim=1) + torch.abs(cmd[:, 2])
  out, num, den = envops.rew_air_time(t, cmd, 0.05, 0.5, 0.5)
  act = (total > 0.5).float()
  torch.testing.assert_close(out, torch.sum(((t > 0.05) & (t < 0.5)).float(), 1) * act)
  in_air = (t > 0).float()
  torch.testing.assert_close(num, (t * in_air).sum(1))
  torch.testing.assert_close(den, in_air.sum(1))
  # sensordata-like slots: [found, fx, fy, fz] per foot -> strided views
  sd = torch.randn(n, 4 * k + 3, device=DEV, generator=g)
  sd[:, 0:4 * k:4] = (torch.rand(n, k, device=DEV, generator=g) > 0.5).float() * 2
  found = sd[:, 0:4 * k:4]
  force = sd.as_strided((n, k, 3), (sd.stride(0), 4, 1), sd.storage_offset() + 1)
  cct = torch.rand(n, k, device=DEV, generator=g) * 0.04 * (torch.rand(n, k, device=DEV, generator=g) > 0.4)
  site = torch.randn(n, 6, 3, device=DEV, generator=g).abs()
  h = site[:, 2:4, 2]
  peak = torch.rand(n, k, device=DEV, generator=g) * 0.2
  peak_ref = peak.clone()
  lim = 0.02 + 1e-8
  cost, pn, pd = envops.rew_swing_height(peak, h, found, cct, cmd, lim, 0.1, 0.05)
  a2 = (total > 0.05).float()
  peak_ref = torch.where(found == 0, torch.maximum(peak_ref, h), peak_ref)
  first = (cct > 0) & (cct < lim)
  ref_cost = torch.sum(torch.square(peak_ref / 0.1 - 1.0) * first.float(), dim=1) * a2
  torch.testing.assert_close(cost, ref_cost, rtol=1e-5, atol=1e-6)
  torch.testing.assert_close(pn, (peak_ref * first.float()).sum(1), rtol=1e-5, atol=1e-6)
  torch.testing.assert_close(pd, first.float().sum(1))
  assert torch.equal(peak, peak_ref.masked_fill(first, 0.0))
  lc, ln, ld = envops.rew_soft_landing(force, cct, cmd, lim, 0.05)
  impact = torch.norm(force, dim=-1) * first.float()
  torch.testing.assert_close(lc, impact.sum(1) * a2, rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(ln, impact.sum(1), rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(ld, first.float().sum(1))


def test_root_frame_and_joint_action_match_formulas():
  from mjlab_amd.entity.data import compute_velocity_from_cvel

  n = 4096
  g = torch.Generator(device=DEV).manual_seed(40)
  xpos, com = torch.randn(n, 5, 3, device=DEV, generator=g), torch.randn(n, 5, 3, device=DEV, generator=g)
  xquat = torch.randn(n, 5, 4, device=DEV, generator=g)
  xquat = xquat / xquat.norm(dim=-1, keepdim=True)
  cvel = torch.randn(n, 5, 6, device=DEV, generator=g)
  grav = torch.tensor([0.0, 0.0, -1.0], device=DEV).repeat(n, 1)
  fwd = torch.tensor([1.0, 0.0, 0.0], device=DEV).repeat(n, 1)
  r = 1
  out = envops.root_frame(xpos[:, r], xquat[:, r], com[:, r], cvel[:, r], grav, fwd)
  q = xquat[:, r]
  v = compute_velocity_from_cvel(xpos[:, r], com[:, r], cvel[:, r])
  f = M.quat_apply(q, fwd)
  ref = torch.cat([v, M.quat_apply_inverse(q, v[:, :3]), M.quat_apply_inverse(q, v[:, 3:]), M.quat_apply_inverse(q, grav),
                   torch.atan2(f[:, 1], f[:, 0])[:, None]], dim=1)
  torch.testing.assert_close(out, ref, rtol=1e-5, atol=2e-5)
  d = 29
  inp = torch.randn(n, d, device=DEV, generator=g)
  action, raw, proc = torch.randn(n, d, device=DEV, generator=g), torch.zeros(n, d, device=DEV), torch.zeros(n, d, device=DEV)
  prev = torch.zeros(n, d, device=DEV)
  a0 = action.clone()
  scale, offset = torch.rand(n, d, device=DEV, generator=g), torch.randn(n, d, device=DEV, generator=g)
  assert envops.joint_action(inp, action, prev, raw, proc, scale, offset)
  assert torch.equal(prev, a0) and torch.equal(action, inp) and torch.equal(raw, inp)
  torch.testing.assert_close(proc, torch.addcmul(offset, inp, scale), rtol=1e-6, atol=1e-6)
  assert envops.joint_action(inp, action, prev, raw, proc, 0.5, offset)
  torch.testing.assert_close(proc, offset + inp * 0.5, rtol=1e-6, atol=1e-6)


def test_motion_command_kernels_match_formulas():
  """Tracking MotionCommand: adaptive sampling, frame refresh and the resampled
  robot state vs the torch formulas of tasks/tracking/mdp/commands.py fed the
  same device-stream draws."""
  import math

  n, B, K, T = 4096, 11, 3, 500
  g = torch.Generator(device=DEV).manual_seed(50)
  ctr = _ctr(61)
  mask = torch.rand(n, device=DEV, generator=g) < 0.2
  term = torch.rand(n, device=DEV, generator=g) < 0.5
  ts = torch.randint(0, T, (n,), device=DEV, generator=g)
  ts0 = ts.clone()
  bin_failed = torch.rand(B, device=DEV, generator=g)
  cur = torch.zeros(B, device=DEV)
  kern = torch.tensor([0.8 ** i for i in range(K)], device=DEV)
  kern = kern / kern.sum()
  met = [torch.zeros(n, device=DEV) for _ in range(3)]
  P = envops._ptr
  native.check(native.lib().mjh_motion_adaptive(P(mask), P(term), P(ts), P(bin_failed), P(cur), P(kern), B, K, T, 0.1,
                                                *[P(x) for x in met], *_args(ctr), n, _s()), "ma")
  failed = mask & term
  cb = torch.clamp((ts0 * B) // T, 0, B - 1)
  ref_cur = torch.zeros(B, device=DEV).scatter_add_(0, cb, failed.float())
  torch.testing.assert_close(cur, ref_cur)
  p = bin_failed + 0.1 / B
  idx = torch.clamp(torch.arange(B, device=DEV)[:, None] + torch.arange(K, device=DEV)[None], max=B - 1)
  p = (p[idx] * kern[None]).sum(-1)
  p = p / p.sum()
  cdf = torch.cumsum(p.double(), 0)
  u = envops.uniform_draws(SEED, KEY, ctr, 2 * n, DEV).view(n, 2)
  bins = torch.searchsorted(cdf, (u[:, 0].double() * cdf[-1]).contiguous(), right=True).clamp_(max=B - 1)
  new = ((bins.float() + u[:, 1]) / B * (T - 1)).long()
  ref_ts = torch.where(mask, new, ts0)
  assert (ts != ref_ts).float().mean().item() < 1e-3  # bin boundaries: float32 vs float64 CDF
  H = -(p * (p + 1e-12).log()).sum()
  torch.testing.assert_close(met[0], (H / math.log(B)).expand(n), rtol=1e-5, atol=1e-6)
  torch.testing.assert_close(met[1], p.max().expand(n), rtol=1e-5, atol=1e-6)
  torch.testing.assert_close(met[2], (p.argmax().float() / B).expand(n))
  # frame refresh
  nj, nb = 29, 14
  W = 2 * nj + 13 * nb
  table = torch.randn(T, W, device=DEV, generator=g)
  frame = torch.zeros(n, W, device=DEV)
  bpw = torch.zeros(n, nb, 3, device=DEV)
  org = torch.randn(n, 3, device=DEV, generator=g)
  native.check(native.lib().mjh_motion_frame(P(table), P(ts), P(frame), W, 2 * nj, nb, P(bpw), P(org), 3, n, _s()), "mf")
  ref_frame = table[ts]
  assert torch.equal(frame, ref_frame)
  torch.testing.assert_close(bpw, ref_frame[:, 2 * nj:2 * nj + 3 * nb].view(n, nb, 3) + org[:, None, :])
  # resampled robot state
  q = frame[:, 2 * nj + 3 * nb:2 * nj + 7 * nb].view(n, nb, 4)
  q /= q.norm(dim=-1, keepdim=True)
  qpos, qvel = torch.zeros(n, 7 + nj, device=DEV), torch.zeros(n, 6 + nj, device=DEV)
  lo = torch.rand(n, nj, device=DEV, generator=g) - 1.5
  lim = torch.stack([lo, lo + 2.0], -1).contiguous()
  F6 = ctypes.c_float * 6
  pr = ([-0.05, -0.05, -0.01, -0.1, -0.1, -0.2], [0.05, 0.05, 0.01, 0.1, 0.1, 0.2])
  vr = ([-0.5, -0.5, -0.2, -0.52, -0.52, -0.78], [0.5, 0.5, 0.2, 0.52, 0.52, 0.78])
  ctr2 = _ctr(62)
  native.check(native.lib().mjh_motion_reset(
    P(frame), W, nj, 2 * nj, 2 * nj + 3 * nb, 2 * nj + 7 * nb, 2 * nj + 10 * nb, P(bpw), 3 * nb, P(mask), F6(*pr[0]),
    F6(*pr[1]), F6(*vr[0]), F6(*vr[1]), 1, 1, -0.52, 0.52, P(lim), 2 * nj, P(qpos), 7 + nj, 0, 7, P(qvel), 6 + nj, 0, 6,
    *_args(ctr2), n, _s()), "mr")
  S = 12 + nj
  uu = envops.uniform_draws(SEED, KEY, ctr2, n * S, DEV).view(n, S)
  T6 = lambda v: torch.tensor(v, device=DEV)  # noqa: E731
  rp = uu[:, 0:6] * (T6(pr[1]) - T6(pr[0])) + T6(pr[0])
  rv = uu[:, 6:12] * (T6(vr[1]) - T6(vr[0])) + T6(vr[0])
  root_pos = bpw[:, 0] + rp[:, 0:3]
  root_q = M.quat_mul(M.quat_from_euler_xyz(rp[:, 3], rp[:, 4], rp[:, 5]), q[:, 0])
  lin = frame[:, 2 * nj + 7 * nb:2 * nj + 7 * nb + 3] + rv[:, 0:3]
  ang = frame[:, 2 * nj + 10 * nb:2 * nj + 10 * nb + 3] + rv[:, 3:6]
  jp = torch.clip(frame[:, :nj] + (uu[:, 12:] * 1.04 - 0.52), lim[:, :, 0], lim[:, :, 1])
  ref_q = torch.cat([root_pos, root_q, jp], 1)
  ref_v = torch.cat([lin, M.quat_apply_inverse(root_q, ang), frame[:, nj:2 * nj]], 1)
  m2 = mask[:, None]
  torch.testing.assert_close(qpos, torch.where(m2, ref_q, 0.0), rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(qvel, torch.where(m2, ref_v, 0.0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("quat", [False, True])
def test_rew_exp_err_matches_tracking_formula(quat):
  n, nb, nbe = 4096, 14, 30
  d = 4 if quat else 3
  g = torch.Generator(device=DEV).manual_seed(70 + quat)
  a = torch.randn(n, nb, d, device=DEV, generator=g)
  big = torch.randn(n, nbe, 6 if not quat else 4, device=DEV, generator=g)
  b = big[..., :d]
  if quat:
    a, b = a / a.norm(dim=-1, keepdim=True), b / b.norm(dim=-1, keepdim=True)
  ra = torch.tensor([0, 3, 5, 13], dtype=torch.int32, device=DEV)
  rb = torch.tensor([1, 7, 2, 29], dtype=torch.int32, device=DEV)
  out = envops.rew_exp_err(a, b, 0.3, quat, ra, rb)
  x, y = a[:, ra.long()], b[:, rb.long()]
  err = M.quat_error_magnitude(x, y) ** 2 if quat else torch.sum(torch.square(x - y), dim=-1)
  torch.testing.assert_close(out, torch.exp(-err.mean(-1) / 0.09), rtol=2e-5, atol=1e-6)



def test_obs_src_rows_of_slot_records():
  """(n, k, 3) force slots at a row stride of 4 (sensordata records) flattened in-kernel."""
  from mjlab_amd.managers.manager_term_config import ObservationTermCfg

  n, k = 2048, 2
  g = torch.Generator(device=DEV).manual_seed(80)
  sd = torch.randn(n, 4 * k + 1, device=DEV, generator=g) * 50
  f = sd.as_strided((n, k, 3), (sd.stride(0), 4, 1), sd.storage_offset() + 1)
  src = envops.ObsSrc(f, envops.OBS_SIGNED_LOG1P)
  tc = ObservationTermCfg(func=lambda env: None)
  out = torch.empty(n, 3 * k, device=DEV)
  assert envops.obs_group([src], [(tc, 0, 3 * k, None, None, 1.0)], None, out)
  ff = f.reshape(n, -1)
  torch.testing.assert_close(out, torch.sign(ff) * torch.log1p(torch.abs(ff)), rtol=1e-6, atol=1e-6)
