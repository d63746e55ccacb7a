"""Fused env-layer kernels (csrc/mjh_envops.hip) vs their torch formulas."""

import pytest
import torch

from mjlab_amd import envops
from mjlab_amd.entity.data import compute_velocity_from_cvel
from mjlab_amd.utils import math as M

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _q(n, g):
  q = torch.randn(n, 4, generator=g, device=DEV)
  return q / q.norm(dim=-1, keepdim=True)


def test_quat_kernels_match_torch():
  g = torch.Generator(device=DEV).manual_seed(0)
  n = 5000
  pose = torch.cat([torch.randn(n, 3, device=DEV, generator=g), _q(n, g)], dim=1)  # strided quaternion view
  q = pose[:, 3:7]
  vel = torch.randn(n, 6, device=DEV, generator=g)
  v = vel[:, 0:3]
  torch.testing.assert_close(envops.quat_apply_inverse(q, v), M.quat_apply_inverse(q, v), rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(envops.quat_apply(q, v), M.quat_apply(q, v), rtol=1e-5, atol=1e-5)
  q2 = _q(n, g)
  torch.testing.assert_close(envops.quat_mul(q, q2), M.quat_mul(q.contiguous(), q2), rtol=1e-5, atol=1e-5)
  qb = q2[:1].expand(n, -1)  # row stride 0 broadcast
  torch.testing.assert_close(envops.quat_mul(q, qb), M.quat_mul(q.contiguous(), qb.contiguous()), rtol=1e-5, atol=1e-5)


def test_velocity_from_cvel_matches_torch():
  g = torch.Generator(device=DEV).manual_seed(1)
  n = 3000
  xpos, com, cvel = (torch.randn(n, k, device=DEV, generator=g) for k in (3, 3, 6))
  torch.testing.assert_close(
    envops.velocity_from_cvel(xpos, com, cvel, compute_velocity_from_cvel), compute_velocity_from_cvel(xpos, com, cvel),
    rtol=1e-5, atol=1e-5,
  )


def test_air_time_kernel_matches_torch_rule():
  g = torch.Generator(device=DEV).manual_seed(2)
  n, k = 1000, 2
  sd = torch.zeros(n, 7, device=DEV)
  cols = torch.tensor([1, 5], dtype=torch.int32, device=DEV)
  st = [torch.rand(n, k, device=DEV, generator=g) * (torch.rand(n, k, device=DEV, generator=g) > 0.5) for _ in range(4)]
  last_time = torch.rand(n, device=DEV, generator=g)
  time = last_time + 0.005
  sd[:, 1] = (torch.rand(n, device=DEV, generator=g) > 0.5).float() * 2
  sd[:, 5] = (torch.rand(n, device=DEV, generator=g) > 0.5).float()
  ca, la, cc, lc = (t.clone() for t in st)
  # torch rule (contact_sensor.py air-time tracking)
  el = (time - last_time)[:, None]
  is_c = sd[:, [1, 5]] > 0
  first_c = (ca > 0) & is_c
  first_d = (cc > 0) & ~is_c
  la_ref = torch.where(first_c, ca + el, la)
  ca_ref = torch.where(~is_c, ca + el, torch.zeros_like(ca))
  lc_ref = torch.where(first_d, cc + el, lc)
  cc_ref = torch.where(is_c, cc + el, torch.zeros_like(cc))
  lt = last_time.clone()
  assert envops.air_time_update(sd, cols, time, lt, ca, la, cc, lc)
  torch.cuda.synchronize()
  for a, b in ((ca, ca_ref), (la, la_ref), (cc, cc_ref), (lc, lc_ref), (lt, time)):
    torch.testing.assert_close(a, b)


def test_obs_term_kernel_matches_torch():
  g = torch.Generator(device=DEV).manual_seed(3)
  n = 777
  x = torch.randn(n, 10, device=DEV, generator=g)[:, 2:7]  # strided input
  out = torch.full((n, 12), -7.0, device=DEV)
  u = torch.rand(n, 12, device=DEV, generator=g)
  assert envops.obs_term(x, out[:, 3:8], u[:, 3:8], -0.5, 0.25, (-1.0, 1.5), 0.25)
  ref = torch.clamp(x + (u[:, 3:8] * 0.75 - 0.5), -1.0, 1.5) * 0.25
  torch.testing.assert_close(out[:, 3:8], ref)
  assert (out[:, :3] == -7.0).all() and (out[:, 8:] == -7.0).all()
  v = torch.randn(n, device=DEV, generator=g)  # 1-D term
  assert envops.obs_term(v, out[:, 0:1], None, 0.0, 0.0, None, 2.0)
  torch.testing.assert_close(out[:, 0], v * 2.0)


def test_fused_observation_group_matches_generic():
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 64
  env = ManagerBasedRlEnv(cfg, device=DEV)
  env.reset()
  env.step(torch.zeros(64, 29, device=DEV))
  om = env.observation_manager
  assert om._fused["critic"] is not None and om._fused["policy"] is not None
  fused = om.compute_group("critic")
  plan = om._fused.pop("critic")
  generic = om.compute_group("critic")
  om._fused["critic"] = plan
  torch.testing.assert_close(fused, generic, rtol=1e-6, atol=1e-6)


def test_fused_reward_terms_match_torch(monkeypatch):
  """Every reward term of the G1 task, fused kernels vs their torch formulas."""
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 128
  env = ManagerBasedRlEnv(cfg, device=DEV)
  env.reset()
  g = torch.Generator(device=DEV).manual_seed(5)
  for _ in range(8):
    env.step(2 * torch.rand(128, 29, device=DEV, generator=g) - 1)
  rm = env.reward_manager

  def evaluate():
    out = {}
    for name, tcfg in zip(rm._term_names, rm._term_cfgs):
      if name == "foot_swing_height":
        continue  # stateful (peak heights): evaluated once per step only
      out[name] = tcfg.func(env, **tcfg.params).clone()
    return out

  fused = evaluate()
  for fn in ("rew_track", "rew_flat_orientation", "rew_sqsum", "rew_diffsq", "rew_pos_limits", "rew_posture", "rew_feet"):
    monkeypatch.setattr(envops, fn, lambda *a, **k: None)
  ref = evaluate()
  for name in fused:
    torch.testing.assert_close(fused[name].float(), ref[name].float(), rtol=2e-5, atol=2e-5, msg=name)


def test_fused_velocity_command_matches_torch():
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 256
  env = ManagerBasedRlEnv(cfg, device=DEV)
  env.reset()
  for _ in range(5):
    env.step(torch.zeros(256, 29, device=DEV))
  term = env.command_manager.get_term("twist")
  term.time_left[::3] = 0.001  # force resampling in a third of the envs
  fields = ("vel_command_b", "heading_target", "heading_error", "is_heading_env", "is_standing_env", "time_left",
            "command_counter")
  snap = {f: getattr(term, f).clone() for f in fields}
  msnap = {k: v.clone() for k, v in term.metrics.items()}
  u = torch.rand(256, 8, device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
  assert term._compute_fused(env.step_dt, u)
  fused = {f: getattr(term, f).clone() for f in fields}
  fm = {k: v.clone() for k, v in term.metrics.items()}
  for f in fields:
    getattr(term, f).copy_(snap[f])
  for k in term.metrics:
    term.metrics[k].copy_(msnap[k])
  term._compute_torch(env.step_dt, u)
  for f in fields:
    torch.testing.assert_close(fused[f], getattr(term, f), rtol=1e-5, atol=1e-5, msg=f)
  for k in fm:
    torch.testing.assert_close(fm[k], term.metrics[k], rtol=1e-5, atol=1e-5, msg=k)


def test_rotation_kernels_match_torch():
  """quat_from_euler_xyz, quat_error_magnitude, subtract_frame_transforms (+ matrix
  columns) and the MotionCommand relative targets vs the torch formulas."""
  g = torch.Generator(device=DEV).manual_seed(3)
  n, k = 1024, 14
  draws = torch.rand(n, 6, device=DEV, generator=g) * 2 - 1  # strided rpy view
  rpy = draws[:, 3:6]
  torch.testing.assert_close(envops.quat_from_euler_xyz(rpy), M.quat_from_euler_xyz(rpy[:, 0], rpy[:, 1], rpy[:, 2]),
                             rtol=1e-6, atol=1e-6)
  q1, q2 = _q(n * k, g).view(n, k, 4), _q(n * k, g).view(n, k, 4)
  q2[:5] = q1[:5]  # zero error: the small-angle branch
  torch.testing.assert_close(envops.quat_error_magnitude(q1, q2), M.quat_error_magnitude(q1, q2), rtol=1e-5, atol=1e-5)
  frame = torch.randn(n, 32, 7, device=DEV, generator=g)  # strided (env, body) layout like body_link_pose
  frame[..., 3:7] = _q(n * 32, g).view(n, 32, 4)
  t01, q01 = frame[:, 5, 0:3], frame[:, 5, 3:7]
  t02, q02 = frame[:, 8:8 + k, 0:3], frame[:, 8:8 + k, 3:7]
  t_ref, q_ref = M.subtract_frame_transforms(t01[:, None].expand(-1, k, -1), q01[:, None].expand(-1, k, -1), t02, q02)
  t12, q12 = envops.frame_subtract(t01, q01, t02, q02)
  torch.testing.assert_close(t12, t_ref, rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(q12, q_ref, rtol=1e-5, atol=1e-5)
  _, m12 = envops.frame_subtract(t01, q01, t02, q02, want_t=False, qcols=2)
  torch.testing.assert_close(m12, M.matrix_from_quat(q_ref)[..., :2].reshape(n, k, 6), rtol=1e-5, atol=1e-5)
  t1, _ = envops.frame_subtract(t01, q01, frame[:, 9, 0:3], frame[:, 9, 3:7], want_q=False)  # one target per env
  torch.testing.assert_close(t1, t_ref[:, 1], rtol=1e-5, atol=1e-5)
  # motion-relative targets (commands.py:383-405)
  ap, aq, rp, rq = frame[:, 1, 0:3], frame[:, 1, 3:7], frame[:, 2, 0:3], frame[:, 2, 3:7]
  bp, bq = frame[:, 10:10 + k, 0:3], frame[:, 10:10 + k, 3:7]
  op, oq = torch.empty(n, k, 3, device=DEV), torch.empty(n, k, 4, device=DEV)
  assert envops.motion_relative(ap, aq, rp, rq, bp, bq, op, oq)
  dpos = rp[:, None].repeat(1, k, 1).clone()
  dpos[..., 2] = ap[:, None, 2]
  dori = M.yaw_quat(M.quat_mul(rq[:, None].repeat(1, k, 1), M.quat_inv(aq[:, None].repeat(1, k, 1))))
  torch.testing.assert_close(oq, M.quat_mul(dori, bq.contiguous()), rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(op, dpos + M.quat_apply(dori, bp - ap[:, None]), rtol=1e-5, atol=1e-5)


def test_reward_combine_matches_torch():
  g = torch.Generator(device=DEV).manual_seed(4)
  n, T = 777, 9
  base = torch.randn(n, 2 * T, device=DEV, generator=g)
  vals = [base[:, 2 * i] for i in range(T)]  # strided term vectors
  vals[3] = None  # weight-0 term
  w = torch.randn(T, device=DEV, generator=g)
  w[3] = 0.0
  dt = 0.02
  sums0 = torch.randn(n, T, device=DEV, generator=g)
  rew, step, sums = torch.empty(n, device=DEV), torch.empty(n, T, device=DEV), sums0.clone()
  assert envops.reward_combine(vals, w, dt, rew, step, sums)
  raw = torch.stack([v if v is not None else torch.zeros(n, device=DEV) for v in vals], 1)
  weighted = raw * (w * dt)
  torch.testing.assert_close(step, raw * w, rtol=1e-6, atol=1e-6)
  torch.testing.assert_close(sums, sums0 + weighted, rtol=1e-6, atol=1e-6)
  torch.testing.assert_close(rew, weighted.sum(1), rtol=1e-5, atol=1e-6)


def test_obs_group_kernel_matches_per_term():
  g = torch.Generator(device=DEV).manual_seed(5)
  n = 513
  a = torch.randn(n, 10, device=DEV, generator=g)
  xs = [a[:, 0:3], a[:, 5], torch.randn(n, 7, device=DEV, generator=g)]
  plan = [(None, 0, 3, (-0.5, 0.5), None, 0.25), (None, 3, 1, None, (-0.1, 0.1), 1.0), (None, 4, 7, (-1.0, 2.0), (-1.0, 1.0), 2.0)]
  u = torch.rand(n, 11, device=DEV, generator=g)
  out = torch.full((n, 11), float("nan"), device=DEV)
  assert envops.obs_group(xs, plan, u, out)
  ref = torch.cat([
    (xs[0] + (u[:, 0:3] * 1.0 - 0.5)) * 0.25,
    xs[1].view(-1, 1).clip(-0.1, 0.1),
    (xs[2] + (u[:, 4:11] * 3.0 - 1.0)).clip(-1.0, 1.0) * 2.0,
  ], 1)
  torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)


def test_gz_above_kernel_matches_torch():
  """bad_orientation's fused test (-cos(limit) < g_z <= 1) equals the torch
  formula on the same float32 values, including g_z just above 1 and at the
  threshold."""
  import math

  from mjlab_amd import envops

  g = torch.rand(4096, 3, device="cuda:0") * 2.2 - 1.1
  thr = -math.cos(1.2)
  g[:4, 2] = torch.tensor([1.0, 1.0000001, float(torch.tensor(thr, dtype=torch.float32)), -1.0])
  got = envops.gz_above(g[:, 2], thr)
  ref = (g[:, 2] > thr) & (g[:, 2] <= 1.0)
  assert torch.equal(got, ref)


def test_sum_ratios_with_mean_sqrt_term():
  """The reward pass's ratio-log launch: sum(num)/max(sum(den),1) terms and a
  den-less term (mean(sqrt(num)): Metrics/angular_momentum_mean) against
  torch, float32 summation-order tolerance."""
  from mjlab_amd import envops

  n = 4096
  a, b, c = torch.rand(n, device="cuda:0"), (torch.rand(n, device="cuda:0") > 0.5).float(), torch.rand(n, device="cuda:0")
  out = torch.zeros(2, device="cuda:0")
  assert envops.sum_ratios([(a, b), (c, None)], out)
  ref = torch.stack([a.sum() / b.sum().clamp(min=1), torch.sqrt(c).mean()])
  torch.testing.assert_close(out, ref, rtol=1e-5, atol=0)
