"""Observation delay and history (reference ``utils/buffers``, ``observation_manager.py:176-188``).

Three layers of evidence:
* golden vectors from the reference's own CircularBuffer / DelayBuffer / ObservationManager
  (tools/make_golden_obs.py -> tests/golden/obs_buffers.npz): the same appends, resets and
  seeded draws replayed here must give identical frames, lags and observations;
* the reference's unit tests (``tests/test_circular_buffer.py``, ``test_delay_buffer.py``,
  ``test_observation_delay.py``, ``test_observation_history.py``) restated on this package;
* capture safety: the buffers' state lives in device tensors updated in place, so a
  CUDA/HIP graph replay advances them (tests/test_gpu_env.py covers the env on the GPU;
  here a CPU check that no attribute is rebound by a step).
"""

from pathlib import Path
from types import SimpleNamespace
from unittest.mock import Mock

import numpy as np
import pytest
import torch

from mjlab_amd.envs import mdp as gmdp
from mjlab_amd.managers.manager_term_config import ObservationGroupCfg, ObservationTermCfg
from mjlab_amd.managers.observation_manager import ObservationManager
from mjlab_amd.utils.buffers import CircularBuffer, DelayBuffer

G = np.load(Path(__file__).parent / "golden" / "obs_buffers.npz")
RESETS = {4: [1, 3], 9: [0], 11: None}  # tools/make_golden_obs.py


def _ids(t):
  return None if RESETS[t] is None else torch.tensor(RESETS[t])


# ---- golden replays ----------------------------------------------------------------------
def test_circular_buffer_matches_reference_golden():
  x, lags = torch.from_numpy(G["cb_x"]), torch.from_numpy(G["cb_lags"])
  T, B, _ = x.shape
  cb = CircularBuffer(max_len=4, batch_size=B, device="cpu")
  for t in range(T):
    if t in RESETS:
      cb.reset(batch_ids=RESETS[t])
    cb.append(x[t])
    assert torch.equal(cb.buffer, torch.from_numpy(G["cb_hist"][t])), t
    assert torch.equal(cb[lags[t]], torch.from_numpy(G["cb_lagged"][t])), t
    assert torch.equal(cb.current_length, torch.from_numpy(G["cb_len"][t])), t


@pytest.mark.parametrize("k", range(5))
def test_delay_buffer_matches_reference_golden(k):
  lo, hi, per_env, hold, period, phase = G["db_cases"][k]
  x = torch.from_numpy(G["cb_x"])
  T, B, _ = x.shape
  gen = torch.Generator().manual_seed(100 + k)
  db = DelayBuffer(int(lo), int(hi), batch_size=B, device="cpu", per_env=bool(per_env), hold_prob=float(hold),
                   update_period=int(period), per_env_phase=bool(phase), generator=gen)
  for t in range(T):
    if t in RESETS:
      db.reset(batch_ids=_ids(t))
    db.append(x[t])
    y = db.compute()
    assert torch.equal(db.current_lags, torch.from_numpy(G[f"db{k}_lags"][t])), (k, t)
    assert torch.equal(y, torch.from_numpy(G[f"db{k}_y"][t])), (k, t)


def test_delay_buffer_bool_mask_reset_equals_index_reset():
  """The env resets with boolean masks; the reference takes index lists: same state."""
  x = torch.from_numpy(G["cb_x"])
  T, B, _ = x.shape
  bufs = [DelayBuffer(0, 3, batch_size=B, update_period=2, hold_prob=0.2, generator=torch.Generator().manual_seed(5))
          for _ in range(2)]
  for t in range(T):
    if t in RESETS:
      m = torch.from_numpy(G["resets"][t])
      bufs[0].reset(batch_ids=_ids(t))
      bufs[1].reset(batch_ids=m)
    ys = []
    for b in bufs:
      b.append(x[t])
      ys.append(b.compute())
    assert torch.equal(ys[0], ys[1]) and torch.equal(bufs[0].current_lags, bufs[1].current_lags)


def test_observation_manager_delay_history_matches_reference_golden():
  seq = torch.from_numpy(G["om_seq"])
  T, B = G["om_policy"].shape[0], seq.shape[1]
  torch.manual_seed(21)
  env = Mock()
  env.num_envs, env.device, env.step_dt = B, "cpu", 0.02
  state = {"t": 0}
  term_a = lambda env: seq[state["t"], :, :3].clone()  # noqa: E731
  term_b = lambda env: seq[state["t"], :, 3:].clone() * 10.0  # noqa: E731
  cfg = {
    "policy": ObservationGroupCfg(terms={
      "a": ObservationTermCfg(func=term_a, params={}, clip=(-1.0, 1.0), scale=2.0, delay_min_lag=0, delay_max_lag=2,
                              history_length=3, flatten_history_dim=True),
      "b": ObservationTermCfg(func=term_b, params={}, delay_min_lag=1, delay_max_lag=3, delay_update_period=2),
    }),
    "critic": ObservationGroupCfg(terms={"a": ObservationTermCfg(func=term_a, params={}, history_length=2,
                                                                 flatten_history_dim=False)},
                                  concatenate_terms=False),
  }
  om = ObservationManager(cfg, env)
  assert om.group_obs_dim["policy"] == tuple(G["om_dims"])
  for t in range(T):
    state["t"] = t + 1
    if t in RESETS:
      om.reset(env_ids=_ids(t))
    o = om.compute(update_history=(t % 5 != 2))
    assert torch.equal(o["policy"], torch.from_numpy(G["om_policy"][t])), t
    assert torch.equal(o["critic"]["a"], torch.from_numpy(G["om_critic"][t])), t


def test_generic_rewards_match_reference_golden():
  tau, qd, pg = (torch.from_numpy(G[k]) for k in ("rw_tau", "rw_qd", "rw_pg"))
  asset = SimpleNamespace(data=SimpleNamespace(actuator_force=tau, joint_vel=qd, projected_gravity_b=pg))
  env = SimpleNamespace(scene={"robot": asset})
  torch.testing.assert_close(gmdp.electrical_power_cost(env), torch.from_numpy(G["rw_electrical_power_cost"]), rtol=0,
                             atol=0)
  torch.testing.assert_close(gmdp.flat_orientation_l2(env), torch.from_numpy(G["rw_flat_orientation_l2"]), rtol=0, atol=0)


# ---- the reference's unit tests, restated ------------------------------------------------
def test_circular_buffer_order_overwrite_and_backfill():
  cb = CircularBuffer(max_len=3, batch_size=2, device="cpu")
  cb.append(torch.tensor([[1.0], [2.0]]))
  assert torch.equal(cb.buffer[:, :, 0], torch.tensor([[1.0, 1.0, 1.0], [2.0, 2.0, 2.0]]))  # first push back-fills
  assert torch.equal(cb.current_length, torch.tensor([1, 1]))
  cb.append(torch.tensor([[3.0], [4.0]]))
  cb.append(torch.tensor([[5.0], [6.0]]))
  cb.append(torch.tensor([[7.0], [8.0]]))  # overwrites the oldest
  assert torch.equal(cb.buffer[:, :, 0], torch.tensor([[3.0, 5.0, 7.0], [4.0, 6.0, 8.0]]))
  cb.reset(batch_ids=[1])
  assert torch.equal(cb.current_length, torch.tensor([3, 0]))
  assert torch.count_nonzero(cb.buffer[1]) == 0
  cb.append(torch.tensor([[9.0], [99.0]]))
  assert torch.equal(cb.buffer[:, :, 0], torch.tensor([[5.0, 7.0, 9.0], [99.0, 99.0, 99.0]]))
  # LIFO lags, clamped to the frames a row holds
  assert torch.equal(cb[torch.tensor([0, 0])][:, 0], torch.tensor([9.0, 99.0]))
  assert torch.equal(cb[torch.tensor([2, 5])][:, 0], torch.tensor([5.0, 99.0]))
  assert torch.equal(cb[1][:, 0], torch.tensor([7.0, 99.0]))
  cb.reset()
  assert torch.equal(cb.current_length, torch.tensor([0, 0])) and torch.count_nonzero(cb.buffer) == 0


def test_circular_buffer_errors():
  with pytest.raises(ValueError):
    CircularBuffer(max_len=0, batch_size=1, device="cpu")
  cb = CircularBuffer(max_len=2, batch_size=2, device="cpu")
  with pytest.raises(ValueError):
    cb.append(torch.zeros(1, 1))
  with pytest.raises(RuntimeError):
    _ = cb.buffer
  with pytest.raises(RuntimeError):
    _ = cb[torch.tensor([0, 0])]
  cb.append(torch.zeros(2, 1))
  with pytest.raises(ValueError):
    _ = cb[torch.tensor([0])]
  assert cb.buffer.dtype == torch.float32


def test_delay_buffer_constant_and_zero_lag():
  db = DelayBuffer(min_lag=2, max_lag=2, batch_size=1)
  got = []
  for v in (1.0, 2.0, 3.0, 4.0, 5.0):
    db.append(torch.tensor([[v]]))
    got.append(db.compute().item())
  assert got == [1.0, 1.0, 1.0, 2.0, 3.0]  # lag clamped to the frames held, then T - 2
  z = DelayBuffer(min_lag=0, max_lag=0, batch_size=2)
  z.append(torch.tensor([[1.0], [2.0]]))
  assert torch.equal(z.compute(), torch.tensor([[1.0], [2.0]]))


def test_delay_buffer_value_matches_lag_and_modes():
  buf = DelayBuffer(0, 2, batch_size=3, generator=torch.Generator().manual_seed(1234))
  for t in range(6):
    buf.append(torch.full((3, 1), float(t)))
    y = buf.compute()
    for e in range(3):
      assert y[e].item() == float(t - min(int(buf.current_lags[e]), t))
  shared = DelayBuffer(0, 3, batch_size=4, per_env=False)
  for t in range(10):
    shared.append(torch.full((4, 1), float(t)))
    shared.compute()
  assert torch.all(shared.current_lags == shared.current_lags[0])
  held = DelayBuffer(0, 3, batch_size=1, update_period=1, hold_prob=1.0, generator=torch.Generator().manual_seed(7))
  for t in range(20):
    held.append(torch.tensor([[float(t)]]))
    held.compute()
    assert held.current_lags.item() == 0  # never resampled: stays at its initial lag
  per = DelayBuffer(0, 10, batch_size=1, update_period=3, per_env_phase=False, generator=torch.Generator().manual_seed(123))
  lags = []
  for t in range(12):
    per.append(torch.tensor([[float(t)]]))
    per.compute()
    lags.append(per.current_lags.item())
  assert all(lags[i] == lags[i - i % 3] for i in range(12))  # resampled at steps 0, 3, 6, 9 only


def test_delay_buffer_reset_and_validation():
  buf = DelayBuffer(1, 2, batch_size=3, generator=torch.Generator().manual_seed(9))
  for t in range(3):
    buf.append(torch.arange(1, 4).float().unsqueeze(1) * 10 + t)
    buf.compute()
  before = buf.current_lags.clone()
  buf.reset(batch_ids=torch.tensor([1]))
  assert buf.current_lags[1] == 0 and buf._step_count[1] == 0 and buf.current_lags[0] == before[0]
  assert torch.count_nonzero(buf.compute()[1]) == 0  # zeros until the row's next append
  buf.append(torch.tensor([[111.0], [999.0], [333.0]]))
  assert buf.compute()[1].item() == 999.0
  with pytest.raises(RuntimeError, match="Buffer not initialized"):
    DelayBuffer(0, 3).compute()
  for kw, msg in (({"min_lag": -1}, "min_lag must be >= 0"), ({"min_lag": 5, "max_lag": 3}, "max_lag.*must be >= min_lag"),
                  ({"hold_prob": 1.5}, "hold_prob must be in"), ({"update_period": -1}, "update_period must be >= 0")):
    with pytest.raises(ValueError, match=msg):
      DelayBuffer(**kw)


@pytest.fixture
def counter_env():
  env = Mock()
  env.num_envs, env.device, env.step_dt = 4, "cpu", 0.02
  c = {"v": 0}

  def f(env):
    c["v"] += 1
    return torch.full((env.num_envs, 3), float(c["v"]))

  return env, f


def _om(env, **kw):
  return ObservationManager({"policy": ObservationGroupCfg(terms={"obs1": ObservationTermCfg(params={}, **kw)})}, env)


def test_observation_delay_pipeline(counter_env):
  env, f = counter_env
  m = _om(env, func=f, delay_min_lag=1, delay_max_lag=1, scale=2.0)  # the term is evaluated once here (value 1)
  assert m.group_obs_dim["policy"] == (3,)
  assert [m.compute()["policy"][0, 0].item() for _ in range(3)] == [4.0, 4.0, 6.0]  # scale before delay
  c = {"v": 0}

  def f2(env):
    c["v"] += 1
    return torch.full((env.num_envs, 3), float(c["v"]))

  m2 = _om(env, func=f2, delay_min_lag=1, delay_max_lag=1, history_length=2, flatten_history_dim=False)
  assert m2.group_obs_dim["policy"] == (2, 3)
  h = [m2.compute(update_history=u)["policy"][0, :, 0].tolist() for u in (False, True, True)]
  assert h == [[2.0, 2.0], [2.0, 2.0], [2.0, 3.0]]  # delay before history


def test_observation_history_pipeline(counter_env):
  env, f = counter_env
  m = _om(env, func=f, history_length=3, flatten_history_dim=False)
  assert m.group_obs_dim["policy"] == (3, 3)
  first = m.compute(update_history=True)["policy"]
  assert torch.equal(first[0, :, 0], torch.tensor([2.0, 2.0, 2.0]))  # one append, back-filled
  hb = m._group_obs_term_history_buffer["policy"]["obs1"]
  assert hb._pointer == 0 and torch.all(hb._num_pushes == 1)
  m.compute(update_history=True)
  before = m.compute(update_history=True)["policy"].clone()
  assert torch.equal(before[0, :, 0], torch.tensor([2.0, 3.0, 4.0]))
  m.reset(env_ids=torch.tensor([0, 2]))
  after = m.compute(update_history=False)["policy"]
  assert torch.count_nonzero(after[0]) == 0 and torch.count_nonzero(after[2]) == 0
  assert torch.equal(after[1], before[1])
  refill = m.compute(update_history=True)["policy"]
  # value 6 (5 went to the update_history=False call): back-filled rows, continuing rows
  assert torch.equal(refill[0, :, 0], torch.tensor([6.0, 6.0, 6.0])) and torch.equal(refill[1, :, 0],
                                                                                    torch.tensor([3.0, 4.0, 6.0]))


def test_group_history_override_and_mixed_concat(counter_env):
  env, f = counter_env
  m = ObservationManager({"policy": ObservationGroupCfg(history_length=5, flatten_history_dim=False,
                                                        terms={"obs1": ObservationTermCfg(func=f, params={},
                                                                                          history_length=2)})}, env)
  assert m.group_obs_dim["policy"] == (5, 3) and m.compute()["policy"].shape == (4, 5, 3)
  env2 = Mock()
  env2.num_envs, env2.device = 4, "cpu"
  m2 = ObservationManager({"policy": ObservationGroupCfg(terms={
    "h": ObservationTermCfg(func=lambda e: torch.ones(4, 3), params={}, history_length=2),
    "n": ObservationTermCfg(func=lambda e: torch.zeros(4, 2), params={})})}, env2)
  assert m2.group_obs_dim["policy"] == (8,) and m2.compute()["policy"].shape == (4, 8)


def test_buffer_state_is_updated_in_place():
  """Capture safety: a step advances the same tensors a captured graph would hold."""
  db = DelayBuffer(0, 3, batch_size=4, update_period=2, hold_prob=0.5)
  db.append(torch.zeros(4, 2))
  ids = {k: id(getattr(db, k)) for k in ("_current_lags", "_step_count", "_phase_offsets")}
  cb = db._buffer
  cid = {k: id(getattr(cb, k)) for k in ("_pointer", "_num_pushes", "_buffer")}
  for t in range(5):
    db.append(torch.full((4, 2), float(t)))
    db.compute()
    db.reset(batch_ids=torch.tensor([True, False, False, True]))
  assert ids == {k: id(getattr(db, k)) for k in ids}
  assert cid == {k: id(getattr(cb, k)) for k in cid}
