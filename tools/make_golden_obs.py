"""Golden vectors for the observation delay / history buffers and two generic reward terms
(run HERE only; the reference imported with inert stand-ins, as tools/make_golden.py).

Runs the reference's own CircularBuffer, DelayBuffer and ObservationManager
(``src/mjlab/utils/buffers``, ``src/mjlab/managers/observation_manager.py``) on seeded
CPU inputs, resets included, and ``electrical_power_cost`` / ``flat_orientation_l2``
(``src/mjlab/envs/mdp/rewards.py:107-126``) on a synthetic entity snapshot. Inputs and
outputs go to tests/golden/obs_buffers.npz (data only).
"""

from __future__ import annotations

import sys
from pathlib import Path
from types import SimpleNamespace
from unittest.mock import Mock

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from make_golden import OUT, setup  # noqa: E402

# (min_lag, max_lag, per_env, hold_prob, update_period, per_env_phase)
DELAY_CASES = [(0, 3, True, 0.0, 0, True), (1, 4, True, 0.3, 0, True), (0, 3, False, 0.0, 3, True),
               (2, 5, True, 0.2, 4, True), (0, 2, True, 0.0, 2, False)]
RESETS = {4: [1, 3], 9: [0], 11: None}  # step -> rows reset before that step's append (None: all)


def _reset_mask(step: int, b: int) -> np.ndarray:
  m = np.zeros(b, dtype=bool)
  if step in RESETS:
    ids = RESETS[step]
    m[:] = ids is None
    if ids is not None:
      m[ids] = True
  return m


def main() -> None:
  setup()
  from mjlab.envs.mdp import rewards as R
  from mjlab.managers.manager_term_config import ObservationGroupCfg, ObservationTermCfg
  from mjlab.managers.observation_manager import ObservationManager
  from mjlab.utils.buffers import CircularBuffer, DelayBuffer

  out: dict[str, np.ndarray] = {}
  g = torch.Generator().manual_seed(11)
  T, B, D = 14, 5, 3
  # ---- CircularBuffer ----
  x = torch.randn(T, B, D, generator=g)
  lags = torch.randint(0, 6, (T, B), generator=g)
  cb = CircularBuffer(max_len=4, batch_size=B, device="cpu")
  hist, lagged, clen = [], [], []
  for t in range(T):
    if t in RESETS:
      cb.reset(batch_ids=RESETS[t])
    cb.append(x[t])
    hist.append(cb.buffer.clone())
    lagged.append(cb[lags[t]].clone())
    clen.append(cb.current_length.clone())
  out.update(cb_x=x.numpy(), cb_lags=lags.numpy(), cb_hist=torch.stack(hist).numpy(), cb_lagged=torch.stack(lagged).numpy(),
             cb_len=torch.stack(clen).numpy())
  out["resets"] = np.stack([_reset_mask(t, B) for t in range(T)])
  # ---- DelayBuffer (seeded generator: the draws are part of the semantics) ----
  for k, (lo, hi, per_env, hold, period, phase) in enumerate(DELAY_CASES):
    gen = torch.Generator().manual_seed(100 + k)
    db = DelayBuffer(lo, hi, batch_size=B, device="cpu", per_env=per_env, hold_prob=hold, update_period=period,
                     per_env_phase=phase, generator=gen)
    ys, ls = [], []
    for t in range(T):
      if t in RESETS:
        db.reset(batch_ids=None if RESETS[t] is None else torch.tensor(RESETS[t]))
      db.append(x[t])
      ys.append(db.compute().clone())
      ls.append(db.current_lags.clone())
    out[f"db{k}_y"] = torch.stack(ys).numpy()
    out[f"db{k}_lags"] = torch.stack(ls).numpy()
  out["db_cases"] = np.array(DELAY_CASES, dtype=np.float64)
  # ---- ObservationManager: noise-free pipeline clip -> scale -> delay -> history ----
  torch.manual_seed(21)
  env = Mock()
  env.num_envs, env.device, env.step_dt = B, "cpu", 0.02
  state = {"t": 0}
  seq = torch.randn(T + 2, B, 4, generator=g)

  def term_a(env):
    return seq[state["t"], :, :3].clone()

  def term_b(env):
    return seq[state["t"], :, 3:].clone() * 10.0

  cfg = {
    "policy": ObservationGroupCfg(terms={
      "a": ObservationTermCfg(func=term_a, params={}, clip=(-1.0, 1.0), scale=2.0, delay_min_lag=0, delay_max_lag=2,
                              history_length=3, flatten_history_dim=True),
      "b": ObservationTermCfg(func=term_b, params={}, delay_min_lag=1, delay_max_lag=3, delay_update_period=2),
    }),
    "critic": ObservationGroupCfg(terms={
      "a": ObservationTermCfg(func=term_a, params={}, history_length=2, flatten_history_dim=False),
    }, concatenate_terms=False),
  }
  om = ObservationManager(cfg, env)
  pol, cri = [], []
  for t in range(T):
    state["t"] = t + 1
    if t in RESETS:
      om.reset(env_ids=None if RESETS[t] is None else torch.tensor(RESETS[t]))
    o = om.compute(update_history=(t % 5 != 2))
    pol.append(o["policy"].clone())
    cri.append(o["critic"]["a"].clone())
  out.update(om_seq=seq.numpy(), om_policy=torch.stack(pol).numpy(), om_critic=torch.stack(cri).numpy(),
             om_dims=np.array(om.group_obs_dim["policy"]))
  # ---- generic rewards ----
  n = 64
  tau, qd = torch.randn(n, 12, generator=g) * 20, torch.randn(n, 12, generator=g) * 3
  pg = torch.randn(n, 3, generator=g) * 0.3
  asset = SimpleNamespace(data=SimpleNamespace(actuator_force=tau, joint_vel=qd, projected_gravity_b=pg))
  renv = SimpleNamespace(scene={"robot": asset})
  out.update(rw_tau=tau.numpy(), rw_qd=qd.numpy(), rw_pg=pg.numpy(),
             rw_electrical_power_cost=R.electrical_power_cost(renv).numpy(),
             rw_flat_orientation_l2=R.flat_orientation_l2(renv).numpy())
  np.savez(OUT / "obs_buffers.npz", **out)
  print("wrote", OUT / "obs_buffers.npz", len(out), "arrays")


if __name__ == "__main__":
  main()
