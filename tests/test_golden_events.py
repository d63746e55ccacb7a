"""randomize_field and the numpy stream against reference-generated vectors.

``tests/golden/events_g1.npz`` (tools/make_golden_events.py): the reference's
``randomize_field`` (``envs/mdp/events.py:256-309``) ran on per-world fields
with its draws recorded; here mjlab_amd's ``randomize_field`` runs on the same
inputs with the same draws injected (its torch.rand calls are fed the
recorded values in call order), on CPU and on the GPU. Exact: the formula is
one float32 multiply-add per element on both sides.
"""

from __future__ import annotations

import json
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from mjlab_amd.envs.mdp import events
from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from tests import rng_np

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def fx():
  return dict(np.load(GOLDEN / "events_g1.npz"))


@pytest.mark.parametrize("dev", [pytest.param("cpu"), pytest.param("cuda:0", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("i", range(4))
def test_randomize_field_matches_reference(fx, i, dev, monkeypatch):
  meta = json.loads(str(fx[f"rf{i}_meta"]))
  ix = {k: torch.tensor(v, dtype=torch.int, device=dev) for k, v in json.loads(str(fx["rf_indexing"])).items()}
  field = torch.as_tensor(fx[f"rf{i}_in"], device=dev).clone()
  env = SimpleNamespace(num_envs=field.shape[0], device=dev, scene={"robot": SimpleNamespace(indexing=SimpleNamespace(**ix))},
                        sim=SimpleNamespace(model=SimpleNamespace(**{meta["field"]: field})))
  draws = torch.as_tensor(fx[f"rf{i}_draws"], device=dev)
  used = [0]

  def rand(*size, device=None, **kw):
    shape = tuple(size[0]) if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)) else tuple(size)
    k = int(np.prod(shape))
    u = draws[used[0] : used[0] + k].reshape(shape)
    used[0] += k
    return u.to(device or dev)

  monkeypatch.setattr(torch, "rand", rand)
  ranges = meta["ranges"]
  ranges = tuple(ranges) if isinstance(ranges, list) else {int(k): tuple(v) for k, v in ranges.items()}
  sc = SceneEntityCfg("robot", **{meta["kind"]: meta["ids"]})
  events.randomize_field(env, torch.as_tensor(fx["rf_mask"], device=dev), meta["field"], ranges, "uniform",
                         meta["operation"], sc, meta["axes"])
  assert used[0] == draws.numel()
  np.testing.assert_array_equal(field.cpu().numpy(), fx[f"rf{i}_out"])


def test_numpy_stream_known_values():
  """mjh_rng.h restated: a few elements computed by hand from the splitmix64
  finalizer (the GPU test checks 4096 elements against the device)."""
  seed, key, step = 1, 2, 3
  b = rng_np.base(seed, key, step)
  z = (b + 1 * rng_np.GOLDEN) & rng_np.M64
  z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & rng_np.M64
  z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & rng_np.M64
  z ^= z >> 31
  assert rng_np.u01(seed, key, step, [0])[0] == np.float32((z >> 40) / 16777216.0)
  u = rng_np.u01(seed, key, step, np.arange(100000))
  assert 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
