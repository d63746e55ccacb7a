"""Compiled model sizes and parameters vs the reference's MJCF + mjlab edits."""

import math

import numpy as np
import pytest

from mjlab_amd.asset_zoo import g1 as g1c
from tests.scenes import g1_scene_model, go1_scene_model


def test_g1_sizes():
  m = g1_scene_model(4)
  assert (m.nbody, m.njnt, m.nq, m.nv, m.nu, m.na) == (32, 30, 36, 35, 29, 0)
  assert m.ngeom == 69
  # 4 XML sensors + feet (2 x found,force) + self-collision found: 12 + 8 + 1
  assert m.nsensordata == 21
  assert (m.nconmax, m.njmax) == (50, 300)


def test_go1_sizes():
  m = go1_scene_model(4)
  assert (m.nbody, m.nq, m.nv, m.nu) == (15, 19, 18, 12)
  assert m.ngeom == 44
  assert m.nsensordata == 54


def test_g1_actuators_follow_constants():
  """kp = gainprm[0], kd = -biasprm[2], forcerange = +-effort (spec_config.py:402-414)."""
  m = g1_scene_model(1)
  names = [n.split("/")[-1] for n in m.names["actuator"]]
  for a in g1c.G1_ARTICULATION.actuators:
    import re

    for i, n in enumerate(names):
      if any(re.fullmatch(e, n) for e in a.joint_names_expr):
        assert m.actuator_gainprm[i, 0] == pytest.approx(a.stiffness, rel=1e-6)
        assert -m.actuator_biasprm[i, 2] == pytest.approx(a.damping, rel=1e-6)
        assert m.actuator_forcerange[i, 1] == pytest.approx(a.effort_limit, rel=1e-6)
  assert all(math.isfinite(v) for v in g1c.G1_ACTION_SCALE.values())


def test_g1_keyframe_and_inertia():
  m = g1_scene_model(1)
  assert m.key_qpos.shape == (m.nq,)
  q = m.key_qpos
  assert np.isclose(np.linalg.norm(q[3:7]), 1.0)
  assert (m.body_mass[2:] > 0).all()
  assert 30.0 < m.body_mass.sum() < 40.0  # G1 29-dof total mass ~33 kg
  assert m.meaninertia > 0
