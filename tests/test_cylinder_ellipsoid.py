"""Plane-cylinder, plane-ellipsoid and sphere-cylinder contacts of the oracle
(oracle.c raw_plane_cylinder / raw_plane_ellipsoid / raw_sphere_cylinder,
restating MuJoCo's mjc_PlaneCylinder and MuJoCo Warp's plane_ellipsoid /
sphere_cylinder) against closed-form geometry. MuJoCo is absent, so these
known answers pin them (parity unpinned by reference vectors); the HIP step is
checked against the oracle in tests/test_gpu_parity.py."""

import numpy as np
import pytest

from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from oracle.oracle import Oracle

PLANE = '<geom name="floor" type="plane" size="5 5 0.1"/>'


def _contacts(bodies: str, plane: str = PLANE, qpos=None):
  xml = f"""<mujoco><option gravity="0 0 0"/><worldbody>{plane}{bodies}</worldbody></mujoco>"""
  m = compile_spec(read_mjcf_string(xml), 16, 64)
  q = m.qpos0[None].copy() if qpos is None else np.asarray(qpos, float)[None]
  out = Oracle(m).run(1, {"qpos": q}, integrate=False)
  n = int(out["ncon"][0, 0])
  return (out["contact_dist"][0, :n], out["contact_pos"][0, : 3 * n].reshape(n, 3),
          out["contact_frame"][0, : 9 * n].reshape(n, 9)[:, :3], m)


def test_cylinder_standing_three_rim_contacts():
  """A cylinder (r 0.1, half height 0.2) standing 0.01 into the floor: three
  contacts on the bottom rim, 120 degrees apart, each at depth 0.01."""
  d, p, nrm, _ = _contacts('<body pos="0 0 0.19"><freejoint/><geom type="cylinder" size="0.1 0.2"/></body>')
  assert len(d) == 3
  np.testing.assert_allclose(d, -0.01, atol=1e-12)
  np.testing.assert_allclose(np.hypot(p[:, 0], p[:, 1]), 0.1, atol=1e-12)
  ang = np.sort(np.mod(np.arctan2(p[:, 1], p[:, 0]), 2 * np.pi))
  np.testing.assert_allclose(np.diff(ang), 2 * np.pi / 3, atol=1e-9)
  np.testing.assert_allclose(p[:, 2], -0.005, atol=1e-12)  # midway between the surfaces
  np.testing.assert_allclose(nrm, np.tile([0, 0, 1], (3, 1)), atol=1e-12)


def test_cylinder_lying_two_end_contacts():
  """Lying along x (rotated 90 degrees about y), 0.02 into the floor: the
  bottom line's two ends, x = +-0.2, depth 0.02."""
  q = [0, 0, 0.08, np.cos(np.pi / 4), 0, np.sin(np.pi / 4), 0]
  d, p, _, _ = _contacts('<body><freejoint/><geom type="cylinder" size="0.1 0.2"/></body>', qpos=q)
  assert len(d) == 2
  np.testing.assert_allclose(d, -0.02, atol=1e-12)
  np.testing.assert_allclose(sorted(p[:, 0]), [-0.2, 0.2], atol=1e-12)
  np.testing.assert_allclose(p[:, 1], 0, atol=1e-12)


def test_ellipsoid_resting_support_point():
  """An ellipsoid (0.3, 0.2, 0.1) tilted 30 degrees about x: the support
  point's height is -sqrt(b^2 sin^2 + c^2 cos^2) below the centre."""
  th = np.pi / 6
  h = np.sqrt(0.2**2 * np.sin(th) ** 2 + 0.1**2 * np.cos(th) ** 2)
  q = [0, 0, h - 0.005, np.cos(th / 2), np.sin(th / 2), 0, 0]
  d, p, nrm, _ = _contacts('<body><freejoint/><geom type="ellipsoid" size="0.3 0.2 0.1"/></body>', qpos=q)
  assert len(d) == 1
  assert d[0] == pytest.approx(-0.005, abs=1e-12)
  assert p[0, 0] == pytest.approx(0, abs=1e-12) and p[0, 2] == pytest.approx(-0.0025, abs=1e-12)
  np.testing.assert_allclose(nrm[0], [0, 0, 1], atol=1e-12)


@pytest.mark.parametrize("where,pos,dist", [
  ("side", [0.18, 0, 0], 0.18 - 0.1 - 0.1),
  ("cap", [0.02, 0, 0.28], 0.28 - 0.2 - 0.1),
  ("rim", [0.16, 0, 0.26], np.hypot(0.06, 0.06) - 0.1),
])
def test_sphere_cylinder_side_cap_rim(where, pos, dist):
  """A sphere (r 0.1) against a static upright cylinder (r 0.1, half height
  0.2): the distance to the shaft, to the cap plane, or to the rim circle."""
  plane = '<geom type="cylinder" size="0.1 0.2"/>'
  d, p, nrm, _ = _contacts(f'<body pos="{pos[0]} {pos[1]} {pos[2]}"><freejoint/><geom type="sphere" size="0.1"/></body>',
                           plane=plane)
  assert len(d) == 1, where
  assert d[0] == pytest.approx(dist, abs=1e-12)
  if where == "cap":
    np.testing.assert_allclose(nrm[0], [0, 0, -1], atol=1e-12)  # from the sphere into the cylinder


def test_ellipsoid_rbound_is_largest_semi_axis():
  _, _, _, m = _contacts('<body pos="0 0 1"><freejoint/><geom type="ellipsoid" size="0.3 0.2 0.1"/></body>')
  assert m.geom_rbound[1] == pytest.approx(0.3)
  assert m.nboxpair == 1 and not m.unsupported_pair_types
