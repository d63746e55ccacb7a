"""Box narrowphase (sphere-box, capsule-box, box-box) in the oracle: analytic
known answers (distance, normal from geom1 to geom2, midpoint position) and a
box resting on a box carrying its weight. The HIP kernel runs the same
algorithms; tests/test_gpu_parity.py::test_box_pairs_parity compares them."""

import math

import numpy as np
import pytest

from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from oracle.oracle import Oracle

BOX = '<geom name="table" type="box" size="0.5 0.5 0.1"/>'


def model(body_xml: str, world_xml: str = BOX):
  xml = f"""<mujoco><compiler angle="radian"/><option timestep="0.002"/><worldbody>{world_xml}
  <body name="b" pos="0 0 0"><freejoint/>{body_xml}</body></worldbody></mujoco>"""
  return compile_spec(read_mjcf_string(xml), 8, 64)


def contacts(m, qpos7):
  q = np.asarray(qpos7, np.float64)[None]
  out = Oracle(m).run(1, {"qpos": q}, integrate=False)
  n = int(out["ncon"][0, 0])
  return n, out["contact_dist"][0, :n], out["contact_pos"][0].reshape(-1, 3)[:n], out["contact_frame"][0].reshape(-1, 9)[:n, :3]


def test_sphere_on_box_face():
  m = model('<geom type="sphere" size="0.1"/>')
  n, d, p, f = contacts(m, [0.1, 0.2, 0.19, 1, 0, 0, 0])
  assert n == 1
  assert d[0] == pytest.approx(-0.01, abs=1e-12)
  np.testing.assert_allclose(f[0], [0, 0, -1], atol=1e-12)  # pairs are ordered by type: sphere (geom1) -> table
  np.testing.assert_allclose(p[0], [0.1, 0.2, 0.095], atol=1e-12)


def test_sphere_centre_inside_box_leaves_through_nearest_face():
  m = model('<geom type="sphere" size="0.05"/>')
  n, d, p, f = contacts(m, [0.45, 0.0, 0.0, 1, 0, 0, 0])
  assert n == 1
  assert d[0] == pytest.approx(-0.1, abs=1e-12)
  np.testing.assert_allclose(np.abs(f[0]), [1, 0, 0], atol=1e-12)
  np.testing.assert_allclose(p[0], [0.45, 0, 0], atol=1e-12)


def test_capsule_lying_on_box_two_contacts():
  m = model('<geom type="capsule" size="0.05 0.2" euler="0 1.5707963267948966 0"/>')
  n, d, p, f = contacts(m, [0, 0, 0.14, 1, 0, 0, 0])
  assert n == 2
  np.testing.assert_allclose(d, [-0.01, -0.01], atol=1e-9)
  np.testing.assert_allclose(sorted(p[:, 0]), [-0.2, 0.2], atol=1e-9)
  np.testing.assert_allclose(p[:, 2], [0.095, 0.095], atol=1e-9)
  np.testing.assert_allclose(np.abs(f[:, 2]), [1, 1], atol=1e-9)


def _box_sdf(bs, q):
  o = np.abs(q) - bs
  out = np.linalg.norm(np.maximum(o, 0))
  return out if out > 0 else o.max()


def test_capsule_across_box_edge_nearest_point():
  """A tilted capsule over the table's edge: one contact whose distance is the
  segment's minimum signed distance to the box minus the radius (dense
  sampling of the segment)."""
  ang = 0.7
  m = model(f'<geom type="capsule" size="0.04 0.25" euler="0 {ang} 0.3"/>')
  pos = np.array([0.55, 0.1, 0.16])
  n, d, p, f = contacts(m, [*pos, 1, 0, 0, 0])
  # the capsule axis (euler xyz, moving axes): Ry(ang) Rz(0.3) z = (sin ang, 0, cos ang)
  ax = np.array([math.sin(ang), 0.0, math.cos(ang)])
  ts = np.linspace(-0.25, 0.25, 200001)
  sd = min(_box_sdf(np.array([0.5, 0.5, 0.1]), pos + t * ax) for t in ts[::50])
  assert n == 1
  assert d[0] == pytest.approx(sd - 0.04, abs=2e-5)


def test_box_resting_on_box_face_four_corners():
  m = model('<geom type="box" size="0.1 0.1 0.1"/>')
  n, d, p, f = contacts(m, [0.05, -0.1, 0.19, 1, 0, 0, 0])
  assert n == 4
  np.testing.assert_allclose(d, [-0.01] * 4, atol=1e-12)
  np.testing.assert_allclose(f, np.tile([0, 0, 1.0], (4, 1)), atol=1e-12)
  np.testing.assert_allclose(p[:, 2], [0.095] * 4, atol=1e-12)
  got = sorted(map(tuple, np.round(p[:, :2], 9)))
  assert got == sorted([(0.15, 0.0), (0.15, -0.2), (-0.05, 0.0), (-0.05, -0.2)])


def test_box_box_edge_edge():
  """Two cubes, the lower turned 45 deg about x, the upper 45 deg about y:
  their crossing edges touch at one point; penetration 0.01."""
  s2 = math.sqrt(2.0)
  world = '<geom name="a" type="box" size="0.1 0.1 0.1" euler="0.7853981633974483 0 0"/>'
  m = model('<geom type="box" size="0.1 0.1 0.1" euler="0 0.7853981633974483 0"/>', world)
  n, d, p, f = contacts(m, [0, 0, 0.2 * s2 - 0.01, 1, 0, 0, 0])
  assert n == 1
  assert d[0] == pytest.approx(-0.01, abs=1e-9)
  np.testing.assert_allclose(f[0], [0, 0, 1], atol=1e-9)
  np.testing.assert_allclose(p[0], [0, 0, 0.1 * s2 - 0.005], atol=1e-9)


def test_separated_boxes_no_contact():
  m = model('<geom type="box" size="0.1 0.1 0.1"/>')
  assert contacts(m, [0.0, 0.0, 0.21, 1, 0, 0, 0])[0] == 0
  assert contacts(m, [0.7, 0.0, 0.1, 1, 0, 0, 0])[0] == 0


def test_box_on_box_carries_its_weight():
  """A 2 kg cube dropped onto the table comes to rest; the constraint force
  on its free joint carries m g."""
  m = model('<geom type="box" size="0.1 0.1 0.1" mass="2"/>')
  orc = Oracle(m)
  st = {"qpos": np.array([[0.05, -0.1, 0.205, 1, 0, 0, 0]])}
  fz = []
  for _ in range(400):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    fz.append(out["qfrc_constraint"][0, 2])
  assert np.mean(fz[-100:]) == pytest.approx(2.0 * 9.81, rel=0.01)
  assert abs(st["qpos"][0, 2] - 0.2) < 2e-3 and np.abs(st["qvel"]).max() < 1e-2
