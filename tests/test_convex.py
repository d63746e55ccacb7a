"""The general convex narrowphase (GJK + EPA, csrc/mjh_convex.h, compiled into
the oracle and the HIP step) against known answers.

MuJoCo collides every pair without a dedicated function (sphere-ellipsoid,
capsule-{ellipsoid,cylinder}, ellipsoid-{ellipsoid,cylinder,box},
cylinder-{cylinder,box}) with its convex collider, one contact per pair
(engine_collision_convex.c / engine_collision_gjk.c; MuJoCo Warp
collision_gjk.py). MuJoCo is absent here, so the oracle's contacts are pinned
by (1) closed-form configurations (axis-aligned stacks whose depth, normal and
witness points follow from the geometry), (2) an independent numpy
statement of the same quantity for random poses: the penetration depth of two
convex bodies is min over unit u of h1(u) + h2(-u) (h = support function,
written here from the shapes' definitions), the contact normal its minimiser,
and (3) a resting ellipsoid carrying its weight at the documented soft-contact
penetration (tests/test_soft_constraint.py). Normals point from geom1 to geom2
(pairs are ordered by geom type). The HIP step is checked against the oracle
in tests/test_gpu_parity.py::test_convex_pairs_parity."""

import numpy as np
import pytest

from mjlab_amd.spec.compiler import CONVEX_PAIRS, compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from mjlab_amd.utils import rot
from oracle.oracle import Oracle

NAMES = {2: "sphere", 3: "capsule", 4: "ellipsoid", 5: "cylinder", 6: "box"}


def _geom(t: int, size, extra: str = "") -> str:
  return f'<geom type="{NAMES[t]}" size="{" ".join(str(float(s)) for s in size)}" {extra}/>'


def _pair(t1, s1, q1, t2, s2, q2, margin=0.0, static2=False):
  """Contacts of geom (t1, s1) on a free body at pose q1 (pos + quat) and geom
  (t2, s2) at q2 (free, or static at q2 with static2). Returns dist, pos,
  normal, geom pairs and the model."""
  mg = f'margin="{margin}"'
  b1 = f'<body name="a"><freejoint/>{_geom(t1, s1, mg)}</body>'
  if static2:
    p, q = q2[:3], q2[3:]
    b2 = _geom(t2, s2, f'pos="{p[0]} {p[1]} {p[2]}" quat="{q[0]} {q[1]} {q[2]} {q[3]}" {mg}')
  else:
    b2 = f'<body name="b"><freejoint/>{_geom(t2, s2, mg)}</body>'
  xml = f'<mujoco><option gravity="0 0 0"/><worldbody>{b2 if static2 else ""}{b1}{"" if static2 else b2}</worldbody></mujoco>'
  m = compile_spec(read_mjcf_string(xml), 8, 64)
  assert not m.unsupported_pair_types
  qpos = np.asarray(q1, float) if static2 else np.concatenate([q1, q2])
  out = Oracle(m).run(1, {"qpos": qpos[None]}, integrate=False)
  n = int(out["ncon"][0, 0])
  geoms = out["contact_geom"][0, : 2 * n].reshape(n, 2)
  return (out["contact_dist"][0, :n], out["contact_pos"][0, : 3 * n].reshape(n, 3),
          out["contact_frame"][0, : 9 * n].reshape(n, 9)[:, :3], geoms, m)


def _pose(p, q=(1, 0, 0, 0)):
  return np.concatenate([np.asarray(p, float), np.asarray(q, float)])


def _axis_quat(axis, ang):
  return rot.axis_angle_to_quat(np.asarray(axis, float), ang)


# ---------------------------------------------------------------- closed forms
def test_sphere_ellipsoid_on_principal_axes():
  """A sphere (r 0.1) pressed 0.02 into a static ellipsoid (0.3, 0.2, 0.25)
  along its z and x axes: depth 0.02, normal from the sphere (geom1) into the
  ellipsoid, the contact midway between the surfaces."""
  for p, nrm, mid in (([0, 0, 0.33], [0, 0, -1], [0, 0, 0.24]), ([0.38, 0, 0], [-1, 0, 0], [0.29, 0, 0])):
    d, pos, n, _, _ = _pair(2, [0.1], _pose(p), 4, [0.3, 0.2, 0.25], _pose([0, 0, 0]), static2=True)
    assert len(d) == 1
    assert d[0] == pytest.approx(-0.02, abs=1e-7)
    np.testing.assert_allclose(n[0], nrm, atol=1e-6)
    np.testing.assert_allclose(pos[0], mid, atol=1e-6)


def test_ellipsoid_stack_and_margin():
  """Two ellipsoids (0.3, 0.2, 0.1) stacked on z: 0.19 apart -> depth 0.01;
  0.205 apart with margin 0.01 -> a contact at dist +0.005; 0.215 apart -> none."""
  s = [0.3, 0.2, 0.1]
  d, pos, n, g, _ = _pair(4, s, _pose([0, 0, 0.19]), 4, s, _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.01, abs=1e-7)
  assert abs(n[0, 2]) == pytest.approx(1, abs=1e-9)
  np.testing.assert_allclose(pos[0], [0, 0, 0.095], atol=1e-6)
  d, _, _, _, _ = _pair(4, s, _pose([0, 0, 0.205]), 4, s, _pose([0, 0, 0]), margin=0.01, static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(0.005, abs=1e-7)
  d, _, _, _, _ = _pair(4, s, _pose([0, 0, 0.215]), 4, s, _pose([0, 0, 0]), margin=0.01, static2=True)
  assert len(d) == 0


def test_cylinders_side_by_side_and_crossed():
  """Parallel upright cylinders (r 0.1, half height 0.2) 0.19 apart on x:
  depth 0.01 along x (a line contact: the point lies on the shared band);
  one lying along x across the other's cap, 0.01 deep: normal along z."""
  s = [0.1, 0.2]
  d, pos, n, _, _ = _pair(5, s, _pose([0.19, 0, 0]), 5, s, _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.01, abs=1e-7)
  assert abs(n[0, 0]) == pytest.approx(1, abs=1e-9)
  assert pos[0, 0] == pytest.approx(0.095, abs=1e-6) and abs(pos[0, 1]) < 1e-6 and abs(pos[0, 2]) <= 0.2 + 1e-9
  lying = _axis_quat([0, 1, 0], np.pi / 2)
  d, pos, n, _, _ = _pair(5, s, _pose([0, 0, 0.29], lying), 5, s, _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.01, abs=1e-7)
  assert abs(n[0, 2]) == pytest.approx(1, abs=1e-9)
  assert pos[0, 2] == pytest.approx(0.195, abs=1e-6) and np.hypot(pos[0, 0], pos[0, 1]) <= 0.1 + 1e-9


def test_cylinder_standing_on_box():
  """A cylinder (geom1) standing 0.01 into a static box's top face: normal
  from the cylinder into the box (0, 0, -1), the contact on the cap disc."""
  d, pos, n, _, _ = _pair(5, [0.1, 0.2], _pose([0.05, -0.1, 0.29]), 6, [0.5, 0.5, 0.1], _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.01, abs=1e-7)
  np.testing.assert_allclose(n[0], [0, 0, -1], atol=1e-9)
  assert pos[0, 2] == pytest.approx(0.095, abs=1e-6)
  assert np.hypot(pos[0, 0] - 0.05, pos[0, 1] + 0.1) <= 0.1 + 1e-9


def test_capsule_across_cylinder_cap():
  """A capsule (r 0.05, half length 0.2) lying along x over an upright
  cylinder's cap (top at 0.2), 0.01 deep: normal from the capsule down."""
  d, pos, n, _, _ = _pair(3, [0.05, 0.2], _pose([0, 0, 0.24], _axis_quat([0, 1, 0], np.pi / 2)), 5, [0.1, 0.2],
                          _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.01, abs=1e-7)
  np.testing.assert_allclose(n[0], [0, 0, -1], atol=1e-9)
  assert pos[0, 2] == pytest.approx(0.195, abs=1e-6) and abs(pos[0, 0]) <= 0.1 + 1e-9


def test_tilted_ellipsoid_on_box_support_point():
  """An ellipsoid (0.3, 0.2, 0.1) tilted 30 degrees about x, 0.005 into a box
  top (z = 0.1): its lowest point is sqrt(b^2 sin^2 + c^2 cos^2) below the
  centre, at y = (b^2 - c^2) sin cos / that height; the contact lies midway."""
  th = np.pi / 6
  b, c = 0.2, 0.1
  h = np.sqrt(b**2 * np.sin(th) ** 2 + c**2 * np.cos(th) ** 2)
  y = -(b**2 - c**2) * np.sin(th) * np.cos(th) / h
  d, pos, n, _, _ = _pair(4, [0.3, b, c], _pose([0, 0, 0.1 + h - 0.005], _axis_quat([1, 0, 0], th)), 6,
                          [0.5, 0.5, 0.1], _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.005, abs=1e-7)
  np.testing.assert_allclose(n[0], [0, 0, -1], atol=1e-6)
  # the ellipsoid's support point is unique: the contact is pinned to it
  assert abs(abs(pos[0, 1]) - abs(y)) < 2e-4 and pos[0, 2] == pytest.approx(0.0975, abs=1e-6)


def test_ellipsoid_on_cylinder_cap_and_capsule_on_ellipsoid():
  d, pos, n, _, _ = _pair(4, [0.15, 0.1, 0.07], _pose([0.02, 0, 0.266]), 5, [0.1, 0.2], _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.004, abs=1e-7)
  np.testing.assert_allclose(n[0], [0, 0, -1], atol=1e-6)
  np.testing.assert_allclose(pos[0], [0.02, 0, 0.198], atol=1e-5)
  # a capsule along y resting across an ellipsoid's top (c = 0.07): 0.003 deep
  d, pos, n, _, _ = _pair(3, [0.04, 0.1], _pose([0, 0, 0.107], _axis_quat([1, 0, 0], np.pi / 2)), 4, [0.15, 0.1, 0.07],
                          _pose([0, 0, 0]), static2=True)
  assert len(d) == 1 and d[0] == pytest.approx(-0.003, abs=1e-7)
  np.testing.assert_allclose(n[0], [0, 0, -1], atol=1e-6)
  np.testing.assert_allclose(pos[0], [0, 0, 0.0685], atol=1e-5)


# ---------------------------------------------------------------- support-function statement
def _support(t, size, R, c, U):
  """Support points of a shape (type t, size, rotation R, centre c) along the
  rows of U, from the shapes' definitions (independent of the C code)."""
  L = U @ R  # local directions
  if t == 2:
    P = np.zeros_like(L)
  elif t == 3:
    P = np.zeros_like(L)
    P[:, 2] = np.where(L[:, 2] >= 0, size[1], -size[1])
  elif t == 4:
    S = np.asarray(size[:3])
    P = S**2 * L / np.linalg.norm(S * L, axis=1, keepdims=True)
  elif t == 5:
    rl = np.linalg.norm(L[:, :2], axis=1, keepdims=True)
    P = np.zeros_like(L)
    P[:, :2] = size[0] * L[:, :2] / np.maximum(rl, 1e-300)
    P[:, 2] = np.where(L[:, 2] >= 0, size[1], -size[1])
  else:
    P = np.where(L >= 0, 1.0, -1.0) * np.asarray(size[:3])
  W = P @ R.T + c
  if t in (2, 3):
    W = W + size[0] * U / np.linalg.norm(U, axis=1, keepdims=True)
  return W


def _overlap(A, B, U):
  """h_A(u) + h_B(-u): the overlap of the two bodies' extents along u."""
  U = np.atleast_2d(U)
  U = U / np.linalg.norm(U, axis=1, keepdims=True)
  ha = np.einsum("ij,ij->i", _support(*A, U), U)
  hb = np.einsum("ij,ij->i", _support(*B, -U), -U)
  return ha + hb


def _min_overlap(A, B):
  """min over unit u of the overlap (dense Fibonacci sphere, then Nelder-Mead
  in the tangent plane of the best few directions)."""
  from scipy.optimize import minimize

  k = 40000
  i = np.arange(k) + 0.5
  phi, z = np.pi * (1 + 5**0.5) * i, 1 - 2 * i / k
  U = np.stack([np.sqrt(1 - z * z) * np.cos(phi), np.sqrt(1 - z * z) * np.sin(phi), z], 1)
  f = _overlap(A, B, U)
  best_f, best_u = np.inf, None
  for j in np.argsort(f)[:6]:
    u0 = U[j]
    t1 = np.cross(u0, [1.0, 0, 0] if abs(u0[0]) < 0.9 else [0, 1.0, 0])
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(u0, t1)
    res = minimize(lambda x: _overlap(A, B, u0 + x[0] * t1 + x[1] * t2)[0], np.zeros(2), method="Nelder-Mead",
                   options={"xatol": 1e-10, "fatol": 1e-12, "maxiter": 4000})
    if res.fun < best_f:
      u = u0 + res.x[0] * t1 + res.x[1] * t2
      best_f, best_u = res.fun, u / np.linalg.norm(u)
  return best_f, best_u


def _random_size(t, rng):
  if t == 2:
    return [rng.uniform(0.05, 0.15)]
  if t in (3, 5):
    return [rng.uniform(0.04, 0.12), rng.uniform(0.05, 0.2)]
  return list(rng.uniform(0.05, 0.2, 3))


@pytest.mark.parametrize("kind", sorted(CONVEX_PAIRS))
def test_random_poses_match_support_function_minimum(kind):
  """Random sizes and orientations, geom2 placed so the pair overlaps: the
  oracle's dist equals -min_u (h1(u) + h2(-u)) and its normal attains that
  minimum (the overlap along it equals the depth), both to 1e-6."""
  t1, t2 = kind
  rng = np.random.default_rng(100 + 10 * t1 + t2)
  done = 0
  while done < 4:
    s1, s2 = _random_size(t1, rng), _random_size(t2, rng)
    q1, q2 = rng.normal(size=4), rng.normal(size=4)
    q1, q2 = q1 / np.linalg.norm(q1), q2 / np.linalg.norm(q2)
    R1, R2 = rot.quat_to_mat(q1), rot.quat_to_mat(q2)
    u = rng.normal(size=3)
    u /= np.linalg.norm(u)
    A = (t1, s1, R1, np.zeros(3))
    # place geom2 along u, overlapping geom1 by about 10 % of the smaller size
    reach = _overlap(A, (t2, s2, R2, np.zeros(3)), u)[0]
    c2 = u * (reach - 0.1 * min(min(s1), min(s2)))
    B = (t2, s2, R2, c2)
    fmin, umin = _min_overlap(A, B)
    if not 1e-3 < fmin < 0.5 * min(min(s1), min(s2)):
      continue
    d, pos, n, g, m = _pair(t1, s1, _pose([0, 0, 0], q1), t2, s2, _pose(c2, q2), static2=True)
    # in the model the static geom2 is geom 0, the free body's geom1 is geom 1; pairs run type-ascending
    assert len(d) == 1, (kind, fmin)
    first_is_1 = int(m.geom_type[g[0, 0]]) == t1 and (t1 != t2 or g[0, 0] == 1)
    P, Q = (A, B) if first_is_1 else (B, A)
    assert d[0] == pytest.approx(-fmin, abs=1e-6), (kind, d[0], fmin)
    assert _overlap(P, Q, n[0])[0] == pytest.approx(fmin, abs=1e-6), (kind, n[0], umin)
    # the contact lies between the two bodies' extreme points along the normal
    lo = np.dot(_support(*Q, -n[0][None])[0], n[0])
    hi = np.dot(_support(*P, n[0][None])[0], n[0])
    assert np.dot(pos[0], n[0]) == pytest.approx(0.5 * (lo + hi), abs=3e-6)
    done += 1


def test_ellipsoid_pair_witness_points():
  """Strictly convex pairs have unique witness points: the contact is the
  midpoint of geom1's support along n and geom2's along -n."""
  rng = np.random.default_rng(7)
  done = 0
  while done < 4:
    s1, s2 = list(rng.uniform(0.06, 0.2, 3)), list(rng.uniform(0.06, 0.2, 3))
    q1, q2 = rng.normal(size=4), rng.normal(size=4)
    q1, q2 = q1 / np.linalg.norm(q1), q2 / np.linalg.norm(q2)
    u = rng.normal(size=3)
    u /= np.linalg.norm(u)
    A = (4, s1, rot.quat_to_mat(q1), np.zeros(3))
    reach = _overlap(A, (4, s2, rot.quat_to_mat(q2), np.zeros(3)), u)[0]
    c2 = u * (reach - 0.02)
    B = (4, s2, rot.quat_to_mat(q2), c2)
    if _min_overlap(A, B)[0] < 1e-3:  # overlapping along u, separated along another direction
      continue
    d, pos, n, g, _ = _pair(4, s1, _pose([0, 0, 0], q1), 4, s2, _pose(c2, q2), static2=True)
    assert len(d) == 1
    P, Q = (A, B) if g[0, 0] == 1 else (B, A)
    mid = 0.5 * (_support(*P, n[0][None])[0] + _support(*Q, -n[0][None])[0])
    np.testing.assert_allclose(pos[0], mid, atol=1e-6)
    done += 1


# ---------------------------------------------------------------- dynamics
def test_ellipsoid_resting_on_box_carries_its_weight():
  """A 1.5 kg ellipsoid (0.2, 0.15, 0.1) dropped flat onto a static box comes
  to rest on one contact below its centre at the documented soft-contact
  penetration r* (default solref/solimp, pyramidal condim 3), carrying m g."""
  xml = """<mujoco><option timestep="0.005"/><worldbody><geom type="box" size="0.5 0.5 0.1"/>
  <body name="e" pos="0 0 0.22"><freejoint/><geom type="ellipsoid" size="0.2 0.15 0.1" mass="1.5"/></body>
  </worldbody></mujoco>"""
  m = compile_spec(read_mjcf_string(xml), 8, 64)
  orc = Oracle(m)
  st = {"qpos": m.qpos0[None].copy()}
  for _ in range(600):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
  from tests.test_soft_constraint import rest_penetration

  rs = rest_penetration((0.02, 1.0), (0.9, 0.95, 0.001, 0.5, 2.0), m.timestep)
  assert int(out["ncon"][0, 0]) == 1
  assert st["qpos"][0, 2] - 0.2 == pytest.approx(rs, rel=1e-4)
  assert abs(st["qvel"][0]).max() < 1e-5  # a slow residual rocking on the curved bottom
  assert out["qfrc_constraint"][0, 2] == pytest.approx(1.5 * 9.81, rel=1e-3)
