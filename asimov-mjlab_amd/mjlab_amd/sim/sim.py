"""Simulation: the drop-in replacement for mjlab's MuJoCo-Warp boundary.

Same surface as ``src/mjlab/sim/sim.py:97-199``: ``Simulation(num_envs, cfg,
model, device)`` with ``.mj_model``, ``.model``/``.data`` bridges,
``expand_model_fields``, ``forward``, ``step``, ``create_graph`` and a
``nan_guard``. ``MujocoCfg`` / ``SimulationCfg`` mirror ``sim.py:42-94``.

Differences by construction (MI355X-first):
* torch allocates every buffer; the HIP library only receives raw pointers
  through the ``mjh_model``/``mjh_data`` descriptors (include/mjh_abi.h);
* ``step``/``forward`` launch one kernel each on torch's current stream, and
  are replayed from ``torch.cuda.CUDAGraph`` (hipGraph) captures;
* there is no CPU physics fallback: on a non-GPU device the bridges work (host
  logic, indexing, writes) but ``step``/``forward`` raise.
"""

from __future__ import annotations

import ctypes
import json
import os
from collections import deque
from contextlib import contextmanager
from dataclasses import dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Literal

import numpy as np
import torch

from mjlab_amd.sim import abi, native
from mjlab_amd.utils.capture import GraphSlot
from mjlab_amd.sim.sim_data import Epoch, BATCHED_STATIC, DATA_SHAPES, MODEL_SHAPES, Bridge, make_opt, shape_of
from mjlab_amd.spec.compiler import Model

_INTEGRATORS = {"euler": 0, "implicitfast": 3}
_SOLVERS = {"pgs": 0, "cg": 1, "newton": 2}
_CONES = {"pyramidal": 0, "elliptic": 1}


@dataclass
class MujocoCfg:
  timestep: float = 0.002
  integrator: Literal["euler", "implicitfast"] = "implicitfast"
  impratio: float = 1.0
  cone: Literal["pyramidal", "elliptic"] = "pyramidal"
  jacobian: Literal["auto", "dense", "sparse"] = "auto"
  solver: Literal["newton", "cg", "pgs"] = "newton"
  iterations: int = 100
  tolerance: float = 1e-8
  ls_iterations: int = 50
  ls_tolerance: float = 0.01
  gravity: tuple[float, float, float] = (0, 0, -9.81)

  def apply(self, model: Model) -> None:
    if self.cone not in _CONES:
      raise ValueError(f"unknown friction cone {self.cone!r}")
    if self.solver not in _SOLVERS:
      raise ValueError(f"unknown solver {self.solver!r}")
    if self.solver == "pgs" and self.cone == "elliptic":
      # MuJoCo C's PGS projects each elliptic contact with a small QCQP; the
      # device PGS (mjh_step.hip) handles pyramidal cones, limits and friction loss
      raise NotImplementedError("the PGS solver supports pyramidal cones only (use Newton or CG for elliptic)")
    model.cone = _CONES[self.cone]
    model.solver = _SOLVERS[self.solver]
    model.jacobian = {"dense": 0, "sparse": 1, "auto": 2}[self.jacobian]
    model.integrator = _INTEGRATORS[self.integrator]
    model.timestep = self.timestep
    model.impratio = self.impratio
    model.gravity = np.array(self.gravity, dtype=np.float64)
    model.iterations = self.iterations
    model.tolerance = self.tolerance
    model.ls_iterations = self.ls_iterations
    model.ls_tolerance = self.ls_tolerance


@dataclass
class NanGuardCfg:
  enabled: bool = False
  buffer_size: int = 100
  output_dir: str = "/tmp/mjlab/nan_dumps"
  max_envs_to_dump: int = 5


class NanGuard:
  """Rolling buffer of physics states, dumped to disk when NaN/Inf appears
  (``src/mjlab/utils/nan_guard.py:26-171``).

  Disabled (the default) every call is a no-op. Enabled, ``capture`` copies
  the mjSTATE_PHYSICS state of every world to the host before each step (one
  sync per step: a debugging aid, as in the reference) and ``check_and_dump``
  writes the buffered states of the first ``max_envs_to_dump`` non-finite
  worlds to ``nan_dump_<timestamp>.npz``. The state layout is MuJoCo's
  mjSTATE_PHYSICS = [qpos (nq), qvel (nv), act (na)] in float64 (the models
  here have no plugin or history state). ``_metadata`` is the same dict object
  array the reference writes (``nan_guard.py:135-150``; read by
  ``scripts/nan_viz.py:31`` with ``.item()``). MuJoCo is absent, so the model
  cannot be saved as MJB: it is written as MJCF (``model_<timestamp>.xml``,
  ``spec.mjcf.model_to_mjcf``), which ``MjModel.from_xml_path`` loads with the
  same body/dof/geom order; ``mjlab_amd.utils.nan_guard.load_nan_dump`` reads
  both files (the reference viewer needs ``from_xml_path`` in place of
  ``from_binary_path`` for this one file).
  """

  def __init__(self, cfg: NanGuardCfg, num_envs: int, model) -> None:
    self.cfg = cfg
    self.enabled = cfg.enabled
    self.num_envs = num_envs
    self.tripped: torch.Tensor | None = None
    if not self.enabled:
      return
    self.buffer_size = cfg.buffer_size
    self.output_dir = Path(cfg.output_dir)
    self.max_envs_to_dump = cfg.max_envs_to_dump
    self.buffer: deque = deque(maxlen=self.buffer_size)
    self.step_counter = 0
    self._dumped = False
    self.model = model
    self.state_size = int(model.nq + model.nv + model.na)

  def capture(self, data) -> None:
    if not self.enabled:
      return
    parts = [data.qpos, data.qvel] + ([data.act] if self.model.na > 0 else [])
    states = torch.cat([p.reshape(p.shape[0], -1) for p in parts], dim=1).double().cpu().numpy()
    self.buffer.append({"step": self.step_counter, "states": states})
    self.step_counter += 1

  @contextmanager
  def watch(self, data):
    self.capture(data)
    yield
    self.check_and_dump(data)

  @staticmethod
  def detect_nans(data) -> torch.Tensor:
    """Per-world bool: NaN/Inf in qpos, qvel, qacc or qacc_warmstart (nan_guard.py:86-104)."""
    m = torch.zeros(data.qpos.shape[0], dtype=torch.bool, device=data.qpos.device)
    for t in (data.qpos, data.qvel, data.qacc, data.qacc_warmstart):
      m |= ~torch.isfinite(t).all(dim=-1)
    return m

  def check_and_dump(self, data) -> bool:
    if not self.enabled or self._dumped:
      return False
    bad = self.detect_nans(data)
    if not bool(bad.any()):
      return False
    ids = torch.where(bad)[0].cpu().numpy().tolist()
    self.tripped = bad.nonzero().flatten()
    self._dump_buffer(ids)
    self._dumped = True
    return True

  def _dump_buffer(self, nan_env_ids: list[int]) -> Path:
    self.output_dir.mkdir(parents=True, exist_ok=True)
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    fname = self.output_dir / f"nan_dump_{stamp}.npz"
    mname = self.output_dir / f"model_{stamp}.xml"
    envs = nan_env_ids[: self.max_envs_to_dump]
    out = {f"states_step_{it['step']:06d}": it["states"][envs] for it in self.buffer}
    meta = {
      "num_envs_total": self.num_envs, "num_envs_dumped": len(envs), "nan_env_ids": nan_env_ids,
      "dumped_env_ids": list(envs), "state_size": self.state_size, "buffer_size": len(self.buffer),
      "detection_step": self.step_counter, "timestamp": stamp, "model_file": mname.name,
      "note": "States in mjSTATE_PHYSICS layout [qpos, qvel, act] (float64); use mj_setState to restore. "
      "Model saved as MJCF (MjModel.from_xml_path).",
    }
    out["_metadata"] = np.array(meta, dtype=object)
    np.savez_compressed(fname, **out)
    from mjlab_amd.spec.mjcf import model_to_mjcf

    mname.write_text(model_to_mjcf(self.model))
    for link, target in ((self.output_dir / "nan_dump_latest.npz", fname), (self.output_dir / "model_latest.xml", mname)):
      link.unlink(missing_ok=True)
      link.symlink_to(target.name)
    print(f"[NanGuard] Detected NaN/Inf at step {self.step_counter}; envs {nan_env_ids[:10]}; "
          f"dumped {len(envs)} envs x {len(self.buffer)} states to {fname}")
    return fname


@dataclass(kw_only=True)
class SimulationCfg:
  nconmax: int | None = None
  njmax: int | None = None
  ls_parallel: bool = True
  contact_sensor_maxmatch: int = 64
  # worlds handed to workgroups in order of their previous step's cost (one counting-sort
  # launch before each physics launch): G1 4096 0.741 -> 0.700 ms per step launch
  balance_worlds: bool = True
  # model-specialised step kernel for a model outside the built-in table
  # (mjlab_amd/sim/jit.py): "auto" compiles a launch plugin once per launch plan
  # (cached), "cached" only uses one already built, "off" keeps the generic
  # instance; default from MJH_SPECIALIZE (the test suite sets "cached")
  specialize: str = field(default_factory=lambda: os.environ.get("MJH_SPECIALIZE", "auto"))
  mujoco: MujocoCfg = field(default_factory=MujocoCfg)
  nan_guard: NanGuardCfg = field(default_factory=NanGuardCfg)


_TORCH_DT = {"float": torch.float32, "int": torch.int32, "mjh_i64": torch.int64}


class Simulation:
  # captured graphs live outside the instance (utils/capture.py: capture-safe release)
  step_graph = GraphSlot()
  forward_graph = GraphSlot()

  def __init__(self, num_envs: int, cfg: SimulationCfg, model: Model, device: str) -> None:
    self.cfg = cfg
    self.device = device
    self.num_envs = num_envs
    self._mj_model = model
    cfg.mujoco.apply(model)
    if cfg.njmax is not None:
      model.njmax = int(cfg.njmax)
    # Contacts: the reference's nconmax sizes a pool shared by all worlds ("one
    # world may have more than nconmax contacts", sim.py:81-85; MuJoCo Warp
    # allocates nconmax x nworld). Each world here gets max(nconmax, njmax)
    # slots: a world keeps more than nconmax contacts while others hold fewer
    # (beyond njmax its rows overflow anyway). The slot count does not depend
    # on the world count, so the model-specialised kernels' plans hold for any
    # num_envs; the pool's total is not enforced across worlds.
    share = int(cfg.nconmax) if cfg.nconmax is not None else int(getattr(model, "ncon_share", model.nconmax))
    model.ncon_share = share
    model.nconmax = max(share, int(model.njmax))
    if cfg.contact_sensor_maxmatch > 64:  # keep the exact-match guarantee below: at most 64 slots
      model.nconmax = max(share, min(model.nconmax, 64))
    # the kernel keeps one wave lane per contact-sensor match (64): a cap above 64
    # is honoured exactly when no world can hold more than 64 contacts, since a
    # sensor never matches more contacts than the world has
    if cfg.contact_sensor_maxmatch > 64 and model.nconmax > 64:
      raise ValueError(f"contact_sensor_maxmatch={cfg.contact_sensor_maxmatch} > 64 needs nconmax <= 64 per world "
                       f"(got nconmax={model.nconmax}): the contact sensor keeps at most 64 matches")
    if cfg.contact_sensor_maxmatch < 1:
      raise ValueError("contact_sensor_maxmatch must be >= 1")
    model.contact_sensor_maxmatch = cfg.contact_sensor_maxmatch
    model.ls_parallel = int(bool(cfg.ls_parallel))  # wp_model.opt.ls_parallel (sim.py:117)
    self.sizes = abi.model_sizes(model)
    # A scene's env-origin sites (Model.nsite_origin, the leading world sites) are
    # static: the kernel's model view starts after them (ksizes, offset site
    # pointers, shifted sensor site ids) and writes its sites into the wide
    # site_xpos / site_xmat rows after the static block written here once.
    self._nsite0 = int(getattr(model, "nsite_origin", 0))
    self.ksizes = dict(self.sizes, nsite=self.sizes["nsite"] - self._nsite0)
    if self._nsite0:
      site_obj = 6  # mjOBJ_SITE
      for t, i in ((model.sensor_objtype, model.sensor_objid), (model.sensor_reftype, model.sensor_refid)):
        if ((np.asarray(t) == site_obj) & (np.asarray(i) < self._nsite0)).any():
          raise NotImplementedError("a sensor references an env-origin site (static, not simulated per world)")

    # ---- model buffers (torch-owned) ----
    host = abi.model_host_arrays(model)
    self._model_flat: dict[str, torch.Tensor] = {}
    self._wstride: dict[str, int] = {}
    self._fields = {f.name: f for f in abi.model_array_fields()}
    for f in abi.model_array_fields():
      self._model_flat[f.name] = torch.as_tensor(host[f.name], dtype=_TORCH_DT[f.ctype], device=device).contiguous()
      if f.kind == "MW":
        self._wstride[f.name] = 0
    model_views = {n: self._model_view(n) for n in self._model_flat}
    self._model_bridge = Bridge(model_views, extra={"opt": make_opt(model, cfg)}, nworld=num_envs)

    # ---- data buffers ----
    # one slab, array f at num_envs * (words per world of the arrays before it),
    # header order: specialised kernel instances derive every data pointer
    # from qpos with compile-time offsets (mjh_data_is_slab)
    self._data_flat: dict[str, torch.Tensor] = {}
    counts = [(f, max(1, abi.count(f, self.ksizes))) for f in abi.data_array_fields()]
    self._slab = torch.zeros(num_envs * sum(c for _, c in counts), dtype=torch.float32, device=device)
    off = 0
    for f, c in counts:
      v = self._slab[off * num_envs : (off + c) * num_envs].view(num_envs, c)
      self._data_flat[f.name] = v if _TORCH_DT[f.ctype] == torch.float32 else v.view(_TORCH_DT[f.ctype])
      off += c
    self._data_flat["qpos"][:] = torch.as_tensor(model.qpos0, dtype=torch.float32, device=device)
    if int(model.nmocap) > 0:  # mj_resetData: mocap poses start at the bodies' model poses
      mb = np.argsort(np.where(model.body_mocapid >= 0, model.body_mocapid, np.iinfo(np.int32).max))[: int(model.nmocap)]
      self._data_flat["mocap_pos"][:] = torch.as_tensor(np.asarray(model.body_pos)[mb].reshape(-1), dtype=torch.float32)
      self._data_flat["mocap_quat"][:] = torch.as_tensor(np.asarray(model.body_quat)[mb].reshape(-1), dtype=torch.float32)
    if self._nsite0:
      # the wide site outputs: (num_envs, nsite) with the static env-origin block
      # (world body at the origin: xpos = site_pos, xmat = R(site_quat))
      n0, ns = self._nsite0, self.sizes["nsite"]
      sp = torch.as_tensor(np.asarray(model.site_pos)[:n0], dtype=torch.float32)
      sq = np.asarray(model.site_quat)[:n0]
      from mjlab_amd.utils import rot

      sm = torch.as_tensor(np.stack([rot.quat_to_mat(q).reshape(-1) for q in sq]) if n0 else np.zeros((0, 9)),
                           dtype=torch.float32)
      xp = torch.zeros(num_envs, ns * 3, dtype=torch.float32, device=device)
      xm = torch.zeros(num_envs, ns * 9, dtype=torch.float32, device=device)
      xp[:, : n0 * 3] = sp.reshape(1, -1).to(device)
      xm[:, : n0 * 9] = sm.reshape(1, -1).to(device)
      self._data_flat["site_xpos"], self._data_flat["site_xmat"] = xp, xm
    data_views = {n: self._data_view(n) for n in self._data_flat}
    self.epoch = Epoch()
    self._data_bridge = Bridge(data_views, extra={"epoch": self.epoch}, nworld=num_envs)

    self._build_structs()
    self.use_cuda_graph = str(device).startswith("cuda") and torch.cuda.is_available()
    self.step_graph = None
    self.forward_graph = None
    self.nan_guard = NanGuard(cfg.nan_guard, num_envs, model)
    self._kernel = {"kind": "generic", "index": -1, "reason": "not selected"}
    if self.use_cuda_graph:
      native.check(native.lib().mjh_model_check(ctypes.addressof(self._mstruct)), "mjh_model_check")
      self._select_kernel()
      self._launch_forward()
      self.create_graph()

  # ---- descriptors ----
  def _model_view(self, name: str) -> torch.Tensor:
    flat = self._model_flat[name]
    if name in MODEL_SHAPES:
      shp = shape_of(MODEL_SHAPES[name], self.sizes)
      if name in self._wstride or name in BATCHED_STATIC:
        if flat.numel() == 0:  # empty field (e.g. no actuators): dim0 cannot be inferred
          return flat.view(self.num_envs if name in self._wstride else 1, *shp)
        return flat.view(-1, *shp)
      return flat.view(*shp)
    return flat

  def _data_view(self, name: str) -> torch.Tensor:
    flat = self._data_flat[name]
    shp = shape_of(DATA_SHAPES.get(name, (flat.shape[1],)), self.sizes)
    if shp == ():
      return flat.view(-1)
    if 0 in shp:
      return flat[:, :0].reshape(flat.shape[0], *shp)
    return flat.view(flat.shape[0], *shp)

  def _build_structs(self) -> None:
    MS = abi.model_struct()
    DS = abi.data_struct()
    ms = MS()
    for k, v in self.ksizes.items():
      setattr(ms, k, v)
    for k, v in abi.model_options(self._mj_model).items():
      setattr(ms, k, v)
    n0 = self._nsite0
    # the kernel's site arrays start after the static env-origin sites
    site_skip = {"site_bodyid": n0, "site_pos": 3 * n0, "site_quat": 4 * n0}
    if n0 and not hasattr(self, "_ksensor"):
      ids = {}
      for tn, idn in (("sensor_objtype", "sensor_objid"), ("sensor_reftype", "sensor_refid")):
        t, i = self._model_flat[tn], self._model_flat[idn]
        ids[idn] = torch.where(t == 6, i - n0, i).contiguous()
      self._ksensor = ids
    for name, t in self._model_flat.items():
      ptr = t.data_ptr() + site_skip.get(name, 0) * t.element_size()
      if n0 and name in ("sensor_objid", "sensor_refid"):
        ptr = self._ksensor[name].data_ptr()
      setattr(ms, name, ptr)
      if name in self._wstride:
        setattr(ms, name + "_wstride", self._wstride[name])
    # packed model image scratch (staged into LDS by every launch)
    if not hasattr(self, "_image"):
      words = int(native.lib().mjh_image_words(ctypes.addressof(ms))) if self._native_ok() else 16
      self._image = torch.zeros(words + 4, dtype=torch.float32, device=self.device)
    ms.image = self._image.data_ptr()
    ms.image_words = self._image.numel()
    ds = DS()
    ds.nworld = self.num_envs
    if not hasattr(self, "_scratch"):
      words = int(native.lib().mjh_scratch_words(ctypes.addressof(ms))) if self._native_ok() else 16
      # zeroed: the split step's per-world position snapshots start invalid
      self._scratch = torch.zeros(self.num_envs * words, dtype=torch.float32, device=self.device)
      self._scratch_words = words
    ds.scratch = self._scratch.data_ptr()
    ds.scratch_words = self._scratch_words
    # worlds are handed to waves in order of last step's constraint count
    # (refreshed on the device before every launch; results are order-free)
    if not hasattr(self, "_order"):
      self._order = torch.arange(self.num_envs, dtype=torch.int64, device=self.device)
      self._order_keys = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
      self._order_cost = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
    ds.world_order = self._order.data_ptr() if self.cfg.balance_worlds else None
    for name, t in self._data_flat.items():
      setattr(ds, name, t.data_ptr())
    if n0:  # wide site outputs: world w's kernel site s at w * nsite + n0 + s
      ds.site_wstride = self.sizes["nsite"]
      ds.site_off = n0
    self._mstruct, self._dstruct = ms, ds
    # the same descriptor with the fused contact-sensor timers (attach_air_time)
    self._dstruct_at = None
    at = getattr(self, "_air_time", None)
    if at is not None:
      dsa = DS()
      ctypes.memmove(ctypes.addressof(dsa), ctypes.addressof(ds), ctypes.sizeof(DS))
      cols, tensors = at
      for name, t in zip(("last_time", "cur_air", "last_air", "cur_con", "last_con"), tensors):
        setattr(dsa, "at_" + name, t.data_ptr())
      dsa.at_k = len(cols)
      for j, c in enumerate(cols):
        dsa.at_cols[j] = int(c)
      self._dstruct_at = dsa
    # bumped whenever the descriptors change: graphs that baked them are stale
    # and are re-captured lazily by the next step()/forward()
    self.struct_version = getattr(self, "struct_version", 0) + 1
    self.step_graph = None
    self.forward_graph = None

  def _native_ok(self) -> bool:
    try:
      native.lib()
      return True
    except native.NativeLibraryError:
      if str(self.device).startswith("cuda"):
        raise
      return False

  def set_option(self, **kw) -> None:
    """Change solver/integrator options after construction (re-captures graphs)."""

    for k, v in kw.items():
      setattr(self._mj_model, k, v)
    self._build_structs()
    if self.use_cuda_graph:
      self._select_kernel()
      self.create_graph()

  def _select_kernel(self) -> None:
    """The step-kernel instance of this model: a built-in specialisation, a launch
    plugin (built once per plan, mjlab_amd/sim/jit.py) or the generic instance."""
    from mjlab_amd.sim import jit

    mode = getattr(self.cfg, "specialize", "auto")
    if mode == "off":
      k = int(native.lib().mjh_spec_index(ctypes.addressof(self._mstruct)))
      self._kernel = {"kind": "builtin", "index": k} if k >= 0 else {"kind": "generic", "index": -1, "reason": "off"}
      return
    self._kernel = jit.ensure(ctypes.addressof(self._mstruct), self._mj_model, name=getattr(self._mj_model, "name", "model"),
                              compile_missing=(mode == "auto"))

  def kernel_instance(self) -> dict:
    """Which step-kernel instance runs: {"kind": "builtin"|"plugin"|"generic", "index": ..}."""
    return dict(self._kernel)

  # ---- reference API ----
  @property
  def mj_model(self) -> Model:
    return self._mj_model

  @property
  def mj_data(self):
    return None

  @property
  def wp_model(self) -> Bridge:
    return self._model_bridge

  @property
  def wp_data(self) -> Bridge:
    return self._data_bridge

  @property
  def data(self) -> Bridge:
    return self._data_bridge

  @property
  def model(self) -> Bridge:
    return self._model_bridge

  def expand_model_fields(self, fields: tuple[str, ...]) -> None:
    invalid = [f for f in fields if not hasattr(self._mj_model, f)]
    if invalid:
      raise ValueError(f"Fields not found in model: {invalid}")
    not_expandable = [f for f in fields if f not in self._wstride]
    if not_expandable:
      raise ValueError(f"Fields cannot be expanded per world: {not_expandable}")
    for name in fields:
      if self._wstride[name] != 0:
        continue
      src = self._model_flat[name]
      n = src.numel()
      dst = torch.empty(self.num_envs * n, dtype=src.dtype, device=src.device)
      if self.use_cuda_graph:
        native.check(
          native.lib().mjh_repeat(
            ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()), n, self.num_envs,
            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
          ),
          "mjh_repeat",
        )
      else:
        dst.copy_(src.repeat(self.num_envs))
      self._model_flat[name] = dst
      self._wstride[name] = n
      self._model_bridge._rebind(name, self._model_view(name))
    self._build_structs()

  def create_graph(self) -> None:
    self.step_graph = None
    self.forward_graph = None
    if not self.use_cuda_graph:
      return
    # no warm-up launch here: it would run a real forward (and overwrite
    # qacc_warmstart); the constructor's first forward() already set the
    # kernels' LDS attributes outside any capture
    from mjlab_amd.utils.capture import no_gc

    with no_gc():
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g):
        self._launch_step()
      g2 = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g2):
        self._launch_forward()
    self.step_graph = g
    self.forward_graph = g2

  def _stream(self) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

  def _refresh_order(self) -> None:
    # default: the step library rewrites world_order inside its pack launch
    # (mjh_set_world_ordering, set at load); the separate launch is the A/B path
    if self.cfg.balance_worlds and self.num_envs > 1 and os.environ.get("MJH_PACK_ORDER") == "0":
      # expected cost of a world ~ (solver iterations + 2) x constraint rows of
      # its previous step; most expensive first (one counting-sort launch)
      native.check(native.lib().mjh_order_worlds(ctypes.c_void_p(self.data.solver_niter.data_ptr()),
                                                 ctypes.c_void_p(self.data.nefc.data_ptr()),
                                                 ctypes.c_void_p(self._order.data_ptr()), self.num_envs, self._stream()),
                   "mjh_order_worlds")

  def attach_air_time(self, cols, last_time, cur_air, last_air, cur_con, last_con) -> bool:
    """Fuse a contact sensor's air/contact timers into the physics step: a step
    launched with ``step(air_time=True)`` updates them at its end (mjh_data.at_*,
    the arithmetic of ContactSensor._update_air_time_tracking), replacing the
    timer launch of Scene.update after each decimation substep. cols: the
    sensordata columns of the sensor's `found` slots (at most 7), one per timer
    column. Returns False (nothing attached) for layouts the kernel does not
    take. Plain ``step()`` never touches the timers."""
    ts = (last_time, cur_air, last_air, cur_con, last_con)
    if not self.use_cuda_graph or not (0 < len(cols) <= 7):
      return False
    if not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ts):
      return False
    if last_time.numel() != self.num_envs or any(t.shape != (self.num_envs, len(cols)) for t in ts[1:]):
      return False
    self._air_time = (list(cols), ts)
    self._build_structs()
    return True

  def model_version(self) -> int:
    """Sum of the model buffers' torch version counters: changes whenever a
    model field is written in place through torch (views share their base's
    counter). Host state, read when a launch is issued (or captured)."""
    return sum(t._version for t in self._model_flat.values())

  def _launch_step(self, keep_image: bool = False, air_time: bool = False) -> None:
    self._refresh_order()
    # the packed image is reused only while no model field has been written
    # since the launch that packed it (an action term that writes
    # gains between decimation substeps must not be ignored)
    ver = self.model_version()
    if keep_image and (ver != getattr(self, "_packed_version", None) or os.environ.get("MJH_KEEP_IMAGE") == "0"):
      keep_image = False
    if not keep_image:
      self._packed_version = ver
    fn = native.lib().mjh_step_keep_image if keep_image else native.lib().mjh_step
    ds = self._dstruct_at if (air_time and self._dstruct_at is not None) else self._dstruct
    native.check(fn(ctypes.addressof(self._mstruct), ctypes.addressof(ds), self._stream()), "mjh_step")

  def _launch_forward(self) -> None:
    self._refresh_order()
    self._packed_version = self.model_version()
    native.check(
      native.lib().mjh_forward(ctypes.addressof(self._mstruct), ctypes.addressof(self._dstruct), self._stream()),
      "mjh_forward",
    )

  def _require_gpu(self) -> None:
    if not self.use_cuda_graph:
      raise native.NativeLibraryError(
        f"Simulation on device '{self.device}': the physics step runs only on the HIP path (no CPU fallback)"
      )

  def forward(self) -> None:
    self._require_gpu()
    self.epoch.bump()
    if torch.cuda.is_current_stream_capturing():
      self._launch_forward()
      return
    if self.forward_graph is None:
      self.create_graph()
    self.forward_graph.replay()

  def forward_gated(self, gate: torch.Tensor) -> None:
    """``forward()`` for all worlds iff the device scalar ``gate`` is non-zero.

    The decision is taken on the device, so the env step can call this inside
    a captured graph where the reference syncs on ``len(reset_env_ids) > 0``
    (``manager_based_rl_env.py:133-137``)."""
    self._require_gpu()
    self.epoch.bump()
    if gate.dtype not in (torch.bool, torch.uint8) or gate.numel() != 1 or not gate.is_cuda:
      raise ValueError("gate must be a one-element bool/uint8 device tensor")
    self._refresh_order()
    self._packed_version = self.model_version()
    native.check(
      native.lib().mjh_forward_gated(
        ctypes.addressof(self._mstruct), ctypes.addressof(self._dstruct), ctypes.c_void_p(gate.data_ptr()), self._stream()
      ),
      "mjh_forward_gated",
    )

  def step(self, keep_image: bool = False, air_time: bool = False) -> None:
    """One physics step. Inside an enclosing capture only: keep_image reuses
    the model image packed for the previous launch on this stream (for
    substeps between which no model field changes); air_time also updates the
    attached contact-sensor timers (attach_air_time) at the end of the step."""
    self._require_gpu()
    self.epoch.bump()
    if torch.cuda.is_current_stream_capturing():
      self._launch_step(keep_image, air_time)  # being captured into an enclosing (env-step) graph
      return
    if self.step_graph is None:
      self.create_graph()
    with self.nan_guard.watch(self.data):
      self.step_graph.replay()

  # ---- utilities ----
  def flag_stats(self) -> torch.Tensor:
    """(6,) int64 device tensor: worlds whose physics passes since the last call
    dropped contacts (nconmax) / constraint rows (efc capacity) / went
    non-finite, then the running totals of the same; clears data.flags_acc.
    No host sync (one single-workgroup launch; capturable)."""
    if not hasattr(self, "_flag_stats"):
      self._flag_stats = torch.zeros(6, dtype=torch.int64, device=self.device)
    fa = self.data.flags_acc.view(-1)
    if self.use_cuda_graph:
      native.check(native.lib().mjh_flag_stats(ctypes.c_void_p(fa.data_ptr()), fa.numel(),
                                               ctypes.c_void_p(self._flag_stats.data_ptr()), self._stream()),
                   "mjh_flag_stats")
    else:
      cur = torch.stack([((fa & b) != 0).sum() for b in (1, 2, 4)])
      self._flag_stats[:3] = cur
      self._flag_stats[3:] += cur
      fa.zero_()
    return self._flag_stats

  def debug_fields(self) -> dict[str, torch.Tensor]:
    """Debug copies of the last step/forward's mass matrix ``qM`` (N, nv, nv)
    and constraint Jacobian ``efc_J`` (N, njmax, nv; rows < nefc), MuJoCo's
    d.qM / d.efc_J, for parity tests (mjh_debug_fields)."""
    self._require_gpu()
    nv, nj = self.sizes["nv"], self.sizes["njmax"]
    qM = torch.zeros(self.num_envs, nv, nv, dtype=torch.float32, device=self.device)
    J = torch.zeros(self.num_envs, nj, nv, dtype=torch.float32, device=self.device)
    native.check(native.lib().mjh_debug_fields(ctypes.addressof(self._mstruct), ctypes.addressof(self._dstruct),
                                               ctypes.c_void_p(qM.data_ptr()), ctypes.c_void_p(J.data_ptr()),
                                               self._stream()), "mjh_debug_fields")
    return {"qM": qM, "efc_J": J}

  def efc_capacity(self) -> int:
    return int(native.lib().mjh_efc_capacity(ctypes.addressof(self._mstruct)))

  def lds_row_capacity(self) -> int:
    """Constraint rows a world keeps in LDS; a world with more runs the rest of
    its step with them in global scratch (same results)."""
    return int(native.lib().mjh_lds_rows(ctypes.addressof(self._mstruct)))

  def scratch_bytes(self) -> int:
    return int(native.lib().mjh_scratch_bytes(ctypes.addressof(self._mstruct)))

  def state_dict(self) -> dict[str, torch.Tensor]:
    """Physics state (qpos, qvel, act, ctrl, qacc_warmstart, time) for checkpoint/resume."""
    return {k: self._data_flat[k].clone() for k in ("qpos", "qvel", "act", "ctrl", "qacc_warmstart", "time", "mocap_pos",
                                                      "mocap_quat")}

  def load_state_dict(self, state: dict[str, torch.Tensor]) -> None:
    for k, v in state.items():
      self._data_flat[k].copy_(v)
    self.epoch.bump()


def detect_nans(data) -> torch.Tensor:
  """Per-world bool: non-finite qpos/qvel/qacc/qacc_warmstart (``utils/nan_guard.py:86-104``)."""
  return NanGuard.detect_nans(data)
