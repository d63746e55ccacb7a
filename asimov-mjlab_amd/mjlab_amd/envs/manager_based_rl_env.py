"""Manager-based environments (``src/mjlab/envs/manager_based_env.py`` and
``src/mjlab/envs/manager_based_rl_env.py``).

Same construction order, step order and reset semantics as the reference
(``manager_based_rl_env.py:126-176``, ``_reset_idx`` ``:210-245``). What is
different is *how* a step executes on the device:

* resets are boolean masks, never ``nonzero()`` index lists, and the
  "any env reset -> ``sim.forward()``" branch is decided on the device by
  ``mjh_forward_gated`` — so the whole env step (action processing,
  ``decimation`` physics steps, terminations, rewards, masked resets, the gated
  forward, commands, interval events, observations) has no host sync and is
  captured into ONE HIP graph, replayed each call to ``step``;
* host-side schedules (curricula on ``common_step_counter``) run before the
  replay; if they change a value baked into the graph (a reward weight), the
  graph is re-captured. Command ranges live in device tensors and need no
  re-capture.

Returned tensors are the graph's persistent buffers: they are overwritten by
the next ``step`` (clone to keep them), as with any CUDA/HIP graph output.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any

import numpy as np
import torch

from mjlab_amd.utils.capture import GraphSlot

from mjlab_amd.envs.mdp.events import reset_scene_to_default
from mjlab_amd.managers.action_manager import ActionManager
from mjlab_amd.managers.command_manager import CommandManager, NullCommandManager
from mjlab_amd.managers.curriculum_manager import CurriculumManager, NullCurriculumManager
from mjlab_amd.managers.event_manager import EventManager
from mjlab_amd.managers.manager_base import as_mask
from mjlab_amd.managers.manager_term_config import EventTermCfg
from mjlab_amd.managers.observation_manager import ObservationManager
from mjlab_amd.managers.reward_manager import RewardManager
from mjlab_amd.managers.termination_manager import TerminationManager
from mjlab_amd.scene import Scene, SceneCfg
from mjlab_amd.sim.sim import Simulation, SimulationCfg


def _nullctx():
  import contextlib

  return contextlib.nullcontext()


@dataclass
class Box:
  """Shape-only stand-in for ``gym.spaces.Box`` (gymnasium is not a dependency)."""

  shape: tuple[int, ...]
  low: float = -math.inf
  high: float = math.inf


@dataclass(kw_only=True)
class ManagerBasedEnvCfg:
  decimation: int
  scene: SceneCfg
  observations: dict
  actions: dict
  events: dict = field(default_factory=lambda: {"reset_scene_to_default": EventTermCfg(func=reset_scene_to_default, mode="reset")})
  seed: int | None = None
  sim: SimulationCfg = field(default_factory=SimulationCfg)
  viewer: Any = None


@dataclass(kw_only=True)
class ManagerBasedRlEnvCfg(ManagerBasedEnvCfg):
  episode_length_s: float
  rewards: dict
  terminations: dict
  commands: dict | None = None
  curriculum: dict | None = None
  is_finite_horizon: bool = False


class _EnvSeed:
  """``seed`` as the reference's staticmethod on the class (``Env.seed(s)``) and as
  a method on an instance (``env.seed(s)``, which also reseeds the device stream)."""

  def __init__(self, fn):
    self._fn = fn
    self.__doc__ = fn.__doc__

  def __get__(self, obj, objtype=None):
    fn = self._fn
    return lambda seed=-1: fn(obj, seed)


def seed_rng(seed: int) -> None:
  """``src/mjlab/utils/random.py``: seed python/numpy/torch."""
  import random

  random.seed(seed)
  np.random.seed(seed)
  torch.manual_seed(seed)


class ManagerBasedEnv:
  def __init__(self, cfg: ManagerBasedEnvCfg, device: str) -> None:
    self.cfg = cfg
    self._air_sensor = None  # a contact sensor whose timers ride on the physics launch (ManagerBasedRlEnv)
    if cfg.seed is not None:
      cfg.seed = self.seed(cfg.seed)
    self._sim_step_counter = 0
    # device random stream of the fused reset/event/command kernels (envops.rng_args):
    # seed from torch's generator (seeded above), counter = env steps taken
    self._rng_ctr = torch.zeros((), dtype=torch.long, device=device)
    self._reseed_stream()
    self.extras: dict = {"log": {}}
    self.obs_buf: dict = {}
    self.scene = Scene(cfg.scene, device=device)
    self.sim = Simulation(num_envs=self.scene.num_envs, cfg=cfg.sim, model=self.scene.compile(), device=device)
    if "cuda" in str(device) and torch.cuda.is_available():
      torch.cuda.set_device(device)
    self.scene.initialize(self.sim.mj_model, self.sim.model, self.sim.data)
    self.load_managers()

  num_envs = property(lambda self: self.scene.num_envs)
  physics_dt = property(lambda self: self.cfg.sim.mujoco.timestep)
  step_dt = property(lambda self: self.cfg.sim.mujoco.timestep * self.cfg.decimation)
  device = property(lambda self: self.sim.device)

  def load_managers(self) -> None:
    self.event_manager = EventManager(self.cfg.events, self)
    self.sim.expand_model_fields(self.event_manager.domain_randomization_fields)
    self.action_manager = ActionManager(self.cfg.actions, self)
    self.observation_manager = ObservationManager(self.cfg.observations, self)
    if type(self) is ManagerBasedEnv and "startup" in self.event_manager.available_modes:
      self.event_manager.apply(mode="startup")
      self.sim.create_graph()

  @_EnvSeed
  def seed(self, seed: int = -1) -> int:
    """Seed python/numpy/torch (``manager_based_env.py:171-177``, a staticmethod
    there) and, when called on an env, restart the device random stream from that
    seed, so ``reset(seed=s)`` reproduces the fused kernels' draws exactly as it
    reproduces the reference's torch draws. ``ManagerBasedRlEnv.seed(42)`` on the
    class seeds the host generators only, as the reference's static method does."""
    if seed == -1:
      seed = int(np.random.randint(0, 10_000))
    seed_rng(seed)
    if self is not None and hasattr(self, "_rng_ctr"):
      self._reseed_stream()
    return seed

  def _reseed_stream(self) -> None:
    """(seed, call counter, step counter) of the device stream from torch's
    (freshly seeded) generator. The step counter restarts in place (captured
    graphs hold its pointer); captured graphs are dropped because they baked
    the old seed and call keys."""
    self._rng_seed = int(torch.randint(0, 2**62, (1,)).item())
    self.__dict__["_rng_calls"] = 0
    self._reset_epoch = 0
    self._rng_ctr.zero_()
    self._graph = None

  def _begin_rng_phase(self, outside_step: bool) -> None:
    """Call keys restart at every env step (draws differ per step through the
    device step counter), so an eager step and a graph replay of it draw the
    same numbers; calls made outside the step (``reset()``) take a separate
    key range per call so they never repeat a step's draws."""
    if outside_step:
      self._reset_epoch += 1
      self.__dict__["_rng_calls"] = self._reset_epoch << 32
    else:
      self.__dict__["_rng_calls"] = 0

  def reset(self, *, seed: int | None = None, env_ids=None, options=None):
    del options
    if seed is not None:
      self.seed(seed)
    self._begin_rng_phase(outside_step=True)
    self._reset_idx(as_mask(env_ids, self.num_envs, self.device))
    self.scene.write_data_to_sim()
    self.sim.forward()
    self.obs_buf = self.observation_manager.compute(update_history=True)
    return self.obs_buf, self.extras

  def step(self, action: torch.Tensor):
    self._rng_ctr += 1
    self._begin_rng_phase(outside_step=False)
    self.action_manager.process_action(action.to(self.device))
    for _ in range(self.cfg.decimation):
      self._sim_step_counter += 1
      self.action_manager.apply_action()
      self.scene.write_data_to_sim()
      # inside the captured step, the contact-sensor timers ride on the physics
      # launch (Simulation.attach_air_time) instead of a launch per substep
      fused = self._air_sensor is not None and torch.cuda.is_current_stream_capturing()
      self.sim.step(air_time=True) if fused else self.sim.step()
      self.scene.update(dt=self.physics_dt, skip=self._air_sensor if fused else None)
    if "interval" in self.event_manager.available_modes:
      self.event_manager.apply(mode="interval", dt=self.step_dt)
    self.obs_buf = self.observation_manager.compute(update_history=True)
    return self.obs_buf, self.extras

  def close(self) -> None:
    pass

  def _reset_idx(self, mask: torch.Tensor) -> None:
    self.scene.reset(mask)
    if "reset" in self.event_manager.available_modes:
      self.event_manager.apply(mode="reset", env_ids=mask, global_env_step_count=self._sim_step_counter // self.cfg.decimation)
    log = self.extras.setdefault("log", {})
    log.update(self.observation_manager.reset(mask))
    log.update(self.action_manager.reset(mask))
    log.update(self.event_manager.reset(mask))


class ManagerBasedRlEnv(ManagerBasedEnv):
  is_vector_env = True
  _graph = GraphSlot()  # the captured env step (utils/capture.py: capture-safe release)
  metadata = {"render_modes": [None]}

  def __init__(self, cfg: ManagerBasedRlEnvCfg, device: str, render_mode: str | None = None, use_graph: bool | None = None, **kwargs) -> None:
    del kwargs
    self.common_step_counter = 0
    self.episode_length_buf = torch.zeros(cfg.scene.num_envs, device=device, dtype=torch.long)
    self.render_mode = render_mode
    super().__init__(cfg=cfg, device=device)
    n = self.num_envs
    # the managers' persistent output buffers, aliased (graph outputs, no copies)
    self.reset_buf = self.termination_manager._dones_buf
    self.reset_terminated = self.termination_manager._terminated_buf
    self.reset_time_outs = self.termination_manager._truncated_buf
    self.reward_buf = self.reward_manager._reward_buf
    self._any_reset = torch.zeros(1, dtype=torch.bool, device=self.device)
    self._env_step_t = self._rng_ctr  # env steps taken (device), also the random stream's counter
    # device counters [envs reset, env steps that ran the gated forward], accumulated
    # inside the graph (no host sync); read with step_stats()
    self._stats = torch.zeros(2, dtype=torch.long, device=self.device)
    self._action_in = torch.zeros(n, self.action_manager.total_action_dim, device=self.device)
    if use_graph is None:
      # the NaN guard captures and checks the state around every physics step on
      # the host (debug aid), so an enabled guard runs the env step eagerly
      use_graph = str(self.device).startswith("cuda") and torch.cuda.is_available() and not cfg.sim.nan_guard.enabled
    self.use_graph = use_graph
    self._graph: torch.cuda.CUDAGraph | None = None
    self._graph_key = None
    self._graph_out = None
    self._eager_steps = 0
    self._pack_buf: torch.Tensor | None = None
    self.metadata = dict(self.metadata, render_fps=1.0 / self.step_dt)
    # sequential job batches (mjh_batch_begin(1)) for the per-env kernel chains
    # of the termination pass and of the commands + interval events: only when
    # every term in them is one whose fused kernels are batchable, so no torch
    # op in the region reads a batched output before the batch launches
    self._seq_term, self._seq_post = self._sequential_regions() if self.use_graph else (False, False)
    self._seq_reset = self._sequential_reset() if self.use_graph else False
    # one air-time contact sensor may have its timers fused into the physics step
    self._air_sensor = None
    if self.use_graph:
      for sen in getattr(self.scene, "_sensors", {}).values():
        attach = getattr(sen, "attach_air_time_to", None)
        if attach is not None and attach(self.sim):
          self._air_sensor = sen
          break

  def _sequential_regions(self) -> tuple[bool, bool]:
    from mjlab_amd.envs.mdp import events as ev
    from mjlab_amd.envs.mdp import terminations as tm

    # bad_orientation fuses only for a limit in [0, pi] (outside it, its torch acos
    # path would read the root frame recorded in the batch before it launches)
    term_ok = all(c.func is tm.time_out
                  or (c.func is tm.bad_orientation and 0.0 <= float(c.params.get("limit_angle", -1.0)) <= math.pi)
                  for c in self.termination_manager._term_cfgs)
    try:
      from mjlab_amd.tasks.velocity.mdp.velocity_command import UniformVelocityCommand
    except ImportError:  # pragma: no cover
      return term_ok, False
    cmds = [self.command_manager.get_term(n) for n in self.command_manager.active_terms]
    cmd_ok = all(type(t) is UniformVelocityCommand and t.cfg.init_velocity_prob == 0.0 for t in cmds)
    ivals = self.event_manager._mode_term_cfgs.get("interval", [])
    ev_ok = all(c.func is ev.push_by_setting_velocity and not c.is_global_time for c in ivals)
    return term_ok, cmd_ok and ev_ok

  def _sequential_reset(self) -> bool:
    """Whether every reset in _reset_idx is a batchable per-env kernel (or a
    cross-env reduction that reads nothing the batch writes: the episode-log
    means and termination counts), so the masked reset runs as one sequential
    job batch: EntityData.clear_state, the contact-sensor timers, the reset
    events, the action / command / interval-event resets, episode_length."""
    from mjlab_amd.entity.data import EntityData
    from mjlab_amd.envs.mdp import events as ev
    from mjlab_amd.envs.mdp.actions import JointAction
    from mjlab_amd.sensor.builtin_sensor import BuiltinSensor
    from mjlab_amd.sensor.contact_sensor import ContactSensor

    sc = self.scene
    for ent in getattr(sc, "_entities", {}).values():
      d = getattr(ent, "data", None)
      if not isinstance(d, EntityData) or not all(isinstance(d._cols.get(k), slice)
                                                  for k in ("free_joint_v_adr", "xfrc_all", "ctrl_ids")):
        return False
    for sen in getattr(sc, "_sensors", {}).values():
      if not isinstance(sen, ContactSensor) and type(sen).reset is not BuiltinSensor.reset:  # the latter: a no-op
        return False
    om, am, rm, em, tm = (self.observation_manager, self.action_manager, self.reward_manager, self.event_manager,
                          self.termination_manager)
    if (any(getattr(om, "_group_obs_term_history_buffer", {}).values())
        or any(getattr(om, "_group_obs_term_delay_buffer", {}).values()) or getattr(om, "_class_terms", None)):
      return False
    if not all(type(t).reset is JointAction.reset for t in am._terms.values()):
      return False
    # class terms take part only through a reset method (their __call__ runs outside the reset)
    if any(hasattr(c.func, "reset") for c in rm._class_term_cfgs + tm._class_term_cfgs):
      return False
    if any(em._mode_class_term_cfgs.values()):
      return False
    if not all(c.func in (ev.reset_root_state_uniform, ev.reset_joints_by_offset)
               for c in em._mode_term_cfgs.get("reset", [])):
      return False
    if any(c.is_global_time for c in em._mode_term_cfgs.get("interval", [])):
      return False
    try:
      from mjlab_amd.tasks.velocity.mdp.velocity_command import UniformVelocityCommand
    except ImportError:  # pragma: no cover
      return False
    cmds = [self.command_manager.get_term(n) for n in self.command_manager.active_terms]
    return all(type(t) is UniformVelocityCommand and t.cfg.init_velocity_prob == 0.0 for t in cmds)

  def enable_step_pack(self) -> torch.Tensor:
    """Learner-facing outputs packed at the end of every env step, inside the
    captured graph, into one persistent (num_envs, D) float32 buffer
    [obs groups in key order | reward | terminated | truncated]
    (mjlab_amd.distributed.pack_step_outputs): the multi-GPU exchange then
    all-gathers this buffer with no per-step allocation."""

    from mjlab_amd.distributed import packed_width

    if self._pack_buf is None:
      dims = {g: int(np.prod(d)) for g, d in self.observation_manager.group_obs_dim.items()}
      self._pack_buf = torch.empty(self.num_envs, packed_width(dims), device=self.device)
      self._graph = None  # re-capture with the pack at the end of the step
    return self._pack_buf

  @property
  def max_episode_length_s(self) -> float:
    return self.cfg.episode_length_s

  @property
  def max_episode_length(self) -> int:
    return math.ceil(self.max_episode_length_s / self.step_dt)

  def load_managers(self) -> None:
    self.command_manager = CommandManager(self.cfg.commands, self) if self.cfg.commands is not None else NullCommandManager()
    super().load_managers()
    self.termination_manager = TerminationManager(self.cfg.terminations, self)
    self.reward_manager = RewardManager(self.cfg.rewards, self)
    self.curriculum_manager = (
      CurriculumManager(self.cfg.curriculum, self) if self.cfg.curriculum is not None else NullCurriculumManager()
    )
    self._configure_spaces()
    if "startup" in self.event_manager.available_modes:
      self.event_manager.apply(mode="startup")
      self.sim.create_graph()

  def _configure_spaces(self) -> None:
    self.single_observation_space = {}
    for g, dim in self.observation_manager.group_obs_dim.items():
      if self.observation_manager.group_obs_concatenate[g]:
        self.single_observation_space[g] = Box(shape=tuple(dim))
      else:
        names = self.observation_manager.active_terms[g]
        self.single_observation_space[g] = {t: Box(shape=tuple(d)) for t, d in zip(names, dim)}
    self.single_action_space = Box(shape=(sum(self.action_manager.action_term_dim),))
    self.action_space = Box(shape=(self.num_envs, *self.single_action_space.shape))

  # ---- stepping ----
  def step(self, action: torch.Tensor):
    self._host_schedules()
    self._action_in.copy_(action.to(self.device))
    if self.use_graph and self._eager_steps >= 1:
      key = self._capture_key()
      if self._graph is None or key != self._graph_key:
        self._capture(key)
      self._graph.replay()
      self.obs_buf = self._graph_out[0]
      self.extras["log"] = dict(self._graph_out[1])
    else:
      self._step_body()
      self._eager_steps += 1
    self.extras["log"].update(self._curriculum_log)
    self._sim_step_counter += self.cfg.decimation
    self.common_step_counter += 1
    return self.obs_buf, self.reward_buf, self.reset_terminated, self.reset_time_outs, self.extras

  def _host_schedules(self) -> None:
    """Host-side curriculum (``_reset_idx`` runs it first in the reference;
    the velocity curricula depend only on ``common_step_counter``)."""
    self._curriculum_log = {}
    if not isinstance(self.curriculum_manager, NullCurriculumManager):
      self.curriculum_manager.compute(env_ids=None)
      self._curriculum_log = self.curriculum_manager.reset(None)
    self.reward_manager.sync_weights()
    for name in self.command_manager.active_terms:
      t = self.command_manager.get_term(name)
      if hasattr(t, "sync_ranges"):
        t.sync_ranges()

  def _capture_key(self):
    return (self.reward_manager.active_pattern, self.sim.struct_version)

  def _capture(self, key) -> None:
    from mjlab_amd.utils.capture import no_gc

    self._graph = None
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with no_gc(), torch.cuda.graph(g):
      self._step_body()
      out = (self.obs_buf, dict(self.extras["log"]))
    self._graph, self._graph_key, self._graph_out = g, key, out

  def _step_body(self) -> None:
    self._begin_rng_phase(outside_step=False)
    self.action_manager.process_action(self._action_in)
    once = self.action_manager.apply_is_idempotent
    for i in range(self.cfg.decimation):
      if i == 0 or not once:
        self.action_manager.apply_action()
      self.scene.write_data_to_sim()
      # every substep repacks: the pack launch also re-sorts the worlds by the
      # previous substep's cost, which pays more than the launch costs (same-box
      # A/B, profiles/r05f_keep_image_ab.log: 1.597M vs 1.570M env-steps/s with
      # substeps 2-4 reusing the image, mjh_step_keep_image, and its stale order)
      # inside the captured step, the contact-sensor timers ride on the physics
      # launch (Simulation.attach_air_time) instead of a launch per substep
      fused = self._air_sensor is not None and torch.cuda.is_current_stream_capturing()
      self.sim.step(air_time=True) if fused else self.sim.step()
      self.scene.update(dt=self.physics_dt, skip=self._air_sensor if fused else None)
    from mjlab_amd import envops

    # the termination pass: step counters, root frame, time_out, bad_orientation,
    # combine — one per-env chain, one dispatch when batched sequentially
    with envops.JobBatch(self.episode_length_buf, sequential=True) if self._seq_term else _nullctx():
      if self.episode_length_buf.is_cuda:
        envops.step_counters(self.episode_length_buf, self._env_step_t)
      else:
        self.episode_length_buf += 1
        self._env_step_t += 1
      self.termination_manager.compute()  # -> reset_buf / reset_terminated / reset_time_outs
    self.reward_manager.compute(dt=self.step_dt)  # -> reward_buf
    with envops.JobBatch(self.reset_buf, sequential=True) if self._seq_reset else _nullctx():
      self._reset_idx(self.reset_buf)
    self.scene.write_data_to_sim()
    if self.reset_buf.is_cuda:
      from mjlab_amd import envops

      envops.reset_stats(self.reset_buf, self._any_reset, self._stats)
    else:
      torch.any(self.reset_buf, dim=0, keepdim=True, out=self._any_reset)
      self._stats[0] += self.reset_buf.sum()
      self._stats[1:] += self._any_reset
    self.sim.forward_gated(self._any_reset)
    # capacity / NaN statistics of this env step's physics passes (device
    # counters, no sync): worlds that dropped contacts or constraint rows
    fs = self.sim.flag_stats()
    log = self.extras.setdefault("log", {})
    log["Sim/contact_overflow_worlds"] = fs[0]
    log["Sim/efc_overflow_worlds"] = fs[1]
    log["Sim/nonfinite_worlds"] = fs[2]
    # commands and interval events: root frame, velocity command, interval
    # timers, pushes — one per-env chain (sequential batch when every term fuses)
    with envops.JobBatch(self.episode_length_buf, sequential=True) if self._seq_post else _nullctx():
      self.command_manager.compute(dt=self.step_dt)
      if "interval" in self.event_manager.available_modes:
        self.event_manager.apply(mode="interval", dt=self.step_dt)
    self.obs_buf = self.observation_manager.compute(update_history=True)
    if self._pack_buf is not None:
      from mjlab_amd.distributed import pack_step_outputs

      pack_step_outputs(self.obs_buf, self.reward_buf, self.reset_terminated, self.reset_time_outs, out=self._pack_buf)

  def reset(self, *, seed: int | None = None, env_ids=None, options=None):
    del options
    if seed is not None:
      self.seed(seed)
    self._begin_rng_phase(outside_step=True)
    mask = as_mask(env_ids, self.num_envs, self.device)
    self._reset_idx(mask)
    self.scene.write_data_to_sim()
    self.sim.forward()
    self.obs_buf = self.observation_manager.compute(update_history=True)
    self._graph = None  # observation buffers were re-bound
    self._eager_steps = 0
    return self.obs_buf, self.extras

  def _reset_idx(self, mask: torch.Tensor) -> None:
    self.scene.reset(mask)
    if "reset" in self.event_manager.available_modes:
      self.event_manager.apply(mode="reset", env_ids=mask, global_env_step_count=self._env_step_t)
    log = self.extras.setdefault("log", {})
    log.update(self.observation_manager.reset(mask))
    log.update(self.action_manager.reset(mask))
    log.update(self.reward_manager.reset(mask))
    log.update(self.command_manager.reset(mask))
    log.update(self.event_manager.reset(mask))
    log.update(self.termination_manager.reset(mask))
    from mjlab_amd import envops

    if not envops.masked_zero_i64(self.episode_length_buf, mask):
      self.episode_length_buf.masked_fill_(mask, 0)

  def step_stats(self) -> torch.Tensor:
    """Cumulative ``[envs reset, env steps whose gated forward ran]`` (device, long)."""
    return self._stats

  def render(self):
    return None
