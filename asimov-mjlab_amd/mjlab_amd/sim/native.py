"""Loader for the HIP library ``libmjh.so`` (the C ABI in include/mjh_abi.h).

There is no CPU fallback: if the library is missing or was built for another
ABI version, every physics call raises. Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (hipcc, gfx950).
"""

from __future__ import annotations

import collections
import ctypes
from functools import lru_cache
from pathlib import Path

from mjlab_amd.sim import abi

import os

PKG = Path(__file__).resolve().parents[1]
# MJH_LIB selects an alternative build of the same ABI (e.g. the phase-timing
# build libmjh_prof.so used by tools/phase_profile.py).
LIB_PATH = Path(os.environ.get("MJH_LIB", str(PKG / "libmjh.so")))
ABI_VERSION = 17

EXPORTS = (
  "mjh_abi_version",
  "mjh_last_error",
  "mjh_sizeof_model",
  "mjh_sizeof_data",
  "mjh_model_check",
  "mjh_scratch_bytes",
  "mjh_image_words",
  "mjh_set_profile_buffer",
  "mjh_efc_capacity",
  "mjh_lds_rows",
  "mjh_step_keep_image",
  "mjh_plan_ints",
  "mjh_spec_index",
  "mjh_register_spec_plugin",
  "mjh_plugin_index",
  "mjh_data_is_slab",
  "mjh_set_specialization",
  "mjh_set_world_ordering",
  "mjh_set_position_reuse",
  "mjh_split_step",
  "mjh_set_lds_row_cap",
  "mjh_debug_fields",
  "mjh_scratch_words",
  "mjh_step",
  "mjh_forward",
  "mjh_forward_gated",
  "mjh_repeat",
  "mjh_quat_rotate",
  "mjh_quat_mul",
  "mjh_velocity_from_cvel",
  "mjh_air_time_update",
  "mjh_obs_term",
  "mjh_rew_track",
  "mjh_rew_flat_orientation",
  "mjh_rew_sqsum",
  "mjh_rew_diffsq",
  "mjh_rew_pos_limits",
  "mjh_rew_posture",
  "mjh_rew_feet",
  "mjh_velocity_command",
  "mjh_quat_from_euler",
  "mjh_quat_error",
  "mjh_frame_subtract",
  "mjh_motion_relative",
  "mjh_obs_group",
  "mjh_reward_combine",
  "mjh_flag_stats",
  "mjh_masked_means",
  "mjh_masked_counts",
  "mjh_uniform_draws",
  "mjh_uniform_where",
  "mjh_interval_tick",
  "mjh_reset_root_uniform",
  "mjh_reset_joints_offset",
  "mjh_push_velocity",
  "mjh_velocity_resample",
  "mjh_event_mark",
  "mjh_term_combine",
  "mjh_gz_above",
  "mjh_velocity_rows",
  "mjh_masked_zero",
  "mjh_sum_ratios",
  "mjh_rew_air_time",
  "mjh_rew_swing_height",
  "mjh_rew_soft_landing",
  "mjh_joint_action",
  "mjh_root_frame",
  "mjh_order_worlds",
  "mjh_motion_adaptive",
  "mjh_motion_frame",
  "mjh_motion_reset",
  "mjh_rew_exp_err",
  "mjh_step_counters",
  "mjh_reset_stats",
  "mjh_batch_begin",
  "mjh_batch_end",
  "mjh_time_out",
  "mjh_masked_copy",
  "mjh_masked_zero_i64",
)


class NativeLibraryError(RuntimeError):
  pass


@lru_cache(maxsize=1)
def lib() -> ctypes.CDLL:
  if not LIB_PATH.exists():
    raise NativeLibraryError(
      f"{LIB_PATH} not found: the HIP step library is required (no CPU fallback). "
      "Build it with __graft_entry__.build()."
    )
  L = ctypes.CDLL(str(LIB_PATH))
  for name in EXPORTS:
    if not hasattr(L, name):
      raise NativeLibraryError(f"{LIB_PATH} does not export {name}")
  L.mjh_abi_version.restype = ctypes.c_int
  L.mjh_last_error.restype = ctypes.c_char_p
  L.mjh_sizeof_model.restype = ctypes.c_size_t
  L.mjh_sizeof_data.restype = ctypes.c_size_t
  L.mjh_model_check.argtypes = [ctypes.c_void_p]
  L.mjh_scratch_bytes.argtypes = [ctypes.c_void_p]
  L.mjh_efc_capacity.argtypes = [ctypes.c_void_p]
  L.mjh_lds_rows.argtypes = [ctypes.c_void_p]
  L.mjh_plan_ints.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
  L.mjh_spec_index.argtypes = [ctypes.c_void_p]
  L.mjh_register_spec_plugin.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
  L.mjh_plugin_index.argtypes = [ctypes.c_void_p]
  L.mjh_data_is_slab.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
  L.mjh_set_specialization.argtypes = [ctypes.c_int]
  L.mjh_set_world_ordering.argtypes = [ctypes.c_int]
  L.mjh_set_position_reuse.argtypes = [ctypes.c_int]
  L.mjh_set_lds_row_cap.argtypes = [ctypes.c_int]
  L.mjh_debug_fields.argtypes = [ctypes.c_void_p] * 5
  if os.environ.get("MJH_POS_REUSE") == "0":  # A/B timing: the split position pass never skips a world
    L.mjh_set_position_reuse(0)
  # the step launches order the worlds themselves (in the pack launch) unless
  # MJH_PACK_ORDER=0 (A/B: one mjh_order_worlds launch per step from the host)
  L.mjh_set_world_ordering(0 if os.environ.get("MJH_PACK_ORDER") == "0" else 1)
  if os.environ.get("MJH_SPEC") == "0":  # A/B timing: generic kernel instance only
    L.mjh_set_specialization(0)
  L.mjh_image_words.argtypes = [ctypes.c_void_p]
  L.mjh_scratch_words.argtypes = [ctypes.c_void_p]
  L.mjh_scratch_words.restype = ctypes.c_longlong
  L.mjh_set_profile_buffer.argtypes = [ctypes.c_void_p]
  for f in (L.mjh_step, L.mjh_forward, L.mjh_step_keep_image):
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int
  L.mjh_forward_gated.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
  L.mjh_forward_gated.restype = ctypes.c_int
  L.mjh_repeat.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p]
  ll, vp, ci = ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int
  L.mjh_quat_rotate.argtypes = [vp, ll, vp, ll, vp, ll, ci, vp]
  L.mjh_quat_mul.argtypes = [vp, ll, vp, ll, vp, ll, vp]
  L.mjh_velocity_from_cvel.argtypes = [vp, ll, vp, ll, vp, ll, vp, ll, ci, vp]
  L.mjh_air_time_update.argtypes = [vp, ll, vp, ci, vp, vp, vp, vp, vp, vp, ll, vp]
  cf = ctypes.c_float
  L.mjh_obs_term.argtypes = [vp, ll, vp, ll, cf, cf, cf, cf, cf, vp, ll, ci, ll, vp]
  L.mjh_rew_track.argtypes = [vp, ll, vp, ll, cf, ci, vp, ll, vp]
  L.mjh_rew_flat_orientation.argtypes = [vp, ll, vp, ll, cf, vp, ll, vp]
  L.mjh_rew_sqsum.argtypes = [vp, ll, ci, vp, ll, vp]
  L.mjh_rew_diffsq.argtypes = [vp, ll, vp, ll, ci, vp, ll, vp]
  L.mjh_rew_pos_limits.argtypes = [vp, ll, vp, ll, ci, vp, ll, vp]
  L.mjh_rew_posture.argtypes = [vp, ll, vp, ll, vp, vp, vp, vp, ll, cf, cf, ci, vp, ll, vp]
  L.mjh_velocity_command.argtypes = [vp, ll, vp, ll, vp, ll, vp, ll, vp, cf, cf, cf, cf, cf, cf, cf, ci, vp, vp, vp, vp, vp,
                                     vp, vp, vp, vp, ctypes.c_ulonglong, ctypes.c_ulonglong, vp, ll, vp]
  L.mjh_rew_feet.argtypes = [vp, ll, ll, vp, ll, ll, vp, ll, ll, vp, ll, cf, cf, cf, ci, vp, vp, vp, vp, ll, vp]
  L.mjh_quat_from_euler.argtypes = [vp, ll, vp, ll, vp]
  L.mjh_quat_error.argtypes = [vp, ll, vp, ll, vp, ll, vp]
  L.mjh_frame_subtract.argtypes = [vp, ll, vp, ll, vp, ll, ll, vp, ll, ll, ci, vp, vp, ci, ll, vp]
  L.mjh_motion_relative.argtypes = [vp, ll, vp, ll, vp, ll, vp, ll, vp, ll, ll, vp, ll, ll, ci, vp, vp, ll, vp]
  L.mjh_obs_group.argtypes = [vp, ci, vp, ll, vp, ll, ll, ctypes.c_ulonglong, ctypes.c_ulonglong, vp, vp]
  L.mjh_reward_combine.argtypes = [vp, vp, ci, vp, cf, vp, vp, vp, ll, vp]
  L.mjh_flag_stats.argtypes = [vp, ll, vp, vp]
  u64 = ctypes.c_ulonglong
  L.mjh_masked_means.argtypes = [vp, vp, ci, vp, cf, ci, vp, ll, vp]
  L.mjh_masked_counts.argtypes = [vp, ci, vp, vp, ll, vp]
  L.mjh_uniform_draws.argtypes = [vp, ll, u64, u64, vp, vp]
  L.mjh_uniform_where.argtypes = [vp, vp, cf, cf, u64, u64, vp, ll, vp]
  L.mjh_interval_tick.argtypes = [vp, cf, cf, cf, vp, u64, u64, vp, ll, vp]
  L.mjh_reset_root_uniform.argtypes = [vp, ll, ci, vp, ll, ci, vp, vp, ll, vp, ll, vp, vp, vp, vp, ci, ci, u64, u64, vp, ll,
                                       vp]
  L.mjh_reset_joints_offset.argtypes = [vp, ll, ci, vp, ll, ci, ci, vp, vp, ll, vp, ll, vp, ll, cf, cf, cf, cf, ci, ci, u64,
                                        u64, vp, ll, vp]
  L.mjh_push_velocity.argtypes = [vp, ll, ci, vp, ll, ci, vp, vp, ll, vp, vp, u64, u64, vp, ll, vp]
  L.mjh_velocity_resample.argtypes = [vp, vp, cf, cf, cf, cf, ci, ci, vp, vp, vp, vp, vp, vp, u64, u64, vp, ll, vp]
  L.mjh_event_mark.argtypes = [vp, vp, vp, vp, ll, vp]
  L.mjh_term_combine.argtypes = [vp, vp, vp, ci, vp, vp, vp, ll, vp]
  L.mjh_gz_above.argtypes = [vp, ll, ctypes.c_float, vp, ll, vp]
  L.mjh_velocity_rows.argtypes = [vp, ll, ll, vp, ll, vp, ll, vp, vp, ci, ll, vp]
  L.mjh_masked_zero.argtypes = [vp, vp, vp, ci, vp, ll, vp]
  L.mjh_sum_ratios.argtypes = [vp, vp, ci, vp, ll, vp]
  L.mjh_rew_air_time.argtypes = [vp, ll, vp, ll, cf, cf, cf, vp, vp, vp, ci, ll, vp]
  L.mjh_rew_swing_height.argtypes = [vp, vp, ll, ll, vp, ll, ll, vp, ll, vp, ll, cf, cf, cf, vp, vp, vp, ci, ll, vp]
  L.mjh_rew_soft_landing.argtypes = [vp, ll, ll, vp, ll, vp, ll, cf, cf, vp, vp, vp, ci, ll, vp]
  L.mjh_joint_action.argtypes = [vp, ll, vp, vp, vp, vp, vp, ll, cf, vp, ll, cf, ci, ll, vp]
  L.mjh_root_frame.argtypes = [vp, ll, vp, ll, vp, ll, vp, ll, vp, ll, vp, ll, vp, ll, vp]
  L.mjh_order_worlds.argtypes = [vp, vp, vp, ll, vp]
  L.mjh_motion_adaptive.argtypes = [vp, vp, vp, vp, vp, vp, ci, ci, ll, cf, vp, vp, vp, u64, u64, vp, ll, vp]
  L.mjh_step_counters.argtypes = [vp, vp, ll, vp]
  L.mjh_reset_stats.argtypes = [vp, vp, vp, ll, vp]
  L.mjh_batch_begin.argtypes = [ci]
  L.mjh_time_out.argtypes = [vp, ll, vp, ll, vp]
  L.mjh_masked_copy.argtypes = [vp, vp, vp, ll, vp]
  L.mjh_masked_zero_i64.argtypes = [vp, vp, ll, vp]
  L.mjh_batch_end.argtypes = [vp]
  L.mjh_rew_exp_err.argtypes = [vp, ll, ll, vp, vp, ll, ll, vp, ci, ci, ci, cf, vp, ll, vp]
  L.mjh_motion_frame.argtypes = [vp, vp, vp, ci, ci, ci, vp, vp, ll, ll, vp]
  L.mjh_motion_reset.argtypes = [vp, ll, ci, ci, ci, ci, ci, vp, ll, vp, vp, vp, vp, vp, ci, ci, cf, cf, vp, ll, vp, ll, ci, ci,
                                 vp, ll, ci, ci, u64, u64, vp, ll, vp]
  if L.mjh_abi_version() != ABI_VERSION:
    raise NativeLibraryError(f"libmjh ABI {L.mjh_abi_version()} != {ABI_VERSION}")
  if L.mjh_sizeof_model() != ctypes.sizeof(abi.model_struct()):
    raise NativeLibraryError("mjh_model layout mismatch between header parse and library")
  if L.mjh_sizeof_data() != ctypes.sizeof(abi.data_struct()):
    raise NativeLibraryError("mjh_data layout mismatch between header parse and library")
  return L


# launches per C-ABI entry point (host-side tally; tests use it to prove which
# HIP kernels a code path ran)
CALLS: "collections.Counter[str]" = collections.Counter()


def check(rc: int, what: str) -> None:
  CALLS[what] += 1
  if rc != 0:
    msg = lib().mjh_last_error().decode()
    raise RuntimeError(f"{what} failed ({rc}): {msg}")
