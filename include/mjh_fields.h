/* mjh_fields.h — single source of truth for the model/data descriptor layout.
 *
 * Every device buffer the batched step reads or writes is listed here once.
 * C/HIP code expands the lists into struct members (mjh_abi.h); the Python host
 * (mjlab_amd/sim/abi.py) parses these same lines to build matching ctypes
 * structures and to allocate the buffers as torch tensors.
 *
 * Entry forms (COUNT is the per-world element count, written in terms of the
 * size fields):
 *   MS(name)                     int32 size / scalar option (model)
 *   MO(type, name)               scalar option (model)
 *   MA(type, name, COUNT)        model array shared by all worlds
 *   MW(type, name, COUNT)        model array that may be expanded per world:
 *                                pointer + int64 `<name>_wstride` (0 = shared,
 *                                COUNT = one copy per world) — the analogue of
 *                                mjlab's expand_model_fields
 *                                (reference: src/mjlab/sim/randomization.py:20-54,
 *                                field list src/mjlab/envs/mdp/events.py:228-253)
 *   DA(type, name, COUNT)        per-world data array, world-outermost (N, COUNT)
 *
 * Field names follow mjModel/mjData, which is what mjlab indexes
 * (src/mjlab/entity/data.py:75-528, src/mjlab/sim/sim_data.py).
 */

/* ---- sizes ---- */
#define MJH_MODEL_SIZES(MS) \
  MS(nq) MS(nv) MS(nu) MS(na) MS(nbody) MS(njnt) MS(ngeom) MS(nsite)        \
  MS(nsensor) MS(nsensordata) MS(npair) MS(nmocap) MS(nconmax) MS(njmax)     \
  MS(nchain) MS(ncolgeom) MS(nboxpair) MS(sensor_ext_mask)

/* ---- options (mjOption subset used by mjlab's MujocoCfg, sim.py:42-76) ---- */
#define MJH_MODEL_OPTIONS(MO) \
  MO(float, timestep) MO(float, gravity_x) MO(float, gravity_y)             \
  MO(float, gravity_z) MO(float, impratio) MO(float, tolerance)              \
  MO(float, ls_tolerance) MO(int, iterations) MO(int, ls_iterations)         \
  MO(int, integrator) MO(int, cone) MO(int, solver) MO(float, meaninertia)   \
  MO(int, contact_sensor_maxmatch) MO(int, disableflags)                     \
  MO(int, ls_parallel) MO(float, ls_parallel_min_step) MO(float, magnetic_x)  \
  MO(float, magnetic_y) MO(float, magnetic_z)

/* ---- static (shared) model arrays ---- */
#define MJH_MODEL_ARRAYS(MA) \
  MA(int, body_parentid, nbody) MA(int, body_rootid, nbody)                  \
  MA(int, body_weldid, nbody) MA(int, body_jntnum, nbody)                    \
  MA(int, body_jntadr, nbody) MA(int, body_dofnum, nbody)                    \
  MA(int, body_dofadr, nbody) MA(int, body_mocapid, nbody)                   \
  MA(float, body_invweight0, nbody * 2)                                      \
  MA(int, body_chainadr, nbody) MA(int, body_chainnum, nbody)                \
  MA(int, body_chain, nchain)                                                \
  MA(mjh_i64, body_dofmask, nbody) MA(mjh_i64, body_treemask, nbody)     \
  MA(int, jnt_type, njnt) MA(int, jnt_qposadr, njnt) MA(int, jnt_dofadr, njnt) \
  MA(int, jnt_bodyid, njnt) MA(int, jnt_limited, njnt)                       \
  MA(float, jnt_pos, njnt * 3) MA(float, jnt_axis, njnt * 3)                 \
  MA(float, jnt_solref, njnt * 2) MA(float, jnt_solimp, njnt * 5)            \
  MA(float, jnt_margin, njnt) MA(float, qpos_spring, nq)                     \
  MA(int, dof_bodyid, nv) MA(int, dof_jntid, nv) MA(int, dof_parentid, nv)   \
  MA(float, dof_invweight0, nv) MA(float, dof_solref, nv * 2)                \
  MA(float, dof_solimp, nv * 5)                                              \
  MA(int, geom_type, ngeom) MA(int, geom_contype, ngeom)                     \
  MA(int, geom_conaffinity, ngeom) MA(int, geom_condim, ngeom)               \
  MA(int, geom_bodyid, ngeom) MA(int, geom_priority, ngeom)                  \
  MA(float, geom_size, ngeom * 3) MA(float, geom_solmix, ngeom)              \
  MA(float, geom_solref, ngeom * 2) MA(float, geom_solimp, ngeom * 5)        \
  MA(float, geom_margin, ngeom) MA(float, geom_gap, ngeom)                   \
  MA(float, geom_rbound, ngeom) MA(int, geom_colslot, ngeom)                 \
  MA(int, colgeom_id, ncolgeom)                                              \
  MA(int, site_bodyid, nsite)                                                \
  MA(int, actuator_trntype, nu) MA(int, actuator_trnid, nu)                  \
  MA(float, actuator_gear, nu) MA(float, actuator_gainprm, nu * 10)          \
  MA(float, actuator_biasprm, nu * 10) MA(float, actuator_ctrlrange, nu * 2) \
  MA(int, actuator_ctrllimited, nu) MA(float, actuator_forcerange, nu * 2)   \
  MA(int, actuator_forcelimited, nu)                                         \
  MA(int, sensor_type, nsensor) MA(int, sensor_objtype, nsensor)             \
  MA(int, sensor_objid, nsensor) MA(int, sensor_reftype, nsensor)            \
  MA(int, sensor_refid, nsensor) MA(int, sensor_adr, nsensor)                \
  MA(int, sensor_dim, nsensor) MA(int, sensor_intprm, nsensor * 3)           \
  MA(float, sensor_cutoff, nsensor)                                          \
  MA(int, pair_geom1, npair) MA(int, pair_geom2, npair)

/* ---- per-world expandable model arrays (domain randomisation targets) ---- */
#define MJH_MODEL_WARRAYS(MW) \
  MW(float, body_pos, nbody * 3) MW(float, body_quat, nbody * 4)             \
  MW(float, body_ipos, nbody * 3) MW(float, body_iquat, nbody * 4)           \
  MW(float, body_mass, nbody) MW(float, body_inertia, nbody * 3)             \
  MW(float, jnt_range, njnt * 2) MW(float, jnt_stiffness, njnt)              \
  MW(float, dof_armature, nv) MW(float, dof_damping, nv)                     \
  MW(float, dof_frictionloss, nv)                                            \
  MW(float, geom_pos, ngeom * 3) MW(float, geom_quat, ngeom * 4)             \
  MW(float, geom_friction, ngeom * 3) MW(float, geom_rgba, ngeom * 4)        \
  MW(float, site_pos, nsite * 3) MW(float, site_quat, nsite * 4)             \
  MW(float, qpos0, nq)

/* ---- per-world data arrays ---- */
#define MJH_DATA_ARRAYS(DA) \
  DA(float, qpos, nq) DA(float, qvel, nv) DA(float, act, na)                 \
  DA(float, qacc_warmstart, nv) DA(float, ctrl, nu)                          \
  DA(float, qfrc_applied, nv) DA(float, xfrc_applied, nbody * 6)             \
  DA(float, mocap_pos, nmocap * 3) DA(float, mocap_quat, nmocap * 4)         \
  DA(float, time, 1)                                                         \
  DA(float, qacc, nv) DA(float, qacc_smooth, nv)                             \
  DA(float, xpos, nbody * 3) DA(float, xquat, nbody * 4)                     \
  DA(float, xmat, nbody * 9) DA(float, xipos, nbody * 3)                     \
  DA(float, ximat, nbody * 9) DA(float, xanchor, njnt * 3)                   \
  DA(float, xaxis, njnt * 3) DA(float, geom_xpos, ngeom * 3)                 \
  DA(float, geom_xmat, ngeom * 9) DA(float, site_xpos, nsite * 3)            \
  DA(float, site_xmat, nsite * 9) DA(float, subtree_com, nbody * 3)          \
  DA(float, cvel, nbody * 6) DA(float, cacc, nbody * 6)                      \
  DA(float, actuator_force, nu) DA(float, actuator_length, nu)               \
  DA(float, actuator_velocity, nu)                                           \
  DA(float, qfrc_bias, nv) DA(float, qfrc_passive, nv)                       \
  DA(float, qfrc_actuator, nv) DA(float, qfrc_smooth, nv)                    \
  DA(float, qfrc_constraint, nv) DA(float, sensordata, nsensordata)          \
  DA(int, ncon, 1) DA(float, contact_dist, nconmax)                          \
  DA(float, contact_pos, nconmax * 3) DA(float, contact_frame, nconmax * 9)  \
  DA(float, contact_friction, nconmax * 5)                                   \
  DA(float, contact_includemargin, nconmax) DA(int, contact_dim, nconmax)    \
  DA(int, contact_geom, nconmax * 2) DA(int, contact_efc_address, nconmax)   \
  DA(int, nefc, 1) DA(int, efc_type, njmax) DA(int, efc_id, njmax)           \
  DA(float, efc_pos, njmax) DA(float, efc_D, njmax) DA(float, efc_aref, njmax) \
  DA(float, efc_force, njmax) DA(int, solver_niter, 1) DA(int, flags, 1)    \
  DA(int, flags_acc, 1) DA(int, solver_lstrace, 3)
