/* mjh_abi.h — C ABI of the MI355X batched MuJoCo step (libmjh.so).
 *
 * Drop-in boundary for mjlab's physics backend. The reference binds
 *   mujoco_warp.put_model / put_data   (src/mjlab/sim/sim.py:116-126)
 *   mujoco_warp.step / forward         (src/mjlab/sim/sim.py:138-147,186-199)
 *   warp repeat_array_kernel           (src/mjlab/sim/randomization.py:9-54)
 * through Warp's Python FFI. This library replaces those four entry points with
 * plain C functions on raw device pointers:
 *
 *   - Ownership: the caller (torch) allocates every buffer; the library never
 *     allocates or frees device memory and keeps no global mutable state, so
 *     all launches are capturable into a hipGraph (torch.cuda.CUDAGraph).
 *   - Layout: world-outermost, (nworld, COUNT) contiguous float32/int32 arrays
 *     with the mjData field names listed in mjh_fields.h.
 *   - Stream: every call takes the hipStream_t to launch on (as void*), normally
 *     torch.cuda.current_stream().cuda_stream. No call synchronises the host.
 *   - Errors: functions return 0 on success, nonzero on failure, and
 *     mjh_last_error() returns a thread-local message. Runtime overflow of the
 *     per-world contact/constraint capacity (nconmax/njmax) is reported through
 *     the per-world `flags` array (bit 0: contacts dropped, bit 1: constraint
 *     rows dropped, bit 2: non-finite state), never by a host sync; the
 *     `flags_acc` array ORs them across launches until the caller clears it
 *     (mjh_flag_stats counts and clears it on the device).
 */
#ifndef MJH_ABI_H_
#define MJH_ABI_H_

#include <stddef.h>
#include "mjh_fields.h"

typedef long long mjh_i64;

#ifdef __cplusplus
extern "C" {
#endif

#define MJH_ABI_VERSION 17

/* efc_type codes (mjtConstraint) */
#define MJH_CNSTR_FRICTION_DOF 1
#define MJH_CNSTR_LIMIT_JOINT 3
#define MJH_CNSTR_CONTACT_FRICTIONLESS 5
#define MJH_CNSTR_CONTACT_PYRAMIDAL 6
#define MJH_CNSTR_CONTACT_ELLIPTIC 7

/* flags bits */
#define MJH_FLAG_CONTACT_OVERFLOW 1
#define MJH_FLAG_EFC_OVERFLOW 2
#define MJH_FLAG_NONFINITE 4
/* bounds-check builds only (-DMJH_BOUNDS=1): an array index out of its capacity
   was skipped (never set by release builds) */
#define MJH_FLAG_BOUNDS 8

/* integrator codes (mjtIntegrator) */
#define MJH_INT_EULER 0
#define MJH_INT_IMPLICITFAST 3

/* Model descriptor: sizes, options, device pointers. */
typedef struct mjh_model {
#define MJH_X_SIZE(name) int name;
  MJH_MODEL_SIZES(MJH_X_SIZE)
#undef MJH_X_SIZE
#define MJH_X_OPT(type, name) type name;
  MJH_MODEL_OPTIONS(MJH_X_OPT)
#undef MJH_X_OPT
#define MJH_X_ARR(type, name, count) const type* name;
  MJH_MODEL_ARRAYS(MJH_X_ARR)
#undef MJH_X_ARR
#define MJH_X_WARR(type, name, count) const type* name; long long name##_wstride;
  MJH_MODEL_WARRAYS(MJH_X_WARR)
#undef MJH_X_WARR
  /* caller-allocated device scratch for the packed model image
     (mjh_image_words() 32-bit words, 16-byte aligned) */
  float* image;
  int image_words;
  int _pad_image;
} mjh_model;

/* Data descriptor: one pointer per per-world array, (nworld, COUNT). */
typedef struct mjh_data {
  int nworld;
  int _pad;
#define MJH_X_DATA(type, name, count) type* name;
  MJH_DATA_ARRAYS(MJH_X_DATA)
#undef MJH_X_DATA
  /* caller-allocated device scratch: nworld x scratch_words floats
     (scratch_words >= mjh_scratch_words(m)); the step's per-world
     intermediates that do not live in LDS */
  float* scratch;
  long long scratch_words;
  /* optional permutation of [0, nworld) (NULL = identity): the order in which
     worlds are assigned to waves. Results do not depend on it; sorting worlds
     by expected cost balances the waves of a workgroup (and, with one-world
     workgroups, starts the most expensive worlds first). */
  const long long* world_order;
  /* optional fused contact-sensor timers (NULL at_cur_air = none): at the end
     of every physics step (mjh_step; not forward) world w updates the timers
     of ContactSensor._update_air_time_tracking (contact_sensor.py:327-367) for
     its at_k slots from this step's contact flags sensordata[w, at_cols[j]] > 0
     and time: at_cur_air / at_last_air / at_cur_con / at_last_con (nworld,
     at_k), at_last_time (nworld). Replaces the per-substep timer launch of
     Scene.update in the env's decimation loop. Not part of the launch key
     (position reuse is unaffected). */
  float* at_last_time;
  float* at_cur_air;
  float* at_last_air;
  float* at_cur_con;
  float* at_last_con;
  int at_k;
  int at_cols[7];
  /* optional site-output layout (site_wstride 0: compact, (nworld, nsite)):
     world w's site s goes to element w * site_wstride + site_off + s of
     site_xpos / site_xmat (counted in sites), so the outputs can sit inside a
     wider per-world site array whose first site_off sites are static and
     written once by the caller (a scene's env-origin sites; mjlab's
     terrain_importer.py:95-120 puts one per env on the world body). The
     model then describes only the sites after them. */
  long long site_wstride;
  int site_off;
  int _pad_site;
} mjh_data;

/* Version of this ABI (MJH_ABI_VERSION). */
int mjh_abi_version(void);

/* Thread-local message describing the last failure ("" if none). */
const char* mjh_last_error(void);

/* sizeof the descriptors, so a binding can check its struct layout. */
size_t mjh_sizeof_model(void);
size_t mjh_sizeof_data(void);

/* Host-side validation of a model descriptor against the kernel limits
 * (nv <= 64, nbody <= 64, capacity of per-world scratch). Returns 0 if the
 * model can be stepped. Replaces put_model's checks (sim.py:116). */
int mjh_model_check(const mjh_model* m);

/* Words of device scratch the caller must provide in m->image: the packed
 * model image (rewritten by every launch; staged into LDS by 8-world
 * workgroups, read in place by one-world workgroups) + 4 words of launch
 * bookkeeping. */
int mjh_image_words(const mjh_model* m);

/* LDS bytes per workgroup the step kernel uses for this model. */
int mjh_scratch_bytes(const mjh_model* m);

/* Words of per-world global scratch the caller must provide in d->scratch. */
long long mjh_scratch_words(const mjh_model* m);

/* Constraint rows per world (one-world workgroups: njmax; 8-world workgroups:
 * those that fit their LDS, <= njmax); rows beyond it are dropped and reported
 * through flags bit 1. */
int mjh_efc_capacity(const mjh_model* m);
/* Constraint rows a world keeps in LDS (<= mjh_efc_capacity; a world with more
 * keeps them in global scratch for the rest of its step). */
int mjh_lds_rows(const mjh_model* m);

/* Build-time introspection (tools/gen_spec.py): the launch plan of model m as
 * ints — [nvp, model sizes (MJH_MODEL_SIZES order), per-world layout, model
 * image offsets] — written to out (capacity cap). Returns the count, or -1 if
 * cap is too small. Used to compile model-specialized kernel instances whose
 * layout offsets and sizes are compile-time constants. */
int mjh_plan_ints(const mjh_model* m, int* out, int cap);

/* Index of the compiled model-specialised instance the step/forward launches
 * of model m use (-1: the generic instance). */
int mjh_spec_index(const mjh_model* m);

/* Registers a launch plugin: a model-specialised step instance compiled after
 * this library for one launch plan (plan: mjh_plan_ints of the model, nplan
 * ints; fn: the plugin library's mjh_plugin_step, see below). Step/forward
 * launches of a model whose plan equals it, in the slab data layout, with
 * pyramidal cones and the Newton or CG solver, run the plugin's instance
 * after this library's model-image pack (which also orders the worlds).
 * Replaces MuJoCo Warp's per-model kernel generation (mujoco_warp.put_model +
 * the Warp JIT behind mjlab sim.py:116-147: whatever model is put is compiled
 * for). Returns the plugin's index, or -1 on a null function / wrong length.
 * Plugin libraries (mjh_step.hip built with -DMJH_PLUGIN and a one-plan
 * table, mjlab_amd/sim/jit.py) export:
 *   int mjh_plugin_abi(void);                    MJH_ABI_VERSION it was built at
 *   int mjh_plugin_plan(int* out, int cap);      the plan it was built for
 *   int mjh_plugin_step(int step, const int* plan, const mjh_model*,
 *                       const mjh_data*, const unsigned char* gate,
 *                       void* stream, int reuse, unsigned long long key);
 *       0 on success, 3 if plan is not the plugin's (this library passes the
 *       plan it matched, so the plugin never recomputes it) */
int mjh_register_spec_plugin(void* fn, const int* plan, int nplan);

/* Index of the registered plugin the launches of model m use (-1: none; a
 * built-in specialisation, mjh_spec_index >= 0, takes precedence). */
int mjh_plugin_index(const mjh_model* m);

/* 1 if every data array of d lies in one slab, array f at nworld * (words per
 * world of the arrays before f, MJH_DATA_ARRAYS order) from d->qpos — the
 * layout specialised instances require (otherwise the generic one runs). */
int mjh_data_is_slab(const mjh_model* m, const mjh_data* d);

/* 0: always launch the generic instance (A/B timing, tests); 1: default. */
int mjh_set_specialization(int enable);

/* 1: mjh_step / mjh_forward / mjh_forward_gated rewrite data.world_order (when
 * set) on the device before the step, by the same rule as mjh_order_worlds, in
 * the model-image pack launch (no separate launch); 0 (default): the caller
 * supplies world_order. */
int mjh_set_world_ordering(int on);

/* Builds with the split step (mjh_split_step() == 1: a position launch, then a
 * velocity/solver launch): 1 (default) lets the position launch skip a world
 * whose qpos, mocap poses and model (image and per-world fields) are
 * bit-identical to its previous position pass, whose results are still in the
 * world's scratch (e.g. the first physics step after a forward — the env step's
 * reset-forward, manager_based_rl_env.py:133-137). Results are bit-identical
 * either way. Applies to launches issued after the call (a captured graph keeps
 * the setting it was captured with). A build whose MJH_PRESET keeps part of the
 * position stage in LDS never reuses (the call is accepted and ignored).
 * Returns mjh_split_step(). */
int mjh_set_position_reuse(int on);

/* Test / diagnostic: cap the constraint rows a one-world workgroup keeps in LDS
 * (0, the default: as many as its LDS budget holds). A world with more rows runs
 * the rest of its step with the row arrays in global scratch; the results are
 * the same either way. A cap changes the launch plan, so the generic kernel
 * instance runs. Applies to launches issued after the call. */
int mjh_set_lds_row_cap(int rows);

/* 1 if this build launches the step as two kernels (position, then velocity /
 * solver / integration), 0 for the single fused launch. */
int mjh_split_step(void);

/* Debug copies of the mass matrix and the constraint Jacobian of the last
 * mjh_step / mjh_forward on d (kept in d->scratch): qM as (nworld, nv, nv),
 * efc_J as (nworld, njmax, nv), rows < nefc written. For parity tests
 * (MuJoCo's d.qM / d.efc_J); not part of the step. */
int mjh_debug_fields(const mjh_model* m, const mjh_data* d, float* qM, float* efc_J, void* stream);

/* Diagnostic builds only (-DMJH_PROFILE): per-world phase timestamps. */
int mjh_set_profile_buffer(void* ptr);

/* One physics step (mj_step: forward + implicitfast/Euler integration) for all
 * nworld worlds. Replaces mjwarp.step (sim.py:193-199). */
int mjh_step(const mjh_model* m, const mjh_data* d, void* stream);

/* mjh_step without the model-image pack launch that precedes every other
 * step / forward: the image (and the world order) of the previous launch on
 * this stream are reused. For the env's decimation substeps after the first,
 * between which nothing writes a model field (manager_based_rl_env.py:114-119:
 * actions write ctrl, data). The caller guarantees that; results are then
 * identical to mjh_step's. */
int mjh_step_keep_image(const mjh_model* m, const mjh_data* d, void* stream);

/* Forward dynamics only (no integration, time unchanged). Replaces
 * mjwarp.forward (sim.py:186-191). */
int mjh_forward(const mjh_model* m, const mjh_data* d, void* stream);

/* mjh_forward, executed only if the device byte *gate is non-zero (read by the
 * kernel, so the decision needs no host sync and can sit inside a captured
 * graph). Replaces the host-side `if len(reset_env_ids) > 0: sim.forward()`
 * of manager_based_rl_env.py:133-137. */
int mjh_forward_gated(const mjh_model* m, const mjh_data* d, const unsigned char* gate, void* stream);

/* Tile src[0:nelem] into dst[w*nelem:(w+1)*nelem] for w < nworld.
 * Replaces repeat_array_kernel (randomization.py:9-17). */
int mjh_repeat(float* dst, const float* src, long long nelem, int nworld, void* stream);

/* ---- fused env-layer kernels (mjh_envops.hip) ----
 * Rows are addressed by a row stride in floats (last-dim stride 1); outputs are
 * contiguous. They replace chains of torch ops in mjlab's entity/sensor reads,
 * with the same formulas (isaaclab/utils/math.py, contact_sensor.py:327-367). */

/* out[i] = q[i] (x) v[i] (x) q[i]^-1, or with q^-1 when inverse != 0
 * (quat_apply / quat_apply_inverse). */
int mjh_quat_rotate(const float* q, long long qs, const float* v, long long vs, float* out, long long n, int inverse,
                    void* stream);

/* out[i] = p[i] * q[i] (quat_mul). */
int mjh_quat_mul(const float* p, long long ps, const float* q, long long qs, float* out, long long n, void* stream);

/* out[i] = [cvel_lin - cvel_ang x (com - pos), cvel_ang] (entity/data.py:20-31) for
 * n rows; rows i share com row i / k (k bodies/sites per env). */
int mjh_velocity_from_cvel(const float* pos, long long ps, const float* com, long long cs, const float* cvel, long long vs,
                           float* out, long long n, int k, void* stream);

/* Contact-sensor air/contact timers for k tracked slots whose `found` values
 * sit at sensordata[:, cols[j]] (contact_sensor.py:327-367). */
int mjh_air_time_update(const float* sensordata, long long sds, const int* cols, int k, const float* time,
                        float* last_time, float* cur_air, float* last_air, float* cur_con, float* last_con, long long n,
                        void* stream);

/* One observation term's noise -> clip -> scale, written into its column slice
 * of the group buffer (observation_manager.py:163-176). u: U[0,1) draws (NULL:
 * no noise); clipping is skipped when cmin > cmax. */
int mjh_obs_term(const float* x, long long xs, const float* u, long long us, float lo, float hi, float cmin, float cmax,
                 float scale, float* out, long long os, int w, long long n, void* stream);

/* ---- fused MDP terms (mjh_mdp.hip): one launch per reward term ----
 * Formulas of src/mjlab/tasks/velocity/mdp/rewards.py and envs/mdp/rewards.py. */
int mjh_rew_track(const float* cmd, long long cs, const float* v, long long vs, float inv_std2, int angular, float* out,
                  long long n, void* stream);
int mjh_rew_flat_orientation(const float* q, long long qs, const float* g, long long gs, float inv_std2, float* out,
                             long long n, void* stream);
int mjh_rew_sqsum(const float* x, long long xs, int k, float* out, long long n, void* stream);
int mjh_rew_diffsq(const float* a, long long as, const float* b, long long bs, int k, float* out, long long n, void* stream);
int mjh_rew_pos_limits(const float* q, long long qs, const float* lim, long long ls, int k, float* out, long long n,
                       void* stream);
int mjh_rew_posture(const float* q, long long qs, const float* q0, long long q0s, const float* std_stand,
                    const float* std_walk, const float* std_run, const float* cmd, long long cs, float walk_thr,
                    float run_thr, int k, float* out, long long n, void* stream);
int mjh_rew_feet(const float* z, long long zs, long long zcs, const float* vel, long long vs, long long vcs, const float* found,
                 long long fs,
                 long long fcs, const float* cmd, long long cs, float target, float thr_clear, float thr_slip, int k,
                 float* clearance, float* slip, float* slip_vsum, float* slip_cnt, long long n, void* stream);

/* UniformVelocityCommand.compute for all envs (velocity_command.py:65-101):
 * metrics, timers, masked resampling from u (N, 8) uniform draws (u NULL:
 * draws e*8 + j of the (seed, key, *ctr) device stream), heading control,
 * standing override. Boolean buffers are torch.bool (1 byte). */
int mjh_velocity_command(const float* lin_b, long long ls, const float* ang_b, long long as, const float* root_q,
                         long long qs, const float* u, long long us, const float* ranges, float dt, float inv_max_step,
                         float t_lo, float t_hi, float rel_heading, float rel_standing, float stiffness,
                         int heading_command, float* cmd, float* heading_target, float* heading_error,
                         unsigned char* is_heading, unsigned char* is_standing, float* time_left, long long* counter,
                         float* err_xy, float* err_yaw, unsigned long long seed, unsigned long long key,
                         const mjh_i64* ctr, long long n, void* stream);

/* ---- rotations for resets and motion tracking (mjh_envops.hip) ----
 * Formulas of isaaclab/utils/math.py as restated in mjlab_amd/utils/math.py. */

/* out[i] = quat_from_euler_xyz(rpy[i][0], rpy[i][1], rpy[i][2]) (math.py quat_from_euler_xyz;
 * used by events.py:45-84 reset_root_state_uniform and tracking/mdp/commands.py:332). */
int mjh_quat_from_euler(const float* rpy, long long rs, float* out, long long n, void* stream);

/* out[i] = |axis_angle(q1[i] (x) conj(q2[i]))| (quat_error_magnitude, used by
 * tracking/mdp/rewards.py:33-40 and commands.py:227-242). */
int mjh_quat_error(const float* q1, long long s1, const float* q2, long long s2, float* out, long long n, void* stream);

/* subtract_frame_transforms (math.py) for n = envs x k target rows: frame e = i / k
 * (row stride s*), target j = i % k at e * s + j * r (env stride s, row stride r):
 * t12[i] = quat_apply(q01^-1, t02 - t01), q12[i] = q01^-1 (x) q02; either output may
 * be NULL; qcols > 0 writes the first qcols columns of matrix_from_quat(q12)
 * row-major instead of q12 (tracking/mdp/observations.py:18-69). */
int mjh_frame_subtract(const float* t01, long long st01, const float* q01, long long sq01, const float* t02,
                       long long st02, long long rt02, const float* q02, long long sq02, long long rq02, int k,
                       float* t12, float* q12, int qcols, long long n, void* stream);

/* MotionCommand anchor-relative body targets (tracking/mdp/commands.py:383-405)
 * for n = envs x k body rows (body arrays: env stride s*, row stride r*). */
int mjh_motion_relative(const float* ap, long long sap, const float* aq, long long saq, const float* rp, long long srp,
                        const float* rq, long long srq, const float* bp, long long sbp, long long rbp, const float* bq,
                        long long sbq, long long rbq, int k, float* out_p, float* out_q, long long n, void* stream);

/* ---- manager-level fusion (mjh_mgr.hip) ---- */
#define MJH_MAX_TERMS 32

/* One observation term of a concatenated group: its (n, w) input rows (row
 * stride xs floats) land in columns [off, off + w) of the group buffer after
 * noise (U[0,1) draws u[:, off + j] mapped to [lo, hi), when noise != 0),
 * clipping (skipped when cmin > cmax) and scaling. */
typedef struct mjh_obs_term_desc {
  const float* x;
  long long xs;
  int w;
  int off;
  float lo, hi, cmin, cmax, scale;
  int noise;
  /* the term's value from a strided input: x[e * xs + j * xcs] (xd > 1: rows
     of xd contiguous floats, x[e * xs + (j / xd) * xcs + j % xd]), then op:
     MJH_OBS_COPY, MJH_OBS_SUB (minus y[e * ys + j]), MJH_OBS_POSITIVE (x > 0 as
     0/1), MJH_OBS_SIGNED_LOG1P (sign(x) * log1p(|x|)) */
  const float* y;
  long long ys;
  long long xcs;
  int op;
  int xd;
} mjh_obs_term_desc;

#define MJH_OBS_COPY 0
#define MJH_OBS_SUB 1
#define MJH_OBS_POSITIVE 2
#define MJH_OBS_SIGNED_LOG1P 3

/* ObservationManager.compute for one concatenated group in one launch
 * (observation_manager.py:156-195); terms are read from host memory at call
 * time. Noise draws: u[e * us + col] when u != NULL, else element
 * e * width + col of the (seed, key, *ctr) device stream (mjh_uniform_draws). */
int mjh_obs_group(const mjh_obs_term_desc* terms, int nterms, const float* u, long long us, float* out, long long os,
                  long long n, unsigned long long seed, unsigned long long key, const mjh_i64* ctr, void* stream);

/* RewardManager.compute's combination step (reward_manager.py:76-88) for nterms
 * term vectors values[t] (row stride strides[t]; NULL = weight-0 term, value 0):
 * step_reward[e, t] = v * w[t]; sums[e, t] += v * (w[t] * dt); reward[e] = sum_t. */
int mjh_reward_combine(const float* const* values, const long long* strides, int nterms, const float* weights, float dt,
                       float* reward, float* step_reward, float* sums, long long n, void* stream);

/* One dispatch per reward pass for the per-term kernels (replaces the reward
 * terms' separate launches inside RewardManager.compute, reward_manager.py:
 * 76-88, where every term is an independent per-env function). Between
 * mjh_batch_begin and mjh_batch_end the batchable term entry points
 * (mjh_rew_track, _flat_orientation, _sqsum, _diffsq, _pos_limits, _posture,
 * _feet, _air_time, _swing_height, _soft_landing) record their job instead of
 * launching it; mjh_batch_end launches the recorded jobs, one kernel per source
 * file (blockIdx.y = job), on the stream they were recorded with (or `stream`).
 * The jobs must not read each other's outputs; other launches made while the
 * batch is open run before it. Outputs are bit-identical to the separate
 * launches. Per thread (not shared across host threads).
 * sequential != 0: each env's jobs run in the order they were recorded (one
 * thread per env; consecutive jobs of one source file in one dispatch), for a
 * chain of per-env kernels whose jobs read earlier jobs' outputs of the same
 * env only (the env step's termination pass: mjh_step_counters, mjh_root_frame,
 * mjh_time_out, mjh_gz_above, mjh_term_combine; the commands and interval
 * events: mjh_velocity_command, mjh_interval_tick, mjh_push_velocity; the
 * masked resets: mjh_masked_zero, mjh_masked_copy, mjh_masked_zero_i64,
 * mjh_event_mark, mjh_reset_root_uniform, mjh_reset_joints_offset,
 * mjh_velocity_resample, mjh_uniform_where). */
int mjh_batch_begin(int sequential);
int mjh_batch_end(void* stream);

/* Capacity/NaN statistics from the sticky per-world flags (data->flags_acc),
 * one workgroup, no host sync: stats[0..2] = worlds with contacts dropped /
 * constraint rows dropped / non-finite state since the last call, stats[3..5]
 * += the same (running totals); flags_acc is cleared. */
int mjh_flag_stats(int* flags_acc, long long nworld, mjh_i64* stats, void* stream);


/* ---- reset path, events and commands (mjh_fuse.hip) ----
 * Masks are torch.bool (1 byte per env; NULL = every env). Random draws are
 * U[0,1) from a counter-based generator keyed (seed, key, *ctr, element index):
 * ctr is a device step counter (NULL = 0), so a captured graph draws anew at
 * every replay; mjh_uniform_draws exposes the same stream (tests). */

/* out[t] = scale * sum_{mask} cols[t][e] / max(count(mask), 1); zero_rows != 0
 * also clears the masked entries (RewardManager.reset, reward_manager.py:55-70;
 * CommandTerm.reset metrics, command_manager.py:34-47). One workgroup. */
int mjh_masked_means(float* const* cols, const long long* strides, int ncols, const unsigned char* mask, float scale,
                     int zero_rows, float* out, long long n, void* stream);

/* out[t] = count(flags[t] & mask) (TerminationManager.reset episode logs,
 * termination_manager.py:84-96). One workgroup. */
int mjh_masked_counts(const unsigned char* const* flags, int nflags, const unsigned char* mask, mjh_i64* out, long long n,
                      void* stream);

/* out[i] = U[0,1) element i of the (seed, key, *ctr) stream. */
int mjh_uniform_draws(float* out, long long n, unsigned long long seed, unsigned long long key, const mjh_i64* ctr,
                      void* stream);

/* t[e] = U[lo, hi) (element e) where mask[e] (command / interval-event timers,
 * command_manager.py:40-47, event_manager.py:95-108). */
int mjh_uniform_where(float* t, const unsigned char* mask, float lo, float hi, unsigned long long seed,
                      unsigned long long key, const mjh_i64* ctr, long long n, void* stream);

/* Interval-event timers (event_manager.py:120-145): t -= dt; due = t < 1e-6;
 * due timers redrawn from U[lo, hi) (element e); due written as bool. */
int mjh_interval_tick(float* t, float dt, float lo, float hi, unsigned char* due, unsigned long long seed,
                      unsigned long long key, const mjh_i64* ctr, long long n, void* stream);

/* reset_root_state_uniform (envs/mdp/events.py:45-84) with EntityData's root
 * pose / velocity writes (entity/data.py:112-151) for the masked envs: pose
 * offsets U[pose_lo, pose_hi) (elements e*12 + 0..5, if pose_rand), velocity
 * offsets U[vel_lo, vel_hi) (e*12 + 6..11, if vel_rand); root_state rows are
 * [pos 3, quat 4, lin vel 3, ang vel 3] (world frame); qpos[qadr..+7] = pos +
 * offset + origin, quat (x) euler(offset); qvel[vadr..+6] = [lin, ang in the new
 * body frame]. */
int mjh_reset_root_uniform(float* qpos, long long qs, int qadr, float* qvel, long long vs, int vadr,
                           const unsigned char* mask, const float* root_state, long long rss, const float* origins,
                           long long os, const float* pose_lo, const float* pose_hi, const float* vel_lo,
                           const float* vel_hi, int pose_rand, int vel_rand, unsigned long long seed,
                           unsigned long long key, const mjh_i64* ctr, long long n, void* stream);

/* reset_joints_by_offset (envs/mdp/events.py:87-121) for k consecutive joints
 * (qpos columns qadr.., qvel columns vadr..): default + U[pos_lo, pos_hi)
 * (elements e*2k + j) clamped to lim (N, k, 2), default velocity + U[vel_lo,
 * vel_hi) (e*2k + k + j), written for the masked envs. */
int mjh_reset_joints_offset(float* qpos, long long qs, int qadr, float* qvel, long long vs, int vadr, int k,
                            const unsigned char* mask, const float* def_pos, long long dps, const float* def_vel,
                            long long dvs, const float* lim, long long ls, float pos_lo, float pos_hi, float vel_lo,
                            float vel_hi, int pos_rand, int vel_rand, unsigned long long seed, unsigned long long key,
                            const mjh_i64* ctr, long long n, void* stream);

/* push_by_setting_velocity (envs/mdp/events.py:124-137): vel_w + U[lo, hi)
 * (elements e*6 + j) written as the free joint's qvel for the masked envs. */
int mjh_push_velocity(const float* qpos, long long qs, int qadr, float* qvel, long long vs, int vadr,
                      const unsigned char* mask, const float* vel_w, long long vws, const float* lo, const float* hi,
                      unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n, void* stream);

/* UniformVelocityCommand resampling of the masked envs (command_manager.py:40-47,
 * velocity_command.py:103-123): timer U[t_lo, t_hi) (element e*8), command
 * over ranges (4 x [lo, hi]: lin_x, lin_y, ang_z, heading) from e*8 + 1..4,
 * heading env (e*8 + 5 <= rel_heading), standing env (e*8 + 6 <= rel_standing);
 * the counter restarts at 1 when reset != 0, else increments. */
int mjh_velocity_resample(const unsigned char* mask, const float* ranges, float t_lo, float t_hi, float rel_heading,
                          float rel_standing, int heading_command, int reset, float* cmd, float* heading_target,
                          unsigned char* is_heading, unsigned char* is_standing, float* time_left, mjh_i64* counter,
                          unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n,
                          void* stream);

/* TerminationManager.compute's combination (termination_manager.py:54-82) for
 * nterms bool term vectors: term_dones[t] = values[t]; truncated = OR of the
 * time-out terms, terminated = OR of the others, dones = truncated | terminated. */
/* out[e] = -cos(limit) < g[e * gs] <= 1 (thr = -cos(limit)): bad_orientation
 * (envs/mdp/terminations.py, torch.acos(-g_z).abs() > limit_angle) on the
 * projected gravity's z column, one launch. */
/* time_out (envs/mdp/terminations.py): out[e] = episode_length[e] >= max_len
 * (batchable). */
int mjh_time_out(const mjh_i64* episode_length, long long max_len, unsigned char* out, long long n, void* stream);

int mjh_gz_above(const float* g, long long gs, float thr, unsigned char* out, long long n, void* stream);

int mjh_term_combine(const unsigned char* const* values, unsigned char* const* term_dones, const int* time_out, int nterms,
                     unsigned char* truncated, unsigned char* terminated, unsigned char* dones, long long n,
                     void* stream);

/* compute_velocity_from_cvel for k rows per env read in place (EntityData
 * body/site/geom velocities, entity/data.py:200-260): row j of env e at pos +
 * e*pes + j*prs, its body's cvel at cvel + e*ves + 6*body[j], root subtree com
 * at com + e*cs; out (n*k, 6) = [lin - ang x (com - pos), ang]. */
int mjh_velocity_rows(const float* pos, long long pes, long long prs, const float* com, long long cs, const float* cvel,
                      long long ves, const int* body, float* out, int k, long long n, void* stream);

/* Zero the masked rows of ntensors float tensors (row t: widths[t] floats at
 * ptrs[t] + e * row_strides[t]) in one launch (managers' masked_fill_ chains). */
int mjh_masked_zero(float* const* ptrs, const long long* row_strides, const int* widths, int ntensors,
                    const unsigned char* mask, long long n, void* stream);

/* Masked per-env copies for the reset path (batchable): dst[e] = src[e] where
 * mask[e] (ContactSensor.reset's last_time, contact_sensor.py:210-216), and
 * dst64[e] = 0 where mask[e] (episode_length_buf.masked_fill_,
 * manager_based_rl_env.py:245). */
int mjh_masked_copy(float* dst, const float* src, const unsigned char* mask, long long n, void* stream);
int mjh_masked_zero_i64(mjh_i64* dst, const unsigned char* mask, long long n, void* stream);

/* out[t] = sum(num[t]) / max(sum(den[t]), 1) over n envs (reward-term metric
 * logs, tasks/velocity/mdp/rewards.py); den[t] NULL: mean(sqrt(num[t]))
 * (Metrics/angular_momentum_mean). One workgroup per term. */
int mjh_sum_ratios(const float* const* num, const float* const* den, int nterms, float* out, long long n, void* stream);

/* Contact-timing rewards of the velocity task (tasks/velocity/mdp/rewards.py),
 * one launch each, per env over its k feet; cmd NULL = no command gating, else
 * x (|cmd_xy| + |cmd_yaw| > cmd_thr). num/den receive the per-env parts of the
 * term's metric log (sum(num) / max(sum(den), 1), see mjh_sum_ratios).
 * Strides: *es per env, *cs / *ss per foot. first contact: 0 < contact time < first_lim. */
int mjh_rew_air_time(const float* t, long long ts, const float* cmd, long long cs, float tmin, float tmax, float cmd_thr,
                     float* out, float* num, float* den, int k, long long n, void* stream);
int mjh_rew_swing_height(float* peak, const float* h, long long hes, long long hcs, const float* found, long long fes,
                         long long fcs, const float* cct, long long cts, const float* cmd, long long cs, float first_lim,
                         float target, float cmd_thr, float* out, float* num, float* den, int k, long long n,
                         void* stream);
int mjh_rew_soft_landing(const float* f, long long fes, long long fss, const float* cct, long long cts, const float* cmd,
                         long long cs, float first_lim, float cmd_thr, float* out, float* num, float* den, int k,
                         long long n, void* stream);

/* ActionManager.process_action with one JointAction term (action_manager.py:
 * 107-116, joint_actions.py:90-108), contiguous (n, d) buffers: prev = action;
 * action = raw = input; processed = raw * scale + offset, scale / offset from
 * rows (stride ss / os) or the scalars scale0 / offset0 when NULL. */
int mjh_joint_action(const float* input, long long is, float* action, float* prev, float* raw, float* processed,
                     const float* scale, long long ss, float scale0, const float* offset, long long os, float offset0,
                     int d, long long n, void* stream);

/* The root body's EntityData frame reads from one forward pass, out (n, 16) =
 * [root_link_vel_w 6 | root_link_lin_vel_b 3 | root_link_ang_vel_b 3 |
 * projected_gravity_b 3 | heading_w 1] (entity/data.py; quat_apply(_inverse),
 * compute_velocity_from_cvel of utils/math.py / data.py). Row strides *s. */
int mjh_root_frame(const float* xpos, long long ps, const float* xquat, long long qs, const float* com, long long cs,
                   const float* cvel, long long vs, const float* grav, long long gs, const float* fwd, long long fs,
                   float* out, long long n, void* stream);

/* A permutation of the worlds for mjh_data.world_order: most expensive first by
 * the previous step's (solver_niter + 2) * nefc (counting sort in 256 buckets,
 * one workgroup), so the worlds sharing a workgroup take similar time. */
int mjh_order_worlds(const int* solver_niter, const int* nefc, long long* order, long long n, void* stream);

/* ---- motion tracking command (tasks/tracking/mdp/commands.py), mjh_fuse.hip ---- */

/* MotionCommand._adaptive_sampling (commands.py:258-307) for the masked envs in
 * one workgroup: failed-bin histogram into cur_failed (when some masked env
 * terminated), p = smooth(bin_failed + ratio / nbins, kern[ksize]) / sum,
 * time steps by inverse CDF (draws 2e, 2e + 1), metrics when any env resampled.
 * nbins <= 4096. */
int mjh_motion_adaptive(const unsigned char* mask, const unsigned char* terminated, long long* time_steps,
                        const float* bin_failed, float* cur_failed, const float* kern, int nbins, int ksize,
                        long long T, float ratio, float* m_entropy, float* m_top1p, float* m_top1b,
                        unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n, void* stream);

/* MotionCommand._refresh_frame: frame[e] = table[time_steps[e]] (width floats);
 * body_pos_w (n, nb, 3) = the frame's body positions (columns pos_off..) + origins. */
int mjh_motion_frame(const float* table, const long long* time_steps, float* frame, int width, int pos_off, int nb,
                     float* body_pos_w, const float* origins, long long os, long long n, void* stream);

/* MotionCommand._resample_command's robot state write for the masked envs
 * (commands.py:309-375): reference root pose/velocity + U offsets (draws e*S +
 * 0..11), joints + U[jlo, jhi) (e*S + 12 + j) clipped to lim (n, nj, 2), S = 12
 * + nj; written into qpos/qvel (root free joint at root_q/root_v, joints at
 * joint_q/joint_v; angular velocity into the new body frame). */
int mjh_motion_reset(const float* frame, long long fs, int nj, int pos_off, int quat_off, int lin_off, int ang_off,
                     const float* body_pos_w, long long bps, const unsigned char* mask, const float* pose_lo,
                     const float* pose_hi, const float* vel_lo, const float* vel_hi, int pose_any, int vel_any, float jlo,
                     float jhi, const float* lim, long long ls, float* qpos, long long qs, int root_q, int joint_q,
                     float* qvel, long long vs, int root_v, int joint_v, unsigned long long seed,
                     unsigned long long key, const mjh_i64* ctr, long long n, void* stream);

/* Gaussian tracking rewards (tasks/tracking/mdp/rewards.py): out[e] =
 * exp(-mean_j err_j * inv_std2) over k rows; row j of a at a + e*aes + ra[j]*ars
 * (ra NULL: j), likewise b; err_j = sum of squared differences over d columns,
 * or quat_error_magnitude(a_j, b_j)^2 when quat != 0. */
int mjh_rew_exp_err(const float* a, long long aes, long long ars, const int* ra, const float* b, long long bes,
                    long long brs, const int* rb, int k, int d, int quat, float inv_std2, float* out, long long n,
                    void* stream);

/* Env-step bookkeeping (manager_based_rl_env.py:111-152): episode_length[e] +=
 * 1 for all n envs and *step += 1 (step may be NULL). */
int mjh_step_counters(mjh_i64* episode_length, mjh_i64* step, long long n, void* stream);

/* any_reset[0] = any(reset); stats[0] += count(reset); stats[1] += any_reset
 * (the gated forward's decision and the env's device counters). One workgroup. */
int mjh_reset_stats(const unsigned char* reset, unsigned char* any_reset, mjh_i64* stats, long long n, void* stream);

/* EventManager reset bookkeeping (event_manager.py:146-156): last[e] = *step,
 * once[e] = 1 for the masked envs. */
int mjh_event_mark(int* last, unsigned char* once, const unsigned char* mask, const mjh_i64* step, long long n,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MJH_ABI_H_ */
