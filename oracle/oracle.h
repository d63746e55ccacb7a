/* oracle.h — CPU restatement of the batched mj_step (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle and the CPU baseline ("port") for the HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. The product path (mjlab_amd + libmjh.so) never links or calls it.
 *
 * Parity status: the reference's physics lives in third-party MuJoCo Warp
 * (git e605c40, pyproject.toml:108) and MuJoCo C 3.4.0.dev, neither vendored
 * nor installable here. This file restates MuJoCo's published
 * pipeline; it is pinned by analytic known answers (tests/test_oracle_physics.py)
 * and by golden vectors from mjlab's importable torch layers, not by a run of
 * the reference step: physics numerics are "parity unpinned" against MuJoCo.
 *
 * Compiled twice: ORACLE_REAL=double (parity reference) and float.
 */
#ifndef ORACLE_H_
#define ORACLE_H_

#include <stddef.h>

#include "../include/mjh_fields.h"

#ifndef ORACLE_REAL
#define ORACLE_REAL double
#endif
typedef ORACLE_REAL real;
typedef long long mjh_i64;

#define OT_float real
#define OT_int int
#define OT_mjh_i64 mjh_i64

typedef struct or_model {
#define X_SIZE(name) int name;
  MJH_MODEL_SIZES(X_SIZE)
#undef X_SIZE
#define X_OPT(type, name) OT_##type name;
  MJH_MODEL_OPTIONS(X_OPT)
#undef X_OPT
#define X_ARR(type, name, count) const OT_##type* name;
  MJH_MODEL_ARRAYS(X_ARR)
#undef X_ARR
#define X_WARR(type, name, count) const OT_##type* name; long long name##_wstride;
  MJH_MODEL_WARRAYS(X_WARR)
#undef X_WARR
} or_model;

typedef struct or_data {
  int nworld;
  int _pad;
#define X_DATA(type, name, count) OT_##type* name;
  MJH_DATA_ARRAYS(X_DATA)
#undef X_DATA
} or_data;

#ifdef __cplusplus
extern "C" {
#endif
/* Run mj_step (integrate=1) or mj_forward (integrate=0) on worlds [w0, w1),
 * with nthreads OpenMP threads (<=0: library default). Returns 0 on success. */
int oracle_run(const or_model* m, or_data* d, int w0, int w1, int integrate, int nthreads);
/* Debug copies written by the next oracle_run calls (NULL: off): qM as
 * (nworld, nv, nv), efc_J as (nworld, njmax, nv) (rows < nefc written), and
 * lsgap (nworld): the smallest relative cost gap between the best and the
 * runner-up step size over the world's parallel line searches (INFINITY if
 * none ran) — a near-tie a float32 step may decide the other way; lstrace
 * (nworld): 1 if the solver stopped at the iteration cap without meeting its
 * tolerance (the step-size choices are in data.solver_lstrace). */
void oracle_set_debug(real* qM, real* efc_J, real* lsgap, long long* lstrace);
/* Follow mode (parallel line search only): each world replays the device's
 * discrete choices — solver_niter iterations, the step-size index of each from
 * solver_lstrace (inputs then) — instead of its own argmin and stopping test;
 * lsgap then reports the worst relative cost excess of a replayed choice over
 * the float64 argmin (a correct device choice is a near-tie: excess ~ 0). The
 * warm-start choice (bit 30 of solver_lstrace[1]: start from qacc_smooth) is
 * replayed as well. */
void oracle_set_follow(int on);
/* The parallel line search's candidate costs at one solver iteration,
 * (nworld, 64), or with iteration = -1 at every iteration < 15, (nworld, 15, 64)
 * (NULL: off). */
void oracle_set_ls_scan(int on);
/* diagnostics: 0 MuJoCo's Newton/CG stop test (improvement or gradient below
   tolerance), 1 the improvement test only (tools/iteration_analysis.py) */
void oracle_set_stop_mode(int mode);
void oracle_set_lscost(real* cost, int iteration);
size_t oracle_sizeof_model(void);
size_t oracle_sizeof_data(void);
int oracle_real_bytes(void);
#ifdef __cplusplus
}
#endif
#endif
