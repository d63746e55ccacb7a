/* oracle.c — serial CPU restatement of mj_step for the parity oracle.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h). One world at a time, in the order of
 * MuJoCo's published pipeline (mj_step = mj_forward + integration):
 *   kinematics -> com_pos -> crb -> tree LDL^T factor (mj_factorI) -> collision
 *   -> make_constraint -> com_vel -> passive -> rne -> actuation ->
 *   acceleration -> Newton solver -> sensors -> implicitfast/Euler integration.
 * Reference anchors: mjlab's solver/integrator options sim.py:42-76 and
 * velocity_env_cfg.py:53-61; actuator semantics spec_config.py:402-414;
 * contact sensor semantics contact_sensor.py:16-47,472-533.
 * Deliberately written differently from the HIP kernel (tree-sparse LDL^T,
 * level-order recursions, dense serial loops) so that agreement is evidence.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MINVAL 1e-15
#define PI 3.14159265358979323846
#define MINIMP 0.0001
#define MAXIMP 0.9999

#define WF(m, f, w) ((m)->f + (long long)(w) * (m)->f##_wstride)

/* ---------------------------------------------------------------- math */
static void mul_quat(real r[4], const real a[4], const real b[4]) {
  real t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof(t));
}
static real norm3(const real v[3]) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static real dot3(const real a[3], const real b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void cross3(real r[3], const real a[3], const real b[3]) {
  real t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof(t));
}
static void normalize4(real q[4]) {
  real n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  } else {
    for (int i = 0; i < 4; i++) q[i] /= n;
  }
}
static real normalize3(real v[3]) {
  real n = norm3(v);
  if (n < MINVAL) {
    v[0] = 1; v[1] = v[2] = 0;
  } else {
    v[0] /= n; v[1] /= n; v[2] /= n;
  }
  return n;
}
static void quat2mat(real m[9], const real q[4]) {
  real w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
static void mat_vec(real r[3], const real m[9], const real v[3]) {
  real t[3] = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
               m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
  memcpy(r, t, sizeof(t));
}
static void matT_vec(real r[3], const real m[9], const real v[3]) {
  real t[3] = {m[0] * v[0] + m[3] * v[1] + m[6] * v[2], m[1] * v[0] + m[4] * v[1] + m[7] * v[2],
               m[2] * v[0] + m[5] * v[1] + m[8] * v[2]};
  memcpy(r, t, sizeof(t));
}
static void mat_mul(real r[9], const real a[9], const real b[9]) {
  real t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof(t));
}
static void rot_quat(real r[3], const real v[3], const real q[4]) {
  real m[9];
  quat2mat(m, q);
  mat_vec(r, m, v);
}
static void axis_angle(real q[4], const real axis[3], real ang) {
  real s = sin(ang * 0.5);
  q[0] = cos(ang * 0.5); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
/* spatial motion cross product  res = v x m  (v, m: [ang; lin]) */
/* the rotation vector (axis x angle, angle in (-pi, pi]) of a quaternion (MuJoCo mju_quat2Vel, dt = 1) */
static real quat2vel(real r[3], const real q[4]) {
  real ax[3] = {q[1], q[2], q[3]};
  const real s = normalize3(ax);
  real ang = 2 * atan2(s, q[0]);
  if (ang > PI) ang -= 2 * PI;
  for (int k = 0; k < 3; k++) r[k] = ax[k] * ang;
  return ang;
}
/* r such that qa = qb * exp(r) (MuJoCo mju_subQuat) */
static void sub_quat(real r[3], const real qa[4], const real qb[4]) {
  const real qbc[4] = {qb[0], -qb[1], -qb[2], -qb[3]};
  real d[4];
  mul_quat(d, qbc, qa);
  quat2vel(r, d);
}

static void cross_motion(real r[6], const real v[6], const real m[6]) {
  real t[6];
  t[0] = -v[2] * m[1] + v[1] * m[2];
  t[1] = v[2] * m[0] - v[0] * m[2];
  t[2] = -v[1] * m[0] + v[0] * m[1];
  t[3] = -v[2] * m[4] + v[1] * m[5] - v[5] * m[1] + v[4] * m[2];
  t[4] = v[2] * m[3] - v[0] * m[5] + v[5] * m[0] - v[3] * m[2];
  t[5] = -v[1] * m[3] + v[0] * m[4] - v[4] * m[0] + v[3] * m[1];
  memcpy(r, t, sizeof(t));
}
/* spatial force cross product  res = v x* f */
static void cross_force(real r[6], const real v[6], const real f[6]) {
  real t[6];
  t[0] = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  t[1] = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  t[2] = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  t[3] = -v[2] * f[4] + v[1] * f[5];
  t[4] = v[2] * f[3] - v[0] * f[5];
  t[5] = -v[1] * f[3] + v[0] * f[4];
  memcpy(r, t, sizeof(t));
}
/* 10-vector inertia (I about com frame origin, h = m*c, m) times motion */
static void inert_vec(real r[6], const real in[10], const real v[6]) {
  r[0] = in[0] * v[0] + in[3] * v[1] + in[4] * v[2] - in[8] * v[4] + in[7] * v[5];
  r[1] = in[3] * v[0] + in[1] * v[1] + in[5] * v[2] + in[8] * v[3] - in[6] * v[5];
  r[2] = in[4] * v[0] + in[5] * v[1] + in[2] * v[2] - in[7] * v[3] + in[6] * v[4];
  r[3] = in[8] * v[1] - in[7] * v[2] + in[9] * v[3];
  r[4] = in[6] * v[2] - in[8] * v[0] + in[9] * v[4];
  r[5] = in[7] * v[0] - in[6] * v[1] + in[9] * v[5];
}
/* velocity/acceleration of a spatial vector at point p, rotated into frame rot (if given) */
static void transform_motion(real res[6], const real vec[6], const real p[3], const real c[3], const real* rot) {
  real dif[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]}, t[3], out[6];
  cross3(t, dif, vec);
  out[0] = vec[0]; out[1] = vec[1]; out[2] = vec[2];
  out[3] = vec[3] - t[0]; out[4] = vec[4] - t[1]; out[5] = vec[5] - t[2];
  if (rot) {
    matT_vec(res, rot, out);
    matT_vec(res + 3, rot, out + 3);
  } else {
    memcpy(res, out, sizeof(out));
  }
}

/* a spatial force [torque; force] about c moved to point p (torque - (p - c) x force),
   optionally rotated into the frame rot (mju_transformSpatial, flg_force 1) */
static void transform_force(real res[6], const real vec[6], const real p[3], const real c[3], const real* rot) {
  real dif[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]}, t[3], out[6];
  cross3(t, dif, vec + 3);
  out[0] = vec[0] - t[0]; out[1] = vec[1] - t[1]; out[2] = vec[2] - t[2];
  out[3] = vec[3]; out[4] = vec[4]; out[5] = vec[5];
  if (rot) {
    matT_vec(res, rot, out);
    matT_vec(res + 3, rot, out + 3);
  } else {
    memcpy(res, out, sizeof(out));
  }
}

/* ---------------------------------------------------------------- workspace */
typedef struct {
  real dist, pos[3], frame[9], friction[5], solref[2], solimp[5], includemargin;
  int dim, geom[2], efc_address;
} contact_t;

static real* g_dbg_lscost;
static int g_dbg_lscost_it;
static real* g_dbg_conv;
static real* g_dbg_warm;
static int g_ls_scan = 0;
static int g_stop_mode = 0;  /* 0: MuJoCo's Newton/CG stop test; 1: improvement test only */
static _Thread_local real g_dbg_scan_cost[64];

typedef struct {
  real *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis, *subtree_com;
  real *cinert, *crb, *cdof, *cdof_dot, *cvel, *cacc, *cfrc;
  real *gxpos, *gxmat, *sxpos, *sxmat;
  real *M, *LD, *H, *qvel, *qpos, *qacc, *qacc_smooth, *qfrc_smooth, *qfrc_bias, *qfrc_passive,
      *qfrc_actuator, *qfrc_constraint, *act_force, *act_length, *act_vel, *tmpv, *tmpv2, *grad, *search,
      *Ma, *Mv, *Mgrad, *qacc_int, *cg_g, *cg_mg;
  real *J, *efc_pos, *efc_margin, *efc_D, *efc_R, *efc_aref, *efc_fl, *jaref, *jv, *efc_force, *jtmp;
  int *efc_type, *efc_id;
  int nefc, ncon, flags, niter;
  real lsgap; /* parallel line search: smallest relative cost gap best vs runner-up */
  unsigned lstrace[3];        /* solver_lstrace: step-size index (6 bits) of iterations 5w..5w+4 in word w */
  int capped;                 /* the solver stopped at the iteration cap, unconverged */
  int conv;                   /* the last iteration passed the convergence test */
  int follow, fniter;         /* follow mode: replay fniter iterations with the given choices */
  int warm_smooth;            /* the solve started from qacc_smooth (not qacc_warmstart) */
  int wi;
  unsigned ftrace[3];
  real lsexcess;              /* follow mode: worst relative cost excess of a given choice */
  contact_t* con;
} ws_t;

static void* xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

static void ws_alloc(ws_t* w, const or_model* m) {
  int nb = m->nbody, nv = m->nv, nj = m->njnt;
  memset(w, 0, sizeof(*w));
#define AR(p, n) w->p = (real*)xcalloc((size_t)(n), sizeof(real))
  AR(xpos, 3 * nb); AR(xquat, 4 * nb); AR(xmat, 9 * nb); AR(xipos, 3 * nb); AR(ximat, 9 * nb);
  AR(xanchor, 3 * nj); AR(xaxis, 3 * nj); AR(subtree_com, 3 * nb); AR(cinert, 10 * nb); AR(crb, 10 * nb);
  AR(cdof, 6 * nv); AR(cdof_dot, 6 * nv); AR(cvel, 6 * nb); AR(cacc, 6 * nb); AR(cfrc, 6 * nb);
  AR(gxpos, 3 * m->ngeom); AR(gxmat, 9 * m->ngeom); AR(sxpos, 3 * m->nsite); AR(sxmat, 9 * m->nsite);
  AR(M, nv * nv); AR(LD, nv * nv); AR(H, nv * nv); AR(qvel, nv); AR(qpos, m->nq); AR(qacc, nv);
  AR(qacc_smooth, nv); AR(qfrc_smooth, nv); AR(qfrc_bias, nv); AR(qfrc_passive, nv); AR(qfrc_actuator, nv);
  AR(qfrc_constraint, nv); AR(act_force, m->nu); AR(act_length, m->nu); AR(act_vel, m->nu);
  AR(tmpv, nv); AR(tmpv2, nv); AR(grad, nv); AR(search, nv); AR(Ma, nv); AR(Mv, nv); AR(Mgrad, nv);
  AR(qacc_int, nv); AR(cg_g, nv); AR(cg_mg, nv);
  AR(J, (size_t)m->njmax * nv); AR(efc_pos, m->njmax); AR(efc_margin, m->njmax); AR(efc_D, m->njmax);
  AR(efc_R, m->njmax); AR(efc_aref, m->njmax); AR(efc_fl, m->njmax); AR(jaref, m->njmax); AR(jv, m->njmax);
  AR(efc_force, m->njmax); AR(jtmp, m->njmax);
#undef AR
  w->efc_type = (int*)xcalloc(m->njmax, sizeof(int));
  w->efc_id = (int*)xcalloc(m->njmax, sizeof(int));
  w->con = (contact_t*)xcalloc(m->nconmax, sizeof(contact_t));
}

static void ws_free(ws_t* w) {
  real** ptrs[] = {&w->xpos, &w->xquat, &w->xmat, &w->xipos, &w->ximat, &w->xanchor, &w->xaxis, &w->subtree_com,
                   &w->cinert, &w->crb, &w->cdof, &w->cdof_dot, &w->cvel, &w->cacc, &w->cfrc, &w->gxpos, &w->gxmat,
                   &w->sxpos, &w->sxmat, &w->M, &w->LD, &w->H, &w->qvel, &w->qpos, &w->qacc, &w->qacc_smooth,
                   &w->qfrc_smooth, &w->qfrc_bias, &w->qfrc_passive, &w->qfrc_actuator, &w->qfrc_constraint,
                   &w->act_force, &w->act_length, &w->act_vel, &w->tmpv, &w->tmpv2, &w->grad, &w->search, &w->Ma,
                   &w->Mv, &w->Mgrad, &w->qacc_int, &w->cg_g, &w->cg_mg, &w->J, &w->efc_pos, &w->efc_margin, &w->efc_D, &w->efc_R,
                   &w->efc_aref, &w->efc_fl, &w->jaref, &w->jv, &w->efc_force, &w->jtmp};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); i++) free(*ptrs[i]);
  free(w->efc_type);
  free(w->efc_id);
  free(w->con);
}

/* ---------------------------------------------------------------- smooth dynamics */
static void kinematics(const or_model* m, const or_data* d, int wi, ws_t* w) {
  const real* bpos = WF(m, body_pos, wi);
  const real* bquat = WF(m, body_quat, wi);
  const real* qpos0 = WF(m, qpos0, wi);
  w->xquat[0] = 1;
  quat2mat(w->xmat, w->xquat);
  for (int b = 1; b < m->nbody; b++) {
    int p = m->body_parentid[b];
    real* xp = w->xpos + 3 * b;
    real* xq = w->xquat + 4 * b;
    int ja = m->body_jntadr[b], jn = m->body_jntnum[b];
    const int mid = m->body_mocapid[b];
    if (mid >= 0) { /* mocap body (child of the world): pose from mocap_pos / mocap_quat */
      const real* mp = d->mocap_pos + ((size_t)wi * m->nmocap + mid) * 3;
      const real* mq = d->mocap_quat + ((size_t)wi * m->nmocap + mid) * 4;
      xp[0] = mp[0]; xp[1] = mp[1]; xp[2] = mp[2];
      xq[0] = mq[0]; xq[1] = mq[1]; xq[2] = mq[2]; xq[3] = mq[3];
      normalize4(xq);
      quat2mat(w->xmat + 9 * b, xq);
      continue;
    }
    if (jn == 1 && m->jnt_type[ja] == 0) {
      const real* q = w->qpos + m->jnt_qposadr[ja];
      xp[0] = q[0]; xp[1] = q[1]; xp[2] = q[2];
      xq[0] = q[3]; xq[1] = q[4]; xq[2] = q[5]; xq[3] = q[6];
      normalize4(xq);
      memcpy(w->xanchor + 3 * ja, xp, 3 * sizeof(real));
      quat2mat(w->xmat + 9 * b, xq);
      real* ax = w->xaxis + 3 * ja;
      ax[0] = w->xmat[9 * b + 2]; ax[1] = w->xmat[9 * b + 5]; ax[2] = w->xmat[9 * b + 8];
      continue;
    }
    real t[3];
    mat_vec(t, w->xmat + 9 * p, bpos + 3 * b);
    for (int k = 0; k < 3; k++) xp[k] = w->xpos[3 * p + k] + t[k];
    mul_quat(xq, w->xquat + 4 * p, bquat + 4 * b);
    for (int j = ja; j < ja + jn; j++) {
      real* anc = w->xanchor + 3 * j;
      real* ax = w->xaxis + 3 * j;
      rot_quat(ax, m->jnt_axis + 3 * j, xq);
      rot_quat(anc, m->jnt_pos + 3 * j, xq);
      for (int k = 0; k < 3; k++) anc[k] += xp[k];
      int qa = m->jnt_qposadr[j];
      if (m->jnt_type[j] == 2) { /* slide */
        real d = w->qpos[qa] - qpos0[qa];
        for (int k = 0; k < 3; k++) xp[k] += ax[k] * d;
      } else if (m->jnt_type[j] == 3) { /* hinge */
        real ql[4], v[3];
        axis_angle(ql, m->jnt_axis + 3 * j, w->qpos[qa] - qpos0[qa]);
        mul_quat(xq, xq, ql);
        rot_quat(v, m->jnt_pos + 3 * j, xq);
        for (int k = 0; k < 3; k++) xp[k] = anc[k] - v[k];
      } else if (m->jnt_type[j] == 1) { /* ball: the normalised qpos quaternion, about the anchor */
        real ql[4] = {w->qpos[qa], w->qpos[qa + 1], w->qpos[qa + 2], w->qpos[qa + 3]}, v[3];
        normalize4(ql);
        mul_quat(xq, xq, ql);
        rot_quat(v, m->jnt_pos + 3 * j, xq);
        for (int k = 0; k < 3; k++) xp[k] = anc[k] - v[k];
      }
    }
    normalize4(xq);
    quat2mat(w->xmat + 9 * b, xq);
  }
  /* inertial frames, geoms, sites */
  const real* ipos = WF(m, body_ipos, wi);
  const real* iquat = WF(m, body_iquat, wi);
  for (int b = 0; b < m->nbody; b++) {
    real t[3], im[9];
    mat_vec(t, w->xmat + 9 * b, ipos + 3 * b);
    for (int k = 0; k < 3; k++) w->xipos[3 * b + k] = w->xpos[3 * b + k] + t[k];
    quat2mat(im, iquat + 4 * b);
    mat_mul(w->ximat + 9 * b, w->xmat + 9 * b, im);
  }
  const real* gpos = WF(m, geom_pos, wi);
  const real* gquat = WF(m, geom_quat, wi);
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    real t[3], gm[9];
    mat_vec(t, w->xmat + 9 * b, gpos + 3 * g);
    for (int k = 0; k < 3; k++) w->gxpos[3 * g + k] = w->xpos[3 * b + k] + t[k];
    quat2mat(gm, gquat + 4 * g);
    mat_mul(w->gxmat + 9 * g, w->xmat + 9 * b, gm);
  }
  const real* spos = WF(m, site_pos, wi);
  const real* squat = WF(m, site_quat, wi);
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    real t[3], sm[9];
    mat_vec(t, w->xmat + 9 * b, spos + 3 * s);
    for (int k = 0; k < 3; k++) w->sxpos[3 * s + k] = w->xpos[3 * b + k] + t[k];
    quat2mat(sm, squat + 4 * s);
    mat_mul(w->sxmat + 9 * s, w->xmat + 9 * b, sm);
  }
}

static void com_pos(const or_model* m, int wi, ws_t* w) {
  const real* mass = WF(m, body_mass, wi);
  const real* inertia = WF(m, body_inertia, wi);
  int nb = m->nbody;
  real* msum = w->tmpv;  /* nv may be < nbody; use a local buffer instead */
  real* mb = (real*)calloc((size_t)nb * 4, sizeof(real));
  (void)msum;
  for (int b = 0; b < nb; b++) {
    mb[4 * b + 3] = mass[b];
    for (int k = 0; k < 3; k++) mb[4 * b + k] = mass[b] * w->xipos[3 * b + k];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    for (int k = 0; k < 4; k++) mb[4 * p + k] += mb[4 * b + k];
  }
  for (int b = 0; b < nb; b++) {
    for (int k = 0; k < 3; k++)
      w->subtree_com[3 * b + k] = mb[4 * b + 3] < MINVAL ? w->xipos[3 * b + k] : mb[4 * b + k] / mb[4 * b + 3];
  }
  free(mb);
  /* cinert: inertia about subtree_com[root] in world orientation */
  for (int b = 0; b < nb; b++) {
    real* ci = w->cinert + 10 * b;
    const real* R = w->ximat + 9 * b;
    const real* c = w->subtree_com + 3 * m->body_rootid[b];
    real d[3] = {w->xipos[3 * b] - c[0], w->xipos[3 * b + 1] - c[1], w->xipos[3 * b + 2] - c[2]};
    real I[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        real s = 0;
        for (int k = 0; k < 3; k++) s += R[3 * i + k] * inertia[3 * b + k] * R[3 * j + k];
        I[3 * i + j] = s;
      }
    real mm = mass[b], dd = dot3(d, d);
    ci[0] = I[0] + mm * (dd - d[0] * d[0]);
    ci[1] = I[4] + mm * (dd - d[1] * d[1]);
    ci[2] = I[8] + mm * (dd - d[2] * d[2]);
    ci[3] = I[1] - mm * d[0] * d[1];
    ci[4] = I[2] - mm * d[0] * d[2];
    ci[5] = I[5] - mm * d[1] * d[2];
    ci[6] = mm * d[0]; ci[7] = mm * d[1]; ci[8] = mm * d[2]; ci[9] = mm;
  }
  /* cdof */
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    const real* c = w->subtree_com + 3 * m->body_rootid[b];
    real off[3] = {c[0] - w->xanchor[3 * j], c[1] - w->xanchor[3 * j + 1], c[2] - w->xanchor[3 * j + 2]};
    switch (m->jnt_type[j]) {
      case 0:
        for (int k = 0; k < 3; k++) {
          real* cd = w->cdof + 6 * (da + k);
          memset(cd, 0, 6 * sizeof(real));
          cd[3 + k] = 1;
        }
        for (int k = 0; k < 3; k++) {
          real* cd = w->cdof + 6 * (da + 3 + k);
          real ax[3] = {w->xmat[9 * b + k], w->xmat[9 * b + 3 + k], w->xmat[9 * b + 6 + k]};
          memcpy(cd, ax, 3 * sizeof(real));
          cross3(cd + 3, ax, off);
        }
        break;
      case 1: /* ball: rotations about the body's axes (mj_comPos) */
        for (int k = 0; k < 3; k++) {
          real* cd = w->cdof + 6 * (da + k);
          real ax[3] = {w->xmat[9 * b + k], w->xmat[9 * b + 3 + k], w->xmat[9 * b + 6 + k]};
          memcpy(cd, ax, 3 * sizeof(real));
          cross3(cd + 3, ax, off);
        }
        break;
      case 2: {
        real* cd = w->cdof + 6 * da;
        memset(cd, 0, 3 * sizeof(real));
        memcpy(cd + 3, w->xaxis + 3 * j, 3 * sizeof(real));
        break;
      }
      case 3: {
        real* cd = w->cdof + 6 * da;
        memcpy(cd, w->xaxis + 3 * j, 3 * sizeof(real));
        cross3(cd + 3, w->xaxis + 3 * j, off);
        break;
      }
    }
  }
}

static void crb(const or_model* m, int wi, ws_t* w) {
  int nv = m->nv;
  memcpy(w->crb, w->cinert, sizeof(real) * 10 * m->nbody);
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) w->crb[10 * p + k] += w->crb[10 * b + k];
  }
  memset(w->M, 0, sizeof(real) * nv * nv);
  const real* arm = WF(m, dof_armature, wi);
  for (int i = 0; i < nv; i++) {
    real buf[6];
    inert_vec(buf, w->crb + 10 * m->dof_bodyid[i], w->cdof + 6 * i);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      real s = 0;
      for (int k = 0; k < 6; k++) s += w->cdof[6 * j + k] * buf[k];
      w->M[i * nv + j] = s;
      w->M[j * nv + i] = s;
    }
    w->M[i * nv + i] += arm[i];
  }
}

/* tree LDL^T (mj_factorI): LD holds L (strict lower, tree pattern) and D on the diagonal */
static void factor_tree(const or_model* m, const real* A, real* LD) {
  int nv = m->nv;
  memcpy(LD, A, sizeof(real) * nv * nv);
  for (int k = nv - 1; k >= 0; k--) {
    if (LD[k * nv + k] < MINVAL) LD[k * nv + k] = MINVAL;
    real invD = 1.0 / LD[k * nv + k];
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) {
      real t = LD[k * nv + i];
      for (int j = i; j >= 0; j = m->dof_parentid[j]) LD[i * nv + j] -= t * invD * LD[k * nv + j];
      LD[k * nv + i] = t * invD;
    }
  }
}
static void solve_tree(const or_model* m, const real* LD, real* x) {
  int nv = m->nv;
  for (int k = nv - 1; k >= 0; k--)
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) x[i] -= LD[k * nv + i] * x[k];
  for (int k = 0; k < nv; k++) x[k] /= LD[k * nv + k];
  for (int k = 0; k < nv; k++)
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) x[k] -= LD[k * nv + i] * x[i];
}

static void com_vel(const or_model* m, ws_t* w) {
  memset(w->cvel, 0, 6 * sizeof(real));
  for (int b = 1; b < m->nbody; b++) {
    real cv[6];
    memcpy(cv, w->cvel + 6 * m->body_parentid[b], sizeof(cv));
    for (int j = m->body_jntadr[b]; j < m->body_jntadr[b] + m->body_jntnum[b] && m->body_jntnum[b] > 0; j++) {
      int da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == 0) {
        for (int k = 0; k < 3; k++) {
          memset(w->cdof_dot + 6 * (da + k), 0, 6 * sizeof(real));
          for (int c = 0; c < 6; c++) cv[c] += w->cdof[6 * (da + k) + c] * w->qvel[da + k];
        }
        for (int k = 3; k < 6; k++) cross_motion(w->cdof_dot + 6 * (da + k), cv, w->cdof + 6 * (da + k));
        for (int k = 3; k < 6; k++)
          for (int c = 0; c < 6; c++) cv[c] += w->cdof[6 * (da + k) + c] * w->qvel[da + k];
      } else if (m->jnt_type[j] == 1) { /* ball: all three from the parent's velocity (mj_comVel) */
        for (int k = 0; k < 3; k++) cross_motion(w->cdof_dot + 6 * (da + k), cv, w->cdof + 6 * (da + k));
        for (int k = 0; k < 3; k++)
          for (int c = 0; c < 6; c++) cv[c] += w->cdof[6 * (da + k) + c] * w->qvel[da + k];
      } else {
        cross_motion(w->cdof_dot + 6 * da, cv, w->cdof + 6 * da);
        for (int c = 0; c < 6; c++) cv[c] += w->cdof[6 * da + c] * w->qvel[da];
      }
    }
    memcpy(w->cvel + 6 * b, cv, sizeof(cv));
  }
}

/* RNE: cacc from qacc (NULL: bias only), cfrc_body, returns generalized force in out */
static void rne(const or_model* m, ws_t* w, const real* qacc, real* out) {
  real g[3] = {m->gravity_x, m->gravity_y, m->gravity_z};
  real* cacc = w->cacc;
  memset(cacc, 0, 6 * sizeof(real));
  cacc[3] = -g[0]; cacc[4] = -g[1]; cacc[5] = -g[2];
  for (int b = 1; b < m->nbody; b++) {
    real* a = cacc + 6 * b;
    memcpy(a, cacc + 6 * m->body_parentid[b], 6 * sizeof(real));
    for (int d = m->body_dofadr[b]; d < m->body_dofadr[b] + m->body_dofnum[b] && m->body_dofnum[b] > 0; d++) {
      for (int c = 0; c < 6; c++) {
        a[c] += w->cdof_dot[6 * d + c] * w->qvel[d];
        if (qacc) a[c] += w->cdof[6 * d + c] * qacc[d];
      }
    }
    real f1[6], f2[6], f3[6];
    inert_vec(f1, w->cinert + 10 * b, a);
    inert_vec(f2, w->cinert + 10 * b, w->cvel + 6 * b);
    cross_force(f3, w->cvel + 6 * b, f2);
    for (int c = 0; c < 6; c++) w->cfrc[6 * b + c] = f1[c] + f3[c];
  }
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p > 0)
      for (int c = 0; c < 6; c++) w->cfrc[6 * p + c] += w->cfrc[6 * b + c];
  }
  if (out)
    for (int d = 0; d < m->nv; d++) {
      real s = 0;
      for (int c = 0; c < 6; c++) s += w->cdof[6 * d + c] * w->cfrc[6 * m->dof_bodyid[d] + c];
      out[d] = s;
    }
}

/* translational/rotational jacobian column of dof d at point p for body b (0 if d not in chain) */
static int in_chain(const or_model* m, int b, int d) {
  int db = m->dof_bodyid[d];
  for (int k = b; k > 0; k = m->body_parentid[k])
    if (k == db) return 1;
  return 0;
}
static void jac_col(const or_model* m, ws_t* w, int b, const real p[3], int d, real jp[3], real jr[3]) {
  if (!in_chain(m, b, d)) {
    jp[0] = jp[1] = jp[2] = jr[0] = jr[1] = jr[2] = 0;
    return;
  }
  const real* cd = w->cdof + 6 * d;
  const real* c = w->subtree_com + 3 * m->body_rootid[b];
  real off[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]}, t[3];
  cross3(t, cd, off);
  for (int k = 0; k < 3; k++) {
    jp[k] = cd[3 + k] + t[k];
    jr[k] = cd[k];
  }
}

static void passive_actuation(const or_model* m, int wi, ws_t* w, const real* ctrl, const real* qfrc_applied,
                              const real* xfrc) {
  int nv = m->nv;
  const real* damping = WF(m, dof_damping, wi);
  const real* stiff = WF(m, jnt_stiffness, wi);
  memset(w->qfrc_passive, 0, sizeof(real) * nv);
  for (int j = 0; j < m->njnt; j++) {
    int t = m->jnt_type[j];
    if ((t == 2 || t == 3) && stiff[j] != 0) {
      int qa = m->jnt_qposadr[j];
      w->qfrc_passive[m->jnt_dofadr[j]] -= stiff[j] * (w->qpos[qa] - m->qpos_spring[qa]);
    } else if (t == 1 && stiff[j] != 0) { /* ball: the rotation vector from the spring pose (mju_subQuat) */
      real dif[3];
      sub_quat(dif, w->qpos + m->jnt_qposadr[j], m->qpos_spring + m->jnt_qposadr[j]);
      for (int k = 0; k < 3; k++) w->qfrc_passive[m->jnt_dofadr[j] + k] -= stiff[j] * dif[k];
    }
  }
  for (int d = 0; d < nv; d++) w->qfrc_passive[d] -= damping[d] * w->qvel[d];
  memset(w->qfrc_actuator, 0, sizeof(real) * nv);
  for (int i = 0; i < m->nu; i++) {
    int j = m->actuator_trnid[i];
    real gear = m->actuator_gear[i];
    real len = gear * w->qpos[m->jnt_qposadr[j]];
    real vel = gear * w->qvel[m->jnt_dofadr[j]];
    real c = ctrl[i];
    if (m->actuator_ctrllimited[i]) {
      real lo = m->actuator_ctrlrange[2 * i], hi = m->actuator_ctrlrange[2 * i + 1];
      c = c < lo ? lo : (c > hi ? hi : c);
    }
    const real* gp = m->actuator_gainprm + 10 * i;
    const real* bp = m->actuator_biasprm + 10 * i;
    real f = gp[0] * c + bp[0] + bp[1] * len + bp[2] * vel;
    if (m->actuator_forcelimited[i]) {
      real lo = m->actuator_forcerange[2 * i], hi = m->actuator_forcerange[2 * i + 1];
      f = f < lo ? lo : (f > hi ? hi : f);
    }
    w->act_force[i] = f;
    w->act_length[i] = len;
    w->act_vel[i] = vel;
    w->qfrc_actuator[m->jnt_dofadr[j]] += gear * f;
  }
  /* smooth force */
  for (int d = 0; d < nv; d++)
    w->qfrc_smooth[d] = w->qfrc_passive[d] - w->qfrc_bias[d] + qfrc_applied[d] + w->qfrc_actuator[d];
  /* xfrc_applied at body com */
  for (int b = 1; b < m->nbody; b++) {
    const real* f = xfrc + 6 * b;
    if (!(f[0] || f[1] || f[2] || f[3] || f[4] || f[5])) continue;
    for (int d = 0; d < nv; d++) {
      real jp[3], jr[3];
      jac_col(m, w, b, w->xipos + 3 * b, d, jp, jr);
      w->qfrc_smooth[d] += dot3(jp, f) + dot3(jr, f + 3);
    }
  }
}

/* ---------------------------------------------------------------- collision */
static void make_frame(real f[9]) {
  normalize3(f);
  if (norm3(f + 3) < 0.5) {
    f[3] = f[4] = f[5] = 0;
    if (f[1] < 0.5 && f[1] > -0.5) f[4] = 1; else f[5] = 1;
  }
  real d = dot3(f, f + 3);
  for (int k = 0; k < 3; k++) f[3 + k] -= d * f[k];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

static int raw_sphere_sphere(contact_t* c, real margin, const real p1[3], real r1, const real p2[3], real r2) {
  real dif[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  real cd = norm3(dif);
  if (cd > margin + r1 + r2) return 0;
  real n[3];
  if (cd < MINVAL) { n[0] = 1; n[1] = n[2] = 0; }
  else { n[0] = dif[0] / cd; n[1] = dif[1] / cd; n[2] = dif[2] / cd; }
  c->dist = cd - r1 - r2;
  for (int k = 0; k < 3; k++) {
    c->pos[k] = p1[k] + n[k] * (r1 + 0.5 * c->dist);
    c->frame[k] = n[k];
    c->frame[3 + k] = 0;
  }
  return 1;
}
static int raw_plane_sphere(contact_t* c, real margin, const real pp[3], const real pm[9], const real sp[3], real r) {
  real n[3] = {pm[2], pm[5], pm[8]};
  real dif[3] = {sp[0] - pp[0], sp[1] - pp[1], sp[2] - pp[2]};
  real cd = dot3(dif, n);
  if (cd > margin + r) return 0;
  c->dist = cd - r;
  for (int k = 0; k < 3; k++) {
    c->pos[k] = sp[k] - n[k] * (r + 0.5 * c->dist);
    c->frame[k] = n[k];
    c->frame[3 + k] = 0;
  }
  return 1;
}

/* Near-ties in the box functions' discrete choices (nearest face, separating
   axis, incident face, kept clip points) go to the earlier candidate unless the
   later one wins by BOX_TIE x the boxes' size scale, so a float32 and a float64
   evaluation choose alike (the kernel uses the same rule). */
#define BOX_TIE 1e-5
/* ---- box pairs (sphere-box, capsule-box, box-box). Boxes: centre bp,
   rotation bm (row-major, column k = axis k), half sizes bs. Normals point from
   geom1 to geom2 (pairs are ordered by type, so the box is geom2 except in
   box-box). The kernel (csrc/mjh_step.hip, box_* functions) runs the same
   algorithms in float32. */
static void to_box(const real bp[3], const real bm[9], const real p[3], real out[3]) {
  real d[3] = {p[0] - bp[0], p[1] - bp[1], p[2] - bp[2]};
  for (int k = 0; k < 3; k++) out[k] = bm[k] * d[0] + bm[3 + k] * d[1] + bm[6 + k] * d[2];
}
static void from_box(const real bm[9], const real v[3], real out[3]) {
  for (int k = 0; k < 3; k++) out[k] = bm[3 * k] * v[0] + bm[3 * k + 1] * v[1] + bm[3 * k + 2] * v[2];
}

/* sphere (centre sp, radius r; geom1) - box (geom2): the box point closest to
   the centre; a centre inside the box leaves through its nearest face
   (MuJoCo Warp collision_primitive.sphere_box, restated) */
static int raw_sphere_box(contact_t* c, real margin, const real sp[3], real r, const real bp[3], const real bm[9],
                          const real bs[3]) {
  real lc[3], cl[3], dif[3];
  to_box(bp, bm, sp, lc);
  for (int k = 0; k < 3; k++) {
    cl[k] = lc[k] < -bs[k] ? -bs[k] : (lc[k] > bs[k] ? bs[k] : lc[k]);
    dif[k] = cl[k] - lc[k];
  }
  real dist = norm3(dif);
  if (dist - r > margin) return 0;
  real nl[3] = {0, 0, 0}, pl[3];
  if (dist <= MINVAL) {
    /* inside: the nearest face (ties to the lower axis, the negative face first) */
    real closest = 2 * (bs[0] + bs[1] + bs[2]), tie = BOX_TIE * (bs[0] + bs[1] + bs[2]);
    int kf = 0;
    for (int i = 0; i < 6; i++) {
      real fd = fabs((i & 1 ? 1 : -1) * bs[i >> 1] - lc[i >> 1]);
      if (closest > fd + tie) { closest = fd; kf = i; }
    }
    nl[kf >> 1] = kf & 1 ? -1 : 1; /* from the sphere into the box */
    for (int k = 0; k < 3; k++) pl[k] = lc[k] + nl[k] * (r - closest) * 0.5;
    c->dist = -closest - r;
  } else {
    for (int k = 0; k < 3; k++) nl[k] = dif[k] / dist;
    for (int k = 0; k < 3; k++) pl[k] = 0.5 * (cl[k] + lc[k] + nl[k] * r);
    c->dist = dist - r;
  }
  real pw[3];
  from_box(bm, pl, pw);
  from_box(bm, nl, c->frame);
  for (int k = 0; k < 3; k++) {
    c->pos[k] = bp[k] + pw[k];
    c->frame[3 + k] = 0;
  }
  return 1;
}

/* signed distance of a box-frame point to the box (convex) */
static real box_sdf(const real bs[3], const real q[3]) {
  real o[3], out = 0, in = -1e30;
  for (int k = 0; k < 3; k++) {
    o[k] = fabs(q[k]) - bs[k];
    real e = o[k] > 0 ? o[k] : 0;
    out += e * e;
    if (o[k] > in) in = o[k];
  }
  return out > 0 ? sqrt(out) : in;
}

/* capsule (centre cp, axis ax, half length h, radius r; geom1) - box (geom2):
   both segment ends as spheres when both touch (a capsule lying on a face),
   otherwise one sphere at the segment point nearest the box (the signed
   distance is convex along the segment: golden-section search, 40 steps) */
static int raw_capsule_box(contact_t* out, real margin, const real cp[3], const real ax[3], real h, real r,
                           const real bp[3], const real bm[9], const real bs[3]) {
  real a[3], b[3];
  for (int k = 0; k < 3; k++) { a[k] = cp[k] + ax[k] * h; b[k] = cp[k] - ax[k] * h; }
  contact_t ca, cb;
  int na = raw_sphere_box(&ca, margin, a, r, bp, bm, bs), nb = raw_sphere_box(&cb, margin, b, r, bp, bm, bs);
  if (na && nb) {
    out[0] = ca;
    out[1] = cb;
    for (int i = 0; i < 2; i++) memcpy(out[i].frame + 3, ax, 3 * sizeof(real));
    return 2;
  }
  real la[3], lb[3];
  to_box(bp, bm, a, la);
  to_box(bp, bm, b, lb);
  const real g = 0.6180339887498949;
  real lo = 0, hi = 1, x1 = hi - g * (hi - lo), x2 = lo + g * (hi - lo), q[3];
  for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x1;
  real f1 = box_sdf(bs, q);
  for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x2;
  real f2 = box_sdf(bs, q);
  for (int it = 0; it < 40; it++) {
    if (f1 <= f2) {
      hi = x2; x2 = x1; f2 = f1; x1 = hi - g * (hi - lo);
      for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x1;
      f1 = box_sdf(bs, q);
    } else {
      lo = x1; x1 = x2; f1 = f2; x2 = lo + g * (hi - lo);
      for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x2;
      f2 = box_sdf(bs, q);
    }
  }
  real t = 0.5 * (lo + hi), p[3];
  for (int k = 0; k < 3; k++) p[k] = a[k] + (b[k] - a[k]) * t;
  int n = raw_sphere_box(out, margin, p, r, bp, bm, bs);
  if (n) memcpy(out[0].frame + 3, ax, 3 * sizeof(real));
  return n;
}

/* box (geom1) - box (geom2): separating-axis test over the 15 axes (3 + 3
   face normals, 9 edge-edge cross products; face axes preferred within 5 %);
   a face axis clips the incident face of the other box against the reference
   face's side planes (up to 8 points, the deepest kept and then up to 3 more,
   each farthest from those kept), an edge-edge axis gives the closest points
   of the two support edges */
static int raw_box_box(contact_t* out, real margin, const real pa[3], const real ma[9], const real sa[3],
                       const real pb[3], const real mb[9], const real sb[3]) {
  real A[3][3], B[3][3], d[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = ma[3 * k + i]; B[i][k] = mb[3 * k + i]; }
  real best = 1e30, bn[3] = {0, 0, 0}, tie = BOX_TIE * (sa[0] + sa[1] + sa[2] + sb[0] + sb[1] + sb[2]);
  int bk = -1;
  for (int k = 0; k < 15; k++) {
    real L[3];
    if (k < 3) memcpy(L, A[k], sizeof(L));
    else if (k < 6) memcpy(L, B[k - 3], sizeof(L));
    else cross3(L, A[(k - 6) / 3], B[(k - 6) % 3]);
    real ln = norm3(L);
    if (ln < 1e-6) continue;
    for (int q = 0; q < 3; q++) L[q] /= ln;
    real ra = 0, rb = 0;
    for (int i = 0; i < 3; i++) { ra += sa[i] * fabs(dot3(A[i], L)); rb += sb[i] * fabs(dot3(B[i], L)); }
    real dl = dot3(d, L), ov = ra + rb - fabs(dl);
    if (ov < -margin) return 0;
    real score = k < 6 ? ov : ov * 1.05 + 1e-9; /* prefer face axes */
    if (score < best - tie) {
      best = score;
      bk = k;
      for (int q = 0; q < 3; q++) bn[q] = dl < 0 ? -L[q] : L[q]; /* from A to B */
    }
  }
  if (bk < 0) return 0;
  if (bk < 6) {
    /* reference face: of A (normal bn) or of B (normal -bn); incident box the other */
    int refA = bk < 3;
    const real *rp = refA ? pa : pb, *ip = refA ? pb : pa, *rs = refA ? sa : sb, *is = refA ? sb : sa;
    real (*R)[3] = refA ? A : B, (*I)[3] = refA ? B : A;
    real nr[3];
    for (int q = 0; q < 3; q++) nr[q] = refA ? bn[q] : -bn[q]; /* out of the reference face */
    int ra = refA ? bk : bk - 3;
    /* incident face: the face of the other box most opposed to nr */
    int ia = 0;
    real mx = -1;
    for (int i = 0; i < 3; i++) {
      real v = fabs(dot3(I[i], nr));
      if (v > mx + BOX_TIE) { mx = v; ia = i; }
    }
    real isg = dot3(I[ia], nr) > 0 ? -1 : 1;
    real fc[3];
    for (int q = 0; q < 3; q++) fc[q] = ip[q] + I[ia][q] * is[ia] * isg;
    int u = (ia + 1) % 3, v = (ia + 2) % 3;
    real poly[16][3], tmpp[16][3];
    int np = 4;
    for (int c = 0; c < 4; c++) {
      real su = (c == 0 || c == 3) ? 1 : -1, sv = (c < 2) ? 1 : -1;
      for (int q = 0; q < 3; q++) poly[c][q] = fc[q] + I[u][q] * is[u] * su + I[v][q] * is[v] * sv;
    }
    /* clip against the 4 side planes of the reference face */
    for (int e = 0; e < 4 && np > 0; e++) {
      int axis = e < 2 ? (ra + 1) % 3 : (ra + 2) % 3;
      real sg = (e & 1) ? -1 : 1;
      real off = dot3(R[axis], rp) * sg + rs[axis];
      int nn = 0;
      for (int i = 0; i < np; i++) {
        const real *P = poly[i], *Q = poly[(i + 1) % np];
        real dp = sg * dot3(R[axis], P) - off, dq = sg * dot3(R[axis], Q) - off;
        if (dp <= 0) { memcpy(tmpp[nn++], P, 3 * sizeof(real)); }
        if ((dp <= 0) != (dq <= 0)) {
          real t = dp / (dp - dq);
          for (int q = 0; q < 3; q++) tmpp[nn][q] = P[q] + (Q[q] - P[q]) * t;
          nn++;
        }
      }
      np = nn;
      memcpy(poly, tmpp, sizeof(real) * 3 * nn);
    }
    /* depth below the reference face */
    real rfc = dot3(nr, rp) + rs[ra] * fabs(dot3(R[ra], nr));
    real dep[16];
    int keep[16], nk = 0;
    for (int i = 0; i < np; i++) {
      dep[i] = dot3(nr, poly[i]) - rfc;
      if (dep[i] <= margin) keep[nk++] = i;
    }
    if (nk == 0) return 0;
    int sel[4], ns = 0;
    int di = keep[0];
    for (int j = 1; j < nk; j++) if (dep[keep[j]] < dep[di] - tie) di = keep[j];
    sel[ns++] = di;
    while (ns < 4 && ns < nk) {
      int bj = -1;
      real bd = -1;
      for (int j = 0; j < nk; j++) {
        int i = keep[j], used = 0;
        real md = 1e30;
        for (int s2 = 0; s2 < ns; s2++) {
          if (sel[s2] == i) used = 1;
          real dd[3] = {poly[i][0] - poly[sel[s2]][0], poly[i][1] - poly[sel[s2]][1], poly[i][2] - poly[sel[s2]][2]};
          real dn = norm3(dd);
          if (dn < md) md = dn;
        }
        if (!used && md > bd + tie) { bd = md; bj = i; }
      }
      if (bj < 0) break;
      sel[ns++] = bj;
    }
    for (int i = 0; i < ns; i++) {
      contact_t* c = out + i;
      c->dist = dep[sel[i]];
      for (int q = 0; q < 3; q++) {
        c->pos[q] = poly[sel[i]][q] - nr[q] * 0.5 * c->dist;
        c->frame[q] = bn[q];
        c->frame[3 + q] = 0;
      }
    }
    return ns;
  }
  /* edge-edge: the support edges (along A_i and B_j) */
  int ai = (bk - 6) / 3, bj = (bk - 6) % 3;
  real ca[3], cb[3];
  memcpy(ca, pa, sizeof(ca));
  memcpy(cb, pb, sizeof(cb));
  for (int i = 0; i < 3; i++) {
    if (i != ai) {
      real sg = dot3(A[i], bn) > 0 ? 1 : -1;
      for (int q = 0; q < 3; q++) ca[q] += A[i][q] * sa[i] * sg;
    }
    if (i != bj) {
      real sg = dot3(B[i], bn) > 0 ? -1 : 1;
      for (int q = 0; q < 3; q++) cb[q] += B[i][q] * sb[i] * sg;
    }
  }
  /* closest points of the segments ca + s A_ai (|s| <= sa[ai]), cb + t B_bj */
  real w0[3] = {ca[0] - cb[0], ca[1] - cb[1], ca[2] - cb[2]};
  real aa = dot3(A[ai], A[ai]), ab = dot3(A[ai], B[bj]), bb = dot3(B[bj], B[bj]);
  real da = dot3(A[ai], w0), db = dot3(B[bj], w0), den = aa * bb - ab * ab;
  real s = den > 1e-12 ? (ab * db - bb * da) / den : 0;
  s = s < -sa[ai] ? -sa[ai] : (s > sa[ai] ? sa[ai] : s);
  real t = (ab * s + db) / bb;
  t = t < -sb[bj] ? -sb[bj] : (t > sb[bj] ? sb[bj] : t);
  s = (ab * t - da) / aa;
  s = s < -sa[ai] ? -sa[ai] : (s > sa[ai] ? sa[ai] : s);
  real p1[3], p2[3];
  for (int q = 0; q < 3; q++) { p1[q] = ca[q] + A[ai][q] * s; p2[q] = cb[q] + B[bj][q] * t; }
  real dd[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  real dist = dot3(dd, bn);
  if (dist > margin) return 0;
  out[0].dist = dist;
  for (int q = 0; q < 3; q++) {
    out[0].pos[q] = 0.5 * (p1[q] + p2[q]);
    out[0].frame[q] = bn[q];
    out[0].frame[3 + q] = 0;
  }
  return 1;
}

/* plane (geom1) - cylinder (geom2, radius r, half height h): MuJoCo's
   mjc_PlaneCylinder / MuJoCo Warp collision_primitive.plane_cylinder,
   restated: the rim point of the nearer cap closest to the plane, the same rim
   direction on the farther cap, then the nearer cap's rim points 120 degrees
   either side of the first (a cylinder standing on the plane: 3 contacts;
   lying on it: 2) */
static int raw_plane_cylinder(contact_t* out, real margin, const real pp[3], const real pm[9], const real cp[3],
                              const real cm[9], real r, real h) {
  const real n[3] = {pm[2], pm[5], pm[8]};
  real ax[3] = {cm[2], cm[5], cm[8]};
  real prjaxis = dot3(n, ax);
  if (prjaxis > 0) {
    for (int k = 0; k < 3; k++) ax[k] = -ax[k];
    prjaxis = -prjaxis;
  }
  const real dif[3] = {cp[0] - pp[0], cp[1] - pp[1], cp[2] - pp[2]};
  const real dist0 = dot3(dif, n);
  real vec[3];
  for (int k = 0; k < 3; k++) vec[k] = ax[k] * prjaxis - n[k];
  const real len = norm3(vec);
  if (len < MINVAL) { /* axis along the normal: any rim direction */
    for (int k = 0; k < 3; k++) vec[k] = cm[3 * k] * r;
  } else {
    for (int k = 0; k < 3; k++) vec[k] *= r / len;
  }
  const real prjvec = dot3(vec, n);
  for (int k = 0; k < 3; k++) ax[k] *= h;
  prjaxis *= h;
  int cnt = 0;
  for (int e = 0; e < 2; e++) {
    const real sg = e == 0 ? 1 : -1, dist = dist0 + sg * prjaxis + prjvec;
    if (dist > margin) continue;
    contact_t* c = out + cnt++;
    c->dist = dist;
    for (int k = 0; k < 3; k++) {
      c->pos[k] = cp[k] + vec[k] + sg * ax[k] - n[k] * 0.5 * dist;
      c->frame[k] = n[k];
      c->frame[3 + k] = 0;
    }
  }
  const real dist = dist0 + prjaxis - 0.5 * prjvec;
  if (dist <= margin) {
    real side[3];
    cross3(side, vec, ax);
    const real sl = norm3(side);
    for (int k = 0; k < 3; k++) side[k] = sl > MINVAL ? side[k] * (r * sqrt(3.0) * 0.5 / sl) : 0;
    for (int e = 0; e < 2; e++) {
      const real sg = e == 0 ? 1 : -1;
      contact_t* c = out + cnt++;
      c->dist = dist;
      for (int k = 0; k < 3; k++) {
        c->pos[k] = cp[k] + ax[k] - 0.5 * vec[k] + sg * side[k] - n[k] * 0.5 * dist;
        c->frame[k] = n[k];
        c->frame[3 + k] = 0;
      }
    }
  }
  return cnt;
}

/* plane (geom1) - ellipsoid (geom2, semi-axes s): the ellipsoid's support
   point against the plane normal (MuJoCo Warp plane_ellipsoid, restated):
   in the ellipsoid frame p = -S^2 n_l / |S n_l| */
static int raw_plane_ellipsoid(contact_t* c, real margin, const real pp[3], const real pm[9], const real ep[3],
                               const real em[9], const real s[3]) {
  const real n[3] = {pm[2], pm[5], pm[8]};
  real nl[3], u[3], pl[3], pw[3];
  for (int k = 0; k < 3; k++) nl[k] = em[k] * n[0] + em[3 + k] * n[1] + em[6 + k] * n[2];
  for (int k = 0; k < 3; k++) u[k] = s[k] * nl[k];
  const real ul = norm3(u);
  for (int k = 0; k < 3; k++) pl[k] = -s[k] * u[k] / (ul > MINVAL ? ul : MINVAL);
  for (int k = 0; k < 3; k++) pw[k] = em[3 * k] * pl[0] + em[3 * k + 1] * pl[1] + em[3 * k + 2] * pl[2];
  real dif[3];
  for (int k = 0; k < 3; k++) dif[k] = ep[k] + pw[k] - pp[k];
  const real dist = dot3(dif, n);
  if (dist > margin) return 0;
  c->dist = dist;
  for (int k = 0; k < 3; k++) {
    c->pos[k] = ep[k] + pw[k] - n[k] * 0.5 * dist;
    c->frame[k] = n[k];
    c->frame[3 + k] = 0;
  }
  return 1;
}

/* sphere (geom1, radius rs) - cylinder (geom2, radius r, half height h)
   (MuJoCo Warp sphere_cylinder, restated): against the side when the centre
   projects onto the shaft, against the cap when it lies over the cap disc
   (inside: whichever surface is nearer), otherwise against the rim circle */
static int raw_sphere_cylinder(contact_t* c, real margin, const real sp[3], real rs, const real cp[3], const real cm[9],
                               real r, real h) {
  const real ax[3] = {cm[2], cm[5], cm[8]};
  const real v[3] = {sp[0] - cp[0], sp[1] - cp[1], sp[2] - cp[2]};
  const real x = dot3(v, ax);
  real pr[3];
  for (int k = 0; k < 3; k++) pr[k] = v[k] - ax[k] * x;
  const real pr2 = dot3(pr, pr);
  int side = fabs(x) < h, cap = pr2 < r * r;
  if (side && cap) { /* centre inside: the nearer surface */
    if (h - fabs(x) < r - sqrt(pr2)) side = 0; else cap = 0;
  }
  if (side) { /* the shaft point level with the centre, as a sphere of radius r */
    real q[3];
    for (int k = 0; k < 3; k++) q[k] = cp[k] + ax[k] * x;
    return raw_sphere_sphere(c, margin, sp, rs, q, r);
  }
  if (cap) { /* the cap plane, normal from the sphere into the cylinder */
    const real sg = x > 0 ? 1 : -1;
    real nrm[3], q[3];
    for (int k = 0; k < 3; k++) { nrm[k] = -sg * ax[k]; q[k] = cp[k] + sg * ax[k] * h; }
    real d[3];
    for (int k = 0; k < 3; k++) d[k] = sp[k] - q[k];
    const real dist = -dot3(d, nrm) - rs;
    if (dist > margin) return 0;
    c->dist = dist;
    for (int k = 0; k < 3; k++) {
      c->pos[k] = sp[k] + nrm[k] * (rs + 0.5 * dist);
      c->frame[k] = nrm[k];
      c->frame[3 + k] = 0;
    }
    return 1;
  }
  /* the rim: the circle point nearest the centre, as a sphere of radius 0 */
  const real prl = sqrt(pr2);
  real q[3];
  const real sg = x > 0 ? 1 : -1;
  for (int k = 0; k < 3; k++) q[k] = cp[k] + sg * ax[k] * h + (prl > MINVAL ? pr[k] * (r / prl) : 0);
  return raw_sphere_sphere(c, margin, sp, rs, q, 0);
}

/* the general convex pairs (sphere-ellipsoid, capsule-{ellipsoid,cylinder},
   ellipsoid-{ellipsoid,cylinder,box}, cylinder-{cylinder,box}): GJK + EPA,
   one contact (asimov-mjlab_amd/csrc/mjh_convex.h, shared with the kernel and
   pinned by tests/test_convex.py's known answers) */
#define CVX_REAL real
#include "mjh_convex.h"

static int convex_pair(int t1, int t2) {
  if (t1 < 2 || t2 < 2) return 0;
  return t2 == 4 || (t2 == 5 && t1 != 2) || (t2 == 6 && (t1 == 4 || t1 == 5));
}

static int collide(const or_model* m, ws_t* w, int g1, int g2, real margin, contact_t* out) {
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const real *p1 = w->gxpos + 3 * g1, *m1 = w->gxmat + 9 * g1, *s1 = m->geom_size + 3 * g1;
  const real *p2 = w->gxpos + 3 * g2, *m2 = w->gxmat + 9 * g2, *s2 = m->geom_size + 3 * g2;
  if (t1 == 0 && t2 == 2) return raw_plane_sphere(out, margin, p1, m1, p2, s2[0]);
  if (t1 == 0 && t2 == 3) {
    real ax[3] = {m2[2], m2[5], m2[8]}, a[3], b[3];
    for (int k = 0; k < 3; k++) { a[k] = p2[k] + ax[k] * s2[1]; b[k] = p2[k] - ax[k] * s2[1]; }
    int n1 = raw_plane_sphere(out, margin, p1, m1, a, s2[0]);
    int n2 = raw_plane_sphere(out + n1, margin, p1, m1, b, s2[0]);
    if (n1) memcpy(out[0].frame + 3, ax, 3 * sizeof(real));
    if (n2) memcpy(out[n1].frame + 3, ax, 3 * sizeof(real));
    return n1 + n2;
  }
  if (t1 == 0 && t2 == 6) {
    real n[3] = {m1[2], m1[5], m1[8]};
    real dif[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    real dist = dot3(dif, n);
    int cnt = 0;
    for (int i = 0; i < 8 && cnt < 4; i++) {
      real v[3] = {0, 0, 0};
      for (int k = 0; k < 3; k++) {
        real s = (i & (1 << k)) ? s2[k] : -s2[k];
        v[0] += m2[k] * s; v[1] += m2[3 + k] * s; v[2] += m2[6 + k] * s;
      }
      real ld = dot3(n, v);
      if (dist + ld > margin) continue;
      contact_t* c = out + cnt++;
      c->dist = dist + ld;
      for (int k = 0; k < 3; k++) {
        c->pos[k] = p2[k] + v[k] - n[k] * 0.5 * c->dist;
        c->frame[k] = n[k];
        c->frame[3 + k] = 0;
      }
    }
    return cnt;
  }
  if (t1 == 2 && t2 == 2) return raw_sphere_sphere(out, margin, p1, s1[0], p2, s2[0]);
  if (t1 == 2 && t2 == 3) {
    real ax[3] = {m2[2], m2[5], m2[8]};
    real dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    real x = dot3(dif, ax);
    x = x < -s2[1] ? -s2[1] : (x > s2[1] ? s2[1] : x);
    real v[3] = {p2[0] + ax[0] * x, p2[1] + ax[1] * x, p2[2] + ax[2] * x};
    return raw_sphere_sphere(out, margin, p1, s1[0], v, s2[0]);
  }
  if (t1 == 3 && t2 == 3) {
    real a1[3] = {m1[2] * s1[1], m1[5] * s1[1], m1[8] * s1[1]};
    real a2[3] = {m2[2] * s2[1], m2[5] * s2[1], m2[8] * s2[1]};
    real dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    real ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    real u = -dot3(a1, dif), v = dot3(a2, dif), det = ma * mc - mb * mb;
    real v1[3], v2[3];
    if (fabs(det) >= MINVAL) {
      real x1 = (mc * u - mb * v) / det, x2 = (ma * v - mb * u) / det;
      if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
      else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
      if (x2 > 1) { x2 = 1; x1 = (u - mb) / ma; x1 = x1 < -1 ? -1 : (x1 > 1 ? 1 : x1); }
      else if (x2 < -1) { x2 = -1; x1 = (u + mb) / ma; x1 = x1 < -1 ? -1 : (x1 > 1 ? 1 : x1); }
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
      return raw_sphere_sphere(out, margin, v1, s1[0], v2, s2[0]);
    }
    /* parallel axes: test segment end points */
    int n = 0;
    for (int e = 0; e < 2 && n < 2; e++) {
      real x1 = e ? -1 : 1;
      real x2 = (v - mb * x1) / mc;
      x2 = x2 < -1 ? -1 : (x2 > 1 ? 1 : x2);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
      n += raw_sphere_sphere(out + n, margin, v1, s1[0], v2, s2[0]);
    }
    for (int e = 0; e < 2 && n < 2; e++) {
      real x2 = e ? -1 : 1;
      real x1 = (u - mb * x2) / ma;
      x1 = x1 < -1 ? -1 : (x1 > 1 ? 1 : x1);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
      n += raw_sphere_sphere(out + n, margin, v1, s1[0], v2, s2[0]);
    }
    return n;
  }
  if (t1 == 0 && t2 == 4) return raw_plane_ellipsoid(out, margin, p1, m1, p2, m2, s2);
  if (t1 == 0 && t2 == 5) return raw_plane_cylinder(out, margin, p1, m1, p2, m2, s2[0], s2[1]);
  if (t1 == 2 && t2 == 5) return raw_sphere_cylinder(out, margin, p1, s1[0], p2, m2, s2[0], s2[1]);
  if (t1 == 2 && t2 == 6) return raw_sphere_box(out, margin, p1, s1[0], p2, m2, s2);
  if (t1 == 3 && t2 == 6) {
    real ax[3] = {m1[2], m1[5], m1[8]};
    return raw_capsule_box(out, margin, p1, ax, s1[1], s1[0], p2, m2, s2);
  }
  if (t1 == 6 && t2 == 6) return raw_box_box(out, margin, p1, m1, s1, p2, m2, s2);
  if (convex_pair(t1, t2)) {
    real n[3];
    if (!cvx_collide(t1, p1, m1, s1, t2, p2, m2, s2, margin, &out->dist, out->pos, n)) return 0;
    for (int k = 0; k < 3; k++) {
      out->frame[k] = n[k];
      out->frame[3 + k] = 0;
    }
    return 1;
  }
  return 0; /* unsupported pairs are rejected by the compiler */
}

static void collision(const or_model* m, int wi, ws_t* w) {
  const real* fr = WF(m, geom_friction, wi);
  w->ncon = 0;
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
    real margin = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
    real gap = m->geom_gap[g1] > m->geom_gap[g2] ? m->geom_gap[g1] : m->geom_gap[g2];
    /* bounding-sphere broadphase */
    if (m->geom_type[g1] == 0) {
      const real* pm = w->gxmat + 9 * g1;
      real n[3] = {pm[2], pm[5], pm[8]};
      real dif[3] = {w->gxpos[3 * g2] - w->gxpos[3 * g1], w->gxpos[3 * g2 + 1] - w->gxpos[3 * g1 + 1],
                     w->gxpos[3 * g2 + 2] - w->gxpos[3 * g1 + 2]};
      if (dot3(dif, n) > margin + m->geom_rbound[g2]) continue;
    } else {
      real dif[3] = {w->gxpos[3 * g2] - w->gxpos[3 * g1], w->gxpos[3 * g2 + 1] - w->gxpos[3 * g1 + 1],
                     w->gxpos[3 * g2 + 2] - w->gxpos[3 * g1 + 2]};
      if (norm3(dif) > margin + m->geom_rbound[g1] + m->geom_rbound[g2]) continue;
    }
    contact_t tmp[4];
    memset(tmp, 0, sizeof(tmp));
    int n = collide(m, w, g1, g2, margin, tmp);
    /* contact parameters */
    int condim;
    real fri[3], solref[2], solimp[5];
    int pr1 = m->geom_priority[g1], pr2 = m->geom_priority[g2];
    if (pr1 != pr2) {
      int g = pr1 > pr2 ? g1 : g2;
      condim = m->geom_condim[g];
      for (int k = 0; k < 3; k++) fri[k] = fr[3 * g + k];
      for (int k = 0; k < 2; k++) solref[k] = m->geom_solref[2 * g + k];
      for (int k = 0; k < 5; k++) solimp[k] = m->geom_solimp[5 * g + k];
    } else {
      condim = m->geom_condim[g1] > m->geom_condim[g2] ? m->geom_condim[g1] : m->geom_condim[g2];
      for (int k = 0; k < 3; k++) fri[k] = fr[3 * g1 + k] > fr[3 * g2 + k] ? fr[3 * g1 + k] : fr[3 * g2 + k];
      real s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2], mix;
      if (s1 >= MINVAL && s2 >= MINVAL) mix = s1 / (s1 + s2);
      else if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
      else mix = s1 < MINVAL ? 0.0 : 1.0;
      const real *r1 = m->geom_solref + 2 * g1, *r2 = m->geom_solref + 2 * g2;
      if (r1[0] > 0 && r2[0] > 0)
        for (int k = 0; k < 2; k++) solref[k] = mix * r1[k] + (1 - mix) * r2[k];
      else
        for (int k = 0; k < 2; k++) solref[k] = r1[k] < r2[k] ? r1[k] : r2[k];
      for (int k = 0; k < 5; k++) solimp[k] = mix * m->geom_solimp[5 * g1 + k] + (1 - mix) * m->geom_solimp[5 * g2 + k];
    }
    for (int i = 0; i < n; i++) {
      if (w->ncon >= m->nconmax) {
        w->flags |= 1;
        break;
      }
      contact_t* c = w->con + w->ncon++;
      *c = tmp[i];
      make_frame(c->frame);
      c->dim = condim;
      c->geom[0] = g1;
      c->geom[1] = g2;
      c->friction[0] = fri[0]; c->friction[1] = fri[0]; c->friction[2] = fri[1];
      c->friction[3] = fri[2]; c->friction[4] = fri[2];
      memcpy(c->solref, solref, sizeof(solref));
      memcpy(c->solimp, solimp, sizeof(solimp));
      c->includemargin = margin - gap;
      c->efc_address = -1;
    }
  }
}

/* ---------------------------------------------------------------- constraints */
static void efc_row_params(const or_model* m, ws_t* w, int r, real pos_aref, real pos_imp, real invweight,
                           const real* solref, const real* solimp, real margin, real jqvel) {
  real timeconst = solref[0], dampratio = solref[1];
  real dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (timeconst < 2 * m->timestep && solref[0] > 0) timeconst = 2 * m->timestep;
  dmin = dmin < MINIMP ? MINIMP : (dmin > MAXIMP ? MAXIMP : dmin);
  dmax = dmax < MINIMP ? MINIMP : (dmax > MAXIMP ? MAXIMP : dmax);
  width = width < MINVAL ? MINVAL : width;
  mid = mid < MINIMP ? MINIMP : (mid > MAXIMP ? MAXIMP : mid);
  power = power < 1 ? 1 : power;
  real k = 1.0 / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  real b = 2.0 / (dmax * timeconst);
  if (solref[0] <= 0) k = -solref[0] / (dmax * dmax);
  if (solref[1] <= 0) b = -solref[1] / dmax;
  real x = fabs(pos_imp) / width, imp;
  if (x > 1) {
    imp = dmax;
  } else {
    real y;
    if (x < mid) y = pow(x, power) / pow(mid, power - 1);
    else y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
    imp = dmin + y * (dmax - dmin);
    imp = imp < dmin ? dmin : (imp > dmax ? dmax : imp);
  }
  real R = invweight * (1 - imp) / imp;
  if (R < MINVAL) R = MINVAL;
  w->efc_R[r] = R;
  w->efc_D[r] = 1.0 / R;
  w->efc_aref[r] = -k * imp * pos_aref - b * jqvel;
  w->efc_pos[r] = pos_aref + margin;
  w->efc_margin[r] = margin;
}

static int new_row(const or_model* m, ws_t* w) {
  if (w->nefc >= m->njmax) {
    w->flags |= 2;
    return -1;
  }
  int r = w->nefc++;
  memset(w->J + (size_t)r * m->nv, 0, sizeof(real) * m->nv);
  w->efc_fl[r] = 0;
  return r;
}

static void make_constraint(const or_model* m, int wi, ws_t* w) {
  int nv = m->nv;
  w->nefc = 0;
  const real* fl = WF(m, dof_frictionloss, wi);
  const real* rng = WF(m, jnt_range, wi);
  /* dof friction loss */
  for (int d = 0; d < nv; d++) {
    if (fl[d] <= 0) continue;
    int r = new_row(m, w);
    if (r < 0) return;
    w->J[r * nv + d] = 1;
    w->efc_type[r] = 1;
    w->efc_id[r] = d;
    w->efc_fl[r] = fl[d];
    efc_row_params(m, w, r, 0, 0, m->dof_invweight0[d], m->dof_solref + 2 * d, m->dof_solimp + 5 * d, 0,
                   w->qvel[d]);
  }
  /* joint limits */
  for (int j = 0; j < m->njnt; j++) {
    int t = m->jnt_type[j];
    if (m->jnt_limited[j] && t == 1) {
      /* ball: the rotation angle against the larger range bound, J = -(rotation axis)
         on the joint's three dofs (mj_instantiateLimit) */
      real ax[3];
      const real ang = fabs(quat2vel(ax, w->qpos + m->jnt_qposadr[j]));
      normalize3(ax);
      const real amax = rng[2 * j] > rng[2 * j + 1] ? rng[2 * j] : rng[2 * j + 1];
      const real pos = amax - ang - m->jnt_margin[j];
      if (pos >= 0) continue;
      int r = new_row(m, w);
      if (r < 0) return;
      const int d = m->jnt_dofadr[j];
      real jv = 0;
      for (int k = 0; k < 3; k++) {
        w->J[r * nv + d + k] = -ax[k];
        jv -= ax[k] * w->qvel[d + k];
      }
      w->efc_type[r] = 3;
      w->efc_id[r] = j;
      efc_row_params(m, w, r, pos, pos, m->dof_invweight0[d], m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j,
                     m->jnt_margin[j], jv);
      continue;
    }
    if (!m->jnt_limited[j] || (t != 2 && t != 3)) continue;
    real q = w->qpos[m->jnt_qposadr[j]];
    real dlo = q - rng[2 * j], dhi = rng[2 * j + 1] - q;
    real pos = (dlo < dhi ? dlo : dhi) - m->jnt_margin[j];
    if (pos >= 0) continue;
    int r = new_row(m, w);
    if (r < 0) return;
    int d = m->jnt_dofadr[j];
    real jj = dlo < dhi ? 1 : -1;
    w->J[r * nv + d] = jj;
    w->efc_type[r] = 3;
    w->efc_id[r] = j;
    efc_row_params(m, w, r, pos, pos, m->dof_invweight0[d], m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j,
                   m->jnt_margin[j], jj * w->qvel[d]);
  }
  /* contacts */
  for (int ci = 0; ci < w->ncon; ci++) {
    contact_t* c = w->con + ci;
    real pos = c->dist - c->includemargin;
    if (pos >= 0) continue;
    int b1 = m->geom_bodyid[c->geom[0]], b2 = m->geom_bodyid[c->geom[1]];
    /* elliptic cones (opt.cone == mjCONE_ELLIPTIC): one row per contact
       dimension (MuJoCo Warp constraint.py _efc_contact_elliptic, restated):
       row 0 the normal, row j the frame direction j (tangents, then torsion and
       rolling from the rotational Jacobian); the friction rows have no position
       term (aref from the velocity only), impedance from the normal's distance,
       invweight / impratio (times friction0^2 / friction_{j-1}^2 for j > 1) */
    int ell = m->cone == 1 && c->dim > 1;
    int nrow = c->dim == 1 ? 1 : (ell ? c->dim : 2 * (c->dim - 1));
    real invw = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    if (c->dim > 1 && !ell) {
      real f0 = c->friction[0];
      invw = invw + f0 * f0 * invw;
      invw = invw * 2 * f0 * f0 / m->impratio;
    }
    /* relative translational / rotational jacobians (b2 minus b1), projected on frame */
    real* jf = (real*)calloc((size_t)6 * nv, sizeof(real)); /* rows: n, t1, t2 (trans), n, t1, t2 (rot) */
    for (int d = 0; d < nv; d++) {
      real jp1[3], jr1[3], jp2[3], jr2[3];
      jac_col(m, w, b1, c->pos, d, jp1, jr1);
      jac_col(m, w, b2, c->pos, d, jp2, jr2);
      real dp[3] = {jp2[0] - jp1[0], jp2[1] - jp1[1], jp2[2] - jp1[2]};
      real dr[3] = {jr2[0] - jr1[0], jr2[1] - jr1[1], jr2[2] - jr1[2]};
      for (int a = 0; a < 3; a++) {
        jf[a * nv + d] = dot3(c->frame + 3 * a, dp);
        jf[(3 + a) * nv + d] = dot3(c->frame + 3 * a, dr);
      }
    }
    c->efc_address = w->nefc;
    for (int e = 0; e < nrow; e++) {
      int r = new_row(m, w);
      if (r < 0) {
        free(jf);
        return;
      }
      real* Jr = w->J + (size_t)r * nv;
      real pos_aref = pos, invw_r = invw;
      if (c->dim == 1) {
        for (int d = 0; d < nv; d++) Jr[d] = jf[d];
        w->efc_type[r] = 5;
      } else if (ell) {
        for (int d = 0; d < nv; d++) Jr[d] = jf[e * nv + d];
        w->efc_type[r] = 7;
        real f0 = c->friction[0];
        /* the cone's scale per row: mu = friction0 / sqrt(impratio) (the
           regularised cone), friction_{j-1} for row j */
        w->efc_fl[r] = e == 0 ? f0 / sqrt(m->impratio) : c->friction[e - 1];
        if (e > 0) {
          pos_aref = 0;
          invw_r = invw / m->impratio;
          if (e > 1) invw_r *= f0 * f0 / (c->friction[e - 1] * c->friction[e - 1]);
        }
      } else {
        int k = e / 2 + 1;                           /* friction direction 1..dim-1 */
        const real* jt = k < 3 ? jf + k * nv : jf + (3 + k - 3) * nv; /* tangent (trans) or torsion/roll (rot) */
        real fk = c->friction[k - 1];
        real sgn = (e % 2 == 0) ? 1 : -1;
        for (int d = 0; d < nv; d++) Jr[d] = jf[d] + sgn * fk * jt[d];
        w->efc_type[r] = 6;
      }
      w->efc_id[r] = ci;
      real jq = 0;
      for (int d = 0; d < nv; d++) jq += Jr[d] * w->qvel[d];
      efc_row_params(m, w, r, pos_aref, pos, invw_r, c->solref, c->solimp, c->includemargin, jq);
    }
    free(jf);
  }
}

/* ---------------------------------------------------------------- solver */
static void mat_vec_n(const real* A, const real* x, real* y, int n) {
  for (int i = 0; i < n; i++) {
    real s = 0;
    for (int j = 0; j < n; j++) s += A[i * n + j] * x[j];
    y[i] = s;
  }
}

/* constraint state at jaref: force, cost; returns hessian weight (D if quadratic else 0) */
static real row_eval(const ws_t* w, int r, real jaref, real* force, real* cost) {
  real D = w->efc_D[r];
  if (w->efc_type[r] == 1) {
    real f = w->efc_fl[r], R = w->efc_R[r];
    if (jaref >= R * f) { *force = -f; *cost = f * jaref - 0.5 * R * f * f; return 0; }
    if (jaref <= -R * f) { *force = f; *cost = -f * jaref - 0.5 * R * f * f; return 0; }
    *force = -D * jaref; *cost = 0.5 * D * jaref * jaref; return D;
  }
  if (jaref < 0) { *force = -D * jaref; *cost = 0.5 * D * jaref * jaref; return D; }
  *force = 0; *cost = 0; return 0;
}

/* elliptic cone contact at jar (its dim rows from r0): MuJoCo Warp solver.py
   _update_constraint_efc (CONTACT_ELLIPTIC), MuJoCo engine_solver.c, restated.
   U0 = mu jar0, Uj = friction_{j-1} jarj (the scales in efc_fl), N = U0,
   T = |U1..|: the top zone (N >= mu T) is free; the bottom zone
   (mu N + T <= 0) makes every row quadratic; between them the cone: cost
   0.5 Dm (N - mu T)^2 with Dm = D0 / (mu^2 (1 + mu^2)). Writes the rows'
   forces and, when H is given, the cost's Hessian in jar (dim x dim); returns
   the cost. */
static real cone_eval(const ws_t* w, int r0, int dim, const real* jar, real* force, real* H) {
  const real mu = w->efc_fl[r0];
  real U[6], TT = 0;
  U[0] = jar[0] * mu;
  for (int j = 1; j < dim; j++) {
    U[j] = jar[j] * w->efc_fl[r0 + j];
    TT += U[j] * U[j];
  }
  const real N = U[0], T = TT > 0 ? sqrt(TT) : 0;
  if (H) memset(H, 0, sizeof(real) * dim * dim);
  if (N >= mu * T || (T <= 0 && N >= 0)) { /* top zone */
    for (int j = 0; j < dim; j++) force[j] = 0;
    return 0;
  }
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) { /* bottom zone */
    real cost = 0;
    for (int j = 0; j < dim; j++) {
      const real D = w->efc_D[r0 + j];
      force[j] = -D * jar[j];
      cost += 0.5 * D * jar[j] * jar[j];
      if (H) H[j * dim + j] = D;
    }
    return cost;
  }
  const real m2 = mu * mu * (1 + mu * mu);
  const real Dm = w->efc_D[r0] / (m2 > MINVAL ? m2 : MINVAL), NmT = N - mu * T;
  force[0] = -Dm * NmT * mu;
  for (int j = 1; j < dim; j++) force[j] = -force[0] / T * U[j] * w->efc_fl[r0 + j];
  if (H) {
    /* in U: [1, -mu U^T / T; -mu U / T, mu N U U^T / T^3 + (mu^2 - mu N / T) I],
       then scaled by Dm and the row scales on both sides */
    real s[6];
    s[0] = mu;
    for (int j = 1; j < dim; j++) s[j] = w->efc_fl[r0 + j];
    H[0] = 1;
    for (int j = 1; j < dim; j++) H[j] = H[j * dim] = -mu * U[j] / T;
    for (int j = 1; j < dim; j++)
      for (int k = 1; k < dim; k++)
        H[j * dim + k] = mu * N * U[j] * U[k] / (T * T * T) + (j == k ? mu * mu - mu * N / T : 0);
    for (int j = 0; j < dim; j++)
      for (int k = 0; k < dim; k++) H[j * dim + k] *= Dm * s[j] * s[k];
  }
  return 0.5 * Dm * NmT * NmT;
}

/* the rows' total cost at jar (cones per contact); sabs (if given) gathers
   the magnitudes of the terms (the float32 evaluation's error scale) */
static real rows_cost(const or_model* m, const ws_t* w, const real* jar, real* sabs) {
  real cost = 0;
  for (int r = 0; r < w->nefc; r++) {
    real f[6], c;
    if (w->efc_type[r] == 7) {
      const int dim = w->con[w->efc_id[r]].dim;
      c = cone_eval(w, r, dim, jar + r, f, NULL);
      r += dim - 1;
    } else {
      row_eval(w, r, jar[r], f, &c);
    }
    cost += c;
    if (sabs) *sabs += fabs(c);
  }
  (void)m;
  return cost;
}

/* update forces/cost/qfrc_constraint at current jaref; returns total cost */
static real update_constraint(const or_model* m, ws_t* w, const real* qacc_smooth) {
  int nv = m->nv;
  real cost = 0;
  memset(w->qfrc_constraint, 0, sizeof(real) * nv);
  for (int r = 0; r < w->nefc; r++) {
    real f[6], c;
    int nr = 1;
    if (w->efc_type[r] == 7) {
      nr = w->con[w->efc_id[r]].dim;
      c = cone_eval(w, r, nr, w->jaref + r, f, NULL);
    } else {
      row_eval(w, r, w->jaref[r], f, &c);
    }
    cost += c;
    for (int j = 0; j < nr; j++) {
      w->efc_force[r + j] = f[j];
      for (int d = 0; d < nv; d++) w->qfrc_constraint[d] += w->J[(size_t)(r + j) * nv + d] * f[j];
    }
    r += nr - 1;
  }
  real gauss = 0;
  for (int d = 0; d < nv; d++) gauss += 0.5 * (w->Ma[d] - w->qfrc_smooth[d]) * (w->qacc[d] - qacc_smooth[d]);
  return cost + gauss;
}

static int chol_dense(real* A, int n) {
  for (int j = 0; j < n; j++) {
    real s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (s < MINVAL) s = MINVAL;
    real d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      real t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 0;
}
static void chol_solve(const real* L, real* x, int n) {
  for (int i = 0; i < n; i++) {
    real s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    real s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

static void newton_direction(const or_model* m, ws_t* w) {
  int nv = m->nv;
  for (int d = 0; d < nv; d++) w->grad[d] = w->Ma[d] - w->qfrc_smooth[d] - w->qfrc_constraint[d];
  memcpy(w->H, w->M, sizeof(real) * nv * nv);
  for (int r = 0; r < w->nefc; r++) {
    if (w->efc_type[r] == 7) {
      /* cone contact: J_c^T Hc J_c */
      const int dim = w->con[w->efc_id[r]].dim;
      real f[6], Hc[36];
      cone_eval(w, r, dim, w->jaref + r, f, Hc);
      for (int a = 0; a < dim; a++)
        for (int b = 0; b < dim; b++) {
          const real h = Hc[a * dim + b];
          if (h == 0) continue;
          const real *Ja = w->J + (size_t)(r + a) * nv, *Jb = w->J + (size_t)(r + b) * nv;
          for (int i = 0; i < nv; i++) {
            if (Ja[i] == 0) continue;
            for (int j = 0; j <= i; j++) w->H[i * nv + j] += h * Ja[i] * Jb[j];
          }
        }
      r += dim - 1;
      continue;
    }
    real f, c, h = row_eval(w, r, w->jaref[r], &f, &c);
    if (h == 0) continue;
    const real* Jr = w->J + (size_t)r * nv;
    for (int i = 0; i < nv; i++) {
      if (Jr[i] == 0) continue;
      for (int j = 0; j <= i; j++) w->H[i * nv + j] += h * Jr[i] * Jr[j];
    }
  }
  chol_dense(w->H, nv);
  memcpy(w->Mgrad, w->grad, sizeof(real) * nv);
  chol_solve(w->H, w->Mgrad, nv);
  for (int d = 0; d < nv; d++) w->search[d] = -w->Mgrad[d];
}

/* CG (opt.solver == mjSOL_CG): MuJoCo's primal solver with the search
   direction from M instead of the Hessian (engine_solver.c mj_solPrimal,
   restated; MuJoCo Warp solver.py): Mgrad = M^-1 grad from M's factor, the
   first search -Mgrad, later ones Polak-Ribiere: search = -Mgrad + max(0, beta)
   search, beta = grad.(Mgrad - Mgrad_old) / max(mjMINVAL, grad_old.Mgrad_old) */
static void cg_direction(const or_model* m, ws_t* w, int first) {
  int nv = m->nv;
  for (int d = 0; d < nv; d++) w->grad[d] = w->Ma[d] - w->qfrc_smooth[d] - w->qfrc_constraint[d];
  memcpy(w->Mgrad, w->grad, sizeof(real) * nv);
  solve_tree(m, w->LD, w->Mgrad);
  real beta = 0;
  if (!first) {
    real num = 0, den = 0;
    for (int d = 0; d < nv; d++) {
      num += w->grad[d] * (w->Mgrad[d] - w->cg_mg[d]);
      den += w->cg_g[d] * w->cg_mg[d];
    }
    beta = num / (den > 1e-15 ? den : (real)1e-15);
    if (beta < 0) beta = 0;
  }
  for (int d = 0; d < nv; d++) {
    w->search[d] = first ? -w->Mgrad[d] : -w->Mgrad[d] + beta * w->search[d];
    w->cg_g[d] = w->grad[d];
    w->cg_mg[d] = w->Mgrad[d];
  }
}

static void direction(const or_model* m, ws_t* w, int first) {
  if (m->solver == 1)
    cg_direction(m, w, first);
  else
    newton_direction(m, w);
}

/* adds the rows' first and second derivatives along jv at step alpha */
static void rows_derivs(ws_t* w, real alpha, real* d1, real* d2) {
  for (int r = 0; r < w->nefc; r++) {
    if (w->efc_type[r] == 7) {
      const int dim = w->con[w->efc_id[r]].dim;
      real jar[6], f[6], Hc[36];
      for (int j = 0; j < dim; j++) jar[j] = w->jaref[r + j] + alpha * w->jv[r + j];
      cone_eval(w, r, dim, jar, f, Hc);
      for (int a = 0; a < dim; a++) {
        *d1 -= f[a] * w->jv[r + a];
        for (int b = 0; b < dim; b++) *d2 += w->jv[r + a] * Hc[a * dim + b] * w->jv[r + b];
      }
      r += dim - 1;
      continue;
    }
    real ja = w->jaref[r] + alpha * w->jv[r], f, c;
    real h = row_eval(w, r, ja, &f, &c);
    *d1 -= f * w->jv[r];
    *d2 += h * w->jv[r] * w->jv[r];
  }
}

/* exact line search on the convex piecewise-quadratic cost along search */
static real linesearch(const or_model* m, ws_t* w) {
  int nv = m->nv;
  mat_vec_n(w->M, w->search, w->Mv, nv);
  for (int r = 0; r < w->nefc; r++) {
    real s = 0;
    for (int d = 0; d < nv; d++) s += w->J[(size_t)r * nv + d] * w->search[d];
    w->jv[r] = s;
  }
  real g1 = 0, g2 = 0;
  for (int d = 0; d < nv; d++) {
    g1 += w->search[d] * (w->Ma[d] - w->qfrc_smooth[d]);
    g2 += w->search[d] * w->Mv[d];
  }
  if (m->ls_parallel) {
    /* MuJoCo Warp's parallel line search (solver.py linesearch_parallel,
       restated): the cost at nlsp = ls_iterations step sizes log-spaced over
       [ls_parallel_min_step, 1]; the cheapest wins (the smallest on ties) */
    int nlsp = m->ls_iterations;
    real lmin = log((real)m->ls_parallel_min_step);
    real lstep = (0 - lmin) / (nlsp - 1 > 1 ? (real)(nlsp - 1) : (real)1);
    real best = INFINITY, second = INFINITY;
    int bi = 0;
    /* follow mode: the step size the device chose at this iteration (its
       solver_lstrace), if recorded; its cost excess over the best is reported */
    int fi = -1;
    if (w->follow && w->niter < 15) fi = (int)((w->ftrace[w->niter / 5] >> (6 * (w->niter % 5))) & 63u);
    real cf = 0, c0 = 0, sf = 0, sb = 0;
    for (int k = 0; k < nlsp; k++) {
      real a = exp(lmin + k * lstep), c = a * (g1 + 0.5 * a * g2);
      /* magnitude of the summed terms: the float32 evaluation's error scale */
      real s = fabs(a * g1) + fabs(0.5 * a * a * g2);
      for (int r = 0; r < w->nefc; r++) w->jtmp[r] = w->jaref[r] + a * w->jv[r];
      c += rows_cost(m, w, w->jtmp, &s);
      if (k == fi) { cf = c; sf = s; }
      if (k < 64) g_dbg_scan_cost[k] = c;
      if (c < best) sb = s;
      if (k == 0) c0 = c;
      if (g_dbg_lscost && k < 64) {
        if (g_dbg_lscost_it < 0 && w->niter < 15)
          g_dbg_lscost[((size_t)w->wi * 15 + w->niter) * 64 + k] = c;
        else if (w->niter == g_dbg_lscost_it)
          g_dbg_lscost[(size_t)w->wi * 64 + k] = c;
      }
      if (c < best) {
        second = best;
        best = c;
        bi = k;
      } else if (c < second) {
        second = c;
      }
    }
    /* gaps relative to the search's decrease from its smallest step (~ the
       current cost): a near-tie can be decided differently in float32 */
    real dec = c0 - best;
    if (nlsp > 1 && dec > 0) {
      real gap = (second - best) / dec;
      if (gap < w->lsgap) w->lsgap = gap;
    }
    if (g_ls_scan && fi < 0) {
      /* diagnostics: the device's rule (scan down from the full step, stop at
         the first increase) on the same candidate costs */
      int k = nlsp - 1;
      while (k > 0 && g_dbg_scan_cost[k - 1] <= g_dbg_scan_cost[k]) k--;
      bi = k;
    }
    if (fi >= 0 && fi < nlsp) {
      /* floor: float32 resolution of the cost (an iteration at convergence
         decreases it by ~nothing, where any choice is a tie) */
      real den = (dec > 0 ? dec : 0) + 1e-5 * (sf > sb ? sf : sb);
      real ex = den > 0 ? (cf - best) / den : 0;
      if (ex > w->lsexcess) w->lsexcess = ex;
      bi = fi;
    }
    if (w->niter < 15) w->lstrace[w->niter / 5] |= (unsigned)(bi & 63) << (6 * (w->niter % 5));
    return exp(lmin + bi * lstep);
  }
  /* derivative of cost(alpha) */
#define DERIVS(alpha, d1, d2)                                         \
  do {                                                                \
    d1 = g1 + (alpha) * g2;                                           \
    d2 = g2;                                                          \
    rows_derivs(w, alpha, &d1, &d2);                                  \
  } while (0)
  real d10, d20;
  DERIVS(0.0, d10, d20);
  if (!(d10 < 0)) return 0;
  real gtol = m->ls_tolerance * fabs(d10);
  real lo = 0, hi = -1, alpha = -d10 / d20;
  for (int it = 0; it < m->ls_iterations; it++) {
    real d1, d2;
    DERIVS(alpha, d1, d2);
    if (fabs(d1) <= gtol) break;
    if (d1 < 0) lo = alpha; else hi = alpha;
    real an = alpha - d1 / d2;
    if (an <= lo || (hi >= 0 && an >= hi)) an = hi >= 0 ? 0.5 * (lo + hi) : 2 * alpha;
    alpha = an;
  }
#undef DERIVS
  return alpha;
}

/* PGS (opt.solver == mjSOL_PGS): MuJoCo's projected Gauss-Seidel on the dual
   problem (engine_solver.c mj_solPGS and the dual warm start of
   engine_forward.c, restated from MuJoCo's published algorithm; MuJoCo Warp
   implements CG and Newton only, so this follows MuJoCo C):
     minimise 0.5 f' AR f + f' b,  AR = J M^-1 J' + diag(R),  b = J qacc_smooth - aref,
   one row at a time: res = b_i + AR_i f, f_i -= res / AR_ii, projected onto
   the row's set (friction loss: [-fl, fl]; limits and contact rows: f >= 0);
   a row update whose cost change 0.5 AR_ii d^2 + d res exceeds 1e-10 is undone.
   An iteration is one sweep over the rows; stop when the sweep's improvement
   (the summed cost decrease) times 1 / (meaninertia nv) is below tolerance.
   Warm start: the forces of qacc_warmstart's constraint state (jar = J qacc_ws -
   aref), replaced by zero when their dual cost is positive. Result:
   qfrc_constraint = J' f, qacc = qacc_smooth + M^-1 qfrc_constraint. Elliptic
   cones are not supported here (MuJoCo solves a small cone QCQP per contact;
   the Python layer refuses that combination). */
static void solve_pgs(const or_model* m, ws_t* w, const real* warm) {
  const int nv = m->nv, n = w->nefc;
  const real scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  real* MJ = (real*)xcalloc((size_t)n * nv, sizeof(real)); /* rows: M^-1 J_r' */
  real* A = (real*)xcalloc((size_t)n * n, sizeof(real));
  real* b = (real*)xcalloc((size_t)n, sizeof(real));
  real* f = w->efc_force;
  for (int r = 0; r < n; r++) {
    memcpy(MJ + (size_t)r * nv, w->J + (size_t)r * nv, sizeof(real) * nv);
    solve_tree(m, w->LD, MJ + (size_t)r * nv);
  }
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) {
      real s = 0;
      for (int d = 0; d < nv; d++) s += w->J[(size_t)i * nv + d] * MJ[(size_t)j * nv + d];
      A[(size_t)i * n + j] = s;
    }
    A[(size_t)i * n + i] += w->efc_R[i];
    real s = 0;
    for (int d = 0; d < nv; d++) s += w->J[(size_t)i * nv + d] * w->qacc_smooth[d];
    b[i] = s - w->efc_aref[i];
  }
  /* warm start */
  for (int r = 0; r < n; r++) {
    real s = 0, c;
    for (int d = 0; d < nv; d++) s += w->J[(size_t)r * nv + d] * warm[d];
    row_eval(w, r, s - w->efc_aref[r], f + r, &c);
  }
  real wc = 0;
  for (int i = 0; i < n; i++) {
    real af = 0;
    for (int j = 0; j < n; j++) af += A[(size_t)i * n + j] * f[j];
    wc += f[i] * (b[i] + 0.5 * af);
  }
  if (g_dbg_warm) {
    g_dbg_warm[2 * (size_t)w->wi] = wc;
    g_dbg_warm[2 * (size_t)w->wi + 1] = 0;
  }
  w->warm_smooth = wc > 0;
  if (wc > 0) memset(f, 0, sizeof(real) * n);
  for (int it = 0; it < m->iterations; it++) {
    if (w->follow && it >= w->fniter) break;
    real improvement = 0;
    for (int i = 0; i < n; i++) {
      real res = b[i];
      for (int j = 0; j < n; j++) res += A[(size_t)i * n + j] * f[j];
      const real aii = A[(size_t)i * n + i], old = f[i];
      real fi = old - res / (aii < MINVAL ? MINVAL : aii);
      if (w->efc_type[i] == 1) {
        const real fl = w->efc_fl[i];
        fi = fi < -fl ? -fl : (fi > fl ? fl : fi);
      } else if (fi < 0) {
        fi = 0;
      }
      const real dl = fi - old;
      real change = 0.5 * dl * dl * aii + dl * res;
      if (change > 1e-10) {
        fi = old;
        change = 0;
      }
      f[i] = fi;
      improvement -= change;
    }
    w->niter++;
    const int conv = improvement * scale < m->tolerance;
    if (g_dbg_conv && it < 15) {
      real* cv = g_dbg_conv + ((size_t)w->wi * 15 + it) * 4;
      cv[0] = improvement * scale;
      cv[1] = NAN;
      cv[2] = NAN;
      cv[3] = NAN;
    }
    w->conv = conv;
    if (!w->follow && conv) break;
    if (it == m->iterations - 1 && !conv) w->capped = 1;
  }
  memset(w->qfrc_constraint, 0, sizeof(real) * nv);
  for (int r = 0; r < n; r++)
    for (int d = 0; d < nv; d++) w->qfrc_constraint[d] += w->J[(size_t)r * nv + d] * f[r];
  memcpy(w->qacc, w->qfrc_constraint, sizeof(real) * nv);
  solve_tree(m, w->LD, w->qacc);
  for (int d = 0; d < nv; d++) w->qacc[d] += w->qacc_smooth[d];
  for (int r = 0; r < n; r++) {
    real s = 0;
    for (int d = 0; d < nv; d++) s += w->J[(size_t)r * nv + d] * w->qacc[d];
    w->jaref[r] = s - w->efc_aref[r];
  }
  free(MJ);
  free(A);
  free(b);
}

static void solve(const or_model* m, ws_t* w, const real* warm) {
  int nv = m->nv;
  real scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  w->niter = 0;
  if (w->nefc == 0) {
    memcpy(w->qacc, w->qacc_smooth, sizeof(real) * nv);
    memset(w->qfrc_constraint, 0, sizeof(real) * nv);
    return;
  }
  if (m->solver == 0) {
    solve_pgs(m, w, warm);
    return;
  }
  /* warmstart: keep the lower-cost of qacc_warmstart and qacc_smooth */
  memcpy(w->qacc, warm, sizeof(real) * nv);
  mat_vec_n(w->M, w->qacc, w->Ma, nv);
  for (int r = 0; r < w->nefc; r++) {
    real s = 0;
    for (int d = 0; d < nv; d++) s += w->J[(size_t)r * nv + d] * w->qacc[d];
    w->jaref[r] = s - w->efc_aref[r];
  }
  real cost = update_constraint(m, w, w->qacc_smooth);
  for (int r = 0; r < w->nefc; r++) {
    real s = 0;
    for (int d = 0; d < nv; d++) s += w->J[(size_t)r * nv + d] * w->qacc_smooth[d];
    w->jtmp[r] = s - w->efc_aref[r];
  }
  real cost_smooth = rows_cost(m, w, w->jtmp, NULL);
  if (g_dbg_warm) {
    g_dbg_warm[2 * (size_t)w->wi] = cost;
    g_dbg_warm[2 * (size_t)w->wi + 1] = cost_smooth;
  }
  int from_smooth = w->follow ? (int)((w->ftrace[0] >> 30) & 1u) : cost > cost_smooth;
  w->warm_smooth = from_smooth;
  if (from_smooth) {
    memcpy(w->qacc, w->qacc_smooth, sizeof(real) * nv);
    memcpy(w->Ma, w->qfrc_smooth, sizeof(real) * nv);
    mat_vec_n(w->M, w->qacc, w->Ma, nv);
    for (int r = 0; r < w->nefc; r++) {
      real s = 0;
      for (int d = 0; d < nv; d++) s += w->J[(size_t)r * nv + d] * w->qacc[d];
      w->jaref[r] = s - w->efc_aref[r];
    }
    cost = update_constraint(m, w, w->qacc_smooth);
  }
  direction(m, w, 1);
  for (int it = 0; it < m->iterations; it++) {
    if (w->follow && it >= w->fniter) break;
    real alpha = linesearch(m, w);
    if (alpha == 0) break;
    for (int d = 0; d < nv; d++) {
      w->qacc[d] += alpha * w->search[d];
      w->Ma[d] += alpha * w->Mv[d];
    }
    for (int r = 0; r < w->nefc; r++) w->jaref[r] += alpha * w->jv[r];
    real old = cost;
    cost = update_constraint(m, w, w->qacc_smooth);
    direction(m, w, 0);
    w->niter++;
    real gn = 0;
    for (int d = 0; d < nv; d++) gn += w->grad[d] * w->grad[d];
    real improvement = scale * (old - cost), gradient = scale * sqrt(gn);
    /* g_stop_mode 1 (diagnostics, tools/iteration_analysis.py): the improvement
       test alone -- what a float32 solver is left with when its gradient's
       rounding floor lies above the tolerance */
    int conv = improvement < m->tolerance || (g_stop_mode == 0 && gradient < m->tolerance);
    if (g_dbg_conv && it < 15) {
      real* cv = g_dbg_conv + ((size_t)w->wi * 15 + it) * 4;
      real gm = 0;
      for (int d = 0; d < nv; d++) {
        const real t = fabs(w->Ma[d]) + fabs(w->qfrc_smooth[d]) + fabs(w->qfrc_constraint[d]);
        gm += t * t;
      }
      cv[0] = improvement;
      cv[1] = gradient;
      cv[2] = scale * (fabs(old) + fabs(cost));
      cv[3] = scale * sqrt(gm);
    }
    w->conv = conv;
    if (!w->follow && conv) break;
    if (it == m->iterations - 1 && !conv) w->capped = 1; /* stopped by the iteration cap, unconverged */
  }
}

/* ---------------------------------------------------------------- sensors */
static int subtree_has(const or_model* m, int root, int b) {
  for (int k = b; k >= 0; k = k ? m->body_parentid[k] : -1) {
    if (k == root) return 1;
    if (k == 0) break;
  }
  return 0;
}
static int obj_match(const or_model* m, int type, int id, int g) {
  if (id < 0) return 1;
  int b = m->geom_bodyid[g];
  if (type == 5) return g == id;
  if (type == 1) return b == id;
  if (type == 2) return subtree_has(m, id, b);
  return 0;
}

static void contact_force(const or_model* m, ws_t* w, int ci, real f[6]) {
  contact_t* c = w->con + ci;
  memset(f, 0, 6 * sizeof(real));
  if (c->efc_address < 0) return;
  const real* ef = w->efc_force + c->efc_address;
  if (c->dim == 1) { f[0] = ef[0]; return; }
  if (m->cone == 1) { /* elliptic: the rows are the frame components */
    for (int k = 0; k < c->dim; k++) f[k] = ef[k];
    return;
  }
  for (int e = 0; e < 2 * (c->dim - 1); e++) f[0] += ef[e];
  for (int k = 1; k < c->dim; k++) f[k] = c->friction[k - 1] * (ef[2 * k - 2] - ef[2 * k - 1]);
}

/* rotation -> unit quaternion (mju_mat2Quat: branch of the largest component, no sign normalisation) */
static void mat2quat(real q[4], const real* R) {
  real tr = R[0] + R[4] + R[8];
  if (tr > 0) {
    real sq = sqrt(tr + 1) * 2;
    q[0] = 0.25 * sq; q[1] = (R[7] - R[5]) / sq; q[2] = (R[2] - R[6]) / sq; q[3] = (R[3] - R[1]) / sq;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    real sq = sqrt(1 + R[0] - R[4] - R[8]) * 2;
    q[0] = (R[7] - R[5]) / sq; q[1] = 0.25 * sq; q[2] = (R[1] + R[3]) / sq; q[3] = (R[2] + R[6]) / sq;
  } else if (R[4] > R[8]) {
    real sq = sqrt(1 + R[4] - R[0] - R[8]) * 2;
    q[0] = (R[2] - R[6]) / sq; q[1] = (R[1] + R[3]) / sq; q[2] = 0.25 * sq; q[3] = (R[5] + R[7]) / sq;
  } else {
    real sq = sqrt(1 + R[8] - R[0] - R[4]) * 2;
    q[0] = (R[3] - R[1]) / sq; q[1] = (R[2] + R[6]) / sq; q[2] = (R[5] + R[7]) / sq; q[3] = 0.25 * sq;
  }
  normalize4(q);
}

/* a sensor object's frame (mj_sensorPos): body = inertial frame, xbody =
   body frame, geom, site; *bd: the body it moves with */
static void obj_frame(const or_model* m, const ws_t* w, int type, int id, const real** pos, const real** mat, int* bd) {
  switch (type) {
    case 1: *pos = w->xipos + 3 * id; *mat = w->ximat + 9 * id; *bd = id; break;
    case 2: *pos = w->xpos + 3 * id; *mat = w->xmat + 9 * id; *bd = id; break;
    case 5: *pos = w->gxpos + 3 * id; *mat = w->gxmat + 9 * id; *bd = m->geom_bodyid[id]; break;
    default: *pos = w->sxpos + 3 * id; *mat = w->sxmat + 9 * id; *bd = m->site_bodyid[id]; break;
  }
}

/* its orientation as a quaternion: xbody copies xquat, body composes the
   inertial frame's quaternion, geom / site convert their matrix */
static void obj_quat(const or_model* m, const ws_t* w, int wi, int type, int id, real q[4]) {
  if (type == 2) {
    memcpy(q, w->xquat + 4 * id, 4 * sizeof(real));
  } else if (type == 1) {
    mul_quat(q, w->xquat + 4 * id, WF(m, body_iquat, wi) + 4 * id);
  } else {
    const real *p, *R;
    int b;
    obj_frame(m, w, type, id, &p, &R, &b);
    mat2quat(q, R);
  }
}

/* its 6D velocity [angular; linear at the frame origin] in the world frame
   (mj_objectVelocity, flg_local 0) */
static void obj_vel(const or_model* m, const ws_t* w, int type, int id, real v[6]) {
  const real *p, *R;
  int b;
  obj_frame(m, w, type, id, &p, &R, &b);
  transform_motion(v, w->cvel + 6 * b, p, w->subtree_com + 3 * m->body_rootid[b], NULL);
}

/* cfrc_int (mj_rnePostConstraint): per body I a + v x* I v minus the external
   wrench (xfrc_applied at the body com; contact forces at the contact point:
   - on geom1's body, + on geom2's body, world body excluded), about the root's
   subtree com, then accumulated from the leaves to the root (6 * nbody) */
static void cfrc_interaction(const or_model* m, ws_t* w, const real* xfrc, real* fi) {
  const int nb = m->nbody;
  memset(fi, 0, 6 * sizeof(real) * nb);
  for (int b = 1; b < nb; b++) {
    real t1[6], t2[6], t3[6];
    inert_vec(t1, w->cinert + 10 * b, w->cacc + 6 * b);
    inert_vec(t2, w->cinert + 10 * b, w->cvel + 6 * b);
    cross_force(t3, w->cvel + 6 * b, t2);
    const real* f = xfrc + 6 * b;
    const real* c = w->subtree_com + 3 * m->body_rootid[b];
    real r[3] = {w->xipos[3 * b] - c[0], w->xipos[3 * b + 1] - c[1], w->xipos[3 * b + 2] - c[2]}, rf[3];
    cross3(rf, r, f);
    for (int k = 0; k < 3; k++) {
      fi[6 * b + k] = t1[k] + t3[k] - (f[3 + k] + rf[k]);
      fi[6 * b + 3 + k] = t1[3 + k] + t3[3 + k] - f[k];
    }
  }
  for (int ci = 0; ci < w->ncon; ci++) {
    const contact_t* con = w->con + ci;
    real F[6], Fw[3], Tw[3];
    contact_force(m, w, ci, F);
    matT_vec(Fw, con->frame, F);
    matT_vec(Tw, con->frame, F + 3);
    for (int side = 0; side < 2; side++) {
      const int b = m->geom_bodyid[con->geom[side]];
      if (b == 0) continue;
      const real sg = side ? 1 : -1;
      const real* c = w->subtree_com + 3 * m->body_rootid[b];
      real r[3] = {con->pos[0] - c[0], con->pos[1] - c[1], con->pos[2] - c[2]}, t[3];
      cross3(t, r, Fw);
      for (int k = 0; k < 3; k++) {
        fi[6 * b + k] -= sg * (Tw[k] + t[k]);
        fi[6 * b + 3 + k] -= sg * Fw[k];
      }
    }
  }
  for (int b = nb - 1; b > 0; b--) {
    const int p = m->body_parentid[b];
    if (p > 0)
      for (int k = 0; k < 6; k++) fi[6 * p + k] += fi[6 * b + k];
  }
}

/* ---- rays (mj_ray's primitive intersections, engine_ray.c): distance along a
   unit ray to the geom's surface, -1 for no hit; a x^2 + 2 b x + c = 0 gives
   the smallest non-negative root (ray_quad) */
static real ray_quad(real a, real b, real c, real x[2]) {
  real det = b * b - a * c;
  if (det < MINVAL) { x[0] = x[1] = -1; return -1; }
  det = sqrt(det);
  x[0] = (-b - det) / a;
  x[1] = (-b + det) / a;
  return x[0] >= 0 ? x[0] : (x[1] >= 0 ? x[1] : -1);
}

static real ray_geom(int type, const real* size, const real* pos, const real* mat, const real* pnt, const real* vec) {
  real dif[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]}, lp[3], lv[3], xx[2];
  matT_vec(lp, mat, dif);
  matT_vec(lv, mat, vec);
  real x = -1, sol;
  switch (type) {
    case 0: { /* plane: from the front side, within the rendered rectangle when sized */
      if (lv[2] > -MINVAL) return -1;
      x = -lp[2] / lv[2];
      if (x < 0) return -1;
      const real p0 = lp[0] + x * lv[0], p1 = lp[1] + x * lv[1];
      return ((size[0] <= 0 || fabs(p0) <= size[0]) && (size[1] <= 0 || fabs(p1) <= size[1])) ? x : -1;
    }
    case 2: /* sphere */
      return ray_quad(dot3(lv, lv), dot3(lv, lp), dot3(lp, lp) - size[0] * size[0], xx);
    case 3: { /* capsule: the round side between the flat ends, then the two caps */
      sol = ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1],
                     lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0], xx);
      if (sol >= 0 && fabs(lp[2] + sol * lv[2]) <= size[1]) x = sol;
      for (int side = -1; side <= 1; side += 2) {
        real ld[3] = {lp[0], lp[1], lp[2] - side * size[1]};
        ray_quad(dot3(lv, lv), dot3(lv, ld), dot3(ld, ld) - size[0] * size[0], xx);
        for (int i = 0; i < 2; i++)
          if (xx[i] >= 0 && side * (lp[2] + xx[i] * lv[2]) >= size[1] && (x < 0 || xx[i] < x)) x = xx[i];
      }
      return x;
    }
    case 4: { /* ellipsoid */
      real a = 0, b = 0, c = -1;
      for (int i = 0; i < 3; i++) {
        const real si = 1 / (size[i] * size[i]);
        a += si * lv[i] * lv[i]; b += si * lv[i] * lp[i]; c += si * lp[i] * lp[i];
      }
      return ray_quad(a, b, c, xx);
    }
    case 5: { /* cylinder: the flat faces within the radius, then the round side */
      if (fabs(lv[2]) > MINVAL)
        for (int side = -1; side <= 1; side += 2) {
          sol = (side * size[1] - lp[2]) / lv[2];
          if (sol < 0) continue;
          const real p0 = lp[0] + sol * lv[0], p1 = lp[1] + sol * lv[1];
          if (p0 * p0 + p1 * p1 <= size[0] * size[0] && (x < 0 || sol < x)) x = sol;
        }
      sol = ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1],
                     lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0], xx);
      if (sol >= 0 && fabs(lp[2] + sol * lv[2]) <= size[1] && (x < 0 || sol < x)) x = sol;
      return x;
    }
    case 6: /* box: the six faces */
      for (int i = 0; i < 3; i++) {
        if (fabs(lv[i]) <= MINVAL) continue;
        for (int side = -1; side <= 1; side += 2) {
          sol = (side * size[i] - lp[i]) / lv[i];
          if (sol < 0) continue;
          const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
          if (fabs(lp[i1] + sol * lv[i1]) <= size[i1] && fabs(lp[i2] + sol * lv[i2]) <= size[i2] && (x < 0 || sol < x))
            x = sol;
        }
      }
      return x;
    default:
      return -1;
  }
}

/* rangefinder (mj_sensorPos -> mj_ray): along the site's z axis, every geom but
   the site body's and the invisible ones (rgba alpha 0), nearest hit or -1 */
static real rangefinder(const or_model* m, const ws_t* w, int wi, int site) {
  const real* R = w->sxmat + 9 * site;
  const real vec[3] = {R[2], R[5], R[8]};
  const real* rgba = WF(m, geom_rgba, wi);
  const real* gsize = m->geom_size;
  const int bex = m->site_bodyid[site];
  real best = -1;
  for (int g = 0; g < m->ngeom; g++) {
    if (m->geom_bodyid[g] == bex || rgba[4 * g + 3] == 0) continue;
    const real d = ray_geom(m->geom_type[g], gsize + 3 * g, w->gxpos + 3 * g, w->gxmat + 9 * g, w->sxpos + 3 * site, vec);
    if (d >= 0 && (best < 0 || d < best)) best = d;
  }
  return best;
}

static void sensors(const or_model* m, ws_t* w, int wi, real time, const real* xfrc, real* sd) {
  real* fint = NULL;  /* cfrc_int, computed at the first force / torque sensor */
  for (int s = 0; s < m->nsensor; s++) {
    int type = m->sensor_type[s], id = m->sensor_objid[s];
    real* out = sd + m->sensor_adr[s];
    const int rtype = m->sensor_reftype[s], rid = m->sensor_refid[s];
    switch (type) {
      case 30: case 41: case 42: case 43: { /* framepos / frame{x,y,z}axis, optionally in the ref frame */
        const real *p, *R, *pr, *Rr;
        int b, br;
        obj_frame(m, w, m->sensor_objtype[s], id, &p, &R, &b);
        real v[3];
        if (type == 30) memcpy(v, p, sizeof(v));
        else for (int k = 0; k < 3; k++) v[k] = R[3 * k + (type - 41)];
        if (rid >= 0) {
          obj_frame(m, w, rtype, rid, &pr, &Rr, &br);
          if (type == 30) for (int k = 0; k < 3; k++) v[k] -= pr[k];
          matT_vec(out, Rr, v);
        } else {
          memcpy(out, v, sizeof(v));
        }
        break;
      }
      case 31: { /* framequat, optionally relative to the ref frame: q_ref^-1 q */
        real q[4];
        obj_quat(m, w, wi, m->sensor_objtype[s], id, q);
        if (rid >= 0) {
          real qr[4], qc[4];
          obj_quat(m, w, wi, rtype, rid, qr);
          qc[0] = qr[0]; qc[1] = -qr[1]; qc[2] = -qr[2]; qc[3] = -qr[3];
          mul_quat(out, qc, q);
        } else {
          memcpy(out, q, sizeof(q));
        }
        break;
      }
      case 44: case 45: { /* framelinvel / frameangvel (mj_sensorVel): world frame, or relative
                             to the ref frame and expressed in it */
        real v[6];
        obj_vel(m, w, m->sensor_objtype[s], id, v);
        if (rid < 0) {
          memcpy(out, type == 44 ? v + 3 : v, 3 * sizeof(real));
          break;
        }
        real vr[6], rel[3], dp[3], t[3];
        const real *p, *R, *pr, *Rr;
        int b, br;
        obj_vel(m, w, rtype, rid, vr);
        obj_frame(m, w, m->sensor_objtype[s], id, &p, &R, &b);
        obj_frame(m, w, rtype, rid, &pr, &Rr, &br);
        if (type == 44) {
          for (int k = 0; k < 3; k++) dp[k] = p[k] - pr[k];
          cross3(t, vr, dp);
          for (int k = 0; k < 3; k++) rel[k] = v[3 + k] - vr[3 + k] - t[k];
        } else {
          for (int k = 0; k < 3; k++) rel[k] = v[k] - vr[k];
        }
        matT_vec(out, Rr, rel);
        break;
      }
      case 46: case 47: { /* framelinacc / frameangacc (mj_objectAcceleration, world frame): cacc at
                             the frame origin plus the Coriolis term w x v */
        const real *p, *R;
        int b;
        obj_frame(m, w, m->sensor_objtype[s], id, &p, &R, &b);
        const real* c = w->subtree_com + 3 * m->body_rootid[b];
        real a[6], v[6], t[3];
        transform_motion(a, w->cacc + 6 * b, p, c, NULL);
        if (type == 47) { memcpy(out, a, 3 * sizeof(real)); break; }
        transform_motion(v, w->cvel + 6 * b, p, c, NULL);
        cross3(t, v, v + 3);
        for (int k = 0; k < 3; k++) out[k] = a[3 + k] + t[k];
        break;
      }
      case 20: case 21: case 22: { /* jointlimitpos / vel / frc: the joint's limit row, 0 when inactive */
        out[0] = 0;
        for (int r = 0; r < w->nefc; r++) {
          if (w->efc_type[r] != 3 || w->efc_id[r] != id) continue;
          if (type == 20) {
            out[0] = w->efc_pos[r] - w->efc_margin[r];
          } else if (type == 21) {
            real v = 0;
            for (int i = 0; i < m->nv; i++) v += w->J[r * m->nv + i] * w->qvel[i];
            out[0] = v;
          } else {
            out[0] = w->efc_force[r];
          }
          break;
        }
        break;
      }
      case 4: case 5: { /* force / torque: cfrc_int of the site's body at the site, in the site frame */
        if (!fint) {
          fint = (real*)malloc(6 * sizeof(real) * m->nbody);
          cfrc_interaction(m, w, xfrc, fint);
        }
        const int b = m->site_bodyid[id];
        real v[6];
        transform_force(v, fint + 6 * b, w->sxpos + 3 * id, w->subtree_com + 3 * m->body_rootid[b], w->sxmat + 9 * id);
        memcpy(out, type == 4 ? v + 3 : v, 3 * sizeof(real));
        break;
      }
      case 7: out[0] = rangefinder(m, w, wi, id); break;
      case 6: { /* magnetometer: the global field in the site frame */
        const real mg[3] = {m->magnetic_x, m->magnetic_y, m->magnetic_z};
        matT_vec(out, w->sxmat + 9 * id, mg);
        break;
      }
      case 13: out[0] = w->act_length[id]; break;
      case 14: out[0] = w->act_vel[id]; break;
      case 15: out[0] = w->act_force[id]; break;
      case 16: out[0] = w->qfrc_actuator[m->jnt_dofadr[id]]; break;
      case 18: { /* ballquat: the normalised joint quaternion */
        real q[4];
        memcpy(q, w->qpos + m->jnt_qposadr[id], sizeof(q));
        normalize4(q);
        memcpy(out, q, sizeof(q));
        break;
      }
      case 19: memcpy(out, w->qvel + m->jnt_dofadr[id], 3 * sizeof(real)); break;
      case 50: out[0] = time; break;
      case 48: { /* e_potential (mj_energyPos): gravity and joint springs */
        const real g[3] = {m->gravity_x, m->gravity_y, m->gravity_z};
        const real* stiff = WF(m, jnt_stiffness, wi);
        real e = 0;
        for (int b = 1; b < m->nbody; b++) e -= w->cinert[10 * b + 9] * dot3(g, w->xipos + 3 * b);
        for (int j = 0; j < m->njnt; j++) {
          if (stiff[j] == 0) continue;
          const int qa = m->jnt_qposadr[j], t = m->jnt_type[j];
          if (t == 2 || t == 3) {
            const real dq = w->qpos[qa] - m->qpos_spring[qa];
            e += 0.5 * stiff[j] * dq * dq;
          } else if (t == 1) {
            real dif[3];
            sub_quat(dif, w->qpos + qa, m->qpos_spring + qa);
            e += 0.5 * stiff[j] * dot3(dif, dif);
          }
        }
        out[0] = e;
        break;
      }
      case 49: { /* e_kinetic (mj_energyVel): qvel' M qvel / 2 */
        real e = 0;
        for (int i = 0; i < m->nv; i++)
          for (int j = 0; j < m->nv; j++) e += w->qvel[i] * w->M[i * m->nv + j] * w->qvel[j];
        out[0] = 0.5 * e;
        break;
      }
      case 3: { /* gyro */
        int b = m->site_bodyid[id];
        matT_vec(out, w->sxmat + 9 * id, w->cvel + 6 * b);
        break;
      }
      case 2: { /* velocimeter */
        int b = m->site_bodyid[id];
        real v[6];
        transform_motion(v, w->cvel + 6 * b, w->sxpos + 3 * id, w->subtree_com + 3 * m->body_rootid[b],
                         w->sxmat + 9 * id);
        memcpy(out, v + 3, 3 * sizeof(real));
        break;
      }
      case 1: { /* accelerometer */
        int b = m->site_bodyid[id];
        const real* c = w->subtree_com + 3 * m->body_rootid[b];
        real a[6], v[6], t[3];
        transform_motion(a, w->cacc + 6 * b, w->sxpos + 3 * id, c, w->sxmat + 9 * id);
        transform_motion(v, w->cvel + 6 * b, w->sxpos + 3 * id, c, w->sxmat + 9 * id);
        cross3(t, v, v + 3);
        for (int k = 0; k < 3; k++) out[k] = a[3 + k] + t[k];
        break;
      }
      case 9: out[0] = w->qpos[m->jnt_qposadr[id]]; break;
      case 10: out[0] = w->qvel[m->jnt_dofadr[id]]; break;
      case 34: memcpy(out, w->subtree_com + 3 * id, 3 * sizeof(real)); break;
      case 35:
      case 36: { /* subtree linear velocity / angular momentum about subtree com */
        real msum = 0, lin[3] = {0, 0, 0}, L[3] = {0, 0, 0};
        const real* mass = m->body_mass; /* world 0 copy is fine only if not expanded; use per-world below */
        (void)mass;
        const real* c = w->subtree_com + 3 * id;
        /* per-body com velocity */
        for (int b = 1; b < m->nbody; b++) {
          if (!subtree_has(m, id, b)) continue;
          real bm = w->cinert[10 * b + 9];
          real v[6];
          transform_motion(v, w->cvel + 6 * b, w->xipos + 3 * b, w->subtree_com + 3 * m->body_rootid[b], NULL);
          msum += bm;
          for (int k = 0; k < 3; k++) lin[k] += bm * v[3 + k];
        }
        real vc[3] = {0, 0, 0};
        if (msum > MINVAL) for (int k = 0; k < 3; k++) vc[k] = lin[k] / msum;
        if (type == 35) { memcpy(out, vc, sizeof(vc)); break; }
        for (int b = 1; b < m->nbody; b++) {
          if (!subtree_has(m, id, b)) continue;
          real bm = w->cinert[10 * b + 9];
          real v[6], Iw[3], dv[3], dx[3], t[3];
          transform_motion(v, w->cvel + 6 * b, w->xipos + 3 * b, w->subtree_com + 3 * m->body_rootid[b], NULL);
          /* I_b * omega in world: R diag(I) R' omega; use cinert-independent body inertia via ximat */
          const real* R = w->ximat + 9 * b;
          real wl[3];
          matT_vec(wl, R, v);
          /* inertia diag recovered from crb is not available; cinert holds I about root com.
             Use the rotational inertia about the body com: I_com = I_root - m(|d|^2 - dd') */
          real d[3] = {w->xipos[3 * b] - w->subtree_com[3 * m->body_rootid[b]],
                       w->xipos[3 * b + 1] - w->subtree_com[3 * m->body_rootid[b] + 1],
                       w->xipos[3 * b + 2] - w->subtree_com[3 * m->body_rootid[b] + 2]};
          const real* ci = w->cinert + 10 * b;
          real dd = dot3(d, d);
          real I[9] = {ci[0] - bm * (dd - d[0] * d[0]), ci[3] + bm * d[0] * d[1], ci[4] + bm * d[0] * d[2],
                       ci[3] + bm * d[0] * d[1], ci[1] - bm * (dd - d[1] * d[1]), ci[5] + bm * d[1] * d[2],
                       ci[4] + bm * d[0] * d[2], ci[5] + bm * d[1] * d[2], ci[2] - bm * (dd - d[2] * d[2])};
          (void)wl;
          mat_vec(Iw, I, v);
          for (int k = 0; k < 3; k++) { dx[k] = w->xipos[3 * b + k] - c[k]; dv[k] = (v[3 + k] - vc[k]) * bm; }
          cross3(t, dx, dv);
          for (int k = 0; k < 3; k++) L[k] += Iw[k] + t[k];
        }
        memcpy(out, L, sizeof(L));
        break;
      }
      case 40: { /* contact sensor */
        int bits = m->sensor_intprm[3 * s], reduce = m->sensor_intprm[3 * s + 1], nslot = m->sensor_intprm[3 * s + 2];
        int rtype = m->sensor_reftype[s], rid = m->sensor_refid[s], otype = m->sensor_objtype[s];
        int dim = m->sensor_dim[s];
        memset(out, 0, sizeof(real) * dim);
        int match[64], flip[64], nmatch = 0;
        for (int ci = 0; ci < w->ncon && nmatch < m->contact_sensor_maxmatch && nmatch < 64; ci++) {
          int g1 = w->con[ci].geom[0], g2 = w->con[ci].geom[1];
          if (obj_match(m, otype, id, g1) && obj_match(m, rtype, rid, g2)) { match[nmatch] = ci; flip[nmatch++] = 0; }
          else if (obj_match(m, otype, id, g2) && obj_match(m, rtype, rid, g1)) { match[nmatch] = ci; flip[nmatch++] = 1; }
        }
        if (nmatch == 0) break;
        /* per-match data */
        real F[64][6], Fw[64][3], Tw[64][3];
        for (int k = 0; k < nmatch; k++) {
          contact_t* c = w->con + match[k];
          contact_force(m, w, match[k], F[k]);
          real sgn = flip[k] ? 1 : -1; /* force on primary = +F if primary is geom2 */
          for (int a = 0; a < 3; a++) {
            Fw[k][a] = sgn * (F[k][0] * c->frame[a] + F[k][1] * c->frame[3 + a] + F[k][2] * c->frame[6 + a]);
            Tw[k][a] = sgn * (F[k][3] * c->frame[a] + F[k][4] * c->frame[3 + a] + F[k][5] * c->frame[6 + a]);
          }
        }
        int order[64], nfill;
        for (int k = 0; k < nmatch; k++) order[k] = k;
        if (reduce == 1 || reduce == 2) { /* stable sort by dist asc / contact-frame force norm desc */
          real key[64];
          for (int k = 0; k < nmatch; k++) key[k] = reduce == 1 ? w->con[match[k]].dist : -norm3(F[k]);
          for (int k = 0; k < nmatch; k++) {
            int rank = 0;
            for (int j = 0; j < nmatch; j++) rank += (key[j] < key[k] || (key[j] == key[k] && j < k)) ? 1 : 0;
            order[rank] = k;
          }
        }
        real* o = out;
        if (reduce == 3) {
          real net[3] = {0, 0, 0}, tq[3] = {0, 0, 0}, cen[3] = {0, 0, 0}, wsum = 0, mind = 1e30;
          for (int k = 0; k < nmatch; k++) {
            real fn = norm3(Fw[k]);
            for (int a = 0; a < 3; a++) { net[a] += Fw[k][a]; cen[a] += fn * w->con[match[k]].pos[a]; }
            wsum += fn;
            if (w->con[match[k]].dist < mind) mind = w->con[match[k]].dist;
          }
          for (int a = 0; a < 3; a++) cen[a] = wsum > MINVAL ? cen[a] / wsum : w->con[match[0]].pos[a];
          for (int k = 0; k < nmatch; k++) {
            real r[3], t[3];
            for (int a = 0; a < 3; a++) r[a] = w->con[match[k]].pos[a] - cen[a];
            cross3(t, r, Fw[k]);
            for (int a = 0; a < 3; a++) tq[a] += t[a] + Tw[k][a];
          }
          if (bits & 1) *o++ = nmatch;
          if (bits & 2) { memcpy(o, net, 3 * sizeof(real)); o += 3; }
          if (bits & 4) { memcpy(o, tq, 3 * sizeof(real)); o += 3; }
          if (bits & 8) *o++ = mind;
          if (bits & 16) { memcpy(o, cen, 3 * sizeof(real)); o += 3; }
          if (bits & 32) { real z[3] = {0, 0, 0}; memcpy(o, z, sizeof(z)); o += 3; }
          if (bits & 64) { real z[3] = {0, 0, 0}; memcpy(o, z, sizeof(z)); o += 3; }
          break;
        }
        nfill = nmatch < nslot ? nmatch : nslot;
        for (int sl = 0; sl < nfill; sl++) {
          int k = order[sl];
          contact_t* c = w->con + match[k];
          real sg = flip[k] ? -1 : 1;
          if (bits & 1) *o++ = nmatch;
          if (bits & 2) { memcpy(o, F[k], 3 * sizeof(real)); o += 3; }
          if (bits & 4) { memcpy(o, F[k] + 3, 3 * sizeof(real)); o += 3; }
          if (bits & 8) *o++ = c->dist;
          if (bits & 16) { memcpy(o, c->pos, 3 * sizeof(real)); o += 3; }
          if (bits & 32) { for (int a = 0; a < 3; a++) *o++ = sg * c->frame[a]; }
          if (bits & 64) { for (int a = 0; a < 3; a++) *o++ = sg * c->frame[3 + a]; }
        }
        break;
      }
    }
    /* cutoff: not for quaternions and axes (mjDATATYPE_QUATERNION / _AXIS) or contact records */
    if (m->sensor_cutoff[s] > 0 && type == 7) { /* mjDATATYPE_POSITIVE: clipped above only (a miss stays -1) */
      if (out[0] > m->sensor_cutoff[s]) out[0] = m->sensor_cutoff[s];
    } else if (m->sensor_cutoff[s] > 0 && type != 31 && type != 18 && (type < 41 || type > 43) && type != 40)
      for (int k = 0; k < m->sensor_dim[s]; k++) {
        real cut = m->sensor_cutoff[s];
        out[k] = out[k] < -cut ? -cut : (out[k] > cut ? cut : out[k]);
      }
  }
  free(fint);
}

/* ---------------------------------------------------------------- driver */
/* optional per-world debug copies (oracle_set_debug): the mass matrix qM
   (nv x nv, dense) and the constraint Jacobian efc_J (njmax x nv, rows < nefc) */
static real* g_dbg_lscost = NULL; /* (nworld, 32): candidate costs at one iteration */
static int g_dbg_lscost_it = 0;
static real* g_dbg_qM = NULL;
static real* g_dbg_J = NULL;
static real* g_dbg_lsgap = NULL;
static long long* g_dbg_lstrace = NULL;
/* the solver's own discrete decisions (oracle_set_decisions), evaluated at every
   iteration also in follow mode: per world 15 x {improvement, gradient, the
   scaled cost magnitude |old| + |cost|, the scaled magnitude of the gradient's
   terms |Ma| + |qfrc_smooth| + |qfrc_constraint|} (the convergence test's
   inputs and their float32 resolution scales, NaN where no iteration ran), and {cost at qacc_warmstart, cost at qacc_smooth}
   (the warm-start comparison) */
static real* g_dbg_conv = NULL;
static real* g_dbg_warm = NULL;
static int g_follow = 0;

static void world_step(const or_model* m, or_data* d, int wi, int integrate, ws_t* w) {
  int nq = m->nq, nv = m->nv, nu = m->nu, nb = m->nbody;
  const real* qpos_in = d->qpos + (size_t)wi * nq;
  memcpy(w->qpos, qpos_in, sizeof(real) * nq);
  memcpy(w->qvel, d->qvel + (size_t)wi * nv, sizeof(real) * nv);
  const real* ctrl = d->ctrl + (size_t)wi * nu;
  const real* qfrc_applied = d->qfrc_applied + (size_t)wi * nv;
  const real* xfrc = d->xfrc_applied + (size_t)wi * nb * 6;
  w->flags = 0;
  w->lsgap = INFINITY;
  w->lstrace[0] = w->lstrace[1] = w->lstrace[2] = 0u;
  w->warm_smooth = 0;
  w->wi = wi;
  w->capped = 0;
  w->conv = 0;
  w->lsexcess = 0;
  w->follow = g_follow && m->ls_parallel;
  if (w->follow) {
    w->fniter = d->solver_niter[wi];
    for (int k = 0; k < 3; k++) w->ftrace[k] = (unsigned)d->solver_lstrace[3 * wi + k];
  }

  kinematics(m, d, wi, w);
  com_pos(m, wi, w);
  crb(m, wi, w);
  factor_tree(m, w->M, w->LD);
  collision(m, wi, w);
  com_vel(m, w);
  rne(m, w, NULL, w->qfrc_bias);
  passive_actuation(m, wi, w, ctrl, qfrc_applied, xfrc);
  make_constraint(m, wi, w);
  memcpy(w->qacc_smooth, w->qfrc_smooth, sizeof(real) * nv);
  solve_tree(m, w->LD, w->qacc_smooth);
  solve(m, w, d->qacc_warmstart + (size_t)wi * nv);
  rne(m, w, w->qacc, NULL); /* cacc with constraint accelerations (accelerometer) */
  real* sd = d->sensordata + (size_t)wi * m->nsensordata;
  sensors(m, w, wi, d->time[wi], xfrc, sd);

  /* outputs of the forward pass */
  memcpy(d->xpos + (size_t)wi * nb * 3, w->xpos, sizeof(real) * nb * 3);
  memcpy(d->xquat + (size_t)wi * nb * 4, w->xquat, sizeof(real) * nb * 4);
  memcpy(d->xmat + (size_t)wi * nb * 9, w->xmat, sizeof(real) * nb * 9);
  memcpy(d->xipos + (size_t)wi * nb * 3, w->xipos, sizeof(real) * nb * 3);
  memcpy(d->ximat + (size_t)wi * nb * 9, w->ximat, sizeof(real) * nb * 9);
  memcpy(d->xanchor + (size_t)wi * m->njnt * 3, w->xanchor, sizeof(real) * m->njnt * 3);
  memcpy(d->xaxis + (size_t)wi * m->njnt * 3, w->xaxis, sizeof(real) * m->njnt * 3);
  memcpy(d->geom_xpos + (size_t)wi * m->ngeom * 3, w->gxpos, sizeof(real) * m->ngeom * 3);
  memcpy(d->geom_xmat + (size_t)wi * m->ngeom * 9, w->gxmat, sizeof(real) * m->ngeom * 9);
  memcpy(d->site_xpos + (size_t)wi * m->nsite * 3, w->sxpos, sizeof(real) * m->nsite * 3);
  memcpy(d->site_xmat + (size_t)wi * m->nsite * 9, w->sxmat, sizeof(real) * m->nsite * 9);
  memcpy(d->subtree_com + (size_t)wi * nb * 3, w->subtree_com, sizeof(real) * nb * 3);
  memcpy(d->cvel + (size_t)wi * nb * 6, w->cvel, sizeof(real) * nb * 6);
  memcpy(d->cacc + (size_t)wi * nb * 6, w->cacc, sizeof(real) * nb * 6);
  memcpy(d->actuator_force + (size_t)wi * nu, w->act_force, sizeof(real) * nu);
  memcpy(d->actuator_length + (size_t)wi * nu, w->act_length, sizeof(real) * nu);
  memcpy(d->actuator_velocity + (size_t)wi * nu, w->act_vel, sizeof(real) * nu);
  memcpy(d->qfrc_bias + (size_t)wi * nv, w->qfrc_bias, sizeof(real) * nv);
  memcpy(d->qfrc_passive + (size_t)wi * nv, w->qfrc_passive, sizeof(real) * nv);
  memcpy(d->qfrc_actuator + (size_t)wi * nv, w->qfrc_actuator, sizeof(real) * nv);
  memcpy(d->qfrc_smooth + (size_t)wi * nv, w->qfrc_smooth, sizeof(real) * nv);
  memcpy(d->qfrc_constraint + (size_t)wi * nv, w->qfrc_constraint, sizeof(real) * nv);
  memcpy(d->qacc_smooth + (size_t)wi * nv, w->qacc_smooth, sizeof(real) * nv);
  memcpy(d->qacc + (size_t)wi * nv, w->qacc, sizeof(real) * nv);
  d->ncon[wi] = w->ncon;
  for (int ci = 0; ci < w->ncon; ci++) {
    contact_t* c = w->con + ci;
    size_t o = (size_t)wi * m->nconmax + ci;
    d->contact_dist[o] = c->dist;
    memcpy(d->contact_pos + 3 * o, c->pos, 3 * sizeof(real));
    memcpy(d->contact_frame + 9 * o, c->frame, 9 * sizeof(real));
    memcpy(d->contact_friction + 5 * o, c->friction, 5 * sizeof(real));
    d->contact_includemargin[o] = c->includemargin;
    d->contact_dim[o] = c->dim;
    d->contact_geom[2 * o] = c->geom[0];
    d->contact_geom[2 * o + 1] = c->geom[1];
    d->contact_efc_address[o] = c->efc_address;
  }
  d->nefc[wi] = w->nefc;
  for (int r = 0; r < w->nefc; r++) {
    size_t o = (size_t)wi * m->njmax + r;
    d->efc_type[o] = w->efc_type[r];
    d->efc_id[o] = w->efc_id[r];
    d->efc_pos[o] = w->efc_pos[r];
    d->efc_D[o] = w->efc_D[r];
    d->efc_aref[o] = w->efc_aref[r];
    d->efc_force[o] = w->efc_force[r];
  }
  d->solver_niter[wi] = w->niter;
  if (g_dbg_qM) memcpy(g_dbg_qM + (size_t)wi * nv * nv, w->M, sizeof(real) * nv * nv);
  if (g_dbg_lsgap) g_dbg_lsgap[wi] = w->follow ? w->lsexcess : w->lsgap;
  d->solver_lstrace[3 * wi] = (int)(w->lstrace[0] | ((unsigned)w->warm_smooth << 30));
  d->solver_lstrace[3 * wi + 1] = (int)(w->lstrace[1] | ((unsigned)(w->conv && !w->follow) << 30));
  d->solver_lstrace[3 * wi + 2] = (int)w->lstrace[2];
  if (g_dbg_lstrace) g_dbg_lstrace[wi] = (long long)w->capped;
  if (g_dbg_J) memcpy(g_dbg_J + (size_t)wi * m->njmax * nv, w->J, sizeof(real) * (size_t)w->nefc * nv);

  if (integrate) {
    real dt = m->timestep;
    const real* damping = WF(m, dof_damping, wi);
    real* qa = w->qacc_int;
    if (m->integrator == 3) {
      /* implicitfast: (M - dt*qDeriv) qacc = qfrc_smooth + qfrc_constraint,
         qDeriv = actuator velocity gains (skipped when force-clamped) - dof damping */
      memcpy(w->H, w->M, sizeof(real) * nv * nv);
      for (int dd = 0; dd < nv; dd++) w->H[dd * nv + dd] += dt * damping[dd];
      for (int i = 0; i < nu; i++) {
        if (m->actuator_forcelimited[i]) {
          real f = w->act_force[i];
          if (f <= m->actuator_forcerange[2 * i] || f >= m->actuator_forcerange[2 * i + 1]) continue;
        }
        int dof = m->jnt_dofadr[m->actuator_trnid[i]];
        real g = m->actuator_gear[i];
        w->H[dof * nv + dof] -= dt * g * g * m->actuator_biasprm[10 * i + 2];
      }
      factor_tree(m, w->H, w->LD);
      for (int dd = 0; dd < nv; dd++) qa[dd] = w->qfrc_smooth[dd] + w->qfrc_constraint[dd];
      solve_tree(m, w->LD, qa);
    } else {
      int anyd = 0;
      for (int dd = 0; dd < nv; dd++) anyd |= damping[dd] > 0;
      if (anyd) {
        memcpy(w->H, w->M, sizeof(real) * nv * nv);
        for (int dd = 0; dd < nv; dd++) w->H[dd * nv + dd] += dt * damping[dd];
        factor_tree(m, w->H, w->LD);
        mat_vec_n(w->M, w->qacc, qa, nv);
        solve_tree(m, w->LD, qa);
      } else {
        memcpy(qa, w->qacc, sizeof(real) * nv);
      }
    }
    real* qvel = d->qvel + (size_t)wi * nv;
    real* qpos = d->qpos + (size_t)wi * nq;
    for (int dd = 0; dd < nv; dd++) w->qvel[dd] += dt * qa[dd];
    for (int j = 0; j < m->njnt; j++) {
      int q0 = m->jnt_qposadr[j], v0 = m->jnt_dofadr[j];
      if (m->jnt_type[j] == 0) {
        for (int k = 0; k < 3; k++) w->qpos[q0 + k] += dt * w->qvel[v0 + k];
        real* q = w->qpos + q0 + 3;
        real om[3] = {w->qvel[v0 + 3], w->qvel[v0 + 4], w->qvel[v0 + 5]};
        real ang = dt * normalize3(om), qr[4];
        axis_angle(qr, om, ang);
        normalize4(q);
        mul_quat(q, q, qr);
        normalize4(q);
      } else if (m->jnt_type[j] == 1) { /* ball: mju_quatIntegrate */
        real* q = w->qpos + q0;
        real om[3] = {w->qvel[v0], w->qvel[v0 + 1], w->qvel[v0 + 2]};
        real ang = dt * normalize3(om), qr[4];
        axis_angle(qr, om, ang);
        normalize4(q);
        mul_quat(q, q, qr);
        normalize4(q);
      } else {
        w->qpos[q0] += dt * w->qvel[v0];
      }
    }
    memcpy(qvel, w->qvel, sizeof(real) * nv);
    memcpy(qpos, w->qpos, sizeof(real) * nq);
    d->time[wi] += dt;
  }
  memcpy(d->qacc_warmstart + (size_t)wi * nv, w->qacc, sizeof(real) * nv);
  for (int k = 0; k < nq; k++) if (!isfinite(d->qpos[(size_t)wi * nq + k])) w->flags |= 4;
  for (int k = 0; k < nv; k++) if (!isfinite(d->qvel[(size_t)wi * nv + k]) || !isfinite(w->qacc[k])) w->flags |= 4;
  d->flags[wi] = w->flags;
  d->flags_acc[wi] |= w->flags;
}

int oracle_run(const or_model* m, or_data* d, int w0, int w1, int integrate, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    ws_t w;
    ws_alloc(&w, m);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (int wi = w0; wi < w1; wi++) world_step(m, d, wi, integrate, &w);
    ws_free(&w);
  }
  (void)nthreads;
  return 0;
}

void oracle_set_follow(int on) { g_follow = on; }

void oracle_set_ls_scan(int on) { g_ls_scan = on; }

void oracle_set_stop_mode(int mode) { g_stop_mode = mode; }

void oracle_set_lscost(real* cost, int iteration) {
  g_dbg_lscost = cost;
  g_dbg_lscost_it = iteration;
}

void oracle_set_decisions(real* conv, real* warm) {
  g_dbg_conv = conv;
  g_dbg_warm = warm;
}

void oracle_set_debug(real* qM, real* efc_J, real* lsgap, long long* lstrace) {
  g_dbg_qM = qM;
  g_dbg_J = efc_J;
  g_dbg_lsgap = lsgap;
  g_dbg_lstrace = lstrace;
}

size_t oracle_sizeof_model(void) { return sizeof(or_model); }
size_t oracle_sizeof_data(void) { return sizeof(or_data); }
int oracle_real_bytes(void) { return (int)sizeof(real); }
