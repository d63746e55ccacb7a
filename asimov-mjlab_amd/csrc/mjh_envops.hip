// mjh_envops.hip — fused elementwise kernels for the env layer (gfx950).
//
// The manager-based env evaluates its terms as chains of small torch ops
// (each a separate ~4 us launch at 4096 envs, even inside a captured graph).
// These kernels fuse the hottest chains into one launch each, with exactly the
// formulas of the torch versions in mjlab_amd/utils/math.py and
// sensor/contact_sensor.py (which restate the reference's Isaac Lab math,
// src/mjlab/third_party/isaaclab/isaaclab/utils/math.py, and the contact
// sensor's air-time tracking, src/mjlab/sensor/contact_sensor.py:327-367).
// Rows are addressed with a row stride (last-dim stride 1), so strided views
// such as pose[:, 3:7] need no copy.
#include <hip/hip_runtime.h>

#include "../../include/mjh_abi.h"

namespace {

__global__ void quat_rotate_kernel(const float* __restrict__ q, long long qs, const float* __restrict__ v, long long vs,
                                   float* __restrict__ out, long long n, float sgn) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* a = q + i * qs;
  const float* b = v + i * vs;
  const float w = a[0], x = a[1], y = a[2], z = a[3];
  const float vx = b[0], vy = b[1], vz = b[2];
  // t = 2 (xyz x v); out = v +- w t + xyz x t   (quat_apply / quat_apply_inverse)
  const float tx = 2.f * (y * vz - z * vy), ty = 2.f * (z * vx - x * vz), tz = 2.f * (x * vy - y * vx);
  float* o = out + 3 * i;
  o[0] = (vx + sgn * w * tx) + (y * tz - z * ty);
  o[1] = (vy + sgn * w * ty) + (z * tx - x * tz);
  o[2] = (vz + sgn * w * tz) + (x * ty - y * tx);
}

__global__ void quat_mul_kernel(const float* __restrict__ p, long long ps, const float* __restrict__ q, long long qs,
                                float* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* a = p + i * ps;
  const float* b = q + i * qs;
  const float w1 = a[0], x1 = a[1], y1 = a[2], z1 = a[3];
  const float w2 = b[0], x2 = b[1], y2 = b[2], z2 = b[3];
  const float ww = (z1 + x1) * (x2 + y2);
  const float yy = (w1 - y1) * (w2 + z2);
  const float zz = (w1 + y1) * (w2 - z2);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
  float* o = out + 4 * i;
  o[0] = qq - ww + (z1 - y1) * (y2 - z2);
  o[1] = qq - xx + (x1 + w1) * (x2 + w2);
  o[2] = qq - yy + (w1 - x1) * (y2 + z2);
  o[3] = qq - zz + (z1 + y1) * (w2 - x2);
}

__global__ void velocity_from_cvel_kernel(const float* __restrict__ pos, long long ps, const float* __restrict__ com,
                                          long long cs, const float* __restrict__ cvel, long long vs,
                                          float* __restrict__ out, long long n, int k) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = pos + i * ps;
  const float* c = com + (i / k) * cs;  // k rows (bodies/sites) share their env's com
  const float* v = cvel + i * vs;
  const float ox = c[0] - p[0], oy = c[1] - p[1], oz = c[2] - p[2];
  const float wx = v[0], wy = v[1], wz = v[2];
  float* o = out + 6 * i;
  o[0] = v[3] - (wy * oz - wz * oy);
  o[1] = v[4] - (wz * ox - wx * oz);
  o[2] = v[5] - (wx * oy - wy * ox);
  o[3] = wx; o[4] = wy; o[5] = wz;
}

// one thread per env: its k slots, then the env's last_time (read before, so
// every slot sees the pre-update value)
__global__ void air_time_kernel(const float* __restrict__ sensordata, long long sds, const int* __restrict__ cols, int k,
                                const float* __restrict__ time, float* last_time, float* cur_air, float* last_air,
                                float* cur_con, float* last_con, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float now = time[e];
  const float el = now - last_time[e];
  for (int j = 0; j < k; j++) {
    const long long t = e * k + j;
    const bool is_c = sensordata[e * sds + cols[j]] > 0.f;
    const float ca = cur_air[t], cc = cur_con[t];
    if (ca > 0.f && is_c) last_air[t] = ca + el;
    cur_air[t] = is_c ? 0.f : ca + el;
    if (cc > 0.f && !is_c) last_con[t] = cc + el;
    cur_con[t] = is_c ? cc + el : 0.f;
  }
  last_time[e] = now;
}

inline int grid(long long n) { return (int)((n + 255) / 256); }

inline int finish() { return hipGetLastError() == hipSuccess ? 0 : 2; }

}  // namespace

extern "C" {

int mjh_quat_rotate(const float* q, long long qs, const float* v, long long vs, float* out, long long n, int inverse,
                    void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(quat_rotate_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, q, qs, v, vs, out, n,
                     inverse ? -1.f : 1.f);
  return finish();
}

int mjh_quat_mul(const float* p, long long ps, const float* q, long long qs, float* out, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(quat_mul_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, p, ps, q, qs, out, n);
  return finish();
}

int mjh_velocity_from_cvel(const float* pos, long long ps, const float* com, long long cs, const float* cvel, long long vs,
                           float* out, long long n, int k, void* stream) {
  if (n <= 0 || k <= 0) return 0;
  hipLaunchKernelGGL(velocity_from_cvel_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, pos, ps, com, cs, cvel,
                     vs, out, n, k);
  return finish();
}

int mjh_air_time_update(const float* sensordata, long long sds, const int* cols, int k, const float* time,
                        float* last_time, float* cur_air, float* last_air, float* cur_con, float* last_con, long long n,
                        void* stream) {
  if (n <= 0 || k <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(air_time_kernel, dim3(grid(n)), dim3(256), 0, s, sensordata, sds, cols, k, time, last_time,
                     cur_air, last_air, cur_con, last_con, n);
  return finish();
}

}  // extern "C"

// ---- observation term post-processing, written into its slice of the group
// buffer: out = clip(x + (u * (hi - lo) + lo), cmin, cmax) * scale
// (observation_manager.py:163-176: noise -> clip -> scale; u = U[0,1) draws,
// null when the term has no noise; clip skipped when cmin > cmax)
namespace {
__global__ void obs_term_kernel(const float* __restrict__ x, long long xs, const float* __restrict__ u, long long us,
                                float lo, float hi, float cmin, float cmax, float scale, float* __restrict__ out,
                                long long os, int w, long long n) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * w) return;
  const long long e = t / w;
  const int j = (int)(t - e * w);
  float v = x[e * xs + j];
  if (u) v = v + (u[e * us + j] * (hi - lo) + lo);
  if (cmin <= cmax) v = fminf(fmaxf(v, cmin), cmax);
  out[e * os + j] = v * scale;
}
}  // namespace

extern "C" int mjh_obs_term(const float* x, long long xs, const float* u, long long us, float lo, float hi, float cmin,
                            float cmax, float scale, float* out, long long os, int w, long long n, void* stream) {
  if (n <= 0 || w <= 0) return 0;
  hipLaunchKernelGGL(obs_term_kernel, dim3((int)((n * w + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, xs, u, us,
                     lo, hi, cmin, cmax, scale, out, os, w, n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---- rotations for resets and motion tracking -----------------------------
// Formulas of utils/math.py (isaaclab/utils/math.py): quat_from_euler_xyz,
// quat_inv, quat_mul, quat_apply, yaw_quat, axis_angle_from_quat,
// matrix_from_quat, subtract_frame_transforms.
namespace {
struct Q4 {
  float w, x, y, z;
};
__device__ __forceinline__ Q4 ld4(const float* p) { return Q4{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ Q4 qmul(Q4 a, Q4 b) {
  const float ww = (a.z + a.x) * (b.x + b.y);
  const float yy = (a.w - a.y) * (b.w + b.z);
  const float zz = (a.w + a.y) * (b.w - b.z);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (a.z - a.x) * (b.x - b.y));
  return Q4{qq - ww + (a.z - a.y) * (b.y - b.z), qq - xx + (a.x + a.w) * (b.x + b.w), qq - yy + (a.w - a.x) * (b.y + b.z),
            qq - zz + (a.z + a.y) * (b.w - b.x)};
}
__device__ __forceinline__ Q4 qinv(Q4 q) {
  float n2 = q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z;
  n2 = fmaxf(n2, 1e-9f);
  return Q4{q.w / n2, -q.x / n2, -q.y / n2, -q.z / n2};
}
// quat_apply: v + w t + xyz x t, t = 2 xyz x v
__device__ __forceinline__ void qapply(Q4 q, const float v[3], float o[3]) {
  const float tx = (q.y * v[2] - q.z * v[1]) * 2.f, ty = (q.z * v[0] - q.x * v[2]) * 2.f, tz = (q.x * v[1] - q.y * v[0]) * 2.f;
  o[0] = v[0] + q.w * tx + (q.y * tz - q.z * ty);
  o[1] = v[1] + q.w * ty + (q.z * tx - q.x * tz);
  o[2] = v[2] + q.w * tz + (q.x * ty - q.y * tx);
}
__device__ __forceinline__ Q4 qyaw(Q4 q) {
  const float yaw = atan2f(2.f * (q.w * q.z + q.x * q.y), 1.f - 2.f * (q.y * q.y + q.z * q.z));
  const float c = cosf(yaw / 2.f), s = sinf(yaw / 2.f);
  const float nrm = sqrtf(c * c + s * s);
  return Q4{c / nrm, 0.f, 0.f, s / nrm};
}
// |axis_angle_from_quat(q)|
__device__ __forceinline__ float qangle(Q4 q) {
  const float sg = q.w < 0.f ? -1.f : 1.f;
  const float w = q.w * sg, x = q.x * sg, y = q.y * sg, z = q.z * sg;
  const float mag = sqrtf(x * x + y * y + z * z);
  const float half = atan2f(mag, w);
  const float ang = 2.f * half;
  const float s = fabsf(ang) > 1e-6f ? sinf(half) / ang : 0.5f - ang * ang / 48.f;
  const float ax = x / s, ay = y / s, az = z / s;
  return sqrtf(ax * ax + ay * ay + az * az);
}
// first `nc` columns of matrix_from_quat(q), row-major (3 x nc)
__device__ __forceinline__ void qmat(Q4 q, int nc, float* o) {
  const float two_s = 2.f / (q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  const float m[9] = {1.f - two_s * (q.y * q.y + q.z * q.z), two_s * (q.x * q.y - q.z * q.w), two_s * (q.x * q.z + q.y * q.w),
                      two_s * (q.x * q.y + q.z * q.w), 1.f - two_s * (q.x * q.x + q.z * q.z), two_s * (q.y * q.z - q.x * q.w),
                      two_s * (q.x * q.z - q.y * q.w), two_s * (q.y * q.z + q.x * q.w), 1.f - two_s * (q.x * q.x + q.y * q.y)};
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < nc; c++) o[r * nc + c] = m[r * 3 + c];
}

__global__ void quat_from_euler_kernel(const float* __restrict__ rpy, long long rs, float* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* a = rpy + i * rs;
  const float cy = cosf(a[2] * 0.5f), sy = sinf(a[2] * 0.5f);
  const float cr = cosf(a[0] * 0.5f), sr = sinf(a[0] * 0.5f);
  const float cp = cosf(a[1] * 0.5f), sp = sinf(a[1] * 0.5f);
  float* o = out + 4 * i;
  o[0] = cy * cr * cp + sy * sr * sp;
  o[1] = cy * sr * cp - sy * cr * sp;
  o[2] = cy * cr * sp + sy * sr * cp;
  o[3] = sy * cr * cp - cy * sr * sp;
}

__global__ void quat_error_kernel(const float* __restrict__ q1, long long s1, const float* __restrict__ q2, long long s2,
                                  float* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Q4 b = ld4(q2 + i * s2);
  out[i] = qangle(qmul(ld4(q1 + i * s1), Q4{b.w, -b.x, -b.y, -b.z}));
}

// T12 = T01^-1 T02 for n rows; rows i use frame row i / k
__global__ void frame_subtract_kernel(const float* __restrict__ t01, long long st01, const float* __restrict__ q01,
                                      long long sq01, const float* __restrict__ t02, long long st02, long long rt02,
                                      const float* __restrict__ q02, long long sq02, long long rq02, int k,
                                      float* __restrict__ t12, float* __restrict__ q12, int qcols, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long f = i / k, j = i - f * k;
  const Q4 q10 = qinv(ld4(q01 + f * sq01));
  if (t12) {
    const float* a = t01 + f * st01;
    const float* b = t02 + f * st02 + j * rt02;
    const float d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    qapply(q10, d, t12 + 3 * i);
  }
  if (q12) {
    const Q4 r = qmul(q10, ld4(q02 + f * sq02 + j * rq02));
    if (qcols == 0) {
      float* o = q12 + 4 * i;
      o[0] = r.w; o[1] = r.x; o[2] = r.y; o[3] = r.z;
    } else {
      qmat(r, qcols, q12 + 3 * qcols * i);
    }
  }
}

// MotionCommand._update_command targets (tracking/mdp/commands.py:383-405):
// per env delta = (robot anchor xy, motion anchor z), yaw(robot_q * motion_q^-1);
// per body: q_rel = delta (x) q_body, p_rel = delta_pos + delta (x) (p_body - anchor)
__global__ void motion_relative_kernel(const float* __restrict__ ap, long long sap, const float* __restrict__ aq,
                                       long long saq, const float* __restrict__ rp, long long srp,
                                       const float* __restrict__ rq, long long srq, const float* __restrict__ bp,
                                       long long sbp, long long rbp, const float* __restrict__ bq, long long sbq,
                                       long long rbq, int k, float* __restrict__ out_p, float* __restrict__ out_q,
                                       long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long e = i / k, j = i - e * k;
  const float* a = ap + e * sap;
  const float* r = rp + e * srp;
  const Q4 dq = qyaw(qmul(ld4(rq + e * srq), qinv(ld4(aq + e * saq))));
  const Q4 qr = qmul(dq, ld4(bq + e * sbq + j * rbq));
  float* oq = out_q + 4 * i;
  oq[0] = qr.w; oq[1] = qr.x; oq[2] = qr.y; oq[3] = qr.z;
  const float* b = bp + e * sbp + j * rbp;
  const float d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  float t[3];
  qapply(dq, d, t);
  float* op = out_p + 3 * i;
  op[0] = r[0] + t[0]; op[1] = r[1] + t[1]; op[2] = a[2] + t[2];
}
}  // namespace

extern "C" {
int mjh_quat_from_euler(const float* rpy, long long rs, float* out, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(quat_from_euler_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, rpy, rs, out, n);
  return finish();
}

int mjh_quat_error(const float* q1, long long s1, const float* q2, long long s2, float* out, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(quat_error_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, q1, s1, q2, s2, out, n);
  return finish();
}

int mjh_frame_subtract(const float* t01, long long st01, const float* q01, long long sq01, const float* t02,
                       long long st02, long long rt02, const float* q02, long long sq02, long long rq02, int k,
                       float* t12, float* q12, int qcols, long long n, void* stream) {
  if (n <= 0 || k <= 0) return 0;
  if (qcols < 0 || qcols > 3) return 1;
  hipLaunchKernelGGL(frame_subtract_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, t01, st01, q01, sq01, t02,
                     st02, rt02, q02, sq02, rq02, k, t12, q12, qcols, n);
  return finish();
}

int mjh_motion_relative(const float* ap, long long sap, const float* aq, long long saq, const float* rp, long long srp,
                        const float* rq, long long srq, const float* bp, long long sbp, long long rbp, const float* bq,
                        long long sbq, long long rbq, int k, float* out_p, float* out_q, long long n, void* stream) {
  if (n <= 0 || k <= 0) return 0;
  hipLaunchKernelGGL(motion_relative_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, ap, sap, aq, saq, rp, srp,
                     rq, srq, bp, sbp, rbp, bq, sbq, rbq, k, out_p, out_q, n);
  return finish();
}
}  // extern "C"
