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

__global__ void air_time_kernel(const float* __restrict__ sensordata, long long sds, const int* __restrict__ cols, int k,
                                const float* __restrict__ time, float* last_time, float* cur_air, float* last_air,
                                float* cur_con, float* last_con, long long n) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * k) return;
  const long long e = t / k;
  const int j = (int)(t - e * k);
  const float now = time[e];
  const float el = now - last_time[e];
  const bool is_c = sensordata[e * sds + cols[j]] > 0.f;
  const float ca = cur_air[t], cc = cur_con[t];
  if (ca > 0.f && is_c) last_air[t] = ca + el;
  cur_air[t] = is_c ? 0.f : ca + el;
  if (cc > 0.f && !is_c) last_con[t] = cc + el;
  cur_con[t] = is_c ? cc + el : 0.f;
}

// last_time is written by a second launch so every (env, slot) thread above
// reads the pre-update value
__global__ void copy_kernel(const float* __restrict__ src, float* __restrict__ dst, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
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
  hipLaunchKernelGGL(air_time_kernel, dim3(grid(n * k)), dim3(256), 0, s, sensordata, sds, cols, k, time, last_time,
                     cur_air, last_air, cur_con, last_con, n);
  hipLaunchKernelGGL(copy_kernel, dim3(grid(n)), dim3(256), 0, s, time, last_time, n);
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
