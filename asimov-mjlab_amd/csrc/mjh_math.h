// mjh_math.h — device math for the batched step (float32, gfx950).
#pragma once
#include <hip/hip_runtime.h>

#define MJH_MINVAL 1e-15f
#define MJH_MINIMP 0.0001f
#define MJH_MAXIMP 0.9999f

namespace mjh {

__device__ __forceinline__ void quat_mul(float r[4], const float a[4], const float b[4]) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}

__device__ __forceinline__ void quat_normalize(float q[4]) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MJH_MINVAL) {
    q[0] = 1.f; q[1] = q[2] = q[3] = 0.f;
  } else {
    float inv = 1.f / n;
    q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
  }
}

__device__ __forceinline__ void quat2mat(float m[9], const float q[4]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1.f - 2.f * (y * y + z * z); m[1] = 2.f * (x * y - w * z); m[2] = 2.f * (x * z + w * y);
  m[3] = 2.f * (x * y + w * z); m[4] = 1.f - 2.f * (x * x + z * z); m[5] = 2.f * (y * z - w * x);
  m[6] = 2.f * (x * z - w * y); m[7] = 2.f * (y * z + w * x); m[8] = 1.f - 2.f * (x * x + y * y);
}

// rotation -> unit quaternion (mju_mat2Quat: the branch of the largest component, no sign normalisation)
__device__ __forceinline__ void mat2quat(float q[4], const float* R) {
  const float tr = R[0] + R[4] + R[8];
  if (tr > 0.f) {
    const float sq = sqrtf(tr + 1.f) * 2.f;
    q[0] = 0.25f * sq; q[1] = (R[7] - R[5]) / sq; q[2] = (R[2] - R[6]) / sq; q[3] = (R[3] - R[1]) / sq;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    const float sq = sqrtf(1.f + R[0] - R[4] - R[8]) * 2.f;
    q[0] = (R[7] - R[5]) / sq; q[1] = 0.25f * sq; q[2] = (R[1] + R[3]) / sq; q[3] = (R[2] + R[6]) / sq;
  } else if (R[4] > R[8]) {
    const float sq = sqrtf(1.f + R[4] - R[0] - R[8]) * 2.f;
    q[0] = (R[2] - R[6]) / sq; q[1] = (R[1] + R[3]) / sq; q[2] = 0.25f * sq; q[3] = (R[5] + R[7]) / sq;
  } else {
    const float sq = sqrtf(1.f + R[8] - R[0] - R[4]) * 2.f;
    q[0] = (R[3] - R[1]) / sq; q[1] = (R[2] + R[6]) / sq; q[2] = (R[5] + R[7]) / sq; q[3] = 0.25f * sq;
  }
  quat_normalize(q);
}

__device__ __forceinline__ void mat_vec(float r[3], const float* m, const float v[3]) {
  float a = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float b = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float c = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}

__device__ __forceinline__ void matT_vec(float r[3], const float* m, const float v[3]) {
  float a = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float b = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float c = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}

__device__ __forceinline__ void mat_mul(float r[9], const float* a, const float* b) {
  float t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = t[i];
}

__device__ __forceinline__ float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__device__ __forceinline__ void cross3(float r[3], const float* a, const float* b) {
  float x = a[1] * b[2] - a[2] * b[1];
  float y = a[2] * b[0] - a[0] * b[2];
  float z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}

__device__ __forceinline__ float normalize3(float v[3]) {
  float n = sqrtf(dot3(v, v));
  if (n < MJH_MINVAL) {
    v[0] = 1.f; v[1] = v[2] = 0.f;
  } else {
    float inv = 1.f / n;
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
  }
  return n;
}

__device__ __forceinline__ void axis_angle(float q[4], const float* axis, float ang) {
  float s, c;
  sincosf(0.5f * ang, &s, &c);
  q[0] = c; q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}

// the rotation vector (axis x angle, angle in (-pi, pi]) of a quaternion
// (MuJoCo mju_quat2Vel with dt = 1); returns the angle
__device__ __forceinline__ float quat2vel(float r[3], const float* q) {
  float ax[3] = {q[1], q[2], q[3]};
  const float s = normalize3(ax);
  float ang = 2.f * atan2f(s, q[0]);
  if (ang > 3.14159265358979f) ang -= 6.28318530717959f;
  r[0] = ax[0] * ang; r[1] = ax[1] * ang; r[2] = ax[2] * ang;
  return ang;
}

// r such that qa = qb * exp(r) (MuJoCo mju_subQuat)
__device__ __forceinline__ void sub_quat(float r[3], const float* qa, const float* qb) {
  const float qbc[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, a[4] = {qa[0], qa[1], qa[2], qa[3]};
  float d[4];
  quat_mul(d, qbc, a);
  quat2vel(r, d);
}

// spatial motion cross product r = v x m   ([ang; lin] convention)
__device__ __forceinline__ void cross_motion(float r[6], const float* v, const float* m) {
  float t0 = -v[2] * m[1] + v[1] * m[2];
  float t1 = v[2] * m[0] - v[0] * m[2];
  float t2 = -v[1] * m[0] + v[0] * m[1];
  float t3 = -v[2] * m[4] + v[1] * m[5] - v[5] * m[1] + v[4] * m[2];
  float t4 = v[2] * m[3] - v[0] * m[5] + v[5] * m[0] - v[3] * m[2];
  float t5 = -v[1] * m[3] + v[0] * m[4] - v[4] * m[0] + v[3] * m[1];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}

// spatial force cross product r = v x* f
__device__ __forceinline__ void cross_force(float r[6], const float* v, const float* f) {
  float t0 = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  float t1 = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  float t2 = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  float t3 = -v[2] * f[4] + v[1] * f[5];
  float t4 = v[2] * f[3] - v[0] * f[5];
  float t5 = -v[1] * f[3] + v[0] * f[4];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}

// 10-vector com inertia (Ixx Iyy Izz Ixy Ixz Iyz, m*c, m) times motion vector
__device__ __forceinline__ void inert_vec(float r[6], const float* in, const float* v) {
  r[0] = in[0] * v[0] + in[3] * v[1] + in[4] * v[2] - in[8] * v[4] + in[7] * v[5];
  r[1] = in[3] * v[0] + in[1] * v[1] + in[5] * v[2] + in[8] * v[3] - in[6] * v[5];
  r[2] = in[4] * v[0] + in[5] * v[1] + in[2] * v[2] - in[7] * v[3] + in[6] * v[4];
  r[3] = in[8] * v[1] - in[7] * v[2] + in[9] * v[3];
  r[4] = in[6] * v[2] - in[8] * v[0] + in[9] * v[4];
  r[5] = in[7] * v[0] - in[6] * v[1] + in[9] * v[5];
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

}  // namespace mjh
