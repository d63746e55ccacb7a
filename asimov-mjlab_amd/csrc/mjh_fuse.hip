// mjh_fuse.hip — fused reset-path / event / command kernels for the env layer
// (gfx950).
//
// The masked reset of a manager-based env (manager_based_rl_env.py:210-245 of
// the reference: events, then every manager's reset with its episode logs) is
// ~80 small torch launches per env step at 4096 envs, each a few microseconds
// of dispatch for microseconds of work. These kernels do each manager's (or
// event term's) whole masked update in one launch:
//   * masked column means (+ row clear) — RewardManager.reset episode sums,
//     CommandTerm.reset metrics;
//   * masked flag counts — TerminationManager.reset episode logs;
//   * uniform draws selected by a mask — interval-event and command timers;
//   * reset_root_state_uniform / reset_joints_by_offset /
//     push_by_setting_velocity (envs/mdp/events.py) with their EntityData
//     writes into qpos / qvel;
//   * UniformVelocityCommand resampling (velocity_command.py:103-123).
//
// Random draws come from a counter-based generator (splitmix64 finalizer over
// seed, call-site key, a device step counter and the element index): stateless,
// so the draws of a captured graph change with the step counter at every
// replay and no host RNG state is consumed inside the graph. Distributions are
// the reference's (U[lo, hi) per element); the stream is not torch's (the
// reference's stream is already not reproduced by mask-based resets).
#include <hip/hip_runtime.h>

#include "../../include/mjh_abi.h"
#include "mjh_batch.h"
#include "mjh_rng.h"

namespace {

constexpr int kBlock = 256;
inline int grid(long long n) { return (int)((n + kBlock - 1) / kBlock); }
int finish() { return hipGetLastError() == hipSuccess ? 0 : 2; }

using mjh::Rng;

__device__ __forceinline__ bool on(const unsigned char* mask, long long e) { return mask == nullptr || mask[e] != 0; }

// ---- rotations (formulas of mjh_envops.hip / utils/math.py) ------------------
__device__ __forceinline__ void qmul(float o[4], const float a[4], const float b[4]) {
  const float ww = (a[3] + a[1]) * (b[1] + b[2]);
  const float yy = (a[0] - a[2]) * (b[0] + b[3]);
  const float zz = (a[0] + a[2]) * (b[0] - b[3]);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (a[3] - a[1]) * (b[1] - b[2]));
  o[0] = qq - ww + (a[3] - a[2]) * (b[2] - b[3]);
  o[1] = qq - xx + (a[1] + a[0]) * (b[1] + b[0]);
  o[2] = qq - yy + (a[0] - a[1]) * (b[2] + b[3]);
  o[3] = qq - zz + (a[3] + a[2]) * (b[0] - b[1]);
}
__device__ __forceinline__ void qeuler(float o[4], float roll, float pitch, float yaw) {
  const float cy = cosf(yaw * 0.5f), sy = sinf(yaw * 0.5f);
  const float cr = cosf(roll * 0.5f), sr = sinf(roll * 0.5f);
  const float cp = cosf(pitch * 0.5f), sp = sinf(pitch * 0.5f);
  o[0] = cy * cr * cp + sy * sr * sp;
  o[1] = cy * sr * cp - sy * cr * sp;
  o[2] = cy * cr * sp + sy * sr * cp;
  o[3] = sy * cr * cp - cy * sr * sp;
}
// quat_apply_inverse(q, v)
__device__ __forceinline__ void qrot_inv(float o[3], const float q[4], const float v[3]) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  const float tx = 2.f * (y * v[2] - z * v[1]), ty = 2.f * (z * v[0] - x * v[2]), tz = 2.f * (x * v[1] - y * v[0]);
  o[0] = (v[0] - w * tx) + (y * tz - z * ty);
  o[1] = (v[1] - w * ty) + (z * tx - x * tz);
  o[2] = (v[2] - w * tz) + (x * ty - y * tx);
}

// ---- masked reductions (one workgroup; fixed summation order) ---------------
struct ColArgs {
  float* c[MJH_MAX_TERMS];
  long long cs[MJH_MAX_TERMS];
  int ncols;
};

// wave64 sum (all lanes get the total)
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kRedBlock = 1024;  // one workgroup of 16 waves per column

// blockIdx.x = column: masked row count and masked column sum (each thread
// accumulates rows tid, tid + 1024, ...), wave + LDS reduction; the column's
// masked rows are cleared when zero_rows. With no row masked, out[t] keeps its
// value: the reference writes its episode logs only from _reset_idx, which runs
// only when some env resets, so the log holds the last reset's values
// (manager_based_rl_env.py:133-135, 216-238)
__global__ __launch_bounds__(kRedBlock) void masked_means_kernel(const ColArgs a, const unsigned char* __restrict__ mask,
                                                                  float scale, int zero_rows, float* __restrict__ out,
                                                                  long long n) {
  __shared__ float part[2][kRedBlock / 64];
  const int t = blockIdx.x;
  float* const col = a.c[t];
  const long long cs = a.cs[t];
  float s = 0.f, cnt = 0.f;
  for (long long e = threadIdx.x; e < n; e += kRedBlock) {
    if (!on(mask, e)) continue;
    cnt += 1.f;
    s += col[e * cs];
    if (zero_rows) col[e * cs] = 0.f;
  }
  s = wsum(s);
  cnt = wsum(cnt);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][wv] = s;
    part[1][wv] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ts = 0.f, tc = 0.f;
#pragma unroll
    for (int w = 0; w < kRedBlock / 64; w++) {
      ts += part[0][w];
      tc += part[1][w];
    }
    if (tc > 0.f) out[t] = ts / tc * scale;
  }
}

struct FlagArgs {
  const unsigned char* f[MJH_MAX_TERMS];
  int nflags;
};

__global__ __launch_bounds__(kRedBlock) void masked_counts_kernel(const FlagArgs a, const unsigned char* __restrict__ mask,
                                                                   mjh_i64* __restrict__ out, long long n) {
  __shared__ int part[MJH_MAX_TERMS][kRedBlock / 64];
  __shared__ int any_masked;
  int acc[MJH_MAX_TERMS];
#pragma unroll
  for (int t = 0; t < MJH_MAX_TERMS; t++) acc[t] = 0;
  if (threadIdx.x == 0) any_masked = 0;
  __syncthreads();
  for (long long e = threadIdx.x; e < n; e += kRedBlock) {
    if (!on(mask, e)) continue;
    any_masked = 1;  // benign race: every writer stores 1
#pragma unroll
    for (int t = 0; t < MJH_MAX_TERMS; t++)
      if (t < a.nflags) acc[t] += a.f[t][e] ? 1 : 0;
  }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < MJH_MAX_TERMS; t++) {
    if (t < a.nflags) {
      int v = acc[t];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) part[t][wv] = v;
    }
  }
  __syncthreads();
  if (any_masked && threadIdx.x < (unsigned)a.nflags) {  // no env masked: keep the last counts
    long long s = 0;
#pragma unroll
    for (int w = 0; w < kRedBlock / 64; w++) s += part[threadIdx.x][w];
    out[threadIdx.x] = s;
  }
}

// ---- masked draws -------------------------------------------------------------
__global__ void uniform_draws_kernel(float* __restrict__ out, long long n, unsigned long long seed,
                                     unsigned long long key, const mjh_i64* ctr) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = Rng(seed, key, ctr).u01(i);
}

struct UniformWhereJob {
  static constexpr int kKind = 120;
  float* t; const unsigned char* mask; float lo; float hi; unsigned long long seed; unsigned long long key;
  const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    if (on(mask, e)) t[e] = Rng(seed, key, ctr).u01(e) * (hi - lo) + lo;
  }
};

// interval event timers (event_manager.py:120-145): t -= dt; due = t < 1e-6;
// due timers are redrawn from U[lo, hi)
struct IntervalTickJob {
  static constexpr int kKind = 110;
  float* t; float dt; float lo; float hi; unsigned char* due; unsigned long long seed; unsigned long long key;
  const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    const float v = t[e] - dt;
    const bool d = v < 1e-6f;
    t[e] = d ? Rng(seed, key, ctr).u01(e) * (hi - lo) + lo : v;
    due[e] = d ? 1 : 0;
  }
};

// ---- event terms ----------------------------------------------------------------
struct Range6 {
  float lo[6], hi[6];
};

// reset_root_state_uniform (envs/mdp/events.py:45-84): draws u[e, 0:6] for the
// pose, u[e, 6:12] for the velocity (element index e * 12 + j)
struct ResetRootJob {
  static constexpr int kKind = 121;
  float* qpos; long long qs; int qadr; float* qvel; long long vs; int vadr; const unsigned char* mask;
  const float* rs; long long rss; const float* org; long long os; Range6 pose; Range6 vel; int pose_rand; int vel_rand;
  unsigned long long seed; unsigned long long key; const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    if (!on(mask, e)) return;
    const Rng rng(seed, key, ctr);
    const float* r = rs + e * rss;
    float p6[6], v6[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      p6[j] = pose_rand ? rng.u01(e * 12 + j) * (pose.hi[j] - pose.lo[j]) + pose.lo[j] : 0.f;
      v6[j] = vel_rand ? rng.u01(e * 12 + 6 + j) * (vel.hi[j] - vel.lo[j]) + vel.lo[j] : 0.f;
    }
    float qe[4], q[4];
    qeuler(qe, p6[3], p6[4], p6[5]);
    const float q0[4] = {r[3], r[4], r[5], r[6]};
    qmul(q, q0, qe);
    float* qp = qpos + e * qs + qadr;
    const float* o = org + e * os;
    qp[0] = r[0] + p6[0] + o[0];
    qp[1] = r[1] + p6[1] + o[1];
    qp[2] = r[2] + p6[2] + o[2];
    qp[3] = q[0]; qp[4] = q[1]; qp[5] = q[2]; qp[6] = q[3];
    // write_root_link_velocity: linear in the world frame, angular in the new body frame
    const float w[3] = {r[10] + v6[3], r[11] + v6[4], r[12] + v6[5]};
    float wb[3];
    qrot_inv(wb, q, w);
    float* qv = qvel + e * vs + vadr;
    qv[0] = r[7] + v6[0]; qv[1] = r[8] + v6[1]; qv[2] = r[9] + v6[2];
    qv[3] = wb[0]; qv[4] = wb[1]; qv[5] = wb[2];
  }
};

// reset_joints_by_offset (envs/mdp/events.py:87-121) for k consecutive joints:
// draws u[e, 0:k] position offsets, u[e, k:2k] velocity offsets
// the per-joint kernel below as a per-env job (sequential batches): the same
// element arithmetic for j = 0..k-1
struct ResetJointsJob {
  static constexpr int kKind = 122;
  float* qpos; long long qs; int qadr; float* qvel; long long vs; int vadr; int k; const unsigned char* mask;
  const float* dp; long long dps; const float* dv; long long dvs; const float* lim; long long ls; float plo; float phi;
  float vlo; float vhi; int prand; int vrand; unsigned long long seed; unsigned long long key; const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    if (!on(mask, e)) return;
    const Rng rng(seed, key, ctr);
    for (int j = 0; j < k; j++) {
      float p = dp[e * dps + j];
      if (prand) p += rng.u01(e * 2 * k + j) * (phi - plo) + plo;
      const float* l = lim + e * ls + 2 * j;
      p = fminf(fmaxf(p, l[0]), l[1]);
      float v = dv[e * dvs + j];
      if (vrand) v += rng.u01(e * 2 * k + k + j) * (vhi - vlo) + vlo;
      qpos[e * qs + qadr + j] = p;
      qvel[e * vs + vadr + j] = v;
    }
  }
};
__global__ void reset_joints_offset_kernel(float* __restrict__ qpos, long long qs, int qadr, float* __restrict__ qvel,
                                           long long vs, int vadr, int k, const unsigned char* __restrict__ mask,
                                           const float* __restrict__ dp, long long dps, const float* __restrict__ dv,
                                           long long dvs, const float* __restrict__ lim, long long ls, float plo,
                                           float phi, float vlo, float vhi, int prand, int vrand,
                                           unsigned long long seed, unsigned long long key, const mjh_i64* ctr,
                                           long long n) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * k) return;
  const long long e = t / k;
  const int j = (int)(t - e * k);
  if (!on(mask, e)) return;
  const Rng rng(seed, key, ctr);
  float p = dp[e * dps + j];
  if (prand) p += rng.u01(e * 2 * k + j) * (phi - plo) + plo;
  const float* l = lim + e * ls + 2 * j;
  p = fminf(fmaxf(p, l[0]), l[1]);
  float v = dv[e * dvs + j];
  if (vrand) v += rng.u01(e * 2 * k + k + j) * (vhi - vlo) + vlo;
  qpos[e * qs + qadr + j] = p;
  qvel[e * vs + vadr + j] = v;
}

// push_by_setting_velocity (envs/mdp/events.py:124-137): root_link_vel_w + U6,
// written as the free joint's qvel (angular part into the body frame)
struct PushVelocityJob {
  static constexpr int kKind = 111;
  const float* qpos; long long qs; int qadr; float* qvel; long long vs; int vadr; const unsigned char* mask;
  const float* vw; long long vws; Range6 r; unsigned long long seed; unsigned long long key; const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    if (!on(mask, e)) return;
    const Rng rng(seed, key, ctr);
    const float* v = vw + e * vws;
    float u[6];
#pragma unroll
    for (int j = 0; j < 6; j++) u[j] = v[j] + (rng.u01(e * 6 + j) * (r.hi[j] - r.lo[j]) + r.lo[j]);
    const float* qp = qpos + e * qs + qadr;
    const float q[4] = {qp[3], qp[4], qp[5], qp[6]};
    float wb[3];
    qrot_inv(wb, q, u + 3);
    float* qv = qvel + e * vs + vadr;
    qv[0] = u[0]; qv[1] = u[1]; qv[2] = u[2];
    qv[3] = wb[0]; qv[4] = wb[1]; qv[5] = wb[2];
  }
};

// ---- command terms --------------------------------------------------------------
// CommandTerm.reset + UniformVelocityCommand._resample_command for the masked
// envs (command_manager.py:34-47, velocity_command.py:103-123): draws per env
// u[e, 0] timer, u[e, 1:5] lin_x / lin_y / ang_z / heading, u[e, 5] heading env,
// u[e, 6] standing env (element e * 8 + j). `reset` != 0: the counter restarts
// (masked_fill 0, then += 1), else it is incremented.
struct VelocityResampleJob {
  static constexpr int kKind = 123;
  const unsigned char* mask; const float* ranges; float t_lo; float t_hi; float rel_heading; float rel_standing;
  int heading_command; int reset; float* cmd; float* heading_target; unsigned char* is_heading; unsigned char* is_standing;
  float* time_left; mjh_i64* counter; unsigned long long seed; unsigned long long key; const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    if (!on(mask, e)) return;
    const Rng rng(seed, key, ctr);
    const long long b = e * 8;
    time_left[e] = rng.u01(b) * (t_hi - t_lo) + t_lo;
#pragma unroll
    for (int j = 0; j < 3; j++) cmd[e * 3 + j] = rng.u01(b + 1 + j) * (ranges[2 * j + 1] - ranges[2 * j]) + ranges[2 * j];
    if (heading_command) {
      heading_target[e] = rng.u01(b + 4) * (ranges[7] - ranges[6]) + ranges[6];
      is_heading[e] = rng.u01(b + 5) <= rel_heading ? 1 : 0;
    }
    is_standing[e] = rng.u01(b + 6) <= rel_standing ? 1 : 0;
    counter[e] = reset ? 1 : counter[e] + 1;
  }
};

// EventManager reset bookkeeping (event_manager.py:146-156): last = step, once = 1
struct EventMarkJob {
  static constexpr int kKind = 124;
  static constexpr int kFlags = mjh_batch::kReadsCounter;  // reads the step counter
  int* last; unsigned char* once; const unsigned char* mask; const mjh_i64* step;
  __device__ __forceinline__ void run(long long e) const {
    if (!on(mask, e)) return;
    last[e] = step ? (int)*step : 0;
    once[e] = 1;
  }
};

// TerminationManager.compute's combination (termination_manager.py:54-82):
// per-term done flags copied out, OR-ed into truncated (time-out terms) or
// terminated, dones = truncated | terminated
struct TermArgs {
  const unsigned char* v[MJH_MAX_TERMS];
  unsigned char* d[MJH_MAX_TERMS];
  int time_out[MJH_MAX_TERMS];
  int nterms;
};

// bad_orientation (envs/mdp/terminations.py): acos(-g_z) > limit as
// -cos(limit) < g_z <= 1, one launch (instead of two compares and an AND)
struct GzAboveJob {
  static constexpr int kKind = 112;
  const float* g; long long gs; float thr; unsigned char* out;
  __device__ __forceinline__ void run(long long e) const {
    const float gz = g[e * gs];
    out[e] = (gz > thr && gz <= 1.f) ? 1 : 0;
  }
};
// time_out (envs/mdp/terminations.py): episode_length >= max
struct TimeOutJob {
  static constexpr int kKind = 113;
  const mjh_i64* len; mjh_i64 max_len; unsigned char* out;
  __device__ __forceinline__ void run(long long e) const { out[e] = len[e] >= max_len ? 1 : 0; }
};

// the combine for up to 6 terms as a batchable job (the kernel below takes any number)
struct TermCombineJob {
  static constexpr int kKind = 114;
  const unsigned char* v[6]; unsigned char* d[6]; int time_out_mask; int nterms;
  unsigned char* truncated; unsigned char* terminated; unsigned char* dones;
  __device__ __forceinline__ void run(long long e) const {
    unsigned char tr = 0, te = 0;
#pragma unroll
    for (int t = 0; t < 6; t++) {
      if (t < nterms) {
        const unsigned char x = v[t][e] ? 1 : 0;
        d[t][e] = x;
        if ((time_out_mask >> t) & 1) tr |= x;
        else te |= x;
      }
    }
    truncated[e] = tr;
    terminated[e] = te;
    dones[e] = tr | te;
  }
};
__global__ void term_combine_kernel(const TermArgs a, unsigned char* __restrict__ truncated,
                                    unsigned char* __restrict__ terminated, unsigned char* __restrict__ dones, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  unsigned char tr = 0, te = 0;
#pragma unroll
  for (int t = 0; t < MJH_MAX_TERMS; t++) {
    if (t < a.nterms) {
      const unsigned char v = a.v[t][e] ? 1 : 0;
      a.d[t][e] = v;
      if (a.time_out[t]) tr |= v;
      else te |= v;
    }
  }
  truncated[e] = tr;
  terminated[e] = te;
  dones[e] = tr | te;
}

// compute_velocity_from_cvel (entity/data.py:25-30 of the reference restated)
// for k rows per env read in place: point j of env e at pos + e*pes + j*prs,
// its body's cvel at cvel + e*ves + 6*body[j], the root subtree com at
// com + e*cs; out (n*k, 6) = [lin - ang x (com - pos), ang]
__global__ void velocity_rows_kernel(const float* __restrict__ pos, long long pes, long long prs,
                                     const float* __restrict__ com, long long cs, const float* __restrict__ cvel,
                                     long long ves, const int* __restrict__ body, float* __restrict__ out, int k,
                                     long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * k) return;
  const long long e = i / k;
  const int j = (int)(i - e * k);
  const float* p = pos + e * pes + j * prs;
  const float* c = com + e * cs;
  const float* v = cvel + e * ves + 6ll * body[j];
  const float ox = c[0] - p[0], oy = c[1] - p[1], oz = c[2] - p[2];
  const float ax = v[0], ay = v[1], az = v[2];
  float* o = out + 6 * i;
  o[0] = v[3] - (ay * oz - az * oy);
  o[1] = v[4] - (az * ox - ax * oz);
  o[2] = v[5] - (ax * oy - ay * ox);
  o[3] = ax; o[4] = ay; o[5] = az;
}

// zero the rows of several float tensors where mask (one launch for a
// manager's masked_fill_(mask, 0) chain): tensor t holds w[t] floats per row
struct ZeroArgs {
  float* p[MJH_MAX_TERMS];
  long long rs[MJH_MAX_TERMS];
  int w[MJH_MAX_TERMS];
  int ntensors, wmax;
};

// masked_zero for up to 6 tensors as a per-env job (sequential batches)
struct MaskedZeroJob {
  static constexpr int kKind = 125;
  float* p[6]; long long rs[6]; int w[6]; int nt; const unsigned char* mask;
  __device__ __forceinline__ void run(long long e) const {
    if (!on(mask, e)) return;
    for (int t = 0; t < nt; t++)
      for (int j = 0; j < w[t]; j++) p[t][e * rs[t] + j] = 0.f;
  }
};
// dst[e] = mask[e] ? src[e] : dst[e] (float); dst64[e] = mask[e] ? 0 : dst64[e] (int64)
struct MaskedCopyJob {
  static constexpr int kKind = 126;
  float* dst; const float* src; const unsigned char* mask;
  __device__ __forceinline__ void run(long long e) const {
    if (mask[e]) dst[e] = src[e];
  }
};
struct MaskedZeroI64Job {
  static constexpr int kKind = 127;
  mjh_i64* dst; const unsigned char* mask;
  __device__ __forceinline__ void run(long long e) const {
    if (mask[e]) dst[e] = 0;
  }
};
__global__ void masked_zero_kernel(const ZeroArgs a, const unsigned char* __restrict__ mask, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int t = blockIdx.y;
  if (i >= n * a.wmax || t >= a.ntensors) return;
  const long long e = i / a.wmax;
  const int j = (int)(i - e * a.wmax);
  if (j < a.w[t] && on(mask, e)) a.p[t][e * a.rs[t] + j] = 0.f;
}

// sum(num[t]) / max(sum(den[t]), 1) over all envs (the per-step metric logs of
// the reward terms, e.g. rewards.py Metrics/*_mean); one workgroup
struct RatioArgs {
  const float* num[MJH_MAX_TERMS];
  const float* den[MJH_MAX_TERMS];
  int nterms;
};

// blockIdx.x = term
__global__ __launch_bounds__(1024) void sum_ratios_kernel(const RatioArgs a, float* __restrict__ out, long long n) {
  __shared__ float part[2][16];
  const int t = blockIdx.x;
  float x = 0.f, y = 0.f;
  // den NULL: mean(sqrt(num)) (e.g. Metrics/angular_momentum_mean)
  const float* dn = a.den[t];
  for (long long e = threadIdx.x; e < n; e += 1024) {
    x += dn ? a.num[t][e] : sqrtf(a.num[t][e]);
    y += dn ? dn[e] : 1.f;
  }
  x = wsum(x);
  y = wsum(y);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][wv] = x;
    part[1][wv] = y;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sx = 0.f, sy = 0.f;
    for (int w = 0; w < 16; w++) {
      sx += part[0][w];
      sy += part[1][w];
    }
    out[t] = sx / fmaxf(sy, 1.f);
  }
}

// ---- contact-timing rewards of the velocity task (tasks/velocity/mdp/rewards.py)
// One thread per env over its k feet; `cmd` NULL = no command gating, else the
// term is multiplied by (|cmd_xy| + |cmd_yaw| > cmd_thr). num/den: per-env
// parts of the term's metric log (sum(num) / max(sum(den), 1), mjh_sum_ratios).
__device__ __forceinline__ float cmd_active(const float* cmd, long long cs, long long e, float thr) {
  if (!cmd) return 1.f;
  const float* c = cmd + e * cs;
  return (sqrtf(c[0] * c[0] + c[1] * c[1]) + fabsf(c[2])) > thr ? 1.f : 0.f;
}

// the contact-timing reward terms as batchable jobs (mjh_batch.h; run(e) is
// the term for env e)
// feet_air_time: sum((t > tmin) & (t < tmax)) * active; log air_time_mean
struct AirTimeJob {
  static constexpr int kKind = 101;
  const float* t; long long ts; const float* cmd; long long cs; float tmin; float tmax; float cmd_thr;
  float* out; float* num; float* den; int k;
  __device__ __forceinline__ void run(long long e) const {
    float r = 0.f, a = 0.f, b = 0.f;
    for (int j = 0; j < k; j++) {
      const float x = t[e * ts + j];
      r += (x > tmin && x < tmax) ? 1.f : 0.f;
      const float in_air = x > 0.f ? 1.f : 0.f;
      a += x * in_air;
      b += in_air;
    }
    out[e] = r * cmd_active(cmd, cs, e, cmd_thr);
    num[e] = a;
    den[e] = b;
  }
};

// feet_swing_height: peak = in_air ? max(peak, h) : peak; first contact =
// 0 < contact_time < first_lim; cost = sum((peak / target - 1)^2 * first) *
// active; log peak_height_mean; peak cleared where first
struct SwingHeightJob {
  static constexpr int kKind = 102;
  float* peak; const float* h; long long hes; long long hcs; const float* found; long long fes; long long fcs;
  const float* cct; long long cts; const float* cmd; long long cs; float first_lim; float target; float cmd_thr;
  float* out; float* num; float* den; int k;
  __device__ __forceinline__ void run(long long e) const {
    float c = 0.f, a = 0.f, b = 0.f;
    for (int j = 0; j < k; j++) {
      float p = peak[e * k + j];
      if (found[e * fes + j * fcs] == 0.f) p = fmaxf(p, h[e * hes + j * hcs]);
      const float ct = cct[e * cts + j];
      const float first = (ct > 0.f && ct < first_lim) ? 1.f : 0.f;
      const float err = p / target - 1.f;
      c += err * err * first;
      a += p * first;
      b += first;
      peak[e * k + j] = first != 0.f ? 0.f : p;
    }
    out[e] = c * cmd_active(cmd, cs, e, cmd_thr);
    num[e] = a;
    den[e] = b;
  }
};

// soft_landing: sum(|force| * first) * active; log landing_force_mean
struct SoftLandingJob {
  static constexpr int kKind = 103;
  const float* f; long long fes; long long fss; const float* cct; long long cts; const float* cmd; long long cs;
  float first_lim; float cmd_thr; float* out; float* num; float* den; int k;
  __device__ __forceinline__ void run(long long e) const {
    float c = 0.f, b = 0.f;
    for (int j = 0; j < k; j++) {
      const float* v = f + e * fes + j * fss;
      const float ct = cct[e * cts + j];
      const float first = (ct > 0.f && ct < first_lim) ? 1.f : 0.f;
      c += sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) * first;
      b += first;
    }
    out[e] = c * cmd_active(cmd, cs, e, cmd_thr);
    num[e] = c;
    den[e] = b;
  }
};


// ActionManager.process_action with one JointAction term (action_manager.py:
// 107-116, joint_actions.py:90-108): prev = action; action = raw = input;
// processed = raw * scale + offset (scale / offset: per-column rows, or the
// scalars when the pointer is NULL)
__global__ void joint_action_kernel(const float* __restrict__ input, long long is, float* __restrict__ action,
                                    float* __restrict__ prev, float* __restrict__ raw, float* __restrict__ processed,
                                    const float* __restrict__ scale, long long ss, float scale0,
                                    const float* __restrict__ offset, long long os, float offset0, int d, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * d) return;
  const long long e = i / d;
  const int j = (int)(i - e * d);
  const float a = input[e * is + j];
  prev[i] = action[i];
  action[i] = a;
  raw[i] = a;
  const float sc = scale ? scale[e * ss + j] : scale0;
  const float of = offset ? offset[e * os + j] : offset0;
  processed[i] = fmaf(a, sc, of);
}

// The root body's frame quantities EntityData derives from one forward pass
// (entity/data.py): out[e] = [root_link_vel_w (lin, ang) 6 | lin_vel_b 3 |
// ang_vel_b 3 | projected_gravity_b 3 | heading_w 1]; quaternion rotations as
// quat_apply(_inverse) (utils/math.py), velocity as compute_velocity_from_cvel
__device__ __forceinline__ void qrot(float o[3], const float q[4], const float v[3], float sgn) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  const float tx = 2.f * (y * v[2] - z * v[1]), ty = 2.f * (z * v[0] - x * v[2]), tz = 2.f * (x * v[1] - y * v[0]);
  o[0] = (v[0] + sgn * w * tx) + (y * tz - z * ty);
  o[1] = (v[1] + sgn * w * ty) + (z * tx - x * tz);
  o[2] = (v[2] + sgn * w * tz) + (x * ty - y * tx);
}

struct RootFrameJob {
  static constexpr int kKind = 115;
  static constexpr int kFlags = mjh_batch::kProducer;  // read by reward / termination jobs and torch in the same pass
  const float* xpos; long long ps; const float* xquat; long long qs; const float* com; long long cs;
  const float* cvel; long long vs; const float* grav; long long gs; const float* fwd; long long fs; float* out;
  __device__ __forceinline__ void run(long long e) const {
    const float* p = xpos + e * ps;
    const float* c = com + e * cs;
    const float* v = cvel + e * vs;
    const float q[4] = {xquat[e * qs], xquat[e * qs + 1], xquat[e * qs + 2], xquat[e * qs + 3]};
    const float ox = c[0] - p[0], oy = c[1] - p[1], oz = c[2] - p[2];
    const float ang[3] = {v[0], v[1], v[2]};
    const float lin[3] = {v[3] - (ang[1] * oz - ang[2] * oy), v[4] - (ang[2] * ox - ang[0] * oz), v[5] - (ang[0] * oy - ang[1] * ox)};
    float* o = out + 16 * e;
    o[0] = lin[0]; o[1] = lin[1]; o[2] = lin[2];
    o[3] = ang[0]; o[4] = ang[1]; o[5] = ang[2];
    qrot(o + 6, q, lin, -1.f);
    qrot(o + 9, q, ang, -1.f);
    const float g[3] = {grav[e * gs], grav[e * gs + 1], grav[e * gs + 2]};
    qrot(o + 12, q, g, -1.f);
    const float f0[3] = {fwd[e * fs], fwd[e * fs + 1], fwd[e * fs + 2]};
    float f[3];
    qrot(f, q, f0, 1.f);
    o[15] = atan2f(f[1], f[0]);
  }
};

// World order for the step kernel's workgroups (mjh_data.world_order): worlds
// bucketed by their previous step's cost (solver_niter + 2) * nefc, most
// expensive first (counting sort, one workgroup), so the 8 worlds sharing a
// workgroup's LDS take similar time. Within a bucket the order is arbitrary:
// results do not depend on it.
constexpr int kOrderBuckets = 256;

__global__ __launch_bounds__(1024) void order_worlds_kernel(const int* __restrict__ niter, const int* __restrict__ nefc,
                                                           long long* __restrict__ order, long long n) {
  __shared__ int cnt[kOrderBuckets];
  __shared__ int base[kOrderBuckets];
  for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const int key = (niter[e] + 2) * nefc[e];
    const int b = kOrderBuckets - 1 - min(key >> 4, kOrderBuckets - 1);  // descending cost
    atomicAdd(&cnt[b], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < kOrderBuckets; b++) {
      base[b] = acc;
      acc += cnt[b];
    }
  }
  __syncthreads();
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const int key = (niter[e] + 2) * nefc[e];
    const int b = kOrderBuckets - 1 - min(key >> 4, kOrderBuckets - 1);
    order[atomicAdd(&base[b], 1)] = e;
  }
}

// ---- motion tracking command (tasks/tracking/mdp/commands.py) -------------------
constexpr int kMaxBins = 4096;

// MotionCommand._adaptive_sampling for the envs in mask, one workgroup:
// failed-bin histogram (kept only when some resampled env failed), sampling
// probabilities p = smooth(bin_failed + ratio / B) / sum, time steps drawn by
// inverse CDF (draws e*2, e*2+1 of the stream), and the sampling metrics
// (entropy, top-1 probability, top-1 bin) written to every env when some env
// resampled (commands.py:258-307)
__global__ __launch_bounds__(1024) void motion_adaptive_kernel(
    const unsigned char* __restrict__ mask, const unsigned char* __restrict__ terminated, long long* __restrict__ ts,
    const float* __restrict__ bin_failed, float* __restrict__ cur_failed, const float* __restrict__ kern, int B, int K,
    long long T, float ratio, float* __restrict__ m_entropy, float* __restrict__ m_top1p, float* __restrict__ m_top1b,
    unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n) {
  __shared__ float p[kMaxBins];
  __shared__ float cdf[kMaxBins];
  __shared__ int hist[kMaxBins];
  __shared__ int anyfail, anymask;
  __shared__ float H, pmax, imax;
  for (int b = threadIdx.x; b < B; b += blockDim.x) hist[b] = 0;
  if (threadIdx.x == 0) anyfail = anymask = 0;
  __syncthreads();
  const long long Tc = T > 1 ? T : 1;
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const bool m = mask[e] != 0;
    if (m) anymask = 1;
    if (m && terminated[e]) {
      long long b = (ts[e] * B) / Tc;
      b = b < 0 ? 0 : (b > B - 1 ? B - 1 : b);
      atomicAdd(&hist[b], 1);
      anyfail = 1;
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if (anyfail) cur_failed[b] = (float)hist[b];
    p[b] = bin_failed[b] + ratio / (float)B;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    float v = 0.f;
    for (int k = 0; k < K; k++) v += p[min(b + k, B - 1)] * kern[k];
    cdf[b] = v;  // smoothed, unnormalised
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; b++) s += cdf[b];
    float c = 0.f, h = 0.f, mx = -1.f;
    int im = 0;
    for (int b = 0; b < B; b++) {
      const float q = cdf[b] / s;
      p[b] = q;
      c += q;
      cdf[b] = c;
      h -= q * logf(q + 1e-12f);
      if (q > mx) { mx = q; im = b; }
    }
    H = h;
    pmax = mx;
    imax = (float)im;
  }
  __syncthreads();
  const Rng rng(seed, key, ctr);
  const float total = cdf[B - 1];
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    if (mask[e]) {
      const float target = rng.u01(2 * e) * total;
      int lo = 0, hi = B;  // first b with cdf[b] > target (searchsorted right)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] <= target) lo = mid + 1; else hi = mid;
      }
      const int bin = lo > B - 1 ? B - 1 : lo;
      ts[e] = (long long)(((float)bin + rng.u01(2 * e + 1)) / (float)B * (float)(T - 1));
    }
    if (anymask) {
      m_entropy[e] = H / logf((float)B);
      m_top1p[e] = pmax;
      m_top1b[e] = imax / (float)B;
    }
  }
}

// MotionCommand._refresh_frame: frame[e] = table[ts[e]]; body_pos_w = the
// frame's body positions + env origin (commands.py:134-181)
__global__ void motion_frame_kernel(const float* __restrict__ table, const long long* __restrict__ ts,
                                    float* __restrict__ frame, int W, int pos_off, int nb, float* __restrict__ body_pos_w,
                                    const float* __restrict__ org, long long os, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * W) return;
  const long long e = i / W;
  const int c = (int)(i - e * W);
  const float v = table[ts[e] * W + c];
  frame[i] = v;
  const int r = c - pos_off;
  if (r >= 0 && r < 3 * nb) body_pos_w[e * 3 * nb + r] = v + org[e * os + r % 3];
}

// MotionCommand._resample_command's state write for the masked envs
// (commands.py:309-375): root = reference root + pose offsets (U[pose], draws
// e*S + 0..5; quat = euler(offset) (x) reference quat), velocity + U[vel] (e*S +
// 6..11), joints = reference + U[jlo, jhi) (e*S + 12 + j) clipped to the soft
// limits, joint velocities = reference; written as EntityData root/joint state
// (angular velocity into the new body frame); S = 12 + nj
__global__ void motion_reset_kernel(const float* __restrict__ frame, long long fs, int nj, int pos_off, int quat_off,
                                    int lin_off, int ang_off, const float* __restrict__ body_pos_w, long long bps,
                                    const unsigned char* __restrict__ mask, const Range6 pose, const Range6 vel,
                                    int pose_any, int vel_any, float jlo, float jhi, const float* __restrict__ lim,
                                    long long ls, float* __restrict__ qpos, long long qs, int rq, int jq,
                                    float* __restrict__ qvel, long long vs, int rv, int jv, unsigned long long seed,
                                    unsigned long long key, const mjh_i64* ctr, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n || !mask[e]) return;
  const Rng rng(seed, key, ctr);
  const long long S = 12 + nj;
  const float* f = frame + e * fs;
  float pos[3] = {body_pos_w[e * bps], body_pos_w[e * bps + 1], body_pos_w[e * bps + 2]};
  float q[4] = {f[quat_off], f[quat_off + 1], f[quat_off + 2], f[quat_off + 3]};
  float lin[3] = {f[lin_off], f[lin_off + 1], f[lin_off + 2]};
  float ang[3] = {f[ang_off], f[ang_off + 1], f[ang_off + 2]};
  if (pose_any) {
    float r[6];
    for (int j = 0; j < 6; j++) r[j] = rng.u01(e * S + j) * (pose.hi[j] - pose.lo[j]) + pose.lo[j];
    pos[0] += r[0]; pos[1] += r[1]; pos[2] += r[2];
    float qe[4], q2[4];
    qeuler(qe, r[3], r[4], r[5]);
    qmul(q2, qe, q);
    q[0] = q2[0]; q[1] = q2[1]; q[2] = q2[2]; q[3] = q2[3];
  }
  if (vel_any) {
    float r[6];
    for (int j = 0; j < 6; j++) r[j] = rng.u01(e * S + 6 + j) * (vel.hi[j] - vel.lo[j]) + vel.lo[j];
    lin[0] += r[0]; lin[1] += r[1]; lin[2] += r[2];
    ang[0] += r[3]; ang[1] += r[4]; ang[2] += r[5];
  }
  float* qp = qpos + e * qs;
  float* qv = qvel + e * vs;
  for (int j = 0; j < nj; j++) {
    float v = f[j] + (rng.u01(e * S + 12 + j) * (jhi - jlo) + jlo);
    const float* l = lim + e * ls + 2 * j;
    v = fminf(fmaxf(v, l[0]), l[1]);
    qp[jq + j] = v;
    qv[jv + j] = f[nj + j];
  }
  qp[rq] = pos[0]; qp[rq + 1] = pos[1]; qp[rq + 2] = pos[2];
  qp[rq + 3] = q[0]; qp[rq + 4] = q[1]; qp[rq + 5] = q[2]; qp[rq + 6] = q[3];
  float wb[3];
  qrot_inv(wb, q, ang);
  qv[rv] = lin[0]; qv[rv + 1] = lin[1]; qv[rv + 2] = lin[2];
  qv[rv + 3] = wb[0]; qv[rv + 4] = wb[1]; qv[rv + 5] = wb[2];
}

// |axis_angle_from_quat(a (x) conj(b))| (quat_error_magnitude, utils/math.py;
// the formula of mjh_envops.hip)
__device__ __forceinline__ float quat_err(const float* a, const float* b) {
  const float bc[4] = {b[0], -b[1], -b[2], -b[3]};
  float q[4];
  qmul(q, a, bc);
  const float sg = q[0] < 0.f ? -1.f : 1.f;
  const float w = q[0] * sg, x = q[1] * sg, y = q[2] * sg, z = q[3] * sg;
  const float mag = sqrtf(x * x + y * y + z * z);
  const float half = atan2f(mag, w);
  const float ang = 2.f * half;
  const float s = fabsf(ang) > 1e-6f ? sinf(half) / ang : 0.5f - ang * ang / 48.f;
  const float ax = x / s, ay = y / s, az = z / s;
  return sqrtf(ax * ax + ay * ay + az * az);
}

// Gaussian tracking rewards (tasks/tracking/mdp/rewards.py): out[e] =
// exp(-mean_j err_j * inv_std2) over k rows, row j of a at a + e*aes +
// ra[j]*ars (ra NULL: j), likewise b; err_j = sum_c (a - b)^2 over d columns
// (quat = 0), or quat_error_magnitude(a_j, b_j)^2 (quat != 0)
__global__ void rew_exp_err_kernel(const float* __restrict__ a, long long aes, long long ars, const int* __restrict__ ra,
                                   const float* __restrict__ b, long long bes, long long brs, const int* __restrict__ rb,
                                   int k, int d, int quat, float inv_std2, float* __restrict__ out, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float s = 0.f;
  for (int j = 0; j < k; j++) {
    const float* x = a + e * aes + (long long)(ra ? ra[j] : j) * ars;
    const float* y = b + e * bes + (long long)(rb ? rb[j] : j) * brs;
    if (quat) {
      const float q = quat_err(x, y);
      s += q * q;
    } else {
      for (int c = 0; c < d; c++) s += (x[c] - y[c]) * (x[c] - y[c]);
    }
  }
  out[e] = expf(-(s / (float)k) * inv_std2);
}

// env-step bookkeeping (manager_based_rl_env.py:111-152): every episode
// length += 1 and the env-step counter += 1 (the device random stream's counter)
struct StepCountersJob {
  static constexpr int kKind = 116;
  static constexpr int kFlags = mjh_batch::kWritesCounter;  // thread 0 advances the step counter
  mjh_i64* episode_length; mjh_i64* step;
  __device__ __forceinline__ void run(long long e) const {
    episode_length[e] += 1;
    if (e == 0 && step) *step += 1;
  }
};

// after the terminations: any_reset = any(reset); stats[0] += count(reset),
// stats[1] += any_reset (the gated forward's decision and its counters); one workgroup
__global__ __launch_bounds__(1024) void reset_stats_kernel(const unsigned char* __restrict__ reset,
                                                          unsigned char* __restrict__ any_reset, mjh_i64* __restrict__ stats,
                                                          long long n) {
  __shared__ int part[16];
  int c = 0;
  for (long long e = threadIdx.x; e < n; e += 1024) c += reset[e] ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < 16; w++) t += part[w];
    any_reset[0] = t > 0 ? 1 : 0;
    stats[0] += t;
    stats[1] += t > 0 ? 1 : 0;
  }
}

// ---- UniformVelocityCommand.compute (velocity_command.py:65-101 and
// command_manager.py:53-67) for all envs in one launch: metric accumulation,
// timer countdown, masked resampling from u (N, 8) uniform draws
// [timer, lin_x, lin_y, ang_z, heading, heading-env, standing-env, unused],
// heading control and standing override.

__device__ __forceinline__ float wrap_to_pi_f(float a) {
  const float two_pi = 6.283185307179586f, pi = 3.141592653589793f;
  float r = fmodf(a, two_pi);  // torch.remainder: fmod, then shift into [0, 2pi)
  if (r != 0.f && r < 0.f) r += two_pi;
  return r > pi ? r - two_pi : r;
}

struct VelocityCommandJob {
  static constexpr int kKind = 20;
  const float* lin_b; long long ls; const float* ang_b; long long as; const float* root_q; long long qs;
  const float* u; long long us; const float* ranges; float dt; float inv_max_step; float t_lo; float t_hi;
  float rel_heading; float rel_standing; float stiffness; int heading_command; float* cmd; float* heading_target;
  float* heading_error; bool* is_heading; bool* is_standing; float* time_left; long long* counter; float* err_xy;
  float* err_yaw; unsigned long long seed; unsigned long long key; const mjh_i64* ctr;
  __device__ __forceinline__ void run(long long e) const {
    float* c = cmd + 3 * e;
    const float* lv = lin_b + e * ls;
    const float* av = ang_b + e * as;
    // _update_metrics (before the resample, on the previous command)
    const float dx = c[0] - lv[0], dy = c[1] - lv[1];
    err_xy[e] += sqrtf(dx * dx + dy * dy) * inv_max_step;
    err_yaw[e] += fabsf(c[2] - av[2]) * inv_max_step;
    // countdown + resample
    float tl = time_left[e] - dt;
    float ud[8];
    const float* ue = u ? u + e * us : ud;
    if (tl <= 0.f) {
      if (!u) {  // draws e*8 + j of the env's device stream (mjh_rng.h)
        const mjh::Rng rng(seed, key, ctr);
#pragma unroll
        for (int j = 0; j < 8; j++) ud[j] = rng.u01(8 * e + j);
      }
      tl = ue[0] * (t_hi - t_lo) + t_lo;
#pragma unroll
      for (int k = 0; k < 3; k++) c[k] = ue[1 + k] * (ranges[2 * k + 1] - ranges[2 * k]) + ranges[2 * k];
      if (heading_command) {
        heading_target[e] = ue[4] * (ranges[7] - ranges[6]) + ranges[6];
        is_heading[e] = ue[5] <= rel_heading;
      }
      is_standing[e] = ue[6] <= rel_standing;
      counter[e] += 1;
    }
    time_left[e] = tl;
    // _update_command
    if (heading_command) {
      const float* q = root_q + e * qs;
      const float w = q[0], x = q[1], y = q[2], z = q[3];
      // quat_apply(q, [1, 0, 0]) with the quat_rotate_kernel's operation order
      const float tx = 2.f * (y * 0.f - z * 0.f), ty = 2.f * (z * 1.f - x * 0.f), tz = 2.f * (x * 0.f - y * 1.f);
      const float fx = (1.f + w * tx) + (y * tz - z * ty);
      const float fy = (0.f + w * ty) + (z * tx - x * tz);
      const float herr = wrap_to_pi_f(heading_target[e] - atan2f(fy, fx));
      heading_error[e] = herr;
      if (is_heading[e]) c[2] = fminf(fmaxf(stiffness * herr, ranges[4]), ranges[5]);
    }
    if (is_standing[e]) c[0] = c[1] = c[2] = 0.f;
  }
};


// this file's batchable jobs (mjh_batch.h)
struct FuseJobs {
  __device__ static void run(const mjh_batch::Job& j, long long e) {
    mjh_run_as<AirTimeJob>(j, e) || mjh_run_as<SwingHeightJob>(j, e) || mjh_run_as<SoftLandingJob>(j, e) ||
        mjh_run_as<IntervalTickJob>(j, e) || mjh_run_as<PushVelocityJob>(j, e) || mjh_run_as<GzAboveJob>(j, e) ||
        mjh_run_as<TimeOutJob>(j, e) || mjh_run_as<TermCombineJob>(j, e) || mjh_run_as<RootFrameJob>(j, e) ||
        mjh_run_as<StepCountersJob>(j, e) || mjh_run_as<VelocityCommandJob>(j, e) || mjh_run_as<UniformWhereJob>(j, e) ||
        mjh_run_as<ResetRootJob>(j, e) || mjh_run_as<ResetJointsJob>(j, e) || mjh_run_as<VelocityResampleJob>(j, e) ||
        mjh_run_as<EventMarkJob>(j, e) || mjh_run_as<MaskedZeroJob>(j, e) || mjh_run_as<MaskedCopyJob>(j, e) ||
        mjh_run_as<MaskedZeroI64Job>(j, e);
  }
};
const bool kFuseRegistered = mjh_batch::register_unit(mjh_batch::kFuse, mjh_batch_launch<FuseJobs>);

template <class J>
int submit_job(const J& j, long long n, void* stream) {
  return mjh_batch::submit(mjh_batch::kFuse, j, n, (hipStream_t)stream, mjh_job_kernel<J>);
}
}  // namespace

extern "C" {

int mjh_masked_means(float* const* cols, const long long* strides, int ncols, const unsigned char* mask, float scale,
                     int zero_rows, float* out, long long n, void* stream) {
  if (ncols <= 0) return 0;
  if (ncols > MJH_MAX_TERMS) return 1;
  ColArgs a{};
  for (int t = 0; t < ncols; t++) {
    a.c[t] = cols[t];
    a.cs[t] = strides[t];
  }
  a.ncols = ncols;
  hipLaunchKernelGGL(masked_means_kernel, dim3(ncols), dim3(kRedBlock), 0, (hipStream_t)stream, a, mask, scale, zero_rows, out, n);
  return finish();
}

int mjh_masked_counts(const unsigned char* const* flags, int nflags, const unsigned char* mask, mjh_i64* out, long long n,
                      void* stream) {
  if (nflags <= 0) return 0;
  if (nflags > MJH_MAX_TERMS) return 1;
  FlagArgs a{};
  for (int t = 0; t < nflags; t++) a.f[t] = flags[t];
  a.nflags = nflags;
  hipLaunchKernelGGL(masked_counts_kernel, dim3(1), dim3(kRedBlock), 0, (hipStream_t)stream, a, mask, out, n);
  return finish();
}

int mjh_uniform_draws(float* out, long long n, unsigned long long seed, unsigned long long key, const mjh_i64* ctr,
                      void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(uniform_draws_kernel, dim3(grid(n)), dim3(kBlock), 0, (hipStream_t)stream, out, n, seed, key, ctr);
  return finish();
}

int mjh_uniform_where(float* t, const unsigned char* mask, float lo, float hi, unsigned long long seed,
                      unsigned long long key, const mjh_i64* ctr, long long n, void* stream) {
  return submit_job(UniformWhereJob{t, mask, lo, hi, seed, key, ctr}, n, stream);
}

int mjh_interval_tick(float* t, float dt, float lo, float hi, unsigned char* due, unsigned long long seed,
                      unsigned long long key, const mjh_i64* ctr, long long n, void* stream) {
  return submit_job(IntervalTickJob{t, dt, lo, hi, due, seed, key, ctr}, n, stream);
}

int mjh_reset_root_uniform(float* qpos, long long qs, int qadr, float* qvel, long long vs, int vadr,
                           const unsigned char* mask, const float* root_state, long long rss, const float* origins,
                           long long os, const float* pose_lo, const float* pose_hi, const float* vel_lo,
                           const float* vel_hi, int pose_rand, int vel_rand, unsigned long long seed,
                           unsigned long long key, const mjh_i64* ctr, long long n, void* stream) {
  Range6 p{}, v{};
  for (int j = 0; j < 6; j++) {
    p.lo[j] = pose_lo[j]; p.hi[j] = pose_hi[j];
    v.lo[j] = vel_lo[j]; v.hi[j] = vel_hi[j];
  }
  return submit_job(ResetRootJob{qpos, qs, qadr, qvel, vs, vadr, mask, root_state, rss, origins, os, p, v, pose_rand, vel_rand,
                                 seed, key, ctr}, n, stream);
}

int mjh_reset_joints_offset(float* qpos, long long qs, int qadr, float* qvel, long long vs, int vadr, int k,
                            const unsigned char* mask, const float* def_pos, long long dps, const float* def_vel,
                            long long dvs, const float* lim, long long ls, float pos_lo, float pos_hi, float vel_lo,
                            float vel_hi, int pos_rand, int vel_rand, unsigned long long seed, unsigned long long key,
                            const mjh_i64* ctr, long long n, void* stream) {
  if (n <= 0 || k <= 0) return 0;
  // inside a batch: a per-env job; otherwise one thread per (env, joint)
  const ResetJointsJob j{qpos, qs, qadr, qvel, vs, vadr, k, mask, def_pos, dps, def_vel, dvs, lim, ls, pos_lo, pos_hi, vel_lo,
                         vel_hi, pos_rand, vel_rand, seed, key, ctr};
  if (mjh_batch::add(mjh_batch::kFuse, ResetJointsJob::kKind, n, &j, sizeof(j), (hipStream_t)stream,
                     mjh_batch::job_flags<ResetJointsJob>()))
    return 0;
  hipLaunchKernelGGL(reset_joints_offset_kernel, dim3(grid(n * k)), dim3(kBlock), 0, (hipStream_t)stream, qpos, qs, qadr,
                     qvel, vs, vadr, k, mask, def_pos, dps, def_vel, dvs, lim, ls, pos_lo, pos_hi, vel_lo, vel_hi,
                     pos_rand, vel_rand, seed, key, ctr, n);
  return finish();
}

int mjh_push_velocity(const float* qpos, long long qs, int qadr, float* qvel, long long vs, int vadr,
                      const unsigned char* mask, const float* vel_w, long long vws, const float* lo, const float* hi,
                      unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n, void* stream) {
  Range6 r{};
  for (int j = 0; j < 6; j++) {
    r.lo[j] = lo[j];
    r.hi[j] = hi[j];
  }
  return submit_job(PushVelocityJob{qpos, qs, qadr, qvel, vs, vadr, mask, vel_w, vws, r, seed, key, ctr}, n, stream);
}

int mjh_velocity_resample(const unsigned char* mask, const float* ranges, float t_lo, float t_hi, float rel_heading,
                          float rel_standing, int heading_command, int reset, float* cmd, float* heading_target,
                          unsigned char* is_heading, unsigned char* is_standing, float* time_left, mjh_i64* counter,
                          unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n,
                          void* stream) {
  return submit_job(VelocityResampleJob{mask, ranges, t_lo, t_hi, rel_heading, rel_standing, heading_command, reset, cmd,
                                        heading_target, is_heading, is_standing, time_left, counter, seed, key, ctr}, n, stream);
}

int mjh_event_mark(int* last, unsigned char* once, const unsigned char* mask, const mjh_i64* step, long long n,
                   void* stream) {
  return submit_job(EventMarkJob{last, once, mask, step}, n, stream);
}

int mjh_gz_above(const float* g, long long gs, float thr, unsigned char* out, long long n, void* stream) {
  return submit_job(GzAboveJob{g, gs, thr, out}, n, stream);
}

int mjh_time_out(const mjh_i64* episode_length, long long max_len, unsigned char* out, long long n, void* stream) {
  return submit_job(TimeOutJob{episode_length, max_len, out}, n, stream);
}

int mjh_term_combine(const unsigned char* const* values, unsigned char* const* term_dones, const int* time_out, int nterms,
                     unsigned char* truncated, unsigned char* terminated, unsigned char* dones, long long n,
                     void* stream) {
  if (n <= 0) return 0;
  if (nterms > MJH_MAX_TERMS) return 1;
  if (nterms <= 6) {
    TermCombineJob j{};
    for (int t = 0; t < nterms; t++) {
      j.v[t] = values[t];
      j.d[t] = term_dones[t];
      j.time_out_mask |= time_out[t] ? 1 << t : 0;
    }
    j.nterms = nterms;
    j.truncated = truncated;
    j.terminated = terminated;
    j.dones = dones;
    return submit_job(j, n, stream);
  }
  TermArgs a{};
  for (int t = 0; t < nterms; t++) {
    a.v[t] = values[t];
    a.d[t] = term_dones[t];
    a.time_out[t] = time_out[t];
  }
  a.nterms = nterms;
  hipLaunchKernelGGL(term_combine_kernel, dim3(grid(n)), dim3(kBlock), 0, (hipStream_t)stream, a, truncated, terminated,
                     dones, n);
  return finish();
}

int mjh_velocity_rows(const float* pos, long long pes, long long prs, const float* com, long long cs, const float* cvel,
                      long long ves, const int* body, float* out, int k, long long n, void* stream) {
  if (n <= 0 || k <= 0) return 0;
  hipLaunchKernelGGL(velocity_rows_kernel, dim3(grid(n * k)), dim3(kBlock), 0, (hipStream_t)stream, pos, pes, prs, com, cs,
                     cvel, ves, body, out, k, n);
  return finish();
}

int mjh_masked_zero(float* const* ptrs, const long long* row_strides, const int* widths, int ntensors,
                    const unsigned char* mask, long long n, void* stream) {
  if (n <= 0 || ntensors <= 0) return 0;
  if (ntensors > MJH_MAX_TERMS) return 1;
  if (ntensors <= 6) {  // inside a batch: a per-env job
    MaskedZeroJob j{};
    for (int t = 0; t < ntensors; t++) {
      j.p[t] = ptrs[t];
      j.rs[t] = row_strides[t];
      j.w[t] = widths[t];
    }
    j.nt = ntensors;
    j.mask = mask;
    if (mjh_batch::add(mjh_batch::kFuse, MaskedZeroJob::kKind, n, &j, sizeof(j), (hipStream_t)stream,
                       mjh_batch::job_flags<MaskedZeroJob>()))
      return 0;
  }
  ZeroArgs a{};
  a.wmax = 0;
  for (int t = 0; t < ntensors; t++) {
    a.p[t] = ptrs[t];
    a.rs[t] = row_strides[t];
    a.w[t] = widths[t];
    if (widths[t] > a.wmax) a.wmax = widths[t];
  }
  a.ntensors = ntensors;
  hipLaunchKernelGGL(masked_zero_kernel, dim3(grid(n * a.wmax), ntensors), dim3(kBlock), 0, (hipStream_t)stream, a, mask, n);
  return finish();
}

int mjh_masked_copy(float* dst, const float* src, const unsigned char* mask, long long n, void* stream) {
  return submit_job(MaskedCopyJob{dst, src, mask}, n, stream);
}

int mjh_masked_zero_i64(mjh_i64* dst, const unsigned char* mask, long long n, void* stream) {
  return submit_job(MaskedZeroI64Job{dst, mask}, n, stream);
}

int mjh_sum_ratios(const float* const* num, const float* const* den, int nterms, float* out, long long n, void* stream) {
  if (n <= 0 || nterms <= 0) return 0;
  if (nterms > MJH_MAX_TERMS) return 1;
  RatioArgs a{};
  for (int t = 0; t < nterms; t++) {
    a.num[t] = num[t];
    a.den[t] = den[t];
  }
  a.nterms = nterms;
  hipLaunchKernelGGL(sum_ratios_kernel, dim3(nterms), dim3(1024), 0, (hipStream_t)stream, a, out, n);
  return finish();
}

int mjh_rew_air_time(const float* t, long long ts, const float* cmd, long long cs, float tmin, float tmax, float cmd_thr,
                     float* out, float* num, float* den, int k, long long n, void* stream) {
  return submit_job(AirTimeJob{t, ts, cmd, cs, tmin, tmax, cmd_thr, out, num, den, k}, n, stream);
}

int mjh_rew_swing_height(float* peak, const float* h, long long hes, long long hcs, const float* found, long long fes,
                         long long fcs, const float* cct, long long cts, const float* cmd, long long cs, float first_lim,
                         float target, float cmd_thr, float* out, float* num, float* den, int k, long long n,
                         void* stream) {
  return submit_job(SwingHeightJob{peak, h, hes, hcs, found, fes, fcs, cct, cts, cmd, cs, first_lim, target, cmd_thr, out, num,
                                   den, k}, n, stream);
}

int mjh_rew_soft_landing(const float* f, long long fes, long long fss, const float* cct, long long cts, const float* cmd,
                         long long cs, float first_lim, float cmd_thr, float* out, float* num, float* den, int k,
                         long long n, void* stream) {
  return submit_job(SoftLandingJob{f, fes, fss, cct, cts, cmd, cs, first_lim, cmd_thr, out, num, den, k}, n, stream);
}

int mjh_joint_action(const float* input, long long is, float* action, float* prev, float* raw, float* processed,
                     const float* scale, long long ss, float scale0, const float* offset, long long os, float offset0,
                     int d, long long n, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  hipLaunchKernelGGL(joint_action_kernel, dim3(grid(n * d)), dim3(kBlock), 0, (hipStream_t)stream, input, is, action, prev,
                     raw, processed, scale, ss, scale0, offset, os, offset0, d, n);
  return finish();
}

int mjh_root_frame(const float* xpos, long long ps, const float* xquat, long long qs, const float* com, long long cs,
                   const float* cvel, long long vs, const float* grav, long long gs, const float* fwd, long long fs,
                   float* out, long long n, void* stream) {
  return submit_job(RootFrameJob{xpos, ps, xquat, qs, com, cs, cvel, vs, grav, gs, fwd, fs, out}, n, stream);
}

int mjh_order_worlds(const int* solver_niter, const int* nefc, long long* order, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(order_worlds_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, solver_niter, nefc, order, n);
  return finish();
}

int mjh_motion_adaptive(const unsigned char* mask, const unsigned char* terminated, long long* time_steps,
                        const float* bin_failed, float* cur_failed, const float* kern, int nbins, int ksize,
                        long long T, float ratio, float* m_entropy, float* m_top1p, float* m_top1b,
                        unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n, void* stream) {
  if (n <= 0) return 0;
  if (nbins <= 0 || nbins > kMaxBins || ksize <= 0) return 1;
  hipLaunchKernelGGL(motion_adaptive_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, mask, terminated, time_steps,
                     bin_failed, cur_failed, kern, nbins, ksize, T, ratio, m_entropy, m_top1p, m_top1b, seed, key, ctr, n);
  return finish();
}

int mjh_motion_frame(const float* table, const long long* time_steps, float* frame, int width, int pos_off, int nb,
                     float* body_pos_w, const float* origins, long long os, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(motion_frame_kernel, dim3(grid(n * width)), dim3(kBlock), 0, (hipStream_t)stream, table, time_steps,
                     frame, width, pos_off, nb, body_pos_w, origins, os, n);
  return finish();
}

int mjh_motion_reset(const float* frame, long long fs, int nj, int pos_off, int quat_off, int lin_off, int ang_off,
                     const float* body_pos_w, long long bps, const unsigned char* mask, const float* pose_lo,
                     const float* pose_hi, const float* vel_lo, const float* vel_hi, int pose_any, int vel_any, float jlo,
                     float jhi, const float* lim, long long ls, float* qpos, long long qs, int root_q, int joint_q,
                     float* qvel, long long vs, int root_v, int joint_v, unsigned long long seed,
                     unsigned long long key, const mjh_i64* ctr, long long n, void* stream) {
  if (n <= 0) return 0;
  Range6 p{}, v{};
  for (int j = 0; j < 6; j++) {
    p.lo[j] = pose_lo[j]; p.hi[j] = pose_hi[j];
    v.lo[j] = vel_lo[j]; v.hi[j] = vel_hi[j];
  }
  hipLaunchKernelGGL(motion_reset_kernel, dim3(grid(n)), dim3(kBlock), 0, (hipStream_t)stream, frame, fs, nj, pos_off,
                     quat_off, lin_off, ang_off, body_pos_w, bps, mask, p, v, pose_any, vel_any, jlo, jhi, lim, ls, qpos,
                     qs, root_q, joint_q, qvel, vs, root_v, joint_v, seed, key, ctr, n);
  return finish();
}

int mjh_rew_exp_err(const float* a, long long aes, long long ars, const int* ra, const float* b, long long bes,
                    long long brs, const int* rb, int k, int d, int quat, float inv_std2, float* out, long long n,
                    void* stream) {
  if (n <= 0 || k <= 0) return 0;
  hipLaunchKernelGGL(rew_exp_err_kernel, dim3(grid(n)), dim3(kBlock), 0, (hipStream_t)stream, a, aes, ars, ra, b, bes, brs, rb,
                     k, d, quat, inv_std2, out, n);
  return finish();
}

int mjh_step_counters(mjh_i64* episode_length, mjh_i64* step, long long n, void* stream) {
  return submit_job(StepCountersJob{episode_length, step}, n, stream);
}

int mjh_reset_stats(const unsigned char* reset, unsigned char* any_reset, mjh_i64* stats, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(reset_stats_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, reset, any_reset, stats, n);
  return finish();
}

}  // extern "C"
extern "C" int mjh_velocity_command(const float* lin_b, long long ls, const float* ang_b, long long as, const float* root_q,
                                    long long qs, const float* u, long long us, const float* ranges, float dt,
                                    float inv_max_step, float t_lo, float t_hi, float rel_heading, float rel_standing,
                                    float stiffness, int heading_command, float* cmd, float* heading_target,
                                    float* heading_error, unsigned char* is_heading, unsigned char* is_standing,
                                    float* time_left, long long* counter, float* err_xy, float* err_yaw,
                                    unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n,
                                    void* stream) {
  return submit_job(VelocityCommandJob{lin_b, ls, ang_b, as, root_q, qs, u, us, ranges, dt, inv_max_step, t_lo, t_hi,
                                   rel_heading, rel_standing, stiffness, heading_command, cmd, heading_target,
                                   heading_error, reinterpret_cast<bool*>(is_heading), reinterpret_cast<bool*>(is_standing),
                                   time_left, counter, err_xy, err_yaw, seed, key, ctr}, n, stream);
}
