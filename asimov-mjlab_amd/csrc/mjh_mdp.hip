// mjh_mdp.hip — fused MDP term kernels for the velocity task (gfx950).
//
// Each kernel computes one reward/observation term for all envs in a single
// launch, with the formula of the torch term it replaces
// (src/mjlab/tasks/velocity/mdp/rewards.py, src/mjlab/envs/mdp/rewards.py);
// the torch versions in mjlab_amd remain the semantics and the CPU path.
// Row-strided inputs (last-dim stride 1) let views such as qpos[:, 7:] or
// pose[:, 3:7] be read in place.
#include <hip/hip_runtime.h>

#include "../../include/mjh_abi.h"
#include "mjh_batch.h"
#include "mjh_rng.h"

namespace {

inline int grid(long long n) { return (int)((n + 255) / 256); }
inline int finish() { return hipGetLastError() == hipSuccess ? 0 : 2; }

__device__ __forceinline__ float cmd_total(const float* c) { return sqrtf(c[0] * c[0] + c[1] * c[1]) + fabsf(c[2]); }

// Reward terms as batchable jobs (mjh_batch.h): run(e) is the term's formula
// for env e; the ABI entry points launch the job's own kernel or append it to
// the reward pass's batch.

// exp(-(|c_xy - v_xy|^2 + v_z^2) / std2)            track_linear_velocity
// exp(-((c_z - w_z)^2 + |w_xy|^2) / std2)            track_angular_velocity
struct TrackJob {
  static constexpr int kKind = 1;
  const float* cmd; long long cs; const float* v; long long vs; float inv_std2; int angular; float* out;
  __device__ __forceinline__ void run(long long e) const {
    const float* c = cmd + e * cs;
    const float* a = v + e * vs;
    float err;
    if (angular) {
      const float dz = c[2] - a[2];
      err = dz * dz + (a[0] * a[0] + a[1] * a[1]);
    } else {
      const float dx = c[0] - a[0], dy = c[1] - a[1];
      err = (dx * dx + dy * dy) + a[2] * a[2];
    }
    out[e] = expf(-err * inv_std2);
  }
};

// exp(-|(q^-1 g)_xy|^2 / std2)                        flat_orientation (body path)
struct FlatJob {
  static constexpr int kKind = 2;
  const float* q; long long qs; const float* g; long long gs; float inv_std2; float* out;
  __device__ __forceinline__ void run(long long e) const {
    const float* a = q + e * qs;
    const float* b = g + e * gs;
    const float w = a[0], x = a[1], y = a[2], z = a[3];
    const float tx = 2.f * (y * b[2] - z * b[1]), ty = 2.f * (z * b[0] - x * b[2]), tz = 2.f * (x * b[1] - y * b[0]);
    const float gx = (b[0] - w * tx) + (y * tz - z * ty);
    const float gy = (b[1] - w * ty) + (z * tx - x * tz);
    out[e] = expf(-(gx * gx + gy * gy) * inv_std2);
  }
};

// sum_j x_j^2 over the first k columns                 body_angular_velocity (k=2), angular momentum (k=3)
struct SqsumJob {
  static constexpr int kKind = 3;
  const float* x; long long xs; int k; float* out;
  __device__ __forceinline__ void run(long long e) const {
    const float* a = x + e * xs;
    float s = 0.f;
    for (int j = 0; j < k; j++) s += a[j] * a[j];
    out[e] = s;
  }
};

// sum_j (a_j - b_j)^2                                  action_rate_l2
struct DiffsqJob {
  static constexpr int kKind = 4;
  const float* a; long long as; const float* b; long long bs; int k; float* out;
  __device__ __forceinline__ void run(long long e) const {
    float s = 0.f;
    // unrolled so a batch of the row's strided loads is in flight at once (the
    // sum keeps its order: bit-identical)
#pragma unroll 8
    for (int j = 0; j < k; j++) {
      const float d = a[e * as + j] - b[e * bs + j];
      s += d * d;
    }
    out[e] = s;
  }
};

// sum_j max(lo_j - q_j, 0) + max(q_j - hi_j, 0)       joint_pos_limits (lim: (N, k, 2))
struct PosLimitsJob {
  static constexpr int kKind = 5;
  const float* q; long long qs; const float* lim; long long ls; int k; float* out;
  __device__ __forceinline__ void run(long long e) const {
    float s = 0.f;
#pragma unroll 8
    for (int j = 0; j < k; j++) {
      const float v = q[e * qs + j], lo = lim[e * ls + 2 * j], hi = lim[e * ls + 2 * j + 1];
      s += -fminf(v - lo, 0.f);
      s += fmaxf(v - hi, 0.f);
    }
    out[e] = s;
  }
};

// exp(-mean_j (q_j - q0_j)^2 / std_j^2), std by command speed band   variable_posture
struct PostureJob {
  static constexpr int kKind = 6;
  const float* q; long long qs; const float* q0; long long q0s; const float* std_stand; const float* std_walk;
  const float* std_run; const float* cmd; long long cs; float walk_thr; float run_thr; int k; float* out;
  __device__ __forceinline__ void run(long long e) const {
    const float tot = cmd_total(cmd + e * cs);
    const float* sd = tot < walk_thr ? std_stand : (tot < run_thr ? std_walk : std_run);
    float s = 0.f;
#pragma unroll 8
    for (int j = 0; j < k; j++) {
      const float d = q[e * qs + j] - q0[e * q0s + j];
      s += d * d / (sd[j] * sd[j]);
    }
    out[e] = expf(-s / (float)k);
  }
};

// per-foot terms on k sites (site z, site linear velocity (N, k, 3)):
//   clearance: sum_j |z_j - target| * |v_xy,j|                     (feet_clearance; z_j at column stride zcs)
//   slip:      sum_j |v_xy,j|^2 * [found_j > 0]                   (feet_slip)
// both x [command total > threshold]; also writes sum_j |v_xy| * [found] and
// sum_j [found] for the slip metric.
struct FeetJob {
  static constexpr int kKind = 7;
  const float* z; long long zs; long long zcs; const float* vel; long long vs; long long vcs; const float* found; long long fs;
  long long fcs; const float* cmd; long long cs; float target; float thr_clear; float thr_slip; int k;
  float* clearance; float* slip; float* slip_vsum; float* slip_cnt;
  __device__ __forceinline__ void run(long long e) const {
    const float tot = cmd_total(cmd + e * cs);
    float cl = 0.f, sl = 0.f, vs_ = 0.f, cnt = 0.f;
    for (int j = 0; j < k; j++) {
      const float* v = vel + e * vs + vcs * j;
      const float vn = sqrtf(v[0] * v[0] + v[1] * v[1]);
      cl += fabsf(z[e * zs + zcs * j] - target) * vn;
      if (found) {
        const float in = found[e * fs + fcs * j] > 0.f ? 1.f : 0.f;
        sl += vn * vn * in;
        vs_ += vn * in;
        cnt += in;
      }
    }
    if (clearance) clearance[e] = cl * (tot > thr_clear ? 1.f : 0.f);
    if (found) {
      slip[e] = sl * (tot > thr_slip ? 1.f : 0.f);
      slip_vsum[e] = vs_;
      slip_cnt[e] = cnt;
    }
  }
};

// the reward pass's batch kernel for this file's jobs
__global__ void mdp_batch_kernel(const mjh_batch::Pack p) {
  const mjh_batch::Job& j = p.jobs[blockIdx.y];
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= j.n) return;
  switch (j.kind) {
    case TrackJob::kKind: reinterpret_cast<const TrackJob*>(j.a)->run(e); break;
    case FlatJob::kKind: reinterpret_cast<const FlatJob*>(j.a)->run(e); break;
    case SqsumJob::kKind: reinterpret_cast<const SqsumJob*>(j.a)->run(e); break;
    case DiffsqJob::kKind: reinterpret_cast<const DiffsqJob*>(j.a)->run(e); break;
    case PosLimitsJob::kKind: reinterpret_cast<const PosLimitsJob*>(j.a)->run(e); break;
    case PostureJob::kKind: reinterpret_cast<const PostureJob*>(j.a)->run(e); break;
    case FeetJob::kKind: reinterpret_cast<const FeetJob*>(j.a)->run(e); break;
    default: break;
  }
}

void mdp_batch_launch(const mjh_batch::Pack& p, hipStream_t s) {
  hipLaunchKernelGGL(mdp_batch_kernel, dim3(mjh_batch::grid1(p.nmax), p.njobs), dim3(256), 0, s, p);
}
const bool kMdpRegistered = mjh_batch::register_unit(mjh_batch::kMdp, mdp_batch_launch);

template <class J>
int submit(const J& j, long long n, void* stream) {
  return mjh_batch::submit(mjh_batch::kMdp, j, n, (hipStream_t)stream, mjh_job_kernel<J>);
}

}  // namespace

extern "C" {

int mjh_rew_track(const float* cmd, long long cs, const float* v, long long vs, float inv_std2, int angular, float* out,
                  long long n, void* stream) {
  return submit(TrackJob{cmd, cs, v, vs, inv_std2, angular, out}, n, stream);
}

int mjh_rew_flat_orientation(const float* q, long long qs, const float* g, long long gs, float inv_std2, float* out,
                             long long n, void* stream) {
  return submit(FlatJob{q, qs, g, gs, inv_std2, out}, n, stream);
}

int mjh_rew_sqsum(const float* x, long long xs, int k, float* out, long long n, void* stream) {
  return submit(SqsumJob{x, xs, k, out}, n, stream);
}

int mjh_rew_diffsq(const float* a, long long as, const float* b, long long bs, int k, float* out, long long n, void* stream) {
  return submit(DiffsqJob{a, as, b, bs, k, out}, n, stream);
}

int mjh_rew_pos_limits(const float* q, long long qs, const float* lim, long long ls, int k, float* out, long long n,
                       void* stream) {
  return submit(PosLimitsJob{q, qs, lim, ls, k, out}, n, stream);
}

int mjh_rew_posture(const float* q, long long qs, const float* q0, long long q0s, const float* std_stand,
                    const float* std_walk, const float* std_run, const float* cmd, long long cs, float walk_thr,
                    float run_thr, int k, float* out, long long n, void* stream) {
  return submit(PostureJob{q, qs, q0, q0s, std_stand, std_walk, std_run, cmd, cs, walk_thr, run_thr, k, out}, n, stream);
}

int mjh_rew_feet(const float* z, long long zs, long long zcs, const float* vel, long long vs, long long vcs, const float* found, long long fs,
                 long long fcs, const float* cmd, long long cs, float target, float thr_clear, float thr_slip, int k,
                 float* clearance, float* slip, float* slip_vsum, float* slip_cnt, long long n, void* stream) {
  return submit(FeetJob{z, zs, zcs, vel, vs, vcs, found, fs, fcs, cmd, cs, target, thr_clear, thr_slip, k, clearance, slip,
                        slip_vsum, slip_cnt}, n, stream);
}

}  // extern "C"

// ---- UniformVelocityCommand.compute (velocity_command.py:65-101 and
// command_manager.py:53-67) for all envs in one launch: metric accumulation,
// timer countdown, masked resampling from u (N, 8) uniform draws
// [timer, lin_x, lin_y, ang_z, heading, heading-env, standing-env, unused],
// heading control and standing override.
namespace {
__device__ __forceinline__ float wrap_to_pi_f(float a) {
  const float two_pi = 6.283185307179586f, pi = 3.141592653589793f;
  float r = fmodf(a, two_pi);  // torch.remainder: fmod, then shift into [0, 2pi)
  if (r != 0.f && r < 0.f) r += two_pi;
  return r > pi ? r - two_pi : r;
}

__global__ void velocity_command_kernel(const float* lin_b, long long ls, const float* ang_b, long long as,
                                        const float* root_q, long long qs, const float* u, long long us,
                                        const float* ranges, float dt, float inv_max_step, float t_lo, float t_hi,
                                        float rel_heading, float rel_standing, float stiffness, int heading_command,
                                        float* cmd, float* heading_target, float* heading_error, bool* is_heading,
                                        bool* is_standing, float* time_left, long long* counter, float* err_xy,
                                        float* err_yaw, unsigned long long seed, unsigned long long key,
                                        const mjh_i64* ctr, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
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
}  // namespace

extern "C" int mjh_velocity_command(const float* lin_b, long long ls, const float* ang_b, long long as, const float* root_q,
                                    long long qs, const float* u, long long us, const float* ranges, float dt,
                                    float inv_max_step, float t_lo, float t_hi, float rel_heading, float rel_standing,
                                    float stiffness, int heading_command, float* cmd, float* heading_target,
                                    float* heading_error, unsigned char* is_heading, unsigned char* is_standing,
                                    float* time_left, long long* counter, float* err_xy, float* err_yaw,
                                    unsigned long long seed, unsigned long long key, const mjh_i64* ctr, long long n,
                                    void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(velocity_command_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, lin_b, ls, ang_b, as, root_q,
                     qs, u, us, ranges, dt, inv_max_step, t_lo, t_hi, rel_heading, rel_standing, stiffness, heading_command,
                     cmd, heading_target, heading_error, reinterpret_cast<bool*>(is_heading),
                     reinterpret_cast<bool*>(is_standing), time_left, counter, err_xy, err_yaw, seed, key, ctr, n);
  return finish();
}
