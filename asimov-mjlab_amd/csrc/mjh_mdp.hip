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


// this file's batchable jobs (mjh_batch.h)
struct MdpJobs {
  __device__ static void run(const mjh_batch::Job& j, long long e) {
    mjh_run_as<TrackJob>(j, e) || mjh_run_as<FlatJob>(j, e) || mjh_run_as<SqsumJob>(j, e) ||
        mjh_run_as<DiffsqJob>(j, e) || mjh_run_as<PosLimitsJob>(j, e) || mjh_run_as<PostureJob>(j, e) ||
        mjh_run_as<FeetJob>(j, e);
  }
};
const bool kMdpRegistered = mjh_batch::register_unit(mjh_batch::kMdp, mjh_batch_launch<MdpJobs>);

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

