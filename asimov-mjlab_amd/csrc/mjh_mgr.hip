// mjh_mgr.hip — manager-level fused kernels (gfx950): one launch per
// observation group and one per reward pass, replacing a launch per term plus
// the stack / weight / accumulate / sum chain. Term descriptors are passed by
// value in the kernel arguments, so a captured graph bakes them like any other
// launch parameter (no host->device copy inside the env step).
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/mjh_abi.h"
#include "mjh_batch.h"
#include "mjh_rng.h"

namespace {

struct ObsArgs {
  mjh_obs_term_desc t[MJH_MAX_TERMS];
  int nterms;
  int width;  // group width: element index of the device-stream noise draw
  unsigned long long seed, key;
  const mjh_i64* ctr;
};

// blockIdx.y = term; out[e, off + j] = clip(f(x[e, j]) + noise, cmin, cmax) * scale
// (observation_manager.py:163-176: term -> noise -> clip -> scale), f the
// term's elementwise op on its strided input (MJH_OBS_*)
__global__ void obs_group_kernel(const ObsArgs a, const float* __restrict__ u, long long us, float* __restrict__ out,
                                 long long os, long long n) {
  const mjh_obs_term_desc& d = a.t[blockIdx.y];
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * d.w) return;
  const long long e = t / d.w;
  const int j = (int)(t - e * d.w);
  float v = d.xd > 1 ? d.x[e * d.xs + (j / d.xd) * d.xcs + j % d.xd] : d.x[e * d.xs + j * d.xcs];
  if (d.op == MJH_OBS_SUB) v -= d.y[e * d.ys + j];
  else if (d.op == MJH_OBS_POSITIVE) v = v > 0.f ? 1.f : 0.f;
  else if (d.op == MJH_OBS_SIGNED_LOG1P) v = (v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f)) * log1pf(fabsf(v));
  if (d.noise) {
    const float r = u ? u[e * us + d.off + j] : mjh::Rng(a.seed, a.key, a.ctr).u01(e * a.width + d.off + j);
    v = v + (r * (d.hi - d.lo) + d.lo);
  }
  if (d.cmin <= d.cmax) v = fminf(fmaxf(v, d.cmin), d.cmax);
  out[e * os + d.off + j] = v * d.scale;
}

// one workgroup: count the worlds per flag bit, publish, accumulate, clear
__global__ void flag_stats_kernel(int* __restrict__ flags, long long n, mjh_i64* __restrict__ stats) {
  __shared__ int cnt[3];
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  int c0 = 0, c1 = 0, c2 = 0;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    const int f = flags[i];
    c0 += f & MJH_FLAG_CONTACT_OVERFLOW ? 1 : 0;
    c1 += f & MJH_FLAG_EFC_OVERFLOW ? 1 : 0;
    c2 += f & MJH_FLAG_NONFINITE ? 1 : 0;
    flags[i] = 0;
  }
  if (c0) atomicAdd(&cnt[0], c0);  // LDS atomics
  if (c1) atomicAdd(&cnt[1], c1);
  if (c2) atomicAdd(&cnt[2], c2);
  __syncthreads();
  if (threadIdx.x < 3) {
    stats[threadIdx.x] = cnt[threadIdx.x];
    stats[3 + threadIdx.x] += cnt[threadIdx.x];
  }
}

struct RewArgs {
  const float* v[MJH_MAX_TERMS];
  long long vs[MJH_MAX_TERMS];
  int nterms;
};

// reward_manager.py:76-88: weighted = term * (weight * dt); step_reward = term * weight;
// sums += weighted; reward = sum_t weighted (terms with a null pointer are 0)
__global__ void reward_combine_kernel(const RewArgs a, const float* __restrict__ w, float dt, float* __restrict__ reward,
                                      float* __restrict__ step_reward, float* __restrict__ sums, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int T = a.nterms;
  // every term's value loaded before the first store (the stores may alias the
  // term buffers as far as the compiler knows, so a load behind one waits for it)
  float xs[MJH_MAX_TERMS];
#pragma unroll
  for (int i = 0; i < MJH_MAX_TERMS; i++) xs[i] = (i < T && a.v[i]) ? a.v[i][e * a.vs[i]] : 0.f;
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < MJH_MAX_TERMS; i++) {
    if (i >= T) break;
    const float x = xs[i];
    const float wi = w[i];
    const float wd = wi * dt;
    const float weighted = x * wd;
    step_reward[e * T + i] = x * wi;
    sums[e * T + i] += weighted;
    r += weighted;
  }
  reward[e] = r;
}

}  // namespace

// ---- the job batch's host side (mjh_batch.h) ----------------------------------
namespace mjh_batch {
namespace {
struct State {
  bool open = false;
  bool seq = false;
  int cur = -1;  // sequential batches: the unit of the jobs recorded last
  bool counter_written = false;  // sequential batches: a recorded, not yet launched kWritesCounter job
  hipStream_t stream = nullptr;
  Pack pack[kUnits];
};
thread_local State g_state;
Launcher g_launch[kUnits] = {};

void flush_unit(State& st, int u) {
  Pack& p = st.pack[u];
  if (p.njobs > 0 && g_launch[u]) g_launch[u](p, st.stream, st.seq);
  p.njobs = 0;
  p.nmax = 0;
}
}  // namespace

bool register_unit(int unit, Launcher f) {
  if (unit < 0 || unit >= kUnits) return false;
  g_launch[unit] = f;
  return true;
}

bool add(int unit, int kind, long long n, const void* args, size_t bytes, hipStream_t s, int flags) {
  State& st = g_state;
  if (!st.open || unit < 0 || unit >= kUnits || !g_launch[unit] || bytes > (size_t)kArgBytes) return false;
  // a producer's output is read inside the pass: in an independent batch it
  // runs now (ahead of the batch, on the same stream), never recorded
  if (!st.seq && (flags & kProducer)) return false;
  if (s != st.stream) {  // a job on another stream: everything recorded so far goes first
    if (st.seq) {
      if (st.cur >= 0) flush_unit(st, st.cur);
    } else {
      for (int u = 0; u < kUnits; u++) flush_unit(st, u);
    }
    st.stream = s;
  }
  if (st.seq && st.cur != unit && st.cur >= 0) flush_unit(st, st.cur);  // keep the recorded order
  // a counter reader after the counter's writer: the writer's dispatch ends first
  if (st.seq && (flags & kReadsCounter) && st.counter_written) {
    for (int u = 0; u < kUnits; u++) flush_unit(st, u);
    st.counter_written = false;
  }
  st.cur = unit;
  Pack& p = st.pack[unit];
  if (p.njobs == kMaxJobs) flush_unit(st, unit);
  if (flags & kWritesCounter) st.counter_written = true;
  Job& j = p.jobs[p.njobs++];
  j.kind = kind;
  j.pad = 0;
  j.n = n;
  std::memcpy(j.a, args, bytes);
  if (n > p.nmax) p.nmax = n;
  return true;
}
}  // namespace mjh_batch

extern "C" {

int mjh_batch_begin(int sequential) {
  mjh_batch::g_state.open = true;
  mjh_batch::g_state.seq = sequential != 0;
  mjh_batch::g_state.cur = -1;
  mjh_batch::g_state.counter_written = false;
  mjh_batch::g_state.stream = nullptr;
  for (auto& p : mjh_batch::g_state.pack) p.njobs = 0, p.nmax = 0;
  return 0;
}

int mjh_batch_end(void* stream) {
  auto& st = mjh_batch::g_state;
  if (!st.open) return 0;
  if (!st.stream) st.stream = (hipStream_t)stream;
  if (st.seq) {
    if (st.cur >= 0) mjh_batch::flush_unit(st, st.cur);
  } else {
    for (int u = 0; u < mjh_batch::kUnits; u++) mjh_batch::flush_unit(st, u);
  }
  st.open = false;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int mjh_obs_group(const mjh_obs_term_desc* terms, int nterms, const float* u, long long us, float* out, long long os,
                  long long n, unsigned long long seed, unsigned long long key, const mjh_i64* ctr, void* stream) {
  if (n <= 0 || nterms <= 0) return 0;
  if (nterms > MJH_MAX_TERMS) return 1;
  ObsArgs a;
  int wmax = 0, width = 0;
  for (int i = 0; i < nterms; i++) {
    a.t[i] = terms[i];
    if (terms[i].w > wmax) wmax = terms[i].w;
    if (terms[i].off + terms[i].w > width) width = terms[i].off + terms[i].w;
    if (terms[i].op == MJH_OBS_SUB && !terms[i].y) return 1;
  }
  a.nterms = nterms;
  a.width = width;
  a.seed = seed;
  a.key = key;
  a.ctr = ctr;
  const long long items = n * wmax;
  hipLaunchKernelGGL(obs_group_kernel, dim3((unsigned)((items + 255) / 256), (unsigned)nterms), dim3(256), 0,
                     (hipStream_t)stream, a, u, us, out, os, n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int mjh_reward_combine(const float* const* values, const long long* strides, int nterms, const float* weights, float dt,
                       float* reward, float* step_reward, float* sums, long long n, void* stream) {
  if (n <= 0) return 0;
  if (nterms > MJH_MAX_TERMS || nterms < 0) return 1;
  RewArgs a;
  for (int i = 0; i < nterms; i++) {
    a.v[i] = values[i];
    a.vs[i] = strides[i];
  }
  a.nterms = nterms;
  hipLaunchKernelGGL(reward_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a,
                     weights, dt, reward, step_reward, sums, n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int mjh_flag_stats(int* flags_acc, long long nworld, mjh_i64* stats, void* stream) {
  hipLaunchKernelGGL(flag_stats_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, flags_acc, nworld, stats);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
