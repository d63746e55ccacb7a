// mjh_mgr.hip — manager-level fused kernels (gfx950): one launch per
// observation group and one per reward pass, replacing a launch per term plus
// the stack / weight / accumulate / sum chain. Term descriptors are passed by
// value in the kernel arguments, so a captured graph bakes them like any other
// launch parameter (no host->device copy inside the env step).
#include <hip/hip_runtime.h>

#include "../../include/mjh_abi.h"

namespace {

struct ObsArgs {
  mjh_obs_term_desc t[MJH_MAX_TERMS];
  int nterms;
};

// blockIdx.y = term; out[e, off + j] = clip(x[e, j] + noise, cmin, cmax) * scale
// (observation_manager.py:163-176: noise -> clip -> scale)
__global__ void obs_group_kernel(const ObsArgs a, const float* __restrict__ u, long long us, float* __restrict__ out,
                                 long long os, long long n) {
  const mjh_obs_term_desc& d = a.t[blockIdx.y];
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * d.w) return;
  const long long e = t / d.w;
  const int j = (int)(t - e * d.w);
  float v = d.x[e * d.xs + j];
  if (d.noise) v = v + (u[e * us + d.off + j] * (d.hi - d.lo) + d.lo);
  if (d.cmin <= d.cmax) v = fminf(fmaxf(v, d.cmin), d.cmax);
  out[e * os + d.off + j] = v * d.scale;
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
  float r = 0.f;
  for (int i = 0; i < T; i++) {
    const float x = a.v[i] ? a.v[i][e * a.vs[i]] : 0.f;
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

extern "C" {

int mjh_obs_group(const mjh_obs_term_desc* terms, int nterms, const float* u, long long us, float* out, long long os,
                  long long n, void* stream) {
  if (n <= 0 || nterms <= 0) return 0;
  if (nterms > MJH_MAX_TERMS) return 1;
  ObsArgs a;
  int wmax = 0;
  for (int i = 0; i < nterms; i++) {
    a.t[i] = terms[i];
    if (terms[i].noise && !u) return 1;
    if (terms[i].w > wmax) wmax = terms[i].w;
  }
  a.nterms = nterms;
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

}  // extern "C"
