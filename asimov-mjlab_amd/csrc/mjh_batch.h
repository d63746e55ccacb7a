// mjh_batch.h — one launch for a pass of independent per-env env-layer kernels.
//
// A captured env step replays ~50 small env-layer kernels; each is a separate
// dispatch whose cost (~5 us on 4,096 envs) is its launch and memory latency,
// not its work. Kernels that the env layer evaluates as a group of mutually
// independent per-env jobs (the reward terms of one reward pass) are written
// as job structs whose run(e) is the kernel body; their C-ABI entry points
// either launch the job's own kernel (no batch open) or append the job to the
// open batch. mjh_batch_end launches every translation unit's batch kernel
// once: blockIdx.y selects the job, blockIdx.x * blockDim.x + threadIdx.x the
// env, so the batched pass runs the same arithmetic as the separate launches
// (bit-identical outputs) in one dispatch per file. Jobs in a batch must not
// read each other's outputs (the reward terms read sim state, EntityData and
// commands only); anything launched while a batch is open runs before it.
// A sequential batch (mjh_batch_begin(1)) instead runs each env's jobs in the
// order they were recorded, one thread per env (consecutive jobs of the same
// file in one dispatch): for chains of per-env kernels where a job reads an
// earlier job's output for the same env only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <type_traits>

namespace mjh_batch {

constexpr int kArgBytes = 240;  // the largest job struct (static_assert in submit)
constexpr int kMaxJobs = 10;    // per translation unit and launch (kernel arguments: ~2.6 KB)
enum Unit { kMdp = 0, kFuse = 1, kUnits = 2 };

struct Job {
  int kind;
  int pad;
  long long n;
  alignas(16) unsigned char a[kArgBytes];
};

struct Pack {
  int njobs;
  int pad;
  long long nmax;
  Job jobs[kMaxJobs];
};

// seq = false: the jobs are independent (blockIdx.y = job); seq = true: thread
// e runs the jobs in recorded order for env e (per-env dependencies kept)
typedef void (*Launcher)(const Pack&, hipStream_t, bool seq);

// Job flags (a job struct declares `static constexpr int kFlags`; a member
// named `ctr` adds kReadsCounter):
// * kProducer: other jobs or torch read the output within the same pass (the
//   root frame), so in an independent batch the job launches at once instead
//   of being recorded (the batch's jobs may not read each other's outputs);
// * kWritesCounter: the job advances the device step counter from one thread
//   (the step counters); kReadsCounter: the job reads that counter (the random
//   streams, event marks). In a sequential batch a reader recorded after a
//   writer starts a new dispatch, so every thread sees the advanced counter.
enum Flags { kProducer = 1, kWritesCounter = 2, kReadsCounter = 4 };
template <class J, class = void> struct declared_flags : std::integral_constant<int, 0> {};
template <class J> struct declared_flags<J, std::void_t<decltype(J::kFlags)>> : std::integral_constant<int, J::kFlags> {};
template <class J, class = void> struct has_ctr : std::false_type {};
template <class J> struct has_ctr<J, std::void_t<decltype(&J::ctr)>> : std::true_type {};
template <class J> constexpr int job_flags() { return declared_flags<J>::value | (has_ctr<J>::value ? kReadsCounter : 0); }

// host side (mjh_mgr.hip): register a unit's batch launcher; append a job to
// the open batch (false: no batch open, or a producer in an independent batch:
// the caller launches the job itself)
bool register_unit(int unit, Launcher f);
bool add(int unit, int kind, long long n, const void* args, size_t bytes, hipStream_t s, int flags);

inline int grid1(long long n) { return (int)((n + 255) / 256); }

// launch job J's own kernel, or append it to the open batch
template <class J>
int submit(int unit, const J& j, long long n, hipStream_t s, void (*kernel)(J, long long)) {
  static_assert(sizeof(J) <= kArgBytes, "job struct exceeds the batch slot");
  if (n <= 0) return 0;
  if (add(unit, J::kKind, n, &j, sizeof(J), s, job_flags<J>())) return 0;
  hipLaunchKernelGGL(kernel, dim3(grid1(n)), dim3(256), 0, s, j, n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace mjh_batch

// the per-job kernel of a job struct J (J::run(e) is the body)
template <class J>
__global__ void mjh_job_kernel(const J j, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) j.run(e);
}

// a unit's batch kernels; D::run(job, e) switches on the job kind
template <class D>
__global__ void mjh_batch2d_kernel(const mjh_batch::Pack p) {
  const mjh_batch::Job& j = p.jobs[blockIdx.y];
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < j.n) D::run(j, e);
}
template <class D>
__global__ void mjh_batchseq_kernel(const mjh_batch::Pack p) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < p.njobs; k++) {
    const mjh_batch::Job& j = p.jobs[k];
    if (e < j.n) D::run(j, e);
  }
}
template <class D>
void mjh_batch_launch(const mjh_batch::Pack& p, hipStream_t s, bool seq) {
  if (seq)
    hipLaunchKernelGGL(mjh_batchseq_kernel<D>, dim3(mjh_batch::grid1(p.nmax)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(mjh_batch2d_kernel<D>, dim3(mjh_batch::grid1(p.nmax), p.njobs), dim3(256), 0, s, p);
}
// dispatch a job of kind J::kKind to J::run
template <class J>
__device__ __forceinline__ bool mjh_run_as(const mjh_batch::Job& j, long long e) {
  if (j.kind != J::kKind) return false;
  reinterpret_cast<const J*>(j.a)->run(e);
  return true;
}
