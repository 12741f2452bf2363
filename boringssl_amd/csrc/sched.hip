// sched.hip -- record scheduling for ragged batches (gfx950).
//
// The bulk kernels give each record a fixed group of lanes and step a wave's
// records together, so a wave runs as long as its longest record.  For
// batches with per-record lengths this builds a processing order grouped by
// length class, longest first (a counting sort on length/256 into 64 classes),
// so the records a wave or tile handles together have similar lengths.  The
// order only changes which records are processed together, never where a
// record's output goes, so results are identical with or without it.
#include <hip/hip_runtime.h>

#include "internal.h"

namespace bssl_amd {
namespace {

constexpr int kClasses = kSchedClasses;  // (internal.h: the split words derive from these)
constexpr int kThreads = 256;
constexpr int kPerThread = 16;  // records per thread in the scatter pass

__device__ __forceinline__ int length_class(uint64_t len) {
  const uint64_t c = len / kSchedClassBytes;
  return c >= kClasses - 1 ? 0 : kClasses - 1 - (int)c;  // longest first
}

__global__ __launch_bounds__(kThreads) void class_histogram(const uint64_t *__restrict__ lengths,
                                                           uint64_t n, uint32_t *hist) {
  __shared__ uint32_t h[kClasses];
  if (threadIdx.x < kClasses) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kThreads)
    atomicAdd(&h[length_class(lengths[i])], 1u);
  __syncthreads();
  if (threadIdx.x < kClasses && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// Exclusive prefix sum of the 64 class counts (one wave).
__global__ void class_offsets(const uint32_t *hist, uint32_t *cursor) {
  const int l = threadIdx.x;
  uint32_t v = hist[l], x = v;
#pragma unroll
  for (int o = 1; o < kClasses; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, kClasses);
    if (l >= o) x += y;
  }
  cursor[l] = x - v;
}

// Each block reserves, per class, a contiguous range for its records with one
// global atomic per class, then places them with LDS atomics.
__global__ __launch_bounds__(kThreads) void class_scatter(const uint64_t *__restrict__ lengths,
                                                         uint64_t n, uint32_t *cursor,
                                                         uint32_t *__restrict__ order) {
  __shared__ uint32_t cnt[kClasses], base[kClasses];
  if (threadIdx.x < kClasses) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t first = (uint64_t)blockIdx.x * kThreads * kPerThread;
  int cls[kPerThread];
  uint32_t rank[kPerThread];
#pragma unroll
  for (int k = 0; k < kPerThread; k++) {
    const uint64_t i = first + (uint64_t)k * kThreads + threadIdx.x;
    cls[k] = i < n ? length_class(lengths[i]) : -1;
    rank[k] = cls[k] >= 0 ? atomicAdd(&cnt[cls[k]], 1u) : 0u;
  }
  __syncthreads();
  if (threadIdx.x < kClasses)
    base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]) : 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPerThread; k++) {
    const uint64_t i = first + (uint64_t)k * kThreads + threadIdx.x;
    if (cls[k] >= 0) order[base[cls[k]] + rank[k]] = (uint32_t)i;
  }
}

}  // namespace

int build_length_order(const uint64_t *lengths, uint64_t n, uint32_t *order, uint32_t *scratch,
                       void *stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint32_t *hist = scratch, *cursor = scratch + kClasses;
  if (hipMemsetAsync(hist, 0, kClasses * sizeof(uint32_t), s) != hipSuccess) return 1;
  const uint64_t hb = (n + kThreads * 16 - 1) / (kThreads * 16);
  hipLaunchKernelGGL(class_histogram, dim3((unsigned)(hb < 4096 ? hb : 4096)), dim3(kThreads), 0,
                     s, lengths, n, hist);
  hipLaunchKernelGGL(class_offsets, dim3(1), dim3(kClasses), 0, s, hist, cursor);
  const uint64_t sb = (n + kThreads * kPerThread - 1) / (kThreads * kPerThread);
  hipLaunchKernelGGL(class_scatter, dim3((unsigned)sb), dim3(kThreads), 0, s, lengths, n, cursor,
                     order);
  return (int)hipGetLastError();
}

}  // namespace bssl_amd
