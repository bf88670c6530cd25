// FPR at 95 % recall on device: the per-pair descriptor distance of the eval loop
// (hardnet/HardNet.py:458) followed by ErrorRateAt95Recall (hardnet/EvalMetrics.py:6-19).
//
//   d_i   = sqrt(sum_k (a_ik - p_ik)^2)                       (fp32, like the reference)
//   key_i = 1 / (1 / (d_i + 1e-8) + 1e-8)                      (scores -> distances, fp32)
//   labels sorted by key (stable LSD radix sort, hipCUB); t = first i with
//   cumsum(labels)[i] >= 0.95 * sum(labels); FP = #0 in [0,t), TN = #0 in [t,n).
//
// Ties: numpy's argsort (quicksort) orders equal keys implementation-defined; the radix
// sort here is stable.  Results can differ only when equal keys with different labels
// straddle the threshold (documented in tests/test_gpu_parity.py).
#include <hipcub/hipcub.hpp>

#include "hn_common.h"
#include "hn_internal.h"

namespace {

__global__ __launch_bounds__(256) void k_pair_dist(const float* __restrict__ a, const float* __restrict__ p,
                                                   int64_t n, int dim, float* __restrict__ d,
                                                   float* __restrict__ key, int* __restrict__ idx) {
  // one wave per pair, lanes stride over the descriptor
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  float s = 0.f;
  for (int k = lane; k < dim; k += 64) {
    const float df = a[i * dim + k] - p[i * dim + k];
    s = fmaf(df, df, s);
  }
  s = wave_sum(s);
  if (lane == 0) {
    const float dist = sqrtf(s);
    if (d) d[i] = dist;
    const float score = 1.0f / (dist + 1e-8f);
    key[i] = 1.0f / (score + 1e-8f);
    idx[i] = (int)i;
  }
}

__global__ __launch_bounds__(256) void k_gather_labels(const int* __restrict__ perm,
                                                       const int* __restrict__ labels, int64_t n,
                                                       int* __restrict__ sorted) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) sorted[i] = labels[perm[i]] != 0 ? 1 : 0;
}

// first index with cumsum >= thr  (cumsum is non-decreasing -> atomicMin over candidates)
__global__ __launch_bounds__(256) void k_threshold(const long long* __restrict__ cum, int64_t n,
                                                   unsigned long long* __restrict__ first) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long total = cum[n - 1];
  const double thr = 0.95 * (double)total;
  const bool hit = (double)cum[i] >= thr;
  const bool prev = i > 0 && (double)cum[i - 1] >= thr;
  if (hit && !prev) atomicMin(first, (unsigned long long)i);
}

__global__ void k_fpr(const long long* __restrict__ cum, int64_t n,
                      const unsigned long long* __restrict__ first, double* __restrict__ out) {
  const long long t = (long long)*first;  // n if never reached (np.argmax of all-False -> 0)
  const long long ti = t >= n ? 0 : t;
  const long long ones_before = ti > 0 ? cum[ti - 1] : 0;
  const long long total = cum[n - 1];
  const long long fp = ti - ones_before;
  const long long tn = (n - ti) - (total - ones_before);
  // the reference divides 0/0 (Python raises); report NaN for "no negatives"
  *out = (fp + tn) > 0 ? (double)fp / (double)(fp + tn) : __builtin_nan("");
}

struct Ws {
  size_t off_dist_keys, off_keys_sorted, off_idx, off_idx_sorted, off_lab, off_cum, off_first,
      off_tmp, tmp_bytes, total;
};

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

hipError_t layout(int64_t n, Ws& w) {
  size_t sort_tmp = 0, scan_tmp = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (const float*)nullptr,
                                                    (float*)nullptr, (const int*)nullptr,
                                                    (int*)nullptr, (int)n);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveSum(nullptr, scan_tmp, (const int*)nullptr,
                                       (long long*)nullptr, (int)n);
  if (e != hipSuccess) return e;
  size_t o = 0;
  w.off_dist_keys = o; o = align256(o + n * 4);
  w.off_keys_sorted = o; o = align256(o + n * 4);
  w.off_idx = o; o = align256(o + n * 4);
  w.off_idx_sorted = o; o = align256(o + n * 4);
  w.off_lab = o; o = align256(o + n * 4);
  w.off_cum = o; o = align256(o + n * 8);
  w.off_first = o; o = align256(o + 8);
  w.tmp_bytes = std::max(sort_tmp, scan_tmp);
  w.off_tmp = o; o = align256(o + w.tmp_bytes);
  w.total = o;
  return hipSuccess;
}

}  // namespace

hipError_t hn_fpr95_ws_bytes(int64_t n, size_t* bytes) {
  Ws w{};
  hipError_t e = layout(n, w);
  *bytes = w.total;
  return e;
}

hipError_t hn_launch_fpr95(const float* a, const float* p, const int* labels, int64_t n, int dim,
                           float* dists, double* fpr, void* ws, size_t ws_bytes, hipStream_t st) {
  Ws w{};
  hipError_t e = layout(n, w);
  if (e != hipSuccess) return e;
  if (ws_bytes < w.total) return hipErrorInvalidValue;
  char* b = static_cast<char*>(ws);
  float* key = reinterpret_cast<float*>(b + w.off_dist_keys);
  float* key_s = reinterpret_cast<float*>(b + w.off_keys_sorted);
  int* idx = reinterpret_cast<int*>(b + w.off_idx);
  int* idx_s = reinterpret_cast<int*>(b + w.off_idx_sorted);
  int* lab = reinterpret_cast<int*>(b + w.off_lab);
  long long* cum = reinterpret_cast<long long*>(b + w.off_cum);
  unsigned long long* first = reinterpret_cast<unsigned long long*>(b + w.off_first);
  void* tmp = b + w.off_tmp;
  hipLaunchKernelGGL(k_pair_dist, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, a, p, n, dim,
                     dists, key, idx);
  size_t tb = w.tmp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key_s, idx, idx_s, (int)n, 0, 32, st);
  if (e != hipSuccess) return e;
  const unsigned g = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_gather_labels, dim3(g), dim3(256), 0, st, idx_s, labels, n, lab);
  tb = w.tmp_bytes;
  e = hipcub::DeviceScan::InclusiveSum(tmp, tb, lab, cum, (int)n, st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(first, 0xFF, 8, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_threshold, dim3(g), dim3(256), 0, st, cum, n, first);
  hipLaunchKernelGGL(k_fpr, dim3(1), dim3(1), 0, st, cum, n, first, fpr);
  return hipGetLastError();
}
