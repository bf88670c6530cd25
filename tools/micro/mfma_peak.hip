// Microbenchmark: sustained MFMA rate with operands in registers, 1 or 2 waves per SIMD,
// NACC independent accumulators per wave (NACC = 1: a fully dependent chain).  Calibrates the
// MFMA ceiling the conv kernels are measured against.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC, bool BIG>
__global__ __launch_bounds__(256) void k_peak(float* out, int iters, float seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(seed + threadIdx.x * 1e-3f + j); b[j] = (__bf16)(seed - j); }
  f32x16 acc[NACC];
  f32x4 acc4[NACC];
  for (int i = 0; i < NACC; ++i) { acc[i] = f32x16{}; acc4[i] = f32x4{}; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if (BIG) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
      else acc4[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc4[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15] + acc4[i][0];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int NACC, bool BIG>
void run(int cus, float* out, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 40000 / NACC;
  for (int wps = 1; wps <= 2; ++wps) {
    const int grid = cus * wps;  // 4 waves per block
    k_peak<NACC, BIG><<<grid, 256>>>(out, 100, 1.f);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    k_peak<NACC, BIG><<<grid, 256>>>(out, iters, 1.f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double n = (double)NACC * iters * wps;  // MFMAs per SIMD
    const double flops = 2.0 * (BIG ? 32 * 32 * 16 : 16 * 16 * 32) * n * cus * 4;
    printf("{\"mfma\": \"%s\", \"acc_chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.1f, "
           "\"ns_per_mfma_per_simd\": %.3f}\n",
           BIG ? "32x32x16" : "16x16x32", NACC, wps, ms, flops / ms / 1e9, ms * 1e6 / n);
  }
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  (void)hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  run<4, true>(cus, out, e0, e1);
  run<1, true>(cus, out, e0, e1);
  run<4, false>(cus, out, e0, e1);
  run<1, false>(cus, out, e0, e1);
  run<2, false>(cus, out, e0, e1);
  return 0;
}
