// Shared device/host helpers for the gfx950 descriptor kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define HN_DEV __device__ __forceinline__

// Split an fp32 value into bf16 hi + bf16 lo (x ~= hi + lo to ~16 mantissa bits).
// The product a*b is then evaluated on the bf16 MFMA as ah*bh + ah*bl + al*bh
// ("bf16x3"); the dropped al*bl term is ~2^-16 relative (1.1e-5 max
// abs on the descriptor vs the 1e-4 budget).
HN_DEV void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = (__bf16)x;
  lo = (__bf16)(x - (float)hi);
}

// 8 fp32 -> 8 bf16 hi + 8 bf16 lo packed as two 16-byte vectors.
HN_DEV void split8(const float4& a, const float4& b, uint4& hi, uint4& lo) {
  __bf16 h[8], l[8];
  split_bf16(a.x, h[0], l[0]); split_bf16(a.y, h[1], l[1]);
  split_bf16(a.z, h[2], l[2]); split_bf16(a.w, h[3], l[3]);
  split_bf16(b.x, h[4], l[4]); split_bf16(b.y, h[5], l[5]);
  split_bf16(b.z, h[6], l[6]); split_bf16(b.w, h[7], l[7]);
  hi = *reinterpret_cast<const uint4*>(h);
  lo = *reinterpret_cast<const uint4*>(l);
}

HN_DEV bf16x8 as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

HN_DEV f32x16 mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                    f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  return acc;
}

HN_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the 32 lanes of one half-wave (lanes l and l^k for k < 32).
HN_DEV float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
