// Shared device/host helpers for the gfx950 descriptor kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));  // arithmetic on it emits v_pk_fma_f32

#define HN_DEV __device__ __forceinline__

// ReLU as one integer max: every float with the sign bit set (negative, -0, -NaN) is a negative int, so
// max_i32(bits, 0) = max(x, +0) for each non-NaN x (a +NaN passes through, as torch.relu's does; a NaN
// with the sign bit set becomes +0 where torch.relu would propagate it -- a divergence only for -NaN
// activations, which the eval path's finite weights and inputs do not produce).
// fmaxf(x, 0.f) costs two v_max_f32 when x comes from an MFMA or a load: the compiler first quiets a
// possible signalling NaN (v_max_f32 x, x, x), which was 5-8 % of the fused kernels' instructions.
HN_DEV float relu0(float x) { return __builtin_bit_cast(float, __builtin_elementwise_max(__builtin_bit_cast(int, x), 0)); }
HN_DEV f32x4 relu4(f32x4 v) { return f32x4{relu0(v[0]), relu0(v[1]), relu0(v[2]), relu0(v[3])}; }

// Split an fp32 value into bf16 hi + bf16 lo (x ~= hi + lo to ~16 mantissa bits).
// The product a*b is then evaluated on the bf16 MFMA as ah*bh + ah*bl + al*bh
// ("bf16x3"); the dropped al*bl term is ~2^-16 relative (1.1e-5 max
// abs on the descriptor vs the 1e-4 budget).
HN_DEV void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = (__bf16)x;
  lo = (__bf16)(x - (float)hi);
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// 8 fp32 -> 8 bf16 hi + 8 bf16 lo packed as two 16-byte vectors.  Built as vector
// elements (no local arrays + pointer casts, which hipcc can leave in scratch).
HN_DEV void split8(const float4& a, const float4& b, uint4& hi, uint4& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  bf16x8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (__bf16)v[j];
    l[j] = (__bf16)(v[j] - (float)h[j]);
  }
  hi = __builtin_bit_cast(uint4, h);
  lo = __builtin_bit_cast(uint4, l);
}

HN_DEV bf16x8 as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

// fp16 variant of the split ("fp16x3"): 11-bit halves, so hi + lo carries ~22 bits and the
// dropped lo*lo term is ~2^-22 relative -- used where activations are range-bounded (the
// NAS front: no input_norm, ReLU outputs of O(1)); same MFMA rate as bf16.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// (v_fma_mix{lo,hi}_f16 for the lo half -- one instruction per value -- measured slower on
// gfx950: k_irf 12.3 -> 13.7 ms; so did v_fma_mix_f32 for x - f32(hi), two
// instructions per value instead of three: wang2 17.6 -> 16.8, wang4 20.0 -> 19.4 Mpatches/s)
HN_DEV void split8_f16(const float4& a, const float4& b, uint4& hi, uint4& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  f16x8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (_Float16)v[j];
    l[j] = (_Float16)(v[j] - (float)h[j]);
  }
  hi = __builtin_bit_cast(uint4, h);
  lo = __builtin_bit_cast(uint4, l);
}
HN_DEV f16x8 as_f16x8(const uint4& v) { return __builtin_bit_cast(f16x8, v); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Buffer resource over [base, base + bytes): the descriptor lives in SGPRs, loads take a
// per-lane byte offset (one VGPR) plus a wave-uniform soffset/immediate, so unrolled
// K-loops do not keep one 64-bit address per load live (cdna_hip_programming.md T8/T20).
HN_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
HN_DEV uint4 buf_load16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// a store beyond the resource's byte count is dropped by the hardware (no branch, so the
// compiler's vmcnt accounting stays exact)
HN_DEV void buf_store16(__amdgpu_buffer_rsrc_t r, const uint4& v, unsigned voff, unsigned soff) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, voff, soff, 0);
}

HN_DEV f32x16 mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                    f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  return acc;
}

HN_DEV f32x16 mfma3_f16(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl,
                        f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
  return acc;
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
// the same split-precision product on the 16x16x32 f16 MFMA (4 accumulator entries per lane)
HN_DEV f32x4_t mfma3_f16_16(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, f32x4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  return acc;
}

// Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8); remap so that
// consecutive logical tiles run on the same XCD and share its L2.
HN_DEV int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
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
