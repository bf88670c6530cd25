// k_c12: HardNet input_norm + conv0 + conv1 + conv2 (hardnet/HardNet.py:281-289, 306-310) in
// one kernel, so the two 128 KB/patch activations a0 and a1 never reach HBM: the kernel reads
// the 4 KB patch and writes a2 (64 KB/patch, [P,16,16,64] fp32 NHWC).
//
// Persistent workgroups of 8 waves walk a contiguous range of whole patches, each in 4 bands
// of 4 conv2 output rows, in order.  a0 and a1 live in LDS ring buffers of 10 / 9 rows, so a
// band computes only its 8 new a0 rows and 8 new a1 rows (no halo recompute).  Per band:
//   P1 stem : the new a0 rows on the MFMA (32x32x16 bf16x3, K = 9 taps + the bias in K slot 9
//             against a constant-1 input), ReLU, split to
//             bf16 hi/lo -> ring W0.
//   P2 conv1: the new a1 rows as 16x16x32 bf16x3 MFMA tiles (16 pixels x 16 channels, K = 32
//             channels per tap), each wave owning one 16-channel half with its 9 taps of
//             weights resident in VGPRs; BN+ReLU, split -> ring W1 (even/odd columns split for
//             the stride-2 reads of conv2).
//   P3 conv2: 4 rows x 16 pixels x 64 channels as 16x16x32 tiles, each wave owning one
//             16-channel quarter (weights resident); BN+ReLU -> float4 stores of a2.
// LDS pixel stride 160 B (bf16 hi 64 B | lo 64 B | pad 32 B): every ds_read_b128 of a
// 16x16x32 operand (lane: pixel l & 15, channels 8 (l >> 4) ..) hits 16 distinct 16-byte
// slots per 16-lane group (tests/test_lds_banks.py).  Window stores are widened to b128 with
// permlane swaps.  Two barriers per band: P3 of band b overlaps P1 of band b+1 across waves.
#include "hn_common.h"
#include "hn_internal.h"
#include "hn_preproc.h"

#include <algorithm>
#include <cstdlib>

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int PXB = 160;                // bytes per pixel in W0 / W1
constexpr int W0C = 34, W1C = 33;       // columns (x = -1 .. 32 / -1 .. 31)
// ring geometry for RB2 conv2 output rows per band
template <int RB2>
struct C12Ring {
  static constexpr int NA0 = 2 * RB2 + 2;      // a0 ring rows: a band's conv1 reads 2 RB2 + 2 a0 rows
  static constexpr int NA1 = 2 * RB2 + 1;      // a1 ring rows: a band's conv2 reads 2 RB2 + 1 a1 rows
  static constexpr int W0B = NA0 * W0C * PXB;  // RB2 4: 59,840   RB2 2: 32,640
  static constexpr int W1B = NA1 * W1C * PXB;  // RB2 4: 47,520   RB2 2: 26,400
};

HN_DEV f32x4v mfma16(const uint4& a, const uint4& b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}

HN_DEV uint2 pack_bf16x4(float a, float b, float c, float d, uint2& lo) {
  bf16x4 h, l;
  h[0] = (__bf16)a; l[0] = (__bf16)(a - (float)h[0]);
  h[1] = (__bf16)b; l[1] = (__bf16)(b - (float)h[1]);
  h[2] = (__bf16)c; l[2] = (__bf16)(c - (float)h[2]);
  h[3] = (__bf16)d; l[3] = (__bf16)(d - (float)h[3]);
  lo = __builtin_bit_cast(uint2, l);
  return __builtin_bit_cast(uint2, h);
}

// W1 column slot of a1 column x (x = -1 .. 31): even (x + 1) -> (x + 1) / 2, odd -> 17 + x / 2
HN_DEV int w1_slot(int x) { return ((x + 1) & 1) ? 17 + (x >> 1) : (x + 1) >> 1; }

// ABL (ablation builds for profiling only; 0 in production): bit 6 = phase time stamps (below),
// bit 5 reads every conv2 fragment
// from tap 0 (L1-resident weights), bit 3 skips P1 entirely,
// bit 4 skips the P2/P3 B-fragment LDS reads; bit 0 skips P1's MFMA work,
// bit 1 skips P2's, bit 2 skips P3's (the phases still run their LDS traffic and barriers).
//
// Every wave holds both conv1 16-channel groups (144 VGPRs of weights), so each P2 B fragment
// feeds two output groups.  Configurations (NW waves, RB2 rows per band, WPE waves per SIMD):
//   <8, 4, 2>: one workgroup per CU (107 KB of rings), two waves per SIMD;
//   <4, 4, 1>: one workgroup per CU, one wave per SIMD (512-register file);
//   <4, 2, 2>: two workgroups per CU (59 KB of rings each) with independent barriers, so one
//              workgroup's MFMA phases run while the other waits at a barrier.
// P3I: P3 walks taps, each with both output rows' B fragments (one tap ahead) and the two rows'
// accumulator chains interleaved MFMA by MFMA; conv2 fragments WA taps ahead (P3I = 0: steps
// of one (tap, row), fragments 2 taps ahead).
// P2I: P2 walks taps with both 16-pixel halves' B fragments one tap ahead, so the 4 accumulator
// chains (2 halves x 2 groups) interleave MFMA by MFMA (P2I = 0: steps of one (tap, half), 2
// chains at a time).
// Tried and removed (same-box A/B): P1's operands read during the previous P3 (-1.3 % vs 7,
// nothing on top of PRIO); P1's row computed inside the previous P3 with its MFMAs spread over
// P3's steps (+5-10 %: the register file then holds conv2 fragments only one tap ahead); the
// 29 split-stem products K-packed into two independent MFMAs instead of the dependent mfma3
// chain (+1 %: P1 is not bound by its MFMA latency).
// U8 (preprocessing fused into the patch load): -1 = fp32 [P,1,32,32] input;
// HN_RESIZE_NONE / _CV2_LINEAR / _PIL_BILINEAR = uint8 patches (32x32 / 64x64) resized,
// /255'd and Normalize'd in the load (hn_preproc.h, the same arithmetic as hn_preprocess), so
// the input costs 1 / 4 KiB of HBM per patch and no intermediate fp32 tensor exists.
template <int ABL, int NW, int RB2, int WPE, bool P3I = false, int WA = 2, bool P2I = false, int PRIO = 0,
          int U8 = -1>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_c12(
    const void* __restrict__ in_, float* __restrict__ out, const float* __restrict__ stem_w,
    const float* __restrict__ stem_b, const uint4* __restrict__ w1p, const float* __restrict__ b1,
    const uint4* __restrict__ w2p, const float* __restrict__ b2, int P, float eps, float pmean,
    float pstd, int pnorm) {
  constexpr int NA0 = C12Ring<RB2>::NA0, NA1 = C12Ring<RB2>::NA1;
  constexpr int W0B = C12Ring<RB2>::W0B, W1B = C12Ring<RB2>::W1B;
  __shared__ __attribute__((aligned(16))) char s_w0[W0B];
  __shared__ __attribute__((aligned(16))) char s_w1[W1B];
  __shared__ float s_in[34 * 34];
  __shared__ float red[2 * NW];
  // P3: RB2 / 2 wave sets, each taking two output rows (set s: rows s and s + RB2 / 2); the
  // NCH2 waves of a set split the 4 16-channel quarters, G2 each
  constexpr int NSET = RB2 / 2, NCH2 = NW / NSET, G2 = 4 / NCH2;
  constexpr int G1 = 2, NCH1 = 2 / G1;  // conv1 output groups per wave / waves sharing a P2 unit
  static_assert(NSET * NCH2 == NW && G2 * NCH2 == 4, "P3 work split");
  // XST (the 4-wave, 2-row-band form): P3's a2 tile leaves through an LDS staging buffer so that each
  // store instruction writes 4 whole 256-byte pixel rows (1 KB contiguous) instead of 16 64-byte
  // quarters; 16-byte chunk q of pixel x at slot q ^ (x & 7) (the P3 writes and the read-back are
  // conflict-free).  The read-back + stores of band b run after the next band's P1 barrier (no extra
  // barrier; the buffer is rewritten only after the following one).
  constexpr bool XST = NW == 4 && NSET == 1 && G2 == 1 && (ABL & 192) == 0;
  __shared__ __attribute__((aligned(16))) float s_st[XST ? 2 * 16 * 64 : 4];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r32 = lane & 31, h32 = lane >> 5;  // 32x32x16 lane roles (stem)
  const int c16 = lane & 15, g16 = lane >> 4;  // 16x16x32 lane roles (conv1/conv2)

  // whole patches per workgroup (contiguous), their 4 bands in order: consecutive bands
  // share a0 / a1 rows, which stay in the LDS ring buffers (no halo recompute)
  const long per = ((long)P + gridDim.x - 1) / gridDim.x;
  const long pb = (long)xcd_remap(blockIdx.x, gridDim.x) * per;
  const long pe = min((long)P, pb + per);
  if (pb >= pe) return;  // workgroup-uniform

  // ---- one-time init: zero both windows (borders and never-written slots stay zero) ----
  for (int i = t; i < W0B / 16; i += NW * 64) reinterpret_cast<uint4*>(s_w0)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < W1B / 16; i += NW * 64) reinterpret_cast<uint4*>(s_w1)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < 34 * 34; i += NW * 64) s_in[i] = 0.f;

  // stem A operand (32x32x16): lane (channel r32, taps 8*h32 ..), bf16 hi/lo
  // (kept in LDS, [lane][hi|lo], read once per P1 row: frees 8 VGPRs for the P3 pipeline)
  __shared__ __attribute__((aligned(16))) uint4 s_stem[64][2];
  if (t < 64) {
    bf16x8 sah, sal;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // K slot 9 carries the bias (its B input is 1.0)
      const int tap = 8 * h32 + j;
      const float v = tap < 9 ? stem_w[tap * 32 + r32] : (tap == 9 ? stem_b[r32] : 0.f);
      sah[j] = (__bf16)v;
      sal[j] = (__bf16)(v - (float)sah[j]);
    }
    s_stem[lane][0] = __builtin_bit_cast(uint4, sah);
    s_stem[lane][1] = __builtin_bit_cast(uint4, sal);
  }
  // conv1 / conv2 A operands resident in registers: [tap][group][plane]
  const int cs1 = w % NCH1, cs2 = w % NCH2;
  uint4 a1w[9][G1][2];
  // biases in LDS (read in the epilogues; frees their registers)
  // (the stem bias too: a global load in P1 would queue behind the previous P3's output
  // stores in the in-order vmcnt counter)
  __shared__ __attribute__((aligned(16))) float s_b0[32], s_b1[32], s_b2[64];
  for (int i = t; i < 128; i += NW * 64) {
    if (i < 32) s_b0[i] = stem_b[i];
    else if (i < 64) s_b1[i - 32] = b1[i - 32];
    else s_b2[i - 64] = b2[i - 64];
  }
#pragma unroll
  for (int g = 0; g < G1; ++g) {
    const int chh = cs1 * G1 + g;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) a1w[tap][g][pl] = w1p[((tap * 2 + chh) * 2 + pl) * 64 + lane];
  }
  // conv2 A fragments are streamed from L2 per tap (2 taps ahead): the register file holds
  // both conv1 groups instead, so each P2 B fragment feeds two output groups
  auto w2_frag = [&](int tap, int g, int pl) {
    if constexpr ((ABL & 32) != 0) tap = 0;  // timing only: L1-resident conv2 fragments
    int i = ((tap * 4 + cs2 * G2 + g) * 2 + pl) * 64 + lane;
    asm volatile("" : "+v"(i));  // keep the load here (not hoisted out of the patch loop)
    return w2p[i];
  };

  // P1 operands of a0 row y: the im2col taps (K slot 9 = 1.0 carries the bias) and the stem A
  auto p1_fetch = [&](int y, float (&xv)[8], uint4& sa0, uint4& sa1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tap = 8 * h32 + j;
      xv[j] = tap < 9 ? s_in[(y + tap / 3) * 34 + r32 + tap % 3] : (tap == 9 ? 1.f : 0.f);
    }
    sa0 = s_stem[lane][0];
    sa1 = s_stem[lane][1];
  };
  // P1 epilogue: ReLU, split to bf16 hi/lo, a0 row y -> its W0 ring slot
  auto p1_store = [&](int y, const f32x16& c0) {
    char* rowp = s_w0 + ((y + 1) % NA0) * W0C * PXB;
    // lane (px, h) holds channels 8q + 4h .. +3; permlane32_swap pairs (q, q+1) so that
    // lanes 0-31 hold channels 8q .. 8q+7 and lanes 32-63 channels 8q+8 .. 8q+15 of the
    // same pixel (T21): 4 ds_write_b128 instead of 8 ds_write_b64
    uint2 hi[4], lo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)  // (the bias came in through K slot 9)
      hi[q] = pack_bf16x4(fmaxf(c0[4 * q], 0.f), fmaxf(c0[4 * q + 1], 0.f), fmaxf(c0[4 * q + 2], 0.f),
                          fmaxf(c0[4 * q + 3], 0.f), lo[q]);
    char* o = rowp + (r32 + 1) * PXB + 16 * h32;
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      auto sw = [](uint2& a, uint2& b) {
        const auto rx = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
        a.x = rx[0]; b.x = rx[1]; a.y = ry[0]; b.y = ry[1];
      };
      sw(hi[k], hi[k + 1]);
      sw(lo[k], lo[k + 1]);
      *reinterpret_cast<uint4*>(o + 16 * k) = make_uint4(hi[k].x, hi[k].y, hi[k + 1].x, hi[k + 1].y);
      *reinterpret_cast<uint4*>(o + 64 + 16 * k) = make_uint4(lo[k].x, lo[k].y, lo[k + 1].x, lo[k + 1].y);
    }
  };
  // ABL bit 6 (timing only): per-wave s_memtime stamps at the phase boundaries of every band of
  // the workgroup's third patch, written past the sub-chunk's a2 output and the head input that
  // follows it (out + P * 24576 floats: tools/c12_timeline.py gives the workspace that much room)
  long long* const dbg =
      reinterpret_cast<long long*>(out + (long)P * 24576) + ((long)blockIdx.x * NW + w) * 128;
  long patch_ts = -1;
#define HN_C12_TS(K)                                                                        \
  if constexpr ((ABL & 192) != 0) {                                                          \
    if (patch == patch_ts && lane == 0) dbg[band * 6 + (K)] = (long long)__builtin_amdgcn_s_memtime(); \
  }
#define HN_C12_TS2(K)                                                                       \
  if constexpr ((ABL & 128) != 0) {                                                         \
    if (patch == patch_ts && lane == 0) dbg[48 + band * 4 + (K)] = (long long)__builtin_amdgcn_s_memtime(); \
  }
  // the next patch's pixels are fetched one patch ahead (U8: its raw bytes; resized at use)
  constexpr int PPT = 1024 / (NW * 64);  // patch pixels per thread (2 or 4)
  typedef float pxv __attribute__((ext_vector_type(PPT)));
  const float* in = static_cast<const float*>(in_);
  const uint8_t* in8 = static_cast<const uint8_t*>(in_);
  constexpr int INB = U8 == HN_RESIZE_NONE ? 1024 : 4096;  // bytes per uint8 patch
  const int py = (PPT * t) >> 5, px = (PPT * t) & 31;      // this thread's pixels (py, px ..)
  pxv vnext;
  hnpre::U8Px<U8 < 0 ? HN_RESIZE_NONE : U8, PPT> rnext;
  if constexpr (U8 < 0)
    vnext = reinterpret_cast<const pxv*>(in + pb * 1024)[t];
  else
    rnext.load(in8 + pb * INB, py, px);
  long pend_patch = -1;  // XST: the band whose a2 rows wait in s_st (patch, first row)
  int pend_row = 0;
  auto xst_flush = [&]() {  // wave w: row w >> 1, pixels 8 (w & 1) + (lane >> 4) + 4 j, chunk lane & 15
    const int ry = w >> 1, q = lane & 15;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int x = 8 * (w & 1) + (lane >> 4) + 4 * j;
      const f32x4v v = *reinterpret_cast<const f32x4v*>(s_st + ((ry * 16 + x) * 16 + (q ^ (x & 7))) * 4);
      *reinterpret_cast<f32x4v*>(out + ((pend_patch * 16 + pend_row + ry) * 16 + x) * 64 + 4 * q) = v;
    }
  };
#pragma unroll 1
  for (long patch = pb; patch < pe; ++patch) {
    if constexpr ((ABL & 192) != 0) patch_ts = pb + 2;
    {
      pxv v;
      if constexpr (U8 < 0) {
        v = vnext;
        if (patch + 1 < pe) vnext = reinterpret_cast<const pxv*>(in + (patch + 1) * 1024)[t];
      } else {
        int q[PPT];
        rnext.resized(py, px, q);
#pragma unroll
        for (int j = 0; j < PPT; ++j) v[j] = hnpre::to_input(q[j], pmean, pstd, pnorm);
        if (patch + 1 < pe) rnext.load(in8 + (patch + 1) * INB, py, px);
      }
      float mean = 0.f, sd = 1.f;
      if (eps >= 0.f) {  // input_norm: (x - mean) / (std_unbiased + eps), HardNet.py:306-310
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < PPT; ++j) a += v[j];
        const float s = wave_sum(a);
        if (lane == 0) red[w] = s;
        __syncthreads();  // (also: every wave is past the previous patch's P1 reads of s_in)
        a = 0.f;
#pragma unroll
        for (int i = 0; i < NW; ++i) a += red[i];
        mean = a * (1.f / 1024.f);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < PPT; ++j) q += (v[j] - mean) * (v[j] - mean);
        q = wave_sum(q);
        if (lane == 0) red[NW + w] = q;
        __syncthreads();
        a = 0.f;
#pragma unroll
        for (int i = 0; i < NW; ++i) a += red[NW + i];
        sd = sqrtf(a * (1.f / 1023.f)) + eps;
      } else {
        __syncthreads();
      }
      const float inv = 1.f / sd;  // as k_conv_ws's stem: (x - mean) * (1/sd)
      const int q0 = PPT * t, y = q0 >> 5, x = q0 & 31;
#pragma unroll
      for (int j = 0; j < PPT; ++j) s_in[(y + 1) * 34 + x + 1 + j] = (v[j] - mean) * inv;
      __syncthreads();
    }
#pragma unroll 1
  for (int band = 0; band < 16 / RB2; ++band) {
    HN_C12_TS(0);
    const int r0 = band * RB2;
    // PRIO & 3: wave priority raised over P1 -- a short serial latency chain that every wave of
    // the workgroup waits for at the next barrier -- so its VALU and MFMA issue ahead of the
    // other workgroup's waves on the same SIMD (MI355X_MICROARCH.md, two waves per SIMD, item 4);
    // PRIO >> 2: P3's level (P3 -> P1 -> barrier)
    if constexpr ((PRIO & 3) != 0) __builtin_amdgcn_s_setprio(PRIO & 3);
    // ---- P1: the band's new a0 rows -> W0 ring (slot (y + 1) % NA0) ------------------------
    // band 0: rows -1 .. 8 (row -1 is conv1's zero padding); band b: rows 8b+1 .. 8b+8
    const int ybeg = band == 0 ? -1 : 2 * RB2 * band + 1, nrows = band == 0 ? 2 * RB2 + 2 : 2 * RB2;
#pragma unroll 1
    for (int ri = w; ri < ((ABL & 8) ? 0 : nrows); ri += NW) {
      const int y = ybeg + ri;  // a0 row
      char* rowp = s_w0 + ((y + 1) % NA0) * W0C * PXB;
      if (y < 0 || y >= 32) {  // zero padding row (interior columns)
        for (int i = lane; i < 32 * (PXB / 16); i += 64)
          reinterpret_cast<uint4*>(rowp + PXB)[i] = make_uint4(0, 0, 0, 0);
        continue;
      }
      float xv[8];
      uint4 sa0, sa1;
      p1_fetch(y, xv, sa0, sa1);
      bf16x8 xh, xl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[j] = (__bf16)xv[j];
        xl[j] = (__bf16)(xv[j] - (float)xh[j]);
      }
      if constexpr ((ABL & 128) != 0) {  // sub-stamp a: operands read and split
        asm volatile("" ::"v"(xh[0]), "v"(xl[7]));
        HN_C12_TS2(0);
      }
      const f32x16 c0 = (ABL & 1) ? f32x16{} : mfma3(as_bf16x8(sa0), as_bf16x8(sa1), xh, xl, f32x16{});
      if constexpr ((ABL & 128) != 0) {  // sub-stamp b: the MFMA chain's result is available
        float z = c0[0] + c0[15];
        asm volatile("" : "+v"(z));
        if (z == 1234.5f) dbg[127] = 0;
        HN_C12_TS2(1);
      }
      p1_store(y, c0);
      HN_C12_TS2(2);  // sub-stamp c: epilogue issued (the stamp's wait also drains the LDS stores)
    }
    HN_C12_TS(1);
    if constexpr (PRIO != 0) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    HN_C12_TS(2);
    if constexpr (XST) {  // the previous band's a2 rows (every wave's P3 staging writes are past the barrier)
      if (pend_patch >= 0) xst_flush();
    }

    // ---- P2: conv1 -> W1 ring (units: new a1 row, both 16-pixel halves; G1 groups) ----------
    // band b: a1 rows 2 RB2 b .. + 2 RB2 - 1 (+ row -1, conv2's zero padding, in band 0).  The two halves
    // are independent accumulator chains interleaved on the MFMA pipe (a single chain of
    // dependent 16x16x32 MFMAs issues at ~half rate).
    const int y1beg = 2 * RB2 * band;
    if (band == 0 && w < NCH1) {  // zero padding row -1 of a1: this wave's channel groups
      char* zrow = s_w1 + (0 * W1C) * PXB;
#pragma unroll
      for (int hx = 0; hx < 2; ++hx)
#pragma unroll
        for (int g = 0; g < G1; ++g) {
          char* dst = zrow + w1_slot(16 * hx + c16) * PXB + 32 * (cs1 * G1 + g) + 8 * g16;
          *reinterpret_cast<uint2*>(dst) = make_uint2(0, 0);
          *reinterpret_cast<uint2*>(dst + 64) = make_uint2(0, 0);
        }
    }
#pragma unroll 1
    for (int u = w / NCH1; u < 2 * RB2; u += NW / NCH1) {
      const int y1 = y1beg + u;
      f32x4v acc[2][G1];
#pragma unroll
      for (int g = 0; g < G1; ++g)  // the bias is the chains' initial accumulator
        acc[0][g] = acc[1][g] = *reinterpret_cast<const f32x4v*>(s_b1 + 16 * (cs1 * G1 + g) + 4 * g16);
      // the 3 a0 rows y1 - 1 .. y1 + 1 sit in ring slots (y1 + dy) % NA0; half 1 is 16 columns on
      const char* srow[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) srow[dy] = s_w0 + (((y1 + dy) % NA0) * W0C + c16) * PXB + 16 * g16;
      if constexpr (P2I) {
        // taps: both halves' B fragments one tap ahead; the 2 x G1 accumulator chains are
        // interleaved MFMA by MFMA (dependent distance 2 G1 instead of G1)
        uint4 bq[2][2][2];  // [buffer][half][plane]
        auto bptr = [&](int tn, int hn) { return srow[tn / 3] + (tn % 3 + 16 * hn) * PXB; };
#pragma unroll
        for (int hn = 0; hn < 2; ++hn) {
          bq[0][hn][0] = *reinterpret_cast<const uint4*>(bptr(0, hn));
          bq[0][hn][1] = *reinterpret_cast<const uint4*>(bptr(0, hn) + 64);
        }
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          if (tap + 1 < 9) {
#pragma unroll
            for (int hn = 0; hn < 2; ++hn) {
              bq[(tap + 1) & 1][hn][0] = *reinterpret_cast<const uint4*>(bptr(tap + 1, hn));
              bq[(tap + 1) & 1][hn][1] = *reinterpret_cast<const uint4*>(bptr(tap + 1, hn) + 64);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          const uint4(&b)[2][2] = bq[tap & 1];
          if constexpr ((ABL & 2) != 0) {
#pragma unroll
            for (int g = 0; g < G1; ++g)
#pragma unroll
              for (int hx = 0; hx < 2; ++hx) acc[hx][g][0] += __builtin_bit_cast(float, b[hx][0].x ^ b[hx][1].y);
            continue;
          }
#pragma unroll
          for (int g = 0; g < G1; ++g)
#pragma unroll
            for (int hx = 0; hx < 2; ++hx) acc[hx][g] = mfma16(a1w[tap][g][1], b[hx][0], acc[hx][g]);
#pragma unroll
          for (int g = 0; g < G1; ++g)
#pragma unroll
            for (int hx = 0; hx < 2; ++hx) acc[hx][g] = mfma16(a1w[tap][g][0], b[hx][1], acc[hx][g]);
#pragma unroll
          for (int g = 0; g < G1; ++g)
#pragma unroll
            for (int hx = 0; hx < 2; ++hx) acc[hx][g] = mfma16(a1w[tap][g][0], b[hx][0], acc[hx][g]);
        }
      } else {
      // steps j = (tap, half): B fragments one step ahead (two register sets); each feeds
      // the G1 groups, and consecutive steps alternate between the two halves' chains
      uint4 bh[2], bl[2];
      bh[0] = *reinterpret_cast<const uint4*>(srow[0]);
      bl[0] = *reinterpret_cast<const uint4*>(srow[0] + 64);
#pragma unroll
      for (int j = 0; j < 18; ++j) {
        const int tap = j >> 1, hx = j & 1;
        if (j + 1 < 18) {
          const int tn = (j + 1) >> 1, hn = (j + 1) & 1;
          const char* p = srow[tn / 3] + (tn % 3 + 16 * hn) * PXB;
          bh[(j + 1) & 1] = *reinterpret_cast<const uint4*>(p);
          bl[(j + 1) & 1] = *reinterpret_cast<const uint4*>(p + 64);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the next step's reads ahead of these MFMAs
#pragma unroll
        for (int g = 0; g < G1; ++g) {
          if (ABL & 2) {
            acc[hx][g][0] += __builtin_bit_cast(float, bh[j & 1].x ^ bl[j & 1].y);
          } else {
            acc[hx][g] = mfma16(a1w[tap][g][1], bh[j & 1], acc[hx][g]);
            acc[hx][g] = mfma16(a1w[tap][g][0], bl[j & 1], acc[hx][g]);
            acc[hx][g] = mfma16(a1w[tap][g][0], bh[j & 1], acc[hx][g]);
          }
        }
      }
      }
      char* prow = s_w1 + ((y1 + 1) % NA1) * W1C * PXB;
#pragma unroll
      for (int hx = 0; hx < 2; ++hx) {
        char* pix = prow + w1_slot(16 * hx + c16) * PXB;
#pragma unroll
        for (int g = 0; g < G1; ++g) {
          const f32x4v r = __builtin_elementwise_max(acc[hx][g], f32x4v{});
          // lane (c, g16) holds channels 4g16 .. +3; permlane16_swap (odd rows of vdst <-> even
          // rows of src) leaves the even row with hi channels 4g16 .. +7 and the odd row with lo
          // channels 4g16-4 .. +3: one ds_write_b128 per lane instead of two ds_write_b64
          uint2 lo;
          uint2 hi = pack_bf16x4(r[0], r[1], r[2], r[3], lo);
          const auto rx = __builtin_amdgcn_permlane16_swap(hi.x, lo.x, false, false);
          const auto ry = __builtin_amdgcn_permlane16_swap(hi.y, lo.y, false, false);
          hi.x = rx[0]; lo.x = rx[1]; hi.y = ry[0]; lo.y = ry[1];
          char* d16 = pix + 32 * (cs1 * G1 + g) + 16 * (g16 >> 1) + 64 * (g16 & 1);
          *reinterpret_cast<uint4*>(d16) = make_uint4(hi.x, hi.y, lo.x, lo.y);
        }
      }
    }
    HN_C12_TS(3);
    // the first WA taps of this wave's conv2 fragments, in flight across the barrier
    uint4 wq[WA + 1][G2][2];
#pragma unroll
    for (int tap = 0; tap < WA; ++tap)
#pragma unroll
      for (int g = 0; g < G2; ++g)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) wq[tap][g][pl] = w2_frag(tap, g, pl);
    __syncthreads();
    HN_C12_TS(4);

    if constexpr ((PRIO >> 2) != 0) __builtin_amdgcn_s_setprio((PRIO >> 2) & 3);  // P3 too (P3 -> P1 -> barrier)
    // ---- P3: conv2 (stride 2) -> a2 in HBM (units: output rows oy and oy + 2 together; this
    // wave's G2 quarters) ----------------------------------------------------------------------
    {
      const int oy0 = w / NCH2;  // rows oy0 and oy0 + NSET
      f32x4v acc[2][G2];
#pragma unroll
      for (int g = 0; g < G2; ++g)  // the bias is the chains' initial accumulator
        acc[0][g] = acc[1][g] = *reinterpret_cast<const f32x4v*>(s_b2 + 16 * (cs2 * G2 + g) + 4 * g16);
      // output column c16 reads a1 column 2*c16 - 1 + dx: W1 slot c16 (dx 0), 17 + c16 (dx 1),
      // c16 + 1 (dx 2); a1 rows 2 (r0 + oy) - 1 + dy sit in ring slots (2 (r0 + oy) + dy) % NA1
      const char* srow[2][3];
#pragma unroll
      for (int ry = 0; ry < 2; ++ry)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
          srow[ry][dy] = s_w1 + (((2 * (r0 + oy0 + NSET * ry) + dy) % NA1) * W1C + c16) * PXB + 16 * g16;
      if constexpr (P3I) {
        // taps: both rows' B fragments one tap ahead; conv2 fragments WA taps ahead
        auto bptr = [&](int tn, int rn) {
          const int dy = tn / 3, dx = tn % 3;
          return srow[rn][dy] + (dx == 1 ? 17 : (dx >> 1)) * PXB;
        };
        uint4 bf[2][2][2];  // [buffer][row][plane]
#pragma unroll
        for (int rn = 0; rn < 2; ++rn) {
          bf[0][rn][0] = *reinterpret_cast<const uint4*>(bptr(0, rn));
          bf[0][rn][1] = *reinterpret_cast<const uint4*>(bptr(0, rn) + 64);
        }
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          if (tap + WA < 9) {
#pragma unroll
            for (int g = 0; g < G2; ++g)
#pragma unroll
              for (int pl = 0; pl < 2; ++pl) wq[(tap + WA) % (WA + 1)][g][pl] = w2_frag(tap + WA, g, pl);
          }
          if (tap + 1 < 9) {
#pragma unroll
            for (int rn = 0; rn < 2; ++rn) {
              bf[(tap + 1) & 1][rn][0] = *reinterpret_cast<const uint4*>(bptr(tap + 1, rn));
              bf[(tap + 1) & 1][rn][1] = *reinterpret_cast<const uint4*>(bptr(tap + 1, rn) + 64);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          const uint4(&b)[2][2] = bf[tap & 1];
#pragma unroll
          for (int g = 0; g < G2; ++g) {
            const uint4* wc = wq[tap % (WA + 1)][g];
            acc[0][g] = mfma16(wc[1], b[0][0], acc[0][g]);
            acc[1][g] = mfma16(wc[1], b[1][0], acc[1][g]);
            acc[0][g] = mfma16(wc[0], b[0][1], acc[0][g]);
            acc[1][g] = mfma16(wc[0], b[1][1], acc[1][g]);
            acc[0][g] = mfma16(wc[0], b[0][0], acc[0][g]);
            acc[1][g] = mfma16(wc[0], b[1][0], acc[1][g]);
          }
        }
      } else {
      // steps j = (tap, row): B fragments one step ahead; conv2 fragments 2 taps ahead
      uint4 bh[2], bl[2];
      bh[0] = *reinterpret_cast<const uint4*>(srow[0][0]);
      bl[0] = *reinterpret_cast<const uint4*>(srow[0][0] + 64);
#pragma unroll
      for (int j = 0; j < 18; ++j) {
        const int tap = j >> 1, ry = j & 1;
        if (ry == 0 && tap + WA < 9) {
#pragma unroll
          for (int g = 0; g < G2; ++g)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) wq[(tap + WA) % (WA + 1)][g][pl] = w2_frag(tap + WA, g, pl);
        }
        if (j + 1 < 18) {
          const int tn = (j + 1) >> 1, rn = (j + 1) & 1;
          const int dy = tn / 3, dx = tn % 3;
          const char* p = srow[rn][dy] + (dx == 1 ? 17 : (dx >> 1)) * PXB;
          bh[(j + 1) & 1] = *reinterpret_cast<const uint4*>(p);
          bl[(j + 1) & 1] = *reinterpret_cast<const uint4*>(p + 64);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < G2; ++g) {
          if (ABL & 4) {
            acc[ry][g][0] += __builtin_bit_cast(float, bh[j & 1].x ^ bl[j & 1].y);
          } else {
            const uint4* wc = wq[tap % (WA + 1)][g];
            acc[ry][g] = mfma16(wc[1], bh[j & 1], acc[ry][g]);
            acc[ry][g] = mfma16(wc[0], bl[j & 1], acc[ry][g]);
            acc[ry][g] = mfma16(wc[0], bh[j & 1], acc[ry][g]);
          }
        }
      }
      }
      if constexpr (XST) {
#pragma unroll
        for (int ry = 0; ry < 2; ++ry)
          *reinterpret_cast<f32x4v*>(s_st + ((ry * 16 + c16) * 16 + ((4 * cs2 + g16) ^ (c16 & 7))) * 4) =
              __builtin_elementwise_max(acc[ry][0], f32x4v{});
        pend_patch = patch;
        pend_row = r0 + oy0;
      } else {
#pragma unroll
      for (int ry = 0; ry < 2; ++ry) {
        float* o = out + ((patch * 16 + r0 + oy0 + NSET * ry) * 16 + c16) * 64 + 4 * g16;
#pragma unroll
        for (int g = 0; g < G2; ++g)
          *reinterpret_cast<f32x4v*>(o + 16 * (cs2 * G2 + g)) =
              __builtin_elementwise_max(acc[ry][g], f32x4v{});
      }
      }
    }
    HN_C12_TS(5);
    // no barrier: the next band's P1 writes only W0, which P3 does not read; its first
    // barrier orders this P3's W1 reads before the next P2's W1 writes
  }  // band
  }  // patch
  if constexpr (XST) {  // the last band's rows
    __syncthreads();
    xst_flush();
  }
}


#ifdef HN_EXPERIMENTS  // measured slower than k_c12 cfg 12 (24.2 vs 20.4 ms per step, same box): experiments library only
// ------------------------------------------------------------------------------------------
// k_c12h: the same computation with the roles split per SIMD.  One workgroup per CU of 8 waves:
// waves 0-3 (one per SIMD, 256-register budget) run only conv1 (P2) and conv2 (P3) of band g on
// the MFMA; waves 4-7 (the SIMDs' second waves) run the stem (P1) of band g + 1, the next patch's
// input_norm and the stores of band g - 1's a2 rows meanwhile.  In k_c12 every wave runs P1 -> P2
// -> P3 in sequence and P1 (3 % of the MFMA work, a latency chain of LDS reads, split, 3 MFMAs,
// split, LDS stores) costs ~17 % of each band on every SIMD; here it runs beside the MFMA stream.
// Two barriers per band: X_g (W1 rows of band g complete) and E_g (band g's a2 tile staged, band
// g + 1's W0 rows complete).  Rings: W0 12 rows (P1 of band g + 1 -- or of the next patch's band 0
// -- writes while P2 of band g reads), W1 5 rows; conv1's A fragments in LDS (the 4 MFMA waves
// read the same ones), conv2's quarter of each MFMA wave resident in its registers.
// U8: as k_c12 (the patch load preprocesses uint8 patches; -1 = fp32).
template <int U8 = -1>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_c12h(
    const void* __restrict__ in_, float* __restrict__ out, const float* __restrict__ stem_w,
    const float* __restrict__ stem_b, const uint4* __restrict__ w1p, const float* __restrict__ b1,
    const uint4* __restrict__ w2p, const float* __restrict__ b2, int P, float eps, float pmean, float pstd,
    int pnorm) {
  constexpr int NA0 = 12, NA1 = 5;
  __shared__ __attribute__((aligned(16))) char s_w0[NA0 * W0C * PXB];
  __shared__ __attribute__((aligned(16))) char s_w1[NA1 * W1C * PXB];
  __shared__ __attribute__((aligned(16))) uint4 s_a1w[9 * 2 * 2 * 64];  // conv1 A fragments [tap][g][plane][lane]
  __shared__ __attribute__((aligned(16))) float s_in[2][34 * 34];      // normalised patch, by patch parity
  __shared__ __attribute__((aligned(16))) uint4 s_stem[64][2];
  __shared__ __attribute__((aligned(16))) float s_st[2 * 16 * 64];     // a2 staging (k_c12's XST)
  __shared__ __attribute__((aligned(16))) float s_b1[32], s_b2[64];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool mw = w < 4;  // MFMA wave (one per SIMD)
  const int hw = w & 3;   // index within the role
  const int r32 = lane & 31, h32 = lane >> 5;
  const int c16 = lane & 15, g16 = lane >> 4;

  const long per = ((long)P + gridDim.x - 1) / gridDim.x;
  const long pb = (long)xcd_remap(blockIdx.x, gridDim.x) * per;
  const long pe = min((long)P, pb + per);
  if (pb >= pe) return;  // workgroup-uniform
  const long G = (pe - pb) * 8;  // bands (2 conv2 rows each)

  // ---- one-time init ----
  for (int i = t; i < NA0 * W0C * PXB / 16; i += 512) reinterpret_cast<uint4*>(s_w0)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < NA1 * W1C * PXB / 16; i += 512) reinterpret_cast<uint4*>(s_w1)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < 2 * 34 * 34; i += 512) (&s_in[0][0])[i] = 0.f;
  for (int i = t; i < 9 * 2 * 2 * 64; i += 512) s_a1w[i] = w1p[i];
  if (t < 64) {
    bf16x8 sah, sal;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // K slot 9 carries the bias (its B input is 1.0)
      const int tap = 8 * h32 + j;
      const float v = tap < 9 ? stem_w[tap * 32 + r32] : (tap == 9 ? stem_b[r32] : 0.f);
      sah[j] = (__bf16)v;
      sal[j] = (__bf16)(v - (float)sah[j]);
    }
    s_stem[lane][0] = __builtin_bit_cast(uint4, sah);
    s_stem[lane][1] = __builtin_bit_cast(uint4, sal);
  }
  for (int i = t; i < 96; i += 512) {
    if (i < 32) s_b1[i] = b1[i];
    else s_b2[i - 32] = b2[i - 32];
  }

  // W0 slot of a0 row y (-1 .. 32) of the workgroup's patch pl; W1 slot of a1 row y (-1 .. 31)
  auto w0row = [&](long pl, int y) { return s_w0 + (int)((pl * 34 + y + 1) % NA0) * W0C * PXB; };
  auto w1row = [&](int y) { return s_w1 + ((y + 1) % NA1) * W1C * PXB; };

  // ---- helper side: input_norm (wave 4), P1, a2 stores ----
  const float* in = static_cast<const float*>(in_);
  const uint8_t* in8 = static_cast<const uint8_t*>(in_);
  constexpr int INB = U8 == HN_RESIZE_NONE ? 1024 : 4096;
  float4 vn[4];
  hnpre::U8Px<U8 < 0 ? HN_RESIZE_NONE : U8, 4> rn[4];
  auto patch_fetch = [&](long p) {  // lane's 16 pixels: 4 runs of 4 at px = 4 (lane + 64 k)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (U8 < 0) {
        vn[k] = reinterpret_cast<const float4*>(in + p * 1024)[lane + 64 * k];
      } else {
        const int px = 4 * (lane + 64 * k);
        rn[k].load(in8 + p * INB, px >> 5, px & 31);
      }
    }
  };
  auto patch_norm = [&](long p) {  // input_norm (HardNet.py:306-310) of the fetched patch -> s_in[p & 1]
    float v[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (U8 < 0) {
        v[4 * k] = vn[k].x; v[4 * k + 1] = vn[k].y; v[4 * k + 2] = vn[k].z; v[4 * k + 3] = vn[k].w;
      } else {
        const int px = 4 * (lane + 64 * k);
        int q[4];
        rn[k].resized(px >> 5, px & 31, q);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * k + j] = hnpre::to_input(q[j], pmean, pstd, pnorm);
      }
    }
    float mean = 0.f, sd = 1.f;
    if (eps >= 0.f) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) a += v[j];
      mean = wave_sum(a) * (1.f / 1024.f);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) q += (v[j] - mean) * (v[j] - mean);
      sd = sqrtf(wave_sum(q) * (1.f / 1023.f)) + eps;
    }
    const float inv = 1.f / sd;  // as k_c12
    float* si = s_in[p & 1];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int px = 4 * (lane + 64 * k), y = px >> 5, x = px & 31;
#pragma unroll
      for (int j = 0; j < 4; ++j) si[(y + 1) * 34 + x + 1 + j] = (v[4 * k + j] - mean) * inv;
    }
  };
  // P1: the new a0 rows of band g (helper wave hw: rows ri = hw, hw + 4)
  auto p1_band = [&](long g) {
    const long pl = g >> 3;
    const int band = (int)(g & 7);
    const float* si = s_in[(pb + pl) & 1];
    const int ybeg = band == 0 ? -1 : 4 * band + 1, nrows = band == 0 ? 6 : 4;
#pragma unroll 1
    for (int ri = hw; ri < nrows; ri += 4) {
      const int y = ybeg + ri;
      char* rowp = w0row(pl, y);
      if (y < 0 || y >= 32) {  // zero padding row (interior columns)
        for (int i = lane; i < 32 * (PXB / 16); i += 64) reinterpret_cast<uint4*>(rowp + PXB)[i] = make_uint4(0, 0, 0, 0);
        continue;
      }
      bf16x8 xh, xl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * h32 + j;
        const float xv = tap < 9 ? si[(y + tap / 3) * 34 + r32 + tap % 3] : (tap == 9 ? 1.f : 0.f);
        xh[j] = (__bf16)xv;
        xl[j] = (__bf16)(xv - (float)xh[j]);
      }
      const f32x16 c0 = mfma3(as_bf16x8(s_stem[lane][0]), as_bf16x8(s_stem[lane][1]), xh, xl, f32x16{});
      uint2 hi[4], lo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        hi[q] = pack_bf16x4(fmaxf(c0[4 * q], 0.f), fmaxf(c0[4 * q + 1], 0.f), fmaxf(c0[4 * q + 2], 0.f),
                            fmaxf(c0[4 * q + 3], 0.f), lo[q]);
      char* o = rowp + (r32 + 1) * PXB + 16 * h32;
#pragma unroll
      for (int k = 0; k < 4; k += 2) {
        auto sw = [](uint2& a, uint2& b) {
          const auto rx = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
          const auto ry = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
          a.x = rx[0]; b.x = rx[1]; a.y = ry[0]; b.y = ry[1];
        };
        sw(hi[k], hi[k + 1]);
        sw(lo[k], lo[k + 1]);
        *reinterpret_cast<uint4*>(o + 16 * k) = make_uint4(hi[k].x, hi[k].y, hi[k + 1].x, hi[k + 1].y);
        *reinterpret_cast<uint4*>(o + 64 + 16 * k) = make_uint4(lo[k].x, lo[k].y, lo[k + 1].x, lo[k + 1].y);
      }
    }
  };
  // a2 rows 2 band .. 2 band + 1 of band g from s_st (k_c12's xst_flush: 4 whole pixel rows per store)
  auto flush = [&](long g) {
    const long patch = pb + (g >> 3);
    const int row0 = 2 * (int)(g & 7), ry = hw >> 1, q = lane & 15;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int x = 8 * (hw & 1) + (lane >> 4) + 4 * j;
      const f32x4v v = *reinterpret_cast<const f32x4v*>(s_st + ((ry * 16 + x) * 16 + (q ^ (x & 7))) * 4);
      *reinterpret_cast<f32x4v*>(out + ((patch * 16 + row0 + ry) * 16 + x) * 64 + 4 * q) = v;
    }
  };

  if (!mw) {
    if (hw == 0) {
      patch_fetch(pb);
      patch_norm(pb);
    }
    __syncthreads();  // B0: s_in of the first patch
    p1_band(0);
    if (hw == 0 && pb + 1 < pe) patch_fetch(pb + 1);
    __syncthreads();  // B1: band 0's W0 rows
#pragma unroll 1
    for (long g = 0; g < G; ++g) {
      // part 1, beside P2(g): band g - 1's a2 rows, P1 of band g + 1
      if (g > 0) flush(g - 1);
      if (g + 1 < G) p1_band(g + 1);
      __syncthreads();  // X_g
      // part 2, beside P3(g): the next patch's input_norm (band 0), its pixels fetched a band ahead
      if (hw == 0 && (g & 7) == 0) {
        const long pn = pb + (g >> 3) + 1;
        if (pn < pe) patch_norm(pn);
        if (pn + 1 < pe) patch_fetch(pn + 1);
      }
      __syncthreads();  // E_g
    }
    flush(G - 1);
    return;
  }

  // ---- MFMA side: P2 (conv1) and P3 (conv2) of every band ----
  uint4 w2r[9][2];  // this wave's conv2 quarter (hw), both planes, resident
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) w2r[tap][pl] = w2p[((tap * 4 + hw) * 2 + pl) * 64 + lane];
  __syncthreads();  // B0
  __syncthreads();  // B1
#pragma unroll 1
  for (long g = 0; g < G; ++g) {
    const long pl = g >> 3;
    const int band = (int)(g & 7);
    // ---- P2: a1 row y1 = 4 band + hw, both 16-pixel halves, both 16-channel groups ----
    {
      const int y1 = 4 * band + hw;
      if (band == 0 && hw == 0) {  // a1 row -1 (conv2's zero padding), every channel
        char* zrow = w1row(-1);
        for (int i = lane; i < W1C * (PXB / 16); i += 64) reinterpret_cast<uint4*>(zrow)[i] = make_uint4(0, 0, 0, 0);
      }
      f32x4v acc[2][2];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
        acc[0][gg] = acc[1][gg] = *reinterpret_cast<const f32x4v*>(s_b1 + 16 * gg + 4 * g16);
      const char* srow[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) srow[dy] = w0row(pl, y1 - 1 + dy) + c16 * PXB + 16 * g16;
      uint4 bq[2][2][2], aq[2][2][2];  // [buffer][half | group][plane]
      auto fetch = [&](int tn, uint4 (&b)[2][2], uint4 (&a)[2][2]) {
#pragma unroll
        for (int hn = 0; hn < 2; ++hn) {
          const char* p = srow[tn / 3] + (tn % 3 + 16 * hn) * PXB;
          b[hn][0] = *reinterpret_cast<const uint4*>(p);
          b[hn][1] = *reinterpret_cast<const uint4*>(p + 64);
        }
#pragma unroll
        for (int gg = 0; gg < 2; ++gg)
#pragma unroll
          for (int pln = 0; pln < 2; ++pln) a[gg][pln] = s_a1w[((tn * 2 + gg) * 2 + pln) * 64 + lane];
      };
      fetch(0, bq[0], aq[0]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) fetch(tap + 1, bq[(tap + 1) & 1], aq[(tap + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const uint4(&b)[2][2] = bq[tap & 1];
        const uint4(&a)[2][2] = aq[tap & 1];
#pragma unroll
        for (int gg = 0; gg < 2; ++gg)
#pragma unroll
          for (int hx = 0; hx < 2; ++hx) acc[hx][gg] = mfma16(a[gg][1], b[hx][0], acc[hx][gg]);
#pragma unroll
        for (int gg = 0; gg < 2; ++gg)
#pragma unroll
          for (int hx = 0; hx < 2; ++hx) acc[hx][gg] = mfma16(a[gg][0], b[hx][1], acc[hx][gg]);
#pragma unroll
        for (int gg = 0; gg < 2; ++gg)
#pragma unroll
          for (int hx = 0; hx < 2; ++hx) acc[hx][gg] = mfma16(a[gg][0], b[hx][0], acc[hx][gg]);
        __builtin_amdgcn_sched_barrier(0);
      }
      char* prow = w1row(y1);
#pragma unroll
      for (int hx = 0; hx < 2; ++hx) {
        char* pix = prow + w1_slot(16 * hx + c16) * PXB;
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const f32x4v r = __builtin_elementwise_max(acc[hx][gg], f32x4v{});
          uint2 lo;
          uint2 hi = pack_bf16x4(r[0], r[1], r[2], r[3], lo);
          const auto rx = __builtin_amdgcn_permlane16_swap(hi.x, lo.x, false, false);
          const auto ry = __builtin_amdgcn_permlane16_swap(hi.y, lo.y, false, false);
          hi.x = rx[0]; lo.x = rx[1]; hi.y = ry[0]; lo.y = ry[1];
          char* d16 = pix + 32 * gg + 16 * (g16 >> 1) + 64 * (g16 & 1);
          *reinterpret_cast<uint4*>(d16) = make_uint4(hi.x, hi.y, lo.x, lo.y);
        }
      }
    }
    __syncthreads();  // X_g
    // ---- P3: conv2 rows 2 band, 2 band + 1, this wave's 16-channel quarter ----
    {
      f32x4v acc[2];
      acc[0] = acc[1] = *reinterpret_cast<const f32x4v*>(s_b2 + 16 * hw + 4 * g16);
      const char* srow[2][3];
#pragma unroll
      for (int ry = 0; ry < 2; ++ry)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) srow[ry][dy] = w1row(2 * (2 * band + ry) - 1 + dy) + c16 * PXB + 16 * g16;
      auto bptr = [&](int tn, int rn) {
        const int dx = tn % 3;
        return srow[rn][tn / 3] + (dx == 1 ? 17 : (dx >> 1)) * PXB;
      };
      uint4 bf[2][2][2];  // [buffer][row][plane]
#pragma unroll
      for (int rn = 0; rn < 2; ++rn) {
        bf[0][rn][0] = *reinterpret_cast<const uint4*>(bptr(0, rn));
        bf[0][rn][1] = *reinterpret_cast<const uint4*>(bptr(0, rn) + 64);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) {
#pragma unroll
          for (int rn = 0; rn < 2; ++rn) {
            bf[(tap + 1) & 1][rn][0] = *reinterpret_cast<const uint4*>(bptr(tap + 1, rn));
            bf[(tap + 1) & 1][rn][1] = *reinterpret_cast<const uint4*>(bptr(tap + 1, rn) + 64);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint4(&b)[2][2] = bf[tap & 1];
        acc[0] = mfma16(w2r[tap][1], b[0][0], acc[0]);
        acc[1] = mfma16(w2r[tap][1], b[1][0], acc[1]);
        acc[0] = mfma16(w2r[tap][0], b[0][1], acc[0]);
        acc[1] = mfma16(w2r[tap][0], b[1][1], acc[1]);
        acc[0] = mfma16(w2r[tap][0], b[0][0], acc[0]);
        acc[1] = mfma16(w2r[tap][0], b[1][0], acc[1]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int ry = 0; ry < 2; ++ry)
        *reinterpret_cast<f32x4v*>(s_st + ((ry * 16 + c16) * 16 + ((4 * hw + g16) ^ (c16 & 7))) * 4) =
            __builtin_elementwise_max(acc[ry], f32x4v{});
    }
    __syncthreads();  // E_g
  }
}
#endif  // HN_EXPERIMENTS

}  // namespace

// HN_C12_CFG variants of the direct k_c12 (12 is the product library's direct-conv1 fallback; the default is
// 15 = k_c12s, hn_c12w.hip).  The experiments library also has the measured-slower forms:
//   0 <8 waves, 4-row bands, 2 waves/SIMD>   1 <4, 4, 1> (512-register file)
//   2 <4 waves, 2-row bands, 2 workgroups/CU>
//   3 / 4: 0 with tap-interleaved P3, conv2 fragments 2 / 3 taps ahead;  5 / 6: the same for 2
//   7 / 8: 2 / 5 with the tap-interleaved P2 (both halves' chains MFMA by MFMA);  9: 0 with it
//   10 / 11: 7 with the P1 wave priority raised to 1 / 3;  12: 7 with P3 and P1 at priority 1
//   13: k_c12h (MFMA / helper waves split per SIMD);  14: k_c12w (conv1 as F(4,3), hn_c12w.hip)
#ifdef HN_EXPERIMENTS
#define HN_C12_CFGS(X)                                                                   \
  X(0, 8, 4, 2, false, 2, false, 0) X(1, 4, 4, 1, false, 2, false, 0) X(2, 4, 2, 2, false, 2, false, 0) \
  X(3, 8, 4, 2, true, 2, false, 0) X(4, 8, 4, 2, true, 3, false, 0) X(5, 4, 2, 2, true, 2, false, 0)     \
  X(6, 4, 2, 2, true, 3, false, 0) X(7, 4, 2, 2, false, 2, true, 0) X(8, 4, 2, 2, true, 2, true, 0)      \
  X(9, 8, 4, 2, false, 2, true, 0) X(10, 4, 2, 2, false, 2, true, 1) X(11, 4, 2, 2, false, 2, true, 3) \
  X(12, 4, 2, 2, false, 2, true, 5)
#else
#define HN_C12_CFGS(X) X(12, 4, 2, 2, false, 2, true, 5)
#endif  // (P1, P3) at priority (2, 1) / (1, 2) / (2, 2): within the box noise of 12, removed

bool hn_c12_cfg_ok(int cfg, int abl) {
  if (cfg == kC12Split) {  // k_c12s (hn_c12w.hip)
#ifdef HN_EXPERIMENTS
    return abl == 0 || abl == 1 || abl == 2 || abl == 4 || abl == 6 || abl == 64 || abl == 65 || abl == 66 || abl == 72 ||
           abl == 80 || abl == 84 || abl == 88 || abl == 116 || abl == 86 || abl == 340 || abl == 576 || abl == 1088;
#else
    return abl == 0;
#endif
  }
#ifdef HN_EXPERIMENTS
  if (cfg == kC12Wino)  // k_c12w (hn_c12w.hip)
    return abl == 0 || abl == 1 || abl == 2 || abl == 4 || abl == 6 || abl == 64 || abl == 192;
  if (cfg < 0 || cfg > 13) return false;
#else
  if (cfg != 12) return false;
#endif
  if (!abl) return true;
#ifdef HN_EXPERIMENTS
  switch (cfg) {
    case 0: return abl == 1 || abl == 6 || abl == 8;
    case 2: return abl == 6 || abl == 8;
    case 12: return abl == 1 || abl == 6 || abl == 8 || abl == 32 || abl == 64 || abl == 192;
  }
#endif
  return false;
}

hipError_t hn_launch_c12(const float* in, float* out, const HardnetDev& d, int P, float eps,
                         hipStream_t st, const HnU8In* u8) {
  if (P <= 0) return hipSuccess;
  // the calling model's HN_C12_CFG (and, in the HN_EXPERIMENTS library, HN_C12_ABL), hn_create
  const int cfg = hn_knobs().c12_cfg;  // same-box A/Bs: 12 2-4 % < 7 1.5 % < 2 4.5 % < 0
  const int abl = hn_knobs().c12_abl;
  if (!hn_c12_cfg_ok(cfg, abl)) return hipErrorInvalidValue;
#ifdef HN_EXPERIMENTS
  if (cfg == kC12Wino) return hn_launch_c12w(in, out, d, P, eps, st, u8, abl);
#endif
  if (cfg == kC12Split) return hn_launch_c12s(in, out, d, P, eps, st, u8);
  if (u8 && ((cfg != 12 && cfg != 13) || abl)) return hipErrorInvalidValue;  // the uint8 loads: production builds only
  const void* fn = nullptr;
  int nw = 0;
  switch (cfg) {
#define HN_C12_FN(C, W, R, E, I, A, Q, PR)                               \
  case C:                                                                \
    fn = reinterpret_cast<const void*>(&k_c12<0, W, R, E, I, A, Q, PR>); \
    nw = W;                                                              \
    break;
    HN_C12_CFGS(HN_C12_FN)
#undef HN_C12_FN
#ifdef HN_EXPERIMENTS
    case 13:
      fn = reinterpret_cast<const void*>(&k_c12h<-1>);
      nw = 8;
      break;
#endif
  }
  if (!fn) return hipErrorInvalidValue;
  int resident = 0;
  const hipError_t e = hn_resident_blocks(fn, nw * 64, 0, &resident);
  if (e != hipSuccess) return e;
  const int grid = (int)std::min<long>((long)P, resident);
  const void* src = u8 ? u8->in : static_cast<const void*>(in);
  const float pm = u8 ? u8->mean : 0.f, ps = u8 ? u8->stdv : 1.f;
  const int pn = u8 ? u8->normalize : 0;
#define HN_C12_GO(A, W, R, E, I, WA, Q, PR, ...)                                                 \
  hipLaunchKernelGGL((k_c12<A, W, R, E, I, WA, Q, PR, ##__VA_ARGS__>), dim3(grid), dim3(W * 64), 0, st, src, \
                     out, d.stem_w, d.stem_b, static_cast<const uint4*>(d.c12_w1), d.bias[1],   \
                     static_cast<const uint4*>(d.c12_w2), d.bias[2], P, eps, pm, ps, pn)
#ifdef HN_EXPERIMENTS
#define HN_C12H_GO(U)                                                                                        \
  hipLaunchKernelGGL((k_c12h<U>), dim3(grid), dim3(512), 0, st, src, out, d.stem_w, d.stem_b,               \
                     static_cast<const uint4*>(d.c12_w1), d.bias[1], static_cast<const uint4*>(d.c12_w2),   \
                     d.bias[2], P, eps, pm, ps, pn)
  if (cfg == 13) {
    if (!u8) HN_C12H_GO(-1);
    else if (u8->resize == HN_RESIZE_NONE) HN_C12H_GO(HN_RESIZE_NONE);
    else if (u8->resize == HN_RESIZE_CV2_LINEAR) HN_C12H_GO(HN_RESIZE_CV2_LINEAR);
    else if (u8->resize == HN_RESIZE_PIL_BILINEAR) HN_C12H_GO(HN_RESIZE_PIL_BILINEAR);
    else return hipErrorInvalidValue;
#undef HN_C12H_GO
    return hipGetLastError();
  }
#endif
  if (u8) {
    switch (u8->resize) {
      case HN_RESIZE_NONE: HN_C12_GO(0, 4, 2, 2, false, 2, true, 5, HN_RESIZE_NONE); break;
      case HN_RESIZE_CV2_LINEAR: HN_C12_GO(0, 4, 2, 2, false, 2, true, 5, HN_RESIZE_CV2_LINEAR); break;
      case HN_RESIZE_PIL_BILINEAR: HN_C12_GO(0, 4, 2, 2, false, 2, true, 5, HN_RESIZE_PIL_BILINEAR); break;
      default: return hipErrorInvalidValue;
    }
  } else if (abl) {
#ifdef HN_EXPERIMENTS
    if (cfg == 0) {
      switch (abl) {
        case 1: HN_C12_GO(1, 8, 4, 2, false, 2, false, 0); break;
        case 6: HN_C12_GO(6, 8, 4, 2, false, 2, false, 0); break;
        case 8: HN_C12_GO(8, 8, 4, 2, false, 2, false, 0); break;
      }
    } else if (cfg == 2) {
      switch (abl) {
        case 6: HN_C12_GO(6, 4, 2, 2, false, 2, false, 0); break;
        case 8: HN_C12_GO(8, 4, 2, 2, false, 2, false, 0); break;
      }
    } else if (cfg == 12) {
      switch (abl) {
        case 1: HN_C12_GO(1, 4, 2, 2, false, 2, true, 5); break;
        case 6: HN_C12_GO(6, 4, 2, 2, false, 2, true, 5); break;
        case 8: HN_C12_GO(8, 4, 2, 2, false, 2, true, 5); break;
        case 32: HN_C12_GO(32, 4, 2, 2, false, 2, true, 5); break;
        case 64: HN_C12_GO(64, 4, 2, 2, false, 2, true, 5); break;
        case 64 + 128: HN_C12_GO(192, 4, 2, 2, false, 2, true, 5); break;
      }
    }
#endif
  } else {
    switch (cfg) {
#define HN_C12_CASE(C, W, R, E, I, A, Q, PR) \
  case C: HN_C12_GO(0, W, R, E, I, A, Q, PR); break;
      HN_C12_CFGS(HN_C12_CASE)
#undef HN_C12_CASE
    }
  }
#undef HN_C12_GO
  return hipGetLastError();
}
