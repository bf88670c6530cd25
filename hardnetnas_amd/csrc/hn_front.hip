// Fused NAS front: the stem ConvBNRelu(1->32, 3x3) (model_supernet.py:57-58,
// fbnet_builder.py:352-404) and the first searched layer (SEARCH_SPACE2[0] = (32, 32, s2),
// lookup_table_builder.py:22-45) in one kernel, so the two 128 KB/patch tensors of the
// 32x32 stage (stem output, pw output) never reach HBM.
//
//   MODE FRONT_IRF:     IRFBlock pw 1x1 (groups, BN, ReLU) [+ ChannelShuffle] -> dw kxk s2
//                       (BN, ReLU) -> pwl 1x1 (groups, BN)  (fbnet_builder.py:455-570);
//                       writes the layer-0 output [P,16,16,32] (SE, if any, follows as k_se).
//   MODE FRONT_MAXPOOL: the "skip" op at stride 2 = MaxPool2d(3, 2, 1)
//                       (fbnet_builder.py:202-228); writes [P,16,16,32].
//
// Persistent workgroups (4 waves) walk whole patches, each in 4 bands of 4 output rows; for
// MID = 32 the pw rows live in an LDS ring shared by consecutive bands (8 new rows per band),
// for wider MID a band's 2*3+k rows are recomputed.  Rows are produced one per wave: a wave
// computes the stem for one image row (32 pixels) as one fp16x3 MFMA tile whose output
// layout (lane = pixel, 16 channels per lane) is directly the pw B operand, keeps it in
// registers, and runs
// the 1x1 conv for each 32-channel chunk of MID as a 32x32x32 fp16x3 MFMA tile (weights =
// A operand, BN scale folded, shuffle folded into the row order, groups densified).  The
// chunk's pw rows go to LDS; the depthwise conv reads them from LDS (fp32 VALU), each lane
// producing exactly the 8 channels it holds as a pwl B operand, so the pwl fp16x3 MFMA
// accumulates over the MID chunks in registers; only the 32-channel block output reaches HBM.
#include "hn_common.h"
#include "hn_internal.h"
#include "hn_preproc.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int FRONT_IRF = 0, FRONT_MAXPOOL = 1;
constexpr int RB = 4;   // output rows per band
constexpr int PS = 36;  // floats per pixel in the LDS pw band (32 channels + 4 pad)

// dw/maxpool read mapping: lane -> (pixel ox in 0..7, channel quad q) chosen so that every
// 16-lane ds_read_b128 group (MI355X_MICROARCH.md LDS) hits 16 distinct 16-byte slots of a
// bank row for the s2 window reads (slot = 2*ox + q + 9*dx mod 16 at PS = 36 floats);
// derived in tests/test_lds_banks.py::test_front_dw_lane_map.  Encoded ox*8 + q.
__constant__ unsigned char kDwLane[64] = {
    0,  1,  2,  3,  46, 47, 8,  9,  10, 11, 12, 13, 4,  5,  6,  7,  20, 21, 28, 29, 14, 15,
    22, 23, 30, 31, 38, 39, 36, 37, 44, 45, 52, 53, 54, 55, 58, 59, 60, 61, 62, 63, 24, 25,
    16, 17, 18, 19, 32, 33, 40, 41, 26, 27, 34, 35, 42, 43, 50, 51, 48, 49, 56, 57};

// LDS pw row layout (IRF form): columns c (pad included) split even / odd -- even c at position
// c / 2, odd c at HALF + c / 2 -- so the dw's stride-2 window reads of consecutive output
// pixels hit consecutive positions (pixel stride PS = 36 floats = 9 slots: 16 distinct 16-byte
// slots per ds_read_b128 group), and the row stride is a multiple of 64 floats so the two
// output rows a 16-lane group mixes see the same slot pattern (tests/test_lds_banks.py).  The
// maxpool form keeps the plain column order (its lane map kDwLane is built for it).
//
// RING (MID = 32 and the maxpool form): the chunk's pw rows live in an LDS ring of IR rows
// (slot (y + PAD) % IR) that persists across the 4 bands of a patch, so a band computes only
// its 8 new stem/pw rows.  MID > 32 recomputes the band's halo rows for every chunk.
// NF (no fold, the default): the pwl runs as 16x16x32 tiles -- wave w owns the band's output row w
// (16 pixels), lane (pixel l & 15, channels 8 (l >> 4) .. + 7) computes its dw channels and is directly
// that MFMA's B operand -- so no wave holds a partial K sum and the fold through LDS (two barriers
// per band) goes; for MID = 32 the dw weights are loaded into LDS once per workgroup.
// U8 (preprocessing fused into the patch load, as k_c12): -1 = fp32 [P,1,32,32]
// input; HN_RESIZE_NONE / _CV2_LINEAR = uint8 patches (32x32 / 64x64) resized, /255'd and
// Normalize'd in the load by hn_preproc.h (the arithmetic of hn_preprocess), so the input costs
// 1 / 4 KiB of HBM per patch and no intermediate fp32 tensor exists.  HN_RESIZE_PIL_BILINEAR: the raw
// 4 KiB are prefetched coalesced and staged in the free pw ring (one extra barrier per patch): its
// 12-register per-thread window fetched ahead took the k3 front from three workgroups per CU to two.
template <int K, int MID, int MODE, bool NORM, bool NF, int U8 = -1, bool P5 = false, bool X3 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == FRONT_IRF && K == 3 && MID == 32 ? 3 : MODE == FRONT_IRF && MID == 32 ? 2 : 1))) void k_front(const void* __restrict__ in_,
                                               float* __restrict__ out,
                                               const uint4* __restrict__ spack,  // stem A operand
                                               const float* __restrict__ stem_b,  // [32]
                                               const uint4* __restrict__ apack,
                                               const float* __restrict__ pw_b,  // [MID] (dw order)
                                               const float* __restrict__ dw_w,  // [K*K][MID]
                                               const float* __restrict__ dw_b,  // [MID]
                                               const uint4* __restrict__ pwl_a,  // [1][MID/16][2][64]
                                               const float* __restrict__ pwl_b,  // [32]
                                               const uint4* __restrict__ pwl_a16,  // [MID/32][2][2][64]
                                               int P, float eps, float pmean, float pstd, int pnorm) {
  constexpr int KK = MODE == FRONT_MAXPOOL ? 3 : K;
  constexpr int PAD = KK / 2;
  constexpr int IR = 2 * (RB - 1) + KK;  // pw rows a band reads (ring size)
  constexpr int PC = 32 + 2 * PAD;       // columns incl. zero padding
  // LEAN (k3 IRF, MID = 32): the waves take only the band's real (non-padding) stem/pw rows
  // -- at most 8, two row tiles per wave instead of three -- and the stem / pw biases are read
  // from LDS where used instead of held in 32 VGPRs: 162 instead of 210 registers, three
  // workgroups per CU instead of two (wang2 front 6.7 -> 6.1 ms).  Elsewhere the extra LDS
  // round trips on the row's latency chain cost more than they free (k5: register-bound at two
  // workgroups either way; maxpool: LDS-bound at three).
  constexpr bool LEAN = MODE == FRONT_IRF && K == 3 && MID == 32;
  // PAIR5 (k5, MID = 32): the k3 form's two-rows-per-gather stem on the k5 ring (8 new rows per
  // band; band 0 has a ninth real row, which wave 0 computes alone as tile 2); biases stay in
  // registers (the k5 front is LDS-bound at two workgroups per CU, not register-bound)
  constexpr bool PAIR5 = P5 && MODE == FRONT_IRF && K == 5 && MID == 32;
  constexpr bool RL = LEAN || PAIR5;  // the waves take only the band's real rows
  constexpr int NT = LEAN ? 2 : PAIR5 ? 3 : (IR + 3) / 4;  // row tiles per wave (at most)
  constexpr int OC = 32;  // layer-0 output channels (SEARCH_SPACE2[0] = (32, 32, 2))
  constexpr int DYU = KK == 3 ? 3 : 1;  // k5: rolled dy loop keeps VGPRs (and occupancy) in check
  constexpr bool RING = MID == 32;
  constexpr bool SPLIT = MODE == FRONT_IRF;                  // even/odd column split
  constexpr int HALF = (PC + 1) / 2;                         // first odd-column position
  // XCH (the k5 front, MID = 32): the dw runs per channel group with its weights in SGPRs and crosses to
  // the pwl's operand layout through s_x (see the dw phase); s_dw is not used
  // (X3, HN_FRONT_XCH3=1: the same for the k3 front)
  constexpr bool XCH = NF && (PAIR5 || (X3 && K == 3 && MID == 32 && MODE == FRONT_IRF));
  // SW (X3): 32-float pw pixels (no pad floats) with the 16-byte channel chunk c of ring position pos
  // stored at c ^ swz(pos) -- the XCH dw reads and the pw epilogue writes stay conflict-free
  // (tests/test_lds_banks.py::test_front_x3_swizzle_conflict_free) and the ring shrinks by 1/9, so
  // the k3 XCH front fits three workgroups per CU (52 KB)
  constexpr bool SW = XCH && K == 3;
  constexpr int PSX = SW ? 32 : PS;
  auto swz = [](int pos) { return SW ? (pos + 3 * (pos >> 1)) & 7 : 0; };
  constexpr int RS = SPLIT ? (PC * PSX + 63) / 64 * 64 : PC * PSX;  // row stride (floats)
  static_assert(IR >= 8, "ring holds a band's 8 new rows");
  __shared__ float s_in[34 * 34];
  __shared__ __attribute__((aligned(16))) float s_pw[IR * RS];
  __shared__ __attribute__((aligned(16))) float s_dw[XCH ? 4 : KK * KK * 32 + 32];
  __shared__ uint4 s_x[XCH ? 2 * 4 * 16 * 4 : 1];  // [hi / lo][band row][column][16-byte chunk]
  __shared__ float red[8];
  // stem bias and (MID = 32: the single chunk's) pw bias, read where used (fewer live VGPRs)
  __shared__ __attribute__((aligned(16))) float s_sb[32], s_pwb[32];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int px = lane & 31, h = lane >> 5;
  // NF lane permutations (bank conflicts; tests/test_lds_banks.py::test_front_nf_*).  pxm: the image
  // column that stem / pw MFMA column px stands for -- columns 0-15 take the pixels whose padded column
  // PAD + pxm is even, 16-31 the odd ones, in order -- so each 8-lane group of the pw epilogue's
  // ds_write_b128 covers 8 consecutive positions of one half of the even / odd-split pw row (2-way
  // conflicted in column order).  dwx (below): the output column of 16x16 pwl column l & 15 -- columns
  // {0-3, 12-15} the even ones, {4-11} the odd ones -- so the dw window reads of a ds_read_b128 lane group
  // (mixing those two sets with channel offsets 8 apart) hit 16 distinct slots (2-way in order).
  const int pxm = NF ? 2 * (px & 15) + (((px >> 4) & 1) ^ (PAD & 1)) : px;
  const int l16 = lane & 15;
  const int dwx = l16 < 4 ? 2 * l16 : l16 < 12 ? 2 * (l16 - 4) + 1 : 2 * (l16 - 8);
  // persistent: whole patches per workgroup, their 4 bands in order
  const long per = ((long)P + gridDim.x - 1) / gridDim.x;
  const long pb = (long)xcd_remap(blockIdx.x, gridDim.x) * per;
  const long pe = min((long)P, pb + per);
  if (pb >= pe) return;  // workgroup-uniform

  // position of padded column c in a pw row
  auto colpos = [](int c) { return SPLIT ? ((c & 1) ? HALF + (c >> 1) : c >> 1) : c; };
  // ---- one-time init: zero s_in (its frame stays zero) and the pw pad columns ---------------
  for (int i = t; i < 34 * 34; i += 256) s_in[i] = 0.f;
  for (int i = t; i < IR * 2 * PAD * (PSX / 4); i += 256) {  // left/right pad columns
    const int ri = i / (2 * PAD * (PSX / 4)), rem = i % (2 * PAD * (PSX / 4)), c = rem / (PSX / 4);
    reinterpret_cast<float4*>(s_pw)[(ri * RS + colpos(c < PAD ? c : 32 + c) * PSX) / 4 + rem % (PSX / 4)] =
        make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const f16x8 sah = as_f16x8(spack[lane]), sal = as_f16x8(spack[64 + lane]);
  constexpr bool LDSB = LEAN;
  // PAIR (the k3 no-fold front): wave w computes the band's stem rows 2w, 2w + 1 from ONE B operand,
  // the 4 x 3 input window of the two rows (K slot 3 dy + dx, dy = 0..3; slots 12..15 carry any valid
  // input against zero weights), with the row-y taps in K slots 0..8 (spack op 0) and the row-(y + 1)
  // taps in slots 3..11 (op 1): one gather and one hi / lo split per two rows
  constexpr bool PAIR = (LEAN && NF) || PAIR5;
  f16x8 sah2{}, sal2{};
  int toff[8] = {};  // PAIR: this lane's s_in offsets of its 8 K slots, from (row y0, column px)
  if constexpr (PAIR) {
    sah2 = as_f16x8(spack[128 + lane]);
    sal2 = as_f16x8(spack[192 + lane]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = min(8 * h + j, 11);
      toff[j] = (k / 3) * 34 + k % 3;
    }
  }
  if (t < 32) s_sb[t] = stem_b[t];
  else if (t < 64 && MID == 32) s_pwb[t - 32] = pw_b[t - 32];
  // (visible after the first patch's barriers)
  // 32 channels of a bias vector in the MFMA accumulator order (lane (px, h): acc[4q + r] =
  // channel 4h + 8q + r) -- the initial accumulator, so the epilogues are ReLU only
  auto bias16 = [&](const float* b) {
    f32x16 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(b + 8 * q + 4 * h);
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
    return v;
  };
  f32x16 sbr = {};  // !LDSB: the stem bias in registers
  if constexpr (!LDSB) sbr = bias16(stem_b);
  const int lm = kDwLane[lane], dq = lm & 7, dox = lm >> 3;
  auto slot_of = [](int y) { return (y + PAD + IR) % IR; };  // ring slot of pw row y

  constexpr bool DW_ONCE = NF && MID == 32 && MODE == FRONT_IRF;  // one chunk: its dw weights never change
  if constexpr (DW_ONCE && !XCH) {
    for (int i = t; i < KK * KK * 8 + 8; i += 256) {
      float4 wv;
      if (i < KK * KK * 8)
        wv = *reinterpret_cast<const float4*>(dw_w + (i >> 3) * MID + 4 * (i & 7));
      else
        wv = *reinterpret_cast<const float4*>(dw_b + 4 * (i - KK * KK * 8));
      reinterpret_cast<float4*>(s_dw)[i] = wv;
    }
  }
  // INV (MID = 32: one chunk): the chunk's pw / pwl operands and biases are loop-invariant.  They
  // are loaded here and consumed by an empty asm before the patch loop, so that no load from
  // outside the loops is still pending at the band loop: otherwise the compiler flushes vmcnt to
  // zero in front of the band loop (a loop with stores, no loads and operands loaded outside it),
  // which also waited for the next patch's prefetch issued just before -- an exposed HBM latency
  // per patch.
  constexpr bool INV = MID == 32 && MODE == FRONT_IRF;
  f16x8 iah0{}, ial0{}, iah1{}, ial1{};
  f16x8 ilp[4] = {};
  f32x16 ipwb = {};
  f32x4_t ib16[2] = {};
  if constexpr (INV) {
    iah0 = as_f16x8(apack[lane]);
    ial0 = as_f16x8(apack[64 + lane]);
    iah1 = as_f16x8(apack[128 + lane]);
    ial1 = as_f16x8(apack[192 + lane]);
    asm volatile("" ::"v"(iah0), "v"(ial0), "v"(iah1), "v"(ial1));
    if constexpr (NF) {
#pragma unroll
      for (int k = 0; k < 4; ++k) ilp[k] = as_f16x8(pwl_a16[64 * k + lane]);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const float4 b = *reinterpret_cast<const float4*>(pwl_b + 16 * tt + 4 * (lane >> 4));
        ib16[tt] = f32x4_t{b.x, b.y, b.z, b.w};
      }
      asm volatile("" ::"v"(ilp[0]), "v"(ilp[1]), "v"(ilp[2]), "v"(ilp[3]), "v"(ib16[0]), "v"(ib16[1]));
    }
    if constexpr (!LDSB) {
      ipwb = bias16(pw_b);
      asm volatile("" ::"v"(ipwb));
    }
    if constexpr (!LDSB) asm volatile("" ::"v"(sbr));
  }
  const float* in = static_cast<const float*>(in_);
  const uint8_t* in8 = static_cast<const uint8_t*>(in_);
  constexpr int INB = U8 == HN_RESIZE_NONE ? 1024 : 4096;  // bytes per uint8 patch
  const int iy = t >> 3, ix = 4 * (t & 7);                  // this thread's 4 pixels (iy, ix ..)
  // the next patch's pixels are fetched one patch ahead (U8: its raw bytes -- 1 / 4 registers for
  // NONE / CV2, as many as the fp32 form -- resized at use).  PIL: the 4 KiB patch is fetched ahead
  // coalesced (16 bytes per thread, 4 registers), staged in the pw ring once the previous patch is
  // done with it, and every thread reads its 4 x 10-byte window from there (its 12-register window
  // fetched ahead cost the k3 front its third workgroup per CU)
  constexpr bool PILS = U8 == HN_RESIZE_PIL_BILINEAR;
  static_assert(!PILS || (!NORM && IR * RS * 4 >= 4096), "PIL staging: no input_norm, a ring of >= 4 KiB");
  float4 vnext;
  hnpre::U8Px<U8 < 0 || PILS ? HN_RESIZE_NONE : U8, 4> rnext;
  uint4 rawnext;
  if constexpr (U8 < 0)
    vnext = reinterpret_cast<const float4*>(in + pb * 1024)[t];
  else if constexpr (PILS)
    rawnext = reinterpret_cast<const uint4*>(in8 + pb * INB)[t];
  else
    rnext.load(in8 + pb * INB, iy, ix);
#pragma unroll 1
  for (long patch = pb; patch < pe; ++patch) {
    // ---- patch (+ input_norm) to LDS; the next patch's pixels are prefetched ---------------
    float4 v;
    if constexpr (U8 < 0) {
      v = vnext;
      if (patch + 1 < pe) vnext = reinterpret_cast<const float4*>(in + (patch + 1) * 1024)[t];
    } else if constexpr (PILS) {
      __syncthreads();  // the previous patch is done with the ring
      reinterpret_cast<uint4*>(s_pw)[t] = rawnext;
      if (patch + 1 < pe) rawnext = reinterpret_cast<const uint4*>(in8 + (patch + 1) * INB)[t];
      __syncthreads();
      hnpre::U8Px<HN_RESIZE_PIL_BILINEAR, 4> wpx;
      wpx.load(reinterpret_cast<const uint8_t*>(s_pw), iy, ix);
      int q[4];
      wpx.resized(iy, ix, q);
      v = make_float4(hnpre::to_input(q[0], pmean, pstd, pnorm), hnpre::to_input(q[1], pmean, pstd, pnorm),
                      hnpre::to_input(q[2], pmean, pstd, pnorm), hnpre::to_input(q[3], pmean, pstd, pnorm));
    } else {
      int q[4];
      rnext.resized(iy, ix, q);
      v = make_float4(hnpre::to_input(q[0], pmean, pstd, pnorm), hnpre::to_input(q[1], pmean, pstd, pnorm),
                      hnpre::to_input(q[2], pmean, pstd, pnorm), hnpre::to_input(q[3], pmean, pstd, pnorm));
      if (patch + 1 < pe) rnext.load(in8 + (patch + 1) * INB, iy, ix);
    }
    float mean = 0.f, sd = 1.f;
    if (NORM) {  // (x - mean) / (std_unbiased + eps), as k_stem
      const float s = wave_sum(v.x + v.y + v.z + v.w);
      if (lane == 0) red[w] = s;
      __syncthreads();
      mean = (red[0] + red[1] + red[2] + red[3]) * (1.f / 1024.f);
      const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
      const float q = wave_sum(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
      if (lane == 0) red[4 + w] = q;
      __syncthreads();
      sd = sqrtf((red[4] + red[5] + red[6] + red[7]) * (1.f / 1023.f)) + eps;
    }
    __syncthreads();  // the previous patch is done with s_in and the ring
    {
      const int q = 4 * t, y = q >> 5, x = q & 31;
      float* d = s_in + (y + 1) * 34 + x + 1;
      if (NORM) {
        d[0] = (v.x - mean) / sd; d[1] = (v.y - mean) / sd;
        d[2] = (v.z - mean) / sd; d[3] = (v.w - mean) / sd;
      } else {
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    }
    __syncthreads();

#pragma unroll 1
    for (int band = 0; band < 4; ++band) {
      const int r0 = band * RB;
      // pw rows this band computes: all IR rows 2 r0 - PAD .. (band 0 / no ring), or the 8
      // rows after the previous band's last one (ring)
      const int ylast = 2 * r0 + 6 + PAD;
      const int ybeg = (RING && band > 0) ? ylast - 7 : 2 * r0 - PAD;
      // LEAN: the real rows yr0 .. go to the waves round-robin and the padding rows are
      // zero-filled apart; otherwise all rows ybeg .. ylast round-robin
      const int yr0 = RL ? max(ybeg, 0) : ybeg;
      const int nreal = RL ? min(ylast, 31) + 1 - yr0 : ylast + 1 - ybeg;

      // ---- phase A: stem rows on the MFMA ------------------------------------------------
      // A = stem weights [32 ch][16 = 9 taps + 0], B = im2col of one image row (lane: pixel
      // px, taps 8h..8h+7).  C leaves channel 4h + 8q + r (i = 4q + r) of pixel px in acc[i];
      // that order is used as-is as the pw contraction index (pw weights are packed to match).
      auto zero_row = [&](int y) {  // zero padding row of the pw output (whole row)
        float4* d = reinterpret_cast<float4*>(s_pw + slot_of(y) * RS);
        for (int j = lane; j < RS / 4; j += 64) d[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      };
      if constexpr (RL)
        for (int y = ybeg + w; y <= ylast; y += 4)
          if (y < 0 || y >= 32) zero_row(y);
      uint4 bh[NT][2], bl[NT][2];
      // row tile i of this wave: band row 2w + i (PAIR; PAIR5's tile 2: band row 8) or w + 4i
      // (PAIR5: the window base row y5 = min(y0, 30) keeps the 4-row window inside s_in; a wave
      // whose y0 is 31 takes row 31 as op 1 of the window at 30, and drops tile 0 = row 30)
      const int y5 = min(yr0 + 2 * w, 30);
      auto row_of = [&](int i) { return PAIR5 ? (i < 2 ? y5 - yr0 + i : 8) : PAIR ? 2 * w + i : w + 4 * i; };
      auto tile_on = [&](int i) {  // PAIR5: tile i holds a real row this wave owns
        const int ri = row_of(i);
        return i < 2 ? (ri >= 2 * w && ri < nreal) : (w == 0 && nreal > 8);
      };
      if constexpr (PAIR) {
        static_assert(!PAIR || NT == 2 || PAIR5, "two rows per wave");
        const int y0 = PAIR5 ? y5 : yr0 + 2 * w;  // rows y0, y0 + 1 (LEAN bands hold 8 real rows)
        const float* sb = s_in + y0 * 34 + pxm;
        float tp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tp[j] = sb[toff[j]];
        uint4 xh, xl;
        split8_f16(make_float4(tp[0], tp[1], tp[2], tp[3]), make_float4(tp[4], tp[5], tp[6], tp[7]), xh, xl);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const f32x16 c = i == 0 ? mfma3_f16(sah, sal, as_f16x8(xh), as_f16x8(xl), LDSB ? bias16(s_sb) : sbr)
                                  : mfma3_f16(sah2, sal2, as_f16x8(xh), as_f16x8(xl), LDSB ? bias16(s_sb) : sbr);
          float4 o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            o[q] = make_float4(relu0(c[4 * q]), relu0(c[4 * q + 1]), relu0(c[4 * q + 2]),
                               relu0(c[4 * q + 3]));
          split8_f16(o[0], o[1], bh[i][0], bl[i][0]);
          split8_f16(o[2], o[3], bh[i][1], bl[i][1]);
        }
      }
#pragma unroll
      for (int i = (PAIR5 ? 2 : 0); i < (PAIR && !PAIR5 ? 0 : NT); ++i) {
        const int ri = row_of(i), y = yr0 + ri;
        if (PAIR5 ? !tile_on(i) : ri >= nreal) continue;  // wave-uniform; such tiles are never read
        if (!LEAN && (y < 0 || y >= 32)) {
          zero_row(y);
          continue;
        }
        float tp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = 8 * h + j;  // h = 1 holds tap 8 and zeros
          tp[j] = tap < 9 ? s_in[(y + tap / 3) * 34 + pxm + tap % 3] : 0.f;
        }
        uint4 xh, xl;
        split8_f16(make_float4(tp[0], tp[1], tp[2], tp[3]), make_float4(tp[4], tp[5], tp[6], tp[7]), xh, xl);
        const f32x16 c = mfma3_f16(sah, sal, as_f16x8(xh), as_f16x8(xl), LDSB ? bias16(s_sb) : sbr);
        float4 o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = make_float4(relu0(c[4 * q]), relu0(c[4 * q + 1]), relu0(c[4 * q + 2]),
                             relu0(c[4 * q + 3]));
        if (MODE == FRONT_MAXPOOL) {
          float4* d = reinterpret_cast<float4*>(s_pw + slot_of(y) * RS + colpos(PAD + px) * PS);
#pragma unroll
          for (int q = 0; q < 4; ++q) d[2 * q + h] = o[q];
        } else {
          split8_f16(o[0], o[1], bh[i][0], bl[i][0]);
          split8_f16(o[2], o[3], bh[i][1], bl[i][1]);
        }
      }

      if (MODE == FRONT_MAXPOOL) {
        __syncthreads();
        // MaxPool2d(3, 2, 1): padding never wins since every window holds a ReLU output >= 0
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int p = 8 * (w + 4 * j) + dox, orr = p >> 4, ox = p & 15;
          float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int dy = 0; dy < 3; ++dy) {
            const float* rp = s_pw + slot_of(2 * (r0 + orr) - 1 + dy) * RS;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
              const float4 a = *reinterpret_cast<const float4*>(rp + (2 * ox + dx) * PS + 4 * dq);
              m.x = fmaxf(m.x, a.x); m.y = fmaxf(m.y, a.y); m.z = fmaxf(m.z, a.z); m.w = fmaxf(m.w, a.w);
            }
          }
          *reinterpret_cast<float4*>(out + ((patch * 16 + r0 + orr) * 16 + ox) * 32 + 4 * dq) = m;
        }
        __syncthreads();  // reads done before the next band's rows overwrite ring slots
        continue;
      }

      // ---- phases B/C/D per 32-channel chunk of MID -------------------------------------
      f32x16 oacc = {};
      f32x4_t o16[2];  // NF: pwl output channels 16 tile + 4 (lane >> 4) + j of pixel lane & 15, from the bias
      if constexpr (NF) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          if constexpr (INV) {
            o16[tt] = ib16[tt];
          } else {
            const float4 b = *reinterpret_cast<const float4*>(pwl_b + 16 * tt + 4 * (lane >> 4));
            o16[tt] = f32x4_t{b.x, b.y, b.z, b.w};
          }
        }
      }
#pragma unroll 1
      for (int m = 0; m < MID / 32; ++m) {
        // dw weights + bias of the chunk
        if (!DW_ONCE)
        for (int i = t; i < KK * KK * 8 + 8; i += 256) {
          float4 wv;
          if (i < KK * KK * 8)
            wv = *reinterpret_cast<const float4*>(dw_w + (i >> 3) * MID + 32 * m + 4 * (i & 7));
          else
            wv = *reinterpret_cast<const float4*>(dw_b + 32 * m + 4 * (i - KK * KK * 8));
          reinterpret_cast<float4*>(s_dw)[i] = wv;
        }
        const uint4* ap = apack + (size_t)m * 4 * 64 + lane;
        const f16x8 ah0 = INV ? iah0 : as_f16x8(ap[0]), al0 = INV ? ial0 : as_f16x8(ap[64]);
        const f16x8 ah1 = INV ? iah1 : as_f16x8(ap[128]), al1 = INV ? ial1 : as_f16x8(ap[192]);
        f32x16 bias;  // pw bias as the initial accumulator (LDSB: read per row from LDS)
        if constexpr (!LDSB) bias = INV ? ipwb : bias16(pw_b + 32 * m);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          const int ri = row_of(i), y = yr0 + ri;
          if (PAIR5 ? !tile_on(i) : (ri >= nreal || y < 0 || y >= 32)) continue;
          if constexpr (LDSB) bias = bias16(s_pwb);
          f32x16 acc = mfma3_f16(ah0, al0, as_f16x8(bh[i][0]), as_f16x8(bl[i][0]), bias);
          acc = mfma3_f16(ah1, al1, as_f16x8(bh[i][1]), as_f16x8(bl[i][1]), acc);
          const int pos = colpos(PAD + pxm);
          float4* d = reinterpret_cast<float4*>(s_pw + slot_of(y) * RS + pos * PSX);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            d[(2 * q + h) ^ swz(pos)] = make_float4(relu0(acc[4 * q]), relu0(acc[4 * q + 1]),
                                       relu0(acc[4 * q + 2]), relu0(acc[4 * q + 3]));
        }
        __syncthreads();
        if constexpr (NF) {
          uint4 xh, xl;
          if constexpr (XCH) {
            // wave w computes channel group w (8 channels) of all four band rows, lane (row lane >> 4, output
            // column lane & 15): the dw weights are wave-uniform and come from SGPRs (scalar loads of dw_w /
            // dw_b) instead of a broadcast ds_read_b128 per 4 channels and tap -- half the front's LDS
            // reads.  The results cross to the pwl's (column, channel group) lane layout through s_x, chunk
            // g of column c at g ^ ((c >> 1) & 3) (writes and reads conflict-free, tests/test_lds_banks.py).
            const int cg = __builtin_amdgcn_readfirstlane(w), rr = lane >> 4, ox = lane & 15, c0 = 8 * cg;
            const float* const wsrc = dw_w + 32 * m + c0;
            f32x4 a0 = *reinterpret_cast<const f32x4*>(dw_b + 32 * m + c0);
            f32x4 a1 = *reinterpret_cast<const f32x4*>(dw_b + 32 * m + c0 + 4);
#pragma unroll DYU
            for (int dy = 0; dy < KK; ++dy) {
              const float* rp = s_pw + slot_of(2 * (r0 + rr) - PAD + dy) * RS;
#pragma unroll
              for (int dx = 0; dx < KK; ++dx) {
                const float* wp = wsrc + (dy * KK + dx) * MID;
                const int pos = (dx & 1) ? HALF + ox + (dx >> 1) : ox + (dx >> 1);
                const float* ip = rp + pos * PSX;
                const int sz = swz(pos);
                a0 = __builtin_elementwise_fma(*reinterpret_cast<const f32x4*>(wp),
                                               *reinterpret_cast<const f32x4*>(ip + 4 * ((2 * cg) ^ sz)), a0);
                a1 = __builtin_elementwise_fma(*reinterpret_cast<const f32x4*>(wp + 4),
                                               *reinterpret_cast<const f32x4*>(ip + 4 * ((2 * cg + 1) ^ sz)), a1);
              }
            }
            a0 = relu4(a0);
            a1 = relu4(a1);
            split8_f16(make_float4(a0.x, a0.y, a0.z, a0.w), make_float4(a1.x, a1.y, a1.z, a1.w), xh, xl);
            const int wc = cg ^ ((ox >> 1) & 3);
            s_x[((0 * 4 + rr) * 16 + ox) * 4 + wc] = xh;
            s_x[((1 * 4 + rr) * 16 + ox) * 4 + wc] = xl;
            __syncthreads();  // every channel group of the band's pixels in s_x
            const int kg = lane >> 4, rc = kg ^ ((l16 >> 1) & 3);
            xh = s_x[((0 * 4 + w) * 16 + l16) * 4 + rc];
            xl = s_x[((1 * 4 + w) * 16 + l16) * 4 + rc];
          } else {  // dw of band row w, 8 channels of pixel dwx -> 16x16x32 pwl
            const int ox = dwx, c0 = 8 * (lane >> 4);
            f32x4 a0 = *reinterpret_cast<const f32x4*>(s_dw + KK * KK * 32 + c0);
            f32x4 a1 = *reinterpret_cast<const f32x4*>(s_dw + KK * KK * 32 + c0 + 4);
#pragma unroll DYU
            for (int dy = 0; dy < KK; ++dy) {
              const float* rp = s_pw + slot_of(2 * (r0 + w) - PAD + dy) * RS + c0;
#pragma unroll
              for (int dx = 0; dx < KK; ++dx) {
                const float* wp = s_dw + (dy * KK + dx) * 32 + c0;
                const float* ip = rp + ((dx & 1) ? HALF + ox + (dx >> 1) : ox + (dx >> 1)) * PS;
                a0 = __builtin_elementwise_fma(*reinterpret_cast<const f32x4*>(wp), *reinterpret_cast<const f32x4*>(ip), a0);
                a1 = __builtin_elementwise_fma(*reinterpret_cast<const f32x4*>(wp + 4), *reinterpret_cast<const f32x4*>(ip + 4), a1);
              }
            }
            a0 = relu4(a0);
            a1 = relu4(a1);
            split8_f16(make_float4(a0.x, a0.y, a0.z, a0.w), make_float4(a1.x, a1.y, a1.z, a1.w), xh, xl);
          }
          const uint4* lp = pwl_a16 + (size_t)m * 4 * 64 + lane;
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
            o16[tt] = mfma3_f16_16(INV ? ilp[2 * tt] : as_f16x8(lp[128 * tt]), INV ? ilp[2 * tt + 1] : as_f16x8(lp[128 * tt + 64]),
                                   as_f16x8(xh), as_f16x8(xl), o16[tt]);
          // s_dw (and, without the ring, s_pw) is rewritten next; XCH: the next band's s_x writes come after
          // its own first barrier, which every wave reaches only after these reads
          if constexpr (!XCH) __syncthreads();
          continue;
        }
        // dw straight into the pwl B-operand layout: wave w owns band pixel tile (w & 1) and
        // K-step (w >> 1) of this chunk; lane (px, h) computes channels 16*(w>>1) + 8h .. +7
        // of band pixel 32*(w&1) + px, splits them and multiplies with the pwl weights of
        // that K-step.  Waves 2/3 hold partial sums over the odd K-steps, folded in below.
        {
          const int p = 32 * (w & 1) + px, orr = p >> 4, ox = p & 15, c0 = 16 * (w >> 1) + 8 * h;
          f32x4 a0 = *reinterpret_cast<const f32x4*>(s_dw + KK * KK * 32 + c0);
          f32x4 a1 = *reinterpret_cast<const f32x4*>(s_dw + KK * KK * 32 + c0 + 4);
#pragma unroll DYU
          for (int dy = 0; dy < KK; ++dy) {
            const float* rp = s_pw + slot_of(2 * (r0 + orr) - PAD + dy) * RS + c0;
#pragma unroll
            for (int dx = 0; dx < KK; ++dx) {
              const float* wp = s_dw + (dy * KK + dx) * 32 + c0;
              // column 2 ox + dx: position ox + dx / 2 (even dx) or HALF + ox + dx / 2 (odd)
              const float* ip = rp + ((dx & 1) ? HALF + ox + (dx >> 1) : ox + (dx >> 1)) * PS;
              a0 = __builtin_elementwise_fma(*reinterpret_cast<const f32x4*>(wp), *reinterpret_cast<const f32x4*>(ip), a0);
              a1 = __builtin_elementwise_fma(*reinterpret_cast<const f32x4*>(wp + 4), *reinterpret_cast<const f32x4*>(ip + 4), a1);
            }
          }
          a0 = relu4(a0);
          a1 = relu4(a1);
          uint4 xh, xl;
          split8_f16(make_float4(a0.x, a0.y, a0.z, a0.w), make_float4(a1.x, a1.y, a1.z, a1.w), xh, xl);
          const uint4* lp = pwl_a + ((size_t)(2 * m + (w >> 1)) * 2) * 64 + lane;
          oacc = mfma3_f16(as_f16x8(lp[0]), as_f16x8(lp[64]), as_f16x8(xh), as_f16x8(xl), oacc);
        }
        __syncthreads();  // s_dw (and, without the ring, s_pw) is rewritten next
      }
      if constexpr (NF) {  // band row r0 + w, pixel lane & 15: 4 consecutive channels per tile
        // (whole 128-byte rows per store after a DPP row rotation measured slower: wang2 front 5.07 -> 5.26 ms)
        float* dst = out + ((patch * 16 + r0 + w) * 16 + (XCH ? l16 : dwx)) * OC + 4 * (lane >> 4);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          *reinterpret_cast<float4*>(dst + 16 * tt) = make_float4(o16[tt][0], o16[tt][1], o16[tt][2], o16[tt][3]);
        continue;
      }
      // fold the odd-K-step partial sums of waves 2/3 into waves 0/1 through the interior
      // of the ring slots of rows ybeg, ybeg + 1 (recomputed by the next band, never the
      // rows it keeps; the pad columns stay zero): lanes 0-31 use the 16 interior even-column
      // positions 1 .., lanes 32-63 the 16 interior odd-column positions HALF + PAD - 1 ..
      auto fold_at = [&](int row) {
        return reinterpret_cast<float4*>(s_pw + slot_of(row) * RS + (h ? HALF + PAD - 1 : 1) * PS) + px * 4;
      };
      static_assert(16 * PS >= 32 * 16, "a half-wave's partial sums fit 16 interior positions");
      if (w >= 2) {
        float4* d = fold_at(ybeg + (w - 2));
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = make_float4(oacc[4 * q], oacc[4 * q + 1], oacc[4 * q + 2], oacc[4 * q + 3]);
      }
      __syncthreads();
      if (w < 2) {  // output pixel 32w + px of the band = row r0 + (32w + px) / 16
        const float4* d = fold_at(ybeg + w);
        const int p = 32 * w + px;
        float* dst = out + ((patch * 16 + r0 + (p >> 4)) * 16 + (p & 15)) * OC;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v4 = d[q];
          const float4 b = *reinterpret_cast<const float4*>(pwl_b + 8 * q + 4 * h);
          *reinterpret_cast<float4*>(dst + 8 * q + 4 * h) =
              make_float4(oacc[4 * q] + v4.x + b.x, oacc[4 * q + 1] + v4.y + b.y,
                          oacc[4 * q + 2] + v4.z + b.z, oacc[4 * q + 3] + v4.w + b.w);
        }
      }
      __syncthreads();  // fold reads done before the next band rewrites those ring slots
    }
  }
}

template <int K, int MID, int MODE, bool NORM, bool NF, int U8 = -1, bool P5 = false, bool X3 = false>
hipError_t front_launch_nf(const HnFrontArgs& a, int P, float eps, hipStream_t st, const HnU8In* u8 = nullptr) {
  int resident = 0;  // persistent grid: every workgroup resident at once
  const hipError_t e =
      hn_resident_blocks(reinterpret_cast<const void*>(&k_front<K, MID, MODE, NORM, NF, U8, P5, X3>), 256, 0, &resident);
  if (e != hipSuccess) return e;
  const void* src = u8 ? static_cast<const void*>(u8->in) : static_cast<const void*>(a.in);
  hipLaunchKernelGGL((k_front<K, MID, MODE, NORM, NF, U8, P5, X3>), dim3(std::min(P, resident)), dim3(256), 0, st, src,
                     a.out, a.spack, a.stem_b, a.apack, a.pw_b, a.dw_w, a.dw_b, a.pwl_a, a.pwl_b, a.pwl_a16, P,
                     eps, u8 ? u8->mean : 0.f, u8 ? u8->stdv : 1.f, u8 ? u8->normalize : 0);
  return hipGetLastError();
}

// the production form of (K, MID, MODE): the no-fold pwl for the k3 IRF fronts and the k5 MID-32 one,
// the latter with paired stem rows (same-box A/B, wang3 front ms per step: fold form 8.94, + dy loop
// unrolled 8.56, no fold 9.19, no fold + dy unrolled 8.54, paired rows with the fold 8.16, paired rows
// without it 8.13 (the default), both + dy unrolled 8.0-8.4)
template <int K, int MID, int MODE>
constexpr bool front_nf() { return MODE == FRONT_IRF && (K == 3 || (K == 5 && MID == 32)); }
template <int K, int MID, int MODE>
constexpr bool front_p5() { return MODE == FRONT_IRF && K == 5 && MID == 32; }

template <int K, int MID, int MODE, bool NORM>
hipError_t front_launch_t(const HnFrontArgs& a, int P, float eps, hipStream_t st, const HnU8In* u8) {
  // HN_FRONT_FOLD=1: the 32x32x16 pwl with the partial-sum fold through LDS (the round-2 form;
  // wang2 front k3 6.12 -> 5.59 ms without it; the k5 front without the fold alone was 6 % slower, with
  // the paired stem rows 9 % faster than the fold form)
  const bool nf = front_nf<K, MID, MODE>() && !hn_knobs().front_fold && a.pwl_a16;
  if (u8) {  // uint8 loads (every resize mode): the production form without input_norm only (hn_api.hip u8_fused)
    if constexpr (NORM) {
      return hipErrorInvalidValue;
    } else {
      if (nf != front_nf<K, MID, MODE>()) return hipErrorInvalidValue;
      constexpr bool NFD = front_nf<K, MID, MODE>(), P5D = front_p5<K, MID, MODE>();
      switch (u8->resize) {
        case HN_RESIZE_NONE: return front_launch_nf<K, MID, MODE, false, NFD, HN_RESIZE_NONE, P5D>(a, P, eps, st, u8);
        case HN_RESIZE_CV2_LINEAR:
          return front_launch_nf<K, MID, MODE, false, NFD, HN_RESIZE_CV2_LINEAR, P5D>(a, P, eps, st, u8);
        case HN_RESIZE_PIL_BILINEAR:
          return front_launch_nf<K, MID, MODE, false, NFD, HN_RESIZE_PIL_BILINEAR, P5D>(a, P, eps, st, u8);
      }
      return hipErrorInvalidValue;
    }
  }
  if constexpr (K == 3 && MID == 32 && MODE == FRONT_IRF)
    if (nf && hn_knobs().front_xch3) return front_launch_nf<K, MID, MODE, NORM, true, -1, false, true>(a, P, eps, st);
  if (nf) return front_launch_nf<K, MID, MODE, NORM, true, -1, front_p5<K, MID, MODE>()>(a, P, eps, st);
  return front_launch_nf<K, MID, MODE, NORM, false>(a, P, eps, st);
}

template <int K, int MID, int MODE>
hipError_t front_launch(const HnFrontArgs& a, int P, bool norm, float eps, hipStream_t st, const HnU8In* u8) {
  return norm ? front_launch_t<K, MID, MODE, true>(a, P, eps, st, u8)
              : front_launch_t<K, MID, MODE, false>(a, P, eps, st, u8);
}

}  // namespace

bool hn_front_supported(int k, int mid) {
  return (k == 3 || k == 5) && (mid == 32 || mid == 96 || mid == 128);
}

hipError_t hn_launch_front(const HnFrontArgs& a, int P, int k, int mid, bool maxpool, bool norm,
                           float eps, hipStream_t st, const HnU8In* u8) {
  if (P <= 0) return hipSuccess;
  if (maxpool) return front_launch<3, 32, FRONT_MAXPOOL>(a, P, norm, eps, st, u8);
#define HN_FRONT(KK, MM) \
  if (k == KK && mid == MM) return front_launch<KK, MM, FRONT_IRF>(a, P, norm, eps, st, u8);
  HN_FRONT(3, 32) HN_FRONT(3, 96) HN_FRONT(3, 128) HN_FRONT(5, 32) HN_FRONT(5, 96) HN_FRONT(5, 128)
#undef HN_FRONT
  return hipErrorInvalidValue;
}
