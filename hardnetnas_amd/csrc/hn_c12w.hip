// k_c12w: HardNet input_norm + conv0 + conv1 + conv2 (hardnet/HardNet.py:281-289, 306-310) in one
// kernel, as k_c12 (hn_c12.hip, production configuration 12: 4 waves, bands of 2 conv2 output rows,
// two workgroups per CU), with conv1 as a 1-D Winograd F(4,3) along x.
//
// conv1 (9.4 of the kernel's 14.2 MMAC per patch) per output row and tile T of 4 columns
// (4T .. 4T + 3) reads the 6 input columns d_i = a0[4T - 1 + i]; with the Toom-Cook points
// 0, 1, -1, 1/2, -1/2, inf the 6 transformed inputs V = B^T d meet U_xi[ky] = sum_kx G[xi][kx]
// W[ky][kx] (fp64 on the host, then bf16 hi / lo) in 6 x 3 GEMMs of K = 32 channels, and
// y = A^T m: 18 multiplies per 4 outputs and input channel instead of 36, so conv1's MFMA work
// halves (k_c12's drops by a third).  tests/precision/wino1d_precision.py: 1.7e-5 max abs from the
// fp64 reference with conv1, conv3 and conv5 transformed (1.0e-5 all direct; the budget is 1e-4).
//
// Per band (P1 -> barrier -> P2 -> barrier -> P3, as k_c12):
//   P1 stem: the band's new a0 rows (one per wave), 32x32x16 bf16x3 MFMA as k_c12, ReLU; the fp32
//            row is staged in its own W0 ring slot (144-byte columns: the stores and the transform's
//            reads are conflict-free), read back as lane (tile T, 4-channel chunk) = 6 columns,
//            transformed (12 FMAs per channel), split to bf16 hi / lo and written over the staging
//            as V records (xi, T): 128 B = 32 channels hi | lo, 16-byte chunk c at c ^ T.
//   P2 conv1: wave (group g = w & 1 of 16 output channels, row pair rp = w >> 1): N = 16 = 8 tiles
//            x 2 a1 rows, its 6 x 3 x 2 U fragments resident (144 VGPRs, as k_c12's direct
//            weights); 18 (ky, xi) steps of 3 MFMAs; the output transform, bias (in m1, whose A^T
//            column is all ones), ReLU, split -> ring W1 (unchanged layout: even / odd columns apart).
//   P3 conv2: k_c12's (each wave a 16-channel quarter of the band's 2 x 16 output pixels), the a2
//            tile staged through LDS and stored as whole 256-byte pixel rows after the next P1.
// LDS 78.6 KB: W0 6 rows x 6 KB, W1 5 rows x 5,280 B, the normalised patch, the a2 staging.
#include "hn_common.h"
#include "hn_internal.h"
#include "hn_preproc.h"

#include <algorithm>

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

#ifdef HN_EXPERIMENTS
constexpr int NW = 4;                   // k_c12w: waves per workgroup
constexpr int NA0 = 6, NA1 = 5;         // k_c12w: ring rows (a band's conv1 reads 6 a0 rows, conv2 5 a1 rows)
#endif
constexpr int VROW = 6 * 8 * 128;       // W0 ring: bytes per a0 row (6 xi x 8 tiles x 128 B)
constexpr int PXB = 160, W1C = 33;      // W1: bytes per pixel, column slots (x = -1 .. 31)
constexpr int W1ROW = W1C * PXB;
constexpr int IRS = 72, IPL = 35 * IRS; // normalised patch planes: bytes per row (36 bf16) / plane

// The stem (conv0, 1 -> 32 channels, 3x3) as one 16x16x32 MFMA per channel half, the three bf16x3
// products and the bias packed along K: K-group 0 = x_hi(tap j) . w_hi(tap j), 1 = x_lo . w_hi,
// 2 = x_hi . w_lo (taps j = 0 .. 7), 3 = x_hi(8) w_hi(8), x_lo(8) w_hi(8), x_hi(8) w_lo(8), 1 . b_hi,
// 1 . b_lo, 0, 0, 0 (the A side is built once into s_stem, the B side per view in P1).

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

// lane (c, g16) holds 4 channels hi / lo; permlane16_swap (odd rows of vdst <-> even rows of src)
// leaves the even 16-lane row with the hi halves of 8 channels and the odd row with their lo halves
HN_DEV uint4 swap_hilo(uint2 hi, uint2 lo) {
  const auto rx = __builtin_amdgcn_permlane16_swap(hi.x, lo.x, false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(hi.y, lo.y, false, false);
  return make_uint4(rx[0], ry[0], rx[1], ry[1]);
}

// W1 column slot of a1 column x (x = -1 .. 31): even (x + 1) -> (x + 1) / 2, odd -> 17 + x / 2
HN_DEV int w1_slot(int x) { return ((x + 1) & 1) ? 17 + (x >> 1) : (x + 1) >> 1; }

#ifdef HN_EXPERIMENTS  // k_c12w (HN_C12_CFG=14): measured slower than k_c12s, experiments library only
// U8: -1 = fp32 [P,1,32,32] input; HN_RESIZE_* = uint8 patches preprocessed in the load (hn_preproc.h)
// ABL (timing builds of the experiments library only; 0 in production): bit 0 / 1 / 2 skip the stem /
// conv1 / conv2 MFMAs, bit 6 stamps s_memtime at the phase boundaries of every band of each
// workgroup's third patch (k_c12's layout, tools/c12_timeline.py), bit 7 also inside P1
// PD2 / PD3: how many steps ahead P2 / P3 read their B fragments from LDS (rings of PD + 1)
template <int U8 = -1, int ABL = 0, int PD2 = 1, int PD3 = 1>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_c12w(
    const void* __restrict__ in_, float* __restrict__ out, const float* __restrict__ stem_w,
    const float* __restrict__ stem_b, const uint4* __restrict__ w1u, const float* __restrict__ b1,
    const uint4* __restrict__ w2p, const float* __restrict__ b2, int P, float eps, float pmean,
    float pstd, int pnorm) {
  __shared__ __attribute__((aligned(16))) char s_w0[NA0 * VROW];
  __shared__ __attribute__((aligned(16))) char s_w1[NA1 * W1ROW];
  // the normalised patch as bf16 hi / lo planes: [plane][row -1 .. 33][column -2 .. 33], 72-byte rows
  __shared__ __attribute__((aligned(16))) char s_in[2 * IPL];
  __shared__ float red[2 * NW];
  __shared__ __attribute__((aligned(16))) float s_st[2 * 16 * 64];  // a2 staging (k_c12's XST)
  __shared__ __attribute__((aligned(16))) uint4 s_stem[2][64];        // K-packed stem A per channel half
  __shared__ __attribute__((aligned(16))) float s_b1[32], s_b2[64];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // lane-derived addresses are recomputed in each phase from an opaque copy of the lane index (one
  // or two VALU each) instead of being held in registers across the band loop
  auto opaque_lane = [&]() {
    int l = lane;
    asm volatile("" : "+v"(l));
    return l;
  };

  const long per = ((long)P + gridDim.x - 1) / gridDim.x;
  const long pb = (long)xcd_remap(blockIdx.x, gridDim.x) * per;
  const long pe = min((long)P, pb + per);
  if (pb >= pe) return;  // workgroup-uniform

  for (int i = t; i < NA0 * VROW / 16; i += NW * 64) reinterpret_cast<uint4*>(s_w0)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < NA1 * W1ROW / 16; i += NW * 64) reinterpret_cast<uint4*>(s_w1)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < 2 * IPL / 16; i += NW * 64) reinterpret_cast<uint4*>(s_in)[i] = make_uint4(0, 0, 0, 0);
  if (t < 128) {  // stem A (16x16x32) of channel half t >> 6 with the bf16x3 products K-packed (stem_b1)
    const int l = t & 63, ch = 16 * (t >> 6) + (l & 15), gk = l >> 4;
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = 0.f;
      bool lo = false;
      if (gk < 3) {
        v = stem_w[j * 32 + ch];
        lo = gk == 2;
      } else if (j < 3) {
        v = stem_w[8 * 32 + ch];
        lo = j == 2;
      } else if (j < 5) {
        v = stem_b[ch];
        lo = j == 4;
      }
      const __bf16 h = (__bf16)v;
      a[j] = lo ? (__bf16)(v - (float)h) : h;
    }
    s_stem[t >> 6][l] = __builtin_bit_cast(uint4, a);
  }
  for (int i = t; i < 96; i += NW * 64) {
    if (i < 32) s_b1[i] = b1[i];
    else s_b2[i - 32] = b2[i - 32];
  }
  // conv1 U fragments resident: [xi][ky][plane] of this wave's 16-channel group
  const int g1 = w & 1, rp = w >> 1;
  uint4 uw[6][3][2];
#pragma unroll
  for (int xi = 0; xi < 6; ++xi)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) uw[xi][ky][pl] = w1u[(((xi * 3 + ky) * 2 + g1) * 2 + pl) * 64 + lane];
  // conv2 A fragments of this wave's quarter, streamed from L2 two taps ahead
  auto w2_frag = [&](int tap, int pl) {
    int i = ((tap * 4 + w) * 2 + pl) * 64 + lane;
    asm volatile("" : "+v"(i));  // keep the load here (not hoisted out of the patch loop)
    return w2p[i];
  };

  constexpr int PPT = 1024 / (NW * 64);  // patch pixels per thread
  typedef float pxv __attribute__((ext_vector_type(PPT)));
  const float* in = static_cast<const float*>(in_);
  const uint8_t* in8 = static_cast<const uint8_t*>(in_);
  constexpr int INB = U8 == HN_RESIZE_NONE ? 1024 : 4096;
  const int py = (PPT * t) >> 5, px = (PPT * t) & 31;
  pxv vnext;
  hnpre::U8Px<U8 < 0 ? HN_RESIZE_NONE : U8, PPT> rnext;
  if constexpr (U8 < 0)
    vnext = reinterpret_cast<const pxv*>(in + pb * 1024)[t];
  else
    rnext.load(in8 + pb * INB, py, px);
  long pend_patch = -1;  // the band whose a2 rows wait in s_st
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
  const int ph = w & 1, pr = w >> 1;  // P1: the wave's channel half and row pair
  long long* const dbg =
      reinterpret_cast<long long*>(out + (long)P * 24576) + ((long)blockIdx.x * NW + w) * 128;
  long patch_ts = -1;
#define HN_W_TS(K)                                                                                      \
  if constexpr ((ABL & 192) != 0) {                                                                      \
    if (patch == patch_ts && lane == 0) dbg[band * 6 + (K)] = (long long)__builtin_amdgcn_s_memtime(); \
  }
#define HN_W_TS2(K)                                                                                     \
  if constexpr ((ABL & 128) != 0) {                                                                     \
    if (patch == patch_ts && lane == 0 && q == pr) dbg[48 + band * 4 + (K)] = (long long)__builtin_amdgcn_s_memtime(); \
  }

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
        __syncthreads();
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
      const float inv = 1.f / sd;
      const int q0 = PPT * t, y = q0 >> 5, x = q0 & 31;
      static_assert(PPT == 4, "4 pixels per thread");
      uint32_t hw[2], lw[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float a = (v[2 * j] - mean) * inv, b = (v[2 * j + 1] - mean) * inv;
        const __bf16 ha = (__bf16)a, hb = (__bf16)b;
        const __bf16 la = (__bf16)(a - (float)ha), lb = (__bf16)(b - (float)hb);
        hw[j] = (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
        lw[j] = (uint32_t)__builtin_bit_cast(uint16_t, la) | ((uint32_t)__builtin_bit_cast(uint16_t, lb) << 16);
      }
      char* o = s_in + (y + 1) * IRS + (x + 2) * 2;
      reinterpret_cast<uint32_t*>(o)[0] = hw[0];
      reinterpret_cast<uint32_t*>(o)[1] = hw[1];
      reinterpret_cast<uint32_t*>(o + IPL)[0] = lw[0];
      reinterpret_cast<uint32_t*>(o + IPL)[1] = lw[1];
      __syncthreads();
    }
#pragma unroll 1
    for (int band = 0; band < 8; ++band) {
      const int r0 = 2 * band;  // conv2 output rows r0, r0 + 1
      HN_W_TS(0);
      __builtin_amdgcn_s_setprio(1);
      // ---- P1: the band's new a0 rows -> V records in W0 (row y in slot (y + 1) % 6) ---------------
      // wave (pair pr, channel half ph); band 0: rows -1 (zero), 0 .. 4 (pairs 0, 2, 4; row 5 is not
      // written), band b: pairs 4b + 1, 4b + 3 (row 32 is zeroed after its pair)
      if (band == 0)
        for (int i = t; i < VROW / 16; i += NW * 64) reinterpret_cast<uint4*>(s_w0)[i] = make_uint4(0, 0, 0, 0);
      const int npair = band == 0 ? 3 : 2;
#pragma unroll 1
      for (int q = pr; q < npair; q += 2) {
        const int y0 = band == 0 ? 2 * q : 4 * band + 1 + 2 * q;
        // lane roles (16x16x32, N = 8 tiles x 2 a0 rows): tile pT, row pj of the pair; K-group g16
        // reads the lo plane (1) or the hi plane (0, 2, 3)
        const int ln = opaque_lane(), g16 = ln >> 4, pT = ln & 7, pj = (ln >> 3) & 1;
        const bool pg3 = g16 == 3;
        const int pbase = (g16 == 1 ? IPL : 0) + pj * IRS + 8 * pT;  // + (y0 + dy) * IRS: window row dy
        const int lbase = IPL + pj * IRS + 8 * pT;                     // the lo plane (tap 8's x_lo)
        const int pchunk = ((2 * ph + (g16 >> 1)) + 4 * (g16 & 1)) ^ pT;  // V chunk written after the swap
        // window rows y - 1 .. y + 1 (y = y0 + pj), columns 4 pT - 2 .. 4 pT + 5, this lane's plane
        uint32_t R[3][4], L[4];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const uint2 a = *reinterpret_cast<const uint2*>(s_in + pbase + (y0 + dy) * IRS);
          const uint2 b = *reinterpret_cast<const uint2*>(s_in + pbase + (y0 + dy) * IRS + 8);
          R[dy][0] = a.x; R[dy][1] = a.y; R[dy][2] = b.x; R[dy][3] = b.y;
        }
        {
          const uint2 a = *reinterpret_cast<const uint2*>(s_in + lbase + (y0 + 2) * IRS);
          const uint2 b = *reinterpret_cast<const uint2*>(s_in + lbase + (y0 + 2) * IRS + 8);
          L[0] = a.x; L[1] = a.y; L[2] = b.x; L[3] = b.y;
        }
        const uint4 sa = s_stem[ph][ln];
        // pair (W(dy, c), W(dy, c + 1)) of window row dy
        auto pair = [&](int dy, int c) -> uint32_t {
          return (c & 1) ? __builtin_amdgcn_alignbit(R[dy][(c + 1) >> 1], R[dy][(c - 1) >> 1], 16) : R[dy][c >> 1];
        };
        f32x4v acc[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {  // view i: a0 column 4 pT - 1 + i
          const int p = i & 1;
          const uint32_t sel = p ? 0x07060302u : 0x05040100u;
          uint4 b;
          b.x = pair(0, i);
          b.y = __builtin_amdgcn_perm(R[1][i >> 1], R[0][(i + 2) >> 1], sel);  // (W(0, i + 2), W(1, i))
          b.z = pair(1, i + 1);
          b.w = pair(2, i);
          // K-group 3: (x_hi(8), x_lo(8)), (x_hi(8), 1), (1, 0), 0 with tap 8 = W(2, i + 2)
          const uint32_t s0 = __builtin_amdgcn_perm(L[(i + 2) >> 1], R[2][(i + 2) >> 1], sel);
          const uint32_t s1 = __builtin_amdgcn_perm(0x3F80u, R[2][(i + 2) >> 1], p ? 0x05040302u : 0x05040100u);
          b.x = pg3 ? s0 : b.x;
          b.y = pg3 ? s1 : b.y;
          b.z = pg3 ? 0x3F80u : b.z;
          b.w = pg3 ? 0u : b.w;
          acc[i] = (ABL & 1) ? f32x4v{} : mfma16(sa, b, f32x4v{});
        }
        if constexpr ((ABL & 128) != 0) {  // sub-stamp a: the stem's results are available
          float z = acc[0][0] + acc[5][3];
          asm volatile("" : "+v"(z));
          if (z == 1234.5f) dbg[127] = 0;
          HN_W_TS2(0);
        }
        // V = B^T relu(d) (points 0, 1, -1, 1/2, -1/2, inf), channels 16 ph + 4 g16 + c; columns -1 (view 0
        // of tile 0) and 32 (view 5 of tile 7) are conv1's zero padding, not the stem evaluated there:
        // their coefficients (d0 only enters V0, d5 only V5) are zeroed per lane
        const float k0 = pT == 0 ? 0.f : 0.25f, k5 = pT == 7 ? 0.f : 1.f;
        float V[6][4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float d0 = fmaxf(acc[0][c], 0.f), d1 = fmaxf(acc[1][c], 0.f), d2 = fmaxf(acc[2][c], 0.f);
          const float d3 = fmaxf(acc[3][c], 0.f), d4 = fmaxf(acc[4][c], 0.f), d5 = fmaxf(acc[5][c], 0.f);
          V[0][c] = fmaf(k0, d0, fmaf(-1.25f, d2, d4));
          const float pa = fmaf(-0.25f, d2, d4), pb_ = fmaf(-0.25f, d1, d3);
          V[1][c] = pa + pb_;
          V[2][c] = pa - pb_;
          const float pc = d4 - d2, pe_ = d3 - d1;
          V[3][c] = fmaf(0.5f, pe_, pc);
          V[4][c] = fmaf(-0.5f, pe_, pc);
          V[5][c] = fmaf(k5, d5, fmaf(0.25f, d1, -1.25f * d3));
        }
        HN_W_TS2(1);
        char* S = s_w0 + ((y0 + pj + 1) % NA0) * VROW + pT * 128 + 16 * pchunk;
        const bool wr = !(band == 0 && q == 2 && pj == 1);  // band 0's row 5 belongs to band 1
#pragma unroll
        for (int xi = 0; xi < 6; ++xi) {
          uint2 lo;
          const uint2 hi = pack_bf16x4(V[xi][0], V[xi][1], V[xi][2], V[xi][3], lo);
          const uint4 vv = swap_hilo(hi, lo);
          if (wr) *reinterpret_cast<uint4*>(S + xi * 1024) = vv;
        }
        HN_W_TS2(2);  // sub-stamp c: V records issued (the stamp's wait drains the LDS stores)
      }
      if (band == 7 && pr == 1) {  // a0 row 32 (conv1's zero padding): this wave's channel half
        char* S = s_w0 + (33 % NA0) * VROW;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int idx = k * 64 + lane, rec = idx >> 2, cc = idx & 3;
          const int c = (cc & 1) + 2 * ph + 4 * (cc >> 1);
          *reinterpret_cast<uint4*>(S + rec * 128 + 16 * (c ^ (rec & 7))) = make_uint4(0, 0, 0, 0);
        }
      }
      HN_W_TS(1);
      __builtin_amdgcn_s_setprio(0);
      __syncthreads();
      HN_W_TS(2);
      if (pend_patch >= 0) xst_flush();  // the previous band's a2 rows

      // ---- P2: conv1 (F(4,3)) -> W1 ring: a1 rows 4 band + 2 rp + j (j = lane bit 3), group g1 ------
      if (band == 0 && rp == 0) {  // a1 row -1 (conv2's zero padding): this wave's channel group
        const int c16 = lane & 15, g16 = lane >> 4;
#pragma unroll
        for (int hx = 0; hx < 2; ++hx) {
          char* dst = s_w1 + w1_slot(16 * hx + c16) * PXB + 32 * g1 + 8 * g16;
          *reinterpret_cast<uint2*>(dst) = make_uint2(0, 0);
          *reinterpret_cast<uint2*>(dst + 64) = make_uint2(0, 0);
        }
      }
      {
        const int ln = opaque_lane(), g16 = ln >> 4, tj = (ln >> 3) & 1, tt = ln & 7;
        f32x4v acc[6];
#pragma unroll
        for (int xi = 0; xi < 6; ++xi) acc[xi] = f32x4v{};
        acc[1] = *reinterpret_cast<const f32x4v*>(s_b1 + 16 * g1 + 4 * g16);  // the bias rides in m1
        const char* vrow[3];  // a0 row 4 band + 2 rp + tj - 1 + ky: ring slot (row + 1) % 6
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) vrow[ky] = s_w0 + ((4 * band + 2 * rp + tj + ky) % NA0) * VROW + tt * 128;
        const int ohi = 16 * (g16 ^ tt), olo = 16 * ((4 + g16) ^ tt);
        constexpr int R2 = PD2 + 1;
        uint4 bh[R2], bl[R2];
        auto ld2 = [&](int s) {
          bh[s % R2] = *reinterpret_cast<const uint4*>(vrow[s / 6] + (s % 6) * 1024 + ohi);
          bl[s % R2] = *reinterpret_cast<const uint4*>(vrow[s / 6] + (s % 6) * 1024 + olo);
        };
#pragma unroll
        for (int s = 0; s < PD2; ++s) ld2(s);
#pragma unroll
        for (int s = 0; s < 18; ++s) {
          const int ky = s / 6, xi = s % 6;
          if (s + PD2 < 18) ld2(s + PD2);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((ABL & 2) != 0) {
            acc[xi][0] += __builtin_bit_cast(float, bh[s % R2].x ^ bl[s % R2].y);
            continue;
          }
          acc[xi] = mfma16(uw[xi][ky][1], bh[s % R2], acc[xi]);
          acc[xi] = mfma16(uw[xi][ky][0], bl[s % R2], acc[xi]);
          acc[xi] = mfma16(uw[xi][ky][0], bh[s % R2], acc[xi]);
        }
        // y = A^T m: lane (tile tt, row tj, channels 16 g1 + 4 g16 ..) -> columns 4 tt .. 4 tt + 3
        f32x4v yv[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float s12 = acc[1][c] + acc[2][c], d12 = acc[1][c] - acc[2][c];
          const float s34 = acc[3][c] + acc[4][c], d34 = acc[3][c] - acc[4][c];
          yv[0][c] = acc[0][c] + s12 + s34;
          yv[1][c] = fmaf(0.5f, d34, d12);
          yv[2][c] = fmaf(0.25f, s34, s12);
          yv[3][c] = fmaf(0.125f, d34, d12) + acc[5][c];
        }
        char* prow = s_w1 + ((4 * band + 2 * rp + tj + 1) % NA1) * W1ROW + 32 * g1 + 16 * (g16 >> 1) + 64 * (g16 & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint2 lo;
          const uint2 hi = pack_bf16x4(fmaxf(yv[i][0], 0.f), fmaxf(yv[i][1], 0.f), fmaxf(yv[i][2], 0.f),
                                       fmaxf(yv[i][3], 0.f), lo);
          *reinterpret_cast<uint4*>(prow + w1_slot(4 * tt + i) * PXB) = swap_hilo(hi, lo);
        }
      }
      HN_W_TS(3);
      uint4 wq[3][2];  // conv2 fragments, the first two taps in flight across the barrier
#pragma unroll
      for (int tap = 0; tap < 2; ++tap)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) wq[tap][pl] = w2_frag(tap, pl);
      __syncthreads();
      HN_W_TS(4);

      __builtin_amdgcn_s_setprio(1);
      // ---- P3: conv2 (stride 2), output rows r0, r0 + 1, this wave's 16-channel quarter ----------
      {
        const int ln = opaque_lane(), c16 = ln & 15, g16 = ln >> 4;
        f32x4v acc[2];
        acc[0] = acc[1] = *reinterpret_cast<const f32x4v*>(s_b2 + 16 * w + 4 * g16);
        // output column c16 reads a1 column 2 c16 - 1 + dx: W1 slot c16 (dx 0), 17 + c16 (dx 1),
        // c16 + 1 (dx 2); a1 rows 2 (r0 + ry) - 1 + dy sit in ring slots (2 (r0 + ry) + dy) % 5
        const char* srow[2][3];
#pragma unroll
        for (int ry = 0; ry < 2; ++ry)
#pragma unroll
          for (int dy = 0; dy < 3; ++dy) srow[ry][dy] = s_w1 + (((2 * (r0 + ry) + dy) % NA1) * W1C + c16) * PXB + 16 * g16;
        constexpr int R3 = PD3 + 1;
        uint4 bh[R3], bl[R3];
        auto ld3 = [&](int j) {
          const int tn = j >> 1, rn = j & 1;
          const int dy = tn / 3, dx = tn % 3;
          const char* p = srow[rn][dy] + (dx == 1 ? 17 : (dx >> 1)) * PXB;
          bh[j % R3] = *reinterpret_cast<const uint4*>(p);
          bl[j % R3] = *reinterpret_cast<const uint4*>(p + 64);
        };
#pragma unroll
        for (int j = 0; j < PD3; ++j) ld3(j);
#pragma unroll
        for (int j = 0; j < 18; ++j) {
          const int tap = j >> 1, ry = j & 1;
          if (ry == 0 && tap + 2 < 9) {
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) wq[(tap + 2) % 3][pl] = w2_frag(tap + 2, pl);
          }
          if (j + PD3 < 18) ld3(j + PD3);
          __builtin_amdgcn_sched_barrier(0);
          const uint4* wc = wq[tap % 3];
          if constexpr ((ABL & 4) != 0) {
            acc[ry][0] += __builtin_bit_cast(float, bh[j % R3].x ^ bl[j % R3].y ^ wc[0].x);
            continue;
          }
          acc[ry] = mfma16(wc[1], bh[j % R3], acc[ry]);
          acc[ry] = mfma16(wc[0], bl[j % R3], acc[ry]);
          acc[ry] = mfma16(wc[0], bh[j % R3], acc[ry]);
        }
#pragma unroll
        for (int ry = 0; ry < 2; ++ry)
          *reinterpret_cast<f32x4v*>(s_st + ((ry * 16 + c16) * 16 + ((4 * w + g16) ^ (c16 & 7))) * 4) =
              __builtin_elementwise_max(acc[ry], f32x4v{});
        pend_patch = patch;
        pend_row = r0;
      }
      HN_W_TS(5);
      // no barrier: the next band's P1 writes only W0, which P3 does not read; its barrier orders this
      // P3's W1 reads before the next P2's W1 writes
    }  // band
  }  // patch
  __syncthreads();
  xst_flush();
#undef HN_W_TS
#undef HN_W_TS2
}

#endif  // HN_EXPERIMENTS

// ----------------------------------------------------------------------------------------------------
// k_c12s: k_c12w's arithmetic (the K-packed stem, conv1 as F(4,3), direct conv2 -- bit-identical to it)
// with the roles split per SIMD and the bands software-pipelined.  In k_c12 / k_c12w every wave runs
// P1 -> P2 -> P3 of its band behind two barriers, and the phase timelines (tools/c12_timeline.py) show
// the band set by the prioritised P1 + P3 of both workgroups of a CU, with P2 in their shadow: halving
// P2's MFMA work (k_c12w) moved little.  Here one workgroup of 8 waves per CU (waves w and w + 4 share
// a SIMD) runs, between two barriers of step g:
//   A-waves 0-3: P2 of band g (conv1, U resident: 144 VGPRs), as k_c12w's P2;
//   B-waves 4-7: P3 of band g - 1 (conv2 with this wave's quarter of its weights resident: 72 VGPRs, so
//                no weight stream from L2), P1 of band g + 1 (k_c12w's), the a2 stores of band g - 2 and,
//                spread over bands 2-6, the input_norm of the next patch (s_in double-buffered).
// So every SIMD has one conv1 and one conv2 MFMA stream in flight at once and the stem's latency chain
// runs beside them.  Rings over the workgroup's whole patch range (row G = 32 patch + y): W0 10 a0 rows
// (P2 of band g reads 6 while P1 of band g + 1 writes 4), W1 10 a1 rows (P3 of band g - 1 reads 5 while
// P2 of band g writes 4), each with one more all-zero row that the padding rows (-1, 32) read.  LDS
// 152.5 KB, one workgroup per CU.
//
// P2's N index n stands for tile n >> 1 of a1 row n & 1 (k_c12w: tile n & 7, row n >> 3), so each 8-lane group
// of its epilogue's ds_write_b128 holds 4 tiles x 2 rows: 2-way at the 160-byte W1 pixel instead of 8 tiles of one
// row on 2 distinct 16-byte positions (4-way).  Its V-record reads stay conflict-free because W0 rows are padded
// to VROW + 128 (adjacent rows in opposite halves of the 256-byte bank row; only reads of the zero row collide),
// and the W1 ring has 10 rows so that the ring's wrap (-9 rows) keeps row pairs apart as +1 does
// (tests/test_lds_banks.py::test_c12s_*).  P3's reads are k_c12w's (conflict-free, immediate offsets).
constexpr int SNA0 = 10, SNA1 = 10;
constexpr int SVROW = VROW + 128;

// PRB: the B-waves' wave priority (1: their VALU-heavy stem chain and conv2 issue ahead of conv1)
// ABL (experiments library only): bit 0 / 1 / 2 skip the stem / conv1 / conv2 MFMAs, bit 3 / 4 the B-waves'
// P3 / P1 phases entirely; bit 6 stamps
// s_memtime at the phase boundaries of the steps of each workgroup's third patch (tools/c12_timeline.py)
// P1A: P1 runs on the A-waves (after P2) instead of the B-waves (after P3)
// P1I: P1 on the B-waves with its pieces inside P3's MFMA stream
// ILV: P2 / P3 with independent accumulator chains interleaved MFMA by MFMA
template <int U8 = -1, int PD2 = 1, int PD3 = 1, int PRB = 1, int ABL = 0, bool P1A = false, bool P1I = false,
          bool ILV = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_c12s(
    const void* __restrict__ in_, float* __restrict__ out, const float* __restrict__ stem_w,
    const float* __restrict__ stem_b, const uint4* __restrict__ w1u, const float* __restrict__ b1,
    const uint4* __restrict__ w2p, const float* __restrict__ b2, int P, float eps, float pmean,
    float pstd, int pnorm) {
  __shared__ __attribute__((aligned(16))) char s_w0[(SNA0 + 1) * SVROW];
  __shared__ __attribute__((aligned(16))) char s_w1[(SNA1 + 1) * W1ROW];
  __shared__ __attribute__((aligned(16))) char s_in[2][2 * IPL];
  __shared__ __attribute__((aligned(16))) float s_st[2][2 * 16 * 64];  // a2 staging, by band parity
  __shared__ __attribute__((aligned(16))) uint4 s_stem[2][64];
  __shared__ __attribute__((aligned(16))) float s_b0[32], s_b1[32], s_b2[64];
  __shared__ float red[8];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool isA = w < 4;
  const int aw = w & 3;  // index within the role

  const long per = ((long)P + gridDim.x - 1) / gridDim.x;
  const long pb = (long)xcd_remap(blockIdx.x, gridDim.x) * per;
  const long pe = min((long)P, pb + per);
  if (pb >= pe) return;  // workgroup-uniform
  const int np = (int)(pe - pb), G = 8 * np;

  for (int i = t; i < (SNA0 + 1) * SVROW / 16; i += 512) reinterpret_cast<uint4*>(s_w0)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < (SNA1 + 1) * W1ROW / 16; i += 512) reinterpret_cast<uint4*>(s_w1)[i] = make_uint4(0, 0, 0, 0);
  for (int i = t; i < 4 * IPL / 16; i += 512) reinterpret_cast<uint4*>(&s_in[0][0])[i] = make_uint4(0, 0, 0, 0);
  if (t < 128) {  // stem A (16x16x32) of channel half t >> 6, K-packed as k_c12w's without the bias slots
    const int l = t & 63, ch = 16 * (t >> 6) + (l & 15), gk = l >> 4;
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = 0.f;
      bool lo = false;
      if (gk < 3) {
        v = stem_w[j * 32 + ch];
        lo = gk == 2;
      } else if (j < 3) {
        v = stem_w[8 * 32 + ch];
        lo = j == 2;
      }
      const __bf16 h = (__bf16)v;
      a[j] = lo ? (__bf16)(v - (float)h) : h;
    }
    s_stem[t >> 6][l] = __builtin_bit_cast(uint4, a);
  }
  for (int i = t; i < 128; i += 512) {
    if (i < 32) s_b1[i] = b1[i];
    else if (i < 96) s_b2[i - 32] = b2[i - 32];
    else s_b0[i - 96] = stem_b[i - 96];
  }
  auto opaque_lane = [&]() {
    int l = lane;
    asm volatile("" : "+v"(l));
    return l;
  };
  long long* const dbg = reinterpret_cast<long long*>(out + (long)P * 24576) + ((long)blockIdx.x * 8 + w) * 128;
#define HN_S_TS(K)                                                                                           \
  if constexpr ((ABL & 64) != 0) {                                                                           \
    if (g >= 16 && g < 24 && lane == 0) dbg[(g - 16) * 6 + (K)] = (long long)__builtin_amdgcn_s_memtime();   \
  }
  // ABL & 64: every wave's start / end in the 100 MHz clock (slots 120 / 121), for the launch's tail
#define HN_S_RT(K)                                                                                           \
  if constexpr ((ABL & 64) != 0) {                                                                           \
    if (lane == 0) dbg[120 + (K)] = (long long)__builtin_amdgcn_s_memrealtime();                             \
  }
  HN_S_RT(0);

  // P1 of band gq (k_c12w's): a0 rows -> V records, slot (32 p + y) % 10; the padding rows are not
  // stored (the zero row stands for them).  p1_front: the window reads, the B operands and the 6 stem
  // MFMAs of pair q; p1_back: ReLU, the transform, the split and the V stores (none for a band past the
  // range: gq >= G).
  const int ph = aw & 1, pr = aw >> 1;  // the wave's channel half and row pair (in its role)
  auto p1_y0 = [&](int gq, int q) { const int band = gq & 7; return band == 0 ? 2 * q : 4 * band + 1 + 2 * q; };
  struct P1Ctx {  // one pair-iteration of P1 in flight
    uint32_t R[3][4], L[4];
    uint4 sa;
    f32x4v bias0, acc[6];
    float V[6][4];
    float k0, k5;  // V0's / V5's coefficient of the padding columns -1 / 32 (zero on tiles 0 / 7)
    char* S;       // this lane's V record chunk in the row's ring slot (xi adds 1 KB)
    bool wr, pg3;
  };
  auto p1_read = [&](int gq, int q, P1Ctx& c) {  // the window (issued; consumed by p1_mfma) + lane roles
    const int y0 = p1_y0(gq, q);
    const char* sin = s_in[(gq >> 3) & 1];
    const int ln = opaque_lane(), g16 = ln >> 4, pT = ln & 7, pj = (ln >> 3) & 1;
    const int pbase = (g16 == 1 ? IPL : 0) + pj * IRS + 8 * pT;
    const int lbase = IPL + pj * IRS + 8 * pT;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const uint2 a = *reinterpret_cast<const uint2*>(sin + pbase + (y0 + dy) * IRS);
      const uint2 b = *reinterpret_cast<const uint2*>(sin + pbase + (y0 + dy) * IRS + 8);
      c.R[dy][0] = a.x; c.R[dy][1] = a.y; c.R[dy][2] = b.x; c.R[dy][3] = b.y;
    }
    {
      const uint2 a = *reinterpret_cast<const uint2*>(sin + lbase + (y0 + 2) * IRS);
      const uint2 b = *reinterpret_cast<const uint2*>(sin + lbase + (y0 + 2) * IRS + 8);
      c.L[0] = a.x; c.L[1] = a.y; c.L[2] = b.x; c.L[3] = b.y;
    }
    c.pg3 = g16 == 3;
    c.k0 = pT == 0 ? 0.f : 0.25f;
    c.k5 = pT == 7 ? 0.f : 1.f;
    {
      const int p = gq >> 3, band = gq & 7, y = y0 + pj;
      const int pchunk = ((2 * ph + (g16 >> 1)) + 4 * (g16 & 1)) ^ pT;
      c.S = s_w0 + ((32 * p + y) % SNA0) * SVROW + pT * 128 + 16 * pchunk;
      // row 5 belongs to band 1; row 32 is padding; a band past the range stores nothing
      c.wr = gq < G && y <= 31 && !(band == 0 && y == 5);
    }
    c.sa = s_stem[ph][ln];
    // the stem bias is the accumulators' initial value (exact fp32); K-group 3's slots 3 .. 7 are zero
    // on the A side, so only its first two B dwords need the tap-8 values
    c.bias0 = *reinterpret_cast<const f32x4v*>(s_b0 + 16 * ph + 4 * g16);
  };
  auto p1_mfma = [&](P1Ctx& c, int i0, int i1) {  // views i0 .. i1 - 1: B operands + stem MFMAs
    const bool pg3 = c.pg3;
    auto pair = [&](int dy, int cc) -> uint32_t {
      return (cc & 1) ? __builtin_amdgcn_alignbit(c.R[dy][(cc + 1) >> 1], c.R[dy][(cc - 1) >> 1], 16)
                      : c.R[dy][cc >> 1];
    };
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const int pp = i & 1;
      const uint32_t sel = pp ? 0x07060302u : 0x05040100u;
      uint4 b;
      b.x = pair(0, i);
      b.y = __builtin_amdgcn_perm(c.R[1][i >> 1], c.R[0][(i + 2) >> 1], sel);
      b.z = pair(1, i + 1);
      b.w = pair(2, i);
      // K-group 3: (x_hi(8), x_lo(8)), (x_hi(8), -) with tap 8 = W(2, i + 2)
      const uint32_t s0 = __builtin_amdgcn_perm(c.L[(i + 2) >> 1], c.R[2][(i + 2) >> 1], sel);
      const uint32_t s1 = pp ? (c.R[2][(i + 2) >> 1] >> 16) : c.R[2][(i + 2) >> 1];
      b.x = pg3 ? s0 : b.x;
      b.y = pg3 ? s1 : b.y;
      c.acc[i] = (ABL & 1) ? f32x4v{} : mfma16(c.sa, b, c.bias0);
    }
  };
  auto p1_vt = [&](P1Ctx& c, int ch) {  // ReLU + V = B^T d (points 0, 1, -1, 1/2, -1/2, inf), channel ch
    const float k0 = c.k0, k5 = c.k5;
    const float d0 = fmaxf(c.acc[0][ch], 0.f), d1 = fmaxf(c.acc[1][ch], 0.f), d2 = fmaxf(c.acc[2][ch], 0.f);
    const float d3 = fmaxf(c.acc[3][ch], 0.f), d4 = fmaxf(c.acc[4][ch], 0.f), d5 = fmaxf(c.acc[5][ch], 0.f);
    c.V[0][ch] = fmaf(k0, d0, fmaf(-1.25f, d2, d4));
    const float pa = fmaf(-0.25f, d2, d4), pb_ = fmaf(-0.25f, d1, d3);
    c.V[1][ch] = pa + pb_;
    c.V[2][ch] = pa - pb_;
    const float pc = d4 - d2, pe_ = d3 - d1;
    c.V[3][ch] = fmaf(0.5f, pe_, pc);
    c.V[4][ch] = fmaf(-0.5f, pe_, pc);
    c.V[5][ch] = fmaf(k5, d5, fmaf(0.25f, d1, -1.25f * d3));
  };
  auto p1_store = [&](P1Ctx& c, int xi) {  // split V_xi to bf16 hi / lo -> its V record chunk
    uint2 lo;
    const uint2 hi = pack_bf16x4(c.V[xi][0], c.V[xi][1], c.V[xi][2], c.V[xi][3], lo);
    const uint4 vv = swap_hilo(hi, lo);
    if (c.wr) *reinterpret_cast<uint4*>(c.S + xi * 1024) = vv;
  };
  auto p1_front = [&](int gq, int q, P1Ctx& c) {
    p1_read(gq, q, c);
    p1_mfma(c, 0, 6);
  };
  auto p1_back = [&](P1Ctx& c) {
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) p1_vt(c, ch);
#pragma unroll
    for (int xi = 0; xi < 6; ++xi) p1_store(c, xi);
  };
  auto p1 = [&](int gq) {
    const int npair = (gq & 7) == 0 ? 3 : 2;
#pragma unroll 1
    for (int q = pr; q < npair; q += 2) {
      P1Ctx c;
      p1_front(gq, q, c);
      p1_back(c);
    }
  };

  if (isA) {
    // ================================ A-waves: P2 (conv1) ================================
    const int g1 = aw & 1, rp = aw >> 1;
    uint4 uw[6][3][2];
#pragma unroll
    for (int xi = 0; xi < 6; ++xi)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) uw[xi][ky][pl] = w1u[(((xi * 3 + ky) * 2 + g1) * 2 + pl) * 64 + lane];
    for (int k = 0; k < 3; ++k) __syncthreads();  // the B-waves' prologue: input_norm
    if constexpr (P1A) p1(0);
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g <= G; ++g) {
      HN_S_TS(0);
      if (g < G) {
        const int p = g >> 3, band = g & 7;
        const int ln = opaque_lane(), g16 = ln >> 4, tj = ln & 1, tt = (ln >> 1) & 7;
        f32x4v acc[6];
#pragma unroll
        for (int xi = 0; xi < 6; ++xi) acc[xi] = f32x4v{};
        acc[1] = *reinterpret_cast<const f32x4v*>(s_b1 + 16 * g1 + 4 * g16);  // the bias rides in m1
        const char* vrow[3];  // a0 row r = 4 band + 2 rp + tj - 1 + ky: slot (32 p + r) % 10, padding -> 10
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int r = 4 * band + 2 * rp + tj - 1 + ky;
          const int slot = (r < 0 || r > 31) ? SNA0 : (32 * p + r) % SNA0;
          vrow[ky] = s_w0 + slot * SVROW + tt * 128;
        }
        const int ohi = 16 * (g16 ^ tt), olo = 16 * ((4 + g16) ^ tt);
        constexpr int R2 = PD2 + 1;
        uint4 bh[R2], bl[R2];
        auto ld2 = [&](int s) {
          if constexpr ((ABL & 32) != 0) {  // timing: one B fragment for every step (no LDS stream)
            if (s > 0) { bh[s % R2] = bh[0]; bl[s % R2] = bl[0]; return; }
          }
          bh[s % R2] = *reinterpret_cast<const uint4*>(vrow[s / 6] + (s % 6) * 1024 + ohi);
          bl[s % R2] = *reinterpret_cast<const uint4*>(vrow[s / 6] + (s % 6) * 1024 + olo);
        };
        if constexpr (ILV) {
          // groups of three xi (one ky): each product of the three chains in turn, so dependent MFMAs
          // are three apart (an MFMA reading the previous one's result as C right after it stalls)
          uint4 gh[2][3], gl[2][3];
          auto ldg = [&](int q) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              const int st = 3 * q + i;
              gh[q & 1][i] = *reinterpret_cast<const uint4*>(vrow[st / 6] + (st % 6) * 1024 + ohi);
              gl[q & 1][i] = *reinterpret_cast<const uint4*>(vrow[st / 6] + (st % 6) * 1024 + olo);
            }
          };
          ldg(0);
#pragma unroll
          for (int q = 0; q < 6; ++q) {
            if (q + 1 < 6) ldg(q + 1);
            __builtin_amdgcn_sched_barrier(0);
            const int ky = q >> 1, x0 = 3 * (q & 1);
#pragma unroll
            for (int i = 0; i < 3; ++i) acc[x0 + i] = mfma16(uw[x0 + i][ky][1], gh[q & 1][i], acc[x0 + i]);
#pragma unroll
            for (int i = 0; i < 3; ++i) acc[x0 + i] = mfma16(uw[x0 + i][ky][0], gl[q & 1][i], acc[x0 + i]);
#pragma unroll
            for (int i = 0; i < 3; ++i) acc[x0 + i] = mfma16(uw[x0 + i][ky][0], gh[q & 1][i], acc[x0 + i]);
          }
        } else {
#pragma unroll
        for (int s = 0; s < PD2; ++s) ld2(s);
#pragma unroll
        for (int s = 0; s < 18; ++s) {
          const int ky = s / 6, xi = s % 6;
          if (s + PD2 < 18) ld2(s + PD2);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((ABL & 2) != 0) {
            acc[xi][0] += __builtin_bit_cast(float, bh[s % R2].x ^ bl[s % R2].y);
            continue;
          }
          acc[xi] = mfma16(uw[xi][ky][1], bh[s % R2], acc[xi]);
          acc[xi] = mfma16(uw[xi][ky][0], bl[s % R2], acc[xi]);
          acc[xi] = mfma16(uw[xi][ky][0], bh[s % R2], acc[xi]);
        }
        }
        f32x4v yv[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float s12 = acc[1][c] + acc[2][c], d12 = acc[1][c] - acc[2][c];
          const float s34 = acc[3][c] + acc[4][c], d34 = acc[3][c] - acc[4][c];
          yv[0][c] = acc[0][c] + s12 + s34;
          yv[1][c] = fmaf(0.5f, d34, d12);
          yv[2][c] = fmaf(0.25f, s34, s12);
          yv[3][c] = fmaf(0.125f, d34, d12) + acc[5][c];
        }
        char* prow = s_w1 + ((32 * p + 4 * band + 2 * rp + tj) % SNA1) * W1ROW + 32 * g1 + 16 * (g16 >> 1) +
                     64 * (g16 & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint2 lo;
          const uint2 hi = pack_bf16x4(fmaxf(yv[i][0], 0.f), fmaxf(yv[i][1], 0.f), fmaxf(yv[i][2], 0.f),
                                       fmaxf(yv[i][3], 0.f), lo);
          *reinterpret_cast<uint4*>(prow + w1_slot(4 * tt + i) * PXB) = swap_hilo(hi, lo);
        }
      }
      if constexpr (P1A) {
        if (g + 1 < G) p1(g + 1);
      }
      HN_S_TS(1);
      __syncthreads();
      HN_S_TS(2);
    }
    HN_S_RT(1);
    return;
  }

  // ================================ B-waves: P3 (conv2), P1 (stem), input_norm, stores ================
  const int bt = t - 256;  // 0 .. 255
  uint4 w2r[9][2];         // this wave's conv2 quarter, resident
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) w2r[tap][pl] = w2p[((tap * 4 + aw) * 2 + pl) * 64 + lane];
  if constexpr (PRB != 0) __builtin_amdgcn_s_setprio(PRB);

  // input_norm of a patch in three pieces (one per step, the barriers between them order the reductions)
  const float* in = static_cast<const float*>(in_);
  const uint8_t* in8 = static_cast<const uint8_t*>(in_);
  constexpr int INB = U8 == HN_RESIZE_NONE ? 1024 : 4096;
  const int py = (4 * bt) >> 5, px = (4 * bt) & 31;
  typedef float pxv __attribute__((ext_vector_type(4)));
  pxv v;
  hnpre::U8Px<U8 < 0 ? HN_RESIZE_NONE : U8, 4> raw;
  float mean = 0.f;
  auto norm_load = [&](long patch) {
    if constexpr (U8 < 0) v = reinterpret_cast<const pxv*>(in + patch * 1024)[bt];
    else raw.load(in8 + patch * INB, py, px);
  };
  auto norm_sum = [&]() {
    if constexpr (U8 >= 0) {
      int q[4];
      raw.resized(py, px, q);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = hnpre::to_input(q[j], pmean, pstd, pnorm);
    }
    if (eps >= 0.f) {
      const float s = wave_sum(v[0] + v[1] + v[2] + v[3]);
      if (lane == 0) red[aw] = s;
    }
  };
  auto norm_var = [&]() {
    if (eps >= 0.f) {
      mean = (red[0] + red[1] + red[2] + red[3]) * (1.f / 1024.f);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) q += (v[j] - mean) * (v[j] - mean);
      q = wave_sum(q);
      if (lane == 0) red[4 + aw] = q;
    }
  };
  auto norm_write = [&](int buf) {  // (x - mean) / (std_unbiased + eps) -> bf16 hi / lo planes
    float sd = 1.f, mu = 0.f;
    if (eps >= 0.f) {
      mu = mean;
      sd = sqrtf((red[4] + red[5] + red[6] + red[7]) * (1.f / 1023.f)) + eps;
    }
    const float inv = 1.f / sd;
    uint32_t hw[2], lw[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float a = (v[2 * j] - mu) * inv, b = (v[2 * j + 1] - mu) * inv;
      const __bf16 ha = (__bf16)a, hb = (__bf16)b;
      const __bf16 la = (__bf16)(a - (float)ha), lb = (__bf16)(b - (float)hb);
      hw[j] = (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
      lw[j] = (uint32_t)__builtin_bit_cast(uint16_t, la) | ((uint32_t)__builtin_bit_cast(uint16_t, lb) << 16);
    }
    char* o = s_in[buf] + (py + 1) * IRS + (px + 2) * 2;
    reinterpret_cast<uint32_t*>(o)[0] = hw[0];
    reinterpret_cast<uint32_t*>(o)[1] = hw[1];
    reinterpret_cast<uint32_t*>(o + IPL)[0] = lw[0];
    reinterpret_cast<uint32_t*>(o + IPL)[1] = lw[1];
  };

  // P3 of band gq: conv2, this wave's quarter, output rows 2 band, 2 band + 1 -> s_st[gq & 1]; hook(j)
  // runs after step j's MFMAs are issued (P1's pieces fill P3's MFMA shadow in the fused schedule)
  auto p3h = [&](int gq, auto&& hook) {
    const int p = gq >> 3, band = gq & 7;
    const int ln = opaque_lane(), c16 = ln & 15, g16 = ln >> 4;
    f32x4v acc[2];
    acc[0] = acc[1] = *reinterpret_cast<const f32x4v*>(s_b2 + 16 * aw + 4 * g16);
    const char* srow[2][3];  // a1 row r = 4 band + 2 ry - 1 + dy: slot (32 p + r) % 10, row -1 -> 10
#pragma unroll
    for (int ry = 0; ry < 2; ++ry)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int r = 4 * band + 2 * ry - 1 + dy;
        const int slot = r < 0 ? SNA1 : (32 * p + r) % SNA1;
        srow[ry][dy] = s_w1 + (slot * W1C + c16) * PXB + 16 * g16;
      }
    constexpr int R3 = PD3 + 1;
    uint4 bh[R3], bl[R3];
    auto ld3 = [&](int j) {
      const int tn = j >> 1, rn = j & 1;
      const int dy = tn / 3, dx = tn % 3;
      const char* pp = srow[rn][dy] + (dx == 1 ? 17 : (dx >> 1)) * PXB;
      bh[j % R3] = *reinterpret_cast<const uint4*>(pp);
      bl[j % R3] = *reinterpret_cast<const uint4*>(pp + 64);
    };
    if constexpr (ILV) {
      // per tap both rows' chains interleaved MFMA by MFMA (dependent MFMAs two apart)
      uint4 th[2][2], tl[2][2];
      auto ldt = [&](int tap) {
#pragma unroll
        for (int rn = 0; rn < 2; ++rn) {
          const int dy = tap / 3, dx = tap % 3;
          const char* pp = srow[rn][dy] + (dx == 1 ? 17 : (dx >> 1)) * PXB;
          th[tap & 1][rn] = *reinterpret_cast<const uint4*>(pp);
          tl[tap & 1][rn] = *reinterpret_cast<const uint4*>(pp + 64);
        }
      };
      ldt(0);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) ldt(tap + 1);
        __builtin_amdgcn_sched_barrier(0);
        const uint4(&h)[2] = th[tap & 1];
        const uint4(&l)[2] = tl[tap & 1];
        acc[0] = mfma16(w2r[tap][1], h[0], acc[0]);
        acc[1] = mfma16(w2r[tap][1], h[1], acc[1]);
        acc[0] = mfma16(w2r[tap][0], l[0], acc[0]);
        acc[1] = mfma16(w2r[tap][0], l[1], acc[1]);
        acc[0] = mfma16(w2r[tap][0], h[0], acc[0]);
        acc[1] = mfma16(w2r[tap][0], h[1], acc[1]);
        hook(2 * tap);
        hook(2 * tap + 1);
      }
    } else {
#pragma unroll
    for (int j = 0; j < PD3; ++j) ld3(j);
#pragma unroll
    for (int j = 0; j < 18; ++j) {
      const int tap = j >> 1, ry = j & 1;
      if (j + PD3 < 18) ld3(j + PD3);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((ABL & 4) != 0) {
        acc[ry][0] += __builtin_bit_cast(float, bh[j % R3].x ^ bl[j % R3].y ^ w2r[tap][0].x);
        continue;
      }
      acc[ry] = mfma16(w2r[tap][1], bh[j % R3], acc[ry]);
      acc[ry] = mfma16(w2r[tap][0], bl[j % R3], acc[ry]);
      acc[ry] = mfma16(w2r[tap][0], bh[j % R3], acc[ry]);
      hook(j);
    }
    }
    float* st = s_st[gq & 1];
#pragma unroll
    for (int ry = 0; ry < 2; ++ry)
      *reinterpret_cast<f32x4v*>(st + ((ry * 16 + c16) * 16 + ((4 * aw + g16) ^ (c16 & 7))) * 4) =
          __builtin_elementwise_max(acc[ry], f32x4v{});
  };
  auto p3 = [&](int gq) { p3h(gq, [](int) {}); };
  // a2 rows of band gq from s_st[gq & 1]: wave row aw >> 1, pixels 8 (aw & 1) + (lane >> 4) + 4 j
  auto flush = [&](int gq) {
    const long patch = pb + (gq >> 3);
    const int row = 2 * (gq & 7) + (aw >> 1), q = lane & 15;
    const float* st = s_st[gq & 1];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int x = 8 * (aw & 1) + (lane >> 4) + 4 * j;
      const f32x4v vv = *reinterpret_cast<const f32x4v*>(st + (((aw >> 1) * 16 + x) * 16 + (q ^ (x & 7))) * 4);
      *reinterpret_cast<f32x4v*>(out + ((patch * 16 + row) * 16 + x) * 64 + 4 * q) = vv;
    }
  };

  // prologue: the first patch's input_norm, P1 of its band 0
  norm_load(pb);
  norm_sum();
  __syncthreads();
  norm_var();
  __syncthreads();
  norm_write(0);
  __syncthreads();
  if constexpr (!P1A) p1(0);
  __syncthreads();
#pragma unroll 1
  for (int g = 0; g <= G; ++g) {
    const int band = g & 7;
    const int pn = (g >> 3) + 1;  // the next patch (relative), prepared over bands 2 .. 6
    HN_S_TS(0);
    if (g >= 2) flush(g - 2);
    HN_S_TS(1);
    if constexpr (P1I) {
      // P1 of band g + 1 inside P3 of band g - 1 (pair pr; band 0's third pair separately): its window reads
      // ahead of P3, its B operands and stem MFMAs after P3's steps 0 / 1, ReLU + transform after steps 3-6,
      // the V stores after steps 7-12
      P1Ctx c1;
      if (g >= 1) {
        p1_read(g + 1, pr, c1);
        p3h(g - 1, [&](int j) {
          if (j == 0) p1_mfma(c1, 0, 3);
          else if (j == 1) p1_mfma(c1, 3, 6);
          else if (j >= 3 && j < 7) p1_vt(c1, j - 3);
          else if (j >= 7 && j < 13) p1_store(c1, j - 7);
        });
      } else {
        p1_front(g + 1, pr, c1);
        p1_back(c1);
      }
      HN_S_TS(2);
      if (((g + 1) & 7) == 0 && g + 1 < G && pr == 0) {
        P1Ctx c2;
        p1_front(g + 1, 2, c2);
        p1_back(c2);
      }
    } else {
      if ((ABL & 8) == 0 && g >= 1) p3(g - 1);
      HN_S_TS(2);
      if constexpr (!P1A) {
        if ((ABL & 16) == 0 && g + 1 < G) p1(g + 1);
      }
    }
    HN_S_TS(3);
    if (g < G && pn < np) {
      if (band == 2) norm_load(pb + pn);
      else if (band == 4) norm_sum();
      else if (band == 5) norm_var();
      else if (band == 6) norm_write(pn & 1);
    }
    HN_S_TS(4);
    __syncthreads();
    HN_S_TS(5);
  }
  flush(G - 1);
  HN_S_RT(1);
#undef HN_S_TS
#undef HN_S_RT
}

}  // namespace

#ifdef HN_EXPERIMENTS
hipError_t hn_launch_c12w(const float* in, float* out, const HardnetDev& d, int P, float eps, hipStream_t st,
                          const HnU8In* u8, int abl) {
  if (P <= 0) return hipSuccess;
  if (!d.c12_w1w) return hipErrorInvalidValue;
  int resident = 0;
  const hipError_t e = hn_resident_blocks(reinterpret_cast<const void*>(&k_c12w<-1>), NW * 64, 0, &resident);
  if (e != hipSuccess) return e;
  const int grid = (int)std::min<long>((long)P, resident);
  const void* src = u8 ? u8->in : static_cast<const void*>(in);
  const float pm = u8 ? u8->mean : 0.f, ps = u8 ? u8->stdv : 1.f;
  const int pn = u8 ? u8->normalize : 0;
#define HN_C12W_GO(U, ...)                                                                                \
  hipLaunchKernelGGL((k_c12w<U, ##__VA_ARGS__>), dim3(grid), dim3(NW * 64), 0, st, src, out, d.stem_w, d.stem_b,        \
                     static_cast<const uint4*>(d.c12_w1w), d.bias[1], static_cast<const uint4*>(d.c12_w2), \
                     d.bias[2], P, eps, pm, ps, pn)
  const int pd = hn_knobs().c12w_pd;
  if (!u8 && !abl && pd != 11) {
    switch (pd) {
      case 21: HN_C12W_GO(-1, 0, 2, 1); break;
      case 31: HN_C12W_GO(-1, 0, 3, 1); break;
      case 12: HN_C12W_GO(-1, 0, 1, 2); break;
      case 22: HN_C12W_GO(-1, 0, 2, 2); break;
      case 32: HN_C12W_GO(-1, 0, 3, 2); break;
      case 33: HN_C12W_GO(-1, 0, 3, 3); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (abl) {
#ifdef HN_EXPERIMENTS
    if (u8) return hipErrorInvalidValue;
    switch (abl) {
      case 1: HN_C12W_GO(-1, 1); break;
      case 2: HN_C12W_GO(-1, 2); break;
      case 4: HN_C12W_GO(-1, 4); break;
      case 6: HN_C12W_GO(-1, 6); break;
      case 64: HN_C12W_GO(-1, 64); break;
      case 192: HN_C12W_GO(-1, 192); break;
      default: return hipErrorInvalidValue;
    }
#else
    return hipErrorInvalidValue;
#endif
  } else if (!u8) HN_C12W_GO(-1);
  else if (u8->resize == HN_RESIZE_NONE) HN_C12W_GO(HN_RESIZE_NONE);
  else if (u8->resize == HN_RESIZE_CV2_LINEAR) HN_C12W_GO(HN_RESIZE_CV2_LINEAR);
  else if (u8->resize == HN_RESIZE_PIL_BILINEAR) HN_C12W_GO(HN_RESIZE_PIL_BILINEAR);
  else return hipErrorInvalidValue;
#undef HN_C12W_GO
  return hipGetLastError();
}

#endif  // HN_EXPERIMENTS

hipError_t hn_launch_c12s(const float* in, float* out, const HardnetDev& d, int P, float eps, hipStream_t st,
                          const HnU8In* u8) {
  if (P <= 0) return hipSuccess;
  if (!d.c12_w1w) return hipErrorInvalidValue;
  int resident = 0;
  const hipError_t e = hn_resident_blocks(reinterpret_cast<const void*>(&k_c12s<-1>), 512, 0, &resident);
  if (e != hipSuccess) return e;
  const int grid = (int)std::min<long>((long)P, resident);
  const void* src = u8 ? u8->in : static_cast<const void*>(in);
  const float pm = u8 ? u8->mean : 0.f, ps = u8 ? u8->stdv : 1.f;
  const int pn = u8 ? u8->normalize : 0;
#define HN_C12S_GO(U, ...)                                                                                \
  hipLaunchKernelGGL((k_c12s<U, ##__VA_ARGS__>), dim3(grid), dim3(512), 0, st, src, out, d.stem_w, d.stem_b, \
                     static_cast<const uint4*>(d.c12_w1w), d.bias[1], static_cast<const uint4*>(d.c12_w2),   \
                     d.bias[2], P, eps, pm, ps, pn)
#ifdef HN_EXPERIMENTS
  const int pd = hn_knobs().c12w_pd;
  const int abl = hn_knobs().c12_abl + (hn_knobs().c12w_pd == 21 && hn_knobs().c12_abl == 84 ? 1000 : 0);
  if (abl) {
    if (u8) return hipErrorInvalidValue;
    switch (abl) {
      case 1: HN_C12S_GO(-1, 1, 1, 1, 1); break;
      case 2: HN_C12S_GO(-1, 1, 1, 1, 2); break;
      case 4: HN_C12S_GO(-1, 1, 1, 1, 4); break;
      case 6: HN_C12S_GO(-1, 1, 1, 1, 6); break;
      case 64: HN_C12S_GO(-1, 1, 1, 1, 64); break;
      case 65: HN_C12S_GO(-1, 1, 1, 1, 64, true); break;
      case 66: HN_C12S_GO(-1, 1, 1, 1, 64, false, true); break;
      case 64 + 8: HN_C12S_GO(-1, 1, 1, 1, 64 + 8); break;    // timing: no P3
      case 64 + 16: HN_C12S_GO(-1, 1, 1, 1, 64 + 16); break;  // timing: no P1
      case 64 + 24: HN_C12S_GO(-1, 1, 1, 1, 64 + 24); break;  // timing: neither (P2 alone)
      case 64 + 20: HN_C12S_GO(-1, 1, 1, 1, 64 + 20); break;  // timing: P3 without MFMAs, no P1
      case 64 + 20 + 32: HN_C12S_GO(-1, 1, 1, 1, 64 + 20 + 32); break;  // + P2 without its LDS stream
      case 64 + 20 + 256: HN_C12S_GO(-1, 1, 1, 1, 64 + 20, false, false, true); break;  // 84, interleaved
      case 64 + 20 + 2: HN_C12S_GO(-1, 1, 1, 1, 64 + 20 + 2); break;  // 84 without the conv1 MFMAs
      case 64 + 512: HN_C12S_GO(-1, 1, 1, 1, 64, false, false, true); break;  // stamps, interleaved
      case 64 + 1024: HN_C12S_GO(-1, 1, 1, 1, 64, false, true, true); break;  // stamps, interleaved + P1 in P3
      case 64 + 20 + 1000: HN_C12S_GO(-1, 2, 1, 1, 64 + 20); break;  // the same, P2 two steps ahead
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (!u8 && pd != 11) {
    switch (pd) {
      case 21: HN_C12S_GO(-1, 2, 1); break;
      case 22: HN_C12S_GO(-1, 2, 2); break;
      case 10: HN_C12S_GO(-1, 1, 1, 0); break;  // B-waves at priority 0
      case 1: HN_C12S_GO(-1, 1, 1, 1, 0, true); break;  // P1 on the A-waves
      case 2: HN_C12S_GO(-1, 1, 1, 0, 0, true); break;  // P1 on the A-waves, B-waves at priority 0
      case 3: HN_C12S_GO(-1, 1, 1, 1, 0, false, true); break;  // P1 split around P3 on the B-waves
      case 4: HN_C12S_GO(-1, 1, 1, 0, 0, false, true); break;  // the same, B-waves at priority 0
      case 5: HN_C12S_GO(-1, 1, 1, 1, 0, false, false, true); break;  // interleaved MFMA chains
      case 6: HN_C12S_GO(-1, 1, 1, 1, 0, false, true, true); break;   // + P1 inside P3
      case 7: HN_C12S_GO(-1, 1, 1, 0, 0, false, true, true); break;   // + B-waves at priority 0
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
#endif  // HN_EXPERIMENTS
  if (!u8) HN_C12S_GO(-1);
  else if (u8->resize == HN_RESIZE_NONE) HN_C12S_GO(HN_RESIZE_NONE);
  else if (u8->resize == HN_RESIZE_CV2_LINEAR) HN_C12S_GO(HN_RESIZE_CV2_LINEAR);
  else if (u8->resize == HN_RESIZE_PIL_BILINEAR) HN_C12S_GO(HN_RESIZE_PIL_BILINEAR);
  else return hipErrorInvalidValue;
#undef HN_C12S_GO
  return hipGetLastError();
}
