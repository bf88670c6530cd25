// Fused IRF block (fbnet_builder.py:455-570) for the searched layers 1..5 (SEARCH_SPACE2,
// lookup_table_builder.py:22-45; resolutions 16x16 .. 4x4):
//
//   y = pwl(dw(shuffle(pw(x)))) [+ x]        (SE, when present, runs after as k_se)
//
// in one kernel, so the MID-channel intermediates (pw output, dw output) never reach HBM:
// the block reads x once and writes y once (the residual comes from the x operands already
// in registers).
//
// Persistent workgroups (4 waves) walk a contiguous range of tiles of NI = 256 input pixels
// (NPB whole patches: 1 at 16x16, 4 at 8x8, 16 -- or 8 when CIN = 128 -- at 4x4), prefetching
// the next tile's input into registers.  Per 32-channel chunk of MID:
//   pw  : 1x1 conv as 32x32 fp16x3 MFMA tiles (weights = A, BN folded, ChannelShuffle folded
//         into the row order, groups densified).  B operands (x, split into fp16 hi/lo) are
//         loaded once per tile and stay in registers across chunks.  bias+ReLU -> LDS (fp32).
//   dw  : kxk depthwise conv (stride S, pad k/2, BN, ReLU) on the VALU from LDS, fp32, each
//         thread sliding a register window along a run of R output pixels of one row for 4
//         channels; result -> LDS (fp32).
//   pwl : 1x1 conv (BN, no ReLU) as fp16x3 MFMA tiles accumulating over the chunks in
//         registers (+ the residual as identity-weight K-steps); bias, float4 stores.
#include "hn_common.h"
#include "hn_internal.h"

#include <algorithm>

namespace {

constexpr int PS = 36;  // floats per pixel in the LDS tiles (32 channels + 4 pad)

// 256 input pixels per tile; 128 for the 128-channel blocks and the 64-channel e1 blocks (the
// wang2 / wang4 irf2 pair at 8x8: three workgroups per CU in 40 KB, 156-166 VGPRs; same-box A/B
// irf2 -1.2 / -2.7 %).  The 64-channel e3 / e4 blocks keep 256 (FDLNet's irf +4 % at 128: half the
// weight reuse of their 192 / 256-channel 1x1 operands).
template <int CIN, int HIN, int MID>
struct IrfTile {
  static constexpr int NPB = (CIN == 128 || (CIN == 64 && MID == 64)) ? 128 / (HIN * HIN) : 256 / (HIN * HIN);
  static constexpr int NI = NPB * HIN * HIN;  // input pixels per workgroup
};

template <int CIN, int COUT, int HIN, int S, int K, int MID>
struct IrfShape {
  static constexpr int HOUT = HIN / S, PAD = K / 2;
  static constexpr int NPB = IrfTile<CIN, HIN, MID>::NPB, NI = IrfTile<CIN, HIN, MID>::NI;
  static constexpr int NO = NPB * HOUT * HOUT;           // output pixels per workgroup
  static constexpr int TI = NI / 32 / 4;                 // pw pixel tiles per wave
  static constexpr int KS = CIN / 16;                    // pw K-steps
  static constexpr int NOT = NO / 32, NCT = COUT / 32;   // pwl pixel tiles, cout tiles
  static constexpr int TW = NOT * NCT / 4;               // pwl tiles per wave
  static constexpr int R = S == 1 ? 4 : 2;               // dw run length (output pixels per thread)
  static constexpr int RUNS = NO / R;                    // runs per chunk (x 8 channel quads)
  static constexpr int WIN = (R - 1) * S + K;            // input columns of a run window
  static constexpr bool RES = S == 1 && CIN == COUT;
  static_assert(NI % 128 == 0 && NO % 32 == 0 && (NOT * NCT) % 4 == 0, "tile shape");
  static_assert(HOUT % R == 0, "dw run must stay in one row");
  static constexpr int LDS_PW = NI * PS, LDS_DW = NO * PS, LDS_W = K * K * 32 + 32;  // floats
};

// The block's work on one tile once its pw B operands (x split into fp16 hi / lo, pixel tiles
// 4i + w of the tile, lane: pixel, 8 channels) are in registers: per 32-channel chunk of MID the
// pw (fp16x3 MFMA, bias + ReLU -> LDS), the dw (VALU, register window), the pwl accumulated in
// registers; then the residual as identity-weight K-steps.  Leaves the pwl output (bias included)
// in acc[i] = 32 x 32 tile (pixel tile (4i + w) % NOT, channel tile (4i + w) / NOT); lane (px, h):
// acc[4q + r] = channel 8q + 4h + r of pixel px.  Ends with a barrier (s_pw / s_dw free).
// MODE (k_irf2's three-workgroups-per-CU form, 53 KB of LDS): IRF_WPAD keeps the dw weights in the
// 16-byte pad slot of each s_pw pixel (float4 i at pixel i) instead of s_w; IRF_BAND (+ WPAD, the
// stride-1 256-pixel tile) runs the dw in two bands of 8 output rows through a 16 KB band buffer
// s_dw (128 pixels x 32 floats, 16-byte chunk c of band pixel p at c ^ band_sw(p): the pwl operand
// reads and the dw stores both conflict-free, tests/test_lds_banks.py) with the pwl of each band
// right after it -- the thread's two dw items are exactly the two bands, and wave w's pwl tile of
// band b is its acc[b].
constexpr int IRF_PLAIN = 0, IRF_WPAD = 1, IRF_BAND = 2;
HN_DEV int band_sw(int p) { return ((p >> 1) & 1) | (((p >> 4) & 1) << 1) | (((p >> 2) & 1) << 2); }

template <int CIN, int COUT, int HIN, int S, int K, int MID, int MODE = IRF_PLAIN>
HN_DEV void irf_core(const uint4 (&bh)[IrfShape<CIN, COUT, HIN, S, K, MID>::TI][CIN / 16],
                     const uint4 (&bl)[IrfShape<CIN, COUT, HIN, S, K, MID>::TI][CIN / 16],
                     f32x16 (&acc)[IrfShape<CIN, COUT, HIN, S, K, MID>::TW], const uint4* __restrict__ pw_a,
                     const float* __restrict__ pw_b, const float* __restrict__ dw_w, const float* __restrict__ dw_b,
                     const uint4* __restrict__ pwl_a, const float* __restrict__ pwl_b, float* s_pw, float* s_dw,
                     float* s_w) {
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  constexpr int HOUT = Sh::HOUT, PAD = Sh::PAD, TI = Sh::TI, KS = Sh::KS, NOT = Sh::NOT, TW = Sh::TW, R = Sh::R,
                RUNS = Sh::RUNS, WIN = Sh::WIN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int px = lane & 31, h = lane >> 5;
  constexpr bool WPAD = MODE != IRF_PLAIN, BAND = MODE == IRF_BAND;
  static_assert(!WPAD || Sh::NI >= K * K * 8 + 8, "a pad slot per weight float4");
  static_assert(!BAND || (S == 1 && Sh::NO == 256 && HOUT == 16 && TW == 2 && Sh::NCT == 1),
                "the band form is the 16x16 stride-1 32 -> 32 block");
  // dw weight / bias float4 i (i < K*K*8: tap i / 8, channel quad i % 8; then the bias quads)
  auto wslot = [&](int i) -> float* { return WPAD ? s_pw + i * PS + 32 : s_w + 4 * i; };
  // pwl accumulators start at the pwl bias, so the epilogue is stores only
#pragma unroll
  for (int i = 0; i < TW; ++i) {
    const int ct = (4 * i + w) / NOT;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(pwl_b + 32 * ct + 8 * q + 4 * h);
      acc[i][4 * q] = b.x; acc[i][4 * q + 1] = b.y; acc[i][4 * q + 2] = b.z; acc[i][4 * q + 3] = b.w;
    }
  }
#pragma unroll 1
  for (int m = 0; m < MID / 32; ++m) {
    // dw weights + bias of the chunk (float4 t of K*K*8 + 8).  RING (the 64- and 128-channel blocks,
    // KS >= 4): loaded with the pw's first operands and stored to LDS after the pw, so their L2 round
    // trip hides behind the pw MFMAs (the clamped index keeps the load unconditional); the 32-channel
    // blocks keep the up-front store (same-box A/B: the RING form cost wang3's irf 2.42 -> 2.59 ms)
    static_assert(K * K * 8 + 8 <= 256, "one dw weight float4 per thread");
    constexpr int NWQ = K * K * 8 + 8;
    constexpr bool RING = KS >= 4;
    const int iw = t < NWQ ? t : NWQ - 1;
    const float* const wsrc =
        iw < K * K * 8 ? dw_w + (iw >> 3) * MID + 32 * m + 4 * (iw & 7) : dw_b + 32 * m + 4 * (iw - K * K * 8);
    float4 wv;
    if constexpr (!RING)
      if (t < NWQ) *reinterpret_cast<float4*>(wslot(t)) = *reinterpret_cast<const float4*>(wsrc);
    // ---- pw --------------------------------------------------------------------------
    {
      f32x16 bias;  // pw bias as the initial accumulator (epilogue: ReLU only)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(pw_b + 32 * m + 8 * q + 4 * h);
        bias[4 * q] = b.x; bias[4 * q + 1] = b.y; bias[4 * q + 2] = b.z; bias[4 * q + 3] = b.w;
      }
      f32x16 c[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) c[i] = bias;
      auto pw_frag = [&](int s, uint4 (&d)[2]) {
        const uint4* ap = pw_a + ((size_t)(m * KS + s) * 2) * 64 + lane;
        d[0] = ap[0];
        d[1] = ap[64];
      };
      if constexpr (RING) {
        // the weight fragments one K-step ahead (ring of two): left to itself the scheduler reused one
        // register pair for every K-step of the 64-channel blocks, i.e. load -> vmcnt(0) -> MFMA, one L2
        // round trip per K-step (same-box A/B: wang2 irf2 9.26 -> 8.40 ms)
        uint4 fa[2][2];
        pw_frag(0, fa[0]);
        wv = *reinterpret_cast<const float4*>(wsrc);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (s + 1 < KS) pw_frag(s + 1, fa[(s + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
          const f16x8 ah = as_f16x8(fa[s & 1][0]), al = as_f16x8(fa[s & 1][1]);
#pragma unroll
          for (int i = 0; i < TI; ++i) c[i] = mfma3_f16(ah, al, as_f16x8(bh[i][s]), as_f16x8(bl[i][s]), c[i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          uint4 f[2];
          pw_frag(s, f);
          const f16x8 ah = as_f16x8(f[0]), al = as_f16x8(f[1]);
#pragma unroll
          for (int i = 0; i < TI; ++i) c[i] = mfma3_f16(ah, al, as_f16x8(bh[i][s]), as_f16x8(bl[i][s]), c[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        float4* d = reinterpret_cast<float4*>(s_pw + ((4 * i + w) * 32 + px) * PS);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          d[2 * q + h] = make_float4(relu0(c[i][4 * q]), relu0(c[i][4 * q + 1]),
                                     relu0(c[i][4 * q + 2]), relu0(c[i][4 * q + 3]));
      }
    }
    if constexpr (RING)
      if (t < NWQ) *reinterpret_cast<float4*>(wslot(t)) = wv;
    __syncthreads();
    // ---- dw: thread item = (run of R output pixels in one row, channel quad q) -----------
    // (BAND: item k of the thread is band k, computed and consumed by the pwl in turn)
    auto dw_item = [&](int it) {
      // lane -> (run, channel quad): each 16-lane ds_read_b128 group holds 4 runs x 4 quads,
      // whose window reads land in 16 distinct bank slots (slot = 4 run + q + 9 dx mod 16)
      const int q = (lane & 3) | ((lane >> 5) << 2), run = (it >> 6) * 8 + ((lane >> 2) & 7);
      const int o0 = run * R;  // first output pixel (tile-local)
      const int pl = o0 / (HOUT * HOUT), oy = (o0 / HOUT) % HOUT, ox0 = o0 % HOUT;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(wslot(K * K * 8 + q));
      f32x4 o[R];
#pragma unroll
      for (int r = 0; r < R; ++r) o[r] = b4;
      const int ix0 = ox0 * S - PAD;
#pragma unroll 1
      for (int dy = 0; dy < K; ++dy) {
        const int iy = oy * S + dy - PAD;
        if (iy < 0 || iy >= HIN) continue;
        const float* rowp = s_pw + ((pl * HIN + iy) * HIN) * PS + 4 * q;
        f32x4 win[WIN];
#pragma unroll
        for (int c = 0; c < WIN; ++c) {
          const int ix = ix0 + c;
          win[c] = (ix >= 0 && ix < HIN) ? *reinterpret_cast<const f32x4*>(rowp + ix * PS) : f32x4{};
        }
#pragma unroll
        for (int dx = 0; dx < K; ++dx) {
          const f32x4 wv = *reinterpret_cast<const f32x4*>(wslot((dy * K + dx) * 8 + q));
#pragma unroll
          for (int r = 0; r < R; ++r) o[r] = __builtin_elementwise_fma(wv, win[r * S + dx], o[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const f32x4 v = relu4(o[r]);
        if constexpr (BAND) {
          const int p = (o0 + r) & 127;  // band pixel
          *reinterpret_cast<f32x4*>(s_dw + p * 32 + 4 * (q ^ band_sw(p))) = v;
        } else {
          *reinterpret_cast<f32x4*>(s_dw + (o0 + r) * PS + 4 * q) = v;
        }
      }
    };
    // ---- pwl (accumulate this chunk's 32 mid channels = 2 K-steps) into acc[i] -------------
    auto pwl_tile = [&](int i) {
      const int tile = 4 * i + w, pt = tile % NOT, ct = tile / NOT;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float4 v0, v1;
        if constexpr (BAND) {
          const int p = (pt & 3) * 32 + px, c = 4 * s + 2 * h;
          v0 = *reinterpret_cast<const float4*>(s_dw + p * 32 + 4 * (c ^ band_sw(p)));
          v1 = *reinterpret_cast<const float4*>(s_dw + p * 32 + 4 * ((c + 1) ^ band_sw(p)));
        } else {
          const float4* src = reinterpret_cast<const float4*>(s_dw + (pt * 32 + px) * PS + 16 * s + 8 * h);
          v0 = src[0];
          v1 = src[1];
        }
        uint4 xh, xl;
        split8_f16(v0, v1, xh, xl);
        const uint4* ap = pwl_a + ((size_t)(ct * (MID / 16) + 2 * m + s) * 2) * 64 + lane;
        acc[i] = mfma3_f16(as_f16x8(ap[0]), as_f16x8(ap[64]), as_f16x8(xh), as_f16x8(xl), acc[i]);
      }
    };
    if constexpr (BAND) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        dw_item(t + 256 * b);
        __syncthreads();
        pwl_tile(b);
        if (b == 0) __syncthreads();  // band 1 rewrites the band buffer
      }
    } else {
#pragma unroll 1
      for (int it = t; it < RUNS * 8; it += 256) dw_item(it);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TW; ++i) pwl_tile(i);
    }
    __syncthreads();  // s_pw / s_dw / s_w are rewritten by the next chunk
  }

  // ---- residual: y += x as two more MFMA K-steps per tile with an identity A operand
  // against the x B operands already in registers (x = hi + lo to ~2^-22; no second read of
  // x from HBM).  With S = 1, NI = NO, so the wave's pwl pixel tiles are its pw tiles.
  if constexpr (Sh::RES) {
#pragma unroll
    for (int i = 0; i < TW; ++i) {
      constexpr int TPW = NOT / 4;  // pixel tiles per wave (= TI)
      const int ii = i % TPW, ct = i / TPW;
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        f16x8 id;
#pragma unroll
        for (int j = 0; j < 8; ++j) id[j] = (_Float16)((px == 16 * sl + 8 * h + j) ? 1.f : 0.f);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(id, as_f16x8(bl[ii][2 * ct + sl]), acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(id, as_f16x8(bh[ii][2 * ct + sl]), acc[i], 0, 0, 0);
      }
    }
  }
}

// pwl output tiles -> y in HBM: each 32-pixel x 32-channel tile goes through a per-wave scratch in
// s_pw (free after the core's last barrier), so that every float4 store instruction writes 8 whole
// 128-byte pixel rows instead of 32 pixels x 32 bytes.  Ends with a barrier.
template <int CIN, int COUT, int HIN, int S, int K, int MID>
HN_DEV void irf_store(const f32x16 (&acc)[IrfShape<CIN, COUT, HIN, S, K, MID>::TW], float* __restrict__ y, long p0,
                      int npv, float* s_pw) {
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  constexpr int HOUT = Sh::HOUT, NOT = Sh::NOT, TW = Sh::TW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, px = lane & 31, h = lane >> 5;
  float* scr = s_pw + w * 32 * PS;
  static_assert(Sh::NI * PS >= 4 * 32 * PS, "scratch fits in s_pw");
#pragma unroll
  for (int i = 0; i < TW; ++i) {
    const int tile = 4 * i + w, pt = tile % NOT, ct = tile / NOT;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(scr + px * PS + 8 * q + 4 * h) =
          make_float4(acc[i][4 * q], acc[i][4 * q + 1], acc[i][4 * q + 2], acc[i][4 * q + 3]);
    __builtin_amdgcn_wave_barrier();  // (one wave: its LDS accesses execute in order)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pl = 8 * k + (lane >> 3), c4 = lane & 7, o = pt * 32 + pl;
      if (o < npv * HOUT * HOUT)
        *reinterpret_cast<float4*>(y + (p0 * (HOUT * HOUT) + o) * COUT + 32 * ct + 4 * c4) =
            *reinterpret_cast<const float4*>(scr + pl * PS + 4 * c4);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  __syncthreads();  // the scratch (s_pw) is rewritten by the next tile's pw
}

// The block's input tile from HBM into registers (pixel tiles 4i + w, 8 channels per lane), zero
// past the batch's last patch
template <int CIN, int COUT, int HIN, int S, int K, int MID>
HN_DEV void irf_load(float4* pa, float4* pb, const float* __restrict__ x, long tile, int P) {  // [TI][KS]
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, px = lane & 31, h = lane >> 5;
  const long q0 = tile * Sh::NPB;
  const int nv = (int)min<long>(Sh::NPB, P - q0);
#pragma unroll
  for (int i = 0; i < Sh::TI; ++i) {
    const int p = (4 * i + w) * 32 + px;
    const bool ok = p < nv * HIN * HIN;
#pragma unroll
    for (int s = 0; s < Sh::KS; ++s) {
      pa[i * Sh::KS + s] = pb[i * Sh::KS + s] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok) {
        const float4* src = reinterpret_cast<const float4*>(x + (q0 * (HIN * HIN) + p) * CIN + 16 * s + 8 * h);
        pa[i * Sh::KS + s] = src[0];
        pb[i * Sh::KS + s] = src[1];
      }
    }
  }
}

// The block's shared memory: pw rows, dw outputs, dw weights (one array, carved)
template <int CIN, int COUT, int HIN, int S, int K, int MID>
constexpr int irf_lds_floats() {
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  return Sh::LDS_PW + Sh::LDS_DW + Sh::LDS_W;
}

// The 64 -> 128 stride-2 and the 128-channel (4x4) blocks are held to 168 VGPRs, three
// workgroups per CU (their LDS allows three; the k5 forms spill 20-25 dwords and still gain):
// wang2 / wang4 / FDLNet irf -1 to -2 %.  The CIN = 32 blocks (16x16) run three workgroups per CU
// too, in <= 53 KB of LDS: the stride-1 ones in the band form (IRF_BAND), the stride-2 ones with the
// dw weights in the s_pw pad slots (IRF_WPAD); every block is one tile per workgroup (the round-2
// persistent register prefetch of the next tile is gone: see k_irf2).
template <int CIN, int S>
constexpr int irf_mode() { return CIN == 32 ? (S == 1 ? IRF_BAND : IRF_WPAD) : IRF_PLAIN; }
template <int CIN, int COUT, int HIN, int S, int K, int MID>
constexpr int irf_smem_floats() {
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  constexpr int M = irf_mode<CIN, S>();
  return M == IRF_BAND ? Sh::LDS_PW + 128 * 32 : M == IRF_WPAD ? Sh::LDS_PW + Sh::LDS_DW : irf_lds_floats<CIN, COUT, HIN, S, K, MID>();
}

template <int CIN, int COUT, int HIN, int S, int K, int MID>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CIN == 64 && S == 1 && MID != 64 ? 1 : 3))) void k_irf(const float* __restrict__ x, float* __restrict__ y,
                                             const uint4* __restrict__ pw_a,   // [MID/32][CIN/16][2][64]
                                             const float* __restrict__ pw_b,   // [MID] dw order
                                             const float* __restrict__ dw_w,   // [K*K][MID]
                                             const float* __restrict__ dw_b,   // [MID]
                                             const uint4* __restrict__ pwl_a,  // [COUT/32][MID/16][2][64]
                                             const float* __restrict__ pwl_b,  // [COUT]
                                             int P) {
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  constexpr int NPB = Sh::NPB, TI = Sh::TI, KS = Sh::KS, TW = Sh::TW, MODE = irf_mode<CIN, S>();
  constexpr int SMEM = irf_smem_floats<CIN, COUT, HIN, S, K, MID>();
  static_assert((CIN == 64 && S == 1 && MID != 64) || 3 * SMEM * 4 <= 160 * 1024, "three workgroups per CU");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float* s_pw = smem;
  float* s_dw = smem + Sh::LDS_PW;
  float* s_w = s_dw + Sh::LDS_DW;  // (IRF_PLAIN only)
  const int tile = (int)blockIdx.x;  // one tile per workgroup
  if (tile * NPB >= P) return;       // workgroup-uniform
  float4 pa[TI][KS], pb[TI][KS];
  irf_load<CIN, COUT, HIN, S, K, MID>(&pa[0][0], &pb[0][0], x, tile, P);
  const long p0 = (long)tile * NPB;  // first patch of the tile
  const int npv = (int)min<long>(NPB, P - p0);
  uint4 bh[TI][KS], bl[TI][KS];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int s = 0; s < KS; ++s) split8_f16(pa[i][s], pb[i][s], bh[i][s], bl[i][s]);
  f32x16 acc[TW];
  irf_core<CIN, COUT, HIN, S, K, MID, MODE>(bh, bl, acc, pw_a, pw_b, dw_w, dw_b, pwl_a, pwl_b, s_pw, s_dw, s_w);
  irf_store<CIN, COUT, HIN, S, K, MID>(acc, y, p0, npv, s_pw);
}

// Two consecutive blocks on the same tile (A at stride 1, so its output tile is B's input tile:
// SEARCH_SPACE2 layers 1 -> 2 at 16x16 and 3 -> 4 at 8x8): A's pwl output goes to LDS (over A's
// then free pw / dw buffers) instead of HBM, B's pw B operands are read back from there -- the
// A -> B activation (32 / 16 KB per patch each way) never reaches HBM.
// CA = 32 (the 16x16 pair): three workgroups per CU in 53 KB of LDS -- A's dw in two bands
// through a 16 KB buffer and both blocks' dw weights in the s_pw pad slots (IRF_BAND / IRF_WPAD) --
// at <= 168 VGPRs; CA = 64: two workgroups per CU, the plain layout.
template <int CA>
constexpr int irf2_mode_a() { return CA == 32 ? IRF_BAND : IRF_PLAIN; }
template <int CA>
constexpr int irf2_mode_b() { return CA == 32 ? IRF_WPAD : IRF_PLAIN; }

template <int CA, int HI, int KA, int MA, int CB, int KB, int MB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_irf2(
    const float* __restrict__ x, float* __restrict__ y, HnIrfArgs A, HnIrfArgs Bk, int P) {
  using SA = IrfShape<CA, CA, HI, 1, KA, MA>;
  using SB = IrfShape<CA, CB, HI, 2, KB, MB>;
  static_assert(SA::NPB == SB::NPB && SA::NO == SB::NI, "A's output tile is B's input tile");
  constexpr int NPB = SA::NPB, XS = CA + 4;  // A -> B tile in LDS: [pixel][CA + 4 floats]
  constexpr int MA_ = irf2_mode_a<CA>(), MB_ = irf2_mode_b<CA>();
  constexpr int LA = MA_ == IRF_BAND ? SA::LDS_PW + 128 * 32 : irf_lds_floats<CA, CA, HI, 1, KA, MA>();
  constexpr int LB = MB_ == IRF_WPAD ? SB::LDS_PW + SB::LDS_DW : irf_lds_floats<CA, CB, HI, 2, KB, MB>();
  constexpr int LX = SA::NO * XS;
  constexpr int LDS = LA > LB ? (LA > LX ? LA : LX) : (LB > LX ? LB : LX);
  static_assert(3 * LDS * 4 <= 160 * 1024, "three workgroups per CU");
  __shared__ __attribute__((aligned(16))) float smem[LDS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, px = lane & 31, h = lane >> 5;
  // one tile per workgroup (not persistent, no register prefetch of the next tile: the other
  // workgroups on the CU hide the load; the 32 freed registers measured -5 % irf2 time on wang2,
  // 10.03 -> 9.53 ms, same box)
  const int tile = (int)blockIdx.x;
  if (tile * NPB >= P) return;  // workgroup-uniform
  float4 pa[SA::TI][SA::KS], pb[SA::TI][SA::KS];
  {
    irf_load<CA, CA, HI, 1, KA, MA>(&pa[0][0], &pb[0][0], x, tile, P);
    const long p0 = (long)tile * NPB;
    const int npv = (int)min<long>(NPB, P - p0);
    {
      uint4 bh[SA::TI][SA::KS], bl[SA::TI][SA::KS];
#pragma unroll
      for (int i = 0; i < SA::TI; ++i)
#pragma unroll
        for (int s = 0; s < SA::KS; ++s) split8_f16(pa[i][s], pb[i][s], bh[i][s], bl[i][s]);
      f32x16 acc[SA::TW];
      irf_core<CA, CA, HI, 1, KA, MA, MA_>(bh, bl, acc, A.pw_a, A.pw_b, A.dw_w, A.dw_b, A.pwl_a, A.pwl_b, smem,
                                           smem + SA::LDS_PW, smem + SA::LDS_PW + SA::LDS_DW);
      // A's output tile -> LDS [pixel][XS] (lane (px, h): channels 8q + 4h .. + 3 of pixel px)
#pragma unroll
      for (int i = 0; i < SA::TW; ++i) {
        const int tl = 4 * i + w, pt = tl % SA::NOT, ct = tl / SA::NOT;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<float4*>(smem + (pt * 32 + px) * XS + 32 * ct + 8 * q + 4 * h) =
              make_float4(acc[i][4 * q], acc[i][4 * q + 1], acc[i][4 * q + 2], acc[i][4 * q + 3]);
      }
    }
    __syncthreads();
    // B's pw B operands from the LDS tile (pixel tiles 4i + w, 8 channels per lane), then B
    uint4 bh[SB::TI][SB::KS], bl[SB::TI][SB::KS];
#pragma unroll
    for (int i = 0; i < SB::TI; ++i)
#pragma unroll
      for (int s = 0; s < SB::KS; ++s) {
        const float4* src = reinterpret_cast<const float4*>(smem + ((4 * i + w) * 32 + px) * XS + 16 * s + 8 * h);
        split8_f16(src[0], src[1], bh[i][s], bl[i][s]);
      }
    __syncthreads();  // the tile's LDS is B's pw / dw buffers from here
    f32x16 acc[SB::TW];
    irf_core<CA, CB, HI, 2, KB, MB, MB_>(bh, bl, acc, Bk.pw_a, Bk.pw_b, Bk.dw_w, Bk.dw_b, Bk.pwl_a, Bk.pwl_b, smem,
                                    smem + SB::LDS_PW, smem + SB::LDS_PW + SB::LDS_DW);
    irf_store<CA, CB, HI, 2, KB, MB>(acc, y, p0, npv, smem);
  }
}

#ifdef HN_EXPERIMENTS
// (experiments library, HN_IRF3=1: measured slower -- wang4 irf2 + irf 5.09 -> irf3 5.68 ms per step)
// Three consecutive blocks on one tile: k_irf2's 8x8 pair (A: 64 -> 64 stride 1, B: 64 -> 128 stride 2;
// SEARCH_SPACE2 layers 3 -> 4) and C, the 4x4 stride-1 128 -> 128 e1 block after it (layer 5), on B's output
// tile -- 2 patches = 32 pixels x 128 channels -- so the B -> C activation (8 KB per patch each way) never
// reaches HBM and C costs no launch of its own.  C's tile is
// a single 32-pixel MFMA tile, so its work is split by channel chunk instead of by pixel tile: wave w runs
// C's pw for mid chunk w (all CB / 16 K-steps, its B operands split from an LDS copy of B's output), that
// chunk's depthwise conv (RUNS x 8 = 64 items: one per lane), and -- after a workgroup barrier -- the pwl for
// output-channel tile w over the MID chunks in irf_core's order, then the residual as identity-weight
// K-steps.  Every C output is the same products added in the same order as k_irf's: bit-identical.
template <int CA, int HI, int KA, int MA, int CB, int KB, int MB, int KC, int MC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_irf3(
    const float* __restrict__ x, float* __restrict__ y, HnIrfArgs A, HnIrfArgs Bk, HnIrfArgs Cc, int P) {
  using SA = IrfShape<CA, CA, HI, 1, KA, MA>;
  using SB = IrfShape<CA, CB, HI, 2, KB, MB>;
  constexpr int HC = HI / 2, NC = SB::NO;      // C's resolution and its tile's pixels
  constexpr int KSC = CB / 16, NCH = MC / 32;  // C's pw K-steps and mid chunks
  static_assert(SA::NPB == SB::NPB && SA::NO == SB::NI, "A's output tile is B's input tile");
  static_assert(NC == 32 && SB::TW == 1 && SB::NCT == 4 && NCH == 4, "C: one pixel tile, one mid chunk per wave");
  static_assert(irf2_mode_a<CA>() == IRF_PLAIN && irf2_mode_b<CA>() == IRF_PLAIN, "the 64-channel pair");
  constexpr int NPB = SA::NPB, XS = CA + 4, XC = CB + 4;
  constexpr int CW = KC * KC * 8 + 8;          // C's dw weight + bias float4s per chunk
  constexpr int LA = irf_lds_floats<CA, CA, HI, 1, KA, MA>(), LB = irf_lds_floats<CA, CB, HI, 2, KB, MB>();
  constexpr int LX = SA::NO * XS, LCX = NC * XC;
  constexpr int C_PW = 0, C_W = NCH * NC * PS, C_DW = C_W + NCH * CW * 4, LC = C_DW + NCH * NC * PS;
  constexpr int L1 = LA > LB ? LA : LB, L2 = LX > LCX ? LX : LCX, L3 = L1 > L2 ? L1 : L2;
  constexpr int LDS = L3 > LC ? L3 : LC;
  static_assert(3 * LDS * 4 <= 160 * 1024, "three workgroups per CU");
  __shared__ __attribute__((aligned(16))) float smem[LDS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, px = lane & 31, h = lane >> 5;
  const int tile = (int)blockIdx.x;
  if (tile * NPB >= P) return;  // workgroup-uniform
  const long p0 = (long)tile * NPB;
  const int npv = (int)min<long>(NPB, P - p0);
  f32x16 accb[1];
  {
    float4 pa[SA::TI][SA::KS], pb[SA::TI][SA::KS];
    irf_load<CA, CA, HI, 1, KA, MA>(&pa[0][0], &pb[0][0], x, tile, P);
    {
      uint4 bh[SA::TI][SA::KS], bl[SA::TI][SA::KS];
#pragma unroll
      for (int i = 0; i < SA::TI; ++i)
#pragma unroll
        for (int s = 0; s < SA::KS; ++s) split8_f16(pa[i][s], pb[i][s], bh[i][s], bl[i][s]);
      f32x16 acc[SA::TW];
      irf_core<CA, CA, HI, 1, KA, MA, IRF_PLAIN>(bh, bl, acc, A.pw_a, A.pw_b, A.dw_w, A.dw_b, A.pwl_a, A.pwl_b, smem,
                                                 smem + SA::LDS_PW, smem + SA::LDS_PW + SA::LDS_DW);
#pragma unroll
      for (int i = 0; i < SA::TW; ++i) {
        const int tl = 4 * i + w, pt = tl % SA::NOT, ct = tl / SA::NOT;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<float4*>(smem + (pt * 32 + px) * XS + 32 * ct + 8 * q + 4 * h) =
              make_float4(acc[i][4 * q], acc[i][4 * q + 1], acc[i][4 * q + 2], acc[i][4 * q + 3]);
      }
    }
    __syncthreads();
    uint4 bh[SB::TI][SB::KS], bl[SB::TI][SB::KS];
#pragma unroll
    for (int i = 0; i < SB::TI; ++i)
#pragma unroll
      for (int s = 0; s < SB::KS; ++s) {
        const float4* src = reinterpret_cast<const float4*>(smem + ((4 * i + w) * 32 + px) * XS + 16 * s + 8 * h);
        split8_f16(src[0], src[1], bh[i][s], bl[i][s]);
      }
    __syncthreads();
    irf_core<CA, CB, HI, 2, KB, MB, IRF_PLAIN>(bh, bl, accb, Bk.pw_a, Bk.pw_b, Bk.dw_w, Bk.dw_b, Bk.pwl_a, Bk.pwl_b,
                                               smem, smem + SB::LDS_PW, smem + SB::LDS_PW + SB::LDS_DW);
  }
  // B's output (wave w: pixels 0..31, channels 32 w ..) -> LDS [pixel][XC]; C's pw B operands from it
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(smem + px * XC + 32 * w + 8 * q + 4 * h) =
        make_float4(accb[0][4 * q], accb[0][4 * q + 1], accb[0][4 * q + 2], accb[0][4 * q + 3]);
  __syncthreads();
  uint4 ch[KSC], cl[KSC];
#pragma unroll
  for (int s = 0; s < KSC; ++s) {
    const float4* src = reinterpret_cast<const float4*>(smem + px * XC + 16 * s + 8 * h);
    split8_f16(src[0], src[1], ch[s], cl[s]);
  }
  __syncthreads();  // the region is C's pw / dw buffers from here
  // ---- C: pw of mid chunk m = w (bias + ReLU) -> this wave's [32 pixels][PS] ------------------
  const int m = w;
  float* s_pwc = smem + C_PW + w * NC * PS;
  float* s_wc = smem + C_W + w * CW * 4;
  float* s_dwa = smem + C_DW;
  for (int i = lane; i < CW; i += 64) {
    const float* src = i < KC * KC * 8 ? Cc.dw_w + (i >> 3) * MC + 32 * m + 4 * (i & 7)
                                       : Cc.dw_b + 32 * m + 4 * (i - KC * KC * 8);
    *reinterpret_cast<float4*>(s_wc + 4 * i) = *reinterpret_cast<const float4*>(src);
  }
  {
    f32x16 c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(Cc.pw_b + 32 * m + 8 * q + 4 * h);
      c[4 * q] = b.x; c[4 * q + 1] = b.y; c[4 * q + 2] = b.z; c[4 * q + 3] = b.w;
    }
#pragma unroll
    for (int s = 0; s < KSC; ++s) {
      const uint4* ap = Cc.pw_a + ((size_t)(m * KSC + s) * 2) * 64 + lane;
      c = mfma3_f16(as_f16x8(ap[0]), as_f16x8(ap[64]), as_f16x8(ch[s]), as_f16x8(cl[s]), c);
    }
    float4* d = reinterpret_cast<float4*>(s_pwc + px * PS);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d[2 * q + h] = make_float4(relu0(c[4 * q]), relu0(c[4 * q + 1]), relu0(c[4 * q + 2]), relu0(c[4 * q + 3]));
  }
  __builtin_amdgcn_wave_barrier();  // (one wave: its LDS accesses execute in order)
  asm volatile("" ::: "memory");
  // ---- C: depthwise KC x KC (stride 1, pad KC / 2, BN, ReLU) of chunk m: lane = (4-pixel row run, quad) -----
  {
    constexpr int R = 4, PAD = KC / 2, WIN = R - 1 + KC;
    static_assert(HC == R && NC / R * 8 == 64, "one run (a whole row) per lane");
    const int q = (lane & 3) | ((lane >> 5) << 2), run = (lane >> 2) & 7;
    const int o0 = run * R, pl = o0 / (HC * HC), oy = (o0 / HC) % HC;
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(s_wc + 4 * (KC * KC * 8 + q));
    f32x4 o[R];
#pragma unroll
    for (int r = 0; r < R; ++r) o[r] = b4;
#pragma unroll 1
    for (int dy = 0; dy < KC; ++dy) {
      const int iy = oy + dy - PAD;
      if (iy < 0 || iy >= HC) continue;
      const float* rowp = s_pwc + ((pl * HC + iy) * HC) * PS + 4 * q;
      f32x4 win[WIN];
#pragma unroll
      for (int c = 0; c < WIN; ++c) {
        const int ix = c - PAD;
        win[c] = (ix >= 0 && ix < HC) ? *reinterpret_cast<const f32x4*>(rowp + ix * PS) : f32x4{};
      }
#pragma unroll
      for (int dx = 0; dx < KC; ++dx) {
        const f32x4 wv = *reinterpret_cast<const f32x4*>(s_wc + 4 * ((dy * KC + dx) * 8 + q));
#pragma unroll
        for (int r = 0; r < R; ++r) o[r] = __builtin_elementwise_fma(wv, win[r + dx], o[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      *reinterpret_cast<f32x4*>(s_dwa + (m * NC + o0 + r) * PS + 4 * q) = relu4(o[r]);
  }
  __syncthreads();
  // ---- C: pwl (output-channel tile ct = w over the MID chunks, irf_core's order) + residual ---------------
  const int ct = w;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b = *reinterpret_cast<const float4*>(Cc.pwl_b + 32 * ct + 8 * q + 4 * h);
    acc[4 * q] = b.x; acc[4 * q + 1] = b.y; acc[4 * q + 2] = b.z; acc[4 * q + 3] = b.w;
  }
#pragma unroll
  for (int mm = 0; mm < NCH; ++mm)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float4* src = reinterpret_cast<const float4*>(s_dwa + (mm * NC + px) * PS + 16 * s + 8 * h);
      uint4 xh, xl;
      split8_f16(src[0], src[1], xh, xl);
      const uint4* ap = Cc.pwl_a + ((size_t)(ct * (MC / 16) + 2 * mm + s) * 2) * 64 + lane;
      acc = mfma3_f16(as_f16x8(ap[0]), as_f16x8(ap[64]), as_f16x8(xh), as_f16x8(xl), acc);
    }
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    f16x8 id;
#pragma unroll
    for (int j = 0; j < 8; ++j) id[j] = (_Float16)((px == 16 * sl + 8 * h + j) ? 1.f : 0.f);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(id, as_f16x8(cl[2 * ct + sl]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(id, as_f16x8(ch[2 * ct + sl]), acc, 0, 0, 0);
  }
  // ---- C's output tile -> y through this wave's (dead) pw chunk region: 128-byte pixel rows per store ------
  float* scr = s_pwc;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(scr + px * PS + 8 * q + 4 * h) =
        make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int pl = 8 * k + (lane >> 3), c4 = lane & 7;
    if (pl < npv * HC * HC)
      *reinterpret_cast<float4*>(y + (p0 * (HC * HC) + pl) * CB + 32 * ct + 4 * c4) =
          *reinterpret_cast<const float4*>(scr + pl * PS + 4 * c4);
  }
}

#endif  // HN_EXPERIMENTS

// A 16x16 stride-2 block (32 -> 64, SEARCH_SPACE2 layer 2) followed -- after any identity skips -- by the
// channel-changing stride-2 "skip" op at 8x8 (layer 4: MaxPool2d(3, 2, 1) then ConvBNRelu 1x1 64 -> 128,
// fbnet_builder.py:202-228; wang3's layers 2-4, fbnet_modeldef.py:30-95): the block's 8x8x64 output
// stays in LDS and the pooled 1x1 conv runs in the same workgroup, so the 16 KB / patch layer-2 output
// never reaches HBM (write + read back by k_skip_s2).  The skip arithmetic is k_skip_s2's (hn_nas.hip)
// step for step -- pooling max over the clamped 3x3 window, fp16 hi / lo split of the pooled value and of
// the weights, the same 32x32x16 fp16x3 K-loop from the bias -- so the result is bit-identical to the
// unfused pair (tests/test_gpu_parity.py).  One patch per workgroup (NPB = 1): wave w computes output
// channels 32 w .. + 31 of the 16 pooled pixels (MFMA columns 16 .. 31 repeat them and are not stored).
template <int K, int MID>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_irf_skip(
    const float* __restrict__ x, float* __restrict__ y, HnIrfArgs A,
    const uint4* __restrict__ sa,     // [128/32][64/16][plane 2][lane 64] x 8 fp16 (pack_1x1_a)
    const float* __restrict__ sbias,  // [128]
    int P) {
  constexpr int CIN = 32, COUT = 64, HIN = 16, S = 2;
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  constexpr int TI = Sh::TI, KS = Sh::KS, TW = Sh::TW, MODE = irf_mode<CIN, S>();
  constexpr int SMEM = irf_smem_floats<CIN, COUT, HIN, S, K, MID>();
  static_assert(Sh::NPB == 1 && TW == 1 && Sh::NOT == 2 && Sh::NCT == 2, "one 8x8x64 patch per workgroup");
  constexpr int XS = COUT + 4;             // block output in LDS: [64 pixels][68 floats]
  constexpr int SC = 128, SKS = COUT / 16;  // skip output channels, K-steps
  constexpr int LY = 64 * XS, LB = SKS * 2 * 64 * 4, LO = 4 * 32 * 36;
  static_assert(LY + LB + LO <= SMEM, "the skip's buffers fit in the block's LDS");
  static_assert(3 * SMEM * 4 <= 160 * 1024, "three workgroups per CU");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  const int tile = (int)blockIdx.x;  // = patch
  if (tile >= P) return;             // workgroup-uniform
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, px = lane & 31, h = lane >> 5;
  f32x16 acc[TW];
  {
    float4 pa[TI][KS], pb[TI][KS];
    irf_load<CIN, COUT, HIN, S, K, MID>(&pa[0][0], &pb[0][0], x, tile, P);
    uint4 bh[TI][KS], bl[TI][KS];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int s = 0; s < KS; ++s) split8_f16(pa[i][s], pb[i][s], bh[i][s], bl[i][s]);
    irf_core<CIN, COUT, HIN, S, K, MID, MODE>(bh, bl, acc, A.pw_a, A.pw_b, A.dw_w, A.dw_b, A.pwl_a, A.pwl_b, smem,
                                             smem + Sh::LDS_PW, smem + Sh::LDS_PW + Sh::LDS_DW);
  }
  // the skip's weights (k_skip_s2's A operand, split on the host the way k_skip_s2 splits it: row = output
  // channel 32 w + px, K-step ks = input channels 16 ks + 8 h + j) are loaded now, consumed after the pooling
  uint4 wa[SKS][2];
#pragma unroll
  for (int ks = 0; ks < SKS; ++ks) {
    wa[ks][0] = sa[((w * SKS + ks) * 2) * 64 + lane];
    wa[ks][1] = sa[((w * SKS + ks) * 2 + 1) * 64 + lane];
  }
  float* s_y = smem;
  uint4* s_b = reinterpret_cast<uint4*>(smem + LY);  // [ks][plane][lane]
  float* s_o = smem + LY + LB + w * 32 * 36;         // per-wave output staging
  {  // block output tile (pixel tile pt, channel tile ct) -> s_y; lane (px, h): channels 8q + 4h .. + 3
    const int pt = w % Sh::NOT, ct = w / Sh::NOT;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(s_y + (pt * 32 + px) * XS + 32 * ct + 8 * q + 4 * h) =
          make_float4(acc[0][4 * q], acc[0][4 * q + 1], acc[0][4 * q + 2], acc[0][4 * q + 3]);
  }
  __syncthreads();
  {  // pool: thread = (pooled pixel o, channel quad c4); the padding row / column -1 is replaced by 0
    const int o = t >> 4, c4 = t & 15, oy = o >> 2, ox = o & 3;
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = max(2 * oy - 1 + ky, 0);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = max(2 * ox - 1 + kx, 0);
        const float4 a = *reinterpret_cast<const float4*>(s_y + (yy * 8 + xx) * XS + 4 * c4);
        m.x = fmaxf(m.x, a.x); m.y = fmaxf(m.y, a.y); m.z = fmaxf(m.z, a.z); m.w = fmaxf(m.w, a.w);
      }
    }
    typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
    f16x4_t hi, lo;
    hi[0] = (_Float16)m.x; lo[0] = (_Float16)(m.x - (float)hi[0]);
    hi[1] = (_Float16)m.y; lo[1] = (_Float16)(m.y - (float)hi[1]);
    hi[2] = (_Float16)m.z; lo[2] = (_Float16)(m.z - (float)hi[2]);
    hi[3] = (_Float16)m.w; lo[3] = (_Float16)(m.w - (float)hi[3]);
    const int ks = c4 >> 2, ln = ((c4 >> 1) & 1) * 32 + o, half = c4 & 1;
#pragma unroll
    for (int d = 0; d < 2; ++d) {  // MFMA columns o and o + 16 (the latter never stored)
      reinterpret_cast<uint2*>(&s_b[(ks * 2 + 0) * 64 + ln + 16 * d])[half] = __builtin_bit_cast(uint2, hi);
      reinterpret_cast<uint2*>(&s_b[(ks * 2 + 1) * 64 + ln + 16 * d])[half] = __builtin_bit_cast(uint2, lo);
    }
  }
  f32x16 c;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b = *reinterpret_cast<const float4*>(sbias + 32 * w + 8 * q + 4 * h);
    c[4 * q] = b.x; c[4 * q + 1] = b.y; c[4 * q + 2] = b.z; c[4 * q + 3] = b.w;
  }
  __syncthreads();
#pragma unroll
  for (int ks = 0; ks < SKS; ++ks)
    c = mfma3_f16(as_f16x8(wa[ks][0]), as_f16x8(wa[ks][1]), as_f16x8(s_b[(ks * 2) * 64 + lane]),
                  as_f16x8(s_b[(ks * 2 + 1) * 64 + lane]), c);
  // bias + ReLU -> per-wave staging -> 16 pixels x 128-byte rows of channels 32 w .. + 31
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(s_o + px * 36 + 8 * q + 4 * h) =
        make_float4(relu0(c[4 * q]), relu0(c[4 * q + 1]), relu0(c[4 * q + 2]), relu0(c[4 * q + 3]));
  __builtin_amdgcn_wave_barrier();  // (one wave: its LDS accesses execute in order)
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int pl = 8 * k + (lane >> 3), c4 = lane & 7;
    *reinterpret_cast<float4*>(y + ((long)tile * 16 + pl) * SC + 32 * w + 4 * c4) =
        *reinterpret_cast<const float4*>(s_o + pl * 36 + 4 * c4);
  }
}

// The max-pool NAS front (layer 0 = the strided "skip": stem ConvBNRelu 1 -> 32 then MaxPool2d(3, 2, 1),
// model_supernet.py:57-58, fbnet_builder.py:202-228; k_front's FRONT_MAXPOOL form, hn_front.hip) and -- past an
// identity skip at layer 1 -- the first IRF block, the 16x16 stride-2 32 -> COUT one (SEARCH_SPACE2 layer 2,
// wang4's ir_k5_s2; fbnet_builder.py:455-570), in one persistent kernel: the 16x16x32 front output (32 KB per
// patch written by k_front and read back by k_irf, the 8x8 net's largest HBM stream) never leaves the workgroup.
// Per patch: the front's 4 bands (stem rows on the MFMA into the 9-row ring, the 3x3 / 2 max-pool of each band's
// 4 output rows) keep their pooled float4s in registers (8 per thread); after the last band they go to an LDS
// tile [256 pixels][36 floats] over the then dead ring, the block's pw B operands are read from it (k_irf2's
// A -> B hand-off), and irf_core / irf_store run as in k_irf.  s_in stays apart (4.6 KB), the ring (44 KB) and
// the block's buffers (46 KB) share one region: 50.7 KB, three workgroups per CU as both kernels it replaces.
// Every value takes the arithmetic of k_front + k_irf in the same order: bit-identical to the two-kernel path
// (tests/test_gpu_parity.py::test_maxpool_front_irf_kernel_is_bit_identical).
namespace mpf {
// k_front's dw/maxpool read lane map (hn_front.hip kDwLane; tests/test_lds_banks.py::test_front_dw_lane_map)
__constant__ unsigned char kLane[64] = {
    0,  1,  2,  3,  46, 47, 8,  9,  10, 11, 12, 13, 4,  5,  6,  7,  20, 21, 28, 29, 14, 15,
    22, 23, 30, 31, 38, 39, 36, 37, 44, 45, 52, 53, 54, 55, 58, 59, 60, 61, 62, 63, 24, 25,
    16, 17, 18, 19, 32, 33, 40, 41, 26, 27, 34, 35, 42, 43, 50, 51, 48, 49, 56, 57};
constexpr int IR = 9, PC = 34, RS = PC * PS;  // ring rows (2 (RB - 1) + 3), padded columns, row stride (floats)
}  // namespace mpf

template <int K, int MID, bool NORM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_mpfront_irf(
    const float* __restrict__ in, float* __restrict__ y, const uint4* __restrict__ spack,
    const float* __restrict__ stem_b, HnIrfArgs A, int P, float eps) {
  constexpr int CIN = 32, COUT = 64, HIN = 16, S = 2;
  using Sh = IrfShape<CIN, COUT, HIN, S, K, MID>;
  constexpr int TI = Sh::TI, KS = Sh::KS, TW = Sh::TW, MODE = irf_mode<CIN, S>();
  static_assert(Sh::NPB == 1 && MODE == IRF_WPAD, "one 16x16 patch per tile, dw weights in the pad slots");
  constexpr int XS = CIN + 4;                         // the front output tile: [256 pixels][36 floats]
  constexpr int RING = mpf::IR * mpf::RS;             // floats
  constexpr int BLK = irf_smem_floats<CIN, COUT, HIN, S, K, MID>();
  constexpr int REG = RING > BLK ? RING : BLK;
  static_assert(256 * XS <= REG, "the tile fits the shared region");
  static_assert(3 * (REG + 34 * 34 + 8) * 4 <= 160 * 1024, "three workgroups per CU");
  __shared__ __attribute__((aligned(16))) float s_reg[REG];  // ring | front output tile | block buffers
  __shared__ float s_in[34 * 34];
  __shared__ float red[8];
  __shared__ __attribute__((aligned(16))) float s_sb[32];  // the stem bias, read where used (registers: the block)
  float* const s_pw = s_reg;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int px = lane & 31, h = lane >> 5;
  const long per = ((long)P + gridDim.x - 1) / gridDim.x;
  const long pb = (long)xcd_remap(blockIdx.x, gridDim.x) * per;
  const long pe = min((long)P, pb + per);
  if (pb >= pe) return;  // workgroup-uniform

  for (int i = t; i < 34 * 34; i += 256) s_in[i] = 0.f;  // the frame stays zero (only 32 x 32 rewritten)
  if (t < 32) s_sb[t] = stem_b[t];
  const int lm = mpf::kLane[lane], dq = lm & 7, dox = lm >> 3;
  auto slot_of = [](int yy) { return (yy + 1 + mpf::IR) % mpf::IR; };  // ring slot of stem row yy (PAD 1)
  float4 vnext = reinterpret_cast<const float4*>(in + pb * 1024)[t];
#pragma unroll 1
  for (long patch = pb; patch < pe; ++patch) {
    float4 v = vnext;
    if (patch + 1 < pe) vnext = reinterpret_cast<const float4*>(in + (patch + 1) * 1024)[t];
    float mean = 0.f, sd = 1.f;
    if (NORM) {  // (x - mean) / (std_unbiased + eps), as k_front
      const float s0 = wave_sum(v.x + v.y + v.z + v.w);
      if (lane == 0) red[w] = s0;
      __syncthreads();
      mean = (red[0] + red[1] + red[2] + red[3]) * (1.f / 1024.f);
      const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
      const float q = wave_sum(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
      if (lane == 0) red[4 + w] = q;
      __syncthreads();
      sd = sqrtf((red[4] + red[5] + red[6] + red[7]) * (1.f / 1023.f)) + eps;
    }
    __syncthreads();  // the previous patch is done with s_in and the shared region
    {
      const int q = 4 * t, yy = q >> 5, xx = q & 31;
      float* d = s_in + (yy + 1) * 34 + xx + 1;
      if (NORM) {
        d[0] = (v.x - mean) / sd; d[1] = (v.y - mean) / sd;
        d[2] = (v.z - mean) / sd; d[3] = (v.w - mean) / sd;
      } else {
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    }
    // the ring's left pad column (x = -1; the block's buffers overwrote it): zero, as k_front's one-time init
    for (int i = t; i < mpf::IR * (PS / 4); i += 256)
      reinterpret_cast<float4*>(s_pw)[(i / (PS / 4)) * (mpf::RS / 4) + i % (PS / 4)] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    // the stem A operand (L2-resident) per patch: not held in registers through the block's phase
    const f16x8 sah = as_f16x8(spack[lane]), sal = as_f16x8(spack[64 + lane]);
    // the pooled output, band b, j -> pixel (4 b + orr, ox), channels 4 dq .. + 3, in mp[b][j] after the
    // band loop (a register FIFO shifted once per band: the loop stays rolled)
    float4 mp[4][2];
#pragma unroll 1
    for (int band = 0; band < 4; ++band) {
      const int r0 = band * 4;
      const int ylast = 2 * r0 + 7, ybeg = band > 0 ? ylast - 7 : -1;  // the ring's new rows
      const int nreal = ylast + 1 - ybeg;
#pragma unroll
      for (int i = 0; i < 3; ++i) {  // stem row tiles w + 4 i (k_front's non-PAIR phase A)
        const int ri = w + 4 * i, yy = ybeg + ri;
        if (ri >= nreal) continue;  // wave-uniform
        if (yy < 0 || yy >= 32) {   // padding row of the stem output
          float4* d = reinterpret_cast<float4*>(s_pw + slot_of(yy) * mpf::RS);
          for (int j = lane; j < mpf::RS / 4; j += 64) d[j] = make_float4(0.f, 0.f, 0.f, 0.f);
          continue;
        }
        float tp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = 8 * h + j;  // h = 1 holds tap 8 and zeros
          tp[j] = tap < 9 ? s_in[(yy + tap / 3) * 34 + px + tap % 3] : 0.f;
        }
        uint4 xh, xl;
        split8_f16(make_float4(tp[0], tp[1], tp[2], tp[3]), make_float4(tp[4], tp[5], tp[6], tp[7]), xh, xl);
        f32x16 sbr;  // the stem bias in the accumulator order (lane (px, h): acc[4q + r] = channel 4h + 8q + r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 b = *reinterpret_cast<const float4*>(s_sb + 8 * q + 4 * h);
          sbr[4 * q] = b.x; sbr[4 * q + 1] = b.y; sbr[4 * q + 2] = b.z; sbr[4 * q + 3] = b.w;
        }
        const f32x16 c = mfma3_f16(sah, sal, as_f16x8(xh), as_f16x8(xl), sbr);
        float4* d = reinterpret_cast<float4*>(s_pw + slot_of(yy) * mpf::RS + (1 + px) * PS);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          d[2 * q + h] = make_float4(relu0(c[4 * q]), relu0(c[4 * q + 1]), relu0(c[4 * q + 2]), relu0(c[4 * q + 3]));
      }
      __syncthreads();
      // MaxPool2d(3, 2, 1): padding never wins since every window holds a ReLU output >= 0
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pp = 8 * (w + 4 * j) + dox, orr = pp >> 4, ox = pp & 15;
        float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const float* rp = s_pw + slot_of(2 * (r0 + orr) - 1 + dy) * mpf::RS;
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) {
            const float4 a = *reinterpret_cast<const float4*>(rp + (2 * ox + dx) * PS + 4 * dq);
            m.x = fmaxf(m.x, a.x); m.y = fmaxf(m.y, a.y); m.z = fmaxf(m.z, a.z); m.w = fmaxf(m.w, a.w);
          }
        }
#pragma unroll
        for (int b = 0; b < 3; ++b) mp[b][j] = mp[b + 1][j];
        mp[3][j] = m;
      }
      __syncthreads();  // reads done before the next band's rows (or the output tile) overwrite ring slots
    }
    // the front output tile -> LDS [pixel][XS] over the dead ring; the block's pw B operands from it
#pragma unroll
    for (int band = 0; band < 4; ++band)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pp = 8 * (w + 4 * j) + dox;
        *reinterpret_cast<float4*>(s_reg + (band * 64 + pp) * XS + 4 * dq) = mp[band][j];
      }
    __syncthreads();
    uint4 bh[TI][KS], bl[TI][KS];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float4* src = reinterpret_cast<const float4*>(s_reg + ((4 * i + w) * 32 + px) * XS + 16 * s + 8 * h);
        split8_f16(src[0], src[1], bh[i][s], bl[i][s]);
      }
    __syncthreads();  // the region is the block's pw / dw buffers from here
    f32x16 acc[TW];
    irf_core<CIN, COUT, HIN, S, K, MID, MODE>(bh, bl, acc, A.pw_a, A.pw_b, A.dw_w, A.dw_b, A.pwl_a, A.pwl_b, s_reg,
                                             s_reg + Sh::LDS_PW, s_reg + Sh::LDS_PW + Sh::LDS_DW);
    irf_store<CIN, COUT, HIN, S, K, MID>(acc, y, patch, 1, s_reg);
  }
}

template <int CIN, int COUT, int HIN, int S, int K, int MID>
hipError_t irf_launch(const HnIrfArgs& a, int P, hipStream_t st) {
  constexpr int NPB = IrfTile<CIN, HIN, MID>::NPB;
  hipLaunchKernelGGL((k_irf<CIN, COUT, HIN, S, K, MID>), dim3((P + NPB - 1) / NPB), dim3(256), 0, st, a.x, a.y,
                     a.pw_a, a.pw_b, a.dw_w, a.dw_b, a.pwl_a, a.pwl_b, P);
  return hipGetLastError();
}

template <int CA, int HI, int KA, int MA, int CB, int KB, int MB>
hipError_t irf2_launch(const HnIrfArgs& a, const HnIrfArgs& b, int P, hipStream_t st) {
  constexpr int NPB = IrfTile<CA, HI, MA>::NPB;
  hipLaunchKernelGGL((k_irf2<CA, HI, KA, MA, CB, KB, MB>), dim3((P + NPB - 1) / NPB), dim3(256), 0, st, a.x, b.y, a,
                     b, P);
  return hipGetLastError();
}

#ifdef HN_EXPERIMENTS
template <int KA, int KB, int KC>
hipError_t irf3_launch(const HnIrfArgs& a, const HnIrfArgs& b, const HnIrfArgs& c, int P, hipStream_t st) {
  constexpr int NPB = IrfTile<64, 8, 64>::NPB;
  hipLaunchKernelGGL((k_irf3<64, 8, KA, 64, 128, KB, 64, KC, 128>), dim3((P + NPB - 1) / NPB), dim3(256), 0, st, a.x,
                     c.y, a, b, c, P);
  return hipGetLastError();
}
#endif

}  // namespace

#ifdef HN_EXPERIMENTS
// three consecutive blocks fused (k_irf3): k_irf2's 8x8 pair (64 -> 64 stride 1 mid 64, then 64 -> 128 stride 2
// mid 64: e1 / s2 ops at SEARCH_SPACE2 layers 3 -> 4) and the 4x4 128 -> 128 e1 block of layer 5, kernels 3 / 5
bool hn_irf3_supported(int ka, int ma, int kb, int mb, int kc, int mc) {
  return ma == 64 && mb == 64 && mc == 128 && (ka == 3 || ka == 5) && (kb == 3 || kb == 5) && (kc == 3 || kc == 5);
}

hipError_t hn_launch_irf3(const HnIrfArgs& a, const HnIrfArgs& b, const HnIrfArgs& c, int P, int ka, int kb, int kc,
                          hipStream_t st) {
  if (P <= 0) return hipSuccess;
#define HN_IRF3_GO(KA, KB, KC) \
  if (ka == KA && kb == KB && kc == KC) return irf3_launch<KA, KB, KC>(a, b, c, P, st);
  HN_IRF3_GO(3, 3, 3) HN_IRF3_GO(3, 3, 5) HN_IRF3_GO(3, 5, 3) HN_IRF3_GO(3, 5, 5)
  HN_IRF3_GO(5, 3, 3) HN_IRF3_GO(5, 3, 5) HN_IRF3_GO(5, 5, 3) HN_IRF3_GO(5, 5, 5)
#undef HN_IRF3_GO
  return hipErrorInvalidValue;
}
#endif

// two consecutive blocks fused (k_irf2): A = (CA -> CA, stride 1, kernel KA, mid MA) at HI x HI,
// B = (CA -> CB, stride 2, KB, MB); e = 1 / s2 ops (mid = CA) at SEARCH_SPACE2 layers 1 -> 2 and 3 -> 4
#define HN_IRF2_SHAPES(X) \
  X(32, 16, 3, 32, 64, 3, 32) X(32, 16, 3, 32, 64, 5, 32) X(32, 16, 5, 32, 64, 3, 32) X(32, 16, 5, 32, 64, 5, 32) \
  X(64, 8, 3, 64, 128, 3, 64) X(64, 8, 3, 64, 128, 5, 64) X(64, 8, 5, 64, 128, 3, 64) X(64, 8, 5, 64, 128, 5, 64)

bool hn_irf2_supported(int ca, int hi, int ka, int ma, int cb, int kb, int mb) {
#define HN_IRF2_SUP(CA, HI, KA, MA, CB, KB, MB) \
  if (ca == CA && hi == HI && ka == KA && ma == MA && cb == CB && kb == KB && mb == MB) return true;
  HN_IRF2_SHAPES(HN_IRF2_SUP)
#undef HN_IRF2_SUP
  return false;
}

hipError_t hn_launch_irf2(const HnIrfArgs& a, const HnIrfArgs& b, int P, int ca, int hi, int ka, int ma, int cb,
                          int kb, int mb, hipStream_t st) {
  if (P <= 0) return hipSuccess;
#define HN_IRF2_GO(CA, HI, KA, MA, CB, KB, MB) \
  if (ca == CA && hi == HI && ka == KA && ma == MA && cb == CB && kb == KB && mb == MB) \
    return irf2_launch<CA, HI, KA, MA, CB, KB, MB>(a, b, P, st);
  HN_IRF2_SHAPES(HN_IRF2_GO)
#undef HN_IRF2_GO
  return hipErrorInvalidValue;
}

// layer 2 (32 -> 64, 16x16, stride 2; e1 / e3 / e4, k3 / k5) + the 8x8 64 -> 128 skip (k_irf_skip)
bool hn_irf_skip_supported(int cin, int cout, int hin, int s, int k, int mid) {
  return cin == 32 && cout == 64 && hin == 16 && s == 2 && (k == 3 || k == 5) && (mid == 32 || mid == 96 || mid == 128);
}

hipError_t hn_launch_irf_skip(const HnIrfArgs& a, const uint4* skip_a, const float* skip_b, int P, int k, int mid,
                              hipStream_t st) {
  if (P <= 0) return hipSuccess;
#define HN_IRFSK_GO(KK, MM)                                                                               \
  if (k == KK && mid == MM) {                                                                             \
    hipLaunchKernelGGL((k_irf_skip<KK, MM>), dim3(P), dim3(256), 0, st, a.x, a.y, a, skip_a, skip_b, P); \
    return hipGetLastError();                                                                             \
  }
  HN_IRFSK_GO(3, 32) HN_IRFSK_GO(3, 96) HN_IRFSK_GO(3, 128) HN_IRFSK_GO(5, 32) HN_IRFSK_GO(5, 96) HN_IRFSK_GO(5, 128)
#undef HN_IRFSK_GO
  return hipErrorInvalidValue;
}

// max-pool front + the 16x16 stride-2 32 -> 64 block (k_mpfront_irf): k3 / k5, e1 / e3 / e4 (mid 32 / 96 / 128)
bool hn_mpfront_irf_supported(int cin, int cout, int hin, int s, int k, int mid) {
  return hn_irf_skip_supported(cin, cout, hin, s, k, mid);
}

hipError_t hn_launch_mpfront_irf(const float* in, const uint4* spack, const float* stem_b, const HnIrfArgs& a, int P,
                                 int k, int mid, bool norm, float eps, hipStream_t st) {
  if (P <= 0) return hipSuccess;
#define HN_MPF_GO(KK, MM, NN)                                                                                      \
  if (k == KK && mid == MM && norm == NN) {                                                                        \
    int resident = 0; /* persistent grid: every workgroup resident at once */                                      \
    const hipError_t e = hn_resident_blocks(reinterpret_cast<const void*>(&k_mpfront_irf<KK, MM, NN>), 256, 0, &resident); \
    if (e != hipSuccess) return e;                                                                                 \
    hipLaunchKernelGGL((k_mpfront_irf<KK, MM, NN>), dim3(std::min(P, resident)), dim3(256), 0, st, in, a.y, spack, \
                       stem_b, a, P, eps);                                                                         \
    return hipGetLastError();                                                                                      \
  }
  HN_MPF_GO(3, 32, false) HN_MPF_GO(3, 96, false) HN_MPF_GO(3, 128, false)
  HN_MPF_GO(5, 32, false) HN_MPF_GO(5, 96, false) HN_MPF_GO(5, 128, false)
#undef HN_MPF_GO
  return hipErrorInvalidValue;
}

// SEARCH_SPACE2 layers 1..5 (cin, cout, hin, stride) x k in {3,5} x e in {1,3,4}
#define HN_IRF_SHAPES(X, K)                                                                     \
  X(32, 32, 16, 1, K, 32) X(32, 32, 16, 1, K, 96) X(32, 32, 16, 1, K, 128)                       \
  X(32, 64, 16, 2, K, 32) X(32, 64, 16, 2, K, 96) X(32, 64, 16, 2, K, 128)                       \
  X(64, 64, 8, 1, K, 64) X(64, 64, 8, 1, K, 192) X(64, 64, 8, 1, K, 256)                         \
  X(64, 128, 8, 2, K, 64) X(64, 128, 8, 2, K, 192) X(64, 128, 8, 2, K, 256)                      \
  X(128, 128, 4, 1, K, 128) X(128, 128, 4, 1, K, 384) X(128, 128, 4, 1, K, 512)

bool hn_irf_supported(int cin, int cout, int hin, int s, int k, int mid) {
#define HN_IRF_SUP(CI, CO, HI, SS, KK, MM) \
  if (cin == CI && cout == CO && hin == HI && s == SS && k == KK && mid == MM) return true;
  HN_IRF_SHAPES(HN_IRF_SUP, 3) HN_IRF_SHAPES(HN_IRF_SUP, 5)
#undef HN_IRF_SUP
  return false;
}

hipError_t hn_launch_irf(const HnIrfArgs& a, int P, int cin, int cout, int hin, int s, int k, int mid,
                         hipStream_t st) {
  if (P <= 0) return hipSuccess;
#define HN_IRF_GO(CI, CO, HI, SS, KK, MM) \
  if (cin == CI && cout == CO && hin == HI && s == SS && k == KK && mid == MM) \
    return irf_launch<CI, CO, HI, SS, KK, MM>(a, P, st);
  HN_IRF_SHAPES(HN_IRF_GO, 3) HN_IRF_SHAPES(HN_IRF_GO, 5)
#undef HN_IRF_GO
  return hipErrorInvalidValue;
}
