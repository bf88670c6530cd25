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

template <int CIN, int HIN>
struct IrfTile {
  static constexpr int NPB = CIN == 128 ? 128 / (HIN * HIN) : 256 / (HIN * HIN);
  static constexpr int NI = NPB * HIN * HIN;  // input pixels per workgroup
};

// The 64 -> 128 stride-2 and the 128-channel (4x4) blocks are held to 168 VGPRs, three
// workgroups per CU (their LDS allows three; the k5 forms spill 20-25 dwords and still gain):
// wang2 / wang4 / FDLNet irf -1 to -2 %.  The 32 -> 64 stride-2 blocks lose with the same cap
// (+6 % irf: their register prefetch of the next tile spills).
template <int CIN, int COUT, int HIN, int S, int K, int MID>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((CIN == 64 && S == 2) || CIN == 128 ? 3 : 1))) void k_irf(const float* __restrict__ x, float* __restrict__ y,
                                             const uint4* __restrict__ pw_a,   // [MID/32][CIN/16][2][64]
                                             const float* __restrict__ pw_b,   // [MID] dw order
                                             const float* __restrict__ dw_w,   // [K*K][MID]
                                             const float* __restrict__ dw_b,   // [MID]
                                             const uint4* __restrict__ pwl_a,  // [COUT/32][MID/16][2][64]
                                             const float* __restrict__ pwl_b,  // [COUT]
                                             int P) {
  constexpr int HOUT = HIN / S, PAD = K / 2;
  constexpr int NPB = IrfTile<CIN, HIN>::NPB, NI = IrfTile<CIN, HIN>::NI;
  constexpr int NO = NPB * HOUT * HOUT;           // output pixels per workgroup
  constexpr int TI = NI / 32 / 4;                 // pw pixel tiles per wave
  constexpr int KS = CIN / 16;                    // pw K-steps
  constexpr int NOT = NO / 32, NCT = COUT / 32;   // pwl pixel tiles, cout tiles
  constexpr int TW = NOT * NCT / 4;               // pwl tiles per wave
  constexpr int R = S == 1 ? 4 : 2;               // dw run length (output pixels per thread)
  constexpr int RUNS = NO / R;                    // runs per chunk (x 8 channel quads)
  constexpr int WIN = (R - 1) * S + K;            // input columns of a run window
  constexpr bool RES = S == 1 && CIN == COUT;
  static_assert(NI % 128 == 0 && NO % 32 == 0 && (NOT * NCT) % 4 == 0, "tile shape");
  static_assert(HOUT % R == 0, "dw run must stay in one row");
  __shared__ __attribute__((aligned(16))) float s_pw[NI * PS];
  __shared__ __attribute__((aligned(16))) float s_dw[NO * PS];
  __shared__ __attribute__((aligned(16))) float s_w[K * K * 32 + 32];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int px = lane & 31, h = lane >> 5;
  // persistent: a contiguous range of tiles per workgroup; the next tile's input is
  // prefetched into registers while the current one is computed
  // register prefetch + persistence only where the VGPR budget allows it without losing
  // occupancy (CIN = 32); otherwise one tile per workgroup
  constexpr bool PREF = CIN == 32;
  const int ntiles = (P + NPB - 1) / NPB;
  const int per = PREF ? (ntiles + (int)gridDim.x - 1) / (int)gridDim.x : 1;
  const int tbeg = (int)blockIdx.x * per, tend = PREF ? min(ntiles, tbeg + per) : tbeg + 1;
  if (tbeg >= ntiles) return;  // workgroup-uniform

  float4 pa[TI][KS], pb[TI][KS];
#define HN_IRF_LOAD(TILE)                                                                   \
  {                                                                                         \
    const long q0 = (long)(TILE) * NPB;                                                     \
    const int nv = (int)min<long>(NPB, P - q0);                                             \
    _Pragma("unroll") for (int i = 0; i < TI; ++i) {                                        \
      const int p = (4 * i + w) * 32 + px;                                                  \
      const bool ok = p < nv * HIN * HIN;                                                   \
      _Pragma("unroll") for (int s = 0; s < KS; ++s) {                                      \
        pa[i][s] = pb[i][s] = make_float4(0.f, 0.f, 0.f, 0.f);                              \
        if (ok) {                                                                           \
          const float4* src = reinterpret_cast<const float4*>(                              \
              x + (q0 * (HIN * HIN) + p) * CIN + 16 * s + 8 * h);                           \
          pa[i][s] = src[0];                                                                \
          pb[i][s] = src[1];                                                                \
        }                                                                                   \
      }                                                                                     \
    }                                                                                       \
  }
  if (PREF) HN_IRF_LOAD(tbeg)
#pragma unroll 1
  for (int tile = tbeg; tile < tend; ++tile) {
  if (!PREF) HN_IRF_LOAD(tile)
  const long p0 = (long)tile * NPB;  // first patch of the tile
  const int npv = (int)min<long>(NPB, P - p0);

  // ---- pw B operands: pixel tiles 4i + w of the workgroup tile (lane: pixel, 8 channels) --
  uint4 bh[TI][KS], bl[TI][KS];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int s = 0; s < KS; ++s) split8_f16(pa[i][s], pb[i][s], bh[i][s], bl[i][s]);
  if (PREF && tile + 1 < tend) HN_IRF_LOAD(tile + 1)

  // pwl accumulators start at the pwl bias (lane (px, h): acc[4q + r] = channel 8q + 4h + r
  // of the tile's 32 output channels), so the epilogue is stores only
  f32x16 acc[TW];
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
    // dw weights + bias of the chunk
    for (int i = t; i < K * K * 8 + 8; i += 256) {
      float4 wv;
      if (i < K * K * 8)
        wv = *reinterpret_cast<const float4*>(dw_w + (i >> 3) * MID + 32 * m + 4 * (i & 7));
      else
        wv = *reinterpret_cast<const float4*>(dw_b + 32 * m + 4 * (i - K * K * 8));
      reinterpret_cast<float4*>(s_w)[i] = wv;
    }
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
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const uint4* ap = pw_a + ((size_t)(m * KS + s) * 2) * 64 + lane;
        const f16x8 ah = as_f16x8(ap[0]), al = as_f16x8(ap[64]);
#pragma unroll
        for (int i = 0; i < TI; ++i) c[i] = mfma3_f16(ah, al, as_f16x8(bh[i][s]), as_f16x8(bl[i][s]), c[i]);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        float4* d = reinterpret_cast<float4*>(s_pw + ((4 * i + w) * 32 + px) * PS);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          d[2 * q + h] = make_float4(fmaxf(c[i][4 * q], 0.f), fmaxf(c[i][4 * q + 1], 0.f),
                                     fmaxf(c[i][4 * q + 2], 0.f), fmaxf(c[i][4 * q + 3], 0.f));
      }
    }
    __syncthreads();
    // ---- dw: thread item = (run of R output pixels in one row, channel quad q) -----------
#pragma unroll 1
    for (int it = t; it < RUNS * 8; it += 256) {
      // lane -> (run, channel quad): each 16-lane ds_read_b128 group holds 4 runs x 4 quads,
      // whose window reads land in 16 distinct bank slots (slot = 4 run + q + 9 dx mod 16)
      const int q = (lane & 3) | ((lane >> 5) << 2), run = (it >> 6) * 8 + ((lane >> 2) & 7);
      const int o0 = run * R;  // first output pixel (tile-local)
      const int pl = o0 / (HOUT * HOUT), oy = (o0 / HOUT) % HOUT, ox0 = o0 % HOUT;
      const f32x4 b4 = reinterpret_cast<const f32x4*>(s_w + K * K * 32)[q];
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
          const f32x4 wv = reinterpret_cast<const f32x4*>(s_w + (dy * K + dx) * 32)[q];
#pragma unroll
          for (int r = 0; r < R; ++r) o[r] = __builtin_elementwise_fma(wv, win[r * S + dx], o[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
        *reinterpret_cast<f32x4*>(s_dw + (o0 + r) * PS + 4 * q) = __builtin_elementwise_max(o[r], f32x4{});
    }
    __syncthreads();
    // ---- pwl (accumulate this chunk's 32 mid channels = 2 K-steps) -----------------------
#pragma unroll
    for (int i = 0; i < TW; ++i) {
      const int tile = 4 * i + w, pt = tile % NOT, ct = tile / NOT;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float4* src = reinterpret_cast<const float4*>(s_dw + (pt * 32 + px) * PS + 16 * s + 8 * h);
        uint4 xh, xl;
        split8_f16(src[0], src[1], xh, xl);
        const uint4* ap = pwl_a + ((size_t)(ct * (MID / 16) + 2 * m + s) * 2) * 64 + lane;
        acc[i] = mfma3_f16(as_f16x8(ap[0]), as_f16x8(ap[64]), as_f16x8(xh), as_f16x8(xl), acc[i]);
      }
    }
    __syncthreads();  // s_pw / s_dw / s_w are rewritten by the next chunk
  }

  // ---- residual: y += x as two more MFMA K-steps per tile with an identity A operand
  // against the x B operands already in registers (x = hi + lo to ~2^-22; no second read of
  // x from HBM).  With S = 1, NI = NO, so the wave's pwl pixel tiles are its pw tiles.
  if (RES) {
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

  // ---- epilogue (the bias is in the accumulators): each 32-pixel x 32-channel tile goes through
  // a per-wave scratch in s_pw (free after the last chunk's barrier), so that every float4 store
  // instruction writes 8 whole 128-byte pixel rows instead of 32 pixels x 32 bytes ---------------
  float* scr = s_pw + w * 32 * PS;
  static_assert(NI * PS >= 4 * 32 * PS, "scratch fits in s_pw");
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
  }  // tile loop
#undef HN_IRF_LOAD
}

template <int CIN, int COUT, int HIN, int S, int K, int MID>
hipError_t irf_launch(const HnIrfArgs& a, int P, hipStream_t st) {
  constexpr int NPB = IrfTile<CIN, HIN>::NPB;
  const void* fn = reinterpret_cast<const void*>(&k_irf<CIN, COUT, HIN, S, K, MID>);
  int resident = 0;  // persistent grid: every workgroup resident at once
  const hipError_t e = hn_resident_blocks(fn, 256, 0, &resident);
  if (e != hipSuccess) return e;
  const int grid = CIN == 32 ? std::min((P + NPB - 1) / NPB, resident) : (P + NPB - 1) / NPB;
  hipLaunchKernelGGL((k_irf<CIN, COUT, HIN, S, K, MID>), dim3(grid), dim3(256), 0, st, a.x, a.y, a.pw_a,
                     a.pw_b, a.dw_w, a.dw_b, a.pwl_a, a.pwl_b, P);
  return hipGetLastError();
}

}  // namespace

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
