// Train-mode stock HardNet on the GPU: the forward with BatchNorm batch
// statistics (and running-statistics update), Dropout(0.3), and the backward to every conv
// weight (and optionally the input), as the reference's training step runs it through autograd
// (hardnet/HardNet.py:379-441 over the module of :275-315).
//
// Layout: activations are kept channel-major across the whole batch, CNHW ([C][B][H][W]), so
//   * each conv is ONE implicit GEMM over the whole batch, its column matrix never stored (the
//     B-operand loader computes the im2col / col2im addresses; K = Cin*k*k):
//                     forward  Y  [Cout][BHW]  = W [Cout][K] . col,
//                     wgrad    dW [Cout][K]    = dY [Cout][BHW] . col^T  (split-K, fp64 sums),
//                     dgrad    dX [Cin][BHinWin] = Wt [Cin][Cout k k] . gather(dY);
//   * BatchNorm's per-channel batch statistics are reductions over one contiguous row.
// GEMMs run on the f32 MFMA (exact fp32 products, fp64 sums across split-K slices).
// Saved for the backward (the workspace the caller keeps between the calls): the normalised
// pre-ReLU output z of every BN layer, its 1/sqrt(var + eps), the normalised input and the
// per-patch input std.  The next layer's input relu(z) (x mask / (1 - p) after the dropout) is
// formed on the fly in the im2col loader; the dropout mask is a counter hash of (seed, element),
// so the backward recomputes it instead of storing it.
#include "hn_common.h"
#include "hn_internal.h"
#include "hn_train_kernels.h"

#include <algorithm>
#include <cstring>

namespace {
// conv weights W [cout][cin][3][3] (raw, or flipped and transposed for the data gradient:
// W'[ci][co][tap] = W[co][ci][8 - tap]) -> the bf16x3 MFMA fragments of the inference conv kernels
// (hn_api.hip pack_conv3x3 layout [cin/32][tap][ks][cout/32][plane][lane][8]), on the GPU since
// the weights change every step
__global__ __launch_bounds__(256) void k_pack3x3(const float* __restrict__ w, int cin_w, int cout_w, int flip,
                                                 unsigned short* __restrict__ out) {
  const int cin = flip ? cout_w : cin_w, cout = flip ? cin_w : cout_w, ntot = cout / 32;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // one (hi, lo) pair per thread
  if (e >= (long)cin * cout * 9) return;
  const int j = (int)(e & 7), lane = (int)((e >> 3) & 63);
  long r = e >> 9;
  const int nt = (int)(r % ntot);
  r /= ntot;
  const int ks = (int)(r & 1);
  r >>= 1;
  const int tap = (int)(r % 9), cc = (int)(r / 9);
  const int n = nt * 32 + (lane & 31), c = cc * 32 + ks * 16 + (lane >> 5) * 8 + j;
  const float v = flip ? w[((long)c * cin_w + n) * 9 + 8 - tap] : w[((long)n * cin_w + c) * 9 + tap];
  const __bf16 hv = (__bf16)v, lv = (__bf16)(v - (float)hv);
  const long o = ((((long)(cc * 9 + tap) * 2 + ks) * ntot + nt) * 2 * 64 + lane) * 8 + j;
  out[o] = __builtin_bit_cast(unsigned short, hv);
  out[o + 64 * 8] = __builtin_bit_cast(unsigned short, lv);
}

// CNHW [C][B][HW] (relu optional) <-> NHWC [B][HW][C] through a 64-pixel x C LDS tile: both sides
// coalesced.  grid (HW / 64, B)
__global__ __launch_bounds__(256) void k_cnhw_to_nhwc(const float* __restrict__ z, int C, long B, int HW, int relu,
                                                      float* __restrict__ out) {
  __shared__ float tile[128][65];
  const long b = blockIdx.y;
  const int p0 = blockIdx.x * 64, t = threadIdx.x;
  for (int i = t; i < C * 64; i += 256) {
    const int c = i >> 6, p = i & 63;
    float v = z[((long)c * B + b) * HW + p0 + p];
    tile[c][p] = relu ? fmaxf(v, 0.f) : v;
  }
  __syncthreads();
  for (int i = t; i < C * 64; i += 256) {
    const int p = i / C, c = i % C;
    out[(b * HW + p0 + p) * C + c] = tile[c][p];
  }
}
__global__ __launch_bounds__(256) void k_nhwc_to_cnhw(const float* __restrict__ in, int C, long B, int HW,
                                                      float* __restrict__ z) {
  __shared__ float tile[128][65];
  const long b = blockIdx.y;
  const int p0 = blockIdx.x * 64, t = threadIdx.x;
  for (int i = t; i < C * 64; i += 256) {
    const int p = i / C, c = i % C;
    tile[c][p] = in[(b * HW + p0 + p) * C + c];
  }
  __syncthreads();
  for (int i = t; i < C * 64; i += 256) {
    const int c = i >> 6, p = i & 63;
    z[((long)c * B + b) * HW + p0 + p] = tile[c][p];
  }
}

unsigned grid_for(long n) { return (unsigned)std::min<long>((n + 255) / 256, 65536); }

// conv6's data gradient (8x8 kernel over an 8x8 input, one output position): the column matrix
// dcol [(ci, p)][b] = W^T . dY is the gradient itself, in [ci][p][b] order -- transpose each ci's
// 64 x n block to [ci][b][p] through an LDS tile (coalesced on both sides)
__global__ __launch_bounds__(256) void k_col6_to_cnhw(const float* __restrict__ dcol, long B, long n0, long n,
                                                      float* __restrict__ din) {
  __shared__ float tile[64][65];
  const int ci = blockIdx.x, t = threadIdx.x;
  const long b0 = (long)blockIdx.y * 64;
  for (int i = t; i < 64 * 64; i += 256) {
    const int p = i >> 6, bb = i & 63;
    tile[p][bb] = b0 + bb < n ? dcol[((long)ci * 64 + p) * n + b0 + bb] : 0.f;
  }
  __syncthreads();
  for (int i = t; i < 64 * 64; i += 256) {
    const int bb = i >> 6, p = i & 63;
    if (b0 + bb < n) din[((long)ci * B + n0 + b0 + bb) * 64 + p] = tile[p][bb];
  }
}

// ------------------------------------------------------------------------------------------
// weight gradient of a stride-1 3x3 layer (conv1 / conv3 / conv5):
//   dW[co][ci][tap] = sum over (b, y, x) of dY[co][b][y][x] . X[ci][b][y + dy - 1][x + dx - 1]
// with X = relu(z of the previous layer) (CNHW).  One wave per (32 co x 32 ci) block and run of
// patches, all 9 taps in registers (9 f32 MFMA accumulators, v_mfma_f32_32x32x2_f32: exact fp32
// products); the wave streams its patches row by row through its own LDS: the dY row and a ring
// of three X rows with zero halo columns (rows -1 and H are zero rows), so the 9 shifted operands
// are plain ds_read_b32 at padded (odd) row strides -- no im2col index arithmetic.  Each wave
// writes its partial sums as one split-K slice (slice = chunk * 4 + wave; k_splitk_sum adds the
// slices in fp64).  Chunk = 4096 / (H * H) patches, 1,024 positions per wave.
// ------------------------------------------------------------------------------------------
template <int CIN, int COUT, int H>
struct Wg3Cfg {
  static constexpr int NPC = 4096 / (H * H);   // patches per workgroup chunk (4 waves)
  static constexpr int NPW = NPC / 4;          // patches per wave
  static constexpr int RSY = H + 1;            // dY row stride (floats): odd -> conflict-free
  static constexpr int XW = H + 2;             // X row with halo
  static constexpr int RSX = (3 * XW) | 1;     // per-channel ring stride (odd)
  static constexpr int WAVE_F = 32 * RSY + 32 * RSX;  // floats of LDS per wave
  static constexpr int NCO = COUT / 32, NCI = CIN / 32;
  static_assert(NPW >= 1 && NPC % 4 == 0, "chunking");
};

// The workgroup's one split-K slice of dW: its 4 waves' 9 tap accumulators summed in wave order (w0 + w1 + w2
// + w3, fp32) through LDS, one tap per round (16 KB), wave w adding and storing accumulator rows 4w .. 4w + 3;
// k_splitk_sum then adds the slices in fp64.  (One slice per wave made the slice sum 4x longer.)
template <int CIN, int COUT>
HN_DEV void wgrad_slice_write(const f32x16 (&acc)[9], float* smem, float* __restrict__ dst, int co0, int ci0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    __syncthreads();  // (the waves are done with their rings / the previous tap's reads)
#pragma unroll
    for (int i = 0; i < 16; ++i) smem[(w * 16 + i) * 64 + lane] = acc[t][i];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = 4 * w + k;
      float v = smem[i * 64 + lane];
#pragma unroll
      for (int src = 1; src < 4; ++src) v += smem[(src * 16 + i) * 64 + lane];
      dst[(long)(co0 + 8 * w + 4 * h + k) * (CIN * 9) + (ci0 + r) * 9 + t] = v;  // i = 4q + e: q = w, e = k
    }
  }
}

// NS: as k_fwd3's row segments -- the chunk's NPC units are (patch, segment of H / NS rows), so a small batch
// gets NS times the waves (and NS times the split-K slices; each product lands in the same fp64 slice sum)
template <int CIN, int COUT, int H, int NS = 1>
__global__ __launch_bounds__(256) void k_wgrad3(const float* __restrict__ zx, const float* __restrict__ dY, long B,
                                                float* __restrict__ part) {
  using C = Wg3Cfg<CIN, COUT, H>;
  constexpr int HS = H / NS;
  static_assert(4 * C::WAVE_F >= 4 * 16 * 64, "the slice reduction's round fits the rings");
  __shared__ float smem[4 * C::WAVE_F];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int blk = blockIdx.x, co0 = (blk / C::NCI) * 32, ci0 = (blk % C::NCI) * 32;
  const long chunk = blockIdx.y;
  float* sy = smem + w * C::WAVE_F;  // [32 co][RSY]
  float* sx = sy + 32 * C::RSY;      // [32 ci][3 slots][XW] (+pad)
  // halo columns and unused pad stay zero for the kernel's lifetime
  for (int i = lane; i < 32 * C::RSX; i += 64) sx[i] = 0.f;
  __builtin_amdgcn_wave_barrier();
  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x16{};
  constexpr int HH = H * H, NPR = 32 * H / 64;  // floats per lane of one 32-channel row
  static_assert(NPR >= 1 && (32 * H) % 64 == 0, "row split");
  // one 32-channel row (channels c0.., patch b, row y) of src: lane -> NPR consecutive floats
  auto load_row = [&](const float* src, int c0, long b, int y, float (&v)[NPR], bool relu) {
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int e = lane * NPR + i, c = e / H, x = e % H;
      float t = 0.f;
      if (y >= 0 && y < H) t = src[((long)(c0 + c) * B + b) * HH + y * H + x];
      v[i] = relu ? fmaxf(t, 0.f) : t;
    }
  };
  auto put_y = [&](const float (&v)[NPR]) {
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int e = lane * NPR + i, c = e / H, x = e % H;
      sy[c * C::RSY + x] = v[i];
    }
  };
  auto put_x = [&](const float (&v)[NPR], int y) {  // row y (-1 .. H) into its ring slot
    const int slot = (y + 1) % 3;
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int e = lane * NPR + i, c = e / H, x = e % H;
      sx[c * C::RSX + slot * C::XW + 1 + x] = v[i];
    }
  };
#pragma unroll 1
  for (int pi = 0; pi < C::NPW; ++pi) {
    const long u = chunk * C::NPC + w + 4 * pi;
    const long b = u / NS;
    if (b >= B) break;  // wave-uniform
    const int ys = (int)(u % NS) * HS, ye = ys + HS;
    float vy[NPR], vx[NPR];
    // prologue: X rows ys - 1, ys, ys + 1 and dY row ys (the ring slot of row y is (y + 1) % 3)
    load_row(zx, ci0, b, ys - 1, vx, true); put_x(vx, ys - 1);
    load_row(zx, ci0, b, ys, vx, true);     put_x(vx, ys);
    load_row(zx, ci0, b, ys + 1, vx, true); put_x(vx, ys + 1);
    load_row(dY, co0, b, ys, vy, false);    put_y(vy);
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int y = ys; y < ye; ++y) {
      // prefetch dY row y + 1 and X row y + 2 while row y's MFMAs run
      if (y + 1 < ye) load_row(dY, co0, b, y + 1, vy, false);
      load_row(zx, ci0, b, y + 2, vx, true);
      const float* xr[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) xr[dy] = sx + r * C::RSX + ((y + dy) % 3) * C::XW;  // row y + dy - 1
#pragma unroll
      for (int m = 0; m < H / 2; ++m) {  // positions x = 2m + h
        const int x = 2 * m + h;
        const float av = sy[r * C::RSY + x];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            acc[dy * 3 + dx] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xr[dy][x + dx], acc[dy * 3 + dx], 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (y + 1 < ye) put_y(vy);
      put_x(vx, y + 2);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
  // acc[t][4q + e] = dW row co0 + 8q + 4h + e, column (ci0 + r) * 9 + t
  wgrad_slice_write<CIN, COUT>(acc, smem, part + chunk * (long)COUT * CIN * 9, co0, ci0);
}

static int wgrad3_ns(long B) { return B >= 2048 ? 1 : B >= 1024 ? 2 : 4; }  // (B x NS waves per layer)

template <int CIN, int COUT, int H>
hipError_t wgrad3(const float* zx, const float* dY, long B, float* dW, float* part, hipStream_t st) {
  using C = Wg3Cfg<CIN, COUT, H>;
  const int ns = wgrad3_ns(B);
  const long chunks = (B * ns + C::NPC - 1) / C::NPC;
  auto go = [&](auto nsc) {
    constexpr int NS = decltype(nsc)::value;
    hipLaunchKernelGGL((k_wgrad3<CIN, COUT, H, NS>), dim3(C::NCO * C::NCI, (unsigned)chunks), dim3(256), 0, st, zx,
                       dY, B, part);
  };
  if (ns == 4) go(std::integral_constant<int, 4>{});
  else if (ns == 2) go(std::integral_constant<int, 2>{});
  else go(std::integral_constant<int, 1>{});
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  GemmArgs g{nullptr, nullptr, dW, COUT, (long)CIN * 9, 0, 0, 0, 0, 0, (long)CIN * 9, 1, 1.f, 0.f};
  hipLaunchKernelGGL(k_splitk_sum, dim3((unsigned)((g.M * g.N + 63) / 64)), dim3(1024), 0, st, g,
                     (int)chunks, part);
  return hipGetLastError();
}

// slices k_wgrad3 writes for layer l (0 if it does not take that layer)
static long wgrad3_slices(int l, long B) {
  const int npc = l == 1 ? Wg3Cfg<32, 32, 32>::NPC : l == 3 ? Wg3Cfg<64, 64, 16>::NPC : l == 5 ? Wg3Cfg<128, 128, 8>::NPC : 0;
  return npc ? (B * wgrad3_ns(B) + npc - 1) / npc : 0;  // one slice per workgroup chunk
}

// ------------------------------------------------------------------------------------------
// forward of a stride-1 3x3 layer (conv1 / conv3 / conv5) on the f32 MFMA, the same streaming as
// k_wgrad3: z[co][b][p] = sum over (ci, tap) of W[co][ci][tap] . X[ci][b][p shifted by tap].  A wave
// owns whole patches; per group of G = 32 / H output rows (32 positions = the MFMA's N) it holds
// all COUT / 32 accumulator blocks, reads the shifted X operand from its LDS ring of G + 2 zero-
// haloed input rows (all CIN channels) and the weights W[co][ci][0..8] straight from L2 (9 taps
// contiguous: three loads per lane per input-channel pair, prefetched one pair ahead).
// ------------------------------------------------------------------------------------------
template <int CIN, int COUT, int H>
struct Fw3Cfg {
  static constexpr int G = 32 / H, R = G + 2;  // output rows per step, ring slots
  static constexpr int XW = H + 2;
  static constexpr int RSX = (R * XW) | 1;     // per-channel ring stride (odd)
  static constexpr int WAVE_F = CIN * RSX;
  static constexpr int NCO = COUT / 32;
  static constexpr int NLD = G * CIN * H / 64;  // floats per lane of one step's new rows
  static_assert(32 % H == 0 && (G * CIN * H) % 64 == 0, "geometry");
};

// NS: each patch's H output rows in NS segments of H / NS, one wave each (its own ring, primed with the
// segment's halo rows) -- small train batches (the reference's 512 pairs: 512 waves for 1,024 SIMDs at NS = 1)
// get NS times the waves; every output keeps its K order, so the result is the same bit for bit
template <int CIN, int COUT, int H, int NS = 1>
__global__ __launch_bounds__(256) void k_fwd3(const float* __restrict__ zx, int relu, const float* __restrict__ W,
                                              long B, float* __restrict__ z) {
  using C = Fw3Cfg<CIN, COUT, H>;
  constexpr int G = C::G, HS = H / NS;
  static_assert(HS % G == 0, "whole steps per segment");
  __shared__ float smem[4 * C::WAVE_F];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  float* sx = smem + w * C::WAVE_F;  // [CIN][R slots][XW] (+pad)
  for (int i = lane; i < C::WAVE_F; i += 64) sx[i] = 0.f;
  __builtin_amdgcn_wave_barrier();
  constexpr int HH = H * H;
  const long u = (long)blockIdx.x * 4 + w;  // one (patch, row segment) per wave
  const long b = u / NS;
  const int ys = (int)(u % NS) * HS, ye = ys + HS;
  if (b >= B) return;
  // input rows y0 .. y0 + G - 1 of all CIN channels (zero outside the patch): lane -> NLD floats
  auto load_rows = [&](int y0, float (&v)[C::NLD]) {
#pragma unroll
    for (int i = 0; i < C::NLD; ++i) {
      const int e = lane * C::NLD + i, c = e / (G * H), rr = (e / H) % G, x = e % H, y = y0 + rr;
      float t = 0.f;
      if (y >= 0 && y < H) t = zx[((long)c * B + b) * HH + y * H + x];
      v[i] = relu ? fmaxf(t, 0.f) : t;
    }
  };
  auto put_rows = [&](int y0, const float (&v)[C::NLD], int ymax) {  // rows y0 .. min(y0 + G - 1, ymax)
#pragma unroll
    for (int i = 0; i < C::NLD; ++i) {
      const int e = lane * C::NLD + i, c = e / (G * H), rr = (e / H) % G, x = e % H, y = y0 + rr;
      if (y <= ymax) sx[c * C::RSX + ((y + 1 + C::R) % C::R) * C::XW + 1 + x] = v[i];
    }
  };
  {  // prologue: rows ys - 1 .. ys + G into the ring
    float v[C::NLD];
    load_rows(ys - 1, v);
    put_rows(ys - 1, v, ys + G);
#pragma unroll 1
    for (int y0 = ys + G - 1; y0 <= ys + G; y0 += G) {
      load_rows(y0, v);
      put_rows(y0, v, ys + G);
    }
  }
  __builtin_amdgcn_wave_barrier();
  // this lane's output position within the step: row rr0 = r / H, column x0 = r % H
  const int rr0 = r / H, x0 = r % H;
  const float* wl = W + (long)r * CIN * 9 + h * 9;  // W[co = cb * 32 + r][ci = 2 j + h][0..8]
  // conv1 (32 -> 32): the lane's whole weight slice (16 channel pairs x 9 taps) stays in registers
  // for the kernel's lifetime, so the K-loop issues no L2 weight loads
  constexpr bool WREG = C::NCO == 1 && CIN / 2 * 9 <= 144;
  float wr[WREG ? CIN / 2 : 1][9];
  if constexpr (WREG) {
#pragma unroll
    for (int j = 0; j < CIN / 2; ++j)
#pragma unroll
      for (int t = 0; t < 9; ++t) wr[j][t] = wl[j * 18 + t];
  }
#pragma unroll 1
  for (int y = ys; y < ye; y += G) {
    float nv[C::NLD];
    if (y + G < ye) load_rows(y + G + 1, nv);  // rows y + G + 1 .. y + 2G (zero past the patch)
    f32x16 acc[C::NCO];
#pragma unroll
    for (int cb = 0; cb < C::NCO; ++cb) acc[cb] = f32x16{};
    if constexpr (WREG) {
#pragma unroll
      for (int j = 0; j < CIN / 2; ++j) {
        const float* xc = sx + (2 * j + h) * C::RSX;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                wr[j][dy * 3 + dx], xc[((y + rr0 + dy - 1 + 1 + C::R) % C::R) * C::XW + x0 + dx], acc[0], 0, 0, 0);
      }
    } else {
    float wc[C::NCO][9], wn[C::NCO][9];
    auto ldw = [&](int j, float (&wv)[C::NCO][9]) {
#pragma unroll
      for (int cb = 0; cb < C::NCO; ++cb)
#pragma unroll
        for (int t = 0; t < 9; ++t) wv[cb][t] = wl[(long)cb * 32 * CIN * 9 + j * 18 + t];
    };
    ldw(0, wc);
#pragma unroll 1
    for (int j = 0; j < CIN / 2; ++j) {
      if (j + 1 < CIN / 2) ldw(j + 1, wn);
      const float* xc = sx + (2 * j + h) * C::RSX;
      float bv[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
          bv[dy * 3 + dx] = xc[((y + rr0 + dy - 1 + 1 + C::R) % C::R) * C::XW + x0 + dx];
#pragma unroll
      for (int cb = 0; cb < C::NCO; ++cb)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][t], bv[t], acc[cb], 0, 0, 0);
      if (j + 1 < CIN / 2) {
#pragma unroll
        for (int cb = 0; cb < C::NCO; ++cb)
#pragma unroll
          for (int t = 0; t < 9; ++t) wc[cb][t] = wn[cb][t];
      }
    }
    }
    // acc[cb][4q + e]: co = 32 cb + 8q + 4h + e, position r of the step -> CNHW
#pragma unroll
    for (int cb = 0; cb < C::NCO; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 32 * cb + 8 * q + 4 * h + e;
          z[((long)co * B + b) * HH + (y + rr0) * H + x0] = acc[cb][4 * q + e];
        }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (y + G < ye) put_rows(y + G + 1, nv, 1 << 30);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// k_fwd3s: k_fwd3 with the ring shared by NWP waves of a workgroup that split the output channels
// (one 32-channel block each) -- 4 / NWP patches per workgroup.  Per patch one ring instead of NWP,
// so conv3 (NWP 2, 37 KB per workgroup) and conv5 (NWP 4, 31 KB) run 4-5 waves per SIMD instead
// of one and the MFMA chains of different waves hide each other's ring and weight loads.
// NS: as k_fwd3's (row segments of H / NS per (patch, segment) unit, 4 / NWP units per workgroup)
template <int CIN, int COUT, int H, int NWP, int NS = 1>
__global__ __launch_bounds__(256) void k_fwd3s(const float* __restrict__ zx, int relu, const float* __restrict__ W,
                                               long B, float* __restrict__ z) {
  using C = Fw3Cfg<CIN, COUT, H>;
  constexpr int G = C::G, PPB = 4 / NWP, NLDT = C::NLD / NWP, HH = H * H, HS = H / NS;
  static_assert(HS % G == 0, "whole steps per segment");
  static_assert(C::NCO == NWP && C::NLD % NWP == 0, "one 32-channel block per wave");
  __shared__ float smem[PPB * C::WAVE_F];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int lp = w / NWP, cb = w % NWP;  // local patch, output-channel block
  float* sx = smem + lp * C::WAVE_F;
  for (int i = threadIdx.x; i < PPB * C::WAVE_F; i += 256) smem[i] = 0.f;
  __syncthreads();
  const long u = (long)blockIdx.x * PPB + lp;
  const long b = u / NS;
  const int ys = (int)(u % NS) * HS, ye = ys + HS;
  const bool valid = b < B;  // no early return: the waves of a workgroup meet at barriers
  auto load_rows = [&](int y0, float (&v)[NLDT]) {  // this wave's share of rows y0 .. y0 + G - 1
#pragma unroll
    for (int i = 0; i < NLDT; ++i) {
      const int e = (cb * 64 + lane) * NLDT + i, c = e / (G * H), rr = (e / H) % G, x = e % H, y = y0 + rr;
      float t = 0.f;
      if (valid && y >= 0 && y < H) t = zx[((long)c * B + b) * HH + y * H + x];
      v[i] = relu ? fmaxf(t, 0.f) : t;
    }
  };
  auto put_rows = [&](int y0, const float (&v)[NLDT], int ymax) {
#pragma unroll
    for (int i = 0; i < NLDT; ++i) {
      const int e = (cb * 64 + lane) * NLDT + i, c = e / (G * H), rr = (e / H) % G, x = e % H, y = y0 + rr;
      if (y <= ymax) sx[c * C::RSX + ((y + 1 + C::R) % C::R) * C::XW + 1 + x] = v[i];
    }
  };
  {
    float v[NLDT];
    load_rows(ys - 1, v);
    put_rows(ys - 1, v, ys + G);
#pragma unroll 1
    for (int y0 = ys + G - 1; y0 <= ys + G; y0 += G) {
      load_rows(y0, v);
      put_rows(y0, v, ys + G);
    }
  }
  __syncthreads();
  const int rr0 = r / H, x0 = r % H;
  const float* wl = W + (long)(cb * 32 + r) * CIN * 9 + h * 9;  // W[co][ci = 2 j + h][0..8]
#pragma unroll 1
  for (int y = ys; y < ye; y += G) {
    float nv[NLDT];
    if (y + G < ye) load_rows(y + G + 1, nv);
    f32x16 acc = f32x16{};
    float wc[9], wn[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wc[t] = wl[t];
#pragma unroll 2
    for (int j = 0; j < CIN / 2; ++j) {
      if (j + 1 < CIN / 2)
#pragma unroll
        for (int t = 0; t < 9; ++t) wn[t] = wl[(j + 1) * 18 + t];
      const float* xc = sx + (2 * j + h) * C::RSX;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(
              wc[dy * 3 + dx], xc[((y + rr0 + dy - 1 + 1 + C::R) % C::R) * C::XW + x0 + dx], acc, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) wc[t] = wn[t];
    }
    if (valid)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 32 * cb + 8 * q + 4 * h + e;
          z[((long)co * B + b) * HH + (y + rr0) * H + x0] = acc[4 * q + e];
        }
    __syncthreads();
    if (y + G < ye) put_rows(y + G + 1, nv, 1 << 30);
    __syncthreads();
  }
}

// row segments per patch: enough (patch, segment) waves for two per SIMD (2,048) at small batches
static int fwd3_ns(long waves) { return waves >= 2048 ? 1 : waves >= 1024 ? 2 : 4; }

template <int CIN, int COUT, int H>
hipError_t fwd3s(const float* zx, bool relu, const float* W, long B, float* z, hipStream_t st) {
  constexpr int NWP = COUT / 32, PPB = 4 / NWP;
  const int ns = std::min(fwd3_ns(B * NWP), H / Fw3Cfg<CIN, COUT, H>::G);
  auto go = [&](auto nsc) {
    constexpr int NS = decltype(nsc)::value;
    hipLaunchKernelGGL((k_fwd3s<CIN, COUT, H, NWP, NS>), dim3((unsigned)((B * NS + PPB - 1) / PPB)), dim3(256), 0, st,
                       zx, relu ? 1 : 0, W, B, z);
  };
  constexpr int NSMAX = H / Fw3Cfg<CIN, COUT, H>::G;  // (whole G-row steps per segment)
  if constexpr (NSMAX >= 4) {
    if (ns >= 4) {
      go(std::integral_constant<int, 4>{});
      return hipGetLastError();
    }
  }
  if constexpr (NSMAX >= 2) {
    if (ns >= 2) {
      go(std::integral_constant<int, 2>{});
      return hipGetLastError();
    }
  }
  go(std::integral_constant<int, 1>{});
  return hipGetLastError();
}

// W'[ci][co][tap] = W[co][ci][8 - tap]: the data gradient of a stride-1 3x3 conv is the same conv
// of dY with these weights
__global__ __launch_bounds__(256) void k_wflip(const float* __restrict__ w, int cout, int cin, float* __restrict__ wf) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)cout * cin * 9) return;
  const int t = (int)(e % 9), ci = (int)((e / 9) % cin), co = (int)(e / (9L * cin));
  wf[((long)ci * cout + co) * 9 + 8 - t] = w[e];
}

template <int CIN, int COUT, int H>
hipError_t fwd3(const float* zx, bool relu, const float* W, long B, float* z, hipStream_t st) {
  const int ns = std::min(fwd3_ns(B), H / Fw3Cfg<CIN, COUT, H>::G);
  auto go = [&](auto nsc) {
    constexpr int NS = decltype(nsc)::value;
    hipLaunchKernelGGL((k_fwd3<CIN, COUT, H, NS>), dim3((unsigned)((B * NS + 3) / 4)), dim3(256), 0, st, zx,
                       relu ? 1 : 0, W, B, z);
  };
  constexpr int NSMAX = H / Fw3Cfg<CIN, COUT, H>::G;  // (whole G-row steps per segment)
  if constexpr (NSMAX >= 4) {
    if (ns >= 4) {
      go(std::integral_constant<int, 4>{});
      return hipGetLastError();
    }
  }
  if constexpr (NSMAX >= 2) {
    if (ns >= 2) {
      go(std::integral_constant<int, 2>{});
      return hipGetLastError();
    }
  }
  go(std::integral_constant<int, 1>{});
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// the stride-2 3x3 pad-1 layers (conv2: 32 -> 64 at 32 -> 16, conv4: 64 -> 128 at 16 -> 8), the same
// per-wave LDS streaming on the f32 MFMA as the stride-1 kernels above.
//
// k_fwd2: forward.  Output rows y .. y + G - 1 (G = 32 / HO: 32 positions = the MFMA's N) read
// input rows 2y - 1 .. 2y + 2G - 1 from a ring of R = 2G + 1 rows of all CIN channels (column 0 is
// the zero pad at x = -1, the ring starts zeroed, so row -1 is the zero pad too); each step loads
// the next 2G rows while its MFMAs run.
// ------------------------------------------------------------------------------------------
template <int CIN, int COUT, int HI>
struct Fw2Cfg {
  static constexpr int HO = HI / 2, G = 32 / HO, R = 2 * G + 1;
  static constexpr int XW = HI + 1;
  static constexpr int RSX = (R * XW) | 1;
  static constexpr int WAVE_F = CIN * RSX;
  static constexpr int NCO = COUT / 32;
  static constexpr int NLD = 2 * G * CIN * HI / 64;  // floats per lane of one step's 2G new rows
  static_assert(32 % HO == 0 && (2 * G * CIN * HI) % 64 == 0 && HO >= G, "geometry");
};

// NWP waves share one patch's ring and split its output-channel blocks (NWP > 1: 4 / NWP patches
// per workgroup, workgroup barriers; NWP = 1: one patch per wave, wave barriers).
// NS: output rows in NS segments of HO / NS per (patch, segment) unit (k_fwd3's small-batch split)
template <int CIN, int COUT, int HI, int NWP, int NS = 1>
__global__ __launch_bounds__(256) void k_fwd2(const float* __restrict__ zx, int relu, const float* __restrict__ W,
                                              long B, float* __restrict__ z) {
  using C = Fw2Cfg<CIN, COUT, HI>;
  constexpr int G = C::G, HO = C::HO, HHI = HI * HI, PPB = 4 / NWP, CPW = C::NCO / NWP, NLDT = C::NLD / NWP;
  constexpr int HS = HO / NS;
  static_assert(HS % G == 0, "whole steps per segment");
  static_assert(C::NCO % NWP == 0 && C::NLD % NWP == 0, "split");
  __shared__ float smem[PPB * C::WAVE_F];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int lp = w / NWP, wp = w % NWP;
  float* sx = smem + lp * C::WAVE_F;  // [CIN][R slots][XW] (+pad); input row k in slot (k + 1) % R
  auto sync = [&] {
    if constexpr (NWP > 1) __syncthreads();
    else {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  };
  for (int i = (NWP > 1 ? threadIdx.x : lane); i < (NWP > 1 ? PPB : 1) * C::WAVE_F; i += (NWP > 1 ? 256 : 64))
    (NWP > 1 ? smem : sx)[i] = 0.f;
  sync();
  const long u = (long)blockIdx.x * PPB + lp;
  const long b = u / NS;
  const int ys = (int)(u % NS) * HS, ye = ys + HS;
  const bool valid = b < B;
  if (NWP == 1 && !valid) return;
  auto load_rows = [&](int y0, float (&v)[NLDT]) {  // this wave's share of input rows y0 .. y0 + 2G - 1
#pragma unroll
    for (int i = 0; i < NLDT; ++i) {
      const int e = (wp * 64 + lane) * NLDT + i, c = e / (2 * G * HI), rr = (e / HI) % (2 * G), x = e % HI;
      const int y = y0 + rr;
      const float t = valid && y >= 0 && y < HI ? zx[((long)c * B + b) * HHI + y * HI + x] : 0.f;
      v[i] = relu ? fmaxf(t, 0.f) : t;
    }
  };
  auto put_rows = [&](int y0, const float (&v)[NLDT], int ymax) {
#pragma unroll
    for (int i = 0; i < NLDT; ++i) {
      const int e = (wp * 64 + lane) * NLDT + i, c = e / (2 * G * HI), rr = (e / HI) % (2 * G), x = e % HI;
      if (y0 + rr <= ymax) sx[c * C::RSX + ((y0 + rr + 1 + C::R) % C::R) * C::XW + 1 + x] = v[i];
    }
  };
  {  // prologue: input rows 2 ys - 1 .. 2 ys + 2G - 1 (row -1: the zero pad)
    float v[NLDT];
    load_rows(2 * ys - 1, v);
    put_rows(2 * ys - 1, v, 2 * ys + 2 * G - 1);
    load_rows(2 * ys + 2 * G - 1, v);
    put_rows(2 * ys + 2 * G - 1, v, 2 * ys + 2 * G - 1);
  }
  sync();
  const int rr0 = r / HO, x0 = r % HO;
  const float* wl = W + (long)(wp * CPW * 32 + r) * CIN * 9 + h * 9;  // W[co = (wp CPW + cb) 32 + r][ci = 2 j + h]
#pragma unroll 1
  for (int y = ys; y < ye; y += G) {
    float nv[NLDT];
    if (y + G < ye) load_rows(2 * (y + G), nv);
    f32x16 acc[CPW];
#pragma unroll
    for (int cb = 0; cb < CPW; ++cb) acc[cb] = f32x16{};
    float wc[CPW][9], wn[CPW][9];
    auto ldw = [&](int j, float (&wv)[CPW][9]) {
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
        for (int t = 0; t < 9; ++t) wv[cb][t] = wl[(long)cb * 32 * CIN * 9 + j * 18 + t];
    };
    // the 9 shifted operands of channel pair j: input row 2 (y + rr0) + dy - 1 -> slot (2 (y + rr0) + dy) % R;
    // read one pair ahead so the MFMA chain does not wait on the LDS latency
    auto ldb = [&](int j, float (&bv)[9]) {
      const float* xc = sx + (2 * j + h) * C::RSX;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) bv[dy * 3 + dx] = xc[((2 * (y + rr0) + dy) % C::R) * C::XW + 2 * x0 + dx];
    };
    float bv[9], bn[9];
    ldw(0, wc);
    ldb(0, bv);
#pragma unroll 1
    for (int j = 0; j < CIN / 2; ++j) {
      if (j + 1 < CIN / 2) {
        ldw(j + 1, wn);
        ldb(j + 1, bn);
      }
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][t], bv[t], acc[cb], 0, 0, 0);
      if (j + 1 < CIN / 2) {
#pragma unroll
        for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
          for (int t = 0; t < 9; ++t) wc[cb][t] = wn[cb][t];
#pragma unroll
        for (int t = 0; t < 9; ++t) bv[t] = bn[t];
      }
    }
    if (valid)
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int co = 32 * (wp * CPW + cb) + 8 * q + 4 * h + e;
            z[((long)co * B + b) * (HO * HO) + (y + rr0) * HO + x0] = acc[cb][4 * q + e];
          }
    sync();
    if (y + G < ye) put_rows(2 * (y + G), nv, 1 << 30);
    sync();
  }
}

// (patch, row segment) units: B NS waves x NWP (shared rings) reach two per SIMD at small batches
template <int HS, int G, class F>
static void launch_ns(int ns, F&& go) {
  if constexpr (HS / G >= 4) {
    if (ns >= 4) return go(std::integral_constant<int, 4>{});
  }
  if constexpr (HS / G >= 2) {
    if (ns >= 2) return go(std::integral_constant<int, 2>{});
  }
  go(std::integral_constant<int, 1>{});
}

template <int CIN, int COUT, int HI, int NWP = (COUT / 32 >= 4 ? 4 : COUT / 32)>
hipError_t fwd2(const float* zx, bool relu, const float* W, long B, float* z, hipStream_t st, bool shared) {
  using C = Fw2Cfg<CIN, COUT, HI>;
  const int nwp = shared ? NWP : 1;
  launch_ns<C::HO, C::G>(fwd3_ns(B * nwp), [&](auto nsc) {
    constexpr int NS = decltype(nsc)::value;
    if (shared)
      hipLaunchKernelGGL((k_fwd2<CIN, COUT, HI, NWP, NS>), dim3((unsigned)((B * NS + 4 / NWP - 1) / (4 / NWP))),
                         dim3(256), 0, st, zx, relu ? 1 : 0, W, B, z);
    else
      hipLaunchKernelGGL((k_fwd2<CIN, COUT, HI, 1, NS>), dim3((unsigned)((B * NS + 3) / 4)), dim3(256), 0, st, zx,
                         relu ? 1 : 0, W, B, z);
  });
  return hipGetLastError();
}

// k_dgrad2: data gradient, without the 3 of 4 zero taps of the transposed conv.  Input pixel
// (2m + py, 2n + px) of channel ci collects W[co][ci][ky][kx] . dY[co][m + (ky == 0)][n + (kx == 0)]
// over its parity class's taps (py = 0: ky = 1; py = 1: ky = 2 at m and ky = 0 at m + 1; the same
// in x): 1 + 2 + 2 + 4 = 9 MFMAs per output-channel pair for the four pixels of a 2x2 cell.  A wave
// owns whole patches; per step of G = 32 / HO cell rows it reads dY rows m .. m + G of all CO
// channels from its LDS ring (row HO and column HO are zero) and W[co][ci][0..8] from L2 (no flip),
// and stores each cell row pair (px = 0, 1) as one float2.
template <int CO, int CI, int HO>
struct Dg2Cfg {
  static constexpr int G = 32 / HO, R = G + 1, XW = HO + 1;
  static constexpr int RSX = (R * XW) | 1;
  static constexpr int WAVE_F = CO * RSX;
  static constexpr int NCI = CI / 32;
  static constexpr int NLD = G * CO * HO / 64;
  static_assert(32 % HO == 0 && (G * CO * HO) % 64 == 0 && HO >= G, "geometry");
};

template <int CO, int CI, int HO, int NWP, int NS = 1>
__global__ __launch_bounds__(256) void k_dgrad2(const float* __restrict__ dY, const float* __restrict__ W, long B,
                                                float* __restrict__ din) {
  using C = Dg2Cfg<CO, CI, HO>;
  constexpr int G = C::G, HI = 2 * HO, HH = HO * HO, PPB = 4 / NWP, CPW = C::NCI / NWP, NLDT = C::NLD / NWP;
  constexpr int HS = HO / NS;  // cell rows per (patch, segment) unit
  static_assert(HS % G == 0, "whole steps per segment");
  static_assert(C::NCI % NWP == 0 && C::NLD % NWP == 0, "split");
  __shared__ float smem[PPB * C::WAVE_F];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int lp = w / NWP, wp = w % NWP;  // local patch, this wave's share of the input-channel blocks
  float* sx = smem + lp * C::WAVE_F;  // [CO][R slots][XW]; dY row k in slot k % R
  auto sync = [&] {
    if constexpr (NWP > 1) __syncthreads();
    else {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  };
  for (int i = (NWP > 1 ? threadIdx.x : lane); i < (NWP > 1 ? PPB : 1) * C::WAVE_F; i += (NWP > 1 ? 256 : 64))
    (NWP > 1 ? smem : sx)[i] = 0.f;
  sync();
  const long u = (long)blockIdx.x * PPB + lp;
  const long b = u / NS;
  const int ys = (int)(u % NS) * HS, ye = ys + HS;
  const bool valid = b < B;
  if (NWP == 1 && !valid) return;
  auto load_rows = [&](int y0, float (&v)[NLDT]) {  // dY rows y0 .. y0 + G - 1 (zero past the patch)
#pragma unroll
    for (int i = 0; i < NLDT; ++i) {
      const int e = (wp * 64 + lane) * NLDT + i, c = e / (G * HO), rr = (e / HO) % G, x = e % HO, y = y0 + rr;
      v[i] = valid && y < HO ? dY[((long)c * B + b) * HH + y * HO + x] : 0.f;
    }
  };
  auto put_rows = [&](int y0, const float (&v)[NLDT], int ymax) {
#pragma unroll
    for (int i = 0; i < NLDT; ++i) {
      const int e = (wp * 64 + lane) * NLDT + i, c = e / (G * HO), rr = (e / HO) % G, x = e % HO, y = y0 + rr;
      if (y <= ymax) sx[c * C::RSX + (y % C::R) * C::XW + x] = v[i];
    }
  };
  {  // prologue: rows ys .. ys + G
    float v[NLDT];
    load_rows(ys, v);
    put_rows(ys, v, ys + G);
    load_rows(ys + G, v);
    put_rows(ys + G, v, ys + G);
  }
  sync();
  const int rr0 = r / HO, n0 = r % HO;
  const float* wl = W + ((long)h * CI + wp * CPW * 32 + r) * 9;  // W[co = 2 j + h][ci = (wp CPW + cb) 32 + r]
#pragma unroll 1
  for (int y = ys; y < ye; y += G) {
    float nv[NLDT];
    if (y + G < ye) load_rows(y + G + 1, nv);
    f32x16 acc[4][CPW];  // [2 py + px][ci block]
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb) acc[k][cb] = f32x16{};
    float wc[CPW][9], wn[CPW][9];
    auto ldw = [&](int j, float (&wv)[CPW][9]) {
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
        for (int t = 0; t < 9; ++t) wv[cb][t] = wl[(long)j * 2 * CI * 9 + cb * 32 * 9 + t];
    };
    ldw(0, wc);
#pragma unroll 1
    for (int j = 0; j < CO / 2; ++j) {
      if (j + 1 < CO / 2) ldw(j + 1, wn);
      const float* xc = sx + (2 * j + h) * C::RSX;
      const int s0 = ((y + rr0) % C::R) * C::XW + n0, s1 = ((y + rr0 + 1) % C::R) * C::XW + n0;
      const float b00 = xc[s0], b01 = xc[s0 + 1], b10 = xc[s1], b11 = xc[s1 + 1];
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb) {
        acc[0][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][4], b00, acc[0][cb], 0, 0, 0);
        acc[1][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][5], b00, acc[1][cb], 0, 0, 0);
        acc[2][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][7], b00, acc[2][cb], 0, 0, 0);
        acc[3][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][8], b00, acc[3][cb], 0, 0, 0);
        acc[1][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][3], b01, acc[1][cb], 0, 0, 0);
        acc[3][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][6], b01, acc[3][cb], 0, 0, 0);
        acc[2][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][1], b10, acc[2][cb], 0, 0, 0);
        acc[3][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][2], b10, acc[3][cb], 0, 0, 0);
        acc[3][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[cb][0], b11, acc[3][cb], 0, 0, 0);
      }
      if (j + 1 < CO / 2) {
#pragma unroll
        for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
          for (int t = 0; t < 9; ++t) wc[cb][t] = wn[cb][t];
      }
    }
    // acc[2 py + px][cb][4q + e]: ci = 32 cb + 8q + 4h + e, input pixel (2 (y + rr0) + py, 2 n0 + px)
    if (valid)
#pragma unroll
    for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ci = 32 * (wp * CPW + cb) + 8 * q + 4 * h + e;
          float* o = din + ((long)ci * B + b) * (HI * HI) + 2 * (y + rr0) * HI + 2 * n0;
#pragma unroll
          for (int py = 0; py < 2; ++py)
            *reinterpret_cast<float2*>(o + py * HI) = make_float2(acc[2 * py][cb][4 * q + e], acc[2 * py + 1][cb][4 * q + e]);
        }
    sync();
    if (y + G < ye) put_rows(y + G + 1, nv, 1 << 30);
    sync();
  }
}

template <int CO, int CI, int HO>
hipError_t dgrad2(const float* dY, const float* W, long B, float* din, hipStream_t st, bool shared) {
  constexpr int NWP = CI / 32 >= 4 ? 4 : CI / 32;
  using C = Dg2Cfg<CO, CI, HO>;
  const bool sh = shared && NWP > 1;
  launch_ns<HO, C::G>(fwd3_ns(B * (sh ? NWP : 1)), [&](auto nsc) {
    constexpr int NS = decltype(nsc)::value;
    if (sh)
      hipLaunchKernelGGL((k_dgrad2<CO, CI, HO, NWP, NS>), dim3((unsigned)((B * NS + 4 / NWP - 1) / (4 / NWP))),
                         dim3(256), 0, st, dY, W, B, din);
    else
      hipLaunchKernelGGL((k_dgrad2<CO, CI, HO, 1, NS>), dim3((unsigned)((B * NS + 3) / 4)), dim3(256), 0, st, dY, W, B,
                         din);
  });
  return hipGetLastError();
}

// k_wgrad2: weight gradient, k_wgrad3's streaming with the stride: per output row y the wave holds
// the dY row and X rows 2y - 1, 2y, 2y + 1 (ring of 3, column 0 = the zero pad at x = -1), so tap
// (dy, dx) of position x is the ds_read at column 2x + dx.  Chunk = 2048 / HO^2 patches (>= 4).
template <int CIN, int COUT, int HO>
struct Wg2Cfg {
  static constexpr int HI = 2 * HO;
  static constexpr int NPC = 2048 / (HO * HO) >= 4 ? 2048 / (HO * HO) : 4;
  static constexpr int NPW = NPC / 4;
  static constexpr int RSY = HO + 1;
  static constexpr int XW = HI + 1;
  static constexpr int RSX = (3 * XW) | 1;
  static constexpr int WAVE_F = 32 * RSY + 32 * RSX;
  static constexpr int NCO = COUT / 32, NCI = CIN / 32;
  static constexpr int NPY = 32 * HO / 64, NPX = 32 * HI / 64;  // floats per lane of a dY / X row
  static_assert(NPY >= 1 && NPC % 4 == 0 && HO % 2 == 0, "geometry");
};

template <int CIN, int COUT, int HO, int NS = 1>
__global__ __launch_bounds__(256) void k_wgrad2(const float* __restrict__ zx, const float* __restrict__ dY, long B,
                                                float* __restrict__ part) {
  using C = Wg2Cfg<CIN, COUT, HO>;
  constexpr int HI = C::HI, HS = HO / NS;  // (output rows per (patch, segment) unit)
  static_assert(4 * C::WAVE_F >= 4 * 16 * 64, "the slice reduction's round fits the rings");
  __shared__ float smem[4 * C::WAVE_F];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int blk = blockIdx.x, co0 = (blk / C::NCI) * 32, ci0 = (blk % C::NCI) * 32;
  const long chunk = blockIdx.y;
  float* sy = smem + w * C::WAVE_F;  // [32 co][RSY]
  float* sx = sy + 32 * C::RSY;      // [32 ci][3 slots][XW]; X row k in slot (k + 1) % 3
  for (int i = lane; i < 32 * C::RSX; i += 64) sx[i] = 0.f;
  __builtin_amdgcn_wave_barrier();
  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x16{};
  auto load_y = [&](long b, int y, float (&v)[C::NPY]) {
#pragma unroll
    for (int i = 0; i < C::NPY; ++i) {
      const int e = lane * C::NPY + i, c = e / HO, x = e % HO;
      v[i] = dY[((long)(co0 + c) * B + b) * (HO * HO) + y * HO + x];
    }
  };
  auto put_y = [&](const float (&v)[C::NPY]) {
#pragma unroll
    for (int i = 0; i < C::NPY; ++i) {
      const int e = lane * C::NPY + i, c = e / HO, x = e % HO;
      sy[c * C::RSY + x] = v[i];
    }
  };
  auto load_x = [&](long b, int y, float (&v)[C::NPX]) {  // relu(X) row y (0 .. HI - 1)
#pragma unroll
    for (int i = 0; i < C::NPX; ++i) {
      const int e = lane * C::NPX + i, c = e / HI, x = e % HI;
      v[i] = fmaxf(zx[((long)(ci0 + c) * B + b) * (HI * HI) + y * HI + x], 0.f);
    }
  };
  auto put_x = [&](const float (&v)[C::NPX], int y) {
    const int slot = (y + 1) % 3;
#pragma unroll
    for (int i = 0; i < C::NPX; ++i) {
      const int e = lane * C::NPX + i, c = e / HI, x = e % HI;
      sx[c * C::RSX + slot * C::XW + 1 + x] = v[i];
    }
  };
#pragma unroll 1
  for (int pi = 0; pi < C::NPW; ++pi) {
    const long u = chunk * C::NPC + w + 4 * pi;
    const long b = u / NS;
    if (b >= B) break;  // wave-uniform
    const int ys = (int)(u % NS) * HS, ye = ys + HS;
    float vy[C::NPY], va[C::NPX], vb[C::NPX];
    // prologue: X row 2 ys - 1 (zeros for ys = 0: the pad), rows 2 ys and 2 ys + 1, dY row ys
    if (ys == 0) {
      for (int i = 0; i < C::NPX; ++i) va[i] = 0.f;
    } else {
      load_x(b, 2 * ys - 1, va);
    }
    put_x(va, 2 * ys - 1);
    load_x(b, 2 * ys, va); put_x(va, 2 * ys);
    load_x(b, 2 * ys + 1, va); put_x(va, 2 * ys + 1);
    load_y(b, ys, vy); put_y(vy);
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int y = ys; y < ye; ++y) {
      const bool more = y + 1 < ye;  // prefetch dY row y + 1 and X rows 2y + 2, 2y + 3
      if (more) {
        load_y(b, y + 1, vy);
        load_x(b, 2 * y + 2, va);
        load_x(b, 2 * y + 3, vb);
      }
      const float* xr[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) xr[dy] = sx + r * C::RSX + ((2 * y + dy) % 3) * C::XW;  // X row 2y + dy - 1
#pragma unroll
      for (int m = 0; m < HO / 2; ++m) {  // positions x = 2m + h
        const int x = 2 * m + h;
        const float av = sy[r * C::RSY + x];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            acc[dy * 3 + dx] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xr[dy][2 * x + dx], acc[dy * 3 + dx], 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (more) {
        put_y(vy);
        put_x(va, 2 * y + 2);
        put_x(vb, 2 * y + 3);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
  wgrad_slice_write<CIN, COUT>(acc, smem, part + chunk * (long)COUT * CIN * 9, co0, ci0);
}

template <int CIN, int COUT, int HO>
hipError_t wgrad2(const float* zx, const float* dY, long B, float* dW, float* part, hipStream_t st) {
  using C = Wg2Cfg<CIN, COUT, HO>;
  const int ns = wgrad3_ns(B);
  const long chunks = (B * ns + C::NPC - 1) / C::NPC;
  auto go = [&](auto nsc) {
    constexpr int NS = decltype(nsc)::value;
    hipLaunchKernelGGL((k_wgrad2<CIN, COUT, HO, NS>), dim3(C::NCO * C::NCI, (unsigned)chunks), dim3(256), 0, st, zx,
                       dY, B, part);
  };
  if (ns == 4) go(std::integral_constant<int, 4>{});
  else if (ns == 2) go(std::integral_constant<int, 2>{});
  else go(std::integral_constant<int, 1>{});
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  GemmArgs g{nullptr, nullptr, dW, COUT, (long)CIN * 9, 0, 0, 0, 0, 0, (long)CIN * 9, 1, 1.f, 0.f};
  hipLaunchKernelGGL(k_splitk_sum, dim3((unsigned)((g.M * g.N + 63) / 64)), dim3(1024), 0, st, g,
                     (int)chunks, part);
  return hipGetLastError();
}


static long wgrad2_slices(int l, long B) {
  const int npc = l == 2 ? Wg2Cfg<32, 64, 16>::NPC : l == 4 ? Wg2Cfg<64, 128, 8>::NPC : 0;
  return npc ? (B * wgrad3_ns(B) + npc - 1) / npc : 0;  // one slice per workgroup chunk
}

// implicit-im2col convs of one layer (compile-time geometry): the forward Y = W . col and the
// weight gradient dW = dY . col^T over the whole batch, with no column matrix in memory
template <int C, int H, int KS, int S, int PAD>
hipError_t conv_fwd(const ActIn& a, long B, const float* W, int cout, float* z, float* part, hipStream_t st) {
  using L = Im2colB<C, H, KS, S, PAD, false>;
  const long n = B * L::HWO, K = (long)C * KS * KS;
  GemmArgs g{W, nullptr, z, cout, n, K, K, 1, 2, 1, n, 1, 1.f, 0.f};  // B contiguous along N
  return gemm(g, st, part, L{a, B});
}
// dX [C][B H H] = Wt [C][COUT KK] . col2im-gather(dY), Wt transposed into `wt` first
template <int C, int H, int KS, int S, int PAD>
hipError_t conv_dgrad(const float* dY, long B, const float* W, int cout, float* wt, float* dX, hipStream_t st) {
  constexpr int KK = KS * KS;
  const long nw = (long)cout * C * KK;
  hipLaunchKernelGGL(k_wt, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, W, cout, C, KK, wt);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long n = B * H * H, K = (long)cout * KK;
  GemmArgs g{wt, nullptr, dX, C, n, K, K, 1, 2, 1, n, 1, 1.f, 0.f};
  if (cout == 32)
    return gemm(g, st, nullptr, Col2imB<32, H, KS, S, PAD>{dY, B});
  if (cout == 64)
    return gemm(g, st, nullptr, Col2imB<64, H, KS, S, PAD>{dY, B});
  return gemm(g, st, nullptr, Col2imB<128, H, KS, S, PAD>{dY, B});
}
template <int C, int H, int KS, int S, int PAD>
hipError_t conv_wgrad(const ActIn& a, long B, const float* dY, int cout, float* dW, float* part, hipStream_t st) {
  using L = Im2colB<C, H, KS, S, PAD, true>;
  const long n = B * L::HWO, K = (long)C * KS * KS;
  GemmArgs g{dY, nullptr, dW, cout, K, n, n, 1, 1, 2, K, 1, 1.f, 0.f};  // B contiguous along K (= pos)
  return gemm(g, st, part, L{a, B});
}
#define HN_TRAIN_LAYERS(X) \
  X(0, 1, 32, 3, 1, 1) X(1, 32, 32, 3, 1, 1) X(2, 32, 32, 3, 2, 1) X(3, 64, 16, 3, 1, 1) X(4, 64, 16, 3, 2, 1) \
  X(5, 128, 8, 3, 1, 1) X(6, 128, 8, 8, 1, 0)
hipError_t conv_fwd_l(int l, const ActIn& a, long B, const float* W, int cout, float* z, float* part,
                      hipStream_t st) {
#define HN_F(L_, C, H, KS, S, PAD) \
  if (l == L_) return conv_fwd<C, H, KS, S, PAD>(a, B, W, cout, z, part, st);
  HN_TRAIN_LAYERS(HN_F)
#undef HN_F
  return hipErrorInvalidValue;
}
hipError_t conv_wgrad_l(int l, const ActIn& a, long B, const float* dY, int cout, float* dW, float* part,
                        hipStream_t st) {
#define HN_W(L_, C, H, KS, S, PAD) \
  if (l == L_) return conv_wgrad<C, H, KS, S, PAD>(a, B, dY, cout, dW, part, st);
  HN_TRAIN_LAYERS(HN_W)
#undef HN_W
  return hipErrorInvalidValue;
}
hipError_t conv_dgrad_l(int l, const float* dY, long B, const float* W, int cout, float* wt, float* dX,
                        hipStream_t st) {
#define HN_D(L_, C, H, KS, S, PAD) \
  if (l == L_) return conv_dgrad<C, H, KS, S, PAD>(dY, B, W, cout, wt, dX, st);
  HN_TRAIN_LAYERS(HN_D)
#undef HN_D
  return hipErrorInvalidValue;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
const HnTrainLayer kHardnetTrainLayers[7] = {
    // cin, cout, hin, ks, s, pad
    {1, 32, 32, 3, 1, 1},   {32, 32, 32, 3, 1, 1}, {32, 64, 32, 3, 2, 1}, {64, 64, 16, 3, 1, 1},
    {64, 128, 16, 3, 2, 1}, {128, 128, 8, 3, 1, 1}, {128, 128, 8, 8, 1, 0}};

static long hout_of(const HnTrainLayer& l) { return (l.hin + 2 * l.pad - l.ks) / l.s + 1; }

// patches per dgrad column chunk: col = K x (n Ho Wo) floats within kColBudget
static constexpr size_t kColBudget = (size_t)256 << 20;
static long chunk_of(const HnTrainLayer& l, long B) {
  const long ho = hout_of(l);
  const size_t per = (size_t)l.cin * l.ks * l.ks * ho * ho * sizeof(float);
  return std::max<long>(1, std::min<long>(B, (long)(kColBudget / per)));
}

HnTrainWs hn_train_layout(long B) {
  // Two regions.  "saved" holds what the backward reads (one per forward call: autograd keeps it
  // until the backward has run); "scratch" is transient (the caller may reuse it between calls).
  HnTrainWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) / 256 * 256;
    return o;
  };
  w.xn = take((size_t)B * 1024 * 4);
  w.inv_sd = take((size_t)B * 4);
  size_t maxact = (size_t)B * 1024;
  for (int l = 0; l < 7; ++l) {
    const long ho = hout_of(kHardnetTrainLayers[l]);
    w.z[l] = take((size_t)kHardnetTrainLayers[l].cout * B * ho * ho * 4);
    w.rstd[l] = take((size_t)kHardnetTrainLayers[l].cout * 4);
    maxact = std::max(maxact, (size_t)kHardnetTrainLayers[l].cout * B * ho * ho);
  }
  w.saved_total = off;
  off = 0;  // scratch offsets
  w.g0 = take(maxact * 4);
  w.g1 = take(maxact * 4);
  size_t col = 0;  // the strided / 8x8 dgrads' column chunk
  for (int l = 0; l < 7; ++l) {
    const HnTrainLayer& L = kHardnetTrainLayers[l];
    if (L.s == 1 && L.ks == 3) continue;
    const long ho = hout_of(L);
    col = std::max(col, (size_t)L.cin * L.ks * L.ks * chunk_of(L, B) * ho * ho * 4);
  }
  w.col = take(col);
  size_t part = 0;  // split-K partials of the weight gradients (one GEMM over the whole batch)
  for (int l = 0; l < 7; ++l) {
    const HnTrainLayer& L = kHardnetTrainLayers[l];
    const long ho = hout_of(L), kk = B * ho * ho;
    part = std::max(part, (size_t)L.cout * L.cin * L.ks * L.ks * ((kk + hn_knobs().train_splitk - 1) / hn_knobs().train_splitk) * 4);
  }
  part = std::max(part, (size_t)512 * GBM * GBN * 4);  // small-grid forward splits (S <= ceil(256 / tiles))
  part = std::max(part, (size_t)32 * 9 * wgrad0_slices(B) * 4);  // k_wgrad0's slices
  for (int l = 1; l <= 5; ++l) {  // k_wgrad3's / k_wgrad2's slices
    const HnTrainLayer& L = kHardnetTrainLayers[l];
    part = std::max(part, (size_t)L.cout * L.cin * 9 * (wgrad3_slices(l, B) + wgrad2_slices(l, B)) * 4);
  }
  w.part = take(part);
  w.bnpart = take((size_t)128 * kBnSlices * 2 * sizeof(double));
  w.wt = take((size_t)128 * 128 * 64 * sizeof(float));  // a transposed weight (conv6 is the largest)
  w.bnmean = take((size_t)2 * 128 * sizeof(float));
  // the bf16x3 conv path (HN_TRAIN_F32 bit 0 or 1 off): NHWC in / out (the largest activation:
  // 32 x 32 x 32 per patch), one packed layer (conv5: 128 x 128 x 9 x 2 bf16 pairs), a zero bias
  const bool bf16x3 = (hn_knobs().train_f32 & 3) != 3;
  w.nhwc0 = take(bf16x3 ? (size_t)B * 32 * 1024 * 4 : 0);
  w.nhwc1 = take(bf16x3 ? (size_t)B * 32 * 1024 * 4 : 0);
  w.wpack = take(bf16x3 ? (size_t)128 * 128 * 9 * 2 * 2 * 2 : 0);
  w.zero = take(128 * sizeof(float));
  w.scratch_total = off;
  return w;
}

#define HCK(x)                        \
  do {                                \
    hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return e_;  \
  } while (0)

// conv layer l (1..5) as the inference kernels' bf16x3 MFMA conv over NHWC: CNHW `x` (relu'd if
// asked) -> NHWC -> conv (flip: the data gradient, input = the conv's output space) -> CNHW `y`
static hipError_t conv_bf16x3(int l, bool flip, const float* x, bool relu, long B, const float* W, float* y,
                              char* sc, const HnTrainWs& L, hipStream_t st) {
  const HnTrainLayer& S = kHardnetTrainLayers[l];
  const long ho = hout_of(S);
  const int cin = flip ? S.cout : S.cin, cout = flip ? S.cin : S.cout;
  const int hin = flip ? (int)ho : S.hin, hout = flip ? S.hin : (int)ho;
  float* a = reinterpret_cast<float*>(sc + L.nhwc0);
  float* o = reinterpret_cast<float*>(sc + L.nhwc1);
  unsigned short* wp = reinterpret_cast<unsigned short*>(sc + L.wpack);
  hipLaunchKernelGGL(k_cnhw_to_nhwc, dim3(hin * hin / 64, (unsigned)B), dim3(256), 0, st, x, cin, B, hin * hin,
                     relu ? 1 : 0, a);
  hipLaunchKernelGGL(k_pack3x3, dim3((S.cin * S.cout * 9 + 255) / 256), dim3(256), 0, st, W, S.cin, S.cout,
                     flip ? 1 : 0, wp);
  HCK(hipGetLastError());
  HCK(hn_launch_conv_raw(l, wp, reinterpret_cast<const float*>(sc + L.zero), a, o, (int)B, st));
  hipLaunchKernelGGL(k_nhwc_to_cnhw, dim3(hout * hout / 64, (unsigned)B), dim3(256), 0, st, o, cout, B,
                     hout * hout, y);
  return hipGetLastError();
}

hipError_t hn_train_forward(const float* in, long B, const float* const* W, float* const* rmean, float* const* rvar,
                            float mom, float bn_eps, float in_eps, float l2_eps, float drop_p,
                            unsigned long long seed, float* out, char* sv, char* sc, hipStream_t st) {
  const HnTrainWs L = hn_train_layout(B);
  HCK(hipMemsetAsync(sc + L.zero, 0, 128 * sizeof(float), st));  // the bf16x3 convs' zero bias
  float* xn = reinterpret_cast<float*>(sv + L.xn);
  hipLaunchKernelGGL(k_input_norm, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, in, B, in_eps, xn,
                     reinterpret_cast<float*>(sv + L.inv_sd));
  HCK(hipGetLastError());
  for (int l = 0; l < 7; ++l) {
    const HnTrainLayer& S = kHardnetTrainLayers[l];
    const long ho = hout_of(S), hw = ho * ho;
    // this layer's input: the normalised patch, or relu(z) of the previous layer (x the dropout
    // mask before conv6, HardNet.py:299)
    const ActIn a{l == 0 ? xn : reinterpret_cast<const float*>(sv + L.z[l - 1]), l > 0 ? 1 : 0,
                  l == 6 ? drop_p : 0.f, seed};
    float* z = reinterpret_cast<float*>(sv + L.z[l]);
    const int tf = hn_knobs().train_f32;
    if (l == 0 && !(tf & 64)) {  // conv0: k_fwd0 (taps as the MFMA's K)
      hipLaunchKernelGGL(k_fwd0, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, xn, W[0], B, z);
      HCK(hipGetLastError());
    } else if (l >= 1 && l <= 5 && !(tf & 1))  // conv1..5: the bf16x3 MFMA conv kernels
      HCK(conv_bf16x3(l, false, a.z, true, B, W[l], z, sc, L, st));
    else if ((l == 1 || l == 3 || l == 5) && !(tf & 8)) {  // stride-1 3x3: k_fwd3 (f32 MFMA)
      if (l == 1) HCK((fwd3<32, 32, 32>(a.z, true, W[l], B, z, st)));
      const bool sh = !(tf & 128);  // conv3 / conv5: the shared-ring form
      if (l == 3) HCK((sh ? fwd3s<64, 64, 16> : fwd3<64, 64, 16>)(a.z, true, W[l], B, z, st));
      if (l == 5) HCK((sh ? fwd3s<128, 128, 8> : fwd3<128, 128, 8>)(a.z, true, W[l], B, z, st));
    } else if ((l == 2 || l == 4) && !(tf & 32)) {  // stride-2 3x3: k_fwd2 (f32 MFMA)
      // conv2: one ring per wave (shared by 2 waves measured 0.64 vs 0.31 ms); conv4: one ring per two
      // waves (one per wave needs 128 prefetch registers per lane and spills)
      if (l == 2) HCK((fwd2<32, 64, 32>(a.z, true, W[l], B, z, st, (tf & 128) != 0)));
      if (l == 4) HCK((fwd2<64, 128, 16, 2>(a.z, true, W[l], B, z, st, !(tf & 128))));
    } else
      HCK(conv_fwd_l(l, a, B, W[l], S.cout, z, reinterpret_cast<float*>(sc + L.part), st));  // Y = W . im2col(a)
    {
      const int NS = bn_slices(S.cout, B * hw);
      double* part = reinterpret_cast<double*>(sc + L.bnpart);
      float* rstd = reinterpret_cast<float*>(sv + L.rstd[l]);
      hipLaunchKernelGGL(k_bn_part, dim3(S.cout, NS), dim3(256), 0, st, z, B * hw, NS, part);
      hipLaunchKernelGGL(k_bn_apply, bn_row_grid(S.cout, B * hw), dim3(256), 0, st, z, B * hw, part, NS, bn_eps, mom,
                         rmean ? rmean[l] : nullptr, rvar ? rvar[l] : nullptr, rstd);
      HCK(hipGetLastError());
    }
  }
  hipLaunchKernelGGL(k_l2_fwd, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st,
                     reinterpret_cast<const float*>(sv + L.z[6]), B, l2_eps, out);
  return hipGetLastError();
}

hipError_t hn_train_backward(const float* dout, long B, const float* const* W, float* const* dW, float* din,
                             float l2_eps, float drop_p, unsigned long long seed, char* sv, char* sc, hipStream_t st) {
  const HnTrainWs L = hn_train_layout(B);
  HCK(hipMemsetAsync(sc + L.zero, 0, 128 * sizeof(float), st));
  const float* xn = reinterpret_cast<const float*>(sv + L.xn);
  float* gbuf[2] = {reinterpret_cast<float*>(sc + L.g0), reinterpret_cast<float*>(sc + L.g1)};
  // g: gradient w.r.t. layer l's output activation a_l (a_6 = z_6 into the L2 norm; a_5 =
  // dropout(relu(z_5)); a_l = relu(z_l) below), then in place w.r.t. its conv output
  float* g = gbuf[0];
  hipLaunchKernelGGL(k_l2_bwd, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st,
                     reinterpret_cast<const float*>(sv + L.z[6]), dout, B, l2_eps, g);
  HCK(hipGetLastError());
  for (int l = 6; l >= 0; --l) {
    const HnTrainLayer& S = kHardnetTrainLayers[l];
    const long ho = hout_of(S), hw = ho * ho, K = (long)S.cin * S.ks * S.ks;
    {
      const int NS = bn_slices(S.cout, B * hw);
      double* part = reinterpret_cast<double*>(sc + L.bnpart);
      const float* zl = reinterpret_cast<const float*>(sv + L.z[l]);
      hipLaunchKernelGGL(k_bn_bwd_part, dim3(S.cout, NS), dim3(256), 0, st, g, zl, B * hw, NS, l < 6 ? 1 : 0,
                         l == 5 ? drop_p : 0.f, seed, part);
      hipLaunchKernelGGL(k_bn_bwd_apply, bn_row_grid(S.cout, B * hw), dim3(256), 0, st, g, zl, B * hw, part, NS,
                         reinterpret_cast<const float*>(sv + L.rstd[l]), l < 6 ? 1 : 0, l == 5 ? drop_p : 0.f, seed);
      HCK(hipGetLastError());
    }
    const ActIn a{l == 0 ? xn : reinterpret_cast<const float*>(sv + L.z[l - 1]), l > 0 ? 1 : 0,
                  l == 6 ? drop_p : 0.f, seed};
    float* gin = gbuf[(7 - l) & 1];  // gradient w.r.t. this layer's input activation
    const bool want_in = l > 0 || din;
    // dW [Cout][K] = dY [Cout][B hw] . im2col(a)^T (split-K slices summed in fp64)
    float* part = reinterpret_cast<float*>(sc + L.part);
    if (l == 0 && !(hn_knobs().train_f32 & 64)) {  // conv0: k_wgrad0 (taps as the MFMA's N)
      const long ns = wgrad0_slices(B);
      hipLaunchKernelGGL(k_wgrad0, dim3((unsigned)(ns / 4)), dim3(256), 0, st, xn, g, B, part);
      HCK(hipGetLastError());
      GemmArgs gs{nullptr, nullptr, dW[0], 32, 9, 0, 0, 0, 0, 0, 9, 1, 1.f, 0.f};
      hipLaunchKernelGGL(k_splitk_sum, dim3((unsigned)((32 * 9 + 63) / 64)), dim3(1024), 0, st, gs, (int)ns, part);
      HCK(hipGetLastError());
    } else if ((l == 1 || l == 3 || l == 5) && !(hn_knobs().train_f32 & 4)) {  // stride-1 3x3: k_wgrad3
      const float* zx = reinterpret_cast<const float*>(sv + L.z[l - 1]);
      if (l == 1) HCK((wgrad3<32, 32, 32>(zx, g, B, dW[l], part, st)));
      if (l == 3) HCK((wgrad3<64, 64, 16>(zx, g, B, dW[l], part, st)));
      if (l == 5) HCK((wgrad3<128, 128, 8>(zx, g, B, dW[l], part, st)));
    } else if ((l == 2 || l == 4) && !(hn_knobs().train_f32 & 32)) {  // stride-2 3x3: k_wgrad2
      const float* zx = reinterpret_cast<const float*>(sv + L.z[l - 1]);
      if (l == 2) HCK((wgrad2<32, 64, 16>(zx, g, B, dW[l], part, st)));
      if (l == 4) HCK((wgrad2<64, 128, 8>(zx, g, B, dW[l], part, st)));
    } else {
      HCK(conv_wgrad_l(l, a, B, g, S.cout, dW[l], part, st));
    }
    if (want_in && S.s == 1 && S.ks == 3 && l >= 1 && !(hn_knobs().train_f32 & 16)) {
      // stride-1 3x3 (Cin = Cout): the data gradient is k_fwd3 over dY with the flipped weights
      float* wf = reinterpret_cast<float*>(sc + L.wt);
      hipLaunchKernelGGL(k_wflip, dim3((unsigned)((S.cout * S.cin * 9 + 255) / 256)), dim3(256), 0, st, W[l], S.cout,
                         S.cin, wf);
      HCK(hipGetLastError());
      if (l == 1) HCK((fwd3<32, 32, 32>(g, false, wf, B, gin, st)));
      const bool sh = !(hn_knobs().train_f32 & 128);
      if (l == 3) HCK((sh ? fwd3s<64, 64, 16> : fwd3<64, 64, 16>)(g, false, wf, B, gin, st));
      if (l == 5) HCK((sh ? fwd3s<128, 128, 8> : fwd3<128, 128, 8>)(g, false, wf, B, gin, st));
    } else if (want_in && S.s == 1 && S.ks == 3 && l >= 1 && !(hn_knobs().train_f32 & 2)) {
      // stride-1 3x3 (conv1 / conv3 / conv5: Cin = Cout): the data gradient is the same conv with
      // the weights flipped and transposed, on the bf16x3 MFMA conv kernels
      HCK(conv_bf16x3(l, true, g, false, B, W[l], gin, sc, L, st));
    } else if (want_in && S.s == 1 && S.ks == 3) {
      // stride-1 3x3: d a_{l-1} [Cin][B H H] = implicit col2im-gather GEMM Wt . dY (every tap lands)
      HCK(conv_dgrad_l(l, g, B, W[l], S.cout, reinterpret_cast<float*>(sc + L.wt), gin, st));
    } else if (want_in && (l == 2 || l == 4) && !(hn_knobs().train_f32 & 32)) {
      // stride-2 3x3: k_dgrad2 (the parity classes' taps only, f32 MFMA)
      const bool sh = !(hn_knobs().train_f32 & 128);
      if (l == 2) HCK((dgrad2<64, 32, 16>(g, W[l], B, gin, st, sh)));
      if (l == 4) HCK((dgrad2<128, 64, 8>(g, W[l], B, gin, st, sh)));
    } else if (want_in) {
      // stride 2 (3 of 4 taps miss a given input pixel) and the 8x8 conv6 (one tap per pixel):
      // dcol [K][n hw] = W^T [K][Cout] . dY, then the gather col2im, in chunks of patches
      float* col = reinterpret_cast<float*>(sc + L.col);
      const long nc = chunk_of(S, B);
      for (long n0 = 0; n0 < B; n0 += nc) {
        const long n = std::min(nc, B - n0);
        GemmArgs gd{W[l], g + n0 * hw, col, K, n * hw, S.cout, 1, K, B * hw, 1, n * hw, 1, 1.f, 0.f};
        HCK(gemm(gd, st));
        if (S.ks == 8 && ho == 1)  // conv6: the column matrix is the gradient, transposed
          hipLaunchKernelGGL(k_col6_to_cnhw, dim3(S.cin, (unsigned)((n + 63) / 64)), dim3(256), 0, st, col, B, n0,
                             n, gin);
        else
          hipLaunchKernelGGL(k_col2im, dim3(grid_for((long)S.cin * n * S.hin * S.hin)), dim3(256), 0, st, col,
                             S.cin, B, S.hin, S.hin, S.ks, S.s, S.pad, (int)ho, (int)ho, n0, n, gin);
        HCK(hipGetLastError());
      }
    }
    g = gin;
  }
  if (din) {
    // input_norm with detached mean / std (HardNet.py:309-310): d input = d xn / (std + eps)
    hipLaunchKernelGGL(k_scale_rows, dim3(grid_for(B * 1024)), dim3(256), 0, st, g, B,
                       reinterpret_cast<const float*>(sv + L.inv_sd));
    HCK(hipGetLastError());
    HCK(hipMemcpyAsync(din, g, (size_t)B * 1024 * 4, hipMemcpyDeviceToDevice, st));
  }
  return hipSuccess;
}
