// Winograd F(2x2, 3x3) for the stride-1 3x3 convs of stock HardNet (hardnet/HardNet.py:290-291
// conv3: 64 -> 64 at 16x16, :296-297 conv5: 128 -> 128 at 8x8; BN folded into the weights,
// ReLU fused).  Y = A^T [ (G g G^T) . (B^T d B) ] A per 2x2 output tile (Lavin & Gray): 16
// independent GEMMs (one per transform position xi) of [tiles x CIN] x [CIN x COUT], 2.25x
// fewer multiplies than the direct 3x3 implicit GEMM.  The GEMMs run on the bf16 MFMA in bf16x3
// split precision like the direct kernels (hn_common.h mfma3); the transforms are fp32 VALU.
//
// Work item = NPB patches (128 output tiles) x 32 output channels; 4 waves, one per SIMD, each
// owning 32 tiles x 32 channels x all 16 xi (256 accumulator registers), so the output
// transform is in-register.  Per stage (16 input channels):
//   * global_load_lds (16 B, lane-linear) fills the OTHER buffer with the next stage's input
//     image d and its U fragments while this stage computes;
//   * each lane reads its tile's 4x4 window (8 channels) from LDS, forms B^T d B in fp32,
//     splits to bf16 hi/lo as the MFMA A operand (rows = tiles) and runs 16 x mfma3 against the
//     U fragments (B operand, columns = output channels).
// LDS image of d: [patch][y][x & 1][x >> 1][16 channels], the 16-byte chunk q of a pixel in row y
// stored at q ^ ((y >> 1) & 3): every ds_read_b128 of the window reads is bank-conflict free
// (even/odd columns apart: stride-2 tiles hit consecutive pixels).  Window pixels outside the
// patch read a 64-byte zero block after the image.
#include "hn_common.h"
#include "hn_internal.h"

#include <type_traits>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int CIN, int COUT, int H>
struct WinoCfg {
  static constexpr int TPR = H / 2, TPP = TPR * TPR;  // tiles per row / per patch
  static constexpr int NW = 4, TB = NW * 32;          // waves, tiles per work item
  static constexpr int NPB = TB / TPP;                 // patches per work item
  static constexpr int NKS = CIN / 16, NCB = COUT / 32;
  static constexpr int DIMG = NPB * H * H * 64;        // d image per stage (16 fp32 channels)
  static constexpr int DB = DIMG + 64;                 // + zero block
  static constexpr int UIMG = 16 * 2 * 64 * 16;        // [xi][plane][lane] x 16 B
  static constexpr int UOFF = 2 * DB;
  static constexpr int SCR = 2 * DB + 2 * UIMG;       // epilogue transpose, 32 x 32 floats per wave
  static constexpr int SMEM = SCR + NW * 32 * 32 * 4;
  static constexpr int GLD = DIMG / (NW * 1024), GLU = UIMG / (NW * 1024);
  static_assert(TB % TPP == 0 && GLD * NW * 1024 == DIMG && GLU * NW * 1024 == UIMG, "tiling");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

HN_DEV void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)lds, 16, 0, 0);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// fp32 pair -> bf16 hi pair + bf16 lo pair, packed: v_cvt_pk_bf16_f32, two bit ops, one
// v_pk_add_f32, v_cvt_pk_bf16_f32 (the same rounding as hn_common.h split8)
HN_DEV void split2(float a, float b, unsigned& hi, unsigned& lo) {
  hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
  const float la = a - __builtin_bit_cast(float, hi << 16);
  const float lb = b - __builtin_bit_cast(float, hi & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{la, lb}, bf16x2));
}

// (scalar fp32 throughout: packed v_pk_add_f32 costs ~4x a v_sub_f32 in issue slots beside MFMAs,
// MI355X_MICROARCH.md cycle constants)
HN_DEV void split_v(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint4 h, l;
  split2(v[0], v[1], h.x, l.x);
  split2(v[2], v[3], h.y, l.y);
  split2(v[4], v[5], h.z, l.z);
  split2(v[6], v[7], h.w, l.w);
  hi = as_bf16x8(h);
  lo = as_bf16x8(l);
}

template <int CIN, int COUT, int H, int ABL = 0>
__global__ __launch_bounds__(256, 1) void k_wino(const float* __restrict__ in, float* __restrict__ out,
                                                 const uint4* __restrict__ wu, const float* __restrict__ bias,
                                                 int P) {
  using C = WinoCfg<CIN, COUT, H>;
  // one LDS object per buffer: a ds_read of this stage's buffer then provably does not alias
  // the global_load_lds filling the other one (same object + run-time lane offsets make hipcc
  // wait vmcnt(0) before the read, serialising the prefetch)
  // buffer b = [d image | zero block | U fragments]
  __shared__ __attribute__((aligned(16))) char sb0[C::DB + C::UIMG], sb1[C::DB + C::UIMG];
  __shared__ __attribute__((aligned(16))) float sscr[C::NW * 1024];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, rb = xcd_remap(blockIdx.x, nwg);
  const int ngroups = (P + C::NPB - 1) / C::NPB;
  const int nitems = ngroups * C::NCB;
  const int my_items = rb < nitems ? (nitems - 1 - rb) / nwg + 1 : 0;
  const int NS = my_items * C::NKS;
  if (NS == 0) return;

  // zero blocks of both buffers (never written by the loads)
  if (tid < 8) *reinterpret_cast<uint4*>(((tid >> 2) ? sb1 : sb0) + C::DIMG + (tid & 3) * 16) = uint4{0, 0, 0, 0};

  // ---- loader: chunk L = (wave * GLD + i) * 64 + lane of the d image = pixel L >> 2 (patch
  // uniform per instruction: 64 chunks never straddle a patch), stored chunk L & 3 = source
  // chunk (L & 3) ^ ((y >> 1) & 3) ----
  static_assert((H * H * 4) % 64 == 0, "one instruction = one patch");
  // stage s's data into buffer `b` (the last stage re-loads itself into the idle buffer: no
  // branch, so a stage stays one basic block)
  auto issue = [&](int s, int b) {
    const int it = rb + (s / C::NKS) * nwg, ks = s % C::NKS;
    const int pg = it / C::NCB, cb = it % C::NCB;
    char* dbuf = b ? sb1 : sb0;
#pragma unroll
    for (int i = 0; i < C::GLD; ++i) {
      const int L0 = (wave * C::GLD + i) * 64;  // uniform
      const int pp = L0 / (H * H * 4);
      const int p = min(pg * C::NPB + pp, P - 1);
      const int pix = (L0 % (H * H * 4) + lane) >> 2;
      const int xh = pix % (H / 2), xp = (pix / (H / 2)) & 1, y = pix / H;
      const int q = (lane & 3) ^ ((y >> 1) & 3);
      glds16(in + (size_t)p * (H * H * CIN) + (y * H + 2 * xh + xp) * CIN + 4 * q + 16 * ks,
             dbuf + (wave * C::GLD + i) * 1024);
    }
    const char* usrc = reinterpret_cast<const char*>(wu) + (size_t)(cb * C::NKS + ks) * C::UIMG + lane * 16;
    char* ubuf = (b ? sb1 : sb0) + C::DB;
#pragma unroll
    for (int i = 0; i < C::GLU; ++i)
      glds16(usrc + (wave * C::GLU + i) * 1024, ubuf + (wave * C::GLU + i) * 1024);
  };

  // ---- compute: this lane's tile window (A operand row = tile lane & 31, channels 8h..8h+7) ----
  const int h = lane >> 5;
  int off[4][4], dj[4];
  {
    const int t = wave * 32 + (lane & 31);
    const int pp = t / C::TPP, tt = t % C::TPP, ty = tt / C::TPR, tx = tt % C::TPR;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int y = 2 * ty + r - 1;
      const bool vy = (unsigned)y < (unsigned)H;
      const int s = (y >> 1) & 3;
      dj[r] = vy ? 16 * (((2 * h + 1) ^ s) - ((2 * h) ^ s)) : 16;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int x = 2 * tx + c - 1;
        const bool v = vy && (unsigned)x < (unsigned)H;
        off[r][c] = v ? (((pp * H + y) * 2 + (x & 1)) * (H / 2) + (x >> 1)) * 64 + 16 * ((2 * h) ^ s)
                      : C::DIMG + 16;  // +-16 stays inside the zero block
      }
    }
  }

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // items outer, stages inner: the accumulators are zeroed at the top of each item (no
  // conditional reset inside the stage loop, which makes hipcc keep them in VGPRs and copy)
#pragma unroll 1
  for (int k = 0; k < my_items; ++k) {
  f32x16 acc[16];
  // FIRST: the item's first stage starts each accumulator chain from an inline-constant zero
  // (no 256 v_accvgpr_write to clear them)
  auto stage = [&](int ks, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    const int s = k * C::NKS + ks;
    // NKS is even, so the buffer of stage s is ks & 1: a compile-time offset once the stages are
    // unrolled (with a run-time one hipcc cannot tell the next stage's global_load_lds target
    // from this stage's reads and waits vmcnt(0) before the first ds_read)
    static_assert(C::NKS % 2 == 0, "buffer parity = ks parity");
    if constexpr (!(ABL & 2)) issue(min(s + 1, NS - 1), (ks + 1) & 1);
    const char* D = (ks & 1) ? sb1 : sb0;
    // per-stage opaque copies of the lane offsets: the base differs per buffer, and hoisted
    // base + offset sums for both buffers would cost 2 x 20 registers
    int offs[4][4], djs[4], lofs = lane * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      djs[r] = dj[r];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        offs[r][c] = off[r][c];
        asm volatile("" : "+v"(offs[r][c]));
      }
    }
    asm volatile("" : "+v"(lofs));
    const char* U = D + C::DB + lofs;
    auto ldrow = [&](int r, float (&v)[4][8]) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(D + offs[r][c]);
        const f32x4 b = *reinterpret_cast<const f32x4*>(D + offs[r][c] + djs[r]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[c][e] = a[e];
          v[c][4 + e] = b[e];
        }
      }
    };
    auto ldu = [&](int xi, uint4 (&u)[2]) {
      u[0] = *reinterpret_cast<const uint4*>(U + xi * 2048);
      u[1] = *reinterpret_cast<const uint4*>(U + xi * 2048 + 1024);
    };
    // column transform of row t (B^T d)_i: position j
    auto vcol = [&](const float (&t)[4][8], int j, bf16x8& vh, bf16x8& vl) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (j == 0) v[e] = t[0][e] - t[2][e];
        if (j == 1) v[e] = t[1][e] + t[2][e];
        if (j == 2) v[e] = t[2][e] - t[1][e];
        if (j == 3) v[e] = t[1][e] - t[3][e];
      }
      split_v(v, vh, vl);
    };
    // rows of B^T d: t0 = d0 - d2, t1 = d1 + d2, t2 = d2 - d1, t3 = d1 - d3, each row pair read
    // from LDS just before its group so only t (and one pair in flight) stays live.  Software
    // pipeline per xi: MFMAs of xi, then the U reads of xi + 2 and the column transform + split
    // of xi + 1 (VALU under the MFMAs), one scheduling region per xi.
    float ra[4][8], rb2[4][8], t[4][8], t2[4][8];
    uint4 ub[3][2];
    ldrow(0, ra);
    ldrow(2, rb2);
    ldu(0, ub[0]);
    ldu(1, ub[1]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) t[c][e] = ra[c][e] - rb2[c][e];
    bf16x8 vh[2], vl[2];
    vcol(t, 0, vh[0], vl[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      if constexpr (ABL & 8)
        acc[xi][0] += __builtin_bit_cast(float, __builtin_bit_cast(uint4, vh[xi & 1]).x ^ __builtin_bit_cast(uint4, vl[xi & 1]).y ^ ub[xi % 3][0].z ^ ub[xi % 3][1].w);
      else
        acc[xi] = mfma3(vh[xi & 1], vl[xi & 1], as_bf16x8(ub[xi % 3][0]), as_bf16x8(ub[xi % 3][1]),
                        FIRST ? f32x16{} : acc[xi]);
      if (xi + 2 < 16) ldu(xi + 2, ub[(xi + 2) % 3]);
      if (xi == 1) { ldrow(1, ra); ldrow(2, rb2); }
      if (xi == 10) { ldrow(1, ra); ldrow(3, rb2); }
      const int n = xi + 1;
      if (n < 16) {
        if (n == 4) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              t[c][e] = ra[c][e] + rb2[c][e];
              t2[c][e] = rb2[c][e] - ra[c][e];
            }
        }
        if (n == 12) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) t[c][e] = ra[c][e] - rb2[c][e];
        }
        if (n >= 8 && n < 12)
          vcol(t2, n & 3, vh[n & 1], vl[n & 1]);
        else
          vcol(t, n & 3, vh[n & 1], vl[n & 1]);
      }
      // each dependent MFMA of the chain waits ~32 cycles for its predecessor: fill the gaps
      // with the next xi's transform and the LDS reads
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 15, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 15, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 15, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 64, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

  };
  using yes = std::integral_constant<bool, true>;
  using no = std::integral_constant<bool, false>;
  stage(0, yes{});
  if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // straight-line stages: a loop-carried accumulator set that fills the whole AGPR file makes
  // the register allocator copy it at the loop boundary (spills)
#pragma unroll
  for (int ks = 1; ks < C::NKS - 1; ++ks) {
    stage(ks, no{});
    if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // the last stage, its barrier and the output transform in one basic block: the accumulators
  // then reach the epilogue one vector at a time instead of being copied out of AGPRs at a
  // loop exit all at once (256 VGPRs -> spills)
  stage(C::NKS - 1, no{});
  __builtin_amdgcn_sched_barrier(0);  // keep the epilogue's accumulator reads out of the MFMA stage
  if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  {
      // output transform Y = A^T M A (A^T = [1 1 1 0; 0 1 -1 -1]), + bias, ReLU.  Lane: column
      // = output channel, accumulator element 4q + e = tile 8q + 4h + e.  Walked xi by xi (one
      // accumulator vector in VGPRs at a time): sc = the column transform of row i, y += A^T[a][i] sc.
      const int it = rb + k * nwg;
      const int pg = it / C::NCB, cb = it % C::NCB;
      const float bv = bias[cb * 32 + (lane & 31)];
      f32x16 y00 = f32x16{}, y01 = f32x16{}, y10 = f32x16{}, y11 = f32x16{};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x16 s0 = acc[4 * i];
        __builtin_amdgcn_sched_barrier(0);
        f32x16 s1 = acc[4 * i + 1];
        s0 += s1;
        __builtin_amdgcn_sched_barrier(0);
        const f32x16 m2 = acc[4 * i + 2];
        s0 += m2;
        s1 -= m2;
        __builtin_amdgcn_sched_barrier(0);
        s1 -= acc[4 * i + 3];
        if (i < 3) { y00 += s0; y01 += s1; }
        if (i == 1) { y10 += s0; y11 += s1; }
        if (i >= 2) { y10 -= s0; y11 -= s1; }
        __builtin_amdgcn_sched_barrier(0);
      }
      // + bias, ReLU; each output position (a, b) of the 2x2 tiles goes through this wave's LDS
      // scratch [tile 32][channel 32] so that 8 lanes store one pixel's 128-byte channel run
      float* scr = sscr + wave * 1024;
      const int rt = lane >> 3, c4 = lane & 7;  // read side: tile rt + 8 k, channels 4 c4 ..
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const f32x16& yv = ab == 0 ? y00 : ab == 1 ? y01 : ab == 2 ? y10 : y11;
#pragma unroll
        for (int x = 0; x < 16; ++x)
          scr[(8 * (x >> 2) + 4 * h + (x & 3)) * 32 + (lane & 31)] = fmaxf(yv[x] + bv, 0.f);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const int m = wave * 32 + rt + 8 * k4;
          const int pp = m / C::TPP, tt = m % C::TPP, ty = tt / C::TPR, tx = tt % C::TPR;
          const int p = pg * C::NPB + pp;
          const f32x4 v = *reinterpret_cast<const f32x4*>(scr + (rt + 8 * k4) * 32 + 4 * c4);
          if (p < P && (!(ABL & 4) || v[0] == 1234.5f))
            *reinterpret_cast<f32x4*>(out + (((size_t)p * H + 2 * ty + (ab >> 1)) * H + 2 * tx + (ab & 1)) * COUT +
                                      cb * 32 + 4 * c4) = v;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
  }
  }
}


template <int CIN, int COUT, int H, int ABL = 0>
hipError_t launch_wino(const float* in, float* out, const void* wu, const float* bias, int P, hipStream_t st) {
  using C = WinoCfg<CIN, COUT, H>;
  const void* fn = reinterpret_cast<const void*>(&k_wino<CIN, COUT, H, ABL>);
  int resident = 0;
  const hipError_t e = hn_resident_blocks(fn, 256, 0, &resident);  // LDS is static (C::SMEM)
  if (e != hipSuccess) return e;
  if (resident < 1) return hipErrorLaunchOutOfResources;
  const int items = (P + C::NPB - 1) / C::NPB * C::NCB;
  const int grid = std::min(items, resident);
  hipLaunchKernelGGL((k_wino<CIN, COUT, H, ABL>), dim3(grid), dim3(256), 0, st, in, out,
                     static_cast<const uint4*>(wu), bias, P);
  return hipGetLastError();
}

}  // namespace

// layer 3 (64 -> 64, 16x16) or 5 (128 -> 128, 8x8)
hipError_t hn_launch_wino(int layer, const HardnetDev& d, const float* in, float* out, int P, hipStream_t st) {
  if (P <= 0) return hipSuccess;
  if (!d.wino[layer]) return hipErrorInvalidValue;
#ifdef HN_EXPERIMENTS
#define HN_WABL(A) \
  if (hn_knobs().dbg == A) \
    return layer == 3 ? launch_wino<64, 64, 16, A>(in, out, d.wino[3], d.bias[3], P, st) \
                      : launch_wino<128, 128, 8, A>(in, out, d.wino[5], d.bias[5], P, st);
  HN_WABL(1) HN_WABL(2) HN_WABL(3) HN_WABL(4) HN_WABL(8) HN_WABL(12) HN_WABL(15)
#undef HN_WABL
#endif
  switch (layer) {
    case 3: return launch_wino<64, 64, 16>(in, out, d.wino[3], d.bias[3], P, st);
    case 5: return launch_wino<128, 128, 8>(in, out, d.wino[5], d.bias[5], P, st);
  }
  return hipErrorInvalidValue;
}
