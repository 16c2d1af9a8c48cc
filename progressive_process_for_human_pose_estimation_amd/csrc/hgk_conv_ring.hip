// 1x1 / stride-1 convolutions of the big hourglass levels (64x64, bf16): the LDS-DMA RING kernel.
//
// These launches (ResidualBlock conv1 / conv3 forward and their input gradients,
// try_with_torch.py:186,192; lin / ll_ at try_with_torch.py:249,292) move ~100-170 MB per launch at
// a few MFMA cycles per byte: HBM-bound. The tiled implicit-GEMM kernel reaches 3.2-3.8 TB/s on
// them because each workgroup keeps one 8 KB k-tile of input in flight at a time (four dependent
// round trips per tile; register-prefetching further ahead costs occupancy). This kernel is built
// around keeping bytes in flight instead:
// * ONE 8-wave workgroup per CU, persistent over a contiguous range of 32-pixel blocks;
// * every operand a block needs from memory — the input rows x[32][K] and, when fused, the
//   residual / accumulate source and the BN-backward input y[32][Cout] — goes global -> LDS by
//   LDS-DMA (global_load_lds_dwordx4, no registers) into a RING of R slots: R-1 blocks (~100 KB
//   per CU) are in flight while one is computed. Waits are counted vmcnt (every vector-memory
//   op a wave issues per block is a compile-time count), never vmcnt(0) in the loop;
// * each wave keeps its packed weight slice in REGISTERS for the whole launch (32 output
//   channels x K: 32-64 VGPRs) — weights never touch LDS;
// * the fused BN(+ReLU) input transform is applied once per element, in place in the slot, by
//   all 512 threads (a thread's 16-B chunks always hold the same 8 channels: its constants are
//   loop-invariant), one barrier before the MFMAs;
// * transposed MFMA (weights = A operand, pixels = B operand; weight rows permuted so a lane's 8
//   output channels are consecutive): bias / residual / ReLU / bf16 round / 16-B stores straight
//   from the accumulators; the BN statistics (two passes over the block's stored values: sum,
//   then sum of squared deviations, each reduced over the 16 pixels of a DPP row) are
//   Chan-merged in registers over U consecutive blocks and emitted as one partial row per
//   (U blocks, pixel group) from an LDS stash at the end of the launch (channel-major
//   [C][3][rows], hgk_bn_finalize's format); the fused BN-backward sums (sum g, sum g*xhat over
//   the STORED dA, hgk_bn_bwd_reduce's [rows][2][C] format) likewise;
// * folded BatchNorm-backward apply (MODE bit 16, the input gradient of a conv whose OUTPUT fed a
//   train-mode BN(+ReLU)): the x part holds that BN's upstream gradient dA and a fourth part its
//   input y; the transform pass turns dA into dy = hgk_bn_bwd_apply's value (bnb_apply, same
//   bits), in place, and also stores it (vout): the conv's weight gradient reads it later. The
//   separate apply pass (read dA, y; write dy; read dy again here) disappears;
// * twin launches (two convolutions with the same weights: an hourglass level's up- and
//   down-branch blocks) are one block list: blocks [0, nb0) segment 0, the rest segment 1.
// LDS layout of a slot: the parts (x | res | bn-y), rows of 16-B chunks, chunk c of pixel p at
// position c ^ (p & 15) — conflict-free for the ds_read_b128 fragment and epilogue reads
// (the swizzle is applied to the per-lane DMA source address); 64-channel parts (128-B rows, two
// pixels per 256-B bank period) take c ^ ((p >> 1) & 7) (ring_swz).
#include <algorithm>

#include "hgk_common.h"
#include "hgk_conv.h"

namespace hgk {

struct RingSeg {
  const bf16_t* x;
  const bf16_t* res;
  bf16_t* y;
  const float* pre_scale;
  const float* pre_shift;
  float* stats;
  const bf16_t* bby;
  const float *bsc, *bsh, *bmu, *bis;
  float* bpart;
  // folded BN-backward apply (MODE & 16): BN input y [M][K], forward scale / shift (ReLU mask),
  // coefficients [4][K] (k0, k1, k2, mean), materialised dy [M][K]
  const bf16_t* vgy;
  const float *vsc, *vsh, *vco;
  bf16_t* vout;
  int rows;  // partial rows of this segment (stats_R)
};

struct RingArgs {
  RingSeg s[2];
  const bf16_t* w;
  const float* bias;
  int w_ld;
  int pre_relu, post_relu, bb_relu, vg_relu;
  int nb0;   // blocks of segment 0
  int nrg;   // row groups (U blocks each) of both segments
  int nrg0;  // row groups of segment 0
};

// pixels per block: 16 * (pixel groups) * 2, i.e. two 16-pixel MFMA tiles per wave (64 for 128
// output channels, 32 for 256), unless that makes a slot larger than 32 KB (BN-backward and
// residual variants at 128 output channels: 32)
// NW = 4: two 4-wave workgroups per CU (half the LDS each, slots <= 16 KB, 16-pixel blocks when
// a 32-pixel slot would not fit) — the two workgroups' blocks interleave on every SIMD instead of
// all eight waves running each phase in lock step
// 64 output channels: 2 channel groups, so 4 (NW 8) / 2 (NW 4) pixel groups of 16-pixel tiles;
// 64 input channels: blocks grow until the x part is whole 1-KB-per-wave DMA rounds (ring_bp)
static constexpr int kRingU = 4;         // blocks per partial-row group
static constexpr int kRingRGMax = 8;     // row groups per workgroup (LDS stash)
#ifndef HGK_RING_NW4_KB
#define HGK_RING_NW4_KB 48
#endif
__host__ __device__ constexpr int ring_bytes(int NW) { return NW == 8 ? 128 * 1024 : HGK_RING_NW4_KB * 1024; }
__host__ __device__ constexpr int ring_slot_bytes(int bp, int K, int COUT, int MODE) {
  return bp * 2 * (K + ((MODE & 2) ? COUT : 0) + ((MODE & 4) ? COUT : 0) + ((MODE & 16) ? K : 0));
}
// every part of a slot whole DMA rounds (NW x 1 KB)
__host__ __device__ constexpr bool ring_parts_ok(int bp, int K, int COUT, int MODE, int NW) {
  return (bp * K * 2) % (NW * 1024) == 0 && (bp * COUT * 2) % (NW * 1024) == 0;
}
__host__ __device__ constexpr int ring_bp(int K, int COUT, int MODE, int NW = 8) {
  const int PG = COUT < 32 ? 1 : NW / (COUT / 32) > 0 ? NW / (COUT / 32) : 1;
  const int lim = NW == 8 ? 32768 : 16384;
  if (ring_slot_bytes(PG * 32, K, COUT, MODE) <= lim && ring_parts_ok(PG * 32, K, COUT, MODE, NW)) return PG * 32;
  int bp = PG * 16;
  while (bp < 1024 && !ring_parts_ok(bp, K, COUT, MODE, NW)) bp *= 2;
  return bp;
}
// the configuration's wave split, ring depth and transform mapping hold (RingCfg's static_asserts)
__host__ __device__ constexpr bool ring_cfg_ok(int K, int COUT, int MODE, int NW) {
  const int bp = ring_bp(K, COUT, MODE, NW), CG = COUT / 32;
  if (CG < 1 || NW % CG != 0) return false;
  const int PG = NW / CG, NT = 64 * NW;
  const int R = ring_bytes(NW) / ring_slot_bytes(bp, K, COUT, MODE);
  return (bp / 16) / PG >= 1 && ring_parts_ok(bp, K, COUT, MODE, NW) && R >= 3 &&
         (bp * (K / 8)) % NT == 0 && NT % (K / 8) == 0 && (!(MODE & 16) || NW == 8);
}
// swizzle of 16-B chunk slots in a pixel row of `chunks` chunks (>= 16: 256-B rows; 8: 128-B rows)
__host__ __device__ constexpr int ring_swz(int chunks, int p) { return chunks >= 16 ? (p & 15) : ((p >> 1) & 7); }

template <int K, int COUT, int MODE, int NW = 8>
struct RingCfg {
  static constexpr bool PRE = MODE & 1, RES = (MODE & 2) != 0, BBM = (MODE & 4) != 0,
                        STATS = (MODE & 8) != 0, VG = (MODE & 16) != 0;
  static constexpr int NT = 64 * NW;           // threads
  static constexpr int DRB = NW * 1024;         // bytes of one DMA round (1 KB per wave)
  static constexpr int BP = ring_bp(K, COUT, MODE, NW);
  static constexpr int CG = COUT / 32;          // channel groups of 32
  static constexpr int PG = NW / CG;            // pixel groups (waves per channel group)
  static constexpr int PTW = (BP / 16) / PG;    // 16-pixel MFMA tiles per wave
  static constexpr int KS = K / 32;             // MFMA k-steps
  static constexpr int XB = BP * K * 2;
  static constexpr int RBY = RES ? BP * COUT * 2 : 0;
  static constexpr int YBY = BBM ? BP * COUT * 2 : 0;
  static constexpr int VGY = VG ? BP * K * 2 : 0;
  static constexpr int SB = XB + RBY + YBY + VGY;  // slot bytes
  static constexpr int D = SB / DRB;            // 1-KB DMAs per wave per block
  static constexpr int R0 = ring_bytes(NW) / SB;
#ifndef HGK_ABL_RING_RMAX
#define HGK_ABL_RING_RMAX 12
#endif
  static constexpr int R = R0 > HGK_ABL_RING_RMAX ? HGK_ABL_RING_RMAX : R0;   // ring slots
  static constexpr int TCH = BP * (K / 8) / NT;  // transform chunks per thread per block
  // 16-B stores per wave per block: the epilogue's, and the folded apply's dy chunks (VG)
#ifdef HGK_ABL_RING_NOSTORE  // ablation: no epilogue stores (wrong results; timing only)
  static constexpr int ST = VG ? TCH : 0;
#else
  static constexpr int ST = PTW + (VG ? TCH : 0);
#endif
  static constexpr int NROWS = kRingRGMax * PG; // stash rows
  static constexpr int XCH = K / 8, CCH = COUT / 8;  // 16-B chunks per pixel row
  static_assert(PG * CG == NW && PTW >= 1, "wave split");
  static_assert(XB % DRB == 0 && RBY % DRB == 0 && YBY % DRB == 0 && VGY % DRB == 0,
                "parts of whole DMA rounds");
  static_assert(TCH >= 1 && TCH * NT == BP * (K / 8) && NT % (K / 8) == 0, "transform mapping");
  static_assert(!VG || NW == 8, "the folded apply's transform assumes one channel chunk per thread");
  static_assert(!(VG && PRE), "a folded BN-backward apply and a BN forward transform exclude each other");
  static_assert(R >= 3, "ring depth");  // R - 2 blocks in flight at a wait
};

// s_waitcnt vmcnt(min(base + i * st, 63)) for the runtime i in [0, N]
template <int BASE, int ST, int N>
__device__ __forceinline__ void ring_wait(int i) {
  if constexpr (N > 0) {
    if (i < N) {
      ring_wait<BASE, ST, N - 1>(i);
      return;
    }
  }
  constexpr int X = BASE + N * ST > 63 ? 63 : BASE + N * ST;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
}

template <int K, int COUT, int MODE, int NW = 8>
__global__ __launch_bounds__(64 * NW) void conv1x1_ring_kernel(RingArgs ra) {
  typedef RingCfg<K, COUT, MODE, NW> C;
  constexpr int NT = C::NT;
  constexpr int BP = C::BP, PG = C::PG, CG = C::CG, PTW = C::PTW, KS = C::KS, R = C::R, D = C::D;
  __shared__ __attribute__((aligned(16))) char ring[R * C::SB];
  __shared__ __attribute__((aligned(16))) float stash[C::NROWS * 2 * COUT];
  __shared__ __attribute__((aligned(16))) float sPre[C::PRE ? 2 * 2 * K : 4];      // [seg][scale|shift][K]
  __shared__ __attribute__((aligned(16))) float sBb[C::BBM ? 2 * 4 * COUT : 4];    // [seg][sc|sh|mu|is][COUT]
  __shared__ __attribute__((aligned(16))) float sVg[C::VG ? 2 * 6 * K : 4];        // [seg][sc|sh|k0|k1|k2|mu][K]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, q = lane >> 4;
  // XCD-contiguous workgroup order: the workgroups of one XCD walk neighbouring row groups, so
  // a 128-B line of channel-major partial slots is written from one L2
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int vid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int rg0 = (int)((long)vid * ra.nrg / G), rg1 = (int)((long)(vid + 1) * ra.nrg / G);
  const int nbw = (rg1 - rg0) * kRingU;
  if (nbw <= 0) return;  // workgroup-uniform

  const int cgi = wave % CG, pgi = wave / CG;
  const int cb = cgi * 32;  // this wave's first output channel

  // ---- DMA geometry: instruction j of this wave = 1-KB piece j * NW + wave of the slot ----
  int doff[D];  // element offset of this lane's 16 B within the block's part
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const int gb = (j * NW + wave) * 1024 + lane * 16;
    int s, rowc, cols;
    if (j * C::DRB < C::XB) {
      s = gb / 16; rowc = C::XCH; cols = K;
    } else if (j * C::DRB < C::XB + C::RBY) {
      s = (gb - C::XB) / 16; rowc = C::CCH; cols = COUT;
    } else if (j * C::DRB < C::XB + C::RBY + C::YBY) {
      s = (gb - C::XB - C::RBY) / 16; rowc = C::CCH; cols = COUT;
    } else {  // VG: the BN input, laid out as the x part
      s = (gb - C::XB - C::RBY - C::YBY) / 16; rowc = C::XCH; cols = K;
    }
    const int p = s / rowc, c = (s % rowc) ^ ring_swz(rowc, p);
    doff[j] = p * cols + c * 8;
  }
  // block b (workgroup-local, clamped: the tail re-loads the last block into a free slot so the
  // per-iteration op count stays fixed) -> slot
  auto issue = [&](int b, int slot) __attribute__((always_inline)) {
    b = min(b, nbw - 1);
    const int gbk = rg0 * kRingU + b;
    const bool sg = gbk >= ra.nb0;
    const long pix0 = (long)(gbk - (sg ? ra.nb0 : 0)) * BP;
    const bf16_t* bx = (sg ? ra.s[1].x : ra.s[0].x) + pix0 * K;
    const bf16_t* brs = nullptr;
    const bf16_t* bby = nullptr;
    const bf16_t* bvg = nullptr;
    if constexpr (C::RES) brs = (sg ? ra.s[1].res : ra.s[0].res) + pix0 * COUT;
    if constexpr (C::BBM) bby = (sg ? ra.s[1].bby : ra.s[0].bby) + pix0 * COUT;
    if constexpr (C::VG) bvg = (sg ? ra.s[1].vgy : ra.s[0].vgy) + pix0 * K;
    char* sbase = ring + slot * C::SB;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const bf16_t* src = j * C::DRB < C::XB ? bx
                          : j * C::DRB < C::XB + C::RBY ? brs
                          : j * C::DRB < C::XB + C::RBY + C::YBY ? bby : bvg;
      dma16(src + doff[j], sbase + (j * NW + wave) * 1024);
    }
  };

#pragma unroll
  for (int b = 0; b < R - 1; ++b) issue(b, b);

  // ---- per-launch constants -> registers / LDS (compiler-visible loads, all waited for below) ----
  bf16x8 wreg[2][KS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // MFMA row rho of tile j <-> channel cb + 8 (rho >> 2) + 4 j + (rho & 3): a lane's accumulator
    // rows of tiles 0 and 1 are 8 consecutive channels
    const int ch = cb + 8 * (lr >> 2) + 4 * j + (lr & 3);
    const bf16_t* wp = ra.w + (long)ch * ra.w_ld + q * 8;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) wreg[j][kk] = *reinterpret_cast<const bf16x8*>(wp + kk * 32);
  }
  float bias8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias8[e] = ra.bias ? ra.bias[cb + 8 * q + e] : 0.f;
  constexpr int UPRE = (4 * K + NT - 1) / NT, UBB = (8 * COUT + NT - 1) / NT,
                UVG = (12 * K + NT - 1) / NT;
  float cpre[UPRE];
  if constexpr (C::PRE) {
    // 4 * K values: [seg][scale|shift][K]
#pragma unroll
    for (int u = 0; u < UPRE; ++u) {
      cpre[u] = 0.f;
      const int i = tid + u * NT;
      if (i < 4 * K) {
        const int sg = i / (2 * K), part = (i / K) & 1, c = i % K;
        const float* src = part ? ra.s[sg].pre_shift : ra.s[sg].pre_scale;
        cpre[u] = src ? src[c] : 0.f;
      }
    }
  }
  float cbb[UBB];
  if constexpr (C::BBM) {
#pragma unroll
    for (int u = 0; u < UBB; ++u) {
      cbb[u] = 0.f;
      const int i = tid + u * NT;
      if (i < 8 * COUT) {
        const int sg = i / (4 * COUT), part = (i / COUT) & 3, c = i % COUT;
        const RingSeg& s = ra.s[sg];
        const float* src = part == 0 ? s.bsc : part == 1 ? s.bsh : part == 2 ? s.bmu : s.bis;
        cbb[u] = src ? src[c] : 0.f;
      }
    }
  }

  float cvg[UVG];
  if constexpr (C::VG) {
    // 12 * K values: [seg][sc|sh|k0|k1|k2|mu][K]
#pragma unroll
    for (int u = 0; u < UVG; ++u) {
      cvg[u] = 0.f;
      const int i = tid + u * NT;
      if (i < 12 * K) {
        const int sg = i / (6 * K), part = (i / K) % 6, c = i % K;
        const RingSeg& s = ra.s[sg];
        const float* src = part == 0 ? s.vsc : part == 1 ? s.vsh : s.vco + (part - 2) * K;
        cvg[u] = src[c];
      }
    }
  }
  // constants -> LDS. Their loads went out right behind the prologue DMAs: the compiler's
  // vmcnt(0) before these stores waits for both in one round trip
  if constexpr (C::PRE) {
#pragma unroll
    for (int u = 0; u < UPRE; ++u)
      if (tid + u * NT < 4 * K) sPre[tid + u * NT] = cpre[u];
  }
  if constexpr (C::BBM) {
#pragma unroll
    for (int u = 0; u < UBB; ++u)
      if (tid + u * NT < 8 * COUT) sBb[tid + u * NT] = cbb[u];
  }
  if constexpr (C::VG) {
#pragma unroll
    for (int u = 0; u < UVG; ++u)
      if (tid + u * NT < 12 * K) sVg[tid + u * NT] = cvg[u];
  }
  // the weight / bias registers: waited for here, not inside the loop
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(bias8[e]));
  {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) asm volatile("" ::"v"(wreg[j][kk]));
  }

  // ---- fragment / epilogue LDS offsets (fixed per lane) ----
  // x fragment of tile t, k-step kk: pixel p = pt*16 + lr, chunk kk*4 + q at (kk*4+q) ^ lr
  int xo[PTW][4];
#pragma unroll
  for (int t = 0; t < PTW; ++t) {
    const int p = (pgi * PTW + t) * 16 + lr;
#pragma unroll
    for (int kl = 0; kl < 4; ++kl) xo[t][kl] = p * K * 2 + (((kl * 4 + q) ^ ring_swz(C::XCH, p)) << 4);
  }
  // epilogue (res / bn-y parts): pixel p, chunk cb/8 + q
  int eo[PTW];
#pragma unroll
  for (int t = 0; t < PTW; ++t) {
    const int p = (pgi * PTW + t) * 16 + lr;
    eo[t] = p * COUT * 2 + ((((cb >> 3) + q) ^ ring_swz(C::CCH, p)) << 4);
  }
  // transform pass: thread -> chunks tid + NT u of the x part (pixel tp + u NT / XCH); its channel
  // chunk is fixed when NT / XCH is a multiple of 16 (the swizzle period), else it alternates
  constexpr int TCH = BP * C::XCH / NT;
  constexpr int TPU = NT / C::XCH;  // pixels per transform step
  const int tp = tid / C::XCH, tc = (tid % C::XCH) ^ ring_swz(C::XCH, tp);

  // BN(+ReLU) of one 16-B chunk (8 bf16) in place: packed fp32 FMAs, one v_cvt_pk_bf16_f32 and
  // one v_pk_max_i16 per pair (floor 0 = ReLU, INT16_MIN = none: a bf16 is negative iff its
  // int16 image is)
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const short floor16 = ra.pre_relu ? (short)0 : (short)-32768;
  auto transform = [&](int slot, bool sg) __attribute__((always_inline)) {
    f32x2 s2[4], b2[4];
    auto load_consts = [&](int tcu) __attribute__((always_inline)) {
      const float* ps = sPre + (sg ? 2 * K : 0) + tcu * 8;
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const float4 s4 = *reinterpret_cast<const float4*>(ps + e);
        const float4 b4 = *reinterpret_cast<const float4*>(ps + K + e);
        s2[e / 2] = f32x2{s4.x, s4.y}; s2[e / 2 + 1] = f32x2{s4.z, s4.w};
        b2[e / 2] = f32x2{b4.x, b4.y}; b2[e / 2 + 1] = f32x2{b4.z, b4.w};
      }
    };
    load_consts(tc);
#pragma unroll
    for (int u = 0; u < TCH; ++u) {
      if constexpr (TPU % 16 != 0) {
        if (u > 0) load_consts((tid % C::XCH) ^ ring_swz(C::XCH, tp + u * TPU));
      }
      uint4* cp = reinterpret_cast<uint4*>(ring + slot * C::SB + (tid + u * NT) * 16);
      const uint4 v = *cp;
      const uint32_t in[4] = {v.x, v.y, v.z, v.w};
      uint32_t out[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        f32x2 f = {__uint_as_float(in[h] << 16), __uint_as_float(in[h] & 0xffff0000u)};
        f = f * s2[h] + b2[h];
        const bf16x2_t r2 = __builtin_convertvector(f, bf16x2_t);
        s16x2 qv = __builtin_bit_cast(s16x2, r2);
        qv = __builtin_elementwise_max(qv, (s16x2){floor16, floor16});
        out[h] = __builtin_bit_cast(uint32_t, qv);
      }
      *cp = make_uint4(out[0], out[1], out[2], out[3]);
    }
  };
  // folded BN-backward apply of block b in `slot` (b clamped like issue(): the tail re-transforms
  // the re-loaded last block and re-stores the same values, keeping the per-iteration op count)
  auto transform_vg = [&](int slot, int b) __attribute__((always_inline)) {
    b = min(b, nbw - 1);
    const int gbk = rg0 * kRingU + b;
    const bool sg = gbk >= ra.nb0;
    const long pix0 = (long)(gbk - (sg ? ra.nb0 : 0)) * BP;
    const float* kv = sVg + (sg ? 6 * K : 0) + tc * 8;
    float vsc[8], vsh[8], vk0[8], vk1[8], vk2[8], vmu[8];
#pragma unroll
    for (int e = 0; e < 8; e += 4) {
      const float4 a0 = *reinterpret_cast<const float4*>(kv + e);
      const float4 a1 = *reinterpret_cast<const float4*>(kv + K + e);
      const float4 a2 = *reinterpret_cast<const float4*>(kv + 2 * K + e);
      const float4 a3 = *reinterpret_cast<const float4*>(kv + 3 * K + e);
      const float4 a4 = *reinterpret_cast<const float4*>(kv + 4 * K + e);
      const float4 a5 = *reinterpret_cast<const float4*>(kv + 5 * K + e);
      vsc[e] = a0.x; vsc[e + 1] = a0.y; vsc[e + 2] = a0.z; vsc[e + 3] = a0.w;
      vsh[e] = a1.x; vsh[e + 1] = a1.y; vsh[e + 2] = a1.z; vsh[e + 3] = a1.w;
      vk0[e] = a2.x; vk0[e + 1] = a2.y; vk0[e + 2] = a2.z; vk0[e + 3] = a2.w;
      vk1[e] = a3.x; vk1[e + 1] = a3.y; vk1[e + 2] = a3.z; vk1[e + 3] = a3.w;
      vk2[e] = a4.x; vk2[e + 1] = a4.y; vk2[e + 2] = a4.z; vk2[e + 3] = a4.w;
      vmu[e] = a5.x; vmu[e + 1] = a5.y; vmu[e + 2] = a5.z; vmu[e + 3] = a5.w;
    }
    bf16_t* vo = sg ? ra.s[1].vout : ra.s[0].vout;
    const bool vrelu = ra.vg_relu != 0;
#pragma unroll
    for (int u = 0; u < C::TCH; ++u) {
      char* cp = ring + slot * C::SB + (tid + u * NT) * 16;
      float fd[8], fy[8], o[8];
      unpack16<bf16_t>(*reinterpret_cast<const uint4*>(cp), fd);
      unpack16<bf16_t>(*reinterpret_cast<const uint4*>(cp + C::XB + C::RBY + C::YBY), fy);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = bnb_apply(fd[e], fy[e], vsc[e], vsh[e], vk0[e], vk1[e], vk2[e], vmu[e], vrelu);
      const uint4 pk = pack16<bf16_t>(o);
      *reinterpret_cast<uint4*>(cp) = pk;
      store16(vo + (pix0 + tp + u * TPU) * K + tc * 8, pk);
    }
  };
  auto seg_of = [&](int i, long& pix0) __attribute__((always_inline)) {
    const int gbk = rg0 * kRingU + i;
    const bool sg = gbk >= ra.nb0;
    pix0 = (long)(gbk - (sg ? ra.nb0 : 0)) * BP;
    return sg;
  };
  // the constants in LDS (every thread's stores) and block 0 (every wave's pieces)
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"((R - 2) * D) : "memory");
  __syncthreads();
  if constexpr (C::PRE) {
    // block 0 transformed before the loop
    long p0;
    const bool sg0 = seg_of(0, p0);
    transform(0, sg0);
  }
  if constexpr (C::VG) transform_vg(0, 0);

  // Per iteration ONE barrier: at the top, block i + 1 has landed (counted vmcnt) and every wave
  // is done with iteration i - 1, whose slot takes the DMA of block i + R - 1. Block i was
  // transformed in iteration i - 1; block i + 1 is transformed here, behind block i's MFMAs.
  const int nrgw = rg1 - rg0;
#pragma unroll 1
  for (int gi = 0; gi < nrgw; ++gi) {
    uint4 keep[kRingU][PTW];         // STATS: the stored outputs of the row group (bf16 x 8)
    float bs1[8], bs2[8];            // BBM: per-lane sum g, sum g * xhat over the row group
#pragma unroll
    for (int e = 0; e < 8; ++e) { bs1[e] = 0.f; bs2[e] = 0.f; }
    // the row group's segment (segments hold whole row groups): its BN-backward constants
    float sc[8], sh[8], is[8], mis[8];
    if constexpr (C::BBM) {
      long pg0;
      const bool sgg = seg_of(gi * kRingU, pg0);
      const float* kb = sBb + (sgg ? 4 * COUT : 0) + cb + 8 * q;
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const float4 v0 = *reinterpret_cast<const float4*>(kb + e);
        const float4 v1 = *reinterpret_cast<const float4*>(kb + COUT + e);
        const float4 v2 = *reinterpret_cast<const float4*>(kb + 2 * COUT + e);
        const float4 v3 = *reinterpret_cast<const float4*>(kb + 3 * COUT + e);
        sc[e] = v0.x; sc[e + 1] = v0.y; sc[e + 2] = v0.z; sc[e + 3] = v0.w;
        sh[e] = v1.x; sh[e + 1] = v1.y; sh[e + 2] = v1.z; sh[e + 3] = v1.w;
        is[e] = v3.x; is[e + 1] = v3.y; is[e + 2] = v3.z; is[e + 3] = v3.w;
        mis[e] = -v2.x * v3.x; mis[e + 1] = -v2.y * v3.y;
        mis[e + 2] = -v2.z * v3.z; mis[e + 3] = -v2.w * v3.w;
      }
    }
    // STATS keeps every block's stored outputs in registers (keep[j]: j must be a compile-time
    // index -> the U blocks unrolled); otherwise a rolled loop (registers)
    constexpr int JU = C::STATS ? kRingU : 1, JR = C::STATS ? 1 : kRingU;
#pragma unroll
    for (int ju = 0; ju < JU; ++ju)
#pragma unroll 1
    for (int jr = 0; jr < JR; ++jr) {
      const int j = C::STATS ? ju : jr;
      const int i = gi * kRingU + j;
      const int slot = i % R;
      char* sb = ring + slot * C::SB;
      ring_wait<(R - 3) * D, C::ST, R - 2>(i);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's transform writes
      // raw s_barrier: __syncthreads' release fence would drain the stores and DMAs in flight
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(i + R - 1, (i + R - 1) % R);
      long pix0;
      const bool sg = seg_of(i, pix0);
      auto transform_next = [&]() __attribute__((always_inline)) {
        if constexpr (C::PRE) {
          if (i + 1 < nbw) {
            long pn;
            const bool sgn = seg_of(i + 1, pn);
            transform((i + 1) % R, sgn);
          }
        }
        if constexpr (C::VG) transform_vg((i + 1) % R, i + 1);
      };
#ifndef HGK_ABL_RING_XFORM_LATE
      transform_next();
#endif
      // ---- MFMA: acc[t][j] = W[tile j rows] x X[pixel tile t]^T over K ----
      f32x4 acc[PTW][2];
#pragma unroll
      for (int t = 0; t < PTW; ++t) {
        acc[t][0] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#ifndef HGK_ABL_RING_NOMFMA  // ablation: no MFMAs (wrong results; timing only)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int t = 0; t < PTW; ++t) {
          const bf16x8 xv = *reinterpret_cast<const bf16x8*>(sb + xo[t][kk & 3] + (kk >> 2) * 256);
          acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[0][kk], xv, acc[t][0], 0, 0, 0);
          acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[1][kk], xv, acc[t][1], 0, 0, 0);
        }
      }
#endif
#ifdef HGK_ABL_RING_XFORM_LATE
      transform_next();  // behind the MFMAs (their latency hidden by its VALU / LDS work)
#endif
      // ---- epilogue: lane = 8 consecutive channels cb + 8q .. of pixel (tile t, lr) ----
      bf16_t* ys = sg ? ra.s[1].y : ra.s[0].y;
#pragma unroll
      for (int t = 0; t < PTW; ++t) {
        float f[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = acc[t][0][r] + bias8[r];
          f[4 + r] = acc[t][1][r] + bias8[4 + r];
        }
        if constexpr (C::RES) {
          float rv[8];
          unpack16<bf16_t>(*reinterpret_cast<const uint4*>(sb + C::XB + eo[t]), rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += rv[e];
        }
        if (ra.post_relu)
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
        const uint4 pk = pack16<bf16_t>(f);
        const long p = pix0 + (pgi * PTW + t) * 16 + lr;
#ifndef HGK_ABL_RING_NOSTORE
        store16(ys + p * COUT + cb + 8 * q, pk);
#endif
        if constexpr (C::STATS) keep[ju][t] = pk;
        if constexpr (C::BBM) {
          // BN-backward partial sums over the STORED dA: g = dA [relu mask of the BN output]
          float fs[8], yv[8];
          unpack16<bf16_t>(pk, fs);
          unpack16<bf16_t>(*reinterpret_cast<const uint4*>(sb + C::XB + C::RBY + eo[t]), yv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gv = (ra.bb_relu && !(fmaf(yv[e], sc[e], sh[e]) > 0.f)) ? 0.f : fs[e];
            bs1[e] += gv;
            bs2[e] = fmaf(gv, fmaf(yv[e], is[e], mis[e]), bs2[e]);
          }
        }
      }
    }
    // ---- row group done: reduce over the 16 pixels of each DPP row, stash the partial row ----
    float o1[8], o2[8];
    if constexpr (C::STATS) {
      // two passes over the row group's kRingU * 16 * PTW stored values per channel
      float vals[kRingU][PTW][8];
#pragma unroll
      for (int j = 0; j < kRingU; ++j)
#pragma unroll
        for (int t = 0; t < PTW; ++t) unpack16<bf16_t>(keep[j][t], vals[j][t]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < kRingU; ++j)
#pragma unroll
          for (int t = 0; t < PTW; ++t) sum += vals[j][t][e];
        o1[e] = sum;
      }
      row_allreduce<8>(o1);
      constexpr float inv_n = 1.f / (kRingU * 16 * PTW);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float mu = o1[e] * inv_n;
        float d2 = 0.f;
#pragma unroll
        for (int j = 0; j < kRingU; ++j)
#pragma unroll
          for (int t = 0; t < PTW; ++t) {
            const float d = vals[j][t][e] - mu;
            d2 = fmaf(d, d, d2);
          }
        o2[e] = d2;
      }
      row_allreduce<8>(o2);
    }
    if constexpr (C::BBM) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { o1[e] = bs1[e]; o2[e] = bs2[e]; }
      row_allreduce<8>(o1);
      row_allreduce<8>(o2);
    }
    if constexpr (C::STATS || C::BBM) {
      const int row = gi * PG + pgi;  // workgroup-local stash row
      if (lr == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          stash[(row * 2 + 0) * COUT + cb + 8 * q + e] = o1[e];
          stash[(row * 2 + 1) * COUT + cb + 8 * q + e] = o2[e];
        }
      }
    }
  }

  if constexpr (C::STATS || C::BBM) {
    __syncthreads();
    // this workgroup's rows: row groups [rg0, rg1) x pixel groups, each segment's rows contiguous
    const int nrow = (rg1 - rg0) * PG;
    for (int idx = tid; idx < nrow * COUT; idx += NT) {
      int ch, lrow;
      if constexpr (C::STATS) { ch = idx / nrow; lrow = idx - ch * nrow; }  // rows fastest
      else { lrow = idx / COUT; ch = idx - lrow * COUT; }                    // channels fastest
      const int rg = rg0 + lrow / PG, pg = lrow % PG;
      const bool s1 = rg >= ra.nrg0;
      const int row = (rg - (s1 ? ra.nrg0 : 0)) * PG + pg;
      const float a = stash[(lrow * 2 + 0) * COUT + ch], b = stash[(lrow * 2 + 1) * COUT + ch];
      if constexpr (C::STATS) {
        float* st = s1 ? ra.s[1].stats : ra.s[0].stats;
        const int Rs = s1 ? ra.s[1].rows : ra.s[0].rows;
        st[((long)ch * 3 + 0) * Rs + row] = a;
        st[((long)ch * 3 + 1) * Rs + row] = b;
        st[((long)ch * 3 + 2) * Rs + row] = (float)(kRingU * 16 * PTW);
      } else {
        float* bp = s1 ? ra.s[1].bpart : ra.s[0].bpart;
        bp[((long)row * 2 + 0) * COUT + ch] = a;
        bp[((long)row * 2 + 1) * COUT + ch] = b;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static int ring_mode(const ConvFwdArgs& a) {
  return (a.pre_scale ? 1 : 0) | (a.res ? 2 : 0) | (a.bb_partial ? 4 : 0) | (a.stats ? 8 : 0) |
         (a.vg_y ? 16 : 0);
}

// (K, Cout, mode) combinations with an instantiation: the ResidualBlock's conv1 forward
// (256 -> 128, BN in, stats out) and conv3 forward (128 -> 256, BN in, residual, stats out), their
// input gradients (128 -> 256 accumulate + BN-backward partials; 256 -> 128 BN-backward
// partials), and plain / statistics-only 256 -> 256 launches (lin, ll_);
// mode 20: conv1's input gradient with the BN2-backward apply folded in (its upstream gradient in);
// round 5, the 64-channel launches: the stem block (ResidualBlock(64, 128) at 128x128: conv1
// 64 -> 64, conv3 64 -> 128 + the skip conv4 64 -> 128, their input gradients), residual2's
// 128 -> 64 / 64 -> 128 at 64x64, and the heads' 64 -> 256 (try_with_torch.py:286-297; the
// statistics-only / plain variants: hourglass_compare's BN-followed convs): 1.1-1.5x
// the tiled kernel per launch (scripts/ring64_bench.py). The heads' 256 -> 64 and the 128 -> 64
// input gradients with BN-backward sums stay tiled (0.91-0.94x on the ring, profiles/r05_ring64_ab.txt)
static constexpr bool ring_have(int K, int Cout, int mode) {
  if (K == 256 && Cout == 128) return mode == 9 || mode == 4 || mode == 6 || mode == 8 || mode == 0 || mode == 2;
  if (K == 128 && Cout == 256)
    return mode == 11 || mode == 6 || mode == 4 || mode == 10 || mode == 8 || mode == 9 || mode == 0 || mode == 2 ||
           mode == 20;
  if (K == 256 && Cout == 256) return mode == 8 || mode == 9 || mode == 0 || mode == 2 || mode == 4 || mode == 1;
  if (K == 128 && Cout == 128) return mode == 0 || mode == 8 || mode == 9;
  if (K == 64 && Cout == 64) return mode == 9 || mode == 4;
  if (K == 64 && Cout == 128) return mode == 0 || mode == 11 || mode == 4 || mode == 8 || mode == 9;
  if (K == 128 && Cout == 64) return mode == 0 || mode == 9;
  if (K == 64 && Cout == 256) return mode == 10 || mode == 2 || mode == 4 || mode == 0 || mode == 8;
  return false;
}
// the ring_have table at run time (the dispatch's K / Cout pairs)
static bool ring_pair(int K, int Cout) {
  return (K == 256 && (Cout == 128 || Cout == 256)) || (K == 128 && (Cout == 256 || Cout == 128 || Cout == 64)) ||
         (K == 64 && (Cout == 64 || Cout == 128 || Cout == 256));
}

// waves per workgroup: 8 (one workgroup per CU) or, for Cout <= 128 without the folded apply,
// 4 (two per CU: -0 to -4 % per launch at 64x64, and the small launches of ring_small_ok; +0.4 %
// img/s same-box, profiles/r03_ring_nw.txt); route HGK_ROUTE_RING_NW = 8 forces the 8-wave kernel
static int ring_nw(int K, int Cout, int mode) {
  return route(HGK_ROUTE_RING_NW) == 4 && Cout <= 128 && !(mode & 16) && ring_cfg_ok(K, Cout, mode, 4) ? 4 : 8;
}

// rows at and above which a (twin) launch takes the ring kernel (HGK_ROUTE_RING_MINM; 0 = off;
// default 16384: the 32x32 level's convs at N = 32 (+0.6 %) and at N = 16 (try_with_aspp, +1.7 %),
// profiles/r04_route_ab.txt, r04_aspp_route_ab.txt)
static long ring_min_m() { return route(HGK_ROUTE_RING_MINM); }

static bool ring_shape_ok(const ConvFwdArgs& a) {
  // the instantiation table first: ring_bp() needs Cout in {128, 256}
  if (!ring_pair(a.Cin, a.Cout) || !ring_have(a.Cin, a.Cout, ring_mode(a))) return false;
  const int mode = ring_mode(a), nw = ring_nw(a.Cin, a.Cout, mode);
  return a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && a.H == a.Ho && a.W == a.Wo &&
         a.M % (ring_bp(a.Cin, a.Cout, mode, nw) * kRingU) == 0 && a.w_ld % 8 == 0;
}

// below ring_min_m(): the 4-wave kernel's smaller launches that beat the tiled routes
// (scripts/ring_bench.py, K 256 -> 128: @32 single x1.4-1.6, @16+8 twin x1.6-1.8; @16 single and
// @32+16 twin stay tiled). Route HGK_ROUTE_RING_SMALL = 0 disables
static bool ring_small_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1) {
  if (!route(HGK_ROUTE_RING_SMALL) || a.Cin != 256 || ring_nw(a.Cin, a.Cout, ring_mode(a)) != 4) return false;
  if (!a1) return a.M >= 32768;
  const long m = a.M + a1->M;
  return m >= 10240 && m <= 16384;
}

bool ring_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1) {
  const long minm = ring_min_m();
  if (minm <= 0 || !ring_shape_ok(a) || a.vg_part || (a1 && a1->vg_part)) return false;  // no folded finalize
  if (!a1) return a.M >= minm || ring_small_ok(a, nullptr);
  return ring_shape_ok(*a1) && ring_mode(*a1) == ring_mode(a) && a1->Cin == a.Cin &&
         a1->Cout == a.Cout && (a.M + a1->M >= minm || ring_small_ok(a, a1));
}

template <int K, int COUT, int MODE>
static void ring_launch_t(hipStream_t st, const RingArgs& ra, int grid, int nw) {
  if constexpr (COUT <= 128 && !(MODE & 16) && ring_cfg_ok(K, COUT, MODE, 4)) {
    if (nw == 4) {
      hipLaunchKernelGGL((conv1x1_ring_kernel<K, COUT, MODE, 4>), dim3(grid), dim3(256), 0, st, ra);
      return;
    }
  }
  hipLaunchKernelGGL((conv1x1_ring_kernel<K, COUT, MODE>), dim3(grid), dim3(512), 0, st, ra);
}

template <int K, int COUT>
static bool ring_dispatch_mode(hipStream_t st, const RingArgs& ra, int grid, int mode, int nw) {
  switch (mode) {
#define HGK_RING_CASE(m)                                 \
  case m:                                                \
    if constexpr (ring_have(K, COUT, m)) {               \
      ring_launch_t<K, COUT, m>(st, ra, grid, nw);       \
      return true;                                       \
    }                                                    \
    return false;
    HGK_RING_CASE(0) HGK_RING_CASE(1) HGK_RING_CASE(2) HGK_RING_CASE(4) HGK_RING_CASE(6)
    HGK_RING_CASE(8) HGK_RING_CASE(9) HGK_RING_CASE(10) HGK_RING_CASE(11) HGK_RING_CASE(20)
#undef HGK_RING_CASE
    default: return false;
  }
}

int launch_ring(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1) {
  const int mode = ring_mode(a0);
  if (a1 && (ring_mode(*a1) != mode || a1->Cin != a0.Cin || a1->Cout != a0.Cout)) {
    set_error("conv_fwd ring: twin segments differ");
    return HGK_ERR_ARG;
  }
  const bool stats = (mode & 8) != 0, bbm = (mode & 4) != 0;
  const int nw = ring_nw(a0.Cin, a0.Cout, mode);
  const int PG = nw / (a0.Cout / 32);
  RingArgs ra;
  memset(&ra, 0, sizeof(ra));
  int nb[2] = {0, 0}, nrg[2] = {0, 0};
  for (int s = 0; s < 2; ++s) {
    const ConvFwdArgs* a = s == 0 ? &a0 : a1;
    if (!a) break;
    nb[s] = (int)(a->M / ring_bp(a0.Cin, a0.Cout, mode, nw));
    nrg[s] = nb[s] / kRingU;
    RingSeg& g = ra.s[s];
    g.x = reinterpret_cast<const bf16_t*>(a->x);
    g.res = reinterpret_cast<const bf16_t*>(a->res);
    g.y = reinterpret_cast<bf16_t*>(a->y);
    g.pre_scale = a->pre_scale;
    g.pre_shift = a->pre_shift;
    g.stats = a->stats;
    g.bby = reinterpret_cast<const bf16_t*>(a->bb_y);
    g.bsc = a->bb_scale; g.bsh = a->bb_shift; g.bmu = a->bb_mean; g.bis = a->bb_invstd;
    g.bpart = a->bb_partial;
    g.vgy = reinterpret_cast<const bf16_t*>(a->vg_y);
    g.vsc = a->vg_scale; g.vsh = a->vg_shift; g.vco = a->vg_coef;
    g.vout = reinterpret_cast<bf16_t*>(a->vg_out);
    g.rows = nrg[s] * PG;
    if ((stats || bbm) && g.rows > kMaxStatsRows) {
      set_error("conv_fwd ring: %d partial rows exceed the maximum %d", g.rows, kMaxStatsRows);
      return HGK_ERR_UNSUPPORTED;
    }
  }
  if (!a1) ra.s[1] = ra.s[0];
  ra.w = reinterpret_cast<const bf16_t*>(a0.w);
  ra.bias = a0.bias;
  ra.w_ld = a0.w_ld;
  ra.pre_relu = a0.pre_relu;
  ra.post_relu = a0.post_relu;
  ra.bb_relu = a0.bb_relu;
  ra.vg_relu = a0.vg_relu;
  if (a1 && a1->vg_relu != a0.vg_relu) {
    set_error("conv_fwd ring: twin segments differ in the folded apply's ReLU");
    return HGK_ERR_ARG;
  }
  ra.nb0 = nb[0];
  ra.nrg0 = nrg[0];
  ra.nrg = nrg[0] + nrg[1];
  // one (NW 8) or two (NW 4) workgroups per CU (LDS), at most kRingRGMax row groups each
#ifndef HGK_RING_NW4_GRID
#define HGK_RING_NW4_GRID 512
#endif
  int grid = std::min(ra.nrg, nw == 4 ? HGK_RING_NW4_GRID : 256);
  grid = std::max(grid, ceil_div(ra.nrg, kRingRGMax));
  bool ok = false;
  const int K = a0.Cin, Cout = a0.Cout;
  if (K == 256 && Cout == 128) ok = ring_dispatch_mode<256, 128>(st, ra, grid, mode, nw);
  else if (K == 128 && Cout == 256) ok = ring_dispatch_mode<128, 256>(st, ra, grid, mode, nw);
  else if (K == 256 && Cout == 256) ok = ring_dispatch_mode<256, 256>(st, ra, grid, mode, nw);
  else if (K == 128 && Cout == 128) ok = ring_dispatch_mode<128, 128>(st, ra, grid, mode, nw);
  else if (K == 64 && Cout == 64) ok = ring_dispatch_mode<64, 64>(st, ra, grid, mode, nw);
  else if (K == 64 && Cout == 128) ok = ring_dispatch_mode<64, 128>(st, ra, grid, mode, nw);
  else if (K == 128 && Cout == 64) ok = ring_dispatch_mode<128, 64>(st, ra, grid, mode, nw);
  else if (K == 64 && Cout == 256) ok = ring_dispatch_mode<64, 256>(st, ra, grid, mode, nw);
  if (!ok) {
    set_error("conv_fwd ring: no kernel for K %d Cout %d mode %d", K, Cout, mode);
    return HGK_ERR_UNSUPPORTED;
  }
  HGK_LAUNCH_CHECK();
  a0.stats_R = ra.s[0].rows;
  if (a1) a1->stats_R = ra.s[1].rows;
  if (rows0) *rows0 = (stats || bbm) ? ra.s[0].rows : 0;
  if (rows1) *rows1 = (stats || bbm) && a1 ? ra.s[1].rows : 0;
  return HGK_OK;
}

}  // namespace hgk
