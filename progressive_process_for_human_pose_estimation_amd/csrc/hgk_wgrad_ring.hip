// Weight gradients of the big 1x1 convolutions on an LDS-DMA RING (round 6).
//
// dW[co][ci] = sum_p dy[p][co] * x'[p][ci] (+ db[co] = sum_p dy[p][co]) over every use of a shared
// weight (the ResidualBlock conv1 256->128 / conv3 128->256 of each hourglass level and of
// residual4, lin / ll_ 256->256: try_with_torch.py:186,192,248,295), x' = relu?(BN(x)) of that use.
// These launches stream 0.3-1.2 GB of bf16 dy / x each at ~2 MFMA cycles per byte: HBM-bound. The
// register-staged tiled kernel (conv_wgrad_multi_kernel<bf16,128,128>) keeps one 64-pixel stage
// (32 KB) per workgroup in flight and reads one operand once per tile: ~0.5 of 8 TB/s on
// algorithmic bytes. This kernel keeps bytes in flight instead (the conv1x1_ring_kernel recipe):
// * ONE 8-wave workgroup per CU, owning one (use, pixel range, 128- or 256-row co-tile): the whole
//   K (= Cin) of the weight is one tile, so each use's x rows are read once per co-tile and dy
//   rows once (256x256 weights: two co-tiles, adjacent on one XCD so the second x read is an L2 hit);
// * 32-pixel blocks: the dy rows [32][BMO] and x rows [32][K] go global -> LDS by LDS-DMA
//   (global_load_lds_dwordx4, no registers) into a RING of R = 6 slots (24 KB each: 3 - 4 blocks,
//   72 - 96 KB, in flight per CU); waits are counted vmcnt (3 DMAs per wave per block, nothing else
//   in the loop touches vector memory), one barrier per block;
// * the use's BN(+ReLU) transform of x runs once per element, in place in the slot, one block
//   ahead of the MFMAs (a thread's 16-B chunks always hold the same 8 channels: its 16 constants
//   are loaded once — a workgroup never crosses uses); the bias sums come from the same pass over
//   the dy chunks (fixed thread -> chunk map, fixed-order LDS reduction at the end);
// * MFMA 16x16x32 bf16, A = dy (co rows), B = x' (ci columns), both read as transposed fragments
//   (ds_read_b64_tr_b16, 8 pixels of one channel per lane) from rows whose 16-B chunks are
//   XOR-swizzled by (p & 7) << 1: the 8 rows x 2 chunks a 32-lane half reads hit 16 distinct
//   16-B bank groups (conflict-free), and every DMA instruction still writes 1 KB contiguously;
// * the accumulators (the workgroup's whole co-tile x K, 64 fp32 per lane) go to the use's split
//   slab once at the end (slab_rmw's [S][Cout][K] layout, accumulate when split < s_init): the
//   reduction (hgk_conv_wgrad_finish*) is unchanged.
// Deterministic (fixed block order per workgroup, fixed slab / bias order); not bitwise the tiled
// kernel's (another fp32 summation order and split plan): gated against torch fp32 and the tiled
// route (tests/test_gpu_wgrad_ring.py).
#include <algorithm>

#include "hgk_common.h"
#include "hgk_conv.h"

namespace hgk {

#ifndef HGK_WR_BP
#define HGK_WR_BP 32
#endif
static constexpr int kWrBP = HGK_WR_BP;  // pixels per block (BP / 32 MFMA k-steps)
#ifndef HGK_WR_SLOTS
#define HGK_WR_SLOTS 6
#endif
static constexpr int kWrSlots = HGK_WR_SLOTS;  // ring depth
static constexpr int kWrMaxSrc = 40;    // uses per launch (the tiled multi launch's limit)

struct WgRingSrc {
  const bf16_t* x;
  const bf16_t* dy;
  const float* pre_scale;
  const float* pre_shift;
  int pre_relu;
  int nb;  // 32-pixel blocks of this use
  int s0;  // its first split (slab index)
  int ns;  // its splits
};

struct WgRingArgs {
  WgRingSrc src[kWrMaxSrc];
  float* slab;    // [slab_cap][Cout][K]
  float* slab_b;  // [slab_cap][Cout] or null
  int nsrc, S, T, Cout, s_init;
};
static_assert(sizeof(WgRingArgs) <= 4096, "kernel argument segment");

__device__ __forceinline__ int wr_swz(int p) { return (p & 7) << 1; }

// s_waitcnt vmcnt(X) with X a compile-time count
template <int X>
__device__ __forceinline__ void wr_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X > 63 ? 63 : X) : "memory");
}

template <int BMO, int K>
#ifndef HGK_WR_WPE
#define HGK_WR_WPE 2
#endif
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(HGK_WR_WPE)))
void conv1x1_wgrad_ring_kernel(WgRingArgs ra) {
  constexpr int NT = 512, NW = 8;
  constexpr int CD = BMO / 8, CX = K / 8;            // 16-B chunks per dy / x row
  constexpr int DB = kWrBP * BMO * 2, XBY = kWrBP * K * 2;
  constexpr int SB = DB + XBY;                       // slot bytes
  constexpr int D = SB / (NW * 1024);                // 1-KB DMAs per wave per block
  constexpr int R = kWrSlots;
  static_assert(DB % (NW * 1024) == 0 && XBY % (NW * 1024) == 0, "whole DMA rounds per part");
  static_assert(CD >= 16 && CX >= 16, "swizzle needs >= 16 chunks per row");
  constexpr int WM = 2, WN = 4, WTM = BMO / WM, WTN = K / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave tile");
  constexpr int TX = kWrBP * CX / NT;  // x chunks per thread (transform)
  constexpr int TD = kWrBP * CD / NT;  // dy chunks per thread (bias)
  static_assert(TX >= 1 && TD >= 1 && (NT / CX) % 8 == 0 && (NT / CD) % 8 == 0,
                "a thread's chunks keep one channel chunk (swizzle period 8 rows)");
  __shared__ __attribute__((aligned(16))) char ring[R * SB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  // block -> (co-tile, split): the T co-tiles of a split sit 8 blocks apart (one XCD)
  const int bid = blockIdx.x, slotg = bid >> 3;
  const int tile = slotg % ra.T;
  const int split = (slotg / ra.T) * 8 + (bid & 7);
  if (split >= ra.S) return;  // workgroup-uniform
  int si = 0;
  while (si + 1 < ra.nsrc && split >= ra.src[si + 1].s0) ++si;
  const WgRingSrc& sr = ra.src[si];
  const int j = split - sr.s0;
  const int b0 = (int)((long)j * sr.nb / sr.ns), b1 = (int)((long)(j + 1) * sr.nb / sr.ns);
  const int nbw = b1 - b0;
  const int Cout = ra.Cout, co0 = tile * BMO;
  const bf16_t* __restrict__ xg = sr.x;
  const bf16_t* __restrict__ dyg = sr.dy;

  // ---- DMA geometry: instruction d of this wave = 1-KB piece d * NW + wave of the slot ----
  // (the dy part is whole DMA rounds, so whether DMA d is a dy piece is known at compile time)
  int doff[D];  // element offset of this lane's 16 B within a block (pixel 0 of the block)
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int gb = (d * NW + wave) * 1024 + lane * 16;
    if (d * NW * 1024 < DB) {
      const int s = gb / 16, p = s / CD, c = (s % CD) ^ wr_swz(p);
      doff[d] = p * Cout + co0 + c * 8;
    } else {
      const int s = (gb - DB) / 16, p = s / CX, c = (s % CX) ^ wr_swz(p);
      doff[d] = p * K + c * 8;
    }
  }
  auto issue = [&](int b, int slot) __attribute__((always_inline)) {
    b = b0 + min(b, nbw - 1);  // the tail re-loads the last block: fixed op count per iteration
    const long pix0 = (long)b * kWrBP;
    char* sbase = ring + slot * SB;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const bf16_t* src = d * NW * 1024 < DB ? dyg + pix0 * Cout : xg + pix0 * K;
      dma16(src + doff[d], sbase + (d * NW + wave) * 1024);
    }
  };
#pragma unroll
  for (int b = 0; b < R - 1; ++b) issue(b, b);

  // ---- per-workgroup constants (compiler-visible loads, waited for once below) ----
  const int xp = tid / CX, xc = (tid % CX) ^ wr_swz(xp);  // logical x chunk of this thread
  const bool has_pre = sr.pre_scale != nullptr;
  float ps[8], pb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ps[e] = has_pre ? sr.pre_scale[xc * 8 + e] : 1.f;
    pb[e] = has_pre ? sr.pre_shift[xc * 8 + e] : 0.f;
  }
  const bool relu = sr.pre_relu != 0;
  const bool do_bias = ra.slab_b != nullptr;
  float bsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bsum[e] = 0.f;

  // fragment byte offsets within a slot (lo rows; hi rows = +16 rows): row 4 lg + (lr >> 2),
  // columns 4 (lr & 3) .. +3 of fragment i / j (one 8-B half of a 16-B chunk)
  const int prow = 4 * lg + (lr >> 2), p4 = lr & 3;
  int offA[FM], offB[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int col = wm * WTM + i * 16 + 4 * p4;
    offA[i] = prow * BMO * 2 + ((((col >> 3) ^ wr_swz(prow))) << 4) + (col & 7) * 2;
  }
#pragma unroll
  for (int jj = 0; jj < FN; ++jj) {
    const int col = wn * WTN + jj * 16 + 4 * p4;
    offB[jj] = DB + prow * K * 2 + ((((col >> 3) ^ wr_swz(prow))) << 4) + (col & 7) * 2;
  }

  // in-place BN(+ReLU) of block `slot`'s x chunks and the bias sums of its dy chunks
  auto prep = [&](int slot) __attribute__((always_inline)) {
    char* sb = ring + slot * SB;
    if (has_pre) {
#pragma unroll
      for (int u = 0; u < TX; ++u) {
        uint4* cp = reinterpret_cast<uint4*>(sb + DB + (tid + u * NT) * 16);
        *cp = bn_relu_chunk<bf16_t>(*cp, ps, pb, relu);
      }
    }
    if (do_bias) {
#pragma unroll
      for (int u = 0; u < TD; ++u) {
        float f[8];
        unpack16<bf16_t>(*reinterpret_cast<const uint4*>(sb + (tid + u * NT) * 16), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[e] += f[e];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the constants (compiler vmcnt(0) at their first use waits for them and the prologue DMAs in
  // one round trip) and block 0 of every wave
  wr_wait<(R - 2) * D>();
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(ps[e]), "v"(pb[e]));
  __syncthreads();
  prep(0);

  typedef short s16x8 __attribute__((ext_vector_type(8)));
#pragma unroll 1
  for (int i = 0; i < nbw; ++i) {
    // block i + 1 landed (this wave's pieces; every wave's after the barrier), block i prepared
    wr_wait<(R - 3) * D>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // raw: __syncthreads' fence would drain the DMAs in flight
    asm volatile("" ::: "memory");
    issue(i + R - 1, (i + R - 1) % R);
    const char* sb0 = ring + (i % R) * SB;
    if (i + 1 < nbw) prep((i + 1) % R);
#pragma unroll
    for (int kk = 0; kk < kWrBP / 32; ++kk) {
    const char* sb = sb0 + kk * 32 * BMO * 2;  // dy rows 32 kk ..; the x part: + kk * 32 * K * 2 below
    const int xk = kk * 32 * (K - BMO) * 2;
    bf16x8 av[FM], bv[FN];
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      const char* p = sb + offA[a];
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(p + 16 * BMO * 2));
      s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      av[a] = __builtin_bit_cast(bf16x8, c);
    }
#pragma unroll
    for (int b = 0; b < FN; ++b) {
      const char* p = sb + xk + offB[b];
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(p + 16 * K * 2));
      s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bv[b] = __builtin_bit_cast(bf16x8, c);
    }
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }
  // drain the tail's re-loads before the LDS is reused / released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  float* slab = ra.slab + (long)split * Cout * K;
  slab_rmw<FM, FN>(slab, K, Cout, split < ra.s_init, co0 + wm * WTM + lg * 4, wn * WTN + lr, acc);
  if (do_bias) {
    // threads t, t + CD, ... hold dy chunk (t % CD) ^ swz: fixed-order sum over the NT / CD rows
    float* red = reinterpret_cast<float*>(ring);  // [NT / CD][BMO]
    const int dp = tid / CD, dc = (tid % CD) ^ wr_swz(dp);
#pragma unroll
    for (int e = 0; e < 8; ++e) red[dp * BMO + dc * 8 + e] = bsum[e];
    __syncthreads();
    for (int c = tid; c < BMO; c += NT) {
      float s = 0.f;
      for (int r = 0; r < NT / CD; ++r) s += red[r * BMO + c];
      float* d = &ra.slab_b[(long)split * Cout + co0 + c];
      *d = split < ra.s_init ? *d + s : s;
    }
  }
}

// ---- host side ----
bool wgrad_ring_shape_ok(int Cout, int Cin) {
  return (Cout == 128 && Cin == 256) || (Cout == 256 && Cin == 128) || (Cout == 256 && Cin == 256);
}

// srcs: the uses (bf16 NHWC, 1x1 / stride 1 / pad 0: M pixels each, M % 32 == 0). Plans the splits
// (every use >= 1, the rest by its share of the blocks, total <= 256 / co-tiles and <= slab_cap)
// and launches. Returns the splits written (slabs [0, S)), or -1 when the shapes do not fit.
int launch_wgrad_ring(hipStream_t st, const void* const* xs, const void* const* dys,
                      const float* const* pscale, const float* const* pshift, const int* prelu,
                      const long* Ms, int nsrc, float* slab, float* slab_b, int slab_cap, int s_init,
                      int Cout, int Cin) {
  if (nsrc < 1 || nsrc > kWrMaxSrc || !wgrad_ring_shape_ok(Cout, Cin)) return -1;
  static_assert(kWrBP % 32 == 0, "whole MFMA k-steps per block");
  const int BMO = (Cout == 256 && Cin == 128) ? 256 : 128;
  const int T = Cout / BMO;
  long nb_tot = 0;
  for (int i = 0; i < nsrc; ++i) {
    if (Ms[i] % kWrBP != 0 || Ms[i] <= 0) return -1;
    nb_tot += Ms[i] / kWrBP;
  }
  const int G = std::min(256 / T, slab_cap);
  if (G < nsrc) return -1;
  WgRingArgs a;
  int s = 0;
  for (int i = 0; i < nsrc; ++i) {
    WgRingSrc& w = a.src[i];
    w.x = reinterpret_cast<const bf16_t*>(xs[i]);
    w.dy = reinterpret_cast<const bf16_t*>(dys[i]);
    w.pre_scale = pscale[i];
    w.pre_shift = pshift[i];
    w.pre_relu = prelu[i];
    w.nb = (int)(Ms[i] / kWrBP);
    const long extra = (long)(G - nsrc) * w.nb / nb_tot;
    w.ns = (int)std::min<long>(w.nb, 1 + extra);
    w.s0 = s;
    s += w.ns;
  }
  a.slab = slab;
  a.slab_b = slab_b;
  a.nsrc = nsrc;
  a.S = s;
  a.T = T;
  a.Cout = Cout;
  a.s_init = s_init;
  const unsigned grid = (unsigned)(((s + 7) / 8) * 8 * T);
  if (BMO == 128) {
    if (Cin == 256) hipLaunchKernelGGL((conv1x1_wgrad_ring_kernel<128, 256>), dim3(grid), dim3(512), 0, st, a);
    else return -1;
  } else {
    hipLaunchKernelGGL((conv1x1_wgrad_ring_kernel<256, 128>), dim3(grid), dim3(512), 0, st, a);
  }
  return s;
}

}  // namespace hgk
