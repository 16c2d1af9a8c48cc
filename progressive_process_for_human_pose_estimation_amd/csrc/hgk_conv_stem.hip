// The stem convolution of every model (try_with_torch.py:262 / creatModel: nn.Conv2d(3, 64, 7, 2, 3)
// on the 256x256 image, ReLU after it, BN statistics of its output for residual1's bn1):
// 7x7 / stride 2 / pad 3 over the channel-padded NHWC input (8 stored channels: one 16-B chunk per
// pixel, channels 3..7 zero), 64 output channels, 128x128 output.
//
// The implicit GEMM (SMALLC path) gathered each output pixel's 49 taps as 16-B chunks per k-tile,
// 7 dependent k-tiles per 128x64 tile: 163 us for 10 GFLOP (the image is 33.5 MB). Here a
// workgroup runs a contiguous range of output rows (128 pixels x 64 channels each; ~8 per
// workgroup, two workgroups per CU), the next row's input loads in flight behind the current
// row's epilogue:
//   * the 7 input rows it needs ((2*128 + 5) positions each, zero padding applied) go to LDS once,
//     stored by column PARITY (stride 2: the 16 pixels of a fragment read 16 consecutive 16-B
//     slots of one parity row — conflict-free);
//   * every wave keeps its 16 output channels' weights in REGISTERS for all 14 k32 steps (4 taps x
//     8 channels each; K = 392 padded to 448 with zero weights, whose taps read a clamped valid
//     position), loaded once per workgroup — no weight traffic through LDS;
//   * 4 waves of 128 pixels x 16 channels: v_mfma_f32_16x16x32_bf16 with the pixels as A
//     (fragment = one tap's 8 channels of one pixel) and the weights as B;
//   * epilogue in registers: bias, bf16 rounding, ReLU, the statistics partial row of the stored
//     values (sum, M2 about the row mean, count: one row per output row, the implicit GEMM's rows
//     of 128 pixels, XCD-slot order), the tile staged in LDS for 16-B stores.
#include <algorithm>

#include "hgk_common.h"
#include "hgk_conv.h"

namespace hgk {

static constexpr int kStemWo = 128;   // output row = one workgroup tile
static constexpr int kStemKS = 14;    // k32 steps over K = 49 taps x 8 channels, padded to 448

template <int WO>
__global__ __launch_bounds__(256, 2) void conv_stem_kernel(ConvFwdArgs a, int nrows) {
  typedef bf16_t T;
  constexpr int NT = 256, BM = WO, BN = 64;
  constexpr int NP = 2 * WO + 5;   // input positions of a row: wi = -3 .. 2 WO + 1
  constexpr int HP = WO + 3;       // slots per (row, parity)
  constexpr int HALO = 7 * 2 * HP * 16;
  // waves: 16 output channels x all 128 pixels each (weights 56 registers per lane; the 2 x 2 split
  // needs 112 and spills once the epilogue and the next row's loads are live)
  constexpr int WM = 1, WN = 4, WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int LDC = BN + 8;
  constexpr int EPI = BM * LDC * 2 + 2 * WM * BN * 4;  // staged tile | per-wave-row channel sums
  constexpr int NCH = 7 * NP, HL = (NCH + NT - 1) / NT;
  // the halo and the epilogue's staging have their own LDS (the next row's halo is written while
  // the stores of this row may still read the staged tile)
  __shared__ __attribute__((aligned(16))) char sHalo[HALO];
  __shared__ __attribute__((aligned(16))) char sEpi[EPI];
  __shared__ float sBias[BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 15, lg = lane >> 4;
  // a contiguous run of output rows (key n * Ho + ho) per workgroup
  const int r0 = (int)((long)blockIdx.x * nrows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * nrows / gridDim.x);
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);

  // input rows of output row `orow` -> registers (zero padding applied); hd: LDS slot by parity
  uint4 hv[HL];
  int hd[HL];
  auto load_halo = [&](int orow) __attribute__((always_inline)) {
    const int n = orow / a.Ho, ho = orow - n * a.Ho;
#pragma unroll
    for (int j = 0; j < HL; ++j) {
      const int q = tid + j * NT;
      const int kh = q / NP, p = q - kh * NP;
      const int hi = 2 * ho - 3 + kh, wi = p - 3;
      const bool ok = q < NCH && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
      hv[j] = ok ? load16(x + (((long)n * a.H + hi) * a.W + wi) * 8) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    const int q = tid + j * NT;
    const int kh = q / NP, p = q - kh * NP;
    hd[j] = q < NCH ? ((kh * 2 + (p & 1)) * HP + (p >> 1)) * 16 : -1;
  }
  if (r0 >= r1) return;  // workgroup-uniform, before any barrier
  load_halo(r0);
  // this wave's weight fragments, loaded once for the whole run: output channel lr of tile j,
  // k = 32 s + 8 lg .. + 7
  bf16x8 wb[kStemKS][FN];
#pragma unroll
  for (int s = 0; s < kStemKS; ++s)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      wb[s][j] = *reinterpret_cast<const bf16x8*>(w + (long)(wn * WTN + j * 16 + lr) * a.w_ld + s * 32 + lg * 8);
  if (tid < BN) sBias[tid] = a.bias ? a.bias[tid] : 0.f;
  // LDS offset of this lane's tap at k-step s (taps past 48 meet zero weights: read tap 48's valid
  // slot); a few ALU ops per step instead of 14 live registers
  auto toff = [&](int s) __attribute__((always_inline)) {
    const int tap = min(4 * s + lg, 48);
    const int kh = (tap * 37) >> 8, kw = tap - kh * 7;  // tap / 7 for tap < 64
    return ((kh * 2 + (kw & 1)) * HP + (kw >> 1)) * 16;
  };
  const int pbase = (wm * WTM + lr) * 16;  // this lane's pixel (output column) in its first tile
  T* Cs = reinterpret_cast<T*>(sEpi);
  float* red = reinterpret_cast<float*>(sEpi + BM * LDC * sizeof(T));  // [sum | M2][WM][BN]
  T* __restrict__ y = reinterpret_cast<T*>(a.y);

  for (int orow = r0; orow < r1; ++orow) {
#pragma unroll
    for (int j = 0; j < HL; ++j)
      if (hd[j] >= 0) *reinterpret_cast<uint4*>(sHalo + hd[j]) = hv[j];
    __syncthreads();  // the halo is in; every wave is past the previous row's epilogue

    // ---- MFMA stream: 14 k-steps x FM x FN, no synchronisation ----
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // software-pipelined: k-step s + 1's fragment reads go out before step s's MFMAs; the
    // scheduling barrier keeps the compiler from hoisting further reads (registers: the weights
    // already hold 112 per lane)
    bf16x8 av[2][FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) av[0][i] = *reinterpret_cast<const bf16x8*>(sHalo + toff(0) + pbase + i * 256);
#pragma unroll
    for (int s = 0; s < kStemKS; ++s) {
      if (s + 1 < kStemKS) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          av[(s + 1) & 1][i] = *reinterpret_cast<const bf16x8*>(sHalo + toff(s + 1) + pbase + i * 256);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[s & 1][i], wb[s][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: bias, bf16 rounding, ReLU (post_relu) in registers (the stored values); the
    // statistics partial row from them (sum, then M2 about the row mean: the lanes of a wave by
    // shuffles, wave rows through LDS in a fixed order); the tile staged in LDS for 16-B stores ----
    float s1[FN];
    const bool relu = a.post_relu != 0;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = wn * WTN + j * 16 + lr;
      const float bj = sBias[c];
      s1[j] = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int rbase = wm * WTM + i * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = to_f(from_f<T>(acc[i][j][r] + bj));
          const T tv = from_f<T>(relu ? fmaxf(o, 0.f) : o);
          const float v = to_f(tv);
          acc[i][j][r] = v;
          s1[j] += v;
          Cs[(rbase + lg * 4 + r) * LDC + c] = tv;
        }
      }
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      if (lg == 0) red[wm * BN + c] = s1[j];
    }
    __syncthreads();  // tile staged, sums in; every halo read of this row is done
    const long prow = a.stats ? xcd_slot(orow, a.stats_R) : 0;
    float q1[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = wn * WTN + j * 16 + lr;
      float sm = red[c];
#pragma unroll
      for (int h = 1; h < WM; ++h) sm += red[h * BN + c];
      const float mean = sm / (float)BM;
      q1[j] = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[i][j][r] - mean;
          q1[j] += d * d;
        }
      q1[j] += __shfl_xor(q1[j], 16, 64);
      q1[j] += __shfl_xor(q1[j], 32, 64);
      if (lg == 0) red[(WM + wm) * BN + c] = q1[j];
      if (a.stats && wm == 0 && lg == 0) {
        a.stats[((long)c * 3 + 0) * a.stats_R + prow] = sm;
        a.stats[((long)c * 3 + 2) * a.stats_R + prow] = (float)BM;
      }
    }
    if (orow + 1 < r1) load_halo(orow + 1);  // in flight behind the stores and the next barrier
    // the output row: 128 pixels x 64 channels, 16-B chunks
#pragma unroll
    for (int u = 0; u < BM * BN / 8 / NT; ++u) {
      const int q = tid + u * NT, px = q / (BN / 8), cc = q - px * (BN / 8);
      store16(y + ((long)orow * WO + px) * BN + cc * 8,
              *reinterpret_cast<const typename Vec16<T>::type*>(&Cs[px * LDC + cc * 8]));
    }
    __syncthreads();  // M2 halves in
    if (a.stats && tid < BN) {
      float qq = red[WM * BN + tid];
#pragma unroll
      for (int h = 1; h < WM; ++h) qq += red[(WM + h) * BN + tid];
      a.stats[((long)tid * 3 + 1) * a.stats_R + prow] = qq;
    }
  }
}

bool stem_ok(const ConvFwdArgs& a) {
  return route(HGK_ROUTE_STEM) != 0 && a.Cin == 8 && a.KH == 7 && a.KW == 7 && a.stride == 2 &&
         a.pad == 3 && a.dil == 1 && a.Cout == 64 && a.Wo == kStemWo && a.W <= 2 * kStemWo + 1 &&
         a.w_ld >= kStemKS * 32 && a.w_ld % 8 == 0 && !a.pre_scale && !a.res && !a.bb_partial &&
         !a.vg_y && !a.fold_part && a.M / kStemWo <= kMaxStatsRows && a.M % kStemWo == 0;
}

// workgroups: two per CU (LDS 56 KB, <= 256 registers per lane), each a run of ~8 output rows
int launch_stem(hipStream_t st, ConvFwdArgs& a, int* rows_out) {
  const int g = (int)(a.M / kStemWo);
  a.stats_R = g;
  const int grid = std::min(g, 512);
  hipLaunchKernelGGL(conv_stem_kernel<kStemWo>, dim3(grid), dim3(256), 0, st, a, g);
  HGK_LAUNCH_CHECK();
  if (rows_out) *rows_out = a.stats ? g : 0;
  return HGK_OK;
}

}  // namespace hgk
