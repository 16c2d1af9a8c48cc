// The stem convolution of every model (try_with_torch.py:262 / creatModel: nn.Conv2d(3, 64, 7, 2, 3)
// on the 256x256 image, ReLU after it, BN statistics of its output for residual1's bn1):
// 7x7 / stride 2 / pad 3 over the channel-padded NHWC input (8 stored channels: one 16-B chunk per
// pixel, channels 3..7 zero), 64 output channels, 128x128 output.
//
// The implicit GEMM (SMALLC path) gathered each output pixel's 49 taps as 16-B chunks per k-tile,
// 7 dependent k-tiles per 128x64 tile: 163 us for 10 GFLOP (the image is 33.5 MB). Here a
// workgroup owns ONE output row (128 pixels x 64 channels):
//   * the 7 input rows it needs ((2*128 + 5) positions each, zero padding applied) go to LDS once,
//     stored by column PARITY (stride 2: the 16 pixels of a fragment read 16 consecutive 16-B
//     slots of one parity row — conflict-free);
//   * every wave keeps its 32 output channels' weights in REGISTERS for all 14 k32 steps (4 taps x
//     8 channels each; K = 392 padded to 448 with zero weights, whose taps read a clamped valid
//     position) — no weight traffic through LDS;
//   * 2 x 2 waves of 64 pixels x 32 channels: v_mfma_f32_16x16x32_bf16 with the pixels as A
//     (fragment = one tap's 8 channels of one pixel) and the weights as B;
//   * the shared epilogue (epi_store_half): bias, ReLU, bf16 store, statistics partial row of the
//     stored values — one row per output row, the implicit GEMM's rows (128 pixels each).
#include "hgk_common.h"
#include "hgk_conv.h"

namespace hgk {

static constexpr int kStemWo = 128;   // output row = one workgroup tile
static constexpr int kStemKS = 14;    // k32 steps over K = 49 taps x 8 channels, padded to 448

template <int WO>
__global__ __launch_bounds__(256, 2) void conv_stem_kernel(ConvFwdArgs a) {
  typedef bf16_t T;
  constexpr int NT = 256, BM = WO, BN = 64;
  constexpr int NP = 2 * WO + 5;   // input positions of a row: wi = -3 .. 2 WO + 1
  constexpr int HP = WO + 3;       // slots per (row, parity)
  constexpr int HALO = 7 * 2 * HP * 16;
  constexpr int WM = 2, WN = 2, WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int LDC = BN + 8, ECH = BN / 8, ERPP = NT / ECH;
  constexpr int EPI = BM * LDC * 2 + ERPP * BN * 4 + BN * 4;
  constexpr int SMEM = HALO > EPI ? HALO : EPI;
  constexpr int NCH = 7 * NP, HL = (NCH + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  __shared__ float sBias[BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int orow = blockIdx.x;  // output row key n * Ho + ho
  const int n = orow / a.Ho, ho = orow - n * a.Ho;
  const long m0 = (long)orow * WO;
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);

  // ---- one burst: the input rows (registers -> LDS below) and this wave's weight fragments ----
  uint4 hv[HL];
  int hd[HL];
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    const int q = tid + j * NT;
    const int kh = q / NP, p = q - kh * NP;
    const int hi = 2 * ho - 3 + kh, wi = p - 3;
    const bool ok = q < NCH && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
    hv[j] = ok ? load16(x + (((long)n * a.H + hi) * a.W + wi) * 8) : make_uint4(0u, 0u, 0u, 0u);
    hd[j] = q < NCH ? ((kh * 2 + (p & 1)) * HP + (p >> 1)) * 16 : -1;
  }
  bf16x8 wb[kStemKS][FN];  // B fragments: output channel lr of tile j, k = 32 s + 8 lg .. + 7
#pragma unroll
  for (int s = 0; s < kStemKS; ++s)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      wb[s][j] = *reinterpret_cast<const bf16x8*>(w + (long)(wn * WTN + j * 16 + lr) * a.w_ld + s * 32 + lg * 8);
  if (tid < BN) sBias[tid] = a.bias ? a.bias[tid] : 0.f;
#pragma unroll
  for (int j = 0; j < HL; ++j)
    if (hd[j] >= 0) *reinterpret_cast<uint4*>(smem + hd[j]) = hv[j];
  // this lane's tap per k-step (taps past 48 meet zero weights: read tap 48's valid slot)
  int toff[kStemKS];
#pragma unroll
  for (int s = 0; s < kStemKS; ++s) {
    const int tap = min(4 * s + lg, 48);
    const int kh = tap / 7, kw = tap - kh * 7;
    toff[s] = ((kh * 2 + (kw & 1)) * HP + (kw >> 1)) * 16;
  }
  __syncthreads();

  // ---- MFMA stream: 14 k-steps x FM x FN, no synchronisation ----
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int pbase = (wm * WTM + lr) * 16;  // this lane's pixel (output column) in its first tile
#pragma unroll
  for (int s = 0; s < kStemKS; ++s) {
    bf16x8 av[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) av[i] = *reinterpret_cast<const bf16x8*>(smem + toff[s] + pbase + i * 256);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], wb[s][j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // every halo read is done: the epilogue reuses the LDS

  // ---- epilogue: the shared staged / coalesced / statistics path ----
  T* Cs = reinterpret_cast<T*>(smem);
  float* red = reinterpret_cast<float*>(smem + BM * LDC * sizeof(T));
  float* bmean = red + ERPP * BN;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = wn * WTN + j * 16 + lr;
    const float bj = sBias[c];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rbase = wm * WTM + i * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(rbase + lg * 4 + r) * LDC + c] = from_f<T>(acc[i][j][r] + bj);
    }
  }
  __syncthreads();
  epi_store_half<T, BM, BN, NT, BM, 1>(a, Cs, red, bmean, m0, 0, 0, tid, orow);
}

bool stem_ok(const ConvFwdArgs& a) {
  return route(HGK_ROUTE_STEM) != 0 && a.Cin == 8 && a.KH == 7 && a.KW == 7 && a.stride == 2 &&
         a.pad == 3 && a.dil == 1 && a.Cout == 64 && a.Wo == kStemWo && a.W <= 2 * kStemWo + 1 &&
         a.w_ld >= kStemKS * 32 && a.w_ld % 8 == 0 && !a.pre_scale && !a.res && !a.bb_partial &&
         !a.vg_y && !a.fold_part && a.M / kStemWo <= kMaxStatsRows && a.M % kStemWo == 0;
}

int launch_stem(hipStream_t st, ConvFwdArgs& a, int* rows_out) {
  const int g = (int)(a.M / kStemWo);
  a.stats_R = g;
  hipLaunchKernelGGL(conv_stem_kernel<kStemWo>, dim3(g), dim3(256), 0, st, a);
  HGK_LAUNCH_CHECK();
  if (rows_out) *rows_out = a.stats ? g : 0;
  return HGK_OK;
}

}  // namespace hgk
