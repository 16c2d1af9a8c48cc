// Implicit-GEMM convolutions on MFMA for gfx950 (forward / input-grad-as-forward / weight grad).
//
// Forward: GEMM rows = output pixels m (NHWC), cols = output channels, contraction k over
// (kh, kw, ci). A tile = the (BN+ReLU-transformed) input pixels of one filter tap and BK input
// channels (16-byte vector loads of channel-contiguous NHWC rows), B tile = packed weights
// [Cout][K]. Both staged through LDS, k-contiguous rows, read as MFMA fragments:
//   fp32 : v_mfma_f32_16x16x4_f32   (exact fp32 fma chain; the parity path)
//   bf16 : v_mfma_f32_16x16x32_bf16 (fp32 accumulate)
// Epilogue fuses bias, residual add (in place allowed), optional ReLU and the per-channel
// (sum, sum^2) partials that the following BatchNorm needs (no second pass over y).
//
// Weight grad: GEMM rows = out channels, cols = k, contraction over output pixels, split over
// workgroups into fp32 partial slabs, reduced in a fixed order (deterministic) by a second kernel
// that ACCUMULATES into the canonical [Cout][Cin][KH][KW] fp32 grad (shared weights).
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "hgk_common.h"
#include "hgk_conv.h"

namespace hgk {


template <typename T>
struct MfmaTraits;
template <>
struct MfmaTraits<float> {
  static constexpr int KSTEP = 4;   // k per MFMA
  static constexpr int BK = 32;     // k per LDS stage
  static constexpr int PAD = 4;     // LDS row padding (elements; rows stay 16-byte aligned)
};
template <>
struct MfmaTraits<bf16_t> {
  static constexpr int KSTEP = 32;
  static constexpr int BK = 64;
  static constexpr int PAD = 16;  // 160-B rows: the 16-lane ds_read_b128 groups hit 16 distinct slots
};


// BN-constant LDS layout: for VEC = 8 the low and high 4-channel halves of every 8-channel
// chunk live in two separate contiguous arrays, so lanes reading consecutive chunks hit
// consecutive 16-B slots. (Generic Cin not a multiple of 8 keeps the identity layout.)
template <int VEC>
__device__ __forceinline__ int pre_perm(int c, int Cin) {
  if (VEC != 8 || (Cin & 7)) return c;
  return ((c >> 2) & 1) * (Cin >> 1) + (c >> 3) * 4 + (c & 3);
}
template <int VEC>
__device__ __forceinline__ void pre_load(const float* sPre, int cb, int Cin, float* ps, float* pb) {
  if constexpr (VEC == 8) {
    const int lo = (cb >> 3) * 4, hi = (Cin >> 1) + (cb >> 3) * 4;
    const float4 s0 = *reinterpret_cast<const float4*>(&sPre[lo]);
    const float4 s1 = *reinterpret_cast<const float4*>(&sPre[hi]);
    const float4 b0 = *reinterpret_cast<const float4*>(&sPre[kMaxPreC + lo]);
    const float4 b1 = *reinterpret_cast<const float4*>(&sPre[kMaxPreC + hi]);
    ps[0] = s0.x; ps[1] = s0.y; ps[2] = s0.z; ps[3] = s0.w;
    ps[4] = s1.x; ps[5] = s1.y; ps[6] = s1.z; ps[7] = s1.w;
    pb[0] = b0.x; pb[1] = b0.y; pb[2] = b0.z; pb[3] = b0.w;
    pb[4] = b1.x; pb[5] = b1.y; pb[6] = b1.z; pb[7] = b1.w;
  } else {
#pragma unroll
    for (int e = 0; e < VEC; ++e) { ps[e] = sPre[cb + e]; pb[e] = sPre[kMaxPreC + cb + e]; }
  }
}


// --------------------------------------------------------------------------------------------
// forward conv
// --------------------------------------------------------------------------------------------
// SMALLC: Cin == one 16-byte chunk (the channel-padded network input): a k-tile spans BK/VEC
// filter taps and each thread's chunk is one whole pixel of ITS tap (up to 64 taps, e.g. 7x7).
// Occupancy: the bf16 MFMA paths are held to 4 waves per SIMD (<= 128 VGPRs, accumulators out
// of AGPRs): the 1x1 convs are latency/HBM-bound and gain more from a 4th resident workgroup than
// they lose to register pressure (no spills; 1x1 @64x64 kernels 10-15 % faster, step +3 %)
#ifndef HGK_FWD64_WPE
#define HGK_FWD64_WPE 4
#endif
#ifndef HGK_SMALLC_WPE
#define HGK_SMALLC_WPE 0  // 4 waves/SIMD for the RGB-stem path too (ablation)
#endif
template <typename T, int BM, int BN, bool GENERIC, bool SMALLC, int PF>
constexpr int fwd_waves_per_eu() {
  if (PF > 1) return 1;  // few-workgroup (all-ahead) launches: registers are free
  return (sizeof(T) == 2 && !GENERIC && (!SMALLC || HGK_SMALLC_WPE)) ? (BM * BN <= 64 * 64 ? HGK_FWD64_WPE : 4) : 1;
}

// PF > 1: all-ahead mode for few-workgroup launches (small hourglass levels): the host limits a
// workgroup to PF k-tiles (split-K) and all of their loads are issued up front.
// KG > 1 (with PF > 1): KG groups of 64*WM*WN threads share the output tile and split its
// k-tiles (group g takes kt0 + g, kt0 + g + KG, ...): the serial chain of a small-level 3x3 conv
// (18 k-tiles) shrinks KG-fold without a split-K workspace + epilogue launch. Partial tiles are
// added in LDS in a fixed group order (deterministic); group 0 runs the epilogue.
//
// Twin launches (hgk_conv_fwd_twin): one grid runs TWO convolutions with the same weights on
// different inputs (an hourglass level's up-branch and down-branch blocks share their
// ResidualBlock): M-tiles [0, t0) take segment a0, tiles [t0, ...) segment a1 with tile index
// mx - t0. Single launches pass t0 = kNoTwin.
#ifdef HGK_FWD_TRACE  // timing build (scripts/fwd_trace.py only): phase stamps of workgroups 0-511
__device__ unsigned long long g_fwdtrace[512 * 16];
#define FT_STAMP(k)                                                                       \
  do {                                                                                    \
    const unsigned ft_b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;  \
    if (threadIdx.x == 0 && ft_b < 512) g_fwdtrace[ft_b * 16 + (k)] = wall_clock64();     \
  } while (0)
#else
#define FT_STAMP(k)
#endif

template <typename T, int BM, int BN, int WM, int WN, bool GENERIC, bool SPLITK, bool SMALLC, int PF,
          int KG>
__device__ __forceinline__ void conv_fwd_body(const ConvFwdArgs& a, int mx, int ny, bool seg1);

template <typename T, int BM, int BN, int WM, int WN, bool GENERIC, bool SPLITK = false,
          bool SMALLC = false, int PF = 1, int KG = 1, bool TWIN = false>
__global__ __launch_bounds__(64 * WM * WN * KG)
__attribute__((amdgpu_waves_per_eu((fwd_waves_per_eu<T, BM, BN, GENERIC, SMALLC, PF>()))))
void conv_fwd_kernel(ConvFwdArgs a0, ConvFwdArgs a1, int t0) {
  FT_STAMP(0);
  // tile order: the gy output-channel tiles of one M-tile get block ids b, b+8, ... (same XCD,
  // dispatched together), so the A tile is fetched from HBM once and re-read from that XCD's L2
  int mx = blockIdx.x, ny = blockIdx.y;
  if (!SPLITK && gridDim.y > 1) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int b = blockIdx.y * gx + blockIdx.x;
    const int g = b / (8 * gy);
    const int cnt = min(8, gx - g * 8);
    const int r = b - g * 8 * gy;
    ny = r / cnt;
    mx = g * 8 + (r - ny * cnt);
  }
  if constexpr (TWIN) {
    const bool seg1 = mx >= t0;
    alignas(8) uint32_t wr[kArgWords];
    twin_pick(a0, a1, seg1, wr);
    const ConvFwdArgs& a = *reinterpret_cast<const ConvFwdArgs*>(wr);
    conv_fwd_body<T, BM, BN, WM, WN, GENERIC, SPLITK, SMALLC, PF, KG>(a, seg1 ? mx - t0 : mx, ny, seg1);
  } else {
    conv_fwd_body<T, BM, BN, WM, WN, GENERIC, SPLITK, SMALLC, PF, KG>(a0, mx, ny, false);
  }
}


template <typename T, int BM, int BN, int WM, int WN, bool GENERIC, bool SPLITK, bool SMALLC, int PF,
          int KG>
__device__ __forceinline__ void conv_fwd_body(const ConvFwdArgs& a, int mx, int ny, bool seg1) {
  FT_STAMP(1);
  constexpr int NT = 64 * WM * WN;  // threads of ONE k-group
  static_assert(KG == 1 || PF > 1, "k-groups: all-ahead mode only");
  constexpr int BK = MfmaTraits<T>::BK;
  constexpr int LDK = BK + MfmaTraits<T>::PAD;
  constexpr int VEC = Vec16<T>::N;
  constexpr int CPR = BK / VEC;          // 16-byte chunks per tile row
  constexpr int RPP = NT / CPR;          // rows per load pass
  constexpr int A_PASSES = BM / RPP;
  constexpr int B_PASSES = (BN + RPP - 1) / RPP;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert(BM % RPP == 0, "tile rows");
  static_assert(FM >= 1 && FN >= 1, "wave tile");
  // epilogue: the output tile is staged through LDS in NH row-halves of HROWS rows, then written
  // (and residual-read, BN-stat-reduced) with 16-byte coalesced accesses
  constexpr int NH = (BM * BN * (int)sizeof(T) > 32768) ? 2 : 1;
  constexpr int HROWS = BM / NH;
  constexpr int LDC = BN + 16 / (int)sizeof(T);
  constexpr int ECH = BN / VEC;           // 16-byte chunks per output row
  constexpr int ERPP = NT / ECH;          // rows per epilogue pass
  constexpr int MAIN_BYTES = (BM + BN) * LDK * (int)sizeof(T);
  constexpr int EPI_BYTES = HROWS * LDC * (int)sizeof(T) + ERPP * BN * 4 + BN * 4;
  constexpr int RED_BYTES = (KG - 1) * BM * BN * 4;
  constexpr int SMEM0 = KG * MAIN_BYTES > EPI_BYTES ? KG * MAIN_BYTES : EPI_BYTES;
  constexpr int SMEM = SMEM0 > RED_BYTES ? SMEM0 : RED_BYTES;
  static_assert(NT % ECH == 0 && HROWS % ERPP == 0, "epilogue mapping");
  static_assert(BN <= NT, "bias staging");

  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  __shared__ __attribute__((aligned(16))) float sPre[2 * kMaxPreC];  // BN scale | shift
  __shared__ float sBias[BN];
  // folded BN finalize: the two half-channel threads' partial sums
  __shared__ double sFold[PF > 1 && KG == 1 && !GENERIC && !SMALLC && sizeof(T) == 2 ? NT : 1];
  const int g = KG > 1 ? (int)threadIdx.x / NT : 0;   // k-group
  const int tid = KG > 1 ? (int)threadIdx.x % NT : (int)threadIdx.x;
  T* As = reinterpret_cast<T*>(smem + g * MAIN_BYTES);
  T* Bs = As + BM * LDK;

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long m0 = (long)mx * BM;
  const int n0 = ny * BN;
  const int HoWo = a.Ho * a.Wo;
  // folded BN finalize (all-ahead launches only; host: Cin <= NT, rows <= kFoldRows, rows % 4 == 0)
  constexpr bool FOLDK = PF > 1 && KG == 1 && !GENERIC && !SMALLC && sizeof(T) == 2;
  const bool fold = FOLDK && a.fold_part != nullptr;
  const bool has_pre = a.pre_scale != nullptr || fold;
  // per-channel constants: their loads are issued right after the row geometry (clamped,
  // unconditional), every k-tile's loads right behind them, and they are written to LDS only
  // then — one round trip for all. The bias goes to LDS for the epilogue (no load after the k
  // loop).
  constexpr int PRE_IT = kMaxPreC / NT;
  float pre_s[PRE_IT], pre_b[PRE_IT];
  // fold: this thread's share of its channel's partial rows (sum | M2 | n runs, 16-B loads,
  // clamped). Cin <= NT / 2: two threads per channel (fh = 0, 1) take alternate row quads
  FoldRegs<FOLDK ? kFoldRows / 4 : 1> fr;
  fold_setup(a, fold, tid, NT, fr);
  float bias_v;

  // per-thread row geometry (fixed over the k loop)
  const int cv = tid % CPR;
  const int r0 = tid / CPR;
  // per row: element offset of its (kh=0, kw=0) tap pixel (may point outside the image) and a
  // bitmask of the filter taps that land inside it -> a k-tile's A address is one add
  int rb_off[A_PASSES];
  typedef typename std::conditional<SMALLC, uint64_t, uint32_t>::type TapMask;
  TapMask rb_mask[A_PASSES];
  if constexpr (!GENERIC) {
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      long m = m0 + r0 + i * RPP;
      rb_off[i] = 0;
      rb_mask[i] = 0u;
      if (m < a.M) {
        int n = (int)a.fd_howo.div((uint32_t)m);
        int rem = (int)(m - (long)n * HoWo);
        int ho = (int)a.fd_wo.div((uint32_t)rem), wo = rem - ho * a.Wo;
        const int h0 = ho * a.stride - a.pad, w0 = wo * a.stride - a.pad;
        rb_off[i] = ((n * a.H + h0) * a.W + w0) * a.Cin;
        TapMask mk = 0u;
        for (int kh = 0; kh < a.KH; ++kh) {
          const int hi = h0 + kh * a.dil;
          for (int kw = 0; kw < a.KW; ++kw) {
            const int wi = w0 + kw * a.dil;
            if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) mk |= (TapMask)1 << (kh * a.KW + kw);
          }
        }
        rb_mask[i] = mk;
      }
    }
  }

  // the per-channel constants' loads go out only now, after the row geometry: a load in flight
  // across the geometry's tap loops made the compiler wait for it there (one more serial memory
  // round trip per launch: 1.3-1.7 us of the small-level launches, scripts/fwd_trace.py)
  if (fold) {
    fold_issue(a, fr);
  } else if (has_pre) {
#pragma unroll
    for (int it = 0; it < PRE_IT; ++it) {
      const int c = min(tid + it * NT, a.Cin - 1);
      pre_s[it] = a.pre_scale[c];
      pre_b[it] = a.pre_shift[c];
    }
  }
  bias_v = (a.bias && tid < BN) ? a.bias[min(n0 + tid, a.Cout - 1)] : 0.f;
  FT_STAMP(2);
  typedef typename Vec16<T>::type V;
  static_assert(PF == 1 || (!GENERIC && !SMALLC), "PF > 1: vectorised path only");
  V areg_s[PF][A_PASSES];
  V breg_s[PF][B_PASSES];
  float ag[GENERIC ? (BM * BK / NT) : 1];
  uint32_t ag_in = 0u;  // GENERIC: which of this thread's elements are in-image taps
  static_assert(!GENERIC || BM * BK / NT <= 32, "generic in-image mask");
  const int nk = (a.K + BK - 1) / BK;

  auto load_tiles = [&](int kt, int st) __attribute__((always_inline)) {
    V* areg = areg_s[st];
    V* breg = breg_s[st];
    const int k0 = kt * BK;
    if constexpr (SMALLC) {
      const int tap = kt * CPR + cv;  // this thread's tap; its chunk = all Cin channels
      const int kh = (int)a.fd_kw.div((uint32_t)tap), kw = tap - kh * a.KW;
      const int tap_off = (kh * a.dil * a.W + kw * a.dil) * a.Cin;
      const bool tap_ok = tap < a.KH * a.KW;
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) {
        const bool ok = tap_ok && ((rb_mask[i] >> tap) & 1u);
        areg[i] = ok ? load16(x + (rb_off[i] + tap_off)) : V{};
      }
    } else if constexpr (!GENERIC) {
      const int tap = (int)a.fd_cin.div((uint32_t)k0);
      const int c0 = k0 - tap * a.Cin;
      const int kh = (int)a.fd_kw.div((uint32_t)tap), kw = tap - kh * a.KW;
      const int tap_off = (kh * a.dil * a.W + kw * a.dil) * a.Cin + c0 + cv * VEC;
      // branch-free: a padding tap loads a valid in-image address (zeroed at store time), so
      // the loads of several k-tiles in flight keep counted (not vmcnt(0)) waits
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) {
        const bool ok = (rb_mask[i] >> tap) & 1u;
        areg[i] = load16(x + (ok ? rb_off[i] + tap_off : c0 + cv * VEC));
      }
    } else {
      // raw values; the BN(+ReLU) transform runs in store_tiles (sPre is written after the first
      // k-tile's loads are issued)
      ag_in = 0u;
#pragma unroll
      for (int j = 0; j < BM * BK / NT; ++j) {
        int e = tid + j * NT;
        int r = e / BK, kc = e - (e / BK) * BK;
        long m = m0 + r;
        int kidx = k0 + kc;
        float v = 0.f;
        if (m < a.M && kidx < a.K) {
          int tap = (int)a.fd_cin.div((uint32_t)kidx), ci = kidx - tap * a.Cin;
          int kh = (int)a.fd_kw.div((uint32_t)tap), kw = tap - kh * a.KW;
          int n = (int)a.fd_howo.div((uint32_t)m);
          int rem = (int)(m - (long)n * HoWo);
          int ho = (int)a.fd_wo.div((uint32_t)rem), wo = rem - ho * a.Wo;
          int hi = ho * a.stride - a.pad + kh * a.dil, wi = wo * a.stride - a.pad + kw * a.dil;
          if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) {
            v = to_f(x[(((long)n * a.H + hi) * a.W + wi) * a.Cin + ci]);
            ag_in |= 1u << j;
          }
        }
        ag[j] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      int r = r0 + i * RPP;
      if (BN % RPP == 0 || r < BN) breg[i] = load16(w + (long)(n0 + r) * a.w_ld + k0 + cv * VEC);
    }
  };

  auto store_tiles = [&](int kt, int st) __attribute__((always_inline)) {
    V* areg = areg_s[st];
    V* breg = breg_s[st];
    const int k0 = kt * BK;
    if constexpr (SMALLC) {
      const int tap = kt * CPR + cv;
      float ps[VEC], pb[VEC];
      if (has_pre) pre_load<VEC>(sPre, 0, a.Cin, ps, pb);
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) {
        const int r = r0 + i * RPP;
        const bool ok = tap < a.KH * a.KW && ((rb_mask[i] >> tap) & 1u);
        const V v = (has_pre && ok) ? bn_relu_chunk<T>(areg[i], ps, pb, a.pre_relu != 0) : areg[i];
        store16(&As[r * LDK + cv * VEC], v);
      }
    } else if constexpr (!GENERIC) {
      const int tap = (int)a.fd_cin.div((uint32_t)k0);
      const int c0 = k0 - tap * a.Cin;
      float ps[VEC], pb[VEC];
      if (has_pre) pre_load<VEC>(sPre, c0 + cv * VEC, a.Cin, ps, pb);
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) {
        const int r = r0 + i * RPP;
        const bool ok = (rb_mask[i] >> tap) & 1u;
        // padding taps stay exactly 0 (the conv pads AFTER BN+ReLU)
        const V v = !ok ? V{} : has_pre ? bn_relu_chunk<T>(areg[i], ps, pb, a.pre_relu != 0) : areg[i];
        store16(&As[r * LDK + cv * VEC], v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < BM * BK / NT; ++j) {
        int e = tid + j * NT;
        int r = e / BK, kc = e - (e / BK) * BK;
        float v = ag[j];
        if (has_pre && ((ag_in >> j) & 1u)) {  // padding taps stay exactly 0
          const int kidx = k0 + kc;
          const int tap = (int)a.fd_cin.div((uint32_t)kidx), ci = kidx - tap * a.Cin;
          const int pc = pre_perm<VEC>(ci, a.Cin);
          v = v * sPre[pc] + sPre[kMaxPreC + pc];
          if (a.pre_relu) v = fmaxf(v, 0.f);
        }
        As[r * LDK + kc] = from_f<T>(v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      int r = r0 + i * RPP;
      if (BN % RPP == 0 || r < BN) store16(&Bs[r * LDK + cv * VEC], breg[i]);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  auto mma_tile = [&]() {
    if constexpr (sizeof(T) == 4) {
      const float* Af = reinterpret_cast<const float*>(As);
      const float* Bf = reinterpret_cast<const float*>(Bs);
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        float av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) av[i] = Af[(wm * WTM + i * 16 + lr) * LDK + kk * 4 + lg];
#pragma unroll
        for (int j = 0; j < FN; ++j) bv[j] = Bf[(wn * WTN + j * 16 + lr) * LDK + kk * 4 + lg];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          av[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WTM + i * 16 + lr) * LDK + kk * 32 + lg * 8]);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bv[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WTN + j * 16 + lr) * LDK + kk * 32 + lg * 8]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // split-K (small M): this workgroup multiplies k-tiles [kt0, kt1) only
  const int kt0 = SPLITK ? (int)blockIdx.z * a.kt_per_split : 0;
  const int kt1 = SPLITK ? min(nk, kt0 + a.kt_per_split) : nk;
#pragma unroll
  for (int s = 0; s < PF; ++s) {
    const int k = kt0 + g + KG * s;  // KG == 1: kt0 + s
    if (k < kt1) load_tiles(k, s);
  }
  FT_STAMP(3);

  if (fold) {
    // the finalize of the BN in front of this conv, from its partials (loads issued above, ahead
    // of the k-tiles); the launch's (segment's) first workgroup publishes it
    fold_merge(a, fr, tid, sFold, mx == 0 && ny == 0 && (!SPLITK || blockIdx.z == 0), pre_s[0],
               pre_b[0]);
  }
  if (has_pre) {
    // permuted so a 16-lane ds_read_b128 group reads 16 CONTIGUOUS 16-B chunks (conflict-free)
#pragma unroll
    for (int it = 0; it < PRE_IT; ++it) {
      const int c = tid + it * NT;
      if (c < a.Cin) {
        const int pc = pre_perm<VEC>(c, a.Cin);
        sPre[pc] = pre_s[it];
        sPre[kMaxPreC + pc] = pre_b[it];
      }
    }
  }
  if (tid < BN) sBias[tid] = (n0 + tid < a.Cout) ? bias_v : 0.f;
  FT_STAMP(4);
  __syncthreads();
  FT_STAMP(5);
  if constexpr (KG > 1) {
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      if (kt0 + KG * s >= kt1) break;  // uniform: no group has a k-tile at this step
      const int k = kt0 + g + KG * s;
      if (k < kt1) store_tiles(k, s);
      __syncthreads();
      if (k < kt1) mma_tile();
      __syncthreads();
    }
    // fixed-order cross-group sum of the partial tiles (layout [slot][NT]: conflict-free)
    constexpr int NACC = FM * FN * 4;
    float* xr = reinterpret_cast<float*>(smem);
    if (g > 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            xr[((g - 1) * NACC + (i * FN + j) * 4 + r) * NT + tid] = acc[i][j][r];
    }
    __syncthreads();
    if (g == 0) {
      for (int gg = 1; gg < KG; ++gg)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc[i][j][r] += xr[((gg - 1) * NACC + (i * FN + j) * 4 + r) * NT + tid];
    }
  } else {
  store_tiles(kt0, 0);
  __syncthreads();
  FT_STAMP(6);

  if constexpr (PF == 1) {
    for (int kt = kt0; kt < kt1; ++kt) {
      if (kt + 1 < kt1) load_tiles(kt + 1, 0);
      mma_tile();
      __syncthreads();
      if (kt + 1 < kt1) {
        store_tiles(kt + 1, 0);
        __syncthreads();
      }
    }
  } else {
    // all-ahead (few-workgroup launches, host guarantees kt1 - kt0 <= PF): every k-tile's loads
    // were issued above before any wait, so the whole K range costs ONE memory round trip
    // (a rolling prefetch lost its overlap to conservative vmcnt(0) waits at the loop back-edge)
#pragma unroll
    for (int s = 1; s < PF; ++s) {
      if (kt0 + s - 1 < kt1) {
        mma_tile();
        __syncthreads();
        FT_STAMP(6 + s);
        if (kt0 + s < kt1) {
          store_tiles(kt0 + s, s);
          __syncthreads();
        }
      }
    }
    if (kt0 + PF - 1 < kt1) mma_tile();
  }
  }  // KG == 1
  FT_STAMP(11);

  if constexpr (SPLITK) {
    if (g != 0) return;  // k-groups: group 0 holds the summed tile
    // raw fp32 partial tile; conv_splitk_epilogue_kernel sums the splits in a fixed order
    float* ws = a.split_ws + (long)blockIdx.z * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * WTN + j * 16 + lr;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long row = m0 + wm * WTM + i * 16 + lg * 4 + r;
          if (col < a.Cout && row < a.M) {
            if (KG == 1 && a.split_ctr)  // sc1 (write-through): read by another CU's fix-up
              __hip_atomic_store(ws + row * a.Cout + col, acc[i][j][r], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            else
              ws[row * a.Cout + col] = acc[i][j][r];
          }
        }
    }
    if constexpr (KG == 1) {
      if (a.split_ctr) {
        // split-K fix-up: the last split of this tile to arrive sums all splits (fixed split
        // order: bitwise what conv_splitk_epilogue_kernel computes) and runs the epilogue —
        // one launch instead of two. Arrival: every wave's sc1 stores drained, a barrier, one
        // agent-scope add whose returned value names the last arriver (MI355X_MICROARCH.md,
        // hand-off table row 1); the last arriver resets the counter for the next launch.
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* ctr = a.split_ctr + blockIdx.y * gridDim.x + blockIdx.x;
        if (threadIdx.x == 0) {
          const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const int last = old == (int)gridDim.z - 1;
          if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_last = last;
        }
        __syncthreads();
        FT_STAMP(12);
        if (s_last) splitk_epilogue_body<T, BM, BN, true>(a, mx, n0);
        FT_STAMP(15);
      }
    }
    return;
  }

  // ---- epilogue ----
  T* Cs = reinterpret_cast<T*>(smem);                                   // [HROWS][LDC]
  float* red = reinterpret_cast<float*>(smem + HROWS * LDC * sizeof(T));  // [ERPP][BN]
  float* bmean = red + ERPP * BN;                                      // [BN]
  float bias_r[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bias_r[j] = sBias[wn * WTN + j * 16 + lr];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    __syncthreads();  // main-loop tiles / previous half no longer read
    // 1) fragments -> LDS (acc + bias, rounded to T)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rbase = wm * WTM + i * 16;
      if (g != 0 || rbase < h * HROWS || rbase >= (h + 1) * HROWS) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * WTN + j * 16 + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(rbase - h * HROWS + lg * 4 + r) * LDC + c] = from_f<T>(acc[i][j][r] + bias_r[j]);
      }
    }
    __syncthreads();
    FT_STAMP(12 + h);
    epi_store_half<T, BM, BN, NT, HROWS, NH>(a, Cs, red, bmean, m0, n0, h, tid, mx, g == 0);
  }
  FT_STAMP(15);
}

// --------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 forward conv (and every 3x3 input gradient), bf16, Cin % 64 == 0:
// spatial halo tiling. A workgroup owns TH x 16 output pixels of one image and 128 output
// channels. Per 64-channel input chunk the (TH+2) x 18 halo of the input is staged ONCE in LDS,
// already BN(+ReLU)-transformed and zero-padded, and all 9 taps read their A fragments from it at
// shifted positions — the implicit GEMM above re-loads and re-transforms every input pixel once
// per tap (9x the global loads and the VALU work). Weights stream per (tap, chunk) through a
// 3-deep LDS-DMA ring (two steps in flight behind counted vmcnt waits: with one, every step waited
// a full L2 round trip for its 16 KB); the halo is single-buffered (restaged between chunks)
// to pay for the third weight slot. LDS rows are 128 B with 16-B chunk c of position p in slot
// c ^ (p & 7): conflict-free for the shifted fragment reads and the halo writes alike. 73 KB
// LDS -> 2 workgroups per CU.
// --------------------------------------------------------------------------------------------
// KG = 2 (the 32x32 level: one workgroup per CU, 18 serial tap steps): two 4-wave groups, each
// with its own halo buffer and weight ring, take alternate 64-channel chunks; their partial tiles
// are added in LDS (fixed order) and group 0 runs the epilogue.
// BN = 64: the 64-channel 3x3 of the stem block at 128x128 (one 64-channel chunk)
template <int TH, int KG, int BN>
__device__ __forceinline__ void halo_body(const ConvFwdArgs& a, int tile, int nt);

// TWIN: one grid over two convolutions' tiles (see conv_fwd_kernel), tiles [0, t0) segment a0
template <int TH, int KG = 1, int BN = 128, bool TWIN = false>
__global__ __launch_bounds__(256 * KG) void conv3x3_halo_kernel(ConvFwdArgs a0, ConvFwdArgs a1,
                                                               int t0) {
  // tile coordinates: blockIdx.x = (image, tile row, tile col), blockIdx.y = output-channel tile;
  // XCD-contiguous remap so neighbouring tiles (shared halo rows) share an L2
  const int gx = gridDim.x, gy = gridDim.y, nb = gx * gy;
  const int bid = blockIdx.y * gx + blockIdx.x;
  const int xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
  const int vid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = vid / gy, nt = vid - tile * gy;
  if constexpr (TWIN) {
    const bool seg1 = tile >= t0;
    alignas(8) uint32_t wr[kArgWords];
    twin_pick(a0, a1, seg1, wr);
    halo_body<TH, KG, BN>(*reinterpret_cast<const ConvFwdArgs*>(wr), seg1 ? tile - t0 : tile, nt);
  } else {
    halo_body<TH, KG, BN>(a0, tile, nt);
  }
}

template <int TH, int KG, int BN>
__device__ __forceinline__ void halo_body(const ConvFwdArgs& a, int tile, int nt) {
  typedef bf16_t T;
  constexpr int NT = 256, TW = 16;
  constexpr int BM = TH * TW;
  constexpr int WM = 2, WN = 2, WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int HW = TW + 2, HPOS = (TH + 2) * HW;
  constexpr int RB = 128;
  constexpr int HALO = HPOS * RB, BBYTES = BN * RB;
  constexpr int HCH = HPOS * 8, HLD = (HCH + NT - 1) / NT;
  constexpr int B_LD = BN * 8 / NT;
  constexpr int NBUF = 3;
  constexpr int OFF_B = HALO;
  constexpr int MAIN = OFF_B + NBUF * BBYTES;
  constexpr int NH = 1, HROWS = BM;
  constexpr int LDC = BN + 8, ECH = BN / 8, ERPP = NT / ECH;
  constexpr int EPI = HROWS * LDC * 2 + ERPP * BN * 4 + BN * 4;
  static_assert(EPI <= MAIN, "epilogue fits the main-loop LDS");
  static_assert((KG - 1) * BM * BN * 4 <= KG * MAIN, "group reduction fits");
  __shared__ __attribute__((aligned(16))) char smem[KG * MAIN];
  // BN scale | shift of all input channels (Cin <= kHaloPreC) and the bias, staged once
  __shared__ __attribute__((aligned(16))) float sPre[2 * kHaloPreC];
  __shared__ float sBias[BN];

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);
  const int g = KG > 1 ? (int)threadIdx.x / NT : 0;
  const int tid = KG > 1 ? (int)threadIdx.x % NT : (int)threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  char* gsm = smem + g * MAIN;  // this group's halo buffer + weight ring
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int tiles_w = a.W / TW, tiles_img = (a.H / TH) * tiles_w;
  const int img = tile / tiles_img, trem = tile - img * tiles_img;
  const int h0 = (trem / tiles_w) * TH, w0 = (trem % tiles_w) * TW;
  const int n0 = nt * BN;
  const bool has_pre = a.pre_scale != nullptr;
  const bool relu = a.pre_relu != 0;

  // halo staging: thread t handles chunks q = t + j*256 -> position q/8, channel slot t%8
  const int c8 = tid & 7;
  int hoff[HLD];      // element offset of the position's pixel (channel 0), or -1 if padding
  int hdst[HLD];      // LDS byte offset within a halo buffer, or -1 past the halo
#pragma unroll
  for (int j = 0; j < HLD; ++j) {
    const int q = tid + j * NT;
    const int pos = q >> 3;
    hdst[j] = q < HCH ? pos * RB + ((c8 ^ (pos & 7)) << 4) : -1;
    const int hr = pos / HW, hc = pos - hr * HW;
    const int hi = h0 - 1 + hr, wi = w0 - 1 + hc;
    const bool in = q < HCH && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
    hoff[j] = in ? ((img * a.H + hi) * a.W + wi) * a.Cin : -1;
  }
  uint4 hreg[HLD];
#ifdef HGK_ABL_HALO_VG2
  // ablation (timing only, wrong results): the cost of a folded BN-backward apply — a second
  // operand loaded with the halo and every interior chunk stored once more
  uint4 yreg[HLD];
#endif
  auto halo_load = [&](int cc) {
#pragma unroll
    for (int j = 0; j < HLD; ++j) {
      const int off = hoff[j] >= 0 ? hoff[j] : 0;  // padding: any in-bounds row, zeroed below
      hreg[j] = *reinterpret_cast<const uint4*>(x + off + cc * 64 + c8 * 8);
#ifdef HGK_ABL_HALO_VG2
      yreg[j] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.y) + off + cc * 64 + c8 * 8);
#endif
    }
  };
  auto halo_store = [&](int cc) {
    float ps[8], pb[8];
    if (has_pre) {
      const float4 s0 = *reinterpret_cast<const float4*>(sPre + cc * 64 + c8 * 8);
      const float4 s1 = *reinterpret_cast<const float4*>(sPre + cc * 64 + c8 * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(sPre + kHaloPreC + cc * 64 + c8 * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(sPre + kHaloPreC + cc * 64 + c8 * 8 + 4);
      ps[0] = s0.x; ps[1] = s0.y; ps[2] = s0.z; ps[3] = s0.w;
      ps[4] = s1.x; ps[5] = s1.y; ps[6] = s1.z; ps[7] = s1.w;
      pb[0] = b0.x; pb[1] = b0.y; pb[2] = b0.z; pb[3] = b0.w;
      pb[4] = b1.x; pb[5] = b1.y; pb[6] = b1.z; pb[7] = b1.w;
    }
    char* hb = gsm;
#pragma unroll
    for (int j = 0; j < HLD; ++j) {
      if (hdst[j] < 0) continue;
      uint4 v = hreg[j];
      if (has_pre) v = bn_relu_chunk<bf16_t>(v, ps, pb, relu);
#ifdef HGK_ABL_HALO_VG2
      {
        float fd[8], fy[8], o[8];
        unpack16<bf16_t>(v, fd);
        unpack16<bf16_t>(yreg[j], fy);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = bnb_apply(fd[e], fy[e], 1.f, 0.f, 0.5f, 0.25f, 0.f, 0.1f, true);
        v = pack16<bf16_t>(o);
        const int q = tid + j * NT, pos = q >> 3, hr = pos / HW, hc = pos - hr * HW;
        if (hoff[j] >= 0 && hr >= 1 && hr <= TH && hc >= 1 && hc <= TW)
          *reinterpret_cast<uint4*>(reinterpret_cast<T*>(a.y) + hoff[j] * a.Cout / a.Cin + cc * 64 + c8 * 8) = v;
      }
#endif
      const uint32_t keep = hoff[j] >= 0 ? 0xffffffffu : 0u;  // zero padding AFTER the transform
      v.x &= keep; v.y &= keep; v.z &= keep; v.w &= keep;
      *reinterpret_cast<uint4*>(hb + hdst[j]) = v;
    }
  };
  // weight DMA: LDS row (wave*B_LD + j)*8 + lane/8 <- packed row n0 + that, chunk (lane%8)^(lane/8)
  const int gch = (lane & 7) ^ (lane >> 3);
  const T* wrow[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j)
    wrow[j] = w + (long)(n0 + (wave * B_LD + j) * 8 + (lane >> 3)) * a.w_ld + gch * 8;
  const int ncc = a.Cin / 64;
  const int nsteps = 9 * ncc / KG;  // this group's steps (host: ncc % KG == 0)
  auto issue_b = [&](int lstep, int buf) {
    // group-local step -> (chunk, tap): this group's chunks are g, g + KG, ...
    const int cc = (lstep / 9) * KG + g, tap = lstep - (lstep / 9) * 9;
    const int k0 = tap * a.Cin + cc * 64;
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      dma16(wrow[j] + k0, gsm + OFF_B + buf * BBYTES + (wave * B_LD + j) * 8 * RB);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: per-channel constants, weights of step 0 and the halo of chunk 0 in flight
  // together (one round trip), constants -> LDS, then the halo of chunk 0 staged
  float pv_s = 0.f, pv_b = 0.f;
  if (has_pre) {
    const int c = min(tid, a.Cin - 1);
    pv_s = a.pre_scale[c];
    pv_b = a.pre_shift[c];
  }
  const float bias_v = (a.bias && tid < BN) ? a.bias[min(n0 + tid, a.Cout - 1)] : 0.f;
  issue_b(0, 0);
  if (nsteps > 1) issue_b(1, 1);
  halo_load(g);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (has_pre && tid < a.Cin) { sPre[tid] = pv_s; sPre[kHaloPreC + tid] = pv_b; }
  if (tid < BN) sBias[tid] = (n0 + tid < a.Cout) ? bias_v : 0.f;
  __syncthreads();
  halo_store(g);

  for (int cc = g; cc < ncc; cc += KG) {
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int step = ((cc - g) / KG) * 9 + tap;  // group-local
      // this step's weights landed: younger in the vm queue are the next step's B_LD DMAs and,
      // at taps 1-2, the next chunk's halo loads (issued at tap 0) -> counted waits. The
      // barrier publishes the weights (and the halo) and retires every read of the slot
      // refilled below (last read at step - 1)
      if (step + 1 >= nsteps)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      else if ((tap == 1 || tap == 2) && cc + KG < ncc)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(B_LD + HLD) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(B_LD) : "memory");
      __builtin_amdgcn_s_barrier();
#ifndef HGK_ABL_HALO_NODMA  // ablation: weights of steps 0-1 only (wrong results; timing only)
      if (step + 2 < nsteps) issue_b(step + 2, (step + 2) % NBUF);
#endif
      if (tap == 0 && cc + KG < ncc) halo_load(cc + KG);   // lands behind the weight DMAs
      const char* Hb = gsm;
      const char* Bb = gsm + OFF_B + (step % NBUF) * BBYTES;
      const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int cidx = kk * 4 + lg;
        bf16x8 av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int pos = (wm * FM + i + kh) * HW + lr + kw;
          av[i] = *reinterpret_cast<const bf16x8*>(Hb + pos * RB + ((cidx ^ (pos & 7)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bv[j] = *reinterpret_cast<const bf16x8*>(Bb + (wn * WTN + j * 16 + lr) * RB +
                                                   ((cidx ^ (lr & 7)) << 4));
#ifdef HGK_ABL_HALO_NOMFMA  // ablation: fragments read, no MFMAs (wrong results; timing only)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(av[i]), "v"(bv[j]));
#else
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
#endif
      }
    }
    if (cc + KG < ncc) {
      // every wave is done with this chunk's halo: restage it with the next chunk (its loads,
      // issued at tap 0, are older than the two weight steps in flight)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * B_LD) : "memory");
      __syncthreads();
      halo_store(cc + KG);
    }
  }
  if constexpr (KG > 1) {
    // fixed-order cross-group sum of the partial tiles (layout [slot][NT]: conflict-free)
    constexpr int NACC = FM * FN * 4;
    __syncthreads();  // every group is done with its halo / weight buffers
    float* xr = reinterpret_cast<float*>(smem);
    if (g > 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            xr[((g - 1) * NACC + (i * FN + j) * 4 + r) * NT + tid] = acc[i][j][r];
    }
    __syncthreads();
    if (g == 0) {
      for (int gg = 1; gg < KG; ++gg)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc[i][j][r] += xr[((gg - 1) * NACC + (i * FN + j) * 4 + r) * NT + tid];
    }
  }

  // ---- epilogue: the shared staged / coalesced / statistics path over the spatial tile ----
  __syncthreads();
  T* Cs = reinterpret_cast<T*>(smem);
  float* red = reinterpret_cast<float*>(smem + HROWS * LDC * sizeof(T));
  float* bmean = red + ERPP * BN;
  float bias_r[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bias_r[j] = sBias[wn * WTN + j * 16 + lr];
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rbase = wm * WTM + i * 16;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * WTN + j * 16 + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(rbase + lg * 4 + r) * LDC + c] = from_f<T>(acc[i][j][r] + bias_r[j]);
      }
    }
  }
  __syncthreads();
  const long m0 = ((long)img * a.Ho + h0) * a.Wo + w0;
  epi_store_half<T, BM, BN, NT, HROWS, NH, TW>(a, Cs, red, bmean, m0, n0, 0, tid, tile, g == 0);
}

// split-K epilogue: sum the ksplit fp32 partial tiles (fixed order), + bias, then the shared
// coalesced store / residual / ReLU / statistics epilogue.
template <typename T, int BM, int BN, bool SC1 = false>
__device__ __forceinline__ void splitk_epilogue_body(const ConvFwdArgs& a, int bx, int n0);

template <typename T, int BM, int BN, bool TWIN = false>
__global__ __launch_bounds__(256) void conv_splitk_epilogue_kernel(ConvFwdArgs a0, ConvFwdArgs a1,
                                                                    int t0) {
  if constexpr (TWIN) {  // twin launch: see conv_fwd_kernel
    const bool seg1 = (int)blockIdx.x >= t0;
    alignas(8) uint32_t wr[kArgWords];
    twin_pick(a0, a1, seg1, wr);
    const ConvFwdArgs& a = *reinterpret_cast<const ConvFwdArgs*>(wr);
    splitk_epilogue_body<T, BM, BN>(a, (int)blockIdx.x - (seg1 ? t0 : 0), blockIdx.y * BN);
  } else {
    splitk_epilogue_body<T, BM, BN>(a0, blockIdx.x, blockIdx.y * BN);
  }
}

// SC1: the in-conv fix-up (conv_fwd_body): every load of the other splits' partials is an sc1
// load (L1 bypassed; the producers stored them sc1 and drained before their arrival add)
template <typename T, int BM, int BN, bool SC1>
__device__ __forceinline__ void splitk_epilogue_body(const ConvFwdArgs& a, int bx, int n0) {
  constexpr int NT = 256;
  constexpr int NH = (BM * BN * (int)sizeof(T) > 32768) ? 2 : 1;
  constexpr int HROWS = BM / NH;
  constexpr int LDC = BN + 16 / (int)sizeof(T);
  constexpr int ECH = BN / 4;     // float4 chunks per row of the fp32 partials
  constexpr int ERPP = NT / ECH;
  constexpr int SVEC = Vec16<T>::N;
  constexpr int SRPP = NT / (BN / SVEC);
  __shared__ __attribute__((aligned(16))) char smem[HROWS * LDC * sizeof(T) + SRPP * BN * 4 + BN * 4];
  T* Cs = reinterpret_cast<T*>(smem);
  float* red = reinterpret_cast<float*>(smem + HROWS * LDC * sizeof(T));
  float* bmean = red + SRPP * BN;
  const int tid = threadIdx.x;
  const long m0 = (long)bx * BM;
  const int cv = tid % ECH, r0 = tid / ECH;
  const int col = n0 + cv * 4;
  constexpr int RPT = HROWS / ERPP;  // rows per thread per half
  static_assert(HROWS % ERPP == 0, "rows per thread");
  const bool vec = (a.Cout & 3) == 0 && col + 4 <= a.Cout;
  // bias: loaded once up front (not a guarded load per element after the sums)
  float bias4[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bias4[e] = a.bias ? a.bias[min(col + e, a.Cout - 1)] : 0.f;
#pragma unroll 1
  for (int h = 0; h < NH; ++h) {
    __syncthreads();
    float v[RPT][4];
#pragma unroll
    for (int u = 0; u < RPT; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[u][e] = 0.f;
    if (vec) {
      // clamped, unconditional 16-B loads: 4 splits x RPT rows in flight, each row summed in
      // split order (deterministic)
      const float* src[RPT];
#pragma unroll
      for (int u = 0; u < RPT; ++u)
        src[u] = a.split_ws + min(m0 + h * HROWS + r0 + u * ERPP, a.M - 1) * a.Cout + col;
      const long sstride = a.M * a.Cout;
      for (int sp = 0; sp < a.ksplit; sp += 4) {
        float4 q[RPT][4];
        if constexpr (SC1) {
          f32x4 qv[RPT][4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const long so = (long)min(sp + k, a.ksplit - 1) * sstride;
#pragma unroll
            for (int u = 0; u < RPT; ++u)
              asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(qv[u][k]) : "v"(src[u] + so) : "memory");
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
              asm volatile("" : "+v"(qv[u][k]));  // the values are read after the wait only
              q[u][k] = make_float4(qv[u][k][0], qv[u][k][1], qv[u][k][2], qv[u][k][3]);
            }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const long so = (long)min(sp + k, a.ksplit - 1) * sstride;
#pragma unroll
            for (int u = 0; u < RPT; ++u) q[u][k] = *reinterpret_cast<const float4*>(src[u] + so);
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (sp + k >= a.ksplit) break;
#pragma unroll
          for (int u = 0; u < RPT; ++u) {
            v[u][0] += q[u][k].x; v[u][1] += q[u][k].y;
            v[u][2] += q[u][k].z; v[u][3] += q[u][k].w;
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        const long row = m0 + h * HROWS + r0 + u * ERPP;
        if (row >= a.M) continue;
        for (int sp = 0; sp < a.ksplit; ++sp) {
          const float* src = a.split_ws + ((long)sp * a.M + row) * a.Cout + col;
          for (int e = 0; e < 4; ++e)
            if (col + e < a.Cout)
              v[u][e] += SC1 ? __hip_atomic_load(src + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : src[e];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(r0 + u * ERPP) * LDC + cv * 4 + e] = from_f<T>(v[u][e] + (col + e < a.Cout ? bias4[e] : 0.f));
    __syncthreads();
    epi_store_half<T, BM, BN, NT, HROWS, NH>(a, Cs, red, bmean, m0, n0, h, tid, bx);
  }
}

#ifdef HGK_FWD_TRACE
}  // namespace hgk
extern "C" int hgk_debug_fwd_trace(void* dst, int reset) {
  if (reset) {
    static unsigned long long zero[512 * 16];
    return hipMemcpyToSymbol(HIP_SYMBOL(hgk::g_fwdtrace), zero, sizeof(zero)) == hipSuccess ? 0 : 1;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(hgk::g_fwdtrace), sizeof(hgk::g_fwdtrace)) == hipSuccess ? 0 : 1;
}
namespace hgk {
#endif

// host: stats rows a conv_fwd launch with tile BM x BN reports
template <typename T, int BM, int BN>
constexpr int conv_stats_halves() {
  return (BM * BN * (int)sizeof(T) > 32768) ? 2 : 1;
}

// --------------------------------------------------------------------------------------------
// weight gradient
// --------------------------------------------------------------------------------------------
struct ConvWgradArgs {
  const void* x;
  const void* dy;
  const float* pre_scale;
  const float* pre_shift;
  float* slab;    // [S][Cout][K]
  float* slab_b;  // [S][Cout] or null
  int pre_relu;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, dil;
  int K;
  long M;
  long pix_per_split;
  FastDiv fd_howo, fd_wo, fd_cin, fd_kw;
  int gco, gk, S;  // co-tiles, k-tiles, pixel splits (1-D grid, XCD-grouped)
  int s_init;       // slabs [0, s_init) already hold partials of earlier uses: accumulate into them
};

template <typename T>
struct WgradTraits;
template <>
struct WgradTraits<float> {
  static constexpr int BP = 64;  // pixels per LDS stage
  static constexpr int PAD = 4;
};
template <>
struct WgradTraits<bf16_t> {
  static constexpr int BP = 64;
  static constexpr int PAD = 16;  // row stride = 8 (mod 64) dwords for 128-wide, 40 for 64-wide
};

template <typename T, int BMO, int BNO, int WM, int WN, bool GENERIC>
__global__ __launch_bounds__(64 * WM * WN) void conv_wgrad_kernel(ConvWgradArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BP = WgradTraits<T>::BP;
  constexpr int PADW = WgradTraits<T>::PAD;
  constexpr int LDD = BMO + PADW;  // Ds[BP][LDD]
  constexpr int LDX = BNO + PADW;  // Xs[BP][LDX]
  constexpr int VEC = Vec16<T>::N;
  constexpr int CPR_D = BMO / VEC, RPP_D = NT / CPR_D, D_PASSES = BP / RPP_D;
  constexpr int CPR_X = BNO / VEC, RPP_X = NT / CPR_X, X_PASSES = BP / RPP_X;
  constexpr int WTM = BMO / WM, WTN = BNO / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert(D_PASSES >= 1 && X_PASSES >= 1, "tile");
  constexpr int GEL = (BP * BNO) / NT;  // generic elements per thread

  __shared__ __attribute__((aligned(16))) T Ds[BP * LDD];
  __shared__ __attribute__((aligned(16))) T Xs[BP * LDX];
  __shared__ __attribute__((aligned(16))) float sPre[2 * kMaxPreC];

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.dy);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware decomposition (speed only, never correctness): blocks b and b+8 share an XCD under
  // round-robin dispatch, so the gco*gk tiles of ONE pixel split are given block ids that differ by
  // multiples of 8 -> they re-read that split's dy / input rows from the same 4 MB L2, not HBM.
  const int b = blockIdx.x;
  const int tiles = a.gco * a.gk;
  const int slot = b >> 3;
  const int group = slot / tiles;
  const int tile = slot - group * tiles;
  const int split = group * 8 + (b & 7);
  if (split >= a.S) return;
  const int co0 = (tile % a.gco) * BMO;
  const int k_tile = tile / a.gco;
  const int k0 = k_tile * BNO;
  const long p_begin = (long)split * a.pix_per_split;
  const long p_end = min(a.M, p_begin + a.pix_per_split);
  const int HoWo = a.Ho * a.Wo;
  const bool has_pre = a.pre_scale != nullptr;
  const bool do_bias = a.slab_b != nullptr && k_tile == 0;
  if (has_pre) {
    for (int c = tid; c < a.Cin; c += NT) {
      sPre[c] = a.pre_scale[c];
      sPre[kMaxPreC + c] = a.pre_shift[c];
    }
    __syncthreads();
  }

  int tap = 0, c0 = 0, kh = 0, kw = 0;
  if (!GENERIC) {
    tap = k0 / a.Cin;
    c0 = k0 - tap * a.Cin;
    kh = tap / a.KW;
    kw = tap - kh * a.KW;
  }
  const int cvd = tid % CPR_D, rd0 = tid / CPR_D;
  const int cvx = tid % CPR_X, rx0 = tid / CPR_X;

  typedef typename Vec16<T>::type V;
  constexpr int DEL = (BP * BMO) / NT;  // generic dy elements per thread
  V dreg[GENERIC ? 1 : D_PASSES];
  float dg[GENERIC ? DEL : 1];
  V xreg[GENERIC ? 1 : X_PASSES];
  bool xval[GENERIC ? 1 : X_PASSES];
  float xg[GENERIC ? GEL : 1];

  auto load = [&](long p0) {
    if constexpr (!GENERIC) {
#pragma unroll
      for (int i = 0; i < D_PASSES; ++i) {
        long m = p0 + rd0 + i * RPP_D;
        int co = co0 + cvd * VEC;
        if (m < p_end && co < a.Cout)
          dreg[i] = load16(dy + m * a.Cout + co);
        else
          dreg[i] = V{};
      }
    } else {
#pragma unroll
      for (int j = 0; j < DEL; ++j) {
        int e = tid + j * NT;
        int r = e / BMO, c = e - (e / BMO) * BMO;
        long m = p0 + r;
        int co = co0 + c;
        dg[j] = (m < p_end && co < a.Cout) ? to_f(dy[m * a.Cout + co]) : 0.f;
      }
    }
    if constexpr (!GENERIC) {
#pragma unroll
      for (int i = 0; i < X_PASSES; ++i) {
        long m = p0 + rx0 + i * RPP_X;
        bool ok = false;
        if (m < p_end) {
          int n = (int)a.fd_howo.div((uint32_t)m);
          int rem = (int)(m - (long)n * HoWo);
          int ho = (int)a.fd_wo.div((uint32_t)rem), wo = rem - ho * a.Wo;
          int hi = ho * a.stride - a.pad + kh * a.dil, wi = wo * a.stride - a.pad + kw * a.dil;
          if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) {
            ok = true;
            xreg[i] = load16(x + (((long)n * a.H + hi) * a.W + wi) * a.Cin + c0 + cvx * VEC);
          }
        }
        if (!ok) xreg[i] = V{};
        xval[i] = ok;
      }
    } else {
#pragma unroll
      for (int j = 0; j < GEL; ++j) {
        int e = tid + j * NT;
        int r = e / BNO, kc = e - (e / BNO) * BNO;
        long m = p0 + r;
        int kidx = k0 + kc;
        float v = 0.f;
        if (m < p_end && kidx < a.K) {
          int tp = (int)a.fd_cin.div((uint32_t)kidx), ci = kidx - tp * a.Cin;
          int kh2 = (int)a.fd_kw.div((uint32_t)tp), kw2 = tp - kh2 * a.KW;
          int n = (int)a.fd_howo.div((uint32_t)m);
          int rem = (int)(m - (long)n * HoWo);
          int ho = (int)a.fd_wo.div((uint32_t)rem), wo = rem - ho * a.Wo;
          int hi = ho * a.stride - a.pad + kh2 * a.dil, wi = wo * a.stride - a.pad + kw2 * a.dil;
          if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) {
            v = to_f(x[(((long)n * a.H + hi) * a.W + wi) * a.Cin + ci]);
            if (has_pre) {
              v = v * sPre[ci] + sPre[kMaxPreC + ci];
              if (a.pre_relu) v = fmaxf(v, 0.f);
            }
          }
        }
        xg[j] = v;
      }
    }
  };
  auto store = [&]() {
    if constexpr (!GENERIC) {
#pragma unroll
      for (int i = 0; i < D_PASSES; ++i) store16(&Ds[(rd0 + i * RPP_D) * LDD + cvd * VEC], dreg[i]);
    } else {
#pragma unroll
      for (int j = 0; j < DEL; ++j) {
        int e = tid + j * NT;
        int r = e / BMO, c = e - (e / BMO) * BMO;
        Ds[r * LDD + c] = from_f<T>(dg[j]);
      }
    }
    if constexpr (!GENERIC) {
#pragma unroll
      for (int i = 0; i < X_PASSES; ++i) {
        T* dst = &Xs[(rx0 + i * RPP_X) * LDX + cvx * VEC];
        if (has_pre && xval[i]) {
          float f[VEC];
          unpack16<T>(xreg[i], f);
          const int cb = c0 + cvx * VEC;
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            float v = f[e] * sPre[cb + e] + sPre[kMaxPreC + cb + e];
            f[e] = a.pre_relu ? fmaxf(v, 0.f) : v;
          }
          store16(dst, pack16<T>(f));
        } else {
          store16(dst, xreg[i]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < GEL; ++j) {
        int e = tid + j * NT;
        int r = e / BNO, kc = e - (e / BNO) * BNO;
        Xs[r * LDX + kc] = from_f<T>(xg[j]);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;

  const int lr = lane & 15, lg = lane >> 4;
  if (p_begin < p_end) {
    load(p_begin);
    store();
    __syncthreads();
  }
  for (long p0 = p_begin; p0 < p_end; p0 += BP) {
    const bool more = p0 + BP < p_end;
    if (more) load(p0 + BP);
    if (do_bias && tid < BMO) {
#pragma unroll 4
      for (int p = 0; p < BP; ++p) bacc += to_f(Ds[p * LDD + tid]);
    }
    if constexpr (sizeof(T) == 4) {
      const float* Df = reinterpret_cast<const float*>(Ds);
      const float* Xf = reinterpret_cast<const float*>(Xs);
#pragma unroll
      for (int kk = 0; kk < BP / 4; ++kk) {
        float av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) av[i] = Df[(kk * 4 + lg) * LDD + wm * WTM + i * 16 + lr];
#pragma unroll
        for (int j = 0; j < FN; ++j) bv[j] = Xf[(kk * 4 + lg) * LDX + wn * WTN + j * 16 + lr];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // transposed LDS reads (ds_read_b64_tr_b16): lane (g = lane>>4, i = lane&15) receives
      // column i of 4 consecutive pixel rows. The contraction order is free as long as A and B
      // agree, so fragment element j of group g is pixel 4g+j (j<4) / 16+4g+(j-4) (j>=4): each
      // tr instruction then reads 8 CONSECUTIVE rows per 32-lane half, which the row padding maps
      // to 8 disjoint bank slots (conflict-free).
      const int q = lr >> 2, p4 = lr & 3;
      typedef short s16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int kk = 0; kk < BP / 32; ++kk) {
        bf16x8 av[FM], bv[FN];
        const int prow = kk * 32 + 4 * lg + q;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const T* base = &Ds[prow * LDD + wm * WTM + i * 16 + 4 * p4];
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + 16 * LDD));
          s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          av[i] = __builtin_bit_cast(bf16x8, c);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const T* base = &Xs[prow * LDX + wn * WTN + j * 16 + 4 * p4];
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + 16 * LDX));
          s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bv[j] = __builtin_bit_cast(bf16x8, c);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }

  // partial slab [split][Cout][K]
  slab_rmw<FM, FN>(a.slab + (long)split * a.Cout * a.K, a.K, a.Cout, split < a.s_init,
                   co0 + wm * WTM + lg * 4, k0 + wn * WTN + lr, acc);
  if (do_bias && tid < BMO && co0 + tid < a.Cout) {
    float* d = &a.slab_b[(long)split * a.Cout + co0 + tid];
    *d = split < a.s_init ? *d + bacc : bacc;
  }
}

// --------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 weight gradient, bf16, Cin % 64 == 0, Cout % 64 == 0: spatial halo
// tiling. A workgroup owns (64 output channels) x (64 input channels) x (all 9 taps) for a run of
// TH x 16-pixel spatial tiles (its split); NINE waves, wave t accumulates tap t's 64 x 64 block.
// Per tile the dy rows [128 px][64 co] and the BN(+ReLU)-transformed, zero-padded input halo
// [(TH+2) x 18][64 ci] are staged ONCE and every tap reads its B fragments from the halo at a
// shifted position — the per-tap implicit GEMM re-loads and re-transforms the input 9x and dy
// once per k-tile. Both operands are read as transposed fragments (ds_read_b64_tr_b16) from
// 160-B-pitch rows (conflict-free for any row offset). Three LDS stages, one barrier per tile:
// while tile st is multiplied, tile st + 1 is already staged and the loads of tile st + 2 fly
// in registers — a tile's loads get a whole tile of MFMAs to land (with two stages the staging
// of tile st + 1 waited on loads issued just before the MFMAs: latency-bound, MFMA busy 0.18).
// --------------------------------------------------------------------------------------------
#ifdef HGK_WG_TRACE  // timing build (scripts/wgrad_trace.py): stamps of workgroups 0-255
// [wg][64]: 0 entry, 1 prologue done, per tile st < 15: 2+4st staged, 3+4st loads issued,
// 4+4st MFMAs issued, 5+4st barrier passed; 62 slab stores issued, 63 exit
__device__ unsigned long long g_wgtrace[256 * 64];
#define WG_STAMP(k)                                                                  \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 256 && (k) < 64)                            \
      g_wgtrace[blockIdx.x * 64 + (k)] = wall_clock64();                             \
  } while (0)
#else
#define WG_STAMP(k)
#endif

#ifndef HGK_WG_PRIO
#define HGK_WG_PRIO 0
#endif
// One use of the weight in a multi-use halo launch (route HGK_ROUTE_WG_HALO_MULTI): the uses'
// spatial tiles are concatenated (use i owns global tiles [t0, t0 + N (H/TH) (W/16))) and the
// splits run over the concatenation, so a split may cross from one use into the next — every
// slab element is read-modified-written ONCE per launch instead of once per use.
struct HaloSrc {
  const void* x;
  const void* dy;
  const float* pre_scale;
  const float* pre_shift;
  int pre_relu, N, H, W;
  int t0;
};
static constexpr int kMaxHaloSrc = 40;
struct HaloMultiArgs {
  ConvWgradArgs a;  // shared channels, slabs, split plan; x / dy / N / H / W unused
  int nsrc, t_total;
  HaloSrc src[kMaxHaloSrc];
};
static_assert(sizeof(HaloMultiArgs) <= 4096, "kernel argument segment");

template <int TH, bool MULTI>
__device__ __forceinline__ void wgrad_halo_body(const ConvWgradArgs& a, const HaloSrc* srcs,
                                                int nsrc, int t_total_multi) {
  typedef bf16_t T;
  WG_STAMP(0);
  constexpr int NT = 512, TW = 16, BP = TH * TW, HW = TW + 2, HPOS = (TH + 2) * HW;
  constexpr int LD = 80;  // elements per staged row (160 B)
  constexpr int DBUF = BP * LD, XBUF = HPOS * LD;
  constexpr int DCH = BP * 8, XCH = HPOS * 8;
  constexpr int DLD = (DCH + NT - 1) / NT, XLD = (XCH + NT - 1) / NT;
  static_assert(BP == 128, "4 x 32-pixel MFMA k-steps per tile");
  constexpr int NSTG = 3;
  __shared__ __attribute__((aligned(16))) T smem[NSTG * (DBUF + XBUF)];
  T* const Ds = smem;                 // [NSTG][BP][LD]
  T* const Xs = smem + NSTG * DBUF;   // [NSTG][HPOS][LD]

  const int b = blockIdx.x;
  const int tiles = a.gco * a.gk;  // (co-tile, ci-chunk) pairs
  const int slot = b >> 3;
  const int group = slot / tiles;
  const int tile = slot - group * tiles;
  const int split = group * 8 + (b & 7);  // a split's workgroups share an XCD (and its L2)
  if (split >= a.S) return;
  const int co0 = (tile % a.gco) * 64;
  const int ci0 = (tile / a.gco) * 64;
  const int t_total = MULTI ? t_total_multi : a.N * ((a.H / TH) * (a.W / TW));
  const int t_begin = split * (int)a.pix_per_split;
  const int t_end = min(t_total, t_begin + (int)a.pix_per_split);
  const int nstage = max(0, t_end - t_begin);

  // the source being loaded (MULTI: the use owning the next tile to load; its geometry is
  // wave-uniform and switched in load() when its tiles run out)
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.dy);
  int cH = a.H, cW = a.W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;  // wave w: tap w + 1/8 of tap 8
  const int c8 = tid & 7;  // this thread's 8-channel chunk in every staged row (512 % 8 == 0)
  // the BN(+ReLU) of the source being STAGED (MULTI: s_src, which lags the load cursor)
  bool has_pre = a.pre_scale != nullptr;
  bool relu = a.pre_relu != 0;
  const bool do_bias = a.slab_b != nullptr && ci0 == 0;
  float ps[8], pb[8], bsum[8];
  auto pre_load = [&](const float* sc, const float* sh) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ps[e] = sc ? sc[ci0 + c8 * 8 + e] : 1.f;
      pb[e] = sc ? sh[ci0 + c8 * 8 + e] : 0.f;
    }
  };
  int l_src = 0, l_left = 0, s_src = 0;
  int l_img, l_h0, l_w0;  // the next tile to load
  if (MULTI) {
    int s = 0;
    while (s + 1 < nsrc && srcs[s + 1].t0 <= t_begin) ++s;
    const HaloSrc& u = srcs[s];
    x = reinterpret_cast<const T*>(u.x);
    dy = reinterpret_cast<const T*>(u.dy);
    cH = u.H;
    cW = u.W;
    const int tiles_img = (cH / TH) * (cW / TW);
    l_src = s_src = s;
    l_left = u.N * tiles_img - (t_begin - u.t0);
    has_pre = u.pre_scale != nullptr;
    relu = u.pre_relu != 0;
    pre_load(u.pre_scale, u.pre_shift);
  } else {
    pre_load(a.pre_scale, a.pre_shift);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) bsum[e] = 0.f;
  {
    const int tiles_w = cW / TW, tiles_img = (cH / TH) * tiles_w;
    const int tb = MULTI ? t_begin - srcs[l_src].t0 : t_begin;
    const int img = tb / tiles_img, trem = tb - img * tiles_img;
    l_img = img;
    l_h0 = (trem / tiles_w) * TH;
    l_w0 = (trem % tiles_w) * TW;
  }
  uint4 rd[DLD], rx[XLD];
  bool xok[XLD];

  // per-thread element offsets of its chunks relative to the tile's first pixel (32-bit: the
  // host checks M * max(Cin, Cout) < 2^31) and the halo chunks' (row, column) in the halo; per
  // tile only the tile's base pixel moves (kept in scalars, stepped tile by tile: no divisions)
  int doff[DLD], xoff[XLD], xhr[XLD], xhc[XLD];
  auto offsets = [&](int W) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < DLD; ++j) {
      const int px = min(tid + j * NT, DCH - 1) >> 3;
      doff[j] = ((px >> 4) * W + (px & 15)) * a.Cout + co0 + c8 * 8;
    }
#pragma unroll
    for (int j = 0; j < XLD; ++j) {
      const int pos = min(tid + j * NT, XCH - 1) >> 3;
      const int hr = pos / HW, hc = pos - hr * HW;
      xoff[j] = ((hr - 1) * W + (hc - 1)) * a.Cin + ci0 + c8 * 8;
    }
  };
  offsets(cW);
#pragma unroll
  for (int j = 0; j < XLD; ++j) {
    const int q = tid + j * NT;
    const int pos = min(q, XCH - 1) >> 3;
    const int hr = pos / HW, hc = pos - hr * HW;
    // q >= XCH (a thread without this chunk) never passes the bounds test below
    xhr[j] = q < XCH ? hr - 1 : -(1 << 20);
    xhc[j] = hc - 1;
  }

  // loads tile st (tiles are loaded in order: l_* is its position) and returns its source
  auto load = [&](int st, uint4* rd, uint4* rx, bool* xok) __attribute__((always_inline)) {
    (void)st;
    if (MULTI) {
      if (l_left == 0) {  // the current use is exhausted: the next one starts at its tile 0
        const HaloSrc& u = srcs[++l_src];
        x = reinterpret_cast<const T*>(u.x);
        dy = reinterpret_cast<const T*>(u.dy);
        cH = u.H;
        cW = u.W;
        l_left = u.N * ((cH / TH) * (cW / TW));
        l_img = l_h0 = l_w0 = 0;
        offsets(cW);
      }
      --l_left;
    }
    const int img = l_img, h0 = l_h0, w0 = l_w0;
    l_w0 += TW;
    if (l_w0 == cW) {
      l_w0 = 0;
      l_h0 += TH;
      if (l_h0 == cH) { l_h0 = 0; ++l_img; }
    }
    const long tpix = ((long)img * cH + h0) * cW + w0;
    const T* dyt = dy + tpix * a.Cout;
    const T* xt = x + tpix * a.Cin;
#pragma unroll
    for (int j = 0; j < DLD; ++j) rd[j] = *reinterpret_cast<const uint4*>(dyt + doff[j]);
#pragma unroll
    for (int j = 0; j < XLD; ++j) {
      const bool ok = (unsigned)(h0 + xhr[j]) < (unsigned)cH && (unsigned)(w0 + xhc[j]) < (unsigned)cW;
      rx[j] = *reinterpret_cast<const uint4*>(ok ? xt + xoff[j] : x + ci0 + c8 * 8);
      xok[j] = ok;
    }
    return l_src;
  };
  auto store = [&](int buf, const uint4* rd, const uint4* rx, const bool* xok, int src) __attribute__((always_inline)) {
    if (MULTI && src != s_src) {  // the staged tile belongs to the next use: its BN
      s_src = src;
      const HaloSrc& u = srcs[src];
      has_pre = u.pre_scale != nullptr;
      relu = u.pre_relu != 0;
      pre_load(u.pre_scale, u.pre_shift);
    }
    T* D = Ds + buf * DBUF;
    T* X = Xs + buf * XBUF;
#pragma unroll
    for (int j = 0; j < DLD; ++j) {
      const int q = tid + j * NT;
      if (q < DCH) {
        *reinterpret_cast<uint4*>(D + (q >> 3) * LD + c8 * 8) = rd[j];
        if (do_bias) {
          float f[8];
          unpack16<T>(rd[j], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) bsum[e] += f[e];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < XLD; ++j) {
      const int q = tid + j * NT;
      if (q < XCH) {
        uint4 v = rx[j];
        if (has_pre) v = bn_relu_chunk<bf16_t>(v, ps, pb, relu);
        const uint32_t keep = xok[j] ? 0xffffffffu : 0u;  // zero padding AFTER the transform
        v.x &= keep; v.y &= keep; v.z &= keep; v.w &= keep;
        *reinterpret_cast<uint4*>(X + (q >> 3) * LD + c8 * 8) = v;
      }
    }
  };

  // wave w owns tap w's 4x4 fragment tiles plus tiles (w/2, 2(w%2)..+1) of tap 8: 18 tiles per
  // wave, two waves per SIMD, every SIMD equally loaded (9 waves would leave one SIMD with 3)
  f32x4 acc[4][4], acc8[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc8[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc8[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, lg = lane >> 4, q4 = lr >> 2, p4 = lr & 3;
  const int kh = wave / 3, kw = wave - kh * 3;
  const int i8 = wave >> 1, j8 = (wave & 1) * 2;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
#ifndef HGK_ABL_WG_NOPIPE
  // software-pipelined: the fragments of k-step kk + 1 are read from LDS before the MFMAs of
  // k-step kk issue (two fragment sets in registers), so LDS latency hides behind the matrix work
  struct WgFrag { bf16x8 av[4], bv[4], a8, b8[2]; };
  auto rd_tr = [&](const T* base, int stride) __attribute__((always_inline)) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + stride));
    const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, c);
  };
  auto frag_load = [&](const T* D, const T* X, int kk, WgFrag& f) __attribute__((always_inline)) {
    const int prow = kk * 32 + 4 * lg + q4;
    const int pos = (2 * kk + kh) * HW + 4 * lg + q4 + kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) f.av[i] = rd_tr(D + prow * LD + i * 16 + 4 * p4, 16 * LD);
#pragma unroll
    for (int j = 0; j < 4; ++j) f.bv[j] = rd_tr(X + pos * LD + j * 16 + 4 * p4, HW * LD);
    f.a8 = rd_tr(D + prow * LD + i8 * 16 + 4 * p4, 16 * LD);
    const int pos8 = (2 * kk + 2) * HW + 4 * lg + q4 + 2;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) f.b8[jj] = rd_tr(X + pos8 * LD + (j8 + jj) * 16 + 4 * p4, HW * LD);
  };
  auto frag_mma = [&](const WgFrag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.av[i], f.bv[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
      acc8[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a8, f.b8[jj], acc8[jj], 0, 0, 0);
  };
  auto compute = [&](int buf) {
    const T* D = Ds + buf * DBUF;
    const T* X = Xs + buf * XBUF;
    WgFrag f[2];
    frag_load(D, X, 0, f[0]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk + 1 < 4) frag_load(D, X, kk + 1, f[(kk + 1) & 1]);
      frag_mma(f[kk & 1]);
    }
  };
#else
  auto compute = [&](int buf) {
    const T* D = Ds + buf * DBUF;
    const T* X = Xs + buf * XBUF;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      // contraction order: fragment element e of lane group g <-> tile pixel kk*32 + 4g + e
      // (e < 4, tile row 2kk) / kk*32 + 16 + 4g + e - 4 (tile row 2kk+1), for A and B alike
      const int prow = kk * 32 + 4 * lg + q4;
      const int pos = (2 * kk + kh) * HW + 4 * lg + q4 + kw;
      bf16x8 av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const T* base = D + prow * LD + i * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 16 * LD));
        const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        av[i] = __builtin_bit_cast(bf16x8, c);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const T* base = X + pos * LD + j * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + HW * LD));
        const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bv[j] = __builtin_bit_cast(bf16x8, c);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      // this wave's share of tap 8 (kh = kw = 2)
      {
        const T* base = D + prow * LD + i8 * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 16 * LD));
        const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 a8 = __builtin_bit_cast(bf16x8, c);
        const int pos8 = (2 * kk + 2) * HW + 4 * lg + q4 + 2;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const T* xb = X + pos8 * LD + (j8 + jj) * 16 + 4 * p4;
          const s16x4 l8 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb));
          const s16x4 h8 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb + HW * LD));
          const s16x8 c8v = {l8[0], l8[1], l8[2], l8[3], h8[0], h8[1], h8[2], h8[3]};
          acc8[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, __builtin_bit_cast(bf16x8, c8v),
                                                             acc8[jj], 0, 0, 0);
        }
      }
    }
  };
#endif

  // iteration st: stage tile st + 1 (its loads were issued one iteration ago) into stage
  // (st + 1) % 3 — last read by compute(st - 2), before the previous barrier — then issue tile
  // st + 2's loads into the freed registers and multiply tile st
  int r_src = 0;  // the source of the tile held in rd / rx
  if (nstage > 0) {
    // both prologue tiles' loads in flight together (a second register set for tile 1)
    uint4 rd1[DLD], rx1[XLD];
    bool xok1[XLD];
    const int s0 = load(0, rd, rx, xok);
    if (nstage > 1) r_src = load(1, rd1, rx1, xok1);
    store(0, rd, rx, xok, s0);
#pragma unroll
    for (int j = 0; j < DLD; ++j) rd[j] = rd1[j];
#pragma unroll
    for (int j = 0; j < XLD; ++j) { rx[j] = rx1[j]; xok[j] = xok1[j]; }
  }
  __syncthreads();
  WG_STAMP(1);
  // The two waves of a SIMD (w and w + 4) take the tile's phases in opposite order: waves 0-3
  // stage tile st + 1 and issue tile st + 2's loads, then multiply tile st; waves 4-7 multiply
  // first. Staging writes stage (st + 1) % 3, the MFMAs read stage st % 3, so the orders are
  // interchangeable inside the iteration — and each SIMD's MFMA pipe now runs one wave's matrix
  // work while its partner stages (in lock step, every SIMD idled through staging + load issue,
  // ~1 us of the 2.6 us per tile: scripts/wgrad_trace.py, profiles/r04_wgrad_trace.txt).
#ifdef HGK_ABL_WG_LOCKSTEP
  const bool mfma_first = false;
#else
  const bool mfma_first = wave >= 4;
#endif
#if HGK_WG_PRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half loses arbitration
#endif
  for (int st = 0, cur = 0; st < nstage; ++st) {
    const int nxt = cur == NSTG - 1 ? 0 : cur + 1;
    if (mfma_first) compute(cur);
    if (st + 1 < nstage) store(nxt, rd, rx, xok, r_src);
    WG_STAMP(2 + 4 * st);
#ifndef HGK_ABL_WG_NOLOAD
    if (st + 2 < nstage) r_src = load(st + 2, rd, rx, xok);
#endif
    WG_STAMP(3 + 4 * st);
    if (!mfma_first) compute(cur);
    WG_STAMP(4 + 4 * st);
    __syncthreads();
    WG_STAMP(5 + 4 * st);
    cur = nxt;
  }
#ifdef HGK_ABL_WG_NOSLAB
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
  asm volatile("" ::"v"(acc8[0]), "v"(acc8[1]));
  return;
#endif

  // partial slab [split][Cout][K], k = tap * Cin + ci
  float* slab = a.slab + (long)split * a.Cout * a.K;
  const bool accum = split < a.s_init;
  // all of a row-group's slab loads are issued before its stores (see slab_rmw)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* base = slab + (long)(co0 + i * 16 + lg * 4) * a.K + wave * a.Cin + ci0 + lr;
    float old[4][4];
    if (accum) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[j][r] = base[(long)r * a.K + j * 16];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        base[(long)r * a.K + j * 16] = accum ? old[j][r] + acc[i][j][r] : acc[i][j][r];
  }
  {
    float* base = slab + (long)(co0 + i8 * 16 + lg * 4) * a.K + 8 * a.Cin + ci0 + j8 * 16 + lr;
    float old[2][4];
    if (accum) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[jj][r] = base[(long)r * a.K + jj * 16];
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        base[(long)r * a.K + jj * 16] = accum ? old[jj][r] + acc8[jj][r] : acc8[jj][r];
  }
  WG_STAMP(62);
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);  // [NT/8][64]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(tid >> 3) * 64 + c8 * 8 + e] = bsum[e];
    __syncthreads();
    if (tid < 64) {
      float sb = 0.f;
      for (int r = 0; r < NT / 8; ++r) sb += red[r * 64 + tid];
      float* d = &a.slab_b[(long)split * a.Cout + co0 + tid];
      *d = split < a.s_init ? *d + sb : sb;
    }
  }
  WG_STAMP(63);
}

template <int TH>
__global__ __launch_bounds__(512) void conv3x3_wgrad_halo_kernel(ConvWgradArgs a) {
  wgrad_halo_body<TH, false>(a, nullptr, 0, 0);
}

template <int TH>
__global__ __launch_bounds__(512) void conv3x3_wgrad_halo_multi_kernel(HaloMultiArgs m) {
  wgrad_halo_body<TH, true>(m.a, m.src, m.nsrc, m.t_total);
}

// --------------------------------------------------------------------------------------------
// The halo weight gradient with LDS-DMA staging (route HGK_ROUTE_WG_DMA): the same workgroup
// tiles, splits, tap-per-wave MFMA schedule, summation order and slab epilogue as
// conv3x3_wgrad_halo_kernel (bitwise equal results), but the dy tile and the raw input halo go
// global -> LDS by global_load_lds_dwordx4 (no register round trip, no ds_write), and the BN+ReLU
// transform of the input runs in place on the chunks each lane itself DMA'd (its own counted
// vmcnt orders them: no extra barrier). Staged rows are 128 B with 16-B chunk c of row r in slot
// c ^ (r & 7): a 1-KB DMA block is 8 whole rows and lane L always carries channel chunk
// (L & 7) ^ (L >> 3) — its BN scale / shift stay in registers — and the transposed fragment
// reads stay conflict-free (8 consecutive rows per 32-lane half hit 8 distinct slots x 2 bank
// halves). Out-of-image halo positions DMA a zero page and skip the transform (zero AFTER BN).
// --------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) uint4 g_wgdma_zero[4];

template <int TH, bool PRE>
__global__ __launch_bounds__(512) void conv3x3_wgrad_dma_kernel(ConvWgradArgs a) {
  typedef bf16_t T;
  constexpr int NT = 512, NW = 8, TW = 16, BP = TH * TW, HW = TW + 2, HPOS = (TH + 2) * HW;
  static_assert(BP == 128, "4 x 32-pixel MFMA k-steps per tile");
  constexpr int RB = 128;                          // bytes per staged row (64 channels)
  constexpr int DBLK = BP / 8;                     // 1-KB DMA blocks of the dy tile (8 rows each)
  constexpr int XBLK = (HPOS + 7) / 8;             // ... of the input halo (last one partly dummy)
  constexpr int NBLK = DBLK + XBLK;
  constexpr int DBYTES = DBLK * 1024, XBYTES = XBLK * 1024, STG = DBYTES + XBYTES;
  constexpr int NSTG = 3;
  constexpr int MAXB = (NBLK + NW - 1) / NW;       // DMA blocks per wave per tile (<=)
  static_assert(NSTG * STG <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NSTG * STG];

  const int b = blockIdx.x;
  const int tiles = a.gco * a.gk;
  const int slot = b >> 3;
  const int group = slot / tiles;
  const int tile = slot - group * tiles;
  const int split = group * 8 + (b & 7);
  if (split >= a.S) return;
  const int co0 = (tile % a.gco) * 64;
  const int ci0 = (tile / a.gco) * 64;
  const int tiles_w = a.W / TW, tiles_img = (a.H / TH) * tiles_w;
  const int t_total = a.N * tiles_img;
  const int t_begin = split * (int)a.pix_per_split;
  const int t_end = min(t_total, t_begin + (int)a.pix_per_split);
  const int nstage = max(0, t_end - t_begin);

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.dy);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c8 = tid & 7;  // the bias partial's channel chunk (as conv3x3_wgrad_halo_kernel)
  const bool relu = a.pre_relu != 0;
  const bool do_bias = a.slab_b != nullptr && ci0 == 0;
  // this lane's DMA channel chunk, the same in every block
  const int cl = (lane & 7) ^ ((lane >> 3) & 7);
  float ps[8], pb[8], bsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ps[e] = PRE ? a.pre_scale[ci0 + cl * 8 + e] : 1.f;
    pb[e] = PRE ? a.pre_shift[ci0 + cl * 8 + e] : 0.f;
    bsum[e] = 0.f;
  }
  const int nb = (NBLK - wave + NW - 1) / NW;  // this wave's blocks: wave, wave + 8, ...
  const char* const zero = reinterpret_cast<const char*>(g_wgdma_zero);

  // issue this wave's DMA blocks of tile st into stage buf
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    const int t = t_begin + st;
    const int img = t / tiles_img, trem = t - img * tiles_img;
    const int h0 = (trem / tiles_w) * TH, w0 = (trem % tiles_w) * TW;
    char* const sb = smem + buf * STG;
#pragma unroll
    for (int i = 0; i < MAXB; ++i) {
      const int blk = wave + i * NW;
      if (blk < NBLK) {
        const int row = (blk < DBLK ? blk : blk - DBLK) * 8 + (lane >> 3);
        const void* src;
        if (blk < DBLK) {
          const long pix = ((long)img * a.H + h0 + (row >> 4)) * a.W + w0 + (row & 15);
          src = dy + pix * a.Cout + co0 + cl * 8;
        } else {
          const int hr = row / HW, hc = row - hr * HW;
          const int hi = h0 - 1 + hr, wi = w0 - 1 + hc;
          const bool ok = row < HPOS && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
          src = ok ? (const void*)(x + (((long)img * a.H + hi) * a.W + wi) * a.Cin + ci0 + cl * 8)
                   : (const void*)zero;
        }
        dma16(src, sb + (blk < DBLK ? blk * 1024 : DBYTES + (blk - DBLK) * 1024));
      }
    }
  };
  // BN+ReLU of the input chunks this lane DMA'd for tile st (in stage buf), in place
  auto transform = [&](int st, int buf) __attribute__((always_inline)) {
    if constexpr (PRE) {
      const int t = t_begin + st;
      const int img = t / tiles_img, trem = t - img * tiles_img;
      const int h0 = (trem / tiles_w) * TH, w0 = (trem % tiles_w) * TW;
      char* const xb = smem + buf * STG + DBYTES;
      (void)img;
#pragma unroll
      for (int i = 0; i < MAXB; ++i) {
        const int blk = wave + i * NW;
        if (blk >= DBLK && blk < NBLK) {
          const int row = (blk - DBLK) * 8 + (lane >> 3);
          const int hr = row / HW, hc = row - hr * HW;
          const int hi = h0 - 1 + hr, wi = w0 - 1 + hc;
          const bool ok = row < HPOS && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
          uint4* cp = reinterpret_cast<uint4*>(xb + (blk - DBLK) * 1024 + lane * 16);
          if (ok) *cp = bn_relu_chunk<bf16_t>(*cp, ps, pb, relu);
        }
      }
    }
  };
  // wait until this wave's DMAs of the tile before the last `younger` blocks have landed
  auto wait_older = [&](bool younger) __attribute__((always_inline)) {
    if (!younger) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (nb == MAXB) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXB - 1) : "memory");
    }
  };
  static_assert(NBLK % NW != 0 && NBLK > NW * (MAXB - 1), "two per-wave block counts");

  f32x4 acc[4][4], acc8[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc8[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc8[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, lg = lane >> 4, q4 = lr >> 2, p4 = lr & 3;
  const int kh = wave / 3, kw = wave - kh * 3;
  const int i8 = wave >> 1, j8 = (wave & 1) * 2;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  // row R, channels 16 * f + 4 * p4 .. + 3 (8 B inside 16-B chunk 2 f + (p4 >> 1))
  auto at = [&](const char* base, int R, int f) __attribute__((always_inline)) {
    return base + R * RB + ((((2 * f + (p4 >> 1)) ^ (R & 7))) << 4) + ((p4 & 1) << 3);
  };
  auto rd_tr = [&](const char* lo, const char* hi) __attribute__((always_inline)) {
    const s16x4 l = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lo));
    const s16x4 h = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(hi));
    const s16x8 c = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
    return __builtin_bit_cast(bf16x8, c);
  };
  struct WgFrag { bf16x8 av[4], bv[4], a8, b8[2]; };
  auto frag_load = [&](const char* D, const char* X, int kk, WgFrag& f) __attribute__((always_inline)) {
    const int prow = kk * 32 + 4 * lg + q4;
    const int pos = (2 * kk + kh) * HW + 4 * lg + q4 + kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) f.av[i] = rd_tr(at(D, prow, i), at(D, prow + 16, i));
#pragma unroll
    for (int j = 0; j < 4; ++j) f.bv[j] = rd_tr(at(X, pos, j), at(X, pos + HW, j));
    f.a8 = rd_tr(at(D, prow, i8), at(D, prow + 16, i8));
    const int pos8 = (2 * kk + 2) * HW + 4 * lg + q4 + 2;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) f.b8[jj] = rd_tr(at(X, pos8, j8 + jj), at(X, pos8 + HW, j8 + jj));
  };
  auto frag_mma = [&](const WgFrag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.av[i], f.bv[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
      acc8[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a8, f.b8[jj], acc8[jj], 0, 0, 0);
  };
  auto compute = [&](int buf) {
    const char* D = smem + buf * STG;
    const char* X = D + DBYTES;
    if (do_bias) {
      // conv3x3_wgrad_halo_kernel's per-thread bias order: rows tid >> 3, + 64; chunk c8
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = (tid >> 3) + 64 * j;
        float f[8];
        unpack16<T>(*reinterpret_cast<const uint4*>(D + r * RB + ((c8 ^ (r & 7)) << 4)), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[e] += f[e];
      }
    }
    WgFrag f[2];
    frag_load(D, X, 0, f[0]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk + 1 < 4) frag_load(D, X, kk + 1, f[(kk + 1) & 1]);
      frag_mma(f[kk & 1]);
    }
  };

  // prologue: tiles 0 and 1 in flight, tile 0 landed and transformed
  if (nstage > 0) {
    issue(0, 0);
    if (nstage > 1) issue(1, 1);
    wait_older(nstage > 1);
    transform(0, 0);
  }
  __syncthreads();
  // iteration st: issue tile st + 2 into the stage compute(st - 1) released before the last
  // barrier; multiply tile st; tile st + 1 (issued one iteration ago) lands and is transformed.
  // Waves 4-7 multiply first, 0-3 transform first (the SIMD's two waves in opposite phases).
  const bool mfma_first = wave >= 4;
  for (int st = 0, cur = 0; st < nstage; ++st) {
    const int nxt = cur == NSTG - 1 ? 0 : cur + 1;
    const int nxt2 = nxt == NSTG - 1 ? 0 : nxt + 1;
    if (st + 2 < nstage) issue(st + 2, nxt2);
    if (mfma_first) compute(cur);
    if (st + 1 < nstage) {
      wait_older(st + 2 < nstage);
      transform(st + 1, nxt);
    }
    if (!mfma_first) compute(cur);
    __syncthreads();
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // partial slab [split][Cout][K], k = tap * Cin + ci (conv3x3_wgrad_halo_kernel's epilogue)
  float* slab = a.slab + (long)split * a.Cout * a.K;
  const bool accum = split < a.s_init;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* base = slab + (long)(co0 + i * 16 + lg * 4) * a.K + wave * a.Cin + ci0 + lr;
    float old[4][4];
    if (accum) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[j][r] = base[(long)r * a.K + j * 16];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        base[(long)r * a.K + j * 16] = accum ? old[j][r] + acc[i][j][r] : acc[i][j][r];
  }
  {
    float* base = slab + (long)(co0 + i8 * 16 + lg * 4) * a.K + 8 * a.Cin + ci0 + j8 * 16 + lr;
    float old[2][4];
    if (accum) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[jj][r] = base[(long)r * a.K + jj * 16];
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        base[(long)r * a.K + jj * 16] = accum ? old[jj][r] + acc8[jj][r] : acc8[jj][r];
  }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);  // [NT/8][64]
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(tid >> 3) * 64 + c8 * 8 + e] = bsum[e];
    __syncthreads();
    if (tid < 64) {
      float sb = 0.f;
      for (int r = 0; r < NT / 8; ++r) sb += red[r * 64 + tid];
      float* d = &a.slab_b[(long)split * a.Cout + co0 + tid];
      *d = split < a.s_init ? *d + sb : sb;
    }
  }
}

// One source of weight-grad pixels: an (input, output-grad) tensor pair of one use of a weight.
// m_begin = first pixel of the source in the launch's concatenated pixel space.
struct WgradSrc {
  const void* x;
  const void* dy;
  const float* pre_scale;
  const float* pre_shift;
  long m_begin;
  int M, H, W, Ho, Wo, pre_relu;
  FastDiv fd_howo, fd_wo;
};
// sources per launch: 40 covers every shared weight of the models in one launch (the small
// levels' blocks are used 32 times per step: 24 took two under-filled launches each)
static constexpr int kMaxWgradSrc = 40;
// hgk_conv_wgrad_accum_multi: several uses of ONE weight (same Cin / Cout / filter) in one launch
struct ConvWgradMultiArgs {
  ConvWgradArgs a;  // shared geometry, slabs, split plan; a.M = total pixels of all sources
  int nsrc;
  WgradSrc src[kMaxWgradSrc];
};
static_assert(sizeof(ConvWgradMultiArgs) <= 4096, "kernel argument segment");

// Weight-grad main body for channel counts that vectorise (Cin % BNO == 0, Cout % VEC == 0).
// One workgroup = one (co-tile, k-tile) of one pixel split (XCD-grouped, see below). Per stage of
// BP output pixels: dy rows [BP][BMO] and the tap-shifted, BN+ReLU-transformed input rows
// [BP][BNO] are loaded branch-free (clamped addresses + select), kept in registers while the
// previous stage is multiplied (double-buffered LDS, ONE barrier per stage), then read back as
// transposed MFMA fragments. The bias grad (column sums of dy) is accumulated from the dy
// registers of k-tile 0 workgroups. A split's pixel range may span several sources (the multi-use
// launch): the staged loop runs once per source it intersects, into the same accumulators.
// SMALLC: Cin == one 16-byte chunk (channel-padded network input): a k-tile spans BNO/VEC taps
// and each thread's x chunk is one whole pixel of its own tap.
template <typename T, int BMO, int BNO, int WM, int WN, bool SMALLC>
__device__ __forceinline__ void wgrad_fast_body(const ConvWgradArgs& a, const WgradSrc* srcs,
                                                int nsrc, int b) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BP = 64;
  constexpr int PADW = sizeof(T) == 2 ? 16 : 4;
  constexpr int LDD = BMO + PADW, LDX = BNO + PADW;
  constexpr int VEC = Vec16<T>::N;
  constexpr int CPR_D = BMO / VEC, RPP_D = NT / CPR_D, D_PASSES = BP / RPP_D;
  constexpr int CPR_X = BNO / VEC, RPP_X = NT / CPR_X, X_PASSES = BP / RPP_X;
  constexpr int WTM = BMO / WM, WTN = BNO / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert(D_PASSES >= 1 && X_PASSES >= 1 && NT % CPR_D == 0 && NT % CPR_X == 0, "tile");
  constexpr int DBUF = BP * LDD, XBUF = BP * LDX;

  __shared__ __attribute__((aligned(16))) T Ds[2 * DBUF];
  __shared__ __attribute__((aligned(16))) T Xs[2 * XBUF];
  float* sBias = reinterpret_cast<float*>(Ds);  // [RPP_D][BMO], reused after the last stage
  static_assert(RPP_D * BMO * 4 <= 2 * DBUF * (int)sizeof(T), "bias scratch");

  const int tiles = a.gco * a.gk;
  const int slot = b >> 3;
  const int group = slot / tiles;
  const int tile = slot - group * tiles;
  const int split = group * 8 + (b & 7);
  if (split >= a.S) return;
  const int co0 = (tile % a.gco) * BMO;
  const int k_tile = tile / a.gco;
  const int k0 = k_tile * BNO;
  const long P0 = (long)split * a.pix_per_split;
  const long P1 = min(a.M, P0 + a.pix_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const bool do_bias = a.slab_b != nullptr && k_tile == 0;
  const int cvd = tid % CPR_D, rd0 = tid / CPR_D;
  const int cvx = tid % CPR_X, rx0 = tid / CPR_X;
  // tap of this thread's x chunk: the workgroup's (one tap per k-tile), or for SMALLC its own
  const int tap = SMALLC ? k0 / VEC + cvx : (int)a.fd_cin.div((uint32_t)k0);
  const int c0 = SMALLC ? 0 : k0 - tap * a.Cin;
  const int xc = SMALLC ? 0 : c0 + cvx * VEC;  // first channel of this thread's x chunk
  const bool tap_ok = !SMALLC || tap < a.KH * a.KW;
  const int kh = (int)a.fd_kw.div((uint32_t)tap), kw = tap - kh * a.KW;
  const int dh = kh * a.dil - a.pad, dw = kw * a.dil - a.pad;
  const bool d_chunk_ok = co0 + cvd * VEC < a.Cout;  // last co-tile may be partial

  typedef typename Vec16<T>::type V;
  struct Regs {
    V d[D_PASSES], x[X_PASSES];
    bool ok[X_PASSES];
  };
  Regs R0;  // register stage: next stage's loads fly while the current stage is multiplied
  float bsum[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) bsum[e] = 0.f;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, lg = lane >> 4;

  for (int si = 0; si < nsrc; ++si) {
    const WgradSrc& sr = srcs[si];
    const long lo = max(P0, sr.m_begin), hi_ = min(P1, sr.m_begin + (long)sr.M);
    if (lo >= hi_) continue;  // workgroup-uniform
    const long p_begin = lo - sr.m_begin, p_end = hi_ - sr.m_begin;
    const int nstage = (int)((p_end - p_begin + BP - 1) / BP);
    const T* __restrict__ x = reinterpret_cast<const T*>(sr.x);
    const T* __restrict__ dy = reinterpret_cast<const T*>(sr.dy);
    const int HoWo = sr.Ho * sr.Wo;
    const bool has_pre = sr.pre_scale != nullptr;
    const bool pre_relu = sr.pre_relu != 0;
    // this thread's input channels are fixed for the whole source: BN constants in registers
    float pre_s[VEC], pre_b[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      pre_s[e] = has_pre ? sr.pre_scale[xc + e] : 1.f;
      pre_b[e] = has_pre ? sr.pre_shift[xc + e] : 0.f;
    }
    const T* dcol = dy + co0 + cvd * VEC;
    const T* xcol = x + xc;

    auto load = [&](int st, Regs& R) {
      const long p0 = p_begin + (long)st * BP;
#pragma unroll
      for (int i = 0; i < D_PASSES; ++i) {
        const long m = p0 + rd0 + i * RPP_D;
        // Cout % VEC == 0 on this path, so a 16-B chunk is entirely inside or outside the row
        const bool ok = m < p_end && d_chunk_ok;
        V v = ok ? load16(dcol + m * a.Cout) : V{};
        R.d[i] = v;
      }
#pragma unroll
      for (int i = 0; i < X_PASSES; ++i) {
        const long m = p0 + rx0 + i * RPP_X;
        const int mm = (int)(m < p_end ? m : p_begin);
        const int n = (int)sr.fd_howo.div((uint32_t)mm);
        const int rem = mm - n * HoWo;
        const int ho = (int)sr.fd_wo.div((uint32_t)rem), wo = rem - ho * sr.Wo;
        const int hi = ho * a.stride + dh, wi = wo * a.stride + dw;
        const bool ok = tap_ok && m < p_end && hi >= 0 && hi < sr.H && wi >= 0 && wi < sr.W;
        const int hc = ok ? hi : 0, wc = ok ? wi : 0;
        V v = load16(xcol + ((long)(n * sr.H + hc) * sr.W + wc) * a.Cin);
        R.x[i] = ok ? v : V{};
        R.ok[i] = ok;
      }
    };
    auto store = [&](int buf, const Regs& R) {
      T* D = Ds + buf * DBUF;
      T* X = Xs + buf * XBUF;
#pragma unroll
      for (int i = 0; i < D_PASSES; ++i) {
        store16(&D[(rd0 + i * RPP_D) * LDD + cvd * VEC], R.d[i]);
        if (do_bias) {
          float f[VEC];
          unpack16<T>(R.d[i], f);
#pragma unroll
          for (int e = 0; e < VEC; ++e) bsum[e] += f[e];
        }
      }
#pragma unroll
      for (int i = 0; i < X_PASSES; ++i) {
        V v = R.x[i];
#ifdef HGK_ABL_NO_PRE
        if (false) {
#else
        if (has_pre) {
#endif
          float f[VEC];
          unpack16<T>(v, f);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            const float t = f[e] * pre_s[e] + pre_b[e];
            f[e] = pre_relu ? fmaxf(t, 0.f) : t;
          }
          v = R.ok[i] ? pack16<T>(f) : V{};  // padding taps stay exactly 0 after the transform
        }
        store16(&X[(rx0 + i * RPP_X) * LDX + cvx * VEC], v);
      }
    };
    auto compute = [&](int cur) {
      const T* D = Ds + cur * DBUF;
      const T* X = Xs + cur * XBUF;
      if constexpr (sizeof(T) == 4) {
        const float* Df = reinterpret_cast<const float*>(D);
        const float* Xf = reinterpret_cast<const float*>(X);
#pragma unroll
        for (int kk = 0; kk < BP / 4; ++kk) {
          float av[FM], bv[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) av[i] = Df[(kk * 4 + lg) * LDD + wm * WTM + i * 16 + lr];
#pragma unroll
          for (int j = 0; j < FN; ++j) bv[j] = Xf[(kk * 4 + lg) * LDX + wn * WTN + j * 16 + lr];
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
      } else {
        // fragment element j of lane group g <-> pixel 4g+j (j<4) / 16+4g+(j-4): each
        // ds_read_b64_tr_b16 reads 8 consecutive rows per 32-lane half -> conflict-free
        const int q = lr >> 2, p4 = lr & 3;
        typedef short s16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int kk = 0; kk < BP / 32; ++kk) {
          bf16x8 av[FM], bv[FN];
          const int prow = kk * 32 + 4 * lg + q;
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const T* base = &D[prow * LDD + wm * WTM + i * 16 + 4 * p4];
#ifdef HGK_ABL_NO_TR
            s16x4 lo4 = {(short)base[0].v, 0, 0, 0}, hi4 = {0, 0, 0, 0};
#else
            s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
            s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 16 * LDD));
#endif
            s16x8 c = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            av[i] = __builtin_bit_cast(bf16x8, c);
          }
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const T* base = &X[prow * LDX + wn * WTN + j * 16 + 4 * p4];
            s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
            s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 16 * LDX));
            s16x8 c = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            bv[j] = __builtin_bit_cast(bf16x8, c);
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
      }
    };
    if (nstage > 0) {
      load(0, R0);
      store(0, R0);
    }
    __syncthreads();
    for (int st = 0; st < nstage; ++st) {
      const bool more = st + 1 < nstage;
      if (more) load(st + 1, R0);
      compute(st & 1);
      if (more) store((st + 1) & 1, R0);  // that buffer was last read before the previous barrier
      __syncthreads();
    }
  }

  // partial slab [split][Cout][K]
  slab_rmw<FM, FN>(a.slab + (long)split * a.Cout * a.K, a.K, a.Cout, split < a.s_init,
                   co0 + wm * WTM + lg * 4, k0 + wn * WTN + lr, acc);
  if (do_bias) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) sBias[rd0 * BMO + cvd * VEC + e] = bsum[e];
    __syncthreads();
    for (int c = tid; c < BMO; c += NT) {
      float sb = 0.f;
      for (int r = 0; r < RPP_D; ++r) sb += sBias[r * BMO + c];
      if (co0 + c < a.Cout) {
        float* d = &a.slab_b[(long)split * a.Cout + co0 + c];
        *d = split < a.s_init ? *d + sb : sb;
      }
    }
  }
}

__host__ __device__ inline WgradSrc wgrad_src_of(const ConvWgradArgs& a) {
  return WgradSrc{a.x, a.dy, a.pre_scale, a.pre_shift, 0L, (int)a.M, a.H, a.W, a.Ho, a.Wo,
                  a.pre_relu, a.fd_howo, a.fd_wo};
}

template <typename T, int BMO, int BNO, int WM, int WN, bool SMALLC = false>
__global__ __launch_bounds__(64 * WM * WN) HGK_WPE_WGRAD void conv_wgrad_fast_kernel(ConvWgradArgs a) {
  const WgradSrc s = wgrad_src_of(a);
  wgrad_fast_body<T, BMO, BNO, WM, WN, SMALLC>(a, &s, 1, blockIdx.x);
}

template <typename T, int BMO, int BNO, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) HGK_WPE_WGRAD void conv_wgrad_multi_kernel(ConvWgradMultiArgs m) {
  wgrad_fast_body<T, BMO, BNO, WM, WN, false>(m.a, m.src, m.nsrc, blockIdx.x);
}

// hgk_conv_wgrad_accum_batch: jobs of DIFFERENT weights (one use each, one tile plan) in one
// grid; job j owns blocks [off[j], off[j + 1]) (multiples of 8: the XCD grouping is kept) and runs
// exactly its single launch's body
static constexpr int kWgBatch = 12;
struct WgradBatchArgs {
  ConvWgradArgs a[kWgBatch];
  WgradSrc src[kWgBatch];
  int off[kWgBatch + 1];
  int n;
};
static_assert(sizeof(WgradBatchArgs) <= 4096, "kernel argument segment");

template <typename T, int BMO, int BNO, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) HGK_WPE_WGRAD void conv_wgrad_batch_kernel(WgradBatchArgs m) {
  int j = 0;
  while (j + 1 < m.n && (int)blockIdx.x >= m.off[j + 1]) ++j;
  wgrad_fast_body<T, BMO, BNO, WM, WN, false>(m.a[j], &m.src[j], 1, (int)blockIdx.x - m.off[j]);
}

// dw[co][ci][kh][kw] += sum_s slab[s][co][k], k = (kh*KW+kw)*Cin+ci ; db[co] += sum_s slab_b[s][co]
// A workgroup owns 64 float4 columns; its G waves each sum every G-th split with 8 loads in
// flight (G = 16 for many splits: ~one HBM round trip per wave instead of S/4 serial ones), then
// the G wave sums are added in a fixed order through LDS (deterministic). Slabs are over the
// STORED channel counts; only the logical [Cout_log][Cin_log] part exists in the canonical weight
// (channel-padded heads).
template <int G>
__global__ __launch_bounds__(64 * G) void wgrad_reduce_kernel(
    const float* __restrict__ slab, const float* __restrict__ slab_b, float* __restrict__ dw,
    float* __restrict__ db, int S, int Cout, int K, int Cin, int KH, int KW, int Cout_log,
    int Cin_log) {
  constexpr int U = 8;
  __shared__ float4 part[G][64];
  const long total = (long)Cout * K;
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const long i0 = ((long)blockIdx.x * 64 + lane) * 4;
  const bool vec = (total & 3) == 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 < total) {
    if (vec) {
      for (int s0 = grp; s0 < S; s0 += G * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int sc = min(s0 + G * u, S - 1);  // clamped: all U loads issued together
          v[u] = *reinterpret_cast<const float4*>(slab + (long)sc * total + i0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (s0 + G * u < S) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
        }
      }
    } else {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = grp; s < S; s += G)
        for (int u = 0; u < 4; ++u)
          if (i0 + u < total) t[u] += slab[(long)s * total + i0 + u];
      acc = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
  part[grp][lane] = acc;
  __syncthreads();
  if (grp == 0 && i0 < total) {
    float r[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int q = 1; q < G; ++q) {
      const float4 p = part[q][lane];
      r[0] += p.x; r[1] += p.y; r[2] += p.z; r[3] += p.w;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long idx = i0 + u;
      if (idx >= total) break;
      const int co = (int)(idx / K);
      const int k = (int)(idx - (long)co * K);
      const int tap = k / Cin, ci = k - tap * Cin;
      const int kh = tap / KW, kw = tap - kh * KW;
      if (co < Cout_log && ci < Cin_log)
        dw[(((long)co * Cin_log + ci) * KH + kh) * KW + kw] += r[u];
    }
  }
  if (db && (long)blockIdx.x * 64 < Cout_log) {
    // bias: the first ceil(Cout/64) workgroups, lane = channel, the G waves split the slabs
    const int c = blockIdx.x * 64 + lane;
    const int cc = min(c, Cout - 1);
    float sb = 0.f;
    for (int s0 = grp; s0 < S; s0 += G * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = slab_b[(long)min(s0 + G * u, S - 1) * Cout + cc];
#pragma unroll
      for (int u = 0; u < U; ++u) sb += (s0 + G * u < S) ? v[u] : 0.f;
    }
    __syncthreads();
    float* pb = reinterpret_cast<float*>(part);
    pb[grp * 64 + lane] = sb;
    __syncthreads();
    if (grp == 0 && c < Cout_log) {
      float r = pb[lane];
      for (int q = 1; q < G; ++q) r += pb[q * 64 + lane];
      db[c] += r;
    }
  }
}

// Every weight's slab reduction of one flush point in ONE launch (hgk_conv_wgrad_finish_multi):
// workgroups [b0_i, b0_{i+1}) reduce weight i exactly as wgrad_reduce_kernel<G_i> would (G_i = 16
// waves per 256-element column chunk for >= 64 slabs, else 4), so the result is bitwise the same.
// A G = 4 weight's workgroup takes 16 / G = 4 consecutive chunks, one per 4-wave group: every wave
// works (with one chunk per workgroup, 12 of 16 waves idled and the unshared models' reduction —
// mostly weights of < 64 slabs, 2.4 GB per hourglass_compare step — streamed at 2.3 TB/s).
static constexpr int kFinMulti = 32;
struct WgradFinDesc {
  const float* slab;
  const float* slab_b;
  float* dw;
  float* db;
  int S, Cout, K, Cin, KH, KW, Cout_log, Cin_log, b0;
};
struct WgradFinMultiArgs {
  WgradFinDesc d[kFinMulti];
  int n;
};

__global__ __launch_bounds__(1024) void wgrad_reduce_multi_kernel(WgradFinMultiArgs m) {
  constexpr int U = 8;
  __shared__ float4 part[16][64];
  int i = 0;
  while (i + 1 < m.n && (int)blockIdx.x >= m.d[i + 1].b0) ++i;
  const WgradFinDesc& d = m.d[i];
  const int bx = (int)blockIdx.x - d.b0;
  const int G = d.S >= 64 ? 16 : 4, NSUB = 16 / G;
  const float* __restrict__ slab = d.slab;
  const int S = d.S, Cout = d.Cout, K = d.K, Cin = d.Cin, KW = d.KW, KH = d.KH;
  const long total = (long)Cout * K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = wave / G, grp = wave - sub * G;  // column chunk of the workgroup, slab group
  const long chunk = (long)bx * NSUB + sub;
  const long i0 = (chunk * 64 + lane) * 4;
  const bool vec = (total & 3) == 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 < total) {
    if (vec) {
      for (int s0 = grp; s0 < S; s0 += G * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int sc = min(s0 + G * u, S - 1);
          v[u] = *reinterpret_cast<const float4*>(slab + (long)sc * total + i0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (s0 + G * u < S) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
        }
      }
    } else {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = grp; s < S; s += G)
        for (int u = 0; u < 4; ++u)
          if (i0 + u < total) t[u] += slab[(long)s * total + i0 + u];
      acc = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (grp == 0 && i0 < total) {
    float r[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int q = 1; q < G; ++q) {
      const float4 p = part[sub * G + q][lane];
      r[0] += p.x; r[1] += p.y; r[2] += p.z; r[3] += p.w;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long idx = i0 + u;
      if (idx >= total) break;
      const int co = (int)(idx / K);
      const int k = (int)(idx - (long)co * K);
      const int tap = k / Cin, ci = k - tap * Cin;
      const int kh = tap / KW, kw = tap - kh * KW;
      if (co < d.Cout_log && ci < d.Cin_log)
        d.dw[(((long)co * d.Cin_log + ci) * KH + kh) * KW + kw] += r[u];
    }
  }
  if (d.db && (long)bx * NSUB * 64 < d.Cout_log) {  // workgroup-uniform (barriers inside)
    const int c = (int)chunk * 64 + lane;
    const int cc = min(c, Cout - 1);
    float sb = 0.f;
    for (int s0 = grp; s0 < S; s0 += G * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = d.slab_b[(long)min(s0 + G * u, S - 1) * Cout + cc];
#pragma unroll
      for (int u = 0; u < U; ++u) sb += (s0 + G * u < S) ? v[u] : 0.f;
    }
    __syncthreads();
    float* pb = reinterpret_cast<float*>(part);
    pb[wave * 64 + lane] = sb;
    __syncthreads();
    if (grp == 0 && c < d.Cout_log) {
      float r = pb[sub * G * 64 + lane];
      for (int q = 1; q < G; ++q) r += pb[(sub * G + q) * 64 + lane];
      d.db[c] += r;
    }
  }
}

// canonical fp32 [Cout][Cin][KH][KW] -> packed [rows_pad][w_ld]
__device__ __forceinline__ float pack_weight_value(const float* __restrict__ w, long idx, int w_ld,
                                                   int Cout, int Cin, int KH, int KW, int dgrad,
                                                   int Cout_st, int Cin_st) {
  const int r = (int)(idx / w_ld);
  const int k = (int)(idx - (long)r * w_ld);
  float v = 0.f;
  if (!dgrad) {
    // row = co, k = (kh*KW+kw)*Cin_st + ci  (ci >= Cin: channel padding of the stored input)
    if (r < Cout && k < KH * KW * Cin_st) {
      int tap = k / Cin_st, ci = k - tap * Cin_st;
      int kh = tap / KW, kw = tap - kh * KW;
      if (ci < Cin) v = w[(((long)r * Cin + ci) * KH + kh) * KW + kw];
    }
  } else {
    // row = ci, k = (kh'*KW+kw')*Cout_st + co ; value w[co][ci][KH-1-kh'][KW-1-kw']
    if (r < Cin && k < KH * KW * Cout_st) {
      int tap = k / Cout_st, co = k - tap * Cout_st;
      int kh = tap / KW, kw = tap - kh * KW;
      if (co < Cout) v = w[(((long)co * Cin + r) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)];
    }
  }
  return v;
}

template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, T* __restrict__ out, int w_ld,
                                   int rows_pad, int Cout, int Cin, int KH, int KW, int dgrad,
                                   int Cout_st, int Cin_st) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)rows_pad * w_ld) return;
  out[idx] = from_f<T>(pack_weight_value(w, idx, w_ld, Cout, Cin, KH, KW, dgrad, Cout_st, Cin_st));
}

// every weight of a training step packed in ONE launch (blockIdx.y = descriptor): a step packs
// ~60 weight layouts, each launch ~4.7 us mostly fixed cost
static constexpr int kPackMulti = 48;
struct PackMultiArgs {
  hgk_pack_desc d[kPackMulti];
  int n;
};

// a thread packs 8 consecutive elements of a packed row (w_ld % 64 == 0): one 16-B (bf16) store,
// 32-bit index arithmetic once per chunk; when the stored channel count is a multiple of 8 the
// chunk is 8 consecutive channels of one tap (every layout of the models), else per element
template <typename T>
__global__ __launch_bounds__(256) void pack_weight_multi_kernel(PackMultiArgs a) {
  const hgk_pack_desc& d = a.d[blockIdx.y];
  const int cpr = d.w_ld / 8;  // chunks per packed row
  const int total = (d.rows_store + 127) / 128 * 128 * cpr;
  const int dg = d.for_dgrad;
  const int Cst = dg ? d.Cout_store : d.Cin_store;  // channels per tap in a packed row
  const int Klen = d.KH * d.KW * Cst;
  const int rows = dg ? d.Cin : d.Cout, cl = dg ? d.Cout : d.Cin;  // logical row / channel counts
  const bool grp8 = (Cst & 7) == 0;
  T* out = reinterpret_cast<T*>(d.packed);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < total; c += gridDim.x * blockDim.x) {
    const int r = c / cpr;
    const int k0 = (c - r * cpr) * 8;
    float v[8];
    if (grp8) {
      const int tap = k0 / Cst, c0 = k0 - tap * Cst;
      const int kh = tap / d.KW, kw = tap - kh * d.KW;
      const bool ok = r < rows && k0 < Klen;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = c0 + e;
        v[e] = 0.f;
        if (ok && ch < cl)
          v[e] = dg ? d.w[(((long)ch * d.Cin + r) * d.KH + (d.KH - 1 - kh)) * d.KW + (d.KW - 1 - kw)]
                    : d.w[(((long)r * d.Cin + ch) * d.KH + kh) * d.KW + kw];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = pack_weight_value(d.w, (long)c * 8 + e, d.w_ld, d.Cout, d.Cin, d.KH, d.KW, dg,
                                 d.Cout_store, d.Cin_store);
    }
    constexpr int VN = Vec16<T>::N;  // round-to-nearest-even as from_f
#pragma unroll
    for (int q = 0; q < 8 / VN; ++q) store16(out + (long)c * 8 + q * VN, pack16<T>(v + q * VN));
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
// split-K plan for small-M launches (the 8x8 / 4x4 hourglass levels have too few M-tiles to
// fill 256 CUs, and each would otherwise walk all K = 9*Cin serially)

static int fwd_ksplit(long blocks, int nk) {
  static const int min_blocks = 128;
  static const int target = 256;
  static const int min_nk = 5;  // 1x1 (<= 4 k-tiles): no split
  if (blocks >= min_blocks || nk < min_nk) return 1;
  int ks = (int)std::min<long>(nk, std::max<long>(1, (target + blocks - 1) / blocks));
  const int per = (nk + ks - 1) / ks;
  return (nk + per - 1) / per;
}

template <typename T, int BM, int BN, int WM, int WN>
static int launch_fwd_smallc(hipStream_t st, ConvFwdArgs& a, int* rows_out) {
  const int gx = ceil_div(a.M, BM), gy = ceil_div(a.Cout, BN);
  constexpr int NH = conv_stats_halves<T, BM, BN>();
  if ((a.stats || a.bb_partial) && gx * NH > kMaxStatsRows) {
    set_error("conv_fwd: %d stats rows exceed the maximum %d", gx * NH, kMaxStatsRows);
    return HGK_ERR_UNSUPPORTED;
  }
  a.stats_R = gx * NH;
  hipLaunchKernelGGL((conv_fwd_kernel<T, BM, BN, WM, WN, false, false, true>), dim3(gx, gy),
                     dim3(64 * WM * WN), 0, st, a, a, kNoTwin);
  HGK_LAUNCH_CHECK();
  if (rows_out) *rows_out = (a.stats || a.bb_partial) ? gx * NH : 0;
  return HGK_OK;
}

// split-K plan of an implicit-GEMM launch. Few-workgroup launches (the small hourglass levels)
// take the all-ahead kernel: at most `ka` k-tiles per workgroup, all loads issued up front (one
// memory round trip instead of one per k-tile); ks grows until every split fits. HGK_AHEAD=0
// disables, HGK_AHEAD_BLOCKS caps the tile count it applies to.
static int fwd_plan(long blocks, int nk, int ka, bool* ahead) {
  static const int on = 1;
  static const long maxb = 512;
  int ks = fwd_ksplit(blocks, nk);
  *ahead = false;
  if (on && blocks <= maxb && nk >= 2) {
    *ahead = true;
    const int per = (nk + ks - 1) / ks;
    if (per > ka) {
      const int ks2 = (nk + ka - 1) / ka;
      const int per2 = (nk + ks2 - 1) / ks2;
      ks = (nk + per2 - 1) / per2;
    }
  }
  return ks;
}

template <int BM, int BN>
constexpr int ahead_tiles() { return BM * BN <= 64 * 64 ? 6 : 4; }

// a1 != nullptr: twin launch (segment a1's M-tiles follow a's; same weights, Cout, K and plan;
// the split-K workspace holds a's partials then a1's)
#define HGK_FWD_LAUNCH(SK, PFV, KGV, GRID, BLK)                                                   \
  do {                                                                                            \
    if (a1)                                                                                       \
      hipLaunchKernelGGL((conv_fwd_kernel<T, BM, BN, WM, WN, false, SK, false, PFV, KGV, true>),  \
                         GRID, BLK, 0, st, a, b, t0);                                             \
    else                                                                                          \
      hipLaunchKernelGGL((conv_fwd_kernel<T, BM, BN, WM, WN, false, SK, false, PFV, KGV, false>), \
                         GRID, BLK, 0, st, a, b, t0);                                             \
  } while (0)
#define HGK_EPI_LAUNCH()                                                                          \
  do {                                                                                            \
    if (a1)                                                                                       \
      hipLaunchKernelGGL((conv_splitk_epilogue_kernel<T, BM, BN, true>), dim3(gx, gy), dim3(256), \
                         0, st, a, b, t0);                                                        \
    else                                                                                          \
      hipLaunchKernelGGL((conv_splitk_epilogue_kernel<T, BM, BN, false>), dim3(gx, gy),           \
                         dim3(256), 0, st, a, b, t0);                                             \
  } while (0)
template <typename T, int BM, int BN, int WM, int WN>
static int launch_fwd(hipStream_t st, ConvFwdArgs& a, bool generic, int* rows_out, void* ws,
                      size_t ws_bytes, ConvFwdArgs* a1 = nullptr, int* rows_out1 = nullptr) {
  const int gx0 = ceil_div(a.M, BM), gy = ceil_div(a.Cout, BN);
  const int gx1 = a1 ? ceil_div(a1->M, BM) : 0;
  const int gx = gx0 + gx1;
  const long Mtot = a.M + (a1 ? a1->M : 0);
  constexpr int NH = conv_stats_halves<T, BM, BN>();
  if ((a.stats || a.bb_partial) && std::max(gx0, gx1) * NH > kMaxStatsRows) {
    set_error("conv_fwd: %d stats rows exceed the maximum %d", std::max(gx0, gx1) * NH, kMaxStatsRows);
    return HGK_ERR_UNSUPPORTED;
  }
  a.stats_R = gx0 * NH;
  if (a1) a1->stats_R = gx1 * NH;
  const int t0 = a1 ? gx0 : kNoTwin;
  ConvFwdArgs& b = a1 ? *a1 : a;
  // workspace: [kSplitCtrBytes of tile arrival counters][fp32 partials of a (and a1)]
  float* wsp = ws ? reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + kSplitCtrBytes) : nullptr;
  auto set_split = [&](int ks_, int per, bool fixup) {
    int* ctr = fixup && ks_ > 1 && ws && (long)gx * gy <= kSplitCtrBytes / 4 ? reinterpret_cast<int*>(ws)
                                                                             : nullptr;
    a.ksplit = ks_;
    a.kt_per_split = per;
    a.split_ws = wsp;
    a.split_ctr = ctr;
    if (a1) {
      a1->ksplit = ks_;
      a1->kt_per_split = per;
      a1->split_ws = wsp ? wsp + (long)ks_ * a.M * a.Cout : nullptr;
      a1->split_ctr = ctr;
    }
  };
  const int nk = (a.K + MfmaTraits<T>::BK - 1) / MfmaTraits<T>::BK;
  constexpr int KA = ahead_tiles<BM, BN>();
  bool ahead = false;
  int ks = 1;
  if (!generic) {
    ks = fwd_plan((long)gx * gy, nk, KA, &ahead);
    if (!ws || (ks > 1 && (size_t)ks * Mtot * a.Cout * sizeof(float) + kSplitCtrBytes > ws_bytes)) {
      ks = 1;
      ahead = ahead && nk <= KA;
    }
  }
  // k-groups: 3 groups of a 64x64 tile hold 3 x KA k-tiles -> fewer (usually no) splits
  constexpr int KGN = 3;
  static const int kg_on = 1;
  if constexpr (BM == 64 && BN == 64) {
    static const long kg_maxb = 512;
    const int ks2 = (nk + KA * KGN - 1) / (KA * KGN);
    const bool ws_fits = ks2 == 1 || (ws && (size_t)ks2 * Mtot * a.Cout * sizeof(float) + kSplitCtrBytes <= ws_bytes);
    // only for >= 128 tiles (the 16x16 level): with fewer tiles (8x8, 4x4) split-K's extra
    // workgroups beat the groups' shorter chain (3x3 @8x8: 13.4 vs 14.4 us)
    static const long kg_minb = 128;
    if (kg_on && !generic && nk > KA && (long)gx * gy <= kg_maxb && (long)gx * gy >= kg_minb &&
        ws_fits) {
      if (a.fold_part || (a1 && a1->fold_part)) {
        set_error("conv_fwd: the folded BN finalize has no k-group launch (hgk_conv_fold_ok)");
        return HGK_ERR_UNSUPPORTED;
      }
      set_split(ks2, (nk + ks2 - 1) / ks2, false);  // k-groups: the epilogue kernel
      dim3 grid2((unsigned)gx, (unsigned)gy, (unsigned)ks2);
      const dim3 blk2(64 * WM * WN * KGN);
      if (ks2 > 1)
        HGK_FWD_LAUNCH(true, KA, KGN, grid2, blk2);
      else
        HGK_FWD_LAUNCH(false, KA, KGN, grid2, blk2);
      HGK_LAUNCH_CHECK();
      if (ks2 > 1) {
        HGK_EPI_LAUNCH();
        HGK_LAUNCH_CHECK();
      }
      if (rows_out) *rows_out = (a.stats || a.bb_partial) ? gx0 * NH : 0;
      if (rows_out1) *rows_out1 = (a.stats || a.bb_partial) ? gx1 * NH : 0;
      return HGK_OK;
    }
  }
  if ((a.fold_part || (a1 && a1->fold_part)) && (generic || !ahead)) {
    set_error("conv_fwd: the folded BN finalize needs the all-ahead launch (hgk_conv_fold_ok)");
    return HGK_ERR_UNSUPPORTED;
  }
  const int fixup = (int)route(HGK_ROUTE_SPLITK_FIXUP);  // 0: the epilogue kernel (A/B, tests)
  set_split(ks, (nk + ks - 1) / ks, fixup != 0);
  dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)ks);
  const dim3 blk(64 * WM * WN);
  if (generic) {
    if (a1) {
      set_error("conv_fwd_twin: generic (unvectorised) convolutions have no twin launch");
      return HGK_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL((conv_fwd_kernel<T, BM, BN, WM, WN, true>), grid, blk, 0, st, a, b, t0);
  } else if (ahead) {
    if (ks > 1)
      HGK_FWD_LAUNCH(true, KA, 1, grid, blk);
    else
      HGK_FWD_LAUNCH(false, KA, 1, grid, blk);
  } else if (ks > 1)
    HGK_FWD_LAUNCH(true, 1, 1, grid, blk);
  else
    HGK_FWD_LAUNCH(false, 1, 1, grid, blk);
  HGK_LAUNCH_CHECK();
  if (ks > 1 && !a.split_ctr) {
    HGK_EPI_LAUNCH();
    HGK_LAUNCH_CHECK();
  }
  if (rows_out1) *rows_out1 = (a.stats || a.bb_partial) ? gx1 * NH : 0;
  if (rows_out) *rows_out = (a.stats || a.bb_partial) ? gx0 * NH : 0;
  return HGK_OK;
}

template <int TH, int BN = 128>
static int launch_halo(hipStream_t st, ConvFwdArgs& a, int* rows_out) {
  const int gx = a.N * (a.H / TH) * (a.W / 16), gy = ceil_div(a.Cout, BN);
  if ((a.stats || a.bb_partial) && gx > kMaxStatsRows) {
    set_error("conv_fwd: %d stats rows exceed the maximum %d", gx, kMaxStatsRows);
    return HGK_ERR_UNSUPPORTED;
  }
  a.stats_R = gx;
  // <= 512 tiles (the 32x32 level: about one workgroup per CU): two k-groups halve the chain
  static const int kg = 1;
  bool done = false;
  if constexpr (BN == 128 && TH <= 8) {
    if (kg && (long)gx * gy <= 512 && (a.Cin / 64) % 2 == 0) {
      hipLaunchKernelGGL((conv3x3_halo_kernel<TH, 2>), dim3(gx, gy), dim3(512), 0, st, a, a, kNoTwin);
      done = true;
    }
  }
  if constexpr (BN == 64 && TH <= 8) {
    if (!done && (route(HGK_ROUTE_HALO_BN64) & 6) && a.Cout % 128 == 0 && (a.Cin / 64) % 2 == 0) {
      hipLaunchKernelGGL((conv3x3_halo_kernel<TH, 2, 64>), dim3(gx, gy), dim3(512), 0, st, a, a, kNoTwin);
      done = true;
    }
  }
  if (!done)
    hipLaunchKernelGGL((conv3x3_halo_kernel<TH, 1, BN>), dim3(gx, gy), dim3(256), 0, st, a, a,
                       kNoTwin);
  HGK_LAUNCH_CHECK();
  if (rows_out) *rows_out = (a.stats || a.bb_partial) ? gx : 0;
  return HGK_OK;
}

// twin halo launch: both segments tiled TH x 16 (BN = 128), one grid; k-groups as launch_halo
// for the combined tile count
template <int TH>
static int launch_halo_twin(hipStream_t st, ConvFwdArgs& a, ConvFwdArgs& b, int* rows0,
                            int* rows1) {
  const int g0 = a.N * (a.H / TH) * (a.W / 16), g1 = b.N * (b.H / TH) * (b.W / 16);
  const int gy = ceil_div(a.Cout, 128);
  if ((a.stats || a.bb_partial) && std::max(g0, g1) > kMaxStatsRows) {
    set_error("conv_fwd_twin: %d stats rows exceed the maximum %d", std::max(g0, g1), kMaxStatsRows);
    return HGK_ERR_UNSUPPORTED;
  }
  a.stats_R = g0;
  b.stats_R = g1;
  const int gx = g0 + g1;
  static const int kg = 1;
  if (kg && (long)gx * gy <= 512 && (a.Cin / 64) % 2 == 0)
    hipLaunchKernelGGL((conv3x3_halo_kernel<TH, 2, 128, true>), dim3(gx, gy), dim3(512), 0, st, a, b,
                       g0);
  else
    hipLaunchKernelGGL((conv3x3_halo_kernel<TH, 1, 128, true>), dim3(gx, gy), dim3(256), 0, st, a, b,
                       g0);
  HGK_LAUNCH_CHECK();
  if (rows0) *rows0 = (a.stats || a.bb_partial) ? g0 : 0;
  if (rows1) *rows1 = (b.stats || b.bb_partial) ? g1 : 0;
  return HGK_OK;
}

// implicit-GEMM tile: 0 = 128 x 64, 1 = 64 x 128, 2 = 64 x 64 (+ split-K when few workgroups).
// 64 x 128 (each wave 32 x 64) measured fastest on every large-M shape with Cout >= 128
// (scripts/conv_bench.py); small M -> 64 x 64 tiles and split-K.
static int fwd_tile(long M, int Cout) {
  static const int wide_min = 512;  // 256: -0.2 % (same box)
  if (Cout <= 64) return M >= 128L * 256 ? 0 : 2;
  return (long)ceil_div(M, 64) * ceil_div(Cout, 128) >= wide_min ? 1 : 2;
}

#ifndef HGK_HALO64_TH
// output rows per tile of the 64-output-channel 3x3 halo launches (16: half the weight re-streaming
// per pixel, measured within noise of 8, profiles/r05_halo64_th16_ab.txt)
#define HGK_HALO64_TH 8
#endif
// kernel family a forward launch takes (conv_fwd_t); twin launches need kRouteImplicit for both
enum { kRouteImplicit, kRouteSmallC, kRouteHalo8, kRouteHalo64, kRouteHalo4, kRouteRing, kRouteRow3,
       kRouteImg, kRouteStem };

template <typename T>
static int fwd_route(const ConvFwdArgs& a) {
  // the channel-padded network input (Cin = one 16-B chunk): the 7x7 / stride-2 stem of the models
  // (bf16), else any small-channel input conv
  if constexpr (sizeof(T) == 2)
    if (stem_ok(a)) return kRouteStem;
  if (a.Cin == Vec16<T>::N && a.KH * a.KW <= 64 && a.Cout <= 64 && a.M >= 128L * 256 &&
      1)
    return kRouteSmallC;
  if constexpr (sizeof(T) == 2) {
    const bool generic = (a.Cin % MfmaTraits<T>::BK) != 0 || a.KH * a.KW > 32;
    // 3x3 / stride 1 / pad 1 on tileable images: the halo kernel (each input pixel staged once
    // per 64-channel chunk instead of once per tap)
    const int halo = 1;
    if (ring_ok(a)) return kRouteRing;
    if (row3_ok(a)) return kRouteRow3;
    if (img_ok(a)) return kRouteImg;
    const bool h33 = halo && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.dil == 1 &&
                     a.Cin % 64 == 0 && a.Cin <= kHaloPreC && a.W % 16 == 0;
#ifndef HGK_HALO8_MINT
#define HGK_HALO8_MINT 256  // 8x16-pixel tiles from which 8-row tiles are used (else 4-row)
#endif
    static const long halo8_mint = HGK_HALO8_MINT;
    if (h33 && a.Cout % 128 == 0 && a.H % 8 == 0 &&
        (long)a.N * (a.H / 8) * (a.W / 16) * (a.Cout / 128) >= halo8_mint)
      return kRouteHalo8;
    // 64 output channels (the stem block's 3x3 at 128x128 and its input gradient)
    static const int halo64 = 1;
    if (h33 && halo64 && a.Cout == 64 && a.H % HGK_HALO64_TH == 0 && (long)a.N * (a.H / 8) * (a.W / 16) >= 256)
      return kRouteHalo64;
    // the 16x16 level: 4x16-pixel tiles (128 at N = 32), two k-groups per workgroup
    static const int halo4 = 1;
    if (h33 && halo4 && a.Cout % 128 == 0 && a.H % 4 == 0 &&
        (long)a.N * (a.H / 4) * (a.W / 16) * (a.Cout / 128) >= 128)
      return kRouteHalo4;
  }
  return kRouteImplicit;
}

template <typename T>
static int conv_fwd_t(hipStream_t st, ConvFwdArgs& a, int* rows_out, void* ws, size_t ws_bytes,
                      ConvFwdArgs* a1 = nullptr, int* rows_out1 = nullptr) {
  const bool generic = (a.Cin % MfmaTraits<T>::BK) != 0 || a.KH * a.KW > 32;
  const long Mt = a.M + (a1 ? a1->M : 0);
  switch (a1 ? kRouteImplicit : fwd_route<T>(a)) {
    case kRouteSmallC: return launch_fwd_smallc<T, 128, 64, 4, 1>(st, a, rows_out);
    case kRouteStem: return launch_stem(st, a, rows_out);
    case kRouteRing: return launch_ring(st, a, nullptr, rows_out, nullptr);
    case kRouteRow3: return launch_row3(st, a, nullptr, rows_out, nullptr);
    case kRouteImg: return launch_img(st, a, nullptr, rows_out, nullptr);
    case kRouteHalo8:
      // route halo_bn64 & 4: 64-channel tiles where 128-channel ones leave <= 128 workgroups
      // (the 32x32 level at N <= 16: +0.3 % on try_with_aspp; at 256 workgroups, N = 32, slower)
#ifndef HGK_HALO_BN64_MAXWG
#define HGK_HALO_BN64_MAXWG 128
#endif
      if ((route(HGK_ROUTE_HALO_BN64) & 4) && a.Cout % 128 == 0 &&
          (long)a.N * (a.H / 8) * (a.W / 16) * (a.Cout / 128) <= HGK_HALO_BN64_MAXWG)
        return launch_halo<8, 64>(st, a, rows_out);
      return launch_halo<8>(st, a, rows_out);
    case kRouteHalo64: return launch_halo<HGK_HALO64_TH, 64>(st, a, rows_out);
    case kRouteHalo4:
      // route halo_bn64: 64-channel output tiles (twice the workgroups: 128 -> 256 at N = 32)
      if ((route(HGK_ROUTE_HALO_BN64) & 3) && a.Cout % 64 == 0) return launch_halo<4, 64>(st, a, rows_out);
      return launch_halo<4>(st, a, rows_out);
    default: break;
  }
  switch (fwd_tile(Mt, a.Cout)) {
    case 0: return launch_fwd<T, 128, 64, 4, 1>(st, a, generic, rows_out, ws, ws_bytes, a1, rows_out1);
    case 1: return launch_fwd<T, 64, 128, 2, 2>(st, a, generic, rows_out, ws, ws_bytes, a1, rows_out1);
    default: return launch_fwd<T, 64, 64, 2, 2>(st, a, generic, rows_out, ws, ws_bytes, a1, rows_out1);
  }
}

// upper bound of the weight-grad pixel splits (slab sets are allocated for this many)
#ifndef HGK_WG_TARGET
#define HGK_WG_TARGET 512
#endif
#ifndef HGK_WG_SMAX
#define HGK_WG_SMAX 256
#endif
static constexpr int kMaxWgradSplits = HGK_WG_SMAX > 256 ? HGK_WG_SMAX : 256;

struct WgradPlan {
  int bmo, bno, S;
  long pix_per_split;
  bool generic, smallc;
};

// full-width tiles (HGK_ROUTE_WG_FULL): the whole 128x256 / 256x128 1x1 weight in one 8-wave
// workgroup, so each use's dy and x rows are read once (the 128x128 tiling reads the operand it
// does not tile once per tile); bf16 only (106 KB of LDS: one workgroup per CU)
static bool wgrad_full_ok(int dtype, long M, int Cin, int Cout, int K) {
  const long minm = route(HGK_ROUTE_WG_FULL);
  return minm > 0 && M >= minm && dtype == HGK_BF16 && K == Cin &&
         ((Cout == 128 && Cin == 256) || (Cout == 256 && Cin == 128));
}

#ifndef HGK_SMALLC_BNO
// k columns per weight-gradient tile of the channel-padded stem: 128 (16 taps; dy re-read 4x instead
// of 7x): 124 -> 95.5 us per N=32 launch; 256 (one workgroup per CU by LDS) 123 us
// (profiles/r05_stem_wgrad_bno.txt)
#define HGK_SMALLC_BNO 128
#endif
static WgradPlan wgrad_plan(int dtype, long M, int Cin, int Cout, int K, long target_wg = 0,
                            double slab_cap = 2.0) {
  WgradPlan p;
  const int vec = dtype == HGK_BF16 ? 8 : 4;
  p.smallc = Cin == vec && K / Cin <= 64 && (Cout % 8) == 0;
  p.generic = !p.smallc && ((Cin % 64) != 0 || (Cout % 8) != 0);
  const int BP = 64;
  const bool small = M <= 16384;  // hourglass levels <= 16x16 at N=32
  p.bmo = (Cout <= 64 || small) ? 64 : 128;
  p.bno = (!p.generic && Cin % 128 == 0 && p.bmo == 128) ? 128 : 64;  // launch_wgrad's tiles
  if (p.smallc && p.bmo == 64 && dtype == HGK_BF16) p.bno = HGK_SMALLC_BNO;  // the stem: taps per k-tile
  if (wgrad_full_ok(dtype, M, Cin, Cout, K)) {
    p.bmo = Cout;
    p.bno = K;
  }
  const long tiles = (long)ceil_div(Cout, p.bmo) * ceil_div(K, p.bno);
  const long nsub = (M + BP - 1) / BP;
  // split-K over pixels: ~1.5 workgroups per CU in total, >= min_stages stages per workgroup,
  // and the fp32 partial slabs (S * Cout * K * 4 B, written then re-read) capped at ~2x the
  // bytes of dy + input the GEMM itself reads -> small levels get few splits, many tiles
  // target_wg: a batched launch's share (hgk_conv_wgrad_accum_batch, route wg_batch_target)
  const long target = target_wg > 0 ? target_wg : HGK_WG_TARGET;
  static const long min_stages = 4;
  const double elt = dtype == HGK_BF16 ? 2.0 : 4.0;
  const double main_bytes = (double)M * (Cin + Cout) * elt;
  const double slab_unit = (double)Cout * K * 4.0 * 2.0;
  const long s_bytes = std::max(4L, (long)(slab_cap * main_bytes / slab_unit));
  static const long smax = std::min<long>(kMaxWgradSplits, HGK_WG_SMAX);
  long S = std::min<long>(smax, (target + tiles - 1) / tiles);
  S = std::min(S, std::max(1L, nsub / min_stages));
  S = std::min(S, s_bytes);
  S = std::max(S, 1L);
  long per = (nsub + S - 1) / S;
  p.pix_per_split = per * BP;
  p.S = (int)((M + p.pix_per_split - 1) / p.pix_per_split);
  return p;
}

template <typename T, int BMO, int BNO, int WM, int WN>
static void launch_wgrad(hipStream_t st, ConvWgradArgs& a, const WgradPlan& p) {
  a.gco = ceil_div(a.Cout, BMO);
  a.gk = ceil_div(a.K, BNO);
  a.S = p.S;
  const long s_pad = ((long)p.S + 7) / 8 * 8;
  dim3 grid((unsigned)(s_pad * a.gco * a.gk));
  if (p.generic)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, BMO, BNO, WM, WN, true>), grid, dim3(64 * WM * WN), 0, st, a);
  else if (p.smallc)
    hipLaunchKernelGGL((conv_wgrad_fast_kernel<T, BMO, BNO, 2, 4, true>), grid, dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_fast_kernel<T, BMO, BNO, 2, 4>), grid, dim3(512), 0, st, a);
}

// the channel-padded stem with wider k tiles (HGK_SMALLC_BNO > 64): dy re-read fewer times
template <typename T, int BMO, int BNO>
static void launch_wgrad_smallc(hipStream_t st, ConvWgradArgs& a, const WgradPlan& p) {
  a.gco = ceil_div(a.Cout, BMO);
  a.gk = ceil_div(a.K, BNO);
  a.S = p.S;
  const long s_pad = ((long)p.S + 7) / 8 * 8;
  hipLaunchKernelGGL((conv_wgrad_fast_kernel<T, BMO, BNO, 2, 4, true>), dim3((unsigned)(s_pad * a.gco * a.gk)),
                     dim3(512), 0, st, a);
}

// full-width tiles (wgrad_full_ok): one workgroup per split
template <int BMO, int BNO>
static void launch_wgrad_full(hipStream_t st, ConvWgradArgs& a, const WgradPlan& p) {
  a.gco = 1;
  a.gk = 1;
  a.S = p.S;
  const long s_pad = ((long)p.S + 7) / 8 * 8;
  hipLaunchKernelGGL((conv_wgrad_fast_kernel<bf16_t, BMO, BNO, 2, 4>), dim3((unsigned)s_pad), dim3(512), 0,
                     st, a);
}

template <typename T, int BMO, int BNO>
static void launch_wgrad_multi(hipStream_t st, ConvWgradMultiArgs& m, const WgradPlan& p) {
  m.a.gco = ceil_div(m.a.Cout, BMO);
  m.a.gk = ceil_div(m.a.K, BNO);
  m.a.S = p.S;
  const long s_pad = ((long)p.S + 7) / 8 * 8;
  hipLaunchKernelGGL((conv_wgrad_multi_kernel<T, BMO, BNO, 2, 4>),
                     dim3((unsigned)(s_pad * m.a.gco * m.a.gk)), dim3(512), 0, st, m);
}

// ConvWgradArgs + its one WgradSrc for a batch job (hgk_conv_wgrad_accum_multi's setup, nsrc = 1)
static int wgrad_job_args(int dtype, const hgk_wgrad_job& j, ConvWgradArgs& a, WgradSrc& w,
                          WgradPlan& p, long target_wg = 0) {
  HGK_CHECK_ARG(j.slabs && j.slab_cap > 0 && j.slabs_init >= 0 && j.slabs_init <= j.slab_cap,
                "conv_wgrad_accum_batch: bad slabs");
  HGK_CHECK_ARG(j.Cin % 64 == 0 && j.Cout % 8 == 0 && j.KH > 0 && j.KW > 0 && j.stride > 0 &&
                    j.dil > 0 && j.pad >= 0,
                "conv_wgrad_accum_batch: unsupported geometry (Cin %d, Cout %d)", j.Cin, j.Cout);
  const hgk_wgrad_src& u = j.src;
  HGK_CHECK_ARG(u.x && u.dy && u.N > 0 && u.H > 0 && u.W > 0, "conv_wgrad_accum_batch: source");
  HGK_CHECK_ARG(u.pre_scale == nullptr || u.pre_shift != nullptr, "conv_wgrad_accum_batch: pre_shift");
  const int K = j.KH * j.KW * j.Cin;
  a.x = a.dy = nullptr; a.pre_scale = a.pre_shift = nullptr; a.pre_relu = 0;
  a.N = a.H = a.W = a.Ho = a.Wo = 0;
  a.Cin = j.Cin; a.Cout = j.Cout; a.KH = j.KH; a.KW = j.KW;
  a.stride = j.stride; a.pad = j.pad; a.dil = j.dil; a.K = K;
  a.fd_cin = FastDiv(j.Cin); a.fd_kw = FastDiv(j.KW);
  w.x = u.x; w.dy = u.dy; w.pre_scale = u.pre_scale; w.pre_shift = u.pre_shift;
  w.pre_relu = u.pre_relu; w.H = u.H; w.W = u.W;
  w.Ho = (u.H + 2 * j.pad - j.dil * (j.KH - 1) - 1) / j.stride + 1;
  w.Wo = (u.W + 2 * j.pad - j.dil * (j.KW - 1) - 1) / j.stride + 1;
  HGK_CHECK_ARG(w.Ho > 0 && w.Wo > 0, "conv_wgrad_accum_batch: empty output");
  const long M = (long)u.N * w.Ho * w.Wo;
  HGK_CHECK_ARG(M * (long)std::max(j.Cin, j.Cout) < (1L << 31), "conv_wgrad_accum_batch: tensor too large");
  w.M = (int)M;
  w.m_begin = 0;
  w.fd_howo = FastDiv(w.Ho * w.Wo); w.fd_wo = FastDiv(w.Wo);
  a.M = M;
  a.slab = reinterpret_cast<float*>(j.slabs);
  a.slab_b = j.with_bias ? a.slab + (size_t)j.slab_cap * j.Cout * K : nullptr;
  a.s_init = j.slabs_init;
  // route wg_batch_slab_x10: a batched (single-use) weight's slabs capped at this / 10 x its
  // operand bytes (default 5: +0.7 % on hourglass_compare; multi-use weights keep 2x, where a
  // lower cap measured slower, profiles/r05_wg_slab_cap_ab.txt)
  p = wgrad_plan(dtype, M, j.Cin, j.Cout, K, target_wg,
                 (double)route(HGK_ROUTE_WG_BATCH_SLAB_X10) / 10.0);
  HGK_CHECK_ARG(!p.generic && !p.smallc, "conv_wgrad_accum_batch: unsupported channel counts");
  HGK_CHECK_ARG(p.S <= j.slab_cap, "conv_wgrad: %d splits > slab capacity %d", p.S, j.slab_cap);
  a.pix_per_split = p.pix_per_split;
  a.S = p.S;
  return HGK_OK;
}

template <typename T, int BMO, int BNO>
static void launch_wgrad_batch(hipStream_t st, WgradBatchArgs& m) {
  hipLaunchKernelGGL((conv_wgrad_batch_kernel<T, BMO, BNO, 2, 4>), dim3((unsigned)m.off[m.n]),
                     dim3(512), 0, st, m);
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_max_stats_rows(void) { return kMaxStatsRows; }

int hgk_conv_w_ld(int K) { return ((K + 63) / 64) * 64; }

struct BnBwdFuse {
  const void* y;
  const float *scale, *shift, *mean, *invstd;
  int relu;
  float* partial;
  int* rows_out;
};

// ConvFwdArgs of one convolution (shared by the single and the twin entry points)
static int build_fwd_args(ConvFwdArgs& a, const void* x, const void* w, int w_ld, const float* bias,
                          const void* res, void* y, const float* pre_scale, const float* pre_shift,
                          int pre_relu, int post_relu, float* stats, int N, int H, int W, int Cin,
                          int Cout, int KH, int KW, int stride, int pad, int dil) {
  HGK_CHECK_ARG(x && w && y, "conv_fwd: null tensor");
  HGK_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 &&
                    dil > 0 && pad >= 0,
                "conv_fwd: bad shape");
  a.x = x; a.w = w; a.bias = bias; a.res = res; a.y = y;
  a.pre_scale = pre_scale; a.pre_shift = pre_shift; a.stats = stats;
  a.pre_relu = pre_relu; a.post_relu = post_relu;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW;
  a.stride = stride; a.pad = pad; a.dil = dil;
  a.Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  a.Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  HGK_CHECK_ARG(a.Ho > 0 && a.Wo > 0, "conv_fwd: empty output");
  a.K = KH * KW * Cin;
  a.w_ld = w_ld;
  HGK_CHECK_ARG(w_ld >= a.K && w_ld % 64 == 0, "conv_fwd: w_ld %d invalid for K %d", w_ld, a.K);
  HGK_CHECK_ARG(pre_scale == nullptr || pre_shift != nullptr, "conv_fwd: pre_shift missing");
  HGK_CHECK_ARG(pre_scale == nullptr || Cin <= kMaxPreC, "conv_fwd: fused BN over %d > %d channels",
                Cin, kMaxPreC);
  a.M = (long)N * a.Ho * a.Wo;
  HGK_CHECK_ARG(a.M * (long)std::max(Cin, Cout) < (1L << 31), "conv_fwd: tensor too large");
  a.fd_howo = FastDiv(a.Ho * a.Wo); a.fd_wo = FastDiv(a.Wo);
  a.fd_cin = FastDiv(Cin); a.fd_kw = FastDiv(KW);
  a.split_ws = nullptr; a.ksplit = 1; a.kt_per_split = 0; a.split_ctr = nullptr;
  a.bb_y = nullptr; a.bb_scale = a.bb_shift = a.bb_mean = a.bb_invstd = nullptr;
  a.bb_partial = nullptr; a.bb_relu = 0;
  a.vg_y = nullptr; a.vg_scale = a.vg_shift = a.vg_coef = nullptr; a.vg_out = nullptr; a.vg_relu = 0;
  a.vg_part = nullptr; a.vg_rows = 0; a.vg_training = 0; a.vg_M = 0; a.vg_mean = a.vg_invstd = nullptr;
  a.vg_dgamma = a.vg_dbeta = nullptr; a.vg_add = nullptr;
  a.fold_part = nullptr; a.fold_rows = 0; a.fold_M = 0; a.fold_gamma = a.fold_beta = nullptr;
  a.fold_eps = 0.f; a.fold_stat = nullptr; a.fold_rec = nullptr;
  a.stats_R = 0;
  return HGK_OK;
}

static int set_bnbwd(ConvFwdArgs& a, int dtype, const BnBwdFuse* bb) {
  HGK_CHECK_ARG(bb->y && bb->scale && bb->shift && bb->mean && bb->invstd && bb->partial,
                "conv_fwd_bnbwd: null BN operand");
  HGK_CHECK_ARG(a.stats == nullptr, "conv_fwd_bnbwd: statistics and BN-backward fusion are exclusive");
  HGK_CHECK_ARG(a.Cout % (dtype == HGK_BF16 ? 8 : 4) == 0, "conv_fwd_bnbwd: Cout %d not a 16-B multiple",
                a.Cout);
  a.bb_y = bb->y; a.bb_scale = bb->scale; a.bb_shift = bb->shift; a.bb_mean = bb->mean;
  a.bb_invstd = bb->invstd; a.bb_partial = bb->partial; a.bb_relu = bb->relu;
  return HGK_OK;
}

// the folded BN-backward apply (hgk_conv_fwd_bnbwd_vg / hgk_conv_seg.vg): bf16, and only the
// ring, row-streaming and image-tile kernels stage it (vgrad_route_ok) — any other route would
// read the upstream gradient as if it were dy. With vg->partial the finalize is folded too.
static int set_vgrad(ConvFwdArgs& a, int dtype, const hgk_bn_vgrad* vg) {
  HGK_CHECK_ARG(vg->y && vg->scale && vg->shift && (vg->coef || vg->partial) && vg->out,
                "conv_fwd: null operand of the folded BN-backward apply");
  HGK_CHECK_ARG(dtype == HGK_BF16, "conv_fwd: the folded BN-backward apply is bf16 only");
  HGK_CHECK_ARG(a.pre_scale == nullptr, "conv_fwd: folded apply and BN input transform exclude each other");
  a.vg_y = vg->y; a.vg_scale = vg->scale; a.vg_shift = vg->shift; a.vg_coef = vg->coef;
  a.vg_out = vg->out; a.vg_relu = vg->relu;
  if (vg->partial) {
    HGK_CHECK_ARG(vg->mean && vg->invstd && vg->M > 0 && vg->rows > 0,
                  "conv_fwd: null operand of the folded BN-backward finalize");
    a.vg_part = vg->partial; a.vg_rows = vg->rows; a.vg_M = vg->M; a.vg_training = vg->training;
    a.vg_mean = vg->mean; a.vg_invstd = vg->invstd; a.vg_dgamma = vg->dgamma; a.vg_dbeta = vg->dbeta;
    a.vg_add = vg->add;
    HGK_CHECK_ARG(vg->add == nullptr || vg->add != vg->out, "conv_fwd: folded apply's add aliases its output");
  } else {
    HGK_CHECK_ARG(vg->add == nullptr, "conv_fwd: a folded apply's add needs the folded finalize");
  }
  return HGK_OK;
}

// a kernel stages the folded BN-backward apply (and, with vg_part, its finalize: image tiles only)
static bool vgrad_route_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1) {
  return ring_ok(a, a1) || row3_ok(a, a1) || img_ok(a, a1);
}

// the folded BN finalize (hgk_conv_fwd_fold / hgk_conv_seg.fold)
static int set_fold(ConvFwdArgs& a, int dtype, const hgk_bn_fold* f) {
  HGK_CHECK_ARG(f->partial && f->stat && f->rec && f->M > 0, "conv_fwd_fold: null operand");
  HGK_CHECK_ARG(f->rows > 0 && f->rows <= kFoldRows && f->rows % 4 == 0,
                "conv_fwd_fold: %d partial rows (1..%d, multiple of 4)", f->rows, kFoldRows);
  HGK_CHECK_ARG(dtype == HGK_BF16, "conv_fwd_fold: bf16 only");
  HGK_CHECK_ARG(a.Cin <= 256, "conv_fwd_fold: %d input channels > 256", a.Cin);
  HGK_CHECK_ARG(a.pre_scale == nullptr, "conv_fwd_fold: the fold provides the input transform");
  a.fold_part = f->partial; a.fold_rows = f->rows; a.fold_M = f->M;
  a.fold_gamma = f->gamma; a.fold_beta = f->beta; a.fold_eps = f->eps;
  a.fold_stat = f->stat; a.fold_rec = f->rec;
  return HGK_OK;
}

// launch_fwd's plan for a (twin) conv with a sufficient workspace: the all-ahead implicit-GEMM
// launch with one k-group — the only one that folds a BN finalize
static bool fold_route_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1) {
  const bool generic = (a.Cin % MfmaTraits<bf16_t>::BK) != 0 || a.KH * a.KW > 32;
  if (generic || a.Cin > 256) return false;
  // the image-tile kernel folds too (where the dispatch gives it the launch)
  if (!ring_ok(a, a1) && !row3_ok(a, a1) && img_ok(a, a1)) return true;
  if (a1) {
    if (ring_ok(a, a1) || fwd_route<bf16_t>(a) != kRouteImplicit || fwd_route<bf16_t>(*a1) != kRouteImplicit)
      return false;
  } else if (fwd_route<bf16_t>(a) != kRouteImplicit) {
    return false;
  }
  const long Mt = a.M + (a1 ? a1->M : 0);
  const int tile = fwd_tile(Mt, a.Cout);
  const int BM = tile == 0 ? 128 : 64, BN = tile == 1 ? 128 : 64;
  const long blocks = ((long)ceil_div(a.M, BM) + (a1 ? ceil_div(a1->M, BM) : 0)) * ceil_div(a.Cout, BN);
  const int nk = (a.K + MfmaTraits<bf16_t>::BK - 1) / MfmaTraits<bf16_t>::BK;
  const int KA = BM * BN <= 64 * 64 ? 6 : 4;
  if (BM == 64 && BN == 64 && nk > KA && blocks <= 512 && blocks >= 128) return false;  // k-groups
  bool ahead = false;
  fwd_plan(blocks, nk, KA, &ahead);
  return ahead;
}

static int conv_fwd_impl(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                         const float* bias, const void* res, void* y, const float* pre_scale,
                         const float* pre_shift, int pre_relu, int post_relu, float* stats,
                         int* rows_out, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                         int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                         const BnBwdFuse* bb, const hgk_bn_vgrad* vg = nullptr,
                         const hgk_bn_fold* fold = nullptr) {
  ConvFwdArgs a;
  {
    const int rc0 = build_fwd_args(a, x, w, w_ld, bias, res, y, pre_scale, pre_shift, pre_relu,
                                   post_relu, stats, N, H, W, Cin, Cout, KH, KW, stride, pad, dil);
    if (rc0 != HGK_OK) return rc0;
  }
  if (bb) {
    const int rcb = set_bnbwd(a, dtype, bb);  // partial rows = the launch's statistics rows
    if (rcb != HGK_OK) return rcb;
  }
  if (vg) {
    const int rcv = set_vgrad(a, dtype, vg);
    if (rcv != HGK_OK) return rcv;
    if (!vgrad_route_ok(a, nullptr)) {
      set_error("conv_fwd: no kernel folds the BN-backward apply for this shape (hgk_conv_vgrad_ok)");
      return HGK_ERR_UNSUPPORTED;
    }
  }
  if (fold) {
    const int rcf = set_fold(a, dtype, fold);
    if (rcf != HGK_OK) return rcf;
    if (!fold_route_ok(a, nullptr)) {
      set_error("conv_fwd_fold: no all-ahead launch for this shape (hgk_conv_fold_ok)");
      return HGK_ERR_UNSUPPORTED;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  int rows = 0;
  int rc;
  HGK_DISPATCH_DTYPE(dtype, T, rc = conv_fwd_t<T>(st, a, &rows, workspace, ws_bytes));
  if (rc == HGK_OK) {
    if (rows_out) *rows_out = stats ? rows : 0;
    if (bb && bb->rows_out) *bb->rows_out = rows;
  }
  return rc;
}

int hgk_conv_fwd(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                 const float* bias, const void* res, void* y, const float* pre_scale,
                 const float* pre_shift, int pre_relu, int post_relu, float* stats, int* rows_out,
                 int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                 int dil, void* workspace, size_t ws_bytes) {
  return conv_fwd_impl(stream, dtype, x, w, w_ld, bias, res, y, pre_scale, pre_shift, pre_relu,
                       post_relu, stats, rows_out, N, H, W, Cin, Cout, KH, KW, stride, pad, dil,
                       workspace, ws_bytes, nullptr);
}

int hgk_conv_fwd_bnbwd(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                       const void* res, void* y, int N, int H, int W, int Cin, int Cout, int KH,
                       int KW, int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                       const void* bn_y, const float* bn_scale, const float* bn_shift, int bn_relu,
                       const float* bn_mean, const float* bn_invstd, float* bn_partial,
                       int* bn_rows) {
  BnBwdFuse f{bn_y, bn_scale, bn_shift, bn_mean, bn_invstd, bn_relu, bn_partial, bn_rows};
  return conv_fwd_impl(stream, dtype, x, w, w_ld, nullptr, res, y, nullptr, nullptr, 0, 0,
                       nullptr, nullptr, N, H, W, Cin, Cout, KH, KW, stride, pad, dil, workspace,
                       ws_bytes, &f);
}

int hgk_conv_fwd_bnbwd_vg(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                          const void* res, void* y, int N, int H, int W, int Cin, int Cout, int KH,
                          int KW, int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                          const void* bn_y, const float* bn_scale, const float* bn_shift,
                          int bn_relu, const float* bn_mean, const float* bn_invstd,
                          float* bn_partial, int* bn_rows, const hgk_bn_vgrad* vg) {
  HGK_CHECK_ARG(vg != nullptr, "conv_fwd_bnbwd_vg: null folded apply");
  BnBwdFuse f{bn_y, bn_scale, bn_shift, bn_mean, bn_invstd, bn_relu, bn_partial, bn_rows};
  return conv_fwd_impl(stream, dtype, x, w, w_ld, nullptr, res, y, nullptr, nullptr, 0, 0,
                       nullptr, nullptr, N, H, W, Cin, Cout, KH, KW, stride, pad, dil, workspace,
                       ws_bytes, &f, vg);
}

int hgk_conv_fwd_fold(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                      const float* bias, const void* res, void* y, int pre_relu, int post_relu,
                      float* stats, int* rows_out, int N, int H, int W, int Cin, int Cout, int KH,
                      int KW, int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                      const hgk_bn_fold* fold) {
  HGK_CHECK_ARG(fold != nullptr, "conv_fwd_fold: null fold");
  return conv_fwd_impl(stream, dtype, x, w, w_ld, bias, res, y, nullptr, nullptr, pre_relu,
                       post_relu, stats, rows_out, N, H, W, Cin, Cout, KH, KW, stride, pad, dil,
                       workspace, ws_bytes, nullptr, nullptr, fold);
}

int hgk_conv_fwd_kernel_family(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin,
                               int Cout, int KH, int KW, int stride, int pad, int dil) {
  HGK_CHECK_ARG(dtype == HGK_F32 || dtype == HGK_BF16, "kernel_family: dtype %d", dtype);
  void* p = reinterpret_cast<void*>(256);
  float* fp = reinterpret_cast<float*>(256);
  const int w_ld = (KH * KW * Cin + 63) / 64 * 64;
  ConvFwdArgs a[2];
  const int n = N1 > 0 ? 2 : 1;
  for (int s = 0; s < n; ++s) {
    const int rc = build_fwd_args(a[s], p, p, w_ld, nullptr, nullptr, p, nullptr, nullptr, 1, 0, fp,
                                  s ? N1 : N0, s ? H1 : H0, s ? W1 : W0, Cin, Cout, KH, KW, stride,
                                  pad, dil);
    if (rc != HGK_OK) return rc;
  }
  auto fam = [](int r) {
    switch (r) {
      case kRouteSmallC: return (int)HGK_KFAM_SMALLC;
      case kRouteStem: return (int)HGK_KFAM_STEM;
      case kRouteHalo8: case kRouteHalo64: case kRouteHalo4: return (int)HGK_KFAM_HALO;
      case kRouteRing: return (int)HGK_KFAM_RING;
      case kRouteRow3: return (int)HGK_KFAM_ROW3;
      case kRouteImg: return (int)HGK_KFAM_IMG;
      default: return (int)HGK_KFAM_IMPLICIT;
    }
  };
  if (dtype == HGK_F32) {
    if (n == 1) return fam(fwd_route<float>(a[0]));
    return (fwd_route<float>(a[0]) == kRouteImplicit && fwd_route<float>(a[1]) == kRouteImplicit)
               ? (int)HGK_KFAM_IMPLICIT : (int)HGK_KFAM_SPLIT;
  }
  if (n == 1) return fam(fwd_route<bf16_t>(a[0]));
  // the twin dispatch of hgk_conv_fwd_twin, in its order
  const int r0 = fwd_route<bf16_t>(a[0]), r1 = fwd_route<bf16_t>(a[1]);
  if (ring_ok(a[0], &a[1])) return HGK_KFAM_RING;
  if (row3_ok(a[0], &a[1])) return HGK_KFAM_ROW3;
  if (img_ok(a[0], &a[1])) return HGK_KFAM_IMG;
  if (Cin % 64 == 0 && KH * KW <= 32 && r0 == kRouteImplicit && r1 == kRouteImplicit) return HGK_KFAM_IMPLICIT;
  if (r0 == kRouteHalo8 && r1 == kRouteHalo8) return HGK_KFAM_HALO;
  return HGK_KFAM_SPLIT;
}

int hgk_conv_fold_ok(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin, int Cout,
                     int KH, int KW, int stride, int pad, int dil, int rows0, int rows1) {
  if (dtype != HGK_BF16) return 0;
  void* p = reinterpret_cast<void*>(256);
  float* fp = reinterpret_cast<float*>(256);
  const int w_ld = (KH * KW * Cin + 63) / 64 * 64;
  ConvFwdArgs a[2];
  const int n = N1 > 0 ? 2 : 1;
  for (int s = 0; s < n; ++s) {
    if (build_fwd_args(a[s], p, p, w_ld, nullptr, nullptr, p, nullptr, nullptr, 1, 0, fp,
                       s ? N1 : N0, s ? H1 : H0, s ? W1 : W0, Cin, Cout, KH, KW, stride, pad,
                       dil) != HGK_OK)
      return 0;
    hgk_bn_fold f{fp, s ? rows1 : rows0, 1, nullptr, nullptr, 1e-5f, fp, reinterpret_cast<double*>(p)};
    if (set_fold(a[s], dtype, &f) != HGK_OK) return 0;
  }
  return fold_route_ok(a[0], n == 2 ? &a[1] : nullptr) ? 1 : 0;
}

int hgk_conv_vgrad_ok(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin, int Cout,
                      int KH, int KW, int stride, int pad, int dil, int bn_bwd) {
  if (dtype != HGK_BF16) return 0;
  // shape-only check: stand-in pointers, never dereferenced
  void* p = reinterpret_cast<void*>(256);
  const float* fp = reinterpret_cast<const float*>(256);
  const int w_ld = (KH * KW * Cin + 63) / 64 * 64;
  hgk_bn_vgrad vg{p, fp, fp, fp, 1, p, nullptr, 0, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr};
  BnBwdFuse bb{p, fp, fp, fp, fp, 1, const_cast<float*>(fp), nullptr};
  ConvFwdArgs a[2];
  const int n = N1 > 0 ? 2 : 1;
  for (int s = 0; s < n; ++s) {
    if (build_fwd_args(a[s], p, p, w_ld, nullptr, nullptr, p, nullptr, nullptr, 0, 0, nullptr,
                       s ? N1 : N0, s ? H1 : H0, s ? W1 : W0, Cin, Cout, KH, KW, stride, pad,
                       dil) != HGK_OK)
      return 0;
    if (bn_bwd && set_bnbwd(a[s], dtype, &bb) != HGK_OK) return 0;
    if (set_vgrad(a[s], dtype, &vg) != HGK_OK) return 0;
  }
  return vgrad_route_ok(a[0], n == 2 ? &a[1] : nullptr) ? 1 : 0;
}

int hgk_conv_vgrad_fin_ok(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin,
                          int Cout, int KH, int KW, int stride, int pad, int dil, int bn_bwd,
                          int rows0, int rows1, int add) {
  if (dtype != HGK_BF16) return 0;
  void* p = reinterpret_cast<void*>(256);
  float* fp = reinterpret_cast<float*>(256);
  const int w_ld = (KH * KW * Cin + 63) / 64 * 64;
  BnBwdFuse bb{p, fp, fp, fp, fp, 1, fp, nullptr};
  ConvFwdArgs a[2];
  const int n = N1 > 0 ? 2 : 1;
  for (int s = 0; s < n; ++s) {
    if (build_fwd_args(a[s], p, p, w_ld, nullptr, nullptr, p, nullptr, nullptr, 0, 0, nullptr,
                       s ? N1 : N0, s ? H1 : H0, s ? W1 : W0, Cin, Cout, KH, KW, stride, pad,
                       dil) != HGK_OK)
      return 0;
    const long M = (long)(s ? N1 : N0) * (s ? H1 : H0) * (s ? W1 : W0);
    hgk_bn_vgrad vg{p, fp, fp, nullptr, 1, reinterpret_cast<void*>(512), fp, s ? rows1 : rows0, M,
                    fp, fp, 1, fp, fp, add ? p : nullptr};
    if (bn_bwd && set_bnbwd(a[s], dtype, &bb) != HGK_OK) return 0;
    if (set_vgrad(a[s], dtype, &vg) != HGK_OK) return 0;
  }
  return vgrad_route_ok(a[0], n == 2 ? &a[1] : nullptr) ? 1 : 0;
}

size_t hgk_conv_fwd_workspace(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                              int stride, int pad, int dil) {
  const int Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  const long M = (long)N * Ho * Wo;
  const int K = KH * KW * Cin;
  const int BK = dtype == HGK_BF16 ? 64 : 32;
  const int nk = (K + BK - 1) / BK;
  // tile choice mirrors conv_fwd_t (split-K only on the implicit-GEMM path)
  const int tile = fwd_tile(M, Cout);
  const int BM = tile == 0 ? 128 : 64, BN = tile == 1 ? 128 : 64;
  const long blocks = (long)ceil_div(M, BM) * ceil_div(Cout, BN);
  if (Cin % BK != 0 || KH * KW > 32) return 0;  // generic path: no split-K
  bool ahead = false;
  const int ks = fwd_plan(blocks, nk, BM * BN <= 64 * 64 ? 6 : 4, &ahead);
  return ks > 1 ? (size_t)ks * M * Cout * sizeof(float) + kSplitCtrBytes : 0;
}

int hgk_conv_fwd_twin(hgk_stream_t stream, int dtype, const void* w, int w_ld, const float* bias,
                      int pre_relu, int post_relu, int Cin, int Cout, int KH, int KW, int stride,
                      int pad, int dil, const hgk_conv_seg* seg, void* workspace, size_t ws_bytes) {
  HGK_CHECK_ARG(seg != nullptr, "conv_fwd_twin: null segments");
  ConvFwdArgs a[2];
  for (int s = 0; s < 2; ++s) {
    const hgk_conv_seg& g = seg[s];
    const int rc = build_fwd_args(a[s], g.x, w, w_ld, bias, g.res, g.y, g.pre_scale, g.pre_shift,
                                  pre_relu, post_relu, g.stats, g.N, g.H, g.W, Cin, Cout, KH, KW,
                                  stride, pad, dil);
    if (rc != HGK_OK) return rc;
    if (g.bb_partial) {
      BnBwdFuse f{g.bb_y, g.bb_scale, g.bb_shift, g.bb_mean, g.bb_invstd, g.bb_relu, g.bb_partial,
                  g.bb_rows};
      const int rcb = set_bnbwd(a[s], dtype, &f);
      if (rcb != HGK_OK) return rcb;
    }
    if (g.vg) {
      const int rcv = set_vgrad(a[s], dtype, g.vg);
      if (rcv != HGK_OK) return rcv;
    }
    if (g.fold) {
      const int rcf = set_fold(a[s], dtype, g.fold);
      if (rcf != HGK_OK) return rcf;
    }
  }
  if (a[0].fold_part || a[1].fold_part) {
    // both segments fold, in one all-ahead twin launch
    HGK_CHECK_ARG(a[0].fold_part && a[1].fold_part, "conv_fwd_twin: only one segment folds a BN finalize");
    if (!fold_route_ok(a[0], &a[1])) {
      set_error("conv_fwd_twin: no all-ahead twin launch folds these BN finalizes (hgk_conv_fold_ok)");
      return HGK_ERR_UNSUPPORTED;
    }
  }
  if (a[0].vg_y || a[1].vg_y) {
    // both segments fold the apply, in one ring launch (no other kernel stages it)
    HGK_CHECK_ARG(a[0].vg_y && a[1].vg_y, "conv_fwd_twin: only one segment folds the BN-backward apply");
    HGK_CHECK_ARG((a[0].vg_part == nullptr) == (a[1].vg_part == nullptr) &&
                      (a[0].vg_add == nullptr) == (a[1].vg_add == nullptr) &&
                      a[0].vg_dgamma == a[1].vg_dgamma && a[0].vg_dbeta == a[1].vg_dbeta,
                  "conv_fwd_twin: segments differ in the folded BN-backward finalize");
    if (!vgrad_route_ok(a[0], &a[1])) {
      set_error("conv_fwd_twin: no kernel folds the BN-backward apply for these shapes (hgk_conv_vgrad_ok)");
      return HGK_ERR_UNSUPPORTED;
    }
  }
  HGK_CHECK_ARG((a[0].stats == nullptr) == (a[1].stats == nullptr) &&
                    (a[0].bb_partial == nullptr) == (a[1].bb_partial == nullptr),
                "conv_fwd_twin: segments differ in statistics / BN-backward outputs");
  hipStream_t st = (hipStream_t)stream;
  int rows[2] = {0, 0};
  int rc = HGK_OK;
  HGK_DISPATCH_DTYPE(dtype, T, {
    const bool vec = Cin % MfmaTraits<T>::BK == 0 && KH * KW <= 32;
    const int r0 = fwd_route<T>(a[0]), r1 = fwd_route<T>(a[1]);
    // twin halo only where both segments take 8-row tiles on their own (64x64 + 32x32): at
    // 32x32 + 16x16 the combined grid (320 two-group tiles) ends in a partial round and measured
    // 41 vs 23.8 + 14.7 us for the two launches (4-row tiles for both: slower still)
    const int twin_halo = 1;
    const bool halo0 = r0 == kRouteHalo8 || (twin_halo == 2 && r0 == kRouteHalo4);
    const bool halo1 = r1 == kRouteHalo8 || (twin_halo == 2 && r1 == kRouteHalo4);
    if (sizeof(T) == 2 && ring_ok(a[0], &a[1])) {
      // the big-level 1x1 pair (64x64 + 32x32): one ring launch over both block lists
      rc = launch_ring(st, a[0], &a[1], &rows[0], &rows[1]);
    } else if (sizeof(T) == 2 && row3_ok(a[0], &a[1])) {
      // the big-level 3x3 pair (64x64 + 32x32): one row-streaming grid
      rc = launch_row3(st, a[0], &a[1], &rows[0], &rows[1]);
    } else if (sizeof(T) == 2 && img_ok(a[0], &a[1])) {
      // a small-level pair (16x16 + 8x8, 8x8 + 4x4): one image-tile grid
      rc = launch_img(st, a[0], &a[1], &rows[0], &rows[1]);
    } else if (vec && r0 == kRouteImplicit && r1 == kRouteImplicit && 1) {
      rc = conv_fwd_t<T>(st, a[0], &rows[0], workspace, ws_bytes, &a[1], &rows[1]);
    } else if (sizeof(T) == 2 && halo0 && halo1 && twin_halo) {
      // both 3x3 segments take the halo kernel: one grid, 8-row tiles when both heights allow
      // them
      const int th = 8;
      if (th == 8 && a[0].H % 8 == 0 && a[1].H % 8 == 0)
        rc = launch_halo_twin<8>(st, a[0], a[1], &rows[0], &rows[1]);
      else
        rc = launch_halo_twin<4>(st, a[0], a[1], &rows[0], &rows[1]);
    } else {
      // a segment routes to a specialised kernel (halo 3x3, ring 1x1): one launch each
      for (int s = 0; s < 2 && rc == HGK_OK; ++s)
        rc = conv_fwd_t<T>(st, a[s], &rows[s], workspace, ws_bytes);
    }
  });
  if (rc != HGK_OK) return rc;
  for (int s = 0; s < 2; ++s) {
    if (seg[s].rows_out) *seg[s].rows_out = a[s].stats ? rows[s] : 0;
    if (a[s].bb_partial && seg[s].bb_rows) *seg[s].bb_rows = rows[s];
  }
  return HGK_OK;
}

size_t hgk_conv_fwd_twin_workspace(int dtype, int N0, int H0, int W0, int N1, int H1, int W1,
                                   int Cin, int Cout, int KH, int KW, int stride, int pad, int dil) {
  size_t best = std::max(hgk_conv_fwd_workspace(dtype, N0, H0, W0, Cin, Cout, KH, KW, stride, pad, dil),
                         hgk_conv_fwd_workspace(dtype, N1, H1, W1, Cin, Cout, KH, KW, stride, pad, dil));
  auto outm = [&](int N, int H, int W) {
    const int Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
    const int Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
    return (long)N * Ho * Wo;
  };
  const long M0 = outm(N0, H0, W0), M1 = outm(N1, H1, W1);
  const int K = KH * KW * Cin;
  const int BK = dtype == HGK_BF16 ? 64 : 32;
  const int nk = (K + BK - 1) / BK;
  if (Cin % BK != 0 || KH * KW > 32) return best;
  const int tile = fwd_tile(M0 + M1, Cout);
  const int BM = tile == 0 ? 128 : 64, BN = tile == 1 ? 128 : 64;
  const long blocks = ((long)ceil_div(M0, BM) + ceil_div(M1, BM)) * ceil_div(Cout, BN);
  bool ahead = false;
  const int ks = fwd_plan(blocks, nk, BM * BN <= 64 * 64 ? 6 : 4, &ahead);
  if (ks > 1) best = std::max(best, (size_t)ks * (M0 + M1) * Cout * sizeof(float) + kSplitCtrBytes);
  return best;
}

int hgk_pack_conv_weight_multi(hgk_stream_t stream, int dtype, const hgk_pack_desc* descs, int n) {
  HGK_CHECK_ARG(descs && n >= 0, "pack_multi: bad args");
  hipStream_t st = (hipStream_t)stream;
  for (int b = 0; b < n; b += kPackMulti) {
    PackMultiArgs a;
    a.n = std::min(kPackMulti, n - b);
    long most = 0;
    for (int i = 0; i < a.n; ++i) {
      const hgk_pack_desc& d = descs[b + i];
      HGK_CHECK_ARG(d.w && d.packed, "pack_multi: null");
      HGK_CHECK_ARG(d.Cout_store >= d.Cout && d.Cin_store >= d.Cin, "pack_multi: stored < logical");
      const int rows = d.for_dgrad ? d.Cin_store : d.Cout_store;
      const int K = d.KH * d.KW * (d.for_dgrad ? d.Cout_store : d.Cin_store);
      HGK_CHECK_ARG(d.rows_store == rows, "pack_multi: rows_store must be the stored row count");
      HGK_CHECK_ARG(d.w_ld >= K && d.w_ld % 64 == 0, "pack_multi: bad w_ld");
      a.d[i] = d;
      most = std::max(most, (long)((rows + 127) / 128 * 128) * d.w_ld / 8);
    }
    HGK_CHECK_ARG(most * 8 < (1L << 31), "pack_multi: layout too large");
    const unsigned gx = (unsigned)std::min<long>(ceil_div(most, 256), 1024);
    HGK_DISPATCH_DTYPE(dtype, T, {
      hipLaunchKernelGGL(pack_weight_multi_kernel<T>, dim3(gx, (unsigned)a.n), dim3(256), 0, st, a);
    });
    HGK_LAUNCH_CHECK();
  }
  return HGK_OK;
}

int hgk_pack_conv_weight(hgk_stream_t stream, int dtype, const float* w, void* packed, int w_ld,
                         int Cout, int Cin, int KH, int KW, int for_dgrad, int Cout_store,
                         int Cin_store) {
  HGK_CHECK_ARG(w && packed, "pack: null");
  HGK_CHECK_ARG(Cout_store >= Cout && Cin_store >= Cin, "pack: stored channels < logical");
  const int rows = for_dgrad ? Cin_store : Cout_store;
  const int K = KH * KW * (for_dgrad ? Cout_store : Cin_store);
  HGK_CHECK_ARG(w_ld >= K && w_ld % 64 == 0, "pack: bad w_ld");
  const int rows_pad = ((rows + 127) / 128) * 128;
  const long total = (long)rows_pad * w_ld;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(pack_weight_kernel<T>, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st,
                       w, reinterpret_cast<T*>(packed), w_ld, rows_pad, Cout, Cin, KH, KW, for_dgrad,
                       Cout_store, Cin_store);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_conv_wgrad_max_splits(void) { return kMaxWgradSplits; }

#ifdef HGK_WG_TRACE
extern "C" int hgk_debug_wg_trace(void* dst, int reset) {
  if (reset) {
    static unsigned long long zero[256 * 64];
    return hipMemcpyToSymbol(HIP_SYMBOL(hgk::g_wgtrace), zero, sizeof(zero)) == hipSuccess ? 0 : 1;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(hgk::g_wgtrace), sizeof(hgk::g_wgtrace)) == hipSuccess ? 0 : 1;
}
#endif

// spatial tiles per split of the 3x3 halo weight-grad kernel, or 0 when it does not apply;
// *S_out = splits. ~256 workgroups in total.
static int halo_wgrad_plan(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                           int stride, int pad, int dil, int* S_out) {
  if (dtype != HGK_BF16 || KH != 3 || KW != 3 || stride != 1 || pad != 1 || dil != 1 ||
      Cin % 64 || Cout % 64 || H % 8 || W % 16 || Cin > kMaxPreC || !1)
    return 0;
  const int t_total = N * (H / 8) * (W / 16);
  const int tiles = (Cout / 64) * (Cin / 64);
  if (t_total < 128) return 0;  // the 16x16 level and below: implicit GEMM measured faster
#ifndef HGK_HWG_SMAX
#define HGK_HWG_SMAX 256  // 96: -0.24 % (profiles/r03_wgrad_split_ab.txt; the 64-channel 3x3 at 128x128 filled 96 of 256 CUs)
#endif
  int S = std::max(1, std::min(HGK_HWG_SMAX, 256 / tiles));
  S = std::min(S, t_total);
  const int per = (t_total + S - 1) / S;
  *S_out = (t_total + per - 1) / per;
  return per;
}

size_t hgk_conv_wgrad_slab_bytes(int Cin, int Cout, int KH, int KW, int slab_cap) {
  return (size_t)slab_cap * ((size_t)Cout * KH * KW * Cin + Cout) * sizeof(float);
}

size_t hgk_conv_wgrad_workspace(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                int stride, int pad, int dil) {
  const int Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  const long M = (long)N * Ho * Wo;
  const int K = KH * KW * Cin;
  int hS = 0;
  if (halo_wgrad_plan(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, dil, &hS) > 0)
    return hgk_conv_wgrad_slab_bytes(Cin, Cout, KH, KW, hS);
  WgradPlan p = wgrad_plan(dtype, M, Cin, Cout, K);
  return hgk_conv_wgrad_slab_bytes(Cin, Cout, KH, KW, p.S);
}

int hgk_conv_wgrad_accum(hgk_stream_t stream, int dtype, const void* x, const void* dy,
                         const float* pre_scale, const float* pre_shift, int pre_relu,
                         void* slabs, int slab_cap, int slabs_init, int with_bias, int* splits_out,
                         int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int dil) {
  HGK_CHECK_ARG(x && dy && slabs && slab_cap > 0 && slabs_init >= 0 && slabs_init <= slab_cap,
                "conv_wgrad_accum: bad args");
  HGK_CHECK_ARG(pre_scale == nullptr || (pre_shift != nullptr && Cin <= kMaxPreC),
                "conv_wgrad: fused BN over %d channels unsupported", Cin);
  ConvWgradArgs a;
  a.x = x; a.dy = dy; a.pre_scale = pre_scale; a.pre_shift = pre_shift; a.pre_relu = pre_relu;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW;
  a.stride = stride; a.pad = pad; a.dil = dil;
  a.Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  a.Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  a.K = KH * KW * Cin;
  a.M = (long)N * a.Ho * a.Wo;
  HGK_CHECK_ARG(a.M * (long)std::max(Cin, Cout) < (1L << 31), "conv_wgrad: tensor too large");
  a.fd_howo = FastDiv(a.Ho * a.Wo); a.fd_wo = FastDiv(a.Wo);
  a.fd_cin = FastDiv(Cin); a.fd_kw = FastDiv(KW);
  a.slab = reinterpret_cast<float*>(slabs);
  a.slab_b = with_bias ? a.slab + (size_t)slab_cap * Cout * a.K : nullptr;
  a.s_init = slabs_init;
  hipStream_t st = (hipStream_t)stream;
  int hS = 0;
  const int hper = halo_wgrad_plan(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, dil, &hS);
  if (hper > 0) {
    HGK_CHECK_ARG(hS <= slab_cap, "conv_wgrad: %d splits > slab capacity %d", hS, slab_cap);
    a.gco = Cout / 64;
    a.gk = Cin / 64;
    a.S = hS;
    a.pix_per_split = hper;  // spatial tiles per split
    const long s_pad = ((long)hS + 7) / 8 * 8;
    const dim3 grid((unsigned)(s_pad * a.gco * a.gk));
    if (route(HGK_ROUTE_WG_DMA) && pre_scale)
      hipLaunchKernelGGL((conv3x3_wgrad_dma_kernel<8, true>), grid, dim3(512), 0, st, a);
    else if (route(HGK_ROUTE_WG_DMA))
      hipLaunchKernelGGL((conv3x3_wgrad_dma_kernel<8, false>), grid, dim3(512), 0, st, a);
    else
      hipLaunchKernelGGL((conv3x3_wgrad_halo_kernel<8>), grid, dim3(512), 0, st, a);
    HGK_LAUNCH_CHECK();
    if (splits_out) *splits_out = hS;
    return HGK_OK;
  }
  WgradPlan p = wgrad_plan(dtype, a.M, Cin, Cout, a.K);
  HGK_CHECK_ARG(p.S <= slab_cap, "conv_wgrad: %d splits > slab capacity %d", p.S, slab_cap);
  a.pix_per_split = p.pix_per_split;
  if (dtype == HGK_F32) {
    if (p.bmo == 64) launch_wgrad<float, 64, 64, 2, 2>(st, a, p);
    else if (p.bno == 128) launch_wgrad<float, 128, 128, 2, 2>(st, a, p);
    else launch_wgrad<float, 128, 64, 2, 2>(st, a, p);
  } else if (dtype == HGK_BF16) {
    if (p.bmo == 128 && p.bno == 256) launch_wgrad_full<128, 256>(st, a, p);
    else if (p.bmo == 256 && p.bno == 128) launch_wgrad_full<256, 128>(st, a, p);
    else if (p.smallc && p.bmo == 64 && p.bno != 64) launch_wgrad_smallc<bf16_t, 64, HGK_SMALLC_BNO>(st, a, p);
    else if (p.bmo == 64) launch_wgrad<bf16_t, 64, 64, 2, 2>(st, a, p);
    else if (p.bno == 128) launch_wgrad<bf16_t, 128, 128, 2, 2>(st, a, p);
    else launch_wgrad<bf16_t, 128, 64, 2, 2>(st, a, p);
  } else {
    set_error("conv_wgrad: dtype");
    return HGK_ERR_ARG;
  }
  HGK_LAUNCH_CHECK();
  if (splits_out) *splits_out = p.S;
  return HGK_OK;
}

int hgk_conv_wgrad_accum_multi(hgk_stream_t stream, int dtype, const hgk_wgrad_src* src, int nsrc,
                               void* slabs, int slab_cap, int slabs_init, int with_bias,
                               int* splits_out, int Cin, int Cout, int KH, int KW, int stride,
                               int pad, int dil) {
  HGK_CHECK_ARG(src && nsrc > 0 && slabs && slab_cap > 0 && slabs_init >= 0 &&
                    slabs_init <= slab_cap,
                "conv_wgrad_accum_multi: bad args");
  HGK_CHECK_ARG(dtype == HGK_BF16 || dtype == HGK_F32, "conv_wgrad_accum_multi: dtype");
  HGK_CHECK_ARG(Cin % 64 == 0 && Cout % 8 == 0 && KH > 0 && KW > 0 && stride > 0 && dil > 0 &&
                    pad >= 0,
                "conv_wgrad_accum_multi: unsupported geometry (Cin %d, Cout %d)", Cin, Cout);
  hipStream_t st = (hipStream_t)stream;
  const int K = KH * KW * Cin;
  int init = slabs_init;
  // every source valid before the first launch (an error leaves the slabs untouched)
  for (int i = 0; i < nsrc; ++i) {
    const hgk_wgrad_src& u = src[i];
    HGK_CHECK_ARG(u.x && u.dy && u.N > 0 && u.H > 0 && u.W > 0, "conv_wgrad_accum_multi: source %d", i);
    HGK_CHECK_ARG(u.pre_scale == nullptr || u.pre_shift != nullptr, "conv_wgrad_accum_multi: pre_shift");
    HGK_CHECK_ARG((long)u.N * u.H * u.W * (long)std::max(Cin, Cout) < (1L << 31),
                  "conv_wgrad_accum_multi: tensor too large");
  }
  // route wg_halo_multi: the halo-tileable uses of a bf16 3x3 weight in one halo launch over
  // their concatenated tiles (the rest below)
  std::vector<hgk_wgrad_src> rest;
  const long halo_min = route(HGK_ROUTE_WG_HALO_MULTI);
  if (halo_min > 0 && dtype == HGK_BF16 && KH == 3 && KW == 3 && stride == 1 && pad == 1 &&
      dil == 1 && Cout % 64 == 0 && Cin <= kMaxPreC) {
    std::vector<int> hal;
    long t_all = 0;
    for (int i = 0; i < nsrc; ++i) {
      const hgk_wgrad_src& u = src[i];
      if (u.H % 8 == 0 && u.W % 16 == 0) {
        hal.push_back(i);
        t_all += (long)u.N * (u.H / 8) * (u.W / 16);
      } else {
        rest.push_back(u);
      }
    }
    if (!hal.empty() && t_all >= halo_min) {
      const int pairs = (Cout / 64) * (Cin / 64);
      // halo_wgrad_plan's split count over a launch's concatenated tiles; every launch's is
      // checked against the slab capacity before the first launch
      auto plan = [&](size_t c0, int* per_out) {
        const int n = (int)std::min<size_t>(kMaxHaloSrc, hal.size() - c0);
        int t = 0;
        for (int i = 0; i < n; ++i) {
          const hgk_wgrad_src& u = src[hal[c0 + i]];
          t += u.N * (u.H / 8) * (u.W / 16);
        }
        int S = std::max(1, std::min(HGK_HWG_SMAX, 256 / pairs));
        S = std::min(S, t);
        const int per = (t + S - 1) / S;
        if (per_out) *per_out = per;
        return (t + per - 1) / per;
      };
      for (size_t c0 = 0; c0 < hal.size(); c0 += kMaxHaloSrc) {
        const int S = plan(c0, nullptr);
        HGK_CHECK_ARG(S <= slab_cap, "conv_wgrad: %d splits > slab capacity %d", S, slab_cap);
      }
      for (size_t c0 = 0; c0 < hal.size(); c0 += kMaxHaloSrc) {
        const int n = (int)std::min<size_t>(kMaxHaloSrc, hal.size() - c0);
        HaloMultiArgs m;
        ConvWgradArgs& a = m.a;
        a.x = a.dy = nullptr; a.pre_scale = a.pre_shift = nullptr; a.pre_relu = 0;
        a.N = a.H = a.W = a.Ho = a.Wo = 0;
        a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW;
        a.stride = stride; a.pad = pad; a.dil = dil; a.K = K;
        int t = 0;
        for (int i = 0; i < n; ++i) {
          const hgk_wgrad_src& u = src[hal[c0 + i]];
          HaloSrc& h = m.src[i];
          h.x = u.x; h.dy = u.dy; h.pre_scale = u.pre_scale; h.pre_shift = u.pre_shift;
          h.pre_relu = u.pre_relu; h.N = u.N; h.H = u.H; h.W = u.W;
          h.t0 = t;
          t += u.N * (u.H / 8) * (u.W / 16);
        }
        m.nsrc = n;
        m.t_total = t;
        a.M = (long)t * 128;
        int per = 0;
        const int S = plan(c0, &per);
        a.gco = Cout / 64;
        a.gk = Cin / 64;
        a.S = S;
        a.pix_per_split = per;
        a.slab = reinterpret_cast<float*>(slabs);
        a.slab_b = with_bias ? a.slab + (size_t)slab_cap * Cout * K : nullptr;
        a.s_init = init;
        const long s_pad = ((long)S + 7) / 8 * 8;
        hipLaunchKernelGGL((conv3x3_wgrad_halo_multi_kernel<8>), dim3((unsigned)(s_pad * pairs)),
                           dim3(512), 0, st, m);
        HGK_LAUNCH_CHECK();
        init = std::max(init, S);
      }
      if (rest.empty()) {
        if (splits_out) *splits_out = init;
        return HGK_OK;
      }
      src = rest.data();
      nsrc = (int)rest.size();
    }
  }
  // route wg_ring: the LDS-DMA ring kernel (hgk_wgrad_ring.hip) for big bf16 1x1 uses
  const long ring_min = route(HGK_ROUTE_WG_RING);
  if (ring_min > 0 && dtype == HGK_BF16 && KH == 1 && KW == 1 && stride == 1 && pad == 0 &&
      wgrad_ring_shape_ok(Cout, Cin)) {
    long mt = 0;
    bool ok = true;
    for (int i = 0; i < nsrc; ++i) {
      const hgk_wgrad_src& u = src[i];
      HGK_CHECK_ARG(u.x && u.dy && u.N > 0 && u.H > 0 && u.W > 0, "conv_wgrad_accum_multi: source %d", i);
      HGK_CHECK_ARG(u.pre_scale == nullptr || u.pre_shift != nullptr, "conv_wgrad_accum_multi: pre_shift");
      const long M = (long)u.N * u.H * u.W;
      HGK_CHECK_ARG(M * (long)std::max(Cin, Cout) < (1L << 31), "conv_wgrad_accum_multi: tensor too large");
      ok = ok && M % 32 == 0;
      mt += M;
    }
    if (ok && mt >= ring_min) {
      for (int c0 = 0; c0 < nsrc; c0 += kMaxWgradSrc) {
        const int n = std::min(kMaxWgradSrc, nsrc - c0);
        const void* xs[kMaxWgradSrc];
        const void* dys[kMaxWgradSrc];
        const float* psc[kMaxWgradSrc];
        const float* psh[kMaxWgradSrc];
        int prl[kMaxWgradSrc];
        long Ms[kMaxWgradSrc];
        for (int i = 0; i < n; ++i) {
          const hgk_wgrad_src& u = src[c0 + i];
          xs[i] = u.x; dys[i] = u.dy; psc[i] = u.pre_scale; psh[i] = u.pre_shift;
          prl[i] = u.pre_relu; Ms[i] = (long)u.N * u.H * u.W;
        }
        float* sl = reinterpret_cast<float*>(slabs);
        const int S = launch_wgrad_ring(st, xs, dys, psc, psh, prl, Ms, n, sl,
                                        with_bias ? sl + (size_t)slab_cap * Cout * K : nullptr,
                                        slab_cap, init, Cout, Cin);
        HGK_CHECK_ARG(S > 0, "conv_wgrad_accum_multi: ring plan failed (%d uses)", n);
        HGK_LAUNCH_CHECK();
        init = std::max(init, S);
      }
      if (splits_out) *splits_out = init;
      return HGK_OK;
    }
  }
  for (int c0 = 0; c0 < nsrc; c0 += kMaxWgradSrc) {
    const int n = std::min(kMaxWgradSrc, nsrc - c0);
    ConvWgradMultiArgs m;
    ConvWgradArgs& a = m.a;
    a.x = a.dy = nullptr; a.pre_scale = a.pre_shift = nullptr; a.pre_relu = 0;
    a.N = a.H = a.W = a.Ho = a.Wo = 0;
    a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW;
    a.stride = stride; a.pad = pad; a.dil = dil; a.K = K;
    a.fd_cin = FastDiv(Cin); a.fd_kw = FastDiv(KW);
    long mtot = 0;
    for (int i = 0; i < n; ++i) {
      const hgk_wgrad_src& u = src[c0 + i];
      HGK_CHECK_ARG(u.x && u.dy && u.N > 0 && u.H > 0 && u.W > 0, "conv_wgrad_accum_multi: source %d", c0 + i);
      HGK_CHECK_ARG(u.pre_scale == nullptr || u.pre_shift != nullptr, "conv_wgrad_accum_multi: pre_shift");
      WgradSrc& w = m.src[i];
      w.x = u.x; w.dy = u.dy; w.pre_scale = u.pre_scale; w.pre_shift = u.pre_shift;
      w.pre_relu = u.pre_relu; w.H = u.H; w.W = u.W;
      w.Ho = (u.H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
      w.Wo = (u.W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
      HGK_CHECK_ARG(w.Ho > 0 && w.Wo > 0, "conv_wgrad_accum_multi: empty output");
      const long M = (long)u.N * w.Ho * w.Wo;
      HGK_CHECK_ARG(M * (long)std::max(Cin, Cout) < (1L << 31), "conv_wgrad_accum_multi: tensor too large");
      w.M = (int)M;
      w.m_begin = mtot;
      w.fd_howo = FastDiv(w.Ho * w.Wo); w.fd_wo = FastDiv(w.Wo);
      mtot += M;
    }
    m.nsrc = n;
    a.M = mtot;
    a.slab = reinterpret_cast<float*>(slabs);
    a.slab_b = with_bias ? a.slab + (size_t)slab_cap * Cout * K : nullptr;
    a.s_init = init;
    WgradPlan p = wgrad_plan(dtype, mtot, Cin, Cout, K);
    HGK_CHECK_ARG(!p.generic && !p.smallc, "conv_wgrad_accum_multi: unsupported channel counts");
    HGK_CHECK_ARG(p.S <= slab_cap, "conv_wgrad: %d splits > slab capacity %d", p.S, slab_cap);
    a.pix_per_split = p.pix_per_split;
    if (dtype == HGK_F32) {
      if (p.bmo == 64) launch_wgrad_multi<float, 64, 64>(st, m, p);
      else if (p.bno == 128) launch_wgrad_multi<float, 128, 128>(st, m, p);
      else launch_wgrad_multi<float, 128, 64>(st, m, p);
    } else {
      if (p.bmo == 128 && p.bno == 256) launch_wgrad_multi<bf16_t, 128, 256>(st, m, p);
      else if (p.bmo == 256 && p.bno == 128) launch_wgrad_multi<bf16_t, 256, 128>(st, m, p);
      else if (p.bmo == 64) launch_wgrad_multi<bf16_t, 64, 64>(st, m, p);
      else if (p.bno == 128) launch_wgrad_multi<bf16_t, 128, 128>(st, m, p);
      else launch_wgrad_multi<bf16_t, 128, 64>(st, m, p);
    }
    HGK_LAUNCH_CHECK();
    init = std::max(init, p.S);
  }
  if (splits_out) *splits_out = init;
  return HGK_OK;
}

int hgk_conv_wgrad_accum_batch(hgk_stream_t stream, int dtype, const hgk_wgrad_job* jobs, int n,
                               int* splits_out) {
  HGK_CHECK_ARG(n >= 0 && (n == 0 || (jobs && splits_out)), "conv_wgrad_accum_batch: bad args");
  HGK_CHECK_ARG(dtype == HGK_BF16 || dtype == HGK_F32, "conv_wgrad_accum_batch: dtype");
  hipStream_t st = (hipStream_t)stream;
  WgradBatchArgs m;
  int bmo = 0, bno = 0;
  auto flush = [&]() -> int {
    if (m.n == 0) return HGK_OK;
    if (dtype == HGK_F32) {
      if (bmo == 64) launch_wgrad_batch<float, 64, 64>(st, m);
      else if (bno == 128) launch_wgrad_batch<float, 128, 128>(st, m);
      else launch_wgrad_batch<float, 128, 64>(st, m);
    } else {
      if (bmo == 64) launch_wgrad_batch<bf16_t, 64, 64>(st, m);
      else if (bno == 128) launch_wgrad_batch<bf16_t, 128, 128>(st, m);
      else launch_wgrad_batch<bf16_t, 128, 64>(st, m);
    }
    HGK_LAUNCH_CHECK();
    m.n = 0;
    return HGK_OK;
  };
  m.n = 0;
  m.off[0] = 0;
  // route wg_batch_target: the batch's workgroups (all jobs together) instead of each job's own
  // HGK_WG_TARGET — a batch of many weights fills the chip with few pixel splits per weight, and
  // the fp32 partial slabs (S x the weight, written here and re-read by the reduction) shrink
  // with S. Each job gets its share of the tiles-weighted total.
  const long tgt = route(HGK_ROUTE_WG_BATCH_TARGET);
  auto tiles128 = [](const hgk_wgrad_job& j) {
    return (long)ceil_div(j.Cout, 128) * ceil_div(j.KH * j.KW * j.Cin, 128);
  };
  double per_launch = 0.0;  // 128x128 tiles of one launch's jobs (kWgBatch per launch)
  if (tgt > 0 && n > 1) {
    long tiles_all = 0;
    for (int i = 0; i < n; ++i) tiles_all += tiles128(jobs[i]);
    per_launch = (double)tiles_all * std::min(n, kWgBatch) / n;
  }
  // every job's plan first; then the jobs go out grouped by tile shape (one instantiation per
  // launch: fewer, fuller launches than the engine's interleaved order) and, inside a group, longest
  // per-workgroup pixel range first, so the long workgroups are dispatched before the short ones
  // fill the tail. Each job keeps its own tiles, splits and slabs: the results do not depend on
  // the order (bitwise).
  std::vector<ConvWgradArgs> va(n);
  std::vector<WgradSrc> vw(n);
  std::vector<WgradPlan> vp(n);
  std::vector<int> order, full;
  // validate and plan EVERY job before the first launch: an invalid job returns its error with
  // no slab accumulated and splits_out untouched (the caller's slab bookkeeping stays consistent)
  for (int i = 0; i < n; ++i) {
    // S = tgt / per_launch splits for every job: job i's own target is S x its tiles
    const long tj = per_launch > 0.0 ? std::max(1L, (long)(tgt * tiles128(jobs[i]) / per_launch)) : 0;
    const int rc = wgrad_job_args(dtype, jobs[i], va[i], vw[i], vp[i], tj);
    if (rc != HGK_OK) return rc;
    // route wg_full, and a halo-tileable bf16 3x3 use of wg_halo_multi's size: their own launch
    // (hgk_conv_wgrad_accum_multi with one source: the halo kernel's single-use plan)
    const hgk_wgrad_job& jb = jobs[i];
    const long hmin = route(HGK_ROUTE_WG_HALO_MULTI);
    const bool halo = hmin > 0 && dtype == HGK_BF16 && jb.KH == 3 && jb.KW == 3 && jb.stride == 1 &&
                      jb.pad == 1 && jb.dil == 1 && jb.Cin % 64 == 0 && jb.Cout % 64 == 0 &&
                      jb.Cin <= kMaxPreC && jb.src.H % 8 == 0 && jb.src.W % 16 == 0 &&
                      (long)jb.src.N * (jb.src.H / 8) * (jb.src.W / 16) >= hmin;
    // (a single-use 1x1 stays in the batch: the ring launch per job measured slower than the
    // batched tiled launch, profiles/r06_ring64.txt)
    if (vp[i].bmo == 256 || vp[i].bno == 256 || halo) full.push_back(i);
    else order.push_back(i);
  }
  for (int i : full) {
    const hgk_wgrad_job& j = jobs[i];
    const int r2 = hgk_conv_wgrad_accum_multi(stream, dtype, &j.src, 1, j.slabs, j.slab_cap,
                                              j.slabs_init, j.with_bias, &splits_out[i], j.Cin,
                                              j.Cout, j.KH, j.KW, j.stride, j.pad, j.dil);
    if (r2 != HGK_OK) return r2;
  }
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    if (vp[x].bmo != vp[y].bmo) return vp[x].bmo > vp[y].bmo;
    if (vp[x].bno != vp[y].bno) return vp[x].bno > vp[y].bno;
    return vp[x].pix_per_split > vp[y].pix_per_split;
  });
  for (int i : order) {
    ConvWgradArgs& a = va[i];
    const WgradPlan& p = vp[i];
    if (m.n > 0 && (p.bmo != bmo || p.bno != bno || m.n == kWgBatch)) {
      const int r2 = flush();
      if (r2 != HGK_OK) return r2;
      m.off[0] = 0;
    }
    bmo = p.bmo;
    bno = p.bno;
    a.gco = ceil_div(a.Cout, bmo);
    a.gk = ceil_div(a.K, bno);
    const long s_pad = ((long)p.S + 7) / 8 * 8;
    m.a[m.n] = a;
    m.src[m.n] = vw[i];
    m.off[m.n + 1] = m.off[m.n] + (int)(s_pad * a.gco * a.gk);
    ++m.n;
    splits_out[i] = std::max(jobs[i].slabs_init, p.S);
  }
  return flush();
}

int hgk_conv_wgrad_finish(hgk_stream_t stream, const void* slabs, int slab_cap, int nslabs,
                          float* dw, float* db, int Cin, int Cout, int KH, int KW, int Cin_log,
                          int Cout_log) {
  HGK_CHECK_ARG(slabs && dw && nslabs >= 1 && nslabs <= slab_cap, "conv_wgrad_finish: bad args");
  HGK_CHECK_ARG(Cin_log <= Cin && Cout_log <= Cout && Cin_log > 0 && Cout_log > 0,
                "conv_wgrad_finish: logical channels exceed stored");
  const int K = KH * KW * Cin;
  const float* slab = reinterpret_cast<const float*>(slabs);
  const float* slab_b = db ? slab + (size_t)slab_cap * Cout * K : nullptr;
  hipStream_t st = (hipStream_t)stream;
  const long cols4 = ((long)Cout * K + 3) / 4;
  if (nslabs >= 64)
    hipLaunchKernelGGL(wgrad_reduce_kernel<16>, dim3((unsigned)ceil_div(cols4, 64)), dim3(1024), 0,
                       st, slab, slab_b, dw, db, nslabs, Cout, K, Cin, KH, KW, Cout_log, Cin_log);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<4>, dim3((unsigned)ceil_div(cols4, 64)), dim3(256), 0,
                       st, slab, slab_b, dw, db, nslabs, Cout, K, Cin, KH, KW, Cout_log, Cin_log);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_conv_wgrad_finish_multi(hgk_stream_t stream, const hgk_wgrad_fin* f, int n) {
  HGK_CHECK_ARG(n >= 0 && (n == 0 || f), "conv_wgrad_finish_multi: bad args");
  hipStream_t st = (hipStream_t)stream;
  for (int b = 0; b < n; b += kFinMulti) {
    WgradFinMultiArgs m;
    m.n = std::min(kFinMulti, n - b);
    int blocks = 0;
    for (int i = 0; i < m.n; ++i) {
      const hgk_wgrad_fin& e = f[b + i];
      HGK_CHECK_ARG(e.slabs && e.dw && e.nslabs >= 1 && e.nslabs <= e.slab_cap,
                    "conv_wgrad_finish_multi: entry %d", b + i);
      HGK_CHECK_ARG(e.Cin_log <= e.Cin && e.Cout_log <= e.Cout && e.Cin_log > 0 && e.Cout_log > 0,
                    "conv_wgrad_finish_multi: entry %d logical channels", b + i);
      const int K = e.KH * e.KW * e.Cin;
      const float* slab = reinterpret_cast<const float*>(e.slabs);
      WgradFinDesc& d = m.d[i];
      d.slab = slab;
      d.slab_b = e.db ? slab + (size_t)e.slab_cap * e.Cout * K : nullptr;
      d.dw = e.dw; d.db = e.db;
      d.S = e.nslabs; d.Cout = e.Cout; d.K = K; d.Cin = e.Cin; d.KH = e.KH; d.KW = e.KW;
      d.Cout_log = e.Cout_log; d.Cin_log = e.Cin_log;
      d.b0 = blocks;
      blocks += ceil_div(((long)e.Cout * K + 3) / 4, e.nslabs >= 64 ? 64 : 256);
    }
    hipLaunchKernelGGL(wgrad_reduce_multi_kernel, dim3((unsigned)blocks), dim3(1024), 0, st, m);
    HGK_LAUNCH_CHECK();
  }
  return HGK_OK;
}

int hgk_conv_wgrad(hgk_stream_t stream, int dtype, const void* x, const void* dy,
                   const float* pre_scale, const float* pre_shift, int pre_relu, float* dw,
                   float* db, void* workspace, size_t ws_bytes, int N, int H, int W, int Cin,
                   int Cout, int KH, int KW, int stride, int pad, int dil, int Cin_log,
                   int Cout_log) {
  HGK_CHECK_ARG(x && dy && dw && workspace, "conv_wgrad: null");
  const size_t unit = hgk_conv_wgrad_slab_bytes(Cin, Cout, KH, KW, 1);
  const int cap = (int)std::min<size_t>(kMaxWgradSplits, ws_bytes / unit);
  HGK_CHECK_ARG(cap >= 1, "conv_wgrad: workspace too small");
  int S = 0;
  int rc = hgk_conv_wgrad_accum(stream, dtype, x, dy, pre_scale, pre_shift, pre_relu, workspace,
                                cap, 0, db != nullptr, &S, N, H, W, Cin, Cout, KH, KW, stride, pad,
                                dil);
  if (rc) return rc;
  return hgk_conv_wgrad_finish(stream, workspace, cap, S, dw, db, Cin, Cout, KH, KW, Cin_log,
                               Cout_log);
}

}  // extern "C"
