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
#include <algorithm>

#include "hgk_common.h"

namespace hgk {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

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
  static constexpr int PAD = 8;
};

struct ConvFwdArgs {
  const void* x;
  const void* w;
  const float* bias;
  const void* res;
  void* y;
  const float* pre_scale;
  const float* pre_shift;
  float* stats;
  int pre_relu, post_relu;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, dil;
  int K, w_ld;
  long M;
};

// --------------------------------------------------------------------------------------------
// forward conv
// --------------------------------------------------------------------------------------------
template <typename T, int BM, int BN, int WM, int WN, bool GENERIC>
__global__ __launch_bounds__(64 * WM * WN) void conv_fwd_kernel(ConvFwdArgs a) {
  constexpr int NT = 64 * WM * WN;
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

  __shared__ __attribute__((aligned(16))) T As[BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LDK];

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int HoWo = a.Ho * a.Wo;
  const bool has_pre = a.pre_scale != nullptr;

  // per-thread row geometry (fixed over the k loop)
  const int cv = tid % CPR;
  const int r0 = tid / CPR;
  int rb_h[A_PASSES], rb_w[A_PASSES];
  long rb_pix[A_PASSES];
  if constexpr (!GENERIC) {
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      long m = m0 + r0 + i * RPP;
      if (m < a.M) {
        int n = (int)(m / HoWo);
        int rem = (int)(m - (long)n * HoWo);
        int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
        rb_h[i] = ho * a.stride - a.pad;
        rb_w[i] = wo * a.stride - a.pad;
        rb_pix[i] = (long)n * a.H * a.W;
      } else {
        rb_h[i] = -(1 << 29);
        rb_w[i] = 0;
        rb_pix[i] = 0;
      }
    }
  }

  typedef typename Vec16<T>::type V;
  V areg[A_PASSES];
  V breg[B_PASSES];
  float ag[GENERIC ? (BM * BK / NT) : 1];
  const int nk = (a.K + BK - 1) / BK;

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK;
    if constexpr (!GENERIC) {
      const int tap = k0 / a.Cin;
      const int c0 = k0 - tap * a.Cin;
      const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) {
        int hi = rb_h[i] + kh * a.dil, wi = rb_w[i] + kw * a.dil;
        if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) {
          areg[i] = load16(x + (rb_pix[i] + (long)hi * a.W + wi) * a.Cin + c0 + cv * VEC);
        } else {
          areg[i] = V{};
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < BM * BK / NT; ++j) {
        int e = tid + j * NT;
        int r = e / BK, kc = e - (e / BK) * BK;
        long m = m0 + r;
        int kidx = k0 + kc;
        float v = 0.f;
        if (m < a.M && kidx < a.K) {
          int tap = kidx / a.Cin, ci = kidx - (kidx / a.Cin) * a.Cin;
          int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
          int n = (int)(m / HoWo);
          int rem = (int)(m - (long)n * HoWo);
          int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
          int hi = ho * a.stride - a.pad + kh * a.dil, wi = wo * a.stride - a.pad + kw * a.dil;
          if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) {
            v = to_f(x[(((long)n * a.H + hi) * a.W + wi) * a.Cin + ci]);
            if (has_pre) {
              v = v * a.pre_scale[ci] + a.pre_shift[ci];
              if (a.pre_relu) v = fmaxf(v, 0.f);
            }
          }
        }
        ag[j] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      int r = r0 + i * RPP;
      if (r < BN) breg[i] = load16(w + (long)(n0 + r) * a.w_ld + k0 + cv * VEC);
    }
  };

  auto store_tiles = [&](int kt) {
    const int k0 = kt * BK;
    if constexpr (!GENERIC) {
      const int tap = k0 / a.Cin;
      const int c0 = k0 - tap * a.Cin;
      const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) {
        int r = r0 + i * RPP;
        int hi = rb_h[i] + kh * a.dil, wi = rb_w[i] + kw * a.dil;
        bool valid = hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
        if (has_pre && valid) {
          float f[VEC];
          unpack16<T>(areg[i], f);
          const int cb = c0 + cv * VEC;
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            float v = f[e] * a.pre_scale[cb + e] + a.pre_shift[cb + e];
            f[e] = a.pre_relu ? fmaxf(v, 0.f) : v;
          }
          store16(&As[r * LDK + cv * VEC], pack16<T>(f));
        } else {
          store16(&As[r * LDK + cv * VEC], areg[i]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < BM * BK / NT; ++j) {
        int e = tid + j * NT;
        int r = e / BK, kc = e - (e / BK) * BK;
        As[r * LDK + kc] = from_f<T>(ag[j]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      int r = r0 + i * RPP;
      if (r < BN) store16(&Bs[r * LDK + cv * VEC], breg[i]);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int lr = lane & 15, lg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tiles(kt + 1);
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
    __syncthreads();
    if (kt + 1 < nk) {
      store_tiles(kt + 1);
      __syncthreads();
    }
  }

  // ---- epilogue ----
  T* __restrict__ y = reinterpret_cast<T*>(a.y);
  const T* res = reinterpret_cast<const T*>(a.res);
  // store; keep the stored (rounded) values in acc for the two-pass column statistics
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wn * WTN + j * 16 + lr;
    const bool cok = col < a.Cout;
    const float bb = (cok && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long row = m0 + wm * WTM + i * 16 + lg * 4 + r;
        if (cok && row < a.M) {
          float v = acc[i][j][r] + bb;
          const long off = row * a.Cout + col;
          if (res) v += to_f(res[off]);
          if (a.post_relu) v = fmaxf(v, 0.f);
          T tv = from_f<T>(v);
          y[off] = tv;
          acc[i][j][r] = to_f(tv);
        }
      }
    }
  }
  if (a.stats) {
    // per-column (sum, M2 about the block mean, count) of this M-tile: two passes over the
    // register-resident values, so the variance never suffers E[x^2]-E[x]^2 cancellation
    // (a train-mode BN over as few as 2 values — the 1x1 innermost level — needs that).
    const long nrows = min((long)BM, a.M - m0);
    __syncthreads();  // As / Bs no longer needed
    float* red = reinterpret_cast<float*>(As);   // [WM][BN]
    float* bmean = reinterpret_cast<float*>(Bs);  // [BN]
    auto row_ok = [&](int i, int r) { return m0 + wm * WTM + i * 16 + lg * 4 + r < a.M; };
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row_ok(i, r)) sm += acc[i][j][r];
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      if (lg == 0) red[wm * BN + wn * WTN + j * 16 + lr] = sm;
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < WM; ++i) sm += red[i * BN + c];
      bmean[c] = sm / (float)nrows;
      const int col = n0 + c;
      if (col < a.Cout) {
        a.stats[((long)blockIdx.x * 3 + 0) * a.Cout + col] = sm;
        a.stats[((long)blockIdx.x * 3 + 2) * a.Cout + col] = (float)nrows;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const float mu = bmean[wn * WTN + j * 16 + lr];
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row_ok(i, r)) {
            const float d = acc[i][j][r] - mu;
            q += d * d;
          }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lg == 0) red[wm * BN + wn * WTN + j * 16 + lr] = q;
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < WM; ++i) q += red[i * BN + c];
      const int col = n0 + c;
      if (col < a.Cout) a.stats[((long)blockIdx.x * 3 + 1) * a.Cout + col] = q;
    }
  }
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
};

template <typename T>
struct WgradTraits;
template <>
struct WgradTraits<float> {
  static constexpr int BP = 32;  // pixels per LDS stage
  static constexpr int PAD = 4;
};
template <>
struct WgradTraits<bf16_t> {
  static constexpr int BP = 32;
  static constexpr int PAD = 8;
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

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.dy);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int co0 = blockIdx.x * BMO;
  const int k0 = blockIdx.y * BNO;
  const int split = blockIdx.z;
  const long p_begin = (long)split * a.pix_per_split;
  const long p_end = min(a.M, p_begin + a.pix_per_split);
  const int HoWo = a.Ho * a.Wo;
  const bool has_pre = a.pre_scale != nullptr;
  const bool do_bias = a.slab_b != nullptr && blockIdx.y == 0;

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
          int n = (int)(m / HoWo);
          int rem = (int)(m - (long)n * HoWo);
          int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
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
          int tp = kidx / a.Cin, ci = kidx - (kidx / a.Cin) * a.Cin;
          int kh2 = tp / a.KW, kw2 = tp - (tp / a.KW) * a.KW;
          int n = (int)(m / HoWo);
          int rem = (int)(m - (long)n * HoWo);
          int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
          int hi = ho * a.stride - a.pad + kh2 * a.dil, wi = wo * a.stride - a.pad + kw2 * a.dil;
          if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) {
            v = to_f(x[(((long)n * a.H + hi) * a.W + wi) * a.Cin + ci]);
            if (has_pre) {
              v = v * a.pre_scale[ci] + a.pre_shift[ci];
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
            float v = f[e] * a.pre_scale[cb + e] + a.pre_shift[cb + e];
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
      // column i of rows 8g..8g+3 / 8g+4..8g+7 -> fragment element j <-> pixel 8g+j
      const int q = lr >> 2, p4 = lr & 3;
#pragma unroll
      for (int kk = 0; kk < BP / 32; ++kk) {
        bf16x8 av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const T* base = &Ds[(kk * 32 + 8 * lg + q) * LDD + wm * WTM + i * 16 + 4 * p4];
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + 4 * LDD));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          av[i] = __builtin_bit_cast(bf16x8, c);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const T* base = &Xs[(kk * 32 + 8 * lg + q) * LDX + wn * WTN + j * 16 + 4 * p4];
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + 4 * LDX));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
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
  float* slab = a.slab + (long)split * a.Cout * a.K;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int kc = k0 + wn * WTN + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * WTM + i * 16 + lg * 4 + r;
        if (co < a.Cout && kc < a.K) slab[(long)co * a.K + kc] = acc[i][j][r];
      }
    }
  }
  if (do_bias && tid < BMO && co0 + tid < a.Cout)
    a.slab_b[(long)split * a.Cout + co0 + tid] = bacc;
}

// dw[co][ci][kh][kw] += sum_s slab[s][co][k], k = (kh*KW+kw)*Cin+ci ; db[co] += sum_s slab_b[s][co]
// Fixed summation order over s (deterministic); 4 consecutive k per thread, 4 slabs in flight.
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ slab_b,
                                    float* __restrict__ dw, float* __restrict__ db, int S, int Cout,
                                    int K, int Cin, int KH, int KW) {
  const long total = (long)Cout * K;
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 < total) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const bool vec = (i0 + 4 <= total) && ((total & 3) == 0);
    int s = 0;
    if (vec) {
      for (; s + 4 <= S; s += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(slab + (long)(s + u) * total + i0);
#pragma unroll
        for (int u = 0; u < 4; ++u) { acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w; }
      }
      for (; s < S; ++s) {
        float4 v = *reinterpret_cast<const float4*>(slab + (long)s * total + i0);
        acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
      }
    } else {
      for (; s < S; ++s)
        for (int u = 0; u < 4; ++u)
          if (i0 + u < total) acc[u] += slab[(long)s * total + i0 + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long idx = i0 + u;
      if (idx >= total) break;
      const int co = (int)(idx / K);
      const int k = (int)(idx - (long)co * K);
      const int tap = k / Cin, ci = k - tap * Cin;
      const int kh = tap / KW, kw = tap - kh * KW;
      dw[(((long)co * Cin + ci) * KH + kh) * KW + kw] += acc[u];
    }
  }
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (db && t < Cout) {
    float sb = 0.f;
    for (int i = 0; i < S; ++i) sb += slab_b[(long)i * Cout + t];
    db[t] += sb;
  }
}

// canonical fp32 [Cout][Cin][KH][KW] -> packed [rows_pad][w_ld]
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, T* __restrict__ out, int w_ld,
                                   int rows_pad, int Cout, int Cin, int KH, int KW, int dgrad) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)rows_pad * w_ld) return;
  const int r = (int)(idx / w_ld);
  const int k = (int)(idx - (long)r * w_ld);
  float v = 0.f;
  if (!dgrad) {
    // row = co, k = (kh*KW+kw)*Cin + ci
    if (r < Cout && k < KH * KW * Cin) {
      int tap = k / Cin, ci = k - tap * Cin;
      int kh = tap / KW, kw = tap - kh * KW;
      v = w[(((long)r * Cin + ci) * KH + kh) * KW + kw];
    }
  } else {
    // row = ci, k = (kh'*KW+kw')*Cout + co ; value w[co][ci][KH-1-kh'][KW-1-kw']
    if (r < Cin && k < KH * KW * Cout) {
      int tap = k / Cout, co = k - tap * Cout;
      int kh = tap / KW, kw = tap - kh * KW;
      v = w[(((long)co * Cin + r) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)];
    }
  }
  out[idx] = from_f<T>(v);
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
static constexpr int kMaxStatsRows = 8192;

template <typename T, int BM, int BN, int WM, int WN>
static int launch_fwd(hipStream_t st, ConvFwdArgs& a, bool generic, int* rows_out) {
  dim3 grid((unsigned)ceil_div(a.M, BM), (unsigned)ceil_div(a.Cout, BN));
  if (a.stats && (int)grid.x > kMaxStatsRows) {
    set_error("conv_fwd: %d stats rows exceed the maximum %d", (int)grid.x, kMaxStatsRows);
    return HGK_ERR_UNSUPPORTED;
  }
  if (generic)
    hipLaunchKernelGGL((conv_fwd_kernel<T, BM, BN, WM, WN, true>), grid, dim3(64 * WM * WN), 0, st, a);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<T, BM, BN, WM, WN, false>), grid, dim3(64 * WM * WN), 0, st, a);
  if (rows_out) *rows_out = a.stats ? (int)grid.x : 0;
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

template <typename T>
static int conv_fwd_t(hipStream_t st, ConvFwdArgs& a, int* rows_out) {
  const bool generic = (a.Cin % MfmaTraits<T>::BK) != 0;
  const long tiles128 = (long)ceil_div(a.M, 128) * ceil_div(a.Cout, 128);
  if (a.Cout <= 64) {
    if (a.M >= 128L * 256) return launch_fwd<T, 128, 64, 4, 1>(st, a, generic, rows_out);
    return launch_fwd<T, 64, 64, 2, 2>(st, a, generic, rows_out);
  }
  if (tiles128 >= 256) return launch_fwd<T, 128, 128, 2, 2>(st, a, generic, rows_out);
  return launch_fwd<T, 64, 64, 2, 2>(st, a, generic, rows_out);
}

struct WgradPlan {
  int bmo, bno, S;
  long pix_per_split;
  bool generic;
};

static WgradPlan wgrad_plan(int dtype, long M, int Cin, int Cout, int K) {
  WgradPlan p;
  p.bmo = Cout <= 64 ? 64 : 128;
  p.bno = 64;
  p.generic = (Cin % 64) != 0 || (Cout % 8) != 0;
  const int BP = 32;
  const long tiles = (long)ceil_div(Cout, p.bmo) * ceil_div(K, p.bno);
  const long nsub = (M + BP - 1) / BP;
  long S = std::min<long>(64, (512 + tiles - 1) / tiles);
  // keep >= 4 pixel stages per workgroup
  S = std::min(S, std::max(1L, nsub / 4));
  S = std::max(S, 1L);
  long per = (nsub + S - 1) / S;
  p.pix_per_split = per * BP;
  p.S = (int)((M + p.pix_per_split - 1) / p.pix_per_split);
  (void)dtype;
  return p;
}

template <typename T, int BMO, int BNO, int WM, int WN>
static void launch_wgrad(hipStream_t st, ConvWgradArgs& a, const WgradPlan& p) {
  dim3 grid((unsigned)ceil_div(a.Cout, BMO), (unsigned)ceil_div(a.K, BNO), (unsigned)p.S);
  if (p.generic)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, BMO, BNO, WM, WN, true>), grid, dim3(64 * WM * WN), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<T, BMO, BNO, WM, WN, false>), grid, dim3(64 * WM * WN), 0, st, a);
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_max_stats_rows(void) { return kMaxStatsRows; }

int hgk_conv_w_ld(int K) { return ((K + 63) / 64) * 64; }

int hgk_conv_fwd(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                 const float* bias, const void* res, void* y, const float* pre_scale,
                 const float* pre_shift, int pre_relu, int post_relu, float* stats, int* rows_out,
                 int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                 int dil) {
  HGK_CHECK_ARG(x && w && y, "conv_fwd: null tensor");
  HGK_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 &&
                    dil > 0 && pad >= 0,
                "conv_fwd: bad shape");
  ConvFwdArgs a;
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
  a.M = (long)N * a.Ho * a.Wo;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, return conv_fwd_t<T>(st, a, rows_out));
}

int hgk_pack_conv_weight(hgk_stream_t stream, int dtype, const float* w, void* packed, int w_ld,
                         int Cout, int Cin, int KH, int KW, int for_dgrad) {
  HGK_CHECK_ARG(w && packed, "pack: null");
  const int rows = for_dgrad ? Cin : Cout;
  const int K = KH * KW * (for_dgrad ? Cout : Cin);
  HGK_CHECK_ARG(w_ld >= K && w_ld % 64 == 0, "pack: bad w_ld");
  const int rows_pad = ((rows + 127) / 128) * 128;
  const long total = (long)rows_pad * w_ld;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(pack_weight_kernel<T>, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st,
                       w, reinterpret_cast<T*>(packed), w_ld, rows_pad, Cout, Cin, KH, KW, for_dgrad);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

size_t hgk_conv_wgrad_workspace(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                int stride, int pad, int dil) {
  const int Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  const long M = (long)N * Ho * Wo;
  const int K = KH * KW * Cin;
  WgradPlan p = wgrad_plan(dtype, M, Cin, Cout, K);
  return (size_t)p.S * ((size_t)Cout * K + Cout) * sizeof(float);
}

int hgk_conv_wgrad(hgk_stream_t stream, int dtype, const void* x, const void* dy,
                   const float* pre_scale, const float* pre_shift, int pre_relu, float* dw,
                   float* db, void* workspace, size_t ws_bytes, int N, int H, int W, int Cin,
                   int Cout, int KH, int KW, int stride, int pad, int dil) {
  HGK_CHECK_ARG(x && dy && dw && workspace, "conv_wgrad: null");
  ConvWgradArgs a;
  a.x = x; a.dy = dy; a.pre_scale = pre_scale; a.pre_shift = pre_shift; a.pre_relu = pre_relu;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW;
  a.stride = stride; a.pad = pad; a.dil = dil;
  a.Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  a.Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  a.K = KH * KW * Cin;
  a.M = (long)N * a.Ho * a.Wo;
  WgradPlan p = wgrad_plan(dtype, a.M, Cin, Cout, a.K);
  const size_t need = (size_t)p.S * ((size_t)Cout * a.K + Cout) * sizeof(float);
  HGK_CHECK_ARG(ws_bytes >= need, "conv_wgrad: workspace %zu < %zu", ws_bytes, need);
  a.slab = reinterpret_cast<float*>(workspace);
  a.slab_b = db ? a.slab + (size_t)p.S * Cout * a.K : nullptr;
  a.pix_per_split = p.pix_per_split;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == HGK_F32) {
    if (p.bmo == 64) launch_wgrad<float, 64, 64, 2, 2>(st, a, p);
    else launch_wgrad<float, 128, 64, 2, 2>(st, a, p);
  } else if (dtype == HGK_BF16) {
    if (p.bmo == 64) launch_wgrad<bf16_t, 64, 64, 2, 2>(st, a, p);
    else launch_wgrad<bf16_t, 128, 64, 2, 2>(st, a, p);
  } else {
    set_error("conv_wgrad: dtype");
    return HGK_ERR_ARG;
  }
  HGK_LAUNCH_CHECK();
  const long total = std::max(((long)Cout * a.K + 3) / 4, (long)Cout);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st,
                     a.slab, a.slab_b, dw, db, p.S, Cout, a.K, Cin, KH, KW);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

}  // extern "C"
