// Down/up-sampling, loss, layout glue and the optimizer step (NHWC, 16-byte channel vectors).
//  maxpool2   : nn.MaxPool2d(2)              try_with_torch.py:220,226,265,279
//  upsample2  : F.interpolate(x2, bilinear, align_corners=True) + skip add  :238-239
//               (nearest x2 + add: hourglass_compare.py:532-542, model.py:82-83)
//  mse        : nn.MSELoss() per stack        :305-308,333-341
//  adam       : torch.optim.Adam(lr=1e-5)     :317,344
#include <algorithm>

#include "hgk_common.h"

namespace hgk {

static int ew_grid(long n) {
  long g = (n + 255) / 256;
  return (int)std::min<long>(std::max<long>(g, 1), 256L * 16);
}

// ---------------------------------------------------------------- maxpool 2x2 / stride 2
template <typename T>
__global__ void maxpool2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H,
                                    int W, int C, FastDiv fcv, FastDiv fw, FastDiv fh) {
  constexpr int VEC = Vec16<T>::N;
  const int Ho = H / 2, Wo = W / 2, CV = C / VEC;
  const int total = N * Ho * Wo * CV;  // < 2^31 (host-checked): 32-bit index math
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int p = (int)fcv.div((uint32_t)i), cv = i - p * CV;
    const int q = (int)fw.div((uint32_t)p), wo = p - q * Wo;
    const int n = (int)fh.div((uint32_t)q), ho = q - n * Ho;
    const T* base = x + (((long)n * H + 2 * ho) * W + 2 * wo) * C + cv * VEC;
    float m[VEC], f[VEC];
    unpack16<T>(load16(base), m);
    const long offs[3] = {(long)C, (long)W * C, (long)W * C + C};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      unpack16<T>(load16(base + offs[t]), f);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (f[e] > m[e] || f[e] != f[e]) m[e] = f[e];
    }
    store16(y + (long)i * VEC, pack16<T>(m));
  }
}

// dx for each 2x2 window: dy goes to the first maximum in scan order (0,0),(0,1),(1,0),(1,1)
template <typename T>
__global__ void maxpool2_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                    T* __restrict__ dx, int N, int H, int W, int C,
                                    int accumulate, FastDiv fcv, FastDiv fw, FastDiv fh) {
  constexpr int VEC = Vec16<T>::N;
  const int Ho = H / 2, Wo = W / 2, CV = C / VEC;
  const int total = N * Ho * Wo * CV;  // < 2^31 (host-checked): 32-bit index math
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int p = (int)fcv.div((uint32_t)i), cv = i - p * CV;
    const int q = (int)fw.div((uint32_t)p), wo = p - q * Wo;
    const int n = (int)fh.div((uint32_t)q), ho = q - n * Ho;
    const long b = (((long)n * H + 2 * ho) * W + 2 * wo) * C + cv * VEC;
    const long offs[4] = {0, (long)C, (long)W * C, (long)W * C + C};
    float v[4][VEC], g[VEC];
#pragma unroll
    for (int t = 0; t < 4; ++t) unpack16<T>(load16(x + b + offs[t]), v[t]);
    unpack16<T>(load16(dy + (long)i * VEC), g);
    int arg[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float m = v[0][e];
      int a = 0;
#pragma unroll
      for (int t = 1; t < 4; ++t)
        if (v[t][e] > m || v[t][e] != v[t][e]) { m = v[t][e]; a = t; }
      arg[e] = a;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float o[VEC];
      if (accumulate) unpack16<T>(load16(dx + b + offs[t]), o);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float c = (arg[e] == t) ? g[e] : 0.f;
        o[e] = accumulate ? o[e] + c : c;
      }
      store16(dx + b + offs[t], pack16<T>(o));
    }
  }
}

// ---------------------------------------------------------------- x2 up-sampling
// PyTorch index/weight rule (align_corners=True): scale = (in-1)/(out-1) in fp32,
// src = scale*dst, i0 = floor(src), i1 = i0 + (i0 < in-1), l1 = src - i0, l0 = 1 - l1.
__device__ __forceinline__ void lin_idx(int dst, int in, float scale, int& i0, int& i1, float& l0,
                                        float& l1) {
  float src = scale * (float)dst;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = src - (float)i0;
  l1 = fminf(fmaxf(l1, 0.f), 1.f);
  l0 = 1.f - l1;
}

template <typename T>
__global__ void upsample2_add_kernel(int mode, const T* __restrict__ low, const T* skip, T* out,
                                     int N, int h, int w, int C) {
  constexpr int VEC = Vec16<T>::N;
  const int H = 2 * h, W = 2 * w, CV = C / VEC;
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  const long total = (long)N * H * W * CV;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    long p = i / CV;
    const int ow = (int)(p % W);
    p /= W;
    const int oh = (int)(p % H);
    const int n = (int)(p / H);
    float r[VEC];
    const T* lb = low + (long)n * h * w * C + cv * VEC;
    if (mode == HGK_UP_NEAREST) {
      unpack16<T>(load16(lb + ((long)(oh >> 1) * w + (ow >> 1)) * C), r);
    } else {
      int h0, h1, w0, w1;
      float hl0, hl1, wl0, wl1;
      lin_idx(oh, h, sh, h0, h1, hl0, hl1);
      lin_idx(ow, w, sw, w0, w1, wl0, wl1);
      float a[VEC], b[VEC], c[VEC], d[VEC];
      unpack16<T>(load16(lb + ((long)h0 * w + w0) * C), a);
      unpack16<T>(load16(lb + ((long)h0 * w + w1) * C), b);
      unpack16<T>(load16(lb + ((long)h1 * w + w0) * C), c);
      unpack16<T>(load16(lb + ((long)h1 * w + w1) * C), d);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        r[e] = hl0 * (wl0 * a[e] + wl1 * b[e]) + hl1 * (wl0 * c[e] + wl1 * d[e]);
    }
    if (skip) {
      float s[VEC];
      unpack16<T>(load16(skip + i * VEC), s);
#pragma unroll
      for (int e = 0; e < VEC; ++e) r[e] = s[e] + r[e];
    }
    store16(out + i * VEC, pack16<T>(r));
  }
}

// ---------------------------------------------------------------- producers with BN statistics
// maxpool2 / upsample2(+add) outputs always feed a train-mode BatchNorm (the next residual
// block's bn1): these variants emit that BN's statistics partials as they store, instead of a
// separate hgk_bn_stats pass re-reading the tensor. Row plan as bn_stats: a workgroup owns a range
// of output pixels, thread (cv, rp) owns channel chunk cv of rows rp, rp + rpp, ...; per-thread
// sums shifted by its first stored value, Chan-merged across rp in a fixed order; partials in the
// channel-major layout [C][3][G] (see bn_finalize).
#ifndef HGK_SAMP_U
#define HGK_SAMP_U 2
#endif
static constexpr int kSampNT = 256, kSampU = HGK_SAMP_U;  // output rows per thread in flight

struct SampPlan {
  int tpr, rpp, G;
  long rows_per_block;
};

template <typename T>
static bool samp_plan(long M, int C, SampPlan& p) {
  constexpr int VEC = Vec16<T>::N;
  if (C % VEC != 0) return false;
  p.tpr = C / VEC;
  if (kSampNT % p.tpr != 0) return false;
  p.rpp = kSampNT / p.tpr;
  long per = std::max<long>((long)p.rpp * 4, (M + 2047) / 2048);
  per = ((per + p.rpp - 1) / p.rpp) * p.rpp;
  p.G = (int)((M + per - 1) / per);
  p.rows_per_block = per;
  return true;
}

// one output pixel's VEC channels: OP 0 = 2x2 max of x, OP 1 = x2 up-sample of low (+ skip)
template <typename T, int OP>
__device__ __forceinline__ void samp_value(long r, int cv, int C, const T* __restrict__ src,
                                           const T* skip, int mode, int N, int h, int w,
                                           float sh, float sw, FastDiv fdw, FastDiv fdh, float* v) {
  constexpr int VEC = Vec16<T>::N;
  if constexpr (OP == 0) {
    // src = x [N][h][w][C] (full resolution), output [N][h/2][w/2]
    // fdw / fdh divide by the OUTPUT width / height (32-bit magic division: M < 2^31)
    const int Wo = w / 2, Ho = h / 2;
    const uint32_t p = fdw.div((uint32_t)r);
    const int wo = (int)((uint32_t)r - p * Wo);
    const int n = (int)fdh.div(p);
    const int ho = (int)(p - (uint32_t)n * Ho);
    const T* base = src + (((long)n * h + 2 * ho) * w + 2 * wo) * C + cv * VEC;
    typename Vec16<T>::type q[4];
    q[0] = load16(base);
    q[1] = load16(base + C);
    q[2] = load16(base + (long)w * C);
    q[3] = load16(base + (long)w * C + C);
    float f[VEC];
    unpack16<T>(q[0], v);
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      unpack16<T>(q[t], f);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (f[e] > v[e] || f[e] != f[e]) v[e] = f[e];
    }
  } else {
    // src = low [N][h][w][C], output [N][2h][2w]
    const int H = 2 * h, W = 2 * w;
    const uint32_t p = fdw.div((uint32_t)r);
    const int ow = (int)((uint32_t)r - p * W);
    const int n = (int)fdh.div(p);
    const int oh = (int)(p - (uint32_t)n * H);
    const T* lb = src + (long)n * h * w * C + cv * VEC;
    typename Vec16<T>::type sk;
    if (skip) sk = load16(skip + r * C + cv * VEC);
    if (mode == HGK_UP_NEAREST) {
      unpack16<T>(load16(lb + ((long)(oh >> 1) * w + (ow >> 1)) * C), v);
    } else {
      int h0, h1, w0, w1;
      float hl0, hl1, wl0, wl1;
      lin_idx(oh, h, sh, h0, h1, hl0, hl1);
      lin_idx(ow, w, sw, w0, w1, wl0, wl1);
      const typename Vec16<T>::type qa = load16(lb + ((long)h0 * w + w0) * C);
      const typename Vec16<T>::type qb = load16(lb + ((long)h0 * w + w1) * C);
      const typename Vec16<T>::type qc = load16(lb + ((long)h1 * w + w0) * C);
      const typename Vec16<T>::type qd = load16(lb + ((long)h1 * w + w1) * C);
      float a[VEC], b[VEC], c[VEC], d[VEC];
      unpack16<T>(qa, a);
      unpack16<T>(qb, b);
      unpack16<T>(qc, c);
      unpack16<T>(qd, d);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        v[e] = hl0 * (wl0 * a[e] + wl1 * b[e]) + hl1 * (wl0 * c[e] + wl1 * d[e]);
    }
    if (skip) {
      float f[VEC];
      unpack16<T>(sk, f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[e] = f[e] + v[e];
    }
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kSampNT) void sample_stats_kernel(
    const T* __restrict__ src, const T* skip, T* out, int mode, int N, int h, int w,  // skip may alias out
    long M, int C, long rows_per_block, int tpr, int rpp, FastDiv fdw, FastDiv fdh,
    float* __restrict__ partial) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rpp][C][3]
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  const int H = 2 * h, W = 2 * w;
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  float k[VEC], s[VEC], q[VEC];
  int n = 0;
#pragma unroll
  for (int e = 0; e < VEC; ++e) { k[e] = 0.f; s[e] = 0.f; q[e] = 0.f; }
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kSampU * rpp) {
    float v[kSampU][VEC];
#pragma unroll
    for (int u = 0; u < kSampU; ++u) {
      const long r = min(r0 + u * rpp, r_end - 1);  // clamped: loads of both rows in flight
      samp_value<T, OP>(r, cv, C, src, skip, mode, N, h, w, sh, sw, fdw, fdh, v[u]);
    }
#pragma unroll
    for (int u = 0; u < kSampU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      const typename Vec16<T>::type pv = pack16<T>(v[u]);
      store16(out + r * C + cv * VEC, pv);
      float f[VEC];
      unpack16<T>(pv, f);  // statistics of the STORED values
      if (n == 0) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) k[e] = f[e];
      }
      ++n;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float d = f[e] - k[e];
        s[e] += d;
        q[e] += d * d;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    float* dst = &red[((long)rp * C + cv * VEC + e) * 3];
    const float mean = n ? k[e] + s[e] / (float)n : 0.f;
    dst[0] = (float)n;
    dst[1] = mean;
    dst[2] = n ? fmaxf(q[e] - s[e] * s[e] / (float)n, 0.f) : 0.f;
  }
  __syncthreads();
  const long slot = xcd_slot(blockIdx.x, gridDim.x);
  for (int c = tid; c < C; c += kSampNT) {
    float na = 0.f, ma = 0.f, m2a = 0.f;
    for (int i = 0; i < rpp; ++i) {
      const float* sp = &red[((long)i * C + c) * 3];
      const float nb = sp[0];
      if (nb == 0.f) continue;
      const float nab = na + nb;
      const float delta = sp[1] - ma;
      ma += delta * (nb / nab);
      m2a += sp[2] + delta * delta * (na * nb / nab);
      na = nab;
    }
    partial[((long)c * 3 + 0) * gridDim.x + slot] = ma * na;
    partial[((long)c * 3 + 1) * gridDim.x + slot] = m2a;
    partial[((long)c * 3 + 2) * gridDim.x + slot] = na;
  }
}

template <typename T, int OP>
static int launch_sample_stats(hipStream_t st, const T* src, const T* skip, T* out, int mode,
                               int N, int h, int w, long M, int C, float* partial, int* rows_out) {
  SampPlan p;
  HGK_CHECK_ARG(samp_plan<T>(M, C, p), "sample_stats: unsupported C=%d", C);
  const size_t lds = (size_t)p.rpp * C * 3 * sizeof(float);
  const int Wout = OP == 0 ? w / 2 : 2 * w, Hout = OP == 0 ? h / 2 : 2 * h;
  HGK_CHECK_ARG(M * C < (1L << 31), "sample_stats: tensor too large");
  hipLaunchKernelGGL((sample_stats_kernel<T, OP>), dim3(p.G), dim3(kSampNT), lds, st, src, skip,
                     out, mode, N, h, w, M, C, p.rows_per_block, p.tpr, p.rpp,
                     FastDiv((uint32_t)Wout), FastDiv((uint32_t)Hout), partial);
  HGK_LAUNCH_CHECK();
  if (rows_out) *rows_out = p.G;
  return HGK_OK;
}

// gather-form backward: for each low-res pixel, sum the weighted grads of every output pixel
// whose interpolation touches it (no atomics; deterministic)
__device__ __forceinline__ float lin_w(int dst, int in, float scale, int target) {
  int i0, i1;
  float l0, l1;
  lin_idx(dst, in, scale, i0, i1, l0, l1);
  return (i0 == target ? l0 : 0.f) + (i1 == target ? l1 : 0.f);
}

template <typename T>
__global__ void upsample2_bwd_kernel(int mode, const T* __restrict__ dout, T* dlow, int N, int h,
                                     int w, int C, int accumulate, FastDiv fcv, FastDiv fw,
                                     FastDiv fh) {
  constexpr int VEC = Vec16<T>::N;
  const int H = 2 * h, W = 2 * w, CV = C / VEC;
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  const int total = N * h * w * CV;  // < 2^31 (host-checked): 32-bit index math
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int p = (int)fcv.div((uint32_t)i), cv = i - p * CV;
    const int q = (int)fw.div((uint32_t)p), iw = p - q * w;
    const int n = (int)fh.div((uint32_t)q), ih = q - n * h;
    const T* db = dout + (long)n * H * W * C + cv * VEC;
    float acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
    if (mode == HGK_UP_NEAREST) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float f[VEC];
        unpack16<T>(load16(db + ((long)(2 * ih + (t >> 1)) * W + (2 * iw + (t & 1))) * C), f);
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] += f[e];
      }
    } else {
      // output rows whose source lies in (ih-1, ih+1)
      int oh_lo = 0, oh_hi = H - 1, ow_lo = 0, ow_hi = W - 1;
      if (sh > 0.f) {
        oh_lo = max(0, (int)floorf((float)(ih - 1) / sh) - 1);
        oh_hi = min(H - 1, (int)ceilf((float)(ih + 1) / sh) + 1);
      }
      if (sw > 0.f) {
        ow_lo = max(0, (int)floorf((float)(iw - 1) / sw) - 1);
        ow_hi = min(W - 1, (int)ceilf((float)(iw + 1) / sw) + 1);
      }
      for (int oh = oh_lo; oh <= oh_hi; ++oh) {
        const float wh = lin_w(oh, h, sh, ih);
        if (wh == 0.f) continue;
        for (int ow = ow_lo; ow <= ow_hi; ++ow) {
          const float ww = lin_w(ow, w, sw, iw);
          if (ww == 0.f) continue;
          float f[VEC];
          unpack16<T>(load16(db + ((long)oh * W + ow) * C), f);
          const float wt = wh * ww;
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[e] += wt * f[e];
        }
      }
    }
    if (accumulate) {
      float o[VEC];
      unpack16<T>(load16(dlow + (long)i * VEC), o);
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] += o[e];
    }
    store16(dlow + (long)i * VEC, pack16<T>(acc));
  }
}

// ---------------------------------------------------------------- MSE
static constexpr int kMseBlocks = 1024;
__global__ void mse_kernel(const float* __restrict__ out, const float* __restrict__ tgt, long n,
                           float* __restrict__ partial, float* __restrict__ grad, float gscale) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float d = out[i] - tgt[i];
    s += d * d;
    if (grad) grad[i] = gscale * d;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void mse_finalize_kernel(const float* __restrict__ partial, int rows, long n,
                                    float* loss, int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < rows; i += blockDim.x) s += (double)partial[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)((red[0] + red[1] + red[2] + red[3]) / (double)n);
    loss[0] = accumulate ? loss[0] + v : v;
  }
}

// ---------------------------------------------------------------- per-stack MSE on the NHWC heads
// All nStack heads of one step in ONE launch (round 6). A workgroup takes tiles of 32 consecutive
// pixels of one head: the NCHW fp32 target of the tile's K logical channels is staged in LDS with
// row loads along the pixels, then each thread owns one 16-B (8-channel) chunk of one pixel of the
// head's NHWC output (dtype, Cs stored channels; consecutive lanes = consecutive chunks of a pixel
// row: every head read and gradient write is contiguous), reads the chunk only when it holds
// logical channels (c < K: 3 of the 8 chunks of the 17 heatmaps in a 64-channel store), writes the
// NHWC gradient (pad channels zero) and adds (o - t)^2 to a per-workgroup partial (fixed order:
// wave shuffles, then the 4 waves). The per-element values are the ones nhwc_to_nchw -> mse_kernel
// -> nchw_to_nhwc produced (same fp32 difference and scale, one rounding to dtype); only the loss
// summation order differs. kMseHeadsMax heads per launch.
static constexpr int kMseHeadsMax = 8;
static constexpr int kMseHeadBlocks = 1024;  // workgroups per head (partial rows per head)
static constexpr int kMseTilePx = 32;       // pixels per workgroup tile
static constexpr int kMseMaxK = 64;         // logical channels the LDS target tile holds
struct MseHeadsArgs {
  const void* head[kMseHeadsMax];
  void* grad[kMseHeadsMax];
};

template <typename T>
__global__ __launch_bounds__(256) void mse_heads_kernel(MseHeadsArgs a, const float* __restrict__ tgt,
                                                        int P, int HW, int K, int Cs, float gscale,
                                                        float* __restrict__ partial) {
  __shared__ float red[4];
  __shared__ float tt[kMseMaxK][kMseTilePx];  // the tile's target, [channel][pixel]
  const int hd = blockIdx.y, tid = threadIdx.x;
  const T* __restrict__ hv = reinterpret_cast<const T*>(a.head[hd]);
  T* __restrict__ gv = reinterpret_cast<T*>(a.grad[hd]);
  const int CH = Cs / 8;                    // 8-channel chunks per pixel
  const int tiles = (P + kMseTilePx - 1) / kMseTilePx;
  float s = 0.f;
  for (int tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
    const int p0 = tl * kMseTilePx;
    __syncthreads();  // the previous tile's target reads are done
    for (int j = tid; j < K * kMseTilePx; j += blockDim.x) {
      const int c = j / kMseTilePx, px = j - c * kMseTilePx, p = p0 + px;
      if (p < P) {
        const int n = p / HW, q = p - n * HW;
        tt[c][px] = tgt[((long)n * K + c) * HW + q];
      }
    }
    __syncthreads();
    for (int j = tid; j < kMseTilePx * CH; j += blockDim.x) {
      const int px = j / CH, c0 = (j - px * CH) * 8, p = p0 + px;
      if (p >= P) continue;
      T* gp = gv + (long)p * Cs + c0;
      float g[8];
      if (c0 < K) {
        const T* hp = hv + (long)p * Cs + c0;
        float o[8];
        unpack16<T>(*reinterpret_cast<const typename Vec16<T>::type*>(hp), o);
        if constexpr (sizeof(T) == 4) unpack16<T>(*reinterpret_cast<const typename Vec16<T>::type*>(hp + 4), o + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (c0 + e < K) {
            const float d = o[e] - tt[c0 + e][px];
            s += d * d;
            g[e] = gscale * d;
          } else {
            g[e] = 0.f;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = 0.f;
      }
      store16(gp, pack16<T>(g));
      if constexpr (sizeof(T) == 4) store16(gp + 4, pack16<T>(g + 4));
    }
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) partial[hd * gridDim.x + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// loss[0] = sum over heads, in head order, of (sum of the head's partial rows, fp64) / numel —
// hgk_mse_finalize's arithmetic per head, with its accumulate chain
__global__ void mse_heads_finalize_kernel(const float* __restrict__ partial, int nheads, int rows,
                                          long n, float* loss) {
  __shared__ double red[4];
  float acc = 0.f;
  for (int h = 0; h < nheads; ++h) {
    double s = 0.0;
    for (int i = threadIdx.x; i < rows; i += blockDim.x) s += (double)partial[h * rows + i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    const float v = (float)((red[0] + red[1] + red[2] + red[3]) / (double)n);
    acc = h == 0 ? v : acc + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = acc;
}

// ---------------------------------------------------------------- layout glue
// NCHW fp32 [N][C][H][W] <-> NHWC dtype [N][H][W][Cs], Cs >= C (channel-padded storage; the pad
// channels are written as zeros)
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ src, T* __restrict__ dst, int N,
                                    int C, int H, int W, int Cs) {
  const long total = (long)N * Cs * H * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cs);
    long p = i / Cs;
    const int wv = (int)(p % W);
    p /= W;
    const int hv = (int)(p % H);
    const int n = (int)(p / H);
    dst[i] = from_f<T>(c < C ? src[(((long)n * C + c) * H + hv) * W + wv] : 0.f);
  }
}

// Pixel-per-thread forms (Cs a multiple of the 16-B vector, pixel count < 2^31): a thread reads
// its pixel's C channels from the NCHW planes (consecutive threads = consecutive pixels of a
// plane, so every plane read is coalesced) and writes the pixel's Cs channels with 16-B stores;
// 32-bit index math (the element-wise form spent its time in 64-bit divisions per element)
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc_pix_kernel(const float* __restrict__ src,
                                                               T* __restrict__ dst, int P, int HW,
                                                               FastDiv fd_hw, int C, int Cs) {
  constexpr int VEC = Vec16<T>::N;
  for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < P; pix += gridDim.x * blockDim.x) {
    const int n = (int)fd_hw.div((uint32_t)pix), hw = pix - n * HW;
    const float* sp = src + (long)n * C * HW + hw;
    T* dp = dst + (long)pix * Cs;
    for (int c0 = 0; c0 < Cs; c0 += VEC) {
      float f[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) f[e] = c0 + e < C ? sp[(long)(c0 + e) * HW] : 0.f;
      store16(dp + c0, pack16<T>(f));
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void nhwc_to_nchw_pix_kernel(const T* __restrict__ src,
                                                               float* __restrict__ dst, int P,
                                                               int HW, FastDiv fd_hw, int C, int Cs) {
  constexpr int VEC = Vec16<T>::N;
  for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < P; pix += gridDim.x * blockDim.x) {
    const int n = (int)fd_hw.div((uint32_t)pix), hw = pix - n * HW;
    const T* sp = src + (long)pix * Cs;
    float* dp = dst + (long)n * C * HW + hw;
    for (int c0 = 0; c0 < C; c0 += VEC) {
      float f[VEC];
      unpack16<T>(load16(sp + c0), f);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (c0 + e < C) dp[(long)(c0 + e) * HW] = f[e];
    }
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ src, float* __restrict__ dst, int N,
                                    int C, int H, int W, int Cs) {
  const long total = (long)N * C * H * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int wv = (int)(i % W);
    long p = i / W;
    const int hv = (int)(p % H);
    p /= H;
    const int c = (int)(p % C);
    const int n = (int)(p / C);
    dst[i] = to_f(src[(((long)n * H + hv) * W + wv) * Cs + c]);
  }
}

// y = a (+ b) (+ y): 16-byte chunks (all three loads of a chunk issued before its store), then a
// channel-range copy between NHWC tensors (torch.cat along channels and its backward, used by the
// progressive heads' concat re-injection, try_with_aspp.py:327-334): for every pixel m,
// dst[m][dc0 + c] (+)= src[m][sc0 + c], c < nch. 16-B vectors when every offset allows it.
template <typename T, bool VECTOR>
__global__ void channel_copy_kernel(const T* __restrict__ src, int sC, int sc0, T* dst, int dC,
                                    int dc0, int nch, long M, int accumulate) {
  constexpr int VEC = VECTOR ? Vec16<T>::N : 1;
  const int cv_n = nch / VEC;
  const long total = M * cv_n;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long m = i / cv_n;
    const int c = (int)(i - m * cv_n) * VEC;
    const T* sp = src + m * sC + sc0 + c;
    T* dp = dst + m * dC + dc0 + c;
    if constexpr (VECTOR) {
      float f[VEC];
      unpack16<T>(load16(sp), f);
      if (accumulate) {
        float g[VEC];
        unpack16<T>(load16(dp), g);
#pragma unroll
        for (int e = 0; e < VEC; ++e) f[e] += g[e];
      }
      store16(dp, pack16<T>(f));
    } else {
      float v = to_f(*sp);
      if (accumulate) v += to_f(*dp);
      *dp = from_f<T>(v);
    }
  }
}

// global average pool / 1x1 broadcast (try_more_layer.py's live ASPP image-pool branch):
// y[n, c] = scale * sum_p x[n, p, c] (+ y): one thread per (image, channel), fixed-order sum over
// the positions (deterministic); consecutive threads = consecutive channels (coalesced)
template <typename T>
__global__ void spatial_sum_kernel(const T* __restrict__ x, T* y, int N, int HW, int C,
                                   float scale, int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * C) return;
  const long n = i / C;
  const T* p = x + n * HW * C + (i - n * C);
  float s = 0.f;
  for (int q = 0; q < HW; ++q) s += to_f(p[(long)q * C]);
  s *= scale;
  if (accumulate) s += to_f(y[i]);
  y[i] = from_f<T>(s);
}

// y[n, p, c] = scale * x[n, c] (+ y)
template <typename T>
__global__ void spatial_broadcast_kernel(const T* __restrict__ x, T* y, int N, int HW, int C,
                                         float scale, int accumulate) {
  const long total = (long)N * HW * C, per = (long)HW * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long n = i / per;
    const int c = (int)(i % C);
    float v = scale * to_f(x[n * C + c]);
    if (accumulate) v += to_f(y[i]);
    y[i] = from_f<T>(v);
  }
}

// stride-s zero insertion (the input-gradient of a strided conv as a stride-1 conv):
// z[n, j, l, :] = dy[n, j/s, l/s, :] where s | j, s | l (and inside dy), else 0; 16-B chunks
template <typename T, bool VECTOR>
__global__ void zero_insert_kernel(const T* __restrict__ src, T* __restrict__ dst, int N, int h,
                                   int w, int C, int s, int Hz, int Wz) {
  constexpr int VEC = VECTOR ? Vec16<T>::N : 1;
  const int CV = C / VEC;
  const long total = (long)N * Hz * Wz * CV;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    long p = i / CV;
    const int l = (int)(p % Wz);
    p /= Wz;
    const int j = (int)(p % Hz);
    const int n = (int)(p / Hz);
    const int hj = j / s, wl = l / s;
    const bool hit = j - hj * s == 0 && l - wl * s == 0 && hj < h && wl < w;
    const T* sp = src + (((long)n * h + hj) * w + wl) * C + cv * VEC;
    if constexpr (VECTOR) {
      typedef typename Vec16<T>::type V;
      store16(dst + i * VEC, hit ? load16(sp) : V{});
    } else {
      dst[i] = hit ? *sp : from_f<T>(0.f);
    }
  }
}

// scalar tail
template <typename T>
__global__ void add_kernel(const T* a, const T* b, T* y, long n, int accumulate) {
  constexpr int VEC = Vec16<T>::N;
  typedef typename Vec16<T>::type V;
  const long nv = n / VEC;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const V va = load16(a + i * VEC);
    const V vb = b ? load16(b + i * VEC) : V{};
    const V vy = accumulate ? load16(y + i * VEC) : V{};
    float fa[VEC], fb[VEC], fy[VEC];
    unpack16<T>(va, fa);
    unpack16<T>(vb, fb);
    unpack16<T>(vy, fy);
#pragma unroll
    for (int e = 0; e < VEC; ++e) fa[e] += fb[e] + fy[e];
    store16(y + i * VEC, pack16<T>(fa));
  }
  for (long i = nv * VEC + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = to_f(a[i]);
    if (b) v += to_f(b[i]);
    if (accumulate) v += to_f(y[i]);
    y[i] = from_f<T>(v);
  }
}

// ---------------------------------------------------------------- Adam (torch.optim.Adam, L2 wd)
// state[0] = step (device-resident so a captured hipGraph replays with the right bias
// correction), state[1] = 1 - beta1^step, state[2] = sqrt(1 - beta2^step)
__global__ void adam_prep_kernel(float* state, float b1, float b2) {
  const float step = state[0] + 1.f;
  state[0] = step;
  state[1] = 1.f - powf(b1, step);
  state[2] = sqrtf(1.f - powf(b2, step));
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                            float* __restrict__ m, float* __restrict__ v, long n, float lr,
                            float b1, float b2, float eps, float wd,
                            const float* __restrict__ state) {
  const float bc1 = state[1], bc2s = state[2];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (wd != 0.f) gi += wd * p[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    // torch single-tensor Adam: denom = sqrt(v)/sqrt(bc2) + eps; p -= lr/bc1 * m / denom
    const float denom = sqrtf(vi) / bc2s + eps;
    p[i] -= (lr / bc1) * mi / denom;
  }
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_maxpool2_fwd(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int H, int W,
                     int C) {
  HGK_CHECK_ARG(x && y && H >= 2 && W >= 2, "maxpool2_fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    HGK_CHECK_ARG(C % Vec16<T>::N == 0, "maxpool2_fwd: C=%d", C);
    long total = (long)N * (H / 2) * (W / 2) * (C / Vec16<T>::N);
    HGK_CHECK_ARG(N >= 0 && C >= 0 && total * Vec16<T>::N < (1L << 31), "maxpool2_fwd: too large");
    if (total == 0) return HGK_OK;
    hipLaunchKernelGGL(maxpool2_fwd_kernel<T>, dim3(ew_grid(total)), dim3(256), 0, st,
                       reinterpret_cast<const T*>(x), reinterpret_cast<T*>(y), N, H, W, C,
                       FastDiv(C / Vec16<T>::N), FastDiv(W / 2), FastDiv(H / 2));
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_maxpool2_fwd_stats(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int H,
                           int W, int C, float* partial, int* rows_out) {
  HGK_CHECK_ARG(x && y && partial && H >= 2 && W >= 2, "maxpool2_fwd_stats: bad args");
  hipStream_t st = (hipStream_t)stream;
  int rc = HGK_OK;
  HGK_DISPATCH_DTYPE(dtype, T, {
    rc = launch_sample_stats<T, 0>(st, reinterpret_cast<const T*>(x), nullptr,
                                   reinterpret_cast<T*>(y), 0, N, H, W,
                                   (long)N * (H / 2) * (W / 2), C, partial, rows_out);
  });
  return rc;
}

int hgk_maxpool2_bwd(hgk_stream_t stream, int dtype, const void* x, const void* dy, void* dx,
                     int N, int H, int W, int C, int accumulate) {
  HGK_CHECK_ARG(x && dy && dx, "maxpool2_bwd: null");
  HGK_CHECK_ARG(H % 2 == 0 && W % 2 == 0, "maxpool2_bwd: odd H/W not supported");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    HGK_CHECK_ARG(C % Vec16<T>::N == 0, "maxpool2_bwd: C=%d", C);
    long total = (long)N * (H / 2) * (W / 2) * (C / Vec16<T>::N);
    HGK_CHECK_ARG(N >= 0 && H >= 0 && W >= 0 && C >= 0 && total * Vec16<T>::N < (1L << 31),
                  "maxpool2_bwd: too large");
    if (total == 0) return HGK_OK;
    hipLaunchKernelGGL(maxpool2_bwd_kernel<T>, dim3(ew_grid(total)), dim3(256), 0, st,
                       reinterpret_cast<const T*>(x), reinterpret_cast<const T*>(dy),
                       reinterpret_cast<T*>(dx), N, H, W, C, accumulate,
                       FastDiv(C / Vec16<T>::N), FastDiv(W / 2), FastDiv(H / 2));
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_upsample2_add_fwd(hgk_stream_t stream, int dtype, int mode, const void* low,
                          const void* skip, void* out, int N, int h, int w, int C) {
  HGK_CHECK_ARG(low && out && (mode == HGK_UP_BILINEAR_AC || mode == HGK_UP_NEAREST),
                "upsample2_add_fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    HGK_CHECK_ARG(C % Vec16<T>::N == 0, "upsample2: C=%d", C);
    long total = (long)N * 4 * h * w * (C / Vec16<T>::N);
    hipLaunchKernelGGL(upsample2_add_kernel<T>, dim3(ew_grid(total)), dim3(256), 0, st, mode,
                       reinterpret_cast<const T*>(low), reinterpret_cast<const T*>(skip),
                       reinterpret_cast<T*>(out), N, h, w, C);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_upsample2_add_fwd_stats(hgk_stream_t stream, int dtype, int mode, const void* low,
                                const void* skip, void* out, int N, int h, int w, int C,
                                float* partial, int* rows_out) {
  HGK_CHECK_ARG(low && out && partial && (mode == HGK_UP_BILINEAR_AC || mode == HGK_UP_NEAREST),
                "upsample2_add_fwd_stats: bad args");
  hipStream_t st = (hipStream_t)stream;
  int rc = HGK_OK;
  HGK_DISPATCH_DTYPE(dtype, T, {
    rc = launch_sample_stats<T, 1>(st, reinterpret_cast<const T*>(low),
                                   reinterpret_cast<const T*>(skip), reinterpret_cast<T*>(out),
                                   mode, N, h, w, (long)N * 4 * h * w, C, partial, rows_out);
  });
  return rc;
}

int hgk_upsample2_bwd(hgk_stream_t stream, int dtype, int mode, const void* dout, void* dlow,
                      int N, int h, int w, int C, int accumulate) {
  HGK_CHECK_ARG(dout && dlow && (mode == HGK_UP_BILINEAR_AC || mode == HGK_UP_NEAREST),
                "upsample2_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    HGK_CHECK_ARG(C % Vec16<T>::N == 0, "upsample2_bwd: C=%d", C);
    long total = (long)N * h * w * (C / Vec16<T>::N);
    HGK_CHECK_ARG(N >= 0 && h >= 0 && w >= 0 && C >= 0 && total * Vec16<T>::N < (1L << 31),
                  "upsample2_bwd: too large");
    if (total == 0) return HGK_OK;
    hipLaunchKernelGGL(upsample2_bwd_kernel<T>, dim3(ew_grid(total)), dim3(256), 0, st, mode,
                       reinterpret_cast<const T*>(dout), reinterpret_cast<T*>(dlow), N, h, w, C,
                       accumulate, FastDiv(C / Vec16<T>::N), FastDiv(w), FastDiv(h));
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_mse_fwd_bwd(hgk_stream_t stream, const float* out, const float* target, long numel,
                    float* loss_partial, int* rows_out, float* grad, float grad_scale) {
  HGK_CHECK_ARG(out && target && loss_partial && numel > 0, "mse: bad args");
  hipStream_t st = (hipStream_t)stream;
  int blocks = (int)std::min<long>(kMseBlocks, (numel + 255) / 256);
  hipLaunchKernelGGL(mse_kernel, dim3(blocks), dim3(256), 0, st, out, target, numel, loss_partial,
                     grad, grad_scale * 2.0f / (float)numel);
  if (rows_out) *rows_out = blocks;
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_mse_finalize(hgk_stream_t stream, const float* loss_partial, int rows, long numel,
                     float* loss, int accumulate) {
  HGK_CHECK_ARG(loss_partial && loss && rows > 0, "mse_finalize: bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(mse_finalize_kernel, dim3(1), dim3(256), 0, st, loss_partial, rows, numel,
                     loss, accumulate);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_mse_heads_nhwc(hgk_stream_t stream, int dtype, const void* const* heads, void* const* grads,
                       int nheads, const float* target, int N, int K, int H, int W, int C_store,
                       float grad_scale, float* loss_partial, float* loss) {
  HGK_CHECK_ARG(heads && grads && target && loss_partial && loss && nheads >= 1 &&
                    nheads <= kMseHeadsMax && N > 0 && K > 0 && H > 0 && W > 0 && C_store >= K &&
                    C_store % 8 == 0,
                "mse_heads: bad args");
  const long P = (long)N * H * W;
  HGK_CHECK_ARG(P * C_store < (1L << 31), "mse_heads: tensor too large");
  MseHeadsArgs a;
  for (int h = 0; h < nheads; ++h) {
    HGK_CHECK_ARG(heads[h] && grads[h] && ((uintptr_t)heads[h] % 16) == 0 && ((uintptr_t)grads[h] % 16) == 0,
                  "mse_heads: head %d pointers", h);
    a.head[h] = heads[h];
    a.grad[h] = grads[h];
  }
  hipStream_t st = (hipStream_t)stream;
  const long numel = P * K;
  const float gscale = grad_scale * 2.0f / (float)numel;
  HGK_CHECK_ARG(K <= kMseMaxK, "mse_heads: %d heatmaps > %d", K, kMseMaxK);
  const int blocks = (int)std::min<long>(kMseHeadBlocks, (P + kMseTilePx - 1) / kMseTilePx);
  HGK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(mse_heads_kernel<T>, dim3(blocks, nheads), dim3(256), 0, st, a, target, (int)P,
                       H * W, K, C_store, gscale, loss_partial);
  });
  HGK_LAUNCH_CHECK();
  hipLaunchKernelGGL(mse_heads_finalize_kernel, dim3(1), dim3(256), 0, st, loss_partial, nheads,
                     blocks, numel, loss);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_mse_heads_partial_rows(void) { return kMseHeadsMax * kMseHeadBlocks; }

int hgk_nchw_to_nhwc(hgk_stream_t stream, int dtype, const float* src, void* dst, int N, int C,
                     int H, int W, int C_store) {
  HGK_CHECK_ARG(src && dst && C_store >= C, "nchw_to_nhwc: bad args");
  hipStream_t st = (hipStream_t)stream;
  long total = (long)N * C_store * H * W;
  const long P = (long)N * H * W;
  HGK_DISPATCH_DTYPE(dtype, T, {
    if (C_store % Vec16<T>::N == 0 && P < (1L << 31) && ((uintptr_t)dst % 16) == 0) {
      hipLaunchKernelGGL(nchw_to_nhwc_pix_kernel<T>, dim3(ew_grid(P)), dim3(256), 0, st, src,
                         reinterpret_cast<T*>(dst), (int)P, H * W, FastDiv((uint32_t)(H * W)), C,
                         C_store);
    } else {
      hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(ew_grid(total)), dim3(256), 0, st, src,
                         reinterpret_cast<T*>(dst), N, C, H, W, C_store);
    }
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_nhwc_to_nchw(hgk_stream_t stream, int dtype, const void* src, float* dst, int N, int C,
                     int H, int W, int C_store) {
  HGK_CHECK_ARG(src && dst && C_store >= C, "nhwc_to_nchw: bad args");
  hipStream_t st = (hipStream_t)stream;
  long total = (long)N * C * H * W;
  const long P = (long)N * H * W;
  HGK_DISPATCH_DTYPE(dtype, T, {
    if (C_store % Vec16<T>::N == 0 && P < (1L << 31) && ((uintptr_t)src % 16) == 0) {
      hipLaunchKernelGGL(nhwc_to_nchw_pix_kernel<T>, dim3(ew_grid(P)), dim3(256), 0, st,
                         reinterpret_cast<const T*>(src), dst, (int)P, H * W,
                         FastDiv((uint32_t)(H * W)), C, C_store);
    } else {
      hipLaunchKernelGGL(nhwc_to_nchw_kernel<T>, dim3(ew_grid(total)), dim3(256), 0, st,
                         reinterpret_cast<const T*>(src), dst, N, C, H, W, C_store);
    }
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_channel_copy(hgk_stream_t stream, int dtype, const void* src, int src_C, int src_c0,
                     void* dst, int dst_C, int dst_c0, int nch, long M, int accumulate) {
  HGK_CHECK_ARG(src && dst && M >= 0 && nch >= 0, "channel_copy: null / negative");
  HGK_CHECK_ARG(src_c0 >= 0 && src_c0 + nch <= src_C && dst_c0 >= 0 && dst_c0 + nch <= dst_C,
                "channel_copy: channel range outside the tensors");
  if (M == 0 || nch == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    constexpr int V = Vec16<T>::N;
    const bool vec = (src_C | src_c0 | dst_C | dst_c0 | nch) % V == 0 &&
                     ((uintptr_t)src | (uintptr_t)dst) % 16 == 0;
    const long items = M * (vec ? nch / V : nch);
    if (vec)
      hipLaunchKernelGGL((channel_copy_kernel<T, true>), dim3(ew_grid(items)), dim3(256), 0, st,
                         reinterpret_cast<const T*>(src), src_C, src_c0, reinterpret_cast<T*>(dst),
                         dst_C, dst_c0, nch, M, accumulate);
    else
      hipLaunchKernelGGL((channel_copy_kernel<T, false>), dim3(ew_grid(items)), dim3(256), 0, st,
                         reinterpret_cast<const T*>(src), src_C, src_c0, reinterpret_cast<T*>(dst),
                         dst_C, dst_c0, nch, M, accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_zero_insert(hgk_stream_t stream, int dtype, const void* src, void* dst, int N, int h, int w,
                    int C, int stride, int Hz, int Wz) {
  HGK_CHECK_ARG(src && dst && N >= 0 && h > 0 && w > 0 && C > 0 && stride > 0 && Hz > 0 && Wz > 0,
                "zero_insert: bad args");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    constexpr int V = Vec16<T>::N;
    const bool vec = C % V == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0;
    const long items = (long)N * Hz * Wz * (vec ? C / V : C);
    if (vec)
      hipLaunchKernelGGL((zero_insert_kernel<T, true>), dim3(ew_grid(items)), dim3(256), 0, st,
                         reinterpret_cast<const T*>(src), reinterpret_cast<T*>(dst), N, h, w, C,
                         stride, Hz, Wz);
    else
      hipLaunchKernelGGL((zero_insert_kernel<T, false>), dim3(ew_grid(items)), dim3(256), 0, st,
                         reinterpret_cast<const T*>(src), reinterpret_cast<T*>(dst), N, h, w, C,
                         stride, Hz, Wz);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_spatial_sum(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int HW, int C,
                    float scale, int accumulate) {
  HGK_CHECK_ARG(x && y && N >= 0 && HW > 0 && C > 0, "spatial_sum: null / bad shape");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(spatial_sum_kernel<T>, dim3((unsigned)(((long)N * C + 255) / 256)), dim3(256),
                       0, st, reinterpret_cast<const T*>(x), reinterpret_cast<T*>(y), N, HW, C,
                       scale, accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_spatial_broadcast(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int HW,
                          int C, float scale, int accumulate) {
  HGK_CHECK_ARG(x && y && N >= 0 && HW > 0 && C > 0, "spatial_broadcast: null / bad shape");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(spatial_broadcast_kernel<T>, dim3(ew_grid((long)N * HW * C)), dim3(256), 0,
                       st, reinterpret_cast<const T*>(x), reinterpret_cast<T*>(y), N, HW, C, scale,
                       accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_add(hgk_stream_t stream, int dtype, const void* a, const void* b, void* y, long n,
            int accumulate) {
  HGK_CHECK_ARG(a && y && n >= 0, "add: null");
  if (n == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    HGK_CHECK_ARG(((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) % 16 == 0, "add: tensors not 16-B aligned");
    hipLaunchKernelGGL(add_kernel<T>, dim3(ew_grid((n + Vec16<T>::N - 1) / Vec16<T>::N)), dim3(256), 0, st,
                       reinterpret_cast<const T*>(a), reinterpret_cast<const T*>(b),
                       reinterpret_cast<T*>(y), n, accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_adam_step(hgk_stream_t stream, float* param, const float* grad, float* exp_avg,
                  float* exp_avg_sq, long n, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float* step_state) {
  HGK_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && step_state, "adam: bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, st, step_state, beta1, beta2);
  HGK_LAUNCH_CHECK();
  hipLaunchKernelGGL(adam_kernel, dim3(ew_grid(n)), dim3(256), 0, st, param, grad, exp_avg,
                     exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, step_state);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

}  // extern "C"
