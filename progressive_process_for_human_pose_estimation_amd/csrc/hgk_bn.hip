// Train-mode BatchNorm2d (+ fused ReLU) statistics, finalisation and backward, NHWC.
// Reference semantics: torch.nn.BatchNorm2d as used by try_with_torch.py:184,187,190,249 —
// batch mean / biased variance to normalise, unbiased variance into running_var, momentum 0.1,
// eps 1e-5; ReLU(True) after it (:185). All cross-workgroup sums go through per-workgroup
// partial slabs reduced in a fixed order (fp64 in the finalisers).
#include <algorithm>

#include "hgk_common.h"

namespace hgk {

static constexpr int kStatsNT = 256;
static constexpr int kMaxRows = 8192;

struct RowPlan {
  int tpr, rpp, G;
  long rows_per_block;
};

template <typename T>
static bool row_plan(long M, int C, RowPlan& p) {
  constexpr int VEC = Vec16<T>::N;
  if (C % VEC != 0) return false;
  p.tpr = C / VEC;
  if (kStatsNT % p.tpr != 0) return false;
  p.rpp = kStatsNT / p.tpr;
  // >= 8 passes per block, <= 2048 blocks
  long per = std::max<long>((long)p.rpp * 8, (M + 2047) / 2048);
  per = ((per + p.rpp - 1) / p.rpp) * p.rpp;
  p.G = (int)((M + per - 1) / per);
  p.rows_per_block = per;
  return true;
}

// Statistics partials, layout [b][3][C]: (sum, M2 about the block mean, count) of block b's rows.
// Each thread accumulates its rows shifted by its first value (well conditioned), the threads of
// a channel are merged with Chan's parallel rule, and bn_finalize merges the blocks the same way
// in fp64: no E[x^2]-E[x]^2 cancellation even for a BN over 2 values (1x1 innermost level, N=2).
template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_stats_kernel(const T* __restrict__ x, long M, int C,
                                                            long rows_per_block, int tpr, int rpp,
                                                            float* __restrict__ partial) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rpp][C][3]
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float k[VEC], s[VEC], q[VEC];
  int n = 0;
#pragma unroll
  for (int e = 0; e < VEC; ++e) { k[e] = 0.f; s[e] = 0.f; q[e] = 0.f; }
  if (r_begin + rp < r_end) unpack16<T>(load16(x + (r_begin + rp) * C + cv * VEC), k);
  for (long r = r_begin + rp; r < r_end; r += rpp) {
    float f[VEC];
    unpack16<T>(load16(x + r * C + cv * VEC), f);
    ++n;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float d = f[e] - k[e];
      s[e] += d;
      q[e] += d * d;
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
  for (int c = tid; c < C; c += kStatsNT) {
    float na = 0.f, ma = 0.f, m2a = 0.f;
    for (int i = 0; i < rpp; ++i) {
      const float* src = &red[((long)i * C + c) * 3];
      const float nb = src[0];
      if (nb == 0.f) continue;
      const float nab = na + nb;
      const float delta = src[1] - ma;
      ma += delta * (nb / nab);
      m2a += src[2] + delta * delta * (na * nb / nab);
      na = nab;
    }
    partial[((long)blockIdx.x * 3 + 0) * C + c] = ma * na;
    partial[((long)blockIdx.x * 3 + 1) * C + c] = m2a;
    partial[((long)blockIdx.x * 3 + 2) * C + c] = na;
  }
}

// Finalisers: one workgroup per 16 channels, 64 row-phases x 16 channels = 1024 threads, fp64
// tree reduction in LDS (the partial rows are read in parallel, not by one thread per channel).
static constexpr int kFinCh = 16, kFinRp = 64, kFinNT = kFinCh * kFinRp;

__device__ __forceinline__ double fin_reduce(double v, double* red, int tx, int ty) {
  red[ty * kFinCh + tx] = v;
  __syncthreads();
  for (int h = kFinRp / 2; h > 0; h >>= 1) {
    if (ty < h) red[ty * kFinCh + tx] += red[(ty + h) * kFinCh + tx];
    __syncthreads();
  }
  const double r = red[tx];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kFinNT) void bn_finalize_kernel(
    const float* __restrict__ partial, int rows, long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* running_mean, float* running_var, float momentum,
    float eps, int training, float* mean, float* invstd, float* scale, float* shift) {
  __shared__ double red[kFinNT];
  const int tx = threadIdx.x % kFinCh, ty = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + tx;
  const bool ok = c < C;
  double mu = 0.0, var = 0.0;
  if (training) {
    double s = 0.0;
    if (ok)
      for (int r = ty; r < rows; r += kFinRp) s += (double)partial[((long)r * 3 + 0) * C + c];
    mu = fin_reduce(s, red, tx, ty) / (double)M;
    double m2 = 0.0;
    if (ok)
      for (int r = ty; r < rows; r += kFinRp) {
        const double nb = partial[((long)r * 3 + 2) * C + c];
        if (nb == 0.0) continue;
        const double d = (double)partial[((long)r * 3 + 0) * C + c] / nb - mu;
        m2 += (double)partial[((long)r * 3 + 1) * C + c] + nb * d * d;
      }
    m2 = fin_reduce(m2, red, tx, ty);
    var = m2 / (double)M;
    if (ty == 0 && ok && running_mean) {
      const double unbiased = M > 1 ? m2 / (double)(M - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mu);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unbiased);
    }
  } else if (ok) {
    mu = running_mean[c];
    var = running_var[c];
  }
  if (ty != 0 || !ok) return;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  const float sc = g * is;
  mean[c] = (float)mu;
  invstd[c] = is;
  scale[c] = sc;
  shift[c] = b - (float)mu * sc;
}

// backward partials: g = dA * [y*scale+shift > 0]; sum g, sum g*xhat
template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_bwd_reduce_kernel(
    const T* __restrict__ dA, const T* __restrict__ y, long M, int C, long rows_per_block, int tpr,
    int rpp, const float* __restrict__ scale, const float* __restrict__ shift, int relu,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ partial) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sc[VEC], sh[VEC], mu[VEC], is[VEC], s[VEC], q[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    sc[e] = scale[c]; sh[e] = shift[c]; mu[e] = mean[c]; is[e] = invstd[c];
    s[e] = 0.f; q[e] = 0.f;
  }
  for (long r = r_begin + rp; r < r_end; r += rpp) {
    float fd[VEC], fy[VEC];
    unpack16<T>(load16(dA + r * C + cv * VEC), fd);
    unpack16<T>(load16(y + r * C + cv * VEC), fy);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float g = fd[e];
      if (relu && !(fy[e] * sc[e] + sh[e] > 0.f)) g = 0.f;
      s[e] += g;
      q[e] += g * ((fy[e] - mu[e]) * is[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    red[((long)rp * C + cv * VEC + e) * 2 + 0] = s[e];
    red[((long)rp * C + cv * VEC + e) * 2 + 1] = q[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += kStatsNT) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < rpp; ++i) {
      a += red[((long)i * C + c) * 2 + 0];
      b += red[((long)i * C + c) * 2 + 1];
    }
    partial[((long)blockIdx.x * 2 + 0) * C + c] = a;
    partial[((long)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

__global__ __launch_bounds__(kFinNT) void bn_bwd_finalize_kernel(
    const float* __restrict__ partial, int rows, long M, int C, const float* __restrict__ scale,
    const float* __restrict__ mean, const float* __restrict__ invstd, int training, float* dgamma,
    float* dbeta, float* coef) {
  __shared__ double red[kFinNT];
  const int tx = threadIdx.x % kFinCh, ty = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + tx;
  const bool ok = c < C;
  double sg = 0.0, sgx = 0.0;
  if (ok)
    for (int r = ty; r < rows; r += kFinRp) {
      sg += (double)partial[((long)r * 2 + 0) * C + c];
      sgx += (double)partial[((long)r * 2 + 1) * C + c];
    }
  sg = fin_reduce(sg, red, tx, ty);
  sgx = fin_reduce(sgx, red, tx, ty);
  if (ty != 0 || !ok) return;
  if (dgamma) dgamma[c] += (float)sgx;
  if (dbeta) dbeta[c] += (float)sg;
  const double sc = scale[c];
  double c1 = 0.0, c2 = 0.0;
  if (training) {
    // dy = scale * (g - mean(g) - xhat * mean(g*xhat)),  xhat = (y - mean) * invstd
    //    = coef0*g + coef1*(y - mean) + coef2   (centred form: no cancellation when y ~ mean)
    c1 = -sc * (double)invstd[c] * sgx / (double)M;
    c2 = -sc * sg / (double)M;
  }
  coef[c] = (float)sc;
  coef[C + c] = (float)c1;
  coef[2 * C + c] = (float)c2;
  coef[3 * C + c] = mean[c];
}

// Apply kernels: the same row plan as the reductions — a thread owns VEC channels for the whole
// launch, so its per-channel constants live in registers; rows are streamed with 16-B accesses.
template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_bwd_apply_kernel(
    const T* __restrict__ dA, const T* __restrict__ y, long M, int C, long rows_per_block, int tpr,
    int rpp, const float* __restrict__ scale, const float* __restrict__ shift, int relu,
    const float* __restrict__ coef, const T* add, T* dy, int accumulate) {
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sc[VEC], sh[VEC], k0[VEC], k1[VEC], k2[VEC], mu[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    sc[e] = scale[c]; sh[e] = shift[c];
    k0[e] = coef[c]; k1[e] = coef[C + c]; k2[e] = coef[2 * C + c]; mu[e] = coef[3 * C + c];
  }
  for (long r = r_begin + rp; r < r_end; r += rpp) {
    const long off = r * C + cv * VEC;
    float fd[VEC], fy[VEC], fa[VEC], fo[VEC], o[VEC];
    unpack16<T>(load16(dA + off), fd);
    unpack16<T>(load16(y + off), fy);
    if (add) unpack16<T>(load16(add + off), fa);
    if (accumulate) unpack16<T>(load16(dy + off), fo);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float g = fd[e];
      if (relu && !(fy[e] * sc[e] + sh[e] > 0.f)) g = 0.f;
      float v = k0[e] * g + k1[e] * (fy[e] - mu[e]) + k2[e];
      if (add) v += fa[e];
      if (accumulate) v += fo[e];
      o[e] = v;
    }
    store16(dy + off, pack16<T>(o));
  }
}

template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_apply_kernel(
    const T* __restrict__ x, long M, int C, long rows_per_block, int tpr, int rpp,
    const float* __restrict__ scale, const float* __restrict__ shift, int relu, T* __restrict__ y) {
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) { sc[e] = scale[cv * VEC + e]; sh[e] = shift[cv * VEC + e]; }
  for (long r = r_begin + rp; r < r_end; r += rpp) {
    const long off = r * C + cv * VEC;
    float f[VEC];
    unpack16<T>(load16(x + off), f);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float v = f[e] * sc[e] + sh[e];
      f[e] = relu ? fmaxf(v, 0.f) : v;
    }
    store16(y + off, pack16<T>(f));
  }
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_bn_stats(hgk_stream_t stream, int dtype, const void* x, long M, int C, float* partial,
                 int* rows_out) {
  HGK_CHECK_ARG(x && partial && M > 0 && C > 0, "bn_stats: bad args");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_stats: unsupported C=%d", C);
    HGK_CHECK_ARG(p.G <= kMaxRows, "bn_stats: too many rows");
    size_t lds = (size_t)p.rpp * C * 3 * sizeof(float);
    hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(p.G), dim3(kStatsNT), lds, st,
                       reinterpret_cast<const T*>(x), M, C, p.rows_per_block, p.tpr, p.rpp,
                       partial);
    if (rows_out) *rows_out = p.G;
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_finalize(hgk_stream_t stream, const float* partial, int rows, long M, int C,
                    const float* gamma, const float* beta, float* running_mean,
                    float* running_var, float momentum, float eps, int training, float* mean,
                    float* invstd, float* scale, float* shift) {
  HGK_CHECK_ARG(mean && invstd && scale && shift, "bn_finalize: null outputs");
  HGK_CHECK_ARG(!training || (partial && rows > 0), "bn_finalize: partials missing");
  HGK_CHECK_ARG(training || (running_mean && running_var), "bn_finalize: eval needs running stats");
  HGK_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr), "bn_finalize: running pair");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(C, kFinCh)), dim3(kFinNT), 0, st, partial, rows,
                     M, C, gamma, beta, running_mean, running_var, momentum, eps, training, mean,
                     invstd, scale, shift);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_apply(hgk_stream_t stream, int dtype, const void* x, long M, int C, const float* scale,
                 const float* shift, int relu, void* y) {
  HGK_CHECK_ARG(x && y && scale && shift, "bn_apply: null");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_apply: unsupported C=%d", C);
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(p.G), dim3(kStatsNT), 0, st,
                       reinterpret_cast<const T*>(x), M, C, p.rows_per_block, p.tpr, p.rpp, scale,
                       shift, relu, reinterpret_cast<T*>(y));
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_reduce(hgk_stream_t stream, int dtype, const void* dA, const void* y, long M,
                      int C, const float* scale, const float* shift, int relu, const float* mean,
                      const float* invstd, float* partial, int* rows_out) {
  HGK_CHECK_ARG(dA && y && scale && shift && mean && invstd && partial, "bn_bwd_reduce: null");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_bwd_reduce: unsupported C=%d", C);
    HGK_CHECK_ARG(p.G <= kMaxRows, "bn_bwd_reduce: too many rows");
    size_t lds = (size_t)p.rpp * C * 2 * sizeof(float);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(p.G), dim3(kStatsNT), lds, st,
                       reinterpret_cast<const T*>(dA), reinterpret_cast<const T*>(y), M, C,
                       p.rows_per_block, p.tpr, p.rpp, scale, shift, relu, mean, invstd, partial);
    if (rows_out) *rows_out = p.G;
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_finalize(hgk_stream_t stream, const float* partial, int rows, long M, int C,
                        const float* scale, const float* mean, const float* invstd, int training,
                        float* dgamma, float* dbeta, float* coef) {
  HGK_CHECK_ARG(partial && scale && mean && invstd && coef && rows > 0, "bn_bwd_finalize: null");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(C, kFinCh)), dim3(kFinNT), 0, st, partial,
                     rows, M, C, scale, mean, invstd, training, dgamma, dbeta, coef);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_apply(hgk_stream_t stream, int dtype, const void* dA, const void* y, long M, int C,
                     const float* scale, const float* shift, int relu, const float* coef,
                     const void* add, void* dy, int accumulate) {
  HGK_CHECK_ARG(dA && y && scale && shift && coef && dy, "bn_bwd_apply: null");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_bwd_apply: unsupported C=%d", C);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(p.G), dim3(kStatsNT), 0, st,
                       reinterpret_cast<const T*>(dA), reinterpret_cast<const T*>(y), M, C,
                       p.rows_per_block, p.tpr, p.rpp, scale, shift, relu, coef,
                       reinterpret_cast<const T*>(add), reinterpret_cast<T*>(dy), accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

}  // extern "C"
