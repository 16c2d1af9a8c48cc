// Progressive-head losses of the reference's train.py:
//   Costomer_CrossEntropyLoss          bootstrapped top-k pixel CE      train.py:343-362
//   Costomer_CrossEntropyLoss_with_mask  CE x mask, mean                train.py:365-376
//   Costomer_MSELoss_with_mask         (a-b)^2 x mask, mean             train.py:379-391
//   Costomer_MSELoss                   bootstrapped top-k squared error train.py:394-408
// as three building blocks: per-pixel softmax CE (+ its gradient), per-element squared difference
// (+ gradient), and a deterministic per-row top-k selection (radix select on order-preserving
// float keys; ties at the threshold go to the lowest indices; fixed-order fp64 row sums).
// Module outputs are NCHW fp32 (the engine's output format); targets int64 class maps.
#include <algorithm>

#include "hgk_common.h"

namespace hgk {

static int loss_grid(long n) {
  return (int)std::min<long>(std::max<long>((n + 255) / 256, 1), 256L * 16);
}

static constexpr long kIgnoreIndex = -100;  // nn.CrossEntropyLoss / F.nll_loss default
static constexpr int kCeBlocks = 1024;  // partial rows of hgk_ce_fwd_bwd (<= the MSE finalize's)

// loss[n, p] = (mask[n, p] *) (logsumexp_k x[n, k, p] - x[n, t, p]); one thread per pixel
// (consecutive threads = consecutive pixels: coalesced for every class plane)
__global__ void ce_pixels_kernel(const float* __restrict__ x, const long* __restrict__ t,
                                 const float* __restrict__ mask, int N, int K, long P,
                                 float* __restrict__ loss, int* __restrict__ bad) {
  const long total = (long)N * P;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long n = i / P, p = i - n * P;
    const float* xp = x + n * K * P + p;
    const long tt = t[i];
    if (tt == kIgnoreIndex || tt < 0 || tt >= K) {
      if (tt != kIgnoreIndex) *bad = 1;
      loss[i] = 0.f;
      continue;
    }
    float m = xp[0];
    for (int k = 1; k < K; ++k) m = fmaxf(m, xp[(long)k * P]);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += expf(xp[(long)k * P] - m);
    float v = (m + logf(s)) - xp[tt * P];
    if (mask) v *= mask[i];
    loss[i] = v;
  }
}

// dx[n, k, p] = g * mult * w[n, p] (* mask) * (softmax_k - [k == t]); g = *gscale (device scalar:
// the incoming loss gradient, no host sync)
__global__ void ce_grad_kernel(const float* __restrict__ x, const long* __restrict__ t,
                               const float* __restrict__ w, const float* __restrict__ mask,
                               int N, int K, long P, const float* __restrict__ gscale, float mult,
                               float* __restrict__ dx) {
  const long total = (long)N * P;
  const float g = (gscale ? *gscale : 1.f) * mult;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long n = i / P, p = i - n * P;
    const float* xp = x + n * K * P + p;
    float* dp = dx + n * K * P + p;
    const long tt = t[i];
    float gw = g;
    if (w) gw *= w[i];
    if (mask) gw *= mask[i];
    if (tt < 0 || tt >= K) gw = 0.f;
    float m = xp[0];
    for (int k = 1; k < K; ++k) m = fmaxf(m, xp[(long)k * P]);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += expf(xp[(long)k * P] - m);
    const float inv = 1.f / s;
    for (int k = 0; k < K; ++k) {
      const float sm = expf(xp[(long)k * P] - m) * inv;
      dp[(long)k * P] = gw * (sm - (k == tt ? 1.f : 0.f));
    }
  }
}

// out[n, c, p] = (mask[n, p] *) (a - b)^2  (a, b: [N, C, P])
__global__ void sqdiff_kernel(const float* __restrict__ a, const float* __restrict__ b,
                              const float* __restrict__ mask, int N, int C, long P,
                              float* __restrict__ out) {
  const long total = (long)N * C * P;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const float d = a[i] - b[i];
    float v = d * d;
    if (mask) {
      const long n = i / ((long)C * P);
      v *= mask[n * P + (i % P)];
    }
    out[i] = v;
  }
}

// da[i] = g * mult * 2 (a - b) (* w[i]) (* mask[n, p])
__global__ void sqdiff_grad_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                   const float* __restrict__ w, const float* __restrict__ mask,
                                   int N, int C, long P, const float* __restrict__ gscale,
                                   float mult, float* __restrict__ da) {
  const long total = (long)N * C * P;
  const float g = (gscale ? *gscale : 1.f) * mult * 2.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    float v = g * (a[i] - b[i]);
    if (w) v *= w[i];
    if (mask) {
      const long n = i / ((long)C * P);
      v *= mask[n * P + (i % P)];
    }
    da[i] = v;
  }
}

// Fused nn.CrossEntropyLoss forward + backward of a progressive head for the Trainer
// (try_with_aspp.py:356-358,393-396: CE(out0, background), CE(out1, skeleton)): per pixel
// lse = logsumexp_k x[n, k, p]; loss = lse - x[n, t, p]; dx[n, k, p] = gscale (softmax_k - [k == t]).
// Per-workgroup partial sums of the pixel losses (fixed order: wave sums, then 4 waves) go to
// partial[blockIdx.x] for hgk_mse_finalize (mean = sum / (N P)). A target outside [0, K) sets
// *bad and contributes 0 loss / 0 gradient. That includes ignore_index (-100): the fused head does
// not support ignored pixels (PyTorch would drop them from the mean's count too), so they are
// rejected like any other out-of-range class (Trainer.step raises on the flag).
__global__ __launch_bounds__(256) void ce_fwd_bwd_kernel(const float* __restrict__ x,
                                                         const long* __restrict__ t, int K, long P,
                                                         long total, float* __restrict__ partial,
                                                         float* __restrict__ dx, float gscale,
                                                         int* __restrict__ bad) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long n = i / P, p = i - n * P;
    const float* xp = x + n * K * P + p;
    float* dp = dx + n * K * P + p;
    const long tt = t[i];
    const bool ok = tt >= 0 && tt < K;
    if (!ok) *bad = 1;
    float m = xp[0];
    for (int k = 1; k < K; ++k) m = fmaxf(m, xp[(long)k * P]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(xp[(long)k * P] - m);
    const float inv = 1.f / se;
    const float g = ok ? gscale : 0.f;
    float xt = 0.f;
    for (int k = 0; k < K; ++k) {
      const float xv = xp[(long)k * P];
      if (k == tt) xt = xv;
      dp[(long)k * P] = g * (expf(xv - m) * inv - (k == tt ? 1.f : 0.f));
    }
    if (ok) s += (m + logf(se)) - xt;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// order-preserving key of a float (larger float <-> larger unsigned key)
__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

static constexpr int kTopkNT = 1024;

// one workgroup per row: sel[n, i] = 1 for the k largest values of row n (ties at the k-th value:
// lowest indices first), 0 otherwise; sums[n] = sum of the selected values (per-thread fp64 sums in
// index order, fixed-order tree). Radix select, 4 passes of 8 bits (integer LDS histograms).
__global__ __launch_bounds__(kTopkNT) void topk_select_kernel(const float* __restrict__ v, long L,
                                                              long k, float* __restrict__ sel,
                                                              float* __restrict__ sums) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_bin;
  __shared__ long s_rem;
  __shared__ int scan[kTopkNT];
  __shared__ double dred[kTopkNT];
  const int tid = threadIdx.x;
  const float* row = v + (long)blockIdx.x * L;
  float* srow = sel + (long)blockIdx.x * L;
  unsigned prefix = 0, pmask = 0;
  long rem = k;  // how many of the keys matching `prefix` are still to be taken from the top
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = tid; b < 256; b += kTopkNT) hist[b] = 0;
    __syncthreads();
    for (long i = tid; i < L; i += kTopkNT) {
      const unsigned key = fkey(row[i]);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      long cum = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (cum + (long)hist[b] >= rem) break;
        cum += hist[b];
      }
      s_bin = (unsigned)b;
      s_rem = rem - cum;
    }
    __syncthreads();
    prefix |= s_bin << shift;
    pmask |= 255u << shift;
    rem = s_rem;
    __syncthreads();
  }
  // prefix = the k-th largest key; take every larger key and the first `rem` keys equal to it
  const unsigned T = prefix;
  long taken = 0;
  double acc = 0.0;
  for (long base = 0; base < L; base += kTopkNT) {
    const long i = base + tid;
    const float x = i < L ? row[i] : 0.f;
    const unsigned key = fkey(x);
    const int tie = (i < L && key == T) ? 1 : 0;
    scan[tid] = tie;
    __syncthreads();
    // inclusive Hillis-Steele scan of the tie flags (index order)
    for (int o = 1; o < kTopkNT; o <<= 1) {
      const int add = tid >= o ? scan[tid - o] : 0;
      __syncthreads();
      scan[tid] += add;
      __syncthreads();
    }
    const long rank = taken + scan[tid] - tie;  // ties before this index
    const bool take = i < L && (key > T || (tie && rank < rem));
    if (i < L) srow[i] = take ? 1.f : 0.f;
    if (take) acc += (double)x;
    taken += scan[kTopkNT - 1];
    __syncthreads();
  }
  dred[tid] = acc;
  __syncthreads();
  for (int o = kTopkNT / 2; o > 0; o >>= 1) {
    if (tid < o) dred[tid] += dred[tid + o];
    __syncthreads();
  }
  if (tid == 0) sums[blockIdx.x] = (float)dred[0];
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_ce_pixels(hgk_stream_t stream, const float* logits, const long* target, const float* mask,
                  int N, int K, long P, float* loss, int* bad) {
  HGK_CHECK_ARG(logits && target && loss && bad && N >= 0 && K > 0 && P > 0, "ce_pixels: bad args");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_pixels_kernel, dim3(loss_grid((long)N * P)), dim3(256), 0, st, logits,
                     target, mask, N, K, P, loss, bad);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_ce_grad(hgk_stream_t stream, const float* logits, const long* target, const float* weight,
                const float* mask, int N, int K, long P, const float* gscale, float mult,
                float* dlogits) {
  HGK_CHECK_ARG(logits && target && dlogits && N >= 0 && K > 0 && P > 0, "ce_grad: bad args");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_grad_kernel, dim3(loss_grid((long)N * P)), dim3(256), 0, st, logits, target,
                     weight, mask, N, K, P, gscale, mult, dlogits);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_sqdiff(hgk_stream_t stream, const float* a, const float* b, const float* mask, int N, int C,
               long P, float* out) {
  HGK_CHECK_ARG(a && b && out && N >= 0 && C > 0 && P > 0, "sqdiff: bad args");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sqdiff_kernel, dim3(loss_grid((long)N * C * P)), dim3(256), 0, st, a, b, mask,
                     N, C, P, out);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_sqdiff_grad(hgk_stream_t stream, const float* a, const float* b, const float* weight,
                    const float* mask, int N, int C, long P, const float* gscale, float mult,
                    float* da) {
  HGK_CHECK_ARG(a && b && da && N >= 0 && C > 0 && P > 0, "sqdiff_grad: bad args");
  if (N == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sqdiff_grad_kernel, dim3(loss_grid((long)N * C * P)), dim3(256), 0, st, a, b,
                     weight, mask, N, C, P, gscale, mult, da);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_ce_fwd_bwd(hgk_stream_t stream, const float* logits, const long* target, int N, int K,
                   long P, float* loss_partial, int* rows_out, float* dlogits, float grad_scale,
                   int* bad) {
  HGK_CHECK_ARG(logits && target && loss_partial && dlogits && bad && N > 0 && K > 0 && P > 0,
                "ce_fwd_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  const long total = (long)N * P;
  const int blocks = (int)std::min<long>(kCeBlocks, (total + 255) / 256);
  hipLaunchKernelGGL(ce_fwd_bwd_kernel, dim3(blocks), dim3(256), 0, st, logits, target, K, P,
                     total, loss_partial, dlogits, grad_scale / (float)total, bad);
  if (rows_out) *rows_out = blocks;
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_topk_select(hgk_stream_t stream, const float* values, int rows, long L, long k,
                    float* sel, float* sums) {
  HGK_CHECK_ARG(values && sel && sums && rows >= 0 && L > 0 && k >= 1 && k <= L,
                "topk_select: bad args (k %ld of %ld)", k, L);
  if (rows == 0) return HGK_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(topk_select_kernel, dim3(rows), dim3(kTopkNT), 0, st, values, L, k, sel, sums);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

}  // extern "C"
