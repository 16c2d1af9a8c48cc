// The two components either side of the training hot path:
//   * Gaussian heatmap targets  (try_with_torch.py:104-130, the dataset's __getitem__)
//   * PCKh evaluation           (train.py:759-791, class PCKh)
// Both are tiny next to the step but run per batch; on the GPU they keep the input pipeline and
// the evaluator off the host. Integer / index work is bit-exact with the reference (tests pin
// them against vectors produced by executing the reference's code).
#include <math.h>

#include "hgk_common.h"

namespace hgk {

// one workgroup per (image, joint) map; only the LAST annotation of an image counts (the
// reference re-creates Gauss_map inside its per-annotation loop, :113)
__global__ __launch_bounds__(256) void gauss_targets_kernel(const float* __restrict__ kps,
                                                            const int* __restrict__ counts,
                                                            const float* __restrict__ wh, int P,
                                                            int K, int Hm, int Wm, double inv2s2,
                                                            float* __restrict__ out) {
  const int b = blockIdx.x / K, k = blockIdx.x - b * K;
  const int cnt = counts[b];
  float* o = out + (long)blockIdx.x * Hm * Wm;
  bool on = false;
  long x = 0, y = 0;
  if (cnt > 0) {
    const float* kp = kps + (((long)b * P + (cnt - 1)) * K + k) * 3;
    on = kp[2] > 0.f;
    // (kp / w * 64).astype(int): float64 arithmetic, truncation toward zero (:110-111)
    x = (long)((double)kp[0] / (double)wh[2 * b] * (double)Wm);
    y = (long)((double)kp[1] / (double)wh[2 * b + 1] * (double)Hm);
  }
  for (int i = threadIdx.x; i < Hm * Wm; i += blockDim.x) {
    const long row = i / Wm, col = i - row * Wm;
    float v = 0.f;
    if (on) {
      const long d2 = (col - x) * (col - x) + (row - y) * (row - y);
      v = (float)exp(-(double)d2 * inv2s2);  // float64 exp, then the float32 tensor (:130)
    }
    o[i] = v;
  }
}

struct PckhThresholds {
  float t[11];
};

// one workgroup per (image, joint): label = first row-major pixel with target == j+1, prediction
// = first row-major maximum of channel j+1; per-threshold hit bits + "labelled" bit 11
__global__ __launch_bounds__(256) void pckh_joint_kernel(const float* __restrict__ x,
                                                         const int* __restrict__ target,
                                                         const double* __restrict__ rect, int C,
                                                         int HW, int W, PckhThresholds th,
                                                         int* __restrict__ preds,
                                                         int* __restrict__ labels,
                                                         int* __restrict__ bits) {
  __shared__ float sv[256];
  __shared__ int si[256], sl[256];
  const int b = blockIdx.x / C, j = blockIdx.x - b * C;
  const int tid = threadIdx.x;
  const int* tg = target + (long)b * HW;
  const bool has_ch = j + 1 < C;  // the reference would raise IndexError for j + 1 == C
  const float* ch = x + ((long)b * C + (has_ch ? j + 1 : 0)) * HW;
  float best = -INFINITY;
  int bi = HW, li = HW;
  for (int i = tid; i < HW; i += 256) {  // increasing i: the first hit / strict > keeps the first
    const float v = ch[i];
    if (v > best || bi == HW) { best = v; bi = i; }
    if (li == HW && tg[i] == j + 1) li = i;
  }
  sv[tid] = best; si[tid] = bi; sl[tid] = li;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      const float ov = sv[tid + s];
      const int oi = si[tid + s];
      if (ov > sv[tid] || (ov == sv[tid] && oi < si[tid])) { sv[tid] = ov; si[tid] = oi; }
      sl[tid] = min(sl[tid], sl[tid + s]);
    }
    __syncthreads();
  }
  if (tid != 0) return;
  const long o = ((long)b * C + j) * 2;
  int out_bits = 0;
  if (sl[0] < HW && has_ch) {
    const int ly = sl[0] / W, lx = sl[0] - ly * W;
    const int py = si[0] / W, px = si[0] - py * W;
    const double* r = rect + 4 * b;
    const float standard =
        (float)(sqrt((r[0] - r[2]) * (r[0] - r[2]) + (r[1] - r[3]) * (r[1] - r[3])) * 0.6);
    const int d2 = (ly - py) * (ly - py) + (lx - px) * (lx - px);
    const float dist = (float)sqrt((double)d2) / standard;  // float32 tensor / float32 scalar
    out_bits = 1 << 11;
    for (int s = 0; s < 11; ++s)
      if (dist < th.t[s]) out_bits |= 1 << s;
    preds[o] = px; preds[o + 1] = py;
    labels[o] = lx; labels[o + 1] = ly;
  } else {
    preds[o] = 0; preds[o + 1] = 0;
    labels[o] = 0; labels[o + 1] = 0;
  }
  bits[(long)b * C + j] = out_bits;
}

__global__ void pckh_acc_kernel(const int* __restrict__ bits, int B, int C, double* __restrict__ acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * 11) return;
  const int b = i / 11, s = i - b * 11;
  double correct = 0.0, total = 0.0;
  for (int j = 0; j < C; ++j) {
    const int v = bits[(long)b * C + j];
    if (v & (1 << 11)) {
      total += 1.0;
      if (v & (1 << s)) correct += 1.0;
    }
  }
  acc[i] = correct / total;  // nan when no joint is labelled, as the reference
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_gauss_targets(hgk_stream_t stream, const float* kps, const int* counts, const float* wh,
                      int B, int P, int K, int Hm, int Wm, float sigma, float* out) {
  HGK_CHECK_ARG(kps && counts && wh && out && B > 0 && P > 0 && K > 0 && Hm > 0 && Wm > 0 &&
                    sigma > 0.f,
                "gauss_targets: bad args");
  hipLaunchKernelGGL(gauss_targets_kernel, dim3(B * K), dim3(256), 0, (hipStream_t)stream, kps,
                     counts, wh, P, K, Hm, Wm, 1.0 / (2.0 * (double)sigma * (double)sigma), out);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_pckh(hgk_stream_t stream, const float* x, const int* target, const double* rect, int B,
             int C, int H, int W, int* preds, int* labels, int* scratch, double* acc) {
  HGK_CHECK_ARG(x && target && rect && preds && labels && scratch && acc && B > 0 && C > 1 &&
                    H > 0 && W > 0,
                "pckh: bad args");
  PckhThresholds th;
  for (int s = 0; s < 11; ++s) th.t[s] = (float)(0.0 + s * 0.05);  // np.arange(0, 0.55, 0.05)
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(pckh_joint_kernel, dim3(B * C), dim3(256), 0, st, x, target, rect, C, H * W,
                     W, th, preds, labels, scratch);
  HGK_LAUNCH_CHECK();
  hipLaunchKernelGGL(pckh_acc_kernel, dim3(ceil_div(B * 11, 256)), dim3(256), 0, st, scratch, B, C,
                     acc);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

}  // extern "C"
