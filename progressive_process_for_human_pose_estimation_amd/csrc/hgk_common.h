// Shared device/host helpers for libhgk (stacked-hourglass kernels for gfx950 / MI355X).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/hgk.h"

// occupancy hints (ablation hooks: override with -DHGK_WPE_...= at build time). Weight-grad
// MFMA kernels: 4 waves per SIMD (<= 128 VGPRs, no spills) -> two 8-wave workgroups per CU
// (was 135 VGPRs, one workgroup): step +2.6 %
#ifndef HGK_WPE_WGRAD
#define HGK_WPE_WGRAD __attribute__((amdgpu_waves_per_eu(4)))
#endif
#ifndef HGK_WPE_BWDAPPLY
#define HGK_WPE_BWDAPPLY
#endif

namespace hgk {

// ---- error reporting across the C-ABI (thread-local message, negative return codes) ----
void set_error(const char* fmt, ...);
// current value of a routing knob (HGK_ROUTE_*, include/hgk.h; hgk_util.cpp)
long route(int knob);

#define HGK_CHECK_ARG(cond, ...)                \
  do {                                          \
    if (!(cond)) {                              \
      ::hgk::set_error(__VA_ARGS__);            \
      return HGK_ERR_ARG;                       \
    }                                           \
  } while (0)

#define HGK_LAUNCH_CHECK()                                                   \
  do {                                                                       \
    hipError_t e__ = hipGetLastError();                                      \
    if (e__ != hipSuccess) {                                                 \
      ::hgk::set_error("HIP launch error %s at %s:%d", hipGetErrorString(e__), \
                       __FILE__, __LINE__);                                  \
      return HGK_ERR_HIP;                                                    \
    }                                                                        \
  } while (0)

// ---- storage types: fp32, or bf16 kept as raw uint16 bits ----
struct bf16_t {
  uint16_t v;
};

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16_t x) { return __uint_as_float(((uint32_t)x.v) << 16); }

template <typename T>
__device__ __forceinline__ T from_f(float x);
template <>
__device__ __forceinline__ float from_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ bf16_t from_f<bf16_t>(float x) {
  // hardware round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950; keeps NaN a NaN)
  bf16_t r;
  r.v = __builtin_bit_cast(uint16_t, (__bf16)x);
  return r;
}

// 16-byte vector of T: 4 floats or 8 bf16
template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
  static constexpr int N = 4;
  typedef float4 type;
};
template <>
struct Vec16<bf16_t> {
  static constexpr int N = 8;
  typedef uint4 type;
};

template <typename T>
__device__ __forceinline__ void unpack16(const typename Vec16<T>::type& v, float* f);
template <>
__device__ __forceinline__ void unpack16<float>(const float4& v, float* f) {
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
template <>
__device__ __forceinline__ void unpack16<bf16_t>(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

template <typename T>
__device__ __forceinline__ typename Vec16<T>::type pack16(const float* f);
template <>
__device__ __forceinline__ float4 pack16<float>(const float* f) {
  return make_float4(f[0], f[1], f[2], f[3]);
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
template <>
__device__ __forceinline__ uint4 pack16<bf16_t>(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bf16x2_t h = {(__bf16)f[2 * i], (__bf16)f[2 * i + 1]};  // one v_cvt_pk_bf16_f32
    w[i] = __builtin_bit_cast(uint32_t, h);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <typename T>
__device__ __forceinline__ typename Vec16<T>::type load16(const T* p) {
  return *reinterpret_cast<const typename Vec16<T>::type*>(p);
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const typename Vec16<T>::type& v) {
  *reinterpret_cast<typename Vec16<T>::type*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Slot of producer workgroup `m` of `n` in a channel-major statistics partial array ([C][3][n]):
// a bijection on [0, n) that makes the slots of one XCD (m & 7, the round-robin dispatch) one
// contiguous run. Row-indexed slots put every 64-B line of a channel's partials on 8 XCDs, each
// L2 writing it back partially: the 1x1 conv at 64x64 wrote 1.47x its output bytes (PMC).
__device__ __forceinline__ long xcd_slot(long m, long n) {
  const long x = m & 7, q = n >> 3, r = n & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (m >> 3);
}

// BatchNorm(+ReLU) backward apply of one element: g = dA * [relu: y*scale + shift > 0],
// dy = k0*g + k1*(y - mu) + k2 (hgk_bn_bwd_finalize's coefficients). Explicit fmaf: the apply
// kernels and the convolutions that fold the apply into their operand staging
// (hgk_conv_fwd_bnbwd_vg) round identically, so both paths give the same bits.
__device__ __forceinline__ float bnb_apply(float dA, float y, float sc, float sh, float k0,
                                           float k1, float k2, float mu, bool relu) {
  const float g = (relu && !(fmaf(y, sc, sh) > 0.f)) ? 0.f : dA;
  return fmaf(k0, g, fmaf(k1, y - mu, k2));
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Division by a runtime-invariant divisor with a multiply-high (n < 2^31), as PyTorch's
// IntDivider: the hot gather loops divide pixel indices by Wo, Ho*Wo, Cin, KW every element.
struct FastDiv {
  uint32_t d, mul, shr;
  FastDiv() : d(1), mul(0), shr(0) {}
  explicit FastDiv(uint32_t dv) : d(dv) {
    for (shr = 0; shr < 32; ++shr)
      if ((1u << shr) >= d) break;
    const uint64_t one = 1;
    const uint64_t magic = ((one << 32) * ((one << shr) - d)) / d + 1;
    mul = (uint32_t)magic;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t t = __umulhi(n, mul);
    return (t + n) >> shr;
  }
};

}  // namespace hgk

#define HGK_DISPATCH_DTYPE(dt, T, ...)                         \
  do {                                                         \
    if ((dt) == HGK_F32) {                                     \
      typedef float T;                                         \
      __VA_ARGS__;                                             \
    } else if ((dt) == HGK_BF16) {                             \
      typedef ::hgk::bf16_t T;                                 \
      __VA_ARGS__;                                             \
    } else {                                                   \
      ::hgk::set_error("unsupported dtype %d", (int)(dt));    \
      return HGK_ERR_ARG;                                      \
    }                                                          \
  } while (0)
