// Grid-barrier price at the small hourglass levels' workgroup counts (round-5 verdict, item 2:
// "commit a grid-barrier microbenchmark at 8/16/32/64 workgroups; the 4.1 us figure was at 256").
//
// One phase = what a fused small-level ResidualBlock would do between two convolutions: every
// workgroup publishes a BN-statistics partial row (2 floats x 256 channels = 2 KB, plain stores),
// a grid barrier (monotonic agent-scope counter: every storing wave drains, lane 0 releases at
// agent scope and adds, polls relaxed with s_sleep, acquires once; bounded spin), then every
// workgroup reads all G partial rows (the merge a consumer needs). Per-phase cost = (time of a
// launch with 17 phases - time with 1 phase) / 16. Placements: "spread" (G workgroups, dealt over
// the 8 XCDs) and "xcd" (8G workgroups launched, only those with blockIdx % 8 == 0 take part: one
// XCD under the observed round-robin dealing — speed only, the protocol does not assume it).
// "launch" = the same phase as its own kernel, P launches back to back (the boundary it replaces),
// from the host stream and replayed as a hipGraph (the engine's mode). Two merges: "serial" (round 5:
// one thread per channel reads the G rows one after another — G dependent round trips, what the
// round-5 verdict flagged: the payload columns then measured that loop, not the barrier) and
// "parallel" (round 6: every thread owns one float4 column chunk of every RG-th row, all its loads
// issued in one burst into registers, then the RG row groups add through LDS in a fixed order —
// one memory round trip per phase whatever G). The payload-0 rows are the barrier itself.
//
// build: hipcc --offload-arch=gfx950 -O3 scripts/grid_barrier_bench.hip -o scripts/bin/grid_barrier_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef __attribute__((address_space(1))) unsigned gu32;

// round 5: thread i sums channel i over the G rows, one load after another
__device__ float merge_serial(const float* all, int G, int nf) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < nf; i += 256) {
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += all[(size_t)g * nf + i];
    acc += s * 1e-6f;
  }
  return acc;
}

// round 6: nf / 4 float4 column chunks x RG = 1024 / nf row groups; thread (rg, c) loads rows rg,
// rg + RG, ... of chunk c, up to 64 loads in flight, then the row groups meet in LDS (fixed order)
__device__ float merge_parallel(const float* all, int G, int nf, float4* red) {
  const int tid = threadIdx.x;
  if (nf == 0) return 0.f;
  const int chunks = nf / 4, RG = 256 / chunks;
  const int c = tid % chunks, rg = tid / chunks;
  const float4* a4 = reinterpret_cast<const float4*>(all);
  constexpr int MAXL = 64;
  float4 v[MAXL];
#pragma unroll
  for (int k = 0; k < MAXL; ++k) {
    const int g = rg + k * RG;
    v[k] = g < G ? a4[(size_t)g * chunks + c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < MAXL; ++k) {
    s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w;
  }
  red[tid] = s;
  __syncthreads();
  float acc = 0.f;
  if (rg == 0) {
    float4 t = red[c];
    for (int r = 1; r < RG; ++r) {
      const float4 u = red[r * chunks + c];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    acc = (t.x + t.y + t.z + t.w) * 1e-6f;
  }
  __syncthreads();
  return acc;
}

__global__ __launch_bounds__(256) void phases_kernel(unsigned* counter, float* payload, float* out,
                                                     unsigned* timeout, int G, int stride, int P,
                                                     int nf, int use_barrier, int par) {
  __shared__ float4 red[256];
  const int bid = blockIdx.x, tid = threadIdx.x;
  if (bid % stride) return;  // not a participant (workgroup-uniform exit before any barrier)
  const int me = bid / stride;
  float acc = 0.f;
  for (int ph = 0; ph < P; ++ph) {
    float* mine = payload + ((size_t)(ph & 1) * G + me) * nf;
    for (int i = tid; i < nf; i += 256) mine[i] = acc + (float)(i + ph + me);
    if (use_barrier) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (unsigned)(ph + 1) * (unsigned)G;
        unsigned spins = 0;
        while (__hip_atomic_load((gu32*)counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1u << 22)) {
            __hip_atomic_store((gu32*)timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      // the merge: every workgroup reads all G partial rows
      const float* all = payload + (size_t)(ph & 1) * G * nf;
      acc += par ? merge_parallel(all, G, nf, red) : merge_serial(all, G, nf);
    }
  }
  out[me * 256 + tid] = acc;
}

// the same phase as its own launch: read the previous launch's rows, publish this one's
__global__ __launch_bounds__(256) void one_phase_kernel(float* payload, float* out, int G, int stride,
                                                        int ph, int nf, int par) {
  __shared__ float4 red[256];
  const int bid = blockIdx.x, tid = threadIdx.x;
  if (bid % stride) return;
  const int me = bid / stride;
  const float* all = payload + (size_t)((ph + 1) & 1) * G * nf;
  float acc = par ? merge_parallel(all, G, nf, red) : merge_serial(all, G, nf);
  float* mine = payload + ((size_t)(ph & 1) * G + me) * nf;
  for (int i = tid; i < nf; i += 256) mine[i] = acc + (float)(i + ph + me);
  out[me * 256 + tid] = acc;
}

int main() {
  unsigned *counter, *timeout;
  float *payload, *out;
  const int GMAX = 256, NF = 512;
  CK(hipMalloc(&counter, 64));
  CK(hipMalloc(&timeout, 64));
  CK(hipMalloc(&payload, sizeof(float) * 2 * GMAX * NF));
  CK(hipMalloc(&out, sizeof(float) * GMAX * 256));
  CK(hipMemset(timeout, 0, 64));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int REPS = 50;
  printf("G,placement,merge,payload_bytes,us_per_launch_P1,us_per_launch_P17,us_per_phase,us_per_boundary_launch,us_per_boundary_launch_graph\n");
  for (int G : {8, 16, 32, 64, 128, 256}) {
    for (int stride : {1, 8}) {
      if (G * stride > 2048) continue;
      for (int nfp : {0, NF, 2 * NF}) {
       const int nf = nfp == 2 * NF ? NF : nfp, par = nfp == 2 * NF;  // (0, serial, parallel)
        float t[2];
        int Ps[2] = {1, 17};
        for (int k = 0; k < 2; ++k) {
          // warm-up
          for (int r = 0; r < 3; ++r) {
            CK(hipMemsetAsync(counter, 0, 64, st));
            hipLaunchKernelGGL(phases_kernel, dim3(G * stride), dim3(256), 0, st, counter, payload, out,
                               timeout, G, stride, Ps[k], nf, 1, par);
          }
          CK(hipEventRecord(e0, st));
          for (int r = 0; r < REPS; ++r) {
            CK(hipMemsetAsync(counter, 0, 64, st));
            hipLaunchKernelGGL(phases_kernel, dim3(G * stride), dim3(256), 0, st, counter, payload, out,
                               timeout, G, stride, Ps[k], nf, 1, par);
          }
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          CK(hipEventElapsedTime(&t[k], e0, e1));
          t[k] = t[k] * 1000.f / REPS;
        }
        // boundary: 16 dependent single-phase launches
        float tb;
        for (int r = 0; r < 3; ++r)
          hipLaunchKernelGGL(one_phase_kernel, dim3(G * stride), dim3(256), 0, st, payload, out, G, stride, r, nf, par);
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < REPS * 16; ++r)
          hipLaunchKernelGGL(one_phase_kernel, dim3(G * stride), dim3(256), 0, st, payload, out, G, stride, r, nf, par);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tb, e0, e1));
        tb = tb * 1000.f / (REPS * 16);
        // the same 16 dependent launches captured in a hipGraph (how the engine replays a step)
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int r = 0; r < 16; ++r)
          hipLaunchKernelGGL(one_phase_kernel, dim3(G * stride), dim3(256), 0, st, payload, out, G, stride, r, nf, par);
        CK(hipStreamEndCapture(st, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < REPS; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float tg;
        CK(hipEventElapsedTime(&tg, e0, e1));
        tg = tg * 1000.f / (REPS * 16);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
        printf("%d,%s,%s,%d,%.2f,%.2f,%.3f,%.3f,%.3f\n", G, stride == 1 ? "spread" : "xcd",
               nf == 0 ? "-" : (par ? "parallel" : "serial"), nf * 4, t[0], t[1],
               (t[1] - t[0]) / 16.f, tb, tg);
        fflush(stdout);
      }
    }
  }
  unsigned to = 0;
  CK(hipMemcpy(&to, timeout, 4, hipMemcpyDeviceToHost));
  printf("timeout_flag,%u\n", to);
  CK(hipDeviceSynchronize());
  return to ? 2 : 0;
}
