// Diagnostic: what RotatE's sweep inner loop costs per element on MI355X with operands in
// registers (no LDS, no barriers), against variants that remove one piece at a time. The
// sweep itself (k_sweep_valu<2>) runs at 44.8 SIMD-cycles per 64 elements (C4, 73.5 ms); this
// says how much of that the arithmetic alone takes at the same occupancy (3 waves / SIMD).
//   V0 the sweep's sequence: dr, di, v = fma(di, di, dr*dr), y = rsq(v), s = v*y, h = y/2,
//      e = fma(-s, s, v), acc += fma(e, h, s), min3 of v's bits per two elements
//   V1 V0 without the min tracking
//   V2 V0 with rsq replaced by a multiply (the rsq's cost)
//   V3 V0 with the last row's rsq interleaved (no software pipeline: rsq used right away)
//   V4 v_sqrt_f32 instead of rsq + Newton (not exact; rate only)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define KEEP(x) asm volatile("" : "+v"(x))

template <int V>
__device__ __forceinline__ void body(float* out, int iters, float seed);
template <int V>
__global__ __launch_bounds__(256, 3) void k(float* out, int iters, float seed) { body<V>(out, iters, seed); }
template <int V>
__global__ __launch_bounds__(256, 2) void k2(float* out, int iters, float seed) { body<V>(out, iters, seed); }
template <int V>
__device__ __forceinline__ void body(float* out, int iters, float seed) {
  float qa[8], qb[8], xv[8], yv[8], acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    qa[i] = seed + threadIdx.x * 1e-3f + i;
    qb[i] = seed * 0.5f + i * 0.25f;
    xv[i] = seed * 0.3f - i;
    yv[i] = seed * 0.7f + i * 0.125f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
  }
  uint32_t lo = 0xFFFFFFFFu;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { KEEP(qa[i]); KEEP(qb[i]); KEEP(xv[i]); KEEP(yv[i]); }
    float v[8], y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dr = qa[0] - xv[j], di = qb[0] - yv[j];
      v[j] = __builtin_fmaf(di, di, dr * dr);
      y[j] = V == 2 ? v[j] * 0.75f : (V == 4 || V == 7) ? __builtin_amdgcn_sqrtf(v[j]) : __builtin_amdgcn_rsqf(v[j]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float vn[8], yn[8];
      if (i + 1 < 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dr = qa[i + 1] - xv[j], di = qb[i + 1] - yv[j];
          vn[j] = __builtin_fmaf(di, di, dr * dr);
          yn[j] = V == 2 ? vn[j] * 0.75f : (V == 4 || V == 7) ? __builtin_amdgcn_sqrtf(vn[j]) : __builtin_amdgcn_rsqf(vn[j]);
        }
      }
      if (V != 3) __builtin_amdgcn_sched_barrier(0);
      if (V >= 5) {  // Newton step in phases across the row's 8 elements: 8 independent chains
        float sv[8], hv[8], ev[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { sv[j] = v[j] * y[j]; hv[j] = 0.5f * y[j]; }
        if (V == 5) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) ev[j] = __builtin_fmaf(-sv[j], sv[j], v[j]);
        if (V == 5) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) sv[j] = __builtin_fmaf(ev[j], hv[j], sv[j]);
        if (V == 5) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          lo = min(min(lo, __float_as_uint(v[j])), __float_as_uint(v[j + 1]));
          acc[i][j] = acc[i][j] + sv[j];
          acc[i][j + 1] = acc[i][j + 1] + sv[j + 1];
        }
      } else
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        if (V != 1) lo = min(min(lo, __float_as_uint(v[j])), __float_as_uint(v[j + 1]));
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float vv = v[j + u], yy = y[j + u];
          float m;
          if (V == 4) {
            m = yy;
          } else {
            const float s = vv * yy, h = 0.5f * yy;
            const float e = __builtin_fmaf(-s, s, vv);
            m = __builtin_fmaf(e, h, s);
          }
          acc[i][j + u] = acc[i][j + u] + m;
        }
      }
      if (i + 1 < 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] = vn[j]; y[j] = yn[j]; }
      }
    }
  }
  float s = (float)lo;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[i][j];
  if (s == 12345.0f) out[0] = s;
}

__global__ __launch_bounds__(256) void kt(float* out, int iters, float a) {
  float x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = __builtin_amdgcn_rsqf(x[c]) + a;
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  if (s == 12345.0f) out[0] = s;
}

int main() {
  float* out;
  if (hipMalloc(&out, 4) != hipSuccess) return 2;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2048, blocks = 256 * 3;  // 3 x 256-thread workgroups per CU = 3 waves / SIMD
  auto run = [&](auto kern, const char* name) {
    float best = 1e9f;
    for (int r = 0; r < 4; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0.37f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    // elements per SIMD: waves per SIMD (3) x iters x 64 pairs; cycles at 2.4 GHz
    const double wave_elems = 3.0 * iters * 64;
    printf("%-28s %8.3f ms  %6.2f SIMD-cycles per wave-element (at 2.4 GHz)\n", name, best,
           best * 1e-3 * 2.4e9 / wave_elems);
  };
  run(k<0>, "V0 sweep sequence");
  run(k<1>, "V1 no min tracking");
  run(k<2>, "V2 rsq -> mul");
  run(k<3>, "V3 no sched barrier");
  run(k<4>, "V4 v_sqrt_f32 only");
  run(k<5>, "V5 phased Newton (barriers)");
  run(k<6>, "V6 phased Newton (free)");
  run(k2<5>, "V5 at 2 waves/SIMD bound");
  run(k<7>, "V7 V0 with v_sqrt as the trans");
  for (int w = 1; w <= 8; w *= 2) {  // trans throughput vs waves per SIMD: 8 chains of rsq + add
    float best = 1e9f;
    for (int r = 0; r < 4; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kt, dim3(256 * w), dim3(256), 0, 0, out, iters * 8, 0.999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("rsq+add chains, %d waves/SIMD: %.2f SIMD-cycles per rsq+add pair\n", w,
           best * 1e-3 * 2.4e9 / ((double)w * iters * 8 * 8));
  }
  return 0;
}
