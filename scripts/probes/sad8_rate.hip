// Diagnostic: issue rate of v_sad_u8 / v_msad_u8 (four 8-bit |a - b| per dword) next to v_sad_u16 and
// the f32 sub + abs-add chain on MI355X -- the candidate inner op of an 8-bit TransE L1 pre-filter.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define KEEP(x) asm volatile("" : "+v"(x))

__global__ void sem(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_sad_u16(a[i], b[i], c[i]);
}

template <int OPK>
__global__ __launch_bounds__(256, 4) void rate(uint32_t* out, int iters, uint32_t seed) {
  uint32_t qa[8], xv[8], acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    qa[i] = seed * (threadIdx.x + i);
    xv[i] = seed ^ (threadIdx.x * 7 + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { KEEP(qa[i]); KEEP(xv[i]); }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (OPK == 0) acc[i][j] = __builtin_amdgcn_sad_u16(qa[i], xv[j], acc[i][j]); else if (OPK == 2) acc[i][j] = __builtin_amdgcn_sad_u8(qa[i], xv[j], acc[i][j]); else if (OPK == 3) acc[i][j] = __builtin_amdgcn_msad_u8(qa[i], xv[j], acc[i][j]);
        else acc[i][j] = __float_as_uint(__uint_as_float(acc[i][j]) + fabsf(__uint_as_float(qa[i]) - __uint_as_float(xv[j])));
      }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[i][j];
  if (s == 12345u) out[0] = s;
}

int main() {
  const int n = 8;
  uint32_t ha[n] = {0x00050003u, 0xFFFF0000u, 0x00000000u, 0x12345678u, 0x0001FFFFu, 0x80008000u, 7u, 0x00070000u};
  uint32_t hb[n] = {0x00020009u, 0x0000FFFFu, 0xFFFFFFFFu, 0x87654321u, 0xFFFF0001u, 0x7FFF8001u, 9u, 0x00090000u};
  uint32_t hc[n] = {10u, 0u, 1u, 0u, 5u, 0u, 0u, 100u};
  uint32_t *a, *b, *c, *o;
  hipMalloc(&a, 4 * n); hipMalloc(&b, 4 * n); hipMalloc(&c, 4 * n); hipMalloc(&o, 4 * n);
  hipMemcpy(a, ha, 4 * n, hipMemcpyHostToDevice); hipMemcpy(b, hb, 4 * n, hipMemcpyHostToDevice);
  hipMemcpy(c, hc, 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, a, b, c, o, n);
  uint32_t ho[n];
  hipMemcpy(ho, o, 4 * n, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const int lo = (int)(ha[i] & 0xFFFF) - (int)(hb[i] & 0xFFFF), hi = (int)(ha[i] >> 16) - (int)(hb[i] >> 16);
    const uint32_t both = (uint32_t)(abs(lo) + abs(hi)) + hc[i], low_only = (uint32_t)abs(lo) + hc[i];
    printf("a %08x b %08x c %u -> %u  (both halves %u, low half only %u)\n", ha[i], hb[i], hc[i], ho[i], both, low_only);
    bad += ho[i] != both;
  }
  printf("semantics: %s\n", bad ? "NOT the sum of both halves" : "sum of |a - b| over both 16-bit halves + c");
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4096, blocks = 256 * 4;
  for (int v = 0; v < 4; ++v) {
    float best = 1e9f;
    for (int r = 0; r < 4; ++r) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(rate<0>, dim3(blocks), dim3(256), 0, 0, o, iters, 3u);
      else if (v == 1) hipLaunchKernelGGL(rate<1>, dim3(blocks), dim3(256), 0, 0, o, iters, 3u); else if (v == 2) hipLaunchKernelGGL(rate<2>, dim3(blocks), dim3(256), 0, 0, o, iters, 3u); else hipLaunchKernelGGL(rate<3>, dim3(blocks), dim3(256), 0, 0, o, iters, 3u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    const double wave_instr = 4.0 * iters * 64 * (v == 0 ? 1 : 2);  // per SIMD (4 waves / SIMD)
    printf("%s: %.3f ms, %.2f SIMD-cycles per wave-instruction at 2.4 GHz\n", v == 0 ? "v_sad_u16 chains" : v == 2 ? "v_sad_u8" : v == 3 ? "v_msad_u8" :
           "f32 sub + abs-add chains", best, best * 1e-3 * 2.4e9 / wave_instr);
  }
  return bad ? 1 : 0;
}
