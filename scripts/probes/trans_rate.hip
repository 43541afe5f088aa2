// Diagnostic: issue rate of f32 VALU ops vs the transcendental v_rsq_f32 on MI355X, with
// 8 independent chains per thread and 4 waves per SIMD (1024-thread blocks x 2 per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NRSQ>
__global__ __launch_bounds__(256) void k(float* out, int iters, float a) {
  float x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (c < NRSQ) x[c] = __builtin_amdgcn_rsqf(x[c]) + a;  // 1 trans + 1 add
      else x[c] = x[c] * a + a;                            // 2 ops (mul, add; no contraction)
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  if (s == 12345.0f) out[0] = s;
}

int main() {
  float* out; hipMalloc(&out, 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4096, blocks = 256 * 16;  // 16 x 256-thread blocks per CU = 16 waves / SIMD
  auto run = [&](auto kern, const char* name, int nrsq) {
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    const double wave_instr = (double)blocks * 4 * iters * (nrsq * 2 + (8 - nrsq) * 2);  // wave-level instrs
    printf("%-10s %8.3f ms  %.3f ns per wave-instr per SIMD\n", name, best, best * 1e6 / (wave_instr / 1024));
  };
  run(k<0>, "0 rsq/8", 0);
  run(k<1>, "1 rsq/8", 1);
  run(k<2>, "2 rsq/8", 2);
  run(k<4>, "4 rsq/8", 4);
  run(k<8>, "8 rsq/8", 8);
  return 0;
}
