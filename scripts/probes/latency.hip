// Diagnostic microbenchmark: dispatch cost of many one-wave workgroups and the cost of
// dependent global-load rounds (pointer chase through an L2/MALL-resident table).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__global__ void k_empty(int* out) { if (threadIdx.x == 1000) out[0] = 1; }

__global__ void k_chase(const int* __restrict__ next, int rounds, int n, int* out) {
  int i = (blockIdx.x * 64 + threadIdx.x) % n;
  for (int r = 0; r < rounds; ++r) i = next[i];
  if (i == -1) out[0] = i;
}

int main() {
  const int n = 1 << 22;  // 16 MB table
  std::vector<int> h(n);
  uint64_t s = 1;
  for (int i = 0; i < n; ++i) { s = s * 6364136223846793005ULL + 1442695040888963407ULL; h[i] = (int)((s >> 33) % n); }
  int *d, *out;
  hipMalloc(&d, n * 4); hipMalloc(&out, 4);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int blocks : {1024, 4096, 11607, 35192}) {
    for (int rounds : {0, 1, 4, 10}) {
      float best = 1e9;
      for (int it = 0; it < 5; ++it) {
        hipEventRecord(a);
        if (rounds == 0) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(64), 0, 0, out);
        else hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(64), 0, 0, d, rounds, n, out);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
      }
      printf("blocks %6d x 64 thr, %2d dependent rounds: %8.1f us\n", blocks, rounds, best * 1e3);
    }
  }
  // 256-thread blocks, same number of waves
  for (int rounds : {1, 4, 10}) {
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_chase, dim3(11607 / 4 + 1), dim3(256), 0, 0, d, rounds, n, out);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    printf("blocks %6d x 256 thr, %2d dependent rounds: %8.1f us\n", 11607 / 4 + 1, rounds, best * 1e3);
  }
  return 0;
}
