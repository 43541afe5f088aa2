// Diagnostic: dependent-load latency with one active lane per wave, and coalesced
// (wave-contiguous) dependent rounds, over many one-wave workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__global__ void k_chase1(const int* __restrict__ next, int rounds, int n, int* out) {
  if (threadIdx.x != 0) return;
  int i = (blockIdx.x * 977) % n;
  for (int r = 0; r < rounds; ++r) i = next[i];
  if (i == -1) out[0] = i;
}
__global__ void k_chase_coal(const int* __restrict__ next, int rounds, int n, int* out) {
  int base = (blockIdx.x * 977) % (n - 64);
  int v = 0;
  for (int r = 0; r < rounds; ++r) {
    v = next[base + threadIdx.x];
    base = __shfl(v, 0) % (n - 64);
  }
  if (v == -1) out[0] = v;
}

int main() {
  const int n = 1 << 22;
  std::vector<int> h(n);
  uint64_t s = 1;
  for (int i = 0; i < n; ++i) { s = s * 6364136223846793005ULL + 1442695040888963407ULL; h[i] = (int)((s >> 33) % n); }
  int *d, *out;
  hipMalloc(&d, n * 4); hipMalloc(&out, 4);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int kind = 0; kind < 2; ++kind)
    for (int blocks : {256, 11607, 35192})
      for (int rounds : {1, 10, 40}) {
        float best = 1e9;
        for (int it = 0; it < 5; ++it) {
          hipEventRecord(a);
          if (kind == 0) hipLaunchKernelGGL(k_chase1, dim3(blocks), dim3(64), 0, 0, d, rounds, n, out);
          else hipLaunchKernelGGL(k_chase_coal, dim3(blocks), dim3(64), 0, 0, d, rounds, n, out);
          hipEventRecord(b); hipEventSynchronize(b);
          float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("%s blocks %6d, %2d rounds: %8.1f us\n", kind ? "coalesced" : "one-lane ", blocks, rounds, best * 1e3);
      }
  return 0;
}
