// Exhaustive check that RotatE's sweep magnitude keeps its bits when the Newton step's halving
// moves from the rsq estimate (h = y / 2, fma(e, h, s)) to the residual (e / 2 by the VOP3
// output modifier div:2 of the fma that forms it, fma(e / 2, y, s)): one multiply less per
// element. Compares the two sequences with each other and with IEEE sqrtf over every float
// bit pattern below +inf. Diagnostic.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ float mag_h(float v) {  // the sweep's sequence before
  const float y = __builtin_amdgcn_rsqf(v);
  const float s = v * y, h = 0.5f * y;
  const float e = __builtin_fmaf(-s, s, v);
  return __builtin_fmaf(e, h, s);
}
__device__ __forceinline__ float mag_omod(float v) {  // e / 2 from the output modifier
  const float y = __builtin_amdgcn_rsqf(v);
  const float s = v * y;
  float e2;
  asm("v_fma_f32 %0, -%1, %1, %2 div:2" : "=v"(e2) : "v"(s), "v"(v));
  return __builtin_fmaf(e2, y, s);
}

__global__ void k(uint32_t base, uint32_t n, unsigned long long* diff_all, unsigned long long* diff_hi,
                  unsigned long long* ieee_hi) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = base + i;
  const float x = __uint_as_float(b);
  const float fa = mag_h(x), fo = mag_omod(x);
  const uint32_t o = __float_as_uint(fo);
  const bool hi = b >= 0x0F800000u;  // v >= 2^-96: the range the sweep trusts
  if (__float_as_uint(fa) != o && !(fa != fa && fo != fo)) {
    atomicAdd(diff_all, 1ull);
    if (hi) atomicAdd(diff_hi, 1ull);
  }
  if (hi && o != __float_as_uint(sqrtf(x))) atomicAdd(ieee_hi, 1ull);
}

int main() {
  unsigned long long* d;
  if (hipMalloc(&d, 24) != hipSuccess || hipMemset(d, 0, 24) != hipSuccess) return 2;
  const uint64_t top = 0x7F800000ull, chunk = 1ull << 28;
  for (uint64_t base = 0; base < top; base += chunk) {
    const uint32_t n = (uint32_t)(base + chunk > top ? top - base : chunk);
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, (uint32_t)base, n, d, d + 1, d + 2);
  }
  unsigned long long h[3];
  if (hipMemcpy(h, d, 24, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("omod vs h sequence: %llu differing inputs (%llu of them >= 2^-96); omod vs IEEE sqrtf >= 2^-96: %llu\n",
         h[0], h[1], h[2]);
  return (h[1] == 0 && h[2] == 0) ? 0 : 1;
}
