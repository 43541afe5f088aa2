// Exhaustive error bound of the raw v_sqrt_f32 against the correctly rounded IEEE sqrtf over
// every non-negative float below +inf (and +inf itself): the largest distance in ulps (bit
// patterns of two non-negative floats) for normal inputs, and the largest absolute error for
// denormal inputs. This bound is what the RotatE sweep's fast filter relies on. Diagnostic.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(uint32_t base, uint32_t n, uint32_t* max_ulp, uint32_t* max_ulp_at, uint32_t* max_abs_den,
                  uint32_t* bad_special) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = base + i;
  const float x = __uint_as_float(b);
  const float a = __builtin_amdgcn_sqrtf(x), c = sqrtf(x);
  const uint32_t ab = __float_as_uint(a), cb = __float_as_uint(c);
  if (b >= 0x7F800000u || b == 0u) {  // +inf, +0: must be exact
    if (ab != cb) atomicAdd(bad_special, 1u);
    return;
  }
  if ((ab >> 31) || ab >= 0x7F800000u) { atomicAdd(bad_special, 1u); return; }  // negative / inf / NaN
  const uint32_t d = ab > cb ? ab - cb : cb - ab;
  if (b < 0x00800000u) {  // denormal input: absolute error, as float bits of |a - c|
    const float e = fabsf(a - c);
    atomicMax(max_abs_den, __float_as_uint(e));
  } else if (d) {
    atomicMax(max_ulp, d);
    if (d > 1) atomicMax(max_ulp_at, b);
  }
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 16) != hipSuccess || hipMemset(d, 0, 16) != hipSuccess) return 2;
  const uint64_t top = 0x7F800000ull, chunk = 1ull << 28;
  for (uint64_t base = 0; base <= top; base += chunk) {
    const uint32_t n = (uint32_t)(base + chunk > top + 1 ? top + 1 - base : chunk);
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, (uint32_t)base, n, d, d + 1, d + 2, d + 3);
  }
  uint32_t h[4];
  if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("v_sqrt_f32 vs sqrtf: max %u ulp on normal inputs (largest input beyond 1 ulp 0x%08x); "
         "max abs error on denormal inputs %g; special-case mismatches %u\n",
         h[0], h[1], (double)__builtin_bit_cast(float, h[2]), h[3]);
  return (h[0] <= 1 && h[3] == 0) ? 0 : 1;
}
