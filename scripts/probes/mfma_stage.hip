// Diagnostic: where the f32 MFMA sweep loses issue rate. One stage = KS K rows = KS/2 k pairs
// x 4 v_mfma_f32_32x32x2_f32 per wave (2 x 2 blocks of 32 x 32, as k_sweep_mfma), 256-thread
// workgroups, OCC per CU. Variants add, one at a time, what the sweep's stage carries:
//   0 register operands only          1 + operands read from LDS per k pair (lgkmcnt per pair)
//   2 + a workgroup barrier per stage 3 + per-stage global loads of the next stage (register
//   staged, issued at the top of the stage, L2-resident source) written to the other LDS buffer
//   4 the loads as global_load_lds into a 3-stage ring, two stages in flight (counted vmcnt)
//   5 global_load_lds into 2 slots, one stage in flight (issued after the stage's barrier)
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_stage scripts/probes/mfma_stage.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int T = 128;

template <int V, int KS, int OCC>
__global__ __launch_bounds__(256, OCC) void k(const float* __restrict__ src, float* out, int stages,
                                              int64_t src_rows) {
  constexpr int NB = (V == 4) ? 3 : 2;
  constexpr int RING = (V == 5) ? 2 : 3;
  __shared__ __attribute__((aligned(16))) float smem[NB * KS * T * 2];
  float(*sq)[KS][T] = reinterpret_cast<float(*)[KS][T]>(smem);
  float(*se)[KS][T] = reinterpret_cast<float(*)[KS][T]>(smem + NB * KS * T);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wq = wave >> 1, we = wave & 1, lrow = lane >> 5, lcol = lane & 31;
  for (int i = tid; i < NB * KS * T; i += 256) {
    (&sq[0][0][0])[i] = 1e-3f * (i & 127);
    (&se[0][0][0])[i] = 1e-3f * ((i >> 3) & 127);
  }
  __syncthreads();
  floatx16 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  float ra0 = lane * 1e-3f, ra1 = ra0 + 1.0f, rb0 = ra0 * 0.5f, rb1 = ra0 + 2.0f;
  const int srow = tid >> 5, sc4 = tid & 31;
  // big sources: each stage reads a different far-apart slice (HBM streaming, as C5's table)
  auto src_row = [&](int s) { return ((int64_t)blockIdx.x * 7919 + (int64_t)s * KS * 61) % (src_rows - KS); };
  // V4: wave w fills rows (KS/4) w .. of both operands, 2 rows (1 KB) per instruction
  auto issue = [&](int s) {
    const int slot = s % RING;
    const int64_t r0 = src_row(s);
#pragma unroll
    for (int i = 0; i < KS / 8; ++i) {
      const int row = (KS / 4) * wave + 2 * i;
      const float* p = src + (r0 + row + lrow) * 512 + lcol * 4;
      __builtin_amdgcn_global_load_lds(p, (lds_ptr_t)&sq[slot][row][0], 16, 0, 0);
      __builtin_amdgcn_global_load_lds(p + 256, (lds_ptr_t)&se[slot][row][0], 16, 0, 0);
    }
  };
  float4 g[KS / 4];
  int buf = 0;
  if constexpr (V == 4) {
    issue(0);
    issue(1);
  }
  if constexpr (V == 5) issue(0);
  for (int s = 0; s < stages; ++s) {
    if constexpr (V == 3) {
      const float* p = src + (src_row(s) + srow) * 512 + sc4 * 4;
#pragma unroll
      for (int i = 0; i < KS / 8; ++i) {
        g[2 * i] = *reinterpret_cast<const float4*>(p + 8 * i * 512);
        g[2 * i + 1] = *reinterpret_cast<const float4*>(p + 8 * i * 512 + 256);
      }
      __builtin_amdgcn_sched_barrier(0);  // loads stay at the top of the stage (hipcc sinks them)
    }
    if constexpr (V == 4) {
      if (s + 1 < stages) {
        if constexpr (KS == 16) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (s + 2 < stages) issue(s + 2);
      buf = s % 3;
    }
    if constexpr (V == 5) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of stage s landed
      __builtin_amdgcn_s_barrier();                     // all parts landed; slot (s+1)%2 is free
      if (s + 1 < stages) issue(s + 1);
      buf = s & 1;
    }
#pragma unroll
    for (int kp2 = 0; kp2 < KS; kp2 += 2) {
      float a0 = ra0, a1 = ra1, b0 = rb0, b1 = rb1;
      if constexpr (V >= 1) {
        a0 = sq[buf][kp2 + lrow][wq * 64 + lcol];
        a1 = sq[buf][kp2 + lrow][wq * 64 + 32 + lcol];
        b0 = se[buf][kp2 + lrow][we * 64 + lcol];
        b1 = se[buf][kp2 + lrow][we * 64 + 32 + lcol];
      }
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if constexpr (V == 3) {
#pragma unroll
      for (int i = 0; i < KS / 8; ++i) {
        *reinterpret_cast<float4*>(&sq[buf ^ 1][srow + 8 * i][sc4 * 4]) = g[2 * i];
        *reinterpret_cast<float4*>(&se[buf ^ 1][srow + 8 * i][sc4 * 4]) = g[2 * i + 1];
      }
    }
    if constexpr (V == 2 || V == 3) {
      __syncthreads();
      buf ^= 1;
    }
  }
  float t = 0.0f;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int r = 0; r < 16; ++r) t += acc[a][b][r];
  if (t == 1234.5f) out[tid] = t;
}

// V6: one 512-thread workgroup per CU over a 256 (q) x 128 (e) tile: 8 waves as 4 (q) x 2 (e),
// each 64 x 64 as before, register-staged K stages: 25 % less staging per MFMA than two 128 x
// 128 workgroups, but both waves of a SIMD now meet at the same barrier
template <int KS>
__global__ __launch_bounds__(512, 1) void k6(const float* __restrict__ src, float* out, int stages, int64_t src_rows) {
  constexpr int TQ2 = 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * KS * (TQ2 + T)];
  float(*sq)[KS][TQ2] = reinterpret_cast<float(*)[KS][TQ2]>(smem);
  float(*se)[KS][T] = reinterpret_cast<float(*)[KS][T]>(smem + 2 * KS * TQ2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wq = wave >> 1, we = wave & 1, lrow = lane >> 5, lcol = lane & 31;
  for (int i = tid; i < 2 * KS * TQ2; i += 512) (&sq[0][0][0])[i] = 1e-3f * (i & 127);
  for (int i = tid; i < 2 * KS * T; i += 512) (&se[0][0][0])[i] = 1e-3f * ((i >> 3) & 127);
  __syncthreads();
  floatx16 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  auto src_row = [&](int s) { return ((int64_t)blockIdx.x * 7919 + (int64_t)s * KS * 61) % (src_rows - KS); };
  // per stage: q 256 x KS floats (thread: KS/16 float4 rows of 64 threads per 256 cols), e 128 x KS
  const int qrow = tid >> 6, qc4 = tid & 63;   // q: 8 rows per pass, 64 float4 per row
  const int erow = tid >> 5, ec4 = tid & 31;   // e: 16 rows per pass, 32 float4 per row
  float4 gq[KS / 8], ge[KS / 16];
  int buf = 0;
  for (int s = 0; s < stages; ++s) {
    const float* p = src + src_row(s) * 512;
#pragma unroll
    for (int i = 0; i < KS / 8; ++i) gq[i] = *reinterpret_cast<const float4*>(p + (qrow + 8 * i) * 512 + qc4 * 4);
#pragma unroll
    for (int i = 0; i < KS / 16; ++i)
      ge[i] = *reinterpret_cast<const float4*>(p + (erow + 16 * i) * 512 + 256 + ec4 * 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kp2 = 0; kp2 < KS; kp2 += 2) {
      const float a0 = sq[buf][kp2 + lrow][wq * 64 + lcol], a1 = sq[buf][kp2 + lrow][wq * 64 + 32 + lcol];
      const float b0 = se[buf][kp2 + lrow][we * 64 + lcol], b1 = se[buf][kp2 + lrow][we * 64 + 32 + lcol];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < KS / 8; ++i) *reinterpret_cast<float4*>(&sq[buf ^ 1][qrow + 8 * i][qc4 * 4]) = gq[i];
#pragma unroll
    for (int i = 0; i < KS / 16; ++i) *reinterpret_cast<float4*>(&se[buf ^ 1][erow + 16 * i][ec4 * 4]) = ge[i];
    __syncthreads();
    buf ^= 1;
  }
  float t = 0.0f;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int r = 0; r < 16; ++r) t += acc[a][b][r];
  if (t == 1234.5f) out[tid] = t;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  int64_t src_rows = 1 << 13;  // 16 MB source: L2 / Infinity-Cache resident
  const int64_t big_rows = (int64_t)1 << 20;  // 2 GB source: HBM
  float* src;
  (void)hipMalloc(&src, big_rows * 512 * sizeof(float));
  (void)hipMemset(src, 0, big_rows * 512 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int kflat = 32000;  // K rows per workgroup (stages x KS)
  auto run = [&](auto kern, const char* name, int per_cu, int ks, int threads = 256) {
    const int blocks = cus * per_cu, stages = kflat / ks;
    float best = 1e9f;
    for (int r = 0; r < 4; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, src, out, stages, src_rows);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double flops = (double)blocks * (threads / 64) * stages * (ks / 2) * 4 * (32.0 * 32 * 2 * 2);
    printf("%-40s %s KS %2d  %d/CU  %8.3f ms  %7.1f TF  %.3f of 157.3\n", name, src_rows > 100000 ? "HBM" : "L2 ", ks, per_cu, best, flops / best / 1e9,
           flops / best / 1e9 / 157.3);
  };
  run(k<0, 16, 2>, "V0 register operands", 2, 16);
  run(k<1, 16, 2>, "V1 + LDS operand reads", 2, 16);
  run(k<2, 16, 2>, "V2 + barrier per stage", 2, 16);
  for (int big = 0; big < 2; ++big) {
    src_rows = big ? big_rows : (1 << 13);
    run(k<3, 16, 2>, "V3 + global->LDS staging (early)", 2, 16);
    run(k<4, 16, 2>, "V4 glds ring, 2 stages in flight", 2, 16);
    run(k<3, 32, 2>, "V3 + global->LDS staging (early)", 2, 32);
    run(k<4, 16, 3>, "V4 glds ring, 2 stages in flight", 3, 16);
    run(k<5, 16, 2>, "V5 glds 2 slots, 1 stage in flight", 2, 16);
    run(k<5, 32, 2>, "V5 glds 2 slots, 1 stage in flight", 2, 32);
    run(k6<32>, "V6 256x128 tile, 8 waves, 1/CU", 1, 32, 512);
    run(k6<16>, "V6 256x128 tile, 8 waves, 1/CU", 1, 16, 512);
  }
  (void)hipFree(src);
  (void)hipFree(out);
  return 0;
}
