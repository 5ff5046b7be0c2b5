// FP32 MFMA (v_mfma_f32_32x32x2_f32) rate calibration at the BST kernel's occupancy
// (512-thread workgroups, one per CU, 2 waves / SIMD).  Variants:
//   0  register operands only, NCH independent accumulator chains per wave
//   1  A operand float4 from LDS (one chunk ahead), B from registers
//   2  A from LDS, B float4 streamed from a 64 KB global weight (L2-resident), 1-chunk prefetch
//   3  A from LDS, B streamed in 4-chunk super-chunks, double buffered (bst_block WStream)
//   4  A from LDS, B float4 from LDS
//   5+ MLP-shaped (mlp_core.h): 1024-thread workgroups (4 waves / SIMD), v_mfma_f32_16x16x4_f32,
//      one 16-row A tile from LDS, TPW weight tiles streamed with a PD-chunk register ring
// Prints achieved TFLOP/s and cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ unsigned long long g_cycles;
template <int NCH, int MODE>
__global__ __launch_bounds__(512) void calib(const float* __restrict__ W, float* out, int iters) {
  __shared__ float A[64 * 132];
  const unsigned long long t0 = clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * 132; i += 512) A[i] = 0.001f * (i & 7);
  __syncthreads();
  f32x16 acc[NCH];
  for (int j = 0; j < NCH; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  const float* arow = A + ((wave >> 2) * 32 + (lane & 31)) * 132 + 4 * (lane >> 5);
  const float* wrow = W + ((wave & 3) * 32 + (lane & 31)) * 128 + 4 * (lane >> 5);
  f4 a = {1.f, 2.f, 3.f, 4.f}, bb = {0.5f, 0.25f, 0.125f, 1.f};
  f4 bn = bb;
  if (MODE == 3) {
    f4 bq[2][4];
    for (int c = 0; c < 4; ++c) bq[0][c] = *reinterpret_cast<const f4*>(wrow + 8 * c);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 4; ++c) bq[(s + 1) & 1][c] = *reinterpret_cast<const f4*>(wrow + 32 * ((s + 1) & 3) + 8 * c);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const f4 an = *reinterpret_cast<const f4*>(arow + 8 * ((4 * s + c + 1) & 15));
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < NCH; ++j)
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], bq[s & 1][c][e], acc[j], 0, 0, 0);
          a = an;
        }
      }
    }
  }
  const float* lrow = A + ((wave & 1) * 32 + (lane & 31)) * 132 + 4 * (lane >> 5) + 64;
  for (int it = 0; it < (MODE == 3 ? 0 : iters); ++it) {
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      f4 an = a, bc = bb;
      if (MODE >= 1) an = *reinterpret_cast<const f4*>(arow + 8 * ((c + 1) & 15));
      if (MODE == 4) bc = *reinterpret_cast<const f4*>(lrow + 4 * (c & 7));
      if (MODE == 2) {
        bc = bn;
        bn = *reinterpret_cast<const f4*>(wrow + 8 * ((c + 1) & 15));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < NCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], bc[e], acc[j], 0, 0, 0);
      if (MODE >= 1) a = an;
    }
  }
  float s = 0.f;
  for (int j = 0; j < NCH; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) atomicAdd(&g_cycles, clock64() - t0);
}

// dynamic LDS padding that forces one 512-thread workgroup per CU (2 waves / SIMD), like bst_block
constexpr size_t kPadLds = 120 * 1024;

template <int NCH, int MODE>
void run(const float* W, float* out, int cus) {
  const int iters = 200;
  hipFuncSetAttribute((const void*)calib<NCH, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  calib<NCH, MODE><<<cus, 512, kPadLds>>>(W, out, iters);
  unsigned long long z = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(g_cycles), &z, 8);
  hipEventRecord(e0);
  calib<NCH, MODE><<<cus, 512, kPadLds>>>(W, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfma = (double)cus * 8 * iters * 16 * 4 * NCH;  // per wave: iters*16 chunks*4*NCH
  const double tf = mfma * 32 * 32 * 2 * 2 / (ms * 1e-3) / 1e12;
  unsigned long long cyc;
  hipMemcpyFromSymbol(&cyc, HIP_SYMBOL(g_cycles), 8);
  const double per_wg = (double)cyc / cus, mfma_per_simd = 2.0 * iters * 16 * 4 * NCH;
  printf("mode %d chains %d: %.3f ms  %.1f TFLOP/s  (%.1f%% of 157.3)  clock64 %.1f cyc/MFMA/SIMD, %.2f GHz\n",
         MODE, NCH, ms, tf, 100 * tf / 157.3, per_wg / mfma_per_simd, per_wg / (ms * 1e6));
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// MLP-shaped stream: K = 512 (32 chunks of 16), W tile rows read from a 256 KB weight (L2),
// TPW tiles per wave, ring depth PD, A one chunk ahead (APF) or in the same chunk.
template <int TPW, int PD, bool APF, bool SPLIT>
__global__ __launch_bounds__(1024) void calib_mlp(const float* __restrict__ W, float* out, int iters) {
  __shared__ float A[16 * 516];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 16 * 516; i += 1024) A[i] = 0.001f * (i & 7);
  __syncthreads();
  const int li = lane & 15, kq = 4 * (lane >> 4);
  constexpr int KC = 32;
  const float* wrow[TPW];
  for (int j = 0; j < TPW; ++j) wrow[j] = W + (size_t)(16 * ((wave + 16 * j) & 15) + li) * 512 + kq;
  f32x4 acc[TPW][2];
  for (int j = 0; j < TPW; ++j) acc[j][0] = acc[j][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const float* arow = A + li * 516 + kq;
  for (int it = 0; it < iters; ++it) {
    f32x4 ring[PD][TPW];
#pragma unroll
    for (int s = 0; s < PD; ++s)
#pragma unroll
      for (int j = 0; j < TPW; ++j) ring[s][j] = *reinterpret_cast<const f32x4*>(wrow[j] + 16 * s);
    f32x4 an = *reinterpret_cast<const f32x4*>(arow);
    for (int c0 = 0; c0 < KC; c0 += PD) {
#pragma unroll
      for (int s = 0; s < PD; ++s) {
        const int c = c0 + s;
        f32x4 av;
        if (APF) {
          av = an;
          an = *reinterpret_cast<const f32x4*>(arow + 16 * min(c + 1, KC - 1));
        } else {
          av = *reinterpret_cast<const f32x4*>(arow + 16 * c);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < TPW; ++j) {
            f32x4& a = acc[j][SPLIT ? (e & 1) : 0];
            a = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], ring[s][j][e], a, 0, 0, 0);
          }
        const int cn = min(c + PD, KC - 1);
#pragma unroll
        for (int j = 0; j < TPW; ++j) ring[s][j] = *reinterpret_cast<const f32x4*>(wrow[j] + 16 * cn);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  float sacc = 0.f;
  for (int j = 0; j < TPW; ++j)
    for (int r = 0; r < 4; ++r) sacc += acc[j][0][r] + acc[j][1][r];
  out[blockIdx.x * 1024 + threadIdx.x] = sacc;
}

template <int TPW, int PD, bool APF, bool SPLIT>
void run_mlp(const float* W, float* out, int cus) {
  const int iters = 100;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  calib_mlp<TPW, PD, APF, SPLIT><<<cus, 1024>>>(W, out, iters);
  hipEventRecord(e0);
  calib_mlp<TPW, PD, APF, SPLIT><<<cus, 1024>>>(W, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = (double)cus * 16 * iters * 32 * 4 * TPW * 16 * 16 * 4 * 2;
  printf("mlp TPW %d PD %d Aprefetch %d split-acc %d: %.3f ms  %.1f TFLOP/s (%.1f%%)\n", TPW, PD, (int)APF,
         (int)SPLIT, ms, flop / (ms * 1e-3) / 1e12, 100 * flop / (ms * 1e-3) / 157.3e12);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float *W, *out;
  hipMalloc(&W, 128 * 128 * 4);
  hipMemset(W, 0, 128 * 128 * 4);
  hipMalloc(&out, (size_t)cus * 512 * 4);
  printf("%d CUs\n", cus);
  run<1, 0>(W, out, cus);
  run<2, 0>(W, out, cus);
  run<4, 0>(W, out, cus);
  run<1, 1>(W, out, cus);
  run<2, 1>(W, out, cus);
  run<1, 2>(W, out, cus);
  run<2, 2>(W, out, cus);
  run<1, 3>(W, out, cus);
  run<2, 3>(W, out, cus);
  run<1, 4>(W, out, cus);
  run<2, 4>(W, out, cus);
  float* W2;
  hipMalloc(&W2, 512 * 512 * 4);
  hipMemset(W2, 0, 512 * 512 * 4);
  run_mlp<1, 4, false, false>(W2, out, cus);
  run_mlp<1, 4, true, false>(W2, out, cus);
  run_mlp<1, 4, true, true>(W2, out, cus);
  run_mlp<1, 8, true, true>(W2, out, cus);
  run_mlp<2, 4, false, false>(W2, out, cus);
  run_mlp<2, 4, true, false>(W2, out, cus);
  run_mlp<2, 8, true, false>(W2, out, cus);
  return 0;
}
