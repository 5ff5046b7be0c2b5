// Weight-stream intake probe (tools only, not part of the library): how fast one CU takes in a
// weight image that every CU reads (L2-resident after the first touch), the access pattern of the
// streamed MLP tails (mlp_stream.h): 256 workgroups x 16 waves, wave w reads its own 1 KiB
// fragments of an image of `kb` KiB, all CUs the same image.
//   mode 0: global_load_dwordx4 into an R-deep register ring (the tails' scheme), summed
//   mode 1: LDS-DMA (global_load_lds_dwordx4) into a per-wave ring of S 1-KiB LDS slots, counted
//           vmcnt, each slot read back by ds_read_b128 and summed
//   mode 2: mode 0 with the loads issued nontemporal
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

constexpr int kWaves = 16;

template <int R>
__global__ __launch_bounds__(1024) void ring_regs(const float* __restrict__ img, int nfrag, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // wave w reads fragments w, w + 16, ... (1 KiB each)
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int n = nfrag / kWaves;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[(int64_t)(wave + kWaves * i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      acc += ring[j];
      if (i + j + R < n) ring[j] = base[(int64_t)(wave + kWaves * (i + j + R)) * 64];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

template <int R>
__global__ __launch_bounds__(1024) void ring_regs_nt(const float* __restrict__ img, int nfrag, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int n = nfrag / kWaves;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = __builtin_nontemporal_load(base + (int64_t)(wave + kWaves * i) * 64);
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      acc += ring[j];
      if (i + j + R < n) ring[j] = __builtin_nontemporal_load(base + (int64_t)(wave + kWaves * (i + j + R)) * 64);
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// S slots of 1 KiB per wave in LDS; S - 1 DMA loads in flight ahead of the slot being read
template <int S>
__global__ __launch_bounds__(1024) void ring_dma(const float* __restrict__ img, int nfrag, float* out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* slots = sm + wave * S * 256;
  const float* base = img + 4 * lane;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int n = nfrag / kWaves;
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    __builtin_amdgcn_global_load_lds((glb_void*)(base + (int64_t)(wave + kWaves * i) * 256), (lds_void*)(slots + 256 * i),
                                     16, 0, 0);
  for (int i = 0; i < n; ++i) {
    if (i + S - 1 < n)
      __builtin_amdgcn_global_load_lds((glb_void*)(base + (int64_t)(wave + kWaves * (i + S - 1)) * 256),
                                       (lds_void*)(slots + 256 * ((i + S - 1) % S)), 16, 0, 0);
    // slot i % S complete: S - 1 younger loads may stay in flight (fewer at the tail)
    if (i + S - 1 < n)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S - 1) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const f4 v = *reinterpret_cast<const f4*>(slots + 256 * (i % S) + 4 * lane);
    acc += v;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read before it is refilled
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// The same streams with each 1 KiB fragment consumed as the B operand of MF 16x16x4 f32 MFMAs
// (MF = 4: a one-tile layer of the tails, 4 waves per SIMD): does the intake hold with the matrix
// pipe busy?
template <int R, int MF>
__global__ __launch_bounds__(1024) void ring_regs_mfma(const float* __restrict__ img, int nfrag, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
  const int n = nfrag / kWaves;  // a multiple of R here
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[(int64_t)(wave + kWaves * i) * 64];
  for (int i = 0; i < n - R; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
      for (int m = 0; m < MF; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j][m & 3], acc, 0, 0, 0);
      ring[j] = base[(int64_t)(wave + kWaves * (i + j + R)) * 64];
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int m = 0; m < MF; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j][m & 3], acc, 0, 0, 0);
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

template <int S, int MF>
__global__ __launch_bounds__(1024) void ring_dma_mfma(const float* __restrict__ img, int nfrag, float* out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* slots = sm + wave * S * 256;
  const float* base = img + 4 * lane;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
  const int n = nfrag / kWaves;
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    __builtin_amdgcn_global_load_lds((glb_void*)(base + (int64_t)(wave + kWaves * i) * 256), (lds_void*)(slots + 256 * i),
                                     16, 0, 0);
  for (int i = 0; i < n; ++i) {
    if (i + S - 1 < n) {
      __builtin_amdgcn_global_load_lds((glb_void*)(base + (int64_t)(wave + kWaves * (i + S - 1)) * 256),
                                       (lds_void*)(slots + 256 * ((i + S - 1) % S)), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S - 1) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const f4 v = *reinterpret_cast<const f4*>(slots + 256 * (i % S) + 4 * lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int m = 0; m < MF; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, v[m & 3], acc, 0, 0, 0);
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// MFMA only, no loads: n chunks of MF MFMAs per wave on C independent accumulator chains (the
// pipe's rate with 4 waves per SIMD and 1 or 2 chains per wave)
template <int MF, int C>
__global__ __launch_bounds__(1024) void mfma_only(int n, float* out) {
  const int lane = threadIdx.x & 63;
  f4 acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = (f4){0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane, b = 2.0f - lane;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int m = 0; m < MF; ++m) acc[m % C] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m % C], 0, 0, 0);
  }
  f4 t = acc[0];
#pragma unroll
  for (int c = 1; c < C; ++c) t += acc[c];
  if (t[0] + t[1] + t[2] + t[3] == 12345.f) out[threadIdx.x] = t[0];
}

// loads + MFMA with the chunk's MFMAs alternating over 2 accumulator chains
template <int R, int MF>
__global__ __launch_bounds__(1024) void ring_regs_mfma2(const float* __restrict__ img, int nfrag, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const float a = 1.0f + lane;
  const int n = nfrag / kWaves;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[(int64_t)(wave + kWaves * i) * 64];
  for (int i = 0; i < n - R; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        if (m & 1)
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j][m & 3], acc1, 0, 0, 0);
        else
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j][m & 3], acc0, 0, 0, 0);
      }
      ring[j] = base[(int64_t)(wave + kWaves * (i + j + R)) * 64];
    }
  }
  acc0 += acc1;
  if (acc0[0] + acc0[1] + acc0[2] + acc0[3] == 12345.f) out[threadIdx.x] = acc0[0];
}

int main() {
  const int kb_list[] = {128, 896, 2560};
  float* img;
  float* out;
  const int max_kb = 4096;
  hipMalloc(&img, (size_t)max_kb * 1024);
  hipMalloc(&out, 1024 * sizeof(float));
  std::vector<float> h((size_t)max_kb * 256, 0.5f);
  hipMemcpy(img, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)ring_dma<4>, hipFuncAttributeMaxDynamicSharedMemorySize, kWaves * 4 * 1024);
  hipFuncSetAttribute((const void*)ring_dma<8>, hipFuncAttributeMaxDynamicSharedMemorySize, kWaves * 8 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int kb : kb_list) {
    const int nfrag = kb;  // 1 KiB fragments
    for (int mode = 0; mode < 5; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: ring_regs<8><<<256, 1024>>>(img, nfrag, out); break;
          case 1: ring_regs<4><<<256, 1024>>>(img, nfrag, out); break;
          case 2: ring_regs_nt<8><<<256, 1024>>>(img, nfrag, out); break;
          case 3: ring_dma<4><<<256, 1024, kWaves * 4 * 1024>>>(img, nfrag, out); break;
          default: ring_dma<8><<<256, 1024, kWaves * 8 * 1024>>>(img, nfrag, out); break;
        }
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = 1e3 * ms / it;
      const char* names[] = {"regs R=8", "regs R=4", "regs R=8 nt", "dma S=4", "dma S=8"};
      printf("image %5d KiB  %-12s %8.2f us per launch  %7.1f GB/s per CU\n", kb, names[mode], us,
             kb * 1024.0 / (us * 1e-6) / 1e9);
    }
  }
  hipFuncSetAttribute((const void*)ring_dma_mfma<4, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kWaves * 4 * 1024);
  hipFuncSetAttribute((const void*)ring_dma_mfma<4, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, kWaves * 4 * 1024);
  for (int kb : {896, 2560}) {
    for (int mode = 0; mode < 6; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: ring_regs_mfma<4, 4><<<256, 1024>>>(img, kb, out); break;
          case 1: ring_regs_mfma<8, 4><<<256, 1024>>>(img, kb, out); break;
          case 2: ring_dma_mfma<4, 4><<<256, 1024, kWaves * 4 * 1024>>>(img, kb, out); break;
          case 3: ring_regs_mfma<4, 8><<<256, 1024>>>(img, kb, out); break;
          case 4: ring_regs_mfma<8, 8><<<256, 1024>>>(img, kb, out); break;
          default: ring_dma_mfma<4, 8><<<256, 1024, kWaves * 4 * 1024>>>(img, kb, out); break;
        }
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = 1e3 * ms / it;
      const char* names[] = {"regs4 mf4", "regs8 mf4", "dma4 mf4", "regs4 mf8", "regs8 mf8", "dma4 mf8"};
      // MFMA floor: kb fragments x MF MFMAs x 32 cycles / 4 SIMDs
      printf("image %5d KiB  %-10s %8.2f us  %7.1f GB/s per CU  (MFMA floor %.1f kcycles per SIMD)\n", kb, names[mode],
             us, kb * 1024.0 / (us * 1e-6) / 1e9, kb * (mode % 3 == 0 || mode == 1 || mode == 2 ? (mode < 3 ? 4 : 8) : 8) * 32.0 / 4 / 1e3);
    }
  }
  for (int mode = 0; mode < 4; ++mode) {
    const int kb = 896;
    auto launch = [&]() {
      switch (mode) {
        case 0: mfma_only<4, 1><<<256, 1024>>>(kb / kWaves, out); break;
        case 1: mfma_only<4, 2><<<256, 1024>>>(kb / kWaves, out); break;
        case 2: mfma_only<4, 4><<<256, 1024>>>(kb / kWaves, out); break;
        default: ring_regs_mfma2<8, 4><<<256, 1024>>>(img, kb, out); break;
      }
    };
    for (int w = 0; w < 5; ++w) launch();
    hipEventRecord(a);
    const int it = 50;
    for (int w = 0; w < it; ++w) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const char* names[] = {"mfma only, 1 chain", "mfma only, 2 chains", "mfma only, 4 chains", "regs8 mf4 2 chains"};
    printf("896-KiB schedule  %-22s %8.2f us  (MFMA floor 28.7 kcycles per SIMD)\n", names[mode], 1e3 * ms / it);
  }
  hipError_t e = hipGetLastError();
  printf("status: %s\n", hipGetErrorString(e));
  return 0;
}
