// Weight-image layout probe (tools only, not part of the library): does the ORDER in which the 16
// waves of every CU walk a shared L2-resident image change the intake rate?  256 workgroups x 16
// waves, R = 8 register ring of 1 KiB fragments, each fragment optionally feeding 4
// v_mfma_f32_16x16x4_f32 (one tile-chunk of the streamed tails, mlp_stream.h).
//   contiguous : step i, wave w reads fragment 16 i + w (the 16 waves read 16 adjacent KiB)
//   tile-major : wave w reads fragments w n + i (its own tile's chunks, n = fragments per wave):
//                the packed-weight layout the tails use, tiles n KiB apart
//   tile-major+pad : the same with tiles n + 1 KiB apart (breaks the common stride)
//   tile-major+xor : the same fragments, the tile base permuted per CU (blockIdx-dependent
//                rotation of the wave -> tile map), so CUs in lockstep read different tiles
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/stream_layout_probe tools/stream_layout_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kWaves = 16, R = 8;

template <int MODE, int MF>
__global__ __launch_bounds__(1024) void walk(const float* __restrict__ img, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  const int tile = MODE == 3 ? (wave + blockIdx.x) & (kWaves - 1) : wave;
  auto frag = [&](int i) -> int64_t {
    if (MODE == 0) return (int64_t)kWaves * i + wave;
    if (MODE == 2) return (int64_t)tile * (n + 1) + i;
    return (int64_t)tile * n + i;
  };
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[frag(i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (MF == 0) {
        acc += ring[j];
      } else {
#pragma unroll
        for (int m = 0; m < MF; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j][m & 3], acc, 0, 0, 0);
      }
      if (i + j + R < n) ring[j] = base[frag(i + j + R) * 64];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// Two 16-row tiles per fragment (RT = 2, or two CUs splitting a layer's columns for 32 rows): 8 MFMAs
// per fragment on two accumulator chains, over half the image
__global__ __launch_bounds__(1024) void walk_rt2(const float* __restrict__ img, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const float a0 = 1.0f + lane, a1 = 2.0f - lane;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[((int64_t)wave * n + i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, ring[j][m], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, ring[j][m], acc1, 0, 0, 0);
      }
      if (i + j + R < n) ring[j] = base[((int64_t)wave * n + i + j + R) * 64];
    }
  }
  acc0 += acc1;
  if (acc0[0] + acc0[1] + acc0[2] + acc0[3] == 12345.f) out[threadIdx.x] = acc0[0];
}

// walk<1, 4> with the accumulator held in AGPRs (the MFMA's C / D in the accumulation registers, as
// inline asm; the compiler's own choice is the VGPR form): does keeping the 4-register accumulator
// out of the VGPR file leave the load returns their write bandwidth?
__global__ __launch_bounds__(1024) void walk_agpr(const float* __restrict__ img, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[((int64_t)wave * n + i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(ring[j][m]));
      if (i + j + R < n) ring[j] = base[((int64_t)wave * n + i + j + R) * 64];
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 2" ::: "memory");
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// The same MFMA stream with its B fragments read from LDS (a 64-KiB resident image, ds_read_b128)
// instead of global memory: the cost of the VMEM instructions themselves
__global__ __launch_bounds__(1024) void walk_lds(const float* __restrict__ img, int n, float* out) {
  __shared__ f4 lds[64 * 64];  // 64 fragments of 1 KiB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * 64; i += 1024) lds[i] = reinterpret_cast<const f4*>(img)[i];
  __syncthreads();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
  f4 cur = lds[((wave * 4) & 63) * 64 + lane];
  for (int i = 0; i < n; ++i) {
    const f4 nxt = lds[((wave * 4 + i + 1) & 63) * 64 + lane];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, cur[m], acc, 0, 0, 0);
    cur = nxt;
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// walk<1, 4> with the ring refilled two fragments at a time (two loads back to back, then their 8
// MFMAs): the same instruction counts, a different issue pattern
__global__ __launch_bounds__(1024) void walk_pairs(const float* __restrict__ img, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[((int64_t)wave * n + i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; j += 2) {
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j][m], acc, 0, 0, 0);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j + 1][m], acc, 0, 0, 0);
      if (i + j + R < n) {
        ring[j] = base[((int64_t)wave * n + i + j + R) * 64];
        ring[j + 1] = base[((int64_t)wave * n + i + j + 1 + R) * 64];
      }
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// walk<1, 4> with the ring refilled G fragments at a time (G loads back to back after G fragments' MFMAs)
template <int G>
__global__ __launch_bounds__(1024) void walk_groups(const float* __restrict__ img, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[((int64_t)wave * n + i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; j += G) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j + g][m], acc, 0, 0, 0);
      if (i + j + R < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) ring[j + g] = base[((int64_t)wave * n + i + j + g + R) * 64];
      }
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// walk_groups<4> with the wave's priority raised around its MFMA burst (P = 1) or around its load
// burst (P = 2)
template <int P>
__global__ __launch_bounds__(1024) void walk_prio(const float* __restrict__ img, int n, float* out) {
  constexpr int G = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[R];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
#pragma unroll
  for (int i = 0; i < R; ++i) ring[i] = base[((int64_t)wave * n + i) * 64];
  for (int i = 0; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; j += G) {
      if (P == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j + g][m], acc, 0, 0, 0);
      if (P == 1) __builtin_amdgcn_s_setprio(0);
      if (P == 2) __builtin_amdgcn_s_setprio(1);
      if (i + j + R < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) ring[j + g] = base[((int64_t)wave * n + i + j + g + R) * 64];
      }
      if (P == 2) __builtin_amdgcn_s_setprio(0);
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

// walk_groups with an RR-deep ring
template <int RR, int G>
__global__ __launch_bounds__(1024) void walk_ring(const float* __restrict__ img, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = reinterpret_cast<const f4*>(img) + lane;
  f4 ring[RR];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + lane;
#pragma unroll
  for (int i = 0; i < RR; ++i) ring[i] = base[((int64_t)wave * n + i) * 64];
  for (int i = 0; i < n; i += RR) {
#pragma unroll
    for (int j = 0; j < RR; j += G) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int m = 0; m < 4; ++m)
          if (i + j + g < n) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ring[j + g][m], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (i + j + g + RR < n) ring[j + g] = base[((int64_t)wave * n + i + j + g + RR) * 64];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

int main() {
  float* img;
  float* out;
  const int max_kb = 4096;
  hipMalloc(&img, (size_t)max_kb * 1024);
  hipMalloc(&out, 1024 * sizeof(float));
  std::vector<float> h((size_t)max_kb * 256, 0.5f);
  hipMemcpy(img, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"contiguous", "tile-major", "tile-major+pad", "tile-major+rot"};
  for (int mf : {0, 4}) {
    for (int kb : {512, 896, 2560}) {  // per-layer image sizes: DCN/DIN 512->256 layer, DIN fcn, DeepFM
      const int n = kb / kWaves;
      for (int round = 0; round < 2; ++round) {
        for (int mode = 0; mode < 4; ++mode) {
          auto launch = [&]() {
            if (mf == 0) {
              switch (mode) {
                case 0: walk<0, 0><<<256, 1024>>>(img, n, out); break;
                case 1: walk<1, 0><<<256, 1024>>>(img, n, out); break;
                case 2: walk<2, 0><<<256, 1024>>>(img, n, out); break;
                default: walk<3, 0><<<256, 1024>>>(img, n, out); break;
              }
            } else {
              switch (mode) {
                case 0: walk<0, 4><<<256, 1024>>>(img, n, out); break;
                case 1: walk<1, 4><<<256, 1024>>>(img, n, out); break;
                case 2: walk<2, 4><<<256, 1024>>>(img, n, out); break;
                default: walk<3, 4><<<256, 1024>>>(img, n, out); break;
              }
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
          printf("mf %d image %5d KiB  %-16s %8.2f us  %7.1f GB/s per CU%s\n", mf, kb, names[mode], us,
                 kb * 1024.0 / (us * 1e-6) / 1e9, mf ? "  (MFMA floor: n x 4 x 32 cycles x 4 waves per SIMD)" : "");
        }
      }
    }
  }
  // the same walk (tile-major, MFMA) on fewer workgroups: one workgroup per CU, dispatched round-robin
  // over the 8 XCDs, so grid g puts g / 8 CUs on each XCD's L2.  A per-CU intake limit keeps the time;
  // a shared per-XCD L2 limit shortens it as the CUs per XCD drop.
  for (int round = 0; round < 2; ++round) {
    for (int grid : {256, 192, 128, 64, 32, 8}) {
      const int kb = 896, n = kb / kWaves;
      for (int w = 0; w < 5; ++w) walk<1, 4><<<grid, 1024>>>(img, n, out);
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) walk<1, 4><<<grid, 1024>>>(img, n, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = 1e3 * ms / it;
      printf("grid %3d (%2d CUs per XCD) image 896 KiB tile-major mf 4  %8.2f us  %7.1f GB/s per CU\n", grid, grid / 8,
             us, kb * 1024.0 / (us * 1e-6) / 1e9);
    }
  }
  // the same MFMA count per CU from half the bytes: 896 KiB x 4 MFMAs per fragment against 448 KiB x 8
  for (int round = 0; round < 2; ++round) {
    for (int mode = 0; mode < 2; ++mode) {
      const int kb = mode ? 448 : 896, n = kb / kWaves;
      auto launch = [&]() {
        if (mode) walk_rt2<<<256, 1024>>>(img, n, out);
        else walk<1, 4><<<256, 1024>>>(img, n, out);
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("%s  %8.2f us (MFMA floor 13.7 us at 2.1 GHz)\n",
             mode ? "448 KiB, 8 MFMAs per fragment on 2 chains (32 rows per fragment)"
                  : "896 KiB, 4 MFMAs per fragment on 1 chain (16 rows per fragment) ", 1e3 * ms / it);
    }
  }
  for (int round = 0; round < 2; ++round) {
    for (int mode = 0; mode < 2; ++mode) {
      const int kb = 896, n = kb / kWaves;
      auto launch = [&]() {
        if (mode) walk_agpr<<<256, 1024>>>(img, n, out);
        else walk<1, 4><<<256, 1024>>>(img, n, out);
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("896 KiB mf 4, accumulator in %s  %8.2f us\n", mode ? "AGPRs" : "VGPRs", 1e3 * ms / it);
    }
  }
  // more waves per SIMD: two 16-wave workgroups per CU (grid 512: 8 waves per SIMD), each walking
  // the whole image — twice the work of grid 256; 2x the time means no gain from the extra waves
  for (int round = 0; round < 2; ++round) {
    for (int grid : {256, 512}) {
      const int kb = 896, n = kb / kWaves;
      for (int w = 0; w < 5; ++w) walk<1, 4><<<grid, 1024>>>(img, n, out);
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) walk<1, 4><<<grid, 1024>>>(img, n, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("896 KiB mf 4, grid %d (%d waves per SIMD)  %8.2f us\n", grid, grid / 64, 1e3 * ms / it);
    }
  }
  for (int round = 0; round < 2; ++round) {
    for (int mode = 0; mode < 3; ++mode) {
      const int kb = 896, n = kb / kWaves;
      auto launch = [&]() {
        if (mode == 0) walk<1, 4><<<256, 1024>>>(img, n, out);
        else if (mode == 1) walk_lds<<<256, 1024>>>(img, n, out);
        else walk_pairs<<<256, 1024>>>(img, n, out);
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const char* nm[] = {"global fragments, one load per 4 MFMAs", "LDS fragments (ds_read_b128)",
                          "global fragments, loads in pairs"};
      printf("896-KiB walk mf 4: %-40s %8.2f us\n", nm[mode], 1e3 * ms / it);
    }
  }
  for (int round = 0; round < 2; ++round) {
    for (int g : {1, 2, 4, 8}) {
      const int kb = 896, n = kb / kWaves;
      auto launch = [&]() {
        if (g == 1) walk_groups<1><<<256, 1024>>>(img, n, out);
        else if (g == 2) walk_groups<2><<<256, 1024>>>(img, n, out);
        else if (g == 4) walk_groups<4><<<256, 1024>>>(img, n, out);
        else walk_groups<8><<<256, 1024>>>(img, n, out);
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("896-KiB walk mf 4: ring refilled %d at a time  %8.2f us\n", g, 1e3 * ms / it);
    }
  }
  for (int round = 0; round < 2; ++round) {
    for (int pm = 0; pm < 3; ++pm) {
      const int kb = 896, n = kb / kWaves;
      auto launch = [&]() {
        if (pm == 0) walk_groups<4><<<256, 1024>>>(img, n, out);
        else if (pm == 1) walk_prio<1><<<256, 1024>>>(img, n, out);
        else walk_prio<2><<<256, 1024>>>(img, n, out);
      };
      for (int w = 0; w < 5; ++w) launch();
      hipEventRecord(a);
      const int it = 50;
      for (int w = 0; w < it; ++w) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const char* nm[] = {"refill 4, no priority", "refill 4, setprio 1 over the MFMAs", "refill 4, setprio 1 over the loads"};
      printf("896-KiB walk mf 4: %-36s %8.2f us\n", nm[pm], 1e3 * ms / it);
    }
  }
  for (int round = 0; round < 2; ++round) {
    for (int v = 0; v < 5; ++v) {
      const int kb = 896, n = kb / kWaves;
      auto launch = [&]() {
        switch (v) {
          case 0: walk_ring<8, 4><<<256, 1024>>>(img, n, out); break;
          case 1: walk_ring<12, 4><<<256, 1024>>>(img, n, out); break;
          case 2: walk_ring<16, 4><<<256, 1024>>>(img, n, out); break;
          case 3: walk_ring<12, 6><<<256, 1024>>>(img, n, out); break;
          default: walk_ring<16, 8><<<256, 1024>>>(img, n, out); break;
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
      const char* nm[] = {"ring 8, bursts of 4", "ring 12, bursts of 4", "ring 16, bursts of 4", "ring 12, bursts of 6",
                          "ring 16, bursts of 8"};
      printf("896-KiB walk mf 4: %-22s %8.2f us\n", nm[v], 1e3 * ms / it);
    }
  }
  hipError_t e = hipGetLastError();
  printf("status: %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
