// Round-6 gather probe: (a) known-byte calibration of FETCH_SIZE for the access
// shapes of the embedding gather, (b) the copy ceiling re-timed, (c) field-major gather variants.
//
// (a) calibration kernels over a 2 GiB table of 128-B rows (16.7 M rows, far beyond the 256 MiB
//     Infinity Cache), N = 2,097,152 DISTINCT random rows read once each:
//       cal_rows128   whole 128-B rows (8 lanes x 16 B per row, 8 rows per wave-instruction)
//       cal_rows64    the first 64 B of each row
//       cal_word4     one 4-B word per row (64 rows per wave-instruction)
//     Known bytes: N x 128, N x 64, N x 4 (+ N x 8 of indices, streamed).
// (b) copy: 2 GiB -> 2 GiB, float4, 4 loads in flight per lane.
// (c) the DeepFM gather (configs[1] tables: 30 fields x 1e6 rows x 32 fp32 + first-order weights,
//     8,048 algorithmic B/sample) at batch 4096 / 65536:
//       sm          one wave per sample (the round-5 kernel's structure), tables or packed rows
//       fm<U>       FIELD-MAJOR: a wave owns 8 samples (lane = sample slot x quad) and walks the
//                   fields in order, U fields' rows in flight; every wave on the chip sweeps field
//                   f at about the same time, so field f's 4-MB first-order table is re-read from
//                   the on-die caches instead of costing a 128-B HBM line per lookup
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_probe2.hip -o tools/bin/gather_probe2
//   tools/bin/gather_probe2 [only-substring]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int F = 30, D = 32, G = 8, RS = 36;

// non-zero table contents (RANDOM=1): a hash of the element index as a float in [-1, 1)
__global__ void fill_hash(float* __restrict__ p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = (float)(h & 0xffffff) / 8388608.0f - 1.0f;
  }
}

// ---------------------------------------------------------------- (a) calibration
template <int U>
__global__ __launch_bounds__(256) void cal_rows128(const float* __restrict__ tab, const int64_t* __restrict__ idx,
                                                   int64_t n, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, q = lane & 7, j = lane >> 3;
  const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  f32x4 acc = {0, 0, 0, 0};
  for (int64_t p0 = gw * 8 * U; p0 < n; p0 += nw * 8 * U) {
    int64_t r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + 8 * u + j;
      r[u] = p < n ? idx[p] : -1;
    }
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = r[u] >= 0 ? *reinterpret_cast<const f32x4*>(tab + r[u] * 32 + 4 * q) : (f32x4){0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) sink[0] = 1.f;
}

template <int U>
__global__ __launch_bounds__(256) void cal_rows64(const float* __restrict__ tab, const int64_t* __restrict__ idx,
                                                  int64_t n, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, q = lane & 3, j = lane >> 2;  // 16 rows x 4 quads
  const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  f32x4 acc = {0, 0, 0, 0};
  for (int64_t p0 = gw * 16 * U; p0 < n; p0 += nw * 16 * U) {
    int64_t r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + 16 * u + j;
      r[u] = p < n ? idx[p] : -1;
    }
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = r[u] >= 0 ? *reinterpret_cast<const f32x4*>(tab + r[u] * 32 + 4 * q) : (f32x4){0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) sink[0] = 1.f;
}

template <int U>
__global__ __launch_bounds__(256) void cal_word4(const float* __restrict__ tab, const int64_t* __restrict__ idx,
                                                 int64_t n, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  float acc = 0.f;
  for (int64_t p0 = gw * 64 * U; p0 < n; p0 += nw * 64 * U) {
    int64_t r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + 64 * u + lane;
      r[u] = p < n ? idx[p] : -1;
    }
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = r[u] >= 0 ? tab[r[u] * 32] : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc == 12345.f) sink[0] = 1.f;
}

// index stream alone (the calibration kernels' index reads, to subtract)
__global__ __launch_bounds__(256) void cal_index_only(const int64_t* __restrict__ idx, int64_t n,
                                                      float* __restrict__ sink) {
  int64_t acc = 0;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) acc += idx[p];
  if (acc == 1234567) sink[0] = 1.f;
}

// ---------------------------------------------------------------- (b) copy
template <int U>
__global__ __launch_bounds__(256) void copy_u(const f32x4* __restrict__ a, f32x4* __restrict__ o, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      v[u] = i < n ? __builtin_nontemporal_load(a + i) : (f32x4){0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n) __builtin_nontemporal_store(v[u], o + i);
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_u(const f32x4* __restrict__ a, int64_t n, float* __restrict__ sink) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  f32x4 acc = {0, 0, 0, 0};
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      v[u] = i < n ? a[i] : (f32x4){0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) sink[0] = 1.f;
}

// ---------------------------------------------------------------- (c) gather variants
struct Tabs {
  const float* second[32];
  const float* first[32];
  const float* packed[32];
  const int64_t* idx[32];
};

// one wave per sample (round-5 fm_gather_kernel structure): lane = (field slot j of 8, quad q)
template <bool PACKED>
__global__ __launch_bounds__(256) void sm_gather(Tabs t, int64_t batch, float* __restrict__ deep,
                                                 float* __restrict__ fm1, float* __restrict__ fm2) {
  constexpr int J = 64 / G, NI = (F + J - 1) / J;
  const int lane = threadIdx.x & 63, q = lane % G, j = lane / G;
  const int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (b >= batch) return;
  f32x4 v[NI];
  float w1[NI];
  int64_t r[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int f = i * J + j;
    r[i] = f < F ? t.idx[f][b] : 0;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int f = i * J + j < F ? i * J + j : F - 1;
    const float* row = PACKED ? t.packed[f] + r[i] * RS : t.second[f] + r[i] * D;
    v[i] = *reinterpret_cast<const f32x4*>(row + 4 * q);
    w1[i] = q == 0 ? (PACKED ? row[D] : t.first[f][r[i]]) : 0.f;
  }
  f32x4 s = {0, 0, 0, 0}, sq = {0, 0, 0, 0};
  float fo = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int f = i * J + j;
    if (f < F) {
      *reinterpret_cast<f32x4*>(deep + b * (F * D) + f * D + 4 * q) = v[i];
      s += v[i];
      sq += v[i] * v[i];
      fo += w1[i];
    }
  }
#pragma unroll
  for (int o = G; o < 64; o <<= 1) {
    s.x += __shfl_xor(s.x, o, 64);
    s.y += __shfl_xor(s.y, o, 64);
    s.z += __shfl_xor(s.z, o, 64);
    s.w += __shfl_xor(s.w, o, 64);
    sq.x += __shfl_xor(sq.x, o, 64);
    sq.y += __shfl_xor(sq.y, o, 64);
    sq.z += __shfl_xor(sq.z, o, 64);
    sq.w += __shfl_xor(sq.w, o, 64);
    fo += __shfl_xor(fo, o, 64);
  }
  float part = (s.x * s.x - sq.x) + (s.y * s.y - sq.y) + (s.z * s.z - sq.z) + (s.w * s.w - sq.w);
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if (lane == 0) {
    fm2[b] = 0.5f * part;
    fm1[b] = fo;
  }
}

// field-major: a wave owns 8 samples (lane = sample slot j, quad q) and walks the fields in order,
// U fields in flight (indices of the U fields first, then their rows).  NTS: nontemporal deep_in
// stores; PF: the next round's indices issued before this round's rows are consumed.
template <int U, bool PACKED, int WPB, bool NTS = false, bool PF = false>
__global__ __launch_bounds__(64 * WPB) void fmaj_gather(Tabs t, int64_t batch, float* __restrict__ deep,
                                                        float* __restrict__ fm1, float* __restrict__ fm2) {
  const int lane = threadIdx.x & 63, q = lane & 7, j = lane >> 3;
  const int64_t b = (((int64_t)blockIdx.x * 64 * WPB + threadIdx.x) >> 6) * 8 + j;
  const bool live = b < batch;
  const int64_t bb = live ? b : 0;
  f32x4 s = {0, 0, 0, 0}, sq = {0, 0, 0, 0};
  float fo = 0.f;
  int64_t r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) r[u] = u < F ? t.idx[u][bb] : 0;
  for (int f0 = 0; f0 < F; f0 += U) {
    if (!PF && f0 > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = f0 + u < F ? t.idx[f0 + u][bb] : 0;
    }
    f32x4 v[U];
    float w1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = f0 + u < F ? f0 + u : F - 1;
      const float* row = PACKED ? t.packed[f] + r[u] * RS : t.second[f] + r[u] * D;
      v[u] = *reinterpret_cast<const f32x4*>(row + 4 * q);
      w1[u] = q == 0 ? (PACKED ? row[D] : t.first[f][r[u]]) : 0.f;
    }
    if (PF) {
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = f0 + U + u < F ? t.idx[f0 + U + u][bb] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (f0 + u < F) {
        if (live) {
          f32x4* o = reinterpret_cast<f32x4*>(deep + b * (F * D) + (f0 + u) * D + 4 * q);
          if (NTS)
            __builtin_nontemporal_store(v[u], o);
          else
            *o = v[u];
        }
        s += v[u];
        sq += v[u] * v[u];
        fo += w1[u];
      }
    }
  }
  float part = (s.x * s.x - sq.x) + (s.y * s.y - sq.y) + (s.z * s.z - sq.z) + (s.w * s.w - sq.w);
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) part += __shfl_xor(part, o, 64);
  if (live && q == 0) {
    fm2[b] = 0.5f * part;
    fm1[b] = fo;
  }
}

// ---------------------------------------------------------------- driver
template <typename L>
float time_ms(L launch, int iters = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

static const char* g_only = nullptr;
static bool want(const char* name) { return !g_only || strstr(name, g_only); }

int main(int argc, char** argv) {
  if (argc > 1) g_only = argv[1];
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float* sink;
  CK(hipMalloc(&sink, 256));
  // ---------------- (a) calibration
  {
    const int64_t R = 1ll << 24;  // 16.7 M rows x 128 B = 2 GiB
    const int64_t N = 1ll << 21;  // distinct rows read
    float* tab;
    int64_t* idx;
    CK(hipMalloc(&tab, (size_t)R * 128));
    CK(hipMemset(tab, 0, (size_t)R * 128));
    if (getenv("RANDOM")) fill_hash<<<4096, 256>>>(tab, R * 32, 4u);
    CK(hipMalloc(&idx, (size_t)N * 8));
    std::vector<int64_t> h(R);
    std::iota(h.begin(), h.end(), 0);
    std::mt19937_64 rng(7);
    for (int64_t i = 0; i < N; ++i) std::swap(h[i], h[i + (int64_t)(rng() % (uint64_t)(R - i))]);
    CK(hipMemcpy(idx, h.data(), (size_t)N * 8, hipMemcpyHostToDevice));
    const unsigned grid = (unsigned)(cus * 8);  // 32 waves per CU
    auto rep = [&](const char* name, float ms, double bytes) {
      printf("cal %-22s %8.2f us  %8.1f GB/s of %.1f MB known bytes (+%.1f MB indices)  %.1f Mrows/s\n", name,
             ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / 1e6, N * 8 / 1e6, N / (ms * 1e-3) / 1e6);
    };
    if (want("cal_rows128")) rep("cal_rows128<4>", time_ms([&] { cal_rows128<4><<<grid, 256>>>(tab, idx, N, sink); }), N * 128.0);
    if (want("cal_rows128")) rep("cal_rows128<8>", time_ms([&] { cal_rows128<8><<<grid, 256>>>(tab, idx, N, sink); }), N * 128.0);
    if (want("cal_rows64")) rep("cal_rows64<4>", time_ms([&] { cal_rows64<4><<<grid, 256>>>(tab, idx, N, sink); }), N * 64.0);
    if (want("cal_word4")) rep("cal_word4<4>", time_ms([&] { cal_word4<4><<<grid, 256>>>(tab, idx, N, sink); }), N * 4.0);
    if (want("cal_word4")) rep("cal_word4<8>", time_ms([&] { cal_word4<8><<<grid, 256>>>(tab, idx, N, sink); }), N * 4.0);
    if (want("cal_index")) rep("cal_index_only", time_ms([&] { cal_index_only<<<grid, 256>>>(idx, N, sink); }), 0.0);
    CK(hipFree(tab));
    CK(hipFree(idx));
  }
  // ---------------- (b) copy ceiling
  if (want("copy") || want("read")) {
    const int64_t n = (2ll << 30) / 16;
    f32x4 *a, *o;
    CK(hipMalloc(&a, (size_t)n * 16));
    CK(hipMalloc(&o, (size_t)n * 16));
    CK(hipMemset(a, 0, (size_t)n * 16));
    CK(hipMemset(o, 0, (size_t)n * 16));
    if (getenv("RANDOM")) fill_hash<<<4096, 256>>>((float*)a, n * 4, 5u);
    for (int mult : {4, 8, 16}) {
      const unsigned grid = (unsigned)(cus * mult);
      float ms = time_ms([&] { copy_u<4><<<grid, 256>>>(a, o, n); }, 10);
      printf("copy 2 GiB -> 2 GiB  U4 grid %5u: %8.1f GB/s (read + write)\n", grid, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
      ms = time_ms([&] { copy_u<8><<<grid, 256>>>(a, o, n); }, 10);
      printf("copy 2 GiB -> 2 GiB  U8 grid %5u: %8.1f GB/s (read + write)\n", grid, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
      ms = time_ms([&] { copy_u<2><<<grid, 256>>>(a, o, n); }, 10);
      printf("copy 2 GiB -> 2 GiB  U2 grid %5u: %8.1f GB/s (read + write)\n", grid, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
      ms = time_ms([&] { read_u<4><<<grid, 256>>>(a, n, sink); }, 10);
      printf("read 2 GiB           U4 grid %5u: %8.1f GB/s\n", grid, 1.0 * n * 16 / (ms * 1e-3) / 1e9);
    }
    CK(hipFree(a));
    CK(hipFree(o));
  }
  // ---------------- (c) gather variants
  {
    const int64_t V = 1000000, Bmax = 65536;
    float *second, *first, *packed, *deep, *f1, *f2;
    int64_t* idx;
    CK(hipMalloc(&second, (size_t)F * V * D * 4));
    CK(hipMalloc(&first, (size_t)F * V * 4));
    CK(hipMalloc(&packed, (size_t)F * V * RS * 4));
    CK(hipMalloc(&idx, (size_t)F * Bmax * 8));
    CK(hipMalloc(&deep, (size_t)Bmax * F * D * 4));
    CK(hipMalloc(&f1, Bmax * 4));
    CK(hipMalloc(&f2, Bmax * 4));
    CK(hipMemset(second, 0, (size_t)F * V * D * 4));
    CK(hipMemset(first, 0, (size_t)F * V * 4));
    CK(hipMemset(packed, 0, (size_t)F * V * RS * 4));
    if (getenv("RANDOM")) {  // non-zero contents (does the data change the rate?)
      fill_hash<<<4096, 256>>>(second, (int64_t)F * V * D, 1u);
      fill_hash<<<4096, 256>>>(first, (int64_t)F * V, 2u);
      fill_hash<<<4096, 256>>>(packed, (int64_t)F * V * RS, 3u);
      CK(hipDeviceSynchronize());
      printf("tables filled with hashed values\n");
    }
    std::vector<int64_t> h((size_t)F * Bmax);
    std::mt19937_64 rng(11);
    for (auto& x : h) x = (int64_t)(rng() % (uint64_t)V);
    CK(hipMemcpy(idx, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    Tabs t;
    for (int f = 0; f < 32; ++f) {
      const int ff = f < F ? f : 0;
      t.second[f] = second + (size_t)ff * V * D;
      t.first[f] = first + (size_t)ff * V;
      t.packed[f] = packed + (size_t)ff * V * RS;
      t.idx[f] = idx + (size_t)ff * Bmax;
    }
    const double bps = 30.0 * (8 + 128 + 4) + 30 * 128 + 8;
    for (int64_t B : {(int64_t)4096, Bmax}) {
      auto rep = [&](const char* name, float ms) {
        printf("gather B %6ld %-26s %8.2f us  %7.1f GB/s alg  (%.3f of 8 TB/s)\n", (long)B, name, ms * 1e3,
               bps * B / (ms * 1e-3) / 1e9, bps * B / (ms * 1e-3) / 8e12);
      };
      const unsigned gs = (unsigned)((B + 3) / 4);
      if (want("sm_tables")) rep("sm_tables", time_ms([&] { sm_gather<false><<<gs, 256>>>(t, B, deep, f1, f2); }));
      if (want("sm_packed")) rep("sm_packed", time_ms([&] { sm_gather<true><<<gs, 256>>>(t, B, deep, f1, f2); }));
      const unsigned g4 = (unsigned)((B / 8 + 3) / 4), g1 = (unsigned)(B / 8);
#define FM_CASE(UU, PK, WPB, GRID, NAME, ...) \
  if (want(NAME)) rep(NAME, time_ms([&] { fmaj_gather<UU, PK, WPB, ##__VA_ARGS__><<<GRID, 64 * WPB>>>(t, B, deep, f1, f2); }));
      FM_CASE(3, false, 4, g4, "fm3_tables")
      FM_CASE(5, false, 4, g4, "fm5_tables")
      FM_CASE(6, false, 4, g4, "fm6_tables")
      FM_CASE(10, false, 4, g4, "fm10_tables")
      FM_CASE(5, false, 4, g4, "fm5_tables_nts", true, false)
      FM_CASE(5, false, 4, g4, "fm5_tables_pf", false, true)
      FM_CASE(5, false, 4, g4, "fm5_tables_nts_pf", true, true)
      FM_CASE(6, false, 4, g4, "fm6_tables_nts_pf", true, true)
      FM_CASE(10, false, 4, g4, "fm10_tables_nts_pf", true, true)
      FM_CASE(5, false, 1, g1, "fm5_tables_w1_nts_pf", true, true)
      FM_CASE(5, false, 2, (unsigned)((B / 8 + 1) / 2), "fm5_tables_w2_nts_pf", true, true)
      FM_CASE(10, true, 4, g4, "fm10_packed")
#undef FM_CASE
    }
  }
  return 0;
}
