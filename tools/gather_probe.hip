// Embedding-gather ceiling probe (DeepFM configs[1] shape): 30 fields x 1e6 rows x 32 fp32
// second-order tables + 30 x 1e6 first-order weights, batch B, deep_in [B, 960] written.
// Times kernel variants with hipEvents and prints algorithmic GB/s (8,048 B/sample basis).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_probe.hip -o tools/bin/gather_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
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
constexpr int F = 30, D = 32, G = 8;

struct Tabs {
  const float* second[32];
  const float* first[32];
  const int64_t* idx[32];
};

// Variant knobs: UNI = wave index made uniform (scalar pointer loads); FIRST = load first-order
// weights; FM = compute sums + LDS reduction; NT = nontemporal row loads / deep_in stores.
template <bool UNI, bool FIRST, bool FM, bool NT>
__global__ __launch_bounds__(256) void fm_probe(Tabs t, int64_t batch, float* __restrict__ deep_in,
                                                float* __restrict__ fm1, float* __restrict__ fm2) {
  constexpr int SPW = 64 / G;
  __shared__ float red[4][9][64];
  const int lane = threadIdx.x & 63;
  const int wave = UNI ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : (threadIdx.x >> 6);
  const int q = lane % G;
  const int64_t b = (int64_t)blockIdx.x * SPW + lane / G;
  constexpr int FPW = 8;
  f32x4 s = {0, 0, 0, 0}, sq = {0, 0, 0, 0};
  float fo = 0.f;
  const float* rp[FPW];
  const float* wp[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int f = wave + 4 * j;
    const int64_t r = f < F ? t.idx[f][b] : 0;
    rp[j] = f < F ? t.second[f] + r * D : nullptr;
    wp[j] = (FIRST && f < F && q == 0) ? t.first[f] + r : nullptr;
  }
  f32x4 v[FPW];
  float w1[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    if (rp[j]) {
      const f32x4* p = reinterpret_cast<const f32x4*>(rp[j] + 4 * q);
      v[j] = NT ? __builtin_nontemporal_load(p) : *p;
    } else {
      v[j] = (f32x4){0, 0, 0, 0};
    }
    w1[j] = wp[j] ? wp[j][0] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int f = wave + 4 * j;
    if (f < F) {
      f32x4* o = reinterpret_cast<f32x4*>(deep_in + b * (F * D) + f * D + 4 * q);
      if (NT)
        __builtin_nontemporal_store(v[j], o);
      else
        *o = v[j];
      s += v[j];
      sq += v[j] * v[j];
      fo += w1[j];
    }
  }
  if (!FM) {
    if (q == 0 && wave == 0) fm1[b] = fo + s.x + sq.y;
    return;
  }
  red[wave][0][lane] = s.x;
  red[wave][1][lane] = s.y;
  red[wave][2][lane] = s.z;
  red[wave][3][lane] = s.w;
  red[wave][4][lane] = sq.x;
  red[wave][5][lane] = sq.y;
  red[wave][6][lane] = sq.z;
  red[wave][7][lane] = sq.w;
  red[wave][8][lane] = fo;
  __syncthreads();
  if (wave != 0) return;
  float S[4] = {0, 0, 0, 0}, Q[4] = {0, 0, 0, 0}, FO = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      S[c] += red[w][c][lane];
      Q[c] += red[w][4 + c][lane];
    }
    FO += red[w][8][lane];
  }
  float part = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) part += S[c] * S[c] - Q[c];
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if (q == 0) {
    fm2[b] = 0.5f * part;
    fm1[b] = FO;
  }
}

// Flattened variant: a wave walks (sample, field) pairs in deep_in order, 8 pairs per
// instruction, U instructions in flight; no FM (pure gather + contiguous write ceiling).
template <int U>
__global__ __launch_bounds__(256) void flat_probe(Tabs t, int64_t batch, float* __restrict__ deep_in) {
  const int lane = threadIdx.x & 63, q = lane & 7, r = lane >> 3;
  const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t p0 = gw * (8 * U);
  const int64_t np = batch * F;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t p = p0 + 8 * u + r;
    v[u] = (f32x4){0, 0, 0, 0};
    if (p < np) {
      const int64_t b = p / F;
      const int f = (int)(p - b * F);
      const int64_t row = t.idx[f][b];
      v[u] = *reinterpret_cast<const f32x4*>(t.second[f] + row * D + 4 * q);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t p = p0 + 8 * u + r;
    if (p < np) *reinterpret_cast<f32x4*>(deep_in + p * D + 4 * q) = v[u];
  }
}


// Sample-major: lane = (field slot j, quad q), a wave walks one sample per NS-step with its
// fields 8 per instruction; the sample's 3,840-B deep_in row is written contiguously; FM sums
// reduced across field slots by xor-shuffles (no LDS, no barrier).
template <int NS>
__global__ __launch_bounds__(256) void sm_probe(Tabs t, int64_t batch, float* __restrict__ deep_in,
                                                float* __restrict__ fm1, float* __restrict__ fm2) {
  constexpr int J = 64 / G, NI = (F + J - 1) / J;
  const int lane = threadIdx.x & 63, q = lane % G, j = lane / G;
  const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  for (int64_t b0 = gw * NS; b0 < batch; b0 += nw * NS) {
    f32x4 v[NS][NI];
    float w1[NS][NI];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int64_t b = b0 + n;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int f = i * J + j;
        const bool ok = b < batch && f < F;
        const int64_t r = ok ? t.idx[f][b] : 0;
        v[n][i] = ok ? *reinterpret_cast<const f32x4*>(t.second[f] + r * D + 4 * q) : (f32x4){0, 0, 0, 0};
        w1[n][i] = (ok && q == 0) ? t.first[f][r] : 0.f;
      }
    }
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int64_t b = b0 + n;
      f32x4 s = {0, 0, 0, 0}, sq = {0, 0, 0, 0};
      float fo = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int f = i * J + j;
        if (b < batch && f < F) *reinterpret_cast<f32x4*>(deep_in + b * (F * D) + f * D + 4 * q) = v[n][i];
        s += v[n][i];
        sq += v[n][i] * v[n][i];
        fo += w1[n][i];
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
      if (lane == 0 && b < batch) {
        fm2[b] = 0.5f * part;
        fm1[b] = fo;
      }
    }
  }
}

__global__ void copy_probe(const f32x4* __restrict__ a, f32x4* __restrict__ o, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = a[i];
}

template <typename L>
float time_ms(L launch, int iters = 30) {
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

int main(int argc, char** argv) {
  const int64_t V = 1000000;
  float *second, *first, *deep, *f1, *f2;
  int64_t* idx;
  const int64_t Bmax = 65536;
  CK(hipMalloc(&second, (size_t)F * V * D * 4));
  CK(hipMalloc(&first, (size_t)F * V * 4));
  CK(hipMalloc(&idx, (size_t)F * Bmax * 8));
  CK(hipMalloc(&deep, (size_t)Bmax * F * D * 4));
  CK(hipMalloc(&f1, Bmax * 4));
  CK(hipMalloc(&f2, Bmax * 4));
  CK(hipMemset(second, 0, (size_t)F * V * D * 4));
  CK(hipMemset(first, 0, (size_t)F * V * 4));
  const double bytes_per_sample = 30.0 * (8 + 128 + 4) + 30 * 128 + 8;
  for (int64_t span : {V}) {
    std::vector<int64_t> h((size_t)F * Bmax);
    srand(7);
    for (auto& x : h) x = (int64_t)(((uint64_t)rand() * 2654435761ull + rand()) % (uint64_t)span);
    CK(hipMemcpy(idx, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    Tabs t;
    for (int f = 0; f < 32; ++f) {
      const int ff = f < F ? f : 0;
      t.second[f] = second + (size_t)ff * V * D;
      t.first[f] = first + (size_t)ff * V;
      t.idx[f] = idx + (size_t)ff * Bmax;
    }
    for (int64_t B : {(int64_t)4096, Bmax}) {
      const unsigned blocks = (unsigned)(B / 8);
      auto rep = [&](const char* name, float ms) {
        printf("span %7ld B %6ld %-28s %8.2f us  %7.1f GB/s alg  (%.3f of 8 TB/s)\n", (long)span, (long)B, name,
               ms * 1e3, bytes_per_sample * B / (ms * 1e-3) / 1e9, bytes_per_sample * B / (ms * 1e-3) / 8e12);
      };
      rep("current", time_ms([&] { fm_probe<false, true, true, false><<<blocks, 256>>>(t, B, deep, f1, f2); }));
      rep("uniform-wave", time_ms([&] { fm_probe<true, true, true, false><<<blocks, 256>>>(t, B, deep, f1, f2); }));
      rep("uniform+nt", time_ms([&] { fm_probe<true, true, true, true><<<blocks, 256>>>(t, B, deep, f1, f2); }));
      rep("no-first-order", time_ms([&] { fm_probe<true, false, true, false><<<blocks, 256>>>(t, B, deep, f1, f2); }));
      rep("no-fm-reduce", time_ms([&] { fm_probe<true, true, false, false><<<blocks, 256>>>(t, B, deep, f1, f2); }));
      for (int wpc : {32, 64, 1 << 20}) {
        const unsigned g1 = (unsigned)std::min<int64_t>((B + 3) / 4, 256 * wpc / 4);
        const unsigned g2 = (unsigned)std::min<int64_t>((B / 2 + 3) / 4, 256 * wpc / 4);
        char nm[64];
        snprintf(nm, sizeof nm, "sample-major NS1 w/CU %d", wpc);
        rep(nm, time_ms([&] { sm_probe<1><<<g1, 256>>>(t, B, deep, f1, f2); }));
        snprintf(nm, sizeof nm, "sample-major NS2 w/CU %d", wpc);
        rep(nm, time_ms([&] { sm_probe<2><<<g2, 256>>>(t, B, deep, f1, f2); }));
      }
      rep("flat U4 (rows only)", time_ms([&] {
            flat_probe<4><<<(unsigned)((B * F / 32 + 3) / 4), 256>>>(t, B, deep);
          }));
      rep("flat U8 (rows only)", time_ms([&] {
            flat_probe<8><<<(unsigned)((B * F / 64 + 3) / 4), 256>>>(t, B, deep);
          }));
    }
  }
  // streaming copy reference: 2 x 1 GiB
  const int64_t n = (1ll << 30) / 16;
  float ms = time_ms([&] { copy_probe<<<4096, 256>>>((const f32x4*)second, (f32x4*)(second + (size_t)4 * n), n); }, 10);
  printf("copy 1 GiB -> 1 GiB: %.1f GB/s (read+write)\n", 2.0 * n * 16 / (ms * 1e-3) / 1e9);
  return 0;
}
