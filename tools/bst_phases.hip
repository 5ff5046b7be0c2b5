// Per-phase cycle breakdown of bst_block_kernel (rk_bst_forward_blocks) on random data.
// Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DRK_BST_PHASES -I include \
//     -I <pkg>/csrc tools/bst_phases.hip <pkg>/csrc/runtime.hip <pkg>/csrc/bst_small.hip <pkg>/csrc/mlp.hip \
//     -o tools/bin/bst_phases && tools/bin/bst_phases
// Phases (thread 0, cycles between consecutive barriers, summed over workgroups):
//   0 gather | 1 V | 2 Q/K | 3 attention | 4 O-proj | 5 LN1 | 6 FFN1 | 7 FFN2 | 8 LN2 + pooling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "bst_block.hip"

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static float* dev_random(size_t n, float scale, std::mt19937& g) {
  std::normal_distribution<float> d(0.f, scale);
  std::vector<float> h(n);
  for (auto& v : h) v = d(g);
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 2048;
  const int T = 64, D = 128, V = 100000, iters = 20;
  std::mt19937 g(1);
  float* table = dev_random((size_t)V * D, 1.f, g);
  std::vector<int64_t> seq(B * T), len(B);
  std::uniform_int_distribution<int64_t> ri(0, V - 1), rl(1, T);
  for (auto& v : seq) v = ri(g);
  for (auto& v : len) v = rl(g);
  int64_t *dseq, *dlen;
  CK(hipMalloc(&dseq, seq.size() * 8));
  CK(hipMalloc(&dlen, len.size() * 8));
  CK(hipMemcpy(dseq, seq.data(), seq.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlen, len.data(), len.size() * 8, hipMemcpyHostToDevice));
  const float* params[17];
  params[0] = dev_random((size_t)(T + 1) * D, 1.f, g);
  for (int k = 1; k <= 12; ++k) params[k] = dev_random((k % 2) ? (size_t)D * D : D, 0.09f, g);
  for (int k = 13; k < 17; ++k) params[k] = dev_random(D, 0.2f, g);
  const float scalars[3] = {1e-5f, 1e-5f, 0.01f};
  float* pool;
  CK(hipMalloc(&pool, (size_t)B * D * 4));
  auto run = [&]() {
    if (rk_bst_forward_blocks(table, V, D, dseq, T, T, dlen, B, D, 4, 1, params, scalars, pool, D, 0, nullptr)) {
      fprintf(stderr, "launch failed: %s\n", rk_last_error());
      exit(1);
    }
  };
  run();
  CK(hipDeviceSynchronize());
#ifdef RK_BST_PHASES
  unsigned long long zero[16] = {0};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rk::g_bst_phase), zero, sizeof(zero)));
  unsigned long long zw[80] = {0};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rk::g_bst_wave), zw, sizeof(zw)));
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) run();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("batch %lld  %.1f us/launch\n", (long long)B, 1e3 * ms / iters);
#ifdef RK_BST_PHASES
  unsigned long long ph[16];
  CK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(rk::g_bst_phase), sizeof(ph)));
  const char* names[9] = {"gather", "v_proj", "qk_proj", "attention", "o_proj", "ln1", "ffn1", "ffn2", "ln2+pool"};
  unsigned long long tot = 0;
  for (int i = 0; i < 9; ++i) tot += ph[i];
  for (int i = 0; i < 9; ++i)
    printf("  %-10s %8.0f cycles/WG  %5.1f%%\n", names[i], (double)ph[i] / (iters * B), 100.0 * ph[i] / tot);
  printf("  total      %8.0f cycles/WG\n", (double)tot / (iters * B));
  unsigned long long wv[10][8];
  CK(hipMemcpyFromSymbol(wv, HIP_SYMBOL(rk::g_bst_wave), sizeof(wv)));
  const char* marks[5] = {"v_proj", "qk_proj", "o_proj", "ffn1", "ffn2"};
  const int mp[5] = {1, 2, 4, 6, 7};
  for (int i = 0; i < 5; ++i) {
    printf("  %-10s phase %6.0f, MFMA loop done per wave:", marks[i], (double)ph[mp[i]] / (iters * B));
    for (int w = 0; w < 8; ++w) printf(" %6.0f", (double)wv[i][w] / (iters * B));
    printf("\n  %-10s        %6s  epilogue done (before barrier):", "", "");
    for (int w = 0; w < 8; ++w) printf(" %6.0f", (double)wv[5 + i][w] / (iters * B));
    printf("\n");
  }
#endif
  return 0;
}
