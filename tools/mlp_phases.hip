// Per-layer cycle breakdown of mlp_kernel (rk_mlp_forward) on random packed weights.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DRK_MLP_PHASES -I include -I <pkg>/csrc \
//     tools/mlp_phases.hip <pkg>/csrc/runtime.hip -o tools/bin/mlp_phases
// Shapes: dcn (64->512->256->128, ReLU, head), deepfm (960->512->256->128, BN+ReLU, head),
// batch 4096.  Prints, per layer, the average cycles (wave 0 of each workgroup) from the layer's
// start to: MFMA loop done, epilogue stored, barrier passed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "mlp.hip"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
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

static void run_shape(const char* name, int K0, std::vector<int> widths, bool bn, int64_t M) {
  std::mt19937 g(7);
  float* x = dev_random((size_t)M * K0, 1.f, g);
  std::vector<rk_mlp_layer> L(widths.size());
  int K = K0;
  for (size_t l = 0; l < widths.size(); ++l) {
    const int n = widths[l];
    float* w = dev_random((size_t)n * K, 0.05f, g);
    int64_t rows, cols;
    rk_mlp_packed_size(n, K, &rows, &cols);
    float* packed;
    CK(hipMalloc(&packed, rows * cols * 4));
    rk_mlp_pack_weight(w, K, n, K, packed, nullptr);
    L[l] = {};
    L[l].w = packed;
    L[l].ldw = cols;
    L[l].n = n;
    L[l].act = RK_ACT_RELU;
    L[l].bias = dev_random(n, 0.1f, g);
    if (bn) {
      L[l].pre_scale = dev_random(n, 1.f, g);
      L[l].pre_shift = dev_random(n, 0.1f, g);
    }
    K = n;
  }
  rk_epilogue head = {};
  head.head_w = dev_random(K, 0.1f, g);
  head.head_b = dev_random(1, 0.1f, g);
  float *logit, *prob;
  CK(hipMalloc(&logit, M * 4));
  CK(hipMalloc(&prob, M * 4));
  head.head_logit = logit;
  head.head_prob = prob;
  auto run = [&]() {
    if (rk_mlp_forward(x, K0, M, K0, L.data(), (int)L.size(), &head, nullptr, 0, nullptr)) {
      fprintf(stderr, "rk_mlp_forward: %s\n", rk_last_error());
      exit(1);
    }
  };
  run();
  CK(hipDeviceSynchronize());
  unsigned long long zero[3 * RK_MLP_MAX_LAYERS + 2] = {0};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rk::g_mlp_phase), zero, sizeof(zero)));
  const int iters = 20;
  // single-launch wall span of the grid (first workgroup start -> last workgroup end)
  unsigned long long span0[5] = {~0ull, 0, 0, 0, 0};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rk::g_mlp_span), span0, sizeof(span0)));
  run();
  CK(hipDeviceSynchronize());
  unsigned long long span[5];
  CK(hipMemcpyFromSymbol(span, HIP_SYMBOL(rk::g_mlp_span), sizeof(span)));
  {
    static unsigned wg[8192][4];
    CK(hipMemcpyFromSymbol(wg, HIP_SYMBOL(rk::g_mlp_wg), sizeof(wg)));
    const int64_t n = (M + 15) / 16;
    // CU key = XCC_ID and HW_ID bits [15:8] (cu, sh, se); count workgroups per CU
    std::vector<int> per(8 * 256, 0);
    for (int64_t i = 0; i < n && i < 8192; ++i) per[(wg[i][1] & 7) * 256 + ((wg[i][0] >> 8) & 0xFF)]++;
    int cus_used = 0, shared = 0;
    for (int c : per) {
      cus_used += c > 0;
      shared += c > 1 ? c : 0;
    }
    double d_alone = 0, d_shared = 0;
    int n_alone = 0, n_shared = 0;
    for (int64_t i = 0; i < n && i < 8192; ++i) {
      const bool sh = per[(wg[i][1] & 7) * 256 + ((wg[i][0] >> 8) & 0xFF)] > 1;
      (sh ? d_shared : d_alone) += wg[i][2] / 100.0;
      (sh ? n_shared : n_alone)++;
    }
    printf("  %d distinct CUs for %lld workgroups; %d workgroups share a CU (mean %.1f us) vs alone (mean %.1f us)\n",
           cus_used, (long long)n, shared, n_shared ? d_shared / n_shared : 0.0, n_alone ? d_alone / n_alone : 0.0);
  }
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rk::g_mlp_phase), zero, sizeof(zero)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) run();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long ph[3 * RK_MLP_MAX_LAYERS + 2];
  CK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(rk::g_mlp_phase), sizeof(ph)));
  const char* rows = getenv("RANKOPS_MLP_ROWS");
  const int64_t wgs = (M + (rows && atoi(rows) == 32 ? 31 : 15)) / (rows && atoi(rows) == 32 ? 32 : 16);
  printf("%s: M=%lld  %.1f us/launch  (%lld workgroups), grid span %.1f us, last workgroup starts at %.1f us\n",
         name, (long long)M, 1e3 * ms / iters, (long long)wgs, (span[1] - span[0]) / 100.0, (span[2] - span[0]) / 100.0);
  printf("  workgroup wall time: mean %.1f us, max %.1f us\n", span[4] / 100.0 / wgs, span[3] / 100.0);
  printf("  input staged %7.0f cycles, workgroup total %7.0f cycles\n",
         ph[3 * RK_MLP_MAX_LAYERS] / ((double)iters * wgs), ph[3 * RK_MLP_MAX_LAYERS + 1] / ((double)iters * wgs));
  for (size_t l = 0; l < widths.size(); ++l) {
    const double d = (double)iters * wgs;
    printf("  layer %zu (n=%d): loop %7.0f  epilogue %7.0f  barrier %7.0f cycles\n", l, widths[l], ph[3 * l] / d,
           ph[3 * l + 1] / d, ph[3 * l + 2] / d);
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("%d CUs\n", cus);
  run_shape("dcn", 50, {512, 256, 128}, false, 4096);
  run_shape("dcn-2k", 50, {512, 256, 128}, false, 2048);
  run_shape("deepfm", 960, {512, 256, 128}, true, 4096);
  return 0;
}
