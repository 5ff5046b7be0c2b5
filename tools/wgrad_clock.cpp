// Diagnostic: per-workgroup s_memtime / s_memrealtime stamps of rk_gemm_wgrad at the BST shape
// (N = K = 128, R = 131072): effective clock, workgroup start spread and durations.
// Build: hipcc --offload-arch=gfx950 -O3 -DRK_WGRAD_STAMP -I<csrc> tools/wgrad_clock.cpp <csrc>/wgrad.hip <csrc>/runtime.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
extern "C" int rk_gemm_wgrad(int64_t, int64_t, int64_t, const float*, int64_t, const float*, const float*, int64_t,
                             float*, int64_t, float*, int32_t, float*, int64_t, void*);
extern "C" int64_t rk_gemm_wgrad_workspace_floats(int64_t, int64_t, int64_t);
namespace rk { __device__ uint64_t g_wgrad_stamp[4 * 4096]; }
int main() {
  const int64_t N = 128, K = 128, R = 131072;
  float *A, *B, *C, *db, *ws;
  (void)hipMalloc(&A, R * N * 4); (void)hipMalloc(&B, R * K * 4); (void)hipMalloc(&C, N * K * 4);
  (void)hipMalloc(&db, N * 4);
  const int64_t nws = rk_gemm_wgrad_workspace_floats(N, K, R);
  (void)hipMalloc(&ws, nws * 4);
  (void)hipMemset(A, 0, R * N * 4); (void)hipMemset(B, 0, R * K * 4);
  for (int i = 0; i < 200; ++i) rk_gemm_wgrad(N, K, R, A, N, nullptr, B, K, C, K, db, 0, ws, nws, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint64_t> st(4 * 4096);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(rk::g_wgrad_stamp), st.size() * 8);
  int n = 0;
  uint64_t rmin = ~0ull;
  for (int b = 0; b < 4096; ++b) if (st[4 * b + 2]) { rmin = std::min(rmin, st[4 * b + 2]); ++n; }
  std::vector<double> clk, dur, start;
  for (int b = 0; b < n; ++b) {
    const double dt = (double)(st[4 * b + 1] - st[4 * b]), dr = (double)(st[4 * b + 3] - st[4 * b + 2]);
    clk.push_back(dt / dr * 0.1);  // GHz (realtime at 100 MHz)
    dur.push_back(dr * 0.01);      // us
    start.push_back((st[4 * b + 2] - rmin) * 0.01);
  }
  std::sort(clk.begin(), clk.end()); std::sort(dur.begin(), dur.end()); std::sort(start.begin(), start.end());
  printf("workgroups %d\nclock GHz  min %.2f med %.2f max %.2f\nduration us min %.1f med %.1f max %.1f\n", n, clk[0],
         clk[n / 2], clk[n - 1], dur[0], dur[n / 2], dur[n - 1]);
  printf("start offset us: p10 %.1f p50 %.1f p90 %.1f max %.1f\n", start[n / 10], start[n / 2], start[9 * n / 10],
         start[n - 1]);
  return 0;
}
