// Layout probe for v_mfma_f32_4x4x1f32 (16 blocks) with CBSZ/ABID broadcast, and for
// v_permlane16_swap / v_permlane32_swap on gfx950: prints which lane's A / B operand lands in which
// output lane/register, so bst_small.hip's operand arrangement can be checked against hardware.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma4_probe.hip -o tools/bin/mfma4_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));

template <int CBSZ, int ABID>
__global__ void probe(float* out, int mode) {
  const int l = threadIdx.x;
  // mode 0: A = lane + 1, B = 1 -> out = the A lane feeding D[i][j]; mode 1: A = 1, B = lane + 1
  const float a = mode == 0 ? (float)(l + 1) : 1.f;
  const float b = mode == 0 ? 1.f : (float)(l + 1);
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, CBSZ, ABID, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

__global__ void swaps(int* out) {
  const int l = threadIdx.x;
  auto p32 = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  auto p16 = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  out[l * 4 + 0] = p32[0];
  out[l * 4 + 1] = p32[1];
  out[l * 4 + 2] = p16[0];
  out[l * 4 + 3] = p16[1];
}

int main() {
  float* d;
  int* di;
  hipMalloc(&d, 256 * sizeof(float));
  hipMalloc(&di, 256 * sizeof(int));
  float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    for (int v = 0; v < 2; ++v) {
      if (v == 0) probe<0, 0><<<1, 64>>>(d, mode);
      else probe<2, 1><<<1, 64>>>(d, mode);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("mode %s, cbsz/abid %s: out lane:reg=src-lane\n", mode ? "B" : "A", v ? "2/1" : "0/0");
      for (int l = 0; l < 64; ++l) {
        printf("%2d:", l);
        for (int r = 0; r < 4; ++r) printf(" %3d", (int)h[l * 4 + r] - 1);
        printf(l % 4 == 3 ? "\n" : " |");
      }
    }
  }
  swaps<<<1, 64>>>(di);
  int hi[256];
  hipMemcpy(hi, di, sizeof(hi), hipMemcpyDeviceToHost);
  printf("permlane swaps (vdst = lane, vsrc = 100 + lane): lane: p32[0] p32[1] p16[0] p16[1]\n");
  for (int l = 0; l < 64; ++l) printf("%2d: %3d %3d %3d %3d%s", l, hi[4 * l], hi[4 * l + 1], hi[4 * l + 2], hi[4 * l + 3], l % 4 == 3 ? "\n" : " | ");
  hipFree(d);
  hipFree(di);
  return 0;
}
