// Latency probe (tools only, not part of the library): cycles from kernel entry until a value read
// through a pointer taken from (a) the kernel-argument block by a per-lane vector load, (b) the
// kernel-argument block by a scalar load, (c) a small device buffer that stays L2-resident across
// launches — the first dependent round trip of the DCN / DeepFM prologues (their segment
// descriptors live in the kernel arguments).  Build: hipcc --offload-arch=gfx950 -O3 -o
// gpurun_out/kernarg_probe tools/kernarg_probe.hip ; run on the box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Args {
  const int64_t* p[8];
  const int64_t* desc;  // device copy of p
  unsigned long long* out;
  int mode;
};

__global__ __launch_bounds__(64) void probe(Args a) {
  const unsigned long long t0 = clock64();
  const int lane = threadIdx.x;
  const int64_t* ip;
  if (a.mode == 0) {
    ip = a.p[lane & 7];  // per-lane index into the argument block: vector load
  } else if (a.mode == 1) {
    ip = a.p[0];  // uniform: scalar load
  } else {
    ip = reinterpret_cast<const int64_t* const*>(a.desc)[lane & 7];
  }
  const int64_t v = ip[blockIdx.x];
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = clock64();
  if (lane == 0) a.out[blockIdx.x] = (t1 - t0) + (v == 123456789 ? 1 : 0);
}

int main() {
  const int nb = 256;
  int64_t* data;
  int64_t* desc;
  unsigned long long* out;
  hipMalloc(&data, 8 * 4096 * sizeof(int64_t));
  hipMemset(data, 0, 8 * 4096 * sizeof(int64_t));
  hipMalloc(&desc, 8 * sizeof(int64_t*));
  hipMalloc(&out, nb * sizeof(unsigned long long));
  Args a = {};
  std::vector<const int64_t*> ptrs(8);
  for (int i = 0; i < 8; ++i) a.p[i] = ptrs[i] = data + 4096 * i;
  hipMemcpy(desc, ptrs.data(), 8 * sizeof(int64_t*), hipMemcpyHostToDevice);
  a.desc = desc;
  a.out = out;
  const char* names[3] = {"kernarg, per-lane vector load", "kernarg, scalar load", "device descriptor buffer"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
      a.mode = m;
      for (int w = 0; w < 5; ++w) probe<<<nb, 64>>>(a);
      hipDeviceSynchronize();
      std::vector<unsigned long long> h(nb);
      hipMemcpy(h.data(), out, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      std::vector<unsigned long long> s(h);
      std::sort(s.begin(), s.end());
      printf("%-32s cycles to first dependent value: min %llu med %llu max %llu\n", names[m], s[0], s[nb / 2],
             s[nb - 1]);
    }
  return 0;
}
