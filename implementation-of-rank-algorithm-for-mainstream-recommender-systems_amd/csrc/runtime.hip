// Host runtime of the rankops C ABI: error text, per-device flag word, CU count.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>

#include "common.h"

namespace rk {

namespace {
thread_local char g_err[512] = "";
constexpr int kMaxDevices = 64;
uint32_t* g_flags[kMaxDevices] = {nullptr};
int g_cus[kMaxDevices] = {0};
std::mutex g_mu;

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  return dev;
}
}  // namespace

void raise_lds_limit(const void* kern, int bytes) {
  struct Entry {
    const void* kern;
    int dev, bytes;
  };
  static Entry done[256];
  static int n = 0;
  const int dev = current_device();
  std::lock_guard<std::mutex> lock(g_mu);
  for (int i = 0; i < n; ++i)
    if (done[i].kern == kern && done[i].dev == dev && done[i].bytes >= bytes) return;
  // static LDS (timing builds add some) counts against the same 160 KiB
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, kern) == hipSuccess) bytes = std::min<int>(bytes, 160 * 1024 - (int)fa.sharedSizeBytes);
  if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    (void)hipGetLastError();  // leave no sticky error for the launch check that follows
  if (n < 256) done[n++] = Entry{kern, dev, bytes};
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(RK_ERR_LAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
  return RK_OK;
}

uint32_t* device_flags() {
  int dev = current_device();
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  return g_flags[dev];
}

int num_cus() {
  int dev = current_device();
  if (dev < 0 || dev >= kMaxDevices) return 256;
  if (g_cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_cus[dev] = n;
  }
  return g_cus[dev];
}

}  // namespace rk

RK_API int32_t rk_abi_version(void) { return RK_ABI_VERSION; }

RK_API const char* rk_last_error(void) { return rk::g_err; }

RK_API int rk_init(int32_t device) {
  if (device < 0 || device >= rk::kMaxDevices) return rk::fail(RK_ERR_INVALID, "rk_init: bad device %d", device);
  std::lock_guard<std::mutex> lock(rk::g_mu);
  if (rk::g_flags[device]) return RK_OK;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return rk::fail(RK_ERR_RUNTIME, "rk_init: hipGetDevice failed");
  if (hipSetDevice(device) != hipSuccess) return rk::fail(RK_ERR_RUNTIME, "rk_init: hipSetDevice(%d) failed", device);
  uint32_t* p = nullptr;
  hipError_t e = hipMalloc(&p, 64);
  if (e == hipSuccess) e = hipMemset(p, 0, 64);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return rk::fail(RK_ERR_RUNTIME, "rk_init: %s", hipGetErrorString(e));
  rk::g_flags[device] = p;
  return RK_OK;
}

RK_API int rk_error_flags(int32_t device, uint32_t* flags, int32_t reset) {
  if (!flags) return rk::fail(RK_ERR_INVALID, "rk_error_flags: null output");
  if (device < 0 || device >= rk::kMaxDevices || !rk::g_flags[device])
    return rk::fail(RK_ERR_INVALID, "rk_error_flags: device %d not initialised", device);
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(flags, rk::g_flags[device], sizeof(uint32_t), hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) e = hipMemset(rk::g_flags[device], 0, sizeof(uint32_t));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return rk::fail(RK_ERR_RUNTIME, "rk_error_flags: %s", hipGetErrorString(e));
  return RK_OK;
}
