// Probe: latency of hipStreamWaitValue32 on plain device memory (the peer exchange's
// stream-level wait), a waiter kernel spinning on the same flag, and back-to-back
// empty launches for reference.  Usage: ./waitvalue
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && p) p[1] += 1; }
__global__ void k_stamp(long long* t, int i) { if (threadIdx.x == 0) t[i] = wall_clock64(); }
__global__ void k_set(int* f, int v, long long* t, int i, long long delay) {
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < delay) __builtin_amdgcn_s_sleep(2);
    t[i] = wall_clock64();
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void k_wait(int* f, int v, long long* t, int i) {
  if (threadIdx.x == 0) {
    long long n = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < v && ++n < (1LL << 26)) __builtin_amdgcn_s_sleep(1);
    t[i] = wall_clock64();
  }
}

int main() {
  int dev = 0, attr = 0;
  CK(hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, dev));
  int rate = 0;
  CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev));  // kHz
  printf("CanUseStreamWaitValue=%d wall_clock_kHz=%d\n", attr, rate);
  int* f;
  long long* t;
  CK(hipMalloc(&f, 64));
  CK(hipMalloc(&t, 8 * 4096));
  CK(hipMemset(f, 0, 64));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  const double us = 1000.0 / rate;
  // 1) empty launches back to back
  for (int w = 0; w < 2; w++) {
    CK(hipStreamSynchronize(a));
    auto c0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, a, nullptr);
    CK(hipStreamSynchronize(a));
    auto c1 = std::chrono::steady_clock::now();
    printf("empty launch: %.2f us each\n", std::chrono::duration<double, std::micro>(c1 - c0).count() / 1000);
  }
  // 2) satisfied waits between empty launches
  CK(hipMemset(f, 0x7f, 4));
  for (int w = 0; w < 2; w++) {
    CK(hipStreamSynchronize(a));
    auto c0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) {
      CK(hipStreamWaitValue32(a, f, 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
      hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, a, nullptr);
    }
    CK(hipStreamSynchronize(a));
    auto c1 = std::chrono::steady_clock::now();
    printf("satisfied wait + empty launch: %.2f us each\n", std::chrono::duration<double, std::micro>(c1 - c0).count() / 1000);
  }
  // 3) a wait released by a kernel on another stream: release -> next kernel start
  for (int rep = 0; rep < 5; rep++) {
    CK(hipMemset(f, 0, 4));
    CK(hipDeviceSynchronize());
    CK(hipStreamWaitValue32(a, f, 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, a, t, 1);
    hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, b, f, 1, t, 0, (long long)(200 / us));
    CK(hipDeviceSynchronize());
    long long h[2];
    CK(hipMemcpy(h, t, 16, hipMemcpyDeviceToHost));
    printf("stream wait released -> next kernel: %.2f us\n", (h[1] - h[0]) * us);
  }
  // 4) a spinning waiter kernel released by another stream's kernel
  for (int rep = 0; rep < 5; rep++) {
    CK(hipMemset(f, 0, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, a, f, 1, t, 1);
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, a, t, 2);
    hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, b, f, 1, t, 0, (long long)(200 / us));
    CK(hipDeviceSynchronize());
    long long h[3];
    CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
    printf("spin waiter: release -> waiter sees %.2f us, -> next kernel %.2f us\n", (h[1] - h[0]) * us, (h[2] - h[0]) * us);
  }
  printf("done\n");
  return 0;
}
