// Host cost of a kernel launch on this runtime (diagnostic): hipLaunchKernelGGL of an empty kernel
// with 0 / 16 arguments, hipGetLastError, on a non-blocking stream, 2000 calls each, GPU kept busy
// by the launches themselves (no synchronisation inside the timed loops).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty0() {}
__global__ void k_empty16(const float *a, const float *b, const float *c, const float *d, int e, int f, float g,
                          float h, int *i, float *j, unsigned long long *k, int *l, int *m, int n, void *o, void *p) {
  if (e == -12345 && threadIdx.x == 0) *i = 1;
}

struct Args16 {
  const float *a, *b, *c, *d;
  int e, f;
  float g, h;
  int *i;
  float *j;
  unsigned long long *k;
  int *l, *m;
  int n;
  void *o, *p;
};
__global__ void k_struct16(Args16 x) {
  if (x.e == -12345 && threadIdx.x == 0) *x.i = 1;
}
__global__ void k_empty4(const float *a, const float *b, int e, float *j) {
  if (e == -12345 && threadIdx.x == 0) *j = 1.f;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipLaunchKernelGGL(k_empty0, dim3(1), dim3(64), 0, s);
  hipStreamSynchronize(s);
  const int n = 2000;
  using C = std::chrono::steady_clock;
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = C::now();
    for (int r = 0; r < n; ++r) hipLaunchKernelGGL(k_empty0, dim3(1312), dim3(256), 0, s);
    auto t1 = C::now();
    hipStreamSynchronize(s);
    auto t2 = C::now();
    for (int r = 0; r < n; ++r)
      hipLaunchKernelGGL(k_empty16, dim3(1312), dim3(256), 0, s, nullptr, nullptr, nullptr, nullptr, 1, 2, 1.f, 2.f,
                         nullptr, nullptr, nullptr, nullptr, nullptr, 3, nullptr, nullptr);
    auto t3 = C::now();
    hipStreamSynchronize(s);
    auto t4 = C::now();
    for (int r = 0; r < n; ++r) (void)hipGetLastError();
    auto t5 = C::now();
    const Args16 x{nullptr, nullptr, nullptr, nullptr, 1, 2, 1.f, 2.f, nullptr, nullptr, nullptr, nullptr, nullptr, 3,
                   nullptr, nullptr};
    for (int r = 0; r < n; ++r) hipLaunchKernelGGL(k_struct16, dim3(1312), dim3(256), 0, s, x);
    auto t6 = C::now();
    hipStreamSynchronize(s);
    auto t7 = C::now();
    for (int r = 0; r < n; ++r) hipLaunchKernelGGL(k_empty4, dim3(1312), dim3(256), 0, s, nullptr, nullptr, 1, nullptr);
    auto t8 = C::now();
    hipStreamSynchronize(s);
    void *kargs[1] = {const_cast<Args16 *>(&x)};
    auto t9 = C::now();
    for (int r = 0; r < n; ++r)
      (void)hipLaunchKernel(reinterpret_cast<const void *>(k_struct16), dim3(1312), dim3(256), kargs, 0, s);
    auto t10 = C::now();
    hipStreamSynchronize(s);
    const double us = 1e-3 / n;
    printf("launch0 %.2f us  launch16 %.2f us  struct16 %.2f us  launch4 %.2f us  hipLaunchKernel(struct16) %.2f us  "
           "getlasterror %.3f us\n",
           std::chrono::duration<double, std::nano>(t1 - t0).count() * us,
           std::chrono::duration<double, std::nano>(t3 - t2).count() * us,
           std::chrono::duration<double, std::nano>(t6 - t5).count() * us,
           std::chrono::duration<double, std::nano>(t8 - t7).count() * us,
           std::chrono::duration<double, std::nano>(t10 - t9).count() * us,
           std::chrono::duration<double, std::nano>(t5 - t4).count() * us);
  }
  return 0;
}
