// Instruction-fetch cost: a kernel with ~NI straight-line VALU instructions (8 independent fma
// chains), run cold (after kernels with other code) and then warm (the same kernel again).
// Prints the median in-kernel time (entry -> end, wave 0 of each WG) of each instance.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
#define CK(x) do { if ((x) != hipSuccess) { printf("error %s line %d\n", #x, __LINE__); return 1; } } while (0)
template <int NI, int SALT>
__global__ __launch_bounds__(64) void body(float* out, unsigned long long* ts, float s) {
  unsigned long long t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x[j] = s * (threadIdx.x + j + SALT);
    asm volatile("" : "+v"(x[j]));
  }
#pragma unroll
  for (int i = 0; i < NI / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = __builtin_fmaf(x[j], 1.0001f + 1e-7f * (i & 7), 0.5f + SALT);
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc += x[j];
  asm volatile("" ::"v"(acc));
  unsigned long long t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) { ts[2 * blockIdx.x] = t0; ts[2 * blockIdx.x + 1] = t1; }
}
template <int NI>
int run(const char* tag) {
  const int nb = 256;
  float* out; unsigned long long* ts;
  CK(hipMalloc(&out, nb * 64 * 4 * 4)); CK(hipMalloc(&ts, nb * 16 * 3));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  // evictors: other code of the same size
  hipLaunchKernelGGL((body<NI, 1>), dim3(nb), dim3(64), 0, st, out + nb * 64, ts + 2 * nb * 2, 1.f);
  hipLaunchKernelGGL((body<NI, 2>), dim3(nb), dim3(64), 0, st, out + 2 * nb * 64, ts + 2 * nb * 2, 1.f);
  hipLaunchKernelGGL((body<NI, 3>), dim3(nb), dim3(64), 0, st, out + 3 * nb * 64, ts + 2 * nb * 2, 1.f);
  hipLaunchKernelGGL((body<NI, 0>), dim3(nb), dim3(64), 0, st, out, ts, 1.f);           // cold
  hipLaunchKernelGGL((body<NI, 0>), dim3(nb), dim3(64), 0, st, out, ts + 2 * nb, 1.f);  // warm
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  std::vector<double> c, w;
  std::vector<unsigned long long> h(4 * nb);
  for (int it = 0; it < 60; ++it) {
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    if (it < 10) continue;
    CK(hipMemcpy(h.data(), ts, nb * 32, hipMemcpyDeviceToHost));
    for (int j = 0; j < nb; ++j) {
      c.push_back((h[2 * j + 1] - h[2 * j]) * 10.0);
      w.push_back((h[2 * nb + 2 * j + 1] - h[2 * nb + 2 * j]) * 10.0);
    }
  }
  std::sort(c.begin(), c.end()); std::sort(w.begin(), w.end());
  printf("%s (~%d VALU instrs): cold median %.0f ns p90 %.0f | warm median %.0f ns p90 %.0f\n", tag, NI,
         c[c.size() / 2], c[c.size() * 9 / 10], w[w.size() / 2], w[w.size() * 9 / 10]);
  return 0;
}
int main() {
  run<256>("256");
  run<1024>("1k");
  run<2048>("2k");
  run<4096>("4k");
  return 0;
}
