// Does kernarg preloading (-mllvm -amdgpu-kernarg-preload-count) shorten the time from a
// workgroup's first instruction to its first global load landing, for a chain of dependent
// graph-replayed kernels whose kernel arguments are L2-cold (a 64 MB sweep between replays)?
// Build twice (with and without the flag) and compare.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
#define CK(x) do { if ((x) != hipSuccess) { printf("error %s line %d\n", #x, __LINE__); return 1; } } while (0)
__global__ void k(const float* __restrict__ a, float* __restrict__ b, int n, unsigned long long* __restrict__ ts) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int i = blockIdx.x * 256 + threadIdx.x;
  float v = i < n ? a[i] : 0.f;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  b[i] = v * 2.f;
  if (threadIdx.x == 0) { ts[2 * blockIdx.x] = t0; ts[2 * blockIdx.x + 1] = t1; }
}
__global__ void sweep(const float4* __restrict__ x, float4* __restrict__ y, int n) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) { float4 v = x[i]; acc.x += v.x; }
  if (acc.x == 12345.f) y[0] = acc;
}
int main() {
  const int nb = 64, n = nb * 256, L = 16, NS = 16 << 20;
  float *a, *b; unsigned long long* ts; float4* big;
  CK(hipMalloc(&a, n * 4 * (L + 1))); CK(hipMalloc(&ts, nb * 16 * L)); CK(hipMalloc(&big, NS * 16));
  CK(hipMemset(a, 0, n * 4 * (L + 1))); CK(hipMemset(big, 0, NS * 16));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int l = 0; l < L; ++l)
    hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, s, a + l * n, a + (l + 1) * n, n, ts + 2 * nb * l);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<double> d, gap; double tot = 0; int cnt = 0;
  std::vector<unsigned long long> h(2 * nb * L);
  for (int it = 0; it < 120; ++it) {
    hipLaunchKernelGGL(sweep, dim3(1024), dim3(256), 0, s, big, big, NS);
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    if (it < 20) continue;
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); tot += ms; ++cnt;
    CK(hipMemcpy(h.data(), ts, nb * 16 * L, hipMemcpyDeviceToHost));
    for (int l = 0; l < L; ++l)
      for (int j = 0; j < nb; ++j) d.push_back((h[2 * (nb * l + j) + 1] - h[2 * (nb * l + j)]) * 10.0);
  }
  std::sort(d.begin(), d.end());
  printf("entry -> first load landed: median %.0f ns  p10 %.0f  p90 %.0f ; graph of %d kernels %.2f us per kernel\n",
         d[d.size() / 2], d[d.size() / 10], d[d.size() * 9 / 10], L, 1000.0 * tot / cnt / L);
  return 0;
}
