// Microbenchmark: per-kernel cost of back-to-back dependent launches on one stream
// (empty kernel / one 16 KB load per WG / 256 WGs), eager vs hipGraph replay.
// Build: hipcc --offload-arch=gfx950 -O3 -o launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 9999999) out[0] = 1.f;
}
__global__ void k_load(const float4* in, float* out) {
  float4 v = in[blockIdx.x * 256 + threadIdx.x];
  float s = v.x + v.y + v.z + v.w;
  if (s == 12345.f) out[blockIdx.x] = s;
}
__global__ void k_chain(const float* in, float* out) {  // read what the previous launch wrote
  const int i = blockIdx.x * 256 + threadIdx.x;
  out[i] = in[i] * 1.0001f + 1.f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <class F>
float time_seq(hipStream_t s, int n, F launch, bool graph) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipGraphExec_t ex = nullptr;
  if (graph) {
    hipGraph_t g;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; ++i) launch(i);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    (void)hipGraphLaunch(ex, s);
  } else {
    for (int i = 0; i < n; ++i) launch(i);
  }
  (void)hipStreamSynchronize(s);
  (void)hipEventRecord(a, s);
  for (int rep = 0; rep < 5; ++rep) {
    if (graph) (void)hipGraphLaunch(ex, s);
    else for (int i = 0; i < n; ++i) launch(i);
  }
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  if (ex) (void)hipGraphExecDestroy(ex);
  return ms * 1000.f / (5 * n);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *buf0, *buf1;
  CK(hipMalloc(&buf0, 64 << 20));
  CK(hipMalloc(&buf1, 64 << 20));
  CK(hipMemset(buf0, 0, 64 << 20));
  CK(hipMemset(buf1, 0, 64 << 20));
  const int n = 200;
  for (int graph = 0; graph < 2; ++graph) {
    for (int wgs : {1, 16, 256, 1024}) {
      float t0 = time_seq(s, n, [&](int) { hipLaunchKernelGGL(k_empty, dim3(wgs), dim3(256), 0, s, buf1); }, graph);
      float t1 = time_seq(s, n, [&](int) { hipLaunchKernelGGL(k_load, dim3(wgs), dim3(256), 0, s, (const float4*)buf0, buf1); }, graph);
      float t2 = time_seq(s, n, [&](int i) {
        float* a = (i & 1) ? buf1 : buf0;
        float* b = (i & 1) ? buf0 : buf1;
        hipLaunchKernelGGL(k_chain, dim3(wgs), dim3(256), 0, s, a, b);
      }, graph);
      printf("%s WGs=%4d  empty %6.2f us  load16KB/WG %6.2f us  chain %6.2f us per kernel\n",
             graph ? "graph" : "eager", wgs, t0, t1, t2);
    }
  }
  return 0;
}
