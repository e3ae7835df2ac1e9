// Kernel launches through a function pointer -- the form libsfx's launch() uses
// (hipLaunchKernelGGL on a `void (*)(Args...)` parameter) -- eagerly and from a captured graph,
// next to a direct launch.  Built plain and with -Xarch_host -fsanitize=function (build.sh fnptr)
// to tell whether UBSan's function check changes what such a launch does (the round-3 runner hang
// under runner_ubsan_full).  Prints what each launch left in memory and the launch's error code.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_set(int* p, int v) { p[threadIdx.x] = v; }

template <typename... KArgs, typename... Args>
hipError_t launch_fp(void (*kern)(KArgs...), hipStream_t s, Args... args) {
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, s, args...);
  return hipGetLastError();
}

static int read0(const int* d) {
  int h[64] = {};
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -999;
  return h[0];
}

int main() {
  int* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
  (void)hipMemset(d, 0, 64 * sizeof(int));
  hipStream_t s;
  (void)hipStreamCreate(&s);
  int bad = 0;
  hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, s, d, 1);
  hipError_t e = hipGetLastError();
  (void)hipStreamSynchronize(s);
  int v = read0(d);
  std::printf("direct launch:            value %d (want 1), error %s\n", v, hipGetErrorString(e));
  bad |= v != 1;
  e = launch_fp(k_set, s, d, 2);
  (void)hipStreamSynchronize(s);
  v = read0(d);
  std::printf("function-pointer launch:  value %d (want 2), error %s\n", v, hipGetErrorString(e));
  bad |= v != 2;
  hipGraph_t g = nullptr;
  hipGraphExec_t ex = nullptr;
  hipError_t ec = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  e = launch_fp(k_set, s, d, 3);
  hipError_t ee = hipStreamEndCapture(s, &g);
  size_t nodes = 0;
  if (g) (void)hipGraphGetNodes(g, nullptr, &nodes);
  hipError_t ei = g ? hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) : hipErrorUnknown;
  hipError_t el = ex ? hipGraphLaunch(ex, s) : hipErrorUnknown;
  (void)hipStreamSynchronize(s);
  v = read0(d);
  std::printf("captured pointer launch:  value %d (want 3), nodes %zu, errors begin %s / launch %s / end %s / "
              "instantiate %s / replay %s\n",
              v, nodes, hipGetErrorString(ec), hipGetErrorString(e), hipGetErrorString(ee), hipGetErrorString(ei),
              hipGetErrorString(el));
  bad |= v != 3;
  std::printf(bad ? "fnptr: MISMATCH\n" : "fnptr: all launches ran\n");
  return bad;
}
