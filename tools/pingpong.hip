// tools/pingpong.hip -- latency of the native runner's host <-> device hand-off
// for two ways of staging a step's inputs:
//   pull  inputs and the go word in host-coherent memory (hipHostMalloc): the gate kernel polls
//         go across PCIe and copies the inputs across PCIe -- what sfx_runner does;
//   push  inputs and go in fine-grained device memory the host writes through the BAR: the
//         gate polls HBM and copies from HBM.
// Per iteration k the host waits for iteration k-1's published result, writes NB bytes of
// inputs and bumps go; on the device, gate(k) (wait, copy) and check(k) (verify the copy, hold
// the GPU for `busy` so host launches stay off the measured path, publish to host memory) were
// launched ahead.  Device timestamps (100 MHz): handoff = gate(k) saw go - check(k-1) published,
// copy = gate(k) copy done - saw go.  Medians over the iterations, in µs.
// Build: hipcc --offload-arch=gfx950 -O2 tools/pingpong.hip -o tools/pingpong
// Run:   tools/pingpong pull|push [bytes] [iters]
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Res {
  long long seq, bad;
};
struct Stamp {
  long long go, cp, pub;
};

__global__ void k_gate(const long long* go, long long want, const uint4* src, uint4* dst, int n16, int* tmo,
                       Stamp* ts) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
      if (wall_clock64() - t0 > 200000000LL) {  // 2 s
        ok = 0;
        __hip_atomic_store(tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    ts[want].go = wall_clock64();
  }
  __syncthreads();
  if (!ok) return;
  for (int i = threadIdx.x; i < n16; i += 256) dst[i] = src[i];
  __syncthreads();
  if (threadIdx.x == 0) ts[want].cp = wall_clock64();
}

__global__ void k_check(const uint4* dst, int n16, long long seq, Res* res, Stamp* ts, long long busy) {
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n16; i += 256) {
    const uint4 v = dst[i];
    if (v.x != (unsigned)seq || v.w != (unsigned)i) atomicAdd(&bad, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < busy) __builtin_amdgcn_s_sleep(8);
    ts[seq].pub = wall_clock64();
    __hip_atomic_store(&res->bad, (long long)bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&res->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const bool push = argc > 1 && std::strcmp(argv[1], "push") == 0;
  const int nbytes = argc > 2 ? std::atoi(argv[2]) : 6912;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 2000;
  const int n16 = nbytes / 16, W = 8;
  uint4 *src = nullptr, *dst = nullptr;
  long long* go = nullptr;
  Res* res = nullptr;
  int* tmo = nullptr;
  Stamp* ts = nullptr;
  if (push) {
    CK(hipExtMallocWithFlags((void**)&src, nbytes, hipDeviceMallocFinegrained));
    CK(hipExtMallocWithFlags((void**)&go, 64, hipDeviceMallocFinegrained));
  } else {
    CK(hipHostMalloc((void**)&src, nbytes, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&go, 64, hipHostMallocCoherent | hipHostMallocMapped));
  }
  CK(hipHostMalloc((void**)&res, sizeof(Res), hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&tmo, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipMalloc((void**)&dst, nbytes));
  CK(hipMalloc((void**)&ts, sizeof(Stamp) * (iters + 2)));
  CK(hipMemset(go, 0, 64));
  CK(hipDeviceSynchronize());
  signal(SIGSEGV, on_segv);
  signal(SIGBUS, on_segv);
  if (sigsetjmp(g_jb, 1)) {
    std::printf("{\"mode\": \"%s\", \"host_access\": false}\n", push ? "push" : "pull");
    return 0;
  }
  volatile long long probe = *go;  // push: a host load through the BAR (faults without host access)
  (void)probe;
  *go = 0;
  signal(SIGSEGV, SIG_DFL);
  signal(SIGBUS, SIG_DFL);
  res->seq = 0;
  res->bad = 0;
  *tmo = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<uint4> shadow(n16);
  auto launch = [&](long long k) {
    hipLaunchKernelGGL(k_gate, dim3(1), dim3(256), 0, st, go, k, src, dst, n16, tmo, ts);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, st, dst, n16, k, res, ts, 3000LL);  // 30 µs
  };
  for (long long k = 1; k <= W && k <= iters; ++k) launch(k);
  for (long long k = 1; k <= iters; ++k) {
    if (k > 1)
      while (__atomic_load_n(&res->seq, __ATOMIC_ACQUIRE) < k - 1)
        if (__atomic_load_n(tmo, __ATOMIC_RELAXED)) {
          std::fprintf(stderr, "gate timeout at %lld\n", k);
          return 2;
        }
    if (res->bad) {
      std::fprintf(stderr, "bad inputs at %lld: %lld\n", k - 1, res->bad);
      return 3;
    }
    for (int i = 0; i < n16; ++i) shadow[i] = make_uint4((unsigned)k, 0u, 0u, (unsigned)i);
    std::memcpy((void*)src, shadow.data(), nbytes);
    _mm_sfence();
    __atomic_store_n(go, k, __ATOMIC_RELEASE);
    _mm_sfence();
    if (k + W <= iters) launch(k + W);
  }
  CK(hipStreamSynchronize(st));
  if (res->bad) {
    std::fprintf(stderr, "bad inputs at the last iteration: %lld\n", res->bad);
    return 3;
  }
  std::vector<Stamp> h(iters + 2);
  CK(hipMemcpy(h.data(), ts, sizeof(Stamp) * (iters + 2), hipMemcpyDeviceToHost));
  std::vector<double> handoff, copy;
  for (int k = 2 + 100; k <= iters; ++k) {
    handoff.push_back(0.01 * (double)(h[k].go - h[k - 1].pub));
    copy.push_back(0.01 * (double)(h[k].cp - h[k].go));
  }
  std::printf("{\"mode\": \"%s\", \"host_access\": true, \"bytes\": %d, \"iters\": %d, \"handoff_us\": %.2f, "
              "\"copy_us\": %.2f}\n",
              push ? "push" : "pull", nbytes, iters, median(handoff), median(copy));
  return 0;
}
