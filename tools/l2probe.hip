// Operand-fetch microbenchmark (in-kernel s_memrealtime stamps, 10 ns ticks): 256 workgroups (one
// per CU) each load a chunk of KB kilobytes with every load issued before the first wait, then
// sum it.  Reported: the median workgroup's load time (entry to last load landed) and the span of
// the launch (first entry to last exit), for
//   - the chunk just written by the previous launch on the reader's own XCD (shift 0) or another
//     XCD (shift 1), with plain / write-through (sc1) stores;
//   - the same chunk re-read by the next launch (again);
//   - a chunk not written for a while (after a 512 MB memset: HBM);
//   - dword loads (one float per lane per instruction) instead of float4.
// Per-CU fetch rate = KB / load time.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/l2probe tools/l2probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int NB = 256;
constexpr int MAXKB = 96;

__global__ void k_one() {}

__device__ __forceinline__ long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(256) void k_write(float4* buf, int nf4, int wt, float v) {
  float4* c = buf + (size_t)blockIdx.x * nf4;
  const float4 x = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
  for (int i = threadIdx.x; i < nf4; i += 256) {
    if (!wt) {
      c[i] = x;
    } else {
      float* p = reinterpret_cast<float*>(c + i);
      __hip_atomic_store(p, x.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 1, x.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 2, x.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 3, x.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// NJ float4 per thread (NJ * 4 KB per workgroup), all requested before the first use
template <int NJ>
__global__ __launch_bounds__(256) void k_read4(const float4* buf, int nf4, int shift, long long* st, float* out) {
  const long long t0 = rt();
  const int src = (blockIdx.x + shift) % NB;
  const float4* c = buf + (size_t)src * nf4;
  float4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = c[threadIdx.x + 256 * j];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += acc[j].x + acc[j].y + acc[j].z + acc[j].w;
  __syncthreads();
  const long long t1 = rt();
  if (threadIdx.x == 0) {
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = t1;
  }
  if (s == -12345.f) out[blockIdx.x] = s;
}

// the same bytes with dword loads: 16 consecutive lanes read 64 contiguous bytes (the k_bwd pattern)
template <int NJ>
__global__ __launch_bounds__(256) void k_read1(const float* buf, int nf, int shift, long long* st, float* out) {
  const long long t0 = rt();
  const int src = (blockIdx.x + shift) % NB;
  const float* c = buf + (size_t)src * nf;
  float acc[NJ * 4];
#pragma unroll
  for (int j = 0; j < NJ * 4; ++j) acc[j] = c[threadIdx.x + 256 * j];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ * 4; ++j) s += acc[j];
  __syncthreads();
  const long long t1 = rt();
  if (threadIdx.x == 0) {
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = t1;
  }
  if (s == -12345.f) out[blockIdx.x] = s;
}

struct Res {
  double med_us, span_us;
};

Res summarize(const std::vector<long long>& h) {
  std::vector<double> d(NB);
  long long lo = h[0], hi = h[1];
  for (int b = 0; b < NB; ++b) {
    d[b] = (h[2 * b + 1] - h[2 * b]) * 0.01;
    lo = std::min(lo, h[2 * b]);
    hi = std::max(hi, h[2 * b + 1]);
  }
  std::nth_element(d.begin(), d.begin() + NB / 2, d.end());
  return {d[NB / 2], (hi - lo) * 0.01};
}

int main() {
  float4* buf = nullptr;
  float4* cold = nullptr;
  float* out = nullptr;
  float* junk = nullptr;
  long long* st = nullptr;
  const size_t bytes = (size_t)NB * MAXKB * 1024;
  const size_t junk_n = (size_t)512 << 20;
  if (hipMalloc(&buf, bytes) || hipMalloc(&cold, bytes) || hipMalloc(&out, NB * 4) || hipMalloc(&junk, junk_n) ||
      hipMalloc(&st, NB * 16))
    return 1;
  (void)hipMemset(cold, 0, bytes);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  std::vector<long long> h(2 * NB);
  const int reps = 40;
  auto run = [&](int kb, int kind, const float4* b, int shift) {
    const int nf4 = kb * 64;
    switch (kind * 1000 + kb) {
      case 12: hipLaunchKernelGGL(k_read4<3>, dim3(NB), dim3(256), 0, s, b, nf4, shift, st, out); break;
      case 24: hipLaunchKernelGGL(k_read4<6>, dim3(NB), dim3(256), 0, s, b, nf4, shift, st, out); break;
      case 48: hipLaunchKernelGGL(k_read4<12>, dim3(NB), dim3(256), 0, s, b, nf4, shift, st, out); break;
      case 96: hipLaunchKernelGGL(k_read4<24>, dim3(NB), dim3(256), 0, s, b, nf4, shift, st, out); break;
      case 1012: hipLaunchKernelGGL(k_read1<3>, dim3(NB), dim3(256), 0, s, (const float*)b, nf4 * 4, shift, st, out); break;
      case 1048: hipLaunchKernelGGL(k_read1<12>, dim3(NB), dim3(256), 0, s, (const float*)b, nf4 * 4, shift, st, out); break;
      default: break;
    }
  };
  auto collect = [&]() {
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), st, NB * 16, hipMemcpyDeviceToHost);
    return summarize(h);
  };
  std::printf("%-44s %6s %9s %9s %9s\n", "case (256 workgroups, one per CU)", "KB", "load_us", "span_us", "GB/s/CU");
  // does a small launch in between move the block -> XCD deal of the next launch?
  for (int mid : {0, 1, 3, 8}) {
    for (int shift : {0, 1}) {
      double m1 = 0;
      for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_write, dim3(NB), dim3(256), 0, s, buf, 96 * 64, 0, (float)r);
        if (mid) hipLaunchKernelGGL(k_one, dim3(mid), dim3(64), 0, s);
        run(96, 0, buf, shift);
        m1 += collect().med_us;
      }
      std::printf("plain write, %d-block launch between, shift %d %6d %9.2f\n", mid, shift, 96, m1 / reps);
    }
  }
  for (int kb : {12, 24, 48, 96}) {
    for (int kind : {0, 1}) {
      if (kind == 1 && kb != 12 && kb != 48) continue;
      for (int wt : {0, 1}) {
        for (int shift : {0, 1}) {
          double m1 = 0, s1 = 0, m2 = 0, s2 = 0;
          for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_write, dim3(NB), dim3(256), 0, s, buf, kb * 64, wt, (float)r);
            run(kb, kind, buf, shift);
            Res a = collect();
            run(kb, kind, buf, shift);
            Res b2 = collect();
            m1 += a.med_us, s1 += a.span_us, m2 += b2.med_us, s2 += b2.span_us;
          }
          char name[96];
          std::snprintf(name, sizeof name, "%s loads, %s write, %s XCD", kind ? "dword" : "float4", wt ? "sc1" : "plain",
                        shift ? "other" : "own");
          std::printf("%-44s %6d %9.2f %9.2f %9.1f\n", name, kb, m1 / reps, s1 / reps, kb * 1.024 / (m1 / reps));
          std::snprintf(name, sizeof name, "  ... read again by the next launch");
          std::printf("%-44s %6d %9.2f %9.2f %9.1f\n", name, kb, m2 / reps, s2 / reps, kb * 1.024 / (m2 / reps));
        }
      }
    }
    double mc = 0, sc = 0;
    for (int r = 0; r < reps; ++r) {
      (void)hipMemsetAsync(junk, r & 0xff, junk_n, s);
      run(kb, 0, cold, 0);
      Res a = collect();
      mc += a.med_us, sc += a.span_us;
    }
    std::printf("%-44s %6d %9.2f %9.2f %9.1f\n", "float4, cold (after a 512 MB memset)", kb, mc / reps, sc / reps,
                kb * 1.024 / (mc / reps));
  }
  return 0;
}
