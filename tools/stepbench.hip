// Per-launch timing of the C2 all-task step (T = 8, H = 256 x 2, B = 32) through the engine path
// (sfx_step_all / sfx_step_finish, eager launches with packet timestamps: the bench's live
// instrumentation).  Prints, per launch position of a step with the standard launch count, the
// kernel kind, mean / min duration and the launch's algorithmic bytes -- the A/B harness for
// kernel variants (compile a variant with -D..., run both on one box).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/stepbench tools/stepbench.hip -ldl
// Run: tools/stepbench [steps=300] [skip=1]   (skip=0: SFX_SKIP=0, every policy recomputes)
#include "../deep-successor-features-for-transfer_amd/csrc/sfx.hip"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

namespace {
unsigned g_seed = 12345u;
float urand() { return ((g_seed = g_seed * 1664525u + 1013904223u) >> 8) * (1.f / 16777216.f); }
}  // namespace

int main(int argc, char** argv) {
  const int steps = argc > 1 ? std::atoi(argv[1]) : 300;
  if (argc > 2 && argv[2][0] == '0') setenv("SFX_SKIP", "0", 1);
  const int T = 8, n_s = 17, H = 256, A = 7, d = 8, B = 32, acts[2] = {1, 1};
  sfx_t hh = nullptr;
  if (sfx_create(&hh, T, n_s, H, 2, acts, A, d, B, 0, nullptr) != SFX_OK) {
    std::fprintf(stderr, "sfx_create: %s\n", sfx_last_error());
    return 1;
  }
  sfx_handle* h = hh;
  std::vector<float> p(sfx_head_numel(hh));
  for (int t = 0; t < T; ++t) {
    // torch-like init: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) per layer is not needed for timing; keep
    // the values small so the TD errors stay finite over many steps
    for (float& x : p) x = (urand() - 0.5f) * 0.1f;
    if (sfx_load_head(hh, t, 0, p.data()) || sfx_load_head(hh, t, 1, p.data())) return 1;
    std::vector<float> w(d);
    for (float& x : w) x = (urand() - 0.5f) * 0.02f;
    if (sfx_load_w(hh, t, w.data())) return 1;
  }
  sfx_set_adam(hh, 1e-3, 0.0, 1e-3, 0.0, 0.9, 0.999, 1e-8);
  sfx_set_target_update_ev(hh, 1000);
  // a pool of minibatches (device), cycled
  const int pool = 64;
  const size_t per = (size_t)B * (2 * n_s + d + 1) + 2 * n_s + d + 1;
  std::vector<float> hf(per * pool);
  for (float& x : hf) x = urand() * 2.f - 1.f;
  std::vector<int64_t> ha((size_t)B * pool);
  for (auto& a : ha) a = (int64_t)(urand() * A) % A;
  float* df = nullptr;
  int64_t* da = nullptr;
  if (hipMalloc(&df, hf.size() * 4) || hipMalloc(&da, ha.size() * 8)) return 1;
  for (int i = 0; i < pool; ++i) {  // gamma 0.9, phi in [0, 1)
    float* b = hf.data() + per * i;
    for (int k = 0; k < B * d; ++k) b[2 * B * n_s + k] = 0.5f * (b[2 * B * n_s + k] + 1.f);
    for (int k = 0; k < B; ++k) b[2 * B * n_s + B * d + k] = 0.9f;
  }
  (void)hipMemcpy(df, hf.data(), hf.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(da, ha.data(), ha.size() * 8, hipMemcpyHostToDevice);
  std::map<int, std::vector<double>> by_len;  // launch count -> per-position sums
  std::map<int, std::vector<double>> mins, bytes;
  std::map<int, std::vector<int>> kinds;
  std::map<int, int> nsteps;
  for (int it = 0; it < steps + 50; ++it) {
    const float* b = df + per * (it % pool);
    const float *S = b, *S1 = b + B * n_s, *phi = b + 2 * B * n_s, *gam = phi + B * d, *tail = gam + B;
    h->prof = it >= 50;
    const size_t before = h->prof_recs.size();
    if (sfx_step_all(hh, S, da + (size_t)B * (it % pool), phi, S1, gam, B, 1, it % T, tail, tail + d, 1e-3f,
                     tail + 1, it % T, 1, nullptr) != SFX_OK) {
      std::fprintf(stderr, "sfx_step_all: %s\n", sfx_last_error());
      return 1;
    }
    int64_t out[3];
    if (sfx_step_finish(hh, out) != SFX_OK) {
      std::fprintf(stderr, "sfx_step_finish: %s\n", sfx_last_error());
      return 1;
    }
    if (!h->prof) continue;
    (void)hipStreamSynchronize(h->stream);
    const int n = (int)(h->prof_recs.size() - before);
    auto& sum = by_len[n];
    auto& mn = mins[n];
    auto& by = bytes[n];
    auto& kd = kinds[n];
    if (sum.empty()) {
      sum.assign(n, 0.0);
      mn.assign(n, 1e30);
      by.assign(n, 0.0);
      kd.assign(n, -1);
    }
    for (int i = 0; i < n; ++i) {
      const auto& r = h->prof_recs[before + i];
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, r.a, r.b);
      sum[i] += 1e3 * ms;
      mn[i] = std::min(mn[i], 1e3 * (double)ms);
      by[i] = r.bytes;
      kd[i] = r.kind;
    }
    nsteps[n] += 1;
    for (auto& r : h->prof_recs) {
      h->prof_pool.push_back(r.a);
      h->prof_pool.push_back(r.b);
    }
    h->prof_recs.clear();
  }
  static const char* kname[] = {"fwd", "tdg", "bwd", "gpi", "lms", "ver", "tsf"};
  long long chk = 0, skp = 0;
  sfx_skip_stats(hh, &chk, &skp, 0);
  std::printf("stepbench: %d steps, policies checked %lld, skipped %lld\n", steps, chk, skp);
  for (auto& kv : by_len) {
    const int n = kv.first, ns = nsteps[n];
    double tot = 0.0;
    for (double s : kv.second) tot += s / ns;
    std::printf("== %d launches per step: %d steps, %.2f us of launches per step\n", n, ns, tot);
    double kb = 0.0;
    int nb = 0;
    for (int i = 0; i < n; ++i) {
      std::printf("  %2d %-4s mean %7.2f  min %7.2f us  %8.0f KB\n", i, kname[kinds[n][i]], kv.second[i] / ns,
                  mins[n][i], bytes[n][i] / 1024.0);
      if (kinds[n][i] == 2) {
        kb += kv.second[i] / ns;
        ++nb;
      }
    }
    if (nb) std::printf("  K_BWD mean %.2f us over %d launches per step\n", kb / nb, nb);
  }
  sfx_destroy(hh);
  return 0;
}
