// Host-side sanitizer run of the native env-step runner (csrc/sfx_runner.inc) -- the host/device
// protocol VERDICT r2 called the riskiest code in the product: pre-launched gated graphs, the
// result ring, gate time-outs with cancel / re-issue, the hold word, host rounds on the side
// stream and the recompute after a drain, env-callback errors that cancel the queue.
//
// Built by tools/hostsan/build.sh with libsfx's sources compiled in and AddressSanitizer +
// UndefinedBehaviorSanitizer on the HOST code only (every -fsanitize= after -Xarch_host: the
// kernels are the product's, unchanged).  Runs each schedule through those paths with small heads
// and checks the C ABI's status codes and counters; any heap / stack / UB finding aborts the run
// with the sanitizer's report.  Progress lines go to stdout.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/sfx.h"

#define CK(x)                                                                         \
  do {                                                                                \
    const int rc_ = (x);                                                              \
    if (rc_ != 0) {                                                                   \
      std::fprintf(stderr, "FAIL %s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, \
                   sfx_last_error());                                                 \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

namespace {

constexpr int NS = 17, H = 32, A = 7, D = 8;

unsigned long long g_rng = 0x9E3779B97F4A7C15ull;
float urand() {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (float)((g_rng >> 40) * (1.0 / 16777216.0));
}

sfx_t make_handle(int T) {
  const int acts[2] = {SFX_ACT_RELU, SFX_ACT_RELU};
  sfx_t h = nullptr;
  CK(sfx_create(&h, T, NS, H, 2, acts, A, D, 32, 0, nullptr));
  CK(sfx_set_adam(h, 1e-3, 0.0, 1e-3, 0.0, 0.9, 0.999, 1e-8));
  CK(sfx_set_target_update_ev(h, 1000));
  const int P = sfx_head_numel(h);
  std::vector<float> p(P), w(D);
  for (int t = 0; t < T; ++t) {
    for (float& x : p) x = (urand() - 0.5f) * 0.2f;
    for (float& x : w) x = urand() * 0.1f;
    CK(sfx_load_head(h, t, 0, p.data()));
    CK(sfx_load_head(h, t, 1, p.data()));
    CK(sfx_load_w(h, t, w.data()));
  }
  return h;
}

struct Env {  // a host env with an optional injected failure (exercises the cancel-on-error path)
  int steps = 0, fail_at = -1;
};
int env_reset(void* ctx, int, float* s0) {
  (void)ctx;
  for (int i = 0; i < NS; ++i) s0[i] = urand() - 0.5f;
  return 0;
}
int env_step(void* ctx, int task, int action, float* s1, float* phi, float* r, int* term) {
  Env* e = static_cast<Env*>(ctx);
  if (e->fail_at >= 0 && e->steps == e->fail_at) {
    e->fail_at = -1;
    return 7;
  }
  e->steps += 1;
  for (int i = 0; i < NS; ++i) s1[i] = urand() - 0.5f + 0.01f * (float)action;
  for (int k = 0; k < D; ++k) phi[k] = urand();
  *r = phi[task % D];
  *term = (e->steps % 37) == 0;
  return 0;
}

void stats(const char* tag, sfx_runner_t R) {
  long long n = 0, pre = 0, hr = 0, rt = 0, rc = 0;
  double wait = 0;
  CK(sfx_runner_stats(R, &n, &pre, &hr, &wait));
  CK(sfx_runner_retried(R, &rt));
  CK(sfx_runner_recomputed(R, &rc));
  std::printf("  %-34s env_steps %lld prelaunched %lld host_round_steps %lld retried %lld recomputed %lld\n", tag, n,
              pre, hr, rt, rc);
  std::fflush(stdout);
}

// one schedule through: plain pipelined steps, 10 ns gates (every queued step cancelled and
// re-issued) with forced host rounds (recompute after the drain), an env error mid-run, records
void scenario(const char* name, int schedule, int T, bool callbacks) {
  std::printf("%s (T=%d, %s env)\n", name, T, callbacks ? "callback" : "built-in");
  std::fflush(stdout);
  sfx_t h = make_handle(T);
  if (schedule == 3) {  // one rank, no transport: nothing to reduce
    CK(sfx_shard_setup(h, T, 0));
    CK(sfx_set_comm_host(h, nullptr, nullptr, 0, 1));
  }
  if (schedule == 2) {
    CK(sfx_tsf_setup(h, 16, 3, 1.0f, 1e-3, 0.0, 1e-3, 0.0));
    const int Pg = 3 * (2 * NS + 1) + 16 * NS + 16, Ph = D * 16 + D;
    std::vector<float> g(Pg), hh(Ph);
    for (int t = 0; t < T; ++t) {
      for (float& x : g) x = (urand() - 0.5f) * 0.2f;
      CK(sfx_tsf_load_g(h, t, g.data()));
    }
    for (float& x : hh) x = (urand() - 0.5f) * 0.2f;
    CK(sfx_tsf_load_h(h, hh.data()));
  }
  Env env;
  sfx_runner_t R = nullptr;
  CK(sfx_runner_create(&R, h, 16, 300, 0.9f, 0.3f, 0.05f, 25, 1, 11ull, callbacks ? env_reset : nullptr,
                       callbacks ? env_step : nullptr, callbacks ? &env : nullptr));
  CK(sfx_runner_config(R, schedule, 1, callbacks ? 0.0f : 0.02f));
  CK(sfx_runner_record(R, 64));
  CK(sfx_runner_prefill(R, 40));
  CK(sfx_runner_set_task(R, T - 1));
  CK(sfx_runner_warm(R));
  CK(sfx_runner_run(R, 120));
  stats("pipelined", R);
  // 10 ns gate bound: every pre-launched step is cancelled at its gate and issued again
  CK(sfx_runner_gate_timeout(R, 1e-8));
  CK(sfx_runner_run(R, 30));
  if (schedule == 0 || schedule == 3) {  // + forced host rounds: the recompute after the drain
    CK(sfx_debug_force_rerun(h, 1));
    CK(sfx_runner_run(R, 20));
    CK(sfx_debug_force_rerun(h, -1));
  }
  stats("10 ns gates (+ forced host rounds)", R);
  CK(sfx_runner_gate_timeout(R, 5.0));
  if (callbacks) {  // an env error in the middle of a run: the queue is cancelled, the run fails
    env.fail_at = env.steps + 9;
    const int rc = sfx_runner_run(R, 40);
    if (rc == 0) {
      std::fprintf(stderr, "FAIL %s: the injected env error did not fail the run\n", name);
      std::exit(1);
    }
    std::printf("  env error returned %d: %s\n", rc, sfx_last_error());
  }
  CK(sfx_runner_run(R, 60));  // usable afterwards
  stats("after", R);
  const int nrec = sfx_runner_recorded(R);
  int64_t off[10];
  CK(sfx_runner_layout(R, off));
  std::vector<unsigned char> stage((size_t)off[9]);
  int64_t meta[6];
  for (int i = 0; i < nrec; i += 7) CK(sfx_runner_get_record(R, i, stage.data(), meta));
  int64_t act[3];
  CK(sfx_runner_action(R, act));
  std::vector<float> p((size_t)sfx_head_numel(h));
  for (int t = 0; t < T; ++t) {
    CK(sfx_get_head(h, t, 0, p.data()));
    for (float x : p)
      if (!std::isfinite(x)) {
        std::fprintf(stderr, "FAIL %s: non-finite parameter in head %d\n", name, t);
        std::exit(1);
      }
  }
  std::printf("  records %d, action (%lld, %lld, %lld)\n", nrec, (long long)act[0], (long long)act[1],
              (long long)act[2]);
  CK(sfx_runner_destroy(R));
  CK(sfx_destroy(h));
}

// the engine's all-task update (sfx_update_all: graph-captured speculative rounds, settled by the
// next call) without the runner: device inputs, five steps, finite and moved parameters
void engine_scenario() {
  std::printf("engine update_all (T=3)\n");
  std::fflush(stdout);
  const int T = 3, B = 32;
  sfx_t h = make_handle(T);
  std::vector<float> s(B * NS), s1(B * NS), phi(B * D), g(B, 0.9f), p0((size_t)sfx_head_numel(h)), p1(p0.size());
  std::vector<int64_t> a(B);
  float *dS, *dS1, *dphi, *dg;
  int64_t* da;
  if (hipMalloc(&dS, 4 * s.size()) || hipMalloc(&dS1, 4 * s1.size()) || hipMalloc(&dphi, 4 * phi.size()) ||
      hipMalloc(&dg, 4 * g.size()) || hipMalloc(&da, 8 * a.size())) {
    std::fprintf(stderr, "FAIL engine: hipMalloc\n");
    std::exit(1);
  }
  CK(sfx_get_head(h, 1, 0, p0.data()));
  for (int it = 0; it < 5; ++it) {
    for (float& x : s) x = urand() - 0.5f;
    for (float& x : s1) x = urand() - 0.5f;
    for (float& x : phi) x = urand();
    for (int64_t& x : a) x = (int64_t)(urand() * A) % A;
    if (hipMemcpy(dS, s.data(), 4 * s.size(), hipMemcpyHostToDevice) ||
        hipMemcpy(dS1, s1.data(), 4 * s1.size(), hipMemcpyHostToDevice) ||
        hipMemcpy(dphi, phi.data(), 4 * phi.size(), hipMemcpyHostToDevice) ||
        hipMemcpy(dg, g.data(), 4 * g.size(), hipMemcpyHostToDevice) ||
        hipMemcpy(da, a.data(), 8 * a.size(), hipMemcpyHostToDevice)) {
      std::fprintf(stderr, "FAIL engine: hipMemcpy\n");
      std::exit(1);
    }
    CK(sfx_update_all(h, dS, da, dphi, dS1, dg, B, nullptr));
  }
  CK(sfx_get_head(h, 1, 0, p1.data()));  // settles the last step
  bool moved = false;
  for (size_t i = 0; i < p1.size(); ++i) {
    if (!std::isfinite(p1[i])) {
      std::fprintf(stderr, "FAIL engine: non-finite parameter\n");
      std::exit(1);
    }
    moved = moved || p1[i] != p0[i];
  }
  std::printf("  5 steps, parameters %s\n", moved ? "moved" : "UNCHANGED");
  std::fflush(stdout);
  (void)hipFree(dS);
  (void)hipFree(dS1);
  (void)hipFree(dphi);
  (void)hipFree(dg);
  (void)hipFree(da);
  CK(sfx_destroy(h));
}

// the drop-in's fused agent step (round 6): sfx_replay_put_gather (append + replay in one launch,
// copying the next state and φ into the fused step's fixed inputs), sfx_update_all_select (LMS with a
// host or a device reward, update, next GPI through host words), sfx_settle (host rounds forced on
// odd steps: the posted-verdict wait and the host rounds' selection), sfx_graph_stats
void dropin_scenario() {
  std::printf("drop-in fused step (T=3)\n");
  std::fflush(stdout);
  const int T = 3, B = 16, CAP = 64;
  sfx_t h = make_handle(T);
  float *rs, *rphi, *rs1, *S, *S1, *PHI, *G, *x, *lphi, *q, *st, *sp, *s1p, *rdev;
  int64_t *ra, *Aout, *task, *ap;
  if (hipMalloc(&rs, 4 * CAP * NS) || hipMalloc(&rphi, 4 * CAP * D) || hipMalloc(&rs1, 4 * CAP * NS) ||
      hipMalloc(&ra, 8 * CAP) || hipMalloc(&S, 4 * B * NS) || hipMalloc(&S1, 4 * B * NS) || hipMalloc(&PHI, 4 * B * D) ||
      hipMalloc(&G, 4 * B) || hipMalloc(&Aout, 8 * B) || hipMalloc(&x, 4 * NS) || hipMalloc(&lphi, 4 * D) ||
      hipMalloc(&q, 4 * T * A) || hipMalloc(&task, 8) || hipMalloc(&st, 4 * NS) || hipMalloc(&sp, 4 * D) ||
      hipMalloc(&s1p, 4 * NS) || hipMalloc(&ap, 8) || hipMalloc(&rdev, 4)) {
    std::fprintf(stderr, "FAIL dropin: hipMalloc\n");
    std::exit(1);
  }
  (void)hipMemset(rs, 0, 4 * CAP * NS);
  (void)hipMemset(rs1, 0, 4 * CAP * NS);
  (void)hipMemset(rphi, 0, 4 * CAP * D);
  (void)hipMemset(ra, 0, 8 * CAP);
  int64_t* hidx = nullptr;  // indices and γ in coherent host memory, as the drop-in hands them over
  if (sfx_host_alloc(8 * (B + B), reinterpret_cast<void**>(&hidx)) != 0) {
    std::fprintf(stderr, "FAIL dropin: sfx_host_alloc\n");
    std::exit(1);
  }
  float* hgam = reinterpret_cast<float*>(hidx + B);
  std::vector<float> hs(NS), hp(D), hs1(NS);
  for (int it = 0; it < 8; ++it) {
    for (float& v : hs) v = urand() - 0.5f;
    for (float& v : hp) v = urand();
    for (float& v : hs1) v = urand() - 0.5f;
    const int64_t a = (int64_t)(urand() * A) % A;
    const float r = urand();
    if (hipMemcpy(st, hs.data(), 4 * NS, hipMemcpyHostToDevice) || hipMemcpy(sp, hp.data(), 4 * D, hipMemcpyHostToDevice) ||
        hipMemcpy(s1p, hs1.data(), 4 * NS, hipMemcpyHostToDevice) || hipMemcpy(ap, &a, 8, hipMemcpyHostToDevice) ||
        hipMemcpy(rdev, &r, 4, hipMemcpyHostToDevice)) {
      std::fprintf(stderr, "FAIL dropin: hipMemcpy\n");
      std::exit(1);
    }
    const int j = it % CAP, size = it + 1 < B ? B : it + 1;
    for (int b = 0; b < B; ++b) {
      hidx[b] = b % 2 ? j : (int64_t)(urand() * size) % size;  // every other draw: the new row
      hgam[b] = 0.9f;
    }
    CK(sfx_replay_put_gather(nullptr, rs, rphi, rs1, ra, nullptr, j, st, sp, s1p, ap, x, lphi, hidx,
                             reinterpret_cast<const float*>(hgam), B, S, PHI, S1, Aout, G, NS, D));
    CK(sfx_debug_force_rerun(h, it % 2 ? 1 : -1));
    CK(sfx_update_all_select(h, S, Aout, PHI, S1, G, B, nullptr, x, 1, q, task, 1, lphi, r, it % 4 >= 2 ? rdev : nullptr,
                             0.05f));
    int hr = -1;
    CK(sfx_settle(h, &hr, nullptr));
    if ((it % 2) && hr <= 0) {
      std::fprintf(stderr, "FAIL dropin: forced host rounds did not run (%d)\n", hr);
      std::exit(1);
    }
  }
  std::vector<float> hq(T * A);
  int64_t ht = -1;
  if (hipMemcpy(hq.data(), q, 4 * T * A, hipMemcpyDeviceToHost) || hipMemcpy(&ht, task, 8, hipMemcpyDeviceToHost)) {
    std::fprintf(stderr, "FAIL dropin: hipMemcpy back\n");
    std::exit(1);
  }
  for (float v : hq)
    if (!std::isfinite(v)) {
      std::fprintf(stderr, "FAIL dropin: non-finite q\n");
      std::exit(1);
    }
  long long cap_n = 0, launches = 0, cached = 0;
  CK(sfx_graph_stats(h, &cap_n, &launches, &cached));
  std::printf("  8 steps, task %lld, graphs captured %lld, launches %lld, cached %lld\n", (long long)ht, cap_n, launches,
              cached);
  std::fflush(stdout);
  for (void* p : {(void*)rs, (void*)rphi, (void*)rs1, (void*)ra, (void*)S, (void*)S1, (void*)PHI, (void*)G, (void*)Aout,
                  (void*)x, (void*)lphi, (void*)q, (void*)task, (void*)st, (void*)sp, (void*)s1p, (void*)ap, (void*)rdev})
    (void)hipFree(p);
  CK(sfx_host_free(hidx));
  CK(sfx_destroy(h));
}

}  // namespace

int main() {
  // HOSTSAN_BISECT=1: the engine path first, then the all-task runner eager (no graphs), then
  // without pre-launched graphs -- the first one that stops narrows a hang down
  // HOSTSAN_BISECT=2: the all-task runner with the result published by its own k_publish (no
  // k_ver fold); HOSTSAN_BISECT=4: the plain all-task scenario alone
  if (const char* b = std::getenv("HOSTSAN_BISECT"); b && b[0] == '4') {
    scenario("all-task", 0, 3, false);
    std::printf("hostsan: bisect scenario clean\n");
    return 0;
  }
  if (const char* b = std::getenv("HOSTSAN_BISECT"); b && b[0] == '2') {
    setenv("SFX_FOLD_PUBLISH", "0", 1);
    scenario("all-task, separate k_publish", 0, 3, false);
    std::printf("hostsan: bisect scenario clean\n");
    return 0;
  }
  if (const char* b = std::getenv("HOSTSAN_BISECT"); b && b[0] == '1') {
    engine_scenario();
    setenv("SFX_GRAPHS", "0", 1);
    scenario("all-task, eager launches", 0, 3, false);
    unsetenv("SFX_GRAPHS");
    setenv("SFX_RUNNER_PIPELINE", "0", 1);
    scenario("all-task, graphs, no pre-launch", 0, 3, false);
    unsetenv("SFX_RUNNER_PIPELINE");
  }
  engine_scenario();
  dropin_scenario();
  scenario("all-task", 0, 3, false);
  scenario("all-task", 0, 4, true);
  scenario("active-task", 1, 3, true);
  scenario("tsf (K=3)", 2, 3, false);
  scenario("sharded, one rank, no collective", 3, 4, false);
  std::printf("hostsan: all scenarios clean\n");
  // every handle is destroyed above; skip the HIP / HSA runtimes' static teardown, where ASan's
  // device-allocator hook can recycle a quarantined device chunk after the HSA runtime unloaded
  // (round 5: "sanitizer_allocator_device.h:125 dev_runtime_unloaded_" at __cxa_finalize)
  std::fflush(nullptr);
  std::_Exit(0);
}
