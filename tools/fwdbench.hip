// Microbenchmark of the post-update forward launches (layers 1..3 of the C2 shape, T = 8, H = 256)
// in the group layouts the all-task step uses: the plain post-update forward (one group, 33 rows)
// and the look-ahead's four-group row-split launch, plus variants that isolate one
// factor each (target heads vs online, 2 / 3 / 4 column tiles, the 33-row groups in one 48-row tile or two, L2 flushed
// before each repetition).  It compiles libsfx's translation unit in (#include) to call run_fwd
// directly and reads the per-launch packet timestamps the bench instrumentation records.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/fwdbench tools/fwdbench.hip -ldl
#include "../deep-successor-features-for-transfer_amd/csrc/sfx.hip"

#include <cstdio>
#include <vector>

namespace {

struct Variant {
  const char* name;
  std::vector<FwdGroup> groups;
  int M;
  int tp;      // SFX_AHEAD_TP
  bool flush;  // stream 256 MB through the L2s before each repetition
  int tail = 1;  // SFX_FWD_TAIL
};

int run_variant(sfx_handle* h, const Variant& v, float* junk, size_t junk_n, int reps, double* per_layer) {
  h->ahead_tp = v.tp;
  h->fwd_tail = v.tail;
  FwdExtra vx;
  vx.l0 = 1;
  for (int l = 0; l < 3; ++l) per_layer[l] = 0.0;
  int n = 0;
  for (int it = 0; it < reps + 5; ++it) {
    if (v.flush) (void)hipMemsetAsync(junk, it & 0xff, junk_n * sizeof(float), h->stream);
    h->prof = it >= 5;
    const size_t before = h->prof_recs.size();
    int rc = SFX_OK;
    switch (v.groups.size()) {
      case 1: rc = run_fwd(h, {v.groups[0]}, v.M, nullptr, nullptr, vx); break;
      case 3: rc = run_fwd(h, {v.groups[0], v.groups[1], v.groups[2]}, v.M, nullptr, nullptr, vx); break;
      default: rc = run_fwd(h, {v.groups[0], v.groups[1], v.groups[2], v.groups[3]}, v.M, nullptr, nullptr, vx);
    }
    if (rc) return rc;
    if (hipStreamSynchronize(h->stream) != hipSuccess) return SFX_E_HIP;
    if (!h->prof) continue;
    for (size_t i = before; i < h->prof_recs.size(); ++i) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, h->prof_recs[i].a, h->prof_recs[i].b);
      per_layer[(i - before) % 3] += 1e3 * ms;
    }
    ++n;
    for (auto& r : h->prof_recs) {
      h->prof_pool.push_back(r.a);
      h->prof_pool.push_back(r.b);
    }
    h->prof_recs.clear();
  }
  h->prof = false;
  for (int l = 0; l < 3; ++l) per_layer[l] /= n;
  return SFX_OK;
}

}  // namespace

int main() {
  const int T = 8, acts[2] = {1, 1};
  sfx_t hh = nullptr;
  if (sfx_create(&hh, T, 17, 256, 2, acts, 7, 8, 32, 0, nullptr) != SFX_OK) {
    std::fprintf(stderr, "sfx_create: %s\n", sfx_last_error());
    return 1;
  }
  sfx_handle* h = hh;
  std::vector<float> p(sfx_head_numel(hh));
  unsigned s = 1;
  for (float& x : p) x = ((s = s * 1664525u + 1013904223u) >> 8) * (1.f / 16777216.f) * 0.1f - 0.05f;
  for (int t = 0; t < T; ++t)
    if (sfx_load_head(hh, t, 0, p.data()) || sfx_load_head(hh, t, 1, p.data())) return 1;
  const size_t junk_n = 64u << 20;  // 256 MB
  float* junk = nullptr;
  if (hipMalloc(&junk, junk_n * sizeof(float)) != hipSuccess) return 1;
  const FwdGroup gv{R_V, P_NEW, 0, 0, T, 33, 0}, gns{R_NS, P_NEW, 0, 0, T, 32, 1},
      gn1{R_NS1, P_NEW, 0, 0, T, 32, 1}, gnt{R_NS1T, P_TARGET, 0, 0, T, 32, 1}, gno{R_NS1T, P_NEW, 0, 0, T, 32, 1};
  const std::vector<Variant> vs = {
      {"plain R_V 33 rows (round-0 post-update)", {gv}, 33, 4, false, 0},
      {"plain R_V 33 rows, one 48-row tile", {gv}, 33, 4, false, 2},
      {"look-ahead 4 groups, TP 4, 33 rows in 2 tiles", {gv, gns, gn1, gnt}, 33, 4, false, 0},
      {"look-ahead 4 groups, TP 3, 33 rows in 2 tiles", {gv, gns, gn1, gnt}, 33, 3, false, 0},
      {"look-ahead 4 groups, TP 2, 33 rows in 2 tiles", {gv, gns, gn1, gnt}, 33, 2, false, 0},
      {"look-ahead 4 groups, TP 4, 48-row tail tile", {gv, gns, gn1, gnt}, 33, 4, false, 1},
      {"look-ahead 4 groups, TP 3, 48-row tail tile", {gv, gns, gn1, gnt}, 33, 3, false, 1},
      {"look-ahead 4 groups, TP 2, 48-row tail tile", {gv, gns, gn1, gnt}, 33, 2, false, 1},
      {"4 groups TP 3 tail, target group on online", {gv, gns, gn1, gno}, 33, 3, false, 1},
      {"look-ahead 4 groups TP 3 tail, L2 flushed", {gv, gns, gn1, gnt}, 33, 3, true, 1},
  };
  std::printf("%-48s %9s %9s %9s  (us per launch, mean of 200; layers 1 / 2 / 3)\n", "variant", "L1", "L2", "L3");
  for (const Variant& v : vs) {
    double us[3];
    if (run_variant(h, v, junk, junk_n, 200, us) != SFX_OK) {
      std::fprintf(stderr, "%s: %s\n", v.name, sfx_last_error());
      return 1;
    }
    std::printf("%-48s %9.2f %9.2f %9.2f\n", v.name, us[0], us[1], us[2]);
  }
  (void)hipFree(junk);
  sfx_destroy(hh);
  return 0;
}
