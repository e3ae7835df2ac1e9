// sfx.hip -- libsfx.so: C ABI (include/sfx.h) + launch orchestration for gfx950.
//
// Device state of one handle (T local ψ heads), all fp32:
//   online/adam_m/adam_v : [2][T][P]  packed heads, double-buffered (slot per head in `mask`)
//   target               : [T][P]
//   w, wm, wv            : [T][dpad]  reward weights and their Adam moments
//   step                 : [T]        Adam step per head (device-resident)
//   act                  : [role][T][actSize]   per-layer outputs, rows = max_batch + 1
//   dz                   : [T][actSize]         per-layer output gradients
//   rowloss              : [T][MMAX]            per-row TD loss of the last update
//   spec_next            : [T][MMAX]            speculated next actions of the all-task step
// Kernels take the whole geometry by value (sfx::Geo) and derive every pointer from it.
// Each entry point's launch sequence is captured once into a hipGraph (keyed by its
// arguments, including the slot mask) and replayed afterwards; SFX_GRAPHS=0 disables graphs.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <map>
#include <random>
#include <string>
#include <functional>
#include <tuple>
#include <utility>
#include <vector>

#include "sfx_kernels.h"
#include "sfx_gpiw.h"
#include "sfx_tsf.h"
#include "sfx_phi.h"
#include "../../include/sfx.h"

using namespace sfx;

static thread_local std::string g_err;

// RCCL is resolved at run time (dlopen), on the first communicator call: libsfx.so loads -- and
// runs every single-rank path -- on a host without RCCL; only the sharded collectives need it.
struct RcclApi {
  bool ok = false;
  std::string why;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t*, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
static const RcclApi& rccl() {
  static const RcclApi api = [] {
    RcclApi a;
    void* lib = nullptr;
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"})
      if ((lib = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (!lib) {
      a.why = "RCCL not found (dlopen librccl.so.1)";
      return a;
    }
    bool all = true;
    auto sym = [&](auto& f, const char* n) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(lib, n));
      all = all && f != nullptr;
    };
    sym(a.GetUniqueId, "ncclGetUniqueId");
    sym(a.CommInitRank, "ncclCommInitRank");
    sym(a.AllReduce, "ncclAllReduce");
    sym(a.CommDestroy, "ncclCommDestroy");
    sym(a.CommAbort, "ncclCommAbort");
    sym(a.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(a.CommSplit, "ncclCommSplit");
    sym(a.CommCount, "ncclCommCount");
    sym(a.CommUserRank, "ncclCommUserRank");
    sym(a.GetErrorString, "ncclGetErrorString");
    a.ok = all;
    if (!all) a.why = "RCCL lacks a needed entry point";
    return a;
  }();
  return api;
}

#define SFX_FAIL(code, msg) \
  do {                      \
    g_err = (msg);          \
    return (code);          \
  } while (0)

#define HIPCHK(x)                                                     \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_);         \
      return SFX_E_HIP;                                               \
    }                                                                 \
  } while (0)

#define LAUNCHCHK()                                                   \
  do {                                                                \
    hipError_t e_ = hipGetLastError();                                \
    if (e_ != hipSuccess) {                                           \
      g_err = std::string("kernel launch: ") + hipGetErrorString(e_); \
      return SFX_E_HIP;                                               \
    }                                                                 \
  } while (0)

#define RC(x)            \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)

namespace {

inline int align4(int x) { return (x + 3) & ~3; }
inline int align8(int x) { return (x + 7) & ~7; }  // weight blocks: 16-B aligned rows of the bf16 copy too
inline int cdiv(int a, int b) { return (a + b - 1) / b; }

struct GraphKey {
  int op, a0, a1, a2, a3, a4, a5, a6;
  unsigned long long mask;
  const void* p[12];
  bool operator<(const GraphKey& o) const { return std::memcmp(this, &o, sizeof(GraphKey)) < 0; }
};

// what the host reads back after a fused step: GPI task, greedy action, first re-run policy
struct StepOut {
  int64_t sel[2];
  int flag;
  unsigned done;  // k_ver arrivals when it publishes (reset by the last arrival)
  int posted;     // host copy: the final k_ver posted sel / flag (VerArgs::h_posted)
  int pad_;
};

}  // namespace

struct sfx_handle {
  int T = 0, n_s = 0, H = 0, nh = 0, A = 0, d = 0, O = 0, NL = 0, Mmax = 0, device = 0;
  int P = 0, Ptorch = 0, dpad = 0, actSize = 0;
  std::vector<LayerGeo> L;
  std::vector<int> actOff;
  hipStream_t stream = nullptr;  // caller's stream: everything is ordered on it
  hipStream_t cap = nullptr;     // private stream used only to capture graphs
  bool use_graphs = true;
  int fwd_tpw = FWD_TPW; // column tiles per workgroup (layer-0+1 forward, oversubscribed launches); SFX_FWD_TPW=1: one
  SelScratch* selk = nullptr;  // k_sel1m's per-head keys and arrival counter
  int ncu = 256;         // compute units of the device
  AdamHP hp_psi{1e-3, 0.0, 0.9, 0.999, 1e-8};
  AdamHP hp_w{1e-3, 0.0, 0.9, 0.999, 1e-8};
  int target_update_ev = 1000;
  std::vector<int> since_target, host_step;
  unsigned long long mask = 0;  // bit t: current slot of head t
  std::map<GraphKey, hipGraphExec_t> graphs;
  std::map<GraphKey, bool> graph_posts;  // fused steps whose final k_ver posts to hout (no copy)
  std::map<GraphKey, int> keys_seen;     // library-call keys launched eagerly once (run_graph)
  long long graph_eager = 0;             // those eager launches (sfx_graph_stats)
  Geo G{};
  // event instrumentation (bench roofline): packet timestamps per launch, eager only
  bool prof = false;
  struct ProfRec {
    int kind;
    double bytes;
    hipEvent_t a, b;
  };
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> prof_pool;
  // pending fused step (sfx_step_all -> sfx_step_finish)
  bool lazy_finish = false;  // sfx_update_all enqueued a step whose verdict settle() collects
  struct Pending {
    bool active = false, update = false, sel = false;
    int B = 0, use_gpi = 1, task = 0, sel_use_gpi = 1;
    const float *S = nullptr, *S1 = nullptr, *phi = nullptr, *gamma = nullptr, *s_next = nullptr;
    const int64_t* a = nullptr;
    float* losses = nullptr;
    // native runner look-ahead: pre -- this step's minibatch roles were filled by the
    // step before (no step-start forward; the gate resets the flag and runs the LMS); ax / aM --
    // the next step's minibatch states [NS | NS1] (aM rows each), forwarded by this step's final
    // round into the other copy of the minibatch roles
    bool pre = false;
    const float* ax = nullptr;
    int aM = 0;
    bool posted = false;  // the step's final k_ver posts its verdict to hout (wait on hout->posted)
    // sfx_update_all_select: the selection's q table [T*A] and GPI task of s_next (gpi_row's
    // q_out / task_out, as sfx_gpi writes them)
    float* q_out = nullptr;
    int64_t* task_out = nullptr;
    const unsigned long long* out_ind = nullptr;  // q_out / task_out through host words instead
  } pend;
  // step statistics
  long long steps_spec = 0, steps_fallback = 0, policies_rerun = 0, rounds_total = 0;
  long long graph_captures = 0, graph_launches = 0;  // sfx_graph_stats
  int force_rerun_from = -1;  // test hook: treat the speculation as failed from this policy on
  int spec_rounds = 2;        // speculative rounds launched on the device per fused step
  bool spec_rounds_auto = true;  // spec_rounds follows T_glob (auto_spec_rounds) until set explicitly
  // sharded heads (sfx_shard_*): this handle's heads are global [off, off + T) of Tg; w has Tg rows
  int Tg = 0, off = 0;
  struct sfx_tsf_state* tsf = nullptr;  // TSF-DQN state (sfx_tsf_setup)
  struct sfx_phi_state* phi = nullptr;  // learned φ (sfx_phi_setup)
  // collective of the sharded step (sfx_comm_init / sfx_set_comm / sfx_set_comm_host): all-reduce
  // (MAX) of fp32 buffers over the ranks that share the source tasks
  int comm_rank = 0, comm_world = 0;  // world 0: no communicator
  ncclComm_t comm = nullptr;
  bool comm_owned = false;
  // host rounds' own communicator (ncclCommSplit of comm, always owned): the collectives of a
  // step's host rounds (side stream) and of the pre-launched next step (step stream) never share
  // a communicator, so the runner pre-launches at N > 1 too
  ncclComm_t comm_rounds = nullptr;
  bool rounds_comm = false;  // coll_max uses comm_rounds (set while the runner runs host rounds)
  bool comm_dead = false;    // aborted after a collective timed out (sfx_runner_wait_timeout)
  std::string comm_err;
  long long* dstall = nullptr;  // test hook (sfx_debug_stall): one-shot stall of the sharded finish
  bool comm_force = false;  // SFX_RCCL_WORLD1=1: call RCCL even with one rank (tests)
  int (*host_ar)(void*, int32_t*, int) = nullptr;  // host transport: (ctx, host buffer, count)
  void* host_ar_ctx = nullptr;
  int32_t* host_ar_buf = nullptr;  // pinned staging of the host transport
  size_t host_ar_cap = 0;
  // sharded step, sortable int32: maxima buffers xb[2] ([Tg][Mmax][A] ++ q table [Tg][A]) and the
  // pre-step part xge ([Tg][Mmax][A]) of the fused path (shard_fused)
  int *xb[2] = {nullptr, nullptr}, *xge = nullptr;
  // sharded TSF step (runner schedule sharded_tsf): the active policy's GPI maxima [Mmax][A] and the
  // owner's h / w_task ++ the selection table [Ph + d + Tg * A] (sortable / raw int32 words)
  int *tsx = nullptr, *tsz = nullptr;
  int *qh = nullptr, *qhs = nullptr;  // local heads' own maxima terms (FwdArgs::qh), qhs inside qh's block
  bool shard_qa = true;  // SFX_SHARD_QA=0: maxima by separate k_qmax launches
  struct ShardPending {
    bool active = false;
    int B = 0;
    const float *S = nullptr, *S1 = nullptr, *phi = nullptr, *gamma = nullptr, *s_next = nullptr;
    const int64_t* a = nullptr;
  } spend;

  float *online = nullptr, *target = nullptr, *am = nullptr, *av = nullptr;
  float *w = nullptr, *wm = nullptr, *wv = nullptr;
  int* step = nullptr;
  int* dcancel = nullptr;  // Geo::cancel: written by runner gates, 0 otherwise
  AdamC* adamc = nullptr;
  float *act = nullptr, *dz = nullptr, *rowloss = nullptr;
  int64_t* spec_next = nullptr;  // [2][T][MMAX]: next actions of even / odd speculative rounds
  int* skip = nullptr;            // [T]: the policy repeats the previous round (BwdArgs::skip)
  unsigned long long* skipc = nullptr;  // [0] policies checked, [1] skipped (rounds >= 1)
  bool skip_rounds = true;        // SFX_SKIP=0: every round recomputes every policy
  StepOut* dout = nullptr;  // device
  // set by the runner while it captures a step: the final k_ver (with action selection)
  // publishes to pub_res instead of a separate k_publish; pub_folded reports that it did
  HostResult* pub_res = nullptr;
  const long long* pub_dctr = nullptr;
  bool pub_folded = false;
  bool fold_publish = true;  // SFX_FOLD_PUBLISH=0: always a separate k_publish
  // bf16 operand mode (sfx_set_precision): bf16 copies of the online [2][T][P] / target [T][P]
  // parameters feed the forward and dX MFMAs; fp32 master weights, moments and accumulators
  bool bf16 = false;
  __bf16* on16 = nullptr;
  __bf16* tg16 = nullptr;
  // split-N dX of wide layers (run_bwd): partial tiles and per-(head, tile) arrival counters
  int dxs_max = 1, dx_ntile = 1;
  float* dxpart = nullptr;
  unsigned* dxctr = nullptr;
  StepOut* hout = nullptr;  // pinned host (coherent, mapped: the final k_ver may write it)
  // set by sfx_step_all while it records a step: the final round's k_ver posts flag and selection
  // to hout (run_ver post_host), which then needs no copy after the step (hout_posted)
  bool post_hout = false, hout_posted = false;
  // host-coherent inputs of sfx_update_all_select, written before each launch: [0] the fused LMS's
  // reward (float), [1] / [2] the selection's q / task output pointers (GpiArgs::out_ind)
  unsigned long long* xin = nullptr;
  // recorded after a fused step's graph (which ends with the StepOut copy): sfx_step_finish waits
  // for the step itself, not for work queued behind it (the drop-in's speculative GPI graph)
  hipEvent_t ev_step = nullptr;
  // generation of the handle's device state: bumped by every launch and every parameter / moment /
  // role write made outside the native runner (touch()); a runner whose look-ahead chain was
  // recorded at another generation drops it (the minibatch roles or the weights it forwarded with
  // may have been overwritten in between: ADVICE r4)
  unsigned long long gen = 0;
  int in_runner = 0;  // > 0 while a sfx_runner_* call drives the handle

  int slot(int head) const { return (int)((mask >> head) & 1ull); }
  unsigned long long all_bits() const { return T >= 64 ? ~0ull : ((1ull << T) - 1ull); }
  float* online_cur(int head) const { return online + ((size_t)slot(head) * T + head) * P; }
  float* am_cur(int head) const { return am + ((size_t)slot(head) * T + head) * P; }
  float* av_cur(int head) const { return av + ((size_t)slot(head) * T + head) * P; }
  float* target_of(int head) const { return target + (size_t)head * P; }
  __bf16* on16_cur(int head) const { return on16 + ((size_t)slot(head) * T + head) * P; }
  __bf16* tg16_of(int head) const { return tg16 + (size_t)head * P; }
};

namespace {

inline void touch(sfx_handle* h) {
  if (!h->in_runner) ++h->gen;
}

void clear_graphs(sfx_handle* h) {
  for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
  h->graphs.clear();
  h->graph_posts.clear();
}

enum { K_FWD = 0, K_TDG = 1, K_BWD = 2, K_GPI = 3, K_LMS = 4, K_VER = 5, K_TSF = 6, K_NKIND = 7 };

hipEvent_t prof_event(sfx_handle* h) {
  if (!h->prof_pool.empty()) {
    hipEvent_t e = h->prof_pool.back();
    h->prof_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Launch a kernel; when instrumentation is on, the dispatch packet itself records start and
// stop timestamps into an event pair (hipExtLaunchKernelGGL: the timestamps rocprofv3 reads).
//
// The kernel is launched through the runtime entry point with an explicit argument array, not with
// `kern<<<...>>>` on the pointer: a triple-chevron call through a pointer to a kernel is an indirect
// call to its host handle, and a host build with clang's -fsanitize=function compiled that call
// away -- the call configuration was pushed and no kernel launched, so the runner's first update
// step never published (profiles/r05_ubsan_fn_disasm.txt).
template <typename... KArgs, std::size_t... I>
void launch_argv(sfx_handle* h, int kind, double bytes, const void* kern, dim3 grid, dim3 block,
                 std::tuple<KArgs...>& t, std::index_sequence<I...>) {
  void* argv[sizeof...(KArgs) > 0 ? sizeof...(KArgs) : 1] = {static_cast<void*>(&std::get<I>(t))...};
  if (!h->prof) {
    (void)hipLaunchKernel(kern, grid, block, argv, 0, h->stream);  // errors: LAUNCHCHK / hipGetLastError
    return;
  }
  hipEvent_t a = prof_event(h), b = prof_event(h);
  (void)hipExtLaunchKernel(kern, grid, block, argv, 0, h->stream, a, b, 0);
  h->prof_recs.push_back({kind, bytes, a, b});
}

template <typename... KArgs, typename... Args>
void launch(sfx_handle* h, int kind, double bytes, void (*kern)(KArgs...), dim3 grid, dim3 block, Args... args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "launch: argument count");
  touch(h);
  std::tuple<KArgs...> t(args...);  // each argument converted to the kernel's parameter type
  launch_argv(h, kind, bytes, reinterpret_cast<const void*>(kern), grid, block, t, std::index_sequence_for<KArgs...>{});
}

// graph ops of the library's entry points (sfx_gpi 1, sfx_select_action 2, sfx_update 3,
// sfx_step_all / sfx_update_all* 5, sfx_successors 21, sfx_test_actions 26, TSF 20 / 22-24,
// learned φ 30): the first call with a new key runs eagerly (run_graph)
bool eager_first_sight(int op) {
  return op == 1 || op == 2 || op == 3 || op == 5 || op == 21 || op == 26 || op == 20 || (op >= 22 && op <= 24) ||
         op == 30;
}

// Capture `body` (which launches on h->stream) into a graph keyed by `key`, then replay
// (launch = false: instantiate only -- sfx_runner_warm).
template <class F>
int run_graph(sfx_handle* h, const GraphKey& key, F body, bool launch_it = true) {
  touch(h);
  if (!h->use_graphs || h->prof) return launch_it ? body() : SFX_OK;
  auto it = h->graphs.find(key);
  if (it == h->graphs.end() && launch_it && eager_first_sight(key.op)) {
    // a library call whose key this handle has not seen: launch it eagerly and capture it only
    // when the same key comes again -- callers that pass fresh buffers every call (a new key each
    // time) would otherwise pay a capture and an instantiation per call
    int& n = h->keys_seen[key];
    if (n++ == 0) {
      if (h->keys_seen.size() > 4096) h->keys_seen.clear();
      h->graph_eager += 1;
      return body();
    }
  }
  if (it == h->graphs.end()) {
    hipStream_t saved = h->stream;
    h->stream = h->cap;
    HIPCHK(hipStreamBeginCapture(h->cap, hipStreamCaptureModeThreadLocal));
    const int rc = body();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(h->cap, &g);
    h->stream = saved;
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    HIPCHK(e);
    hipGraphExec_t ex = nullptr;
    const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPCHK(ei);
    if (h->graphs.size() > 256) clear_graphs(h);
    it = h->graphs.emplace(key, ex).first;
    h->graph_captures += 1;
  }
  if (launch_it) {
    HIPCHK(hipGraphLaunch(it->second, h->stream));
    h->graph_launches += 1;
  }
  return SFX_OK;
}

GraphKey make_key(int op, std::initializer_list<int> ints, unsigned long long mask,
                  std::initializer_list<const void*> ptrs) {
  GraphKey k;
  std::memset(&k, 0, sizeof(k));
  k.op = op;
  int* dst[7] = {&k.a0, &k.a1, &k.a2, &k.a3, &k.a4, &k.a5, &k.a6};
  int i = 0;
  for (int v : ints) *dst[i++] = v;
  k.mask = mask;
  i = 0;
  for (const void* p : ptrs) k.p[i++] = p;
  return k;
}

struct FwdExtra {
  int l0 = 0;            // first layer to run
  int lN = -1;           // layers [l0, lN) (-1: through the last)
  const float* xc = nullptr;  // layer-0 input of groups with xsel 3
  int lms_head = -1;     // LMS in block 0 of layer 0
  const float* lms_phi = nullptr;
  const float* lms_r = nullptr;
  const unsigned long long* lms_r_ind = nullptr;  // FwdArgs::lms_r_ind
  float lms_alpha = 0.f;
  int* flag = nullptr;   // reset to flag_value in block 0 of the first layer
  int flag_value = 0;
  // sharded step: GPI maxima accumulated by the last layer's tiles of group role qa_role
  int qa_role = -1, qa_M = 0, qa_row = -1, qa_task = 0, qa_use_gpi = 1;
  int *qa_all = nullptr, *qa_ge = nullptr, *qa_lt = nullptr, *qa_sel = nullptr;
  const int* skip = nullptr;  // post-update forward of rounds r >= 1 (FwdArgs::skip; one group)
  int* qh = nullptr;          // sharded rounds: the local heads' maxima terms (FwdArgs::qh)
  int* qhs = nullptr;
  // the first launch when it is the fused layer-0+1 one (k_fwd<true, 8, true, BF, TP>): issued by
  // the caller instead, with workgroups of its own riding along (TSF: k_fwd_tsf); returns true when
  // it launched
  std::function<bool(const FwdArgs& F, dim3 grid, double bytes)> ride_l0;
};

int run_fwd(sfx_handle* h, std::initializer_list<FwdGroup> groups, int M, const float* xa, const float* xb,
            const FwdExtra& ex = FwdExtra()) {
  FwdArgs F{};
  F.M = M;
  F.xa = xa;
  F.xb = xb;
  F.xc = ex.xc;
  F.mask = h->mask;
  F.lms_head = -1;
  F.qa_role = -1;
  F.skip = ex.skip;
  if (ex.skip && (ex.flag || ex.lms_head >= 0 || (ex.qa_role >= 0 && !ex.qh)))
    SFX_FAIL(SFX_E_STATE, "run_fwd: head skipping needs no LMS / flag / maxima");
  int ninst = 0;
  bool uniform = true;  // every group covers heads 0..T-1: XCD-aware grid possible
  FwdGroup* slots[4] = {&F.g0, &F.g1, &F.g2, &F.g3};
  for (const FwdGroup& g : groups) {
    *slots[F.ngroups++] = g;
    ninst += g.n;
    uniform = uniform && g.head0 == 0 && g.n == h->T;
  }
  F.xcd = uniform && h->T > 1 ? 1 : 0;
  F.nh = h->T;
  // layers 0 and 1 in one launch when layer 0 is small (its rows recomputed per tile in LDS)
  const bool fuse01 = ex.l0 == 0 && h->NL >= 3 && h->L[0].K <= L0_KMAX && h->L[0].N <= L0_NMAX && h->L[1].K % 32 == 0;
  const int lend = ex.lN >= 0 ? ex.lN : h->NL;
  if (fuse01 && lend < 2) SFX_FAIL(SFX_E_STATE, "run_fwd: the fused layer-0+1 launch needs layer 1");
  for (int l = fuse01 ? 1 : ex.l0; l < lend; ++l) {
    const LayerGeo& L = h->L[l];
    const bool l0 = fuse01 && l == 1;
    F.N = L.N;
    F.K = L.K;
    F.act = L.actOut;
    F.wOff = L.wOff;
    F.bOff = L.bOff;
    F.xOff = l == 0 || l0 ? -1 : h->actOff[l - 1];
    F.yOff = h->actOff[l];
    F.w0Off = h->L[0].wOff;
    F.b0Off = h->L[0].bOff;
    F.K0 = h->L[0].K;
    F.y0Off = h->actOff[0];
    const bool first = l == ex.l0 || l0;
    F.lms_head = first ? ex.lms_head : -1;
    F.lms_phi = ex.lms_phi;
    F.lms_r = ex.lms_r;
    F.lms_r_ind = first ? ex.lms_r_ind : nullptr;
    F.lms_alpha = ex.lms_alpha;
    F.flag = first ? ex.flag : nullptr;
    F.flag_value = ex.flag_value;
    const bool qa = ex.qa_role >= 0 && l == h->NL - 1;  // the maxima come from the ψ output layer
    // the vector path needs K % (256/NW) == 0 and 16-B aligned rows of X (layer 0 reads the caller's S)
    const bool aligned = l > 0 || ((uintptr_t)xa % 16 == 0 && (uintptr_t)xb % 16 == 0);
    bool own = false;  // groups with their own rows on an XCD grid: per-group row tiles (FwdArgs::rowsplit)
    if (F.xcd)
      for (const FwdGroup& g : groups) own = own || (g.m > 0 && g.m != M);
    F.ntN = cdiv(L.N, 16);
    // a group's last row tile takes up to 16 more rows (FwdArgs::tail; plain 8-wave vector launches):
    // on row-split launches with more 32-row tiles than CUs (the look-ahead's hidden layers: 640 ->
    // 512 tiles, paired into 256 workgroups; tools/fwdbench 6.8 / 6.4 us against 7.8 / 7.5 for 240
    // workgroups of 3 tiles without it -- it is slower where the tiles already fit the chip)
    long tiles32 = 0;
    for (const FwdGroup& g : groups) tiles32 += (long)F.ntN * cdiv(own && g.m > 0 ? g.m : M, 32) * g.n;
    F.tail = !l0 && !qa && (L.K % 32) == 0 && aligned && own && tiles32 > h->ncu ? 1 : 0;
    F.ntM = fwd_row_tiles(M, F.tail);
    F.tpw = 1;
    long tiles = (long)F.ntN * F.ntM * ninst;
    F.rowsplit = 0;
    if (own) {
      int* mt[4] = {&F.mt0, &F.mt1, &F.mt2, &F.mt3};
      int gi = 0;
      F.ntMs = 0;
      tiles = 0;
      for (const FwdGroup& g : groups) {
        *mt[gi++] = fwd_row_tiles(g.m > 0 ? g.m : M, F.tail);
        F.ntMs += *mt[gi - 1];
        tiles += (long)F.ntN * *mt[gi - 1] * g.n;
      }
      F.rowsplit = 1;
    }
    if (qa) {
      F.qa_role = ex.qa_role;
      F.qa_Tg = h->Tg;
      F.qa_off = h->off;
      F.qa_M = ex.qa_M;
      F.qa_all = ex.qa_all;
      F.qa_ge = ex.qa_ge;
      F.qa_lt = ex.qa_lt;
      F.qa_sel = ex.qa_sel;
      F.qa_row = ex.qa_row;
      F.qa_task = ex.qa_task;
      F.qa_use_gpi = ex.qa_use_gpi;
      F.qh = ex.qh;
      F.qhs = ex.qhs;
    }
    // two column tiles per workgroup (an L0 launch's in-tile layer 0 computed once for them, a
    // plain launch's X operands loaded once) when the tiles would put two workgroups on at least
    // half the CUs and, paired, fit the two workgroups a CU holds: C2's first forward of three roles
    // (384 tiles -> 192 workgroups, +1 %); the TSF look-ahead select's layer-0+1 and layer-2
    // launches (544 tiles: unpaired, the last 32 waited a whole workgroup body for a slot);
    // Hopper TSF's 288 tiles stay unpaired (pairing measured 1 % slower) (the look-ahead's
    // row-split launches pair above that too: 640 tiles of 32 x 16 measured 11.8 us unpaired, their
    // workgroups dispatched over 5 us)
    if (!qa && h->fwd_tpw > 1 && F.ntN > 1 && 2 * tiles >= 3L * h->ncu && (tiles <= 4L * h->ncu || F.rowsplit) &&
        (l0 || ((L.K % 32) == 0 && aligned)))
      F.tpw = h->fwd_tpw;
    const int ntNb = cdiv(F.ntN, F.tpw);
    const dim3 grid = F.xcd ? dim3(8 * cdiv(h->T, 8) * ntNb * (F.rowsplit ? F.ntMs : F.ntM * F.ngroups))
                            : dim3(ntNb, ninst, F.ntM);
    double by = 0.0;
    for (const FwdGroup& g : groups) {  // each group at its own rows
      const double m = g.m > 0 ? g.m : M;
      by += 4.0 * g.n * ((double)L.N * L.K + L.N + m * L.K + m * L.N);
      if (l0) by += 4.0 * g.n * ((double)h->L[0].N * h->L[0].K + h->L[0].N + m * h->L[0].K);
    }
    const bool tp2 = F.tpw > 1;
    const bool gemv = !l0 && !qa && M <= GEMV_M && L.N >= GEMV_N && L.K % 16 == 0 &&
                      (l > 0 || ((uintptr_t)xa % 16 == 0 && (uintptr_t)xb % 16 == 0));
    if (gemv) {
      launch(h, K_FWD, by, k_fwd_gemv, dim3(cdiv(L.N, 64), ninst), dim3(256), h->G, F);
    } else if (l0) {
      if (!(ex.ride_l0 && !F.xcd && ex.ride_l0(F, grid, by)))
        launch(h, K_FWD, by,
               tp2 ? (h->bf16 ? k_fwd<true, 8, true, true, 2> : k_fwd<true, 8, true, false, 2>)
                   : (h->bf16 ? k_fwd<true, 8, true, true> : k_fwd<true, 8, true>),
               grid, dim3(512), h->G, F);
    } else {  // (the tpw rule above requires the vector path)
      const bool vec = (L.K % 32) == 0 && aligned;
      launch(h, K_FWD, by,
             !vec ? k_fwd<false, 8, false>
                  : tp2 ? (h->bf16 ? k_fwd<true, 8, false, true, 2> : k_fwd<true, 8, false, false, 2>)
                        : (h->bf16 ? k_fwd<true, 8, false, true> : k_fwd<true, 8, false>),
             grid, dim3(512), h->G, F);
    }
  }
  LAUNCHCHK();
  return SFX_OK;
}

// GPI over many heads (sfx_gpiw.h): one workgroup per (row, WPC policies) instead of one per
// (policy, row) once a row's q table (T·A entries) outgrows a workgroup
bool wide_gpi(const sfx_handle* h) {
  return (long)h->T * h->A > 256 && h->d % 4 == 0 && h->d <= 16 && h->A <= WAMAX;
}

#define SFX_WIDE(K) (h->d == 4 ? K<1> : h->d == 8 ? K<2> : h->d == 12 ? K<3> : K<4>)

int run_tdg(sfx_handle* h, int pol0, int npol, int guess, int M, int use_gpi, const int64_t* a, const float* phi,
            const float* gamma, int64_t* next, int next_stride, int* flag = nullptr, const int* xmax = nullptr,
            int poloff = 0, const float* dz_scale = nullptr, const int64_t* prev = nullptr, bool skip = false) {
  const double nt = use_gpi ? h->T : 1;
  const double by = 4.0 * npol * M * (nt * h->O + 2.0 * h->O + 2.0 * h->d + 4);
  if (use_gpi && !xmax && !dz_scale && wide_gpi(h)) {
    TdgwArgs W{};
    W.M = M;
    W.pol0 = pol0;
    W.npol = npol;
    W.guess = guess;
    W.next_stride = next_stride;
    W.flag_value = h->T;
    W.a = a;
    W.phi = phi;
    W.gamma = gamma;
    W.next = next;
    W.flag = flag;
    W.prev = skip ? prev : nullptr;
    W.skip = skip ? h->skip : nullptr;
    W.skipc = skip ? h->skipc : nullptr;
    launch(h, K_TDG, by, SFX_WIDE(k_tdgw), dim3(M, cdiv(npol, WPC)), dim3(256), h->G, W);
    LAUNCHCHK();
    return SFX_OK;
  }
  TdgArgs A{};
  A.dz_scale = dz_scale;
  A.xmax = xmax;
  A.poloff = poloff;
  A.M = M;
  A.use_gpi = use_gpi;
  A.pol0 = pol0;
  A.npol = npol;
  A.guess = guess;
  A.flag = flag;
  A.flag_value = h->T;
  A.next_stride = next_stride;
  A.a = a;
  A.phi = phi;
  A.gamma = gamma;
  A.next = next;
  A.prev = skip ? prev : nullptr;
  A.skip = skip ? h->skip : nullptr;
  A.skipc = skip ? h->skipc : nullptr;
  launch(h, K_TDG, by, k_tdg, dim3(M, npol), dim3(256), h->G, A);
  LAUNCHCHK();
  return SFX_OK;
}

// K2 inputs for run_bwd: fused into the first backward launch when the 32-row LDS tiles fit,
// else launched as k_tdg right before it.
struct TdgSpec {
  int use_gpi = 1, guess = R_S1, next_stride = 0;
  const int64_t* a = nullptr;
  const float* gamma = nullptr;
  int64_t* next = nullptr;
  int* flag = nullptr;
  const int* xmax = nullptr;    // sharded heads: all-reduced GPI maxima [T_glob][M][A] (sortable)
  int poloff = 0;               // global index of local head 0
  // sharded step: the fused-TD launch re-initialises the next round's maxima (BwdArgs::xi_*)
  const int* xi_src = nullptr;
  int* xi_dst = nullptr;
  int xi_copy = 0, xi_n = 0;
  // rounds r >= 1: round r-1's next actions; policies that repeat them skip (BwdArgs::tdg_prev)
  const int64_t* prev = nullptr;
  bool skip = false;
  // learned φ (sfx_phi.inc): output gradient scaled by a device scalar
  const float* dz_scale = nullptr;
};

// 0: K2 as its own launch; 1: fused, d <= 8; 2: fused, d <= 16 (see tdg_rows)
int tdg_variant(const sfx_handle* h) {
  if ((h->d & 3) != 0 || h->O > TDG_ROWS_O || h->A > 128) return 0;
  const long ta = (long)h->T * h->A;
  if (h->d <= 8 && 32 * ta <= 256 * 8) return 1;
  if (h->d <= 16 && 32 * ta <= 256 * 4) return 2;
  return 0;
}

bool can_fuse_tdg(const sfx_handle* h) { return tdg_variant(h) != 0; }

struct BwdExtra {
  int inc_step = 1;
  bool fuse_v0 = false;  // post-update forward of layer 0 into vRole (rows S1 ++ s_next)
  int vRole = R_V;
  const float* v_x = nullptr;
  const float* v_xn = nullptr;
  bool skip_fwd = false;      // in: the caller skips the post-update forward of skipped heads
  const float* ax = nullptr;  // look-ahead rows of the fused forward (BwdArgs::ax), aM rows each
  int aM = 0, a_noskip = 0;
  bool* skip_armed = nullptr; // out: this round's launches decide and honour BwdArgs::skip
  // launch `li` (tiles `ntile` of one head, grid dim3(ntile)) issued by the caller instead, with
  // extra workgroups of its own riding along (TSF: k_bwd_tsf); returns true when it launched.
  // tail_at: the launch holding the loss tail and (not fused) the Adam step bump
  std::function<bool(int li, int tail_at, const BwdArgs& A, int ntile, double bytes)> ride;
};

bool can_fuse_v0(const sfx_handle* h, int vM) { return h->L[0].K <= KFUSE && vM * h->L[0].K <= VFUSE; }
// the fused forward with the look-ahead rows as well (2 aM rows after vM, 16-B aligned, whole float4s)
bool can_fuse_ahead(const sfx_handle* h, int vM, int aM) {
  const int K = h->L[0].K;
  return can_fuse_v0(h, vM) && ((vM * K + 3) & ~3) + 2 * aM * K <= VFUSE && (2 * aM * K) % 4 == 0;
}

int run_bwd(sfx_handle* h, int head0, int nhead, int M, const float* x0, const float* phi, const float* r,
            float* losses, const TdgSpec& td, const BwdExtra& ex = BwdExtra()) {
  const bool fuse = can_fuse_tdg(h) && ((uintptr_t)phi & 15) == 0 &&  // fused K2 reads φ rows as float4
                    (!td.xmax || 32 * h->A <= 1024);                     // and up to 4 maxima per thread
  if (!fuse && td.xi_dst) SFX_FAIL(SFX_E_STATE, "run_bwd: maxima re-initialisation needs the fused TD launch");
  // round skipping: decided in the fused TD launch (M <= 32: one row tile per policy) or, unfused,
  // by the TD launch's per-policy arrivals (tdg_skip_report)
  const bool armed = td.skip && (fuse ? M <= 32 : true);
  if (!fuse)
    RC(run_tdg(h, head0, nhead, td.guess, M, td.use_gpi, td.a, phi, td.gamma, td.next, td.next_stride, td.flag,
               td.xmax, td.poloff, td.dz_scale, td.prev, armed));
  BwdArgs A{};
  A.xcd = nhead > 1 ? 1 : 0;
  A.nhead = nhead;
  A.step_in_tail = fuse ? 0 : 1;
  A.tdg_use_gpi = td.use_gpi;
  A.tdg_guess = td.guess;
  A.tdg_next_stride = td.next_stride;
  A.tdg_a = td.a;
  A.tdg_gamma = td.gamma;
  A.tdg_next = td.next;
  A.tdg_xmax = td.xmax;
  A.tdg_poloff = td.poloff;
  A.flag = td.flag;
  A.flag_value = h->T;
  A.dz_scale = td.dz_scale;
  if (armed && fuse) {
    A.tdg_prev = td.prev;
    A.skip = h->skip;
    A.skipc = h->skipc;
    A.skip_v0 = ex.skip_fwd ? 1 : 0;
  }
  if (armed) {
    A.skip = h->skip;
    A.skip_v0 = ex.skip_fwd ? 1 : 0;
  }
  if (ex.skip_armed) *ex.skip_armed = armed;
  const int tail_at = fuse ? 1 : 0;  // launch index of the loss tail (needs every row's loss)
  const bool need_tail = losses || r || !fuse;  // losses, a w step or the Adam step bump
  const double tdg_bytes = 4.0 * nhead * M * ((td.use_gpi ? h->T : 1) * h->O + 2.0 * h->O + 2.0 * h->d + 4);
  A.M = M;
  A.head0 = head0;
  A.mask = h->mask;
  A.hp = h->hp_psi;
  A.hpw = h->hp_w;
  A.x0 = x0;
  A.phi = phi;
  A.r = r;
  A.train_w = r != nullptr;
  A.losses = losses;
  A.inc_step = ex.inc_step;
  auto dw_tiles = [&](int l) { return cdiv(h->L[l].N, 32) * cdiv(h->L[l].K, 64); };
  auto geo = [&](int l) {
    const LayerGeo& L = h->L[l];
    RoleGeo r{};
    r.N = L.N;
    r.K = L.K;
    r.wOff = L.wOff;
    r.bOff = L.bOff;
    r.actIn = L.actIn;
    r.xOff = l == 0 ? -1 : h->actOff[l - 1];
    r.dzOff = h->actOff[l];
    r.dzIn = l == 0 ? 0 : h->actOff[l - 1];
    return r;
  };
  // algorithmic bytes: dX reads W, dZ, X and writes dZ_{l-1}; dW reads dZ, X and does Adam's
  // read p,m,v + write p,m,v (24 B per parameter)
  auto dx_bytes = [&](int l) {
    const LayerGeo& L = h->L[l];
    return 4.0 * ((double)L.N * L.K + (double)M * L.N + 2.0 * M * L.K);
  };
  auto dw_bytes = [&](int l) {
    const LayerGeo& L = h->L[l];
    return 24.0 * ((double)L.N * L.K + L.N) + 4.0 * ((double)M * L.N + (double)M * L.K);
  };
  for (int l = h->NL - 1; l >= 1; --l) {
    const int li = h->NL - 1 - l;
    A.tdg = fuse && li == 0 ? 1 : 0;
    A.xi_src = A.tdg ? td.xi_src : nullptr;
    A.xi_dst = A.tdg ? td.xi_dst : nullptr;
    A.xi_copy = td.xi_copy;
    A.xi_n = td.xi_n;
    const double by = nhead * (dx_bytes(l) + (l + 1 <= h->NL - 1 ? dw_bytes(l + 1) : 0.0)) + (A.tdg ? tdg_bytes : 0.0);
    A.ra = geo(l);
    A.na = cdiv(M, 32) * cdiv(h->L[l].K, 16);
    // wide layers: the dX tiles split N in <= 256-wide chunks over workgroups (not in a fused
    // TD launch)
    A.dxs = 1;
    if (!A.tdg && h->dxpart && h->L[l].N > DX_SPLIT_N && M <= 32 * cdiv(h->Mmax, 32) &&
        nhead <= h->T) {
      A.dxs = cdiv(h->L[l].N, DX_SPLIT_N);
      A.dxpart = h->dxpart;
      A.dxctr = h->dxctr;
      A.na *= A.dxs;
    }
    if (l + 1 <= h->NL - 1) {
      A.rb = geo(l + 1);
      A.nb = dw_tiles(l + 1);
    } else {
      A.nb = 0;
    }
    A.nc = 0;
    A.tail = li == tail_at && need_tail ? 1 : 0;
    const int ntile = A.tdg ? A.na : A.na + A.nb + A.nc + A.tail;
    const dim3 grid = A.xcd ? dim3(8 * cdiv(nhead, 8) * ntile) : dim3(ntile, nhead);
    if (A.tdg && tdg_variant(h) == 1)  // d <= 8
      launch(h, K_BWD, by, k_bwd_tdg<2, 8>, grid, dim3(256), h->G, A);
    else if (A.tdg)
      launch(h, K_BWD, by, k_bwd_tdg<4, 4>, grid, dim3(256), h->G, A);
    else if (!(ex.ride && nhead == 1 && !A.xcd && ex.ride(li, tail_at, A, ntile, by)))
      launch(h, K_BWD, by, h->bf16 ? k_bwd<true> : k_bwd<false>, grid, dim3(256), h->G, A);
  }
  A.na = 0;
  A.dxs = 1;
  A.tdg = 0;
  A.xi_dst = nullptr;
  A.xi_src = nullptr;
  A.rb = geo(1);
  A.nb = dw_tiles(1);
  A.rc = geo(0);
  A.nc = dw_tiles(0);
  A.tail = h->NL - 1 == tail_at && need_tail ? 1 : 0;
  A.fuse_v0 = ex.fuse_v0 ? 1 : 0;
  A.vM = M + (ex.v_xn ? 1 : 0);
  A.vOff = h->actOff[0];
  A.vRole = ex.vRole;
  A.act0 = h->L[0].actOut;
  A.v_x = ex.v_x;
  A.v_xn = ex.v_xn;
  A.ax = ex.fuse_v0 ? ex.ax : nullptr;
  A.aM = ex.fuse_v0 && ex.ax ? ex.aM : 0;
  A.a_noskip = ex.a_noskip;
  const int ntile = A.nb + A.nc + A.tail;
  if (!(ex.ride && nhead == 1 && !A.xcd && ex.ride(h->NL - 1, tail_at, A, ntile, nhead * (dw_bytes(1) + dw_bytes(0)))))
    launch(h, K_BWD, nhead * (dw_bytes(1) + dw_bytes(0)), h->bf16 ? k_bwd<true> : k_bwd<false>,
           A.xcd ? dim3(8 * cdiv(nhead, 8) * ntile) : dim3(ntile, nhead), dim3(256), h->G, A);
  LAUNCHCHK();
  return SFX_OK;
}

GpiArgs gpi_args(int role, int rowoff, int row0, const float* w, float* psi, float* q, int64_t* task, int64_t* next,
                 int64_t* sel, int select_task, int use_gpi, int M) {
  GpiArgs A{};
  A.M = M;
  A.role = role;
  A.row0 = row0;
  A.rowoff = rowoff;
  A.select_task = select_task;
  A.use_gpi = use_gpi;
  A.w = w;
  A.psi_out = psi;
  A.q_out = q;
  A.task_out = task;
  A.next_out = next;
  A.sel_out = sel;
  return A;
}

int run_gpi(sfx_handle* h, const GpiArgs& A) {
  launch(h, K_GPI, 4.0 * A.M * ((double)h->T * h->O * (A.psi_out ? 2 : 1) + h->d + (A.q_out ? h->T * h->A : 0)),
         k_gpi, dim3(A.M), dim3(256), h->G, A);
  LAUNCHCHK();
  return SFX_OK;
}

int run_ver(sfx_handle* h, int M, int npol, bool sel, int post, const GpiArgs& g, const int64_t* spec,
            bool post_host = false) {
  VerArgs V{};
  V.M = M;
  V.post = post;
  V.npol = npol;
  V.sel = sel ? 1 : 0;
  V.spec_stride = MMAX;
  V.spec_next = spec;
  V.flag = &h->dout->flag;
  V.g = g;
  const int TA = h->T * h->A;
  V.rows = TA >= 256 ? 1 : (256 / TA < M ? 256 / TA : M);
  const bool wide = wide_gpi(h) && npol > 1;
  const dim3 grid = wide ? dim3(M, cdiv(npol, WPC) + 1) : dim3(npol + 1, cdiv(M, V.rows));
  if (sel && h->pub_res && h->fold_publish) {
    V.pub = h->pub_res;
    V.pub_dctr = h->pub_dctr;
    V.done = &h->dout->done;
    V.nblocks = (int)(grid.x * grid.y);
    h->pub_folded = true;
  } else if (post_host) {  // the step's verdict and selection straight to h->hout (no copy after)
    V.h_sel = h->hout->sel;
    V.h_flag = &h->hout->flag;
    V.h_posted = &h->hout->posted;
    V.done = &h->dout->done;
    V.nblocks = (int)(grid.x * grid.y);
    h->hout_posted = true;
  }
  const double by = 4.0 * (double)M * npol * h->T * h->O + 4.0 * h->T * h->O;
  if (wide)
    launch(h, K_VER, by, SFX_WIDE(k_verw), grid, dim3(256), h->G, V);
  else
    launch(h, K_VER, by, k_ver, grid, dim3(256), h->G, V);
  LAUNCHCHK();
  return SFX_OK;
}

void after_update(sfx_handle* h, int t) {
  h->host_step[t] += 1;
  h->since_target[t] += 1;
}

int maybe_sync_target(sfx_handle* h, int t) {
  if (h->since_target[t] >= h->target_update_ev) {
    touch(h);
    HIPCHK(hipMemcpyAsync(h->target_of(t), h->online_cur(t), sizeof(float) * h->P, hipMemcpyDeviceToDevice,
                          h->stream));
    if (h->bf16)
      HIPCHK(hipMemcpyAsync(h->tg16_of(t), h->on16_cur(t), sizeof(__bf16) * h->P, hipMemcpyDeviceToDevice,
                            h->stream));
    h->since_target[t] = 0;
  }
  return SFX_OK;
}

// torch packing <-> aligned packing of one head
void pack_head(const sfx_handle* h, const float* src, float* dst) {
  std::memset(dst, 0, sizeof(float) * h->P);
  size_t off = 0;
  for (const LayerGeo& L : h->L) {
    std::memcpy(dst + L.wOff, src + off, sizeof(float) * L.N * L.K);
    off += (size_t)L.N * L.K;
    std::memcpy(dst + L.bOff, src + off, sizeof(float) * L.N);
    off += L.N;
  }
}

void unpack_head(const sfx_handle* h, const float* src, float* dst) {
  size_t off = 0;
  for (const LayerGeo& L : h->L) {
    std::memcpy(dst + off, src + L.wOff, sizeof(float) * L.N * L.K);
    off += (size_t)L.N * L.K;
    std::memcpy(dst + off, src + L.bOff, sizeof(float) * L.N);
    off += L.N;
  }
}

bool valid_head(const sfx_handle* h, int t) { return h && t >= 0 && t < h->T; }
bool valid_w(const sfx_handle* h, int t) { return h && t >= 0 && t < h->Tg; }

// the bf16 copy of n parameters (round to nearest even), on the handle's stream
__global__ void k_to_bf16(const float* __restrict__ src, __bf16* __restrict__ dst, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = (__bf16)src[i];
}

int refresh_bf16(sfx_handle* h, const float* src, __bf16* dst, long long n) {
  touch(h);
  hipLaunchKernelGGL(k_to_bf16, dim3((unsigned)std::min<long long>(1024, (n + 255) / 256)), dim3(256), 0, h->stream, src,
                     dst, n);
  LAUNCHCHK();
  return SFX_OK;
}

void free_all(sfx_handle* h) {
  clear_graphs(h);
  for (auto& r : h->prof_recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (hipEvent_t e : h->prof_pool) (void)hipEventDestroy(e);
  for (void* p : {(void*)h->online, (void*)h->target, (void*)h->am, (void*)h->av, (void*)h->w, (void*)h->wm,
                  (void*)h->wv, (void*)h->step, (void*)h->dcancel, (void*)h->adamc, (void*)h->act, (void*)h->dz, (void*)h->rowloss, (void*)h->spec_next, (void*)h->skip, (void*)h->skipc,
                  (void*)h->dout, (void*)h->dxpart, (void*)h->dxctr, (void*)h->qh, (void*)h->selk})
    if (p) (void)hipFree(p);
  if (h->hout) (void)hipHostFree(h->hout);
  if (h->xin) (void)hipHostFree(h->xin);
  if (h->ev_step) (void)hipEventDestroy(h->ev_step);
  if (h->on16) (void)hipFree(h->on16);
  if (h->tg16) (void)hipFree(h->tg16);
  if (h->host_ar_buf) (void)hipHostFree(h->host_ar_buf);
  for (int* p : {h->tsx, h->tsz})
    if (p) (void)hipFree(p);
  for (int* p : {h->xb[0], h->xb[1]})  // xge lives in xb[0]'s block
    if (p) (void)hipFree(p);
  if (h->comm_rounds) (void)rccl().CommDestroy(h->comm_rounds);
  if (h->comm && h->comm_owned) (void)rccl().CommDestroy(h->comm);
  if (h->dstall) (void)hipFree(h->dstall);
  if (h->cap) (void)hipStreamDestroy(h->cap);
}

// Device rounds of the all-task step when the caller has not chosen (sfx_set_spec_rounds 0): the
// chain of the reference's in-order loop (agents/sfdqn.py:57-60) is T_glob policies deep, and the
// rounds a step needs grow with it -- measured (tools/spec_sim.py, the bench's synthetic Reacher
// stream, 2 device rounds): 10-13 % of steps need more at T = 8, 27 % at 16, 45-60 % at 32, 80 %
// at 64; with 3 they are 0-1 % at 16, 2-4 % at 32, 2-8 % at 64.  A third round in a step that
// verified after two costs its TD launch and early-exiting tiles (every policy skips); a host round
// costs a host round trip on top of the round -- at T = 8 the host rounds are cheaper overall
// (DESIGN.md §4), from 16 on the third device round.
int auto_spec_rounds(int T_glob) { return T_glob >= 16 ? 3 : 2; }

// Role of round r's post-update forward.  The launches of a round run in stream order, so every
// round can write the same role (round r's TD launch has read round r-1's values before its
// forward overwrites them) -- which lets a head whose policy repeats round r-1 skip its forward.
inline int round_role(const sfx_handle*, int) { return R_V; }
// next actions of speculative round r (two buffers: round r reads round r-1's while it writes)
inline int64_t* spec_buf(sfx_handle* h, int r) { return h->spec_next + (size_t)(r & 1) * h->T * MMAX; }

// One speculative round r of the all-task update: every policy takes its GPI next actions
// with heads t < i seen through role `guess` (round 0: the pre-step heads), every head
// updates from its read slot into its write slot, the post-update forward of S1 (++ s_next)
// lands in round_role(r).  Only a final round runs k_ver (flag the first policy whose actions
// were wrong; action selection): an earlier round's verdict would be overwritten unread.
int launch_round(sfx_handle* h, const sfx_handle::Pending& p, int r, bool final) {
  const int T = h->T, B = p.B;
  const int guess = r == 0 ? R_S1 : round_role(h, r - 1), out = round_role(h, r);
  const float* wsel = h->w + (size_t)p.task * h->dpad;
  TdgSpec td;
  td.use_gpi = p.use_gpi;
  td.guess = guess;
  td.a = p.a;
  td.gamma = p.gamma;
  td.next = spec_buf(h, r);
  td.next_stride = MMAX;
  td.flag = &h->dout->flag;
  td.prev = r > 0 ? spec_buf(h, r - 1) : nullptr;
  td.skip = h->skip_rounds;
  BwdExtra bx;
  bx.inc_step = r == 0 ? 1 : 0;  // later rounds redo the same optimizer step
  bool armed = false;
  bx.skip_fwd = true;  // one role for every round (round_role)
  bx.skip_armed = &armed;
  // the s_next row rides along in every round that a later round may skip heads after: a skipped
  // head's row must already be in the role when the final round's selection reads it
  const bool want_sel = p.sel && (final || bx.skip_fwd);
  bx.fuse_v0 = can_fuse_v0(h, B + 1);
  bx.vRole = out;
  bx.v_x = p.S1;
  bx.v_xn = want_sel ? p.s_next : nullptr;
  const int vM = B + (want_sel ? 1 : 0);
  // look-ahead: the final round (device or host) also forwards the next step's minibatch into the
  // other copy of the minibatch roles; the first round that does (the last device round) computes
  // them for every head, skipped or not -- later host rounds skip them with the rest of a head.
  // (Forwarding them in round 0 instead, so that an all-skip round 1 leaves its forwards empty,
  // measured 9 % slower: DESIGN.md §8.)
  const bool ahead = final && p.ax && p.aM > 0 && bx.fuse_v0 && can_fuse_ahead(h, vM, p.aM);
  const int a_noskip = ahead && r <= h->spec_rounds - 1 ? 1 : 0;
  if (ahead) {
    bx.ax = p.ax;
    bx.aM = p.aM;
    bx.a_noskip = a_noskip;
  }
  RC(run_bwd(h, 0, T, B, p.S, p.phi, nullptr, p.losses, td, bx));
  if (bx.fuse_v0) {
    FwdExtra vx;
    vx.l0 = 1;
    vx.skip = armed && r > 0 && bx.skip_fwd ? h->skip : nullptr;
    if (ahead)
      RC(run_fwd(h, {{out, P_NEW, 0, 0, T, vM, 0}, {R_NS, P_NEW, 0, 0, T, p.aM, a_noskip},
                     {R_NS1, P_NEW, 0, 0, T, p.aM, a_noskip}, {R_NS1T, P_TARGET, 0, 0, T, p.aM, a_noskip}},
                 std::max(vM, p.aM), nullptr, nullptr, vx));
    else
      RC(run_fwd(h, {{out, P_NEW, 0, 0, T}}, vM, nullptr, nullptr, vx));
  } else {
    RC(run_fwd(h, {{out, P_NEW, 2, 0, T}}, B, p.S1, p.S1));
  }
  if (!final) return SFX_OK;
  const bool sel = p.sel && bx.fuse_v0;
  const bool verify = p.use_gpi != 0;
  GpiArgs gs = gpi_args(out, B, 0, wsel, nullptr, p.q_out, p.task_out, nullptr, h->dout->sel, p.task, p.sel_use_gpi, 1);
  gs.out_ind = p.out_ind;
  // the ver launch posts the verdict to the host itself when nothing after it changes the selection
  if (verify || sel)
    RC(run_ver(h, B, verify ? T : 1, sel, out, gs, spec_buf(h, r), h->post_hout && (sel || !p.sel)));
  if (p.sel && !bx.fuse_v0) {  // selection through the plain forward path
    RC(run_fwd(h, {{R_A, P_NEW, 1, 0, T}}, 1, p.s_next, nullptr));
    gs.role = R_A;
    gs.rowoff = 0;
    RC(run_gpi(h, gs));
  }
  return SFX_OK;
}

// The fused step: LMS + forward of the minibatch, then `rounds` speculative rounds (or just
// LMS + action selection when there is no minibatch yet).
// SFDQN.get_Q_values + action choice for one state (sfdqn.py:577-596; agents/sfdqn.py:39-45):
// forward of every head on s, GPI with w of `task`, selection into out[2] = (c, a).
// With `pub` (runner steps) the step's result is published after the selection: inside k_sel1m, or
// by k_publish after k_gpi.
// the look-ahead TSF forward's tail riding along in the selection launch (k_sel1m_tsft)
struct TsfTail {
  TsfArgs A;  // fwd_mode 2
  const float* gfl;
  int nblk;
  double bytes;
};
int select_pick(sfx_handle* h, int task, int use_gpi, float* q, int64_t* out, const SelPub* pub,
                const TsfTail* tail = nullptr);
int select_body(sfx_handle* h, const float* s, int task, int use_gpi, float* q, int64_t* out,
                const SelPub* pub = nullptr) {
  RC(run_fwd(h, {{R_A, P_ONLINE, 1, 0, h->T}}, 1, s, nullptr));
  return select_pick(h, task, use_gpi, q, out, pub);
}

// the choice from role R_A row 0 (GPI with w of `task`, or `task`'s own q) and the publication
int select_pick(sfx_handle* h, int task, int use_gpi, float* q, int64_t* out, const SelPub* pub,
                const TsfTail* tail) {
  const GpiArgs g = gpi_args(R_A, 0, 0, h->w + (size_t)task * h->dpad, nullptr, q, nullptr, nullptr, out, task, use_gpi, 1);
  const int TA = h->T * h->A;
  if (h->T <= 64 && h->A <= 256) {  // one workgroup per head, the last one picks
    const SelPub P = pub ? *pub : SelPub{};
    const dim3 grid(h->T), block((unsigned)(cdiv(h->A, 64) * 64));
    const double by = 4.0 * ((double)TA * h->d + h->d + (q ? TA : 0));
    if (tail) {  // the TSF tail's workgroups first, 256-thread workgroups
      void (*k)(Geo, GpiArgs, SelPub, SelScratch*, TsfArgs, const float*, int) = nullptr;
      const int vw = h->d % 4 == 0 ? 4 : h->d % 2 == 0 ? 2 : 1;
      const int np = tail->A.np;
#define SFX_SEL_TAIL(V) \
  k = np == 4 ? k_sel1m_tsft<V, 4> : np == 8 ? k_sel1m_tsft<V, 8> : np == 16 ? k_sel1m_tsft<V, 16> : k_sel1m_tsft<V, 32>
      if (vw == 4)
        SFX_SEL_TAIL(4);
      else if (vw == 2)
        SFX_SEL_TAIL(2);
      else
        SFX_SEL_TAIL(1);
#undef SFX_SEL_TAIL
      launch(h, K_GPI, by + tail->bytes, k, dim3(tail->nblk + h->T), dim3(256), h->G, g, P, h->selk, tail->A,
             tail->gfl, tail->nblk);
      LAUNCHCHK();
      return SFX_OK;
    }
    if (h->d % 4 == 0)
      launch(h, K_GPI, by, k_sel1m<4>, grid, block, h->G, g, P, h->selk);
    else if (h->d % 2 == 0)
      launch(h, K_GPI, by, k_sel1m<2>, grid, block, h->G, g, P, h->selk);
    else
      launch(h, K_GPI, by, k_sel1m<1>, grid, block, h->G, g, P, h->selk);
    LAUNCHCHK();
    return SFX_OK;
  }
  RC(run_gpi(h, g));
  if (pub && pub->res) {
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, h->stream, (const int64_t*)out, pub->flag, pub->res, pub->dctr,
                       pub->cancel, pub->nonfin);
    LAUNCHCHK();
  }
  return SFX_OK;
}

// DeepSF.update_successor of one head (sfdqn.py:303-371): forwards, GPI / own-ψ next actions,
// TD target, backward + Adam (+ l2 and the w step when r is given).  Launches only.
// pre: the previous runner step's look-ahead select (select_ahead_body) already forwarded this
// minibatch with the current heads into the roles this step reads: start at the TD target.
int update_body(sfx_handle* h, int policy, const float* S, const int64_t* a, const float* r, const float* phi,
                const float* S1, const float* gamma, int B, int use_gpi, float* losses, int64_t* next,
                bool pre = false) {
  if (pre) {
  } else if (use_gpi) {
    RC(run_fwd(h, {{R_S, P_ONLINE, 1, policy, 1}, {R_S1T, P_TARGET, 2, policy, 1}, {R_S1, P_ONLINE, 2, 0, h->T}}, B,
               S, S1));
  } else {
    RC(run_fwd(h, {{R_S, P_ONLINE, 1, policy, 1}, {R_S1T, P_TARGET, 2, policy, 1}, {R_S1, P_ONLINE, 2, policy, 1}},
               B, S, S1));
  }
  TdgSpec td;
  td.use_gpi = use_gpi;
  td.a = a;
  td.gamma = gamma;
  td.next = next;
  td.next_stride = B;
  return run_bwd(h, policy, 1, B, S, phi, r, losses, td);
}

// TSFDQN.update_successor (sfx_tsf.inc)
int tsf_body(sfx_handle* h, int policy, const float* S, const int64_t* a, const float* r, const float* phi,
             const float* S1, const float* gamma, int B, int use_gpi, float* losses, int64_t* next,
             const int* xmax = nullptr, bool pre = false);
int tsf_fwd_with(sfx_handle* h, int policy, int B, const float* S, const float* S1, const float* phi,
                 const std::function<int(const FwdExtra&)>& fwd, const float* xc, int mode = 0);
bool tsf_tail_rider(sfx_handle* h, int policy, int B, const float* S, const float* S1, const float* phi, TsfTail* out);

// The action for s_next (select_body) with the look-ahead of the active-task / TSF runner steps
// (DESIGN.md §5): the next step's minibatch -- states ax[0, B), next states ax[B, 2B), TSF: its φ
// rows axphi -- is forwarded with this step's post-update heads into the other copy of the
// minibatch roles: ψ(S1) of every head (R_NS1; the next step's GPI), ψ(S) and ψ⁻(S1) of the active
// head (R_NS, R_NS1T) and, for TSF, its φ̃ and flow states (the TSF forward riding in the first
// launch) -- so the next step starts at its TD target.  Layers 0 .. NL-2 of the selection row
// (R_A, its own group) and of the minibatch share launches; then the selection's last layer, the
// choice and the publication; the minibatch's last layer comes after them, so it runs while the
// host turns the published action into the next step's inputs.
// task: the active LOCAL head, or -1 when another rank owns it (the sharded TSF schedule: this
// rank forwards the next minibatch's S1 through its heads only).  pick: the selection in place of
// select_pick (sharded: this rank's q-table slice, the all-reduce, the pick and its publication).
int select_ahead_body(sfx_handle* h, const float* s, const float* ax, const float* axphi, int B, int task,
                      int use_gpi, int64_t* out, const SelPub* pub, const std::function<int()>* pick = nullptr) {
  const int T = h->T, n_s = h->n_s;
  const float* S = ax;
  const float* S1 = ax + (size_t)B * n_s;
  const auto early = [&](const FwdExtra& fx0) -> int {
    FwdExtra fx = fx0;
    fx.lN = h->NL - 1;
    fx.xc = s;
    if (task < 0) return run_fwd(h, {{R_A, P_ONLINE, 3, 0, T, 1, 0}, {R_NS1, P_ONLINE, 2, 0, T, B, 0}}, B, S, S1, fx);
    return run_fwd(h, {{R_A, P_ONLINE, 3, 0, T, 1, 0}, {R_NS1, P_ONLINE, 2, 0, T, B, 0}, {R_NS, P_ONLINE, 1, task, 1, B, 0},
                       {R_NS1T, P_TARGET, 2, task, 1, B, 0}},
                   B, S, S1, fx);
  };
  // TSF: the chains in the first launch, the Linear of g and φ̃ (the tail) in the selection
  // launch when it can take them, so they run beside the selection instead of after the chains
  TsfTail tail;
  const bool split = axphi && !pick && task >= 0 && T <= 64 && h->A <= 256 &&
                     tsf_tail_rider(h, task, B, S, S1, axphi, &tail);
  if (axphi && task >= 0)
    RC(tsf_fwd_with(h, task, B, S, S1, axphi, early, s, split ? 1 : 0));
  else
    RC(early(FwdExtra()));
  FwdExtra last;
  last.l0 = h->NL - 1;
  RC(run_fwd(h, {{R_A, P_ONLINE, 3, 0, T}}, 1, nullptr, nullptr, last));
  if (pick)
    RC((*pick)());
  else
    RC(select_pick(h, task, use_gpi, nullptr, out, pub, split ? &tail : nullptr));
  if (task < 0) return run_fwd(h, {{R_NS1, P_ONLINE, 2, 0, T}}, B, nullptr, nullptr, last);
  return run_fwd(h, {{R_NS1, P_ONLINE, 2, 0, T}, {R_NS, P_ONLINE, 1, task, 1}, {R_NS1T, P_TARGET, 2, task, 1}}, B,
                 nullptr, nullptr, last);
}


int launch_step_all(sfx_handle* h, const sfx_handle::Pending& p, int lms_task, const float* lms_phi, const float* lms_r,
                    float lms_alpha, int rounds) {
  const int T = h->T, B = p.B;
  FwdExtra ex;
  ex.lms_head = lms_task;
  ex.lms_phi = lms_phi;
  ex.lms_r = lms_r;
  if (h->xin && lms_r == reinterpret_cast<const float*>(h->xin + 3)) {  // sfx_update_all_select, device reward
    ex.lms_r = nullptr;
    ex.lms_r_ind = h->xin + 3;
  }
  ex.lms_alpha = lms_alpha;
  ex.flag = &h->dout->flag;
  ex.flag_value = T;
  if (!p.update) {
    const float* wsel = h->w + (size_t)p.task * h->dpad;
    RC(run_fwd(h, {{R_A, P_ONLINE, 1, 0, T}}, 1, p.s_next, nullptr, ex));
    GpiArgs gs = gpi_args(R_A, 0, 0, wsel, nullptr, p.q_out, p.task_out, nullptr, h->dout->sel, p.task,
                          p.sel_use_gpi, 1);
    gs.out_ind = p.out_ind;
    return run_gpi(h, gs);
  }
  // a look-ahead step (p.pre) starts at its TD launch: the step before forwarded its minibatch
  // into these roles, its gate reset the flag and ran the LMS
  if (!p.pre)
    RC(run_fwd(h, {{R_S, P_ONLINE, 1, 0, T}, {R_S1T, P_TARGET, 2, 0, T}, {R_S1, P_ONLINE, 2, 0, T}}, B, p.S, p.S1, ex));
  for (int r = 0; r < rounds; ++r) RC(launch_round(h, p, r, r == rounds - 1));
  return SFX_OK;
}

}  // namespace

// The drop-in's agents.buffer ring (sfx/dropin/agents/buffer.py; agents/buffer.py:34-82): one
// launch appends a transition's row to every field, one launch gathers a minibatch -- in place of
// a framework copy per field and an index_select per field.
__global__ void k_replay_put(float* __restrict__ rs, float* __restrict__ rphi, float* __restrict__ rs1,
                             int64_t* __restrict__ ra, long long j, const float* __restrict__ s,
                             const float* __restrict__ phi, const float* __restrict__ s1, const int64_t* __restrict__ a,
                             int n_s, int d) {
  for (int k = threadIdx.x; k < n_s; k += blockDim.x) {
    rs[j * n_s + k] = s[k];
    rs1[j * n_s + k] = s1[k];
  }
  for (int k = threadIdx.x; k < d; k += blockDim.x) rphi[j * d + k] = phi[k];
  if (threadIdx.x == 0) ra[j] = *a;
}

// agents/buffer.py append (:62-82) and the replay right after it (:34-60) in one launch: workgroup B
// writes ring row j from the new transition (and copies its next state / φ into s1c / phic, the
// fixed inputs of a fused selection and LMS, when given); workgroup b < B gathers row idx[b] --
// from the new transition's own vectors when idx[b] == j (that row is being written beside it).
struct PutGather {
  float *rs, *rphi, *rs1;
  int64_t* ra;
  const float* rg;  // γ ring on the device, or null: γ from gam
  long long j;
  const float *s, *phi, *s1;
  const int64_t* a;
  float *s1c, *phic;
  const int64_t* idx;
  const float* gam;
  float *S, *PHI, *S1, *G;
  int64_t* A;
  int B, n_s, d;
};
__global__ void k_replay_put_gather(PutGather P) {
  const int b = blockIdx.x, n_s = P.n_s, d = P.d;
  if (b == P.B) {
    for (int k = threadIdx.x; k < n_s; k += blockDim.x) {
      P.rs[P.j * n_s + k] = P.s[k];
      const float v = P.s1[k];
      P.rs1[P.j * n_s + k] = v;
      if (P.s1c) P.s1c[k] = v;
    }
    for (int k = threadIdx.x; k < d; k += blockDim.x) {
      const float v = P.phi[k];
      P.rphi[P.j * d + k] = v;
      if (P.phic) P.phic[k] = v;
    }
    if (threadIdx.x == 0) P.ra[P.j] = *P.a;
    return;
  }
  const long long i = P.idx[b];
  const bool fresh = i == P.j;
  const float* xs = fresh ? P.s : P.rs + i * n_s;
  const float* xs1 = fresh ? P.s1 : P.rs1 + i * n_s;
  const float* xphi = fresh ? P.phi : P.rphi + i * d;
  for (int k = threadIdx.x; k < n_s; k += blockDim.x) {
    P.S[(size_t)b * n_s + k] = xs[k];
    P.S1[(size_t)b * n_s + k] = xs1[k];
  }
  for (int k = threadIdx.x; k < d; k += blockDim.x) P.PHI[(size_t)b * d + k] = xphi[k];
  if (threadIdx.x == 0) {
    P.A[b] = fresh ? *P.a : P.ra[i];
    P.G[b] = P.rg ? P.rg[i] : P.gam[b];
  }
}

// workgroup b: row idx[b] of each field; γ from the packed copy (gam) or from the ring (rg)
__global__ void k_replay_gather(const float* __restrict__ rs, const float* __restrict__ rphi,
                                const float* __restrict__ rs1, const int64_t* __restrict__ ra,
                                const float* __restrict__ rg, const int64_t* __restrict__ idx,
                                const float* __restrict__ gam, float* __restrict__ S, float* __restrict__ PHI,
                                float* __restrict__ S1, int64_t* __restrict__ Aout, float* __restrict__ G, int n_s,
                                int d) {
  const int b = blockIdx.x;
  const long long i = idx[b];
  for (int k = threadIdx.x; k < n_s; k += blockDim.x) {
    S[(size_t)b * n_s + k] = rs[i * n_s + k];
    S1[(size_t)b * n_s + k] = rs1[i * n_s + k];
  }
  for (int k = threadIdx.x; k < d; k += blockDim.x) PHI[(size_t)b * d + k] = rphi[i * d + k];
  if (threadIdx.x == 0) {
    Aout[b] = ra[i];
    G[b] = rg ? rg[i] : gam[b];
  }
}

// A launch whose final k_ver posts the verdict to host memory (VerArgs::h_posted): wait for that
// word -- it lands before the launch's completion signal reaches the host, and polling it skips
// the runtime's wake-up.  Bounded (1 s); false when it did not come (the caller then waits for
// the launch itself, which reports any error).
bool wait_posted(sfx_handle* h) {
  volatile int* posted = &h->hout->posted;
  const auto t0 = std::chrono::steady_clock::now();
  for (long spins = 0; !*posted; ++spins)
    if ((spins & 1023) == 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 1.0)
      return false;
  std::atomic_thread_fence(std::memory_order_acquire);
  return true;
}

// sfx_update_all returns once its step is enqueued; the speculation verdict -- and host rounds,
// should the device rounds leave a policy unverified -- is collected by the next API call on the
// handle (every entry point settles first), so the host never waits on a step it has not asked
// a result of.
static int settle(sfx_handle* h) {
  if (!h || !h->lazy_finish) return SFX_OK;
  h->lazy_finish = false;
  return sfx_step_finish(h, nullptr);
}

extern "C" {

const char* sfx_version(void) { return "sfx 0.3 gfx950 fp32-mfma graphs speculative-gpi"; }

int sfx_replay_put(void* stream, float* rs, float* rphi, float* rs1, int64_t* ra, long long j, const float* s,
                   const float* phi, const float* s1, const int64_t* a, int n_s, int d) {
  if (!rs || !rphi || !rs1 || !ra || !s || !phi || !s1 || !a || j < 0 || n_s < 1 || d < 1)
    SFX_FAIL(SFX_E_ARG, "sfx_replay_put: bad arguments");
  hipLaunchKernelGGL(k_replay_put, dim3(1), dim3(64), 0, (hipStream_t)stream, rs, rphi, rs1, ra, j, s, phi, s1, a, n_s,
                     d);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_host_alloc(size_t bytes, void** out) {
  if (!out || bytes == 0) SFX_FAIL(SFX_E_ARG, "sfx_host_alloc: bad arguments");
  *out = nullptr;
  if (hipHostMalloc(out, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    SFX_FAIL(SFX_E_HIP, "sfx_host_alloc: hipHostMalloc failed");
  std::memset(*out, 0, bytes);
  return SFX_OK;
}

int sfx_host_free(void* p) {
  if (p) (void)hipHostFree(p);
  return SFX_OK;
}

int sfx_replay_gather(void* stream, const float* rs, const float* rphi, const float* rs1, const int64_t* ra,
                      const float* rg, const int64_t* idx, const float* gam, int B, float* S, float* PHI, float* S1,
                      int64_t* A, float* G, int n_s, int d) {
  if (!rs || !rphi || !rs1 || !ra || !idx || (!rg && !gam) || B < 1 || !S || !PHI || !S1 || !A || !G || n_s < 1 ||
      d < 1)
    SFX_FAIL(SFX_E_ARG, "sfx_replay_gather: bad arguments");
  hipLaunchKernelGGL(k_replay_gather, dim3(B), dim3(64), 0, (hipStream_t)stream, rs, rphi, rs1, ra, rg, idx, gam, S,
                     PHI, S1, A, G, n_s, d);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_replay_put_gather(void* stream, float* rs, float* rphi, float* rs1, int64_t* ra, const float* rg, long long j,
                          const float* s, const float* phi, const float* s1, const int64_t* a, float* s1_copy,
                          float* phi_copy, const int64_t* idx, const float* gam, int B, float* S, float* PHI, float* S1,
                          int64_t* A, float* G, int n_s, int d) {
  if (!rs || !rphi || !rs1 || !ra || j < 0 || !s || !phi || !s1 || !a || !idx || (!rg && !gam) || B < 1 || !S ||
      !PHI || !S1 || !A || !G || n_s < 1 || d < 1)
    SFX_FAIL(SFX_E_ARG, "sfx_replay_put_gather: bad arguments");
  const PutGather P{rs, rphi, rs1, ra, rg, j, s, phi, s1, a, s1_copy, phi_copy, idx, gam, S, PHI, S1, G, A, B, n_s, d};
  hipLaunchKernelGGL(k_replay_put_gather, dim3(B + 1), dim3(64), 0, (hipStream_t)stream, P);
  LAUNCHCHK();
  return SFX_OK;
}
const char* sfx_last_error(void) { return g_err.c_str(); }

// Bounds-check builds (-DSFX_CHECK, libsfx_check.so): failed device bounds checks since the last
// reset; -1 in the product build.  first_host: up to 8 records (line, a, b, c).
int sfx_check_failures(long long* count, long long* first_host, int reset) {
  if (!count) SFX_FAIL(SFX_E_ARG, "null argument");
#ifdef SFX_CHECK
  unsigned n = 0;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(&n, HIP_SYMBOL(sfx::g_chk_n), sizeof(n)));
  if (first_host) HIPCHK(hipMemcpyFromSymbol(first_host, HIP_SYMBOL(sfx::g_chk_rec), sizeof(long long) * 32));
  if (reset) {
    const unsigned z = 0;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(sfx::g_chk_n), &z, sizeof(z)));
  }
  *count = n;
#else
  (void)first_host;
  (void)reset;
  *count = -1;
#endif
  return SFX_OK;
}

#ifdef SFX_PROBE
// Debug builds: copy out (and reset) the kernel timing probe records; returns the count.
int sfx_probe_dump(void* out_host, int max_recs) {
  unsigned n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(sfx::g_probe_n), sizeof(n)) != hipSuccess) return -1;
  if (n > sfx::PROBE_N) n = sfx::PROBE_N;
  if ((int)n > max_recs) n = (unsigned)max_recs;
  if (n && hipMemcpyFromSymbol(out_host, HIP_SYMBOL(sfx::g_probe), n * sizeof(sfx::ProbeRec)) != hipSuccess) return -1;
  const unsigned z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(sfx::g_probe_n), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)n;
}
#endif

int sfx_create(sfx_t* out, int T, int n_s, int H, int n_hidden, const int* acts, int A, int d, int max_batch,
               int device, void* stream) {
  if (!out) SFX_FAIL(SFX_E_ARG, "out is null");
  *out = nullptr;
  if (T < 1 || T > 64 || n_s < 1 || H < 1 || n_hidden < 0 || n_hidden + 2 > NLMAX || A < 1 || d < 1 ||
      max_batch < 1)
    SFX_FAIL(SFX_E_ARG, "bad geometry (1 <= T <= 64 heads per handle)");
  if (d > DMAX || max_batch + 1 > MMAX || (long)T * A > QMAX || (long)A * d > OMAX)
    SFX_FAIL(SFX_E_ARG, "geometry exceeds kernel limits (d<=256, batch<1024, T*A<=8192, A*d<=4096)");
  for (int i = 0; i < n_hidden; ++i)
    if (!acts || acts[i] < ACT_NONE || acts[i] > ACT_TANH) SFX_FAIL(SFX_E_ARG, "bad activation code");
  HIPCHK(hipSetDevice(device));
  sfx_handle* h = new sfx_handle();
  h->T = T;
  h->n_s = n_s;
  h->H = H;
  h->nh = n_hidden;
  h->A = A;
  h->d = d;
  h->O = A * d;
  h->NL = n_hidden + 2;
  h->Mmax = max_batch;
  h->device = device;
  h->stream = (hipStream_t)stream;
  h->dpad = align4(d);
  const char* eg = std::getenv("SFX_GRAPHS");
  h->use_graphs = !(eg && eg[0] == '0');
  const char* efp = std::getenv("SFX_FOLD_PUBLISH");
  h->fold_publish = !(efp && efp[0] == '0');
  {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
      h->ncu = ncu;
  }
  const char* etp = std::getenv("SFX_FWD_TPW");
  h->fwd_tpw = etp && etp[0] == '1' ? 1 : FWD_TPW;
  const char* eqa = std::getenv("SFX_SHARD_QA");
  h->shard_qa = !(eqa && eqa[0] == '0');
  const char* esk = std::getenv("SFX_SKIP");
  h->skip_rounds = !(esk && esk[0] == '0');
  int off = 0, ptorch = 0;
  for (int l = 0; l < h->NL; ++l) {
    LayerGeo Lr{};
    if (l == 0) {
      Lr.N = H; Lr.K = n_s; Lr.actOut = ACT_NONE;
    } else if (l == h->NL - 1) {
      Lr.N = h->O; Lr.K = H; Lr.actOut = ACT_NONE;
    } else {
      Lr.N = H; Lr.K = H; Lr.actOut = acts[l - 1];
    }
    Lr.actIn = l > 0 ? h->L[l - 1].actOut : ACT_NONE;
    Lr.wOff = align8(off);
    off = Lr.wOff + Lr.N * Lr.K;
    Lr.bOff = align4(off);
    off = Lr.bOff + Lr.N;
    ptorch += Lr.N * Lr.K + Lr.N;
    h->L.push_back(Lr);
  }
  h->P = (off + 63) & ~63;
  h->Ptorch = ptorch;
  int aoff = 0;
  for (int l = 0; l < h->NL; ++l) {
    h->actOff.push_back(aoff);
    aoff += align4((max_batch + 1) * h->L[l].N);  // +1 row: the next state of the fused step
  }
  h->actSize = (aoff + 63) & ~63;
  h->Tg = T;
  h->spec_rounds = auto_spec_rounds(T);
  h->since_target.assign(T, 0);
  h->host_step.assign(T, 0);

  const size_t headBytes = sizeof(float) * (size_t)T * h->P;
  const size_t wBytes = sizeof(float) * (size_t)T * h->dpad;
  int rc = SFX_OK;
  auto alloc = [&](void** p, size_t bytes) {
    if (rc != SFX_OK) return;
    if (hipMalloc(p, bytes) != hipSuccess || hipMemset(*p, 0, bytes) != hipSuccess) {
      g_err = "hipMalloc failed";
      rc = SFX_E_HIP;
    }
  };
  alloc((void**)&h->online, 2 * headBytes);
  alloc((void**)&h->target, headBytes);
  alloc((void**)&h->am, 2 * headBytes);
  alloc((void**)&h->av, 2 * headBytes);
  alloc((void**)&h->w, wBytes);
  alloc((void**)&h->wm, wBytes);
  alloc((void**)&h->wv, wBytes);
  alloc((void**)&h->step, sizeof(int) * T);
  alloc((void**)&h->dcancel, 64);
  alloc((void**)&h->adamc, sizeof(AdamC) * T);
  {  // split-N dX: every layer's N split into <= 256-wide chunks, tiles of 32 rows x 16 columns
    int nmax = 0, kmax = 0;
    for (const LayerGeo& L : h->L) {
      nmax = std::max(nmax, L.N);
      kmax = std::max(kmax, L.K);
    }
    h->dxs_max = std::max(1, cdiv(nmax, DX_SPLIT_N));
    h->dx_ntile = cdiv(max_batch, 32) * cdiv(kmax, 16);
    if (h->dxs_max > 1) {
      alloc((void**)&h->dxpart, sizeof(float) * 512 * (size_t)T * h->dx_ntile * h->dxs_max);
      alloc((void**)&h->dxctr, sizeof(unsigned) * (size_t)T * h->dx_ntile);
    }
  }
  alloc((void**)&h->act, sizeof(float) * (size_t)NROLE * T * h->actSize);
  alloc((void**)&h->dz, sizeof(float) * (size_t)T * h->actSize);
  alloc((void**)&h->rowloss, sizeof(float) * (size_t)T * MMAX);
  alloc((void**)&h->spec_next, sizeof(int64_t) * 2 * (size_t)T * MMAX);
  alloc((void**)&h->skip, sizeof(int) * 2 * (size_t)T);  // skip [T] | the unfused TD launch's report words [T]
  alloc((void**)&h->skipc, 64);
  alloc((void**)&h->dout, sizeof(StepOut));
  alloc((void**)&h->selk, sizeof(SelScratch));
  if (rc == SFX_OK &&
      hipHostMalloc((void**)&h->hout, sizeof(StepOut), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    g_err = "hipHostMalloc failed";
    rc = SFX_E_HIP;
  }
  if (rc == SFX_OK && hipEventCreateWithFlags(&h->ev_step, hipEventDisableTiming) != hipSuccess) {
    g_err = "hipEventCreate failed";
    rc = SFX_E_HIP;
  }
  if (rc == SFX_OK && hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking) != hipSuccess) {
    g_err = "hipStreamCreate failed";
    rc = SFX_E_HIP;
  }
  if (rc != SFX_OK) {
    free_all(h);
    delete h;
    return rc;
  }
  Geo& G = h->G;
  G.T = T;
  G.NL = h->NL;
  G.A = A;
  G.d = d;
  G.O = h->O;
  G.dpad = h->dpad;
  G.P = h->P;
  G.actSize = h->actSize;
  G.online = h->online;
  G.target = h->target;
  G.am = h->am;
  G.av = h->av;
  G.w = h->w;
  G.wm = h->wm;
  G.wv = h->wv;
  G.step = h->step;
  G.adamc = h->adamc;
  G.act = h->act;
  G.dz = h->dz;
  G.rowloss = h->rowloss;
  G.cancel = h->dcancel;
  G.nonfin = h->dcancel + 8;  // sticky non-finite TD flag (sfx_nonfinite)
  G.lastOff = h->actOff[h->NL - 1];
#ifdef SFX_CHECK
  G.ext_dxpart = h->dxpart ? 512LL * T * h->dx_ntile * h->dxs_max : 0;
#endif
  *out = h;
  return SFX_OK;
}

void tsf_release(sfx_handle* h);
void phi_release(sfx_handle* h);

int sfx_destroy(sfx_t h) {
  if (!h) return SFX_OK;
  (void)settle(h);
  (void)hipStreamSynchronize(h->stream);
  tsf_release(h);
  phi_release(h);
  free_all(h);
  delete h;
  return SFX_OK;
}

int sfx_set_stream(sfx_t h, void* stream) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->stream = (hipStream_t)stream;
  return SFX_OK;
}

int sfx_set_graphs(sfx_t h, int enable) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->use_graphs = enable != 0;
  if (!h->use_graphs) clear_graphs(h);
  return SFX_OK;
}

int sfx_head_numel(sfx_t h) { return h ? h->Ptorch : SFX_E_ARG; }

int sfx_set_adam(sfx_t h, double lr_psi, double wd_psi, double lr_w, double wd_w, double beta1, double beta2,
                 double eps) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->hp_psi = AdamHP{lr_psi, wd_psi, beta1, beta2, eps};
  h->hp_w = AdamHP{lr_w, wd_w, beta1, beta2, eps};
  clear_graphs(h);  // hyper-parameters are baked into captured launches
  return SFX_OK;
}

int sfx_load_head(sfx_t h, int t, int which, const float* params_host) {
  RC(settle(h));
  if (!valid_head(h, t) || !params_host) SFX_FAIL(SFX_E_ARG, "bad head / pointer");
  std::vector<float> buf(h->P);
  pack_head(h, params_host, buf.data());
  HIPCHK(hipStreamSynchronize(h->stream));
  touch(h);
  HIPCHK(hipMemcpyAsync(which ? h->target_of(t) : h->online_cur(t), buf.data(), sizeof(float) * h->P,
                        hipMemcpyHostToDevice, h->stream));
  if (h->bf16) RC(refresh_bf16(h, which ? h->target_of(t) : h->online_cur(t), which ? h->tg16_of(t) : h->on16_cur(t), h->P));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

int sfx_get_head(sfx_t h, int t, int which, float* params_host) {
  RC(settle(h));
  if (!valid_head(h, t) || !params_host) SFX_FAIL(SFX_E_ARG, "bad head / pointer");
  std::vector<float> buf(h->P);
  HIPCHK(hipMemcpyAsync(buf.data(), which ? h->target_of(t) : h->online_cur(t), sizeof(float) * h->P,
                        hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  unpack_head(h, buf.data(), params_host);
  return SFX_OK;
}

int sfx_load_adam(sfx_t h, int t, const float* m_host, const float* v_host, int step) {
  RC(settle(h));
  if (!valid_head(h, t) || !m_host || !v_host || step < 0) SFX_FAIL(SFX_E_ARG, "bad args");
  std::vector<float> bm(h->P), bv(h->P);
  pack_head(h, m_host, bm.data());
  pack_head(h, v_host, bv.data());
  HIPCHK(hipStreamSynchronize(h->stream));
  touch(h);
  HIPCHK(hipMemcpyAsync(h->am_cur(t), bm.data(), sizeof(float) * h->P, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->av_cur(t), bv.data(), sizeof(float) * h->P, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->step + t, &step, sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->host_step[t] = step;
  return SFX_OK;
}

int sfx_get_adam(sfx_t h, int t, float* m_host, float* v_host, int* step) {
  RC(settle(h));
  if (!valid_head(h, t)) SFX_FAIL(SFX_E_ARG, "bad head");
  std::vector<float> bm(h->P), bv(h->P);
  int st = 0;
  HIPCHK(hipMemcpyAsync(bm.data(), h->am_cur(t), sizeof(float) * h->P, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(bv.data(), h->av_cur(t), sizeof(float) * h->P, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(&st, h->step + t, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (m_host) unpack_head(h, bm.data(), m_host);
  if (v_host) unpack_head(h, bv.data(), v_host);
  if (step) *step = st;
  return SFX_OK;
}

int sfx_load_w(sfx_t h, int t, const float* w_host) {
  RC(settle(h));
  if (!valid_w(h, t) || !w_host) SFX_FAIL(SFX_E_ARG, "bad args");
  HIPCHK(hipStreamSynchronize(h->stream));
  touch(h);
  HIPCHK(hipMemcpyAsync(h->w + (size_t)t * h->dpad, w_host, sizeof(float) * h->d, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

// w_t with its Adam moments (the sfdqn.py l2 path's w optimizer state; checkpoint resume)
int sfx_load_w_state(sfx_t h, int t, const float* w_host, const float* wm_host, const float* wv_host) {
  RC(settle(h));
  if (!valid_w(h, t) || !w_host || !wm_host || !wv_host) SFX_FAIL(SFX_E_ARG, "bad args");
  HIPCHK(hipStreamSynchronize(h->stream));
  const size_t o = (size_t)t * h->dpad, n = sizeof(float) * h->d;
  touch(h);
  HIPCHK(hipMemcpyAsync(h->w + o, w_host, n, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->wm + o, wm_host, n, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->wv + o, wv_host, n, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

int sfx_get_w(sfx_t h, int t, float* w_host, float* wm_host, float* wv_host) {
  RC(settle(h));
  if (!valid_w(h, t)) SFX_FAIL(SFX_E_ARG, "bad head");
  const size_t o = (size_t)t * h->dpad, n = sizeof(float) * h->d;
  if (w_host) HIPCHK(hipMemcpyAsync(w_host, h->w + o, n, hipMemcpyDeviceToHost, h->stream));
  if (wm_host) HIPCHK(hipMemcpyAsync(wm_host, h->wm + o, n, hipMemcpyDeviceToHost, h->stream));
  if (wv_host) HIPCHK(hipMemcpyAsync(wv_host, h->wv + o, n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

int sfx_w_ptr(sfx_t h, int t, float** w_dev) {
  RC(settle(h));
  if (!valid_w(h, t) || !w_dev) SFX_FAIL(SFX_E_ARG, "bad args");
  *w_dev = h->w + (size_t)t * h->dpad;
  return SFX_OK;
}

int sfx_gpi(sfx_t h, const float* S, int B, const float* w, float* psi, float* q, int64_t* task, int64_t* next) {
  if (!h || !S || !w || B < 1) SFX_FAIL(SFX_E_ARG, "bad args");
  auto gpi = [&]() -> int {
    const GraphKey key = make_key(1, {B}, h->mask, {S, w, psi, q, task, next});
    return run_graph(h, key, [&]() -> int {
      for (int row0 = 0; row0 < B; row0 += h->Mmax) {
        const int m = B - row0 < h->Mmax ? B - row0 : h->Mmax;
        RC(run_fwd(h, {{R_G, P_ONLINE, 1, 0, h->T}}, m, S + (size_t)row0 * h->n_s, nullptr));
        RC(run_gpi(h, gpi_args(R_G, 0, row0, w, psi, q, task, next, nullptr, 0, 0, m)));
      }
      return SFX_OK;
    });
  };
  if (h->lazy_finish && h->pend.active && h->pend.update) {
    // An all-task update (sfx_update_all) is pending its verdict.  Queue this GPI behind it first,
    // on the slots that update writes (h->mask flips to them when the verdict is collected), so it
    // runs while the host waits for the verdict; only when the verdict needs host rounds -- which
    // rewrite those slots -- is it queued again behind them.  (The drop-in's agent loop calls GPI
    // right after the update: the wait then ends with the GPI done, not before it is launched.)
    const unsigned long long m0 = h->mask;
    h->mask = m0 ^ h->all_bits();
    const int rc = gpi();
    h->mask = m0;
    RC(rc);
    const long long fb = h->steps_fallback;
    RC(settle(h));
    if (h->steps_fallback == fb) return SFX_OK;
    return gpi();
  }
  RC(settle(h));
  return gpi();
}

int sfx_successors(sfx_t h, const float* S, int B, int which, float* psi) {
  RC(settle(h));
  if (!h || !S || !psi || B < 1 || (which != 0 && which != 1)) SFX_FAIL(SFX_E_ARG, "bad args");
  const GraphKey key = make_key(21, {B, which}, h->mask, {S, psi});
  return run_graph(h, key, [&]() -> int {
    for (int row0 = 0; row0 < B; row0 += h->Mmax) {
      const int m = B - row0 < h->Mmax ? B - row0 : h->Mmax;
      RC(run_fwd(h, {{R_G, which ? P_TARGET : P_ONLINE, 1, 0, h->T}}, m, S + (size_t)row0 * h->n_s, nullptr));
      RC(run_gpi(h, gpi_args(R_G, 0, row0, h->w, psi, nullptr, nullptr, nullptr, nullptr, 0, 0, m)));
    }
    return SFX_OK;
  });
}

int sfx_select_action(sfx_t h, const float* s, int task_index, int use_gpi, float* q, int64_t* out) {
  RC(settle(h));
  if (!h || !s || !out || task_index < 0 || task_index >= h->T) SFX_FAIL(SFX_E_ARG, "bad args");
  use_gpi = use_gpi ? 1 : 0;
  const GraphKey key = make_key(2, {task_index, use_gpi}, h->mask, {s, q, out});
  return run_graph(h, key, [&]() -> int { return select_body(h, s, task_index, use_gpi, q, out); });
}

int sfx_test_actions(sfx_t h, const float* S, int E, const float* W, int w_stride, float* q, int64_t* out) {
  RC(settle(h));
  if (!h || !S || !W || !out || E < 1 || w_stride < h->d) SFX_FAIL(SFX_E_ARG, "bad args");
  const GraphKey key = make_key(26, {E, w_stride}, h->mask, {S, W, q, out});
  return run_graph(h, key, [&]() -> int {
    for (int row0 = 0; row0 < E; row0 += h->Mmax) {
      const int m = E - row0 < h->Mmax ? E - row0 : h->Mmax;
      RC(run_fwd(h, {{R_G, P_ONLINE, 1, 0, h->T}}, m, S + (size_t)row0 * h->n_s, nullptr));
      GpiArgs g = gpi_args(R_G, 0, row0, W, nullptr, q, nullptr, nullptr, out, 0, 1, m);
      g.w_stride = w_stride;
      g.sel_stride = 2;
      RC(run_gpi(h, g));
    }
    return SFX_OK;
  });
}

int sfx_test_reward_updates(sfx_t h, int E, const float* phi, const float* r, float* W, int w_stride, double lr,
                            double wd, float* loss) {
  RC(settle(h));
  if (!h || !phi || !r || !W || !loss || E < 1 || w_stride < h->d) SFX_FAIL(SFX_E_ARG, "bad args");
  launch(h, K_GPI, 12.0 * E * h->d, k_sf_test_mapper, dim3(cdiv(E, 64)), dim3(64), E, h->d, phi, r, W, w_stride,
         (float)(-lr), (float)wd, loss);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_update(sfx_t h, int policy, const float* S, const int64_t* a, const float* r, const float* phi,
               const float* S1, const float* gamma, int B, int use_gpi, float* losses, int64_t* next) {
  RC(settle(h));
  if (!valid_head(h, policy) || !S || !a || !phi || !S1 || !gamma) SFX_FAIL(SFX_E_ARG, "bad args");
  if (B < 1 || B > h->Mmax) SFX_FAIL(SFX_E_ARG, "batch exceeds max_batch");
  use_gpi = use_gpi ? 1 : 0;
  const GraphKey key = make_key(3, {policy, use_gpi, B}, h->mask, {S, a, r, phi, S1, gamma, losses, next});
  RC(run_graph(h, key, [&]() -> int { return update_body(h, policy, S, a, r, phi, S1, gamma, B, use_gpi, losses, next); }));
  h->mask ^= 1ull << policy;
  after_update(h, policy);
  return maybe_sync_target(h, policy);
}

static int step_all_impl(sfx_t h, const float* S, const int64_t* a, const float* phi, const float* S1,
                         const float* gamma, int B, int use_gpi, int lms_task, const float* lms_phi,
                         const float* lms_r, float lms_alpha, const float* s_next, int task_index, int sel_use_gpi,
                         float* losses, float* q_out, int64_t* task_out,
                         const unsigned long long* out_ind = nullptr) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  if (h->pend.active) SFX_FAIL(SFX_E_STATE, "sfx_step_all: previous step not finished");
  const bool update = B > 0;
  if (update && (!S || !a || !phi || !S1 || !gamma || B > h->Mmax)) SFX_FAIL(SFX_E_ARG, "bad minibatch");
  if (lms_task >= h->T || (lms_task >= 0 && (!lms_phi || !lms_r))) SFX_FAIL(SFX_E_ARG, "bad LMS args");
  if (s_next && (task_index < 0 || task_index >= h->T)) SFX_FAIL(SFX_E_ARG, "bad task_index");
  if (!update && !s_next) SFX_FAIL(SFX_E_ARG, "nothing to do");
  sfx_handle::Pending p;
  p.active = true;
  p.update = update;
  p.sel = s_next != nullptr;
  p.B = update ? B : 0;
  p.use_gpi = use_gpi ? 1 : 0;
  p.task = s_next ? task_index : 0;
  p.sel_use_gpi = sel_use_gpi ? 1 : 0;
  p.S = S;
  p.S1 = S1;
  p.phi = phi;
  p.gamma = gamma;
  p.a = a;
  p.s_next = s_next;
  p.losses = losses;
  p.q_out = s_next && !out_ind ? q_out : nullptr;
  p.task_out = s_next && !out_ind ? task_out : nullptr;
  p.out_ind = s_next ? out_ind : nullptr;
  unsigned alpha_bits;
  std::memcpy(&alpha_bits, &lms_alpha, 4);
  const GraphKey key = make_key(5, {p.B, p.use_gpi, lms_task, p.task, p.sel_use_gpi, (int)alpha_bits, h->spec_rounds}, h->mask,
                                {S, a, phi, S1, gamma, lms_phi, lms_r, s_next, losses, p.q_out, p.task_out, p.out_ind});
  const int rounds = p.use_gpi ? h->spec_rounds : 1;
  h->hout->posted = 0;  // the step before has been collected: nothing writes hout now
  bool recorded = false;
  RC(run_graph(h, key, [&]() -> int {
    h->post_hout = true;
    h->hout_posted = false;
    const int rc = launch_step_all(h, p, lms_task, lms_phi, lms_r, lms_alpha, rounds);
    h->post_hout = false;
    RC(rc);
    recorded = true;
    p.posted = h->hout_posted;
    if (h->use_graphs && !h->prof) h->graph_posts[key] = p.posted;
    if (!h->hout_posted) HIPCHK(hipMemcpyAsync(h->hout, h->dout, sizeof(StepOut), hipMemcpyDeviceToHost, h->stream));
    return SFX_OK;
  }));
  if (!recorded) {  // a cached graph: what its recording found
    const auto it = h->graph_posts.find(key);
    p.posted = it != h->graph_posts.end() && it->second;
  }
  HIPCHK(hipEventRecord(h->ev_step, h->stream));
  h->pend = p;
  return SFX_OK;
}

int sfx_step_all(sfx_t h, const float* S, const int64_t* a, const float* phi, const float* S1, const float* gamma,
                 int B, int use_gpi, int lms_task, const float* lms_phi, const float* lms_r, float lms_alpha,
                 const float* s_next, int task_index, int sel_use_gpi, float* losses) {
  return step_all_impl(h, S, a, phi, S1, gamma, B, use_gpi, lms_task, lms_phi, lms_r, lms_alpha, s_next, task_index,
                       sel_use_gpi, losses, nullptr, nullptr);
}

int sfx_step_finish(sfx_t h, int64_t* out_host) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  if (!h->pend.active) SFX_FAIL(SFX_E_STATE, "sfx_step_finish without sfx_step_all");
  sfx_handle::Pending p = h->pend;
  h->pend.active = false;
  if (!p.posted || !wait_posted(h)) HIPCHK(hipEventSynchronize(h->ev_step));
  int first = h->T, dev_flag = h->T;
  if (p.update) {
    first = p.use_gpi ? h->hout->flag : h->T;
    if (first < 0 || first > h->T) SFX_FAIL(SFX_E_STATE, "corrupt speculation flag");
    if (h->force_rerun_from >= 0 && h->force_rerun_from < first) first = h->force_rerun_from;
    int r = p.use_gpi ? h->spec_rounds : 1;
    dev_flag = first;
    h->steps_spec += 1;
    if (first < h->T) {
      h->steps_fallback += 1;
      h->policies_rerun += h->T - first;
    }
    // more rounds until every policy's next actions are verified (each round fixes >= 1 head)
    while (first < h->T) {
      if (r > h->T + 1) SFX_FAIL(SFX_E_STATE, "speculation did not converge");
      RC(launch_round(h, p, r, true));
      HIPCHK(hipMemcpyAsync(h->hout, h->dout, sizeof(StepOut), hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));
      ++r;
      first = h->hout->flag;
      if (first < 0 || first > h->T) SFX_FAIL(SFX_E_STATE, "corrupt speculation flag");
      if (h->force_rerun_from >= 0 && r <= h->spec_rounds + 1 && h->force_rerun_from < first) first = h->force_rerun_from;
    }
    h->rounds_total += r;
    h->mask ^= h->all_bits();
    for (int t = 0; t < h->T; ++t) {
      after_update(h, t);
      RC(maybe_sync_target(h, t));
    }
  }
  if (out_host) {
    out_host[0] = p.sel ? h->hout->sel[0] : -1;
    out_host[1] = p.sel ? h->hout->sel[1] : -1;
    out_host[2] = dev_flag;
  }
  return SFX_OK;
}

int sfx_set_precision(sfx_t h, int precision) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  if (precision != SFX_PREC_FP32 && precision != SFX_PREC_BF16) SFX_FAIL(SFX_E_ARG, "unknown precision");
  touch(h);
  const bool want = precision == SFX_PREC_BF16;
  if (want == h->bf16) return SFX_OK;
  HIPCHK(hipStreamSynchronize(h->stream));
  clear_graphs(h);
  if (want) {
    const size_t n = (size_t)h->T * h->P;
    if (!h->on16 && hipMalloc((void**)&h->on16, sizeof(__bf16) * 2 * n) != hipSuccess)
      SFX_FAIL(SFX_E_HIP, "hipMalloc(bf16 copy) failed");
    if (!h->tg16 && hipMalloc((void**)&h->tg16, sizeof(__bf16) * n) != hipSuccess)
      SFX_FAIL(SFX_E_HIP, "hipMalloc(bf16 copy) failed");
    RC(refresh_bf16(h, h->online, h->on16, (long long)(2 * n)));
    RC(refresh_bf16(h, h->target, h->tg16, (long long)n));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  h->bf16 = want;
  h->G.on16 = want ? h->on16 : nullptr;
  h->G.tg16 = want ? h->tg16 : nullptr;
  return SFX_OK;
}

int sfx_get_precision(sfx_t h) { return h ? (h->bf16 ? SFX_PREC_BF16 : SFX_PREC_FP32) : SFX_E_ARG; }

int sfx_set_huber(sfx_t h, float delta) {
  RC(settle(h));
  if (!h || !(delta >= 0.f) || !std::isfinite(delta)) SFX_FAIL(SFX_E_ARG, "huber delta must be finite and >= 0");
  if (delta == h->G.huber) return SFX_OK;
  HIPCHK(hipStreamSynchronize(h->stream));
  clear_graphs(h);  // Geo is baked into captured launches
  h->G.huber = delta;
  return SFX_OK;
}

float sfx_get_huber(sfx_t h) { return h ? h->G.huber : -1.f; }

int sfx_set_spec_rounds(sfx_t h, int rounds) {
  RC(settle(h));
  if (!h || rounds < 0) SFX_FAIL(SFX_E_ARG, "bad args");
  h->spec_rounds_auto = rounds == 0;
  h->spec_rounds = rounds == 0 ? auto_spec_rounds(h->Tg) : rounds;
  return SFX_OK;
}

int sfx_step_stats(sfx_t h, long long* steps, long long* fallbacks, long long* rerun_policies, long long* rounds) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  if (rounds) *rounds = h->rounds_total;
  if (steps) *steps = h->steps_spec;
  if (fallbacks) *fallbacks = h->steps_fallback;
  if (rerun_policies) *rerun_policies = h->policies_rerun;
  return SFX_OK;
}

int sfx_graph_stats(sfx_t h, long long* captures, long long* launches, long long* cached) {
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  if (captures) *captures = h->graph_captures;
  if (launches) *launches = h->graph_launches + h->graph_eager;
  if (cached) *cached = (long long)h->graphs.size();
  return SFX_OK;
}

int sfx_skip_stats(sfx_t h, long long* checked, long long* skipped, int reset) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  unsigned long long c[2] = {0, 0};
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(c, h->skipc, sizeof(c), hipMemcpyDeviceToHost));
  if (checked) *checked = (long long)c[0];
  if (skipped) *skipped = (long long)c[1];
  if (reset) {
    HIPCHK(hipMemset(h->skipc, 0, sizeof(c)));
  }
  return SFX_OK;
}

int sfx_nonfinite(sfx_t h, int* flag_host, int reset) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  int v = 0;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(&v, h->G.nonfin, sizeof(int), hipMemcpyDeviceToHost));
  if (flag_host) *flag_host = v;
  if (reset) HIPCHK(hipMemset(h->G.nonfin, 0, sizeof(int)));
  return SFX_OK;
}

int sfx_debug_force_rerun(sfx_t h, int first_policy) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->force_rerun_from = first_policy;
  return SFX_OK;
}

int sfx_update_all(sfx_t h, const float* S, const int64_t* a, const float* phi, const float* S1, const float* gamma,
                   int B, float* losses) {
  if (!h || !S || !a || !phi || !S1 || !gamma) SFX_FAIL(SFX_E_ARG, "bad args");
  if (B < 1 || B > h->Mmax) SFX_FAIL(SFX_E_ARG, "batch exceeds max_batch");
  RC(settle(h));
  RC(sfx_step_all(h, S, a, phi, S1, gamma, B, 1, -1, nullptr, nullptr, 0.f, nullptr, 0, 1, losses));
  h->lazy_finish = true;  // the verdict is collected by the next call (settle)
  return SFX_OK;
}

int sfx_update_all_select(sfx_t h, const float* S, const int64_t* a, const float* phi, const float* S1,
                          const float* gamma, int B, float* losses, const float* s_next, int task_index, float* q_out,
                          int64_t* task_out, int lms_task, const float* lms_phi, float lms_r, const float* lms_r_dev,
                          float lms_alpha) {
  if (!h || !S || !a || !phi || !S1 || !gamma || !s_next) SFX_FAIL(SFX_E_ARG, "bad args");
  if (B < 1 || B > h->Mmax) SFX_FAIL(SFX_E_ARG, "batch exceeds max_batch");
  if (task_index < 0 || task_index >= h->T) SFX_FAIL(SFX_E_ARG, "bad task_index");
  if (lms_task >= h->T || (lms_task >= 0 && !lms_phi)) SFX_FAIL(SFX_E_ARG, "bad LMS args");
  RC(settle(h));  // the step before has completed: nothing reads xin any more
  if (!h->xin && hipHostMalloc((void**)&h->xin, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    SFX_FAIL(SFX_E_HIP, "hipHostMalloc failed");
  // read by the step's launches (kernel arguments would change the captured graph every step)
  std::memcpy(h->xin, &lms_r, sizeof(float));
  h->xin[1] = (unsigned long long)(uintptr_t)q_out;
  h->xin[2] = (unsigned long long)(uintptr_t)task_out;
  h->xin[3] = (unsigned long long)(uintptr_t)lms_r_dev;
  // the reward: the value in xin[0], or the device float whose address xin[3] holds
  const float* rp = lms_task < 0 ? nullptr : reinterpret_cast<const float*>(lms_r_dev ? h->xin + 3 : h->xin);
  RC(step_all_impl(h, S, a, phi, S1, gamma, B, 1, lms_task, lms_phi, rp, lms_alpha, s_next, task_index, 1, losses,
                   q_out, task_out, h->xin + 1));
  h->lazy_finish = true;  // the verdict (host rounds redo the selection) is collected by the next call
  return SFX_OK;
}

int sfx_settle(sfx_t h, int* host_rounds, int64_t* sel) {
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  const long long r0 = h->rounds_total, s0 = h->steps_spec;
  int64_t out[3] = {-1, -1, -1};
  if (h->lazy_finish) {
    h->lazy_finish = false;
    RC(sfx_step_finish(h, out));
  }
  if (sel) {
    sel[0] = out[0];
    sel[1] = out[1];
  }
  if (host_rounds) {
    // rounds run by this settle beyond the device rounds of the step it collected
    const long long ran = h->rounds_total - r0, dev = h->steps_spec > s0 ? h->spec_rounds : 0;
    *host_rounds = (int)(ran > dev ? ran - dev : 0);
  }
  return SFX_OK;
}

int sfx_lms(sfx_t h, int t, const float* phi, const float* r, float alpha) {
  RC(settle(h));
  if (!valid_w(h, t) || !phi || !r) SFX_FAIL(SFX_E_ARG, "bad args");
  launch(h, K_LMS, 4.0 * (3.0 * h->d + 1), k_lms, dim3(1), dim3(256), h->w + (size_t)t * h->dpad, phi, r, alpha,
         h->d, 0.f);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_lms_value(sfx_t h, int t, const float* phi, float r, float alpha) {
  RC(settle(h));
  if (!valid_w(h, t) || !phi) SFX_FAIL(SFX_E_ARG, "bad args");
  launch(h, K_LMS, 4.0 * (3.0 * h->d), k_lms, dim3(1), dim3(256), h->w + (size_t)t * h->dpad, phi,
         static_cast<const float*>(nullptr), alpha, h->d, r);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_set_target_update_ev(sfx_t h, int ev) {
  RC(settle(h));
  if (!h || ev < 1) SFX_FAIL(SFX_E_ARG, "bad args");
  h->target_update_ev = ev;
  return SFX_OK;
}

int sfx_get_since_target(sfx_t h, int t, int* count) {
  RC(settle(h));
  if (!valid_head(h, t) || !count) SFX_FAIL(SFX_E_ARG, "bad args");
  *count = h->since_target[t];
  return SFX_OK;
}

int sfx_set_since_target(sfx_t h, int t, int count) {
  RC(settle(h));
  if (!valid_head(h, t) || count < 0) SFX_FAIL(SFX_E_ARG, "bad args");
  h->since_target[t] = count;
  return SFX_OK;
}

int sfx_sync_target(sfx_t h, int t) {
  RC(settle(h));
  if (!valid_head(h, t)) SFX_FAIL(SFX_E_ARG, "bad head");
  touch(h);
  HIPCHK(hipMemcpyAsync(h->target_of(t), h->online_cur(t), sizeof(float) * h->P, hipMemcpyDeviceToDevice, h->stream));
  return SFX_OK;
}

int sfx_prof_enable(sfx_t h, int enable) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->prof = enable != 0;
  return SFX_OK;
}

int sfx_prof_collect(sfx_t h, int kind, int* count, double* total_us, double* bytes) {
  RC(settle(h));
  if (!h || kind < 0 || kind >= K_NKIND) SFX_FAIL(SFX_E_ARG, "bad args");
  HIPCHK(hipStreamSynchronize(h->stream));
  int n = 0;
  double us = 0.0, by = 0.0;
  for (auto& r : h->prof_recs) {
    if (r.kind != kind) continue;
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, r.a, r.b));
    ++n;
    us += 1000.0 * ms;
    by += r.bytes;
  }
  if (count) *count = n;
  if (total_us) *total_us = us;
  if (bytes) *bytes = by;
  return SFX_OK;
}

int sfx_prof_reset(sfx_t h) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  for (auto& r : h->prof_recs) {
    h->prof_pool.push_back(r.a);
    h->prof_pool.push_back(r.b);
  }
  h->prof_recs.clear();
  return SFX_OK;
}

int sfx_synchronize(sfx_t h) {
  RC(settle(h));
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

}  // extern "C"

#include "sfx_comm.inc"
#include "sfx_shard.inc"
#include "sfx_runner.inc"
#include "sfx_tsf.inc"
#include "sfx_phi.inc"
