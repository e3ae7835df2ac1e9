// sfx_kernels.h -- gfx950 device code for the successor-feature hot path.
//
// fp32 end to end: the dense products run on the exact-f32 matrix cores
// (v_mfma_f32_16x16x4_f32, a k-ordered fmaf chain), element-wise work on VALU.
//
// Every problem here is tiny (minibatch M <= 32, heads of ~150k parameters), so each
// kernel is LATENCY bound: the design rules are (1) every pointer is computed from
// kernel arguments (no descriptor loads, no dynamically indexed kernel-argument arrays
// in front of the data loads), (2) all global loads a thread needs are issued before the
// first use (compile-time unrolled, predicated), (3) optimizer state is prefetched before
// the MFMA chain, (4) as few dependent launches per env step as the algorithm allows.
//
// Online head state (params, Adam m, v) is double-buffered: head t reads slot
// (mask >> t) & 1 and an optimizer step writes the other slot.  Nothing is updated in
// place, so a speculative update can be discarded (see k_ver) and no launch both reads
// and rewrites a weight.
//
// Reference behaviour being implemented is cited per kernel (paths relative to
// /root/reference/source).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace sfx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int NLMAX = 8;      // Linear layers per head (n_hidden <= 6)
constexpr int MT = 32;        // minibatch rows per tile
constexpr int QMAX = 8192;    // T*A entries of the per-row GPI scratch in LDS
constexpr int OMAX = 4096;    // A*d (row of a ψ output) held in LDS
constexpr int DMAX = 256;     // feature dimension d
constexpr int MMAX = 1024;    // rows of one update
constexpr int KFUSE = 64;     // layer-0 fan-in up to which the post-update forward is fused
constexpr int GEMV_N = 512;   // layer width from which a forward of <= GEMV_M rows runs k_fwd_gemv
constexpr int GEMV_M = 4;
constexpr int DX_SPLIT_N = 256;  // dX of a layer wider than this splits N over workgroups
constexpr int VFUSE = 4096;   // (rows x fan-in) of that forward's input, staged in LDS
constexpr int TQF = 4096;     // 32 rows x (T*A) q values / 32 rows x A*d gradients of the fused TD target

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };
// activation-block roles: ψ(S) online (saved for backward), ψ⁻(S1) target, ψ(S1) online
// before the step, GPI scratch, action selection, and two alternating buffers of
// ψ(S1 ++ s_next) online after a speculative round of the step
// Minibatch roles R_S / R_S1T / R_S1 exist twice: Geo::mb (0 or R_NS) picks the copy the current
// step uses, R_NS / R_NS1T / R_NS1 name the other copy -- the native runner's look-ahead forward
// (sfx_runner) fills the next step's minibatch roles from the final round's
// post-update forward, so that step starts at its TD launch.
enum { R_S = 0, R_S1T = 1, R_S1 = 2, R_G = 3, R_A = 4, R_V = 5, R_V2 = 6, R_NS = 7, R_NS1T = 8, R_NS1 = 9, NROLE = 10 };
// parameter sets a forward instance can read
enum { P_ONLINE = 0, P_TARGET = 1, P_NEW = 2 };

__device__ __forceinline__ float act_fwd(float x, int code) {
  if (code == ACT_RELU) return x > 0.f ? x : 0.f;
  if (code == ACT_TANH) return tanhf(x);
  return x;
}

// Gradient through an activation expressed via its OUTPUT y (ATen threshold_backward /
// tanh_backward: grad * (1 - y*y)).
__device__ __forceinline__ float act_bwd(float gy, float y, int code) {
  if (code == ACT_RELU) return y > 0.f ? gy : 0.f;
  if (code == ACT_TANH) return __fmul_rn(gy, __fsub_rn(1.f, __fmul_rn(y, y)));
  return gy;
}

// Timing probe (debug builds with -DSFX_PROBE only): wave 0 of each workgroup logs
// s_memrealtime (100 MHz) at entry (t[0]), at up to four marks (t[1] kernel arguments
// landed, t[2] operands landed / MFMA done, t[3], t[4] free) and after its stores completed
// (t[5]), for tools/probe_run.py.
#ifdef SFX_PROBE
struct ProbeRec {
  unsigned kid, blk;
  unsigned long long t[10];
};
constexpr unsigned PROBE_N = 1u << 16;
__device__ ProbeRec g_probe[PROBE_N];
__device__ unsigned g_probe_n;
__shared__ unsigned long long s_probe_t[10];
#define PROBE_T(v)                                                                 \
  const unsigned long long v = __builtin_amdgcn_s_memrealtime();                   \
  if (threadIdx.x == 0)                                                            \
    for (int i_ = 1; i_ < 9; ++i_) s_probe_t[i_] = 0
#define PROBE_AT(i) \
  do { if (threadIdx.x == 0) s_probe_t[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define PROBE_MARKA() \
  do { __builtin_amdgcn_s_waitcnt(0); PROBE_AT(1); } while (0)
#define PROBE_MARK() PROBE_AT(2)
#define PROBE_REC(kid, t0)                                                         \
  do {                                                                             \
    __builtin_amdgcn_s_waitcnt(0);                                                 \
    const unsigned long long t5_ = __builtin_amdgcn_s_memrealtime();               \
    if (threadIdx.x == 0) {                                                        \
      const unsigned i_ = atomicAdd(&g_probe_n, 1u);                               \
      if (i_ < PROBE_N)                                                            \
        g_probe[i_] = ProbeRec{(unsigned)(kid), blockIdx.x + 65536u * blockIdx.y,  \
                               {t0, s_probe_t[1], s_probe_t[2], s_probe_t[3], s_probe_t[4],   \
                                s_probe_t[5], s_probe_t[6], s_probe_t[7], s_probe_t[8], t5_}}; \
    }                                                                              \
  } while (0)
#else
#define PROBE_T(v)
#define PROBE_AT(i)
#define PROBE_MARK()
#define PROBE_MARKA()
#define PROBE_REC(kid, t0)
#endif

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 operand mode (sfx_set_precision): v_mfma_f32_16x16x32_bf16 -- lane l holds A[row l&15]
// [k = 8(l>>4) + j] and B[k = 8(l>>4) + j][col l&15], j = 0..7; C as the f32 16x16x4 form.  The
// 8 k of a lane are the KL-consecutive k the fp32 tiles already give each lane group, so a tile
// swaps its 8 f32 k-steps for one bf16 step (the reduction order changes: not bit-exact).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ floatx4 mfma_bf16(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 to_bf16x8(const float* v) {  // round to nearest even
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}
__device__ __forceinline__ bf16x8 ld_bf16x8(const __bf16* p) {  // 16-B aligned
  return *reinterpret_cast<const bf16x8*>(p);
}

// Loads / stores of data handed between workgroups INSIDE one launch (the split-N dX partial
// tiles): C = true makes them coherent -- sc1 (L1-bypassing) dword loads and write-through
// stores, the hand-off form of MI355X_MICROARCH.md's validated table (sc1 stores, every storing
// wave's vmcnt(0), one agent-scope arrival per workgroup, sc1 poll, barrier, sc1 loads).
// C = false: plain accesses (data from an earlier launch; the kernel boundary orders it).
template <bool C>
__device__ __forceinline__ float ldc(const float* p) {
  if constexpr (C) return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool C>
__device__ __forceinline__ void stc(float* p, float v) {
#ifdef SFX_WT_ALL  // experiment: every hand-off store to a later launch write-through too
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  if constexpr (C) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
#endif
}
template <bool C>
__device__ __forceinline__ float4 ldc4(const float* p) {  // 16-B aligned
  if constexpr (C) return make_float4(ldc<true>(p), ldc<true>(p + 1), ldc<true>(p + 2), ldc<true>(p + 3));
  else return *reinterpret_cast<const float4*>(p);
}

// 16 consecutive floats row[kb .. kb+15] (zero where !ok / outside [0, K)).  `vec` must be
// wave-uniform (K % 64 == 0 with 16-B aligned rows): then four predicated float4 loads.
template <bool C = false>
__device__ __forceinline__ void load16u(float (&v)[16], const float* row, int kb, int K, bool ok, bool vec) {
  if (vec) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = ok ? ldc4<C>(row + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[4 * q] = t.x;
      v[4 * q + 1] = t.y;
      v[4 * q + 2] = t.z;
      v[4 * q + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (ok && kb + j < K) ? ldc<C>(row + kb + j) : 0.f;
  }
}

// -------------------------------------------------------------------------------------
// Handle geometry, passed by value to every kernel (all pointers derive from it).
// -------------------------------------------------------------------------------------
// Device bounds checks (SURVEY §5 "HIP debug mode with bounds asserts"; the `check` build,
// -DSFX_CHECK, Makefile target `check` -> libsfx_check.so): SFX_CHK(cond, a, b, c) counts a failed
// condition, records the first ones (file line, a, b, c) and prints them.  It does not trap:
// a fault would take the shared GPU box down; the test harness reads the count after every test
// (sfx_check_failures, tests/conftest.py) and fails the test.  Compiled out of the product build.
#ifdef SFX_CHECK
__device__ unsigned g_chk_n;
__device__ long long g_chk_rec[8][4];
__device__ __noinline__ void sfx_chk_fail(const char* file, int line, long long a, long long b, long long c) {
  const unsigned i = atomicAdd(&g_chk_n, 1u);
  if (i < 8) {
    g_chk_rec[i][0] = line;
    g_chk_rec[i][1] = a;
    g_chk_rec[i][2] = b;
    g_chk_rec[i][3] = c;
  }
  if (i < 4)
    printf("SFX_CHECK %s:%d failed: %lld %lld %lld (block %u, %u thread %u)\n", file, line, a, b, c, blockIdx.x,
           blockIdx.y, threadIdx.x);
}
#define SFX_CHK(cond, a, b, c)                                                                       \
  do {                                                                                               \
    if (!(cond)) sfx_chk_fail(__FILE__, __LINE__, (long long)(a), (long long)(b), (long long)(c)); \
  } while (0)
#else
#define SFX_CHK(cond, a, b, c) \
  do {                         \
  } while (0)
#endif

struct LayerGeo {
  int N, K, wOff, bOff, actIn, actOut;  // actIn: activation that produced this layer's input
};

struct AdamC;

struct Geo {
  int T, NL, A, d, O, dpad;
  long long P;        // packed head stride (floats)
  long long actSize;  // one (role, head) activation block (floats)
  float* online;      // [2][T][P]   slot-major
  float* target;      // [T][P]
  float* am;          // [2][T][P]   Adam m of ψ
  float* av;          // [2][T][P]   Adam v of ψ
  float* w;           // [T][dpad]
  float* wm;
  float* wv;
  int* step;          // [T]
  AdamC* adamc;       // [T] ψ-Adam constants of each head's current step (written where step is bumped)
  float* act;         // [NROLE][T][actSize]
  float* dz;          // [T][actSize]
  float* rowloss;     // [T][MMAX] per-row Σ (c - t)^2 of the last TD target
  const int* cancel;  // runner steps: 1 when the step's gate cancelled it (see step_cancelled)
  int* nonfin;        // SURVEY §5 failure detection: set (sticky) when a TD error comes out non-finite
  int lastOff;        // offset of the last layer's output inside an activation block
  // bf16 operand mode: bf16 copies of the online [2][T][P] and target [T][P] parameters (the
  // fp32 ones stay the master copy; the Adam epilogue rewrites the copy of every weight it
  // updates).  Null in fp32 mode.
  __bf16* on16;
  __bf16* tg16;
  int mb;          // 0 or R_NS: the physical copy of the minibatch roles this launch calls R_S .. R_S1
  float huber;     // ψ loss: 0 = MSELoss (the reference's), δ > 0 = HuberLoss(delta = δ) (opt-in, td_grad)
#ifdef SFX_CHECK
  long long ext_dxpart;  // floats of the split-N dX partials
#endif

  __device__ __forceinline__ int phys_role(int role) const {
    return role < R_G ? role + mb : role >= R_NS ? role - R_NS + (R_NS - mb) : role;
  }
  // off: per-layer offset inside a block (passed per launch as a scalar, never indexed)
  __device__ __forceinline__ float* actp(int role, int head, int off) const {
    SFX_CHK(phys_role(role) >= 0 && phys_role(role) < NROLE && head >= 0 && head < T && off >= 0 && off < actSize,
            role, head, off);
    return act + ((long long)phys_role(role) * T + head) * actSize + off;
  }
  __device__ __forceinline__ float* dzp(int head, int off) const {
    SFX_CHK(head >= 0 && head < T && off >= 0 && off < actSize, head, off, actSize);
    return dz + (long long)head * actSize + off;
  }
  // element idx of the block at `off` (role, head) stays inside that (role, head) block
  __device__ __forceinline__ void chk_act(int off, long long idx) const {
    SFX_CHK(off + idx >= 0 && off + idx < actSize, off, idx, actSize);
  }
  __device__ __forceinline__ long long slot_off(int slot, int head) const {
    return ((long long)slot * T + head) * P;
  }
};

__device__ __forceinline__ int rslot(unsigned long long mask, int head) { return (int)((mask >> head) & 1ull); }

// GPI maxima handed between ranks travel as "sortable" int32: an order-preserving map of the
// fp32 value (-0 folded into +0), so all-reduce(MAX) and atomicMax run on plain int32 and the
// decoded max is exactly the fp32 max.  SORT_EMPTY (INT_MIN) marks an entry no head filled.
constexpr int SORT_EMPTY = (int)0x80000000;
__host__ __device__ __forceinline__ int sortable(float f) {
  union { float f; int i; } u;
  u.f = f + 0.f;
  return u.i >= 0 ? u.i : u.i ^ 0x7FFFFFFF;
}
__host__ __device__ __forceinline__ float unsortable(int i) {
  union { float f; int i; } u;
  u.i = i >= 0 ? i : i ^ 0x7FFFFFFF;
  return u.f;
}

// dst[j] = src[j] for j < n_copy, SORT_EMPTY for n_copy <= j < n; grid-strided over a launch
__device__ __forceinline__ void fill_sortable(int* dst, const int* src, int n_copy, int n, int gtid, int gthreads) {
  for (int j = gtid; j < n; j += gthreads) dst[j] = j < n_copy ? src[j] : SORT_EMPTY;
}

// A runner step whose gate cancelled it (the host aborted, or the gate timed out waiting for the
// host) runs its launches anyway -- they are already queued -- but must not commit: every store
// to persistent state (parameters and moments of the write slot, Adam step counters, w, g, h) is
// predicated on this word, written by the step's gate (0 outside runner steps).  Read once at
// entry, used only at the stores, so its latency overlaps the operand loads.
__device__ __forceinline__ int step_cancelled(const int* c) { return __builtin_nontemporal_load(c); }

// Division by a runtime divisor 1 <= d, for 0 <= x < 2^22: one multiply by a float reciprocal
// and one correction step (a hardware integer divide is a ~40-instruction sequence, and the
// index arithmetic of the GPI / TD loops used dozens of them per thread).
struct FDiv {
  int d;
  float inv;
};
__device__ __forceinline__ FDiv fdiv(int d) { return FDiv{d, __frcp_rn((float)d)}; }
__device__ __forceinline__ int operator/(int x, const FDiv& f) {
  int q = (int)((float)x * f.inv);
  const int r = x - q * f.d;
  return q + (r >= f.d) - (r < 0);
}

// XCD-aware decode of a 1-D grid of 8 * ceil(nhead / 8) * ntile blocks into (head, tile):
// workgroups are dealt round-robin over the 8 XCDs, so every tile of head h runs on the XCD
// of slot h % 8 and the head's parameters, Adam state and activations stay in that XCD's L2
// from one launch to the next.  Returns false for the padding blocks.
__device__ __forceinline__ bool xcd_decode(int b, int nhead, int ntile, int& head, int& tile) {
  const int hp = (nhead + 7) >> 3, k = b >> 3;
  const int kq = hp == 1 ? k : k / fdiv(hp);
  head = (b & 7) + 8 * (k - kq * hp);
  tile = kq;
  return head < nhead && tile < ntile;
}

// -------------------------------------------------------------------------------------
// Adam, torch 2.10 single-tensor semantics (torch/optim/adam.py:457,476,531-547):
//   g += wd*p ; m = lerp(m, g, 1-b1) ; v = v*b2 + ((1-b2)*g)*g
//   p += (-lr/bc1 * m) / (sqrt(v)/sqrt(bc2) + eps)
// Hyper-parameters arrive as doubles (Python floats) and are narrowed exactly where
// ATen narrows its Scalar arguments.
// -------------------------------------------------------------------------------------
struct AdamHP {
  double lr, wd, b1, b2, eps;
};

struct AdamC {
  float omb1, b2, omb2, eps, wd, bc2s, nss;
};

template <bool C>
__device__ __forceinline__ AdamC load_adamc(const AdamC* p) {
  if constexpr (!C) {
    return *p;
  } else {
    const float* f = reinterpret_cast<const float*>(p);
    AdamC c;
    c.omb1 = ldc<true>(f);
    c.b2 = ldc<true>(f + 1);
    c.omb2 = ldc<true>(f + 2);
    c.eps = ldc<true>(f + 3);
    c.wd = ldc<true>(f + 4);
    c.bc2s = ldc<true>(f + 5);
    c.nss = ldc<true>(f + 6);
    return c;
  }
}

__device__ __forceinline__ AdamC adam_consts(const AdamHP& hp, int step) {
  AdamC c;
  const double bc1 = 1.0 - pow(hp.b1, (double)step);
  const double bc2 = 1.0 - pow(hp.b2, (double)step);
  c.nss = (float)(-(hp.lr / bc1));
  c.bc2s = (float)sqrt(bc2);
  c.omb1 = (float)(1.0 - hp.b1);
  c.b2 = (float)hp.b2;
  c.omb2 = (float)(1.0 - hp.b2);
  c.eps = (float)hp.eps;
  c.wd = (float)hp.wd;
  return c;
}

// The Adam epilogue's stores (parameters, moments: ≈6 MB per dW launch at C2) are write-through
// (sc1): a kernel boundary costs ≈1.45 µs plus the writeback of what the predecessor left dirty in
// L2 (MI355X_MICROARCH.md, "boundary": + B / 6 TB/s), and the Adam tiles are the largest writers.
// A/B on one box (tools/ab_libs.sh): plain parameters + non-temporal moments 7380 / 7396,
// write-through 7544 / 7567 env-steps/s, non-temporal everything 7357 / 7364.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#ifdef SFX_NO_WT  // diagnostics: the earlier stores (plain parameters, non-temporal moments)
__device__ __forceinline__ void st_moment(float* p, float v) { __builtin_nontemporal_store(v, p); }
template <bool C>
__device__ __forceinline__ void st_param(float* p, float v) { stc<C>(p, v); }
#else
__device__ __forceinline__ void st_moment(float* p, float v) { st_wt(p, v); }
template <bool C>
__device__ __forceinline__ void st_param(float* p, float v) { st_wt(p, v); }
#endif

__device__ __forceinline__ void adam_apply(float& pp, float& mm, float& vv, float g, const AdamC& c) {
  if (c.wd != 0.f) g = __fadd_rn(g, __fmul_rn(c.wd, pp));
  mm = __builtin_fmaf(c.omb1, __fsub_rn(g, mm), mm);  // vectorized lerp: fmadd(w, end-start, start)
  vv = __fadd_rn(__fmul_rn(vv, c.b2), __fmul_rn(__fmul_rn(c.omb2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), c.bc2s), c.eps);
  pp = __fadd_rn(pp, __fdiv_rn(__fmul_rn(c.nss, mm), denom));
}

__device__ __forceinline__ void adam_el(float* p, float* m, float* v, float g, const AdamC& c) {
  float pp = *p, mm = *m, vv = *v;
  adam_apply(pp, mm, vv, g, c);
  *p = pp;
  *m = mm;
  *v = vv;
}

// -------------------------------------------------------------------------------------
// K1  Forward of one Linear (+activation) for a set of (role, head) instances:
//   Y[M,N] = act(X[M,K] W[N,K]^T + b)      (nn.Linear of the ψ lambda,
//                                            main_sfdqn_torch.py:57-71)
// Grid: (ceil(N/16), n_inst, ceil(M/32)), 256 threads.  A workgroup owns a 32x16 output
// tile; its 4 waves split K in 64-wide chunks, each wave runs two 16x16x4 f32 MFMA
// chains, partial tiles are summed through LDS in wave order (deterministic).
// Instances come in up to 4 groups of consecutive heads sharing (role, param set, input).
// Block (0,0,0) of a layer-0 launch may also run the env step's LMS reward fit
// (features/successor.py:164-167) and reset the speculation flag.
// -------------------------------------------------------------------------------------
struct FwdGroup {
  int role, which, xsel, head0, n;  // which: P_*; xsel: 1 -> xa, 2 -> xb, 3 -> xc
  int m;       // rows of this group (0: FwdArgs::M); tiles past them exit
  int noskip;  // FwdArgs::skip does not apply (look-ahead groups of the final device round)
};

struct FwdArgs {
  int M, N, K, act, wOff, bOff, xOff, yOff;  // xOff < 0: layer input is xa / xb
  int ngroups, lms_head, flag_value, xcd;  // xcd: 1-D XCD-aware grid (every group has heads 0..nh-1)
  int nh, ntN, ntM, tpw;  // tpw: column tiles per workgroup (L0 launches; else 1)
  // rowsplit (XCD grids of groups with their own rows, FwdGroup::m): group g has mt_g row tiles
  // and the grid holds ntMs = Σ mt_g of them per (head, column tile) -- no workgroups for rows a
  // group does not have
  int rowsplit, mt0, mt1, mt2, mt3, ntMs;
  // tail: a group's last row tile also takes up to 16 rows past its 32 (a third 16-row MFMA block;
  // plain vector launches only): the 33-row post-update roles in one row tile, not two
  int tail, pad_t;
  int w0Off, b0Off, K0, y0Off;  // L0 launches: layer 0 (K0 -> K, identity) computed in-tile, stored at y0Off
  unsigned long long mask;
  FwdGroup g0, g1, g2, g3;
  const float* xa;
  const float* xb;
  const float* xc;       // a third layer-0 input (the look-ahead select: s_next beside the next minibatch)
  const float* lms_phi;  // LMS (lms_head >= 0): w[lms_head] += α (r - φ·w) φ
  const float* lms_r;
  // or, non-null: a host-coherent word holding r's device address (a device reward tensor of the
  // caller's that changes every step, read without changing the captured launch)
  const unsigned long long* lms_r_ind;
  float lms_alpha;
  int* flag;             // set to flag_value when non-null
  // sharded step (d | 16): GPI maxima accumulated by the last layer's tiles of group role qa_role
  // (see q_accumulate); qa_role < 0: off
  int qa_role, qa_Tg, qa_off, qa_M;
  int* qa_all;   // max over every local head (X of round 0)
  int* qa_ge;    // max over local heads with global index >= policy (the pre-step part)
  int* qa_lt;    // max over local heads with global index < policy (post-update rounds)
  int* qa_sel;   // [Tg][A] selection table of row qa_row with w of qa_task (null: none)
  int qa_row, qa_task, qa_use_gpi, pad3_;
  // sharded rounds: every computed tile also stores its head's terms, qh[head][i][b][a] and the
  // selection row's qhs[head][a]; a head that skips the round (skip) replays them (q_replay)
  int* qh;
  int* qhs;
  // post-update forward of speculative rounds r >= 1: heads whose policy repeats round r-1
  // (BwdArgs::skip) keep the values that round left in the role -- their tiles exit at once
  const int* skip;
};

// The sharded step's GPI maxima, fused into the forward of the ψ output layer: a 32 x 16 tile
// of head t holds whole actions (16 / d of them), so it forms q[i][b][a] = ψ_t(s1_b)[a]·w_i for
// every global policy i straight from the tile (the GPI kernels' k-ordered fmaf chain) and
// atomically maxes it (sortable int32) into X[i][b][a] -- for all i (round 0: every head enters
// through its pre-step values), for i <= t (the pre-step part of later rounds) or for i > t (heads
// already updated in the reference's order: agents/sfdqn.py:57-60).  Row qa_row (s_next) fills the
// selection table with w of the active task.  Replaces a k_qmax launch per round.
constexpr int QA_WMAX = 2048;  // Tg * d of the policies' w rows staged in LDS
__device__ void q_accumulate(const Geo& G, const FwdArgs& F, int head, int tN, int tM, const float* sT) {
  __shared__ float sw[QA_WMAX];
  const int d = G.d, Aa = G.A, Tg = F.qa_Tg, tid = threadIdx.x, nt = blockDim.x;
  const int n0 = tN * 16, m0 = tM * 32, na = 16 / d, a0 = n0 / d, tg = F.qa_off + head;
  for (int j = tid; j < Tg * d; j += nt) {
    const int i = j / d;
    sw[j] = G.w[(long long)i * G.dpad + (j - i * d)];
  }
  __syncthreads();
  const int mrows = F.qa_M - m0 < 32 ? F.qa_M - m0 : 32;
  const int per_i = (mrows > 0 ? mrows : 0) * na;
  for (int it = tid; it < Tg * per_i; it += nt) {
    const int i = it / per_i, rem = it - i * per_i, bl = rem / na, al = rem - bl * na, a = a0 + al;
    if (a >= Aa) continue;
    const bool all = F.qa_all != nullptr, ge = F.qa_ge && tg >= i, lt = F.qa_lt && tg < i;
    if (!all && !ge && !lt) continue;
    const float* p = sT + bl * 16 + al * d;
    const float* w = sw + i * d;
    float q = 0.f;
    for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], w[k], q);
    const int v = sortable(q);
    SFX_CHK(i < Tg && m0 + bl < F.qa_M && head < G.T, i, m0 + bl, head);
    const size_t o = ((size_t)i * F.qa_M + m0 + bl) * Aa + a;
    if (all) atomicMax(F.qa_all + o, v);
    if (ge) atomicMax(F.qa_ge + o, v);
    if (lt) atomicMax(F.qa_lt + o, v);
    if (F.qh) F.qh[(((size_t)head * Tg + i) * F.qa_M + m0 + bl) * Aa + a] = v;
  }
  const int rl = F.qa_row - m0;
  if ((F.qa_sel || F.qhs) && rl >= 0 && rl < 32 && (F.qa_use_gpi || tg == F.qa_task))
    for (int al = tid; al < na; al += nt) {
      const int a = a0 + al;
      if (a >= Aa) continue;
      const float* p = sT + rl * 16 + al * d;
      const float* w = sw + F.qa_task * d;
      float q = 0.f;
      for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], w[k], q);
      const int v = sortable(q);
      if (F.qa_sel) F.qa_sel[(size_t)tg * Aa + a] = v;
      if (F.qhs) F.qhs[(size_t)head * Aa + a] = v;
    }
}

// A head whose policy repeats the previous round (BwdArgs::skip) has the same post-update ψ as
// then: its tiles add the terms they stored in that round (q_accumulate's qh / qhs) instead of
// recomputing them.
__device__ void q_replay(const Geo& G, const FwdArgs& F, int head, int tN, int tM) {
  const int d = G.d, Aa = G.A, Tg = F.qa_Tg, tid = threadIdx.x, nt = blockDim.x;
  const int n0 = tN * 16, m0 = tM * 32, na = 16 / d, a0 = n0 / d, tg = F.qa_off + head;
  const int mrows = F.qa_M - m0 < 32 ? F.qa_M - m0 : 32;
  const int per_i = (mrows > 0 ? mrows : 0) * na;
  for (int it = tid; it < Tg * per_i; it += nt) {
    const int i = it / per_i, rem = it - i * per_i, bl = rem / na, al = rem - bl * na, a = a0 + al;
    if (a >= Aa || !F.qa_lt || tg >= i) continue;
    const int v = F.qh[(((size_t)head * Tg + i) * F.qa_M + m0 + bl) * Aa + a];
    atomicMax(F.qa_lt + ((size_t)i * F.qa_M + m0 + bl) * Aa + a, v);
  }
  const int rl = F.qa_row - m0;
  if (F.qa_sel && rl >= 0 && rl < 32 && (F.qa_use_gpi || tg == F.qa_task))
    for (int al = tid; al < na; al += nt) {
      const int a = a0 + al;
      if (a < Aa) F.qa_sel[(size_t)tg * Aa + a] = F.qhs[(size_t)head * Aa + a];
    }
}

// LMS reward fit (features/successor.py:164-167) by one workgroup: w += α (r - Σ φ⊙w) φ, the sum
// in index order; no store when `cx` (a cancelled runner step).
__device__ void lms_apply(float* w, const float* phi, const float* r, float alpha, int d, int cx) {
  __shared__ float s_p[DMAX];
  __shared__ float s_e;
  const int tid = threadIdx.x;
  const float wk = tid < d ? w[tid] : 0.f, pk = tid < d ? phi[tid] : 0.f;
  if (tid < d) s_p[tid] = __fmul_rn(pk, wk);
  __syncthreads();
  if (tid == 0) {
    float rf = 0.f;
    for (int k = 0; k < d; ++k) rf = __fadd_rn(rf, s_p[k]);
    s_e = __fmul_rn(alpha, __fsub_rn(r[0], rf));
  }
  __syncthreads();
  if (tid < d && !cx) w[tid] = __fadd_rn(wk, __fmul_rn(s_e, pk));
}

__device__ void lms_block(const Geo& G, const FwdArgs& F) {
  const float* r = F.lms_r_ind ? reinterpret_cast<const float*>(F.lms_r_ind[0]) : F.lms_r;
  lms_apply(G.w + (long long)F.lms_head * G.dpad, F.lms_phi, r, F.lms_alpha, G.d, step_cancelled(G.cancel));
}

// L0 = true (layer-1 launches of a forward from the states): the workgroup first computes the
// 32 x K layer-0 rows it needs, a0 = X W0ᵀ + b0 (layer 0 has no activation), into LDS -- each
// column tile recomputes them (K0 is the small state width), the tile-0 workgroups publish
// them for the backward -- and feeds them to the layer-1 MFMAs from LDS: one launch less.
constexpr int L0_KMAX = 64, L0_NMAX = 256;  // layer-0 fan-in / width handled in-tile

// One 32-row x 16-column output tile of instance y (flattened over the groups).  C: coherent
// accesses (data handed between workgroups inside the launch).
// instance y of a forward launch -> its group (y becomes the index inside the group)
__device__ __forceinline__ FwdGroup fwd_group(const FwdArgs& F, int& y) {
  int gs = 0;
  if (F.ngroups > 1 && y >= F.g0.n) { y -= F.g0.n; gs = 1; }
  if (F.ngroups > 2 && gs == 1 && y >= F.g1.n) { y -= F.g1.n; gs = 2; }
  if (F.ngroups > 3 && gs == 2 && y >= F.g2.n) { y -= F.g2.n; gs = 3; }
  auto pick = [gs](int a, int b, int c, int d) { return gs == 0 ? a : gs == 1 ? b : gs == 2 ? c : d; };
  FwdGroup g;
  g.role = pick(F.g0.role, F.g1.role, F.g2.role, F.g3.role);
  g.which = pick(F.g0.which, F.g1.which, F.g2.which, F.g3.which);
  g.xsel = pick(F.g0.xsel, F.g1.xsel, F.g2.xsel, F.g3.xsel);
  g.head0 = pick(F.g0.head0, F.g1.head0, F.g2.head0, F.g3.head0);
  g.n = pick(F.g0.n, F.g1.n, F.g2.n, F.g3.n);
  g.m = pick(F.g0.m, F.g1.m, F.g2.m, F.g3.m);
  g.noskip = pick(F.g0.noskip, F.g1.noskip, F.g2.noskip, F.g3.noskip);
  return g;
}

constexpr int FWD_TPW = 2;  // column tiles per workgroup (FwdArgs::tpw <= TP)

// row tiles of an m-row group (FwdArgs::tail: the last one covers up to 48 rows)
__host__ __device__ __forceinline__ int fwd_row_tiles(int m, int tail) {
  return tail && m > 32 ? (m + 15) >> 5 : (m + 31) >> 5;
}

// TP > 1: the workgroup computes column tiles tN .. tN + tpw - 1 of its rows -- an L0 launch's
// layer-0 rows computed once for them, a plain launch's X operands loaded once for them (launches
// that would otherwise put more workgroups than CUs on the chip)
template <bool VEC, int NW, bool L0, bool C, bool BF = false, int TP = 1>
__device__ __forceinline__ void fwd_tile(const Geo& G, const FwdArgs& F, int y, int tN, int tM, float* sT = nullptr) {
  constexpr int TPW = TP;
  static_assert(TP == 1 || VEC, "several tiles per workgroup: vector tiles only");
  const int ntile = TP == 1 ? 1 : (F.ntN - tN < F.tpw ? F.ntN - tN : F.tpw);
  static_assert(!(L0 && C), "the in-tile layer 0 reads only inputs of earlier launches");
  static_assert(!BF || (VEC && !C), "bf16 operands: vector tiles of plain launches");
  constexpr int KW = 256 / NW;  // K chunk of one wave per iteration (NW waves cover 256)
  constexpr int KL = KW / 4;    // consecutive k per lane (4 lane groups per MFMA k-step)
  // instance -> (group, head) by scalar selects of each field (no dynamic kernarg indexing, and
  // no FwdGroup copy: conditionally copied structs were demoted to scratch, 17 dwords per lane)
  const FwdGroup grp = fwd_group(F, y);
  const int head = grp.head0 + y;
  const int M = grp.m > 0 ? grp.m : F.M, N = F.N, K = F.K;
  if (tM >= fwd_row_tiles(M, F.tail)) return;  // a group with fewer rows than the launch (block-uniform)
  const float* P = grp.which == P_TARGET ? G.target + (long long)head * G.P
                                         : G.online + G.slot_off(rslot(F.mask, head) ^ (grp.which == P_NEW), head);
  const float* X = F.xOff < 0 ? (grp.xsel == 1 ? F.xa : grp.xsel == 2 ? F.xb : F.xc) : G.actp(grp.role, head, F.xOff);
  float* Y = G.actp(grp.role, head, F.yOff);
  const int m0 = tM * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int ma = m0 + r, mb = m0 + 16 + r, mc = m0 + 32 + r;
  const bool oka = ma < M, okb = mb < M;
  // FwdArgs::tail: rows m0 + 32 .. m0 + 47 as a third MFMA block (block-uniform)
  constexpr bool EXT = VEC && !L0 && !C;
  const bool ext = EXT && F.tail && M - m0 > 32;
  const bool okc = ext && mc < M;
  const float* Pw = P + F.wOff;
  // bf16 mode: the W operand from the bf16 copy (same packing, 16-B aligned rows: wOff % 8 == 0)
  const __bf16* Pw16 = nullptr;
  if constexpr (BF)
    Pw16 = (grp.which == P_TARGET ? G.tg16 + (long long)head * G.P
                                  : G.on16 + G.slot_off(rslot(F.mask, head) ^ (grp.which == P_NEW), head)) +
           F.wOff;
  // the reducing threads fetch their biases early
  const int Lx = threadIdx.x & 63;
  float biasv[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int col = (tN + j) * 16 + (Lx & 15);
    biasv[j] = (j < ntile && threadIdx.x < (ext ? 192 : 128) && col < N) ? ldc<C>(P + F.bOff + col) : 0.f;
  }
  constexpr int AS = L0 ? L0_NMAX + 4 : 4;  // LDS row stride of a0 (padded against bank conflicts)
  __shared__ __align__(16) float sA[L0 ? 32 * AS : 4];
  // L0: the first K chunk of this lane's W rows (every tile of the workgroup) is requested before
  // layer 0 is computed, so its latency overlaps the in-tile layer 0 instead of following it
  float4 wpre[TPW][VEC && L0 && !BF ? KL / 4 : 1];
  bf16x8 wpre16[TPW][BF && L0 ? KL / 8 : 1];
  if constexpr (VEC && L0 && !BF) {
    const int kb0 = wave * KW + g * KL;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int nj = (tN + j) * 16 + r;
      const bool ok = j < ntile && nj < N && kb0 < K;
#pragma unroll
      for (int q = 0; q < KL / 4; ++q)
        wpre[j][q] = ok ? ldc4<C>(Pw + (size_t)nj * K + kb0 + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if constexpr (BF && L0) {
    const int kb0 = wave * KW + g * KL;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int nj = (tN + j) * 16 + r;
      const bool ok = j < ntile && nj < N && kb0 < K;
#pragma unroll
      for (int q = 0; q < KL / 8; ++q) wpre16[j][q] = ok ? ld_bf16x8(Pw16 + (size_t)nj * K + kb0 + 8 * q) : bf16x8{};
    }
  }
  if constexpr (L0) {
    __shared__ float sX[32 * L0_KMAX];
    const int K0 = F.K0;
    // a0 = X W0ᵀ + b0 by MFMA: wave w owns layer-0 columns [32w, 32w + 32) (+32·NW ...), K0 in
    // k-steps of 4.  The W0 / b0 operands of the first column block are requested together
    // with the X rows, before the barrier (one memory latency, not one per k-step).
    const float* W0 = P + F.w0Off;
    const float* b0 = P + F.b0Off;
    float* Y0 = G.actp(grp.role, head, F.y0Off);
    constexpr int KS = L0_KMAX / 4;
    float wA[KS], wB[KS], bA, bB;
    auto load_w0 = [&](int cb) {
      const int nA = cb + r, nB = cb + 16 + r;
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        const int kk = 4 * q + g;
        const bool okk = kk < K0;
        wA[q] = okk && nA < K ? W0[(size_t)nA * K0 + kk] : 0.f;
        wB[q] = okk && nB < K ? W0[(size_t)nB * K0 + kk] : 0.f;
      }
      bA = nA < K ? b0[nA] : 0.f;
      bB = nB < K ? b0[nB] : 0.f;
    };
    int cb = wave * 32;
    load_w0(cb);
    for (int j = threadIdx.x; j < 32 * K0; j += 64 * NW) {
      const int rr = j / fdiv(K0), kk = j - rr * K0;
      sX[j] = m0 + rr < M ? X[(size_t)(m0 + rr) * K0 + kk] : 0.f;
    }
    __syncthreads();
    PROBE_AT(3);
    for (; cb < K; cb += 32 * NW) {
      floatx4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c10 = c00, c11 = c00;
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        if (4 * q < K0) {
          const int kk = 4 * q + g;
          const bool okk = kk < K0;
          const float x0 = okk ? sX[r * K0 + kk] : 0.f, x1 = okk ? sX[(16 + r) * K0 + kk] : 0.f;
          c00 = mfma4(x0, wA[q], c00);
          c01 = mfma4(x0, wB[q], c01);
          c10 = mfma4(x1, wA[q], c10);
          c11 = mfma4(x1, wB[q], c11);
        }
      }
      // (no array of pointers to the accumulators: it put them in scratch memory)
      auto put = [&](const floatx4& c, int q) {
        const int cc = cb + (q & 1) * 16 + r;
        if (cc < K) {
          const float bb = (q & 1) ? bB : bA;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rr = (q >> 1) * 16 + g * 4 + i;
            const float v = __fadd_rn(c[i], bb);
            sA[rr * AS + cc] = v;
            if (tN == 0 && m0 + rr < M) {
              G.chk_act(F.y0Off, (long long)(m0 + rr) * K + cc);
              Y0[(size_t)(m0 + rr) * K + cc] = v;
            }
          }
        }
      };
      put(c00, 0);
      put(c01, 1);
      put(c10, 2);
      put(c11, 3);
      if (cb + 32 * NW < K) load_w0(cb + 32 * NW);
    }
    __syncthreads();
    PROBE_AT(4);
  }
  const float* xra = L0 ? sA + r * AS : X + (size_t)ma * K;
  const float* xrb = L0 ? sA + (16 + r) * AS : X + (size_t)mb * K;
  const float* xrc = X + (size_t)(okc ? mc : 0) * K;
  __shared__ floatx4 red[NW][EXT ? 3 : 2][64];
  floatx4 acc0[TPW], acc1[TPW], acc2[EXT ? TPW : 1];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc0[j] = acc1[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < (EXT ? TPW : 1); ++j) acc2[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* wrj[TPW];
  const __bf16* wr16j[TPW];
  bool oknj[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int n = (tN + j) * 16 + r;
    oknj[j] = j < ntile && n < N;
    wrj[j] = Pw + (size_t)(oknj[j] ? n : 0) * K;
    wr16j[j] = BF ? Pw16 + (size_t)(oknj[j] ? n : 0) * K : nullptr;
  }
  for (int kc = wave * KW; kc < K && BF; kc += 256) {
    // bf16 operands: per lane KL consecutive k as KL / 8 MFMA steps of 8 (the fp32 path's k
    // assignment, regrouped), X rounded to bf16 in registers, W from the bf16 copy
    const int kb = kc + g * KL;
    float a0[KL], a1[KL], a2[EXT ? KL : 1];
#pragma unroll
    for (int q = 0; q < KL / 4; ++q) {
      float4 ta, tb;
      if constexpr (L0) {
        ta = reinterpret_cast<const float4*>(xra + kb)[q];
        tb = reinterpret_cast<const float4*>(xrb + kb)[q];
      } else {
        ta = oka ? *reinterpret_cast<const float4*>(xra + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        tb = okb ? *reinterpret_cast<const float4*>(xrb + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      a0[4 * q] = ta.x; a0[4 * q + 1] = ta.y; a0[4 * q + 2] = ta.z; a0[4 * q + 3] = ta.w;
      a1[4 * q] = tb.x; a1[4 * q + 1] = tb.y; a1[4 * q + 2] = tb.z; a1[4 * q + 3] = tb.w;
      if constexpr (EXT) {
        const float4 tc = okc ? *reinterpret_cast<const float4*>(xrc + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        a2[4 * q] = tc.x; a2[4 * q + 1] = tc.y; a2[4 * q + 2] = tc.z; a2[4 * q + 3] = tc.w;
      }
    }
    bf16x8 w16[TPW][KL / 8];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int q = 0; q < KL / 8; ++q) {
        if constexpr (L0)
          w16[j][q] = kc == wave * KW ? wpre16[j][q] : (oknj[j] ? ld_bf16x8(wr16j[j] + kb + 8 * q) : bf16x8{});
        else
          w16[j][q] = oknj[j] ? ld_bf16x8(wr16j[j] + kb + 8 * q) : bf16x8{};
      }
#pragma unroll
    for (int q = 0; q < KL / 8; ++q) {
      const bf16x8 x0 = to_bf16x8(a0 + 8 * q), x1 = to_bf16x8(a1 + 8 * q);
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        acc0[j] = mfma_bf16(x0, w16[j][q], acc0[j]);
        acc1[j] = mfma_bf16(x1, w16[j][q], acc1[j]);
      }
    }
    if constexpr (EXT)
      if (ext)
#pragma unroll
        for (int q = 0; q < KL / 8; ++q) {
          const bf16x8 x2 = to_bf16x8(a2 + 8 * q);
#pragma unroll
          for (int j = 0; j < TPW; ++j) acc2[j] = mfma_bf16(x2, w16[j][q], acc2[j]);
        }
  }
  for (int kc = wave * KW; kc < K && !BF; kc += 256) {
    const int kb = kc + g * KL;
    float a0[KL], a1[KL], bw[TPW][KL], a2[EXT ? KL : 1];
    if constexpr (VEC) {  // K % KW == 0, rows 16-B aligned: KL/4 float4 per operand row
#pragma unroll
      for (int q = 0; q < KL / 4; ++q) {
        float4 ta, tb;
        if constexpr (L0) {  // a0 from LDS
          ta = reinterpret_cast<const float4*>(xra + kb)[q];
          tb = reinterpret_cast<const float4*>(xrb + kb)[q];
        } else {
          ta = oka ? ldc4<C>(xra + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
          tb = okb ? ldc4<C>(xrb + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          float4 tw;
          if constexpr (L0 && !BF) {
            tw = kc == wave * KW ? wpre[j][q]
                                 : (oknj[j] ? ldc4<C>(wrj[j] + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f));
          } else {
            tw = oknj[j] ? ldc4<C>(wrj[j] + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
          }
          bw[j][4 * q] = tw.x; bw[j][4 * q + 1] = tw.y; bw[j][4 * q + 2] = tw.z; bw[j][4 * q + 3] = tw.w;
        }
        a0[4 * q] = ta.x; a0[4 * q + 1] = ta.y; a0[4 * q + 2] = ta.z; a0[4 * q + 3] = ta.w;
        a1[4 * q] = tb.x; a1[4 * q + 1] = tb.y; a1[4 * q + 2] = tb.z; a1[4 * q + 3] = tb.w;
        if constexpr (EXT) {
          const float4 tc = okc ? ldc4<C>(xrc + kb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
          a2[4 * q] = tc.x; a2[4 * q + 1] = tc.y; a2[4 * q + 2] = tc.z; a2[4 * q + 3] = tc.w;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < KL; ++i) {
        const bool kin = kb + i < K;
        if constexpr (L0) {
          a0[i] = (oka && kin) ? xra[kb + i] : 0.f;
          a1[i] = (okb && kin) ? xrb[kb + i] : 0.f;
        } else {
          a0[i] = (oka && kin) ? ldc<C>(xra + kb + i) : 0.f;
          a1[i] = (okb && kin) ? ldc<C>(xrb + kb + i) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < TPW; ++j) bw[j][i] = (oknj[j] && kin) ? ldc<C>(wrj[j] + kb + i) : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < KL; ++i)
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        acc0[j] = mfma4(a0[i], bw[j][i], acc0[j]);
        acc1[j] = mfma4(a1[i], bw[j][i], acc1[j]);
      }
    if constexpr (EXT)
      if (ext)
#pragma unroll
        for (int i = 0; i < KL; ++i)
#pragma unroll
          for (int j = 0; j < TPW; ++j) acc2[j] = mfma4(a2[i], bw[j][i], acc2[j]);
  }
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
  if (j >= ntile) continue;  // block-uniform
  const int n0 = (tN + j) * 16, col = n0 + (Lx & 15);
  const float bias = biasv[j];
  PROBE_MARK();
  if (j > 0) __syncthreads();  // the previous tile's reduction has read red
  red[wave][0][lane] = acc0[j];
  red[wave][1][lane] = acc1[j];
  if constexpr (EXT)
    if (ext) red[wave][EXT ? 2 : 1][lane] = acc2[EXT ? j : 0];
  __syncthreads();
  if (threadIdx.x < (ext ? 192 : 128)) {
    const int s = threadIdx.x >> 6;
    floatx4 v = red[0][s][Lx];
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) v += red[w2][s][Lx];
    if (col < N) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * s + (Lx >> 4) * 4 + i;
        const float o = act_fwd(__fadd_rn(v[i], bias), F.act);
        if (row < M) {
          G.chk_act(F.yOff, (long long)row * N + col);
          stc<C>(Y + (size_t)row * N + col, o);
        }
        if (sT) sT[(row - m0) * 16 + (col - n0)] = row < M ? o : 0.f;
      }
    }
  }
  }  // tiles
}

constexpr int qa_tile_floats(bool L0) { return L0 ? 1 : 32 * 16; }  // L0 launches never accumulate

// workgroup (bx, by, bz) of a forward launch's grid (k_fwd; k_fwd_tsf after its TSF blocks)
template <bool VEC, int NW, bool L0, bool BF, int TP>
__device__ __forceinline__ void fwd_body(const Geo& G, const FwdArgs& F, int bx, int by, int bz) {
  PROBE_T(pt0);
  int y = by, tN = bx, tM = bz;
  const int ntNb = TP > 1 ? (F.ntN + F.tpw - 1) / F.tpw : F.ntN;  // workgroups along N
  if (F.xcd) {  // head h's tiles on the XCD of slot h % 8 (see xcd_decode)
    const int b = bx, hp = (F.nh + 7) >> 3, k = b >> 3;
    const int r = hp == 1 ? k : k / fdiv(hp), hd = (b & 7) + 8 * (k - r * hp);
    const int rN = r / fdiv(ntNb);
    int gi;
    tN = r - rN * ntNb;
    if (F.rowsplit) {
      tM = rN;
      gi = 0;
      if (tM >= F.mt0) {
        tM -= F.mt0;
        gi = 1;
        if (tM >= F.mt1) {
          tM -= F.mt1;
          gi = 2;
          if (tM >= F.mt2) {
            tM -= F.mt2;
            gi = 3;
          }
        }
      }
    } else {
      gi = rN / fdiv(F.ntM);
      tM = rN - gi * F.ntM;
    }
    if (hd >= F.nh || gi >= F.ngroups) return;
    y = gi * F.nh + hd;
  }
  if constexpr (TP > 1) tN *= F.tpw;
  bool qa = false;
  int head = 0;
  if (F.qa_role >= 0) {  // the sharded step's maxima from this tile (last layer, group role qa_role)
    int yy = y;
    const FwdGroup grp = fwd_group(F, yy);
    qa = grp.role == F.qa_role;
    head = grp.head0 + yy;
  }
  if (F.skip) {  // instance y is the head inside its group
    int yy = y;
    const FwdGroup grp = fwd_group(F, yy);
    if (!grp.noskip && __builtin_nontemporal_load(F.skip + grp.head0 + yy)) {
      if (qa && F.qh) q_replay(G, F, head, tN, tM);  // its maxima terms as that round stored them
      return;
    }
  }
  __shared__ float sT[qa_tile_floats(L0)];
  fwd_tile<VEC, NW, L0, false, BF, TP>(G, F, y, tN, tM, qa ? sT : nullptr);
  if (qa) q_accumulate(G, F, head, tN, tM, sT);
  if (tN == 0 && tM == 0 && by == 0 && (F.xcd ? bx == 0 : true)) {
    if (F.flag && threadIdx.x == 0) *F.flag = F.flag_value;
    if (F.lms_head >= 0) lms_block(G, F);
  }
  PROBE_REC(L0 ? 2 : 1, pt0);
}

template <bool VEC, int NW, bool L0, bool BF = false, int TP = 1>
__global__ __launch_bounds__(64 * NW) void k_fwd(Geo G, FwdArgs F) {
  fwd_body<VEC, NW, L0, BF, TP>(G, F, blockIdx.x, blockIdx.y, blockIdx.z);
}

// K1b  Forward of a wide layer (N >= GEMV_N) for a few rows (M <= GEMV_M: the B = 1 action
// choice): GEMV-shaped, no MFMA.  Grid (ceil(N / 64), n_inst), 256 threads; a wave owns 16
// output columns, 4 lanes per column each summing K / 4 products (lane q takes k = 16 i + 4 q
// .. + 3, so the 4 lanes of a column read 64 contiguous bytes of its W row per step), a quad
// DPP butterfly finishes the dot.  Every W and X load of a lane is issued before the first FMA.
__global__ __launch_bounds__(256) void k_fwd_gemv(Geo G, FwdArgs F) {
  PROBE_T(pt0);
  int y = blockIdx.y;
  const FwdGroup grp = fwd_group(F, y);
  const int head = grp.head0 + y;
  if (F.skip && __builtin_nontemporal_load(F.skip + head)) return;
  const int M = F.M, N = F.N, K = F.K;
  const float* P = grp.which == P_TARGET ? G.target + (long long)head * G.P
                                         : G.online + G.slot_off(rslot(F.mask, head) ^ (grp.which == P_NEW), head);
  const float* X = F.xOff < 0 ? (grp.xsel == 1 ? F.xa : grp.xsel == 2 ? F.xb : F.xc) : G.actp(grp.role, head, F.xOff);
  float* Y = G.actp(grp.role, head, F.yOff);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane & 3;
  const int n = blockIdx.x * 64 + wave * 16 + (lane >> 2);
  const bool okn = n < N;
  const float* wr = P + F.wOff + (size_t)(okn ? n : 0) * K;
  float acc[GEMV_M];
#pragma unroll
  for (int m = 0; m < GEMV_M; ++m) acc[m] = 0.f;
  // K in chunks of 256 (4 lanes x 16 steps x float4); K % 16 == 0 (checked by the host)
  for (int kc = 0; kc < K; kc += 256) {
    float4 wv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = kc + 16 * i + 4 * q;
      wv[i] = k < K ? *reinterpret_cast<const float4*>(wr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int m = 0; m < GEMV_M; ++m) {
      if (m < M) {
        const float* xr = X + (size_t)m * K;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int k = kc + 16 * i + 4 * q;
          const float4 xv = k < K ? *reinterpret_cast<const float4*>(xr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
          acc[m] = __builtin_fmaf(xv.x, wv[i].x, acc[m]);
          acc[m] = __builtin_fmaf(xv.y, wv[i].y, acc[m]);
          acc[m] = __builtin_fmaf(xv.z, wv[i].z, acc[m]);
          acc[m] = __builtin_fmaf(xv.w, wv[i].w, acc[m]);
        }
      }
    }
  }
  const float bias = okn ? P[F.bOff + n] : 0.f;
#pragma unroll
  for (int m = 0; m < GEMV_M; ++m) {
    float v = acc[m];
    v = __fadd_rn(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
    v = __fadd_rn(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
    if (m < M && okn && q == 0) Y[(size_t)m * N + n] = act_fwd(__fadd_rn(v, bias), F.act);
  }
  PROBE_REC(19, pt0);
}

// The ψ loss of one element x = c - t of the merged-clone TD target.  MSELoss(mean) (the
// reference's, sfdqn.py:341-342): gradient (2/N) x, loss x².  Opt-in HuberLoss(delta = δ, mean)
// (north_star's wording): gradient (1/N) clamp(x, -δ, δ) as torch's
// huber_loss_backward forms it (±(1/N)·δ outside), loss 0.5 x² for |x| < δ, else δ (|x| - 0.5 δ).
// The loss tail divides Σ rowloss by N = M·O for both.
__device__ __forceinline__ float td_norm(const Geo& G, int M, int O, const float* dz_scale) {
  const float n = (float)((G.huber > 0.f ? 1.0 : 2.0) / ((double)M * (double)O));
  return dz_scale ? __fmul_rn(n, *dz_scale) : n;
}
__device__ __forceinline__ float td_grad(float huber, float norm, float x) {
  if (huber > 0.f) {
    const float nd = __fmul_rn(norm, huber);
    return x < -huber ? -nd : (x > huber ? nd : __fmul_rn(norm, x));
  }
  return __fmul_rn(norm, x);
}
__device__ __forceinline__ float td_loss(float huber, float x) {
  if (huber > 0.f) {
    const float z = fabsf(x);
    return z < huber ? __fmul_rn(__fmul_rn(0.5f, z), z) : __fmul_rn(huber, __fsub_rn(z, __fmul_rn(0.5f, huber)));
  }
  return __fmul_rn(x, x);
}

// -------------------------------------------------------------------------------------
// K2  TD target and output gradient, one workgroup per (policy, minibatch row b)
// (sfdqn.py:313-341; features/deep.py:101-120):
//   a'_b = argmax_a max_t ψ_t(s1_b)[a]·w_i        (GPI branch)
//        = argmax_a ψ_i(s1_b)[a]·w_i              (own-ψ branch)
//   t_b  = φ_b + γ_b ψ⁻_i(s1_b)[a'_b]
//   g[b, a_b, :] = 2 (c[b,a_b,:] - t_b) / (M*A*d), 0 elsewhere  (MSE vs merged clone)
//   rowloss[i][b] = Σ_k (c[b,a_b,k] - t_b[k])^2
// Policy i takes ψ_t(s1) of heads t < i from role `guess` and of heads t >= i from R_S1
// (before the step).  In the reference's in-order loop heads t < i are already updated;
// guess = R_S1 speculates they did not move, guess = R_V uses the post-update values
// of the previous speculative round (see k_ver).
// Grid (M, npol), 256 threads.  Policies pol0 .. pol0+npol-1.
// -------------------------------------------------------------------------------------
// Round skipping for the TD launches that are not the fused one (k_tdg, k_tdgw; BwdArgs::skip):
// every workgroup covering rows of policy `pol` reports whether any of its rows' next actions
// differ from the previous round's (prev; null in round 0: always "differs") with ONE relaxed
// atomic add on the policy's word -- 1 per report, + 2^16 when it differs -- so the count and the
// verdict travel in the same word and no release / acquire (an L2 write-back per workgroup on
// gfx950's 8 XCDs) is needed; the report that completes the count (`nrep`) writes skip[pol] (read
// by the later launches of the round: the kernel boundary orders it), counts the statistics and
// re-arms the word ([T] after skip[T]) for the next launch.
__device__ __forceinline__ void tdg_skip_report(int* skip, unsigned long long* skipc, int pol, int T, bool differs,
                                                bool have_prev, int nrep) {
  int* word = skip + T + pol;
  const int old = __hip_atomic_fetch_add(word, differs ? 0x10001 : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((old & 0xFFFF) == nrep - 1) {
    const bool any = (old >> 16) != 0 || differs;
    skip[pol] = any ? 0 : 1;
    if (skipc && have_prev) {
      atomicAdd(skipc, 1ull);
      if (!any) atomicAdd(skipc + 1, 1ull);
    }
    __hip_atomic_store(word, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct TdgArgs {
  int M, use_gpi, pol0, npol, guess, next_stride, flag_value, pad_;
  const int64_t* a;
  const float* phi;
  const float* gamma;
  int64_t* next;  // next[(policy - pol0) * next_stride + b] or null
  int* flag;      // reset to flag_value by block (0, 0) when non-null
  // sharded heads: max over ALL heads of q[b, t, a] (all-reduced across ranks, sortable int32),
  // indexed by the global policy poloff + pol; replaces the local GPI reduction when non-null
  const int* xmax;
  int poloff, pad2_;
  const float* dz_scale;  // learned φ: the output gradient is scaled by the loss coefficient λ (device)
  // round skipping (tdg_skip_report): prev = the previous round's next actions (same indexing as
  // next; null in round 0), skip / skipc as BwdArgs; skip null: no skipping
  const int64_t* prev;
  int* skip;
  unsigned long long* skipc;
};

__global__ __launch_bounds__(256) void k_tdg(Geo G, TdgArgs A) {
  PROBE_T(pt0);
  const int b = blockIdx.x, pol = A.pol0 + blockIdx.y, tid = threadIdx.x;
  const int T = G.T, Aa = G.A, d = G.d, O = G.O, M = A.M, NLm = G.lastOff;
  __shared__ float s_w[DMAX];
  __shared__ float s_q[QMAX];
  __shared__ float s_t[OMAX];  // ψ⁻_i(s1_b) row
  __shared__ float s_m[256];
  __shared__ float s_sq[DMAX];
  __shared__ int s_next;
  const float* wrow = G.w + (long long)pol * G.dpad;
  for (int k = tid; k < d; k += 256) s_w[k] = wrow[k];
  if (A.flag && b == 0 && blockIdx.y == 0 && tid == 0) *A.flag = A.flag_value;
  const float* trow = G.actp(R_S1T, pol, NLm) + (size_t)b * O;
  for (int o = tid; o < O; o += 256) s_t[o] = trow[o];
  const int ab = (int)A.a[b];
  const bool aok = ab >= 0 && ab < Aa;
  float cval = 0.f, phik = 0.f;
  const float gam = A.gamma[b];
  if (tid < d) {
    phik = A.phi[(size_t)b * d + tid];
    if (aok) cval = G.actp(R_S, pol, NLm)[(size_t)b * O + ab * d + tid];
  }
  __syncthreads();
  if (A.xmax) {
    const int* xr = A.xmax + ((size_t)(A.poloff + pol) * M + b) * Aa;
    for (int a = tid; a < Aa; a += 256) s_m[a] = unsortable(xr[a]);
  } else {
    const int t0 = A.use_gpi ? 0 : pol, nt = A.use_gpi ? T : 1;
    const FDiv fA = fdiv(Aa);
    for (int idx = tid; idx < nt * Aa; idx += 256) {
      const int tq = idx / fA, t = t0 + tq, a = idx - tq * Aa;
      const float* p = G.actp(t < pol ? A.guess : R_S1, t, NLm) + (size_t)b * O + a * d;
      float q = 0.f;
#pragma unroll 8
      for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
      s_q[idx] = q;
    }
    __syncthreads();
    for (int a = tid; a < Aa; a += 256) {  // max over heads for each action (torch.max(q1, axis=1))
      float mx = s_q[a];
      for (int t = 1; t < nt; ++t) mx = fmaxf(mx, s_q[t * Aa + a]);
      s_m[a] = mx;
    }
  }
  __syncthreads();
  if (tid == 0) {  // argmax over actions, first index on ties
    int am = 0;
    float qm = s_m[0];
    for (int a = 1; a < Aa; ++a)
      if (s_m[a] > qm) {
        qm = s_m[a];
        am = a;
      }
    s_next = am;
    SFX_CHK(b < A.next_stride || !A.next, b, A.next_stride, 0);
    if (A.next) A.next[(size_t)blockIdx.y * A.next_stride + b] = am;
    if (A.skip)
      tdg_skip_report(A.skip, A.skipc, pol, T, !A.prev || A.prev[(size_t)blockIdx.y * A.next_stride + b] != am,
                      A.prev != nullptr, M);
  }
  __syncthreads();
  const float norm = td_norm(G, M, O, A.dz_scale);
  float* grow = G.dzp(pol, NLm) + (size_t)b * O;
  const float* crow = G.actp(R_S, pol, NLm) + (size_t)b * O;
  const int an = s_next;
  for (int o = tid; o < O; o += 256) {
    float gv = 0.f;
    if (aok && o >= ab * d && o < ab * d + d) {
      const int k = o - ab * d;
      const float tg = __fadd_rn(A.phi[(size_t)b * d + k], __fmul_rn(gam, s_t[an * d + k]));
      gv = td_grad(G.huber, norm, __fsub_rn(crow[o], tg));
    }
    grow[o] = gv;
  }
  float dsq = 0.f;
  if (tid < d && aok) {
    const float diff = __fsub_rn(cval, __fadd_rn(phik, __fmul_rn(gam, s_t[an * d + tid])));
    dsq = td_loss(G.huber, diff);
    if (!__builtin_isfinite(diff) && G.nonfin) atomicOr(G.nonfin, 1);
  }
  if (tid < d) s_sq[tid] = dsq;
  __syncthreads();
  if (tid == 0) {  // row Σ diff^2 in feature order
    float s = 0.f;
    for (int k = 0; k < d; ++k) s = __fadd_rn(s, s_sq[k]);
    SFX_CHK(pol >= 0 && pol < G.T && b < MMAX, pol, b, 0);
    G.rowloss[(long long)pol * MMAX + b] = s;
  }
  PROBE_REC(17, pt0);
}

// -------------------------------------------------------------------------------------
// K3  Backward through the ψ MLP with Adam fused into the weight-gradient epilogue
// (autograd of sfdqn.py:344-345 + optim.step() at :362).
//   dX role : dZ_{l-1} = (dZ_l W_l) ⊙ act'(X_l)        32x16 tile, split over the 4 waves
//   dW role : dW_l = dZ_l^T X_l ; db_l = Σ_m dZ_l ; Adam(W_l, b_l) read slot -> write slot
//   tail    : (first launch only) l1 from the per-row losses, optional l2 = MSE(w_i·φ, r)
//             with one Adam step on w_i (sfdqn.py:340-342), Adam step counter += 1.
// Layers are walked in a ping-pong (dX of l with dW of l+1) so each launch needs only one
// dZ.  With fuse_v0 the layer-0 dW tiles also run the post-update forward of layer 0 for
// the rows of S1 (and s_next) into R_V from the freshly written parameters.
// blockIdx.x selects the role: [0, na) dX; [na, na+nb) dW rb; [.., +nc) dW rc; then tail.
// blockIdx.y = head - head0.
// -------------------------------------------------------------------------------------
struct RoleGeo {
  int N, K, wOff, bOff, actIn;
  int xOff;   // input activation offset (R_S block); < 0: the minibatch states x0
  int dzOff;  // this layer's output-gradient offset (dz block)
  int dzIn;   // dX role: offset of the gradient it writes (layer l-1)
};

struct BwdArgs {
  int M, na, nb, nc, tail, head0, train_w, inc_step;
  int xcd, nhead;               // xcd: 1-D XCD-aware grid (xcd_decode) over nhead heads
  int step_in_tail;             // 1: the tail bumps the Adam step; 0: dX tile 0 of this launch does
  int tdg, tdg_use_gpi, tdg_guess, tdg_next_stride, flag_value, pad2_;  // fused TD target (K2)
  const int64_t* tdg_a;
  const float* tdg_gamma;
  int64_t* tdg_next;
  const int* tdg_xmax;  // sharded heads: all-reduced GPI maxima (see TdgArgs::xmax)
  int tdg_poloff, pad3_;
  int* flag;
  int fuse_v0, vM, vOff, act0;  // fused forward: rows (S1 ++ s_next), layer-0 offset, layer-0 act
  int vRole, dxs;               // role block the fused forward writes; dX split over N (1: none)
  unsigned long long mask;
  // dxs > 1 (wide layers): the dX tiles of one (head, tile) split N over dxs workgroups; each
  // writes its partial tile to dxpart (coherent stores), arrives on dxctr[head][tile], and the
  // last to arrive sums the partials in split order (deterministic) and stores dZ_{l-1}
  float* dxpart;
  unsigned* dxctr;
  RoleGeo ra, rb, rc;  // dX role (layer la), dW roles (lb, lc)
  AdamHP hp, hpw;
  const float* x0;     // layer-0 input (the minibatch states S)
  const float* phi;    // tail: [M, d]
  const float* r;      // tail: [M] rewards (train_w)
  float* losses;       // tail: [n_head][3] (l1+l2, l1, l2) or null
  const float* v_x;    // fused forward input rows 0..M-1 (S1)
  const float* v_xn;   // fused forward input row M (s_next) or null
  // look-ahead rows of the fused forward (runner steps): ax = [NS (aM rows) | NS1 (aM
  // rows)], the next step's minibatch states; layer 0 of NS -> R_NS, NS1 -> R_NS1 with the
  // post-update weights and NS1 -> R_NS1T with the target weights.  aM = 0: none.  a_noskip: the
  // layer-0 tiles of a head that skips this round still compute them (first round that has them)
  const float* ax;
  int aM, a_noskip;
  // sharded step: the fused-TD launch re-initialises the next round's maxima buffer (xi_dst[j] =
  // xi_src[j] for j < xi_copy, SORT_EMPTY up to xi_n) -- its last reader was an earlier launch
  const int* xi_src;
  int* xi_dst;
  int xi_copy, xi_n;
  // speculative rounds r >= 1 (fused TD launch only): tdg_prev = round r-1's next actions
  // [head][MMAX].  A policy whose next actions all equal them repeats round r-1's update bit
  // for bit -- same targets, same gradients, same Adam step from the same read slot into the same
  // write slot -- so its tiles skip: the TD launch sets skip[head] (0 or 1, every round: round 0
  // has no tdg_prev and clears it) and the later launches of the round test it.  The post-update
  // forward still runs for every head (reading the write slot, which already holds the result).
  // skipc: [0] policies checked, [1] policies skipped (statistics).
  const int64_t* tdg_prev;
  int* skip;
  unsigned long long* skipc;
  int skip_v0, pad4_;  // skipped heads' layer-0 tiles: 1 = the post-update forward skips them too
  // learned φ (features/deep_phi.py): the output gradient scaled by λ (device scalar)
  const float* dz_scale;
};

__device__ __forceinline__ const float* layer_input(const Geo& G, const BwdArgs& A, int head, int xOff) {
  return xOff < 0 ? A.x0 : G.actp(R_S, head, xOff);
}

// K2 fused into the first backward launch: the TD target and output gradient of the 32 rows
// m0.. of policy `pol` (the arithmetic of k_tdg, in the same order), left in LDS (s.dz, row
// stride O) for this tile's dX.  The k-tile 0 workgroup of each row tile also publishes dZ,
// the per-row losses and the next actions for the later launches.
// Every global load is issued in stage A (one memory latency); stages B-E run from LDS.
// Shapes (can_fuse_tdg): d = 4V <= 4 VMAX, 32·T·A <= 256 U, A·d <= 128.
constexpr int TDG_ROWS_O = 128;  // max A*d of a fused row tile
struct TdgSmem {
  float w[32], gam[32], ph[32 * 16];
  int a[32], n[32];
  float q[2048], m[32 * 128];
  float tt[32 * TDG_ROWS_O], tc[32 * TDG_ROWS_O];
  float dz[32 * TDG_ROWS_O];
};

// Returns 1 when the policy repeats the previous round's update (BwdArgs::tdg_prev): then the
// output gradient and the row losses are left as that round wrote them.
template <int VMAX, int U, bool C>
__device__ int tdg_rows(const Geo& G, const BwdArgs& A, int pol, int m0, bool pub, TdgSmem& sm) {
  const int tid = threadIdx.x, T = G.T, Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff, M = A.M;
  const int nb = M - m0 < 32 ? M - m0 : 32;
  const bool xm = A.tdg_xmax != nullptr;
  const int t0 = A.tdg_use_gpi ? 0 : pol, nt = A.tdg_use_gpi ? T : 1, TA = nt * Aa, n = xm ? 0 : nb * TA, V = d >> 2;
  const int guess = A.tdg_guess;
  const FDiv fTA = fdiv(TA), fA = fdiv(Aa);
  // ---- stage A: all global loads
  float4 v[U][VMAX];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int idx = tid + u * 256;
    const bool ok = idx < n;
    const int bl = idx / fTA, rem = idx - bl * TA, tq = rem / fA, t = t0 + tq, a = rem - tq * Aa;
    const float4* p = reinterpret_cast<const float4*>(G.actp(t < pol ? guess : R_S1, ok ? t : 0, NLm) +
                                                      (ok ? (size_t)(m0 + bl) * O + a * d : 0));
#pragma unroll
    for (int j = 0; j < VMAX; ++j) v[u][j] = (ok && j < V) ? p[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int n4 = (nb * O) >> 2;  // row tiles are whole float4s (O % 4 == 0)
  const float4* tg4 = reinterpret_cast<const float4*>(G.actp(R_S1T, pol, NLm) + (size_t)m0 * O);
  const float4* cu4 = reinterpret_cast<const float4*>(G.actp(R_S, pol, NLm) + (size_t)m0 * O);
  float4 tt[4], tc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 256;
    tt[u] = i < n4 ? tg4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    tc[u] = i < n4 ? cu4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int np4 = (nb * d) >> 2;
  const float4 ph = tid < np4 ? reinterpret_cast<const float4*>(A.phi + (size_t)m0 * d)[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float wk = tid < d ? G.w[(long long)pol * G.dpad + tid] : 0.f;
  const int ab_l = tid < nb ? (int)A.tdg_a[m0 + tid] : 0;
  const float gam_l = tid < nb ? A.tdg_gamma[m0 + tid] : 0.f;
  int xv[4];  // raw sortable ints: decoded after the barrier, so no wait is placed here
  if (xm) {  // the all-reduced maxima rows of this policy: stage C's output
    const int* xr = A.tdg_xmax + ((size_t)(A.tdg_poloff + pol) * M + m0) * Aa;
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = tid + u * 256 < nb * Aa ? xr[tid + u * 256] : 0;
  }
  // the previous round's next action of this thread's row, requested with the other operands
  // (stage D compares against it; a load there would cost a dependent round trip)
  const int64_t* prev = A.tdg_prev ? A.tdg_prev + (size_t)(pol - A.head0) * A.tdg_next_stride + m0 : nullptr;
  const int64_t prev_l = prev && tid < nb ? prev[tid] : -1;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 256;
    if (i < n4) {
      reinterpret_cast<float4*>(sm.tt)[i] = tt[u];
      reinterpret_cast<float4*>(sm.tc)[i] = tc[u];
      reinterpret_cast<float4*>(sm.dz)[i] = make_float4(0.f, 0.f, 0.f, 0.f);  // stage E fills the taken actions
    }
  }
  if (tid < np4) reinterpret_cast<float4*>(sm.ph)[tid] = ph;
  if (tid < d) sm.w[tid] = wk;
  if (tid < nb) {
    sm.a[tid] = ab_l;
    sm.gam[tid] = gam_l;
  }
  __syncthreads();
  PROBE_AT(3);
  if (xm) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (tid + u * 256 < nb * Aa) sm.m[tid + u * 256] = unsortable(xv[u]);
  }
  // ---- stage B: q = ψ·w, one fmaf chain per dot in k order
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int idx = tid + u * 256;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VMAX; ++j) {
      if (j < V) {
        q = __builtin_fmaf(v[u][j].x, sm.w[4 * j], q);
        q = __builtin_fmaf(v[u][j].y, sm.w[4 * j + 1], q);
        q = __builtin_fmaf(v[u][j].z, sm.w[4 * j + 2], q);
        q = __builtin_fmaf(v[u][j].w, sm.w[4 * j + 3], q);
      }
    }
    if (idx < n) sm.q[idx] = q;
  }
  __syncthreads();
  PROBE_AT(5);
  // ---- stage C: max over heads per (row, action)   (torch.max(q1, axis=1))
  for (int i = tid; i < (xm ? 0 : nb * Aa); i += 256) {
    const int bl = i / fA, a = i - bl * Aa;
    const float* qb = sm.q + bl * TA + a;
    float mx = qb[0];
    for (int t = 1; t < nt; ++t) mx = fmaxf(mx, qb[t * Aa]);
    sm.m[i] = mx;
  }
  __syncthreads();
  PROBE_AT(6);
  // ---- stage D: first argmax over actions
  int differs = prev == nullptr || m0 != 0 || nb != M;  // skipping needs every row of the policy
  for (int bl = tid; bl < nb; bl += 256) {
    const float* mb = sm.m + bl * Aa;
    int am = 0;
    float qm = mb[0];
    for (int a = 1; a < Aa; ++a)
      if (mb[a] > qm) {
        qm = mb[a];
        am = a;
      }
    sm.n[bl] = am;
    if (prev && (bl == tid ? prev_l : prev[bl]) != am) differs = 1;
    SFX_CHK(!(pub && A.tdg_next) || (m0 + bl < A.tdg_next_stride && pol - A.head0 >= 0), pol, m0 + bl,
            A.tdg_next_stride);
    if (pub && A.tdg_next) A.tdg_next[(size_t)(pol - A.head0) * A.tdg_next_stride + m0 + bl] = am;
  }
  const int same = !__syncthreads_or(differs);
  if (pub && A.skip && tid == 0) {
    A.skip[pol] = same;
    if (A.skipc && prev) {
      atomicAdd(A.skipc, 1ull);
      if (same) atomicAdd(A.skipc + 1, 1ull);
    }
  }
  if (same) return 1;
  PROBE_AT(4);
  // ---- stage E: output gradient rows -- nonzero only at the taken action: one thread per
  // (row, feature) of it -- and the rows' squared errors (into sm.q, free after stage C)
  const float norm = td_norm(G, M, O, A.dz_scale);
  const FDiv fd = fdiv(d);
  float* sq = sm.q;
  int nf = 0;
  for (int i = tid; i < nb * d; i += 256) {
    const int bl = i / fd, k = i - bl * d, ab = sm.a[bl];
    float e2 = 0.f;
    if (ab >= 0 && ab < Aa) {
      const float tg = __fadd_rn(sm.ph[bl * d + k], __fmul_rn(sm.gam[bl], sm.tt[bl * O + sm.n[bl] * d + k]));
      const float diff = __fsub_rn(sm.tc[bl * O + ab * d + k], tg);
      sm.dz[bl * O + ab * d + k] = td_grad(G.huber, norm, diff);
      e2 = td_loss(G.huber, diff);
      nf |= !__builtin_isfinite(diff);
    }
    sq[i] = e2;
  }
  if (__syncthreads_or(nf) && tid == 0 && G.nonfin) atomicOr(G.nonfin, 1);
  PROBE_AT(7);
  if (pub) {
    float4* gout4 = reinterpret_cast<float4*>(G.dzp(pol, NLm) + (size_t)m0 * O);
    for (int i = tid; i < n4; i += 256) {
      const float4 v = reinterpret_cast<const float4*>(sm.dz)[i];
      if constexpr (C) {
        float* o = reinterpret_cast<float*>(gout4 + i);
        stc<true>(o, v.x);
        stc<true>(o + 1, v.y);
        stc<true>(o + 2, v.z);
        stc<true>(o + 3, v.w);
      } else {
        gout4[i] = v;
      }
    }
    for (int bl = tid; bl < nb; bl += 256) {  // row Σ diff^2 in feature order
      float sacc = 0.f;
      for (int k = 0; k < d; ++k) sacc = __fadd_rn(sacc, sq[bl * d + k]);
      SFX_CHK(pol >= 0 && pol < G.T && m0 + bl < MMAX, pol, m0 + bl, 0);
      G.rowloss[(long long)pol * MMAX + m0 + bl] = sacc;
    }
  }
  PROBE_AT(8);
  return 0;
}

template <bool TDG, int VMAX = 2, int U = 8, bool C = false, bool BF = false>
__device__ __forceinline__ void role_dx(const Geo& G, const BwdArgs& A, int head, int tile, floatx4 (*red)[2][64]) {
  static_assert(!(BF && (TDG || C)), "bf16 dX: the plain dX tiles only (the fused TD launch stays fp32)");
  const RoleGeo L = A.ra;
  const int N = L.N, K = L.K, M = A.M;
  const int ntk = (K + 15) >> 4;
  // split of N (TDG launches never split: their N <= 128)
  const int split = TDG ? 0 : tile % A.dxs;
  tile = TDG ? tile : tile / A.dxs;
  const int nchunk = ((N + A.dxs - 1) / A.dxs + 63) & ~63;
  const int nbeg = split * nchunk, nend = min(N, nbeg + nchunk);
  const int k0 = (tile % ntk) * 16, m0 = (tile / ntk) * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const float* W = G.online + G.slot_off(rslot(A.mask, head), head) + L.wOff;
  const float* Xin = layer_input(G, A, head, L.xOff);
  float* out = G.dzp(head, L.dzIn);
  const int ma = m0 + r, mb = m0 + 16 + r, kk = k0 + r;
  const bool oka = ma < M, okb = mb < M, okk = kk < K;
  // activation outputs the reducing threads will need
  const int s = (threadIdx.x >> 6) & 1, Lx = threadIdx.x & 63, col = k0 + (Lx & 15);
  float xin[4] = {0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 128 && col < K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + 16 * s + (Lx >> 4) * 4 + i;
      if (row < M) xin[i] = Xin[(size_t)row * K + col];
    }
  }
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (TDG) {
    // N = A*d <= 128: at most one 64-wide chunk per wave; its W slice is fetched before K2
    __shared__ TdgSmem sm;
    if (tile == 0 && A.inc_step && threadIdx.x == 0 && !step_cancelled(G.cancel)) {  // no dW reads them in this launch
      const int st = G.step[head] + 1;
      const AdamC ac = adam_consts(A.hp, st);
      if constexpr (C) {  // read by this launch's dW tiles
        __hip_atomic_store(G.step + head, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float* f = reinterpret_cast<float*>(G.adamc + head);
        stc<true>(f, ac.omb1);
        stc<true>(f + 1, ac.b2);
        stc<true>(f + 2, ac.omb2);
        stc<true>(f + 3, ac.eps);
        stc<true>(f + 4, ac.wd);
        stc<true>(f + 5, ac.bc2s);
        stc<true>(f + 6, ac.nss);
      } else {
        G.step[head] = st;
        G.adamc[head] = ac;
      }
    }
    if (A.flag && tile == 0 && head == A.head0 && threadIdx.x == 0) *A.flag = A.flag_value;
    // the 16 k-steps of each 64-wide chunk are split over the waves (4 or 8 steps each); the
    // partial sums meet in the reduction below
    const int wpc = N > 64 ? 2 : 4, jw = 16 / wpc, j0 = (wave % wpc) * jw;
    const int nb = (wave / wpc) * 64 + g * 16;
    float bw[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      bw[j] = (j >= j0 && j < j0 + jw && okk && nb + j < N) ? W[(size_t)(nb + j) * K + kk] : 0.f;
    if (tdg_rows<VMAX, U, C>(G, A, head, m0, tile % ntk == 0, sm)) return;  // repeats round r-1 (block-uniform)
    const float* da = sm.dz + (size_t)r * N + nb;
    const float* db = sm.dz + (size_t)(16 + r) * N + nb;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j >= j0 && j < j0 + jw) {
        const bool okj = nb + j < N;
        acc0 = mfma4(oka && okj ? da[j] : 0.f, bw[j], acc0);
        acc1 = mfma4(okb && okj ? db[j] : 0.f, bw[j], acc1);
      }
    }
  } else {
    const float* dZ = G.dzp(head, L.dzOff);
    const bool vec = (N & 63) == 0;
    for (int nc = nbeg + wave * 64; nc < nend; nc += 256) {
      const int nb = nc + g * 16;
      float a0[16], a1[16], bw[16];
      load16u<C>(a0, dZ + (size_t)ma * N, nb, nend, oka, vec);
      load16u<C>(a1, dZ + (size_t)mb * N, nb, nend, okb, vec);
      if constexpr (BF) {
        // the reduction index n = nb + 8s + j as element j of bf16 step s (a permutation of the
        // fp32 path's k-steps); W from the bf16 copy of the read slot
        const __bf16* W16 = G.on16 + G.slot_off(rslot(A.mask, head), head) + L.wOff;
        bf16x8 w16[2];
#pragma unroll
        for (int j = 0; j < 16; ++j)
          w16[j >> 3][j & 7] = (okk && nb + j < nend) ? W16[(size_t)(nb + j) * K + kk] : (__bf16)0.f;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          acc0 = mfma_bf16(to_bf16x8(a0 + 8 * s2), w16[s2], acc0);
          acc1 = mfma_bf16(to_bf16x8(a1 + 8 * s2), w16[s2], acc1);
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) bw[j] = (okk && nb + j < nend) ? W[(size_t)(nb + j) * K + kk] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        acc0 = mfma4(a0[j], bw[j], acc0);
        acc1 = mfma4(a1[j], bw[j], acc1);
      }
    }
  }
  PROBE_MARK();
  red[wave][0][lane] = acc0;
  red[wave][1][lane] = acc1;
  __syncthreads();
  if (!TDG && A.dxs > 1) {  // partial tile -> dxpart; the last of the dxs splits finishes it
    const int ntile = ((M + 31) >> 5) * ntk;
    const size_t pt = ((size_t)(head - A.head0) * ntile + tile) * A.dxs;
    __shared__ int s_last;
    if (threadIdx.x < 128) {
      floatx4 v = red[0][s][Lx];
      v += red[1][s][Lx];
      v += red[2][s][Lx];
      v += red[3][s][Lx];
      float* o = A.dxpart + ((pt + split) * 128 + threadIdx.x) * 4;
#ifdef SFX_CHECK
      SFX_CHK((long long)((pt + split) * 128 + threadIdx.x) * 4 + 3 < G.ext_dxpart, pt, split, G.ext_dxpart);
#endif
#pragma unroll
      for (int i = 0; i < 4; ++i) stc<true>(o + i, v[i]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned* ctr = A.dxctr + (size_t)(head - A.head0) * ntile + tile;
      const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == (unsigned)A.dxs - 1;
      if (s_last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last || threadIdx.x >= 128) return;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < A.dxs; ++q) {
      const float* o = A.dxpart + ((pt + q) * 128 + threadIdx.x) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __fadd_rn(v[i], ldc<true>(o + i));
    }
    if (col < K) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * s + (Lx >> 4) * 4 + i;
        if (row < M) {
          G.chk_act(L.dzIn, (long long)row * K + col);
          stc<C>(out + (size_t)row * K + col, act_bwd(v[i], xin[i], L.actIn));
        }
      }
    }
    return;
  }
  if (threadIdx.x < 128) {
    floatx4 v = red[0][s][Lx];
    v += red[1][s][Lx];
    v += red[2][s][Lx];
    v += red[3][s][Lx];
    if (col < K) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * s + (Lx >> 4) * 4 + i;
        if (row < M) {
          G.chk_act(L.dzIn, (long long)row * K + col);
          stc<C>(out + (size_t)row * K + col, act_bwd(v[i], xin[i], L.actIn));
        }
      }
    }
  }
}

// post-update forward of layer 0 for the 32 output rows this tile just optimised
// (input rows staged in LDS by role_dw: sX[m * K + k], m < vM); with look-ahead rows also
// (sX[aoff + m * K + k], m < 2 aM) those rows into R_NS / R_NS1 and, with the target weights sWt,
// NS1 into R_NS1T.  vrows = false: the look-ahead rows only (a skipped head).
__device__ __forceinline__ int v0_aoff(const BwdArgs& A, int K) { return (A.vM * K + 3) & ~3; }
constexpr int V0S = KFUSE + 4;  // LDS row stride of the tile's weights: lane (r, g) hits bank 4r + g

// One 16-row x 16-column MFMA tile of the fused layer-0 forward: rows [m0, m0 + 16) of x (row
// stride K, `rows` valid) times this lane's weight row w (K floats), bias bb, into Y (row stride
// N).  Every LDS operand is read before the first MFMA (K <= KFUSE: at most 16 k-steps), in the
// k-ordered accumulation of k_fwd's layer-0 path.
template <bool C>
__device__ __forceinline__ void v0_tile(const float* x, int K, int m0, int rows, const float* w, float bb, int act,
                                        float* Y, int N, int n, long long lim) {
  constexpr int KS = 8;  // k-steps whose operands are read together (K <= 32: one batch)
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4, ma = m0 + r;
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 4 * KS) {
    float a[KS], b[KS];
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      const int k = k0 + 4 * q + g;
      a[q] = (k < K && ma < rows) ? x[ma * K + k] : 0.f;
      b[q] = k < K ? w[k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < KS; ++q)
      if (k0 + 4 * q < K) c = mfma4(a[q], b[q], c);
  }
  if (n < N) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + g * 4 + i;
      if (m < rows) {
        SFX_CHK((long long)m * N + n < lim, m, n, lim);
        stc<C>(Y + (size_t)m * N + n, act_fwd(__fadd_rn(c[i], bb), act));
      }
    }
  }
}

template <bool C>
__device__ __forceinline__ void fused_v0(const Geo& G, const BwdArgs& A, const RoleGeo& L, int head, int nbase, const float* sW,
                         const float* sB, const float* sX, const float* sWt = nullptr, const float* sBt = nullptr,
                         bool vrows = true, bool landed = false) {
  // the look-ahead LDS-DMA has landed (role_dw waits for it before its Adam stores: landed)
  if (A.aM > 0 && !landed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  PROBE_AT(3);
  const int K = L.K, N = L.N, VM = A.vM;
  // wave w owns column half (w & 1) and row tiles (w >> 1), (w >> 1) + 2, ...
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15;
  const int nl = (wave & 1) * 16 + r, n = nbase + nl;
  const float bias = sB[nl];
  if (vrows) {
    float* Y = G.actp(A.vRole, head, A.vOff);
    for (int mt = wave >> 1; mt * 16 < VM; mt += 2)
      v0_tile<C>(sX, K, mt * 16, VM, sW + nl * V0S, bias, A.act0, Y, N, n, G.actSize - A.vOff);
  }
  PROBE_AT(4);
  if (A.aM > 0) {
    // 16-row tiles of three products: NS -> R_NS and NS1 -> R_NS1 with the post-update weights,
    // NS1 -> R_NS1T with the target weights (row stride K in sWt)
    const int aM = A.aM, nt = (aM + 15) >> 4;
    const float* xa = sX + v0_aoff(A, K);
    const float bt = sBt[nl];
    for (int it = wave >> 1; it < 3 * nt; it += 2) {
      const int which = it / nt, mt = it - which * nt;
      v0_tile<C>(xa + (which ? aM * K : 0), K, mt * 16, aM, which == 2 ? sWt + nl * K : sW + nl * V0S,
                 which == 2 ? bt : bias, A.act0, G.actp(which == 0 ? R_NS : which == 1 ? R_NS1 : R_NS1T, head, A.vOff),
                 N, n, G.actSize - A.vOff);
    }
  }
  PROBE_AT(5);
}

typedef __attribute__((address_space(3))) void* tsf_lds_t;

// LDS-DMA staging: dst[j] = *src(j) for j < n (global_load_lds_dword; wave-uniform LDS base +
// lane * 4, per-lane global address, no VGPR destination), by waves [w0, w0 + nw) of the
// workgroup; src(j) == nullptr marks a padding word, zeroed by a plain LDS store instead.
// Nothing waits here: the loads of every staging call stay in flight together until the
// caller's next __syncthreads().
template <class F>
__device__ __forceinline__ void glds(float* dst, int n, F src, int w0 = 0, int nw = 4) {
  const int lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) - w0;
  if (wv < 0 || wv >= nw) return;
  for (int c = wv; c * 64 < n; c += nw) {
    const int j = c * 64 + lane;
    const float* p = j < n ? src(j) : nullptr;
    if (p)
      __builtin_amdgcn_global_load_lds((const void*)p, (tsf_lds_t)(dst + c * 64), 4, 0, 0);
    else if (j < n)
      dst[j] = 0.f;
  }
}

// LDS of the fused post-update layer-0 forward, one instance per kernel for both of its callers
// (role_dw's layer-0 tiles and role_v0_only): the tile's weights and biases, the input rows, the
// target weights and biases of the look-ahead rows.
struct V0Smem {
  float sW[32 * V0S];
  float sB[32];
  float sWt[32 * KFUSE];
  float sBt[32];
  __align__(16) float sX[VFUSE];
};
__device__ __forceinline__ V0Smem& v0_smem() {
  __shared__ V0Smem sm;
  return sm;
}

// The look-ahead operands by LDS-DMA (no registers; they land while the tile does its dW): the
// 2 aM input rows (BwdArgs::ax) at sX + v0_aoff, the target weights of columns [nbase, nbase + 32)
// (32 contiguous rows of K floats; row stride K in sWt) and their biases.  Landed at fused_v0.
__device__ __forceinline__ void v0_stage_ahead(const Geo& G, const BwdArgs& A, const RoleGeo& L, int head, int nbase,
                                               V0Smem& sm) {
  const int K = L.K, ncol = L.N - nbase < 32 ? L.N - nbase : 32;
  const float* ax = A.ax;
  glds(sm.sX + v0_aoff(A, K), 2 * A.aM * K, [&](int j) -> const float* { return ax + j; });
  const float* Pt = G.target + (long long)head * G.P;
  const float* tw = Pt + L.wOff + (size_t)nbase * K;
  glds(sm.sWt, 32 * K, [&](int j) -> const float* { return j < ncol * K ? tw + j : nullptr; });
  const float* tb = Pt + L.bOff + nbase;
  glds(sm.sBt, 32, [&](int j) -> const float* { return j < ncol ? tb + j : nullptr; }, 0, 1);
}

// A layer-0 dW tile of a policy that repeats the previous round (BwdArgs::skip): no gradient,
// no Adam -- the write slot already holds this round's weights -- only the fused post-update
// forward of its 32 columns, from those weights (the bits role_dw would have staged): every row
// (vrows), or the look-ahead rows alone (BwdArgs::a_noskip).
// Fused layers have K <= KFUSE <= 64: one k-tile, so tile = column tile.
__device__ __forceinline__ void role_v0_only(const Geo& G, const BwdArgs& A, int head, const RoleGeo& L, int tile, bool vrows) {
  const int N = L.N, K = L.K, M = A.M, tid = threadIdx.x, nbase = tile * 32;
  const float* Pw = G.online + G.slot_off(rslot(A.mask, head) ^ 1, head);
  V0Smem& sm = v0_smem();
  float* sW = sm.sW;
  float* sB = sm.sB;
  float* sX = sm.sX;
  if (A.aM > 0) v0_stage_ahead(G, A, L, head, nbase, sm);
  const FDiv fK = fdiv(K);
  for (int j = tid; j < 32 * K; j += 256) {
    const int nl = j / fK, k = j - nl * K;
    sW[nl * V0S + k] = nbase + nl < N ? Pw[L.wOff + (size_t)(nbase + nl) * K + k] : 0.f;
  }
  if (tid < 32) sB[tid] = nbase + tid < N ? Pw[L.bOff + nbase + tid] : 0.f;
  if (vrows) {
    const int nxs = A.vM * K;
    for (int j = tid; j < nxs; j += 256) sX[j] = j < M * K ? A.v_x[j] : A.v_xn[j - M * K];
  }
  fused_v0<false>(G, A, L, head, nbase, sW, sB, sX, sm.sWt, sm.sBt, vrows);
}

template <bool C = false, bool BF = false>
__device__ __forceinline__ void role_dw(const Geo& G, const BwdArgs& A, int head, const RoleGeo& L, int tile, bool fuse) {
  const int N = L.N, K = L.K, M = A.M;
  const int ntk = (K + 63) >> 6;
  const int kt = tile % ntk, nt = tile / ntk;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int nbase = nt * 32, n0 = nbase + (wave & 1) * 16, k0 = kt * 64 + (wave >> 1) * 32;
  const float* dZ = G.dzp(head, L.dzOff);
  const float* X = layer_input(G, A, head, L.xOff);
  const int rs = rslot(A.mask, head);
  const long long ro = G.slot_off(rs, head), wo = G.slot_off(rs ^ 1, head);
  const float* Pr = G.online + ro;
  const float* Mr = G.am + ro;
  const float* Vr = G.av + ro;
  float* Pw = G.online + wo;
  float* Mw = G.am + wo;
  float* Vw = G.av + wo;
  const AdamC c = load_adamc<C>(G.adamc + head);  // bias corrections of this step (double pow once per head)
  const int cx = step_cancelled(G.cancel);
  const int nn = n0 + r, kb0 = k0 + r, kb1 = k0 + 16 + r;
  // prefetch the optimizer state of the 8 weights this lane will update
  float pp[8], pm[8], pv[8];
  bool ok[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + g * 4 + i;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = h ? kb1 : kb0;
      const int e = i * 2 + h;
      ok[e] = n < N && k < K;
      const size_t off = (size_t)L.wOff + (size_t)n * K + k;
      pp[e] = ok[e] ? Pr[off] : 0.f;
      pm[e] = ok[e] ? Mr[off] : 0.f;
      pv[e] = ok[e] ? Vr[off] : 0.f;
    }
  }
  // bias of column n0 + r: lane r of waves 0/1 (k-half 0) of the kt == 0 tiles.  Its gradient
  // Σ_m dZ[m][n] comes from the dZ operands already in registers (no extra loads: a lane
  // stays under the 63 outstanding loads the vmcnt counter tracks).
  const bool dob = kt == 0 && wave < 2 && g == 0 && nn < N;
  const int nbias = nn;
  float bp = 0.f, bm = 0.f, bv = 0.f;
  if (dob) {
    bp = Pr[L.bOff + nbias];
    bm = Mr[L.bOff + nbias];
    bv = Vr[L.bOff + nbias];
  }
  // fused forward input (S1 rows ++ s_next), requested with the rest, parked in LDS below: the S1
  // rows as float4 (4 loads per lane, not 16: with the Adam state and the MFMA operands a lane
  // stays under the 63 loads vmcnt tracks), the s_next row one float per lane
  constexpr int XQ = VFUSE / 1024;
  float4 xs[XQ];
  float xn = 0.f;
  const int nx = fuse ? M * K : 0;
  const int nxn = fuse && A.v_xn ? K : 0;
  if (fuse && A.aM > 0) v0_stage_ahead(G, A, L, head, nbase, v0_smem());
  if (fuse) {
    if ((nx & 3) == 0 && (reinterpret_cast<uintptr_t>(A.v_x) & 15) == 0) {
#pragma unroll
      for (int q = 0; q < XQ; ++q) {
        const int j = threadIdx.x + 256 * q;
        xs[q] = 4 * j < nx ? reinterpret_cast<const float4*>(A.v_x)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {  // rows not whole float4s: the same layout from dword loads
#pragma unroll
      for (int q = 0; q < XQ; ++q) {
        const int j = 4 * (threadIdx.x + 256 * q);
        xs[q].x = j < nx ? A.v_x[j] : 0.f;
        xs[q].y = j + 1 < nx ? A.v_x[j + 1] : 0.f;
        xs[q].z = j + 2 < nx ? A.v_x[j + 2] : 0.f;
        xs[q].w = j + 3 < nx ? A.v_x[j + 3] : 0.f;
      }
    }
    if ((int)threadIdx.x < nxn) xn = A.v_xn[threadIdx.x];
  }
  __builtin_amdgcn_sched_barrier(0);  // keep those loads ahead of the MFMA operands
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  for (int mc = 0; mc < M; mc += MT) {
    float av[MT / 4], bv0[MT / 4], bv1[MT / 4];
#pragma unroll
    for (int j = 0; j < MT / 4; ++j) {
      const int m = mc + 4 * j + g;
      const bool okm = m < M;
      av[j] = (okm && nn < N) ? ldc<C>(dZ + (size_t)m * N + nn) : 0.f;
      bv0[j] = (okm && kb0 < K) ? X[(size_t)m * K + kb0] : 0.f;
      bv1[j] = (okm && kb1 < K) ? X[(size_t)m * K + kb1] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < MT / 4; ++j) {
      acc0 = mfma4(av[j], bv0[j], acc0);
      acc1 = mfma4(av[j], bv1[j], acc1);
    }
#pragma unroll
    for (int j = 0; j < MT / 4; ++j) bsum = __fadd_rn(bsum, av[j]);  // rows mc + 4j + g
  }
  // + the other three row classes (lanes r + 16, r + 32, r + 48), fixed order
  bsum = __fadd_rn(bsum, __shfl_xor(bsum, 16));
  bsum = __fadd_rn(bsum, __shfl_xor(bsum, 32));
  // the look-ahead LDS-DMA (issued first) waited for here, before the Adam stores are issued: a
  // wait after them (in fused_v0) would also wait for every store to drain
  if (fuse && A.aM > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PROBE_MARK();
  V0Smem& sm = v0_smem();
  float* sW = sm.sW;
  float* sB = sm.sB;
  float* sX = sm.sX;
  if (fuse) {
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int j = threadIdx.x + 256 * q;
      if (4 * j + 3 < nx) {
        reinterpret_cast<float4*>(sX)[j] = xs[q];
      } else if (4 * j < nx) {  // the last, partial float4
        sX[4 * j] = xs[q].x;
        if (4 * j + 1 < nx) sX[4 * j + 1] = xs[q].y;
        if (4 * j + 2 < nx) sX[4 * j + 2] = xs[q].z;
      }
    }
    if ((int)threadIdx.x < nxn) sX[nx + threadIdx.x] = xn;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + g * 4 + i;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = i * 2 + h;
      if (ok[e]) {
        const int k = h ? kb1 : kb0;
        const size_t off = (size_t)L.wOff + (size_t)n * K + k;
        SFX_CHK((long long)off < G.P, L.wOff, n, k);
        adam_apply(pp[e], pm[e], pv[e], h ? acc1[i] : acc0[i], c);
        if (!cx) {
          st_param<C>(Pw + off, pp[e]);
          st_moment(Mw + off, pm[e]);
          st_moment(Vw + off, pv[e]);
          // the bf16 copy of the write slot (2-byte stores: an LDS transpose into 16-byte row stores
          // measured slower -- its barrier costs more than the stores, profiles/r06_probe_bf16_lds.txt)
          if constexpr (BF) G.on16[wo + off] = (__bf16)pp[e];
        }
        if (fuse) sW[(n - nbase) * V0S + k] = pp[e];
      }
    }
  }
  if (dob) {
    adam_apply(bp, bm, bv, bsum, c);
    if (!cx) {
      st_param<C>(Pw + L.bOff + nbias, bp);
      st_moment(Mw + L.bOff + nbias, bm);
      st_moment(Vw + L.bOff + nbias, bv);
      if constexpr (BF) G.on16[wo + L.bOff + nbias] = (__bf16)bp;
    }
    if (fuse) sB[nbias - nbase] = bp;
  }
  if (fuse) fused_v0<C>(G, A, L, head, nbase, sW, sB, sX, sm.sWt, sm.sBt, true, true);
}

// loss finalisation, optional w step, Adam step counter (one workgroup per head)
// Deterministic block sum (fixed pairwise tree over 256 partials) -- result in every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int s = 128; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = __fadd_rn(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// loss finalisation, optional w step, Adam step counter (one workgroup per head).  The host
// drops the tail when it has nothing to do (no losses requested, no w step, step bumped in
// the fused TD launch).
__device__ __forceinline__ void role_tail(const Geo& G, const BwdArgs& A, int head) {
  const int M = A.M, d = G.d, tid = threadIdx.x;
  __shared__ float s_e[MMAX];
  __shared__ float s_red[256];
  __shared__ float s_phi[2048];
  const int step = A.step_in_tail && A.inc_step ? G.step[head] + 1 : G.step[head];
  const int cx = step_cancelled(G.cancel);
  const float* rl = G.rowloss + (long long)head * MMAX;
  float* w = G.w + (long long)head * G.dpad;
  float part = 0.f;  // this thread's rows of Σ_b rowloss (b = tid, tid + 256, ...)
  for (int b = tid; b < M; b += 256) part = __fadd_rn(part, rl[b]);
  float l2 = 0.f;
  if (A.train_w) {
    // r_fit = w·φ_b ; e_b = r_fit - r_b ; dw = Σ_b (2/M) e_b φ_b   (sfdqn.py:340-342)
    const bool lds_phi = M * d <= 2048;
    if (lds_phi)
      for (int j = tid; j < M * d; j += 256) s_phi[j] = A.phi[j];
    __syncthreads();
    const float* ph = lds_phi ? s_phi : A.phi;
    float se = 0.f;
    for (int b = tid; b < M; b += 256) {
      float rf = 0.f;
      for (int k = 0; k < d; ++k) rf = __builtin_fmaf(w[k], ph[(size_t)b * d + k], rf);
      s_e[b] = __fsub_rn(rf, A.r[b]);
      se = __builtin_fmaf(s_e[b], s_e[b], se);
    }
    se = block_sum(se, s_red);  // also orders s_e for the readers below
    const AdamC c = adam_consts(A.hpw, step);
    const float nrm = (float)(2.0 / (double)M);
    float gw = 0.f;
    if (tid < d) {
      for (int b = 0; b < M; ++b) gw = __builtin_fmaf(__fmul_rn(nrm, s_e[b]), ph[(size_t)b * d + tid], gw);
    }
    __syncthreads();
    if (tid < d && !cx) adam_el(w + tid, G.wm + (long long)head * G.dpad + tid, G.wv + (long long)head * G.dpad + tid, gw, c);
    l2 = (float)((double)se / (double)M);
  }
  const float s = A.losses ? block_sum(part, s_red) : 0.f;
  if (tid == 0) {
    const float l1 = (float)((double)s / ((double)M * (double)G.O));
    if (A.losses) {
      float* lo = A.losses + 3 * (head - A.head0);
      lo[0] = __fadd_rn(l1, l2);
      lo[1] = l1;
      lo[2] = l2;
    }
    if (A.step_in_tail && !cx) {
      G.step[head] = step;
      G.adamc[head] = adam_consts(A.hp, step);
    }
  }
}

// tile bx of head `head` of a backward launch (k_bwd; k_bwd_tsf after its TSF blocks)
template <bool BF>
__device__ __forceinline__ void bwd_body(const Geo& G, const BwdArgs& A, int head, int bx, floatx4 (*red)[2][64]) {
  PROBE_T(pt0);
  PROBE_MARKA();
  const bool skip = A.skip && __builtin_nontemporal_load(A.skip + head) != 0;  // repeats round r-1
  // tiles of a head in dispatch order, longest first so they request their operands before the
  // bulk of the launch does: layer-0 dW (+ the fused post-update forward), dW, dX, tail
  if (bx < A.nc) {
    if (skip) {
      if (A.fuse_v0 && (!A.skip_v0 || (A.aM > 0 && A.a_noskip))) role_v0_only(G, A, head, A.rc, bx, !A.skip_v0);
      return;
    }
    role_dw<false, BF>(G, A, head, A.rc, bx, A.fuse_v0 != 0);
    PROBE_REC(6, pt0);
    return;
  }
  bx -= A.nc;
  if (bx < A.nb) {
    if (skip) return;
    role_dw<false, BF>(G, A, head, A.rb, bx, false);
    PROBE_REC(5, pt0);
    return;
  }
  bx -= A.nb;
  if (bx < A.na) {
    if (skip) return;
    role_dx<false, 2, 8, false, BF>(G, A, head, bx, red);
    PROBE_REC(4, pt0);
    return;
  }
  role_tail(G, A, head);
}

template <bool BF = false>
__global__ __launch_bounds__(256) void k_bwd(Geo G, BwdArgs A) {
  __shared__ floatx4 red[4][2][64];
  int head = A.head0 + blockIdx.y, bx = blockIdx.x;
  if (A.xcd) {
    if (!xcd_decode(blockIdx.x, A.nhead, A.na + A.nb + A.nc + A.tail, head, bx)) return;
    head += A.head0;
  }
  bwd_body<BF>(G, A, head, bx, red);
}

// First backward launch with K2 fused: dX of the last layer only (A.na tiles per head).
template <int VMAX, int U>
__global__ __launch_bounds__(256) void k_bwd_tdg(Geo G, BwdArgs A) {
  __shared__ floatx4 red[4][2][64];
  PROBE_T(pt0);
  if (A.xi_dst)
    fill_sortable(A.xi_dst, A.xi_src, A.xi_copy, A.xi_n, (blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x,
                  gridDim.x * gridDim.y * 256);
  int head = A.head0 + blockIdx.y, bx = blockIdx.x;
  if (A.xcd) {
    if (!xcd_decode(blockIdx.x, A.nhead, A.na, head, bx)) return;
    head += A.head0;
  }
  PROBE_MARKA();
  role_dx<true, VMAX, U>(G, A, head, bx, red);
  PROBE_REC(3, pt0);
}

// -------------------------------------------------------------------------------------
// K4  GPI reduction over heads (SF.GPI_w, features/successor.py:243-246;
// sfdqn.py:235-240) and action selection (sfdqn.py:585-594).  One workgroup per row.
//   task = argmax_t max_a q ; next = argmax_a max_t q ; sel = (c, argmax_a q[c])
// -------------------------------------------------------------------------------------
struct GpiArgs {
  int M, role, row0, select_task, use_gpi, rowoff;  // rowoff: first row of the role block used
  int w_stride, sel_stride;  // > 0: row b's w at w + b*w_stride, its (c, a) at sel_out + b*sel_stride
  const float* w;
  float* psi_out;   // [B, T, A, d] or null  (row b -> row0 + b)
  float* q_out;     // [B, T, A] or null
  int64_t* task_out;
  int64_t* next_out;
  int64_t* sel_out;  // [2] or null
  // sfx_update_all_select: q_out / task_out read at run time from host-coherent words (written by
  // the host before each launch), so a captured step serves fresh output tensors every time
  const unsigned long long* out_ind;
};

// argmax helpers: (value, index) packed so that an integer max picks the largest value and,
// among equal values, the smallest index (torch.argmax's first-index rule); -0 == +0.
__device__ __forceinline__ unsigned long long argmax_key(float v, int idx) {
  const unsigned int u = __float_as_uint(__fadd_rn(v, 0.f));
  const unsigned int o = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)o << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)idx);
}
__device__ __forceinline__ int argmax_idx(unsigned long long key) { return (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull)); }
__device__ __forceinline__ unsigned long long wave_max(unsigned long long k) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const unsigned long long o = __shfl_xor(k, m, 64);
    k = o > k ? o : k;
  }
  return k;
}

// The argmaxes of one row's q = ψ·w (s_q[t * A + a], in LDS, complete): head maxima and action
// maxima by the nthr threads of the workgroup, then the first-index argmaxes by wave 0.  Returns
// (in wave 0) the selection (c, a) packed as c * A + a, or -1 without a selection output.
__device__ __forceinline__ int gpi_pick(const GpiArgs& A, const float* s_q, float* s_mt, float* s_ma, int T, int Aa,
                                        long long ob, int64_t* so, int nthr) {
  const int tid = threadIdx.x;
  for (int t = tid; t < T; t += nthr) {  // max over actions per head (torch.max(q, axis=2))
    float mx = s_q[t * Aa];
    for (int a = 1; a < Aa; ++a) mx = fmaxf(mx, s_q[t * Aa + a]);
    s_mt[t] = mx;
  }
  for (int a = tid; a < Aa; a += nthr) {  // max over heads per action (torch.max(q1, axis=1))
    float mx = s_q[a];
    for (int t = 1; t < T; ++t) mx = fmaxf(mx, s_q[t * Aa + a]);
    s_ma[a] = mx;
  }
  __syncthreads();
  int picked = -1;
  if (tid < 64) {  // first-index argmaxes by one wave
    unsigned long long kt = 0ull, ka = 0ull;
    for (int t = tid; t < T; t += 64) {
      const unsigned long long k = argmax_key(s_mt[t], t);
      kt = k > kt ? k : kt;
    }
    for (int a = tid; a < Aa; a += 64) {
      const unsigned long long k = argmax_key(s_ma[a], a);
      ka = k > ka ? k : ka;
    }
    const int tb = argmax_idx(wave_max(kt)), ab = argmax_idx(wave_max(ka));
    const int c = A.use_gpi ? tb : A.select_task;
    unsigned long long kc = 0ull;
    if (so)
      for (int a = tid; a < Aa; a += 64) {
        const unsigned long long k = argmax_key(s_q[c * Aa + a], a);
        kc = k > kc ? k : kc;
      }
    const int act = so ? argmax_idx(wave_max(kc)) : 0;
    if (so) picked = c * Aa + act;
    if (tid == 0) {
      if (A.task_out) A.task_out[ob] = tb;
      if (A.next_out) A.next_out[ob] = ab;
      if (so) {  // sc1 stores: k_ver's last workgroup may publish them in this launch
        __hip_atomic_store(so, (int64_t)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(so + 1, (int64_t)act, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  return picked;
}

__device__ void gpi_row(const Geo& G, const GpiArgs& A0, int b) {
  GpiArgs A = A0;
  if (A.out_ind) {  // issued first: the round trip to host memory overlaps the dot products
    A.q_out = reinterpret_cast<float*>(A.out_ind[0]);
    A.task_out = reinterpret_cast<int64_t*>(A.out_ind[1]);
  }
  const int tid = threadIdx.x;
  const int T = G.T, Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff, TA = T * Aa;
  __shared__ float s_q[QMAX];
  __shared__ float s_w[DMAX];
  __shared__ float s_mt[256], s_ma[256];
  const long long ob = (long long)(A.row0 + b);
  const int lb = A.rowoff + b;
  const FDiv fA = fdiv(Aa);
  const float* wr = A.w + ob * A.w_stride;
  int64_t* so = A.sel_out ? A.sel_out + ob * A.sel_stride : nullptr;
  if (A.psi_out) {
    const FDiv fO = fdiv(O);
    for (int idx = tid; idx < T * O; idx += 256) {
      const int t = idx / fO, o = idx - t * O;
      A.psi_out[(ob * T + t) * O + o] = G.actp(A.role, t, NLm)[(size_t)lb * O + o];
    }
  }
  if (TA <= 256 && (d & 3) == 0 && d <= 16 && ((uintptr_t)wr & 15) == 0) {  // one dot per thread, ψ and w requested together
    const int V4 = d >> 2, t = tid / fA, a = tid - t * Aa;
    const bool act = tid < TA;
    const float4* p4 = reinterpret_cast<const float4*>(G.actp(A.role, act ? t : 0, NLm) + (size_t)lb * O + (act ? a * d : 0));
    const float4* w4 = reinterpret_cast<const float4*>(wr);
    float4 pv[4], wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pv[j] = (act && j < V4) ? p4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      wv[j] = j < V4 ? w4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < V4) {
        q = __builtin_fmaf(pv[j].x, wv[j].x, q);
        q = __builtin_fmaf(pv[j].y, wv[j].y, q);
        q = __builtin_fmaf(pv[j].z, wv[j].z, q);
        q = __builtin_fmaf(pv[j].w, wv[j].w, q);
      }
    }
    if (act) {
      s_q[tid] = q;
      if (A.q_out) A.q_out[(ob * T + t) * Aa + a] = q;
    }
  } else {
    for (int k = tid; k < d; k += 256) s_w[k] = wr[k];
    __syncthreads();
    for (int idx = tid; idx < TA; idx += 256) {
      const int t = idx / fA, a = idx - t * Aa;
      const float* p = G.actp(A.role, t, NLm) + (size_t)lb * O + a * d;
      float q = 0.f;
#pragma unroll 8
      for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
      s_q[idx] = q;
      if (A.q_out) A.q_out[(ob * T + t) * Aa + a] = q;
    }
  }
  __syncthreads();
  gpi_pick(A, s_q, s_mt, s_ma, T, Aa, ob, so, 256);
}
__global__ __launch_bounds__(256) void k_gpi(Geo G, GpiArgs A) {
  PROBE_T(pt0);
  gpi_row(G, A, blockIdx.x);
  PROBE_REC(16, pt0);
}

// -------------------------------------------------------------------------------------
// K5  Verification of a speculative round of the all-task update + action selection.
// Block i in [1, T): recompute policy i's next actions with heads t < i AFTER this round's
// update (role `post`) and heads t >= i before it (R_S1) -- what policy i sees in the
// reference's in-order loop (agents/sfdqn.py:59-60) -- and compare with the actions the
// round used.  Mismatch: atomicMin(flag, i).  Heads below the flag are exact (induction
// from policy 0, which only sees pre-step heads); the next round re-derives every
// policy's actions from this round's post-update values and fixes at least one more head.
// Block npol (when sel): GPI action for s_next (row M of `post`) with w[select_task].
// -------------------------------------------------------------------------------------
struct HostResult {  // host-coherent; seq written last
  long long sel0, sel1;
  int flag, err;       // err (slot 0 only): a gate timed out (set by the gate itself, system scope)
  int cancelled;       // the published step was cancelled at its gate: nothing of it committed
  int nonfinite;       // the handle's non-finite TD flag (Geo::nonfin) when the step published
  long long seq;
};
// Results live in a ring of RES_RING slots, step seq in slot seq % RES_RING: steps queued behind
// the host that get cancelled at their gates (runner gate bound) still publish, and must not
// overwrite the result of the step the host is waiting for (> the runner's pre-launch span).
constexpr int RES_RING = 64;

// Post the step's result (selected action, speculation verdict) to host-coherent memory;
// seq is written last (system release).  The inputs are read with coherent (sc1) loads.
__device__ __forceinline__ void publish_result(const int64_t* sel, const int* flag, HostResult* ring,
                                               const long long* dctr, const int* cancel, const int* nonfin) {
  const long long s0 = __hip_atomic_load(sel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long s1 = __hip_atomic_load(sel + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int cx = __hip_atomic_load(cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long seq = __hip_atomic_load(dctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  HostResult* out = ring + (seq & (RES_RING - 1));
  out->sel0 = s0;
  out->sel1 = s1;
  out->flag = f;
  out->cancelled = cx;
  out->nonfinite = nonfin ? __hip_atomic_load(nonfin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  __threadfence_system();
  __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct VerArgs {
  int M, npol, sel, spec_stride, post, rows;  // rows: minibatch rows per workgroup
  const int64_t* spec_next;  // [T][spec_stride]
  int* flag;
  GpiArgs g;                 // action selection for s_next
  // k_publish folded in (runner steps): every workgroup arrives on `done`; the last one to
  // arrive (told by the value its add returns) publishes.  Null: no publication.
  HostResult* pub;
  const long long* pub_dctr;
  unsigned* done;
  int nblocks, pad_;
  // library steps (sfx_step_all / sfx_update_all*): the last workgroup to arrive copies the
  // selection and the flag to host-coherent memory instead of a copy after the launch.  Null: no.
  int64_t* h_sel;
  int* h_flag;
  int* h_posted;  // set to 1 last: the host waits for it instead of the launch's completion
};

// The step's verdict and selection to host-coherent memory (VerArgs::h_sel / h_flag), read with
// coherent loads after the arrivals, written with system scope; the launch's completion (the
// host waits for it) makes them visible.
__device__ __forceinline__ void post_verdict(const VerArgs& V) {
  const long long s0 = __hip_atomic_load(V.g.sel_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long s1 = __hip_atomic_load(V.g.sel_out + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int f = __hip_atomic_load(V.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(V.h_sel, s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(V.h_sel + 1, s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(V.h_flag, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __hip_atomic_store(V.h_posted, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Grid (npol + 1, ceil(M / rows)): one workgroup per (policy, `rows` minibatch rows), each
// thread one q = ψ·w dot product, so every load is issued before the first reduction.
__device__ void ver_block(const Geo& G, const VerArgs& V) {
  const int i = blockIdx.x, tid = threadIdx.x;
  if (i == V.npol) {
    if (V.sel && blockIdx.y == 0) gpi_row(G, V.g, 0);
    return;
  }
  if (i == 0) return;  // policy 0 sees only pre-update heads: always exact
  const int T = G.T, Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff, TA = T * Aa;
  const FDiv fTA = fdiv(TA), fA = fdiv(Aa);
  const int b0 = blockIdx.y * V.rows;
  const int nb = V.M - b0 < V.rows ? V.M - b0 : V.rows;
  if (nb <= 0) return;
  __shared__ float s_q[QMAX];
  __shared__ float s_m[QMAX];
  __shared__ float s_w[DMAX];
  __shared__ int s_bad;
  PROBE_MARKA();
  const float* wrow = G.w + (long long)i * G.dpad;
  const int n = nb * TA;
  SFX_CHK(!(tid < nb) || b0 + tid < V.spec_stride, i, b0 + tid, V.spec_stride);
  const int spec = tid < nb ? (int)V.spec_next[(size_t)i * V.spec_stride + b0 + tid] : 0;
  if (tid == 0) s_bad = 0;
  if (n <= 256 && (d & 3) == 0 && d <= 16) {
    // one dot per thread; ψ, w and the speculated action all requested before the first wait
    const int V4 = d >> 2;
    const int bl = tid / fTA, rem = tid - bl * TA, t = rem / fA, a = rem - t * Aa;
    const bool act = tid < n;
    const float4* p4 = reinterpret_cast<const float4*>(
        G.actp(t < i ? V.post : R_S1, act ? t : 0, NLm) + (act ? (size_t)(b0 + bl) * O + a * d : 0));
    const float4* w4 = reinterpret_cast<const float4*>(wrow);
    float4 pv[4], wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pv[j] = (act && j < V4) ? p4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      wv[j] = j < V4 ? w4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < V4) {
        q = __builtin_fmaf(pv[j].x, wv[j].x, q);
        q = __builtin_fmaf(pv[j].y, wv[j].y, q);
        q = __builtin_fmaf(pv[j].z, wv[j].z, q);
        q = __builtin_fmaf(pv[j].w, wv[j].w, q);
      }
    }
    if (act) s_q[tid] = q;
  } else {
    for (int k = tid; k < d; k += 256) s_w[k] = wrow[k];
    __syncthreads();
    for (int idx = tid; idx < n; idx += 256) {
      const int bl = idx / fTA, rem = idx - bl * TA, t = rem / fA, a = rem - t * Aa;
      const float* p = G.actp(t < i ? V.post : R_S1, t, NLm) + (size_t)(b0 + bl) * O + a * d;
      float q = 0.f;
#pragma unroll 8
      for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
      s_q[idx] = q;
    }
  }
  PROBE_MARK();
  __syncthreads();
  for (int j = tid; j < nb * Aa; j += 256) {  // max over heads per (row, action)
    const int bl = j / fA, a = j - bl * Aa;
    const float* qb = s_q + bl * TA + a;
    float mx = qb[0];
    for (int t = 1; t < T; ++t) mx = fmaxf(mx, qb[t * Aa]);
    s_m[j] = mx;
  }
  __syncthreads();
  if (tid < nb) {  // first argmax over actions vs the speculated next action
    const float* mb = s_m + tid * Aa;
    int am = 0;
    float best = mb[0];
    for (int a = 1; a < Aa; ++a)
      if (mb[a] > best) {
        best = mb[a];
        am = a;
      }
    if (am != spec) s_bad = 1;
  }
  __syncthreads();
  if (tid == 0 && s_bad) atomicMin(V.flag, i);
}

__global__ __launch_bounds__(256) void k_ver(Geo G, VerArgs V) {
  PROBE_T(pt0);
  ver_block(G, V);
  if (V.pub || V.h_flag) {
    // every wave's stores (the selection, the flag) are ordered before the arrival by the barrier
    // and the arrival's agent-scope release; the last arrival acquires them all before it reads
    // the selection and the flag and publishes (the counter is re-armed by the last arrival and by
    // every runner gate: GateArgs::rearm)
    __syncthreads();
    PROBE_AT(3);
    if (threadIdx.x == 0) {
      const unsigned prev = __hip_atomic_fetch_add(V.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      PROBE_AT(4);
      if (prev == (unsigned)V.nblocks - 1) {
        if (V.pub)
          publish_result(V.g.sel_out, V.flag, V.pub, V.pub_dctr, G.cancel, G.nonfin);
        else
          post_verdict(V);
        PROBE_AT(5);
        __hip_atomic_store(V.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  PROBE_REC(8, pt0);
}

// LMS reward fit (features/successor.py:164-167): w += α (r - Σ φ⊙w) φ
// rv: the reward as a value (sfx_lms_value) when r is null
__global__ void k_lms(float* __restrict__ w, const float* __restrict__ phi, const float* __restrict__ r,
                      float alpha, int d, float rv) {
  __shared__ float s_p[DMAX];
  const int tid = threadIdx.x;
  const float wk = tid < d ? w[tid] : 0.f, pk = tid < d ? phi[tid] : 0.f;
  if (tid < d) s_p[tid] = __fmul_rn(pk, wk);
  __syncthreads();
  __shared__ float s_e;
  if (tid == 0) {
    float rf = 0.f;
    for (int k = 0; k < d; ++k) rf = __fadd_rn(rf, s_p[k]);
    s_e = __fmul_rn(alpha, __fsub_rn(r ? r[0] : rv, rf));
  }
  __syncthreads();
  if (tid < d) w[tid] = __fadd_rn(wk, __fmul_rn(s_e, pk));
}

// SFDQN.update_test_reward_mapper (agents/sfdqn.py:168-184) for E test tasks, one lane per task:
// a fresh SGD(lr, weight_decay=wd) step on the bias-free Linear(d, 1) w_e with the loss
// MSE(w_e(φ_e), r_e) -- y = w·φ, loss = (y - r)², ∂w = 2(y - r) φ (mse_loss_backward: 2/N with
// N = 1), d_p = ∂w + wd·w, w += -lr·d_p (torch/optim/sgd.py single-tensor, no momentum).  The
// loss is the pre-step value, as the reference returns it.  lr / wd are narrowed where ATen
// narrows its Scalar arguments.
__global__ __launch_bounds__(64) void k_sf_test_mapper(int E, int d, const float* __restrict__ phi,
                                                       const float* __restrict__ r, float* __restrict__ W,
                                                       int w_stride, float neg_lr, float wd,
                                                       float* __restrict__ loss) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float* f = phi + (long long)e * d;
  float* w = W + (long long)e * w_stride;
  float y = 0.f;
  for (int k = 0; k < d; ++k) y = __builtin_fmaf(w[k], f[k], y);
  const float diff = __fsub_rn(y, r[e]);
  const float gy = __fmul_rn(2.f, diff);
  for (int k = 0; k < d; ++k) {
    const float wk = w[k];
    const float dp = __fadd_rn(__fmul_rn(gy, f[k]), __fmul_rn(wd, wk));
    w[k] = __builtin_fmaf(neg_lr, dp, wk);
  }
  loss[e] = __fmul_rn(diff, diff);
}

}  // namespace sfx

namespace sfx {

// -------------------------------------------------------------------------------------
// Env-step runner plumbing (sfx_runner_*): the host prepares step j's inputs in pinned,
// host-coherent memory and bumps `go`; the graph of step j -- launched ahead, while step
// j-1 still runs -- opens with k_gate, which waits for go >= seq and copies the inputs into
// device memory, and closes with k_publish, which posts the selected action and the
// speculation verdict back to host memory.  Every spin is bounded by `timeout` ticks of
// the 100 MHz wall clock; on expiry the gate records the failure and lets the launch drain.
// -------------------------------------------------------------------------------------
struct GateArgs {
  const uint4* src;  // host-coherent staging
  uint4* dst;        // device staging
  int n16;           // 16-byte words
  int pad_;
  const long long* go;  // host-coherent: last step whose inputs the host has written
  long long* dctr;      // device: last step a gate opened (this gate opens dctr + 1)
  long long timeout;
  int* err;             // host-coherent
  const int* hcancel;   // written by the host (sfx_runner abort): cancel every step still waiting
  const int* hold;      // written by the host while it runs host rounds of the step before (see below)
  long long hard;       // bound of a held wait (ticks)
  int* cancel;          // device: this step's verdict for its kernels (Geo::cancel)
  int* clr;             // sharded steps: SORT_EMPTY-fill clr[0, nclr) (round 0's maxima buffers)
  int nclr, pad2_;
  // a look-ahead step (its minibatch forward ran in the step before): the step-start work of the
  // forward's block 0 moves here -- the speculation flag reset and the LMS reward fit
  int* flag;
  int flag_value, lms_d;
  float* lms_w;
  const float* lms_phi;  // in the staging the gate copies from
  const float* lms_r;
  float lms_alpha, pad3_;
  unsigned *rearm0, *rearm1;  // arrival counters of the step's folded publications (k_ver, k_sel1m)
};

// Wait for the host's go of this step (bounded); 1 if the step may run, 0 if it is cancelled.
// One thread.  dctr advances either way, so the gates of later steps keep their numbering.
// A cancelled step's launches still run (without committing) and overwrite the handle's
// transient buffers, so no gate may give up while the host runs host rounds of the step before
// on the side stream (they read those buffers).  The host raises `hold` before such rounds and
// then reads err; a gate past its bound writes err and then reads `hold` -- each side flushing
// its write before its read (the host reads the word back through the BAR, the gate reads err
// back across PCIe), so at least one of them sees the other: either the host sees err = 1 and
// drains the cancelled steps before its rounds (runner_abort), or the gate sees hold = 1, takes
// its err back and keeps waiting (up to `hard`).
__device__ __forceinline__ int gate_wait(const GateArgs& g) {
  int ok = 1;
  const long long want = __hip_atomic_load(g.dctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const long long t0 = wall_clock64();
  unsigned it = 0;
  bool held = false;
  while (__hip_atomic_load(g.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if ((++it & 15) == 0 && __hip_atomic_load(g.hcancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
      ok = 0;
      break;
    }
    const long long el = wall_clock64() - t0;
    if (el > g.timeout && (!held || (it & 15) == 0)) {
      __hip_atomic_store(g.err, 1, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
      (void)__hip_atomic_load(g.err, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);  // the store has landed
      if (el > g.hard || !g.hold || !__hip_atomic_load(g.hold, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM)) {
        ok = 0;
        break;
      }
      __hip_atomic_store(g.err, 0, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);  // held: not given up
      held = true;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __hip_atomic_store(g.dctr, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *g.cancel = ok ? 0 : 1;
  // the step's folded publications count their arrivals from zero whatever an earlier launch left
  if (g.rearm0) __hip_atomic_store(g.rearm0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (g.rearm1) __hip_atomic_store(g.rearm1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ok;
}

// Queue-sharing probe (runner setup): k_qwait spins, bounded, on a device word that k_qset --
// launched afterwards on another stream -- sets.  If both streams feed the same hardware queue
// the set only runs after the wait gave up, and `seen` stays 0.
__global__ void k_qwait(const int* word, int* seen, long long timeout) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  int s = 0;
  while (!(s = __hip_atomic_load(word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) && wall_clock64() - t0 < timeout)
    __builtin_amdgcn_s_sleep(8);
  __hip_atomic_store(seen, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_qset(int* word) {
  if (threadIdx.x == 0) __hip_atomic_store(word, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_gate(GateArgs g) {
  __shared__ int ok;
  PROBE_T(pt0);
  if (threadIdx.x == 0) ok = gate_wait(g);
  __syncthreads();
  if (!ok) return;
  // after the wait: until then a step before this one may still be running its host rounds
  if (g.clr) fill_sortable(g.clr, nullptr, 0, g.nclr, threadIdx.x, 256);
  PROBE_MARK();
  for (int i = threadIdx.x; i < g.n16; i += 256) g.dst[i] = g.src[i];
  if (g.flag && threadIdx.x == 0) *g.flag = g.flag_value;
  if (g.lms_w) lms_apply(g.lms_w, g.lms_phi, g.lms_r, g.lms_alpha, g.lms_d, 0);
  PROBE_REC(9, pt0);
}


// -------------------------------------------------------------------------------------
// Device-resident replay (opt-in, sfx_runner_device_replay): the ring
// lives in HBM and the gate of each step appends the step's transition and draws the
// uniform minibatch itself, so the host hands over one transition (≈ 2n_s + d + 8 words)
// instead of the collated batch.  Index b of a step with key k over a ring of `size` rows:
//   x = splitmix64(k + (b + 1)·0x9E3779B97F4A7C15),  idx = ((x >> 32) · size) >> 32
// (replay_index below; the host mirror uses the same function, so the recorded minibatch
// of a step is the one the device gathered).
// -------------------------------------------------------------------------------------
struct ReplayMeta {  // tail of the host staging, written by the host per step
  long long a, slot, size;
  unsigned long long key;
  float r, gamma;
  int have, pad_;
};

__host__ __device__ inline unsigned replay_index(unsigned long long key, int b, long long size) {
  unsigned long long x = key + (unsigned long long)(b + 1) * 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (unsigned)(((x >> 32) * (unsigned long long)size) >> 32);
}

struct ReplayGateArgs {
  GateArgs g;         // src/dst/n16 cover [tail0, bytes) of the staging: s_next, φ1, r1, transition
  int tail0;          // 16-byte word where the host-written tail starts
  int n_s, d, B;
  int off_s, off_s1, off_phi, off_a, off_g, off_rb;  // device minibatch fields (bytes)
  int tr_s, tr_s1, tr_phi, tr_meta;                  // transition fields (bytes, from tail0)
  float *rs, *rs1, *rphi, *rr, *rg;                  // ring [cap][...]
  long long* ra;
};

constexpr int REPLAY_TAIL_MAX = 4096;  // bytes of the staged tail held in LDS

__global__ __launch_bounds__(256) void k_gate_replay(ReplayGateArgs A) {
  __shared__ int ok;
  __shared__ __attribute__((aligned(16))) unsigned char tail[REPLAY_TAIL_MAX];
  const GateArgs& g = A.g;
  PROBE_T(pt0);
  if (threadIdx.x == 0) ok = gate_wait(g);
  __syncthreads();
  if (!ok) return;
  // after the wait: until then a step before this one may still be running its host rounds
  if (g.clr) fill_sortable(g.clr, nullptr, 0, g.nclr, threadIdx.x, 256);
  PROBE_MARK();
  uint4* lt = reinterpret_cast<uint4*>(tail);
  for (int i = threadIdx.x; i < g.n16; i += 256) {
    const uint4 v = g.src[A.tail0 + i];
    lt[i] = v;
    g.dst[A.tail0 + i] = v;
  }
  __syncthreads();
  const ReplayMeta& m = *reinterpret_cast<const ReplayMeta*>(tail + A.tr_meta);
  const float* ts = reinterpret_cast<const float*>(tail + A.tr_s);
  const float* ts1 = reinterpret_cast<const float*>(tail + A.tr_s1);
  const float* tphi = reinterpret_cast<const float*>(tail + A.tr_phi);
  const int n_s = A.n_s, d = A.d;
  const long long slot = m.slot;  // < 0: no transition this step (first action of an episode)
  // append (agents/buffer.py:34-50); the gathers below take row `slot` from LDS, so they do
  // not depend on these stores being visible within this launch
  if (slot >= 0) {
    for (int k = threadIdx.x; k < n_s; k += 256) {
      A.rs[slot * n_s + k] = ts[k];
      A.rs1[slot * n_s + k] = ts1[k];
    }
    for (int k = threadIdx.x; k < d; k += 256) A.rphi[slot * d + k] = tphi[k];
    if (threadIdx.x == 0) {
      A.rr[slot] = m.r;
      A.rg[slot] = m.gamma;
      A.ra[slot] = m.a;
    }
  }
  if (!m.have) {
    PROBE_REC(9, pt0);
    return;
  }
  // uniform minibatch (agents/buffer.py:52-64): row b of every field from ring row idx_b
  unsigned char* dst = reinterpret_cast<unsigned char*>(g.dst);
  float* S = reinterpret_cast<float*>(dst + A.off_s);
  float* S1 = reinterpret_cast<float*>(dst + A.off_s1);
  float* PHI = reinterpret_cast<float*>(dst + A.off_phi);
  const int w = 2 * n_s + d;
  for (int e = threadIdx.x; e < A.B * w; e += 256) {
    const int b = e / w, k = e - b * w;
    const long long i = replay_index(m.key, b, m.size);
    const bool own = i == slot;
    if (k < n_s)
      S[b * n_s + k] = own ? ts[k] : A.rs[i * n_s + k];
    else if (k < 2 * n_s)
      S1[b * n_s + k - n_s] = own ? ts1[k - n_s] : A.rs1[i * n_s + k - n_s];
    else
      PHI[b * d + k - 2 * n_s] = own ? tphi[k - 2 * n_s] : A.rphi[i * d + k - 2 * n_s];
  }
  for (int b = threadIdx.x; b < A.B; b += 256) {
    const long long i = replay_index(m.key, b, m.size);
    const bool own = i == slot;
    reinterpret_cast<long long*>(dst + A.off_a)[b] = own ? m.a : A.ra[i];
    reinterpret_cast<float*>(dst + A.off_g)[b] = own ? m.gamma : A.rg[i];
    reinterpret_cast<float*>(dst + A.off_rb)[b] = own ? m.r : A.rr[i];
  }
  PROBE_REC(9, pt0);
}

__global__ void k_publish(const int64_t* sel, const int* flag, HostResult* out, const long long* dctr,
                          const int* cancel, const int* nonfin) {
  PROBE_T(pt0);
  if (threadIdx.x == 0) publish_result(sel, flag, out, dctr, cancel, nonfin);
  PROBE_REC(18, pt0);
}

// -------------------------------------------------------------------------------------
// K4m  The action for one state (select_body: SFDQN.get_Q_values + the choice, sfdqn.py:577-596)
// over T workgroups, one head each: a row of A dots of d (a few KB per workgroup -- one workgroup
// reading all T·A·d floats, at a memory latency per ~8 KB in flight, took 10-12 µs at Hopper width,
// k_gpi 8-9 µs), the heads combined by the last workgroup to arrive (k_ver's hand-off: each
// workgroup's lane 0 stores its head's (max_a q key, argmax_a) write-through, waits for the store,
// then adds to the arrival counter; the add's return tells the last one, which reads the keys
// write-through, picks, publishes and re-arms the counter).  Per head: q in gpi_row's k order
// (bit-identical); the head maximum as gpi_pick forms it; the task as its first-index argmax over
// heads (argmax_key(max_a q_t, t)); the action as the first-index argmax over a of q[c][a].  The
// runner's publication (k_publish) is folded into the last workgroup.  Launch: grid T, 64·⌈A/64⌉
// threads; selections only (no task_out / next_out).
// -------------------------------------------------------------------------------------
struct SelPub {
  HostResult* res;  // null: no publication
  const long long* dctr;
  const int* flag;
  const int* cancel;
  const int* nonfin;
};
constexpr int SEL1_DC = 64;  // ψ operands per thread requested at once

struct SelScratch {
  unsigned long long key[64];  // per head: argmax_key(max_a q_t, t)
  int act[64];                 // per head: first argmax_a q_t[a]
  unsigned done;               // arrivals (re-armed to 0 by the last)
};

// head t's workgroup of k_sel1m
template <int VW>  // d % VW == 0
__device__ __forceinline__ void sel1m_body(const Geo& G, const GpiArgs& A, const SelPub& P, SelScratch* S, int t) {
  PROBE_T(pt0);
  __shared__ float s_w[DMAX];
  __shared__ float s_q[256];
  const int tid = threadIdx.x;
  const int T = G.T, Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff;
  const long long ob = A.row0;
  const float* wr = A.w + ob * A.w_stride;
  int64_t* so = A.sel_out ? A.sel_out + ob * A.sel_stride : nullptr;
  const bool act = tid < Aa;
  const float* p = G.actp(A.role, t, NLm) + (size_t)A.rowoff * O + (size_t)(act ? tid : 0) * d;
  using vec = typename std::conditional<VW == 4, float4, typename std::conditional<VW == 2, float2, float>::type>::type;
  for (int k = tid; k < d; k += blockDim.x) s_w[k] = wr[k];
  float q = 0.f;
  for (int k0 = 0; k0 < d; k0 += SEL1_DC) {
    vec v[SEL1_DC / VW];
#pragma unroll
    for (int j = 0; j < SEL1_DC / VW; ++j) {
      const int k = k0 + j * VW;
      v[j] = act && k < d ? *reinterpret_cast<const vec*>(p + k) : vec{};
    }
    if (k0 == 0) __syncthreads();  // s_w
#pragma unroll
    for (int j = 0; j < SEL1_DC / VW; ++j) {
      const int k = k0 + j * VW;
      if (k < d) {
        const float* e = reinterpret_cast<const float*>(&v[j]);
#pragma unroll
        for (int u = 0; u < VW; ++u) q = __builtin_fmaf(e[u], s_w[k + u], q);
      }
    }
  }
  if (act) {
    s_q[tid] = q;
    if (A.q_out) A.q_out[(ob * T + t) * Aa + tid] = q;
  }
  __syncthreads();
  if (tid < 64) {
    // head maximum as gpi_pick forms it (sequential fmaxf over a), first-index argmax over a
    float mx = s_q[0];
    for (int a = 1; a < Aa; ++a) mx = fmaxf(mx, s_q[a]);
    unsigned long long ka = 0ull;
    for (int a = tid; a < Aa; a += 64) {
      const unsigned long long k = argmax_key(s_q[a], a);
      ka = k > ka ? k : ka;
    }
    const int am = argmax_idx(wave_max(ka));
    if (tid == 0) {
      __hip_atomic_store(S->key + t, argmax_key(mx, t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(S->act + t, am, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // release this head's key, acquire every earlier arrival's (the last arrival reads them all)
      const unsigned prev = __hip_atomic_fetch_add(&S->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned)T - 1) {
        unsigned long long best = 0ull;
        for (int u = 0; u < T; ++u) {
          const unsigned long long k = __hip_atomic_load(S->key + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          best = k > best ? k : best;
        }
        const int c = A.use_gpi ? argmax_idx(best) : A.select_task;
        const int a = __hip_atomic_load(S->act + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (so) {
          __hip_atomic_store(so, (int64_t)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(so + 1, (int64_t)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (P.res) publish_result(so, P.flag, P.res, P.dctr, P.cancel, P.nonfin);
        }
        __hip_atomic_store(&S->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  PROBE_REC(16, pt0);
}

template <int VW>
__global__ __launch_bounds__(256) void k_sel1m(Geo G, GpiArgs A, SelPub P, SelScratch* S) {
  sel1m_body<VW>(G, A, P, S, blockIdx.x);
}

}  // namespace sfx

namespace sfx {

// -------------------------------------------------------------------------------------
// Sharded heads: rank g owns heads [off, off + T) of T_glob; w is replicated
// ([T_glob][dpad]).  GPI over all heads = all-reduce(MAX) of per-rank maxima, which is exact
// (max is order-free) and keeps argmax first-index tie-breaking.
// -------------------------------------------------------------------------------------
// q[idx] = Σ_k p_idx[k] w[k] for idx < n, one fmaf chain in k order per dot (the order every
// GPI kernel uses, so argmaxes agree bit for bit).  d = 4V <= 4 VMAX with 16-B aligned rows:
// U dots per thread with every load issued before the first FMA; other d: scalar loop.
template <int VMAX, int U, class PF>
__device__ __forceinline__ void qdots_vec(int n, int d, const float* s_w, float* s_q, PF ptr) {
  const int V = d >> 2;
  for (int base = threadIdx.x; base < n; base += 256 * U) {
    float4 v[U][VMAX];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * 256;
      const float4* p = reinterpret_cast<const float4*>(ptr(idx < n ? idx : 0));
#pragma unroll
      for (int j = 0; j < VMAX; ++j) v[u][j] = (idx < n && j < V) ? p[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * 256;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < VMAX; ++j) {
        if (j < V) {
          q = __builtin_fmaf(v[u][j].x, s_w[4 * j], q);
          q = __builtin_fmaf(v[u][j].y, s_w[4 * j + 1], q);
          q = __builtin_fmaf(v[u][j].z, s_w[4 * j + 2], q);
          q = __builtin_fmaf(v[u][j].w, s_w[4 * j + 3], q);
        }
      }
      if (idx < n) s_q[idx] = q;
    }
  }
}

template <class PF>
__device__ __forceinline__ void qdots(int n, int d, const float* s_w, float* s_q, PF ptr) {
  if ((d & 3) == 0 && d <= 8) {
    qdots_vec<2, 8>(n, d, s_w, s_q, ptr);
  } else if ((d & 3) == 0 && d <= 16) {
    qdots_vec<4, 4>(n, d, s_w, s_q, ptr);
  } else {
    for (int idx = threadIdx.x; idx < n; idx += 256) {
      const float* p = ptr(idx);
      float q = 0.f;
#pragma unroll 8
      for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
      s_q[idx] = q;
    }
  }
}

struct QmaxArgs {
  int M, Tg, off, guess, rows, pol0, tsel, pad_;
  int* X;  // [npol][M][A]: max over this rank's heads of q[b, t, a] with w of policy pol0 + blockIdx.x,
           // sortable int32 (tsel >= 0: only local head tsel, the own-ψ branch of TSF's next actions)
};

// K5: grid (Tg, ceil(M / rows)).  Head t (global off + t) enters policy i's GPI through role
// `guess` if off + t < i (already updated in the reference's order) else R_S1.
__global__ __launch_bounds__(256) void k_qmax(Geo G, QmaxArgs Q) {
  const int i = Q.pol0 + blockIdx.x, tid = threadIdx.x;
  const int T = Q.tsel >= 0 ? 1 : G.T, t0 = Q.tsel >= 0 ? Q.tsel : 0;
  const int Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff, TA = T * Aa;
  const FDiv fTA = fdiv(TA), fA = fdiv(Aa);
  const int b0 = blockIdx.y * Q.rows;
  const int nb = Q.M - b0 < Q.rows ? Q.M - b0 : Q.rows;
  if (nb <= 0) return;
  __shared__ float s_w[DMAX];
  __shared__ float s_q[QMAX];
  const float* wrow = G.w + (long long)i * G.dpad;
  for (int k = tid; k < d; k += 256) s_w[k] = wrow[k];
  __syncthreads();
  const int off = Q.off, guess = Q.guess;
  qdots(nb * TA, d, s_w, s_q, [&](int idx) {
    const int bl = idx / fTA, rem = idx - bl * TA, t = t0 + rem / fA, a = rem - (t - t0) * Aa;
    return G.actp(off + t < i ? guess : R_S1, t, NLm) + (size_t)(b0 + bl) * O + a * d;
  });
  __syncthreads();
  for (int j = tid; j < nb * Aa; j += 256) {
    const int bl = j / fA, a = j - bl * Aa;
    const float* qb = s_q + bl * TA + a;
    float mx = qb[0];
    for (int t = 1; t < T; ++t) mx = fmaxf(mx, qb[t * Aa]);
    Q.X[((size_t)blockIdx.x * Q.M + b0 + bl) * Aa + a] = sortable(mx);
  }
}

// first argmax (torch.argmax tie-breaking) of A sortable maxima
__device__ __forceinline__ int first_argmax(const int* x, int Aa) {
  int am = 0;
  float b = unsortable(x[0]);
  for (int a = 1; a < Aa; ++a) {
    const float v = unsortable(x[a]);
    if (v > b) {
      b = v;
      am = a;
    }
  }
  return am;
}

// K6: first policy whose next actions differ between the TD maxima X (from the guesses) and
// the verification maxima Y (from the post-update heads); Tg if none.  One workgroup.
__global__ __launch_bounds__(256) void k_sverify(const int* X, const int* Y, int Tg, int M, int Aa, int* flag) {
  __shared__ int s_min;
  if (threadIdx.x == 0) s_min = Tg;
  __syncthreads();
  int mine = Tg;
  const FDiv fM = fdiv(M);
  for (int j = threadIdx.x; j < Tg * M; j += 256) {
    if (first_argmax(X + (size_t)j * Aa, Aa) != first_argmax(Y + (size_t)j * Aa, Aa)) mine = min(mine, j / fM);
  }
  atomicMin(&s_min, mine);
  __syncthreads();
  if (threadIdx.x == 0) *flag = s_min;
}

// K7: this rank's best (q, global t*A + a) for action selection in row `row` of role `role`
// with w of task `task`, packed into an order-preserving int64 so all-reduce(MAX) returns the
// reference's pick (argmax_t max_a, then argmax_a; first index on ties).  !use_gpi: only
// head `task` competes (c = task_index).
struct KeyArgs {
  int role, row, task, use_gpi, off, pad_;
  long long* key;
};

__device__ __forceinline__ unsigned int orderable(float q) {
  const unsigned int u = __float_as_uint(q);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void k_skey(Geo G, KeyArgs K) {
  __shared__ unsigned long long s_best;
  __shared__ float s_w[DMAX];
  const int tid = threadIdx.x, T = G.T, Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff;
  if (tid == 0) s_best = 0ull;
  const float* wrow = G.w + (long long)K.task * G.dpad;
  for (int k = tid; k < d; k += 256) s_w[k] = wrow[k];
  __syncthreads();
  unsigned long long best = 0ull;
  const FDiv fA = fdiv(Aa);
  for (int j = tid; j < T * Aa; j += 256) {
    const int t = j / fA, a = j - t * Aa, tg = K.off + t;
    if (!K.use_gpi && tg != K.task) continue;
    const float* p = G.actp(K.role, t, NLm) + (size_t)K.row * O + a * d;
    float q = 0.f;
#pragma unroll 8
    for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
    q = __fadd_rn(q, 0.f);  // -0 -> +0: torch's argmax treats them as equal
    const unsigned long long key =
        ((unsigned long long)orderable(q) << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)(tg * Aa + a));
    best = key > best ? key : best;
  }
  atomicMax(&s_best, best);
  __syncthreads();
  // unsigned order -> signed order (all-reduce MAX runs on int64); 0 (nothing here) -> INT64_MIN
  if (tid == 0) *K.key = (long long)(s_best ^ 0x8000000000000000ull);
}

// -------------------------------------------------------------------------------------
// The sharded env step in the native runner (sfx_runner schedule "sharded").
// Action selection goes through the same all-reduce(MAX) as the verification maxima: this
// rank writes q[t][a] = ψ_t(s_next)[a]·w_task of its own heads into its slice of a [T_glob][A]
// table and SORT_EMPTY into every other slice, so the all-reduced table is the full GPI q table
// on every rank; k_sfinish then picks argmax_t max_a and argmax_a (first index on ties:
// SF.GPI_w + agent argmax, features/successor.py:223-273).
// -------------------------------------------------------------------------------------
struct SselArgs {
  int role, row, task, use_gpi, off, Tg;
  int* q;  // [Tg][A] sortable
};

// grid cdiv(Tg * A, 256)
__global__ __launch_bounds__(256) void k_ssel(Geo G, SselArgs S) {
  __shared__ float s_w[DMAX];
  const int tid = threadIdx.x, Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff;
  const float* wrow = G.w + (long long)S.task * G.dpad;
  for (int k = tid; k < d; k += 256) s_w[k] = wrow[k];
  __syncthreads();
  const int j = blockIdx.x * 256 + tid;
  if (j >= S.Tg * Aa) return;
  const int tg = j / Aa, a = j - tg * Aa, t = tg - S.off;
  int q = SORT_EMPTY;
  if (t >= 0 && t < G.T && (S.use_gpi || tg == S.task)) {
    const float* p = G.actp(S.role, t, NLm) + (size_t)S.row * O + a * d;
    float acc = 0.f;
#pragma unroll 8
    for (int k = 0; k < d; ++k) acc = __builtin_fmaf(p[k], s_w[k], acc);  // the GPI kernels' k order
    q = sortable(acc);
  }
  S.q[j] = q;
}

struct SfinArgs {
  const int* X;  // [Tg][M][A] all-reduced TD maxima of the last round (null: no update this step)
  const int* Y;  // [Tg][M][A] all-reduced verification maxima
  const int* q;  // [Tg][A] all-reduced selection table
  int Tg, M, A, pad_;
  int* flag;     // first policy whose next actions changed (Tg: verified)
  int64_t* sel;  // (GPI task c, greedy action a)
  HostResult* pub;        // runner steps: publish (flag, sel) to the host (k_publish folded in)
  const long long* dctr;
  const int* cancel;
  const int* nonfin;      // Geo::nonfin
  long long* stall;       // test hook (sfx_debug_stall): one-shot delay before the publication
};

// One workgroup of 1024 threads: verification of the speculated next actions (k_sverify), the env
// action, and in runner steps the publication of both.
__global__ __launch_bounds__(1024) void k_sfinish(SfinArgs F) {
  __shared__ int s_min;
  __shared__ unsigned long long s_best;
  const int tid = threadIdx.x, Aa = F.A;
  if (tid == 0) {
    s_min = F.Tg;
    s_best = 0ull;
  }
  __syncthreads();
  int mine = F.Tg;
  if (F.X) {
    const FDiv fM = fdiv(F.M);
    for (int j = tid; j < F.Tg * F.M; j += blockDim.x)
      if (first_argmax(F.X + (size_t)j * Aa, Aa) != first_argmax(F.Y + (size_t)j * Aa, Aa)) mine = min(mine, j / fM);
  }
  // packed (q, first index) keys as k_skey: the max key is argmax_t max_a, then argmax_a
  unsigned long long best = 0ull;
  for (int j = tid; j < F.Tg * Aa; j += blockDim.x) {
    const int qi = F.q[j];
    if (qi == SORT_EMPTY) continue;
    const unsigned long long key =
        ((unsigned long long)orderable(unsortable(qi)) << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)j);
    best = key > best ? key : best;
  }
  atomicMin(&s_min, mine);
  atomicMax(&s_best, best);
  __syncthreads();
  if (tid == 0) {
    const unsigned idx = 0xFFFFFFFFu - (unsigned)(s_best & 0xFFFFFFFFull);
    const long long c = idx / (unsigned)Aa, a = idx % (unsigned)Aa;
    *F.flag = s_min;
    F.sel[0] = c;
    F.sel[1] = a;
    if (F.stall) {  // bounded by the host's value (<= 60 s), consumed once
      const long long n = *F.stall;
      if (n > 0) {
        *F.stall = 0;
        const long long t0 = wall_clock64();
        while (wall_clock64() - t0 < n) __builtin_amdgcn_s_sleep(127);
      }
    }
    if (F.pub) {
      const long long seq = *F.dctr;
      HostResult* pub = F.pub + (seq & (RES_RING - 1));  // the step's slot of the result ring
      pub->sel0 = c;
      pub->sel1 = a;
      pub->flag = s_min;
      pub->cancelled = *F.cancel;
      pub->nonfinite = F.nonfin ? __hip_atomic_load(F.nonfin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      __threadfence_system();
      __hip_atomic_store(&pub->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}


// -------------------------------------------------------------------------------------
// TSF-DQN with the heads sharded (BASELINE config C5; the native runner's "sharded_tsf"
// schedule): after the active task's owner has updated (tsfdqn.py:588-709), the
// shared h and w_task go from the owner to every rank as ONE all-reduce(MAX) over int32 words --
// the owner contributes their raw bits, every other rank INT_MIN, and max(b, INT_MIN) = b for
// every 32-bit pattern b, so the reduced words are the owner's bits exactly (a broadcast, -0 and
// NaN payloads included).  k_tsx_pack fills the words, k_tsx_unpack writes them back (every rank;
// the owner rewrites its own values; nothing in a cancelled step).
// -------------------------------------------------------------------------------------
struct TsxArgs {
  int nsh, Ph, own, pad_;
  float* hp;     // h parameters [Ph]
  float* w;      // w_task row [nsh - Ph]
  int* z;        // [nsh]
  const int* cancel;
};

__global__ __launch_bounds__(256) void k_tsx_pack(TsxArgs X) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < X.nsh) X.z[j] = X.own ? __float_as_int(j < X.Ph ? X.hp[j] : X.w[j - X.Ph]) : (int)0x80000000;
}

__global__ __launch_bounds__(256) void k_tsx_unpack(TsxArgs X) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= X.nsh || step_cancelled(X.cancel)) return;
  const float v = __int_as_float(X.z[j]);
  if (j < X.Ph)
    X.hp[j] = v;
  else
    X.w[j - X.Ph] = v;
}

}  // namespace sfx
