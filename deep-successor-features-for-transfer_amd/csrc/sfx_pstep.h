// sfx_pstep.h -- the all-task env step (agents/sfdqn.py:57-60 over features/deep.py:93-131) as ONE
// persistent launch per env step: k_pstep.
//
// Why.  The launch path (sfx.hip launch_step_all / launch_round) runs a step as ~19 dependent
// launches; every launch pays a kernel boundary (≈1.5-3 µs) plus a fresh operand fetch (2-4 µs)
// before it computes anything, and rounds whose policies all repeat still pay their launches.
// Here one launch of 256 workgroups (one per CU) runs the whole step: head t of T <= 8 lives on
// XCD t (its 32 CUs), each workgroup ("rank" r of its head) owns the hidden units [8r, 8r+8) of
// every hidden layer and action r of the output layer, and the phases of the step are separated
// by in-launch hand-offs instead of launch boundaries:
//   intra-head edges  -- activations / output gradients of one head, 32 producers -> 32
//                        consumers, published write-through (sc1) and signalled on the head's
//                        arrival counter (every storing wave drains, one lane per workgroup adds,
//                        the consumer polls sc1 and reads sc1: MI355X_MICROARCH.md's validated
//                        hand-off form; placement-independent -- XCC_ID only groups for speed);
//   cross-head edge   -- once per speculative round: every output-layer rank folds its q = ψ·w
//                        into the GPI maxima of every policy with agent-scope atomicMax (sortable
//                        int32, as the sharded step does) and adds to one counter.
// Weights are never staged by a launch boundary: each phase requests its weight slice (read slot
// of the head, L2/MALL-resident across steps) BEFORE it waits for its hand-off.
// Speculative rounds loop on the device until every policy's next actions repeat the previous
// round (the verification of sfx.hip's k_ver, evaluated by every workgroup from the same maxima),
// so a step never needs host rounds and never launches a round whose policies all repeat.
//
// Per round r (policy i = the head's index, sfx.hip §4 speculation):
//   a'_i(b)   = argmax_a max(max_{t<i} q_t^{post(r-1)}, max_{t>=i} q_t^{pre})      (r = 0: pre only)
//   converged = r >= 1 and a'_i(r) == a'_i(r-1) for every policy i   -> result of round r-1
//   skip_i    = r >= 1 and a'_i(r) == a'_i(r-1)                     -> head i keeps round r-1
//   else: TD target + output gradient (k_tdg arithmetic) -> dX / dW + Adam per layer (read slot ->
//         write slot) -> post-update forward of S1 ++ s_next -> maxima of round r for policies > i.
// The result equals the launch path's (same schedule, same skip rule, same Adam), evaluated in a
// different fp32 summation order for the dense products (VALU fmaf chains in k order instead of
// fp32 MFMA tiles): parity is checked against the oracle like every other path.
//
// Limits (host-checked, else the launch path runs): T <= 8 heads, hidden width 256, 1..4 hidden
// layers, n_s <= 64, A <= 32 actions, d <= 32, A·d <= 1024, B <= 32, fp32, GPI next actions, no
// per-step losses, and the LDS budget below.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sfx {

constexpr int PS_R = 32;               // workgroups (ranks) per head
constexpr int PS_H = 256;              // hidden width
constexpr int PS_J = PS_H / PS_R;      // hidden units per rank
constexpr int PS_MB = 32;              // minibatch rows
constexpr int PS_RMAX = 10;            // round buffers: rounds 0 .. T (T <= 8) + the pre-step part
constexpr int PS_NLMAX = 6;            // Linear layers
constexpr int PS_XS = PS_H + 4;        // LDS row stride of staged activations / weight rows (floats)
constexpr int PS_CSET = 32 * 18;       // counter words per parity set (each counter on its own 128 B)
constexpr int PS_GRID = 256;
constexpr int PS_MAXAS = 32;           // actions

struct PsLayer {
  int N, K, wOff, bOff, act;  // act: activation applied to this layer's output
};

struct PsArgs {
  int T, B, n_s, A, d, O, NL, task;
  int sel_use_gpi, lms_task, K0S, nsel;
  float lms_alpha, norm;
  unsigned long long mask;
  long long timeout;
  AdamHP hp;
  PsLayer L[PS_NLMAX];
  // LDS carve (floats), computed by the host (ps_smem)
  int o_sx, o_phi, o_gam, o_ab, o_w, o_own, o_dz, o_dzn, o_g3, o_g3m, o_ap, o_ac, o_cr, o_qs, o_wc3, o_psi, o_pst, o_nb,
      o_st;
  const float *S, *S1, *phi, *gamma, *s_next, *lms_phi, *lms_r;
  const int64_t* a;
  // workspace: intra-head hand-off buffers (rewritten every launch)
  float* xs;    // [T][NL-1][3*PS_MB][H]: step-start outputs of layers 0..NL-2 (rows S | S1 | S1 target)
  float* psit;  // [T][PS_MB][O]: ψ⁻(s1)
  float* cr;    // [T][PS_MB][d]: ψ_i(s_b)[a_b]
  float* dzb;   // [T][NL-1][PS_MB][H]: output gradients of hidden layers (index = layer)
  float* xv;    // [T][NL-1][PS_MB+1][H]: post-update forward of S1 ++ s_next, layers 0..NL-2
  // cross-head: two parity sets (launch k uses set k & 1 and clears the other for launch k + 1)
  int* xq;                  // [2][PS_RMAX][T][PS_MB][A]: round r's maxima over heads t < i (r = 0: pre-step)
  int* xge;                 // [2][T][PS_MB][A]: pre-step maxima over heads t >= i
  unsigned long long* sel;  // [2][PS_RMAX]: selection key of round r - 1's post-update heads
  unsigned* cnt;            // [2][PS_CSET]: tickets per XCD, arrivals per head, q arrivals, exits
  unsigned* epoch;          // launch counter (parity)
  int* err;                 // nonzero: a bounded wait gave up (host: the step failed)
  int64_t* sel_out;         // dout->sel
  int* flag;                // dout->flag: T when verified (always, unless err)
  HostResult* pub;          // runner: result ring (null: none)
  const long long* pub_dctr;
  unsigned long long* stats;  // [0] steps, [1] rounds computed, [2] policies checked, [3] skipped
  int* trace;  // [PS_RMAX][8][PS_MB + 1]: per round and head, the next actions it used (+ 1 computed / 0 skipped)
  long long* timeline;  // optional (SFX_PSTEP_PROBE=1): [8][PS_TL] wall-clock marks of rank 0 of each head
};
constexpr int PS_TL = 64;
#define PS_MARK0(i)                                                                              \
  do {                                                                                           \
    if (r == 0) PS_MARK(i);                                                                      \
  } while (0)
#define PS_MARK(i)                                                                               \
  do {                                                                                           \
    if (P.timeline && rank == 0 && tid == 0 && head < 8 && (i) < PS_TL) P.timeline[head * PS_TL + (i)] = wall_clock64(); \
  } while (0)

__device__ __forceinline__ unsigned ps_xcc() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xF;
}
__device__ __forceinline__ float ps_ld(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ps_ldi(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ps_st(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte sc1 (L1-bypassing) load of bytes another workgroup published in this launch
__device__ __forceinline__ float4 ps_ld4(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ps_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Hand-off producer side: every storing wave drains its sc1 stores, then ONE lane adds.
__device__ __forceinline__ void ps_arrive(unsigned* c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Consumer side: one lane polls (sc1, bounded), the workgroup joins at a barrier; returns false
// (and sets *err) when the wait gave up or another workgroup already did.
__device__ __forceinline__ bool ps_wait(const PsArgs& P, unsigned* c, unsigned target, int* s_ok) {
  if (threadIdx.x == 0) {
    int ok = 1;
    const long long t0 = wall_clock64();
    unsigned it = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if ((++it & 31) == 0 &&
          (wall_clock64() - t0 > P.timeout || __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_fetch_or(P.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_ok = ok;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
  return *s_ok != 0;
}

// rows x 256 floats at src (global, published in this launch) -> LDS dst at row stride PS_XS
template <int CH>
__device__ __forceinline__ void ps_stage(const float* src, int rows, float* dst) {
  const __amdgpu_buffer_rsrc_t r = ps_rsrc(src, (unsigned)rows * PS_H * 4u);
  const int n4 = rows * (PS_H / 4);
  for (int i0 = 0; i0 < n4; i0 += 256 * CH) {
    float4 v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int i = i0 + c * 256 + threadIdx.x;
      v[c] = i < n4 ? ps_ld4(r, i * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int i = i0 + c * 256 + threadIdx.x;
      if (i < n4) *reinterpret_cast<float4*>(dst + (i >> 6) * PS_XS + ((i & 63) << 2)) = v[c];
    }
  }
}

// k-ordered fmaf chain of two LDS rows (16-B aligned, K % 4 == 0)
__device__ __forceinline__ float ps_dot(const float* x, const float* w, int K) {
  float acc = 0.f;
  for (int k = 0; k < K; k += 4) {
    const float4 a = *reinterpret_cast<const float4*>(x + k);
    const float4 b = *reinterpret_cast<const float4*>(w + k);
    acc = __builtin_fmaf(a.x, b.x, acc);
    acc = __builtin_fmaf(a.y, b.y, acc);
    acc = __builtin_fmaf(a.z, b.z, acc);
    acc = __builtin_fmaf(a.w, b.w, acc);
  }
  return acc;
}

// order-preserving u32 of a float (the high word of the selection key)
__device__ __forceinline__ unsigned ps_ukey(float q) { return (unsigned)sortable(q) ^ 0x80000000u; }

// Per-thread state that every speculative round of a step re-reads is made resident ONCE per step:
// the Adam state (p, m, v of the read slot) of this rank's rows of every layer and the columns
// X_l[b][tid] of the step-start activations that the dW sums need live in registers; the weight
// column slices of the dX products, ψ⁻(s1) and c in LDS; the post-update weights a round produces
// stay in LDS for that round's forward.  A round then pays only its hand-offs.
// NH hidden Linear layers (NL = NH + 2), DC = ceil(d / 8) chunks of 8 output rows per rank.
template <int NH, int DC>
__global__ __launch_bounds__(256) void k_pstep(Geo G, PsArgs P) {
  constexpr int NL = NH + 2;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ int s_rank, s_ok, s_flag;
  __shared__ AdamC s_ac;
  const int tid = threadIdx.x;
  const int T = P.T, B = P.B, A = P.A, d = P.d, O = P.O, n_s = P.n_s, K0S = P.K0S;
  const unsigned ep = __hip_atomic_load(P.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int par = (int)(ep & 1u);
  unsigned* cnt = P.cnt + par * PS_CSET;
  const int nxq = PS_RMAX * T * PS_MB * A, nxge = T * PS_MB * A;
  int* xq = P.xq + (size_t)par * nxq;
  int* xge = P.xge + (size_t)par * nxge;
  unsigned long long* sel = P.sel + par * PS_RMAX;
  {  // clear the other parity set for the next launch (plain stores; the kernel boundary publishes them)
    const int q = par ^ 1, gt = blockIdx.x * 256 + tid, gn = gridDim.x * 256;
    unsigned* c2 = P.cnt + q * PS_CSET;
    for (int i = gt; i < PS_CSET; i += gn) c2[i] = 0u;
    int* x2 = P.xq + (size_t)q * nxq;
    for (int i = gt; i < nxq; i += gn) x2[i] = SORT_EMPTY;
    int* g2 = P.xge + (size_t)q * nxge;
    for (int i = gt; i < nxge; i += gn) g2[i] = SORT_EMPTY;
    if (gt < PS_RMAX) P.sel[q * PS_RMAX + gt] = 0ull;
  }
  const unsigned xcc = ps_xcc();
  if (tid == 0)
    s_rank = xcc < 8 ? (int)__hip_atomic_fetch_add(cnt + 32 * xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : PS_R;
  __syncthreads();
  const int head = (int)xcc, rank = s_rank, hd = head & 7;
  const bool active = head < T && rank < PS_R;
  const int cancelled = step_cancelled(G.cancel);
  const bool work = active && !cancelled;
  unsigned* hctr = cnt + 32 * (8 + hd);
  unsigned* qctr = cnt + 32 * 16;
  unsigned* fin = cnt + 32 * 17;
  const bool outr = rank < A;  // this rank owns action `rank` of the output layer
  unsigned e = 0;              // intra-head edges completed so far
  int rounds = 0;              // the converged round (the result is round rounds - 1's)
  bool ok = true;
  int r = 0;                   // current round (PS_MARK0)
  // LDS carve (sfx_pstep.inc pstep_carve)
  float* sx = sm + P.o_sx;     // [97][K0S]: S | S1 | S1 | s_next
  float* sphi = sm + P.o_phi;  // [32][d]
  float* sgam = sm + P.o_gam;  // [32]
  int* sab = reinterpret_cast<int*>(sm + P.o_ab);  // [32]
  float* sw = sm + P.o_w;      // [T][d] reward weights (the active task's after LMS)
  float* own = sm + P.o_own;   // [NL-1][32][8]: own columns of the step-start S-row activations
  // dZ columns and the masked output gradient are stored transposed (row b contiguous per column)
  // so the dW sums read 4 rows per 16-byte LDS read
  float* sdz = sm + P.o_dz;    // [8][32]: own columns of the current output gradient
  float* sdzn = sm + P.o_dzn;  // [8][32]: ... of the next (lower) layer
  float* g3 = sm + P.o_g3;     // [32][d]: TD gradient at the taken action
  float* g3m = sm + P.o_g3m;   // [d][32] (transposed): the same, zero in rows whose action is not this rank's
  int* ap = reinterpret_cast<int*>(sm + P.o_ap);  // [8][32] next actions of the previous round
  int* ac = reinterpret_cast<int*>(sm + P.o_ac);  // [8][32] ... of this round
  float* scr = sm + P.o_cr;    // [32][d] ψ_i(s_b)[a_b]
  float* qs = sm + P.o_qs;     // [8][32] saved post-update q of this rank's action (skip re-publication)
  float* wc3 = sm + P.o_wc3;   // [O][8]: output-layer weights of this rank's hidden columns (read slot)
  float* psi = sm + P.o_psi;   // [33][d]: ψ of this rank's action
  float* pst = sm + P.o_pst;   // [32][O]: ψ⁻(s1) of this head
  float* nb = sm + P.o_nb;     // [NL-1][8] post-update biases of this rank's hidden units; [NL-1][..] output
  float* st = sm + P.o_st;     // staging
  // round-time staging layout: [33][XS] hand-off rows | WcT [NH][8][XS] | Wn [NH][8][XS] | Wno [8 DC][XS] | W0n
  float* WcT = st + (PS_MB + 1) * PS_XS;
  float* Wn = WcT + NH * PS_J * PS_XS;
  float* Wno = Wn + NH * PS_J * PS_XS;
  float* W0n = Wno + 8 * DC * PS_XS;
  unsigned long long qkey = 0ull;
  int step0 = 0;
  const int rs = rslot(P.mask, hd), wsl = rs ^ 1;
  const float* pon = G.online + G.slot_off(rs, hd);  // read slot (pre-step)
  float* pnew = G.online + G.slot_off(wsl, hd);      // write slot
  const float* mrd = G.am + G.slot_off(rs, hd);
  const float* vrd = G.av + G.slot_off(rs, hd);
  float* mwr = G.am + G.slot_off(wsl, hd);
  float* vwr = G.av + G.slot_off(wsl, hd);
  const float* ptg = G.target + (long long)hd * G.P;
  const int j = tid & 7, g = tid >> 3;  // (hidden column, row group) of the 8-column phases
  const int c0 = PS_J * (rank & 31);    // this rank's first hidden unit
  const int arow = (rank & 31) * d;     // this rank's first output row
  float* xsh = P.xs + (size_t)hd * (NL - 1) * 3 * PS_MB * PS_H;
  float* dzh = P.dzb + (size_t)hd * (NL - 1) * PS_MB * PS_H;
  float* xvh = P.xv + (size_t)hd * (NL - 1) * (PS_MB + 1) * PS_H;
  float* psith = P.psit + (size_t)hd * PS_MB * O;
  float* crh = P.cr + (size_t)hd * PS_MB * d;

  // ---- register-resident Adam state of this rank's rows (read slot: written by no one in this launch)
  float pw[NH][PS_J][3];      // hidden layer l = 1..NH, rows c0 + jj, column tid
  // output rows arow + 8c + u, column tid (output ranks): registers for DC = 1 only; wider output
  // slices read their (read-slot) Adam state at the update instead -- at DC >= 2 the resident copy
  // pushed the kernel into heavy register spilling, and the DC = 3 build lost resident state
  // (tests/test_gpu_pstep.py caught it at d = 20)
  constexpr bool PO_REG = DC == 1;
  float po[PO_REG ? DC : 1][8][3];
  float p0[3] = {0.f, 0.f, 0.f};  // layer 0: entry tid of rows c0.. (8 n_s <= 256 entries)
  float pb[NL - 1][3];        // threads < 8: bias c0 + tid of layers 0 .. NH
  float pbo[3] = {0.f, 0.f, 0.f};  // threads < d: output bias arow + tid
  float xc[NH + 1][PS_MB];    // X_l[b][tid] of the step-start S rows, l = 0 .. NH (X_NH: output ranks)
  if (work) {
#pragma unroll
    for (int l = 0; l < NH; ++l)
#pragma unroll
      for (int jj = 0; jj < PS_J; ++jj) {
        const size_t wi = P.L[l + 1].wOff + (size_t)(c0 + jj) * PS_H + tid;
        pw[l][jj][0] = pon[wi];
        pw[l][jj][1] = mrd[wi];
        pw[l][jj][2] = vrd[wi];
      }
    if constexpr (PO_REG) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool okk = outr && u < d;
        const size_t wi = P.L[NL - 1].wOff + (size_t)(arow + u) * PS_H + tid;
        po[0][u][0] = okk ? pon[wi] : 0.f;
        po[0][u][1] = okk ? mrd[wi] : 0.f;
        po[0][u][2] = okk ? vrd[wi] : 0.f;
      }
    }
    if (tid < PS_J * n_s) {
      const size_t wi = P.L[0].wOff + (size_t)c0 * n_s + tid;
      p0[0] = pon[wi];
      p0[1] = mrd[wi];
      p0[2] = vrd[wi];
    }
#pragma unroll
    for (int l = 0; l < NL - 1; ++l) {
      const size_t bi = P.L[l].bOff + c0 + (tid & 7);
      pb[l][0] = tid < PS_J ? pon[bi] : 0.f;
      pb[l][1] = tid < PS_J ? mrd[bi] : 0.f;
      pb[l][2] = tid < PS_J ? vrd[bi] : 0.f;
    }
    if (outr && tid < d) {
      const size_t bi = P.L[NL - 1].bOff + arow + tid;
      pbo[0] = pon[bi];
      pbo[1] = mrd[bi];
      pbo[2] = vrd[bi];
    }
    // ---------------- inputs: S | S1 | S1 | s_next (K padded to K0S), φ, γ, a, w (+ LMS)
    for (int i = tid; i < 97 * K0S; i += 256) {
      const int row = i / K0S, k = i - row * K0S;
      float v = 0.f;
      if (k < n_s) {
        if (row < 32) v = row < B ? P.S[row * n_s + k] : 0.f;
        else if (row < 96) v = (row & 31) < B ? P.S1[(row & 31) * n_s + k] : 0.f;
        else v = P.s_next[k];
      }
      sx[i] = v;
    }
    for (int i = tid; i < PS_MB * d; i += 256) sphi[i] = i < B * d ? P.phi[i] : 0.f;
    if (tid < PS_MB) {
      sgam[tid] = tid < B ? P.gamma[tid] : 0.f;
      sab[tid] = tid < B ? (int)P.a[tid] : -1;
    }
    for (int i = tid; i < T * d; i += 256) {
      const int t = i / d;
      sw[i] = G.w[(long long)t * G.dpad + (i - t * d)];
    }
    step0 = G.step[head];
    __syncthreads();
    if (P.lms_task >= 0 && tid == 0) {  // features/successor.py:164-167, k_lms's order
      float* w = sw + P.lms_task * d;
      float rf = 0.f;
      for (int k = 0; k < d; ++k) rf = __fadd_rn(rf, __fmul_rn(P.lms_phi[k], w[k]));
      const float ee = __fmul_rn(P.lms_alpha, __fsub_rn(P.lms_r[0], rf));
      for (int k = 0; k < d; ++k) w[k] = __fadd_rn(w[k], __fmul_rn(ee, P.lms_phi[k]));
    }
    __syncthreads();
  }

  // ---------------- step-start forward, layer 0 (K = n_s): rows S, S1 (online), S1 (target)
  PS_MARK(0);
  if (work) {
    const PsLayer L0 = P.L[0];
    float* W0s = st;  // [2][8][K0S] online, target rows c0..c0+7; then the 2 x 8 biases
    {
      const int n0 = PS_J * n_s;  // the 8 rows are contiguous in the packed head
      for (int i = tid; i < 2 * n0 + 2 * PS_J; i += 256) {
        if (i < 2 * n0) {
          const int which = i >= n0, ii = i - which * n0, jj = ii / n_s, k = ii - jj * n_s;
          W0s[(which * PS_J + jj) * K0S + k] = (which ? ptg : pon)[L0.wOff + (size_t)c0 * n_s + ii];
        } else {
          const int ii = i - 2 * n0;
          W0s[2 * PS_J * K0S + ii] = (ii >= PS_J ? ptg : pon)[L0.bOff + c0 + (ii & 7)];
        }
      }
      __syncthreads();
    }
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int k = 0; k < n_s; ++k) {
      const float wk = W0s[j * K0S + k], tk = W0s[(PS_J + j) * K0S + k];
      a0 = __builtin_fmaf(sx[g * K0S + k], wk, a0);
      a1 = __builtin_fmaf(sx[(32 + g) * K0S + k], wk, a1);
      a2 = __builtin_fmaf(sx[(64 + g) * K0S + k], tk, a2);
    }
    const float bo0 = W0s[2 * PS_J * K0S + j], bt0 = W0s[2 * PS_J * K0S + PS_J + j];
    const float y0 = act_fwd(__fadd_rn(a0, bo0), L0.act);
    const float y1 = act_fwd(__fadd_rn(a1, bo0), L0.act);
    const float y2 = act_fwd(__fadd_rn(a2, bt0), L0.act);
    ps_st(xsh + (size_t)g * PS_H + c0 + j, y0);
    ps_st(xsh + (size_t)(32 + g) * PS_H + c0 + j, y1);
    ps_st(xsh + (size_t)(64 + g) * PS_H + c0 + j, y2);
    own[g * 8 + j] = y0;
    ps_arrive(hctr);
    ++e;
    // the Adam constants of this step (double precision, as ATen forms them: one lane, off the
    // critical path -- the next hand-off takes longer)
    if (tid == 64) s_ac = adam_consts(P.hp, step0 + 1);
    PS_MARK(1);
  }
  // ---------------- step-start forward, hidden layers 1 .. NH
#pragma unroll
  for (int l = 1; l <= NH; ++l) {
    if (work && ok) {
    const PsLayer Ll = P.L[l];
    float* X = st;                 // [96][PS_XS]
    float* Wst = st + 96 * PS_XS;  // [16][PS_XS]: online rows c0.., target rows c0..
    for (int i = tid; i < 16 * 64; i += 256) {  // weight rows first: they do not depend on the hand-off
      const int row = i >> 6, c4 = (i & 63) << 2;
      const float* src = (row < 8 ? pon : ptg) + Ll.wOff + (size_t)(c0 + (row & 7)) * PS_H + c4;
      *reinterpret_cast<float4*>(Wst + row * PS_XS + c4) = *reinterpret_cast<const float4*>(src);
    }
    const float bo = pon[Ll.bOff + c0 + j], bt = ptg[Ll.bOff + c0 + j];
    ok = ps_wait(P, hctr, PS_R * e, &s_ok);
    if (ok) {
    ps_stage<12>(xsh + (size_t)(l - 1) * 3 * PS_MB * PS_H, 96, X);
    __syncthreads();
#pragma unroll
    for (int b = 0; b < PS_MB; ++b) xc[l - 1][b] = X[b * PS_XS + tid];  // X_{l-1}[b][tid], S rows
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    {
      const float* x0 = X + g * PS_XS;
      const float* x1 = X + (32 + g) * PS_XS;
      const float* x2 = X + (64 + g) * PS_XS;
      const float* w0 = Wst + j * PS_XS;
      const float* w1 = Wst + (8 + j) * PS_XS;
      for (int k = 0; k < PS_H; k += 4) {
        const float4 wa = *reinterpret_cast<const float4*>(w0 + k);
        const float4 wb = *reinterpret_cast<const float4*>(w1 + k);
        const float4 v0 = *reinterpret_cast<const float4*>(x0 + k);
        const float4 v1 = *reinterpret_cast<const float4*>(x1 + k);
        const float4 v2 = *reinterpret_cast<const float4*>(x2 + k);
        a0 = __builtin_fmaf(v0.x, wa.x, a0); a0 = __builtin_fmaf(v0.y, wa.y, a0);
        a0 = __builtin_fmaf(v0.z, wa.z, a0); a0 = __builtin_fmaf(v0.w, wa.w, a0);
        a1 = __builtin_fmaf(v1.x, wa.x, a1); a1 = __builtin_fmaf(v1.y, wa.y, a1);
        a1 = __builtin_fmaf(v1.z, wa.z, a1); a1 = __builtin_fmaf(v1.w, wa.w, a1);
        a2 = __builtin_fmaf(v2.x, wb.x, a2); a2 = __builtin_fmaf(v2.y, wb.y, a2);
        a2 = __builtin_fmaf(v2.z, wb.z, a2); a2 = __builtin_fmaf(v2.w, wb.w, a2);
      }
    }
    const float y0 = act_fwd(__fadd_rn(a0, bo), Ll.act);
    const float y1 = act_fwd(__fadd_rn(a1, bo), Ll.act);
    const float y2 = act_fwd(__fadd_rn(a2, bt), Ll.act);
    float* out = xsh + (size_t)l * 3 * PS_MB * PS_H;
    ps_st(out + (size_t)g * PS_H + c0 + j, y0);
    ps_st(out + (size_t)(32 + g) * PS_H + c0 + j, y1);
    ps_st(out + (size_t)(64 + g) * PS_H + c0 + j, y2);
    own[(l * 32 + g) * 8 + j] = y0;
    ps_arrive(hctr);
    ++e;
    PS_MARK(1 + l);
    }
    }
  }
  // ---------------- step-start output layer (rank a < A): c rows, ψ⁻(s1), pre-step maxima
  const PsLayer LO = P.L[NL - 1];
  if (work && ok && outr) {
    float* X = st;                 // [96][PS_XS]
    float* Wst = st + 96 * PS_XS;  // [d][PS_XS]: online rows of action `rank`, then target
    for (int i = tid; i < d * 64; i += 256) {
      const int row = i >> 6, c4 = (i & 63) << 2;
      *reinterpret_cast<float4*>(Wst + row * PS_XS + c4) =
          *reinterpret_cast<const float4*>(pon + LO.wOff + (size_t)(arow + row) * PS_H + c4);
    }
    // target rows: beside the online rows when the staging holds both (96 + 2d <= 112 rows), else
    // over them once the online rows are done
    const bool tw_lds = 96 + 2 * d <= 112;
    float* Wtg = tw_lds ? Wst + d * PS_XS : Wst;
    if (tw_lds)
      for (int i = tid; i < d * 64; i += 256) {
        const int row = i >> 6, c4 = (i & 63) << 2;
        *reinterpret_cast<float4*>(Wtg + row * PS_XS + c4) =
            *reinterpret_cast<const float4*>(ptg + LO.wOff + (size_t)(arow + row) * PS_H + c4);
      }
    ok = ps_wait(P, hctr, PS_R * e, &s_ok);
    if (ok) {
      ps_stage<12>(xsh + (size_t)(NL - 2) * 3 * PS_MB * PS_H, 96, X);
      __syncthreads();
#pragma unroll
      for (int b = 0; b < PS_MB; ++b) xc[NH][b] = X[b * PS_XS + tid];
      for (int i = tid; i < 64 * d; i += 256) {  // online: S rows -> c, S1 rows -> psi
        const int row = i / d, k = i - row * d;
        const float y = __fadd_rn(ps_dot(X + row * PS_XS, Wst + k * PS_XS, PS_H), pon[LO.bOff + arow + k]);
        if (row < 32) {
          if (row < B && sab[row] == rank) ps_st(crh + row * d + k, y);
        } else {
          psi[(row - 32) * d + k] = y;
        }
      }
      __syncthreads();
      if (!tw_lds) {
        for (int i = tid; i < d * 64; i += 256) {
          const int row = i >> 6, c4 = (i & 63) << 2;
          *reinterpret_cast<float4*>(Wtg + row * PS_XS + c4) =
              *reinterpret_cast<const float4*>(ptg + LO.wOff + (size_t)(arow + row) * PS_H + c4);
        }
        __syncthreads();
      }
      for (int i = tid; i < B * d; i += 256) {  // target: ψ⁻(s1_b)[rank][k]
        const int b = i / d, k = i - b * d;
        const float y = __fadd_rn(ps_dot(X + (64 + b) * PS_XS, Wtg + k * PS_XS, PS_H), ptg[LO.bOff + arow + k]);
        ps_st(psith + b * O + arow + k, y);
      }
      // pre-step maxima: policy i <= head takes this head through xge, i > head through xq[0]
      for (int i = tid; i < T * B; i += 256) {
        const int pi = i / B, b = i - pi * B;
        float q = 0.f;
        for (int k = 0; k < d; ++k) q = __builtin_fmaf(psi[b * d + k], sw[pi * d + k], q);
        int* dst = pi <= head ? xge + (pi * PS_MB + b) * A + rank : xq + (pi * PS_MB + b) * A + rank;
        __hip_atomic_fetch_max(dst, sortable(q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ps_arrive(qctr);
    }
  }
  PS_MARK(6);
  // ---------------- operands of every round that do not change from round to round (read slot):
  // the dX weight slices W_l[:, c0 .. c0+7] (transposed) and W_out[:, c0 .. c0+7]
  if (work && ok) {
    __syncthreads();  // the step-start staging is dead: WcT overlaps it
#pragma unroll
    for (int l = 1; l <= NH; ++l) {
      const float4* src = reinterpret_cast<const float4*>(pon + P.L[l].wOff + (size_t)tid * PS_H + c0);
      const float4 lo = src[0], hi = src[1];
      float* w = WcT + (l - 1) * PS_J * PS_XS;
      w[0 * PS_XS + tid] = lo.x; w[1 * PS_XS + tid] = lo.y; w[2 * PS_XS + tid] = lo.z; w[3 * PS_XS + tid] = lo.w;
      w[4 * PS_XS + tid] = hi.x; w[5 * PS_XS + tid] = hi.y; w[6 * PS_XS + tid] = hi.z; w[7 * PS_XS + tid] = hi.w;
    }
    for (int o = tid; o < O; o += 256) {
      const float4* src = reinterpret_cast<const float4*>(pon + LO.wOff + (size_t)o * PS_H + c0);
      *reinterpret_cast<float4*>(wc3 + o * 8) = src[0];
      *reinterpret_cast<float4*>(wc3 + o * 8 + 4) = src[1];
    }
  }
  const unsigned qper = (unsigned)(T * A);
  __syncthreads();
  const AdamC adc = s_ac;
  for (r = 0; work && ok; ++r) {
    if (!(ok = ps_wait(P, qctr, qper * (unsigned)(r + 1), &s_ok))) break;
    PS_MARK(8 + 8 * (r < 6 ? r : 5));
    // next actions of every policy (each workgroup the same, from the same maxima): every load
    // issued before the first compare; round 0 also takes ψ⁻(s1) and c of this head into LDS
    int chg = 0, chg_own = 0;
    if (r == 0) {
      for (int i = tid; i < B * O; i += 256) pst[i] = ps_ld(psith + i);
      for (int i = tid; i < B * d; i += 256) scr[i] = ps_ld(crh + i);
    }
    {  // the round's maxima of every policy, max(xq[r], xge), into LDS (the staging rows are free)
      int* mx = reinterpret_cast<int*>(st);
      const int n = T * PS_MB * A;
      const int* xr = xq + (size_t)r * n;
      for (int i0 = 0; i0 < n; i0 += 256 * 8) {
        int xv[8], gv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * 256 + tid;
          xv[u] = i < n ? ps_ldi(xr + i) : 0;
          gv[u] = i < n ? ps_ldi(xge + i) : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + u * 256 + tid < n) mx[i0 + u * 256 + tid] = max(xv[u], gv[u]);
      }
    }
    __syncthreads();
    if (tid < T * B) {
      const int pi = tid / B, b = tid - pi * B;
      const int* m = reinterpret_cast<const int*>(st) + (pi * PS_MB + b) * A;
      int best = 0, bv = m[0];
      for (int aa = 1; aa < A; ++aa)
        if (m[aa] > bv) {
          bv = m[aa];
          best = aa;
        }
      ac[pi * PS_MB + b] = best;
      if (r > 0 && best != ap[pi * PS_MB + b]) {
        chg = 1;
        chg_own = pi == head;
      }
    }
    const int any = __syncthreads_or(chg);
    const int own_chg = __syncthreads_or(chg_own);
    if (r > 0 && !any) {
      rounds = r;
      if (rank == 0 && head == 0 && tid == 0) P.trace[PS_RMAX * 8 * (PS_MB + 1)] = r;
      break;
    }
    if (r > T) {  // every round fixes at least one more policy
      __hip_atomic_fetch_or(P.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = false;
      break;
    }
    const bool skip = r > 0 && !own_chg;
    if (tid == 0 && rank == 0 && r > 0) {
      __hip_atomic_fetch_add(P.stats + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (skip) __hip_atomic_fetch_add(P.stats + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int i = tid; i < T * PS_MB; i += 256) ap[i] = ac[i];
    if (rank == 0 && tid <= PS_MB)  // the round's record of this head (sfx_pstep_trace)
      P.trace[(r * 8 + head) * (PS_MB + 1) + tid] = tid < PS_MB ? ac[head * PS_MB + tid] : (skip ? 0 : 1);
    int* xqn = xq + (size_t)(r + 1) * T * PS_MB * A;  // this round's post-update maxima (policies > head)
    if (skip) {  // the policy repeats round r - 1: re-publish that round's terms
      if (outr) {
        for (int i = tid; i < T * B; i += 256) {
          const int pi = i / B, b = i - pi * B;
          if (pi > head)
            __hip_atomic_fetch_max(xqn + (pi * PS_MB + b) * A + rank, sortable(qs[pi * PS_MB + b]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0 && qkey) __hip_atomic_fetch_max(sel + r + 1, qkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ps_arrive(qctr);
      }
      continue;
    }
    // ---- TD target and output gradient (k_tdg's arithmetic), every rank the same
    const int* an = ac + head * PS_MB;
    int nf = 0;
    for (int i = tid; i < PS_MB * d; i += 256) {
      const int b = i / d, k = i - b * d;
      float gv = 0.f;
      if (b < B && sab[b] >= 0 && sab[b] < A) {
        const float tg = __fadd_rn(sphi[b * d + k], __fmul_rn(sgam[b], pst[b * O + an[b] * d + k]));
        const float diff = __fsub_rn(scr[b * d + k], tg);
        gv = __fmul_rn(P.norm, diff);
        nf |= !__builtin_isfinite(diff);
      }
      g3[i] = gv;
      g3m[k * PS_MB + b] = b < B && sab[b] == rank ? gv : 0.f;
    }
    if (__syncthreads_or(nf) && tid == 0 && rank == 0) atomicOr(G.nonfin, 1);
    PS_MARK0(40);
    {  // dX of layer NH (sparse: row b's gradient sits at action a_b) -> dZ_NH, published
      float dx = 0.f;
      const int ab = g < B ? sab[g] : -1;
      if (ab >= 0 && ab < A)
        for (int k = 0; k < d; ++k) dx = __builtin_fmaf(g3[g * d + k], wc3[(ab * d + k) * 8 + j], dx);
      const float z = g < B ? act_bwd(dx, own[(NH * 32 + g) * 8 + j], P.L[NH].act) : 0.f;
      sdz[j * PS_MB + g] = z;
      ps_st(dzh + ((size_t)NH * PS_MB + g) * PS_H + c0 + j, z);
    }
    ps_arrive(hctr);
    ++e;
    PS_MARK0(41);
    if (outr) {  // dW / db + Adam of the output rows of action `rank` (read slot -> write slot)
#pragma unroll 1
      for (int c = 0; c < DC; ++c) {  // rolled: an unrolled DC >= 2 body spills
        float pl[8][3];  // DC >= 2: this chunk's read-slot Adam state, all loads issued up front
        if constexpr (!PO_REG) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const size_t wi = LO.wOff + (size_t)(arow + (8 * c + u < d ? 8 * c + u : 0)) * PS_H + tid;
            pl[u][0] = pon[wi];
            pl[u][1] = mrd[wi];
            pl[u][2] = vrd[wi];
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = 8 * c + u;
          if (k < d) {
            float gw = 0.f;  // rows of other actions hold exact zeros in g3m: the same sum
#pragma unroll
            for (int b = 0; b < PS_MB; b += 4) {
              const float4 gg = *reinterpret_cast<const float4*>(g3m + k * PS_MB + b);
              gw = __builtin_fmaf(gg.x, xc[NH][b], gw);
              gw = __builtin_fmaf(gg.y, xc[NH][b + 1], gw);
              gw = __builtin_fmaf(gg.z, xc[NH][b + 2], gw);
              gw = __builtin_fmaf(gg.w, xc[NH][b + 3], gw);
            }
            float pp, mm, vv;
            if constexpr (PO_REG) {
              pp = po[0][u][0];
              mm = po[0][u][1];
              vv = po[0][u][2];
            } else {
              pp = pl[u][0];
              mm = pl[u][1];
              vv = pl[u][2];
            }
            adam_apply(pp, mm, vv, gw, adc);
            const size_t wi = LO.wOff + (size_t)(arow + k) * PS_H + tid;
            pnew[wi] = pp;
            mwr[wi] = mm;
            vwr[wi] = vv;
            Wno[k * PS_XS + tid] = pp;
          }
        }
      }
      if (tid < d) {
        float gb = 0.f;
#pragma unroll
        for (int b = 0; b < PS_MB; b += 4) {  // other actions' rows and rows past B: exact zeros
          const float4 g4 = *reinterpret_cast<const float4*>(g3m + tid * PS_MB + b);
          gb = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(gb, g4.x), g4.y), g4.z), g4.w);
        }
        float pp = pbo[0], mm = pbo[1], vv = pbo[2];
        adam_apply(pp, mm, vv, gb, adc);
        const size_t bi = LO.bOff + arow + tid;
        pnew[bi] = pp;
        mwr[bi] = mm;
        vwr[bi] = vv;
        nb[(NL - 1) * PS_J + tid] = pp;
      }
    }
    PS_MARK0(42);
    // ---- hidden layers NH .. 1: dX of layer l-1 (published) || dW + Adam of layer l (own rows)
#pragma unroll
    for (int l = NH; l >= 1; --l) {
      if (ok) {
      const PsLayer Ll = P.L[l];
      float* DZ = st;  // [32][PS_XS]
      PS_MARK0(43 + 4 * (NH - l));
      ok = ps_wait(P, hctr, PS_R * e, &s_ok);
      if (ok) {
      ps_stage<8>(dzh + (size_t)l * PS_MB * PS_H, PS_MB, DZ);
      __syncthreads();
      PS_MARK0(44 + 4 * (NH - l));
      {  // dX_{l-1}[g][c0 + j]
        const float dx = ps_dot(DZ + g * PS_XS, WcT + ((l - 1) * PS_J + j) * PS_XS, PS_H);
        const float z = g < B ? act_bwd(dx, own[((l - 1) * 32 + g) * 8 + j], P.L[l - 1].act) : 0.f;
        sdzn[j * PS_MB + g] = z;
        if (l - 1 >= 1) ps_st(dzh + ((size_t)(l - 1) * PS_MB + g) * PS_H + c0 + j, z);
      }
      if (l - 1 >= 1) {
        ps_arrive(hctr);
        ++e;
      } else {
        __syncthreads();
      }
      PS_MARK0(45 + 4 * (NH - l));
      // dW_l[c0 + jj][tid] = Σ_b dZ_l[b][c0 + jj] X_{l-1}[b][tid], db_l; Adam from registers
#pragma unroll
      for (int jj = 0; jj < PS_J; ++jj) {
        float gw = 0.f;  // rows past B hold exact zeros in sdz
#pragma unroll
        for (int b = 0; b < PS_MB; b += 4) {
          const float4 z4 = *reinterpret_cast<const float4*>(sdz + jj * PS_MB + b);
          gw = __builtin_fmaf(z4.x, xc[l - 1][b], gw);
          gw = __builtin_fmaf(z4.y, xc[l - 1][b + 1], gw);
          gw = __builtin_fmaf(z4.z, xc[l - 1][b + 2], gw);
          gw = __builtin_fmaf(z4.w, xc[l - 1][b + 3], gw);
        }
        float pp = pw[l - 1][jj][0], mm = pw[l - 1][jj][1], vv = pw[l - 1][jj][2];
        adam_apply(pp, mm, vv, gw, adc);
        const size_t wi = Ll.wOff + (size_t)(c0 + jj) * PS_H + tid;
        pnew[wi] = pp;
        mwr[wi] = mm;
        vwr[wi] = vv;
        Wn[((l - 1) * PS_J + jj) * PS_XS + tid] = pp;
      }
      if (tid < PS_J) {
        float gb = 0.f;
#pragma unroll
        for (int b = 0; b < PS_MB; b += 4) {  // rows past B: exact zeros (the same sum)
          const float4 z4 = *reinterpret_cast<const float4*>(sdz + tid * PS_MB + b);
          gb = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(gb, z4.x), z4.y), z4.z), z4.w);
        }
        float pp = pb[l][0], mm = pb[l][1], vv = pb[l][2];
        adam_apply(pp, mm, vv, gb, adc);
        const size_t bi = Ll.bOff + c0 + tid;
        pnew[bi] = pp;
        mwr[bi] = mm;
        vwr[bi] = vv;
        nb[l * PS_J + tid] = pp;
      }
      __syncthreads();
      PS_MARK0(46 + 4 * (NH - l));
      sdz[tid] = sdzn[tid];
      __syncthreads();
      }
      }
    }
    if (!ok) break;
    // ---- layer 0: dW0 + Adam of rows c0.., then the post-update forward of S1 ++ s_next
    {
      const PsLayer L0 = P.L[0];
      if (tid < PS_J * n_s) {
        const int jj = tid / n_s, k = tid - jj * n_s;
        float gw = 0.f;
#pragma unroll
        for (int b = 0; b < PS_MB; b += 4) {
          const float4 z4 = *reinterpret_cast<const float4*>(sdz + jj * PS_MB + b);
          gw = __builtin_fmaf(z4.x, sx[b * K0S + k], gw);
          gw = __builtin_fmaf(z4.y, sx[(b + 1) * K0S + k], gw);
          gw = __builtin_fmaf(z4.z, sx[(b + 2) * K0S + k], gw);
          gw = __builtin_fmaf(z4.w, sx[(b + 3) * K0S + k], gw);
        }
        float pp = p0[0], mm = p0[1], vv = p0[2];
        adam_apply(pp, mm, vv, gw, adc);
        const size_t wi = L0.wOff + (size_t)c0 * n_s + tid;
        pnew[wi] = pp;
        mwr[wi] = mm;
        vwr[wi] = vv;
        W0n[jj * K0S + k] = pp;
      }
      if (tid < PS_J) {
        float gb = 0.f;
#pragma unroll
        for (int b = 0; b < PS_MB; b += 4) {  // rows past B: exact zeros (the same sum)
          const float4 z4 = *reinterpret_cast<const float4*>(sdz + tid * PS_MB + b);
          gb = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(gb, z4.x), z4.y), z4.z), z4.w);
        }
        float pp = pb[0][0], mm = pb[0][1], vv = pb[0][2];
        adam_apply(pp, mm, vv, gb, adc);
        const size_t bi = L0.bOff + c0 + tid;
        pnew[bi] = pp;
        mwr[bi] = mm;
        vwr[bi] = vv;
        nb[tid] = pp;
      }
      __syncthreads();
      PS_MARK0(51);
      for (int i = tid; i < (PS_MB + 1) * PS_J; i += 256) {
        const int row = i >> 3, jj = i & 7;
        const float* xr = sx + (row < PS_MB ? 32 + row : 96) * K0S;
        float acc = 0.f;
        for (int k = 0; k < n_s; ++k) acc = __builtin_fmaf(xr[k], W0n[jj * K0S + k], acc);
        ps_st(xvh + (size_t)row * PS_H + c0 + jj, act_fwd(__fadd_rn(acc, nb[jj]), L0.act));
      }
      ps_arrive(hctr);
      ++e;
      PS_MARK(12 + 8 * (r < 6 ? r : 5));
    }
    // ---- post-update forward, hidden layers 1 .. NH (own rows from LDS)
#pragma unroll
    for (int l = 1; l <= NH; ++l) {
      if (ok) {
      const PsLayer Ll = P.L[l];
      float* X = st;  // [33][PS_XS]
      PS_MARK0(53 + 3 * (l - 1));
      ok = ps_wait(P, hctr, PS_R * e, &s_ok);
      if (ok) {
      ps_stage<9>(xvh + (size_t)(l - 1) * (PS_MB + 1) * PS_H, PS_MB + 1, X);
      __syncthreads();
      PS_MARK0(54 + 3 * (l - 1));
      const float bn = nb[l * PS_J + j];
      for (int row = g; row < PS_MB + 1; row += 32) {
        const float y = act_fwd(__fadd_rn(ps_dot(X + row * PS_XS, Wn + ((l - 1) * PS_J + j) * PS_XS, PS_H), bn), Ll.act);
        ps_st(xvh + ((size_t)l * (PS_MB + 1) + row) * PS_H + c0 + j, y);
      }
      ps_arrive(hctr);
      ++e;
      PS_MARK0(55 + 3 * (l - 1));
      }
      }
    }
    if (!ok) break;
    // ---- post-update output layer (rank a < A): this round's maxima for policies > head, selection key
    if (outr) {
      float* X = st;  // [33][PS_XS]
      PS_MARK0(59);
      if (!(ok = ps_wait(P, hctr, PS_R * e, &s_ok))) break;
      PS_MARK(13 + 8 * (r < 6 ? r : 5));
      ps_stage<9>(xvh + (size_t)NH * (PS_MB + 1) * PS_H, PS_MB + 1, X);
      __syncthreads();
      float yv[5];
#pragma unroll
      for (int u = 0; u < 5; ++u) {
        const int i = tid + u * 256;
        const int row = i / d, k = i - row * d;
        yv[u] = i < (PS_MB + 1) * d ? __fadd_rn(ps_dot(X + row * PS_XS, Wno + k * PS_XS, PS_H), nb[(NL - 1) * PS_J + k]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 5; ++u)
        if (tid + u * 256 < (PS_MB + 1) * d) psi[tid + u * 256] = yv[u];
      __syncthreads();
      for (int i = tid; i < T * B; i += 256) {
        const int pi = i / B, b = i - pi * B;
        float q = 0.f;
        for (int k = 0; k < d; ++k) q = __builtin_fmaf(psi[b * d + k], sw[pi * d + k], q);
        qs[pi * PS_MB + b] = q;
        if (pi > head)
          __hip_atomic_fetch_max(xqn + (pi * PS_MB + b) * A + rank, sortable(q), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
      if (tid == 0) {
        qkey = 0ull;
        if (P.nsel && (P.sel_use_gpi || head == P.task)) {
          float q = 0.f;
          for (int k = 0; k < d; ++k) q = __builtin_fmaf(psi[PS_MB * d + k], sw[P.task * d + k], q);
          qkey = ((unsigned long long)ps_ukey(q) << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)(head * A + rank));
          __hip_atomic_fetch_max(sel + r + 1, qkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      ps_arrive(qctr);
      PS_MARK(14 + 8 * (r < 6 ? r : 5));
    }
  }
  // ---------------- commit and publish
  PS_MARK(62);
  __syncthreads();
  if (tid == 0) s_flag = __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (work && ok && s_flag == 0 && rank == 0 && tid == 0) G.step[head] = step0 + 1;
  if (active && rank == 0 && head == 0 && tid == 0) {
    const int err = __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long c = -1, a = -1;
    int flag = T;
    if (cancelled) {
      flag = T;
    } else if (!ok || err) {
      flag = -1;
    } else {
      if (P.lms_task >= 0)
        for (int k = 0; k < d; ++k) G.w[(long long)P.lms_task * G.dpad + k] = sw[P.lms_task * d + k];
      if (P.nsel) {
        const unsigned long long key = __hip_atomic_load(sel + rounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned idx = 0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull);
        c = idx / (unsigned)A;
        a = idx % (unsigned)A;
      }
      __hip_atomic_fetch_add(P.stats, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(P.stats + 1, (unsigned long long)rounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    P.sel_out[0] = c;
    P.sel_out[1] = a;
    *P.flag = flag;
    if (P.pub) {
      const long long seq = *P.pub_dctr;
      HostResult* out = P.pub + (seq & (RES_RING - 1));
      out->sel0 = c;
      out->sel1 = a;
      out->flag = flag;
      out->cancelled = cancelled;
      out->nonfinite = __hip_atomic_load(G.nonfin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // the last workgroup out advances the launch counter (the next launch takes the other set)
  __syncthreads();
  PS_MARK(63);
  if (tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(fin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1)
      __hip_atomic_store(P.epoch, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Placement census (host check before the persistent step is used): per XCC_ID, how many of a
// 256-workgroup launch with k_pstep's LDS footprint landed there.
__global__ __launch_bounds__(256) void k_pstep_census(unsigned* counts) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (threadIdx.x == 0) {
    sm[0] = 0.f;
    atomicAdd(counts + (ps_xcc() & 15), 1u);
  }
}

}  // namespace sfx

// Host-side workspace of the persistent step (sfx_pstep.inc; global, like the other handle states)
struct sfx_pstep_state {
  float* fbuf = nullptr;  // xs | psit | cr | dzb | xv
  float *xs = nullptr, *psit = nullptr, *cr = nullptr, *dzb = nullptr, *xv = nullptr;
  int* ibuf = nullptr;  // xq [2][...] | xge [2][...]
  int *xq = nullptr, *xge = nullptr;
  size_t nxq = 0, nxge = 0;
  unsigned long long* sel = nullptr;    // [2][PS_RMAX]
  unsigned* cnt = nullptr;              // [2][PS_CSET] | epoch | err
  unsigned long long* stats = nullptr;  // [4]
  int* trace = nullptr;                 // [PS_RMAX][8][PS_MB + 1] + the last launch's converged round
  long long* timeline = nullptr;        // SFX_PSTEP_PROBE=1: [8][PS_TL]
  int lds_floats = 0;
  sfx::PsArgs base{};  // geometry and LDS carve
};
