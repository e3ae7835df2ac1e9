// sfx_tsf.h -- TSF-DQN's transformed features (tsfdqn.py:588-709, tsfdqn_nf.py): device side.
//
// Per task i a state transform g_i (K planar flows z <- z + u_k tanh(w_k·z + b_k), then
// Linear(n_s, G); K = 0 is tsfdqn.py's plain Linear) and ONE affine map h = Linear(G, d) shared
// by all tasks give the transformed features
//     φ̃ = (h(g_i(s)) + h(g_i(s1))) ⊙ φ
// which replace φ in the TD target (t = φ̃ + γ ψ⁻_i(s1)[a'], so l1 trains g_i and h too) and in
// l2 = MSE(w_i·φ̃, r); loss = l1 + β l2 and one Adam step over {ψ_i, w_i, g_i, h}.
//
// The ψ part runs through the SF-DQN kernels with φ̃ as the features; these kernels do the rest:
//   k_tsf_fwd<NP>   before the TD target: φ̃, the saved flow states / tanh outputs / g features,
//                   and a snapshot of g_i, h, w_i as they were before the step.  A workgroup
//                   owns TSF_PB batch indices (their s and s1 rows); a row's planar-flow chain
//                   runs in ONE lane (z in NP registers, w_k·z as packed FMAs in three
//                   independent chains, flow parameters as wave-uniform scalar loads), so a
//                   flow step holds no cross-lane reduction.  NP = n_s rounded up to 4.
//   k_tsf_bwd<NP>   after the ψ backward, one launch of four workgroup roles that all read the
//                   snapshot (so no role sees another's Adam writes):
//                     flow rows  TSF_FR rows each: dg, then the reverse flow chain, one lane per
//                                row, the flow states staged in LDS; each row's terms of the
//                                flow-parameter gradients into `part`
//                     h          256 parameters of the shared h each: gradient + Adam
//                     g-Linear   TSF_QS output columns of g_i's Linear each: dg, gradient + Adam
//                     w          l2, the w_i gradient + Adam, the loss row
//   k_tsf_flow      flow parameters: sum of the per-row terms (fixed order) + Adam (K > 0).
// Limits (checked by sfx_tsf_setup): n_s <= 32, B <= 64, d <= 128, G <= 256, d*G4 <= 8192 (G4: G
// rounded up to 4), 2B*G <= 8192, B*d <= 4096, K(2 n_s + 1) + G(n_s + 1) <= 4096, G*NP <= 4096,
// K tsf_fst(NP) <= TSF_FA, and the flow-row staging TSF_FR K <= TSF_TS, TSF_FR G <= 2048,
// TSF_FR d <= 2048.
#pragma once

namespace sfx {

constexpr int TSF_NS = 32;     // max n_s
constexpr int TSF_LDS = 8192;  // floats per staged operand (flows, W_h, g features)
constexpr int TSF_TS = 1024;   // tanh outputs staged per flow-row workgroup: TSF_FR x K
constexpr int TSF_QS = 16;     // g-Linear output columns per backward workgroup
constexpr int TSF_PB = 8;      // forward: batch indices per workgroup (2 TSF_PB flow rows)
constexpr int TSF_FR = 8;      // backward: flow rows per flow-row workgroup
constexpr int TSF_SCR = 64 * TSF_NS;  // TsfArgs::scratch floats (one row per chain lane)
constexpr int TSF_FA = 8192;   // flows staged in the chain layout: K x tsf_fst(NP)
constexpr int TSF_SM = TSF_TS + TSF_LDS / 2 + TSF_LDS + 3 * 2048 + TSF_FA;  // k_tsf_bwd LDS (floats)

// NP: n_s rounded up to a power of two >= 4 -- the width of a flow row (spread over tsf_lpr(NP)
// lanes) and the row stride of the saved flow states (zs [K+1][2B][NP], 16-byte rows); the per-row gradient terms `part` are
// [K][2B][tsf_pst(NP)]: dz_{k+1} (the gradient reaching z_{k+1}) at [0, NP), da_k at NP --
// k_tsf_flow forms the w / u terms da_k z_k and dz_{k+1} t_k from them and the saved states.
__host__ __device__ constexpr int tsf_np(int n_s) { return n_s <= 4 ? 4 : n_s <= 8 ? 8 : n_s <= 16 ? 16 : 32; }
// lanes per flow row (each holds NP / lanes = 4 or 8 state components)
__host__ __device__ constexpr int tsf_lpr(int np) { return np / 4 < 4 ? np / 4 : 4; }
__host__ __device__ constexpr int tsf_pst(int np) { return np + 4; }
// a flow in the chain layout (LDS): w at [0, NP), u at [NP, 2NP), b at 2NP, c at 2NP + 1, zeros
// elsewhere
__host__ __device__ constexpr int tsf_fst(int np) { return 2 * np + 4; }

struct TsfArgs {
  int pol, B, n_s, G, K, d, Pg, Ph, O, lastOff;
  float beta;
  int nflow, nh, nlin;  // k_tsf_bwd roles: flow-row / h / g-Linear workgroups, then one w workgroup
  int np;               // tsf_np(n_s)
  int fwd_mode;         // the forward: 0 whole, 1 staging + chains + images (no Linear / φ̃), 2 Linear + φ̃ only
  int pad_m_;
  const float* S;
  const float* S1;
  const float* phi;
  const float* r;
  const int64_t* a;
  float* g;  // [T][Pg]: flow k at k*(2n_s+1) (w[n_s], b, u[n_s]); Linear W[G][n_s] at K*(2n_s+1), then b[G]
  // [T][K][tsf_fst(NP)]: the same flows in the chain layout (zeros in the padding), kept by every
  // writer of g's flows (the flows' Adam in tsf_flow_block, the host loads): the forward and the
  // backward's flow rows stage it with one contiguous 16-byte LDS-DMA.  The c slots hold the
  // look-ahead coefficients of the last forward (which the backward after it uses as they are)
  float* gch;
  float* gm;
  float* gv;
  float* hp;  // [Ph]: W_h[d][G] then b_h[d]
  float* hm;  // [T][Ph] (each task's optimizer keeps its own moments of the shared h)
  float* hv;
  float* zs;     // [K+1][2B][NP] flow states (rows 0..B-1: s, B..2B-1: s1)
  float* ts;     // tanh outputs [2B / TSF_FR groups][K][TSF_FR]: a backward flow-row workgroup's block is contiguous (tsf_ts_at)
  float* gfeat;  // [2B][G]
  float* tphi;   // [B][d]
  float* part;   // [K][2B][tsf_pst(NP)] per-row flow gradients (dz_{k+1}, da_k)
  float* scratch;  // [TSF_SCR]: stores of flow-chain lanes past the batch (never read)
  float* bimg;   // [NP][G4] W_l transposed, then [G][D4] W_h transposed: the pre-step values, written by the
                 // forward for the backward's flow rows (one contiguous LDS-DMA there)
  float* snap;   // [Pg + Ph + d]: g_i, h, w_i before this step (written by k_tsf_fwd)
  float* losses; // [3]: [1] = l1 (written by the ψ tail); [0], [2] written here
  const float* dzlast;  // output gradient of the policy's ψ head [B][O] (written by K2)
  const int* step;      // Adam step of the policy (already bumped by the ψ path)
  const int* cancel;    // runner steps: the gate's cancel word (Geo::cancel); no commit when set
  float* w;             // [d] reward weights of the policy (+ moments; its global row when sharded)
  float* wm;
  float* wv;
  AdamHP hpw, hpg, hph;
  AdamHP hpf;  // the planar flows' Adam (hpg, or lr = 0 when frozen: sfx_tsf_freeze_flows)
};

__device__ __forceinline__ int tsf_flow_stride(int n_s) { return 2 * n_s + 1; }
// tanh output t_k of flow row `row` in TsfArgs::ts
__host__ __device__ __forceinline__ long long tsf_ts_at(int row, int k, int K) {
  return ((long long)(row / TSF_FR) * K + k) * TSF_FR + row % TSF_FR;
}

// LDS carve of the backward roles (float offsets, 16-byte aligned), from the geometry: the
// flow-row role, the h / g-Linear / w roles and k_tsf_flow's flows each start at 0 of the same
// buffer.  k_tsf_bwd holds TSF_SM floats (enough for every geometry sfx_tsf_setup accepts);
// k_bwd_tsf, which shares its workgroups' LDS with the ψ backward tiles, holds TSFX_SM, and the
// host rides the TSF backward along only when the carve fits (tsf_bwd_lds(...).total).
constexpr int TSFX_SM = 20480;
__host__ __device__ constexpr int tsf_r4(int n) { return (n + 3) & ~3; }
__host__ __device__ constexpr int tsf_imax(int a, int b) { return a > b ? a : b; }
struct TsfBwdLds {
  int t, wlT, whT, dg, da, gc, fa, flow_total;  // flow-row role
  int rda, rgf, rzk, rtp, rgc, rdg, role_total;  // h / g-Linear / w roles
  int fdz, fda, ft, fk_total;                    // k_tsf_flow (s_z at 0)
  int total;
};
__host__ __device__ inline TsfBwdLds tsf_bwd_lds(int K, int np, int G, int d, int B) {
  TsfBwdLds L{};
  const int FR = TSF_FR, G4 = tsf_r4(G), D4 = tsf_r4(d), R2 = 2 * B;
  int o = 0;
  L.t = o;   o += tsf_r4(K * FR);
  L.wlT = o; o += np * G4;
  L.whT = o; o += G * D4;
  L.dg = o;  o += tsf_r4(tsf_imax(FR * G4, FR * d));  // φ̃ rows while staging
  L.da = o;  o += tsf_r4(FR * d);
  L.gc = o;  o += tsf_imax(FR * D4, FR * np);
  L.fa = o;  o += K * tsf_fst(np);
  L.flow_total = K > 0 ? o : 0;
  o = 0;
  L.rda = o; o += tsf_r4(B * d);
  L.rgf = o;                                            // h role: [2B][G]; g-Linear: W_h columns, z_K
  L.rzk = o + tsf_r4(d * TSF_QS);
  o += tsf_imax(tsf_r4(R2 * G), tsf_r4(d * TSF_QS) + R2 * np);
  L.rtp = o; o += tsf_r4(B * d);
  L.rgc = o; o += tsf_r4(B * d);
  L.rdg = o; o += B * TSF_QS;
  L.role_total = o;
  L.fdz = R2 * np;
  L.fda = 2 * R2 * np;
  L.ft = L.fda + tsf_r4(R2);
  L.fk_total = K > 0 ? L.ft + tsf_r4(R2) : 0;
  L.total = tsf_imax(tsf_imax(L.flow_total, L.role_total), L.fk_total);
  return L;
}

// LDS carve of k_tsf_fwd (float offsets, 16-byte aligned), from the geometry; k_fwd_tsf (the
// forward riding along in the ψ forward's first launch) holds TSFXF_SM floats of it.
constexpr int TSFXF_SM = 20480;
struct TsfFwdLds {
  int fa, wl, wh, gf, z, ph, bl, bh, total;
};
__host__ __device__ inline TsfFwdLds tsf_fwd_lds(int K, int np, int G, int d) {
  TsfFwdLds L{};
  const int GP = tsf_r4(G), RPW = 2 * TSF_PB;
  int o = 0;
  L.fa = o; o += K * tsf_fst(np);  // flows, chain layout
  L.wl = o; o += G * (np + 4);     // Linear of g: [G][NP + 4] (the padded stride: conflict-free b128 reads)
  L.wh = o; o += d * GP;           // W_h: [d][GP]
  L.gf = o; o += RPW * GP;         // g features [RPW][GP]
  L.z = o;  o += RPW * np;         // z_K rows [RPW][NP]
  L.ph = o; o += tsf_r4(TSF_PB * d);  // φ rows [PB][d]
  L.bl = o; o += tsf_r4(G);
  L.bh = o; o += tsf_r4(d);
  L.total = o;
  return L;
}
// LDS carve of the forward's tail alone (tsf_fwd_tail): W_l transposed [NP][GP], W_h [d][GP], g
// features [RPW][GP], the z_K rows, φ rows, b_l, b_h
struct TsfTailLds {
  int wlT, wh, gf, z, ph, bl, bh, total;
};
__host__ __device__ inline TsfTailLds tsf_tail_lds(int np, int G, int d) {
  TsfTailLds L{};
  const int GP = tsf_r4(G), RPW = 2 * TSF_PB;
  int o = 0;
  L.wlT = o; o += np * GP;
  L.wh = o;  o += d * GP;
  L.gf = o;  o += RPW * GP;
  L.z = o;   o += RPW * np;
  L.ph = o;  o += tsf_r4(TSF_PB * d);
  L.bl = o;  o += tsf_r4(G);
  L.bh = o;  o += tsf_r4(d);
  L.total = o;
  return L;
}
constexpr int TSF_FWD_SM = TSF_FA + TSF_LDS / 2 + TSF_LDS + TSF_LDS / 2 + 2 * TSF_PB * TSF_NS + 1024 + 512;

// tanh without branches: for |x| < 0.625 the same odd minimax polynomial (same coefficients,
// same operation order) as the device library's tanhf, else 1 − 2 / (e^{2|x|} + 1) by v_exp /
// v_rcp; both are evaluated and selected, so a flow step's chain has no exec-mask branches.
__device__ __forceinline__ float tsf_tanh(float x) {
  const float ax = fabsf(x), x2 = __fmul_rn(x, x);
  float p = __builtin_fmaf(x2, __int_as_float(0xbbbac73d), __int_as_float(0x3ca908c9));
  p = __builtin_fmaf(x2, p, __int_as_float(0xbd5c1c4e));
  p = __builtin_fmaf(x2, p, __int_as_float(0x3e088382));
  p = __builtin_fmaf(x2, p, __int_as_float(0xbeaaaa99));
  const float small = __builtin_fmaf(x2, __fmul_rn(ax, p), ax);
  const float e = __expf(__fadd_rn(ax, ax));
  const float large = __builtin_fmaf(__builtin_amdgcn_rcpf(__fadd_rn(e, 1.f)), -2.f, 1.f);
  return copysignf(ax < 0.625f ? small : large, x);
}

typedef float tsf_f2 __attribute__((ext_vector_type(2)));
typedef float tsf_f4 __attribute__((ext_vector_type(4)));

// A flow row runs on LPR = tsf_lpr(NP) neighbouring lanes, lane j holding NL = NP / LPR
// components [j NL, (j+1) NL) of the state.  One planar flow's parameters as lane j needs them
// (chain layout, tsf_fst): its parts of w and u, b and the look-ahead coefficient
// c_k = w_{k+1}·u_k; LDS reads at the same addresses for every row (broadcast), 16 bytes at a time.
template <int NL>
struct TsfFlow {
  float w[NL], u[NL], b, c;
};

template <int NL, int NP>
__device__ __forceinline__ void tsf_flow_ld(TsfFlow<NL>& F, const float* f, int j) {
  const float* fw = f + j * NL;
  const float* fu = f + NP + j * NL;
#pragma unroll
  for (int q = 0; q < NL / 4; ++q) {
    const tsf_f4 w4 = *(const tsf_f4*)(fw + 4 * q), u4 = *(const tsf_f4*)(fu + 4 * q);
    F.w[4 * q] = w4.x; F.w[4 * q + 1] = w4.y; F.w[4 * q + 2] = w4.z; F.w[4 * q + 3] = w4.w;
    F.u[4 * q] = u4.x; F.u[4 * q + 1] = u4.y; F.u[4 * q + 2] = u4.z; F.u[4 * q + 3] = u4.w;
  }
  const tsf_f2 bc = *(const tsf_f2*)(f + 2 * NP);
  F.b = bc.x;
  F.c = bc.y;
}

// this lane's part of x·y: NL/2 packed FMAs in (up to) three independent chains
template <int NL>
__device__ __forceinline__ float tsf_dot(const tsf_f2 (&x)[NL / 2], const float (&y)[NL]) {
  tsf_f2 c0 = {0.f, 0.f}, c1 = {0.f, 0.f}, c2 = {0.f, 0.f};
#pragma unroll
  for (int p = 0; p < NL / 2; ++p) {
    const tsf_f2 yy = {y[2 * p], y[2 * p + 1]};
    if (p % 3 == 0)
      c0 = __builtin_elementwise_fma(x[p], yy, c0);
    else if (p % 3 == 1)
      c1 = __builtin_elementwise_fma(x[p], yy, c1);
    else
      c2 = __builtin_elementwise_fma(x[p], yy, c2);
  }
  return __fadd_rn(__fadd_rn(__fadd_rn(c0.x, c0.y), __fadd_rn(c1.x, c1.y)), __fadd_rn(c2.x, c2.y));
}

// the row's full sum from its LPR lanes' parts (DPP quad_perm xor 1, then xor 2: every lane of
// the row gets the same value, as IEEE addition commutes)
template <int LPR>
__device__ __forceinline__ float tsf_row_sum(float v) {
  if (LPR >= 2) v = __fadd_rn(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  if (LPR >= 4) v = __fadd_rn(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  return v;
}

// x += s·y (packed)
template <int NL>
__device__ __forceinline__ void tsf_axpy(tsf_f2 (&x)[NL / 2], float s, const float (&y)[NL]) {
  const tsf_f2 ss = {s, s};
#pragma unroll
  for (int p = 0; p < NL / 2; ++p) x[p] = __builtin_elementwise_fma((tsf_f2){y[2 * p], y[2 * p + 1]}, ss, x[p]);
}

// dst[0, NL) = x (16-byte stores)
template <int NL>
__device__ __forceinline__ void tsf_store(float* dst, const tsf_f2 (&x)[NL / 2]) {
#pragma unroll
  for (int q = 0; q < NL / 4; ++q) *(tsf_f4*)(dst + 4 * q) = (tsf_f4){x[2 * q].x, x[2 * q].y, x[2 * q + 1].x, x[2 * q + 1].y};
}

// c_k = w_{k+1}·u_k (c_{K-1} = 0) into the chain layout, by ALL 64 lanes of one wave (lane per
// flow); the wave's own later LDS reads see these stores (in-order LDS queue per wave)
template <int NP>
__device__ __forceinline__ void tsf_lookahead(float* s_fa, int K) {
  constexpr int FA = tsf_fst(NP);
  for (int k = threadIdx.x & 63; k < K; k += 64) {
    float c = 0.f;
    if (k + 1 < K)
      for (int i = 0; i < NP; ++i) c = __builtin_fmaf(s_fa[(k + 1) * FA + i], s_fa[k * FA + NP + i], c);
    s_fa[k * FA + 2 * NP + 1] = c;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a·b over n4 16-byte groups of two LDS rows, four independent lanes of accumulation
__device__ __forceinline__ float tsf_dot4(const float* a, const float* b, int n4) {
  tsf_f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int q = 0; q < n4; ++q) acc = __builtin_elementwise_fma(*(const tsf_f4*)(a + 4 * q), *(const tsf_f4*)(b + 4 * q), acc);
  return __fadd_rn(__fadd_rn(acc.x, acc.y), __fadd_rn(acc.z, acc.w));
}

// glds16_rows: rows of 16-byte groups, dst[r][4 g .. 4 g + 3] = src[r * stride + 4 g ..] for r <
// rows, g < row4 (dst dense; src rows 16-byte aligned), by the workgroup's first four waves;
// completes at the caller's next __syncthreads()
__device__ __forceinline__ void glds16_rows(float* dst, const float* src, int rows, int stride, int row4) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, n4 = rows * row4;
  if (wv >= 4) return;
  for (int c = wv; c * 64 < n4; c += 4) {
    const int e = c * 64 + lane;
    if (e < n4) {
      const int r = e / row4, g = e - r * row4;
      __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)r * stride + 4 * g), (tsf_lds_t)(dst + c * 256), 16,
                                       0, 0);
    }
  }
}

// glds / tsf_lds_t (LDS-DMA staging): sfx_kernels.h.  glds16: a contiguous copy of n4 16-byte
// groups (16-byte aligned source and destination) by global_load_lds_dwordx4, one KB per wave
// instruction, by waves [w0, w0 + nw); completes at the caller's next __syncthreads()
__device__ __forceinline__ void glds16(float* dst, const float* src, int n4, int w0 = 0, int nw = 4) {
  const int lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) - w0;
  if (wv < 0 || wv >= nw) return;
  for (int c = wv; c * 64 < n4; c += nw)
    if (c * 64 + lane < n4)
      __builtin_amdgcn_global_load_lds((const void*)(src + 4 * (c * 64 + lane)), (tsf_lds_t)(dst + c * 256), 16, 0, 0);
}

// Rows [0, n) of the minibatch (row rl is batch index bmap(rl)), staged for the backward roles:
// φ̃ and φ rows, r, the taken actions, the pre-step w_i, then (second round trip) the taken
// action's row of the ψ output gradient; dr_b = β (2/B) (w·φ̃_b − r_b) and
//   daff[b][c] = (−∂l1/∂t[b][c] + dr_b w_c) φ[b][c]
// (the gradient reaching h's output through the TD targets and through w·φ̃).  Returns this
// thread's share of Σ_b (w·φ̃_b − r_b)² (l2 numerator).  Callers may have staging loads of their
// own in flight; the first barrier here retires them too.  Ends with a barrier.
template <class BMap>
__device__ float tsf_stage_daff(const TsfArgs& A, int n, BMap bmap, float* s_tp, float* s_da, float* s_gc,
                                float* s_dr, float* s_w, float* s_r, int* s_ab) {
  const int tid = threadIdx.x, d = A.d, O = A.O;
  const float* wold = A.snap + A.Pg + A.Ph;
  const FDiv fd = fdiv(d);
  float rv = 0.f;
  int av = 0;
  if (tid < n) {
    const int b = bmap(tid);
    rv = A.r[b];
    av = (int)A.a[b];
  }
  glds(s_w, d, [&](int j) { return wold + j; });
  glds(s_tp, n * d, [&](int j) { const int rl = j / fd; return A.tphi + (size_t)bmap(rl) * d + (j - rl * d); });
  glds(s_da, n * d, [&](int j) { const int rl = j / fd; return A.phi + (size_t)bmap(rl) * d + (j - rl * d); });
  if (tid < n) {
    s_r[tid] = rv;
    s_ab[tid] = av;
  }
  __syncthreads();
  PROBE_AT(5);
  glds(s_gc, n * d, [&](int j) {
    const int rl = j / fd, ab = s_ab[rl];
    return (ab >= 0 && ab * d < O) ? A.dzlast + (size_t)bmap(rl) * O + ab * d + (j - rl * d) : A.dzlast;
  });
  float se = 0.f;
  const float bnorm = __fmul_rn(A.beta, (float)(2.0 / (double)A.B));
  if (tid < n) {
    float rf = 0.f;
    for (int j = 0; j < d; ++j) rf = __builtin_fmaf(s_tp[tid * d + j], s_w[j], rf);
    const float e = __fsub_rn(rf, s_r[tid]);
    se = __fmul_rn(e, e);
    s_dr[tid] = __fmul_rn(bnorm, e);
  }
  __syncthreads();
  PROBE_AT(6);
  for (int j = tid; j < n * d; j += 256) {
    const int rl = j / fd, c = j - rl * d, ab = s_ab[rl];
    const float gc = (ab >= 0 && ab * d < O) ? s_gc[j] : 0.f;
    const float dt = __fadd_rn(-gc, __fmul_rn(s_dr[rl], s_w[c]));
    s_da[j] = __fmul_rn(dt, s_da[j]);
  }
  __syncthreads();
  return se;
}

// grid cdiv(B, TSF_PB), 256 threads; TSF_PB batch indices (their s rows and s1 rows) per WG.
// gfl = A.g + pol Pg (g_i).
//   A  all waves: the flows into LDS (chain layout), then c_k = w_{k+1}·u_k;
//   B  wave 0, one lane per row: the planar-flow chain.  With q_{k+1} = w_{k+1}·z_k + b_{k+1}
//      (known before t_k) the next pre-activation is a_{k+1} = q_{k+1} + t_k c_k, so a flow
//      step's critical path is tanh + one FMA; z_{k+1} = z_k + u_k t_k and the stores of z_k, t_k
//      run beside it.  Waves 1-3 meanwhile stage the Linear of g, W_h, b_h and φ, and write the
//      snapshot of g_i, h, w_i (read by k_tsf_bwd) from global memory;
//   C  Linear(n_s, G) of g for the workgroup's rows, then φ̃ = (h(g(s)) + h(g(s1))) ⊙ φ.
// workgroup blk of nblk (threads past 256 of a wider workgroup -- k_fwd_tsf's -- only join the
// barriers); sm holds tsf_fwd_lds(...).total floats
template <int NP>
__device__ __forceinline__ void tsf_fwd_tail(const TsfArgs& A, const float* __restrict__ gfl, float* sm, int blk);

template <int NP>
__device__ __forceinline__ void tsf_fwd_body(const TsfArgs& A, const float* __restrict__ gfl, float* sm, int blk,
                                             int nblk) {
  if (A.fwd_mode == 2) {
    tsf_fwd_tail<NP>(A, gfl, sm, blk);
    return;
  }
  constexpr int PB = TSF_PB, RPW = 2 * PB, FA = tsf_fst(NP), WLS = NP + 4;  // WLS: s_wl's row stride
  const int tid = threadIdx.x, n_s = A.n_s, G = A.G, K = A.K, d = A.d, B = A.B, R2 = 2 * B;
  const int fs = tsf_flow_stride(n_s), nfl = K * fs, GP = (G + 3) & ~3;
  const TsfFwdLds L = tsf_fwd_lds(K, NP, G, d);
  float *s_fa = sm + L.fa, *s_wl = sm + L.wl, *s_wh = sm + L.wh, *s_gf = sm + L.gf, *s_z = sm + L.z;
  float *s_ph = sm + L.ph, *s_bl = sm + L.bl, *s_bh = sm + L.bh;
  const int b0 = blk * PB, nb = min(PB, B - b0);
  __shared__ int s_sync;  // waves 1-3 meet on it before writing the backward's image
  if (tid == 0) s_sync = 0;
  PROBE_T(t0_);
  glds16(s_fa, A.gch + (size_t)A.pol * K * FA, K * FA / 4);  // the flows, chain layout
  // flow row rl = tid / LPR on lanes [LPR rl, LPR rl + LPR) (components [hf NL, hf NL + NL) each):
  // rows 0..PB-1 the s rows of batch indices b0.., PB.. the s1 rows
  constexpr int LPR = tsf_lpr(NP), NL = NP / LPR;
  const int rl = tid / LPR, hf = tid % LPR;
  const bool s1row = rl >= PB;
  const int b = b0 + (s1row ? rl - PB : rl);
  const bool valid = rl < RPW && b < B;
  const int row = s1row ? B + b : b;
  tsf_f2 z[NL / 2];
  if (rl < RPW) {
    const float* src = (s1row ? A.S1 : A.S) + (size_t)(valid ? b : 0) * n_s;
#pragma unroll
    for (int p = 0; p < NL / 2; ++p) {
      const int i = hf * NL + 2 * p;
      z[p] = (tsf_f2){valid && i < n_s ? src[i] : 0.f, valid && i + 1 < n_s ? src[i + 1] : 0.f};
    }
  }
  PROBE_AT(4);
  __syncthreads();
  PROBE_AT(5);
  if (tid < 64) {
    tsf_lookahead<NP>(s_fa, K);
    // the coefficients into the chain-layout copy too: the backward's flow rows read these flows
    // (its own launch comes before their Adam step) with c already in place
    if (blk == 0)
      for (int k = tid; k < K; k += 64)
        A.gch[((size_t)A.pol * K + k) * FA + 2 * NP + 1] = s_fa[k * FA + 2 * NP + 1];
    if (rl < RPW) {
      // rows past the batch write their (unused) states to a scratch row, so the loop body is one
      // basic block: the LDS reads for step k + 2 issue at its top
      float* zrow = valid ? A.zs + (size_t)row * NP + hf * NL : A.scratch + rl * TSF_NS + hf * NL;
      float* trow = valid ? A.ts + tsf_ts_at(row, 0, K) : A.scratch + rl * TSF_NS + NP;  // both lanes: the same t
      const size_t zstep = valid ? (size_t)R2 * NP : 0, tstep = valid ? (size_t)TSF_FR : 0;
      PROBE_AT(1);
      // flows k (F0) and k + 1 (F1) in registers; flow k + 2's LDS reads are issued a full step
      // before their use
      TsfFlow<NL> F0, F1, F2;
      float a = 0.f;
      if (K > 0) {
        tsf_flow_ld<NL, NP>(F0, s_fa, hf);
        tsf_flow_ld<NL, NP>(F1, s_fa + min(1, K - 1) * FA, hf);
        a = __fadd_rn(tsf_row_sum<LPR>(tsf_dot<NL>(z, F0.w)), F0.b);
      }
      // one flow step: Fa = flow k, Fb = flow k + 1, Fc <- flow k + 2; the loop rotates the three
      // register sets by name (unrolled by 3), so no step copies parameters
      auto step = [&](const TsfFlow<NL>& Fa, const TsfFlow<NL>& Fb, TsfFlow<NL>& Fc, int k) {
        // w_{k+1}·z_k + b_{k+1}: off the critical path
        const float q = __fadd_rn(tsf_row_sum<LPR>(tsf_dot<NL>(z, Fb.w)), Fb.b);
        // flow k + 2's reads go out after the dot has read flow k + 1, so the wait for flow k + 1's
        // reads (issued a step ago) does not also wait for these
        tsf_flow_ld<NL, NP>(Fc, s_fa + min(k + 2, K - 1) * FA, hf);
        const float t = tsf_tanh(a);
        tsf_store<NL>(zrow, z);
        *trow = t;
        zrow += zstep;
        trow += tstep;
        a = __builtin_fmaf(t, Fa.c, q);
        tsf_axpy<NL>(z, t, Fa.u);
      };
      // K mod 3 steps first, then groups of three with no exit between their steps (an exit
      // branch lets the compiler sink each step's flow reads past it, next to their use)
      int k = 0;
      const int rem = K % 3;
      if (rem == 0) {
        for (; k < K; k += 3) {
          step(F0, F1, F2, k);
          step(F1, F2, F0, k + 1);
          step(F2, F0, F1, k + 2);
        }
      } else if (rem == 1) {
        step(F0, F1, F2, k++);
        for (; k < K; k += 3) {
          step(F1, F2, F0, k);
          step(F2, F0, F1, k + 1);
          step(F0, F1, F2, k + 2);
        }
      } else {
        step(F0, F1, F2, k++);
        step(F1, F2, F0, k++);
        for (; k < K; k += 3) {
          step(F2, F0, F1, k);
          step(F0, F1, F2, k + 1);
          step(F1, F2, F0, k + 2);
        }
      }
      tsf_store<NL>(zrow, z);
      tsf_store<NL>(s_z + rl * NP + hf * NL, z);
      PROBE_AT(2);
    }
  } else if (tid < 256) {
    const FDiv fws = fdiv(WLS), fgp = fdiv(GP);
    const float* Wl = gfl + nfl;
    glds(s_wl, G * WLS, [&](int j) -> const float* {
      const int c = j / fws, i = j - c * WLS;
      return i < n_s ? Wl + c * n_s + i : nullptr;
    }, 1, 3);
    glds(s_bl, G, [&](int j) { return Wl + G * n_s + j; }, 1, 3);
    glds(s_wh, d * GP, [&](int j) -> const float* {
      const int c = j / fgp, q = j - c * GP;
      return q < G ? A.hp + c * G + q : nullptr;
    }, 1, 3);
    glds(s_bh, d, [&](int j) { return A.hp + d * G + j; }, 1, 3);
    glds(s_ph, nb * d, [&](int j) { return A.phi + (size_t)b0 * d + j; }, 1, 3);
    // this workgroup's slice of the pre-step snapshot of g_i, h, w_i
    const int S = A.Pg + A.Ph + d, per = (S + nblk - 1) / nblk;
    const int lo = blk * per, hi = min(S, lo + per);
    for (int j = lo + tid - 64; j < hi; j += 192)
      A.snap[j] = j < A.Pg ? gfl[j] : (j < A.Pg + A.Ph ? A.hp[j - A.Pg] : A.w[j - A.Pg - A.Ph]);
    // this workgroup's slice of the backward flow rows' staging image (TsfArgs::bimg): W_l and W_h
    // transposed, from the LDS copies once every one of waves 1-3 has landed its part of them (a
    // wave's own LDS-DMA is complete at its vmcnt(0); the waves meet on an LDS counter -- wave 0 is
    // in the flow chain)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((tid & 63) == 0) __hip_atomic_fetch_add(&s_sync, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&s_sync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 3) __builtin_amdgcn_s_sleep(1);
    const int D4 = (d + 3) & ~3, nwl = NP * GP, nimg = nwl + G * D4;
    const int ip = (nimg + nblk - 1) / nblk, ilo = blk * ip, ihi = min(nimg, ilo + ip);
    const FDiv fd4 = fdiv(D4);
    for (int j = ilo + tid - 64; j < ihi; j += 192) {
      float v;
      if (j < nwl) {
        const int i = j / fgp, q = j - i * GP;
        v = q < G ? s_wl[q * WLS + i] : 0.f;
      } else {
        const int jj = j - nwl, q = jj / fd4, c = jj - q * D4;
        v = c < d ? s_wh[c * GP + q] : 0.f;
      }
      A.bimg[j] = v;
    }
  }
  __syncthreads();
  if (A.fwd_mode == 1) {  // the Linear and φ̃ run later, in the selection launch (tsf_fwd_tail)
    PROBE_REC(10, t0_);
    return;
  }
  if (tid < 256) {  // Linear(n_s, G) of g for this workgroup's rows (columns past G: zero)
    const FDiv fgp = fdiv(GP);
    for (int j = tid; j < RPW * GP; j += 256) {
      const int r = j / fgp, c = j - r * GP;
      float v = 0.f;
      if (c < G) {
        v = __fadd_rn(tsf_dot4(s_z + r * NP, s_wl + c * WLS, NP / 4), s_bl[c]);
        const int bb = b0 + (r >= PB ? r - PB : r);
        if (bb < B) A.gfeat[(size_t)(r >= PB ? B + bb : bb) * G + c] = v;
      }
      s_gf[j] = v;
    }
  }
  __syncthreads();
  PROBE_AT(3);
  // φ̃ = (h(g(s)) + h(g(s1))) ⊙ φ
  const FDiv fd = fdiv(d);
  for (int j = tid; j < (tid < 256 ? nb * d : 0); j += 256) {
    const int r = j / fd, c = j - r * d, bb = b0 + r;
    const float h0 = tsf_dot4(s_gf + r * GP, s_wh + c * GP, GP / 4);
    const float h1 = tsf_dot4(s_gf + (PB + r) * GP, s_wh + c * GP, GP / 4);
    const float hb = s_bh[c];
    const float aff = __fadd_rn(__fadd_rn(h0, hb), __fadd_rn(h1, hb));
    A.tphi[(size_t)bb * d + c] = __fmul_rn(aff, s_ph[j]);
  }
  PROBE_REC(10, t0_);
}

// The forward's Linear of g and φ̃ for workgroup blk's rows (TsfArgs::fwd_mode 2: the chains ran
// in an earlier launch with mode 1).  Operands: the chain's final states z_K (TsfArgs::zs), W_l
// transposed from the backward's image (TsfArgs::bimg, written by that launch), W_h as stored, the
// biases and φ -- the same values and the same arithmetic as the whole forward's tail.
template <int NP>
__device__ __forceinline__ void tsf_fwd_tail(const TsfArgs& A, const float* __restrict__ gfl, float* sm, int blk) {
  constexpr int PB = TSF_PB, RPW = 2 * PB;
  const int tid = threadIdx.x, n_s = A.n_s, G = A.G, K = A.K, d = A.d, B = A.B, R2 = 2 * B;
  const int nfl = K * tsf_flow_stride(n_s), GP = (G + 3) & ~3;
  const TsfTailLds L = tsf_tail_lds(NP, G, d);
  float *s_wlT = sm + L.wlT, *s_wh = sm + L.wh, *s_gf = sm + L.gf, *s_z = sm + L.z;
  float *s_ph = sm + L.ph, *s_bl = sm + L.bl, *s_bh = sm + L.bh;
  const int b0 = blk * PB, nb = min(PB, B - b0);
  PROBE_T(t0_);
  if (tid < 256) {
    glds16(s_wlT, A.bimg, NP * GP / 4);
    if (GP == G && (((uintptr_t)A.hp) & 15) == 0) {
      glds16(s_wh, A.hp, d * GP / 4);
    } else {
      const FDiv fgp = fdiv(GP);
      glds(s_wh, d * GP, [&](int j) -> const float* {
        const int c = j / fgp, q = j - c * GP;
        return q < G ? A.hp + c * G + q : nullptr;
      });
    }
    glds(s_z, RPW * NP, [&](int j) -> const float* {
      const int r = j / NP, i = j - r * NP, bb = b0 + (r >= PB ? r - PB : r);
      return bb < B ? A.zs + ((size_t)K * R2 + (r >= PB ? B + bb : bb)) * NP + i : nullptr;
    });
    glds(s_bl, G, [&](int j) { return gfl + nfl + G * n_s + j; });
    glds(s_bh, d, [&](int j) { return A.hp + d * G + j; });
    glds(s_ph, nb * d, [&](int j) { return A.phi + (size_t)b0 * d + j; });
  }
  __syncthreads();
  if (tid < 256) {  // Linear(n_s, G): tsf_dot4's four accumulators over i mod 4, W_l read transposed
    const FDiv fgp = fdiv(GP);
    for (int j = tid; j < RPW * GP; j += 256) {
      const int r = j / fgp, c = j - r * GP;
      float v = 0.f;
      if (c < G) {
        const float* zr = s_z + r * NP;
        tsf_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NP / 4; ++q) {
          const tsf_f4 wv = {s_wlT[(4 * q) * GP + c], s_wlT[(4 * q + 1) * GP + c], s_wlT[(4 * q + 2) * GP + c],
                             s_wlT[(4 * q + 3) * GP + c]};
          acc = __builtin_elementwise_fma(*(const tsf_f4*)(zr + 4 * q), wv, acc);
        }
        v = __fadd_rn(__fadd_rn(__fadd_rn(acc.x, acc.y), __fadd_rn(acc.z, acc.w)), s_bl[c]);
        const int bb = b0 + (r >= PB ? r - PB : r);
        if (bb < B) A.gfeat[(size_t)(r >= PB ? B + bb : bb) * G + c] = v;
      }
      s_gf[j] = v;
    }
  }
  __syncthreads();
  // φ̃ = (h(g(s)) + h(g(s1))) ⊙ φ
  const FDiv fd = fdiv(d);
  for (int j = tid; j < (tid < 256 ? nb * d : 0); j += 256) {
    const int r = j / fd, c = j - r * d, bb = b0 + r;
    const float h0 = tsf_dot4(s_gf + r * GP, s_wh + c * GP, GP / 4);
    const float h1 = tsf_dot4(s_gf + (PB + r) * GP, s_wh + c * GP, GP / 4);
    const float hb = s_bh[c];
    const float aff = __fadd_rn(__fadd_rn(h0, hb), __fadd_rn(h1, hb));
    A.tphi[(size_t)bb * d + c] = __fmul_rn(aff, s_ph[j]);
  }
  PROBE_REC(10, t0_);
}

template <int NP>
__global__ __launch_bounds__(256) void k_tsf_fwd(TsfArgs A, const float* __restrict__ gfl) {
  __shared__ __attribute__((aligned(16))) float sm[TSF_FWD_SM];
  SFX_CHK(threadIdx.x || tsf_fwd_lds(A.K, NP, A.G, A.d).total <= TSF_FWD_SM, tsf_fwd_lds(A.K, NP, A.G, A.d).total,
          TSF_FWD_SM, 0);
  tsf_fwd_body<NP>(A, gfl, sm, blockIdx.x, gridDim.x);
}

// flow-row role: rows [f FR, (f+1) FR) of the 2B rows; lanes 0..FR-1 of wave 0 run the reverse
// flow chains (one row each).  The pre-step flows come from TsfArgs::gch (their Adam step runs in a
// later launch), W_l / W_h transposed from TsfArgs::bimg (the forward's image).  With r_k = dz_{k+1}·u_{k-1}
// (known before da_k) the next chain value is su_{k-1} = dz_k·u_{k-1} = r_k + da_k c_{k-1}, so a
// step's critical path is two operations (da_k = su_k (1 - t_k^2), then that FMA); the update
// dz_k = dz_{k+1} + da_k w_k and the stores of dz_{k+1}, da_k run beside it.
template <int NP>
__device__ __forceinline__ void tsf_bwd_flows(const TsfArgs& A, const float* __restrict__ sfl, float* sm, float* s_dr, float* s_w,
                              float* s_r, int* s_ab, int f) {
  constexpr int FR = TSF_FR, PST = tsf_pst(NP), FA = tsf_fst(NP);
  const int tid = threadIdx.x, n_s = A.n_s, G = A.G, K = A.K, d = A.d, B = A.B, R2 = 2 * B;
  const int D4 = (d + 3) & ~3, G4 = (G + 3) & ~3;   // rows padded to 16 bytes (zeros)
  const TsfBwdLds L = tsf_bwd_lds(K, NP, G, d, B);
  float* s_t = sm + L.t;                            // [K][FR]
  float* s_wlT = sm + L.wlT;                        // Linear of g (pre-step), transposed: [NP][G4]
  float* s_whT = sm + L.whT;                        // W_h (pre-step), transposed: [G][D4]
  float* s_dg = sm + L.dg;                          // [FR][G4] (φ̃ rows while staging)
  float* s_da = sm + L.da;                          // [FR][d]
  float* s_gc = sm + L.gc;                          // ψ output gradient rows; daff [FR][D4]; dz_K [FR][NP]
  float* s_fa = sm + L.fa;                          // [K][FA] flows, chain layout
  PROBE_T(t0_);
  const int r0 = f * FR;
  const int nr = min(FR, R2 - r0);
  // stage everything up front (LDS-DMA, all in flight together): the flows from the chain-layout
  // copy (the flows' Adam runs in a later launch, so it still holds the pre-step values), W_l and
  // W_h transposed, this workgroup's tanh outputs
  glds16(s_fa, A.gch + (size_t)A.pol * K * FA, K * FA / 4);
  glds16(s_wlT, A.bimg, (NP * G4 + G * D4) / 4);  // W_l, W_h transposed (adjacent in the carve and the image)
  glds16(s_t, A.ts + tsf_ts_at(r0, 0, K), K * FR / 4);  // this workgroup's [K][FR] block (rows past nr unused)
  PROBE_AT(4);
  (void)tsf_stage_daff(A, nr, [&](int rl) { const int row = r0 + rl; return row < B ? row : row - B; }, s_dg, s_da,
                       s_gc, s_dr, s_w, s_r, s_ab);
  PROBE_AT(1);
  // daff rows in 16-byte rows (rows past nr: zero)
  float* s_dap = s_gc;
  for (int j = tid; j < FR * D4; j += 256) {
    const int rl = j / D4, c = j - rl * D4;
    s_dap[j] = rl < nr && c < d ? s_da[rl * d + c] : 0.f;
  }
  __syncthreads();
  // dg = daff W_h (the same for a batch index's s row and s1 row)
  {
    const FDiv fg4 = fdiv(G4);
    for (int j = tid; j < FR * G4; j += 256) {
      const int rl = j / fg4, q = j - rl * G4;
      s_dg[j] = q < G ? tsf_dot4(s_dap + rl * D4, s_whT + q * D4, D4 / 4) : 0.f;
    }
  }
  __syncthreads();
  // dz_K = dg W_lin (zero past n_s), one thread per (row, component)
  float* s_dz = s_gc;
  if (tid < FR * NP) {
    const int rl = tid / NP, i = tid - rl * NP;
    s_dz[tid] = i < n_s ? tsf_dot4(s_dg + rl * G4, s_wlT + i * G4, G4 / 4) : 0.f;
  }
  __syncthreads();
  PROBE_AT(2);
  constexpr int LPR = tsf_lpr(NP), NL = NP / LPR;
  if (tid >= 64 || K == 0) return;
  // c_k = w_{k+1}·u_k came with the flows: the forward that staged these flows stored them
  if (tid >= LPR * FR) return;
  // row rl on lanes [LPR rl, LPR rl + LPR) (components [hf NL, hf NL + NL) each)
  const int rl = tid / LPR, hf = tid % LPR, row = r0 + rl;
  const bool valid = row < R2;
  tsf_f2 dz[NL / 2];
#pragma unroll
  for (int p = 0; p < NL / 2; ++p) dz[p] = *(const tsf_f2*)(s_dz + rl * NP + hf * NL + 2 * p);
  // rows past 2B write to a scratch row (one basic block per step, as in k_tsf_fwd)
  float* pk = valid ? A.part + ((size_t)(K - 1) * R2 + row) * PST + hf * NL : A.scratch + rl * TSF_NS + hf * NL;
  float* pda = valid ? A.part + ((size_t)(K - 1) * R2 + row) * PST + NP : A.scratch + rl * TSF_NS + NP;
  const size_t pstep = valid ? (size_t)R2 * PST : 0;
  PROBE_AT(3);
  // flows k (F0) and k - 1 (F1) in registers; flow k - 2's LDS reads go out a step ahead
  TsfFlow<NL> F0, F1, F2;
  tsf_flow_ld<NL, NP>(F0, s_fa + (K - 1) * FA, hf);
  tsf_flow_ld<NL, NP>(F1, s_fa + max(K - 2, 0) * FA, hf);
  float t = s_t[(K - 1) * FR + rl];
  float su = tsf_row_sum<LPR>(tsf_dot<NL>(dz, F0.u));  // dz_K·u_{K-1}
  // one reverse step: Fa = flow k, Fb = flow k - 1, Fc <- flow k - 2 (rotated by name, as in
  // k_tsf_fwd); tb = t_{k-1}, tc <- t_{k-2}
  float t1 = s_t[max(K - 2, 0) * FR + rl], t2 = 0.f;
  auto step = [&](const TsfFlow<NL>& Fa, const TsfFlow<NL>& Fb, TsfFlow<NL>& Fc, float ta, float& tc, int k) {
    const float rn = tsf_row_sum<LPR>(tsf_dot<NL>(dz, Fb.u));  // dz_{k+1}·u_{k-1}: off the critical path
    // flow k - 2's reads after the dot has read flow k - 1 (as in k_tsf_fwd)
    tsf_flow_ld<NL, NP>(Fc, s_fa + max(k - 2, 0) * FA, hf);
    tc = s_t[max(k - 2, 0) * FR + rl];
    const float da = __fmul_rn(su, __fsub_rn(1.f, __fmul_rn(ta, ta)));
    tsf_store<NL>(pk, dz);
    *pda = da;  // both lanes: the same value
    pk -= pstep;
    pda -= pstep;
    su = __builtin_fmaf(da, Fb.c, rn);
    tsf_axpy<NL>(dz, da, Fa.w);
  };
  // K mod 3 steps first, then groups of three (as in k_tsf_fwd)
  int k = K - 1;
  const int rem = K % 3;
  if (rem == 0) {
    for (; k >= 0; k -= 3) {
      step(F0, F1, F2, t, t2, k);
      step(F1, F2, F0, t1, t, k - 1);
      step(F2, F0, F1, t2, t1, k - 2);
    }
  } else if (rem == 1) {
    step(F0, F1, F2, t, t2, k--);
    for (; k >= 0; k -= 3) {
      step(F1, F2, F0, t1, t, k);
      step(F2, F0, F1, t2, t1, k - 1);
      step(F0, F1, F2, t, t2, k - 2);
    }
  } else {
    step(F0, F1, F2, t, t2, k--);
    step(F1, F2, F0, t1, t, k--);
    for (; k >= 0; k -= 3) {
      step(F2, F0, F1, t2, t1, k);
      step(F0, F1, F2, t, t2, k - 1);
      step(F1, F2, F0, t1, t, k - 2);
    }
  }
  PROBE_REC(11, t0_);
}

// workgroup `role` of the backward (grid nflow + nh + nlin + 1, 256 threads; roles: see the
// header comment); sm holds tsf_bwd_lds(...).total floats
template <int NP>
__device__ __forceinline__ void tsf_bwd_block(const TsfArgs& A, const float* __restrict__ sfl, float* sm, float* s_dr, float* s_r,
                              float* s_w, float* s_red, int* s_ab, int role) {
  const int tid = threadIdx.x, n_s = A.n_s, G = A.G, K = A.K, d = A.d, B = A.B, R2 = 2 * B;
  const int fs = tsf_flow_stride(n_s), nfl = K * fs;
  if (role < A.nflow) {
    tsf_bwd_flows<NP>(A, sfl, sm, s_dr, s_w, s_r, s_ab, role);
    return;
  }
  role -= A.nflow;
  PROBE_T(t0_);
  const float* snap = A.snap;
  const int step = *A.step;
  const int cx = step_cancelled(A.cancel);
  const FDiv fG = fdiv(G);
  // LDS (tsf_bwd_lds): daff | role operands | φ̃ rows | ψ gradient rows | g-Linear dg
  const TsfBwdLds L = tsf_bwd_lds(K, NP, G, d, B);
  float* s_da = sm + L.rda;
  float* s_tp = sm + L.rtp;
  float* s_gc = sm + L.rgc;
  const bool wrole = role == A.nh + A.nlin;
  float* s_gf = sm + L.rgf;   // h role: [2B][G]
  float* s_whs = sm + L.rgf;  // g-Linear role: [d][TSF_QS] pre-step W_h columns
  float* s_zk = sm + L.rzk;   // g-Linear role: [2B][NP] z_K
  float* s_dg = sm + L.rdg;   // g-Linear role: [B][TSF_QS]
  const int q0 = (role - A.nh) * TSF_QS, nq = min(TSF_QS, G - q0);
  // staging by 16-byte LDS-DMA where the rows allow it (one KB per wave instruction; the dword
  // form issues one 256-byte request per wave instruction at ≈140 ns each)
  if (!wrole && role < A.nh) {
    if (((R2 * G) & 3) == 0 && (((uintptr_t)A.gfeat) & 15) == 0)
      glds16(s_gf, A.gfeat, R2 * G / 4);
    else
      glds(s_gf, R2 * G, [&](int j) { return A.gfeat + j; });
  } else if (!wrole) {
    const float* wh = snap + A.Pg;
    if ((G & 3) == 0 && (((uintptr_t)wh) & 15) == 0) {
      // W_h rows' columns [q0, q0 + TSF_QS): past G (the last role) the group reads on into the
      // next row / b_h (finite values; those columns' dg is zeroed below)
      glds16_rows(s_whs, wh + q0, d, G, TSF_QS / 4);
    } else {
      glds(s_whs, d * TSF_QS, [&](int j) {
        const int c = j / TSF_QS, qq = j - c * TSF_QS;
        return wh + c * G + q0 + (qq < nq ? qq : 0);  // columns past G: zeroed below
      });
    }
    glds16(s_zk, A.zs + (size_t)K * R2 * NP, R2 * NP / 4);  // NP is a multiple of 4
  }
  const float se = tsf_stage_daff(A, B, [](int rl) { return rl; }, s_tp, s_da, s_gc, s_dr, s_w, s_r, s_ab);
  PROBE_AT(1);
  if (wrole) {  // l2, g_w = drᵀ φ̃, Adam on w_i, the loss row
    const float sse = block_sum(se, s_red);
    if (tid < d) {
      float gw = 0.f;
      for (int b = 0; b < B; ++b) gw = __builtin_fmaf(s_dr[b], s_tp[b * d + tid], gw);
      if (!step_cancelled(A.cancel)) adam_el(A.w + tid, A.wm + tid, A.wv + tid, gw, adam_consts(A.hpw, step));
    }
    if (tid == 0 && A.losses) {
      const float l2 = (float)((double)sse / (double)B);
      A.losses[2] = l2;
      A.losses[0] = __fadd_rn(A.losses[1], __fmul_rn(A.beta, l2));
    }
    PROBE_REC(14, t0_);
    return;
  }
  if (role < A.nh) {  // h role: g_Wh = daffᵀ g(s) + daffᵀ g(s1), g_bh = 2 Σ_b daff
    const int j = role * 256 + tid;
    float g = 0.f;
    if (j >= A.Ph) {
    } else if (j < d * G) {
      const int c = j / fG, q = j - c * G;
      float g0 = 0.f, g1 = 0.f;
      for (int b = 0; b < B; ++b) {
        g0 = __builtin_fmaf(s_da[b * d + c], s_gf[b * G + q], g0);
        g1 = __builtin_fmaf(s_da[b * d + c], s_gf[(B + b) * G + q], g1);
      }
      g = __fadd_rn(g0, g1);
    } else {
      const int c = j - d * G;
      float sb = 0.f;
      for (int b = 0; b < B; ++b) sb = __fadd_rn(sb, s_da[b * d + c]);
      g = __fmul_rn(2.f, sb);
    }
    const long long ho = (long long)A.pol * A.Ph;
    if (j < A.Ph && !cx) adam_el(A.hp + j, A.hm + ho + j, A.hv + ho + j, g, adam_consts(A.hph, step));
    PROBE_REC(12, t0_);
    return;
  }
  // g-Linear role: columns [q0, q0 + nq) of g_i's Linear(n_s, G)
  for (int j = tid; j < B * TSF_QS; j += 256) {
    const int b = j / TSF_QS, qq = j - b * TSF_QS;
    float acc = 0.f;
    for (int c = 0; c < d; ++c) acc = __builtin_fmaf(s_da[b * d + c], s_whs[c * TSF_QS + qq], acc);
    s_dg[j] = qq < nq ? acc : 0.f;
  }
  __syncthreads();
  const AdamC cg = adam_consts(A.hpg, step);
  float* gp = A.g + (long long)A.pol * A.Pg;
  float* gm = A.gm + (long long)A.pol * A.Pg;
  float* gv = A.gv + (long long)A.pol * A.Pg;
  for (int j = tid; j < (cx ? 0 : nq * (n_s + 1)); j += 256) {
    const int qq = j / (n_s + 1), i = j - qq * (n_s + 1);
    int o;
    float g;
    if (i < n_s) {  // dW = dgᵀ z_K(s) + dgᵀ z_K(s1)
      float g0 = 0.f, g1 = 0.f;
      for (int b = 0; b < B; ++b) {
        g0 = __builtin_fmaf(s_dg[b * TSF_QS + qq], s_zk[b * NP + i], g0);
        g1 = __builtin_fmaf(s_dg[b * TSF_QS + qq], s_zk[(B + b) * NP + i], g1);
      }
      g = __fadd_rn(g0, g1);
      o = nfl + (q0 + qq) * n_s + i;
    } else {  // db = Σ dg + Σ dg
      float sb = 0.f;
      for (int b = 0; b < B; ++b) sb = __fadd_rn(sb, s_dg[b * TSF_QS + qq]);
      g = __fadd_rn(sb, sb);
      o = nfl + G * n_s + q0 + qq;
    }
    adam_el(gp + o, gm + o, gv + o, g, cg);
  }
  PROBE_REC(13, t0_);
}

template <int NP>
__global__ __launch_bounds__(256) void k_tsf_bwd(TsfArgs A, const float* __restrict__ sfl) {
  __shared__ __attribute__((aligned(16))) float sm[TSF_SM];
  __shared__ float s_dr[64], s_r[64], s_w[256], s_red[256];
  __shared__ int s_ab[64];
  SFX_CHK(threadIdx.x || tsf_bwd_lds(A.K, NP, A.G, A.d, A.B).total <= TSF_SM, tsf_bwd_lds(A.K, NP, A.G, A.d, A.B).total,
          TSF_SM, 1);
  tsf_bwd_block<NP>(A, sfl, sm, s_dr, s_r, s_w, s_red, s_ab, blockIdx.x);
}

// flow parameters: Σ over the s rows + Σ over the s1 rows of the per-row terms (the two
// g_backward calls of the reference), then Adam.  grid K (one workgroup per flow), 256 threads:
// the flow's saved states z_k, tanh outputs t_k and the rows' (dz_{k+1}, da_k) into LDS, then
// thread e of [0, 2 n_s + 1) sums its parameter's terms row by row:
//   w_i: da_k z_k[i]     b: da_k     u_i: dz_{k+1}[i] t_k
// sm: tsf_bwd_lds(...).fk_total floats
__device__ __forceinline__ void tsf_flow_block(const TsfArgs& A, float* sm, int k) {
  const int tid = threadIdx.x, n_s = A.n_s, fs = tsf_flow_stride(n_s), B = A.B, R2 = 2 * B, NP = A.np;
  const int PST = tsf_pst(NP);
  const TsfBwdLds L = tsf_bwd_lds(A.K, NP, A.G, A.d, B);
  float *s_z = sm, *s_dz = sm + L.fdz, *s_da = sm + L.fda, *s_t = sm + L.ft;
  PROBE_T(t0_);
  const FDiv fnp = fdiv(NP);
  glds16(s_z, A.zs + (size_t)k * R2 * NP, R2 * NP / 4);  // NP is a multiple of 4
  if ((PST & 3) == 0)
    glds16_rows(s_dz, A.part + (size_t)k * R2 * PST, R2, PST, NP / 4);
  else
    glds(s_dz, R2 * NP, [&](int j) {
      const int r = j / fnp;
      return A.part + ((size_t)k * R2 + r) * PST + (j - r * NP);
    });
  glds(s_da, R2, [&](int j) { return A.part + ((size_t)k * R2 + j) * PST + NP; });
  glds(s_t, R2, [&](int j) { return A.ts + tsf_ts_at(j, k, A.K); });
  __syncthreads();
  if (tid >= fs) return;
  const int e = tid;
  float g0 = 0.f, g1 = 0.f;
  if (e < n_s) {
    for (int r = 0; r < B; ++r) g0 = __fadd_rn(g0, __fmul_rn(s_da[r], s_z[r * NP + e]));
    for (int r = B; r < R2; ++r) g1 = __fadd_rn(g1, __fmul_rn(s_da[r], s_z[r * NP + e]));
  } else if (e == n_s) {
    for (int r = 0; r < B; ++r) g0 = __fadd_rn(g0, s_da[r]);
    for (int r = B; r < R2; ++r) g1 = __fadd_rn(g1, s_da[r]);
  } else {
    const int i = e - n_s - 1;
    for (int r = 0; r < B; ++r) g0 = __fadd_rn(g0, __fmul_rn(s_dz[r * NP + i], s_t[r]));
    for (int r = B; r < R2; ++r) g1 = __fadd_rn(g1, __fmul_rn(s_dz[r * NP + i], s_t[r]));
  }
  const float g = __fadd_rn(g0, g1);
  const long long go = (long long)A.pol * A.Pg + (long long)k * fs + e;
  if (!step_cancelled(A.cancel)) {
    adam_el(A.g + go, A.gm + go, A.gv + go, g, adam_consts(A.hpf, *A.step));
    // the chain-layout copy (TsfArgs::gch): w at e, b at 2NP, u at NP + (e - n_s - 1)
    const int slot = e < n_s ? e : e == n_s ? 2 * NP : NP + (e - n_s - 1);
    A.gch[((long long)A.pol * A.K + k) * tsf_fst(NP) + slot] = A.g[go];
  }
  PROBE_REC(15, t0_);
}

// TsfArgs::gch of one head from its packed flows (after a host load of g): workgroup k writes
// flow k's chain-layout row, zeros in the padding and c slots
__global__ __launch_bounds__(64) void k_tsf_gch(const float* __restrict__ g, float* __restrict__ gch, int n_s, int np) {
  const int k = blockIdx.x, FA = tsf_fst(np), fs = tsf_flow_stride(n_s);
  const float* f = g + (long long)k * fs;
  for (int e = threadIdx.x; e < FA; e += blockDim.x) {
    float v = 0.f;
    if (e < n_s)
      v = f[e];
    else if (e >= np && e < np + n_s)
      v = f[n_s + 1 + (e - np)];
    else if (e == 2 * np)
      v = f[n_s];
    gch[(long long)k * FA + e] = v;
  }
}

__global__ __launch_bounds__(256) void k_tsf_flow(TsfArgs A) {
  __shared__ __attribute__((aligned(16))) float sm[2 * 128 * TSF_NS + 256];  // 2B <= 128 rows
  SFX_CHK(threadIdx.x || tsf_bwd_lds(A.K, A.np, A.G, A.d, A.B).fk_total <= 2 * 128 * TSF_NS + 256,
          tsf_bwd_lds(A.K, A.np, A.G, A.d, A.B).fk_total, 2 * 128 * TSF_NS + 256, 2);
  tsf_flow_block(A, sm, blockIdx.x);
}

// A ψ backward launch (k_bwd's tiles) with TSF-DQN's backward riding along in the same grid
// (sfx_tsf.inc): blocks [0, ntsf) run TSF work -- mode 1 k_tsf_bwd's roles, mode 2 k_tsf_flow's
// flows -- and the rest k_bwd's tiles of one head.  The TSF chains (≈24 µs at K = 100) then run
// beside the ψ tiles instead of as launches of their own on the step's critical path; the LDS
// of the two halves is allocated side by side (k_bwd's + TSFX_SM floats), so the host rides
// along only when the TSF carve fits and the grid stays within one workgroup per CU.
template <int NP, bool BF>
__global__ __launch_bounds__(256) void k_bwd_tsf(Geo G, BwdArgs A, TsfArgs T, const float* __restrict__ sfl,
                                                  int mode, int ntsf) {
  __shared__ floatx4 red[4][2][64];
  __shared__ __attribute__((aligned(16))) float sm[TSFX_SM];
  __shared__ float s_dr[64], s_r[64], s_w[256], s_red[256];
  __shared__ int s_ab[64];
  const int bx = blockIdx.x;
  if (bx < ntsf) {
    SFX_CHK(threadIdx.x || (mode == 1 ? tsf_bwd_lds(T.K, NP, T.G, T.d, T.B).total : tsf_bwd_lds(T.K, T.np, T.G, T.d, T.B).fk_total) <= TSFX_SM,
            mode, tsf_bwd_lds(T.K, NP, T.G, T.d, T.B).total, TSFX_SM);
    if (mode == 1)
      tsf_bwd_block<NP>(T, sfl, sm, s_dr, s_r, s_w, s_red, s_ab, bx);
    else
      tsf_flow_block(T, sm, bx);
    return;
  }
  bwd_body<BF>(G, A, A.head0, bx - ntsf, red);
}

// The ψ forward's first launch (layers 0 + 1 from the states, k_fwd<true, 8, true, BF>) with
// k_tsf_fwd's workgroups riding along first in the same grid: the flow chains run beside the ψ
// tiles.  (gx, gy) = the ψ launch's own grid; its workgroup r is (r % gx, r / gx % gy, r / gx gy).
template <int NP, bool BF, int TP>
__global__ __launch_bounds__(512) void k_fwd_tsf(Geo G, FwdArgs F, TsfArgs T, const float* __restrict__ gfl,
                                                  int ntsf, int gx, int gy) {
  __shared__ __attribute__((aligned(16))) float sm[TSFXF_SM];
  const int b = blockIdx.x;
  if (b < ntsf) {
    SFX_CHK(threadIdx.x || tsf_fwd_lds(T.K, NP, T.G, T.d).total <= TSFXF_SM, tsf_fwd_lds(T.K, NP, T.G, T.d).total,
            TSFXF_SM, 3);
    tsf_fwd_body<NP>(T, gfl, sm, b, ntsf);
    return;
  }
  const int r = b - ntsf;
  fwd_body<true, 8, true, BF, TP>(G, F, r % gx, (r / gx) % gy, r / (gx * gy));
}

// The one-state selection (k_sel1m: a workgroup per head, the last to arrive picks and publishes)
// with the look-ahead TSF forward's tail (Linear of g, φ̃: TsfArgs::fwd_mode 2) riding along first
// in its grid (select_ahead_body): its chains ran in the select's first launch (mode 1), and the
// tail runs beside the selection instead of after the chains there.  256-thread workgroups.
template <int VW, int NP>
__global__ __launch_bounds__(256) void k_sel1m_tsft(Geo G, GpiArgs A, SelPub P, SelScratch* S, TsfArgs T,
                                                     const float* __restrict__ gfl, int ntsf) {
  __shared__ __attribute__((aligned(16))) float sm[TSFXF_SM];
  const int b = blockIdx.x;
  if (b < ntsf) {
    SFX_CHK(threadIdx.x || tsf_tail_lds(NP, T.G, T.d).total <= TSFXF_SM, tsf_tail_lds(NP, T.G, T.d).total, TSFXF_SM, 5);
    tsf_fwd_tail<NP>(T, gfl, sm, b);
    return;
  }
  sel1m_body<VW>(G, A, P, S, b - ntsf);
}

// -------------------------------------------------------------------------------------
// TSF test tasks: TSFDQN.get_test_action (tsfdqn.py:859-870) and
// update_test_reward_mapper (tsfdqn.py:917-997).  A test task mixes the source tasks with
// ω̂ = ω / Σω and fits its reward weights w and ω by Adam on
//   l1 = MSE(Σ_t ω̂_t ψ_t(s)[a], φ̃ + γ Σ_t ω̂_t ψ⁻_t(s1)[a1]),  l2 = (w·φ̃ - r)²,
//   loss = l1 + β l2 + λ Σ|ω|,   φ̃ = φ ⊙ (h(Σ_t ω̂_t g_t(s)) + h(Σ_t ω̂_t g_t(s1))),
// ψ, ψ⁻ and g_t held fixed (no_grad), then ω ≥ 1e-7.  B = 1: tiny, latency-bound kernels.
// -------------------------------------------------------------------------------------
struct TsfTestArgs {
  int T, n_s, G, K, A, d, O, Pg, lastOff, pad_;
  long long actSize;
  const float* s;        // [n_s] (k_tsf_test_g)
  const float* s1;
  const float* g;        // [T][Pg] g_t parameters (TsfArgs::g packing)
  const float* hp;       // [d][G] W_h then [d] b_h
  float* gfeat;          // [T][2][G]: g_t(s), g_t(s1)
  const float* psi;      // ψ_t(s):  row 0 of an activation role, head stride actSize, at lastOff
  const float* psi1;     // ψ⁻_t(s1)
  const float* phi;      // [d]
  const int64_t* a;      // device scalars (the actions the agent took / will take)
  const int64_t* a1;
  float r, gamma, beta, lasso;
  float* w;              // [d] the test task's reward weights (in place)
  float* omega;          // [T] (in place)
  float* mom;            // [2d + 2T]: m_w, v_w, m_ω, v_ω
  int step;              // Adam step after this update (1-based)
  int pad2_;
  AdamHP hpw, hpo;
  float* losses;         // [3]: loss, l2, l1 (the reference's return order)
  int64_t* act_out;      // k_tsf_test_act: the greedy action
  // Lockstep test phase (sfx_tsf_test_actions / sfx_tsf_test_updates): row e of a launch is test
  // task e -- its state rows s/s1 [E][n_s], ψ row e of the forward, φ [E][d], a/a1 [E], w / ω /
  // moments at their row strides, losses [E][3], act_out [E]; rowp [E][6] = r, lr_w, wd_w, lr_ω,
  // wd_ω, step of each task's own optimizer (nullptr: the scalar fields above, E = 1).
  int w_stride, o_stride, mom_stride, pad3_;
  const float* rowp;
};

// The arguments of test task e (row e of a lockstep launch); e = 0 with rowp == nullptr is the
// single-task call unchanged.
__device__ inline TsfTestArgs tsf_test_row(const TsfTestArgs& A0, int e) {
  TsfTestArgs A = A0;
  if (A.s) A.s += (long long)e * A.n_s;
  if (A.s1) A.s1 += (long long)e * A.n_s;
  if (A.gfeat) A.gfeat += (long long)e * 2 * A.T * A.G;
  if (A.psi) A.psi += (long long)e * A.O;
  if (A.psi1) A.psi1 += (long long)e * A.O;
  if (A.phi) A.phi += (long long)e * A.d;
  if (A.a) A.a += e;
  if (A.a1) A.a1 += e;
  if (A.w) A.w += (long long)e * A.w_stride;
  if (A.omega) A.omega += (long long)e * A.o_stride;
  if (A.mom) A.mom += (long long)e * A.mom_stride;
  if (A.losses) A.losses += (long long)e * 3;
  if (A.act_out) A.act_out += e;
  if (A.rowp) {
    const float* p = A.rowp + (long long)e * 6;
    A.r = p[0];
    A.hpw.lr = p[1];
    A.hpw.wd = p[2];
    A.hpo.lr = p[3];
    A.hpo.wd = p[4];
    A.step = (int)p[5];
  }
  return A;
}

// g_t(s), g_t(s1) for every task: one wave per task, lanes 0..31 row s, 32..63 row s1, one state
// component per lane through the K planar flows (w_k·z by a xor butterfly within the 32-lane
// half), then Linear(n_s, G) from LDS.
__global__ __launch_bounds__(64) void k_tsf_test_g(TsfTestArgs A0) {
  const TsfTestArgs A = tsf_test_row(A0, blockIdx.y);
  const int t = blockIdx.x, lane = threadIdx.x, row = lane >> 5, j = lane & 31, n_s = A.n_s, G = A.G;
  const float* gp = A.g + (long long)t * A.Pg;
  const bool on = j < n_s;
  float z = on ? (row ? A.s1 : A.s)[j] : 0.f;
  const int fs = 2 * n_s + 1;
  for (int k = 0; k < A.K; ++k) {
    const float* f = gp + (long long)k * fs;
    const float wk = on ? f[j] : 0.f, uk = on ? f[n_s + 1 + j] : 0.f, bk = f[n_s];
    float v = __fmul_rn(wk, z);
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o, 32));
    const float th = tsf_tanh(__fadd_rn(v, bk));
    z = __fadd_rn(z, __fmul_rn(uk, th));
  }
  __shared__ float sz[2][TSF_NS];
  if (on) sz[row][j] = z;
  __syncthreads();
  const float* W = gp + (long long)A.K * fs;
  const float* b = W + (long long)G * n_s;
  for (int idx = lane; idx < 2 * G; idx += 64) {
    const int rr = idx >= G ? 1 : 0, o = idx - rr * G;
    float acc = 0.f;
    for (int q = 0; q < n_s; ++q) acc = __builtin_fmaf(W[(long long)o * n_s + q], sz[rr][q], acc);
    A.gfeat[((long long)t * 2 + rr) * G + o] = __fadd_rn(acc, b[o]);
  }
}

// The greedy test action: argmax_a Σ_k w_k Σ_t ω̂_t ψ_t(s)[a][k] (first index on ties), one WG.
__global__ __launch_bounds__(256) void k_tsf_test_act(TsfTestArgs A0) {
  const TsfTestArgs A = tsf_test_row(A0, blockIdx.x);
  __shared__ float s_on[64];
  __shared__ float s_q[256];
  const int tid = threadIdx.x, T = A.T, d = A.d;
  if (tid == 0) {
    float S = 0.f;
    for (int t = 0; t < T; ++t) S = __fadd_rn(S, A.omega[t]);
    for (int t = 0; t < T; ++t) s_on[t] = __fdiv_rn(A.omega[t], S);
  }
  __syncthreads();
  for (int a = tid; a < A.A; a += 256) {
    float q = 0.f;
    for (int k = 0; k < d; ++k) {
      float m = 0.f;
      for (int t = 0; t < T; ++t) m = __fadd_rn(m, __fmul_rn(A.psi[(long long)t * A.actSize + A.lastOff + a * d + k], s_on[t]));
      q = __builtin_fmaf(m, A.w[k], q);
    }
    s_q[a] = q;
  }
  __syncthreads();
  if (tid == 0) {
    int best = 0;
    for (int a = 1; a < A.A; ++a)
      if (s_q[a] > s_q[best]) best = a;
    *A.act_out = best;
  }
}

// One update_test_reward_mapper step, one WG (T <= 64, d <= 256, G <= 512).
__global__ __launch_bounds__(256) void k_tsf_test_step(TsfTestArgs A0) {
  const TsfTestArgs A = tsf_test_row(A0, blockIdx.x);
  const int tid = threadIdx.x, T = A.T, d = A.d, G = A.G;
  __shared__ float s_om[64], s_on[64], s_dn[64];
  __shared__ float s_ws[2][512], s_gws[512];
  __shared__ float s_tphi[256], s_de[256], s_gaff[256], s_w[256];
  __shared__ float s_S, s_rfit, s_l1, s_sumdn;
  const int a = (int)*A.a, a1 = (int)*A.a1;
  const float* Wh = A.hp;
  const float* bh = A.hp + (long long)d * G;
  if (tid < T) s_om[tid] = A.omega[tid];
  if (tid < d) s_w[tid] = A.w[tid];
  __syncthreads();
  if (tid == 0) {
    float S = 0.f;
    for (int t = 0; t < T; ++t) S = __fadd_rn(S, s_om[t]);
    s_S = S;
    for (int t = 0; t < T; ++t) s_on[t] = __fdiv_rn(s_om[t], S);
  }
  __syncthreads();
  // weighted g features of s and s1
  for (int idx = tid; idx < 2 * G; idx += 256) {
    const int rr = idx >= G ? 1 : 0, o = idx - rr * G;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc = __fadd_rn(acc, __fmul_rn(A.gfeat[((long long)t * 2 + rr) * G + o], s_on[t]));
    s_ws[rr][o] = acc;
  }
  __syncthreads();
  // φ̃, the two ω-mixed successor rows, the TD error
  if (tid < d) {
    float h0 = 0.f, h1 = 0.f;
    for (int g = 0; g < G; ++g) {
      h0 = __builtin_fmaf(Wh[(long long)tid * G + g], s_ws[0][g], h0);
      h1 = __builtin_fmaf(Wh[(long long)tid * G + g], s_ws[1][g], h1);
    }
    const float aff = __fadd_rn(__fadd_rn(h0, bh[tid]), __fadd_rn(h1, bh[tid]));
    const float tphi = __fmul_rn(A.phi[tid], aff);
    float cur = 0.f, nx = 0.f;
    for (int t = 0; t < T; ++t) {
      cur = __fadd_rn(cur, __fmul_rn(A.psi[(long long)t * A.actSize + A.lastOff + a * d + tid], s_on[t]));
      nx = __fadd_rn(nx, __fmul_rn(A.psi1[(long long)t * A.actSize + A.lastOff + a1 * d + tid], s_on[t]));
    }
    const float e = __fsub_rn(cur, __fadd_rn(tphi, __fmul_rn(A.gamma, nx)));
    s_tphi[tid] = tphi;
    s_de[tid] = e;
  }
  __syncthreads();
  if (tid == 0) {
    float se = 0.f, rf = 0.f;
    for (int k = 0; k < d; ++k) {
      se = __builtin_fmaf(s_de[k], s_de[k], se);
      rf = __builtin_fmaf(s_tphi[k], s_w[k], rf);
    }
    s_l1 = __fdiv_rn(se, (float)d);
    s_rfit = rf;
  }
  __syncthreads();
  const float q = __fmul_rn(A.beta, __fmul_rn(2.f, __fsub_rn(s_rfit, A.r)));  // dloss / dr_fit
  const float nd = __fdiv_rn(2.f, (float)d);
  if (tid < d) {
    const float de = __fmul_rn(nd, s_de[tid]);                    // dl1 / dcur
    s_gaff[tid] = __fmul_rn(__fadd_rn(-de, __fmul_rn(q, s_w[tid])), A.phi[tid]);
    s_de[tid] = de;
  }
  __syncthreads();
  for (int g = tid; g < G; g += 256) {  // d aff / d (mixed g features): W_hᵀ gaff (both rows alike)
    float acc = 0.f;
    for (int k = 0; k < d; ++k) acc = __builtin_fmaf(Wh[(long long)k * G + g], s_gaff[k], acc);
    s_gws[g] = acc;
  }
  __syncthreads();
  if (tid < T) {  // dloss / d ω̂_t
    float v = 0.f;
    for (int k = 0; k < d; ++k) {
      v = __builtin_fmaf(s_de[k], A.psi[(long long)tid * A.actSize + A.lastOff + a * d + k], v);
      v = __builtin_fmaf(-__fmul_rn(A.gamma, s_de[k]), A.psi1[(long long)tid * A.actSize + A.lastOff + a1 * d + k], v);
    }
    for (int g = 0; g < G; ++g)
      v = __builtin_fmaf(s_gws[g], __fadd_rn(A.gfeat[((long long)tid * 2) * G + g], A.gfeat[((long long)tid * 2 + 1) * G + g]), v);
    s_dn[tid] = v;
  }
  __syncthreads();
  if (tid == 0) {
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc = __builtin_fmaf(s_on[t], s_dn[t], acc);
    s_sumdn = acc;
    float l1n = 0.f;
    for (int t = 0; t < T; ++t) l1n = __fadd_rn(l1n, fabsf(s_om[t]));
    const float l2 = __fmul_rn(__fsub_rn(s_rfit, A.r), __fsub_rn(s_rfit, A.r));
    const float loss = __fadd_rn(__fadd_rn(s_l1, __fmul_rn(A.beta, l2)), __fmul_rn(A.lasso, l1n));
    A.losses[0] = loss;
    A.losses[1] = l2;
    A.losses[2] = s_l1;
  }
  __syncthreads();
  float* mw = A.mom;
  float* vw = A.mom + d;
  float* mo = A.mom + 2 * d;
  float* vo = A.mom + 2 * d + T;
  if (tid < d) adam_el(A.w + tid, mw + tid, vw + tid, __fmul_rn(q, s_tphi[tid]), adam_consts(A.hpw, A.step));
  if (tid < T) {
    const float om = s_om[tid];
    const float sg = om > 0.f ? 1.f : (om < 0.f ? -1.f : 0.f);
    const float g = __fadd_rn(__fdiv_rn(__fsub_rn(s_dn[tid], s_sumdn), s_S), __fmul_rn(A.lasso, sg));
    float pp = om, mm = mo[tid], vv = vo[tid];
    adam_apply(pp, mm, vv, g, adam_consts(A.hpo, A.step));
    mo[tid] = mm;
    vo[tid] = vv;
    A.omega[tid] = fmaxf(pp, 1e-7f);
  }
}

}  // namespace sfx
