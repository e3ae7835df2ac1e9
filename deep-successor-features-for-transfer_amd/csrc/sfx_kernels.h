// sfx_kernels.h -- gfx950 device code for the successor-feature hot path.
//
// fp32 end to end: the dense products run on the exact-f32 matrix cores
// (v_mfma_f32_16x16x4_f32, a k-ordered fmaf chain), element-wise work on VALU.
// Reference behaviour being implemented is cited per kernel (paths relative to
// /root/reference/source).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sfx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int NLMAX = 8;        // Linear layers per head (n_hidden <= 6)
constexpr int TDG_QMAX = 8192;  // M*A entries of the per-row GPI scratch in LDS
constexpr int TDG_MMAX = 1024;
constexpr int TDG_DMAX = 256;

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

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

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 16 consecutive floats row[kb .. kb+15], zero outside [0, K) or when !ok.
__device__ __forceinline__ void load16(float (&v)[16], const float* row, int kb, int K, bool ok) {
  if (ok && kb + 16 <= K && ((reinterpret_cast<uintptr_t>(row + kb) & 15u) == 0)) {
    const float4* p = reinterpret_cast<const float4*>(row + kb);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = p[q];
      v[4 * q + 0] = t.x;
      v[4 * q + 1] = t.y;
      v[4 * q + 2] = t.z;
      v[4 * q + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (ok && kb + j < K) ? row[kb + j] : 0.f;
  }
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

__device__ __forceinline__ void adam_el(float* __restrict__ p, float* __restrict__ m,
                                        float* __restrict__ v, float g, const AdamC& c) {
  float pp = *p, mm = *m, vv = *v;
  if (c.wd != 0.f) g = __fadd_rn(g, __fmul_rn(c.wd, pp));
  mm = __builtin_fmaf(c.omb1, __fsub_rn(g, mm), mm);  // vectorized lerp: fmadd(w, end-start, start)
  vv = __fadd_rn(__fmul_rn(vv, c.b2), __fmul_rn(__fmul_rn(c.omb2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), c.bc2s), c.eps);
  pp = __fadd_rn(pp, __fdiv_rn(__fmul_rn(c.nss, mm), denom));
  *p = pp;
  *m = mm;
  *v = vv;
}

// -------------------------------------------------------------------------------------
// Forward of one Linear (+activation) for a batch of (head, input-stream) instances:
//   Y[M,N] = act(X[M,K] W[N,K]^T + b)      (nn.Linear of the ψ lambda,
//                                            main_sfdqn_torch.py:57-71)
// Grid: (ceil(N/16), n_inst, ceil(M/32)), 256 threads.  A workgroup owns a 32x16 output
// tile; its 4 waves split K in 64-wide chunks, each wave runs two 16x16x4 f32 MFMA
// chains (rows m0..m0+15, m0+16..m0+31), partial tiles are summed through LDS in wave
// order (deterministic).
// -------------------------------------------------------------------------------------
struct FwdInst {
  const float* X;  // layer input (used when xsel == 0)
  const float* W;  // [N, K]
  const float* b;  // [N]
  float* Y;        // [M, N]
  int xsel;        // 0: X, 1: kernel arg xa, 2: kernel arg xb
  int pad_;
};

__global__ __launch_bounds__(256) void k_fwd(const FwdInst* __restrict__ insts, int M, int N, int K,
                                             int act, const float* __restrict__ xa,
                                             const float* __restrict__ xb) {
  const FwdInst in = insts[blockIdx.y];
  const float* X = in.xsel == 0 ? in.X : (in.xsel == 1 ? xa : xb);
  const int n0 = blockIdx.x * 16, m0 = blockIdx.z * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int ma = m0 + r, mb = m0 + 16 + r, n = n0 + r;
  const bool oka = ma < M, okb = mb < M, okn = n < N;
  const float* xra = X + (size_t)ma * K;
  const float* xrb = X + (size_t)mb * K;
  const float* wr = in.W + (size_t)n * K;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int kc = wave * 64; kc < K; kc += 256) {
    const int kb = kc + g * 16;
    float a0[16], a1[16], bw[16];
    load16(a0, xra, kb, K, oka);
    load16(a1, xrb, kb, K, okb);
    load16(bw, wr, kb, K, okn);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0 = mfma4(a0[j], bw[j], acc0);
      acc1 = mfma4(a1[j], bw[j], acc1);
    }
  }
  __shared__ floatx4 red[4][2][64];
  red[wave][0][lane] = acc0;
  red[wave][1][lane] = acc1;
  __syncthreads();
  if (threadIdx.x < 128) {
    const int s = threadIdx.x >> 6, L = threadIdx.x & 63;
    floatx4 v = red[0][s][L];
    v += red[1][s][L];
    v += red[2][s][L];
    v += red[3][s][L];
    const int col = n0 + (L & 15);
    if (col < N) {
      const float bias = in.b[col];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * s + (L >> 4) * 4 + i;
        if (row < M) in.Y[(size_t)row * N + col] = act_fwd(__fadd_rn(v[i], bias), act);
      }
    }
  }
}

// -------------------------------------------------------------------------------------
// TD target and output gradient for one policy (sfdqn.py:313-345; features/deep.py:101-122)
//   a'_b = argmax_a max_t ψ_t(s1_b)[a]·w_i        (GPI branch)
//        = argmax_a ψ_i(s1_b)[a]·w_i              (own-ψ branch)
//   t_b  = φ_b + γ_b ψ⁻_i(s1_b)[a'_b]
//   g[b, a_b, :] = 2 (c[b,a_b,:] - t_b) / (M*A*d), 0 elsewhere  (MSE vs merged clone)
//   l1 = Σ (c - t)^2 / (M*A*d);  optional l2 = MSE(w_i·φ, r) with one Adam step on w_i.
// One 256-thread workgroup per policy instance.
// -------------------------------------------------------------------------------------
struct TdgInst {
  int policy;
  int pad_;
  const float* c;     // ψ_i(S)    [M, O]
  const float* tpsi;  // ψ⁻_i(S1)  [M, O]
  const float* psiN;  // ψ_t(S1)   head t at psiN + t * psiN_stride, [M, O]
  float* w;           // w_i [d]
  float* wm;
  float* wv;
  int* step;          // Adam step counter of head i (incremented here when inc_step)
  float* g;           // [M, O]
};

struct TdgArgs {
  int M, T, A, d, use_gpi, train_w, inc_step, pad_;
  long long psiN_stride;
  const int64_t* a;
  const float* phi;
  const float* gamma;
  const float* r;
  float* losses;      // [n_inst][3] = (l1 + l2, l1, l2) or null
  int64_t* next;      // [n_inst][M] or null
  AdamHP hpw;
};

__device__ __forceinline__ float block_sum256(float v, float* sh) {
  // deterministic tree sum over the 256 threads of a block
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] = __fadd_rn(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  const float out = sh[0];
  __syncthreads();
  return out;
}

__global__ __launch_bounds__(256) void k_tdg(const TdgInst* __restrict__ insts, TdgArgs A) {
  const TdgInst I = insts[blockIdx.x];
  const int M = A.M, Aa = A.A, d = A.d, O = Aa * d, tid = threadIdx.x;
  __shared__ float s_w[TDG_DMAX];
  __shared__ float s_q[TDG_QMAX];
  __shared__ int s_next[TDG_MMAX];
  __shared__ float s_red[256];
  const int step = *I.step + 1;
  for (int k = tid; k < d; k += 256) s_w[k] = I.w[k];
  __syncthreads();
  // q over (b, a): max over heads (GPI) or own head
  for (int idx = tid; idx < M * Aa; idx += 256) {
    const int b = idx / Aa, a = idx - b * Aa;
    float best = -INFINITY;
    const int t0 = A.use_gpi ? 0 : I.policy, t1 = A.use_gpi ? A.T : I.policy + 1;
    for (int t = t0; t < t1; ++t) {
      const float* p = I.psiN + (long long)t * A.psiN_stride + (size_t)b * O + a * d;
      float q = 0.f;
      for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
      best = (t == t0 || q > best) ? q : best;
    }
    s_q[idx] = best;
  }
  for (int idx = tid; idx < M * O; idx += 256) I.g[idx] = 0.f;
  __syncthreads();
  for (int b = tid; b < M; b += 256) {
    int am = 0;
    float qm = s_q[b * Aa];
    for (int a = 1; a < Aa; ++a) {
      const float q = s_q[b * Aa + a];
      if (q > qm) { qm = q; am = a; }
    }
    s_next[b] = am;
    if (A.next) A.next[(size_t)blockIdx.x * M + b] = am;
  }
  __threadfence_block();
  __syncthreads();
  const float norm = (float)(2.0 / ((double)M * (double)O));
  float sq = 0.f;
  for (int idx = tid; idx < M * d; idx += 256) {
    const int b = idx / d, k = idx - b * d;
    const int ab = (int)A.a[b];
    if (ab < 0 || ab >= Aa) continue;  // invalid action: contributes nothing (never indexes out of range)
    const float tg = __fadd_rn(A.phi[idx], __fmul_rn(A.gamma[b], I.tpsi[(size_t)b * O + s_next[b] * d + k]));
    const float diff = __fsub_rn(I.c[(size_t)b * O + ab * d + k], tg);
    I.g[(size_t)b * O + ab * d + k] = __fmul_rn(norm, diff);
    sq = __builtin_fmaf(diff, diff, sq);
  }
  const float l1 = (float)((double)block_sum256(sq, s_red) / ((double)M * (double)O));
  float l2 = 0.f;
  if (A.train_w) {
    // r_fit = w·φ_b ; e_b = r_fit - r_b ; dw = Σ_b (2/M) e_b φ_b   (sfdqn.py:340-342)
    __shared__ float s_e[TDG_MMAX];
    float se = 0.f;
    for (int b = tid; b < M; b += 256) {
      float rf = 0.f;
      for (int k = 0; k < d; ++k) rf = __builtin_fmaf(s_w[k], A.phi[(size_t)b * d + k], rf);
      const float e = __fsub_rn(rf, A.r[b]);
      s_e[b] = __fmul_rn((float)(2.0 / (double)M), e);
      se = __builtin_fmaf(e, e, se);
    }
    l2 = (float)((double)block_sum256(se, s_red) / (double)M);
    const AdamC c = adam_consts(A.hpw, step);
    for (int k = tid; k < d; k += 256) {
      float gw = 0.f;
      for (int b = 0; b < M; ++b) gw = __builtin_fmaf(s_e[b], A.phi[(size_t)b * d + k], gw);
      adam_el(I.w + k, I.wm + k, I.wv + k, gw, c);
    }
  }
  if (tid == 0) {
    if (A.losses) {
      float* lo = A.losses + 3 * blockIdx.x;
      lo[0] = __fadd_rn(l1, l2);
      lo[1] = l1;
      lo[2] = l2;
    }
    if (A.inc_step) *I.step = step;
  }
}

// -------------------------------------------------------------------------------------
// Backward through the ψ MLP with Adam fused into the weight-gradient epilogue
// (autograd of sfdqn.py:344-345 + optim.step() at :362).
//
// Layers are processed in a ping-pong so no launch both reads and rewrites a weight:
// the launch that back-propagates through layer l (dX role, reads W_l) is the one that
// finishes the weight gradient of layer l+1 and applies Adam to it (dW roles).
//   dX role : dZ_{l-1} = (dZ_l W_l) ⊙ act'(X_l)        32x16 tile, split over the 4 waves
//   dW role : dW_l = dZ_l^T X_l ; db_l = Σ_m dZ_l ; Adam(W_l, b_l)
// blockIdx.x selects the role: [0, na) dX of layer la; [na, na+nb) dW of lb;
// [na+nb, na+nb+nc) dW of lc.  blockIdx.y = updated head instance.
// -------------------------------------------------------------------------------------
struct LayerGeo {
  int N, K, wOff, bOff, actIn;  // actIn: activation that produced this layer's input
};

struct BwdInst {
  float* P;                   // packed params of the head (online)
  float* Mo;                  // Adam m
  float* Vo;                  // Adam v
  const int* step;            // Adam step (already incremented by k_tdg)
  const float* X[NLMAX];      // input of each layer (X[0] == null -> BwdArgs.x0)
  float* dZ[NLMAX];           // gradient w.r.t. each layer's output (pre-activation)
};

struct BwdArgs {
  int M, na, nb, nc, la, lb, lc, pad_;
  LayerGeo L[NLMAX];
  AdamHP hp;
  const float* x0;
};

__device__ void role_dx(const BwdArgs& A, const BwdInst& I, int tile, floatx4 (*red)[2][64]) {
  const LayerGeo L = A.L[A.la];
  const int N = L.N, K = L.K, M = A.M;
  const int ntk = (K + 15) >> 4;
  const int k0 = (tile % ntk) * 16, m0 = (tile / ntk) * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const float* dZ = I.dZ[A.la];
  const float* W = I.P + L.wOff;
  const int ma = m0 + r, mb = m0 + 16 + r, kk = k0 + r;
  const bool oka = ma < M, okb = mb < M, okk = kk < K;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int nc = wave * 64; nc < N; nc += 256) {
    const int nb = nc + g * 16;
    float a0[16], a1[16], bw[16];
    load16(a0, dZ + (size_t)ma * N, nb, N, oka);
    load16(a1, dZ + (size_t)mb * N, nb, N, okb);
#pragma unroll
    for (int j = 0; j < 16; ++j) bw[j] = (okk && nb + j < N) ? W[(size_t)(nb + j) * K + kk] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0 = mfma4(a0[j], bw[j], acc0);
      acc1 = mfma4(a1[j], bw[j], acc1);
    }
  }
  red[wave][0][lane] = acc0;
  red[wave][1][lane] = acc1;
  __syncthreads();
  if (threadIdx.x < 128) {
    const int s = threadIdx.x >> 6, Lx = threadIdx.x & 63;
    floatx4 v = red[0][s][Lx];
    v += red[1][s][Lx];
    v += red[2][s][Lx];
    v += red[3][s][Lx];
    const int col = k0 + (Lx & 15);
    if (col < K) {
      const float* Xin = I.X[A.la];
      float* out = I.dZ[A.la - 1];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * s + (Lx >> 4) * 4 + i;
        if (row < M) out[(size_t)row * K + col] = act_bwd(v[i], Xin[(size_t)row * K + col], L.actIn);
      }
    }
  }
}

__device__ void role_dw(const BwdArgs& A, const BwdInst& I, int l, int tile) {
  const LayerGeo L = A.L[l];
  const int N = L.N, K = L.K, M = A.M;
  const int ntk = (K + 63) >> 6;
  const int kt = tile % ntk, nt = tile / ntk;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int nbase = nt * 32, n0 = nbase + (wave & 1) * 16, k0 = kt * 64 + (wave >> 1) * 32;
  const float* dZ = I.dZ[l];
  const float* X = I.X[l] ? I.X[l] : A.x0;
  const int nn = n0 + r, kb0 = k0 + r, kb1 = k0 + 16 + r;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int mb = 0; mb < M; mb += 4) {
    const int m = mb + g;
    const bool okm = m < M;
    const float a = (okm && nn < N) ? dZ[(size_t)m * N + nn] : 0.f;
    const float b0 = (okm && kb0 < K) ? X[(size_t)m * K + kb0] : 0.f;
    const float b1 = (okm && kb1 < K) ? X[(size_t)m * K + kb1] : 0.f;
    acc0 = mfma4(a, b0, acc0);
    acc1 = mfma4(a, b1, acc1);
  }
  const AdamC c = adam_consts(A.hp, *I.step);
  float* P = I.P + L.wOff;
  float* Mo = I.Mo + L.wOff;
  float* Vo = I.Vo + L.wOff;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + g * 4 + i;
    if (n < N) {
      if (kb0 < K) adam_el(P + (size_t)n * K + kb0, Mo + (size_t)n * K + kb0, Vo + (size_t)n * K + kb0, acc0[i], c);
      if (kb1 < K) adam_el(P + (size_t)n * K + kb1, Mo + (size_t)n * K + kb1, Vo + (size_t)n * K + kb1, acc1[i], c);
    }
  }
  if (kt == 0 && threadIdx.x < 32) {
    const int n = nbase + threadIdx.x;
    if (n < N) {
      float s = 0.f;
      for (int m = 0; m < M; ++m) s = __fadd_rn(s, dZ[(size_t)m * N + n]);
      adam_el(I.P + L.bOff + n, I.Mo + L.bOff + n, I.Vo + L.bOff + n, s, c);
    }
  }
}

__global__ __launch_bounds__(256) void k_bwd(const BwdInst* __restrict__ insts, BwdArgs A) {
  __shared__ floatx4 red[4][2][64];
  const BwdInst& I = insts[blockIdx.y];
  int bx = blockIdx.x;
  if (bx < A.na) {
    role_dx(A, I, bx, red);
    return;
  }
  bx -= A.na;
  if (bx < A.nb) {
    role_dw(A, I, A.lb, bx);
    return;
  }
  bx -= A.nb;
  role_dw(A, I, A.lc, bx);
}

// -------------------------------------------------------------------------------------
// GPI reduction over heads (SF.GPI_w, features/successor.py:243-246; sfdqn.py:235-240)
// psiN: head t rows at psiN + t*stride, [M, O].  One workgroup per row b.
// Also serves action selection (sfdqn.py:585-594): out[0] = c, out[1] = argmax_a q[c].
// -------------------------------------------------------------------------------------
struct GpiArgs {
  int M, T, A, d, row0, select_task, use_gpi, pad_;
  long long stride;
  const float* psiN;
  const float* w;
  float* psi_out;   // [B, T, A, d] or null  (row b -> row0 + b)
  float* q_out;     // [B, T, A] or null
  int64_t* task_out;
  int64_t* next_out;
  int64_t* sel_out;  // [2] (action selection) or null
};

__global__ __launch_bounds__(256) void k_gpi(GpiArgs A) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = A.T, Aa = A.A, d = A.d, O = Aa * d;
  __shared__ float s_q[TDG_QMAX];
  __shared__ float s_w[TDG_DMAX];
  for (int k = tid; k < d; k += 256) s_w[k] = A.w[k];
  __syncthreads();
  const long long ob = (long long)(A.row0 + b);
  for (int idx = tid; idx < T * Aa; idx += 256) {
    const int t = idx / Aa, a = idx - t * Aa;
    const float* p = A.psiN + (long long)t * A.stride + (size_t)b * O + a * d;
    float q = 0.f;
    for (int k = 0; k < d; ++k) q = __builtin_fmaf(p[k], s_w[k], q);
    s_q[idx] = q;
    if (A.q_out) A.q_out[(ob * T + t) * Aa + a] = q;
  }
  if (A.psi_out) {
    for (int idx = tid; idx < T * O; idx += 256) {
      const int t = idx / O, o = idx - t * O;
      A.psi_out[(ob * T + t) * O + o] = A.psiN[(long long)t * A.stride + (size_t)b * O + o];
    }
  }
  __syncthreads();
  if (tid == 0) {
    // task = argmax_t max_a q ; next = argmax_a max_t q  (first index on ties)
    int tb = 0;
    float tv = -INFINITY;
    for (int t = 0; t < T; ++t) {
      float mx = s_q[t * Aa];
      for (int a = 1; a < Aa; ++a) mx = s_q[t * Aa + a] > mx ? s_q[t * Aa + a] : mx;
      if (t == 0 || mx > tv) { tv = mx; tb = t; }
    }
    int ab = 0;
    float av = -INFINITY;
    for (int a = 0; a < Aa; ++a) {
      float mx = s_q[a];
      for (int t = 1; t < T; ++t) mx = s_q[t * Aa + a] > mx ? s_q[t * Aa + a] : mx;
      if (a == 0 || mx > av) { av = mx; ab = a; }
    }
    if (A.task_out) A.task_out[ob] = tb;
    if (A.next_out) A.next_out[ob] = ab;
    if (A.sel_out) {
      const int c = A.use_gpi ? tb : A.select_task;
      int act = 0;
      float best = s_q[c * Aa];
      for (int a = 1; a < Aa; ++a)
        if (s_q[c * Aa + a] > best) { best = s_q[c * Aa + a]; act = a; }
      A.sel_out[0] = c;
      A.sel_out[1] = act;
    }
  }
}

// LMS reward fit (features/successor.py:164-167): w += α (r - Σ φ⊙w) φ
__global__ void k_lms(float* __restrict__ w, const float* __restrict__ phi, const float* __restrict__ r,
                      float alpha, int d) {
  __shared__ float s_red[256];
  const int tid = threadIdx.x;
  float p = 0.f;
  for (int k = tid; k < d; k += 256) p = __fadd_rn(p, __fmul_rn(phi[k], w[k]));
  const float rfit = block_sum256(p, s_red);
  const float e = __fmul_rn(alpha, __fsub_rn(r[0], rfit));
  for (int k = tid; k < d; k += 256) w[k] = __fadd_rn(w[k], __fmul_rn(e, phi[k]));
}

}  // namespace sfx
