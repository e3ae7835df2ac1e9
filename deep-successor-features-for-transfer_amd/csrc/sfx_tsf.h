// sfx_tsf.h -- TSF-DQN's transformed features (tsfdqn.py:588-709, tsfdqn_nf.py): device side.
//
// Per task i a state transform g_i (K planar flows z <- z + u_k tanh(w_k·z + b_k), then
// Linear(n_s, G); K = 0 is tsfdqn.py's plain Linear) and ONE affine map h = Linear(G, d) shared
// by all tasks give the transformed features
//     φ̃ = (h(g_i(s)) + h(g_i(s1))) ⊙ φ
// which replace φ in the TD target (t = φ̃ + γ ψ⁻_i(s1)[a'], so l1 trains g_i and h too) and in
// l2 = MSE(w_i·φ̃, r); loss = l1 + β l2 and one Adam step over {ψ_i, w_i, g_i, h}.
//
// The ψ part runs through the SF-DQN kernels with φ̃ as the features; these two single-
// workgroup kernels do the rest: k_tsf_fwd (φ̃ and the saved activations) before the TD
// target, k_tsf_bwd (w_i, g_i, h gradients + Adam, l2) after the ψ backward.
// Limits (checked by sfx_tsf_setup): n_s <= 32, B <= 64, d*G <= 8192, 2B*G <= 8192,
// B*d <= 4096, B*G <= 4096, K(2 n_s + 1) + G(n_s + 1) <= 4096.
#pragma once

namespace sfx {

constexpr int TSF_NS = 32;     // max n_s (flow state in registers)
constexpr int TSF_LDS = 8192;  // floats per staged operand (flows, W_h, g features)

struct TsfArgs {
  int pol, B, n_s, G, K, d, Pg, Ph, O, lastOff;
  float beta;
  const float* S;
  const float* S1;
  const float* phi;
  const float* r;
  const int64_t* a;
  float* g;  // [T][Pg]: flow k at k*(2n_s+1) (w[n_s], b, u[n_s]); Linear W[G][n_s] at K*(2n_s+1), then b[G]
  float* gm;
  float* gv;
  float* hp;  // [Ph]: W_h[d][G] then b_h[d]
  float* hm;  // [T][Ph] (each task's optimizer keeps its own moments of the shared h)
  float* hv;
  float* zs;     // [K+1][2B][n_s] flow states (rows 0..B-1: s, B..2B-1: s1)
  float* ts;     // [K][2B] tanh outputs
  float* gfeat;  // [2B][G]
  float* tphi;   // [B][d]
  float* part;   // [K][2B][2n_s+1] per-row flow-parameter gradients
  float* losses; // [3]: [1] = l1 (written by the ψ tail); [0], [2] written here
  const float* dzlast;  // output gradient of the policy's ψ head [B][O] (written by K2)
  const int* step;      // Adam step of the policy (already bumped by the ψ path)
  float* w;             // [d] reward weights of the policy (+ moments)
  float* wm;
  float* wv;
  AdamHP hpw, hpg, hph;
};

__device__ __forceinline__ int tsf_flow_stride(int n_s) { return 2 * n_s + 1; }

__global__ __launch_bounds__(256) void k_tsf_fwd(TsfArgs A) {
  __shared__ float s_fl[TSF_LDS];  // flow parameters, then the Linear of g
  __shared__ float s_wh[TSF_LDS];  // W_h
  __shared__ float s_gf[TSF_LDS];  // g features of the 2B rows
  __shared__ float s_z[4 * TSF_NS * 32];
  const int tid = threadIdx.x, n_s = A.n_s, G = A.G, K = A.K, d = A.d, B = A.B, R2 = 2 * B;
  const int fs = tsf_flow_stride(n_s), nfl = K * fs, nlin = G * n_s + G;
  const float* gp = A.g + (long long)A.pol * A.Pg;
  for (int j = tid; j < nfl + nlin; j += 256) s_fl[j] = gp[j];
  for (int j = tid; j < d * G; j += 256) s_wh[j] = A.hp[j];
  __syncthreads();
  // planar flows, one thread per row (state in registers); save z_k and t_k for the backward
  for (int row = tid; row < R2; row += 256) {
    const float* x = row < B ? A.S + (size_t)row * n_s : A.S1 + (size_t)(row - B) * n_s;
    float z[TSF_NS];
#pragma unroll
    for (int i = 0; i < TSF_NS; ++i) z[i] = i < n_s ? x[i] : 0.f;
    for (int k = 0; k < K; ++k) {
      const float* f = s_fl + k * fs;
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < TSF_NS; ++i)
        if (i < n_s) acc = __builtin_fmaf(z[i], f[i], acc);
      const float t = tanhf(__fadd_rn(acc, f[n_s]));
      float* zk = A.zs + ((size_t)k * R2 + row) * n_s;
#pragma unroll
      for (int i = 0; i < TSF_NS; ++i)
        if (i < n_s) {
          zk[i] = z[i];
          z[i] = __fadd_rn(z[i], __fmul_rn(f[n_s + 1 + i], t));
        }
      A.ts[(size_t)k * R2 + row] = t;
    }
    float* zK = A.zs + ((size_t)K * R2 + row) * n_s;
#pragma unroll
    for (int i = 0; i < TSF_NS; ++i)
      if (i < n_s) {
        zK[i] = z[i];
        s_z[row * n_s + i] = z[i];
      }
  }
  __syncthreads();
  // Linear(n_s, G) of g
  const float* Wl = s_fl + nfl;
  const float* bl = Wl + G * n_s;
  for (int j = tid; j < R2 * G; j += 256) {
    const int row = j / fdiv(G), c = j - row * G;
    float acc = 0.f;
    for (int i = 0; i < n_s; ++i) acc = __builtin_fmaf(s_z[row * n_s + i], Wl[c * n_s + i], acc);
    const float v = __fadd_rn(acc, bl[c]);
    s_gf[j] = v;
    A.gfeat[j] = v;
  }
  __syncthreads();
  // φ̃ = (h(g(s)) + h(g(s1))) ⊙ φ
  const float* bh = A.hp + d * G;
  for (int j = tid; j < B * d; j += 256) {
    const int b = j / fdiv(d), c = j - b * d;
    float h0 = 0.f, h1 = 0.f;
    for (int q = 0; q < G; ++q) {
      h0 = __builtin_fmaf(s_gf[b * G + q], s_wh[c * G + q], h0);
      h1 = __builtin_fmaf(s_gf[(B + b) * G + q], s_wh[c * G + q], h1);
    }
    const float bb = bh[c];
    const float aff = __fadd_rn(__fadd_rn(h0, bb), __fadd_rn(h1, bb));
    A.tphi[j] = __fmul_rn(aff, A.phi[j]);
  }
}

__global__ __launch_bounds__(256) void k_tsf_bwd(TsfArgs A) {
  __shared__ float s_wh[TSF_LDS];      // W_h before its update (+ dg [B][G] when it fits)
  __shared__ float s_gf[TSF_LDS];      // g features [2B][G]
  __shared__ float s_da[TSF_LDS / 2];  // daff [B][d]
  __shared__ float s_tp[TSF_LDS / 2];  // φ̃ [B][d], then dg [B][G] when it does not fit after W_h
  __shared__ float s_fl[TSF_LDS / 2];  // g parameters (flows + Linear) before the update
  __shared__ float s_w[256], s_gw[256], s_dr[64], s_red[256];
  const int tid = threadIdx.x, n_s = A.n_s, G = A.G, K = A.K, d = A.d, B = A.B, R2 = 2 * B, O = A.O;
  const int fs = tsf_flow_stride(n_s), nfl = K * fs, nlin = G * n_s + G;
  const FDiv fd = fdiv(d), fG = fdiv(G);
  float* gp = A.g + (long long)A.pol * A.Pg;
  for (int j = tid; j < d * G; j += 256) s_wh[j] = A.hp[j];
  for (int j = tid; j < R2 * G; j += 256) s_gf[j] = A.gfeat[j];
  for (int j = tid; j < B * d; j += 256) s_tp[j] = A.tphi[j];
  for (int j = tid; j < nfl + nlin; j += 256) s_fl[j] = gp[j];
  if (tid < d) s_w[tid] = A.w[tid];
  __syncthreads();
  // l2 = MSE(w·φ̃, r): dr_b = β (2/B) (r_fit_b - r_b)
  float se = 0.f;
  const float bnorm = __fmul_rn(A.beta, (float)(2.0 / (double)B));
  for (int b = tid; b < B; b += 256) {
    float rf = 0.f;
    for (int j = 0; j < d; ++j) rf = __builtin_fmaf(s_tp[b * d + j], s_w[j], rf);
    const float e = __fsub_rn(rf, A.r[b]);
    se = __builtin_fmaf(e, e, se);
    s_dr[b] = __fmul_rn(bnorm, e);
  }
  se = block_sum(se, s_red);
  // g_w = drᵀ φ̃ ; dφ̃ = -g_l1[b, a_b, :] + dr w ; daff = dφ̃ ⊙ φ
  if (tid < d) {
    float gw = 0.f;
    for (int b = 0; b < B; ++b) gw = __builtin_fmaf(s_dr[b], s_tp[b * d + tid], gw);
    s_gw[tid] = gw;
  }
  for (int j = tid; j < B * d; j += 256) {
    const int b = j / fd, c = j - b * d;
    const int ab = (int)A.a[b];
    const float gc = (ab >= 0 && ab * d < O) ? A.dzlast[(size_t)b * O + ab * d + c] : 0.f;
    const float dt = __fadd_rn(-gc, __fmul_rn(s_dr[b], s_w[c]));
    s_da[j] = __fmul_rn(dt, A.phi[j]);
  }
  __syncthreads();
  const int step = *A.step;
  // h: g_Wh = daffᵀ g(s) + daffᵀ g(s1) ; g_bh = 2 Σ_b daff   (Adam with this task's moments)
  {
    const AdamC c = adam_consts(A.hph, step);
    float* hm = A.hm + (long long)A.pol * A.Ph;
    float* hv = A.hv + (long long)A.pol * A.Ph;
    for (int j = tid; j < d * G; j += 256) {
      const int c0 = j / fG, q = j - c0 * G;
      float g0 = 0.f, g1 = 0.f;
      for (int b = 0; b < B; ++b) {
        g0 = __builtin_fmaf(s_da[b * d + c0], s_gf[b * G + q], g0);
        g1 = __builtin_fmaf(s_da[b * d + c0], s_gf[(B + b) * G + q], g1);
      }
      adam_el(A.hp + j, hm + j, hv + j, __fadd_rn(g0, g1), c);
    }
    for (int c0 = tid; c0 < d; c0 += 256) {
      float sb = 0.f;
      for (int b = 0; b < B; ++b) sb = __fadd_rn(sb, s_da[b * d + c0]);
      adam_el(A.hp + d * G + c0, hm + d * G + c0, hv + d * G + c0, __fmul_rn(2.f, sb), c);
    }
  }
  // w
  if (tid < d) adam_el(A.w + tid, A.wm + tid, A.wv + tid, s_gw[tid], adam_consts(A.hpw, step));
  // dg = daff W_h (identical for the s and s1 rows)
  __syncthreads();
  float* s_dg = s_wh + d * G;  // after W_h in the same buffer when it fits, else reuse s_tp
  const bool dg_in_wh = d * G + B * G <= TSF_LDS;
  if (!dg_in_wh) s_dg = s_tp;
  for (int j = tid; j < B * G; j += 256) {
    const int b = j / fG, q = j - b * G;
    float acc = 0.f;
    for (int c0 = 0; c0 < d; ++c0) acc = __builtin_fmaf(s_da[b * d + c0], s_wh[c0 * G + q], acc);
    s_dg[j] = acc;
  }
  __syncthreads();
  const AdamC cg = adam_consts(A.hpg, step);
  float* gm = A.gm + (long long)A.pol * A.Pg;
  float* gv = A.gv + (long long)A.pol * A.Pg;
  const float* Wl = s_fl + nfl;
  // Linear of g: dW = dgᵀ z_K(s) + dgᵀ z_K(s1) ; db = Σ dg + Σ dg
  for (int j = tid; j < G * n_s; j += 256) {
    const int q = j / fdiv(n_s), i = j - q * n_s;
    float g0 = 0.f, g1 = 0.f;
    for (int b = 0; b < B; ++b) {
      g0 = __builtin_fmaf(s_dg[b * G + q], A.zs[((size_t)K * R2 + b) * n_s + i], g0);
      g1 = __builtin_fmaf(s_dg[b * G + q], A.zs[((size_t)K * R2 + B + b) * n_s + i], g1);
    }
    adam_el(gp + nfl + j, gm + nfl + j, gv + nfl + j, __fadd_rn(g0, g1), cg);
  }
  for (int q = tid; q < G; q += 256) {
    float sb = 0.f;
    for (int b = 0; b < B; ++b) sb = __fadd_rn(sb, s_dg[b * G + q]);
    const int o = nfl + G * n_s + q;
    adam_el(gp + o, gm + o, gv + o, __fadd_rn(sb, sb), cg);
  }
  // planar flows, backward per row: dz = dg W ; for k = K-1..0: t = t_k, da = (dz·u_k)(1 - t²),
  // per-row parts du_k = dz t, dw_k = da z_k, db_k = da ; dz += da w_k
  for (int row = tid; row < R2 && K > 0; row += 256) {
    const int b = row < B ? row : row - B;
    float dz[TSF_NS];
#pragma unroll
    for (int i = 0; i < TSF_NS; ++i) {
      float acc = 0.f;
      if (i < n_s)
        for (int q = 0; q < G; ++q) acc = __builtin_fmaf(s_dg[b * G + q], Wl[q * n_s + i], acc);
      dz[i] = acc;
    }
    for (int k = K - 1; k >= 0; --k) {
      const float* f = s_fl + k * fs;
      const float t = A.ts[(size_t)k * R2 + row];
      const float* zk = A.zs + ((size_t)k * R2 + row) * n_s;
      float* pr = A.part + ((size_t)k * R2 + row) * fs;
      float su = 0.f;
#pragma unroll
      for (int i = 0; i < TSF_NS; ++i)
        if (i < n_s) {
          su = __builtin_fmaf(dz[i], f[n_s + 1 + i], su);
          pr[n_s + 1 + i] = __fmul_rn(dz[i], t);
        }
      const float da = __fmul_rn(su, __fsub_rn(1.f, __fmul_rn(t, t)));
#pragma unroll
      for (int i = 0; i < TSF_NS; ++i)
        if (i < n_s) {
          pr[i] = __fmul_rn(da, zk[i]);
          dz[i] = __fadd_rn(dz[i], __fmul_rn(da, f[i]));
        }
      pr[n_s] = da;
    }
  }
  __syncthreads();
  // flow parameter gradients: Σ over the s rows + Σ over the s1 rows, then Adam
  for (int j = tid; j < nfl; j += 256) {
    const int k = j / fdiv(fs), e = j - k * fs;
    float g0 = 0.f, g1 = 0.f;
    for (int b = 0; b < B; ++b) {
      g0 = __fadd_rn(g0, A.part[((size_t)k * R2 + b) * fs + e]);
      g1 = __fadd_rn(g1, A.part[((size_t)k * R2 + B + b) * fs + e]);
    }
    adam_el(gp + j, gm + j, gv + j, __fadd_rn(g0, g1), cg);
  }
  if (tid == 0 && A.losses) {
    const float l2 = (float)((double)se / (double)B);
    A.losses[2] = l2;
    A.losses[0] = __fadd_rn(A.losses[1], __fmul_rn(A.beta, l2));
  }
}

}  // namespace sfx
