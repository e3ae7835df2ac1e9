// sfx_phi.h -- learned φ: features/deep_phi.py DeepSF_PHI.update_successor
// (:93-224), the library of main_sfdqn_phi_torch.py / agents/sfdqn_phi.py.  Device side.
//
// φ = phi_net(s ⊕ a ⊕ s1): Linear(n_in, hid) + ReLU, n_mid × (Linear(hid, hid) + ReLU),
// Linear(hid, d) -- main_sfdqn_phi_torch.py's phi_model_lambda with n_in = 2 n_s + 1, hid = 2 n_in.
// The update of policy i (the ψ part runs through the SF-DQN kernels with φ as the features,
// the output gradient scaled by λ_i and a fresh Adam):
//   k_phi_fwd   φ of the B rows, every hidden activation kept for the backward
//   (ψ forwards, TD target with φ, ψ backward + fresh-Adam step, l1 = psi_loss)
//   k_phi_bwd   dφ_b = -λ ∂l1/∂t_b (the ψ launch's output gradient at the taken action, already
//               scaled) + (2/B)(w·φ_b + b - r_b) w; backward through the φ net, then one fresh
//               Adam step on every φ parameter, on w_i and its bias, and λ_i ← clamp(λ_i + step
//               of ascent on psi_loss, 1e-2, 1e6); losses (loss, psi_loss, phi_loss, λ_i).
// A fresh Adam (the reference builds torch.optim.Adam inside every update) has zero moments and
// step 1: p -= lr / (1 - β1) · m / (√v / √(1 - β2) + ε) with m = (1 - β1) g, v = (1 - β2) g².
// One workgroup each: the net is tiny (n_in <= 64, hid <= 128, d <= 64) and B <= 64.
#pragma once

namespace sfx {

constexpr int PHI_IN = 64, PHI_HID = 128, PHI_B = 64, PHI_L = 8;

struct PhiArgs {
  int n_in, hid, n_mid, d, B, n_s, O, lastOff;
  int pol, pad_;
  float* p;            // [P] the φ net in torch packing (per Linear: W [out][in], b [out])
  float* acts;         // [L][B][hid] post-activation outputs of the hidden layers; [B][n_in] input after
  float* phis;         // [B][d]
  const float* S;      // [B][n_s]
  const float* S1;
  const int64_t* a;
  const float* r;      // [B]
  const float* dzlast; // [B][O]: the ψ output gradient of policy pol (λ-scaled), nonzero at a_b only
  float* w;            // [d] w_i (the reward model's weight row)
  float* wb;           // w_i's bias
  float* lam;          // λ_i
  float* losses;       // [4]: loss, psi_loss (losses[1] written by the ψ tail), phi_loss, λ_i after
  AdamHP hp;           // lr of every parameter group (1e-3 in features/deep_phi.py), β, ε
};

__device__ __forceinline__ int phi_layer_in(const PhiArgs& A, int l) { return l == 0 ? A.n_in : A.hid; }
__device__ __forceinline__ int phi_layer_out(const PhiArgs& A, int l) { return l == A.n_mid + 1 ? A.d : A.hid; }
__device__ __forceinline__ long long phi_layer_off(const PhiArgs& A, int l) {
  long long off = 0;
  for (int j = 0; j < l; ++j) off += (long long)phi_layer_out(A, j) * (phi_layer_in(A, j) + 1);
  return off;
}

// one freshly built Adam's first step on p with gradient g (maximize: ascent)
__device__ __forceinline__ float fresh_adam(float p, float g, const AdamC& c, bool maximize = false) {
  float m = 0.f, v = 0.f;
  adam_apply(p, m, v, maximize ? -g : g, c);
  return p;
}

__global__ __launch_bounds__(256) void k_phi_fwd(PhiArgs A) {
  __shared__ float sx[PHI_B * PHI_HID], sy[PHI_B * PHI_HID];
  const int tid = threadIdx.x, B = A.B, n_s = A.n_s, L = A.n_mid + 2;
  float* in_keep = A.acts + (long long)(L - 1) * B * A.hid;  // the layer-0 input, kept for dW
  for (int j = tid; j < B * A.n_in; j += 256) {
    const int b = j / A.n_in, k = j - b * A.n_in;
    const float v = k < n_s ? A.S[(long long)b * n_s + k]
                            : (k == n_s ? (float)A.a[b] : A.S1[(long long)b * n_s + (k - n_s - 1)]);
    sx[b * A.n_in + k] = v;
    in_keep[j] = v;
  }
  __syncthreads();
  float* x = sx;
  float* y = sy;
  for (int l = 0; l < L; ++l) {
    const int K = phi_layer_in(A, l), N = phi_layer_out(A, l);
    const float* W = A.p + phi_layer_off(A, l);
    const float* bias = W + (long long)N * K;
    const bool last = l == L - 1;
    for (int j = tid; j < B * N; j += 256) {
      const int b = j / N, o = j - b * N;
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc = __builtin_fmaf(x[b * K + k], W[(long long)o * K + k], acc);
      acc = __fadd_rn(acc, bias[o]);
      if (last) {
        A.phis[(long long)b * N + o] = acc;
      } else {
        acc = fmaxf(acc, 0.f);
        y[b * N + o] = acc;
        A.acts[((long long)l * B + b) * A.hid + o] = acc;
      }
    }
    __syncthreads();
    float* t = x;
    x = y;
    y = t;
  }
}

__global__ __launch_bounds__(256) void k_phi_bwd(PhiArgs A) {
  __shared__ float sg[PHI_B * PHI_HID], sg2[PHI_B * PHI_HID];
  __shared__ float s_w[PHI_IN], s_e[PHI_B];
  const int tid = threadIdx.x, B = A.B, d = A.d, L = A.n_mid + 2;
  const AdamC c1 = adam_consts(A.hp, 1);
  if (tid < d) s_w[tid] = A.w[tid];
  __syncthreads();
  const float wb = *A.wb;
  // r_fit_b - r_b with w_i before its step
  for (int b = tid; b < B; b += 256) {
    float rf = 0.f;
    for (int k = 0; k < d; ++k) rf = __builtin_fmaf(A.phis[(long long)b * d + k], s_w[k], rf);
    s_e[b] = __fsub_rn(__fadd_rn(rf, wb), A.r[b]);
  }
  __syncthreads();
  const float nrm = (float)(2.0 / (double)B);
  // dφ = -dz[b][a_b][:] (λ-scaled ∂l1/∂c; ∂/∂t is its negative) + (2/B) e_b w
  for (int j = tid; j < B * d; j += 256) {
    const int b = j / d, k = j - b * d;
    const int ab = (int)A.a[b];
    const float dz = A.dzlast[(long long)b * A.O + ab * d + k];
    sg[b * d + k] = __fadd_rn(-dz, __fmul_rn(__fmul_rn(nrm, s_e[b]), s_w[k]));
  }
  __syncthreads();
  // w_i, its bias (gradients Σ_b (2/B) e_b φ_b, Σ_b (2/B) e_b), phi_loss
  if (tid < d) {
    float g = 0.f;
    for (int b = 0; b < B; ++b) g = __builtin_fmaf(__fmul_rn(nrm, s_e[b]), A.phis[(long long)b * d + tid], g);
    A.w[tid] = fresh_adam(s_w[tid], g, c1);
  }
  if (tid == 0) {
    float gb = 0.f, sse = 0.f;
    for (int b = 0; b < B; ++b) {
      gb = __fadd_rn(gb, __fmul_rn(nrm, s_e[b]));
      sse = __builtin_fmaf(s_e[b], s_e[b], sse);
    }
    *A.wb = fresh_adam(wb, gb, c1);
    const float phi_loss = (float)((double)sse / (double)B);
    const float psi_loss = A.losses[1];
    const float lam = *A.lam;
    A.losses[0] = __fadd_rn(phi_loss, __fmul_rn(lam, psi_loss));
    A.losses[2] = phi_loss;
    const float ln = fminf(fmaxf(fresh_adam(lam, psi_loss, c1, true), 1e-2f), 1e6f);
    *A.lam = ln;
    A.losses[3] = ln;
  }
  // backward through the net, layer L-1 .. 0: dW, db (Σ over rows), then dX through the ReLU
  float* g = sg;
  float* gn = sg2;
  for (int l = L - 1; l >= 0; --l) {
    const int K = phi_layer_in(A, l), N = phi_layer_out(A, l);
    float* W = A.p + phi_layer_off(A, l);
    float* bias = W + (long long)N * K;
    const float* X = l == 0 ? A.acts + (long long)(L - 1) * B * A.hid : A.acts + (long long)(l - 1) * B * A.hid;
    const int xs = l == 0 ? A.n_in : A.hid;
    // dX first (reads W before its update)
    if (l > 0) {
      for (int j = tid; j < B * K; j += 256) {
        const int b = j / K, k = j - b * K;
        float acc = 0.f;
        for (int o = 0; o < N; ++o) acc = __builtin_fmaf(g[b * N + o], W[(long long)o * K + k], acc);
        gn[b * K + k] = X[(long long)b * xs + k] > 0.f ? acc : 0.f;  // ReLU of the layer below
      }
    }
    __syncthreads();
    for (int j = tid; j < N * K; j += 256) {
      const int o = j / K, k = j - o * K;
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc = __builtin_fmaf(g[b * N + o], X[(long long)b * xs + k], acc);
      W[j] = fresh_adam(W[j], acc, c1);
    }
    for (int o = tid; o < N; o += 256) {
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc = __fadd_rn(acc, g[b * N + o]);
      bias[o] = fresh_adam(bias[o], acc, c1);
    }
    __syncthreads();
    float* t = g;
    g = gn;
    gn = t;
  }
}

}  // namespace sfx
