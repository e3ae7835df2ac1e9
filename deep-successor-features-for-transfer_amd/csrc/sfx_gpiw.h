// sfx_gpiw.h -- GPI over many heads (T·A > 256: BASELINE config C4's 64 source tasks on one GPU and
// the all-task step at large T).  Included by sfx.hip after sfx_kernels.h.
//
// The per-row kernels (k_tdg, k_ver, k_qmax: one workgroup per (policy, row), one q = ψ·w dot per
// thread, then a serial max over heads) read every head's ψ row once PER POLICY: at T = 64 that is
// 64 × 30 MB of L2 traffic per launch and a 64-step dependent max per action -- 20 / 53 / 20 µs.
// Here one workgroup takes one minibatch row b and a chunk of WPC policies: lane = head (heads
// past 64 loop), wave w = the actions a ≡ w (mod 4).  A lane loads its head's ψ rows of the row
// once (both roles: heads before the policy in the reference's order read `lt`, the others `ge`),
// forms q for each policy of the chunk with the SAME k-ordered fmaf chain as every other GPI
// kernel (so maxima and argmaxes are bit-identical to theirs), and the wave takes the max over
// heads with shuffles (max is exact and order-free).  features/deep.py:101-103 (GPI next actions),
// sfdqn.py:313-316, features/successor.py:223-246.
#pragma once

namespace sfx {

constexpr int WPC = 8;     // policies per workgroup
constexpr int WAMAX = 32;  // actions (wide kernels)

// max over the 64 lanes of a wave, the result in every lane: DPP within rows of 16 (xor 1, xor 2,
// half-row mirror, row mirror: one VALU op each), then the four row maxima by readlane -- instead of
// six ds_bpermute shuffles per reduction (max is exact and order-free)
#define SFX_DPP_MAX(v, ctrl) \
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false)))
__device__ __forceinline__ float wave_fmax(float v) {
  SFX_DPP_MAX(v, 0xB1);   // quad_perm [1,0,3,2]
  SFX_DPP_MAX(v, 0x4E);   // quad_perm [2,3,0,1]
  SFX_DPP_MAX(v, 0x141);  // row_half_mirror
  SFX_DPP_MAX(v, 0x140);  // row_mirror
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
#undef SFX_DPP_MAX

// s_m[j][a] = max over this handle's heads t of ψ_{role(t)}(row b)[a]·w_{i0+j} for j < ni, where
// role(t) = lt if off + t < i0 + j else ge.  s_w[j][k]: the policies' w rows (in LDS, complete).
// d = 4 VD.  Every thread of the workgroup calls it; a barrier follows inside.  A wave takes the
// actions a = wave, wave + 4 (then + 8 ...), both of a pair's ψ rows requested before the first dot.
template <int VD>
__device__ __forceinline__ void wide_maxima(const Geo& G, int b, int i0, int ni, int off, int lt, int ge,
                                            const float (*s_w)[16], float (*s_m)[WAMAX]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int T = G.T, Aa = G.A, O = G.O, NLm = G.lastOff;
  const bool two = lt != ge;
  for (int a0 = wave; a0 < Aa; a0 += 8) {
    float mx[2][WPC];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < WPC; ++j) mx[u][j] = -INFINITY;
    for (int t0 = 0; t0 < T; t0 += 64) {  // wave-uniform trip count
      const int t = t0 + lane;
      const bool ok = t < T;
      float4 pl[2][VD], pg[2][VD];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int a = a0 + 4 * u;
        const bool oka = ok && a < Aa;
        const size_t ro = (size_t)b * O + (size_t)(oka ? a : 0) * 4 * VD;
        const float4* rl = reinterpret_cast<const float4*>(G.actp(lt, ok ? t : 0, NLm) + ro);
        const float4* rg = reinterpret_cast<const float4*>(G.actp(ge, ok ? t : 0, NLm) + ro);
#pragma unroll
        for (int v = 0; v < VD; ++v) {
          pl[u][v] = oka ? rl[v] : make_float4(0.f, 0.f, 0.f, 0.f);
          pg[u][v] = oka && two ? rg[v] : pl[u][v];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < WPC; ++j) {
          if (j < ni) {
            const bool before = off + t < i0 + j;
            float q = 0.f;
#pragma unroll
            for (int v = 0; v < VD; ++v) {
              const float4 p = before ? pl[u][v] : pg[u][v];
              q = __builtin_fmaf(p.x, s_w[j][4 * v], q);
              q = __builtin_fmaf(p.y, s_w[j][4 * v + 1], q);
              q = __builtin_fmaf(p.z, s_w[j][4 * v + 2], q);
              q = __builtin_fmaf(p.w, s_w[j][4 * v + 3], q);
            }
            if (ok) mx[u][j] = fmaxf(mx[u][j], q);
          }
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int a = a0 + 4 * u;
      if (a < Aa) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < WPC; ++j) {
          const float m = wave_fmax(mx[u][j]);
          if (lane == 0 && j < ni) s_m[j][a] = m;
        }
      }
    }
  }
  __syncthreads();
}

// the first argmax over actions of s_m[j] (torch.argmax's first index; -0 == +0)
__device__ __forceinline__ int wide_argmax(const float* m, int Aa) {
  int am = 0;
  float qm = m[0];
  for (int a = 1; a < Aa; ++a)
    if (m[a] > qm) {
      qm = m[a];
      am = a;
    }
  return am;
}

// the policies' w rows into LDS (s_w[j][k], k < d)
__device__ __forceinline__ void wide_load_w(const Geo& G, int i0, int ni, float (*s_w)[16]) {
  const int tid = threadIdx.x, d = G.d;
  if (tid < WPC * 16) {
    const int j = tid >> 4, k = tid & 15;
    s_w[j][k] = j < ni && k < d ? G.w[(long long)(i0 + j) * G.dpad + k] : 0.f;
  }
}

// k_qmax over many heads: X[(i - pol0) * M + b][a] = sortable(max over local heads), grid
// (M, cdiv(npol, WPC)).  QmaxArgs as k_qmax (tsel < 0 only).
template <int VD>
__global__ __launch_bounds__(256) void k_qmaxw(Geo G, QmaxArgs Q) {
  __shared__ float s_w[WPC][16];
  __shared__ float s_m[WPC][WAMAX];
  const int b = blockIdx.x, i0 = blockIdx.y * WPC, ni = min(WPC, Q.Tg - i0);  // pol0 == 0 (host)
  wide_load_w(G, i0, ni, s_w);
  __syncthreads();
  wide_maxima<VD>(G, b, i0, ni, Q.off, Q.guess, R_S1, s_w, s_m);
  const int Aa = G.A;
  for (int e = threadIdx.x; e < ni * Aa; e += 256) {
    const int j = e / Aa, a = e - j * Aa;
    Q.X[((size_t)(i0 + j) * Q.M + b) * Aa + a] = sortable(s_m[j][a]);
  }
}

// k_ver over many heads: policy i's next actions from the round's post-update heads (t < i) and
// the pre-step heads (t >= i) against the ones the round used; flag = first policy that differs.
// Grid (M, cdiv(npol, WPC) + 1): the extra chunk's row-0 workgroup selects the env action (gpi_row);
// the publication folds in as in k_ver (VerArgs::pub: the last workgroup to arrive posts it).
template <int VD>
__global__ __launch_bounds__(256) void k_verw(Geo G, VerArgs V) {
  __shared__ float s_w[WPC][16];
  __shared__ float s_m[WPC][WAMAX];
  __shared__ int s_bad;
  const int b = blockIdx.x, chunk = blockIdx.y, nchunk = gridDim.y - 1;
  if (chunk == nchunk) {
    if (V.sel && b == 0) gpi_row(G, V.g, 0);
  } else {
    const int i0 = chunk * WPC, ni = min(WPC, V.npol - i0);
    if (threadIdx.x == 0) s_bad = V.npol;
    wide_load_w(G, i0, ni, s_w);
    __syncthreads();
    wide_maxima<VD>(G, b, i0, ni, 0, V.post, R_S1, s_w, s_m);
    if (threadIdx.x < ni && i0 + threadIdx.x > 0) {  // policy 0 sees only pre-update heads: exact
      const int j = threadIdx.x;
      const int am = wide_argmax(s_m[j], G.A);
      SFX_CHK(b < V.spec_stride, i0 + j, b, V.spec_stride);
      if (am != (int)V.spec_next[(size_t)(i0 + j) * V.spec_stride + b]) atomicMin(&s_bad, i0 + j);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_bad < V.npol) atomicMin(V.flag, s_bad);
  }
  if (V.pub || V.h_flag) {  // as k_ver: the barrier + agent-scope arrival order every wave's stores before it
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = __hip_atomic_fetch_add(V.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned)V.nblocks - 1) {
        if (V.pub)
          publish_result(V.g.sel_out, V.flag, V.pub, V.pub_dctr, G.cancel, G.nonfin);
        else
          post_verdict(V);
        __hip_atomic_store(V.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

struct TdgwArgs {
  int M, pol0, npol, guess, next_stride, flag_value;
  const int64_t* a;
  const float* phi;
  const float* gamma;
  int64_t* next;    // next[(pol - pol0) * next_stride + b]
  int* flag;        // reset to flag_value by workgroup (0, 0)
  const int64_t* prev;  // round skipping (tdg_skip_report); null: no previous round
  int* skip;
  unsigned long long* skipc;
};

// K2 over many heads (the GPI branch of k_tdg; sfdqn.py:313-341, features/deep.py:101-120): grid
// (M, cdiv(npol, WPC)), policies pol0 .. pol0 + npol - 1 (local heads).  The next actions of WPC policies for row b, then each policy's TD target,
// output-gradient row and row loss with k_tdg's arithmetic in k_tdg's order.
template <int VD>
__global__ __launch_bounds__(256) void k_tdgw(Geo G, TdgwArgs W) {
  __shared__ float s_w[WPC][16];
  __shared__ float s_m[WPC][WAMAX];
  __shared__ int s_n[WPC];
  const int b = blockIdx.x, i0 = W.pol0 + blockIdx.y * WPC, ni = min(WPC, W.pol0 + W.npol - i0), tid = threadIdx.x;
  const int Aa = G.A, d = G.d, O = G.O, NLm = G.lastOff, M = W.M;
  if (W.flag && b == 0 && blockIdx.y == 0 && tid == 0) *W.flag = W.flag_value;
  wide_load_w(G, i0, ni, s_w);
  __syncthreads();
  wide_maxima<VD>(G, b, i0, ni, 0, W.guess, R_S1, s_w, s_m);
  if (tid < ni) {
    const int am = wide_argmax(s_m[tid], Aa);
    s_n[tid] = am;
    const size_t ni_ = (size_t)(i0 + tid - W.pol0) * W.next_stride + b;
    SFX_CHK(b < W.next_stride, i0 + tid, b, W.next_stride);
    if (W.next) W.next[ni_] = am;
    if (W.skip) tdg_skip_report(W.skip, W.skipc, i0 + tid, G.T, !W.prev || W.prev[ni_] != am, W.prev != nullptr, M);
  }
  __syncthreads();
  const int ab = (int)W.a[b];
  const bool aok = ab >= 0 && ab < Aa;
  const float gam = W.gamma[b];
  const float norm = td_norm(G, M, O, nullptr);
  // output-gradient rows: nonzero only at the taken action (k_tdg's stage, one thread per entry)
  for (int e = tid; e < ni * O; e += 256) {
    const int j = e / O, o = e - j * O, pol = i0 + j;
    float gv = 0.f;
    if (aok && o >= ab * d && o < ab * d + d) {
      const int k = o - ab * d;
      const float tv = G.actp(R_S1T, pol, NLm)[(size_t)b * O + s_n[j] * d + k];
      const float tg = __fadd_rn(W.phi[(size_t)b * d + k], __fmul_rn(gam, tv));
      gv = td_grad(G.huber, norm, __fsub_rn(G.actp(R_S, pol, NLm)[(size_t)b * O + o], tg));
    }
    G.dzp(pol, NLm)[(size_t)b * O + o] = gv;
  }
  // row losses, Σ over features in feature order (one thread per policy)
  if (tid < ni) {
    const int pol = i0 + tid;
    float s = 0.f;
    int nf = 0;
    if (aok) {
      const float* trow = G.actp(R_S1T, pol, NLm) + (size_t)b * O + s_n[tid] * d;
      const float* crow = G.actp(R_S, pol, NLm) + (size_t)b * O + ab * d;
      for (int k = 0; k < d; ++k) {
        const float diff = __fsub_rn(crow[k], __fadd_rn(W.phi[(size_t)b * d + k], __fmul_rn(gam, trow[k])));
        s = __fadd_rn(s, td_loss(G.huber, diff));
        nf |= !__builtin_isfinite(diff);
      }
    }
    if (nf && G.nonfin) atomicOr(G.nonfin, 1);
    SFX_CHK(pol >= 0 && pol < G.T && b < MMAX, pol, b, 0);
    G.rowloss[(long long)pol * MMAX + b] = s;
  }
}

}  // namespace sfx
