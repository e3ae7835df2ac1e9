// sfx.hip -- libsfx.so: C ABI (include/sfx.h) + launch orchestration for gfx950.
//
// Device state of one handle (T local ψ heads), all fp32:
//   online/target/adam_m/adam_v : [T][P]      packed heads, every tensor 16-B aligned
//   w, wm, wv                   : [T][dpad]   reward weights and their Adam moments
//   step                        : [T]         Adam step per head (device-resident)
//   act                         : [role][T][actSize]   per-layer outputs, rows = max_batch
//   dz                          : [T][actSize]         per-layer output gradients
// Every kernel reads its pointers from static descriptor tables built at create time,
// so the per-call host work is a handful of launches with scalar arguments.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sfx_kernels.h"
#include "../../include/sfx.h"

using namespace sfx;

static thread_local std::string g_err;

#define SFX_FAIL(code, msg)  \
  do {                       \
    g_err = (msg);           \
    return (code);           \
  } while (0)

#define HIPCHK(x)                                                            \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_);                \
      return SFX_E_HIP;                                                      \
    }                                                                        \
  } while (0)

#define LAUNCHCHK()                                                          \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      g_err = std::string("kernel launch: ") + hipGetErrorString(e_);        \
      return SFX_E_HIP;                                                      \
    }                                                                        \
  } while (0)

namespace {

struct Layer {
  int N, K, wOff, bOff, actOut;
};

enum Role { R_S = 0, R_S1T = 1, R_S1 = 2, R_G = 3, R_A = 4, NROLE = 5 };

inline int align4(int x) { return (x + 3) & ~3; }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace

struct sfx_handle {
  int T = 0, n_s = 0, H = 0, nh = 0, A = 0, d = 0, O = 0, NL = 0, Mmax = 0, device = 0;
  int P = 0, Ptorch = 0, dpad = 0, actSize = 0;
  std::vector<Layer> L;
  std::vector<int> actOff;
  hipStream_t stream = nullptr;
  AdamHP hp_psi{1e-3, 0.0, 0.9, 0.999, 1e-8};
  AdamHP hp_w{1e-3, 0.0, 0.9, 0.999, 1e-8};
  int target_update_ev = 1000;
  std::vector<int> since_target, host_step;

  float *online = nullptr, *target = nullptr, *am = nullptr, *av = nullptr;
  float *w = nullptr, *wm = nullptr, *wv = nullptr;
  int* step = nullptr;
  float* act = nullptr;
  float* dz = nullptr;

  FwdInst* d_fwd = nullptr;
  BwdInst* d_bwd = nullptr;
  TdgInst* d_tdg = nullptr;
  // fwd plan bases (index into d_fwd)
  std::vector<int> plan_upd[2];  // [use_gpi][policy]
  int plan_all = 0;
  std::vector<int> plan_refwd;   // [policy]
  int plan_gpi = 0, plan_act = 0;

  float* actp(int role, int head, int layer) const {
    return act + ((size_t)role * T + head) * actSize + actOff[layer];
  }
  float* dzp(int head, int layer) const { return dz + (size_t)head * actSize + actOff[layer]; }
  float* params(int which, int head) const { return (which ? target : online) + (size_t)head * P; }
};

namespace {

struct InstSpec {
  int role, head, which, xsel;
};

int add_fwd_plan(const sfx_handle* h, std::vector<FwdInst>& all, const std::vector<InstSpec>& specs) {
  const int base = (int)all.size();
  for (int l = 0; l < h->NL; ++l) {
    for (const InstSpec& s : specs) {
      FwdInst f{};
      const float* p = h->params(s.which, s.head);
      f.W = p + h->L[l].wOff;
      f.b = p + h->L[l].bOff;
      f.Y = h->actp(s.role, s.head, l);
      if (l == 0) {
        f.xsel = s.xsel;
        f.X = nullptr;
      } else {
        f.xsel = 0;
        f.X = h->actp(s.role, s.head, l - 1);
      }
      all.push_back(f);
    }
  }
  return base;
}

int run_fwd(sfx_handle* h, int base, int ninst, int M, const float* xa, const float* xb) {
  for (int l = 0; l < h->NL; ++l) {
    const Layer& L = h->L[l];
    hipLaunchKernelGGL(k_fwd, dim3(cdiv(L.N, 16), ninst, cdiv(M, 32)), dim3(256), 0, h->stream,
                       h->d_fwd + base + (size_t)l * ninst, M, L.N, L.K, L.actOut, xa, xb);
  }
  LAUNCHCHK();
  return SFX_OK;
}

int run_bwd(sfx_handle* h, int desc, int ninst, int M, const float* x0) {
  BwdArgs A{};
  A.M = M;
  for (int l = 0; l < h->NL; ++l) {
    const Layer& L = h->L[l];
    A.L[l] = LayerGeo{L.N, L.K, L.wOff, L.bOff, l > 0 ? h->L[l - 1].actOut : ACT_NONE};
  }
  A.hp = h->hp_psi;
  A.x0 = x0;
  auto dw_tiles = [&](int l) { return cdiv(h->L[l].N, 32) * cdiv(h->L[l].K, 64); };
  for (int l = h->NL - 1; l >= 1; --l) {
    A.la = l;
    A.na = cdiv(M, 32) * cdiv(h->L[l].K, 16);
    if (l + 1 <= h->NL - 1) {
      A.lb = l + 1;
      A.nb = dw_tiles(l + 1);
    } else {
      A.lb = -1;
      A.nb = 0;
    }
    A.lc = -1;
    A.nc = 0;
    hipLaunchKernelGGL(k_bwd, dim3(A.na + A.nb, ninst), dim3(256), 0, h->stream, h->d_bwd + desc, A);
  }
  A.la = -1;
  A.na = 0;
  A.lb = 1;
  A.nb = dw_tiles(1);
  A.lc = 0;
  A.nc = dw_tiles(0);
  hipLaunchKernelGGL(k_bwd, dim3(A.nb + A.nc, ninst), dim3(256), 0, h->stream, h->d_bwd + desc, A);
  LAUNCHCHK();
  return SFX_OK;
}

int run_tdg(sfx_handle* h, int policy, int M, int use_gpi, const int64_t* a, const float* r,
            const float* phi, const float* gamma, float* losses, int64_t* next) {
  TdgArgs A{};
  A.M = M;
  A.T = h->T;
  A.A = h->A;
  A.d = h->d;
  A.use_gpi = use_gpi;
  A.train_w = r != nullptr;
  A.inc_step = 1;
  A.psiN_stride = h->actSize;
  A.a = a;
  A.phi = phi;
  A.gamma = gamma;
  A.r = r;
  A.hpw = h->hp_w;
  A.losses = losses;
  A.next = next;
  hipLaunchKernelGGL(k_tdg, dim3(1), dim3(256), 0, h->stream, h->d_tdg + policy, A);
  LAUNCHCHK();
  return SFX_OK;
}

void after_update(sfx_handle* h, int t) {
  h->host_step[t] += 1;
  h->since_target[t] += 1;
}

int maybe_sync_target(sfx_handle* h, int t) {
  if (h->since_target[t] >= h->target_update_ev) {
    HIPCHK(hipMemcpyAsync(h->params(1, t), h->params(0, t), sizeof(float) * h->P,
                          hipMemcpyDeviceToDevice, h->stream));
    h->since_target[t] = 0;
  }
  return SFX_OK;
}

// torch packing <-> aligned packing of one head
void pack_head(const sfx_handle* h, const float* src, float* dst) {
  std::memset(dst, 0, sizeof(float) * h->P);
  size_t off = 0;
  for (const Layer& L : h->L) {
    std::memcpy(dst + L.wOff, src + off, sizeof(float) * L.N * L.K);
    off += (size_t)L.N * L.K;
    std::memcpy(dst + L.bOff, src + off, sizeof(float) * L.N);
    off += L.N;
  }
}

void unpack_head(const sfx_handle* h, const float* src, float* dst) {
  size_t off = 0;
  for (const Layer& L : h->L) {
    std::memcpy(dst + off, src + L.wOff, sizeof(float) * L.N * L.K);
    off += (size_t)L.N * L.K;
    std::memcpy(dst + off, src + L.bOff, sizeof(float) * L.N);
    off += L.N;
  }
}

bool valid_head(const sfx_handle* h, int t) { return h && t >= 0 && t < h->T; }

int free_all(sfx_handle* h) {
  (void)hipFree(h->online);
  (void)hipFree(h->target);
  (void)hipFree(h->am);
  (void)hipFree(h->av);
  (void)hipFree(h->w);
  (void)hipFree(h->wm);
  (void)hipFree(h->wv);
  (void)hipFree(h->step);
  (void)hipFree(h->act);
  (void)hipFree(h->dz);
  (void)hipFree(h->d_fwd);
  (void)hipFree(h->d_bwd);
  (void)hipFree(h->d_tdg);
  return SFX_OK;
}

}  // namespace

extern "C" {

const char* sfx_version(void) { return "sfx 0.1 gfx950 fp32-mfma"; }
const char* sfx_last_error(void) { return g_err.c_str(); }

int sfx_create(sfx_t* out, int T, int n_s, int H, int n_hidden, const int* acts, int A, int d,
               int max_batch, int device, void* stream) {
  if (!out) SFX_FAIL(SFX_E_ARG, "out is null");
  *out = nullptr;
  if (T < 1 || n_s < 1 || H < 1 || n_hidden < 0 || n_hidden + 2 > NLMAX || A < 1 || d < 1 ||
      max_batch < 1)
    SFX_FAIL(SFX_E_ARG, "bad geometry");
  if (d > TDG_DMAX || max_batch > TDG_MMAX || (long)max_batch * A > TDG_QMAX || (long)T * A > TDG_QMAX)
    SFX_FAIL(SFX_E_ARG, "geometry exceeds kernel limits (d<=256, batch<=1024, batch*A and T*A <= 8192)");
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
  // layers
  int off = 0, ptorch = 0;
  for (int l = 0; l < h->NL; ++l) {
    Layer Lr{};
    if (l == 0) {
      Lr.N = H; Lr.K = n_s; Lr.actOut = ACT_NONE;
    } else if (l == h->NL - 1) {
      Lr.N = h->O; Lr.K = H; Lr.actOut = ACT_NONE;
    } else {
      Lr.N = H; Lr.K = H; Lr.actOut = acts[l - 1];
    }
    Lr.wOff = align4(off);
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
    aoff += align4(max_batch * h->L[l].N);
  }
  h->actSize = (aoff + 63) & ~63;
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
  alloc((void**)&h->online, headBytes);
  alloc((void**)&h->target, headBytes);
  alloc((void**)&h->am, headBytes);
  alloc((void**)&h->av, headBytes);
  alloc((void**)&h->w, wBytes);
  alloc((void**)&h->wm, wBytes);
  alloc((void**)&h->wv, wBytes);
  alloc((void**)&h->step, sizeof(int) * T);
  alloc((void**)&h->act, sizeof(float) * (size_t)NROLE * T * h->actSize);
  alloc((void**)&h->dz, sizeof(float) * (size_t)T * h->actSize);
  if (rc != SFX_OK) {
    free_all(h);
    delete h;
    return rc;
  }

  // static launch descriptors
  std::vector<FwdInst> fwd;
  for (int g = 0; g < 2; ++g) {
    for (int i = 0; i < T; ++i) {
      std::vector<InstSpec> specs = {{R_S, i, 0, 1}, {R_S1T, i, 1, 2}};
      if (g) {
        for (int t = 0; t < T; ++t) specs.push_back({R_S1, t, 0, 2});
      } else {
        specs.push_back({R_S1, i, 0, 2});
      }
      h->plan_upd[g].push_back(add_fwd_plan(h, fwd, specs));
    }
  }
  {
    std::vector<InstSpec> specs;
    for (int t = 0; t < T; ++t) specs.push_back({R_S, t, 0, 1});
    for (int t = 0; t < T; ++t) specs.push_back({R_S1T, t, 1, 2});
    for (int t = 0; t < T; ++t) specs.push_back({R_S1, t, 0, 2});
    h->plan_all = add_fwd_plan(h, fwd, specs);
  }
  for (int i = 0; i < T; ++i) h->plan_refwd.push_back(add_fwd_plan(h, fwd, {{R_S1, i, 0, 2}}));
  {
    std::vector<InstSpec> g, a;
    for (int t = 0; t < T; ++t) {
      g.push_back({R_G, t, 0, 1});
      a.push_back({R_A, t, 0, 1});
    }
    h->plan_gpi = add_fwd_plan(h, fwd, g);
    h->plan_act = add_fwd_plan(h, fwd, a);
  }
  std::vector<BwdInst> bwd(T);
  std::vector<TdgInst> tdg(T);
  for (int i = 0; i < T; ++i) {
    BwdInst& b = bwd[i];
    b.P = h->params(0, i);
    b.Mo = h->am + (size_t)i * h->P;
    b.Vo = h->av + (size_t)i * h->P;
    b.step = h->step + i;
    for (int l = 0; l < NLMAX; ++l) {
      b.X[l] = (l >= 1 && l < h->NL) ? h->actp(R_S, i, l - 1) : nullptr;
      b.dZ[l] = l < h->NL ? h->dzp(i, l) : nullptr;
    }
    TdgInst& t = tdg[i];
    t.policy = i;
    t.c = h->actp(R_S, i, h->NL - 1);
    t.tpsi = h->actp(R_S1T, i, h->NL - 1);
    t.psiN = h->actp(R_S1, 0, h->NL - 1);
    t.w = h->w + (size_t)i * h->dpad;
    t.wm = h->wm + (size_t)i * h->dpad;
    t.wv = h->wv + (size_t)i * h->dpad;
    t.step = h->step + i;
    t.g = h->dzp(i, h->NL - 1);
  }
  auto upload = [&](void** dst, const void* src, size_t bytes) {
    if (rc != SFX_OK) return;
    if (hipMalloc(dst, bytes) != hipSuccess || hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      g_err = "descriptor upload failed";
      rc = SFX_E_HIP;
    }
  };
  upload((void**)&h->d_fwd, fwd.data(), sizeof(FwdInst) * fwd.size());
  upload((void**)&h->d_bwd, bwd.data(), sizeof(BwdInst) * bwd.size());
  upload((void**)&h->d_tdg, tdg.data(), sizeof(TdgInst) * tdg.size());
  if (rc != SFX_OK) {
    free_all(h);
    delete h;
    return rc;
  }
  *out = h;
  return SFX_OK;
}

int sfx_destroy(sfx_t h) {
  if (!h) return SFX_OK;
  (void)hipStreamSynchronize(h->stream);
  free_all(h);
  delete h;
  return SFX_OK;
}

int sfx_set_stream(sfx_t h, void* stream) {
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->stream = (hipStream_t)stream;
  return SFX_OK;
}

int sfx_head_numel(sfx_t h) { return h ? h->Ptorch : SFX_E_ARG; }

int sfx_set_adam(sfx_t h, double lr_psi, double wd_psi, double lr_w, double wd_w, double beta1,
                 double beta2, double eps) {
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  h->hp_psi = AdamHP{lr_psi, wd_psi, beta1, beta2, eps};
  h->hp_w = AdamHP{lr_w, wd_w, beta1, beta2, eps};
  return SFX_OK;
}

int sfx_load_head(sfx_t h, int t, int which, const float* params_host) {
  if (!valid_head(h, t) || !params_host) SFX_FAIL(SFX_E_ARG, "bad head / pointer");
  std::vector<float> buf(h->P);
  pack_head(h, params_host, buf.data());
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpyAsync(h->params(which, t), buf.data(), sizeof(float) * h->P, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

int sfx_get_head(sfx_t h, int t, int which, float* params_host) {
  if (!valid_head(h, t) || !params_host) SFX_FAIL(SFX_E_ARG, "bad head / pointer");
  std::vector<float> buf(h->P);
  HIPCHK(hipMemcpyAsync(buf.data(), h->params(which, t), sizeof(float) * h->P, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  unpack_head(h, buf.data(), params_host);
  return SFX_OK;
}

int sfx_load_adam(sfx_t h, int t, const float* m_host, const float* v_host, int step) {
  if (!valid_head(h, t) || !m_host || !v_host || step < 0) SFX_FAIL(SFX_E_ARG, "bad args");
  std::vector<float> bm(h->P), bv(h->P);
  pack_head(h, m_host, bm.data());
  pack_head(h, v_host, bv.data());
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpyAsync(h->am + (size_t)t * h->P, bm.data(), sizeof(float) * h->P, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->av + (size_t)t * h->P, bv.data(), sizeof(float) * h->P, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->step + t, &step, sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->host_step[t] = step;
  return SFX_OK;
}

int sfx_get_adam(sfx_t h, int t, float* m_host, float* v_host, int* step) {
  if (!valid_head(h, t)) SFX_FAIL(SFX_E_ARG, "bad head");
  std::vector<float> bm(h->P), bv(h->P);
  int st = 0;
  HIPCHK(hipMemcpyAsync(bm.data(), h->am + (size_t)t * h->P, sizeof(float) * h->P, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(bv.data(), h->av + (size_t)t * h->P, sizeof(float) * h->P, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(&st, h->step + t, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (m_host) unpack_head(h, bm.data(), m_host);
  if (v_host) unpack_head(h, bv.data(), v_host);
  if (step) *step = st;
  return SFX_OK;
}

int sfx_load_w(sfx_t h, int t, const float* w_host) {
  if (!valid_head(h, t) || !w_host) SFX_FAIL(SFX_E_ARG, "bad args");
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpyAsync(h->w + (size_t)t * h->dpad, w_host, sizeof(float) * h->d, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

int sfx_get_w(sfx_t h, int t, float* w_host, float* wm_host, float* wv_host) {
  if (!valid_head(h, t)) SFX_FAIL(SFX_E_ARG, "bad head");
  const size_t o = (size_t)t * h->dpad, n = sizeof(float) * h->d;
  if (w_host) HIPCHK(hipMemcpyAsync(w_host, h->w + o, n, hipMemcpyDeviceToHost, h->stream));
  if (wm_host) HIPCHK(hipMemcpyAsync(wm_host, h->wm + o, n, hipMemcpyDeviceToHost, h->stream));
  if (wv_host) HIPCHK(hipMemcpyAsync(wv_host, h->wv + o, n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

int sfx_w_ptr(sfx_t h, int t, float** w_dev) {
  if (!valid_head(h, t) || !w_dev) SFX_FAIL(SFX_E_ARG, "bad args");
  *w_dev = h->w + (size_t)t * h->dpad;
  return SFX_OK;
}

int sfx_gpi(sfx_t h, const float* S, int B, const float* w, float* psi, float* q, int64_t* task,
            int64_t* next) {
  if (!h || !S || !w || B < 1) SFX_FAIL(SFX_E_ARG, "bad args");
  for (int row0 = 0; row0 < B; row0 += h->Mmax) {
    const int m = B - row0 < h->Mmax ? B - row0 : h->Mmax;
    int rc = run_fwd(h, h->plan_gpi, h->T, m, S + (size_t)row0 * h->n_s, nullptr);
    if (rc) return rc;
    GpiArgs G{};
    G.M = m;
    G.T = h->T;
    G.A = h->A;
    G.d = h->d;
    G.row0 = row0;
    G.stride = h->actSize;
    G.psiN = h->actp(R_G, 0, h->NL - 1);
    G.w = w;
    G.psi_out = psi;
    G.q_out = q;
    G.task_out = task;
    G.next_out = next;
    hipLaunchKernelGGL(k_gpi, dim3(m), dim3(256), 0, h->stream, G);
    LAUNCHCHK();
  }
  return SFX_OK;
}

int sfx_select_action(sfx_t h, const float* s, int task_index, int use_gpi, float* q, int64_t* out) {
  if (!h || !s || !out || task_index < 0 || task_index >= h->T) SFX_FAIL(SFX_E_ARG, "bad args");
  int rc = run_fwd(h, h->plan_act, h->T, 1, s, nullptr);
  if (rc) return rc;
  GpiArgs G{};
  G.M = 1;
  G.T = h->T;
  G.A = h->A;
  G.d = h->d;
  G.select_task = task_index;
  G.use_gpi = use_gpi;
  G.stride = h->actSize;
  G.psiN = h->actp(R_A, 0, h->NL - 1);
  G.w = h->w + (size_t)task_index * h->dpad;
  G.q_out = q;
  G.sel_out = out;
  hipLaunchKernelGGL(k_gpi, dim3(1), dim3(256), 0, h->stream, G);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_update(sfx_t h, int policy, const float* S, const int64_t* a, const float* r, const float* phi,
               const float* S1, const float* gamma, int B, int use_gpi, float* losses, int64_t* next) {
  if (!valid_head(h, policy) || !S || !a || !phi || !S1 || !gamma) SFX_FAIL(SFX_E_ARG, "bad args");
  if (B < 1 || B > h->Mmax) SFX_FAIL(SFX_E_ARG, "batch exceeds max_batch");
  use_gpi = use_gpi ? 1 : 0;
  const int ninst = 2 + (use_gpi ? h->T : 1);
  int rc = run_fwd(h, h->plan_upd[use_gpi][policy], ninst, B, S, S1);
  if (rc) return rc;
  if ((rc = run_tdg(h, policy, B, use_gpi, a, r, phi, gamma, losses, next))) return rc;
  if ((rc = run_bwd(h, policy, 1, B, S))) return rc;
  after_update(h, policy);
  return maybe_sync_target(h, policy);
}

int sfx_update_all(sfx_t h, const float* S, const int64_t* a, const float* phi, const float* S1,
                   const float* gamma, int B, float* losses) {
  if (!h || !S || !a || !phi || !S1 || !gamma) SFX_FAIL(SFX_E_ARG, "bad args");
  if (B < 1 || B > h->Mmax) SFX_FAIL(SFX_E_ARG, "batch exceeds max_batch");
  int rc = run_fwd(h, h->plan_all, 3 * h->T, B, S, S1);
  if (rc) return rc;
  for (int i = 0; i < h->T; ++i) {
    if ((rc = run_tdg(h, i, B, 1, a, nullptr, phi, gamma, losses ? losses + 3 * i : nullptr, nullptr))) return rc;
    if ((rc = run_bwd(h, i, 1, B, S))) return rc;
    if (i + 1 < h->T && (rc = run_fwd(h, h->plan_refwd[i], 1, B, S, S1))) return rc;
    after_update(h, i);
  }
  for (int i = 0; i < h->T; ++i)
    if ((rc = maybe_sync_target(h, i))) return rc;
  return SFX_OK;
}

int sfx_lms(sfx_t h, int t, const float* phi, const float* r, float alpha) {
  if (!valid_head(h, t) || !phi || !r) SFX_FAIL(SFX_E_ARG, "bad args");
  hipLaunchKernelGGL(k_lms, dim3(1), dim3(256), 0, h->stream, h->w + (size_t)t * h->dpad, phi, r, alpha, h->d);
  LAUNCHCHK();
  return SFX_OK;
}

int sfx_set_target_update_ev(sfx_t h, int ev) {
  if (!h || ev < 1) SFX_FAIL(SFX_E_ARG, "bad args");
  h->target_update_ev = ev;
  return SFX_OK;
}

int sfx_get_since_target(sfx_t h, int t, int* count) {
  if (!valid_head(h, t) || !count) SFX_FAIL(SFX_E_ARG, "bad args");
  *count = h->since_target[t];
  return SFX_OK;
}

int sfx_set_since_target(sfx_t h, int t, int count) {
  if (!valid_head(h, t) || count < 0) SFX_FAIL(SFX_E_ARG, "bad args");
  h->since_target[t] = count;
  return SFX_OK;
}

int sfx_sync_target(sfx_t h, int t) {
  if (!valid_head(h, t)) SFX_FAIL(SFX_E_ARG, "bad head");
  HIPCHK(hipMemcpyAsync(h->params(1, t), h->params(0, t), sizeof(float) * h->P, hipMemcpyDeviceToDevice,
                        h->stream));
  return SFX_OK;
}

int sfx_synchronize(sfx_t h) {
  if (!h) SFX_FAIL(SFX_E_ARG, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  return SFX_OK;
}

}  // extern "C"
