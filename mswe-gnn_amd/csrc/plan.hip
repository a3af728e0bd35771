// Host side of the C ABI (include/mswegnn.h): graph plan (internal numbering, CSR by
// destination, pooling / unpooling maps), weight packing for the gfx950 kernels, the
// per-step schedule of MSGNN.forward / GNN.forward and the fused rollout.
//
// Reference semantics followed (sdat2/mSWE-GNN):
//   MSGNN.forward  models/gnn.py:267-350     GNN.forward  models/gnn.py:102-152
//   SWEGNN.forward models/gnn.py:387-445     rollout_test training/train.py:67-95
//   update_batch_multiscale training/train.py:31-65 (batched node_ptr layout)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/mswegnn.h"
#include "engine.h"

using namespace msw;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return fail(MSW_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));     \
  } while (0)

inline int tiles(int n) { return (n + 15) / 16; }


struct Blob {
  std::vector<float> h;
  int alloc(size_t n) {  // 64-float (256 B) aligned chunk
    size_t off = (h.size() + 63) / 64 * 64;
    h.resize(off + n, 0.f);
    return (int)off;
  }
};

// Pack W (original [out_dim][in_dim]) as the A operand of v_mfma_f32_16x16x4_f32,
// [tout][tin][lane][4]: lane l, k-step r of input tile ti for output tile to holds
// W[16 to + (l & 15)][16 ti + 4 (l >> 4) + r] (see kernels_impl.h for the register layout).
// in_map(k) / out_map(o) give the original column / row of packed input feature k /
// output feature o, or -1 for a zero pad.
template <class InMap, class OutMap>
int pack_operand(Blob& B, const float* W, int in_dim, int tout, int tin, InMap in_map,
                 OutMap out_map) {
  const int off = B.alloc((size_t)tout * tin * 64 * 4);
  float* A = B.h.data() + off;
  for (int to = 0; to < tout; ++to)
    for (int ti = 0; ti < tin; ++ti)
      for (int lane = 0; lane < 64; ++lane)
        for (int r = 0; r < 4; ++r) {
          const int o = out_map(16 * to + (lane & 15));
          const int k = in_map(16 * ti + 4 * (lane >> 4) + r);
          float v = 0.f;
          if (o >= 0 && k >= 0) v = W[(size_t)o * in_dim + k];
          A[(((size_t)to * tin + ti) * 64 + lane) * 4 + r] = v;
        }
  return off;
}

int pack_bias(Blob& B, const float* b, int out_dim, int tout) {
  if (!b) return -1;
  const int off = B.alloc((size_t)16 * tout);
  for (int o = 0; o < out_dim; ++o) B.h[off + o] = b[o];
  return off;
}

int act_code(int a) { return (a >= 0 && a <= 7) ? a : -1; }

// Pack a make_mlp stack (natural feature order in and out).
int pack_mlp(Blob& B, const msw_mlp& m, MlpDev& d, int first_in_tiles_override = -1) {
  if (m.n_layers < 1 || m.n_layers > kMaxLayers)
    return fail(MSW_ERR_UNSUPPORTED, "MLP depth must be 1.." + std::to_string(kMaxLayers));
  d.n = m.n_layers;
  for (int i = 0; i < m.n_layers; ++i) {
    const msw_linear& L = m.layer[i];
    if (!L.weight || L.in_features <= 0 || L.out_features <= 0)
      return fail(MSW_ERR_INVALID, "MLP layer without weight");
    if (act_code(L.act) < 0) return fail(MSW_ERR_INVALID, "unknown activation code");
    const int tin = (i == 0 && first_in_tiles_override > 0) ? first_in_tiles_override : tiles(L.in_features);
    const int tout = tiles(L.out_features);
    const int din = L.in_features, dout = L.out_features;
    d.l[i].tin = tin;
    d.l[i].tout = tout;
    d.l[i].a_off = pack_operand(B, L.weight, din, tout, tin,
                                [&](int k) { return k < din ? k : -1; },
                                [&](int o) { return o < dout ? o : -1; });
    d.l[i].b_off = pack_bias(B, L.bias, dout, tout);
    d.l[i].act = L.act;
    d.l[i].slope = L.act_param;
  }
  return MSW_OK;
}

template <class T>
int dalloc(T** p, size_t n, int64_t& counter) {
  if (n == 0) n = 1;
  HIP_TRY(hipMalloc((void**)p, n * sizeof(T)));
  counter += (int64_t)(n * sizeof(T));
  return MSW_OK;
}

template <class T>
int upload(T** p, const std::vector<T>& v, int64_t& counter) {
  int rc = dalloc(p, v.size(), counter);
  if (rc) return rc;
  if (!v.empty()) HIP_TRY(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return MSW_OK;
}

}  // namespace

hipError_t rowmlp_dispatch(int NT, const RowMlpArgs& ra) {
  switch (NT) {
    case 1: return launch_rowmlp<1>(ra, nullptr);
    case 2: return launch_rowmlp<2>(ra, nullptr);
    default: return launch_rowmlp<4>(ra, nullptr);
  }
}

// ============================================================================ plan
struct ScaleCSR {
  int n0 = 0, ns = 0;     // internal node range
  int E = 0;              // edges of this scale
  int* rowptr = nullptr;  // [ns+1]
  int* src = nullptr;     // [E] internal ids, CSR order
  int* dst = nullptr;     // [E]
  std::vector<int> eorig; // CSR position -> original edge id
};

struct LevelMaps {            // level l: coarse scale l+1, fine scale l
  int I = 0;
  int* pool_rowptr = nullptr; // by coarse (local to scale l+1)
  int* pool_child = nullptr;
  int* un_rowptr = nullptr;   // by fine (local to scale l)
  int* un_src = nullptr;      // coarse ids
  int* un_dst = nullptr;      // fine ids
};

struct Proc {                 // one SWEGNN layer bound to a scale (or intra level)
  int scale = 0;
  int K = 0, normalize = 1, with_filter = 1, with_gradient = 1, upwind = 0;
  int h1t = 1;
  int a_u = -1, a_v = -1, a_o = -1;
  float* Pe = nullptr;        // [E][32*h1t] (processors with edge features)
  int b1_off = -1;            // bias of layer 1 (blob)
  int act1 = 0;
  float slope1 = 0.f;
  MlpDev rest{};              // layers 2..L, offsets relative to rest_base
  int rest_base = 0, rest_count = 0;
  std::vector<int> wt_off;    // packed filters 1..K (blob offsets)
  int prelu = 0;              // every edge-MLP activation is PReLU
};

struct msw_plan {
  int device = 0;
  int model_type = 0, F = 32, NT = 2, S = 1, p = 3, nnf = 8, dyn = 6, nstat_raw = 2;
  int with_wl = 1, skip = 1, ef = 1;
  int N = 0;
  int64_t E = 0;
  bool identity = true;
  std::vector<int> perm, iperm;  // internal -> graph, graph -> internal
  std::vector<ScaleCSR> sc;
  std::vector<LevelMaps> lv;
  std::vector<Proc> procs, unpools;
  MlpDev stat{}, dynm{}, dec{}, edge_enc{};
  int gnn_act = 0;
  float gnn_slope = 0.f;
  int enc_prelu = 0, dec_prelu = 0;
  int resw_off = -1;
  Blob blob;
  float* dW = nullptr;
  int* perm_d = nullptr;
  int* bc_slot_d = nullptr;
  std::vector<int> bc_rows_set;  // internal rows currently holding a BC slot
  RolloutIO* io_d = nullptr;
  float *X = nullptr, *xs = nullptr, *xd0 = nullptr, *bufA = nullptr, *bufB = nullptr;
  float *xin = nullptr, *xdown = nullptr, *xup = nullptr, *U = nullptr, *V = nullptr, *s = nullptr;
  float* gnnbuf[2] = {nullptr, nullptr};
  int h1t_max = 1;
  int64_t dev_bytes = 0;
  int64_t forward_calls = 0, rollout_steps = 0;
  int kernels_per_step = 0;
  int use_graph = 1;
  hipStream_t cap_stream = nullptr;
  hipGraphExec_t step_exec = nullptr;
  const float* last_x = nullptr;  // input the forward-mode kernels were built for
  std::vector<void*> owned;
  ~msw_plan() {
    if (step_exec) (void)hipGraphExecDestroy(step_exec);
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    for (void* q : owned) (void)hipFree(q);
  }
};

namespace {

template <class T>
int palloc(msw_plan* P, T** p, size_t n) {
  int rc = dalloc(p, n, P->dev_bytes);
  if (!rc) P->owned.push_back(*p);
  return rc;
}
template <class T>
int pupload(msw_plan* P, T** p, const std::vector<T>& v) {
  int rc = upload(p, v, P->dev_bytes);
  if (!rc) P->owned.push_back(*p);
  return rc;
}

// Stable counting sort of (key, payload) pairs by key in [0, nkeys).
void csr_build(int nkeys, const std::vector<int>& key, std::vector<int>& rowptr,
               std::vector<int>& order) {
  rowptr.assign(nkeys + 1, 0);
  for (int k : key) rowptr[k + 1]++;
  for (int i = 0; i < nkeys; ++i) rowptr[i + 1] += rowptr[i];
  std::vector<int> pos(rowptr.begin(), rowptr.end() - 1);
  order.assign(key.size(), 0);
  for (size_t e = 0; e < key.size(); ++e) order[pos[key[e]]++] = (int)e;
}

// SWEGNN layer -> packed Proc.  edge_in: width of the per-edge features it consumes.
int build_proc(msw_plan* P, const msw_swegnn& g, int scale, bool intra, Proc& pr) {
  const int F = P->F;
  pr.scale = scale;
  pr.K = g.K;
  pr.normalize = g.normalize;
  pr.with_filter = g.with_filter_matrix;
  pr.with_gradient = g.with_gradient;
  pr.upwind = g.upwind_mode;
  if (g.K < 1 && !intra) return fail(MSW_ERR_UNSUPPORTED, "SWEGNN with K < 1");
  const msw_mlp& m = g.edge_mlp;
  if (m.n_layers < 1 || m.n_layers > kMaxLayers)
    return fail(MSW_ERR_UNSUPPORTED, "edge MLP depth must be 1..4");
  const msw_linear& L1 = m.layer[0];
  const int ef = g.edge_features;
  if (L1.in_features != 4 * F + ef) return fail(MSW_ERR_INVALID, "edge MLP input width != 4F + edge_features");
  const int H1 = L1.out_features;
  if (H1 != (m.n_layers > 1 ? 2 * F : F)) return fail(MSW_ERR_UNSUPPORTED, "edge MLP hidden width must be 2F");
  for (int i = 1; i < m.n_layers; ++i)
    if (m.layer[i].in_features != 2 * F || m.layer[i].out_features != (i == m.n_layers - 1 ? F : 2 * F))
      return fail(MSW_ERR_UNSUPPORTED, "edge MLP layer widths must be 2F -> ... -> F");
  pr.h1t = tiles(H1);
  P->h1t_max = std::max(P->h1t_max, pr.h1t);
  const int din = L1.in_features;
  const float* W1 = L1.weight;
  auto outm = [&](int o) { return o < H1 ? o : -1; };
  // U: [x_s (tiles 0..T-1) | x_d (tiles T..2T-1)] of the ROW (source) node
  auto in_u = [&](int k) {
    if (k < F) return k;                                     // x_s[row]  cols [0, F)
    return k < 2 * F ? 2 * F + (k - F) : -1;                 // x_d[row]  cols [2F, 3F)
  };
  auto in_v = [&](int k) {
    if (k < F) return F + k;                                 // x_s[col]  cols [F, 2F)
    return k < 2 * F ? 3 * F + (k - F) : -1;                 // x_d[col]  cols [3F, 4F)
  };
  pr.a_u = pack_operand(P->blob, W1, din, pr.h1t, 2 * P->NT, in_u, outm);
  pr.a_v = pack_operand(P->blob, W1, din, pr.h1t, 2 * P->NT, in_v, outm);
  pr.act1 = L1.act;
  pr.slope1 = L1.act_param;
  if (L1.bias) {
    pr.b1_off = P->blob.alloc(16 * pr.h1t);
    for (int o = 0; o < H1; ++o) P->blob.h[pr.b1_off + o] = L1.bias[o];
  } else {
    pr.b1_off = P->blob.alloc(16 * pr.h1t);  // zeros
  }
  if (g.with_filter_matrix && !intra) {
    if (!g.filter) return fail(MSW_ERR_INVALID, "with_filter_matrix but no filter weights");
    // filter 0 as an MFMA operand over the x_in tiles: O = W0 . x_in
    pr.a_o = pack_operand(P->blob, g.filter[0], F, P->NT, P->NT,
                          [&](int k) { return k < F ? k : -1; },
                          [&](int o) { return o < F ? o : -1; });
    for (int k = 1; k <= g.K; ++k)  // filters 1..K as MFMA operands of the hop kernel
      pr.wt_off.push_back(pack_operand(P->blob, g.filter[k], F, P->NT, P->NT,
                                       [&](int q) { return q < F ? q : -1; },
                                       [&](int o) { return o < F ? o : -1; }));
  } else if (g.with_filter_matrix && intra) {
    return fail(MSW_ERR_UNSUPPORTED, "intra-scale SWEGNN with filter matrix");
  } else if (!intra) {
    // out = x_d.clone() (gnn.py:404): identity operand, exact (1*x + 0*y sums)
    std::vector<float> I((size_t)F * F, 0.f);
    for (int i = 0; i < F; ++i) I[(size_t)i * F + i] = 1.f;
    pr.a_o = pack_operand(P->blob, I.data(), F, P->NT, P->NT,
                          [&](int k) { return k < F ? k : -1; },
                          [&](int o) { return o < F ? o : -1; });
  }
  // layers 2..L contiguous (staged to LDS by the edge kernel)
  pr.rest.n = m.n_layers - 1;
  Blob rb;
  for (int i = 1; i < m.n_layers; ++i) {
    const msw_linear& L = m.layer[i];
    const int tin = tiles(L.in_features), tout = tiles(L.out_features);
    const int di = L.in_features, dout = L.out_features;
    pr.rest.l[i - 1].tin = tin;
    pr.rest.l[i - 1].tout = tout;
    pr.rest.l[i - 1].a_off = pack_operand(rb, L.weight, di, tout, tin,
                                          [&](int k) { return k < di ? k : -1; },
                                          [&](int o) { return o < dout ? o : -1; });
    pr.rest.l[i - 1].b_off = pack_bias(rb, L.bias, dout, tout);
    pr.rest.l[i - 1].act = L.act;
    pr.rest.l[i - 1].slope = L.act_param;
  }
  if (m.layer[m.n_layers - 1].out_features != F) return fail(MSW_ERR_INVALID, "edge MLP output != F");
  pr.prelu = 1;
  for (int i = 0; i < m.n_layers; ++i) pr.prelu &= (m.layer[i].act == MSW_ACT_PRELU);
  pr.rest_count = (int)((rb.h.size() + 3) / 4 * 4);
  pr.rest_base = P->blob.alloc(pr.rest_count);
  std::copy(rb.h.begin(), rb.h.end(), P->blob.h.begin() + pr.rest_base);
  if ((size_t)pr.rest_count * 4 > 160 * 1024)
    return fail(MSW_ERR_UNSUPPORTED, "edge MLP weights exceed LDS");
  return MSW_OK;
}

template <int NT>
int run_proc(msw_plan* P, const Proc& pr, const float* xin, float* out, int post_act,
             float post_slope, hipStream_t st, int& nk) {
  const ScaleCSR& g = P->sc[pr.scale];
  NodeProjArgs np{};
  np.r0 = g.n0; np.R = g.ns; np.xs = P->xs; np.xin = xin;
  np.a_u = pr.a_u; np.a_v = pr.a_v; np.a_o = pr.a_o; np.W = P->dW;
  np.U = P->U; np.V = P->V; np.O = P->bufA; np.h1t = pr.h1t;
  HIP_TRY(launch_node_proj<NT>(np, st)); ++nk;
  EdgeMlpArgs em{};
  em.E = g.E; em.src = g.src; em.dst = g.dst; em.U = P->U; em.V = P->V; em.Pe = pr.Pe;
  em.b1 = P->dW + pr.b1_off; em.h1t = pr.h1t; em.act1 = pr.act1; em.slope1 = pr.slope1;
  em.rest = pr.rest; em.W = P->dW + pr.rest_base; em.w_count = pr.rest_count;
  em.normalize = pr.normalize; em.s = P->s; em.prelu_only = pr.prelu;
  HIP_TRY(launch_edge_mlp<NT>(em, st)); ++nk;
  const float* cur = P->bufA;
  for (int k = 1; k <= pr.K; ++k) {
    float* nxt = (k == pr.K) ? out : (cur == P->bufA ? P->bufB : P->bufA);
    HopArgs h{};
    h.n0 = g.n0; h.R = g.ns; h.rowptr = g.rowptr; h.src = g.src; h.s = P->s; h.in = cur;
    h.out = nxt; h.A = pr.wt_off.empty() ? nullptr : P->dW + pr.wt_off[k - 1]; h.skip = nullptr; h.own_zero = 0;
    h.grad = pr.with_gradient; h.upwind = pr.upwind;
    h.post_act = (k == pr.K) ? post_act : 0; h.post_slope = post_slope;
    HIP_TRY(launch_hop<NT>(h, st)); ++nk;
    cur = nxt;
  }
  return MSW_OK;
}

// intra_scale_gnn[i] on level l: coarse rows (scale l+1) of `xo` -> fine rows of `dst`
template <int NT>
int run_unpool(msw_plan* P, const Proc& pr, int l, const float* xo, float* dst, hipStream_t st,
               int& nk) {
  const ScaleCSR& cs = P->sc[l + 1];
  const ScaleCSR& fs = P->sc[l];
  const LevelMaps& m = P->lv[l];
  NodeProjArgs np{};
  np.xs = P->xs; np.W = P->dW; np.U = P->U; np.V = P->V; np.O = nullptr; np.h1t = pr.h1t;
  np.r0 = cs.n0; np.R = cs.ns; np.xin = xo; np.a_u = pr.a_u; np.a_v = -1; np.a_o = -1;
  HIP_TRY(launch_node_proj<NT>(np, st)); ++nk;
  np.r0 = fs.n0; np.R = fs.ns; np.xin = nullptr; np.a_u = -1; np.a_v = pr.a_v;
  HIP_TRY(launch_node_proj<NT>(np, st)); ++nk;
  EdgeMlpArgs em{};
  em.E = m.I; em.src = m.un_src; em.dst = m.un_dst; em.U = P->U; em.V = P->V; em.Pe = nullptr;
  em.b1 = P->dW + pr.b1_off; em.h1t = pr.h1t; em.act1 = pr.act1; em.slope1 = pr.slope1;
  em.rest = pr.rest; em.W = P->dW + pr.rest_base; em.w_count = pr.rest_count;
  em.normalize = pr.normalize; em.s = P->s; em.prelu_only = pr.prelu;
  HIP_TRY(launch_edge_mlp<NT>(em, st)); ++nk;
  HopArgs h{};
  h.n0 = fs.n0; h.R = fs.ns; h.rowptr = m.un_rowptr; h.src = m.un_src; h.s = P->s; h.in = xo;
  h.out = dst; h.A = nullptr; h.skip = P->skip ? P->xdown : nullptr; h.own_zero = 1;
  h.grad = pr.with_gradient; h.upwind = pr.upwind; h.post_act = 0; h.post_slope = 0.f;
  HIP_TRY(launch_hop<NT>(h, st)); ++nk;
  return MSW_OK;
}

// One forward.  x_src/perm: input rows (forward mode: graph rows via perm; rollout: the
// internal state X with perm = null).  y: forward-mode output (null in rollout mode).
template <int NT>
int enqueue_step(msw_plan* P, const float* x_src, const int* perm, float* y, bool rollout,
                 hipStream_t st) {
  int nk = 0;
  EncodeArgs ea{};
  ea.x = x_src; ea.perm = perm; ea.N = P->N; ea.nnf = P->nnf; ea.nstat_raw = P->nstat_raw;
  ea.with_wl = P->with_wl; ea.dyn = P->dyn; ea.stat = P->stat; ea.dynm = P->dynm; ea.W = P->dW;
  ea.xs = P->xs; ea.xd = P->xd0; ea.xd_rows = P->sc[0].n0 + P->sc[0].ns;
  ea.io = rollout ? P->io_d : nullptr;
  ea.prelu_only = P->enc_prelu;
  HIP_TRY(launch_encode<NT>(ea, st)); ++nk;
  const float* dec_in = nullptr;
  int pre_act = 0;
  float pre_slope = 0.f;
  int rc = MSW_OK;
  if (P->model_type == 0) {
    const int S = P->S;
    for (int i = 0; i < S - 1; ++i) {
      rc = run_proc<NT>(P, P->procs[i], i == 0 ? P->xd0 : P->xin, P->xdown, 0, 0.f, st, nk);
      if (rc) return rc;
      PoolArgs pa{};
      pa.n0 = P->sc[i + 1].n0; pa.R = P->sc[i + 1].ns; pa.rowptr = P->lv[i].pool_rowptr;
      pa.child = P->lv[i].pool_child; pa.in = P->xdown; pa.out = P->xin;
      HIP_TRY(launch_pool<NT>(pa, st)); ++nk;
    }
    for (int i = 0; i < S; ++i) {
      const int j = S - 1 + i;
      const float* in = (S == 1) ? P->xd0 : P->xin;
      rc = run_proc<NT>(P, P->procs[j], in, P->xup, 0, 0.f, st, nk);
      if (rc) return rc;
      if (i < S - 1) {
        const int l = S - 2 - i;
        rc = run_unpool<NT>(P, P->unpools[i], l, P->xup, P->xin, st, nk);
        if (rc) return rc;
      }
    }
    dec_in = P->xup;
    pre_act = P->gnn_act;
    pre_slope = P->gnn_slope;
  } else {
    const float* cur = P->xd0;
    for (size_t j = 0; j < P->procs.size(); ++j) {
      float* out = P->gnnbuf[j & 1];
      rc = run_proc<NT>(P, P->procs[j], cur, out, P->gnn_act, P->gnn_slope, st, nk);
      if (rc) return rc;
      cur = out;
    }
    dec_in = cur;
  }
  DecodeArgs da{};
  da.N = P->N; da.nnf = P->nnf; da.dyn = P->dyn; da.p = P->p; da.xup = dec_in;
  da.pre_act = pre_act; da.pre_slope = pre_slope; da.dec = P->dec; da.W = P->dW;
  da.resw = P->resw_off >= 0 ? P->dW + P->resw_off : nullptr;
  da.X = const_cast<float*>(x_src);
  da.perm = P->identity ? nullptr : P->perm_d;
  da.y = y; da.io = rollout ? P->io_d : nullptr; da.bc_slot = P->bc_slot_d;
  da.prelu_only = P->dec_prelu;
  HIP_TRY(launch_decode<NT>(da, st)); ++nk;
  P->kernels_per_step = nk;
  return MSW_OK;
}

int step_dispatch(msw_plan* P, const float* x_src, const int* perm, float* y, bool rollout,
                  hipStream_t st) {
  switch (P->NT) {
    case 1: return enqueue_step<1>(P, x_src, perm, y, rollout, st);
    case 2: return enqueue_step<2>(P, x_src, perm, y, rollout, st);
    default: return enqueue_step<4>(P, x_src, perm, y, rollout, st);
  }
}

int build_graph_plan(msw_plan* P, const msw_graph_desc* g) {
  const int S = P->S, G = g->num_graphs;
  if (g->num_nodes <= 0 || g->num_nodes > (1LL << 30)) return fail(MSW_ERR_INVALID, "num_nodes out of range");
  if (g->num_edges < 0 || g->num_edges > (1LL << 31) - 64) return fail(MSW_ERR_INVALID, "num_edges out of range");
  if (G < 1 || !g->node_ptr) return fail(MSW_ERR_INVALID, "node_ptr missing");
  if (g->num_scales != S) return fail(MSW_ERR_INVALID, "graph num_scales != model num_scales");
  const int N = (int)g->num_nodes;
  P->N = N;
  P->E = g->num_edges;
  // internal numbering: scale-major, graph-major inside a scale
  P->perm.clear();
  P->sc.assign(S, ScaleCSR{});
  for (int s = 0; s < S; ++s) {
    P->sc[s].n0 = (int)P->perm.size();
    for (int gi = 0; gi < G; ++gi) {
      const int64_t a = g->node_ptr[gi * (S + 1) + s], b = g->node_ptr[gi * (S + 1) + s + 1];
      if (a < 0 || b < a || b > N) return fail(MSW_ERR_INVALID, "node_ptr out of range");
      for (int64_t v = a; v < b; ++v) P->perm.push_back((int)v);
    }
    P->sc[s].ns = (int)P->perm.size() - P->sc[s].n0;
  }
  if ((int)P->perm.size() != N) return fail(MSW_ERR_INVALID, "node_ptr does not cover every node exactly once");
  P->iperm.assign(N, -1);
  for (int i = 0; i < N; ++i) {
    if (P->iperm[P->perm[i]] != -1) return fail(MSW_ERR_INVALID, "node_ptr ranges overlap");
    P->iperm[P->perm[i]] = i;
  }
  P->identity = true;
  for (int i = 0; i < N; ++i)
    if (P->perm[i] != i) { P->identity = false; break; }
  // per-scale CSR by destination
  const int64_t E = g->num_edges;
  if (g->edge_ptr[0] != 0 || g->edge_ptr[S] != E) return fail(MSW_ERR_INVALID, "edge_ptr must span [0, E]");
  for (int s = 0; s < S; ++s) {
    ScaleCSR& c = P->sc[s];
    const int64_t a = g->edge_ptr[s], b = g->edge_ptr[s + 1];
    if (b < a) return fail(MSW_ERR_INVALID, "edge_ptr not monotone");
    c.E = (int)(b - a);
    std::vector<int> key(c.E), srcv(c.E), dstv(c.E);
    for (int64_t e = a; e < b; ++e) {
      const int64_t r = g->edge_index[e], cl = g->edge_index[E + e];
      if (r < 0 || r >= N || cl < 0 || cl >= N) return fail(MSW_ERR_INVALID, "edge_index out of range");
      const int ri = P->iperm[r], ci = P->iperm[cl];
      if (ri < c.n0 || ri >= c.n0 + c.ns || ci < c.n0 || ci >= c.n0 + c.ns)
        return fail(MSW_ERR_INVALID, "edge of scale " + std::to_string(s) + " leaves the scale");
      key[e - a] = ci - c.n0;
      srcv[e - a] = ri;
      dstv[e - a] = ci;
    }
    std::vector<int> rowptr, order;
    csr_build(c.ns, key, rowptr, order);
    std::vector<int> so(c.E), dso(c.E);
    c.eorig.resize(c.E);
    for (int i = 0; i < c.E; ++i) {
      so[i] = srcv[order[i]];
      dso[i] = dstv[order[i]];
      c.eorig[i] = (int)(a + order[i]);
    }
    int rc;
    if ((rc = pupload(P, &c.rowptr, rowptr)) || (rc = pupload(P, &c.src, so)) || (rc = pupload(P, &c.dst, dso)))
      return rc;
  }
  // intra-scale levels
  P->lv.assign(S > 1 ? S - 1 : 0, LevelMaps{});
  if (S > 1) {
    if (!g->intra_edge_index || !g->intra_edge_ptr) return fail(MSW_ERR_INVALID, "intra edges missing");
    const int64_t I = g->num_intra_edges;
    for (int l = 0; l < S - 1; ++l) {
      LevelMaps& m = P->lv[l];
      const ScaleCSR& cs = P->sc[l + 1];
      const ScaleCSR& fs = P->sc[l];
      const int64_t a = g->intra_edge_ptr[l], b = g->intra_edge_ptr[l + 1];
      if (a < 0 || b < a || b > I) return fail(MSW_ERR_INVALID, "intra_edge_ptr out of range");
      m.I = (int)(b - a);
      std::vector<int> ck(m.I), fk(m.I), cv(m.I), fv(m.I);
      for (int64_t e = a; e < b; ++e) {
        const int64_t co = g->intra_edge_index[e], fi = g->intra_edge_index[I + e];
        if (co < 0 || co >= N || fi < 0 || fi >= N) return fail(MSW_ERR_INVALID, "intra edge out of range");
        const int ci = P->iperm[co], fii = P->iperm[fi];
        if (ci < cs.n0 || ci >= cs.n0 + cs.ns || fii < fs.n0 || fii >= fs.n0 + fs.ns)
          return fail(MSW_ERR_INVALID, "intra edge of level " + std::to_string(l) + " not (coarse, fine)");
        ck[e - a] = ci - cs.n0;
        fk[e - a] = fii - fs.n0;
        cv[e - a] = ci;
        fv[e - a] = fii;
      }
      std::vector<int> rp, order;
      csr_build(cs.ns, ck, rp, order);
      std::vector<int> child(m.I);
      for (int i = 0; i < m.I; ++i) child[i] = fv[order[i]];
      int rc;
      if ((rc = pupload(P, &m.pool_rowptr, rp)) || (rc = pupload(P, &m.pool_child, child))) return rc;
      csr_build(fs.ns, fk, rp, order);
      std::vector<int> us(m.I), ud(m.I);
      for (int i = 0; i < m.I; ++i) {
        us[i] = cv[order[i]];
        ud[i] = fv[order[i]];
      }
      if ((rc = pupload(P, &m.un_rowptr, rp)) || (rc = pupload(P, &m.un_src, us)) ||
          (rc = pupload(P, &m.un_dst, ud)))
        return rc;
    }
  }
  return MSW_OK;
}

}  // namespace

namespace {
template <int NT>
int bench_kernel(msw_plan* P, int kernel, int scale, int iters, int64_t* units, hipStream_t st) {
  if (scale < 0 || scale >= P->S) return fail(MSW_ERR_INVALID, "scale out of range");
  const Proc* pr = nullptr;
  for (auto& q : P->procs)
    if (q.scale == scale) { pr = &q; break; }
  const ScaleCSR& g = P->sc[scale];
  int64_t rows = 0, edges = 0;
  for (int it = 0; it < iters; ++it) {
    if (kernel == 0 || kernel == 1 || kernel == 2) {
      if (!pr) return fail(MSW_ERR_INVALID, "no processor on that scale");
      if (kernel == 0) {
        HopArgs h{};
        h.n0 = g.n0; h.R = g.ns; h.rowptr = g.rowptr; h.src = g.src; h.s = P->s; h.in = P->bufA;
        h.out = P->bufB; h.A = pr->wt_off.empty() ? nullptr : P->dW + pr->wt_off[0];
        h.grad = pr->with_gradient; h.upwind = pr->upwind;
        HIP_TRY(launch_hop<NT>(h, st));
        rows = g.ns; edges = g.E;
      } else if (kernel == 1) {
        EdgeMlpArgs em{};
        em.E = g.E; em.src = g.src; em.dst = g.dst; em.U = P->U; em.V = P->V; em.Pe = pr->Pe;
        em.b1 = P->dW + pr->b1_off; em.h1t = pr->h1t; em.act1 = pr->act1; em.slope1 = pr->slope1;
        em.rest = pr->rest; em.W = P->dW + pr->rest_base; em.w_count = pr->rest_count;
        em.normalize = pr->normalize; em.s = P->s; em.prelu_only = pr->prelu;
        HIP_TRY(launch_edge_mlp<NT>(em, st));
        rows = 0; edges = g.E;
      } else {
        NodeProjArgs np{};
        np.r0 = g.n0; np.R = g.ns; np.xs = P->xs; np.xin = P->xin;
        np.a_u = pr->a_u; np.a_v = pr->a_v; np.a_o = pr->a_o; np.W = P->dW;
        np.U = P->U; np.V = P->V; np.O = P->bufA; np.h1t = pr->h1t;
        HIP_TRY(launch_node_proj<NT>(np, st));
        rows = g.ns; edges = 0;
      }
    } else if (kernel == 3) {
      if (scale < 1) return fail(MSW_ERR_INVALID, "pooling targets scale >= 1");
      PoolArgs pa{};
      pa.n0 = g.n0; pa.R = g.ns; pa.rowptr = P->lv[scale - 1].pool_rowptr;
      pa.child = P->lv[scale - 1].pool_child; pa.in = P->xdown; pa.out = P->bufB;
      HIP_TRY(launch_pool<NT>(pa, st));
      rows = g.ns; edges = P->lv[scale - 1].I;
    } else if (kernel == 4) {
      EncodeArgs ea{};
      ea.x = P->X; ea.perm = nullptr; ea.N = P->N; ea.nnf = P->nnf; ea.nstat_raw = P->nstat_raw;
      ea.with_wl = P->with_wl; ea.dyn = P->dyn; ea.stat = P->stat; ea.dynm = P->dynm; ea.W = P->dW;
      ea.xs = P->bufA; ea.xd = P->bufB; ea.xd_rows = P->sc[0].n0 + P->sc[0].ns; ea.io = nullptr;
      ea.prelu_only = P->enc_prelu;
      HIP_TRY(launch_encode<NT>(ea, st));
      rows = P->N; edges = 0;
    } else if (kernel == 5) {
      DecodeArgs da{};
      da.N = P->N; da.nnf = P->nnf; da.dyn = P->dyn; da.p = P->p; da.xup = P->xup;
      da.pre_act = P->gnn_act; da.pre_slope = P->gnn_slope; da.dec = P->dec; da.W = P->dW;
      da.resw = P->resw_off >= 0 ? P->dW + P->resw_off : nullptr;
      da.X = P->X; da.perm = P->identity ? nullptr : P->perm_d; da.y = P->bufB; da.io = nullptr;
      da.bc_slot = P->bc_slot_d; da.prelu_only = P->dec_prelu;
      HIP_TRY(launch_decode<NT>(da, st));
      rows = P->N; edges = 0;
    } else {
      return fail(MSW_ERR_INVALID, "unknown kernel id");
    }
  }
  if (units) { units[0] = rows; units[1] = edges; }
  return MSW_OK;
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

const char* msw_last_error(void) { return g_err.c_str(); }

int64_t msw_struct_size(const char* name) {
  if (!name) return -1;
  if (!strcmp(name, "msw_linear")) return sizeof(msw_linear);
  if (!strcmp(name, "msw_mlp")) return sizeof(msw_mlp);
  if (!strcmp(name, "msw_swegnn")) return sizeof(msw_swegnn);
  if (!strcmp(name, "msw_model_desc")) return sizeof(msw_model_desc);
  if (!strcmp(name, "msw_graph_desc")) return sizeof(msw_graph_desc);
  if (!strcmp(name, "msw_plan_stats")) return sizeof(msw_plan_stats);
  return -1;
}
int msw_abi_version(void) { return MSW_ABI_VERSION; }

int msw_plan_create(const msw_graph_desc* g, const msw_model_desc* m, int device,
                    msw_plan** out_plan) {
  if (!g || !m || !out_plan) return fail(MSW_ERR_INVALID, "null argument");
  *out_plan = nullptr;
  if (m->model_type != 0 && m->model_type != 1) return fail(MSW_ERR_INVALID, "model_type must be 0 (MSGNN) or 1 (GNN)");
  if (m->hid_features != 16 && m->hid_features != 32 && m->hid_features != 64)
    return fail(MSW_ERR_UNSUPPORTED, "hid_features must be 16, 32 or 64");
  if (m->learned_pooling) return fail(MSW_ERR_UNSUPPORTED, "learned_pooling=True is not implemented");
  HIP_TRY(hipSetDevice(device));
  std::unique_ptr<msw_plan> P(new msw_plan());
  P->device = device;
  P->model_type = m->model_type;
  P->F = m->hid_features;
  P->NT = P->F / 16;
  P->S = m->model_type == 0 ? m->num_scales : 1;
  P->p = m->previous_t;
  P->nnf = m->num_node_features;
  P->dyn = 2 * P->p;
  P->nstat_raw = P->nnf - P->dyn;
  P->with_wl = m->with_WL;
  P->skip = m->skip_connections;
  P->gnn_act = m->gnn_act;
  P->gnn_slope = m->gnn_act_param;
  if (P->S < 1) return fail(MSW_ERR_INVALID, "num_scales < 1");
  if (P->nstat_raw < 1 || P->nstat_raw + P->with_wl > 16 || P->dyn > 16)
    return fail(MSW_ERR_UNSUPPORTED, "node feature layout (static / dynamic widths)");
  if (m->model_type == 0 && m->num_processors != 2 * P->S - 1)
    return fail(MSW_ERR_INVALID, "MSGNN needs 2S-1 processors");
  if (m->model_type == 0 && m->num_unpool != P->S - 1)
    return fail(MSW_ERR_INVALID, "MSGNN needs S-1 intra-scale layers");
  if (m->model_type == 1 && m->num_processors < 1) return fail(MSW_ERR_INVALID, "GNN needs >= 1 layer");

  int rc = build_graph_plan(P.get(), g);
  if (rc) return rc;
  const int F = P->F, N = P->N;

  // ---- weights
  if ((rc = pack_mlp(P->blob, m->static_encoder, P->stat))) return rc;
  if ((rc = pack_mlp(P->blob, m->dynamic_encoder, P->dynm))) return rc;
  if ((rc = pack_mlp(P->blob, m->decoder, P->dec))) return rc;
  {
    auto all_prelu = [](const msw_mlp& mm) {
      for (int i = 0; i < mm.n_layers; ++i)
        if (mm.layer[i].act != MSW_ACT_PRELU) return 0;
      return 1;
    };
    P->enc_prelu = all_prelu(m->static_encoder) & all_prelu(m->dynamic_encoder);
    P->dec_prelu = all_prelu(m->decoder);
  }
  auto chain_ok = [&](const msw_mlp& mm, int last_out) {
    for (int i = 0; i < mm.n_layers; ++i) {
      const int want = (i == mm.n_layers - 1) ? last_out : F;
      if (mm.layer[i].out_features != want) return false;
      if (i > 0 && mm.layer[i].in_features != F) return false;
    }
    return true;
  };
  if (!chain_ok(m->static_encoder, F) || !chain_ok(m->dynamic_encoder, F) || !chain_ok(m->decoder, 2) ||
      (m->edge_mlp && !chain_ok(m->edge_encoder, F)) || m->decoder.layer[0].in_features != F)
    return fail(MSW_ERR_UNSUPPORTED, "encoder/decoder hidden widths must equal hid_features");
  if (m->static_encoder.layer[0].in_features != P->nstat_raw + P->with_wl)
    return fail(MSW_ERR_INVALID, "static encoder input width");
  if (m->dynamic_encoder.layer[0].in_features != P->dyn) return fail(MSW_ERR_INVALID, "dynamic encoder input width");
  if (m->decoder.layer[m->decoder.n_layers - 1].out_features != 2) return fail(MSW_ERR_INVALID, "decoder output != 2");
  if (m->residual_weights) {
    P->resw_off = P->blob.alloc(2 * P->p);
    for (int i = 0; i < 2 * P->p; ++i) P->blob.h[P->resw_off + i] = m->residual_weights[i];
  }
  const int ef_raw = g->num_edge_features;
  if (m->edge_mlp) {
    if ((rc = pack_mlp(P->blob, m->edge_encoder, P->edge_enc))) return rc;
    if (m->edge_encoder.layer[0].in_features != ef_raw) return fail(MSW_ERR_INVALID, "edge encoder input width");
    if (ef_raw > 16) return fail(MSW_ERR_UNSUPPORTED, "more than 16 raw edge features");
  } else if (ef_raw > F) {
    return fail(MSW_ERR_UNSUPPORTED, "more raw edge features than F");
  }
  const int ef = m->edge_mlp ? F : ef_raw;
  P->procs.resize(m->num_processors);
  for (int j = 0; j < m->num_processors; ++j) {
    const int S = P->S;
    const int scale = P->model_type == 1 ? 0 : (j <= S - 1 ? j : 2 * S - 2 - j);
    if (m->processors[j].edge_features != ef) return fail(MSW_ERR_INVALID, "processor edge_features mismatch");
    if ((rc = build_proc(P.get(), m->processors[j], scale, false, P->procs[j]))) return rc;
  }
  P->unpools.resize(P->model_type == 0 ? m->num_unpool : 0);
  for (size_t i = 0; i < P->unpools.size(); ++i) {
    if (m->unpool[i].edge_features != 0) return fail(MSW_ERR_INVALID, "intra-scale layer with edge features");
    if (m->unpool[i].K != 1) return fail(MSW_ERR_UNSUPPORTED, "intra-scale layer with K != 1");
    if ((rc = build_proc(P.get(), m->unpool[i], P->S - 2 - (int)i, true, P->unpools[i]))) return rc;
  }

  // ---- device buffers
  if ((rc = pupload(P.get(), &P->dW, P->blob.h))) return rc;
  if ((rc = pupload(P.get(), &P->perm_d, P->perm))) return rc;
  std::vector<int> minus1(N, -1);
  if ((rc = pupload(P.get(), &P->bc_slot_d, minus1))) return rc;
  if ((rc = palloc(P.get(), &P->io_d, 1))) return rc;
  int Emax = 1;
  for (auto& c : P->sc) Emax = std::max(Emax, c.E);
  for (auto& l : P->lv) Emax = std::max(Emax, l.I);
  const size_t NF = (size_t)N * F;
  const size_t NH = (size_t)N * 16 * P->h1t_max;
  float** bufs[] = {&P->xs, &P->xd0, &P->bufA, &P->bufB, &P->xin, &P->xdown, &P->xup};
  for (float** b : bufs) {
    if ((rc = palloc(P.get(), b, NF))) return rc;
    HIP_TRY(hipMemset(*b, 0, NF * sizeof(float)));
  }
  if (P->model_type == 1) {
    P->gnnbuf[0] = P->xin;
    P->gnnbuf[1] = P->xdown;
  }
  if ((rc = palloc(P.get(), &P->U, NH)) || (rc = palloc(P.get(), &P->V, NH))) return rc;
  if ((rc = palloc(P.get(), &P->s, (size_t)Emax * F))) return rc;
  if ((rc = palloc(P.get(), &P->X, (size_t)N * P->nnf))) return rc;

  // ---- static per-edge features: edge encoder + edge part of each processor's layer 1
  if (P->E > 0) {
    const int64_t E = P->E;
    std::vector<float> ea((size_t)E * ef_raw);
    // CSR order, scale by scale (matching ScaleCSR::eorig)
    std::vector<int64_t> sbase(P->S + 1, 0);
    for (int s = 0; s < P->S; ++s) sbase[s + 1] = sbase[s] + P->sc[s].E;
    for (int s = 0; s < P->S; ++s)
      for (int i = 0; i < P->sc[s].E; ++i)
        for (int f = 0; f < ef_raw; ++f)
          ea[(size_t)(sbase[s] + i) * ef_raw + f] = g->edge_attr[(size_t)P->sc[s].eorig[i] * ef_raw + f];
    float* ea_d = nullptr;
    float* enc_d = nullptr;
    int64_t tmp_bytes = 0;
    if ((rc = upload(&ea_d, ea, tmp_bytes))) return rc;
    const float* feat = ea_d;
    int feat_stride = ef_raw, feat_dim = ef_raw;
    if (m->edge_mlp) {
      if ((rc = dalloc(&enc_d, (size_t)E * F, tmp_bytes))) return rc;
      RowMlpArgs ra{};
      ra.mode = 0;
      ra.in = ea_d; ra.in_stride = ef_raw; ra.in_dim = ef_raw; ra.R = (int)E; ra.m = P->edge_enc;
      ra.W = P->dW; ra.out = enc_d; ra.out_stride = F; ra.out_tiles = P->NT;
      HIP_TRY(rowmlp_dispatch(P->NT, ra));
      feat = enc_d; feat_stride = F; feat_dim = F;
    }
    for (size_t j = 0; j < P->procs.size(); ++j) {
      Proc& pr = P->procs[j];
      const msw_linear& L1 = m->processors[j].edge_mlp.layer[0];
      const int H1 = L1.out_features;
      // single-layer MLP: Pe = W1[:, 4F:4F+ef] . feat + b1 (no activation)
      Blob tb;
      MlpDev md{};
      md.n = 1;
      md.l[0].tin = P->NT;       // k_rowmlp<NT, 1>: one NT -> 2NT layer (zero padded)
      md.l[0].tout = 2 * P->NT;
      md.l[0].a_off = pack_operand(tb, L1.weight, L1.in_features, 2 * P->NT, P->NT,
                                   [&](int k) { return k < feat_dim ? 4 * F + k : -1; },
                                   [&](int o) { return o < H1 ? o : -1; });
      md.l[0].b_off = -1;
      if (L1.bias) {
        md.l[0].b_off = tb.alloc(16 * 2 * P->NT);
        for (int o = 0; o < H1; ++o) tb.h[md.l[0].b_off + o] = L1.bias[o];
      }
      md.l[0].act = 0;
      float* tw = nullptr;
      if ((rc = upload(&tw, tb.h, tmp_bytes))) return rc;
      const ScaleCSR& c = P->sc[pr.scale];
      if ((rc = palloc(P.get(), &pr.Pe, (size_t)std::max(c.E, 1) * 16 * pr.h1t))) return rc;
      RowMlpArgs ra{};
      ra.mode = 1;
      ra.in = feat + (size_t)sbase[pr.scale] * feat_stride; ra.in_stride = feat_stride;
      ra.in_dim = feat_dim; ra.R = c.E; ra.m = md; ra.W = tw;
      ra.out = pr.Pe; ra.out_stride = 16 * pr.h1t; ra.out_tiles = pr.h1t;
      HIP_TRY(rowmlp_dispatch(P->NT, ra));
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipFree(tw));
    }
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(ea_d));
    if (enc_d) HIP_TRY(hipFree(enc_d));
  }
  HIP_TRY(hipDeviceSynchronize());
  *out_plan = P.release();
  return MSW_OK;
}

int msw_plan_destroy(msw_plan* plan) {
  if (!plan) return MSW_OK;
  (void)hipSetDevice(plan->device);
  (void)hipDeviceSynchronize();
  delete plan;
  return MSW_OK;
}

int msw_forward(msw_plan* P, const float* x, float* y, void* stream) {
  if (!P || !x || !y) return fail(MSW_ERR_INVALID, "null argument");
  HIP_TRY(hipSetDevice(P->device));
  hipStream_t st = (hipStream_t)stream;
  int rc = step_dispatch(P, x, P->identity ? nullptr : P->perm_d, y, false, st);
  if (rc) return rc;
  P->forward_calls++;
  return MSW_OK;
}

int msw_set_graph_capture(msw_plan* P, int enable) {
  if (!P) return fail(MSW_ERR_INVALID, "null plan");
  P->use_graph = enable ? 1 : 0;
  return MSW_OK;
}

int msw_rollout(msw_plan* P, const float* x0, const float* bc, int32_t bc_tstride,
                const int32_t* node_bc, int32_t n_bc, int32_t type_bc, int32_t T, float* out,
                void* stream) {
  if (!P || !x0 || (!out && T > 0)) return fail(MSW_ERR_INVALID, "null argument");
  if (T < 0) return fail(MSW_ERR_INVALID, "T < 0");
  if (T == 0) return MSW_OK;
  if (n_bc > 0 && (!bc || !node_bc)) return fail(MSW_ERR_INVALID, "BC arrays missing");
  if (n_bc > 0 && bc_tstride < T) return fail(MSW_ERR_INVALID, "BC has fewer time entries than T");
  if (type_bc != 1 && type_bc != 2) return fail(MSW_ERR_INVALID, "type_BC must be 1 or 2 (dataset.py:499-506)");
  HIP_TRY(hipSetDevice(P->device));
  hipStream_t st = (hipStream_t)stream;
  // BC slots (internal rows) and the device I/O record, set by kernels whose arguments
  // carry the values: no host buffer lifetime issue and no host synchronisation.
  std::vector<int> rows;
  for (int b = 0; b < n_bc; ++b) {
    if (node_bc[b] < 0 || node_bc[b] >= P->N) return fail(MSW_ERR_INVALID, "node_BC out of range");
    rows.push_back(P->iperm[node_bc[b]]);
  }
  if (rows != P->bc_rows_set) {
    for (size_t i = 0; i < P->bc_rows_set.size(); i += kSlotBatch) {
      SlotArgs sa{};
      sa.slot = P->bc_slot_d;
      sa.n = (int)std::min(P->bc_rows_set.size() - i, (size_t)kSlotBatch);
      for (int k = 0; k < sa.n; ++k) { sa.row[k] = P->bc_rows_set[i + k]; sa.val[k] = -1; }
      HIP_TRY(launch_set_slots(sa, st));
    }
    for (size_t i = 0; i < rows.size(); i += kSlotBatch) {
      SlotArgs sa{};
      sa.slot = P->bc_slot_d;
      sa.n = (int)std::min(rows.size() - i, (size_t)kSlotBatch);
      for (int k = 0; k < sa.n; ++k) { sa.row[k] = rows[i + k]; sa.val[k] = (int)(i + k); }
      HIP_TRY(launch_set_slots(sa, st));
    }
    P->bc_rows_set = rows;
  }
  RolloutIO io{};
  io.bc = bc; io.out = out; io.bc_tstride = bc_tstride; io.type_bc = type_bc; io.T = T; io.step = -1;
  HIP_TRY(launch_set_io(P->io_d, io, st));
  InitArgs ia{};
  ia.x0 = x0; ia.perm = P->identity ? nullptr : P->perm_d; ia.N = P->N; ia.nnf = P->nnf;
  ia.dyn = P->dyn; ia.p = P->p; ia.X = P->X; ia.io = P->io_d; ia.bc_slot = P->bc_slot_d;
  HIP_TRY(launch_init_state(ia, st));
  if (P->use_graph && T > 0) {
    if (!P->step_exec) {
      if (!P->cap_stream) HIP_TRY(hipStreamCreateWithFlags(&P->cap_stream, hipStreamNonBlocking));
      hipGraph_t graph = nullptr;
      HIP_TRY(hipStreamBeginCapture(P->cap_stream, hipStreamCaptureModeThreadLocal));
      int rc = step_dispatch(P, P->X, nullptr, nullptr, true, P->cap_stream);
      hipError_t ce = hipStreamEndCapture(P->cap_stream, &graph);
      if (rc) return rc;
      if (ce != hipSuccess) return fail(MSW_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
      hipError_t ie = hipGraphInstantiate(&P->step_exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      if (ie != hipSuccess) {
        P->step_exec = nullptr;
        return fail(MSW_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
      }
    }
    for (int t = 0; t < T; ++t) HIP_TRY(hipGraphLaunch(P->step_exec, st));
  } else {
    for (int t = 0; t < T; ++t) {
      int rc = step_dispatch(P, P->X, nullptr, nullptr, true, st);
      if (rc) return rc;
    }
  }
  P->rollout_steps += T;
  P->forward_calls += T;
  return MSW_OK;
}

int msw_bench_kernel(msw_plan* P, int32_t kernel, int32_t scale, int32_t iters, int64_t* units,
                     void* stream) {
  if (!P || iters < 0) return fail(MSW_ERR_INVALID, "bad argument");
  HIP_TRY(hipSetDevice(P->device));
  hipStream_t st = (hipStream_t)stream;
  switch (P->NT) {
    case 1: return bench_kernel<1>(P, kernel, scale, iters, units, st);
    case 2: return bench_kernel<2>(P, kernel, scale, iters, units, st);
    default: return bench_kernel<4>(P, kernel, scale, iters, units, st);
  }
}

int msw_debug_buffer(msw_plan* P, const char* name, float* dst, void* stream) {
  if (!P || !name || !dst) return fail(MSW_ERR_INVALID, "null argument");
  const float* src = nullptr;
  if (!strcmp(name, "x_s")) src = P->xs;
  else if (!strcmp(name, "x_d")) src = P->xd0;
  else if (!strcmp(name, "x_down")) src = P->xdown;
  else if (!strcmp(name, "x_in")) src = P->xin;
  else if (!strcmp(name, "x_up")) src = P->model_type == 0 ? P->xup : nullptr;
  if (!src) return fail(MSW_ERR_INVALID, std::string("unknown buffer ") + name);
  if (!P->identity) return fail(MSW_ERR_UNSUPPORTED, "debug buffers only for identity numbering");
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipMemcpy2DAsync(dst, P->F * sizeof(float), src, P->F * sizeof(float), P->F * sizeof(float),
                           P->N, hipMemcpyDeviceToDevice, st));
  return MSW_OK;
}

int msw_plan_get_stats(const msw_plan* P, msw_plan_stats* s) {
  if (!P || !s) return fail(MSW_ERR_INVALID, "null argument");
  s->num_nodes = P->N;
  s->num_edges = P->E;
  s->num_scales = P->S;
  s->hid_features = P->F;
  s->padded_features = P->F;
  s->kernels_per_step = P->kernels_per_step;
  s->forward_calls = P->forward_calls;
  s->rollout_steps = P->rollout_steps;
  s->device_bytes = P->dev_bytes;
  s->graph_captured = P->step_exec != nullptr;
  return MSW_OK;
}

}  // extern "C"
