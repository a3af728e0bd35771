// Host side of the C ABI (include/mswegnn.h): graph plan (16-row-aligned internal
// numbering, CSR by destination, edge tiles, pooling / unpooling maps), weight packing
// for the gfx950 kernels, the per-step schedule of MSGNN.forward / GNN.forward and the
// fused rollout (one hipGraph per step, replayed T times).
//
// Reference semantics followed (sdat2/mSWE-GNN):
//   MSGNN.forward  models/gnn.py:267-350     GNN.forward  models/gnn.py:102-152
//   SWEGNN.forward models/gnn.py:387-445     rollout_test training/train.py:67-95
//   update_batch_multiscale training/train.py:31-65 (batched node_ptr layout)
#include <atomic>
#include <cmath>
#include <cstdio>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/mswegnn.h"
#include "tiling.h"
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

inline int tiles16(int n) { return (n + 15) / 16; }

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
// W[16 to + (l & 15)][16 ti + 4 (l >> 4) + r] (register layout: kernels_impl.h).
// in_map(k) / out_map(o): original column / row of packed input feature k / output
// feature o, or -1 for a zero pad.
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

// Every layer gets a bias vector (zeros for bias=False): the kernels add it unconditionally.
int pack_bias(Blob& B, const float* b, int out_dim, int tout) {
  const int off = B.alloc((size_t)16 * tout);
  if (b)
    for (int o = 0; o < out_dim; ++o) B.h[off + o] = b[o];
  return off;
}

// Pack a make_mlp stack (natural feature order in and out).
int pack_mlp(Blob& B, const msw_mlp& m, MlpDev& d) {
  if (m.n_layers < 1 || m.n_layers > kMaxLayers)
    return fail(MSW_ERR_UNSUPPORTED, "MLP depth must be 1.." + std::to_string(kMaxLayers));
  d.n = m.n_layers;
  for (int i = 0; i < m.n_layers; ++i) {
    const msw_linear& L = m.layer[i];
    if (!L.weight || L.in_features <= 0 || L.out_features <= 0)
      return fail(MSW_ERR_INVALID, "MLP layer without weight");
    if (L.act < 0 || L.act > 7) return fail(MSW_ERR_INVALID, "unknown activation code");
    const int tin = tiles16(L.in_features), tout = tiles16(L.out_features);
    const int din = L.in_features, dout = L.out_features;
    d.l[i].tin = tin;
    d.l[i].tout = tout;
    d.l[i].a_off = pack_operand(B, L.weight, din, tout, tin, [&](int k) { return k < din ? k : -1; },
                                [&](int o) { return o < dout ? o : -1; });
    d.l[i].b_off = pack_bias(B, L.bias, dout, tout);
    d.l[i].act = L.act;
    d.l[i].slope = L.act_param;
  }
  return MSW_OK;
}

// every activation of the MLP is a PReLU with slope <= 1, slope != 0: the compile-time PReLU
// kernels (kernels/k_base.h act_static<1>: max(x, slope x)); otherwise the run-time switch
int all_prelu(const msw_mlp& m) {
  for (int i = 0; i < m.n_layers; ++i) {
    const float s = m.layer[i].act_param;
    if (m.layer[i].act != MSW_ACT_PRELU || !(s <= 1.f && s != 0.f)) return 0;
  }
  return 1;
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

hipError_t rowmlp_dispatch(int NT, const RowMlpArgs& ra, hipStream_t st = nullptr) {
  switch (NT) {
    case 1: return launch_rowmlp<1>(ra, st);
    case 2: return launch_rowmlp<2>(ra, st);
    default: return launch_rowmlp<4>(ra, st);
  }
}

}  // namespace

// ============================================================================ plan
struct ScaleCSR {
  int n0 = 0, ns = 0;           // internal rows [n0, n0+ns) (n0 is a multiple of 16)
  int E = 0;                    // edges of this scale
  LaneRec* recs = nullptr;      // [ntiles][16]
  int ntiles = 0;
  EdgeChunk* chunks = nullptr;  // [nchunks][16] dense edge chunks (k_edge_mlp)
  int nchunks = 0;
  int* rptr = nullptr;          // row-layout middle hops (k_hop_rows, large scales): CSR by
  int2* redge = nullptr;        // destination, {source row, s slot} per edge

  std::vector<int> porig;       // tile-padded edge slot -> original edge id, -1 = padding
  std::vector<LaneRec> hrecs;   // host copy of recs (fused pooling slots, PoolSlot)
};

struct LevelMaps {              // level l: coarse scale l+1, fine scale l
  int I = 0;
  PoolRec* pool_recs = nullptr; // per coarse row (scale l+1): its children (engine.h PoolRec)
  LaneRec* pool_erecs = nullptr; // edge tiles of coarse nodes and their children (<= 16 per tile)
  int pool_etiles = 0;
  int* pool_child = nullptr;    // internal fine rows, reference order
  PoolSlot* pool_slots = nullptr; // per edge slot of the coarse scale: children of its source /
                                  // destination (pooling fused into the coarse edge hop)
  int2* parent_slots = nullptr;   // per edge slot of the fine scale: parents of its source /
                                  // destination (unpooling fused into the fine edge hop)
  LaneRec* un_recs = nullptr;   // fine nodes (scale l) and their coarse parents
  int un_ntiles = 0;
};

struct Proc {                   // one SWEGNN layer bound to a scale (or an intra level)
  int scale = 0;
  int K = 0, normalize = 1, with_filter = 1, with_gradient = 1, upwind = 0;
  int h1t = 1;
  int a_u = -1, a_v = -1, a_o = -1;  // projection operands ([x_s | x_d] -> U, V, O)
  int a_vu = -1;                // intra layers: V from x_s only (fine rows)
  float* Pe = nullptr;          // [E][16*h1t] (layers with edge features)
  int b1_off = -1;              // bias of the first edge-MLP layer
  int act1 = 0;
  float slope1 = 0.f;
  MlpDev rest{};                // layers 2..L
  std::vector<int> filt;        // packed filters 1..K
  int prelu = 0;
  int par = 0;                  // buffer set (execution index & 1)
};

// RCCL, bound at run time: the copy already in the process (PyTorch's) or librccl.so.1.
struct RcclApi {
  ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*groupStart)() = nullptr;
  ncclResult_t (*groupEnd)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*errStr)(ncclResult_t) = nullptr;
  bool ok = false;
};
static RcclApi& rccl() {
  static RcclApi api = [] {
    RcclApi a;
    void* h = RTLD_DEFAULT;
    if (!dlsym(h, "ncclSend")) {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) return a;
    }
    a.getUniqueId = (decltype(a.getUniqueId))dlsym(h, "ncclGetUniqueId");
    a.commInitRank = (decltype(a.commInitRank))dlsym(h, "ncclCommInitRank");
    a.commDestroy = (decltype(a.commDestroy))dlsym(h, "ncclCommDestroy");
    a.groupStart = (decltype(a.groupStart))dlsym(h, "ncclGroupStart");
    a.groupEnd = (decltype(a.groupEnd))dlsym(h, "ncclGroupEnd");
    a.send = (decltype(a.send))dlsym(h, "ncclSend");
    a.recv = (decltype(a.recv))dlsym(h, "ncclRecv");
    a.errStr = (decltype(a.errStr))dlsym(h, "ncclGetErrorString");
    a.ok = a.getUniqueId && a.commInitRank && a.commDestroy && a.groupStart && a.groupEnd && a.send &&
           a.recv && a.errStr;
    return a;
  }();
  return api;
}

// One kernel launch of a step, arguments fixed at plan time (forward mode patches the
// input / output pointers per call).
enum LaunchKind { L_ENCODE, L_EDGE_HOP, L_HOP, L_POOL, L_EXCHANGE, L_EPI, L_EDGE_MLP, L_DECODE };

// Halo exchange before a gathering launch (partitioned meshes, msw_plan_create_part):
// refresh the halo rows of up to two of the plan's buffers on one scale.
enum BufId { B_U0, B_U1, B_O0, B_O1, B_T0, B_T1 };
struct ExchangeArgs {
  Common c;
  int scale;
  int nbuf;
  int buf[2];    // BufId
  int width[2];  // floats per row
};
struct Launch {
  int kind;
  int scale;                    // destination scale (bench hook)
  union {
    EncodeArgs enc;
    EdgeHopArgs eh;
    HopArgs hop;
    PoolArgs pool;
    ExchangeArgs xch;
    EpiArgs ep;
    DecodeArgs dec;
  };
  Launch() { memset((void*)this, 0, sizeof(*this)); }
  Common& common() {
    switch (kind) {
      case L_ENCODE: return enc.c;
      case L_EDGE_HOP:
      case L_EDGE_MLP: return eh.c;
      case L_HOP: return hop.c;
      case L_EXCHANGE: return xch.c;
      case L_EPI: return ep.c;
      case L_DECODE: return dec.c;
      default: return pool.c;
    }
  }
};

// Engine switches: read ONCE per plan (knobs_from_env) from MSW_* environment variables.
// Defaults are the measured-best settings; every switch flips a schedule between variants
// that are bit-identical (each has a -m gpu test that flips it), so a stray variable can
// change speed, never results.  bench.py records the MSW_* variables of its process.
struct Knobs {
  int split_edge_mlp = -1;  // MSW_SPLIT_EDGE_MLP  F = 64 split edge MLP: -1 size rule, 0 / 1 force
  int pool_fuse = 1;        // MSW_POOL_FUSE       mean pooling fused into the coarse first launch
  int unpool_fuse = 1;      // MSW_UNPOOL_FUSE     F = 32 unpooling fused into the fine first launch
  int defer_decode = -1;    // MSW_DEFER_DECODE    decoder in the next step's encoder: -1 size rule
  int hop_rows = -1;        // MSW_HOP_ROWS        row-layout middle hops: -1 size rule, 0 off, 2 all
  int coop2_direct = 1;     // MSW_COOP2_DIRECT    F = 64 two-wave edge hop, blob-read MLP: 0 / 1 / 2
  int coop2_f64 = 1;        // MSW_COOP2_F64       F = 64 two-wave edge hops: 0 off, 2 also for four
  int enc_coop = -1;        // MSW_ENC_COOP        cooperative encoder: -1 size rule, 0 / 1 force
  int eh_loop = 0;          // MSW_EH_LOOP         grid-stride fused edge hops at any size
  int hop_split = -1;       // MSW_HOP_SPLIT       feature-split middle hops: -1 = F = 64 rule
  int pool_wide = 1;        // MSW_POOL_WIDE       2F / 16 waves per pooling tile
  int tile_pack = 1;        // MSW_TILE_PACK       degree-aware destination order
  int xcd_max = 1;          // MSW_XCD_MAX         XCD packing of small grids (0 = all eight XCDs)
  int coop_waves = -1;      // MSW_COOP_WAVES      cooperative kernels while P x tiles <= this (-1 default)
  int epi_split_tiles = -1; // MSW_EPI_SPLIT_TILES row-epilogue threshold in edge tiles (-1 default)
  int trace_encode = 0;     // MSW_TRACE_ENCODE    diagnostic builds (-DMSW_TRACE): encoder marks only
};
inline Knobs knobs_from_env() {
  Knobs k;
  const struct { const char* name; int* v; } tab[] = {
      {"MSW_SPLIT_EDGE_MLP", &k.split_edge_mlp}, {"MSW_POOL_FUSE", &k.pool_fuse},
      {"MSW_UNPOOL_FUSE", &k.unpool_fuse}, {"MSW_DEFER_DECODE", &k.defer_decode}, {"MSW_HOP_ROWS", &k.hop_rows},
      {"MSW_COOP2_DIRECT", &k.coop2_direct}, {"MSW_COOP2_F64", &k.coop2_f64}, {"MSW_ENC_COOP", &k.enc_coop},
      {"MSW_EH_LOOP", &k.eh_loop},
      {"MSW_HOP_SPLIT", &k.hop_split}, {"MSW_POOL_WIDE", &k.pool_wide}, {"MSW_TILE_PACK", &k.tile_pack},
      {"MSW_XCD_MAX", &k.xcd_max}, {"MSW_COOP_WAVES", &k.coop_waves},
      {"MSW_EPI_SPLIT_TILES", &k.epi_split_tiles}, {"MSW_TRACE_ENCODE", &k.trace_encode}};
  for (const auto& t : tab)
    if (const char* e = getenv(t.name)) *t.v = atoi(e);
  return k;
}

struct msw_plan {
  int device = 0;
  int model_type = 0, F = 32, NT = 2, S = 1, p = 3, nnf = 8, dyn = 6, nstat_raw = 2;
  int with_wl = 1, skip = 1;
  int N = 0, Npad = 0;
  int64_t E = 0;
  std::vector<int> perm, iperm;  // internal -> graph (-1 padding), graph -> internal
  std::vector<ScaleCSR> sc;
  std::vector<LevelMaps> lv;
  std::vector<Proc> procs, unpools;
  MlpDev stat{}, dynm{}, dec{}, edge_enc{};
  int gnn_act = 0;
  float gnn_slope = 0.f;
  int resw_off = -1;
  int prelu = 0;
  Blob blob;
  float* dW = nullptr;
  int* perm_d = nullptr;
  int* bc_slot_d = nullptr;
  float* zrow_d = nullptr;
  std::vector<int> bc_rows_set;
  RolloutIO* io_d = nullptr;
  // Edge terms of the processors' first edge-MLP layer (edge encoder, gnn.py:281-282, then
  // Pe = W1[:, 4F:] . enc + b1 per processor): static for a graph, computed at plan creation
  // for msw_forward and recomputed at the start of every msw_rollout (edge_jobs, in order).
  std::vector<RowMlpArgs> edge_jobs;
  // O / U / V of consecutive SWEGNN layers alternate between two sets (Proc::par): the
  // last hop of layer j reads O[j&1] (K = 1: also U/V[j&1]) while its epilogue writes the
  // projection of layer j+1.  T[0] / T[1] carry the intermediate hops.
  float *X = nullptr, *xs = nullptr, *xd0 = nullptr;
  float *O[2] = {nullptr, nullptr}, *T[2] = {nullptr, nullptr};
  float *xdown = nullptr, *xup = nullptr, *xgnn = nullptr;
  float *U[2] = {nullptr, nullptr}, *V[2] = {nullptr, nullptr};
  float *Uu = nullptr, *Vu = nullptr, *s = nullptr;
  int h1t_max = 1;
  int64_t dev_bytes = 0;
  int64_t forward_calls = 0, rollout_steps = 0;
  // RCCL transport: ncclSend / ncclRecv calls issued (eagerly or into a captured graph) and
  // rollout steps whose halo exchanges ran over RCCL (eager steps and graph replays)
  int64_t rccl_calls = 0, rccl_steps = 0;
  int kernels_per_step = 0;
  std::vector<Launch> sched_fwd, sched_roll;  // one forward step: forward / rollout mode
  int use_graph = 1;
  // A layer's last hop on a scale with at least this many edge tiles runs as a middle hop
  // + a row epilogue launch (engine.h EpiArgs); MSW_EPI_SPLIT_TILES overrides (0: never).
  // Measured on MI355X (profiles/r01_v7/ab_epi_split.txt).
  int epi_split_tiles = 8192;
  // partitioned mesh (msw_plan_create_part): per scale, the halo rows received from / the
  // owned rows sent to each peer (internal rows, concatenated in peer order)
  struct XchPeer { int peer, roff, rcount, soff, scount; };
  struct XchScale {
    int nrecv = 0, nsend = 0;
    int* recv_rows = nullptr;
    int* send_rows = nullptr;
    std::vector<XchPeer> peers;
  };
  int part_rank = -1;
  std::vector<XchScale> xch;
  ncclComm_t comm = nullptr;
  float *xsend = nullptr, *xrecv = nullptr;
  hipStream_t cap_stream = nullptr;
  hipGraphExec_t step_exec = nullptr;   // one rollout step
  hipGraphExec_t multi_exec = nullptr;  // graph_steps consecutive steps (one graph launch)
  // Forward mode (msw_forward, the reference's own rollout loop calls it once per step): the
  // forward schedule captured once with fixed device I/O slots; a call copies x into fwd_x,
  // replays the graph and copies fwd_y out -- three stream operations instead of ~35 eager
  // launches (host-launch-bound at ~3.5 us each).
  hipGraphExec_t fwd_exec = nullptr;
  float *fwd_x = nullptr, *fwd_y = nullptr;
  // Steps per graph launch: consecutive launches of one graph leave a ~8.5 us gap on the
  // device (measured, rocprofv3 step breakdown), inside a graph the steps run back to back.
  int graph_steps = 16;
  // Cooperative kernels (several waves per tile: edge hop, last hop, pooling) while
  // waves-per-tile x tiles <= coop_waves (MSW_COOP_WAVES; 0: never).
  // small one-round grids on at most this many XCDs (engine.h Common::xcd, MSW_XCD_MAX;
  // 0 = all eight)
  int xcd_max = 1;
  int coop_waves = 1024;
  Knobs kn;                 // engine switches of this plan (knobs_from_env)
  // set when a fused (un)pooling launch's weight region would not fit its kernel's LDS cap
  // (edge_coop_lds_cap): the schedule is rebuilt with the pooling / unpooling launches
  int no_fuse = 0;
  std::vector<void*> owned;
  // In-process group of partitioned plans (msw_group_rollout): the group's steps captured as
  // graphs too (every part's launches and the halo copies between their buffers), held by the
  // group's plan 0 and keyed by the members' identities and graph generations
  uint64_t uid = 0;              // unique per plan created in this process
  int graph_gen = 0;             // advanced whenever this plan's captured arguments go stale
  int group_graph = 1;           // msw_set_graph_capture(plans[0], 0): the group steps eagerly
  hipGraphExec_t group_one = nullptr, group_multi = nullptr;
  std::vector<uint64_t> group_key;
  void drop_group_graphs() {
    if (group_one) (void)hipGraphExecDestroy(group_one);
    if (group_multi) (void)hipGraphExecDestroy(group_multi);
    group_one = group_multi = nullptr;
    group_key.clear();
  }
  void drop_graphs() {
    if (step_exec) (void)hipGraphExecDestroy(step_exec);
    if (multi_exec) (void)hipGraphExecDestroy(multi_exec);
    if (fwd_exec) (void)hipGraphExecDestroy(fwd_exec);
    step_exec = multi_exec = fwd_exec = nullptr;
    drop_group_graphs();
    ++graph_gen;
  }
  ~msw_plan() {
    drop_graphs();
    if (comm && rccl().ok) (void)rccl().commDestroy(comm);
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
// host I2 pairs (graph_build.h) into a device int2 array (same layout)
int pupload(msw_plan* P, int2** p, const std::vector<I2>& v) {
  static_assert(sizeof(I2) == sizeof(int2), "I2 mirrors int2");
  int rc = palloc(P, p, v.size());
  if (!rc && !v.empty()) HIP_TRY(hipMemcpy(*p, v.data(), v.size() * sizeof(I2), hipMemcpyHostToDevice));
  return rc;
}


// SWEGNN layer -> packed Proc (gnn.py:352-445).
int build_proc(msw_plan* P, const msw_swegnn& g, int scale, bool intra, Proc& pr) {
  const int F = P->F, NT = P->NT;
  pr.scale = scale;
  pr.K = g.K;
  pr.normalize = g.normalize;
  pr.with_filter = g.with_filter_matrix;
  pr.with_gradient = g.with_gradient;
  pr.upwind = g.upwind_mode;
  if (g.K < 1) return fail(MSW_ERR_UNSUPPORTED, "SWEGNN with K < 1");
  const msw_mlp& m = g.edge_mlp;
  if (m.n_layers < 1 || m.n_layers > kMaxLayers) return fail(MSW_ERR_UNSUPPORTED, "edge MLP depth must be 1..4");
  const msw_linear& L1 = m.layer[0];
  const int ef = g.edge_features;
  if (L1.in_features != 4 * F + ef) return fail(MSW_ERR_INVALID, "edge MLP input width != 4F + edge_features");
  const int H1 = L1.out_features;
  if (H1 != (m.n_layers > 1 ? 2 * F : F)) return fail(MSW_ERR_UNSUPPORTED, "edge MLP hidden width must be 2F");
  for (int i = 1; i < m.n_layers; ++i)
    if (m.layer[i].in_features != 2 * F || m.layer[i].out_features != (i == m.n_layers - 1 ? F : 2 * F))
      return fail(MSW_ERR_UNSUPPORTED, "edge MLP layer widths must be 2F -> ... -> F");
  pr.h1t = tiles16(H1);
  P->h1t_max = std::max(P->h1t_max, pr.h1t);
  const int din = L1.in_features;
  const float* W1 = L1.weight;
  auto outm = [&](int o) { return o < H1 ? o : -1; };
  // cat(x_s[row], x_s[col], x_d[row], x_d[col], e_ij) (gnn.py:414-420): U takes the row
  // (source) blocks, V the col (receiving) blocks; packed input = [x_s (F) | x_d (F)]
  auto in_u = [&](int k) { return k < F ? k : (k < 2 * F ? 2 * F + (k - F) : -1); };
  auto in_v = [&](int k) { return k < F ? F + k : (k < 2 * F ? 3 * F + (k - F) : -1); };
  pr.a_u = pack_operand(P->blob, W1, din, pr.h1t, 2 * NT, in_u, outm);
  pr.a_v = pack_operand(P->blob, W1, din, pr.h1t, 2 * NT, in_v, outm);
  if (intra)  // fine rows enter with x_d = 0: V from the x_s block alone
    pr.a_vu = pack_operand(P->blob, W1, din, pr.h1t, NT, [&](int k) { return k < F ? F + k : -1; }, outm);
  pr.act1 = L1.act;
  pr.slope1 = L1.act_param;
  pr.b1_off = P->blob.alloc(16 * pr.h1t);
  if (L1.bias)
    for (int o = 0; o < H1; ++o) P->blob.h[pr.b1_off + o] = L1.bias[o];
  auto idF = [&](int q) { return q < F ? q : -1; };
  if (g.with_filter_matrix) {
    if (intra) return fail(MSW_ERR_UNSUPPORTED, "intra-scale SWEGNN with filter matrix");
    if (!g.filter) return fail(MSW_ERR_INVALID, "with_filter_matrix but no filter weights");
    pr.a_o = pack_operand(P->blob, g.filter[0], F, NT, NT, idF, idF);
    for (int k = 1; k <= g.K; ++k) pr.filt.push_back(pack_operand(P->blob, g.filter[k], F, NT, NT, idF, idF));
  } else if (!intra) {
    // out = x_d.clone() (gnn.py:404): identity operand, exact (1*x + 0*y sums)
    std::vector<float> I((size_t)F * F, 0.f);
    for (int i = 0; i < F; ++i) I[(size_t)i * F + i] = 1.f;
    pr.a_o = pack_operand(P->blob, I.data(), F, NT, NT, idF, idF);
  }
  pr.rest.n = m.n_layers - 1;
  for (int i = 1; i < m.n_layers; ++i) {
    const msw_linear& L = m.layer[i];
    const int di = L.in_features, dout = L.out_features;
    LayerDev& d = pr.rest.l[i - 1];
    d.tin = tiles16(di);
    d.tout = tiles16(dout);
    d.a_off = pack_operand(P->blob, L.weight, di, d.tout, d.tin, [&](int k) { return k < di ? k : -1; },
                           [&](int o) { return o < dout ? o : -1; });
    d.b_off = pack_bias(P->blob, L.bias, dout, d.tout);
    d.act = L.act;
    d.slope = L.act_param;
  }
  pr.prelu = all_prelu(m);
  return MSW_OK;
}

NpDesc np_of(msw_plan* P, const Proc& pr) {
  NpDesc d{};
  d.a_u = pr.a_u; d.a_v = pr.a_v; d.a_o = pr.a_o; d.h1t = pr.h1t;
  d.U = P->U[pr.par]; d.V = P->V[pr.par]; d.O = P->O[pr.par];
  return d;
}
NpDesc np_none() {
  NpDesc d{};
  d.a_u = d.a_v = d.a_o = -1;
  d.h1t = 1;
  return d;
}

Common common_of(msw_plan* P) {
  Common c{};
  c.W = P->dW; c.perm = P->perm_d; c.nnf = P->nnf; c.dyn = P->dyn; c.p = P->p; c.zrow = P->zrow_d;
  c.xcd_max = P->xcd_max;
  c.nstat_raw = P->nstat_raw; c.with_wl = P->with_wl; c.prelu = P->prelu;
  return c;
}

DecDesc dec_of(msw_plan* P, const float* x_src, bool rollout, float* y) {
  DecDesc d{};
  d.on = 1;
  d.pre_act = P->model_type == 0 ? P->gnn_act : 0;
  d.pre_slope = P->gnn_slope;
  d.dec = P->dec;
  d.resw_off = P->resw_off;
  d.X = x_src;
  d.x_internal = rollout ? 1 : 0;
  d.y = y;
  d.io = rollout ? P->io_d : nullptr;
  d.bc_slot = P->bc_slot_d;
  return d;
}

// One SWEGNN layer on its scale: fused edge-MLP + hop 1, then hops 2..K; the last hop
// runs `epi` (and stores its output to `out` if non-null).  out_0 is in O[par].
// Partitioned mesh: refresh the halo rows of `bufs` on `scale` before a gathering launch.
void sched_exchange(msw_plan* P, std::vector<Launch>& q, int scale, std::initializer_list<std::pair<int, int>> bufs) {
  if (P->xch.empty() || P->xch[scale].peers.empty()) return;
  Launch L;
  L.kind = L_EXCHANGE;
  L.scale = scale;
  L.xch.c = common_of(P);
  L.xch.scale = scale;
  for (auto& b : bufs) {
    L.xch.buf[L.xch.nbuf] = b.first;
    L.xch.width[L.xch.nbuf] = b.second;
    ++L.xch.nbuf;
  }
  q.push_back(L);
}

constexpr int kSplitMlpTiles = 1024;  // F = 64: split edge MLP from this many edge tiles up
// the layer's edge MLP runs alone (k_edge_mlp) and hop 1 as a k_hop launch
bool edge_mlp_split(const msw_plan* P, const Proc& pr) {
  if (P->NT != 4 || pr.K < 2 || P->part_rank >= 0) return false;  // F = 64 only (F = 32: -3.4 %)
  return P->kn.split_edge_mlp >= 0 ? P->kn.split_edge_mlp != 0 : P->sc[pr.scale].ntiles >= kSplitMlpTiles;
}
void sched_proc(msw_plan* P, std::vector<Launch>& q, const Proc& pr, float* out, const Epilogue& epi,
                const PoolFuse* pool = nullptr) {
  const ScaleCSR& g = P->sc[pr.scale];
  const Common c = common_of(P);
  sched_exchange(P, q, pr.scale, {{pr.par ? B_U1 : B_U0, 16 * pr.h1t}, {pr.par ? B_O1 : B_O0, P->F}});
  Launch L1;
  L1.kind = L_EDGE_HOP;
  L1.scale = pr.scale;
  EdgeHopArgs& eh = L1.eh;
  eh.c = c; eh.n0 = g.n0; eh.recs = g.recs; eh.ntiles = g.ntiles; eh.xs = P->xs; eh.U = P->U[pr.par]; eh.V = P->V[pr.par]; eh.Pe = pr.Pe;
  eh.b1_off = pr.b1_off; eh.h1t = pr.h1t; eh.act1 = pr.act1; eh.slope1 = pr.slope1;
  eh.rest = pr.rest; eh.normalize = pr.normalize;
  eh.c.prelu = P->prelu & pr.prelu;
  eh.s = pr.K > 1 ? P->s : nullptr;
  eh.in = P->O[pr.par]; eh.own_zero = 0; eh.grad = pr.with_gradient; eh.upwind = pr.upwind;
  eh.filt_a = pr.filt.empty() ? -1 : pr.filt[0];
  eh.skip = nullptr;
  eh.last = pr.K == 1;
  eh.out = pr.K == 1 ? out : P->T[0];
  eh.epi = epi;
  if (pool) eh.pool = *pool;  // U / V / O of this layer formed in the launch (no pooling launch)
  // F = 64 scales beyond one round of the fused kernel (one wave per SIMD): the edge MLP
  // alone over dense edge chunks (k_edge_mlp, two waves per SIMD) + hop 1 as a k_hop launch
  // (MSW_SPLIT_EDGE_MLP=0/1 overrides the size rule)
  const bool split = edge_mlp_split(P, pr);
  if (split) {
    L1.kind = L_EDGE_MLP;
    eh.chunks = g.chunks; eh.nchunks = g.nchunks;
    q.push_back(L1);
    Launch H;
    H.kind = L_HOP;
    H.scale = pr.scale;
    HopArgs& h = H.hop;
    h.c = c;
    h.n0 = g.n0; h.recs = g.recs; h.ntiles = g.ntiles;
    h.nrows = g.ns; h.rptr = g.rptr; h.redge = g.redge;
    h.s = P->s; h.xs = P->xs;
    h.in = P->O[pr.par]; h.out = P->T[0];
    h.filt_a = eh.filt_a;
    h.grad = pr.with_gradient; h.upwind = pr.upwind;
    h.last = 0;
    h.epi = epi;
    q.push_back(H);
  } else {
    q.push_back(L1);
  }
  const float* cur = P->T[0];
  for (int k = 2; k <= pr.K;) {
    sched_exchange(P, q, pr.scale, {{cur == P->T[0] ? B_T0 : B_T1, P->F}});
    // one launch per hop (hop chains -- several hops per launch with the halo recomputed --
    // measured 0.7-1.6 % slower under graph replay, profiles/r01_v7/ab_chains.txt; removed)
    const int m = 1;
    const bool last = k == pr.K;
    float* nxt = last ? out : (cur == P->T[0] ? P->T[1] : P->T[0]);
    Launch L;
    L.scale = pr.scale;
    {
      // the last hop of a large scale: a middle hop into the free ping-pong buffer, then
      // the epilogue on dense node tiles (not on parts: their schedules must stay equal)
      // (only an epilogue with MFMA work gains: a bare store of the layer's output costs a
      // whole extra pass over the rows)
      const bool mfma_epi = epi.np.a_u >= 0 || epi.np.a_v >= 0 || epi.np.a_o >= 0 || epi.uu_a >= 0 || epi.dec.on;
      const bool split = last && mfma_epi && P->part_rank < 0 && P->epi_split_tiles > 0 &&
                         g.ntiles >= P->epi_split_tiles;
      L.kind = L_HOP;
      HopArgs& h = L.hop;
      h.c = c;
      h.n0 = g.n0; h.recs = g.recs; h.ntiles = g.ntiles;
      h.nrows = g.ns; h.rptr = g.rptr; h.redge = g.redge;
      h.s = P->s; h.xs = P->xs;
      h.in = cur; h.out = split ? (cur == P->T[0] ? P->T[1] : P->T[0]) : nxt;
      h.filt_a = pr.filt.empty() ? -1 : pr.filt[k - 1];
      h.grad = pr.with_gradient; h.upwind = pr.upwind;
      h.last = last && !split;
      h.epi = epi;
      if (split) {
        q.push_back(L);
        Launch LE;
        LE.kind = L_EPI;
        LE.scale = pr.scale;
        EpiArgs& ea = LE.ep;
        ea.c = c;
        ea.n0 = g.n0; ea.ns = g.ns; ea.ntiles = (g.ns + kRowsPerWave - 1) / kRowsPerWave;
        ea.in = h.out; ea.xs = P->xs; ea.out = nxt;
        ea.epi = epi;
        L = LE;
      }
    }
    q.push_back(L);
    cur = nxt;
    k += m;
  }
}

constexpr int kMaxFusedPoolBlocks = 256;  // one 4-wave workgroup (two tiles) per CU, one round
// Mean pooling into coarse scale s fused into the first launch of the processor on s
// (k_edge_coop with EdgeHopArgs::pool): F = 32, the scale small enough for the two-wave
// cooperative edge hop in one round (set_grid_cap's k_edge_coop rule), not on parts (their
// halo exchange sits between the two launches).  MSW_POOL_FUSE=0 keeps the pooling launch.
bool pool_fusable(const msw_plan* P, int s, const Proc& pr) {
  if (!P->kn.pool_fuse || P->no_fuse || (P->NT != 2 && P->NT != 4) || P->part_rank >= 0 || s <= 0 || s >= P->S) return false;
  const ScaleCSR& g = P->sc[s];
  // K > 1: the launch is not the layer's last hop (k_edge_coop runs no unpool / decoder epilogue)
  if (pr.scale != s || pr.K < 2 || edge_mlp_split(P, pr) || !P->lv[s - 1].pool_slots || g.ntiles <= 0)
    return false;
  // the scales the cooperative kernels take in one round (F = 32: two waves per tile; F = 64:
  // four, or two with two tiles per workgroup)
  return P->coop_waves > 0 && 2L * g.ntiles <= std::min(P->coop_waves, kWaves * kMaxFusedPoolBlocks);
}

// The unpooling layer into fine scale s fused into the first launch of the processor on s
// (k_edge_coop with PoolFuse::parent), as pool_fusable, F = 32 only (at F = 64 its 384-MFMA
// unpooling MLP per side outweighs the launch it saves: zenodo4_f64 -2.5 %,
// profiles/r03/ab_unpool_fuse_f64.txt); MSW_UNPOOL_FUSE=0 keeps the unpooling launch.
bool unpool_fusable(const msw_plan* P, int s, const Proc& pr, const Proc& up) {
  if (!P->kn.unpool_fuse || P->no_fuse || P->NT != 2 || P->part_rank >= 0 || s < 0 || s + 1 >= P->S) return false;
  const ScaleCSR& g = P->sc[s];
  if (pr.scale != s || pr.K < 2 || edge_mlp_split(P, pr) || !P->lv[s].parent_slots || g.ntiles <= 0) return false;
  if (up.h1t > 2 * P->NT || up.K != 1) return false;
  return P->coop_waves > 0 && 2L * g.ntiles <= std::min(P->coop_waves, kWaves * kMaxFusedPoolBlocks);
}

// One forward.  Forward mode: the encoder reads graph rows of x (via perm) and the decoder
// writes y (both patched per call); rollout mode: the internal state X is updated in place
// by the decoder epilogue.
void sched_step(msw_plan* P, std::vector<Launch>& q, bool rollout) {
  q.clear();
  const int S = P->S;
  const Common c = common_of(P);
  Launch LE;
  LE.kind = L_ENCODE;
  EncodeArgs& ea = LE.enc;
  ea.c = c;
  ea.x = rollout ? P->X : nullptr; ea.x_internal = rollout ? 1 : 0; ea.Npad = P->Npad; ea.S = S;
  for (int s = 0; s < S; ++s) {
    ea.n0[s] = P->sc[s].n0;
    ea.ns[s] = P->sc[s].ns;
    ea.vu_a[s] = -1;
  }
  ea.n0[S] = P->Npad;
  ea.stat = P->stat; ea.dynm = P->dynm; ea.xs = P->xs; ea.xd = P->xd0;
  ea.np0 = np_of(P, P->procs[0]);
  ea.io = rollout ? P->io_d : nullptr;
  ea.vu_h1t = 1;
  if (P->model_type == 0 && S > 1) {
    for (int l = 0; l < S - 1; ++l) ea.vu_a[l] = P->unpools[S - 2 - l].a_vu;  // level l <- intra_scale_gnn[S-2-l]
    ea.vu_h1t = P->unpools[0].h1t;
    ea.Vu = P->Vu;
  }
  const DecDesc dd = dec_of(P, rollout ? P->X : nullptr, rollout, nullptr);
  // rollout mode: the decoder of step t runs in the encoder launch of step t + 1 (and in a
  // final decode-only launch after the last step, msw_rollout); its input is the last
  // layer's output, stored by that layer's last hop (x_up rows / the GNN's last layer)
  // Deferred where the step is latency-bound (zenodo4 +3.2 %, the batch of 8 +1.8 %); on
  // meshes whose finest scale has >= kDeferMaxTiles edge tiles the decoder stays in the last
  // hops' row epilogue (config 5: -1.2 % deferred; profiles/r02_v3/ab_defer_decode.txt).
  // MSW_DEFER_DECODE=0/1 overrides.
  // Forward mode (msw_forward, the reference's own step loop): the decoder leaves the last
  // hops for one row-local launch after the schedule (k_decode_fwd), by the same size rule.
  constexpr int kDeferMaxTiles = 65536;
  bool defer = P->sc[0].ntiles < kDeferMaxTiles;
  if (P->kn.defer_decode >= 0) defer = P->kn.defer_decode != 0;
  if (!rollout && !P->xch.empty()) defer = false;  // parts of a split mesh: decoded in their last hops
  ea.dec = dd;
  ea.dec.on = defer && rollout ? 1 : 0;
  ea.dec_in = P->model_type == 0 ? P->xup : P->xgnn;
  ea.decode_only = 0;
  q.push_back(LE);
  DecDesc dl = dd;  // the last hops' decoder: forward mode, or rollout mode not deferred
  dl.on = defer ? 0 : 1;
  if (P->model_type == 0) {
    Epilogue none{};
    none.np = np_none(); none.uu_a = -1; none.dec.on = 0;
    PoolFuse fuse{};
    for (int i = 0; i < S - 1; ++i) {  // fine -> coarse
      sched_proc(P, q, P->procs[i], P->xdown, none, fuse.slots ? &fuse : nullptr);
      const LevelMaps& m = P->lv[i];
      fuse = PoolFuse{};
      if (pool_fusable(P, i + 1, P->procs[i + 1])) {  // the next processor's first launch pools
        fuse.slots = m.pool_slots; fuse.child = m.pool_child; fuse.in = P->xdown;
        fuse.np = np_of(P, P->procs[i + 1]);
        continue;
      }
      Launch L;
      L.kind = L_POOL;
      L.scale = i + 1;
      PoolArgs& pa = L.pool;
      pa.c = c; pa.n0 = P->sc[i + 1].n0; pa.ns = P->sc[i + 1].ns;
      pa.rtiles = (pa.ns + 15) / 16; pa.etiles = m.pool_etiles;
      pa.rows = 1; pa.ntiles = pa.rtiles;  // set_grid_cap picks the layout
      pa.recs = m.pool_recs; pa.erecs = m.pool_erecs; pa.child = m.pool_child;
      pa.in = P->xdown; pa.xs = P->xs;
      pa.np = np_of(P, P->procs[i + 1]);
      q.push_back(L);
    }
    PoolFuse ufuse{};
    for (int i = 0; i < S; ++i) {      // coarse -> fine
      const int j = S - 1 + i, s = S - 1 - i;
      Epilogue e{};
      e.np = np_none();
      e.uu_a = -1;
      if (s > 0) {
        const Proc& up = P->unpools[i];
        e.uu_a = up.a_u; e.uu_h1t = up.h1t; e.Uu = P->Uu;
      }
      e.dec = dl;  // every scale's rows are decoded once final (gnn.py:335-348)
      sched_proc(P, q, P->procs[j], P->xup, e, i == 0 && fuse.slots ? &fuse : ufuse.parent ? &ufuse : nullptr);
      ufuse = PoolFuse{};
      if (s > 0) {                      // intra_scale_gnn[i] on level s-1 (+ skip) + projection
        const Proc& up = P->unpools[i];
        const ScaleCSR& fs = P->sc[s - 1];
        const LevelMaps& m = P->lv[s - 1];
        if (unpool_fusable(P, s - 1, P->procs[j + 1], up)) {  // the next processor's first launch unpools
          ufuse.parent = m.parent_slots; ufuse.cpad = P->sc[s].n0;
          ufuse.Uu = P->Uu; ufuse.Vu = P->Vu; ufuse.xc = P->xup; ufuse.skip = P->skip ? P->xdown : nullptr;
          ufuse.b1_off = up.b1_off; ufuse.h1t = up.h1t; ufuse.act1 = up.act1; ufuse.slope1 = up.slope1;
          ufuse.rest = up.rest; ufuse.normalize = up.normalize; ufuse.grad = up.with_gradient;
          ufuse.upwind = up.upwind; ufuse.post_act = 0; ufuse.post_slope = 0.f;
          ufuse.np = np_of(P, P->procs[j + 1]);
          continue;
        }
        Launch L;
        L.kind = L_EDGE_HOP;
        L.scale = s - 1;
        EdgeHopArgs& eh = L.eh;
        eh.c = c; eh.c.prelu = P->prelu & up.prelu;
        eh.n0 = fs.n0; eh.recs = m.un_recs; eh.ntiles = m.un_ntiles;
        eh.xs = P->xs; eh.U = P->Uu; eh.V = P->Vu;
        eh.Pe = nullptr; eh.b1_off = up.b1_off; eh.h1t = up.h1t; eh.act1 = up.act1;
        eh.slope1 = up.slope1; eh.rest = up.rest; eh.normalize = up.normalize; eh.s = nullptr;
        eh.in = P->xup; eh.own_zero = 1; eh.grad = up.with_gradient; eh.upwind = up.upwind;
        eh.filt_a = -1; eh.skip = P->skip ? P->xdown : nullptr; eh.out = nullptr; eh.last = 1;
        eh.epi.np = np_of(P, P->procs[j + 1]); eh.epi.uu_a = -1; eh.epi.dec.on = 0;
        q.push_back(L);
      }
    }
  } else {
    const int L = (int)P->procs.size();
    for (int j = 0; j < L; ++j) {
      Epilogue e{};
      e.post_act = P->gnn_act; e.post_slope = P->gnn_slope;
      e.np = j + 1 < L ? np_of(P, P->procs[j + 1]) : np_none();
      e.uu_a = -1;
      if (j + 1 == L) e.dec = dl; else e.dec.on = 0;
      sched_proc(P, q, P->procs[j], P->xgnn, e);
    }
  }
  if (defer && !rollout) {  // forward mode: the deferred decoder, after everything else
    Launch LD;
    LD.kind = L_DECODE;
    LD.scale = 0;
    DecodeArgs& da = LD.dec;
    da.c = c;
    da.c.xcd_max = 0;
    da.Npad = P->Npad;
    da.in = ea.dec_in;
    da.dec = dd;
    da.dec.on = 1;
    q.push_back(LD);
  }
  if (defer && rollout)  // the step counter the next step's encoder reads advances here
    for (Launch& L : q)
      if (L.kind == L_EDGE_HOP || L.kind == L_EDGE_MLP) {
        L.eh.step_inc = &P->io_d->step;
        break;
      }
}

// ---------------------------------------------------------------------------- weight regions
// Copies the operands one launch reads into a contiguous blob region and rewrites the
// launch's offsets to LDS offsets (kernels stage the region per workgroup).
struct RegionBuilder {
  Blob& B;
  int base, shift;
  std::map<int, int> memo;
  RegionBuilder(Blob& b, int sh) : B(b), shift(sh) { base = B.alloc(0); }
  int put(int off, int len) {
    if (off < 0) return off;
    auto it = memo.find(off);
    if (it != memo.end()) return it->second;
    len = (len + 3) & ~3;
    std::vector<float> tmp(len, 0.f);
    for (int i = 0; i < len && off + i < (int)B.h.size(); ++i) tmp[i] = B.h[off + i];
    const int pos = (int)B.h.size();
    B.h.insert(B.h.end(), tmp.begin(), tmp.end());
    const int r = pos - base + shift;
    memo[off] = r;
    return r;
  }
  int pos() const { return (int)B.h.size() - base; }
  WReg done(int split = -1) const {
    const int len = (int)B.h.size() - base;
    return WReg{base, len, split < 0 ? len : split};
  }
};

struct Relocator {
  int NT, p;
  void layer(RegionBuilder& R, LayerDev& L) {
    L.a_off = R.put(L.a_off, L.tout * L.tin * 256);
    L.b_off = R.put(L.b_off, 16 * L.tout);
  }
  void mlp(RegionBuilder& R, MlpDev& m) {
    for (int i = 0; i < m.n; ++i) layer(R, m.l[i]);
  }
  void np(RegionBuilder& R, NpDesc& d) {
    d.a_u = R.put(d.a_u, d.h1t * 2 * NT * 256);
    d.a_v = R.put(d.a_v, d.h1t * 2 * NT * 256);
    d.a_o = R.put(d.a_o, NT * NT * 256);
  }
  void epi(RegionBuilder& R, Epilogue& e) {
    np(R, e.np);
    e.uu_a = R.put(e.uu_a, e.uu_h1t * 2 * NT * 256);
    if (e.dec.on) {
      mlp(R, e.dec.dec);
      e.dec.resw_off = R.put(e.dec.resw_off, 2 * p);
    }
  }
};

constexpr int kMaxRegionFloats = (160 * 1024) / 4 - kWaves * kRowsPerWave * (3 * 32 + 4);  // minus the F=32 slab

// mlp_only (F = 64): only the edge hops' MLP operands (b1, layers 2..L) get a region -- when
// it fits beside the edge slab; every other operand stays a blob offset.
int relocate(msw_plan* P, std::vector<Launch>& q, bool mlp_only = false) {
  Relocator rl{P->NT, P->p};
  for (Launch& L : q) {
    WReg* reg = nullptr;
    int tot = 0;
    if (mlp_only) {
      if (L.kind != L_EDGE_HOP && L.kind != L_EDGE_MLP) continue;
      EdgeHopArgs& a = L.eh;
      const int len = 16 * a.h1t + [&] {
        int n = 0;
        for (int i = 0; i < a.rest.n; ++i) n += a.rest.l[i].tout * a.rest.l[i].tin * 256 + 16 * a.rest.l[i].tout;
        return n;
      }();
      const int slab = kWaves * kRowsPerWave * (48 * P->NT + 4) * (int)sizeof(float);
      if ((len + 255) / 256 * 256 * (int)sizeof(float) + slab > 160 * 1024) continue;  // stays in the blob
      RegionBuilder R(P->blob, 0);
      a.b1_off = R.put(a.b1_off, 16 * a.h1t);
      rl.mlp(R, a.rest);
      a.reg = R.done();
      a.reg_nf = a.reg.len;
      a.filt_l = -1;
      continue;
    }
    if (L.kind == L_ENCODE) {
      // one contiguous region per scale (one LDS-DMA copy per workgroup): the static
      // encoder first -- identical relative offsets in every scale's region -- then the
      // dynamic encoder + projection 0 (scale 0) and that scale's unpool V operand
      EncodeArgs& a = L.enc;
      const MlpDev stat0 = a.stat, dec0 = a.dec.dec;
      const int resw0 = a.dec.resw_off;
      a.reg = WReg{0, 0, 0};
      a.lds_floats = 0;
      for (int s = 0; s < a.S; ++s) {
        RegionBuilder Rs(P->blob, 0);
        MlpDev st = stat0;
        rl.mlp(Rs, st);
        a.stat = st;
        if (a.dec.on) {  // the decoder (rollout mode): same offsets in every scale's region
          MlpDev dm = dec0;
          rl.mlp(Rs, dm);
          a.dec.dec = dm;
          a.dec.resw_off = Rs.put(resw0, 2 * P->p);
        }
        if (s == 0) {
          rl.mlp(Rs, a.dynm);
          rl.np(Rs, a.np0);
        }
        a.vu_a[s] = Rs.put(a.vu_a[s], a.vu_h1t * P->NT * 256);
        a.sreg[s] = Rs.done();
        a.lds_floats = std::max(a.lds_floats, a.sreg[s].len);
      }
      tot = (a.lds_floats + 255) / 256 * 256;
    } else if (L.kind == L_EDGE_MLP) {
      EdgeHopArgs& a = L.eh;  // the MLP operands only
      RegionBuilder R(P->blob, 0);
      a.b1_off = R.put(a.b1_off, 16 * a.h1t);
      rl.mlp(R, a.rest);
      a.reg = R.done();
      a.reg_nf = a.reg.len;
      a.filt_l = -1;
      reg = &a.reg;
    } else if (L.kind == L_EDGE_HOP) {
      EdgeHopArgs& a = L.eh;
      RegionBuilder R(P->blob, 0);
      a.b1_off = R.put(a.b1_off, 16 * a.h1t);
      rl.mlp(R, a.rest);
      if (a.pool.parent) {  // fused unpooling: its edge MLP, then the projection
        a.pool.b1_off = R.put(a.pool.b1_off, 16 * a.pool.h1t);
        rl.mlp(R, a.pool.rest);
      }
      if (a.pool.slots || a.pool.parent) rl.np(R, a.pool.np);  // fused (un)pooling: before the MLP
      const int split = R.pos();  // operands after this one stream in behind the MLP
      if (a.last) rl.epi(R, a.epi);
      // filt_a stays a blob offset (the one-tile-per-wave variant loads it into registers and
      // stages the region without it); the grid-stride variant reads this trailing copy
      a.reg_nf = R.pos();
      a.filt_l = R.put(a.filt_a, P->NT * P->NT * 256);
      a.reg = R.done(split);
      reg = &a.reg;
    } else if (L.kind == L_EXCHANGE || L.kind == L_DECODE) {
      continue;  // no LDS weight region (the forward decode reads its operands from the blob)
    } else if (L.kind == L_EPI) {
      EpiArgs& a = L.ep;
      RegionBuilder R(P->blob, 0);
      rl.epi(R, a.epi);
      a.reg = R.done();
      reg = &a.reg;
    } else if (L.kind == L_HOP) {
      HopArgs& a = L.hop;
      if (!a.last) continue;  // middle hops load their filter from the blob (k_hop<.., false>)
      RegionBuilder R(P->blob, 0);  // filt_a stays a blob offset (k_hop loads it into registers)
      rl.epi(R, a.epi);
      a.reg = R.done();
      reg = &a.reg;
    } else {
      PoolArgs& a = L.pool;
      RegionBuilder R(P->blob, 0);
      rl.np(R, a.np);
      a.reg = R.done();
      reg = &a.reg;
    }
    if (reg) tot = (reg->len + 255) / 256 * 256;  // LDS-DMA chunks
    if (tot > kMaxRegionFloats)
      return fail(MSW_ERR_UNSUPPORTED, "weights of one launch exceed the LDS budget (" + std::to_string(tot * 4) + " B)");
  }
  return MSW_OK;
}

// Grid cap of a grid-stride launch: the workgroups the chip holds at once, so that each
// stages its weight region once (large meshes) and none waits for a second wave of blocks.
int resident_of(int NT, int kind, int prelu, int last, size_t bytes, int loop) {
  switch (NT) {
    case 1: return resident_blocks<1>(kind, prelu, last, bytes, loop);
    case 2: return resident_blocks<2>(kind, prelu, last, bytes, loop);
    default: return resident_blocks<4>(kind, prelu, last, bytes, loop);
  }
}
template <class A>
void caps(msw_plan* P, A& a, int kind, int prelu, int last, int floats) {
  a.max_blocks = resident_of(P->NT, kind, prelu, last, (size_t)floats * 4, 1);
  a.fit_blocks = resident_of(P->NT, kind, prelu, last, (size_t)floats * 4, 0);
}
constexpr int kHopLoopTiles = 65536;
// middle hops of scales with at least this many edge tiles run in the row layout
// (k_hop_rows; MSW_HOP_ROWS=0 keeps the edge tiles)
constexpr int kRowHopMinTiles = kHopLoopTiles;
// MSW_HOP_ROWS=2: every middle hop in the row layout, at any size (parity tests)
bool row_hops_forced(const msw_plan* P) { return P->kn.hop_rows == 2; }
constexpr long kEncCoopWaves = 4096;
void set_grid_cap(msw_plan* P, Launch& L) {
  // XCD packing (Common::xcd_max) applies to the hop, edge-hop, pooling and row-epilogue
  // launches (the only one-round grids small enough to fit one XCD)
  if (L.kind != L_HOP && L.kind != L_EDGE_HOP && L.kind != L_POOL && L.kind != L_EPI) L.common().xcd_max = 0;
  switch (L.kind) {
    case L_ENCODE: {
      L.enc.max_blocks = resident_of(P->NT, 0, L.enc.c.prelu, 0, (size_t)L.enc.lds_floats * 4, 0);
      // F = 64: four waves per row tile while that leaves <= 4 waves per SIMD (k_encode_coop;
      // zenodo4_f64 +5.0 %; at F = 32 the halved chains are too short for the seven LDS
      // exchanges: -2.5 %; MSW_ENC_COOP=0/1 overrides)
      bool coop = P->NT == 4 && (long)(L.enc.Npad / kRowsPerWave) * P->NT <= kEncCoopWaves;
      if (P->kn.enc_coop >= 0) coop = P->NT >= 2 && P->kn.enc_coop != 0;
      L.enc.coop = coop ? P->NT : 0;
      // grid-stride (more 64-row chunks than resident workgroups) without the decoder: the
      // encoder's rows (config 5: 1.26 GB per launch) go out as streaming stores
      L.enc.stream = !L.enc.coop && !L.enc.dec.on && L.enc.max_blocks > 0 &&
                     L.enc.Npad / kRowsPerBlock > L.enc.max_blocks;
      break;
    }
    case L_EDGE_MLP: {
      // k_edge_mlp: two waves per SIMD, one chunk each.  (A software-pipelined variant, one wave
      // per SIMD walking ~2 chunks with the next chunk's gathers in flight, spilled once the
      // operands were LDS-typed and lost: zenodo4_f64 27.76 / 27.91 vs 28.08 / 28.09 M,
      // profiles/r04/ab_f64_lds_operands.txt; removed in round 6.)  Waves 4..7 start 2 x 2 k
      // cycles late (k_edge_mlp 22.0 -> 21.2 us, profiles/r05/ab_f64_mlp_stagger.txt).
      L.eh.stagger = kMlpStagger;
      L.eh.max_blocks = resident_of(P->NT, 10, L.eh.c.prelu, 0, (size_t)L.eh.reg.len * 4, 1);
      break;
    }
    case L_EDGE_HOP: {
      EdgeHopArgs& a = L.eh;
      caps(P, a, 1, a.c.prelu, a.last, a.reg.len);
      a.fit_blocks = resident_of(P->NT, 1, a.c.prelu, a.last, (size_t)a.reg_nf * 4, 0);
      // MSW_EH_LOOP=1: the grid-stride variant at any size (parity tests of the large-mesh path)
      if (P->kn.eh_loop && a.max_blocks > 0 && a.ntiles > kWaves) a.fit_blocks = 1;
      // two waves per tile (k_edge_coop) while the tiles leave most SIMDs idle: one tile
      // per wave at most, no grid-stride loop, an epilogue of projections only
      const bool loop = a.fit_blocks > 0 && a.max_blocks > 0 && (a.ntiles + kWaves - 1) / kWaves > a.fit_blocks;
      const bool epi_ok = !a.last || (!a.epi.dec.on && a.epi.uu_a < 0);
      // ... and its grid resident at once (a second round of workgroups costs more than the
      // halved MLP chain saves: measured +4.7 us on the finest unpooling of zenodo4)
      // (F = 32: two waves per tile; F = 64: four, one tile per workgroup)
      const int pw = P->NT == 2 ? 2 : P->NT == 4 ? 4 : 0;
      const int coop_fit = pw ? resident_of(P->NT, 7, a.c.prelu, a.last, (size_t)a.reg_nf * 4, 0) : 0;
      a.coop = (pw && !loop && epi_ok && P->coop_waves > 0 && (long)pw * a.ntiles <= P->coop_waves &&
                (pw * a.ntiles + kWaves - 1) / kWaves <= coop_fit) ? pw : 0;
      // F = 64 where four waves per tile do not fit one round: two, two tiles per workgroup
      // (zenodo4_f64 scale 1: 508 tiles in one round, +2.0 %; MSW_COOP2_F64=0 off, =2 also in
      // place of four, for tests)
      // fused pooling exists in the cooperative kernels only (pool_fusable): F = 32 two waves
      // per tile; F = 64 four, or two where four do not fit one round (below)
      if ((a.pool.slots || a.pool.parent) && P->NT == 2) a.coop = 2;
      const int c2 = P->kn.coop2_f64;
      if (c2 == 2 && a.coop == 4) a.coop = 0;
      a.wdirect = 0;
      if (P->NT == 4 && !a.coop && !loop && epi_ok && P->coop_waves > 0 && 2L * a.ntiles <= P->coop_waves && c2) {
        const int need = (2 * a.ntiles + kWaves - 1) / kWaves;
        const int wd = P->kn.coop2_direct;
        if (need <= resident_of(P->NT, 12, a.c.prelu, a.last, (size_t)a.reg_nf * 4, 0)) {
          a.coop = 2;
          a.wdirect = wd == 2 && a.reg.len > 0;
        } else if (wd != 0 && a.reg.len > 0 && need <= resident_of(P->NT, 12, a.c.prelu, a.last, 0, 0)) {
          // the staged MLP region (96 KB) holds one workgroup per CU: read it from its blob
          // copy instead, two workgroups per CU, and the grid fits one round (the finest
          // unpooling of zenodo4_f64: 652 tiles; MSW_COOP2_DIRECT=0 off)
          a.coop = 2;
          a.wdirect = 1;
        }
      }
      if ((a.pool.slots || a.pool.parent) && !a.coop) a.coop = 2;  // F = 64 fused: two waves per tile, any grid
      break;
    }
    case L_HOP:
      caps(P, L.hop, 2, L.hop.c.prelu, L.hop.last, L.hop.reg.len);
      // one tile per wave below kHopLoopTiles: the grid-stride variant measured 1.1-1.6 % slower on the batch of 8 and
      // dk15, equal on the 1M-node mesh whose finest hop alone it runs 3 % faster
      // (profiles/r01_v7/ab_edge_waves.txt)
      if (L.hop.ntiles < kHopLoopTiles) L.hop.max_blocks = 0;
      {  // F = 64: feature-split middle hops below the grid-stride size (k_hop_split;
         // zenodo4_f64 +4.6 %, F = 32 neutral; MSW_HOP_SPLIT=0/1 overrides the rule)
        bool sp = P->NT == 4 && L.hop.max_blocks == 0;
        if (P->kn.hop_split >= 0) sp = P->kn.hop_split != 0;
        L.hop.split = (sp && P->NT >= 2 && !L.hop.last) ? 1 : 0;
      }
      {  // row layout for the grid-stride middle hops of large scales (k_hop_rows)
        HopArgs& h = L.hop;
        const bool loop = h.fit_blocks > 0 && h.max_blocks > 0 && (h.ntiles + kWaves - 1) / kWaves > h.fit_blocks;
        const bool want = P->kn.hop_rows != 0;
        h.rows = 0;
        if (want && !h.last && (loop || row_hops_forced(P)) && h.rptr && h.redge) {
          h.rows = 1;
          h.split = 0;
          h.max_blocks = resident_of(P->NT, 14, 0, 0, 0, 1);
        }
      }
      {  // a last hop with an epilogue on few tiles: P = F / 16 waves per tile (k_hop_coop)
        HopArgs& h = L.hop;
        const bool loop = h.fit_blocks > 0 && h.max_blocks > 0 && (h.ntiles + kWaves - 1) / kWaves > h.fit_blocks;
        const int pw = P->NT >= 2 ? P->NT : 0;
        h.coop = 0;
        if (h.last && pw && !loop && P->coop_waves > 0 && (long)pw * h.ntiles <= P->coop_waves &&
            (pw * h.ntiles + kWaves - 1) / kWaves <= resident_of(P->NT, 9, h.c.prelu, 1, (size_t)h.reg.len * 4, 0))
          h.coop = pw;
      }
      break;
    case L_EXCHANGE: break;
    case L_DECODE: break;
    case L_EPI:
      caps(P, L.ep, 6, L.ep.c.prelu, 1, L.ep.reg.len);
      break;
    default: {
      // edge tiles while they all fit on the chip at once (latency-bound launch), else rows
      PoolArgs& a = L.pool;
      const int fe = resident_of(P->NT, 5, 0, 0, (size_t)a.reg.len * 4, 0);
      a.rows = !(fe > 0 && (a.etiles + kWaves - 1) / kWaves <= fe);
      a.ntiles = a.rows ? a.rtiles : a.etiles;
      caps(P, a, 3, 0, 0, a.reg.len);
      // two waves per edge tile (projection split) while that grid too is resident at once
      // (F = 32: two waves per tile, F = 64: four)
      const int pw = P->NT >= 2 ? P->NT : 0;
      a.coop = (!a.rows && pw && P->coop_waves > 0 && (long)pw * a.etiles <= P->coop_waves &&
                (pw * a.etiles + kWaves - 1) / kWaves <= fe) ? pw : 0;
      // 2F-wide first edge-MLP layer: 2 * F / 16 waves per tile (one U and one V output tile
      // each) while resident (zenodo4_f64 +1.8 %, zenodo4 +0.6 %, profiles/r02_s4/ab_pool_p8.txt,
      // ab_pool_wide_f32.txt); MSW_POOL_WIDE=0: F / 16 waves; bit-identical either way
      const bool wide = P->kn.pool_wide != 0;
      if (wide && pw && a.coop == pw && a.np.h1t == 2 * pw) {
        const int f8 = resident_of(P->NT, 13, 0, 0, (size_t)a.reg.len * 4, 0);
        if (f8 > 0 && a.etiles <= f8) a.coop = 2 * pw;
      }
      break;
    }
  }
}

// The first cooperative edge hop whose staged weight region exceeds the dynamic LDS
// prepare_kernels allowed its kernel (edge_coop_lds_cap), or nullptr.
const Launch* lds_overflow(const msw_plan* P) {
  for (const auto* q : {&P->sched_fwd, &P->sched_roll})
    for (const Launch& L : *q) {
      if (L.kind != L_EDGE_HOP || !(L.eh.coop == 2 || L.eh.coop == 4) || L.eh.wdirect) continue;
      const int fuse = L.eh.pool.slots ? 1 : L.eh.pool.parent ? 2 : 0;
      const int cap = P->NT == 4 ? edge_coop_lds_cap<4>(L.eh.coop, fuse) : edge_coop_lds_cap<2>(2, fuse);
      if (eh_lds_bytes(L.eh.reg_nf) > (size_t)cap) return &L;
    }
  return nullptr;
}

template <int NT>
hipError_t launch_one(const Launch& L, hipStream_t st) {
  switch (L.kind) {
    case L_ENCODE: return launch_encode<NT>(L.enc, st);
    case L_EDGE_HOP: return launch_edge_hop<NT>(L.eh, st);
    case L_EDGE_MLP: return launch_edge_mlp<NT>(L.eh, st);
    case L_HOP: return launch_hop<NT>(L.hop, st);
    case L_POOL: return launch_pool<NT>(L.pool, st);
    case L_EPI: return launch_epi<NT>(L.ep, st);
    case L_DECODE: return launch_decode<NT>(L.dec, st);
    default: return hipErrorInvalidValue;  // exchanges are run by run_schedule / the group driver
  }
}

float* buf_of(msw_plan* P, int id) {
  switch (id) {
    case B_U0: return P->U[0];
    case B_U1: return P->U[1];
    case B_O0: return P->O[0];
    case B_O1: return P->O[1];
    case B_T0: return P->T[0];
    default: return P->T[1];
  }
}

// RCCL transport: pack the rows every peer needs into one staging buffer, one grouped
// send/recv per peer, unpack into the halo rows.  Stream-ordered (capturable).
int rccl_exchange(msw_plan* P, const ExchangeArgs& a, hipStream_t st) {
  const msw_plan::XchScale& X = P->xch[a.scale];
  if (!P->comm) return fail(MSW_ERR_INVALID, "partitioned plan without a transport (msw_plan_set_comm)");
  RcclApi& r = rccl();
  for (int b = 0; b < a.nbuf; ++b) {
    float* buf = buf_of(P, a.buf[b]);
    const int w = a.width[b];
    HIP_TRY(launch_copy_rows(buf, X.send_rows, P->xsend, nullptr, X.nsend, w, st));
    ncclResult_t e = r.groupStart();
    for (const auto& pe : X.peers) {
      if (e == ncclSuccess && pe.scount > 0 &&
          (e = r.send(P->xsend + (size_t)pe.soff * w, (size_t)pe.scount * w, ncclFloat32, pe.peer, P->comm, st)) ==
              ncclSuccess)
        ++P->rccl_calls;
      if (e == ncclSuccess && pe.rcount > 0 &&
          (e = r.recv(P->xrecv + (size_t)pe.roff * w, (size_t)pe.rcount * w, ncclFloat32, pe.peer, P->comm, st)) ==
              ncclSuccess)
        ++P->rccl_calls;
    }
    const ncclResult_t e2 = r.groupEnd();
    if (e != ncclSuccess || e2 != ncclSuccess)
      return fail(MSW_ERR_HIP, std::string("RCCL halo exchange: ") + r.errStr(e != ncclSuccess ? e : e2));
    HIP_TRY(launch_copy_rows(P->xrecv, nullptr, buf, X.recv_rows, X.nrecv, w, st));
  }
  return MSW_OK;
}

template <int NT>
int run_schedule(msw_plan* P, const std::vector<Launch>& q, hipStream_t st) {
  for (const Launch& L : q) {
    if (L.kind == L_EXCHANGE) {
      int rc = rccl_exchange(P, L.xch, st);
      if (rc) return rc;
    } else {
      HIP_TRY(launch_one<NT>(L, st));
    }
  }
  P->kernels_per_step = (int)q.size();
  return MSW_OK;
}

int schedule_dispatch(msw_plan* P, const std::vector<Launch>& q, hipStream_t st) {
  switch (P->NT) {
    case 1: return run_schedule<1>(P, q, st);
    case 2: return run_schedule<2>(P, q, st);
    default: return run_schedule<4>(P, q, st);
  }
}

// After a rollout's last step: the decoder of that step (the encoder launch of the rollout
// schedule with decode_only set: no encoders run).
int final_decode(msw_plan* P, hipStream_t st) {
  if (P->sched_roll.empty() || P->sched_roll[0].kind != L_ENCODE || !P->sched_roll[0].enc.dec.on)
    return MSW_OK;
  Launch L = P->sched_roll[0];
  L.enc.decode_only = 1;
  if (P->kn.trace_encode) L.enc.c.trace = nullptr;  // keep the last step's encoder marks
  switch (P->NT) {
    case 1: HIP_TRY(launch_one<1>(L, st)); break;
    case 2: HIP_TRY(launch_one<2>(L, st)); break;
    default: HIP_TRY(launch_one<4>(L, st)); break;
  }
  return MSW_OK;
}

// Forward mode: point the encoder at x (graph rows) and the decoder at x / y.
void patch_forward(std::vector<Launch>& q, const float* x, float* y) {
  for (Launch& L : q) {
    if (L.kind == L_ENCODE) L.enc.x = x;
    if (L.kind == L_DECODE) {
      L.dec.dec.X = x;
      L.dec.dec.y = y;
    }
    Epilogue* e = L.kind == L_EDGE_HOP ? &L.eh.epi : L.kind == L_HOP ? &L.hop.epi
                 : L.kind == L_EPI ? &L.ep.epi : nullptr;
    if (e && e->dec.on) {
      e->dec.X = x;
      e->dec.y = y;
    }
  }
}

int build_graph_plan(msw_plan* P, const msw_graph_desc* g) {
  // the host plan (graph_build.h: numbering, CSRs, tiles, records -- also built by the
  // sanitizer harness tests/asan/host_plan_check.cpp), then its device copies
  HostGraph H;
  std::string err;
  int rc = build_host_graph(g, P->S, kRowsPerBlock, P->kn.tile_pack != 0,
                            row_hops_forced(P) ? 0 : kRowHopMinTiles, H, err);
  if (rc) return fail(rc, err);
  P->N = H.N;
  P->E = H.E;
  P->Npad = H.Npad;
  P->perm = std::move(H.perm);
  P->iperm = std::move(H.iperm);
  const int S = P->S;
  P->sc.assign(S, ScaleCSR{});
  for (int s = 0; s < S; ++s) {
    HostScale& h = H.sc[s];
    ScaleCSR& c = P->sc[s];
    c.n0 = h.n0; c.ns = h.ns; c.E = h.E; c.ntiles = h.ntiles; c.nchunks = h.nchunks;
    if ((rc = pupload(P, &c.recs, h.recs))) return rc;
    if (c.nchunks > 0 && (rc = pupload(P, &c.chunks, h.chunks))) return rc;
    if (!h.rptr.empty() && ((rc = pupload(P, &c.rptr, h.rptr)) || (rc = pupload(P, &c.redge, h.redge)))) return rc;
    c.porig = std::move(h.porig);
    c.hrecs = std::move(h.recs);
  }
  P->lv.assign(S > 1 ? S - 1 : 0, LevelMaps{});
  for (int l = 0; l + 1 < S; ++l) {
    HostLevel& h = H.lv[l];
    LevelMaps& m = P->lv[l];
    m.I = h.I; m.pool_etiles = h.pool_etiles; m.un_ntiles = h.un_ntiles;
    if ((rc = pupload(P, &m.pool_erecs, h.pool_erecs)) || (rc = pupload(P, &m.pool_recs, h.pool_recs)) ||
        (rc = pupload(P, &m.pool_child, h.pool_child)) || (rc = pupload(P, &m.un_recs, h.un_recs)))
      return rc;
    if (!h.pool_slots.empty() && (rc = pupload(P, &m.pool_slots, h.pool_slots))) return rc;
    if (!h.parent_slots.empty() && (rc = pupload(P, &m.parent_slots, h.parent_slots))) return rc;
  }
  return MSW_OK;
}

// Re-launch one kernel of the rollout schedule (first of its kind on `scale`), with its
// rollout side effects removed: no epilogue (the output goes to a scratch buffer), no
// rollout step advance.
int bench_kernel(msw_plan* P, int kernel, int scale, int iters, int64_t* units, hipStream_t st) {
  if (scale < 0 || scale >= P->S) return fail(MSW_ERR_INVALID, "scale out of range");
  if (P->sched_roll.empty()) return fail(MSW_ERR_INVALID, "run a rollout before bench_kernel");
  static const int kind_of[] = {L_HOP, L_EDGE_HOP, L_POOL, L_ENCODE, L_EDGE_HOP};
  if (kernel < 0 || kernel > 4) return fail(MSW_ERR_INVALID, "unknown kernel id");
  const bool unpool = kernel == 4;  // the intra-scale (unpooling) layer into `scale`
  const Launch* src = nullptr;
  for (const Launch& L : P->sched_roll)
    if ((L.kind == kind_of[kernel] || (kernel == 1 && L.kind == L_EDGE_MLP)) &&
        (L.kind == L_ENCODE || L.scale == scale) &&
        (L.kind != L_EDGE_HOP || (L.eh.own_zero != 0) == unpool)) {
      if (!src) src = &L;
      if (L.kind == L_HOP && !L.hop.last) { src = &L; break; }  // prefer a middle hop
      if (L.kind != L_HOP) break;
    }
  if (!src) return fail(MSW_ERR_INVALID, "no such kernel on that scale");
  Launch L = *src;
  const ScaleCSR& g = P->sc[scale];
  int64_t rows = g.ns, edges = g.E;
  if (L.kind == L_HOP && L.hop.last) { L.hop.last = 0; L.hop.out = P->T[1]; }
  if (L.kind == L_EDGE_HOP && L.eh.last && !unpool) { L.eh.last = 0; L.eh.out = P->T[1]; }
  if (L.kind == L_EDGE_HOP || L.kind == L_EDGE_MLP) L.eh.step_inc = nullptr;  // the rollout's step counter stays put
  if (unpool) edges = P->lv[scale].I;  // the unpool epilogue only writes the next layer's U/V/O
  if (L.kind == L_POOL) edges = P->lv[scale - 1].I;
  if (L.kind == L_ENCODE) { L.enc.io = nullptr; L.enc.dec.on = 0; rows = P->N; edges = 0; }
  std::vector<Launch> q(1, L);
  for (int it = 0; it < iters; ++it) {
    int rc = schedule_dispatch(P, q, st);
    if (rc) return rc;
  }
  P->kernels_per_step = (int)P->sched_roll.size();
  if (units) { units[0] = rows; units[1] = edges; }
  return MSW_OK;
}

}  // namespace

int msw::set_error(int code, const char* msg) { return fail(code, msg ? msg : ""); }

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
  if (!strcmp(name, "msw_exchange_desc")) return sizeof(msw_exchange_desc);
  if (!strcmp(name, "msw_swegnn_train_desc")) return sizeof(msw_swegnn_train_desc);
  if (!strcmp(name, "msw_swegnn_grads")) return sizeof(msw_swegnn_grads);
  if (!strcmp(name, "msw_mlp_train_desc")) return sizeof(msw_mlp_train_desc);
  if (!strcmp(name, "msw_mlp_grads")) return sizeof(msw_mlp_grads);
  return -1;
}

int msw_abi_version(void) { return MSW_ABI_VERSION; }

}  // extern "C"

namespace {

// Partitioned mesh: per-scale receive / send row lists (local graph rows -> internal rows).
int build_exchange(msw_plan* P, const msw_exchange_desc* d) {
  // the lists (graph_build.h build_host_exchange, validated against the plan's numbering)
  HostGraph H;  // the numbering only
  H.N = P->N;
  H.iperm = P->iperm;
  H.sc.resize(P->S);
  for (int s = 0; s < P->S; ++s) { H.sc[s].n0 = P->sc[s].n0; H.sc[s].ns = P->sc[s].ns; }
  std::vector<HostXchScale> X;
  std::string err;
  int rc = build_host_exchange(H, P->part_rank, d, X, err);
  if (rc) return fail(rc, err);
  P->xch.assign(P->S, msw_plan::XchScale{});
  size_t most = 1;
  for (int s = 0; s < P->S; ++s) {
    msw_plan::XchScale& Y = P->xch[s];
    Y.nrecv = (int)X[s].recv_rows.size();
    Y.nsend = (int)X[s].send_rows.size();
    for (const XchPeer& pe : X[s].peers) Y.peers.push_back(msw_plan::XchPeer{pe.peer, pe.roff, pe.rcount, pe.soff, pe.scount});
    if ((rc = pupload(P, &Y.recv_rows, X[s].recv_rows)) || (rc = pupload(P, &Y.send_rows, X[s].send_rows))) return rc;
    most = std::max(most, (size_t)std::max(Y.nrecv, Y.nsend));
  }
  const size_t floats = most * 2 * P->F;  // widest exchanged row: U (2F)
  if ((rc = palloc(P, &P->xsend, floats)) || (rc = palloc(P, &P->xrecv, floats))) return rc;
  return MSW_OK;
}

int plan_create_impl(const msw_graph_desc* g, const msw_model_desc* m, int device,
                     const msw_exchange_desc* xch, int rank, msw_plan** out_plan) {
  if (!g || !m || !out_plan) return fail(MSW_ERR_INVALID, "null argument");
  *out_plan = nullptr;
  if (m->model_type != 0 && m->model_type != 1) return fail(MSW_ERR_INVALID, "model_type must be 0 (MSGNN) or 1 (GNN)");
  if (m->hid_features != 16 && m->hid_features != 32 && m->hid_features != 64)
    return fail(MSW_ERR_UNSUPPORTED, "hid_features must be 16, 32 or 64");
  if (m->learned_pooling) return fail(MSW_ERR_UNSUPPORTED, "learned_pooling=True is not implemented");
  HIP_TRY(hipSetDevice(device));
  std::unique_ptr<msw_plan> P(new msw_plan());
  static std::atomic<uint64_t> next_uid{1};
  P->uid = next_uid++;
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

  P->kn = knobs_from_env();
  if (P->kn.epi_split_tiles >= 0) P->epi_split_tiles = P->kn.epi_split_tiles;
  P->xcd_max = std::max(0, P->kn.xcd_max);
  // F = 64: four-wave cooperative kernels on every scale whose grid stays resident
  // (zenodo4_f64 +3.3 %, profiles/r02_v1/ab_coop_f64.txt); F = 32 keeps 1024 (no gain above)
  if (P->NT == 4) P->coop_waves = 4096;
  if (P->kn.coop_waves >= 0) P->coop_waves = P->kn.coop_waves;
  P->part_rank = xch ? rank : -1;
  int rc = build_graph_plan(P.get(), g);
  if (rc) return rc;
  if (xch && (rc = build_exchange(P.get(), xch))) return rc;
  const int F = P->F, Npad = P->Npad;

  // ---- weights
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
  if ((rc = pack_mlp(P->blob, m->static_encoder, P->stat))) return rc;
  if ((rc = pack_mlp(P->blob, m->dynamic_encoder, P->dynm))) return rc;
  if ((rc = pack_mlp(P->blob, m->decoder, P->dec))) return rc;
  if (m->static_encoder.layer[0].in_features != P->nstat_raw + P->with_wl)
    return fail(MSW_ERR_INVALID, "static encoder input width");
  if (m->dynamic_encoder.layer[0].in_features != P->dyn) return fail(MSW_ERR_INVALID, "dynamic encoder input width");
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
    P->procs[j].par = j & 1;
  }
  P->unpools.resize(P->model_type == 0 ? m->num_unpool : 0);
  for (size_t i = 0; i < P->unpools.size(); ++i) {
    if (m->unpool[i].edge_features != 0) return fail(MSW_ERR_INVALID, "intra-scale layer with edge features");
    if (m->unpool[i].K != 1) return fail(MSW_ERR_UNSUPPORTED, "intra-scale layer with K != 1");
    if (m->unpool[i].with_gradient) return fail(MSW_ERR_UNSUPPORTED, "intra-scale layer with gradient");
    if ((rc = build_proc(P.get(), m->unpool[i], P->S - 2 - (int)i, true, P->unpools[i]))) return rc;
  }
  P->prelu = all_prelu(m->static_encoder) & all_prelu(m->dynamic_encoder) & all_prelu(m->decoder);

  // ---- device buffers
  if ((rc = pupload(P.get(), &P->perm_d, P->perm))) return rc;
  if ((rc = pupload(P.get(), &P->zrow_d, std::vector<float>(kZeroRow, 0.f)))) return rc;
  std::vector<int> minus1(Npad, -1);
  if ((rc = pupload(P.get(), &P->bc_slot_d, minus1))) return rc;
  if ((rc = palloc(P.get(), &P->io_d, 1))) return rc;
  HIP_TRY(hipMemset(P->io_d, 0, sizeof(RolloutIO)));
  int Emax = 1;  // tile-padded edge slots of the largest scale
  for (auto& c : P->sc) Emax = std::max(Emax, c.ntiles * kRowsPerWave);
  const size_t NF = (size_t)Npad * F;
  const size_t NH = (size_t)Npad * 16 * P->h1t_max;
  float** bufs[] = {&P->xs, &P->xd0, &P->O[0], &P->O[1], &P->T[0], &P->T[1], &P->xdown, &P->xup, &P->xgnn};
  for (float** b : bufs) {
    if ((rc = palloc(P.get(), b, NF))) return rc;
    HIP_TRY(hipMemset(*b, 0, NF * sizeof(float)));
  }
  float** hbufs[] = {&P->U[0], &P->V[0], &P->U[1], &P->V[1], &P->Uu, &P->Vu};
  for (float** b : hbufs) {
    if ((rc = palloc(P.get(), b, NH))) return rc;
    HIP_TRY(hipMemset(*b, 0, NH * sizeof(float)));
  }
  if ((rc = palloc(P.get(), &P->s, (size_t)Emax * F))) return rc;
  if ((rc = palloc(P.get(), &P->X, (size_t)Npad * P->nnf))) return rc;
  HIP_TRY(hipMemset(P->X, 0, (size_t)Npad * P->nnf * sizeof(float)));
  if (P->E > 0)
    for (Proc& pr : P->procs)
      if ((rc = palloc(P.get(), &pr.Pe, (size_t)std::max(P->sc[pr.scale].ntiles * kRowsPerWave, 1) * 16 * pr.h1t)))
        return rc;

  // ---- launch schedules (forward / rollout), per-launch weight regions, weight upload
  switch (P->NT) {
    case 1: HIP_TRY(prepare_kernels<1>()); break;
    case 2: HIP_TRY(prepare_kernels<2>()); break;
    default: HIP_TRY(prepare_kernels<4>()); break;
  }
  const size_t blob0 = P->blob.h.size();
  for (;;) {
    sched_step(P.get(), P->sched_fwd, false);
    sched_step(P.get(), P->sched_roll, true);
    const bool mlp_only = P->NT > 2;  // F = 64: only the edge-MLP operands fit in LDS
    if ((rc = relocate(P.get(), P->sched_fwd, mlp_only)) || (rc = relocate(P.get(), P->sched_roll, mlp_only)))
      return rc;
    for (auto* q : {&P->sched_fwd, &P->sched_roll})
      for (Launch& L : *q) set_grid_cap(P.get(), L);
    // every cooperative edge hop's staged region must fit the LDS its kernel was given; a
    // fused (un)pooling launch that does not (e.g. F = 32 with mlp_layers = 4: two edge MLPs
    // + the projection) falls back to the separate pooling / unpooling launches
    const Launch* bad = lds_overflow(P.get());
    if (!bad) break;
    if (P->no_fuse || !(bad->eh.pool.slots || bad->eh.pool.parent))
      return fail(MSW_ERR_UNSUPPORTED, "weights of a cooperative edge hop exceed its LDS budget (" +
                                           std::to_string(eh_lds_bytes(bad->eh.reg_nf)) + " B)");
    P->no_fuse = 1;
    P->blob.h.resize(blob0);  // drop the regions of the fused schedule
  }
  P->blob.alloc(256);  // slack: LDS-DMA chunks may read up to 255 floats past a region
  if ((rc = pupload(P.get(), &P->dW, P->blob.h))) return rc;
  for (auto* q : {&P->sched_fwd, &P->sched_roll})
    for (Launch& L : *q) L.common().W = P->dW;

  // ---- static per-edge features: edge encoder + edge part of each processor's layer 1
  if (P->E > 0) {
    // tile-padded edge slots, scale by scale (ScaleCSR::porig); padding slots get zeros
    std::vector<int64_t> sbase(P->S + 1, 0);
    for (int s = 0; s < P->S; ++s) sbase[s + 1] = sbase[s] + (int64_t)P->sc[s].ntiles * kRowsPerWave;
    const int64_t E = sbase[P->S];
    std::vector<float> ea((size_t)std::max<int64_t>(E, 1) * ef_raw, 0.f);
    for (int s = 0; s < P->S; ++s)
      for (size_t q = 0; q < P->sc[s].porig.size(); ++q)
        if (P->sc[s].porig[q] >= 0)
          for (int f = 0; f < ef_raw; ++f)
            ea[(size_t)(sbase[s] + q) * ef_raw + f] = g->edge_attr[(size_t)P->sc[s].porig[q] * ef_raw + f];
    float* ea_d = nullptr;
    float* enc_d = nullptr;
    if ((rc = pupload(P.get(), &ea_d, ea))) return rc;
    const float* feat = ea_d;
    int feat_stride = ef_raw, feat_dim = ef_raw;
    if (m->edge_mlp) {
      if ((rc = palloc(P.get(), &enc_d, (size_t)E * F))) return rc;
      RowMlpArgs ra{};
      ra.mode = 0;
      ra.in = ea_d; ra.in_stride = ef_raw; ra.in_dim = ef_raw; ra.R = (int)E; ra.m = P->edge_enc;
      ra.W = P->dW; ra.out = enc_d; ra.out_stride = F; ra.out_tiles = P->NT;
      P->edge_jobs.push_back(ra);
      feat = enc_d; feat_stride = F; feat_dim = F;
    }
    for (size_t j = 0; j < P->procs.size(); ++j) {
      Proc& pr = P->procs[j];
      const msw_linear& L1 = m->processors[j].edge_mlp.layer[0];
      const int H1 = L1.out_features;
      Blob tb;  // Pe = W1[:, 4F:4F+ef] . feat + b1: one NT -> 2NT layer (zero padded)
      MlpDev md{};
      md.n = 1;
      md.l[0].tin = P->NT;
      md.l[0].tout = 2 * P->NT;
      md.l[0].a_off = pack_operand(tb, L1.weight, L1.in_features, 2 * P->NT, P->NT,
                                   [&](int k) { return k < feat_dim ? 4 * F + k : -1; },
                                   [&](int o) { return o < H1 ? o : -1; });
      md.l[0].b_off = pack_bias(tb, L1.bias, H1, 2 * P->NT);
      md.l[0].act = 0;
      float* tw = nullptr;
      if ((rc = pupload(P.get(), &tw, tb.h))) return rc;
      const ScaleCSR& c = P->sc[pr.scale];
      RowMlpArgs ra{};
      ra.mode = 1;
      ra.in = feat + (size_t)sbase[pr.scale] * feat_stride; ra.in_stride = feat_stride;
      ra.in_dim = feat_dim; ra.R = c.ntiles * kRowsPerWave; ra.m = md; ra.W = tw;
      ra.out = pr.Pe; ra.out_stride = 16 * pr.h1t; ra.out_tiles = pr.h1t;
      P->edge_jobs.push_back(ra);
    }
    for (const RowMlpArgs& ra : P->edge_jobs) HIP_TRY(rowmlp_dispatch(P->NT, ra));
  }
  HIP_TRY(hipDeviceSynchronize());
  if (xch) P->use_graph = 0;  // partitioned plans: the RCCL exchanges run eagerly
  *out_plan = P.release();
  return MSW_OK;
}

// BC slots (internal rows), the device I/O record and the initial state of a rollout, set
// by kernels whose arguments carry the values: no host buffer lifetime issue, no host sync.
int rollout_prologue(msw_plan* P, const float* x0, const float* bc, int32_t bc_tstride,
                     const int32_t* node_bc, int32_t n_bc, int32_t type_bc, int32_t T, float* out,
                     hipStream_t st) {
  if (!P || !x0 || !out) return fail(MSW_ERR_INVALID, "null argument");
  if (n_bc > 0 && (!bc || !node_bc)) return fail(MSW_ERR_INVALID, "BC arrays missing");
  if (n_bc > 0 && bc_tstride < T) return fail(MSW_ERR_INVALID, "BC has fewer time entries than T");
  if (type_bc != 1 && type_bc != 2) return fail(MSW_ERR_INVALID, "type_BC must be 1 or 2 (dataset.py:499-506)");
  HIP_TRY(hipSetDevice(P->device));
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
  for (const RowMlpArgs& ra : P->edge_jobs) HIP_TRY(rowmlp_dispatch(P->NT, ra, st));
  RolloutIO io{};
  io.bc = bc; io.out = out; io.bc_tstride = bc_tstride; io.type_bc = type_bc; io.T = T; io.step = -1;
  HIP_TRY(launch_set_io(P->io_d, io, st));
  InitArgs ia{};
  ia.x0 = x0; ia.perm = P->perm_d; ia.N = P->Npad; ia.nnf = P->nnf;
  ia.dyn = P->dyn; ia.p = P->p; ia.X = P->X; ia.io = P->io_d; ia.bc_slot = P->bc_slot_d;
  HIP_TRY(launch_init_state(ia, st));
  return MSW_OK;
}

// Capture what `enqueue(stream)` launches on the plan's capture stream into `*exec`.
template <class Fn>
int capture_graph(msw_plan* P, hipGraphExec_t* exec, Fn enqueue) {
  if (!P->cap_stream) HIP_TRY(hipStreamCreateWithFlags(&P->cap_stream, hipStreamNonBlocking));
  hipGraph_t graph = nullptr;
  HIP_TRY(hipStreamBeginCapture(P->cap_stream, hipStreamCaptureModeThreadLocal));
  const int rc = enqueue(P->cap_stream);
  const hipError_t ce = hipStreamEndCapture(P->cap_stream, &graph);
  if (rc) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  if (ce != hipSuccess) return fail(MSW_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
  const hipError_t ie = hipGraphInstantiate(exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ie != hipSuccess) {
    *exec = nullptr;
    return fail(MSW_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
  }
  return MSW_OK;
}

// In-process transport (msw_group_rollout): halo rows of plan k's buffer gathered straight
// from the owning plans' buffers, using each owner's send list for k.
int loopback_exchange(msw_plan* const* plans, int k, const ExchangeArgs& a, hipStream_t st) {
  msw_plan* P = plans[k];
  const msw_plan::XchScale& X = P->xch[a.scale];
  for (const auto& pe : X.peers) {
    if (pe.rcount == 0) continue;
    msw_plan* Q = plans[pe.peer];
    const msw_plan::XchScale& Y = Q->xch[a.scale];
    const msw_plan::XchPeer* back = nullptr;
    for (const auto& qe : Y.peers)
      if (qe.peer == k) back = &qe;
    if (!back || back->scount != pe.rcount)
      return fail(MSW_ERR_INVALID, "exchange lists of plans " + std::to_string(k) + " and " +
                                       std::to_string(pe.peer) + " disagree");
    for (int b = 0; b < a.nbuf; ++b) {
      if (Q == P) {  // self entry: staged, as the RCCL transport does (the row sets may overlap)
        HIP_TRY(launch_copy_rows(buf_of(P, a.buf[b]), Y.send_rows + back->soff, P->xsend, nullptr, pe.rcount,
                                 a.width[b], st));
        HIP_TRY(launch_copy_rows(P->xsend, nullptr, buf_of(P, a.buf[b]), X.recv_rows + pe.roff, pe.rcount,
                                 a.width[b], st));
      } else {
        HIP_TRY(launch_copy_rows(buf_of(Q, a.buf[b]), Y.send_rows + back->soff, buf_of(P, a.buf[b]),
                                 X.recv_rows + pe.roff, pe.rcount, a.width[b], st));
      }
    }
  }
  return MSW_OK;
}

template <int NT>
int group_step(msw_plan* const* plans, int n, hipStream_t st) {
  const size_t L = plans[0]->sched_roll.size();
  for (size_t i = 0; i < L; ++i)
    for (int k = 0; k < n; ++k) {
      const Launch& l = plans[k]->sched_roll[i];
      if (l.kind == L_EXCHANGE) {
        int rc = loopback_exchange(plans, k, l.xch, st);
        if (rc) return rc;
      } else {
        HIP_TRY(launch_one<NT>(l, st));
      }
    }
  return MSW_OK;
}

}  // namespace

extern "C" {

int msw_plan_create(const msw_graph_desc* g, const msw_model_desc* m, int device, msw_plan** out_plan) {
  return plan_create_impl(g, m, device, nullptr, -1, out_plan);
}

int msw_plan_create_part(const msw_graph_desc* g, const msw_model_desc* m, int device,
                         const msw_exchange_desc* xch, int32_t rank, msw_plan** out_plan) {
  if (!xch || rank < 0) return fail(MSW_ERR_INVALID, "exchange descriptor missing or rank < 0");
  if (xch->num_entries < 0 || (xch->num_entries > 0 && (!xch->peer || !xch->scale || !xch->recv_ptr ||
                                                         !xch->send_ptr)))
    return fail(MSW_ERR_INVALID, "exchange descriptor arrays missing");
  return plan_create_impl(g, m, device, xch, rank, out_plan);
}

int msw_comm_unique_id(char* uid128) {
  if (!uid128) return fail(MSW_ERR_INVALID, "null argument");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  if (!rccl().ok) return fail(MSW_ERR_UNSUPPORTED, "RCCL not found in the process nor as librccl.so.1");
  ncclUniqueId id;
  const ncclResult_t e = rccl().getUniqueId(&id);
  if (e != ncclSuccess) return fail(MSW_ERR_HIP, std::string("ncclGetUniqueId: ") + rccl().errStr(e));
  memcpy(uid128, &id, sizeof(id));
  return MSW_OK;
}

int msw_plan_set_comm(msw_plan* P, const char* uid128, int32_t nranks, int32_t rank) {
  if (!P || !uid128) return fail(MSW_ERR_INVALID, "null argument");
  if (P->part_rank < 0) return fail(MSW_ERR_INVALID, "plan is not partitioned (msw_plan_create_part)");
  if (rank != P->part_rank || nranks <= rank) return fail(MSW_ERR_INVALID, "rank does not match the plan's part");
  if (!rccl().ok) return fail(MSW_ERR_UNSUPPORTED, "RCCL not found in the process nor as librccl.so.1");
  HIP_TRY(hipSetDevice(P->device));
  if (P->comm) {
    (void)rccl().commDestroy(P->comm);
    P->comm = nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, uid128, sizeof(id));
  const ncclResult_t e = rccl().commInitRank(&P->comm, nranks, id, rank);
  if (e != ncclSuccess) {
    P->comm = nullptr;
    return fail(MSW_ERR_HIP, std::string("ncclCommInitRank: ") + rccl().errStr(e));
  }
  return MSW_OK;
}

int msw_group_rollout(msw_plan* const* plans, int32_t num_plans, const float* const* x0,
                      const float* const* bc, const int32_t* bc_tstride, const int32_t* const* node_bc,
                      const int32_t* n_bc, int32_t type_bc, int32_t T, float* const* out, void* stream) {
  if (!plans || num_plans <= 0 || !x0 || !bc || !bc_tstride || !node_bc || !n_bc || !out)
    return fail(MSW_ERR_INVALID, "null argument");
  if (T < 0) return fail(MSW_ERR_INVALID, "T < 0");
  const msw_plan* P0 = plans[0];
  for (int k = 0; k < num_plans; ++k) {
    const msw_plan* P = plans[k];
    if (!P) return fail(MSW_ERR_INVALID, "null plan");
    if (P->part_rank != k) return fail(MSW_ERR_INVALID, "plans[k] must be the plan of part k");
    if (P->device != P0->device || P->NT != P0->NT) return fail(MSW_ERR_INVALID, "plans on different devices / widths");
    if (P->sched_roll.size() != P0->sched_roll.size())
      return fail(MSW_ERR_INVALID, "plans with different step schedules");
    for (size_t i = 0; i < P->sched_roll.size(); ++i)
      if (P->sched_roll[i].kind != P0->sched_roll[i].kind)
        return fail(MSW_ERR_INVALID, "plans with different step schedules");
    for (const auto& X : P->xch)
      for (const auto& pe : X.peers)
        if (pe.peer >= num_plans) return fail(MSW_ERR_INVALID, "exchange peer outside the group");
  }
  if (T == 0) return MSW_OK;
  hipStream_t st = (hipStream_t)stream;
  for (int k = 0; k < num_plans; ++k) {
    int rc = rollout_prologue(plans[k], x0[k], bc[k], bc_tstride[k], node_bc[k], n_bc[k], type_bc, T, out[k], st);
    if (rc) return rc;
  }
  auto step = [&](hipStream_t s) {
    return P0->NT == 1 ? group_step<1>(plans, num_plans, s)
         : P0->NT == 2 ? group_step<2>(plans, num_plans, s)
                       : group_step<4>(plans, num_plans, s);
  };
  msw_plan* G0 = plans[0];
  if (G0->group_graph) {
    // every part's launches and the halo copies of `steps` consecutive steps in one graph,
    // replayed as msw_rollout replays its own (the parts' device-side I/O records were written
    // by their prologues; the kernels read the step counters from them)
    std::vector<uint64_t> key;
    for (int k = 0; k < num_plans; ++k) {
      key.push_back(plans[k]->uid);
      key.push_back((uint64_t)plans[k]->graph_gen);
    }
    if (key != G0->group_key) {
      G0->drop_group_graphs();
      G0->group_key = key;
    }
    auto capture = [&](hipGraphExec_t* exec, int steps) -> int {
      return capture_graph(G0, exec, [&](hipStream_t cs) {
        int rc = MSW_OK;
        for (int k = 0; k < steps && !rc; ++k) rc = step(cs);
        return rc;
      });
    };
    const int G = std::max(1, G0->graph_steps);
    int rc;
    if (G > 1 && T >= G && !G0->group_multi && (rc = capture(&G0->group_multi, G))) return rc;
    if ((G == 1 || T % G) && !G0->group_one && (rc = capture(&G0->group_one, 1))) return rc;
    int t = 0;
    if (G > 1)
      for (; t + G <= T; t += G) HIP_TRY(hipGraphLaunch(G0->group_multi, st));
    for (; t < T; ++t) HIP_TRY(hipGraphLaunch(G0->group_one, st));
  } else {
    for (int t = 0; t < T; ++t)
      if (int rc = step(st)) return rc;
  }
  for (int k = 0; k < num_plans; ++k)
    if (int rc = final_decode(plans[k], st)) return rc;
  for (int k = 0; k < num_plans; ++k) {
    plans[k]->rollout_steps += T;
    plans[k]->forward_calls += T;
  }
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
  if (P->use_graph) {
    // the schedule reads fwd_x and writes fwd_y (graph numbering, like x and y)
    const size_t xb = (size_t)P->N * P->nnf * sizeof(float), yb = (size_t)P->N * 2 * sizeof(float);
    if (!P->fwd_exec) {
      if (!P->fwd_x) {
        int rc = palloc(P, &P->fwd_x, (size_t)P->N * P->nnf);
        if (!rc) rc = palloc(P, &P->fwd_y, (size_t)P->N * 2);
        if (rc) return rc;
      }
      patch_forward(P->sched_fwd, P->fwd_x, P->fwd_y);
      int rc = capture_graph(P, &P->fwd_exec, [&](hipStream_t cs) { return schedule_dispatch(P, P->sched_fwd, cs); });
      if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(P->fwd_x, x, xb, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipGraphLaunch(P->fwd_exec, st));
    HIP_TRY(hipMemcpyAsync(y, P->fwd_y, yb, hipMemcpyDeviceToDevice, st));
  } else {
    patch_forward(P->sched_fwd, x, y);
    int rc = schedule_dispatch(P, P->sched_fwd, st);
    if (rc) return rc;
  }
  P->forward_calls++;
  return MSW_OK;
}

int msw_set_graph_capture(msw_plan* P, int enable) {
  if (!P) return fail(MSW_ERR_INVALID, "null plan");
  P->use_graph = enable ? 1 : 0;  // the plan's own rollout / forward graphs only
  return MSW_OK;
}

int msw_set_group_graph(msw_plan* P, int enable) {
  if (!P) return fail(MSW_ERR_INVALID, "null plan");
  P->group_graph = enable ? 1 : 0;
  P->drop_group_graphs();
  return MSW_OK;
}

int msw_rollout(msw_plan* P, const float* x0, const float* bc, int32_t bc_tstride,
                const int32_t* node_bc, int32_t n_bc, int32_t type_bc, int32_t T, float* out,
                void* stream) {
  if (!P || !x0 || (!out && T > 0)) return fail(MSW_ERR_INVALID, "null argument");
  if (T < 0) return fail(MSW_ERR_INVALID, "T < 0");
  if (T == 0) return MSW_OK;
  hipStream_t st = (hipStream_t)stream;
  int prc = rollout_prologue(P, x0, bc, bc_tstride, node_bc, n_bc, type_bc, T, out, st);
  if (prc) return prc;
  if (P->use_graph) {
    // capture `steps` consecutive rollout steps into one executable graph
    auto capture = [&](hipGraphExec_t* exec, int steps) -> int {
      return capture_graph(P, exec, [&](hipStream_t cs) {
        int rc = MSW_OK;
        for (int k = 0; k < steps && !rc; ++k) rc = schedule_dispatch(P, P->sched_roll, cs);
        return rc;
      });
    };
    const int G = std::max(1, P->graph_steps);
    int rc;
    if (G > 1 && T >= G && !P->multi_exec && (rc = capture(&P->multi_exec, G))) return rc;
    if ((G == 1 || T % G) && !P->step_exec && (rc = capture(&P->step_exec, 1))) return rc;
    int t = 0;
    if (G > 1)
      for (; t + G <= T; t += G) HIP_TRY(hipGraphLaunch(P->multi_exec, st));
    for (; t < T; ++t) HIP_TRY(hipGraphLaunch(P->step_exec, st));
  } else {
    for (int t = 0; t < T; ++t) {
      int rc = schedule_dispatch(P, P->sched_roll, st);
      if (rc) return rc;
    }
  }
  if (int rc = final_decode(P, st)) return rc;
  P->rollout_steps += T;
  P->forward_calls += T;
  if (P->comm)
    for (const auto& X : P->xch)
      if (!X.peers.empty()) {
        P->rccl_steps += T;
        break;
      }
  return MSW_OK;
}

int msw_bench_kernel(msw_plan* P, int32_t kernel, int32_t scale, int32_t iters, int64_t* units,
                     void* stream) {
  if (!P || iters < 0) return fail(MSW_ERR_INVALID, "bad argument");
  HIP_TRY(hipSetDevice(P->device));
  hipStream_t st = (hipStream_t)stream;
  return bench_kernel(P, kernel, scale, iters, units, st);
}

int msw_debug_buffer(msw_plan* P, const char* name, float* dst, void* stream) {
  if (!P || !name || !dst) return fail(MSW_ERR_INVALID, "null argument");
  const float* src = nullptr;
  if (!strcmp(name, "x_s")) src = P->xs;
  else if (!strcmp(name, "x_d")) src = P->xd0;
  else if (!strcmp(name, "x_down")) src = P->model_type == 0 ? P->xdown : nullptr;
  else if (!strcmp(name, "x_up")) src = P->model_type == 0 ? P->xup : nullptr;
  if (!src) return fail(MSW_ERR_INVALID, std::string("unknown buffer ") + name);
  // debug only: synchronous host round trip into graph numbering
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  std::vector<float> h((size_t)P->Npad * P->F), o((size_t)P->N * P->F);
  HIP_TRY(hipMemcpy(h.data(), src, h.size() * sizeof(float), hipMemcpyDeviceToHost));
  for (int i = 0; i < P->Npad; ++i)
    if (P->perm[i] >= 0)
      std::copy(h.begin() + (size_t)i * P->F, h.begin() + (size_t)(i + 1) * P->F, o.begin() + (size_t)P->perm[i] * P->F);
  HIP_TRY(hipMemcpy(dst, o.data(), o.size() * sizeof(float), hipMemcpyHostToDevice));
  return MSW_OK;
}

int msw_set_trace(msw_plan* P, uint64_t* buf) {
  if (!P) return fail(MSW_ERR_INVALID, "null plan");
  // MSW_TRACE_ENCODE: the encoder launches only (a rollout then leaves the marks of its last
  // step's encoder: the deferred decoder + encoders, tools/trace_kernels.py)
  const bool enc_only = P->kn.trace_encode != 0;
  for (auto* q : {&P->sched_fwd, &P->sched_roll})
    for (Launch& L : *q)
      L.common().trace = (!enc_only || L.kind == L_ENCODE) ? reinterpret_cast<unsigned long long*>(buf) : nullptr;
  P->drop_graphs();  // the captured steps hold the old arguments
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
  s->graph_captured = P->step_exec != nullptr || P->multi_exec != nullptr || P->fwd_exec != nullptr;
  s->rccl_calls = P->rccl_calls;
  s->rccl_steps = P->rccl_steps;
  return MSW_OK;
}

}  // extern "C"
