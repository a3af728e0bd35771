/*
 * mswegnn.h -- C ABI of the MI355X (gfx950) multi-scale SWE-GNN rollout engine.
 *
 * Drop-in boundary for the hot path of sdat2/mSWE-GNN.  The reference
 * has no FFI/plugin layer: its hot path sits behind the Python nn.Module API
 *   MSGNN.forward(graph)   models/gnn.py:267-350
 *   GNN.forward(graph)     models/gnn.py:102-152   (type_GNN='SWEGNN')
 *   rollout_test(model,b)  training/train.py:67-95
 * and the package's Python host side (mswe-gnn_amd/models/gnn.py, training/train.py)
 * binds the entry points below through ctypes (mswe-gnn_amd/mswegnn/_lib.py); the binding
 * a maintainer would add on the reference side is shown in INTEGRATION.md.
 *
 * Conventions
 *   - plain C types, no torch types; all float data is fp32, row-major.
 *   - host pointers are read only during msw_plan_create (graph + weights are copied to
 *     device memory the plan owns); device pointers passed to msw_forward / msw_rollout
 *     are owned by the caller and must stay valid until the stream has executed the work.
 *   - every function returns MSW_OK (0) or a negative MSW_ERR_* code and never aborts;
 *     msw_last_error() returns a thread-local message for the last failure.
 *   - a plan is bound to one device and is not re-entrant: one stream at a time.
 *   - msw_forward / msw_rollout enqueue asynchronously on `stream` (a hipStream_t, NULL =
 *     default stream) and never synchronise the host.
 */
#ifndef MSWEGNN_H
#define MSWEGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSW_ABI_VERSION 1

#define MSW_OK 0
#define MSW_ERR_INVALID (-1)     /* bad argument / inconsistent graph or model description */
#define MSW_ERR_HIP (-2)         /* HIP runtime error (allocation, launch, ...)           */
#define MSW_ERR_UNSUPPORTED (-3) /* configuration outside what the engine implements      */

/* Activation codes: activation_functions(), models/models.py:149-169. */
enum msw_activation {
  MSW_ACT_NONE = 0,
  MSW_ACT_PRELU = 1, /* single learned slope (nn.PReLU() default num_parameters=1) */
  MSW_ACT_RELU = 2,
  MSW_ACT_LEAKYRELU = 3, /* slope 0.1 */
  MSW_ACT_ELU = 4,
  MSW_ACT_SWISH = 5, /* SiLU */
  MSW_ACT_SIGMOID = 6,
  MSW_ACT_TANH = 7
};

/* One nn.Linear followed by its activation (make_mlp, models/models.py:121-146:
 * the activation follows EVERY layer, including the last). */
typedef struct {
  int32_t in_features;
  int32_t out_features;
  const float* weight; /* host [out_features][in_features] */
  const float* bias;   /* host [out_features] or NULL (bias=False) */
  int32_t act;         /* enum msw_activation */
  float act_param;     /* PReLU slope */
} msw_linear;

#define MSW_MAX_MLP_LAYERS 4
typedef struct {
  int32_t n_layers;
  msw_linear layer[MSW_MAX_MLP_LAYERS];
} msw_mlp;

/* One SWEGNN layer (models/gnn.py:352-445). */
typedef struct {
  int32_t K;                  /* hops */
  int32_t normalize;          /* s_ij / ||s_ij||, NaN -> 0  (gnn.py:424-426) */
  int32_t with_filter_matrix; /* filter_matrix[0..K] (gnn.py:381-384) */
  int32_t with_gradient;      /* (out[col]-out[row]) * s  vs  s * out[row] (gnn.py:429-435) */
  int32_t upwind_mode;        /* clamp negative gradients (gnn.py:431-432) */
  int32_t edge_features;      /* width of edge_attr fed to this layer; 0 for intra_scale_gnn */
  msw_mlp edge_mlp;           /* input 4F + edge_features -> 2F -> ... -> F */
  const float* const* filter; /* K+1 host pointers to [F][F] (bias-free) or NULL */
} msw_swegnn;

/* Model description.  model_type 0 = MSGNN (models/gnn.py:154-350),
 * 1 = GNN with type_GNN='SWEGNN' (models/gnn.py:13-152). */
typedef struct {
  int32_t model_type;
  int32_t hid_features;      /* F: 16, 32 or 64 supported (F=16 runs zero-padded to 32) */
  int32_t num_scales;        /* S (GNN: 1) */
  int32_t previous_t;        /* p */
  int32_t num_node_features; /* static + 2p */
  int32_t with_WL;           /* append DEM + h_t to the static input (gnn.py:288-291) */
  int32_t skip_connections;  /* MSGNN x_down skips (gnn.py:330-331) */
  int32_t learned_pooling;   /* must be 0 (no shipped config uses it) */
  int32_t gnn_act;           /* MSGNN: on x_up (gnn.py:335-336); GNN: after every layer */
  float gnn_act_param;
  /* residual: res_var = sum_tau residual_weights[tau][var] * x[:, dyn + 2 tau + var]
   * (models/models.py:50-77 folded to a [p][2] matrix by the host; NULL = none) */
  const float* residual_weights;
  int32_t edge_mlp;      /* edge encoder present (gnn.py:203-206) */
  msw_mlp edge_encoder;  /* raw edge features -> F */
  msw_mlp static_encoder;
  msw_mlp dynamic_encoder;
  msw_mlp decoder; /* F -> ... -> 2 */
  int32_t num_processors;        /* MSGNN: 2S-1 (down 0..S-2, coarsest, up); GNN: n_GNN_layers */
  const msw_swegnn* processors;
  int32_t num_unpool;            /* MSGNN: S-1 intra_scale_gnn; GNN: 0 */
  const msw_swegnn* unpool;
} msw_model_desc;

/* Graph description in the reference's layout:
 *   - nodes of graph g, scale s: [node_ptr[g*(S+1)+s], node_ptr[g*(S+1)+s+1])
 *     (a single Data: num_graphs=1; a Batch after update_batch_multiscale, train.py:31-65)
 *   - edge_index[0] = row (source j), edge_index[1] = col (target i); scale s edges are
 *     [edge_ptr[s], edge_ptr[s+1]) (scale-major)
 *   - intra_edge_index rows (coarse, fine), level l (coarse scale l+1, fine scale l) is
 *     [intra_edge_ptr[l], intra_edge_ptr[l+1]). */
typedef struct {
  int64_t num_nodes;
  int32_t num_scales;
  int32_t num_graphs;
  const int64_t* node_ptr; /* [num_graphs][num_scales+1] */
  int64_t num_edges;
  const int64_t* edge_index; /* [2][num_edges] */
  const float* edge_attr;    /* [num_edges][num_edge_features] */
  int32_t num_edge_features;
  const int64_t* edge_ptr; /* [num_scales+1] */
  int64_t num_intra_edges;
  const int64_t* intra_edge_index; /* [2][num_intra_edges] */
  const int64_t* intra_edge_ptr;   /* [num_scales] */
} msw_graph_desc;

typedef struct msw_plan msw_plan;

/* Statistics for tests / benchmarks. */
typedef struct {
  int64_t num_nodes;
  int64_t num_edges;
  int32_t num_scales;
  int32_t hid_features;
  int32_t padded_features;
  int32_t kernels_per_step;  /* launches one forward enqueues */
  int64_t forward_calls;     /* forwards executed through the HIP path so far */
  int64_t rollout_steps;     /* rollout steps executed through the HIP path so far */
  int64_t device_bytes;      /* device memory owned by the plan */
  int32_t graph_captured;    /* a hipGraph of one rollout step is instantiated */
  int64_t rccl_calls;        /* ncclSend / ncclRecv calls this plan issued (eagerly, or recorded
                                into a captured rollout graph) */
  int64_t rccl_steps;        /* rollout steps whose halo exchanges ran over RCCL (eager or replayed) */
} msw_plan_stats;

/* Halo exchange of one rank of a single mesh split over several ranks (SURVEY §8 f2,
 * mswegnn/partition.py).  The graph given to msw_plan_create_part is the rank's LOCAL graph
 * (owned nodes + halo nodes, in-edges of owned nodes only).  An entry = one (scale, peer)
 * pair: the rows this rank receives from `peer` (its halo rows of that scale, local graph
 * numbering) and the rows it sends to `peer` (its owned rows the peer holds as halo, in the
 * peer's receive order).  Exchanged before every launch that gathers from other nodes:
 * U and out_0 before a layer's first hop, out_k before each further hop.  An entry whose peer
 * is the rank itself (equal receive and send counts) copies send row k to receive row k through
 * the transport -- RCCL send / recv to self in a one-rank communicator. */
typedef struct msw_exchange_desc {
  int32_t num_entries;
  const int32_t* peer;       /* [num_entries] peer rank */
  const int32_t* scale;      /* [num_entries] scale of the entry */
  const int64_t* recv_ptr;   /* [num_entries + 1] offsets into recv_rows */
  const int32_t* recv_rows;
  const int64_t* send_ptr;   /* [num_entries + 1] offsets into send_rows */
  const int32_t* send_rows;
} msw_exchange_desc;

/* Build CSR-by-destination per scale, pooling/unpooling maps, pack the weights for
 * the gfx950 kernels, allocate workspaces.  Host-synchronous; call once per graph. */
int msw_plan_create(const msw_graph_desc* graph, const msw_model_desc* model, int device,
                    msw_plan** out_plan);
int msw_plan_destroy(msw_plan* plan);

/* msw_plan_create for one rank of a partitioned mesh: `xch` describes its halo exchange
 * (hop pairs are not used: their halo is two rings deep).  The exchange itself runs either
 * over RCCL (msw_plan_set_comm, one process per GPU, inside msw_rollout; launched eagerly:
 * a partitioned plan is created with graph capture off, and msw_set_graph_capture(plan, 1) is
 * the only way to capture the RCCL exchanges too) or between plans of one process
 * (msw_group_rollout, validation on one GPU: the group's steps are captured as hipGraphs held
 * by plans[0] -- msw_set_group_graph(plans[0], 0) steps it eagerly). */
int msw_plan_create_part(const msw_graph_desc* graph, const msw_model_desc* model, int device,
                         const msw_exchange_desc* xch, int32_t rank, msw_plan** out_plan);

/* RCCL transport.  msw_comm_unique_id writes an ncclUniqueId (128 bytes) on the rank that
 * creates it; every rank then calls msw_plan_set_comm with the same bytes.  RCCL is bound
 * at run time from the process (the copy PyTorch loaded) or librccl.so.1. */
int msw_comm_unique_id(char* uid128);
int msw_plan_set_comm(msw_plan* plan, const char* uid128, int32_t nranks, int32_t rank);

/* All ranks' plans of one partitioned mesh in ONE process, stepped in lockstep with the
 * halo exchange done by device copies between the plans (no RCCL): validates the
 * decomposition on a single GPU.  Per-plan arrays: x0, bc, bc_tstride, node_bc, n_bc, out
 * as msw_rollout takes them. */
int msw_group_rollout(msw_plan* const* plans, int32_t num_plans, const float* const* x0,
                      const float* const* bc, const int32_t* bc_tstride,
                      const int32_t* const* node_bc, const int32_t* n_bc, int32_t type_bc,
                      int32_t T, float* const* out, void* stream);

/* One forward (MSGNN.forward / GNN.forward): x [N][num_node_features] -> y [N][2].
 * Does not modify x.  Equivalent to models/gnn.py:267-350 (MSGNN) or :102-152 (GNN).
 * With graph capture on (the default), the first call captures the forward schedule into a
 * hipGraph over plan-owned I/O slots; every call then enqueues copy x -> slot, one graph
 * launch, copy slot -> y (the reference's per-step rollout loop, train.py:87-95, calls this
 * once per step). */
int msw_forward(msw_plan* plan, const float* x, float* y, void* stream);

/* Autoregressive rollout (rollout_test, training/train.py:67-95 with
 * apply_boundary_condition / use_prediction, utils/dataset.py:486-529):
 *   for t in 0..T-1: x[node_bc, dyn + (type_bc-1) + 2 tau] = bc[b][tau][t]
 *                    pred = forward(x); x = shift(x, pred); out[:, :, t] = pred
 * x0 [N][nnf] (device, not modified), bc [n_bc][p][T_bc] device with T_bc >= T,
 * node_bc host int32 [n_bc] (node ids in the graph's numbering), out [N][2][T] device. */
int msw_rollout(msw_plan* plan, const float* x0, const float* bc, int32_t bc_time_stride,
                const int32_t* node_bc, int32_t n_bc, int32_t type_bc, int32_t T, float* out,
                void* stream);

/* Copy an internal per-node buffer ("x_s", "x_d", "x_down", "x_up") of the last forward
 * into dst (device, [N][F], graph numbering).  Debug / parity localisation only. */
int msw_debug_buffer(msw_plan* plan, const char* name, float* dst, void* stream);

/* Enable (1) / disable (0) graph capture of this plan's own rollout steps and msw_forward
 * (default 1, partitioned plans 0; 0 = every launch enqueued eagerly).  With a communicator
 * set, 1 captures the RCCL halo exchanges into the rollout graphs too. */
int msw_set_graph_capture(msw_plan* plan, int enable);
/* msw_group_rollout's own graphs (default 1): only the flag of the group's plans[0] is read,
 * and it is independent of msw_set_graph_capture. */
int msw_set_group_graph(msw_plan* plans0, int enable);

int msw_plan_get_stats(const msw_plan* plan, msw_plan_stats* stats);


/* Re-launch one kernel of the step `iters` times on `stream` (benchmark / roofline hook;
 * call after a forward or rollout: it reuses the plan's workspaces and overwrites scratch).
 *   kernel: 0 = middle hop (first processor on `scale`), 1 = fused edge MLP + hop 1
 *           (same processor), 2 = mean pooling + projection into `scale` (scale >= 1),
 *           3 = node encoders (+ projection of processor 0), 4 = unpooling layer into
 *           `scale` (scale < S-1) with its projection epilogue.
 * units_out (optional) receives {rows, edges} processed by ONE launch. */
int msw_bench_kernel(msw_plan* plan, int32_t kernel, int32_t scale, int32_t iters,
                     int64_t* units_out, void* stream);

/* On-device rollout evaluation (the reference's test-time metrics, finest scale only;
 * utils/miscellaneous.py:116-199, training/loss.py:8-35,120-169).  pred, real: device
 * [N][2][T] (graph numbering, as msw_rollout writes them); fine_ranges: host int64
 * [num_sims][2], the finest-scale row range of each simulation (node_ptr[g][0],
 * node_ptr[g][1]); thresholds: host float [n_thr] (n_thr <= 4) water-depth thresholds;
 * area: device float [N] cell areas by graph row (data.area), or NULL.
 * Outputs (device): sums written (fp64, workgroup partials added in a fixed order -- bit-
 * reproducible; stream-ordered scratch from hipMallocAsync), counts ZEROED by the caller
 * (exact integer atomics):
 *   sums   double [num_sims][T][10]: sum|dh|, sum|dv|, sum dh^2, sum dv^2, the same four
 *          over rows with dh != 0 or dv != 0 (mask_on_water), that row count, and the
 *          stored volume sum(area * h_pred) (0 when area is NULL);
 *   counts uint64 [num_sims][T][n_thr][4]: TP, TN, FP, FN of h_pred > thr vs h_real > thr.
 * Stream-ordered, no host synchronisation; needs no plan. */
int msw_rollout_metrics(const float* pred, const float* real, int32_t T, const int64_t* fine_ranges,
                        int32_t num_sims, const float* thresholds, int32_t n_thr, const float* area,
                        double* sums, uint64_t* counts, void* stream);

/* ---- Training: autograd through one SWEGNN processor ------------------------
 * Replaces the autograd of SWEGNN.forward (models/gnn.py:387-445) the reference trains through
 * in training_step (training/train.py:125-145).  Stateless: every buffer is device memory the
 * caller owns (mswegnn/autograd.py allocates them as torch tensors).  Parameters are the
 * layer's own tensors: edge_mlp Linear weights [width[l+1]][width[l]] / biases, single-slope
 * PReLU parameters, filter_matrix[k].weight [F][F]. */
#define MSW_MAX_HOPS 8
typedef struct {
  int64_t num_nodes, num_edges;
  int32_t F;             /* dynamic_node_features = static = edge_output_size */
  int32_t edge_features; /* width of edge_attr (0 for intra_scale_gnn) */
  int32_t K;             /* hops, 1..MSW_MAX_HOPS */
  int32_t n_layers;      /* edge MLP depth, 1..MSW_MAX_MLP_LAYERS */
  int32_t width[MSW_MAX_MLP_LAYERS + 1]; /* width[0] = 4F + edge_features, width[n_layers] = F */
  int32_t act[MSW_MAX_MLP_LAYERS];       /* enum msw_activation after each layer */
  int32_t normalize, with_filter_matrix, with_gradient, upwind_mode;
  /* graph, device int32: row / col = edge_index[0] / [1]; CSR by destination (col) and by
   * source (row), edges of a node in reference (edge_index) order */
  const int32_t *row, *col;
  const int32_t *in_ptr, *in_edge;   /* [N + 1], [E] */
  const int32_t *out_ptr, *out_edge; /* [N + 1], [E] */
  const float* weight[MSW_MAX_MLP_LAYERS];
  const float* bias[MSW_MAX_MLP_LAYERS];  /* NULL = bias=False */
  const float* slope[MSW_MAX_MLP_LAYERS]; /* device scalar (PReLU) or NULL */
  const float* filter[MSW_MAX_HOPS + 1];  /* with_filter_matrix: K + 1 matrices */
} msw_swegnn_train_desc;

/* Gradient outputs (device; written, not accumulated).  d_x_d is required; any other NULL
 * pointer skips that gradient. */
typedef struct {
  float *d_x_s, *d_x_d, *d_edge_attr;
  float* d_weight[MSW_MAX_MLP_LAYERS];
  float* d_bias[MSW_MAX_MLP_LAYERS];
  float* d_slope[MSW_MAX_MLP_LAYERS];
  float* d_filter[MSW_MAX_HOPS + 1];
} msw_swegnn_grads;

/* Floats of the forward's saved state (kept until the backward) and of the backward's scratch. */
int msw_swegnn_train_workspace(const msw_swegnn_train_desc* desc, int64_t* saved_floats,
                               int64_t* scratch_floats);
/* out [N][F] = SWEGNN(x_s, x_d, edge_attr); `saved` receives the MLP inputs / pre-activations,
 * s_ij, ||h||, out_k, the aggregated messages and the activity flags of every hop. */
int msw_swegnn_train_forward(const msw_swegnn_train_desc* desc, const float* x_s, const float* x_d,
                             const float* edge_attr, float* saved, float* out, void* stream);
/* Gradients of all inputs and parameters given grad_out [N][F] and the forward's `saved`. */
int msw_swegnn_train_backward(const msw_swegnn_train_desc* desc, const float* x_s, const float* x_d,
                              const float* edge_attr, const float* saved, const float* grad_out,
                              const msw_swegnn_grads* grads, float* scratch, void* stream);

/* ---- Training: autograd through one make_mlp stack --------------------------
 * Replaces the autograd of a make_mlp Sequential (models/models.py:121-146: Linear + activation
 * after every layer, no dropout / layer norm) -- the model's edge / node encoders and node
 * decoder (models/gnn.py:204-215, 239-240) -- in training_step (training/train.py:125-145). */
typedef struct {
  int64_t rows;
  int32_t n_layers;                      /* 1..MSW_MAX_MLP_LAYERS */
  int32_t width[MSW_MAX_MLP_LAYERS + 1]; /* width[0] = input features, width[n_layers] = output */
  int32_t act[MSW_MAX_MLP_LAYERS];       /* enum msw_activation after each layer */
  const float* weight[MSW_MAX_MLP_LAYERS]; /* [width[l+1]][width[l]] */
  const float* bias[MSW_MAX_MLP_LAYERS];   /* NULL = bias=False */
  const float* slope[MSW_MAX_MLP_LAYERS];  /* device scalar (PReLU) or NULL */
} msw_mlp_train_desc;

/* Gradient outputs (device; written, not accumulated); NULL skips that gradient. */
typedef struct {
  float* d_x;
  float* d_weight[MSW_MAX_MLP_LAYERS];
  float* d_bias[MSW_MAX_MLP_LAYERS];
  float* d_slope[MSW_MAX_MLP_LAYERS];
} msw_mlp_grads;

int msw_mlp_train_workspace(const msw_mlp_train_desc* desc, int64_t* saved_floats, int64_t* scratch_floats);
/* out [rows][width[n_layers]] = MLP(x [rows][width[0]]); `saved` receives every layer's
 * pre-activation and the hidden layers' outputs. */
int msw_mlp_train_forward(const msw_mlp_train_desc* desc, const float* x, float* saved, float* out, void* stream);
/* Gradients of the input and the parameters given grad_out and the forward's `saved`. */
int msw_mlp_train_backward(const msw_mlp_train_desc* desc, const float* x, const float* saved,
                           const float* grad_out, const msw_mlp_grads* grads, float* scratch, void* stream);

/* ---- Training: autograd of the mean pooling ----------------------------------
 * Replaces MSGNN._pooling (models/gnn.py:242-257, learnable=False, reduce='mean') and its
 * autograd: pooling edge e maps fine[e] -> coarse[e] (intra_mesh_edge_index rows (coarse,
 * fine), gnn.py:310); cptr / cedge = CSR of the pooling edges by coarse node, fptr / fedge by
 * fine node ([N + 1], [E], edges in pooling-edge order).  out[c] = sum of x[fine] over c's
 * edges / max(#edges, 1), rows without children 0; deterministic (no atomics). */
int msw_pool_mean_forward(int64_t num_nodes, int32_t F, const int32_t* fine, const int32_t* cptr,
                          const int32_t* cedge, const float* x, float* out, void* stream);
int msw_pool_mean_backward(int64_t num_nodes, int32_t F, const int32_t* coarse, const int32_t* cptr,
                           const int32_t* fptr, const int32_t* fedge, const float* grad_out, float* grad_x,
                           void* stream);

/* Diagnostics: route per-phase timestamps of wave 0 of workgroup 0 of every launch to the
 * device buffer `buf` (uint64[20]: {shader clock, 100 MHz clock} for phase marks 0..9).
 * Only builds compiled with -DMSW_TRACE record anything; NULL disables. */
int msw_set_trace(msw_plan* plan, uint64_t* buf);

/* sizeof() of a descriptor struct ("msw_linear", "msw_mlp", "msw_swegnn",
 * "msw_model_desc", "msw_graph_desc", "msw_plan_stats"); -1 if unknown.  Pure host code:
 * lets FFI bindings verify their struct layouts without a GPU. */
int64_t msw_struct_size(const char* name);
const char* msw_last_error(void);
int msw_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MSWEGNN_H */
