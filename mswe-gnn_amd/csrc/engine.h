// Internal interface between the host plan (plan.hip) and the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

namespace msw {

constexpr int kMaxLayers = 4;

// One packed layer for the MFMA chain.  `a_off` indexes the packed operand
// [tout][tin][r4][lane][4] (floats) in a weight blob, `b_off` a bias padded to 32*tout
// (-1 = none).  tin/tout count 32-wide feature tiles.
struct LayerDev {
  int tin, tout;
  int a_off, b_off;
  int act;
  float slope;
};
struct MlpDev {
  int n;
  LayerDev l[kMaxLayers];
};

// Device-resident rollout I/O record: kernels read it so that one captured step graph
// can be replayed for every time step and every rollout call.
struct RolloutIO {
  const float* bc;  // [n_bc][p][bc_tstride]
  float* out;       // [N][2][T] (graph numbering)
  int bc_tstride;
  int type_bc;
  int T;
  int step;         // current step, advanced by the encoder kernel of each step
};

struct EncodeArgs {
  const float* x;      // [N][nnf] rows; row of internal node i is perm ? perm[i] : i
  const int* perm;
  int N, nnf, nstat_raw, with_wl, dyn;
  MlpDev stat, dynm;
  const float* W;
  float* xs;  // [N][FP]
  float* xd;  // [N][FP]
  int xd_rows;  // dynamic encoder only needed for the first `xd_rows` internal rows
  RolloutIO* io;  // non-null in rollout mode: advance io->step
};

struct RowMlpArgs {
  const float* in; int in_stride, in_dim;
  int R;
  MlpDev m;
  const float* W;
  float* out; int out_stride;
};

struct NodeProjArgs {
  int r0, R;                 // internal rows [r0, r0+R)
  const float* xs;           // [N][FP]
  const float* xin;          // [N][FP] or null (zeros)
  int a_u, a_v, a_o;         // packed operand offsets (-1 = output not wanted)
  const float* W;
  float* U; float* V;        // [N][H1P]
  float* O;                  // [N][FP]
  int h1t;                   // tiles of U / V
};

struct EdgeMlpArgs {
  int E;
  const int* src; const int* dst;  // CSR order
  const float* U; const float* V;  // [N][H1P]
  const float* Pe;                 // [E][H1P] (edge part of layer 1 incl. its bias) or null
  const float* b1;                 // layer-1 bias [H1P] used when Pe is null
  int h1t;
  int act1; float slope1;
  MlpDev rest;                     // layers 2..L (offsets relative to W)
  const float* W;                  // blob base of `rest` (staged to LDS)
  int w_count;                     // floats of W to stage
  int normalize;
  float* s;                        // [E][FP]
};

struct HopArgs {
  int n0, R;               // destination rows [n0, n0+R)
  const int* rowptr;       // [R+1] into src / s
  const int* src;
  const float* s;          // [E][FP]
  const float* in;         // [N][FP] or null (zero rows)
  float* out;              // [N][FP]
  const float* WT;         // [FP][FP] transposed filter or null
  const float* skip;       // [N][FP] or null
  int own_zero;            // destination rows read as zero (intra_scale_gnn fine rows)
  int grad, upwind, post_act; float post_slope;
};

struct PoolArgs {
  int n0, R;
  const int* rowptr;
  const int* child;
  const float* in;
  float* out;
};

struct DecodeArgs {
  int N, nnf, dyn, p;
  const float* xup;        // [N][FP]
  int pre_act; float pre_slope;
  MlpDev dec;
  const float* W;
  const float* resw;       // [p][2] or null
  float* X;                // state rows (residual source); internal rows, or external via perm
  const int* perm;         // internal -> graph numbering
  float* y;                // forward mode: [N][2] graph numbering (null in rollout mode)
  RolloutIO* io;           // rollout mode
  const int* bc_slot;      // [N] internal -> BC row or -1
};

struct InitArgs {
  const float* x0; const int* perm; int N, nnf, dyn, p;
  float* X;
  RolloutIO* io;
  const int* bc_slot;
};

constexpr int kSlotBatch = 64;
struct SlotArgs {
  int* slot;
  int n;
  int row[kSlotBatch];
  int val[kSlotBatch];
};
hipError_t launch_set_slots(const SlotArgs& a, hipStream_t st);
hipError_t launch_set_io(RolloutIO* dst, const RolloutIO& v, hipStream_t st);

template <int FP> hipError_t launch_encode(const EncodeArgs& a, hipStream_t st);
template <int FP> hipError_t launch_rowmlp(const RowMlpArgs& a, hipStream_t st);
template <int FP> hipError_t launch_node_proj(const NodeProjArgs& a, hipStream_t st);
template <int FP> hipError_t launch_edge_mlp(const EdgeMlpArgs& a, hipStream_t st);
template <int FP> hipError_t launch_hop(const HopArgs& a, hipStream_t st);
template <int FP> hipError_t launch_pool(const PoolArgs& a, hipStream_t st);
template <int FP> hipError_t launch_decode(const DecodeArgs& a, hipStream_t st);
hipError_t launch_init_state(const InitArgs& a, hipStream_t st);

}  // namespace msw
