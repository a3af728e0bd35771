// Internal interface between the host plan (plan.hip) and the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

namespace msw {

constexpr int kMaxLayers = 4;
constexpr int kRowsPerWave = 16;  // v_mfma_f32_16x16x4_f32: 16 rows (nodes / edges) per wave
constexpr int kWaves = 4;         // waves per 256-thread block
constexpr int kRowsPerBlock = kRowsPerWave * kWaves;

// One packed layer of an MFMA chain.  `a_off` indexes the packed A operand
// [tout][tin][lane][4] (floats, 16-feature tiles) in a weight blob, `b_off` a bias padded
// to 16*tout (-1 = none).
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
  float* xs;  // [N][F]
  float* xd;  // [N][F]
  int xd_rows;  // dynamic encoder only needed for the first `xd_rows` internal rows
  RolloutIO* io;  // non-null in rollout mode: advance io->step
  int prelu_only; // every MLP activation is PReLU: compile-time activation kernel
};

struct RowMlpArgs {
  int mode;  // 0: edge encoder chain (<= 16 raw features -> F ... -> F); 1: one F -> 2F layer
  const float* in; int in_stride, in_dim;
  int R;
  MlpDev m;
  const float* W;
  float* out; int out_stride, out_tiles;
};

// Node-side part of a SWEGNN layer's first edge-MLP layer and filter 0.  Output tiles are
// enumerated [U (h1t) | V (h1t) | O (T)]; blockIdx.y selects a pair of them.
struct NodeProjArgs {
  int r0, R;                 // internal rows [r0, r0+R)
  const float* xs;           // [N][F]
  const float* xin;          // [N][F] or null (zeros)
  int a_u, a_v, a_o;         // packed operand offsets (-1 = output not wanted)
  const float* W;
  float* U; float* V;        // [N][16*h1t]
  float* O;                  // [N][F]
  int h1t;                   // 16-feature tiles of U / V
};

struct EdgeMlpArgs {
  int E;
  const int* src; const int* dst;  // CSR order
  const float* U; const float* V;  // [N][16*h1t]
  const float* Pe;                 // [E][16*h1t] (edge part of layer 1 incl. its bias) or null
  const float* b1;                 // layer-1 bias [16*h1t] used when Pe is null
  int h1t;
  int act1; float slope1;
  MlpDev rest;                     // layers 2..L (offsets relative to W)
  const float* W;                  // blob base of `rest` (staged to LDS)
  int w_count;                     // floats of W to stage
  int normalize;
  int prelu_only;
  float* s;                        // [E][F]
};

struct HopArgs {
  int n0, R;               // destination rows [n0, n0+R)
  const int* rowptr;       // [R+1] into src / s
  const int* src;
  const float* s;          // [E][F]
  const float* in;         // [N][F]
  float* out;              // [N][F]
  const float* A;          // packed filter W_{k+1} [T][T] operand, or null (no filter)
  const float* skip;       // [N][F] or null
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
  const float* xup;        // [N][F]
  int pre_act; float pre_slope;
  MlpDev dec;
  const float* W;
  const float* resw;       // [p][2] or null
  float* X;                // state rows (residual source); internal rows, or external via perm
  const int* perm;         // internal -> graph numbering
  float* y;                // forward mode: [N][2] graph numbering (null in rollout mode)
  RolloutIO* io;           // rollout mode
  const int* bc_slot;      // [N] internal -> BC row or -1
  int prelu_only;
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

// NT = F / 16 feature tiles (F = 16, 32, 64 -> NT = 1, 2, 4)
template <int NT> hipError_t launch_encode(const EncodeArgs& a, hipStream_t st);
template <int NT> hipError_t launch_rowmlp(const RowMlpArgs& a, hipStream_t st);
template <int NT> hipError_t launch_node_proj(const NodeProjArgs& a, hipStream_t st);
template <int NT> hipError_t launch_edge_mlp(const EdgeMlpArgs& a, hipStream_t st);
template <int NT> hipError_t launch_hop(const HopArgs& a, hipStream_t st);
template <int NT> hipError_t launch_pool(const PoolArgs& a, hipStream_t st);
template <int NT> hipError_t launch_decode(const DecodeArgs& a, hipStream_t st);
hipError_t launch_init_state(const InitArgs& a, hipStream_t st);

}  // namespace msw
