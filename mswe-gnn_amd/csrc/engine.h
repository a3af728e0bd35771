// Internal interface between the host plan (plan.hip) and the gfx950 kernels
// (kernels_impl.h, instantiated per F in kernels_nt*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "graph_build.h"  // kRowsPerWave, kMaxScales and the host-built records (LaneRec, ...)

namespace msw {

constexpr int kMaxLayers = 4;
constexpr int kWaves = 4;  // waves per block (tiles per workgroup)
constexpr int kRowsPerBlock = kRowsPerWave * kWaves;
constexpr int kXcds = 8, kCusPerXcd = 32;  // MI355X: 8 XCDs x 32 CUs (workgroup i -> XCD i % 8)

// One packed layer of an MFMA chain.  `a_off` indexes the packed A operand
// [tout][tin][lane][4] (floats, 16-feature tiles) in the weight blob, `b_off` a bias
// padded to 16*tout (-1 = none).
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

// Weight region of one launch: blob floats [off, off+len) (len % 4 == 0) copied into LDS
// by every workgroup before use; the operand offsets in that launch's arguments are then
// LDS offsets (plan.hip: relocate).  F = 64 launches read the blob in place (len = 0).
struct WReg {
  int off, len;
  int split;  // floats needed before the epilogue; [split, len) = epilogue operands (or len)
};
template <int NT> constexpr bool kStaged = NT <= 2;

// Device-resident rollout I/O record: kernels read it so that one captured step graph
// can be replayed for every time step and every rollout call.
struct RolloutIO {
  const float* bc;  // [n_bc][p][bc_tstride]
  float* out;       // [N][2][T] (graph numbering)
  int bc_tstride;
  int type_bc;
  int T;
  int step;         // rollout mode: -1 before step 0; advanced once per step -- by the encoder
                    // when the last hops decode, by the first edge-MLP launch when the decoder
                    // is deferred to the next encoder (which then reads t - 1, the step it decodes)
};

// Node projection of one SWEGNN layer from [x_s ; x_in] of a node tile:
//   U = W1[:, x_s(row) | x_d(row)] [x_s; x_in]   (gnn.py:414-417, row = source node)
//   V = W1[:, x_s(col) | x_d(col)] [x_s; x_in]   (col = receiving node)
//   O = filter_matrix[0] x_in                    (gnn.py:401-402; identity without filter)
// An offset < 0 = that output is not produced.
struct NpDesc {
  int a_u, a_v, a_o;
  int h1t;
  float* U; float* V; float* O;
};

// Decoder + rollout bookkeeping for a node tile (gnn.py:335-348, models.py:50-91,
// dataset.py:486-529, train.py:88-95).
struct DecDesc {
  int on;
  int pre_act; float pre_slope;
  MlpDev dec;
  int resw_off;            // [p][2] residual matrix in the blob, -1 = none
  const float* X;          // residual source: rollout state (internal rows) or forward input
  int x_internal;          // X rows are internal (rollout) or graph rows (forward, via perm)
  float* y;                // forward mode: [N][2] graph numbering
  RolloutIO* io;           // rollout mode (X internal rows, updated in place)
  const int* bc_slot;      // [Npad] internal -> BC row or -1
};

// Kernels load unconditionally: a load under a run-time flag compiles to a branch behind
// which the compiler drains the memory counter, serialising the prologue's loads.  A flag
// that switches a load off points it at Common::zrow (or clamps the index) instead.
constexpr int kZeroRow = 256;
struct Common {
  const float* W;          // weight blob
  const int* perm;         // internal -> graph numbering (-1 = padding row)
  int nnf, dyn, p, nstat_raw, with_wl;
  int prelu;               // every MLP activation is PReLU (compile-time activation path)
  const float* zrow;       // kZeroRow zeros: the address of a load a flag switches off
  unsigned long long* trace;  // diagnostic builds (-DMSW_TRACE): per-phase timestamps of wave 0
  int xcd_max;             // XCD packing of small grids: at most this many XCDs (0 = off)
  int xcd;                 // set by the launcher: this launch runs on XCDs 0 .. xcd-1 (0 = all)
};

// Encoder.  Scale ranges start at multiples of 64 rows, so a workgroup has one scale.
struct EncodeArgs {
  Common c;
  int max_blocks;          // grid cap (resident workgroups), <= 0 = one per 64-row chunk
  WReg reg;                // unused (len 0)
  WReg sreg[kMaxScales];   // per scale: static encoder, dynamic encoder & projection 0
                           // (s = 0), unpool V -- the static encoder at the same offsets
  int lds_floats;          // max over s of sreg[s].len
  const float* x;          // input rows (forward: graph rows via perm; rollout: X)
  int x_internal;
  int Npad;
  int S;
  int n0[kMaxScales + 1];  // padded scale starts, n0[S] = Npad
  int ns[kMaxScales];      // valid rows per scale
  MlpDev stat, dynm;
  float* xs;               // [Npad][F]
  float* xd;               // [Npad][F] (scale-0 rows)
  NpDesc np0;              // projection of processor 0 (scale 0, x_in = x_d)
  int vu_a[kMaxScales];    // unpool V (x_s part) for fine rows of level s, -1 = none
  int vu_h1t;
  float* Vu;
  RolloutIO* io;           // rollout mode with the decoder in the last hops: advance io->step
  // Rollout mode: the decoder of the PREVIOUS step runs here, row-locally, before the
  // encoders (its input, the last SWEGNN layer's output, is stored by that layer's last
  // hop): prediction -> rollout output, window shift + BC of this step into X, and the
  // encoders read the updated state.  dec.on = 0 in forward mode (the decoder then runs in
  // the last hops' epilogues).  decode_only = 1: the rollout's final decode (no encoders).
  DecDesc dec;
  const float* dec_in;     // [Npad][F] decoder input rows (x_up / the GNN's last layer output)
  int decode_only;
  int coop;                // = NT: k_encode_coop (NT waves per 16-row tile), else k_encode
  int stream;              // 1: streaming stores (grid-stride launch without the decoder)
};

struct Epilogue {
  int post_act; float post_slope;  // GNN: gnn_activation after every SWEGNN layer
  NpDesc np;                       // projection of the next layer from [x_s; out]
  int uu_a; int uu_h1t; float* Uu; // unpool U from [x_s; out] (coarse rows)
  DecDesc dec;
};

// Fused: edge MLP (s_ij for every edge, stored for the later hops) + hop 1
// (+ epilogue when the layer has K = 1; intra-scale unpooling is such a layer).
// Records built on the host (graph_build.h): LaneRec, EdgeChunk, PoolRec, PoolSlot.
struct PoolFuse {
  const PoolSlot* slots;           // [ntiles][16], null = not fused
  const int* child;                // internal fine rows, reference order (PoolArgs::child)
  const float* in;                 // x_down (fine rows)
  NpDesc np;                       // projection of the processor (outputs not stored)
  // ... or the unpooling layer into this scale fused instead (slots null, parent set): the
  // intra-scale SWEGNN of each slot's two nodes (one in-edge from the coarse parent, own rows
  // zero, + skip), then the projection np -- the unpooling launch's work, in this launch
  const int2* parent;              // [ntiles][16] {parent of the slot's source, of the lane's
                                   // destination}: coarse internal rows, -1 = none
  int cpad;                        // a real coarse row (absent parents load it)
  const float* Uu; const float* Vu;  // unpool U (coarse rows) / V (fine rows) [Npad][16*h1t]
  const float* xc;                 // x_up (coarse rows): the parent's out_0
  const float* skip;               // + skip rows (x_down) or null
  int b1_off, h1t, act1; float slope1;
  MlpDev rest;                     // the unpooling layer's edge MLP layers 2..L
  int normalize, grad, upwind;
  int post_act; float post_slope;
};

constexpr int kMlpStagger = 2;  // k_edge_mlp start stagger (profiles/r05/ab_f64_mlp_stagger.txt)
struct EdgeHopArgs {
  Common c;
  WReg reg;                        // [MLP | epilogue operands | filter W_1]
  int reg_nf;                      // floats without the trailing filter copy (one-tile-per-wave
                                   // variant, which keeps the filter in registers)
  int max_blocks;                  // grid cap of the grid-stride variant (resident workgroups)
  int fit_blocks;                  // workgroups of the one-tile-per-wave variant the chip holds
  int n0;                          // first internal row of the destination scale
  const LaneRec* recs; int ntiles; // [ntiles][16]
  const float* xs;
  const float* U; const float* V;  // [Npad][16*h1t]
  const float* Pe;                 // [16 ntiles][16*h1t] or null (then bias b1_off)
  int b1_off;
  int h1t;
  int act1; float slope1;
  MlpDev rest;                     // layers 2..L
  int normalize;
  float* s;                        // [16 ntiles][F] (null: not needed later)
  const float* in;                 // out_0 rows [Npad][F]
  int own_zero;                    // destination rows read as zero (intra_scale_gnn)
  int grad, upwind;
  int filt_a;                      // packed filter W_1, -1 = none (blob offset)
  int filt_l;                      // the same operand in the launch's LDS region (grid-stride variant)
  const float* skip;               // + skip rows (unpool), or null
  float* out;                      // out_1 rows, or null
  int last;                        // last hop of the layer: run the epilogue
  Epilogue epi;
  int coop;                        // waves per tile (k_edge_coop: MFMA output tiles split
                                   // across them), 0/1 = one wave per tile
  int stagger;                     // k_edge_mlp: waves 4..7 start this many x 2 k cycles late
                                   // (kMlpStagger)
  int wdirect;                     // k_edge_coop4: read the MLP region from its blob copy
                                   // (c.W + reg.off) instead of staging it in LDS
  int* step_inc;                   // rollout mode, first edge-MLP launch of a step:
                                   // &RolloutIO::step, advanced once (workgroup 0, lane 0)
  const EdgeChunk* chunks; int nchunks;  // k_edge_mlp: dense 16-edge chunks [nchunks][16]
  PoolFuse pool;                   // mean pooling + projection fused in (k_edge_coop only)
};

// Hops 2..K over the same edge tiles as the fused first hop.
struct HopArgs {
  Common c;
  WReg reg;
  int max_blocks;                  // grid cap of the grid-stride variant (resident workgroups)
  int fit_blocks;                  // workgroups of the one-tile-per-wave variant the chip holds
  int n0;                  // first internal row of the scale
  const LaneRec* recs; int ntiles;
  const float* s;          // [16 ntiles][F]
  const float* xs;
  const float* in;         // [Npad][F]
  float* out;              // [Npad][F]
  int filt_a;              // packed filter W_{k+1}, -1 = none
  int grad, upwind;
  int last;
  Epilogue epi;
  int coop;          // last hop: waves per tile (k_hop_coop), 0 = one
  int split;         // middle hop: features split over two waves per tile (k_hop_split)
  // middle hop in the row layout (k_hop_rows, large meshes): 16 consecutive destinations per
  // wave, each lane row pulling its in-edges from the scale's CSR by destination
  int rows;
  int nrows;         // destinations of the scale (local rows [0, nrows) = internal n0 + k)
  const int* rptr;   // [nrows + 1] CSR offsets (local destination order)
  const int2* redge; // [E] {internal source row, tile-padded s slot}, reference edge order
};

// Mean pooling into the coarse rows + projection of the next processor.

struct PoolArgs {
  Common c;
  WReg reg;
  int max_blocks;                  // grid cap of the grid-stride variant (resident workgroups)
  int fit_blocks;                  // workgroups of the one-tile-per-wave variant the chip holds
  int n0, ns;              // internal rows [n0, n0 + ns) of the coarse scale
  int rows;                // 1: row layout (k_pool), 0: edge tiles (k_pool_edge)
  int ntiles;              // tiles of the chosen layout
  const PoolRec* recs;     // row layout: 16 consecutive coarse rows per tile, one record each
  const LaneRec* erecs;    // edge tiles: children <= 16 per tile (16 lane records per tile)
  int rtiles, etiles;      // tile counts of the two layouts
  const int* child;        // internal fine rows, in reference (intra edge) order
  const float* in;         // x_down
  const float* xs;
  NpDesc np;
  int coop;                // edge tiles: 2 = two waves per tile (projection split), else one
};

// Epilogue of a layer's last hop on dense 16-row node tiles (large scales, plan.hip
// sched_proc): the hop runs as a middle hop and stores its result rows (before post_act);
// this launch applies what follows the hop (node_epilogue) to rows [n0, n0 + ns).  An edge
// tile holds ~5 destinations of its <= 16 rows on a triangular mesh, so the epilogue's
// MFMA chains (projections, decoder) run on 3x fewer tiles here.
struct EpiArgs {
  Common c;
  WReg reg;                // epilogue operands (LDS region)
  int max_blocks, fit_blocks;
  int n0, ns, ntiles;      // ntiles = ceil(ns / 16)
  const float* in;         // the last hop's result rows
  const float* xs;
  float* out;              // the layer's output rows (may be `in`, or null)
  Epilogue epi;
};

// Forward mode (msw_forward), decoder deferred out of the last hops: one row-local launch
// after the schedule decodes every node from the stored last-layer rows (gnn.py:335-348,
// models.py:50-91), as the rollout's encoder does for the previous step.
struct DecodeArgs {
  Common c;                // c.W: the blob (the decoder operands stay blob offsets)
  int Npad;                // rows [0, Npad), 16 per wave; padding rows (perm -1) skipped
  const float* in;         // [Npad][F] the last layer's output rows (x_up / the GNN's last layer)
  DecDesc dec;             // forward variant: X = the forward input (graph rows), y = output
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

struct RowMlpArgs {
  int mode;  // 0: edge encoder chain (<= 16 raw features -> F ... -> F); 1: one F -> 2F layer
  const float* in; int in_stride, in_dim;
  int R;
  MlpDev m;
  const float* W;
  float* out; int out_stride, out_tiles;
};

// dynamic LDS of a launch: its weight region rounded up to whole 1-KB LDS-DMA chunks
// (kChunk floats); the edge hop stages its MLP region at every width
constexpr int kChunk = 256;
constexpr size_t eh_lds_bytes(int floats) {
  return (size_t)((floats + kChunk - 1) / kChunk * kChunk) * sizeof(float);
}
// Dynamic-LDS cap of the cooperative edge hop (k_edge_coop / k_edge_coop4) with `pw` waves
// per tile, with fused (un)pooling or not: 160 KB minus its static slabs and exchange buffers.
// prepare_kernels sets exactly this; plan creation checks every such launch against it.
template <int NT>
constexpr int edge_coop_lds_cap(int pw, int fuse) {
  if constexpr (NT == 4) {
    return 160 * 1024 - (kWaves / pw) * (kRowsPerWave * (48 * NT + 4) * 4 + 2 * kRowsPerWave * (32 * NT + 4) * 4);
  } else {
    const int st = kWaves * kRowsPerWave * (48 * NT + 4) * 4 + (kWaves / 2) * 2 * kRowsPerWave * (32 * NT + 4) * 4;
    // fused (un)pooling: + the source rank's U | O exchange rows (one slab per tile)
    const int ps = fuse ? (kWaves / 2) * kRowsPerWave * (48 * NT + 4) * 4 : 0;
    return 160 * 1024 - st - ps;
  }
}
// Records `msg` as msw_last_error() (thread-local) and returns `code` (plan.hip).
int set_error(int code, const char* msg);

hipError_t launch_set_slots(const SlotArgs& a, hipStream_t st);
hipError_t launch_set_io(RolloutIO* dst, const RolloutIO& v, hipStream_t st);
hipError_t launch_init_state(const InitArgs& a, hipStream_t st);
hipError_t launch_copy_rows(const float* src, const int* srows, float* dst, const int* drows, int n, int width,
                            hipStream_t st);

// NT = F / 16 feature tiles (F = 16, 32, 64 -> NT = 1, 2, 4)
template <int NT> hipError_t prepare_kernels();
// kind 0 encode, 1 edge_hop, 2 hop, 3 pool, 5 pool edge tiles, 6 row epilogue (and the
// cooperative / split / row-layout variants, kernels_impl.h kernel_of)
template <int NT> int resident_blocks(int kind, int prelu, int last, size_t dyn_bytes, int loop);
template <int NT> hipError_t launch_encode(const EncodeArgs& a, hipStream_t st);
template <int NT> hipError_t launch_edge_hop(const EdgeHopArgs& a, hipStream_t st);
template <int NT> hipError_t launch_edge_mlp(const EdgeHopArgs& a, hipStream_t st);
template <int NT> hipError_t launch_hop(const HopArgs& a, hipStream_t st);
template <int NT> hipError_t launch_pool(const PoolArgs& a, hipStream_t st);
template <int NT> hipError_t launch_epi(const EpiArgs& a, hipStream_t st);
template <int NT> hipError_t launch_rowmlp(const RowMlpArgs& a, hipStream_t st);
template <int NT> hipError_t launch_decode(const DecodeArgs& a, hipStream_t st);

}  // namespace msw
