// gfx950 (MI355X, CDNA4) kernels of the multi-scale SWE-GNN rollout (templates; the
// kernels_nt*.hip units instantiate them for F = 16, 32, 64).
//
// Layout
//  * every F-wide node / edge vector is fp32, row-major, unpadded (stride F).
//  * A wave owns 16 ROWS (nodes or edges).  Lane l works on row j = l & 15 and, in lane
//    group g = l >> 4, holds features 16t + 4g + r (r = 0..3) of every 16-feature tile t
//    in one f32x4 per tile.  That is the accumulator layout of v_mfma_f32_16x16x4_f32 with
//    the row on the MFMA column (C/D: col = l & 15, row = 4(l >> 4) + r) and, register
//    for register, the B operand of the next layer (k-step (t, r): lane group g supplies
//    feature 16t + 4g + r).  Layers chain in registers: no shuffles between layers; the
//    A operands (weights) of a launch are staged once per workgroup in LDS.  Packed A operand: A[to][ti][lane][r] = W[16 to + (l & 15)][16 ti + 4 (l >> 4) + r].
//  * f32 in / f32 accumulate MFMA = exact fp32 fma chains (no TF32 on gfx950).
//  * message passing runs on edge tiles (whole destination neighbourhoods, <= 16 edges):
//    one lane per edge computes its message, the destination lane sums them from LDS in
//    the reference's edge order -- no atomics, bit-reproducible run to run.
//  * one rollout step = encoder (+ projection of processor 0) -> per processor: fused
//    edge-MLP+hop-1, hops 2..K (the last with an epilogue: next projection / unpool
//    projection / decoder + rollout update) -> pooling+projection / unpooling+projection.
#pragma once
#include "engine.h"

namespace msw {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 64 * kWaves;
// Grid-stride (LOOP) variants of the tile kernels run 8-wave workgroups when their weights
// are staged in LDS (F <= 32): one staged copy per 8 waves instead of per 4 halves the
// staging traffic of a large mesh and the LDS the copies take.
template <int NT, bool LOOP>
constexpr int waves_of() { return LOOP && NT <= 2 ? 8 : kWaves; }
// the grid-stride middle / last hop (k_hop, large meshes): its own workgroup size
#ifndef MSW_HOP_WAVES
#define MSW_HOP_WAVES 8
#endif
template <int NT, bool LOOP>
constexpr int hop_waves() { return LOOP && NT <= 2 ? MSW_HOP_WAVES : kWaves; }
// the fused edge MLP + hop keeps one tile per wave in flight in its grid-stride loop:
// a software-pipelined loop (next tile's gathers during the MLP) needs > 256 registers,
// i.e. one wave per SIMD, and measured 24 % slower on the 1M-node mesh
#ifndef MSW_EDGE_WAVES
#define MSW_EDGE_WAVES 12   // grid-stride, with epilogue (LST = 1): 3 waves per SIMD
#endif
#ifndef MSW_EDGE_WAVES0
#define MSW_EDGE_WAVES0 16  // grid-stride, no epilogue (LST = 0): 4 waves per SIMD
#endif
// Workgroup of the grid-stride edge MLP + hop: as many waves as the register budget allows
// per SIMD, times 4 -- one workgroup per CU, so one staged weight copy serves all of them.
template <int NT, bool LOOP, int LST = 1>
constexpr int edge_waves() { return LOOP && NT <= 2 ? (LST ? MSW_EDGE_WAVES : MSW_EDGE_WAVES0) : kWaves; }
template <int NT, bool LOOP, int LST>
constexpr int edge_eu() { return LOOP && NT <= 2 ? edge_waves<NT, LOOP, LST>() / 4 : 1; }

#define MSW_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// ---------------------------------------------------------------------------- helpers
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ float hsum(f32x4 v) { return (v.x + v.y) + (v.z + v.w); }
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// sum over the 4 lane groups holding one row (lanes j, j+16, j+32, j+48): gfx950's
// v_permlane16_swap / v_permlane32_swap exchange rows of 16 lanes in registers (no LDS
// round trip as ds_bpermute would take); every lane gets (g0 + g1) + (g2 + g3).
__device__ __forceinline__ float row_sum(float v) {
  const unsigned u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const unsigned us = __float_as_uint(s);
  const auto b = __builtin_amdgcn_permlane32_swap(us, us, false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
// XCD packing (Common::xcd = k > 0, small one-round grids): the launch has 8x the workgroups
// it needs and only those the dispatcher places on XCDs 0 .. k-1 (workgroup i -> XCD i % 8)
// work.  The XCDs start a launch's workgroups up to ~1.3 us apart, most of a small hop's
// span; on k XCDs the skew is k XCDs' instead of eight.  Logical workgroup, -1 = idle.
__device__ __forceinline__ int logical_block(const Common& c) {
  const int b = blockIdx.x;
  if (c.xcd <= 0) return b;
  const int x = b % kXcds;
  return x < c.xcd ? (b / kXcds) * c.xcd + x : -1;
}
__device__ __forceinline__ int wave_row0() { return (blockIdx.x * kWaves + wave_id()) * kRowsPerWave; }

// activation_functions, models/models.py:149-169
template <int ACT>
__device__ __forceinline__ float act_static(float x, float slope) {
  if constexpr (ACT == 1) return x > 0.f ? x : slope * x;       // PReLU
  else if constexpr (ACT == 2) return x > 0.f ? x : 0.f;        // ReLU
  else if constexpr (ACT == 3) return x > 0.f ? x : 0.1f * x;   // LeakyReLU(0.1)
  else if constexpr (ACT == 4) return x > 0.f ? x : expm1f(x);  // ELU
  else if constexpr (ACT == 5) return x / (1.f + expf(-x));     // SiLU
  else if constexpr (ACT == 6) return 1.f / (1.f + expf(-x));   // Sigmoid
  else if constexpr (ACT == 7) return tanhf(x);                 // Tanh
  else return x;
}
template <int ACT, int N>
__device__ __forceinline__ void act_tiles_static(f32x4 (&v)[N], float slope) {
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[t][r] = act_static<ACT>(v[t][r], slope);
}
// ACT >= 0: activation fixed at compile time (PReLU kernels of the shipped configs);
// ACT < 0: one wave-uniform switch outside the element loops.
template <int ACT, int N>
__device__ __forceinline__ void act_tiles(f32x4 (&v)[N], int act, float slope) {
  if constexpr (ACT >= 0) {
    act_tiles_static<ACT, N>(v, slope);
  } else {
    switch (act) {
      case 1: act_tiles_static<1, N>(v, slope); break;
      case 2: act_tiles_static<2, N>(v, slope); break;
      case 3: act_tiles_static<3, N>(v, slope); break;
      case 4: act_tiles_static<4, N>(v, slope); break;
      case 5: act_tiles_static<5, N>(v, slope); break;
      case 6: act_tiles_static<6, N>(v, slope); break;
      case 7: act_tiles_static<7, N>(v, slope); break;
      default: break;
    }
  }
}

// acc[to] = sum_ti A[to][ti] in[ti]; A packed [TOUT][TIN].  Shapes are compile-time only:
// a run-time bound here puts a branch after every MFMA (accumulator read-back + s_nop),
// which measured ~130 cycles per 32-cycle MFMA.  The TOUT accumulators are independent
// chains interleaved per k-step (40-cycle dependent MFMA latency).
template <int TIN, int TOUT>
__device__ __forceinline__ void proj(const f32x4 (&in)[TIN], f32x4 (&acc)[TOUT],
                                     const float* __restrict__ A, int lane) {
#pragma unroll
  for (int to = 0; to < TOUT; ++to) acc[to] = zero4();
#pragma unroll
  for (int ti = 0; ti < TIN; ++ti) {
    f32x4 w[TOUT];
#pragma unroll
    for (int to = 0; to < TOUT; ++to) w[to] = ld4(A + ((size_t)(to * TIN + ti) * 64 + lane) * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int to = 0; to < TOUT; ++to) acc[to] = MSW_MFMA(w[to][r], in[ti][r], acc[to]);
  }
}

// nn.Linear (+ bias, + activation), compile-time shape TIN -> TOUT (make_mlp layer,
// models/models.py:121-146).
template <int TIN, int TOUT, int ACT>
__device__ __forceinline__ void mfma_layer(const f32x4 (&in)[TIN], f32x4 (&out)[TOUT],
                                           const LayerDev& L, const float* __restrict__ W,
                                           int lane, int g) {
  f32x4 acc[TOUT];
  proj<TIN, TOUT>(in, acc, W + L.a_off, lane);
#pragma unroll
  for (int to = 0; to < TOUT; ++to) acc[to] = acc[to] + ld4(W + L.b_off + 16 * to + 4 * g);  // zeros if bias=False
  act_tiles<ACT, TOUT>(acc, L.act, L.slope);
#pragma unroll
  for (int to = 0; to < TOUT; ++to) out[to] = acc[to];
}

// make_mlp chain IN0 -> T -> ... -> T -> TL: the layer count is a run-time value, every
// layer's shape is fixed at compile time (first IN0->T, or IN0->TL if m.n == 1; middle
// T->T; last T->TL), so all register arrays are statically indexed.
template <int IN0, int T, int TL, int ACT>
__device__ __forceinline__ void run_mlp(const f32x4 (&in)[IN0], f32x4 (&out)[TL], const MlpDev& m,
                                        const float* __restrict__ W, int lane, int g) {
  if (m.n == 1) {
    mfma_layer<IN0, TL, ACT>(in, out, m.l[0], W, lane, g);
    return;
  }
  f32x4 h[T];
  mfma_layer<IN0, T, ACT>(in, h, m.l[0], W, lane, g);
  for (int li = 1; li + 1 < m.n; ++li) {
    f32x4 h2[T];
    mfma_layer<T, T, ACT>(h, h2, m.l[li], W, lane, g);
#pragma unroll
    for (int t = 0; t < T; ++t) h[t] = h2[t];
  }
  mfma_layer<T, TL, ACT>(h, out, m.l[m.n - 1], W, lane, g);
}

template <int N>
__device__ __forceinline__ void load_row(f32x4 (&v)[N], const float* row, int g) {
#pragma unroll
  for (int t = 0; t < N; ++t) v[t] = ld4(row + 16 * t + 4 * g);
}
template <int N>
__device__ __forceinline__ void store_row(float* row, const f32x4 (&v)[N], int ntiles, int g) {
#pragma unroll
  for (int t = 0; t < N; ++t)
    if (t < ntiles) st4(row + 16 * t + 4 * g, v[t]);
}

// ---------------------------------------------------------------------------- epilogues
// Projection of a SWEGNN layer (U, V, O) from [x_s ; x_in] of a node tile; H1T = tiles of
// the first edge-MLP layer (2F, or F for one-layer MLPs).
template <int NT, int H1T>
__device__ __forceinline__ void np_project_t(const f32x4 (&xs)[NT], const f32x4 (&xin)[NT],
                                             const NpDesc& d, const float* W, size_t n, bool valid,
                                             int lane, int g) {
  constexpr int F = 16 * NT, T2 = 2 * NT;
  f32x4 in[T2];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    in[t] = xs[t];
    in[NT + t] = xin[t];
  }
  if (d.a_u >= 0) {
    f32x4 acc[H1T];
    proj<T2, H1T>(in, acc, W + d.a_u, lane);
    if (valid) store_row<H1T>(d.U + n * (16 * H1T), acc, H1T, g);
  }
  if (d.a_v >= 0) {
    f32x4 acc[H1T];
    proj<T2, H1T>(in, acc, W + d.a_v, lane);
    if (valid) store_row<H1T>(d.V + n * (16 * H1T), acc, H1T, g);
  }
  if (d.a_o >= 0) {
    f32x4 acc[NT];
    proj<NT, NT>(xin, acc, W + d.a_o, lane);
    if (valid) store_row<NT>(d.O + n * F, acc, NT, g);
  }
}
template <int NT>
__device__ __forceinline__ void np_project(const f32x4 (&xs)[NT], const f32x4 (&xin)[NT],
                                           const NpDesc& d, const float* W, size_t n, bool valid,
                                           int lane, int g) {
  if (d.h1t == 2 * NT)
    np_project_t<NT, 2 * NT>(xs, xin, d, W, n, valid, lane, g);
  else
    np_project_t<NT, NT>(xs, xin, d, W, n, valid, lane, g);
}

// U (or V) = W[:, blocks] [x_s ; x] with H1T output tiles, TIN input tiles.
template <int TIN, int H1T, int NT>
__device__ __forceinline__ void side_proj_t(const f32x4 (&in)[TIN], const float* A, float* dst, size_t n,
                                            bool valid, int lane, int g) {
  f32x4 acc[H1T];
  proj<TIN, H1T>(in, acc, A, lane);
  if (valid) store_row<H1T>(dst + n * (16 * H1T), acc, H1T, g);
}
template <int TIN, int NT>
__device__ __forceinline__ void side_proj(const f32x4 (&in)[TIN], int h1t, const float* A, float* dst,
                                          size_t n, bool valid, int lane, int g) {
  if (h1t == 2 * NT)
    side_proj_t<TIN, 2 * NT, NT>(in, A, dst, n, valid, lane, g);
  else
    side_proj_t<TIN, NT, NT>(in, A, dst, n, valid, lane, g);
}

// Everything an epilogue reads from HBM that does not depend on the tile's result, loaded
// with the tile's gathers at kernel start instead of after the hop (one latency less on the
// chain): x_s rows for the projections, the decoder's dynamic state columns, the step.
constexpr int kMaxDyn = 16;
template <int NT>
struct EpiPre {
  f32x4 xs[NT];
  float xd[kMaxDyn];  // X[row, nstat : nnf] (lane group 0 uses it)
  int ext, step;
  int bc;             // the row's BC slot (rollout mode), -1 = none
  float bcv[kMaxDyn / 2];  // deferred decoder: the row's BC values of step + 1 (bc_prefetch)
};
// Deferred decoder (k_encode): the BC values the state update writes, loaded with the tile's
// other inputs instead of after the decoder chain (a BC row's wave would otherwise wait for
// one more global load on the launch's critical path).
template <int NT>
__device__ __forceinline__ void bc_prefetch(EpiPre<NT>& p, const DecDesc& d, const Common& c) {
  const RolloutIO* io = d.io;
  const bool on = p.bc >= 0 && p.step + 1 < io->bc_tstride;
  const float* bp = on ? io->bc + (size_t)p.bc * c.p * io->bc_tstride + p.step + 1 : c.zrow;
  const int ts = on ? io->bc_tstride : 0;
#pragma unroll
  for (int u = 0; u < kMaxDyn / 2; ++u) p.bcv[u] = u < c.p ? bp[u * ts] : 0.f;
}
template <int NT>
__device__ __forceinline__ void epi_prefetch(EpiPre<NT>& p, const Epilogue& e, const Common& c,
                                             const float* xs_rows, size_t n, int g) {
  constexpr int F = 16 * NT;
  if (e.np.a_u >= 0 || e.np.a_v >= 0 || e.np.a_o >= 0 || e.uu_a >= 0) load_row<NT>(p.xs, xs_rows + n * F, g);
  if (e.dec.on) {
    p.ext = c.perm ? c.perm[n] : (int)n;
    p.step = e.dec.io ? e.dec.io->step : 0;
    p.bc = e.dec.bc_slot ? e.dec.bc_slot[n] : -1;  // here, not after the decoder chain
    const size_t row = e.dec.x_internal ? n : (size_t)(p.ext > 0 ? p.ext : 0);
    const float* xr = e.dec.X + row * c.nnf + (c.nnf - c.dyn);
#pragma unroll
    for (int k = 0; k < kMaxDyn; ++k) p.xd[k] = k < c.dyn ? xr[k] : 0.f;
  }
}
// tanh(x_up) -> node_decoder -> + learned residual -> ReLU -> small-depth mask
// (gnn.py:335-348, models.py:50-91); rollout mode: use_prediction + BC of the next step
// (dataset.py:486-529) and the rollout write (train.py:88-95).
// decode_tail: what follows the decoder MLP (o = its output tile: h, |q| in lane group 0)
template <int NT>
__device__ __forceinline__ void decode_tail(const f32x4 (&o)[1], const DecDesc& d, const Common& c,
                                            const EpiPre<NT>& pre, int n, bool valid, int g);
template <int NT, int ACT>
__device__ __forceinline__ void decode_rows(const f32x4 (&xup)[NT], const DecDesc& d, const Common& c,
                                            const EpiPre<NT>& pre, int n, bool valid, int lane, int g) {
#pragma clang fp contract(off)
  f32x4 x0[NT], o[1];
#pragma unroll
  for (int t = 0; t < NT; ++t) x0[t] = xup[t];
  act_tiles<-1, NT>(x0, d.pre_act, d.pre_slope);
  run_mlp<NT, NT, 1, ACT>(x0, o, d.dec, c.W, lane, g);
  decode_tail<NT>(o, d, c, pre, n, valid, g);
}
template <int NT>
__device__ __forceinline__ void decode_tail(const f32x4 (&o)[1], const DecDesc& d, const Common& c,
                                            const EpiPre<NT>& pre, int n, bool valid, int g) {
#pragma clang fp contract(off)
  if (!valid || g) return;  // lane group 0 holds output features 0 (h) and 1 (|q|)
  const int ext = pre.ext;
  if (ext < 0) return;
  float* xw = const_cast<float*>(d.X) + (size_t)(d.x_internal ? n : ext) * c.nnf + (c.nnf - c.dyn);
  float h = o[0].x, v = o[0].y;
  if (d.resw_off >= 0) {
    const float* rw = c.W + d.resw_off;
    float rh = pre.xd[0] * rw[0];
    float rv = pre.xd[1] * rw[1];
#pragma unroll
    for (int tau = 1; tau < kMaxDyn / 2; ++tau) {
      if (tau < c.p) {
        rh = rh + pre.xd[2 * tau] * rw[2 * tau];
        rv = rv + pre.xd[2 * tau + 1] * rw[2 * tau + 1];
      }
    }
    h = h + rh;
    v = v + rv;
  }
  h = h > 0.f ? h : 0.f;  // torch.relu
  v = v > 0.f ? v : 0.f;
  const float hm = h * (fabsf(h) > 1e-4f ? 1.f : 0.f);  // _mask_small_WD(epsilon=1e-4)
  const float vm = v * (h != 0.f ? 1.f : 0.f);
  if (!d.io) {
    d.y[(size_t)ext * 2 + 0] = hm;
    d.y[(size_t)ext * 2 + 1] = vm;
    return;
  }
  RolloutIO* io = d.io;
  const int t = pre.step;
  io->out[((size_t)ext * 2 + 0) * io->T + t] = hm;
  io->out[((size_t)ext * 2 + 1) * io->T + t] = vm;
  // use_prediction: shift the window by one step, the prediction becomes the newest pair
#pragma unroll
  for (int k = 0; k + 2 < kMaxDyn; ++k)
    if (k + 2 < c.dyn) xw[k] = pre.xd[k + 2];
  xw[c.dyn - 2] = hm;
  xw[c.dyn - 1] = vm;
  const int b = pre.bc;
  if (b >= 0 && t + 1 < io->bc_tstride) {
    for (int tau = 0; tau < c.p; ++tau)
      xw[(io->type_bc - 1) + 2 * tau] = io->bc[((size_t)b * c.p + tau) * io->bc_tstride + t + 1];
  }
}

// Rollout mode, in the NEXT step's encoder: the decoder of a 16-row node tile (x: the last
// SWEGNN layer's output rows, pre-activation applied here) + decode_tail's arithmetic (the
// same operations in the same order) and state update.  Every lane of a row ends with the
// row's new dynamic columns in nd (window shifted, prediction appended, BC of step t + 1);
// lane group 0 writes the rollout output and the state row.  W: the decoder operands.
template <int NT>
__device__ __forceinline__ void decode_state_tail(const f32x4 (&o)[1], const DecDesc& d, const Common& c,
                                                  const float* W, const EpiPre<NT>& pre, int n, bool valid,
                                                  int lane, int g, float (&nd)[kMaxDyn]);
template <int NT, int ACT>
__device__ __forceinline__ void decode_state(const f32x4 (&x)[NT], const DecDesc& d, const Common& c,
                                             const float* W, const EpiPre<NT>& pre, int n, bool valid,
                                             int lane, int g, float (&nd)[kMaxDyn]) {
#pragma clang fp contract(off)
  f32x4 x0[NT], o[1];
#pragma unroll
  for (int t = 0; t < NT; ++t) x0[t] = x[t];
  act_tiles<-1, NT>(x0, d.pre_act, d.pre_slope);
  run_mlp<NT, NT, 1, ACT>(x0, o, d.dec, W, lane, g);
  decode_state_tail<NT>(o, d, c, W, pre, n, valid, lane, g, nd);
}
template <int NT>
__device__ __forceinline__ void decode_state_tail(const f32x4 (&o)[1], const DecDesc& d, const Common& c,
                                                  const float* W, const EpiPre<NT>& pre, int n, bool valid,
                                                  int lane, int g, float (&nd)[kMaxDyn]) {
#pragma clang fp contract(off)
  // output features 0 (h) and 1 (|q|) live in lane group 0: every lane of the row takes them
  float h = __shfl(o[0].x, lane & 15), v = __shfl(o[0].y, lane & 15);
  if (d.resw_off >= 0) {
    const float* rw = W + d.resw_off;
    float rh = pre.xd[0] * rw[0];
    float rv = pre.xd[1] * rw[1];
#pragma unroll
    for (int tau = 1; tau < kMaxDyn / 2; ++tau) {
      if (tau < c.p) {
        rh = rh + pre.xd[2 * tau] * rw[2 * tau];
        rv = rv + pre.xd[2 * tau + 1] * rw[2 * tau + 1];
      }
    }
    h = h + rh;
    v = v + rv;
  }
  h = h > 0.f ? h : 0.f;  // torch.relu
  v = v > 0.f ? v : 0.f;
  const float hm = h * (fabsf(h) > 1e-4f ? 1.f : 0.f);  // _mask_small_WD(epsilon=1e-4)
  const float vm = v * (h != 0.f ? 1.f : 0.f);
  // use_prediction (window shift) + apply_boundary_condition of the next step; selects keep
  // nd in registers (run-time column indices would put it in scratch)
  const RolloutIO* io = d.io;
  const int t = pre.step, b = pre.bc;
  const bool bc_on = b >= 0 && t + 1 < io->bc_tstride;
  const int c0 = io->type_bc - 1;
#pragma unroll
  for (int k = 0; k < kMaxDyn; ++k) {
    float val = k + 2 < c.dyn ? pre.xd[k + 2] : (k == c.dyn - 2 ? hm : (k == c.dyn - 1 ? vm : 0.f));
    const int tau = (k - c0) >> 1;
    float bv = 0.f;  // pre.bcv[tau] by selects (a run-time register index would use scratch)
#pragma unroll
    for (int u = 0; u < kMaxDyn / 2; ++u) bv = u == tau ? pre.bcv[u] : bv;
    if (bc_on && k >= c0 && ((k - c0) & 1) == 0 && tau < c.p) val = bv;
    nd[k] = val;
  }
  if (!valid || g || pre.ext < 0) return;
  const int ext = pre.ext;
  io->out[((size_t)ext * 2 + 0) * io->T + t] = hm;
  io->out[((size_t)ext * 2 + 1) * io->T + t] = vm;
  float* xw = const_cast<float*>(d.X) + (size_t)n * c.nnf + (c.nnf - c.dyn);
#pragma unroll
  for (int k = 0; k < kMaxDyn; ++k)
    if (k < c.dyn) xw[k] = nd[k];
}

// What follows the last hop of a SWEGNN layer, on the layer's destination rows.
template <int NT, int ACT>
__device__ __forceinline__ void node_epilogue(f32x4 (&res)[NT], const Epilogue& e, const Common& c,
                                              const EpiPre<NT>& pre, float* out, int n,
                                              bool valid, int lane, int g) {
  constexpr int F = 16 * NT, T2 = 2 * NT;
  if (e.post_act) act_tiles<-1, NT>(res, e.post_act, e.post_slope);
  if (out && valid) store_row<NT>(out + (size_t)n * F, res, NT, g);
  const bool np = e.np.a_u >= 0 || e.np.a_v >= 0 || e.np.a_o >= 0;
  if (np || e.uu_a >= 0) {
    const f32x4(&xs)[NT] = pre.xs;
    if (np) np_project<NT>(xs, res, e.np, c.W, n, valid, lane, g);
    if (e.uu_a >= 0) {
      f32x4 in[T2];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        in[t] = xs[t];
        in[NT + t] = res[t];
      }
      side_proj<T2, NT>(in, e.uu_h1t, c.W + e.uu_a, e.Uu, n, valid, lane, g);
    }
  }
  if (e.dec.on) decode_rows<NT, ACT>(res, e.dec, c, pre, n, valid, lane, g);
}

// ---------------------------------------------------------------------------- tracing
// Diagnostic builds only (-DMSW_TRACE, tools/trace_kernels.py): wave 0 of workgroup 0 drains
// its memory counters and records {shader clock, 100 MHz clock} at each phase mark, so the
// dependent-latency chain of one launch can be read phase by phase.
#ifdef MSW_TRACE
// Every workgroup also records its start (mark 0, thread 0) and the end of its last wave
// (mark 9, max over waves) in 100 MHz ticks at trace[32 + 2 b] / [33 + 2 b], b < kTraceWG.
constexpr int kTraceWG = 8192;
#define MSW_MARK(c, k)                                                          \
  do {                                                                          \
    if ((c).trace && blockIdx.x == 0 && threadIdx.x < 64) {                     \
      __builtin_amdgcn_s_waitcnt(0);                                            \
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();               \
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();           \
      if (threadIdx.x == 0) { (c).trace[2 * (k)] = t0; (c).trace[2 * (k) + 1] = t1; } \
    }                                                                           \
    if ((c).trace && (k) == 0 && threadIdx.x == 0 && blockIdx.x < kTraceWG)     \
      (c).trace[32 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();       \
    if ((c).trace && (k) == 9 && blockIdx.x < kTraceWG) {                       \
      __builtin_amdgcn_s_waitcnt(0);                                            \
      const unsigned long long te = __builtin_amdgcn_s_memrealtime();           \
      if ((threadIdx.x & 63) == 0) atomicMax(&(c).trace[33 + 2 * blockIdx.x], te); \
    }                                                                           \
  } while (0)
#else
#define MSW_MARK(c, k) \
  do {                 \
  } while (0)
#endif

// ---------------------------------------------------------------------------- staging
// LDS-DMA staging (global_load_lds_dwordx4): one wave instruction copies 1 KB (256 floats)
// of the region straight into LDS, no VGPR round trip.  Copies the 256-float chunks that
// cover [first, last) floats of the region; a partial final chunk reads up to 255 floats
// past the region (the blob and the LDS allocation are padded for it).
template <int WV = kWaves>
__device__ __forceinline__ void stage_glds(float* smem, const float* __restrict__ W, WReg r, int first, int last) {
  const int lane = threadIdx.x & 63;
  for (int ch = first / kChunk + wave_id(); ch * kChunk < last; ch += WV)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(W + r.off + ch * kChunk + lane * 4),
        (__attribute__((address_space(3))) void*)(smem + ch * kChunk), 16, 0, 0);
}
__device__ __forceinline__ int chunk_ceil(int n) { return (n + kChunk - 1) / kChunk * kChunk; }

// ---------------------------------------------------------------------------- encoder
// Static / dynamic node encoders incl. the water-level feature (MSGNN.forward
// gnn.py:284-294, GNN.forward :112-123) + projection of processor 0 + the x_s part of
// every unpooling layer's V.  One workgroup = 64 rows of one scale.
// DEC: the rollout variant that decodes the previous step first (EncodeArgs::dec.on); the
// other variant keeps the encoders' register budget (four waves per SIMD) for forward mode
// and the large meshes whose last hops decode.
template <int NT, int ACT, bool DEC>
__global__ __launch_bounds__(kBlock) void k_encode(EncodeArgs a) {
  constexpr int F = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  MSW_MARK(a.c, 0);
  Common c = a.c;
  // rollout mode: the step whose prediction this launch decodes (the previous one; -1 at
  // step 0, whose state k_init_state wrote)
  const int dstep = DEC ? a.dec.io->step : -1;
  // rollout mode, decoder in the last hops (large meshes): advance the step they read
  if (!a.dec.on && a.io && blockIdx.x == 0 && threadIdx.x == 0) a.io->step += 1;
  const int nchunks = a.Npad / kRowsPerBlock;
  int staged = -1;  // scale whose region is in LDS
  // grid-stride over 64-row chunks (scale ranges are 64-aligned: a chunk has one scale);
  // the per-scale weight region is re-staged only when the scale changes
  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int rb = chunk * kRowsPerBlock;
    int s = 0;
    while (s + 1 < a.S && rb >= a.n0[s + 1]) ++s;
    const int n = rb + wave_id() * kRowsPerWave + j;
    const bool valid = (n - a.n0[s]) < a.ns[s];
    const int ext = a.c.perm ? a.c.perm[n] : n;
    const int xrow = a.x_internal ? (valid ? n : a.n0[s]) : (valid ? ext : 0);
    const float* xr = a.x + (size_t)xrow * a.c.nnf;
    const int nstat = a.c.nstat_raw;
    float raw[4], dyn[4];
    float wlv;
    EpiPre<NT> pre;
    f32x4 xu[NT];
    // the decoder's inputs, loaded before the weight staging and whatever the step (at step
    // 0 nothing reads them): not behind the load of the step counter, whose dependent loads
    // (the BC values) are issued after the staging barrier, in flight during the decoder MLP
    if (DEC) {
      load_row<NT>(xu, a.dec_in + (size_t)n * F, g);
      pre.ext = ext;
      pre.bc = a.dec.bc_slot[n];
#pragma unroll
      for (int k = 0; k < kMaxDyn; ++k) pre.xd[k] = k < c.dyn ? xr[nstat + k] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * g + r;
      raw[r] = f < nstat ? xr[f] : 0.f;
      dyn[r] = f < a.c.dyn ? xr[nstat + f] : 0.f;
    }
    wlv = xr[nstat - 1] + xr[a.c.nnf - 2];  // water level = bed elevation + depth
    MSW_MARK(c, 1);
    if constexpr (kStaged<NT>) {
      if (s != staged) {  // uniform across the workgroup: every wave walks the same chunks
        if (staged >= 0) __syncthreads();  // everyone is done with the old region
        stage_glds(smem, a.c.W, a.sreg[s], 0, a.sreg[s].len);
        __syncthreads();
        staged = s;
      }
    }
    // weight reads straight from the LDS pointer (not through c.W, which the compiler cannot
    // prove to be LDS across the loop: it emitted flat loads, which wait on vmcnt too)
    const float* Wl = kStaged<NT> ? (const float*)smem : c.W;
    if (DEC && dstep >= 0) {  // decode the previous step; the encoders read the updated state
      pre.step = dstep;
      bc_prefetch<NT>(pre, a.dec, c);
      float nd[kMaxDyn];
      decode_state<NT, ACT>(xu, a.dec, c, Wl, pre, n, valid, lane, g, nd);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 4 * g + r;
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < kMaxDyn; ++k) v = (k == f && f < c.dyn) ? nd[k] : v;
        dyn[r] = v;
      }
      float hn = 0.f;
#pragma unroll
      for (int k = 0; k < kMaxDyn; ++k) hn = (k == c.dyn - 2) ? nd[k] : hn;
      wlv = xr[nstat - 1] + hn;
    }
    if (DEC && a.decode_only) continue;
    MSW_MARK(c, 2);
    f32x4 xs[NT];
    {
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (c.with_wl && 4 * g + r == nstat) ? wlv : raw[r];
      const f32x4 in[1] = {v};
      run_mlp<1, NT, NT, ACT>(in, xs, a.stat, Wl, lane, g);
      if (valid) store_row<NT>(a.xs + (size_t)n * F, xs, NT, g);
    }
    MSW_MARK(c, 5);
    if (s == 0) {
      f32x4 xd[NT];
      const f32x4 in[1] = {f32x4{dyn[0], dyn[1], dyn[2], dyn[3]}};
      run_mlp<1, NT, NT, ACT>(in, xd, a.dynm, Wl, lane, g);
      if (valid && a.xd) store_row<NT>(a.xd + (size_t)n * F, xd, NT, g);
      MSW_MARK(c, 6);
      np_project<NT>(xs, xd, a.np0, Wl, n, valid, lane, g);
    }
    MSW_MARK(c, 8);
    if (a.vu_a[s] >= 0) side_proj<NT, NT>(xs, a.vu_h1t, Wl + a.vu_a[s], a.Vu, n, valid, lane, g);
  }
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- message passing
// One wave = one edge tile (whole destination neighbourhoods, <= 16 edges, <= 16 nodes).
// Lane j is edge slot j in the edge phase and destination j in the node phase; per-node
// rows the edges need (V, out at the destination) are loaded ONCE by the node lanes and
// handed to the edge lanes through the wave's LDS slab, the messages go back through the
// same slab (no atomics; every destination sums its messages in the reference's edge
// order).
struct Lanes {
  bool ev, nv;
  int dl, q0, q1;
  size_t sr, n;   // source row (edge lane) / destination row (node lane), safe rows if absent
  size_t p;       // tile-padded edge slot
};
__device__ __forceinline__ Lanes lanes_of(const LaneRec& r, int tile, int j, int n0) {
  Lanes L;
  L.ev = r.src >= 0;
  L.nv = r.n >= 0;
  L.dl = L.ev ? r.dl : 0;
  L.sr = (size_t)(L.ev ? r.src : n0);
  L.n = (size_t)(L.nv ? r.n : n0);
  L.q0 = r.q & 255;
  L.q1 = L.nv ? (r.q >> 8) : L.q0;
  L.p = (size_t)tile * kRowsPerWave + j;
  return L;
}
__device__ __forceinline__ LaneRec load_rec(const LaneRec* recs, int tile, int j) {
  const int4 v = reinterpret_cast<const int4*>(recs)[(size_t)tile * kRowsPerWave + j];
  return LaneRec{v.x, v.y, v.z, v.w};
}

// msg_e = active(e) * (out[col] - out[row]) * s_e  (or s_e * out[row])   (gnn.py:406-435)
template <int NT>
__device__ __forceinline__ void put_message(float* slab_row, const f32x4 (&os)[NT], const f32x4 (&od)[NT],
                                            const f32x4 (&sv)[NT], bool ev, int grad, int upwind, int g) {
#pragma clang fp contract(off)
  float rs = 0.f, rd = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    rs += hsum(os[t]);
    rd += hsum(od[t]);
  }
  const bool act = (row_sum(rs) != 0.f) || (row_sum(rd) != 0.f);  // gnn.py:408-411
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f32x4 gv;
    if (grad) {
      gv = od[t] - os[t];  // out[col] - out[row]
      if (upwind) {
        gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
        gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
      }
    } else {
      gv = os[t];          // s_ij * out[row]
    }
    const f32x4 m = gv * sv[t];
    st4(slab_row + 16 * t + 4 * g, (ev && act) ? m : zero4());
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
}

// Node phase: agg = sum of the node's messages (edge order).
template <int NT, int STRIDE>
__device__ __forceinline__ void gather_messages(f32x4 (&agg)[NT], const float* slab, int q0, int q1, int g) {
#pragma clang fp contract(off)
  wave_lds_sync();
#pragma unroll
  for (int t = 0; t < NT; ++t) agg[t] = zero4();
  for (int q = q0; q < q1; ++q) {
#pragma unroll
    for (int t = 0; t < NT; ++t) agg[t] = agg[t] + ld4(slab + q * STRIDE + 16 * t + 4 * g);
  }
}

// res += W agg (filter; agg is already in B-operand layout) or res += agg
template <int NT>
__device__ __forceinline__ void apply_filter(f32x4 (&res)[NT], const f32x4 (&agg)[NT], int filt_a,
                                             const float* W, int lane) {
#pragma clang fp contract(off)
  if (filt_a >= 0) {
    f32x4 acc[NT];
    proj<NT, NT>(agg, acc, W + filt_a, lane);
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = res[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = res[t] + agg[t];
  }
}

// Tile kernels: LOOP = false -> one tile per wave, the tile's HBM gathers issued before the
// weight staging (latency-bound meshes); LOOP = true -> grid capped at the resident
// workgroups, each stages its weight region ONCE and walks tiles grid-stride (large
// meshes).  In the loop the lane id is made opaque per iteration so that the compiler does
// not hoist every lane-derived weight address out of the loop (it pinned ~55 VGPRs).
__device__ __forceinline__ int opaque_lane() {
  int ln = (int)(threadIdx.x & 63);
  asm volatile("" : "+v"(ln));
  return ln;
}

// Filter A operand straight from the blob into registers (small: NT x NT tiles), issued at
// kernel start; apply_filter_regs = apply_filter with the operand already in registers.
template <int NT>
__device__ __forceinline__ void load_filter(f32x4 (&wf)[NT][NT], const float* W, int filt_a, int lane) {
  const int fa = filt_a >= 0 ? filt_a : 0;  // unconditional (unused without a filter)
#pragma unroll
  for (int to = 0; to < NT; ++to)
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) wf[to][ti] = ld4(W + fa + ((size_t)(to * NT + ti) * 64 + lane) * 4);
}
template <int NT>
__device__ __forceinline__ void apply_filter_regs(f32x4 (&res)[NT], const f32x4 (&agg)[NT], int filt_a,
                                                  const f32x4 (&wf)[NT][NT]) {
#pragma clang fp contract(off)
  if (filt_a >= 0) {
    f32x4 acc[NT];
#pragma unroll
    for (int to = 0; to < NT; ++to) acc[to] = zero4();
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int to = 0; to < NT; ++to) acc[to] = MSW_MFMA(wf[to][ti][r], agg[ti][r], acc[to]);
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = res[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = res[t] + agg[t];
  }
}

// ---------------------------------------------------------------------------- edge MLP + hop 1
//  edges: s_ij = normalize(MLP(x_s[row], x_s[col], x_d[row], x_d[col], e_ij))
//         (gnn.py:414-426; first layer pre-split: h1 = act(U[row] + V[col] + Pe[e]));
//         computed ONCE per layer -- its inputs do not change across the K hops.
//  nodes: out_1 = out_0 + W_1 agg [+ skip] -> store, or the epilogue when K = 1.
template <int NT>
struct EdgeHopRows {  // everything one tile reads from HBM
  Lanes L;
  f32x4 Us[2 * NT], Ps[2 * NT], Vn[2 * NT], os[NT], inn[NT], sk[NT];
  EpiPre<NT> pre;  // a.last only
};
// LST = 0: the launch never runs an epilogue (compiled out: fewer live scalars, no SGPR
// spills into VGPR lanes in the grid-stride loop); LST = 1: a.last decides.
template <int NT, int LST>
__device__ __forceinline__ void edge_hop_gather(EdgeHopRows<NT>& r, const EdgeHopArgs& a, const LaneRec& rec,
                                                int tile, int j, int g) {
  constexpr int F = 16 * NT, T2 = 2 * NT;
  r.L = lanes_of(rec, tile, j, a.n0);
  const Lanes& L = r.L;
  const int hs = 16 * a.h1t;
  const float* z = a.c.zrow;
  const float* Ub = a.U + L.sr * hs;
  const float* Vb = a.V + L.n * hs;
  const float* Pb = a.Pe ? a.Pe + L.p * hs : z;
#pragma unroll
  for (int t = 0; t < T2; ++t) {  // unconditional loads, tiles past h1t read zeros
    const int off = 16 * t + 4 * g;
    const bool on = t < a.h1t;
    r.Us[t] = ld4((on ? Ub : z) + off);
    r.Vn[t] = ld4((on ? Vb : z) + off);
    r.Ps[t] = ld4((on ? Pb : z) + off);
  }
  load_row<NT>(r.os, a.in + L.sr * F, g);
  load_row<NT>(r.inn, a.own_zero ? z : a.in + L.n * F, g);
  load_row<NT>(r.sk, a.skip ? a.skip + L.n * F : z, g);
  if (LST && a.last) epi_prefetch<NT>(r.pre, a.epi, a.c, a.xs, L.n, g);
}
template <int NT, int LST>
__device__ __forceinline__ void edge_hop_load(EdgeHopRows<NT>& r, const EdgeHopArgs& a, int tile, int j, int g) {
  edge_hop_gather<NT, LST>(r, a, load_rec(a.recs, tile, j), tile, j, g);
}
// Wm: the MLP operands (b1, layers 2..L) -- the staged region; c.W: everything else (the
// same region for F <= 32, the blob for F = 64, whose epilogue operands do not fit in LDS).
template <int NT, int ACT, int XS, bool FREG = true>
__device__ __forceinline__ void edge_hop_core(const EdgeHopRows<NT>& r, const EdgeHopArgs& a, const Common& c,
                                              const float* Wm, const f32x4 (&wf)[NT][NT], float* slab, int j,
                                              int lane, int g, f32x4 (&res_out)[NT]) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, T2 = 2 * NT;
  const Lanes& L = r.L;
  // node rows -> edge lanes
  float* my = slab + j * XS;
  store_row<T2>(my, r.Vn, T2, g);
  store_row<NT>(my + 16 * T2, r.inn, NT, g);
  wave_lds_sync();
  const float* dr = slab + L.dl * XS;
  f32x4 H[T2], od[NT];
  // unconditional LDS reads + selects: reads under the run-time h1t / Pe flags compiled to
  // a branch and an lgkmcnt(0) wait per tile
  const int b1 = a.b1_off >= 0 ? a.b1_off : 0;
  f32x4 vr[T2], br[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int off = 16 * t + 4 * g;
    vr[t] = ld4(dr + off);
    br[t] = ld4(Wm + b1 + off);
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const f32x4 p = a.Pe ? r.Ps[t] : br[t];
    H[t] = (t < a.h1t) ? (r.Us[t] + vr[t]) + p : zero4();
  }
  load_row<NT>(od, dr + 16 * T2, g);
  MSW_MARK(c, 4);
  act_tiles<ACT, T2>(H, a.act1, a.slope1);
  f32x4 sv[NT];
  if (a.rest.n > 0) {
    run_mlp<T2, T2, NT, ACT>(H, sv, a.rest, Wm, lane, g);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) sv[t] = H[t];
  }
  MSW_MARK(c, 5);
  if (a.normalize) {
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) ss += hsum(sv[t] * sv[t]);
    const float nrm = sqrtf(row_sum(ss));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 q = sv[t] / nrm;
      q.x = (q.x == q.x) ? q.x : 0.f;  // masked_fill_(isnan, 0)
      q.y = (q.y == q.y) ? q.y : 0.f;
      q.z = (q.z == q.z) ? q.z : 0.f;
      q.w = (q.w == q.w) ? q.w : 0.f;
      sv[t] = q;
    }
  }
  if (a.s) store_row<NT>(a.s + L.p * F, sv, NT, g);  // padding slots too: never read
  put_message<NT>(my, r.os, od, sv, L.ev, a.grad, a.upwind, g);  // the slab row is free again
  MSW_MARK(c, 6);
  f32x4 agg[NT], res[NT];
  gather_messages<NT, XS>(agg, slab, L.q0, L.q1, g);
  MSW_MARK(c, 7);
#pragma unroll
  for (int t = 0; t < NT; ++t) res[t] = r.inn[t];
  if constexpr (FREG)
    apply_filter_regs<NT>(res, agg, a.filt_a, wf);
  else  // filter operand in the staged LDS region (fewer live registers in the loop)
    apply_filter<NT>(res, agg, a.filt_l, c.W, lane);
  MSW_MARK(c, 8);
  if (a.skip) {
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = res[t] + r.sk[t];
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) res_out[t] = res[t];
}
template <int NT, int ACT, int LST>
__device__ __forceinline__ void edge_hop_finish(f32x4 (&res)[NT], const EdgeHopRows<NT>& r, const EdgeHopArgs& a,
                                                const Common& c, int lane, int g) {
  constexpr int F = 16 * NT;
  const Lanes& L = r.L;
  if (LST && a.last) {
    node_epilogue<NT, ACT>(res, a.epi, c, r.pre, a.out, L.n, L.nv, lane, g);
  } else if (L.nv && a.out) {
    store_row<NT>(a.out + L.n * F, res, NT, g);
  }
}
template <int NT, int ACT, bool LOOP, int LST>
__global__ __launch_bounds__((64 * edge_waves<NT, LOOP, LST>())) __attribute__((amdgpu_waves_per_eu(edge_eu<NT, LOOP, LST>())))
void k_edge_hop(EdgeHopArgs a) {
  constexpr int WV = edge_waves<NT, LOOP, LST>();
  // slab row: V | out, +4 floats so the 16 rows of a b128 access hit distinct LDS banks
  constexpr int XS = 16 * 2 * NT + 16 * NT + 4;
  __shared__ __attribute__((aligned(16))) float slab[WV][kRowsPerWave][XS];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int stride = gridDim.x * WV;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  int tile = xb * WV + w;
  Common c = a.c;
  MSW_MARK(c, 0);
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  f32x4 wf[NT][NT];
  if constexpr (!LOOP || !kStaged<NT>)
    load_filter<NT>(wf, a.c.W, a.filt_a, lane);  // blob offset (not part of the LDS region)
  if constexpr (!LOOP) {
    const bool live = tile < a.ntiles;
    EdgeHopRows<NT> r;
    edge_hop_load<NT, LST>(r, a, live ? tile : 0, j, g);  // idle waves stay in bounds
    MSW_MARK(c, 1);
    // weights the MLP needs now; the epilogue's operands (unpool / K = 1 projections)
    // stream into LDS behind the MLP and are waited for at the epilogue barrier
    const bool split = kStaged<NT> && a.reg.split < a.reg_nf;
    const float* Wm = c.W;
    if constexpr (kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.split);
      __syncthreads();
      c.W = smem;
      Wm = smem;
      if (split) stage_glds<WV>(smem, a.c.W, a.reg, chunk_ceil(a.reg.split), a.reg_nf);
    } else if (a.reg.len > 0) {  // F = 64: the MLP region alone (plan.hip relocate)
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      Wm = smem;
    }
    MSW_MARK(c, 2);
    f32x4 res[NT];
    if (live) edge_hop_core<NT, ACT, XS>(r, a, c, Wm, wf, &slab[w][0][0], j, lane, g, res);
    if (split) __syncthreads();  // every wave: the epilogue operands have landed
    if (live) edge_hop_finish<NT, ACT, LST>(res, r, a, c, lane, g);
  } else {
    const float* Wm = c.W;
    if constexpr (kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      c.W = smem;
      Wm = smem;
    } else if (a.reg.len > 0) {  // F = 64: the MLP region alone
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      Wm = smem;
    }
    for (; tile < a.ntiles; tile += stride) {
      const int ln = opaque_lane(), gg = ln >> 4, jj = ln & 15;
      EdgeHopRows<NT> q;
      edge_hop_load<NT, LST>(q, a, tile, jj, gg);
      f32x4 res[NT];
      edge_hop_core<NT, ACT, XS, !kStaged<NT>>(q, a, c, Wm, wf, &slab[w][0][0], jj, ln, gg, res);
      edge_hop_finish<NT, ACT, LST>(res, q, a, c, ln, gg);
    }
  }
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- edge MLP alone
// F = 64 scales whose edge tiles exceed one round of the fused kernel (plan.hip sched_proc,
// MSW_SPLIT_EDGE_MLP): the edge MLP of a layer's first hop on its own, s for every edge;
// hop 1 then runs as a k_hop launch.  Without the hop state (source / own rows, filter,
// node -> edge slab) the kernel fits two waves per SIMD where the fused kernel runs one, and
// it needs no whole neighbourhoods: it walks dense chunks of 16 real edges (EdgeChunk), so
// the last partly filled round of the tile order disappears (zenodo4: 2,050 tiles on 1,024
// fused waves = three rounds; 1,927 chunks on 2,048 waves = one).  The arithmetic is
// edge_hop_core's, operation for operation: s is bit-identical.
constexpr int kMlpWaves = 8;
template <int NT, int ACT>
__global__ __launch_bounds__(64 * kMlpWaves) __attribute__((amdgpu_waves_per_eu(2)))
void k_edge_mlp(EdgeHopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, T2 = 2 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = wave_id();
  const int stride = gridDim.x * kMlpWaves;
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  const float* Wm = a.c.W;
  if (a.reg.len > 0) {
    stage_glds<kMlpWaves>(smem, a.c.W, a.reg, 0, a.reg.len);
    __syncthreads();
    Wm = smem;
  }
  const int hs = 16 * a.h1t;
  const float* z = a.c.zrow;
  const int b1 = a.b1_off >= 0 ? a.b1_off : 0;
  for (int ch = blockIdx.x * kMlpWaves + w; ch < a.nchunks; ch += stride) {
    const int ln = opaque_lane(), g = ln >> 4, j = ln & 15;
    const int4 e = reinterpret_cast<const int4*>(a.chunks)[(size_t)ch * kRowsPerWave + j];
    const bool ev = e.z >= 0;
    const float* Ub = a.U + (size_t)(ev ? e.x : a.n0) * hs;
    const float* Vb = a.V + (size_t)(ev ? e.y : a.n0) * hs;
    const float* Pb = a.Pe && ev ? a.Pe + (size_t)e.z * hs : z;
    f32x4 H[T2];
#pragma unroll
    for (int t = 0; t < T2; ++t) {  // unconditional loads, tiles past h1t read zeros
      const int off = 16 * t + 4 * g;
      const bool on = t < a.h1t;
      const f32x4 u = ld4((on ? Ub : z) + off);
      const f32x4 v = ld4((on ? Vb : z) + off);
      const f32x4 pe = ld4((on ? Pb : z) + off);
      const f32x4 p = a.Pe ? pe : ld4(Wm + b1 + off);
      H[t] = on ? (u + v) + p : zero4();
    }
    act_tiles<ACT, T2>(H, a.act1, a.slope1);
    f32x4 sv[NT];
    if (a.rest.n > 0) {
      run_mlp<T2, T2, NT, ACT>(H, sv, a.rest, Wm, ln, g);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) sv[t] = H[t];
    }
    if (a.normalize) {
      float ss = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) ss += hsum(sv[t] * sv[t]);
      const float nrm = sqrtf(row_sum(ss));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 q = sv[t] / nrm;
        q.x = (q.x == q.x) ? q.x : 0.f;  // masked_fill_(isnan, 0)
        q.y = (q.y == q.y) ? q.y : 0.f;
        q.z = (q.z == q.z) ? q.z : 0.f;
        q.w = (q.w == q.w) ? q.w : 0.f;
        sv[t] = q;
      }
    }
    if (ev) store_row<NT>(a.s + (size_t)e.z * F, sv, NT, g);
  }
}

// k_edge_mlp software-pipelined (F = 64, MSW_MLP_PIPE): one wave per SIMD, each wave walks
// ~2 chunks and issues the next chunk's U / V / Pe gathers (1.5 KB per edge) before the
// current chunk's MLP (384 MFMAs), so the gathers of chunk n+1 run under the MFMA chain of
// chunk n instead of every wave of the launch gathering, then multiplying, in lockstep.  Same
// operations on the same operands as k_edge_mlp: s is bit-identical.
constexpr int kMlpPipeWaves = 4;
template <int NT>
struct MlpFetch {
  f32x4 u[2 * NT], v[2 * NT], p[2 * NT];
  int4 e;
};
template <int NT>
__device__ __forceinline__ void mlp_fetch(MlpFetch<NT>& f, const EdgeHopArgs& a, int ch, int j, int g) {
  constexpr int T2 = 2 * NT;
  const int hs = 16 * a.h1t;
  const float* z = a.c.zrow;
  f.e = reinterpret_cast<const int4*>(a.chunks)[(size_t)ch * kRowsPerWave + j];
  const bool ev = f.e.z >= 0;
  const float* Ub = a.U + (size_t)(ev ? f.e.x : a.n0) * hs;
  const float* Vb = a.V + (size_t)(ev ? f.e.y : a.n0) * hs;
  const float* Pb = a.Pe && ev ? a.Pe + (size_t)f.e.z * hs : z;
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int off = 16 * t + 4 * g;
    const bool on = t < a.h1t;
    f.u[t] = ld4((on ? Ub : z) + off);
    f.v[t] = ld4((on ? Vb : z) + off);
    f.p[t] = ld4((on ? Pb : z) + off);
  }
}
template <int NT, int ACT>
__global__ __launch_bounds__(64 * kMlpPipeWaves) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_edge_mlp_pipe(EdgeHopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, T2 = 2 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = wave_id();
  const int stride = gridDim.x * kMlpPipeWaves;
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  const int ln = opaque_lane(), g = ln >> 4, j = ln & 15;
  int ch = blockIdx.x * kMlpPipeWaves + w;
  MlpFetch<NT> f;
  if (ch < a.nchunks) mlp_fetch<NT>(f, a, ch, j, g);  // in flight during the weight staging
  const float* Wm = a.c.W;
  if (a.reg.len > 0) {
    stage_glds<kMlpPipeWaves>(smem, a.c.W, a.reg, 0, a.reg.len);
    __syncthreads();
    Wm = smem;
  }
  const int b1 = a.b1_off >= 0 ? a.b1_off : 0;
  for (; ch < a.nchunks; ch += stride) {
    f32x4 H[T2];
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      const f32x4 p = a.Pe ? f.p[t] : ld4(Wm + b1 + 16 * t + 4 * g);
      H[t] = t < a.h1t ? (f.u[t] + f.v[t]) + p : zero4();
    }
    const int4 e = f.e;
    if (ch + stride < a.nchunks) mlp_fetch<NT>(f, a, ch + stride, j, g);
    act_tiles<ACT, T2>(H, a.act1, a.slope1);
    f32x4 sv[NT];
    if (a.rest.n > 0) {
      run_mlp<T2, T2, NT, ACT>(H, sv, a.rest, Wm, ln, g);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) sv[t] = H[t];
    }
    if (a.normalize) {
      float ss = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) ss += hsum(sv[t] * sv[t]);
      const float nrm = sqrtf(row_sum(ss));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 q = sv[t] / nrm;
        q.x = (q.x == q.x) ? q.x : 0.f;  // masked_fill_(isnan, 0)
        q.y = (q.y == q.y) ? q.y : 0.f;
        q.z = (q.z == q.z) ? q.z : 0.f;
        q.w = (q.w == q.w) ? q.w : 0.f;
        sv[t] = q;
      }
    }
    if (e.z >= 0) store_row<NT>(a.s + (size_t)e.z * F, sv, NT, g);
  }
}

// ---------------------------------------------------------------------------- cooperative edge hop
// The fused edge MLP + hop with P waves per tile, for scales whose tiles are far fewer than
// the chip's SIMDs (the MLP chain of one wave is then the launch's critical path): every
// wave of a tile group loads the tile and does the (cheap) VALU / LDS work itself; the MFMA
// work -- each MLP layer, the filter, the epilogue projections -- is split by output tile,
// rank r computing tiles [r T/P, (r+1) T/P), the parts exchanged through LDS.  Same
// operations on the same operands as k_edge_hop (every output element is one MFMA chain
// in k order either way): bit-identical results.
// a[k TS + t] for the rank's k, with compile-time register indices (a run-time index into a
// register array would move it to scratch)
template <int N, int TS>
__device__ __forceinline__ f32x4 pick(const f32x4 (&a)[N], int r, int t) {
  f32x4 v = a[t];
#pragma unroll
  for (int k = 1; k < N / TS; ++k) v = (r == k) ? a[k * TS + t] : v;
  return v;
}
template <int T, int P>
__device__ __forceinline__ void coop_exchange(const f32x4* sub, f32x4 (&full)[T], float* buf, int xw, int r,
                                              int j, int g) {
  constexpr int TS = T / P;
#pragma unroll
  for (int t = 0; t < TS; ++t) st4(buf + j * xw + 16 * (r * TS + t) + 4 * g, sub[t]);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < T; ++t) full[t] = ld4(buf + j * xw + 16 * t + 4 * g);
}
// nn.Linear + bias + activation on output tiles [to0, to0 + TS) of a TIN -> T layer
template <int TIN, int TS, int ACT>
__device__ __forceinline__ void mfma_layer_sub(const f32x4 (&in)[TIN], f32x4 (&out)[TS], const LayerDev& L,
                                               const float* __restrict__ W, int to0, int lane, int g) {
  f32x4 acc[TS];
  proj<TIN, TS>(in, acc, W + L.a_off + (size_t)to0 * TIN * 256, lane);
#pragma unroll
  for (int to = 0; to < TS; ++to) acc[to] = acc[to] + ld4(W + L.b_off + 16 * (to0 + to) + 4 * g);
  act_tiles<ACT, TS>(acc, L.act, L.slope);
#pragma unroll
  for (int to = 0; to < TS; ++to) out[to] = acc[to];
}
// run_mlp with each layer's output tiles split over the P ranks; buffers alternate per layer
template <int IN0, int T, int TL, int ACT, int P>
__device__ __forceinline__ void coop_run_mlp(const f32x4 (&in)[IN0], f32x4 (&out)[TL], const MlpDev& m,
                                             const float* __restrict__ W, int lane, int g, int j, int r,
                                             float* buf0, float* buf1, int xw) {
  if (m.n == 1) {
    f32x4 o[TL / P];
    mfma_layer_sub<IN0, TL / P, ACT>(in, o, m.l[0], W, r * (TL / P), lane, g);
    coop_exchange<TL, P>(o, out, buf0, xw, r, j, g);
    return;
  }
  f32x4 h[T];
  {
    f32x4 o[T / P];
    mfma_layer_sub<IN0, T / P, ACT>(in, o, m.l[0], W, r * (T / P), lane, g);
    coop_exchange<T, P>(o, h, buf0, xw, r, j, g);
  }
  for (int li = 1; li + 1 < m.n; ++li) {
    f32x4 o[T / P];
    mfma_layer_sub<T, T / P, ACT>(h, o, m.l[li], W, r * (T / P), lane, g);
    coop_exchange<T, P>(o, h, (li & 1) ? buf1 : buf0, xw, r, j, g);
  }
  f32x4 o[TL / P];
  mfma_layer_sub<T, TL / P, ACT>(h, o, m.l[m.n - 1], W, r * (TL / P), lane, g);
  coop_exchange<TL, P>(o, out, ((m.n - 1) & 1) ? buf1 : buf0, xw, r, j, g);
}
// np_project with the output tiles of U, V and O split over the ranks (each stores its part)
template <int TIN, int TS>
__device__ __forceinline__ void proj_store_part(const f32x4 (&in)[TIN], const float* A, int r, float* dst, size_t n,
                                                int ntl, bool valid, int lane, int g) {
  f32x4 acc[TS];
  proj<TIN, TS>(in, acc, A + (size_t)r * TS * TIN * 256, lane);
  if (valid) {
#pragma unroll
    for (int t = 0; t < TS; ++t) st4(dst + n * (16 * ntl) + 16 * (r * TS + t) + 4 * g, acc[t]);
  }
}
template <int NT, int H1T, int P>
__device__ __forceinline__ void np_project_coop(const f32x4 (&xs)[NT], const f32x4 (&xin)[NT], const NpDesc& d,
                                                const float* W, size_t n, bool valid, int r, int lane, int g) {
  constexpr int T2 = 2 * NT;
  f32x4 in[T2];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    in[t] = xs[t];
    in[NT + t] = xin[t];
  }
  if (d.a_u >= 0) proj_store_part<T2, H1T / P>(in, W + d.a_u, r, d.U, n, H1T, valid, lane, g);
  if (d.a_v >= 0) proj_store_part<T2, H1T / P>(in, W + d.a_v, r, d.V, n, H1T, valid, lane, g);
  if constexpr (P <= NT) {
    if (d.a_o >= 0) proj_store_part<NT, NT / P>(xin, W + d.a_o, r, d.O, n, NT, valid, lane, g);
  } else {  // more ranks than O tiles: ranks 0..NT-1 take one O tile each
    if (d.a_o >= 0 && r < NT) proj_store_part<NT, 1>(xin, W + d.a_o, r, d.O, n, NT, valid, lane, g);
  }
}

// ---- pooling fused into the coarse scale's first edge-MLP + hop (EdgeHopArgs::pool)
// The tile's two ranks split the pooling: rank 0 forms the SOURCE side of its edge lanes
// (mean of the source's children, U and O = out_0 of the source), rank 1 the DESTINATION side
// of its node lanes (V and O of the destination) -- each loads only its side's children.
template <int NT>
struct PoolIn {
  f32x4 c[kPoolInline][NT];  // children rows of this rank's node (absent ones: a real row)
  f32x4 xs[NT];              // x_s of that node
  int cnt, off;              // child count, offset into PoolFuse::child
};
// edge_hop_gather with U / V / out rows replaced by the pooling inputs (issued before the
// weight staging, like every tile load); rank r: 0 = source side, 1 = destination side
template <int NT, int LST>
__device__ __forceinline__ void edge_pool_load(EdgeHopRows<NT>& r, PoolIn<NT>& pi, const EdgeHopArgs& a, int tile,
                                               int j, int g, int rank) {
  constexpr int F = 16 * NT, T2 = 2 * NT;
  const LaneRec rec = load_rec(a.recs, tile, j);
  const int4* sp = reinterpret_cast<const int4*>(a.pool.slots + (size_t)tile * kRowsPerWave + j) + (rank ? 2 : 0);
  const int4 r0 = sp[0], r1 = sp[1];
  r.L = lanes_of(rec, tile, j, a.n0);
  const Lanes& L = r.L;
  const int hs = 16 * a.h1t;
  const float* z = a.c.zrow;
  const float* Pb = a.Pe ? a.Pe + L.p * hs : z;
#pragma unroll
  for (int t = 0; t < T2; ++t) r.Ps[t] = ld4((t < a.h1t ? Pb : z) + 16 * t + 4 * g);
  const int ci[kPoolInline] = {r0.x, r0.y, r0.z, r0.w};
#pragma unroll
  for (int k = 0; k < kPoolInline; ++k) load_row<NT>(pi.c[k], a.pool.in + (size_t)ci[k] * F, g);
  pi.cnt = r1.x; pi.off = r1.y;
  load_row<NT>(pi.xs, a.xs + (rank ? L.n : L.sr) * F, g);
  load_row<NT>(r.sk, a.skip ? a.skip + L.n * F : z, g);
  if (LST && a.last) epi_prefetch<NT>(r.pre, a.epi, a.c, a.xs, L.n, g);
}
// mean of the children (k_pool / k_pool_edge: summed from zero in reference order, divided
// by max(count, 1)) -- the same operations, so the same bits
template <int NT>
__device__ __forceinline__ void pool_mean(f32x4 (&m)[NT], const PoolIn<NT>& pi, const EdgeHopArgs& a, int g) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
#pragma unroll
  for (int t = 0; t < NT; ++t) m[t] = zero4();
#pragma unroll
  for (int k = 0; k < kPoolInline; ++k)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 s2 = m[t] + pi.c[k][t];
      m[t] = k < pi.cnt ? s2 : m[t];
    }
  for (int k = kPoolInline; k < pi.cnt; ++k) {
    f32x4 y[NT];
    load_row<NT>(y, a.pool.in + (size_t)a.pool.child[pi.off + k] * F, g);
#pragma unroll
    for (int t = 0; t < NT; ++t) m[t] = m[t] + y[t];
  }
  const float fc = (float)(pi.cnt > 0 ? pi.cnt : 1);
#pragma unroll
  for (int t = 0; t < NT; ++t) m[t] = m[t] / fc;
}
// np_project's proj calls on the pooled row: h = U (rank 0) or V (rank 1) of [x_s; x], o = O x
// (out_0; x itself without a filter matrix)
template <int NT, int H1T>
__device__ __forceinline__ void pool_project_t(f32x4 (&h)[2 * NT], f32x4 (&o)[NT], const f32x4 (&xp)[NT],
                                               const f32x4 (&xs)[NT], const NpDesc& d, const float* W, int lane,
                                               int rank) {
  constexpr int T2 = 2 * NT;
  f32x4 in[T2], acc[H1T];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    in[t] = xs[t];
    in[NT + t] = xp[t];
  }
  proj<T2, H1T>(in, acc, W + (rank ? d.a_v : d.a_u), lane);
#pragma unroll
  for (int t = 0; t < T2; ++t) h[t] = t < H1T ? acc[t < H1T ? t : 0] : zero4();
  if (d.a_o >= 0) {
    proj<NT, NT>(xp, o, W + d.a_o, lane);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) o[t] = xp[t];
  }
}
// rank 0 -> (q.Us, q.os) of its edge lanes, rank 1 -> (q.Vn, q.inn) of its node lanes, from
// the side's row xp and its x_s; then rank 0 publishes U | O rows in pb, rank 1 V | O rows in
// both ranks' slabs (XS-strided, edge_hop_core's node-row layout); after the barrier each
// rank reads the other side back.
template <int NT, int XS>
__device__ __forceinline__ void side_project_exchange(EdgeHopRows<NT>& q, const f32x4 (&xp)[NT], const f32x4 (&xs)[NT],
                                                      const NpDesc& np, const float* W, int lane, int g, int j,
                                                      int rank, float* pb, float* slab0, float* slab1) {
  constexpr int T2 = 2 * NT;
  f32x4 h[T2], o[NT];
  if (np.h1t == T2)
    pool_project_t<NT, T2>(h, o, xp, xs, np, W, lane, rank);
  else
    pool_project_t<NT, NT>(h, o, xp, xs, np, W, lane, rank);
  if (rank == 0) {
    store_row<T2>(pb + j * XS, h, T2, g);
    store_row<NT>(pb + j * XS + 16 * T2, o, NT, g);
  } else {
    store_row<T2>(slab0 + j * XS, h, T2, g);
    store_row<NT>(slab0 + j * XS + 16 * T2, o, NT, g);
    store_row<T2>(slab1 + j * XS, h, T2, g);
    store_row<NT>(slab1 + j * XS + 16 * T2, o, NT, g);
  }
  __syncthreads();
  if (rank == 0) {
#pragma unroll
    for (int t = 0; t < T2; ++t) q.Us[t] = h[t];
#pragma unroll
    for (int t = 0; t < NT; ++t) q.os[t] = o[t];
    load_row<NT>(q.inn, slab0 + j * XS + 16 * T2, g);
  } else {
    load_row<T2>(q.Us, pb + j * XS, g);
    load_row<NT>(q.os, pb + j * XS + 16 * T2, g);
#pragma unroll
    for (int t = 0; t < NT; ++t) q.inn[t] = o[t];
  }
}

// ---- the unpooling layer into this scale fused in (PoolFuse::parent): per side node v (the
// slot's source on rank 0, the lane's destination on rank 1) the intra-scale SWEGNN's one
// edge parent(v) -> v (gnn.py:323-331 with own rows zero, K = 1, no filter) + skip -- the
// unpooling launch's operations in its order (k_edge_coop / k_edge_hop, LST epilogue)
template <int NT>
struct UnpoolIn {
  f32x4 uc[2 * NT], vv[2 * NT];  // unpool U of the parent, unpool V of v
  f32x4 xc[NT], sk[NT], xs[NT];  // the parent's out_0 (x_up), v's skip row, v's x_s
  bool ev;                       // v has a parent
};
template <int NT, int LST>
__device__ __forceinline__ void edge_unpool_load(EdgeHopRows<NT>& r, UnpoolIn<NT>& u, const EdgeHopArgs& a, int tile,
                                                 int j, int g, int rank) {
  constexpr int F = 16 * NT, T2 = 2 * NT;
  const PoolFuse& d = a.pool;
  const LaneRec rec = load_rec(a.recs, tile, j);
  const int2 pp = d.parent[(size_t)tile * kRowsPerWave + j];
  r.L = lanes_of(rec, tile, j, a.n0);
  const Lanes& L = r.L;
  const float* z = a.c.zrow;
  {
    const int hs = 16 * a.h1t;
    const float* Pb = a.Pe ? a.Pe + L.p * hs : z;
#pragma unroll
    for (int t = 0; t < T2; ++t) r.Ps[t] = ld4((t < a.h1t ? Pb : z) + 16 * t + 4 * g);
  }
  const size_t v = rank ? L.n : L.sr;
  const int pc = rank ? pp.y : pp.x;
  u.ev = pc >= 0;
  const size_t c = (size_t)(pc >= 0 ? pc : d.cpad);
  const int hs = 16 * d.h1t;
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const bool on = t < d.h1t;
    u.uc[t] = ld4((on ? d.Uu + c * hs : z) + 16 * t + 4 * g);
    u.vv[t] = ld4((on ? d.Vu + v * hs : z) + 16 * t + 4 * g);
  }
  load_row<NT>(u.xc, d.xc + c * F, g);
  load_row<NT>(u.sk, d.skip ? d.skip + v * F : z, g);
  load_row<NT>(u.xs, a.xs + v * F, g);
  load_row<NT>(r.sk, a.skip ? a.skip + L.n * F : z, g);
  if (LST && a.last) epi_prefetch<NT>(r.pre, a.epi, a.c, a.xs, L.n, g);
}
template <int NT>
__device__ __forceinline__ void unpool_row(f32x4 (&res)[NT], const UnpoolIn<NT>& u, const EdgeHopArgs& a,
                                           const float* W, int lane, int g) {
#pragma clang fp contract(off)
  constexpr int T2 = 2 * NT;
  const PoolFuse& d = a.pool;
  f32x4 H[T2];
  const int b1 = d.b1_off >= 0 ? d.b1_off : 0;
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const f32x4 br = ld4(W + b1 + 16 * t + 4 * g);
    H[t] = (t < d.h1t) ? (u.uc[t] + u.vv[t]) + br : zero4();
  }
  act_tiles<-1, T2>(H, d.act1, d.slope1);
  f32x4 sv[NT];
  if (d.rest.n > 0) {
    run_mlp<T2, T2, NT, -1>(H, sv, d.rest, W, lane, g);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) sv[t] = H[t];
  }
  if (d.normalize) {
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) ss += hsum(sv[t] * sv[t]);
    const float nrm = sqrtf(row_sum(ss));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 q = sv[t] / nrm;
      q.x = (q.x == q.x) ? q.x : 0.f;  // masked_fill_(isnan, 0)
      q.y = (q.y == q.y) ? q.y : 0.f;
      q.z = (q.z == q.z) ? q.z : 0.f;
      q.w = (q.w == q.w) ? q.w : 0.f;
      sv[t] = q;
    }
  }
  // put_message with the destination's rows zero (own_zero), then its one-edge sum
  float rs = 0.f, rd = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    rs += hsum(u.xc[t]);
    rd += hsum(zero4());
  }
  const bool act = (row_sum(rs) != 0.f) || (row_sum(rd) != 0.f);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f32x4 gv;
    if (d.grad) {
      gv = zero4() - u.xc[t];
      if (d.upwind) {
        gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
        gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
      }
    } else {
      gv = u.xc[t];
    }
    const f32x4 m = gv * sv[t];
    const f32x4 agg = zero4() + ((u.ev && act) ? m : zero4());
    res[t] = (zero4() + agg) + u.sk[t];
  }
  if (d.post_act) act_tiles<-1, NT>(res, d.post_act, d.post_slope);
}

// FUSE: 0 plain, 1 pooling fused in (PoolFuse::slots), 2 unpooling fused in (PoolFuse::parent)
template <int NT, int ACT, int LST, int P, int FUSE = 0>
__global__ __launch_bounds__(64 * kWaves) void k_edge_coop(EdgeHopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, T2 = 2 * NT;
  constexpr int XS = 16 * 2 * NT + 16 * NT + 4;  // per-wave slab row, as k_edge_hop
  constexpr int XW = 16 * T2 + 4;                // exchange buffer row
  constexpr int G = kWaves / P;                  // tile groups per workgroup
  __shared__ __attribute__((aligned(16))) float slab_all[kWaves][kRowsPerWave][XS];
  __shared__ __attribute__((aligned(16))) float xbuf[G][2][kRowsPerWave][XW];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int grp = w / P, r = w % P;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  const int tile = xb * G + grp;
  const bool live = tile < a.ntiles;
  Common c = a.c;
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  f32x4 wf[NT][NT];
  load_filter<NT>(wf, a.c.W, a.filt_a, lane);
  EdgeHopRows<NT> q;
  [[maybe_unused]] PoolIn<NT> pin;
  [[maybe_unused]] UnpoolIn<NT> uin;
  if constexpr (FUSE == 1)
    edge_pool_load<NT, LST>(q, pin, a, live ? tile : 0, j, g, r);
  else if constexpr (FUSE == 2)
    edge_unpool_load<NT, LST>(q, uin, a, live ? tile : 0, j, g, r);
  else
    edge_hop_load<NT, LST>(q, a, live ? tile : 0, j, g);  // dead groups compute tile 0, store nothing
  const bool split = a.reg.split < a.reg_nf;
  stage_glds<kWaves>(smem, a.c.W, a.reg, 0, a.reg.split);
  __syncthreads();
  c.W = smem;
  if (split) stage_glds<kWaves>(smem, a.c.W, a.reg, chunk_ceil(a.reg.split), a.reg_nf);
  if constexpr (FUSE != 0) {
    static_assert(P == 2, "fused pooling / unpooling: a source rank and a destination rank");
    __shared__ __attribute__((aligned(16))) float pbuf[G][kRowsPerWave][XS];
    f32x4 xp[NT];
    if constexpr (FUSE == 1)
      pool_mean<NT>(xp, pin, a, g);
    else
      unpool_row<NT>(xp, uin, a, c.W, lane, g);
    side_project_exchange<NT, XS>(q, xp, FUSE == 1 ? pin.xs : uin.xs, a.pool.np, c.W, lane, g, j, r,
                                  &pbuf[grp][0][0], &slab_all[grp * P][0][0], &slab_all[grp * P + 1][0][0]);
  }
  float* slab = &slab_all[w][0][0];
  float* b0 = &xbuf[grp][0][0][0];
  float* b1p = &xbuf[grp][1][0][0];
  const Lanes& L = q.L;
  // ---- as edge_hop_core up to the MLP (every rank)
  float* my = slab + j * XS;
  if constexpr (FUSE == 0) {  // fused (un)pooling: the destination rank stored them (barrier above)
    store_row<T2>(my, q.Vn, T2, g);
    store_row<NT>(my + 16 * T2, q.inn, NT, g);
    wave_lds_sync();
  }
  const float* dr = slab + L.dl * XS;
  f32x4 H[T2], od[NT];
  const int b1 = a.b1_off >= 0 ? a.b1_off : 0;
  f32x4 vr[T2], br[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int off = 16 * t + 4 * g;
    vr[t] = ld4(dr + off);
    br[t] = ld4(c.W + b1 + off);
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const f32x4 p = a.Pe ? q.Ps[t] : br[t];
    H[t] = (t < a.h1t) ? (q.Us[t] + vr[t]) + p : zero4();
  }
  load_row<NT>(od, dr + 16 * T2, g);
  act_tiles<ACT, T2>(H, a.act1, a.slope1);
  f32x4 sv[NT];
  if (a.rest.n > 0) {
    coop_run_mlp<T2, T2, NT, ACT, P>(H, sv, a.rest, c.W, lane, g, j, r, b0, b1p, XW);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) sv[t] = H[t];
  }
  if (a.normalize) {
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) ss += hsum(sv[t] * sv[t]);
    const float nrm = sqrtf(row_sum(ss));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 v = sv[t] / nrm;
      v.x = (v.x == v.x) ? v.x : 0.f;  // masked_fill_(isnan, 0)
      v.y = (v.y == v.y) ? v.y : 0.f;
      v.z = (v.z == v.z) ? v.z : 0.f;
      v.w = (v.w == v.w) ? v.w : 0.f;
      sv[t] = v;
    }
  }
  if (live && r == 0 && a.s) store_row<NT>(a.s + L.p * F, sv, NT, g);
  put_message<NT>(my, q.os, od, sv, L.ev, a.grad, a.upwind, g);
  f32x4 agg[NT];
  gather_messages<NT, XS>(agg, slab, L.q0, L.q1, g);
  // ---- filter on this rank's output tiles, + skip, exchanged into the full row
  constexpr int TS = NT / P;
  f32x4 rs[TS];
#pragma unroll
  for (int t = 0; t < TS; ++t) rs[t] = pick<NT, TS>(q.inn, r, t);
  if (a.filt_a >= 0) {
    f32x4 wr[TS][NT];  // this rank's filter rows, selected with compile-time indices
#pragma unroll
    for (int to = 0; to < TS; ++to)
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) {
        f32x4 v = wf[to][ti];
#pragma unroll
        for (int k = 1; k < P; ++k) v = (r == k) ? wf[k * TS + to][ti] : v;
        wr[to][ti] = v;
      }
    f32x4 acc[TS];
#pragma unroll
    for (int to = 0; to < TS; ++to) acc[to] = zero4();
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int to = 0; to < TS; ++to) acc[to] = MSW_MFMA(wr[to][ti][rr], agg[ti][rr], acc[to]);
#pragma unroll
    for (int t = 0; t < TS; ++t) rs[t] = rs[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < TS; ++t) rs[t] = rs[t] + pick<NT, TS>(agg, r, t);
  }
  if (a.skip) {
#pragma unroll
    for (int t = 0; t < TS; ++t) rs[t] = rs[t] + pick<NT, TS>(q.sk, r, t);
  }
  f32x4 res[NT];
  // the buffer the MLP's last exchange did not use (its readers may still be reading that one)
  coop_exchange<NT, P>(rs, res, (a.rest.n & 1) ? b1p : b0, XW, r, j, g);
  if (split) __syncthreads();  // every wave: the epilogue operands have landed
  // ---- finish: store, or the epilogue (projections split over the ranks)
  if (LST && a.last) {
    const Epilogue& e = a.epi;
    if (e.post_act) act_tiles<-1, NT>(res, e.post_act, e.post_slope);
    if (live && r == 0 && a.out && L.nv) store_row<NT>(a.out + L.n * F, res, NT, g);
    if (e.np.h1t == T2)
      np_project_coop<NT, T2, P>(q.pre.xs, res, e.np, c.W, L.n, live && L.nv, r, lane, g);
    else
      np_project_coop<NT, NT, P>(q.pre.xs, res, e.np, c.W, L.n, live && L.nv, r, lane, g);
  } else if (live && r == 0 && L.nv && a.out) {
    store_row<NT>(a.out + L.n * F, res, NT, g);
  }
}

// Fused pooling on k_edge_coop4 (F = 64): ranks [0, P/2) form the source side, [P/2, P) the
// destination side; the P/2 ranks of a side split its U (V) and O output tiles.  dst_row: the
// lane's row [h (16 T2) | o (16 NT)] -- the exchange rows (source) or the node slab (destination).
template <int NT, int P, int H1T>
__device__ __forceinline__ void pool_project_part(float* dst_row, const f32x4 (&xp)[NT], const f32x4 (&xs)[NT],
                                                  const NpDesc& d, const float* W, int lane, int g, int side,
                                                  int part) {
  constexpr int NPART = P / 2, T2 = 2 * NT, TU = H1T / NPART, TO = NT / NPART;
  static_assert(H1T % NPART == 0 && NT % NPART == 0, "whole output tiles per rank");
  f32x4 in[T2], acc[TU];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    in[t] = xs[t];
    in[NT + t] = xp[t];
  }
  proj<T2, TU>(in, acc, W + (side ? d.a_v : d.a_u) + (size_t)part * TU * T2 * 256, lane);
#pragma unroll
  for (int t = 0; t < TU; ++t) st4(dst_row + 16 * (part * TU + t) + 4 * g, acc[t]);
  if (part == 0)
#pragma unroll
    for (int t = H1T; t < T2; ++t) st4(dst_row + 16 * t + 4 * g, zero4());  // U / V tiles past h1t
  f32x4 o[TO];
  if (d.a_o >= 0) {
    proj<NT, TO>(xp, o, W + d.a_o + (size_t)part * TO * NT * 256, lane);
  } else {
#pragma unroll
    for (int t = 0; t < TO; ++t) o[t] = pick<NT, TO>(xp, part, t);
  }
#pragma unroll
  for (int t = 0; t < TO; ++t) st4(dst_row + 16 * T2 + 16 * (part * TO + t) + 4 * g, o[t]);
}

// F = 64 (NT = 4): the whole workgroup (4 waves) on one tile, one slab shared by the four
// ranks (rank 0 writes the node rows and the messages) so that the 96 KB edge-MLP region
// still fits beside it; the epilogue's operands stay in the blob (F = 64 relocation).
// P = 2: two tiles per workgroup, two waves each (a slab and exchange buffers per tile);
// P = 4: the whole workgroup on one tile.
// FUSE: 0 plain, 1 pooling fused in (F = 64 keeps the unpooling launch: its 384-MFMA MLP per
// side costs more than the launch it saves, zenodo4_f64 -2.5 %, profiles/r03/ab_unpool_fuse_f64.txt)
template <int ACT, int LST, int P = 4, int FUSE = 0>
__global__ __launch_bounds__(64 * kWaves) void k_edge_coop4(EdgeHopArgs a) {
#pragma clang fp contract(off)
  static_assert(FUSE == 0 || FUSE == 1, "k_edge_coop4: plain or fused pooling");
  constexpr int NT = 4, F = 16 * NT, T2 = 2 * NT, G = kWaves / P, TS = NT / P;
  constexpr int XS = 16 * 2 * NT + 16 * NT + 4;
  constexpr int XW = 16 * T2 + 4;
  __shared__ __attribute__((aligned(16))) float slab_g[G][kRowsPerWave][XS];
  __shared__ __attribute__((aligned(16))) float xbuf_g[G][2][kRowsPerWave][XW];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int grp = w / P, r = w % P;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  const int tile0 = xb * G + grp;
  const bool live = tile0 < a.ntiles;  // dead groups compute tile 0 and store nothing
  const int tile = live ? tile0 : 0;
  float (&slab)[kRowsPerWave][XS] = slab_g[grp];
  float (&xbuf)[2][kRowsPerWave][XW] = xbuf_g[grp];
  Common c = a.c;  // c.W stays the blob: the epilogue reads it there
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  // this rank's filter rows (out tiles r TS .. r TS + TS - 1): wr[t][ti] = W_1 block (r TS + t, ti)
  f32x4 wr[TS][NT];
  {
    const int fa = a.filt_a >= 0 ? a.filt_a : 0;
#pragma unroll
    for (int t = 0; t < TS; ++t)
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) wr[t][ti] = ld4(c.W + fa + ((size_t)((r * TS + t) * NT + ti) * 64 + lane) * 4);
  }
  EdgeHopRows<NT> q;
  [[maybe_unused]] PoolIn<NT> pin;
  [[maybe_unused]] const int side = r >= P / 2;  // fused pooling: 0 source side, 1 destination side
  if constexpr (FUSE == 1)
    edge_pool_load<NT, LST>(q, pin, a, tile, j, g, side);
  else
    edge_hop_load<NT, LST>(q, a, tile, j, g);
  const Lanes& L = q.L;
  // the MLP region: staged in LDS, or (wdirect: two workgroups per CU) read from its blob copy
  if (a.reg.len > 0 && !a.wdirect) stage_glds<kWaves>(smem, c.W, a.reg, 0, a.reg.len);
  const float* Wm = a.reg.len > 0 ? (a.wdirect ? c.W + a.reg.off : (const float*)smem) : c.W;
  float* my = &slab[j][0];
  if constexpr (FUSE != 0) {
    // source side -> exchange rows (in xbuf, free until the MLP), destination side -> the
    // node slab; projection operands from the blob (c.W), its output tiles split over the
    // ranks of a side
    constexpr int XPB = 16 * T2 + 16 * NT + 4;
    static_assert(kRowsPerWave * XPB <= 2 * kRowsPerWave * XW, "exchange rows fit the xbuf pair");
    float* pb = &xbuf[0][0][0] + j * XPB;
    f32x4 xp[NT];
    pool_mean<NT>(xp, pin, a, g);
    const f32x4(&xsr)[NT] = pin.xs;
    if (a.pool.np.h1t == T2)
      pool_project_part<NT, P, T2>(side ? my : pb, xp, xsr, a.pool.np, c.W, lane, g, side, r % (P / 2));
    else
      pool_project_part<NT, P, NT>(side ? my : pb, xp, xsr, a.pool.np, c.W, lane, g, side, r % (P / 2));
    __syncthreads();
    load_row<T2>(q.Us, pb, g);
    load_row<NT>(q.os, pb + 16 * T2, g);
  } else if (r == 0) {
    store_row<T2>(my, q.Vn, T2, g);
    store_row<NT>(my + 16 * T2, q.inn, NT, g);
  }
  __syncthreads();  // node rows and the MLP region have landed (fused pooling: and every rank
                    // has read its exchange rows before the MLP's exchanges reuse xbuf)
  const float* dr = &slab[L.dl][0];
  f32x4 H[T2], od[NT];
  const int b1 = a.b1_off >= 0 ? a.b1_off : 0;
  f32x4 vr[T2], br[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int off = 16 * t + 4 * g;
    vr[t] = ld4(dr + off);
    br[t] = ld4(Wm + b1 + off);
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const f32x4 p = a.Pe ? q.Ps[t] : br[t];
    H[t] = (t < a.h1t) ? (q.Us[t] + vr[t]) + p : zero4();
  }
  load_row<NT>(od, dr + 16 * T2, g);
  act_tiles<ACT, T2>(H, a.act1, a.slope1);
  f32x4 sv[NT];
  if (a.rest.n > 0) {
    coop_run_mlp<T2, T2, NT, ACT, P>(H, sv, a.rest, Wm, lane, g, j, r, &xbuf[0][0][0], &xbuf[1][0][0], XW);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) sv[t] = H[t];
  }
  if (a.normalize) {
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) ss += hsum(sv[t] * sv[t]);
    const float nrm = sqrtf(row_sum(ss));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 v = sv[t] / nrm;
      v.x = (v.x == v.x) ? v.x : 0.f;  // masked_fill_(isnan, 0)
      v.y = (v.y == v.y) ? v.y : 0.f;
      v.z = (v.z == v.z) ? v.z : 0.f;
      v.w = (v.w == v.w) ? v.w : 0.f;
      sv[t] = v;
    }
  }
  if (live && r == 0 && a.s) store_row<NT>(a.s + L.p * F, sv, NT, g);
  // every rank has read the slab's node rows before the first MLP exchange barrier: rank 0
  // may overwrite them with the messages (a.rest.n == 0 has no barrier: add one)
  if (a.rest.n == 0) __syncthreads();
  if (r == 0) put_message<NT>(my, q.os, od, sv, L.ev, a.grad, a.upwind, g);
  __syncthreads();
  f32x4 agg[NT];
  gather_messages<NT, XS>(agg, &slab[0][0], L.q0, L.q1, g);
  // this rank's tile of inn / agg / skip by address (a 4-way select over a register array
  // was turned back into a scratch-indexed load): inn sits past the messages in the slab row
  f32x4 rs[TS];
#pragma unroll
  for (int t = 0; t < TS; ++t) rs[t] = ld4(&slab[j][16 * T2 + 16 * (r * TS + t) + 4 * g]);
  if (a.filt_a >= 0) {
    f32x4 acc[TS];
#pragma unroll
    for (int t = 0; t < TS; ++t) acc[t] = zero4();
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int t = 0; t < TS; ++t) acc[t] = MSW_MFMA(wr[t][ti][rr], agg[ti][rr], acc[t]);
#pragma unroll
    for (int t = 0; t < TS; ++t) rs[t] = rs[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < TS; ++t) {
      f32x4 ag = zero4();
      for (int qq = L.q0; qq < L.q1; ++qq) ag = ag + ld4(&slab[qq][16 * (r * TS + t) + 4 * g]);
      rs[t] = rs[t] + ag;
    }
  }
  if (a.skip) {
#pragma unroll
    for (int t = 0; t < TS; ++t) rs[t] = rs[t] + ld4(a.skip + L.n * F + 16 * (r * TS + t) + 4 * g);
  }
  f32x4 res[NT];
  coop_exchange<NT, P>(rs, res, (a.rest.n & 1) ? &xbuf[1][0][0] : &xbuf[0][0][0], XW, r, j, g);
  if (LST && a.last) {
    const Epilogue& e = a.epi;
    if (e.post_act) act_tiles<-1, NT>(res, e.post_act, e.post_slope);
    if (live && r == 0 && a.out && L.nv) store_row<NT>(a.out + L.n * F, res, NT, g);
    if (e.np.h1t == T2)
      np_project_coop<NT, T2, P>(q.pre.xs, res, e.np, c.W, L.n, L.nv && live, r, lane, g);
    else
      np_project_coop<NT, NT, P>(q.pre.xs, res, e.np, c.W, L.n, L.nv && live, r, lane, g);
  } else if (live && r == 0 && L.nv && a.out) {
    store_row<NT>(a.out + L.n * F, res, NT, g);
  }
}

template <int NT>
static const void* edge_coop_kernel(int prelu, int last, int pw = 0, int pool = 0) {
  if constexpr (NT == 2) {  // F = 32: each MLP layer's output tiles halve (F = 16 has one)
    if (pool == 1) {  // pooling fused in (EdgeHopArgs::pool)
      if (last) return prelu ? (const void*)k_edge_coop<NT, 1, 1, 2, 1> : (const void*)k_edge_coop<NT, -1, 1, 2, 1>;
      return prelu ? (const void*)k_edge_coop<NT, 1, 0, 2, 1> : (const void*)k_edge_coop<NT, -1, 0, 2, 1>;
    }
    if (pool == 2) {  // unpooling fused in
      if (last) return prelu ? (const void*)k_edge_coop<NT, 1, 1, 2, 2> : (const void*)k_edge_coop<NT, -1, 1, 2, 2>;
      return prelu ? (const void*)k_edge_coop<NT, 1, 0, 2, 2> : (const void*)k_edge_coop<NT, -1, 0, 2, 2>;
    }
    if (last) return prelu ? (const void*)k_edge_coop<NT, 1, 1, 2> : (const void*)k_edge_coop<NT, -1, 1, 2>;
    return prelu ? (const void*)k_edge_coop<NT, 1, 0, 2> : (const void*)k_edge_coop<NT, -1, 0, 2>;
  } else if constexpr (NT == 4) {  // F = 64: four waves per tile (pw = 2: two)
    if (pool == 1) {  // pooling fused in (EdgeHopArgs::pool)
      if (pw == 2) {
        if (last) return prelu ? (const void*)k_edge_coop4<1, 1, 2, 1> : (const void*)k_edge_coop4<-1, 1, 2, 1>;
        return prelu ? (const void*)k_edge_coop4<1, 0, 2, 1> : (const void*)k_edge_coop4<-1, 0, 2, 1>;
      }
      if (last) return prelu ? (const void*)k_edge_coop4<1, 1, 4, 1> : (const void*)k_edge_coop4<-1, 1, 4, 1>;
      return prelu ? (const void*)k_edge_coop4<1, 0, 4, 1> : (const void*)k_edge_coop4<-1, 0, 4, 1>;
    }
    if (pool == 2) return nullptr;  // F = 64 keeps the unpooling launch
    if (pw == 2) {
      if (last) return prelu ? (const void*)k_edge_coop4<1, 1, 2> : (const void*)k_edge_coop4<-1, 1, 2>;
      return prelu ? (const void*)k_edge_coop4<1, 0, 2> : (const void*)k_edge_coop4<-1, 0, 2>;
    }
    if (last) return prelu ? (const void*)k_edge_coop4<1, 1> : (const void*)k_edge_coop4<-1, 1>;
    return prelu ? (const void*)k_edge_coop4<1, 0> : (const void*)k_edge_coop4<-1, 0>;
  }
  return nullptr;
}

// ---------------------------------------------------------------------------- cooperative encoder
// k_encode with P waves per 16-row tile, for meshes whose row tiles leave most SIMDs idle
// (zenodo4: 864 row tiles, 1,024 SIMDs -- one wave per tile puts the whole chain of decoder,
// encoders, projection 0 and unpool V on one wave): every MFMA layer's output tiles are split
// over the ranks (rank r: tiles [r T/P, (r+1) T/P)) and exchanged through LDS, a layer with
// fewer output tiles than ranks (the decoder's last) runs on every rank.  Every output element
// is the same MFMA chain in the same k order as in k_encode: bit-identical results.
// Exchange buffers alternate with a running count, so a buffer is rewritten only two
// barriers after its last read, also across MLPs.
template <int IN0, int T, int TL, int ACT, int P, int XW>
__device__ __forceinline__ void enc_coop_mlp(const f32x4 (&in)[IN0], f32x4 (&out)[TL], const MlpDev& m,
                                             const float* __restrict__ W, int lane, int g, int j, int r,
                                             float* buf, int& xc) {
  static_assert(T % P == 0, "hidden tiles split evenly over the ranks");
  auto last = [&](const auto& h) {
    constexpr int TI = sizeof(h) / sizeof(f32x4);
    if constexpr (TL % P == 0) {
      f32x4 o[TL / P];
      mfma_layer_sub<TI, TL / P, ACT>(h, o, m.l[m.n - 1], W, r * (TL / P), lane, g);
      coop_exchange<TL, P>(o, out, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
    } else {
      mfma_layer<TI, TL, ACT>(h, out, m.l[m.n - 1], W, lane, g);
    }
  };
  if (m.n == 1) {
    last(in);
    return;
  }
  f32x4 h[T];
  {
    f32x4 o[T / P];
    mfma_layer_sub<IN0, T / P, ACT>(in, o, m.l[0], W, r * (T / P), lane, g);
    coop_exchange<T, P>(o, h, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
  }
  for (int li = 1; li + 1 < m.n; ++li) {
    f32x4 o[T / P];
    mfma_layer_sub<T, T / P, ACT>(h, o, m.l[li], W, r * (T / P), lane, g);
    coop_exchange<T, P>(o, h, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
  }
  last(h);
}
// Workgroup: WV waves = WV / P row tiles (F = 32: eight waves, the four row tiles of k_encode's
// workgroup, so the weight region is staged as often as there; F = 64 reads the blob).
template <int NT> constexpr int enc_coop_waves() { return NT == 2 ? 8 : kWaves; }
template <int NT, int ACT, bool DEC, int P, int WV = enc_coop_waves<NT>()>
__global__ __launch_bounds__(64 * WV) void k_encode_coop(EncodeArgs a) {
  constexpr int F = 16 * NT, T2 = 2 * NT, G = WV / P;
  constexpr int XW = 16 * T2 + 4;
  __shared__ __attribute__((aligned(16))) float xbuf[G][2][kRowsPerWave][XW];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int grp = w / P, r = w % P;
  MSW_MARK(a.c, 0);
  Common c = a.c;
  const int dstep = DEC ? a.dec.io->step : -1;
  if (!a.dec.on && a.io && blockIdx.x == 0 && threadIdx.x == 0) a.io->step += 1;
  // one chunk of G row tiles per workgroup (scale starts are 64-aligned: one scale)
  const int rb = blockIdx.x * (G * kRowsPerWave);
  int s = 0;
  while (s + 1 < a.S && rb >= a.n0[s + 1]) ++s;
  const int n = rb + grp * kRowsPerWave + j;
  const bool valid = (n - a.n0[s]) < a.ns[s];
  const int ext = a.c.perm ? a.c.perm[n] : n;
  const int xrow = a.x_internal ? (valid ? n : a.n0[s]) : (valid ? ext : 0);
  const float* xr = a.x + (size_t)xrow * a.c.nnf;
  const int nstat = a.c.nstat_raw;
  float raw[4], dyn[4];
  float wlv;
  EpiPre<NT> pre;
  f32x4 xu[NT];
  if (DEC) {  // as k_encode: not behind the step counter
    load_row<NT>(xu, a.dec_in + (size_t)n * F, g);
    pre.ext = ext;
    pre.bc = a.dec.bc_slot[n];
#pragma unroll
    for (int k = 0; k < kMaxDyn; ++k) pre.xd[k] = k < c.dyn ? xr[nstat + k] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = 4 * g + q;
    raw[q] = f < nstat ? xr[f] : 0.f;
    dyn[q] = f < a.c.dyn ? xr[nstat + f] : 0.f;
  }
  wlv = xr[nstat - 1] + xr[a.c.nnf - 2];
  MSW_MARK(c, 1);
  if constexpr (kStaged<NT>) {
    stage_glds<WV>(smem, a.c.W, a.sreg[s], 0, a.sreg[s].len);
    __syncthreads();
  }
  const float* Wl = kStaged<NT> ? (const float*)smem : c.W;
  float* buf = &xbuf[grp][0][0][0];
  int xc = 0;
  if (DEC && dstep >= 0) {
#pragma clang fp contract(off)
    pre.step = dstep;
    bc_prefetch<NT>(pre, a.dec, c);
    float nd[kMaxDyn];
    {
      f32x4 x0[NT], o[1];
#pragma unroll
      for (int t = 0; t < NT; ++t) x0[t] = xu[t];
      act_tiles<-1, NT>(x0, a.dec.pre_act, a.dec.pre_slope);
      enc_coop_mlp<NT, NT, 1, ACT, P, XW>(x0, o, a.dec.dec, Wl, lane, g, j, r, buf, xc);
      decode_state_tail<NT>(o, a.dec, c, Wl, pre, n, valid && r == 0, lane, g, nd);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 4 * g + q;
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < kMaxDyn; ++k) v = (k == f && f < c.dyn) ? nd[k] : v;
      dyn[q] = v;
    }
    float hn = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxDyn; ++k) hn = (k == c.dyn - 2) ? nd[k] : hn;
    wlv = xr[nstat - 1] + hn;
  }
  if (DEC && a.decode_only) return;
  MSW_MARK(c, 2);
  f32x4 xs[NT];
  {
    f32x4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (c.with_wl && 4 * g + q == nstat) ? wlv : raw[q];
    const f32x4 in[1] = {v};
    enc_coop_mlp<1, NT, NT, ACT, P, XW>(in, xs, a.stat, Wl, lane, g, j, r, buf, xc);
    if (valid && r == 0) store_row<NT>(a.xs + (size_t)n * F, xs, NT, g);
  }
  MSW_MARK(c, 5);
  if (s == 0) {
    f32x4 xd[NT];
    const f32x4 in[1] = {f32x4{dyn[0], dyn[1], dyn[2], dyn[3]}};
    enc_coop_mlp<1, NT, NT, ACT, P, XW>(in, xd, a.dynm, Wl, lane, g, j, r, buf, xc);
    if (valid && r == P - 1 && a.xd) store_row<NT>(a.xd + (size_t)n * F, xd, NT, g);
    MSW_MARK(c, 6);
    if (a.np0.h1t == T2)
      np_project_coop<NT, T2, P>(xs, xd, a.np0, Wl, n, valid, r, lane, g);
    else
      np_project_coop<NT, NT, P>(xs, xd, a.np0, Wl, n, valid, r, lane, g);
  }
  MSW_MARK(c, 8);
  if (a.vu_a[s] >= 0) {
    if (a.vu_h1t == T2)
      proj_store_part<NT, T2 / P>(xs, Wl + a.vu_a[s], r, a.Vu, n, T2, valid, lane, g);
    else
      proj_store_part<NT, NT / P>(xs, Wl + a.vu_a[s], r, a.Vu, n, NT, valid, lane, g);
  }
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- hop
// Hops 2..K (gnn.py:406-443) over the same tiles:
//   active(e) = rowsum(out[src]) != 0 || rowsum(out[dst]) != 0          (gnn.py:408-411)
//   agg[c]    = sum_e active(e) * (out[c] - out[src]) * s_e  (edge order; gnn.py:430-438)
//   out'[c]   = out[c] + W_{k+1} agg[c]  (MFMA)  -> store, or the epilogue after hop K
// LAST = false: no epilogue, the filter's A operand goes straight from the blob into
// registers at kernel start (no LDS staging, no workgroup barrier).
template <int NT>
struct HopRows {
  Lanes L;
  f32x4 os[NT], sv[NT], inn[NT];
  EpiPre<NT> pre;  // LAST only
};
template <int NT, bool LAST>
__device__ __forceinline__ void hop_gather(HopRows<NT>& r, const HopArgs& a, const LaneRec& rec, int tile, int j,
                                           int g) {
  constexpr int F = 16 * NT;
  r.L = lanes_of(rec, tile, j, a.n0);
  load_row<NT>(r.os, a.in + r.L.sr * F, g);
  load_row<NT>(r.sv, a.s + r.L.p * F, g);
  load_row<NT>(r.inn, a.in + r.L.n * F, g);
  if constexpr (LAST) epi_prefetch<NT>(r.pre, a.epi, a.c, a.xs, r.L.n, g);
}
template <int NT, bool LAST>
__device__ __forceinline__ void hop_load(HopRows<NT>& r, const HopArgs& a, int tile, int j, int g) {
  hop_gather<NT, LAST>(r, a, load_rec(a.recs, tile, j), tile, j, g);
}
template <int NT, int ACT, bool LAST, bool LOOP>
__global__ __launch_bounds__((64 * hop_waves<NT, LOOP>())) void k_hop(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int WV = hop_waves<NT, LOOP>();
  constexpr int F = 16 * NT;
  constexpr int XS = F + 4;  // padded rows: conflict-free b128 LDS accesses
  __shared__ __attribute__((aligned(16))) float slab_all[WV][kRowsPerWave][XS];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int stride = gridDim.x * WV;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  int tile = xb * WV + w;
  Common c = a.c;
  MSW_MARK(c, 0);
  f32x4 wf[NT][NT];
  load_filter<NT>(wf, c.W, a.filt_a, lane);  // blob offset: not part of the LDS region
  float* slab = &slab_all[w][0][0];
  auto core = [&](const HopRows<NT>& r, int j, int lane, int g, f32x4 (&res)[NT]) {
    float* my = slab + j * XS;
    const Lanes& L = r.L;
    store_row<NT>(my, r.inn, NT, g);
    wave_lds_sync();
    f32x4 od[NT];
    load_row<NT>(od, slab + L.dl * XS, g);
    MSW_MARK(c, 4);
    put_message<NT>(my, r.os, od, r.sv, L.ev, a.grad, a.upwind, g);
    MSW_MARK(c, 6);
    f32x4 agg[NT];
    gather_messages<NT, XS>(agg, slab, L.q0, L.q1, g);
    MSW_MARK(c, 7);
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = r.inn[t];
    apply_filter_regs<NT>(res, agg, a.filt_a, wf);
    MSW_MARK(c, 8);
  };
  auto finish = [&](f32x4 (&res)[NT], const HopRows<NT>& r, int lane, int g) {
    const Lanes& L = r.L;
    if constexpr (LAST) {
      node_epilogue<NT, ACT>(res, a.epi, c, r.pre, a.out, L.n, L.nv, lane, g);
    } else {
      if (L.nv) store_row<NT>(a.out + L.n * F, res, NT, g);
    }
  };
  if constexpr (!LOOP) {
    const bool live = tile < a.ntiles;
    HopRows<NT> r;
    hop_load<NT, LAST>(r, a, live ? tile : 0, j, g);
    MSW_MARK(c, 1);
    // the epilogue's operands stream into LDS alongside the tile's gathers
    if constexpr (LAST && kStaged<NT>) stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
    f32x4 res[NT];
    if (live) core(r, j, lane, g, res);
    if constexpr (LAST && kStaged<NT>) {
      __syncthreads();
      c.W = smem;
    }
    MSW_MARK(c, 2);
    if (live) finish(res, r, lane, g);
  } else {
    if constexpr (LAST && kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      c.W = smem;
    }
    // middle hops, software pipeline: tile i+1's gathers and tile i+2's lane record are in
    // flight while tile i computes (the record round trip no longer stalls the wave); the
    // last hop keeps one tile in flight (its epilogue prefetch would double the registers)
    if (LAST) {
      for (; tile < a.ntiles; tile += stride) {
        const int ln = opaque_lane(), gg = ln >> 4, jj = ln & 15;
        HopRows<NT> q;
        hop_load<NT, LAST>(q, a, tile, jj, gg);
        f32x4 res[NT];
        core(q, jj, ln, gg, res);
        finish(res, q, ln, gg);
      }
    } else if (tile < a.ntiles) {
      HopRows<NT> q;
      hop_load<NT, LAST>(q, a, tile, j, g);
      int t1 = tile + stride;
      LaneRec rn = load_rec(a.recs, t1 < a.ntiles ? t1 : tile, j);
      for (;;) {
        const int ln = opaque_lane(), gg = ln >> 4, jj = ln & 15;
        const bool more = t1 < a.ntiles;
        HopRows<NT> qn;
        if (more) {
          hop_gather<NT, LAST>(qn, a, rn, t1, jj, gg);
          const int t2 = t1 + stride;
          rn = load_rec(a.recs, t2 < a.ntiles ? t2 : t1, jj);
        }
        f32x4 res[NT];
        core(q, jj, ln, gg, res);
        finish(res, q, ln, gg);
        if (!more) break;
        q = qn;
        t1 += stride;
      }
    }
  }
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- row-layout middle hop
// Large meshes (grid-stride regime, HBM-bound): a wave owns 16 CONSECUTIVE destination rows of
// the scale; lane row j pulls its own in-edges from the scale's CSR by destination (reference
// edge order: {source row, tile-padded s slot} per edge) -- no lane records, no LDS slab, and
// all 16 rows of the filter MFMA are live (an edge tile holds ~5 destinations of its 16 rows).
// A lane keeps DC edges' source and s rows in flight at once (DC = 4 at F <= 32, 2 at F = 64).
// The arithmetic is k_hop's operation for operation -- the activity predicate's sums, the
// message, agg = ((0 + m_0) + m_1) + ... in edge order, the filter -- so it is bit-identical.
constexpr int kRowHopWaves = 8;
#ifndef MSW_ROW_DC
#define MSW_ROW_DC 3  // edges in flight per lane (F <= 32): 113 VGPRs, 4 waves per SIMD
#endif
template <int NT>
__global__ __launch_bounds__(64 * kRowHopWaves) void k_hop_rows(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  constexpr int DC = NT >= 4 ? 2 : MSW_ROW_DC;
  [[maybe_unused]] const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int stride = gridDim.x * kRowHopWaves;
  const int ntile = (a.nrows + kRowsPerWave - 1) / kRowsPerWave;
  f32x4 wf[NT][NT];  // the filter in registers (in LDS: equal, profiles/r03/ab_rows_variants.jsonl)
  load_filter<NT>(wf, a.c.W, a.filt_a, lane);
  for (int tile = blockIdx.x * kRowHopWaves + w; tile < ntile; tile += stride) {
    const int ln = opaque_lane(), g = ln >> 4, j = ln & 15;
    const int k = tile * kRowsPerWave + j;
    const bool valid = k < a.nrows;
    const int kc = valid ? k : 0;
    const int q0 = a.rptr[kc], q1 = valid ? a.rptr[kc + 1] : q0;
    const size_t n = (size_t)a.n0 + kc;
    f32x4 od[NT];
    load_row<NT>(od, a.in + n * F, g);
    const int deg = q1 - q0;
    int dmax = deg;  // wave-uniform trip count
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) dmax = max(dmax, __shfl_xor(dmax, o));
    float rd = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) rd += hsum(od[t]);
    const bool zd = row_sum(rd) != 0.f;
    f32x4 agg[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) agg[t] = zero4();
    for (int q = 0; q < dmax; q += DC) {
      int2 e[DC];
#pragma unroll
      for (int u = 0; u < DC; ++u)  // absent edges read the row's own entries (never used)
        e[u] = q + u < deg ? a.redge[q0 + q + u] : int2{(int)n, 0};
      f32x4 os[DC][NT], sv[DC][NT];
#pragma unroll
      for (int u = 0; u < DC; ++u) {
        load_row<NT>(os[u], a.in + (size_t)e[u].x * F, g);
        load_row<NT>(sv[u], a.s + (size_t)e[u].y * F, g);
      }
#pragma unroll
      for (int u = 0; u < DC; ++u) {
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) rs += hsum(os[u][t]);
        const bool act = (row_sum(rs) != 0.f) || zd;  // gnn.py:408-411
        const bool has = q + u < deg;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x4 gv;
          if (a.grad) {
            gv = od[t] - os[u][t];
            if (a.upwind) {
              gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
              gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
            }
          } else {
            gv = os[u][t];
          }
          const f32x4 m = act ? gv * sv[u][t] : zero4();
          const f32x4 sum = agg[t] + m;
          agg[t] = has ? sum : agg[t];
        }
      }
    }
    f32x4 res[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = od[t];
    apply_filter_regs<NT>(res, agg, a.filt_a, wf);
    if (valid) store_row<NT>(a.out + n * F, res, NT, g);
  }
}

// ---------------------------------------------------------------------------- feature-split middle hop
// A middle hop (no epilogue) with each edge tile's features split over two waves: rank r
// gathers, messages and sums features [F r / 2, F (r + 1) / 2) only (half the loads per wave,
// twice the waves in flight), the two ranks exchange through LDS what crosses the split --
// the per-lane partial row sums of the activity predicate (recombined in k_hop's order,
// ((h0 + h1) + h2) + h3, on both ranks) and the aggregated messages (the filter's B operand:
// rank r computes output tiles [NT r / 2, NT (r + 1) / 2) over all input tiles in k_hop's k
// order).  Bit-identical to k_hop.
template <int NT>
__global__ __launch_bounds__(kBlock) void k_hop_split(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, TH = NT / 2, G = kWaves / 2;
  constexpr int XS = 16 * TH + 4;
  __shared__ __attribute__((aligned(16))) float slab_all[G][2][kRowsPerWave][XS];
  __shared__ __attribute__((aligned(16))) float hx[G][2][2 * TH][64];  // partial row sums
  __shared__ __attribute__((aligned(16))) f32x4 ax[G][NT][64];          // aggregated messages
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int grp = w / 2, r = w % 2, t0 = r * TH;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  const int tile = xb * G + grp;
  const bool live = tile < a.ntiles;  // dead groups compute tile 0 and store nothing
  MSW_MARK(a.c, 0);
  const Lanes L = lanes_of(load_rec(a.recs, live ? tile : 0, j), live ? tile : 0, j, a.n0);
  f32x4 os[TH], sv[TH], inn[TH];
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    const int off = 16 * (t0 + t) + 4 * g;
    os[t] = ld4(a.in + L.sr * F + off);
    sv[t] = ld4(a.s + L.p * F + off);
    inn[t] = ld4(a.in + L.n * F + off);
  }
  f32x4 wf[TH][NT];  // this rank's output tiles of the filter
  {
    const int fa = a.filt_a >= 0 ? a.filt_a : 0;
#pragma unroll
    for (int to = 0; to < TH; ++to)
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) wf[to][ti] = ld4(a.c.W + fa + ((size_t)((t0 + to) * NT + ti) * 64 + lane) * 4);
  }
  float* slab = &slab_all[grp][r][0][0];
  float* my = slab + j * XS;
#pragma unroll
  for (int t = 0; t < TH; ++t) st4(my + 16 * t + 4 * g, inn[t]);
  wave_lds_sync();
  f32x4 od[TH];
#pragma unroll
  for (int t = 0; t < TH; ++t) od[t] = ld4(slab + L.dl * XS + 16 * t + 4 * g);
  // activity predicate (put_message): per-lane partial sums of both ranks, combined in t order
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    hx[grp][r][t][lane] = hsum(os[t]);
    hx[grp][r][TH + t][lane] = hsum(od[t]);
  }
  __syncthreads();
  float rs = 0.f, rd = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      rs += hx[grp][q][t][lane];
      rd += hx[grp][q][TH + t][lane];
    }
  const bool act = (row_sum(rs) != 0.f) || (row_sum(rd) != 0.f);  // gnn.py:408-411
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    f32x4 gv;
    if (a.grad) {
      gv = od[t] - os[t];
      if (a.upwind) {
        gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
        gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
      }
    } else {
      gv = os[t];
    }
    const f32x4 m = gv * sv[t];
    st4(my + 16 * t + 4 * g, (L.ev && act) ? m : zero4());
  }
  f32x4 agg[TH];
  gather_messages<TH, XS>(agg, slab, L.q0, L.q1, g);
#pragma unroll
  for (int t = 0; t < TH; ++t) ax[grp][t0 + t][lane] = agg[t];
  __syncthreads();
  f32x4 res[TH];
#pragma unroll
  for (int t = 0; t < TH; ++t) res[t] = inn[t];
  if (a.filt_a >= 0) {
    f32x4 full[NT], acc[TH];
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) full[ti] = ax[grp][ti][lane];
#pragma unroll
    for (int to = 0; to < TH; ++to) acc[to] = zero4();
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int to = 0; to < TH; ++to) acc[to] = MSW_MFMA(wf[to][ti][q], full[ti][q], acc[to]);
#pragma unroll
    for (int t = 0; t < TH; ++t) res[t] = res[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < TH; ++t) res[t] = res[t] + agg[t];
  }
  if (live && L.nv) {
#pragma unroll
    for (int t = 0; t < TH; ++t) st4(a.out + L.n * F + 16 * (t0 + t) + 4 * g, res[t]);
  }
  MSW_MARK(a.c, 9);
}

// ---------------------------------------------------------------------------- cooperative last hop
// A layer's last hop + its epilogue with P waves per tile (small scales, as k_edge_coop):
// every rank does the hop's VALU / LDS work; the filter, the projections (next layer U/V/O,
// unpool U) and the decoder's hidden layers are split by output tile and exchanged through
// LDS; the decoder's 2-wide output layer runs on every rank, its tail on rank 0.
template <int NT, int ACT, int P>
__device__ __forceinline__ void node_epilogue_coop(f32x4 (&res)[NT], const Epilogue& e, const Common& c,
                                                   const EpiPre<NT>& pre, float* out, int n, bool valid,
                                                   int r, int lane, int g, int j, float* b0, float* b1, int xw) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, T2 = 2 * NT;
  if (e.post_act) act_tiles<-1, NT>(res, e.post_act, e.post_slope);
  if (out && valid && r == 0) store_row<NT>(out + (size_t)n * F, res, NT, g);
  if (e.np.a_u >= 0 || e.np.a_v >= 0 || e.np.a_o >= 0) {
    if (e.np.h1t == T2)
      np_project_coop<NT, T2, P>(pre.xs, res, e.np, c.W, (size_t)n, valid, r, lane, g);
    else
      np_project_coop<NT, NT, P>(pre.xs, res, e.np, c.W, (size_t)n, valid, r, lane, g);
  }
  if (e.uu_a >= 0) {
    f32x4 in[T2];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      in[t] = pre.xs[t];
      in[NT + t] = res[t];
    }
    if (e.uu_h1t == T2)
      proj_store_part<T2, T2 / P>(in, c.W + e.uu_a, r, e.Uu, (size_t)n, T2, valid, lane, g);
    else
      proj_store_part<T2, NT / P>(in, c.W + e.uu_a, r, e.Uu, (size_t)n, NT, valid, lane, g);
  }
  if (e.dec.on) {
    const DecDesc& d = e.dec;
    f32x4 x0[NT], o[1];
#pragma unroll
    for (int t = 0; t < NT; ++t) x0[t] = res[t];
    act_tiles<-1, NT>(x0, d.pre_act, d.pre_slope);
    const MlpDev& m = d.dec;
    if (m.n == 1) {
      mfma_layer<NT, 1, ACT>(x0, o, m.l[0], c.W, lane, g);
    } else {  // hidden layers split (exchanges alternate b1, b0, ...: b0 held the result row)
      f32x4 h[NT];
      {
        f32x4 p[NT / P];
        mfma_layer_sub<NT, NT / P, ACT>(x0, p, m.l[0], c.W, r * (NT / P), lane, g);
        coop_exchange<NT, P>(p, h, b1, xw, r, j, g);
      }
      for (int li = 1; li + 1 < m.n; ++li) {
        f32x4 p[NT / P];
        mfma_layer_sub<NT, NT / P, ACT>(h, p, m.l[li], c.W, r * (NT / P), lane, g);
        coop_exchange<NT, P>(p, h, (li & 1) ? b0 : b1, xw, r, j, g);
      }
      mfma_layer<NT, 1, ACT>(h, o, m.l[m.n - 1], c.W, lane, g);
    }
    if (r == 0) decode_tail<NT>(o, d, c, pre, n, valid, g);
  }
}

template <int NT, int ACT, int P>
__global__ __launch_bounds__(kBlock) void k_hop_coop(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, TS = NT / P;
  constexpr int XS = F + 4;
  constexpr int XW = 16 * NT + 4;
  constexpr int G = kWaves / P;
  __shared__ __attribute__((aligned(16))) float slab_all[kWaves][kRowsPerWave][XS];
  __shared__ __attribute__((aligned(16))) float xbuf[G][2][kRowsPerWave][XW];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int grp = w / P, r = w % P;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  const int tile = xb * G + grp;
  const bool live = tile < a.ntiles;
  Common c = a.c;
  // this rank's filter rows (out tiles r TS .. r TS + TS - 1), by address
  f32x4 wr[TS][NT];
  {
    const int fa = a.filt_a >= 0 ? a.filt_a : 0;
#pragma unroll
    for (int to = 0; to < TS; ++to)
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) wr[to][ti] = ld4(c.W + fa + ((size_t)((r * TS + to) * NT + ti) * 64 + lane) * 4);
  }
  HopRows<NT> q;
  hop_load<NT, true>(q, a, live ? tile : 0, j, g);  // dead groups compute tile 0, store nothing
  if constexpr (kStaged<NT>) stage_glds<kWaves>(smem, a.c.W, a.reg, 0, a.reg.len);  // epilogue operands
  const Lanes& L = q.L;
  float* slab = &slab_all[w][0][0];
  float* my = slab + j * XS;
  store_row<NT>(my, q.inn, NT, g);
  wave_lds_sync();
  f32x4 od[NT];
  load_row<NT>(od, slab + L.dl * XS, g);
  put_message<NT>(my, q.os, od, q.sv, L.ev, a.grad, a.upwind, g);
  f32x4 agg[NT];
  gather_messages<NT, XS>(agg, slab, L.q0, L.q1, g);
  f32x4 rs[TS];
#pragma unroll
  for (int t = 0; t < TS; ++t) rs[t] = ld4(a.in + L.n * F + 16 * (r * TS + t) + 4 * g);  // inn, by address
  if (a.filt_a >= 0) {
    f32x4 acc[TS];
#pragma unroll
    for (int to = 0; to < TS; ++to) acc[to] = zero4();
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int to = 0; to < TS; ++to) acc[to] = MSW_MFMA(wr[to][ti][rr], agg[ti][rr], acc[to]);
#pragma unroll
    for (int t = 0; t < TS; ++t) rs[t] = rs[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < TS; ++t) {
      f32x4 ag = zero4();
      for (int qq = L.q0; qq < L.q1; ++qq) ag = ag + ld4(slab + qq * XS + 16 * (r * TS + t) + 4 * g);
      rs[t] = rs[t] + ag;
    }
  }
  f32x4 res[NT];
  float* b0 = &xbuf[grp][0][0][0];
  float* b1 = &xbuf[grp][1][0][0];
  coop_exchange<NT, P>(rs, res, b0, XW, r, j, g);  // its barrier also lands the staged operands
  if constexpr (kStaged<NT>) c.W = smem;
  node_epilogue_coop<NT, ACT, P>(res, a.epi, c, q.pre, a.out, (int)L.n, live && L.nv, r, lane, g, j, b0, b1, XW);
}

// ---------------------------------------------------------------------------- persistent hop chain
// Middle hops k .. k+m-1 of one layer on a small scale in ONE launch (engine.h HopChainArgs;
// verdict r3 item 6).  The grid is XCD-packed onto XCD 0 (c.xcd = 1; G <= 32 workgroups, one
// tile per wave, all co-resident: nothing else runs on the stream), so every row a hop writes
// stays in XCD 0's L2: stores and the next hop's row gathers are agent-scope relaxed atomics
// (sc1: served by the L2, never a stale L1 line), and the barrier between hops is a relaxed
// agent-scope counter -- no fences, nothing leaves the XCD.  Per hop the arithmetic is k_hop's
// (LAST = false), operation for operation: bit-identical.  Every spin is bounded: an expired
// spin counts in err[0] and the launch still finishes (results then unreliable, never a
// hang); a participant found off XCD 0 counts in err[1] (the host checks both).
constexpr long kChainSpin = 1L << 22;
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
__device__ __forceinline__ f32x4 ld4_l2(const float* p) {
  f32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}
__device__ __forceinline__ void st4_l2(float* p, f32x4 v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) __hip_atomic_store(p + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int N>
__device__ __forceinline__ void load_row_l2(f32x4 (&v)[N], const float* row, int g) {
#pragma unroll
  for (int t = 0; t < N; ++t) v[t] = ld4_l2(row + 16 * t + 4 * g);
}
// barrier among the chain's G workgroups: every wave's stores have reached the L2 (vmcnt(0))
// before its workgroup arrives
__device__ __forceinline__ void chain_barrier(const HopChainArgs& a, unsigned long long target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(a.ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long n = 0;
    while (__hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++n < kChainSpin)
      __builtin_amdgcn_s_sleep(1);
    if (n >= kChainSpin) atomicAdd(&a.err[0], 1);
  }
  __syncthreads();
}
// LASTPH: the chain's final hop is the layer's last hop (k_hop<.., LAST = true>'s path: its
// epilogue operands -- projections of the next layer, unpool U, forward-mode decoder -- are
// staged into LDS at kernel start, behind the middle hops).
template <int NT, int ACT, bool LASTPH>
__global__ __launch_bounds__(kBlock) void k_hop_chain(HopChainArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  constexpr int XS = F + 4;
  __shared__ __attribute__((aligned(16))) float slab_all[kWaves][kRowsPerWave][XS];
  __shared__ unsigned long long base_s;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int xb = logical_block(a.h.c);
  if (xb < 0) return;
  if (threadIdx.x == 0) {
    if (xcc_id() != 0) atomicAdd(&a.err[1], 1);
    // every launch adds exactly (m - 1) G arrivals and none can pass the first barrier before
    // all G have started: the value read here lies in [base, base + G) of this launch
    const unsigned long long v = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long per = (unsigned long long)(a.m - 1) * a.G;
    base_s = v - v % per;
  }
  __syncthreads();
  const unsigned long long base = base_s;
  const int tile = xb * kWaves + w;
  const bool live = tile < a.h.ntiles;
  const int tl = live ? tile : 0;  // idle waves stay in bounds
  float* slab = &slab_all[w][0][0];
  Common c = a.h.c;
  const Lanes L = lanes_of(load_rec(a.h.recs, tl, j), tl, j, a.h.n0);
  f32x4 sv[NT];
  load_row<NT>(sv, a.h.s + L.p * F, g);  // s is fixed for the layer: plain loads
  [[maybe_unused]] EpiPre<NT> pre;
  if constexpr (LASTPH) {
    if constexpr (kStaged<NT>) stage_glds<kWaves>(smem, c.W, a.h.reg, 0, a.h.reg.len);
    epi_prefetch<NT>(pre, a.h.epi, c, a.h.xs, L.n, g);  // static inputs (x_s rows, X, BC)
  }
  for (int k = 0; k < a.m; ++k) {
    const float* in = a.io[k];
    float* out = a.io[k + 1];
    f32x4 wf[NT][NT];
    load_filter<NT>(wf, a.h.c.W, a.filt[k], lane);
    f32x4 os[NT], inn[NT];
    if (k == 0) {  // written by the previous launch: plain loads
      load_row<NT>(os, in + L.sr * F, g);
      load_row<NT>(inn, in + L.n * F, g);
    } else {
      load_row_l2<NT>(os, in + L.sr * F, g);
      load_row_l2<NT>(inn, in + L.n * F, g);
    }
    if (live) {  // k_hop's core, LAST = false
      float* my = slab + j * XS;
      store_row<NT>(my, inn, NT, g);
      wave_lds_sync();
      f32x4 od[NT];
      load_row<NT>(od, slab + L.dl * XS, g);
      put_message<NT>(my, os, od, sv, L.ev, a.h.grad, a.h.upwind, g);
      f32x4 agg[NT], res[NT];
      gather_messages<NT, XS>(agg, slab, L.q0, L.q1, g);
#pragma unroll
      for (int t = 0; t < NT; ++t) res[t] = inn[t];
      apply_filter_regs<NT>(res, agg, a.filt[k], wf);
      if (LASTPH && k + 1 == a.m) {  // the layer's last hop: k_hop<.., LAST = true>'s finish
        if constexpr (kStaged<NT>) c.W = smem;  // staged at kernel start (every wave passed a barrier since)
        node_epilogue<NT, ACT>(res, a.h.epi, c, pre, out, L.n, L.nv, lane, g);
      } else if (L.nv) {
#pragma unroll
        for (int t = 0; t < NT; ++t) st4_l2(out + L.n * F + 16 * t + 4 * g, res[t]);
      }
    }
    if (k + 1 < a.m) chain_barrier(a, base + (unsigned long long)(k + 1) * a.G);
  }
}

template <int NT>
static const void* hop_coop_kernel(int prelu) {
  if constexpr (NT >= 2) return prelu ? (const void*)k_hop_coop<NT, 1, NT> : (const void*)k_hop_coop<NT, -1, NT>;
  return nullptr;
}

// ---------------------------------------------------------------------------- pooling
// scatter(x[fine], coarse, reduce='mean') (gnn.py:256): children summed in edge order,
// divided by max(count, 1); then the projection of the next processor.  A wave tile is 16
// consecutive coarse rows: lane (row j, group g) walks its own row's children (CSR) and
// sums feature slice g of each -- no lane exchange, every MFMA row of the projection used
// (an edge-tile layout would hold only 4 coarse rows of 4 children each).
template <int NT, bool LOOP>
__global__ __launch_bounds__((64 * waves_of<NT, LOOP>())) void k_pool(PoolArgs a) {
#pragma clang fp contract(off)
  constexpr int WV = waves_of<NT, LOOP>();
  constexpr int F = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int stride = gridDim.x * WV;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  int tile = xb * WV + w;
  Common c = a.c;
  MSW_MARK(c, 0);
  struct Rows {
    f32x4 acc[NT], xs[NT];
    size_t n;
    bool nv;
  };
  auto load = [&](Rows& r, int t, int j, int g) {
    const int i = 16 * t + j;
    r.nv = i < a.ns;
    r.n = (size_t)a.n0 + (r.nv ? i : 0);
    int4 rc = *reinterpret_cast<const int4*>(a.recs + 16 * t + j);
    const int2 ro = *reinterpret_cast<const int2*>(&a.recs[16 * t + j].cnt);
    asm volatile("" : "+v"(rc.x));  // keep the record one unconditional 16-B load
    const int cnt = ro.x, off = ro.y;
    // unconditional loads (absent children re-read child 0 / the row itself): predicated
    // loads made the compiler drain the memory counter before each one
    const int c0 = cnt > 0 ? rc.x : (int)r.n;
    const int ci[kPoolInline] = {c0, cnt > 1 ? rc.y : c0, cnt > 2 ? rc.z : c0, cnt > 3 ? rc.w : c0};
    f32x4 x[kPoolInline][NT];
#pragma unroll
    for (int k = 0; k < kPoolInline; ++k) load_row<NT>(x[k], a.in + (size_t)ci[k] * F, g);
    load_row<NT>(r.xs, a.xs + r.n * F, g);
#pragma unroll
    for (int t2 = 0; t2 < NT; ++t2) r.acc[t2] = zero4();
#pragma unroll
    for (int k = 0; k < kPoolInline; ++k) {
#pragma unroll
      for (int t2 = 0; t2 < NT; ++t2) {
        const f32x4 s2 = r.acc[t2] + x[k][t2];
        r.acc[t2] = k < cnt ? s2 : r.acc[t2];
      }
    }
    for (int k = kPoolInline; k < cnt; ++k) {  // more children than the record holds
      f32x4 y[NT];
      load_row<NT>(y, a.in + (size_t)a.child[off + k] * F, g);
#pragma unroll
      for (int t2 = 0; t2 < NT; ++t2) r.acc[t2] = r.acc[t2] + y[t2];
    }
    const float fc = (float)(cnt > 0 ? cnt : 1);
#pragma unroll
    for (int t2 = 0; t2 < NT; ++t2) r.acc[t2] = r.acc[t2] / fc;
  };
  if constexpr (!LOOP) {
    Rows r0;
    load(r0, tile < a.ntiles ? tile : 0, j, g);
    MSW_MARK(c, 1);
    if constexpr (kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      c.W = smem;
    }
    MSW_MARK(c, 2);
    if (tile < a.ntiles) np_project<NT>(r0.xs, r0.acc, a.np, c.W, r0.n, r0.nv, lane, g);
  } else {
    if constexpr (kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      c.W = smem;
    }
    for (; tile < a.ntiles; tile += stride) {
      const int ln = opaque_lane(), gg = ln >> 4, jj = ln & 15;
      Rows q;
      load(q, tile, jj, gg);
      np_project<NT>(q.xs, q.acc, a.np, c.W, q.n, q.nv, ln, gg);
    }
  }
  MSW_MARK(c, 9);
}

// Small levels (the whole grid resident at once): edge tiles of coarse nodes with <= 16
// children in all, lane j loads child j, the coarse lanes sum through LDS -- four times
// the waves of the row layout, each with a shorter load chain (measured faster while the
// launch is latency-bound).
// P = 2: two waves per tile, both summing the children, the projection's output tiles split
// between them (as k_edge_coop; bit-identical).
// P = WV = 2 * NT (F = 64: eight waves per tile): each rank projects one U and one V output
// tile (ranks 0..NT-1 also one O tile) -- half the projection chain of P = NT.
template <int NT, int P = 1, int WV = kWaves>
__global__ __launch_bounds__(64 * WV) void k_pool_edge(PoolArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  constexpr int XS = F + 4;  // padded rows: conflict-free b128 LDS accesses
  static_assert(WV % P == 0, "whole tiles per workgroup");
  __shared__ __attribute__((aligned(16))) float slab_all[WV][kRowsPerWave][XS];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  int tile = xb * (WV / P) + w / P;
  const int rk = w % P;
  Common c = a.c;
  MSW_MARK(c, 0);
  struct Rows {
    Lanes L;
    f32x4 x[NT], xs[NT];
  };
  auto load = [&](Rows& r, int t, int j, int g) {
    r.L = lanes_of(load_rec(a.erecs, t, j), t, j, a.n0);
    load_row<NT>(r.x, a.in + r.L.sr * F, g);
    load_row<NT>(r.xs, a.xs + r.L.n * F, g);
  };
  float* slab = &slab_all[w][0][0];
  auto run = [&](const Rows& r, int j, int lane, int g) {
    const Lanes& L = r.L;
    store_row<NT>(slab + j * XS, r.x, NT, g);
    f32x4 acc[NT];
    gather_messages<NT, XS>(acc, slab, L.q0, L.q1, g);
    MSW_MARK(c, 7);
    const float cnt = (float)(L.q1 - L.q0 > 0 ? L.q1 - L.q0 : 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = acc[t] / cnt;
    if constexpr (P == 1) {
      np_project<NT>(r.xs, acc, a.np, c.W, L.n, L.nv, lane, g);
    } else {
      if (a.np.h1t == 2 * NT) {
        np_project_coop<NT, 2 * NT, P>(r.xs, acc, a.np, c.W, L.n, L.nv, rk, lane, g);
      } else if constexpr (P <= NT) {  // P > NT is launched for two-layer-wide MLPs only
        np_project_coop<NT, NT, P>(r.xs, acc, a.np, c.W, L.n, L.nv, rk, lane, g);
      }
    }
  };
  Rows r0;
  load(r0, tile < a.ntiles ? tile : 0, j, g);
  MSW_MARK(c, 1);
  if constexpr (kStaged<NT>) {
    stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
    __syncthreads();
    c.W = smem;
  }
  MSW_MARK(c, 2);
  if (tile < a.ntiles) run(r0, j, lane, g);
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- row epilogue
// engine.h EpiArgs: what follows a layer's last hop, on dense node tiles -- tile t = rows
// n0 + 16t .. n0 + 16t + 15, lane (row j, group g) -- instead of on the hop's edge tiles.
// Same operations in the same order as the hop's own epilogue (bit-identical results).
// LOOP: weights staged once per workgroup, the next tile's rows in flight while a tile
// computes.
template <int NT, int ACT, bool LOOP>
__global__ __launch_bounds__((64 * waves_of<NT, LOOP>())) void k_epi(EpiArgs a) {
#pragma clang fp contract(off)
  constexpr int WV = waves_of<NT, LOOP>();
  constexpr int F = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int stride = gridDim.x * WV;
  const int xb = logical_block(a.c);
  if (xb < 0) return;
  int tile = xb * WV + w;
  Common c = a.c;
  MSW_MARK(c, 0);
  struct Rows {
    f32x4 res[NT];
    EpiPre<NT> pre;
    int n;
    bool nv;
  };
  auto load = [&](Rows& r, int t, int j, int g) {
    const int i = 16 * t + j;
    r.nv = i < a.ns;
    r.n = a.n0 + (r.nv ? i : 0);
    load_row<NT>(r.res, a.in + (size_t)r.n * F, g);
    epi_prefetch<NT>(r.pre, a.epi, a.c, a.xs, (size_t)r.n, g);
  };
  if constexpr (!LOOP) {
    Rows r0;
    load(r0, tile < a.ntiles ? tile : 0, j, g);
    MSW_MARK(c, 1);
    if constexpr (kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      c.W = smem;
    }
    MSW_MARK(c, 2);
    if (tile < a.ntiles) node_epilogue<NT, ACT>(r0.res, a.epi, c, r0.pre, a.out, r0.n, r0.nv, lane, g);
  } else {
    if constexpr (kStaged<NT>) {
      stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg.len);
      __syncthreads();
      c.W = smem;
    }
    if (tile < a.ntiles) {
      Rows q;
      load(q, tile, j, g);
      for (;;) {
        const int ln = opaque_lane(), gg = ln >> 4, jj = ln & 15;
        const int t1 = tile + stride;
        const bool more = t1 < a.ntiles;
        Rows qn;
        if (more) load(qn, t1, jj, gg);
        node_epilogue<NT, ACT>(q.res, a.epi, c, q.pre, a.out, q.n, q.nv, ln, gg);
        if (!more) break;
        q = qn;
        tile = t1;
      }
    }
  }
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- plan time
// MODE 0: edge encoder chain (raw <= 16 features -> F -> ... -> F);
// MODE 1: edge part of a SWEGNN layer's first layer, Pe = W1[:, 4F:] e + b1 (F -> 2F).
template <int NT, int MODE>
__global__ __launch_bounds__(kBlock) void k_rowmlp(RowMlpArgs a) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int r0 = wave_row0();
  if (r0 >= a.R) return;
  const int row = r0 + (lane & 15);
  const bool valid = row < a.R;
  const float* xr = a.in + (size_t)(valid ? row : 0) * a.in_stride;
  constexpr int TI = MODE == 0 ? 1 : NT, TO = MODE == 0 ? NT : 2 * NT;
  f32x4 in[TI], out[TO];
#pragma unroll
  for (int t = 0; t < TI; ++t) {
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * t + 4 * g + r;
      v[r] = f < a.in_dim ? xr[f] : 0.f;
    }
    in[t] = v;
  }
  if (MODE == 0)
    run_mlp<TI, NT, TO, -1>(in, out, a.m, a.W, lane, g);
  else
    mfma_layer<TI, TO, -1>(in, out, a.m.l[0], a.W, lane, g);
  if (valid) store_row<TO>(a.out + (size_t)row * a.out_stride, out, a.out_tiles, g);
}

// ---------------------------------------------------------------------------- launchers
static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

template <int NT>
constexpr size_t lds_bytes(int floats) {
  return kStaged<NT> ? (size_t)((floats + kChunk - 1) / kChunk * kChunk) * sizeof(float) : 0;
}

// Allow the dynamic weight regions past the 64 KB default (gfx950: 160 KB per CU).
template <int NT>
hipError_t prepare_kernels() {
  // the largest static slab (edge-MLP rows) of a workgroup of `wv` waves
  auto mx = [](int wv) { return 160 * 1024 - wv * kRowsPerWave * (16 * 2 * NT + 16 * NT + 4) * (int)sizeof(float); };
  constexpr int WL = waves_of<NT, true>();
  const std::pair<const void*, int> fns[] = {
      {(const void*)k_encode<NT, 1, false>, kWaves}, {(const void*)k_encode<NT, -1, false>, kWaves},
      {(const void*)k_encode<NT, 1, true>, kWaves}, {(const void*)k_encode<NT, -1, true>, kWaves},
      {(const void*)k_edge_hop<NT, 1, false, 0>, kWaves}, {(const void*)k_edge_hop<NT, -1, false, 0>, kWaves},
      {(const void*)k_edge_hop<NT, 1, false, 1>, kWaves}, {(const void*)k_edge_hop<NT, -1, false, 1>, kWaves},
      {(const void*)k_edge_hop<NT, 1, true, 0>, edge_waves<NT, true, 0>()},
      {(const void*)k_edge_hop<NT, -1, true, 0>, edge_waves<NT, true, 0>()},
      {(const void*)k_edge_hop<NT, 1, true, 1>, edge_waves<NT, true, 1>()},
      {(const void*)k_edge_hop<NT, -1, true, 1>, edge_waves<NT, true, 1>()},
      {(const void*)k_hop<NT, 1, true, false>, kWaves}, {(const void*)k_hop<NT, -1, true, false>, kWaves},
      {(const void*)k_hop<NT, 1, true, true>, hop_waves<NT, true>()},
      {(const void*)k_hop<NT, -1, true, true>, hop_waves<NT, true>()},
      {(const void*)k_pool<NT, false>, kWaves}, {(const void*)k_pool<NT, true>, WL},
      {(const void*)k_pool_edge<NT>, kWaves}, {(const void*)k_pool_edge<NT, NT >= 2 ? NT : 1>, kWaves},
      {(const void*)k_epi<NT, 1, false>, kWaves}, {(const void*)k_epi<NT, -1, false>, kWaves},
      {(const void*)k_epi<NT, 1, true>, WL}, {(const void*)k_epi<NT, -1, true>, WL}};
  for (const auto& f : fns) {
    hipError_t e = hipFuncSetAttribute(f.first, hipFuncAttributeMaxDynamicSharedMemorySize, mx(f.second));
    if (e != hipSuccess) return e;
  }
  for (const void* f : {(const void*)k_edge_mlp<NT, 1>, (const void*)k_edge_mlp<NT, -1>}) {  // no slab
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  if constexpr (NT >= 2) {  // wide pooling (one tile per workgroup)
    hipError_t e = hipFuncSetAttribute((const void*)k_pool_edge<NT, 2 * NT, 2 * NT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mx(2 * NT));
    if (e != hipSuccess) return e;
  }
  if constexpr (NT >= 2) {  // cooperative encoders
    for (const void* f : {(const void*)k_encode_coop<NT, 1, false, NT>, (const void*)k_encode_coop<NT, -1, false, NT>,
                          (const void*)k_encode_coop<NT, 1, true, NT>, (const void*)k_encode_coop<NT, -1, true, NT>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx(enc_coop_waves<NT>()));
      if (e != hipSuccess) return e;
    }
  }
  if constexpr (NT == 4) {  // F = 64 cooperative encoder on two waves per row tile
    for (const void* f : {(const void*)k_encode_coop<NT, 1, false, 2>, (const void*)k_encode_coop<NT, -1, false, 2>,
                          (const void*)k_encode_coop<NT, 1, true, 2>, (const void*)k_encode_coop<NT, -1, true, 2>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx(enc_coop_waves<NT>()));
      if (e != hipSuccess) return e;
    }
  }
  if constexpr (NT >= 2) {  // cooperative last hops (F = 32, 64)
    for (int prelu = 0; prelu < 2; ++prelu) {
      hipError_t e = hipFuncSetAttribute(hop_coop_kernel<NT>(prelu), hipFuncAttributeMaxDynamicSharedMemorySize, mx(kWaves));
      if (e != hipSuccess) return e;
    }
  }
  if constexpr (NT == 4) {  // F = 64 cooperative edge hops: a slab + exchange buffers per tile
    for (int pw = 2; pw <= 4; pw += 2) {
      for (int prelu = 0; prelu < 2; ++prelu)
        for (int last = 0; last < 2; ++last)
          for (int pool = 0; pool < 2; ++pool) {
            hipError_t e = hipFuncSetAttribute(edge_coop_kernel<NT>(prelu, last, pw, pool),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               edge_coop_lds_cap<NT>(pw, pool));
            if (e != hipSuccess) return e;
          }
    }
  }
  if constexpr (NT == 2) {  // cooperative edge hops: 160 KB minus slabs and exchange buffers
    for (int prelu = 0; prelu < 2; ++prelu)
      for (int last = 0; last < 2; ++last)
        for (int pool = 0; pool < 3; ++pool) {
          hipError_t e = hipFuncSetAttribute(edge_coop_kernel<NT>(prelu, last, 0, pool),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             edge_coop_lds_cap<NT>(2, pool));
          if (e != hipSuccess) return e;
        }
  }
  // persistent hop chains whose final phase is the layer's last hop (epilogue region in LDS)
  for (const void* f : {(const void*)k_hop_chain<NT, 1, true>, (const void*)k_hop_chain<NT, -1, true>}) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx(kWaves));
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int NT>
hipError_t launch_encode(const EncodeArgs& a, hipStream_t st) {
  if (a.Npad <= 0) return hipSuccess;
  if constexpr (NT == 4) {
    if (a.coop == 2) {  // F = 64 on two waves per row tile (MSW_ENC_COOP_P=2)
      constexpr int P = 2, WV = enc_coop_waves<NT>();
      const dim3 grid(a.Npad / ((WV / P) * kRowsPerWave)), block(64 * WV);
      const size_t sh = lds_bytes<NT>(a.lds_floats);
      if (a.dec.on) {
        if (a.c.prelu)
          hipLaunchKernelGGL((k_encode_coop<NT, 1, true, P>), grid, block, sh, st, a);
        else
          hipLaunchKernelGGL((k_encode_coop<NT, -1, true, P>), grid, block, sh, st, a);
      } else if (a.c.prelu) {
        hipLaunchKernelGGL((k_encode_coop<NT, 1, false, P>), grid, block, sh, st, a);
      } else {
        hipLaunchKernelGGL((k_encode_coop<NT, -1, false, P>), grid, block, sh, st, a);
      }
      return hipGetLastError();
    }
  }
  if constexpr (NT >= 2) {
    if (a.coop == NT) {  // P = NT waves per row tile (F = 32: 2, F = 64: 4)
      constexpr int P = NT, WV = enc_coop_waves<NT>();
      const dim3 grid(a.Npad / ((WV / P) * kRowsPerWave)), block(64 * WV);
      const size_t sh = lds_bytes<NT>(a.lds_floats);
      if (a.dec.on) {
        if (a.c.prelu)
          hipLaunchKernelGGL((k_encode_coop<NT, 1, true, P>), grid, block, sh, st, a);
        else
          hipLaunchKernelGGL((k_encode_coop<NT, -1, true, P>), grid, block, sh, st, a);
      } else if (a.c.prelu) {
        hipLaunchKernelGGL((k_encode_coop<NT, 1, false, P>), grid, block, sh, st, a);
      } else {
        hipLaunchKernelGGL((k_encode_coop<NT, -1, false, P>), grid, block, sh, st, a);
      }
      return hipGetLastError();
    }
  }
  const int n = a.Npad / kRowsPerBlock;
  const dim3 grid(a.max_blocks > 0 && n > a.max_blocks ? a.max_blocks : n), block(kBlock);
  const size_t sh = lds_bytes<NT>(a.lds_floats);
  if (a.dec.on) {
    if (a.c.prelu)
      hipLaunchKernelGGL((k_encode<NT, 1, true>), grid, block, sh, st, a);
    else
      hipLaunchKernelGGL((k_encode<NT, -1, true>), grid, block, sh, st, a);
  } else if (a.c.prelu) {
    hipLaunchKernelGGL((k_encode<NT, 1, false>), grid, block, sh, st, a);
  } else {
    hipLaunchKernelGGL((k_encode<NT, -1, false>), grid, block, sh, st, a);
  }
  return hipGetLastError();
}

// XCD packing of a one-round grid of g workgroups (b: the launch's argument copy): the
// fewest XCDs (1, 2, 4 <= c.xcd_max) that hold one workgroup per CU, else all eight
template <class A>
static inline dim3 xcd_grid(A& b, long g) {
  b.c.xcd = 0;
  for (int k = 1; k <= b.c.xcd_max && k < kXcds; k *= 2)
    if (g <= (long)kCusPerXcd * k) {
      b.c.xcd = k;
      return dim3((unsigned)(cdiv(g, k) * kXcds));
    }
  return dim3((unsigned)g);
}

// one tile per wave while that grid is resident at once; grid-stride loop beyond that
template <class A>
static inline bool tile_loop(const A& a) {
  return a.fit_blocks > 0 && a.max_blocks > 0 && cdiv(a.ntiles, kWaves) > a.fit_blocks;
}
template <class A>
static inline int tile_grid(const A& a) {
  return tile_loop(a) ? a.max_blocks : cdiv(a.ntiles, kWaves);
}

template <int NT>
static const void* edge_hop_kernel(int prelu, bool loop, int last) {
  if (loop) {
    if (last) return prelu ? (const void*)k_edge_hop<NT, 1, true, 1> : (const void*)k_edge_hop<NT, -1, true, 1>;
    return prelu ? (const void*)k_edge_hop<NT, 1, true, 0> : (const void*)k_edge_hop<NT, -1, true, 0>;
  }
  if (last) return prelu ? (const void*)k_edge_hop<NT, 1, false, 1> : (const void*)k_edge_hop<NT, -1, false, 1>;
  return prelu ? (const void*)k_edge_hop<NT, 1, false, 0> : (const void*)k_edge_hop<NT, -1, false, 0>;
}
template <int NT>
hipError_t launch_edge_mlp(const EdgeHopArgs& a, hipStream_t st) {
  if (a.nchunks <= 0) return hipSuccess;
  if (a.pipe) {
    const int n = cdiv(a.nchunks, kMlpPipeWaves);
    const dim3 grid(a.max_blocks > 0 && n > a.max_blocks ? a.max_blocks : n), block(64 * kMlpPipeWaves);
    if (a.c.prelu)
      hipLaunchKernelGGL((k_edge_mlp_pipe<NT, 1>), grid, block, eh_lds_bytes(a.reg.len), st, a);
    else
      hipLaunchKernelGGL((k_edge_mlp_pipe<NT, -1>), grid, block, eh_lds_bytes(a.reg.len), st, a);
    return hipGetLastError();
  }
  const int n = cdiv(a.nchunks, kMlpWaves);
  const dim3 grid(a.max_blocks > 0 && n > a.max_blocks ? a.max_blocks : n), block(64 * kMlpWaves);
  if (a.c.prelu)
    hipLaunchKernelGGL((k_edge_mlp<NT, 1>), grid, block, eh_lds_bytes(a.reg.len), st, a);
  else
    hipLaunchKernelGGL((k_edge_mlp<NT, -1>), grid, block, eh_lds_bytes(a.reg.len), st, a);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_edge_hop(const EdgeHopArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  if (a.coop == 2 || a.coop == 4) {  // waves per tile; 4: F = 64, one tile per workgroup
    const int fuse = a.pool.slots ? 1 : a.pool.parent ? 2 : 0;
    const void* f = edge_coop_kernel<NT>(a.c.prelu, a.last, a.coop, fuse);
    if (!f || (fuse && NT == 2 && a.coop != 2)) return hipErrorInvalidValue;
    EdgeHopArgs b = a;
    const dim3 grid = xcd_grid(b, a.coop == 4 ? a.ntiles : cdiv((long)a.ntiles * a.coop, kWaves));
    void* args[] = {&b};
    return hipLaunchKernel(f, grid, dim3(kBlock), args, a.wdirect ? 0 : eh_lds_bytes(a.reg_nf), st);
  }
  if (a.pool.slots || a.pool.parent) return hipErrorInvalidValue;  // fused into k_edge_coop only
  const bool loop = tile_loop(a);
  EdgeHopArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? (a.last ? edge_waves<NT, true, 1>() : edge_waves<NT, true, 0>()) : kWaves));
  const size_t sh = eh_lds_bytes(loop ? a.reg.len : a.reg_nf);
  void* args[] = {&b};
  return hipLaunchKernel(edge_hop_kernel<NT>(a.c.prelu, loop, a.last), grid, block, args, sh, st);
}
template <int NT>
hipError_t launch_hop_kernel(const HopArgs& a, bool loop, dim3 grid, dim3 block, hipStream_t st);
template <int NT>
hipError_t launch_hop(const HopArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  if (a.coop > 1 && a.last) {  // waves per tile = NT (2 for F = 32, 4 for F = 64)
    const void* f = hop_coop_kernel<NT>(a.c.prelu);
    if (!f) return hipErrorInvalidValue;
    HopArgs b = a;
    const dim3 grid = xcd_grid(b, cdiv((long)a.ntiles * a.coop, kWaves));
    void* args[] = {&b};
    return hipLaunchKernel(f, grid, dim3(kBlock), args, lds_bytes<NT>(a.reg.len), st);
  }
  if (a.rows && !a.last) {  // row-layout middle hop (large meshes)
    const int nt = cdiv(a.nrows, kRowsPerWave);
    const int grid = a.max_blocks > 0 ? std::min(a.max_blocks, cdiv(nt, kRowHopWaves)) : cdiv(nt, kRowHopWaves);
    hipLaunchKernelGGL((k_hop_rows<NT>), dim3(grid), dim3(64 * kRowHopWaves), 0, st, a);
    return hipGetLastError();
  }
  if constexpr (NT >= 2) {
    if (a.split && !a.last) {  // feature-split middle hop: two waves per tile
      HopArgs b = a;
      hipLaunchKernelGGL((k_hop_split<NT>), xcd_grid(b, cdiv((long)a.ntiles * 2, kWaves)), dim3(kBlock), 0, st, b);
      return hipGetLastError();
    }
  }
  const bool loop = tile_loop(a);
  HopArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? hop_waves<NT, true>() : kWaves));
  return launch_hop_kernel<NT>(b, loop, grid, block, st);
}
template <int NT>
hipError_t launch_hop_chain(const HopChainArgs& a, hipStream_t st) {
  if (a.h.ntiles <= 0) return hipSuccess;
  if (a.m < 2 || a.m > kMaxChainHops || a.G != cdiv(a.h.ntiles, kWaves) || a.G > kCusPerXcd || a.h.c.xcd_max < 1)
    return hipErrorInvalidValue;  // the grid must be one XCD's, one workgroup per CU
  HopChainArgs b = a;
  b.h.c.xcd = 1;
  const dim3 grid((unsigned)(a.G * kXcds)), block(kBlock);
  if (!a.h.last) {
    hipLaunchKernelGGL((k_hop_chain<NT, 1, false>), grid, block, 0, st, b);
  } else {
    const size_t sh = lds_bytes<NT>(a.h.reg.len);
    if (a.h.c.prelu)
      hipLaunchKernelGGL((k_hop_chain<NT, 1, true>), grid, block, sh, st, b);
    else
      hipLaunchKernelGGL((k_hop_chain<NT, -1, true>), grid, block, sh, st, b);
  }
  return hipGetLastError();
}
template <int NT>
hipError_t launch_hop_kernel(const HopArgs& a, bool loop, dim3 grid, dim3 block, hipStream_t st) {
  if (!a.last) {
    if (loop) hipLaunchKernelGGL((k_hop<NT, 1, false, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((k_hop<NT, 1, false, false>), grid, block, 0, st, a);
  } else {
    const size_t sh = lds_bytes<NT>(a.reg.len);
    if (a.c.prelu) {
      if (loop) hipLaunchKernelGGL((k_hop<NT, 1, true, true>), grid, block, sh, st, a);
      else hipLaunchKernelGGL((k_hop<NT, 1, true, false>), grid, block, sh, st, a);
    } else {
      if (loop) hipLaunchKernelGGL((k_hop<NT, -1, true, true>), grid, block, sh, st, a);
      else hipLaunchKernelGGL((k_hop<NT, -1, true, false>), grid, block, sh, st, a);
    }
  }
  return hipGetLastError();
}
template <int NT>
hipError_t launch_pool(const PoolArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  const size_t sh = lds_bytes<NT>(a.reg.len);
  if (!a.rows) {
    PoolArgs b = a;
    if constexpr (NT >= 2) {  // 2 NT waves per tile (one tile per workgroup)
      if (a.coop == 2 * NT) {
        hipLaunchKernelGGL((k_pool_edge<NT, 2 * NT, 2 * NT>), xcd_grid(b, a.ntiles), dim3(64 * 2 * NT), sh, st, b);
        return hipGetLastError();
      }
    }
    if constexpr (NT >= 2) {  // waves per tile: 2 (F = 32), 4 (F = 64)
      if (a.coop == NT) {
        hipLaunchKernelGGL((k_pool_edge<NT, NT>), xcd_grid(b, cdiv((long)a.ntiles * NT, kWaves)), dim3(kBlock), sh, st, b);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((k_pool_edge<NT>), xcd_grid(b, cdiv(a.ntiles, kWaves)), dim3(kBlock), sh, st, b);
    return hipGetLastError();
  }
  const bool loop = tile_loop(a);
  PoolArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? waves_of<NT, true>() : kWaves));
  if (loop)
    hipLaunchKernelGGL((k_pool<NT, true>), grid, block, sh, st, b);
  else
    hipLaunchKernelGGL((k_pool<NT, false>), grid, block, sh, st, b);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_epi(const EpiArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  const bool loop = tile_loop(a);
  EpiArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? waves_of<NT, true>() : kWaves));
  const size_t sh = lds_bytes<NT>(a.reg.len);
  if (a.c.prelu) {
    if (loop) hipLaunchKernelGGL((k_epi<NT, 1, true>), grid, block, sh, st, b);
    else hipLaunchKernelGGL((k_epi<NT, 1, false>), grid, block, sh, st, b);
  } else {
    if (loop) hipLaunchKernelGGL((k_epi<NT, -1, true>), grid, block, sh, st, b);
    else hipLaunchKernelGGL((k_epi<NT, -1, false>), grid, block, sh, st, b);
  }
  return hipGetLastError();
}
template <int NT>
hipError_t launch_rowmlp(const RowMlpArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  if (a.mode == 1)
    hipLaunchKernelGGL((k_rowmlp<NT, 1>), dim3(cdiv(a.R, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((k_rowmlp<NT, 0>), dim3(cdiv(a.R, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

// Workgroups of one launch resident on the whole chip (grid cap of the grid-stride kernels).
template <int NT, bool LOOP>
static const void* kernel_of(int kind, int prelu, int last) {
  switch (kind) {
    case 0: return prelu ? (const void*)k_encode<NT, 1, false> : (const void*)k_encode<NT, -1, false>;
    case 1: return edge_hop_kernel<NT>(prelu, LOOP, last);
    case 2:
      return !last ? (const void*)k_hop<NT, 1, false, LOOP>
                   : (prelu ? (const void*)k_hop<NT, 1, true, LOOP> : (const void*)k_hop<NT, -1, true, LOOP>);
    case 3: return (const void*)k_pool<NT, LOOP>;
    case 5: return (const void*)k_pool_edge<NT>;
    case 13:
      if constexpr (NT >= 2) return (const void*)k_pool_edge<NT, 2 * NT, 2 * NT>;
      return nullptr;
    case 6: return prelu ? (const void*)k_epi<NT, 1, LOOP> : (const void*)k_epi<NT, -1, LOOP>;
    case 7: return edge_coop_kernel<NT>(prelu, last);
    case 16: return edge_coop_kernel<NT>(prelu, last, 0, 1);
    case 12: return edge_coop_kernel<NT>(prelu, last, 2);
    case 9: return hop_coop_kernel<NT>(prelu);
    case 10: return prelu ? (const void*)k_edge_mlp<NT, 1> : (const void*)k_edge_mlp<NT, -1>;
    case 14: return (const void*)k_hop_rows<NT>;
    case 15: return prelu ? (const void*)k_edge_mlp_pipe<NT, 1> : (const void*)k_edge_mlp_pipe<NT, -1>;
    default: return nullptr;
  }
}
template <int NT>
int resident_blocks(int kind, int prelu, int last, size_t dyn_bytes, int loop) {
  const void* f = loop ? kernel_of<NT, true>(kind, prelu, last) : kernel_of<NT, false>(kind, prelu, last);
  int per_cu = 0, dev = 0, cus = 0;
  if (!f) return 0;
  const size_t dyn = (kind == 1 || kind == 7 || kind == 10 || kind == 12 || kind == 15) ? eh_lds_bytes((int)(dyn_bytes / 4))
                                                     : lds_bytes<NT>((int)(dyn_bytes / 4));
  const int block = kind == 1 ? 64 * (loop ? (last ? edge_waves<NT, true, 1>() : edge_waves<NT, true, 0>()) : kWaves)
                    : kind == 10 ? 64 * kMlpWaves
                    : kind == 15 ? 64 * kMlpPipeWaves
                    : kind == 13 ? 64 * 2 * NT
                    : kind == 14 ? 64 * kRowHopWaves
                    : kind == 2 ? 64 * (loop ? hop_waves<NT, true>() : kWaves)
                    : 64 * (loop && (kind == 3 || kind == 6) ? waves_of<NT, true>() : kWaves);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, block, dyn) != hipSuccess)
    return 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return per_cu > 0 ? per_cu * cus : 0;
}

#define MSW_INSTANTIATE(NT)                                                       \
  template hipError_t prepare_kernels<NT>();                                      \
  template int resident_blocks<NT>(int, int, int, size_t, int);                   \
  template hipError_t launch_encode<NT>(const EncodeArgs&, hipStream_t);          \
  template hipError_t launch_edge_hop<NT>(const EdgeHopArgs&, hipStream_t);       \
  template hipError_t launch_edge_mlp<NT>(const EdgeHopArgs&, hipStream_t);       \
  template hipError_t launch_hop<NT>(const HopArgs&, hipStream_t);                \
  template hipError_t launch_hop_chain<NT>(const HopChainArgs&, hipStream_t);     \
  template hipError_t launch_pool<NT>(const PoolArgs&, hipStream_t);              \
  template hipError_t launch_epi<NT>(const EpiArgs&, hipStream_t);                \
  template hipError_t launch_rowmlp<NT>(const RowMlpArgs&, hipStream_t);

}  // namespace msw
