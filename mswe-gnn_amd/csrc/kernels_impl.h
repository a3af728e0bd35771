// gfx950 (MI355X, CDNA4) kernels of the multi-scale SWE-GNN rollout (templates; the
// kernels_nt*.hip units instantiate them for F = 16, 32, 64).
//
// Layout
//  * every F-wide node / edge vector is fp32, row-major, unpadded (stride F).
//  * A wave owns 16 ROWS (nodes or edges).  Lane l works on row j = l & 15 and, in lane
//    group g = l >> 4, holds features 16t + 4g + r (r = 0..3) of every 16-feature tile t
//    in one f32x4 per tile.  That is exactly the accumulator layout of
//    v_mfma_f32_16x16x4_f32 with the row on the MFMA column (C/D: col = l & 15,
//    row = 4(l >> 4) + r) and, register for register, the B operand of the next layer
//    (k-step (t, r): lane group g supplies feature 16t + 4g + r).  Layers chain in
//    registers: no LDS, no lane shuffles between layers.  Packed A operand:
//    A[to][ti][lane][r] = W[16 to + (l & 15)][16 ti + 4 (l >> 4) + r] (host: plan.hip).
//  * f32 in / f32 accumulate MFMA = exact fp32 fma chains (no TF32 on gfx950).
//  * message passing pulls over CSR-by-destination, 16 destination rows per wave, 16-byte
//    loads; sums run in the reference's edge order; no atomics (bit-reproducible).
#pragma once
#include "engine.h"

namespace msw {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 64 * kWaves;

#define MSW_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// ---------------------------------------------------------------------------- helpers
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ float hsum(f32x4 v) { return (v.x + v.y) + (v.z + v.w); }

// sum over the 4 lane groups holding one row (lanes j, j+16, j+32, j+48)
__device__ __forceinline__ float row_sum(float v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int ACT>
__device__ __forceinline__ float act_static(float x, float slope) {
  if constexpr (ACT == 1) return x > 0.f ? x : slope * x;
  else if constexpr (ACT == 2) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == 3) return x > 0.f ? x : 0.1f * x;
  else if constexpr (ACT == 4) return x > 0.f ? x : expm1f(x);
  else if constexpr (ACT == 5) return x / (1.f + expf(-x));
  else if constexpr (ACT == 6) return 1.f / (1.f + expf(-x));
  else if constexpr (ACT == 7) return tanhf(x);
  else return x;
}
template <int ACT, int N>
__device__ __forceinline__ void act_tiles_static(f32x4 (&v)[N], float slope) {
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[t][r] = act_static<ACT>(v[t][r], slope);
}
// Activation on whole register tiles.  ACT >= 0: fixed at compile time (the PReLU kernels of
// every shipped configuration); ACT < 0: one wave-uniform switch outside the element loops.
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

// One nn.Linear (+ bias, + activation) on register tiles, compile-time shape TIN -> TOUT
// (make_mlp layer, models/models.py:121-146).  The TOUT accumulators are independent
// chains interleaved per k-step (hides the 40-cycle dependent MFMA latency).
template <int TIN, int TOUT, int ACT>
__device__ __forceinline__ void mfma_layer(const f32x4 (&in)[TIN], f32x4 (&out)[TOUT],
                                           const float* __restrict__ A, const float* __restrict__ b,
                                           int act, float slope, int lane, int g) {
  f32x4 acc[TOUT];
#pragma unroll
  for (int to = 0; to < TOUT; ++to) acc[to] = f32x4{0.f, 0.f, 0.f, 0.f};
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
  if (b) {
#pragma unroll
    for (int to = 0; to < TOUT; ++to) acc[to] = acc[to] + ld4(b + 16 * to + 4 * g);
  }
  act_tiles<ACT, TOUT>(acc, act, slope);
#pragma unroll
  for (int to = 0; to < TOUT; ++to) out[to] = acc[to];
}

template <int TIN, int TOUT, int ACT = -1>
__device__ __forceinline__ void run_layer(const f32x4 (&in)[TIN], f32x4 (&out)[TOUT],
                                          const LayerDev& L, const float* __restrict__ W,
                                          int lane, int g) {
  mfma_layer<TIN, TOUT, ACT>(in, out, W + L.a_off, L.b_off >= 0 ? W + L.b_off : nullptr, L.act,
                        L.slope, lane, g);
}

// make_mlp chain IN0 -> T -> ... -> T -> TL: the layer count m.n is a run-time value, every
// layer's shape is fixed at compile time (first IN0->T, or IN0->TL if m.n == 1; middle
// T->T; last T->TL), so all register arrays are statically indexed.
template <int IN0, int T, int TL, int ACT = -1>
__device__ __forceinline__ void run_mlp(const f32x4 (&in)[IN0], f32x4 (&out)[TL], const MlpDev& m,
                                        const float* __restrict__ W, int lane, int g) {
  if (m.n == 1) {
    run_layer<IN0, TL, ACT>(in, out, m.l[0], W, lane, g);
    return;
  }
  f32x4 h[T];
  run_layer<IN0, T, ACT>(in, h, m.l[0], W, lane, g);
  for (int li = 1; li + 1 < m.n; ++li) {
    f32x4 h2[T];
    run_layer<T, T, ACT>(h, h2, m.l[li], W, lane, g);
#pragma unroll
    for (int t = 0; t < T; ++t) h[t] = h2[t];
  }
  run_layer<T, TL, ACT>(h, out, m.l[m.n - 1], W, lane, g);
}

__device__ __forceinline__ int wave_row0() {
  return (blockIdx.x * kWaves + (threadIdx.x >> 6)) * kRowsPerWave;
}

// ---------------------------------------------------------------------------- encoders
// Static / dynamic node encoders incl. the water-level feature
// (MSGNN.forward models/gnn.py:284-294, GNN.forward :112-123).
template <int NT, int ACT>
__global__ __launch_bounds__(kBlock) void k_encode(EncodeArgs a) {
  constexpr int F = 16 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  if (a.io && blockIdx.x == 0 && threadIdx.x == 0) a.io->step += 1;
  const int r0 = wave_row0();
  if (r0 >= a.N) return;
  const int node = r0 + (lane & 15);
  const bool valid = node < a.N;
  const float* xr = a.x + (size_t)(a.perm ? a.perm[valid ? node : 0] : (valid ? node : 0)) * a.nnf;
  f32x4 A[NT];
  // static input [x_s, WL = DEM + h_t] in tile 0: lane group g holds features 4g..4g+3
  {
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * g + r;
      float val = 0.f;
      if (f < a.nstat_raw) val = xr[f];
      else if (a.with_wl && f == a.nstat_raw) val = xr[a.nstat_raw - 1] + xr[a.nnf - 2];
      v[r] = val;
    }
    const f32x4 in[1] = {v};
    run_mlp<1, NT, NT, ACT>(in, A, a.stat, a.W, lane, g);
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.xs + (size_t)node * F + 16 * t + 4 * g, A[t]);
    }
  }
  if (r0 >= a.xd_rows) return;
  {
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * g + r;
      v[r] = f < a.dyn ? xr[a.nstat_raw + f] : 0.f;
    }
    const f32x4 in[1] = {v};
    run_mlp<1, NT, NT, ACT>(in, A, a.dynm, a.W, lane, g);
    if (valid && node < a.xd_rows) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.xd + (size_t)node * F + 16 * t + 4 * g, A[t]);
    }
  }
}

// Plan-time per-row MLPs.  MODE 0: edge encoder chain (raw <= 16 features -> F -> ... -> F);
// MODE 1: edge part of a SWEGNN layer's first layer, Pe = W1[:, 4F:] e + b1 (F -> h1t tiles).
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
    run_mlp<TI, NT, TO>(in, out, a.m, a.W, lane, g);
  else
    run_layer<TI, TO>(in, out, a.m.l[0], a.W, lane, g);
  if (valid) {
#pragma unroll
    for (int t = 0; t < TO; ++t)
      if (t < a.out_tiles) st4(a.out + (size_t)row * a.out_stride + 16 * t + 4 * g, out[t]);
  }
}

// ---------------------------------------------------------------------------- node projection
// U = W1[:, x_s(row) | x_d(row)] [x_s; x_in] (gnn.py:414-417, row = source node)
// V = W1[:, x_s(col) | x_d(col)] [x_s; x_in] (col = receiving node)
// O = filter_matrix[0] x_in                  (gnn.py:401-402)
// blockIdx.y picks two consecutive output tiles of [U | V | O]: 5x the waves of a
// one-wave-per-row-tile kernel, a 32-MFMA chain per wave (latency, not throughput, bounds
// these small launches).
template <int NT>
__global__ __launch_bounds__(kBlock) void k_node_proj(NodeProjArgs a) {
  constexpr int F = 16 * NT, TM = 2 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int r0 = wave_row0();
  if (r0 >= a.R) return;
  const int q0 = 2 * blockIdx.y;  // first output tile of this block
  const int nU = a.h1t;
  const int li = r0 + (lane & 15);
  const bool valid = li < a.R;
  const size_t n = (size_t)a.r0 + (valid ? li : 0);
  f32x4 in[TM];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    in[t] = ld4(a.xs + n * F + 16 * t + 4 * g);
    in[NT + t] = a.xin ? ld4(a.xin + n * F + 16 * t + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int tn = a.xin ? TM : NT;  // x_in = 0: only the x_s tiles contribute
#pragma unroll
  for (int qq = 0; qq < 2; ++qq) {
    const int q = q0 + qq;
    int a_off, ti0, tin, tstride, to;
    float* dst;
    int stride;
    if (q < nU) {
      if (a.a_u < 0) continue;
      a_off = a.a_u; ti0 = 0; tin = tn; tstride = TM; to = q; dst = a.U; stride = 16 * nU;
    } else if (q < 2 * nU) {
      if (a.a_v < 0) continue;
      a_off = a.a_v; ti0 = 0; tin = tn; tstride = TM; to = q - nU; dst = a.V; stride = 16 * nU;
    } else if (q < 2 * nU + NT) {
      if (a.a_o < 0) continue;
      a_off = a.a_o; ti0 = NT; tin = a.xin ? NT : 0; tstride = NT; to = q - 2 * nU; dst = a.O; stride = F;
    } else {
      continue;
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ti = 0; ti < TM; ++ti) {
      if (ti >= ti0 && ti < ti0 + tin) {
        const f32x4 w = ld4(a.W + a_off + ((size_t)(to * tstride + (ti - ti0)) * 64 + lane) * 4);
        acc = MSW_MFMA(w.x, in[ti].x, acc);
        acc = MSW_MFMA(w.y, in[ti].y, acc);
        acc = MSW_MFMA(w.z, in[ti].z, acc);
        acc = MSW_MFMA(w.w, in[ti].w, acc);
      }
    }
    if (valid) st4(dst + n * stride + 16 * to + 4 * g, acc);
  }
}

// ---------------------------------------------------------------------------- edge MLP
// s_ij = MLP(x_s[row], x_s[col], x_d[row], x_d[col], e_ij), normalised (gnn.py:414-426).
// The first layer arrives pre-split: h1 = act(U[row] + V[col] + Pe[e]).  Computed ONCE per
// SWEGNN layer: its inputs do not change across the K hops (gnn.py:414-420 reads x_s, x_d).
template <int NT, int ACT>
__global__ __launch_bounds__(kBlock) void k_edge_mlp(EdgeMlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int F = 16 * NT, TM = 2 * NT;
  for (int i = threadIdx.x * 4; i < a.w_count; i += kBlock * 4) st4(smem + i, ld4(a.W + i));
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int ntiles = (a.E + kRowsPerWave - 1) / kRowsPerWave;
  const int hs = 16 * a.h1t;
  for (int tile = blockIdx.x * kWaves + (threadIdx.x >> 6); tile < ntiles; tile += gridDim.x * kWaves) {
    const int e = tile * kRowsPerWave + (lane & 15);
    const bool valid = e < a.E;
    const int ee = valid ? e : a.E - 1;
    const size_t sr = (size_t)a.src[ee], dc = (size_t)a.dst[ee];
    f32x4 H[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t < a.h1t) {
        const int off = 16 * t + 4 * g;
        const f32x4 u = ld4(a.U + sr * hs + off);
        const f32x4 v = ld4(a.V + dc * hs + off);
        const f32x4 p = a.Pe ? ld4(a.Pe + (size_t)ee * hs + off) : ld4(a.b1 + off);
        H[t] = (u + v) + p;
      } else {
        H[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    act_tiles<ACT, TM>(H, a.act1, a.slope1);
    if (a.rest.n > 0) {
      f32x4 o[NT];
      run_mlp<TM, TM, NT, ACT>(H, o, a.rest, smem, lane, g);
#pragma unroll
      for (int t = 0; t < NT; ++t) H[t] = o[t];
    }
    if (a.normalize) {
      float ss = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) ss += hsum(H[t] * H[t]);
      const float nrm = sqrtf(row_sum(ss));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 q = H[t] / nrm;
        q.x = (q.x == q.x) ? q.x : 0.f;  // masked_fill_(isnan, 0)
        q.y = (q.y == q.y) ? q.y : 0.f;
        q.z = (q.z == q.z) ? q.z : 0.f;
        q.w = (q.w == q.w) ? q.w : 0.f;
        H[t] = q;
      }
    }
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.s + (size_t)e * F + 16 * t + 4 * g, H[t]);
    }
  }
}

// ---------------------------------------------------------------------------- hop
// One SWEGNN hop (gnn.py:406-443), pull over CSR-by-destination, 16 destinations per wave:
//   active(e) = rowsum(out[src]) != 0 || rowsum(out[dst]) != 0          (gnn.py:408-411)
//   agg[c]    = sum_e active(e) * (out[c] - out[src]) * s_e  (edge order; gnn.py:430-438)
//   out'[c]   = out[c] + W_{k+1} agg[c]    (MFMA; + skip, + post activation)
template <int NT>
__global__ __launch_bounds__(kBlock) void k_hop(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int r0 = wave_row0();
  if (r0 >= a.R) return;
  const int li = r0 + (lane & 15);
  const bool valid = li < a.R;
  const size_t c = (size_t)a.n0 + (valid ? li : 0);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 oc[NT], agg[NT];
  float sc = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    oc[t] = a.own_zero ? z : ld4(a.in + c * F + 16 * t + 4 * g);
    sc += hsum(oc[t]);
    agg[t] = z;
  }
  const bool fc = row_sum(sc) != 0.f;
  const int e0 = valid ? a.rowptr[li] : 0, e1 = valid ? a.rowptr[li + 1] : 0;
  for (int e = e0; e < e1; ++e) {
    const size_t sidx = (size_t)a.src[e];
    f32x4 os[NT], sv[NT];
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      os[t] = ld4(a.in + sidx * F + 16 * t + 4 * g);
      sv[t] = ld4(a.s + (size_t)e * F + 16 * t + 4 * g);
      ss += hsum(os[t]);
    }
    const bool act = fc || (row_sum(ss) != 0.f);
    if (act) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 gv;
        if (a.grad) {
          gv = oc[t] - os[t];  // out[col] - out[row]
          if (a.upwind) {
            gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
            gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
          }
        } else {
          gv = os[t];          // s_ij * out[row]
        }
        agg[t] = agg[t] + gv * sv[t];
      }
    }
  }
  f32x4 res[NT];
  if (a.A) {  // filter W_{k+1} on the MFMA, agg already in B-operand layout
    f32x4 acc[NT];
#pragma unroll
    for (int to = 0; to < NT; ++to) acc[to] = z;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      f32x4 w[NT];
#pragma unroll
      for (int to = 0; to < NT; ++to) w[to] = ld4(a.A + ((size_t)(to * NT + ti) * 64 + lane) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int to = 0; to < NT; ++to) acc[to] = MSW_MFMA(w[to][r], agg[ti][r], acc[to]);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = oc[t] + acc[t];
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = oc[t] + agg[t];
  }
  if (a.skip) {
#pragma unroll
    for (int t = 0; t < NT; ++t) res[t] = res[t] + ld4(a.skip + c * F + 16 * t + 4 * g);
  }
  if (a.post_act) act_tiles<-1, NT>(res, a.post_act, a.post_slope);  // GNN gnn_activation
  if (valid) {
#pragma unroll
    for (int t = 0; t < NT; ++t) st4(a.out + c * F + 16 * t + 4 * g, res[t]);
  }
}

// ---------------------------------------------------------------------------- pooling
// scatter(x[fine], coarse, reduce='mean') (gnn.py:256): children summed in edge order,
// divided by max(count, 1).
template <int NT>
__global__ __launch_bounds__(kBlock) void k_pool(PoolArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int r0 = wave_row0();
  if (r0 >= a.R) return;
  const int li = r0 + (lane & 15);
  if (li >= a.R) return;
  const size_t c = (size_t)a.n0 + li;
  const int e0 = a.rowptr[li], e1 = a.rowptr[li + 1];
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = e0; e < e1; ++e) {
    const size_t ch = (size_t)a.child[e];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = acc[t] + ld4(a.in + ch * F + 16 * t + 4 * g);
  }
  const float cnt = (float)(e1 - e0 > 0 ? e1 - e0 : 1);
#pragma unroll
  for (int t = 0; t < NT; ++t) st4(a.out + c * F + 16 * t + 4 * g, acc[t] / cnt);
}

// ---------------------------------------------------------------------------- decoder
// tanh(x_up) -> node_decoder -> + learned residual -> ReLU -> small-depth mask
// (gnn.py:335-348, models.py:50-91); in rollout mode also use_prediction + BC of the next
// step (dataset.py:486-529) and the rollout write (train.py:93-95).
template <int NT, int ACT>
__global__ __launch_bounds__(kBlock) void k_decode(DecodeArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int r0 = wave_row0();
  if (r0 >= a.N) return;
  const int n = r0 + (lane & 15);
  const bool valid = n < a.N;
  const size_t ni = valid ? n : 0;
  f32x4 X0[NT], A[1];
#pragma unroll
  for (int t = 0; t < NT; ++t) X0[t] = ld4(a.xup + ni * F + 16 * t + 4 * g);
  act_tiles<-1, NT>(X0, a.pre_act, a.pre_slope);
  run_mlp<NT, NT, 1, ACT>(X0, A, a.dec, a.W, lane, g);
  if (!valid || g) return;  // lane group 0 holds output features 0 (h) and 1 (|q|)
  const int ext = a.perm ? a.perm[n] : n;
  float* xr = a.X + (size_t)(a.io ? n : ext) * a.nnf;
  const int nstat = a.nnf - a.dyn;
  float h = A[0].x, v = A[0].y;
  if (a.resw) {
    float rh = xr[nstat] * a.resw[0];
    float rv = xr[nstat + 1] * a.resw[1];
    for (int tau = 1; tau < a.p; ++tau) {
      rh = rh + xr[nstat + 2 * tau] * a.resw[2 * tau];
      rv = rv + xr[nstat + 2 * tau + 1] * a.resw[2 * tau + 1];
    }
    h = h + rh;
    v = v + rv;
  }
  h = h > 0.f ? h : 0.f;  // torch.relu
  v = v > 0.f ? v : 0.f;
  const float hm = h * (fabsf(h) > 1e-4f ? 1.f : 0.f);  // _mask_small_WD(epsilon=1e-4)
  const float vm = v * (h != 0.f ? 1.f : 0.f);
  if (!a.io) {
    a.y[(size_t)ext * 2 + 0] = hm;
    a.y[(size_t)ext * 2 + 1] = vm;
    return;
  }
  RolloutIO* io = a.io;
  const int t = io->step;
  io->out[((size_t)ext * 2 + 0) * io->T + t] = hm;
  io->out[((size_t)ext * 2 + 1) * io->T + t] = vm;
  for (int k = 0; k + 2 < a.dyn; ++k) xr[nstat + k] = xr[nstat + k + 2];
  xr[a.nnf - 2] = hm;
  xr[a.nnf - 1] = vm;
  const int b = a.bc_slot ? a.bc_slot[n] : -1;
  if (b >= 0 && t + 1 < io->bc_tstride) {
    for (int tau = 0; tau < a.p; ++tau)
      xr[nstat + (io->type_bc - 1) + 2 * tau] =
          io->bc[((size_t)b * a.p + tau) * io->bc_tstride + t + 1];
  }
}

// ---------------------------------------------------------------------------- launchers
static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

template <int NT>
hipError_t launch_encode(const EncodeArgs& a, hipStream_t st) {
  if (a.N <= 0) return hipSuccess;
  if (a.prelu_only)
    hipLaunchKernelGGL((k_encode<NT, 1>), dim3(cdiv(a.N, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((k_encode<NT, -1>), dim3(cdiv(a.N, kRowsPerBlock)), dim3(kBlock), 0, st, a);
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
template <int NT>
hipError_t launch_node_proj(const NodeProjArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  const int tiles = 2 * a.h1t + NT;
  hipLaunchKernelGGL(k_node_proj<NT>, dim3(cdiv(a.R, kRowsPerBlock), cdiv(tiles, 2)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_edge_mlp(const EdgeMlpArgs& a, hipStream_t st) {
  if (a.E <= 0) return hipSuccess;
  const int tiles = cdiv(a.E, kRowsPerWave);
  const int grid = std::min(cdiv(tiles, kWaves), 256 * 8);
  if (a.prelu_only)
    hipLaunchKernelGGL((k_edge_mlp<NT, 1>), dim3(grid), dim3(kBlock), a.w_count * sizeof(float), st, a);
  else
    hipLaunchKernelGGL((k_edge_mlp<NT, -1>), dim3(grid), dim3(kBlock), a.w_count * sizeof(float), st, a);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_hop(const HopArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hop<NT>, dim3(cdiv(a.R, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_pool(const PoolArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pool<NT>, dim3(cdiv(a.R, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_decode(const DecodeArgs& a, hipStream_t st) {
  if (a.N <= 0) return hipSuccess;
  if (a.prelu_only)
    hipLaunchKernelGGL((k_decode<NT, 1>), dim3(cdiv(a.N, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((k_decode<NT, -1>), dim3(cdiv(a.N, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

#define MSW_INSTANTIATE(NT)                                                       \
  template hipError_t launch_encode<NT>(const EncodeArgs&, hipStream_t);          \
  template hipError_t launch_rowmlp<NT>(const RowMlpArgs&, hipStream_t);          \
  template hipError_t launch_node_proj<NT>(const NodeProjArgs&, hipStream_t);     \
  template hipError_t launch_edge_mlp<NT>(const EdgeMlpArgs&, hipStream_t);       \
  template hipError_t launch_hop<NT>(const HopArgs&, hipStream_t);                \
  template hipError_t launch_pool<NT>(const PoolArgs&, hipStream_t);              \
  template hipError_t launch_decode<NT>(const DecodeArgs&, hipStream_t);

}  // namespace msw
