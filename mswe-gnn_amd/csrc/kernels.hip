// gfx950 (MI355X, CDNA4) kernels of the multi-scale SWE-GNN rollout.
//
// Layout conventions:
//  * every F-wide node / edge vector is stored fp32, row-major, padded to FP (32 or 64)
//    floats with zero pads; F=16 models run zero-padded to FP=32 (exact: pads stay 0).
//  * dense per-row MLPs run on the f32-input MFMA v_mfma_f32_32x32x2_f32 with the ROW
//    (node or edge) on the lane: a wave owns 32 rows, lane l works on row l&31 and holds,
//    for every 32-feature tile t, the 16 features 32t+16h+r (h = l>>5, r = 0..15) in the
//    16 accumulator registers.  Output tile rows are permuted on the host when packing the
//    A operand (weights) so that the accumulator of one layer is, register for register,
//    the B operand of the next: no LDS or lane shuffles between layers.
//  * message passing (hops, pooling) pulls over CSR-by-destination with FP/4 lanes per
//    node and 16-byte loads; sums run in the reference's edge order, no atomics.
#include "engine.h"

namespace msw {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------- helpers
__device__ __forceinline__ float act_fn(int act, float x, float slope) {
  // activation_functions, models/models.py:149-169
  switch (act) {
    case 1: return x > 0.f ? x : slope * x;          // PReLU
    case 2: return x > 0.f ? x : 0.f;                // ReLU
    case 3: return x > 0.f ? x : 0.1f * x;           // LeakyReLU(0.1)
    case 4: return x > 0.f ? x : expm1f(x);          // ELU
    case 5: return x / (1.f + expf(-x));             // SiLU
    case 6: return 1.f / (1.f + expf(-x));           // Sigmoid
    case 7: return tanhf(x);                         // Tanh
    default: return x;
  }
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

__device__ __forceinline__ f32x16 ld16(const float* p) {
  const f32x4 a = ld4(p), b = ld4(p + 4), c = ld4(p + 8), d = ld4(p + 12);
  f32x16 v;
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  v[8] = c.x; v[9] = c.y; v[10] = c.z; v[11] = c.w;
  v[12] = d.x; v[13] = d.y; v[14] = d.z; v[15] = d.w;
  return v;
}
__device__ __forceinline__ void st16(float* p, const f32x16& v) {
  st4(p, f32x4{v[0], v[1], v[2], v[3]});
  st4(p + 4, f32x4{v[4], v[5], v[6], v[7]});
  st4(p + 8, f32x4{v[8], v[9], v[10], v[11]});
  st4(p + 12, f32x4{v[12], v[13], v[14], v[15]});
}

// One output tile: sum over input tiles [ti0, ti0+tn) of A[to][ti - ti0] * in[ti].
// A packed as [tout][tstride][r4][lane][4] floats (host: pack_operand in plan.hip); only the
// first tn of the tstride packed input tiles are used.
template <int TM>
__device__ __forceinline__ f32x16 mfma_tile(const f32x16 (&in)[TM], int ti0, int tn,
                                            const float* __restrict__ A, int to, int lane,
                                            int tstride) {
  f32x16 acc = {};
#pragma unroll
  for (int ti = 0; ti < TM; ++ti) {
    if (ti >= ti0 && ti < ti0 + tn) {
      const f32x4* Ap = reinterpret_cast<const f32x4*>(A) + ((to * tstride + (ti - ti0)) * 4) * 64 + lane;
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const f32x4 a = Ap[r4 * 64];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, in[ti][4 * r4 + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, in[ti][4 * r4 + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, in[ti][4 * r4 + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, in[ti][4 * r4 + 3], acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

__device__ __forceinline__ void bias_act(f32x16& acc, const float* __restrict__ b, int act,
                                         float slope) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = acc[r];
    if (b) v = v + b[r];
    acc[r] = act_fn(act, v, slope);
  }
}

// nn.Linear + activation on register tiles (make_mlp layer, models/models.py:121-146).
template <int TM>
__device__ __forceinline__ void mfma_layer(const f32x16 (&in)[TM], f32x16 (&out)[TM],
                                           const LayerDev& L, const float* __restrict__ W,
                                           int lane, int half) {
#pragma unroll
  for (int to = 0; to < TM; ++to) {
    if (to < L.tout) {
      f32x16 acc = mfma_tile<TM>(in, 0, L.tin, W + L.a_off, to, lane, L.tin);
      bias_act(acc, L.b_off >= 0 ? W + L.b_off + 32 * to + 16 * half : nullptr, L.act, L.slope);
      out[to] = acc;
    }
  }
}

// Layers [LI, m.n) of an MLP (compile-time unrolled, runtime layer count).
template <int TM, int LI, int FIRST>
__device__ __forceinline__ void chain_step(f32x16 (&a)[TM], f32x16 (&b)[TM], const MlpDev& m,
                                           const float* __restrict__ W, int lane, int half) {
  if constexpr (LI < kMaxLayers) {
    if (LI < m.n) {
      if constexpr (((LI - FIRST) & 1) == 0)
        mfma_layer<TM>(a, b, m.l[LI], W, lane, half);
      else
        mfma_layer<TM>(b, a, m.l[LI], W, lane, half);
      chain_step<TM, LI + 1, FIRST>(a, b, m, W, lane, half);
    }
  }
}

// Layers [FIRST, m.n) of an MLP, starting in `a`; the result ends in `a`.
template <int TM, int FIRST>
__device__ __forceinline__ void run_chain(f32x16 (&a)[TM], f32x16 (&b)[TM], const MlpDev& m,
                                          const float* __restrict__ W, int lane, int half) {
  chain_step<TM, FIRST, FIRST>(a, b, m, W, lane, half);
  const bool odd = ((m.n - FIRST) > 0) && ((m.n - FIRST) & 1);
#pragma unroll
  for (int t = 0; t < TM; ++t) a[t] = odd ? b[t] : a[t];
}

// sum over the LPN lanes of a node group (xor butterfly inside the group)
template <int LPN>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < LPN; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------- encoders
// Static / dynamic node encoders incl. the water-level feature
// (MSGNN.forward models/gnn.py:284-294, GNN.forward :112-123).
template <int FP>
__global__ __launch_bounds__(kBlock) void k_encode(EncodeArgs a) {
  constexpr int T = FP / 32;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  if (a.io && blockIdx.x == 0 && threadIdx.x == 0) a.io->step += 1;
  const int node = ((blockIdx.x * kBlock + threadIdx.x) >> 6) * 32 + (lane & 31);
  if (((blockIdx.x * kBlock + threadIdx.x) >> 6) * 32 >= a.N) return;  // whole wave out
  const bool valid = node < a.N;
  const int ni = valid ? node : 0;
  const float* xr = a.x + (size_t)(a.perm ? a.perm[ni] : ni) * a.nnf;
  f32x16 A[T], B[T];
  {
    f32x16 v = {};
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int f = 16 * half + r;
      float val = 0.f;
      if (f < a.nstat_raw) val = xr[f];
      else if (a.with_wl && f == a.nstat_raw) val = xr[a.nstat_raw - 1] + xr[a.nnf - 2];
      v[r] = val;
    }
    A[0] = v;
#pragma unroll
    for (int t = 1; t < T; ++t) A[t] = f32x16{};
    run_chain<T, 0>(A, B, a.stat, a.W, lane, half);
    if (valid) {
#pragma unroll
      for (int t = 0; t < T; ++t) st16(a.xs + (size_t)node * FP + 32 * t + 16 * half, A[t]);
    }
  }
  if (((blockIdx.x * kBlock + threadIdx.x) >> 6) * 32 >= a.xd_rows) return;
  {
    f32x16 v = {};
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int f = 16 * half + r;
      v[r] = f < a.dyn ? xr[a.nstat_raw + f] : 0.f;
    }
    A[0] = v;
#pragma unroll
    for (int t = 1; t < T; ++t) A[t] = f32x16{};
    run_chain<T, 0>(A, B, a.dynm, a.W, lane, half);
    if (valid && node < a.xd_rows) {
#pragma unroll
      for (int t = 0; t < T; ++t) st16(a.xd + (size_t)node * FP + 32 * t + 16 * half, A[t]);
    }
  }
}

// Generic per-row MLP (edge encoder, edge-feature projection of the edge MLP's first layer).
template <int TM>
__global__ __launch_bounds__(kBlock) void k_rowmlp(RowMlpArgs a) {
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const int wbase = ((blockIdx.x * kBlock + threadIdx.x) >> 6) * 32;
  if (wbase >= a.R) return;
  const int row = wbase + (lane & 31);
  const bool valid = row < a.R;
  const float* xr = a.in + (size_t)(valid ? row : 0) * a.in_stride;
  f32x16 A[TM], B[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    f32x16 v = {};
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int f = 32 * t + 16 * half + r;
      v[r] = f < a.in_dim ? xr[f] : 0.f;
    }
    A[t] = v;
  }
  run_chain<TM, 0>(A, B, a.m, a.W, lane, half);
  if (valid) {
    const int tout = a.m.l[a.m.n - 1].tout;
#pragma unroll
    for (int t = 0; t < TM; ++t)
      if (t < tout) st16(a.out + (size_t)row * a.out_stride + 32 * t + 16 * half, A[t]);
  }
}

// ---------------------------------------------------------------------------- node projection
// Node-side part of the SWEGNN edge MLP's first layer and the first filter:
//   U = W1[:, x_s(row) | x_d(row)] . [x_s; x_in]   (gnn.py:414-417, row = source)
//   V = W1[:, x_s(col) | x_d(col)] . [x_s; x_in]   (col = target)
//   O = filter_matrix[0] . x_in                    (gnn.py:401-402)
template <int FP>
__global__ __launch_bounds__(kBlock) void k_node_proj(NodeProjArgs a) {
  constexpr int T = FP / 32, TM = 2 * T;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const int wbase = ((blockIdx.x * kBlock + threadIdx.x) >> 6) * 32;
  if (wbase >= a.R) return;
  const int li = wbase + (lane & 31);
  const bool valid = li < a.R;
  const size_t n = (size_t)a.r0 + (valid ? li : 0);
  f32x16 in[TM];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    in[t] = ld16(a.xs + n * FP + 32 * t + 16 * half);
    in[T + t] = a.xin ? ld16(a.xin + n * FP + 32 * t + 16 * half) : f32x16{};
  }
  const int tn = a.xin ? 2 * T : T;  // with x_in = 0 only the x_s tiles contribute
  if (a.a_u >= 0) {
#pragma unroll
    for (int to = 0; to < TM; ++to)
      if (to < a.h1t) {
        f32x16 acc = mfma_tile<TM>(in, 0, tn, a.W + a.a_u, to, lane, 2 * T);
        if (valid) st16(a.U + n * (32 * a.h1t) + 32 * to + 16 * half, acc);
      }
  }
  if (a.a_v >= 0) {
#pragma unroll
    for (int to = 0; to < TM; ++to)
      if (to < a.h1t) {
        f32x16 acc = mfma_tile<TM>(in, 0, tn, a.W + a.a_v, to, lane, 2 * T);
        if (valid) st16(a.V + n * (32 * a.h1t) + 32 * to + 16 * half, acc);
      }
  }
  if (a.a_o >= 0) {
#pragma unroll
    for (int to = 0; to < T; ++to) {
      f32x16 acc = a.xin ? mfma_tile<TM>(in, T, T, a.W + a.a_o, to, lane, T) : f32x16{};
      if (valid) st16(a.O + n * FP + 32 * to + 16 * half, acc);
    }
  }
}

// ---------------------------------------------------------------------------- edge MLP
// s_ij = MLP(x_s[row], x_s[col], x_d[row], x_d[col], e_ij), normalised (gnn.py:414-426).
// The first layer arrives pre-split: h1 = act(U[row] + V[col] + Pe[e]).  Computed ONCE per
// SWEGNN layer: its inputs (x_s, x_d, e_ij) do not change across the K hops.
template <int FP>
__global__ __launch_bounds__(kBlock) void k_edge_mlp(EdgeMlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int T = FP / 32, TM = 2 * T;
  for (int i = threadIdx.x * 4; i < a.w_count; i += kBlock * 4) st4(smem + i, ld4(a.W + i));
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const int ntiles = (a.E + 31) / 32;
  const int hstride = 32 * a.h1t;
  for (int tile = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); tile < ntiles;
       tile += gridDim.x * (kBlock / 64)) {
    const int e = tile * 32 + (lane & 31);
    const bool valid = e < a.E;
    const int ee = valid ? e : a.E - 1;
    const size_t sr = (size_t)a.src[ee], dc = (size_t)a.dst[ee];
    f32x16 H[TM], G[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t < a.h1t) {
        const int off = 32 * t + 16 * half;
        f32x16 u = ld16(a.U + sr * hstride + off);
        const f32x16 v = ld16(a.V + dc * hstride + off);
        const f32x16 p = a.Pe ? ld16(a.Pe + (size_t)ee * hstride + off) : ld16(a.b1 + off);
#pragma unroll
        for (int r = 0; r < 16; ++r) u[r] = act_fn(a.act1, (u[r] + v[r]) + p[r], a.slope1);
        H[t] = u;
      } else {
        H[t] = f32x16{};
      }
    }
    run_chain<TM, 0>(H, G, a.rest, smem, lane, half);
    if (a.normalize) {
      float ss = 0.f;
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) ss += H[t][r] * H[t][r];
      ss += __shfl_xor(ss, 32);
      const float nrm = sqrtf(ss);
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float q = H[t][r] / nrm;
          H[t][r] = (q == q) ? q : 0.f;  // masked_fill_(isnan, 0)
        }
    }
    if (valid) {
#pragma unroll
      for (int t = 0; t < T; ++t) st16(a.s + (size_t)e * FP + 32 * t + 16 * half, H[t]);
    }
  }
}

// ---------------------------------------------------------------------------- hop
// One SWEGNN hop (gnn.py:406-443) as a pull over CSR-by-destination:
//   active(e) = rowsum(out[src]) != 0 || rowsum(out[dst]) != 0
//   agg[c]    = sum_e active(e) * (out[c] - out[src]) * s_e      (edge order)
//   out'[c]   = out[c] + W_{k+1} agg[c]        (+ skip, + post activation)
template <int FP>
__global__ __launch_bounds__(kBlock) void k_hop(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int LPN = FP / 4;   // lanes per node
  constexpr int NPW = 64 / LPN; // nodes per wave
  constexpr int NPB = NPW * (kBlock / 64);
  constexpr int AS = FP + 4;    // padded LDS row
  __shared__ __attribute__((aligned(16))) float sW[FP * FP];
  __shared__ __attribute__((aligned(16))) float sA[NPB * AS];
  if (a.WT) {
    for (int i = threadIdx.x * 4; i < FP * FP; i += kBlock * 4) st4(sW + i, ld4(a.WT + i));
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane / LPN, j = lane % LPN;
  const int slot = wv * NPW + g;
  const int li = blockIdx.x * NPB + slot;
  const bool valid = li < a.R;
  const size_t c = (size_t)a.n0 + (valid ? li : 0);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const f32x4 oc = (a.in && !a.own_zero) ? ld4(a.in + c * FP + 4 * j) : zero;
  const bool fc = group_sum<LPN>((oc.x + oc.y) + (oc.z + oc.w)) != 0.f;
  f32x4 agg = zero;
  const int e0 = valid ? a.rowptr[li] : 0, e1 = valid ? a.rowptr[li + 1] : 0;
  for (int e = e0; e < e1; ++e) {
    const size_t sidx = (size_t)a.src[e];
    const f32x4 os = ld4(a.in + sidx * FP + 4 * j);
    const bool fs = group_sum<LPN>((os.x + os.y) + (os.z + os.w)) != 0.f;
    const f32x4 sv = ld4(a.s + (size_t)e * FP + 4 * j);
    f32x4 gv;
    if (a.grad) {
      gv = oc - os;  // out[col] - out[row]
      if (a.upwind) {
        gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
        gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
      }
    } else {
      gv = os;       // s_ij * out[row]
    }
    if (fc || fs) agg = agg + gv * sv;
  }
  f32x4 res;
  if (a.WT) {
    st4(sA + slot * AS + 4 * j, agg);
    __syncthreads();
    f32x4 acc = zero;
#pragma unroll
    for (int i4 = 0; i4 < FP / 4; ++i4) {
      const f32x4 av = ld4(sA + slot * AS + 4 * i4);
      const f32x4 w0 = ld4(sW + (4 * i4 + 0) * FP + 4 * j);
      const f32x4 w1 = ld4(sW + (4 * i4 + 1) * FP + 4 * j);
      const f32x4 w2 = ld4(sW + (4 * i4 + 2) * FP + 4 * j);
      const f32x4 w3 = ld4(sW + (4 * i4 + 3) * FP + 4 * j);
      acc = __builtin_elementwise_fma(f32x4{av.x, av.x, av.x, av.x}, w0, acc);
      acc = __builtin_elementwise_fma(f32x4{av.y, av.y, av.y, av.y}, w1, acc);
      acc = __builtin_elementwise_fma(f32x4{av.z, av.z, av.z, av.z}, w2, acc);
      acc = __builtin_elementwise_fma(f32x4{av.w, av.w, av.w, av.w}, w3, acc);
    }
    res = oc + acc;
  } else {
    res = oc + agg;
  }
  if (a.skip) res = res + ld4(a.skip + c * FP + 4 * j);
  if (a.post_act) {
    res.x = act_fn(a.post_act, res.x, a.post_slope); res.y = act_fn(a.post_act, res.y, a.post_slope);
    res.z = act_fn(a.post_act, res.z, a.post_slope); res.w = act_fn(a.post_act, res.w, a.post_slope);
  }
  if (valid) st4(a.out + c * FP + 4 * j, res);
}

// ---------------------------------------------------------------------------- pooling
// scatter(x[fine], coarse, reduce='mean') (gnn.py:256): children summed in edge order,
// divided by max(count, 1).
template <int FP>
__global__ __launch_bounds__(kBlock) void k_pool(PoolArgs a) {
#pragma clang fp contract(off)
  constexpr int LPN = FP / 4, NPW = 64 / LPN, NPB = NPW * (kBlock / 64);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane / LPN, j = lane % LPN;
  const int li = blockIdx.x * NPB + wv * NPW + g;
  if (li >= a.R) return;
  const size_t c = (size_t)a.n0 + li;
  const int e0 = a.rowptr[li], e1 = a.rowptr[li + 1];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int e = e0; e < e1; ++e) acc = acc + ld4(a.in + (size_t)a.child[e] * FP + 4 * j);
  const float cnt = (float)(e1 - e0 > 0 ? e1 - e0 : 1);
  st4(a.out + c * FP + 4 * j, acc / cnt);
}

// ---------------------------------------------------------------------------- decoder
// tanh(x_up) -> node_decoder -> + learned residual -> ReLU -> small-depth mask
// (gnn.py:335-348, models.py:50-91); in rollout mode also use_prediction + BC of the next
// step (dataset.py:486-529) and the rollout write (train.py:93-95).
template <int FP>
__global__ __launch_bounds__(kBlock) void k_decode(DecodeArgs a) {
#pragma clang fp contract(off)
  constexpr int T = FP / 32;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const int wbase = ((blockIdx.x * kBlock + threadIdx.x) >> 6) * 32;
  if (wbase >= a.N) return;
  const int n = wbase + (lane & 31);
  const bool valid = n < a.N;
  const size_t ni = valid ? n : 0;
  f32x16 A[T], B[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    f32x16 v = ld16(a.xup + ni * FP + 32 * t + 16 * half);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = act_fn(a.pre_act, v[r], a.pre_slope);
    A[t] = v;
  }
  run_chain<T, 0>(A, B, a.dec, a.W, lane, half);
  if (!valid || half) return;
  const int ext = a.perm ? a.perm[n] : n;
  float* xr = a.X + (size_t)(a.io ? n : ext) * a.nnf;
  const int nstat = a.nnf - a.dyn;
  float h = A[0][0], v = A[0][1];
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

// x (graph numbering) -> internal rollout state + BC of step 0
__global__ __launch_bounds__(kBlock) void k_init_state(InitArgs a) {
  const int n = blockIdx.x * kBlock + threadIdx.x;
  if (n == 0) a.io->step = -1;
  if (n >= a.N) return;
  const int ext = a.perm ? a.perm[n] : n;
  float* xr = a.X + (size_t)n * a.nnf;
  const float* src = a.x0 + (size_t)ext * a.nnf;
  for (int k = 0; k < a.nnf; ++k) xr[k] = src[k];
  const int b = a.bc_slot ? a.bc_slot[n] : -1;
  if (b >= 0) {
    const int nstat = a.nnf - a.dyn;
    for (int tau = 0; tau < a.p; ++tau)
      xr[nstat + (a.io->type_bc - 1) + 2 * tau] = a.io->bc[((size_t)b * a.p + tau) * a.io->bc_tstride];
  }
}

__global__ void k_set_slots(SlotArgs a) {
  const int i = threadIdx.x;
  if (i < a.n) a.slot[a.row[i]] = a.val[i];
}
__global__ void k_set_io(RolloutIO* dst, RolloutIO v) {
  if (threadIdx.x == 0) *dst = v;
}

// ---------------------------------------------------------------------------- launchers
hipError_t launch_set_slots(const SlotArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_set_slots, dim3(1), dim3(kSlotBatch), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_set_io(RolloutIO* dst, const RolloutIO& v, hipStream_t st) {
  hipLaunchKernelGGL(k_set_io, dim3(1), dim3(64), 0, st, dst, v);
  return hipGetLastError();
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

template <int FP>
hipError_t launch_encode(const EncodeArgs& a, hipStream_t st) {
  if (a.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode<FP>, dim3(cdiv(a.N, 128)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int FP>
hipError_t launch_rowmlp(const RowMlpArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rowmlp<2 * FP / 32>, dim3(cdiv(a.R, 128)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int FP>
hipError_t launch_node_proj(const NodeProjArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_node_proj<FP>, dim3(cdiv(a.R, 128)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int FP>
hipError_t launch_edge_mlp(const EdgeMlpArgs& a, hipStream_t st) {
  if (a.E <= 0) return hipSuccess;
  const int tiles = cdiv(a.E, 32);
  const int grid = std::min(cdiv(tiles, kBlock / 64), 256 * 8);
  hipLaunchKernelGGL(k_edge_mlp<FP>, dim3(grid), dim3(kBlock), a.w_count * sizeof(float), st, a);
  return hipGetLastError();
}
template <int FP>
hipError_t launch_hop(const HopArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  constexpr int NPB = (64 / (FP / 4)) * (kBlock / 64);
  hipLaunchKernelGGL(k_hop<FP>, dim3(cdiv(a.R, NPB)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int FP>
hipError_t launch_pool(const PoolArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  constexpr int NPB = (64 / (FP / 4)) * (kBlock / 64);
  hipLaunchKernelGGL(k_pool<FP>, dim3(cdiv(a.R, NPB)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
template <int FP>
hipError_t launch_decode(const DecodeArgs& a, hipStream_t st) {
  if (a.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_decode<FP>, dim3(cdiv(a.N, 128)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_init_state(const InitArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_init_state, dim3(cdiv(a.N > 0 ? a.N : 1, kBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

#define MSW_INST(FP)                                                              \
  template hipError_t launch_encode<FP>(const EncodeArgs&, hipStream_t);          \
  template hipError_t launch_rowmlp<FP>(const RowMlpArgs&, hipStream_t);          \
  template hipError_t launch_node_proj<FP>(const NodeProjArgs&, hipStream_t);     \
  template hipError_t launch_edge_mlp<FP>(const EdgeMlpArgs&, hipStream_t);       \
  template hipError_t launch_hop<FP>(const HopArgs&, hipStream_t);                \
  template hipError_t launch_pool<FP>(const PoolArgs&, hipStream_t);              \
  template hipError_t launch_decode<FP>(const DecodeArgs&, hipStream_t);
MSW_INST(32)
MSW_INST(64)

}  // namespace msw
