// gfx950 kernels: helpers, epilogues, tracing, LDS-DMA staging.
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

// ---------------------------------------------------------------------------- helpers
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
// Streaming (non-temporal) store for rows a large-mesh launch writes and nothing re-reads
// while they could still sit in L2 / the MALL (config 5's encoder: 1.26 GB per launch, 426 ->
// 367 us; on Zenodo-size meshes the next launch re-reads from cache and the hint loses, so
// only the grid-stride variants use it).  MSW_STREAM_ST=0: plain stores (A/B build variant).
#ifndef MSW_STREAM_ST
#define MSW_STREAM_ST 1
#endif
__device__ __forceinline__ void st4_stream(float* p, f32x4 v) {
  if constexpr (MSW_STREAM_ST)
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  else
    st4(p, v);
}
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

// s_ij / ||s_ij||, NaN -> 0 (gnn.py:424-426) over one edge row held as NT f32x4 per lane (the
// 4 lane groups of the row together), IEEE division.  (Round 6 measured a shared-reciprocal form
// of the compiler's division sequence -- 5 instead of 11 VALU per element, bit-identical -- and
// it ran slower: profiles/r06/ab_fastdiv.txt.)
template <int NT>
__device__ __forceinline__ void normalize_s(f32x4 (&sv)[NT]) {
#pragma clang fp contract(off)
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
// ACT = 1 (the compile-time PReLU of kernels launched with Common::prelu): max(x, slope x),
// two VALU ops instead of three (cmp, mul, select).  For slope <= 1, slope != 0 it equals
// x > 0 ? x : slope x for every x -- infinities and NaN included -- except the sign of a zero
// output when x = +0 and slope < 0 (+0 instead of -0), which no consumer can see: every PReLU
// output feeds an MFMA chain or a sum that starts from +0, or a comparison with 0.  The host
// checks the slopes per plan (plan.hip all_prelu); other slopes run the run-time switch, whose
// PReLU is ACT = 8 (the reference's form).
#ifndef MSW_PRELU_MAX
#define MSW_PRELU_MAX 1  // 0: the reference's form for ACT = 1 too (A/B build variant)
#endif
template <int ACT>
__device__ __forceinline__ float act_static(float x, float slope) {
  if constexpr (ACT == 1) return MSW_PRELU_MAX ? fmaxf(x, slope * x) : (x > 0.f ? x : slope * x);  // PReLU
  else if constexpr (ACT == 8) return x > 0.f ? x : slope * x;  // PReLU, any slope
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
  if constexpr (ACT == 1 && MSW_PRELU_MAX) {  // the products as packed pairs (v_pk_mul_f32)
#pragma unroll
    for (int t = 0; t < N; ++t) {
      const f32x4 m = v[t] * slope;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[t][r] = fmaxf(v[t][r], m[r]);
    }
  } else {
#pragma unroll
    for (int t = 0; t < N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[t][r] = act_static<ACT>(v[t][r], slope);
  }
}
// ACT >= 0: activation fixed at compile time (PReLU kernels of the shipped configs);
// ACT < 0: one wave-uniform switch outside the element loops.
template <int ACT, int N>
__device__ __forceinline__ void act_tiles(f32x4 (&v)[N], int act, float slope) {
  if constexpr (ACT >= 0) {
    act_tiles_static<ACT, N>(v, slope);
  } else {
    switch (act) {
      case 1: act_tiles_static<8, N>(v, slope); break;
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
template <int N, bool STREAM = false>
__device__ __forceinline__ void store_row(float* row, const f32x4 (&v)[N], int ntiles, int g) {
#pragma unroll
  for (int t = 0; t < N; ++t)
    if (t < ntiles) {
      if constexpr (STREAM)
        st4_stream(row + 16 * t + 4 * g, v[t]);
      else
        st4(row + 16 * t + 4 * g, v[t]);
    }
}

// ---------------------------------------------------------------------------- epilogues
// Projection of a SWEGNN layer (U, V, O) from [x_s ; x_in] of a node tile; H1T = tiles of
// the first edge-MLP layer (2F, or F for one-layer MLPs).
template <int NT, int H1T, bool STREAM = false>
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
    if (valid) store_row<H1T, STREAM>(d.U + n * (16 * H1T), acc, H1T, g);
  }
  if (d.a_v >= 0) {
    f32x4 acc[H1T];
    proj<T2, H1T>(in, acc, W + d.a_v, lane);
    if (valid) store_row<H1T, STREAM>(d.V + n * (16 * H1T), acc, H1T, g);
  }
  if (d.a_o >= 0) {
    f32x4 acc[NT];
    proj<NT, NT>(xin, acc, W + d.a_o, lane);
    if (valid) store_row<NT, STREAM>(d.O + n * F, acc, NT, g);
  }
}
template <int NT, bool STREAM = false>
__device__ __forceinline__ void np_project(const f32x4 (&xs)[NT], const f32x4 (&xin)[NT],
                                           const NpDesc& d, const float* W, size_t n, bool valid,
                                           int lane, int g) {
  if (d.h1t == 2 * NT)
    np_project_t<NT, 2 * NT, STREAM>(xs, xin, d, W, n, valid, lane, g);
  else
    np_project_t<NT, NT, STREAM>(xs, xin, d, W, n, valid, lane, g);
}

// U (or V) = W[:, blocks] [x_s ; x] with H1T output tiles, TIN input tiles.
template <int TIN, int H1T, int NT, bool STREAM = false>
__device__ __forceinline__ void side_proj_t(const f32x4 (&in)[TIN], const float* A, float* dst, size_t n,
                                            bool valid, int lane, int g) {
  f32x4 acc[H1T];
  proj<TIN, H1T>(in, acc, A, lane);
  if (valid) store_row<H1T, STREAM>(dst + n * (16 * H1T), acc, H1T, g);
}
template <int TIN, int NT, bool STREAM = false>
__device__ __forceinline__ void side_proj(const f32x4 (&in)[TIN], int h1t, const float* A, float* dst,
                                          size_t n, bool valid, int lane, int g) {
  if (h1t == 2 * NT)
    side_proj_t<TIN, 2 * NT, NT, STREAM>(in, A, dst, n, valid, lane, g);
  else
    side_proj_t<TIN, NT, NT, STREAM>(in, A, dst, n, valid, lane, g);
}

// Everything an epilogue reads from HBM that does not depend on the tile's result, loaded
// with the tile's gathers at kernel start instead of after the hop (one latency less on the
// chain): x_s rows for the projections, the decoder's dynamic state columns, the step.
constexpr int kMaxDyn = 16;
// Rollout-mode encoder: the next step's BC values issued before the weight staging (their
// round trip then overlaps the staging instead of the decoder MLP; zenodo4 +0.65 %,
// profiles/r04/ab_bc_hoist.txt) where there is a staging to overlap (F <= 32); F = 64 reads
// its operands from the blob and measured neutral.
template <int NT>
constexpr bool kBcHoist = NT <= 2;
template <int NT>
struct EpiPre {
  f32x4 xs[NT];
  float xd[kMaxDyn];  // X[row, nstat : nnf] (lane group 0 uses it)
  int ext, step;
  int bc;             // the row's BC slot (rollout mode), -1 = none
  float bcv[kMaxDyn / 2];  // deferred decoder: the row's BC values of step + 1 (bc_prefetch) ...
  float bck[kMaxDyn];      // ... or (BYCOL) the value for each state column it overwrites
};
// Deferred decoder (k_encode): the BC values the state update writes, loaded with the tile's
// other inputs instead of after the decoder chain (a BC row's wave would otherwise wait for
// one more global load on the launch's critical path).
// BYCOL: one load per state column (bck) instead of one per BC value (bcv): the state update
// then reads bck[k] at a compile-time index instead of selecting bcv[(k - c0) / 2] for every
// column (kMaxDyn x kMaxDyn / 2 selects), at the cost of kMaxDyn / 2 more live registers (the
// four-rank F = 64 encoder, at its 128-register cap, keeps bcv)
template <int NT, bool BYCOL = false>
__device__ __forceinline__ void bc_prefetch(EpiPre<NT>& p, const DecDesc& d, const Common& c) {
  const RolloutIO* io = d.io;
  const bool on = p.bc >= 0 && p.step + 1 < io->bc_tstride;
  const float* bp = on ? io->bc + (size_t)p.bc * c.p * io->bc_tstride + p.step + 1 : c.zrow;
  const int ts = on ? io->bc_tstride : 0;
  if constexpr (BYCOL) {  // wave-uniform column -> BC index map; other columns load bp[0], unused
    const int c0 = io->type_bc - 1;
#pragma unroll
    for (int k = 0; k < kMaxDyn; ++k) {
      const int u = (k - c0) >> 1;
      const bool col = k >= c0 && ((k - c0) & 1) == 0 && u < c.p;
      p.bck[k] = bp[col ? u * ts : 0];
    }
  } else {
#pragma unroll
    for (int u = 0; u < kMaxDyn / 2; ++u) p.bcv[u] = u < c.p ? bp[u * ts] : 0.f;
  }
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
template <int NT, bool BYCOL = false>
__device__ __forceinline__ void decode_state_tail(const f32x4 (&o)[1], const DecDesc& d, const Common& c,
                                                  const float* W, const EpiPre<NT>& pre, int n, bool valid,
                                                  int lane, int g, float (&nd)[kMaxDyn]);
template <int NT, int ACT, bool BYCOL = false>
__device__ __forceinline__ void decode_state(const f32x4 (&x)[NT], const DecDesc& d, const Common& c,
                                             const float* W, const EpiPre<NT>& pre, int n, bool valid,
                                             int lane, int g, float (&nd)[kMaxDyn]) {
#pragma clang fp contract(off)
  f32x4 x0[NT], o[1];
#pragma unroll
  for (int t = 0; t < NT; ++t) x0[t] = x[t];
  act_tiles<-1, NT>(x0, d.pre_act, d.pre_slope);
  run_mlp<NT, NT, 1, ACT>(x0, o, d.dec, W, lane, g);
  decode_state_tail<NT, BYCOL>(o, d, c, W, pre, n, valid, lane, g, nd);
}
template <int NT, bool BYCOL>
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
    float bv;
    if constexpr (BYCOL) {
      bv = pre.bck[k];
    } else {  // pre.bcv[tau] by selects (a run-time register index would use scratch)
      bv = 0.f;
#pragma unroll
      for (int u = 0; u < kMaxDyn / 2; ++u) bv = u == tau ? pre.bcv[u] : bv;
    }
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

// The dynamic encoder's input of this lane, state column 4 g + q (0 past dyn), from the row's
// new state nd (every lane of a row holds all of it): a 4-way select on the lane group instead of
// one select per column.
__device__ __forceinline__ float nd_column(const float (&nd)[kMaxDyn], int g, int q, int dyn) {
  static_assert(kMaxDyn == 16, "four lane groups x four columns");
  const float v = g == 0 ? nd[q] : g == 1 ? nd[4 + q] : g == 2 ? nd[8 + q] : nd[12 + q];
  return 4 * g + q < dyn ? v : 0.f;
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
