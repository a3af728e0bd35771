// gfx950 kernels: cooperative edge hops (incl. fused pooling / unpooling).
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

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
// One layer's operands for output tiles [to0, to0 + TS), loaded ahead of the layer (the
// blob operands of F = 64 come from L2: issued one layer early, their round trip overlaps the
// previous layer's MFMA chain and exchange instead of following it); ops_layer is
// mfma_layer_sub's arithmetic in the same order (proj's k order, then the bias).
template <int TIN, int TS>
struct LayerOps {
  f32x4 w[TIN][TS];
  f32x4 b[TS];
};
template <int TIN, int TS>
__device__ __forceinline__ void ops_load(LayerOps<TIN, TS>& o, const LayerDev& L, const float* __restrict__ W,
                                         int to0, int lane, int g) {
  const float* A = W + L.a_off + (size_t)to0 * TIN * 256;
#pragma unroll
  for (int ti = 0; ti < TIN; ++ti)
#pragma unroll
    for (int to = 0; to < TS; ++to) o.w[ti][to] = ld4(A + ((size_t)(to * TIN + ti) * 64 + lane) * 4);
#pragma unroll
  for (int to = 0; to < TS; ++to) o.b[to] = ld4(W + L.b_off + 16 * (to0 + to) + 4 * g);  // zeros if bias=False
}
template <int TIN, int TS, int ACT>
__device__ __forceinline__ void ops_layer(const f32x4 (&in)[TIN], f32x4 (&out)[TS], const LayerOps<TIN, TS>& o,
                                          const LayerDev& L) {
  f32x4 acc[TS];
#pragma unroll
  for (int to = 0; to < TS; ++to) acc[to] = zero4();
#pragma unroll
  for (int ti = 0; ti < TIN; ++ti)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int to = 0; to < TS; ++to) acc[to] = MSW_MFMA(o.w[ti][to][r], in[ti][r], acc[to]);
#pragma unroll
  for (int to = 0; to < TS; ++to) acc[to] = acc[to] + o.b[to];
  act_tiles<ACT, TS>(acc, L.act, L.slope);
#pragma unroll
  for (int to = 0; to < TS; ++to) out[to] = acc[to];
}
// proj with D k-tiles of operands in flight (D = TIN: all issued before the first MFMA); the
// same MFMA chain in the same k order as proj
template <int TIN, int TOUT, int D>
__device__ __forceinline__ void proj_ahead(const f32x4 (&in)[TIN], f32x4 (&acc)[TOUT], const float* __restrict__ A,
                                           int lane) {
  static_assert(D >= 1 && D <= TIN, "prefetch depth");
  f32x4 w[D][TOUT];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int to = 0; to < TOUT; ++to) w[d][to] = ld4(A + ((size_t)(to * TIN + d) * 64 + lane) * 4);
#pragma unroll
  for (int to = 0; to < TOUT; ++to) acc[to] = zero4();
#pragma unroll
  for (int ti = 0; ti < TIN; ++ti) {
    f32x4 cur[TOUT];
#pragma unroll
    for (int to = 0; to < TOUT; ++to) cur[to] = w[ti % D][to];
    if (ti + D < TIN) {
#pragma unroll
      for (int to = 0; to < TOUT; ++to) w[ti % D][to] = ld4(A + ((size_t)(to * TIN + ti + D) * 64 + lane) * 4);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int to = 0; to < TOUT; ++to) acc[to] = MSW_MFMA(cur[to][r], in[ti][r], acc[to]);
  }
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
// np_project with the output tiles of U, V and O split over the ranks (each stores its part);
// D > 0: D k-tiles of operands in flight (proj_ahead), D = 0: proj
template <int TIN, int TS, int D = 0>
__device__ __forceinline__ void proj_store_part(const f32x4 (&in)[TIN], const float* A, int r, float* dst, size_t n,
                                                int ntl, bool valid, int lane, int g) {
  f32x4 acc[TS];
  if constexpr (D > 0)
    proj_ahead<TIN, TS, (D < TIN ? D : TIN)>(in, acc, A + (size_t)r * TS * TIN * 256, lane);
  else
    proj<TIN, TS>(in, acc, A + (size_t)r * TS * TIN * 256, lane);
  if (valid) {
#pragma unroll
    for (int t = 0; t < TS; ++t) st4(dst + n * (16 * ntl) + 16 * (r * TS + t) + 4 * g, acc[t]);
  }
}
template <int NT, int H1T, int P, int D = 0>
__device__ __forceinline__ void np_project_coop(const f32x4 (&xs)[NT], const f32x4 (&xin)[NT], const NpDesc& d,
                                                const float* W, size_t n, bool valid, int r, int lane, int g) {
  constexpr int T2 = 2 * NT;
  f32x4 in[T2];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    in[t] = xs[t];
    in[NT + t] = xin[t];
  }
  if (d.a_u >= 0) proj_store_part<T2, H1T / P, D>(in, W + d.a_u, r, d.U, n, H1T, valid, lane, g);
  if (d.a_v >= 0) proj_store_part<T2, H1T / P, D>(in, W + d.a_v, r, d.V, n, H1T, valid, lane, g);
  if constexpr (P <= NT) {
    if (d.a_o >= 0) proj_store_part<NT, NT / P, D>(xin, W + d.a_o, r, d.O, n, NT, valid, lane, g);
  } else {  // more ranks than O tiles: ranks 0..NT-1 take one O tile each
    if (d.a_o >= 0 && r < NT) proj_store_part<NT, 1, D>(xin, W + d.a_o, r, d.O, n, NT, valid, lane, g);
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
  if (d.normalize) normalize_s<NT>(sv);  // gnn.py:424-426
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
  __shared__ __attribute__((aligned(16))) float pbuf[FUSE ? G : 1][kRowsPerWave][XS];  // FUSE != 0
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
  // FULL: the processors' common shape, see k_edge.h edge_full (with fused (un)pooling: the
  // processor's part -- the fused loads fill the same rows)
  auto body = [&](auto full) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full)::value;
    EdgeHopRows<NT> q;
    [[maybe_unused]] PoolIn<NT> pin;
    [[maybe_unused]] UnpoolIn<NT> uin;
    if constexpr (FUSE == 1)
      edge_pool_load<NT, LST>(q, pin, a, live ? tile : 0, j, g, r);
    else if constexpr (FUSE == 2)
      edge_unpool_load<NT, LST>(q, uin, a, live ? tile : 0, j, g, r);
    else
      edge_hop_load<NT, LST, FULL>(q, a, live ? tile : 0, j, g);  // dead groups compute tile 0, store nothing
    const bool split = a.reg.split < a.reg_nf;
    stage_glds<kWaves>(smem, a.c.W, a.reg, 0, a.reg.split);
    __syncthreads();
    c.W = smem;
    if (split) stage_glds<kWaves>(smem, a.c.W, a.reg, chunk_ceil(a.reg.split), a.reg_nf);
    if constexpr (FUSE != 0) {
      static_assert(P == 2, "fused pooling / unpooling: a source rank and a destination rank");
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
      if constexpr (!FULL) br[t] = ld4(c.W + b1 + off);
    }
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      if constexpr (FULL) {
        H[t] = (q.Us[t] + vr[t]) + q.Ps[t];
      } else {
        const f32x4 p = a.Pe ? q.Ps[t] : br[t];
        H[t] = (t < a.h1t) ? (q.Us[t] + vr[t]) + p : zero4();
      }
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
    if (a.normalize) normalize_s<NT>(sv);  // gnn.py:424-426
    if (live && r == 0 && a.s) store_row<NT>(a.s + L.p * F, sv, NT, g);
    put_message<NT, FULL ? 1 : -1>(my, q.os, od, sv, L.ev, a.grad, a.upwind, g);
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
    if constexpr (!FULL) {
      if (a.skip) {
#pragma unroll
        for (int t = 0; t < TS; ++t) rs[t] = rs[t] + pick<NT, TS>(q.sk, r, t);
      }
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
  };
  if (edge_full(a, NT))
    body(std::true_type{});
  else
    body(std::false_type{});
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
  // FULL: the processors' common shape, see k_edge.h edge_full (with fused pooling: the
  // processor's part -- the fused load fills the same rows)
  const bool full = edge_full(a, NT);
  EdgeHopRows<NT> q;
  [[maybe_unused]] PoolIn<NT> pin;
  [[maybe_unused]] const int side = r >= P / 2;  // fused pooling: 0 source side, 1 destination side
  if constexpr (FUSE == 1)
    edge_pool_load<NT, LST>(q, pin, a, tile, j, g, side);
  else if (full)
    edge_hop_load<NT, LST, true>(q, a, tile, j, g);
  else
    edge_hop_load<NT, LST>(q, a, tile, j, g);
  const Lanes& L = q.L;
  // the MLP region: staged in LDS, or (wdirect: two workgroups per CU) read from its blob copy
  if (a.reg.len > 0 && !a.wdirect) stage_glds<kWaves>(smem, c.W, a.reg, 0, a.reg.len);
  // the MLP operands through a pointer the compiler can prove to be LDS when staged (the
  // run-time LDS-or-blob choice made every weight read a FLAT load, which also waits on vmcnt)
  auto rest = [&](const float* Wm, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
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
      if constexpr (!FULL) br[t] = ld4(Wm + b1 + off);
    }
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      if constexpr (FULL) {
        H[t] = (q.Us[t] + vr[t]) + q.Ps[t];
      } else {
        const f32x4 p = a.Pe ? q.Ps[t] : br[t];
        H[t] = (t < a.h1t) ? (q.Us[t] + vr[t]) + p : zero4();
      }
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
    if (a.normalize) normalize_s<NT>(sv);  // gnn.py:424-426
    if (live && r == 0 && a.s) store_row<NT>(a.s + L.p * F, sv, NT, g);
    // every rank has read the slab's node rows before the first MLP exchange barrier: rank 0
    // may overwrite them with the messages (a.rest.n == 0 has no barrier: add one)
    if (a.rest.n == 0) __syncthreads();
    if (r == 0) put_message<NT, FULL ? 1 : -1>(my, q.os, od, sv, L.ev, a.grad, a.upwind, g);
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
    if (!FULL && a.skip) {
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
  };
  // (four ranks per tile only: the two-rank kernels' register count grew past two workgroups
  // per CU with it, 176 -> 256 VGPRs, and the finest unpooling lost its one-round grid)
  auto run = [&](auto fullc) __attribute__((always_inline)) {
    if constexpr (P == 4) {
      if (a.reg.len > 0 && !a.wdirect)
        rest((const float*)smem, fullc);
      else
        rest(a.reg.len > 0 ? c.W + a.reg.off : c.W, fullc);
    } else {
      rest(a.reg.len > 0 ? (a.wdirect ? c.W + a.reg.off : (const float*)smem) : c.W, fullc);
    }
  };
  if (full)
    run(std::true_type{});
  else
    run(std::false_type{});
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
