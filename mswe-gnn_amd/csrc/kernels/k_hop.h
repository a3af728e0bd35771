// gfx950 kernels: hops 2..K: edge tiles, row layout, feature split, cooperative last hop.
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

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
constexpr int kRowDc = 3;  // edges in flight per lane (F <= 32): 113 VGPRs, 4 waves per SIMD
template <int NT>
__global__ __launch_bounds__(64 * kRowHopWaves) void k_hop_rows(HopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT;
  constexpr int DC = NT >= 4 ? 2 : kRowDc;
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
    if (valid) store_row<NT, true>(a.out + n * F, res, NT, g);  // streaming (large meshes only)
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

template <int NT>
static const void* hop_coop_kernel(int prelu) {
  if constexpr (NT >= 2) return prelu ? (const void*)k_hop_coop<NT, 1, NT> : (const void*)k_hop_coop<NT, -1, NT>;
  return nullptr;
}
