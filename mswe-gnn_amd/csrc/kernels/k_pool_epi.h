// gfx950 kernels: pooling, row epilogue, plan-time row MLPs.
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

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
