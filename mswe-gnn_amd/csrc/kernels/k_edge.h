// gfx950 kernels: message passing, fused edge MLP + hop 1, split edge MLP.
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

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
// GM = 1: gradient messages without upwind known at compile time (the flags then cost no
// per-element selects); GM = -1: the run-time flags
template <int NT, int GM = -1>
__device__ __forceinline__ void put_message(float* slab_row, const f32x4 (&os)[NT], const f32x4 (&od)[NT],
                                            const f32x4 (&sv)[NT], bool ev, int grad_rt, int upwind_rt, int g) {
#pragma clang fp contract(off)
  const int grad = GM == 1 ? 1 : grad_rt, upwind = GM == 1 ? 0 : upwind_rt;
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
// FULL: the processors' common shape, known at compile time -- a 2F-wide first layer with an
// edge term (h1t = 2NT, Pe), own rows read, no skip, gradient messages without upwind
// (edge_full) -- so the run-time flags below cost no per-element selects (a wave-uniform flag
// in a select is still one VALU op per element).  Same loads and arithmetic where both apply.
#ifndef MSW_EDGE_FULL
#define MSW_EDGE_FULL 1  // 0: no FULL specialisation (A/B build variant)
#endif
__device__ __forceinline__ bool edge_full(const EdgeHopArgs& a, int nt) {
  return MSW_EDGE_FULL && a.h1t == 2 * nt && a.Pe && !a.own_zero && !a.skip && a.grad && !a.upwind;
}
template <int NT, int LST, bool FULL = false>
__device__ __forceinline__ void edge_hop_gather(EdgeHopRows<NT>& r, const EdgeHopArgs& a, const LaneRec& rec,
                                                int tile, int j, int g) {
  constexpr int F = 16 * NT, T2 = 2 * NT;
  r.L = lanes_of(rec, tile, j, a.n0);
  const Lanes& L = r.L;
  const int hs = FULL ? 16 * T2 : 16 * a.h1t;
  const float* z = a.c.zrow;
  const float* Ub = a.U + L.sr * hs;
  const float* Vb = a.V + L.n * hs;
  const float* Pb = FULL ? a.Pe + L.p * hs : a.Pe ? a.Pe + L.p * hs : z;
#pragma unroll
  for (int t = 0; t < T2; ++t) {  // unconditional loads, tiles past h1t read zeros
    const int off = 16 * t + 4 * g;
    const bool on = FULL || t < a.h1t;
    r.Us[t] = ld4((on ? Ub : z) + off);
    r.Vn[t] = ld4((on ? Vb : z) + off);
    r.Ps[t] = ld4((on ? Pb : z) + off);
  }
  load_row<NT>(r.os, a.in + L.sr * F, g);
  load_row<NT>(r.inn, !FULL && a.own_zero ? z : a.in + L.n * F, g);
  if constexpr (!FULL) load_row<NT>(r.sk, a.skip ? a.skip + L.n * F : z, g);
  if (LST && a.last) epi_prefetch<NT>(r.pre, a.epi, a.c, a.xs, L.n, g);
}
template <int NT, int LST, bool FULL = false>
__device__ __forceinline__ void edge_hop_load(EdgeHopRows<NT>& r, const EdgeHopArgs& a, int tile, int j, int g) {
  edge_hop_gather<NT, LST, FULL>(r, a, load_rec(a.recs, tile, j), tile, j, g);
}
// Wm: the MLP operands (b1, layers 2..L) -- the staged region; c.W: everything else (the
// same region for F <= 32, the blob for F = 64, whose epilogue operands do not fit in LDS).
template <int NT, int ACT, int XS, bool FREG = true, bool FULL = false>
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
    if constexpr (!FULL) br[t] = ld4(Wm + b1 + off);
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    if constexpr (FULL) {
      H[t] = (r.Us[t] + vr[t]) + r.Ps[t];
    } else {
      const f32x4 p = a.Pe ? r.Ps[t] : br[t];
      H[t] = (t < a.h1t) ? (r.Us[t] + vr[t]) + p : zero4();
    }
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
  if (a.normalize) normalize_s<NT>(sv);  // gnn.py:424-426
  if (a.s) store_row<NT>(a.s + L.p * F, sv, NT, g);  // padding slots too: never read
  put_message<NT, FULL ? 1 : -1>(my, r.os, od, sv, L.ev, a.grad, a.upwind, g);  // the slab row is free again
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
  if constexpr (!FULL) {
    if (a.skip) {
#pragma unroll
      for (int t = 0; t < NT; ++t) res[t] = res[t] + r.sk[t];
    }
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
    // one tile per wave; FULL: see edge_full
    auto body = [&](auto full) __attribute__((always_inline)) {
      constexpr bool FULL = decltype(full)::value;
      const bool live = tile < a.ntiles;
      EdgeHopRows<NT> r;
      edge_hop_load<NT, LST, FULL>(r, a, live ? tile : 0, j, g);  // idle waves stay in bounds
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
      // F = 64: the MLP operands through a pointer the compiler can prove to be LDS (the run-time
      // LDS-or-blob choice made every weight read a FLAT load, which also waits on vmcnt)
      if (!kStaged<NT> && a.reg.len > 0) {
        if (live) edge_hop_core<NT, ACT, XS, true, FULL>(r, a, c, (const float*)smem, wf, &slab[w][0][0], j, lane, g, res);
      } else if (live) {
        edge_hop_core<NT, ACT, XS, true, FULL>(r, a, c, Wm, wf, &slab[w][0][0], j, lane, g, res);
      }
      if (split) __syncthreads();  // every wave: the epilogue operands have landed
      if (live) edge_hop_finish<NT, ACT, LST>(res, r, a, c, lane, g);
    };
    if (edge_full(a, NT))
      body(std::true_type{});
    else
      body(std::false_type{});
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
    auto walk = [&](const float* Wl, auto full) __attribute__((always_inline)) {
      constexpr bool FULL = decltype(full)::value;
      for (; tile < a.ntiles; tile += stride) {
        const int ln = opaque_lane(), gg = ln >> 4, jj = ln & 15;
        EdgeHopRows<NT> q;
        edge_hop_load<NT, LST, FULL>(q, a, tile, jj, gg);
        f32x4 res[NT];
        edge_hop_core<NT, ACT, XS, !kStaged<NT>, FULL>(q, a, c, Wl, wf, &slab[w][0][0], jj, ln, gg, res);
        edge_hop_finish<NT, ACT, LST>(res, q, a, c, ln, gg);
      }
    };
    // the processors' first hops (config 5's finest launches) take the FULL loop
    const bool full = edge_full(a, NT);
    if (!kStaged<NT> && a.reg.len > 0) {  // F = 64: provably LDS (see above)
      if (full)
        walk((const float*)smem, std::true_type{});
      else
        walk((const float*)smem, std::false_type{});
    } else if (full) {
      walk(Wm, std::true_type{});
    } else {
      walk(Wm, std::false_type{});
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
template <int NT>
struct MlpFetch {
  f32x4 u[2 * NT], v[2 * NT], p[2 * NT];
  int4 e;
};
// FULL shape (2F-wide first layer with an edge term): one chunk's U / V / Pe rows, no selects;
// ok = false reads the zero row instead (a launch of another shape)
template <int NT>
__device__ __forceinline__ void mlp_fetch_full(MlpFetch<NT>& f, const EdgeHopArgs& a, int ch, bool ok, int j, int g) {
  constexpr int T2 = 2 * NT, hs = 16 * T2;
  f.e = reinterpret_cast<const int4*>(a.chunks)[(size_t)ch * kRowsPerWave + j];
  const bool ev = ok && f.e.z >= 0;
  const float* z = a.c.zrow;
  const float* Ub = ok ? a.U + (size_t)(ev ? f.e.x : a.n0) * hs : z;
  const float* Vb = ok ? a.V + (size_t)(ev ? f.e.y : a.n0) * hs : z;
  const float* Pb = ev ? a.Pe + (size_t)f.e.z * hs : z;
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int off = 16 * t + 4 * g;
    f.u[t] = ld4(Ub + off);
    f.v[t] = ld4(Vb + off);
    f.p[t] = ld4(Pb + off);
  }
}
template <int NT, int ACT>
__global__ __launch_bounds__(64 * kMlpWaves) __attribute__((amdgpu_waves_per_eu(2)))
void k_edge_mlp(EdgeHopArgs a) {
#pragma clang fp contract(off)
  constexpr int F = 16 * NT, T2 = 2 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = wave_id();
  const int stride = gridDim.x * kMlpWaves;
  const int ch0 = blockIdx.x * kMlpWaves + w;
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  // FULL: a 2F-wide first layer with an edge term (k_edge_hop's edge_full): no per-element
  // selects on the run-time shape flags, and the first chunk's rows are gathered while the
  // weight staging is in flight (issued after it: the in-order memory counter then waits for
  // both at once; the first layer's sums H0 are all that stays live across the barrier)
  const bool full = MSW_EDGE_FULL && a.h1t == T2 && a.Pe;
  f32x4 H0[T2];
  int4 e0;
  // the MLP operands through a pointer the compiler can prove to be LDS (a run-time choice
  // between LDS and the blob made every weight read a FLAT load, which also waits on vmcnt)
  // one chunk: first layer's activation, layers 2..L, normalisation, s stored
  auto chunk = [&](f32x4 (&H)[T2], const int4 e, const float* Wm, int ln, int g) __attribute__((always_inline)) {
    const bool ev = e.z >= 0;
    act_tiles<ACT, T2>(H, a.act1, a.slope1);
    f32x4 sv[NT];
    if (a.rest.n > 0) {
      run_mlp<T2, T2, NT, ACT>(H, sv, a.rest, Wm, ln, g);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) sv[t] = H[t];
    }
    if (a.normalize) normalize_s<NT>(sv);  // gnn.py:424-426
    if (ev) store_row<NT>(a.s + (size_t)e.z * F, sv, NT, g);
  };
  auto run = [&](const float* Wm, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    if constexpr (FULL) {
      if (ch0 < a.nchunks) {  // the first chunk, gathered during the staging
        const int ln = opaque_lane(), g = ln >> 4;
        chunk(H0, e0, Wm, ln, g);
      }
      for (int ch = ch0 + stride; ch < a.nchunks; ch += stride) {
        const int ln = opaque_lane(), g = ln >> 4, j = ln & 15;
        MlpFetch<NT> f;
        mlp_fetch_full<NT>(f, a, ch, true, j, g);
        f32x4 H[T2];
#pragma unroll
        for (int t = 0; t < T2; ++t) H[t] = (f.u[t] + f.v[t]) + f.p[t];
        chunk(H, f.e, Wm, ln, g);
      }
    } else {
      const int hs = 16 * a.h1t;
      const float* z = a.c.zrow;
      const int b1 = a.b1_off >= 0 ? a.b1_off : 0;
      for (int ch = ch0; ch < a.nchunks; ch += stride) {
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
        chunk(H, e, Wm, ln, g);
      }
    }
  };
  if (a.reg.len > 0) stage_glds<kMlpWaves>(smem, a.c.W, a.reg, 0, a.reg.len);
  {
    const int lane = threadIdx.x & 63;
    MlpFetch<NT> f0;
    mlp_fetch_full<NT>(f0, a, ch0 < a.nchunks ? ch0 : 0, full && ch0 < a.nchunks, lane & 15, lane >> 4);
    e0 = f0.e;
#pragma unroll
    for (int t = 0; t < T2; ++t) H0[t] = (f0.u[t] + f0.v[t]) + f0.p[t];
  }
  if (a.reg.len > 0) __syncthreads();
  // stagger: the two waves of a SIMD (w, w + 4) otherwise run the same phase at the same time, so
  // one's VALU work never overlaps the other's MFMA chain
  if (w >= 4)
    for (int k = 0; k < a.stagger; ++k) __builtin_amdgcn_s_sleep(32);
  if (a.reg.len > 0) {
    if (full)
      run(smem, std::true_type{});
    else
      run(smem, std::false_type{});
  } else if (full) {
    run(a.c.W, std::true_type{});
  } else {
    run(a.c.W, std::false_type{});
  }
}
