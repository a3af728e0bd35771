// gfx950 kernels: the grid-stride fused edge MLP + hop 1 with the NEXT tile's gathers in flight
// as LDS-DMA during the current tile's MLP (large meshes; config 5's finest scale).
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

// Why: on the ~1M-node mesh the grid-stride k_edge_hop takes about the SUM of its MFMA floor
// and its HBM floor: each wave gathers a tile, then multiplies, and its four
// co-resident waves do not cover each other.  Holding the next tile's rows in registers needs
// ~70 VGPRs more (two waves per SIMD, measured slower).  Here the rows land in the wave's own
// LDS region instead (global_load_lds, per-lane source address, lane-linear destination), so
// the prefetch costs no VGPRs: as soon as tile i has read its rows (at its start), all of tile
// i+1's are issued, so they have a whole tile's MLP and hop to land; the messages go from edge
// lane to node lane by ds_bpermute, so the region holds nothing else.
//
// Per wave, lane-linear 1-KB pieces (lane l = 16 g + j at byte 16 l of a piece):
//   U  [2NT pieces]  U[src_j]   features 16t + 4g..   (edge lane j)
//   V  [2NT]         V[dst_j]                          (node lane j; edge lanes read lane 16g + dl)
//   P  [2NT]         Pe[slot_j]                        (edge lane j)
//   OS [NT]          out0[src_j]
//   IN [NT]          out0[dst_j]   -- the node lane's own row; od of edge lanes (lane 16g + dl)
//   REC [2][64 dwords]  the lane records of the current / next tile (global_load_lds_dword)
// The arithmetic is edge_hop_core's, operation for operation: bit-identical to k_edge_hop.
//
// Counting: every VMEM operation of the loop is an LDS-DMA or a store (the filter is loaded
// before the workgroup barrier, which drains the counter), so the compiler inserts no vmcnt
// wait of its own there; the waits below are counted by hand (loads, stores and LDS-DMA retire
// in issue order on the one vmcnt counter), each assuming the FEWEST operations that can be
// younger -- a skipped store then only makes a wait stricter, never too weak.
// Workgroup: eight waves (two per SIMD, one workgroup per CU: LDS-bound; MSW_EH_DMA=1) or four
// (one per SIMD, the MFMA chains of one wave per SIMD under the DMA; MSW_EH_DMA=2)
constexpr int kDmaWaves = 8;
template <int NT>
struct DmaLayout {  // floats, per wave
  static constexpr int T2 = 2 * NT;
  static constexpr int U = 0, V = U + T2 * 256, P = V + T2 * 256;
  static constexpr int OS = P + T2 * 256, IN = OS + NT * 256, REC = IN + NT * 256;
  static constexpr int WAVE = REC + 2 * 64;
};
template <int NT>
constexpr size_t dma_lds_bytes(int reg_floats, int waves = kDmaWaves) {
  return eh_lds_bytes(reg_floats) + (size_t)waves * DmaLayout<NT>::WAVE * sizeof(float);
}

__device__ __forceinline__ void glds16(const float* src, float* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const int* src, float* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// issue: one tile's U / V / Pe rows (3 x 2NT LDS-DMA)
template <int NT>
__device__ __forceinline__ void dma_uvp(const EdgeHopArgs& a, const Lanes& L, float* wl, int g) {
  using D = DmaLayout<NT>;
  constexpr int T2 = 2 * NT, hs = 16 * T2;
  const float* Ub = a.U + L.sr * hs + 4 * g;
  const float* Vb = a.V + L.n * hs + 4 * g;
  const float* Pb = a.Pe + L.p * hs + 4 * g;
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    glds16(Ub + 16 * t, wl + D::U + 256 * t);
    glds16(Vb + 16 * t, wl + D::V + 256 * t);
    glds16(Pb + 16 * t, wl + D::P + 256 * t);
  }
}
// issue: one tile's out0 rows at the sources and destinations (2 x NT LDS-DMA)
template <int NT>
__device__ __forceinline__ void dma_oi(const EdgeHopArgs& a, const Lanes& L, float* wl, int g) {
  using D = DmaLayout<NT>;
  constexpr int F = 16 * NT;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    glds16(a.in + L.sr * F + 16 * t + 4 * g, wl + D::OS + 256 * t);
    glds16(a.in + L.n * F + 16 * t + 4 * g, wl + D::IN + 256 * t);
  }
}
// issue: one tile's 16 lane records (1 LDS-DMA of 64 dwords)
template <int NT>
__device__ __forceinline__ void dma_rec(const EdgeHopArgs& a, int tile, float* wl, int slot, int lane) {
  glds4(reinterpret_cast<const int*>(a.recs) + (size_t)tile * 64 + lane, wl + DmaLayout<NT>::REC + 64 * slot);
}
// The record read is hidden from the compiler (inline asm, its own lgkmcnt wait): a plain
// ds_read of it made hipcc put an s_waitcnt vmcnt(0) before it -- draining the out-row DMA the
// loop keeps in flight there (tests/test_host_cpu.py checks the kernel's vmcnt waits).
template <int NT>
__device__ __forceinline__ LaneRec rec_of(const float* wl, int slot, int j) {
  const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(wl + DmaLayout<NT>::REC + 64 * slot + 4 * j);
  int4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return LaneRec{v.x, v.y, v.z, v.w};
}

// The node phase's message sums without LDS: node lane j (lane group g) adds the messages of
// its edge slots q0..q1-1 in edge order, each fetched from lane 16 g + q with ds_bpermute (no
// LDS memory: the wave's region holds the next tile's rows by then).  Same sums in the same
// order as gather_messages.
template <int NT>
__device__ __forceinline__ void gather_bpermute(f32x4 (&agg)[NT], const f32x4 (&m)[NT], int q0, int q1, int g, int j) {
#pragma clang fp contract(off)
#pragma unroll
  for (int t = 0; t < NT; ++t) agg[t] = zero4();
  const int deg = q1 - q0;
  int dmax = deg;  // wave maximum of the in-degree (uniform loop bound)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) dmax = max(dmax, __shfl_xor(dmax, o));
  for (int d = 0; d < dmax; ++d) {
    const bool on = d < deg;
    const int src = (16 * g + (on ? q0 + d : j)) << 2;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(m[t][r])));
      if (on) agg[t] = agg[t] + v;
    }
  }
}

template <int NT, int ACT, int WV = kDmaWaves>
__global__ __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(WV / 4)))
void k_edge_hop_dma(EdgeHopArgs a) {
#pragma clang fp contract(off)
  using D = DmaLayout<NT>;
  constexpr int F = 16 * NT, T2 = 2 * NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];  // the ONLY LDS object (see above)
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, w = wave_id();
  const int stride = gridDim.x * WV;
  const int last_tile = a.ntiles - 1;
  int tile = blockIdx.x * WV + w;
  float* wl = smem + a.dma_off + w * D::WAVE;
  if (a.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *a.step_inc += 1;
  f32x4 wf[NT][NT];
  load_filter<NT>(wf, a.c.W, a.filt_a, lane);  // blob offset; drained by the barrier below
  stage_glds<WV>(smem, a.c.W, a.reg, 0, a.reg_nf);  // without the trailing filter copy
  const bool live = tile < a.ntiles;
  if (live) dma_rec<NT>(a, tile, wl, 0, lane);
  __syncthreads();  // vmcnt(0): weights, the filter, the first record
  if (!live) return;
  Lanes L = lanes_of(rec_of<NT>(wl, 0, j), tile, j, a.n0);
  dma_uvp<NT>(a, L, wl, g);
  dma_oi<NT>(a, L, wl, g);
  dma_rec<NT>(a, min(tile + stride, last_tile), wl, 1, lane);
  int slot = 0;
  bool first = true;
  const float* Wm = smem;
  for (;;) {
    // this tile's rows and the next tile's record have landed: they were issued last (the
    // prologue) or before the previous tile's MLP; younger: the previous tile's s stores (NT)
    // [and its out stores]
    if (first) vm_wait<0>(); else vm_wait<NT>();
    const int ln = opaque_lane();
    f32x4 H[T2], os[NT], od[NT], res[NT];
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      const f32x4 u = ld4(wl + D::U + 256 * t + 4 * lane);
      const f32x4 v = ld4(wl + D::V + 256 * t + 4 * (16 * g + L.dl));
      const f32x4 p = ld4(wl + D::P + 256 * t + 4 * lane);
      H[t] = (u + v) + p;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      os[t] = ld4(wl + D::OS + 256 * t + 4 * lane);
      od[t] = ld4(wl + D::IN + 256 * t + 4 * (16 * g + L.dl));
      res[t] = ld4(wl + D::IN + 256 * t + 4 * lane);
    }
    const int nxt = min(tile + stride, last_tile);
    const Lanes Ln = lanes_of(rec_of<NT>(wl, slot ^ 1, j), nxt, j, a.n0);  // (waits lgkmcnt(0))
    lgkm_wait();  // every read of the region done: it is free for the next tile
    dma_uvp<NT>(a, Ln, wl, g);                                          // 3 x 2NT
    dma_oi<NT>(a, Ln, wl, g);                                           // 2 x NT
    dma_rec<NT>(a, min(tile + 2 * stride, last_tile), wl, slot, lane);  // 1 (this tile's slot: read)
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
    store_row<NT>(a.s + L.p * F, sv, NT, g);  // NT stores (padding slots too: never read)
    f32x4 msg[NT];
    {  // put_message (k_edge.h), kept in registers
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
        if (a.grad) {
          gv = od[t] - os[t];  // out[col] - out[row]
          if (a.upwind) {
            gv.x = gv.x < 0.f ? 0.f : gv.x; gv.y = gv.y < 0.f ? 0.f : gv.y;
            gv.z = gv.z < 0.f ? 0.f : gv.z; gv.w = gv.w < 0.f ? 0.f : gv.w;
          }
        } else {
          gv = os[t];
        }
        const f32x4 m = gv * sv[t];
        msg[t] = (L.ev && act) ? m : zero4();
      }
    }
    f32x4 agg[NT];
    gather_bpermute<NT>(agg, msg, L.q0, L.q1, g, j);
    apply_filter_regs<NT>(res, agg, a.filt_a, wf);
    if (L.nv) store_row<NT>(a.out + L.n * F, res, NT, g);
    if (tile + stride > last_tile) break;
    tile += stride;
    L = Ln;
    slot ^= 1;
    first = false;
  }
  vm_wait<0>();  // the clamped prefetches of the last iteration
}
