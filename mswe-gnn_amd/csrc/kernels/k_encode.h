// gfx950 kernels: node encoders (+ the deferred decoder).
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

// ---------------------------------------------------------------------------- encoder
// Static / dynamic node encoders incl. the water-level feature (MSGNN.forward
// gnn.py:284-294, GNN.forward :112-123) + projection of processor 0 + the x_s part of
// every unpooling layer's V.  One workgroup = 64 rows of one scale.
// DEC: the rollout variant that decodes the previous step first (EncodeArgs::dec.on); the
// other variant keeps the encoders' register budget (four waves per SIMD) for forward mode
// and the large meshes whose last hops decode.
// STREAM (grid-stride launches without DEC, EncodeArgs::stream): the rows go out with
// streaming stores (k_base.h st4_stream).
template <int NT, int ACT, bool DEC, bool STREAM = false>
__global__ __launch_bounds__(kBlock) void k_encode(EncodeArgs a) {
  constexpr bool ST = STREAM && !DEC;
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
    if constexpr (kBcHoist<NT>) {  // the next step's BC values before the weight staging
      if (DEC && dstep >= 0) {
        pre.step = dstep;
        bc_prefetch<NT, true>(pre, a.dec, c);
      }
    }
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
      if constexpr (!kBcHoist<NT>) {
        pre.step = dstep;
        bc_prefetch<NT, true>(pre, a.dec, c);
      }
      float nd[kMaxDyn];
      decode_state<NT, ACT, true>(xu, a.dec, c, Wl, pre, n, valid, lane, g, nd);
#pragma unroll
      for (int r = 0; r < 4; ++r) dyn[r] = nd_column(nd, g, r, c.dyn);
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
      if (valid) store_row<NT, ST>(a.xs + (size_t)n * F, xs, NT, g);
    }
    MSW_MARK(c, 5);
    if (s == 0) {
      f32x4 xd[NT];
      const f32x4 in[1] = {f32x4{dyn[0], dyn[1], dyn[2], dyn[3]}};
      run_mlp<1, NT, NT, ACT>(in, xd, a.dynm, Wl, lane, g);
      if (valid && a.xd) store_row<NT, ST>(a.xd + (size_t)n * F, xd, NT, g);
      MSW_MARK(c, 6);
      np_project<NT, ST>(xs, xd, a.np0, Wl, n, valid, lane, g);
    }
    MSW_MARK(c, 8);
    if (a.vu_a[s] >= 0) side_proj<NT, NT, ST>(xs, a.vu_h1t, Wl + a.vu_a[s], a.Vu, n, valid, lane, g);
  }
  MSW_MARK(c, 9);
}

// ---------------------------------------------------------------------------- forward decode
// Forward mode with the deferred decoder (plan.hip sched_step): decode_rows -- the last hops'
// forward-mode epilogue, operation for operation -- on 16 stored last-layer rows per wave,
// after the whole schedule instead of inside four latency-bound last hops.  The decoder
// operands are read from the blob (a few KB, L2-resident): no staging barrier.
template <int NT, int ACT>
__global__ __launch_bounds__(kBlock) void k_decode_fwd(DecodeArgs a) {
  constexpr int F = 16 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int n = wave_row0() + j;
  if (wave_row0() >= a.Npad) return;  // whole wave past the rows
  const bool valid = n < a.Npad;
  const int nn = valid ? n : 0;
  EpiPre<NT> pre;
  f32x4 xu[NT];
  load_row<NT>(xu, a.in + (size_t)nn * F, g);
  const Common& c = a.c;
  pre.ext = valid ? c.perm[nn] : -1;
  pre.step = 0;
  pre.bc = -1;
  const float* xr = a.dec.X + (size_t)(pre.ext > 0 ? pre.ext : 0) * c.nnf + (c.nnf - c.dyn);
#pragma unroll
  for (int k = 0; k < kMaxDyn; ++k) pre.xd[k] = k < c.dyn ? xr[k] : 0.f;
  decode_rows<NT, ACT>(xu, a.dec, c, pre, nn, valid, lane, g);
}
