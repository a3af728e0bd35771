// gfx950 kernels: cooperative encoder.
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

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
  if constexpr (kBcHoist<NT>) {  // see k_base.h kBcHoist
    if (DEC && dstep >= 0) {
      pre.step = dstep;
      bc_prefetch<NT>(pre, a.dec, c);
    }
  }
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
    if constexpr (!kBcHoist<NT>) {
      pre.step = dstep;
      bc_prefetch<NT>(pre, a.dec, c);
    }
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
