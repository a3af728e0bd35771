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
// enc_coop_mlp with the operands issued ahead (F = 64 reads them from the blob, i.e. from L2:
// one round trip per layer instead of one per k-tile pair + the bias): the first layer's
// operands are loaded by the caller (load(), early -- at kernel start), layer 1's are in flight
// during layer 0's MFMA chain and exchange, deeper layers load theirs at the layer.  PF: every
// layer's rank slice has TS = T / P output tiles (all F = 64 and F = 32 encoder MLPs at P =
// NT); otherwise it is enc_coop_mlp.  Same arithmetic.
template <int IN0, int T, int TL, int ACT, int P, int XW>
struct CoopMlp {
  static constexpr int TS = T / P;
  static constexpr bool XL = TL % P == 0;  // the last layer split over the ranks, else on every rank
  static constexpr bool PF = (XL ? TL / P : TL) == TS;
  LayerOps<IN0, TS> first;
  __device__ __forceinline__ void load(const MlpDev& m, const float* __restrict__ W, int r, int lane, int g) {
    if constexpr (PF) ops_load<IN0, TS>(first, m.l[0], W, (m.n == 1 && !XL) ? 0 : r * TS, lane, g);
  }
  // hook(): called once, after layer 0's MFMA chain (loads for what follows this MLP)
  template <class Hook>
  __device__ __forceinline__ void run(const f32x4 (&in)[IN0], f32x4 (&out)[TL], const MlpDev& m,
                                      const float* __restrict__ W, int lane, int g, int j, int r, float* buf,
                                      int& xc, Hook&& hook) const {
    if constexpr (!PF) {
      hook();
      enc_coop_mlp<IN0, T, TL, ACT, P, XW>(in, out, m, W, lane, g, j, r, buf, xc);
    } else {
      const int tl0 = XL ? r * TS : 0;
      auto finish = [&](const f32x4 (&o)[TS]) {
        if constexpr (XL) {
          coop_exchange<TL, P>(o, out, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
        } else {
#pragma unroll
          for (int t = 0; t < TL; ++t) out[t] = o[t];
        }
      };
      f32x4 o[TS];
      if (m.n == 1) {
        ops_layer<IN0, TS, ACT>(in, o, first, m.l[0]);
        hook();
        finish(o);
        return;
      }
      LayerOps<T, TS> nx;
      ops_load<T, TS>(nx, m.l[1], W, m.n == 2 ? tl0 : r * TS, lane, g);
      ops_layer<IN0, TS, ACT>(in, o, first, m.l[0]);
      hook();
      f32x4 h[T];
      coop_exchange<T, P>(o, h, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
      ops_layer<T, TS, ACT>(h, o, nx, m.l[1]);
      for (int li = 2; li < m.n; ++li) {
        coop_exchange<T, P>(o, h, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
        LayerOps<T, TS> cur;
        ops_load<T, TS>(cur, m.l[li], W, li + 1 == m.n ? tl0 : r * TS, lane, g);
        ops_layer<T, TS, ACT>(h, o, cur, m.l[li]);
      }
      finish(o);
    }
  }
};
// projections' operands: this many k-tiles in flight (0: proj)
constexpr int kEncProjAhead = 4;
// Workgroup: WV waves = WV / P row tiles (F = 32: eight waves, the four row tiles of k_encode's
// workgroup, so the weight region is staged as often as there; F = 64 reads the blob).
template <int NT> constexpr int enc_coop_waves() { return NT == 2 ? 8 : kWaves; }
// at most 128 registers: four waves per SIMD keep the zenodo4 F = 64 grid (3,488 waves) in one round
template <int NT, int ACT, bool DEC, int P, int WV = enc_coop_waves<NT>()>
__global__ __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_coop(EncodeArgs a) {
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
  // the decoder's pre-activation is split over the ranks like its MFMA layers: rank r loads and
  // activates input tiles [r DS, (r + 1) DS) only, the tiles are exchanged before layer 0
  constexpr int DS = NT / P;
  f32x4 xu[DS];
  if (DEC) {  // as k_encode: not behind the step counter
#pragma unroll
    for (int t = 0; t < DS; ++t) xu[t] = ld4(a.dec_in + (size_t)n * F + 16 * (r * DS + t) + 4 * g);
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
  // first-layer operands of the encoder MLPs, in flight from here (F = 64: from L2)
  // (rollout mode: issued inside the decoder, once its own first layer has run)
  CoopMlp<1, NT, NT, ACT, P, XW> stat_mlp, dyn_mlp;
  auto enc_loads = [&]() {
    stat_mlp.load(a.stat, Wl, r, lane, g);
    dyn_mlp.load(a.dynm, Wl, r, lane, g);  // unconditional (scale 0 only uses it): no branch
  };
  auto none = [&]() {};
  const bool decode = DEC && dstep >= 0;
  if (!decode) enc_loads();
  if (decode) {
#pragma clang fp contract(off)
    CoopMlp<NT, NT, 1, ACT, P, XW> dec_mlp;
    dec_mlp.load(a.dec.dec, Wl, r, lane, g);
    if constexpr (!kBcHoist<NT>) {
      pre.step = dstep;
      bc_prefetch<NT>(pre, a.dec, c);
    }
    float nd[kMaxDyn];
    {
      f32x4 x0[NT], o[1];
      act_tiles<-1, DS>(xu, a.dec.pre_act, a.dec.pre_slope);
      coop_exchange<NT, P>(xu, x0, buf + (xc++ & 1) * kRowsPerWave * XW, XW, r, j, g);
      dec_mlp.run(x0, o, a.dec.dec, Wl, lane, g, j, r, buf, xc, enc_loads);
      decode_state_tail<NT>(o, a.dec, c, Wl, pre, n, valid && r == 0, lane, g, nd);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) dyn[q] = nd_column(nd, g, q, c.dyn);
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
    stat_mlp.run(in, xs, a.stat, Wl, lane, g, j, r, buf, xc, none);
    if (valid && r == 0) store_row<NT>(a.xs + (size_t)n * F, xs, NT, g);
  }
  MSW_MARK(c, 5);
  if (s == 0) {
    f32x4 xd[NT];
    const f32x4 in[1] = {f32x4{dyn[0], dyn[1], dyn[2], dyn[3]}};
    dyn_mlp.run(in, xd, a.dynm, Wl, lane, g, j, r, buf, xc, none);
    if (valid && r == P - 1 && a.xd) store_row<NT>(a.xd + (size_t)n * F, xd, NT, g);
    MSW_MARK(c, 6);
    if (a.np0.h1t == T2)
      np_project_coop<NT, T2, P, kEncProjAhead>(xs, xd, a.np0, Wl, n, valid, r, lane, g);
    else
      np_project_coop<NT, NT, P, kEncProjAhead>(xs, xd, a.np0, Wl, n, valid, r, lane, g);
  }
  MSW_MARK(c, 8);
  if (a.vu_a[s] >= 0) {
    if (a.vu_h1t == T2)
      proj_store_part<NT, T2 / P, kEncProjAhead>(xs, Wl + a.vu_a[s], r, a.Vu, n, T2, valid, lane, g);
    else
      proj_store_part<NT, NT / P, kEncProjAhead>(xs, Wl + a.vu_a[s], r, a.Vu, n, NT, valid, lane, g);
  }
  MSW_MARK(c, 9);
}
