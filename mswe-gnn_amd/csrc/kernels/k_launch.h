// gfx950 kernels: launchers and per-F instantiation.
// Part of kernels_impl.h (included inside namespace msw, in this order); see its header
// comment for the register layout and conventions.
#pragma once

// ---------------------------------------------------------------------------- launchers
static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

template <int NT>
constexpr size_t lds_bytes(int floats) {
  return kStaged<NT> ? (size_t)((floats + kChunk - 1) / kChunk * kChunk) * sizeof(float) : 0;
}

// Allow the dynamic weight regions past the 64 KB default (gfx950: 160 KB per CU).
template <int NT>
hipError_t prepare_kernels() {
  // the largest static slab (edge-MLP rows) of a workgroup of `wv` waves
  auto mx = [](int wv) { return 160 * 1024 - wv * kRowsPerWave * (16 * 2 * NT + 16 * NT + 4) * (int)sizeof(float); };
  constexpr int WL = waves_of<NT, true>();
  const std::pair<const void*, int> fns[] = {
      {(const void*)k_encode<NT, 1, false>, kWaves}, {(const void*)k_encode<NT, -1, false>, kWaves},
      {(const void*)k_encode<NT, 1, true>, kWaves}, {(const void*)k_encode<NT, -1, true>, kWaves},
      {(const void*)k_encode<NT, 1, false, true>, kWaves}, {(const void*)k_encode<NT, -1, false, true>, kWaves},
      {(const void*)k_edge_hop<NT, 1, false, 0>, kWaves}, {(const void*)k_edge_hop<NT, -1, false, 0>, kWaves},
      {(const void*)k_edge_hop<NT, 1, false, 1>, kWaves}, {(const void*)k_edge_hop<NT, -1, false, 1>, kWaves},
      {(const void*)k_edge_hop<NT, 1, true, 0>, edge_waves<NT, true, 0>()},
      {(const void*)k_edge_hop<NT, -1, true, 0>, edge_waves<NT, true, 0>()},
      {(const void*)k_edge_hop<NT, 1, true, 1>, edge_waves<NT, true, 1>()},
      {(const void*)k_edge_hop<NT, -1, true, 1>, edge_waves<NT, true, 1>()},
      {(const void*)k_hop<NT, 1, true, false>, kWaves}, {(const void*)k_hop<NT, -1, true, false>, kWaves},
      {(const void*)k_hop<NT, 1, true, true>, hop_waves<NT, true>()},
      {(const void*)k_hop<NT, -1, true, true>, hop_waves<NT, true>()},
      {(const void*)k_pool<NT, false>, kWaves}, {(const void*)k_pool<NT, true>, WL},
      {(const void*)k_pool_edge<NT>, kWaves}, {(const void*)k_pool_edge<NT, NT >= 2 ? NT : 1>, kWaves},
      {(const void*)k_epi<NT, 1, false>, kWaves}, {(const void*)k_epi<NT, -1, false>, kWaves},
      {(const void*)k_epi<NT, 1, true>, WL}, {(const void*)k_epi<NT, -1, true>, WL}};
  for (const auto& f : fns) {
    hipError_t e = hipFuncSetAttribute(f.first, hipFuncAttributeMaxDynamicSharedMemorySize, mx(f.second));
    if (e != hipSuccess) return e;
  }
  for (const void* f : {(const void*)k_edge_mlp<NT, 1>, (const void*)k_edge_mlp<NT, -1>}) {  // no slab
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  if constexpr (NT >= 2) {  // wide pooling (one tile per workgroup)
    hipError_t e = hipFuncSetAttribute((const void*)k_pool_edge<NT, 2 * NT, 2 * NT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mx(2 * NT));
    if (e != hipSuccess) return e;
  }
  if constexpr (NT >= 2) {  // cooperative encoders
    for (const void* f : {(const void*)k_encode_coop<NT, 1, false, NT>, (const void*)k_encode_coop<NT, -1, false, NT>,
                          (const void*)k_encode_coop<NT, 1, true, NT>, (const void*)k_encode_coop<NT, -1, true, NT>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx(enc_coop_waves<NT>()));
      if (e != hipSuccess) return e;
    }
  }
  if constexpr (NT == 4) {  // F = 64 cooperative encoder on two waves per row tile
    for (const void* f : {(const void*)k_encode_coop<NT, 1, false, 2>, (const void*)k_encode_coop<NT, -1, false, 2>,
                          (const void*)k_encode_coop<NT, 1, true, 2>, (const void*)k_encode_coop<NT, -1, true, 2>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx(enc_coop_waves<NT>()));
      if (e != hipSuccess) return e;
    }
  }
  if constexpr (NT >= 2) {  // cooperative last hops (F = 32, 64)
    for (int prelu = 0; prelu < 2; ++prelu) {
      hipError_t e = hipFuncSetAttribute(hop_coop_kernel<NT>(prelu), hipFuncAttributeMaxDynamicSharedMemorySize, mx(kWaves));
      if (e != hipSuccess) return e;
    }
  }
  if constexpr (NT == 4) {  // F = 64 cooperative edge hops: a slab + exchange buffers per tile
    for (int pw = 2; pw <= 4; pw += 2) {
      for (int prelu = 0; prelu < 2; ++prelu)
        for (int last = 0; last < 2; ++last)
          for (int pool = 0; pool < 2; ++pool) {
            hipError_t e = hipFuncSetAttribute(edge_coop_kernel<NT>(prelu, last, pw, pool),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               edge_coop_lds_cap<NT>(pw, pool));
            if (e != hipSuccess) return e;
          }
    }
  }
  if constexpr (NT == 2) {  // cooperative edge hops: 160 KB minus slabs and exchange buffers
    for (int prelu = 0; prelu < 2; ++prelu)
      for (int last = 0; last < 2; ++last)
        for (int pool = 0; pool < 3; ++pool) {
          hipError_t e = hipFuncSetAttribute(edge_coop_kernel<NT>(prelu, last, 0, pool),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             edge_coop_lds_cap<NT>(2, pool));
          if (e != hipSuccess) return e;
        }
  }
  return hipSuccess;
}

template <int NT>
hipError_t launch_encode(const EncodeArgs& a, hipStream_t st) {
  if (a.Npad <= 0) return hipSuccess;
  if constexpr (NT >= 2) {
    if (a.coop == NT) {  // P = NT waves per row tile (F = 32: 2, F = 64: 4)
      constexpr int P = NT, WV = enc_coop_waves<NT>();
      const dim3 grid(a.Npad / ((WV / P) * kRowsPerWave)), block(64 * WV);
      const size_t sh = lds_bytes<NT>(a.lds_floats);
      if (a.dec.on) {
        if (a.c.prelu)
          hipLaunchKernelGGL((k_encode_coop<NT, 1, true, P>), grid, block, sh, st, a);
        else
          hipLaunchKernelGGL((k_encode_coop<NT, -1, true, P>), grid, block, sh, st, a);
      } else if (a.c.prelu) {
        hipLaunchKernelGGL((k_encode_coop<NT, 1, false, P>), grid, block, sh, st, a);
      } else {
        hipLaunchKernelGGL((k_encode_coop<NT, -1, false, P>), grid, block, sh, st, a);
      }
      return hipGetLastError();
    }
  }
  const int n = a.Npad / kRowsPerBlock;
  const dim3 grid(a.max_blocks > 0 && n > a.max_blocks ? a.max_blocks : n), block(kBlock);
  const size_t sh = lds_bytes<NT>(a.lds_floats);
  if (a.stream && !a.dec.on) {
    if (a.c.prelu)
      hipLaunchKernelGGL((k_encode<NT, 1, false, true>), grid, block, sh, st, a);
    else
      hipLaunchKernelGGL((k_encode<NT, -1, false, true>), grid, block, sh, st, a);
    return hipGetLastError();
  }
  if (a.dec.on) {
    if (a.c.prelu)
      hipLaunchKernelGGL((k_encode<NT, 1, true>), grid, block, sh, st, a);
    else
      hipLaunchKernelGGL((k_encode<NT, -1, true>), grid, block, sh, st, a);
  } else if (a.c.prelu) {
    hipLaunchKernelGGL((k_encode<NT, 1, false>), grid, block, sh, st, a);
  } else {
    hipLaunchKernelGGL((k_encode<NT, -1, false>), grid, block, sh, st, a);
  }
  return hipGetLastError();
}

// XCD packing of a one-round grid of g workgroups (b: the launch's argument copy): the
// fewest XCDs (1, 2, 4 <= c.xcd_max) that hold one workgroup per CU, else all eight
template <class A>
static inline dim3 xcd_grid(A& b, long g) {
  b.c.xcd = 0;
  for (int k = 1; k <= b.c.xcd_max && k < kXcds; k *= 2)
    if (g <= (long)kCusPerXcd * k) {
      b.c.xcd = k;
      return dim3((unsigned)(cdiv(g, k) * kXcds));
    }
  return dim3((unsigned)g);
}

// one tile per wave while that grid is resident at once; grid-stride loop beyond that
template <class A>
static inline bool tile_loop(const A& a) {
  return a.fit_blocks > 0 && a.max_blocks > 0 && cdiv(a.ntiles, kWaves) > a.fit_blocks;
}
template <class A>
static inline int tile_grid(const A& a) {
  return tile_loop(a) ? a.max_blocks : cdiv(a.ntiles, kWaves);
}

template <int NT>
static const void* edge_hop_kernel(int prelu, bool loop, int last) {
  if (loop) {
    if (last) return prelu ? (const void*)k_edge_hop<NT, 1, true, 1> : (const void*)k_edge_hop<NT, -1, true, 1>;
    return prelu ? (const void*)k_edge_hop<NT, 1, true, 0> : (const void*)k_edge_hop<NT, -1, true, 0>;
  }
  if (last) return prelu ? (const void*)k_edge_hop<NT, 1, false, 1> : (const void*)k_edge_hop<NT, -1, false, 1>;
  return prelu ? (const void*)k_edge_hop<NT, 1, false, 0> : (const void*)k_edge_hop<NT, -1, false, 0>;
}
template <int NT>
hipError_t launch_edge_mlp(const EdgeHopArgs& a, hipStream_t st) {
  if (a.nchunks <= 0) return hipSuccess;
  const int n = cdiv(a.nchunks, kMlpWaves);
  const dim3 grid(a.max_blocks > 0 && n > a.max_blocks ? a.max_blocks : n), block(64 * kMlpWaves);
  if (a.c.prelu)
    hipLaunchKernelGGL((k_edge_mlp<NT, 1>), grid, block, eh_lds_bytes(a.reg.len), st, a);
  else
    hipLaunchKernelGGL((k_edge_mlp<NT, -1>), grid, block, eh_lds_bytes(a.reg.len), st, a);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_edge_hop(const EdgeHopArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  if (a.coop == 2 || a.coop == 4) {  // waves per tile; 4: F = 64, one tile per workgroup
    const int fuse = a.pool.slots ? 1 : a.pool.parent ? 2 : 0;
    const void* f = edge_coop_kernel<NT>(a.c.prelu, a.last, a.coop, fuse);
    if (!f || (fuse && NT == 2 && a.coop != 2)) return hipErrorInvalidValue;
    EdgeHopArgs b = a;
    const dim3 grid = xcd_grid(b, a.coop == 4 ? a.ntiles : cdiv((long)a.ntiles * a.coop, kWaves));
    void* args[] = {&b};
    return hipLaunchKernel(f, grid, dim3(kBlock), args, a.wdirect ? 0 : eh_lds_bytes(a.reg_nf), st);
  }
  if (a.pool.slots || a.pool.parent) return hipErrorInvalidValue;  // fused into k_edge_coop only
  const bool loop = tile_loop(a);
  EdgeHopArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? (a.last ? edge_waves<NT, true, 1>() : edge_waves<NT, true, 0>()) : kWaves));
  const size_t sh = eh_lds_bytes(loop ? a.reg.len : a.reg_nf);
  void* args[] = {&b};
  return hipLaunchKernel(edge_hop_kernel<NT>(a.c.prelu, loop, a.last), grid, block, args, sh, st);
}
template <int NT>
hipError_t launch_hop_kernel(const HopArgs& a, bool loop, dim3 grid, dim3 block, hipStream_t st);
template <int NT>
hipError_t launch_hop(const HopArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  if (a.coop > 1 && a.last) {  // waves per tile = NT (2 for F = 32, 4 for F = 64)
    const void* f = hop_coop_kernel<NT>(a.c.prelu);
    if (!f) return hipErrorInvalidValue;
    HopArgs b = a;
    const dim3 grid = xcd_grid(b, cdiv((long)a.ntiles * a.coop, kWaves));
    void* args[] = {&b};
    return hipLaunchKernel(f, grid, dim3(kBlock), args, lds_bytes<NT>(a.reg.len), st);
  }
  if (a.rows && !a.last) {  // row-layout middle hop (large meshes)
    const int nt = cdiv(a.nrows, kRowsPerWave);
    const int grid = a.max_blocks > 0 ? std::min(a.max_blocks, cdiv(nt, kRowHopWaves)) : cdiv(nt, kRowHopWaves);
    hipLaunchKernelGGL((k_hop_rows<NT>), dim3(grid), dim3(64 * kRowHopWaves), 0, st, a);
    return hipGetLastError();
  }
  if constexpr (NT >= 2) {
    if (a.split && !a.last) {  // feature-split middle hop: two waves per tile
      HopArgs b = a;
      hipLaunchKernelGGL((k_hop_split<NT>), xcd_grid(b, cdiv((long)a.ntiles * 2, kWaves)), dim3(kBlock), 0, st, b);
      return hipGetLastError();
    }
  }
  const bool loop = tile_loop(a);
  HopArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? hop_waves<NT, true>() : kWaves));
  return launch_hop_kernel<NT>(b, loop, grid, block, st);
}
template <int NT>
hipError_t launch_hop_kernel(const HopArgs& a, bool loop, dim3 grid, dim3 block, hipStream_t st) {
  if (!a.last) {
    if (loop) hipLaunchKernelGGL((k_hop<NT, 1, false, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((k_hop<NT, 1, false, false>), grid, block, 0, st, a);
  } else {
    const size_t sh = lds_bytes<NT>(a.reg.len);
    if (a.c.prelu) {
      if (loop) hipLaunchKernelGGL((k_hop<NT, 1, true, true>), grid, block, sh, st, a);
      else hipLaunchKernelGGL((k_hop<NT, 1, true, false>), grid, block, sh, st, a);
    } else {
      if (loop) hipLaunchKernelGGL((k_hop<NT, -1, true, true>), grid, block, sh, st, a);
      else hipLaunchKernelGGL((k_hop<NT, -1, true, false>), grid, block, sh, st, a);
    }
  }
  return hipGetLastError();
}
template <int NT>
hipError_t launch_pool(const PoolArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  const size_t sh = lds_bytes<NT>(a.reg.len);
  if (!a.rows) {
    PoolArgs b = a;
    if constexpr (NT >= 2) {  // 2 NT waves per tile (one tile per workgroup)
      if (a.coop == 2 * NT) {
        hipLaunchKernelGGL((k_pool_edge<NT, 2 * NT, 2 * NT>), xcd_grid(b, a.ntiles), dim3(64 * 2 * NT), sh, st, b);
        return hipGetLastError();
      }
    }
    if constexpr (NT >= 2) {  // waves per tile: 2 (F = 32), 4 (F = 64)
      if (a.coop == NT) {
        hipLaunchKernelGGL((k_pool_edge<NT, NT>), xcd_grid(b, cdiv((long)a.ntiles * NT, kWaves)), dim3(kBlock), sh, st, b);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((k_pool_edge<NT>), xcd_grid(b, cdiv(a.ntiles, kWaves)), dim3(kBlock), sh, st, b);
    return hipGetLastError();
  }
  const bool loop = tile_loop(a);
  PoolArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? waves_of<NT, true>() : kWaves));
  if (loop)
    hipLaunchKernelGGL((k_pool<NT, true>), grid, block, sh, st, b);
  else
    hipLaunchKernelGGL((k_pool<NT, false>), grid, block, sh, st, b);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_epi(const EpiArgs& a, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  const bool loop = tile_loop(a);
  EpiArgs b = a;
  const dim3 grid = loop ? dim3(tile_grid(a)) : xcd_grid(b, tile_grid(a));
  if (loop) b.c.xcd = 0;
  const dim3 block(64 * (loop ? waves_of<NT, true>() : kWaves));
  const size_t sh = lds_bytes<NT>(a.reg.len);
  if (a.c.prelu) {
    if (loop) hipLaunchKernelGGL((k_epi<NT, 1, true>), grid, block, sh, st, b);
    else hipLaunchKernelGGL((k_epi<NT, 1, false>), grid, block, sh, st, b);
  } else {
    if (loop) hipLaunchKernelGGL((k_epi<NT, -1, true>), grid, block, sh, st, b);
    else hipLaunchKernelGGL((k_epi<NT, -1, false>), grid, block, sh, st, b);
  }
  return hipGetLastError();
}
template <int NT>
hipError_t launch_rowmlp(const RowMlpArgs& a, hipStream_t st) {
  if (a.R <= 0) return hipSuccess;
  if (a.mode == 1)
    hipLaunchKernelGGL((k_rowmlp<NT, 1>), dim3(cdiv(a.R, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((k_rowmlp<NT, 0>), dim3(cdiv(a.R, kRowsPerBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

template <int NT>
hipError_t launch_decode(const DecodeArgs& a, hipStream_t st) {
  if (a.Npad <= 0) return hipSuccess;
  const dim3 grid(cdiv(a.Npad, kRowsPerBlock)), block(kBlock);
  if (a.c.prelu)
    hipLaunchKernelGGL((k_decode_fwd<NT, 1>), grid, block, 0, st, a);
  else
    hipLaunchKernelGGL((k_decode_fwd<NT, -1>), grid, block, 0, st, a);
  return hipGetLastError();
}

// Workgroups of one launch resident on the whole chip (grid cap of the grid-stride kernels).
template <int NT, bool LOOP>
static const void* kernel_of(int kind, int prelu, int last) {
  switch (kind) {
    case 0: return prelu ? (const void*)k_encode<NT, 1, false> : (const void*)k_encode<NT, -1, false>;
    case 1: return edge_hop_kernel<NT>(prelu, LOOP, last);
    case 2:
      return !last ? (const void*)k_hop<NT, 1, false, LOOP>
                   : (prelu ? (const void*)k_hop<NT, 1, true, LOOP> : (const void*)k_hop<NT, -1, true, LOOP>);
    case 3: return (const void*)k_pool<NT, LOOP>;
    case 5: return (const void*)k_pool_edge<NT>;
    case 13:
      if constexpr (NT >= 2) return (const void*)k_pool_edge<NT, 2 * NT, 2 * NT>;
      return nullptr;
    case 6: return prelu ? (const void*)k_epi<NT, 1, LOOP> : (const void*)k_epi<NT, -1, LOOP>;
    case 7: return edge_coop_kernel<NT>(prelu, last);
    case 16: return edge_coop_kernel<NT>(prelu, last, 0, 1);
    case 12: return edge_coop_kernel<NT>(prelu, last, 2);
    case 9: return hop_coop_kernel<NT>(prelu);
    case 10: return prelu ? (const void*)k_edge_mlp<NT, 1> : (const void*)k_edge_mlp<NT, -1>;
    case 14: return (const void*)k_hop_rows<NT>;
    default: return nullptr;
  }
}
template <int NT>
int resident_blocks(int kind, int prelu, int last, size_t dyn_bytes, int loop) {
  const void* f = loop ? kernel_of<NT, true>(kind, prelu, last) : kernel_of<NT, false>(kind, prelu, last);
  int per_cu = 0, dev = 0, cus = 0;
  if (!f) return 0;
  const size_t dyn = (kind == 1 || kind == 7 || kind == 10 || kind == 12) ? eh_lds_bytes((int)(dyn_bytes / 4))
                                                                          : lds_bytes<NT>((int)(dyn_bytes / 4));
  if (dyn > 160 * 1024) return 0;
  const int block = kind == 1 ? 64 * (loop ? (last ? edge_waves<NT, true, 1>() : edge_waves<NT, true, 0>()) : kWaves)
                    : kind == 10 ? 64 * kMlpWaves
                    : kind == 13 ? 64 * 2 * NT
                    : kind == 14 ? 64 * kRowHopWaves
                    : kind == 2 ? 64 * (loop ? hop_waves<NT, true>() : kWaves)
                    : 64 * (loop && (kind == 3 || kind == 6) ? waves_of<NT, true>() : kWaves);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, block, dyn) != hipSuccess)
    return 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return per_cu > 0 ? per_cu * cus : 0;
}

#define MSW_INSTANTIATE(NT)                                                       \
  template hipError_t prepare_kernels<NT>();                                      \
  template int resident_blocks<NT>(int, int, int, size_t, int);                   \
  template hipError_t launch_encode<NT>(const EncodeArgs&, hipStream_t);          \
  template hipError_t launch_edge_hop<NT>(const EdgeHopArgs&, hipStream_t);       \
  template hipError_t launch_edge_mlp<NT>(const EdgeHopArgs&, hipStream_t);       \
  template hipError_t launch_hop<NT>(const HopArgs&, hipStream_t);                \
  template hipError_t launch_pool<NT>(const PoolArgs&, hipStream_t);              \
  template hipError_t launch_epi<NT>(const EpiArgs&, hipStream_t);                \
  template hipError_t launch_rowmlp<NT>(const RowMlpArgs&, hipStream_t);           \
  template hipError_t launch_decode<NT>(const DecodeArgs&, hipStream_t);
