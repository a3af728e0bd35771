// gfx950 (MI355X, CDNA4) kernels of the multi-scale SWE-GNN rollout (templates; the
// kernels_nt*.hip units instantiate them for F = 16, 32, 64).
//
// Layout
//  * every F-wide node / edge vector is fp32, row-major, unpadded (stride F).
//  * A wave owns 16 ROWS (nodes or edges).  Lane l works on row j = l & 15 and, in lane
//    group g = l >> 4, holds features 16t + 4g + r (r = 0..3) of every 16-feature tile t
//    in one f32x4 per tile.  That is the accumulator layout of v_mfma_f32_16x16x4_f32 with
//    the row on the MFMA column (C/D: col = l & 15, row = 4(l >> 4) + r) and, register
//    for register, the B operand of the next layer (k-step (t, r): lane group g supplies
//    feature 16t + 4g + r).  Layers chain in registers: no shuffles between layers; the
//    A operands (weights) of a launch are staged once per workgroup in LDS.  Packed A operand: A[to][ti][lane][r] = W[16 to + (l & 15)][16 ti + 4 (l >> 4) + r].
//  * f32 in / f32 accumulate MFMA = exact fp32 fma chains (no TF32 on gfx950).
//  * message passing runs on edge tiles (whole destination neighbourhoods, <= 16 edges):
//    one lane per edge computes its message, the destination lane sums them from LDS in
//    the reference's edge order -- no atomics, bit-reproducible run to run.
//  * one rollout step = encoder (+ projection of processor 0) -> per processor: fused
//    edge-MLP+hop-1, hops 2..K (the last with an epilogue: next projection / unpool
//    projection / decoder + rollout update) -> pooling+projection / unpooling+projection.
#pragma once
#include <type_traits>

#include "engine.h"

namespace msw {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 64 * kWaves;
// Grid-stride (LOOP) variants of the tile kernels run 8-wave workgroups when their weights
// are staged in LDS (F <= 32): one staged copy per 8 waves instead of per 4 halves the
// staging traffic of a large mesh and the LDS the copies take.
template <int NT, bool LOOP>
constexpr int waves_of() { return LOOP && NT <= 2 ? 8 : kWaves; }
// the grid-stride middle / last hop (k_hop, large meshes): its own workgroup size
template <int NT, bool LOOP>
constexpr int hop_waves() { return LOOP && NT <= 2 ? 8 : kWaves; }
// the fused edge MLP + hop keeps one tile per wave in flight in its grid-stride loop: a
// software-pipelined loop (tile i+1's gathers and tile i+2's record during tile i's MLP) fits
// two waves per SIMD (212 VGPRs, no spills) and measured 5 % slower on the 1M-node mesh than
// four waves per SIMD without it (673 vs 639 us, profiles/r04/ab_eh_pipe_hbm1m.txt; removed)
constexpr int kEdgeWaves = 12;   // grid-stride, with epilogue (LST = 1): 3 waves per SIMD
constexpr int kEdgeWaves0 = 16;  // grid-stride, no epilogue (LST = 0): 4 waves per SIMD
// Workgroup of the grid-stride edge MLP + hop: as many waves as the register budget allows
// per SIMD, times 4 -- one workgroup per CU, so one staged weight copy serves all of them.
template <int NT, bool LOOP, int LST = 1>
constexpr int edge_waves() { return LOOP && NT <= 2 ? (LST ? kEdgeWaves : kEdgeWaves0) : kWaves; }
template <int NT, bool LOOP, int LST>
constexpr int edge_eu() { return LOOP && NT <= 2 ? edge_waves<NT, LOOP, LST>() / 4 : 1; }

#define MSW_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)


#include "kernels/k_base.h"
#include "kernels/k_encode.h"
#include "kernels/k_edge.h"
#include "kernels/k_coop_edge.h"
#include "kernels/k_coop_encode.h"
#include "kernels/k_hop.h"
#include "kernels/k_pool_epi.h"
#include "kernels/k_launch.h"

}  // namespace msw
