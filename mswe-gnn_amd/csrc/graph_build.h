// Host-side graph plan of the C ABI (plan.hip uploads what this builds): the internal
// numbering, per-scale CSR by destination in reference edge order, edge tiles and their lane
// records, dense edge chunks, the row-layout CSR of large scales, the pooling / unpooling
// records of every level (incl. the per-slot records of the fused (un)pooling launches), and
// the halo exchange lists of a partitioned mesh (msw_plan_create_part).
//
// Header-only and free of HIP, so that a host harness builds exactly this code under
// -fsanitize=address,undefined (tests/asan/host_plan_check.cpp, tests/test_host_sanitizer.py).
//
// Reference semantics: MSGNN's per-scale edge slices (edge_ptr, models/gnn.py:302-331), the
// intra-scale (coarse, fine) edges (intra_mesh_edge_index / intra_edge_ptr, gnn.py:310-327),
// the batched node_ptr of update_batch_multiscale (training/train.py:31-65).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/mswegnn.h"
#include "tiling.h"

namespace msw {

constexpr int kRowsPerWave = 16;  // v_mfma_f32_16x16x4_f32: 16 rows (nodes / edges) per wave
constexpr int kMaxScales = 8;
constexpr int kPoolInline = 4;

struct I2 {  // host twin of HIP's int2 (same size and field order)
  int x, y;
};

// Edge tile: whole destination neighbourhoods, <= 16 edges and <= 16 destinations (host).
struct TileRange {
  int node0, nnode, edge0, nedge;  // local node index / local CSR edge index
};
// What lane j of a tile's wave needs, one 16-B load: as edge lane, edge slot j of the tile
// (source row, local lane of its destination); as node lane, destination j (row, slot
// range [q & 255, q >> 8) of its in-edges).  Per-edge arrays (Pe, s) are tile-padded:
// edge slot j of tile t lives at row 16 t + j.
struct LaneRec {
  int src;  // internal source row, -1 = no edge in this slot
  int dl;   // destination lane (0..15) of the edge
  int n;    // internal destination row, -1 = no node in this lane
  int q;    // q0 | q1 << 8
};
// Dense edge chunks of a scale (k_edge_mlp): 16 consecutive real edges of the tile order,
// padding slots skipped; src / dst internal rows and the edge's tile-padded slot p
// (-1 = past the last edge).
struct EdgeChunk {
  int src, dst, p, pad;
};
// Children of one coarse row (32 B, one 16-B + one 8-B load): the first kPoolInline
// internal fine rows, the count, and where the full list starts in PoolArgs::child.
struct alignas(16) PoolRec {
  int c[kPoolInline];
  int cnt, off, pad[2];
};
// Pooling fused into the coarse scale's first edge-MLP + hop launch (k_edge_coop, POOL):
// per tile-padded edge slot of the coarse scale, the children of the slot's source (edge
// lane) and of the lane's destination (node lane), as PoolRec (absent: cnt 0, children =
// a safe fine row).
struct alignas(16) PoolSlot {
  PoolRec src, dst;
};

struct HostScale {
  int n0 = 0, ns = 0;            // internal rows [n0, n0 + ns)
  int E = 0;                     // edges of this scale
  int ntiles = 0, nchunks = 0;
  std::vector<LaneRec> recs;     // [ntiles][16]
  std::vector<EdgeChunk> chunks; // [nchunks][16]
  std::vector<int> porig;        // tile-padded edge slot -> original edge id, -1 = padding
  std::vector<int> rptr;         // row layout (large scales): CSR offsets by local destination
  std::vector<I2> redge;         //   {internal source row, tile-padded s slot} per CSR edge
};
struct HostLevel {               // level l: coarse scale l + 1, fine scale l
  int I = 0;
  std::vector<PoolRec> pool_recs;      // per coarse row (16-row padded)
  std::vector<LaneRec> pool_erecs;     // edge tiles of coarse nodes and their children
  int pool_etiles = 0;
  std::vector<int> pool_child;         // internal fine rows, reference order (>= 1 entry)
  std::vector<PoolSlot> pool_slots;    // per edge slot of the coarse scale (empty: no edges)
  std::vector<LaneRec> un_recs;        // fine nodes and their coarse parents
  int un_ntiles = 0;
  std::vector<I2> parent_slots;        // per edge slot of the fine scale: parents of its two
                                       // nodes (empty: some fine node has > 1 parent)
};
struct HostGraph {
  int N = 0, Npad = 0;
  int64_t E = 0;
  std::vector<int> perm, iperm;        // internal -> graph row (-1 = padding), graph -> internal
  std::vector<HostScale> sc;
  std::vector<HostLevel> lv;
};

// Halo exchange of a partitioned mesh: per scale, the internal rows received from / sent to
// each peer, concatenated in entry order.
struct XchPeer {
  int peer, roff, rcount, soff, scount;
};
struct HostXchScale {
  std::vector<int> recv_rows, send_rows;
  std::vector<XchPeer> peers;
};

// Stable counting sort by key in [0, nkeys): rowptr + order (original indices).
inline void csr_build(int nkeys, const std::vector<int>& key, std::vector<int>& rowptr, std::vector<int>& order) {
  rowptr.assign(nkeys + 1, 0);
  for (int k : key) rowptr[k + 1]++;
  for (int i = 0; i < nkeys; ++i) rowptr[i + 1] += rowptr[i];
  std::vector<int> pos(rowptr.begin(), rowptr.end() - 1);
  order.assign(key.size(), 0);
  for (size_t e = 0; e < key.size(); ++e) order[pos[key[e]]++] = (int)e;
}

// Edge tiles over a CSR by destination: consecutive destinations with <= 16 in-edges and
// <= 16 destinations per tile (whole neighbourhoods, so hop 1 fuses into the edge MLP).
inline int build_tiles(const std::vector<int>& rowptr, std::vector<TileRange>& out, std::string& err) {
  out.clear();
  const int ns = (int)rowptr.size() - 1;
  int a = 0;
  while (a < ns) {
    int b = a, edges = 0;
    while (b < ns && b - a < kRowsPerWave) {
      const int d = rowptr[b + 1] - rowptr[b];
      if (d > kRowsPerWave) {
        err = "node with more than 16 in-edges";
        return MSW_ERR_UNSUPPORTED;
      }
      if (edges + d > kRowsPerWave) break;
      edges += d;
      ++b;
    }
    out.push_back(TileRange{a, b - a, rowptr[a], edges});
    a = b;
  }
  return MSW_OK;
}

// Per-lane tile records of a CSR by destination: `src` = source row of CSR edge i (internal
// numbering), `n0` = first internal row of the destination scale.  porig (optional)
// receives, per tile-padded edge slot, the CSR position or -1.
inline std::vector<LaneRec> make_recs(const std::vector<int>& rowptr, const std::vector<int>& src, int n0,
                                      const std::vector<TileRange>& tiles, std::vector<int>* porig) {
  std::vector<LaneRec> r(tiles.size() * kRowsPerWave, LaneRec{-1, 0, -1, 0});
  if (porig) porig->assign(tiles.size() * kRowsPerWave, -1);
  for (size_t t = 0; t < tiles.size(); ++t) {
    const TileRange& tr = tiles[t];
    LaneRec* L = &r[t * kRowsPerWave];
    for (int j = 0; j < tr.nnode; ++j) {
      const int k = tr.node0 + j;
      const int q0 = rowptr[k] - tr.edge0, q1 = rowptr[k + 1] - tr.edge0;
      L[j].n = n0 + k;
      L[j].q = q0 | (q1 << 8);
      for (int q = q0; q < q1; ++q) {
        L[q].src = src[tr.edge0 + q];
        L[q].dl = j;
        if (porig) (*porig)[t * kRowsPerWave + q] = tr.edge0 + q;
      }
    }
  }
  return r;
}

// The whole host graph plan.  align: scale starts are padded to multiples of this many rows
// (the encoder's workgroup rows: a workgroup never straddles two scales); pack: destinations
// in tiling.h pack_order (else graph order); row_min_tiles: scales with at least this many
// edge tiles get the row-layout CSR (0: every scale).  Returns MSW_OK or an MSW_ERR_* code
// with `err` set.
inline int build_host_graph(const msw_graph_desc* g, int S, int align, bool pack, int row_min_tiles, HostGraph& H,
                            std::string& err) {
  auto bad = [&](int code, const std::string& m) {
    err = m;
    return code;
  };
  if (!g) return bad(MSW_ERR_INVALID, "null graph");
  const int G = g->num_graphs;
  if (S < 1 || S > kMaxScales) return bad(MSW_ERR_UNSUPPORTED, "1 to 8 scales");
  if (g->num_nodes <= 0 || g->num_nodes > (1LL << 30)) return bad(MSW_ERR_INVALID, "num_nodes out of range");
  if (g->num_edges < 0 || g->num_edges > (1LL << 31) - 64) return bad(MSW_ERR_INVALID, "num_edges out of range");
  if (G < 1 || !g->node_ptr) return bad(MSW_ERR_INVALID, "node_ptr missing");
  if (g->num_scales != S) return bad(MSW_ERR_INVALID, "graph num_scales != model num_scales");
  if (g->num_edges > 0 && !g->edge_index) return bad(MSW_ERR_INVALID, "edge_index missing");
  if (!g->edge_ptr) return bad(MSW_ERR_INVALID, "edge_ptr missing");
  const int N = (int)g->num_nodes;
  H = HostGraph{};
  H.N = N;
  H.E = g->num_edges;
  // internal numbering: scale-major (graph-major inside a scale), each graph's destinations of
  // a scale in pack_order, scale starts padded to multiples of `align` rows
  H.sc.assign(S, HostScale{});
  std::vector<int> indeg(pack ? N : 0, 0);
  if (pack)
    for (int64_t e = 0; e < g->num_edges; ++e) {
      const int64_t cl = g->edge_index[g->num_edges + e];
      if (cl >= 0 && cl < N) ++indeg[cl];
    }
  int64_t placed = 0;
  for (int s = 0; s < S; ++s) {
    H.sc[s].n0 = (int)H.perm.size();
    for (int gi = 0; gi < G; ++gi) {
      const int64_t a = g->node_ptr[gi * (S + 1) + s], b = g->node_ptr[gi * (S + 1) + s + 1];
      if (a < 0 || b < a || b > N) return bad(MSW_ERR_INVALID, "node_ptr out of range");
      if ((placed += b - a) > N) return bad(MSW_ERR_INVALID, "node_ptr ranges overlap");
      if (pack) {
        std::vector<int> d((size_t)(b - a));
        for (int64_t v = a; v < b; ++v) d[v - a] = indeg[v];
        for (int k : pack_order(d)) H.perm.push_back((int)(a + k));
      } else {
        for (int64_t v = a; v < b; ++v) H.perm.push_back((int)v);
      }
    }
    H.sc[s].ns = (int)H.perm.size() - H.sc[s].n0;
    H.perm.resize((H.perm.size() + align - 1) / align * align, -1);
  }
  H.Npad = (int)H.perm.size();
  H.iperm.assign(N, -1);
  int covered = 0;
  for (int i = 0; i < H.Npad; ++i) {
    if (H.perm[i] < 0) continue;
    if (H.iperm[H.perm[i]] != -1) return bad(MSW_ERR_INVALID, "node_ptr ranges overlap");
    H.iperm[H.perm[i]] = i;
    ++covered;
  }
  if (covered != N) return bad(MSW_ERR_INVALID, "node_ptr does not cover every node exactly once");
  // per-scale CSR by destination + edge tiles
  const int64_t E = g->num_edges;
  if (g->edge_ptr[0] != 0 || g->edge_ptr[S] != E) return bad(MSW_ERR_INVALID, "edge_ptr must span [0, E]");
  int rc;
  for (int s = 0; s < S; ++s) {
    HostScale& c = H.sc[s];
    const int64_t a = g->edge_ptr[s], b = g->edge_ptr[s + 1];
    if (a < 0 || b < a || b > E) return bad(MSW_ERR_INVALID, "edge_ptr not monotone");
    c.E = (int)(b - a);
    std::vector<int> key(c.E), srcv(c.E);
    for (int64_t e = a; e < b; ++e) {
      const int64_t r = g->edge_index[e], cl = g->edge_index[E + e];
      if (r < 0 || r >= N || cl < 0 || cl >= N) return bad(MSW_ERR_INVALID, "edge_index out of range");
      const int ri = H.iperm[r], ci = H.iperm[cl];
      if (ri < c.n0 || ri >= c.n0 + c.ns || ci < c.n0 || ci >= c.n0 + c.ns)
        return bad(MSW_ERR_INVALID, "edge of scale " + std::to_string(s) + " leaves the scale");
      key[e - a] = ci - c.n0;
      srcv[e - a] = ri;
    }
    std::vector<int> rowptr, order;
    csr_build(c.ns, key, rowptr, order);
    std::vector<int> so(c.E);
    for (int i = 0; i < c.E; ++i) so[i] = srcv[order[i]];
    std::vector<TileRange> tl;
    if ((rc = build_tiles(rowptr, tl, err))) return rc;
    c.ntiles = (int)tl.size();
    std::vector<int> pcsr;
    c.recs = make_recs(rowptr, so, c.n0, tl, &pcsr);
    c.porig.assign(pcsr.size(), -1);
    for (size_t q = 0; q < pcsr.size(); ++q)
      if (pcsr[q] >= 0) c.porig[q] = (int)(a + order[pcsr[q]]);
    for (size_t q = 0; q < c.recs.size(); ++q)
      if (c.recs[q].src >= 0)
        c.chunks.push_back(EdgeChunk{c.recs[q].src, c.recs[q / kRowsPerWave * kRowsPerWave + c.recs[q].dl].n, (int)q, 0});
    c.nchunks = (int)((c.chunks.size() + kRowsPerWave - 1) / kRowsPerWave);
    c.chunks.resize((size_t)c.nchunks * kRowsPerWave, EdgeChunk{-1, -1, -1, 0});
    if (c.ntiles >= row_min_tiles) {  // row-layout middle hops: CSR + s slots
      std::vector<int> slot_of_csr(c.E, -1);
      for (size_t q = 0; q < pcsr.size(); ++q)
        if (pcsr[q] >= 0) slot_of_csr[pcsr[q]] = (int)q;
      c.rptr = rowptr;
      c.redge.resize(std::max(c.E, 1), I2{0, 0});
      for (int i = 0; i < c.E; ++i) c.redge[i] = I2{so[i], slot_of_csr[i]};
    }
  }
  // intra-scale levels
  H.lv.assign(S > 1 ? S - 1 : 0, HostLevel{});
  if (S > 1) {
    if (!g->intra_edge_index || !g->intra_edge_ptr) return bad(MSW_ERR_INVALID, "intra edges missing");
    const int64_t I = g->num_intra_edges;
    for (int l = 0; l < S - 1; ++l) {
      HostLevel& m = H.lv[l];
      const HostScale& cs = H.sc[l + 1];
      const HostScale& fs = H.sc[l];
      const int64_t a = g->intra_edge_ptr[l], b = g->intra_edge_ptr[l + 1];
      if (a < 0 || b < a || b > I) return bad(MSW_ERR_INVALID, "intra_edge_ptr out of range");
      m.I = (int)(b - a);
      std::vector<int> ck(m.I), fk(m.I), cv(m.I), fv(m.I);
      for (int64_t e = a; e < b; ++e) {
        const int64_t co = g->intra_edge_index[e], fi = g->intra_edge_index[I + e];
        if (co < 0 || co >= N || fi < 0 || fi >= N) return bad(MSW_ERR_INVALID, "intra edge out of range");
        const int ci = H.iperm[co], fii = H.iperm[fi];
        if (ci < cs.n0 || ci >= cs.n0 + cs.ns || fii < fs.n0 || fii >= fs.n0 + fs.ns)
          return bad(MSW_ERR_INVALID, "intra edge of level " + std::to_string(l) + " not (coarse, fine)");
        ck[e - a] = ci - cs.n0;
        fk[e - a] = fii - fs.n0;
        cv[e - a] = ci;
        fv[e - a] = fii;
      }
      std::vector<int> rp, order;
      csr_build(cs.ns, ck, rp, order);
      m.pool_child.resize(m.I);
      for (int i = 0; i < m.I; ++i) m.pool_child[i] = fv[order[i]];
      m.pool_recs.resize((size_t)(cs.ns + 15) / 16 * 16);
      for (size_t i = 0; i < m.pool_recs.size(); ++i) {
        PoolRec& r = m.pool_recs[i];
        const int b0 = i < (size_t)cs.ns ? rp[i] : 0, e0 = i < (size_t)cs.ns ? rp[i + 1] : 0;
        r.cnt = e0 - b0;
        r.off = b0;
        r.pad[0] = r.pad[1] = 0;
        for (int k = 0; k < kPoolInline; ++k) r.c[k] = k < e0 - b0 ? m.pool_child[b0 + k] : -1;
      }
      std::vector<TileRange> pt;
      if ((rc = build_tiles(rp, pt, err))) return rc;
      m.pool_etiles = (int)pt.size();
      m.pool_erecs = make_recs(rp, m.pool_child, cs.n0, pt, nullptr);
      if (!cs.recs.empty()) {  // fused pooling: the records of each slot's two coarse nodes
        auto rec_of = [&](int row) {
          PoolRec r{};
          if (row >= cs.n0 && row < cs.n0 + cs.ns) r = m.pool_recs[row - cs.n0];
          const int safe = r.cnt > 0 ? r.c[0] : fs.n0;  // absent children re-read a real row
          for (int k = 0; k < kPoolInline; ++k)
            if (k >= r.cnt) r.c[k] = safe;
          return r;
        };
        m.pool_slots.resize(cs.recs.size());
        for (size_t q = 0; q < m.pool_slots.size(); ++q) {
          m.pool_slots[q].src = rec_of(cs.recs[q].src);
          m.pool_slots[q].dst = rec_of(cs.recs[q].n);
        }
      }
      if (m.pool_child.empty()) m.pool_child.push_back(0);
      csr_build(fs.ns, fk, rp, order);
      std::vector<int> us(m.I);
      for (int i = 0; i < m.I; ++i) us[i] = cv[order[i]];
      std::vector<TileRange> tl;
      if ((rc = build_tiles(rp, tl, err))) return rc;
      m.un_ntiles = (int)tl.size();
      m.un_recs = make_recs(rp, us, fs.n0, tl, nullptr);
      bool one = true;  // fused unpooling: one parent per fine node at most (else the launch stays)
      std::vector<int> par(fs.ns, -1);
      for (int i = 0; i < fs.ns; ++i) {
        if (rp[i + 1] - rp[i] > 1) one = false;
        if (rp[i + 1] > rp[i]) par[i] = us[rp[i]];
      }
      if (one && !fs.recs.empty()) {
        auto par_of = [&](int row) { return row >= fs.n0 && row < fs.n0 + fs.ns ? par[row - fs.n0] : -1; };
        m.parent_slots.resize(fs.recs.size());
        for (size_t q = 0; q < m.parent_slots.size(); ++q)
          m.parent_slots[q] = I2{par_of(fs.recs[q].src), par_of(fs.recs[q].n)};
      }
    }
  }
  return MSW_OK;
}

// Partitioned mesh: per-scale receive / send row lists (local graph rows -> internal rows),
// validated against the plan's numbering (rows in range and on the entry's scale, peers
// other than this rank).
inline int build_host_exchange(const HostGraph& H, int part_rank, const msw_exchange_desc* d,
                               std::vector<HostXchScale>& X, std::string& err) {
  const int S = (int)H.sc.size();
  X.assign(S, HostXchScale{});
  if (!d || d->num_entries < 0) {
    err = "null exchange descriptor";
    return MSW_ERR_INVALID;
  }
  if (d->num_entries > 0 && (!d->scale || !d->peer || !d->recv_ptr || !d->send_ptr)) {
    err = "exchange descriptor arrays missing";
    return MSW_ERR_INVALID;
  }
  for (int i = 0; i < d->num_entries; ++i) {
    const int s = d->scale[i];
    if (s < 0 || s >= S) {
      err = "exchange entry with a bad scale";
      return MSW_ERR_INVALID;
    }
    const HostScale& c = H.sc[s];
    const int64_t r0 = d->recv_ptr[i], r1 = d->recv_ptr[i + 1], s0 = d->send_ptr[i], s1 = d->send_ptr[i + 1];
    if (r1 < r0 || s1 < s0 || r0 < 0 || s0 < 0 || (r1 > r0 && !d->recv_rows) || (s1 > s0 && !d->send_rows)) {
      err = "exchange row ranges malformed";
      return MSW_ERR_INVALID;
    }
    XchPeer pe{d->peer[i], (int)X[s].recv_rows.size(), (int)(r1 - r0), (int)X[s].send_rows.size(), (int)(s1 - s0)};
    if (pe.peer < 0) {
      err = "exchange entry with a bad peer";
      return MSW_ERR_INVALID;
    }
    // an entry with peer == part_rank exchanges rows with the rank itself (RCCL send / recv
    // to self): one-rank communicators, and the transport check on a one-GPU box
    if (pe.peer == part_rank && pe.rcount != pe.scount) {
      err = "self exchange entry: receive and send counts differ";
      return MSW_ERR_INVALID;
    }
    auto conv = [&](const int32_t* rows, int64_t a, int64_t b, std::vector<int>& dst) -> int {
      for (int64_t k = a; k < b; ++k) {
        const int r = rows[k];
        if (r < 0 || r >= H.N) {
          err = "exchange row out of range";
          return MSW_ERR_INVALID;
        }
        const int in = H.iperm[r];
        if (in < c.n0 || in >= c.n0 + c.ns) {
          err = "exchange row not on the entry's scale";
          return MSW_ERR_INVALID;
        }
        dst.push_back(in);
      }
      return MSW_OK;
    };
    int rc;
    if ((rc = conv(d->recv_rows, r0, r1, X[s].recv_rows)) || (rc = conv(d->send_rows, s0, s1, X[s].send_rows)))
      return rc;
    X[s].peers.push_back(pe);
  }
  return MSW_OK;
}

}  // namespace msw
