// Sanitizer harness for the host side of plan creation (SURVEY §5 "optional ASan on host
// code"; tests/test_host_cpu.py builds it with g++ -fsanitize=address,undefined and runs it).
// It drives EXACTLY the code msw_plan_create / msw_plan_create_part run on the host
// (mswe-gnn_amd/csrc/graph_build.h: numbering, CSR by destination, tiling.h pack_order, edge
// tiles and lane records, edge chunks, row-layout CSR, pooling / unpooling records, fused
// (un)pooling slot records, partition exchange lists) on graphs written by the test, and
// checks every structural invariant the kernels rely on.  Any violation, sanitizer report or
// unexpected return code exits non-zero.
//
//   host_plan_check CASES.bin  ->  one JSON line per case on stdout
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "graph_build.h"

using namespace msw;

#define CHECK(cond, ...)                                              \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "CHECK failed (%s:%d): %s: ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                              \
      std::fprintf(stderr, "\n");                                     \
      std::exit(3);                                                   \
    }                                                                 \
  } while (0)

struct Reader {
  FILE* f;
  int64_t i64() {
    int64_t v;
    CHECK(std::fread(&v, 8, 1, f) == 1, "truncated case file");
    return v;
  }
  std::vector<int64_t> vec(int64_t n) {
    CHECK(n >= 0 && n < (1LL << 32), "bad array length %lld", (long long)n);
    std::vector<int64_t> v((size_t)n);
    if (n) CHECK(std::fread(v.data(), 8, (size_t)n, f) == (size_t)n, "truncated array");
    return v;
  }
};

struct Case {
  std::string name;
  int64_t S, G, N, E, I, expect_rc, group, rank;
  std::vector<int64_t> node_ptr, edge_index, edge_ptr, intra_index, intra_ptr;
  bool has_xch = false;
  std::vector<int32_t> peer, scale, recv_rows, send_rows;
  std::vector<int64_t> recv_ptr, send_ptr, l2g;
};

static std::vector<int32_t> as32(const std::vector<int64_t>& v) { return std::vector<int32_t>(v.begin(), v.end()); }

static bool read_case(Reader& r, Case& c) {
  int64_t magic;
  if (std::fread(&magic, 8, 1, r.f) != 1) return false;
  CHECK(magic == 0x45534143, "bad case magic");
  const int64_t nlen = r.i64();
  std::vector<int64_t> nm = r.vec(nlen);
  c.name.assign(nm.begin(), nm.end());
  c.S = r.i64(); c.G = r.i64(); c.N = r.i64(); c.E = r.i64(); c.I = r.i64();
  c.expect_rc = r.i64(); c.group = r.i64(); c.rank = r.i64();
  c.node_ptr = r.vec(c.G * (c.S + 1));
  c.edge_index = r.vec(2 * c.E);
  c.edge_ptr = r.vec(c.S + 1);
  c.intra_index = r.vec(2 * c.I);
  c.intra_ptr = r.vec(c.S > 1 ? c.S : 0);
  const int64_t ne = r.i64();
  c.has_xch = ne >= 0;
  if (c.has_xch) {
    c.peer = as32(r.vec(ne));
    c.scale = as32(r.vec(ne));
    c.recv_ptr = r.vec(ne + 1);
    c.recv_rows = as32(r.vec(c.recv_ptr.back()));
    c.send_ptr = r.vec(ne + 1);
    c.send_rows = as32(r.vec(c.send_ptr.back()));
    c.l2g = r.vec(c.N);
  }
  return true;
}

static msw_graph_desc desc_of(const Case& c) {
  msw_graph_desc g{};
  g.num_nodes = c.N;
  g.num_scales = (int32_t)c.S;
  g.num_graphs = (int32_t)c.G;
  g.node_ptr = c.node_ptr.data();
  g.num_edges = c.E;
  g.edge_index = c.edge_index.data();
  g.edge_attr = nullptr;
  g.num_edge_features = 1;
  g.edge_ptr = c.edge_ptr.data();
  g.num_intra_edges = c.I;
  g.intra_edge_index = c.S > 1 ? c.intra_index.data() : nullptr;
  g.intra_edge_ptr = c.S > 1 ? c.intra_ptr.data() : nullptr;
  return g;
}

// every invariant of one host plan (graph_build.h) the kernels rely on
static void check_plan(const Case& c, const HostGraph& H, int align, bool rows_all) {
  const int S = (int)c.S, N = (int)c.N;
  CHECK(H.Npad % align == 0 && (int)H.perm.size() == H.Npad, "padding");
  for (int i = 0; i < H.Npad; ++i)
    if (H.perm[i] >= 0) CHECK(H.iperm[H.perm[i]] == i, "perm / iperm not inverse at %d", i);
  for (int v = 0; v < N; ++v) CHECK(H.iperm[v] >= 0 && H.perm[H.iperm[v]] == v, "node %d unmapped", v);
  for (int s = 0; s < S; ++s) {
    const HostScale& sc = H.sc[s];
    CHECK(sc.n0 % align == 0, "scale start");
    int64_t want = 0;
    for (int g = 0; g < c.G; ++g) want += c.node_ptr[g * (S + 1) + s + 1] - c.node_ptr[g * (S + 1) + s];
    CHECK(sc.ns == want, "scale %d rows %d != %lld", s, sc.ns, (long long)want);
    for (int i = sc.n0; i < sc.n0 + sc.ns; ++i) CHECK(H.perm[i] >= 0, "hole inside scale %d", s);
    // edge slots: a permutation of the scale's edges; per destination in reference order
    const int64_t ea = c.edge_ptr[s], eb = c.edge_ptr[s + 1];
    CHECK((int64_t)sc.E == eb - ea, "scale edge count");
    CHECK(sc.recs.size() == (size_t)sc.ntiles * kRowsPerWave && sc.porig.size() == sc.recs.size(), "record sizes");
    std::vector<char> seen((size_t)(eb - ea), 0);
    for (int t = 0; t < sc.ntiles; ++t) {
      const LaneRec* L = &sc.recs[(size_t)t * kRowsPerWave];
      int covered = 0, prev_q1 = 0;
      for (int j = 0; j < kRowsPerWave; ++j) {
        if (L[j].n < 0) continue;
        const int q0 = L[j].q & 255, q1 = L[j].q >> 8;
        CHECK(q0 == prev_q1 && q1 >= q0 && q1 <= kRowsPerWave, "tile %d lane %d slot range", t, j);
        prev_q1 = q1;
        CHECK(L[j].n >= sc.n0 && L[j].n < sc.n0 + sc.ns, "destination row outside scale");
        int64_t last = -1;
        for (int q = q0; q < q1; ++q) {
          const int e = sc.porig[(size_t)t * kRowsPerWave + q];
          CHECK(e >= ea && e < eb, "slot edge outside scale");
          CHECK(!seen[e - ea], "edge %d in two slots", e);
          seen[e - ea] = 1;
          CHECK(e > last, "in-edges of a destination out of reference order");
          last = e;
          CHECK(L[q].dl == j, "edge lane's destination lane");
          CHECK(L[q].src == H.iperm[c.edge_index[e]], "edge lane's source row");
          CHECK(L[j].n == H.iperm[c.edge_index[c.E + e]], "edge slot under the wrong destination");
          ++covered;
        }
      }
      for (int q = covered; q < kRowsPerWave; ++q)
        CHECK(L[q].src == -1 && sc.porig[(size_t)t * kRowsPerWave + q] == -1, "padding slot holds an edge");
    }
    for (size_t e = 0; e < seen.size(); ++e) CHECK(seen[e], "edge %zu of scale %d in no slot", e, s);
    // dense chunks: each real slot once
    CHECK(sc.chunks.size() == (size_t)sc.nchunks * kRowsPerWave, "chunk size");
    std::vector<char> cs(sc.recs.size(), 0);
    int real = 0;
    for (const EdgeChunk& k : sc.chunks) {
      if (k.p < 0) continue;
      CHECK(k.p < (int)sc.recs.size() && !cs[k.p] && sc.recs[k.p].src == k.src, "chunk slot");
      cs[k.p] = 1;
      ++real;
    }
    CHECK(real == sc.E, "chunks cover %d of %d edges", real, sc.E);
    // row layout (forced on every scale in the second pass)
    if (rows_all) CHECK(!sc.rptr.empty() || sc.ns == 0, "row layout missing");
    if (!sc.rptr.empty()) {
      CHECK((int)sc.rptr.size() == sc.ns + 1 && sc.rptr[sc.ns] == sc.E, "row CSR size");
      for (int k = 0; k < sc.ns; ++k)
        for (int q = sc.rptr[k]; q < sc.rptr[k + 1]; ++q) {
          const I2 r = sc.redge[q];
          CHECK(r.y >= 0 && r.y < (int)sc.porig.size(), "row edge slot");
          const int e = sc.porig[r.y];
          CHECK(H.iperm[c.edge_index[c.E + e]] == sc.n0 + k && H.iperm[c.edge_index[e]] == r.x, "row edge");
          if (q > sc.rptr[k]) CHECK(sc.porig[sc.redge[q - 1].y] < e, "row edges out of order");
        }
    }
  }
  // levels
  for (int l = 0; l + 1 < S; ++l) {
    const HostLevel& m = H.lv[l];
    const HostScale &cs = H.sc[l + 1], &fs = H.sc[l];
    const int64_t a = c.intra_ptr[l], b = c.intra_ptr[l + 1];
    CHECK(m.I == b - a, "level %d intra count", l);
    std::map<int, std::vector<int>> kids;  // coarse internal row -> fine internal rows (edge order)
    std::map<int, std::vector<int>> pars;
    for (int64_t e = a; e < b; ++e) {
      const int co = H.iperm[c.intra_index[e]], fi = H.iperm[c.intra_index[c.I + e]];
      kids[co].push_back(fi);
      pars[fi].push_back(co);
    }
    CHECK(m.pool_recs.size() % 16 == 0 && m.pool_recs.size() >= (size_t)cs.ns, "pool record size");
    for (int i = 0; i < cs.ns; ++i) {
      const PoolRec& r = m.pool_recs[i];
      const std::vector<int>& k = kids[cs.n0 + i];
      CHECK(r.cnt == (int)k.size(), "pool count");
      for (int q = 0; q < r.cnt; ++q) CHECK(m.pool_child[r.off + q] == k[q], "pool child order");
      for (int q = 0; q < kPoolInline; ++q) CHECK(r.c[q] == (q < r.cnt ? k[q] : -1), "inline children");
    }
    if (!m.pool_slots.empty()) {
      CHECK(m.pool_slots.size() == cs.recs.size(), "pool slot size");
      for (size_t q = 0; q < cs.recs.size(); ++q) {
        const int rows[2] = {cs.recs[q].src, cs.recs[q].n};
        const PoolRec* pr[2] = {&m.pool_slots[q].src, &m.pool_slots[q].dst};
        for (int side = 0; side < 2; ++side) {
          const int row = rows[side];
          const int want = (row >= cs.n0 && row < cs.n0 + cs.ns) ? (int)kids[row].size() : 0;
          CHECK(pr[side]->cnt == want, "slot %zu side %d children", q, side);
          for (int k = 0; k < kPoolInline; ++k) {
            const int v = pr[side]->c[k];
            CHECK(v >= fs.n0 && v < fs.n0 + fs.ns, "slot child row outside the fine scale (a load the kernel issues)");
          }
        }
      }
    }
    int un_edges = 0;
    for (int t = 0; t < m.un_ntiles; ++t)
      for (int j = 0; j < kRowsPerWave; ++j) {
        const LaneRec& L = m.un_recs[(size_t)t * kRowsPerWave + j];
        if (L.src >= 0) {
          ++un_edges;
          const int dst = m.un_recs[(size_t)t * kRowsPerWave + L.dl].n;
          bool ok = false;
          for (int p : pars[dst]) ok = ok || p == L.src;
          CHECK(ok, "unpool edge not an intra edge");
        }
      }
    CHECK(un_edges == m.I, "unpool tiles cover %d of %d intra edges", un_edges, m.I);
    if (!m.parent_slots.empty()) {
      CHECK(m.parent_slots.size() == fs.recs.size(), "parent slot size");
      for (size_t q = 0; q < fs.recs.size(); ++q) {
        const int rows[2] = {fs.recs[q].src, fs.recs[q].n};
        const int got[2] = {m.parent_slots[q].x, m.parent_slots[q].y};
        for (int side = 0; side < 2; ++side) {
          const int row = rows[side];
          const auto it = pars.find(row);
          const int want = (row >= fs.n0 && row < fs.n0 + fs.ns && it != pars.end()) ? it->second[0] : -1;
          CHECK(got[side] == want, "parent of slot %zu side %d", q, side);
        }
      }
    }
  }
}

int main(int argc, char** argv) {
  CHECK(argc == 2, "usage: host_plan_check CASES.bin");
  Reader r{std::fopen(argv[1], "rb")};
  CHECK(r.f, "cannot open %s", argv[1]);
  std::vector<Case> cases;
  Case c;
  while (read_case(r, c)) cases.push_back(c);
  std::fclose(r.f);
  std::map<int64_t, std::vector<std::pair<const Case*, std::vector<HostXchScale>>>> groups;
  std::map<int64_t, std::vector<const HostGraph*>> ghosts;
  std::vector<HostGraph> keep(cases.size());
  for (size_t ci = 0; ci < cases.size(); ++ci) {
    const Case& k = cases[ci];
    const msw_graph_desc g = desc_of(k);
    std::string err;
    HostGraph& H = keep[ci];
    const int rc = build_host_graph(&g, (int)k.S, 64, true, 65536, H, err);
    CHECK(rc == k.expect_rc, "case %s: rc %d (%s), expected %lld", k.name.c_str(), rc, err.c_str(),
          (long long)k.expect_rc);
    if (rc != MSW_OK) {
      std::printf("{\"case\": \"%s\", \"rc\": %d, \"error\": \"%s\"}\n", k.name.c_str(), rc, err.c_str());
      continue;
    }
    check_plan(k, H, 64, false);
    HostGraph H2;  // graph order, row layout on every scale, other alignment
    CHECK(build_host_graph(&g, (int)k.S, 16, false, 0, H2, err) == MSW_OK, "second pass: %s", err.c_str());
    check_plan(k, H2, 16, true);
    std::printf("{\"case\": \"%s\", \"rc\": 0, \"Npad\": %d, \"ntiles\": [", k.name.c_str(), H.Npad);
    for (int s = 0; s < (int)k.S; ++s) std::printf("%s%d", s ? ", " : "", H.sc[s].ntiles);
    std::printf("], \"ntiles_graph_order\": [");
    for (int s = 0; s < (int)k.S; ++s) std::printf("%s%d", s ? ", " : "", H2.sc[s].ntiles);
    std::printf("], \"fused_pool_levels\": [");
    for (int l = 0; l + 1 < (int)k.S; ++l) std::printf("%s%d", l ? ", " : "", (int)!H.lv[l].pool_slots.empty());
    std::printf("], \"fused_unpool_levels\": [");
    for (int l = 0; l + 1 < (int)k.S; ++l) std::printf("%s%d", l ? ", " : "", (int)!H.lv[l].parent_slots.empty());
    std::printf("]");
    if (k.has_xch) {
      msw_exchange_desc d{};
      d.num_entries = (int32_t)k.peer.size();
      d.peer = k.peer.data();
      d.scale = k.scale.data();
      d.recv_ptr = k.recv_ptr.data();
      d.recv_rows = k.recv_rows.data();
      d.send_ptr = k.send_ptr.data();
      d.send_rows = k.send_rows.data();
      std::vector<HostXchScale> X;
      CHECK(build_host_exchange(H, (int)k.rank, &d, X, err) == MSW_OK, "exchange: %s", err.c_str());
      int halo = 0;
      for (const auto& x : X) halo += (int)x.recv_rows.size();
      std::printf(", \"halo_rows\": %d", halo);
      groups[k.group].push_back({&k, X});
      ghosts[k.group].push_back(&H);
    }
    std::printf("}\n");
  }
  // partitions: what rank r receives from p on scale s is what p sends to r, row for row
  // (global ids via each part's local -> global map), and every halo row is received once
  for (auto& [gid, parts] : groups) {
    std::map<int64_t, size_t> by_rank;
    for (size_t i = 0; i < parts.size(); ++i) by_rank[parts[i].first->rank] = i;
    for (size_t i = 0; i < parts.size(); ++i) {
      const Case& a = *parts[i].first;
      const HostGraph& Ha = *ghosts[gid][i];
      for (size_t s = 0; s < parts[i].second.size(); ++s)
        for (const XchPeer& pe : parts[i].second[s].peers) {
          CHECK(by_rank.count(pe.peer), "peer %d of rank %lld missing from group", pe.peer, (long long)a.rank);
          const size_t j = by_rank[pe.peer];
          const Case& b = *parts[j].first;
          const HostGraph& Hb = *ghosts[gid][j];
          const XchPeer* back = nullptr;
          for (const XchPeer& q : parts[j].second[s].peers)
            if (q.peer == a.rank) back = &q;
          CHECK(back && back->scount == pe.rcount, "rank %lld scale %zu: peer %d sends %d rows, %d received",
                (long long)a.rank, s, pe.peer, back ? back->scount : -1, pe.rcount);
          for (int k = 0; k < pe.rcount; ++k) {
            const int ra = parts[i].second[s].recv_rows[pe.roff + k];
            const int sb = parts[j].second[s].send_rows[back->soff + k];
            CHECK(a.l2g[Ha.perm[ra]] == b.l2g[Hb.perm[sb]], "halo row %d: global %lld != %lld", k,
                  (long long)a.l2g[Ha.perm[ra]], (long long)b.l2g[Hb.perm[sb]]);
          }
        }
    }
    std::printf("{\"group\": %lld, \"parts\": %zu, \"exchange\": \"consistent\"}\n", (long long)gid, parts.size());
  }
  return 0;
}
