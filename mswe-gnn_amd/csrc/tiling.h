// Host-side ordering of destinations for the edge tiles (plan.hip build_graph_plan).
// Header-only and free of HIP so that the CPU tests compile it with g++ (tests/test_host_cpu.py).
#pragma once
#include <algorithm>
#include <vector>

namespace msw {

constexpr int kTileEdges = 16;  // = kRowsPerWave: in-edges and destinations per edge tile

// Order of one graph's destinations inside its scale (the internal numbering) so that
// build_tiles' consecutive packing leaves fewer tiles: the graph order, except that a tile the
// next destination cannot fill exactly is topped up from the next kPackWindow destinations --
// a destination that fits when the next one overflows, or (when the remainder the next one
// would leave fits no destination in the window) one or two destinations that close the
// tile at exactly 16 in-edges.  Sums stay per destination in edge order and every row of a
// tile is computed on its own, so results do not depend on the order (bit-identical).
// zenodo4's finest scale: 2,050 -> 2,046 tiles (1,927 = all tiles full).
constexpr int kPackWindow = 64;
inline std::vector<int> pack_order(const std::vector<int>& deg) {
  const int n = (int)deg.size();
  std::vector<char> used(n, 0);
  std::vector<int> out;
  out.reserve(n);
  auto take = [&](int k) { used[k] = 1; out.push_back(k); };
  int head = 0;
  while (head < n) {
    int e = 0, cnt = 0, j = head;
    for (;;) {
      while (j < n && used[j]) ++j;
      if (j >= n || cnt >= kTileEdges) break;
      const int end = std::min(n, j + kPackWindow);
      if (e + deg[j] <= kTileEdges) {
        const int r = kTileEdges - e - deg[j];
        bool fillable = r == 0;
        for (int k = j + 1; k < end && !fillable; ++k) fillable = !used[k] && deg[k] <= r;
        if (!fillable) {  // exact fill of the current remainder with one or two window nodes
          const int R = kTileEdges - e;
          int first[kTileEdges + 1], second[kTileEdges + 1];
          std::fill(first, first + kTileEdges + 1, -1);
          std::fill(second, second + kTileEdges + 1, -1);
          for (int k = j; k < end; ++k) {
            if (used[k] || deg[k] > R) continue;
            if (first[deg[k]] < 0) first[deg[k]] = k;
            else if (second[deg[k]] < 0) second[deg[k]] = k;
          }
          int pa = -1, pb = -1;
          if (first[R] >= 0 && first[R] != j) pa = first[R];
          else if (second[R] >= 0) pa = second[R];
          for (int d = 0; pa < 0 && d <= R - d; ++d) {
            const int a = first[d], b = d == R - d ? second[d] : first[R - d];
            if (a >= 0 && b >= 0 && cnt + 2 <= kTileEdges) { pa = std::min(a, b); pb = std::max(a, b); }
          }
          if (pa >= 0) {
            take(pa);
            if (pb >= 0) take(pb);
            e = kTileEdges;
            cnt += pb >= 0 ? 2 : 1;
            continue;
          }
        }
        take(j);
        e += deg[j];
        ++cnt;
        ++j;
        continue;
      }
      if (cnt == 0) {  // more than 16 in-edges: alone (build_tiles reports it)
        take(j);
        break;
      }
      int best = -1;
      for (int k = j + 1; k < end && best < 0; ++k)
        if (!used[k] && e + deg[k] <= kTileEdges) best = k;
      if (best < 0) break;
      take(best);
      e += deg[best];
      ++cnt;
    }
    while (head < n && used[head]) ++head;
  }
  return out;
}

}  // namespace msw
