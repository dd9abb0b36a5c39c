// topology.cpp — host-side topology builders.
//
// The reference only builds the full mesh (blockchain-simulator.cc:34-51, one
// PointToPoint link per node pair, peers listed in ascending id order).  The
// gossip configuration of BASELINE configs[4] needs a random 8-regular graph,
// which this file generates deterministically from (n, d, seed) and hands out
// in the same CSR form bcsim_set_topology_csr takes: rows ascending, graph
// symmetric, no self-loops, no multi-edges.
#include <algorithm>
#include <cstdint>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/bcsim.h"

namespace {

struct SplitMix {
  uint64_t x;
  uint64_t next() {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return next() % n; }
};

inline uint64_t ekey(uint32_t a, uint32_t b) {
  if (a > b) std::swap(a, b);
  return (static_cast<uint64_t>(a) << 32) | b;
}

}  // namespace

extern "C" int bcsim_topology_random_regular(uint32_t n, uint32_t d, uint64_t seed, uint32_t* row_ptr,
                                             uint32_t* col_idx) {
  if (!row_ptr || !col_idx || n < 2 || d == 0 || d >= n || (static_cast<uint64_t>(n) * d) % 2) return BCSIM_E_INVAL;
  const uint64_t S = static_cast<uint64_t>(n) * d, M = S / 2;
  if (S > 0xffffffffull) return BCSIM_E_INVAL;
  SplitMix rng{seed ^ 0x6a09e667f3bcc909ull};
  // configuration model: every node owns d stubs; a seeded shuffle pairs them
  std::vector<uint32_t> stub(S);
  for (uint64_t k = 0; k < S; ++k) stub[k] = static_cast<uint32_t>(k / d);
  for (uint64_t k = S - 1; k > 0; --k) std::swap(stub[k], stub[rng.below(k + 1)]);
  std::vector<std::pair<uint32_t, uint32_t>> ed(M);
  std::unordered_map<uint64_t, uint32_t> mult;
  mult.reserve(M * 2);
  for (uint64_t m = 0; m < M; ++m) {
    ed[m] = {stub[2 * m], stub[2 * m + 1]};
    ++mult[ekey(ed[m].first, ed[m].second)];
  }
  auto bad = [&](uint64_t m) { return ed[m].first == ed[m].second || mult[ekey(ed[m].first, ed[m].second)] > 1; };
  auto ok_new = [&](uint32_t a, uint32_t b) {
    if (a == b) return false;
    auto it = mult.find(ekey(a, b));
    return it == mult.end() || it->second == 0;
  };
  // repair self-loops and multi-edges by random double-edge swaps (degree preserving)
  std::vector<uint64_t> todo;
  for (uint64_t m = 0; m < M; ++m)
    if (bad(m)) todo.push_back(m);
  uint64_t guard = 0;
  while (!todo.empty()) {
    if (++guard > 100ull * M + 1000000ull) return BCSIM_E_INVAL;
    const uint64_t m = todo.back();
    if (!bad(m)) {
      todo.pop_back();
      continue;
    }
    const uint64_t f = rng.below(M);
    if (f == m) continue;
    uint32_t a = ed[m].first, b = ed[m].second, c = ed[f].first, e = ed[f].second;
    if (rng.next() & 1) std::swap(c, e);
    if (!ok_new(a, c) || !ok_new(b, e) || ekey(a, c) == ekey(b, e)) continue;
    --mult[ekey(a, b)];
    --mult[ekey(ed[f].first, ed[f].second)];
    ed[m] = {a, c};
    ed[f] = {b, e};
    ++mult[ekey(a, c)];
    ++mult[ekey(b, e)];
    todo.pop_back();
  }
  // CSR, rows ascending (reference peer order)
  std::vector<std::vector<uint32_t>> adj(n);
  for (const auto& pr : ed) {
    adj[pr.first].push_back(pr.second);
    adj[pr.second].push_back(pr.first);
  }
  uint32_t k = 0;
  for (uint32_t i = 0; i < n; ++i) {
    row_ptr[i] = k;
    std::sort(adj[i].begin(), adj[i].end());
    for (uint32_t j : adj[i]) col_idx[k++] = j;
  }
  row_ptr[n] = k;
  return BCSIM_OK;
}
