// host_math.cpp — see host_math.h.
#include "host_math.h"

#include <cmath>

namespace bcsim {

int64_t seconds_to_ns(double s, uint32_t time_round) {
  if (s == 0.0) return 0;
  const bool neg = s < 0;
  const double v = neg ? -s : s;
  int e = 0;
  const double m = std::frexp(v, &e);                 // v = m * 2^e
  const uint64_t mant = static_cast<uint64_t>(std::ldexp(m, 53));
  const int shift = (e - 53) + 64;                    // v * 2^64 = mant * 2^shift
  unsigned __int128 fixed;                            // Q64.64, truncated
  if (shift >= 0) {
    fixed = static_cast<unsigned __int128>(mant) << shift;
  } else if (shift > -128) {
    fixed = static_cast<unsigned __int128>(mant) >> (-shift);
  } else {
    fixed = 0;
  }
  const uint64_t whole = static_cast<uint64_t>(fixed >> 64);
  const uint64_t frac = static_cast<uint64_t>(fixed);
  const unsigned __int128 fns = static_cast<unsigned __int128>(frac) * 1000000000ull;
  uint64_t ns = whole * 1000000000ull + static_cast<uint64_t>(fns >> 64);
  const uint64_t rem = static_cast<uint64_t>(fns);
  if (time_round == BCSIM_TIME_ROUND && (rem >> 63)) ++ns;
  return neg ? -static_cast<int64_t>(ns) : static_cast<int64_t>(ns);
}

int64_t frame_tx_ns(uint32_t wire_bytes, uint64_t rate_bps, uint32_t time_round) {
  const double secs = static_cast<double>(wire_bytes) * 8 / static_cast<double>(rate_bps);
  return seconds_to_ns(secs, time_round);
}

MsgTx message_tx(uint32_t payload, uint32_t mtu, uint64_t rate_bps,
                 uint32_t time_round) {
  MsgTx r{0, 0, 0, 0};
  const uint32_t ip_payload = payload + 8;     // UDP header
  const uint32_t room = mtu - 20;              // IPv4 header
  if (ip_payload <= room) {
    r.wire = ip_payload + 22;
    r.last = frame_tx_ns(r.wire, rate_bps, time_round);
    r.total = r.last;
    r.frames = 1;
    return r;
  }
  const uint32_t frag = room & ~7u;            // fragment offsets are 8-byte units
  for (uint32_t left = ip_payload; left > 0;) {
    const uint32_t p = left > frag ? frag : left;
    const uint32_t w = p + 22;
    r.last = frame_tx_ns(w, rate_bps, time_round);
    r.total += r.last;
    r.wire += w;
    ++r.frames;
    left -= p;
  }
  return r;
}

std::vector<int32_t> glibc_stream(uint32_t seed, size_t n) {
  // state ring of 31 words; front index starts 3 ahead of the rear index
  int32_t ring[31];
  int32_t w = static_cast<int32_t>(seed == 0 ? 1u : seed);
  ring[0] = w;
  for (int i = 1; i < 31; ++i) {
    const long hi = w / 127773, lo = w % 127773;
    long nw = 16807 * lo - 2836 * hi;
    if (nw < 0) nw += 2147483647;
    w = static_cast<int32_t>(nw);
    ring[i] = w;
  }
  int front = 3, rear = 0;
  auto step = [&]() -> int32_t {
    const uint32_t sum = static_cast<uint32_t>(ring[front]) + static_cast<uint32_t>(ring[rear]);
    ring[front] = static_cast<int32_t>(sum);
    front = (front + 1) % 31;
    rear = (rear + 1) % 31;
    return static_cast<int32_t>(sum >> 1);
  };
  for (int k = 0; k < 310; ++k) step();
  std::vector<int32_t> out(n);
  for (size_t k = 0; k < n; ++k) out[k] = step();
  return out;
}

// MurmurHash3_x86_32 (public algorithm; ns-3 Hash32 = Murmur3 with seed 0x8BADF00D)
static uint32_t murmur3(const uint8_t* d, uint32_t len, uint32_t h) {
  auto rot = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t i = 0;
  for (; i + 4 <= len; i += 4) {
    uint32_t k = d[i] | (d[i + 1] << 8) | (d[i + 2] << 16) | (static_cast<uint32_t>(d[i + 3]) << 24);
    h ^= rot(k * c1, 15) * c2;
    h = rot(h, 13) * 5 + 0xe6546b64u;
  }
  uint32_t k = 0;
  for (uint32_t j = len & 3; j > 0; --j) k |= static_cast<uint32_t>(d[i + j - 1]) << (8 * (j - 1));
  if (len & 3) h ^= rot(k * c1, 15) * c2;
  h ^= len;
  h = (h ^ (h >> 16)) * 0x85ebca6bu;
  h = (h ^ (h >> 13)) * 0xc2b2ae35u;
  return h ^ (h >> 16);
}

std::vector<uint8_t> fq_flow_map(uint32_t N, const std::vector<uint32_t>& row, const std::vector<uint32_t>& col,
                                 const std::vector<uint32_t>& rev, uint32_t protocol, uint32_t flows,
                                 uint32_t perturbation) {
  const uint32_t E = row[N];
  std::vector<uint32_t> link(E), src(E);
  uint32_t k = 0;  // the mesh loop's link order (blockchain-simulator.cc:34-51): larger endpoint, then smaller
  for (uint32_t a = 0; a < N; ++a)
    for (uint32_t e = row[a]; e < row[a + 1]; ++e) {
      src[e] = a;
      if (col[e] < a) link[e] = link[rev[e]] = k++;
    }
  // client socket k of a node takes ephemeral port 49153 + k, sockets in peer order; Paxos's
  // socket k serves peer k + 1 and peer 0 gets a later one (paxos-node.cc:110-119)
  auto port = [&](uint32_t node, uint32_t idx) -> uint32_t {
    const uint32_t deg = row[node + 1] - row[node];
    if (protocol == BCSIM_PAXOS) return idx ? 49152 + idx : 49153 + deg;
    return 49153 + idx;
  };
  auto flow = [&](uint32_t s, uint32_t d, uint32_t sp, uint32_t dp) {
    uint8_t b[17];
    const uint32_t w[5] = {s, d, 0, 0, perturbation};
    for (int j = 0; j < 4; ++j) {
      b[j] = static_cast<uint8_t>(w[0] >> (24 - 8 * j));
      b[4 + j] = static_cast<uint8_t>(w[1] >> (24 - 8 * j));
      b[13 + j] = static_cast<uint8_t>(w[4] >> (24 - 8 * j));
    }
    b[8] = 17;
    b[9] = static_cast<uint8_t>(sp >> 8);
    b[10] = static_cast<uint8_t>(sp);
    b[11] = static_cast<uint8_t>(dp >> 8);
    b[12] = static_cast<uint8_t>(dp);
    return murmur3(b, 17, 0x8BADF00Du) % flows;
  };
  std::vector<uint8_t> map(E);
  for (uint32_t e = 0; e < E; ++e) {
    const uint32_t s = src[e], d = col[e];
    const uint32_t net = 0x01000000u + (link[e] << 8);  // 1.0.0.0/24, NewNetwork per link
    const uint32_t ia = net + (s > d ? 1u : 2u), ib = net + (d > s ? 1u : 2u);  // node i of the loop is .1
    const uint32_t hA = flow(ia, ib, port(s, e - row[s]), 7071);
    const uint32_t hE = flow(ia, ib, 7071, port(d, rev[e] - row[d]));
    const uint32_t hF = flow(ia, ib, 0, 0);
    const uint32_t sE = hE == hA ? 0u : 1u;
    const uint32_t sF = hF == hA ? 0u : hF == hE ? sE : sE + 1u;
    map[e] = static_cast<uint8_t>(sE << 2 | sF << 4);
  }
  return map;
}

}  // namespace bcsim
