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
std::vector<uint32_t> fq_link_numbers(uint32_t N, const std::vector<uint32_t>& row, const std::vector<uint32_t>& col,
                                      const std::vector<uint32_t>& rev) {
  std::vector<uint32_t> link(row[N]);
  uint32_t k = 0;
  for (uint32_t a = 0; a < N; ++a)
    for (uint32_t e = row[a]; e < row[a + 1]; ++e)
      if (col[e] < a) link[e] = link[rev[e]] = k++;
  return link;
}

}  // namespace bcsim
