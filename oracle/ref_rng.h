// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product library.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// the library built from this directory, and only as the checker / CPU
// baseline, never as the thing measured or shipped.
//
// CPU restatement of the random-number consumption the reference MCTS path
// performs.  Third-party semantics restated here (not vendored in
// /root/reference):
//   * std::mt19937 / std::mt19937_64 and std::shuffle: used directly from the
//     container's libstdc++ 11 (g++ 11.4) -- the same library the reference's
//     open_spiel/algorithms/mcts.cc:275 call binds to on this toolchain.
//   * abseil 20200225.1 `absl::Uniform(rng_, 0u, actions.size())`
//     (mcts.cc:53): restated from abseil's published algorithm
//     (uniform_int_distribution::Generate + FastUniformBits).  The result type
//     is the common type of (unsigned, size_t) = uint64, so the URBG (32-bit
//     mt19937) is drawn twice per call, first draw in the high half, then
//     Lemire's multiply with rejection (64x64->128).  The 32-bit Lemire branch
//     of the same library is pinned by the reference playthrough
//     negotiation(rng_seed=100,...).txt; the two-word order
//     of the 64-bit path is PARITY UNPINNED by any reference fixture.
//   * numpy legacy RandomState (python/algorithms/mcts.py:69 `choice`,
//     :320 `shuffle`): numpy 2.2 `random_interval` / masked bounded uint32
//     restated (the container's numpy is used by tests as an independent check).
#ifndef OS_ORACLE_REF_RNG_H_
#define OS_ORACLE_REF_RNG_H_

#include <cstdint>
#include <random>
#include <vector>

namespace oref {

// absl::Uniform(g, 0u, n) with n:size_t, g: std::mt19937 (32-bit URBG).
// Returns a value in [0, n).  n must be >= 1.
inline uint64_t AbslUniformU64(std::mt19937& g, uint64_t n) {
  // FastUniformBits<uint64_t> over a 32-bit URBG: two draws, first is high.
  auto fast_bits = [&g]() -> uint64_t {
    uint64_t r = static_cast<uint64_t>(g());
    r = (r << 32) + static_cast<uint64_t>(g());
    return r;
  };
  const uint64_t R = n - 1;       // distribution param: [0, n-1]
  const uint64_t Lim = R + 1;     // == n
  uint64_t bits = fast_bits();
  if ((R & Lim) == 0) return bits & R;  // power of two range
  unsigned __int128 product = static_cast<unsigned __int128>(bits) * Lim;
  uint64_t lo = static_cast<uint64_t>(product);
  if (lo < Lim) {
    const uint64_t threshold = (~uint64_t{0} - Lim + 1) % Lim;
    while (lo < threshold) {
      bits = fast_bits();
      product = static_cast<unsigned __int128>(bits) * Lim;
      lo = static_cast<uint64_t>(product);
    }
  }
  return static_cast<uint64_t>(product >> 64);
}

// numpy legacy `random_interval(bitgen, max)` (mask-and-reject on 32-bit words
// when max <= 0xffffffff).  Used by RandomState.shuffle.
inline uint64_t NpRandomInterval(std::mt19937& g, uint64_t max) {
  if (max == 0) return 0;
  uint64_t mask = max;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
  mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  uint64_t value;
  while ((value = (static_cast<uint64_t>(g()) & mask)) > max) {}
  return value;
}

// numpy legacy RandomState.choice(seq) with replace=True, p=None:
// randint(0, n) -> masked bounded uint32 with rng = n - 1; no draw if n == 1.
inline uint64_t NpChoiceIndex(std::mt19937& g, uint64_t n) {
  const uint64_t rng = n - 1;
  if (rng == 0) return 0;
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
  mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  uint64_t value;
  while ((value = (static_cast<uint64_t>(g()) & mask)) > rng) {}
  return value;
}

// absl::Uniform(g, 0.0, 1.0) (spiel.cc:339, SampleAction): abseil 20200225
// uniform_real_distribution<double> = GenerateRealFromBits<double,
// GeneratePositiveTag, /*IncludeZero=*/true>(FastUniformBits<uint64>(g)):
// the leading-zero count of the 64 bits sets the exponent (2^-(clz+1)), the 52
// bits after the leading one the mantissa (value in [0, 1)); then
// a + sample * (b - a) = sample.  The
// 64-bit word order is the one of AbslUniformU64 (parity unpinned, as there).
inline double AbslUniformDouble01(std::mt19937& g) {
  uint64_t bits = static_cast<uint64_t>(g());
  bits = (bits << 32) + static_cast<uint64_t>(g());
  if (bits == 0) return 0.0;
  const int clz = __builtin_clzll(bits);
  bits <<= clz;
  const uint64_t exp = static_cast<uint64_t>(1022 - clz);
  bits >>= 11;  // 63 - kExp: the leading one lands on the implicit bit 52
  const uint64_t val = (exp << 52) | (bits & ((uint64_t{1} << 52) - 1));
  double d;
  __builtin_memcpy(&d, &val, 8);
  return 0.0 + d * (1.0 - 0.0);
}

// numpy legacy RandomState.random_sample(): 53 bits from two words.
inline double NpRandomSample(std::mt19937& g) {
  const uint32_t a = static_cast<uint32_t>(g()) >> 5, b = static_cast<uint32_t>(g()) >> 6;
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// numpy legacy RandomState.choice(a, p=p) index (replace=True, size=None):
// cdf = p.cumsum(); cdf /= cdf[-1]; cdf.searchsorted(random_sample(),
// side='right').
inline size_t NpChoiceP(std::mt19937& g, const std::vector<double>& p) {
  std::vector<double> cdf(p.size());
  double acc = 0.0;
  for (size_t i = 0; i < p.size(); ++i) cdf[i] = acc = acc + p[i];
  const double last = cdf.back();
  for (double& c : cdf) c /= last;
  const double u = NpRandomSample(g);
  size_t k = 0;
  while (k < cdf.size() && cdf[k] <= u) ++k;
  return k;
}

}  // namespace oref

#endif  // OS_ORACLE_REF_RNG_H_
