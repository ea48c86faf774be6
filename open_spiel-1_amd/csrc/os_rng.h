// Bit-exact random-number consumption of the reference MCTS path, for host and
// gfx950:
//   * std::mt19937 streams (mcts.h:105 evaluator rng_, mcts.h:205 bot rng_),
//     seeded with init_genrand (== numpy RandomState legacy seeding);
//   * absl::Uniform(rng_, 0u, actions.size())    (mcts.cc:53)   -> AbslUniform
//   * std::shuffle(legal_actions, rng_), libstdc++ 11 (mcts.cc:275) -> CppShuffle
//   * numpy RandomState.choice / .shuffle (python/algorithms/mcts.py:69, :320)
//
// The MT19937 state (624 words) lives in caller memory (HBM arena on the
// device, a plain array on the host).  Twisting is done lazily, one word at a
// time, in place: producing word i of a new block needs old s[i], old s[i+1]
// and s[(i+397) mod 624], which is new exactly when the standard generator
// uses the new value, so the output sequence is identical to std::mt19937.
#ifndef OS_RNG_H_
#define OS_RNG_H_

#include "os_common.h"

namespace osm {

constexpr int kMtN = 624;
constexpr int kMtM = 397;

OS_HD void mt_seed(uint32_t* s, uint32_t seed) {
  s[0] = seed;
  for (int i = 1; i < kMtN; ++i)
    s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + static_cast<uint32_t>(i);
}

// A 32-bit MT19937 stream over externally owned state.
struct MtStream {
  uint32_t* s;
  int idx;  // next word index within the current block; kMtN => new block
  int pre;  // 1: the current block is already fully twisted (numpy import)
  uint32_t words;  // words drawn (instrumentation for algorithmic bytes)

  OS_HD uint32_t next() {
    ++words;
    if (idx >= kMtN) {
      idx = 0;
      pre = 0;
    }
    const int i = idx;
    if (pre) {
      idx = i + 1;
      return temper(s[i]);
    }
    const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
    const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
    uint32_t y = (s[i] & 0x80000000u) | (s[i1] & 0x7fffffffu);
    uint32_t v = s[im] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    s[i] = v;
    idx = i + 1;
    return temper(v);
  }
  OS_HD static uint32_t temper(uint32_t v) {
    v ^= v >> 11;
    v ^= (v << 7) & 0x9d2c5680u;
    v ^= (v << 15) & 0xefc60000u;
    v ^= v >> 18;
    return v;
  }
  // Brings the state to numpy's (key, pos) form: the whole current block
  // twisted, `idx` words of it consumed.
  OS_HD void finalize() {
    if (pre || idx >= kMtN) return;
    for (int i = idx; i < kMtN; ++i) {
      const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
      const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
      const uint32_t y = (s[i] & 0x80000000u) | (s[i1] & 0x7fffffffu);
      s[i] = s[im] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    pre = 1;
  }
};

// The same stream over a structure-of-arrays batch: word i of this stream at
// s[i * stride] (stride = streams in the batch), so lanes that draw in
// lockstep read and write one contiguous line per word.  No numpy import.
//
// The seeded state is never stored.  During the first block, word i of the
// twist reads seeded words i, i+1 and i+397, all in increasing order, so two
// running cursors of the init_genrand recurrence supply them (`lo0`/`lo1` =
// x_i / x_{i+1}, `hi` = x_{i+397}); only the twisted words are written (for
// i+397 >= 624 and for the later blocks, which read them back).  The output is
// std::mt19937's, and a playout writes 4 B per word drawn instead of the
// 2.5 KB seed.
struct MtStreamSoA {
  uint32_t* s;
  int64_t stride;
  int idx;
  uint32_t words;
  int blk0;  // 1 while the first block is being drawn
  uint32_t lo0, lo1, hi;

  OS_HD static uint32_t seed_step(uint32_t x, int k) {
    return 1812433253u * (x ^ (x >> 30)) + static_cast<uint32_t>(k);
  }
  OS_HD uint32_t& at(int i) const { return s[static_cast<int64_t>(i) * stride]; }
  OS_HD void seed(uint32_t v) {
    lo0 = v;
    lo1 = seed_step(v, 1);
    uint32_t x = lo1;
    for (int k = 2; k <= kMtM; ++k) x = seed_step(x, k);
    hi = x;
    idx = 0;
    blk0 = 1;
    words = 0;
  }
  OS_HD uint32_t next() {
    ++words;
    if (blk0) {
      const int i = idx;
      const uint32_t b = (i + 1 == kMtN) ? at(0) : lo1;
      const uint32_t m = (i + kMtM < kMtN) ? hi : at(i + kMtM - kMtN);
      const uint32_t y = (lo0 & 0x80000000u) | (b & 0x7fffffffu);
      const uint32_t v = m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      at(i) = v;
      lo0 = lo1;
      lo1 = seed_step(lo1, i + 2);
      hi = seed_step(hi, i + kMtM + 1);
      idx = i + 1;
      if (idx == kMtN) blk0 = 0;
      return MtStream::temper(v);
    }
    if (idx >= kMtN) idx = 0;
    const int i = idx;
    const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
    const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
    const uint32_t y = (at(i) & 0x80000000u) | (at(i1) & 0x7fffffffu);
    const uint32_t v = at(im) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    at(i) = v;
    idx = i + 1;
    return MtStream::temper(v);
  }
};

// MtStreamSoA whose first block never touches memory: std::mt19937's word
// t_i of block 0 is y(x_i, x_{i+1}) ^ x_{i+397} for i < 227 and
// y(x_i, x_{i+1}) ^ t_{i-227} for i >= 227, where x are the init_genrand
// words -- so every t_i is a function of x alone: for 227 <= i < 454,
// t_{i-227} = y(x_{i-227}, x_{i-226}) ^ x_{i+170}; for i >= 454 one level
// more, t_{i-227} = y(x_{i-227}, x_{i-226}) ^ y(x_{i-454}, x_{i-453}) ^ x_{i-57}.
// Running cursors over x give every word of the block without storing or
// reading one.  Word 623 reads the new t_0.  Only a stream that leaves block 0
// (> 624 words: a go9 random playout draws ~230) writes block 0 out, from the
// seed, and continues in memory as MtStreamSoA does.
struct MtStreamReg {
  uint32_t* s;
  int64_t stride;
  int idx;
  uint32_t words;
  int blk0;
  uint32_t seed0;
  uint32_t lo0, lo1, hi;   // x_i, x_{i+1}, x_{i+397} (i < 227)
  uint32_t lag0, lag1, mid;  // x_{i-227}, x_{i-226}, x_{i+170} (i >= 227)
  uint32_t lg0, lg1, far;    // x_{i-454}, x_{i-453}, x_{i-57} (i >= 454)
  uint32_t x397;            // x_397 (mid's and far's start)

  OS_HD uint32_t& at(int i) const { return s[static_cast<int64_t>(i) * stride]; }
  OS_HD static uint32_t mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  OS_HD void seed(uint32_t v) {
    seed0 = v;
    lo0 = v;
    lo1 = MtStreamSoA::seed_step(v, 1);
    uint32_t x = lo1;
    for (int k = 2; k <= kMtM; ++k) x = MtStreamSoA::seed_step(x, k);
    hi = x;
    x397 = x;
    lag0 = lag1 = mid = 0;
    lg0 = lg1 = far = 0;
    idx = 0;
    blk0 = 1;
    words = 0;
  }
  // Leaves block 0: writes its 624 words (recomputed from the seed) for the
  // in-memory twist of block 1.
  OS_HD void spill_block0() {
    uint32_t a = seed0, b = MtStreamSoA::seed_step(seed0, 1), h = x397;
    for (int i = 0; i < kMtN; ++i) {
      const uint32_t bb = (i + 1 == kMtN) ? at(0) : b;
      const uint32_t m = (i + kMtM < kMtN) ? h : at(i + kMtM - kMtN);
      at(i) = m ^ mix(a, bb);
      a = b;
      b = MtStreamSoA::seed_step(b, i + 2);
      h = MtStreamSoA::seed_step(h, i + kMtM + 1);
    }
    blk0 = 0;
  }
  OS_HD uint32_t next() {
    ++words;
    if (blk0) {
      const int i = idx;
      if (i < kMtN) {
        uint32_t v;
        if (i < kMtN - kMtM) {  // i < 227
          v = hi ^ mix(lo0, lo1);
          hi = MtStreamSoA::seed_step(hi, i + kMtM + 1);
          if (i + 1 == kMtN - kMtM) {  // the second form starts at 227
            lag0 = seed0;
            lag1 = MtStreamSoA::seed_step(seed0, 1);
            mid = x397;
          }
        } else {
          constexpr int kL = kMtN - kMtM;  // 227
          uint32_t t;                      // t_{i-227}
          if (i < 2 * kL) {
            t = mid ^ mix(lag0, lag1);
            mid = MtStreamSoA::seed_step(mid, i + kMtM - kL + 1);  // x_{i+171}
            if (i + 1 == 2 * kL) {
              lg0 = seed0;
              lg1 = MtStreamSoA::seed_step(seed0, 1);
              far = x397;
            }
          } else {
            t = far ^ mix(lg0, lg1) ^ mix(lag0, lag1);
            lg0 = lg1;
            lg1 = MtStreamSoA::seed_step(lg1, i - 2 * kL + 2);        // x_{i-452}
            far = MtStreamSoA::seed_step(far, i + kMtM - 2 * kL + 1);  // x_{i-56}
          }
          const uint32_t b = (i + 1 == kMtN)
                                 ? x397 ^ mix(seed0, MtStreamSoA::seed_step(seed0, 1))  // new t_0
                                 : lo1;
          v = t ^ mix(lo0, b);
          lag0 = lag1;
          lag1 = MtStreamSoA::seed_step(lag1, i - kL + 2);  // x_{i-225}
        }
        lo0 = lo1;
        lo1 = MtStreamSoA::seed_step(lo1, i + 2);
        idx = i + 1;
        return MtStream::temper(v);
      }
      spill_block0();
      idx = kMtN;
    }
    if (idx >= kMtN) idx = 0;
    const int i = idx;
    const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
    const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
    const uint32_t y = (at(i) & 0x80000000u) | (at(i1) & 0x7fffffffu);
    const uint32_t v = at(im) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    at(i) = v;
    idx = i + 1;
    return MtStream::temper(v);
  }
};

// MtStreamSoA with the next word's twist inputs read ahead: after word i is
// produced, s[i+2] and s[(i+1+397) % 624] are loaded (s[i+1] is already held),
// so the loads of a draw are in flight while the caller works between draws
// instead of stalling it.  The in-place twist order is unchanged: word i reads
// s[(i+397) % 624] after it was rewritten this pass (i >= 227) and, for
// i = 623, s[0] after word 0 of this pass -- each read is issued after the
// store it must see, from the same lane.  Same words as std::mt19937.
struct MtStreamPf {
  uint32_t* s;
  int64_t stride;
  int idx;
  uint32_t words;
  int blk0;  // 1 while the first block is being drawn (MtStreamSoA cursors)
  uint32_t lo0, lo1, hi;
  uint32_t a_i, a_i1, a_im;  // s[idx], s[idx + 1], s[idx + 397] (mod 624), read ahead
  int pre;   // 1: s holds a fully twisted block (numpy import), words idx.. unread

  OS_HD uint32_t& at(int i) const { return s[static_cast<int64_t>(i) * stride]; }
  OS_HD void seed(uint32_t v) {
    lo0 = v;
    lo1 = MtStreamSoA::seed_step(v, 1);
    uint32_t x = lo1;
    for (int k = 2; k <= kMtM; ++k) x = MtStreamSoA::seed_step(x, k);
    hi = x;
    idx = 0;
    blk0 = 1;
    words = 0;
    a_i = a_i1 = a_im = 0;
    pre = 0;
  }
  // numpy legacy (key, p): s holds the twisted block key, p words consumed.
  OS_HD void init_import(int p) {
    blk0 = 0;
    pre = 1;
    idx = p;
    words = 0;
    a_i = a_i1 = a_im = 0;
  }
  OS_HD void prefetch0() {  // the twist of a new block starts at word 0
    a_i = at(0);
    a_i1 = at(1);
    a_im = at(kMtM);
  }
  // Back to numpy's (key, pos) form: returns pos; the rest of a block being
  // twisted is twisted in place (MtStream::finalize).
  OS_HD int finalize() {
    if (pre) return idx;
    if (blk0 || idx == 0) return blk0 ? idx : kMtN;  // idx 0: the last block is used up
    for (int i = idx; i < kMtN; ++i) {
      const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
      const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
      const uint32_t y = (at(i) & 0x80000000u) | (at(i1) & 0x7fffffffu);
      at(i) = at(im) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    return idx;
  }
  OS_HD uint32_t next() {
    ++words;
    if (pre) {
      if (idx < kMtN) return MtStream::temper(at(idx++));
      pre = 0;  // the imported block is used up: twist the next one
      idx = 0;
      prefetch0();
    }
    const int i = idx;
    uint32_t v;
    if (blk0) {
      const uint32_t b = (i + 1 == kMtN) ? at(0) : lo1;
      const uint32_t m = (i + kMtM < kMtN) ? hi : at(i + kMtM - kMtN);
      const uint32_t y = (lo0 & 0x80000000u) | (b & 0x7fffffffu);
      v = m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      at(i) = v;
      lo0 = lo1;
      lo1 = MtStreamSoA::seed_step(lo1, i + 2);
      hi = MtStreamSoA::seed_step(hi, i + kMtM + 1);
      if (i + 1 == kMtN) {  // block 1 reads the stored block 0
        blk0 = 0;
        prefetch0();
      }
    } else {
      const uint32_t y = (a_i & 0x80000000u) | (a_i1 & 0x7fffffffu);
      v = a_im ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      at(i) = v;
      const int j = (i + 1 == kMtN) ? 0 : i + 1;  // the next word
      const int j1 = (j + 1 == kMtN) ? 0 : j + 1;
      const int jm = (j + kMtM >= kMtN) ? j + kMtM - kMtN : j + kMtM;
      a_i = a_i1;  // s[j]: not rewritten since it was read
      a_i1 = at(j1);
      a_im = at(jm);
    }
    idx = (i + 1 == kMtN) ? 0 : i + 1;
    return MtStream::temper(v);
  }
};

// MtStreamPf whose twisted words reach memory 16 at a time.  A lane of
// k_lsearch runs its own search, so its stream stores land one word at a time
// in lines the other 63 lanes never share; between two words of one lane the
// wave writes 63 other lines, and the L2 evicts partly written lines --
// written back as whole sectors (profiles/r04/g9_traffic: the streams were
// about 2/3 of the written lines).  Here each word goes to a 16-word buffer
// (wb, LDS, lane-interleaved: wb[k * wst]) and every 16th word writes the
// group out as four 16-byte stores (stride 1; 624 = 39 x 16, so a block ends on
// a full group).  Every word the twist reads back as "new" (s[i + 397 - 624],
// s[0] for i = 623, the next block's read-ahead) lies in an earlier, already
// stored group, and the "old" words it reads (s[i + 1], s[i + 397] below 624)
// are not yet rewritten, so the stream is std::mt19937's word for word.
struct MtStreamWc : MtStreamPf {
  uint32_t* wb;
  int wst;

  OS_HD void flush(int c, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (n == 16 && stride == 1) {
      uint4* d = reinterpret_cast<uint4*>(s + c);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = make_uint4(wb[(4 * q) * wst], wb[(4 * q + 1) * wst], wb[(4 * q + 2) * wst],
                          wb[(4 * q + 3) * wst]);
      return;
    }
#endif
    for (int k = 0; k < n; ++k) at(c + k) = wb[k * wst];
  }
  OS_HD void put(int i, uint32_t v) {
    wb[(i & 15) * wst] = v;
    if ((i & 15) == 15) flush(i - 15, 16);
  }
  OS_HD int finalize() {
    if (pre) return idx;
    if (blk0 || idx == 0) {
      if (blk0 && (idx & 15)) flush(idx & ~15, idx & 15);  // the block-0 words drawn so far
      return blk0 ? idx : kMtN;
    }
    if (idx & 15) flush(idx & ~15, idx & 15);  // the group being filled
    return MtStreamPf::finalize();
  }
  OS_HD uint32_t next() {
    ++words;
    if (pre) {
      if (idx < kMtN) return MtStream::temper(at(idx++));
      pre = 0;
      idx = 0;
      prefetch0();
    }
    const int i = idx;
    uint32_t v;
    if (blk0) {
      const uint32_t b = (i + 1 == kMtN) ? at(0) : lo1;
      const uint32_t m = (i + kMtM < kMtN) ? hi : at(i + kMtM - kMtN);
      const uint32_t y = (lo0 & 0x80000000u) | (b & 0x7fffffffu);
      v = m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      put(i, v);
      lo0 = lo1;
      lo1 = MtStreamSoA::seed_step(lo1, i + 2);
      hi = MtStreamSoA::seed_step(hi, i + kMtM + 1);
      if (i + 1 == kMtN) {
        blk0 = 0;
        prefetch0();
      }
    } else {
      const uint32_t y = (a_i & 0x80000000u) | (a_i1 & 0x7fffffffu);
      v = a_im ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      put(i, v);
      const int j = (i + 1 == kMtN) ? 0 : i + 1;
      const int j1 = (j + 1 == kMtN) ? 0 : j + 1;
      const int jm = (j + kMtM >= kMtN) ? j + kMtM - kMtN : j + kMtM;
      a_i = a_i1;
      a_i1 = at(j1);
      a_im = at(jm);
    }
    idx = (i + 1 == kMtN) ? 0 : i + 1;
    return MtStream::temper(v);
  }
};

OS_HD uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return static_cast<uint64_t>((static_cast<unsigned __int128>(a) * b) >> 64);
#endif
}

// absl::Uniform(g, 0u, n) for a 32-bit URBG with a 64-bit result type
// (abseil 20200225 uniform_int_distribution<uint64>::Generate over
// FastUniformBits<uint64>: two words, first in the high half; Lemire 64x64
// with rejection).  n >= 1.
template <class G>
OS_HD uint32_t AbslUniform(G& g, uint32_t n) {
  uint64_t hi = g.next();
  uint64_t lo = g.next();
  if ((n & (n - 1u)) == 0) return static_cast<uint32_t>(lo) & (n - 1u);  // 2^k: low bits
  // bits * n with bits = hi:lo and n < 2^32, in 32x32->64 pieces:
  //   P = (hi*n << 32) + lo*n;  P >> 64 = (hi*n + (lo*n >> 32)) >> 32 (no overflow);
  //   P mod 2^64 = low32(mid):low32(lo*n) with mid = hi*n + (lo*n >> 32).
  const uint64_t b = lo * n;
  const uint64_t mid = hi * n + (b >> 32);
  if (static_cast<uint32_t>(mid) != 0 || static_cast<uint32_t>(b) >= n)
    return static_cast<uint32_t>(mid >> 32);  // P mod 2^64 >= n: no rejection test
  uint64_t bits = (hi << 32) | lo;
  uint64_t plo = bits * n;
  uint64_t phi = umulhi64(bits, n);
  {
    const uint64_t thr = (0ull - static_cast<uint64_t>(n)) % n;
    while (plo < thr) {
      hi = g.next();
      lo = g.next();
      bits = (hi << 32) | lo;
      plo = bits * n;
      phi = umulhi64(bits, n);
    }
  }
  return static_cast<uint32_t>(phi);
}

// libstdc++ uniform_int_distribution downscaling (_S_nd, Lemire 32x32->64).
template <class G>
OS_HD uint32_t Lemire32(G& g, uint32_t m) {
  uint64_t p = static_cast<uint64_t>(g.next()) * m;
  uint32_t low = static_cast<uint32_t>(p);
  if (low < m) {
    const uint32_t thr = (0u - m) % m;
    while (low < thr) {
      p = static_cast<uint64_t>(g.next()) * m;
      low = static_cast<uint32_t>(p);
    }
  }
  return static_cast<uint32_t>(p >> 32);
}

// std::shuffle from libstdc++ 11 (bits/stl_algo.h, "pair" path valid for
// n <= 65535 with a 32-bit URBG).  A is a pointer or an indexable view
// (StridedPtr) of any swappable element type.
template <class A, class G>
OS_HD void CppShuffle(A a, int n, G& g) {
  if (n <= 1) return;
  int i = 1;
  if ((n & 1) == 0) {
    uint32_t j = Lemire32(g, 2u);
    auto t = a[1]; a[1] = a[j]; a[j] = t;
    i = 2;
  }
  while (i != n) {
    const uint32_t b0 = static_cast<uint32_t>(i) + 1u;
    const uint32_t b1 = b0 + 1u;
    const uint32_t x = Lemire32(g, b0 * b1);
    const uint32_t p0 = x / b1, p1 = x % b1;
    auto t = a[i]; a[i] = a[p0]; a[p0] = t;
    t = a[i + 1]; a[i + 1] = a[p1]; a[p1] = t;
    i += 2;
  }
}

// absl::Uniform(g, 0.0, 1.0) (spiel.cc:339, SampleAction): abseil 20200225
// uniform_real_distribution<double> over FastUniformBits<uint64> (two words,
// first high, as AbslUniform) through GenerateRealFromBits<double,
// GeneratePositiveTag, true>: the leading zeros set the exponent, the 52 bits
// after the leading one the mantissa.  Pure integer work, so bit-exact on the
// device.
template <class G>
OS_HD double AbslUniformDouble01(G& g) {
  const uint64_t hi = g.next();
  uint64_t bits = (hi << 32) | g.next();
  if (bits == 0) return 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
  const int clz = __clzll(static_cast<long long>(bits));
#else
  const int clz = __builtin_clzll(bits);
#endif
  bits <<= clz;
  const uint64_t val = (static_cast<uint64_t>(1022 - clz) << 52) |
                       ((bits >> 11) & ((1ull << 52) - 1));  // leading one -> bit 52
  double d;
  __builtin_memcpy(&d, &val, 8);
  return d;
}

// numpy legacy RandomState.random_sample(): (a >> 5, b >> 6) -> 53 bits.
template <class G>
OS_HD double NpRandomSample(G& g) {
  const uint32_t a = g.next() >> 5;
  const uint32_t b = g.next() >> 6;
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// spiel.cc:341-366 SampleAction(outcomes, z) over n equiprobable outcomes
// (probability p each, accumulated in order): index of the first outcome with
// sum <= z < sum + p.  The reference's fall-through is a fatal error (z is
// never that close to 1); the last index stands in for it.
OS_HD int SampleEquiprobable(int n, double p, double z) {
  double sum = 0.0;
  for (int k = 0; k < n; ++k) {
    if (sum <= z && z < sum + p) return k;
    sum += p;
  }
  return n - 1;
}

// numpy legacy RandomState.choice(n outcomes, p=[p] * n) index (replace=True,
// size=None): cdf = p.cumsum(); cdf /= cdf[-1]; searchsorted(random_sample(),
// side='right') == the number of cdf entries <= u.
template <class G>
OS_HD int NpChoiceEquiprobable(G& g, int n, double p) {
  double acc = 0.0, last = 0.0;
  for (int k = 0; k < n; ++k) last = acc = acc + p;
  const double u = NpRandomSample(g);
  int idx = 0;
  acc = 0.0;
  for (int k = 0; k < n; ++k) {
    acc = acc + p;
    idx += (acc / last <= u) ? 1 : 0;
  }
  return idx;
}

OS_HD uint32_t np_mask(uint32_t m) {
  m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
  return m;
}

// numpy legacy random_interval(max) (32-bit masked rejection).
template <class G>
OS_HD uint32_t NpRandomInterval(G& g, uint32_t max) {
  if (max == 0) return 0;
  const uint32_t mask = np_mask(max);
  uint32_t v;
  do { v = g.next() & mask; } while (v > max);
  return v;
}

// numpy legacy RandomState.choice(seq of n) -> index (no draw when n == 1).
template <class G>
OS_HD uint32_t NpChoice(G& g, uint32_t n) {
  const uint32_t rng = n - 1;
  if (rng == 0) return 0;
  const uint32_t mask = np_mask(rng);
  uint32_t v;
  do { v = g.next() & mask; } while (v > rng);
  return v;
}

// numpy RandomState.shuffle(list): Fisher-Yates from the end.
template <class A, class G>
OS_HD void NpShuffle(A a, int n, G& g) {
  for (int i = n - 1; i >= 1; --i) {
    uint32_t j = NpRandomInterval(g, static_cast<uint32_t>(i));
    auto t = a[i]; a[i] = a[j]; a[j] = t;
  }
}

}  // namespace osm

#endif  // OS_RNG_H_
