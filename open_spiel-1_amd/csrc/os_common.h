// Common host/device helpers for the MI355X MCTS engine.
//
// Everything in csrc/*.h compiles both for the host (hipcc host pass / g++)
// and for gfx950; the same game state machines back the host State API and
// the device search kernel, so there is one implementation of each rule set.
#ifndef OS_COMMON_H_
#define OS_COMMON_H_

#include <stdint.h>
#include <type_traits>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define OS_HD __host__ __device__ __forceinline__
#define OS_HDNI __host__ __device__
#else
#define OS_HD inline
#define OS_HDNI
#endif

namespace osm {

OS_HD int popc64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(x);
#else
  return __builtin_popcountll(x);
#endif
}

OS_HD int ctz64(uint64_t x) {  // x != 0
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffsll(static_cast<unsigned long long>(x)) - 1;
#else
  return __builtin_ctzll(x);
#endif
}

// Index of the k-th (0-based) set bit of x, ascending.  Requires k < popc(x).
OS_HD int select64(uint64_t x, int k) {
  // Binary search on popcounts of the low half (6 steps, branch-light).
  int base = 0;
  int c = popc64(x & 0xFFFFFFFFull);
  if (k >= c) { k -= c; x >>= 32; base += 32; }
  c = popc64(x & 0xFFFFull);
  if (k >= c) { k -= c; x >>= 16; base += 16; }
  c = popc64(x & 0xFFull);
  if (k >= c) { k -= c; x >>= 8; base += 8; }
  c = popc64(x & 0xFull);
  if (k >= c) { k -= c; x >>= 4; base += 4; }
  c = popc64(x & 0x3ull);
  if (k >= c) { k -= c; x >>= 2; base += 2; }
  c = static_cast<int>(x & 1ull);
  if (k >= c) { base += 1; }
  return base;
}

// Player-indexed pairs without dynamic indexing: a[p] with a runtime p would
// force the whole state into private (scratch) memory on the GPU; selects keep
// it in registers (SGPRs when the player is wave-uniform).
template <class T>
OS_HD T pick(const T* a, int i) {
  return i ? a[1] : a[0];
}
template <class T>
OS_HD void put(T* a, int i, T v) {
  const T v0 = i ? a[0] : v;
  const T v1 = i ? v : a[1];
  a[0] = v0;
  a[1] = v1;
}

// 128-bit bitboard (two u64 words).  Bit i = cell i.
struct B128 {
  uint64_t lo, hi;
};
OS_HD B128 b128(uint64_t lo, uint64_t hi) { B128 r; r.lo = lo; r.hi = hi; return r; }
// Selects on B128 go word by word: a conditional of class type is emitted as
// a select of the two operands' ADDRESSES, which pins both in scratch.
OS_HD B128 sel128(bool c, B128 x, B128 y) {
  const uint64_t lo = c ? x.lo : y.lo;
  const uint64_t hi = c ? x.hi : y.hi;
  return b128(lo, hi);
}
OS_HD B128 pick(const B128* a, int i) {
  const uint64_t l0 = a[0].lo, h0 = a[0].hi, l1 = a[1].lo, h1 = a[1].hi;
  return b128(i ? l1 : l0, i ? h1 : h0);
}
OS_HD void put(B128* a, int i, B128 v) {
  const uint64_t l0 = a[0].lo, h0 = a[0].hi, l1 = a[1].lo, h1 = a[1].hi;
  a[0] = b128(i ? l0 : v.lo, i ? h0 : v.hi);
  a[1] = b128(i ? v.lo : l1, i ? v.hi : h1);
}
OS_HD B128 operator|(B128 a, B128 b) { return b128(a.lo | b.lo, a.hi | b.hi); }
OS_HD B128 operator&(B128 a, B128 b) { return b128(a.lo & b.lo, a.hi & b.hi); }
OS_HD B128 operator^(B128 a, B128 b) { return b128(a.lo ^ b.lo, a.hi ^ b.hi); }
OS_HD B128 operator~(B128 a) { return b128(~a.lo, ~a.hi); }
OS_HD bool operator==(B128 a, B128 b) { return a.lo == b.lo && a.hi == b.hi; }
OS_HD bool operator!=(B128 a, B128 b) { return !(a == b); }
OS_HD bool any(B128 a) { return (a.lo | a.hi) != 0; }
OS_HD int popc(B128 a) { return popc64(a.lo) + popc64(a.hi); }
OS_HD B128 shl(B128 a, int s) {  // 0 < s < 64
  return b128(a.lo << s, (a.hi << s) | (a.lo >> (64 - s)));
}
OS_HD B128 shr(B128 a, int s) {  // 0 < s < 64
  return b128((a.lo >> s) | (a.hi << (64 - s)), a.hi >> s);
}
OS_HD B128 bit128(int i) {
  return i < 64 ? b128(1ull << i, 0) : b128(0, 1ull << (i - 64));
}
OS_HD bool test(B128 a, int i) {
  return i < 64 ? ((a.lo >> i) & 1) : ((a.hi >> (i - 64)) & 1);
}
OS_HD int lowest(B128 a) {  // a != 0
  return a.lo ? ctz64(a.lo) : 64 + ctz64(a.hi);
}
OS_HD int select128(B128 a, int k) {
  int c = popc64(a.lo);
  return k < c ? select64(a.lo, k) : 64 + select64(a.hi, k - c);
}
// Mask of the low n bits (0 <= n <= 128).
OS_HD B128 lowmask128(int n) {
  if (n <= 0) return b128(0, 0);
  if (n < 64) return b128((1ull << n) - 1, 0);
  if (n == 64) return b128(~0ull, 0);
  if (n < 128) return b128(~0ull, (1ull << (n - 64)) - 1);
  return b128(~0ull, ~0ull);
}

// 96-bit bitboard (three u32 words) for boards of at most 96 cells (go up to
// 9 x 9 on the lane kernels, os_kernels.h Go9).  Bit i = cell i, as B128.  A
// B128 word operation is two 32-bit VALU operations and a B128 shift five
// (two 64-bit shifts, the carried-in half, two ORs); here they are three
// (a shift and two funnel shifts, v_alignbit_b32), and a board is three VGPRs.
struct B96 {
  uint32_t w0, w1, w2;
};
OS_HD B96 b96(uint32_t w0, uint32_t w1, uint32_t w2) {
  B96 r;
  r.w0 = w0; r.w1 = w1; r.w2 = w2;
  return r;
}
OS_HD B96 b96_of(const B128& x) {  // the low 96 cells
  return b96(static_cast<uint32_t>(x.lo), static_cast<uint32_t>(x.lo >> 32),
             static_cast<uint32_t>(x.hi));
}
OS_HD B128 b128_of(const B96& x) {
  return b128(static_cast<uint64_t>(x.w0) | (static_cast<uint64_t>(x.w1) << 32), x.w2);
}
OS_HD B96 sel96(bool c, B96 x, B96 y) {  // word by word (see sel128)
  const uint32_t w0 = c ? x.w0 : y.w0;
  const uint32_t w1 = c ? x.w1 : y.w1;
  const uint32_t w2 = c ? x.w2 : y.w2;
  return b96(w0, w1, w2);
}
OS_HD B96 pick(const B96* a, int i) { return sel96(i != 0, a[1], a[0]); }
OS_HD void put(B96* a, int i, B96 v) {
  const B96 v0 = sel96(i != 0, a[0], v), v1 = sel96(i != 0, v, a[1]);
  a[0] = v0;
  a[1] = v1;
}
OS_HD B96 operator|(B96 a, B96 b) { return b96(a.w0 | b.w0, a.w1 | b.w1, a.w2 | b.w2); }
OS_HD B96 operator&(B96 a, B96 b) { return b96(a.w0 & b.w0, a.w1 & b.w1, a.w2 & b.w2); }
OS_HD B96 operator^(B96 a, B96 b) { return b96(a.w0 ^ b.w0, a.w1 ^ b.w1, a.w2 ^ b.w2); }
OS_HD B96 operator~(B96 a) { return b96(~a.w0, ~a.w1, ~a.w2); }
OS_HD bool operator==(B96 a, B96 b) {
  return ((a.w0 ^ b.w0) | (a.w1 ^ b.w1) | (a.w2 ^ b.w2)) == 0u;
}
OS_HD bool operator!=(B96 a, B96 b) { return !(a == b); }
OS_HD bool any(B96 a) { return (a.w0 | a.w1 | a.w2) != 0u; }
OS_HD int popc32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x);
#else
  return __builtin_popcount(x);
#endif
}
OS_HD int ctz32(uint32_t x) {  // x != 0
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffs(static_cast<int>(x)) - 1;
#else
  return __builtin_ctz(x);
#endif
}
OS_HD int popc(B96 a) { return popc32(a.w0) + popc32(a.w1) + popc32(a.w2); }
// Branch-free word choice in lowest / select96 (1) or a branch per word (0).
// A/B knob.
#ifndef OS_SELECT96_FLAT
#define OS_SELECT96_FLAT 1
#endif
// Funnel shifts: the compiler maps (hi << s) | (lo >> (32 - s)) to one
// v_alignbit_b32.
OS_HD B96 shl(B96 a, int s) {  // 0 < s < 32
  return b96(a.w0 << s, (a.w1 << s) | (a.w0 >> (32 - s)), (a.w2 << s) | (a.w1 >> (32 - s)));
}
OS_HD B96 shr(B96 a, int s) {  // 0 < s < 32
  return b96((a.w0 >> s) | (a.w1 << (32 - s)), (a.w1 >> s) | (a.w2 << (32 - s)), a.w2 >> s);
}
OS_HD B96 bit96(int i) {  // 0 <= i < 96
  const uint32_t m = 1u << (i & 31);
  const int q = i >> 5;
  return b96(q == 0 ? m : 0u, q == 1 ? m : 0u, q == 2 ? m : 0u);
}
OS_HD bool test(B96 a, int i) {
  const int q = i >> 5;
  const uint32_t w = q == 0 ? a.w0 : (q == 1 ? a.w1 : a.w2);
  return (w >> (i & 31)) & 1u;
}
// The word first, then one count (as select96): a ternary over three ctz's
// is emitted as exec-mask branches.
OS_HD int lowest(B96 a) {  // a != 0
  if (!OS_SELECT96_FLAT) return a.w0 ? ctz32(a.w0) : (a.w1 ? 32 + ctz32(a.w1) : 64 + ctz32(a.w2));
  const bool z0 = a.w0 == 0u, z01 = z0 && a.w1 == 0u;
  const uint32_t w = z0 ? (z01 ? a.w2 : a.w1) : a.w0;
  const int base = z0 ? (z01 ? 64 : 32) : 0;
#if defined(__HIP_DEVICE_COMPILE__)
  return base + __builtin_ctz(w);  // w != 0
#else
  return base + ctz32(w);
#endif
}
// Index of the k-th (0-based) set bit of x, ascending; k < popc(x).
OS_HD int select32(uint32_t x, int k) {
  int base = 0;
  int c = popc32(x & 0xFFFFu);
  if (k >= c) { k -= c; x >>= 16; base += 16; }
  c = popc32(x & 0xFFu);
  if (k >= c) { k -= c; x >>= 8; base += 8; }
  c = popc32(x & 0xFu);
  if (k >= c) { k -= c; x >>= 4; base += 4; }
  c = popc32(x & 0x3u);
  if (k >= c) { k -= c; x >>= 2; base += 2; }
  c = static_cast<int>(x & 1u);
  if (k >= c) { base += 1; }
  return base;
}
// Branch-free word choice, then one select32: the lanes of a wave pick
// different words, and a branch per word would run every lane through all
// three selects.
OS_HD int select96(B96 a, int k) {  // k < popc(a)
  if (!OS_SELECT96_FLAT) {
    const int c0 = popc32(a.w0);
    if (k < c0) return select32(a.w0, k);
    k -= c0;
    const int c1 = popc32(a.w1);
    return k < c1 ? 32 + select32(a.w1, k) : 64 + select32(a.w2, k - c1);
  }
  const int c0 = popc32(a.w0);
  const int c01 = c0 + popc32(a.w1);
  const bool in0 = k < c0, in1 = k < c01;
  const uint32_t w = in0 ? a.w0 : (in1 ? a.w1 : a.w2);
  const int base = in0 ? 0 : (in1 ? 32 : 64);
  const int kk = k - (in0 ? 0 : (in1 ? c0 : c01));
  return base + select32(w, kk);
}
OS_HD B96 lowmask96(int n) {  // 0 <= n <= 96
  return b96(n >= 32 ? ~0u : (n <= 0 ? 0u : (1u << n) - 1u),
             n >= 64 ? ~0u : (n <= 32 ? 0u : (1u << (n - 32)) - 1u),
             n >= 96 ? ~0u : (n <= 64 ? 0u : (1u << (n - 64)) - 1u));
}

// 384-bit bitboard (six u64 words) for boards above 11 x 11 (hex, go up to
// 19 x 19).  Same operations as B128; every loop is unrolled, so the words
// are only ever indexed by constants.
struct B384 {
  uint64_t w[6];
};
#define OS_B384_MAP(expr) \
  B384 r;                  \
  _Pragma("unroll") for (int i = 0; i < 6; ++i) r.w[i] = (expr); \
  return r
OS_HD B384 operator|(B384 a, B384 b) { OS_B384_MAP(a.w[i] | b.w[i]); }
OS_HD B384 operator&(B384 a, B384 b) { OS_B384_MAP(a.w[i] & b.w[i]); }
OS_HD B384 operator^(B384 a, B384 b) { OS_B384_MAP(a.w[i] ^ b.w[i]); }
OS_HD B384 operator~(B384 a) { OS_B384_MAP(~a.w[i]); }
OS_HD bool operator==(B384 a, B384 b) {
  uint64_t d = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) d |= a.w[i] ^ b.w[i];
  return d == 0;
}
OS_HD bool operator!=(B384 a, B384 b) { return !(a == b); }
OS_HD bool any(B384 a) {
  uint64_t d = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) d |= a.w[i];
  return d != 0;
}
OS_HD int popc(B384 a) {
  int c = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) c += popc64(a.w[i]);
  return c;
}
OS_HD B384 shl(B384 a, int s) {  // 0 < s < 64
  OS_B384_MAP((a.w[i] << s) | (i ? a.w[i ? i - 1 : 0] >> (64 - s) : 0ull));
}
OS_HD B384 shr(B384 a, int s) {  // 0 < s < 64
  OS_B384_MAP((a.w[i] >> s) | (i < 5 ? a.w[i < 5 ? i + 1 : 5] << (64 - s) : 0ull));
}
OS_HD B384 sel384(bool c, B384 x, B384 y) { OS_B384_MAP(c ? x.w[i] : y.w[i]); }
OS_HD B384 bit384(int b) { OS_B384_MAP((b >> 6) == i ? (1ull << (b & 63)) : 0ull); }
OS_HD bool test(B384 a, int b) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) v |= (b >> 6) == i ? a.w[i] : 0ull;
  return (v >> (b & 63)) & 1;
}
OS_HD int lowest(B384 a) {  // a != 0
  int r = -1;
#pragma unroll
  for (int i = 5; i >= 0; --i) r = a.w[i] ? 64 * i + ctz64(a.w[i]) : r;
  return r;
}
OS_HD int select384(B384 a, int k) {  // k < popc(a)
  int r = -1;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int c = popc64(a.w[i]);
    if (r < 0 && k < c) r = 64 * i + select64(a.w[i], k);
    k -= c;
  }
  return r;
}
OS_HD B384 lowmask384(int n) {  // 0 <= n <= 384
  OS_B384_MAP(n >= 64 * (i + 1) ? ~0ull : (n <= 64 * i ? 0ull : (1ull << (n - 64 * i)) - 1));
}
#undef OS_B384_MAP
OS_HD B384 pick(const B384* a, int i) { return sel384(i != 0, a[1], a[0]); }
OS_HD void put(B384* a, int i, B384 v) {
  const B384 v0 = sel384(i != 0, a[0], v), v1 = sel384(i != 0, v, a[1]);
  a[0] = v0;
  a[1] = v1;
}

// Bitboard-width-generic constructors for the game templates (os_games.h).
template <class B>
struct BB;
template <>
struct BB<B128> {
  static constexpr int kBits = 128;
  OS_HD static B128 zero() { return b128(0, 0); }
  OS_HD static B128 bit(int i) { return bit128(i); }
  OS_HD static B128 lowmask(int n) { return lowmask128(n); }
  OS_HD static int select(B128 a, int k) { return select128(a, k); }
  OS_HD static B128 sel(bool c, B128 x, B128 y) { return sel128(c, x, y); }
};
template <>
struct BB<B96> {
  static constexpr int kBits = 96;
  OS_HD static B96 zero() { return b96(0u, 0u, 0u); }
  OS_HD static B96 bit(int i) { return bit96(i); }
  OS_HD static B96 lowmask(int n) { return lowmask96(n); }
  OS_HD static int select(B96 a, int k) { return select96(a, k); }
  OS_HD static B96 sel(bool c, B96 x, B96 y) { return sel96(c, x, y); }
};
template <>
struct BB<B384> {
  static constexpr int kBits = 384;
  OS_HD static B384 zero() { return lowmask384(0); }
  OS_HD static B384 bit(int i) { return bit384(i); }
  OS_HD static B384 lowmask(int n) { return lowmask384(n); }
  OS_HD static int select(B384 a, int k) { return select384(a, k); }
  OS_HD static B384 sel(bool c, B384 x, B384 y) { return sel384(c, x, y); }
};

}  // namespace osm

#endif  // OS_COMMON_H_
