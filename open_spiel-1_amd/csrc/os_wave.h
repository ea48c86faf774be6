// Wave-per-search execution of the MCTS engine on gfx950 (device only).
//
// One 64-lane wavefront runs one independent search.  The game state, the
// tree walk and the random rollout are wave-uniform (SGPRs, scalar 64-bit
// bitboard ops); the lanes are used where the algorithm has data
// parallelism:
//   * MT19937: the 624-word block is twisted cooperatively in LDS (64 words
//     per step), tempered in parallel, and drawn with v_readlane;
//   * selection: lane k loads child k (coalesced) and evaluates its UCT value;
//     a wave argmax (max value, lowest index on ties == mcts.cc's strict '>'
//     scan) picks the child;
//   * expansion: lane k computes the k-th legal action; the libstdc++ /
//     numpy shuffle runs on the lane-distributed array; lane k writes child k;
//   * backup: lane d updates path node d (mcts.cc:351-357) in one step; the
//     MCTS-Solver max^n backup (:359-395) walks up serially, each level's
//     children outcomes read and reduced across lanes;
//   * go: the superko set lives in the lanes (four entries per lane, one
//     compare + ballot per move); rollouts keep chain labels on the lanes
//     (lane l: points l, l + 64), so a chain is one compare + ballot, not a
//     flood (go_rollout_wave).
// The semantics are those of os_mcts.h::mcts_search (checked bit-exact
// against the oracle by tests/test_gpu_parity.py).
#ifndef OS_WAVE_H_
#define OS_WAVE_H_

#include "os_chance.h"
#include "os_mcts.h"

// Where wave-uniformity of the playout / walk state is re-asserted with
// readfirstlane (A/B switches): 0 never, 1 every ply / step, 2 once on entry
// to the loop (so the loop-carried state can stay in SGPRs).  Measured on
// MI355X, C4 4096 x 1024 (profiles/r01/ab_uniform.txt): ROLL/SEL 0/1 25.6 ms,
// 1/1 27.8, 1/0 28.5; with the DPP argmax 0/1 23.75, 2/1 23.3, 2/2 22.8.
#ifndef OS_UNI_ROLL
#define OS_UNI_ROLL 2
#endif
#ifndef OS_UNI_SEL
#define OS_UNI_SEL 2
#endif
#ifndef OS_UNI_MT
#define OS_UNI_MT 0
#endif
// connect_four's walk state needs no entry re-assertion: its selection loop
// is short and the readfirstlanes cost more than the SGPR copies save
// (profiles/r05/ab_knobs: C2 and self-play faster with mode 0; breakthrough
// and go slower), so the mode is a per-game trait.
#ifndef OS_UNI_SEL_C4
#define OS_UNI_SEL_C4 0
#endif
// 1: connect_four's win test in the tree walk on the vector unit (WaveApply).
#ifndef OS_WAVE_APPLY
#define OS_WAVE_APPLY 1
#endif
// 1: connect_four rollouts build their column / height nibbles on the lanes.
#ifndef OS_C4_LANE_SETUP
#define OS_C4_LANE_SETUP 1
#endif
// 1: connect_four expansions take LegalActions()[lane] from a row scan.
#ifndef OS_WAVE_KTH
#define OS_WAVE_KTH 1
#endif
// 1: connect_four rollout lanes test four-in-a-row branch-free.
#ifndef OS_C4_BF_FOUR
#define OS_C4_BF_FOUR 1
#endif
// 1: the register mirror of the root's children is updated by selects.
#ifndef OS_MIRROR_SEL
#define OS_MIRROR_SEL 1
#endif
// UCT argmax screened in f32 (exact f64 only on near ties): 1 narrow games,
// 2 every game.
#ifndef OS_UCT_SCREEN
#define OS_UCT_SCREEN 2
#endif
// 1: tic_tac_toe / connect_four keep the visit path in the lanes (LanePath).
#ifndef OS_LANE_PATH
#define OS_LANE_PATH 1
#endif
// Diagnostic build (-DOS_PHASE_TIMING=1): per-phase shader-clock cycles of the
// wave search, summed over waves into PhaseCycles (os_debug_phase_cycles).
#ifndef OS_PHASE_TIMING
#define OS_PHASE_TIMING 0
#endif
// Phase builds only: the selection's parts for the non-go games, in the go
// slots (tools/phase_single.py prints them as go_legal..go_score): before
// the level loop, the level loop, after it (expansion included), and the
// scoring inside the loop.
#ifndef OS_PHASE_SEL
#define OS_PHASE_SEL 0
#endif
// UCT screen: settle the argmax by one band ballot when the maximum is the
// only child in the near-tie band (A/B knob; 0 = always the identity test).
#ifndef OS_SCREEN_BAND
#define OS_SCREEN_BAND 1
#endif
// Timing-only A/B switch (results not bit-exact): 1 skips the hex end-of-fill
// relaxation, 2 the hex fill-order rank-select loop.
#ifndef OS_AB_HEX
#define OS_AB_HEX 0
#endif

// Issue priority by progress (results unchanged): the wave searches of a
// launch start together and share each SIMD four ways, and the hardware
// arbitrates issue by priority, then age, so without help the youngest waves
// (the last roots) starve and finish last while the SIMD idles around them.
// Every OS_PACE_EVERY simulations a search compares its own simulation count
// with the mean over the searches resident at that moment (one packed
// launch-wide counter: resident searches << 44 | their simulations) and sets
// its priority (s_setprio 0..3) by how far behind or ahead of the mean it is,
// with bands of max_simulations / OS_PACE_BAND.  C2: 9.26 -> 7.2 ms.
#ifndef OS_PACE
#define OS_PACE 1
#endif
// OS_SCREEN_LOG (integer-reward UCT with the f32 screen): 1 takes the
// screen's log(N) from v_log_f32 of the parent count (no per-lane log-table
// gather on the selection chain; the exact f64 log(N) is read only when the
// screen falls back), reduces the screen by integer keys (DPP folded into
// v_max_i32) and bounds the near-tie band with v_sqrt_f32.
#ifndef OS_SCREEN_LOG
#define OS_SCREEN_LOG 1
#endif
#ifndef OS_PACE_EVERY
#define OS_PACE_EVERY 32
#endif
#ifndef OS_PACE_BAND
#define OS_PACE_BAND 32
#endif

namespace osm {

#if OS_PACE
static __device__ unsigned long long g_pace;  // internal linkage: one per game TU
#endif

template <class G>
struct UniSel { static constexpr int kMode = OS_UNI_SEL; };
template <>
struct UniSel<ConnectFour> { static constexpr int kMode = OS_UNI_SEL_C4; };

enum PhaseId { kPhSelect = 0, kPhExpand, kPhRollout, kPhBackup, kPhSolver, kPhTail,
               kPhTwist, kPhTotal,
               // go rollout breakdown (inside kPhRollout): legal + draw, apply
               // (with the superko insert), the insert alone, the final score
               kPhGoLegal, kPhGoApply, kPhGoInsert, kPhGoScore,
               // go apply on the wave (inside kPhGoApply): own chains joined,
               // opponent chains (captures), the mover's chain, the rest
               kPhX0, kPhX1, kPhX2, kPhX3, kNumPhases };
struct PhaseCycles {
  uint64_t c[kNumPhases];
};
// Diagnostic build (-DOS_WAVE_TIMES=1): each wave search also records
// (s_memrealtime at start, at end, HW_ID | XCC_ID << 32) after the phase
// counters, one triple per root (first kWaveTimesMax roots).
#ifndef OS_WAVE_TIMES
#define OS_WAVE_TIMES 0
#endif
constexpr int kWaveTimesMax = 16384;
constexpr int kDbgSlots = kNumPhases + (OS_WAVE_TIMES ? 3 * kWaveTimesMax : 0);
#if OS_PHASE_TIMING
#define OS_PH_NOW() __builtin_amdgcn_s_memtime()
#define OS_PH_ADD(acc, t0) ((acc) += __builtin_amdgcn_s_memtime() - (t0))
#else
#define OS_PH_NOW() 0ull
#define OS_PH_ADD(acc, t0) ((void)(t0))
#endif

__device__ __forceinline__ int lane_id() { return static_cast<int>(threadIdx.x & 63); }

__device__ __forceinline__ uint32_t rl32(uint32_t v, int lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), lane));
}
__device__ __forceinline__ int32_t rli(int32_t v, int lane) {
  return __builtin_amdgcn_readlane(v, lane);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  const uint32_t lo = rl32(static_cast<uint32_t>(v), lane);
  const uint32_t hi = rl32(static_cast<uint32_t>(v >> 32), lane);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ double rld(double v, int lane) {
  return __longlong_as_double(static_cast<long long>(
      rl64(static_cast<uint64_t>(__double_as_longlong(v)), lane)));
}
__device__ __forceinline__ uint32_t wl32(uint32_t v, int lane, uint32_t old) {
  return lane_id() == lane ? v : old;  // v_cmp + v_cndmask
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// An instrumentation counter kept in lane 0 of a VGPR rather than in an
// SGPR: the wave kernels are SGPR-bound (the state, the tree walk and both
// MT streams are scalar), and a spilled SGPR costs far more than one VALU op.
// The pacing counter of one wave (see OS_PACE): `progress` is the work the
// wave has done (simulations), `band` the gap that moves it one priority
// level.
struct Pacer {
  static constexpr int kShift = 44;
  unsigned long long added = 0;  // this wave's share of the counter
  uint32_t reported = 0;
  __device__ __forceinline__ void begin() {
#if OS_PACE
    added = 1ull << kShift;
    if (lane_id() == 0) atomicAdd(&g_pace, added);
#endif
  }
  __device__ __forceinline__ void update(uint32_t progress, int64_t band) {
#if OS_PACE
    const unsigned long long d = progress - reported;
    reported = progress;
    added += d;
    unsigned long long c = 0;
    if (lane_id() == 0) c = atomicAdd(&g_pace, d);
    c = rl64(c, 0) + d;
    const int64_t active = static_cast<int64_t>(c >> kShift);
    const int64_t sum = static_cast<int64_t>(c & ((1ull << kShift) - 1));
    // (mean - progress) * active against band * active
    const int64_t gap = sum - static_cast<int64_t>(progress) * active;
    band *= active;
    if (gap > band) __builtin_amdgcn_s_setprio(3);
    else if (gap > 0) __builtin_amdgcn_s_setprio(2);
    else if (gap > -band) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#else
    (void)progress;
    (void)band;
#endif
  }
  __device__ __forceinline__ void end() {
#if OS_PACE
    if (lane_id() == 0) atomicAdd(&g_pace, 0ull - added);
    __builtin_amdgcn_s_setprio(0);
#endif
  }
};

struct LaneCount {
  uint32_t v;
  __device__ void reset() { v = 0; }
  __device__ void add(uint32_t x) { v += lane_id() == 0 ? x : 0u; }
  __device__ void max(uint32_t x) {
    const uint32_t y = lane_id() == 0 ? x : 0u;
    v = y > v ? y : v;
  }
  __device__ uint32_t get() const { return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 0)); }
};

// Marks a trivially-copyable value as wave-uniform (v_readfirstlane per
// dword) so the compiler keeps it, and everything computed from it, in SGPRs
// and runs the game logic on the scalar unit.
template <class T>
__device__ __forceinline__ T make_uniform(const T& v) {
  static_assert(sizeof(T) % 4 == 0, "dword-sized state expected");
  T out;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
  for (int i = 0; i < static_cast<int>(sizeof(T) / 4); ++i)
    dst[i] = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(src[i])));
  return out;
}

// MT19937 stream whose 624-word state lives in LDS, shared by the wave.
// Draws are wave-uniform.  `cur` holds 64 tempered words of the current block
// (word base + lane in lane `lane`).
struct WaveMt {
  uint32_t* s;     // LDS, 624 words
  uint32_t cur;    // per lane
  uint32_t nxt;    // per lane: tempered word base + lane + 1 (cur of the next lane)
  int base;        // first word index held in cur; kMtN => block exhausted
  int valid;       // words held in cur
  int pos;         // next word (offset in cur)
  LaneCount words;  // draws (instrumentation; lane 0 of a VGPR)
#if OS_PHASE_TIMING
  uint64_t twist_cycles;
#endif

  // Every field is written on every path, and the last store of each path
  // is to the same field: SimplifyCFG otherwise sinks the tail stores of two
  // paths (pos = 0 / pre7 = ...) into one store through a phi of pointers,
  // which leaves pos and pre7 in scratch for the whole kernel.
  __device__ void init_seeded() {  // state = init_genrand output, untwisted
    words.reset();
#if OS_PHASE_TIMING
    twist_cycles = 0;
#endif
    cur = 0;
    nxt = 0;
    pre7 = 0x80000000u;
    base = kMtN;
    valid = 0;
    pos = 0;
  }
  // numpy legacy (key, p): key is a fully twisted block, p words consumed.
  __device__ void init_import(int p) {
    words.reset();
#if OS_PHASE_TIMING
    twist_cycles = 0;
#endif
    const bool live = p < kMtN;
    base = live ? (p & ~63) : kMtN;
    valid = live ? (kMtN - base < 64 ? kMtN - base : 64) : 0;
    load_window(base + lane_id());
    pre7 = use7 && live ? small7() : 0x80000000u;
    pos = live ? p - base : 0;
  }
  // The pair (cur, nxt) of every lane is read once per window, so
  // uniform_lanes() needs no cross-lane shuffle per draw (small7() reads the
  // pairs once per window and shuffles instead).
  // Every lane reads (lanes past the block re-read its last word) and selects,
  // so the LDS reads need no exec-mask branch.
  __device__ void load_window(int i) {
    const uint32_t w0 = MtStream::temper(s[i < kMtN ? i : kMtN - 1]);
    const uint32_t w1 = MtStream::temper(s[i + 1 < kMtN ? i + 1 : kMtN - 1]);
    cur = i < kMtN ? w0 : 0u;
    nxt = !use7 && i + 1 < kMtN ? w1 : 0u;
  }
  __device__ int export_pos() const { return base >= kMtN ? kMtN : base + pos; }

  // Cooperative in-place twist of the whole block (same result as 624 serial
  // steps: word i reads old s[i], old s[i+1] and s[(i+397) % 624], which is
  // new exactly for i >= 227, and every such word lies >= 3 chunks back).
  __device__ void twist() {
    const int l = lane_id();
#if OS_PHASE_TIMING
    const uint64_t t0 = OS_PH_NOW();
#endif
    for (int c = 0; c < kMtN; c += 64) {
      // Lanes past the block (last chunk only) compute on a clamped index and
      // do not store: no exec-mask branch around the reads.
      const int i = c + l < kMtN ? c + l : kMtN - 1;
      const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
      const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
      const uint32_t y = (s[i] & 0x80000000u) | (s[i1] & 0x7fffffffu);
      const uint32_t v = s[im] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      __builtin_amdgcn_wave_barrier();
      if (c + 64 <= kMtN || c + l < kMtN) s[i] = v;  // wave-uniform except the last chunk
      __builtin_amdgcn_wave_barrier();
    }
#if OS_PHASE_TIMING
    OS_PH_ADD(twist_cycles, t0);
#endif
  }
  __device__ void refill() {
    int nb = base + valid;
    if (base >= kMtN || nb >= kMtN) {
      twist();
      nb = 0;
    }
    base = nb;
    valid = kMtN - base < 64 ? kMtN - base : 64;
    load_window(base + lane_id());
    if (use7) pre7 = small7();
    pos = 0;
  }

  // Small-range absl draws precomputed on the vector unit (connect_four
  // rollouts, n = |LegalActions| <= 7): lane l packs, for the word pair
  // (w_l, w_{l+1}) of the window, absl::Uniform(0, n) for n = 1..7 in bits
  // 3(n-1)..3(n-1)+2 (os_rng.h AbslUniform: power-of-two n -> low bits of the
  // second word; else the high half of the 64x32 Lemire product); bit 31 marks
  // a pair without a next word in the window or one that could need absl's
  // rejection step -- uniform_small() then takes the exact scalar path.
  uint32_t pre7;
  int use7;
  __device__ uint32_t small7() const {
    const int l = lane_id();
    const uint32_t hi = cur;
    const uint32_t lo = static_cast<uint32_t>(__shfl_down(static_cast<int>(cur), 1));
    uint32_t pk = (l + 1 >= valid) ? 0x80000000u : 0u;
    for (uint32_t n = 2; n <= 7; ++n) {
      uint32_t r;
      if ((n & (n - 1)) == 0) {
        r = lo & (n - 1);
      } else {
        const uint64_t b = static_cast<uint64_t>(lo) * n;
        const uint64_t mid = static_cast<uint64_t>(hi) * n + (b >> 32);
        if (static_cast<uint32_t>(mid) == 0 && static_cast<uint32_t>(b) < n) pk |= 0x80000000u;
        r = static_cast<uint32_t>(mid >> 32);
      }
      pk |= r << (3 * (n - 1));
    }
    return pk;
  }
  // absl::Uniform(rng, 0u, n) for n <= 7 from the precomputed table, falling
  // back to the exact two-word draw (os_rng.h) when the table cannot answer.
  __device__ __forceinline__ uint32_t uniform_small(uint32_t n) {
    if (pos + 2 <= valid) {
      const uint32_t pk = rl32(pre7, pos);
      if (!(pk >> 31)) {
        pos += 2;
        words.add(2);
        return (pk >> (3 * (n - 1))) & 7u;
      }
    }
    return AbslUniform(*this, n);
  }
  // absl::Uniform(rng, 0u, n) for any n (< 2^32) with the Lemire arithmetic
  // on the vector unit: lane l evaluates the word pair (w_l, w_{l+1}) of the
  // window and the draw reads lane pos.  A pair that straddles the window or
  // whose product could need absl's rejection step (os_rng.h AbslUniform)
  // takes the exact scalar path, so the stream is consumed identically.
  __device__ __forceinline__ uint32_t uniform_lanes(uint32_t n) {
    if (pos + 2 <= valid) {
      const uint32_t hi = cur;
      const uint32_t lo = nxt;
      // Both forms are evaluated and selected (no branch on n).
      const uint32_t m = n - 1;
      const bool pow2 = (n & m) == 0;
      const uint64_t b = static_cast<uint64_t>(lo) * n;
      const uint64_t mid = static_cast<uint64_t>(hi) * n + (b >> 32);
      const bool slow = static_cast<uint32_t>(mid) == 0 && static_cast<uint32_t>(b) < n;
      const uint32_t pm = 0u - static_cast<uint32_t>(pow2);  // all ones for a power of two
      const uint32_t lem = slow ? 0x80000000u : static_cast<uint32_t>(mid >> 32);
      const uint32_t r = (lo & m & pm) | (lem & ~pm);
      const uint32_t v = rl32(r, pos);
      if (!(v >> 31)) {
        pos += 2;
        words.add(2);
        return v;
      }
    }
    return AbslUniform(*this, n);
  }
  // Stream offset of the next word, counted from the start of the block in s
  // (kMtN when that block is used up and the next draw twists).
  __device__ int offset() const { return base >= kMtN ? kMtN : base + pos; }
  // Untempered word q (q < kMtN + 454) of the stream counted like offset(),
  // read without changing the block: the next block's word i follows the
  // in-place twist (it reads s[i], s[i+1] and s[i+397], which is already new
  // for i >= 227), so words of the next block are recomputed from the old.
  __device__ static uint32_t mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  __device__ uint32_t peek_raw(int q) const {
    if (q < kMtN) return s[q];
    const int i = q - kMtN;
    const uint32_t v = mix(s[i], s[i + 1]);
    if (i < kMtN - kMtM) return v ^ s[i + kMtM];
    const int i2 = i - (kMtN - kMtM);
    return v ^ mix(s[i2], s[i2 + 1]) ^ s[i2 + kMtM];
  }
  // Moves the stream to offset q (< 2 kMtN; counted like offset()), twisting
  // the block when q has left it; the window is re-read as refill() would.
  __device__ void seek(int q) {
    if (q >= kMtN) {
      twist();
      q -= kMtN;
    }
    base = q & ~63;
    valid = kMtN - base < 64 ? kMtN - base : 64;
    load_window(base + lane_id());
    pre7 = use7 ? small7() : 0x80000000u;
    pos = q - base;
  }
  __device__ void uniformize() {
    pos = __builtin_amdgcn_readfirstlane(pos);
    valid = __builtin_amdgcn_readfirstlane(valid);
    base = __builtin_amdgcn_readfirstlane(base);
  }
  __device__ uint32_t next() {
#if OS_UNI_MT
    // The counters are wave-uniform; say so, or a divergent loop exit upstream
    // (temporal divergence) leaves them in VGPRs with exec-masked branches.
    pos = __builtin_amdgcn_readfirstlane(pos);
    valid = __builtin_amdgcn_readfirstlane(valid);
    base = __builtin_amdgcn_readfirstlane(base);
#endif
    if (pos >= valid) refill();
    const uint32_t w = rl32(cur, pos);
    ++pos;
    words.add(1);
    return w;
  }
};

// Go superko context for one search per wave (go.cc:199-208).  The whole set
// -- the positions before the root (base) followed by those logged since --
// lives in the lanes: entry i in lane i % 64 of slot i / 64, up to kCap
// entries (a game of n x n <= 11 x 11 logs at most 2 n^2 + 1 <= 243).  A new
// position is compared with every candidate at once (four 64-bit compares and
// one ballot).  Candidates: the base, and entries logged before the most recent
// capture -- without a capture the stone count only grows, so no later
// position can repeat (the same rule as GoCtx, os_games.h).
struct GoWaveCtx {
  static constexpr bool kWaveUniform = true;  // GoT::legal: the scalar-unit form
#if OS_PHASE_TIMING
  uint64_t* sub;  // PhaseCycles::c of the search (go breakdown)
#endif
  static constexpr int kCap = 256;
  const uint64_t* zob;
  const uint64_t* base;   // hashes before the root (global), copied into the slots
  int32_t n_base;
  int32_t n;              // entries held (base included)
  int32_t cand_end;       // entries [0, cand_end) can repeat a new position
  uint64_t s0, s1, s2, s3;  // per lane: entries lane, lane + 64, + 128, + 192

  __device__ void reset() {
    n = n_base;
    cand_end = n_base;
  }
  // Copies the base into the slots (every lane loads its four entries).
  __device__ void init_filters() {
    const int l = lane_id();
    n_base = n_base < kCap ? n_base : kCap;
    s0 = l < n_base ? base[l] : 0ull;
    s1 = l + 64 < n_base ? base[l + 64] : 0ull;
    s2 = l + 128 < n_base ? base[l + 128] : 0ull;
    s3 = l + 192 < n_base ? base[l + 192] : 0ull;
    reset();
  }
  __device__ uint64_t entry(int i) const {
    const int j = i >> 6, q = i & 63;
    const uint64_t v = j == 0 ? s0 : (j == 1 ? s1 : (j == 2 ? s2 : s3));
    return rl64(v, q);
  }
  __device__ bool insert(uint64_t h, bool captured, int stones) {
    (void)stones;
#if OS_PHASE_TIMING
    const uint64_t t0 = OS_PH_NOW();
#endif
    if (captured) cand_end = n;
    bool dup = false;
    if (cand_end > 0) {
      const int l = lane_id();
      const bool hit = (l < cand_end && s0 == h) | (l + 64 < cand_end && s1 == h) |
                       (l + 128 < cand_end && s2 == h) | (l + 192 < cand_end && s3 == h);
      dup = ballot(hit) != 0;
    }
    if (!dup && n < kCap) {
      const int l = lane_id();
      const int j = n >> 6;
      const bool me = l == (n & 63);
      s0 = me && j == 0 ? h : s0;
      s1 = me && j == 1 ? h : s1;
      s2 = me && j == 2 ? h : s2;
      s3 = me && j == 3 ? h : s3;
      ++n;
    }
#if OS_PHASE_TIMING
    OS_PH_ADD(sub[kPhGoInsert], t0);
#endif
    return !dup;
  }
};

// The bot rng of a RESUMABLE wave search (k_waz_step): between launches the
// stream lives in HBM in numpy's (key[624], pos) form -- a fully twisted
// block and the words consumed -- so a launch reads only the 64-word windows
// it draws from.  A twist (block used up) copies the row to LDS and twists it
// there cooperatively (WaveMt::twist); the launch then reads the LDS copy, and
// save() writes the new block back.  The row is never written in place while
// it is being read.
struct WaveMtRow : WaveMt {
  uint32_t* row;  // global, 624 words
  uint32_t* lds;  // LDS scratch, 624 words
  int dirty;
  // p: words consumed (kMtN: the next draw twists -- a fresh seed's state).
  __device__ void init_row(uint32_t* r, uint32_t* scratch, int p, bool row_in_lds) {
    row = r;
    lds = scratch;
    dirty = row_in_lds ? 1 : 0;
    s = row_in_lds ? scratch : r;
    use7 = 0;
    init_import(p);
  }
  __device__ void twist() {
    if (s != lds) {
      for (int i = lane_id(); i < kMtN; i += 64) lds[i] = row[i];
      __builtin_amdgcn_wave_barrier();
      s = lds;
    }
    WaveMt::twist();
    dirty = 1;
  }
  __device__ void refill() {
    int nb = base + valid;
    if (base >= kMtN || nb >= kMtN) {
      twist();
      nb = 0;
    }
    base = nb;
    valid = kMtN - base < 64 ? kMtN - base : 64;
    load_window(base + lane_id());
    pos = 0;
  }
  __device__ uint32_t next() {
    if (pos >= valid) refill();
    const uint32_t w = rl32(cur, pos);
    ++pos;
    words.add(1);
    return w;
  }
  __device__ void save() {
    if (dirty) {
      __builtin_amdgcn_wave_barrier();
      for (int i = lane_id(); i < kMtN; i += 64) row[i] = lds[i];
    }
  }
};

template <class G>
struct WaveCtxOf {
  using type = NoCtx;
};
template <>
struct WaveCtxOf<Go> {
  using type = GoWaveCtx;
};

// Lane-distributed array of up to 128 u16 actions: element i in lane i % 64 of
// slot i / 64.
struct LaneArr {
  uint32_t a0, a1;
  __device__ uint32_t get(int i) const { return i < 64 ? rl32(a0, i) : rl32(a1, i - 64); }
  __device__ void set(int i, uint32_t v) {
    if (i < 64) a0 = wl32(v, i, a0);
    else a1 = wl32(v, i - 64, a1);
  }
  __device__ void swap(int i, int j) {
    if (i == j) return;
    const uint32_t x = get(i), y = get(j);
    set(i, y);
    set(j, x);
  }
};

// x / d for the shuffle's pair draw without the integer-division sequence:
// x * (floor(2^21 / d) + 1) >> 21 is exact for every x < (d - 1) * d,
// 2 <= d <= 131 (checked exhaustively), which covers x < b0 * b1 for every
// supported |LegalActions| (<= 128).
static __constant__ const uint32_t kDivMagic[132] = {
    0u, 2097153u, 1048577u, 699051u, 524289u, 419431u, 349526u, 299594u,
    262145u, 233017u, 209716u, 190651u, 174763u, 161320u, 149797u, 139811u,
    131073u, 123362u, 116509u, 110377u, 104858u, 99865u, 95326u, 91181u,
    87382u, 83887u, 80660u, 77673u, 74899u, 72316u, 69906u, 67651u,
    65537u, 63551u, 61681u, 59919u, 58255u, 56680u, 55189u, 53774u,
    52429u, 51151u, 49933u, 48771u, 47663u, 46604u, 45591u, 44621u,
    43691u, 42800u, 41944u, 41121u, 40330u, 39569u, 38837u, 38131u,
    37450u, 36793u, 36158u, 35545u, 34953u, 34380u, 33826u, 33289u,
    32769u, 32264u, 31776u, 31301u, 30841u, 30394u, 29960u, 29538u,
    29128u, 28729u, 28340u, 27963u, 27595u, 27236u, 26887u, 26547u,
    26215u, 25891u, 25576u, 25267u, 24967u, 24673u, 24386u, 24106u,
    23832u, 23564u, 23302u, 23046u, 22796u, 22551u, 22311u, 22076u,
    21846u, 21621u, 21400u, 21184u, 20972u, 20764u, 20561u, 20361u,
    20165u, 19973u, 19785u, 19600u, 19419u, 19240u, 19066u, 18894u,
    18725u, 18559u, 18397u, 18237u, 18079u, 17925u, 17773u, 17624u,
    17477u, 17332u, 17190u, 17051u, 16913u, 16778u, 16645u, 16514u,
    16385u, 16257u, 16132u, 16009u,
};
__device__ __forceinline__ uint32_t div_pair(uint32_t x, uint32_t d) {
  return (x * kDivMagic[d]) >> 21;
}

// libstdc++ 11 std::shuffle (pair path; os_rng.h CppShuffle) on the lanes.
// The serial form alternates a draw, a division and two swaps per step, all on
// the scalar unit.  Here:
//  1. lane k draws step k's Lemire32 word speculatively: window word pos + k,
//     accepted unless its low product half is below the range (then Lemire
//     could reject: that step is drawn exactly by the serial Lemire32, which
//     refills and rejects as the reference, and the lanes resume after it);
//  2. lane k splits its draw into the step's transposition targets;
//  3. every lane traces its own final position back through the
//     transpositions in reverse (the element at p after the last swap came
//     from the partner of p), so the permutation costs a few vector compares
//     per step instead of cross-lane swaps;
//  4. one bpermute per slot gathers the shuffled array.
// Step k: k < e (n even): (1, x), range 2; else i = 1 + e + 2 (k - e), range
// (i + 1)(i + 2), x -> (i, x / (i + 2)) then (i + 1, x % (i + 2)).
template <class Mt>
__device__ __forceinline__ void wave_shuffle_cpp(LaneArr& a, int n, Mt& g) {
  if (n <= 1) return;
  const int l = lane_id();
  const int e = (n & 1) ? 0 : 1;
  const int S = e + (n - 1 - e) / 2;  // <= 64 for n <= 128
  const uint32_t ik = l < e ? 1u : static_cast<uint32_t>(1 + e + 2 * (l - e));
  const uint32_t range = l < e ? 2u : (ik + 1u) * (ik + 2u);
  uint32_t xs = 0;
  for (int s = 0; s < S;) {
    if (g.pos >= g.valid) g.refill();
    const int cnt = min(S - s, g.valid - g.pos);
    const uint32_t w = static_cast<uint32_t>(
        __shfl(static_cast<int>(g.cur), (g.pos + l - s) & 63));
    const uint64_t p = static_cast<uint64_t>(w) * range;
    const bool mine = l >= s && l < s + cnt;
    const uint64_t flagged = ballot(mine && static_cast<uint32_t>(p) < range);
    const int acc = flagged ? ctz64(flagged) - s : cnt;
    if (mine && l < s + acc) xs = static_cast<uint32_t>(p >> 32);
    g.pos += acc;
    g.words.add(static_cast<uint32_t>(acc));
    s += acc;
    if (acc < cnt) {  // a step Lemire could reject: drawn exactly
      xs = wl32(Lemire32(g, rl32(range, s)), s, xs);
      ++s;
    }
  }
  const uint32_t b1 = ik + 2u;
  const uint32_t qv = l < e ? xs : xs / b1;
  const uint32_t rv = xs - qv * b1;  // unused for the single step
  const bool two = n > 64;
  int p0 = l, p1 = l + 64;
  for (int k = S - 1; k >= 0; --k) {
    const int i = k < e ? 1 : 1 + e + 2 * (k - e);
    if (k >= e) {
      const int r = static_cast<int>(rl32(rv, k));
      p0 = p0 == i + 1 ? r : (p0 == r ? i + 1 : p0);
      if (two) p1 = p1 == i + 1 ? r : (p1 == r ? i + 1 : p1);
    }
    const int q = static_cast<int>(rl32(qv, k));
    p0 = p0 == i ? q : (p0 == q ? i : p0);
    if (two) p1 = p1 == i ? q : (p1 == q ? i : p1);
  }
  const uint32_t s00 = static_cast<uint32_t>(__shfl(static_cast<int>(a.a0), p0 & 63));
  const uint32_t s01 = static_cast<uint32_t>(__shfl(static_cast<int>(a.a1), p0 & 63));
  uint32_t n1 = a.a1;
  if (two) {
    const uint32_t s10 = static_cast<uint32_t>(__shfl(static_cast<int>(a.a0), p1 & 63));
    const uint32_t s11 = static_cast<uint32_t>(__shfl(static_cast<int>(a.a1), p1 & 63));
    n1 = p1 < 64 ? s10 : s11;
  }
  a.a0 = p0 < 64 ? s00 : s01;
  a.a1 = n1;
}

// numpy RandomState.shuffle (os_rng.h NpShuffle: j_i = random_interval(i)
// for i = n - 1 .. 1, swap(a[i], a[j_i])) of a lane-distributed array, for
// long lists (hex, breakthrough, go expansions):
//   draws   found over the stream's 64-word window as in fill_draws_np
//           (the mask only halves when i falls below its top bit; one
//           ballot per draw), lane x holding j_{n-1-x};
//   swaps   each lane traces its final position back through the
//           transpositions (i = 1 first) to the position its element came
//           from, and one gather moves the elements.
// The stream is consumed exactly as the serial shuffle consumes it.
template <class Mt>
__device__ void np_shuffle_lanes(LaneArr& a, int n, Mt& g) {
  if (n <= 1) return;
  g.uniformize();
  const int l = lane_id();
  uint32_t rng = static_cast<uint32_t>(n - 1), mask = np_mask(rng);
  auto window_avail = [&]() -> uint64_t {
    const uint64_t below_valid = g.valid >= 64 ? ~0ull : ((1ull << g.valid) - 1ull);
    return g.pos >= 64 ? 0ull : (below_valid & (~0ull << g.pos));
  };
  uint64_t avail = window_avail();
  uint32_t v = g.cur & mask;
  uint32_t j0 = 0, j1 = 0;
  for (int x = 0; x < n - 1; ++x, --rng) {
    if (rng <= (mask >> 1)) {
      mask >>= 1;
      v = g.cur & mask;
    }
    uint64_t ok = ballot(v <= rng) & avail;
    while (!ok) {  // the window's unread words are all rejected
      g.words.add(static_cast<uint32_t>(g.valid - g.pos));
      g.pos = g.valid;
      g.refill();
      avail = window_avail();
      v = g.cur & mask;
      ok = ballot(v <= rng) & avail;
    }
    const int idx = ctz64(ok);
    const uint64_t low = ok & (0ull - ok);
    avail &= ~((low << 1) - 1ull);
    g.words.add(static_cast<uint32_t>(idx + 1 - g.pos));
    g.pos = idx + 1;
    const uint32_t jv = rl32(v, idx);
    if (x < 64) j0 = wl32(jv, x, j0);
    else j1 = wl32(jv, x - 64, j1);
  }
  // final position -> source position (transpositions undone last-first)
  uint32_t p0 = static_cast<uint32_t>(l), p1 = static_cast<uint32_t>(l + 64);
  for (int i = 1; i <= n - 1; ++i) {
    const int x = n - 1 - i;
    const uint32_t ji = x < 64 ? rl32(j0, x) : rl32(j1, x - 64);
    const uint32_t iu = static_cast<uint32_t>(i);
    p0 = p0 == iu ? ji : (p0 == ji ? iu : p0);
    if (n > 64) p1 = p1 == iu ? ji : (p1 == ji ? iu : p1);
  }
  const uint32_t s00 = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(static_cast<int>((p0 & 63) << 2), static_cast<int>(a.a0)));
  const uint32_t s01 = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(static_cast<int>((p0 & 63) << 2), static_cast<int>(a.a1)));
  uint32_t n1 = a.a1;
  if (n > 64) {
    const uint32_t s10 = static_cast<uint32_t>(
        __builtin_amdgcn_ds_bpermute(static_cast<int>((p1 & 63) << 2), static_cast<int>(a.a0)));
    const uint32_t s11 = static_cast<uint32_t>(
        __builtin_amdgcn_ds_bpermute(static_cast<int>((p1 & 63) << 2), static_cast<int>(a.a1)));
    n1 = p1 < 64 ? s10 : s11;
  }
  a.a0 = p0 < 64 ? s00 : s01;
  a.a1 = n1;
}

// kLaneNp: long numpy shuffles take np_shuffle_lanes (not in go's search
// kernels, where the extra live registers cost the wave kernel its
// occupancy and put state in scratch memory).
template <int Policy, class Rng, bool kLaneNp = true>
__device__ void wave_shuffle(LaneArr& a, int n, Rng& g) {
  if constexpr (Policy == kPolicyCpp && std::is_base_of<WaveMt, Rng>::value) {
    wave_shuffle_cpp(a, n, g);
  } else if (Policy == kPolicyCpp) {  // libstdc++ 11 std::shuffle, pair path
    if (n <= 1) return;
    int i = 1;
    if ((n & 1) == 0) {
      a.swap(1, static_cast<int>(Lemire32(g, 2u)));
      i = 2;
    }
    while (i != n) {
      const uint32_t b0 = static_cast<uint32_t>(i) + 1u, b1 = b0 + 1u;
      const uint32_t x = Lemire32(g, b0 * b1);
      const uint32_t q = div_pair(x, b1);
      a.swap(i, static_cast<int>(q));
      a.swap(i + 1, static_cast<int>(x - q * b1));
      i += 2;
    }
  } else if constexpr (kLaneNp && std::is_base_of<WaveMt, Rng>::value) {  // numpy shuffle
    if (n > 16) {
      np_shuffle_lanes(a, n, g);
    } else {
      for (int i = n - 1; i >= 1; --i)
        a.swap(i, static_cast<int>(NpRandomInterval(g, static_cast<uint32_t>(i))));
    }
  } else {
    for (int i = n - 1; i >= 1; --i)
      a.swap(i, static_cast<int>(NpRandomInterval(g, static_cast<uint32_t>(i))));
  }
}

// v from the lane selected by DPP control `Ctrl`; lanes without a source (or
// rows outside RowMask) keep `v` itself.
template <int Ctrl, int RowMask = 0xf>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int nlo = __builtin_amdgcn_update_dpp(lo, lo, Ctrl, RowMask, 0xf, false);
  const int nhi = __builtin_amdgcn_update_dpp(hi, hi, Ctrl, RowMask, 0xf, false);
  return __hiloint2double(nhi, nlo);
}

// Wave-uniform maximum of v over all 64 lanes (all lanes active) by DPP:
// butterflies within each 16-lane row (quad_perm 1032 / 2301, half-mirror,
// mirror), then the row_bcast15 / row_bcast31 scan across rows; lane 63 ends
// with the maximum.  `Lanes` (<= 64) bounds the lanes that can hold a
// candidate (the others hold -inf), so narrow games skip the cross-row steps.
template <int Lanes>
__device__ __forceinline__ double wave_max_f64(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));  // quad_perm [1,0,3,2]
  if (Lanes > 2) v = fmax(v, dpp_f64<0x4E>(v));   // quad_perm [2,3,0,1]
  if (Lanes > 4) v = fmax(v, dpp_f64<0x141>(v));  // row_half_mirror
  if (Lanes > 8) v = fmax(v, dpp_f64<0x140>(v));  // row_mirror
  if (Lanes > 16) {
    v = fmax(v, dpp_f64<0x142, 0xa>(v));  // row_bcast15 -> rows 1, 3
    v = fmax(v, dpp_f64<0x143, 0xc>(v));  // row_bcast31 -> rows 2, 3
    return rld(v, 63);
  }
  return rld(v, 0);
}

// Wave argmax over a lane-distributed candidate array: element k = l + 64 h
// has value v0 (h = 0) or v1 (h = 1) in lane l; absent elements hold -inf.
// Returns the LOWEST index among the maxima (== the first maximum of
// mcts.cc's strict '>' scan in index order), wave-uniform.  No NaNs occur
// (UCT values are finite, +inf or solver outcomes); -0 == +0 as in '>'.
template <int Lanes, bool TwoSlots>
__device__ __forceinline__ int wave_argmax2(double v0, double v1) {
  const double m = wave_max_f64<Lanes>(TwoSlots ? fmax(v0, v1) : v0);
  const uint64_t b0 = ballot(v0 == m);
  if (b0) return ctz64(b0);
  return 64 + ctz64(ballot(v1 == m));
}

// Maximum of v over the first `Lanes` lanes by DPP (as wave_max_f64),
// wave-uniform.
template <int Ctrl, int RowMask = 0xf>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), Ctrl, RowMask, 0xf, false));
}
template <int Lanes>
__device__ __forceinline__ float wave_max_f32(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));                   // quad_perm [1,0,3,2]
  if (Lanes > 2) v = fmaxf(v, dpp_f32<0x4E>(v));    // quad_perm [2,3,0,1]
  if (Lanes > 4) v = fmaxf(v, dpp_f32<0x141>(v));   // row_half_mirror
  if (Lanes > 8) v = fmaxf(v, dpp_f32<0x140>(v));   // row_mirror
  if (Lanes > 16) {
    v = fmaxf(v, dpp_f32<0x142, 0xa>(v));  // row_bcast15 -> rows 1, 3
    v = fmaxf(v, dpp_f32<0x143, 0xc>(v));  // row_bcast31 -> rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
  }
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// UCT argmax screened in f32 (integer rewards).  Every child's f32 value A_k
// is within E = (1 + |c| sqrt(log N)) 2^-20 of the f64 value V_k that
// mcts.cc:89-100 computes (each f32 step is within 2^-22 relative, the inputs
// n, w < 2^24 convert exactly; solved outcomes are exact;
// tests/test_uct_screen.py).  Let M be the largest A and j the first child
// holding it.  If every other child k has A_k < M - 2E' (E' = 4E) or the same
// (n, w, out) as j -- then V_k == V_j and the lower index j wins the strict
// '>' scan -- then j is the f64 argmax, and it is returned.  Otherwise -1: the
// caller runs the exact f64 argmax.  Child k = l + 64 h is in slot h of lane
// l.  Callers handle unvisited unsolved children (n == 0) first.
__device__ __forceinline__ float uct_screen_value(const Node<int32_t>& c, bool in, int cp,
                                                  float lf, float cf) {
  const float r = __builtin_amdgcn_rcpf(static_cast<float>(c.n));  // 1 ulp
  float a = static_cast<float>(c.w) * r + cf * __builtin_amdgcn_sqrtf(lf * r);  // 1 ulp
  const float o = static_cast<float>(cp == 0 ? c.out : -c.out);
  a = c.out != kUnsolved ? o : a;
  return in ? a : -__builtin_huge_valf();
}
template <int Lanes, bool TwoSlots>
__device__ __forceinline__ int uct_argmax_screen(const Node<int32_t>& c0, bool in0,
                                                 const Node<int32_t>& c1, bool in1, int cp,
                                                 double logN, double uct_c) {
  const float lf = static_cast<float>(logN);
  const float cf = static_cast<float>(uct_c);
  const float a0 = uct_screen_value(c0, in0, cp, lf, cf);
  const float a1 = TwoSlots ? uct_screen_value(c1, in1, cp, lf, cf) : -__builtin_huge_valf();
  const float m = wave_max_f32<Lanes>(TwoSlots ? fmaxf(a0, a1) : a0);
  const uint64_t t0 = ballot(a0 == m);
  const int j = t0 ? static_cast<int>(ctz64(t0)) : 64 + static_cast<int>(ctz64(ballot(a1 == m)));
  const bool hi = TwoSlots && j >= 64;  // wave-uniform
  const int src = j & 63;
  const int32_t nj = rli(hi ? c1.n : c0.n, src), wj = rli(hi ? c1.w : c0.w, src);
  const int32_t oj = rli(static_cast<int32_t>(hi ? c1.out : c0.out), src);
  const float e2 = (1.0f + fabsf(cf) * __builtin_sqrtf(fmaxf(lf, 0.0f))) * 0x1p-17f;  // 2E'
  const float lo = m - e2;
  const bool same0 = c0.n == nj && c0.w == wj && static_cast<int32_t>(c0.out) == oj;
  bool near = in0 && a0 >= lo && !same0;
  if (TwoSlots) {
    const bool same1 = c1.n == nj && c1.w == wj && static_cast<int32_t>(c1.out) == oj;
    near = near || (in1 && a1 >= lo && !same1);
  }
  return ballot(near) ? -1 : j;
}

// Order-preserving int32 key of a non-NaN f32 (an involution: the same map
// decodes), so the screen's wave maximum runs on integers and DPP folds into
// v_max_i32 (no canonicalising v_max_f32 per step).  -0 and +0 get different
// keys; the near-tie test below still sends any such pair to the exact path.
__device__ __forceinline__ int32_t f32_key(float a) {
  const int32_t b = __float_as_int(a);
  return b ^ ((b >> 31) & 0x7FFFFFFF);
}
__device__ __forceinline__ float key_f32(int32_t k) {
  return __int_as_float(k ^ ((k >> 31) & 0x7FFFFFFF));
}
template <int Ctrl, int RowMask = 0xf>
__device__ __forceinline__ int32_t dpp_max_i32(int32_t v) {
  return max(v, __builtin_amdgcn_update_dpp(static_cast<int32_t>(0x80000000u), v, Ctrl,
                                            RowMask, 0xf, false));
}
template <int Lanes>
__device__ __forceinline__ int32_t wave_max_key(int32_t v) {
  v = dpp_max_i32<0xB1>(v);                   // quad_perm [1,0,3,2]
  if (Lanes > 2) v = dpp_max_i32<0x4E>(v);    // quad_perm [2,3,0,1]
  if (Lanes > 4) v = dpp_max_i32<0x141>(v);   // row_half_mirror
  if (Lanes > 8) v = dpp_max_i32<0x140>(v);   // row_mirror
  if (Lanes > 16) {
    v = dpp_max_i32<0x142, 0xa>(v);  // row_bcast15 -> rows 1, 3
    v = dpp_max_i32<0x143, 0xc>(v);  // row_bcast31 -> rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
  }
  return __builtin_amdgcn_readfirstlane(v);
}
// uct_argmax_screen with the parent term lf = log(N) in f32 from v_log_f32
// (within 4 ulp of log(N); tests/test_uct_screen.py bounds the screen with that
// input error), the integer-key maximum and a v_sqrt_f32 band (the band is
// 8E, four times the 2E the argument needs, so its own rounding is immaterial).
template <int Lanes, bool TwoSlots>
__device__ __forceinline__ int uct_argmax_screen_lf(const Node<int32_t>& c0, bool in0,
                                                    const Node<int32_t>& c1, bool in1, int cp,
                                                    float lf, double uct_c) {
  const float cf = static_cast<float>(uct_c);
  const float a0 = uct_screen_value(c0, in0, cp, lf, cf);
  const float a1 = TwoSlots ? uct_screen_value(c1, in1, cp, lf, cf) : -__builtin_huge_valf();
  const int32_t k0 = f32_key(a0), k1 = f32_key(a1);
  const int32_t mk = wave_max_key<Lanes>(TwoSlots ? max(k0, k1) : k0);
  const float e2 = (1.0f + fabsf(cf) * __builtin_amdgcn_sqrtf(lf)) * 0x1p-17f;  // 2E', lf >= 0
  const float lo = key_f32(mk) - e2;
#if OS_SCREEN_BAND
  // The usual case: the maximum is the only child within the band, so no
  // other child is near it and it is the argmax (the lane holding M is always
  // in the band).  One ballot settles it; the identity test below runs only
  // when two or more children share the band.
  {
    const uint64_t b0 = ballot(in0 && a0 >= lo);
    const uint64_t b1 = TwoSlots ? ballot(in1 && a1 >= lo) : 0ull;
    if (popc64(b0) + popc64(b1) == 1) return b0 ? static_cast<int>(ctz64(b0)) : 64 + static_cast<int>(ctz64(b1));
  }
#endif
  const uint64_t t0 = ballot(k0 == mk);
  const int j = t0 ? static_cast<int>(ctz64(t0)) : 64 + static_cast<int>(ctz64(ballot(k1 == mk)));
  const bool hi = TwoSlots && j >= 64;  // wave-uniform
  const int src = j & 63;
  const int32_t nj = rli(hi ? c1.n : c0.n, src), wj = rli(hi ? c1.w : c0.w, src);
  const int32_t oj = rli(static_cast<int32_t>(hi ? c1.out : c0.out), src);
  const bool same0 = c0.n == nj && c0.w == wj && static_cast<int32_t>(c0.out) == oj;
  bool near = in0 && a0 >= lo && !same0;
  if (TwoSlots) {
    const bool same1 = c1.n == nj && c1.w == wj && static_cast<int32_t>(c1.out) == oj;
    near = near || (in1 && a1 >= lo && !same1);
  }
  return ballot(near) ? -1 : j;
}
// log(n) in f32 for the screen: v_log_f32 (log2, 1 ulp) times ln 2.
__device__ __forceinline__ float screen_log(int32_t n) {
  return __builtin_amdgcn_logf(static_cast<float>(n)) * 0x1.62e430p-1f;
}

// Games whose rollout draws use WaveMt::uniform_small (|LegalActions| <= 7,
// C++ policy): the evaluator stream then needs use7 = 1.
template <class G>
struct SmallAbsl {
  static constexpr bool value = false;
};
template <>
struct SmallAbsl<ConnectFour> {
  static constexpr bool value = true;
};

// Lanes that can hold a child of a node (compile-time, per game): the UCT
// argmax only reduces over those; TwoSlots when a node can have > 64 children.
template <class G>
struct WaveWidth {
  static constexpr int kLanes = 64;
  static constexpr bool kTwoSlots = true;
};
template <>
struct WaveWidth<TicTacToe> {  // <= 9 children
  static constexpr int kLanes = 16;
  static constexpr bool kTwoSlots = false;
};
template <>
struct WaveWidth<ConnectFour> {  // <= 7 children
  static constexpr int kLanes = 8;
  static constexpr bool kTwoSlots = false;
};

// SearchNode::UCTValue (mcts.cc:89-100) for the player to move at the parent,
// for lane-distributed children, computed on every lane and
// selected (no exec-mask branches: the scalar unit is the wave kernels'
// binding pipe, and a masked-off f64 division costs the VALU the same cycles).
// Lanes outside the children score -inf.  A zero count divides to inf / NaN
// only in lanes whose value is then discarded.
template <class R>
__device__ __forceinline__ double uct_value_sel(const Node<R>& c, bool in, int cp, double logN,
                                                double uct_c) {
  const double dn = static_cast<double>(c.n);
  const double u = static_cast<double>(c.w) / dn + uct_c * __builtin_sqrt(logN / dn);
  const double o = outcome_for(c.out, cp);
  double v = c.n == 0 ? __builtin_huge_val() : u;
  v = c.out != kUnsolved ? o : v;
  return in ? v : -__builtin_huge_val();
}
// SearchNode::PUCTValue (mcts.cc:102-111) with the uniform prior, likewise
// selected on every lane.
template <class R>
__device__ __forceinline__ double puct_value_sel(const Node<R>& c, bool in, int cp,
                                                 double sqrtN, double cprior) {
  double v = puct_unsolved(static_cast<double>(c.w), c.n, cprior, sqrtN);
  v = c.out != kUnsolved ? outcome_for(c.out, cp) : v;
  return in ? v : -__builtin_huge_val();
}

// Set bits of the wave-uniform mask m in the lanes below this one.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

// Inclusive prefix (OR / sum) over the 16 lanes of each DPP row; lanes that
// would read across the row boundary read 0 (bound_ctrl), the identity.
template <int Shift>
__device__ __forceinline__ uint32_t row_shr(uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x110 + Shift, 0xf, 0xf, true));
}
__device__ __forceinline__ uint32_t row_scan_add(uint32_t v) {
  v += row_shr<1>(v);
  v += row_shr<2>(v);
  v += row_shr<4>(v);
  v += row_shr<8>(v);
  return v;
}
// OR over the lanes j <= i of the same parity as i (stride-2 prefix).
__device__ __forceinline__ uint64_t row_scan_or_stride2(uint64_t v) {
  uint32_t lo = static_cast<uint32_t>(v), hi = static_cast<uint32_t>(v >> 32);
  lo |= row_shr<2>(lo);
  hi |= row_shr<2>(hi);
  lo |= row_shr<4>(lo);
  hi |= row_shr<4>(hi);
  lo |= row_shr<8>(lo);
  hi |= row_shr<8>(hi);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// connect_four random playout (mcts.cc:46-55), lane-parallel and speculative.
// Between two column-fill events the legal set -- hence n = |LegalActions|
// and the ascending action list -- does not change, so the absl draws of the
// next K moves are known up front (WaveMt::small7 holds absl::Uniform(0, n)
// for every word pair of the window).  Lane i plays move i of such a run:
//   column   = legal[k_i(n)]
//   row      = height of that column + earlier run moves into it (prefix sum
//              of one-hot column nibbles over the lanes)
//   board    = mover's stones + stones of the earlier same-parity lanes
//              (stride-2 prefix OR)
//   terminal = has_four(board) || move 42 (connect_four.cc:98-103)
// The run ends at the first terminal lane, the first lane that fills a
// column (the legal set changes after it), the end of the MT window or 16
// moves (one DPP row); a pair the table cannot answer (window edge, possible
// absl rejection) is drawn by the exact serial path as a 1-move run.  Every
// move, word and outcome is the serial rollout's (tests/test_gpu_parity.py).
//
// Under the numpy policy (RandomState.choice, mcts.py:56-63) a run's draws
// all test their words against the same mask and bound (n is fixed), so the
// run's draws are the window's accepted words in order: one ballot marks
// them, ds_permute sends each accepted word's index to the lane of its rank
// (the others to the top lanes), and move i reads its word from there; the
// stream moves past the last draw taken.  n = 1 draws nothing.
template <int Policy = kPolicyCpp, class C>
__device__ int c4_rollout_lanes(ConnectFour::State s, C& ctx, WaveMt& ev) {
  (void)ctx;
  s = make_uniform(s);
  ev.uniformize();
  const int l = lane_id();
  const int i = l & 15;  // run move index (every row computes the same run)
  // Ascending legal columns as nibbles, and column heights as nibbles.
#if OS_C4_LANE_SETUP
  // Lane c < 7 computes column c's nibbles (height at nibble c; c itself at
  // nibble rank-of-c among the legal columns), one row scan sums them (the
  // nibbles are disjoint) and lane 7 holds the total.
  uint32_t cols, heights;
  {
    const uint32_t c = static_cast<uint32_t>(l & 7);
    const uint64_t occ = s.bb[0] | s.bb[1];
    const bool col = c < 7;
    // every lane counts (lane 7 reads the unused bits above column 6); the
    // select keeps the count free of an exec-mask branch
    const uint32_t hc0 = popc64((occ >> (7 * c)) & 0x3full);
    const uint32_t hc = col ? hc0 : 0u;
    const bool lgl = col && ((s.legal >> c) & 1u);
    const uint32_t rank = static_cast<uint32_t>(__builtin_popcount(s.legal & ((1u << c) - 1u)));
    heights = rl32(row_scan_add(hc << (4 * c)), 7);
    cols = rl32(row_scan_add(lgl ? c << (4 * rank) : 0u), 7);
  }
#else
  uint32_t cols = 0;
  {
    int q = 0;
    for (uint32_t m = s.legal; m; m &= m - 1, ++q) cols |= static_cast<uint32_t>(ctz64(m)) << (4 * q);
  }
  uint32_t heights = 0;
  {
    const uint64_t occ = s.bb[0] | s.bb[1];
    for (int c = 0; c < 7; ++c)
      heights |= static_cast<uint32_t>(popc64((occ >> (7 * c)) & 0x3full)) << (4 * c);
  }
#endif
  int p = s.to_play;
  int moves = s.moves;
  uint32_t legal = s.legal;
  uint64_t b0 = s.bb[0], b1 = s.bb[1];
  for (;;) {
    const int n = popc64(legal);
    int K;
    uint32_t k = 0;
    bool serial = false;
    uint32_t widx = 0;  // numpy: window index of move i's word (lane i)
    if constexpr (Policy == kPolicyCpp) {
      K = (ev.valid - ev.pos) >> 1;
      if (K > 16) K = 16;
      if (K > 42 - moves) K = 42 - moves;
      if (K > 0) {
        const uint32_t pk = static_cast<uint32_t>(
            __builtin_amdgcn_ds_bpermute((ev.pos + 2 * i) << 2, static_cast<int>(ev.pre7)));
        const uint64_t fl = ballot(l < K && (pk >> 31) != 0);
        if (fl) K = ctz64(fl);  // lanes before the first unanswerable pair
        k = (pk >> (3 * (n - 1))) & 7u;
      }
    } else {
      K = 42 - moves < 16 ? 42 - moves : 16;
      if (n > 1) {
        const uint32_t rng = static_cast<uint32_t>(n - 1), m = np_mask(rng);
        const bool a = l >= ev.pos && l < ev.valid && (ev.cur & m) <= rng;
        const uint64_t acc = ballot(a);
        const int avail = popc64(acc);
        if (avail < K) K = avail;
        if (K > 0) {
          const uint32_t r = lanes_below(acc);
          const uint32_t dst = a ? r : 63u - (static_cast<uint32_t>(l) - r);
          const uint32_t wi = static_cast<uint32_t>(
              __builtin_amdgcn_ds_permute(static_cast<int>(dst << 2), l));
          widx = static_cast<uint32_t>(
              __builtin_amdgcn_ds_bpermute(static_cast<int>(i << 2), static_cast<int>(wi)));
          k = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(
                  static_cast<int>(widx << 2), static_cast<int>(ev.cur))) & m;
        }
      }
    }
    if (K == 0) {  // one exact serial draw (refills the window as needed)
      k = Policy == kPolicyCpp ? ev.uniform_small(static_cast<uint32_t>(n))
                               : NpChoice(ev, static_cast<uint32_t>(n));
      K = 1;
      serial = true;
    }
    const uint32_t col = (cols >> (4 * k)) & 15u;
    const uint32_t onehot = 1u << (4 * col);
    const uint32_t incl = row_scan_add(onehot);
    const uint32_t h = ((heights + incl - onehot) >> (4 * col)) & 15u;
    const uint64_t fills = ballot(l < K && h == 5);
    int Kr = K;  // moves of this run
    if (fills) {
      const int f = ctz64(fills) + 1;
      if (f < Kr) Kr = f;
    }
    const uint64_t stones = row_scan_or_stride2(1ull << (7 * col + h));
    const uint64_t mine = ((i & 1) ? (p ? b0 : b1) : (p ? b1 : b0)) | stones;
#if OS_C4_BF_FOUR
    // Branch-free on the lanes (the early-exit form diverges per lane).
    const uint64_t m1 = mine & (mine >> 1), m7 = mine & (mine >> 7);
    const uint64_t m6 = mine & (mine >> 6), m8 = mine & (mine >> 8);
    const bool win = ((m1 & (m1 >> 2)) | (m7 & (m7 >> 14)) | (m6 & (m6 >> 12)) |
                      (m8 & (m8 >> 16))) != 0;
#else
    const bool win = ConnectFour::has_four(mine);
#endif
    const uint64_t term = ballot(l < Kr && (win || moves + i + 1 == 42));
    // stream offset in the window after move t's draw (not in serial runs)
    auto advance = [&](int t) {
      int np = ev.pos + 2 * (t + 1);
      if constexpr (Policy != kPolicyCpp) np = n > 1 ? static_cast<int>(rl32(widx, t)) + 1 : ev.pos;
      ev.words.add(np - ev.pos);
      ev.pos = np;
    };
    if (term) {
      const int t = ctz64(term);
      if (!serial) advance(t);
      const uint64_t wins = ballot(win);
      const int winner = p ^ (t & 1);
      return ((wins >> t) & 1) ? (winner == 0 ? 1 : -1) : 0;
    }
    if (!serial) advance(Kr - 1);
    const int last = Kr - 1;
    const uint64_t blast = rl64(mine, last);
    const int plast = p ^ (last & 1);
    if (Kr >= 2) {
      const uint64_t bprev = rl64(mine, last - 1);
      b0 = plast == 0 ? blast : bprev;
      b1 = plast == 0 ? bprev : blast;
    } else {
      if (plast == 0) b0 = blast;
      else b1 = blast;
    }
    heights += rl32(incl, last);
    if ((fills >> last) & 1) {
      const uint32_t kl = rl32(k, last), cl = rl32(col, last);
      legal &= ~(1u << cl);
      const uint32_t below = kl == 0 ? 0u : (cols & ((1u << (4 * kl)) - 1u));
      cols = below | ((cols >> (4 * (kl + 1))) << (4 * kl));
    }
    p ^= Kr & 1;
    moves += Kr;
  }
}

// Inclusive OR scan over the 64 lanes: the DPP row scan, then row_bcast15 /
// row_bcast31 carry rows 0-1 into rows 1-3 (as wave_max_f64).
__device__ __forceinline__ uint32_t wave_scan_or32(uint32_t v) {
  v |= row_shr<1>(v);
  v |= row_shr<2>(v);
  v |= row_shr<4>(v);
  v |= row_shr<8>(v);
  v |= static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v |= static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
}
__device__ __forceinline__ uint64_t wave_scan_or64(uint64_t v) {
  const uint32_t lo = wave_scan_or32(static_cast<uint32_t>(v));
  const uint32_t hi = wave_scan_or32(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Not a playout return value: the lane-parallel playout declines and the
// exact serial loop runs instead (the stream has not moved).
constexpr int kLanesDecline = 2;

// Pairs of u16 packed in a dword: the two cells a lane holds (cell l in the
// low half, cell l + 64 in the high half) -- v_pk_min_u16 / v_pk_max_u16.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                __builtin_bit_cast(u16x2, b)));
}
// Lanes whose bit is set in the wave-uniform mask m (v_cndmask on an SGPR pair).
__device__ __forceinline__ bool in_mask(uint64_t m) {
  return __builtin_amdgcn_inverse_ballot_w64(m);
}

// Move of the fill: the k-th empty cell (ascending) gets fill time tau.  r
// holds each cell's rank among the empty cells (huge for filled or
// off-board cells), so the move is the cell whose rank is k and the cells
// after it move down one rank -- both are "r > k", since ranks follow cell
// order.  Vector-only: no scalar mask per move.
__device__ __forceinline__ void hex_take(uint32_t& r, uint32_t k, uint32_t tau, uint32_t& t) {
  const bool hit = r == k;
  t = hit ? tau : t;
  r = hit ? 0x40000000u : r - (r > k ? 1u : 0u);
}

// hex random playout (mcts.cc:46-55), lane-parallel.  Hex only ever fills
// empty cells, and on n >= 3 a filled board has exactly one player whose
// stones join their two edges (hex.cc:55-184 labels; no draws), so the serial
// playout is recovered from three data-parallel steps:
//   draws  |LegalActions| before move j is n0 - j whatever was played, so
//          lane j draws absl::Uniform(0, n0 - j) from the word pair at
//          offset 2j (os_rng.h AbslUniform; words past the block come from
//          WaveMt::peek_raw).  A pair absl might reject (P mod 2^64 < n)
//          declines the whole playout to the serial path.
//   fill   move j takes the k_j-th empty cell, ascending: one rank-select per
//          move (mbcnt ranks, ballot) -- the only serial chain; each cell
//          records its fill time tau = j + 1 (0 for stones already placed).
//   end    connection is monotone, so the playout ends at the first move
//          after which some player's stones join both edges: the minimum,
//          over far-edge cells, of the bottleneck time d(c) = min over
//          same-colour paths from the near edge of the largest tau on the
//          path.  d is relaxed for both players at once (neighbours of the
//          other colour are cut) until no lane changes: d = min(d,
//          max(tau, min over the six neighbours)), neighbours fetched with
//          ds_bpermute, both cells of a lane in one packed-u16 dword.
// The winner owns the minimising cell; the stream advances by the 2 (T + 1)
// words the serial playout draws for its T + 1 moves.
//
// hex_fill_end: the fill and end steps, from the draws k0 / k1 of moves l and
// l + 64; returns T + 1, the moves the serial playout plays (0: decline).
__device__ inline int hex_fill_end(const Hex::State& s, const GameCfg& g, B128 empty, int n0,
                                   uint32_t k0, uint32_t k1);

// Draws of a fill playout (every move fills one empty cell, so move j draws
// over n0 - j legal actions whatever was played): k0 / k1 = the draws of moves
// l and l + 64, from the stream at offset q0 (WaveMt::offset; words past the
// block come from peek_raw).  false: decline to the serial playout.
//   C++ (absl::Uniform(0, n), os_rng.h AbslUniform): two words per move, lane
//     j reads the pair at 2j; a pair absl might reject (P mod 2^64 < n)
//     declines.
//   numpy (RandomState.choice, mcts.py:56-63; os_rng.h NpChoice: no word when
//     n = 1, else 32-bit words until (w & mask) <= n - 1): the words taken vary,
//     so the draws are found serially over a 64-word window of tempered words
//     on the lanes -- the accepted word of move j is the first unread lane
//     whose word passes move j's test (one compare and ballot; the mask only
//     halves when n - 1 falls below its top bit) -- and e0 / e1 record the
//     offset (from q0) after each move's draw.
__device__ inline bool fill_draws_cpp(WaveMt& ev, int q0, int n0, uint32_t& k0, uint32_t& k1) {
  const int l = lane_id();
  k0 = k1 = 0;
  bool risky = false;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = l + 64 * h;
    uint32_t k = 0;
    if (j < n0) {
      const uint32_t hi = MtStream::temper(ev.peek_raw(q0 + 2 * j));
      const uint32_t lo = MtStream::temper(ev.peek_raw(q0 + 2 * j + 1));
      const uint32_t m = static_cast<uint32_t>(n0 - j);
      if ((m & (m - 1u)) == 0) {
        k = lo & (m - 1u);
      } else {
        const uint64_t b = static_cast<uint64_t>(lo) * m;
        const uint64_t mid = static_cast<uint64_t>(hi) * m + (b >> 32);
        risky |= static_cast<uint32_t>(mid) == 0 && static_cast<uint32_t>(b) < m;
        k = static_cast<uint32_t>(mid >> 32);
      }
    }
    if (h == 0) k0 = k;
    else k1 = k;
  }
  return !ballot(risky);
}

__device__ inline bool fill_draws_np(WaveMt& ev, int q0, int n0, uint32_t& k0, uint32_t& k1,
                                     uint32_t& e0, uint32_t& e1) {
  const int l = lane_id();
  const int qmax = kMtN + (kMtN - kMtM) + (kMtN - kMtM);  // peek_raw's reach
  int wb = 0;  // window base, relative to q0
  auto load = [&](int b) {
    const int q = q0 + b + l;
    return MtStream::temper(ev.peek_raw(q < qmax ? q : qmax - 1));
  };
  uint32_t win = load(0);
  uint32_t rng = static_cast<uint32_t>(n0 - 1), mask = np_mask(rng);
  uint32_t v = win & mask;
  uint64_t avail = ~0ull;  // unread words of the window
  int cur = 0;             // next unread word, relative to q0
  k0 = k1 = e0 = e1 = 0;
  bool fail = false;
  auto draw = [&]() -> uint32_t {
    if (rng == 0) return 0u;  // one legal action: no word
    if (rng <= (mask >> 1)) {
      mask >>= 1;
      v = win & mask;
    }
    uint64_t ok = ballot(v <= rng) & avail;
    while (!ok) {  // the rest of the window is rejected: the next 64 words
      wb += 64;
      if (q0 + wb + 64 > qmax) {
        fail = true;
        return 0u;
      }
      win = load(wb);
      v = win & mask;
      avail = ~0ull;
      ok = ballot(v <= rng);
    }
    const int idx = ctz64(ok);
    const uint64_t low = ok & (0ull - ok);
    avail &= ~((low << 1) - 1ull);  // words up to idx are read (idx = 63: all)
    cur = wb + idx + 1;
    return rl32(v, idx);
  };
  const int nlo = n0 < 64 ? n0 : 64;
  for (int j = 0; j < nlo; ++j, --rng) {
    const uint32_t k = draw();
    if (fail) return false;
    k0 = wl32(k, j, k0);
    e0 = wl32(static_cast<uint32_t>(cur), j, e0);
  }
  for (int j = 64; j < n0; ++j, --rng) {
    const uint32_t k = draw();
    if (fail) return false;
    k1 = wl32(k, j - 64, k1);
    e1 = wl32(static_cast<uint32_t>(cur), j - 64, e1);
  }
  return true;
}

// Moves the stream past the first `tend` moves' draws of a fill playout.
template <int Policy>
__device__ inline void fill_seek(WaveMt& ev, int q0, int tend, uint32_t e0, uint32_t e1) {
  const int used = Policy == kPolicyCpp
                       ? 2 * tend
                       : static_cast<int>(tend <= 64 ? rl32(e0, tend - 1) : rl32(e1, tend - 65));
  ev.seek(q0 + used);
  ev.words.add(used);
}

// hex under either policy (the numpy form: python/algorithms/mcts.py's
// RandomState.choice playouts).
template <int Policy, class C>
__device__ int hex_rollout_lanes(Hex::State s, const GameCfg& g, C& ctx, WaveMt& ev) {
  (void)ctx;
  s = make_uniform(s);
  ev.uniformize();
  if (Hex::terminal(s, g)) return s.result;
  const B128 empty = g.board & ~(s.st[0] | s.st[1]);
  const int n0 = popc(empty);
  const int q0 = ev.offset();
  uint32_t k0, k1, e0 = 0, e1 = 0;
  const bool ok = Policy == kPolicyCpp ? fill_draws_cpp(ev, q0, n0, k0, k1)
                                       : fill_draws_np(ev, q0, n0, k0, k1, e0, e1);
  if (!ok) return kLanesDecline;
  const int tend = hex_fill_end(s, g, empty, n0, k0, k1);
  if (tend == 0) return kLanesDecline;  // unreachable
  const int winner = s.to_play ^ ((tend - 1) & 1);  // the mover of the last stone
  fill_seek<Policy>(ev, q0, tend, e0, e1);
  return winner == 0 ? 1 : -1;
}

// tic_tac_toe random playout, the same way: every move fills an empty cell,
// so the draws, then the fill times (cell c = lane c), then the end -- the
// earliest time a line's three cells hold one player's stones (the latest of
// their fill times; a line already complete would have ended the game), or
// the full board (a draw, tic_tac_toe.cc:80-150).
constexpr uint32_t kTttLineA = 0x20210630u, kTttLineB = 0x44543741u, kTttLineC = 0x68876852u;
template <int Policy>
__device__ int ttt_rollout_lanes(TicTacToe::State s, const GameCfg& g, WaveMt& ev) {
  s = make_uniform(s);
  ev.uniformize();
  if (TicTacToe::terminal(s, g)) return s.winner == 0 ? 1 : (s.winner == 1 ? -1 : 0);
  const int l = lane_id();
  const uint32_t b0 = s.b[0], b1 = s.b[1];
  const uint32_t empty = 0x1FFu & ~(b0 | b1);
  const int n0 = __builtin_popcount(empty);
  const int q0 = ev.offset();
  uint32_t k0, k1, e0 = 0, e1 = 0;
  const bool ok = Policy == kPolicyCpp ? fill_draws_cpp(ev, q0, n0, k0, k1)
                                       : fill_draws_np(ev, q0, n0, k0, k1, e0, e1);
  if (!ok) return kLanesDecline;
  // fill times (0: a stone of the state) and owners of cell l < 9
  uint32_t t = 0;
  const bool on = l < 9;
  uint32_t r = (on && ((empty >> l) & 1u)) ? lanes_below(empty) : 0x40000000u;
  for (int j = 0; j < n0; ++j) hex_take(r, rl32(k0, j), static_cast<uint32_t>(j + 1), t);
  const int p = s.to_play;
  const uint32_t own = t ? static_cast<uint32_t>(p ^ static_cast<int>((t - 1) & 1))
                         : (on ? ((b1 >> l) & 1u) : 0u);
  const uint32_t cell = t | (own << 8);  // fill time | owner << 8
  // line l < 8: cells (A, B, C) from nibble l of the tables
  const int sh = 4 * (l & 7);
  auto at = [&](uint32_t tab) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(
        static_cast<int>(((tab >> sh) & 15u) << 2), static_cast<int>(cell)));
  };
  const uint32_t ca = at(kTttLineA), cb = at(kTttLineB), cc = at(kTttLineC);
  const bool same = ((ca ^ cb) >> 8) == 0 && ((ca ^ cc) >> 8) == 0;
  const uint32_t ta = ca & 0xFFu, tb = cb & 0xFFu, tc = cc & 0xFFu;
  uint32_t done = ta > tb ? ta : tb;
  done = done > tc ? done : tc;
  uint32_t v = (l < 8 && same) ? done : 0xFFu;  // lines of mixed owners never end it
  for (int off = 4; off >= 1; off >>= 1) {      // minimum over lanes 0..7
    const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), off));
    v = o < v ? o : v;
  }
  const uint32_t tw = rl32(v, 0);
  const int tend = tw <= static_cast<uint32_t>(n0) ? static_cast<int>(tw) : n0;
  fill_seek<Policy>(ev, q0, tend, e0, e1);
  if (tw > static_cast<uint32_t>(n0)) return 0;  // full board, no line
  const int winner = p ^ ((tend - 1) & 1);
  return winner == 0 ? 1 : -1;
}

__device__ inline int hex_fill_end(const Hex::State& s, const GameCfg& g, B128 empty, int n0,
                                   uint32_t k0, uint32_t k1) {
  const int l = lane_id();
  const int n = g.rows;
  // Fill times of cells l (t0) and l + 64 (t1); ranks among the empty cells.
  uint32_t t0 = 0, t1 = 0;
  uint32_t r0 = ((empty.lo >> l) & 1) ? lanes_below(empty.lo) : 0x40000000u;
  uint32_t r1 = ((empty.hi >> l) & 1) ? lanes_below(empty.hi) + popc64(empty.lo) : 0x40000000u;
  const int nlo = n0 < 64 ? n0 : 64;
#if OS_AB_HEX == 2  // timing A/B only: fill order = cell order
  t0 = l < n0 ? l + 1 : 0;
  t1 = l + 64 < n0 ? l + 65 : 0;
  if (n0 < 0)
#endif
  for (int j = 0; j < nlo; ++j) {
    const uint32_t k = rl32(k0, j);
    hex_take(r0, k, static_cast<uint32_t>(j + 1), t0);
    hex_take(r1, k, static_cast<uint32_t>(j + 1), t1);
  }
#if OS_AB_HEX == 2
  if (n0 < 0)
#endif
  for (int j = 64; j < n0; ++j) {
    const uint32_t k = rl32(k1, j - 64);
    hex_take(r0, k, static_cast<uint32_t>(j + 1), t0);
    hex_take(r1, k, static_cast<uint32_t>(j + 1), t1);
  }
  // Per cell: colour (stones already placed by the state, move j by the
  // player to move ^ (j & 1)), near / far edge (hex.cc:55-90: black north row
  // -> south row, white west column -> east column), column.
  const int nn = n * n;
  const int p = s.to_play;
  uint32_t tt = 0, dd = 0, far = 0, own = 0;
  int qa = 0, qb = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = l + 64 * h;
    const uint32_t t = h ? t1 : t0;
    const bool on = c < nn;
    const int q = on ? c % n : 0;
    const int r = on ? c / n : 0;
    const uint64_t w1 = h ? s.st[1].hi : s.st[1].lo;
    const int o = t ? (p ^ static_cast<int>((t - 1) & 1)) : static_cast<int>((w1 >> l) & 1);
    const bool nearE = on && (o == 0 ? r == 0 : q == 0);
    const bool farE = on && (o == 0 ? r == n - 1 : q == n - 1);
    const uint32_t tv = on ? t : 0xFFFFu;
    tt |= tv << (16 * h);
    dd |= (nearE ? tv : 0xFFFFu) << (16 * h);
    far |= (farE ? 0u : 0xFFFFu) << (16 * h);
    own |= static_cast<uint32_t>(o) << (16 * h);
    if (h) qb = q;
    else qa = q;
  }
  // The six neighbours (hex.cc:206-222), as lane offsets d: the source lane
  // is (l + d) & 63; the half and the cut (off the board, a row wrap, or the
  // other colour) are per lane and fixed for the whole relaxation.
  const int dl[6] = {-n, -n + 1, -1, 1, n - 1, n};
  int addr[6];
  uint32_t sel[6], cut[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int d = dl[i];
    const int x = l + d;
    addr[i] = (x & 63) << 2;
    // byte selector for v_perm_b32(r, r, sel): low half <- r.hi if x >= 64,
    // high half <- r.lo if x < 0.
    const uint32_t slo = x >= 64 ? 0x0302u : 0x0100u;
    const uint32_t shi = x < 0 ? 0x0100u : 0x0302u;
    sel[i] = slo | (shi << 16);
    const bool wrap_r = (i == 1 || i == 3);  // +col: cut on the last column
    const bool wrap_l = (i == 2 || i == 4);  // -col: cut on the first column
    const int ca = l + d, cb = l + 64 + d;
    const bool xa = ca < 0 || ca >= nn || (wrap_r && qa == n - 1) || (wrap_l && qa == 0);
    const bool xb = cb < 0 || cb >= nn || (wrap_r && qb == n - 1) || (wrap_l && qb == 0);
    const uint32_t r = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(addr[i], static_cast<int>(own)));
    const uint32_t diff = __builtin_amdgcn_perm(r, r, sel[i]) ^ own;  // 0 / 1 per half
    cut[i] = (diff * 0xFFFFu) | (xa ? 0xFFFFu : 0u) | (xb ? 0xFFFF0000u : 0u);
  }
#if OS_AB_HEX == 1  // timing A/B only: no relaxation
  if (n0 < 0)
#endif
  for (;;) {
    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const uint32_t r = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(addr[i], static_cast<int>(dd)));
      m = pk_min16(m, __builtin_amdgcn_perm(r, r, sel[i]) | cut[i]);
    }
    const uint32_t nd = pk_min16(dd, pk_max16(tt, m));
    const bool changed = nd != dd;
    dd = nd;
    if (!ballot(changed)) break;
  }
  // End: the smallest d on a far-edge cell (the loser has none finite).
  const uint32_t fv = dd | far;
  uint32_t v = pk_min16(fv, fv >> 16) & 0xFFFFu;
  for (int off = 32; off >= 1; off >>= 1) {
    const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), off));
    v = o < v ? o : v;
  }
  const uint32_t tend = rl32(v, 0);
  if (tend == 0 || tend > static_cast<uint32_t>(n0)) return 0;  // unreachable
  return static_cast<int>(tend);
}

// pig random playout (mcts.cc:42-71 / mcts.py:56-67) on the wave.  The
// serial playout, run wave-uniformly, spent ~100 scalar and vector
// instructions per move on the generic n-player state machine (every score
// updated, every player tested for a win, f64 chance sampling on the vector
// unit feeding scalar branches).  Here:
//   * each 64-word window of the stream is decoded once on the lanes: lane i
//     holds, for words (i, i + 1), the chance outcome that a chance node
//     drawing at word i would sample (SampleAction over absl::Uniform(0, 1)
//     under the C++ policy, RandomState.choice(p=) under numpy; os_rng.h) and
//     the roll / stop bit a two-action decision drawing there would take
//     (absl: the low word's bit; numpy: the word's bit);
//   * the move loop keeps the turn in scalars -- turn player, turn total,
//     that player's score, the move count -- with the scores on the lanes
//     (lane p = player p, read once per turn): a decision reads one packed
//     lane value, a stop writes one lane, and only the stopping player can
//     have reached the winning score (pig.cc:180-223: the others have not
//     changed since the last test).
// Words drawn per move are those of the serial playout: decisions 2 (absl,
// either action count) or 1 / 0 (numpy, two / one action), chance nodes 2.
template <int Policy, class PG = Pig>
__device__ int pig_rollout_wave(typename PG::State s, const GameCfg& g, WaveMt& ev) {
  s = make_uniform(s);
  ev.uniformize();
  NoCtx nctx;
  if (PG::terminal(s, g)) return PG::ret0(s, g, nctx);
  const int l = lane_id();
  uint32_t sc = 0;  // lane p: score of player p
#pragma unroll
  for (int i = 0; i < PG::kMaxPlayers; ++i) sc = l == i ? static_cast<uint32_t>(s.score[i]) : sc;
  const int win = g.pig_win, hz = g.pig_horizon, np = g.pig_players, dice = g.pig_dice;
  const double p = 1.0 / dice;  // PG::chance_prob
  int tp = s.turn_player, tt = s.turn_total, moves = s.moves;
  bool at_chance = s.cur < 0;
  int cs = static_cast<int>(rl32(sc, tp));
  int wb = ev.offset();  // stream offset of the window's word 0 (current block)
  int c = 0;             // cursor in the window
  int used = 0;          // words drawn
  uint32_t pk = 0;       // per lane: chance outcome | decision bit << 8
  auto load = [&]() {
    const uint32_t w0 = MtStream::temper(ev.peek_raw(wb + l));
    const uint32_t w1 = MtStream::temper(ev.peek_raw(wb + l + 1));
    int k;
    uint32_t bit;
    if (Policy == kPolicyCpp) {
      uint64_t bits = (static_cast<uint64_t>(w0) << 32) | w1;  // AbslUniformDouble01
      double u = 0.0;
      if (bits != 0) {
        const int clz = __clzll(static_cast<long long>(bits));
        bits <<= clz;
        const uint64_t val = (static_cast<uint64_t>(1022 - clz) << 52) |
                             ((bits >> 11) & ((1ull << 52) - 1));
        __builtin_memcpy(&u, &val, 8);
      }
      k = SampleEquiprobable(dice, p, u);
      bit = w1 & 1u;  // AbslUniform(2): the second word's low bit
    } else {
      const double u = ((w0 >> 5) * 67108864.0 + (w1 >> 6)) / 9007199254740992.0;
      double last = 0.0, acc = 0.0;  // NpChoiceEquiprobable
      for (int j = 0; j < dice; ++j) last = acc = acc + p;
      k = 0;
      acc = 0.0;
      for (int j = 0; j < dice; ++j) {
        acc = acc + p;
        k += (acc / last <= u) ? 1 : 0;
      }
      bit = w0 & 1u;  // NpChoice(2): mask 1, never rejected
    }
    pk = static_cast<uint32_t>(k) | (bit << 8);
  };
  auto need = [&](int n) {  // the next n words must lie in the window
    if (c + n <= 64) return;
    wb += c;
    c = 0;
    if (wb >= kMtN) {  // the window left the block: twist it (seek), rebase
      ev.seek(wb);
      wb -= kMtN;
    }
    load();
  };
  load();
  for (;;) {
    if (moves >= hz) break;  // terminal (a winner ends the loop where it is made)
    if (!at_chance) {
      const bool only_stop = cs + tt >= win;  // PG::legal: stop alone
      const int nw = Policy == kPolicyCpp ? 2 : (only_stop ? 0 : 1);
      need(nw + 2);  // the decision's words and the chance pair a roll draws next
      const uint32_t pd = rl32(pk, c), pc = rl32(pk, c + nw);
      const int a = only_stop ? 1 : static_cast<int>((pd >> 8) & 1u);
      c += nw;
      used += nw;
      moves++;
      if (a == 0) {  // roll: the chance node follows in the same step
        if (moves >= hz) {
          at_chance = true;
          break;
        }
        const int o = static_cast<int>(pc & 0xffu) + 1;  // ChanceOutcomes()[k]: k + 1
        c += 2;
        used += 2;
        if (o == 1) {  // pig.cc:208-213
          tt = 0;
          tp = tp + 1 < np ? tp + 1 : 0;
          cs = static_cast<int>(rl32(sc, tp));
        } else {
          tt += o + 1;
        }
        continue;
      }
      cs += tt;  // stop: bank the turn total
      sc = l == tp ? static_cast<uint32_t>(cs) : sc;
      tt = 0;
      tp = tp + 1 < np ? tp + 1 : 0;
      if (cs >= win) break;
      cs = static_cast<int>(rl32(sc, tp));
    } else {
      need(2);
      const int a = static_cast<int>(rl32(pk, c) & 0xffu) + 1;  // ChanceOutcomes()[k]: k + 1
      c += 2;
      used += 2;
      at_chance = false;
      if (a == 1) {  // pig.cc:208-213
        tt = 0;
        tp = tp + 1 < np ? tp + 1 : 0;
        cs = static_cast<int>(rl32(sc, tp));
      } else {
        tt += a + 1;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < PG::kMaxPlayers; ++i) s.score[i] = static_cast<int32_t>(rl32(sc, i));
  s.turn_total = tt;
  s.turn_player = tp;
  s.cur = at_chance ? -1 : tp;
  s.moves = moves;
  ev.seek(wb + c);
  ev.words.add(used);
  return PG::ret0(s, g, nctx);
}

// Inclusive sum over the 64 lanes (the DPP row scan, then the row_bcast15 /
// row_bcast31 carries, as wave_scan_or32).
__device__ __forceinline__ uint32_t wave_scan_add32(uint32_t v) {
  v += row_shr<1>(v);
  v += row_shr<2>(v);
  v += row_shr<4>(v);
  v += row_shr<8>(v);
  v += static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v += static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
}

// Maps of a 4-state automaton, 2 bits per state (state x -> (f >> 2x) & 3).
constexpr uint32_t kMap4Id = 0xE4u;  // identity: 3 2 1 0
__device__ __forceinline__ uint32_t map4_apply(uint32_t f, uint32_t x) { return (f >> (2 * x)) & 3u; }
// g after f: x -> g(f(x)).
__device__ __forceinline__ uint32_t map4_then(uint32_t f, uint32_t g) {
  return map4_apply(g, map4_apply(f, 0)) | (map4_apply(g, map4_apply(f, 1)) << 2) |
         (map4_apply(g, map4_apply(f, 2)) << 4) | (map4_apply(g, map4_apply(f, 3)) << 6);
}
template <int Ctrl, int RowMask>
__device__ __forceinline__ uint32_t map4_from(uint32_t f) {  // a missing source is the identity
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(kMap4Id),
                                                           static_cast<int>(f), Ctrl, RowMask,
                                                           0xf, false));
}
// Inclusive scan of maps in lane order: lane l ends with f_l o ... o f_0.
__device__ __forceinline__ uint32_t wave_scan_map4(uint32_t f) {
  f = map4_then(map4_from<0x111, 0xf>(f), f);  // row_shr:1
  f = map4_then(map4_from<0x112, 0xf>(f), f);  // row_shr:2
  f = map4_then(map4_from<0x114, 0xf>(f), f);  // row_shr:4
  f = map4_then(map4_from<0x118, 0xf>(f), f);  // row_shr:8
  f = map4_then(map4_from<0x142, 0xa>(f), f);  // row_bcast15 -> rows 1, 3
  f = map4_then(map4_from<0x143, 0xc>(f), f);  // row_bcast31 -> rows 2, 3
  return f;
}

// pig random playout (mcts.cc:46-71, pig.cc:187-213) a window of 64 stream
// words at a time, with the turn walked per TURN instead of per node.  What a
// word is for depends only on the words before it, never on the scores: a
// decision draws one word under numpy (RandomState.choice(2)) or two under
// the C++ policy (absl::Uniform(rng, 0u, n)); a roll leads to a chance node
// (SampleAction: two words), a stop or a chance outcome back to a decision.
// The word roles form a 4-state automaton (C++: decision word 1 / 2, chance
// word 1 / 2; numpy: decision, chance 1 / 2), so lane l finds its word's role
// from the start role by a wave scan over the per-lane transition maps.
// Node effects sit at the node's first word: a stop or a 1 ends the turn,
// other outcomes add outcome + 1 to the turn total (pig.cc:211), so turn
// totals are a segmented prefix sum of the lanes' gains, and the scalar unit
// walks the window's turns with one ballot each: the first decision whose
// player reaches win_score by stopping (LegalActions = {stop}: the game ends
// there; numpy then draws nothing), the horizon (the first node with
// total_moves >= horizon), otherwise the turn's bank or bust.  The same
// words, moves and outcomes as the serial walk (pig_rollout_wave).
#ifndef OS_PIG_PAR2
#define OS_PIG_PAR2 1  // A/B knob: 0 = two players walk the turns like n players
#endif
template <int Policy, class PG = Pig>
__device__ int pig_rollout_turns(typename PG::State s, const GameCfg& g, WaveMt& ev) {
  s = make_uniform(s);
  ev.uniformize();
  NoCtx nctx;
  if (PG::terminal(s, g)) return PG::ret0(s, g, nctx);
  constexpr bool kCpp = Policy == kPolicyCpp;
  constexpr uint32_t kDec = 0, kChance = 2;  // node-start roles (1: C++ decision word 2; 3: chance word 2)
  const int l = lane_id();
  const uint64_t below = (1ull << l) - 1ull;
  uint32_t sc = 0;  // lane p: score of player p
#pragma unroll
  for (int i = 0; i < PG::kMaxPlayers; ++i) sc = l == i ? static_cast<uint32_t>(s.score[i]) : sc;
  const int win = g.pig_win, hz = g.pig_horizon, np = g.pig_players, dice = g.pig_dice;
  const double p = 1.0 / dice;  // PG::chance_prob
  int tp = s.turn_player, tt = s.turn_total, moves = s.moves;
  uint32_t role0 = s.cur < 0 ? kChance : kDec;  // numpy: role of the window's word 0
  bool chance0 = s.cur < 0;                      // C++: the window's node 0 is a chance node
  // A lane is a node under the C++ policy (two words each: 64 nodes, 128
  // words per window) and a word under numpy (64 words per window).
  constexpr int kWordsPerLane = kCpp ? 2 : 1;
  int wb = ev.offset();  // stream offset of the window's word 0 (current block)
  int used = 0;          // words drawn
  bool chance_end = false;
  for (;;) {
    const uint32_t w0 = MtStream::temper(ev.peek_raw(wb + kWordsPerLane * l));
    const uint32_t w1 = MtStream::temper(ev.peek_raw(wb + kWordsPerLane * l + 1));
    int o;  // chance action 1..dice if this lane starts a chance node
    if (kCpp) {
      uint64_t bits = (static_cast<uint64_t>(w0) << 32) | w1;  // AbslUniformDouble01
      double u = 0.0;
      if (bits != 0) {
        const int clz = __clzll(static_cast<long long>(bits));
        bits <<= clz;
        const uint64_t val = (static_cast<uint64_t>(1022 - clz) << 52) |
                             ((bits >> 11) & ((1ull << 52) - 1));
        __builtin_memcpy(&u, &val, 8);
      }
      o = SampleEquiprobable(dice, p, u) + 1;
    } else {
      const double u = ((w0 >> 5) * 67108864.0 + (w1 >> 6)) / 9007199254740992.0;
      double last = 0.0, acc = 0.0;  // NpChoiceEquiprobable
      for (int j = 0; j < dice; ++j) last = acc = acc + p;
      int k = 0;
      acc = 0.0;
      for (int j = 0; j < dice; ++j) {
        acc = acc + p;
        k += (acc / last <= u) ? 1 : 0;
      }
      o = k + 1;
    }
    // A decision's action: C++ the low bit of its second word
    // (AbslUniform(2)), numpy the low bit of its word (mask 1, never
    // rejected); 0 = roll.
    const bool stop_here = ((kCpp ? w1 : w0) & 1u) != 0;  // the decision starting here stops
    bool dec, chn;
    uint32_t after = 0;  // numpy: role of the next word
    if (kCpp) {
      // Node types from one ballot: after a node read as a stop the next node
      // is a decision (a stop, and a chance outcome, lead to one), and along
      // a run of roll-reading nodes the types alternate (a roll leads to a
      // chance node, a chance node back to a decision) -- from the last stop
      // below this lane, or from the window's first node.
      const uint64_t m = ballot(stop_here) & below;
      const bool odd = m ? ((l - (63 - static_cast<int>(__clzll(static_cast<long long>(m)))) - 1) & 1)
                         : (l & 1);
      chn = odd != chance0;
      if (m) chn = odd;
      dec = !chn;
    } else {
      // Word roles: a 4-state automaton (decision, -, chance word 1, chance
      // word 2) scanned over the lanes' transition maps.  (Walking the
      // window's stop bits on the scalar unit instead, a few scalar steps per
      // node, was slower: 16.1 -> 19.3 ms per 1000-simulation step,
      // profiles/r06/pig_nodes.)
      const bool own_roll = (w0 & 1u) == 0;
      const uint32_t f = (own_roll ? 2u : 0u) | (1u << 2) | (3u << 4) | (0u << 6);
      const uint32_t F = wave_scan_map4(f);  // role of word l + 1 = F(role0)
      after = map4_apply(F, role0);
      const uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(after), 1));
      const uint32_t role = l == 0 ? role0 : prev;
      dec = role == kDec;
      chn = role == kChance;
    }
    const bool stop = dec && stop_here, bust = chn && o == 1;
    const uint32_t gain = (chn && o != 1) ? static_cast<uint32_t>(o + 1) : 0u;
    const uint64_t endm = ballot(stop || bust);
    const uint64_t dm = ballot(dec);
    const uint32_t P = wave_scan_add32(gain);  // gains up to and including this word
    const int pex = static_cast<int>(P - gain);
    const int mv = moves + static_cast<int>(__builtin_popcountll(dm & below));  // total_moves here
    const uint64_t hzm = ballot((dec || chn) && mv >= hz);
    const int jh = hzm ? static_cast<int>(ctz64(hzm)) : 64;
    int end_words = -1;
    if (np == 2 && OS_PIG_PAR2) {
      // Two players: no walk at all.  Per word: the turns ended before it
      // (mbcnt of the ends), its turn's first word (the last end below it),
      // hence its turn total (gains since that word, one bpermute) and its
      // turn's player (tp flipped per turn); a stop banks its turn total, and
      // each player's banks are one prefix sum, so every decision knows its
      // player's score and the first one that can win by stopping is a
      // ballot away, as is the horizon.
      const uint64_t eb = endm & below;
      const int tix = static_cast<int>(__builtin_popcountll(eb));
      const int seg0 = eb ? 64 - static_cast<int>(__clzll(static_cast<long long>(eb))) : 0;
      const int pstart = __shfl(pex, seg0);
      const int ttj = (tix == 0 ? tt : 0) + pex - pstart;  // turn total before this word
      const int pj = tp ^ (tix & 1);                        // its turn's player
      const uint32_t bank = stop ? static_cast<uint32_t>(ttj) : 0u;
      const uint32_t b0 = pj == 0 ? bank : 0u, b1 = bank - b0;
      const uint32_t S0 = wave_scan_add32(b0), S1 = wave_scan_add32(b1);
      const int E0 = static_cast<int>(S0 - b0), E1 = static_cast<int>(S1 - b1);
      const int sc0 = static_cast<int>(rl32(sc, 0)), sc1 = static_cast<int>(rl32(sc, 1));
      const int csj = pj == 0 ? sc0 + E0 : sc1 + E1;  // its player's banked score
      const uint64_t wm = ballot(dec && csj + ttj >= win);
      const int jw = wm ? static_cast<int>(ctz64(wm)) : 64;
      int n0, n1;
      if (jw < 64 && jw < jh) {  // only stop is legal: bank and win (pig.cc:151-152, 193-199)
        const int p = rli(pj, jw), t = rli(ttj, jw);
        n0 = sc0 + rli(E0, jw) + (p == 0 ? t : 0);
        n1 = sc1 + rli(E1, jw) + (p == 1 ? t : 0);
        tt = 0;
        tp = p ^ 1;
        moves = rli(mv, jw) + 1;
        end_words = kWordsPerLane * jw + (kCpp ? 2 : 0);
        chance_end = false;
      } else if (jh < 64) {  // total_moves reached the horizon before node jh
        n0 = sc0 + rli(E0, jh);
        n1 = sc1 + rli(E1, jh);
        tt = rli(ttj, jh);
        tp = rli(pj, jh);
        moves = rli(mv, jh);
        end_words = kWordsPerLane * jh;
        chance_end = rli(chn ? 1 : 0, jh) != 0;
      } else {  // the whole window: the state after its last word
        n0 = sc0 + static_cast<int>(rl32(S0, 63));
        n1 = sc1 + static_cast<int>(rl32(S1, 63));
        const bool e63 = (endm >> 63) & 1ull;
        tt = e63 ? 0 : rli(ttj, 63) + static_cast<int>(rl32(gain, 63));
        tp = rli(pj, 63) ^ (e63 ? 1 : 0);
      }
      sc = l == 0 ? static_cast<uint32_t>(n0) : (l == 1 ? static_cast<uint32_t>(n1) : sc);
    } else {
      int pos = 0;
      while (pos < 64) {
        const uint64_t from = ~((1ull << pos) - 1ull);
        const uint64_t e = endm & from;
        const int b = e ? static_cast<int>(ctz64(e)) : 64;  // the turn's last node (its first word)
        const int lim = b < 64 ? b : 63;
        const uint64_t seg = from & (lim == 63 ? ~0ull : ((1ull << (lim + 1)) - 1ull));
        const int pexpos = rli(pex, pos);
        const int cs = rli(static_cast<int32_t>(sc), tp);
        const int need = win - cs - tt + pexpos;  // tt + pex_j - pex_pos >= win - cs
        const uint64_t wm = ballot(dec && pex >= need) & seg;
        const int jw = wm ? static_cast<int>(ctz64(wm)) : 64;
        if (jw <= lim || jh <= lim) {
          if (jw < jh) {  // only stop is legal: bank and win (pig.cc:151-152, 193-199)
            const int bank = cs + tt + rli(pex, jw) - pexpos;
            sc = l == tp ? static_cast<uint32_t>(bank) : sc;
            tt = 0;
            tp = tp + 1 < np ? tp + 1 : 0;
            moves = rli(mv, jw) + 1;
            end_words = kWordsPerLane * jw + (kCpp ? 2 : 0);
            chance_end = false;
          } else {  // total_moves reached the horizon before node jh
            tt += rli(pex, jh) - pexpos;
            moves = rli(mv, jh);
            end_words = kWordsPerLane * jh;
            chance_end = rli(chn ? 1 : 0, jh) != 0;
          }
          break;
        }
        if (b == 64) {  // the turn goes on into the next window
          tt += static_cast<int>(rl32(P, 63)) - pexpos;
          break;
        }
        if (rli(dec ? 1 : 0, b) != 0) {  // stop: bank
          const int bank = cs + tt + rli(pex, b) - pexpos;
          sc = l == tp ? static_cast<uint32_t>(bank) : sc;
        }
        tt = 0;  // stop or a 1 (pig.cc:193-199, 205-210)
        tp = tp + 1 < np ? tp + 1 : 0;
        pos = b + 1;
      }
    }
    if (end_words >= 0) {
      used += end_words;
      wb += end_words;
      break;
    }
    moves += static_cast<int>(__builtin_popcountll(dm));
    if (kCpp)  // after node 63: a chance node iff it is a decision that rolls
      chance0 = rli((dec && !stop_here) ? 1 : 0, 63) != 0;
    else
      role0 = static_cast<uint32_t>(rli(static_cast<int32_t>(after), 63));
    used += 64 * kWordsPerLane;
    wb += 64 * kWordsPerLane;
    if (wb >= kMtN) {  // the next window starts in the next block: twist, rebase
      ev.seek(wb);
      wb -= kMtN;
    }
  }
#pragma unroll
  for (int i = 0; i < PG::kMaxPlayers; ++i) s.score[i] = static_cast<int32_t>(rl32(sc, i));
  s.turn_total = tt;
  s.turn_player = tp;
  s.cur = chance_end ? -1 : tp;
  s.moves = moves;
  ev.seek(wb);
  ev.words.add(used);
  return PG::ret0(s, g, nctx);
}

// OS_PIG_TURNS: 1 = pig playouts by turns (pig_rollout_turns), 0 = node by
// node (pig_rollout_wave).  A/B knob.
#ifndef OS_PIG_TURNS
#define OS_PIG_TURNS 1
#endif
// OS_AB_PIG_NOROLL (timing-only attribution builds; results are NOT the
// reference's): 1 = every playout returns at once.
#ifndef OS_AB_PIG_NOROLL
#define OS_AB_PIG_NOROLL 0
#endif
template <int Policy, int kMaxP>
struct ChanceRollout<PigT<kMaxP>, Policy, WaveMt> {
  __device__ static int run(const typename PigT<kMaxP>::State& s, const GameCfg& g, NoCtx&,
                            WaveMt& ev) {
#if OS_AB_PIG_NOROLL
    return 0;
#endif
#if OS_PIG_TURNS
    return pig_rollout_turns<Policy, PigT<kMaxP>>(s, g, ev);
#else
    return pig_rollout_wave<Policy, PigT<kMaxP>>(s, g, ev);
#endif
  }
};

// breakthrough random playout (mcts.cc:46-55) with lanes as board squares.
// The legal set changes every move, so the moves stay serial, but the board
// lives in the lanes: lane q holds its square's black / white bit, and the
// move generation (breakthrough.cc:217-256) is per-lane vector work -- each
// lane tests its own piece's left / forward / right targets against the
// occupancy masks (ballots, so they cost no scalar instruction) and counts
// its legal actions.  LegalActions()[k] (ascending: source square, then
// direction) is the highest lane whose count-below (mbcnt of the three
// per-direction ballots) is <= k; its k - count-below picks the direction in
// (left, forward, right) order.  The scalar unit -- the pipe that binds the
// wave kernels -- keeps only the draw (absl or numpy), the chosen move's
// squares and the win test (breakthrough.cc:306-319).
template <int Policy, bool kOneCol, class Rng>
__device__ int bt_rollout_wave(Breakthrough::State s, const GameCfg& g, Rng& ev) {
  s = make_uniform(s);
  ev.uniformize();
  const int q = lane_id();
  const int c = g.cols;
  const int last_row0 = (g.rows - 1) * c;  // first square of black's goal row
  const int col = q % c;
  const bool notcol0 = col != 0, notcollast = col != c - 1;
  // Per-lane square bits, kept as 0 / 1 words.
  uint32_t bk = static_cast<uint32_t>(s.pc[0] >> q) & 1u;
  uint32_t wt = static_cast<uint32_t>(s.pc[1] >> q) & 1u;
  int winner = s.winner;
  if (winner < 0 && (s.pc[0] == 0 || s.pc[1] == 0)) winner = s.pc[0] == 0 ? 1 : 0;
  if (winner >= 0) return winner == 0 ? 1 : -1;
  // One move of player P (compile-time, so the mover's and the opponent's
  // squares, the step direction and the goal test need no per-move select).
  // Returns kMore while the game goes on, else the playout's return.
  constexpr int kMore = 2;
  auto move = [&](auto pc) -> int {
    constexpr int P = decltype(pc)::value;
    uint32_t& mine = P ? wt : bk;
    uint32_t& theirs = P ? bk : wt;
    const uint64_t occ = ballot((bk | wt) != 0);
    const uint64_t eo = ~occ | ballot(theirs != 0);  // empty or opponent
    const int tf = P == 0 ? q + c : q - c;
    const uint32_t fl = mine & notcol0 & static_cast<uint32_t>(eo >> ((tf - 1) & 63));
    const uint32_t ff = mine & static_cast<uint32_t>(~occ >> (tf & 63));
    const uint32_t fr = mine & notcollast & static_cast<uint32_t>(eo >> ((tf + 1) & 63));
    const uint64_t L = ballot(fl & 1u), F = ballot(ff & 1u), R = ballot(fr & 1u);
    uint32_t below = __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(L), 0u);
    below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(L >> 32), below);
    below = __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(F), below);
    below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(F >> 32), below);
    below = __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(R), below);
    below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(R >> 32), below);
    const uint32_t code = (fl & 1u) | ((ff & 1u) << 1) | ((fr & 1u) << 2);
    const uint32_t n = rl32(below + __builtin_popcount(code), 63);
    // The topmost piece always has a diagonal move unless cols == 1, where
    // the reference indexes an empty LegalActions(); end the playout there.
    if (kOneCol && n == 0) return 0;
    const uint32_t k = Policy == kPolicyCpp ? ev.uniform_lanes(n) : NpChoice(ev, n);
    const uint64_t cand = ballot(code != 0 && below <= k);
    const int src = 63 - __builtin_clzll(cand);
    // Every lane works out the move it would make as the source (the
    // (k - below)-th set direction of its code in (left, forward, right)
    // order, its target and whether that reaches the goal row); the scalar
    // unit then reads one packed word from lane src.
    const uint32_t rem = k - below;
    const uint32_t low = code & (0u - code);           // first set direction
    const uint32_t rest = code & ~low;
    const uint32_t second = rest & (0u - rest);
    const uint32_t pick = rem == 0 ? low : (rem == 1 ? second : rest & ~second);
    const int tl = tf + (pick == 1u ? -1 : (pick == 2u ? 0 : 1));
    const bool goal = P == 0 ? tl >= last_row0 : tl < c;
    const uint32_t mv = rl32(static_cast<uint32_t>(tl & 63) | (goal ? 64u : 0u), src);
    const int tgt = static_cast<int>(mv & 63u);
    mine = (mine & (q != src ? 1u : 0u)) | (q == tgt ? 1u : 0u);
    theirs &= q != tgt ? 1u : 0u;
    // Reaching the goal row or capturing every opposing piece wins.
    if ((mv & 64u) || !ballot(theirs != 0)) return P == 0 ? 1 : -1;
    return kMore;
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  int r = s.to_play == 1 ? move(P1{}) : kMore;
  while (r == kMore) {
    r = move(P0{});
    if (r == kMore) r = move(P1{});
  }
  return r;
}

// ---------------------------------------------------------------------------
// go playouts with chain labels on the lanes (RandomRolloutEvaluator::Evaluate,
// mcts.cc:42-71, on go.cc / go_board.cc rules; same moves and the same words
// drawn as GoT::apply in a scalar loop).
//
// Lane l holds the labels of points l and l + 64.  Every stone carries the
// label of its chain, and a chain's label is one of its own stones, so labels
// of live chains are distinct and a chain is ONE compare + ballot
// (`chain(L) & colour`) instead of a flood whose iterations grow with the
// chain's diameter.  Placing a stone relabels the own chains it joins to the
// new point; captured stones keep stale labels, which the colour mask drops
// (a stale label names an empty point, never a live chain's stone).
#ifndef OS_GO_LANES
#define OS_GO_LANES 1
#endif

struct GoLabels {
  int32_t l0, l1;  // per lane: labels of points lane, lane + 64
  // One select on the lanes and one readlane (no branch on the slot).
  // (A select of the slot and one readlane instead of the branch: 1% slower.)
  __device__ int at(int q) const { return q < 64 ? rli(l0, q) : rli(l1, q - 64); }
  __device__ B128 chain(int lab) const { return b128(ballot(l0 == lab), ballot(l1 == lab)); }
  __device__ void relabel(int from, int to) {
    l0 = l0 == from ? to : l0;
    l1 = l1 == from ? to : l1;
  }
  __device__ void set(int q, int lab) {
    const int l = lane_id();
    l0 = q == l ? lab : l0;
    l1 = q == l + 64 ? lab : l1;
  }
  __device__ void assign(B128 ch, int lab) {
    const int l = lane_id();
    l0 = ((ch.lo >> l) & 1) ? lab : l0;
    l1 = ((ch.hi >> l) & 1) ? lab : l1;
  }
  // Labels of every chain of s (each labelled by its lowest point).
  __device__ void init(const Go::State& s, const GameCfg& g) {
    l0 = l1 = -1;
    B128 todo = s.bw[0] | s.bw[1];
    while (any(todo)) {
      const int q = lowest(todo);
      const B128 col = test(s.bw[0], q) ? s.bw[0] : s.bw[1];
      const B128 ch = Go::flood(bit128(q), col, g);
      todo = todo & ~ch;
      assign(ch, q);
    }
  }
};

// Neighbourhoods on the vector unit.  nbr(x) = the board points with a
// 4-neighbour in x, which is Go::nbr4(x) (adjacency is symmetric); the scalar
// form is four 128-bit shifts, two column masks and the ORs (~30 SALU).  Here
// lane l tests points l and l + 64: x shifted up one row (e = x << n, five
// dwords) puts the neighbours p - n, p - 1, p + 1, p + n of p at bits 0, n - 1,
// n + 1, 2n of the 32-bit window of e at bit p, one v_alignbit away; the
// lane's constant mask (m0 / m1, the edge columns and off-board points
// cleared) picks them and a v_cmp writes the result straight into the mask.
// ~10 VALU + ~6 SALU: the wave search is bound by the scalar unit (one per
// CU, shared by its waves) while the VALU idles.  n <= 15 (2n < 32).
struct GoNbrLanes {
  uint32_t m0, m1;  // per lane
  int n;
  __device__ void init(const GameCfg& g) {
    n = g.rows;
    const int N = g.rows * g.cols;
    const int l = lane_id();
    auto mk = [&](int p) -> uint32_t {
      if (p >= N) return 0u;
      const int c = p % n;
      uint32_t m = 1u | (1u << (2 * n));
      if (c > 0) m |= 1u << (n - 1);
      if (c < n - 1) m |= 1u << (n + 1);
      return m;
    };
    m0 = mk(l);
    m1 = mk(l + 64);
  }
  __device__ B128 any(B128 x) const { return any_but(x, -1); }
  // any(x) without point `skip` (-1: none): the ko point drops out in the same v_cmp.
  __device__ B128 any_but(B128 x, int skip) const {
    const uint64_t elo = x.lo << n;
    const uint64_t ehi = (x.hi << n) | (x.lo >> (64 - n));
    const uint32_t e0 = static_cast<uint32_t>(elo), e1 = static_cast<uint32_t>(elo >> 32);
    const uint32_t e2 = static_cast<uint32_t>(ehi), e3 = static_cast<uint32_t>(ehi >> 32);
    const uint32_t e4 = static_cast<uint32_t>(x.hi >> (64 - n));
    const int l = lane_id();
    const bool up = l >= 32;
    const uint32_t w0 = __builtin_amdgcn_alignbit(up ? e2 : e1, up ? e1 : e0, l & 31);
    const uint32_t w1 = __builtin_amdgcn_alignbit(up ? e4 : e3, up ? e3 : e2, l & 31);
    return b128(ballot((w0 & m0) != 0 && l != skip), ballot((w1 & m1) != 0 && l + 64 != skip));
  }
  // any(bit128(a)): a is p's neighbour iff t = a - p + n is one of p's window
  // bits, so no one-hot set is built and shifted.
  __device__ B128 at(int a) const {
    const int l = lane_id();
    const uint32_t t0 = static_cast<uint32_t>(a - l + n), t1 = static_cast<uint32_t>(a - l - 64 + n);
    const bool h0 = t0 < 32u && ((m0 >> (t0 & 31u)) & 1u);
    const bool h1 = t1 < 32u && ((m1 >> (t1 & 31u)) & 1u);
    return b128(ballot(h0), ballot(h1));
  }
};

// The playout's board relative to the player to move (the state's bw[] is
// rebuilt at the end): no per-move selects of bw[to_play] on the scalar unit.
struct GoSides {
  B128 me, them;
};

// Go::legal with the neighbourhoods on the lanes (same mask, go_board.cc:425-440):
// Go::legal's cand & (nbr4(E) | (hard & nbr4(good))) is E & ~ko & nbr4(E | good),
// one neighbourhood with the ko point dropped in its compare.
__device__ __forceinline__ Go::Legal go_legal_lanes(const Go::State& s, const GoSides& sd,
                                                    const GameCfg& g, const GoNbrLanes& nb) {
  using M = CfgMasks<B128>;
  const B128 E = M::board(g) & ~(sd.me | sd.them);
  const B128 good = (sd.me & ~s.atari) | (sd.them & s.atari);
  const B128 mask = E & nb.any_but(E | good, s.ko);
  Go::Legal l;
  l.mask = mask;
  l.count = popc(mask) + 1;
  l.pass_action = g.rows * g.cols;
  return l;
}

// LegalActions()[k] from the legal mask on the lanes: the lane holding the
// k-th set bit sees exactly k set bits below it (mbcnt); pass is last.
__device__ __forceinline__ int go_kth_lanes(B128 mask, int k, int pass) {
  const int c0 = popc64(mask.lo);
  if (k >= c0 + popc64(mask.hi)) return pass;
  const bool hi = k >= c0;
  const uint64_t w = hi ? mask.hi : mask.lo;
  const uint32_t kk = static_cast<uint32_t>(hi ? k - c0 : k);
  const int l = lane_id();
  const uint32_t below = __builtin_amdgcn_mbcnt_hi(
      static_cast<uint32_t>(w >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(w), 0u));
  const uint64_t b = ballot(((w >> l) & 1) && below == kk);
  return (hi ? 64 : 0) + ctz64(b);
}

// GoT::apply (go_board.cc:217-299 via go.cc:124-216) with chains from labels.
__device__ __forceinline__ void go_apply_lanes(Go::State& s, GoSides& sd, const GameCfg& g,
                                               GoWaveCtx& ctx, GoLabels& lab,
                                               const GoNbrLanes& nbl, int a) {
  using M = CfgMasks<B128>;
  const int c = s.to_play;
  const int pass = g.rows * g.cols;
  s.flags = static_cast<uint8_t>((s.flags & Go::kSuperko) |
                                 ((s.flags & Go::kLastPass) ? Go::kPrevPass : 0));
  if (a == pass) {
    s.ko = -1;
    s.flags |= Go::kLastPass;
    const B128 t = sd.me;
    sd.me = sd.them;
    sd.them = t;
  } else {
#if OS_PHASE_TIMING
    uint64_t tx = OS_PH_NOW();
#endif
    const B128 pb = bit128(a);
    const B128 nb = nbl.at(a);
    const B128 own0 = sd.me;
    const B128 own = own0 | pb;
    B128 opp = sd.them;
    const bool enemy_eye = !any(nb & ~opp);
    s.hash ^= ctx.zob[2 * a + c];
    B128 E = M::board(g) & ~(own | opp);
    // The own chains next to a join the new stone's chain, labelled a.
    B128 on_own = nb & own0;
    while (any(on_own)) {
      const int L = lab.at(lowest(on_own));
      on_own = on_own & ~lab.chain(L);
      lab.relabel(L, a);
    }
    lab.set(a, a);
#if OS_PHASE_TIMING
    OS_PH_ADD(ctx.sub[kPhX0], tx);
    tx = OS_PH_NOW();
#endif
    int captured = 0;
    int cap_pt = -1;
    B128 atari = s.atari;
    B128 capd = b128(0, 0);
    B128 on = nb & opp;
    while (any(on)) {
      const int q = lowest(on);
      const B128 ch = lab.chain(lab.at(q)) & opp;
      on = on & ~ch;
      const B128 libs = nbl.any(ch) & E;
      if (!any(libs)) {
        opp = opp & ~ch;
        E = E | ch;
        capd = capd | ch;
        captured += popc(ch);
        cap_pt = q;
        B128 rem = ch;
        while (any(rem)) {
          const int x = lowest(rem);
          rem = rem & ~bit128(x);
          s.hash ^= ctx.zob[2 * x + (1 - c)];
        }
      }
      atari = (atari & ~ch) | sel128(popc(libs) == 1, ch, b128(0, 0));
    }
#if OS_PHASE_TIMING
    OS_PH_ADD(ctx.sub[kPhX1], tx);
    tx = OS_PH_NOW();
#endif
    // The mover's chain (label a) and, after captures, the own chains next to
    // the captured stones.  (Skipping the liberty counts where the atari set
    // or two empty neighbours settle them was measured slower here: 1.70e7 ->
    // 1.63e7 sims/s at 4096 roots; the lane kernels do use it, GoT::apply.)
    {
      const B128 ch = lab.chain(a) & own;
      atari = (atari & ~ch) | sel128(popc(nbl.any(ch) & E) == 1, ch, b128(0, 0));
      B128 todo = any(capd) ? nbl.any(capd) & own & ~ch : b128(0, 0);
      while (any(todo)) {
        const B128 cx = lab.chain(lab.at(lowest(todo))) & own;
        todo = todo & ~cx;
        atari = (atari & ~cx) | sel128(popc(nbl.any(cx) & E) == 1, cx, b128(0, 0));
      }
    }
#if OS_PHASE_TIMING
    OS_PH_ADD(ctx.sub[kPhX2], tx);
    tx = OS_PH_NOW();
#endif
    s.atari = atari;
    sd.me = opp;  // the next player's stones
    sd.them = own;
    s.ko = static_cast<int16_t>((enemy_eye && captured == 1) ? cap_pt : -1);
#if OS_PHASE_TIMING
    OS_PH_ADD(ctx.sub[kPhX3], tx);
#endif
    if (!ctx.insert(s.hash, captured > 0, popc(own) + popc(opp))) s.flags |= Go::kSuperko;
  }
  s.to_play = static_cast<uint8_t>(1 - c);
  s.moves++;
}

template <int Policy, class Rng>
__device__ int go_rollout_wave(Go::State s, const GameCfg& g, GoWaveCtx& ctx, Rng& ev) {
  s = make_uniform(s);
  ev.uniformize();
  GoLabels lab;
  lab.init(s, g);
  GoNbrLanes nbl;
  nbl.init(g);
  GoSides sd;
  sd.me = pick(s.bw, s.to_play);
  sd.them = pick(s.bw, 1 - s.to_play);
  const int pass = g.rows * g.cols;
  for (;;) {
    if (Go::terminal(s, g)) break;
#if OS_PHASE_TIMING
    const uint64_t t0 = OS_PH_NOW();
#endif
    const Go::Legal l = go_legal_lanes(s, sd, g, nbl);
    uint32_t k;
    if (Policy == kPolicyCpp)
      k = ev.uniform_lanes(static_cast<uint32_t>(l.count));
    else
      k = NpChoice(ev, static_cast<uint32_t>(l.count));
    const int act = go_kth_lanes(l.mask, static_cast<int>(k), pass);
#if OS_PHASE_TIMING
    const uint64_t t1 = OS_PH_NOW();
    OS_PH_ADD(ctx.sub[kPhGoLegal], t0);
#endif
    go_apply_lanes(s, sd, g, ctx, lab, nbl, act);
#if OS_PHASE_TIMING
    OS_PH_ADD(ctx.sub[kPhGoApply], t1);
#endif
  }
  s.bw[0] = sel128(s.to_play == 0, sd.me, sd.them);
  s.bw[1] = sel128(s.to_play == 0, sd.them, sd.me);
#if OS_PHASE_TIMING
  const uint64_t t2 = OS_PH_NOW();
  const int r0 = Go::ret0(s, g, ctx);
  OS_PH_ADD(ctx.sub[kPhGoScore], t2);
  return r0;
#else
  return Go::ret0(s, g, ctx);
#endif
}

template <class G, int Policy, class Rng, class C>
__device__ int wave_rollout(typename G::State s, const GameCfg& g, C& ctx, Rng& ev) {
  if constexpr (std::is_same<G, Breakthrough>::value) {
    (void)ctx;
    return g.cols == 1 ? bt_rollout_wave<Policy, true>(s, g, ev)
                       : bt_rollout_wave<Policy, false>(s, g, ev);
  }
  if constexpr (Policy == kPolicyCpp && SmallAbsl<G>::value) {
    if (ev.use7) return c4_rollout_lanes(s, ctx, ev);
  }
  if constexpr (Policy == kPolicyNumpy && std::is_same<G, ConnectFour>::value)
    return c4_rollout_lanes<kPolicyNumpy>(s, ctx, ev);
  // C++ policy only: the numpy form's serial window draws cost more than
  // the short serial playout they replace (3.56 -> 3.76 ms per 1000-sim step)
  if constexpr (Policy == kPolicyCpp && std::is_same<G, TicTacToe>::value) {
    const int r = ttt_rollout_lanes<Policy>(s, g, ev);
    if (r != kLanesDecline) return r;
  }
#if OS_GO_LANES
  if constexpr (std::is_same<G, Go>::value) return go_rollout_wave<Policy>(s, g, ctx, ev);
#endif
  if constexpr (std::is_same<G, Hex>::value) {
    // n >= 3: on n <= 2 the reference's wrap filter (hex.cc:206-222) leaves
    // filled boards without a winner, so the end-of-fill argument fails.
    if (g.rows >= 3) {
      const int r = hex_rollout_lanes<Policy>(s, g, ctx, ev);
      if (r != kLanesDecline) return r;
    }
  }
#if OS_UNI_ROLL == 2
  s = make_uniform(s);  // uniform on entry => the loop-carried state can stay in SGPRs
  ev.uniformize();
#endif
  for (;;) {
#if OS_UNI_ROLL == 1
    s = make_uniform(s);  // keep the playout on the scalar unit
#endif
    if (G::terminal(s, g)) break;
#if OS_PHASE_TIMING
    const uint64_t t0 = OS_PH_NOW();
#endif
    const typename G::Legal l = G::legal(s, g, ctx);
    uint32_t k;
    if (Policy == kPolicyCpp && SmallAbsl<G>::value)
      k = ev.uniform_small(static_cast<uint32_t>(l.count));
    else if (Policy == kPolicyCpp)
      k = ev.uniform_lanes(static_cast<uint32_t>(l.count));
    else
      k = NpChoice(ev, static_cast<uint32_t>(l.count));
    const int act = l.kth(static_cast<int>(k));
#if OS_PHASE_TIMING
    const uint64_t t1 = OS_PH_NOW();
    if constexpr (std::is_same<G, Go>::value) OS_PH_ADD(ctx.sub[kPhGoLegal], t0);
#endif
    G::apply(s, g, ctx, act);
#if OS_PHASE_TIMING
    if constexpr (std::is_same<G, Go>::value) OS_PH_ADD(ctx.sub[kPhGoApply], t1);
#endif
  }
#if OS_PHASE_TIMING
  const uint64_t t2 = OS_PH_NOW();
  const int r0 = G::ret0(s, g, ctx);
  if constexpr (std::is_same<G, Go>::value) OS_PH_ADD(ctx.sub[kPhGoScore], t2);
  return r0;
#else
  return G::ret0(s, g, ctx);
#endif
}

// A child node as ONE 16-byte load (Node<int32_t> is 16-byte aligned in the
// arena): copying the struct field-wise costs three loads (dwordx3 + two
// ushort) per lane and scan level.
template <class R>
__device__ __forceinline__ Node<R> load_node(const Node<R>* p) {
  return *p;
}
template <>
__device__ __forceinline__ Node<int32_t> load_node(const Node<int32_t>* p) {
  static_assert(sizeof(Node<int32_t>) == 16, "16-byte node");
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  Node<int32_t> c;
  c.first = v.x;
  c.n = static_cast<int32_t>(v.y);
  c.w = static_cast<int32_t>(v.z);
  c.action = static_cast<uint16_t>(v.w & 0xFFFFu);
  c.nchild = static_cast<uint8_t>((v.w >> 16) & 0xFFu);
  c.out = static_cast<int8_t>(v.w >> 24);
  return c;
}

// Paged arena: `pages` (global, null = the reserved
// per-root arena of `cap` nodes) = {pages taken, page_nodes, pool_pages,
// first dynamic page}.  The search starts on its own page (page blockIdx.x:
// `nodes` points there, cap = page_nodes) and takes further pages off the
// launch's counter when a child block does not fit the current one.  Node
// indices stay relative to `nodes` (uint32; dynamic pages lie above).
// k_wsearch leaves the descriptor's address in the kPageDescLds bytes of LDS
// just below `path` (kPageable searches only): read on that rare path, it
// holds no scalar registers across the search, which is at its SGPR budget.
// (kPgTaken ... kPgFirstDynamic: os_mcts.h.)
constexpr int kPageDescLds = 16;

// LegalActions()[k] for lane k (k < count; other lanes get garbage) in the
// wave kernels' expansion.  connect_four: the ascending legal columns as
// nibbles from one row scan (lane c < 7 places c at nibble rank-of-c), then a
// per-lane shift -- no per-lane loop over the mask.
template <class G>
struct WaveKth {
  __device__ __forceinline__ static int kth(const typename G::Legal& lg, int k) {
    return lg.kth(k);
  }
};
template <>
struct WaveKth<ConnectFour> {
  __device__ __forceinline__ static int kth(const ConnectFour::Legal& lg, int k) {
    const uint32_t c = static_cast<uint32_t>(lane_id() & 7);
    const bool lgl = c < 7 && ((lg.mask >> c) & 1u);
    const uint32_t rank = static_cast<uint32_t>(__builtin_popcount(lg.mask & ((1u << c) - 1u)));
    const uint32_t cols = rl32(row_scan_add(lgl ? c << (4 * rank) : 0u), 7);
    return static_cast<int>((cols >> (4 * (k & 7))) & 15u);
  }
};

// State::apply for the wave kernels' tree walk.  connect_four's four-in-a-row
// test runs on the vector unit: lane j tests direction j & 3 (shift 1, 7, 6,
// 8), one ballot ORs them -- the same predicate as ConnectFour::has_four, in
// a handful of VALU ops instead of ~30 dependent 64-bit scalar ops and four
// branches on the scalar unit (the wave kernels' binding pipe).
template <class G>
struct WaveApply {
  template <class C>
  __device__ __forceinline__ static void apply(typename G::State& s, const GameCfg& g, C& ctx,
                                               int a) {
    G::apply(s, g, ctx, a);
  }
};
template <>
struct WaveApply<ConnectFour> {
  template <class C>
  __device__ __forceinline__ static void apply(ConnectFour::State& s, const GameCfg&, C&,
                                               int col) {
    const int p = s.to_play;
    const uint64_t occ = s.bb[0] | s.bb[1];
    const uint64_t colmask = 0x3Full << (7 * col);
    const uint64_t mv = (occ + (1ull << (7 * col))) & colmask;
    const uint64_t mine = pick(s.bb, p) | mv;
    put(s.bb, p, mine);
    s.moves++;
    if (mv & ConnectFour::kTopRow) s.legal &= ~(1u << col);
    // shift 1, 7, 6, 8 for lane & 3 (one byte extract, no exec-mask branch)
    const uint32_t d = (0x08060701u >> (8 * (lane_id() & 3))) & 0xFFu;
    const uint64_t m = mine & (mine >> d);
    if (ballot((m & (m >> (2 * d))) != 0)) s.outcome = p;
    else if (s.moves == 42) s.outcome = 2;
    s.to_play = 1 - p;
  }
};

// The visit path held in the lanes (lane d <-> path entry d) for games whose
// longest path fits a wave (MaxGameLength + 2 <= 64: tic_tac_toe,
// connect_four).  Entries are written by per-lane selects (no exec-mask
// branch, no LDS store), backup reads its own lane's entry, and the solver
// reads entry d with one v_readlane per field.
template <class G>
struct LanePathGame : std::false_type {};
template <>
struct LanePathGame<TicTacToe> : std::true_type {};
template <>
struct LanePathGame<ConnectFour> : std::true_type {};

template <class R>
struct LanePath {
  uint32_t idx = 0, first = 0;
  int32_t n = 0, nc = 0;
  R w = 0;
  __device__ __forceinline__ void set(int d, uint32_t i, uint32_t f, int32_t cn, int32_t cnc,
                                      R cw) {
    const bool me = lane_id() == d;
    idx = me ? i : idx;
    first = me ? f : first;
    n = me ? cn : n;
    nc = me ? cnc : nc;
    w = me ? cw : w;
  }
  __device__ __forceinline__ void set_children(int d, uint32_t f, int32_t cnc) {
    const bool me = lane_id() == d;
    first = me ? f : first;
    nc = me ? cnc : nc;
  }
};

// LDS copy of the search's first kCache arena nodes (os_kernels.h
// OS_NODE_CACHE).  Nodes are allocated in expansion order, so these are the
// tree's top levels, which every simulation walks: selection reads a child
// block that lies wholly below kCache from LDS instead of HBM / MALL.  Every
// store to such a node is written through to both copies.
// K = kCacheAll (-1): the whole arena is in LDS (k_wsearch kLdsTree: a small
// batch whose reserved tree fits the CU's LDS), `k` = the arena's capacity,
// so every block is an LDS block.
constexpr int kCacheAll = -1;
template <class R, int K>
struct NodeCache {
  Node<R>* c;
  uint32_t k;
  __device__ __forceinline__ bool has(uint32_t i) const {
    return K == kCacheAll || (K > 0 && i < static_cast<uint32_t>(K));
  }
  __device__ __forceinline__ bool block(uint32_t first, int n) const {
    return K == kCacheAll || (K > 0 && first + static_cast<uint32_t>(n) <= static_cast<uint32_t>(K));
  }
};

// One search, executed by the whole wave.  `path` (LDS) has path_cap
// entries.  Same contract as mcts_search; kPuct selects children by
// PUCTValue (sp.log_lut then holds sqrt(N)); kCache > 0: `lcache` (LDS)
// holds the first kCache nodes (NodeCache); kCache == kCacheAll: all `cap`.
template <class G, class R, int Policy, bool kPageable = false, bool kPuct = false,
          int kCache = 0, bool kPace = false, class C>
__device__ SearchResult wave_search(const GameCfg& g, const SearchParams& sp,
                                    const typename G::State& root, C& ctx,
                                    Node<R>* nodes, uint32_t cap, WaveMt& bot,
                                    WaveMt& ev, PathEnt<R>* path, int path_cap,
                                    PhaseCycles& ph, Node<R>* lcache = nullptr) {
  const int l = lane_id();
  const NodeCache<R, kCache> nc_ = {lcache, cap};
  const uint64_t t_begin = OS_PH_NOW();
  SearchResult res;
  res.status = kOk;
  res.sims = 0;
  res.gc_runs = 0;
  res.max_depth = 0;
  res.scanned = res.backed = res.expanded = res.solver_scanned = 0;
  LaneCount c_scanned, c_backed, c_expanded, c_solver, c_depth;  // VGPR-resident
  c_scanned.reset();
  c_backed.reset();
  c_expanded.reset();
  c_solver.reset();
  c_depth.reset();
  const int P0 = G::to_move(root);
  if (l == 0) {
    nodes[0].first = 0;
    nodes[0].n = 0;
    nodes[0].w = 0;
    nodes[0].action = 0;
    nodes[0].nchild = 0;
    nodes[0].out = kUnsolved;
    if (kCache != 0) nc_.c[0] = nodes[0];
  }
  // Root statistics persist in registers across simulations.
  uint32_t root_first = 0;
  int32_t root_n = 0;
  int root_nc = 0;
  R root_w = 0;
  int8_t root_out = kUnsolved;
  uint32_t used = 1;
  int nodes_count = 1;
  int gc_limit = 5;
  const double inf = __builtin_huge_val();
  using WW = WaveWidth<G>;
  Node<R> zero_node;
  zero_node.first = 0; zero_node.n = 0; zero_node.w = 0; zero_node.action = 0;
  zero_node.nchild = 0; zero_node.out = kUnsolved;
  double root_logN = sp.log_lut[0];
  // The root's children, register-resident across simulations (lane k holds
  // child k, and k + 64 in the second slot), with log(n) of each; every write
  // to a root child (expansion, leaf outcome, backup, solver, GC) is mirrored
  // here, so the root scan issues no loads.  root_k = this simulation's
  // root child (the depth-1 node of the path).
  Node<R> rc0 = zero_node, rc1 = zero_node;
  double rlg0 = 0.0, rlg1 = 0.0;
  int root_k = 0;
  constexpr bool kLP = OS_LANE_PATH && LanePathGame<G>::value;
  // cur_logN is then only read on the screen's fallback, loaded there.
  constexpr bool kLazyLog = OS_SCREEN_LOG && OS_UCT_SCREEN && sizeof(R) == 4 && !kPuct &&
                            (OS_UCT_SCREEN == 2 || !WW::kTwoSlots);
  LanePath<R> lp;
  if (kLP && path_cap > 64) path_cap = 64;

  Pacer pacer;
  if (kPace) pacer.begin();
  for (int sim = 0; sim < sp.max_simulations; ++sim) {
    if (kPace && (sim & (OS_PACE_EVERY - 1)) == 0 && sim > 0)
      pacer.update(static_cast<uint32_t>(sim), sp.max_simulations / OS_PACE_BAND);
    uint64_t t_ph = OS_PH_NOW();
    typename G::State s = root;
    ctx.reset();
    uint32_t cur_idx = 0;
    uint32_t cur_first = root_first;
    int32_t cur_n = root_n;
    int cur_nc = root_nc;
    double cur_logN = root_logN;  // log(N) of the node being scanned (mcts.cc:99)
    int depth = 0;
    if constexpr (UniSel<G>::kMode == 2) {
      s = make_uniform(s);
      cur_n = __builtin_amdgcn_readfirstlane(cur_n);
      cur_nc = __builtin_amdgcn_readfirstlane(cur_nc);
      cur_first = static_cast<uint32_t>(
          __builtin_amdgcn_readfirstlane(static_cast<int>(cur_first)));
      cur_logN = make_uniform(cur_logN);
      bot.uniformize();
    }
    // ---- selection / expansion ----
    bool pending_expand = false;
#if OS_PHASE_SEL
    constexpr bool kSelPh = !std::is_same<G, Go>::value;
    if (kSelPh) OS_PH_ADD(ph.c[kPhGoLegal], t_ph);
    uint64_t t_loop = OS_PH_NOW();
#endif
    for (;;) {
      if constexpr (UniSel<G>::kMode == 1) {
        s = make_uniform(s);
        cur_n = __builtin_amdgcn_readfirstlane(cur_n);
        cur_nc = __builtin_amdgcn_readfirstlane(cur_nc);
        cur_first = static_cast<uint32_t>(
            __builtin_amdgcn_readfirstlane(static_cast<int>(cur_first)));
        cur_idx = static_cast<uint32_t>(
            __builtin_amdgcn_readfirstlane(static_cast<int>(cur_idx)));
        depth = __builtin_amdgcn_readfirstlane(depth);
      }
      if (G::terminal(s, g) || cur_n <= 0) break;
      // The node to expand ends the descent (its first child is fresh): the
      // expansion runs after the loop, so the per-level loop carries only
      // the selection (no merge of the two paths' values every level).
      if (cur_nc == 0) {
        pending_expand = true;
        break;
      }
      int chosen;
      uint32_t c_action, c_first;
      int32_t c_n;
      int c_nc;
      R c_w;
      // Lane k scores child k (and k + 64); each lane also fetches
      // log(n) of its own child, which is log(N_parent) one level down if
      // that child is chosen, so the next level needs no dependent load.
      const int cp = P0 ^ (depth & 1);
      c_scanned.add(cur_nc);
      Node<R> c0 = zero_node, c1 = zero_node;
      double lg0 = 0.0, lg1 = 0.0;
      const bool in0 = l < cur_nc, in1 = WW::kTwoSlots && l + 64 < cur_nc;
      if (depth == 0) {  // root children: register-resident, no loads
        // Lanes past the last child hold zero_node in the mirror (every
        // write to it keeps that), so no exec mask is needed here.
        c0 = rc0;
        lg0 = rlg0;
        if (in1) {
          c1 = rc1;
          lg1 = rlg1;
        }
      } else {
        // Every lane loads (lanes past the last child re-read child 0, so
        // no exec-mask branch); their values are masked by in0 / in1.
        // A block of the cached top levels comes from LDS (wave-uniform).
        const Node<R>* src = nc_.block(cur_first, cur_nc) ? nc_.c : nodes;
        if (nc_.block(cur_first, cur_nc)) c0 = load_node(nc_.c + cur_first + (in0 ? l : 0));
        else c0 = load_node(nodes + cur_first + (in0 ? l : 0));
        if (!kLazyLog) lg0 = sp.log_lut[c0.n];
        if (in1) {
          c1 = load_node(src + cur_first + l + 64);
          if (!kLazyLog) lg1 = sp.log_lut[c1.n];
        }
      }
#if OS_PHASE_SEL
      const uint64_t t_sc = OS_PH_NOW();
#endif
      if constexpr (kPuct) {
        // PUCTValue (mcts.cc:102-111): unvisited children are not +inf, so
        // every child is scored in f64 (cur_logN holds sqrt(N) here).
        const double cprior = puct_prior_term(sp.uct_c, cur_nc);
        const double v0 = puct_value_sel(c0, in0, cp, cur_logN, cprior);
        const double v1 =
            WW::kTwoSlots ? puct_value_sel(c1, in1, cp, cur_logN, cprior) : -inf;
        chosen = wave_argmax2<WW::kLanes, WW::kTwoSlots>(v0, v1);
      } else {
      // An unvisited unsolved child scores +inf, above every finite UCT
      // value and solver outcome, so the first one in index order wins the
      // strict '>' scan outright: one ballot instead of the f64 UCT values
      // and the wave max.
      const uint64_t f0 = ballot(in0 && c0.out == kUnsolved && c0.n == 0);
      const uint64_t f1 =
          WW::kTwoSlots ? ballot(in1 && c1.out == kUnsolved && c1.n == 0) : 0ull;
      if (f0 | f1) {
        chosen = f0 ? ctz64(f0) : 64 + ctz64(f1);
      } else {
        chosen = -1;
#if OS_UCT_SCREEN
        if constexpr (kLazyLog)
          chosen = uct_argmax_screen_lf<WW::kLanes, WW::kTwoSlots>(c0, in0, c1, in1, cp,
                                                                   screen_log(cur_n), sp.uct_c);
        else if constexpr (sizeof(R) == 4 && (OS_UCT_SCREEN == 2 || !WW::kTwoSlots))
          chosen = uct_argmax_screen<WW::kLanes, WW::kTwoSlots>(c0, in0, c1, in1, cp,
                                                                cur_logN, sp.uct_c);
#endif
      }
      }
      if (kLazyLog && chosen < 0)  // the exact log(N) for the f64 scan
        cur_logN = depth == 0 ? root_logN : sp.log_lut[cur_n];
      if (!kPuct && chosen < 0) {
        const double v0 = uct_value_sel(c0, in0, cp, cur_logN, sp.uct_c);
        const double v1 = WW::kTwoSlots ? uct_value_sel(c1, in1, cp, cur_logN, sp.uct_c) : -inf;
        chosen = wave_argmax2<WW::kLanes, WW::kTwoSlots>(v0, v1);
      }
      if (depth == 0) root_k = chosen;
#if OS_PHASE_SEL
      if (kSelPh) OS_PH_ADD(ph.c[kPhGoScore], t_sc);
#endif
      const int src = chosen & 63;
      const bool hi = WW::kTwoSlots && chosen >= 64;  // wave-uniform
      const Node<R> bc = hi ? c1 : c0;
      c_action = rl32(bc.action, src);
      c_first = rl32(bc.first, src);
      c_n = rli(bc.n, src);
      c_nc = rli(bc.nchild, src);
      if (sizeof(R) == 4) {
        const int32_t wi = rli(static_cast<int32_t>(bc.w), src);
        c_w = static_cast<R>(wi);
      } else {
        c_w = static_cast<R>(rld(static_cast<double>(bc.w), src));
      }
      if (!kLazyLog) cur_logN = rld(hi ? lg1 : lg0, src);
#if OS_WAVE_APPLY
      WaveApply<G>::apply(s, g, ctx, static_cast<int>(c_action));
#else
      G::apply(s, g, ctx, static_cast<int>(c_action));
#endif
      if (++depth >= path_cap) {
        res.status = kPathOverflow;
        goto done;
      }
      cur_idx = cur_first + chosen;
      cur_first = c_first;
      cur_n = c_n;
      cur_nc = c_nc;
      if constexpr (kLP) {
        lp.set(depth, cur_idx, c_first, c_n, c_nc, c_w);
      } else if (l == 0) {
        PathEnt<R>& pe = path[depth];
        pe.idx = cur_idx;
        pe.first = c_first;
        pe.n = c_n;
        pe.nc = c_nc;
        pe.w = c_w;
      }
    }
#if OS_PHASE_SEL
    if (kSelPh) OS_PH_ADD(ph.c[kPhGoApply], t_loop);
    t_loop = OS_PH_NOW();
#endif
    if (pending_expand) {
      int chosen;
      uint32_t c_action, c_first;
      int32_t c_n;
      int c_nc;
      R c_w;
        const uint64_t t_ex = OS_PH_NOW();
        const typename G::Legal lg = G::legal(s, g, ctx);
        const int nc = lg.count;
        LaneArr acts;
#if OS_WAVE_KTH
        const int k0 = WaveKth<G>::kth(lg, l);  // every lane (row scan inside)
        acts.a0 = l < nc ? static_cast<uint32_t>(k0) : 0u;
#else
        acts.a0 = l < nc ? static_cast<uint32_t>(lg.kth(l)) : 0u;
#endif
        acts.a1 = l + 64 < nc ? static_cast<uint32_t>(lg.kth(l + 64)) : 0u;
        wave_shuffle<Policy, WaveMt, !std::is_same<G, Go>::value>(acts, nc, bot);
        if (used + static_cast<uint32_t>(nc) > cap) {
          bool ok = false;
          if constexpr (kPageable) {  // next page of the pool, if there is one
            const uint64_t v = *reinterpret_cast<const volatile uint64_t*>(
                reinterpret_cast<const unsigned char*>(path) - kPageDescLds);
            uint32_t* const pg = reinterpret_cast<uint32_t*>(make_uniform(v));
            if (pg) {
              uint32_t np = 0;
              if (l == 0) np = atomicAdd(pg + kPgTaken, 1u);  // one vector atomic
              const uint4 d = make_uniform(*reinterpret_cast<const uint4*>(pg));
              np = rl32(np, 0) + d.w;  // kPgFirstDynamic
              const uint32_t pn = d.y;  // kPgNodes
              ok = np < d.z;            // kPgPool
              used = (np - blockIdx.x) * pn;
              cap = used + pn;
            }
          }
          if (!ok) {
            res.status = kArenaOverflow;
            goto done;
          }
        }
        const uint32_t first = used;
        used += nc;
        for (int h = 0; h < 2; ++h) {
          const int k = l + 64 * h;
          if (k < nc) {
            Node<R>& c = nodes[first + k];
            c.first = 0;
            c.n = 0;
            c.w = 0;
            c.action = static_cast<uint16_t>(h == 0 ? acts.a0 : acts.a1);
            c.nchild = 0;
            c.out = kUnsolved;
            if (nc_.has(first + k)) nc_.c[first + k] = c;
          }
        }
        if (l == 0) {
          nodes[cur_idx].first = first;
          nodes[cur_idx].nchild = static_cast<uint8_t>(nc);
          if (nc_.has(cur_idx)) {
            nc_.c[cur_idx].first = first;
            nc_.c[cur_idx].nchild = static_cast<uint8_t>(nc);
          }
        }
        if (depth == 0) {
          root_first = first;
          root_nc = nc;
          // Root children live in registers from now on (lane k <-> child k).
          rc0 = zero_node;
          rc1 = zero_node;
          if (l < nc) rc0.action = static_cast<uint16_t>(acts.a0);
          if (WW::kTwoSlots && l + 64 < nc) rc1.action = static_cast<uint16_t>(acts.a1);
          rlg0 = rlg1 = sp.log_lut[0];
          root_k = 0;
        } else {
          if constexpr (kLP) {
            lp.set_children(depth, first, nc);
          } else if (l == 0) {
            path[depth].first = first;
            path[depth].nc = nc;
          }
          if (depth == 1) {  // the expanded node is root child root_k
            if (l == (root_k & 63)) {
              if (root_k < 64) {
                rc0.first = first;
                rc0.nchild = static_cast<uint8_t>(nc);
              } else {
                rc1.first = first;
                rc1.nchild = static_cast<uint8_t>(nc);
              }
            }
          }
        }
        nodes_count += nc;
        c_expanded.add(nc);
        cur_first = first;
        cur_nc = nc;
        chosen = 0;  // all children fresh: +inf, the first one wins
        c_action = acts.get(0);
        c_first = 0;
        c_n = 0;
        c_nc = 0;
        c_w = 0;
        OS_PH_ADD(ph.c[kPhExpand], t_ex);
#if OS_WAVE_APPLY
      WaveApply<G>::apply(s, g, ctx, static_cast<int>(c_action));
#else
      G::apply(s, g, ctx, static_cast<int>(c_action));
#endif
      if (++depth >= path_cap) {
        res.status = kPathOverflow;
        goto done;
      }
      cur_idx = cur_first + chosen;
      cur_first = c_first;
      cur_n = c_n;
      cur_nc = c_nc;
      if constexpr (kLP) {
        lp.set(depth, cur_idx, c_first, c_n, c_nc, c_w);
      } else if (l == 0) {
        PathEnt<R>& pe = path[depth];
        pe.idx = cur_idx;
        pe.first = c_first;
        pe.n = c_n;
        pe.nc = c_nc;
        pe.w = c_w;
      }
    }
    c_depth.max(depth);
    __builtin_amdgcn_wave_barrier();
#if OS_PHASE_SEL
    if (kSelPh) OS_PH_ADD(ph.c[kPhGoInsert], t_loop);
#endif
    OS_PH_ADD(ph.c[kPhSelect], t_ph);
    t_ph = OS_PH_NOW();
    {
      // ---- evaluation ----
      bool solved;
      R rv0, rv1;
      int8_t leaf_out = kUnsolved;
      if (G::terminal(s, g)) {
        const int r0 = G::ret0(s, g, ctx);
        leaf_out = static_cast<int8_t>(r0);
        if (l == 0) {
          nodes[cur_idx].out = leaf_out;
          if (nc_.has(cur_idx)) nc_.c[cur_idx].out = leaf_out;
        }
        if (depth == 1 && l == (root_k & 63)) {
          if (root_k < 64) rc0.out = leaf_out;
          else rc1.out = leaf_out;
        }
        solved = sp.solve != 0;
        rv0 = static_cast<R>(r0);
        rv1 = static_cast<R>(-r0);
      } else {
        solved = false;
        if (sp.n_rollouts == 1) {
          const int r0 = wave_rollout<G, Policy>(s, g, ctx, ev);
          rv0 = static_cast<R>(r0);
          rv1 = static_cast<R>(-r0);
        } else {
          // Every rollout starts from a clone of the leaf (mcts.cc:46-47), so
          // go's position log is rewound to the leaf before each one.
          const auto leaf_ctx = ctx;
          double s0 = 0.0, s1 = 0.0;
          for (int k = 0; k < sp.n_rollouts; ++k) {
            if (k) ctx = leaf_ctx;
            const int r0 = wave_rollout<G, Policy>(s, g, ctx, ev);
            s0 += static_cast<double>(r0);
            s1 += static_cast<double>(-r0);
          }
          rv0 = static_cast<R>(s0 / sp.n_rollouts);
          rv1 = static_cast<R>(s1 / sp.n_rollouts);
        }
      }
      OS_PH_ADD(ph.c[kPhRollout], t_ph);
      t_ph = OS_PH_NOW();
      // ---- backup: every path node at once (lane d <-> depth d) ----
      c_backed.add(depth + 1);
      if constexpr (kLP) {
        if (l <= depth) {  // lane 0 stores the root
          const bool rt = l == 0;
          const int pl = rt ? P0 : (P0 ^ ((l - 1) & 1));
          const uint32_t ix = rt ? 0u : lp.idx;
          Node<R>& nd = nodes[ix];
          const int32_t nn = (rt ? root_n : lp.n) + 1;
          const R nw = (rt ? root_w : lp.w) + (pl == 0 ? rv0 : rv1);
          nd.n = nn;
          nd.w = nw;
          if (nc_.has(ix)) {
            nc_.c[ix].n = nn;
            nc_.c[ix].w = nw;
          }
        }
      } else for (int d0 = 1; d0 <= depth; d0 += 64) {
        const int d = d0 + l;
        if (d <= depth) {
          const PathEnt<R>& pe = path[d];
          const int pl = P0 ^ ((d - 1) & 1);
          Node<R>& nd = nodes[pe.idx];
          nd.n = pe.n + 1;
          nd.w = pe.w + (pl == 0 ? rv0 : rv1);
          if (nc_.has(pe.idx)) {
            nc_.c[pe.idx].n = pe.n + 1;
            nc_.c[pe.idx].w = pe.w + (pl == 0 ? rv0 : rv1);
          }
        }
      }
      root_n += 1;
      root_logN = sp.log_lut[root_n];  // next simulation's root scan
      root_w += P0 == 0 ? rv0 : rv1;
#if OS_MIRROR_SEL
      if (!WW::kTwoSlots) {  // by selects: every lane reloads its log(n)
        const bool me = depth >= 1 && l == root_k;
        rc0.n += me ? 1 : 0;
        rc0.w += me ? (P0 == 0 ? rv0 : rv1) : R(0);
        rlg0 = sp.log_lut[rc0.n];
      } else
#endif
      if (depth >= 1 && l == (root_k & 63)) {  // mirror of path[1]'s update
        if (root_k < 64) {
          rc0.n += 1;
          rc0.w += P0 == 0 ? rv0 : rv1;
          rlg0 = sp.log_lut[rc0.n];
        } else {
          rc1.n += 1;
          rc1.w += P0 == 0 ? rv0 : rv1;
          rlg1 = sp.log_lut[rc1.n];
        }
      }
      if (!kLP && l == 0) {
        nodes[0].n = root_n;
        nodes[0].w = root_w;
        if (kCache != 0) {
          nc_.c[0].n = root_n;
          nc_.c[0].w = root_w;
        }
      }
      OS_PH_ADD(ph.c[kPhBackup], t_ph);
      t_ph = OS_PH_NOW();
      // ---- MCTS-Solver (serial up the path, children reduced across lanes)
      if (solved) {
        uint32_t prev_idx = cur_idx;
        int8_t prev_out = leaf_out;
        for (int d = depth - 1; d >= 0; --d) {
          uint32_t nfirst, nidx;
          int nnc;
          if (d == 0) {
            nfirst = root_first;
            nnc = root_nc;
            nidx = 0;
          } else if constexpr (kLP) {
            nfirst = rl32(lp.first, d);
            nnc = rli(lp.nc, d);
            nidx = rl32(lp.idx, d);
          } else {
            const PathEnt<R>& pe = path[d];
            nfirst = pe.first;
            nnc = pe.nc;
            nidx = pe.idx;
          }
          if (nnc == 0) continue;  // unreachable: path nodes below have children
          const int cpl = P0 ^ (d & 1);
          c_solver.add(nnc);
          bool any_unsolved = false;
          int best_v = -128;
          for (int h = 0; h < (WW::kTwoSlots ? 2 : 1); ++h) {
            const int k = l + 64 * h;
            int8_t co = kUnsolved;
            if (k < nnc) {
              co = (nfirst + k == prev_idx)
                       ? prev_out
                       : (d == 0 ? (h == 0 ? rc0.out : rc1.out)
                                 : (nc_.block(nfirst, nnc) ? nc_.c[nfirst + k].out
                                                           : nodes[nfirst + k].out));
            }
            const bool uns = k < nnc && co == kUnsolved;
            if (ballot(uns)) any_unsolved = true;
            const int v = (k < nnc && co != kUnsolved) ? (cpl == 0 ? co : -co) : -128;
            // Solved values are -1 / 0 / +1: the maximum by three ballots.
            const int m = ballot(v == 1) ? 1 : (ballot(v == 0) ? 0 : (ballot(v == -1) ? -1 : -128));
            if (m > best_v) best_v = m;
          }
          if (best_v > -128 && (!any_unsolved || best_v == 1)) {
            const int8_t no = static_cast<int8_t>(cpl == 0 ? best_v : -best_v);
            if (l == 0) {
              nodes[nidx].out = no;
              if (nc_.has(nidx)) nc_.c[nidx].out = no;
            }
            if (d == 0) root_out = no;
            if (d == 1 && l == (root_k & 63)) {
              if (root_k < 64) rc0.out = no;
              else rc1.out = no;
            }
            prev_idx = nidx;
            prev_out = no;
          } else {
            break;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    OS_PH_ADD(ph.c[kPhSolver], t_ph);
    t_ph = OS_PH_NOW();
    res.sims = sim + 1;
    if (root_out != kUnsolved) break;
    if (Policy == kPolicyCpp) {
      if (root_nc == 1) break;
      if (sp.max_nodes > 1 && nodes_count >= sp.max_nodes) {
        int st = kOk;
        if (l == 0) st = garbage_collect(nodes, used, cap, gc_limit, &nodes_count);
        st = rli(st, 0);
        nodes_count = rli(nodes_count, 0);
        if (st != kOk) {
          res.status = st;
          goto done;
        }
        res.gc_runs++;
        gc_limit = static_cast<int>(gc_limit *
                                    (nodes_count > sp.max_nodes / 2 ? 1.25 : 0.9));
        if (gc_limit < 5) gc_limit = 5;
        __threadfence_block();
        if (kCache != 0) {  // GC rewrote nchild fields: refresh the LDS copy
          const int lim = kCache == kCacheAll ? static_cast<int>(cap) : kCache;
          for (int i = l; i < lim && i < static_cast<int>(used); i += 64) nc_.c[i] = nodes[i];
          __builtin_amdgcn_wave_barrier();
        }
        root_nc = nodes[0].nchild;
        root_first = nodes[0].first;
        // GC may have detached root children's subtrees: reload the mirror.
        rc0 = l < root_nc ? nodes[root_first + l] : zero_node;
        rc1 = WW::kTwoSlots && l + 64 < root_nc ? nodes[root_first + l + 64] : zero_node;
        rlg0 = sp.log_lut[rc0.n];
        rlg1 = sp.log_lut[rc1.n];
      }
    }
    OS_PH_ADD(ph.c[kPhTail], t_ph);
  }
done:
  if (kPace) pacer.end();
  OS_PH_ADD(ph.c[kPhTotal], t_begin);
  res.scanned = c_scanned.get();
  res.backed = c_backed.get();
  res.expanded = c_expanded.get();
  res.solver_scanned = c_solver.get();
  res.max_depth = static_cast<int32_t>(c_depth.get());
  res.nodes = nodes_count;
  res.used = 1 + res.expanded;  // nodes allocated (== used on the reserved arena)
  return res;
}

}  // namespace osm

#endif  // OS_WAVE_H_
