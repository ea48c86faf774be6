// Device-side (and host-side) state machines for the five target games, as
// SoA bitboards.  One implementation per rule set, compiled for gfx950 (the
// search kernel) and for the host (the pyspiel-compatible State API).
//
// Each game G provides, with S = G::State:
//   init(S&, cfg)                       initial position
//   terminal(const S&, cfg)             State::IsTerminal
//   to_move(const S&)                   CurrentPlayer() for non-terminal S
//   Legal legal(const S&, cfg, ctx)     LegalActions() as masks: .count, kth(k)
//   apply(S&, cfg, ctx, action)         State::DoApplyAction
//   ret0(const S&, cfg, ctx)            Returns()[0] at a terminal state
// Legal actions enumerate in ascending action order, exactly as the
// reference's LegalActions() (verified against the playthrough goldens).
//
// Reference rules restated:
//   tic_tac_toe   open_spiel/games/tic_tac_toe.cc:80-150
//   connect_four  open_spiel/games/connect_four.cc:85-185
//   breakthrough  open_spiel/games/breakthrough.cc:119-320
//   hex           open_spiel/games/hex.cc:55-255
//   go            open_spiel/games/go.cc:124-216, go/go_board.cc:217-597
//   pig           open_spiel/games/pig.cc:81-244 (2..10 players; chance nodes)
// Games with chance nodes (G::kHasChance) also provide
//   chance(const S&)                    IsChanceNode()
//   chance_count(cfg), chance_prob(cfg) ChanceOutcomes(): actions kth(0..count)
//                                       of legal(), each with chance_prob
// and to_move() is -1 (kChancePlayerId) at a chance node.
#ifndef OS_GAMES_H_
#define OS_GAMES_H_

#include "os_common.h"

namespace osm {

enum GameKind : int32_t {
  kTicTacToe = 0,
  kConnectFour = 1,
  kBreakthrough = 2,
  kHex = 3,
  kGo = 4,
  kPig = 5,
};

// Runtime game parameters plus precomputed masks.  POD: copied by value into
// kernels.
struct GameCfg {
  int32_t kind;
  int32_t rows, cols;         // breakthrough rows/cols; hex/go: n x n
  int32_t num_actions;        // NumDistinctActions()
  int32_t max_children;       // upper bound on |LegalActions()|
  int32_t max_game_length;    // MaxGameLength()
  float komi;
  int32_t handicap;
  int32_t pig_dice, pig_horizon, pig_win;         // pig diceoutcomes / horizon / winscore
  int32_t pig_players;                            // pig players (2..10)
  uint64_t board64, notcol0_64, notcollast_64;   // breakthrough (<= 64 cells)
  B128 board, notcol0, notcollast;               // hex / go (<= 128 cells)
  // Hex side-neighbour masks.  Equal to notcol0 / notcollast except on n = 2,
  // where the reference's wrap filter (hex.cc:206-222) also drops the genuine
  // left/right and diagonal neighbours, leaving only up/down.
  B128 hex_a, hex_b;
  // The same masks for boards above 11 x 11 (B384; host State API only).
  B384 big_board, big_notcol0, big_notcollast, big_hex_a, big_hex_b;
};

// Board masks of a GameCfg for the bitboard width B.
template <class B>
struct CfgMasks;
template <>
struct CfgMasks<B128> {
  OS_HD static const B128& board(const GameCfg& g) { return g.board; }
  OS_HD static const B128& notcol0(const GameCfg& g) { return g.notcol0; }
  OS_HD static const B128& notcollast(const GameCfg& g) { return g.notcollast; }
  OS_HD static const B128& hex_a(const GameCfg& g) { return g.hex_a; }
  OS_HD static const B128& hex_b(const GameCfg& g) { return g.hex_b; }
};
template <>
struct CfgMasks<B96> {  // the low 96 cells of the B128 masks (go up to 9 x 9)
  OS_HD static B96 board(const GameCfg& g) { return b96_of(g.board); }
  OS_HD static B96 notcol0(const GameCfg& g) { return b96_of(g.notcol0); }
  OS_HD static B96 notcollast(const GameCfg& g) { return b96_of(g.notcollast); }
};
template <>
struct CfgMasks<B384> {
  OS_HD static const B384& board(const GameCfg& g) { return g.big_board; }
  OS_HD static const B384& notcol0(const GameCfg& g) { return g.big_notcol0; }
  OS_HD static const B384& notcollast(const GameCfg& g) { return g.big_notcollast; }
  OS_HD static const B384& hex_a(const GameCfg& g) { return g.big_hex_a; }
  OS_HD static const B384& hex_b(const GameCfg& g) { return g.big_hex_b; }
};

struct NoCtx {
  OS_HD void reset() {}
  OS_HD int mark() const { return 0; }
  OS_HD void rewind(int) {}
};

// ----------------------------------------------------------------------------
// tic_tac_toe: 3x3, bit = cell, x = player 0 first.
struct TicTacToe {
  struct State {
    uint16_t b[2];
    uint8_t to_play;
    int8_t winner;  // -1 none
    uint8_t moves;
    uint8_t pad;
    static constexpr bool kNeedsLog = false;
  };
  using Ctx = NoCtx;
  struct Legal {
    uint32_t mask;
    int count;
    OS_HD int kth(int k) const { return select64(mask, k); }
  };
  OS_HD static bool line(uint32_t b) {
    const uint32_t L[8] = {0007, 0070, 0700, 0111, 0222, 0444, 0421, 0124};
    bool r = false;
    for (int i = 0; i < 8; ++i) r |= (b & L[i]) == L[i];
    return r;
  }
  OS_HD static void init(State& s, const GameCfg&) {
    s.b[0] = s.b[1] = 0; s.to_play = 0; s.winner = -1; s.moves = 0; s.pad = 0;
  }
  OS_HD static bool terminal(const State& s, const GameCfg&) {
    return s.winner >= 0 || s.moves == 9;
  }
  OS_HD static int to_move(const State& s) { return s.to_play; }
  OS_HD static Legal legal(const State& s, const GameCfg&, Ctx&) {
    Legal l;
    l.mask = 0x1FFu & ~(static_cast<uint32_t>(s.b[0]) | s.b[1]);
    l.count = popc64(l.mask);
    return l;
  }
  OS_HD static void apply(State& s, const GameCfg&, Ctx&, int a) {
    const int p = s.to_play;
    const uint16_t mine = static_cast<uint16_t>(pick(s.b, p) | (1u << a));
    put(s.b, p, mine);
    if (line(mine)) s.winner = static_cast<int8_t>(p);
    s.to_play = static_cast<uint8_t>(1 - p);
    s.moves++;
  }
  OS_HD static int ret0(const State& s, const GameCfg&, Ctx&) {
    return s.winner == 0 ? 1 : (s.winner == 1 ? -1 : 0);
  }
  // ObservationTensor (tic_tac_toe.cc:165-175): [3][3][3], plane = CellState
  // {empty, nought (player 1), cross (player 0)}; not player-relative.
  static constexpr int kObsPlanes = 3;
  OS_HD static float obs(const State& s, const GameCfg&, int, int plane, int cell) {
    const int want = (s.b[0] >> cell) & 1 ? 2 : ((s.b[1] >> cell) & 1 ? 1 : 0);
    return plane == want ? 1.0f : 0.0f;
  }
};

// ----------------------------------------------------------------------------
// connect_four: 6 rows x 7 cols, column-major bitboard, 7 bits per column
// (6 cells + an always-empty sentinel), bit = col * 7 + row, row 0 = bottom.
struct ConnectFour {
  // Dword fields (no byte packing on the scalar unit); `legal` is the
  // playable-column mask kept incrementally by apply().
  struct State {
    uint64_t bb[2];
    int32_t to_play;
    int32_t outcome;  // -1 unknown, 0/1 winner, 2 draw
    int32_t moves;
    uint32_t legal;   // bit c = column c not full (LegalActions, ascending)
    static constexpr bool kNeedsLog = false;
  };
  using Ctx = NoCtx;
  static constexpr uint64_t kTopRow = 0x20ull | (0x20ull << 7) | (0x20ull << 14) |
                                      (0x20ull << 21) | (0x20ull << 28) |
                                      (0x20ull << 35) | (0x20ull << 42);
  struct Legal {
    uint32_t mask;  // bit c = column c playable
    int count;
    // k-th set bit of a <= 7-bit mask: drop the k lowest bits.
    OS_HD int kth(int k) const {
      uint32_t m = mask;
      for (int i = 0; i < k; ++i) m &= m - 1;
      return ctz64(m);
    }
  };
  // Four in a row in any direction (column, row, both diagonals).  Early-exit
  // form: measured 3-7% faster in the wave kernel than a branch-free OR of
  // the four tests (profiles/r01/ab_uniform.txt).
  OS_HD static bool has_four(uint64_t b) {
    uint64_t m = b & (b >> 1);
    if (m & (m >> 2)) return true;
    m = b & (b >> 7);
    if (m & (m >> 14)) return true;
    m = b & (b >> 6);
    if (m & (m >> 12)) return true;
    m = b & (b >> 8);
    if (m & (m >> 16)) return true;
    return false;
  }
  OS_HD static void init(State& s, const GameCfg&) {
    s.bb[0] = s.bb[1] = 0; s.to_play = 0; s.outcome = -1; s.moves = 0; s.legal = 0x7f;
  }
  OS_HD static bool terminal(const State& s, const GameCfg&) { return s.outcome >= 0; }
  OS_HD static int to_move(const State& s) { return s.to_play; }
  OS_HD static Legal legal(const State& s, const GameCfg&, Ctx&) {
    Legal l;
    l.mask = s.legal;
    l.count = popc64(s.legal);
    return l;
  }
  OS_HD static void apply(State& s, const GameCfg&, Ctx&, int col) {
    const int p = s.to_play;
    const uint64_t occ = s.bb[0] | s.bb[1];
    const uint64_t colmask = 0x3Full << (7 * col);
    const uint64_t mv = (occ + (1ull << (7 * col))) & colmask;
    const uint64_t mine = pick(s.bb, p) | mv;
    put(s.bb, p, mine);
    s.moves++;
    if (mv & kTopRow) s.legal &= ~(1u << col);  // column now full
    if (has_four(mine)) s.outcome = p;
    else if (s.moves == 42) s.outcome = 2;
    s.to_play = 1 - p;
  }
  OS_HD static int ret0(const State& s, const GameCfg&, Ctx&) {
    return s.outcome == 0 ? 1 : (s.outcome == 1 ? -1 : 0);
  }
  // ObservationTensor(player) (connect_four.cc:211-221): [3][6][7], tensor
  // cell = row * 7 + col with row 0 at the bottom; PlayerRelative (:198-209)
  // puts the OPPONENT's stones in plane 0, the player's own in plane 1, empty
  // cells in plane 2.
  static constexpr int kObsPlanes = 3;
  OS_HD static float obs(const State& s, const GameCfg&, int player, int plane, int cell) {
    const int bit = (cell % 7) * 7 + cell / 7;
    const int q = (s.bb[0] >> bit) & 1 ? 0 : ((s.bb[1] >> bit) & 1 ? 1 : -1);
    const int want = q < 0 ? 2 : (q == player ? 1 : 0);
    return plane == want ? 1.0f : 0.0f;
  }
};

// ----------------------------------------------------------------------------
// breakthrough: rows x cols <= 64, bit = r * cols + c.  Black (player 0)
// starts on rows 0-1 and moves +row; white on the last two rows, -row.
// Action = ((r * cols + c) * 6 + dir) * 2 + capture (mixed base, as
// spiel_utils.cc:45-73 RankActionMixedBase over {rows, cols, 6, 2}).
struct Breakthrough {
  struct State {
    uint64_t pc[2];
    uint8_t to_play;
    int8_t winner;  // -1 none
    uint16_t moves;
    uint32_t pad;
    static constexpr bool kNeedsLog = false;
  };
  using Ctx = NoCtx;
  struct Legal {
    uint64_t L, F, R;  // source squares with a legal left/forward/right move
    int count;
    int player;
    OS_HD int cnt_below(int s) const {  // actions with source < s
      const uint64_t pre = s >= 64 ? ~0ull : ((1ull << s) - 1);
      return popc64(L & pre) + popc64(F & pre) + popc64(R & pre);
    }
    OS_HD int kth(int k) const {
      int lo = 0;
      for (int step = 32; step >= 1; step >>= 1)
        if (cnt_below(lo + step) <= k) lo += step;
      int rem = k - cnt_below(lo);
      const uint64_t bit = 1ull << lo;
      int o;
      if (L & bit) { if (rem == 0) { o = 0; goto done; } --rem; }
      if (F & bit) { if (rem == 0) { o = 1; goto done; } --rem; }
      o = 2;
    done:
      return ((lo * 6 + player * 3 + o) << 1) | (o != 1 ? cap_bit(lo, o) : 0);
    }
    uint64_t opp;
    int cols;
    OS_HD int cap_bit(int src, int o) const {
      int t = player == 0 ? src + cols + (o == 0 ? -1 : 1)
                          : src - cols + (o == 0 ? -1 : 1);
      return static_cast<int>((opp >> t) & 1);
    }
  };
  OS_HD static void init(State& s, const GameCfg& g) {
    const bool two = g.rows >= 6;
    uint64_t black = 0, white = 0;
    for (int c = 0; c < g.cols; ++c) {
      black |= 1ull << c;
      white |= 1ull << ((g.rows - 1) * g.cols + c);
      if (two) {
        black |= 1ull << (g.cols + c);
        white |= 1ull << ((g.rows - 2) * g.cols + c);
      }
    }
    s.pc[0] = black; s.pc[1] = white;
    s.to_play = 0; s.winner = -1; s.moves = 0; s.pad = 0;
  }
  OS_HD static bool terminal(const State& s, const GameCfg&) {
    return s.winner >= 0 || s.pc[0] == 0 || s.pc[1] == 0;
  }
  OS_HD static int to_move(const State& s) { return s.to_play; }
  OS_HD static Legal legal(const State& s, const GameCfg& g, Ctx&) {
    const int p = s.to_play;
    const uint64_t own = pick(s.pc, p), opp = pick(s.pc, 1 - p);
    const uint64_t E = g.board64 & ~(own | opp);
    const uint64_t EO = E | opp;
    const int c = g.cols;
    Legal l;
    if (p == 0) {
      l.L = own & g.notcol0_64 & (EO >> (c - 1));
      l.F = own & (E >> c);
      l.R = own & g.notcollast_64 & (EO >> (c + 1));
    } else {
      l.L = own & g.notcol0_64 & (EO << (c + 1));
      l.F = own & (E << c);
      l.R = own & g.notcollast_64 & (EO << (c - 1));
    }
    l.count = popc64(l.L) + popc64(l.F) + popc64(l.R);
    l.player = p;
    l.opp = opp;
    l.cols = c;
    return l;
  }
  OS_HD static void apply(State& s, const GameCfg& g, Ctx&, int a) {
    const int p = s.to_play;
    const int sq = a >> 1;
    const int dir = sq % 6;
    const int src = sq / 6;
    const int dr = dir < 3 ? 1 : -1;
    const int dc = (dir % 3) - 1;
    const int tgt = src + dr * g.cols + dc;
    const uint64_t tb = 1ull << tgt;
    const uint64_t own = (pick(s.pc, p) & ~(1ull << src)) | tb;
    const uint64_t opp = pick(s.pc, 1 - p) & ~tb;
    s.pc[0] = p ? opp : own;
    s.pc[1] = p ? own : opp;
    const int trow = tgt / g.cols;
    if (p == 0 && trow == g.rows - 1) s.winner = 0;
    else if (p == 1 && trow == 0) s.winner = 1;
    s.to_play = static_cast<uint8_t>(1 - p);
    s.moves++;
  }
  OS_HD static int ret0(const State& s, const GameCfg&, Ctx&) {
    if (s.winner == 0 || s.pc[1] == 0) return 1;
    if (s.winner == 1 || s.pc[0] == 0) return -1;
    return 0;
  }
  // ObservationTensor (breakthrough.cc:326-340, planes :284-300):
  // [3][rows][cols], {black, white, empty}; not player-relative.
  static constexpr int kObsPlanes = 3;
  OS_HD static float obs(const State& s, const GameCfg&, int, int plane, int cell) {
    const int want = (s.pc[0] >> cell) & 1 ? 0 : ((s.pc[1] >> cell) & 1 ? 1 : 2);
    return plane == want ? 1.0f : 0.0f;
  }
};

// ----------------------------------------------------------------------------
// Hex: n x n <= 128 cells, row-major, bit = cell.  Black (player 0) joins
// north-south, white west-east.  Per player: stones, and the stones whose
// group touches edge A (north / west) or edge B (south / east) -- the bitboard
// form of the reference's per-cell edge labels (hex.cc:55-134, flood :149-184).
template <class B>
struct HexT {
  using M = CfgMasks<B>;
  struct State {
    B st[2];
    B ea[2];
    B eb[2];
    int16_t win_cell;  // -1 none
    int8_t result;     // +1 black won, -1 white won, 0 running
    uint8_t to_play;
    uint16_t moves;
    uint16_t pad;
    static constexpr bool kNeedsLog = false;
  };
  using Ctx = NoCtx;
  struct Legal {
    B mask;
    int count;
    OS_HD int kth(int k) const { return BB<B>::select(mask, k); }
  };
  OS_HD static B nbr6(B x, const GameCfg& g) {
    const int n = g.rows;
    B r = shr(x, n) | (shr(x, n - 1) & M::hex_a(g)) | (shr(x, 1) & M::hex_b(g)) |
             (shl(x, 1) & M::hex_a(g)) | (shl(x, n - 1) & M::hex_b(g)) | shl(x, n);
    return r & M::board(g);
  }
  OS_HD static void init(State& s, const GameCfg&) {
    s.st[0] = s.ea[0] = s.eb[0] = BB<B>::zero();
    s.st[1] = s.ea[1] = s.eb[1] = BB<B>::zero();
    s.win_cell = -1; s.result = 0; s.to_play = 0; s.moves = 0; s.pad = 0;
  }
  OS_HD static bool terminal(const State& s, const GameCfg&) { return s.result != 0; }
  OS_HD static int to_move(const State& s) { return s.to_play; }
  OS_HD static Legal legal(const State& s, const GameCfg& g, Ctx&) {
    Legal l;
    l.mask = M::board(g) & ~(s.st[0] | s.st[1]);
    l.count = popc(l.mask);
    return l;
  }
  // Edge flags the stone would get if player p played cell m (hex.cc:55-134).
  OS_HD static void edges_if(const State& s, const GameCfg& g, int p, int m,
                             bool* a, bool* b) {
    const int n = g.rows;
    bool ea, eb;
    if (p == 0) {
      ea = m < n;
      eb = !ea && m >= n * (n - 1);
    } else {
      ea = (m % n) == 0;
      eb = !ea && (m % n) == n - 1;
    }
    const B nb = nbr6(BB<B>::bit(m), g);
    ea |= any(nb & pick(s.ea, p));
    eb |= any(nb & pick(s.eb, p));
    *a = ea;
    *b = eb;
  }
  OS_HD static void apply(State& s, const GameCfg& g, Ctx&, int m) {
    const int p = s.to_play;
    bool a, b;
    edges_if(s, g, p, m, &a, &b);
    const B mb = BB<B>::bit(m);
    const B st = pick(s.st, p) | mb;
    put(s.st, p, st);
    if (a && b) {
      s.result = static_cast<int8_t>(p == 0 ? 1 : -1);
      s.win_cell = static_cast<int16_t>(m);
    } else if (a || b) {
      const B ea = pick(s.ea, p), eb = pick(s.eb, p);
      const B plain = st & ~ea & ~eb;
      B comp = mb;
      for (;;) {
        B nx = comp | (nbr6(comp, g) & plain);
        if (nx == comp) break;
        comp = nx;
      }
      // Both pairs are written on this path (no store sinking through a
      // pointer phi, which would pin the state in scratch).
      put(s.ea, p, BB<B>::sel(a, ea | comp, ea));
      put(s.eb, p, BB<B>::sel(a, eb, eb | comp));
    }
    s.to_play = static_cast<uint8_t>(1 - p);
    s.moves++;
  }
  OS_HD static int ret0(const State& s, const GameCfg&, Ctx&) { return s.result; }
  // ObservationTensor (hex.cc:266-277): [9][n][n], plane = CellState + 4
  // (hex.h:40-61): white win 0, west 1, east 2, plain 3, empty 4, black
  // plain 5, south 6, north 7, win 8.  Edge A = north / west, B = south /
  // east; the winning stone keeps its win label (no flood, hex.cc:149-156).
  static constexpr int kObsPlanes = 9;
  OS_HD static float obs(const State& s, const GameCfg&, int, int plane, int cell) {
    int want = 4;
    for (int p = 0; p < 2; ++p) {
      if (!test(pick(s.st, p), cell)) continue;
      const int sgn = p == 0 ? 1 : -1;
      const int label = cell == s.win_cell ? 4 : (test(pick(s.ea, p), cell) ? 3
                                                  : (test(pick(s.eb, p), cell) ? 2 : 1));
      want = 4 + sgn * label;
    }
    return plane == want ? 1.0f : 0.0f;
  }
};
using Hex = HexT<B128>;
using HexBig = HexT<B384>;  // board_size 12..19 (host State API)

// ----------------------------------------------------------------------------
// Go: n x n <= 121 cells (board_size <= 11), row-major bit = row * n + col
// (the concrete OpenSpiel action id), pass = n * n.  Chains are recomputed by
// bitboard flood fills instead of the reference's pseudo-liberty chain lists;
// on n <= 11 the reference's `in_atari` test (go_board.h:208-212) is exact
// (no u16/u32 wrap) and equals "exactly one distinct liberty", so legality is
// identical.  Positional superko follows go.cc:199-208 with the same Zobrist
// hashes (chess_common.h ZobristTable, seed 2765481) compared for equality.
// 256-bit membership pre-filter (bit = hash >> 56), kept in four named words
// so it stays in registers.
struct Filter256 {
  uint64_t w0, w1, w2, w3;
  OS_HD void clear() { w0 = w1 = w2 = w3 = 0; }
  OS_HD bool has(int b) const {
    const int q = b >> 6;
    const uint64_t w = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
    return (w >> (b & 63)) & 1;
  }
  OS_HD void add(int b) {
    const int q = b >> 6;
    const uint64_t m = 1ull << (b & 63);
    w0 |= q == 0 ? m : 0;
    w1 |= q == 1 ? m : 0;
    w2 |= q == 2 ? m : 0;
    w3 |= q == 3 ? m : 0;
  }
};

// Positional-superko set of one playout / simulation (go.cc:199-208).
// Two positions can only be equal if they have the same number of stones, so
// the log is bucketed by stone count: head[k] is the last entry with k stones
// (+ 1, 0 = none) and link[e] holds entry e's stone count (high half) and the
// previous entry + 1 with the same count (low half).  A new position is compared only with its own bucket -- in random
// playouts under one entry on average, against ~50 candidates for a linear
// scan -- and the buckets give the same answers as testing the whole set.
// Positions before the root (`base`, counts unknown) are scanned behind a
// 256-bit pre-filter.  Arrays may be batch-SoA: element i at [i * stride].
#ifndef OS_GO_NOWALK
#define OS_GO_NOWALK 0
#endif
// Two filter bits per position before the root (1) or one (0).  A lane whose
// hash hits the filter scans the root's history with dependent loads, and the
// wave waits for it: with one bit and a 7-position history a lane hits on ~3%
// of its moves, so at 32 lanes most moves carry some lane's scan; two bits
// make it ~0.2%.  A/B knob; exact either way (a miss proves absence).
#ifndef OS_GO_BASE_FILT2
#define OS_GO_BASE_FILT2 1
#endif
// Contexts of wave-uniform code (GoWaveCtx) declare kWaveUniform.
template <class C, class = void>
struct WaveUniformCtx : std::false_type {};
template <class C>
struct WaveUniformCtx<C, std::void_t<decltype(C::kWaveUniform)>> : std::true_type {};
// OS_GO_LOG_BLOOM: the lane kernels' go superko logs (k_rollouts, k_lsearch)
// keep a 512-bit Bloom filter per lane in LDS in front of the bucket walk
// (GoCtxT::bloom; exact).  A timing A/B without the walk at all
// (OS_GO_NOWALK, not exact) put the walk at 10% of C5 and 17% of g9.
#ifndef OS_GO_LOG_BLOOM
#define OS_GO_LOG_BLOOM 1
#endif
// L: link word.  uint32_t keeps the stone count for rewind (the searches);
// a rollout-only context (k_rollouts, never rewound) stores the uint16_t
// link alone: 2 B less HBM write per logged move.
template <class H, class L = uint32_t, int kBW = 16>
struct GoCtxT {
  const uint64_t* zob;     // [n*n][2] Zobrist values per (cell, colour)
  const uint64_t* base;    // hashes of positions before this search's root
  int32_t n_base;
  uint64_t* log;           // hashes added since the root (capacity cap)
  L* link;                 // [cap] (stone count << 16 |) previous same-count entry + 1
  H* head;                 // [n_heads] last entry + 1 with k stones (cap <= max of H)
  int32_t stride;          // SoA stride of log / link (1: contiguous)
  int32_t head_stride;     // stride of head (k_rollouts: LDS, 64 lanes)
  int32_t n_log;
  int32_t cap;
  int32_t n_heads;         // cells + 1
  Filter256 base_filt;     // base hashes
  // Optional Bloom filter over the log (kBloomWords words, word w at
  // bloom[w * head_stride]; nullptr: none).  A position whose bucket is not
  // empty is compared with it only when both of its filter bits are set --
  // a miss proves absence, so the answers stay exact -- which spares most of
  // the bucket walks' dependent HBM reads (k_rollouts / k_lsearch keep it in
  // LDS next to the bucket heads).
  uint32_t* bloom = nullptr;
  static constexpr int kBloomWords = kBW;  // kBW * 32 bits, 2 bits per position
  static_assert(kBW == 16 || kBW == 32, "Bloom filter of 512 or 1024 bits");
  static constexpr uint32_t kBloomMask = kBW * 32 - 1;
  static constexpr int kBloomShift = kBW == 32 ? 10 : 9;
  // Optional write-combining of the log (k_lsearch; nullptr: none).  A lane's
  // log entries land in lines no other lane shares, one 12-byte entry per
  // move, so the L2 writes back partly written lines; with wlog / wlink set,
  // the open group of kWg entries lives in LDS (entry e at [(e % kWg) * wst])
  // and goes out as whole 64-byte (hashes) / 32-byte (links) stores once full.
  // Entries below the open group are in memory, those in it only in LDS.
  uint64_t* wlog = nullptr;
  L* wlink = nullptr;
  int32_t wst = 64;
  static constexpr int kWg = 8;

  OS_HD bool in_wbuf(int e) const { return wlog != nullptr && e >= (n_log & ~(kWg - 1)); }
  OS_HD uint64_t log_at(int e) const {
    return in_wbuf(e) ? wlog[(e & (kWg - 1)) * wst] : log[static_cast<int64_t>(e) * stride];
  }
  OS_HD L link_at(int e) const {
    return in_wbuf(e) ? wlink[(e & (kWg - 1)) * wst] : link[static_cast<int64_t>(e) * stride];
  }
  OS_HD void flush_group(int g) {  // entries g .. g + kWg - 1 to memory
#if defined(__HIP_DEVICE_COMPILE__)
    if (stride == 1 && sizeof(L) == 4) {
      uint4* dl = reinterpret_cast<uint4*>(log + g);
#pragma unroll
      for (int q = 0; q < kWg / 2; ++q) {
        const uint64_t a = wlog[(2 * q) * wst], b = wlog[(2 * q + 1) * wst];
        dl[q] = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32),
                           static_cast<uint32_t>(b), static_cast<uint32_t>(b >> 32));
      }
      uint4* dk = reinterpret_cast<uint4*>(link + g);
#pragma unroll
      for (int q = 0; q < kWg / 4; ++q)
        dk[q] = make_uint4(static_cast<uint32_t>(wlink[(4 * q) * wst]),
                           static_cast<uint32_t>(wlink[(4 * q + 1) * wst]),
                           static_cast<uint32_t>(wlink[(4 * q + 2) * wst]),
                           static_cast<uint32_t>(wlink[(4 * q + 3) * wst]));
      return;
    }
#endif
    for (int k = 0; k < kWg; ++k) {
      log[static_cast<int64_t>(g + k) * stride] = wlog[k * wst];
      link[static_cast<int64_t>(g + k) * stride] = wlink[k * wst];
    }
  }

  OS_HD static int bbit0(uint64_t h) { return static_cast<int>(h & kBloomMask); }
  OS_HD static int bbit1(uint64_t h) { return static_cast<int>((h >> kBloomShift) & kBloomMask); }
  OS_HD bool bloom_has(uint64_t h) const {
    const int x = bbit0(h), y = bbit1(h);
    return ((bloom[(x >> 5) * head_stride] >> (x & 31)) & 1u) &&
           ((bloom[(y >> 5) * head_stride] >> (y & 31)) & 1u);
  }
  OS_HD void bloom_add(uint64_t h) {
    const int x = bbit0(h), y = bbit1(h);
    bloom[(x >> 5) * head_stride] |= 1u << (x & 31);
    bloom[(y >> 5) * head_stride] |= 1u << (y & 31);
  }
  OS_HD void bloom_clear() {
    for (int w = 0; w < kBloomWords; ++w) bloom[w * head_stride] = 0u;
  }

  // Empties the log (the base stays).
  OS_HD void reset() {
    n_log = 0;
    for (int k = 0; k < n_heads; ++k) head[k * head_stride] = 0;
    if (bloom) bloom_clear();
  }
  // Builds base_filt from base[0, n_base) and resets.
  OS_HD void init_filters() {
    init_base_filter();
    reset();
  }
  // Builds base_filt only: a resumed search keeps its log (os_az.h).
  OS_HD void init_base_filter() {
    base_filt.clear();
    for (int i = 0; i < n_base; ++i) {
      base_filt.add(fbit(base[i]));
      if (OS_GO_BASE_FILT2) base_filt.add(fbit2(base[i]));
    }
  }
  OS_HD static int fbit(uint64_t h) { return static_cast<int>(h >> 56); }
  OS_HD static int fbit2(uint64_t h) { return static_cast<int>((h >> 48) & 255u); }
  // The pre-filter in front of the scan of the positions before the root:
  // both of a hash's two bits set (OS_GO_BASE_FILT2), or its one bit.
  OS_HD bool base_maybe(uint64_t h) const {
    return base_filt.has(fbit(h)) && (!OS_GO_BASE_FILT2 || base_filt.has(fbit2(h)));
  }
  OS_HD bool contains(uint64_t h, int stones) const {
    if (base_maybe(h))
      for (int i = 0; i < n_base; ++i)
        if (base[i] == h) return true;
#if OS_GO_NOWALK  // timing A/B only (not exact): no bucket walk
    return false;
#endif
    if (bloom && head[stones * head_stride] != 0 && !bloom_has(h)) return false;
#if OS_DEBUG_GOLOG
    int steps = 0;
#endif
    for (int e = head[stones * head_stride]; e; e = static_cast<int>(link_at(e - 1) & 0xFFFFu)) {
#if OS_DEBUG_GOLOG
      if (++steps > cap + 2) {
        printf("golog cycle: stones %d head %d e %d n_log %d link %x\n", stones,
               head[stones * head_stride], e, n_log, link[static_cast<int64_t>(e - 1) * stride]);
        return false;
      }
#endif
      if (log_at(e - 1) == h) return true;
    }
    return false;
  }
  // Log position count, and dropping back to it (each rollout of a leaf
  // starts from the leaf's log, mcts.cc:46-47): the buckets are unlinked in
  // reverse order of insertion.
  OS_HD int mark() const { return n_log; }
  OS_HD void rewind(int m) {
    static_assert(sizeof(L) == 4, "rewind needs the stone count in the link");
    const int g0 = n_log & ~(kWg - 1);  // the open group before the rewind
    while (n_log > m) {
      --n_log;
      const uint32_t lk = (wlog && n_log >= g0) ? wlink[(n_log & (kWg - 1)) * wst]
                                                 : link[static_cast<int64_t>(n_log) * stride];
      head[static_cast<int>(lk >> 16) * head_stride] = static_cast<H>(lk & 0xFFFFu);
    }
    if (wlog) {  // an earlier group is open now: its kept entries back into LDS
      const int g = n_log & ~(kWg - 1);
      if (g < g0)
        for (int e = g; e < n_log; ++e) {
          wlog[(e & (kWg - 1)) * wst] = log[static_cast<int64_t>(e) * stride];
          wlink[(e & (kWg - 1)) * wst] = link[static_cast<int64_t>(e) * stride];
        }
    }
    if (bloom) {  // a Bloom filter cannot forget: rebuilt from the entries kept
      bloom_clear();
      for (int e = 0; e < n_log; ++e) bloom_add(log_at(e));
    }
  }
  // Logs the position after a non-pass move; false if it was already present
  // (go.cc:201-205).
  OS_HD bool insert(uint64_t h, bool captured, int stones) {
    (void)captured;
    if (contains(h, stones)) return false;
    if (n_log < cap) {
      const int64_t e = static_cast<int64_t>(n_log) * stride;
      const int hk = stones * head_stride;
      L lk;
      if constexpr (sizeof(L) == 4)
        lk = (static_cast<uint32_t>(stones) << 16) | head[hk];
      else
        lk = static_cast<L>(head[hk]);
      if (wlog) {
        const int w = (n_log & (kWg - 1)) * wst;
        wlog[w] = h;
        wlink[w] = lk;
      } else {
        log[e] = h;
        link[e] = lk;
      }
      head[hk] = static_cast<H>(n_log + 1);
      if (bloom) bloom_add(h);
      ++n_log;
      if (wlog && (n_log & (kWg - 1)) == 0) flush_group(n_log - kWg);
    }
    return true;
  }
};
// The same set for one random playout (k_rollouts) screened by a per-lane
// Bloom filter instead of stone-count buckets: a new position is compared with
// the log only when both of its filter bits are set, and then only with the
// entries logged before the most recent capture (without a capture the stone
// count only grows, so no later position can repeat one -- go.cc:199-208 asks
// the same question of a hash set).  A filter miss proves absence, so the
// answers are exact; the log is written (8 B per move) but read almost never,
// and no link words are kept.  Filter: kWords u32 per playout (1024 bits),
// word w at filt[w * filt_stride] (LDS, lane-interleaved).  No rewind: each
// playout starts from reset().
struct GoCtxBloom {
  static constexpr int kWords = 32;
  const uint64_t* zob;
  const uint64_t* base;   // hashes before the root
  int32_t n_base;
  uint64_t* log;          // [cap], element i at log[i * stride]
  uint32_t* filt;         // [kWords], element w at filt[w * filt_stride]
  int32_t stride;
  int32_t filt_stride;
  int32_t n_log;
  int32_t cand_end;       // entries [0, cand_end) can repeat a new position
  int32_t cap;
  Filter256 base_filt;

  OS_HD void reset() {
    n_log = 0;
    cand_end = 0;
    for (int w = 0; w < kWords; ++w) filt[w * filt_stride] = 0u;
  }
  OS_HD void init_filters() {
    base_filt.clear();
    for (int i = 0; i < n_base; ++i) base_filt.add(GoCtxT<uint8_t>::fbit(base[i]));
    reset();
  }
  OS_HD static int b0(uint64_t h) { return static_cast<int>(h & 1023u); }
  OS_HD static int b1(uint64_t h) { return static_cast<int>((h >> 10) & 1023u); }
  OS_HD bool contains(uint64_t h) const {
    if (base_filt.has(GoCtxT<uint8_t>::fbit(h)))
      for (int i = 0; i < n_base; ++i)
        if (base[i] == h) return true;
    if (cand_end == 0) return false;
    const int x = b0(h), y = b1(h);
    if (!((filt[(x >> 5) * filt_stride] >> (x & 31)) & 1u)) return false;
    if (!((filt[(y >> 5) * filt_stride] >> (y & 31)) & 1u)) return false;
    for (int e = 0; e < cand_end; ++e)
      if (log[static_cast<int64_t>(e) * stride] == h) return true;
    return false;
  }
  OS_HD bool insert(uint64_t h, bool captured, int stones) {
    (void)stones;
    if (captured) cand_end = n_log;
    if (contains(h)) return false;
    if (n_log < cap) {
      log[static_cast<int64_t>(n_log) * stride] = h;
      const int x = b0(h), y = b1(h);
      filt[(x >> 5) * filt_stride] |= 1u << (x & 31);
      filt[(y >> 5) * filt_stride] |= 1u << (y & 31);
      ++n_log;
    }
    return true;
  }
};

// u8 bucket heads (log cap <= 255: boards up to 11 x 11, and the host's
// one-move logs); u16 heads for the longer logs of larger boards (k_lsearch).
using GoCtx = GoCtxT<uint8_t>;
using GoCtxW = GoCtxT<uint16_t>;

// How GoT::apply keeps the atari set (all three exact):
// 0: every touched chain is flooded to its full extent (the round-3 form);
// 1: chains are flooded only where a liberty count is unknown (see apply) --
//    measured slower on the lane kernels (g9 505 vs 496 ms, C5 15.1 vs
//    14.7 ms, profiles/r04/go_ab/): its three branches diverge across lanes;
// 2: as 1, but one kind of flood for every chain whose count is unknown,
//    which stops as soon as it has seen two liberties (flood_libs2): a chain
//    with two liberties is out of atari whatever its extent, so most floods
//    end after one or two steps instead of the chain's diameter.
#ifndef OS_GO_LAZY_ATARI
#define OS_GO_LAZY_ATARI 2
#endif
// Mode 2's captures and own-chain releases as one multi-seed flood each (1)
// or one flood per chain (0).  A/B knob; the same atari set.
#ifndef OS_GO_APPLY_MS
#define OS_GO_APPLY_MS 1
#endif
// With OS_GO_APPLY_MS: the points with two or more empty neighbours first,
// as one bitboard expression (1), or every flood_libs2 from its seed (0).
// Measured slower on g9 (348 -> 356 ms; C5 equal, profiles/r06/tl/): the
// expression costs every move what the floods it spares cost a few.
#ifndef OS_GO_TWO_LIB
#define OS_GO_TWO_LIB 0
#endif

template <class B>
struct GoT {
  using M = CfgMasks<B>;
  struct State {
    B bw[2];     // black, white stones
    B atari;     // stones (both colours) whose chain has exactly one liberty
    uint64_t hash;  // Zobrist hash of the stones
    int16_t ko;     // ko cell or -1
    uint16_t moves; // history length (since the empty board)
    uint8_t to_play;
    uint8_t flags;  // bit0 superko, bit1 last action pass, bit2 previous pass
    uint16_t pad;
    static constexpr bool kNeedsLog = true;
  };
  using Ctx = GoCtx;
  static constexpr uint8_t kSuperko = 1, kLastPass = 2, kPrevPass = 4;

  OS_HD static B nbr4(B x, const GameCfg& g) {
    const int n = g.rows;
    B r = shl(x, n) | shr(x, n) | (shl(x, 1) & M::notcol0(g)) | (shr(x, 1) & M::notcollast(g));
    return r & M::board(g);
  }
  OS_HD static B flood(B seed, B within, const GameCfg& g) {
    B c = seed;
    for (;;) {
      B nx = (c | nbr4(c, g)) & within;
      if (nx == c) return c;
      c = nx;
    }
  }
  // The chain of `seed` within `within`, grown until it is complete or shows
  // two liberties (empty points of E next to it).  Returns the stones reached;
  // *libs = the liberties seen: when popc(*libs) < 2 the chain is complete and
  // *libs are all its liberties.
  OS_HD static B flood_libs2(B seed, B within, B E, const GameCfg& g, B* libs) {
    B c = seed;
    for (;;) {
      const B n4 = nbr4(c, g);
      *libs = n4 & E;
      if (popc(*libs) >= 2) return c;
      const B nx = (c | n4) & within;
      if (nx == c) return c;
      c = nx;
    }
  }
  struct Legal {
    B mask;  // legal board points (pass excluded)
    int count;  // including pass
    int pass_action;
    OS_HD int kth(int k) const {
      const int c = count - 1;
      return k < c ? BB<B>::select(mask, k) : pass_action;
    }
    // act[k] = kth(k) for every k < count: one walk over the set bits (a
    // lowest-bit step per action) instead of a select per action.
    template <class A>
    OS_HD void fill(A& act) const {
      B m = mask;
      int k = 0;
      while (any(m)) {
        const int b = lowest(m);
        act[k++] = static_cast<uint16_t>(b);
        m = m & ~BB<B>::bit(b);
      }
      act[k] = static_cast<uint16_t>(pass_action);
    }
  };
  OS_HD static void init(State& s, const GameCfg&) {
    s.bw[0] = s.bw[1] = s.atari = BB<B>::zero();
    s.hash = 0; s.ko = -1; s.moves = 0; s.to_play = 0; s.flags = 0; s.pad = 0;
  }
  OS_HD static bool terminal(const State& s, const GameCfg& g) {
    if (s.moves < 2) return false;
    return s.moves >= g.max_game_length || (s.flags & kSuperko) ||
           ((s.flags & kLastPass) && (s.flags & kPrevPass));
  }
  OS_HD static int to_move(const State& s) { return s.to_play; }
  template <class C>
  OS_HD static Legal legal(const State& s, const GameCfg& g, C&) {
    const int c = s.to_play;
    const B E = M::board(g) & ~(s.bw[0] | s.bw[1]);
    B cand = E;
    if (s.ko >= 0) cand = cand & ~BB<B>::bit(s.ko);
    // A point with an empty neighbour is legal; a surrounded one iff it joins
    // an own chain that keeps a liberty (>= 2 now) or captures an opponent
    // chain in atari (go_board.cc:425-440).  Every stone's chain has >= 1
    // liberty, so with the atari set both are masks ("good" stones), and
    // cand & (nbr4(E) | nbr4(good)) is one neighbourhood: cand & nbr4(E | good).
    B mask;
    if constexpr (WaveUniformCtx<C>::value) {
      // Wave-uniform (scalar unit): the second neighbourhood only when some
      // point is surrounded -- rare near the root, where the wave search's
      // tree positions are (3% faster there; the lanes prefer one form).
      const B has_lib = nbr4(E, g);
      mask = cand & has_lib;
      const B hard = cand & ~has_lib;
      if (any(hard)) {
        const B own = pick(s.bw, c), opp = pick(s.bw, 1 - c);
        const B good = (own & ~s.atari) | (opp & s.atari);
        mask = mask | (hard & nbr4(good, g));
      }
    } else {
      const B own = pick(s.bw, c), opp = pick(s.bw, 1 - c);
      const B good = (own & ~s.atari) | (opp & s.atari);
      mask = cand & nbr4(E | good, g);
    }
    Legal l;
    l.mask = mask;
    l.count = popc(mask) + 1;
    l.pass_action = g.rows * g.cols;
    return l;
  }
  // C: GoCtx (one search per lane) or a wave-parallel context with the same
  // zob / insert() interface (os_wave.h).
  template <class C>
  OS_HD static void apply(State& s, const GameCfg& g, C& ctx, int a) {
    const int c = s.to_play;
    const int pass = g.rows * g.cols;
    s.flags = static_cast<uint8_t>((s.flags & kSuperko) | ((s.flags & kLastPass) ? kPrevPass : 0));
    if (a == pass) {
      s.ko = -1;
      s.flags |= kLastPass;
      // Hash unchanged: the repetition insert is a no-op for a pass.
    } else {
      const B pb = BB<B>::bit(a);
      const B nb = nbr4(pb, g);
      const B own0 = pick(s.bw, c);
      B own = own0 | pb;
      B opp = pick(s.bw, 1 - c);
      const bool enemy_eye = !any(nb & ~opp);
      s.hash ^= ctx.zob[2 * a + c];
      B E = M::board(g) & ~(own | opp);
      int captured = 0;
      int cap_pt = -1;
      // The atari set changes only for chains the move touches: adjacent
      // opponent chains lose liberty a (captured at zero), the mover's chain
      // through a is new, and own chains next to captured stones gain
      // liberties.  Every other chain keeps its liberties.
      B atari = s.atari;
      B capd = BB<B>::zero();
      B on = nb & opp;
#if OS_GO_LAZY_ATARI == 2
      // Wave-uniform callers (the wave search's tree moves, on the scalar unit)
      // keep the full floods: the early-stopping form costs the numpy-policy
      // wave kernel its registers (248 VGPRs + 1 KB scratch against 115).
      if constexpr (!WaveUniformCtx<C>::value) {
      // Captures: an opponent chain next to a that was in atari had a as its
      // only liberty; `flood(q, opp & atari)` is its chain (two same-coloured
      // atari chains never touch).  Any other opponent chain next to a keeps
      // >= 1 liberty (points freed by this move's captures were stones of its
      // own colour, so they never touch it) and enters atari iff exactly one
      // is left: flood_libs2 answers that without walking the whole chain (a
      // partial answer leaves the set unchanged; another stone of the same
      // chain in `on` only repeats it).  Own chains in atari next to a (they
      // merge into a's chain) or next to captured stones leave the set; a's
      // chain enters it iff it has exactly one liberty.  Same set as mode 0.
      const B opp_at = opp & atari;
#if OS_GO_APPLY_MS
      // The same updates with the captures and the own chains leaving the set
      // each as ONE flood from all their seeds (a flood of a union of seeds
      // is the union of their chains), so the lanes do not diverge over a
      // per-chain capture branch.  own_at is taken before the updates: they
      // change only opponent stones' membership.  With one stone captured
      // (the only case the ko point needs) that stone is the capturing
      // neighbour, lowest(ch).
      const B own_at = own0 & atari;
      B touched = nb & own_at;
      const B caps = on & opp_at;
      if (any(caps)) {
        const B ch = flood(caps, opp_at, g);
        on = on & ~ch;
        opp = opp & ~ch;
        E = E | ch;
        capd = ch;
        captured = popc(ch);
        cap_pt = lowest(ch);
        atari = atari & ~ch;
        touched = touched | (nbr4(ch, g) & own_at);
        B rem = ch;
        while (any(rem)) {
          const int x = lowest(rem);
          rem = rem & ~BB<B>::bit(x);
          s.hash ^= ctx.zob[2 * x + (1 - c)];
        }
      }
#if OS_GO_TWO_LIB
      // Points with two or more empty neighbours, for every point at once
      // (at least two of nbr4's four shifted copies of E): a chain through
      // such a point has two liberties, which is all the first step of
      // flood_libs2 would learn from it.  The opponent neighbours and the new
      // stone that pass it skip their floods, so the lanes seldom enter the
      // per-chain loop at all.
      const int n = g.rows;
      const B t1 = shl(E, n), t2 = shr(E, n);
      const B t3 = shl(E, 1) & M::notcol0(g), t4 = shr(E, 1) & M::notcollast(g);
      const B two = (t1 & t2) | (t3 & t4) | ((t1 | t2) & (t3 | t4));
      on = on & ~two;
      const bool own_two = test(two, a);
#else
      const bool own_two = false;
#endif
      while (any(on)) {
        B libs;
        const B ch = flood_libs2(BB<B>::bit(lowest(on)), opp, E, g, &libs);
        on = on & ~ch;
        atari = atari | BB<B>::sel(popc(libs) == 1, ch, BB<B>::zero());
      }
      if (any(touched)) atari = atari & ~flood(touched, own_at, g);
      if (!own_two) {
        B libs;
        const B ch = flood_libs2(pb, own, E, g, &libs);
        atari = atari | BB<B>::sel(popc(libs) == 1, ch, BB<B>::zero());
      }
#else
      while (any(on)) {
        const int q = lowest(on);
        const B qb = BB<B>::bit(q);
        if (any(qb & opp_at)) {
          const B ch = flood(qb, opp_at, g);
          on = on & ~ch;
          opp = opp & ~ch;
          E = E | ch;
          capd = capd | ch;
          captured += popc(ch);
          cap_pt = q;
          atari = atari & ~ch;
          B rem = ch;
          while (any(rem)) {
            const int x = lowest(rem);
            rem = rem & ~BB<B>::bit(x);
            s.hash ^= ctx.zob[2 * x + (1 - c)];
          }
        } else {
          B libs;
          const B ch = flood_libs2(qb, opp, E, g, &libs);
          on = on & ~ch;
          atari = atari | BB<B>::sel(popc(libs) == 1, ch, BB<B>::zero());
        }
      }
      const B own_at = own0 & atari;
      B touched = (nb | nbr4(capd, g)) & own_at;
      while (any(touched)) {
        const B ch = flood(BB<B>::bit(lowest(touched)), own_at, g);
        touched = touched & ~ch;
        atari = atari & ~ch;
      }
      {
        B libs;
        const B ch = flood_libs2(pb, own, E, g, &libs);
        atari = atari | BB<B>::sel(popc(libs) == 1, ch, BB<B>::zero());
      }
#endif
      } else {
      while (any(on)) {
        const int q = lowest(on);
        const B ch = flood(BB<B>::bit(q), opp, g);
        on = on & ~ch;
        const B libs = nbr4(ch, g) & E;
        if (!any(libs)) {
          opp = opp & ~ch;
          E = E | ch;
          capd = capd | ch;
          captured += popc(ch);
          cap_pt = q;
          B rem = ch;
          while (any(rem)) {
            const int x = lowest(rem);
            rem = rem & ~BB<B>::bit(x);
            s.hash ^= ctx.zob[2 * x + (1 - c)];
          }
        }
        atari = (atari & ~ch) | BB<B>::sel(popc(libs) == 1, ch, BB<B>::zero());
      }
      B todo = pb | (nbr4(capd, g) & own);
      while (any(todo)) {
        const B ch = flood(BB<B>::bit(lowest(todo)), own, g);
        todo = todo & ~ch;
        atari = (atari & ~ch) | BB<B>::sel(popc(nbr4(ch, g) & E) == 1, ch, BB<B>::zero());
      }
      }
#elif OS_GO_LAZY_ATARI
      // Full chain floods only where a liberty count is unknown.  A chain is in
      // `atari` as a whole, and two same-coloured atari chains never touch, so
      // flood(q, colour & atari) is q's chain whenever q is in atari -- a flood
      // over the few atari stones, not the chain's whole extent.
      //  * An opponent chain next to a that was in atari had a as its only
      //    liberty: it is captured.  Otherwise it keeps >= 1 liberty (points
      //    freed by this move's captures never touch it: they were stones of
      //    its own colour), and it enters atari only if it had exactly two; a
      //    stone of it with >= 2 empty neighbours after the move rules that out.
      //  * The mover's new chain is out of atari if its new stone has >= 2 empty
      //    neighbours; the chains it joined leave the atari set with it.
      //  * Own chains next to captured stones gain liberties: any in atari had
      //    exactly one and now have >= 2.
      // Every other chain keeps its liberties.  Same set as the full update.
      const B opp_at = opp & atari;
      while (any(on)) {
        const int q = lowest(on);
        const B qb = BB<B>::bit(q);
        if (any(qb & opp_at)) {
          const B ch = flood(qb, opp_at, g);
          on = on & ~ch;
          opp = opp & ~ch;
          E = E | ch;
          capd = capd | ch;
          captured += popc(ch);
          cap_pt = q;
          atari = atari & ~ch;
          B rem = ch;
          while (any(rem)) {
            const int x = lowest(rem);
            rem = rem & ~BB<B>::bit(x);
            s.hash ^= ctx.zob[2 * x + (1 - c)];
          }
        } else if (popc(nbr4(qb, g) & E) >= 2) {
          on = on & ~qb;
        } else {
          const B ch = flood(qb, opp, g);
          on = on & ~ch;
          atari = atari | BB<B>::sel(popc(nbr4(ch, g) & E) == 1, ch, BB<B>::zero());
        }
      }
      const B own_at = own0 & atari;
      B touched = (nb | nbr4(capd, g)) & own_at;
      while (any(touched)) {
        const B ch = flood(BB<B>::bit(lowest(touched)), own_at, g);
        touched = touched & ~ch;
        atari = atari & ~ch;
      }
      if (popc(nbr4(pb, g) & E) < 2) {
        const B ch = flood(pb, own, g);
        atari = atari | BB<B>::sel(popc(nbr4(ch, g) & E) == 1, ch, BB<B>::zero());
      }
#else
      while (any(on)) {
        const int q = lowest(on);
        const B ch = flood(BB<B>::bit(q), opp, g);
        on = on & ~ch;
        const B libs = nbr4(ch, g) & E;
        if (!any(libs)) {
          opp = opp & ~ch;
          E = E | ch;
          capd = capd | ch;
          captured += popc(ch);
          cap_pt = q;
          B rem = ch;
          while (any(rem)) {
            const int x = lowest(rem);
            rem = rem & ~BB<B>::bit(x);
            s.hash ^= ctx.zob[2 * x + (1 - c)];
          }
        }
        atari = (atari & ~ch) | BB<B>::sel(popc(libs) == 1, ch, BB<B>::zero());
      }
      B todo = pb | (nbr4(capd, g) & own);
      while (any(todo)) {
        const B ch = flood(BB<B>::bit(lowest(todo)), own, g);
        todo = todo & ~ch;
        atari = (atari & ~ch) | BB<B>::sel(popc(nbr4(ch, g) & E) == 1, ch, BB<B>::zero());
      }
#endif
      s.atari = atari;
      s.bw[0] = c ? opp : own;
      s.bw[1] = c ? own : opp;
      s.ko = static_cast<int16_t>((enemy_eye && captured == 1) ? cap_pt : -1);
      if (!ctx.insert(s.hash, captured > 0, popc(own) + popc(opp))) s.flags |= kSuperko;
    }
    s.to_play = static_cast<uint8_t>(1 - c);
    s.moves++;
  }
  // Tromp-Taylor score with the reference's early-abort DFS
  // (go_board.cc:526-597): for every empty point in ascending order that is
  // not yet marked, a DFS over empty points (neighbour order +row, +col, -col,
  // -row; "marked or reached both colours" tested only on entry) counts the
  // points it marks; the count goes to the colour it reached if it reached
  // only one.  DFSs never cross stones, so each empty region is independent:
  //   * a region bordering one colour (or none) is explored whole by its first
  //     DFS -- its size, from a bitboard flood;
  //   * a region bordering both colours is where the early abort matters: the
  //     reference's DFS sequence is replayed on it exactly (tt_mixed_region).
  OS_HD static float score(const State& s, const GameCfg& g) {
    const B E = M::board(g) & ~(s.bw[0] | s.bw[1]);
    int delta = popc(s.bw[0]) - popc(s.bw[1]);
    B todo = E;
    while (any(todo)) {
      const B reg = flood(BB<B>::bit(lowest(todo)), E, g);
      todo = todo & ~reg;
      const B rim = nbr4(reg, g);
      const bool rb = any(rim & s.bw[0]), rw = any(rim & s.bw[1]);
      if (rb && !rw) delta += popc(reg);
      else if (rw && !rb) delta -= popc(reg);
      else if (rb && rw && popc(reg) > 1) delta += tt_mixed_region(s, g, reg);
    }
    float sc = static_cast<float>(delta) - g.komi;
    if (g.handicap >= 2) sc -= static_cast<float>(g.handicap);
    return sc;
  }
  // The reference's DFS sequence on one empty region that borders both
  // colours; returns its contribution to (black - white).  The DFS stack is
  // held as the 2-bit directions taken from the start point (a point's parent
  // is one step back along its direction, and an ancestor resumes at the
  // direction after the one it took), so no per-point stack memory is needed.
  OS_HD static int tt_mixed_region(const State& s, const GameCfg& g, B reg) {
    const int n = g.rows;
    int delta = 0;
    B marked = BB<B>::zero();
    B todo = reg;
    while (any(todo)) {
      const int p0 = lowest(todo);
      todo = todo & ~BB<B>::bit(p0);
      if (test(marked, p0)) continue;
      bool rb = false, rw = false;
      int num = 1;
      marked = marked | BB<B>::bit(p0);
      // 2 bits per DFS level, one word per 32 levels: as many levels as the
      // board has points (B128: 128, B384: 384), words indexed by unrolled
      // selects so they stay in registers.
      constexpr int kNW = static_cast<int>(sizeof(B)) / 4;
      uint64_t path[kNW];
#pragma unroll
      for (int q = 0; q < kNW; ++q) path[q] = 0;
      int depth = 0;  // stack size - 1
      int cur = p0, curd = 0;
      for (;;) {
        if (rb && rw) break;
        if (curd == 4) {  // pop
          if (depth == 0) break;
          --depth;
          const int w = depth >> 5, sh = 2 * (depth & 31);
          uint64_t pw = 0;
#pragma unroll
          for (int q = 0; q < kNW; ++q) pw = w == q ? path[q] : pw;
          const int dir = static_cast<int>((pw >> sh) & 3);
          cur -= dir == 0 ? n : (dir == 1 ? 1 : (dir == 2 ? -1 : -n));
          curd = dir + 1;
          continue;
        }
        const int d = curd++;
        const int r = cur / n, cc = cur - r * n;
        int q;
        if (d == 0) { if (r + 1 >= n) continue; q = cur + n; }
        else if (d == 1) { if (cc + 1 >= n) continue; q = cur + 1; }
        else if (d == 2) { if (cc - 1 < 0) continue; q = cur - 1; }
        else { if (r - 1 < 0) continue; q = cur - n; }
        if (test(s.bw[0], q)) { rb = true; continue; }
        if (test(s.bw[1], q)) { rw = true; continue; }
        if (test(marked, q)) continue;
        marked = marked | BB<B>::bit(q);
        ++num;
        // Slot `depth` <- d (it may hold a popped sibling's direction).
        const int w = depth >> 5, sh = 2 * (depth & 31);
        const uint64_t keep = ~(3ull << sh), m = static_cast<uint64_t>(d) << sh;
#pragma unroll
        for (int q = 0; q < kNW; ++q) path[q] = w == q ? ((path[q] & keep) | m) : path[q];
        ++depth;
        cur = q;
        curd = 0;
      }
      if (rb && !rw) delta += num;
      else if (!rb && rw) delta -= num;
    }
    return delta;
  }
  template <class C>
  OS_HD static int ret0(const State& s, const GameCfg& g, C&) {
    if (s.flags & kSuperko) return 0;
    const float sc = score(s, g);
    return sc > 0 ? 1 : (sc < 0 ? -1 : 0);
  }
  // ObservationTensor (go.cc:102-122): [4][n][n], planes black, white, empty
  // (GoColor order) in BoardPoints order (== action order), then a constant
  // plane = 1 when white is to play (komi bias); not player-relative.
  static constexpr int kObsPlanes = 4;
  OS_HD static float obs(const State& s, const GameCfg&, int, int plane, int cell) {
    if (plane == 3) return s.to_play == 1 ? 1.0f : 0.0f;
    const int want = test(s.bw[0], cell) ? 0 : (test(s.bw[1], cell) ? 1 : 2);
    return plane == want ? 1.0f : 0.0f;
  }
};
using Go = GoT<B128>;
using GoBig = GoT<B384>;  // board_size 12..19 (host State API)
// board_size <= 9 on the lane kernels (k_lsearch, k_rollouts): the same game
// over three-word bitboards, so every board operation issues 3 VALU words
// instead of 4 and a shift 3 instead of 5.  Roots arrive as Go::State records
// (os_kernels.h GoRoot narrows them); bit i is cell i in both.
using Go9 = GoT<B96>;
constexpr int kGo9MaxSide = 9;
OS_HD Go9::State go9_state(const Go::State& r) {
  Go9::State s;
  s.bw[0] = b96_of(r.bw[0]);
  s.bw[1] = b96_of(r.bw[1]);
  s.atari = b96_of(r.atari);
  s.hash = r.hash;
  s.ko = r.ko;
  s.moves = r.moves;
  s.to_play = r.to_play;
  s.flags = r.flags;
  s.pad = r.pad;
  return s;
}

// ----------------------------------------------------------------------------
// pig (pig.cc:81-244), 2..10 players.  A decision node offers roll (0) and
// stop (1) -- only stop once the turn total would reach winscore
// (:225-229).  Roll moves to a chance node whose outcomes are
// 1..diceoutcomes, each with probability 1 / diceoutcomes (:233-244):
// outcome 1 loses the turn total and passes the turn, outcome k > 1 adds
// k + 1 (:204-213, as written).  Stop banks the turn total and passes
// (round robin).  total_moves counts decisions only; terminal at total_moves
// >= horizon or a score >= winscore (:81-92).  Returns (:94-111): the first
// player (in player order) at winscore gets +1, every other -1 / (n - 1);
// nobody: all 0.  The scores live in a fixed array indexed only through
// unrolled selects, so a state held in registers never goes to scratch.
//
// Outcome codes (ret0 / Node::out): two players keep the player-0 value
// {-1, 0, +1}; with n > 2 players a win by player w is 3 + w and "nobody" 0
// (the reference's outcome vectors are determined by them; out_value()).
// kMaxP: the players the state has room for.  Pig (10) is the game of the
// host State API, the state records and every kernel; Pig2 is the same rules
// over two players' arrays, which the wave chance-node search runs for
// two-player pig (ChanceRoot narrows the 10-player root records): every
// score array op is then 2 selects instead of 10 (a single pig step 13.2 ->
// 10.6 ms, profiles/r06/pig2/).
template <int kMaxP>
struct PigT {
  static constexpr int kMaxPlayers = kMaxP;
  struct State {
    int32_t score[kMaxPlayers];
    int32_t turn_total;
    int32_t cur;          // player to move, -1 at a chance node
    int32_t turn_player;
    int32_t moves;        // total_moves_
    static constexpr bool kNeedsLog = false;
  };
  using Ctx = NoCtx;
  static constexpr bool kHasChance = true;
  struct Legal {
    uint32_t mask;
    int count;
    OS_HD int kth(int k) const { return select64(mask, k); }
  };
  OS_HD static int32_t score_of(const State& s, int p) {
    int32_t v = 0;
#pragma unroll
    for (int i = 0; i < kMaxPlayers; ++i) v = i == p ? s.score[i] : v;
    return v;
  }
  OS_HD static void init(State& s, const GameCfg&) {
#pragma unroll
    for (int i = 0; i < kMaxPlayers; ++i) s.score[i] = 0;
    s.turn_total = 0;
    s.cur = 0;
    s.turn_player = 0;
    s.moves = 0;
  }
  // The first player (in player order) whose score reaches winscore, or -1.
  OS_HD static int winner(const State& s, const GameCfg& g) {
    int w = -1;
#pragma unroll
    for (int i = kMaxPlayers - 1; i >= 0; --i)
      w = (i < g.pig_players && s.score[i] >= g.pig_win) ? i : w;
    return w;
  }
  OS_HD static bool terminal(const State& s, const GameCfg& g) {
    return s.moves >= g.pig_horizon || winner(s, g) >= 0;
  }
  OS_HD static int to_move(const State& s) { return s.cur; }
  OS_HD static bool chance(const State& s) { return s.cur < 0; }
  OS_HD static int chance_count(const GameCfg& g) { return g.pig_dice; }
  OS_HD static double chance_prob(const GameCfg& g) { return 1.0 / g.pig_dice; }
  OS_HD static Legal legal(const State& s, const GameCfg& g, Ctx&) {
    Legal l;
    if (s.cur < 0) {
      l.mask = ((1u << g.pig_dice) - 1u) << 1;  // outcomes 1..dice
      l.count = g.pig_dice;
    } else {
      l.mask = score_of(s, s.cur) + s.turn_total >= g.pig_win ? 2u : 3u;
      l.count = popc64(l.mask);
    }
    return l;
  }
  OS_HD static int next_player(int p, const GameCfg& g) {  // NextPlayerRoundRobin
    return p + 1 < g.pig_players ? p + 1 : 0;
  }
  OS_HD static void apply(State& s, const GameCfg& g, Ctx&, int a) {
    if (s.cur >= 0) {
      s.moves++;
      if (a == 0) {
        s.cur = -1;
        return;
      }
#pragma unroll
      for (int i = 0; i < kMaxPlayers; ++i) s.score[i] += i == s.turn_player ? s.turn_total : 0;
      s.turn_total = 0;
      s.turn_player = next_player(s.turn_player, g);
      s.cur = s.turn_player;
    } else if (a == 1) {
      s.turn_total = 0;
      s.turn_player = next_player(s.turn_player, g);
      s.cur = s.turn_player;
    } else {
      s.turn_total += a + 1;
      s.cur = s.turn_player;
    }
  }
  OS_HD static int ret0(const State& s, const GameCfg& g, Ctx&) {
    const int w = winner(s, g);
    if (g.pig_players == 2) return w == 0 ? 1 : (w == 1 ? -1 : 0);
    return w < 0 ? 0 : 3 + w;
  }
  // Returns()[p] of a terminal whose outcome code is `code` (pig.cc:94-111).
  OS_HD static double value(int code, int p, const GameCfg& g) {
    if (code >= 3) return p == code - 3 ? 1.0 : -1.0 / (g.pig_players - 1);
    return static_cast<double>(p == 0 ? code : -code);
  }
  // ObservationTensor (pig.cc:119-168): [1 + players][winscore + 1] one-hot
  // bins of the turn total, then each player's score (the last bin holds >=
  // winscore); as a [1 + players][1][winscore + 1] CHW image.
  static constexpr int kObsPlanes = 1 + kMaxPlayers;  // planes used: 1 + players
  OS_HD static float obs(const State& s, const GameCfg& g, int, int plane, int cell) {
    const int v = plane == 0 ? s.turn_total : score_of(s, plane - 1);
    const int bin = v < g.pig_win ? v : g.pig_win;
    return cell == bin ? 1.0f : 0.0f;
  }
};
using Pig = PigT<10>;
using Pig2 = PigT<2>;

// Returns()[p] of a solved node whose outcome code is `out` (os_mcts.h
// Node::out): the player-0 value of two-player zero-sum games, or the game's
// own decoding (pig with more than two players).
template <class G, class = void>
struct OutValue {
  OS_HD static double value(int out, int p, const GameCfg&) {
    return static_cast<double>(p == 0 ? out : -out);
  }
};
template <class G>
struct OutValue<G, decltype(void(&G::value))> {
  OS_HD static double value(int out, int p, const GameCfg& g) { return G::value(out, p, g); }
};

// Chance-node traits (games without them never reach the chance branches).
template <class G, class = void>
struct HasChance {
  static constexpr bool value = false;
};
template <class G>
struct HasChance<G, decltype(void(G::kHasChance))> {
  static constexpr bool value = G::kHasChance;
};

}  // namespace osm

#endif  // OS_GAMES_H_
