// Host-side game loading, State API and string formatting for libos_mcts.so.
// The rule logic itself is the shared host/device code in os_games.h.
//
// String formats restate the reference's ToString / ActionToString:
//   tic_tac_toe.cc:94-99,:128-138; connect_four.cc:106-110,:160-169;
//   breakthrough.cc:168-189,:247-266; hex.cc:189-196,:227-243;
//   go.cc:133-144 + go_board.cc:478-506.
#include "os_host.h"

#include "os_rng.h"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <sstream>
#include <type_traits>

namespace osm {

namespace {
// std::mt19937(seed)'s output stream, counting the words drawn (same URBG
// range, so generate_canonical consumes it exactly as it consumes the engine
// itself).  A Dirichlet draw takes a few dozen words, so the first block is
// twisted word by word from running cursors of the init_genrand recurrence
// (x[i], x[i+1], x[i+397]) instead of seeding all 624 words and twisting
// them up front -- the device streams' scheme (MtStreamSoA) -- and the full
// state exists only once the first block is used up.
struct CountingMt {
  using result_type = uint32_t;
  uint32_t s[kMtN];   // twisted words of the current block
  uint32_t lo0, lo1, hi;  // seeded x[i], x[i + 1], x[i + 397] (first block)
  int idx = 0;
  bool blk0 = true;
  int64_t words = 0;
  static uint32_t seed_step(uint32_t x, int k) {
    return 1812433253u * (x ^ (x >> 30)) + static_cast<uint32_t>(k);
  }
  explicit CountingMt(uint32_t seed) {
    lo0 = seed;
    lo1 = seed_step(seed, 1);
    uint32_t x = lo1;
    for (int k = 2; k <= kMtM; ++k) x = seed_step(x, k);
    hi = x;
  }
  static constexpr result_type min() { return 0; }
  static constexpr result_type max() { return 0xFFFFFFFFu; }
  result_type operator()() {
    ++words;
    uint32_t v;
    if (blk0) {
      const int i = idx;
      const uint32_t b = (i + 1 == kMtN) ? s[0] : lo1;
      const uint32_t m = (i + kMtM < kMtN) ? hi : s[i + kMtM - kMtN];
      const uint32_t y = (lo0 & 0x80000000u) | (b & 0x7fffffffu);
      v = m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      s[i] = v;
      lo0 = lo1;
      lo1 = seed_step(lo1, i + 2);
      hi = seed_step(hi, i + kMtM + 1);
      if (++idx == kMtN) {
        blk0 = false;
        idx = 0;
        Twist();
      }
    } else {
      v = s[idx];
      if (++idx == kMtN) {
        idx = 0;
        Twist();
      }
    }
    return MtStream::temper(v);
  }
  void Twist() {  // the next block, in place (standard MT19937 recurrence)
    for (int i = 0; i < kMtN; ++i) {
      const uint32_t y = (s[i] & 0x80000000u) | (s[(i + 1) % kMtN] & 0x7fffffffu);
      s[i] = s[(i + kMtM) % kMtN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
  }
};

// The same URBG over a caller-held stream in numpy's (key, pos) form (the
// engine's MtStream import semantics), on a copy of the key.
struct StateMt {
  using result_type = uint32_t;
  std::vector<uint32_t> key;
  MtStream g;
  int64_t words = 0;
  StateMt(const uint32_t* k, int pos) : key(k, k + kMtN), g{nullptr, pos, 1, 0} {
    g.s = key.data();
  }
  static constexpr result_type min() { return 0; }
  static constexpr result_type max() { return 0xFFFFFFFFu; }
  result_type operator()() {
    ++words;
    return g.next();
  }
};

template <class Rng>
int64_t DirichletFrom(Rng& rng, int count, double alpha, double* out) {
  std::gamma_distribution<double> gamma(alpha, 1.0);
  for (int i = 0; i < count; ++i) out[i] = gamma(rng);
  double sum = 0.0;
  for (int i = 0; i < count; ++i) sum += out[i];  // absl::c_accumulate(noise, 0.0)
  for (int i = 0; i < count; ++i) out[i] /= sum;
  return rng.words;
}
}  // namespace

int64_t DirichletNoiseState(const uint32_t* key, int pos, int count, double alpha, double* out) {
  StateMt rng(key, pos);
  return DirichletFrom(rng, count, alpha, out);
}

int64_t DirichletNoise(uint32_t seed, int count, double alpha, double* out) {
  CountingMt rng(seed);
  return DirichletFrom(rng, count, alpha, out);
}

namespace {

bool ParseGameString(const std::string& s, std::string* name,
                     std::map<std::string, std::string>* kv) {
  size_t lp = s.find('(');
  if (lp == std::string::npos) {
    *name = s;
    return !s.empty();
  }
  if (s.back() != ')') return false;
  *name = s.substr(0, lp);
  std::string body = s.substr(lp + 1, s.size() - lp - 2);
  size_t pos = 0;
  while (pos < body.size()) {
    size_t comma = body.find(',', pos);
    if (comma == std::string::npos) comma = body.size();
    std::string item = body.substr(pos, comma - pos);
    size_t eq = item.find('=');
    if (eq == std::string::npos) return false;
    (*kv)[item.substr(0, eq)] = item.substr(eq + 1);
    pos = comma + 1;
  }
  return true;
}

bool GetInt(const std::map<std::string, std::string>& kv, const char* k,
            int dflt, int* out) {
  auto it = kv.find(k);
  if (it == kv.end()) {
    *out = dflt;
    return true;
  }
  char* end = nullptr;
  long v = std::strtol(it->second.c_str(), &end, 10);
  if (end == it->second.c_str() || *end) return false;
  *out = static_cast<int>(v);
  return true;
}

bool GetDouble(const std::map<std::string, std::string>& kv, const char* k,
               double dflt, double* out) {
  auto it = kv.find(k);
  if (it == kv.end()) {
    *out = dflt;
    return true;
  }
  char* end = nullptr;
  double v = std::strtod(it->second.c_str(), &end);
  if (end == it->second.c_str() || *end) return false;
  *out = v;
  return true;
}

template <class B>
void SquareMasksOf(int n, B* board, B* notcol0, B* notcollast, B* hex_a, B* hex_b) {
  *board = BB<B>::lowmask(n * n);
  B col0 = BB<B>::zero(), coll = BB<B>::zero();
  for (int r = 0; r < n; ++r) {
    col0 = col0 | BB<B>::bit(r * n);
    coll = coll | BB<B>::bit(r * n + n - 1);
  }
  *notcol0 = *board & ~col0;
  *notcollast = *board & ~coll;
  const bool n2 = n == 2;
  *hex_a = n2 ? BB<B>::zero() : *notcol0;
  *hex_b = n2 ? BB<B>::zero() : *notcollast;
}

void SquareMasks(int n, GameCfg* c) {
  if (n <= kB128Side)
    SquareMasksOf(n, &c->board, &c->notcol0, &c->notcollast, &c->hex_a, &c->hex_b);
  else
    SquareMasksOf(n, &c->big_board, &c->big_notcol0, &c->big_notcollast, &c->big_hex_a,
                  &c->big_hex_b);
}

std::string FormatDouble(double v) {
  std::ostringstream ss;
  ss << v;
  return ss.str();
}

template <class G>
typename G::State& St(HostState& s) {
  return *reinterpret_cast<typename G::State*>(s.raw);
}
template <class G>
const typename G::State& St(const HostState& s) {
  return *reinterpret_cast<const typename G::State*>(s.raw);
}

// Calls f(G{}) with G the state machine of the game `g` (hex / go boards above
// 11 x 11 use the B384 instantiations).
template <class F>
auto WithGame(const GameCfg& g, F&& f) {
  switch (g.kind) {
    case kTicTacToe: return f(TicTacToe{});
    case kConnectFour: return f(ConnectFour{});
    case kBreakthrough: return f(Breakthrough{});
    case kHex: return g.rows > kB128Side ? f(HexBig{}) : f(Hex{});
    case kPig: return f(Pig{});
    default: return g.rows > kB128Side ? f(GoBig{}) : f(Go{});
  }
}

template <class G>
constexpr bool kIsGo = std::is_same<typename G::Ctx, GoCtx>::value;

}  // namespace

std::string LoadHostGame(const std::string& gs, HostGame* g, bool* unsupported) {
  *unsupported = false;
  std::string name;
  std::map<std::string, std::string> kv;
  if (!ParseGameString(gs, &name, &kv)) return "cannot parse game string '" + gs + "'";
  GameCfg c;
  std::memset(&c, 0, sizeof c);
  auto reject_unknown = [&](std::initializer_list<const char*> allowed) -> std::string {
    for (auto& it : kv) {
      bool ok = false;
      for (const char* a : allowed) ok |= it.first == a;
      if (!ok) return "unknown parameter '" + it.first + "' for game " + name;
    }
    return "";
  };
  if (name == "tic_tac_toe") {
    std::string e = reject_unknown({});
    if (!e.empty()) return e;
    c.kind = kTicTacToe;
    c.rows = c.cols = 3;
    c.num_actions = 9;
    c.max_children = 9;
    c.max_game_length = 9;
    g->canonical = "tic_tac_toe()";
    g->state_bytes = sizeof(TicTacToe::State);
  } else if (name == "connect_four") {
    std::string e = reject_unknown({});
    if (!e.empty()) return e;
    c.kind = kConnectFour;
    c.rows = 6;
    c.cols = 7;
    c.num_actions = 7;
    c.max_children = 7;
    c.max_game_length = 42;
    g->canonical = "connect_four()";
    g->state_bytes = sizeof(ConnectFour::State);
  } else if (name == "breakthrough") {
    std::string e = reject_unknown({"rows", "columns"});
    if (!e.empty()) return e;
    int rows, cols;
    if (!GetInt(kv, "rows", 8, &rows) || !GetInt(kv, "columns", 8, &cols))
      return "bad breakthrough parameter";
    if (rows < 2 || cols < 2) return "breakthrough needs rows, columns >= 2";
    if (rows * cols > 64) {
      *unsupported = true;
      return "breakthrough boards above 64 cells are not supported by this engine";
    }
    c.kind = kBreakthrough;
    c.rows = rows;
    c.cols = cols;
    c.num_actions = rows * cols * 6 * 2;
    c.max_game_length = 2 * (2 * rows - 3) * cols + 1;
    c.max_children = 3 * cols * (rows >= 6 ? 2 : 1);
    uint64_t board = rows * cols == 64 ? ~0ull : ((1ull << (rows * cols)) - 1);
    uint64_t col0 = 0, coll = 0;
    for (int r = 0; r < rows; ++r) {
      col0 |= 1ull << (r * cols);
      coll |= 1ull << (r * cols + cols - 1);
    }
    c.board64 = board;
    c.notcol0_64 = board & ~col0;
    c.notcollast_64 = board & ~coll;
    g->canonical = (rows == 8 && cols == 8 && kv.empty())
                       ? "breakthrough()"
                       : "breakthrough(columns=" + std::to_string(cols) +
                             ",rows=" + std::to_string(rows) + ")";
    g->state_bytes = sizeof(Breakthrough::State);
  } else if (name == "hex") {
    std::string e = reject_unknown({"board_size"});
    if (!e.empty()) return e;
    int n;
    if (!GetInt(kv, "board_size", 11, &n)) return "bad hex board_size";
    if (n < 2 || n > kMaxSide) {
      *unsupported = true;
      return "hex board_size must be in [2, 19] for this engine";
    }
    c.kind = kHex;
    c.rows = c.cols = n;
    c.num_actions = n * n;
    c.max_children = n * n;
    c.max_game_length = n * n;
    SquareMasks(n, &c);
    g->canonical = kv.empty() ? "hex()" : "hex(board_size=" + std::to_string(n) + ")";
    g->state_bytes = n > kB128Side ? sizeof(HexBig::State) : sizeof(Hex::State);
  } else if (name == "go") {
    std::string e = reject_unknown({"board_size", "komi", "handicap"});
    if (!e.empty()) return e;
    int n, handicap;
    double komi;
    if (!GetInt(kv, "board_size", 19, &n) || !GetInt(kv, "handicap", 0, &handicap) ||
        !GetDouble(kv, "komi", 7.5, &komi))
      return "bad go parameter";
    if (n < 2 || n > kMaxSide) {
      *unsupported = true;
      return "go board_size must be in [2, 19] for this engine";
    }
    // Handicap stones sit on 19 x 19 star points (go.cc:56-78): every one must
    // be on the board, where GoBoard::PlayMove's SPIEL_CHECK_EQ(kEmpty, ...)
    // (go_board.cc:263) would otherwise fail.
    for (int p : GoHandicapStones(handicap, 19))
      if (p / 19 >= n || p % 19 >= n)
        return "go handicap " + std::to_string(handicap) + " places a stone off the " +
               std::to_string(n) + "x" + std::to_string(n) + " board";
    c.kind = kGo;
    c.rows = c.cols = n;
    c.num_actions = n * n + 1;
    c.max_children = n * n + 1;
    c.max_game_length = 2 * n * n;
    c.komi = static_cast<float>(komi);
    c.handicap = handicap;
    SquareMasks(n, &c);
    // chess_common.h:113-154 ZobristTable<uint64_t, 441, 2>(seed 2765481),
    // indexed by virtual point (r + 1) * 21 + (c + 1) (go_board.cc:289-299).
    std::vector<uint64_t> vz(441 * 2);
    std::mt19937_64 outer(2765481);
    for (int i = 0; i < 441; ++i) {
      std::mt19937_64 inner(outer());
      vz[2 * i] = inner();
      vz[2 * i + 1] = inner();
    }
    g->zob.assign(static_cast<size_t>(n) * n * 2, 0);
    for (int r = 0; r < n; ++r)
      for (int col = 0; col < n; ++col) {
        int vp = (r + 1) * 21 + col + 1;
        g->zob[2 * (r * n + col)] = vz[2 * vp];
        g->zob[2 * (r * n + col) + 1] = vz[2 * vp + 1];
      }
    std::string canon = "go(";
    bool first = true;
    auto add = [&](const std::string& k, const std::string& v) {
      canon += (first ? "" : ",") + k + "=" + v;
      first = false;
    };
    for (auto& it : kv) {
      if (it.first == "board_size") add("board_size", std::to_string(n));
      else if (it.first == "komi") add("komi", FormatDouble(komi));
      else if (it.first == "handicap") add("handicap", std::to_string(handicap));
    }
    g->canonical = canon + ")";
    g->state_bytes = n > kB128Side ? sizeof(GoBig::State) : sizeof(Go::State);
  } else if (name == "pig") {
    std::string e = reject_unknown({"players", "horizon", "winscore", "diceoutcomes"});
    if (!e.empty()) return e;
    int players, horizon, win, dice;
    if (!GetInt(kv, "players", 2, &players) || !GetInt(kv, "horizon", 1000, &horizon) ||
        !GetInt(kv, "winscore", 100, &win) || !GetInt(kv, "diceoutcomes", 6, &dice))
      return "bad pig parameter";
    if (players < 2 || players > 10 || horizon < 1 || win < 1 || dice < 1)
      return "bad pig parameter";
    if (dice > 30 || win > 4096) {
      *unsupported = true;
      return "pig diceoutcomes must be <= 30 and winscore <= 4096 for this engine";
    }
    c.kind = kPig;
    c.rows = 1;                 // ObservationTensor [3][winscore + 1]
    c.cols = win + 1;
    c.num_actions = 6;          // pig.h:83 (NumDistinctActions is fixed)
    c.max_children = dice > 2 ? dice : 2;
    c.max_game_length = horizon;
    c.pig_dice = dice;
    c.pig_horizon = horizon;
    c.pig_win = win;
    c.pig_players = players;
    std::string canon = "pig(";
    bool first = true;
    for (auto& it : kv) {  // sorted by key, as GameParametersToString
      canon += (first ? "" : ",") + it.first + "=" + std::to_string(std::atoi(it.second.c_str()));
      first = false;
    }
    g->canonical = canon + ")";
    g->state_bytes = sizeof(Pig::State);
  } else {
    *unsupported = true;
    return "game '" + name + "' is not supported by this engine (supported: "
           "tic_tac_toe, connect_four, breakthrough, hex, go, pig)";
  }
  g->cfg = c;
  g->name = name;
  return "";
}

GoCtx HostGoCtx(const HostState& s, HostGoLog* buf) {
  GoCtx ctx;
  std::memset(static_cast<void*>(&ctx), 0, sizeof ctx);
  const GameCfg& g = s.game->cfg;
  ctx.zob = s.game->zob.data();
  ctx.base = s.hashes.data();
  ctx.n_base = static_cast<int32_t>(s.hashes.size());
  buf->bind(&ctx, 4, g.rows * g.cols);  // one apply logs at most one position
  ctx.init_filters();
  return ctx;
}

std::vector<int> GoHandicapStones(int handicap, int n) {
  // go.cc:56-78 HandicapStones: d4 q16 d16 q4 d10 q10 k4 k16 k10 as (row, col),
  // the centre k10 replacing the last stone of an odd count >= 5; none unless
  // 2 <= handicap <= 9.
  static const int kRC[9][2] = {{3, 3}, {15, 15}, {15, 3}, {3, 15}, {9, 3},
                                {9, 15}, {3, 9}, {15, 9}, {9, 9}};
  std::vector<int> pts;
  if (handicap < 2 || handicap > 9) return pts;
  for (int i = 0; i < handicap; ++i) pts.push_back(kRC[i][0] * n + kRC[i][1]);
  if (handicap >= 5 && handicap % 2 == 1) pts[handicap - 1] = 9 * n + 9;
  return pts;
}

void StateInit(HostState* s) {
  std::memset(s->raw, 0, sizeof s->raw);
  s->history.clear();
  s->hashes.clear();
  const GameCfg& g = s->game->cfg;
  WithGame(g, [&](auto tag) {
    using G = decltype(tag);
    G::init(St<G>(*s), g);
    if constexpr (kIsGo<G>) {
      // GoState::ResetBoard (go.cc:211-225): black plays the handicap stones,
      // then white is to move (for any handicap >= 2, even one above 9 that
      // places none); the history stays empty and the repetition set holds
      // only the resulting position.
      typename G::State& st = St<G>(*s);
      if (g.handicap >= 2) {
        for (int p : GoHandicapStones(g.handicap, g.rows)) {
          HostGoLog buf;
          GoCtx ctx = HostGoCtx(*s, &buf);
          st.to_play = 0;
          G::apply(st, g, ctx, p);
        }
        st.to_play = 1;
        st.moves = 0;
        st.flags = 0;
        st.ko = -1;
      }
      s->hashes.push_back(st.hash);  // go.cc:218-224
    }
  });
}

bool StateTerminal(const HostState& s) {
  const GameCfg& g = s.game->cfg;
  return WithGame(g, [&](auto tag) {
    using G = decltype(tag);
    return G::terminal(St<G>(s), g);
  });
}

int StateCurrentPlayer(const HostState& s) {
  if (StateTerminal(s)) return -4;
  return WithGame(s.game->cfg, [&](auto tag) {
    using G = decltype(tag);
    return G::to_move(St<G>(s));
  });
}

namespace {
template <class G>
void LegalOf(const HostState& s, typename G::Ctx& ctx, std::vector<int64_t>* out) {
  const typename G::Legal l = G::legal(St<G>(s), s.game->cfg, ctx);
  for (int k = 0; k < l.count; ++k) out->push_back(l.kth(k));
}
}  // namespace

void StateLegal(const HostState& s, std::vector<int64_t>* out) {
  out->clear();
  if (StateTerminal(s)) return;
  WithGame(s.game->cfg, [&](auto tag) {
    using G = decltype(tag);
    if constexpr (kIsGo<G>) {
      HostGoLog buf;
      GoCtx ctx = HostGoCtx(s, &buf);
      LegalOf<G>(s, ctx, out);
    } else {
      NoCtx nc;
      LegalOf<G>(s, nc, out);
    }
  });
}

bool StateApply(HostState* s, int64_t a) {
  std::vector<int64_t> legal;
  StateLegal(*s, &legal);
  bool ok = false;
  for (int64_t x : legal) ok |= x == a;
  if (!ok) return false;
  const GameCfg& g = s->game->cfg;
  const int ai = static_cast<int>(a);
  WithGame(g, [&](auto tag) {
    using G = decltype(tag);
    if constexpr (kIsGo<G>) {
      HostGoLog buf;
      GoCtx ctx = HostGoCtx(*s, &buf);
      G::apply(St<G>(*s), g, ctx, ai);
      for (int i = 0; i < ctx.n_log; ++i) s->hashes.push_back(buf.log[i]);
    } else {
      NoCtx nc;
      G::apply(St<G>(*s), g, nc, ai);
    }
  });
  s->history.push_back(a);
  return true;
}

bool StateIsChance(const HostState& s) {
  if (StateTerminal(s)) return false;
  return WithGame(s.game->cfg, [&](auto tag) {
    using G = decltype(tag);
    if constexpr (HasChance<G>::value) return G::chance(St<G>(s));
    else return false;
  });
}

void StateChanceOutcomes(const HostState& s, std::vector<std::pair<int64_t, double>>* out) {
  out->clear();
  if (!StateIsChance(s)) return;
  WithGame(s.game->cfg, [&](auto tag) {
    using G = decltype(tag);
    if constexpr (HasChance<G>::value) {
      NoCtx nc;
      const typename G::Legal l = G::legal(St<G>(s), s.game->cfg, nc);
      for (int k = 0; k < l.count; ++k)
        out->emplace_back(l.kth(k), G::chance_prob(s.game->cfg));
    }
  });
}

int NumPlayers(const GameCfg& g) { return g.kind == kPig ? g.pig_players : 2; }

void StateReturns(const HostState& s, double* r) {
  const GameCfg& g = s.game->cfg;
  const int np = NumPlayers(g);
  for (int p = 0; p < np; ++p) r[p] = 0.0;
  if (!StateTerminal(s)) return;
  const int r0 = WithGame(g, [&](auto tag) {
    using G = decltype(tag);
    if constexpr (kIsGo<G>) {
      HostGoLog buf;
      GoCtx ctx = HostGoCtx(s, &buf);
      return G::ret0(St<G>(s), g, ctx);
    } else {
      NoCtx nc;
      return G::ret0(St<G>(s), g, nc);
    }
  });
  if (g.kind == kPig) {  // outcome code -> Returns() (pig.cc:94-111)
    for (int p = 0; p < np; ++p) r[p] = Pig::value(r0, p, g);
    return;
  }
  r[0] = static_cast<double>(r0);
  r[1] = static_cast<double>(-r0);
}

namespace {
template <class G>
int ObsPlanes() { return G::kObsPlanes; }
template <class G>
void ObsFill(const HostState& s, int player, float* out) {
  const GameCfg& g = s.game->cfg;
  const int cells = g.rows * g.cols;
  const int planes = g.kind == kPig ? 1 + g.pig_players : G::kObsPlanes;
  for (int c = 0; c < planes; ++c)
    for (int i = 0; i < cells; ++i) out[c * cells + i] = G::obs(St<G>(s), g, player, c, i);
}
}  // namespace

int ObservationShape(const HostGame& g, int32_t* shape3) {
  const int c = g.cfg.kind == kPig  // pig.cc:118-121: 1 + players planes
                    ? 1 + g.cfg.pig_players
                    : WithGame(g.cfg, [&](auto tag) { return ObsPlanes<decltype(tag)>(); });
  if (shape3) {
    shape3[0] = c;
    shape3[1] = g.cfg.rows;
    shape3[2] = g.cfg.cols;
  }
  return c * g.cfg.rows * g.cfg.cols;
}

void StateObservation(const HostState& s, int player, float* out) {
  WithGame(s.game->cfg, [&](auto tag) { ObsFill<decltype(tag)>(s, player, out); });
}

namespace {

std::string TttString(const TicTacToe::State& s) {
  std::string out;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) {
      int i = r * 3 + c;
      out += (s.b[0] >> i) & 1 ? "x" : ((s.b[1] >> i) & 1 ? "o" : ".");
    }
    if (r < 2) out += "\n";
  }
  return out;
}

std::string C4String(const ConnectFour::State& s) {
  std::string out;
  for (int r = 5; r >= 0; --r) {
    for (int c = 0; c < 7; ++c) {
      int i = c * 7 + r;
      out += (s.bb[0] >> i) & 1 ? "x" : ((s.bb[1] >> i) & 1 ? "o" : ".");
    }
    out += "\n";
  }
  return out;
}

std::string BtString(const Breakthrough::State& s, const GameCfg& g) {
  std::string out;
  for (int r = 0; r < g.rows; ++r) {
    out += static_cast<char>('1' + (g.rows - 1 - r));
    for (int c = 0; c < g.cols; ++c) {
      int i = r * g.cols + c;
      out += (s.pc[0] >> i) & 1 ? "b" : ((s.pc[1] >> i) & 1 ? "w" : ".");
    }
    out += "\n";
  }
  out += " ";
  for (int c = 0; c < g.cols; ++c) out += static_cast<char>('a' + c);
  out += "\n";
  return out;
}

template <class HS>
char HexCellChar(const HS& s, int i) {
  if (test(s.st[0], i)) {
    if (s.win_cell == i) return 'X';
    if (test(s.ea[0], i)) return 'y';
    if (test(s.eb[0], i)) return 'z';
    return 'x';
  }
  if (test(s.st[1], i)) {
    if (s.win_cell == i) return 'O';
    if (test(s.ea[1], i)) return 'p';
    if (test(s.eb[1], i)) return 'q';
    return 'o';
  }
  return '.';
}

template <class HS>
std::string HexString(const HS& s, const GameCfg& g) {
  const int n = g.rows;
  std::string out;
  int line = 0;
  for (int c = 0; c < n * n; ++c) {
    if (c && !(c % n)) {
      out += "\n";
      ++line;
      out += std::string(line, ' ');
    }
    out += HexCellChar(s, c);
    out += " ";
  }
  return out;
}

template <class GS>
std::string GoString(const GS& s, const GameCfg& g, size_t hist) {
  std::ostringstream ss;
  ss << "GoState(komi=" << g.komi << ", to_play=" << (s.to_play == 0 ? "B" : "W")
     << ", history.size()=" << hist << ")\n";
  ss << "\n";
  const int n = g.rows;
  for (int r = n - 1; r >= 0; --r) {
    char buf[16];
    std::snprintf(buf, sizeof buf, "%2d ", r + 1);
    ss << buf;
    for (int c = 0; c < n; ++c) {
      int i = r * n + c;
      ss << (test(s.bw[0], i) ? 'X' : (test(s.bw[1], i) ? 'O' : '+'));
    }
    ss << "\n";
  }
  std::string cols = "ABCDEFGHJKLMNOPQRST";
  ss << "   " << cols.substr(0, n) << "\n";
  return ss.str();
}

}  // namespace

std::string StateToString(const HostState& s) {
  const GameCfg& g = s.game->cfg;
  switch (g.kind) {
    case kTicTacToe: return TttString(St<TicTacToe>(s));
    case kConnectFour: return C4String(St<ConnectFour>(s));
    case kBreakthrough: return BtString(St<Breakthrough>(s), g);
    case kHex:
      return g.rows > kB128Side ? HexString(St<HexBig>(s), g) : HexString(St<Hex>(s), g);
    case kGo:
      return g.rows > kB128Side ? GoString(St<GoBig>(s), g, s.history.size())
                                : GoString(St<Go>(s), g, s.history.size());
    case kPig: {  // pig.cc:246-251 (StrJoin(scores_, " "))
      const Pig::State& p = St<Pig>(s);
      std::string sc;
      for (int i = 0; i < g.pig_players; ++i) sc += (i ? " " : "") + std::to_string(p.score[i]);
      return "Scores: " + sc + ", Turn total: " + std::to_string(p.turn_total) +
             "\nCurrent player: " + std::to_string(p.turn_player) +
             (p.cur < 0 ? " (rolling)\n" : "\n");
    }
  }
  return "";
}

std::string StateActionToString(const HostState& s, int player, int64_t a) {
  const GameCfg& g = s.game->cfg;
  switch (g.kind) {
    case kTicTacToe:
      return std::string(player == 0 ? "x" : "o") + "(" + std::to_string(a / 3) +
             "," + std::to_string(a % 3) + ")";
    case kConnectFour:
      return std::string(player == 0 ? "x" : "o") + std::to_string(a);
    case kBreakthrough: {
      const int cap = static_cast<int>(a & 1);
      const int sq = static_cast<int>(a >> 1);
      const int dir = sq % 6, src = sq / 6;
      const int r1 = src / g.cols, c1 = src % g.cols;
      const int r2 = r1 + (dir < 3 ? 1 : -1), c2 = c1 + (dir % 3) - 1;
      std::string out;
      out += static_cast<char>('a' + c1);
      out += static_cast<char>('1' + (g.rows - 1 - r1));
      out += static_cast<char>('a' + c2);
      out += static_cast<char>('1' + (g.rows - 1 - r2));
      if (cap) out += "*";
      return out;
    }
    case kHex: {
      bool ea, eb;
      if (g.rows > kB128Side)
        HexBig::edges_if(St<HexBig>(s), g, player, static_cast<int>(a), &ea, &eb);
      else
        Hex::edges_if(St<Hex>(s), g, player, static_cast<int>(a), &ea, &eb);
      char ch;
      if (player == 0) ch = ea && eb ? 'X' : (ea ? 'y' : (eb ? 'z' : 'x'));
      else ch = ea && eb ? 'O' : (ea ? 'p' : (eb ? 'q' : 'o'));
      return std::string(1, ch) + "(" + std::to_string(a % g.rows) + "," +
             std::to_string(a / g.rows) + ")";
    }
    case kGo: {
      std::string out = player == 0 ? "B " : "W ";
      if (a == g.rows * g.cols) return out + "PASS";
      const int r = static_cast<int>(a / g.rows), c = static_cast<int>(a % g.rows);
      char col = static_cast<char>('a' + c);
      if (col >= 'i') ++col;
      return out + std::string(1, col) + std::to_string(r + 1);
    }
    case kPig:  // pig.cc:71-79
      if (player < 0) return "chance outcome " + std::to_string(a);
      return a == 0 ? "roll" : "stop";
  }
  return "";
}

}  // namespace osm
