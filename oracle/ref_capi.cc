// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_rng.h header).
// C entry points for ctypes (tests/, smoke(), bench.py cpu_baseline).  The
// names are prefixed `oref_` so they can never be confused with the product
// library's `os_` C-ABI.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ref_games.h"
#include "ref_mcts.h"
#include "ref_rng.h"

using namespace oref;

namespace {
thread_local std::string g_err;

struct OGame {
  std::unique_ptr<RGame> game;
};

std::unique_ptr<RState> Replay(const RGame& g, const int64_t* a, int64_t n) {
  auto s = g.NewInitialState();
  for (int64_t i = 0; i < n; ++i) s->ApplyAction(a[i]);
  return s;
}

void JsonEscape(const std::string& in, std::string* out) {
  for (char c : in) {
    switch (c) {
      case '"': *out += "\\\""; break;
      case '\\': *out += "\\\\"; break;
      case '\n': *out += "\\n"; break;
      default: *out += c;
    }
  }
}

// Per-root search output, child-ordered (the tree's shuffled order).
struct RootOut {
  int32_t* child_action;
  int32_t* child_n;
  double* child_w;
  int8_t* child_out;   // outcome for the child's player, 2 = unsolved
  int32_t* nchild;
  int32_t* root_n;
  double* root_w;
  int8_t* root_out;
  int64_t* best_action;
  int32_t* nodes;
};

// The int8 outcome of the C-ABI: the value (two players), or its sign (pig
// with more players: 1, -1 / (n - 1), 0).
int8_t Sign(double v) { return static_cast<int8_t>(v > 0 ? 1 : (v < 0 ? -1 : 0)); }

void FillOut(const SearchNode& root, int max_children, int64_t r,
             const SearchStats& st, const RootOut& o) {
  int nc = static_cast<int>(root.children.size());
  o.nchild[r] = nc;
  for (int k = nc; k < max_children; ++k) {  // padding, as the C-ABI fills it
    o.child_action[r * max_children + k] = -1;
    o.child_n[r * max_children + k] = 0;
    o.child_w[r * max_children + k] = 0.0;
    o.child_out[r * max_children + k] = 2;
  }
  for (int k = 0; k < nc && k < max_children; ++k) {
    const SearchNode& c = root.children[k];
    o.child_action[r * max_children + k] = static_cast<int32_t>(c.action);
    o.child_n[r * max_children + k] = c.explore_count;
    o.child_w[r * max_children + k] = c.total_reward;
    o.child_out[r * max_children + k] = c.outcome.empty() ? 2 : Sign(c.outcome[c.player]);
  }
  o.root_n[r] = root.explore_count;
  o.root_w[r] = root.total_reward;
  o.root_out[r] = root.outcome.empty() ? 2 : Sign(root.outcome[root.player]);
  o.best_action[r] = nc > 0 ? root.BestChild().action : -1;
  o.nodes[r] = st.nodes;
}
}  // namespace

extern "C" {

const char* oref_last_error() { return g_err.c_str(); }

void* oref_game_new(const char* game_string) {
  std::string err;
  auto g = LoadGame(game_string, &err);
  if (!g) {
    g_err = err;
    return nullptr;
  }
  auto* og = new OGame;
  og->game = std::move(g);
  return og;
}

void oref_game_free(void* g) { delete static_cast<OGame*>(g); }

int oref_game_info(void* g, int32_t* num_actions, int32_t* max_len) {
  auto* og = static_cast<OGame*>(g);
  *num_actions = og->game->NumDistinctActions();
  *max_len = og->game->MaxGameLength();
  return 0;
}

// Replays `actions` and writes a JSON object describing the reached state.
// Returns the number of bytes needed (excluding NUL); truncates to buflen-1.
// go: Tromp-Taylor score of the position after `actions`.
float oref_go_score(void* g, const int64_t* actions, int64_t n) {
  auto* og = static_cast<OGame*>(g);
  return GoScore(*Replay(*og->game, actions, n));
}

int64_t oref_state_json(void* g, const int64_t* actions, int64_t n, char* buf,
                        int64_t buflen) {
  auto* og = static_cast<OGame*>(g);
  auto s = Replay(*og->game, actions, n);
  std::string j = "{\"is_terminal\":";
  j += s->IsTerminal() ? "true" : "false";
  j += ",\"current_player\":" + std::to_string(s->CurrentPlayer());
  auto r = s->Returns();
  char tmp[64];
  j += ",\"returns\":[";
  for (size_t i = 0; i < r.size(); ++i) {
    std::snprintf(tmp, sizeof tmp, "%s%.17g", i ? "," : "", r[i]);
    j += tmp;
  }
  j += "],\"is_chance_node\":";
  j += s->IsChanceNode() ? "true" : "false";
  if (s->IsChanceNode()) {
    j += ",\"chance_outcomes\":[";
    auto co = s->ChanceOutcomes();
    for (size_t i = 0; i < co.size(); ++i) {
      std::snprintf(tmp, sizeof tmp, "%s[%lld,%.17g]", i ? "," : "",
                    static_cast<long long>(co[i].first), co[i].second);
      j += tmp;
    }
    j += "]";
  }
  j += ",\"legal_actions\":[";
  auto la = s->LegalActions();
  for (size_t i = 0; i < la.size(); ++i) {
    if (i) j += ",";
    j += std::to_string(la[i]);
  }
  j += "],\"string_legal_actions\":[";
  for (size_t i = 0; i < la.size(); ++i) {
    if (i) j += ",";
    j += "\"";
    JsonEscape(s->ActionToString(s->CurrentPlayer(), la[i]), &j);
    j += "\"";
  }
  j += "],\"observation_string\":\"";
  JsonEscape(s->ToString(), &j);
  j += "\"}";
  if (buflen > 0) {
    int64_t m = std::min<int64_t>(buflen - 1, static_cast<int64_t>(j.size()));
    std::memcpy(buf, j.data(), m);
    buf[m] = 0;
  }
  return static_cast<int64_t>(j.size());
}

// n random playouts from the replayed root, evaluator seed seeds[i] each
// (one RandomRolloutEvaluator(n_rollouts, seed) per playout).
int oref_rollouts(void* g, const int64_t* actions, int64_t n_actions,
                  int64_t n, int32_t n_rollouts, const uint32_t* seeds,
                  double* out_returns, int32_t* out_moves) {
  auto* og = static_cast<OGame*>(g);
  auto root = Replay(*og->game, actions, n_actions);
  for (int64_t i = 0; i < n; ++i) {
    RandomRolloutEvaluator ev(n_rollouts, seeds[i]);
    if (out_moves) {
      // Count moves of a single rollout separately (diagnostic only).
      std::mt19937 g2(seeds[i]);
      auto ws = root->Clone();
      int m = 0;
      while (!ws->IsTerminal()) {
        auto a = ws->LegalActions();
        ws->ApplyAction(a[AbslUniformU64(g2, a.size())]);
        ++m;
      }
      out_moves[i] = m;
    }
    auto r = ev.Evaluate(*root);
    out_returns[2 * i] = r[0];
    out_returns[2 * i + 1] = r[1];
  }
  return 0;
}

// Batched independent searches (the C++ MCTSBot path, mcts.cc), one bot +
// one RandomRolloutEvaluator per root, `threads` host threads with static
// round-robin root assignment; puct != 0: ChildSelectionPolicy::PUCT.  Writes
// child-ordered outputs.
int oref_mcts_batch(void* g, int64_t num_roots, const int64_t* root_actions,
                    const int64_t* root_offsets, double uct_c,
                    int32_t max_simulations, int32_t n_rollouts,
                    int64_t max_memory_mb, int32_t solve,
                    const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                    int32_t max_children, int32_t* child_action,
                    int32_t* child_n, double* child_w, int8_t* child_out,
                    int32_t* nchild, int32_t* root_n, double* root_w,
                    int8_t* root_out, int64_t* best_action, int32_t* nodes,
                    int32_t threads, int32_t puct) {
  auto* og = static_cast<OGame*>(g);
  RootOut o{child_action, child_n, child_w, child_out, nchild,
            root_n,       root_w,  root_out, best_action, nodes};
  if (threads < 1) threads = 1;
  auto work = [&](int t) {
    for (int64_t r = t; r < num_roots; r += threads) {
      auto state = Replay(*og->game, root_actions + root_offsets[r],
                          root_offsets[r + 1] - root_offsets[r]);
      RandomRolloutEvaluator ev(n_rollouts, eval_seeds[r]);
      MCTSBot bot(*og->game, &ev, uct_c, max_simulations, max_memory_mb,
                  solve != 0, bot_seeds[r], puct != 0);
      SearchStats st;
      auto root = bot.MCTSearch(*state, &st);
      FillOut(*root, max_children, r, st, o);
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
    for (auto& t : ts) t.join();
  }
  return 0;
}

// The Python mcts.py path with one shared numpy RandomState(seed);
// puct != 0: child_selection_fn = SearchNode.puct_value (mcts.py:135-142).
int oref_mcts_numpy(void* g, const int64_t* actions, int64_t n_actions,
                    double uct_c, int32_t max_simulations, int32_t n_rollouts,
                    int32_t solve, uint32_t seed, int32_t max_children,
                    int32_t* child_action, int32_t* child_n, double* child_w,
                    int8_t* child_out, int32_t* nchild, int32_t* root_n,
                    double* root_w, int8_t* root_out, int64_t* best_action,
                    int32_t* nodes, uint32_t* rng_state_out, int32_t puct) {
  auto* og = static_cast<OGame*>(g);
  auto state = Replay(*og->game, actions, n_actions);
  std::mt19937 rng(seed);
  NumpyMCTSBot bot(*og->game, &rng, uct_c, max_simulations, n_rollouts,
                   solve != 0, puct != 0);
  SearchStats st;
  auto root = bot.Search(*state, &st);
  RootOut o{child_action, child_n, child_w, child_out, nchild,
            root_n,       root_w,  root_out, best_action, nodes};
  FillOut(*root, max_children, 0, st, o);
  if (rng_state_out) rng_state_out[0] = rng();  // next raw word, for tests
  return 0;
}

// Raw known-answer vectors: n words of std::mt19937(seed) / mt19937_64.
void oref_mt19937(uint32_t seed, int64_t n, uint32_t* out) {
  std::mt19937 g(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = g();
}
void oref_mt19937_64(uint64_t seed, int64_t n, uint64_t* out) {
  std::mt19937_64 g(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = g();
}
// k draws of absl::Uniform(rng, 0u, n) from mt19937(seed).
void oref_absl_uniform(uint32_t seed, uint64_t n, int64_t k, uint64_t* out) {
  std::mt19937 g(seed);
  for (int64_t i = 0; i < k; ++i) out[i] = AbslUniformU64(g, n);
}
// std::shuffle of [0..n) with mt19937(seed) (libstdc++ of this toolchain).
void oref_std_shuffle(uint32_t seed, int32_t n, int32_t* out) {
  std::mt19937 g(seed);
  std::vector<std::pair<int64_t, double>> v;
  for (int i = 0; i < n; ++i) v.emplace_back(i, 1.0 / n);
  std::shuffle(v.begin(), v.end(), g);
  for (int i = 0; i < n; ++i) out[i] = static_cast<int32_t>(v[i].first);
}

// Wall-clock helper for the CPU baseline: runs oref_mcts_batch on the first
// `num_roots` roots with `threads` threads and returns seconds.
double oref_time_mcts_batch(void* g, int64_t num_roots,
                            const int64_t* root_actions,
                            const int64_t* root_offsets, double uct_c,
                            int32_t max_simulations, int32_t n_rollouts,
                            int64_t max_memory_mb, int32_t solve,
                            const uint32_t* bot_seeds,
                            const uint32_t* eval_seeds, int32_t threads,
                            int64_t* total_sims) {
  auto* og = static_cast<OGame*>(g);
  std::atomic<int64_t> sims{0};
  if (threads < 1) threads = 1;
  auto t0 = std::chrono::steady_clock::now();
  auto work = [&](int t) {
    int64_t local = 0;
    for (int64_t r = t; r < num_roots; r += threads) {
      auto state = Replay(*og->game, root_actions + root_offsets[r],
                          root_offsets[r + 1] - root_offsets[r]);
      RandomRolloutEvaluator ev(n_rollouts, eval_seeds[r]);
      MCTSBot bot(*og->game, &ev, uct_c, max_simulations, max_memory_mb,
                  solve != 0, bot_seeds[r]);
      SearchStats st;
      auto root = bot.MCTSearch(*state, &st);
      local += root->explore_count;
    }
    sims += local;
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
  for (auto& t : ts) t.join();
  auto t1 = std::chrono::steady_clock::now();
  *total_sims = sims.load();
  return std::chrono::duration<double>(t1 - t0).count();
}

// An external evaluator (the VPNetEvaluator role, vpevaluator.cc:70-80):
// Prior / Evaluate delegate to a C callback that sees the state's history.
// kind 1 = Prior: prior_out[a] for every legal a (action-indexed);
// kind 2 = Evaluate: *value_out = player-0 value (returns {v, -v}).
typedef int (*oref_eval_cb)(const int64_t* history, int64_t n, int32_t kind,
                            double* prior_out, double* value_out);

class CallbackEvaluator : public oref::Evaluator {
 public:
  CallbackEvaluator(oref_eval_cb cb, int num_actions) : cb_(cb), buf_(num_actions) {}
  std::vector<double> Evaluate(const RState& state) override {
    double v = 0;
    const auto& h = state.History();
    cb_(h.data(), static_cast<int64_t>(h.size()), 2, buf_.data(), &v);
    return {v, -v};
  }
  std::vector<std::pair<Action, double>> Prior(const RState& state) override {
    const auto& h = state.History();
    double v = 0;
    cb_(h.data(), static_cast<int64_t>(h.size()), 1, buf_.data(), &v);
    std::vector<std::pair<Action, double>> out;
    for (Action a : state.LegalActions()) out.emplace_back(a, buf_[a]);
    return out;  // LegalActions order, as VPNetModel::Inference returns it
  }

 private:
  oref_eval_cb cb_;
  std::vector<double> buf_;
};

// MCTSBot::MCTSearch with an external evaluator and UCT (puct = 0) or PUCT
// (puct = 1) child selection (mcts.cc:297-304) and Dirichlet root noise when
// dirichlet_alpha > 0 (mcts.cc:265-273), one bot seed per root; same output
// layout as oref_mcts_batch.
int oref_mcts_external(void* g, int64_t num_roots, const int64_t* root_actions,
                       const int64_t* root_offsets, double uct_c, int32_t max_simulations,
                       int64_t max_memory_mb, int32_t solve, int32_t puct,
                       double dirichlet_alpha, double dirichlet_epsilon,
                       const uint32_t* bot_seeds, oref_eval_cb cb, int32_t max_children,
                       int32_t* child_action, int32_t* child_n, double* child_w,
                       int8_t* child_out, int32_t* nchild, int32_t* root_n, double* root_w,
                       int8_t* root_out, int64_t* best_action, int32_t* nodes) {
  auto* og = static_cast<OGame*>(g);
  RootOut o{child_action, child_n, child_w, child_out, nchild,
            root_n,       root_w,  root_out, best_action, nodes};
  CallbackEvaluator ev(cb, og->game->NumDistinctActions());
  for (int64_t r = 0; r < num_roots; ++r) {
    auto state = Replay(*og->game, root_actions + root_offsets[r],
                        root_offsets[r + 1] - root_offsets[r]);
    MCTSBot bot(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
                bot_seeds[r], puct != 0, dirichlet_alpha, dirichlet_epsilon);
    SearchStats st;
    auto root = bot.MCTSearch(*state, &st);
    FillOut(*root, max_children, r, st, o);
  }
  return 0;
}

// Self-play as examples/mcts_example.cc:77-136 PlayGame drives it (and
// evaluate_bots.cc:21-60): two MCTSBots (seeds bot_seeds[2g], [2g+1]) sharing
// ONE RandomRolloutEvaluator (eval_seeds[g]; mcts_example.cc:151-157), each
// move = bots[CurrentPlayer]->Step = MCTSearch + BestChild (mcts.cc:219-226),
// until terminal; MCTSBot's InformAction/Restart are no-ops (mcts.h:162-163).
// Per game: actions[g*max_len ...], len[g], returns[2g..2g+1]; visits (may be
// NULL) [g][max_len][num_actions] = action-indexed root child explore counts.
int oref_selfplay(void* g, int64_t num_games, const int64_t* start_actions,
                  const int64_t* start_offsets, double uct_c, int32_t max_simulations,
                  int32_t n_rollouts, int64_t max_memory_mb, int32_t solve,
                  const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                  int32_t max_len, int64_t* actions, int32_t* len, double* returns,
                  int32_t* visits, int32_t threads) {
  auto* og = static_cast<OGame*>(g);
  const int A = og->game->NumDistinctActions();
  if (threads < 1) threads = 1;
  std::atomic<int> err{0};
  auto work = [&](int t) {
    for (int64_t r = t; r < num_games; r += threads) {
      auto state = Replay(*og->game, start_actions + start_offsets[r],
                          start_offsets[r + 1] - start_offsets[r]);
      RandomRolloutEvaluator ev(n_rollouts, eval_seeds[r]);
      MCTSBot b0(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
                 bot_seeds[2 * r]);
      MCTSBot b1(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
                 bot_seeds[2 * r + 1]);
      MCTSBot* bots[2] = {&b0, &b1};
      int m = 0;
      while (!state->IsTerminal()) {
        if (m >= max_len) {
          err = 1;
          break;
        }
        SearchStats st;
        auto root = bots[state->CurrentPlayer()]->MCTSearch(*state, &st);
        const Action a = root->BestChild().action;
        actions[r * max_len + m] = a;
        if (visits) {
          int32_t* v = visits + (r * max_len + m) * static_cast<int64_t>(A);
          for (int i = 0; i < A; ++i) v[i] = 0;
          for (const SearchNode& c : root->children) v[c.action] = c.explore_count;
        }
        state->ApplyAction(a);
        ++m;
      }
      for (int k = m; k < max_len; ++k) actions[r * max_len + k] = -1;
      len[r] = m;
      std::vector<double> ret = state->Returns();
      returns[2 * r] = ret[0];
      returns[2 * r + 1] = ret[1];
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
    for (auto& t : ts) t.join();
  }
  return err.load() ? -1 : 0;
}

// CPU baseline of the external-evaluator search (bench.py --config az): the
// same MCTSBot (PUCT, Dirichlet root noise) with a native evaluator that costs
// nothing -- uniform Prior over LegalActions, Evaluate = {0, 0} -- so the time
// is the search's own; R searches on `threads` host threads.  Returns seconds.
class ZeroEvaluator : public oref::Evaluator {
 public:
  std::vector<double> Evaluate(const RState&) override { return {0.0, 0.0}; }
  std::vector<std::pair<Action, double>> Prior(const RState& state) override {
    const std::vector<Action> legal = state.LegalActions();
    std::vector<std::pair<Action, double>> out;
    for (Action a : legal) out.emplace_back(a, 1.0 / legal.size());
    return out;
  }
};

double oref_time_mcts_zero_eval(void* g, int64_t num_roots, const int64_t* root_actions,
                                const int64_t* root_offsets, double uct_c,
                                int32_t max_simulations, int32_t puct, double dirichlet_alpha,
                                double dirichlet_epsilon, const uint32_t* bot_seeds,
                                int32_t threads, int64_t* total_sims) {
  auto* og = static_cast<OGame*>(g);
  std::atomic<int64_t> sims{0};
  if (threads < 1) threads = 1;
  auto t0 = std::chrono::steady_clock::now();
  auto work = [&](int t) {
    ZeroEvaluator ev;
    int64_t local = 0;
    for (int64_t r = t; r < num_roots; r += threads) {
      auto state = Replay(*og->game, root_actions + root_offsets[r],
                          root_offsets[r + 1] - root_offsets[r]);
      MCTSBot bot(*og->game, &ev, uct_c, max_simulations, 1000, true, bot_seeds[r], puct != 0,
                  dirichlet_alpha, dirichlet_epsilon);
      SearchStats st;
      local += bot.MCTSearch(*state, &st)->explore_count;
    }
    sims += local;
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
  for (auto& t : ts) t.join();
  *total_sims = sims.load();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// AlphaZero's PlayGame (alpha_zero.cc:64-118) over the self-play pairing of
// oref_selfplay (two MCTSBots, seeds bot_seeds[2g], [2g+1], UCT or PUCT,
// sharing RandomRolloutEvaluator(n_rollouts, eval_seeds[g])) with one actor
// std::mt19937(actor_seeds[g]) per game: resign cutoff drawn first
// (alpha_zero.cc:154-157) when `resign`; each move's policy pow(count, 1/T)
// over the root's children (exponent 1 when temperature <= 0), normalised;
// SampleAction before temperature_drop moves (temperature > 0), BestChild
// after; root value total_reward / explore_count; early stop when |root
// value| > cutoff.  policy [g][max_len][A] (action-indexed), root_value
// [g][max_len]; rows past the end are zero.
int oref_selfplay_az(void* g, int64_t num_games, const int64_t* start_actions,
                     const int64_t* start_offsets, double uct_c, int32_t max_simulations,
                     int32_t n_rollouts, int64_t max_memory_mb, int32_t solve, int32_t puct,
                     const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                     const uint32_t* actor_seeds, double temperature, int32_t temperature_drop,
                     int32_t resign, double cutoff_value, double cutoff_probability,
                     int32_t max_len, int64_t* actions, int32_t* len, double* returns,
                     double* policy, double* root_value) {
  auto* og = static_cast<OGame*>(g);
  const int A = og->game->NumDistinctActions();
  for (int64_t r = 0; r < num_games; ++r) {
    auto state = Replay(*og->game, start_actions + start_offsets[r],
                        start_offsets[r + 1] - start_offsets[r]);
    RandomRolloutEvaluator ev(n_rollouts, eval_seeds[r]);
    MCTSBot b0(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
               bot_seeds[2 * r], puct != 0);
    MCTSBot b1(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
               bot_seeds[2 * r + 1], puct != 0);
    MCTSBot* bots[2] = {&b0, &b1};
    std::mt19937 rng(actor_seeds[r]);
    double cutoff = og->game->MaxUtility() + 1;
    if (resign && AbslUniformDouble01(rng) < cutoff_probability) cutoff = cutoff_value;
    std::fill(policy + r * max_len * static_cast<int64_t>(A),
              policy + (r + 1) * max_len * static_cast<int64_t>(A), 0.0);
    std::fill(root_value + r * max_len, root_value + (r + 1) * max_len, 0.0);
    int m = 0;
    bool stopped = false;
    while (!state->IsTerminal()) {
      if (m >= max_len) return -1;
      const Player player = state->CurrentPlayer();
      SearchStats st;
      auto root = bots[player]->MCTSearch(*state, &st);
      std::vector<std::pair<Action, double>> pol;
      for (const SearchNode& c : root->children)
        pol.emplace_back(c.action, temperature > 0 ? std::pow(c.explore_count, 1.0 / temperature)
                                                   : static_cast<double>(c.explore_count));
      double sum = 0;
      for (const auto& x : pol) sum += x.second;  // NormalizePolicy (spiel.cc:327-335)
      for (auto& x : pol) x.second /= sum;
      Action a;
      if (temperature > 0 && m < temperature_drop)
        a = SampleAction(pol, AbslUniformDouble01(rng));
      else
        a = root->BestChild().action;
      const double rv = root->total_reward / root->explore_count;
      for (const auto& x : pol) policy[(r * max_len + m) * static_cast<int64_t>(A) + x.first] = x.second;
      root_value[r * max_len + m] = rv;
      actions[r * max_len + m] = a;
      state->ApplyAction(a);
      ++m;
      if (!state->IsTerminal() && std::abs(rv) > cutoff) {
        returns[2 * r + player] = rv;
        returns[2 * r + 1 - player] = -rv;
        stopped = true;
        break;
      }
    }
    for (int k = m; k < max_len; ++k) actions[r * max_len + k] = -1;
    len[r] = m;
    if (!stopped) {
      const std::vector<double> ret = state->Returns();
      returns[2 * r] = ret[0];
      returns[2 * r + 1] = ret[1];
    }
  }
  return 0;
}

// AlphaZero's actor games (alpha_zero.cc:64-118 PlayGame, :120-135 InitAZBot):
// per game two MCTSBots (seeds bot_seeds[2g], [2g+1]; PUCT or UCT; Dirichlet
// root noise alpha / epsilon) sharing the external evaluator `cb`, one actor
// std::mt19937(actor_seeds[g]): resign cutoff drawn first when `resign`;
// pow(count, 1/T) policy, SampleAction before temperature_drop moves,
// BestChild after; root value; early stop at |value| > cutoff.  Same outputs
// as oref_selfplay_az.
int oref_az_actor(void* g, int64_t num_games, const int64_t* start_actions,
                  const int64_t* start_offsets, double uct_c, int32_t max_simulations,
                  int64_t max_memory_mb, int32_t solve, int32_t puct, double dirichlet_alpha,
                  double dirichlet_epsilon, const uint32_t* bot_seeds,
                  const uint32_t* actor_seeds, double temperature, int32_t temperature_drop,
                  int32_t resign, double cutoff_value, double cutoff_probability,
                  oref_eval_cb cb, int32_t max_len, int64_t* actions, int32_t* len,
                  double* returns, double* policy, double* root_value) {
  auto* og = static_cast<OGame*>(g);
  const int A = og->game->NumDistinctActions();
  CallbackEvaluator ev(cb, A);
  for (int64_t r = 0; r < num_games; ++r) {
    auto state = Replay(*og->game, start_actions + start_offsets[r],
                        start_offsets[r + 1] - start_offsets[r]);
    MCTSBot b0(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
               bot_seeds[2 * r], puct != 0, dirichlet_alpha, dirichlet_epsilon);
    MCTSBot b1(*og->game, &ev, uct_c, max_simulations, max_memory_mb, solve != 0,
               bot_seeds[2 * r + 1], puct != 0, dirichlet_alpha, dirichlet_epsilon);
    MCTSBot* bots[2] = {&b0, &b1};
    std::mt19937 rng(actor_seeds[r]);
    double cutoff = og->game->MaxUtility() + 1;
    if (resign && AbslUniformDouble01(rng) < cutoff_probability) cutoff = cutoff_value;
    std::fill(policy + r * max_len * static_cast<int64_t>(A),
              policy + (r + 1) * max_len * static_cast<int64_t>(A), 0.0);
    std::fill(root_value + r * max_len, root_value + (r + 1) * max_len, 0.0);
    int m = 0;
    bool stopped = false;
    while (!state->IsTerminal()) {
      if (m >= max_len) return -1;
      const Player player = state->CurrentPlayer();
      SearchStats st;
      auto root = bots[player]->MCTSearch(*state, &st);
      std::vector<std::pair<Action, double>> pol;
      for (const SearchNode& c : root->children)
        pol.emplace_back(c.action, std::pow(c.explore_count, 1.0 / temperature));
      double sum = 0;
      for (const auto& x : pol) sum += x.second;
      for (auto& x : pol) x.second /= sum;
      const Action a = m < temperature_drop ? SampleAction(pol, AbslUniformDouble01(rng))
                                            : root->BestChild().action;
      const double rv = root->total_reward / root->explore_count;
      for (const auto& x : pol) policy[(r * max_len + m) * static_cast<int64_t>(A) + x.first] = x.second;
      root_value[r * max_len + m] = rv;
      actions[r * max_len + m] = a;
      state->ApplyAction(a);
      ++m;
      if (!state->IsTerminal() && std::abs(rv) > cutoff) {
        returns[2 * r + player] = rv;
        returns[2 * r + 1 - player] = -rv;
        stopped = true;
        break;
      }
    }
    for (int k = m; k < max_len; ++k) actions[r * max_len + k] = -1;
    len[r] = m;
    if (!stopped) {
      const std::vector<double> ret = state->Returns();
      returns[2 * r] = ret[0];
      returns[2 * r + 1] = ret[1];
    }
  }
  return 0;
}

// mcts_test.cc:24-36 InitBot bots driven by EvaluateBots (evaluate_bots.cc:
// 24-61): num_bots MCTSBots (seeds bot_seeds[i]) sharing ONE
// RandomRolloutEvaluator(n_rollouts, eval_seed); chance nodes sampled by
// SampleAction(outcomes, absl::Uniform(mt19937(seed), 0.0, 1.0)).  Writes the
// game's actions (history[cap]) and Returns() (returns[num_players]); returns
// the history length, or -1 when it exceeds cap.
int64_t oref_evaluate_mcts_bots(void* g, int32_t num_bots, const uint32_t* bot_seeds,
                                int32_t n_rollouts, uint32_t eval_seed, double uct_c,
                                int32_t max_simulations, int64_t max_memory_mb, int32_t solve,
                                uint32_t seed, int64_t* history, int64_t cap,
                                double* returns) {
  auto* og = static_cast<OGame*>(g);
  RandomRolloutEvaluator ev(n_rollouts, eval_seed);
  std::vector<std::unique_ptr<MCTSBot>> bots;
  for (int i = 0; i < num_bots; ++i)
    bots.push_back(std::make_unique<MCTSBot>(*og->game, &ev, uct_c, max_simulations,
                                             max_memory_mb, solve != 0, bot_seeds[i]));
  std::mt19937 rng(seed);
  auto state = og->game->NewInitialState();
  int64_t m = 0;
  while (!state->IsTerminal()) {
    Action a;
    if (state->IsChanceNode()) {
      a = SampleAction(state->ChanceOutcomes(), AbslUniformDouble01(rng));
    } else {
      SearchStats st;
      auto root = bots[state->CurrentPlayer()]->MCTSearch(*state, &st);
      a = root->BestChild().action;  // MCTSBot::Step (mcts.cc:219-226)
    }
    if (m >= cap) return -1;
    history[m++] = a;
    state->ApplyAction(a);
  }
  const auto r = state->Returns();
  for (size_t i = 0; i < r.size(); ++i) returns[i] = r[i];
  return m;
}

}  // extern "C"
