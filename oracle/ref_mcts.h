// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_rng.h header).
//
// Reference-faithful restatement of open_spiel/algorithms/mcts.{h,cc}
// (UCT + MCTS-Solver + RandomRolloutEvaluator + garbage collection) and of the
// Python twin open_spiel/python/algorithms/mcts.py (numpy RandomState
// consumption).  Object-per-node trees, Clone-per-simulation and vector legal
// actions are kept on purpose: this is both the parity oracle and the CPU
// baseline ("port") timed by bench.py.
#ifndef OS_ORACLE_REF_MCTS_H_
#define OS_ORACLE_REF_MCTS_H_

#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>
#include <numeric>
#include <random>
#include <vector>

#include "ref_games.h"
#include "ref_rng.h"

namespace oref {

// mcts.h:78-87 Evaluator interface.
class Evaluator {
 public:
  virtual ~Evaluator() {}
  virtual std::vector<double> Evaluate(const RState& state) = 0;
  virtual std::vector<std::pair<Action, double>> Prior(const RState& state) = 0;
};

// spiel.cc:337-372 SampleAction(outcomes, z): the first outcome whose
// [sum, sum + prob) holds z.
inline Action SampleAction(const std::vector<std::pair<Action, double>>& outcomes, double z) {
  double sum = 0;
  for (const auto& o : outcomes) {
    if (sum <= z && z < sum + o.second) return o.first;
    sum += o.second;
  }
  return outcomes.back().first;  // the reference raises SpielFatalError here
}

// mcts.h:92-106 / mcts.cc:42-71
class RandomRolloutEvaluator : public Evaluator {
 public:
  RandomRolloutEvaluator(int n_rollouts, uint32_t seed)
      : n_rollouts_(n_rollouts), rng_(seed) {}
  std::vector<double> Evaluate(const RState& state) override {
    std::vector<double> result;
    for (int i = 0; i < n_rollouts_; ++i) {
      std::unique_ptr<RState> ws = state.Clone();
      while (!ws->IsTerminal()) {
        if (ws->IsChanceNode()) {  // mcts.cc:47-49
          ws->ApplyAction(SampleAction(ws->ChanceOutcomes(), AbslUniformDouble01(rng_)));
          continue;
        }
        std::vector<Action> actions = ws->LegalActions();
        ws->ApplyAction(actions[AbslUniformU64(rng_, actions.size())]);
      }
      std::vector<double> r = ws->Returns();
      if (result.empty()) {
        result.swap(r);
      } else {
        for (size_t k = 0; k < result.size(); ++k) result[k] += r[k];
      }
    }
    for (double& v : result) v /= n_rollouts_;
    return result;
  }
  // mcts.cc:73-86
  std::vector<std::pair<Action, double>> Prior(const RState& state) override {
    if (state.IsChanceNode()) return state.ChanceOutcomes();
    std::vector<Action> legal = state.LegalActions();
    std::vector<std::pair<Action, double>> prior;
    prior.reserve(legal.size());
    for (Action a : legal) prior.emplace_back(a, 1.0 / legal.size());
    return prior;
  }
  std::mt19937& rng() { return rng_; }

 private:
  int n_rollouts_;
  std::mt19937 rng_;
};

// mcts.h:109-137
struct SearchNode {
  Action action = 0;
  double prior = 0;
  Player player = 0;
  int explore_count = 0;
  double total_reward = 0;
  std::vector<double> outcome;
  std::vector<SearchNode> children;

  SearchNode() {}
  SearchNode(Action a, Player p, double pr) : action(a), prior(pr), player(p) {}

  // mcts.cc:89-100; built with -ffp-contract=off (the reference is built
  // without -march, so x86-64 never contracts a*b+c into an FMA).
  double UCTValue(int parent_explore_count, double uct_c) const {
    if (!outcome.empty()) return outcome[player];
    if (explore_count == 0) return std::numeric_limits<double>::infinity();
    return total_reward / explore_count +
           uct_c * std::sqrt(std::log(parent_explore_count) / explore_count);
  }
  // mcts.cc:102-111
  double PUCTValue(int parent_explore_count, double uct_c) const {
    if (!outcome.empty()) return outcome[player];
    return ((explore_count != 0 ? total_reward / explore_count : 0) +
            uct_c * prior * std::sqrt(parent_explore_count) / (explore_count + 1));
  }
  // mcts.cc:113-123
  bool CompareFinal(const SearchNode& b) const {
    double out = outcome.empty() ? 0 : outcome[player];
    double out_b = b.outcome.empty() ? 0 : b.outcome[b.player];
    if (out != out_b) return out < out_b;
    if (explore_count != b.explore_count) return explore_count < b.explore_count;
    return total_reward < b.total_reward;
  }
  // mcts.cc:125-141 (std::max_element: first maximum)
  const SearchNode& BestChild() const {
    return *std::max_element(
        children.begin(), children.end(),
        [](const SearchNode& a, const SearchNode& b) { return a.CompareFinal(b); });
  }
};

struct SearchStats {
  int nodes = 0;       // nodes_ at the end of the search (mcts.cc:281)
  int gc_runs = 0;
  int sims_run = 0;
};

// mcts.cc:177-192: gamma(alpha, 1) draws from the bot rng, normalised by
// their left-fold sum (absl::c_accumulate).
inline std::vector<double> DirichletNoise(int count, double alpha, std::mt19937* rng) {
  std::vector<double> noise;
  noise.reserve(count);
  std::gamma_distribution<double> gamma(alpha, 1.0);
  for (int i = 0; i < count; ++i) noise.emplace_back(gamma(*rng));
  double sum = std::accumulate(noise.begin(), noise.end(), 0.0);
  for (double& v : noise) v /= sum;
  return noise;
}

// mcts.cc:194-443: UCT or PUCT child selection, optional Dirichlet root noise.
class MCTSBot {
 public:
  MCTSBot(const RGame& game, Evaluator* evaluator, double uct_c,
          int max_simulations, int64_t max_memory_mb, bool solve, uint32_t seed,
          bool puct = false, double dirichlet_alpha = 0.0, double dirichlet_epsilon = 0.0)
      : dirichlet_alpha_(dirichlet_alpha),
        dirichlet_epsilon_(dirichlet_epsilon),
        puct_(puct),
        uct_c_(uct_c),
        max_simulations_(max_simulations),
        max_nodes_(static_cast<int>((max_memory_mb << 20) / kNodeBytes + 1)),
        solve_(solve),
        max_utility_(game.MaxUtility()),
        rng_(seed),
        evaluator_(evaluator) {}

  // sizeof(SearchNode) of the reference on LP64 libstdc++.
  static constexpr int64_t kNodeBytes = 80;

  std::unique_ptr<SearchNode> MCTSearch(const RState& state, SearchStats* st) {
    Player player_id = state.CurrentPlayer();
    nodes_ = 1;
    gc_limit_ = kMinGcLimit;
    auto root = std::make_unique<SearchNode>(kInvalidAction, player_id, 1);
    std::vector<SearchNode*> visit_path;
    std::vector<double> returns;
    visit_path.reserve(64);
    int i = 0;
    for (; i < max_simulations_; ++i) {
      visit_path.clear();
      returns.clear();
      std::unique_ptr<RState> ws = ApplyTreePolicy(root.get(), state, &visit_path);
      bool solved;
      if (ws->IsTerminal()) {
        returns = ws->Returns();
        visit_path.back()->outcome = returns;
        solved = solve_;
      } else {
        returns = evaluator_->Evaluate(*ws);
        solved = false;
      }
      for (auto it = visit_path.rbegin(); it != visit_path.rend(); ++it) {
        SearchNode* node = *it;
        node->total_reward +=
            returns[node->player == kChancePlayerId ? player_id : node->player];
        node->explore_count += 1;
        if (solved && !node->children.empty() &&
            node->children[0].player == kChancePlayerId) {  // mcts.cc:361-374
          const std::vector<double>& outcome = node->children[0].outcome;
          if (!outcome.empty() &&
              std::all_of(node->children.begin() + 1, node->children.end(),
                          [&outcome](const SearchNode& c) { return c.outcome == outcome; }))
            node->outcome = outcome;
          else
            solved = false;
        } else if (solved && !node->children.empty()) {
          Player player = node->children[0].player;
          const SearchNode* best = nullptr;
          bool all_solved = true;
          for (const SearchNode& child : node->children) {
            if (child.outcome.empty()) {
              all_solved = false;
            } else if (best == nullptr ||
                       child.outcome[player] > best->outcome[player]) {
              best = &child;
            }
          }
          if (best != nullptr &&
              (all_solved || best->outcome[player] == max_utility_)) {
            node->outcome = best->outcome;
          } else {
            solved = false;
          }
        }
      }
      if (!root->outcome.empty() || root->children.size() == 1) {
        ++i;
        break;
      }
      if (max_nodes_ > 1 && nodes_ >= max_nodes_) {
        GarbageCollect(root.get());
        gc_limit_ = static_cast<int>(gc_limit_ * (nodes_ > max_nodes_ / 2 ? 1.25 : 0.9));
        gc_limit_ = std::max(kMinGcLimit, gc_limit_);
        if (st) st->gc_runs++;
      }
    }
    if (st) {
      st->nodes = nodes_;
      st->sims_run = i;
    }
    return root;
  }

 private:
  static constexpr int kMinGcLimit = 5;

  std::unique_ptr<RState> ApplyTreePolicy(SearchNode* root, const RState& state,
                                          std::vector<SearchNode*>* path) {
    path->push_back(root);
    std::unique_ptr<RState> ws = state.Clone();
    SearchNode* cur = root;
    while (!ws->IsTerminal() && cur->explore_count > 0) {
      if (cur->children.empty()) {
        auto legal = evaluator_->Prior(*ws);
        if (cur == root && dirichlet_alpha_ > 0) {  // mcts.cc:265-273
          std::vector<double> noise = DirichletNoise(legal.size(), dirichlet_alpha_, &rng_);
          for (size_t i = 0; i < legal.size(); ++i)
            legal[i].second =
                (1 - dirichlet_epsilon_) * legal[i].second + dirichlet_epsilon_ * noise[i];
        }
        std::shuffle(legal.begin(), legal.end(), rng_);
        Player player = ws->CurrentPlayer();
        cur->children.reserve(legal.size());
        for (auto [a, p] : legal) cur->children.emplace_back(a, player, p);
        nodes_ += static_cast<int>(cur->children.capacity());
      }
      SearchNode* chosen = nullptr;
      if (ws->IsChanceNode()) {  // mcts.cc:285-296: sample with the bot rng_
        const Action a = SampleAction(ws->ChanceOutcomes(), AbslUniformDouble01(rng_));
        for (SearchNode& child : cur->children)
          if (child.action == a) {
            chosen = &child;
            break;
          }
      } else {
        double max_value = -std::numeric_limits<double>::infinity();
        for (SearchNode& child : cur->children) {
          double val = puct_ ? child.PUCTValue(cur->explore_count, uct_c_)
                             : child.UCTValue(cur->explore_count, uct_c_);
          if (val > max_value) {
            max_value = val;
            chosen = &child;
          }
        }
      }
      ws->ApplyAction(chosen->action);
      cur = chosen;
      path->push_back(cur);
    }
    return ws;
  }

  void GarbageCollect(SearchNode* node) {
    if (node->children.empty()) return;
    bool clear = node->explore_count < gc_limit_;
    for (SearchNode& c : node->children) GarbageCollect(&c);
    if (clear) {
      nodes_ -= static_cast<int>(node->children.capacity());
      node->children.clear();
      node->children.shrink_to_fit();
    }
  }

  double dirichlet_alpha_;
  double dirichlet_epsilon_;
  bool puct_;
  double uct_c_;
  int max_simulations_;
  int max_nodes_;
  int nodes_ = 0;
  int gc_limit_ = kMinGcLimit;
  bool solve_;
  double max_utility_;
  std::mt19937 rng_;
  Evaluator* evaluator_;
};

// python/algorithms/mcts.py:199-443 with ONE numpy RandomState (MT19937,
// legacy seeding == std::mt19937 init) shared by bot and evaluator, as in
// mcts_test.py:41-54.  Differences from the C++ bot kept: no single-child
// early stop, no GC, shuffle = numpy Fisher-Yates, rollout pick = choice().
class NumpyMCTSBot {
 public:
  NumpyMCTSBot(const RGame& game, std::mt19937* rng, double uct_c,
               int max_simulations, int n_rollouts, bool solve, bool puct = false)
      : uct_c_(uct_c), max_simulations_(max_simulations),
        n_rollouts_(n_rollouts), solve_(solve), puct_(puct),
        max_utility_(game.MaxUtility()), rng_(rng) {}

  std::unique_ptr<SearchNode> Search(const RState& state, SearchStats* st) {
    Player root_player = state.CurrentPlayer();
    auto root = std::make_unique<SearchNode>(kInvalidAction, root_player, 1);
    int i = 0;
    int nodes = 1;
    for (; i < max_simulations_; ++i) {
      std::vector<SearchNode*> path = {root.get()};
      std::unique_ptr<RState> ws = state.Clone();
      SearchNode* cur = root.get();
      while (!ws->IsTerminal() && cur->explore_count > 0) {
        if (cur->children.empty()) {
          std::vector<std::pair<Action, double>> la;
          if (ws->IsChanceNode()) {  // mcts.py:78-79 prior = chance_outcomes()
            la = ws->ChanceOutcomes();
          } else {
            std::vector<Action> legal = ws->LegalActions();
            for (Action a : legal) la.emplace_back(a, 1.0 / legal.size());
          }
          for (size_t k = la.size() - 1; k >= 1; --k) {  // numpy shuffle
            size_t j = NpRandomInterval(*rng_, k);
            std::swap(la[k], la[j]);
          }
          Player player = ws->CurrentPlayer();
          for (auto [a, p] : la) cur->children.emplace_back(a, player, p);
          nodes += static_cast<int>(la.size());
        }
        SearchNode* chosen = nullptr;
        if (ws->IsChanceNode()) {  // mcts.py:326-333
          const Action a = ChanceChoice(*ws);
          for (SearchNode& child : cur->children)
            if (child.action == a) {
              chosen = &child;
              break;
            }
        } else {
          double max_value = -std::numeric_limits<double>::infinity();
          for (SearchNode& child : cur->children) {
            // mcts.py:312-314: max() over child_selection_fn (uct_value or
            // puct_value, mcts.py:124-142; the same arithmetic as mcts.cc).
            double val = puct_ ? child.PUCTValue(cur->explore_count, uct_c_)
                               : child.UCTValue(cur->explore_count, uct_c_);
            if (chosen == nullptr || val > max_value) {
              max_value = val;
              chosen = &child;
            }
          }
        }
        ws->ApplyAction(chosen->action);
        cur = chosen;
        path.push_back(cur);
      }
      std::vector<double> returns;
      bool solved;
      if (ws->IsTerminal()) {
        returns = ws->Returns();
        path.back()->outcome = returns;
        solved = solve_;
      } else {
        returns = Evaluate(*ws);
        solved = false;
      }
      for (auto it = path.rbegin(); it != path.rend(); ++it) {
        SearchNode* node = *it;
        node->total_reward +=
            returns[node->player == kChancePlayerId ? root_player : node->player];
        node->explore_count += 1;
        if (solved && !node->children.empty() &&
            node->children[0].player == kChancePlayerId) {  // mcts.py:415-424
          const std::vector<double>& outcome = node->children[0].outcome;
          bool same = !outcome.empty();
          for (const SearchNode& c : node->children) same = same && c.outcome == outcome;
          if (same) node->outcome = outcome;
          else solved = false;
        } else if (solved && !node->children.empty()) {
          Player player = node->children[0].player;
          const SearchNode* best = nullptr;
          bool all_solved = true;
          for (const SearchNode& child : node->children) {
            if (child.outcome.empty()) all_solved = false;
            else if (best == nullptr || child.outcome[player] > best->outcome[player])
              best = &child;
          }
          if (best != nullptr && (all_solved || best->outcome[player] == max_utility_))
            node->outcome = best->outcome;
          else
            solved = false;
        }
      }
      if (!root->outcome.empty()) {
        ++i;
        break;
      }
    }
    if (st) {
      st->nodes = nodes;
      st->sims_run = i;
    }
    return root;
  }

 private:
  std::vector<double> Evaluate(const RState& state) {
    std::vector<double> result;
    for (int r = 0; r < n_rollouts_; ++r) {
      std::unique_ptr<RState> ws = state.Clone();
      while (!ws->IsTerminal()) {
        if (ws->IsChanceNode()) {  // mcts.py:64-67
          ws->ApplyAction(ChanceChoice(*ws));
          continue;
        }
        std::vector<Action> legal = ws->LegalActions();
        ws->ApplyAction(legal[NpChoiceIndex(*rng_, legal.size())]);
      }
      std::vector<double> ret = ws->Returns();
      if (result.empty()) result = ret;
      else for (size_t k = 0; k < result.size(); ++k) result[k] += ret[k];
    }
    for (double& v : result) v /= n_rollouts_;
    return result;
  }

  // random_state.choice(action_list, p=prob_list) over chance_outcomes().
  Action ChanceChoice(const RState& ws) {
    const auto o = ws.ChanceOutcomes();
    std::vector<double> p;
    for (const auto& e : o) p.push_back(e.second);
    return o[NpChoiceP(*rng_, p)].first;
  }

  double uct_c_;
  int max_simulations_;
  int n_rollouts_;
  bool solve_;
  bool puct_;
  double max_utility_;
  std::mt19937* rng_;
};

}  // namespace oref

#endif  // OS_ORACLE_REF_MCTS_H_
