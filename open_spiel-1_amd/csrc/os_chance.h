// MCTS over games with chance nodes: the search of
// os_mcts.h::mcts_search with the reference's chance handling, for the lane
// layout (one search per lane) and the host check.
//
//   * expansion at a chance node: Prior = ChanceOutcomes() in outcome order
//     (mcts.cc:73-76 / mcts.py:78-79), shuffled like any prior; the children's
//     player is kChancePlayerId (mcts.cc:276);
//   * selection at a chance node: SampleAction(ChanceOutcomes(), rng_) with the
//     BOT stream (mcts.cc:285-296) -- absl::Uniform(rng_, 0.0, 1.0) under the
//     C++ policy, RandomState.choice(actions, p=probs) under numpy
//     (mcts.py:326-333) -- then the child holding that action;
//   * rollouts sample chance nodes the same way from the evaluator stream
//     (mcts.cc:47-49 / mcts.py:64-67);
//   * backup credits a chance node's reward to the root player (mcts.cc:354-355
//     / mcts.py:409-410); the solver proves a chance node only when all its
//     children hold the same outcome (mcts.cc:361-374 / mcts.py:415-424).
// Turns no longer alternate with depth, so each path entry records the player
// choosing at that node.
#ifndef OS_CHANCE_H_
#define OS_CHANCE_H_

#include "os_mcts.h"

namespace osm {

constexpr int kChancePathCap = 256;  // tree depth bound (kPathOverflow beyond it)

// One chance outcome's index in ChanceOutcomes() order.
template <class G, int Policy, class Rng>
OS_HD int sample_chance(const GameCfg& g, Rng& rng) {
  const int n = G::chance_count(g);
  const double p = G::chance_prob(g);
  if (Policy == kPolicyCpp) return SampleEquiprobable(n, p, AbslUniformDouble01(rng));
  return NpChoiceEquiprobable(rng, n, p);
}

// RandomRolloutEvaluator::Evaluate's playout with chance nodes; returns the
// terminal's outcome code (G::ret0).
template <class G, int Policy, class Rng>
OS_HD int rollout_ret0_chance(typename G::State s, const GameCfg& g, typename G::Ctx& ctx,
                              Rng& ev) {
  while (!G::terminal(s, g)) {
    const typename G::Legal l = G::legal(s, g, ctx);
    int k;
    if (G::chance(s)) {
      k = sample_chance<G, Policy>(g, ev);
    } else {
      k = static_cast<int>(Policy == kPolicyCpp
                               ? AbslUniform(ev, static_cast<uint32_t>(l.count))
                               : NpChoice(ev, static_cast<uint32_t>(l.count)));
    }
    G::apply(s, g, ctx, l.kth(k));
  }
  return G::ret0(s, g, ctx);
}

// The playout a search runs at a leaf: the serial one above, unless a
// kernel's stream type has a faster equivalent (os_wave.h specialises this
// for pig on the wave layout).  Same words drawn, same result.
template <class G, int Policy, class Rng>
struct ChanceRollout {
  OS_HD static int run(const typename G::State& s, const GameCfg& g, typename G::Ctx& ctx,
                       Rng& ev) {
    return rollout_ret0_chance<G, Policy>(s, g, ctx, ev);
  }
};

OS_HD int reward_player(int p, int root_player) { return p < 0 ? root_player : p; }

// Evaluate()'s return vector (mcts.cc:42-71) for up to G::kMaxPlayers
// players, indexed through unrolled selects only (registers, no scratch).
template <class G>
struct Returns {
  double v[G::kMaxPlayers];
  // Returns() of a terminal with outcome code `code`.
  OS_HD void set(int code, const GameCfg& g) {
#pragma unroll
    for (int i = 0; i < G::kMaxPlayers; ++i) v[i] = OutValue<G>::value(code, i, g);
  }
  // result[k] += r[k] (the reference sums rollouts in order, then divides).
  OS_HD void add(int code, const GameCfg& g) {
#pragma unroll
    for (int i = 0; i < G::kMaxPlayers; ++i) v[i] += OutValue<G>::value(code, i, g);
  }
  OS_HD void div(int n) {
#pragma unroll
    for (int i = 0; i < G::kMaxPlayers; ++i) v[i] /= n;
  }
  OS_HD double of(int p) const {
    double x = 0.0;
#pragma unroll
    for (int i = 0; i < G::kMaxPlayers; ++i) x = i == p ? v[i] : x;
    return x;
  }
};

// Same contract as mcts_search; path_cap <= kChancePathCap.
template <class G, class R, int Policy, class Rng>
OS_HD SearchResult mcts_search_chance(const GameCfg& g, const SearchParams& sp,
                                      const typename G::State& root,
                                      typename G::Ctx& ctx, Node<R>* nodes, uint32_t cap,
                                      Rng& bot, Rng& ev, PathEnt<R>* path,
                                      uint16_t* actbuf, int path_cap,
                                      uint32_t* pages = nullptr, uint32_t own_page = 0) {
  SearchResult res;
  res.status = kOk;
  res.sims = 0;
  res.gc_runs = 0;
  res.max_depth = 0;
  res.scanned = res.backed = res.expanded = res.solver_scanned = 0;
  const int P0 = G::to_move(root);
  // The player choosing at path node d (-1: chance) lives in path[d].nc, a
  // field this search does not otherwise use: a per-thread array indexed by
  // depth would sit in scratch memory.
  if (path_cap > kChancePathCap) path_cap = kChancePathCap;
  nodes[0].first = 0;
  nodes[0].n = 0;
  nodes[0].w = 0;
  nodes[0].action = 0;
  nodes[0].nchild = 0;
  nodes[0].out = kUnsolved;
  uint32_t used = 1;
  int nodes_count = 1;
  int gc_limit = 5;
  const double inf = __builtin_huge_val();

  for (int sim = 0; sim < sp.max_simulations; ++sim) {
    typename G::State s = root;
    ctx.reset();
    int depth = 0;
    path[0].idx = 0;
    // ---- selection / expansion (ApplyTreePolicy, mcts.cc:255-323) ----
    for (;;) {
      const uint32_t x = path[depth].idx;
      const Node<R> nx = nodes[x];
      if (G::terminal(s, g) || nx.n <= 0) break;
      const int cp = G::to_move(s);  // -1 at a chance node
      path[depth].nc = cp;
      uint32_t first = nx.first;
      int nc = nx.nchild;
      const typename G::Legal l = G::legal(s, g, ctx);
      if (nc == 0) {
        nc = l.count;
        for (int k = 0; k < nc; ++k) actbuf[k] = static_cast<uint16_t>(l.kth(k));
        if (Policy == kPolicyCpp) CppShuffle(actbuf, nc, bot);
        else NpShuffle(actbuf, nc, bot);
        if (used + static_cast<uint32_t>(nc) > cap &&
            !(pages && take_page(pages, own_page, &used, &cap))) {
          res.status = kArenaOverflow;
          goto done;
        }
        first = used;
        used += nc;
        for (int k = 0; k < nc; ++k) {
          Node<R>& c = nodes[first + k];
          c.first = 0;
          c.n = 0;
          c.w = 0;
          c.action = actbuf[k];
          c.nchild = 0;
          c.out = kUnsolved;
        }
        nodes[x].first = first;
        nodes[x].nchild = static_cast<uint8_t>(nc);
        nodes_count += nc;
        res.expanded += nc;
      }
      int chosen = 0;
      if (cp < 0) {
        const int a = l.kth(sample_chance<G, Policy>(g, bot));
        for (int k = 0; k < nc; ++k)
          if (nodes[first + k].action == a) chosen = k;
      } else {
        const double logN = sp.log_lut[nx.n];  // sqrt(N) under PUCT
        const double cprior = puct_prior_term(sp.uct_c, nc);
        double best = -inf;
        res.scanned += nc;
        for (int k = 0; k < nc; ++k) {
          const Node<R> c = nodes[first + k];
          double v;
          if (c.out != kUnsolved) v = OutValue<G>::value(c.out, cp, g);
          else if (sp.puct) v = puct_unsolved(static_cast<double>(c.w), c.n, cprior, logN);
          else if (c.n == 0) v = inf;
          else v = static_cast<double>(c.w) / c.n + sp.uct_c * __builtin_sqrt(logN / c.n);
          if (v > best) {
            best = v;
            chosen = k;
          }
        }
      }
      G::apply(s, g, ctx, nodes[first + chosen].action);
      if (++depth >= path_cap) {
        res.status = kPathOverflow;
        goto done;
      }
      path[depth].idx = first + chosen;
    }
    if (depth > res.max_depth) res.max_depth = depth;
    {
      // ---- evaluation: the n-player return vector ----
      bool solved;
      Returns<G> ret;
      if (G::terminal(s, g)) {
        const int code = G::ret0(s, g, ctx);
        nodes[path[depth].idx].out = static_cast<int8_t>(code);
        solved = sp.solve != 0;
        ret.set(code, g);
      } else {
        solved = false;
        const int leaf_mark = ctx.mark();
        for (int k = 0; k < sp.n_rollouts; ++k) {
          if (k) ctx.rewind(leaf_mark);
          const int code = ChanceRollout<G, Policy, Rng>::run(s, g, ctx, ev);
          if (k) ret.add(code, g);
          else ret.set(code, g);
        }
        // The reference divides by n_rollouts (mcts.cc:69) -- for one rollout
        // x / 1 == x exactly, so the kMaxPlayers f64 divisions are skipped.
        if (sp.n_rollouts != 1) ret.div(sp.n_rollouts);
      }
      // ---- backup + MCTS-Solver (mcts.cc:351-396) ----
      for (int d = depth; d >= 0; --d) {
        Node<R>& nd = nodes[path[d].idx];
        const int pl = d == 0 ? P0 : reward_player(path[d - 1].nc, P0);
        nd.w += static_cast<R>(ret.of(pl));
        nd.n += 1;
        res.backed += 1;
        if (solved && nd.nchild > 0) {
          res.solver_scanned += nd.nchild;
          if (path[d].nc < 0) {  // chance node: all children share one outcome
            const int8_t o = nodes[nd.first].out;
            bool same = o != kUnsolved;
            for (int k = 1; k < nd.nchild; ++k) same = same && nodes[nd.first + k].out == o;
            if (same) nd.out = o;
            else solved = false;
          } else {
            const int cpl = path[d].nc;
            int best = -1;
            int8_t best_out = kUnsolved;
            double bestv = 0.0;
            bool all_solved = true;
            for (int k = 0; k < nd.nchild; ++k) {
              const int8_t co = nodes[nd.first + k].out;
              if (co == kUnsolved) {
                all_solved = false;
              } else {
                const double v = OutValue<G>::value(co, cpl, g);
                if (best < 0 || v > bestv) {
                  best = k;
                  bestv = v;
                  best_out = co;
                }
              }
            }
            if (best >= 0 && (all_solved || bestv == 1.0)) nd.out = best_out;
            else solved = false;
          }
        }
      }
    }
    res.sims = sim + 1;
    if (nodes[0].out != kUnsolved) break;
    if (Policy == kPolicyCpp) {
      if (nodes[0].nchild == 1) break;
      if (sp.max_nodes > 1 && nodes_count >= sp.max_nodes) {
        const int st = garbage_collect(nodes, used, cap, gc_limit, &nodes_count);
        if (st != kOk) {
          res.status = st;
          goto done;
        }
        res.gc_runs++;
        gc_limit = static_cast<int>(gc_limit * (nodes_count > sp.max_nodes / 2 ? 1.25 : 0.9));
        if (gc_limit < 5) gc_limit = 5;
      }
    }
  }
done:
  res.nodes = nodes_count;
  res.used = pages ? 1 + res.expanded : used;  // nodes allocated (mcts_search)
  return res;
}

}  // namespace osm

#endif  // OS_CHANCE_H_
