// Resumable MCTS with an EXTERNAL evaluator (the
// AlphaZero actor boundary) -- host and device (OS_HD).
//
// The reference MCTSBot calls Evaluator::Prior when it expands a node
// (mcts.cc:262-282) and Evaluator::Evaluate on the leaf (mcts.cc:341-348);
// with VPNetEvaluator both are neural-network inferences on (LegalActions,
// ObservationTensor) (vpevaluator.cc:70-98).  A GPU kernel cannot call the
// network, so each search is a state machine: az_step advances it to its next
// evaluator request, writes the request (observation tensor of the player to
// move + legal-action mask) into caller-owned buffers and returns; the caller
// runs the network on ALL pending requests as one batch, writes priors /
// values back, and steps again.  Child selection is UCT (mcts.cc:89-100) or
// PUCT (mcts.cc:102-111); backup, MCTS-Solver, early stop and GC are those of
// mcts.cc:325-428 (same code shape as os_mcts.h::mcts_search).  Results are
// bit-exact with the reference MCTSBot driving the same evaluator.
//
// Dirichlet root noise (mcts.cc:177-192, applied at :265-273): the reference
// draws std::gamma_distribution<double>(alpha, 1) from the bot rng_ at the
// root's expansion, before the shuffle.  The gamma sampler is libstdc++'s
// (Marsaglia-Tsang over a polar-method normal, with libm log / sqrt / pow), so
// its bits are only reproducible with that library: the host runtime draws it
// at prepare time with the real std::gamma_distribution over the same
// mt19937(seed) stream (a fresh bot's rng_ is untouched until the root
// expands) and hands the kernel the normalised noise and the number of words
// it consumed; the kernel mixes the priors and advances its stream by that
// count.  go's positional-superko set of the pending simulation lives in the
// continuation (AzLog), so searches resume mid-descent with it intact.
//
// Fused requests (`raw` != nullptr; os_az_set_requests OS_AZ_REQUESTS_FUSED):
// for an evaluator that is a pure function of (observation, legal actions) --
// VPNetEvaluator is: both calls are one cached inference of the same network
// on the same input (vpevaluator.cc:70-98) -- the leaf's Evaluate request also
// asks for its Prior (kAzBoth).  The priors are parked in legal-action order
// in `raw`, in the arena slots the leaf's children will occupy (nodes[x].first
// is set while nchild is still 0), and the expansion that the reference does
// on the node's next visit takes them from there -- with the bot rng's shuffle
// and Dirichlet mixing at exactly the same point of the stream.  Every
// simulation then costs one evaluator round instead of two; results are
// unchanged for a pure evaluator.
#ifndef OS_AZ_H_
#define OS_AZ_H_

#include "os_mcts.h"

namespace osm {

enum AzStage : int32_t { kAzStart = 0, kAzWaitPrior = 1, kAzWaitValue = 2, kAzDone = 3 };
enum AzRequest : int32_t { kAzNone = 0, kAzPrior = 1, kAzValue = 2, kAzBoth = 3 };

// Request counters of one step: search r adds to shard r % kAzShards; each
// shard on its own 128-B line (kAzShardStride int32s).
constexpr int kAzShards = 256;
constexpr int kAzShardStride = 32;

constexpr int kAzLogCap = 248;  // go: positions after the root on one tree path (<= 2 * 11 * 11)
constexpr int kAzHeads = 122;   // go: stone-count buckets, 0 .. 11 * 11

// go's position log of the pending simulation (GoCtx arrays + fill count);
// empty for games without a history context.
template <bool kLog>
struct AzLog {};
template <>
struct AzLog<true> {
  uint64_t log[kAzLogCap];
  uint32_t link[kAzLogCap];
  uint8_t head[kAzHeads];
  int32_t n_log;
};

OS_HD void az_bind_log(NoCtx&, AzLog<false>&, bool) {}
OS_HD void az_save_log(const NoCtx&, AzLog<false>&) {}
// Points the context at the continuation's log; `resume` restores the count
// (a fresh search resets it at its first simulation).
OS_HD void az_bind_log(GoCtx& c, AzLog<true>& m, bool resume) {
  c.log = m.log;
  c.link = m.link;
  c.head = m.head;
  c.stride = 1;
  c.head_stride = 1;
  c.cap = kAzLogCap;
  c.n_log = resume ? m.n_log : 0;
  c.init_base_filter();
}
OS_HD void az_save_log(const GoCtx& c, AzLog<true>& m) { m.n_log = c.n_log; }

// Dirichlet root noise of one search, drawn by the host (see above):
// noise[j] pairs with the j-th legal action in ascending order; `skip` = MT
// words the draws consumed.  noise == nullptr: alpha = 0 (no noise).
struct AzNoise {
  const double* noise;
  int32_t skip;
  double eps;
};

// Per-search continuation, resident in HBM between steps.
template <class G>
struct AzSlot {
  typename G::State s;  // working state at the pending request
  int32_t stage;
  int32_t sim;
  int32_t depth;
  int32_t nodes_count;
  int32_t gc_limit;
  int32_t mt_idx;       // MtStream idx / pre of the bot rng
  int32_t mt_pre;
  uint32_t used;
  SearchResult res;
  uint32_t path[kMaxPath];
  AzLog<G::State::kNeedsLog> glog;
};

// One search's request / response views (caller-owned buffers).
struct AzIo {
  int32_t* kind;         // out: kAzNone / kAzPrior / kAzValue
  float* obs;            // out: ObservationTensor(current player), obs_size
  uint8_t* legal;        // out: legal-action mask, num_actions
  const double* prior;   // in: action-indexed priors (read for legal actions; kAzPrior, kAzBoth)
  const double* value;   // in: player-0 value (Evaluate returns {v, -v})
};

template <class G>
OS_HD void az_request(const GameCfg& g, const typename G::State& s, int kind, const AzIo& io,
                      int obs_size, int num_actions, typename G::Ctx& ctx) {
  *io.kind = kind;
  const int cells = g.rows * g.cols;
  const int planes = obs_size / cells;
  const int p = G::to_move(s);
  // Cell-major walk of the CHW tensor: the cell's contents are decoded once
  // for all its planes (no per-element division by the cell count).
  for (int c = 0; c < cells; ++c)
    for (int pl = 0; pl < planes; ++pl) io.obs[pl * cells + c] = G::obs(s, g, p, pl, c);
  for (int a = 0; a < num_actions; ++a) io.legal[a] = 0;
  const typename G::Legal l = G::legal(s, g, ctx);
  for (int k = 0; k < l.count; ++k) io.legal[l.kth(k)] = 1;
}

// Advances one search until it needs the evaluator (request written, returns)
// or finishes (kind = kAzNone, stage = kAzDone).  `ctx` is the game's
// history context with its root fields set (go: Zobrist table, the positions
// before the root, n_heads); its log is bound to the continuation here.
// `raw` ([cap], or nullptr for separate Prior / Evaluate requests): the parked
// priors of fused requests (see above).  `np_policy`: the search of
// python/algorithms/mcts.py (mcts.py:292-333, 395-443) -- the expansion's
// shuffle is RandomState.shuffle on the bot's stream, and the search stops
// early only on a solved root (no single-child stop; the caller disables GC).
template <class G>
OS_HD void az_step(const GameCfg& g, const SearchParams& sp, int puct,
                   const typename G::State& root, AzSlot<G>& sl, Node<double>* nodes,
                   double* prior, double* raw, uint32_t cap, MtStream& bot, const AzIo& io,
                   int obs_size, int num_actions, typename G::Ctx& ctx, const AzNoise& nz,
                   bool np_policy = false) {
  az_bind_log(ctx, sl.glog, sl.stage != kAzStart);
  const int P0 = G::to_move(root);
  const double inf = __builtin_huge_val();
  typename G::State s = sl.s;
  int depth = sl.depth;
  int phase;  // 0 new simulation, 1 descend, 2 expand with priors, 3 value ready
  double v0 = 0.0;
  bool solved = false;
  bool from_raw = false;  // phase 2 takes the parked priors of a fused request
  if (sl.stage == kAzDone) {
    *io.kind = kAzNone;
    return;
  }
  if (sl.stage == kAzStart) {
    nodes[0].first = 0;
    nodes[0].n = 0;
    nodes[0].w = 0;
    nodes[0].action = 0;
    nodes[0].nchild = 0;
    nodes[0].out = kUnsolved;
    prior[0] = 1.0;  // SearchNode(kInvalidAction, player_id, 1) (mcts.cc:328)
    sl.used = 1;
    sl.nodes_count = 1;
    sl.gc_limit = 5;
    sl.sim = 0;
    sl.res.status = kOk;
    sl.res.sims = sl.res.gc_runs = sl.res.max_depth = 0;
    sl.res.scanned = sl.res.backed = sl.res.expanded = sl.res.solver_scanned = 0;
    sl.res.rng_words = sl.res.pad = 0;
    phase = 0;
  } else if (sl.stage == kAzWaitPrior) {
    phase = 2;
  } else {
    v0 = *io.value;
    solved = false;
    phase = 3;
    if (raw != nullptr) {
      // Park the leaf's priors (legal order) where its children will live.
      const typename G::Legal l = G::legal(s, g, ctx);
      const int nc = l.count;
      if (sl.used + static_cast<uint32_t>(nc) > cap) {
        sl.res.status = kArenaOverflow;
        phase = -1;
      } else {
        for (int j = 0; j < nc; ++j) raw[sl.used + j] = io.prior[l.kth(j)];
        nodes[sl.path[depth]].first = sl.used;
        sl.used += nc;
      }
    }
  }
  for (;;) {
    if (phase < 0) break;
    if (phase == 0) {
      if (sl.sim >= sp.max_simulations) break;
      s = root;
      ctx.reset();
      depth = 0;
      sl.path[0] = 0;
      phase = 1;
    }
    if (phase == 2) {
      // Prior of the pending node (legal order), shuffled with the bot rng
      // like std::shuffle over (action, prior) pairs (mcts.cc:275-282).
      const uint32_t x = sl.path[depth];
      const typename G::Legal l = G::legal(s, g, ctx);
      const int nc = l.count;
      if (!from_raw && sl.used + static_cast<uint32_t>(nc) > cap) {
        sl.res.status = kArenaOverflow;
        break;
      }
      const bool noisy = x == 0 && nz.noise != nullptr;
      if (noisy)  // dirichlet_noise consumed these words of rng_ (mcts.cc:265-267)
        for (int i = 0; i < nz.skip; ++i) bot.next();
      uint8_t perm[kMaxChildren];
      for (int k = 0; k < nc; ++k) perm[k] = static_cast<uint8_t>(k);
      if (np_policy) NpShuffle(perm, nc, bot);  // mcts.py:320
      else CppShuffle(perm, nc, bot);
      const uint32_t first = from_raw ? nodes[x].first : sl.used;
      for (int k = 0; k < nc; ++k) {
        const int j = perm[k];
        const int a = l.kth(j);
        const double p = from_raw ? raw[first + j] : io.prior[a];
        Node<double>& c = nodes[first + k];
        c.first = 0;
        c.n = 0;
        c.w = 0.0;
        c.action = static_cast<uint16_t>(a);
        c.nchild = 0;
        c.out = kUnsolved;
        // (1 - eps) * p + eps * noise, separately rounded (mcts.cc:269-271)
        prior[first + k] = noisy ? (1.0 - nz.eps) * p + nz.eps * nz.noise[j] : p;
      }
      nodes[x].first = first;
      nodes[x].nchild = static_cast<uint8_t>(nc);
      if (!from_raw) sl.used += nc;
      from_raw = false;
      sl.nodes_count += nc;
      sl.res.expanded += nc;
      phase = 1;
    }
    if (phase == 1) {
      for (;;) {
        const uint32_t x = sl.path[depth];
        const Node<double> nx = nodes[x];
        if (G::terminal(s, g) || nx.n <= 0) break;
        if (nx.nchild == 0 && raw != nullptr && nx.first != 0) {
          from_raw = true;  // parked by this node's fused request: expand now
          break;
        }
        if (nx.nchild == 0) {
          sl.s = s;
          sl.depth = depth;
          az_save_log(ctx, sl.glog);
          sl.stage = kAzWaitPrior;
          az_request<G>(g, s, kAzPrior, io, obs_size, num_actions, ctx);
          return;
        }
        const int cp = P0 ^ (depth & 1);
        const double dN = static_cast<double>(nx.n);
        const double logN = sp.log_lut[nx.n];
        const double sqrtN = __builtin_sqrt(dN);
        double best = -inf;
        int chosen = 0;
        sl.res.scanned += nx.nchild;
        for (int k = 0; k < nx.nchild; ++k) {
          const Node<double> c = nodes[nx.first + k];
          double v;
          if (c.out != kUnsolved) {
            v = outcome_for(c.out, cp);
          } else if (puct) {  // mcts.cc:102-111
            const double q = c.n != 0 ? c.w / static_cast<double>(c.n) : 0.0;
            v = q + sp.uct_c * prior[nx.first + k] * sqrtN / static_cast<double>(c.n + 1);
          } else if (c.n == 0) {
            v = inf;
          } else {
            const double dn = static_cast<double>(c.n);
            v = c.w / dn + sp.uct_c * __builtin_sqrt(logN / dn);
          }
          if (v > best) {
            best = v;
            chosen = k;
          }
        }
        const uint32_t ci = nx.first + chosen;
        G::apply(s, g, ctx, nodes[ci].action);
        if (++depth >= kMaxPath) {
          sl.res.status = kPathOverflow;
          sl.stage = kAzDone;
          *io.kind = kAzNone;
          return;
        }
        sl.path[depth] = ci;
      }
      if (from_raw) {
        phase = 2;
        continue;
      }
      if (depth > sl.res.max_depth) sl.res.max_depth = depth;
      if (G::terminal(s, g)) {
        const int r0 = G::ret0(s, g, ctx);
        nodes[sl.path[depth]].out = static_cast<int8_t>(r0);
        solved = sp.solve != 0;
        v0 = static_cast<double>(r0);
        phase = 3;
      } else {
        sl.s = s;
        sl.depth = depth;
        az_save_log(ctx, sl.glog);
        sl.stage = kAzWaitValue;
        az_request<G>(g, s, raw != nullptr ? kAzBoth : kAzValue, io, obs_size, num_actions, ctx);
        return;
      }
    }
    if (phase == 3) {
      // ---- backup + MCTS-Solver (mcts.cc:351-396) ----
      for (int d = depth; d >= 0; --d) {
        Node<double>& nd = nodes[sl.path[d]];
        const int pl = d == 0 ? P0 : (P0 ^ ((d - 1) & 1));
        nd.w += pl == 0 ? v0 : -v0;
        nd.n += 1;
        sl.res.backed += 1;
        if (solved && nd.nchild > 0) {
          const int cpl = P0 ^ (d & 1);
          sl.res.solver_scanned += nd.nchild;
          int best = -1;
          int8_t best_out = kUnsolved;
          double bestv = 0.0;
          bool all_solved = true;
          for (int k = 0; k < nd.nchild; ++k) {
            const int8_t co = nodes[nd.first + k].out;
            if (co == kUnsolved) {
              all_solved = false;
            } else {
              const double v = outcome_for(co, cpl);
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
      sl.sim += 1;
      sl.res.sims = sl.sim;
      if (nodes[0].out != kUnsolved) break;  // mcts.cc:398-401, mcts.py:440-441
      if (!np_policy && nodes[0].nchild == 1) break;
      if (sp.max_nodes > 1 && sl.nodes_count >= sp.max_nodes) {      // mcts.cc:402-424
        const int st = garbage_collect(nodes, sl.used, cap, sl.gc_limit, &sl.nodes_count);
        if (st != kOk) {
          sl.res.status = st;
          break;
        }
        sl.res.gc_runs++;
        sl.gc_limit = static_cast<int>(sl.gc_limit *
                                       (sl.nodes_count > sp.max_nodes / 2 ? 1.25 : 0.9));
        if (sl.gc_limit < 5) sl.gc_limit = 5;
      }
      phase = 0;
    }
  }
  sl.res.nodes = sl.nodes_count;
  sl.res.used = sl.used;
  sl.stage = kAzDone;
  *io.kind = kAzNone;
}

}  // namespace osm

#endif  // OS_AZ_H_
