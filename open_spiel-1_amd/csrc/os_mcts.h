// UCT MCTS with MCTS-Solver backup and random rollouts over a flat node
// arena: the single-search engine that the gfx950 kernel runs once per lane.
//
// Restates open_spiel/algorithms/mcts.cc (C++ bot: MCTSBot::MCTSearch
// :325-428, ApplyTreePolicy :255-323, UCTValue :89-100, RandomRolloutEvaluator
// ::Evaluate :42-71, GarbageCollect :430-443) and, under kPolicyNumpy, the
// Python twin open_spiel/python/algorithms/mcts.py:292-443 (one shared numpy
// RandomState, no single-child early stop, no GC).
//
// Tree layout: node 0 is the root; the children of a node are one contiguous
// block [first, first + nchild) in expansion (shuffled) order.  A node's
// player is implied by its depth (all five games strictly alternate turns):
// depth 0 -> root player P0, depth d >= 1 -> P0 ^ ((d - 1) & 1).
// Outcomes (the reference's `outcome` vector) are stored as the player-0
// value in {-1, 0, +1}; all five games are two-player zero-sum with returns
// (r, -r), so outcome[p] = p == 0 ? r : -r.  kUnsolved marks an empty vector.
#ifndef OS_MCTS_H_
#define OS_MCTS_H_

#include "os_common.h"
#include "os_games.h"
#include "os_rng.h"

namespace osm {

constexpr int8_t kUnsolved = 2;
constexpr int kPolicyCpp = 0;     // mcts.cc: bot rng + evaluator rng
constexpr int kPolicyNumpy = 1;   // mcts.py: one shared RandomState
constexpr int kMaxPath = 256;     // > every supported MaxGameLength
constexpr int kMaxChildren = 128; // >= every supported |LegalActions|

enum SearchStatus : int32_t {
  kOk = 0,
  kArenaOverflow = 1,   // node arena capacity exceeded
  kPathOverflow = 2,    // tree depth exceeded kMaxPath
  kGcStackOverflow = 3, // no arena space left for the GC traversal stack
  kGameOverflow = 4,    // self-play game longer than the trajectory buffer
};

// W (wide): a 16-bit child count, for go above 15 x 15 (up to 362 children;
// k_lsearch only).  Every other kernel keeps the 16-byte int32 node.
template <class R, bool W = false>
struct Node {
  uint32_t first;   // first child index (valid iff nchild > 0)
  int32_t n;        // explore_count
  R w;              // total_reward (int32 when n_rollouts == 1: exact)
  uint16_t action;
  typename std::conditional<W, uint16_t, uint8_t>::type nchild;
  int8_t out;       // player-0 outcome, or kUnsolved
};

struct SearchParams {
  double uct_c;
  int32_t max_simulations;
  int32_t n_rollouts;
  int32_t solve;
  int32_t max_nodes;        // (max_memory_mb << 20) / sizeof(SearchNode) + 1
  int32_t policy;           // kPolicyCpp / kPolicyNumpy
  int32_t puct;             // 0 UCTValue (mcts.cc:89-100), 1 PUCTValue (:102-111)
  // Parent term of the child value, N in [0, max_simulations], host libm:
  // log(N) under UCT, sqrt(N) under PUCT.
  const double* log_lut;
};

// SearchNode::PUCTValue (mcts.cc:102-111; mcts.py:135-142) of an unsolved
// child with the uniform prior 1 / nchild of RandomRolloutEvaluator::Prior
// (mcts.cc:73-86): cprior = uct_c * prior, sqrtN = sqrt(parent explore count).
// The reference's operation order: Q + ((uct_c * prior) * sqrt(N)) / (n + 1).
OS_HD double puct_prior_term(double uct_c, int nchild) {
  return uct_c * (1.0 / static_cast<double>(nchild));
}
OS_HD double puct_unsolved(double w, int32_t n, double cprior, double sqrtN) {
  const double q = n != 0 ? w / static_cast<double>(n) : 0.0;
  return q + cprior * sqrtN / static_cast<double>(n + 1);
}

#ifndef OS_AB_LANE_NOROLL
#define OS_AB_LANE_NOROLL 0
#endif
// Lane-layout UCT selection screened in f32 (mcts_search; 1) or the f64
// scan alone (0).  A/B knob; both exact.
#ifndef OS_LANE_SCREEN
#define OS_LANE_SCREEN 1
#endif

struct SearchResult {
  int32_t status;
  int32_t sims;     // simulations run (== root explore_count)
  int32_t nodes;    // the reference's nodes_ counter at exit
  uint32_t used;    // arena slots used
  int32_t gc_runs;
  int32_t max_depth;
  // Instrumentation for the algorithmic-bytes model:
  uint32_t scanned;    // child nodes read by UCT selection
  uint32_t backed;     // nodes updated by backup
  uint32_t expanded;   // child nodes written by expansion
  uint32_t solver_scanned;  // child nodes read by the MCTS-Solver backup
  uint32_t rng_words;  // MT19937 words drawn (set by the caller)
  uint32_t pad;
};

OS_HD double outcome_for(int8_t out0, int player) {
  return static_cast<double>(player == 0 ? out0 : -out0);
}

// mcts.cc:113-123 CompareFinal(a, b) == "a < b".
template <class R, bool W>
OS_HD bool final_less(const Node<R, W>& a, int pa, const Node<R, W>& b, int pb) {
  const double oa = a.out == kUnsolved ? 0.0 : outcome_for(a.out, pa);
  const double ob = b.out == kUnsolved ? 0.0 : outcome_for(b.out, pb);
  if (oa != ob) return oa < ob;
  if (a.n != b.n) return a.n < b.n;
  return static_cast<double>(a.w) < static_cast<double>(b.w);
}

// CompareFinal / BestChild with the game's outcome decoding (OutValue: pig
// with more than two players).
template <class G, class R, bool W>
OS_HD bool final_less_g(const Node<R, W>& a, const Node<R, W>& b, int p, const GameCfg& g) {
  const double oa = a.out == kUnsolved ? 0.0 : OutValue<G>::value(a.out, p, g);
  const double ob = b.out == kUnsolved ? 0.0 : OutValue<G>::value(b.out, p, g);
  if (oa != ob) return oa < ob;
  if (a.n != b.n) return a.n < b.n;
  return static_cast<double>(a.w) < static_cast<double>(b.w);
}
template <class G, class R, bool W>
OS_HD int best_child_g(const Node<R, W>* nodes, int child_player, const GameCfg& g) {
  const Node<R, W>& root = nodes[0];
  if (root.nchild == 0) return -1;
  int best = 0;
  for (int k = 1; k < root.nchild; ++k)
    if (final_less_g<G>(nodes[root.first + best], nodes[root.first + k], child_player, g))
      best = k;
  return best;
}
// The C-ABI's int8 outcome of a solved node for player p: the sign of its
// Returns()[p] (== the value in two-player games; with n players +1 / -1 / 0
// stand for 1, -1 / (n - 1) and 0, which the game fixes).
template <class G>
OS_HD int8_t out_sign(int8_t out, int p, const GameCfg& g) {
  if (out == kUnsolved) return kUnsolved;
  const double v = OutValue<G>::value(out, p, g);
  return static_cast<int8_t>(v > 0.0 ? 1 : (v < 0.0 ? -1 : 0));
}

// Index (within the root's children) of BestChild(): std::max_element keeps
// the first maximum (mcts.cc:125-141; mcts.py:160-162 max() likewise).
template <class R>
OS_HD int best_child(const Node<R>* nodes, int child_player) {
  const Node<R>& root = nodes[0];
  if (root.nchild == 0) return -1;
  int best = 0;
  for (int k = 1; k < root.nchild; ++k)
    if (final_less(nodes[root.first + best], child_player, nodes[root.first + k],
                   child_player))
      best = k;
  return best;
}

// One random playout to the end (mcts.cc:46-55 / mcts.py:62-70).
template <class G, int Policy, class Rng, class Ctx>
OS_HD int rollout_ret0(typename G::State s, const GameCfg& g, Ctx& ctx, Rng& ev) {
  while (!G::terminal(s, g)) {
    const typename G::Legal l = G::legal(s, g, ctx);
    const uint32_t k = Policy == kPolicyCpp
                           ? AbslUniform(ev, static_cast<uint32_t>(l.count))
                           : NpChoice(ev, static_cast<uint32_t>(l.count));
    G::apply(s, g, ctx, l.kth(static_cast<int>(k)));
  }
  return G::ret0(s, g, ctx);
}

// Legal types that write LegalActions() into a buffer in one pass (go);
// OS_LEGAL_FILL=0 keeps one kth() per action (A/B knob, same actions).
#ifndef OS_LEGAL_FILL
#define OS_LEGAL_FILL 1
#endif
template <class L, class A, class = void>
struct HasFill : std::false_type {};
template <class L, class A>
struct HasFill<L, A, std::void_t<decltype(std::declval<const L&>().fill(std::declval<A&>()))>>
    : std::true_type {};

template <class R>
struct RewardOps;
template <>
struct RewardOps<int32_t> {
  OS_HD static int32_t from(int r0, int, int) { return r0; }
};

// Arena nodes to reserve for the GC traversal stack (u32 entries; the stack
// never holds more than depth x max_children entries).
OS_HD int64_t GcStackReserve(int max_children, int depth = kMaxPath) {
  return (static_cast<int64_t>(depth) * max_children * 4) / 16 + 64;
}

// GarbageCollect (mcts.cc:430-443): every node with children whose
// explore_count < limit loses them; nodes_ drops by the capacity of every
// such block, including blocks under an already-cleared ancestor (the
// reference recurses before clearing).  Traversal order does not change the
// result.  The DFS stack lives in the unused arena tail.
template <class R, bool W>
OS_HD int garbage_collect(Node<R, W>* nodes, uint32_t used, uint32_t cap, int limit,
                          int* nodes_count) {
  uint32_t* stack = reinterpret_cast<uint32_t*>(nodes + used);
  const uint64_t stack_cap =
      (static_cast<uint64_t>(cap - used) * sizeof(Node<R, W>)) / sizeof(uint32_t);
  uint64_t sp = 0;
  if (stack_cap < 1) return kGcStackOverflow;
  stack[sp++] = 0;
  while (sp > 0) {
    const uint32_t x = stack[--sp];
    Node<R, W>& nx = nodes[x];
    const int nc = nx.nchild;
    if (nc == 0) continue;
    if (sp + nc > stack_cap) return kGcStackOverflow;
    for (int k = 0; k < nc; ++k) stack[sp++] = nx.first + k;
    if (nx.n < limit) {
      *nodes_count -= nc;
      nx.nchild = 0;
    }
  }
  return kOk;
}

// One entry of the current simulation's visit path (mcts.cc visit_path).
// Selection records each visited node's statistics as it reads them while
// scanning the parent's children, so backup only stores (no dependent global
// loads), and entry 0 (the root) persists across simulations.
template <class R>
struct PathEnt {
  uint32_t idx;    // arena index
  uint32_t first;  // first child (valid iff nc > 0)
  int32_t n;       // explore_count before this simulation's backup
  int32_t nc;      // nchild
  R w;             // total_reward before this simulation's backup
};

// Element i of a batch-SoA array at p[i * stride]: the per-search buffers of
// the global-memory lane layout (k_lsearch), where the lanes of a wave hold
// the same index of their own searches in one contiguous line.
template <class T>
struct StridedPtr {
  T* p;
  int64_t stride;
  OS_HD T& operator[](int i) const { return p[static_cast<int64_t>(i) * stride]; }
};

// Page-pool descriptor of the paged arena (os_engine.hip AllocArena), u32
// words: pages taken by this launch, nodes per page, pages in the pool, first
// page handed out dynamically (the searches' own pages come first).
constexpr int kPgTaken = 0, kPgNodes = 1, kPgPool = 2, kPgFirstDynamic = 3;

// The next page of the pool for search `own_page` whose arena `nodes` starts
// at its own page: the child block goes to the start of that page, node
// indices stay relative to the search's first page.  false when the pool is
// exhausted (the batch is then rerun on the reserved arena).
OS_HD bool take_page(uint32_t* pg, uint32_t own_page, uint32_t* used, uint32_t* cap) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t np = atomicAdd(pg + kPgTaken, 1u) + pg[kPgFirstDynamic];
#else
  const uint32_t np = pg[kPgTaken]++ + pg[kPgFirstDynamic];
#endif
  if (np >= pg[kPgPool]) return false;
  *used = (np - own_page) * pg[kPgNodes];
  *cap = *used + pg[kPgNodes];
  return true;
}

// One complete search from `root`.  `bot` and `ev` are the two MT19937
// streams (the same object under kPolicyNumpy).  `actbuf` holds >=
// max_children entries, `path` >= path_cap >= MaxGameLength + 1 entries
// (pointers, or StridedPtr views of batch-SoA buffers).  `pages` (optional)
// is the page pool's descriptor: a child block that does not fit in `cap`
// then goes to the next free page (`own_page` = this search's first page).
template <class G, class R, int Policy, class Rng, class PathA, class ActA, class Ctx, bool W>
OS_HD SearchResult mcts_search(const GameCfg& g, const SearchParams& sp,
                               const typename G::State& root,
                               Ctx& ctx, Node<R, W>* nodes,
                               uint32_t cap, Rng& bot, Rng& ev, PathA path,
                               ActA actbuf, int path_cap, uint32_t* pages = nullptr,
                               uint32_t own_page = 0) {
  SearchResult res;
  res.status = kOk;
  res.sims = 0;
  res.gc_runs = 0;
  res.max_depth = 0;
  res.scanned = res.backed = res.expanded = res.solver_scanned = 0;
  const int P0 = G::to_move(root);
  nodes[0].first = 0;
  nodes[0].n = 0;
  nodes[0].w = 0;
  nodes[0].action = 0;
  nodes[0].nchild = 0;
  nodes[0].out = kUnsolved;
  path[0].idx = 0;
  path[0].first = 0;
  path[0].n = 0;
  path[0].nc = 0;
  path[0].w = 0;
  int8_t root_out = kUnsolved;
  uint32_t used = 1;
  int nodes_count = 1;
  int gc_limit = 5;
  const double inf = __builtin_huge_val();

  for (int sim = 0; sim < sp.max_simulations; ++sim) {
    typename G::State s = root;
    ctx.reset();
    // Current node, carried from the parent's child scan.
    uint32_t cur_idx = 0;
    uint32_t cur_first = path[0].first;
    int32_t cur_n = path[0].n;
    int cur_nc = path[0].nc;
    int depth = 0;
    // ---- selection / expansion (ApplyTreePolicy, mcts.cc:255-323) ----
    while (!G::terminal(s, g) && cur_n > 0) {
      int chosen;
      uint16_t c_action;
      uint32_t c_first;
      int32_t c_n;
      int c_nc;
      R c_w;
      if (cur_nc == 0) {
        const typename G::Legal l = G::legal(s, g, ctx);
        const int nc = l.count;
        if constexpr (OS_LEGAL_FILL && HasFill<typename G::Legal, ActA>::value)
          l.fill(actbuf);
        else
          for (int k = 0; k < nc; ++k) actbuf[k] = static_cast<uint16_t>(l.kth(k));
        if (Policy == kPolicyCpp) CppShuffle(actbuf, nc, bot);
        else NpShuffle(actbuf, nc, bot);
        if (used + static_cast<uint32_t>(nc) > cap &&
            !(pages && take_page(pages, own_page, &used, &cap))) {
          res.status = kArenaOverflow;
          goto done;
        }
        const uint32_t first = used;
        used += nc;
        for (int k = 0; k < nc; ++k) {
          Node<R, W>& c = nodes[first + k];
          c.first = 0;
          c.n = 0;
          c.w = 0;
          c.action = actbuf[k];
          c.nchild = 0;
          c.out = kUnsolved;
        }
        nodes[cur_idx].first = first;
        nodes[cur_idx].nchild = static_cast<decltype(nodes[0].nchild)>(nc);
        path[depth].first = first;
        path[depth].nc = nc;
        nodes_count += nc;
        res.expanded += nc;
        cur_first = first;
        cur_nc = nc;
        // Every fresh child is unvisited and unsolved (UCT +inf), so the
        // strict '>' scan of mcts.cc:310 picks the first one.
        chosen = 0;
        c_action = actbuf[0];
        c_first = 0;
        c_n = 0;
        c_nc = 0;
        c_w = 0;
      } else {
        const int cp = P0 ^ (depth & 1);  // player choosing at this node
        const double logN = sp.log_lut[cur_n];  // sqrt(N) under PUCT
        const double cprior = puct_prior_term(sp.uct_c, cur_nc);
        double best = -inf;
        chosen = 0;
        res.scanned += cur_nc;
        Node<R, W> bc = nodes[cur_first];
        bool screened = false;
#if defined(__HIP_DEVICE_COMPILE__) && OS_LANE_SCREEN
        // UCT with integer rewards: the argmax screened in f32 first, as the
        // wave kernels' uct_argmax_screen (os_wave.h; the same per-child value,
        // within E = (1 + |c| sqrt(log N)) 2^-20 of the f64 one,
        // tests/test_uct_screen.py), in one serial pass per lane.  The first
        // unvisited unsolved child is +inf in f64 and wins the strict '>' scan
        // outright, so the pass stops there.  Otherwise j, the first child
        // holding the f32 maximum m1, is the f64 argmax when every child of a
        // different (n, w, out) scores below m1 - 8E: m2 bounds those children
        // from above (a child of j's identity scores exactly j's value and
        // comes later, so j still wins; when the maximum moves to a new
        // identity the old maximum becomes m2, covering every child seen
        // before).  Any other case runs the exact f64 scan below.
        if constexpr (std::is_same<R, int32_t>::value) {
          if (!sp.puct) {
            const float lf = static_cast<float>(logN);
            const float cf = static_cast<float>(sp.uct_c);
            float m1 = -__builtin_huge_valf(), m2 = -__builtin_huge_valf();
            int j = -1, jinf = -1;
            int32_t jn = 0, jw = 0, jo = 0;
            auto screen = [&](const Node<R, W>& c, int k) {
              if (c.out == kUnsolved && c.n == 0) {
                jinf = k;
                return;
              }
              const float r = __builtin_amdgcn_rcpf(static_cast<float>(c.n));
              float a = static_cast<float>(c.w) * r + cf * __builtin_amdgcn_sqrtf(lf * r);
              const int32_t o = static_cast<int32_t>(c.out);
              a = o != kUnsolved ? static_cast<float>(cp == 0 ? o : -o) : a;
              if (j >= 0 && c.n == jn && c.w == jw && o == jo) return;
              if (a > m1) {
                m2 = m1;
                m1 = a;
                j = k;
                jn = c.n;
                jw = c.w;
                jo = o;
              } else {
                m2 = fmaxf(m2, a);
              }
            };
            int k = 0;
            for (; k + 4 <= cur_nc && jinf < 0; k += 4) {
              const Node<R, W> c0 = nodes[cur_first + k], c1 = nodes[cur_first + k + 1];
              const Node<R, W> c2 = nodes[cur_first + k + 2], c3 = nodes[cur_first + k + 3];
              screen(c0, k);
              if (jinf < 0) screen(c1, k + 1);
              if (jinf < 0) screen(c2, k + 2);
              if (jinf < 0) screen(c3, k + 3);
            }
            for (; k < cur_nc && jinf < 0; ++k) screen(nodes[cur_first + k], k);
            const float e2 = (1.0f + fabsf(cf) * __builtin_amdgcn_sqrtf(fmaxf(lf, 0.0f))) * 0x1p-17f;
            const int pick_k = jinf >= 0 ? jinf : (m2 < m1 - e2 ? j : -1);
            if (pick_k >= 0) {
              chosen = pick_k;
              bc = nodes[cur_first + pick_k];
              screened = true;
            }
          }
        }
#endif
        auto consider = [&](const Node<R, W>& c, int k) {
          double v;
          if (c.out != kUnsolved) {
            v = outcome_for(c.out, cp);
          } else if (sp.puct) {
            v = puct_unsolved(static_cast<double>(c.w), c.n, cprior, logN);
          } else if (c.n == 0) {
            v = inf;
          } else {
            const double dn = static_cast<double>(c.n);
            v = static_cast<double>(c.w) / dn + sp.uct_c * __builtin_sqrt(logN / dn);
          }
          if (v > best) {
            best = v;
            chosen = k;
            bc = c;
          }
        };
        // Four children loaded before any is scored: one memory latency per
        // four nodes on the lane layouts, the same first-maximum order.
        if (!screened) {
          int k = 0;
          for (; k + 4 <= cur_nc; k += 4) {
            const Node<R, W> c0 = nodes[cur_first + k], c1 = nodes[cur_first + k + 1];
            const Node<R, W> c2 = nodes[cur_first + k + 2], c3 = nodes[cur_first + k + 3];
            consider(c0, k);
            consider(c1, k + 1);
            consider(c2, k + 2);
            consider(c3, k + 3);
          }
          for (; k < cur_nc; ++k) consider(nodes[cur_first + k], k);
        }
        c_action = bc.action;
        c_first = bc.first;
        c_n = bc.n;
        c_nc = bc.nchild;
        c_w = bc.w;
      }
      G::apply(s, g, ctx, c_action);
      if (++depth >= path_cap) {
        res.status = kPathOverflow;
        goto done;
      }
      cur_idx = cur_first + chosen;
      cur_first = c_first;
      cur_n = c_n;
      cur_nc = c_nc;
      PathEnt<R>& pe = path[depth];
      pe.idx = cur_idx;
      pe.first = c_first;
      pe.n = c_n;
      pe.nc = c_nc;
      pe.w = c_w;
    }
    if (depth > res.max_depth) res.max_depth = depth;
    // ---- evaluation ----
    {
      bool solved;
      R rv0, rv1;
      if (G::terminal(s, g)) {
        const int r0 = G::ret0(s, g, ctx);
        nodes[cur_idx].out = static_cast<int8_t>(r0);
        if (depth == 0) root_out = static_cast<int8_t>(r0);
        solved = sp.solve != 0;
        rv0 = static_cast<R>(r0);
        rv1 = static_cast<R>(-r0);
      } else {
        solved = false;
        if (sp.n_rollouts == 1) {
#if OS_AB_LANE_NOROLL  // timing A/B only (not the reference's results): no playout
          const int r0 = 0;
#else
          const int r0 = rollout_ret0<G, Policy>(s, g, ctx, ev);
#endif
          rv0 = static_cast<R>(r0);
          rv1 = static_cast<R>(-r0);
        } else {
          // Every rollout starts from a clone of the leaf (mcts.cc:46-47), so
          // go's position log is rewound to the leaf before each one.
          const int leaf_mark = ctx.mark();
          double s0 = 0.0, s1 = 0.0;
          for (int k = 0; k < sp.n_rollouts; ++k) {
            if (k) ctx.rewind(leaf_mark);
            const int r0 = rollout_ret0<G, Policy>(s, g, ctx, ev);
            s0 += static_cast<double>(r0);
            s1 += static_cast<double>(-r0);
          }
          rv0 = static_cast<R>(s0 / sp.n_rollouts);
          rv1 = static_cast<R>(s1 / sp.n_rollouts);
        }
      }
      // ---- backup + MCTS-Solver (mcts.cc:351-396) ----
      for (int d = depth; d >= 0; --d) {
        PathEnt<R>& pe = path[d];
        const int pl = d == 0 ? P0 : (P0 ^ ((d - 1) & 1));
        pe.w += pl == 0 ? rv0 : rv1;
        pe.n += 1;
        Node<R, W>& nd = nodes[pe.idx];
        nd.n = pe.n;
        nd.w = pe.w;
        res.backed += 1;
        if (solved && pe.nc > 0) {
          const int cpl = P0 ^ (d & 1);
          res.solver_scanned += pe.nc;
          int best = -1;
          int8_t best_out = kUnsolved;
          double bestv = 0.0;
          bool all_solved = true;
          for (int k = 0; k < pe.nc; ++k) {
            const int8_t co = nodes[pe.first + k].out;
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
          if (best >= 0 && (all_solved || bestv == 1.0)) {
            nd.out = best_out;
            if (d == 0) root_out = best_out;
          } else {
            solved = false;
          }
        }
      }
    }
    res.sims = sim + 1;
    if (root_out != kUnsolved) break;
    if (Policy == kPolicyCpp) {
      if (path[0].nc == 1) break;
      if (sp.max_nodes > 1 && nodes_count >= sp.max_nodes) {
        const int st = garbage_collect(nodes, used, cap, gc_limit, &nodes_count);
        if (st != kOk) {
          res.status = st;
          goto done;
        }
        res.gc_runs++;
        gc_limit = static_cast<int>(gc_limit *
                                    (nodes_count > sp.max_nodes / 2 ? 1.25 : 0.9));
        if (gc_limit < 5) gc_limit = 5;
        path[0].nc = nodes[0].nchild;  // the root may have lost its children
        path[0].first = nodes[0].first;
      }
    }
  }
done:
  res.nodes = nodes_count;
  // Nodes allocated (== the last used slot on the reserved arena; on the
  // paged arena `used` is an index into a later page).
  res.used = pages ? 1 + res.expanded : used;
  return res;
}


}  // namespace osm

#endif  // OS_MCTS_H_
