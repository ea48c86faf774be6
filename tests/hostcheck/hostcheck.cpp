// TEST INFRASTRUCTURE ONLY — the product's search engine (csrc/os_mcts.h) and
// game state machines compiled for the host CPU with g++, so the CPU test
// suite can check the exact engine logic the gfx950 kernel runs against the
// oracle without a GPU.  Never shipped, never used by bench.py or the C-ABI.
#include <algorithm>
#include <cmath>
#include <memory>
#include <cstring>
#include <string>
#include <vector>

#include "os_host.h"
#include "os_az.h"
#include "os_chance.h"
#include "os_mcts.h"

// 1: searches keep the go superko log's open group in a side buffer as
// k_lsearch does (hc_set_log_wc).
static int g_log_wc = 0;

using namespace osm;

namespace {
thread_local std::string g_err;

template <class G, class R, int Policy>
int RunOne(const HostGame& game, const HostState& root, const SearchParams& sp,
           uint32_t bot_seed, uint32_t eval_seed, uint32_t cap, int32_t max_children,
           int32_t* child_action, int32_t* child_n, double* child_w,
           int8_t* child_out, int32_t* nchild, int32_t* root_n, double* root_w,
           int8_t* root_out, int64_t* best_action, int32_t* nodes_out) {
  std::vector<Node<R>> nodes(cap);
  std::vector<uint32_t> mt(2 * kMtN);
  MtStream bot{mt.data(), kMtN, 0}, ev{mt.data() + kMtN, kMtN, 0};
  mt_seed(bot.s, bot_seed);
  mt_seed(ev.s, eval_seed);
  PathEnt<R> path[kMaxPath];
  uint16_t actbuf[kMaxChildren];
  typename G::Ctx ctx;
  HostGoLog logbuf;
  uint64_t wlog[8];
  uint32_t wlink[8];
  if constexpr (G::State::kNeedsLog) {
    std::memset(static_cast<void*>(&ctx), 0, sizeof ctx);
    ctx.zob = game.zob.data();
    ctx.base = root.hashes.data();
    ctx.n_base = static_cast<int32_t>(root.hashes.size());
    logbuf.bind(&ctx, 248, game.cfg.rows * game.cfg.cols);
    ctx.init_filters();
    if (g_log_wc) {  // k_lsearch's write-combined log (GoCtxT::wlog)
      ctx.wlog = wlog;
      ctx.wlink = wlink;
      ctx.wst = 1;
    }
  }
  const typename G::State& rs = *reinterpret_cast<const typename G::State*>(root.raw);
  SearchResult res;
  if constexpr (HasChance<G>::value)
    res = mcts_search_chance<G, R, Policy>(game.cfg, sp, rs, ctx, nodes.data(), cap, bot, ev,
                                           path, actbuf, kChancePathCap);
  else
    res = mcts_search<G, R, Policy>(game.cfg, sp, rs, ctx, nodes.data(), cap, bot, ev, path,
                                    actbuf, kMaxPath);
  if (res.status != kOk) {
    g_err = "search status " + std::to_string(res.status);
    return -4;
  }
  const int P0 = G::to_move(rs);
  const Node<R>& rn = nodes[0];
  *nchild = rn.nchild;
  for (int k = 0; k < rn.nchild && k < max_children; ++k) {
    const Node<R>& c = nodes[rn.first + k];
    child_action[k] = c.action;
    child_n[k] = c.n;
    child_w[k] = static_cast<double>(c.w);
    child_out[k] = out_sign<G>(c.out, P0, game.cfg);
  }
  *root_n = rn.n;
  *root_w = static_cast<double>(rn.w);
  *root_out = out_sign<G>(rn.out, P0, game.cfg);
  const int b = best_child_g<G>(nodes.data(), P0, game.cfg);
  *best_action = b < 0 ? -1 : nodes[rn.first + b].action;
  *nodes_out = res.nodes;
  return 0;
}

template <class G>
int Dispatch(const HostGame& game, const HostState& root, const SearchParams& sp,
             int policy, uint32_t bs, uint32_t es, uint32_t cap, int32_t mc, int32_t* ca,
             int32_t* cn, double* cw, int8_t* co, int32_t* nch, int32_t* rn,
             double* rw, int8_t* ro, int64_t* ba, int32_t* nd) {
  if (sp.n_rollouts == 1 && game.cfg.pig_players <= 2) {  // else f64 node rewards
    if (policy == kPolicyCpp)
      return RunOne<G, int32_t, kPolicyCpp>(game, root, sp, bs, es, cap, mc, ca, cn, cw,
                                            co, nch, rn, rw, ro, ba, nd);
    return RunOne<G, int32_t, kPolicyNumpy>(game, root, sp, bs, es, cap, mc, ca, cn, cw,
                                            co, nch, rn, rw, ro, ba, nd);
  }
  if (policy == kPolicyCpp)
    return RunOne<G, double, kPolicyCpp>(game, root, sp, bs, es, cap, mc, ca, cn, cw, co,
                                         nch, rn, rw, ro, ba, nd);
  return RunOne<G, double, kPolicyNumpy>(game, root, sp, bs, es, cap, mc, ca, cn, cw, co,
                                         nch, rn, rw, ro, ba, nd);
}
}  // namespace

extern "C" {

const char* hc_last_error() { return g_err.c_str(); }

// Same output layout as oref_mcts_batch.
int hc_mcts_batch(const char* game_string, int64_t num_roots,
                  const int64_t* root_actions, const int64_t* root_offsets,
                  double uct_c, int32_t max_simulations, int32_t n_rollouts,
                  int64_t max_memory_mb, int32_t solve, int32_t policy,
                  const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                  int32_t max_children, int32_t* child_action, int32_t* child_n,
                  double* child_w, int8_t* child_out, int32_t* nchild,
                  int32_t* root_n, double* root_w, int8_t* root_out,
                  int64_t* best_action, int32_t* nodes) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty()) {
    g_err = err;
    return -1;
  }
  // policy bit 8: PUCT child selection (the LUT then holds sqrt(N)).
  const bool puct = (policy >> 8) & 1;
  policy &= 0xff;
  std::vector<double> lut(max_simulations + 2);
  for (size_t i = 0; i < lut.size(); ++i)
    lut[i] = puct ? std::sqrt(static_cast<double>(i)) : std::log(static_cast<double>(i));
  SearchParams sp;
  std::memset(&sp, 0, sizeof sp);
  sp.uct_c = uct_c;
  sp.max_simulations = max_simulations;
  sp.n_rollouts = n_rollouts;
  sp.solve = solve;
  sp.max_nodes = static_cast<int32_t>((max_memory_mb << 20) / 80 + 1);
  sp.policy = policy;
  sp.puct = puct ? 1 : 0;
  sp.log_lut = lut.data();
  const uint32_t cap = 1 + static_cast<uint32_t>(max_simulations) * game.cfg.max_children +
                       static_cast<uint32_t>(GcStackReserve(game.cfg.max_children));
  for (int64_t r = 0; r < num_roots; ++r) {
    HostState hs;
    hs.game = &game;
    StateInit(&hs);
    for (int64_t i = root_offsets[r]; i < root_offsets[r + 1]; ++i) {
      if (!StateApply(&hs, root_actions[i])) {
        g_err = "illegal root action";
        return -1;
      }
    }
    const int64_t o = r * max_children;
    int rc = 0;
    const uint32_t es = eval_seeds[r], bs = bot_seeds[r];
    switch (game.cfg.kind) {
#define HC_CASE(K, G)                                                              \
  case K:                                                                          \
    rc = Dispatch<G>(game, hs, sp, policy, bs, es, cap, max_children,              \
                     child_action + o, child_n + o, child_w + o, child_out + o,    \
                     nchild + r, root_n + r, root_w + r, root_out + r,             \
                     best_action + r, nodes + r);                                  \
    break;
      HC_CASE(kTicTacToe, TicTacToe)
      HC_CASE(kConnectFour, ConnectFour)
      HC_CASE(kBreakthrough, Breakthrough)
      HC_CASE(kHex, Hex)
      HC_CASE(kGo, Go)
      HC_CASE(kPig, Pig)
#undef HC_CASE
    }
    if (rc) return rc;
  }
  return 0;
}

// External-evaluator search (csrc/os_az.h) stepped on the host: every request
// goes to `cb(obs, obs_size, legal, A, kind, prior_out, value_out)`.  Same
// output layout as hc_mcts_batch.
typedef int (*hc_az_cb)(const float* obs, int32_t obs_size, const uint8_t* legal,
                        int32_t num_actions, int32_t kind, double* prior, double* value);
}  // extern "C"

namespace {
template <class G>
int AzRunOne(const HostGame& game, const HostState& root, const SearchParams& sp, int puct,
             uint32_t seed, double alpha, double eps, uint32_t cap, hc_az_cb cb, int32_t mc,
             int32_t* ca, int32_t* cn, double* cw, int8_t* co, int32_t* nch, int32_t* rn,
             double* rw, int8_t* ro, int64_t* ba, int32_t* nd) {
  const int A = game.cfg.num_actions;
  const int obs_size = ObservationShape(game, nullptr);
  std::vector<Node<double>> nodes(cap);
  std::vector<double> prior(cap);
  std::vector<double> raw((puct & 2) ? cap : 0);  // fused requests
  std::vector<uint32_t> mt(kMtN);
  mt_seed(mt.data(), seed);
  MtStream bot{mt.data(), kMtN, 0, 0};
  std::vector<float> obs(obs_size);
  std::vector<uint8_t> legal(A);
  std::vector<double> pri(A);
  double value = 0;
  int32_t kind = 0;
  AzIo io{&kind, obs.data(), legal.data(), pri.data(), &value};
  auto sl = std::make_unique<AzSlot<G>>();
  std::memset(sl.get(), 0, sizeof(AzSlot<G>));
  const typename G::State& rs = *reinterpret_cast<const typename G::State*>(root.raw);
  sl->s = rs;
  typename G::Ctx ctx;
  if constexpr (G::State::kNeedsLog) {
    std::memset(static_cast<void*>(&ctx), 0, sizeof ctx);
    ctx.zob = game.zob.data();
    ctx.base = root.hashes.data();
    ctx.n_base = static_cast<int32_t>(root.hashes.size());
    ctx.n_heads = game.cfg.rows * game.cfg.cols + 1;
  }
  std::vector<double> noise(game.cfg.max_children, 0.0);
  AzNoise nz{nullptr, 0, eps};
  if (alpha > 0) {
    std::vector<int64_t> acts;
    StateLegal(root, &acts);
    nz.skip = static_cast<int32_t>(
        DirichletNoise(seed, static_cast<int>(acts.size()), alpha, noise.data()));
    nz.noise = noise.data();
  }
  for (;;) {
    az_step<G>(game.cfg, sp, puct & 1, rs, *sl, nodes.data(), prior.data(),
               raw.empty() ? nullptr : raw.data(), cap, bot, io, obs_size, A, ctx, nz);
    if (kind == kAzNone) break;
    std::fill(pri.begin(), pri.end(), 0.0);
    cb(obs.data(), obs_size, legal.data(), A, kind, pri.data(), &value);
  }
  if (sl->res.status != kOk) {
    g_err = "search status " + std::to_string(sl->res.status);
    return -4;
  }
  const int P0 = G::to_move(rs);
  const Node<double>& r0 = nodes[0];
  *nch = r0.nchild;
  for (int k = 0; k < r0.nchild && k < mc; ++k) {
    const Node<double>& c = nodes[r0.first + k];
    ca[k] = c.action;
    cn[k] = c.n;
    cw[k] = c.w;
    co[k] = c.out == kUnsolved ? kUnsolved : (P0 == 0 ? c.out : -c.out);
  }
  *rn = r0.n;
  *rw = r0.w;
  *ro = r0.out == kUnsolved ? kUnsolved : (P0 == 0 ? r0.out : -r0.out);
  const int b = best_child(nodes.data(), P0);
  *ba = b < 0 ? -1 : nodes[r0.first + b].action;
  *nd = sl->res.nodes;
  return 0;
}
// One python/algorithms/mcts.py search (numpy policy) with an external
// evaluator, az_step on the host: the bot's RandomState continues from
// (key, pos) and is written back; `noise` (or null) is the caller's
// RandomState.dirichlet draw for the root's legal actions.
template <class G>
int AzRunNumpy(const HostGame& game, const HostState& root, const SearchParams& sp, int puct,
               uint32_t* key, int32_t* pos, const double* noise, double eps, hc_az_cb cb,
               int mc, int32_t* ca, int32_t* cn, double* cw, double* cp, int8_t* co,
               int32_t* nch, int32_t* rn, double* rw, int64_t* ba) {
  const int A = game.cfg.num_actions;
  const int obs_size = ObservationShape(game, nullptr);
  const uint32_t cap = 1 + static_cast<uint32_t>(sp.max_simulations) * game.cfg.max_children;
  std::vector<Node<double>> nodes(cap);
  std::vector<double> prior(cap);
  MtStream bot{key, *pos, 1, 0};
  std::vector<float> obs(obs_size);
  std::vector<uint8_t> legal(A);
  std::vector<double> pri(A);
  double value = 0;
  int32_t kind = 0;
  AzIo io{&kind, obs.data(), legal.data(), pri.data(), &value};
  auto sl = std::make_unique<AzSlot<G>>();
  std::memset(sl.get(), 0, sizeof(AzSlot<G>));
  const typename G::State& rs = *reinterpret_cast<const typename G::State*>(root.raw);
  sl->s = rs;
  typename G::Ctx ctx;
  if constexpr (G::State::kNeedsLog) {
    std::memset(static_cast<void*>(&ctx), 0, sizeof ctx);
    ctx.zob = game.zob.data();
    ctx.base = root.hashes.data();
    ctx.n_base = static_cast<int32_t>(root.hashes.size());
    ctx.n_heads = game.cfg.rows * game.cfg.cols + 1;
  }
  AzNoise nz{noise, 0, eps};
  for (;;) {
    az_step<G>(game.cfg, sp, puct, rs, *sl, nodes.data(), prior.data(), nullptr, cap, bot, io,
               obs_size, A, ctx, nz, /*np_policy=*/true);
    if (kind == kAzNone) break;
    std::fill(pri.begin(), pri.end(), 0.0);
    cb(obs.data(), obs_size, legal.data(), A, kind, pri.data(), &value);
  }
  if (sl->res.status != kOk) {
    g_err = "search status " + std::to_string(sl->res.status);
    return -4;
  }
  *pos = bot.idx >= kMtN ? kMtN : bot.idx;  // numpy (key, pos): the block is fully twisted
  if (!bot.pre && bot.idx < kMtN) {
    // a block being twisted in place: finish it (numpy keeps whole blocks)
    for (int i = bot.idx; i < kMtN; ++i) {
      const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
      const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
      const uint32_t y = (key[i] & 0x80000000u) | (key[i1] & 0x7fffffffu);
      key[i] = key[im] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
  }
  const int P0 = G::to_move(rs);
  const Node<double>& r0 = nodes[0];
  *nch = r0.nchild;
  for (int k = 0; k < r0.nchild && k < mc; ++k) {
    const Node<double>& c = nodes[r0.first + k];
    ca[k] = c.action;
    cn[k] = c.n;
    cw[k] = c.w;
    cp[k] = prior[r0.first + k];
    co[k] = c.out == kUnsolved ? kUnsolved : (P0 == 0 ? c.out : -c.out);
  }
  *rn = r0.n;
  *rw = r0.w;
  const int b = best_child(nodes.data(), P0);
  *ba = b < 0 ? -1 : nodes[r0.first + b].action;
  return 0;
}
}  // namespace

extern "C" {

int hc_az_numpy(const char* game_string, const int64_t* history, int64_t n_history,
                double uct_c, int32_t max_simulations, int32_t solve, int32_t puct,
                uint32_t* key, int32_t* pos, const double* noise, double eps, hc_az_cb cb,
                int32_t max_children, int32_t* child_action, int32_t* child_n, double* child_w,
                double* child_prior, int8_t* child_out, int32_t* nchild, int32_t* root_n,
                double* root_w, int64_t* best_action) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty()) {
    g_err = err;
    return -1;
  }
  std::vector<double> lut(max_simulations + 2);
  for (size_t i = 0; i < lut.size(); ++i) lut[i] = std::log(static_cast<double>(i));
  SearchParams sp;
  std::memset(&sp, 0, sizeof sp);
  sp.uct_c = uct_c;
  sp.max_simulations = max_simulations;
  sp.n_rollouts = 1;
  sp.solve = solve;
  sp.max_nodes = 1;  // mcts.py never garbage-collects
  sp.policy = kPolicyNumpy;
  sp.log_lut = lut.data();
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n_history; ++i) StateApply(&hs, history[i]);
  int rc = 0;
#define HC_AZN(G)                                                                            \
  rc = AzRunNumpy<G>(game, hs, sp, puct, key, pos, noise, eps, cb, max_children, child_action, \
                     child_n, child_w, child_prior, child_out, nchild, root_n, root_w,          \
                     best_action)
  switch (game.cfg.kind) {
    case kTicTacToe: HC_AZN(TicTacToe); break;
    case kConnectFour: HC_AZN(ConnectFour); break;
    case kBreakthrough: HC_AZN(Breakthrough); break;
    case kHex: HC_AZN(Hex); break;
    case kGo: HC_AZN(Go); break;
    default: g_err = "unsupported"; return -2;
  }
#undef HC_AZN
  return rc;
}

int hc_az_batch(const char* game_string, int64_t num_roots, const int64_t* root_actions,
                const int64_t* root_offsets, double uct_c, int32_t max_simulations,
                int64_t max_memory_mb, int32_t solve, int32_t puct, double alpha, double eps,
                const uint32_t* bot_seeds, hc_az_cb cb, int32_t max_children,
                int32_t* child_action, int32_t* child_n, double* child_w, int8_t* child_out,
                int32_t* nchild, int32_t* root_n, double* root_w, int8_t* root_out,
                int64_t* best_action, int32_t* nodes) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty()) {
    g_err = err;
    return -1;
  }
  std::vector<double> lut(max_simulations + 2);
  for (size_t i = 0; i < lut.size(); ++i) lut[i] = std::log(static_cast<double>(i));
  SearchParams sp;
  std::memset(&sp, 0, sizeof sp);
  sp.uct_c = uct_c;
  sp.max_simulations = max_simulations;
  sp.n_rollouts = 1;
  sp.solve = solve;
  sp.max_nodes = static_cast<int32_t>((max_memory_mb << 20) / 80 + 1);
  sp.policy = kPolicyCpp;
  sp.log_lut = lut.data();
  const uint32_t cap = 1 + static_cast<uint32_t>(max_simulations) * game.cfg.max_children +
                       static_cast<uint32_t>(GcStackReserve(game.cfg.max_children));
  for (int64_t r = 0; r < num_roots; ++r) {
    HostState hs;
    hs.game = &game;
    StateInit(&hs);
    for (int64_t i = root_offsets[r]; i < root_offsets[r + 1]; ++i) StateApply(&hs, root_actions[i]);
    const int64_t o = r * max_children;
    int rc = 0;
#define HC_AZ(G)                                                                          \
  rc = AzRunOne<G>(game, hs, sp, puct, bot_seeds[r], alpha, eps, cap, cb, max_children,  \
                   child_action + o, child_n + o, child_w + o, child_out + o, nchild + r, \
                   root_n + r, root_w + r, root_out + r, best_action + r, nodes + r)
    switch (game.cfg.kind) {
      case kTicTacToe: HC_AZ(TicTacToe); break;
      case kConnectFour: HC_AZ(ConnectFour); break;
      case kBreakthrough: HC_AZ(Breakthrough); break;
      case kHex: HC_AZ(Hex); break;
      case kGo: HC_AZ(Go); break;
      default: g_err = "unsupported"; return -2;
    }
#undef HC_AZ
    if (rc) return rc;
  }
  return 0;
}

// The product's host-drawn Dirichlet noise (os_host.cpp), for known answers.
int64_t hc_dirichlet_noise(uint32_t seed, int32_t count, double alpha, double* out) {
  return DirichletNoise(seed, count, alpha, out);
}

// Product RNG primitives (csrc/os_rng.h) on the host, for known-answer tests.
void hc_mt_words(uint32_t seed, int64_t n, uint32_t* out) {
  std::vector<uint32_t> s(kMtN);
  mt_seed(s.data(), seed);
  MtStream g{s.data(), kMtN, 0, 0};
  for (int64_t i = 0; i < n; ++i) out[i] = g.next();
}
// k_rollouts' SoA stream (seeded words by cursors, never stored), interleaved
// with `stride` - 1 other streams' words.
void hc_mt_words_soa(uint32_t seed, int64_t stride, int64_t n, uint32_t* out) {
  std::vector<uint32_t> s(kMtN * stride, 0xdeadbeefu);
  MtStreamSoA g{s.data() + stride - 1, stride, 0, 0};
  g.seed(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = g.next();
}
// k_lsearch's read-ahead SoA stream (MtStreamPf), same interleaving.
void hc_mt_words_pf(uint32_t seed, int64_t stride, int64_t n, uint32_t* out) {
  std::vector<uint32_t> s(kMtN * stride, 0xdeadbeefu);
  MtStreamPf g{s.data() + stride - 1, stride, 0, 0};
  g.seed(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = g.next();
}
// MtStreamPf continuing a numpy (key, pos) state for k draws, exported back.
void hc_mt_pf_roundtrip(uint32_t* key, int32_t* pos, int64_t k, uint32_t* out) {
  MtStreamPf g{key, 1, 0, 0};
  g.init_import(*pos);
  for (int64_t i = 0; i < k; ++i) out[i] = g.next();
  *pos = g.finalize();
}
void hc_set_log_wc(int on) { g_log_wc = on; }
// k_lsearch's write-combined stream (MtStreamWc: 16-word groups), same
// interleaving.
void hc_mt_words_wc(uint32_t seed, int64_t stride, int64_t n, uint32_t* out) {
  std::vector<uint32_t> s(kMtN * stride, 0xdeadbeefu);
  uint32_t wb[16];
  MtStreamWc g{{s.data() + stride - 1, stride, 0, 0}, wb, 1};
  g.seed(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = g.next();
}
// MtStreamWc continuing a numpy (key, pos) state for k draws, exported back.
void hc_mt_wc_roundtrip(uint32_t* key, int32_t* pos, int64_t k, uint32_t* out) {
  uint32_t wb[16];
  MtStreamWc g{{key, 1, 0, 0}, wb, 1};
  g.init_import(*pos);
  for (int64_t i = 0; i < k; ++i) out[i] = g.next();
  *pos = g.finalize();
}
// k_rollouts' register-only first block (MtStreamReg), same interleaving.
void hc_mt_words_reg(uint32_t seed, int64_t stride, int64_t n, uint32_t* out) {
  std::vector<uint32_t> s(kMtN * stride, 0xdeadbeefu);
  MtStreamReg g{s.data() + stride - 1, stride, 0, 0};
  g.seed(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = g.next();
}
void hc_absl_uniform(uint32_t seed, uint32_t n, int64_t k, uint64_t* out) {
  std::vector<uint32_t> s(kMtN);
  mt_seed(s.data(), seed);
  MtStream g{s.data(), kMtN, 0, 0};
  for (int64_t i = 0; i < k; ++i) out[i] = AbslUniform(g, n);
}
// absl::Uniform(rng, 0.0, 1.0) draws (os_rng.h AbslUniformDouble01).
void hc_absl_double(uint32_t seed, int64_t k, double* out) {
  std::vector<uint32_t> s(kMtN);
  mt_seed(s.data(), seed);
  MtStream g{s.data(), kMtN, 0, 0};
  for (int64_t i = 0; i < k; ++i) out[i] = AbslUniformDouble01(g);
}
// numpy RandomState(seed).choice(n, p=[p] * n) indices (NpChoiceEquiprobable).
void hc_np_choice_p(uint32_t seed, int32_t n, int64_t k, int32_t* out) {
  std::vector<uint32_t> s(kMtN);
  mt_seed(s.data(), seed);
  MtStream g{s.data(), kMtN, 0, 0};
  for (int64_t i = 0; i < k; ++i) out[i] = NpChoiceEquiprobable(g, n, 1.0 / n);
}
void hc_cpp_shuffle(uint32_t seed, int32_t n, int32_t* out) {
  std::vector<uint32_t> s(kMtN);
  mt_seed(s.data(), seed);
  MtStream g{s.data(), kMtN, 0, 0};
  std::vector<int32_t> a(n);
  for (int i = 0; i < n; ++i) a[i] = i;
  CppShuffle(a.data(), n, g);
  for (int i = 0; i < n; ++i) out[i] = a[i];
}
// numpy RandomState(seed): k choice(range(n)) draws then one shuffle of n.
void hc_np_ops(uint32_t seed, uint32_t n, int64_t k, uint32_t* choices,
               int32_t* perm, uint32_t* next_word) {
  std::vector<uint32_t> s(kMtN);
  mt_seed(s.data(), seed);
  MtStream g{s.data(), kMtN, 0, 0};
  for (int64_t i = 0; i < k; ++i) choices[i] = NpChoice(g, n);
  std::vector<int32_t> a(n);
  for (uint32_t i = 0; i < n; ++i) a[i] = static_cast<int32_t>(i);
  NpShuffle(a.data(), static_cast<int>(n), g);
  for (uint32_t i = 0; i < n; ++i) perm[i] = a[i];
  *next_word = g.next();
}
// Import a numpy (key, pos) state, draw k words, export back (finalize).
void hc_mt_roundtrip(uint32_t* key, int32_t* pos, int64_t k, uint32_t* out) {
  MtStream g{key, *pos, 1, 0};
  for (int64_t i = 0; i < k; ++i) out[i] = g.next();
  g.finalize();
  *pos = g.idx;
}

// Product go score (os_games.h Go::score) of the position after `actions`.
float hc_go_score(const char* game_string, const int64_t* actions, int64_t n) {
  HostGame game;
  bool unsup = false;
  if (!LoadHostGame(game_string, &game, &unsup).empty()) return -1e30f;
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n; ++i) StateApply(&hs, actions[i]);
  return Go::score(*reinterpret_cast<const Go::State*>(hs.raw), game.cfg);
}

// Product rollouts on the host: RandomRolloutEvaluator::Evaluate per seed.
int hc_rollouts(const char* game_string, const int64_t* actions, int64_t n_actions,
                int64_t n, const uint32_t* seeds, double* out) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty()) {
    g_err = err;
    return -1;
  }
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n_actions; ++i) StateApply(&hs, actions[i]);
  std::vector<uint32_t> mt(kMtN);
  HostGoLog logbuf;
  for (int64_t i = 0; i < n; ++i) {
    MtStream ev{mt.data(), kMtN, 0};
    mt_seed(ev.s, seeds[i]);
    int r0 = 0;
    switch (game.cfg.kind) {
      case kTicTacToe: { NoCtx c; r0 = rollout_ret0<TicTacToe, kPolicyCpp>(*reinterpret_cast<TicTacToe::State*>(hs.raw), game.cfg, c, ev); break; }
      case kConnectFour: { NoCtx c; r0 = rollout_ret0<ConnectFour, kPolicyCpp>(*reinterpret_cast<ConnectFour::State*>(hs.raw), game.cfg, c, ev); break; }
      case kBreakthrough: { NoCtx c; r0 = rollout_ret0<Breakthrough, kPolicyCpp>(*reinterpret_cast<Breakthrough::State*>(hs.raw), game.cfg, c, ev); break; }
      case kHex: { NoCtx c; r0 = rollout_ret0<Hex, kPolicyCpp>(*reinterpret_cast<Hex::State*>(hs.raw), game.cfg, c, ev); break; }
      case kPig: { NoCtx c; r0 = rollout_ret0_chance<Pig, kPolicyCpp>(*reinterpret_cast<Pig::State*>(hs.raw), game.cfg, c, ev); break; }
      case kGo: {
        GoCtx c;
        std::memset(static_cast<void*>(&c), 0, sizeof c);
        c.zob = game.zob.data();
        c.base = hs.hashes.data();
        c.n_base = static_cast<int32_t>(hs.hashes.size());
        logbuf.bind(&c, 248, game.cfg.rows * game.cfg.cols);
        c.init_filters();
        r0 = rollout_ret0<Go, kPolicyCpp>(*reinterpret_cast<Go::State*>(hs.raw), game.cfg, c, ev);
        break;
      }
    }
    out[2 * i] = r0;
    out[2 * i + 1] = -r0;
  }
  return 0;
}

// The same go playouts with the k_rollouts superko screen (GoCtxBloom).
// go playouts with the bucketed superko log behind its Bloom filter
// (GoCtxT::bloom, as k_rollouts / k_lsearch run it).
int hc_rollouts_go_logbloom(const char* game_string, const int64_t* actions, int64_t n_actions,
                            int64_t n, const uint32_t* seeds, double* out) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty() || game.cfg.kind != kGo) {
    g_err = err.empty() ? "go only" : err;
    return -1;
  }
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n_actions; ++i) StateApply(&hs, actions[i]);
  std::vector<uint32_t> mt(kMtN);
  HostGoLog logbuf;
  std::vector<uint32_t> bloom(GoCtx::kBloomWords * 64);
  for (int64_t i = 0; i < n; ++i) {
    MtStream ev{mt.data(), kMtN, 0};
    mt_seed(ev.s, seeds[i]);
    GoCtx c;
    std::memset(static_cast<void*>(&c), 0, sizeof c);
    c.zob = game.zob.data();
    c.base = hs.hashes.data();
    c.n_base = static_cast<int32_t>(hs.hashes.size());
    logbuf.bind(&c, 248, game.cfg.rows * game.cfg.cols);
    c.bloom = bloom.data();
    c.init_filters();
    const int r0 = rollout_ret0<Go, kPolicyCpp>(*reinterpret_cast<Go::State*>(hs.raw), game.cfg,
                                                c, ev);
    out[2 * i] = r0;
    out[2 * i + 1] = -r0;
  }
  return 0;
}

// k_rollouts' go context: the bucketed log with 16-bit links (never rewound)
// behind the Bloom filter (os_kernels.h RollCtx<Go>).
int hc_rollouts_go_link16(const char* game_string, const int64_t* actions, int64_t n_actions,
                          int64_t n, const uint32_t* seeds, double* out) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty() || game.cfg.kind != kGo) {
    g_err = err.empty() ? "go only" : err;
    return -1;
  }
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n_actions; ++i) StateApply(&hs, actions[i]);
  using Ctx16 = GoCtxT<uint8_t, uint16_t>;
  const int cap = 248, cells = game.cfg.rows * game.cfg.cols;
  std::vector<uint32_t> mt(kMtN);
  std::vector<uint64_t> log(cap);
  std::vector<uint16_t> link(cap);
  std::vector<uint8_t> head(cells + 1);
  std::vector<uint32_t> bloom(Ctx16::kBloomWords * 64);
  for (int64_t i = 0; i < n; ++i) {
    MtStream ev{mt.data(), kMtN, 0};
    mt_seed(ev.s, seeds[i]);
    Ctx16 c;
    std::memset(static_cast<void*>(&c), 0, sizeof c);
    c.zob = game.zob.data();
    c.base = hs.hashes.data();
    c.n_base = static_cast<int32_t>(hs.hashes.size());
    c.log = log.data();
    c.link = link.data();
    c.head = head.data();
    c.stride = 1;
    c.head_stride = 1;
    c.cap = cap;
    c.n_heads = cells + 1;
    c.bloom = bloom.data();
    c.init_filters();
    const int r0 = rollout_ret0<Go, kPolicyCpp>(*reinterpret_cast<Go::State*>(hs.raw), game.cfg,
                                                c, ev);
    out[2 * i] = r0;
    out[2 * i + 1] = -r0;
  }
  return 0;
}

// B96 (three u32 words, os_common.h) against B128 on random boards of up to
// 96 cells: every operation GoT uses, with shifts 1..31 and both word-choice
// forms.  Returns the number of mismatching results.
int64_t hc_b96_selftest(uint64_t seed, int64_t n) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  auto mask96 = [](B128 v) { return b128(v.lo, v.hi & 0xFFFFFFFFull); };
  int64_t bad = 0;
  for (int64_t t = 0; t < n; ++t) {
    // sparse and dense boards
    const int dens = static_cast<int>(rnd() % 4);
    B128 a = mask96(b128(rnd(), rnd())), b = mask96(b128(rnd(), rnd()));
    for (int d = 0; d < dens; ++d) {
      a = a & mask96(b128(rnd(), rnd()));
      b = b | mask96(b128(rnd(), rnd()));
    }
    const B96 a9 = b96_of(a), b9 = b96_of(b);
    const int s = 1 + static_cast<int>(rnd() % 31);
    bad += !(b128_of(a9 | b9) == (a | b));
    bad += !(b128_of(a9 & b9) == (a & b));
    bad += !(b128_of(a9 ^ b9) == (a ^ b));
    bad += !(b128_of(~a9 & b9) == (~a & b));
    bad += (a9 == b9) != (a == b);
    bad += any(a9) != any(a);
    bad += popc(a9) != popc(a);
    bad += !(b128_of(shl(a9, s)) == mask96(shl(a, s)));
    bad += !(b128_of(shr(a9, s)) == shr(a, s));
    const int i = static_cast<int>(rnd() % 96);
    bad += !(b128_of(bit96(i)) == bit128(i));
    bad += test(a9, i) != test(a, i);
    bad += !(b128_of(lowmask96(i)) == lowmask128(i));
    if (any(a)) {
      bad += lowest(a9) != lowest(a);
      const int k = static_cast<int>(rnd() % static_cast<uint64_t>(popc(a)));
      bad += select96(a9, k) != select128(a, k);
    }
    const bool c = (rnd() & 1) != 0;
    bad += !(b128_of(sel96(c, a9, b9)) == sel128(c, a, b));
  }
  return bad;
}

// k_rollouts<Go9>: the link16 context over three-word bitboards (os_games.h
// Go9, board_size <= 9), the root narrowed as the kernels narrow it.
int hc_rollouts_go9(const char* game_string, const int64_t* actions, int64_t n_actions,
                    int64_t n, const uint32_t* seeds, double* out) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty() || game.cfg.kind != kGo || game.cfg.rows > kGo9MaxSide) {
    g_err = err.empty() ? "go up to 9 x 9 only" : err;
    return -1;
  }
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n_actions; ++i) StateApply(&hs, actions[i]);
  const Go9::State root = go9_state(*reinterpret_cast<const Go::State*>(hs.raw));
  using Ctx16 = GoCtxT<uint8_t, uint16_t>;
  const int cap = 248, cells = game.cfg.rows * game.cfg.cols;
  std::vector<uint32_t> mt(kMtN);
  std::vector<uint64_t> log(cap);
  std::vector<uint16_t> link(cap);
  std::vector<uint8_t> head(cells + 1);
  std::vector<uint32_t> bloom(Ctx16::kBloomWords * 64);
  for (int64_t i = 0; i < n; ++i) {
    MtStream ev{mt.data(), kMtN, 0};
    mt_seed(ev.s, seeds[i]);
    Ctx16 c;
    std::memset(static_cast<void*>(&c), 0, sizeof c);
    c.zob = game.zob.data();
    c.base = hs.hashes.data();
    c.n_base = static_cast<int32_t>(hs.hashes.size());
    c.log = log.data();
    c.link = link.data();
    c.head = head.data();
    c.stride = 1;
    c.head_stride = 1;
    c.cap = cap;
    c.n_heads = cells + 1;
    c.bloom = bloom.data();
    c.init_filters();
    const int r0 = rollout_ret0<Go9, kPolicyCpp>(root, game.cfg, c, ev);
    out[2 * i] = r0;
    out[2 * i + 1] = -r0;
  }
  return 0;
}

int hc_rollouts_go_bloom(const char* game_string, const int64_t* actions, int64_t n_actions,
                         int64_t n, const uint32_t* seeds, double* out) {
  HostGame game;
  bool unsup = false;
  std::string err = LoadHostGame(game_string, &game, &unsup);
  if (!err.empty() || game.cfg.kind != kGo) {
    g_err = err.empty() ? "go only" : err;
    return -1;
  }
  HostState hs;
  hs.game = &game;
  StateInit(&hs);
  for (int64_t i = 0; i < n_actions; ++i) StateApply(&hs, actions[i]);
  std::vector<uint32_t> mt(kMtN);
  std::vector<uint64_t> log(248);
  std::vector<uint32_t> filt(GoCtxBloom::kWords);
  for (int64_t i = 0; i < n; ++i) {
    MtStream ev{mt.data(), kMtN, 0};
    mt_seed(ev.s, seeds[i]);
    GoCtxBloom c;
    std::memset(static_cast<void*>(&c), 0, sizeof c);
    c.zob = game.zob.data();
    c.base = hs.hashes.data();
    c.n_base = static_cast<int32_t>(hs.hashes.size());
    c.log = log.data();
    c.stride = 1;
    c.filt = filt.data();
    c.filt_stride = 1;
    c.cap = 248;
    c.init_filters();
    const int r0 = rollout_ret0<Go, kPolicyCpp>(*reinterpret_cast<Go::State*>(hs.raw), game.cfg,
                                                c, ev);
    out[2 * i] = r0;
    out[2 * i + 1] = -r0;
  }
  return 0;
}

}  // extern "C"
