// gfx950 kernels of the MCTS engine and their launchers, instantiated once per
// game by os_game_<name>.hip (OS_DEFINE_LAUNCHERS).
//
//   k_wsearch   (OS_LAYOUT_WAVE): one 64-lane wavefront per search; game state
//               wave-uniform in SGPRs, MT19937 streams + visit path in LDS
//               (os_wave.h).
//   k_mcts      (OS_LAYOUT_LANE): one lane per search; game state in VGPRs, MT
//               streams + path / expansion buffers in LDS slices (os_mcts.h).
//   k_wselfplay one wave plays a whole self-play game.
//   k_az_step   external-evaluator search, one resumable step per launch.
//   k_rollouts / k_wrollouts  RandomRolloutEvaluator batches.
// Searches never share memory, so the search kernels use no atomics and are
// bit-exact whatever the scheduling.
#ifndef OS_KERNELS_H_
#define OS_KERNELS_H_

#include "os_chance.h"
#include "os_engine_impl.h"

namespace osx {

// The single-search engine of the lane layout: mcts_search, or its chance-node
// form for games that have chance nodes (os_chance.h).
template <class G, class R, int Policy, class Rng>
__device__ SearchResult lane_search(const GameCfg& g, const SearchParams& sp,
                                    const typename G::State& root, typename G::Ctx& ctx,
                                    Node<R>* nodes, uint32_t cap, Rng& bot, Rng& ev,
                                    PathEnt<R>* path, uint16_t* actbuf, int path_cap,
                                    uint32_t* pages, uint32_t own_page) {
  if constexpr (HasChance<G>::value)
    return mcts_search_chance<G, R, Policy>(g, sp, root, ctx, nodes, cap, bot, ev, path,
                                            actbuf, path_cap, pages, own_page);
  else
    return mcts_search<G, R, Policy>(g, sp, root, ctx, nodes, cap, bot, ev, path, actbuf,
                                     path_cap, pages, own_page);
}



#if OS_PHASE_TIMING || OS_WAVE_TIMES
static __device__ uint64_t g_phase_cycles[kDbgSlots];  // diagnostic build only; internal linkage: one per game TU
#endif


template <class G>
struct CtxMaker;
template <class G>
struct CtxMaker {
  __device__ static NoCtx make(const DevArgs&, int64_t, uint64_t*, uint32_t*, uint8_t*) {
    return NoCtx();
  }
};
template <>
struct CtxMaker<Go> {
  __device__ static GoCtx make(const DevArgs& a, int64_t gr, uint64_t* log, uint32_t* link,
                               uint8_t* head) {
    GoCtx c;
    c.zob = a.zob;
    c.base = a.root_hashes + gr * a.hash_stride;
    c.n_base = a.root_nhash[gr];
    c.log = log;
    c.link = link;
    c.head = head;
    c.stride = 1;
    c.head_stride = 1;
    c.n_log = 0;
    c.cap = kGoLogCap;
    c.n_heads = a.cfg.rows * a.cfg.cols + 1;
    c.init_filters();
    return c;
  }
};

// One wave per workgroup at most (LaunchSearch clamps the block): with the
// default 1024-thread bound the compiler caps VGPRs at 128 and spills the
// search's working set to scratch, and lanes 32-63 of a wave64 running such
// spill-heavy code returned wrong results on MI355X (k_az_step).
template <class G, class R, int Policy>
__global__ __launch_bounds__(64) void k_mcts(DevArgs a) {
  const int64_t lr = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (lr >= a.num_roots) return;
  const int64_t gr = a.root_base + lr;
  // Per-lane LDS slices: [blockDim][2][624] MT19937 words, then
  // [blockDim][path_cap] u32 visit path, then [blockDim][child_cap] u16
  // expansion buffer.  Every per-simulation random word and path entry is an
  // LDS access (~tens of cycles) instead of a dependent HBM/L2 round trip.
  extern __shared__ __align__(16) unsigned char smem[];
  const int nb = blockDim.x;
  const int lane = threadIdx.x;
  uint32_t* mt0 = reinterpret_cast<uint32_t*>(smem) + lane * 2 * kMtN;
  PathEnt<R>* path =
      reinterpret_cast<PathEnt<R>*>(smem + static_cast<size_t>(nb) * 2 * kMtN * 4) +
      lane * a.path_cap;
  uint16_t* actbuf =
      reinterpret_cast<uint16_t*>(
          smem + static_cast<size_t>(nb) * (2 * kMtN * 4 + a.path_cap * sizeof(PathEnt<R>))) +
      lane * a.child_cap;
  MtStream bot{mt0, kMtN, 0};
  MtStream ev{mt0 + kMtN, kMtN, 0};
  const bool shared = Policy == kPolicyNumpy && a.shared_stream;
  if (a.import_state) {
    const uint32_t* g0 = a.mt + lr * 2 * kMtN;
    for (int i = 0; i < 2 * kMtN; ++i) mt0[i] = g0[i];
    bot.idx = a.mt_pos[2 * gr];
    bot.pre = 1;
    ev.idx = a.mt_pos[2 * gr + 1];
    ev.pre = 1;
  } else {
    mt_seed(bot.s, a.bot_seeds[gr]);
    if (!shared) mt_seed(ev.s, a.eval_seeds[gr]);
  }
  const typename G::State root = static_cast<const typename G::State*>(a.roots)[gr];
  uint64_t glog[G::State::kNeedsLog ? kGoLogCap : 1];
  uint32_t glink[G::State::kNeedsLog ? kGoLogCap : 1];
  uint8_t ghead[G::State::kNeedsLog ? kGoHeads : 1];
  typename G::Ctx ctx = CtxMaker<G>::make(a, gr, glog, glink, ghead);
  Node<R>* nodes = static_cast<Node<R>*>(a.arena) + lr * static_cast<int64_t>(a.cap);
  SearchResult res;
  if (Policy == kPolicyNumpy && a.shared_stream)
    res = lane_search<G, R, Policy>(a.cfg, a.sp, root, ctx, nodes, a.cap, bot, bot,
                                    path, actbuf, a.path_cap, a.pages,
                                    static_cast<uint32_t>(lr));
  else
    res = lane_search<G, R, Policy>(a.cfg, a.sp, root, ctx, nodes, a.cap, bot, ev,
                                    path, actbuf, a.path_cap, a.pages,
                                    static_cast<uint32_t>(lr));
  res.rng_words = bot.words + ((Policy == kPolicyNumpy && a.shared_stream) ? 0u : ev.words);
  a.results[gr] = res;
  const Node<R>& rn = nodes[0];
  const int P0 = G::to_move(root);
  const int nc = rn.nchild;
  a.nchild[gr] = nc;
  a.root_n[gr] = rn.n;
  a.root_w[gr] = static_cast<double>(rn.w);
  a.root_out[gr] = out_sign<G>(rn.out, P0, a.cfg);
  const int64_t ob = gr * a.max_children;
  for (int k = 0; k < nc && k < a.max_children; ++k) {
    const Node<R>& c = nodes[rn.first + k];
    a.child_action[ob + k] = c.action;
    a.child_n[ob + k] = c.n;
    a.child_w[ob + k] = static_cast<double>(c.w);
    a.child_out[ob + k] = out_sign<G>(c.out, P0, a.cfg);
  }
  const int b = best_child_g<G>(nodes, P0, a.cfg);
  a.best_action[gr] = b < 0 ? -1 : nodes[rn.first + b].action;
  if (a.import_state) {
    bot.finalize();
    a.mt_pos[2 * gr] = bot.idx;
    if (!a.shared_stream) {
      ev.finalize();
      a.mt_pos[2 * gr + 1] = ev.idx;
    }
    uint32_t* g0 = a.mt + lr * 2 * kMtN;
    for (int i = 0; i < 2 * kMtN; ++i) g0[i] = mt0[i];
  }
}

// ---------------------------------------------------------------------------
// Lane-per-search kernel with the per-search buffers in HBM (go's
// OS_LAYOUT_LANE): one lane per search, 64 searches per wave, so leaf
// rollouts run 64 at a time instead of one per wave (profiles/r03/g9).  The
// bot and evaluator MT19937 streams (MtStreamPf: std::mt19937 words, only the
// twisted words stored, the next word's inputs read ahead), the visit path and
// go's position log are contiguous per search; the expansion buffer, the
// log's bucket heads and the Zobrist table sit in LDS (buffers lane-
// interleaved).  C++ policy; fresh bots, or bots continuing numpy-form
// (key, pos) streams (os_mcts_stateful).
// LDS / HBM capacities of k_lsearch per game: expansion-buffer entries per
// lane (u8 actions), Zobrist words, LDS bucket heads (u8, lane-interleaved;
// boards above 11 x 11 keep u16 heads per search in HBM), position-log cap.
template <class G>
struct LsCaps {
  static constexpr int act = 1, zob = 1, heads = 1, log = 1, bloom = 1;
};
template <>
struct LsCaps<Go> {  // act, heads and bloom per lane
  static constexpr int act = 124, zob = 2 * 121, heads = kGoHeads, log = kGoLogCap,
                       bloom = GoCtx::kBloomWords;
};
// k_lsearch<Go9>'s superko-log Bloom filter: 1024 bits per lane (1) or 512
// (0).  A lane whose position hits the filter in a non-empty bucket walks the
// bucket with dependent loads while its wave waits; late in a playout (~165
// entries) 512 bits give ~23% false hits, 1024 ~8%.  The lane search has the
// LDS for it (32 lanes per block); k_rollouts (64 lanes, four waves per
// SIMD) keeps 512.  A/B knob; exact either way.
#ifndef OS_LS_BLOOM1K
#define OS_LS_BLOOM1K 1
#endif
using GoCtxLs = GoCtxT<uint8_t, uint32_t, OS_LS_BLOOM1K ? 32 : 16>;
template <>
struct LsCaps<Go9> {  // 9 x 9: 82 actions, stone counts 0 .. 81
  static constexpr int act = kGo9MaxSide * kGo9MaxSide + 1,
                       zob = 2 * kGo9MaxSide * kGo9MaxSide,
                       heads = kGo9MaxSide * kGo9MaxSide + 1, log = kGoLogCap,
                       bloom = GoCtxLs::kBloomWords;
};
template <>
struct LsCaps<GoBig> {  // actions up to 361: u16 expansion buffers in HBM
  static constexpr int act = 1, zob = 2 * 361, heads = 1, log = kGoLogCapBig, bloom = 1;
};
template <>
struct LsCaps<HexBig> {  // actions up to 360: u16 expansion buffers in HBM
  static constexpr int act = 1, zob = 1, heads = 1, log = 1, bloom = 1;
};
template <class G>
struct LsWide : std::false_type {};  // Node<R, true>: 16-bit child counts
template <>
struct LsWide<GoBig> : std::true_type {};
template <>
struct LsWide<HexBig> : std::true_type {};

template <class G>
struct LCtx {
  __device__ static NoCtx make(const DevArgs&, int64_t, int64_t, uint8_t*, uint32_t*, int) {
    return NoCtx();
  }
};
template <>
struct LCtx<GoBig> {
  __device__ static GoCtxW make(const DevArgs& a, int64_t gr, int64_t lr, uint8_t*, uint32_t*,
                                int) {
    GoCtxW c;
    c.zob = a.zob;
    c.base = a.root_hashes + gr * a.hash_stride;
    c.n_base = a.root_nhash[gr];
    c.log = a.lglog + lr * kGoLogCapBig;
    c.link = a.lglink + lr * kGoLogCapBig;
    c.head = a.lheads + lr * kGoHeadsBig;
    c.head_stride = 1;
    c.stride = 1;
    c.n_log = 0;
    c.cap = kGoLogCapBig;
    c.n_heads = a.cfg.rows * a.cfg.cols + 1;
    c.init_filters();
    return c;
  }
};
template <>
struct LCtx<Go> {
  // lds_heads / lds_bloom: this lane's column of the block's lane-interleaved
  // arrays (stride `lanes`, the block's width).
  __device__ static GoCtx make(const DevArgs& a, int64_t gr, int64_t lr, uint8_t* lds_heads,
                               uint32_t* lds_bloom, int lanes) {
    GoCtx c;
    c.zob = a.zob;
    c.base = a.root_hashes + gr * a.hash_stride;
    c.n_base = a.root_nhash[gr];
    c.log = a.lglog + lr * kGoLogCap;
    c.link = a.lglink + lr * kGoLogCap;
    c.head = lds_heads;
    c.head_stride = lanes;
#if OS_GO_LOG_BLOOM
    c.bloom = lds_bloom;
#else
    (void)lds_bloom;
#endif
    c.stride = 1;
    c.n_log = 0;
    c.cap = kGoLogCap;
    c.n_heads = a.cfg.rows * a.cfg.cols + 1;
    c.init_filters();
    return c;
  }
};

template <>
struct LCtx<Go9> {  // as LCtx<Go>, with k_lsearch's Bloom width (GoCtxLs)
  __device__ static GoCtxLs make(const DevArgs& a, int64_t gr, int64_t lr, uint8_t* lds_heads,
                                 uint32_t* lds_bloom, int lanes) {
    GoCtxLs c;
    c.zob = a.zob;
    c.base = a.root_hashes + gr * a.hash_stride;
    c.n_base = a.root_nhash[gr];
    c.log = a.lglog + lr * kGoLogCap;
    c.link = a.lglink + lr * kGoLogCap;
    c.head = lds_heads;
    c.head_stride = lanes;
#if OS_GO_LOG_BLOOM
    c.bloom = lds_bloom;
#else
    (void)lds_bloom;
#endif
    c.stride = 1;
    c.n_log = 0;
    c.cap = kGoLogCap;
    c.n_heads = a.cfg.rows * a.cfg.cols + 1;
    c.init_filters();
    return c;
  }
};

// Root records of the lane kernels: the host's G::State, except for Go9,
// whose roots are Go::State records narrowed to three-word bitboards.
template <class G>
struct LaneRoot {
  __device__ static typename G::State load(const void* roots, int64_t i) {
    return static_cast<const typename G::State*>(roots)[i];
  }
};
template <>
struct LaneRoot<Go9> {
  __device__ static Go9::State load(const void* roots, int64_t i) {
    return go9_state(static_cast<const Go::State*>(roots)[i]);
  }
};
// go on the lane kernels, either bitboard width.
template <class G>
struct IsLaneGo : std::integral_constant<bool, std::is_same<G, Go>::value ||
                                                   std::is_same<G, Go9>::value> {};

// k_lsearch's go superko log written 8 entries at a time (GoCtxT::wlog; 1)
// or entry by entry (0).  A/B knob.
#ifndef OS_LS_LOGWC
#define OS_LS_LOGWC 1
#endif
// k_lsearch's MT19937 streams: MtStreamWc (words stored 16 at a time; 1) or
// MtStreamPf (word by word; 0).  A/B knob.
#ifndef OS_LS_WC
#define OS_LS_WC 1
#endif
// Timing-only attribution switches for k_lsearch's HBM traffic (results are
// NOT the reference's; A/B builds only): bit 0 draws the MT19937 words from a
// register xorshift (no stream memory), bit 1 logs no superko positions.
#ifndef OS_LS_AB
#define OS_LS_AB 0
#endif
struct MtStreamNoMem {
  uint32_t x;
  uint32_t words;
  __device__ void seed(uint32_t v) { x = v * 2654435761u + 1u; words = 0; }
  __device__ void init_import(int p) { x = 0x9e3779b9u + static_cast<uint32_t>(p); words = 0; }
  __device__ uint32_t next() {
    ++words;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
  }
  __device__ int finalize() const { return 0; }
};

// kL: searches (active lanes) per wave, the block's width.  A lane runs a
// whole search, so a wave is one dependent instruction stream per lane; at
// 65536 roots, 64 lanes per wave are 1024 waves, one per SIMD, and nothing
// hides a wave's memory and dependency stalls.  Narrower blocks trade VALU /
// SALU issue per search (a wave instruction covers kL searches) for kOcc
// resident waves per SIMD (LaunchLs picks kL from the batch size).
template <class G, class R, int kL, int kOcc>
__global__ __launch_bounds__(64, kOcc) void k_lsearch(DevArgs a) {
  // LDS: go's bucket heads and the expansion buffers, lane-interleaved
  // ([i][kL]), and the Zobrist table (read by every move of every lane).
  __shared__ uint8_t heads[LsCaps<G>::heads * kL];
  __shared__ uint32_t lbloom[OS_GO_LOG_BLOOM ? LsCaps<G>::bloom * kL : 1];  // go: superko log filter
  __shared__ uint8_t acts[LsCaps<G>::act * kL];  // go actions up to 15 x 15 are < 256
  __shared__ uint64_t zob[LsCaps<G>::zob];
  if constexpr (G::State::kNeedsLog) {
    const int nz = 2 * a.cfg.rows * a.cfg.cols;
    for (int i = threadIdx.x; i < nz; i += blockDim.x) zob[i] = a.zob[i];
    __syncthreads();
  }
  const int t = static_cast<int>(threadIdx.x);  // < kL (blockDim.x == kL)
  const int64_t lr = static_cast<int64_t>(blockIdx.x) * kL + t;
  if (lr >= a.num_roots) return;
  const int64_t gr = a.root_base + lr;
  // Per-search contiguous buffers: the lanes of a wave drift apart (each at
  // its own draw count, log length and depth), so a batch-SoA layout would
  // touch a new cache line per word; contiguous, a search reuses its lines.
#if OS_LS_AB & 1
  MtStreamNoMem bot, ev;
#elif OS_LS_WC
  // twisted words written 16 at a time from a lane-interleaved LDS buffer
  __shared__ uint32_t mt_wb[2 * 16 * kL];
  MtStreamWc bot{{a.mt + lr * 2 * kMtN, 1, 0, 0}, mt_wb + t, kL};
  MtStreamWc ev{{a.mt + lr * 2 * kMtN + kMtN, 1, 0, 0}, mt_wb + 16 * kL + t, kL};
#else
  MtStreamPf bot{a.mt + lr * 2 * kMtN, 1, 0, 0};
  MtStreamPf ev{a.mt + lr * 2 * kMtN + kMtN, 1, 0, 0};
#endif
  if (a.import_state) {  // the rows hold numpy-form keys (os_mcts_stateful)
    bot.init_import(a.mt_pos[2 * gr]);
    ev.init_import(a.mt_pos[2 * gr + 1]);
  } else {
    bot.seed(a.bot_seeds[gr]);
    ev.seed(a.eval_seeds[gr]);
  }
  StridedPtr<PathEnt<R>> path{static_cast<PathEnt<R>*>(a.lpath) + lr * a.path_cap, 1};
  auto ctx = LCtx<G>::make(a, gr, lr, heads + t, lbloom + t, kL);
  if constexpr (G::State::kNeedsLog) ctx.zob = zob;
#if OS_LS_LOGWC
  // go: the superko log's open 8-entry group in LDS (GoCtxT::wlog)
  constexpr bool kLogWc = IsLaneGo<G>::value;
  __shared__ uint64_t ls_wlog[kLogWc ? GoCtx::kWg * kL : 1];
  __shared__ uint32_t ls_wlink[kLogWc ? GoCtx::kWg * kL : 1];
  if constexpr (kLogWc) {
    ctx.wlog = ls_wlog + t;
    ctx.wlink = ls_wlink + t;
    ctx.wst = kL;
  }
#endif
#if OS_LS_AB & 2
  if constexpr (G::State::kNeedsLog) ctx.cap = 0;
#endif
  const typename G::State root = LaneRoot<G>::load(a.roots, gr);
  using N = Node<R, LsWide<G>::value>;
  N* nodes = static_cast<N*>(a.arena) + lr * static_cast<int64_t>(a.cap);
  SearchResult res;
  if constexpr (LsWide<G>::value) {
    StridedPtr<uint16_t> act{a.lact + lr * a.child_cap, 1};
    res = mcts_search<G, R, kPolicyCpp>(a.cfg, a.sp, root, ctx, nodes, a.cap, bot, ev, path,
                                        act, a.path_cap, a.pages, static_cast<uint32_t>(lr));
  } else {
    StridedPtr<uint8_t> act{acts + t, kL};
    res = mcts_search<G, R, kPolicyCpp>(a.cfg, a.sp, root, ctx, nodes, a.cap, bot, ev, path,
                                        act, a.path_cap, a.pages, static_cast<uint32_t>(lr));
  }
  res.rng_words = bot.words + ev.words;
  a.results[gr] = res;
  const N& rn = nodes[0];
  const int P0 = G::to_move(root);
  const int nc = rn.nchild;
  a.nchild[gr] = nc;
  a.root_n[gr] = rn.n;
  a.root_w[gr] = static_cast<double>(rn.w);
  a.root_out[gr] = out_sign<G>(rn.out, P0, a.cfg);
  const int64_t ob = gr * a.max_children;
  for (int k = 0; k < nc && k < a.max_children; ++k) {
    const N& c = nodes[rn.first + k];
    a.child_action[ob + k] = c.action;
    a.child_n[ob + k] = c.n;
    a.child_w[ob + k] = static_cast<double>(c.w);
    a.child_out[ob + k] = out_sign<G>(c.out, P0, a.cfg);
  }
  const int b = best_child_g<G>(nodes, P0, a.cfg);
  a.best_action[gr] = b < 0 ? -1 : nodes[rn.first + b].action;
  if (a.import_state) {
    a.mt_pos[2 * gr] = bot.finalize();
    a.mt_pos[2 * gr + 1] = ev.finalize();
  }
}

// ---------------------------------------------------------------------------
// Wave-per-search kernel (default layout): one 64-lane workgroup per search.
template <class G>
struct WaveCtxMaker {
  __device__ static NoCtx make(const DevArgs&, int64_t) { return NoCtx(); }
};
template <>
struct WaveCtxMaker<Go> {
  __device__ static GoWaveCtx make(const DevArgs& a, int64_t gr) {
    GoWaveCtx c;
    c.zob = a.zob;
    c.base = a.root_hashes + gr * a.hash_stride;
    c.n_base = a.root_nhash[gr];
    c.init_filters();
    return c;
  }
};

// Arena nodes of each search kept in LDS by the wave kernel (os_wave.h
// NodeCache): the first OS_NODE_CACHE nodes, i.e. the tree's top levels.
#ifndef OS_NODE_CACHE
#define OS_NODE_CACHE 0  // A/B: 128 / 256 / 512 were no faster
#endif

template <class G, class R>
__host__ __device__ constexpr size_t WaveLdsBytes(int path_cap) {
  return static_cast<size_t>(2 * kMtN * 4) + kPageDescLds +
         static_cast<size_t>(path_cap) * sizeof(PathEnt<R>) +
         static_cast<size_t>(OS_NODE_CACHE) * sizeof(Node<R>) + 16;
}

// Minimum waves per SIMD requested from the register allocator (A/B knob).
#ifndef OS_HEX_OCC
#define OS_HEX_OCC 1
#endif
template <class G>
struct WaveOcc {
  static constexpr int value = 1;
};
template <>
struct WaveOcc<Hex> {
  static constexpr int value = OS_HEX_OCC;
};
#ifndef OS_BT_OCC
#define OS_BT_OCC 1
#endif
template <>
struct WaveOcc<Breakthrough> {
  static constexpr int value = OS_BT_OCC;
};

// kPaged: the search may take pages from the pool (os_wave.h kPg*).  The
// reserved-arena variant is a separate kernel: the cold page-switch path
// costs the selection loop scalar registers (C2 +1.4% time).
// kLdsTree: the search's whole reserved arena has an LDS copy (NodeCache
// kCacheAll, written through to HBM), so selection reads every child block
// from LDS.  For batches of at most one search per CU -- a single bot's step
// -- of the games whose reserved tree fits the CU's LDS (LdsTreeGame).
template <class G>
struct LdsTreeGame : std::false_type {};
template <>
struct LdsTreeGame<TicTacToe> : std::true_type {};
template <>
struct LdsTreeGame<ConnectFour> : std::true_type {};
constexpr int64_t kLdsTreeMaxRoots = 256;  // one search per CU

template <class G, class R, int Policy, bool kPaged, bool kPuct, bool kLdsTree = false>
__global__ __launch_bounds__(64, WaveOcc<G>::value) void k_wsearch(DevArgs a) {
  const int64_t lr = blockIdx.x;
  if (lr >= a.num_roots) return;
#if OS_WAVE_TIMES
  const uint64_t wt_start = __builtin_amdgcn_s_memrealtime();
#endif
  const int64_t gr = a.root_base + lr;
  const int l = lane_id();
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* mt = reinterpret_cast<uint32_t*>(smem);
  // [MT bot | MT evaluator | page descriptor address | path | node cache]
  PathEnt<R>* path = reinterpret_cast<PathEnt<R>*>(smem + 2 * kMtN * 4 + kPageDescLds);
  Node<R>* lcache = reinterpret_cast<Node<R>*>(
      smem + ((2 * kMtN * 4 + kPageDescLds + a.path_cap * sizeof(PathEnt<R>) + 15) &
              ~size_t(15)));
  if (l == 0)
    *reinterpret_cast<uint64_t*>(smem + 2 * kMtN * 4) = reinterpret_cast<uintptr_t>(a.pages);
  const bool shared = Policy == kPolicyNumpy && a.shared_stream;
  WaveMt bot, ev;
  bot.s = mt;
  ev.s = mt + kMtN;
  bot.use7 = 0;
  ev.use7 = SmallAbsl<G>::value && Policy == kPolicyCpp && !shared ? 1 : 0;
  if (a.import_state) {
    const uint32_t* g0 = a.mt + lr * 2 * kMtN;
    for (int i = l; i < 2 * kMtN; i += 64) mt[i] = g0[i];
    __syncthreads();
    bot.init_import(a.mt_pos[2 * gr]);
    ev.init_import(a.mt_pos[2 * gr + 1]);
  } else {
    if (l == 0) {
      mt_seed(bot.s, a.bot_seeds[gr]);
      if (!shared) mt_seed(ev.s, a.eval_seeds[gr]);
    }
    __syncthreads();
    bot.init_seeded();
    ev.init_seeded();
  }
  const typename G::State root =
      make_uniform(static_cast<const typename G::State*>(a.roots)[gr]);
  typename WaveCtxOf<G>::type ctx = WaveCtxMaker<G>::make(a, gr);
  Node<R>* nodes = static_cast<Node<R>*>(a.arena) + lr * static_cast<int64_t>(a.cap);
  PhaseCycles ph = {};  // paged: the root's page is page lr = blockIdx.x
#if OS_PHASE_TIMING
  if constexpr (std::is_same<G, Go>::value) ctx.sub = ph.c;
#endif
  // Issue-priority pacing evens out a batch of resident waves; the LDS-tree
  // launch (a few searches, one per CU) has nothing to pace against, so it
  // skips the counter atomic every OS_PACE_EVERY simulations.
  constexpr bool kPaceSearch = OS_PACE != 0 && !kLdsTree;
  SearchResult res = shared
      ? wave_search<G, R, Policy, kPaged, kPuct, kLdsTree ? kCacheAll : OS_NODE_CACHE,
                    kPaceSearch>(a.cfg, a.sp, root, ctx, nodes, a.cap, bot, bot, path,
                                  a.path_cap, ph, lcache)
      : wave_search<G, R, Policy, kPaged, kPuct, kLdsTree ? kCacheAll : OS_NODE_CACHE,
                    kPaceSearch>(a.cfg, a.sp, root, ctx, nodes, a.cap, bot, ev, path,
                                  a.path_cap, ph, lcache);
  res.rng_words = bot.words.get() + (shared ? 0u : ev.words.get());
#if OS_PHASE_TIMING
  ph.c[kPhTwist] = bot.twist_cycles + (shared ? 0u : ev.twist_cycles);
  if (l == 0)
    for (int i = 0; i < kNumPhases; ++i)
      atomicAdd(reinterpret_cast<unsigned long long*>(&g_phase_cycles[i]),
                static_cast<unsigned long long>(ph.c[i]));
#endif
#if OS_WAVE_TIMES
  if (l == 0 && lr < kWaveTimesMax) {
    uint64_t* wt = g_phase_cycles + kNumPhases + 3 * lr;
    wt[0] = wt_start;
    wt[1] = __builtin_amdgcn_s_memrealtime();
    wt[2] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF804)) |
            (static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF814)) << 32);
  }
#endif
  __threadfence_block();
  const Node<R> rn = nodes[0];
  const int P0 = G::to_move(root);
  const int nc = rn.nchild;
  const int64_t ob = gr * a.max_children;
  for (int k = l; k < nc && k < a.max_children; k += 64) {
    const Node<R> c = nodes[rn.first + k];
    a.child_action[ob + k] = c.action;
    a.child_n[ob + k] = c.n;
    a.child_w[ob + k] = static_cast<double>(c.w);
    a.child_out[ob + k] =
        c.out == kUnsolved ? kUnsolved : static_cast<int8_t>(P0 == 0 ? c.out : -c.out);
  }
  if (l == 0) {
    a.results[gr] = res;
    a.nchild[gr] = nc;
    a.root_n[gr] = rn.n;
    a.root_w[gr] = static_cast<double>(rn.w);
    a.root_out[gr] = rn.out == kUnsolved ? kUnsolved
                                         : static_cast<int8_t>(P0 == 0 ? rn.out : -rn.out);
    const int b = best_child(nodes, P0);
    a.best_action[gr] = b < 0 ? -1 : nodes[rn.first + b].action;
  }
  if (a.import_state) {
    if (l == 0) {
      a.mt_pos[2 * gr] = bot.export_pos();
      if (!shared) a.mt_pos[2 * gr + 1] = ev.export_pos();
    }
    __syncthreads();
    uint32_t* g0 = a.mt + lr * 2 * kMtN;
    for (int i = l; i < 2 * kMtN; i += 64) g0[i] = mt[i];
  }
}


// ---------------------------------------------------------------------------
// Games with chance nodes on the wave layout (mcts.cc:
// 285-296): one wave per search running os_chance.h's mcts_search_chance
// WAVE-UNIFORMLY -- every lane executes the same scalar program on the same
// values (the MT19937 streams are WaveMt windows in LDS, drawn by readlane;
// path and expansion buffer in LDS; identical stores from all lanes).  pig
// offers two actions and six chance outcomes per node and plays its rollouts
// serially, so there is no data parallelism to spread over lanes; the wave
// form gives one search per wave (a small batch spreads over every SIMD) and
// the wave self-play kernel below.  Bit-exact with the oracle's MCTSBot.
template <class G, class R>
__host__ __device__ constexpr size_t WaveChanceLdsBytes(int path_cap) {
  return static_cast<size_t>(2 * kMtN * 4) + static_cast<size_t>(path_cap) * sizeof(PathEnt<R>) +
         static_cast<size_t>(kMaxChildren) * 2;
}

#ifndef OS_CHANCE_LDS_TREE
#define OS_CHANCE_LDS_TREE 1  // A/B knob: 0 = the arena stays in HBM
#endif
// kLdsTree: the search's whole arena lives in LDS (after the MT states, path
// and expansion buffer, 16-byte aligned; the log / sqrt LUT after it), and the
// nodes it used are copied to the HBM arena when it ends, where fetch and
// tree export read them.  For a
// batch of at most one search per CU whose reserved arena fits the CU's LDS
// -- a single bot's step: pig's tree walk, wave-uniform scalar code, then
// reads each node in ~100 cycles instead of an L2 round trip.
template <class R>
__host__ __device__ constexpr size_t ChanceTreeLdsOffset(size_t lds) {
  return (lds + 15) & ~size_t(15);
}
// The root record of search i: the host writes G::State records, except for
// Pig2, whose roots are the 10-player Pig records narrowed to two players.
template <class G>
struct ChanceRoot {
  __device__ static typename G::State load(const void* roots, int64_t i) {
    return static_cast<const typename G::State*>(roots)[i];
  }
};
template <>
struct ChanceRoot<Pig2> {
  __device__ static Pig2::State load(const void* roots, int64_t i) {
    const Pig::State& r = static_cast<const Pig::State*>(roots)[i];
    Pig2::State s;
    s.score[0] = r.score[0];
    s.score[1] = r.score[1];
    s.turn_total = r.turn_total;
    s.cur = r.cur;
    s.turn_player = r.turn_player;
    s.moves = r.moves;
    return s;
  }
};

template <class G, class R, int Policy, bool kLdsTree = false>
__global__ __launch_bounds__(64) void k_wsearch_chance(DevArgs a) {
  const int64_t lr = blockIdx.x;
  if (lr >= a.num_roots) return;
  const int64_t gr = a.root_base + lr;
  const int l = lane_id();
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* mt = reinterpret_cast<uint32_t*>(smem);
  PathEnt<R>* path = reinterpret_cast<PathEnt<R>*>(smem + 2 * kMtN * 4);
  uint16_t* actbuf = reinterpret_cast<uint16_t*>(smem + 2 * kMtN * 4 +
                                                 a.path_cap * sizeof(PathEnt<R>));
  const bool shared = Policy == kPolicyNumpy && a.shared_stream;
  WaveMt bot, ev;
  bot.s = mt;
  ev.s = mt + kMtN;
  bot.use7 = ev.use7 = 0;
  if (a.import_state) {
    const uint32_t* g0 = a.mt + lr * 2 * kMtN;
    for (int i = l; i < 2 * kMtN; i += 64) mt[i] = g0[i];
    __syncthreads();
    bot.init_import(a.mt_pos[2 * gr]);
    ev.init_import(a.mt_pos[2 * gr + 1]);
  } else {
    if (l == 0) {
      mt_seed(bot.s, a.bot_seeds[gr]);
      if (!shared) mt_seed(ev.s, a.eval_seeds[gr]);
    }
    __syncthreads();
    bot.init_seeded();
    ev.init_seeded();
  }
  const typename G::State root = make_uniform(ChanceRoot<G>::load(a.roots, gr));
  typename G::Ctx ctx;
  Node<R>* nodes = static_cast<Node<R>*>(a.arena) + lr * static_cast<int64_t>(a.cap);
  Node<R>* arena = nodes;
  SearchParams sp = a.sp;
  if constexpr (kLdsTree) {
    // [.. | arena (cap nodes) | log / sqrt LUT (max_simulations + 1)]
    const size_t off = ChanceTreeLdsOffset<R>(WaveChanceLdsBytes<G, R>(a.path_cap));
    arena = reinterpret_cast<Node<R>*>(smem + off);
    double* lut = reinterpret_cast<double*>(smem + off + static_cast<size_t>(a.cap) * sizeof(Node<R>));
    for (int i = l; i <= a.sp.max_simulations; i += 64) lut[i] = a.sp.log_lut[i];
    __syncthreads();
    sp.log_lut = lut;
  }
  SearchResult res = shared
      ? mcts_search_chance<G, R, Policy>(a.cfg, sp, root, ctx, arena, a.cap, bot, bot, path,
                                         actbuf, a.path_cap)
      : mcts_search_chance<G, R, Policy>(a.cfg, sp, root, ctx, arena, a.cap, bot, ev, path,
                                         actbuf, a.path_cap);
  res.rng_words = bot.words.get() + (shared ? 0u : ev.words.get());
  if constexpr (kLdsTree) {  // the nodes used, to the HBM arena (coalesced)
    __syncthreads();
    const uint32_t used = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<int>(res.used < a.cap ? res.used : a.cap)));
    for (uint32_t i = static_cast<uint32_t>(l); i < used; i += 64) nodes[i] = arena[i];
  }
  __threadfence_block();
  const Node<R> rn = nodes[0];
  const int P0 = G::to_move(root);
  const int nc = rn.nchild;
  const int64_t ob = gr * a.max_children;
  for (int k = l; k < nc && k < a.max_children; k += 64) {
    const Node<R> c = nodes[rn.first + k];
    a.child_action[ob + k] = c.action;
    a.child_n[ob + k] = c.n;
    a.child_w[ob + k] = static_cast<double>(c.w);
    a.child_out[ob + k] = out_sign<G>(c.out, P0, a.cfg);
  }
  if (l == 0) {
    a.results[gr] = res;
    a.nchild[gr] = nc;
    a.root_n[gr] = rn.n;
    a.root_w[gr] = static_cast<double>(rn.w);
    a.root_out[gr] = out_sign<G>(rn.out, P0, a.cfg);
    const int b = best_child_g<G>(nodes, P0, a.cfg);
    a.best_action[gr] = b < 0 ? -1 : nodes[rn.first + b].action;
  }
  if (a.import_state) {
    if (l == 0) {
      a.mt_pos[2 * gr] = bot.export_pos();
      if (!shared) a.mt_pos[2 * gr + 1] = ev.export_pos();
    }
    __syncthreads();
    uint32_t* g0 = a.mt + lr * 2 * kMtN;
    for (int i = l; i < 2 * kMtN; i += 64) g0[i] = mt[i];
  }
}

// Self-play of a two-player game with chance nodes, one game per wave, as
// examples/mcts_example.cc:77-136 PlayGame drives it: decision nodes ask
// bots[CurrentPlayer]->Step (mcts_search_chance + BestChild, mcts.cc:219-226),
// chance nodes take SampleAction(ChanceOutcomes(), rng) (:103-109) with the
// game's own rng -- actor_seeds[g] (as alpha_zero.cc PlayGame's one rng).
// Every action (chance outcomes included) is recorded; visit rows are zero
// for chance moves.  Wave-uniform, like k_wsearch_chance.
template <class G, class R>
__host__ __device__ constexpr size_t SelfPlayChanceLdsBytes(int path_cap) {
  return static_cast<size_t>(4 * kMtN * 4) + static_cast<size_t>(path_cap) * sizeof(PathEnt<R>) +
         static_cast<size_t>(kMaxChildren) * 2;
}

template <class G, class R>
__global__ __launch_bounds__(64) void k_wselfplay_chance(SpArgs a) {
  const int64_t lg = blockIdx.x;
  if (lg >= a.num_games) return;
  const int64_t gg = a.game_base + lg;
  const int l = lane_id();
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* mt = reinterpret_cast<uint32_t*>(smem);
  PathEnt<R>* path = reinterpret_cast<PathEnt<R>*>(smem + 4 * kMtN * 4);
  uint16_t* actbuf = reinterpret_cast<uint16_t*>(smem + 4 * kMtN * 4 +
                                                 a.path_cap * sizeof(PathEnt<R>));
  WaveMt b0, b1, ev, act;
  b0.s = mt;
  b1.s = mt + kMtN;
  ev.s = mt + 2 * kMtN;
  act.s = mt + 3 * kMtN;
  b0.use7 = b1.use7 = ev.use7 = act.use7 = 0;
  if (l == 0) {
    mt_seed(b0.s, a.bot_seeds[2 * gg]);
    mt_seed(b1.s, a.bot_seeds[2 * gg + 1]);
    mt_seed(ev.s, a.eval_seeds[gg]);
    mt_seed(act.s, a.actor_seeds[gg]);
  }
  __syncthreads();
  b0.init_seeded();
  b1.init_seeded();
  ev.init_seeded();
  act.init_seeded();
  typename G::State s = make_uniform(static_cast<const typename G::State*>(a.starts)[gg]);
  typename G::Ctx ctx;
  Node<R>* nodes = static_cast<Node<R>*>(a.arena) + lg * static_cast<int64_t>(a.cap);
  SearchResult tot;
  tot.status = kOk;
  tot.sims = tot.nodes = tot.gc_runs = tot.max_depth = 0;
  tot.used = tot.scanned = tot.backed = tot.expanded = tot.solver_scanned = 0;
  tot.rng_words = tot.pad = 0;
  int m = 0;
  while (!G::terminal(s, a.cfg)) {
    if (m >= a.max_len) {
      tot.status = kGameOverflow;
      break;
    }
    const typename G::Legal lgl = G::legal(s, a.cfg, ctx);
    int act_i;
    if (G::chance(s)) {
      act_i = lgl.kth(sample_chance<G, kPolicyCpp>(a.cfg, act));
      if (a.visits) {
        int32_t* v = a.visits + (gg * a.max_len + m) * static_cast<int64_t>(a.num_actions);
        for (int i = l; i < a.num_actions; i += 64) v[i] = 0;
      }
    } else {
      const int p = G::to_move(s);
      WaveMt bot = p == 0 ? b0 : b1;
      const SearchResult r = mcts_search_chance<G, R, kPolicyCpp>(
          a.cfg, a.sp, s, ctx, nodes, a.cap, bot, ev, path, actbuf, a.path_cap);
      if (p == 0) b0 = bot;
      else b1 = bot;
      tot.sims += r.sims;
      tot.nodes += r.nodes;
      tot.used = r.used > tot.used ? r.used : tot.used;
      tot.gc_runs += r.gc_runs;
      tot.max_depth = r.max_depth > tot.max_depth ? r.max_depth : tot.max_depth;
      tot.scanned += r.scanned;
      tot.backed += r.backed;
      tot.expanded += r.expanded;
      tot.solver_scanned += r.solver_scanned;
      if (r.status != kOk) {
        tot.status = r.status;
        break;
      }
      __threadfence_block();
      const int b = best_child_g<G>(nodes, p, a.cfg);  // MCTSBot::Step (mcts.cc:222-225)
      const uint32_t rfirst = nodes[0].first;
      const int rnc = nodes[0].nchild;
      act_i = nodes[rfirst + b].action;
      if (a.visits) {
        int32_t* v = a.visits + (gg * a.max_len + m) * static_cast<int64_t>(a.num_actions);
        for (int i = l; i < a.num_actions; i += 64) v[i] = 0;
        __threadfence_block();
        for (int k = l; k < rnc; k += 64) {
          const Node<R> c = nodes[rfirst + k];
          v[c.action] = c.n;
        }
      }
      if (a.obs) {  // ObservationTensor(player to move) of the position searched
        float* o = a.obs + (gg * a.max_len + m) * static_cast<int64_t>(a.obs_size);
        const int cells = a.cfg.rows * a.cfg.cols;
        for (int i = l; i < a.obs_size; i += 64) o[i] = G::obs(s, a.cfg, p, i / cells, i % cells);
      }
    }
    if (l == 0) a.actions[gg * a.max_len + m] = act_i;
    G::apply(s, a.cfg, ctx, act_i);
    s = make_uniform(s);
    ++m;
  }
  for (int i = m + l; i < a.max_len; i += 64) a.actions[gg * a.max_len + i] = -1;
  if (l == 0) {
    a.length[gg] = m;
    const int code = G::ret0(s, a.cfg, ctx);
    a.returns[2 * gg] = OutValue<G>::value(code, 0, a.cfg);
    a.returns[2 * gg + 1] = OutValue<G>::value(code, 1, a.cfg);
    tot.rng_words = b0.words.get() + b1.words.get() + ev.words.get() + act.words.get();
    a.results[gg] = tot;
  }
}


template <class G>
struct SpCtx {  // games without a history context
  __device__ static NoCtx make(const SpArgs&, int64_t) { return NoCtx(); }
  __device__ static void commit(NoCtx&, const SpArgs&, int64_t) {}
};
template <>
struct SpCtx<Go> {
  __device__ static GoWaveCtx make(const SpArgs& a, int64_t gg) {
    GoWaveCtx c;
    c.zob = a.zob;
    c.base = a.hist + gg * a.hash_stride;
    c.n_base = a.hist_n[gg];
    c.init_filters();
    return c;
  }
  // The move just applied logged its position (go.cc:199-208): it joins the
  // game history that the next searches treat as "before the root" (already
  // in the lanes' slots; stored to the history for the host).
  __device__ static void commit(GoWaveCtx& c, const SpArgs& a, int64_t gg) {
    uint64_t* h = a.hist + gg * a.hash_stride;
    const int l = lane_id();
    const uint64_t sl[4] = {c.s0, c.s1, c.s2, c.s3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 64 * j + l;
      if (i >= c.n_base && i < c.n && i < a.hash_stride) h[i] = sl[j];
    }
    __threadfence_block();
    c.n_base = c.n < a.hash_stride ? c.n : a.hash_stride;
    c.reset();
  }
};

template <class G, class R>
__host__ __device__ constexpr size_t SelfPlayLdsBytes(int path_cap) {
  return static_cast<size_t>(4 * kMtN * 4) + static_cast<size_t>(path_cap) * sizeof(PathEnt<R>);
}

// AlphaZero's move choice (alpha_zero.cc:77-95) from the root's children
// (lane k holds child k in slot 0, k + 64 in slot 1): the action index in the
// child block, with the normalised policy (lane-distributed) and the root
// value.  Sums run serially in child order, as NormalizePolicy and
// SampleAction add them (spiel.cc:327-366).
struct AzChoice {
  int child;
  double p0, p1;
};
template <class R>
__device__ AzChoice az_choose(const SpArgs& a, const Node<R>* kids, int rnc, bool sample,
                              WaveMt& act, int best) {
  const int l = lane_id();
  const int32_t n0 = l < rnc ? kids[l].n : 0;
  const int32_t n1 = l + 64 < rnc ? kids[l + 64].n : 0;
  const double* lut = a.pow_lut;
  double p0 = l < rnc ? (lut ? lut[n0] : static_cast<double>(n0)) : 0.0;
  double p1 = l + 64 < rnc ? (lut ? lut[n1] : static_cast<double>(n1)) : 0.0;
  double sum = 0.0;
  for (int k = 0; k < rnc; ++k) sum += k < 64 ? rld(p0, k) : rld(p1, k - 64);
  p0 /= sum;
  p1 /= sum;
  AzChoice c;
  c.p0 = p0;
  c.p1 = p1;
  c.child = best;
  if (sample) {
    const double z = AbslUniformDouble01(act);
    double acc = 0.0;
    c.child = -1;
    for (int k = 0; k < rnc; ++k) {
      const double pk = k < 64 ? rld(p0, k) : rld(p1, k - 64);
      if (c.child < 0 && acc <= z && z < acc + pk) c.child = k;
      acc += pk;
    }
    // SampleAction's SpielFatalError (z beyond the rounded total) cannot
    // stop a kernel: take the last child, as the oracle restatement does.
    if (c.child < 0) c.child = rnc - 1;
  }
  return c;
}

template <class G, class R, bool kPuct>
__global__ __launch_bounds__(64) void k_wselfplay(SpArgs a) {
  const int64_t lg = blockIdx.x;
  if (lg >= a.num_games) return;
  const int64_t gg = a.game_base + lg;
  const int l = lane_id();
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* mt = reinterpret_cast<uint32_t*>(smem);
  PathEnt<R>* path = reinterpret_cast<PathEnt<R>*>(smem + 4 * kMtN * 4);
  WaveMt b0, b1, ev, act;
  b0.s = mt;
  b1.s = mt + kMtN;
  ev.s = mt + 2 * kMtN;
  act.s = mt + 3 * kMtN;
  b0.use7 = b1.use7 = act.use7 = 0;
  ev.use7 = SmallAbsl<G>::value ? 1 : 0;
  const bool actor = a.actor_seeds != nullptr;
  if (l == 0) {
    mt_seed(b0.s, a.bot_seeds[2 * gg]);
    mt_seed(b1.s, a.bot_seeds[2 * gg + 1]);
    mt_seed(ev.s, a.eval_seeds[gg]);
    if (actor) mt_seed(act.s, a.actor_seeds[gg]);
  }
  __syncthreads();
  b0.init_seeded();
  b1.init_seeded();
  ev.init_seeded();
  act.init_seeded();
  // The game's resign cutoff (alpha_zero.cc:154-157), drawn first.
  double cutoff = a.max_utility + 1.0;
  if (actor && a.resign) {
    const double u = AbslUniformDouble01(act);
    if (u < a.cutoff_probability) cutoff = a.cutoff_value;
  }
  typename G::State s = make_uniform(static_cast<const typename G::State*>(a.starts)[gg]);
  typename WaveCtxOf<G>::type ctx = SpCtx<G>::make(a, gg);
  Node<R>* nodes = static_cast<Node<R>*>(a.arena) + lg * static_cast<int64_t>(a.cap);
  PhaseCycles ph = {};
  SearchResult tot;
  tot.status = kOk;
  tot.sims = tot.nodes = tot.gc_runs = tot.max_depth = 0;
  tot.used = tot.scanned = tot.backed = tot.expanded = tot.solver_scanned = 0;
  tot.rng_words = tot.pad = 0;
  int m = 0;
  bool resigned = false;
  double res_value = 0.0;
  int res_player = 0;
  while (!G::terminal(s, a.cfg)) {
    if (m >= a.max_len) {
      tot.status = kGameOverflow;
      break;
    }
    const int p = G::to_move(s);
    WaveMt bot = p == 0 ? b0 : b1;
    const SearchResult r =
        wave_search<G, R, kPolicyCpp, false, kPuct>(a.cfg, a.sp, s, ctx, nodes, a.cap, bot, ev,
                                                    path, a.path_cap, ph);
    if (p == 0) b0 = bot;
    else b1 = bot;
    tot.sims += r.sims;
    tot.nodes += r.nodes;
    tot.used = r.used > tot.used ? r.used : tot.used;
    tot.gc_runs += r.gc_runs;
    tot.max_depth = r.max_depth > tot.max_depth ? r.max_depth : tot.max_depth;
    tot.scanned += r.scanned;
    tot.backed += r.backed;
    tot.expanded += r.expanded;
    tot.solver_scanned += r.solver_scanned;
    if (r.status != kOk) {
      tot.status = r.status;
      break;
    }
    __threadfence_block();
    // MCTSBot::Step: BestChild of the root (mcts.cc:222-225).
    int bi = 0;
    if (l == 0) bi = best_child(nodes, p);
    bi = rli(bi, 0);
    const uint32_t rfirst = static_cast<uint32_t>(rli(static_cast<int>(nodes[0].first), 0));
    const int rnc = rli(nodes[0].nchild, 0);
    // AlphaZero's choice when an actor rng is given (alpha_zero.cc:77-95).
    const bool want_policy = a.policy != nullptr || actor;
    AzChoice ch;
    ch.child = bi;
    ch.p0 = ch.p1 = 0.0;
    if (want_policy)
      ch = az_choose(a, nodes + rfirst, rnc, actor && m < a.temperature_drop, act, bi);
    const int act_i = rli(nodes[rfirst + ch.child].action, 0);
    // root->total_reward / root->explore_count (alpha_zero.cc:92)
    const double rw = rld(static_cast<double>(nodes[0].w), 0);
    const double rv = rw / static_cast<double>(rli(nodes[0].n, 0));
    if (a.visits) {
      int32_t* v = a.visits + (gg * a.max_len + m) * static_cast<int64_t>(a.num_actions);
      for (int i = l; i < a.num_actions; i += 64) v[i] = 0;
      __threadfence_block();
      for (int k = l; k < rnc; k += 64) {
        const Node<R> c = nodes[rfirst + k];
        v[c.action] = c.n;
      }
    }
    if (a.policy) {
      double* pv = a.policy + (gg * a.max_len + m) * static_cast<int64_t>(a.num_actions);
      for (int i = l; i < a.num_actions; i += 64) pv[i] = 0.0;
      __threadfence_block();
      if (l < rnc) pv[nodes[rfirst + l].action] = ch.p0;
      if (l + 64 < rnc) pv[nodes[rfirst + l + 64].action] = ch.p1;
    }
    if (a.root_value && l == 0) a.root_value[gg * a.max_len + m] = rv;
    if (a.obs) {  // ObservationTensor(player to move) of the position searched
      float* o = a.obs + (gg * a.max_len + m) * static_cast<int64_t>(a.obs_size);
      const int cells = a.cfg.rows * a.cfg.cols;
      for (int i = l; i < a.obs_size; i += 64) o[i] = G::obs(s, a.cfg, p, i / cells, i % cells);
    }
    if (l == 0) a.actions[gg * a.max_len + m] = act_i;
    ctx.reset();
    G::apply(s, a.cfg, ctx, act_i);
    SpCtx<G>::commit(ctx, a, gg);
    s = make_uniform(s);
    ++m;
    // alpha_zero.cc:105-110: a decided position ends the game early.
    if (!G::terminal(s, a.cfg) && fabs(rv) > cutoff) {
      resigned = true;
      res_value = rv;
      res_player = p;
      break;
    }
  }
  tot.rng_words = b0.words.get() + b1.words.get() + ev.words.get() + act.words.get();
  for (int k = m + l; k < a.max_len; k += 64) a.actions[gg * a.max_len + k] = -1;
  if (a.visits) {  // rows after the last move are all-zero policy targets
    int32_t* v = a.visits + (gg * a.max_len + m) * static_cast<int64_t>(a.num_actions);
    const int64_t nz = static_cast<int64_t>(a.max_len - m) * a.num_actions;
    for (int64_t i = l; i < nz; i += 64) v[i] = 0;
  }
  if (a.policy) {
    double* pv = a.policy + (gg * a.max_len + m) * static_cast<int64_t>(a.num_actions);
    const int64_t nz = static_cast<int64_t>(a.max_len - m) * a.num_actions;
    for (int64_t i = l; i < nz; i += 64) pv[i] = 0.0;
  }
  if (a.root_value)
    for (int k = m + l; k < a.max_len; k += 64) a.root_value[gg * a.max_len + k] = 0.0;
  if (a.obs) {
    float* o = a.obs + (gg * a.max_len + m) * static_cast<int64_t>(a.obs_size);
    const int64_t nz = static_cast<int64_t>(a.max_len - m) * a.obs_size;
    for (int64_t i = l; i < nz; i += 64) o[i] = 0.0f;
  }
  if (l == 0) {
    a.length[gg] = m;
    if (resigned) {
      a.returns[2 * gg + res_player] = res_value;
      a.returns[2 * gg + 1 - res_player] = -res_value;
    } else {
      const int r0 = G::terminal(s, a.cfg) ? G::ret0(s, a.cfg, ctx) : 0;
      a.returns[2 * gg] = static_cast<double>(r0);
      a.returns[2 * gg + 1] = static_cast<double>(-r0);
    }
    a.results[gg] = tot;
  }
}


// The root fields of the history context; az_step binds the log to the
// search's continuation.
template <class G>
struct AzCtx {
  __device__ static NoCtx make(const AzArgs&, int64_t) { return NoCtx(); }
};
template <>
struct AzCtx<Go> {
  __device__ static GoCtx make(const AzArgs& a, int64_t r) {
    GoCtx c;
    c.zob = a.zob;
    c.base = a.root_hashes + r * a.hash_stride;
    c.n_base = a.root_nhash[r];
    c.n_heads = a.cfg.rows * a.cfg.cols + 1;
    return c;
  }
};

// __launch_bounds__(64) matches the launch and lifts the 128-VGPR cap of the
// default bound: without it the state machine spilled ~800 VGPRs to scratch
// and searches in lanes 32-63 of each wave64 diverged from the oracle
// (test_az.py many_roots); with it nothing spills to scratch.
template <class G>
__global__ __launch_bounds__(64) void k_az_step(AzArgs a) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= a.num_roots) return;
  AzSlot<G>& sl = static_cast<AzSlot<G>*>(a.slots)[r];
  const int stage0 = sl.stage;
  if (stage0 == kAzDone) {
    a.kind[r] = kAzNone;
    return;
  }
  uint32_t* mt = a.mt + r * kMtN;
  if (stage0 == kAzStart) {
    if (a.import_mt) {  // the row already holds the caller's key
      sl.mt_idx = a.mt_pos_in[r];
      sl.mt_pre = 1;
    } else {
      mt_seed(mt, a.bot_seeds[r]);
      sl.mt_idx = kMtN;
      sl.mt_pre = 0;
    }
    sl.depth = 0;
    sl.s = static_cast<const typename G::State*>(a.roots)[r];
  }
  MtStream bot{mt, sl.mt_idx, sl.mt_pre, 0};
  const typename G::State root = static_cast<const typename G::State*>(a.roots)[r];
  Node<double>* nodes = a.arena + r * static_cast<int64_t>(a.cap);
  AzIo io;
  io.kind = a.kind + r;
  io.obs = a.obs + r * a.obs_size;
  io.legal = a.legal + r * a.num_actions;
  io.prior = a.prior_in + r * a.num_actions;
  io.value = a.value_in + r;
  AzNoise nz;
  nz.noise = a.noise ? a.noise + r * a.noise_stride : nullptr;
  nz.skip = a.noise ? a.noise_skip[r] : 0;
  nz.eps = a.noise_eps;
  typename G::Ctx ctx = AzCtx<G>::make(a, r);
  az_step<G>(a.cfg, a.sp, a.puct, root, sl, nodes, a.priors + r * static_cast<int64_t>(a.cap),
             a.raw ? a.raw + r * static_cast<int64_t>(a.cap) : nullptr, a.cap, bot, io,
             a.obs_size, a.num_actions, ctx, nz, a.np_policy != 0);
  sl.mt_idx = bot.idx;
  sl.mt_pre = bot.pre;
  sl.res.rng_words += bot.words;
  if (*io.kind != kAzNone) {
    atomicAdd(a.shards + (blockIdx.x % kAzShards) * kAzShardStride, 1);
    return;
  }
  if (a.import_mt) {  // the bot's rng_ back in numpy (key, pos) form
    bot.finalize();
    a.mt_pos_out[r] = bot.idx;
  }
  // Finished in this step: publish the root's children like the search kernels.
  const int P0 = G::to_move(root);
  const Node<double> rn = nodes[0];
  const int nc = rn.nchild;
  const int64_t ob = r * a.max_children;
  for (int k = 0; k < nc && k < a.max_children; ++k) {
    const Node<double> c = nodes[rn.first + k];
    a.child_action[ob + k] = c.action;
    a.child_n[ob + k] = c.n;
    a.child_w[ob + k] = c.w;
    a.child_out[ob + k] =
        c.out == kUnsolved ? kUnsolved : static_cast<int8_t>(P0 == 0 ? c.out : -c.out);
  }
  a.results[r] = sl.res;
  a.nchild[r] = nc;
  a.root_n[r] = rn.n;
  a.root_w[r] = rn.w;
  a.root_out[r] = rn.out == kUnsolved ? kUnsolved
                                      : static_cast<int8_t>(P0 == 0 ? rn.out : -rn.out);
  const int b = best_child(nodes, P0);
  a.best_action[r] = b < 0 ? -1 : nodes[rn.first + b].action;
}


// ---------------------------------------------------------------------------
// Wave-per-search external-evaluator step (os_az.h semantics; SURVEY §8f rank
// 2).  k_az_step runs one search per LANE with its whole continuation read
// and written per lane -- 16384 searches fill 256 waves, one per CU, each
// lane's chain of dependent HBM accesses exposed.  Here one WAVE advances one
// search, as k_wsearch does: the child scan is one coalesced load (lane k <->
// child k) and a DPP argmax, the expansion's shuffle runs on the lanes, the
// backup updates every path node at once (lane d <-> depth d), and the request
// (observation tensor, legal mask) is written by all lanes.  Between launches
// the continuation stays in the same AzSlot<G> (state, counters, path, go's
// positions since the root) and the bot rng in its HBM row in numpy form
// (WaveMtRow).  GC (mcts.cc:402-424) is not implemented here: the host runs
// k_az_step whenever the node budget could be reached.  Bit-exact with
// az_step (tests/test_az.py, both layouts).
template <class G>
struct WazCtx {
  __device__ static NoCtx make(const AzArgs&, int64_t) { return NoCtx(); }
  __device__ static void load_tail(NoCtx&, const AzSlot<G>&) {}
  __device__ static void save_tail(const NoCtx&, AzSlot<G>&) {}
};
template <>
struct WazCtx<Go> {
  __device__ static GoWaveCtx make(const AzArgs& a, int64_t r) {
    GoWaveCtx c;
    c.zob = a.zob;
    c.base = a.root_hashes + r * a.hash_stride;
    c.n_base = a.root_nhash[r];
    c.init_filters();
    return c;
  }
  // The pending simulation's positions since the root follow the base.
  __device__ static void load_tail(GoWaveCtx& c, const AzSlot<Go>& sl) {
    const int nl = __builtin_amdgcn_readfirstlane(sl.glog.n_log);
    const int l = lane_id();
    uint64_t* sv[4] = {&c.s0, &c.s1, &c.s2, &c.s3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 64 * j + l;
      const bool in = i >= c.n_base && i < c.n_base + nl && i < GoWaveCtx::kCap;
      const uint64_t v = in ? sl.glog.log[i - c.n_base] : 0ull;
      *sv[j] = in ? v : *sv[j];
    }
    c.n = c.n_base + nl < GoWaveCtx::kCap ? c.n_base + nl : GoWaveCtx::kCap;
    // Every held entry stays a candidate (a superset of the capture rule's:
    // positions after the last capture cannot repeat anyway).
    c.cand_end = c.n;
  }
  __device__ static void save_tail(const GoWaveCtx& c, AzSlot<Go>& sl) {
    const int l = lane_id();
    const uint64_t sv[4] = {c.s0, c.s1, c.s2, c.s3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 64 * j + l;
      if (i >= c.n_base && i < c.n && i - c.n_base < kAzLogCap) sl.glog.log[i - c.n_base] = sv[j];
    }
    if (l == 0) sl.glog.n_log = c.n - c.n_base;
  }
};

// Path of the pending simulation on the lanes: entry d in lane d % 64 of slot d / 64.
struct WazPath {
  uint32_t p0, p1, p2, p3;
  __device__ uint32_t at(int d) const {
    const int j = d >> 6, q = d & 63;
    return rl32(j == 0 ? p0 : (j == 1 ? p1 : (j == 2 ? p2 : p3)), q);
  }
  __device__ void set(int d, uint32_t v) {
    const int j = d >> 6;
    const bool me = lane_id() == (d & 63);
    p0 = me && j == 0 ? v : p0;
    p1 = me && j == 1 ? v : p1;
    p2 = me && j == 2 ? v : p2;
    p3 = me && j == 3 ? v : p3;
  }
};

// OS_WAZ_CHECK (debug builds): every computed index of k_waz_step is checked
// before use; a violation ends the search with status 100 + site instead of
// touching memory out of range.
#ifndef OS_WAZ_CHECK
#define OS_WAZ_CHECK 0
#endif
#if OS_WAZ_CHECK
#define WAZ_CHECK(cond, site)                                   \
  do {                                                          \
    if (ballot(!(cond))) {                                      \
      res.status = 100 + (site);                                \
      request = kAzNone;                                        \
      goto finish;                                              \
    }                                                           \
  } while (0)
#else
#define WAZ_CHECK(cond, site) do {} while (0)
#endif

template <class G, bool kPuct>
__global__ __launch_bounds__(64) void k_waz_step(AzArgs a) {
  const int64_t r = blockIdx.x;
  if (r >= a.num_roots) return;
  const int l = lane_id();
#if OS_PHASE_TIMING
  // Diagnostic build: cycles per phase of one launch (prologue = kPhRollout,
  // descent = kPhSelect, expansion = kPhExpand, backup + solver = kPhBackup,
  // request / result writes = kPhTail), summed over the launch's waves.
  PhaseCycles ph = {};
  const uint64_t ph_t0 = OS_PH_NOW();
  uint64_t ph_t = ph_t0;
  auto ph_flush = [&]() {  // sampled: one search in 64 (atomics would serialise the launch)
    ph.c[kPhTotal] = OS_PH_NOW() - ph_t0;
    if (l == 0 && (r & 63) == 0)
      for (int i = 0; i < kNumPhases; ++i)
        atomicAdd(reinterpret_cast<unsigned long long*>(&g_phase_cycles[i]),
                  static_cast<unsigned long long>(ph.c[i]));
  };
#define WAZ_PH(id)                 \
  do {                             \
    const uint64_t t_ = OS_PH_NOW(); \
    ph.c[id] += t_ - ph_t;         \
    ph_t = t_;                     \
  } while (0)
#else
#define WAZ_PH(id) do {} while (0)
#endif
#if OS_WAVE_TIMES
  // Diagnostic build: (start, end, HW_ID | XCC_ID << 32) of every search's
  // wave in the launch that runs its 21st simulation (sim == 20 at entry).
  const uint64_t wt_start = __builtin_amdgcn_s_memrealtime();
  bool wt_on = false;
  auto wt_flush = [&]() {
    if (wt_on && l == 0 && r < kWaveTimesMax) {
      uint64_t* wt = g_phase_cycles + kNumPhases + 3 * r;
      wt[0] = wt_start;
      wt[1] = __builtin_amdgcn_s_memrealtime();
      wt[2] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF804)) |
              (static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF814)) << 32);
    }
  };
#endif
  __shared__ uint32_t mt_lds[kMtN];
  AzSlot<G>& sl = static_cast<AzSlot<G>*>(a.slots)[r];
  int stage = __builtin_amdgcn_readfirstlane(sl.stage);
  if (stage == kAzDone) {
    if (l == 0) a.kind[r] = kAzNone;
#if OS_PHASE_TIMING
    ph_flush();
#endif
    return;
  }
  const GameCfg& g = a.cfg;
  const SearchParams& sp = a.sp;
  const typename G::State root = make_uniform(static_cast<const typename G::State*>(a.roots)[r]);
  const int P0 = G::to_move(root);
  const int A = a.num_actions;
  Node<double>* nodes = a.arena + r * static_cast<int64_t>(a.cap);
  double* prior = a.priors + r * static_cast<int64_t>(a.cap);
  double* raw = a.raw ? a.raw + r * static_cast<int64_t>(a.cap) : nullptr;
  const double* pin = a.prior_in + r * static_cast<int64_t>(A);
  const uint32_t cap = a.cap;
  const double inf = __builtin_huge_val();
  typename WaveCtxOf<G>::type ctx = WazCtx<G>::make(a, r);
#if OS_PHASE_TIMING
  if constexpr (std::is_same<G, Go>::value) ctx.sub = ph.c;
#endif
  WaveMtRow bot;
  typename G::State s;
  int sim, depth, nodes_count;
  uint32_t used;
  SearchResult res;
  WazPath path;
  path.p0 = path.p1 = path.p2 = path.p3 = 0;
  if (stage == kAzStart) {
    int p = kMtN;
    bool in_lds = false;
    if (a.import_mt) {
      p = a.mt_pos_in[r];
    } else {
      if (l == 0) mt_seed(mt_lds, a.bot_seeds[r]);  // init_genrand: twisted at the first draw
      __syncthreads();
      in_lds = true;
    }
    bot.init_row(a.mt + r * kMtN, mt_lds, p, in_lds);
    if (l == 0) {
      Node<double> z;
      z.first = 0; z.n = 0; z.w = 0.0; z.action = 0; z.nchild = 0; z.out = kUnsolved;
      nodes[0] = z;
      prior[0] = 1.0;  // SearchNode(kInvalidAction, player_id, 1) (mcts.cc:328)
    }
    __threadfence_block();
    sim = 0;
    depth = 0;
    nodes_count = 1;
    used = 1;
    res.status = kOk;
    res.sims = res.nodes = res.gc_runs = res.max_depth = 0;
    res.used = res.scanned = res.backed = res.expanded = res.solver_scanned = 0;
    res.rng_words = res.pad = 0;
    s = root;
  } else {
    bot.init_row(a.mt + r * kMtN, mt_lds, __builtin_amdgcn_readfirstlane(sl.mt_idx), false);
    s = make_uniform(sl.s);
    sim = __builtin_amdgcn_readfirstlane(sl.sim);
    depth = __builtin_amdgcn_readfirstlane(sl.depth);
    nodes_count = __builtin_amdgcn_readfirstlane(sl.nodes_count);
    used = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sl.used)));
    res = make_uniform(sl.res);
#if OS_WAVE_TIMES
    wt_on = sim == 20;
#endif
    path.p0 = sl.path[l];
    if (depth >= 64) path.p1 = sl.path[64 + l];
    if (depth >= 128) path.p2 = sl.path[128 + l];
    if (depth >= 192) path.p3 = sl.path[192 + l];
    WazCtx<G>::load_tail(ctx, sl);
  }
  int phase;  // 0 new simulation, 1 descend, 2 expand with priors, 3 value ready, -1 stop
  double v0 = 0.0;
  bool solved = false;
  bool from_raw = false;  // phase 2 takes the parked priors of a fused request
  uint32_t parked_first = 0;
  int request = kAzNone;
  // The node being descended from / expanded: index and its (first, n, nchild).
  uint32_t cur_x = 0, cur_first = 0;
  int32_t cur_n = 0;
  int cur_nc = 0;

  auto legal_lanes = [&](const typename G::Legal& lg, LaneArr& acts) {
    const int nc = lg.count;
    const int k0 = WaveKth<G>::kth(lg, l);
    acts.a0 = l < nc ? static_cast<uint32_t>(k0) : 0u;
    acts.a1 = l + 64 < nc ? static_cast<uint32_t>(lg.kth(l + 64)) : 0u;
  };
  auto reload_cur = [&](uint32_t x) {
    const Node<double> nx = nodes[x];
    cur_x = x;
    cur_first = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(nx.first)));
    cur_n = __builtin_amdgcn_readfirstlane(nx.n);
    cur_nc = __builtin_amdgcn_readfirstlane(nx.nchild);
  };

  if (stage == kAzStart) {
    phase = 0;
  } else if (stage == kAzWaitPrior) {
    phase = 2;
    WAZ_CHECK(path.at(depth) < cap, 1);
    reload_cur(path.at(depth));
  } else {
    v0 = a.value_in[r];
    phase = 3;
    if (raw != nullptr) {
      // Park the leaf's priors (legal order) where its children will live.
      const typename G::Legal lg = G::legal(s, g, ctx);
      const int nc = lg.count;
      if (used + static_cast<uint32_t>(nc) > cap) {
        res.status = kArenaOverflow;
        phase = -1;
      } else {
        LaneArr acts;
        legal_lanes(lg, acts);
        WAZ_CHECK(l >= nc || acts.a0 < static_cast<uint32_t>(A), 2);
        WAZ_CHECK(l + 64 >= nc || acts.a1 < static_cast<uint32_t>(A), 3);
        // The leaf's index is read across lanes BEFORE the lane-0 store: a
        // readlane inside an exec-masked region reads a value the masked
        // lanes never computed.
        const uint32_t leaf = path.at(depth);
        WAZ_CHECK(leaf < cap, 4);
        if (l < nc) raw[used + l] = pin[acts.a0];
        if (l + 64 < nc) raw[used + l + 64] = pin[acts.a1];
        if (l == 0) nodes[leaf].first = used;
        used += nc;
        __threadfence_block();
      }
    }
  }
  WAZ_PH(kPhRollout);
  for (;;) {
    if (phase < 0) break;
    if (phase == 0) {
      if (sim >= sp.max_simulations) break;
      s = root;
      ctx.reset();
      depth = 0;
      path.set(0, 0u);
      reload_cur(0);
      phase = 1;
    }
    if (phase == 2) {
      // Prior of the pending node (legal order), shuffled with the bot rng
      // like std::shuffle over (action, prior) pairs (mcts.cc:275-282).
      const typename G::Legal lg = G::legal(s, g, ctx);
      const int nc = lg.count;
      if (!from_raw && used + static_cast<uint32_t>(nc) > cap) {
        res.status = kArenaOverflow;
        break;
      }
      const bool noisy = cur_x == 0 && a.noise != nullptr;
      if (noisy) {  // dirichlet_noise consumed these words of rng_ (mcts.cc:265-267)
        const int skip = a.noise_skip[r];
        for (int i = 0; i < skip; ++i) bot.next();
      }
      LaneArr acts, perm;
      legal_lanes(lg, acts);
      perm.a0 = static_cast<uint32_t>(l);
      perm.a1 = static_cast<uint32_t>(l + 64);
      if (a.np_policy)  // mcts.py:320
        wave_shuffle<kPolicyNumpy, WaveMtRow, !std::is_same<G, Go>::value>(perm, nc, bot);
      else wave_shuffle<kPolicyCpp>(perm, nc, bot);
      const uint32_t first = from_raw ? parked_first : used;
      WAZ_CHECK(nc >= 1 && nc <= 128, 5);
      WAZ_CHECK(first + static_cast<uint32_t>(nc) <= cap, 6);
      WAZ_CHECK(cur_x < cap, 7);
      WAZ_CHECK(l >= nc || perm.a0 < static_cast<uint32_t>(nc), 8);
      WAZ_CHECK(l + 64 >= nc || perm.a1 < static_cast<uint32_t>(nc), 9);
      WAZ_CHECK(l >= nc || acts.a0 < static_cast<uint32_t>(A), 10);
      const double* noise = a.noise ? a.noise + r * a.noise_stride : nullptr;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = l + 64 * h;
        const int j = static_cast<int>(h == 0 ? perm.a0 : perm.a1);
        const uint32_t x0 = static_cast<uint32_t>(__shfl(static_cast<int>(acts.a0), j & 63));
        const uint32_t x1 = static_cast<uint32_t>(__shfl(static_cast<int>(acts.a1), j & 63));
        const int act = static_cast<int>(j < 64 ? x0 : x1);
        if (k < nc) {
          const double p = from_raw ? raw[first + j] : pin[act];
          Node<double> c;
          c.first = 0; c.n = 0; c.w = 0.0; c.action = static_cast<uint16_t>(act);
          c.nchild = 0; c.out = kUnsolved;
          nodes[first + k] = c;
          // (1 - eps) * p + eps * noise, separately rounded (mcts.cc:269-271)
          prior[first + k] = noisy ? (1.0 - a.noise_eps) * p + a.noise_eps * noise[j] : p;
        }
      }
      if (l == 0) {
        nodes[cur_x].first = first;
        nodes[cur_x].nchild = static_cast<uint8_t>(nc);
      }
      __threadfence_block();
      if (!from_raw) used += nc;
      from_raw = false;
      nodes_count += nc;
      res.expanded += nc;
      cur_first = first;
      cur_nc = nc;
      phase = 1;
      WAZ_PH(kPhExpand);
    }
    if (phase == 1) {
      for (;;) {
        if (G::terminal(s, g) || cur_n <= 0) break;
        if (cur_nc == 0 && raw != nullptr && cur_first != 0) {
          from_raw = true;  // parked by this node's fused request: expand now
          parked_first = cur_first;
          break;
        }
        if (cur_nc == 0) {
          request = kAzPrior;
          break;
        }
        // ---- selection: lane k scores child k (and k + 64) ----
        WAZ_CHECK(cur_first + static_cast<uint32_t>(cur_nc) <= cap, 11);
        const int cp = P0 ^ (depth & 1);
        const bool in0 = l < cur_nc, in1 = l + 64 < cur_nc;
        const Node<double> c0 = nodes[cur_first + (in0 ? l : 0)];
        const Node<double> c1 = nodes[cur_first + (in1 ? l + 64 : 0)];
        double v0s, v1s;
        if constexpr (kPuct) {  // mcts.cc:102-111
          const double sqrtN = __builtin_sqrt(static_cast<double>(cur_n));
          const double pr0 = prior[cur_first + (in0 ? l : 0)];
          const double pr1 = prior[cur_first + (in1 ? l + 64 : 0)];
          const double q0 = c0.n != 0 ? c0.w / static_cast<double>(c0.n) : 0.0;
          const double q1 = c1.n != 0 ? c1.w / static_cast<double>(c1.n) : 0.0;
          double u0 = q0 + sp.uct_c * pr0 * sqrtN / static_cast<double>(c0.n + 1);
          double u1 = q1 + sp.uct_c * pr1 * sqrtN / static_cast<double>(c1.n + 1);
          u0 = c0.out != kUnsolved ? outcome_for(c0.out, cp) : u0;
          u1 = c1.out != kUnsolved ? outcome_for(c1.out, cp) : u1;
          v0s = in0 ? u0 : -inf;
          v1s = in1 ? u1 : -inf;
        } else {  // mcts.cc:89-100
          const double logN = sp.log_lut[cur_n];
          v0s = uct_value_sel(c0, in0, cp, logN, sp.uct_c);
          v1s = uct_value_sel(c1, in1, cp, logN, sp.uct_c);
        }
        const int chosen = wave_argmax2<64, true>(v0s, v1s);
        WAZ_CHECK(chosen >= 0 && chosen < cur_nc, 12);
        res.scanned += cur_nc;
        const int src = chosen & 63;
        const Node<double> bc = chosen >= 64 ? c1 : c0;
        const int act = static_cast<int>(rl32(bc.action, src));
        const uint32_t ci = cur_first + static_cast<uint32_t>(chosen);
        cur_x = ci;
        cur_first = rl32(bc.first, src);
        cur_n = rli(bc.n, src);
        cur_nc = rli(bc.nchild, src);
        G::apply(s, g, ctx, act);
        if (++depth >= kMaxPath) {
          res.status = kPathOverflow;
          break;
        }
        path.set(depth, ci);
      }
      WAZ_PH(kPhSelect);
      if (res.status != kOk) break;
      if (from_raw) {
        phase = 2;
        continue;
      }
      if (request != kAzNone) break;
      if (depth > res.max_depth) res.max_depth = depth;
      if (G::terminal(s, g)) {
        WAZ_CHECK(cur_x < cap, 13);
        const int r0 = G::ret0(s, g, ctx);
        if (l == 0) nodes[cur_x].out = static_cast<int8_t>(r0);
        __threadfence_block();
        solved = sp.solve != 0;
        v0 = static_cast<double>(r0);
        phase = 3;
      } else {
        request = raw != nullptr ? kAzBoth : kAzValue;
        break;
      }
    }
    if (phase == 3) {
      // ---- backup (mcts.cc:351-357): lane d updates path node d ----
      WAZ_CHECK(path.p0 < cap || l > depth, 14);
      WAZ_CHECK(path.p1 < cap || 64 + l > depth, 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = 64 * j + l;
        const uint32_t x = j == 0 ? path.p0 : (j == 1 ? path.p1 : (j == 2 ? path.p2 : path.p3));
        if (d <= depth) {
          const int pl = d == 0 ? P0 : (P0 ^ ((d - 1) & 1));
          Node<double>& nd = nodes[x];
          nd.w = nd.w + (pl == 0 ? v0 : -v0);
          nd.n = nd.n + 1;
        }
      }
      __threadfence_block();
      res.backed += depth + 1;
      // ---- MCTS-Solver (mcts.cc:359-395), from the leaf's parent upward ----
      if (solved) {
        for (int d = depth; d >= 0; --d) {
          const uint32_t x = path.at(d);
          const Node<double> nd = nodes[x];
          const int nc = __builtin_amdgcn_readfirstlane(nd.nchild);
          if (nc <= 0) continue;
          const uint32_t f = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(nd.first)));
          WAZ_CHECK(f + static_cast<uint32_t>(nc) <= cap, 16);
          const int cpl = P0 ^ (d & 1);
          res.solver_scanned += nc;
          const bool in0 = l < nc, in1 = l + 64 < nc;
          const int8_t o0 = in0 ? nodes[f + l].out : kUnsolved;
          const int8_t o1 = in1 ? nodes[f + l + 64].out : kUnsolved;
          const bool un0 = in0 && o0 == kUnsolved, un1 = in1 && o1 == kUnsolved;
          const bool all_solved = (ballot(un0) | ballot(un1)) == 0;
          // the first solved child with the largest value for the mover
          const double w0 = in0 && o0 != kUnsolved ? outcome_for(o0, cpl) : -inf;
          const double w1 = in1 && o1 != kUnsolved ? outcome_for(o1, cpl) : -inf;
          const double m = wave_max_f64<64>(fmax(w0, w1));
          if (m == -inf) {
            solved = false;
            break;
          }
          const uint64_t b0 = ballot(w0 == m);
          const int bi = b0 ? ctz64(b0) : 64 + ctz64(ballot(w1 == m));
          const int8_t bo = static_cast<int8_t>(rli(bi < 64 ? o0 : o1, bi & 63));
          if (all_solved || m == 1.0) {
            if (l == 0) nodes[x].out = bo;
            __threadfence_block();
          } else {
            solved = false;
            break;
          }
        }
      }
      sim += 1;
      res.sims = sim;
      const Node<double> rt = nodes[0];
      const int rout = __builtin_amdgcn_readfirstlane(rt.out);
      const int rnc = __builtin_amdgcn_readfirstlane(rt.nchild);
      WAZ_PH(kPhBackup);
      // mcts.cc:398-401; mcts.py:440-441 stops on a solved root only
      if (rout != kUnsolved || (rnc == 1 && !a.np_policy)) break;
      phase = 0;
    }
  }
  if (request != kAzNone && res.status == kOk) {
    // ---- save the continuation, write the request ----
    res.rng_words += bot.words.get();
    const int mt_pos = bot.export_pos();
    if (l == 0) {
      sl.s = s;
      sl.stage = request == kAzPrior ? kAzWaitPrior : kAzWaitValue;
      sl.sim = sim;
      sl.depth = depth;
      sl.nodes_count = nodes_count;
      sl.used = used;
      sl.mt_idx = mt_pos;
      sl.res = res;
    }
    const uint32_t ps[4] = {path.p0, path.p1, path.p2, path.p3};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (64 * j + l <= depth) sl.path[64 * j + l] = ps[j];
    WazCtx<G>::save_tail(ctx, sl);
    bot.save();
    const int cells = g.rows * g.cols;
    const int osz = a.obs_size;
    const int p = G::to_move(s);
    float* o = a.obs + r * static_cast<int64_t>(osz);
    for (int i = l; i < osz; i += 64) o[i] = G::obs(s, g, p, i / cells, i % cells);
    uint8_t* lm = a.legal + r * static_cast<int64_t>(A);
    for (int i = l; i < A; i += 64) lm[i] = 0;
    __threadfence_block();
    const typename G::Legal lg = G::legal(s, g, ctx);
    LaneArr acts;
    legal_lanes(lg, acts);
    WAZ_CHECK(l >= lg.count || acts.a0 < static_cast<uint32_t>(A), 17);
    if (l < lg.count) lm[acts.a0] = 1;
    if (l + 64 < lg.count) lm[acts.a1] = 1;
    if (l == 0) {
      a.kind[r] = request;
      atomicAdd(a.shards + (r % kAzShards) * kAzShardStride, 1);
    }
#if OS_PHASE_TIMING
    WAZ_PH(kPhTail);
    ph_flush();
#endif
#if OS_WAVE_TIMES
    wt_flush();
#endif
    return;
  }
  // ---- finished (or failed): publish the root's children ----
#if OS_WAZ_CHECK
finish:
#endif
  res.nodes = nodes_count;
  res.used = used;
  res.rng_words += bot.words.get();
  bot.save();
  if (l == 0) {
    sl.stage = kAzDone;
    sl.res = res;
    a.kind[r] = kAzNone;
  }
  const int mt_end = bot.export_pos();
  if (a.import_mt && l == 0) a.mt_pos_out[r] = mt_end;
  __threadfence_block();
  const Node<double> rn = nodes[0];
  const int nc = __builtin_amdgcn_readfirstlane(rn.nchild);
  const uint32_t rf = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(rn.first)));
  const int64_t ob = r * a.max_children;
  for (int k = l; k < nc && k < a.max_children; k += 64) {
    const Node<double> c = nodes[rf + k];
    a.child_action[ob + k] = c.action;
    a.child_n[ob + k] = c.n;
    a.child_w[ob + k] = c.w;
    a.child_out[ob + k] =
        c.out == kUnsolved ? kUnsolved : static_cast<int8_t>(P0 == 0 ? c.out : -c.out);
  }
  if (l == 0) {
    a.results[r] = res;
    a.nchild[r] = nc;
    a.root_n[r] = rn.n;
    a.root_w[r] = rn.w;
    a.root_out[r] = rn.out == kUnsolved ? kUnsolved
                                        : static_cast<int8_t>(P0 == 0 ? rn.out : -rn.out);
    const int b = best_child(nodes, P0);
    a.best_action[r] = b < 0 ? -1 : nodes[rn.first + b].action;
  }
#if OS_PHASE_TIMING
  WAZ_PH(kPhTail);
  ph_flush();
#endif
#if OS_WAVE_TIMES
  wt_flush();
#endif
}
#undef WAZ_PH


// OS_ROLL_BLOOM: go playouts screen the superko log with a per-lane Bloom
// filter in LDS (GoCtxBloom); 0: stone-count buckets (GoCtx).  Measured on C5
// (profiles/r04/ab_go.md): 1 = 21.4 ms, 0 = 14.7 ms, both bit-exact -- the
// buckets stay the default.
#ifndef OS_ROLL_BLOOM
#define OS_ROLL_BLOOM 0
#endif
template <class G>
struct RollCtx {
  using type = NoCtx;
  static constexpr int kLdsWords = 1;
  __device__ static NoCtx make(const RollArgs&, int64_t, uint32_t*) { return NoCtx(); }
};
#if OS_ROLL_BLOOM
template <>
struct RollCtx<Go> {
  using type = GoCtxBloom;
  static constexpr int kLdsWords = GoCtxBloom::kWords * 64;
  __device__ static GoCtxBloom make(const RollArgs& a, int64_t i, uint32_t* lds) {
    GoCtxBloom c;
    c.zob = a.zob;
    c.base = a.root_hashes;
    c.n_base = a.n_root_hashes;
#if OS_ROLL_AOS & 2
    c.log = a.glog + i * kGoLogCap;
    c.stride = 1;
#else
    c.log = a.glog + i;
    c.stride = static_cast<int32_t>(a.n);
#endif
    c.filt = lds + (threadIdx.x & 63);
    c.filt_stride = 64;
    c.cap = kGoLogCap;
    c.init_filters();
    return c;
  }
};
#else
template <>
struct RollCtx<Go> {
  using type = GoCtxT<uint8_t, uint16_t>;  // never rewound: 16-bit links
  // heads (cells + 1 bytes per lane), then the log's Bloom filter
  // (OS_GO_LOG_BLOOM): launched with RollLdsBytes of dynamic LDS.
  static constexpr int kLdsWords = (kGoHeads * 64 + 3) / 4 + GoCtx::kBloomWords * 64;
  // The bucket heads are the only per-move accesses that differ across the
  // lanes (each lane is at its own stone count): they live in LDS, lane-
  // interleaved ([count][64] bytes); the log and links stay batch-SoA in HBM.
  __device__ static type make(const RollArgs& a, int64_t i, uint32_t* lds) {
    return make_bw<16>(a, i, lds);
  }
  // The same context with a kBW-word Bloom filter (k_rollouts' small batches).
  template <int kBW>
  __device__ static GoCtxT<uint8_t, uint16_t, kBW> make_bw(const RollArgs& a, int64_t i,
                                                           uint32_t* lds) {
    uint8_t* lds_heads = reinterpret_cast<uint8_t*>(lds);
    uint16_t* glink = reinterpret_cast<uint16_t*>(a.glink);
    GoCtxT<uint8_t, uint16_t, kBW> c;
    c.zob = a.zob;
    c.base = a.root_hashes;
    c.n_base = a.n_root_hashes;
#if OS_ROLL_AOS & 2
    c.log = a.glog + i * kGoLogCap;
    c.link = glink + i * kGoLogCap;
    c.stride = 1;
#else
    c.log = a.glog + i;
    c.link = glink + i;
    c.stride = static_cast<int32_t>(a.n);
#endif
    c.head = lds_heads + (threadIdx.x & 63);
    c.head_stride = 64;
#if OS_GO_LOG_BLOOM
    c.bloom = lds + (((a.cfg.rows * a.cfg.cols + 1) * 64 + 3) / 4) + (threadIdx.x & 63);
#endif
    c.n_log = 0;
    c.cap = kGoLogCap;
    c.n_heads = a.cfg.rows * a.cfg.cols + 1;
    c.init_filters();
    return c;
  }
};
#endif

template <>
struct RollCtx<Go9> : RollCtx<Go> {};

// k_rollouts' context: batches of at most kRollZobLdsMax playouts (kSmall;
// two waves per SIMD, LDS to spare) give go 9 x 9 a 1024-bit superko-log
// Bloom filter, as the lane search has (GoCtxLs: fewer lanes walking a bucket
// while their wave waits); larger batches keep 512 bits and four resident
// waves per SIMD.  OS_ROLL_BLOOM1K=0: 512 bits everywhere (A/B knob).
#ifndef OS_ROLL_BLOOM1K
#define OS_ROLL_BLOOM1K 1
#endif
template <class G, bool kSmall>
struct RollCtxOf {
  using type = typename RollCtx<G>::type;
  static constexpr int kBloomWords = GoCtx::kBloomWords;
  __device__ static type make(const RollArgs& a, int64_t i, uint32_t* lds) {
    return RollCtx<G>::make(a, i, lds);
  }
};
#if !OS_ROLL_BLOOM
template <>
struct RollCtxOf<Go9, true> {
  static constexpr int kBloomWords = OS_ROLL_BLOOM1K ? 32 : 16;
  using type = GoCtxT<uint8_t, uint16_t, kBloomWords>;
  __device__ static type make(const RollArgs& a, int64_t i, uint32_t* lds) {
    return RollCtx<Go>::make_bw<kBloomWords>(a, i, lds);
  }
};
#endif

template <class G>
struct WaveRollCtx {
  __device__ static NoCtx make(const RollArgs&) { return NoCtx(); }
};
template <>
struct WaveRollCtx<Go> {
  __device__ static GoWaveCtx make(const RollArgs& a) {
    GoWaveCtx c;
    c.zob = a.zob;
    c.base = a.root_hashes;
    c.n_base = a.n_root_hashes;
    c.init_filters();
    return c;
  }
};

// One wave per RandomRolloutEvaluator (n_rollouts playouts from the root).
template <class G>
__global__ __launch_bounds__(64) void k_wrollouts(RollArgs a) {
  const int64_t i = blockIdx.x;
  if (i >= a.n) return;
  __shared__ uint32_t mt[kMtN];
  WaveMt ev;
  ev.s = mt;
  ev.use7 = SmallAbsl<G>::value ? 1 : 0;
  if (lane_id() == 0) mt_seed(mt, a.seeds[i]);
  __syncthreads();
  ev.init_seeded();
  typename WaveCtxOf<G>::type ctx = WaveRollCtx<G>::make(a);
  const typename G::State root = make_uniform(*static_cast<const typename G::State*>(a.root));
  double s0 = 0.0, s1 = 0.0;
  for (int k = 0; k < a.n_rollouts; ++k) {
    ctx.reset();
    const int r0 = wave_rollout<G, kPolicyCpp>(root, a.cfg, ctx, ev);
    s0 += static_cast<double>(r0);
    s1 += static_cast<double>(-r0);
  }
  if (lane_id() == 0) {
    a.out[2 * i] = s0 / a.n_rollouts;
    a.out[2 * i + 1] = s1 / a.n_rollouts;
  }
}

// One lane per RandomRolloutEvaluator.  The lanes of a wave start together
// and draw two words per move in lockstep, so the MT19937 states and go's
// position logs are batch-SoA in HBM: one contiguous line per word / entry.
// A/B switch for the C5 traffic study: bit 0 keeps each playout's MT state
// contiguous ([n][624]), bit 1 its position log ([n][kGoLogCap]).
#ifndef OS_ROLL_AOS
#define OS_ROLL_AOS 0
#endif
// Minimum waves per SIMD asked of k_rollouts' register allocation (A/B knob).
#ifndef OS_ROLL_OCC
#define OS_ROLL_OCC 1
#endif
// kZob: go's Zobrist table staged in LDS by each block (every move of every
// lane reads it) instead of read through the caches.  It pays where few
// waves share a SIMD and each load's latency is exposed: C5's per-rank share
// (131072 playouts, two waves per SIMD) 2.31 -> 2.13 ms; at 2^20 (four
// resident, sixteen per SIMD in all) the per-block fill costs more than it
// saves, 10.59 -> 10.73 ms (profiles/r06/zob/).  RollLaunch picks it by size.
constexpr int64_t kRollZobLdsMax = 131072;
template <class G, bool kZob>
__global__ __launch_bounds__(64, OS_ROLL_OCC) void k_rollouts(RollArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  constexpr bool kZobLds = kZob && IsLaneGo<G>::value;
  __shared__ uint64_t zob_lds[kZobLds ? LsCaps<G>::zob : 1];
  if constexpr (kZobLds) {  // before any lane leaves: the whole block loads it
    const int nz = 2 * a.cfg.rows * a.cfg.cols;
    for (int z = threadIdx.x; z < nz; z += blockDim.x) zob_lds[z] = a.zob[z];
    __syncthreads();
  }
  if (i >= a.n) return;
  // OS_ROLL_MT (A/B): 0 MtStreamSoA, 1 MtStreamReg (first block from seed
  // cursors alone: no MT traffic below 624 words, more VALU), 2 MtStreamPf.
#ifndef OS_ROLL_MT
#define OS_ROLL_MT 0
#endif
#if OS_ROLL_MT == 1
  using RollMt = MtStreamReg;
#elif OS_ROLL_MT == 2
  using RollMt = MtStreamPf;
#else
  using RollMt = MtStreamSoA;
#endif
#if OS_ROLL_AOS & 1
  RollMt ev{a.mt + i * kMtN, 1, 0, 0};
#else
  RollMt ev{a.mt + i, a.n, 0, 0};
#endif
  ev.seed(a.seeds[i]);
  extern __shared__ uint32_t roll_lds[];  // RollLdsBytes<G>(cfg) bytes
  typename RollCtxOf<G, kZob>::type ctx = RollCtxOf<G, kZob>::make(a, i, roll_lds);
  if constexpr (kZobLds) ctx.zob = zob_lds;
  const typename G::State root = LaneRoot<G>::load(a.root, 0);
  double s0 = 0.0, s1 = 0.0;
  uint32_t moves = 0;
  for (int k = 0; k < a.n_rollouts; ++k) {
    ctx.reset();
    if constexpr (HasChance<G>::value) {
      const int r0 = rollout_ret0_chance<G, kPolicyCpp>(root, a.cfg, ctx, ev);
      s0 += static_cast<double>(r0);
      s1 += static_cast<double>(-r0);
      continue;
    }
    // rollout_ret0 (mcts.cc:46-55), counting the moves for the byte model.
    typename G::State s = root;
    while (!G::terminal(s, a.cfg)) {
      const typename G::Legal l = G::legal(s, a.cfg, ctx);
      G::apply(s, a.cfg, ctx, l.kth(static_cast<int>(AbslUniform(ev, static_cast<uint32_t>(l.count)))));
      ++moves;
    }
    const int r0 = G::ret0(s, a.cfg, ctx);
    s0 += static_cast<double>(r0);
    s1 += static_cast<double>(-r0);
  }
  a.out[2 * i] = s0 / a.n_rollouts;
  a.out[2 * i + 1] = s1 / a.n_rollouts;
  a.counters[i] = make_uint2(ev.words, moves);  // (MT words drawn, moves played)
}





// ---------------------------------------------------------------------------
// Launchers (host side of this game's kernels)

template <class R>
size_t LdsPerLane(int path_cap, int child_cap) {
  return static_cast<size_t>(2 * kMtN * 4) + path_cap * sizeof(PathEnt<R>) +
         static_cast<size_t>(child_cap) * 2;
}

template <class G, class R, int Policy, bool kPuct>
int LaunchWaveLdsTree(os_engine* e, DevArgs a, hipStream_t stream, size_t lds) {
  if constexpr (LdsTreeGame<G>::value) {
    auto kfn = &k_wsearch<G, R, Policy, false, kPuct, true>;
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(lds)));
    a.root_base = 0;
    a.num_roots = e->num_roots;  // one chunk (the caller checked chunk_roots)
    hipLaunchKernelGGL(kfn, dim3(static_cast<unsigned>(a.num_roots)), dim3(64), lds, stream, a);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess)
      return Fail(OS_ERR_DEVICE, std::string("k_wsearch launch failed: ") +
                                     hipGetErrorString(err));
    return OS_OK;
  } else {
    (void)e; (void)a; (void)stream; (void)lds;
    return Fail(OS_ERR_UNSUPPORTED, "no LDS-tree kernel for this game");
  }
}

template <class G, class R, int Policy>
int LaunchWaveSearch(os_engine* e, DevArgs a, hipStream_t stream) {
  const size_t lds = WaveLdsBytes<G, R>(a.path_cap);
  if (lds > kLdsBytes) return Fail(OS_ERR_CAPACITY, "wave LDS slice exceeds the CU's LDS");
  // A small batch of a small game: the whole tree in LDS (kLdsTree).
  if (LdsTreeGame<G>::value && a.pages == nullptr && e->num_roots <= kLdsTreeMaxRoots &&
      e->chunk_roots >= e->num_roots && OS_NODE_CACHE == 0) {
    const size_t tree_lds = ((lds + 15) & ~size_t(15)) + static_cast<size_t>(a.cap) * sizeof(Node<R>);
    if (tree_lds <= kLdsBytes)
      return a.sp.puct ? LaunchWaveLdsTree<G, R, Policy, true>(e, a, stream, tree_lds)
                       : LaunchWaveLdsTree<G, R, Policy, false>(e, a, stream, tree_lds);
  }
  // Paged batches run the C++ policy only (SizeArena).
  constexpr bool kCanPage = Policy == kPolicyCpp;
  const bool paged = kCanPage && a.pages != nullptr;
  if (a.pages && !kCanPage) return Fail(OS_ERR_UNSUPPORTED, "paged arena needs the C++ policy");
  // PUCT searches run on the reserved arena only (SizeArena); their kernel
  // is a third instantiation, so the UCT kernels keep their registers.
  const bool puct = a.sp.puct != 0;
  if (puct && paged) return Fail(OS_ERR_UNSUPPORTED, "paged arena with PUCT");
  const void* kfn =
      puct ? reinterpret_cast<const void*>(&k_wsearch<G, R, Policy, false, true>)
           : (paged ? reinterpret_cast<const void*>(&k_wsearch<G, R, Policy, kCanPage, false>)
                    : reinterpret_cast<const void*>(&k_wsearch<G, R, Policy, false, false>));
  HIP_TRY(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds)));
  for (int64_t base = 0; base < e->num_roots; base += e->chunk_roots) {
    const int64_t n = std::min<int64_t>(e->chunk_roots, e->num_roots - base);
    a.root_base = base;
    a.num_roots = n;
    if (puct)
      hipLaunchKernelGGL((k_wsearch<G, R, Policy, false, true>), dim3(static_cast<unsigned>(n)),
                         dim3(64), lds, stream, a);
    else if (paged)
      hipLaunchKernelGGL((k_wsearch<G, R, Policy, kCanPage, false>),
                         dim3(static_cast<unsigned>(n)), dim3(64), lds, stream, a);
    else
      hipLaunchKernelGGL((k_wsearch<G, R, Policy, false, false>), dim3(static_cast<unsigned>(n)),
                         dim3(64), lds, stream, a);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess)
      return Fail(OS_ERR_DEVICE, std::string("k_wsearch launch failed: ") +
                                     hipGetErrorString(err));
  }
  return OS_OK;
}

// Searches per wave of k_lsearch for a chunk of n roots.  Go 9 x 9 .. 11 x 11
// runs 16 lanes per block up to 32768 roots (2048 waves, all resident at two
// per SIMD) and 32 above; boards above 11 x 11 keep 64.  A wave's time is its
// lanes' longest dependent chain plus the union of their divergent paths, so
// narrower waves finish sooner, and they spread a small batch over more SIMDs
// (go9, 256 sims, ms per launch for 16 / 32 / 64 lanes, profiles/r06/g9_lanes:
// 16384 roots 266 / 361 / 408; 32768 roots 332 / 336 / 444; 65536 roots
// 642 / 428 / 442; 131072 roots - / 833 / 881).  block_size (16 / 32 / 64)
// overrides the choice.
template <class G>
int LsLanes(int64_t n, int block_size) {
  if (!IsLaneGo<G>::value) return 64;
  if (block_size == 16 || block_size == 32 || block_size == 64) return block_size;
  return n <= 32768 ? 16 : 32;
}

template <class G, class R>
int LaunchLs(os_engine* e, DevArgs a, hipStream_t stream) {
  if (a.shared_stream)
    return Fail(OS_ERR_UNSUPPORTED, "go's lane layout runs C++-policy bots (separate streams)");
  if ((!LsWide<G>::value && a.child_cap > LsCaps<G>::act) ||
      (G::State::kNeedsLog && 2 * a.cfg.rows * a.cfg.cols > LsCaps<G>::zob))
    return Fail(OS_ERR_UNSUPPORTED, "board too large for k_lsearch");
  for (int64_t base = 0; base < e->num_roots; base += e->chunk_roots) {
    const int64_t n = std::min<int64_t>(e->chunk_roots, e->num_roots - base);
    a.root_base = base;
    a.num_roots = n;
    const int kl = LsLanes<G>(n, e->params.block_size);
    e->search_lanes = kl;
    const unsigned grid = static_cast<unsigned>((n + kl - 1) / kl);
    if constexpr (IsLaneGo<G>::value) {
      if (kl == 16)
        hipLaunchKernelGGL((k_lsearch<G, R, 16, 2>), dim3(grid), dim3(16), 0, stream, a);
      else if (kl == 32)
        hipLaunchKernelGGL((k_lsearch<G, R, 32, 2>), dim3(grid), dim3(32), 0, stream, a);
      else
        hipLaunchKernelGGL((k_lsearch<G, R, 64, 1>), dim3(grid), dim3(64), 0, stream, a);
    } else {
      hipLaunchKernelGGL((k_lsearch<G, R, 64, 1>), dim3(grid), dim3(64), 0, stream, a);
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess)
      return Fail(OS_ERR_DEVICE, std::string("k_lsearch launch failed: ") +
                                     hipGetErrorString(err));
  }
  return OS_OK;
}

// go / hex above 11 x 11: lane-layout C++-policy searches only
// (os_game_go_big.hip, os_game_hex_big.hip).
template <class G>
int LaunchSearchOnly(os_engine* e, const DevArgs& a, hipStream_t stream) {
  if (e->params.layout != OS_LAYOUT_LANE || e->params.policy != OS_POLICY_CPP)
    return Fail(OS_ERR_UNSUPPORTED,
                "go / hex above 11 x 11 run C++-policy searches on the lane layout");
  return e->node_double ? LaunchLs<G, double>(e, a, stream) : LaunchLs<G, int32_t>(e, a, stream);
}

template <class G, class R, int Policy>
int LaunchChanceWave(os_engine* e, DevArgs a, hipStream_t stream) {
  if (a.pages) return Fail(OS_ERR_UNSUPPORTED, "paged arena on the chance-node wave layout");
  const size_t lds = WaveChanceLdsBytes<G, R>(a.path_cap);
  if (lds > kLdsBytes) return Fail(OS_ERR_CAPACITY, "wave LDS slice exceeds the CU's LDS");
  // A small batch whose reserved arenas fit the CU's LDS: the tree in LDS.
  const size_t tree_lds = ChanceTreeLdsOffset<R>(lds) +
                          static_cast<size_t>(a.cap) * sizeof(Node<R>) +
                          static_cast<size_t>(a.sp.max_simulations + 1) * sizeof(double);
  const bool lds_tree = a.pages == nullptr && e->num_roots <= kLdsTreeMaxRoots &&
                        e->chunk_roots >= e->num_roots && tree_lds <= kLdsBytes &&
                        OS_CHANCE_LDS_TREE;
  const void* fn = lds_tree
      ? reinterpret_cast<const void*>(&k_wsearch_chance<G, R, Policy, true>)
      : reinterpret_cast<const void*>(&k_wsearch_chance<G, R, Policy, false>);
  const size_t dyn = lds_tree ? tree_lds : lds;
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(dyn)));
  for (int64_t base = 0; base < e->num_roots; base += e->chunk_roots) {
    const int64_t n = std::min<int64_t>(e->chunk_roots, e->num_roots - base);
    a.root_base = base;
    a.num_roots = n;
    if (lds_tree)
      hipLaunchKernelGGL((k_wsearch_chance<G, R, Policy, true>), dim3(static_cast<unsigned>(n)),
                         dim3(64), dyn, stream, a);
    else
      hipLaunchKernelGGL((k_wsearch_chance<G, R, Policy, false>),
                         dim3(static_cast<unsigned>(n)), dim3(64), dyn, stream, a);
    HIP_TRY(hipGetLastError());
  }
  return OS_OK;
}

template <class G, class R, int Policy>
int LaunchSearch(os_engine* e, DevArgs a, hipStream_t stream) {
  e->search_lanes = 1;  // the wave layouts; the lane launchers below set theirs
  if constexpr (HasChance<G>::value) {
    if (a.path_cap > kChancePathCap) a.path_cap = kChancePathCap;
    if (e->params.layout == OS_LAYOUT_WAVE) {
      // two-player pig: the same search over two-player state arrays (Pig2)
      if constexpr (std::is_same<G, Pig>::value)
        if (a.cfg.pig_players == 2) return LaunchChanceWave<Pig2, R, Policy>(e, a, stream);
      return LaunchChanceWave<G, R, Policy>(e, a, stream);
    }
  } else {
    if (e->params.layout == OS_LAYOUT_WAVE) return LaunchWaveSearch<G, R, Policy>(e, a, stream);
  }
  if constexpr (G::State::kNeedsLog) {
    // go: k_lsearch, per-search buffers in HBM (the LDS-slice kernel k_mcts
    // would hold the superko log in private memory).
    if (Policy != kPolicyCpp) return Fail(OS_ERR_UNSUPPORTED, "k_lsearch runs the C++ policy");
    if constexpr (std::is_same<G, Go>::value)
      if (UseGo9(a.cfg)) return LaunchGo9Search(e, a, stream);  // os_game_go9.hip
    return LaunchLs<G, R>(e, a, stream);
  } else {
  int bs = e->params.block_size > 0 ? e->params.block_size : kDefaultBlock;
  if (bs > 64) bs = 64;  // k_mcts's __launch_bounds__
  const size_t per_lane = LdsPerLane<R>(a.path_cap, a.child_cap);
  if (per_lane * bs > kLdsBytes) bs = static_cast<int>(kLdsBytes / per_lane);
  if (bs < 1) return Fail(OS_ERR_CAPACITY, "per-lane LDS slice exceeds the CU's LDS");
  const size_t lds = per_lane * bs;
  e->search_lanes = bs;
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mcts<G, R, Policy>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds)));
  for (int64_t base = 0; base < e->num_roots; base += e->chunk_roots) {
    const int64_t n = std::min<int64_t>(e->chunk_roots, e->num_roots - base);
    a.root_base = base;
    a.num_roots = n;
    const unsigned grid = static_cast<unsigned>((n + bs - 1) / bs);
    hipLaunchKernelGGL((k_mcts<G, R, Policy>), dim3(grid), dim3(bs), lds, stream, a);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess)
      return Fail(OS_ERR_DEVICE, std::string("k_mcts launch failed: ") +
                                     hipGetErrorString(err));
  }
  return OS_OK;
  }
}

template <class G>
int LaunchForGame(os_engine* e, const DevArgs& a, hipStream_t stream) {
  const bool dbl = e->node_double;
  if (e->params.policy == OS_POLICY_NUMPY) {
    return dbl ? LaunchSearch<G, double, kPolicyNumpy>(e, a, stream)
               : LaunchSearch<G, int32_t, kPolicyNumpy>(e, a, stream);
  }
  return dbl ? LaunchSearch<G, double, kPolicyCpp>(e, a, stream)
             : LaunchSearch<G, int32_t, kPolicyCpp>(e, a, stream);
}

template <class G, class R, bool kPuct>
int SpLaunch(os_engine* e, hipStream_t stream) {
  SpArgs a;
  std::memset(&a, 0, sizeof a);
  a.cfg = e->game.cfg;
  a.sp.uct_c = e->params.uct_c;
  a.sp.max_simulations = e->params.max_simulations;
  a.sp.n_rollouts = e->params.n_rollouts;
  a.sp.solve = e->params.solve;
  a.sp.max_nodes = static_cast<int32_t>((e->params.max_memory_mb << 20) / 80 + 1);
  a.sp.policy = kPolicyCpp;
  a.sp.puct = kPuct ? 1 : 0;
  a.sp.log_lut = static_cast<const double*>(e->d_lut.p);
  a.starts = e->d_roots.p;
  a.bot_seeds = static_cast<const uint32_t*>(e->d_bseed.p);
  a.eval_seeds = static_cast<const uint32_t*>(e->d_eseed.p);
  a.arena = e->d_arena.p;
  a.cap = e->cap;
  a.path_cap = e->game.cfg.max_game_length + 2;
  a.max_len = e->sp_max_len;
  a.num_actions = e->game.cfg.num_actions;
  a.zob = static_cast<const uint64_t*>(e->d_zob.p);
  a.hist = static_cast<uint64_t*>(e->d_rhash.p);
  a.hist_n = static_cast<int32_t*>(e->d_rnh.p);
  a.hash_stride = e->hash_stride;
  a.actions = static_cast<int32_t*>(e->d_sp_act.p);
  a.length = static_cast<int32_t*>(e->d_sp_len.p);
  a.returns = static_cast<double*>(e->d_sp_ret.p);
  a.visits = e->sp_visits ? static_cast<int32_t*>(e->d_sp_vis.p) : nullptr;
  a.obs = e->sp_obs ? static_cast<float*>(e->d_sp_obs.p) : nullptr;
  a.obs_size = ObservationShape(e->game, nullptr);
  a.results = static_cast<SearchResult*>(e->d_res.p);
  const bool actor = !e->sp_actor_seeds.empty();
  a.actor_seeds = actor ? static_cast<const uint32_t*>(e->d_sp_actor.p) : nullptr;
  a.pow_lut = e->sp_opts.temperature > 0.0 ? static_cast<const double*>(e->d_sp_pow.p) : nullptr;
  a.temperature_drop = e->sp_opts.temperature > 0.0 ? e->sp_opts.temperature_drop : 0;
  a.resign = actor && e->sp_opts.resign ? 1 : 0;
  a.cutoff_value = e->sp_opts.cutoff_value;
  a.cutoff_probability = e->sp_opts.cutoff_probability;
  a.max_utility = 1.0;  // every self-play game: Game::MaxUtility() == 1
  a.policy = e->sp_policy ? static_cast<double*>(e->d_sp_pol.p) : nullptr;
  a.root_value = e->sp_values ? static_cast<double*>(e->d_sp_val.p) : nullptr;
  if constexpr (HasChance<G>::value) {
    if (a.path_cap > kChancePathCap) a.path_cap = kChancePathCap;
    const size_t lds = SelfPlayChanceLdsBytes<G, R>(a.path_cap);
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wselfplay_chance<G, R>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(lds)));
    for (int64_t base = 0; base < e->sp_games; base += e->chunk_roots) {
      const int64_t n = std::min<int64_t>(e->chunk_roots, e->sp_games - base);
      a.game_base = base;
      a.num_games = n;
      hipLaunchKernelGGL((k_wselfplay_chance<G, R>), dim3(static_cast<unsigned>(n)), dim3(64),
                         lds, stream, a);
      HIP_TRY(hipGetLastError());
    }
    return OS_OK;
  } else {
  const size_t lds = SelfPlayLdsBytes<G, R>(a.path_cap);
  if (lds > kLdsBytes) return Fail(OS_ERR_CAPACITY, "self-play LDS slice exceeds the CU's LDS");
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wselfplay<G, R, kPuct>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds)));
  for (int64_t base = 0; base < e->sp_games; base += e->chunk_roots) {
    const int64_t n = std::min<int64_t>(e->chunk_roots, e->sp_games - base);
    a.game_base = base;
    a.num_games = n;
    hipLaunchKernelGGL((k_wselfplay<G, R, kPuct>), dim3(static_cast<unsigned>(n)), dim3(64),
                       lds, stream, a);
    HIP_TRY(hipGetLastError());
  }
  return OS_OK;
  }
}

// ---- external-evaluator search (os_az_*) ----
template <class G>
size_t AzSlotBytes() { return sizeof(AzSlot<G>); }

// Sums the step's request shards into *pending and zeroes them (one
// workgroup, one shard per thread); the batch's running request total (an
// int64 after the shards, os_az_requests) grows by the same count.
static __global__ __launch_bounds__(kAzShards) void k_az_pending(int32_t* shards, int32_t* pending) {
  __shared__ int32_t part[kAzShards / 64];
  const int t = threadIdx.x;
  int32_t v = shards[t * kAzShardStride];
  shards[t * kAzShardStride] = 0;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((t & 63) == 0) part[t >> 6] = v;
  __syncthreads();
  if (t == 0) {
    int32_t s = 0;
    for (int i = 0; i < kAzShards / 64; ++i) s += part[i];
    *pending = s;
    *reinterpret_cast<int64_t*>(shards + kAzShards * kAzShardStride) += s;
  }
}

template <class G>
int AzLaunch(os_engine* e, hipStream_t stream) {
  if constexpr (HasChance<G>::value) {
    (void)e;
    (void)stream;
    return Fail(OS_ERR_UNSUPPORTED, "external-evaluator search of games with chance nodes");
  } else {
  AzArgs a;
  std::memset(&a, 0, sizeof a);
  const DevArgs d = MakeArgs(e);
  a.cfg = d.cfg;
  a.sp = d.sp;
  a.puct = e->az_puct;
  a.np_policy = e->az_np;
  a.num_roots = e->num_roots;
  a.roots = d.roots;
  a.slots = e->d_az_slots.p;
  a.arena = static_cast<Node<double>*>(e->d_arena.p);
  a.priors = static_cast<double*>(e->d_az_prior.p);
  a.raw = e->az_fused ? static_cast<double*>(e->d_az_raw.p) : nullptr;
  a.cap = e->cap;
  a.mt = static_cast<uint32_t*>(e->d_mt.p);
  a.bot_seeds = d.bot_seeds;
  a.obs_size = ObservationShape(e->game, nullptr);
  a.num_actions = e->game.cfg.num_actions;
  a.kind = e->az_kind;
  a.obs = e->az_obs;
  a.legal = e->az_legal;
  a.prior_in = e->az_prior;
  a.value_in = e->az_value;
  a.pending = e->az_pending;
  a.shards = static_cast<int32_t*>(e->d_az_shards.p);
  a.import_mt = e->az_import ? 1 : 0;
  a.mt_pos_in = static_cast<const int32_t*>(e->d_az_pos.p);
  a.mt_pos_out = static_cast<int32_t*>(e->d_az_pos.p) + (e->az_import ? e->num_roots : 0);
  if (e->az_noise) {
    a.noise = static_cast<const double*>(e->d_az_noise.p);
    a.noise_skip = static_cast<const int32_t*>(e->d_az_skip.p);
    a.noise_stride = e->game.cfg.max_children;
    a.noise_eps = e->az_eps;
  }
  a.zob = d.zob;
  a.root_hashes = d.root_hashes;
  a.root_nhash = d.root_nhash;
  a.hash_stride = d.hash_stride;
  a.results = d.results;
  a.max_children = d.max_children;
  a.child_action = d.child_action;
  a.child_n = d.child_n;
  a.child_w = d.child_w;
  a.child_out = d.child_out;
  a.nchild = d.nchild;
  a.root_n = d.root_n;
  a.root_w = d.root_w;
  a.root_out = d.root_out;
  a.best_action = d.best_action;
  if (e->num_roots > 0) {
    if (e->az_wave) {  // one wave per search (k_waz_step)
      if (e->az_puct)
        hipLaunchKernelGGL((k_waz_step<G, true>), dim3(static_cast<unsigned>(e->num_roots)),
                           dim3(64), 0, stream, a);
      else
        hipLaunchKernelGGL((k_waz_step<G, false>), dim3(static_cast<unsigned>(e->num_roots)),
                           dim3(64), 0, stream, a);
    } else {
      // Searches per workgroup (one wave): os_mcts_params.block_size, 64 by
      // default.  Fewer lanes per wave spread a small batch over more SIMDs.
      const int bs = e->params.block_size > 0 ? std::min(e->params.block_size, 64) : 64;
      hipLaunchKernelGGL(k_az_step<G>, dim3(static_cast<unsigned>((e->num_roots + bs - 1) / bs)),
                         dim3(bs), 0, stream, a);
    }
    HIP_TRY(hipGetLastError());
  }
  // *pending = the step's request count; the shards are zeroed for the next step.
  hipLaunchKernelGGL(k_az_pending, dim3(1), dim3(kAzShards), 0, stream, a.shards, a.pending);
  HIP_TRY(hipGetLastError());
  return OS_OK;
  }
}

// k_rollouts' dynamic LDS: go's bucket heads for this board size (one byte
// per stone count per lane) and the log's Bloom filter; the heads' static
// bound (11 x 11) would cost occupancy on 9 x 9.
template <class G>
size_t RollLdsBytes(const GameCfg& c, int bloom_words = GoCtx::kBloomWords) {
#if OS_ROLL_BLOOM
  (void)c;
  (void)bloom_words;
  return sizeof(uint32_t) * RollCtx<G>::kLdsWords;
#else
  if constexpr (IsLaneGo<G>::value)
    return 4 * (((c.rows * c.cols + 1) * 64 + 3) / 4 +
                (OS_GO_LOG_BLOOM ? bloom_words * 64 : 0));
  else
    return sizeof(uint32_t) * RollCtx<G>::kLdsWords;
#endif
}

template <class G>
int RollLaunch(os_engine* e, hipStream_t stream) {
  RollArgs a;
  std::memset(&a, 0, sizeof a);
  a.cfg = e->game.cfg;
  a.n = e->roll_n;
  a.n_rollouts = e->roll_nr;
  a.root = e->d_roots.p;
  a.seeds = static_cast<const uint32_t*>(e->d_bseed.p);
  a.mt = static_cast<uint32_t*>(e->d_mt.p);
  a.glog = static_cast<uint64_t*>(e->d_glog.p);
  a.glink = static_cast<uint32_t*>(e->d_glink.p);
  a.counters = static_cast<uint2*>(e->d_roll_cnt.p);
  a.out = static_cast<double*>(e->d_rollout_out.p);
  a.zob = static_cast<const uint64_t*>(e->d_zob.p);
  a.root_hashes = static_cast<const uint64_t*>(e->d_rhash.p);
  a.n_root_hashes = e->roll_nhash;
  const int64_t n = e->roll_n;
  if (e->game.cfg.pig_players > 2)
    return Fail(OS_ERR_UNSUPPORTED, "rollout batches return two players' values");
  if constexpr (!HasChance<G>::value && !std::is_same<G, Go9>::value) {
    if (e->rollout_layout == OS_LAYOUT_WAVE) {
      hipLaunchKernelGGL(k_wrollouts<G>, dim3(static_cast<unsigned>(n)), dim3(64), 0, stream,
                         a);
      HIP_TRY(hipGetLastError());
      return OS_OK;
    }
  }
  if constexpr (std::is_same<G, Go>::value)
    if (UseGo9(a.cfg)) return LaunchGo9Rollouts(e, stream);  // os_game_go9.hip
  {
    // 64 lanes per block: 32-lane blocks (four waves per SIMD at C5's
    // per-rank 131072 playouts instead of two) were slower, 2.36 -> 3.16 ms
    // (profiles/r06/ab_narrow): a wave instruction then serves half as many
    // playouts, and this kernel's VALU is already half busy.
    const int bs = 64;
    const dim3 grid(static_cast<unsigned>((n + bs - 1) / bs));
    if (IsLaneGo<G>::value && n <= kRollZobLdsMax)
      hipLaunchKernelGGL((k_rollouts<G, true>), grid, dim3(bs),
                         RollLdsBytes<G>(a.cfg, RollCtxOf<G, true>::kBloomWords), stream, a);
    else
      hipLaunchKernelGGL((k_rollouts<G, false>), grid, dim3(bs), RollLdsBytes<G>(a.cfg), stream, a);
  }
  HIP_TRY(hipGetLastError());
  return OS_OK;
}

#if OS_PHASE_TIMING || OS_WAVE_TIMES
static int PhaseCycles(uint64_t* out, bool clear) {  // static: per game TU
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_cycles), sizeof(uint64_t) * kDbgSlots));
  if (clear) {
    std::vector<uint64_t> zero(kDbgSlots, 0);
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), zero.data(),
                              sizeof(uint64_t) * kDbgSlots));
  }
  return OS_OK;
}
#else
static int PhaseCycles(uint64_t*, bool) {
  return Fail(OS_ERR_UNSUPPORTED, "built without -DOS_PHASE_TIMING=1");
}
#endif

template <class G>
int SelfPlayEntry(os_engine* e, hipStream_t stream) {
  if constexpr (HasChance<G>::value) {
    // mcts_example.cc PlayGame over two MCTSBots; chance outcomes from the
    // game's rng (actor seeds).  AlphaZero's move choice is not offered here.
    if (e->game.cfg.pig_players != 2)
      return Fail(OS_ERR_UNSUPPORTED, "self-play of chance games runs two players "
                                      "(mcts_example.cc:148-150)");
    if (e->sp_actor_seeds.empty())
      return Fail(OS_ERR_INVALID, "games with chance nodes need os_selfplay_set_options actor "
                                  "seeds: the PlayGame rng that samples chance outcomes");
    if (e->sp_opts.temperature > 0.0 || e->sp_opts.resign || e->sp_policy || e->sp_values)
      return Fail(OS_ERR_UNSUPPORTED, "AlphaZero move choice / targets on chance games");
    const bool puct = e->params.child_selection == OS_SELECT_PUCT;
    if (e->node_double)
      return puct ? SpLaunch<G, double, true>(e, stream) : SpLaunch<G, double, false>(e, stream);
    return puct ? SpLaunch<G, int32_t, true>(e, stream) : SpLaunch<G, int32_t, false>(e, stream);
  } else
  {
    const bool puct = e->params.child_selection == OS_SELECT_PUCT;
    if (e->params.n_rollouts != 1)
      return puct ? SpLaunch<G, double, true>(e, stream) : SpLaunch<G, double, false>(e, stream);
    return puct ? SpLaunch<G, int32_t, true>(e, stream) : SpLaunch<G, int32_t, false>(e, stream);
  }
}

}  // namespace osx

// Defines osx::k<G>Launchers for game G; WITH_AZ = 0 leaves the external-
// evaluator search unsupported for it.
// A non-const host variable: the device pass instantiates the launch code
// (and so every kernel it launches) but does not emit the table itself.
#define OS_DEFINE_SEARCH_ONLY_LAUNCHERS(G)                                            \
  namespace osx {                                                                     \
  extern GameLaunchers k##G##Launchers;                                               \
  GameLaunchers k##G##Launchers = {&LaunchSearchOnly<G>, nullptr, nullptr, nullptr,  \
                                   &PhaseCycles, 0};                                  \
  }

#define OS_DEFINE_LAUNCHERS(G, WITH_AZ)                                          \
  namespace osx {                                                                \
  extern GameLaunchers k##G##Launchers;                                          \
  GameLaunchers k##G##Launchers = {                                              \
      &LaunchForGame<G>, &SelfPlayEntry<G>, (WITH_AZ) ? &AzLaunch<G> : nullptr,  \
      &RollLaunch<G>, &PhaseCycles, (WITH_AZ) ? AzSlotBytes<G>() : 0};           \
  }

#endif  // OS_KERNELS_H_
