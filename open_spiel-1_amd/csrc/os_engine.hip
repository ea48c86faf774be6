// libos_mcts.so — host side of the MI355X MCTS engine and the C-ABI declared
// in include/os_mcts.h.
//
// Execution model: every root is one independent search
// (MCTSBot::MCTSearch, mcts.cc:325-428) with its own flat node arena in HBM.
// This unit prepares batches (root replay, arena sizing, uploads), launches
// the per-game kernels through the launcher table (os_kernels.h,
// os_game_*.hip), fetches results and reports errors.
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <unordered_map>

#include "os_engine_impl.h"

using namespace osm;
using namespace osx;

thread_local std::string osx::g_err;

struct os_game {
  HostGame g;
};
struct os_state {
  HostState s;
};

namespace osx {
namespace {

// Root-parallel reduction: scatter each tree's root
// children to a dense [R][A] action-indexed image, then sum every action's
// column in a fixed order (deterministic, independent of scheduling).
__global__ void k_root_scatter(const int32_t* nchild, const int32_t* cact, const int32_t* cn,
                               const double* cw, int32_t mc, int64_t A, int32_t* dn,
                               double* dw) {
  const int64_t r = blockIdx.x;
  const int nc = nchild[r];
  for (int k = threadIdx.x; k < nc && k < mc; k += blockDim.x) {
    const int32_t act = cact[r * mc + k];
    if (act >= 0 && act < A) {
      dn[r * A + act] = cn[r * mc + k];
      dw[r * A + act] = cw[r * mc + k];
    }
  }
}

__global__ __launch_bounds__(256) void k_root_reduce(const int32_t* dn, const double* dw,
                                                     int64_t R, int64_t A, int64_t* visits,
                                                     double* rewards) {
  __shared__ int64_t sn[256];
  __shared__ double sw[256];
  const int64_t a = blockIdx.x;
  const int t = threadIdx.x;
  int64_t n = 0;
  double w = 0.0;
  for (int64_t r = t; r < R; r += 256) {
    n += dn[r * A + a];
    w += dw[r * A + a];
  }
  sn[t] = n;
  sw[t] = w;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if (t < s) {
      sn[t] += sn[t + s];
      sw[t] += sw[t + s];
    }
    __syncthreads();
  }
  if (t == 0) {
    visits[a] = sn[0];
    rewards[a] = sw[0];
  }
}

// Per-device root sums [ndev][A] (visits, then rewards) added in device order.
__global__ void k_sum_devices(const int64_t* n, const double* w, int32_t ndev, int64_t A,
                              int64_t* visits, double* rewards) {
  const int64_t a = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (a >= A) return;
  int64_t sn = 0;
  double sw = 0.0;
  for (int g = 0; g < ndev; ++g) {
    sn += n[g * A + a];
    sw += w[g * A + a];
  }
  visits[a] = sn;
  rewards[a] = sw;
}

// Outcome counts of a rollout batch: [0] player 0 ahead, [1] player 1 ahead,
// [2] draws (sign of the mean player-0 return of each evaluator).  Grid-stride
// counting, a wave then a workgroup reduction, one atomic per counter per
// workgroup (integer sums: order-independent).
__global__ __launch_bounds__(256) void k_outcome_counts(const double* out, int64_t n,
                                                        unsigned long long* counts) {
  __shared__ unsigned long long part[3][4];
  unsigned long long c0 = 0, c1 = 0, c2 = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const double v = out[2 * i];
    c0 += v > 0.0;
    c1 += v < 0.0;
    c2 += v == 0.0;
  }
  for (int off = 32; off >= 1; off >>= 1) {
    c0 += __shfl_xor(c0, off);
    c1 += __shfl_xor(c1, off);
    c2 += __shfl_xor(c2, off);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][w] = c0;
    part[1][w] = c1;
    part[2][w] = c2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const unsigned long long t = part[threadIdx.x][0] + part[threadIdx.x][1] +
                                 part[threadIdx.x][2] + part[threadIdx.x][3];
    atomicAdd(&counts[threadIdx.x], t);
  }
}


}  // namespace

DevArgs MakeArgs(os_engine* e) {
  DevArgs a;
  std::memset(&a, 0, sizeof a);
  a.cfg = e->game.cfg;
  a.sp.uct_c = e->params.uct_c;
  a.sp.max_simulations = e->params.max_simulations;
  a.sp.n_rollouts = e->params.n_rollouts;
  a.sp.solve = e->params.solve;
  // mcts.cc:201: max_nodes_ = (max_memory_mb << 20) / sizeof(SearchNode) + 1,
  // with sizeof(SearchNode) == 80 on LP64 libstdc++.
  const int64_t mn = (e->params.max_memory_mb << 20) / 80 + 1;
  a.sp.max_nodes = static_cast<int32_t>(mn);
  a.sp.policy = e->params.policy;
  a.sp.puct = e->params.child_selection == OS_SELECT_PUCT ? 1 : 0;
  a.sp.log_lut = static_cast<const double*>(e->d_lut.p);
  a.roots = e->d_roots.p;
  a.bot_seeds = static_cast<const uint32_t*>(e->d_bseed.p);
  a.eval_seeds = static_cast<const uint32_t*>(e->d_eseed.p);
  a.mt = static_cast<uint32_t*>(e->d_mt.p);
  a.arena = e->d_arena.p;
  a.cap = e->cap;
  a.pages = e->paged ? static_cast<uint32_t*>(e->d_page_next.p) : nullptr;
  // Paths hold depth + 1 <= MaxGameLength + 1 nodes; keep slices 4-byte even.
  a.path_cap = e->game.cfg.max_game_length + 2;
  a.child_cap = (e->game.cfg.max_children + 1) & ~1;
  a.import_state = e->import_state ? 1 : 0;
  a.shared_stream = e->shared_stream ? 1 : 0;
  a.mt_pos = static_cast<int32_t*>(e->d_pos.p);
  a.zob = static_cast<const uint64_t*>(e->d_zob.p);
  a.root_hashes = static_cast<const uint64_t*>(e->d_rhash.p);
  a.root_nhash = static_cast<const int32_t*>(e->d_rnh.p);
  a.hash_stride = e->hash_stride;
  a.lstride = e->chunk_roots;
  a.lpath = e->d_lpath.p;
  // k_lsearch writes each search's log row in whole 8-entry groups with
  // 16-byte stores (GoCtxT::flush_group): rows of kGoLogCap entries keep
  // every group 64 B (hashes) / 32 B (links) aligned.
  static_assert(kGoLogCap % GoCtx::kWg == 0, "log rows of whole write groups");
  a.lglog = static_cast<uint64_t*>(e->d_glog.p);
  a.lglink = static_cast<uint32_t*>(e->d_glink.p);
  a.lheads = static_cast<uint16_t*>(e->d_lheads.p);
  a.lact = static_cast<uint16_t*>(e->d_lact.p);
  a.results = static_cast<SearchResult*>(e->d_res.p);
  a.max_children = e->max_children;
  a.child_action = static_cast<int32_t*>(e->d_cact.p);
  a.child_n = static_cast<int32_t*>(e->d_cn.p);
  a.child_w = static_cast<double*>(e->d_cw.p);
  a.child_out = static_cast<int8_t*>(e->d_cout.p);
  a.nchild = static_cast<int32_t*>(e->d_nch.p);
  a.root_n = static_cast<int32_t*>(e->d_rn.p);
  a.root_w = static_cast<double*>(e->d_rw.p);
  a.root_out = static_cast<int8_t*>(e->d_rout.p);
  a.best_action = static_cast<int64_t*>(e->d_best.p);
  return a;
}

}  // namespace osx

namespace {



// Replays a history on the host; returns false if an action is illegal.
bool ReplayRoot(const HostGame& g, const int64_t* a, int64_t n, HostState* s,
                std::string* err) {
  s->game = &g;
  StateInit(s);
  for (int64_t i = 0; i < n; ++i) {
    if (!StateApply(s, a[i])) {
      *err = "illegal action " + std::to_string(a[i]) + " at ply " + std::to_string(i) +
             " of a root history";
      return false;
    }
  }
  return true;
}






int CheckParams(const os_engine* e, const os_mcts_params* p, bool search = true) {
  if (!p) return Fail(OS_ERR_INVALID, "null params");
  // A binding built against an older, shorter os_mcts_params leaves whatever
  // follows its struct here: refuse it instead of reading it as a policy.
  if (p->reserved != 0)
    return Fail(OS_ERR_INVALID, "os_mcts_params.reserved must be 0 (struct size mismatch? "
                                "see os_abi_struct_size)");
  if (p->max_simulations < 0) return Fail(OS_ERR_INVALID, "max_simulations < 0");
  if (p->n_rollouts < 1) return Fail(OS_ERR_INVALID, "n_rollouts must be >= 1");
  if (p->policy != OS_POLICY_CPP && p->policy != OS_POLICY_NUMPY)
    return Fail(OS_ERR_INVALID, "unknown policy");
  if (p->block_size < 0 || p->block_size > 1024)
    return Fail(OS_ERR_INVALID, "block_size must be in [0, 1024]");
  if (p->layout != OS_LAYOUT_WAVE && p->layout != OS_LAYOUT_LANE &&
      p->layout != OS_LAYOUT_AUTO)
    return Fail(OS_ERR_INVALID, "unknown layout");
  if (BigBoard(e->game.cfg)) {
    // k_lsearch only: dynamic path / log capacities, wide nodes.
    if (!search)
      return Fail(OS_ERR_UNSUPPORTED, "go / hex above 11 x 11 run searches only on the device");
    if (p->layout == OS_LAYOUT_WAVE || p->policy != OS_POLICY_CPP)
      return Fail(OS_ERR_UNSUPPORTED,
                  "go / hex above 11 x 11 run C++-policy searches on the lane layout");
    return p->child_selection == OS_SELECT_UCT || p->child_selection == OS_SELECT_PUCT
               ? OS_OK : Fail(OS_ERR_INVALID, "unknown child_selection");
  }
  if (e->game.cfg.max_children > kMaxChildren)
    return Fail(OS_ERR_UNSUPPORTED, "game exceeds kMaxChildren");
  // Games with chance nodes bound the tree depth instead (kChancePathCap;
  // a deeper tree fails the search with kPathOverflow).
  if (e->game.cfg.max_game_length >= kMaxPath && e->game.cfg.kind != kPig)
    return Fail(OS_ERR_UNSUPPORTED, "game exceeds kMaxPath");
  if (p->child_selection != OS_SELECT_UCT && p->child_selection != OS_SELECT_PUCT)
    return Fail(OS_ERR_INVALID, "unknown child_selection");
  if (search && e->game.cfg.kind == kGo && p->layout == OS_LAYOUT_LANE &&
      p->policy != OS_POLICY_CPP)
    return Fail(OS_ERR_UNSUPPORTED,
                "go's lane layout runs the C++ policy (the wave layout runs numpy bots)");
  return OS_OK;
}

// OS_LAYOUT_AUTO: one wave per search.  hex takes the wave layout only where
// its playouts run lane-parallel (C++ policy, n >= 3; os_wave.h
// hex_rollout_lanes: 6.5e7 vs 1.4e7 sims/s at 4096 roots, profiles/r01).
// Breakthrough at C3's 65536 roots: wave 8.3e7 vs lane 3.3e7 sims/s
// (profiles/r02), so a large batch no longer switches to the lane layout.
// go9 at 256 sims (profiles/r06/g9_lanes): wave 1.70e7 / 1.74e7 sims/s at
// 4096 / 8192 roots (about 1.75e7 at 16384, the wave time grows linearly),
// lane (k_lsearch, 16 lanes per wave) 3.7e6 / 5.4e6 / 1.57e7 at 4096 / 8192 /
// 16384 and 2.5e7 at 32768 -- the lane layout needs enough searches to fill
// the chip, so go takes it from 32768 roots.
int32_t ResolveLayout(const GameCfg& cfg, int32_t layout, int64_t R, int32_t policy) {
  if (layout != OS_LAYOUT_AUTO) return layout;
  // pig (chance nodes): one wave per search (k_wsearch_chance) beats a lane
  // per search at every batch size, 1.7x at one root and 4.3x from 64
  // (tools/pig_layout_probe.py, profiles/r04/pig_layout.txt).
  if (cfg.kind == kPig) return OS_LAYOUT_WAVE;
  if (BigBoard(cfg)) return OS_LAYOUT_LANE;  // k_lsearch
  if (cfg.kind == kGo)
    return policy == OS_POLICY_CPP && R >= 32768 ? OS_LAYOUT_LANE : OS_LAYOUT_WAVE;
  // hex: one wave per search under both policies (the numpy policy's
  // playout draws found over a lane window, os_wave.h hex_rollout_lanes_np);
  // boards below 3 x 3 have no lane-parallel playout.
  if (cfg.kind == kHex) return cfg.rows >= 3 ? OS_LAYOUT_WAVE : OS_LAYOUT_LANE;
  return OS_LAYOUT_WAVE;
}

// Per-search HBM buffers of the global-memory lane layout (k_lsearch: go, and
// hex above 11 x 11): visit path, go's position log + links (+ bucket heads
// above 11 x 11), the u16 expansion buffer above 11 x 11 (LDS otherwise).
bool LaneGlobal(const os_engine* e) {
  return (e->game.cfg.kind == kGo || BigBoard(e->game.cfg)) &&
         e->params.layout == OS_LAYOUT_LANE;
}
int LaneLogCap(const GameCfg& c) {
  return c.kind != kGo ? 0 : (GoBigBoard(c) ? kGoLogCapBig : kGoLogCap);
}
size_t LaneGlobalBytes(const os_engine* e) {
  if (!LaneGlobal(e)) return 0;
  const GameCfg& c = e->game.cfg;
  const size_t pe = e->node_double ? sizeof(PathEnt<double>) : sizeof(PathEnt<int32_t>);
  return (c.max_game_length + 2) * pe + static_cast<size_t>(LaneLogCap(c)) * 12 +
         (GoBigBoard(c) ? kGoHeadsBig * 2 : 0) + (BigBoard(c) ? (c.max_children + 1) * 2 : 0);
}

// Nodes per page of the paged arena: room for 64 expansions of the widest
// node, at least 256.
uint32_t PageNodes(int max_children) {
  uint32_t pn = 256;
  while (pn < 64u * static_cast<uint32_t>(max_children)) pn <<= 1;
  return pn;
}
constexpr int64_t kPagedMinRoots = 64;  // below this the reservation is small

// Sizes the search arena of the prepared batch (e->params, e->num_roots):
//  * reserved: the exact worst case 1 + sims * max_children per root (one
//    expansion per simulation at most; plus the GC stack when GC can fire),
//    unless the caller caps it, with roots chunked to fit ~60% of HBM;
//  * paged (arena_mode OS_ARENA_PAGED; the wave layout's C++-policy UCT
//    search or any lane-layout search; no GC, >= 64 roots, and a hint from an
//    earlier fetched run of the same shape): one pool of pages
//    for the whole batch, sized from the pages the earlier runs needed per
//    root (x 1.25 + slack).  A batch that still runs out of pages is rerun on
//    the reserved arena by the fetch (os_engine_arena_info counts it).
int SizeArena(os_engine* e, bool allow_paged) {
  const os_mcts_params* p = &e->params;
  const GameCfg& cfg = e->game.cfg;
  const int64_t R = e->num_roots;
  int64_t worst = 1 + static_cast<int64_t>(p->max_simulations) * cfg.max_children;
  // GC (mcts.cc:402-424) can fire only if the node budget can be reached; its
  // DFS stack then lives in the arena tail, so reserve room for it.
  const int64_t max_nodes = (p->max_memory_mb << 20) / 80 + 1;
  const bool gc_possible = max_nodes > 1 && worst >= max_nodes;
  if (gc_possible)
    worst += GcStackReserve(cfg.max_children, std::max(kMaxPath, cfg.max_game_length + 2));
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  // The arena this engine already holds is released before a larger one.
  const size_t budget = static_cast<size_t>((free_b + e->d_arena.bytes) * 0.6);
  const size_t mt_bytes = 2 * kMtN * 4 + LaneGlobalBytes(e);
  e->paged = false;
  e->page_nodes = 0;
  e->pool_pages = 0;
  const uint32_t pn = PageNodes(cfg.max_children);
  const auto& h = e->arena_hint;
  // The wave layout pages its C++-policy UCT kernel only; the lane layouts'
  // mcts_search takes pages under every policy and child selection.
  const bool pageable_layout =
      (p->layout == OS_LAYOUT_WAVE && p->policy == OS_POLICY_CPP &&
       p->child_selection == OS_SELECT_UCT && e->game.cfg.kind != kPig) ||
      p->layout == OS_LAYOUT_LANE;
  if (allow_paged && e->arena_mode == OS_ARENA_PAGED && pageable_layout &&
      !gc_possible && p->arena_nodes == 0 && R >= kPagedMinRoots &&
      h.sims == p->max_simulations && h.node_bytes == e->node_bytes && h.page_nodes == pn &&
      2 * static_cast<int64_t>(pn) <= worst) {
    const double extra = h.extra_per_root * static_cast<double>(R) * 1.25 +
                         static_cast<double>(R) / 16.0 + 16.0;
    const int64_t pages = R + static_cast<int64_t>(std::ceil(extra));
    const size_t bytes = static_cast<size_t>(pages) * pn * e->node_bytes +
                         static_cast<size_t>(R) * mt_bytes;
    if (pages * static_cast<int64_t>(pn) < (int64_t(1) << 32) && bytes <= budget) {
      e->paged = true;
      e->page_nodes = pn;
      e->pool_pages = static_cast<uint32_t>(pages);
      e->cap = pn;
      e->chunk_roots = R;
      return OS_OK;
    }
  }
  int64_t cap = p->arena_nodes > 0 ? std::min<int64_t>(p->arena_nodes, worst) : worst;
  if (cap < 1) cap = 1;
  if (cap > 0x7FFFFFFF) return Fail(OS_ERR_CAPACITY, "arena too large per root");
  e->cap = static_cast<uint32_t>(cap);
  // Chunk roots so that arena + MT state stay within ~60% of free HBM.
  const size_t per_root = static_cast<size_t>(cap) * e->node_bytes + mt_bytes;
  int64_t chunk = per_root ? static_cast<int64_t>(budget / per_root) : R;
  if (chunk < 1) return Fail(OS_ERR_CAPACITY, "not enough device memory for one root");
  e->chunk_roots = std::max<int64_t>(1, std::min<int64_t>(chunk, std::max<int64_t>(R, 1)));
  return OS_OK;
}

// Allocates the arena SizeArena chose (a pool much smaller than the buffer
// held from an earlier reserved run replaces it, so the footprint shrinks).
int AllocArena(os_engine* e) {
  const size_t need = e->paged
      ? static_cast<size_t>(e->pool_pages) * e->page_nodes * e->node_bytes
      : static_cast<size_t>(e->chunk_roots) * static_cast<size_t>(e->cap) * e->node_bytes;
  if (e->d_arena.bytes > 2 * need) e->d_arena.release();
  e->arena_bytes = need;
  int rc = e->d_arena.ensure(need);
  if (rc || !e->paged) return rc;
  // The descriptor os_wave.h reads: {taken (zeroed per launch), page_nodes,
  // pool_pages, first dynamic page = the roots' own pages}.
  if ((rc = e->d_page_next.ensure(16))) return rc;
  const uint32_t desc[4] = {0u, e->page_nodes, e->pool_pages,
                            static_cast<uint32_t>(e->num_roots)};
  HIP_TRY(hipMemcpy(e->d_page_next.p, desc, sizeof desc, hipMemcpyHostToDevice));
  return OS_OK;
}

// Pages beyond its own that each root of the last fetched run would take in
// the pool: a page fills to at least page_nodes - max_children + 1 nodes
// before a child block spills into the next.
void UpdateArenaHint(os_engine* e) {
  if (e->last_results.empty()) return;
  const int mc = e->game.cfg.max_children;
  const uint32_t pn = PageNodes(mc);
  const int64_t eff = static_cast<int64_t>(pn) - mc + 1;
  double extra = 0.0;
  for (const SearchResult& s : e->last_results) {
    const int64_t a = s.used;
    if (a > eff) extra += static_cast<double>((a - eff + eff - 1) / eff);
  }
  auto& h = e->arena_hint;
  const double per_root = extra / static_cast<double>(e->last_results.size());
  const bool same = h.sims == e->params.max_simulations && h.node_bytes == e->node_bytes &&
                    h.page_nodes == pn;
  h.extra_per_root = same ? std::max(h.extra_per_root, per_root) : per_root;
  h.sims = e->params.max_simulations;
  h.node_bytes = e->node_bytes;
  h.page_nodes = pn;
}

// Parent-count LUT from the host libm, N in [0, sims + 1]: UCTValue's
// std::log(parent_explore_count) (mcts.cc:99), or PUCTValue's
// std::sqrt(parent_explore_count) (mcts.cc:109).  Uploaded only when the
// simulation count or the selection changed.
int UploadLut(os_engine* e, int32_t sims, bool puct) {
  const size_t n = static_cast<size_t>(sims) + 2;
  int rc;
  if ((rc = e->d_lut.ensure(n * 8))) return rc;
  if (e->lut_at == e->d_lut.p && e->lut_n == static_cast<int64_t>(n) &&
      e->lut_puct == (puct ? 1 : 0))
    return OS_OK;
  std::vector<double> lut(n);
  for (size_t i = 0; i < n; ++i)
    lut[i] = puct ? std::sqrt(static_cast<double>(i)) : std::log(static_cast<double>(i));
  HIP_TRY(hipMemcpy(e->d_lut.p, lut.data(), n * 8, hipMemcpyHostToDevice));
  e->lut_at = e->d_lut.p;
  e->lut_n = static_cast<int64_t>(n);
  e->lut_puct = puct ? 1 : 0;
  return OS_OK;
}

// go's Zobrist table, uploaded once per engine.
int UploadZob(os_engine* e) {
  int rc;
  if ((rc = e->d_zob.ensure(e->game.zob.size() * 8))) return rc;
  if (e->zob_at == e->d_zob.p) return OS_OK;
  HIP_TRY(hipMemcpy(e->d_zob.p, e->game.zob.data(), e->game.zob.size() * 8,
                    hipMemcpyHostToDevice));
  e->zob_at = e->d_zob.p;
  return OS_OK;
}

// Batched small copies through the engine's pinned staging buffer: queued on
// the null stream, then one wait.  Only batches of up to kStageMax bytes are
// staged (a single bot's step moves a few hundred bytes, where the copies'
// fixed costs dominate); larger ones copy directly with synchronous
// hipMemcpy, pageable memory on the host side, so the pinned buffer stays
// small and a big prepare never depends on a large hipHostMalloc.
constexpr size_t kStageMax = size_t(1) << 20;

struct Stager {
  os_engine* e;
  size_t off = 0;
  bool direct = false;                        // batch above kStageMax
  std::vector<std::vector<unsigned char>> dn;  // direct mode: download targets
  explicit Stager(os_engine* eng) : e(eng) {}
  int reserve(size_t bytes) {
    direct = bytes > kStageMax;
    if (direct) return OS_OK;
    // The staging buffer is only reused after the previous batch was waited for.
    return e->h_stage.ensure(std::max<size_t>(bytes, 64 << 10));
  }
  unsigned char* slot(size_t bytes) {
    unsigned char* q = e->h_stage.p + off;
    off += (bytes + 255) & ~size_t(255);
    return q;
  }
  int up(void* dst, const void* src, size_t bytes) {
    if (!bytes) return OS_OK;
    if (direct) {
      HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
      return OS_OK;
    }
    unsigned char* q = slot(bytes);
    std::memcpy(q, src, bytes);
    HIP_TRY(hipMemcpyAsync(dst, q, bytes, hipMemcpyHostToDevice, nullptr));
    return OS_OK;
  }
  int down(unsigned char** q, const void* src, size_t bytes) {
    if (direct) {
      dn.emplace_back(std::max<size_t>(bytes, 1));
      *q = dn.back().data();
      if (bytes) HIP_TRY(hipMemcpy(*q, src, bytes, hipMemcpyDeviceToHost));
      return OS_OK;
    }
    *q = slot(bytes);
    if (bytes) HIP_TRY(hipMemcpyAsync(*q, src, bytes, hipMemcpyDeviceToHost, nullptr));
    return OS_OK;
  }
  int wait() {
    HIP_TRY(hipStreamSynchronize(nullptr));
    return OS_OK;
  }
};

// Host side of a batch's roots: every history replayed into its device
// state record (+ go's hash set); `nlegal` (optional): each root's
// |LegalActions|.  Host-only (no HIP call), so os_az_stage can run it while
// the device works on another batch.
int ReplayRoots(const os_engine* e, int64_t R, const int64_t* root_actions,
                const int64_t* root_offsets, std::vector<unsigned char>* roots,
                std::vector<uint64_t>* rh, std::vector<int32_t>* rnh,
                std::vector<int32_t>* nlegal = nullptr) {
  const GameCfg& cfg = e->game.cfg;
  const int sb = e->game.state_bytes;
  const bool go = cfg.kind == kGo;
  const int64_t hs_stride = go ? cfg.max_game_length + 2 : 1;
  roots->assign(static_cast<size_t>(std::max<int64_t>(R, 1)) * sb, 0);
  rh->clear();
  rnh->clear();
  if (go) {
    rh->assign(static_cast<size_t>(std::max<int64_t>(R, 1)) * hs_stride, 0);
    rnh->assign(std::max<int64_t>(R, 1), 0);
  }
  if (nlegal) nlegal->assign(std::max<int64_t>(R, 1), 0);
  return ParallelChunks(R, 1024, [&](int64_t lo, int64_t hi) {
    std::vector<int64_t> la;
    for (int64_t r = lo; r < hi; ++r) {
      HostState hs;
      std::string err;
      if (!ReplayRoot(e->game, root_actions + root_offsets[r],
                      root_offsets[r + 1] - root_offsets[r], &hs, &err))
        return Fail(OS_ERR_INVALID, "root " + std::to_string(r) + ": " + err);
      if (StateTerminal(hs))
        return Fail(OS_ERR_INVALID, "root " + std::to_string(r) + " is terminal");
      if (StateIsChance(hs))  // a bot is only asked to move at decision nodes
        return Fail(OS_ERR_INVALID, "root " + std::to_string(r) + " is a chance node");
      std::memcpy(roots->data() + r * sb, hs.raw, sb);
      if (go) {
        const int64_t nh = static_cast<int64_t>(hs.hashes.size());
        if (nh > hs_stride) return Fail(OS_ERR_CAPACITY, "go hash history too long");
        std::memcpy(rh->data() + r * hs_stride, hs.hashes.data(), nh * 8);
        (*rnh)[r] = static_cast<int32_t>(nh);
      }
      if (nlegal) {
        StateLegal(hs, &la);
        (*nlegal)[r] = static_cast<int32_t>(la.size());
      }
    }
    return 0;
  });
}

// A batch's replayed roots, handed to Prepare instead of the histories.
struct PreRoots {
  const std::vector<unsigned char>* roots;
  const std::vector<uint64_t>* rh;
  const std::vector<int32_t>* rnh;
};

// Uploads roots / seeds, sizes and allocates the arena and outputs.
int Prepare(os_engine* e, const os_mcts_params* p, int64_t R,
            const int64_t* root_actions, const int64_t* root_offsets,
            const uint32_t* bot_seeds, const uint32_t* eval_seeds, bool search = true,
            const PreRoots* pre = nullptr) {
  int rc = CheckParams(e, p, search);
  if (rc) return rc;
  if (R < 0) return Fail(OS_ERR_INVALID, "num_roots < 0");
  HIP_TRY(hipSetDevice(e->device));
  e->params = *p;
  e->params.layout = ResolveLayout(e->game.cfg, p->layout, R, p->policy);
  e->search_layout = e->params.layout;
  e->num_roots = R;
  const GameCfg& cfg = e->game.cfg;
  e->max_children = cfg.max_children;
  // f64 node rewards when they are not integers: rollout means, or pig's
  // -1 / (n - 1) losses with more than two players (pig.cc:94-111).
  e->node_double = !(p->n_rollouts == 1 && cfg.pig_players <= 2);
  e->node_wide = BigBoard(cfg);
  e->node_bytes = static_cast<int>(
      e->node_wide ? (e->node_double ? sizeof(Node<double, true>) : sizeof(Node<int32_t, true>))
                   : (e->node_double ? sizeof(Node<double>) : sizeof(Node<int32_t>)));
  if ((rc = SizeArena(e, true))) return rc;

  // Root states (+ go hash sets) on the host.
  const int sb = e->game.state_bytes;
  const bool go = cfg.kind == kGo;
  e->hash_stride = go ? cfg.max_game_length + 2 : 1;
  std::vector<unsigned char> own_roots;
  std::vector<uint64_t> own_rh;
  std::vector<int32_t> own_rnh;
  if (!pre) {
    if ((rc = ReplayRoots(e, R, root_actions, root_offsets, &own_roots, &own_rh, &own_rnh)))
      return rc;
  }
  const std::vector<unsigned char>& roots = pre ? *pre->roots : own_roots;
  const std::vector<uint64_t>& rh = pre ? *pre->rh : own_rh;
  const std::vector<int32_t>& rnh = pre ? *pre->rnh : own_rnh;
  const size_t Rz = static_cast<size_t>(std::max<int64_t>(R, 1));
  if ((rc = e->d_roots.ensure(Rz * sb))) return rc;
  if ((rc = e->d_bseed.ensure(Rz * 4)) || (rc = e->d_eseed.ensure(Rz * 4))) return rc;
  if (go && ((rc = e->d_rhash.ensure(rh.size() * 8)) || (rc = e->d_rnh.ensure(rnh.size() * 4))))
    return rc;
  {
    Stager st(e);
    const size_t need = Rz * sb + 2 * Rz * 4 + (go ? rh.size() * 8 + rnh.size() * 4 : 0) +
                        6 * 256;
    if ((rc = st.reserve(need)) || (rc = st.up(e->d_roots.p, roots.data(), Rz * sb))) return rc;
    if (R > 0 && ((rc = st.up(e->d_bseed.p, bot_seeds, R * 4)) ||
                  (rc = st.up(e->d_eseed.p, eval_seeds ? eval_seeds : bot_seeds, R * 4))))
      return rc;
    if (go && ((rc = st.up(e->d_rhash.p, rh.data(), rh.size() * 8)) ||
               (rc = st.up(e->d_rnh.p, rnh.data(), rnh.size() * 4))))
      return rc;
    if ((rc = st.wait())) return rc;
  }
  if (go && (rc = UploadZob(e))) return rc;
  if ((rc = UploadLut(e, p->max_simulations, p->child_selection == OS_SELECT_PUCT))) return rc;
  // Work buffers.
  const size_t C = static_cast<size_t>(e->chunk_roots);
  if ((rc = e->d_mt.ensure(C * 2 * kMtN * 4))) return rc;
  if (LaneGlobal(e)) {
    const size_t pe = e->node_double ? sizeof(PathEnt<double>) : sizeof(PathEnt<int32_t>);
    const size_t lc = LaneLogCap(cfg);
    if ((rc = e->d_lpath.ensure(C * (cfg.max_game_length + 2) * pe)) ||
        (rc = e->d_glog.ensure(C * lc * 8)) || (rc = e->d_glink.ensure(C * lc * 4)) ||
        (GoBigBoard(cfg) && (rc = e->d_lheads.ensure(C * kGoHeadsBig * 2))) ||
        (BigBoard(cfg) && (rc = e->d_lact.ensure(C * (cfg.max_children + 1) * 2))))
      return rc;
  }
  if ((rc = AllocArena(e))) return rc;
  const size_t MC = Rz * e->max_children;
  if ((rc = e->d_res.ensure(Rz * sizeof(SearchResult))) || (rc = e->d_cact.ensure(MC * 4)) ||
      (rc = e->d_cn.ensure(MC * 4)) || (rc = e->d_cw.ensure(MC * 8)) ||
      (rc = e->d_cout.ensure(MC)) || (rc = e->d_nch.ensure(Rz * 4)) ||
      (rc = e->d_rn.ensure(Rz * 4)) || (rc = e->d_rw.ensure(Rz * 8)) ||
      (rc = e->d_rout.ensure(Rz)) || (rc = e->d_best.ensure(Rz * 8)) ||
      (rc = e->d_pos.ensure(Rz * 8)))
    return rc;
  e->import_state = false;
  e->shared_stream = false;
  e->roll_ready = false;  // rollouts, searches and self-play share buffers
  e->sp_ready = false;
  e->az_ready = false;
  return OS_OK;
}


int Run(os_engine* e, hipStream_t stream) {
  HIP_TRY(hipSetDevice(e->device));
  if (e->num_roots == 0) return OS_OK;
  const GameLaunchers* L = LaunchersFor(e->game.cfg);
  if (!L) return Fail(OS_ERR_UNSUPPORTED, "unknown game kind");
  if (e->paged) HIP_TRY(hipMemsetAsync(e->d_page_next.p, 0, 4, stream));
  if (!e->time_runs) return L->search(e, MakeArgs(e), stream);
  // os_engine_set_run_timing: an event pair around the search launches
  if (!e->run_ev[0]) {
    HIP_TRY(hipEventCreate(&e->run_ev[0]));
    HIP_TRY(hipEventCreate(&e->run_ev[1]));
  }
  HIP_TRY(hipEventRecord(e->run_ev[0], stream));
  const int rc = L->search(e, MakeArgs(e), stream);
  HIP_TRY(hipEventRecord(e->run_ev[1], stream));
  e->run_timed = rc == OS_OK;
  return rc;
}

// A paged batch in which some search ran out of pool pages is run again on
// the reserved arena (same seeds, so the same searches).
int RerunReserved(os_engine* e) {
  int rc;
  if ((rc = SizeArena(e, false))) return rc;
  if ((rc = e->d_mt.ensure(static_cast<size_t>(e->chunk_roots) * 2 * kMtN * 4))) return rc;
  if ((rc = AllocArena(e))) return rc;
  if ((rc = Run(e, nullptr))) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(e->last_results.data(), e->d_res.p, e->num_roots * sizeof(SearchResult),
                    hipMemcpyDeviceToHost));
  return OS_OK;
}

int Fetch(os_engine* e, int32_t max_children, int32_t* child_action,
          int32_t* child_n, double* child_w, int8_t* child_out, int32_t* nchild,
          int32_t* root_n, double* root_w, int8_t* root_out, int64_t* best_action,
          int32_t* nodes) {
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  const int64_t R = e->num_roots;
  if (R == 0) return OS_OK;
  if (max_children < e->max_children)
    return Fail(OS_ERR_INVALID, "max_children smaller than the game's bound (" +
                                    std::to_string(e->max_children) + ")");
  e->last_results.resize(R);
  HIP_TRY(hipMemcpy(e->last_results.data(), e->d_res.p, R * sizeof(SearchResult),
                    hipMemcpyDeviceToHost));
  if (e->paged) {
    int64_t over = 0;
    for (const SearchResult& s : e->last_results) over += s.status == kArenaOverflow;
    if (over) {
      e->arena_overflows += over;
      e->arena_reruns += 1;
      int rc = RerunReserved(e);
      if (rc) return rc;
    }
  }
  e->last_sims = 0;
  for (int64_t r = 0; r < R; ++r) {
    const SearchResult& s = e->last_results[r];
    if (s.status != kOk) {
      const std::string why = s.status == kArenaOverflow
                            ? "node arena overflow (raise arena_nodes)"
                            : (s.status == kPathOverflow ? "tree path overflow"
                               : s.status == kGcStackOverflow ? "GC stack overflow"
                                 : "search status " + std::to_string(s.status));
      return Fail(OS_ERR_CAPACITY, "root " + std::to_string(r) + ": " + why);
    }
    e->last_sims += s.sims;
    if (nodes) nodes[r] = s.nodes;
  }
  UpdateArenaHint(e);
  const int mcd = e->max_children;
  const size_t M = static_cast<size_t>(R) * mcd;
  // One queue of device-to-pinned copies and one wait (a single bot's step
  // fetches a few hundred bytes: the copies' fixed costs dominate).
  Stager st(e);
  unsigned char *ca8, *cn8, *cw8, *co8, *nch8, *rn8, *rw8, *ro8, *ba8;
  int rc;
  if ((rc = st.reserve(M * 17 + static_cast<size_t>(R) * 25 + 9 * 256)) ||
      (rc = st.down(&ca8, e->d_cact.p, M * 4)) || (rc = st.down(&cn8, e->d_cn.p, M * 4)) ||
      (rc = st.down(&cw8, e->d_cw.p, M * 8)) || (rc = st.down(&co8, e->d_cout.p, M)) ||
      (rc = st.down(&nch8, e->d_nch.p, R * 4)) || (rc = st.down(&rn8, e->d_rn.p, R * 4)) ||
      (rc = st.down(&rw8, e->d_rw.p, R * 8)) || (rc = st.down(&ro8, e->d_rout.p, R)) ||
      (rc = st.down(&ba8, e->d_best.p, R * 8)) || (rc = st.wait()))
    return rc;
  const int32_t* ca = reinterpret_cast<const int32_t*>(ca8);
  const int32_t* cn = reinterpret_cast<const int32_t*>(cn8);
  const double* cw = reinterpret_cast<const double*>(cw8);
  const int8_t* co = reinterpret_cast<const int8_t*>(co8);
  std::memcpy(nchild, nch8, R * 4);
  std::memcpy(root_n, rn8, R * 4);
  std::memcpy(root_w, rw8, R * 8);
  std::memcpy(root_out, ro8, R);
  std::memcpy(best_action, ba8, R * 8);
  for (int64_t r = 0; r < R; ++r) {
    for (int k = 0; k < max_children; ++k) {
      const int64_t o = r * max_children + k;
      if (k < nchild[r] && k < mcd) {
        child_action[o] = ca[r * mcd + k];
        child_n[o] = cn[r * mcd + k];
        child_w[o] = cw[r * mcd + k];
        child_out[o] = co[r * mcd + k];
      } else {
        child_action[o] = -1;
        child_n[o] = 0;
        child_w[o] = 0.0;
        child_out[o] = kUnsolved;
      }
    }
  }
  return OS_OK;
}

// Node capacity per tree: the exact worst case 1 + sims * max_children (one
// expansion per simulation at most), plus the GC stack reserve when GC can
// fire (mcts.cc:402-424), unless the caller caps it.
int ArenaCap(const os_engine* e, const os_mcts_params* p, uint32_t* cap_out) {
  const GameCfg& cfg = e->game.cfg;
  int64_t worst = 1 + static_cast<int64_t>(p->max_simulations) * cfg.max_children;
  const int64_t max_nodes = (p->max_memory_mb << 20) / 80 + 1;
  if (max_nodes > 1 && worst >= max_nodes) worst += GcStackReserve(cfg.max_children);
  int64_t cap = p->arena_nodes > 0 ? std::min<int64_t>(p->arena_nodes, worst) : worst;
  if (cap < 1) cap = 1;
  if (cap > 0x7FFFFFFF) return Fail(OS_ERR_CAPACITY, "arena too large per tree");
  *cap_out = static_cast<uint32_t>(cap);
  return OS_OK;
}

// Self-play batch: replays the start positions, uploads them with the seeds
// and sizes one tree arena per game (reused by every move's search).
int SpPrepare(os_engine* e, const os_mcts_params* p, int64_t G, const int64_t* start_actions,
              const int64_t* start_offsets, const uint32_t* bot_seeds,
              const uint32_t* eval_seeds, int32_t max_len, int32_t record) {
  if (BigBoard(e->game.cfg))
    return Fail(OS_ERR_UNSUPPORTED, "go / hex above 11 x 11 run searches only on the device");
  const bool with_visits = (record & OS_RECORD_VISITS) != 0;
  const bool with_obs = (record & OS_RECORD_OBSERVATIONS) != 0;
  const bool with_policy = (record & OS_RECORD_POLICY) != 0;
  const bool with_values = (record & OS_RECORD_ROOT_VALUES) != 0;
  if (!e->sp_actor_seeds.empty() && static_cast<int64_t>(e->sp_actor_seeds.size()) != G)
    return Fail(OS_ERR_INVALID, "os_selfplay_set_options was given a different game count");
  int rc = CheckParams(e, p);
  if (rc) return rc;
  if (p->policy != OS_POLICY_CPP)
    return Fail(OS_ERR_UNSUPPORTED, "self-play implements the C++ MCTSBot policy only");
  if (G < 0 || max_len < 0) return Fail(OS_ERR_INVALID, "negative size");
  if (G > 0 && (!bot_seeds || !eval_seeds || !start_offsets))
    return Fail(OS_ERR_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->device));
  e->params = *p;
  e->params.layout = OS_LAYOUT_WAVE;
  e->paged = false;  // self-play trees use the reserved arena
  e->node_double = p->n_rollouts != 1;
  e->node_wide = false;
  e->node_bytes = p->n_rollouts == 1 ? static_cast<int>(sizeof(Node<int32_t>))
                                      : static_cast<int>(sizeof(Node<double>));
  if ((rc = ArenaCap(e, p, &e->cap))) return rc;
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const size_t per_game = static_cast<size_t>(e->cap) * e->node_bytes;
  const int64_t chunk = static_cast<int64_t>(free_b * 0.6 / std::max<size_t>(per_game, 1));
  if (chunk < 1) return Fail(OS_ERR_CAPACITY, "not enough device memory for one game");
  e->chunk_roots = std::max<int64_t>(1, std::min<int64_t>(chunk, std::max<int64_t>(G, 1)));
  const GameCfg& cfg = e->game.cfg;
  const int sb = e->game.state_bytes;
  const bool go = cfg.kind == kGo;
  e->hash_stride = go ? cfg.max_game_length + 2 : 1;
  const size_t Gz = static_cast<size_t>(std::max<int64_t>(G, 1));
  std::vector<unsigned char> starts(Gz * sb);
  std::vector<uint64_t> hist(go ? Gz * e->hash_stride : 1, 0);
  std::vector<int32_t> histn(Gz, 0);
  for (int64_t r = 0; r < G; ++r) {
    HostState hs;
    std::string err;
    if (!ReplayRoot(e->game, start_actions + start_offsets[r],
                    start_offsets[r + 1] - start_offsets[r], &hs, &err))
      return Fail(OS_ERR_INVALID, "game " + std::to_string(r) + ": " + err);
    std::memcpy(starts.data() + r * sb, hs.raw, sb);
    if (go) {
      const int64_t nh = static_cast<int64_t>(hs.hashes.size());
      if (nh > e->hash_stride) return Fail(OS_ERR_CAPACITY, "go hash history too long");
      std::memcpy(hist.data() + r * e->hash_stride, hs.hashes.data(), nh * 8);
      histn[r] = static_cast<int32_t>(nh);
    }
  }
  if ((rc = e->d_roots.ensure(Gz * sb)) || (rc = e->d_bseed.ensure(Gz * 8)) ||
      (rc = e->d_eseed.ensure(Gz * 4)) || (rc = e->d_rhash.ensure(hist.size() * 8)) ||
      (rc = e->d_rnh.ensure(Gz * 4)))
    return rc;
  HIP_TRY(hipMemcpy(e->d_roots.p, starts.data(), Gz * sb, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_rhash.p, hist.data(), hist.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_rnh.p, histn.data(), Gz * 4, hipMemcpyHostToDevice));
  if (G > 0) {
    HIP_TRY(hipMemcpy(e->d_bseed.p, bot_seeds, G * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->d_eseed.p, eval_seeds, G * 4, hipMemcpyHostToDevice));
  }
  if (go && (rc = UploadZob(e))) return rc;
  if ((rc = UploadLut(e, p->max_simulations, p->child_selection == OS_SELECT_PUCT))) return rc;
  const size_t lut_n = static_cast<size_t>(p->max_simulations) + 2;
  // AlphaZero move choice: pow(explore_count, 1 / T) from the host libm
  // (alpha_zero.cc:82-83), and the actor rng seeds.
  if (e->sp_opts.temperature > 0.0) {
    std::vector<double> pw(lut_n);
    const double ex = 1.0 / e->sp_opts.temperature;
    for (size_t i = 0; i < pw.size(); ++i) pw[i] = std::pow(static_cast<double>(i), ex);
    if ((rc = e->d_sp_pow.ensure(pw.size() * 8))) return rc;
    HIP_TRY(hipMemcpy(e->d_sp_pow.p, pw.data(), pw.size() * 8, hipMemcpyHostToDevice));
  }
  if (!e->sp_actor_seeds.empty()) {
    if ((rc = e->d_sp_actor.ensure(e->sp_actor_seeds.size() * 4))) return rc;
    HIP_TRY(hipMemcpy(e->d_sp_actor.p, e->sp_actor_seeds.data(), e->sp_actor_seeds.size() * 4,
                      hipMemcpyHostToDevice));
  }
  const size_t L = static_cast<size_t>(std::max(max_len, 1));
  const size_t A = static_cast<size_t>(cfg.num_actions);
  (void)lut_n;
  if ((rc = e->d_arena.ensure(static_cast<size_t>(e->chunk_roots) * per_game)) ||
      (rc = e->d_res.ensure(Gz * sizeof(SearchResult))) ||
      (rc = e->d_sp_act.ensure(Gz * L * 4)) || (rc = e->d_sp_len.ensure(Gz * 4)) ||
      (rc = e->d_sp_ret.ensure(Gz * 16)) ||
      (with_visits && (rc = e->d_sp_vis.ensure(Gz * L * A * 4))) ||
      (with_obs && (rc = e->d_sp_obs.ensure(Gz * L * ObservationShape(e->game, nullptr) * 4))) ||
      (with_policy && (rc = e->d_sp_pol.ensure(Gz * L * A * 8))) ||
      (with_values && (rc = e->d_sp_val.ensure(Gz * L * 8))))
    return rc;
  e->sp_games = G;
  e->sp_max_len = max_len;
  e->sp_visits = with_visits;
  e->sp_obs = with_obs;
  e->sp_policy = with_policy;
  e->sp_values = with_values;
  e->sp_ready = true;
  e->num_roots = 0;       // the search buffers now hold no prepared batch
  e->roll_ready = false;
  e->az_ready = false;
  return OS_OK;
}


int SpRun(os_engine* e, hipStream_t stream) {
  if (!e->sp_ready) return Fail(OS_ERR_INVALID, "os_selfplay_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  if (e->sp_games == 0) return OS_OK;
  const GameLaunchers* L = LaunchersFor(e->game.cfg);
  if (!L || !L->selfplay)
    return Fail(OS_ERR_UNSUPPORTED, "go above 11 x 11 runs searches only on the device");
  return L->selfplay(e, stream);
}

int SpFetch(os_engine* e, int64_t* actions, int32_t* length, double* returns,
            int32_t* visits, float* observations) {
  if (!e->sp_ready) return Fail(OS_ERR_INVALID, "os_selfplay_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  const int64_t G = e->sp_games;
  if (G == 0) return OS_OK;
  e->last_results.resize(G);
  HIP_TRY(hipMemcpy(e->last_results.data(), e->d_res.p, G * sizeof(SearchResult),
                    hipMemcpyDeviceToHost));
  e->last_sims = 0;
  for (int64_t r = 0; r < G; ++r) {
    const SearchResult& s = e->last_results[r];
    if (s.status != kOk) {
      const char* why = s.status == kGameOverflow ? "game longer than max_len"
                        : s.status == kArenaOverflow ? "node arena overflow (raise arena_nodes)"
                        : s.status == kPathOverflow ? "tree path overflow"
                                                    : "GC stack overflow";
      return Fail(OS_ERR_CAPACITY, "game " + std::to_string(r) + ": " + why);
    }
    e->last_sims += s.sims;
  }
  const size_t L = static_cast<size_t>(e->sp_max_len);
  if (actions) {
    std::vector<int32_t> a32(G * L);
    if (L) HIP_TRY(hipMemcpy(a32.data(), e->d_sp_act.p, a32.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < a32.size(); ++i) actions[i] = a32[i];
  }
  if (length) HIP_TRY(hipMemcpy(length, e->d_sp_len.p, G * 4, hipMemcpyDeviceToHost));
  if (returns) HIP_TRY(hipMemcpy(returns, e->d_sp_ret.p, G * 16, hipMemcpyDeviceToHost));
  if (visits) {
    if (!e->sp_visits) return Fail(OS_ERR_INVALID, "prepared without visit recording");
    HIP_TRY(hipMemcpy(visits, e->d_sp_vis.p, G * L * e->game.cfg.num_actions * 4,
                      hipMemcpyDeviceToHost));
  }
  if (observations) {
    if (!e->sp_obs) return Fail(OS_ERR_INVALID, "prepared without observation recording");
    HIP_TRY(hipMemcpy(observations, e->d_sp_obs.p,
                      G * L * ObservationShape(e->game, nullptr) * 4, hipMemcpyDeviceToHost));
  }
  return OS_OK;
}


// bot_keys / bot_pos (both or neither): each search continues a bot rng_
// held in numpy's (key[624], pos) form instead of seeding one.
// Dirichlet root noise of a batch (os_az.h): per root, the normalised
// std::gamma_distribution draws of a fresh MCTSBot(seed) -- or of the stream
// (keys, pos) -- over its nlegal[r] legal actions, and the words they took.
int DrawRootNoise(const os_engine* e, int64_t R, const std::vector<int32_t>& nlegal,
                  const uint32_t* bot_seeds, const uint32_t* bot_keys, const int32_t* bot_pos,
                  double alpha, std::vector<double>* noise, std::vector<int32_t>* skip) {
  const int mc = e->game.cfg.max_children;
  const size_t Rz = static_cast<size_t>(std::max<int64_t>(R, 1));
  noise->assign(Rz * mc, 0.0);
  skip->assign(Rz, 0);
  return ParallelChunks(R, 512, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      const int64_t w =
          bot_keys ? DirichletNoiseState(bot_keys + r * kMtN, bot_pos[r], nlegal[r], alpha,
                                         noise->data() + r * mc)
                   : DirichletNoise(bot_seeds[r], nlegal[r], alpha, noise->data() + r * mc);
      if (w > 0x7FFFFFFF) return Fail(OS_ERR_CAPACITY, "Dirichlet draw too long");
      (*skip)[r] = static_cast<int32_t>(w);
    }
    return 0;
  });
}

int AzPrepare(os_engine* e, const os_mcts_params* p, int32_t puct, int64_t R,
              const int64_t* root_actions, const int64_t* root_offsets,
              const uint32_t* bot_seeds, double alpha, double eps, int32_t* kind, float* obs,
              uint8_t* legal, const double* prior, const double* value, int32_t* pending,
              const uint32_t* bot_keys = nullptr, const int32_t* bot_pos = nullptr,
              const os_engine::AzStaged* stg = nullptr) {
  if (!p) return Fail(OS_ERR_INVALID, "null params");
  const bool import = bot_keys != nullptr;
  std::vector<uint32_t> zero_seeds;
  if (import) {
    if (!bot_pos) return Fail(OS_ERR_INVALID, "bot_keys need bot_pos");
    for (int64_t r = 0; r < R; ++r)
      if (bot_pos[r] < 0 || bot_pos[r] > kMtN) return Fail(OS_ERR_INVALID, "bad rng position");
    zero_seeds.assign(static_cast<size_t>(std::max<int64_t>(R, 1)), 0u);
    bot_seeds = zero_seeds.data();
  }
  if (!(alpha >= 0.0) || !(eps >= 0.0) || eps > 1.0)
    return Fail(OS_ERR_INVALID, "dirichlet_alpha must be >= 0 and epsilon in [0, 1]");
  if (p->policy != OS_POLICY_CPP && p->policy != OS_POLICY_NUMPY)
    return Fail(OS_ERR_INVALID, "unknown policy");
  const bool np = p->policy == OS_POLICY_NUMPY;
  if (np && alpha > 0.0)
    return Fail(OS_ERR_INVALID,
                "OS_POLICY_NUMPY: draw RandomState.dirichlet on the host and pass it with "
                "os_az_set_noise (alpha must be 0 here)");
  if (R > 0 && (!kind || !obs || !legal || !prior || !value || !pending || !bot_seeds))
    return Fail(OS_ERR_INVALID, "null request / response buffer");
  os_mcts_params q = *p;
  q.policy = OS_POLICY_CPP;  // the shuffle is the az kernels' own (e->az_np)
  if (np) q.max_memory_mb = 0;  // mcts.py never garbage-collects
  q.n_rollouts = 2;  // f64 node rewards (Node<double>): values are not integral
  q.child_selection = OS_SELECT_UCT;  // `puct` selects; the LUT stays log(N)
  q.layout = OS_LAYOUT_LANE;
  // The roots' host work: replayed once (records, go hash sets, legal counts
  // for the noise), or taken from os_az_stage.
  int rc = CheckParams(e, &q, false);
  if (rc) return rc;
  if (R < 0) return Fail(OS_ERR_INVALID, "num_roots < 0");
  std::vector<unsigned char> own_roots;
  std::vector<uint64_t> own_rh;
  std::vector<int32_t> own_rnh, nlegal;
  if (!stg && (rc = ReplayRoots(e, R, root_actions, root_offsets, &own_roots, &own_rh, &own_rnh,
                                alpha > 0.0 ? &nlegal : nullptr)))
    return rc;
  const PreRoots pre = stg ? PreRoots{&stg->roots, &stg->rh, &stg->rnh}
                           : PreRoots{&own_roots, &own_rh, &own_rnh};
  rc = Prepare(e, &q, R, root_actions, root_offsets, bot_seeds, bot_seeds,
               /*search=*/false, &pre);  // buffers only: k_az_step runs the search
  if (rc) return rc;
  if (e->chunk_roots < R)
    return Fail(OS_ERR_CAPACITY, "external-evaluator searches must all fit in HBM at once");
  const GameLaunchers* L = LaunchersFor(e->game.cfg);
  if (!L || !L->az) return Fail(OS_ERR_UNSUPPORTED, "game");
  const size_t slot_bytes = L->az_slot_bytes;
  const size_t Rz = static_cast<size_t>(std::max<int64_t>(R, 1));
  if ((rc = e->d_az_slots.ensure(Rz * slot_bytes)) ||
      (rc = e->d_az_prior.ensure(Rz * static_cast<size_t>(e->cap) * 8)))
    return rc;
  // Fused requests park each evaluated leaf's priors until its expansion; the
  // reserved arena (1 + sims * max_children) bounds them, as every simulation
  // parks at most one leaf's children.
  e->az_fused = e->az_requests == OS_AZ_REQUESTS_FUSED;
  if (e->az_fused && (rc = e->d_az_raw.ensure(Rz * static_cast<size_t>(e->cap) * 8))) return rc;
  HIP_TRY(hipMemset(e->d_az_slots.p, 0, Rz * slot_bytes));  // stage kAzStart
  e->az_noise = alpha > 0.0;
  e->az_eps = eps;
  if (e->az_noise) {
    // The root expands once unless GC clears its children (mcts.cc:430-443);
    // the noise is drawn ahead for that one expansion.
    const int64_t max_nodes = (q.max_memory_mb << 20) / 80 + 1;
    const int64_t worst = 1 + static_cast<int64_t>(p->max_simulations) * e->game.cfg.max_children;
    if (max_nodes > 1 && worst >= max_nodes)
      return Fail(OS_ERR_UNSUPPORTED,
                  "Dirichlet noise with a max_memory_mb small enough for GC to fire");
    std::vector<double> own_noise;
    std::vector<int32_t> own_skip;
    if (!stg && (rc = DrawRootNoise(e, R, nlegal, bot_seeds, import ? bot_keys : nullptr,
                                    bot_pos, alpha, &own_noise, &own_skip)))
      return rc;
    const std::vector<double>& noise = stg ? stg->noise : own_noise;
    const std::vector<int32_t>& skip = stg ? stg->skip : own_skip;
    if ((rc = e->d_az_noise.ensure(noise.size() * 8)) || (rc = e->d_az_skip.ensure(Rz * 4)))
      return rc;
    HIP_TRY(hipMemcpy(e->d_az_noise.p, noise.data(), noise.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->d_az_skip.p, skip.data(), Rz * 4, hipMemcpyHostToDevice));
  }
  e->az_import = import;
  if (import && R > 0) {  // keys into the bot rng rows, positions in / out
    HIP_TRY(hipMemcpy(e->d_mt.p, bot_keys, static_cast<size_t>(R) * kMtN * 4,
                      hipMemcpyHostToDevice));
    if ((rc = e->d_az_pos.ensure(static_cast<size_t>(R) * 8))) return rc;
    HIP_TRY(hipMemcpy(e->d_az_pos.p, bot_pos, static_cast<size_t>(R) * 4, hipMemcpyHostToDevice));
  }
  e->az_puct = puct ? 1 : 0;
  e->az_np = np ? 1 : 0;
  {
    // One wave per search unless GC could fire (k_waz_step has no GC; the
    // lane kernel runs mcts.cc:402-424 exactly) or the caller asks for lanes.
    const int64_t max_nodes = (q.max_memory_mb << 20) / 80 + 1;
    const int64_t worst = 1 + static_cast<int64_t>(p->max_simulations) * e->game.cfg.max_children;
    const bool gc_possible = max_nodes > 1 && worst >= max_nodes;
    if (e->az_layout == OS_LAYOUT_WAVE && gc_possible)
      return Fail(OS_ERR_UNSUPPORTED,
                  "the wave external-evaluator layout does not garbage-collect: raise "
                  "max_memory_mb or use OS_LAYOUT_LANE");
    e->az_wave = e->az_layout == OS_LAYOUT_WAVE || (e->az_layout == OS_LAYOUT_AUTO && !gc_possible);
  }
  e->az_kind = kind;
  e->az_obs = obs;
  e->az_legal = legal;
  e->az_prior = prior;
  e->az_value = value;
  e->az_pending = pending;
  // The step's request count: one counter per kAzShards-th of the searches,
  // each on its own 128-B line, summed into *pending after the step
  // (k_az_pending).  A single counter took every search's atomic at one
  // address: k_waz_step 0.208 -> 0.061 ms per launch at 16384 searches.
  {
    const size_t sb = sizeof(int32_t) * osm::kAzShards * osm::kAzShardStride + 64;  // + total
    if ((rc = e->d_az_shards.ensure(sb))) return rc;
    HIP_TRY(hipMemset(e->d_az_shards.p, 0, sb));
  }
  e->az_ready = true;
  e->az_stream = nullptr;
  return OS_OK;
}


int AzStep(os_engine* e, hipStream_t stream) {
  if (!e->az_ready) return Fail(OS_ERR_INVALID, "os_az_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(stream, &cap));
  if (cap == hipStreamCaptureStatusNone) e->az_stream = stream;
  const GameLaunchers* L = LaunchersFor(e->game.cfg);
  if (!L || !L->az) return Fail(OS_ERR_UNSUPPORTED, "game");
  return L->az(e, stream);
}

// Uploads one root + n evaluator seeds for the rollout kernels.
int RollPrepare(os_engine* e, const HostState& root, int64_t n, int32_t nr,
                const uint32_t* seeds) {
  if (BigBoard(e->game.cfg))
    return Fail(OS_ERR_UNSUPPORTED, "go / hex above 11 x 11 run searches only on the device");
  int rc;
  const size_t sb = e->game.state_bytes;
  if ((rc = e->d_roots.ensure(sb))) return rc;
  HIP_TRY(hipMemcpy(e->d_roots.p, root.raw, sb, hipMemcpyHostToDevice));
  if ((rc = e->d_bseed.ensure(std::max<int64_t>(n, 1) * 4))) return rc;
  if (n > 0) HIP_TRY(hipMemcpy(e->d_bseed.p, seeds, n * 4, hipMemcpyHostToDevice));
  if ((rc = e->d_mt.ensure(std::max<int64_t>(n, 1) * kMtN * 4))) return rc;
  if ((rc = e->d_rollout_out.ensure(std::max<int64_t>(n, 1) * 16))) return rc;
  if ((rc = e->d_roll_cnt.ensure(std::max<int64_t>(n, 1) * 8))) return rc;
  HIP_TRY(hipMemset(e->d_roll_cnt.p, 0, std::max<int64_t>(n, 1) * 8));
  e->roll_nhash = 0;
  if (e->game.cfg.kind == kGo) {
    if ((rc = e->d_glog.ensure(std::max<int64_t>(n, 1) * kGoLogCap * 8)) ||
        (rc = e->d_glink.ensure(std::max<int64_t>(n, 1) * kGoLogCap * 4)))
      return rc;
    if ((rc = UploadZob(e))) return rc;
    if ((rc = e->d_rhash.ensure(std::max<size_t>(root.hashes.size(), 1) * 8))) return rc;
    HIP_TRY(hipMemcpy(e->d_rhash.p, root.hashes.data(), root.hashes.size() * 8,
                      hipMemcpyHostToDevice));
    e->roll_nhash = static_cast<int32_t>(root.hashes.size());
  }
  e->roll_n = n;
  e->roll_nr = nr;
  e->roll_ready = true;
  e->num_roots = 0;  // the search buffers now hold no prepared batch
  e->sp_ready = false;
  e->az_ready = false;
  return OS_OK;
}


int RollRun(os_engine* e, hipStream_t stream) {
  if (!e->roll_ready) return Fail(OS_ERR_INVALID, "os_rollouts_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  if (e->roll_n == 0) return OS_OK;
  const GameLaunchers* L = LaunchersFor(e->game.cfg);
  if (!L || !L->rollouts)
    return Fail(OS_ERR_UNSUPPORTED, "go above 11 x 11 runs searches only on the device");
  return L->rollouts(e, stream);
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
extern "C" {

const char* os_last_error(void) { return g_err.c_str(); }

// Diagnostic (no reference counterpart): the first `count` arena nodes (24-B
// Node<double>) and priors of external-evaluator search r, copied to the host.
int os_debug_az_arena(os_engine* e, int64_t r, int32_t count, void* out_nodes,
                      double* out_prior) {
  if (!e || !e->az_ready || r < 0 || r >= e->num_roots || count < 0 ||
      static_cast<uint32_t>(count) > e->cap)
    return Fail(OS_ERR_INVALID, "bad argument");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  const size_t nb = sizeof(Node<double>);
  HIP_TRY(hipMemcpy(out_nodes, static_cast<unsigned char*>(e->d_arena.p) + r * e->cap * nb,
                    count * nb, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(out_prior, static_cast<double*>(e->d_az_prior.p) + r * e->cap, count * 8,
                    hipMemcpyDeviceToHost));
  return OS_OK;
}

int os_debug_phase_cycles(uint64_t* out, int32_t n) {
#if OS_PHASE_TIMING || OS_WAVE_TIMES
  if (!out || n < kDbgSlots) return Fail(OS_ERR_INVALID, "need kDbgSlots slots");
  // Each game's kernels live in their own code object: sum the counters (the
  // wave-time slots of the games that did not run are zero).
  std::vector<uint64_t> acc(kDbgSlots, 0), one(kDbgSlots, 0);
  for (int k = kTicTacToe; k <= kPig; ++k) {
    const int rc = LaunchersFor(k)->phase_cycles(one.data(), true);
    if (rc) return rc;
    for (int i = 0; i < kDbgSlots; ++i) acc[i] += one[i];
  }
  std::memcpy(out, acc.data(), sizeof(uint64_t) * kDbgSlots);
  return kDbgSlots;
#else
  (void)out;
  (void)n;
  return Fail(OS_ERR_UNSUPPORTED, "built without -DOS_PHASE_TIMING=1");
#endif
}

int64_t os_abi_struct_size(const char* name) {
  if (!name) return Fail(OS_ERR_INVALID, "null name");
  const std::string n(name);
  if (n == "os_mcts_params") return sizeof(os_mcts_params);
  if (n == "os_game_info") return sizeof(os_game_info);
  if (n == "os_selfplay_options") return sizeof(os_selfplay_options);
  return Fail(OS_ERR_INVALID, "unknown ABI struct " + n);
}

const char* os_build_info(void) {
  return "libos_mcts: gfx950 search/rollout kernels, one lane per search, "
         "-ffp-contract=off, lazy in-place MT19937";
}

int os_game_load(const char* game_string, os_game** out) {
  if (!game_string || !out) return Fail(OS_ERR_INVALID, "null argument");
  auto g = std::make_unique<os_game>();
  bool unsupported = false;
  std::string err = LoadHostGame(game_string, &g->g, &unsupported);
  if (!err.empty()) return Fail(unsupported ? OS_ERR_UNSUPPORTED : OS_ERR_INVALID, err);
  *out = g.release();
  return OS_OK;
}

void os_game_free(os_game* game) { delete game; }

int os_game_get_info(const os_game* game, os_game_info* o) {
  if (!game || !o) return Fail(OS_ERR_INVALID, "null argument");
  const GameCfg& c = game->g.cfg;
  std::memset(o, 0, sizeof *o);
  o->kind = c.kind;
  o->num_distinct_actions = c.num_actions;
  o->max_game_length = c.max_game_length;
  o->num_players = NumPlayers(c);
  o->max_children = c.max_children;
  o->rows = c.rows;
  o->cols = c.cols;
  o->min_utility = -1.0;
  o->max_utility = 1.0;
  o->utility_sum = 0.0;
  o->komi = c.komi;
  o->handicap = c.handicap;
  o->state_bytes = game->g.state_bytes;
  return OS_OK;
}

static int64_t CopyOut(const std::string& s, char* buf, int64_t cap) {
  if (buf && cap > 0) {
    const int64_t m = std::min<int64_t>(cap - 1, static_cast<int64_t>(s.size()));
    std::memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return static_cast<int64_t>(s.size());
}

int64_t os_game_to_string(const os_game* game, char* buf, int64_t cap) {
  return CopyOut(game->g.canonical, buf, cap);
}

int os_state_new(const os_game* game, os_state** out) {
  if (!game || !out) return Fail(OS_ERR_INVALID, "null argument");
  auto s = std::make_unique<os_state>();
  s->s.game = &game->g;
  StateInit(&s->s);
  *out = s.release();
  return OS_OK;
}

int os_state_clone(const os_state* s, os_state** out) {
  if (!s || !out) return Fail(OS_ERR_INVALID, "null argument");
  *out = new os_state(*s);
  return OS_OK;
}

void os_state_free(os_state* s) { delete s; }

int os_state_apply(os_state* s, int64_t action) {
  if (!s) return Fail(OS_ERR_INVALID, "null state");
  if (!StateApply(&s->s, action))
    return Fail(OS_ERR_INVALID, "illegal action " + std::to_string(action) +
                                    " in state\n" + StateToString(s->s));
  return OS_OK;
}

int32_t os_state_current_player(const os_state* s) { return StateCurrentPlayer(s->s); }
int32_t os_state_is_terminal(const os_state* s) { return StateTerminal(s->s) ? 1 : 0; }
int os_state_returns(const os_state* s, double* out2) {
  StateReturns(s->s, out2);
  return OS_OK;
}
int32_t os_state_is_chance_node(const os_state* s) { return StateIsChance(s->s) ? 1 : 0; }
int32_t os_state_chance_outcomes(const os_state* s, int64_t* actions, double* probs,
                                 int32_t cap) {
  std::vector<std::pair<int64_t, double>> o;
  StateChanceOutcomes(s->s, &o);
  for (int32_t i = 0; i < static_cast<int32_t>(o.size()) && i < cap; ++i) {
    actions[i] = o[i].first;
    probs[i] = o[i].second;
  }
  return static_cast<int32_t>(o.size());
}
int64_t os_game_observation_shape(const os_game* game, int32_t* shape3) {
  if (!game) return Fail(OS_ERR_INVALID, "null game");
  return ObservationShape(game->g, shape3);
}
int64_t os_state_observation_tensor(const os_state* s, int32_t player, float* out,
                                    int64_t cap) {
  if (!s) return Fail(OS_ERR_INVALID, "null state");
  if (player < 0 || player >= NumPlayers(s->s.game->cfg))
    return Fail(OS_ERR_INVALID, "player out of range");
  const int64_t n = ObservationShape(*s->s.game, nullptr);
  if (out && cap >= n) StateObservation(s->s, player, out);
  return n;
}
int32_t os_state_legal_actions(const os_state* s, int64_t* out, int32_t cap) {
  std::vector<int64_t> v;
  StateLegal(s->s, &v);
  for (int32_t i = 0; i < cap && i < static_cast<int32_t>(v.size()); ++i) out[i] = v[i];
  return static_cast<int32_t>(v.size());
}
int32_t os_state_history(const os_state* s, int64_t* out, int32_t cap) {
  const auto& h = s->s.history;
  for (int32_t i = 0; i < cap && i < static_cast<int32_t>(h.size()); ++i) out[i] = h[i];
  return static_cast<int32_t>(h.size());
}
int64_t os_state_to_string(const os_state* s, char* buf, int64_t cap) {
  return CopyOut(StateToString(s->s), buf, cap);
}
int64_t os_state_action_to_string(const os_state* s, int32_t player, int64_t action,
                                  char* buf, int64_t cap) {
  return CopyOut(StateActionToString(s->s, player, action), buf, cap);
}

int os_engine_create(const char* game_string, int32_t device, os_engine** out) {
  if (!game_string || !out) return Fail(OS_ERR_INVALID, "null argument");
  auto e = std::make_unique<os_engine>();
  bool unsupported = false;
  std::string err = LoadHostGame(game_string, &e->game, &unsupported);
  if (!err.empty()) return Fail(unsupported ? OS_ERR_UNSUPPORTED : OS_ERR_INVALID, err);
  const GameCfg& cfg = e->game.cfg;
  if ((cfg.kind == kHex || cfg.kind == kGo) && cfg.rows > kGoDeviceMaxSide)
    return Fail(OS_ERR_UNSUPPORTED,
                "the device engine runs hex / go up to 19 x 19 (lane-layout searches above "
                "11 x 11)");
  int ndev = 0;
  hipError_t he = hipGetDeviceCount(&ndev);
  if (he != hipSuccess || ndev == 0)
    return Fail(OS_ERR_DEVICE, std::string("no HIP device available: ") +
                                   (he != hipSuccess ? hipGetErrorString(he) : "0 devices"));
  if (device < 0 || device >= ndev)
    return Fail(OS_ERR_INVALID, "device index out of range");
  e->device = device;
  HIP_TRY(hipSetDevice(device));
  *out = e.release();
  return OS_OK;
}

int os_engine_destroy(os_engine* e) {
  delete e;
  return OS_OK;
}

int os_engine_prepare(os_engine* e, const os_mcts_params* p, int64_t num_roots,
                      const int64_t* root_actions, const int64_t* root_offsets,
                      const uint32_t* bot_seeds, const uint32_t* eval_seeds) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return Prepare(e, p, num_roots, root_actions, root_offsets, bot_seeds, eval_seeds);
}

int os_engine_run_async(os_engine* e, void* hip_stream) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return Run(e, static_cast<hipStream_t>(hip_stream));
}

int os_engine_fetch(os_engine* e, int32_t max_children, int32_t* child_action,
                    int32_t* child_n, double* child_w, int8_t* child_out,
                    int32_t* nchild, int32_t* root_n, double* root_w,
                    int8_t* root_out, int64_t* best_action, int32_t* nodes) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return Fetch(e, max_children, child_action, child_n, child_w, child_out, nchild,
               root_n, root_w, root_out, best_action, nodes);
}

int64_t os_engine_last_sims(os_engine* e) { return e ? e->last_sims : -1; }

int os_engine_get_layout(os_engine* e, int32_t* layout) {
  if (!e || !layout) return Fail(OS_ERR_INVALID, "null argument");
  if (e->search_layout < 0) return Fail(OS_ERR_INVALID, "no os_engine_prepare batch");
  *layout = e->search_layout;
  return OS_OK;
}

int os_engine_get_searches_per_wave(os_engine* e, int32_t* searches) {
  if (!e || !searches) return Fail(OS_ERR_INVALID, "null argument");
  if (e->search_lanes <= 0) return Fail(OS_ERR_INVALID, "no search launched yet");
  *searches = e->search_lanes;
  return OS_OK;
}

int os_engine_set_rollout_layout(os_engine* e, int32_t layout) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (layout != OS_LAYOUT_WAVE && layout != OS_LAYOUT_LANE)
    return Fail(OS_ERR_INVALID, "unknown layout");
  e->rollout_layout = layout;
  return OS_OK;
}

int os_engine_stats(os_engine* e, int64_t* out) {
  if (!e || !out) return Fail(OS_ERR_INVALID, "null argument");
  for (int i = 0; i < 10; ++i) out[i] = 0;
  for (const SearchResult& s : e->last_results) {
    out[0] += s.sims;
    out[1] += s.scanned;
    out[2] += s.backed;
    out[3] += s.expanded;
    out[4] += s.solver_scanned;
    out[5] += s.rng_words;
    out[6] += s.nodes;
    out[7] += s.used;
    out[8] = std::max<int64_t>(out[8], s.max_depth);
    out[9] += s.gc_runs;
  }
  return OS_OK;
}

int32_t os_engine_node_bytes(os_engine* e) { return e ? e->node_bytes : -1; }
int32_t os_engine_state_bytes(os_engine* e) { return e ? e->game.state_bytes : -1; }

int os_mcts_batch(os_engine* e, const os_mcts_params* p, int64_t num_roots,
                  const int64_t* root_actions, const int64_t* root_offsets,
                  const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                  int32_t max_children, int32_t* child_action, int32_t* child_n,
                  double* child_w, int8_t* child_out, int32_t* nchild,
                  int32_t* root_n, double* root_w, int8_t* root_out,
                  int64_t* best_action, int32_t* nodes) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  int rc = Prepare(e, p, num_roots, root_actions, root_offsets, bot_seeds, eval_seeds);
  if (rc) return rc;
  if ((rc = Run(e, nullptr))) return rc;
  return Fetch(e, max_children, child_action, child_n, child_w, child_out, nchild,
               root_n, root_w, root_out, best_action, nodes);
}

int os_mcts_stateful(os_engine* e, const os_mcts_params* p,
                        const int64_t* root_actions, int64_t n_actions,
                        int32_t shared, uint32_t* bot_key, int32_t* bot_pos,
                        uint32_t* eval_key, int32_t* eval_pos,
                        int32_t max_children, int32_t* child_action,
                        int32_t* child_n, double* child_w, int8_t* child_out,
                        int32_t* nchild, int32_t* root_n, double* root_w,
                        int8_t* root_out, int64_t* best_action, int32_t* nodes) {
  if (!e || !p || !bot_key || !bot_pos) return Fail(OS_ERR_INVALID, "null argument");
  if (shared && p->policy != OS_POLICY_NUMPY)
    return Fail(OS_ERR_INVALID, "a shared stream needs OS_POLICY_NUMPY");
  if (!shared && (!eval_key || !eval_pos))
    return Fail(OS_ERR_INVALID, "separate evaluator stream needs eval_key/eval_pos");
  int64_t offs[2] = {0, n_actions};
  uint32_t zero = 0;
  int rc = Prepare(e, p, 1, root_actions, offs, &zero, &zero);
  if (rc) return rc;
  e->import_state = true;
  e->shared_stream = shared != 0;
  int32_t pos[2] = {*bot_pos, shared ? 0 : *eval_pos};
  {
    Stager st(e);
    if ((rc = st.reserve(2 * kMtN * 4 + 3 * 256)) ||
        (rc = st.up(e->d_mt.p, bot_key, kMtN * 4)) ||
        (!shared && (rc = st.up(static_cast<uint32_t*>(e->d_mt.p) + kMtN, eval_key, kMtN * 4))) ||
        (rc = st.up(e->d_pos.p, pos, 8)))
      return rc;
    // No wait: the null stream runs these copies before the search kernel.
  }
  if ((rc = Run(e, nullptr))) {
    (void)hipStreamSynchronize(nullptr);  // the queued copies still read h_stage
    e->import_state = false;
    return rc;
  }
  rc = Fetch(e, max_children, child_action, child_n, child_w, child_out, nchild, root_n,
             root_w, root_out, best_action, nodes);
  e->import_state = false;
  if (rc) return rc;
  {
    Stager st(e);
    unsigned char *bk, *ek = nullptr, *ps;
    if ((rc = st.reserve(2 * kMtN * 4 + 3 * 256)) || (rc = st.down(&bk, e->d_mt.p, kMtN * 4)) ||
        (!shared &&
         (rc = st.down(&ek, static_cast<uint32_t*>(e->d_mt.p) + kMtN, kMtN * 4))) ||
        (rc = st.down(&ps, e->d_pos.p, 8)) || (rc = st.wait()))
      return rc;
    std::memcpy(bot_key, bk, kMtN * 4);
    std::memcpy(pos, ps, 8);
    *bot_pos = pos[0];
    if (!shared) {
      std::memcpy(eval_key, ek, kMtN * 4);
      *eval_pos = pos[1];
    }
  }
  return OS_OK;
}

// Copies node x into the export arrays at slot o.
extern "C++" template <class N>
static void ExportNodeT(const N& x, uint32_t o, uint32_t first, uint32_t* out_first, int32_t* n,
                        double* w, int32_t* action, int32_t* nchild, int8_t* out0) {
  n[o] = x.n; w[o] = static_cast<double>(x.w); action[o] = x.action; nchild[o] = x.nchild;
  out0[o] = x.out;
  out_first[o] = first;
}

// Tree r of the last run as arrays in arena-index order.  Reserved arena: one
// copy of the tree's `used` nodes.  Paged: the tree's child blocks lie on the
// root's page and on pages taken later (higher page numbers, filled upward),
// so index order is allocation order; walk the tree from the root, reading
// each page once, and renumber the blocks in index order: the same arrays as
// the reserved arena.
extern "C++" template <class N>
static int ExportTree(os_engine* e, int64_t r, uint32_t used, uint32_t* first, int32_t* n,
                      double* w, int32_t* action, int32_t* nchild, int8_t* out0) {
  unsigned char* const arena = static_cast<unsigned char*>(e->d_arena.p);
  if (!e->paged) {
    std::vector<N> raw(used);
    HIP_TRY(hipMemcpy(raw.data(), arena + static_cast<size_t>(r) * e->cap * sizeof(N),
                      used * sizeof(N), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < used; ++i)
      ExportNodeT(raw[i], i, raw[i].first, first, n, w, action, nchild, out0);
    return OS_OK;
  }
  const uint64_t pn = e->page_nodes;
  const uint64_t base = static_cast<uint64_t>(r) * pn;  // node indices are relative to it
  std::map<uint64_t, std::vector<N>> pages;
  auto node_at = [&](uint64_t rel) -> const N* {
    const uint64_t g = base + rel, pg = g / pn;
    auto it = pages.find(pg);
    if (it == pages.end()) {
      std::vector<N> buf(pn);
      if (hipMemcpy(buf.data(), arena + pg * pn * sizeof(N), pn * sizeof(N),
                    hipMemcpyDeviceToHost) != hipSuccess)
        return nullptr;
      it = pages.emplace(pg, std::move(buf)).first;
    }
    return &it->second[g - pg * pn];
  };
  struct Blk { uint32_t rel, cnt; };
  std::vector<Blk> blocks{{0u, 1u}};  // the root is a block of one
  for (size_t b = 0; b < blocks.size(); ++b) {
    for (uint32_t k = 0; k < blocks[b].cnt; ++k) {
      const N* p = node_at(blocks[b].rel + k);
      if (!p) return Fail(OS_ERR_DEVICE, "tree export copy failed");
      if (p->nchild) blocks.push_back({p->first, static_cast<uint32_t>(p->nchild)});
    }
  }
  std::sort(blocks.begin(), blocks.end(), [](const Blk& a, const Blk& b) { return a.rel < b.rel; });
  std::unordered_map<uint32_t, uint32_t> renum;  // block start -> export index
  uint32_t o = 0;
  for (const Blk& b : blocks) { renum[b.rel] = o; o += b.cnt; }
  if (o != used) return Fail(OS_ERR_DEVICE, "paged tree export: node count mismatch");
  o = 0;
  for (const Blk& b : blocks) {
    for (uint32_t k = 0; k < b.cnt; ++k, ++o) {
      const N* p = node_at(b.rel + k);
      // A childless node keeps the reserved arena's first (0).
      ExportNodeT(*p, o, p->nchild ? renum[p->first] : 0u, first, n, w, action, nchild, out0);
    }
  }
  return OS_OK;
}

int os_engine_tree(os_engine* e, int64_t r, int64_t* count, uint32_t* first,
                   int32_t* n, double* w, int32_t* action, int32_t* nchild,
                   int8_t* out0) {
  if (!e || !count) return Fail(OS_ERR_INVALID, "null argument");
  if (r < 0 || r >= e->num_roots || r >= static_cast<int64_t>(e->last_results.size()))
    return Fail(OS_ERR_INVALID, "root index out of range (fetch first)");
  if (e->num_roots > e->chunk_roots)
    return Fail(OS_ERR_UNSUPPORTED, "tree export needs a single-chunk run");
  const uint32_t used = e->last_results[r].used;
  *count = used;
  if (!first) return OS_OK;
  HIP_TRY(hipSetDevice(e->device));
  if (e->node_wide)  // k_lsearch's wide nodes (go / hex above 11 x 11)
    return e->node_double
               ? ExportTree<Node<double, true>>(e, r, used, first, n, w, action, nchild, out0)
               : ExportTree<Node<int32_t, true>>(e, r, used, first, n, w, action, nchild, out0);
  return e->node_double
             ? ExportTree<Node<double>>(e, r, used, first, n, w, action, nchild, out0)
             : ExportTree<Node<int32_t>>(e, r, used, first, n, w, action, nchild, out0);
}

int os_engine_set_arena_mode(os_engine* e, int32_t mode) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (mode != OS_ARENA_RESERVED && mode != OS_ARENA_PAGED)
    return Fail(OS_ERR_INVALID, "unknown arena mode");
  e->arena_mode = mode;
  return OS_OK;
}

int os_engine_arena_info(os_engine* e, int64_t* out) {
  if (!e || !out) return Fail(OS_ERR_INVALID, "null argument");
  out[0] = e->paged ? 1 : 0;
  out[1] = e->paged ? e->page_nodes : e->cap;
  out[2] = e->paged ? e->pool_pages : e->chunk_roots;
  out[3] = static_cast<int64_t>(e->arena_bytes);
  uint32_t dyn = 0;
  if (e->paged && e->d_page_next.p) {
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&dyn, e->d_page_next.p, 4, hipMemcpyDeviceToHost));
  }
  out[4] = e->paged ? e->num_roots + dyn : 0;
  out[5] = e->arena_reruns;
  out[6] = e->arena_overflows;
  // The reserved arena the batch would take: worst case per root x roots.
  const GameCfg& cfg = e->game.cfg;
  out[7] = (1 + static_cast<int64_t>(e->params.max_simulations) * cfg.max_children) *
           e->num_roots * e->node_bytes;
  return OS_OK;
}

int os_az_prepare(os_engine* e, const os_mcts_params* p, int32_t puct, int64_t num_roots,
                  const int64_t* root_actions, const int64_t* root_offsets,
                  const uint32_t* bot_seeds, double dirichlet_alpha,
                  double dirichlet_epsilon, int32_t* dev_kind, float* dev_obs,
                  uint8_t* dev_legal, const double* dev_prior, const double* dev_value,
                  int32_t* dev_pending) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return AzPrepare(e, p, puct, num_roots, root_actions, root_offsets, bot_seeds,
                   dirichlet_alpha, dirichlet_epsilon, dev_kind, dev_obs, dev_legal, dev_prior,
                   dev_value, dev_pending);
}

int os_az_stage(os_engine* e, const os_mcts_params* p, int32_t puct, int64_t num_roots,
                const int64_t* root_actions, const int64_t* root_offsets,
                const uint32_t* bot_seeds, double dirichlet_alpha, double dirichlet_epsilon) {
  if (!e || !p) return Fail(OS_ERR_INVALID, "null argument");
  if (num_roots < 0 || (num_roots > 0 && (!root_offsets || !bot_seeds)))
    return Fail(OS_ERR_INVALID, "bad batch");
  if (p->policy != OS_POLICY_CPP)
    return Fail(OS_ERR_UNSUPPORTED, "os_az_stage: C++-policy batches (seeded bots)");
  if (!(dirichlet_alpha >= 0.0) || !(dirichlet_epsilon >= 0.0) || dirichlet_epsilon > 1.0)
    return Fail(OS_ERR_INVALID, "dirichlet_alpha must be >= 0 and epsilon in [0, 1]");
  os_engine::AzStaged& st = e->az_staged;
  st.ready = false;
  const int64_t R = num_roots;
  st.p = *p;
  st.puct = puct;
  st.R = R;
  st.alpha = dirichlet_alpha;
  st.eps = dirichlet_epsilon;
  st.offs.assign(root_offsets, root_offsets + R + 1);
  st.acts.assign(root_actions, root_actions + (R > 0 ? root_offsets[R] : 0));
  st.seeds.assign(bot_seeds, bot_seeds + R);
  std::vector<int32_t> nlegal;
  int rc = ReplayRoots(e, R, st.acts.data(), st.offs.data(), &st.roots, &st.rh, &st.rnh,
                       dirichlet_alpha > 0.0 ? &nlegal : nullptr);
  if (rc) return rc;
  st.noise.clear();
  st.skip.clear();
  if (dirichlet_alpha > 0.0 &&
      (rc = DrawRootNoise(e, R, nlegal, st.seeds.data(), nullptr, nullptr, dirichlet_alpha,
                          &st.noise, &st.skip)))
    return rc;
  st.ready = true;
  return OS_OK;
}

int os_az_prepare_staged(os_engine* e, int32_t* dev_kind, float* dev_obs, uint8_t* dev_legal,
                         const double* dev_prior, const double* dev_value,
                         int32_t* dev_pending) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  os_engine::AzStaged& st = e->az_staged;
  if (!st.ready) return Fail(OS_ERR_INVALID, "no os_az_stage batch");
  st.ready = false;  // consumed
  return AzPrepare(e, &st.p, st.puct, st.R, st.acts.data(), st.offs.data(), st.seeds.data(),
                   st.alpha, st.eps, dev_kind, dev_obs, dev_legal, dev_prior, dev_value,
                   dev_pending, nullptr, nullptr, &st);
}

int os_az_prepare_stateful(os_engine* e, const os_mcts_params* p, int32_t puct,
                           int64_t num_roots, const int64_t* root_actions,
                           const int64_t* root_offsets, const uint32_t* bot_keys,
                           const int32_t* bot_pos, double dirichlet_alpha,
                           double dirichlet_epsilon, int32_t* dev_kind, float* dev_obs,
                           uint8_t* dev_legal, const double* dev_prior, const double* dev_value,
                           int32_t* dev_pending) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (num_roots > 0 && (!bot_keys || !bot_pos)) return Fail(OS_ERR_INVALID, "null rng state");
  return AzPrepare(e, p, puct, num_roots, root_actions, root_offsets, nullptr, dirichlet_alpha,
                   dirichlet_epsilon, dev_kind, dev_obs, dev_legal, dev_prior, dev_value,
                   dev_pending, bot_keys ? bot_keys : nullptr, bot_pos);
}

int os_az_set_layout(os_engine* e, int32_t layout) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (layout != OS_LAYOUT_WAVE && layout != OS_LAYOUT_LANE && layout != OS_LAYOUT_AUTO)
    return Fail(OS_ERR_INVALID, "unknown layout");
  e->az_layout = layout;
  return OS_OK;
}

int os_engine_set_run_timing(os_engine* e, int32_t on) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  e->time_runs = on != 0;
  e->run_timed = false;
  return OS_OK;
}

int os_engine_last_run_ms(os_engine* e, double* ms) {
  if (!e || !ms) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->run_timed) return Fail(OS_ERR_INVALID, "no timed run (os_engine_set_run_timing)");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipEventSynchronize(e->run_ev[1]));
  float f = 0.0f;
  HIP_TRY(hipEventElapsedTime(&f, e->run_ev[0], e->run_ev[1]));
  *ms = f;
  return OS_OK;
}

int os_az_get_layout(os_engine* e, int32_t* layout) {
  if (!e || !layout) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->az_ready) return Fail(OS_ERR_INVALID, "no os_az_prepare batch");
  *layout = e->az_wave ? OS_LAYOUT_WAVE : OS_LAYOUT_LANE;
  return OS_OK;
}

int os_az_set_noise(os_engine* e, const double* noise, int64_t stride, double eps) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (!e->az_ready) return Fail(OS_ERR_INVALID, "no os_az_prepare batch");
  if (!(eps >= 0.0) || eps > 1.0) return Fail(OS_ERR_INVALID, "epsilon must be in [0, 1]");
  if (e->params.max_memory_mb != 0 &&
      1 + static_cast<int64_t>(e->params.max_simulations) * e->game.cfg.max_children >=
          (e->params.max_memory_mb << 20) / 80 + 1)
    return Fail(OS_ERR_UNSUPPORTED, "root noise with a node budget small enough for GC to fire");
  const int64_t R = e->num_roots;
  const int mc = e->game.cfg.max_children;
  if (!noise) {
    e->az_noise = false;
    return OS_OK;
  }
  if (stride < mc) return Fail(OS_ERR_INVALID, "noise stride below max_children");
  const size_t Rz = static_cast<size_t>(std::max<int64_t>(R, 1));
  std::vector<double> packed(Rz * mc, 0.0);
  for (int64_t r = 0; r < R; ++r)
    std::memcpy(packed.data() + r * mc, noise + r * stride, mc * 8);
  std::vector<int32_t> skip(Rz, 0);  // drawn by the caller: no bot words to skip
  int rc;
  if ((rc = e->d_az_noise.ensure(packed.size() * 8)) || (rc = e->d_az_skip.ensure(Rz * 4)))
    return rc;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipMemcpy(e->d_az_noise.p, packed.data(), packed.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_az_skip.p, skip.data(), Rz * 4, hipMemcpyHostToDevice));
  e->az_noise = true;
  e->az_eps = eps;
  return OS_OK;
}

int os_az_tree_priors(os_engine* e, int64_t r, int64_t count, double* prior) {
  if (!e || !prior) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->az_ready) return Fail(OS_ERR_INVALID, "no os_az_prepare batch");
  if (r < 0 || r >= e->num_roots || r >= static_cast<int64_t>(e->last_results.size()))
    return Fail(OS_ERR_INVALID, "root index out of range (os_az_fetch first)");
  if (count != static_cast<int64_t>(e->last_results[r].used))
    return Fail(OS_ERR_INVALID, "count must be the tree's node count (os_engine_tree)");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipMemcpy(prior, static_cast<const double*>(e->d_az_prior.p) + r * e->cap, count * 8,
                    hipMemcpyDeviceToHost));
  return OS_OK;
}

int os_az_requests(os_engine* e, int64_t* total) {
  if (!e || !total) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->az_ready) return Fail(OS_ERR_INVALID, "no os_az_prepare batch");
  HIP_TRY(hipSetDevice(e->device));
  // k_az_pending wrote the total on the steps' stream: copy it there
  HIP_TRY(hipMemcpyAsync(total, static_cast<int32_t*>(e->d_az_shards.p) + osm::kAzShards * osm::kAzShardStride,
                         8, hipMemcpyDeviceToHost, e->az_stream));
  HIP_TRY(hipStreamSynchronize(e->az_stream));
  return OS_OK;
}

int os_az_set_requests(os_engine* e, int32_t mode) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (mode != OS_AZ_REQUESTS_SEPARATE && mode != OS_AZ_REQUESTS_FUSED)
    return Fail(OS_ERR_INVALID, "unknown request mode");
  e->az_requests = mode;
  return OS_OK;
}

int os_az_export_rng(os_engine* e, uint32_t* bot_keys, int32_t* bot_pos) {
  if (!e || !bot_keys || !bot_pos) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->az_ready || !e->az_import)
    return Fail(OS_ERR_INVALID, "no os_az_prepare_stateful batch");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->az_stream));
  int32_t pending = 0;
  HIP_TRY(hipMemcpy(&pending, e->az_pending, 4, hipMemcpyDeviceToHost));
  if (pending != 0) return Fail(OS_ERR_INVALID, "searches still wait for the evaluator");
  const int64_t R = e->num_roots;
  if (R == 0) return OS_OK;
  HIP_TRY(hipMemcpy(bot_keys, e->d_mt.p, static_cast<size_t>(R) * kMtN * 4,
                    hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(bot_pos, static_cast<int32_t*>(e->d_az_pos.p) + R,
                    static_cast<size_t>(R) * 4, hipMemcpyDeviceToHost));
  return OS_OK;
}

int64_t os_dirichlet_noise(uint32_t seed, int32_t count, double alpha, double* out) {
  if (count < 0 || (count > 0 && !out)) return Fail(OS_ERR_INVALID, "null argument");
  if (!(alpha > 0.0)) return Fail(OS_ERR_INVALID, "alpha must be > 0");
  return DirichletNoise(seed, count, alpha, out);
}

// One thread per row (rows are requests; num_actions is small next to them).
__global__ void k_az_heads(const void* logits, int32_t dtype, int64_t R, int32_t A, int64_t ld,
                           const uint8_t* legal, double* prior, double* value) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= R) return;
  auto get = [&](int a) -> double {
    const int64_t i = r * ld + a;
    if (dtype == 0) return static_cast<double>(static_cast<const float*>(logits)[i]);
    const uint32_t b = static_cast<uint32_t>(static_cast<const uint16_t*>(logits)[i]) << 16;
    return static_cast<double>(__uint_as_float(b));
  };
  const uint8_t* lg = legal + r * A;
  double m = -__builtin_huge_val();
  for (int a = 0; a < A; ++a) m = fmax(m, lg[a] ? get(a) : -1e32);
  double s = 0.0;
  for (int a = 0; a < A; ++a) s += exp((lg[a] ? get(a) : -1e32) - m);
  double* pr = prior + r * A;
  for (int a = 0; a < A; ++a) pr[a] = exp((lg[a] ? get(a) : -1e32) - m) / s;
  value[r] = tanh(get(A));
}

// A one-hidden-layer policy / value network fused with its heads, for a
// batched external-evaluator round (the bench's stand-in network; an
// evaluator may use it through os_az_mlp_heads_async):
//   h      = relu(bf16(obs) . W1)            hidden units, f32 accumulation, bf16
//   logits = bf16(h . Wout)                  A policy logits, then the value logit
//   prior  = softmax over the legal actions, value = tanh   (k_az_heads, f64)
// One wave owns 16 rows.  Both products run on the matrix cores
// (v_mfma_f32_16x16x32_bf16) transposed -- H^T = W1^T . X^T, then
// L^T = Wout^T . H^T -- so the first product's accumulators (hidden on the
// register index, the row on the lane) are the second one's B operand with no
// lane movement: lane group g of a 32-hidden chunk holds hidden units
// {4g..4g+3} of its two 16-unit tiles, and the A operand (Wout) is read in that
// same k order.  Weights: w1t bf16 [hidden][128] (K padded with zeros),
// wout bf16 [16][hidden] (rows A + 1 .. 15 zero); obs_size <= 128,
// hidden <= 256 and a multiple of 32, A + 1 <= 16.
using AzFragAB = __attribute__((ext_vector_type(8))) short;
using AzFragCD = __attribute__((ext_vector_type(4))) float;
constexpr int kAzMlpK = 128;
constexpr int kAzMlpMaxHidden = 256;

__device__ __forceinline__ uint16_t az_bf16(float f) {  // round to nearest even
  const uint32_t u = __float_as_uint(f);
  return static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

__global__ __launch_bounds__(64) void k_az_mlp_heads(const float* obs, int64_t R, int32_t obs_size,
                                                     const uint16_t* w1t, int32_t hidden,
                                                     const uint16_t* wout, int32_t A,
                                                     const uint8_t* legal, double* prior,
                                                     double* value) {
  __shared__ float lg[16][17];
  const int l = threadIdx.x;
  const int g = l >> 4, c16 = l & 15;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * 16;
  const int64_t row = row0 + c16;
  const bool live = row < R;
  // X^T fragments (B of the first product): obs[row][32c + 8g + j], j < 8
  AzFragAB xb[kAzMlpK / 32];
#pragma unroll
  for (int c = 0; c < kAzMlpK / 32; ++c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * c + 8 * g + j;
      const float v = (live && k < obs_size) ? obs[row * obs_size + k] : 0.0f;
      xb[c][j] = static_cast<short>(az_bf16(v));
    }
  }
  const int tiles = hidden / 16;
  AzFragCD out = {0.0f, 0.0f, 0.0f, 0.0f};
  // hidden chunk by chunk (two 16-unit tiles = 32 units): the chunk's H^T
  // tiles, then their contribution to L^T
  for (int c2 = 0; c2 < tiles / 2; ++c2) {
    AzFragCD h[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = 2 * c2 + u;
      AzFragCD acc = {0.0f, 0.0f, 0.0f, 0.0f};
      const uint16_t* wrow = w1t + static_cast<int64_t>(16 * t + c16) * kAzMlpK + 8 * g;
#pragma unroll
      for (int c = 0; c < kAzMlpK / 32; ++c) {
        const AzFragAB a = *reinterpret_cast<const AzFragAB*>(wrow + 32 * c);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xb[c], acc, 0, 0, 0);
      }
      h[u] = acc;  // H^T[16t + 4g + r][row]
    }
    // B of the second product: element j <- hidden 32 c2 + (j < 4 ? 4g + j : 16 + 4g + j - 4)
    AzFragAB hb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = h[j >> 2][j & 3];
      hb[j] = static_cast<short>(az_bf16(v > 0.0f ? v : 0.0f));  // relu, bf16
    }
    // A of the second product: Wout^T[o = c16][same k order]
    const uint16_t* wo = wout + static_cast<int64_t>(c16) * hidden + 32 * c2 + 4 * g;
    AzFragAB ab;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ab[j] = static_cast<short>(wo[j]);
      ab[4 + j] = static_cast<short>(wo[16 + j]);
    }
    out = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, hb, out, 0, 0, 0);
  }
  // L^T[o = 4g + r][row c16] -> LDS [row][o], rounded to bf16 like the GEMM's output
#pragma unroll
  for (int r = 0; r < 4; ++r)
    lg[c16][4 * g + r] = __uint_as_float(static_cast<uint32_t>(az_bf16(out[r])) << 16);
  __syncthreads();
  if (l >= 16 || !live) return;
  // heads (k_az_heads' arithmetic)
  const uint8_t* lm = legal + row * A;
  double m = -__builtin_huge_val();
  for (int a = 0; a < A; ++a) m = fmax(m, lm[a] ? static_cast<double>(lg[l][a]) : -1e32);
  double sum = 0.0;
  for (int a = 0; a < A; ++a) sum += exp((lm[a] ? static_cast<double>(lg[l][a]) : -1e32) - m);
  double* pr = prior + row * A;
  for (int a = 0; a < A; ++a) pr[a] = exp((lm[a] ? static_cast<double>(lg[l][a]) : -1e32) - m) / sum;
  value[row] = tanh(static_cast<double>(lg[l][A]));
}

int os_az_mlp_heads_async(const float* obs, int64_t num_rows, int32_t obs_size,
                          const uint16_t* w1t, int32_t hidden, const uint16_t* wout,
                          int32_t num_actions, const uint8_t* legal, double* prior,
                          double* value, void* hip_stream) {
  if (num_rows < 0 || obs_size < 1 || obs_size > kAzMlpK || hidden < 32 ||
      hidden > kAzMlpMaxHidden || hidden % 32 != 0 || num_actions < 1 || num_actions + 1 > 16)
    return Fail(OS_ERR_INVALID, "bad network shape (obs <= 128, hidden % 32 == 0 and <= 256, "
                                "actions + 1 <= 16)");
  if (num_rows == 0) return OS_OK;
  if (!obs || !w1t || !wout || !legal || !prior || !value)
    return Fail(OS_ERR_INVALID, "null network buffer");
  const unsigned blocks = static_cast<unsigned>((num_rows + 15) / 16);
  hipLaunchKernelGGL(k_az_mlp_heads, dim3(blocks), dim3(64), 0,
                     static_cast<hipStream_t>(hip_stream), obs, num_rows, obs_size, w1t, hidden,
                     wout, num_actions, legal, prior, value);
  HIP_TRY(hipGetLastError());
  return OS_OK;
}

int os_az_heads_async(const void* logits, int32_t dtype, int64_t num_rows, int32_t num_actions,
                      int64_t ld, const uint8_t* legal, double* prior, double* value,
                      void* hip_stream) {
  if (num_rows < 0 || num_actions < 1 || ld < num_actions + 1 || (dtype != 0 && dtype != 1))
    return Fail(OS_ERR_INVALID, "bad heads shape / dtype");
  if (num_rows == 0) return OS_OK;
  if (!logits || !legal || !prior || !value) return Fail(OS_ERR_INVALID, "null heads buffer");
  const unsigned blocks = static_cast<unsigned>((num_rows + 255) / 256);
  hipLaunchKernelGGL(k_az_heads, dim3(blocks), dim3(256), 0,
                     static_cast<hipStream_t>(hip_stream), logits, dtype, num_rows, num_actions,
                     ld, legal, prior, value);
  HIP_TRY(hipGetLastError());
  return OS_OK;
}

int os_az_step_async(os_engine* e, void* hip_stream) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return AzStep(e, static_cast<hipStream_t>(hip_stream));
}

int os_az_fetch(os_engine* e, int32_t max_children, int32_t* child_action, int32_t* child_n,
                double* child_w, int8_t* child_out, int32_t* nchild, int32_t* root_n,
                double* root_w, int8_t* root_out, int64_t* best_action, int32_t* nodes) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (!e->az_ready) return Fail(OS_ERR_INVALID, "os_az_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->az_stream));
  int32_t pending = 0;
  HIP_TRY(hipMemcpy(&pending, e->az_pending, 4, hipMemcpyDeviceToHost));
  if (pending != 0)
    return Fail(OS_ERR_INVALID, std::to_string(pending) +
                                    " searches still wait for the evaluator: step again");
  return Fetch(e, max_children, child_action, child_n, child_w, child_out, nchild, root_n,
               root_w, root_out, best_action, nodes);
}

int os_selfplay_prepare(os_engine* e, const os_mcts_params* p, int64_t num_games,
                        const int64_t* start_actions, const int64_t* start_offsets,
                        const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                        int32_t max_len, int32_t record) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return SpPrepare(e, p, num_games, start_actions, start_offsets, bot_seeds, eval_seeds,
                   max_len, record);
}

int os_selfplay_set_options(os_engine* e, const os_selfplay_options* o, int64_t num_games,
                            const uint32_t* actor_seeds) {
  if (!e || !o) return Fail(OS_ERR_INVALID, "null argument");
  if (o->temperature > 0.0 && !(o->temperature < 1e300))
    return Fail(OS_ERR_INVALID, "temperature must be finite");
  if (o->resign && (!(o->cutoff_probability >= 0.0) || o->cutoff_probability > 1.0))
    return Fail(OS_ERR_INVALID, "cutoff_probability must be in [0, 1]");
  if (num_games < 0 || (num_games > 0 && !actor_seeds))
    return Fail(OS_ERR_INVALID, "actor seeds needed for every game");
  e->sp_opts = *o;
  e->sp_actor_seeds.assign(actor_seeds, actor_seeds + num_games);
  e->sp_ready = false;  // takes effect at the next os_selfplay_prepare
  return OS_OK;
}

int os_selfplay_fetch_targets(os_engine* e, double* policy, double* root_values) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  if (!e->sp_ready) return Fail(OS_ERR_INVALID, "os_selfplay_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  const size_t GL = static_cast<size_t>(e->sp_games) * e->sp_max_len;
  if (policy) {
    if (!e->sp_policy) return Fail(OS_ERR_INVALID, "prepared without OS_RECORD_POLICY");
    HIP_TRY(hipMemcpy(policy, e->d_sp_pol.p, GL * e->game.cfg.num_actions * 8,
                      hipMemcpyDeviceToHost));
  }
  if (root_values) {
    if (!e->sp_values) return Fail(OS_ERR_INVALID, "prepared without OS_RECORD_ROOT_VALUES");
    HIP_TRY(hipMemcpy(root_values, e->d_sp_val.p, GL * 8, hipMemcpyDeviceToHost));
  }
  return OS_OK;
}

int os_selfplay_run_async(os_engine* e, void* hip_stream) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return SpRun(e, static_cast<hipStream_t>(hip_stream));
}

int os_selfplay_fetch(os_engine* e, int64_t* actions, int32_t* length, double* returns,
                      int32_t* visits, float* observations) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return SpFetch(e, actions, length, returns, visits, observations);
}

int os_selfplay(os_engine* e, const os_mcts_params* p, int64_t num_games,
                const int64_t* start_actions, const int64_t* start_offsets,
                const uint32_t* bot_seeds, const uint32_t* eval_seeds, int32_t max_len,
                int64_t* actions, int32_t* length, double* returns, int32_t* visits,
                float* observations) {
  const int32_t record = (visits ? OS_RECORD_VISITS : 0) |
                         (observations ? OS_RECORD_OBSERVATIONS : 0);
  int rc = os_selfplay_prepare(e, p, num_games, start_actions, start_offsets, bot_seeds,
                               eval_seeds, max_len, record);
  if (rc) return rc;
  if ((rc = SpRun(e, nullptr))) return rc;
  return SpFetch(e, actions, length, returns, visits, observations);
}

int os_rollouts_prepare(os_engine* e, const int64_t* root_actions, int64_t n_actions,
                        int64_t n, int32_t n_rollouts, const uint32_t* seeds) {
  if (!e || (n > 0 && !seeds)) return Fail(OS_ERR_INVALID, "null argument");
  if (n < 0) return Fail(OS_ERR_INVALID, "n < 0");
  if (n > 0x7FFFFFFFll * 64) return Fail(OS_ERR_CAPACITY, "too many evaluators");
  if (n_rollouts < 1) return Fail(OS_ERR_INVALID, "n_rollouts must be >= 1");
  HIP_TRY(hipSetDevice(e->device));
  HostState root;
  std::string err;
  if (!ReplayRoot(e->game, root_actions, n_actions, &root, &err))
    return Fail(OS_ERR_INVALID, err);
  return RollPrepare(e, root, n, n_rollouts, seeds);
}

int os_rollouts_run_async(os_engine* e, void* hip_stream) {
  if (!e) return Fail(OS_ERR_INVALID, "null engine");
  return RollRun(e, static_cast<hipStream_t>(hip_stream));
}

int os_rollouts_fetch(os_engine* e, double* out_returns) {
  if (!e || !out_returns) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->roll_ready) return Fail(OS_ERR_INVALID, "os_rollouts_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  if (e->roll_n > 0)
    HIP_TRY(hipMemcpy(out_returns, e->d_rollout_out.p, e->roll_n * 16, hipMemcpyDeviceToHost));
  return OS_OK;
}

int os_rollouts_stats(os_engine* e, int64_t* out) {
  if (!e || !out) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->roll_ready) return Fail(OS_ERR_INVALID, "os_rollouts_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  std::vector<uint32_t> c(static_cast<size_t>(e->roll_n) * 2);
  if (e->roll_n > 0)
    HIP_TRY(hipMemcpy(c.data(), e->d_roll_cnt.p, c.size() * 4, hipMemcpyDeviceToHost));
  out[0] = out[1] = 0;
  for (size_t i = 0; i < c.size(); i += 2) {
    out[0] += c[i];
    out[1] += c[i + 1];
  }
  out[2] = e->game.state_bytes;
  return OS_OK;
}

int os_rollouts_outcomes_async(os_engine* e, int64_t* dev_counts, void* hip_stream) {
  if (!e || !dev_counts) return Fail(OS_ERR_INVALID, "null argument");
  if (!e->roll_ready) return Fail(OS_ERR_INVALID, "os_rollouts_prepare was not called");
  HIP_TRY(hipSetDevice(e->device));
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipMemsetAsync(dev_counts, 0, 3 * sizeof(int64_t), st));
  if (e->roll_n == 0) return OS_OK;
  const int64_t blocks = std::min<int64_t>((e->roll_n + 255) / 256, 512);
  hipLaunchKernelGGL(k_outcome_counts, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     static_cast<const double*>(e->d_rollout_out.p), e->roll_n,
                     reinterpret_cast<unsigned long long*>(dev_counts));
  HIP_TRY(hipGetLastError());
  return OS_OK;
}

int os_rollouts_batch(os_engine* e, const int64_t* root_actions, int64_t n_actions,
                      int64_t n, int32_t n_rollouts, const uint32_t* seeds,
                      double* out_returns) {
  if (!e || (n > 0 && (!seeds || !out_returns))) return Fail(OS_ERR_INVALID, "null argument");
  int rc = os_rollouts_prepare(e, root_actions, n_actions, n, n_rollouts, seeds);
  if (rc) return rc;
  if ((rc = RollRun(e, nullptr))) return rc;
  return os_rollouts_fetch(e, out_returns);
}

int os_engine_root_sums_async(os_engine* e, int32_t num_actions, int64_t* dev_visits,
                              double* dev_rewards, void* hip_stream) {
  if (!e || !dev_visits || !dev_rewards) return Fail(OS_ERR_INVALID, "null argument");
  if (num_actions < e->game.cfg.num_actions)
    return Fail(OS_ERR_INVALID, "num_actions smaller than NumDistinctActions");
  HIP_TRY(hipSetDevice(e->device));
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  const int64_t R = e->num_roots;
  const int64_t A = num_actions;
  int rc;
  if ((rc = e->d_dense_n.ensure(static_cast<size_t>(std::max<int64_t>(R, 1)) * A * 4)) ||
      (rc = e->d_dense_w.ensure(static_cast<size_t>(std::max<int64_t>(R, 1)) * A * 8)))
    return rc;
  if (R > 0) {
    HIP_TRY(hipMemsetAsync(e->d_dense_n.p, 0, R * A * 4, st));
    HIP_TRY(hipMemsetAsync(e->d_dense_w.p, 0, R * A * 8, st));
    hipLaunchKernelGGL(k_root_scatter, dim3(static_cast<unsigned>(R)), dim3(128), 0, st,
                       static_cast<const int32_t*>(e->d_nch.p),
                       static_cast<const int32_t*>(e->d_cact.p),
                       static_cast<const int32_t*>(e->d_cn.p),
                       static_cast<const double*>(e->d_cw.p), e->max_children, A,
                       static_cast<int32_t*>(e->d_dense_n.p),
                       static_cast<double*>(e->d_dense_w.p));
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_root_reduce, dim3(static_cast<unsigned>(A)), dim3(256), 0, st,
                     static_cast<const int32_t*>(e->d_dense_n.p),
                     static_cast<const double*>(e->d_dense_w.p), R, A, dev_visits,
                     dev_rewards);
  HIP_TRY(hipGetLastError());
  return OS_OK;
}

int os_root_parallel(os_engine* const* engines, int32_t ndev, const os_mcts_params* p,
                     const int64_t* root_actions, int64_t n_actions,
                     int64_t trees_per_device, uint32_t seed_base, int32_t num_actions,
                     int64_t* out_visits, double* out_rewards, int64_t* out_sims) {
  if (!engines || ndev < 1 || !p || !out_visits || !out_rewards || trees_per_device < 1 ||
      (n_actions > 0 && !root_actions))
    return Fail(OS_ERR_INVALID, "bad argument");
  for (int g = 0; g < ndev; ++g) {
    if (!engines[g]) return Fail(OS_ERR_INVALID, "null engine");
    for (int h = 0; h < g; ++h)
      if (engines[h] == engines[g]) return Fail(OS_ERR_INVALID, "an engine is listed twice");
    if (engines[g]->game.cfg.kind != engines[0]->game.cfg.kind ||
        engines[g]->game.cfg.num_actions != engines[0]->game.cfg.num_actions)
      return Fail(OS_ERR_INVALID, "engines of different games");
  }
  if (num_actions < engines[0]->game.cfg.num_actions)
    return Fail(OS_ERR_INVALID, "num_actions smaller than NumDistinctActions");
  const int64_t T = trees_per_device;
  const int64_t A = num_actions;
  std::vector<int64_t> acts(static_cast<size_t>(T * n_actions));
  std::vector<int64_t> offs(static_cast<size_t>(T + 1));
  for (int64_t t = 0; t < T; ++t) {
    offs[t] = t * n_actions;
    for (int64_t i = 0; i < n_actions; ++i) acts[t * n_actions + i] = root_actions[i];
  }
  offs[T] = T * n_actions;
  std::vector<uint32_t> bs(T), es(T);
  int rc;
  // Launch every engine's trees and its on-device root sums before any wait.
  for (int g = 0; g < ndev; ++g) {
    os_engine* e = engines[g];
    for (int64_t t = 0; t < T; ++t) {
      bs[t] = seed_base + static_cast<uint32_t>(g * T + t);
      es[t] = bs[t] + (1u << 20);
    }
    if ((rc = Prepare(e, p, T, acts.data(), offs.data(), bs.data(), es.data()))) return rc;
    if ((rc = Run(e, nullptr))) return rc;
    if ((rc = e->d_rp_sum.ensure(static_cast<size_t>(A) * 16))) return rc;
    int64_t* dn = static_cast<int64_t*>(e->d_rp_sum.p);
    if ((rc = os_engine_root_sums_async(e, num_actions, dn, reinterpret_cast<double*>(dn + A),
                                        nullptr)))
      return rc;
  }
  // Validate every search, then gather the per-device sums on engines[0].
  os_engine* e0 = engines[0];
  if ((rc = e0->d_rp_all.ensure(static_cast<size_t>(ndev) * A * 16))) return rc;
  int64_t* all_n = static_cast<int64_t*>(e0->d_rp_all.p);
  double* all_w = reinterpret_cast<double*>(all_n + ndev * A);
  int64_t sims = 0;
  for (int g = 0; g < ndev; ++g) {
    os_engine* e = engines[g];
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    std::vector<SearchResult> res(T);
    HIP_TRY(hipMemcpy(res.data(), e->d_res.p, T * sizeof(SearchResult), hipMemcpyDeviceToHost));
    if (e->paged) {
      // As os_engine_fetch: a paged batch that ran out of pool pages is rerun
      // on the reserved arena (same seeds, same trees) and summed again.
      int64_t over = 0;
      for (const SearchResult& s : res) over += s.status == kArenaOverflow;
      if (over) {
        e->arena_overflows += over;
        e->arena_reruns += 1;
        e->last_results.resize(T);
        if ((rc = RerunReserved(e))) return rc;
        res = e->last_results;
        int64_t* dn = static_cast<int64_t*>(e->d_rp_sum.p);
        if ((rc = os_engine_root_sums_async(e, num_actions, dn,
                                            reinterpret_cast<double*>(dn + A), nullptr)))
          return rc;
        HIP_TRY(hipDeviceSynchronize());
      }
    }
    for (int64_t t = 0; t < T; ++t) {
      if (res[t].status != kOk)
        return Fail(OS_ERR_CAPACITY, "engine " + std::to_string(g) + " tree " +
                                         std::to_string(t) + ": search status " +
                                         std::to_string(res[t].status));
      sims += res[t].sims;
    }
    const int64_t* dn = static_cast<const int64_t*>(e->d_rp_sum.p);
    HIP_TRY(hipMemcpyPeer(all_n + g * A, e0->device, dn, e->device, A * 8));
    HIP_TRY(hipMemcpyPeer(all_w + g * A, e0->device, dn + A, e->device, A * 8));
  }
  HIP_TRY(hipSetDevice(e0->device));
  int64_t* out_n = static_cast<int64_t*>(e0->d_rp_sum.p);  // reused as the result
  double* out_w = reinterpret_cast<double*>(out_n + A);
  hipLaunchKernelGGL(k_sum_devices, dim3(static_cast<unsigned>((A + 127) / 128)), dim3(128), 0,
                     nullptr, all_n, all_w, ndev, A, out_n, out_w);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(out_visits, out_n, A * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(out_rewards, out_w, A * 8, hipMemcpyDeviceToHost));
  if (out_sims) *out_sims = sims;
  return OS_OK;
}

int32_t os_sample_action(const double* probs, int32_t n, uint32_t* key, int32_t* pos) {
  if (!probs || n < 1 || !key || !pos || *pos < 0 || *pos > kMtN)
    return Fail(OS_ERR_INVALID, "bad argument");
  MtStream g{key, *pos, 1, 0};
  const double z = AbslUniformDouble01(g);
  g.finalize();
  *pos = g.idx;
  // spiel.cc:341-366: the first outcome whose [sum, sum + p) holds z.
  double sum = 0.0;
  for (int32_t k = 0; k < n; ++k) {
    if (sum <= z && z < sum + probs[k]) return k;
    sum += probs[k];
  }
  return Fail(OS_ERR_INVALID, "SampleAction: probabilities do not cover z");
}

int64_t os_make_roots(const os_game* game, int64_t num_roots, uint32_t seed_base,
                      int32_t max_plies, int64_t* actions, int64_t* offsets) {
  if (!game || num_roots < 0 || max_plies < 0)
    return Fail(OS_ERR_INVALID, "bad argument");
  std::vector<int64_t> all;
  std::vector<int64_t> offs(1, 0);
  for (int64_t i = 0; i < num_roots; ++i) {
    std::mt19937 g(seed_base + static_cast<uint32_t>(i));
    HostState s;
    s.game = &game->g;
    StateInit(&s);
    const uint32_t k = g() % static_cast<uint32_t>(max_plies + 1);
    std::vector<int64_t> legal;
    for (uint32_t j = 0; j < k; ++j) {
      StateLegal(s, &legal);
      const int64_t a = legal[g() % legal.size()];
      HostState t = s;
      StateApply(&t, a);
      if (StateTerminal(t)) break;
      s = t;
    }
    // A bot moves at decision nodes only: resolve a pending chance node with
    // drawn outcomes (pig), never ending the game.
    while (StateIsChance(s)) {
      StateLegal(s, &legal);
      HostState t = s;
      StateApply(&t, legal[g() % legal.size()]);
      if (StateTerminal(t)) {
        s.history.pop_back();  // undo the roll that led here
        HostState r;
        r.game = s.game;
        StateInit(&r);
        for (int64_t a : s.history) StateApply(&r, a);
        s = r;
        break;
      }
      s = t;
    }
    all.insert(all.end(), s.history.begin(), s.history.end());
    offs.push_back(static_cast<int64_t>(all.size()));
  }
  if (actions) std::memcpy(actions, all.data(), all.size() * 8);
  if (offsets) std::memcpy(offsets, offs.data(), offs.size() * 8);
  return static_cast<int64_t>(all.size());
}

}  // extern "C"
