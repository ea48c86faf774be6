// Engine internals shared by the host translation unit (os_engine.hip: the
// C-ABI, batch preparation, result fetch) and the per-game kernel units
// (os_game_*.hip, built in parallel): kernel argument blocks, device buffers,
// the engine object, error reporting and the per-game launcher table.
#ifndef OS_ENGINE_IMPL_H_
#define OS_ENGINE_IMPL_H_

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/os_mcts.h"
#include "os_az.h"
#include "os_host.h"
#include "os_mcts.h"
#include "os_wave.h"

namespace osx {
using namespace osm;

// Thread-local message of the last failed C-ABI call (os_last_error).
extern thread_local std::string g_err;
inline int Fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Host-side per-root work (root replay, Dirichlet draws) over [0, n) in
// contiguous chunks on up to 16 threads, the calling thread taking the first.
// body(lo, hi) returns 0 or a Fail() code; the lowest failing chunk's code
// and message are returned (the same error a serial loop reports first).
template <class F>
int ParallelChunks(int64_t n, int64_t min_chunk, F body) {
  const int64_t hw = std::max<int64_t>(1, std::thread::hardware_concurrency());
  const int T = static_cast<int>(
      std::min<int64_t>(std::min<int64_t>(hw, 16), (n + min_chunk - 1) / min_chunk));
  if (T <= 1) return body(int64_t{0}, n);
  std::vector<int> rc(T, 0);
  std::vector<std::string> msg(T);
  auto run = [&](int t) {
    rc[t] = body(n * t / T, n * (t + 1) / T);
    if (rc[t]) msg[t] = g_err;  // g_err is thread-local
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(run, t);
  run(0);
  for (std::thread& x : th) x.join();
  for (int t = 0; t < T; ++t)
    if (rc[t]) return Fail(rc[t], msg[t]);
  return 0;
}
#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess)                                                    \
      return ::osx::Fail(OS_ERR_DEVICE, std::string(#expr " failed: ") +    \
                                            hipGetErrorString(_e));          \
  } while (0)

constexpr int kGoLogCap = 248;              // >= 2 * 11 * 11 + 4
constexpr int kGoHeads = 122;               // stone counts 0 .. 11 * 11
// go 12 x 12 .. 19 x 19 on the device (k_lsearch over B384 bitboards, wide
// nodes with 16-bit child counts, u16 actions in an HBM expansion buffer).
constexpr int kGoDeviceMaxSide = 19;
constexpr int kGoLogCapBig = 2 * 19 * 19 + 4;
constexpr int kGoHeadsBig = 19 * 19 + 1;
constexpr size_t kLdsBytes = 160 * 1024;    // LDS per CU on gfx950
constexpr int kDefaultBlock = 16;           // searches (lanes) per workgroup (lane layout)

struct DevArgs {
  GameCfg cfg;
  SearchParams sp;
  int64_t num_roots;      // roots in this launch
  int64_t root_base;      // global index of the first root of this launch
  const void* roots;      // [total] G::State
  const uint32_t* bot_seeds;
  const uint32_t* eval_seeds;
  uint32_t* mt;           // [num_roots][2][624]
  void* arena;            // [num_roots][cap] Node<R>, or the page pool
  uint32_t cap;           // nodes per root, or per page when paged
  uint32_t* pages;        // paged arena descriptor (os_wave.h kPg*), or null
  int32_t path_cap;       // >= MaxGameLength + 1 (LDS path slice per lane)
  int32_t child_cap;      // >= max |LegalActions| (LDS expansion slice)
  int32_t import_state;   // numpy (key, pos) import / export
  int32_t shared_stream;  // numpy: one RandomState for bot + evaluator
  int32_t* mt_pos;        // [total][2] in/out when import_state
  // go
  const uint64_t* zob;
  const uint64_t* root_hashes;  // [total][hash_stride]
  const int32_t* root_nhash;    // [total]
  int32_t hash_stride;
  // Global-memory lane layout (k_lsearch, go): per-search buffers, contiguous
  // per search (the MT streams use `mt` as [chunk][2][624]).
  int64_t lstride;        // searches per launch chunk
  void* lpath;            // [chunk][path_cap] PathEnt<R>
  uint64_t* lglog;        // [chunk][log cap] position logs
  uint32_t* lglink;       // [chunk][log cap] stone count + same-count links
  uint16_t* lheads;       // [chunk][kGoHeadsBig] bucket heads (boards > 11 x 11)
  uint16_t* lact;         // [chunk][child_cap] expansion buffers (boards > 11 x 11)
  // outputs, indexed by global root
  SearchResult* results;
  int32_t max_children;
  int32_t* child_action;
  int32_t* child_n;
  double* child_w;
  int8_t* child_out;
  int32_t* nchild;
  int32_t* root_n;
  double* root_w;
  int8_t* root_out;
  int64_t* best_action;
};

// ---------------------------------------------------------------------------
// Self-play: one wave plays a whole game the way
// examples/mcts_example.cc:77-136 PlayGame does with two MCTSBots sharing one
// RandomRolloutEvaluator: every move is bots[CurrentPlayer]->Step(state) =
// MCTSearch + BestChild (mcts.cc:219-226, 325-428), both bots' rng_ and the
// shared evaluator's rng persist across moves.
struct SpArgs {
  GameCfg cfg;
  SearchParams sp;
  int64_t num_games;      // games in this launch
  int64_t game_base;      // global index of the first game of this launch
  const void* starts;     // [total] G::State
  const uint32_t* bot_seeds;   // [total][2]
  const uint32_t* eval_seeds;  // [total]
  void* arena;            // [num_games][cap] Node<R>
  uint32_t cap;
  int32_t path_cap;
  int32_t max_len;        // trajectory slots per game
  int32_t num_actions;
  // go: per-game position history (grows by one per move)
  const uint64_t* zob;
  uint64_t* hist;         // [total][hash_stride]
  int32_t* hist_n;        // [total]
  int32_t hash_stride;
  // outputs
  int32_t* actions;       // [total][max_len], -1 padded
  int32_t* length;        // [total]
  double* returns;        // [total][2]
  int32_t* visits;        // [total][max_len][num_actions] or null
  float* obs;             // [total][max_len][obs_size] or null
  int32_t obs_size;       // C * H * W
  SearchResult* results;  // [total], summed over the game's searches
  // AlphaZero PlayGame move choice (alpha_zero.cc:64-118; os_selfplay_set_
  // options): policy = pow(explore_count, 1 / T) over the root's children,
  // normalised; SampleAction from the game's actor rng before
  // temperature_drop moves, BestChild after; resign when |root value| >
  // the game's cutoff.  actor_seeds == null: BestChild every move.
  const uint32_t* actor_seeds;  // [total]
  const double* pow_lut;        // pow(n, 1 / T), n in [0, max_simulations]
  int32_t temperature_drop;
  int32_t resign;               // draw the cutoff at game start, apply it
  double cutoff_value, cutoff_probability, max_utility;
  double* policy;               // [total][max_len][num_actions] or null
  double* root_value;           // [total][max_len] or null
};

// ---------------------------------------------------------------------------
// External-evaluator MCTS (os_az.h): one lane per search, one step per launch.
struct AzArgs {
  GameCfg cfg;
  SearchParams sp;
  int32_t puct;
  int32_t np_policy;        // python/algorithms/mcts.py semantics (os_az.h az_step)
  int64_t num_roots;
  const void* roots;        // [R] G::State
  void* slots;              // [R] AzSlot<G>
  Node<double>* arena;      // [R][cap]
  double* priors;           // [R][cap]
  double* raw;              // [R][cap] parked priors of fused requests, or null
  uint32_t cap;
  uint32_t* mt;             // [R][624] bot rng
  const uint32_t* bot_seeds;
  int32_t obs_size;
  int32_t num_actions;
  int32_t* kind;            // [R]
  float* obs;               // [R][obs_size]
  uint8_t* legal;           // [R][A]
  const double* prior_in;   // [R][A]
  const double* value_in;   // [R]
  int32_t* pending;         // requests written by this step
  int32_t* shards;          // kAzShards counters, kAzShardStride apart (zero between steps)
  // Bot rng continuing a caller-held stream (os_az_prepare_stateful): rows of
  // `mt` hold numpy-form keys, mt_pos_in the positions; a finished search
  // writes its stream back in the same form (key row + mt_pos_out).
  int32_t import_mt;
  const int32_t* mt_pos_in;  // [R]
  int32_t* mt_pos_out;       // [R]
  // Dirichlet root noise (alpha > 0): [R][noise_stride] normalised draws in
  // legal-action order + MT words they consumed (host-drawn, os_az.h)
  const double* noise;      // null: no noise
  const int32_t* noise_skip;
  int32_t noise_stride;
  double noise_eps;
  // go: superko context of each root
  const uint64_t* zob;
  const uint64_t* root_hashes;  // [R][hash_stride]
  const int32_t* root_nhash;    // [R]
  int32_t hash_stride;
  // outputs (same layout as the search kernels)
  SearchResult* results;
  int32_t max_children;
  int32_t* child_action;
  int32_t* child_n;
  double* child_w;
  int8_t* child_out;
  int32_t* nchild;
  int32_t* root_n;
  double* root_w;
  int8_t* root_out;
  int64_t* best_action;
};

struct RollArgs {
  GameCfg cfg;
  int64_t n;
  int32_t n_rollouts;
  const void* root;  // one G::State
  const uint32_t* seeds;
  uint32_t* mt;      // [624][n] (k_rollouts, SoA) or [n][624]
  uint64_t* glog;    // go: [kGoLogCap][n] position logs (k_rollouts, SoA)
  uint32_t* glink;   //     [kGoLogCap][n] stone count + same-count links
  uint2* counters;   // [n] (MT words drawn, moves played) (k_rollouts)
  double* out;       // [n][2]
  const uint64_t* zob;
  const uint64_t* root_hashes;
  int32_t n_root_hashes;
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t b) {
    if (b <= bytes && p) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (b == 0) return 0;
    hipError_t e = hipMalloc(&p, b);
    if (e != hipSuccess) {
      p = nullptr;
      return Fail(OS_ERR_DEVICE, std::string("hipMalloc(") + std::to_string(b) +
                                     ") failed: " + hipGetErrorString(e));
    }
    bytes = b;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// Pinned host staging for the per-call copies of small batches (a single
// bot's step): copies into it are queued with hipMemcpyAsync and waited for
// once, instead of one synchronous pageable hipMemcpy each.
struct PinBuf {
  unsigned char* p = nullptr;
  size_t bytes = 0;
  size_t used = 0;
  int ensure(size_t b) {
    if (b <= bytes && p) return 0;
    // Copies queued from the old buffer (a failed call's) finish first.
    if (p) {
      (void)hipStreamSynchronize(nullptr);
      (void)hipHostFree(p);
    }
    p = nullptr;
    bytes = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), b);
    if (e != hipSuccess) {
      p = nullptr;
      return Fail(OS_ERR_DEVICE, std::string("hipHostMalloc failed: ") + hipGetErrorString(e));
    }
    bytes = b;
    return 0;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
};

}  // namespace osx

struct os_engine {
  osm::HostGame game;
  int device = 0;
  // prepared run
  os_mcts_params params{};
  int64_t num_roots = 0;
  int64_t chunk_roots = 0;
  uint32_t cap = 0;
  int node_bytes = 16;
  bool node_double = false;  // Node<double>: f64 rewards
  bool node_wide = false;    // Node<R, true>: 16-bit child counts (go > 11 x 11)
  int32_t max_children = 0;
  int32_t hash_stride = 1;
  bool import_state = false;
  bool shared_stream = false;
  int32_t search_layout = -1;  // layout of the last os_engine_prepare (AUTO resolved)
  int32_t search_lanes = 0;    // searches per wave of the last search launch (1: wave layout)
  int32_t rollout_layout = OS_LAYOUT_LANE;  // 4-140x faster than WAVE (profiles/r01)
  // prepared rollout batch
  int64_t roll_n = 0;
  int32_t roll_nr = 1;
  int32_t roll_nhash = 0;
  bool roll_ready = false;
  // prepared self-play batch
  int64_t sp_games = 0;
  int32_t sp_max_len = 0;
  bool sp_visits = false;
  bool sp_obs = false;
  bool sp_ready = false;
  bool sp_policy = false;   // OS_RECORD_POLICY
  bool sp_values = false;   // OS_RECORD_ROOT_VALUES
  os_selfplay_options sp_opts{};  // os_selfplay_set_options
  std::vector<uint32_t> sp_actor_seeds;
  // prepared external-evaluator batch (os_az_*): caller-owned device buffers
  bool az_ready = false;
  // The stream of the last eager os_az_step_async (a step captured into a
  // graph is replayed on its caller's stream, which ran the eager steps
  // before): os_az_fetch / os_az_requests / os_az_export_rng wait on it
  // alone, not on every stream of the device.
  hipStream_t az_stream = nullptr;
  int32_t az_puct = 0;
  int32_t az_np = 0;  // OS_POLICY_NUMPY external-evaluator batch
  // os_az_stage: the host work of the NEXT os_az_prepare_staged batch, done
  // ahead (inputs, replayed root records + go hash sets, root noise).
  struct AzStaged {
    bool ready = false;
    os_mcts_params p{};
    int32_t puct = 0;
    int64_t R = 0;
    double alpha = 0.0, eps = 0.0;
    std::vector<int64_t> acts, offs;
    std::vector<uint32_t> seeds;
    std::vector<unsigned char> roots;
    std::vector<uint64_t> rh;
    std::vector<int32_t> rnh;
    std::vector<double> noise;
    std::vector<int32_t> skip;
  } az_staged;
  int32_t* az_kind = nullptr;
  float* az_obs = nullptr;
  uint8_t* az_legal = nullptr;
  const double* az_prior = nullptr;
  const double* az_value = nullptr;
  int32_t* az_pending = nullptr;
  double az_eps = 0.0;
  bool az_noise = false;
  bool az_import = false;  // os_az_prepare_stateful
  int32_t az_requests = 0;  // os_az_set_requests (OS_AZ_REQUESTS_SEPARATE)
  bool az_fused = false;    // mode of the prepared batch
  int32_t az_layout = OS_LAYOUT_AUTO;  // os_az_set_layout
  bool az_wave = false;     // the prepared batch runs k_waz_step (one wave per search)
  osx::DevBuf d_az_slots, d_az_prior, d_az_noise, d_az_skip, d_az_pos, d_az_raw, d_az_shards;
  osx::DevBuf d_lpath, d_lheads, d_lact;  // k_lsearch paths, big-board heads / actions
  osx::DevBuf d_roots, d_bseed, d_eseed, d_mt, d_arena, d_lut, d_zob, d_rhash, d_rnh,
      d_pos, d_res, d_cact, d_cn, d_cw, d_cout, d_nch, d_rn, d_rw, d_rout, d_best,
      d_rollout_out, d_dense_n, d_dense_w, d_sp_act, d_sp_len, d_sp_ret, d_sp_vis,
      d_sp_obs, d_glog, d_glink, d_roll_cnt, d_rp_sum, d_rp_all, d_sp_pol, d_sp_val,
      d_sp_actor, d_sp_pow;
  std::vector<osm::SearchResult> last_results;
  int64_t last_sims = 0;
  // Paged arena (os_engine_set_arena_mode).  arena_mode is the
  // caller's choice; `paged` says whether the prepared batch uses the pool.
  int32_t arena_mode = 0;  // OS_ARENA_RESERVED
  bool paged = false;
  uint32_t page_nodes = 0;
  uint32_t pool_pages = 0;
  size_t arena_bytes = 0;  // arena of the prepared batch
  osx::DevBuf d_page_next;
  struct ArenaHint {  // pages beyond the roots' own, per root, of the last runs
    int32_t sims = -1;
    int32_t node_bytes = 0;
    uint32_t page_nodes = 0;
    double extra_per_root = 0.0;
  } arena_hint;
  // Uploaded constants (LUT of the last prepared sims / selection, go's
  // Zobrist table) and the pinned staging of per-call copies.
  int64_t lut_n = -1;
  int32_t lut_puct = -1;
  const void* lut_at = nullptr;
  const void* zob_at = nullptr;
  osx::PinBuf h_stage;
  // os_engine_set_run_timing: HIP events around each search launch
  bool time_runs = false;
  bool run_timed = false;
  hipEvent_t run_ev[2] = {nullptr, nullptr};
  int64_t arena_reruns = 0;     // batches rerun on the reserved arena
  int64_t arena_overflows = 0;  // searches that ran out of pool pages
  ~os_engine() {
    osx::DevBuf* all[] = {&d_roots, &d_bseed, &d_eseed, &d_mt,  &d_arena, &d_lut,
                     &d_zob,   &d_rhash, &d_rnh,   &d_pos, &d_res,   &d_cact,
                     &d_cn,    &d_cw,    &d_cout,  &d_nch, &d_rn,    &d_rw,
                     &d_rout,  &d_best,  &d_rollout_out, &d_dense_n, &d_dense_w,
                     &d_sp_act, &d_sp_len, &d_sp_ret, &d_sp_vis, &d_sp_obs,
                     &d_az_slots, &d_az_prior, &d_az_noise, &d_az_skip, &d_glog, &d_glink,
                     &d_roll_cnt, &d_rp_sum, &d_rp_all, &d_page_next, &d_sp_pol, &d_sp_val,
                     &d_sp_actor, &d_sp_pow, &d_az_pos, &d_az_raw, &d_az_shards, &d_lpath, &d_lheads, &d_lact};
    (void)hipSetDevice(device);
    for (osx::DevBuf* b : all) b->release();
    h_stage.release();
    for (hipEvent_t& ev : run_ev)
      if (ev) (void)hipEventDestroy(ev);
  }
};

namespace osx {

// Kernel arguments of the prepared search batch (os_engine.hip).
DevArgs MakeArgs(os_engine* e);

// Per-game entry points, defined by os_game_<name>.hip.
struct GameLaunchers {
  int (*search)(os_engine*, const DevArgs&, hipStream_t);  // k_wsearch / k_mcts
  int (*selfplay)(os_engine*, hipStream_t);                // k_wselfplay
  int (*az)(os_engine*, hipStream_t);                      // k_az_step, or null
  int (*rollouts)(os_engine*, hipStream_t);                // k_rollouts / k_wrollouts
  int (*phase_cycles)(uint64_t*, bool clear);              // OS_PHASE_TIMING builds
  size_t az_slot_bytes;
};
extern GameLaunchers kTicTacToeLaunchers;
extern GameLaunchers kConnectFourLaunchers;
extern GameLaunchers kBreakthroughLaunchers;
extern GameLaunchers kHexLaunchers;
extern GameLaunchers kGoLaunchers;
extern GameLaunchers kGoBigLaunchers;
extern GameLaunchers kHexBigLaunchers;
extern GameLaunchers kPigLaunchers;

// go / hex above 11 x 11 run lane-layout searches only (k_lsearch over B384
// bitboards; os_game_go_big.hip, os_game_hex_big.hip).
inline bool GoBigBoard(const GameCfg& c) { return c.kind == kGo && c.rows > 11; }
inline bool BigBoard(const GameCfg& c) { return (c.kind == kGo || c.kind == kHex) && c.rows > 11; }

// go up to 9 x 9 on the lane kernels runs GoT<B96> (os_games.h Go9;
// os_game_go9.hip); OS_GO9=0 builds keep GoT<B128> there (A/B knob).
#ifndef OS_GO9
#define OS_GO9 1
#endif
inline bool UseGo9(const GameCfg& c) {
  return OS_GO9 && c.kind == kGo && c.rows <= kGo9MaxSide;
}
int LaunchGo9Search(os_engine* e, const DevArgs& a, hipStream_t stream);  // k_lsearch<Go9>
int LaunchGo9Rollouts(os_engine* e, hipStream_t stream);                  // k_rollouts<Go9>

inline const GameLaunchers* LaunchersFor(int32_t kind) {
  switch (kind) {
    case kTicTacToe: return &kTicTacToeLaunchers;
    case kConnectFour: return &kConnectFourLaunchers;
    case kBreakthrough: return &kBreakthroughLaunchers;
    case kHex: return &kHexLaunchers;
    case kGo: return &kGoLaunchers;
    case kPig: return &kPigLaunchers;
  }
  return nullptr;
}
inline const GameLaunchers* LaunchersFor(const GameCfg& c) {
  if (BigBoard(c)) return c.kind == kGo ? &kGoBigLaunchers : &kHexBigLaunchers;
  return LaunchersFor(c.kind);
}

}  // namespace osx

#endif  // OS_ENGINE_IMPL_H_
