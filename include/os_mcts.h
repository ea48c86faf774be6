/*
 * os_mcts.h — C-ABI of libos_mcts.so, the MI355X-native batched MCTS engine.
 *
 * Drop-in boundary for OpenSpiel's MCTS random-rollout bot path.  Plain C
 * types only (no torch / HIP types in signatures).  Every entry point cites the
 * reference interface it replaces (paths are under open_spiel/ in
 * Tyjch/open_spiel-1).
 *
 * Conventions
 *   - Return value: 0 (OS_OK) on success, < 0 on error; os_last_error()
 *     returns a thread-local message for the last failure on this thread.
 *     The reference reports the same conditions through SpielFatalError
 *     (spiel_utils.cc:94-110), surfaced in Python as RuntimeError
 *     (pyspiel.cc:67-78, :839-840); unsupported game types raise ValueError in
 *     python/algorithms/mcts.py:241-245 — OS_ERR_UNSUPPORTED maps to that.
 *   - The caller owns every host buffer; an engine owns its device memory.
 *   - Calls are synchronous unless named *_async.  One engine per device;
 *     engines on different devices may be driven from different threads.
 *   - Roots cross the ABI as action histories from the initial state (the
 *     reference's default State::Serialize, spiel.h:541): root r is
 *     root_actions[root_offsets[r] .. root_offsets[r+1]).
 *   - Child outputs are in the tree's child order (the shuffled expansion
 *     order of mcts.cc:275), stride max_children per root.
 *   - Outcomes are int8: the value for the node's own player (the reference's
 *     `outcome[player]`), or 2 when the node is unsolved (empty vector).  With
 *     more than two players (pig) it is the value's sign: +1 a win (1), -1 a
 *     loss (-1 / (n - 1)), 0 nobody won (0).
 */
#ifndef OS_MCTS_C_ABI_H_
#define OS_MCTS_C_ABI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OS_OK 0
#define OS_ERR_INVALID (-1)      /* bad argument / illegal action          */
#define OS_ERR_UNSUPPORTED (-2)  /* game or parameter not supported        */
#define OS_ERR_DEVICE (-3)       /* HIP runtime failure                     */
#define OS_ERR_CAPACITY (-4)     /* node arena / path capacity exceeded     */

typedef struct os_game os_game;
typedef struct os_state os_state;
typedef struct os_engine os_engine;

/* Thread-local description of the last error on this thread. */
const char* os_last_error(void);

/* ---- Game / State: replaces pyspiel.load_game / pyspiel.State ------------
 * pyspiel.cc:675-684 load_game; spiel.cc:176-204 LoadGame;
 * game_parameters.cc:101-130 "name(k=v,...)" parsing.                    */
int os_game_load(const char* game_string, os_game** out);
void os_game_free(os_game* game);

typedef struct {
  int32_t kind;               /* 0 ttt, 1 connect_four, 2 breakthrough, 3 hex, 4 go, 5 pig */
  int32_t num_distinct_actions;  /* Game::NumDistinctActions (spiel.h:601-750) */
  int32_t max_game_length;    /* Game::MaxGameLength */
  int32_t num_players;        /* Game::NumPlayers: 2 (pig: `players`, 2..10) */
  int32_t max_children;       /* upper bound on |LegalActions()| */
  int32_t rows, cols;         /* board geometry */
  double min_utility, max_utility, utility_sum;
  double komi;                /* go only */
  int32_t handicap;           /* go only */
  int32_t state_bytes;        /* sizeof the device state record */
} os_game_info;
int os_game_get_info(const os_game* game, os_game_info* out);
/* Canonical game string, e.g. "go(board_size=9,komi=7.5)". Returns length. */
int64_t os_game_to_string(const os_game* game, char* buf, int64_t cap);

/* State (spiel.h:173-592; pybind pyspiel.cc:292-360). */
int os_state_new(const os_game* game, os_state** out);      /* NewInitialState */
int os_state_clone(const os_state* s, os_state** out);      /* Clone (spiel.h:459) */
void os_state_free(os_state* s);
int os_state_apply(os_state* s, int64_t action);            /* ApplyAction (spiel.h:205) */
int32_t os_state_current_player(const os_state* s);         /* CurrentPlayer (-4 terminal) */
int32_t os_state_is_terminal(const os_state* s);            /* IsTerminal (spiel.h:283) */
/* Returns (spiel.h:309): writes num_players values (os_game_info). */
int os_state_returns(const os_state* s, double* out2);
/* IsChanceNode (spiel.h:331; CurrentPlayer() is then -1, kChancePlayerId). */
int32_t os_state_is_chance_node(const os_state* s);
/* ChanceOutcomes (spiel.h:322-327): (action, probability) pairs in outcome
 * order; returns the count (may exceed cap; 0 unless a chance node). */
int32_t os_state_chance_outcomes(const os_state* s, int64_t* actions, double* probs,
                                 int32_t cap);
/* LegalActions (spiel.h:240), ascending; returns the count (may exceed cap). */
int32_t os_state_legal_actions(const os_state* s, int64_t* out, int32_t cap);
int32_t os_state_history(const os_state* s, int64_t* out, int32_t cap);
int64_t os_state_to_string(const os_state* s, char* buf, int64_t cap);
int64_t os_state_action_to_string(const os_state* s, int32_t player,
                                  int64_t action, char* buf, int64_t cap);
/* ObservationTensorShape (spiel.h Game::ObservationTensorShape; per game:
 * tic_tac_toe [3,3,3], connect_four [3,6,7], breakthrough [3,R,C], hex
 * [9,n,n], go [4,n,n]; all CHW): writes shape3 (may be NULL), returns C*H*W. */
int64_t os_game_observation_shape(const os_game* game, int32_t* shape3);
/* State::ObservationTensor(player) (connect_four.cc:211-221,
 * tic_tac_toe.cc:165-175, breakthrough.cc:326-340, hex.cc:266-277,
 * go.cc:102-122) as float32 [C][H][W].  Returns the size; writes only when
 * cap >= size. */
int64_t os_state_observation_tensor(const os_state* s, int32_t player, float* out,
                                    int64_t cap);

/* ---- Engine: replaces algorithms::MCTSBot / RandomRolloutEvaluator --------
 * mcts.h:152-159 MCTSBot(game, evaluator, uct_c, max_simulations,
 * max_memory_mb, solve, seed, verbose); mcts.h:94-95
 * RandomRolloutEvaluator(n_rollouts, seed); pyspiel.cc:499-524.          */
int os_engine_create(const char* game_string, int32_t device, os_engine** out);
int os_engine_destroy(os_engine* e);

/* Kernel layouts: one 64-lane wavefront per search (lanes scan children, twist
 * MT19937, back up the path in parallel), or one lane per search. */
#define OS_LAYOUT_WAVE 0
#define OS_LAYOUT_LANE 1
#define OS_LAYOUT_AUTO 2  /* engine picks per game and batch size */

#define OS_POLICY_CPP 0    /* mcts.cc: std::mt19937 bot + evaluator streams   */
#define OS_POLICY_NUMPY 1  /* mcts.py: numpy RandomState (shared or separate) */

/* Child selection (ChildSelectionPolicy, mcts.h:38-41).  PUCT with the
 * built-in RandomRolloutEvaluator uses its uniform Prior (mcts.cc:73-86). */
#define OS_SELECT_UCT 0
#define OS_SELECT_PUCT 1

typedef struct {
  double uct_c;                 /* MCTSBot uct_c */
  int32_t max_simulations;      /* MCTSBot max_simulations */
  int32_t n_rollouts;           /* RandomRolloutEvaluator n_rollouts */
  int64_t max_memory_mb;        /* MCTSBot max_memory_mb (drives GC, mcts.cc:402) */
  int32_t solve;                /* MCTSBot solve (MCTS-Solver backup) */
  int32_t policy;               /* OS_POLICY_* */
  int32_t block_size;           /* OS_LAYOUT_LANE only: lanes per workgroup (0 = default) */
  int32_t layout;               /* OS_LAYOUT_WAVE (0), OS_LAYOUT_LANE, OS_LAYOUT_AUTO */
  int64_t arena_nodes;          /* 0 = exact worst case; else nodes per root */
  int32_t child_selection;      /* OS_SELECT_UCT (mcts.cc:89-100) or OS_SELECT_PUCT
                                   (mcts.cc:102-111; MCTSBot child_selection_policy,
                                   mcts.h:152-159; mcts.py child_selection_fn) */
  int32_t reserved;             /* must be 0: every call taking params returns
                                   OS_ERR_INVALID otherwise, so a binding built
                                   against a shorter struct fails loudly */
} os_mcts_params;

/* Batched independent searches: MCTSBot::MCTSearch (mcts.cc:325-428) on every
 * root, bot seed bot_seeds[r], evaluator seed eval_seeds[r].  Bit-exact with
 * the reference given the same seeds.  Under OS_POLICY_NUMPY the two seeds
 * seed numpy-style streams (equal seeds => the test's shared RandomState is
 * NOT modelled; use os_mcts_stateful for a shared stream). */
int os_mcts_batch(os_engine* e, const os_mcts_params* p, int64_t num_roots,
                  const int64_t* root_actions, const int64_t* root_offsets,
                  const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                  int32_t max_children, int32_t* child_action,
                  int32_t* child_n, double* child_w, int8_t* child_out,
                  int32_t* nchild, int32_t* root_n, double* root_w,
                  int8_t* root_out, int64_t* best_action, int32_t* nodes);

/* One search whose MT19937 streams persist across calls: the state is passed
 * in numpy's legacy (key[624], pos) form (== libstdc++ mersenne_twister
 * _M_x/_M_p) and updated in place on return.  OS_POLICY_CPP: a stateful
 * MCTSBot (rng_ is never reseeded between MCTSearch calls, mcts.cc:325-333)
 * and its RandomRolloutEvaluator; OS_POLICY_NUMPY: the
 * python/algorithms/mcts.py path with np.random.RandomState objects.
 * shared != 0 (numpy only): one stream (bot_key) serves bot and evaluator
 * (mcts_test.py:41-54); else eval_key/eval_pos is the evaluator's. */
int os_mcts_stateful(os_engine* e, const os_mcts_params* p,
                        const int64_t* root_actions, int64_t n_actions,
                        int32_t shared, uint32_t* bot_key, int32_t* bot_pos,
                        uint32_t* eval_key, int32_t* eval_pos,
                        int32_t max_children, int32_t* child_action,
                        int32_t* child_n, double* child_w, int8_t* child_out,
                        int32_t* nchild, int32_t* root_n, double* root_w,
                        int8_t* root_out, int64_t* best_action, int32_t* nodes);

/* Whole search tree of root r of the last os_mcts_batch / numpy call, for
 * materialising SearchNode objects (mcts.h:109-137).  First call with
 * first == NULL to get the node count in *count. */
int os_engine_tree(os_engine* e, int64_t r, int64_t* count, uint32_t* first,
                   int32_t* n, double* w, int32_t* action, int32_t* nchild,
                   int8_t* out0);

/* Search-tree arena (no reference counterpart: mcts.cc allocates SearchNode
 * children on the heap).  RESERVED (default): every root gets the exact worst
 * case 1 + max_simulations * max_children nodes.  PAGED: once a fetched run
 * has shown how many nodes the searches take, later batches of the same
 * shape (wave layout, C++ policy, >= 64 roots, GC unable to fire,
 * arena_nodes == 0) share
 * one pool of pages sized from it; a batch that still runs out of pages is
 * rerun on the reserved arena inside os_engine_fetch (same seeds, same
 * results).  Device outputs read before the fetch (os_engine_root_sums_async)
 * are those of the overflowed run then: check os_engine_arena_info. */
#define OS_ARENA_RESERVED 0
#define OS_ARENA_PAGED 1
int os_engine_set_arena_mode(os_engine* e, int32_t mode);
/* out[0] 1 if the prepared batch is paged, [1] nodes per page (paged) or per
 * root, [2] pool pages or roots per chunk, [3] arena bytes of the batch, [4]
 * pages taken by the last run (paged; synchronises the device), [5] batches
 * rerun on the reserved arena, [6] searches that ran out of pages, [7] bytes
 * the reserved arena would take for the whole batch.  out has 8 entries. */
int os_engine_arena_info(os_engine* e, int64_t* out);

/* RandomRolloutEvaluator::Evaluate (mcts.cc:42-71) for n independent
 * evaluators, seeds[i], from one root; out_returns[2*i+{0,1}]. */
int os_rollouts_batch(os_engine* e, const int64_t* root_actions,
                      int64_t n_actions, int64_t n, int32_t n_rollouts,
                      const uint32_t* seeds, double* out_returns);
/* The kernel layout the last os_engine_prepare ran the batch on
 * (OS_LAYOUT_WAVE or OS_LAYOUT_LANE; OS_LAYOUT_AUTO resolved by the engine's
 * own rule: go from 32768 C++-policy roots and boards above 11 x 11 take the
 * lane layout, hex below 3 x 3 too, everything else the wave layout). */
int os_engine_get_layout(os_engine* e, int32_t* layout);
/* Searches per wavefront of the last search launch: 1 on the wave layout, the
 * lane layout's block width otherwise (go 9 x 9 .. 11 x 11: 16 up to 32768
 * roots, 32 above).  Reporting only (no reference counterpart). */
int os_engine_get_searches_per_wave(os_engine* e, int32_t* searches);
/* Kernel layout for os_rollouts_batch: OS_LAYOUT_LANE (default: one lane per
 * evaluator) or OS_LAYOUT_WAVE (one wave per evaluator, uniform game code). */
int os_engine_set_rollout_layout(os_engine* e, int32_t layout);

/* ---- External evaluator / PUCT --------------------
 * MCTSBot::MCTSearch (mcts.cc:325-428) whose Evaluator is outside the GPU
 * kernel -- the AlphaZero actor boundary (VPNetEvaluator, vpevaluator.cc:70-98:
 * Evaluate = {v, -v}, Prior = policy over LegalActions, both from (legal
 * actions, ObservationTensor)).  Child selection is UCT (puct = 0,
 * mcts.cc:89-100) or PUCT (puct = 1, mcts.cc:102-111).  Each of num_roots
 * searches (bot rng seed bot_seeds[r]) advances, one os_az_step_async at a
 * time, to its next evaluator request, written into CALLER-OWNED DEVICE
 * buffers so the caller's network reads them in place:
 *   dev_kind[r]          0 none (finished), 1 Prior, 2 Evaluate, 3 both
 *   dev_obs[r][C*H*W]    ObservationTensor(current player), f32
 *   dev_legal[r][A]      legal-action mask (u8)
 * and answered before the next step in
 *   dev_prior[r][A]      f64 action-indexed priors (read for legal actions)
 *   dev_value[r]         f64 player-0 value
 * *dev_pending = number of requests written by the last step (0 = all done).
 * os_az_fetch then returns the root statistics (os_mcts_batch layout).
 * dirichlet_alpha > 0 mixes Dirichlet noise into the root's priors,
 * (1 - dirichlet_epsilon) * prior + dirichlet_epsilon * noise, drawn from the
 * bot rng_ before the root's shuffle (MCTSBot ctor dirichlet_alpha /
 * dirichlet_epsilon, mcts.h:152-159; dirichlet_noise mcts.cc:177-192, used at
 * :265-273); alpha = 0 disables it.  Noise with a memory budget small enough
 * for GC to fire (the root could be re-expanded) is OS_ERR_UNSUPPORTED.
 * All five games (go's superko set travels in the continuation).  p->policy
 * OS_POLICY_CPP: the C++ MCTSBot; OS_POLICY_NUMPY: python/algorithms/mcts.py
 * (RandomState.shuffle expansions, no single-child stop, no GC; its root
 * noise comes from the caller through os_az_set_noise, alpha must be 0). */
int os_az_prepare(os_engine* e, const os_mcts_params* p, int32_t puct, int64_t num_roots,
                  const int64_t* root_actions, const int64_t* root_offsets,
                  const uint32_t* bot_seeds, double dirichlet_alpha,
                  double dirichlet_epsilon, int32_t* dev_kind, float* dev_obs,
                  uint8_t* dev_legal, const double* dev_prior, const double* dev_value,
                  int32_t* dev_pending);
/* os_az_prepare for bots whose rng_ has advanced over earlier searches (an
 * AlphaZero actor's MCTSBots keep one rng_ across a game, mcts.cc:209,
 * 325-333): search r continues the std::mt19937 held in numpy's legacy
 * (bot_keys[r][624], bot_pos[r]) form; the Dirichlet noise is drawn from that
 * stream.  After the searches finish, os_az_export_rng writes the advanced
 * streams back in the same form. */
int os_az_prepare_stateful(os_engine* e, const os_mcts_params* p, int32_t puct,
                           int64_t num_roots, const int64_t* root_actions,
                           const int64_t* root_offsets, const uint32_t* bot_keys,
                           const int32_t* bot_pos, double dirichlet_alpha,
                           double dirichlet_epsilon, int32_t* dev_kind, float* dev_obs,
                           uint8_t* dev_legal, const double* dev_prior, const double* dev_value,
                           int32_t* dev_pending);
int os_az_export_rng(os_engine* e, uint32_t* bot_keys, int32_t* bot_pos);
/* os_az_prepare in two halves, so a batch's host work overlaps the device
 * work of the batch before it.  os_az_stage does only host work (no HIP call:
 * it replays the roots into their device records and draws the root noise)
 * into the engine's staging area; it may run on another host thread while
 * os_az_step_async / os_az_fetch drive the engine's current batch, but not
 * concurrently with another os_az_stage or os_az_prepare*.
 * os_az_prepare_staged then uploads the staged batch and binds the request /
 * response buffers: the same batch os_az_prepare(the staged arguments) would
 * prepare.  C++ policy, seeded bots. */
int os_az_stage(os_engine* e, const os_mcts_params* p, int32_t puct, int64_t num_roots,
                const int64_t* root_actions, const int64_t* root_offsets,
                const uint32_t* bot_seeds, double dirichlet_alpha, double dirichlet_epsilon);
int os_az_prepare_staged(os_engine* e, int32_t* dev_kind, float* dev_obs, uint8_t* dev_legal,
                         const double* dev_prior, const double* dev_value,
                         int32_t* dev_pending);
/* Request mode of the next os_az_prepare*.  OS_AZ_REQUESTS_SEPARATE (default)
 * asks exactly what the reference MCTSBot asks, when it asks it: Prior at an
 * expansion, Evaluate at a leaf -- two evaluator rounds per simulation.
 * OS_AZ_REQUESTS_FUSED, for an evaluator that is a pure function of
 * (observation, legal actions) such as VPNetEvaluator (vpevaluator.cc:70-98,
 * one cached inference serves both calls): every leaf request is kind 3 and
 * its priors are kept for the node's later expansion, so each simulation
 * costs one round.  Results are identical for a pure evaluator. */
#define OS_AZ_REQUESTS_SEPARATE 0
#define OS_AZ_REQUESTS_FUSED 1
int os_az_set_requests(os_engine* e, int32_t mode);
/* Kernel of the next os_az_prepare*: OS_LAYOUT_WAVE (one wavefront per search:
 * coalesced child scans, lane-parallel expansion / backup / request writes),
 * OS_LAYOUT_LANE (one lane per search; the only one that garbage-collects,
 * mcts.cc:402-424) or OS_LAYOUT_AUTO (default: wave unless the node budget can
 * be reached).  Same results either way. */
int os_az_set_layout(os_engine* e, int32_t layout);
/* The kernel the last os_az_prepare* chose (OS_LAYOUT_WAVE or OS_LAYOUT_LANE),
 * AUTO resolved by the engine's own rule. */
int os_az_get_layout(os_engine* e, int32_t* layout);
/* Evaluator requests the batch's steps have written so far (all steps since
 * os_az_prepare*, counted on the device by the step's request reduction). */
int os_az_requests(os_engine* e, int64_t* total);
/* Measurement: with timing on, every search run of the engine (the batch,
 * stateful and rerun paths) is bracketed by a HIP event pair on its stream;
 * os_engine_last_run_ms waits for the last one and returns its duration, so
 * a caller can time a whole bot step and the kernel inside it in one run. */
int os_engine_set_run_timing(os_engine* e, int32_t on);
int os_engine_last_run_ms(os_engine* e, double* ms);
/* Root Dirichlet noise drawn by the CALLER, for the batch of the last
 * os_az_prepare*: noise[r * stride + j] pairs with root r's j-th legal action
 * (ascending), mixed at the root's expansion as (1 - eps) * prior + eps *
 * noise (mcts.py:314-317, mcts.cc:265-273) without consuming bot words.  For
 * OS_POLICY_NUMPY batches, whose noise is RandomState.dirichlet on the
 * caller's own RandomState (mcts.py:315): the caller draws it where the
 * reference does -- first on the stream, since an external evaluator draws
 * nothing before the root's expansion -- and passes the stream after the draw
 * to os_az_prepare_stateful.  noise == NULL removes the noise. */
int os_az_set_noise(os_engine* e, const double* noise, int64_t stride, double eps);
/* Priors of search r's tree nodes in os_engine_tree's node order (the root's
 * is 1; children's are the evaluator's, mixed with the root noise); count =
 * the node count os_engine_tree reports.  After os_az_fetch. */
int os_az_tree_priors(os_engine* e, int64_t r, int64_t count, double* prior);
/* The Dirichlet noise os_az_prepare draws for one fresh MCTSBot(seed) at a
 * root with `count` legal actions: out[count] (normalised, legal-action
 * order); returns the MT19937 words consumed (< 0 on error).  Exposed so the
 * noise can be checked against libstdc++ directly. */
int64_t os_dirichlet_noise(uint32_t seed, int32_t count, double alpha, double* out);
int os_az_step_async(os_engine* e, void* hip_stream);
int os_az_fetch(os_engine* e, int32_t max_children, int32_t* child_action, int32_t* child_n,
                double* child_w, int8_t* child_out, int32_t* nchild, int32_t* root_n,
                double* root_w, int8_t* root_out, int64_t* best_action, int32_t* nodes);
/* Policy / value heads of an evaluator network, fused into one kernel on
 * hip_stream (optional: an evaluator may compute the responses any way it
 * likes).  Row r of `logits` (element stride ld; dtype 0 = f32, 1 = bf16)
 * holds num_actions policy logits, then the value logit.  As the reference
 * network's heads (alpha_zero/model.py:278-282, 304): illegal logits
 * (legal[r * num_actions + a] == 0) become -1e32, prior[r][a] = their softmax,
 * value[r] = tanh(value logit); f64 arithmetic, written straight into the
 * engine's response buffers (dev_prior / dev_value of os_az_prepare).  The
 * reference model evaluates its heads in float32 (TensorFlow softmax / tanh),
 * so these priors agree with a float32 softmax to float32 rounding, not
 * bitwise; search parity is defined on the responses the engine receives,
 * whatever produced them. */
int os_az_heads_async(const void* logits, int32_t dtype, int64_t num_rows, int32_t num_actions,
                      int64_t ld, const uint8_t* legal, double* prior, double* value,
                      void* hip_stream);
/* A whole evaluator round for a one-hidden-layer network, fused into one
 * kernel on hip_stream: h = relu(bf16(obs) . W1) (f32 accumulation, bf16),
 * logits = bf16(h . Wout), then the heads of os_az_heads_async (f64).  obs
 * f32 [num_rows][obs_size] (the engine's dev_obs), w1t bf16 [hidden][128]
 * (W1 transposed, K zero-padded to 128), wout bf16 [16][hidden] (row a =
 * action a's logit weights, row num_actions = the value's, the rest zero).
 * obs_size <= 128, hidden a multiple of 32 and <= 256, num_actions + 1 <= 16.
 * Both products run on the matrix cores (v_mfma_f32_16x16x32_bf16). */
int os_az_mlp_heads_async(const float* obs, int64_t num_rows, int32_t obs_size,
                          const uint16_t* w1t, int32_t hidden, const uint16_t* wout,
                          int32_t num_actions, const uint8_t* legal, double* prior,
                          double* value, void* hip_stream);

/* ---- Self-play -----------------------------------
 * num_games independent games, each played on the device the way
 * examples/mcts_example.cc:77-136 PlayGame drives two MCTSBots sharing ONE
 * RandomRolloutEvaluator (mcts_example.cc:151-157; evaluate_bots.cc:21-60):
 * every move is bots[CurrentPlayer]->Step(state) = MCTSearch + BestChild
 * (mcts.cc:219-226), the bots' rng_ (seeds bot_seeds[2g], bot_seeds[2g+1])
 * and the evaluator's rng (eval_seeds[g]) persisting across moves;
 * MCTSBot::InformAction / Restart are no-ops (mcts.h:162-163).  Game g starts
 * from history start_actions[start_offsets[g] .. start_offsets[g+1]).
 * Outputs: actions[g][max_len] (-1 padded), length[g], returns[g][2]; if
 * visits != NULL, visits[g][move][A] = the root children's explore_count
 * indexed by action (A = NumDistinctActions), i.e. the MCTS policy targets;
 * if observations != NULL, observations[g][move][C*H*W] = ObservationTensor
 * of the position searched, for the player to move (os_state_observation_
 * tensor layout) -- a trajectory buffer for training without a host replay
 * (alpha_zero.cc:50-62).  Rows past the game end are
 * zero.  C++ policy only (OS_POLICY_NUMPY -> OS_ERR_UNSUPPORTED).  A game
 * longer than max_len fails with OS_ERR_CAPACITY. */
int os_selfplay(os_engine* e, const os_mcts_params* p, int64_t num_games,
                const int64_t* start_actions, const int64_t* start_offsets,
                const uint32_t* bot_seeds, const uint32_t* eval_seeds, int32_t max_len,
                int64_t* actions, int32_t* length, double* returns, int32_t* visits,
                float* observations);
/* The same as prepare / run (async, on hip_stream) / fetch (synchronising);
 * `record` is a mask of OS_RECORD_* selecting the optional buffers, which
 * fetch then requires (NULL skips the copy). */
#define OS_RECORD_VISITS 1
#define OS_RECORD_OBSERVATIONS 2
#define OS_RECORD_POLICY 4       /* f64 [G][max_len][A]: the normalised move policy */
#define OS_RECORD_ROOT_VALUES 8  /* f64 [G][max_len]: root total_reward / explore_count */

/* AlphaZero's PlayGame move choice (alpha_zero.cc:64-118) for the next
 * os_selfplay_prepare on this engine.  Each move's policy over the root's
 * children is pow(explore_count, 1 / temperature), normalised
 * (NormalizePolicy, spiel.cc:327-335); while fewer than temperature_drop
 * moves have been played in the game the action is SampleAction(policy,
 * actor rng) (absl::Uniform(rng, 0.0, 1.0), spiel.cc:337-366), then BestChild.
 * The root value is root total_reward / explore_count.  With resign != 0,
 * the game's cutoff is drawn at its start from the same actor rng
 * (alpha_zero.cc:154-157: u < cutoff_probability ? cutoff_value :
 * MaxUtility + 1) and the game stops after a move whose |root value| exceeds
 * it, returns[mover] = root value, returns[other] = -root value (:105-110).
 * actor_seeds[g] seeds game g's std::mt19937 actor rng.  temperature <= 0
 * restores the default (BestChild every move, mcts_example.cc); the policy
 * and root values are then still recorded, with exponent 1. */
typedef struct {
  double temperature;
  int32_t temperature_drop;
  int32_t resign;
  double cutoff_value;
  double cutoff_probability;
} os_selfplay_options;
int os_selfplay_set_options(os_engine* e, const os_selfplay_options* options,
                            int64_t num_games, const uint32_t* actor_seeds);
/* The recorded targets of the last fetched self-play run (NULL skips). */
int os_selfplay_fetch_targets(os_engine* e, double* policy, double* root_values);
int os_selfplay_prepare(os_engine* e, const os_mcts_params* p, int64_t num_games,
                        const int64_t* start_actions, const int64_t* start_offsets,
                        const uint32_t* bot_seeds, const uint32_t* eval_seeds,
                        int32_t max_len, int32_t record);
int os_selfplay_run_async(os_engine* e, void* hip_stream);
int os_selfplay_fetch(os_engine* e, int64_t* actions, int32_t* length, double* returns,
                      int32_t* visits, float* observations);

/* Device-resident rollout pipeline (go playouts/s): prepare
 * uploads the root and n evaluator seeds; run launches the rollout kernel on
 * `hip_stream` without host synchronisation; fetch synchronises and copies
 * out_returns[2*i+{0,1}] (same as os_rollouts_batch, which is prepare + run +
 * fetch).  Preparing rollouts invalidates a prepared search batch and vice
 * versa (they share the engine's root/seed buffers). */
int os_rollouts_prepare(os_engine* e, const int64_t* root_actions, int64_t n_actions,
                        int64_t n, int32_t n_rollouts, const uint32_t* seeds);
int os_rollouts_run_async(os_engine* e, void* hip_stream);
int os_rollouts_fetch(os_engine* e, double* out_returns);
/* Outcome counts of the last rollout run into DEVICE memory dev_counts[3]
 * (int64: player 0 won, player 1 won, draw — by the sign of each evaluator's
 * mean player-0 return), on hip_stream; overwrites dev_counts.  Lets ranks
 * all-reduce the totals without a host round trip. */
int os_rollouts_outcomes_async(os_engine* e, int64_t* dev_counts, void* hip_stream);
/* Instrumentation of the last lane-layout rollout run (k_rollouts), for the
 * algorithmic-bytes model of bench.py: out[0] = MT19937 words drawn, out[1] =
 * moves played (both summed over the batch), out[2] = root state bytes.  No
 * reference counterpart (the reference has no device). */
int os_rollouts_stats(os_engine* e, int64_t* out);

/* Root-parallel MCTS (the reference has no root-parallel
 * driver — each tree is one MCTSBot::MCTSearch, mcts.cc:325-428): action-indexed
 * sums over the prepared roots of the last run of the root children's
 * explore_count and total_reward (mcts.h:117-118), into DEVICE buffers
 * dev_visits[num_actions] (int64) and dev_rewards[num_actions] (f64) on
 * hip_stream, in a fixed summation order (deterministic).  num_actions >=
 * NumDistinctActions.  The caller all-reduces them across GPUs (RCCL). */
int os_engine_root_sums_async(os_engine* e, int32_t num_actions, int64_t* dev_visits,
                              double* dev_rewards, void* hip_stream);

/* Root-parallel MCTS over several devices of ONE process (SURVEY.md §8b B3
 * os_root_parallel, §8e C4; the reference's counterpart is one MCTSBot::
 * MCTSearch per tree, mcts.cc:325-428, e.g. driven by mcts_example.cc):
 * engines[g] (g < ndev; one per device, or several on one device) each grow
 * trees_per_device trees on the same root, the history root_actions[0 ..
 * n_actions); tree t of engine g uses bot seed seed_base + g * T + t and
 * evaluator seed that + 2^20 (T = trees_per_device).  Every engine's search
 * is launched before any wait; each device sums its trees' root children by
 * action (os_engine_root_sums_async), the per-device sums cross to engines[0]'s
 * device peer-to-peer (xGMI) and are added there in engine order, so the
 * result is deterministic.  Writes out_visits[num_actions] (int64, summed
 * explore_count) and out_rewards[num_actions] (f64, summed total_reward) on
 * the host and, if out_sims != NULL, the simulations run.  Synchronous. */
int os_root_parallel(os_engine* const* engines, int32_t ndev, const os_mcts_params* p,
                     const int64_t* root_actions, int64_t n_actions,
                     int64_t trees_per_device, uint32_t seed_base, int32_t num_actions,
                     int64_t* out_visits, double* out_rewards, int64_t* out_sims);

/* ---- Device-resident pipeline (inputs already in HBM; for benchmarks) ---
 * prepare: upload roots + seeds and size the arena; run: launch the search
 * kernel on `hip_stream` (a hipStream_t, or NULL for the null stream) with no
 * host synchronisation; fetch: synchronise and copy results out (same layout
 * as os_mcts_batch). */
int os_engine_prepare(os_engine* e, const os_mcts_params* p, int64_t num_roots,
                      const int64_t* root_actions, const int64_t* root_offsets,
                      const uint32_t* bot_seeds, const uint32_t* eval_seeds);
int os_engine_run_async(os_engine* e, void* hip_stream);
int os_engine_fetch(os_engine* e, int32_t max_children, int32_t* child_action,
                    int32_t* child_n, double* child_w, int8_t* child_out,
                    int32_t* nchild, int32_t* root_n, double* root_w,
                    int8_t* root_out, int64_t* best_action, int32_t* nodes);
/* Summed simulations over the prepared roots of the last run (after fetch). */
int64_t os_engine_last_sims(os_engine* e);
/* Instrumentation of the last fetched run, summed over roots:
 * out[0] sims, [1] children scanned by UCT selection, [2] nodes backed up,
 * [3] children expanded, [4] children scanned by the solver backup,
 * [5] MT19937 words drawn, [6] reference nodes_ counter, [7] arena slots
 * used, [8] max tree depth, [9] GC runs.  out has 10 entries. */
int os_engine_stats(os_engine* e, int64_t* out);
/* Bytes per arena node (16 for n_rollouts == 1, else 24) and per root state. */
int32_t os_engine_node_bytes(os_engine* e);
int32_t os_engine_state_bytes(os_engine* e);

/* Deterministic benchmark roots: root i = initial state plus
 * k_i = g() % (max_plies + 1) uniformly random legal plies drawn from
 * std::mt19937 g(seed_base + i), stopping before any ply that would end the
 * game; a root left at a chance node (pig) gets drawn outcomes until it is a
 * decision node.  Writes histories (offsets has num_roots + 1 entries); returns the
 * total action count, or < 0 on error.  actions may be NULL to size. */
int64_t os_make_roots(const os_game* game, int64_t num_roots, uint32_t seed_base,
                      int32_t max_plies, int64_t* actions, int64_t* offsets);

/* SampleAction(outcomes, rng) (spiel.cc:337-366), as EvaluateBots
 * (evaluate_bots.cc:24-61) samples chance nodes: z = absl::Uniform(rng, 0.0,
 * 1.0) from a std::mt19937 held in numpy's legacy (key[624], pos) form
 * (advanced in place); returns the index of the first outcome whose
 * [sum, sum + probs[k]) holds z, or < 0 on error. */
int32_t os_sample_action(const double* probs, int32_t n, uint32_t* key, int32_t* pos);

/* sizeof of the named ABI struct ("os_mcts_params", "os_game_info",
 * "os_selfplay_options") as this library was built, or OS_ERR_INVALID for an
 * unknown name: lets a binding (ctypes, cgo, JNI) check its own layout once at
 * load time.  No reference counterpart (pybind11 checks types at compile
 * time, pyspiel.cc:499-524). */
int64_t os_abi_struct_size(const char* name);

/* Library/kernel build info string (arch, build flags). */
const char* os_build_info(void);

/* Diagnostic (no reference counterpart): shader-clock cycles per search phase
 * of the wave-layout kernel summed over all waves since the last call
 * (select, expand, rollout, backup, solver, tail, mt-twist, total), then reset.
 * Returns the number of phases written; OS_ERR_UNSUPPORTED unless the library
 * was built with -DOS_PHASE_TIMING=1. */
int os_debug_phase_cycles(uint64_t* out, int32_t n);
/* Diagnostic (no reference counterpart): the first `count` arena nodes
 * (Node<double>, 24 B: first u32, n i32, w f64, action u16, nchild u8, out i8)
 * and priors of search r of the prepared external-evaluator batch. */
int os_debug_az_arena(os_engine* e, int64_t r, int32_t count, void* out_nodes,
                      double* out_prior);

#ifdef __cplusplus
}
#endif

#endif /* OS_MCTS_C_ABI_H_ */
