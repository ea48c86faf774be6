// Host-side game objects shared by the State API and the engine launcher.
#ifndef OS_HOST_H_
#define OS_HOST_H_

#include <cstdint>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "os_games.h"

namespace osm {

// Host state record: any G::State, big-board hex / go included.
constexpr int kStateBytes = 320;  // >= every G::State (HexBig: 296 B)
constexpr int kB128Side = 11;     // hex / go sides on B128 bitboards (device kernels)
constexpr int kMaxSide = 19;      // hex / go sides on B384 bitboards (host State API)

struct HostGame {
  GameCfg cfg;
  std::string name;          // short name
  std::string canonical;     // canonical game string
  std::vector<uint64_t> zob; // go: [n*n][2]
  int state_bytes = 0;
};

// Contiguous storage of one GoCtx's position log on the host.
struct HostGoLog {
  std::vector<uint64_t> log;
  std::vector<uint32_t> link;
  std::vector<uint8_t> head;
  void bind(GoCtx* c, int cap, int cells) {  // cap <= 255
    log.assign(cap, 0);
    link.assign(cap, 0);
    head.assign(cells + 1, 0);
    c->log = log.data();
    c->link = link.data();
    c->head = head.data();
    c->stride = 1;
    c->head_stride = 1;
    c->cap = cap;
    c->n_heads = cells + 1;
  }
};

struct HostState {
  const HostGame* game;
  alignas(16) unsigned char raw[kStateBytes];
  std::vector<int64_t> history;
  std::vector<uint64_t> hashes;  // go: positions seen, incl. the initial one
};

// A GoCtx whose base is the state's whole position history (the reference's
// repetitions_ set, go.h:105-120) and whose log is empty, in `buf`.
GoCtx HostGoCtx(const HostState& s, HostGoLog* buf);

// dirichlet_noise(count, alpha, &rng_) of mcts.cc:177-192 drawn from a fresh
// std::mt19937(seed) with libstdc++'s own std::gamma_distribution<double>
// (its Marsaglia-Tsang sampler and libm calls make the bits), normalised by
// the left-fold sum; writes out[count] and returns the MT words consumed.
int64_t DirichletNoise(uint32_t seed, int count, double alpha, double* out);
// The same draw from a bot rng_ held in numpy's (key[624], pos) form (a bot
// whose stream has advanced over earlier searches).
int64_t DirichletNoiseState(const uint32_t* key, int pos, int count, double alpha, double* out);

// Parses and validates a game string; returns "" on success, else a message.
// `unsupported` is set when the game/parameters are valid OpenSpiel but not
// supported by this engine.
std::string LoadHostGame(const std::string& gs, HostGame* g, bool* unsupported);

// go.cc:56-78 HandicapStones(handicap) as cell indices row * n + col (empty
// unless 2 <= handicap <= 9).
std::vector<int> GoHandicapStones(int handicap, int n);

// Game::NumPlayers (2, or pig's `players`).
int NumPlayers(const GameCfg& g);

void StateInit(HostState* s);
bool StateTerminal(const HostState& s);
int StateCurrentPlayer(const HostState& s);
void StateLegal(const HostState& s, std::vector<int64_t>* out);
// Returns false if the action is illegal.
bool StateApply(HostState* s, int64_t a);
void StateReturns(const HostState& s, double* r);
// IsChanceNode (spiel.h:331) and ChanceOutcomes (spiel.h:322-327, outcome
// order); empty unless the state is a chance node.
bool StateIsChance(const HostState& s);
void StateChanceOutcomes(const HostState& s, std::vector<std::pair<int64_t, double>>* out);
// ObservationTensorShape: {C, H, W}; returns C * H * W.
int ObservationShape(const HostGame& g, int32_t* shape3);
// ObservationTensor(player) as float [C][H][W] (size ObservationShape).
void StateObservation(const HostState& s, int player, float* out);
std::string StateToString(const HostState& s);
std::string StateActionToString(const HostState& s, int player, int64_t a);

// Fills the go context for host-side use (all hashes in `log`).
GoCtx HostGoCtx(const HostState& s, std::vector<uint64_t>* storage);

}  // namespace osm

#endif  // OS_HOST_H_
