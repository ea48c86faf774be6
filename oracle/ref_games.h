// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_rng.h header).
//
// Reference-faithful CPU restatement of the five target games and the subset
// of the OpenSpiel State/Game API the MCTS path calls (spiel.h:173-750).  The
// restatement deliberately keeps the reference's cost structure (virtual
// State, heap Clone, std::vector LegalActions, per-cell board arrays, go's
// chain/pseudo-liberty board) so that it doubles as the CPU baseline.
//
//   tic_tac_toe   open_spiel/games/tic_tac_toe.cc:80-150
//   connect_four  open_spiel/games/connect_four.cc:85-185
//   breakthrough  open_spiel/games/breakthrough.cc:119-320
//   hex           open_spiel/games/hex.cc:55-255
//   go            open_spiel/games/go.cc:124-216, go/go_board.cc:217-597
//   pig           open_spiel/games/pig.cc:81-244 (chance nodes)
#ifndef OS_ORACLE_REF_GAMES_H_
#define OS_ORACLE_REF_GAMES_H_

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

namespace oref {

using Action = int64_t;
using Player = int;
constexpr Player kTerminalPlayerId = -4;   // spiel.h PlayerId::TERMINAL
constexpr Player kChancePlayerId = -1;     // spiel.h PlayerId::CHANCE
constexpr Player kInvalidPlayer = -3;
constexpr Action kInvalidAction = -1;

struct GameParams {
  std::map<std::string, std::string> kv;
  int GetInt(const std::string& k, int dflt) const;
  double GetDouble(const std::string& k, double dflt) const;
};

// Parses "name(k=v,...)" (game_parameters.cc:101-130 semantics for the flat
// case the five games need).
bool ParseGameString(const std::string& s, std::string* name, GameParams* p);

class RGame;

class RState {
 public:
  virtual ~RState() = default;
  virtual Player CurrentPlayer() const = 0;
  virtual std::vector<Action> LegalActions() const = 0;
  virtual bool IsTerminal() const = 0;
  virtual std::vector<double> Returns() const = 0;
  virtual std::unique_ptr<RState> Clone() const = 0;
  virtual std::string ToString() const = 0;
  virtual std::string ActionToString(Player p, Action a) const = 0;
  // spiel.h:331 IsChanceNode (CurrentPlayer() == kChancePlayerId) and
  // ChanceOutcomes (:322-327); only pig has chance nodes.
  bool IsChanceNode() const { return CurrentPlayer() == kChancePlayerId; }
  virtual std::vector<std::pair<Action, double>> ChanceOutcomes() const { return {}; }
  // spiel.h:205-210: ApplyAction = DoApplyAction + history_.push_back.
  void ApplyAction(Action a) {
    DoApplyAction(a);
    history_.push_back(a);
  }
  const std::vector<Action>& History() const { return history_; }

 protected:
  virtual void DoApplyAction(Action a) = 0;
  std::vector<Action> history_;
};

class RGame {
 public:
  virtual ~RGame() = default;
  virtual std::unique_ptr<RState> NewInitialState() const = 0;
  virtual int NumDistinctActions() const = 0;
  virtual int MaxGameLength() const = 0;
  virtual double MaxUtility() const { return 1.0; }
  virtual double MinUtility() const { return -1.0; }
  virtual std::string ShortName() const = 0;
  virtual int NumPlayers() const { return 2; }
};

// Returns nullptr (and sets *err) for unknown games / unsupported params.
// Tromp-Taylor score of a go state's board (go_board.cc:555-597).
float GoScore(const RState& s);

std::unique_ptr<RGame> LoadGame(const std::string& game_string,
                                std::string* err);

}  // namespace oref

#endif  // OS_ORACLE_REF_GAMES_H_
