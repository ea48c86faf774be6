// ORACLE — TEST INFRASTRUCTURE ONLY (see ref_rng.h header).
// Reference-faithful restatement of the five target games; every class cites
// the reference lines whose behaviour it restates.
#include "ref_games.h"

#include <algorithm>
#include <cstdlib>
#include <iomanip>
#include <random>
#include <sstream>

namespace oref {

int GameParams::GetInt(const std::string& k, int dflt) const {
  auto it = kv.find(k);
  return it == kv.end() ? dflt : std::atoi(it->second.c_str());
}
double GameParams::GetDouble(const std::string& k, double dflt) const {
  auto it = kv.find(k);
  return it == kv.end() ? dflt : std::atof(it->second.c_str());
}

bool ParseGameString(const std::string& s, std::string* name, GameParams* p) {
  size_t lp = s.find('(');
  if (lp == std::string::npos) {
    *name = s;
    return !s.empty();
  }
  if (s.back() != ')') return false;
  *name = s.substr(0, lp);
  std::string body = s.substr(lp + 1, s.size() - lp - 2);
  size_t pos = 0;
  while (pos < body.size()) {
    size_t comma = body.find(',', pos);
    if (comma == std::string::npos) comma = body.size();
    std::string item = body.substr(pos, comma - pos);
    size_t eq = item.find('=');
    if (eq == std::string::npos) return false;
    p->kv[item.substr(0, eq)] = item.substr(eq + 1);
    pos = comma + 1;
  }
  return true;
}

// ---------------------------------------------------------------------------
// tic_tac_toe (tic_tac_toe.cc:80-150, tic_tac_toe.h:30-121)
namespace ttt {
enum class Cell { kEmpty, kNought, kCross };
inline Cell PlayerCell(Player p) { return p == 0 ? Cell::kCross : Cell::kNought; }
inline const char* CellStr(Cell c) {
  return c == Cell::kEmpty ? "." : (c == Cell::kNought ? "o" : "x");
}

class State : public RState {
 public:
  State() { board_.fill(Cell::kEmpty); }
  Player CurrentPlayer() const override {
    return IsTerminal() ? kTerminalPlayerId : cur_;
  }
  std::vector<Action> LegalActions() const override {
    std::vector<Action> v;
    if (IsTerminal()) return v;
    for (int c = 0; c < 9; ++c)
      if (board_[c] == Cell::kEmpty) v.push_back(c);
    return v;
  }
  bool IsTerminal() const override {
    return winner_ != kInvalidPlayer || moves_ == 9;
  }
  std::vector<double> Returns() const override {
    if (winner_ == 0) return {1.0, -1.0};
    if (winner_ == 1) return {-1.0, 1.0};
    return {0.0, 0.0};
  }
  std::unique_ptr<RState> Clone() const override {
    return std::make_unique<State>(*this);
  }
  std::string ToString() const override {
    std::string s;
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) s += CellStr(board_[r * 3 + c]);
      if (r < 2) s += "\n";
    }
    return s;
  }
  std::string ActionToString(Player p, Action a) const override {
    return std::string(CellStr(PlayerCell(p))) + "(" + std::to_string(a / 3) +
           "," + std::to_string(a % 3) + ")";
  }

 protected:
  void DoApplyAction(Action a) override {
    board_[a] = PlayerCell(cur_);
    if (HasLine(cur_)) winner_ = cur_;
    cur_ = 1 - cur_;
    moves_ += 1;
  }

 private:
  bool HasLine(Player p) const {
    static const int kLines[8][3] = {{0, 1, 2}, {3, 4, 5}, {6, 7, 8},
                                     {0, 3, 6}, {1, 4, 7}, {2, 5, 8},
                                     {0, 4, 8}, {2, 4, 6}};
    Cell c = PlayerCell(p);
    for (auto& l : kLines)
      if (board_[l[0]] == c && board_[l[1]] == c && board_[l[2]] == c)
        return true;
    return false;
  }
  std::array<Cell, 9> board_;
  Player cur_ = 0;
  Player winner_ = kInvalidPlayer;
  int moves_ = 0;
};

class Game : public RGame {
 public:
  std::unique_ptr<RState> NewInitialState() const override {
    return std::make_unique<State>();
  }
  int NumDistinctActions() const override { return 9; }
  int MaxGameLength() const override { return 9; }
  std::string ShortName() const override { return "tic_tac_toe"; }
};
}  // namespace ttt

// ---------------------------------------------------------------------------
// connect_four (connect_four.cc:85-185, connect_four.h:36-136)
namespace c4 {
constexpr int kRows = 6, kCols = 7;
enum class Cell { kEmpty, kNought, kCross };
enum class Outcome { kP0 = 0, kP1 = 1, kUnknown, kDraw };
inline Cell PlayerCell(Player p) { return p == 0 ? Cell::kCross : Cell::kNought; }
inline const char* CellStr(Cell c) {
  return c == Cell::kEmpty ? "." : (c == Cell::kNought ? "o" : "x");
}

class State : public RState {
 public:
  State() { board_.fill(Cell::kEmpty); }
  Player CurrentPlayer() const override {
    return IsTerminal() ? kTerminalPlayerId : cur_;
  }
  std::vector<Action> LegalActions() const override {
    std::vector<Action> v;
    if (IsTerminal()) return v;
    for (int c = 0; c < kCols; ++c)
      if (At(kRows - 1, c) == Cell::kEmpty) v.push_back(c);
    return v;
  }
  bool IsTerminal() const override { return outcome_ != Outcome::kUnknown; }
  std::vector<double> Returns() const override {
    if (outcome_ == Outcome::kP0) return {1.0, -1.0};
    if (outcome_ == Outcome::kP1) return {-1.0, 1.0};
    return {0.0, 0.0};
  }
  std::unique_ptr<RState> Clone() const override {
    return std::make_unique<State>(*this);
  }
  std::string ToString() const override {
    std::string s;
    for (int r = kRows - 1; r >= 0; --r) {
      for (int c = 0; c < kCols; ++c) s += CellStr(At(r, c));
      s += "\n";
    }
    return s;
  }
  std::string ActionToString(Player p, Action a) const override {
    return std::string(CellStr(PlayerCell(p))) + std::to_string(a);
  }

 protected:
  void DoApplyAction(Action a) override {
    int r = 0;
    while (At(r, a) != Cell::kEmpty) ++r;
    board_[r * kCols + a] = PlayerCell(cur_);
    if (HasLine(cur_)) {
      outcome_ = static_cast<Outcome>(cur_);
    } else if (IsFull()) {
      outcome_ = Outcome::kDraw;
    }
    cur_ = 1 - cur_;
  }

 private:
  Cell At(int r, int c) const { return board_[r * kCols + c]; }
  bool LineFromDir(Player p, int r, int c, int dr, int dc) const {
    if (r + 3 * dr >= kRows || c + 3 * dc >= kCols || r + 3 * dr < 0 ||
        c + 3 * dc < 0)
      return false;
    Cell want = PlayerCell(p);
    for (int i = 0; i < 4; ++i, r += dr, c += dc)
      if (At(r, c) != want) return false;
    return true;
  }
  // Full-board scan, as the reference does after every move (:144-152).
  bool HasLine(Player p) const {
    Cell want = PlayerCell(p);
    for (int c = 0; c < kCols; ++c)
      for (int r = 0; r < kRows; ++r)
        if (At(r, c) == want &&
            (LineFromDir(p, r, c, 0, 1) || LineFromDir(p, r, c, -1, -1) ||
             LineFromDir(p, r, c, -1, 0) || LineFromDir(p, r, c, -1, 1)))
          return true;
    return false;
  }
  bool IsFull() const {
    for (int c = 0; c < kCols; ++c)
      if (At(kRows - 1, c) == Cell::kEmpty) return false;
    return true;
  }
  std::array<Cell, kRows * kCols> board_;
  Player cur_ = 0;
  Outcome outcome_ = Outcome::kUnknown;
};

class Game : public RGame {
 public:
  std::unique_ptr<RState> NewInitialState() const override {
    return std::make_unique<State>();
  }
  int NumDistinctActions() const override { return kCols; }
  int MaxGameLength() const override { return kRows * kCols; }
  std::string ShortName() const override { return "connect_four"; }
};
}  // namespace c4

// ---------------------------------------------------------------------------
// breakthrough (breakthrough.cc:119-320, breakthrough.h:30-143)
namespace bt {
constexpr int kDirs = 6;
constexpr int kDirRow[kDirs] = {1, 1, 1, -1, -1, -1};
constexpr int kDirCol[kDirs] = {-1, 0, 1, -1, 0, 1};
enum class Cell { kEmpty, kBlack, kWhite };
inline Cell PlayerCell(Player p) { return p == 0 ? Cell::kBlack : Cell::kWhite; }
inline Player CellPlayer(Cell c) { return c == Cell::kBlack ? 0 : 1; }
inline Cell Opp(Cell c) { return PlayerCell(1 - CellPlayer(c)); }

// spiel_utils.cc:45-73 mixed-base ranking, bases {rows, cols, 6, 2}.
inline Action Rank(const std::vector<int>& bases, const std::vector<int>& d) {
  Action a = 0;
  int mult = 1;
  for (int i = static_cast<int>(d.size()) - 1; i >= 0; --i) {
    a += d[i] * mult;
    mult *= bases[i];
  }
  return a;
}
inline void Unrank(Action a, const std::vector<int>& bases,
                   std::vector<int>* d) {
  for (int i = static_cast<int>(d->size()) - 1; i >= 0; --i) {
    (*d)[i] = a % bases[i];
    a /= bases[i];
  }
}

class State : public RState {
 public:
  State(int rows, int cols) : rows_(rows), cols_(cols) {
    board_.assign(rows * cols, Cell::kEmpty);
    const bool two = rows >= 6;
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) {
        if (r == 0 || (two && r == 1)) Set(r, c, Cell::kBlack);
        else if (r == rows - 1 || (two && r == rows - 2)) Set(r, c, Cell::kWhite);
      }
    pieces_[0] = pieces_[1] = cols * (two ? 2 : 1);
  }
  Player CurrentPlayer() const override {
    return IsTerminal() ? kTerminalPlayerId : cur_;
  }
  std::vector<Action> LegalActions() const override {
    std::vector<Action> moves;
    if (IsTerminal()) return moves;
    const Player p = CurrentPlayer();
    const Cell mine = PlayerCell(p);
    std::vector<int> bases = {rows_, cols_, kDirs, 2};
    std::vector<int> vals = {0, 0, 0, 0};
    for (int r = 0; r < rows_; ++r)
      for (int c = 0; c < cols_; ++c) {
        if (At(r, c) != mine) continue;
        for (int o = 0; o < kDirs / 2; ++o) {
          int dir = p * kDirs / 2 + o;
          int rp = r + kDirRow[dir], cp = c + kDirCol[dir];
          if (!InBounds(rp, cp)) continue;
          vals[0] = r; vals[1] = c; vals[2] = dir;
          if (At(rp, cp) == Cell::kEmpty) {
            vals[3] = 0;
            moves.push_back(Rank(bases, vals));
          } else if ((o == 0 || o == 2) && At(rp, cp) == Opp(mine)) {
            vals[3] = 1;
            moves.push_back(Rank(bases, vals));
          }
        }
      }
    return moves;
  }
  bool IsTerminal() const override {
    return winner_ >= 0 || pieces_[0] == 0 || pieces_[1] == 0;
  }
  std::vector<double> Returns() const override {
    if (winner_ == 0 || pieces_[1] == 0) return {1.0, -1.0};
    if (winner_ == 1 || pieces_[0] == 0) return {-1.0, 1.0};
    return {0.0, 0.0};
  }
  std::unique_ptr<RState> Clone() const override {
    return std::make_unique<State>(*this);
  }
  std::string ToString() const override {
    std::string s;
    for (int r = 0; r < rows_; ++r) {
      s += static_cast<char>('1' + (rows_ - 1 - r));
      for (int c = 0; c < cols_; ++c) {
        Cell x = At(r, c);
        s += x == Cell::kBlack ? "b" : (x == Cell::kWhite ? "w" : ".");
      }
      s += "\n";
    }
    s += " ";
    for (int c = 0; c < cols_; ++c) s += static_cast<char>('a' + c);
    s += "\n";
    return s;
  }
  std::string ActionToString(Player, Action a) const override {
    std::vector<int> v(4, -1);
    Unrank(a, {rows_, cols_, kDirs, 2}, &v);
    int r2 = v[0] + kDirRow[v[2]], c2 = v[1] + kDirCol[v[2]];
    std::string s;
    s += static_cast<char>('a' + v[1]);
    s += static_cast<char>('1' + (rows_ - 1 - v[0]));
    s += static_cast<char>('a' + c2);
    s += static_cast<char>('1' + (rows_ - 1 - r2));
    if (v[3] == 1) s += "*";
    return s;
  }

 protected:
  void DoApplyAction(Action a) override {
    std::vector<int> v(4, -1);
    Unrank(a, {rows_, cols_, kDirs, 2}, &v);
    int r1 = v[0], c1 = v[1], dir = v[2];
    int r2 = r1 + kDirRow[dir], c2 = c1 + kDirCol[dir];
    if (At(r2, c2) == Cell::kWhite) pieces_[1]--;
    else if (At(r2, c2) == Cell::kBlack) pieces_[0]--;
    Set(r2, c2, At(r1, c1));
    Set(r1, c1, Cell::kEmpty);
    if (cur_ == 0 && r2 == rows_ - 1) winner_ = 0;
    else if (cur_ == 1 && r2 == 0) winner_ = 1;
    cur_ = 1 - cur_;
  }

 private:
  bool InBounds(int r, int c) const {
    return r >= 0 && r < rows_ && c >= 0 && c < cols_;
  }
  Cell At(int r, int c) const { return board_[r * cols_ + c]; }
  void Set(int r, int c, Cell x) { board_[r * cols_ + c] = x; }
  int rows_, cols_;
  Player cur_ = 0;
  int winner_ = kInvalidPlayer;
  std::array<int, 2> pieces_;
  std::vector<Cell> board_;
};

class Game : public RGame {
 public:
  Game(int rows, int cols) : rows_(rows), cols_(cols) {}
  std::unique_ptr<RState> NewInitialState() const override {
    return std::make_unique<State>(rows_, cols_);
  }
  int NumDistinctActions() const override { return rows_ * cols_ * kDirs * 2; }
  int MaxGameLength() const override { return 2 * (2 * rows_ - 3) * cols_ + 1; }
  std::string ShortName() const override { return "breakthrough"; }

 private:
  int rows_, cols_;
};
}  // namespace bt

// ---------------------------------------------------------------------------
// hex (hex.cc:55-255, hex.h:30-131)
namespace hex {
enum Cell : int {
  kEmpty = 0, kWhiteWest = -3, kWhiteEast = -2, kWhiteWin = -4, kWhite = -1,
  kBlackNorth = 3, kBlackSouth = 2, kBlackWin = 4, kBlack = 1
};
inline const char* CellStr(int c) {
  switch (c) {
    case kEmpty: return ".";
    case kWhite: return "o";
    case kWhiteWin: return "O";
    case kWhiteWest: return "p";
    case kWhiteEast: return "q";
    case kBlack: return "x";
    case kBlackWin: return "X";
    case kBlackNorth: return "y";
    case kBlackSouth: return "z";
  }
  return "?";
}

class State : public RState {
 public:
  explicit State(int n) : n_(n), board_(n * n, kEmpty) {}
  Player CurrentPlayer() const override {
    return IsTerminal() ? kTerminalPlayerId : cur_;
  }
  std::vector<Action> LegalActions() const override {
    std::vector<Action> v;
    if (IsTerminal()) return v;
    for (int c = 0; c < n_ * n_; ++c)
      if (board_[c] == kEmpty) v.push_back(c);
    return v;
  }
  bool IsTerminal() const override { return result_ != 0; }
  std::vector<double> Returns() const override { return {result_, -result_}; }
  std::unique_ptr<RState> Clone() const override {
    return std::make_unique<State>(*this);
  }
  std::string ToString() const override {
    std::string s;
    int line = 0;
    for (int c = 0; c < n_ * n_; ++c) {
      if (c && !(c % n_)) {
        s += "\n";
        ++line;
        s += std::string(line, ' ');
      }
      s += CellStr(board_[c]);
      s += " ";
    }
    return s;
  }
  std::string ActionToString(Player p, Action a) const override {
    return std::string(CellStr(StateAfter(p, a))) + "(" +
           std::to_string(a % n_) + "," + std::to_string(a / n_) + ")";
  }

 protected:
  void DoApplyAction(Action a) override {
    int st = StateAfter(cur_, a);
    board_[a] = st;
    if (st == kBlackWin) {
      result_ = 1;
    } else if (st == kWhiteWin) {
      result_ = -1;
    } else if (st != kBlack && st != kWhite) {
      const int plain = cur_ == 0 ? kBlack : kWhite;
      std::vector<int> stack = {static_cast<int>(a)};
      while (!stack.empty()) {
        int cell = stack.back();
        stack.pop_back();
        for (int nb : Adjacent(cell)) {
          if (board_[nb] == plain) {
            board_[nb] = st;
            stack.push_back(nb);
          }
        }
      }
    }
    cur_ = 1 - cur_;
  }

 private:
  // hex.cc:206-222: six neighbours minus off-board / row-wrapping ones.
  std::vector<int> Adjacent(int cell) const {
    std::vector<int> nb = {cell - n_, cell - n_ + 1, cell - 1,
                           cell + 1,  cell + n_ - 1, cell + n_};
    for (int i = 5; i >= 0; --i) {
      if (nb[i] < 0 || nb[i] >= n_ * n_ ||
          (nb[i] % n_ == 0 && cell % n_ == n_ - 1) ||
          (nb[i] % n_ == n_ - 1 && cell % n_ == 0))
        nb.erase(nb.begin() + i);
    }
    return nb;
  }
  int StateAfter(Player p, Action move) const {
    if (p == 0) {
      bool north = false, south = false;
      if (move < n_) north = true;
      else if (move >= n_ * (n_ - 1)) south = true;
      for (int nb : Adjacent(move)) {
        if (board_[nb] == kBlackNorth) north = true;
        else if (board_[nb] == kBlackSouth) south = true;
      }
      if (north && south) return kBlackWin;
      if (north) return kBlackNorth;
      if (south) return kBlackSouth;
      return kBlack;
    }
    bool west = false, east = false;
    if (move % n_ == 0) west = true;
    else if (move % n_ == n_ - 1) east = true;
    for (int nb : Adjacent(move)) {
      if (board_[nb] == kWhiteWest) west = true;
      else if (board_[nb] == kWhiteEast) east = true;
    }
    if (west && east) return kWhiteWin;
    if (west) return kWhiteWest;
    if (east) return kWhiteEast;
    return kWhite;
  }
  int n_;
  std::vector<int> board_;
  Player cur_ = 0;
  double result_ = 0;
};

class Game : public RGame {
 public:
  explicit Game(int n) : n_(n) {}
  std::unique_ptr<RState> NewInitialState() const override {
    return std::make_unique<State>(n_);
  }
  int NumDistinctActions() const override { return n_ * n_; }
  int MaxGameLength() const override { return n_ * n_; }
  std::string ShortName() const override { return "hex"; }

 private:
  int n_;
};
}  // namespace hex

// ---------------------------------------------------------------------------
// go (go.cc:124-216, go/go_board.cc:217-597, go/go_board.h:84-235)
namespace go {
constexpr int kVB = 21;                 // virtual board side (19 + 2 guards)
constexpr int kVP = kVB * kVB;          // 441 virtual points
constexpr uint16_t kInvalidPoint = 0;
constexpr uint16_t kVirtualPass = kVP + 1;
enum Color : uint8_t { kBlack = 0, kWhite = 1, kEmpty = 2, kGuard = 3 };
inline Color Opp(Color c) {
  return c == kBlack ? kWhite : (c == kWhite ? kBlack : c);
}

// chess_common.h:113-154 ZobristTable<uint64_t, 441, 2>(2765481): outer
// mt19937_64 draws one seed per point; each seeds its own mt19937_64 which
// draws the two colour entries (full-range absl distribution = raw draw).
struct Zobrist {
  uint64_t z[kVP][2];
  Zobrist() {
    std::mt19937_64 outer(2765481);
    for (int i = 0; i < kVP; ++i) {
      std::mt19937_64 inner(outer());
      z[i][0] = inner();
      z[i][1] = inner();
    }
  }
};
inline const Zobrist& Z() {
  static const Zobrist* t = new Zobrist();
  return *t;
}

template <typename F>
inline void ForNeighbours(uint16_t p, const F& f) {
  f(static_cast<uint16_t>(p + kVB));
  f(static_cast<uint16_t>(p + 1));
  f(static_cast<uint16_t>(p - 1));
  f(static_cast<uint16_t>(p - kVB));
}

inline uint16_t FromRC(int r, int c) {
  return static_cast<uint16_t>((r + 1) * kVB + c + 1);
}

class Board {
 public:
  explicit Board(int n) : n_(n) {
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) points_.push_back(FromRC(r, c));
    Clear();
  }
  int size() const { return n_; }
  int pass_action() const { return n_ * n_; }
  const std::vector<uint16_t>& points() const { return points_; }
  Color ColorAt(uint16_t p) const { return v_[p].color; }
  bool IsEmpty(uint16_t p) const { return ColorAt(p) == kEmpty; }
  uint64_t Hash() const { return hash_; }
  uint16_t KoPoint() const { return ko_; }

  uint16_t ToVirtual(Action a) const {
    if (a == n_ * n_) return kVirtualPass;
    return FromRC(static_cast<int>(a / n_), static_cast<int>(a % n_));
  }
  Action ToAction(uint16_t vp) const {
    if (vp == kVirtualPass) return n_ * n_;
    return n_ * (vp / kVB - 1) + (vp % kVB - 1);
  }

  void Clear() {
    hash_ = 0;
    for (int i = 0; i < kVP; ++i) {
      v_[i].color = kGuard;
      v_[i].head = v_[i].next = static_cast<uint16_t>(i);
      ch_[i].ResetBorder();
    }
    for (uint16_t p : points_) {
      v_[p].color = kEmpty;
      ch_[p].Reset();
    }
    for (uint16_t p : points_)
      ForNeighbours(p, [this, p](uint16_t n) {
        if (IsEmpty(n)) ChainOf(p).AddLib(n);
      });
    last_captures_.fill(kInvalidPoint);
    ko_ = kInvalidPoint;
  }

  bool InBoard(uint16_t p) const {
    if (p == kInvalidPoint || p == kVirtualPass) return false;
    int r = p / kVB - 1, c = p % kVB - 1;
    return r >= 0 && r < n_ && c >= 0 && c < n_;
  }

  // go_board.cc:416-441
  bool IsLegal(uint16_t p, Color c) const {
    if (p == kVirtualPass) return true;
    if (!InBoard(p)) return false;
    if (!IsEmpty(p) || p == ko_) return false;
    if (ChainOf(p).npl > 0) return true;
    bool lib = false;
    ForNeighbours(p, [&](uint16_t n) {
      lib |= (ColorAt(n) == c && !ChainOf(n).InAtari());
    });
    if (lib) return true;
    bool kills = false;
    ForNeighbours(p, [&](uint16_t n) {
      kills |= (ColorAt(n) == Opp(c) && ChainOf(n).InAtari());
    });
    return kills;
  }

  // go_board.cc:217-247
  void Play(uint16_t p, Color c) {
    if (p == kVirtualPass) {
      ko_ = kInvalidPoint;
      return;
    }
    bool enemy_eye = true;
    ForNeighbours(p, [&](uint16_t n) {
      Color s = ColorAt(n);
      if (s == c || s == kEmpty) enemy_eye = false;
    });
    JoinChainsAround(p, c);
    SetStone(p, c);
    ForNeighbours(p, [this, p](uint16_t n) { ChainOf(n).RemoveLib(p); });
    int captured = CaptureDeadChains(p, c);
    ko_ = (enemy_eye && captured == 1) ? last_captures_[0] : kInvalidPoint;
  }

 private:
  struct Vertex {
    uint16_t head, next;
    Color color;
  };
  struct Chain {
    uint32_t sumsq;
    uint16_t sum;
    uint16_t stones;
    uint16_t npl;
    void ResetBorder() { stones = 0; npl = 4; sum = 32768; sumsq = 2147483648u; }
    void Reset() { stones = 0; npl = 0; sum = 0; sumsq = 0; }
    void Merge(const Chain& o) {
      stones += o.stones; npl += o.npl; sum += o.sum; sumsq += o.sumsq;
    }
    bool InAtari() const {
      return static_cast<uint32_t>(npl) * sumsq ==
             static_cast<uint32_t>(sum) * static_cast<uint32_t>(sum);
    }
    void AddLib(uint16_t p) {
      npl += 1; sum += p; sumsq += static_cast<uint32_t>(p) * p;
    }
    void RemoveLib(uint16_t p) {
      npl -= 1; sum -= p; sumsq -= static_cast<uint32_t>(p) * p;
    }
  };
  Chain& ChainOf(uint16_t p) { return ch_[v_[p].head]; }
  const Chain& ChainOf(uint16_t p) const { return ch_[v_[p].head]; }

  void SetStone(uint16_t p, Color c) {
    hash_ ^= Z().z[p][c == kEmpty ? ColorAt(p) : c];
    v_[p].color = c;
  }
  void InitChain(uint16_t p) {
    v_[p].head = v_[p].next = p;
    Chain& c = ch_[p];
    c.Reset();
    c.stones += 1;
    ForNeighbours(p, [this, &c](uint16_t n) {
      if (IsEmpty(n)) c.AddLib(n);
    });
  }
  // go_board.cc:302-342
  void JoinChainsAround(uint16_t p, Color c) {
    uint16_t big = kInvalidPoint;
    int big_size = 0;
    ForNeighbours(p, [&](uint16_t n) {
      if (ColorAt(n) == c) {
        const Chain& ch = ChainOf(n);
        if (ch.stones > big_size) {
          big_size = ch.stones;
          big = v_[n].head;
        }
      }
    });
    if (big_size == 0) {
      InitChain(p);
      return;
    }
    ForNeighbours(p, [&](uint16_t n) {
      if (ColorAt(n) != c) return;
      uint16_t h = v_[n].head;
      if (h == big) return;
      ch_[big].Merge(ChainOf(n));
      uint16_t cur = n;
      do {
        v_[cur].head = big;
        cur = v_[cur].next;
      } while (cur != n);
      std::swap(v_[big].next, v_[n].next);
    });
    v_[p].next = v_[big].next;
    v_[big].next = p;
    v_[p].head = big;
    ch_[big].stones += 1;
    ForNeighbours(p, [&](uint16_t n) {
      if (IsEmpty(n)) ch_[big].AddLib(n);
    });
  }
  // go_board.cc:348-365
  int CaptureDeadChains(uint16_t p, Color c) {
    int captured = 0, idx = 0;
    ForNeighbours(p, [&](uint16_t n) {
      if (ColorAt(n) == Opp(c) && ChainOf(n).npl == 0) {
        last_captures_[idx++] = v_[n].head;
        captured += ChainOf(n).stones;
        RemoveChain(n);
      }
    });
    for (; idx < 4; ++idx) last_captures_[idx] = kInvalidPoint;
    return captured;
  }
  // go_board.cc:367-384
  void RemoveChain(uint16_t p) {
    uint16_t head = v_[p].head;
    uint16_t cur = p;
    do {
      uint16_t next = v_[cur].next;
      SetStone(cur, kEmpty);
      InitChain(cur);
      ForNeighbours(cur, [&](uint16_t n) {
        if (v_[n].head != head || IsEmpty(n)) ChainOf(n).AddLib(cur);
      });
      cur = next;
    } while (cur != p);
  }

  int n_;
  std::vector<uint16_t> points_;
  std::array<Vertex, kVP> v_;
  std::array<Chain, kVP> ch_;
  uint64_t hash_;
  std::array<uint16_t, 4> last_captures_;
  uint16_t ko_;
};

// go_board.cc:526-553 (early-abort DFS kept verbatim in behaviour).
inline int NumSurrounded(const Board& b, uint16_t p, std::vector<bool>* marked,
                         bool* rb, bool* rw) {
  if ((*marked)[p] || (*rb && *rw)) return 0;
  (*marked)[p] = true;
  int num = 1;
  ForNeighbours(p, [&](uint16_t n) {
    switch (b.ColorAt(n)) {
      case kBlack: *rb = true; break;
      case kWhite: *rw = true; break;
      case kEmpty: num += NumSurrounded(b, n, marked, rb, rw); break;
      case kGuard: break;
    }
  });
  return num;
}

// go_board.cc:555-597
inline float TrompTaylorScore(const Board& b, float komi, int handicap) {
  int delta = 0;
  std::vector<bool> marked(kVP, false);
  for (uint16_t p : b.points()) {
    switch (b.ColorAt(p)) {
      case kBlack: ++delta; break;
      case kWhite: --delta; break;
      case kEmpty: {
        if (marked[p]) continue;
        bool rb = false, rw = false;
        int n = NumSurrounded(b, p, &marked, &rb, &rw);
        if (rb && !rw) delta += n;
        else if (!rb && rw) delta -= n;
        break;
      }
      default: break;
    }
  }
  float score = delta - komi;
  if (handicap >= 2) score -= handicap;
  return score;
}

inline uint16_t MakePoint(const std::string& s) {
  int col = s[0] < 'i' ? s[0] - 'a' : s[0] - 'a' - 1;
  int row = s[1] - '0';
  if (s.size() == 3) row = row * 10 + (s[2] - '0');
  return FromRC(row - 1, col);
}

class State : public RState {
 public:
  State(int n, float komi, int handicap)
      : board_(n), komi_(komi), handicap_(handicap) {
    Reset();
  }
  Player CurrentPlayer() const override {
    return IsTerminal() ? kTerminalPlayerId : static_cast<int>(to_play_);
  }
  std::vector<Action> LegalActions() const override {
    std::vector<Action> v;
    if (IsTerminal()) return v;
    for (uint16_t p : board_.points())
      if (board_.IsLegal(p, to_play_)) v.push_back(board_.ToAction(p));
    v.push_back(board_.pass_action());
    return v;
  }
  bool IsTerminal() const override {
    if (history_.size() < 2) return false;
    const int n = board_.size();
    return history_.size() >= static_cast<size_t>(2 * n * n) || superko_ ||
           (history_[history_.size() - 1] == board_.pass_action() &&
            history_[history_.size() - 2] == board_.pass_action());
  }
  // Tromp-Taylor score of the current board (go_board.cc:555-597).
  float Score() const { return TrompTaylorScore(board_, komi_, handicap_); }
  std::vector<double> Returns() const override {
    if (!IsTerminal()) return {0.0, 0.0};
    if (superko_) return {0.0, 0.0};
    float s = TrompTaylorScore(board_, komi_, handicap_);
    if (s > 0) return {1.0, -1.0};
    if (s < 0) return {-1.0, 1.0};
    return {0.0, 0.0};
  }
  std::unique_ptr<RState> Clone() const override {
    return std::make_unique<State>(*this);
  }
  std::string ToString() const override {
    std::ostringstream ss;
    ss << "GoState(komi=" << komi_ << ", to_play="
       << (to_play_ == kBlack ? "B" : "W")
       << ", history.size()=" << history_.size() << ")\n";
    ss << "\n";
    const int n = board_.size();
    for (int r = n - 1; r >= 0; --r) {
      ss << std::setw(2) << std::setfill(' ') << (r + 1) << " ";
      for (int c = 0; c < n; ++c) {
        Color x = board_.ColorAt(FromRC(r, c));
        ss << (x == kBlack ? 'X' : (x == kWhite ? 'O' : (x == kEmpty ? '+' : '#')));
      }
      ss << std::endl;
    }
    std::string cols = "ABCDEFGHJKLMNOPQRST";
    ss << "   " << cols.substr(0, n) << std::endl;
    return ss.str();
  }
  std::string ActionToString(Player p, Action a) const override {
    std::string s = p == 0 ? "B " : "W ";
    uint16_t vp = board_.ToVirtual(a);
    if (vp == kVirtualPass) return s + "PASS";
    int r = vp / kVB - 1, c = vp % kVB - 1;
    char col = static_cast<char>('a' + c);
    if (col >= 'i') ++col;
    return s + std::string(1, col) + std::to_string(r + 1);
  }

 protected:
  void DoApplyAction(Action a) override {
    board_.Play(board_.ToVirtual(a), to_play_);
    to_play_ = Opp(to_play_);
    bool inserted = reps_.insert(board_.Hash()).second;
    if (!inserted && a != board_.pass_action()) superko_ = true;
  }

 private:
  void Reset() {
    board_.Clear();
    to_play_ = kBlack;
    if (handicap_ >= 2) {  // go.cc:211-217 (HandicapStones is empty above 9)
      static const char* kPlace[9] = {"d4", "q16", "d16", "q4", "d10",
                                      "q10", "k4", "k16", "k10"};
      std::vector<uint16_t> pts;
      for (int i = 0; i < handicap_ && handicap_ <= 9; ++i) pts.push_back(MakePoint(kPlace[i]));
      if (handicap_ <= 9 && handicap_ >= 5 && handicap_ % 2 == 1)
        pts[handicap_ - 1] = MakePoint("k10");
      for (uint16_t p : pts) board_.Play(p, kBlack);
      to_play_ = kWhite;
    }
    reps_.clear();
    reps_.insert(board_.Hash());
    superko_ = false;
  }
  Board board_;
  float komi_;
  int handicap_;
  Color to_play_;
  bool superko_ = false;
  std::unordered_set<uint64_t> reps_;
};

class Game : public RGame {
 public:
  Game(int n, float komi, int handicap) : n_(n), komi_(komi), handicap_(handicap) {}
  std::unique_ptr<RState> NewInitialState() const override {
    return std::make_unique<State>(n_, komi_, handicap_);
  }
  int NumDistinctActions() const override { return n_ * n_ + 1; }
  int MaxGameLength() const override { return 2 * n_ * n_; }
  std::string ShortName() const override { return "go"; }

 private:
  int n_;
  float komi_;
  int handicap_;
};
}  // namespace go

float GoScore(const RState& s) {
  return dynamic_cast<const go::State&>(s).Score();
}


// ---------------------------------------------------------------------------
// pig (pig.cc:81-244): n players; a decision node offers roll (0) / stop (1)
// (only stop once the turn would reach winscore); a roll goes to a chance
// node with outcomes 1..diceoutcomes, each 1/diceoutcomes.  Outcome 1 loses
// the turn total and passes the turn; outcome k > 1 adds k + 1 to the turn
// total (pig.cc:211, as written).  Stop banks the turn total and passes.
// Terminal at total_moves >= horizon or any score >= winscore; the winner gets
// 1, the others -1 / (n - 1); nobody: all 0.
namespace pig {
class State : public RState {
 public:
  State(int players, int dice, int horizon, int win)
      : n_(players), dice_(dice), horizon_(horizon), win_(win), scores_(players, 0) {}
  Player CurrentPlayer() const override { return IsTerminal() ? kTerminalPlayerId : cur_; }
  bool IsTerminal() const override {
    if (moves_ >= horizon_) return true;
    for (int p = 0; p < n_; ++p)
      if (scores_[p] >= win_) return true;
    return false;
  }
  std::vector<Action> LegalActions() const override {
    if (IsTerminal()) return {};
    if (cur_ == kChancePlayerId) {
      std::vector<Action> v;
      for (int i = 0; i < dice_; ++i) v.push_back(i + 1);
      return v;
    }
    if (scores_[cur_] + turn_total_ >= win_) return {1};
    return {0, 1};
  }
  std::vector<std::pair<Action, double>> ChanceOutcomes() const override {
    std::vector<std::pair<Action, double>> o;
    for (int i = 0; i < dice_; ++i) o.emplace_back(i + 1, 1.0 / dice_);
    return o;
  }
  std::vector<double> Returns() const override {
    if (!IsTerminal()) return std::vector<double>(n_, 0.0);
    std::vector<double> r(n_, -1.0 / (n_ - 1));
    for (int p = 0; p < n_; ++p)
      if (scores_[p] >= win_) {
        r[p] = 1.0;
        return r;
      }
    return std::vector<double>(n_, 0.0);
  }
  std::unique_ptr<RState> Clone() const override { return std::make_unique<State>(*this); }
  std::string ToString() const override {
    std::string s = "Scores:";
    for (int p = 0; p < n_; ++p) s += " " + std::to_string(scores_[p]);
    s += ", Turn total: " + std::to_string(turn_total_) + "\nCurrent player: " +
         std::to_string(turn_player_) + (cur_ == kChancePlayerId ? " (rolling)\n" : "\n");
    return s;
  }
  std::string ActionToString(Player p, Action a) const override {
    if (p == kChancePlayerId) return "chance outcome " + std::to_string(a);
    return a == 0 ? "roll" : "stop";
  }

 protected:
  void DoApplyAction(Action a) override {
    if (cur_ >= 0 && a == 0) {
      cur_ = kChancePlayerId;
      ++moves_;
    } else if (cur_ >= 0 && a == 1) {
      scores_[turn_player_] += turn_total_;
      turn_total_ = 0;
      turn_player_ = (turn_player_ + 1) % n_;
      cur_ = turn_player_;
      ++moves_;
    } else if (cur_ == kChancePlayerId) {
      if (a == 1) {
        turn_total_ = 0;
        turn_player_ = (turn_player_ + 1) % n_;
        cur_ = turn_player_;
      } else {
        turn_total_ += static_cast<int>(a) + 1;
        cur_ = turn_player_;
      }
    }
  }

 private:
  int n_, dice_, horizon_, win_;
  int moves_ = 0;
  Player cur_ = 0;
  int turn_player_ = 0;
  std::vector<int> scores_;
  int turn_total_ = 0;
};

class Game : public RGame {
 public:
  Game(int players, int dice, int horizon, int win)
      : n_(players), dice_(dice), horizon_(horizon), win_(win) {}
  std::unique_ptr<RState> NewInitialState() const override {
    return std::make_unique<State>(n_, dice_, horizon_, win_);
  }
  int NumDistinctActions() const override { return 6; }  // pig.h:83
  int MaxGameLength() const override { return horizon_; }
  std::string ShortName() const override { return "pig"; }
  int NumPlayers() const override { return n_; }

 private:
  int n_, dice_, horizon_, win_;
};
}  // namespace pig

std::unique_ptr<RGame> LoadGame(const std::string& gs, std::string* err) {
  std::string name;
  GameParams p;
  if (!ParseGameString(gs, &name, &p)) {
    *err = "cannot parse game string: " + gs;
    return nullptr;
  }
  if (name == "tic_tac_toe") return std::make_unique<ttt::Game>();
  if (name == "connect_four") return std::make_unique<c4::Game>();
  if (name == "breakthrough") {
    int rows = p.GetInt("rows", 8), cols = p.GetInt("columns", 8);
    if (rows < 2 || cols < 2 || rows > 26 || cols > 26) {
      *err = "bad breakthrough size";
      return nullptr;
    }
    return std::make_unique<bt::Game>(rows, cols);
  }
  if (name == "hex") {
    int n = p.GetInt("board_size", 11);
    if (n < 1 || n > 26) {
      *err = "bad hex size";
      return nullptr;
    }
    return std::make_unique<hex::Game>(n);
  }
  if (name == "go") {
    int n = p.GetInt("board_size", 19);
    if (n < 2 || n > 19) {
      *err = "go board_size must be in [2, 19]";
      return nullptr;
    }
    return std::make_unique<go::Game>(n, static_cast<float>(p.GetDouble("komi", 7.5)),
                                      p.GetInt("handicap", 0));
  }
  if (name == "pig") {
    const int players = p.GetInt("players", 2), dice = p.GetInt("diceoutcomes", 6);
    const int horizon = p.GetInt("horizon", 1000), win = p.GetInt("winscore", 100);
    if (players < 2 || players > 10 || dice < 1 || horizon < 1 || win < 1) {
      *err = "bad pig parameters";
      return nullptr;
    }
    return std::make_unique<pig::Game>(players, dice, horizon, win);
  }
  *err = "unknown game: " + name;
  return nullptr;
}

}  // namespace oref
