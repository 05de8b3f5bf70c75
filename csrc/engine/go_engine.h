// Go rules engine + tactical feature extractor (CPU, C++17).
//
// Semantics follow the reference's Lua engine exactly (makedata.lua), so the stored
// planes it produces match the bundled fixture bit for bit:
//   * trial play (play_with_f, makedata.lua:388-391 / apply_f_to_dead_neighbors :234-241):
//     place the stone, clear every adjacent opponent group left with 0 liberties (in the
//     neighbour order up, down, left, right), then clear the player's own group if it has
//     0 liberties (suicide is legal and removes own stones).  Ko is not enforced.
//   * simple ko (an addition, off by default): a move that captures exactly one stone with
//     a lone stone left in atari makes the captured point the ko point — the opponent may
//     not retake there on the next move.  summarize(out, true) marks it in the stored
//     liberty plane as KO_MARK at that EMPTY point (the plane is 0 at every empty point
//     otherwise, so 9-plane files keep their shape and a reader that gates the liberty
//     planes on a stone — every expander here does — sees the reference's 37 planes).
//   * liberties_after / kills (count_kills_and_liberties :304-327)
//   * group liberties (all_ladder_moves_and_liberties :441-479)
//   * ladders (ladder_moves :393-439, recursive) — group size written for the attacker,
//     later groups in row-major scan order overwrite earlier ones
//   * age (update_board :329-354): +1 on every point with 0 < age < 255, then 1 on the
//     played point and every cleared point.
// The board is a flat array indexed x*19 + y (x = first SGF coordinate, 0-based), i.e.
// the reference's hash(x, y) (:188-196).  Flood fills use a stamp-marked visited array
// instead of Lua hash tables.
#pragma once
#include <array>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace dg {

constexpr int N = 19;
constexpr int NN = N * N;

struct Move {
  int player;  // 1 black, 2 white
  int x, y;    // 0-based
};

// Stored planes of one position, layout [plane][x][y] (dataloader.lua:20-27).
enum Plane : int {
  P_STONES = 0, P_LIBS = 1, P_LIBS_AFTER_B = 2, P_LIBS_AFTER_W = 3, P_KILLS_B = 4,
  P_KILLS_W = 5, P_AGE = 6, P_LADDER_B = 7, P_LADDER_W = 8, NUM_STORED = 9
};

// liberty-plane value at the simple-ko point (summarize(out, mark_ko=true))
constexpr uint8_t KO_MARK = 255;

class IllegalMove : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Board {
 public:
  Board();
  void clear();
  uint8_t at(int idx) const { return s_[idx]; }
  const std::array<uint8_t, NN>& stones() const { return s_; }
  const std::array<uint8_t, NN>& ages() const { return age_; }
  void set_stones(const uint8_t* stones);  // 361 values in {0,1,2}; ages untouched, no ko
  // simple-ko point left by the last play() (-1: none)
  int ko() const { return ko_; }

  // Real move with captures and ageing (update_board).  Throws IllegalMove on an
  // occupied point.
  void play(const Move& m);

  // Liberty count of the group at idx (0 for an empty point) and optionally the group
  // members / liberty points.
  int liberties(int idx, std::vector<int>* group = nullptr, std::vector<int>* libs = nullptr);

  // Trial play of `player` at empty idx: returns (kills, liberties of the played stone's
  // group afterwards), board restored on return.
  void kills_and_liberties(int idx, int player, int* kills, int* libs_after);

  // Compute the 9 stored planes for the current position into out[9*361]
  // (age plane = current ages; mark_ko: KO_MARK in the liberty plane at the ko point).
  void summarize(uint8_t* out, bool mark_ko = false);

  // Number of ladder-search nodes visited by the last summarize() (diagnostics).
  long long ladder_nodes() const { return ladder_nodes_; }

 private:
  struct Undo {
    int idx;
    uint8_t prev;
  };
  void put(int idx, uint8_t v, std::vector<Undo>* log);
  // play_with_f: place + resolve captures; `removed_opp` counts cleared opponent stones.
  void place_and_resolve(int idx, int player, std::vector<Undo>* log, int* removed_opp,
                         std::vector<int>* cleared);
  void unwind(std::vector<Undo>& log, size_t to);
  bool ladder_moves(int gx, const int libs2[2], std::vector<int>* result, int depth);

  std::array<uint8_t, NN> s_{};
  std::array<uint8_t, NN> age_{};
  // flood-fill scratch
  std::array<uint32_t, NN> mark_{};
  std::array<uint32_t, NN> lmark_{};
  uint32_t stamp_ = 0;
  std::vector<int> stack_;
  long long ladder_nodes_ = 0;
  int ko_ = -1;
};

// Plays a whole game: optional handicap stones, then the moves; for each move emits the
// stored planes of the position BEFORE it (all_boards, makedata.lua:156-186).
// out: [num_moves][9][361]; returns number of positions written.  Throws IllegalMove.
// mark_ko: each position's simple-ko point marked (Board::summarize).
int game_positions(const std::vector<Move>& handicap, const std::vector<Move>& moves,
                   uint8_t* out, bool mark_ko = false);

// Neighbour table in the reference's order: (-1,0), (1,0), (0,-1), (0,1).
extern int g_nbr[NN][4];
extern int g_nnbr[NN];

}  // namespace dg
