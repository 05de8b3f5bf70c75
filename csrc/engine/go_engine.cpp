// Go rules engine + tactical feature extractor.  See go_engine.h for the semantics
// contract (bit-exact with the reference's makedata.lua on the bundled fixture).
#include "go_engine.h"

#include <algorithm>
#include <cstring>

namespace dg {

int g_nbr[NN][4];
int g_nnbr[NN];

namespace {
struct NbrInit {
  NbrInit() {
    // reference order: directions = {{-1,0},{1,0},{0,-1},{0,1}} (makedata.lua:199)
    const int d[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};
    for (int x = 0; x < N; ++x)
      for (int y = 0; y < N; ++y) {
        const int i = x * N + y;
        g_nnbr[i] = 0;
        for (auto& dd : d) {
          const int a = x + dd[0], b = y + dd[1];
          if (a >= 0 && a < N && b >= 0 && b < N) g_nbr[i][g_nnbr[i]++] = a * N + b;
        }
      }
  }
} g_nbr_init;

constexpr long long kLadderNodeCap = 50000000;  // never reached on real games
}  // namespace

Board::Board() { clear(); }

void Board::clear() {
  s_.fill(0);
  age_.fill(0);
  mark_.fill(0);
  lmark_.fill(0);
  stamp_ = 0;
  ko_ = -1;
}

void Board::set_stones(const uint8_t* stones) {
  std::memcpy(s_.data(), stones, NN);
  ko_ = -1;
}

int Board::liberties(int idx, std::vector<int>* group, std::vector<int>* libs) {
  const uint8_t p = s_[idx];
  if (group) group->clear();
  if (libs) libs->clear();
  if (p == 0) return 0;
  if (++stamp_ == 0) {  // wrap: reset marks
    mark_.fill(0);
    lmark_.fill(0);
    stamp_ = 1;
  }
  const uint32_t st = stamp_;
  int nlib = 0;
  stack_.clear();
  stack_.push_back(idx);
  mark_[idx] = st;
  while (!stack_.empty()) {
    const int h = stack_.back();
    stack_.pop_back();
    if (group) group->push_back(h);
    for (int k = 0; k < g_nnbr[h]; ++k) {
      const int n = g_nbr[h][k];
      const uint8_t v = s_[n];
      if (v == p) {
        if (mark_[n] != st) {
          mark_[n] = st;
          stack_.push_back(n);
        }
      } else if (v == 0 && lmark_[n] != st) {
        lmark_[n] = st;
        ++nlib;
        if (libs) libs->push_back(n);
      }
    }
  }
  return nlib;
}

void Board::put(int idx, uint8_t v, std::vector<Undo>* log) {
  if (log) log->push_back({idx, s_[idx]});
  s_[idx] = v;
}

void Board::unwind(std::vector<Undo>& log, size_t to) {
  while (log.size() > to) {
    const Undo u = log.back();
    log.pop_back();
    s_[u.idx] = u.prev;
  }
}

void Board::place_and_resolve(int idx, int player, std::vector<Undo>* log, int* removed_opp,
                              std::vector<int>* cleared) {
  put(idx, (uint8_t)player, log);
  std::vector<int> grp;
  auto apply_if_dead = [&](int i) {
    if (s_[i] == 0) return;
    if (liberties(i, &grp, nullptr) != 0) return;
    for (int g : grp) {
      if (s_[g] == 3 - player && removed_opp) ++*removed_opp;
      put(g, 0, log);
      if (cleared) cleared->push_back(g);
    }
  };
  const int opp = 3 - s_[idx];
  for (int k = 0; k < g_nnbr[idx]; ++k) {
    const int n = g_nbr[idx][k];
    if (s_[n] == opp) apply_if_dead(n);
  }
  apply_if_dead(idx);
}

void Board::play(const Move& m) {
  const int idx = m.x * N + m.y;
  if (m.x < 0 || m.x >= N || m.y < 0 || m.y >= N) throw IllegalMove("move off board");
  if (s_[idx] != 0) throw IllegalMove("playing somewhere that's already been played!");
  for (int i = 0; i < NN; ++i)
    if (age_[i] > 0 && age_[i] < 255) ++age_[i];
  std::vector<int> cleared;
  int captured = 0;
  place_and_resolve(idx, m.player, nullptr, &captured, &cleared);
  age_[idx] = 1;
  for (int c : cleared) age_[c] = 1;
  // simple ko: one stone captured by a lone stone now in atari (its one liberty is the
  // captured point, which the opponent may not retake at once)
  ko_ = -1;
  if (captured == 1 && s_[idx] == m.player) {
    std::vector<int> grp, lbs;
    if (liberties(idx, &grp, &lbs) == 1 && grp.size() == 1) ko_ = lbs[0];
  }
}

void Board::kills_and_liberties(int idx, int player, int* kills, int* libs_after) {
  std::vector<Undo> log;
  int k = 0;
  place_and_resolve(idx, player, &log, &k, nullptr);
  *libs_after = liberties(idx);
  *kills = k;
  unwind(log, 0);
}

bool Board::ladder_moves(int gx, const int libs2[2], std::vector<int>* result, int depth) {
  const int player = s_[gx];
  const int opp = 3 - player;
  std::vector<Undo> log;
  std::vector<int> newlibs;
  for (int i = 0; i < 2; ++i) {
    if (++ladder_nodes_ > kLadderNodeCap) return false;
    const int a = libs2[i], o = libs2[1 - i];
    place_and_resolve(a, opp, &log, nullptr, nullptr);
    const int n = liberties(a);
    if (n > 2) {
      place_and_resolve(o, player, &log, nullptr, nullptr);
      const int n2 = liberties(o, nullptr, &newlibs);
      if (n2 == 1) {
        result->push_back(a);
      } else if (n2 == 2) {
        const int n3 = liberties(a);
        if (n3 > 1) {
          const int nl[2] = {newlibs[0], newlibs[1]};
          std::vector<int> sub;
          ladder_moves(gx, nl, &sub, depth + 1);
          if (!sub.empty()) result->push_back(a);
        }
      }
    }
    unwind(log, 0);
  }
  return true;
}

void Board::summarize(uint8_t* out, bool mark_ko) {
  uint8_t* st = out + P_STONES * NN;
  uint8_t* lib = out + P_LIBS * NN;
  uint8_t* age = out + P_AGE * NN;
  std::memset(out, 0, NUM_STORED * NN);
  std::memcpy(st, s_.data(), NN);
  std::memcpy(age, age_.data(), NN);
  // liberties_after / kills for both players (all_kills_and_liberties_after :122-141)
  for (int k = 1; k <= 2; ++k) {
    uint8_t* la = out + (P_LIBS_AFTER_B + k - 1) * NN;
    uint8_t* kl = out + (P_KILLS_B + k - 1) * NN;
    for (int i = 0; i < NN; ++i) {
      if (s_[i] != 0) continue;
      int kills = 0, libs = 0;
      kills_and_liberties(i, k, &kills, &libs);
      la[i] = (uint8_t)libs;
      kl[i] = (uint8_t)kills;
    }
  }
  // group liberties + ladders (all_ladder_moves_and_liberties :441-479)
  ladder_nodes_ = 0;
  std::array<uint8_t, NN> considered{};
  std::vector<int> grp, lbs, moves;
  for (int i = 0; i < NN; ++i) {
    if (s_[i] == 0 || considered[i]) continue;
    const int n = liberties(i, &grp, &lbs);
    const std::vector<int> members = grp;
    for (int g : members) {
      considered[g] = 1;
      lib[g] = (uint8_t)n;
    }
    if (n == 2) {
      const int l2[2] = {lbs[0], lbs[1]};
      moves.clear();
      ladder_moves(i, l2, &moves, 0);
      uint8_t* lad = out + (P_LADDER_B + (3 - s_[i]) - 1) * NN;
      for (int mv : moves) lad[mv] = (uint8_t)members.size();
    }
  }
  if (mark_ko && ko_ >= 0) lib[ko_] = KO_MARK;
}

int game_positions(const std::vector<Move>& handicap, const std::vector<Move>& moves,
                   uint8_t* out, bool mark_ko) {
  Board b;
  for (const Move& h : handicap) b.play(h);
  int k = 0;
  for (const Move& m : moves) {
    b.summarize(out + (size_t)k * NUM_STORED * NN, mark_ko);
    b.play(m);
    ++k;
  }
  return k;
}

}  // namespace dg
