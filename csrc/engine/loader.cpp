#include "loader.h"

#include <algorithm>
#include <cstring>

#include "go_engine.h"
#include "t7.h"

namespace dg {

namespace {
inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
}  // namespace

Loader::Loader(std::vector<GameRef> games, int batch, int threads, std::vector<SlotBuffers> slots,
               uint64_t seed, bool position_uniform, const uint8_t* packed_planes,
               const uint8_t* packed_player, const uint8_t* packed_rank,
               const int32_t* packed_label, int64_t start_seq)
    : games_(std::move(games)),
      batch_(batch),
      slots_(std::move(slots)),
      seed_(seed),
      position_uniform_(position_uniform),
      pk_planes_(packed_planes),
      pk_player_(packed_player),
      pk_rank_(packed_rank),
      pk_label_(packed_label) {
  // drop games with no positions (data.lua:73-76)
  games_.erase(std::remove_if(games_.begin(), games_.end(),
                              [](const GameRef& g) { return g.count <= 0; }),
               games_.end());
  if (games_.empty()) throw std::runtime_error("loader: no non-empty games");
  if (slots_.empty()) throw std::runtime_error("loader: no slots");
  cum_.resize(games_.size() + 1, 0);
  for (size_t i = 0; i < games_.size(); ++i) cum_[i + 1] = cum_[i] + games_[i].count;
  slot_seq_.assign(slots_.size(), -1);
  slot_state_.assign(slots_.size(), 0);
  // resume: batch numbers continue from start_seq (slot = seq % nslots)
  produce_next_ = consume_next_ = start_seq;
  threads = std::max(1, threads);
  for (int t = 0; t < threads; ++t) threads_.emplace_back([this] { worker(); });
}

Loader::~Loader() { stop(); }

void Loader::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ && threads_.empty()) return;
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

std::string Loader::last_error() {
  std::lock_guard<std::mutex> lk(mu_);
  return last_error_;
}

std::vector<std::pair<int, int>> Loader::sample_batch(int64_t k) const {
  std::vector<std::pair<int, int>> out(batch_);
  const uint64_t base = splitmix64(seed_ ^ splitmix64((uint64_t)k + 0x1234567ull));
  for (int i = 0; i < batch_; ++i) {
    const uint64_t r = splitmix64(base + (uint64_t)i * 0x9E3779B97F4A7C15ull);
    const uint64_t r2 = splitmix64(r);
    if (position_uniform_) {
      const int64_t pos = (int64_t)(r % (uint64_t)cum_.back());
      const int g = (int)(std::upper_bound(cum_.begin(), cum_.end(), pos) - cum_.begin()) - 1;
      out[i] = {g, (int)(pos - cum_[g]) + 1};
    } else {
      const int g = (int)(r % games_.size());
      out[i] = {g, 1 + (int)(r2 % (uint64_t)games_[g].count)};
    }
  }
  return out;
}

void Loader::fill(int slot, int64_t k) {
  const SlotBuffers& sb = slots_[slot];
  const auto samples = sample_batch(k);
  constexpr int PB = 9 * 361;
  for (int i = 0; i < batch_; ++i) {
    const GameRef& g = games_[samples[i].first];
    const int move = samples[i].second;
    if (pk_planes_) {
      const int64_t idx = g.start + move - 1;
      std::memcpy(sb.planes + (size_t)i * PB, pk_planes_ + (size_t)idx * PB, PB);
      sb.player[i] = pk_player_[idx];
      sb.rank[i] = pk_rank_[idx];
      sb.label[i] = pk_label_[idx];
      continue;
    }
    t7::Position pos;
    std::string err;
    if (t7::read_position_file(g.dir + "/" + std::to_string(move), &pos, &err)) {
      std::memcpy(sb.planes + (size_t)i * PB, pos.planes, PB);
      sb.player[i] = (uint8_t)pos.player;
      const int rk = pos.player == 1 ? pos.rank_black : pos.rank_white;
      sb.rank[i] = (uint8_t)std::max(0, std::min(255, rk));
      sb.label[i] = 19 * (pos.x - 1) + (pos.y - 1);
    } else {
      errors_.fetch_add(1);
      {
        std::lock_guard<std::mutex> lk(mu_);
        last_error_ = g.dir + "/" + std::to_string(move) + ": " + err;
      }
      std::memset(sb.planes + (size_t)i * PB, 0, PB);
      sb.player[i] = 1;
      sb.rank[i] = 0;
      sb.label[i] = -1;  // marks a bad sample (ignored by nothing: caller checks errors())
    }
  }
}

void Loader::worker() {
  const int P = (int)slots_.size();
  while (true) {
    int slot;
    int64_t k;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || slot_state_[produce_next_ % P] == 0; });
      if (stop_) return;
      k = produce_next_++;
      slot = (int)(k % P);
      slot_state_[slot] = 1;
      slot_seq_[slot] = k;
    }
    fill(slot, k);
    {
      std::lock_guard<std::mutex> lk(mu_);
      slot_state_[slot] = 2;
    }
    cv_.notify_all();
  }
}

int Loader::next(int64_t* seq_out) {
  const int P = (int)slots_.size();
  std::unique_lock<std::mutex> lk(mu_);
  const int slot = (int)(consume_next_ % P);
  cv_.wait(lk, [&] {
    return stop_ || (slot_state_[slot] == 2 && slot_seq_[slot] == consume_next_);
  });
  if (stop_) return -1;
  slot_state_[slot] = 3;
  if (seq_out) *seq_out = consume_next_;
  ++consume_next_;
  return slot;
}

void Loader::release(int slot) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (slot < 0 || slot >= (int)slots_.size() || slot_state_[slot] != 3) return;
    slot_state_[slot] = 0;
    slot_seq_[slot] = -1;
  }
  cv_.notify_all();
}

void random_positions(int n, uint64_t seed, int max_moves, std::vector<uint8_t>* planes,
                      std::vector<uint8_t>* player, std::vector<uint8_t>* rank,
                      std::vector<int32_t>* label) {
  constexpr int PB = 9 * 361;
  planes->resize((size_t)n * PB);
  player->resize(n);
  rank->resize(n);
  label->resize(n);
  uint64_t st = splitmix64(seed + 77);
  auto rnd = [&]() { return st = splitmix64(st); };
  int made = 0;
  while (made < n) {
    Board b;
    const int ranks[3] = {0, 1 + (int)(rnd() % 9), 1 + (int)(rnd() % 9)};
    int to_move = 1;
    for (int mv = 0; mv < max_moves && made < n; ++mv) {
      // candidate empty points in random order
      int order[NN];
      int cnt = 0;
      for (int i = 0; i < NN; ++i)
        if (b.at(i) == 0) order[cnt++] = i;
      for (int i = cnt - 1; i > 0; --i) std::swap(order[i], order[rnd() % (i + 1)]);
      int chosen = -1;
      for (int c = 0; c < cnt; ++c) {
        const int idx = order[c];
        // skip single-point own eyes
        bool eye = true;
        for (int k = 0; k < g_nnbr[idx]; ++k)
          if (b.at(g_nbr[idx][k]) != to_move) eye = false;
        if (eye) continue;
        int kills, libs;
        b.kills_and_liberties(idx, to_move, &kills, &libs);
        if (libs == 0) continue;  // suicide
        chosen = idx;
        break;
      }
      if (chosen < 0) break;  // no sensible move: game over
      b.summarize(planes->data() + (size_t)made * PB);
      (*player)[made] = (uint8_t)to_move;
      (*rank)[made] = (uint8_t)ranks[to_move];
      (*label)[made] = chosen;
      ++made;
      b.play({to_move, chosen / N, chosen % N});
      to_move = 3 - to_move;
    }
  }
}

}  // namespace dg
