// Multi-threaded prefetching batch loader (the reference's 32-thread `threads` pool,
// data.lua:11-27 + dataloader.lua:113-125), rebuilt as a C++ producer/consumer ring.
//
//  * Sources: (a) the reference's on-disk layout — one t7 file per position under
//    <game dir>/<k> — or (b) a packed in-memory dataset (planes [N][9][361] + per-position
//    player / rank / label, grouped into games).
//  * Sampling: "game" = pick a game uniformly, then a move uniformly (data.lua:29-37, the
//    reference's non-uniform-over-positions scheme) or "position" = uniform over positions.
//  * Determinism: batch k is drawn from an RNG seeded by (seed, k) and batches are handed
//    out strictly in order k = 0, 1, 2, ... — the result is independent of thread timing.
//  * Output per batch: uint8 planes [B][9][361] (3.2 KB/board — the GPU expands them),
//    uint8 player, uint8 rank-of-player-to-move, int32 label = 19*(x-1) + (y-1), written into
//    caller-provided (pinned) ring slots.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dg {

struct GameRef {
  std::string dir;     // file source: directory holding files 1..count
  int64_t start = 0;   // packed source: first position index
  int count = 0;
};

struct SlotBuffers {
  uint8_t* planes;   // [B][9*361]
  uint8_t* player;   // [B]
  uint8_t* rank;     // [B]
  int32_t* label;    // [B]
};

class Loader {
 public:
  // Packed source arrays must outlive the loader (the Python wrapper keeps them alive).
  Loader(std::vector<GameRef> games, int batch, int threads, std::vector<SlotBuffers> slots,
         uint64_t seed, bool position_uniform, const uint8_t* packed_planes,
         const uint8_t* packed_player, const uint8_t* packed_rank, const int32_t* packed_label,
         int64_t start_seq = 0);
  ~Loader();
  Loader(const Loader&) = delete;

  // Blocks until batch `seq` is ready; returns its slot index (seq % nslots).
  int next(int64_t* seq_out);
  // The consumer is done with this slot (its H2D copy finished): it may be refilled.
  void release(int slot);
  void stop();
  int64_t errors() const { return errors_.load(); }
  std::string last_error();

  // Draw the (game, move) sample list of batch k (exposed for tests of the sampler).
  std::vector<std::pair<int, int>> sample_batch(int64_t k) const;

 private:
  void worker();
  void fill(int slot, int64_t k);

  std::vector<GameRef> games_;
  std::vector<int64_t> cum_;  // prefix sums of counts (position-uniform sampling)
  int batch_;
  std::vector<SlotBuffers> slots_;
  uint64_t seed_;
  bool position_uniform_;
  const uint8_t* pk_planes_;
  const uint8_t* pk_player_;
  const uint8_t* pk_rank_;
  const int32_t* pk_label_;

  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<int64_t> slot_seq_;     // batch currently held by a slot (-1 = free)
  std::vector<int> slot_state_;       // 0 free, 1 filling, 2 ready, 3 consumed (held)
  int64_t produce_next_ = 0;          // next batch number to claim
  int64_t consume_next_ = 0;          // next batch number to hand out
  bool stop_ = false;
  std::vector<std::thread> threads_;
  std::atomic<int64_t> errors_{0};
  std::string last_error_;
};

// Positions of random self-play games (rule-consistent synthetic data): the engine plays
// uniformly random moves that are legal and not suicide and do not fill a single-point eye
// of the mover.  Returns n positions (planes [n][9][361], player, rank, label).
void random_positions(int n, uint64_t seed, int max_moves, std::vector<uint8_t>* planes,
                      std::vector<uint8_t>* player, std::vector<uint8_t>* rank,
                      std::vector<int32_t>* label);

}  // namespace dg
