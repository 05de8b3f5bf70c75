// Sanitizer stress driver for the CPU runtime: the loader's producer /
// consumer ring under many threads and the Go engine from several threads at once.
// Built and run by tools/sanitize.sh with -fsanitize=thread and -fsanitize=address,undefined
// (CPU only — GPU sanitizers are not available on the MI355X pool).
//
// Checks, beyond "no sanitizer report":
//   * determinism: the batch stream is identical for 1, 3 and 8 worker threads (and for a
//     restart at start_seq), independent of thread timing;
//   * the engine's per-position features are identical when computed concurrently.
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../loader.h"

using namespace dg;

static uint64_t fnv(const uint8_t* p, size_t n, uint64_t h) {
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

struct Packed {
  std::vector<uint8_t> planes, player, rank;
  std::vector<int32_t> label;
  std::vector<GameRef> games;
};

static Packed make_packed(int n) {
  Packed d;
  random_positions(n, 42, 120, &d.planes, &d.player, &d.rank, &d.label);
  int64_t start = 0;
  int g = 0;
  while (start < n) {  // games of 5..40 positions
    const int c = std::min<int64_t>(5 + (g * 7) % 36, n - start);
    GameRef r;
    r.start = start;
    r.count = c;
    d.games.push_back(r);
    start += c;
    ++g;
  }
  return d;
}

static uint64_t run_loader(const Packed& d, int threads, int nbatches, int64_t start_seq,
                           bool position_uniform) {
  const int B = 32, nslots = 4;
  std::vector<std::vector<uint8_t>> pl(nslots, std::vector<uint8_t>(B * 9 * 361));
  std::vector<std::vector<uint8_t>> py(nslots, std::vector<uint8_t>(B)), rk(nslots,
                                                                         std::vector<uint8_t>(B));
  std::vector<std::vector<int32_t>> lb(nslots, std::vector<int32_t>(B));
  std::vector<SlotBuffers> slots;
  for (int i = 0; i < nslots; ++i) slots.push_back({pl[i].data(), py[i].data(), rk[i].data(), lb[i].data()});
  Loader L(d.games, B, threads, slots, 7, position_uniform, d.planes.data(), d.player.data(),
           d.rank.data(), d.label.data(), start_seq);
  uint64_t h = 1469598103934665603ull;
  for (int k = 0; k < nbatches; ++k) {
    int64_t seq = -1;
    const int s = L.next(&seq);
    if (seq != start_seq + k) {
      std::fprintf(stderr, "out-of-order batch %lld (want %lld)\n", (long long)seq,
                   (long long)(start_seq + k));
      std::exit(2);
    }
    h = fnv(pl[s].data(), pl[s].size(), h);
    h = fnv((const uint8_t*)lb[s].data(), lb[s].size() * 4, h);
    L.release(s);
  }
  L.stop();
  if (L.errors()) {
    std::fprintf(stderr, "loader errors: %s\n", L.last_error().c_str());
    std::exit(3);
  }
  return h;
}

int main() {
  const Packed d = make_packed(3000);
  for (bool pu : {false, true}) {
    const uint64_t h1 = run_loader(d, 1, 200, 0, pu);
    const uint64_t h3 = run_loader(d, 3, 200, 0, pu);
    const uint64_t h8 = run_loader(d, 8, 200, 0, pu);
    if (h1 != h3 || h1 != h8) {
      std::fprintf(stderr, "loader not deterministic across thread counts\n");
      return 4;
    }
    // resume: batches 100.. from a fresh loader equal the tail of a full run
    const uint64_t tail_a = run_loader(d, 8, 50, 150, pu);
    const uint64_t tail_b = run_loader(d, 2, 50, 150, pu);
    if (tail_a != tail_b) {
      std::fprintf(stderr, "start_seq resume not deterministic\n");
      return 5;
    }
  }
  // engine from several threads: random games, features must match a serial run
  const int T = 6;
  std::vector<uint64_t> par(T), ser(T);
  auto job = [](int t) {
    std::vector<uint8_t> pl, py, rk;
    std::vector<int32_t> lb;
    random_positions(300, 1000 + t, 200, &pl, &py, &rk, &lb);
    return fnv(pl.data(), pl.size(), 1469598103934665603ull);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back([&, t] { par[t] = job(t); });
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t) ser[t] = job(t);
  for (int t = 0; t < T; ++t)
    if (par[t] != ser[t]) {
      std::fprintf(stderr, "engine results differ under concurrency\n");
      return 6;
    }
  std::printf("stress ok\n");
  return 0;
}
