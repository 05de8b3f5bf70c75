// 9 stored planes -> 37 (or 38 with the optional ko plane) network planes on the CPU (the reference's preprocess(),
// dataloader.lua:50-92).  Used by the CPU training path and the data tools; the GPU path
// ships the 9 uint8 planes and expands them with expand_features_kernel.
#include "features.h"

#include <cstring>

#include "go_engine.h"

namespace dg {

void expand_position(const uint8_t* pl, int player, int rank, float* out, int nplanes) {
  constexpr int NP = 361;
  std::memset(out, 0, sizeof(float) * nplanes * NP);
  const int pi = player, op = 3 - player;
  const uint8_t* st = pl;
  const uint8_t* lib = pl + NP;
  const uint8_t* la = pl + (pi == 1 ? 2 : 3) * NP;
  const uint8_t* kill = pl + (pi == 1 ? 4 : 5) * NP;
  const uint8_t* age = pl + 6 * NP;
  const uint8_t* lad = pl + (pi == 1 ? 7 : 8) * NP;
  for (int p = 0; p < NP; ++p) {
    auto set = [&](int c, bool v) { out[c * NP + p] = v ? 1.f : 0.f; };
    set(0, st[p] == 0);
    set(1, st[p] == pi);
    set(2, st[p] == op);
    // group liberties of a stone (an empty point's liberty entry is 0, or the ko mark)
    const int gl = st[p] != 0 ? lib[p] : 0;
    for (int i = 1; i <= 3; ++i) set(2 + i, gl == i);
    set(6, gl >= 4);
    set(7, st[p] == 0 && la[p] == 0);
    for (int i = 1; i <= 5; ++i) set(7 + i, la[p] == i);
    set(13, la[p] >= 6);
    for (int i = 1; i <= 6; ++i) set(13 + i, kill[p] == i);
    set(20, kill[p] >= 7);
    for (int i = 1; i <= 5; ++i) set(20 + i, age[p] == i);
    set(26, lad[p] >= 1);
    // plane 27 stays zero (the reference's RANK + rank off-by-one)
    if (rank >= 1 && rank <= 9) set(27 + rank, true);
    if (nplanes > kNetPlanes) set(37, st[p] == 0 && lib[p] == KO_MARK);
  }
}

}  // namespace dg
