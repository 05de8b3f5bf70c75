// Per-point feature expansion shared by the expansion kernel (elementwise.hip) and the forward
// stack's fused first-layer prologue (conv_stack2.hip): 9 stored uint8 planes of one board
// point -> the 37 network planes, plus v[37] = the optional simple-ko plane (v[38..] stay 0).
// Reference: preprocess() (dataloader.lua:50-92).  pl points at plane 0 of the point (planes
// are NPTS apart), pi = player to move (1 black / 2 white), rk = its rank (1..9).
// The ko point rides in the stored liberty plane as KO_MARK at an empty point
// (csrc/engine/go_engine.h), so the liberty planes are gated on a stone (a no-op for files
// without the mark).  v[37] is always written: a 37-plane model's first layer has zero
// weights on padded input channel 37, so the mark only reaches models built with the ko
// plane (ExperimentConfig.ko_plane).
#pragma once
#include "dg_common.h"

namespace dg {

template <int N>
DG_DEV void expand_point(const uint8_t* pl, int pi, int rk, float (&v)[N]) {
  static_assert(N >= 38, "37 planes + ko");
  constexpr int KO_MARK = 255;
  const int op = 3 - pi;
  const int stone = pl[0 * NPTS];
  const int lib_raw = pl[1 * NPTS];
  const int lib = stone != 0 ? lib_raw : 0;
  const int la = pl[(pi == 1 ? 2 : 3) * NPTS];
  const int kill = pl[(pi == 1 ? 4 : 5) * NPTS];
  const int age = pl[6 * NPTS];
  const int lad = pl[(pi == 1 ? 7 : 8) * NPTS];
#pragma unroll
  for (int c = 0; c < N; ++c) v[c] = 0.f;
  v[0] = stone == 0;
  v[1] = stone == pi;
  v[2] = stone == op;
#pragma unroll
  for (int i = 1; i <= 3; ++i) v[2 + i] = lib == i;
  v[6] = lib >= 4;
  v[7] = (stone == 0) && (la == 0);
#pragma unroll
  for (int i = 1; i <= 5; ++i) v[7 + i] = la == i;
  v[13] = la >= 6;
#pragma unroll
  for (int i = 1; i <= 6; ++i) v[13 + i] = kill == i;
  v[20] = kill >= 7;
#pragma unroll
  for (int i = 1; i <= 5; ++i) v[20 + i] = age == i;
  v[26] = lad >= 1;
  // v[27] stays 0: the reference's dead plane 28 (RANK + rank, rank in 1..9)
#pragma unroll
  for (int r = 1; r <= 9; ++r) v[27 + r] = (rk == r);
  v[37] = (stone == 0) && (lib_raw == KO_MARK);
}

}  // namespace dg
