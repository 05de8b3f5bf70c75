#pragma once
#include <cstdint>

namespace dg {
constexpr int kNetPlanes = 37;
constexpr int kNetPlanesKo = 38;  // + plane 37: the simple-ko point (optional, off by default)
// pl: 9 stored planes [9][361]; out: [nplanes][361] float (0/1), nplanes 37 or 38
void expand_position(const uint8_t* pl, int player, int rank, float* out,
                     int nplanes = kNetPlanes);
}  // namespace dg
