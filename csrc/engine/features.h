#pragma once
#include <cstdint>

namespace dg {
constexpr int kNetPlanes = 37;
// pl: 9 stored planes [9][361]; out: [37][361] float (0/1)
void expand_position(const uint8_t* pl, int player, int rank, float* out);
}  // namespace dg
