// SGF game-record parsing with the reference's token semantics (makedata.lua:6-120).
//
//  * a record is split into lines, lines into pieces on ';', pieces on '['; a piece is a
//    (PROP, value) token only when it has exactly one '[' and ends with ']'
//    (split_sgf :40-58) — so "B[pd]" is a token but "B[pd]C[..]" is not;
//  * moves: B/W tokens with two letters a..s (to_move :60-67); passes ('' or 'tt') and
//    anything else unparsable are skipped;
//  * handicap: lines starting with AB / AW, values between the first '[' and the last ']'
//    split on "][" (handicaps :24-38);
//  * ranks: BR/WR tokens ending in 'd' (amateur dan); otherwise the game has no ranks and
//    is dropped (get_ranks :102-120).
// Fix vs. the reference: both LF and CRLF line endings are accepted (the reference split
// on "\r\n" only, so LF files silently produced no moves).
#pragma once
#include <string>
#include <vector>

#include "go_engine.h"

namespace dg {

struct SgfGame {
  std::vector<Move> moves;
  std::vector<Move> handicap;
  int black_rank = 0;  // dan, 0 = missing / not dan
  int white_rank = 0;
  bool has_ranks() const { return black_rank > 0 && white_rank > 0; }
};

SgfGame parse_sgf(const std::string& text);

}  // namespace dg
