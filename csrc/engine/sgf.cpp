#include "sgf.h"

#include <cstdlib>

namespace dg {

namespace {

std::vector<std::string> split_lines(const std::string& s) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == '\n') {
      size_t end = i;
      if (end > start && s[end - 1] == '\r') --end;
      out.emplace_back(s.substr(start, end - start));
      start = i + 1;
    }
  }
  return out;
}

std::vector<std::string> split_char(const std::string& s, char c) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i)
    if (i == s.size() || s[i] == c) {
      out.emplace_back(s.substr(start, i - start));
      start = i + 1;
    }
  return out;
}

int coord(char c) { return (c >= 'a' && c <= 's') ? c - 'a' : -1; }

bool to_move(const std::string& v, int* x, int* y) {
  if (v.size() != 2) return false;
  *x = coord(v[0]);
  *y = coord(v[1]);
  return *x >= 0 && *y >= 0;
}

int to_rank(const std::string& v) {
  if (v.empty() || v.back() != 'd') return 0;
  const std::string num = v.substr(0, v.size() - 1);
  if (num.empty()) return 0;
  char* end = nullptr;
  const double d = std::strtod(num.c_str(), &end);
  if (end == num.c_str() || *end != '\0') return 0;
  return d > 0 ? (int)d : 0;
}

}  // namespace

SgfGame parse_sgf(const std::string& text) {
  SgfGame g;
  const auto lines = split_lines(text);
  for (const auto& line : lines) {
    // handicap lines (handicaps :24-38): AB[..][..] / AW[..]
    if (line.size() >= 2 && line[0] == 'A' && (line[1] == 'B' || line[1] == 'W')) {
      const int player = line[1] == 'W' ? 2 : 1;
      if (line.size() >= 4) {
        const std::string body = line.substr(3, line.size() - 4);  // sub(4, -2)
        size_t start = 0;
        while (true) {
          const size_t p = body.find("][", start);
          const std::string pos = body.substr(start, p == std::string::npos ? std::string::npos
                                                                             : p - start);
          int x, y;
          if (to_move(pos, &x, &y)) g.handicap.push_back({player, x, y});
          if (p == std::string::npos) break;
          start = p + 2;
        }
      }
    }
    for (const auto& piece : split_char(line, ';')) {
      const auto sub = split_char(piece, '[');
      if (sub.size() != 2 || sub[1].empty() || sub[1].back() != ']') continue;
      const std::string& prop = sub[0];
      const std::string val = sub[1].substr(0, sub[1].size() - 1);
      if (prop == "B" || prop == "W") {
        int x, y;
        if (to_move(val, &x, &y)) g.moves.push_back({prop == "B" ? 1 : 2, x, y});
      } else if (prop == "BR") {
        g.black_rank = to_rank(val);
      } else if (prop == "WR") {
        g.white_rank = to_rank(val);
      }
    }
  }
  return g;
}

}  // namespace dg
