// Torch7 binary serialization (the reference's torch.save / torch.load format) — C++ codec.
//
// Layout (little-endian; EXTERNAL torch7 File.lua semantics, verified on the fixture):
//   int32 type tag: 0 nil, 1 number (float64), 2 string (int32 len + bytes), 3 table,
//   4 torch object, 5 boolean (int32).
//   table: int32 ref-id; if the id was seen before the value is a back-reference, else
//          int32 n followed by n (key, value) objects.
//   torch: int32 ref-id (same back-reference rule), string version ("V 1"), string class;
//          Tensor payload: int32 ndim, int64 sizes[ndim], int64 strides[ndim], int64
//          storageOffset (1-based), storage object; Storage payload: int64 n, raw elements;
//          any other class (e.g. nn modules): one object (normally a table of fields).
// Position files written by the reference's makedata.lua hold
//   {ranks={[1]=b,[2]=w}, flat=true, input=ByteTensor[9][19][19], move={player,x,y}}.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace dg {
namespace t7 {

struct Node;
using NodeP = std::shared_ptr<Node>;

enum class Kind { Nil, Number, String, Table, Tensor, Storage, Boolean, Object };

struct Node {
  Kind kind = Kind::Nil;
  double num = 0.0;
  bool boolean = false;
  std::string str;                               // String
  std::vector<std::pair<NodeP, NodeP>> entries;  // Table (insertion order kept)
  std::string cls;                               // Tensor / Storage / Object class name
  std::string version = "V 1";
  std::vector<int64_t> sizes, strides;           // Tensor
  int64_t offset = 1;                            // Tensor storageOffset (1-based)
  NodeP storage;                                 // Tensor -> Storage
  std::shared_ptr<std::vector<uint8_t>> data;    // Storage raw bytes
  NodeP payload;                                 // Object payload

  // helpers
  static NodeP number(double v);
  static NodeP string(const std::string& s);
  static NodeP boolean_(bool b);
  static NodeP table();
  NodeP get(const std::string& key) const;  // table lookup by string key
  NodeP get(double key) const;              // table lookup by numeric key
  void set(NodeP k, NodeP v) { entries.emplace_back(std::move(k), std::move(v)); }
  int64_t numel() const;
};

class FormatError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// element size of a torch tensor/storage class ("torch.ByteTensor" -> 1, ...); 0 if unknown
int elem_size(const std::string& cls);

NodeP read(const uint8_t* buf, size_t len);
NodeP read_file(const std::string& path);
std::vector<uint8_t> write(const NodeP& root);
void write_file(const std::string& path, const NodeP& root);  // atomic (tmp + rename)

NodeP make_tensor(const std::string& cls, const std::vector<int64_t>& sizes, const void* src,
                  size_t nbytes);

// Contiguous copy of a tensor's elements (handles strides/offset) into out (bytes).
void tensor_bytes(const Node& t, std::vector<uint8_t>* out);

struct Position {
  uint8_t planes[9 * 361];
  int player = 0;     // 1 black, 2 white
  int x = 0, y = 0;   // 1-based SGF coordinates (x = first char)
  int rank_black = 0, rank_white = 0;
};

// Fast decode of one reference position file (schema above), parsing by key.
bool read_position(const uint8_t* buf, size_t len, Position* out, std::string* err);
bool read_position_file(const std::string& path, Position* out, std::string* err);
// Encode a position with the reference's schema (what makedata.lua's torch.save wrote).
std::vector<uint8_t> write_position(const Position& p);

}  // namespace t7
}  // namespace dg
