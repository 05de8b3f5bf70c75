#include "t7.h"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <unordered_map>

namespace dg {
namespace t7 {

namespace {

enum Tag : int32_t { T_NIL = 0, T_NUMBER = 1, T_STRING = 2, T_TABLE = 3, T_TORCH = 4, T_BOOL = 5 };

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  std::unordered_map<int32_t, NodeP> memo;

  void need(size_t n) {
    if ((size_t)(end - p) < n) throw FormatError("t7: truncated input");
  }
  int32_t i32() {
    need(4);
    int32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  int64_t i64() {
    need(8);
    int64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  double f64() {
    need(8);
    double v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  std::string str() {
    const int32_t n = i32();
    if (n < 0) throw FormatError("t7: negative string length");
    need((size_t)n);
    std::string s((const char*)p, (size_t)n);
    p += n;
    return s;
  }

  NodeP object(int depth = 0) {
    if (depth > 512) throw FormatError("t7: nesting too deep");
    const int32_t tag = i32();
    switch (tag) {
      case T_NIL: return std::make_shared<Node>();
      case T_NUMBER: return Node::number(f64());
      case T_STRING: return Node::string(str());
      case T_BOOL: return Node::boolean_(i32() != 0);
      case T_TABLE: {
        const int32_t ref = i32();
        auto it = memo.find(ref);
        if (it != memo.end()) return it->second;
        auto n = Node::table();
        memo[ref] = n;
        const int32_t count = i32();
        if (count < 0) throw FormatError("t7: negative table size");
        for (int32_t i = 0; i < count; ++i) {
          NodeP k = object(depth + 1);
          NodeP v = object(depth + 1);
          n->set(k, v);
        }
        return n;
      }
      case T_TORCH: {
        const int32_t ref = i32();
        auto it = memo.find(ref);
        if (it != memo.end()) return it->second;
        auto n = std::make_shared<Node>();
        memo[ref] = n;
        std::string version = str();
        std::string cls;
        if (version.rfind("V ", 0) == 0) {
          cls = str();
        } else {  // pre-versioning files store the class name directly
          cls = version;
          version = "";
        }
        n->version = version;
        n->cls = cls;
        const bool is_tensor = cls.size() > 6 && cls.compare(cls.size() - 6, 6, "Tensor") == 0;
        const bool is_storage = cls.size() > 7 && cls.compare(cls.size() - 7, 7, "Storage") == 0;
        if (is_tensor && cls.rfind("torch.", 0) == 0) {
          n->kind = Kind::Tensor;
          const int32_t nd = i32();
          if (nd < 0 || nd > 64) throw FormatError("t7: bad tensor ndim");
          n->sizes.resize(nd);
          n->strides.resize(nd);
          for (auto& s : n->sizes) s = i64();
          for (auto& s : n->strides) s = i64();
          n->offset = i64();
          n->storage = object(depth + 1);
        } else if (is_storage && cls.rfind("torch.", 0) == 0) {
          n->kind = Kind::Storage;
          const int64_t count = i64();
          const int es = elem_size(cls);
          if (es == 0 || count < 0) throw FormatError("t7: unsupported storage " + cls);
          const size_t bytes = (size_t)count * es;
          need(bytes);
          n->data = std::make_shared<std::vector<uint8_t>>(p, p + bytes);
          p += bytes;
        } else {
          n->kind = Kind::Object;
          n->payload = object(depth + 1);
        }
        return n;
      }
      default: throw FormatError("t7: unsupported type tag " + std::to_string(tag));
    }
  }
};

struct Writer {
  std::vector<uint8_t> out;
  std::unordered_map<const Node*, int32_t> refs;
  int32_t next_ref = 1;

  void bytes(const void* s, size_t n) {
    const uint8_t* b = (const uint8_t*)s;
    out.insert(out.end(), b, b + n);
  }
  void i32(int32_t v) { bytes(&v, 4); }
  void i64(int64_t v) { bytes(&v, 8); }
  void f64(double v) { bytes(&v, 8); }
  void str(const std::string& s) {
    i32((int32_t)s.size());
    bytes(s.data(), s.size());
  }
  // returns true if this is a back-reference (already written)
  bool ref(const Node* n) {
    auto it = refs.find(n);
    if (it != refs.end()) {
      i32(it->second);
      return true;
    }
    refs[n] = next_ref;
    i32(next_ref++);
    return false;
  }
  void object(const NodeP& n) {
    if (!n) {
      i32(T_NIL);
      return;
    }
    switch (n->kind) {
      case Kind::Nil: i32(T_NIL); break;
      case Kind::Number: i32(T_NUMBER); f64(n->num); break;
      case Kind::String: i32(T_STRING); str(n->str); break;
      case Kind::Boolean: i32(T_BOOL); i32(n->boolean ? 1 : 0); break;
      case Kind::Table:
        i32(T_TABLE);
        if (ref(n.get())) break;
        i32((int32_t)n->entries.size());
        for (auto& kv : n->entries) {
          object(kv.first);
          object(kv.second);
        }
        break;
      case Kind::Tensor:
        i32(T_TORCH);
        if (ref(n.get())) break;
        str(n->version.empty() ? "V 1" : n->version);
        str(n->cls);
        i32((int32_t)n->sizes.size());
        for (auto s : n->sizes) i64(s);
        for (auto s : n->strides) i64(s);
        i64(n->offset);
        object(n->storage);
        break;
      case Kind::Storage: {
        i32(T_TORCH);
        if (ref(n.get())) break;
        str(n->version.empty() ? "V 1" : n->version);
        str(n->cls);
        const int es = elem_size(n->cls);
        const size_t bytes_ = n->data ? n->data->size() : 0;
        i64(es ? (int64_t)(bytes_ / es) : 0);
        if (bytes_) bytes(n->data->data(), bytes_);
        break;
      }
      case Kind::Object:
        i32(T_TORCH);
        if (ref(n.get())) break;
        str(n->version.empty() ? "V 1" : n->version);
        str(n->cls);
        object(n->payload);
        break;
    }
  }
};

std::string storage_class_of(const std::string& tensor_cls) {
  // torch.ByteTensor -> torch.ByteStorage
  return tensor_cls.substr(0, tensor_cls.size() - 6) + "Storage";
}

}  // namespace

NodeP Node::number(double v) {
  auto n = std::make_shared<Node>();
  n->kind = Kind::Number;
  n->num = v;
  return n;
}
NodeP Node::string(const std::string& s) {
  auto n = std::make_shared<Node>();
  n->kind = Kind::String;
  n->str = s;
  return n;
}
NodeP Node::boolean_(bool b) {
  auto n = std::make_shared<Node>();
  n->kind = Kind::Boolean;
  n->boolean = b;
  return n;
}
NodeP Node::table() {
  auto n = std::make_shared<Node>();
  n->kind = Kind::Table;
  return n;
}
NodeP Node::get(const std::string& key) const {
  for (auto& kv : entries)
    if (kv.first && kv.first->kind == Kind::String && kv.first->str == key) return kv.second;
  return nullptr;
}
NodeP Node::get(double key) const {
  for (auto& kv : entries)
    if (kv.first && kv.first->kind == Kind::Number && kv.first->num == key) return kv.second;
  return nullptr;
}
int64_t Node::numel() const {
  int64_t n = 1;
  for (auto s : sizes) n *= s;
  return sizes.empty() ? 0 : n;
}

int elem_size(const std::string& cls) {
  auto has = [&](const char* k) { return cls.find(k) != std::string::npos; };
  if (has("Byte") || has("Char")) return 1;
  if (has("Short") || has("Half")) return 2;
  if (has("Int") || has("Float")) return 4;
  if (has("Long") || has("Double")) return 8;
  return 0;
}

NodeP read(const uint8_t* buf, size_t len) {
  Reader r{buf, buf + len, {}};
  return r.object();
}

static std::vector<uint8_t> slurp(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<uint8_t> buf;
  uint8_t tmp[1 << 15];
  size_t n;
  while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
  std::fclose(f);
  return buf;
}

NodeP read_file(const std::string& path) {
  auto buf = slurp(path);
  return read(buf.data(), buf.size());
}

std::vector<uint8_t> write(const NodeP& root) {
  Writer w;
  w.object(root);
  return std::move(w.out);
}

void write_file(const std::string& path, const NodeP& root) {
  const auto buf = write(root);
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + tmp);
  const size_t n = std::fwrite(buf.data(), 1, buf.size(), f);
  std::fclose(f);
  if (n != buf.size()) throw std::runtime_error("short write " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename " + path);
}

NodeP make_tensor(const std::string& cls, const std::vector<int64_t>& sizes, const void* src,
                  size_t nbytes) {
  auto t = std::make_shared<Node>();
  t->kind = Kind::Tensor;
  t->cls = cls;
  t->sizes = sizes;
  t->strides.resize(sizes.size());
  int64_t st = 1;
  for (int i = (int)sizes.size() - 1; i >= 0; --i) {
    t->strides[i] = st;
    st *= sizes[i];
  }
  t->offset = 1;
  auto s = std::make_shared<Node>();
  s->kind = Kind::Storage;
  s->cls = storage_class_of(cls);
  s->data = std::make_shared<std::vector<uint8_t>>((const uint8_t*)src,
                                                   (const uint8_t*)src + nbytes);
  t->storage = s;
  return t;
}

void tensor_bytes(const Node& t, std::vector<uint8_t>* out) {
  const int es = elem_size(t.cls);
  if (t.kind != Kind::Tensor || !t.storage || !t.storage->data || es == 0)
    throw FormatError("t7: not a readable tensor");
  const int64_t n = t.numel();
  out->resize((size_t)n * es);
  const auto& d = *t.storage->data;
  const int nd = (int)t.sizes.size();
  std::vector<int64_t> idx(nd, 0);
  for (int64_t e = 0; e < n; ++e) {
    int64_t off = t.offset - 1;
    for (int k = 0; k < nd; ++k) off += idx[k] * t.strides[k];
    if (off < 0 || (size_t)(off + 1) * es > d.size()) throw FormatError("t7: tensor out of storage");
    std::memcpy(out->data() + e * es, d.data() + off * es, es);
    for (int k = nd - 1; k >= 0; --k) {
      if (++idx[k] < t.sizes[k]) break;
      idx[k] = 0;
    }
  }
}

bool read_position(const uint8_t* buf, size_t len, Position* out, std::string* err) {
  try {
    NodeP root = read(buf, len);
    if (!root || root->kind != Kind::Table) throw FormatError("root is not a table");
    NodeP in = root->get("input");
    NodeP mv = root->get("move");
    NodeP rk = root->get("ranks");
    if (!in || in->kind != Kind::Tensor) throw FormatError("missing input tensor");
    if (!mv || mv->kind != Kind::Table) throw FormatError("missing move");
    if (in->numel() != 9 * 361 || elem_size(in->cls) != 1) throw FormatError("bad input shape");
    std::vector<uint8_t> planes;
    tensor_bytes(*in, &planes);
    std::memcpy(out->planes, planes.data(), 9 * 361);
    auto num = [](const NodeP& n) {
      if (!n || n->kind != Kind::Number) throw FormatError("expected number");
      return n->num;
    };
    out->player = (int)num(mv->get("player"));
    out->x = (int)num(mv->get("x"));
    out->y = (int)num(mv->get("y"));
    out->rank_black = out->rank_white = 0;
    if (rk && rk->kind == Kind::Table) {
      NodeP b = rk->get(1.0), w = rk->get(2.0);
      if (b && b->kind == Kind::Number) out->rank_black = (int)b->num;
      if (w && w->kind == Kind::Number) out->rank_white = (int)w->num;
    }
    return true;
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
}

bool read_position_file(const std::string& path, Position* out, std::string* err) {
  std::vector<uint8_t> buf;
  try {
    buf = slurp(path);
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
  return read_position(buf.data(), buf.size(), out, err);
}

std::vector<uint8_t> write_position(const Position& p) {
  // Same table shape and key set as flatten_data (dataloader.lua:30-39); key order follows
  // the fixture files (ranks, flat, input, move).
  auto root = Node::table();
  auto ranks = Node::table();
  ranks->set(Node::number(1), Node::number(p.rank_black));
  ranks->set(Node::number(2), Node::number(p.rank_white));
  root->set(Node::string("ranks"), ranks);
  root->set(Node::string("flat"), Node::boolean_(true));
  root->set(Node::string("input"), make_tensor("torch.ByteTensor", {9, 19, 19}, p.planes, 9 * 361));
  auto mv = Node::table();
  mv->set(Node::string("y"), Node::number(p.y));
  mv->set(Node::string("player"), Node::number(p.player));
  mv->set(Node::string("x"), Node::number(p.x));
  root->set(Node::string("move"), mv);
  return write(root);
}

}  // namespace t7
}  // namespace dg
