// pybind11 module `_dgcpu`: Go engine, SGF parser, t7 codec, CPU feature expansion,
// threaded batch loader, parallel SGF -> position transcription.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <sys/stat.h>
#include <thread>

#include "features.h"
#include "go_engine.h"
#include "loader.h"
#include "sgf.h"
#include "t7.h"

namespace py = pybind11;
using namespace dg;

namespace {

using u8arr = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

std::vector<Move> to_moves(const std::vector<std::tuple<int, int, int>>& v) {
  std::vector<Move> m;
  m.reserve(v.size());
  for (auto& t : v) m.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
  return m;
}

py::list moves_py(const std::vector<Move>& v) {
  py::list l;
  for (auto& m : v) l.append(py::make_tuple(m.player, m.x, m.y));
  return l;
}

// ---- t7 <-> Python ----
py::object to_py(const t7::NodeP& n);

py::object key_py(const t7::NodeP& k) {
  if (k && k->kind == t7::Kind::Number) {
    const double d = k->num;
    if (d == (double)(long long)d) return py::int_((long long)d);
    return py::float_(d);
  }
  return to_py(k);
}

py::array tensor_py(const t7::Node& t) {
  std::vector<uint8_t> bytes;
  t7::tensor_bytes(t, &bytes);
  std::string dt;
  const std::string& c = t.cls;
  if (c.find("Byte") != std::string::npos) dt = "uint8";
  else if (c.find("Char") != std::string::npos) dt = "int8";
  else if (c.find("Short") != std::string::npos) dt = "int16";
  else if (c.find("Int") != std::string::npos) dt = "int32";
  else if (c.find("Long") != std::string::npos) dt = "int64";
  else if (c.find("Float") != std::string::npos) dt = "float32";
  else if (c.find("Double") != std::string::npos) dt = "float64";
  else throw std::runtime_error("t7: unsupported tensor class " + c);
  std::vector<py::ssize_t> shape(t.sizes.begin(), t.sizes.end());
  py::array arr(py::dtype(dt), shape);
  std::memcpy(arr.mutable_data(), bytes.data(), bytes.size());
  return arr;
}

py::object to_py(const t7::NodeP& n) {
  if (!n) return py::none();
  switch (n->kind) {
    case t7::Kind::Nil: return py::none();
    case t7::Kind::Number: return py::float_(n->num);
    case t7::Kind::String: return py::str(n->str);
    case t7::Kind::Boolean: return py::bool_(n->boolean);
    case t7::Kind::Table: {
      py::dict d;
      for (auto& kv : n->entries) d[key_py(kv.first)] = to_py(kv.second);
      return d;
    }
    case t7::Kind::Tensor: return tensor_py(*n);
    case t7::Kind::Storage: {
      const int es = t7::elem_size(n->cls);
      const size_t bytes = n->data ? n->data->size() : 0;
      py::array_t<uint8_t> a((py::ssize_t)bytes);
      if (bytes) std::memcpy(a.mutable_data(), n->data->data(), bytes);
      py::dict d;
      d["__torch_class__"] = n->cls;
      d["data"] = a;
      d["elem_size"] = es;
      return d;
    }
    case t7::Kind::Object: {
      py::dict d;
      py::object payload = to_py(n->payload);
      if (py::isinstance<py::dict>(payload)) {
        for (auto item : payload.cast<py::dict>()) d[item.first] = item.second;
      } else {
        d["__payload__"] = payload;
      }
      d["__torch_class__"] = n->cls;
      return d;
    }
  }
  return py::none();
}

t7::NodeP from_py(const py::handle& o);

t7::NodeP array_node(const py::array& a0) {
  py::array a = py::array::ensure(a0, py::array::c_style);
  std::string cls;
  const char k = a.dtype().kind();
  const int sz = (int)a.dtype().itemsize();
  if (k == 'u' && sz == 1) cls = "torch.ByteTensor";
  else if (k == 'i' && sz == 1) cls = "torch.CharTensor";
  else if (k == 'i' && sz == 2) cls = "torch.ShortTensor";
  else if (k == 'i' && sz == 4) cls = "torch.IntTensor";
  else if (k == 'i' && sz == 8) cls = "torch.LongTensor";
  else if (k == 'f' && sz == 4) cls = "torch.FloatTensor";
  else if (k == 'f' && sz == 8) cls = "torch.DoubleTensor";
  else if (k == 'b') {
    a = a.attr("astype")("uint8");
    cls = "torch.ByteTensor";
  } else throw std::runtime_error("t7: unsupported numpy dtype");
  std::vector<int64_t> sizes(a.shape(), a.shape() + a.ndim());
  return t7::make_tensor(cls, sizes, a.data(), (size_t)a.nbytes());
}

t7::NodeP from_py(const py::handle& o) {
  if (o.is_none()) return std::make_shared<t7::Node>();
  if (py::isinstance<py::bool_>(o)) return t7::Node::boolean_(o.cast<bool>());
  if (py::isinstance<py::int_>(o) || py::isinstance<py::float_>(o))
    return t7::Node::number(o.cast<double>());
  if (py::isinstance<py::str>(o)) return t7::Node::string(o.cast<std::string>());
  if (py::isinstance<py::bytes>(o)) return t7::Node::string(o.cast<std::string>());
  if (py::isinstance<py::array>(o)) return array_node(o.cast<py::array>());
  if (py::isinstance<py::dict>(o)) {
    py::dict d = o.cast<py::dict>();
    if (d.contains("__torch_class__")) {
      auto n = std::make_shared<t7::Node>();
      n->kind = t7::Kind::Object;
      n->cls = d["__torch_class__"].cast<std::string>();
      if (d.contains("__payload__")) {
        n->payload = from_py(d["__payload__"]);
      } else {
        auto tbl = t7::Node::table();
        for (auto item : d) {
          const std::string key = py::str(item.first);
          if (key == "__torch_class__") continue;
          tbl->set(from_py(item.first), from_py(item.second));
        }
        n->payload = tbl;
      }
      return n;
    }
    auto tbl = t7::Node::table();
    for (auto item : d) tbl->set(from_py(item.first), from_py(item.second));
    return tbl;
  }
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    auto tbl = t7::Node::table();
    int i = 1;
    for (auto item : o) tbl->set(t7::Node::number(i++), from_py(item));
    return tbl;
  }
  // torch.Tensor or anything with __array__
  if (py::hasattr(o, "numpy")) return array_node(o.attr("detach")().attr("cpu")().attr("numpy")());
  throw std::runtime_error("t7: cannot serialise object of type " +
                           std::string(py::str(o.get_type())));
}

bool file_exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

void mkdirs(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    ::mkdir(cur.c_str(), 0755);
  }
}

std::string read_text(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// One game: parse + replay + write t7 position files 1..N into dst (reference layout).
// Returns number of positions written, 0 if the game has no dan ranks (dropped like
// transcribe_from_to, makedata.lua:550), -1 on an illegal move.  A ".done" marker file is
// written on success (the reference used "file 100 exists" as its only resume marker).
int transcribe_one(const std::string& src, const std::string& dst, bool skip_done, bool mark_ko) {
  if (skip_done && (file_exists(dst + "/.done") || file_exists(dst + "/100"))) return -2;
  const SgfGame g = parse_sgf(read_text(src));
  if (!g.has_ranks()) return 0;
  std::vector<uint8_t> planes(g.moves.size() * NUM_STORED * NN);
  int n;
  try {
    n = game_positions(g.handicap, g.moves, planes.data(), mark_ko);
  } catch (const IllegalMove&) {
    return -1;
  }
  mkdirs(dst);
  for (int k = 0; k < n; ++k) {
    t7::Position p;
    std::memcpy(p.planes, planes.data() + (size_t)k * NUM_STORED * NN, NUM_STORED * NN);
    p.player = g.moves[k].player;
    p.x = g.moves[k].x + 1;
    p.y = g.moves[k].y + 1;
    p.rank_black = g.black_rank;
    p.rank_white = g.white_rank;
    const auto buf = t7::write_position(p);
    const std::string path = dst + "/" + std::to_string(k + 1);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::fwrite(buf.data(), 1, buf.size(), f);
    std::fclose(f);
  }
  FILE* f = std::fopen((dst + "/.done").c_str(), "wb");
  if (f) std::fclose(f);
  return n;
}

class PyLoader {
 public:
  PyLoader(const std::vector<std::tuple<std::string, int64_t, int>>& games, int batch,
           int threads, const std::vector<std::tuple<uintptr_t, uintptr_t, uintptr_t, uintptr_t>>&
               slots,
           uint64_t seed, bool position_uniform, uintptr_t pk_planes, uintptr_t pk_player,
           uintptr_t pk_rank, uintptr_t pk_label, int64_t start_seq) {
    std::vector<GameRef> g;
    for (auto& t : games) g.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
    std::vector<SlotBuffers> sb;
    for (auto& s : slots)
      sb.push_back({(uint8_t*)std::get<0>(s), (uint8_t*)std::get<1>(s), (uint8_t*)std::get<2>(s),
                    (int32_t*)std::get<3>(s)});
    impl_ = std::make_unique<Loader>(std::move(g), batch, threads, std::move(sb), seed,
                                     position_uniform, (const uint8_t*)pk_planes,
                                     (const uint8_t*)pk_player, (const uint8_t*)pk_rank,
                                     (const int32_t*)pk_label, start_seq);
  }
  py::tuple next() {
    int64_t seq = -1;
    int slot;
    {
      py::gil_scoped_release nogil;
      slot = impl_->next(&seq);
    }
    return py::make_tuple(slot, seq);
  }
  void release(int slot) { impl_->release(slot); }
  void stop() {
    py::gil_scoped_release nogil;
    impl_->stop();
  }
  int64_t errors() const { return impl_->errors(); }
  std::string last_error() { return impl_->last_error(); }
  std::vector<std::pair<int, int>> sample_batch(int64_t k) { return impl_->sample_batch(k); }

 private:
  std::unique_ptr<Loader> impl_;
};

}  // namespace

PYBIND11_MODULE(_dgcpu, m) {
  m.doc() = "deep_go_amd CPU runtime: Go engine, SGF, t7 codec, loader";

  m.def("game_positions",
        [](const std::vector<std::tuple<int, int, int>>& handicap,
           const std::vector<std::tuple<int, int, int>>& moves, bool mark_ko) {
          const auto h = to_moves(handicap), mv = to_moves(moves);
          py::array_t<uint8_t> out({(py::ssize_t)mv.size(), (py::ssize_t)9, (py::ssize_t)19,
                                    (py::ssize_t)19});
          {
            py::gil_scoped_release nogil;
            game_positions(h, mv, out.mutable_data(), mark_ko);
          }
          return out;
        },
        py::arg("handicap"), py::arg("moves"), py::arg("mark_ko") = false,
        "stored planes [n,9,19,19] of the position before each move (0-based x,y); mark_ko: "
        "the simple-ko point as KO_MARK in the liberty plane");
  m.def("game_ko_points",
        [](const std::vector<std::tuple<int, int, int>>& handicap,
           const std::vector<std::tuple<int, int, int>>& moves) {
          Board b;
          for (const Move& m : to_moves(handicap)) b.play(m);
          std::vector<int> ko;
          for (const Move& m : to_moves(moves)) {
            ko.push_back(b.ko());
            b.play(m);
          }
          return ko;
        },
        "simple-ko point (x*19+y, -1 none) of the position before each move");
  m.attr("KO_MARK") = (int)KO_MARK;
  m.def("summarize",
        [](u8arr stones, py::object ages) {
          if (stones.size() != NN) throw std::runtime_error("stones must have 361 entries");
          Board b;
          b.set_stones(stones.data());
          py::array_t<uint8_t> out({9, 19, 19});
          b.summarize(out.mutable_data());
          if (!ages.is_none()) {
            u8arr a = ages.cast<u8arr>();
            std::memcpy(out.mutable_data() + P_AGE * NN, a.data(), NN);
          }
          return out;
        },
        py::arg("stones"), py::arg("ages") = py::none());
  m.def("play",
        [](u8arr stones, int player, int x, int y) {
          Board b;
          b.set_stones(stones.data());
          b.play({player, x, y});
          py::array_t<uint8_t> out({19, 19});
          std::memcpy(out.mutable_data(), b.stones().data(), NN);
          return out;
        },
        "stones after a move with captures (0-based x,y); raises on occupied points");
  m.def("parse_sgf", [](const std::string& text) {
    const SgfGame g = parse_sgf(text);
    py::dict d;
    d["moves"] = moves_py(g.moves);
    d["handicap"] = moves_py(g.handicap);
    d["black_rank"] = g.black_rank;
    d["white_rank"] = g.white_rank;
    return d;
  });
  m.def("transcribe_sgf", [](const std::string& text, bool mark_ko) -> py::object {
    const SgfGame g = parse_sgf(text);
    if (!g.has_ranks()) return py::none();
    py::array_t<uint8_t> planes({(py::ssize_t)g.moves.size(), (py::ssize_t)9, (py::ssize_t)19,
                                 (py::ssize_t)19});
    game_positions(g.handicap, g.moves, planes.mutable_data(), mark_ko);
    py::dict d;
    d["planes"] = planes;
    d["moves"] = moves_py(g.moves);
    d["ranks"] = py::make_tuple(g.black_rank, g.white_rank);
    return d;
  }, py::arg("text"), py::arg("mark_ko") = false);
  m.def("transcribe_files",
        [](const std::vector<std::pair<std::string, std::string>>& jobs, int threads,
           bool skip_done, bool mark_ko) {
          std::vector<int> result(jobs.size(), 0);
          std::atomic<size_t> next{0};
          {
            py::gil_scoped_release nogil;
            std::vector<std::thread> pool;
            for (int t = 0; t < std::max(1, threads); ++t)
              pool.emplace_back([&] {
                for (size_t i = next++; i < jobs.size(); i = next++) {
                  try {
                    result[i] = transcribe_one(jobs[i].first, jobs[i].second, skip_done, mark_ko);
                  } catch (const std::exception&) {
                    result[i] = -3;
                  }
                }
              });
            for (auto& th : pool) th.join();
          }
          return result;
        },
        py::arg("jobs"), py::arg("threads") = 8, py::arg("skip_done") = true,
        py::arg("mark_ko") = false,
        "parallel SGF->t7 transcription; per job: #positions, 0 dropped (no dan ranks), "
        "-1 illegal move, -2 skipped (done), -3 I/O error");

  m.def("t7_loads", [](py::bytes b) {
    const std::string s = b;
    return to_py(t7::read((const uint8_t*)s.data(), s.size()));
  });
  m.def("t7_load", [](const std::string& path) { return to_py(t7::read_file(path)); });
  m.def("t7_dumps", [](py::object o) {
    const auto buf = t7::write(from_py(o));
    return py::bytes((const char*)buf.data(), buf.size());
  });
  m.def("t7_save", [](const std::string& path, py::object o) { t7::write_file(path, from_py(o)); });
  m.def("read_position", [](const std::string& path) {
    t7::Position p;
    std::string err;
    if (!t7::read_position_file(path, &p, &err)) throw std::runtime_error(path + ": " + err);
    py::array_t<uint8_t> planes({9, 19, 19});
    std::memcpy(planes.mutable_data(), p.planes, sizeof(p.planes));
    py::dict d;
    d["planes"] = planes;
    d["player"] = p.player;
    d["x"] = p.x;
    d["y"] = p.y;
    d["ranks"] = py::make_tuple(p.rank_black, p.rank_white);
    return d;
  });
  m.def("read_positions",
        [](const std::vector<std::string>& paths, int threads) {
          const size_t n = paths.size();
          py::array_t<uint8_t> planes({(py::ssize_t)n, (py::ssize_t)9, (py::ssize_t)19,
                                       (py::ssize_t)19});
          py::array_t<int32_t> meta({(py::ssize_t)n, (py::ssize_t)5});
          uint8_t* pl = planes.mutable_data();
          int32_t* mt = meta.mutable_data();
          std::atomic<size_t> next{0};
          std::atomic<int> bad{0};
          {
            py::gil_scoped_release nogil;
            std::vector<std::thread> pool;
            for (int t = 0; t < std::max(1, threads); ++t)
              pool.emplace_back([&] {
                for (size_t i = next++; i < n; i = next++) {
                  t7::Position p;
                  std::string err;
                  if (!t7::read_position_file(paths[i], &p, &err)) {
                    ++bad;
                    std::memset(pl + i * 9 * NN, 0, 9 * NN);
                    for (int k = 0; k < 5; ++k) mt[i * 5 + k] = -1;
                    continue;
                  }
                  std::memcpy(pl + i * 9 * NN, p.planes, 9 * NN);
                  mt[i * 5 + 0] = p.player;
                  mt[i * 5 + 1] = p.x;
                  mt[i * 5 + 2] = p.y;
                  mt[i * 5 + 3] = p.rank_black;
                  mt[i * 5 + 4] = p.rank_white;
                }
              });
            for (auto& th : pool) th.join();
          }
          if (bad) throw std::runtime_error(std::to_string(bad.load()) + " unreadable files");
          return py::make_tuple(planes, meta);
        },
        py::arg("paths"), py::arg("threads") = 8,
        "bulk decode: planes [n,9,19,19], meta [n,5] = (player, x, y, rank_b, rank_w)");
  m.def("write_position", [](const std::string& path, u8arr planes, int player, int x, int y,
                             int rank_black, int rank_white) {
    if (planes.size() != 9 * NN) throw std::runtime_error("planes must be 9x19x19");
    t7::Position p;
    std::memcpy(p.planes, planes.data(), sizeof(p.planes));
    p.player = player;
    p.x = x;
    p.y = y;
    p.rank_black = rank_black;
    p.rank_white = rank_white;
    const auto buf = t7::write_position(p);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::fwrite(buf.data(), 1, buf.size(), f);
    std::fclose(f);
  });
  m.def("expand",
        [](u8arr planes, u8arr player, u8arr rank, bool ko) {
          const py::ssize_t B = player.size();
          if (planes.size() != B * 9 * NN) throw std::runtime_error("planes must be [B,9,19,19]");
          const int NPL = ko ? kNetPlanesKo : kNetPlanes;
          py::array_t<float> out({B, (py::ssize_t)NPL, (py::ssize_t)19, (py::ssize_t)19});
          float* o = out.mutable_data();
          const uint8_t* pl = planes.data();
          const uint8_t* py_ = player.data();
          const uint8_t* rk = rank.data();
          {
            py::gil_scoped_release nogil;
            for (py::ssize_t b = 0; b < B; ++b)
              expand_position(pl + b * 9 * NN, py_[b], rk[b], o + b * NPL * NN, NPL);
          }
          return out;
        },
        py::arg("planes"), py::arg("player"), py::arg("rank"), py::arg("ko") = false,
        "9 stored planes -> 37 network planes (float32 0/1); ko: + plane 37, the simple-ko point");
  m.def("random_positions", [](int n, uint64_t seed, int max_moves) {
    std::vector<uint8_t> planes, player, rank;
    std::vector<int32_t> label;
    {
      py::gil_scoped_release nogil;
      random_positions(n, seed, max_moves, &planes, &player, &rank, &label);
    }
    py::array_t<uint8_t> P({(py::ssize_t)n, (py::ssize_t)9, (py::ssize_t)19, (py::ssize_t)19});
    std::memcpy(P.mutable_data(), planes.data(), planes.size());
    py::array_t<uint8_t> PL(n), RK(n);
    py::array_t<int32_t> LB(n);
    std::memcpy(PL.mutable_data(), player.data(), n);
    std::memcpy(RK.mutable_data(), rank.data(), n);
    std::memcpy(LB.mutable_data(), label.data(), n * 4);
    return py::make_tuple(P, PL, RK, LB);
  });

  py::class_<PyLoader>(m, "Loader")
      .def(py::init<const std::vector<std::tuple<std::string, int64_t, int>>&, int, int,
                    const std::vector<std::tuple<uintptr_t, uintptr_t, uintptr_t, uintptr_t>>&,
                    uint64_t, bool, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int64_t>(),
           py::arg("games"), py::arg("batch"), py::arg("threads"), py::arg("slots"),
           py::arg("seed"), py::arg("position_uniform"), py::arg("pk_planes") = 0,
           py::arg("pk_player") = 0, py::arg("pk_rank") = 0, py::arg("pk_label") = 0,
           py::arg("start_seq") = 0)
      .def("next", &PyLoader::next)
      .def("release", &PyLoader::release)
      .def("stop", &PyLoader::stop)
      .def("errors", &PyLoader::errors)
      .def("last_error", &PyLoader::last_error)
      .def("sample_batch", &PyLoader::sample_batch);
}
