// Checkpoint / restart of the native engine in the shard format of the Python front end
// (multigpu_advectiondiffusion_amd/utils/io.py save_checkpoint / load_checkpoint_box):
//
//   "ADVDIFF1" | u64 little-endian header length | JSON header | zero pad to 64 B |
//   the rank's owned box, float64 little-endian, array order (x fastest)
//
// one shard per rank, named PREFIX.rankNNNNN.ckpt.  The header carries the global grid,
// t, it and the shard's global box (box0 + shape).  A restart assembles its block —
// owned cells AND the ghost cells inside the domain, so no halo exchange is needed —
// from whatever shards overlap it: native and Python runs restart from each other's
// shards, on any process count and any slab / Cartesian layout.  The format executes
// nothing on load (no pickle), and both sides stream it plane by plane (no host copy of
// a whole field).  The reference has no checkpoint (only float32
// result.bin snapshots, MultiGPU/Diffusion3d_Baseline/Tools.c:91-119).
#include <algorithm>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <sstream>

#include "runtime.hpp"

namespace advdiff::rt {

static const char kMagic[8] = {'A', 'D', 'V', 'D', 'I', 'F', 'F', '1'};

std::string shard_path(const std::string& prefix, int rank) {
  char tail[32];
  std::snprintf(tail, sizeof tail, ".rank%05d.ckpt", rank);
  return prefix + tail;
}

std::vector<std::string> list_shards(const std::string& prefix) {
  namespace fs = std::filesystem;
  const fs::path p(prefix);
  const fs::path dir = p.has_parent_path() ? p.parent_path() : fs::path(".");
  const std::string head = p.filename().string() + ".rank";
  std::vector<std::string> out;
  if (fs::is_directory(dir))
    for (const auto& e : fs::directory_iterator(dir)) {
      const std::string n = e.path().filename().string();
      if (n.size() > head.size() + 5 && n.compare(0, head.size(), head) == 0 &&
          n.compare(n.size() - 5, 5, ".ckpt") == 0)
        out.push_back(e.path().string());
    }
  std::sort(out.begin(), out.end());
  if (out.empty()) throw std::runtime_error("no checkpoint shards for " + prefix);
  return out;
}

// The raw text of top-level key `key` of a JSON object (number, string or array; nested
// objects are skipped).  Enough for the headers both writers produce (no escaped quotes).
bool json_top_value(const std::string& js, const std::string& key, std::string& raw) {
  int depth = 0;
  for (size_t q = 0; q < js.size(); ++q) {
    const char c = js[q];
    if (c == '{' || c == '[') {
      ++depth;
    } else if (c == '}' || c == ']') {
      --depth;
    } else if (c == '"') {
      const size_t e = js.find('"', q + 1);
      if (e == std::string::npos) return false;
      if (depth == 1 && js.compare(q + 1, e - q - 1, key) == 0) {
        size_t v = js.find(':', e);
        if (v == std::string::npos) return false;
        ++v;
        while (v < js.size() && js[v] == ' ') ++v;
        if (v >= js.size()) return false;
        size_t end = v;
        if (js[v] == '[' || js[v] == '"') {
          end = js.find(js[v] == '[' ? ']' : '"', v + 1);
          if (end == std::string::npos) return false;
          ++end;
        } else {
          while (end < js.size() && js[end] != ',' && js[end] != '}') ++end;
        }
        raw = js.substr(v, end - v);
        return true;
      }
      q = e;  // a key or a string value at any depth: skip it whole
    }
  }
  return false;
}

static std::vector<int64_t> json_ints(const std::string& raw) {
  std::vector<int64_t> v;
  std::string s = raw;
  for (char& c : s)
    if (c == '[' || c == ']' || c == ',') c = ' ';
  std::istringstream is(s);
  long long x;
  while (is >> x) v.push_back(x);
  return v;
}

ShardInfo read_shard_info(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  char magic[8];
  if (!f.read(magic, 8) || std::memcmp(magic, kMagic, 8) != 0)
    throw std::runtime_error(path + ": not an advdiff checkpoint");
  uint64_t n = 0;
  f.read((char*)&n, 8);
  if (!f || n > (1u << 24)) throw std::runtime_error(path + ": bad header length");
  std::string js(n, '\0');
  f.read(js.data(), (std::streamsize)n);
  if (!f) throw std::runtime_error(path + ": truncated header");
  ShardInfo s;
  std::string raw;
  auto need = [&](const char* k) {
    if (!json_top_value(js, k, raw)) throw std::runtime_error(path + ": header lacks " + k);
    return raw;
  };
  s.shape = json_ints(need("shape"));
  s.grid = json_ints(need("grid"));
  s.dtype = need("dtype");
  s.dtype = s.dtype.substr(1, s.dtype.size() - 2);
  s.t = std::stod(need("t"));
  s.it = std::stoll(need("it"));
  if (json_top_value(js, "box0", raw)) {
    s.box0 = json_ints(raw);
  } else {  // slab shards of an older writer: plane0 along axis 0
    s.box0.assign(s.shape.size(), 0);
    s.box0[0] = std::stoll(need("plane0"));
  }
  if (s.box0.size() != s.shape.size() || s.grid.size() != s.shape.size())
    throw std::runtime_error(path + ": inconsistent header");
  if (s.dtype != "float64" && s.dtype != "float32")
    throw std::runtime_error(path + ": unsupported dtype " + s.dtype);
  s.offset = 8 + 8 + n;
  s.offset += (64 - s.offset % 64) % 64;
  return s;
}

// owned / loadable boxes of this rank, array order padded to three axes (2-D: axis 0 is a
// unit axis): local start, global start, extent
void Engine::own_box(int lo[3], int g0[3], int n[3]) const {
  const int off = 3 - p_.dims;
  for (int a = 0; a < 3; ++a) lo[a] = g0[a] = 0, n[a] = 1;
  for (int a = 0; a < p_.dims; ++a) {
    const Slab s = cd_.axis(a);
    lo[off + a] = s.ghost;
    g0[off + a] = s.start();
    n[off + a] = s.count();
  }
}

void Engine::save_checkpoint(const std::string& prefix, const std::string& ic_name) {
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  int lo[3], g0[3], n[3];
  own_box(lo, g0, n);
  const int off = 3 - p_.dims;
  auto list = [&](const int* v) {  // the run's axes of a padded triple, array order
    std::string s = "[";
    for (int a = off; a < 3; ++a) s += (a > off ? ", " : "") + std::to_string(v[a]);
    return s + "]";
  };
  const int pg[3] = {p_.dims == 3 ? cd_.pgrid[0] : 1, cd_.pgrid[p_.dims - 2],
                     cd_.pgrid[p_.dims - 1]};
  char tbuf[64];
  std::snprintf(tbuf, sizeof tbuf, "%.17g", t_);
  const std::string grid = "[" + std::to_string(p_.nx) + ", " + std::to_string(p_.ny) +
                           (p_.dims == 3 ? ", " + std::to_string(p_.nz) : std::string()) + "]";
  auto num = [](double v) {
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", v);
    return std::string(b);
  };
  const std::string lens = "[" + num(p_.L) + ", " + num(p_.W) +
                           (p_.dims == 3 ? ", " + num(p_.H) : std::string()) + "]";
  const bool diff = p_.physics == Physics::Diffusion;
  std::ostringstream h;  // keys sorted, as json.dumps(sort_keys=True) writes them
  h << "{\"box0\": " << list(g0) << ", \"dtype\": \"float64\", \"grid\": " << grid
    << ", \"ic\": \"" << ic_name << "\", \"integrator\": \""
    << (p_.integrator == 1 ? "lsrk45" : "ssprk3") << "\", \"it\": " << it_
    << ", \"lengths\": " << lens << ", \"model\": {\"model\": \""
    << (diff ? "diffusion" : "burgers") << "\", \"radius\": " << p_.radius()
    << ", \"writer\": \"native\"}, \"nplanes\": " << n[off] << ", \"pgrid\": " << list(pg)
    << ", \"plane0\": " << g0[off] << ", \"rank\": " << env_.rank << ", \"shape\": " << list(n)
    << ", \"t\": " << tbuf << ", \"world\": " << env_.size << "}";
  const std::string js = h.str();
  const std::string path = shard_path(prefix, env_.rank);
  namespace fs = std::filesystem;
  if (fs::path(path).has_parent_path()) fs::create_directories(fs::path(path).parent_path());
  const std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    const uint64_t hn = js.size();
    f.write(kMagic, 8);
    f.write((const char*)&hn, 8);
    f.write(js.data(), (std::streamsize)js.size());
    const std::string pad((64 - (16 + js.size()) % 64) % 64, '\0');
    f.write(pad.data(), (std::streamsize)pad.size());
    // the owned box plane by plane along axis 0 (2-D: one plane = the whole field), fp64
    std::vector<char> pl(plane_span());
    std::vector<double> row((size_t)n[2]);
    for (int k = 0; k < n[0]; ++k) {
      HIP_CHECK(hipMemcpy(pl.data(), plane3(u_, lo[0] + k), pl.size(), hipMemcpyDeviceToHost));
      for (int j = 0; j < n[1]; ++j) {
        const size_t base = (size_t)(lo[1] + j) * sy_ + lo[2];
        for (int i = 0; i < n[2]; ++i)
          row[i] = elem_ == 8 ? ((const double*)pl.data())[base + i]
                              : (double)((const float*)pl.data())[base + i];
        f.write((const char*)row.data(), (std::streamsize)(row.size() * sizeof(double)));
      }
    }
    if (!f) throw std::runtime_error("checkpoint: write failed: " + tmp);
  }
  fs::rename(tmp, path);
  tr_->barrier();  // every shard is complete when any rank returns
  if (env_.rank == 0) {
    // shards of an earlier run on more ranks under this prefix would be read back with ours
    const std::string head = fs::path(prefix).filename().string() + ".rank";
    for (const std::string& q : list_shards(prefix)) {
      const std::string n = fs::path(q).filename().string();
      const std::string digits = n.substr(head.size(), n.size() - head.size() - 5);
      if (!digits.empty() && digits.find_first_not_of("0123456789") == std::string::npos &&
          std::stoi(digits) >= env_.size)
        fs::remove(q);
    }
  }
  tr_->barrier();
}

void Engine::load_checkpoint(const std::string& prefix) {
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  const int off = 3 - p_.dims;
  // the block to fill: owned cells + ghosts, clipped to the domain (array order, 3 axes)
  int blo[3], bg0[3], bn[3];
  {
    int lo[3], g0[3], n[3];
    own_box(lo, g0, n);
    const int gshape[3] = {p_.dims == 3 ? p_.nz : 1, p_.ny, p_.nx};
    for (int a = 0; a < 3; ++a) {
      const int G = a >= off ? lo[a] : 0;
      const int s = std::max(g0[a] - G, 0), e = std::min(g0[a] + n[a] + G, gshape[a]);
      bg0[a] = s;
      bn[a] = e - s;
      blo[a] = lo[a] + (s - g0[a]);
    }
  }
  struct Src {
    ShardInfo h;
    int g0[3], n[3];
    std::ifstream f;
  };
  std::vector<Src> srcs;
  double t = 0;
  long long it = 0;
  bool first = true;
  const std::vector<int64_t> want = p_.dims == 3 ? std::vector<int64_t>{p_.nx, p_.ny, p_.nz}
                                                 : std::vector<int64_t>{p_.nx, p_.ny};
  for (const std::string& path : list_shards(prefix)) {
    ShardInfo h = read_shard_info(path);
    if (h.grid != want) throw std::runtime_error(path + ": checkpoint grid differs from the run's");
    if (first) {
      t = h.t, it = h.it, first = false;
    } else if (h.t != t || h.it != it) {  // e.g. stale shards of an earlier, wider run
      throw std::runtime_error(path + ": shard of another checkpoint (it " + std::to_string(h.it) +
                               " vs " + std::to_string(it) + ") under the same prefix");
    }
    Src s;
    for (int a = 0; a < 3; ++a) s.g0[a] = 0, s.n[a] = 1;
    for (int a = 0; a < p_.dims; ++a) s.g0[off + a] = (int)h.box0[a], s.n[off + a] = (int)h.shape[a];
    bool hit = true;
    for (int a = 0; a < 3; ++a)
      hit = hit && std::max(s.g0[a], bg0[a]) < std::min(s.g0[a] + s.n[a], bg0[a] + bn[a]);
    if (!hit) continue;
    s.h = h;
    s.f.open(path, std::ios::binary);
    srcs.push_back(std::move(s));
  }
  const size_t span = plane_span();
  std::vector<char> pl(span), raw;
  long long covered = 0;
  for (int k = 0; k < bn[0]; ++k) {
    char* dev = (char*)plane3(u_, blo[0] + k);
    HIP_CHECK(hipMemcpy(pl.data(), dev, span, hipMemcpyDeviceToHost));
    const int gk = bg0[0] + k;
    for (Src& s : srcs) {
      if (gk < s.g0[0] || gk >= s.g0[0] + s.n[0]) continue;
      const int j0 = std::max(s.g0[1], bg0[1]), j1 = std::min(s.g0[1] + s.n[1], bg0[1] + bn[1]);
      const int i0 = std::max(s.g0[2], bg0[2]), i1 = std::min(s.g0[2] + s.n[2], bg0[2] + bn[2]);
      if (j1 <= j0 || i1 <= i0) continue;
      const size_t es = s.h.dtype == "float64" ? 8 : 4;
      const int ni = i1 - i0;
      // rows of the shard that span its full x extent are contiguous: one read per plane
      // (slab shards always); otherwise one read per row
      const bool whole = ni == s.n[2];
      const int rows_per_read = whole ? j1 - j0 : 1;
      raw.resize((size_t)rows_per_read * ni * es);
      for (int gj = j0; gj < j1; gj += rows_per_read) {
        const size_t idx = ((size_t)(gk - s.g0[0]) * s.n[1] + (gj - s.g0[1])) * s.n[2] + (i0 - s.g0[2]);
        s.f.seekg((std::streamoff)(s.h.offset + idx * es));
        s.f.read(raw.data(), (std::streamsize)raw.size());
        if (!s.f) throw std::runtime_error("checkpoint: truncated shard");
        for (int r = 0; r < rows_per_read; ++r) {
          const size_t base = (size_t)(blo[1] + gj + r - bg0[1]) * sy_ + blo[2] + (i0 - bg0[2]);
          const char* src = raw.data() + (size_t)r * ni * es;
          for (int i = 0; i < ni; ++i) {
            const double v = es == 8 ? ((const double*)src)[i] : ((const float*)src)[i];
            if (elem_ == 8)
              ((double*)pl.data())[base + i] = v;
            else
              ((float*)pl.data())[base + i] = (float)v;
          }
        }
        covered += (long long)rows_per_read * ni;
      }
    }
    HIP_CHECK(hipMemcpy(dev, pl.data(), span, hipMemcpyHostToDevice));
  }
  if (covered > (long long)bn[0] * bn[1] * bn[2])
    throw std::runtime_error("checkpoint " + prefix +
                             ": overlapping shards cover this rank's block more than once "
                             "(shards of two runs?)");
  if (covered != (long long)bn[0] * bn[1] * bn[2])
    throw std::runtime_error("checkpoint " + prefix + " does not cover this rank's block");
  // the stage buffers start as copies of u, exactly as after the initial condition
  HIP_CHECK(hipMemcpyAsync(A_, u_, field_bytes_, hipMemcpyDeviceToDevice, compute_));
  if (B_ && p_.integrator == 1)
    HIP_CHECK(hipMemsetAsync(B_, 0, field_bytes_, compute_));
  else if (B_)
    HIP_CHECK(hipMemcpyAsync(B_, u_, field_bytes_, hipMemcpyDeviceToDevice, compute_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  t_ = t;
  it_ = (int)it;
  tr_->barrier();
}

}  // namespace advdiff::rt
