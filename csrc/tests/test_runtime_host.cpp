// Host-only unit test of the native runtime (no GPU needed; built with ASan + UBSan by
// `make check`): slab decomposition invariants, the TCP star transport's collectives
// across forked ranks, the reference summary block and the checkpoint shard header.
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cassert>
#include <fstream>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

#include "runtime.hpp"

using namespace advdiff::rt;

static int failures = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

// every non-frozen plane is updated by exactly one of interior/blo/bhi, on one rank
static void test_slab_partition() {
  for (int n : {23, 40, 64, 101})
    for (int size : {1, 2, 3, 4, 7})
      for (int ghost : {1, 2, 3, 6}) {
        if (n < size * ghost) continue;
        for (int border : {ghost, ghost + 1}) {
          std::vector<int> hits(n, 0);
          for (int r = 0; r < size; ++r) {
            Slab s;
            s.n = n;
            s.size = size;
            s.rank = r;
            s.ghost = ghost;
            Range in, lo, hi;
            s.split(border, ghost, in, lo, hi);
            const Range full = s.compute_range(border);
            EXPECT(lo.lo == full.lo || lo.empty());
            for (const Range& q : {in, lo, hi})
              for (int l = q.lo; l < q.hi; ++l) {
                EXPECT(l >= ghost && l < ghost + s.count());  // never a ghost plane
                ++hits[s.start() - ghost + l];
              }
            // the interior never reads a ghost plane
            if (!in.empty()) {
              EXPECT(s.lower() < 0 || in.lo - ghost >= ghost);
              EXPECT(s.upper() < 0 || in.hi + ghost <= ghost + s.count());
            }
          }
          for (int g = 0; g < n; ++g)
            EXPECT(hits[g] == ((g >= border && g < n - border) ? 1 : 0));
        }
      }
}

static void test_star_collectives() {
  const int world = 4;
  const int port = 23000 + (int)(getpid() % 20000);
  std::vector<pid_t> kids;
  for (int r = 0; r < world; ++r) {
    pid_t pid = fork();
    if (pid == 0) {
      ProcEnv e;
      e.rank = r;
      e.size = world;
      e.master_port = port;
      auto tr = make_transport(e, "socket");
      int bad = 0;
      bad += tr->allreduce_max(1.5 * r) != 1.5 * (world - 1);
      bad += tr->allreduce_sum(r + 1.0) != world * (world + 1) / 2.0;
      tr->barrier();
      std::vector<char> mine(r + 1, (char)('a' + r));
      std::vector<char> all = tr->gather(mine);
      if (r == 0) bad += std::string(all.begin(), all.end()) != "abbcccdddd";
      else bad += !all.empty();
      std::_Exit(bad);
    }
    kids.push_back(pid);
  }
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    EXPECT(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }
}

static void test_summary_block() {
  Problem p;
  p.nx = 10;
  p.ny = 11;
  p.nz = 12;
  Stats s;
  s.steps = 5;
  s.seconds = 0.5;
  const std::string txt = summary_multigpu("Diffusion-3D", "opt", s, p, 2);
  EXPECT(txt.find("Total effective GFLOPs") != std::string::npos);
  EXPECT(txt.find("3D Grid Size                                 :  10 x 11 x 12") !=
         std::string::npos);
  EXPECT(txt.find("Iterations                                   :  5 x 3 RK steps") !=
         std::string::npos);
  // single-GPU block: the SG heat GFLOPs has no x3 (5 x 1320 x 8e-9 / 0.5 s), Burgers has
  s.t = 0.25;
  const std::string sg = summary_singlegpu("Diffusion-3D", "opt", s, p, {{"MLUPS", "1.0"}});
  EXPECT(sg.find("Total effective GFLOPs                       :  0.000106\n") != std::string::npos);
  EXPECT(sg.find("3D Grid Size                                 :  10 x 11 x 12 \n") != std::string::npos);
  EXPECT(sg.find("Final Time                                   :  0.25\n") != std::string::npos);
  EXPECT(sg.find("MLUPS                                        :  1.0\n") != std::string::npos);
  p.physics = Physics::Burgers;
  EXPECT(summary_singlegpu("B", "o", s, p, {}).find(":  0.000317\n") != std::string::npos);
}

// Cartesian blocks: over all ranks, interior + boundary boxes cover every non-frozen
// cell exactly once; the interior box never reaches a split face's ghost layers; a
// rank's neighbours are symmetric; parse_pgrid validates the product
static void test_cart_partition() {
  const int shapes[][3] = {{30, 26, 41}, {17, 40, 33}};
  const int grids[][3] = {{1, 2, 2}, {2, 1, 2}, {2, 2, 2}, {3, 2, 1}, {1, 1, 4}};
  for (const auto& sh : shapes)
    for (const auto& pg : grids)
      for (int ghost : {2, 6}) {
        Cart c;
        c.dims = 3;
        for (int a = 0; a < 3; ++a) {
          c.shape[a] = sh[a];
          c.pgrid[a] = pg[a];
        }
        c.ghost = ghost;
        bool fits = true;
        for (int a = 0; a < 3; ++a)
          if (c.shape[a] < c.pgrid[a] * std::max(c.ghost_of_axis(a), 1)) fits = false;
        if (!fits) continue;
        const int border = 2;
        std::vector<int> hits((size_t)sh[0] * sh[1] * sh[2], 0);
        for (int r = 0; r < c.size(); ++r) {
          c.rank = r;
          Slab ax[3];
          for (int a = 0; a < 3; ++a) ax[a] = c.axis(a);
          Box in;
          std::vector<Box> bnd;
          c.split_boxes(border, ghost, in, bnd);
          std::vector<Box> all(bnd);
          all.push_back(in);
          for (const Box& b : all) {
            if (b.empty(3)) continue;
            for (int k = b.r[0].lo; k < b.r[0].hi; ++k)
              for (int j = b.r[1].lo; j < b.r[1].hi; ++j)
                for (int i = b.r[2].lo; i < b.r[2].hi; ++i) {
                  const int g[3] = {ax[0].start() - ax[0].ghost + k, ax[1].start() - ax[1].ghost + j,
                                    ax[2].start() - ax[2].ghost + i};
                  ++hits[((size_t)g[0] * sh[1] + g[1]) * sh[2] + g[2]];
                }
          }
          for (int a = 0; a < 3; ++a) {
            if (in.empty(3) || c.pgrid[a] == 1) continue;
            if (c.neighbor(a, -1) >= 0) EXPECT(in.r[a].lo >= ax[a].ghost + ghost);
            if (c.neighbor(a, 1) >= 0) EXPECT(in.r[a].hi <= ax[a].ghost + ax[a].count() - ghost);
            for (int side : {-1, 1}) {
              const int nb = c.neighbor(a, side);
              if (nb < 0) continue;
              Cart o = c;
              o.rank = nb;
              EXPECT(o.neighbor(a, -side) == r);
            }
          }
        }
        for (int z = 0; z < sh[0]; ++z)
          for (int y = 0; y < sh[1]; ++y)
            for (int x = 0; x < sh[2]; ++x) {
              const bool act = z >= border && z < sh[0] - border && y >= border &&
                               y < sh[1] - border && x >= border && x < sh[2] - border;
              EXPECT(hits[((size_t)z * sh[1] + y) * sh[2] + x] == (act ? 1 : 0));
            }
      }
  int pg[3];
  parse_pgrid("2x2x1", 3, 4, pg);
  EXPECT(pg[0] == 2 && pg[1] == 2 && pg[2] == 1);
  bool threw = false;
  try {
    parse_pgrid("2x2", 3, 4, pg);
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT(threw);
}

// a shard as utils/io.py writes it (json.dumps(sort_keys=True): a nested "model" object
// whose keys must not shadow the top-level ones; payload 64-B aligned)
static void test_checkpoint_header() {
  const std::string js =
      "{\"box0\": [8, 0, 0], \"dtype\": \"float64\", \"grid\": [5, 3, 20], \"ic\": \"sine\", "
      "\"integrator\": \"ssprk3\", \"it\": 12, \"lengths\": [1.0, 1.0, 1.0], \"model\": "
      "{\"K\": 1.0, \"it\": 99, \"model\": \"diffusion\", \"shape\": [1], \"t\": 7.5}, "
      "\"nplanes\": 4, \"pgrid\": [2, 1, 1], \"plane0\": 8, \"rank\": 1, \"shape\": [4, 3, 5], "
      "\"t\": 0.0012500000000000002, \"world\": 2}";
  std::string raw;
  EXPECT(json_top_value(js, "it", raw) && raw == "12");
  EXPECT(json_top_value(js, "t", raw) && raw == "0.0012500000000000002");
  EXPECT(json_top_value(js, "shape", raw) && raw == "[4, 3, 5]");
  EXPECT(!json_top_value(js, "K", raw));  // nested only
  // truncated headers: refused, and no out-of-range access (ASan)
  EXPECT(!json_top_value("{\"it\":", "it", raw));
  EXPECT(!json_top_value("{\"shape\": [1, 2", "shape", raw));
  EXPECT(!json_top_value("{\"dtype\": \"float", "dtype", raw));
  EXPECT(!json_top_value("{\"it", "it", raw));
  char tmpl[] = "/tmp/advdiff_ckpt_XXXXXX";
  const int fd = mkstemp(tmpl);
  EXPECT(fd >= 0);
  close(fd);
  {
    std::ofstream f(tmpl, std::ios::binary);
    const uint64_t n = js.size();
    f.write("ADVDIFF1", 8);
    f.write((const char*)&n, 8);
    f.write(js.data(), (std::streamsize)js.size());
  }
  const ShardInfo h = read_shard_info(tmpl);
  EXPECT((h.shape == std::vector<int64_t>{4, 3, 5}));
  EXPECT((h.box0 == std::vector<int64_t>{8, 0, 0}));
  EXPECT((h.grid == std::vector<int64_t>{5, 3, 20}));
  EXPECT(h.dtype == "float64" && h.it == 12 && h.t == 0.0012500000000000002);
  EXPECT(h.offset % 64 == 0 && h.offset >= 16 + js.size() && h.offset < 16 + js.size() + 64);
  std::remove(tmpl);
  EXPECT(shard_path("out/ck", 3) == "out/ck.rank00003.ckpt");
}

// the comm watchdog: fires on a transport's asynchronous error, and on a missing heartbeat
// only while armed; beats keep it quiet (on_fail replaced: no abort, no exit)
namespace {
class FakeTransport final : public Transport {
 public:
  std::atomic<int> err{0};
  std::atomic<int> aborted{0};
  const char* name() const override { return "fake"; }
  void exchange(const std::vector<Msg>&, hipStream_t) override {}
  void halo(const void*, void*, const void*, void*, size_t, int, int, hipStream_t) override {}
  double allreduce_max(double v) override { return v; }
  double allreduce_sum(double v) override { return v; }
  void barrier() override {}
  std::vector<char> gather(const std::vector<char>& l) override { return l; }
  int poll_error() override { return err.load(); }
  void abort() override { ++aborted; }
};
}  // namespace

static void test_watchdog() {
  using namespace std::chrono_literals;
  FakeTransport tr;
  std::atomic<int> fired{0};
  std::string why;
  std::mutex m;
  auto on_fail = [&](const std::string& w) {
    std::lock_guard<std::mutex> g(m);
    why = w;
    ++fired;
  };
  {  // not armed: a silent main thread is fine (setup, output, gathers)
    Watchdog wd(&tr, 0, 0.2, on_fail, 0.02);
    std::this_thread::sleep_for(400ms);
    EXPECT(fired.load() == 0);
    wd.arm();  // armed and beating: quiet
    for (int i = 0; i < 20; ++i) {
      std::this_thread::sleep_for(20ms);
      wd.beat();
    }
    EXPECT(fired.load() == 0);
    std::this_thread::sleep_for(500ms);  // armed, no beat for > timeout: fires once
    EXPECT(fired.load() == 1);
    EXPECT(wd.fired());
    EXPECT(why.find("no progress") != std::string::npos);
  }
  fired = 0;
  {  // an asynchronous transport error fires at once, armed or not
    Watchdog wd(&tr, 0, 100.0, on_fail, 0.02);
    tr.err = 3;
    std::this_thread::sleep_for(200ms);
    EXPECT(fired.load() == 1);
    EXPECT(why.find("asynchronous error 3") != std::string::npos);
  }
  tr.err = 0;
  fired = 0;
  {  // timeout <= 0: off
    Watchdog wd(&tr, 0, 0.0, on_fail, 0.02);
    wd.arm();
    std::this_thread::sleep_for(100ms);
    EXPECT(fired.load() == 0);
  }
}

int main() {
  test_watchdog();
  test_checkpoint_header();
  test_slab_partition();
  test_cart_partition();
  test_star_collectives();
  test_summary_block();
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("runtime host tests: OK\n");
  return 0;
}
