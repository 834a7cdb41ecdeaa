// Host-only unit test of the native runtime (no GPU needed; built with ASan + UBSan by
// `make check`): slab decomposition invariants, the TCP star transport's collectives
// across forked ranks, and the reference summary block.
#include <sys/wait.h>
#include <unistd.h>

#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

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
}

int main() {
  test_slab_partition();
  test_star_collectives();
  test_summary_block();
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("runtime host tests: OK\n");
  return 0;
}
