// Host-side launch helpers shared by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>
#include <stdint.h>

namespace advdiff {

// Number of workgroups we aim for per launch (A/B: 512..4096 within 4 %, 1024 best).  A
// stencil launch needs >> 256 groups to fill the 8 XCDs (MI355X_MICROARCH.md,
// "Workgroup dispatch").
constexpr long long kTargetBlocks = 1024;

// Length of the marching chunk (planes per workgroup) so that the launch has at
// least kTargetBlocks groups while each group marches far enough to amortise the
// 2R-plane prologue of its register window.
inline int knob(const char* name, int def);

inline int pick_chunk(int nrange, long long xyblocks, int minc, int maxc) {
  if (nrange <= 0) return 1;
  constexpr long long target = kTargetBlocks;
  long long want_chunks = (target + xyblocks - 1) / std::max<long long>(xyblocks, 1);
  long long c = (nrange + want_chunks - 1) / std::max<long long>(want_chunks, 1);
  c = std::max<long long>(c, minc);
  c = std::min<long long>(c, maxc);
  return (int)std::max<long long>(c, 1);
}

inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

// Compute units of the current device (cached per device id).
inline int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// Resident workgroups per CU of kernel `fn` at `threads` threads per group, cached per
// (device, kernel).  The preload entry points (advdiff_preload_*) fill the cache for the
// default kernels, so no launch inside a hipGraph capture is the first to ask; a failed
// query is not cached (1 is returned for that launch and the error cleared).
inline int occupancy_per_cu(const void* fn, int threads) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_pair(dev, fn);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, 0) != hipSuccess || nb < 1) {
    (void)hipGetLastError();
    return 1;
  }
  cache.emplace(key, nb);
  return nb;
}

// Chunking of the marched axis for a kernel whose workgroups each pay `warm` planes of
// pipeline warm-up: with `slots` workgroups resident at once (CUs x occupancy), a launch
// of tiles*C groups runs in ceil(tiles*C/slots) rounds of (ceil(n/C) + warm) planes.
// Pick the C in [1, n/minc] that minimises that estimate (fewer, longer chunks amortise
// the warm-up; the round quantisation decides the rest).
inline int pick_chunk_rounds(int n, long long tiles, long long slots, int warm, int minc) {
  if (n <= 0) return 1;
  long long best_cost = -1;
  int best = n;
  const int cmax = std::max(1, n / std::max(minc, 1));
  for (int C = 1; C <= cmax; ++C) {
    const long long len = (n + C - 1) / C;
    const long long rounds = (tiles * C + slots - 1) / slots;
    const long long cost = rounds * (len + warm);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = (int)len;
    }
  }
  return best;
}

// Tuning knobs read once from the environment (ADVDIFF_<NAME>), for A/B experiments
// inside one process; the defaults are the tuned gfx950 choices.
inline int knob(const char* name, int def) {
  char key[64];
  std::snprintf(key, sizeof(key), "ADVDIFF_%s", name);
  const char* v = std::getenv(key);
  return v ? std::atoi(v) : def;
}

}  // namespace advdiff
