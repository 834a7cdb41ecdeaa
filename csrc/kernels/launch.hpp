// Host-side launch helpers shared by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdint.h>

namespace advdiff {

// Number of workgroups we aim for per launch: 256 CUs x 8 resident groups.  A
// stencil launch needs >> 256 groups to fill the 8 XCDs (MI355X_MICROARCH.md,
// "Workgroup dispatch").
constexpr long long kTargetBlocks = 2048;

// Length of the marching chunk (planes per workgroup) so that the launch has at
// least kTargetBlocks groups while each group marches far enough to amortise the
// 2R-plane prologue of its register window.
inline int knob(const char* name, int def);

inline int pick_chunk(int nrange, long long xyblocks, int minc, int maxc) {
  if (nrange <= 0) return 1;
  static const long long target = knob("TARGET_BLOCKS", (int)kTargetBlocks);
  long long want_chunks = (target + xyblocks - 1) / std::max<long long>(xyblocks, 1);
  long long c = (nrange + want_chunks - 1) / std::max<long long>(want_chunks, 1);
  c = std::max<long long>(c, minc);
  c = std::min<long long>(c, maxc);
  return (int)std::max<long long>(c, 1);
}

inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

// Tuning knobs read once from the environment (ADVDIFF_<NAME>), for A/B experiments
// inside one process; the defaults are the tuned gfx950 choices.
inline int knob(const char* name, int def) {
  char key[64];
  std::snprintf(key, sizeof(key), "ADVDIFF_%s", name);
  const char* v = std::getenv(key);
  return v ? std::atoi(v) : def;
}

}  // namespace advdiff
