// Temporally blocked heat-equation kernel: ONE launch = one FULL SSP-RK3 step.
//
// The per-stage kernels (diffusion.hip) move 64 B of HBM traffic per cell and step
// (stage 1: 16 B, stages 2/3: 24 B each) and run at the HBM roof.  This kernel keeps the
// two intermediate stage fields on chip and moves 16 B per cell and step (read u^n once,
// write u^{n+1} once) — the reference has no counterpart; it is the MI355X-first answer
// to a memory-bound stencil (SURVEY.md §2.5 "temporal blocking / wide halos").
//
// Overlapped (trapezoidal) tiling in x/y, a software pipeline in z:
//   * A workgroup = NW waves.  Lane c of a wave is x = i0 - 2R + c (64 columns: one wave
//     = one row of the stage-1 region); wave w owns region rows w, w+NW, ... (RPW rows).
//   * Regions:  S1 (stage 1) = 64 x (TY+4R) points,  S2 = S1 shrunk by R,  S3 (outputs)
//     = S1 shrunk by 2R = (64-4R) x TY.  Redundant stage-1/2 evaluations on the S1/S2
//     rims replace any inter-workgroup communication.
//   * z pipeline: iteration k computes A(k+2R) on S1, B(k+R) on S2 and u^{n+1}(k) on S3.
//     z-neighbours live in per-thread register windows u(k..k+3R), A(k..k+2R),
//     B(k-R..k+R); x/y neighbours come from three double-buffered LDS planes
//     (u(k+2R) incl. an R-cell rim, A(k+R), B(k)) written at the top of the iteration,
//     so ONE barrier per plane orders everything.
//   * Frozen Dirichlet cells (outside the interior box / planes [zlo, zhi)) carry
//     A = B = u, exactly as the per-stage path (whose A/B buffers keep the IC there).
// Every arithmetic step uses the shared fma helpers of common.hpp, so the result is
// BIT-IDENTICAL to three per-stage launches (tests/test_fused_step_gpu.py).
#include "common.hpp"
#include "launch.hpp"
#include "advdiff/kernels.h"

#include <cstdio>
#include <map>
#include <atomic>
#include <mutex>
#include <queue>
#include <tuple>
#include <utility>
#include <vector>

namespace advdiff {

// x/y bounds of a fused-step launch (view coordinates): cells outside [xa0,xa1) x
// [ya0,ya1) are frozen (A = B = u there, never written); u^{n+1} is written on the active
// cells inside [xo0,xo1) x [yo0,yo1).  Slab layout: active = [border, n-border), output =
// everything; Cartesian blocks: active = the global interior seen through the view,
// output = the block (3R inside the view on split axes).
struct Box2 {
  int xa0, xa1, ya0, ya1, xo0, xo1, yo0, yo1;
};

// Work split of a launch: blockIdx -> (x tile, y tile, z chunk of `zchunk` planes; chunks
// z >= gza belong to the second plane range), as many rounds of resident groups as the
// grid needs — the dispatcher balances the load dynamically.  (A persistent schedule —
// one round of groups each marching an equal share of the linearised (tile, plane) space
// — measured 9-11 % slower at 512^3 and was removed: profiles/archive/step_variants_r2.log.  Uneven
// XCD-balanced chunk lengths gained 1.4 % at 512^3 but lost 6-13 % at other sizes and for
// FD2: profiles/split_ab_r3.log, split_sizes_r3.log.)
struct StepSched {
  int gx, gy;       // tiles along x / y
  int gza, zchunk;  // chunks of the first range, planes per chunk
  int edge;         // v3: boundary-anchored edge tiles (axis_tile)
  int zfirst = 0;   // banded schedule (> 0): a 1-D grid of gza bands x gx gy tiles, band 0
                    // of zfirst planes, the others of zchunk (one range only)
};

// Tile placement along one axis of the v3 march (span W = 64 lanes in x, S1R rows in y;
// interior tiles output W - 4R cells, lanes/rows [2R, W-2R)).  Tiles cover the output
// range [P0, P1) = [o0,o1) ∩ [a0,a1) of the launch.  Edge tiles (edge = 1): when P0 is
// the active range's own start a0 (a Dirichlet boundary — the R cells below it are
// frozen, so their stage-1/2 values are exact copies of u), the first tile is anchored
// with its lanes [0,R) on those frozen cells and outputs [R, W-2R): R more cells than an
// interior tile; likewise the last tile at a1.  At 512^3 FD4 this takes 9 x 18 instead
// of 10 x 19 tiles (-15 % stage-1/2/3 work).  The last tile is anchored at P1 and writes
// only from wlo, where the previous tile stopped, so every cell has exactly one writer.
// edge = 0: the same partition without the R-cell extensions (the pre-edge layout).
struct AxisTile {
  int org;      // coordinate of lane / row 0
  int lo, hi;   // stage-3 (output) lanes / rows [lo, hi)
  int wlo;      // first coordinate this tile writes
};

struct AxisSpan {
  int p0, p1, lol, hir;
};
// SH: the output shrink of an interior tile side (2R for the 3-stage step, 5R for the
// two-step 6-stage kernel); an edge tile anchored on frozen Dirichlet cells shrinks by R.
__host__ __device__ inline AxisSpan axis_span(int W, int R, int a0, int a1, int o0, int o1,
                                              int nmax, int edge, int SH) {
  AxisSpan s;
  s.p0 = o0 > a0 ? o0 : a0;
  s.p1 = o1 < a1 ? o1 : a1;
  const bool el = edge && s.p0 == a0 && a0 - R >= 0;
  const bool er = edge && s.p1 == a1 && a1 + R <= nmax;
  s.lol = el ? R : SH;
  s.hir = er ? W - R : W - SH;
  return s;
}

__host__ __device__ inline int axis_tile_count(int W, int R, int a0, int a1, int o0, int o1,
                                               int nmax, int edge, int SH) {
  const AxisSpan s = axis_span(W, R, a0, a1, o0, o1, nmax, edge, SH);
  const int L = s.p1 - s.p0, TO = W - 2 * SH;
  if (L <= s.hir - s.lol) return 1;
  const int rest = L - (W - SH - s.lol) - (s.hir - SH);
  return 2 + (rest > 0 ? (rest + TO - 1) / TO : 0);
}
__host__ __device__ inline int axis_tile_count(int W, int R, int a0, int a1, int o0, int o1,
                                               int nmax, int edge) {
  return axis_tile_count(W, R, a0, a1, o0, o1, nmax, edge, 2 * R);
}

__device__ __forceinline__ AxisTile axis_tile(int t, int n, int W, int R, int a0, int a1,
                                              int o0, int o1, int nmax, int edge, int SH) {
  const AxisSpan s = axis_span(W, R, a0, a1, o0, o1, nmax, edge, SH);
  const int TO = W - 2 * SH;
  const int e0 = s.p0 + (W - SH - s.lol);  // end of tile 0's outputs
  AxisTile a;
  a.lo = t == 0 ? s.lol : SH;
  a.hi = t == n - 1 ? s.hir : W - SH;
  if (t == 0) {
    a.org = s.p0 - s.lol;
    a.wlo = s.p0;
  } else if (t == n - 1) {
    a.org = s.p1 - s.hir;
    a.wlo = e0 + (t - 1) * TO;
  } else {
    a.wlo = e0 + (t - 1) * TO;
    a.org = a.wlo - SH;
  }
  return a;
}
__device__ __forceinline__ AxisTile axis_tile(int t, int n, int W, int R, int a0, int a1,
                                              int o0, int o1, int nmax, int edge) {
  return axis_tile(t, n, W, R, a0, a1, o0, o1, nmax, edge, 2 * R);
}

// Fused halo puts (slab ranks, ipc transport; common.hpp HaloPut): the exchange rides
// inside the step launch over xGMI instead of a boundary launch plus a put launch after it.
using StepPut = HaloPut;

// ---------------------------------------------------------------------------------
// v3 march: the same algorithm (compact rings, trapezoid, one barrier per plane) with
// the code shaped for the gfx950 issue model:
//   * the wave index is made scalar (readfirstlane), so every per-row condition is a
//     scalar branch and never an exec-mask region;
//   * ONE shared LDS block (U0 U1 | A0 A1 B0 B1) and one base VGPR per row and plane
//     kind: every neighbour, the buffer set and the A->B distance are immediate
//     ds_read/ds_write offsets (the march is unrolled 2 NR times, so the set is static);
//   * stage 1 reads its x and y neighbours from the haloed u plane (no divergent edge
//     lanes); stages 2/3 take y from LDS and x by DPP (XS = 1) or LDS (XS = 0);
//   * global traffic uses a scalar plane base + a 32-bit per-lane byte offset (saddr
//     form: no 64-bit VALU address math in the march);
//   * PF: prefetch distance in planes (1 or 2).
// The arithmetic (fd_ctr / fd4_axis / fd2_axis in the fixed order centre, z, x, y) is
// that of the per-stage kernels, so the step is bit-identical to three stage launches.
// (The round-1 "compact ring" march with per-iteration LDS pointers and the 8-slot ring
// kernels were removed after their A/Bs: profiles/kbench_fused_*.log, step_cfgs_*.)
// ---------------------------------------------------------------------------------
template <typename T, int ORDER, int NW, int RPW>
struct V3Geom {
  static constexpr int R = FD<ORDER>::R;
  static constexpr int W = 64;
  static constexpr int S1R = NW * RPW;
  static constexpr int UW = W + 2 * R, UH = S1R + 2 * R;
  static constexpr int USET = UH * UW;             // elements per u plane buffer
  static constexpr int ASET = S1R * W + 2 * R;      // A/B plane buffer (+R pad each side)
  static constexpr int OFF_A = 2 * USET;            // element offset of A0 in the block
  static constexpr int OFF_B = OFF_A + 2 * ASET;    // B0
  static constexpr int TOTAL = OFF_B + 2 * ASET + R * W;  // + pad: PAIR reads past B1
};

// VAR = PRIO + 4 DEFER + 16 PAIR (round 3 A/B of the barrier-synchronised phases; PAIR:
// each wave owns RPW adjacent rows, see row_of).  PRIO: which
// waves run at a raised s_setprio (0 none, 1 the second half, 2 the "busy" waves whose
// rows all carry three stages, 3 graded by the wave's row-stage count: the busiest at 2,
// one row-stage less at 1).  DEFER: which waves DEFER the arithmetic and the store of their
// stage 3 by one plane (0 none, 1 the second half, 2 the non-busy waves): such a wave
// reads the stage's LDS neighbours (as their y-axis sum) before the next barrier and
// computes right after it, while the others start the plane with their stage-1 LDS reads
// — LDS traffic and VALU work of the two groups overlap instead of alternating in lockstep
// (MI355X_MICROARCH.md "Two waves per SIMD", items 4 and 9).  Same arithmetic, bit-
// identical results.
template <typename T, int ORDER, int NW, int RPW, int XS, int PF, bool SEP, int VAR = 0,
          bool PUT = false>
__device__ __forceinline__ void v3_march(
    T* lds, int tx, int ty, int gx, int gy, int edge, int kc0, int kc1,
    const T* __restrict__ uin, T* __restrict__ uout, int nx, int ny, int64_t sy, int64_t sz,
    int nz_alloc, int zlo, int zhi, const Box2& bx, const FdCoef<T>& q1a, const FdCoef<T>& q2a,
    const FdCoef<T>& q3a, const StepPut& put = StepPut{}) {
  // fp64: the stage-1 coefficients live in VGPRs (a "+v" asm operand makes the uniform
  // values look divergent; 8 more VGPRs, same occupancy).  With all twelve fp64
  // coefficients in SGPRs the kernel needs 106 SGPRs and the compiler spills them into
  // VGPR lanes: 20 v_readlane reloads per plane of the FD4 march (148 -> 128 VALU per
  // plane without them).  FD4 512^3 642 -> 614 us, bitwise the same (in-process A/B,
  // profiles/r5/ab/vcoef_ab.log; stage 3 instead of 1: the same).  fp32 keeps SGPRs (no
  // spill there, and 4 more VGPRs would cost the 16 x 2 tile its second workgroup per CU).
  FdCoef<T> q1 = q1a, q2 = q2a, q3 = q3a;
  auto to_v = [](FdCoef<T>& c) {
    asm volatile("" : "+v"(c.kc));
#pragma unroll
    for (int d = 0; d < 3; ++d) asm volatile("" : "+v"(c.k[d]));
  };
  if constexpr (sizeof(T) == 8) to_v(q1);
  using G = V3Geom<T, ORDER, NW, RPW>;
  constexpr int R = G::R, NR = 2 * R + 1, W = G::W, S1R = G::S1R, UW = G::UW, UH = G::UH;
  constexpr int TX = W - 4 * R, TY = S1R - 4 * R;
  constexpr int NT = 64 * NW;
  constexpr int NHALO = UW * UH - W * S1R;
  constexpr int NH = (NHALO + NT - 1) / NT;
  constexpr int E = (int)sizeof(T);
  constexpr int USETB = G::USET * E, ASETB = G::ASET * E, ABB = (G::OFF_B - G::OFF_A) * E;
  static_assert(TY > 0, "tile too small");
  // The A -> B plane distance rides in the 16-bit DS immediate together with the buffer
  // set offset; a tall tile (FD2 12 x 4: 48 rows) overflows it, and then the B planes get
  // base registers of their own (one more VGPR per row)
  constexpr bool SPLITB = ASETB + ABB + (2 * R * W + 2 * R) * E >= 65536;
  constexpr int ABI = SPLITB ? 0 : ABB;  // A -> B distance carried as an immediate
  static_assert(ASETB + ABI + (2 * R * W + 2 * R) * E < 65536, "A/B offsets must fit the 16-bit DS offset");
  static_assert(USETB + (2 * R * UW + 2 * R) * E < 65536, "u offsets must fit");

  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.y);
  const int tid = w * 64 + lane;
  static_assert(TX > 0, "tile too narrow");
  constexpr int PRIO = VAR % 4, DMODE = (VAR / 4) % 4;
  constexpr bool DEFER = DMODE != 0;
  // PAIR: the wave owns RPW ADJACENT rows (w RPW + q) instead of rows w + q NW, so the y
  // neighbours its rows share are read from LDS once and its own rows come from registers
  // (FD4 16 x 2: 8 -> 4 LDS reads per stage and wave; FD2 12 x 3: 6 -> 2)
  constexpr bool PAIR = VAR / 16 != 0;
  // (Round 3, rejected: issuing every LDS read of the plane right after the barrier,
  // before any stage's arithmetic — FD2 542.6 vs 537.8 us, FD4 spills at 128 VGPRs;
  // profiles/step_ab_hoist_r3.log.)
  auto row_of = [&](int q) { return PAIR ? w * RPW + q : w + q * NW; };
  // row-stages of the wave (1 + in S2 + in S3 per row); busy: all in S3
  int nst = 0;
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = row_of(q);
    nst += 1 + (row >= R && row < S1R - R) + (row >= 2 * R && row < S1R - 2 * R);
  }
  const bool busy = nst == 3 * RPW;
  const bool late = DMODE == 1 ? w >= NW / 2 : (DMODE == 2 ? !busy : false);  // scalar
  if constexpr (PRIO == 1) {
    if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (PRIO == 2) {
    if (busy) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (PRIO == 3) {
    if (busy)
      __builtin_amdgcn_s_setprio(2);
    else if (nst == 3 * RPW - 1)
      __builtin_amdgcn_s_setprio(1);
  }
  const AxisTile atx = axis_tile(tx, gx, W, R, bx.xa0, bx.xa1, bx.xo0, bx.xo1, nx, edge);
  const AxisTile aty = axis_tile(ty, gy, S1R, R, bx.ya0, bx.ya1, bx.yo0, bx.yo1, ny, edge);
  const int x = atx.org + lane;
  const bool xin = x >= bx.xa0 && x < bx.xa1;
  const bool xout = x >= max(bx.xo0, atx.wlo) && x < bx.xo1;
  const int ywlo = max(bx.yo0, aty.wlo);
  // lanes of a frozen edge column carry A = B = u, so s2c needs no edge case
  const bool s2c = lane >= R && lane < W - R;
  const bool s3c = lane >= atx.lo && lane < atx.hi;
  const int xc = clampi(x, 0, nx - 1);
  char* lb = (char*)lds;
  // SEP: a compiler memory fence before every LDS read keeps each one a separate
  // ds_read_b64 (2 LDS cycles per wave) instead of a merged ds_read2_b64 (8 cycles for
  // the same two values: half the LDS read throughput, MI355X_MICROARCH.md §LDS)
  auto ld = [&](int off) {
    if constexpr (SEP) asm volatile("" ::: "memory");
    return lds_ld<T>(lb, off);
  };

  // per row: global byte offset, LDS bases (u neighbourhood top-left; A own cell; A
  // neighbourhood top-left for stages 2/3), lane masks
  uint32_t goff[RPW];
  int ub[RPW], aw[RPW], ar[RPW], bw[RPW], br[RPW];
  bool m1[RPW], m2[RPW], m3[RPW];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = row_of(q);
    const int y = aty.org + row;
    const bool inxy = xin && y >= bx.ya0 && y < bx.ya1;
    m1[q] = inxy;
    m2[q] = inxy && s2c;
    m3[q] = inxy && xout && y >= ywlo && y < bx.yo1 && s3c;
    goff[q] = (uint32_t)(clampi(y, 0, ny - 1) * (int)sy + xc) * (uint32_t)E;
    ub[q] = (row * UW + lane) * E;                            // u(row-R+R.., lane-R+R..)
    aw[q] = (G::OFF_A + R + row * W + lane) * E;               // A own cell, set 0
    const int rc = clampi(row, R, S1R - R - 1);                 // in-bounds for masked rows
    ar[q] = (G::OFF_A + R + (rc - R) * W + lane - (XS ? 0 : R)) * E;
    bw[q] = aw[q] + (ABB - ABI);  // B own cell / B neighbourhood (set 0, minus ABI)
    br[q] = ar[q] + (ABB - ABI);
  }
  // PAIR: the wave's first row and its A/B-plane LDS base at row row0 - R (the lowest
  // row any of its y reads touches: immediates stay non-negative)
  const int row0 = w * RPW;
  const int apb = (G::OFF_A + R + (row0 - R) * W + lane) * E;
  (void)apb;
  uint32_t hoff[NH];
  int hl[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    int idx = tid + h * NT;
    hl[h] = -1;
    hoff[h] = 0;
    if (idx < NHALO) {
      int ur, uc;
      if (idx < R * UW) {
        ur = idx / UW;
        uc = idx - ur * UW;
      } else if ((idx -= R * UW) < R * UW) {
        ur = S1R + R + idx / UW;
        uc = idx % UW;
      } else {
        idx -= R * UW;
        ur = R + idx / (2 * R);
        const int cc = idx % (2 * R);
        uc = cc < R ? cc : W + cc;
      }
      hl[h] = (ur * UW + uc) * E;
      hoff[h] = (uint32_t)(clampi(aty.org - R + ur, 0, ny - 1) * (int)sy +
                           clampi(atx.org - R + uc, 0, nx - 1)) * (uint32_t)E;
    }
  }
  const int64_t szb = sz * E;
  auto plane = [&](int k) {  // buffer descriptor of plane k (clamped into the allocation)
    return plane_rsrc((const char*)uin + (int64_t)clampi(k, 0, nz_alloc - 1) * szb);
  };

  T ru[RPW][NR], ra[RPW][NR], rb[RPW][NR], dl[RPW][R];
  const int kst = kc0 - 4 * R;
  {
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
#pragma unroll
      for (int d = 0; d < R - 1; ++d) dl[q][d] = gld<T>(plane(kst + d), goff[q]);
#pragma unroll
      for (int s = 0; s < NR; ++s) {
        const int pl = kst + R - 1 + s;
        ru[q][pl - kst < NR ? pl - kst : pl - kst - NR] = gld<T>(plane(pl), goff[q]);
        ra[q][s] = rb[q][s] = T(0);
      }
    }
  }
  // prefetch ring: slot f holds the planes of iteration k + f (f < PF): un = own column
  // of u(k+f+3R) (enters the register ring), hv = the LDS rim of u(k+f+2R)
  T hv[PF][NH], un[PF][RPW];
#pragma unroll
  for (int f = 0; f < PF; ++f) {  // planes of iterations kst .. kst+PF-1
    const auto p2 = plane(kst + f + 2 * R);
    const auto p3 = plane(kst + f + 3 * R);
#pragma unroll
    for (int h = 0; h < NH; ++h) hv[f][h] = gld<T>(p2, hoff[h]);
#pragma unroll
    for (int q = 0; q < RPW; ++q) un[f][q] = gld<T>(p3, goff[q]);
  }
  const T third = T(1.0 / 3.0);

  // stage 3 of plane kp from its ingredients: centre, z, x (DPP) and the y-axis sum ys,
  // which comes from LDS (the normal path and the deferred one share it; the chain order
  // centre, z, x, y is the per-stage kernels', so results stay bit-identical)
  static_assert(XS, "stage 3 takes its x neighbours by DPP");
  auto s3_finish = [&](int q, int kp, T c, T uo, T zm2, T zm1, T zp1, T zp2, T ys) {
    T acc = fd_ctr(q3.kc, c, third * uo);
    if constexpr (R == 2) {
      acc = fd4_axis(acc, q3.k[2], zm2, zm1, zp1, zp2);
      const T xm1 = wave_shr1(c), xp1 = wave_shl1(c);
      const T xm2 = wave_shr1(xm1), xp2 = wave_shl1(xp1);
      acc = fd4_axis(acc, q3.k[0], xm2, xm1, xp1, xp2);
    } else {
      acc = fd2_axis(acc, q3.k[2], zm1, zp1);
      acc = fd2_axis(acc, q3.k[0], wave_shr1(c), wave_shl1(c));
    }
    acc = fd_apply(acc, q3.k[1], ys);
    acc = pin(acc);
    if (m3[q]) gst<T>(plane_rsrc((char*)uout + (int64_t)kp * szb), goff[q], acc);
    if constexpr (PUT) {
      // kp and the row are scalar: scalar branches
      if (m3[q]) halo_put<T>(put, kp, aty.org + row_of(q), goff[q], acc);
    }
  };
  // the y-axis sum of stage 3 from the B plane of buffer set AO (LDS)
  auto s3_ysum = [&](int q, int AO) {
    const int b = br[q] + AO + ABI;
    if constexpr (R == 2)
      return fd4_sum(ld(b + 0 * W * E), ld(b + 1 * W * E), ld(b + 3 * W * E), ld(b + 4 * W * E));
    else
      return fd2_sum(ld(b + 0 * E), ld(b + 2 * W * E));
  };
  // PAIR: the column of one plane over rows row0-R .. row0+RPW-1+R — the R rows on each
  // side from LDS (base + immediates; rows beyond the region read the U sets / the pad and
  // are used by no computed row), the wave's own rows from registers
  constexpr int NY = RPW + 2 * R;
  auto ywin = [&](T (&y)[NY], int base, int stride, const T* own) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      y[j] = ld(base + j * stride);
      y[R + RPW + j] = ld(base + (R + RPW + j) * stride);
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) y[R + q] = own[q];
  };
  // y-axis sum / axis term of row q from such a window (the same operands, the same order)
  auto ysum_w = [&](const T (&y)[NY], int q) {
    if constexpr (R == 2)
      return fd4_sum(y[q], y[q + 1], y[q + 3], y[q + 4]);
    else
      return fd2_sum(y[q], y[q + 2]);
  };
  auto yaxis_w = [&](T acc, T k, const T (&y)[NY], int q) {
    if constexpr (R == 2)
      return fd4_axis(acc, k, y[q], y[q + 1], y[q + 3], y[q + 4]);
    else
      return fd2_axis(acc, k, y[q], y[q + 2]);
  };
  // deferred stage 3 (late waves, DEFER): the y sum and u^n of the plane, kept in registers
  // across the barrier
  T dys[RPW], duo[RPW];
  (void)dys;
  (void)duo;

  // PH in [0, 2 NR): ring slots and the LDS buffer set (PH & 1) are compile-time.
  // k == kc1 (DEFER only): a pseudo iteration without a top and a barrier that completes
  // the late waves' last deferred stage 3.
  auto body = [&]<int PH>(int k) {
    auto sl = [](int d) { return (PH + d + 4 * NR) % NR; };
    constexpr int UIN = (PH + 3 * R) % NR;
    constexpr int SET = PH & 1;
    constexpr int UO = SET * USETB, AO = SET * ASETB;
    constexpr int PF0 = PH % PF;
    const bool real = !DEFER || k < kc1;  // scalar
    if (real) {
      // ---- top: new u plane enters the ring; LDS planes u(k+2R), A(k+R), B(k) ----
      // the prefetch ring (PF slots) and the delay line (R slots) rotate by renaming:
      // iteration PH consumes prefetch slot PF0 and refills it with plane k+PF
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        dl[q][(PH + R - 1) % R] = ru[q][UIN];
        ru[q][UIN] = un[PF0][q];
        lds_st<T>(lb, ub[q] + UO + (R * UW + R) * E, ru[q][sl(2 * R)]);
        lds_st<T>(lb, aw[q] + AO, ra[q][sl(R)]);
        lds_st<T>(lb, bw[q] + AO + ABI, rb[q][sl(0)]);
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)  // the rim of u(k+2R)
        if (hl[h] >= 0) lds_st<T>(lb, hl[h] + UO, hv[PF0][h]);
      {
        const auto p2 = plane(k + PF + 2 * R);
        const auto p3 = plane(k + PF + 3 * R);
#pragma unroll
        for (int h = 0; h < NH; ++h) hv[PF0][h] = gld<T>(p2, hoff[h]);
#pragma unroll
        for (int q = 0; q < RPW; ++q) un[PF0][q] = gld<T>(p3, goff[q]);
      }
      __syncthreads();
    }
    if constexpr (DEFER) {
      // the late half opens the plane with the previous plane's stage-3 arithmetic (no
      // LDS): B(k-1) and its z neighbours are still in the ring (stage 2 of this plane
      // overwrites them only below)
      if (late && k - 1 >= kc0) {
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
          const int row = row_of(q);
          if (row < aty.lo || row >= aty.hi) continue;  // scalar branch
          s3_finish(q, k - 1, rb[q][sl(-1)], duo[q], rb[q][sl(-3)], rb[q][sl(-2)],
                    rb[q][sl(0)], rb[q][sl(1)], dys[q]);
        }
      }
      if (!real) return;
    }
    // ---- stage 1: A(k+2R) on S1 ----
    const int pz1 = k + 2 * R;
    const bool z1 = pz1 >= zlo && pz1 < zhi;
    T yu[NY], ya[NY], yb[NY];
    const bool ws2 = row0 + RPW > R && row0 < S1R - R;         // scalar: a row in S2
    const bool ws3 = k >= kc0 && row0 + RPW > aty.lo && row0 < aty.hi;  // a row in S3
    if constexpr (PAIR) {
      T own[RPW];
#pragma unroll
      for (int q = 0; q < RPW; ++q) own[q] = ru[q][sl(2 * R)];
      ywin(yu, ub[0] + UO + R * E, UW * E, own);
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int b = ub[q] + UO;
      const T c = ru[q][sl(2 * R)];
      T acc = fd_ctr(q1.kc, c);
      if constexpr (R == 2) {
        acc = fd4_axis(acc, q1.k[2], ru[q][sl(R)], ru[q][sl(R + 1)], ru[q][sl(3 * R - 1)],
                       ru[q][sl(3 * R)]);
        acc = fd4_axis(acc, q1.k[0], ld(b + (2 * UW + 0) * E),
                       ld(b + (2 * UW + 1) * E), ld(b + (2 * UW + 3) * E),
                       ld(b + (2 * UW + 4) * E));
        if constexpr (PAIR)
          acc = yaxis_w(acc, q1.k[1], yu, q);
        else
          acc = fd4_axis(acc, q1.k[1], ld(b + (0 * UW + 2) * E),
                         ld(b + (1 * UW + 2) * E), ld(b + (3 * UW + 2) * E),
                         ld(b + (4 * UW + 2) * E));
      } else {
        acc = fd2_axis(acc, q1.k[2], ru[q][sl(R)], ru[q][sl(3 * R)]);
        acc = fd2_axis(acc, q1.k[0], ld(b + (UW + 0) * E),
                       ld(b + (UW + 2) * E));
        if constexpr (PAIR)
          acc = yaxis_w(acc, q1.k[1], yu, q);
        else
          acc = fd2_axis(acc, q1.k[1], ld(b + 1 * E), ld(b + (2 * UW + 1) * E));
      }
      acc = pin(acc);
      ra[q][sl(2 * R)] = (z1 && m1[q]) ? acc : c;
    }
    // ---- stage 2: B(k+R) on S2 ----
    if (k >= kc0 - 2 * R) {
      const int pz2 = k + R;
      const bool z2 = pz2 >= zlo && pz2 < zhi;
      if constexpr (PAIR) {
        if (ws2) {  // scalar: a row of the wave is in S2
          T own[RPW];
#pragma unroll
          for (int q = 0; q < RPW; ++q) own[q] = ra[q][sl(R)];
          ywin(ya, apb + AO, W * E, own);
        }
      }
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int row = row_of(q);
        const T uo = ru[q][sl(R)];
        if (row < R || row >= S1R - R) {  // scalar branch
          rb[q][sl(R)] = uo;
          continue;
        }
        const int b = ar[q] + AO;
        const T c = ra[q][sl(R)];
        T acc = fd_ctr(q2.kc, c, T(0.75) * uo);
        constexpr int XC = XS ? 0 : R;  // column of the centre relative to the base
        if constexpr (R == 2) {
          acc = fd4_axis(acc, q2.k[2], ra[q][sl(0)], ra[q][sl(1)], ra[q][sl(3)], ra[q][sl(4)]);
          T xm2, xm1, xp1, xp2;
          if constexpr (XS) {
            xm1 = wave_shr1(c);
            xp1 = wave_shl1(c);
            xm2 = wave_shr1(xm1);
            xp2 = wave_shl1(xp1);
          } else {
            xm2 = ld(b + (2 * W + 0) * E);
            xm1 = ld(b + (2 * W + 1) * E);
            xp1 = ld(b + (2 * W + 3) * E);
            xp2 = ld(b + (2 * W + 4) * E);
          }
          acc = fd4_axis(acc, q2.k[0], xm2, xm1, xp1, xp2);
          if constexpr (PAIR)
            acc = yaxis_w(acc, q2.k[1], ya, q);
          else
            acc = fd4_axis(acc, q2.k[1], ld(b + (0 * W + XC) * E),
                           ld(b + (1 * W + XC) * E), ld(b + (3 * W + XC) * E),
                           ld(b + (4 * W + XC) * E));
        } else {
          acc = fd2_axis(acc, q2.k[2], ra[q][sl(0)], ra[q][sl(2)]);
          T xm1, xp1;
          if constexpr (XS) {
            xm1 = wave_shr1(c);
            xp1 = wave_shl1(c);
          } else {
            xm1 = ld(b + (W + 0) * E);
            xp1 = ld(b + (W + 2) * E);
          }
          acc = fd2_axis(acc, q2.k[0], xm1, xp1);
          if constexpr (PAIR)
            acc = yaxis_w(acc, q2.k[1], ya, q);
          else
            acc = fd2_axis(acc, q2.k[1], ld(b + XC * E),
                           ld(b + (2 * W + XC) * E));
        }
        acc = pin(acc);
        rb[q][sl(R)] = (z2 && m2[q]) ? acc : uo;
      }
    }
    // ---- stage 3: u^{n+1}(k) on S3 (late waves: LDS reads now, arithmetic next plane) ----
    if (k >= kc0) {
      if constexpr (PAIR) {
        if (ws3) {  // scalar: a row of the wave is in S3
          T own[RPW];
#pragma unroll
          for (int q = 0; q < RPW; ++q) own[q] = rb[q][sl(0)];
          ywin(yb, apb + (ABB - ABI) + AO + ABI, W * E, own);
        }
      }
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int row = row_of(q);
        if (row < aty.lo || row >= aty.hi) continue;  // scalar branch
        T ys;
        if constexpr (PAIR)
          ys = ysum_w(yb, q);
        else
          ys = s3_ysum(q, AO);
        if (DEFER && late) {
          dys[q] = ys;
          duo[q] = dl[q][PH % R];
        } else {
          s3_finish(q, k, rb[q][sl(0)], dl[q][PH % R], rb[q][sl(-2)], rb[q][sl(-1)],
                    rb[q][sl(1)], rb[q][sl(2)], ys);
        }
      }
    }
  };
  static_assert((2 * NR) % PF == 0 && (2 * NR) % R == 0, "ring phases must repeat");

  // the LDS set of iteration k is (k - kst) & 1: unroll 2 NR so it is static
  const int kend = kc1 + (DEFER ? 1 : 0);
  for (int kb = kst; kb < kend; kb += 2 * NR) {
    [&]<int... P>(std::integer_sequence<int, P...>) {
      (void)((kb + P < kend ? (body.template operator()<P>(kb + P), true) : false) && ...);
    }(std::make_integer_sequence<int, 2 * NR>{});
  }
  // every peer store of this wave acknowledged before the wave (and the dispatch) ends
  if constexpr (PUT) __builtin_amdgcn_s_waitcnt(0);
}

// ---------------------------------------------------------------------------------
// TWO SSP-RK3 steps in one launch, 7-point (FD2) Laplacian: six stages on chip
// (A, B, U1 = u^{n+1}, C, D, U2 = u^{n+2}), u^n read once and u^{n+2} written once —
// 8 B of HBM traffic per cell and step instead of 16.  The FD2 step is the lighter one
// (about a third of the FD4 step's VALU work per cell, 79 % of the copy rate at one step
// per launch: profiles/roofline.md), so it has the VALU headroom to trade: the trapezoid
// rims grow from 2R to 5R per side (the x/y tile outputs 54 x (S1R - 10) of 64 x S1R), and
// the z warm-up from 4R to 10R planes.
// Iteration k of the z march: A(k+5), B(k+4), U1(k+3), C(k+2), D(k+1), U2(k) (R = 1).
// Register rings of 4 slots per plane kind (u k+3..k+6, A k+2..k+5, B k+1..k+4, U1 k..k+3,
// C k-1..k+2, D k-2..k+1), the march unrolled by 4 so every slot and the LDS buffer set
// (k & 1) are static; six double-buffered LDS planes (u with its rim for stage 1's x/y
// neighbours; A, B, U1, C, D for the y neighbours of the stages they feed — x comes from
// the wave's own lanes by DPP) written at the top of the iteration: one barrier per plane.
// The arithmetic is the per-stage kernels' (fd_ctr, fd2_axis / fd_apply in the order
// centre, z, x, y; stage bases a u^n with u^n = U1 for the second step), so two steps
// of this kernel equal two launches of the one-step kernel — and six stage launches —
// bit for bit (tests/test_fused_step_gpu.py).
// ---------------------------------------------------------------------------------
template <typename T, int NW, int RPW>
struct V6Geom {
  static constexpr int R = 1, W = 64, S1R = NW * RPW;
  static constexpr int UW = W + 2 * R, UH = S1R + 2 * R;
  static constexpr int USET = UH * UW;
  static constexpr int ASET = S1R * W + 2 * W;    // + one pad row above and below
  static constexpr int OFF_P = 2 * USET;            // first of the 5 x 2 A-type planes
  static constexpr int TOTAL = OFF_P + 10 * ASET;
};

template <typename T, int NW, int RPW>
__device__ __forceinline__ void v6_march(
    T* lds, int tx, int ty, int gx, int gy, int edge, int kc0, int kc1,
    const T* __restrict__ uin, T* __restrict__ uout, int nx, int ny, int64_t sy, int64_t sz,
    int nz_alloc, int zlo, int zhi, const Box2& bx, const FdCoef<T>& q1a, const FdCoef<T>& q2,
    const FdCoef<T>& q3) {
  // fp64: stage-1 coefficients in VGPRs, as in v3_march (no SGPR spill reloads)
  FdCoef<T> q1 = q1a;
  if constexpr (sizeof(T) == 8) {
    asm volatile("" : "+v"(q1.kc));
#pragma unroll
    for (int d = 0; d < 3; ++d) asm volatile("" : "+v"(q1.k[d]));
  }
  using G = V6Geom<T, NW, RPW>;
  constexpr int R = 1, W = G::W, S1R = G::S1R, UW = G::UW, UH = G::UH, NR = 4, PF = 2;
  constexpr int SH = 5 * R;  // interior output shrink per side
  constexpr int NT = 64 * NW;
  constexpr int NHALO = UW * UH - W * S1R;
  constexpr int NH = (NHALO + NT - 1) / NT;
  constexpr int E = (int)sizeof(T);
  constexpr int USETB = G::USET * E, ASETB = G::ASET * E;
  static_assert(S1R - 2 * SH > 0, "tile too small");
  static_assert(USETB + (2 * UW + 2) * E < 65536 && ASETB + 2 * W * E < 65536,
                "LDS immediates must fit the 16-bit DS offset");

  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.y);
  const int tid = w * 64 + lane;
  const AxisTile atx = axis_tile(tx, gx, W, R, bx.xa0, bx.xa1, bx.xo0, bx.xo1, nx, edge, SH);
  const AxisTile aty = axis_tile(ty, gy, S1R, R, bx.ya0, bx.ya1, bx.yo0, bx.yo1, ny, edge, SH);
  const int x = atx.org + lane;
  const bool xin = x >= bx.xa0 && x < bx.xa1;
  const bool xout = x >= max(bx.xo0, atx.wlo) && x < bx.xo1 && lane >= atx.lo && lane < atx.hi;
  const int ywlo = max(bx.yo0, aty.wlo);
  const int xc = clampi(x, 0, nx - 1);
  char* lb = (char*)lds;
  auto ld = [&](int off) {
    asm volatile("" ::: "memory");  // keep every LDS read a separate ds_read_b64
    return lds_ld<T>(lb, off);
  };

  uint32_t goff[RPW];
  int ub[RPW], pb[RPW];
  bool m1[RPW], m6[RPW];
  int rowq[RPW];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = w + q * NW;  // rows interleaved over the waves
    rowq[q] = row;
    const int y = aty.org + row;
    const bool inxy = xin && y >= bx.ya0 && y < bx.ya1;
    m1[q] = inxy;
    m6[q] = inxy && xout && y >= ywlo && y < bx.yo1 && row >= aty.lo && row < aty.hi;
    goff[q] = (uint32_t)(clampi(y, 0, ny - 1) * (int)sy + xc) * (uint32_t)E;
    ub[q] = (row * UW + lane) * E;                      // u: top-left of the 3x3 window
    pb[q] = (G::OFF_P + W + row * W + lane) * E;        // A-type plane 0, set 0: own cell
  }
  // rows of stage s (1..6) of this tile: [min((s-1)R, lo), max(S1R-(s-1)R, hi)) — an
  // anchored edge tile computes every stage from its first output row
  auto srow = [&](int s, int row) {
    const int lo = min((s - 1) * R, aty.lo), hi = max(S1R - (s - 1) * R, aty.hi);
    return row >= lo && row < hi;
  };
  uint32_t hoff[NH];
  int hl[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    int idx = tid + h * NT;
    hl[h] = -1;
    hoff[h] = 0;
    if (idx < NHALO) {
      int ur, uc;
      if (idx < R * UW) {
        ur = idx / UW;
        uc = idx - ur * UW;
      } else if ((idx -= R * UW) < R * UW) {
        ur = S1R + R + idx / UW;
        uc = idx % UW;
      } else {
        idx -= R * UW;
        ur = R + idx / (2 * R);
        const int cc = idx % (2 * R);
        uc = cc < R ? cc : W + cc;
      }
      hl[h] = (ur * UW + uc) * E;
      hoff[h] = (uint32_t)(clampi(aty.org - R + ur, 0, ny - 1) * (int)sy +
                           clampi(atx.org - R + uc, 0, nx - 1)) * (uint32_t)E;
    }
  }
  const int64_t szb = sz * E;
  auto plane = [&](int k) {
    return plane_rsrc((const char*)uin + (int64_t)clampi(k, 0, nz_alloc - 1) * szb);
  };

  // rings, slot of plane p = (p - kst) % NR
  T ru[RPW][NR], ra[RPW][NR], rb[RPW][NR], r1[RPW][NR], rc[RPW][NR], rd[RPW][NR];
  const int kst = kc0 - 10 * R;
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
#pragma unroll
    for (int s = 0; s < NR; ++s) ra[q][s] = rb[q][s] = r1[q][s] = rc[q][s] = rd[q][s] = T(0);
    // u(kst+3..kst+5) into slots 3, 0, 1 (u(kst+6) arrives at the top of iteration kst)
    ru[q][3] = gld<T>(plane(kst + 3), goff[q]);
    ru[q][0] = gld<T>(plane(kst + 4), goff[q]);
    ru[q][1] = gld<T>(plane(kst + 5), goff[q]);
    ru[q][2] = T(0);
  }
  T hv[PF][NH], un[PF][RPW];
#pragma unroll
  for (int f = 0; f < PF; ++f) {
    const auto p5 = plane(kst + f + 5);
    const auto p6 = plane(kst + f + 6);
#pragma unroll
    for (int h = 0; h < NH; ++h) hv[f][h] = gld<T>(p5, hoff[h]);
#pragma unroll
    for (int q = 0; q < RPW; ++q) un[f][q] = gld<T>(p6, goff[q]);
  }
  const T third = T(1.0 / 3.0), tq = T(0.75);

  auto body = [&]<int PH>(int k) {
    auto sl = [](int d) { return (PH + d + 4 * NR) % NR; };  // slot of plane k + d
    constexpr int SET = PH & 1;
    constexpr int UO = SET * USETB, AO = SET * ASETB;
    constexpr int PF0 = PH % PF;
    constexpr int PA = 0, PB_ = 2 * ASETB, PU = 4 * ASETB, PC = 6 * ASETB, PD = 8 * ASETB;
    // ---- top: u(k+6) enters the ring; LDS planes u(k+5) (+ rim), A(k+4), B(k+3),
    //      U1(k+2), C(k+1), D(k) ----
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      ru[q][sl(6)] = un[PF0][q];
      lds_st<T>(lb, ub[q] + UO + (R * UW + R) * E, ru[q][sl(5)]);
      lds_st<T>(lb + PA, pb[q] + AO, ra[q][sl(4)]);
      lds_st<T>(lb + PB_, pb[q] + AO, rb[q][sl(3)]);
      lds_st<T>(lb + PU, pb[q] + AO, r1[q][sl(2)]);
      lds_st<T>(lb + PC, pb[q] + AO, rc[q][sl(1)]);
      lds_st<T>(lb + PD, pb[q] + AO, rd[q][sl(0)]);
    }
#pragma unroll
    for (int h = 0; h < NH; ++h)
      if (hl[h] >= 0) lds_st<T>(lb, hl[h] + UO, hv[PF0][h]);
    {
      const auto p5 = plane(k + PF + 5);
      const auto p6 = plane(k + PF + 6);
#pragma unroll
      for (int h = 0; h < NH; ++h) hv[PF0][h] = gld<T>(p5, hoff[h]);
#pragma unroll
      for (int q = 0; q < RPW; ++q) un[PF0][q] = gld<T>(p6, goff[q]);
    }
    __syncthreads();

    auto zin = [&](int p) { return p >= zlo && p < zhi; };
    // y neighbours of an A-type plane (base offset PL) at row q
    auto ysum = [&](const char* base, int q) {
      return fd2_sum(lds_ld<T>(base, pb[q] + AO - W * E), lds_ld<T>(base, pb[q] + AO + W * E));
    };
    // ---- stage 1: A(k+5) from u(k+5) (x, y from the LDS u plane with its rim) ----
    {
      const bool zv = zin(k + 5);
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int b = ub[q] + UO;
        const T c = ru[q][sl(5)];
        T acc = fd_ctr(q1.kc, c);
        acc = fd2_axis(acc, q1.k[2], ru[q][sl(4)], ru[q][sl(6)]);
        acc = fd2_axis(acc, q1.k[0], ld(b + (UW + 0) * E), ld(b + (UW + 2) * E));
        acc = fd2_axis(acc, q1.k[1], ld(b + 1 * E), ld(b + (2 * UW + 1) * E));
        acc = pin(acc);
        ra[q][sl(5)] = (zv && m1[q]) ? acc : c;
      }
    }
    // ---- stage 2: B(k+4) from A(k+4) ----
    if (k >= kc0 - 8 * R) {
      const bool zv = zin(k + 4);
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const T uo = ru[q][sl(4)];
        if (!srow(2, rowq[q])) {  // scalar branch
          rb[q][sl(4)] = uo;
          continue;
        }
        const T c = ra[q][sl(4)];
        T acc = fd_ctr(q2.kc, c, tq * uo);
        acc = fd2_axis(acc, q2.k[2], ra[q][sl(3)], ra[q][sl(5)]);
        acc = fd2_axis(acc, q2.k[0], wave_shr1(c), wave_shl1(c));
        acc = fd_apply(acc, q2.k[1], ysum(lb + PA, q));
        acc = pin(acc);
        rb[q][sl(4)] = (zv && m1[q]) ? acc : uo;
      }
    }
    // ---- stage 3: U1(k+3) = u^{n+1} from B(k+3) ----
    if (k >= kc0 - 6 * R) {
      const bool zv = zin(k + 3);
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const T uo = ru[q][sl(3)];
        if (!srow(3, rowq[q])) {
          r1[q][sl(3)] = uo;
          continue;
        }
        const T c = rb[q][sl(3)];
        T acc = fd_ctr(q3.kc, c, third * uo);
        acc = fd2_axis(acc, q3.k[2], rb[q][sl(2)], rb[q][sl(4)]);
        acc = fd2_axis(acc, q3.k[0], wave_shr1(c), wave_shl1(c));
        acc = fd_apply(acc, q3.k[1], ysum(lb + PB_, q));
        acc = pin(acc);
        r1[q][sl(3)] = (zv && m1[q]) ? acc : uo;
      }
    }
    // ---- stage 4: C(k+2) from U1(k+2) (second step, stage 1) ----
    if (k >= kc0 - 4 * R) {
      const bool zv = zin(k + 2);
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const T c = r1[q][sl(2)];
        if (!srow(4, rowq[q])) {
          rc[q][sl(2)] = c;
          continue;
        }
        T acc = fd_ctr(q1.kc, c);
        acc = fd2_axis(acc, q1.k[2], r1[q][sl(1)], r1[q][sl(3)]);
        acc = fd2_axis(acc, q1.k[0], wave_shr1(c), wave_shl1(c));
        acc = fd_apply(acc, q1.k[1], ysum(lb + PU, q));
        acc = pin(acc);
        rc[q][sl(2)] = (zv && m1[q]) ? acc : c;
      }
    }
    // ---- stage 5: D(k+1) from C(k+1), base 3/4 U1(k+1) ----
    if (k >= kc0 - 2 * R) {
      const bool zv = zin(k + 1);
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const T uo = r1[q][sl(1)];
        if (!srow(5, rowq[q])) {
          rd[q][sl(1)] = uo;
          continue;
        }
        const T c = rc[q][sl(1)];
        T acc = fd_ctr(q2.kc, c, tq * uo);
        acc = fd2_axis(acc, q2.k[2], rc[q][sl(0)], rc[q][sl(2)]);
        acc = fd2_axis(acc, q2.k[0], wave_shr1(c), wave_shl1(c));
        acc = fd_apply(acc, q2.k[1], ysum(lb + PC, q));
        acc = pin(acc);
        rd[q][sl(1)] = (zv && m1[q]) ? acc : uo;
      }
    }
    // ---- stage 6: U2(k) = u^{n+2} from D(k), base 1/3 U1(k) -> global ----
    if (k >= kc0) {
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        if (rowq[q] < aty.lo || rowq[q] >= aty.hi) continue;  // scalar branch
        const T c = rd[q][sl(0)];
        T acc = fd_ctr(q3.kc, c, third * r1[q][sl(0)]);
        acc = fd2_axis(acc, q3.k[2], rd[q][sl(-1)], rd[q][sl(1)]);
        acc = fd2_axis(acc, q3.k[0], wave_shr1(c), wave_shl1(c));
        acc = fd_apply(acc, q3.k[1], ysum(lb + PD, q));
        acc = pin(acc);
        if (m6[q]) gst<T>(plane_rsrc((char*)uout + (int64_t)k * szb), goff[q], acc);
      }
    }
  };
  for (int kb = kst; kb < kc1; kb += NR) {
    [&]<int... P>(std::integer_sequence<int, P...>) {
      (void)((kb + P < kc1 ? (body.template operator()<P>(kb + P), true) : false) && ...);
    }(std::make_integer_sequence<int, NR>{});
  }
}

template <typename T, int NW, int RPW>
__global__ __launch_bounds__(64 * NW) void diffusion3d_step2x_kernel(
    const T* __restrict__ uin, T* __restrict__ uout, int nx, int ny, int64_t sy, int64_t sz,
    int nz_alloc, int k0, int k1, StepSched sc, int zlo, int zhi, Box2 bx, FdCoef<T> q1,
    FdCoef<T> q2, FdCoef<T> q3) {
  __shared__ T lds[V6Geom<T, NW, RPW>::TOTAL];
  const Tile3 tile = xcd_tile();
  const int kc0 = k0 + tile.z * sc.zchunk;
  const int kc1 = min(kc0 + sc.zchunk, k1);
  v6_march<T, NW, RPW>(lds, tile.x, tile.y, sc.gx, sc.gy, sc.edge, kc0, kc1, uin, uout, nx, ny,
                       sy, sz, nz_alloc, zlo, zhi, bx, q1, q2, q3);
}

// Waves per SIMD to budget registers for (fp64): as many workgroups as the LDS admits
// (FD4 16 waves: 1/CU -> 4; FD2 12 waves: 2/CU -> 6).  Without it the compiler spent 86
// VGPRs on the FD2 step and lost the second workgroup per CU (-25 %).
template <typename T, int ORDER, int NW, int RPW>
constexpr int step_min_waves() {
  constexpr int lds = (int)sizeof(T) * V3Geom<T, ORDER, NW, RPW>::TOTAL;
  constexpr int wgs = 163840 / lds;
  constexpr int w = wgs * NW / 4;
  return sizeof(T) == 8 ? (w > 8 ? 8 : (w < 1 ? 1 : w)) : 1;
}

// The march variant: DPP x neighbours in stages 2/3 (XS = 1), prefetch distance 2,
// unmerged LDS reads (SEP).  The other (XS, PF, SEP) combinations measured 1-9 % slower
// at 512^3 (profiles/archive/step_variants_r2.log, step_cfgs_edge_r2.log) and were removed.
template <typename T, int ORDER, int NW, int RPW, int VAR, bool PUT = false>
__global__ __launch_bounds__(64 * NW) __attribute__((
    amdgpu_waves_per_eu(step_min_waves<T, ORDER, NW, RPW>()))) void diffusion3d_step_kernel(
    const T* __restrict__ uin, T* __restrict__ uout, int nx, int ny, int64_t sy, int64_t sz,
    int nz_alloc, int k0, int k1, int k0b, int k1b, StepSched sc, int zlo, int zhi,
    Box2 bx, FdCoef<T> q1, FdCoef<T> q2, FdCoef<T> q3, StepPut put) {
  __shared__ T lds[V3Geom<T, ORDER, NW, RPW>::TOTAL];
  int kc0, kc1;
  Tile3 tile;
  if (sc.zfirst > 0) {  // banded: one long band, then short ones fill the last rounds
    tile = xcd_tile_banded(sc.gx * sc.gy, sc.gx);
    if constexpr (PUT) {
      // the long band at the TOP of the range: its workgroups store the upper face as
      // they end and the first short band's store the lower face as they start, so both
      // faces' puts run through the launch (bottom-up, the top band would be dispatched
      // last and bunch the upper peer's stores at the end)
      const int top = k1 - sc.zfirst;
      kc0 = tile.z == 0 ? top : k0 + (tile.z - 1) * sc.zchunk;
      kc1 = tile.z == 0 ? k1 : min(kc0 + sc.zchunk, top);
    } else {
      kc0 = k0 + (tile.z == 0 ? 0 : sc.zfirst + (tile.z - 1) * sc.zchunk);
      kc1 = min(kc0 + (tile.z == 0 ? sc.zfirst : sc.zchunk), k1);
    }
  } else {
    tile = xcd_tile();
    // z chunks of the first range [k0,k1), then (tile.z >= gza) of the second [k0b,k1b)
    const bool second = tile.z >= sc.gza;
    kc0 = second ? k0b + (tile.z - sc.gza) * sc.zchunk : k0 + tile.z * sc.zchunk;
    kc1 = min(kc0 + sc.zchunk, second ? k1b : k1);
  }
  v3_march<T, ORDER, NW, RPW, 1, 2, true, VAR, PUT>(lds, tile.x, tile.y, sc.gx, sc.gy, sc.edge,
                                                  kc0, kc1, uin, uout, nx, ny, sy, sz, nz_alloc,
                                                  zlo, zhi, bx, q1, q2, q3, put);
}

// Banded z schedule: with a whole number of z chunks per column the last round of
// resident workgroups is often part-empty (8-GPU slab rank, 1024 x 1024 x 116 interior
// planes, FD4: 817 columns x 2 chunks = 6.4 rounds of 256).  One long band of every
// column followed by short bands lets the dispatcher fill the last round with short
// workgroups; the band lengths come from a list-scheduling model of one XCD's slots
// (step_bands).  The model ignores L2 locality — workgroups of different bands run side
// by side at different z — and misjudges the memory-bound launches (bench/banded_ab.py,
// profiles/r5/ab/banded_ab.log: 512^3 FD4 +2.5 %, FD2 -10 %; 8-GPU slab rank FD2 +5.4 %;
// 1024 x 512 x 256 rank FD4 -4.2 %, FD2 +10.8 %), so it runs only where it was MEASURED
// faster for that launch (advdiff_diffusion3d_step_sched_pick, at solver / engine
// construction).  ADVDIFF_STEP_BANDED / advdiff_set_step_banded: -1 (default) the
// measured choice (uniform chunks for an unmeasured launch), 0 never, 1 always.  Results
// are bitwise the same for every chunking.
// process-wide setting (atomic: the C API is callable from any host thread); the pick's
// own forced schedule is THREAD-local, so a launch from another thread during a
// measurement keeps its own choice and a concurrent advdiff_set_step_banded survives
static std::atomic<int> g_step_banded{-2};
static thread_local int t_sched_force = -1;  // advdiff_diffusion3d_step_sched_pick only
static int step_banded() {
  int v = g_step_banded.load(std::memory_order_relaxed);
  if (v == -2) {
    int fresh = knob("STEP_BANDED", -1);
    g_step_banded.compare_exchange_strong(v, fresh);
    v = g_step_banded.load(std::memory_order_relaxed);
  }
  return v;
}

// Makespan, in plane-times, of `cols` columns cut into bands (first of `a` planes, then
// `nb` bands of `b`) on `slots` resident workgroups of one XCD, band-major dispatch to the
// earliest free slot; every workgroup also pays `warm` planes of pipeline fill.
static long long band_makespan(long long cols, int a, int nb, int b, int slots, int warm) {
  std::priority_queue<long long, std::vector<long long>, std::greater<long long>> t;
  for (int i = 0; i < std::max(slots, 1); ++i) t.push(0);
  long long end = 0;
  auto run = [&](int len, long long n) {
    for (long long i = 0; i < n; ++i) {
      const long long f = t.top() + len + warm;
      t.pop();
      t.push(f);
      end = std::max(end, f);
    }
  };
  run(a, cols);
  for (int q = 0; q < nb; ++q) run(b, cols);
  return end;
}

// (first band, later band length, number of bands) for n planes of `tiles` columns on
// `slots` resident workgroups (8 XCDs), minimising the model's makespan over uniform
// chunkings and one-long-band + uniform-short-band splits; cached per shape.
struct Bands {
  int zfirst, zchunk, nbands;
};
static Bands step_bands(int n, long long tiles, long long slots, int warm, int minc) {
  static std::mutex mu;
  static std::map<std::tuple<int, long long, long long, int, int>, Bands> cache;
  const auto key = std::make_tuple(n, tiles, slots, warm, minc);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const int xs = (int)std::max<long long>(slots / 8, 1);
  const long long cols = (tiles + 7) / 8;  // one XCD's share of every band
  Bands best{n, n, 1};
  long long bcost = -1;
  auto consider = [&](int a, int nb, int b) {
    const long long c = band_makespan(cols, a, nb, b, xs, warm);
    if (bcost < 0 || c < bcost) {
      bcost = c;
      best = {a, nb > 0 ? b : a, 1 + nb};
    }
  };
  const int cmax = std::max(1, n / std::max(minc, 1));
  for (int C = 1; C <= std::min(cmax, 16); ++C) {  // uniform chunks (as pick_chunk_rounds)
    const int len = (n + C - 1) / C;
    const int nb = (n - len + len - 1) / len;
    consider(len, nb, len);
  }
  const int step = std::max(1, n / 64);
  for (int a = minc; a < n; a += step)  // one long band + 1..3 short ones
    for (int nb = 1; nb <= 3; ++nb) {
      const int b = (n - a + nb - 1) / nb;
      if (b >= std::max(4, minc / 4)) consider(a, nb, b);
    }
  cache[key] = best;
  static const int log = knob("STEP_BANDS_LOG", 0);
  if (log)
    std::fprintf(stderr, "advdiff: fused step %d planes x %lld columns on %lld slots: bands %d + %d x %d (model %lld)\n",
                 n, tiles, slots, best.zfirst, best.nbands - 1, best.zchunk, bcost);
  return best;
}

// v3 edge tiles (axis_tile): always on since round 2 (the plain partition, their A/B
// loser, was removed in round 6 with the other A/B-only knobs)
constexpr int kStepEdge = 1;
// fewest planes per z chunk: 16 (was 32) lets small grids fill one round of CUs
// (201x199x200 FD4: 6 -> 7 chunks, 216 -> 252 groups, 51.6 -> 45.1 us per step); 512^3 and
// 400x200x206 pick the same chunking either way (profiles/archive/heat3d_min_chunk_r2.log)
constexpr int kStepMinChunk = 16;

struct SArgs {
  const void* uin;
  void* uout;
  int nx, ny;
  int64_t sy, sz;
  int nz_alloc;
  int k0, k1, k0b, k1b;  // one or two output plane ranges (second may be empty)
  int zlo, zhi;
  Box2 bx;
  double cx, cy, cz, dt;
  hipStream_t st;
};

// measured schedule per launch (key: element size, order, device, geometry, range, box)
static std::mutex g_sched_mu;
static std::map<std::vector<int64_t>, int> g_sched;
static std::vector<int64_t> sched_key(int esize, int order, int nx, int ny, int64_t sy,
                                      int64_t sz, int nz_alloc, int k0, int k1, int zlo, int zhi,
                                      const Box2& b) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return {esize, order, dev, nx, ny, sy, sz, nz_alloc, k0, k1, zlo, zhi,
          b.xa0, b.xa1, b.ya0, b.ya1, b.xo0, b.xo1, b.yo0, b.yo1};
}
static bool sched_banded(int esize, int order, const SArgs& a) {
  if (t_sched_force >= 0) return t_sched_force > 0;
  const int m = step_banded();
  if (m >= 0) return m > 0;
  const auto key = sched_key(esize, order, a.nx, a.ny, a.sy, a.sz, a.nz_alloc, a.k0, a.k1, a.zlo,
                             a.zhi, a.bx);
  std::lock_guard<std::mutex> g(g_sched_mu);
  auto it = g_sched.find(key);
  return it != g_sched.end() && it->second > 0;
}

template <typename T, int ORDER, int NW, int RPW, int VAR, bool PUT = false>
static hipError_t launch_step(const SArgs& a, const StepPut& put = StepPut{}) {
  constexpr int R = ORDER / 2;
  constexpr int edge = kStepEdge;
  const int gx = axis_tile_count(64, R, a.bx.xa0, a.bx.xa1, a.bx.xo0, a.bx.xo1, a.nx, edge);
  const int gy = axis_tile_count(NW * RPW, R, a.bx.ya0, a.bx.ya1, a.bx.yo0, a.bx.yo1, a.ny, edge);
  // z chunks: minimise (rounds of resident workgroups) x (chunk + 4R warm-up planes);
  // resident workgroups = CUs x occupancy of this instance (LDS / VGPR bound: 1-2 per CU)
  const int per_cu =
      occupancy_per_cu((const void*)diffusion3d_step_kernel<T, ORDER, NW, RPW, VAR, PUT>, 64 * NW);
  constexpr int minc = kStepMinChunk;
  const int na = std::max(a.k1 - a.k0, 0), nb = std::max(a.k1b - a.k0b, 0);
  const long long slots = (long long)device_cus() * per_cu;
  StepSched sc{gx, gy, 0, 0, edge};
  dim3 grid;
  // (PUT, banded: the long band is the top one, see the kernel; uniform chunks: xcd_tile
  // spreads the chunks of a column over the XCDs, so both faces' stores run through the
  // whole launch either way)
  if (nb == 0 && na > 0 && sched_banded((int)sizeof(T), ORDER, a)) {
    const Bands bd = step_bands(na, (long long)gx * gy, slots, 4 * R, minc);
    sc.zfirst = bd.zfirst;
    sc.zchunk = bd.zchunk;
    sc.gza = bd.nbands;
    grid = dim3(gx * gy * bd.nbands, 1, 1);
  } else {
    const int zc = pick_chunk_rounds(na + nb, (long long)gx * gy, slots, 4 * R, minc);
    sc.gza = na > 0 ? div_up(na, zc) : 0;
    sc.zchunk = zc;
    grid = dim3(gx, gy, sc.gza + (nb > 0 ? div_up(nb, zc) : 0));
  }
  // SSP-RK3 stage coefficients b = 1, 1/4, 2/3: exactly the per-stage path's (FdCoef)
  const FdCoef<T> q1 = fd_coef<T>(ORDER, a.cx, a.cy, a.cz, a.dt, 1.0, true);
  const FdCoef<T> q2 = fd_coef<T>(ORDER, a.cx, a.cy, a.cz, a.dt, 0.25, true);
  const FdCoef<T> q3 = fd_coef<T>(ORDER, a.cx, a.cy, a.cz, a.dt, 2.0 / 3.0, true);
  hipLaunchKernelGGL((diffusion3d_step_kernel<T, ORDER, NW, RPW, VAR, PUT>), grid,
                     dim3(64, NW, 1), 0, a.st, (const T*)a.uin, (T*)a.uout, a.nx, a.ny, a.sy,
                     a.sz, a.nz_alloc, a.k0, a.k1, a.k0b, a.k1b, sc, a.zlo, a.zhi, a.bx, q1, q2,
                     q3, put);
  return hipGetLastError();
}

// Phase-overlap variant (v3_march VAR) per order, from the round-3 interleaved A/B at
// 512^3 fp64 (bench/step_ab.py, profiles/step_ab_r3.log; medians of 7 rounds x 10):
//   FD4 (16 x 2): graded priority (VAR 3) 655.5 us vs 691.9 plain (-5.3 %); deferring
//                 stage 3 as well: 669.8 (priority alone wins);
//   FD2 (12 x 3): second half defers stage 3 + graded priority (VAR 7) 549.3 vs 560.7
//                 (-2.0 %); priority alone: 562.6 (no gain);
//   adjacent rows per wave (PAIR, VAR + 16; profiles/step_ab_pair_r3.log, two runs):
//                 FD2 VAR 23 539.1 / 544.1 us vs VAR 7 550.3 / 551.3 (-1.3..2.0 %) -> the
//                 FD2 default; FD4 VAR 19 660.6 vs 644.8 (VAR 3), VAR 23 ties VAR 3 and
//                 VAR 16 (no priority) 658.8 — FD4 keeps VAR 3 (its LDS reads are not
//                 the limit: -37 % of them bought nothing).
// Also rejected in round 3 (profiles/step_ab_xs_cfg_r3.log): stage-2/3 x neighbours from
// LDS instead of DPP (-23 % VALU instructions, FD4 643.9 -> 651.8 us) and a 16 x 3 FD2 tile
// (amplification 1.20 -> 1.16: 540.7 -> 543.5 us) — the step moves 77 % (FD4) / 85 % (FD2)
// of the copy rate once its halo re-reads are counted (67 / 78 % by a later direct count).
// Also rejected: prefetching NR planes ahead instead of 2 (FD4 equal, FD2 +1.6 %,
// profiles/prefetch_ab_r3.log) and pacing the workgroups of an XCD so co-XCD tiles read
// their shared halo rows together (no gain, profiles/pace_ab_r3.log).
// Built instances: the order's default only (FD4 VAR 3, FD2 VAR 23; the plain kernel,
// VAR 0, and the ADVDIFF_STEP_VAR switch were removed in round 6 — re-checked on the
// round-5 pitched layout, one process: FD4 VAR 19 / 23 / 7 at 0.997 / 1.020 / 1.036 x the
// VAR 3 time, FD2 VAR 7 / 19 at 1.031 / 0.993 x VAR 23, profiles/r5/ab/var_pitched_ab.log).
// The template still takes any VAR for a new experiment.
template <int ORDER>
constexpr int kStepVar = ORDER == 4 ? 3 : 23;

// Tile shape per order.  With the edge tiles (axis_tile), interleaved medians at 512^3:
// FD4 16 waves x 2 rows (32 stage-1 rows) 662 us vs 715 us for 12 x 3; FD2 12 x 3 rows
// 535 us vs 549 us for 16 x 2 (profiles/archive/step_cfgs_edge_r2.log).  48 rows overflow the
// 16-bit DS offsets, 10 x 4 spills at 168 VGPRs.
// fp32 uses the fp64 tile shapes.  Round-5 A/B at 256^3-1024^3 of taller fp32 tiles (16 x
// 3 / 4 rows; profiles/r5/ab/step_fp32_ab.log, bitwise equal): FD4 16 x 4 3-4 % faster at
// 384^3 / 512^3 but 4-6 % slower at 640^3-1024^3, FD2 fastest on the fp64 shape.  FD2 8 x 3
// (two workgroups per CU) 5-13 % slower at 384^3-768^3; 12 x 4 (152 VGPRs) +3.6 / +0.5 /
// -7.0 / +3.0 / +10.1 % at 384 / 512 / 640 / 768 / 1024^3, where the two-step launch wins by
// more (profiles/r5/ab/step_tile_ab*.log); FD4 12 x 3 0.94-0.99 x (fd4_tile_ab.log).  The
// alternatives and their switches were removed in round 6.
template <typename T, int ORDER, bool PUT = false>
static hipError_t dispatch_step(const SArgs& a, const StepPut& put = StepPut{}) {
  if constexpr (ORDER == 4)
    return launch_step<T, ORDER, 16, 2, kStepVar<4>, PUT>(a, put);
  else
    return launch_step<T, ORDER, 12, 3, kStepVar<2>, PUT>(a, put);
}

// two-step FD2 launch (v6_march): 12 waves x 2 rows (24 stage-1 rows, 14 output rows;
// six double-buffered LDS planes = 160.6 KB of the CU's 160 KiB)
template <typename T, int NW, int RPW>
static hipError_t launch_step2x(const SArgs& a) {
  constexpr int R = 1, SH = 5 * R;
  constexpr int edge = kStepEdge;
  const int gx = axis_tile_count(64, R, a.bx.xa0, a.bx.xa1, a.bx.xo0, a.bx.xo1, a.nx, edge, SH);
  const int gy = axis_tile_count(NW * RPW, R, a.bx.ya0, a.bx.ya1, a.bx.yo0, a.bx.yo1, a.ny, edge,
                                 SH);
  const int per_cu =
      occupancy_per_cu((const void*)diffusion3d_step2x_kernel<T, NW, RPW>, 64 * NW);
  const int na = std::max(a.k1 - a.k0, 0);
  const long long slots = (long long)device_cus() * per_cu;
  StepSched sc{gx, gy, 0, 0, edge};
  const int zc = pick_chunk_rounds(na, (long long)gx * gy, slots, 10 * R, kStepMinChunk);
  sc.gza = div_up(na, zc);
  sc.zchunk = zc;
  const FdCoef<T> q1 = fd_coef<T>(2, a.cx, a.cy, a.cz, a.dt, 1.0, true);
  const FdCoef<T> q2 = fd_coef<T>(2, a.cx, a.cy, a.cz, a.dt, 0.25, true);
  const FdCoef<T> q3 = fd_coef<T>(2, a.cx, a.cy, a.cz, a.dt, 2.0 / 3.0, true);
  hipLaunchKernelGGL((diffusion3d_step2x_kernel<T, NW, RPW>), dim3(gx, gy, sc.gza),
                     dim3(64, NW, 1), 0, a.st, (const T*)a.uin, (T*)a.uout, a.nx, a.ny, a.sy,
                     a.sz, a.nz_alloc, a.k0, a.k1, sc, a.zlo, a.zhi, a.bx, q1, q2, q3);
  return hipGetLastError();
}

}  // namespace advdiff

// Host-only query of the band model (no GPU): out = {first band, later band length,
// number of bands, modelled makespan in plane-times of the best split, of the best
// uniform chunking}.  For tests and scheduling studies.
extern "C" int advdiff_step_bands_plan(int n, long long tiles, long long slots, int warm,
                                       int minc, long long* out) {
  using namespace advdiff;
  if (out == nullptr || n <= 0 || tiles <= 0 || slots <= 0) return hipErrorInvalidValue;
  const Bands b = step_bands(n, tiles, slots, warm, minc);
  const int xs = (int)std::max<long long>(slots / 8, 1);
  const long long cols = (tiles + 7) / 8;
  long long uni = -1;
  const int cmax = std::max(1, n / std::max(minc, 1));
  for (int C = 1; C <= std::min(cmax, 16); ++C) {
    const int len = (n + C - 1) / C;
    const long long c = band_makespan(cols, len, (n - len + len - 1) / len, len, xs, warm);
    if (uni < 0 || c < uni) uni = c;
  }
  out[0] = b.zfirst;
  out[1] = b.zchunk;
  out[2] = b.nbands;
  out[3] = band_makespan(cols, b.zfirst, b.nbands - 1, b.zchunk, xs, warm);
  out[4] = uni;
  return hipSuccess;
}

extern "C" int advdiff_set_step_banded(int on) {
  const int old = advdiff::step_banded();
  advdiff::g_step_banded.store(on);
  return old;
}

extern "C" int advdiff_diffusion3d_step_box(int dtype, const void* uin, void* uout, int nx,
                                            int ny, int64_t sy, int64_t sz, int nz_alloc, int k0,
                                            int k1, int k0b, int k1b, int zlo, int zhi,
                                            const int* box, int order, double cx, double cy,
                                            double cz, double dt, void* stream) {
  return advdiff_diffusion3d_step_box_ex(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, k0b,
                                         k1b, zlo, zhi, box, order, cx, cy, cz, dt, 0, stream);
}

extern "C" int advdiff_diffusion3d_step_box_ex(int dtype, const void* uin, void* uout, int nx,
                                               int ny, int64_t sy, int64_t sz, int nz_alloc,
                                               int k0, int k1, int k0b, int k1b, int zlo, int zhi,
                                               const int* box, int order, double cx, double cy,
                                               double cz, double dt, int flags, void* stream) {
  using namespace advdiff;
  if (k1 <= k0) {  // only the second range (or nothing)
    k0 = k0b;
    k1 = k1b;
    k0b = k1b = 0;
  }
  if (k1 <= k0) return hipSuccess;
  if (k1b <= k0b) k0b = k1b = 0;
  if (nx <= 0 || ny <= 0 || uin == uout || k0 < 0 || k1 > nz_alloc || k0b < 0 ||
      k1b > nz_alloc || box == nullptr)
    return hipErrorInvalidValue;
  if (sy * (int64_t)ny >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  const Box2 bx{box[0], box[1], box[2], box[3], box[4], box[5], box[6], box[7]};
  (void)flags;  // placement hints (ADVDIFF_EXCLUSIVE): the grid schedule serves all launches
  const SArgs a{uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, k0b, k1b, zlo, zhi, bx,
                cx, cy, cz, dt, (hipStream_t)stream};
  if (dtype == ADVDIFF_F64) {
    if (order == 4) return dispatch_step<double, 4>(a);
    if (order == 2) return dispatch_step<double, 2>(a);
  } else if (dtype == ADVDIFF_F32) {
    if (order == 4) return dispatch_step<float, 4>(a);
    if (order == 2) return dispatch_step<float, 2>(a);
  }
  return hipErrorInvalidValue;
}

// TWO fused SSP-RK3 steps of the 7-point heat equation in one launch (order 2 only, one
// plane range): uout[k0:k1] = RK3(RK3(uin)) on the box's output x/y range, with the
// intermediate u^{n+1} taken over the whole active box — bit-identical to a one-step
// launch on the active box followed by one on the output box.  The planes within 5 of
// [k0, k1) must hold u^n (ghosts included); the frozen cells (outside [zlo, zhi) and the
// box's active x/y range) keep their values.
extern "C" int advdiff_diffusion3d_step2x(int dtype, const void* uin, void* uout, int nx, int ny,
                                          int64_t sy, int64_t sz, int nz_alloc, int k0, int k1,
                                          int zlo, int zhi, const int* box, double cx, double cy,
                                          double cz, double dt, void* stream) {
  using namespace advdiff;
  if (k1 <= k0) return hipSuccess;
  if (nx <= 0 || ny <= 0 || uin == uout || k0 < 0 || k1 > nz_alloc || box == nullptr)
    return hipErrorInvalidValue;
  if (sy * (int64_t)ny >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  const Box2 bx{box[0], box[1], box[2], box[3], box[4], box[5], box[6], box[7]};
  const SArgs a{uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, 0, 0, zlo, zhi, bx,
                cx, cy, cz, dt, (hipStream_t)stream};
  if (dtype == ADVDIFF_F64) return launch_step2x<double, 12, 2>(a);
  if (dtype == ADVDIFF_F32) return launch_step2x<float, 12, 2>(a);
  return hipErrorInvalidValue;
}

// One step or two per launch for this FD2 shape: measured, once per (dtype, shape) and
// process.  The two-step launch halves the HBM traffic but grows the trapezoid rims from
// 2R to 5R; which wins depends on how the two tilings quantise on the 256 CUs: two per
// launch is 9-25 % faster at 384^3, 640^3-1024^3 fp64 and 16-22 % in fp32, but 3 % slower
// at 512^3 fp64, where the one-step tiling fits unusually well (profiles/r5/ab/
// step2_ab.log, step2_sizes.log, step2_chunks.log).  Protocol: 3 warm-up one-step
// launches, then 3 interleaved rounds of two one-step launches and one two-step launch
// (uin -> uout only: uin is untouched, uout's output box is scratch), min per step; two
// per launch only if it is >= 3 % faster.  ADVDIFF_STEP2=0 / 1 forces the choice.
// Synchronous (host waits on events): call it outside any graph capture.
// Banded or uniform z schedule for this fused-step launch, measured: interleaved rounds of
// both schedules uin -> uout (uout is scratch), banded kept only if >= 1.5 % faster; cached
// per launch and consulted by every later launch of it.  Synchronous: call it outside a
// graph capture.  ADVDIFF_STEP_BANDED=0/1 forces (no measurement).
extern "C" int advdiff_diffusion3d_step_sched_pick(int dtype, const void* uin, void* uout,
                                                   int nx, int ny, int64_t sy, int64_t sz,
                                                   int nz_alloc, int k0, int k1, int zlo,
                                                   int zhi, const int* box, int order, double cx,
                                                   double cy, double cz, double dt, void* stream,
                                                   int* banded) {
  using namespace advdiff;
  if (banded == nullptr || box == nullptr || k1 <= k0) return hipErrorInvalidValue;
  const int mode = step_banded();
  if (mode >= 0) {
    *banded = mode;
    return hipSuccess;
  }
  const Box2 bx{box[0], box[1], box[2], box[3], box[4], box[5], box[6], box[7]};
  const auto key = sched_key(dtype == ADVDIFF_F64 ? 8 : 4, order, nx, ny, sy, sz, nz_alloc, k0,
                             k1, zlo, zhi, bx);
  {
    std::lock_guard<std::mutex> g(g_sched_mu);
    auto it = g_sched.find(key);
    if (it != g_sched.end()) {
      *banded = it->second;
      return hipSuccess;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  auto launch = [&](int m) {  // this thread's launches only (t_sched_force)
    t_sched_force = m;
    const int e = advdiff_diffusion3d_step_box_ex(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0,
                                                  k1, 0, 0, zlo, zhi, box, order, cx, cy, cz, dt,
                                                  ADVDIFF_EXCLUSIVE, stream);
    t_sched_force = -1;
    return e;
  };
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  float t[2] = {1e30f, 1e30f};
  for (int w = 0; w < 4 && e == hipSuccess; ++w) e = (hipError_t)launch(w & 1);
  for (int r = 0; r < 4 && e == hipSuccess; ++r)
    for (int m = 0; m < 2 && e == hipSuccess; ++m) {
      float ms = 0.f;
      e = hipEventRecord(e0, st);
      for (int q = 0; q < 3 && e == hipSuccess; ++q) e = (hipError_t)launch(m);
      if (e == hipSuccess) e = hipEventRecord(e1, st);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess) t[m] = std::min(t[m], ms / 3.f);
    }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (e != hipSuccess) return e;
  *banded = t[1] < 0.985f * t[0];
  if (std::getenv("ADVDIFF_STEP_BANDS_LOG"))
    std::fprintf(stderr, "advdiff: fused FD%d %dx%dx%d %s: uniform %.1f us, banded %.1f us -> %s\n",
                 order, nx, ny, k1 - k0, dtype == ADVDIFF_F64 ? "fp64" : "fp32", t[0] * 1e3f,
                 t[1] * 1e3f, *banded ? "banded" : "uniform");
  std::lock_guard<std::mutex> g(g_sched_mu);
  g_sched[key] = *banded;
  return hipSuccess;
}

extern "C" int advdiff_diffusion3d_step2_pick(int dtype, const void* uin, void* uout, int nx,
                                              int ny, int64_t sy, int64_t sz, int nz_alloc,
                                              int k0, int k1, int zlo, int zhi, const int* box,
                                              double cx, double cy, double cz, double dt,
                                              void* stream, int* use2) {
  using namespace advdiff;
  if (use2 == nullptr || box == nullptr) return hipErrorInvalidValue;
  if (const char* v = std::getenv("ADVDIFF_STEP2"); v && (v[0] == '0' || v[0] == '1')) {
    *use2 = v[0] == '1';
    return hipSuccess;
  }
  static std::mutex mu;
  static std::map<std::vector<int64_t>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::vector<int64_t> key{dtype, dev, nx, ny, sy, sz, nz_alloc, k0, k1, zlo, zhi};
  for (int q = 0; q < 8; ++q) key.push_back(box[q]);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) {
      *use2 = it->second;
      return hipSuccess;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  auto one = [&]() {
    return advdiff_diffusion3d_step_box_ex(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1,
                                           0, 0, zlo, zhi, box, 2, cx, cy, cz, dt,
                                           ADVDIFF_EXCLUSIVE, stream);
  };
  auto two = [&]() {
    return advdiff_diffusion3d_step2x(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, zlo,
                                      zhi, box, cx, cy, cz, dt, stream);
  };
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  float t1 = 1e30f, t2 = 1e30f;
  for (int w = 0; w < 3 && e == hipSuccess; ++w) e = (hipError_t)one();
  for (int r = 0; r < 3 && e == hipSuccess; ++r) {
    float ms = 0.f;
    e = hipEventRecord(e0, st);
    if (e == hipSuccess) e = (hipError_t)one();
    if (e == hipSuccess) e = (hipError_t)one();
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) t1 = std::min(t1, ms / 2.f);
    if (e == hipSuccess) e = hipEventRecord(e0, st);
    if (e == hipSuccess) e = (hipError_t)two();
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) t2 = std::min(t2, ms / 2.f);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (e != hipSuccess) return e;
  *use2 = t2 < 0.97f * t1;
  if (std::getenv("ADVDIFF_STEP2_LOG"))
    std::fprintf(stderr, "advdiff: FD2 %dx%dx%d %s: one step %.1f us, two per launch %.1f us/step"
                 " -> %s\n", nx, ny, k1 - k0, dtype == ADVDIFF_F64 ? "fp64" : "fp32",
                 t1 * 1e3f, t2 * 1e3f, *use2 ? "two" : "one");
  std::lock_guard<std::mutex> g(mu);
  cache[key] = *use2;
  return hipSuccess;
}

extern "C" int advdiff_diffusion3d_step2(int dtype, const void* uin, void* uout, int nx, int ny,
                                         int64_t sy, int64_t sz, int nz_alloc, int k0, int k1,
                                         int k0b, int k1b, int zlo, int zhi, int border,
                                         int order, double cx, double cy, double cz, double dt,
                                         void* stream) {
  const int box[8] = {border, nx - border, border, ny - border, 0, nx, 0, ny};
  return advdiff_diffusion3d_step_box(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, k0b,
                                      k1b, zlo, zhi, box, order, cx, cy, cz, dt, stream);
}

extern "C" int advdiff_diffusion3d_step(int dtype, const void* uin, void* uout, int nx, int ny,
                                        int64_t sy, int64_t sz, int nz_alloc, int k0, int k1,
                                        int zlo, int zhi, int border, int order, double cx,
                                        double cy, double cz, double dt, void* stream) {
  return advdiff_diffusion3d_step2(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, 0, 0, zlo,
                                   zhi, border, order, cx, cy, cz, dt, stream);
}

// One full-range slab step whose output planes [lo_k0, lo_k1) / [hi_k0, hi_k1) are also
// stored into the peer planes at dst_lo / dst_hi (the peer's plane for local plane lo_k0 /
// hi_k0; null or an empty range: no peer on that side).  The peer fields must have this
// field's row pitch and plane stride (slab ranks of one grid).  Uniform z chunks.
// One full-range slab step whose output planes also go, system scope, to peers: part p's
// cells (planes [k0[p], k1[p]), rows [y0[p], y1[p])) to dst[p] + (k - k0[p]) pb[p] + the
// own in-plane byte offset (common.hpp HaloPut; up to 6 parts; null dst / empty range:
// skipped).  Every receive box has this field's row pitch.  Banded or uniform z chunks.
extern "C" int advdiff_diffusion3d_step_putv(int dtype, const void* uin, void* uout, int nx,
                                             int ny, int64_t sy, int64_t sz, int nz_alloc,
                                             int k0, int k1, int zlo, int zhi, int border,
                                             int order, double cx, double cy, double cz,
                                             double dt, int nparts, void* const* dst,
                                             const int* pk0, const int* pk1, const int* py0,
                                             const int* py1, const int64_t* pb, void* stream) {
  using namespace advdiff;
  if (k1 <= k0) return hipSuccess;
  if (nx <= 0 || ny <= 0 || uin == uout || k0 < 0 || k1 > nz_alloc) return hipErrorInvalidValue;
  if (sy * (int64_t)ny >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  StepPut put;
  if (nparts > 0 && (dst == nullptr || pk0 == nullptr || pk1 == nullptr || py0 == nullptr ||
                     py1 == nullptr || pb == nullptr))
    return hipErrorInvalidValue;
  if (!make_halo_put(nparts, dst, pk0, pk1, py0, py1, pb, nz_alloc, put))
    return hipErrorInvalidValue;
  const Box2 bx{border, nx - border, border, ny - border, 0, nx, 0, ny};
  const SArgs a{uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, 0, 0, zlo, zhi, bx,
                cx, cy, cz, dt, (hipStream_t)stream};
  if (dtype == ADVDIFF_F64) {
    if (order == 4) return dispatch_step<double, 4, true>(a, put);
    if (order == 2) return dispatch_step<double, 2, true>(a, put);
  } else if (dtype == ADVDIFF_F32) {
    if (order == 4) return dispatch_step<float, 4, true>(a, put);
    if (order == 2) return dispatch_step<float, 2, true>(a, put);
  }
  return hipErrorInvalidValue;
}

// The two-face form: output planes [lo_k0, lo_k1) / [hi_k0, hi_k1) to the peer planes at
// dst_lo / dst_hi (the peer plane of local plane lo_k0 / hi_k0; all rows; this field's
// plane stride).
extern "C" int advdiff_diffusion3d_step_put(int dtype, const void* uin, void* uout, int nx,
                                            int ny, int64_t sy, int64_t sz, int nz_alloc, int k0,
                                            int k1, int zlo, int zhi, int border, int order,
                                            double cx, double cy, double cz, double dt,
                                            void* dst_lo, int lo_k0, int lo_k1, void* dst_hi,
                                            int hi_k0, int hi_k1, void* stream) {
  void* dst[2] = {dst_lo, dst_hi};
  const int pk0[2] = {lo_k0, hi_k0}, pk1[2] = {lo_k1, hi_k1}, py0[2] = {0, 0};
  const int py1[2] = {1 << 30, 1 << 30};
  const int64_t esz = dtype == ADVDIFF_F64 ? 8 : 4, pb[2] = {sz * esz, sz * esz};
  return advdiff_diffusion3d_step_putv(dtype, uin, uout, nx, ny, sy, sz, nz_alloc, k0, k1, zlo,
                                       zhi, border, order, cx, cy, cz, dt, 2, dst, pk0, pk1,
                                       py0, py1, pb, stream);
}

// Code-object preload (see advdiff_preload in aux.hip).
// The default kernels' occupancies are cached here too (launch.hpp occupancy_per_cu), so
// no launch inside a hipGraph capture is the first to query one.
extern "C" int advdiff_preload_diffusion_fused(void) {
  using namespace advdiff;
  hipFuncAttributes a;
  const hipError_t e =
      hipFuncGetAttributes(&a, (const void*)diffusion3d_step_kernel<double, 4, 16, 2, 3>);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<double, 4, 16, 2, 3>, 64 * 16);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<double, 2, 12, 3, 23>, 64 * 12);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<float, 4, 16, 2, 3>, 64 * 16);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<float, 2, 12, 3, 23>, 64 * 12);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<double, 4, 16, 2, 3, true>, 64 * 16);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<double, 2, 12, 3, 23, true>, 64 * 12);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<float, 4, 16, 2, 3, true>, 64 * 16);
  (void)occupancy_per_cu((const void*)diffusion3d_step_kernel<float, 2, 12, 3, 23, true>, 64 * 12);
  (void)occupancy_per_cu((const void*)diffusion3d_step2x_kernel<double, 12, 2>, 64 * 12);
  (void)occupancy_per_cu((const void*)diffusion3d_step2x_kernel<float, 12, 2>, 64 * 12);
  return e;
}
