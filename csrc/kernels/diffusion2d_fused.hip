// 2-D heat equation: ONE full SSP-RK3 step per launch (temporal blocking), gfx950.
//
// The 2-D counterpart of diffusion_fused.hip with no LDS and no barriers at all: every
// wave owns a 64-column strip and marches along y on its own.  Column strip x = i0-2R+lane:
//   stage 1  A(j+2R) on all 64 lanes  (x neighbours by DPP wave shifts; the 2R edge lanes
//            read their missing neighbours straight from the row, prefetched one row ahead)
//   stage 2  B(j+R)  on lanes [R, 64-R)      (x neighbours of A by DPP)
//   stage 3  u(j)    on lanes [2R, 64-2R)    -> 56 output columns per wave (FD4)
// y neighbours come from exact register rings (2R+1 rows of u, A and B; u(j) of stage 3
// from a delay line), as in the 3-D compact-ring kernel.  HBM traffic 16 B/cell/step.
// Bit-identical to three advdiff_diffusion2d_stage launches (same helpers, same order).
// Reference: MultiGPU/Diffusion2d_Baseline (Compute_Laplace + Compute_RK per stage),
// SingleGPU/Diffusion2d{,_PitchedMem,_TextureMem}.
#include "common.hpp"
#include "launch.hpp"
#include "advdiff/kernels.h"

namespace advdiff {

constexpr int kWavesPerBlock2 = 4;

template <typename T, int ORDER>
__global__ __launch_bounds__(64 * kWavesPerBlock2) void diffusion2d_step_kernel(
    const T* __restrict__ uin, T* __restrict__ uout, int nx, int64_t sy, int ny_alloc, int j0,
    int j1, int ylo, int yhi, int ychunk, int nchunks, int ntiles, int xa0, int xa1, int xo0,
    int xo1, FdCoef<T> q1, FdCoef<T> q2, FdCoef<T> q3) {
  constexpr int R = FD<ORDER>::R;
  constexpr int NR = 2 * R + 1;
  constexpr int W = 64;
  constexpr int TX = W - 4 * R;
  const int lane = threadIdx.x;
  const int item = blockIdx.x * kWavesPerBlock2 + threadIdx.y;  // (x-tile, y-chunk)
  if (item >= ntiles * nchunks) return;                          // wave-uniform
  const int tile = item % ntiles, chunk = item / ntiles;
  const int i0 = tile * TX;
  const int x = i0 - 2 * R + lane;
  const int jc0 = j0 + chunk * ychunk;
  const int jc1 = min(jc0 + ychunk, j1);
  const bool xin = x >= xa0 && x < xa1;                 // non-frozen columns
  const bool xout = xin && x >= xo0 && x < xo1;          // columns this launch writes
  const bool s2c = lane >= R && lane < W - R;
  const bool s3c = lane >= 2 * R && lane < W - 2 * R;
  const int xc = clampi(x, 0, nx - 1);
  // edge lanes: columns of the two missing x neighbours (left for lanes < R, right for
  // lanes >= W-R), clamped to the array (those values only feed frozen/unused cells)
  const bool edge = lane < R || lane >= W - R;
  const int e1 = clampi(lane < R ? x - 1 : x + 1, 0, nx - 1);
  const int e2 = clampi(lane < R ? x - 2 : x + 2, 0, nx - 1);
  auto row = [&](int j) { return uin + (int64_t)clampi(j, 0, ny_alloc - 1) * sy; };

  const int jst = jc0 - 4 * R;
  T ru[NR], ra[NR], rb[NR], dl[R];
#pragma unroll
  for (int d = 0; d < R - 1; ++d) dl[d] = row(jst + d)[xc];
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    const int p = jst + R - 1 + s;
    ru[p - jst < NR ? p - jst : p - jst - NR] = row(p)[xc];
    ra[s] = rb[s] = T(0);
  }
  T un = row(jst + 3 * R)[xc];
  T ev1 = T(0), ev2 = T(0);  // edge neighbours of row jst+2R
  if (edge) {
    ev1 = row(jst + 2 * R)[e1];
    ev2 = row(jst + 2 * R)[e2];
  }
  const T third = T(1.0 / 3.0);

  auto body = [&]<int PH>(int j) {
    auto sl = [](int d) { return (PH + d + 4 * NR) % NR; };
    constexpr int UIN = (PH + 3 * R) % NR;
    dl[R - 1] = ru[UIN];  // u(j+R-1) -> delay line
    ru[UIN] = un;
    const T ee1 = ev1, ee2 = ev2;
    if (j + 1 < jc1) {  // prefetch the next row (and its edge neighbours)
      un = row(j + 1 + 3 * R)[xc];
      if (edge) {
        ev1 = row(j + 1 + 2 * R)[e1];
        ev2 = row(j + 1 + 2 * R)[e2];
      }
    }
    // stage 1: A(j+2R) on all lanes
    {
      const T c = ru[sl(2 * R)];
      T acc = fd_ctr(q1.kc, c);  // order: centre, y, x (as the per-stage kernel)
      if constexpr (R == 2) {
        T m1 = wave_shr1(c), p1 = wave_shl1(c);
        T m2 = wave_shr1(m1), p2 = wave_shl1(p1);
        if (lane < R) {  // own x-1, x-2 from the prefetched row values
          m1 = ee1;
          m2 = ee2;
        } else if (lane >= W - R) {
          p1 = ee1;
          p2 = ee2;
        }
        acc = fd4_axis(acc, q1.k[1], ru[sl(R)], ru[sl(R + 1)], ru[sl(3 * R - 1)],
                       ru[sl(3 * R)]);
        acc = fd4_axis(acc, q1.k[0], m2, m1, p1, p2);
      } else {
        T m1 = wave_shr1(c), p1 = wave_shl1(c);
        if (lane == 0) m1 = ee1;
        if (lane == W - 1) p1 = ee1;
        acc = fd2_axis(acc, q1.k[1], ru[sl(R)], ru[sl(3 * R)]);
        acc = fd2_axis(acc, q1.k[0], m1, p1);
      }
      const int p = j + 2 * R;
      const T v = acc;
      ra[sl(2 * R)] = (p >= ylo && p < yhi && xin) ? v : c;
    }
    // stage 2: B(j+R)
    if (j >= jc0 - 2 * R) {
      const T c = ra[sl(R)];
      const T uo = ru[sl(R)];
      T acc = fd_ctr(q2.kc, c, T(0.75) * uo);
      if constexpr (R == 2) {
        const T m1 = wave_shr1(c), p1 = wave_shl1(c);
        acc = fd4_axis(acc, q2.k[1], ra[sl(0)], ra[sl(1)], ra[sl(3)], ra[sl(4)]);
        acc = fd4_axis(acc, q2.k[0], wave_shr1(m1), m1, p1, wave_shl1(p1));
      } else {
        acc = fd2_axis(acc, q2.k[1], ra[sl(0)], ra[sl(2)]);
        acc = fd2_axis(acc, q2.k[0], wave_shr1(c), wave_shl1(c));
      }
      const int p = j + R;
      const T v = acc;
      rb[sl(R)] = (p >= ylo && p < yhi && xin && s2c) ? v : uo;
    }
    // stage 3: u^{n+1}(j)
    if (j >= jc0) {
      const T c = rb[sl(0)];
      const T uo = dl[0];
      T acc = fd_ctr(q3.kc, c, third * uo);
      if constexpr (R == 2) {
        const T m1 = wave_shr1(c), p1 = wave_shl1(c);
        acc = fd4_axis(acc, q3.k[1], rb[sl(-2)], rb[sl(-1)], rb[sl(1)], rb[sl(2)]);
        acc = fd4_axis(acc, q3.k[0], wave_shr1(m1), m1, p1, wave_shl1(p1));
      } else {
        acc = fd2_axis(acc, q3.k[1], rb[sl(-1)], rb[sl(1)]);
        acc = fd2_axis(acc, q3.k[0], wave_shr1(c), wave_shl1(c));
      }
      const T v = acc;
      if (xout && s3c) uout[(int64_t)j * sy + x] = v;
    }
#pragma unroll
    for (int d = 0; d < R - 1; ++d) dl[d] = dl[d + 1];
  };

  for (int jb = jst; jb < jc1; jb += NR) {
    body.template operator()<0>(jb);
    if (jb + 1 < jc1) body.template operator()<1>(jb + 1);
    if (jb + 2 < jc1) body.template operator()<2>(jb + 2);
    if constexpr (NR > 3) {
      if (jb + 3 < jc1) body.template operator()<3>(jb + 3);
      if (jb + 4 < jc1) body.template operator()<4>(jb + 4);
    }
  }
}

template <typename T, int ORDER>
static hipError_t launch_step2d(const void* uin, void* uout, int nx, int64_t sy, int ny_alloc,
                                int j0, int j1, int ylo, int yhi, const int* bx, double cx,
                                double cy, double dt, hipStream_t st) {
  constexpr int R = ORDER / 2;
  constexpr int TX = 64 - 4 * R;
  const int ntiles = div_up(nx, TX);
  // Waves are independent and latency-bound when few: cost(C chunks) ~ (rows per wave +
  // 4R warm-up) x max(1, waves / wave slots), wave slots ~ 4 per SIMD (fitted on 400² ..
  // 16384²: profiles/heat2d_sizes.log).  Small grids get short chunks (more waves), large
  // grids long ones (less warm-up).
  static const int slots = 4 * 4 * device_cus();
  constexpr int minc = 2;
  const int n = j1 - j0;
  int chunks = 1;
  double best = -1.0;
  for (int C = 1; C <= std::max(1, n / minc); ++C) {
    const double len = (double)div_up(n, C);
    const double cost = (len + 4 * R) * std::max(1.0, (double)ntiles * C / slots);
    if (best < 0 || cost < best) {
      best = cost;
      chunks = C;
    }
  }
  const int yc = div_up(n, chunks);
  chunks = div_up(n, yc);
  const int items = ntiles * chunks;
  // SSP-RK3 stage coefficients b = 1, 1/4, 2/3 (the per-stage path's, common.hpp FdCoef)
  hipLaunchKernelGGL((diffusion2d_step_kernel<T, ORDER>), dim3(div_up(items, kWavesPerBlock2)),
                     dim3(64, kWavesPerBlock2, 1), 0, st, (const T*)uin, (T*)uout, nx, sy,
                     ny_alloc, j0, j1, ylo, yhi, yc, chunks, ntiles, bx[0], bx[1], bx[2],
                     bx[3], fd_coef<T>(ORDER, cx, cy, 0.0, dt, 1.0, true),
                     fd_coef<T>(ORDER, cx, cy, 0.0, dt, 0.25, true),
                     fd_coef<T>(ORDER, cx, cy, 0.0, dt, 2.0 / 3.0, true));
  return hipGetLastError();
}

}  // namespace advdiff

extern "C" int advdiff_diffusion2d_step_box(int dtype, const void* uin, void* uout, int nx,
                                            int64_t sy, int ny_alloc, int j0, int j1, int ylo,
                                            int yhi, const int* box, int order, double cx,
                                            double cy, double dt, void* stream) {
  using namespace advdiff;
  if (j1 <= j0) return hipSuccess;
  if (nx <= 0 || uin == uout || j0 < 0 || j1 > ny_alloc || box == nullptr)
    return hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
#define S2D(T, O) \
  return launch_step2d<T, O>(uin, uout, nx, sy, ny_alloc, j0, j1, ylo, yhi, box, cx, cy, dt, st)
  if (dtype == ADVDIFF_F64) {
    if (order == 4) S2D(double, 4);
    if (order == 2) S2D(double, 2);
  } else if (dtype == ADVDIFF_F32) {
    if (order == 4) S2D(float, 4);
    if (order == 2) S2D(float, 2);
  }
#undef S2D
  return hipErrorInvalidValue;
}

extern "C" int advdiff_diffusion2d_step(int dtype, const void* uin, void* uout, int nx,
                                        int64_t sy, int ny_alloc, int j0, int j1, int ylo,
                                        int yhi, int border, int order, double cx, double cy,
                                        double dt, void* stream) {
  const int box[4] = {border, nx - border, 0, nx};
  return advdiff_diffusion2d_step_box(dtype, uin, uout, nx, sy, ny_alloc, j0, j1, ylo, yhi, box,
                                      order, cx, cy, dt, stream);
}

// Code-object preload (see advdiff_preload in aux.hip).
extern "C" int advdiff_preload_diffusion2d_fused(void) {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void*)advdiff::diffusion2d_step_kernel<double, 4>);
}
