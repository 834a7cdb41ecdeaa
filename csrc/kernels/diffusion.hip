// Fused heat-equation SSP-RK3 stage kernels for gfx950.
//
// Replaces the reference's whole family of Laplacian + RK kernels
//   MultiGPU/Diffusion3d_Baseline/Kernels.cu:104-300   (Laplace, LaplaceO2_async,
//                                                      LaplaceO4_async, Compute_RK)
//   SingleGPU/Diffusion3d_{baselineCode,PitchedMem,Blocking}/kernels.cu
//   SingleGPU/Diffusion2d{,_PitchedMem,_TextureMem}/kernels.cu
//   MultiGPU/Diffusion2d_Baseline/Kernels.cu:126-188
// with ONE kernel per dimensionality that computes L(u) and the RK combination in
// the same pass (no Lu array, no uo memcpy): 16-24 B of HBM traffic per cell and
// stage instead of the reference's ~56.
//
// Structure (3-D): a 64 x TY workgroup owns a tile of columns and marches along z.
//   * Each plane of the input is staged ONCE into an LDS ring (tile + R-cell halo in
//     x and y; R+2 slots so a single barrier per plane suffices: the slot written at
//     plane k is neither slot read at plane k-1).
//   * Each thread keeps its own column's z-window (2R+1 values) in registers, fed
//     from the ring, so the z-neighbours cost no extra memory traffic.
//   * The x/y neighbours come from the ring slot of the centre plane (ds_read_b64,
//     64 consecutive doubles per wave: conflict-free).
//   * blockIdx.z splits the z-range into chunks so one launch has >= 2048 groups.
// 2-D uses the same scheme with a row tile marching along y.
#include "common.hpp"
#include "launch.hpp"
#include "advdiff/kernels.h"

namespace advdiff {

template <typename T, int ORDER, int TX, int TY, int MODE>
__global__ __launch_bounds__(TX* TY) void diffusion3d_stage_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int ny, int64_t sy, int64_t sz,
    int k0, int k1, int zchunk, int border, FdCoef<T> q, T a, T b) {
  constexpr int R = FD<ORDER>::R;
  constexpr int LX = TX + 2 * R, LY = TY + 2 * R, NS = R + 2, NT = TX * TY, NE = LX * LY;
  constexpr int NPT = (NE + NT - 1) / NT;  // tile elements staged per thread and plane
  __shared__ T ring[NS][NE];

  const int tx = threadIdx.x, ty = threadIdx.y, tid = ty * TX + tx;
  const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
  const int i = i0 + tx, j = j0 + ty;
  const int kc0 = k0 + (int)blockIdx.z * zchunk;
  const int kc1 = min(kc0 + zchunk, k1);
  const bool active = i >= border && i < nx - border && j >= border && j < ny - border;
  const int own = min(j, ny - 1) * (int)sy + min(i, nx - 1);  // plane-relative
  const int lc = (ty + R) * LX + tx + R;

  // Plane-relative gather offsets of this thread's tile elements (clamped at the array
  // edge: those values only feed cells that are never written).
  int toff[NPT];
#pragma unroll
  for (int r = 0; r < NPT; ++r) {
    const int idx = min(tid + r * NT, NE - 1);
    const int ly = idx / LX, lx = idx - ly * LX;
    toff[r] = clampi(j0 - R + ly, 0, ny - 1) * (int)sy + clampi(i0 - R + lx, 0, nx - 1);
  }
  T pre[NPT];
  auto fetch = [&](int k) {
    const T* src = in + (int64_t)k * sz;
#pragma unroll
    for (int r = 0; r < NPT; ++r) pre[r] = src[toff[r]];
  };
  auto stash = [&](int k) {
    T* s = ring[k % NS];
#pragma unroll
    for (int r = 0; r < NPT; ++r)
      if (NPT * NT == NE || tid + r * NT < NE) s[tid + r * NT] = pre[r];
  };

  T zw[2 * R + 1];
#pragma unroll
  for (int q = 0; q < 2 * R; ++q) zw[q] = in[(int64_t)(kc0 - R + q) * sz + own];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    fetch(kc0 + q);
    stash(kc0 + q);
  }
  fetch(kc0 + R);

  for (int k = kc0; k < kc1; ++k) {
    stash(k + R);                       // plane k+R: loaded one iteration ago
    if (k + 1 < kc1) fetch(k + R + 1);  // keep the next plane's loads in flight
    T ax = T(0);
    if constexpr (reads_aux<MODE>()) ax = aux[(int64_t)k * sz + own];
    __syncthreads();
    zw[2 * R] = ring[(k + R) % NS][lc];
    const T* c = ring[k % NS];
    const T ctr = zw[R];
    T acc = fd_start<T, MODE>(q.kc, ctr, ax, a);  // fixed order: centre, z, x, y
    if constexpr (ORDER == 4) {
      acc = fd4_axis(acc, q.k[2], zw[0], zw[1], zw[3], zw[4]);
      acc = fd4_axis(acc, q.k[0], c[lc - 2], c[lc - 1], c[lc + 1], c[lc + 2]);
      acc = fd4_axis(acc, q.k[1], c[lc - 2 * LX], c[lc - LX], c[lc + LX],
                     c[lc + 2 * LX]);
    } else {
      acc = fd2_axis(acc, q.k[2], zw[0], zw[2]);
      acc = fd2_axis(acc, q.k[0], c[lc - 1], c[lc + 1]);
      acc = fd2_axis(acc, q.k[1], c[lc - LX], c[lc + LX]);
    }
    if (active) fd_store<T, MODE>(out, aux, (int64_t)k * sz + own, ctr, acc, b);
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) zw[q] = zw[q + 1];
  }
}

template <typename T, int ORDER, int TX, int MODE>
__global__ __launch_bounds__(TX) void diffusion2d_stage_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int64_t sy, int j0, int j1,
    int ychunk, int border, FdCoef<T> q, T a, T b) {
  constexpr int R = FD<ORDER>::R;
  constexpr int LX = TX + 2 * R, NS = R + 2;
  __shared__ T ring[NS][LX];

  const int tx = threadIdx.x;
  const int i0 = blockIdx.x * TX, i = i0 + tx;
  const int jc0 = j0 + (int)blockIdx.y * ychunk;
  const int jc1 = min(jc0 + ychunk, j1);
  const bool active = i >= border && i < nx - border;
  const int ic = min(i, nx - 1);
  const int lc = tx + R;
  const int g0 = clampi(i0 - R + tx, 0, nx - 1);
  const int g1 = clampi(i0 - R + TX + tx, 0, nx - 1);

  T p0, p1 = T(0);
  auto fetch = [&](int jj) {
    const T* src = in + (int64_t)jj * sy;
    p0 = src[g0];
    if (tx < 2 * R) p1 = src[g1];
  };
  auto stash = [&](int jj) {
    T* s = ring[jj % NS];
    s[tx] = p0;
    if (tx < 2 * R) s[TX + tx] = p1;
  };

  T yw[2 * R + 1];
#pragma unroll
  for (int q = 0; q < 2 * R; ++q) yw[q] = in[(int64_t)(jc0 - R + q) * sy + ic];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    fetch(jc0 + q);
    stash(jc0 + q);
  }
  fetch(jc0 + R);

  for (int jj = jc0; jj < jc1; ++jj) {
    stash(jj + R);
    if (jj + 1 < jc1) fetch(jj + R + 1);
    T ax = T(0);
    if constexpr (reads_aux<MODE>()) ax = aux[(int64_t)jj * sy + ic];
    __syncthreads();
    yw[2 * R] = ring[(jj + R) % NS][lc];
    const T* c = ring[jj % NS];
    const T ctr = yw[R];
    T acc = fd_start<T, MODE>(q.kc, ctr, ax, a);  // fixed order: centre, y, x
    if constexpr (ORDER == 4) {
      acc = fd4_axis(acc, q.k[1], yw[0], yw[1], yw[3], yw[4]);
      acc = fd4_axis(acc, q.k[0], c[lc - 2], c[lc - 1], c[lc + 1], c[lc + 2]);
    } else {
      acc = fd2_axis(acc, q.k[1], yw[0], yw[2]);
      acc = fd2_axis(acc, q.k[0], c[lc - 1], c[lc + 1]);
    }
    if (active) fd_store<T, MODE>(out, aux, (int64_t)jj * sy + i, ctr, acc, b);
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) yw[q] = yw[q + 1];
  }
}

// ------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------
constexpr int kTX3 = 64, kTY3 = 16;  // 1024-thread groups: one wave per tile row (A/B: profiles/)
constexpr int kTX2 = 256;

struct DArgs {
  const void* in;
  void* aux;
  void* out;
  int nx, ny;
  int64_t sy, sz;
  int lo, hi, border;  // marched-axis range [lo, hi)
  double cx, cy, cz, dt, a, b;
  hipStream_t st;
};

// folded stage coefficients (common.hpp FdCoef): SSP stages scale by b and keep the c
// term; low-storage stages produce d = a du + dt L (b = 1, no c term)
template <typename T, int MODE>
static FdCoef<T> stage_coef(int order, const DArgs& p) {
  const bool ls = MODE == kLs1 || MODE == kLs;
  return fd_coef<T>(order, p.cx, p.cy, p.cz, p.dt, ls ? 1.0 : p.b, !ls);
}

template <typename T, int ORDER, int TY, int MODE>
static hipError_t launch_d3_ty(const DArgs& p) {
  const int gx = div_up(p.nx, kTX3), gy = div_up(p.ny, TY);
  const int zc = pick_chunk(p.hi - p.lo, (long long)gx * gy, 8, 256);
  const int gz = div_up(p.hi - p.lo, zc);
  hipLaunchKernelGGL((diffusion3d_stage_kernel<T, ORDER, kTX3, TY, MODE>), dim3(gx, gy, gz),
                     dim3(kTX3, TY, 1), 0, p.st, (const T*)p.in, (T*)p.aux, (T*)p.out, p.nx,
                     p.ny, p.sy, p.sz, p.lo, p.hi, zc, p.border, stage_coef<T, MODE>(ORDER, p),
                     T(p.a), T(p.b));
  return hipGetLastError();
}

template <typename T, int ORDER, int MODE>
static hipError_t launch_d3(const DArgs& p) {
  // (the 4- and 16-row tiles and their ADVDIFF_D3_TY switch were removed in round 6)
  return launch_d3_ty<T, ORDER, kTY3, MODE>(p);
}

template <typename T, int ORDER, int MODE>
static hipError_t launch_d2(const DArgs& p) {
  const int gx = div_up(p.nx, kTX2);
  const int yc = pick_chunk(p.hi - p.lo, gx, 8, 256);
  const int gy = div_up(p.hi - p.lo, yc);
  hipLaunchKernelGGL((diffusion2d_stage_kernel<T, ORDER, kTX2, MODE>), dim3(gx, gy, 1),
                     dim3(kTX2, 1, 1), 0, p.st, (const T*)p.in, (T*)p.aux, (T*)p.out, p.nx,
                     p.sy, p.lo, p.hi, yc, p.border, stage_coef<T, MODE>(ORDER, p), T(p.a),
                     T(p.b));
  return hipGetLastError();
}

template <typename T, bool THREE_D, int ORDER>
static hipError_t d_by_mode(int mode, const DArgs& p) {
#define DM(M) return THREE_D ? launch_d3<T, ORDER, M>(p) : launch_d2<T, ORDER, M>(p)
  switch (mode) {
    case kSsp1: DM(kSsp1);
    case kSsp: DM(kSsp);
    case kLs1: DM(kLs1);
    default: DM(kLs);
  }
#undef DM
}

static hipError_t run_d(int dtype, bool three_d, int order, bool ls, const DArgs& p) {
  if (p.hi <= p.lo) return hipSuccess;
  const int R = order / 2;
  if ((order != 2 && order != 4) || p.lo < R || p.nx <= 0 || (three_d && p.ny <= 0) ||
      p.in == p.out || (ls && (p.in == p.aux || p.out == p.aux)))
    return hipErrorInvalidValue;
  if (three_d && p.sy * (int64_t)p.ny >= (int64_t(1) << 31))
    return hipErrorInvalidValue;  // 32-bit plane offsets
  const int mode = ls ? (p.a != 0.0 ? kLs : kLs1) : (p.a != 0.0 ? kSsp : kSsp1);
#define DD(T, O) \
  return three_d ? d_by_mode<T, true, O>(mode, p) : d_by_mode<T, false, O>(mode, p)
  if (dtype == ADVDIFF_F64) {
    if (order == 4) DD(double, 4);
    DD(double, 2);
  }
  if (dtype == ADVDIFF_F32) {
    if (order == 4) DD(float, 4);
    DD(float, 2);
  }
#undef DD
  return hipErrorInvalidValue;
}

}  // namespace advdiff

extern "C" int advdiff_diffusion3d_stage(int dtype, const void* in, const void* u0, void* out,
                                         int nx, int ny, int64_t sy, int64_t sz, int k0,
                                         int k1, int border, int order, double cx, double cy,
                                         double cz, double dt, double a, double b,
                                         void* stream) {
  using namespace advdiff;
  const DArgs p{in, const_cast<void*>(u0), out, nx, ny, sy, sz, k0, k1, border,
                cx, cy, cz, dt, a, b, (hipStream_t)stream};
  return run_d(dtype, true, order, false, p);
}

extern "C" int advdiff_diffusion3d_stage_ls(int dtype, const void* in, void* du, void* out,
                                            int nx, int ny, int64_t sy, int64_t sz, int k0,
                                            int k1, int border, int order, double cx,
                                            double cy, double cz, double dt, double A,
                                            double B, void* stream) {
  using namespace advdiff;
  const DArgs p{in, du, out, nx, ny, sy, sz, k0, k1, border, cx, cy, cz, dt, A, B,
                (hipStream_t)stream};
  return run_d(dtype, true, order, true, p);
}

extern "C" int advdiff_diffusion2d_stage(int dtype, const void* in, const void* u0, void* out,
                                         int nx, int64_t sy, int j0, int j1, int border,
                                         int order, double cx, double cy, double dt, double a,
                                         double b, void* stream) {
  using namespace advdiff;
  const DArgs p{in, const_cast<void*>(u0), out, nx, 0, sy, 0, j0, j1, border,
                cx, cy, 0.0, dt, a, b, (hipStream_t)stream};
  return run_d(dtype, false, order, false, p);
}

extern "C" int advdiff_diffusion2d_stage_ls(int dtype, const void* in, void* du, void* out,
                                            int nx, int64_t sy, int j0, int j1, int border,
                                            int order, double cx, double cy, double dt,
                                            double A, double B, void* stream) {
  using namespace advdiff;
  const DArgs p{in, du, out, nx, 0, sy, 0, j0, j1, border, cx, cy, 0.0, dt, A, B,
                (hipStream_t)stream};
  return run_d(dtype, false, order, true, p);
}

// Code-object preload (see advdiff_preload in aux.hip).
extern "C" int advdiff_preload_diffusion(void) {
  hipFuncAttributes a;
  return hipFuncGetAttributes(
      &a, (const void*)advdiff::diffusion3d_stage_kernel<double, 4, advdiff::kTX3, advdiff::kTY3, 0>);
}
