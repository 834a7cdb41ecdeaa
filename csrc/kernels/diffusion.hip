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

template <typename T, int ORDER, int TX, int TY, bool USE_U0>
__global__ __launch_bounds__(TX* TY) void diffusion3d_stage_kernel(
    const T* __restrict__ in, const T* u0, T* out, int nx, int ny, int64_t sy, int64_t sz,
    int k0, int k1, int zchunk, int border, T cx, T cy, T cz, T dt, T a, T b) {
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
    T uo = T(0);
    if constexpr (USE_U0) uo = u0[(int64_t)k * sz + own];
    __syncthreads();
    zw[2 * R] = ring[(k + R) % NS][lc];
    const T* c = ring[k % NS];
    const T ctr = zw[R];
    T lap;
    if constexpr (ORDER == 4) {
      lap = lap3(cx, FD<4>::d2(c[lc - 2], c[lc - 1], ctr, c[lc + 1], c[lc + 2]), cy,
                 FD<4>::d2(c[lc - 2 * LX], c[lc - LX], ctr, c[lc + LX], c[lc + 2 * LX]), cz,
                 FD<4>::d2(zw[0], zw[1], ctr, zw[3], zw[4]));
    } else {
      lap = lap3(cx, FD<2>::d2(c[lc - 1], ctr, c[lc + 1]), cy,
                 FD<2>::d2(c[lc - LX], ctr, c[lc + LX]), cz, FD<2>::d2(zw[0], ctr, zw[2]));
    }
    if (active) out[(int64_t)k * sz + own] = rk_stage<T, USE_U0>(uo, ctr, lap, dt, a, b);
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) zw[q] = zw[q + 1];
  }
}

template <typename T, int ORDER, int TX, bool USE_U0>
__global__ __launch_bounds__(TX) void diffusion2d_stage_kernel(
    const T* __restrict__ in, const T* u0, T* out, int nx, int64_t sy, int j0, int j1,
    int ychunk, int border, T cx, T cy, T dt, T a, T b) {
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
    T uo = T(0);
    if constexpr (USE_U0) uo = u0[(int64_t)jj * sy + ic];
    __syncthreads();
    yw[2 * R] = ring[(jj + R) % NS][lc];
    const T* c = ring[jj % NS];
    const T ctr = yw[R];
    T lap;
    if constexpr (ORDER == 4) {
      lap = lap2(cx, FD<4>::d2(c[lc - 2], c[lc - 1], ctr, c[lc + 1], c[lc + 2]), cy,
                 FD<4>::d2(yw[0], yw[1], ctr, yw[3], yw[4]));
    } else {
      lap = lap2(cx, FD<2>::d2(c[lc - 1], ctr, c[lc + 1]), cy, FD<2>::d2(yw[0], ctr, yw[2]));
    }
    if (active) out[(int64_t)jj * sy + i] = rk_stage<T, USE_U0>(uo, ctr, lap, dt, a, b);
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) yw[q] = yw[q + 1];
  }
}

// ------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------
constexpr int kTX3 = 64, kTY3 = 16;  // 1024-thread groups: one wave per tile row (A/B: profiles/)
constexpr int kTX2 = 256;

template <typename T, int ORDER, int TY, bool USE_U0>
static hipError_t launch_d3_ty(const void* in, const void* u0, void* out, int nx, int ny,
                               int64_t sy, int64_t sz, int k0, int k1, int border, double cx,
                               double cy, double cz, double dt, double a, double b,
                               hipStream_t st) {
  const int gx = div_up(nx, kTX3), gy = div_up(ny, TY);
  const int zc = pick_chunk(k1 - k0, (long long)gx * gy, 8, 256);
  const int gz = div_up(k1 - k0, zc);
  const double s = ORDER == 4 ? 1.0 / 12.0 : 1.0;
  hipLaunchKernelGGL((diffusion3d_stage_kernel<T, ORDER, kTX3, TY, USE_U0>), dim3(gx, gy, gz),
                     dim3(kTX3, TY, 1), 0, st, (const T*)in, (const T*)u0, (T*)out, nx, ny, sy,
                     sz, k0, k1, zc, border, T(cx * s), T(cy * s), T(cz * s), T(dt), T(a), T(b));
  return hipGetLastError();
}

template <typename T, int ORDER, bool USE_U0>
static hipError_t launch_d3(const void* in, const void* u0, void* out, int nx, int ny,
                            int64_t sy, int64_t sz, int k0, int k1, int border, double cx,
                            double cy, double cz, double dt, double a, double b,
                            hipStream_t st) {
  static const int ty = knob("D3_TY", kTY3);
#define TYL(TY) \
  return launch_d3_ty<T, ORDER, TY, USE_U0>(in, u0, out, nx, ny, sy, sz, k0, k1, border, cx, cy, cz, dt, a, b, st)
  switch (ty) {
    case 4: TYL(4);
    case 16: TYL(16);
    default: TYL(8);
  }
#undef TYL
}

template <typename T, int ORDER, bool USE_U0>
static hipError_t launch_d2(const void* in, const void* u0, void* out, int nx, int64_t sy,
                            int j0, int j1, int border, double cx, double cy, double dt,
                            double a, double b, hipStream_t st) {
  const int gx = div_up(nx, kTX2);
  const int yc = pick_chunk(j1 - j0, gx, 8, 256);
  const int gy = div_up(j1 - j0, yc);
  const double s = ORDER == 4 ? 1.0 / 12.0 : 1.0;
  hipLaunchKernelGGL((diffusion2d_stage_kernel<T, ORDER, kTX2, USE_U0>), dim3(gx, gy, 1),
                     dim3(kTX2, 1, 1), 0, st, (const T*)in, (const T*)u0, (T*)out, nx, sy,
                     j0, j1, yc, border, T(cx * s), T(cy * s), T(dt), T(a), T(b));
  return hipGetLastError();
}

template <typename T>
static hipError_t dispatch_d3(const void* in, const void* u0, void* out, int nx, int ny,
                              int64_t sy, int64_t sz, int k0, int k1, int border, int order,
                              double cx, double cy, double cz, double dt, double a, double b,
                              hipStream_t st) {
  const bool use_u0 = a != 0.0;
#define D3(ORD, U) \
  return launch_d3<T, ORD, U>(in, u0, out, nx, ny, sy, sz, k0, k1, border, cx, cy, cz, dt, a, b, st)
  if (order == 4) {
    if (use_u0) D3(4, true); else D3(4, false);
  } else if (order == 2) {
    if (use_u0) D3(2, true); else D3(2, false);
  }
#undef D3
  return hipErrorInvalidValue;
}

template <typename T>
static hipError_t dispatch_d2(const void* in, const void* u0, void* out, int nx, int64_t sy,
                              int j0, int j1, int border, int order, double cx, double cy,
                              double dt, double a, double b, hipStream_t st) {
  const bool use_u0 = a != 0.0;
#define D2(ORD, U) return launch_d2<T, ORD, U>(in, u0, out, nx, sy, j0, j1, border, cx, cy, dt, a, b, st)
  if (order == 4) {
    if (use_u0) D2(4, true); else D2(4, false);
  } else if (order == 2) {
    if (use_u0) D2(2, true); else D2(2, false);
  }
#undef D2
  return hipErrorInvalidValue;
}

}  // namespace advdiff

extern "C" int advdiff_diffusion3d_stage(int dtype, const void* in, const void* u0, void* out,
                                         int nx, int ny, int64_t sy, int64_t sz, int k0,
                                         int k1, int border, int order, double cx, double cy,
                                         double cz, double dt, double a, double b,
                                         void* stream) {
  using namespace advdiff;
  if (k1 <= k0) return hipSuccess;
  const int R = order / 2;
  if (k0 < R || nx <= 0 || ny <= 0 || in == out) return hipErrorInvalidValue;
  if (sy * (int64_t)ny >= (int64_t(1) << 31)) return hipErrorInvalidValue;  // 32-bit plane offsets
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADVDIFF_F64)
    return dispatch_d3<double>(in, u0, out, nx, ny, sy, sz, k0, k1, border, order, cx, cy,
                               cz, dt, a, b, st);
  if (dtype == ADVDIFF_F32)
    return dispatch_d3<float>(in, u0, out, nx, ny, sy, sz, k0, k1, border, order, cx, cy,
                              cz, dt, a, b, st);
  return hipErrorInvalidValue;
}

extern "C" int advdiff_diffusion2d_stage(int dtype, const void* in, const void* u0, void* out,
                                         int nx, int64_t sy, int j0, int j1, int border,
                                         int order, double cx, double cy, double dt, double a,
                                         double b, void* stream) {
  using namespace advdiff;
  if (j1 <= j0) return hipSuccess;
  const int R = order / 2;
  if (j0 < R || nx <= 0 || in == out) return hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADVDIFF_F64)
    return dispatch_d2<double>(in, u0, out, nx, sy, j0, j1, border, order, cx, cy, dt, a, b,
                               st);
  if (dtype == ADVDIFF_F32)
    return dispatch_d2<float>(in, u0, out, nx, sy, j0, j1, border, order, cx, cy, dt, a, b,
                              st);
  return hipErrorInvalidValue;
}
