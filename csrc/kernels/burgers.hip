// Fused WENO5 Burgers SSP-RK3 stage kernels for gfx950.
//
// One kernel evaluates the full RHS  L(u) = -Σ_d ∂_d f(u) [+ C ∇²u]  AND the RK
// stage combination.  It replaces the reference's per-direction sweep kernels
//   MultiGPU/Burgers3d_Baseline/Kernels.cu:225-490   (Compute_dF/dG/dH + Compute_RK,
//                                                    one thread per pencil, uncoalesced)
//   SingleGPU/Burgers3d_WENO5*/kernels.cu           (6 memory variants: global, pitched,
//                                                    shared line tiles, textures, hybrids)
//   MultiGPU/Burgers2d_Baseline/Kernels.cu:214-382
// and the separate viscous Compute_Laplace_Async pass.
//
// The problem is fp64-VALU bound (≈380 VALU ops per cell and stage), so the design
// goals are: compute every face flux exactly once, keep every wave busy, and cut
// divisions (common.hpp: one division per reconstruction side).
//
// 3-D structure: a 64 x TY workgroup (one wave per tile row) marches along z.
//   * Per plane, the tile + 3-cell halo of u is staged in LDS together with the
//     split fluxes f± (computed once per point at staging time).  The next plane's
//     tile is prefetched into registers while the current plane computes.
//   * x faces: each lane computes the face to the right of its cell; y faces: the
//     face above its cell.  The TY missing left faces and the 64 missing bottom faces
//     are computed by the last / first wave (wave-uniform branches), so the tile costs
//     (64·TY + TY + 64) x/y faces instead of twice that.
//   * z faces: each lane keeps f±(k-2..k+3) of its own column in registers; the
//     face k+½ of plane k is reused as face k-½ of plane k+1.
// 2-D: a row tile of 256 lanes marching along y, same scheme.
#include "common.hpp"
#include "launch.hpp"
#include "advdiff/kernels.h"

namespace advdiff {

template <typename T, bool WZ, bool VISC, bool USE_U0, int TX, int TY>
__global__ __launch_bounds__(TX* TY) void burgers3d_stage_kernel(
    const T* __restrict__ in, const T* u0, T* out, int nx, int ny, int64_t sy, int64_t sz,
    int k0, int k1, int zchunk, int border, T rdx, T rdy, T rdz, T vx, T vy, T vz, T dt, T a,
    T b) {
  constexpr int R = 3;
  constexpr int LX = TX + 2 * R, LY = TY + 2 * R, NT = TX * TY;
  constexpr int NPT = (LX * LY + NT - 1) / NT;
  constexpr int FXW = TX + 1;  // x-face row width
  __shared__ T s_u[LY * LX];
  __shared__ T s_p[LY * LX];
  __shared__ T s_m[LY * LX];
  __shared__ T s_fx[TY * FXW];
  __shared__ T s_fy[(TY + 1) * TX];

  const int tx = threadIdx.x, ty = threadIdx.y, tid = ty * TX + tx;
  const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
  const int i = i0 + tx, j = j0 + ty;
  const int kc0 = k0 + (int)blockIdx.z * zchunk;
  const int kc1 = min(kc0 + zchunk, k1);
  const bool active = i >= border && i < nx - border && j >= border && j < ny - border;
  const int64_t own = (int64_t)min(j, ny - 1) * sy + min(i, nx - 1);
  const int lc = (ty + R) * LX + tx + R;

  // Per-thread gather offsets of the tile (plane-relative), computed once.
  int64_t toff[NPT];
#pragma unroll
  for (int r = 0; r < NPT; ++r) {
    const int idx = min(tid + r * NT, LX * LY - 1);
    const int ly = idx / LX, lx = idx - ly * LX;
    const int gi = clampi(i0 - R + lx, 0, nx - 1);
    const int gj = clampi(j0 - R + ly, 0, ny - 1);
    toff[r] = (int64_t)gj * sy + gi;
  }
  T pre[NPT];
  auto fetch_tile = [&](int k) {
    const T* src = in + (int64_t)k * sz;
#pragma unroll
    for (int r = 0; r < NPT; ++r) pre[r] = src[toff[r]];
  };

  // ---- prologue: column window and the face below the first plane ----
  T P[5], M[5], U[5];  // f+(k-2..k+2), f-(k-1..k+3), u(k-2..k+2)
  T fz_lo;
  {
    T uz[6], fp[6], fm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      uz[q] = in[(int64_t)(kc0 - 3 + q) * sz + own];
      lf_split(uz[q], fp[q], fm[q]);
    }
    // face kc0-½ : f+(kc0-3..kc0+1), f-(kc0-2..kc0+2)
    fz_lo = weno5_face<T, WZ>(fp[0], fp[1], fp[2], fp[3], fp[4], fm[1], fm[2], fm[3], fm[4],
                              fm[5]);
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      P[q] = fp[q + 1];
      U[q] = uz[q + 1];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) M[q] = fm[q + 2];
  }
  fetch_tile(kc0);
  T unext = in[(int64_t)(kc0 + 3) * sz + own];

  for (int k = kc0; k < kc1; ++k) {
    __syncthreads();  // previous plane's LDS readers are done
#pragma unroll
    for (int r = 0; r < NPT; ++r) {
      const int idx = tid + r * NT;
      if (NPT * NT == LX * LY || idx < LX * LY) {
        T p, m;
        lf_split(pre[r], p, m);
        s_u[idx] = pre[r];
        s_p[idx] = p;
        s_m[idx] = m;
      }
    }
    // own column: u(k+3) -> f-(k+3) now, f+(k+3)/u(k+3) after the shift
    T pn, mn;
    lf_split(unext, pn, mn);
    M[4] = mn;
    const T un = unext;
    if (k + 1 < kc1) {
      fetch_tile(k + 1);
      unext = in[(int64_t)(k + 4) * sz + own];
    }
    __syncthreads();

    // x face at i+½ and y face at j+½ of this lane's cell
    s_fx[ty * FXW + tx + 1] =
        weno5_face<T, WZ>(s_p[lc - 2], s_p[lc - 1], s_p[lc], s_p[lc + 1], s_p[lc + 2],
                          s_m[lc - 1], s_m[lc], s_m[lc + 1], s_m[lc + 2], s_m[lc + 3]);
    s_fy[(ty + 1) * TX + tx] = weno5_face<T, WZ>(
        s_p[lc - 2 * LX], s_p[lc - LX], s_p[lc], s_p[lc + LX], s_p[lc + 2 * LX],
        s_m[lc - LX], s_m[lc], s_m[lc + LX], s_m[lc + 2 * LX], s_m[lc + 3 * LX]);
    if (ty == 0) {  // bottom faces j0-½ of every column (wave-uniform)
      const int c = 3 * LX + tx + R;  // row j0
      s_fy[tx] = weno5_face<T, WZ>(s_p[c - 3 * LX], s_p[c - 2 * LX], s_p[c - LX], s_p[c],
                                   s_p[c + LX], s_m[c - 2 * LX], s_m[c - LX], s_m[c],
                                   s_m[c + LX], s_m[c + 2 * LX]);
    }
    if (ty == TY - 1 && tx < TY) {  // left faces i0-½ of every row
      const int c = (tx + R) * LX + R;  // (row tx, column i0)
      s_fx[tx * FXW] = weno5_face<T, WZ>(s_p[c - 3], s_p[c - 2], s_p[c - 1], s_p[c],
                                         s_p[c + 1], s_m[c - 2], s_m[c - 1], s_m[c],
                                         s_m[c + 1], s_m[c + 2]);
    }
    const T fz_hi = weno5_face<T, WZ>(P[0], P[1], P[2], P[3], P[4], M[0], M[1], M[2], M[3], M[4]);
    __syncthreads();

    const T ctr = s_u[lc];
    T L = -((s_fx[ty * FXW + tx + 1] - s_fx[ty * FXW + tx]) * rdx +
            (s_fy[(ty + 1) * TX + tx] - s_fy[ty * TX + tx]) * rdy + (fz_hi - fz_lo) * rdz);
    if constexpr (VISC) {
      L += vx * FD<4>::d2(s_u[lc - 2], s_u[lc - 1], ctr, s_u[lc + 1], s_u[lc + 2]) +
           vy * FD<4>::d2(s_u[lc - 2 * LX], s_u[lc - LX], ctr, s_u[lc + LX], s_u[lc + 2 * LX]) +
           vz * FD<4>::d2(U[0], U[1], ctr, U[3], U[4]);
    }
    if (active) {
      const int64_t o = (int64_t)k * sz + own;
      T uo = T(0);
      if constexpr (USE_U0) uo = u0[o];
      out[o] = rk_stage<T, USE_U0>(uo, ctr, L, dt, a, b);
    }
    fz_lo = fz_hi;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      P[q] = P[q + 1];
      M[q] = M[q + 1];
      U[q] = U[q + 1];
    }
    P[4] = pn;
    U[4] = un;
  }
}

template <typename T, bool WZ, bool VISC, bool USE_U0, int TX>
__global__ __launch_bounds__(TX) void burgers2d_stage_kernel(
    const T* __restrict__ in, const T* u0, T* out, int nx, int64_t sy, int j0, int j1,
    int ychunk, int border, T rdx, T rdy, T vx, T vy, T dt, T a, T b) {
  constexpr int R = 3, LX = TX + 2 * R;
  __shared__ T s_u[LX];
  __shared__ T s_p[LX];
  __shared__ T s_m[LX];
  __shared__ T s_fx[TX + 1];

  const int tx = threadIdx.x;
  const int i0 = blockIdx.x * TX, i = i0 + tx;
  const int jc0 = j0 + (int)blockIdx.y * ychunk;
  const int jc1 = min(jc0 + ychunk, j1);
  const bool active = i >= border && i < nx - border;
  const int ic = min(i, nx - 1);
  const int lc = tx + R;
  const int g0 = clampi(i0 - R + tx, 0, nx - 1);
  const int g1 = clampi(i0 - R + TX + tx, 0, nx - 1);

  T pre0, pre1 = T(0);
  auto fetch_row = [&](int jj) {
    const T* src = in + (int64_t)jj * sy;
    pre0 = src[g0];
    if (tx < 2 * R) pre1 = src[g1];
  };

  T P[5], M[5], U[5];
  T fy_lo;
  {
    T uy[6], fp[6], fm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      uy[q] = in[(int64_t)(jc0 - 3 + q) * sy + ic];
      lf_split(uy[q], fp[q], fm[q]);
    }
    fy_lo = weno5_face<T, WZ>(fp[0], fp[1], fp[2], fp[3], fp[4], fm[1], fm[2], fm[3], fm[4],
                              fm[5]);
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      P[q] = fp[q + 1];
      U[q] = uy[q + 1];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) M[q] = fm[q + 2];
  }
  fetch_row(jc0);
  T unext = in[(int64_t)(jc0 + 3) * sy + ic];

  for (int jj = jc0; jj < jc1; ++jj) {
    __syncthreads();
    {
      T p, m;
      lf_split(pre0, p, m);
      s_u[tx] = pre0;
      s_p[tx] = p;
      s_m[tx] = m;
      if (tx < 2 * R) {
        lf_split(pre1, p, m);
        s_u[TX + tx] = pre1;
        s_p[TX + tx] = p;
        s_m[TX + tx] = m;
      }
    }
    T pn, mn;
    lf_split(unext, pn, mn);
    M[4] = mn;
    const T un = unext;
    if (jj + 1 < jc1) {
      fetch_row(jj + 1);
      unext = in[(int64_t)(jj + 4) * sy + ic];
    }
    __syncthreads();
    s_fx[tx + 1] = weno5_face<T, WZ>(s_p[lc - 2], s_p[lc - 1], s_p[lc], s_p[lc + 1],
                                     s_p[lc + 2], s_m[lc - 1], s_m[lc], s_m[lc + 1],
                                     s_m[lc + 2], s_m[lc + 3]);
    if (tx == TX - 1) {  // left face i0-½ (last wave, single lane)
      s_fx[0] = weno5_face<T, WZ>(s_p[0], s_p[1], s_p[2], s_p[3], s_p[4], s_m[1], s_m[2],
                                  s_m[3], s_m[4], s_m[5]);
    }
    const T fy_hi = weno5_face<T, WZ>(P[0], P[1], P[2], P[3], P[4], M[0], M[1], M[2], M[3], M[4]);
    __syncthreads();
    const T ctr = s_u[lc];
    T L = -((s_fx[tx + 1] - s_fx[tx]) * rdx + (fy_hi - fy_lo) * rdy);
    if constexpr (VISC) {
      L += vx * FD<4>::d2(s_u[lc - 2], s_u[lc - 1], ctr, s_u[lc + 1], s_u[lc + 2]) +
           vy * FD<4>::d2(U[0], U[1], ctr, U[3], U[4]);
    }
    if (active) {
      const int64_t o = (int64_t)jj * sy + i;
      T uo = T(0);
      if constexpr (USE_U0) uo = u0[o];
      out[o] = rk_stage<T, USE_U0>(uo, ctr, L, dt, a, b);
    }
    fy_lo = fy_hi;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      P[q] = P[q + 1];
      M[q] = M[q + 1];
      U[q] = U[q + 1];
    }
    P[4] = pn;
    U[4] = un;
  }
}

// ------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------
constexpr int kBTX3 = 64, kBTY3 = 8;
constexpr int kBTX2 = 256;

template <typename T, bool WZ, bool VISC, bool U0, int TY>
static hipError_t launch_b3_ty(const void* in, const void* u0, void* out, int nx, int ny,
                               int64_t sy, int64_t sz, int k0, int k1, int border, double rdx,
                               double rdy, double rdz, double vx, double vy, double vz,
                               double dt, double a, double b, hipStream_t st) {
  const int gx = div_up(nx, kBTX3), gy = div_up(ny, TY);
  const int zc = pick_chunk(k1 - k0, (long long)gx * gy, 8, 256);
  const int gz = div_up(k1 - k0, zc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers3d_stage_kernel<T, WZ, VISC, U0, kBTX3, TY>), dim3(gx, gy, gz),
                     dim3(kBTX3, TY, 1), 0, st, (const T*)in, (const T*)u0, (T*)out, nx, ny, sy,
                     sz, k0, k1, zc, border, T(rdx), T(rdy), T(rdz), T(vx * s), T(vy * s),
                     T(vz * s), T(dt), T(a), T(b));
  return hipGetLastError();
}

template <typename T, bool WZ, bool VISC, bool U0>
static hipError_t launch_b3(const void* in, const void* u0, void* out, int nx, int ny,
                            int64_t sy, int64_t sz, int k0, int k1, int border, double rdx,
                            double rdy, double rdz, double vx, double vy, double vz, double dt,
                            double a, double b, hipStream_t st) {
  static const int ty = knob("B3_TY", kBTY3);
  if (ty == 16)
    return launch_b3_ty<T, WZ, VISC, U0, 16>(in, u0, out, nx, ny, sy, sz, k0, k1, border, rdx,
                                             rdy, rdz, vx, vy, vz, dt, a, b, st);
  return launch_b3_ty<T, WZ, VISC, U0, 8>(in, u0, out, nx, ny, sy, sz, k0, k1, border, rdx, rdy,
                                          rdz, vx, vy, vz, dt, a, b, st);
}

template <typename T, bool WZ, bool VISC, bool U0>
static hipError_t launch_b2(const void* in, const void* u0, void* out, int nx, int64_t sy,
                            int j0, int j1, int border, double rdx, double rdy, double vx,
                            double vy, double dt, double a, double b, hipStream_t st) {
  const int gx = div_up(nx, kBTX2);
  const int yc = pick_chunk(j1 - j0, gx, 4, 256);
  const int gy = div_up(j1 - j0, yc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers2d_stage_kernel<T, WZ, VISC, U0, kBTX2>), dim3(gx, gy, 1),
                     dim3(kBTX2, 1, 1), 0, st, (const T*)in, (const T*)u0, (T*)out, nx, sy, j0,
                     j1, yc, border, T(rdx), T(rdy), T(vx * s), T(vy * s), T(dt), T(a), T(b));
  return hipGetLastError();
}

template <typename T>
static hipError_t dispatch_b3(const void* in, const void* u0, void* out, int nx, int ny,
                              int64_t sy, int64_t sz, int k0, int k1, int border, int wz,
                              double rdx, double rdy, double rdz, double vx, double vy,
                              double vz, double dt, double a, double b, hipStream_t st) {
  const bool visc = vx != 0.0 || vy != 0.0 || vz != 0.0;
  const bool u0f = a != 0.0;
  const int key = (wz ? 4 : 0) | (visc ? 2 : 0) | (u0f ? 1 : 0);
#define B3(W, V, U)                                                                        \
  return launch_b3<T, W, V, U>(in, u0, out, nx, ny, sy, sz, k0, k1, border, rdx, rdy, rdz, \
                               vx, vy, vz, dt, a, b, st)
  switch (key) {
    case 0: B3(false, false, false);
    case 1: B3(false, false, true);
    case 2: B3(false, true, false);
    case 3: B3(false, true, true);
    case 4: B3(true, false, false);
    case 5: B3(true, false, true);
    case 6: B3(true, true, false);
    default: B3(true, true, true);
  }
#undef B3
}

template <typename T>
static hipError_t dispatch_b2(const void* in, const void* u0, void* out, int nx, int64_t sy,
                              int j0, int j1, int border, int wz, double rdx, double rdy,
                              double vx, double vy, double dt, double a, double b,
                              hipStream_t st) {
  const bool visc = vx != 0.0 || vy != 0.0;
  const bool u0f = a != 0.0;
  const int key = (wz ? 4 : 0) | (visc ? 2 : 0) | (u0f ? 1 : 0);
#define B2(W, V, U) \
  return launch_b2<T, W, V, U>(in, u0, out, nx, sy, j0, j1, border, rdx, rdy, vx, vy, dt, a, b, st)
  switch (key) {
    case 0: B2(false, false, false);
    case 1: B2(false, false, true);
    case 2: B2(false, true, false);
    case 3: B2(false, true, true);
    case 4: B2(true, false, false);
    case 5: B2(true, false, true);
    case 6: B2(true, true, false);
    default: B2(true, true, true);
  }
#undef B2
}

}  // namespace advdiff

extern "C" int advdiff_burgers3d_stage(int dtype, const void* in, const void* u0, void* out,
                                       int nx, int ny, int64_t sy, int64_t sz, int k0, int k1,
                                       int border, int weno_z, double rdx, double rdy,
                                       double rdz, double vx, double vy, double vz, double dt,
                                       double a, double b, void* stream) {
  using namespace advdiff;
  if (k1 <= k0) return hipSuccess;
  if (k0 < 3 || nx <= 0 || ny <= 0 || in == out) return hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADVDIFF_F64)
    return dispatch_b3<double>(in, u0, out, nx, ny, sy, sz, k0, k1, border, weno_z, rdx, rdy,
                               rdz, vx, vy, vz, dt, a, b, st);
  if (dtype == ADVDIFF_F32)
    return dispatch_b3<float>(in, u0, out, nx, ny, sy, sz, k0, k1, border, weno_z, rdx, rdy,
                              rdz, vx, vy, vz, dt, a, b, st);
  return hipErrorInvalidValue;
}

extern "C" int advdiff_burgers2d_stage(int dtype, const void* in, const void* u0, void* out,
                                       int nx, int64_t sy, int j0, int j1, int border,
                                       int weno_z, double rdx, double rdy, double vx, double vy,
                                       double dt, double a, double b, void* stream) {
  using namespace advdiff;
  if (j1 <= j0) return hipSuccess;
  if (j0 < 3 || nx <= 0 || in == out) return hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADVDIFF_F64)
    return dispatch_b2<double>(in, u0, out, nx, sy, j0, j1, border, weno_z, rdx, rdy, vx, vy,
                               dt, a, b, st);
  if (dtype == ADVDIFF_F32)
    return dispatch_b2<float>(in, u0, out, nx, sy, j0, j1, border, weno_z, rdx, rdy, vx, vy,
                              dt, a, b, st);
  return hipErrorInvalidValue;
}
