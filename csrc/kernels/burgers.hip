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
#include <utility>

#include "common.hpp"
#include "launch.hpp"
#include "advdiff/kernels.h"

namespace advdiff {

// Scheme-generic fused stage.  Rc = Recon<T, W, WZ>: R = 3 (WENO5) or 4 (WENO7),
// NP = 2R-1 values per side of a face.  MODE: stage epilogue (common.hpp).
template <typename T, int W, bool WZ, bool VISC, int MODE, int TX, int TY>
// WENO7 (136 VGPRs unconstrained): capped at 128 for 4 waves/SIMD = two 8-wave groups
// per CU; a 20-byte spill, -12 % stage time (profiles/archive/kbench_latest.log)
__global__ __launch_bounds__(TX* TY)
__attribute__((amdgpu_waves_per_eu(W == 7 ? 4 : 1))) void burgers3d_stage_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int ny, int64_t sy, int64_t sz, int k0,
    int k1, int zchunk, int border, T rdx, T rdy, T rdz, T vx, T vy, T vz, T dt, T a, T b,
    const double* __restrict__ dtp) {
  using Rc = Recon<T, W, WZ>;
  constexpr int R = Rc::R, NP = 2 * R - 1;
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
  if (dtp != nullptr && !device_dt(dtp, dt)) {  // adaptive run at t_end: out = in
    if (active)
      for (int k = kc0; k < kc1; ++k) out[(int64_t)k * sz + own] = in[(int64_t)k * sz + own];
    return;
  }

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
  // flux at the face to the right of LDS cell c along stride st
  auto lds_face = [&](int c, int st) {
    T pv[NP], mv[NP];
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      pv[d] = s_p[c + (d - R + 1) * st];
      mv[d] = s_m[c + (d - R + 2) * st];
    }
    return Rc::face(pv, mv);
  };

  // ---- prologue: column window and the face below the first plane ----
  T P[NP], M[NP], U[NP];  // f+(k-R+1..k+R-1), f-(k-R+2..k+R), u(k-R+1..k+R-1)
  T KP[3], KM[3];         // WENO5: curvatures of f+ at k-1..k+1 and f- at k..k+2
  T fz_lo;
  {
    T uz[2 * R], fp[2 * R], fm[2 * R];
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) {
      uz[q] = in[(int64_t)(kc0 - R + q) * sz + own];
      lf_split(uz[q], fp[q], fm[q]);
    }
    fz_lo = Rc::face(fp, fm + 1);  // face kc0-½
    if constexpr (W == 5) {  // curvatures carried along z: f+ at kc0-1, kc0; f- at kc0, kc0+1
      KP[0] = weno5_curv(fp[1], fp[2], fp[3]);
      KP[1] = weno5_curv(fp[2], fp[3], fp[4]);
      KM[0] = weno5_curv(fm[2], fm[3], fm[4]);
      KM[1] = weno5_curv(fm[3], fm[4], fm[5]);
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      P[q] = fp[q + 1];
      U[q] = uz[q + 1];
    }
#pragma unroll
    for (int q = 0; q < NP - 1; ++q) M[q] = fm[q + 2];
  }
  fetch_tile(kc0);
  T unext = in[(int64_t)(kc0 + R) * sz + own];

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
    // own column: u(k+R) -> f-(k+R) now, f+(k+R)/u(k+R) after the shift
    T pn, mn;
    lf_split(unext, pn, mn);
    M[NP - 1] = mn;
    const T un = unext;
    if (k + 1 < kc1) {
      fetch_tile(k + 1);
      unext = in[(int64_t)(k + 1 + R) * sz + own];
    }
    __syncthreads();

    // x face at i+½ and y face at j+½ of this lane's cell
    s_fx[ty * FXW + tx + 1] = lds_face(lc, 1);
    s_fy[(ty + 1) * TX + tx] = lds_face(lc, LX);
    if (ty == 0)  // bottom faces j0-½ of every column (wave-uniform)
      s_fy[tx] = lds_face((R - 1) * LX + tx + R, LX);
    if (ty == TY - 1 && tx < TY)  // left faces i0-½ of every row
      s_fx[tx * FXW] = lds_face((tx + R) * LX + R - 1, 1);
    T fz_hi;
    if constexpr (W == 5) {  // two of three curvatures per side come from the last plane
      KP[2] = weno5_curv(P[2], P[3], P[4]);
      KM[2] = weno5_curv(M[2], M[3], M[4]);
      fz_hi = weno5_face_k<T, WZ>(P, M, KP, KM);
      KP[0] = KP[1];
      KP[1] = KP[2];
      KM[0] = KM[1];
      KM[1] = KM[2];
    } else {
      fz_hi = Rc::face(P, M);
    }
    __syncthreads();

    const T ctr = s_u[lc];
    T L = -((s_fx[ty * FXW + tx + 1] - s_fx[ty * FXW + tx]) * rdx +
            (s_fy[(ty + 1) * TX + tx] - s_fy[ty * TX + tx]) * rdy + (fz_hi - fz_lo) * rdz);
    if constexpr (VISC) {
      L += vx * FD<4>::d2(s_u[lc - 2], s_u[lc - 1], ctr, s_u[lc + 1], s_u[lc + 2]) +
           vy * FD<4>::d2(s_u[lc - 2 * LX], s_u[lc - LX], ctr, s_u[lc + LX], s_u[lc + 2 * LX]) +
           vz * FD<4>::d2(U[R - 3], U[R - 2], ctr, U[R], U[R + 1]);
    }
    if (active) {
      const int64_t o = (int64_t)k * sz + own;
      T ax = T(0);
      if constexpr (reads_aux<MODE>()) ax = aux[o];
      stage_store<T, MODE>(out, aux, o, ax, ctr, L, dt, a, b);
    }
    fz_lo = fz_hi;
#pragma unroll
    for (int q = 0; q < NP - 1; ++q) {
      P[q] = P[q + 1];
      M[q] = M[q + 1];
      U[q] = U[q + 1];
    }
    P[NP - 1] = pn;
    U[NP - 1] = un;
  }
}

// ------------------------------------------------------------------------------
// WENO5 3-D stage, v2 (the default for WENO5-JS/Z):
//   * 63-cell x tiles: lane l computes the face to the right of its cell from the LDS
//     tile; the face to its left comes from lane l-1 by one DPP shift, so lane 0 only
//     supplies that face and no wave computes an extra column of faces (v1: the last
//     wave of the tile computed the tile's left faces with 8 of 64 lanes active);
//   * y faces: the face above each row, plus the tile's bottom row of faces by wave 0;
//   * z faces from the lane's register column (two of three curvatures reused);
//   * scaled smoothness indicators (common.hpp w5_*): 32 instead of 40 fp64 ops per side;
//   * the cell value and the z neighbours of the viscous term come from the register
//     column, x/y neighbours from the LDS tile;
//   * DB = false: 2 barriers per plane (faces | stage next tile | combine);
//     DB = true: a double-buffered tile and ONE barrier per plane (2x the LDS).
// Tiles are anchored at the active region (x: border-1, y: border), so a 256-wide grid
// with border 3 takes 4 x tiles.
// ------------------------------------------------------------------------------
template <typename T, bool WZ, bool VISC, int MODE, int TY, bool DB, int WPE>
__global__ __launch_bounds__(64 * TY) __attribute__((amdgpu_waves_per_eu(WPE))) void burgers3d_w5_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int ny, int64_t sy, int64_t sz, int k0,
    int k1, int zchunk, int border, T rdx, T rdy, T rdz, T vx, T vy, T vz, T dt, T a, T b,
    const double* __restrict__ dtp) {
  constexpr int R = 3, NP = 5, TX = 64, TXO = TX - 1;
  constexpr int LX = TX + 2 * R, LY = TY + 2 * R, NT = TX * TY, LT = LX * LY;
  constexpr int NPT = (LT + NT - 1) / NT;
  constexpr int NB = DB ? 2 : 1;
  __shared__ T s_p[NB][LT];
  __shared__ T s_m[NB][LT];
  __shared__ T s_u[VISC ? NB : 1][VISC ? LT : 1];
  __shared__ T s_fy[NB][(TY + 1) * TX];

  const int tx = threadIdx.x, ty = threadIdx.y, tid = ty * TX + tx;
  const int ib = border - 1 + (int)blockIdx.x * TXO;  // x of lane 0 (supplies a face only)
  const int jb = border + (int)blockIdx.y * TY;       // y of wave 0
  const int i = ib + tx, j = jb + ty;
  const int kc0 = k0 + (int)blockIdx.z * zchunk;
  const int kc1 = min(kc0 + zchunk, k1);
  const bool active = tx >= 1 && i < nx - border && j < ny - border;
  const int64_t own = (int64_t)min(j, ny - 1) * sy + min(i, nx - 1);
  const int lc = (ty + R) * LX + tx + R;
  if (dtp != nullptr && !device_dt(dtp, dt)) {  // adaptive run at t_end: out = in
    if (active)
      for (int k = kc0; k < kc1; ++k) out[(int64_t)k * sz + own] = in[(int64_t)k * sz + own];
    return;
  }

  int64_t toff[NPT];
#pragma unroll
  for (int r = 0; r < NPT; ++r) {
    const int idx = min(tid + r * NT, LT - 1);
    const int ly = idx / LX, lx = idx - ly * LX;
    toff[r] = (int64_t)clampi(jb - R + ly, 0, ny - 1) * sy + clampi(ib - R + lx, 0, nx - 1);
  }
  T pre[NPT];
  auto fetch_tile = [&](int k) {
    const T* src = in + (int64_t)k * sz;
#pragma unroll
    for (int r = 0; r < NPT; ++r) pre[r] = src[toff[r]];
  };
  auto stage_tile = [&](int buf) {
#pragma unroll
    for (int r = 0; r < NPT; ++r) {
      const int idx = tid + r * NT;
      if (NPT * NT == LT || idx < LT) {
        T p, m;
        lf_split(pre[r], p, m);
        s_p[buf][idx] = p;
        s_m[buf][idx] = m;
        if constexpr (VISC) s_u[buf][idx] = pre[r];
      }
    }
  };
  auto lds_face = [&](int buf, int c, int st) {
    T pv[NP], mv[NP];
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      pv[d] = s_p[buf][c + (d - R + 1) * st];
      mv[d] = s_m[buf][c + (d - R + 2) * st];
    }
    return w5_face<T, WZ>(pv, mv);
  };

  // ---- prologue: column window, the face below the first plane, the first tile ----
  T P[NP], M[NP], U[NP];  // f+(k-2..k+2), f-(k-1..k+3) (last filled per plane), u(k-2..k+2)
  T KP[3], KM[3];         // C of f+ centred on k-1..k+1, of f- centred on k..k+2
  T fz_lo;
  {
    T uz[2 * R], fp[2 * R], fm[2 * R];
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) {
      uz[q] = in[(int64_t)(kc0 - R + q) * sz + own];
      lf_split(uz[q], fp[q], fm[q]);
    }
    fz_lo = w5_face<T, WZ>(fp, fm + 1);  // face kc0-½
    KP[0] = w5_curv(fp[1], fp[2], fp[3]);
    KP[1] = w5_curv(fp[2], fp[3], fp[4]);
    KM[0] = w5_curv(fm[2], fm[3], fm[4]);
    KM[1] = w5_curv(fm[3], fm[4], fm[5]);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      P[q] = fp[q + 1];
      U[q] = uz[q + 1];
    }
#pragma unroll
    for (int q = 0; q < NP - 1; ++q) M[q] = fm[q + 2];
  }
  fetch_tile(kc0);
  stage_tile(0);
  if (kc0 + 1 < kc1) fetch_tile(kc0 + 1);
  T unext = in[(int64_t)(kc0 + R) * sz + own];
  __syncthreads();

  for (int k = kc0; k < kc1; ++k) {
    const int cb = DB ? ((k - kc0) & 1) : 0;
    // own column: u(k+R) -> f-(k+R) now, f+(k+R)/u(k+R) after the shift
    T pn, mn;
    lf_split(unext, pn, mn);
    M[NP - 1] = mn;
    const T un = unext;
    if (k + 1 < kc1) unext = in[(int64_t)(k + 1 + R) * sz + own];

    const T fx = lds_face(cb, lc, 1);    // x face i+½
    const T fy = lds_face(cb, lc, LX);   // y face j+½
    T fyb = T(0);
    if (ty == 0) fyb = lds_face(cb, (R - 1) * LX + tx + R, LX);  // y faces jb-½ (wave 0)
    T d2x = T(0), d2y = T(0);
    const T ctr = U[R - 1];
    if constexpr (VISC) {
      d2x = FD<4>::d2(s_u[cb][lc - 2], s_u[cb][lc - 1], ctr, s_u[cb][lc + 1], s_u[cb][lc + 2]);
      d2y = FD<4>::d2(s_u[cb][lc - 2 * LX], s_u[cb][lc - LX], ctr, s_u[cb][lc + LX],
                      s_u[cb][lc + 2 * LX]);
    }
    KP[2] = w5_curv(P[2], P[3], P[4]);
    KM[2] = w5_curv(M[2], M[3], M[4]);
    const T fz_hi = w5_face_k<T, WZ>(P, M, KP, KM);
    KP[0] = KP[1];
    KP[1] = KP[2];
    KM[0] = KM[1];
    KM[1] = KM[2];
    s_fy[cb][(ty + 1) * TX + tx] = fy;
    if (ty == 0) s_fy[cb][tx] = fyb;

    if constexpr (!DB) __syncthreads();  // tile k fully read; y faces visible
    if (k + 1 < kc1) {                   // stage tile k+1 (DB: into the other buffer)
      stage_tile(DB ? cb ^ 1 : 0);
      if (k + 2 < kc1) fetch_tile(k + 2);
    }
    if constexpr (DB) __syncthreads();  // y faces of k and tile k+1 visible

    const T fyl = s_fy[cb][ty * TX + tx];
    const T fxl = wave_shr1(fx);  // face i-½ from lane l-1 (column 0: unused)
    T L = -((fx - fxl) * rdx + (fy - fyl) * rdy + (fz_hi - fz_lo) * rdz);
    if constexpr (VISC) {
      L += vx * d2x + vy * d2y + vz * FD<4>::d2(U[R - 3], U[R - 2], ctr, U[R], U[R + 1]);
    }
    if (active) {
      const int64_t o = (int64_t)k * sz + own;
      T ax = T(0);
      if constexpr (reads_aux<MODE>()) ax = aux[o];
      stage_store<T, MODE>(out, aux, o, ax, ctr, L, dt, a, b);
    }
    fz_lo = fz_hi;
#pragma unroll
    for (int q = 0; q < NP - 1; ++q) {
      P[q] = P[q + 1];
      M[q] = M[q + 1];
      U[q] = U[q + 1];
    }
    P[NP - 1] = pn;
    U[NP - 1] = un;
    if constexpr (!DB) __syncthreads();  // tile k+1 visible
  }
}

// ------------------------------------------------------------------------------
// Division helpers of the v9 stage.  Faces are carried as a multiple of the flux (the
// 1/6 or 1/3 of the candidate polynomials is folded into rd* by the launcher) and the one
// division per face is a product with a reciprocal refined by one Newton step
// (w5_combine6: 4 fp64 ops fewer per face than the IEEE-exact fast_div;
// bench/native/divtest.hip measures the variants).
// ------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T fast_div1(T n, T d) {
#pragma clang fp contract(off)
  if constexpr (std::is_same_v<T, double>) {
    T r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, T(1)), r, r);
    const T q = n * r;
    return fma(fma(-d, q, n), r, q);
  } else {
    return n / d;
  }
}

// 6 x the face flux from the two sides (w5_side numerators / weight sums): the common
// numerator times a reciprocal refined by one Newton step (relative error ~2^-46, i.e.
// ~1e-14 of the flux; fast_div1's residual correction to a correctly rounded quotient
// costs 2 more fp64 ops per face and buys nothing the scheme can see)
__device__ __forceinline__ float rcp_hw(float d) { return __builtin_amdgcn_rcpf(d); }
__device__ __forceinline__ f32x2 rcp_hw(f32x2 d) {
  return f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
// fp32 reciprocal: hardware estimate + one Newton step (~1 ulp; packed for pairs)
template <typename T>
__device__ __forceinline__ T rcp_nr(T d) {
#pragma clang fp contract(off)
  const T r = rcp_hw(d);
  return fma(fma(-d, r, T(1)), r, r);
}

// fp32 (one cell or a packed pair) keeps one reciprocal per side: S1 S2 of the JS weights
// can fall below the fp32 normal range.  The IEEE quotients of rounds 1-3 cost ~10
// unpacked ops each; the refined reciprocals are 1 + 2 (packed) ops per element and side.
template <typename T>
__device__ __forceinline__ T w5_combine6(T n1, T S1, T n2, T S2) {
#pragma clang fp contract(off)
  if constexpr (std::is_same_v<T, double>) {
    const T d = S1 * S2;
    T r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, T(1)), r, r);
    return fma(n1, S2, n2 * S1) * r;
  } else {
    return fma(n1, rcp_nr(S1), n2 * rcp_nr(S2));
  }
}

// ------------------------------------------------------------------------------
// WENO5 3-D stage, v9 (default): the v3 algorithm (63-cell x tiles, DPP left x face,
// register z column, double-buffered LDS tile, one barrier per plane) with the z rings
// rotated by renaming (march unrolled by the ring length), the tile's bottom y faces
// rotating over the waves plane by plane, and the per-plane overhead taken out:
//   * the march is unrolled by 10 planes (ring length 5 x buffer-set parity 2), so the
//     LDS buffer set of every plane is a compile-time constant: each LDS access is a
//     loop-invariant lane base + an immediate offset.  The lane's read base sits at the
//     lowest cell any of its reads touches (own cell - 2 rows - 2 columns), so every
//     offset is non-negative and fits the 16-bit DS offset (v6 spends ~15 v_add_u32
//     per plane rebuilding bases);
//   * every prefetch is unconditional: plane indices past the chunk are clamped (SALU)
//     to its last plane, so no branch and no phi copies (v_mov_b64) around the loads;
//     the extra tile staged after the last plane lands in the idle buffer set;
//   * x and y faces use w5_side_h (common.hpp): 37 instead of 41 fp64 ops per side,
//     carried as 3 x the flux; z faces keep w5_side on the z rings (6 x the flux);
//   * (round 6) a lane stages its OWN cell of the next tile from its z rings (f+, f-, u of
//     plane k+1 are already there) and only the tile's halo is loaded and split: half the
//     tile loads, one split per lane instead of two; the lane's own f+ / f- in its x and
//     y faces come from the same registers (no LDS read) — bitwise the same, in the
//     solver +2.6-3.2 % at 256^3 and +5.0-5.4 % at 512^3, where the 32 x 16 tile also
//     stopped spilling (profiles/r6/ab/burgers_own_face_ab.log; staging alone:
//     burgers_own_cell_ab.log, +1.2-1.7 %).
// Requires a plane below 2^31 bytes (v9_fits); TY = 8 only (offsets < 64 KiB).
// ------------------------------------------------------------------------------
//
// TXL: cells per tile row.  64 (default shape): one row per wave, 63 outputs per row, 8
// rows per tile.  32: each wave holds TWO 32-lane rows (lanes 0 and 32 supply a face
// only), 31 outputs per row, 16 rows per tile — the launcher picks it where it wastes
// fewer lanes on the last x tile: a 512 row has 506 active cells = 8.03 tiles of 63
// (9 tiles, 88 % of the lanes busy) but 16.3 of 31 (17 tiles, 93 %); 1024: 94 % -> 96 %.
// The 32 x 16 tile also stages fewer halo cells per output (38 x 22 / (31 x 16) = 1.69
// vs 70 x 14 / (63 x 8) = 1.94).  wave_shr1 hands lane 32 the face of lane 31 — lane 32
// is its row's face-only lane, so the DPP shift needs no change.
// PUT (round 6, slab ranks, ipc transport): the stage's output planes inside put's ranges
// are also stored into the neighbours' ghost planes (common.hpp halo_put2) — one launch per
// stage over every owned plane instead of interior + boundary + put launches.
template <typename T, bool WZ, bool VISC, int MODE, int TXL = 64, bool PK = false,
          bool PUT = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void burgers3d_w5s_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int ny, int64_t sy, int64_t sz, int k0,
    int k1, int k0b, int k1b, int gza, int zchunk, int border, T rdx3, T rdy3, T rdz6, T vx,
    T vy, T vz, T dt, T a, T b, const double* __restrict__ dtp, int xcdmap,
    HaloPut2 put = HaloPut2{}) {
  static_assert(TXL == 64 || TXL == 32, "tile row: 64 or 32 lanes");
  static_assert(!PK || std::is_same_v<T, float>, "packed pairs: fp32");
  static_assert(!(PK && PUT), "halo puts: one cell per lane");
  using V = std::conditional_t<PK, f32x2, T>;  // a lane's value: one cell or a z pair
  constexpr int NW = 8, RW = 64 / TXL;  // waves per workgroup, tile rows per wave
  constexpr int TY = NW * RW, R = 3, NR = 5, TX = TXL, TXO = TX - 1;
  constexpr int LX = TX + 2 * R, LY = TY + 2 * R, NT = 64 * NW, LT = LX * LY;
  constexpr int E = (int)sizeof(V), EG = (int)sizeof(T);  // LDS / global element bytes
  constexpr int NARR = VISC ? 3 : 2;                 // staged arrays: f+, f- [, u]
  constexpr int SET = NARR * LT + (TY + 1) * TX;     // elements per buffer set (+ y faces)
  constexpr int OM = LT * E, OU = 2 * LT * E, OFY = NARR * LT * E, SETB = SET * E;
  constexpr int XO = 2 * LX * E + 2 * E;             // own cell - lane read base
  static_assert(SETB + XO + NARR * LT * E + 3 * LX * E < 65536, "DS immediate offsets");
  __shared__ V lds[2 * SET];
  char* lb = (char*)lds;
  const W5Sgpr<V> kk;  // fp64 constants in SGPRs (VOP3 operands, no v_fmac copies)

  const int tx = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.y);
  const int tid = w * 64 + tx;
  const int col = tx % TX, row = w * RW + tx / TX;  // the lane's cell in the tile
  // xcdmap: XCD-contiguous tile order (common.hpp xcd_tile), so y-adjacent tiles — which
  // share 6 of their staged rows — run together on one XCD's L2
  const Tile3 tl = xcdmap ? xcd_tile() : Tile3{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const int ib = border - 1 + tl.x * TXO;  // x of column 0 (supplies a face only)
  const int jb = border + tl.y * TY;       // y of row 0
  const int i = ib + col, j = jb + row;
  // z chunks of the first plane range [k0, k1), then (tile z >= gza) of the second
  // [k0b, k1b): both boundary slabs of a rank in ONE launch
  const bool second = tl.z >= gza;
  const int kc0 = second ? k0b + (tl.z - gza) * zchunk : k0 + tl.z * zchunk;
  const int kc1 = min(kc0 + zchunk, second ? k1b : k1);
  // PK: the chunk's halves [kc0, kc0 + H) and [kc0 + H, kc1) march side by side, plane
  // k of the first with plane k + H of the second (the second may be one plane shorter:
  // its last iteration is then a dummy — plane indices clamped, stores dropped)
  const int H = PK ? (kc1 - kc0 + 1) / 2 : kc1 - kc0;
  const int kce = kc0 + H;  // end of the march
  const int klast = kce - 1;
  const bool active = col >= 1 && i < nx - border && j < ny - border;
  const uint32_t goff = (uint32_t)(min(j, ny - 1) * (int)sy + min(i, nx - 1)) * (uint32_t)EG;
  const int64_t szb = sz * EG;
  auto plane = [&](const T* base, int k) {
    return plane_rsrc((const char*)base + (int64_t)k * szb);
  };
  if (dtp != nullptr && !device_dt(dtp, dt)) {  // adaptive run at t_end: out = in
    if (active)
      for (int k = kc0; k < kc1; ++k) {
        const T v = gld<T>(plane(in, k), goff);
        gst<T>(plane(out, k), goff, v);
        if constexpr (PUT) halo_put2<T>(put, k, szb, goff, v);
      }
    if constexpr (PUT) __builtin_amdgcn_s_waitcnt(0);
    return;
  }
  // global load of plane k (PK: and of plane k + H, clamped to the last plane the
  // unpacked march reads) / store of plane k (PK: and k + H if it is in the chunk)
  auto gl = [&](const T* base, int k, uint32_t off) -> V {
    if constexpr (PK)
      return V{gld<T>(plane(base, k), off), gld<T>(plane(base, min(k + H, kc1 + R - 1)), off)};
    else
      return gld<T>(plane(base, k), off);
  };
  auto gs = [&](T* base, int k, V v) {
    if constexpr (PK) {
      gst<T>(plane(base, k), goff, v.x);
      if (k + H < kc1) gst<T>(plane(base, k + H), goff, v.y);
    } else {
      gst<T>(plane(base, k), goff, v);
    }
  };

  // Tile staging: a lane's OWN cell of the staged plane comes from its register z column
  // (the rings already hold f+, f- and u of planes k-2..k+2 — the same loads and the same
  // split, so the same bits); only the tile's halo — NHALO = LX LY - TX TY cells, 468 of
  // 980 for the 64 x 8 tile — is loaded and split, by the first NHALO lanes: half the tile
  // loads and one split per lane instead of two (the round-5 kernel staged every cell)
  constexpr int NHALO = LT - TX * TY;
  constexpr int NH = (NHALO + NT - 1) / NT;
  uint32_t hoff[NH];
  int hl[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    int idx = tid + h * NT;
    hl[h] = -1;
    hoff[h] = 0;
    if (idx < NHALO) {
      int ly, lx;
      if (idx < R * LX) {  // the R rows below the tile
        ly = idx / LX;
        lx = idx - ly * LX;
      } else if ((idx -= R * LX) < R * LX) {  // the R rows above it
        ly = TY + R + idx / LX;
        lx = idx % LX;
      } else {  // the R columns left and right of each tile row
        idx -= R * LX;
        ly = R + idx / (2 * R);
        const int c = idx % (2 * R);
        lx = c < R ? c : TX + c;
      }
      hl[h] = (ly * LX + lx) * E;
      hoff[h] = (uint32_t)(clampi(jb - R + ly, 0, ny - 1) * (int)sy +
                           clampi(ib - R + lx, 0, nx - 1)) * (uint32_t)EG;
    }
  }
  // loop-invariant LDS lane bases (byte addresses); everything else is an immediate
  const int lrb = ((row + R) * LX + col + R) * E - XO;  // own-cell reads (and own-cell staging)
  const int brb = col * E;                              // bottom y faces (row R-1) + its store
  const int fyb = ((row + 1) * TX + col) * E;           // y face above the own cell
  V pre[NH];
  auto fetch_tile = [&](int k) {  // the halo of plane k
#pragma unroll
    for (int h = 0; h < NH; ++h) pre[h] = gl(in, k, hoff[h]);
  };
  // SB: byte offset of the buffer set; op, om, ou: the own cell's f+, f-, u (ring values)
  auto stage_tile = [&]<int SB>(V op, V om, V ou) {
    lds_st<V>(lb + lrb, SB + XO, op);
    lds_st<V>(lb + lrb, SB + OM + XO, om);
    if constexpr (VISC) lds_st<V>(lb + lrb, SB + OU + XO, ou);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      if (hl[h] >= 0) {
        V p, m;
        lf_split(pre[h], p, m);
        lds_st<V>(lb + hl[h], SB, p);
        lds_st<V>(lb + hl[h], SB + OM, m);
        if constexpr (VISC) lds_st<V>(lb + hl[h], SB + OU, pre[h]);
      }
    }
  };
  // 3 x flux at the face to the right of the cell at immediate offset c (relative to the
  // base pointer bp) along stride st.  own_face3: the cell is the lane's own, whose f+ and
  // f- (op, om: the ring values) need no LDS read
  auto lds_face3 = [&](const char* bp, int c, int st) {
    V pv[5], mv[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      pv[d] = lds_ld<V>(bp, c + (d - 2) * st);
      mv[d] = lds_ld<V>(bp, c + OM + (d - 1) * st);
    }
    V n1, S1, n2, S2;
    w5_face3_sides<V, WZ>(pv, mv, n1, S1, n2, S2, kk);
    return w5_combine6(n1, S1, n2, S2);
  };
  auto own_face3 = [&](const char* bp, int c, int st, V op, V om) {
    V pv[5], mv[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      pv[d] = d == 2 ? op : lds_ld<V>(bp, c + (d - 2) * st);
      mv[d] = d == 1 ? om : lds_ld<V>(bp, c + OM + (d - 1) * st);
    }
    V n1, S1, n2, S2;
    w5_face3_sides<V, WZ>(pv, mv, n1, S1, n2, S2, kk);
    return w5_combine6(n1, S1, n2, S2);
  };

  // ---- rings: plane p lives in slot (p - kc0 + 2 NR) % NR ----
  V rp[NR], rm[NR], ru[NR], cp[NR], cm[NR], fz[NR];  // f+, f-, u, C(f+), C(f-), 6 x z face
  {
    V uz[2 * R], fp[2 * R], fm[2 * R];  // planes kc0-3 .. kc0+2
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) {
      uz[q] = gl(in, kc0 - R + q, goff);
      lf_split(uz[q], fp[q], fm[q]);
    }
    auto sl = [](int p) { return (p + 2 * NR) % NR; };  // slot of plane kc0 + p
    {  // face kc0-½: the march's z-face arithmetic (bit-identical to it)
      V n1, S1, n2, S2;
      w5_side<V, WZ>(fp[0], fp[1], fp[2], fp[3], fp[4], w5_curv(fp[0], fp[1], fp[2], kk),
                     w5_curv(fp[1], fp[2], fp[3], kk), w5_curv(fp[2], fp[3], fp[4], kk), n1, S1, kk);
      w5_side<V, WZ>(fm[5], fm[4], fm[3], fm[2], fm[1], w5_curv(fm[5], fm[4], fm[3], kk),
                     w5_curv(fm[4], fm[3], fm[2], kk), w5_curv(fm[3], fm[2], fm[1], kk), n2, S2, kk);
      fz[sl(-1)] = w5_combine6(n1, S1, n2, S2);
    }
    cp[sl(-1)] = w5_curv(fp[1], fp[2], fp[3], kk);
    cp[sl(0)] = w5_curv(fp[2], fp[3], fp[4], kk);
    cm[sl(0)] = w5_curv(fm[2], fm[3], fm[4], kk);
    cm[sl(1)] = w5_curv(fm[3], fm[4], fm[5], kk);
#pragma unroll
    for (int q = 1; q < 2 * R; ++q) {  // planes kc0-2 .. kc0+2
      rp[sl(q - R)] = fp[q];
      ru[sl(q - R)] = uz[q];
    }
#pragma unroll
    for (int q = 2; q < 2 * R; ++q) rm[sl(q - R)] = fm[q];  // kc0-1 .. kc0+2
  }
  fetch_tile(kc0);
  stage_tile.template operator()<0>(rp[0], rm[0], ru[0]);  // plane kc0: ring slot 0
  fetch_tile(min(kc0 + 1, klast));
  V un = gl(in, kc0 + R, goff);  // u(k+3) of the current iteration
  V ax = V(0);
  if constexpr (reads_aux<MODE>()) ax = gl(aux, kc0, goff);
  __syncthreads();

  auto body = [&]<int PH>(int k) {
    auto sl = [](int d) { return (PH + d + 2 * NR) % NR; };  // slot of plane k + d
    constexpr int SB = (PH & 1) * SETB, SBN = SETB - SB;    // this / the other set
    // new plane k+3 of the own column: f-(k+3) now; f+(k+3) and u(k+3) after their use
    V pn, mn;
    lf_split(un, pn, mn);
    rm[sl(3)] = mn;
    const V unew = un;
    un = gl(in, min(k + 1, klast) + R, goff);
    V axk = ax;
    if constexpr (reads_aux<MODE>()) ax = gl(aux, min(k + 1, klast), goff);

    const V fy = own_face3(lb + lrb, SB + XO, LX * E, rp[sl(0)], rm[sl(0)]);  // y face j+½
    if (w == (k - kc0) % NW)  // the tile's bottom y faces rotate over the waves
      // (TXL 32: both rows of the wave compute them; identical values, same slots)
      lds_st<V>(lb + brb, SB + OFY, lds_face3(lb + brb, SB + ((R - 1) * LX + R) * E, LX * E));
    lds_st<V>(lb + fyb, SB + OFY, fy);
    const V ctr = ru[sl(0)];
    V d2x = V(0), d2y = V(0), d2z = V(0);
    const V fx = own_face3(lb + lrb, SB + XO, E, rp[sl(0)], rm[sl(0)]);  // x face i+½
    if constexpr (VISC) {
      const int c = SB + OU + XO;
      const char* bp = lb + lrb;
      d2x = fd4_d2k(lds_ld<V>(bp, c - 2 * E), lds_ld<V>(bp, c - E), ctr,
                    lds_ld<V>(bp, c + E), lds_ld<V>(bp, c + 2 * E), kk);
      d2y = fd4_d2k(lds_ld<V>(bp, c - 2 * LX * E), lds_ld<V>(bp, c - LX * E), ctr,
                    lds_ld<V>(bp, c + LX * E), lds_ld<V>(bp, c + 2 * LX * E), kk);
      d2z = fd4_d2k(ru[sl(-2)], ru[sl(-1)], ctr, ru[sl(1)], ru[sl(2)], kk);
    }
    cp[sl(1)] = w5_curv(rp[sl(0)], rp[sl(1)], rp[sl(2)], kk);
    cm[sl(2)] = w5_curv(rm[sl(1)], rm[sl(2)], rm[sl(3)], kk);
    {
      V n1, S1, n2, S2;
      w5_side<V, WZ>(rp[sl(-2)], rp[sl(-1)], rp[sl(0)], rp[sl(1)], rp[sl(2)], cp[sl(-1)],
                     cp[sl(0)], cp[sl(1)], n1, S1, kk);
      w5_side<V, WZ>(rm[sl(3)], rm[sl(2)], rm[sl(1)], rm[sl(0)], rm[sl(-1)], cm[sl(2)],
                     cm[sl(1)], cm[sl(0)], n2, S2, kk);
      fz[sl(0)] = w5_combine6(n1, S1, n2, S2);  // face k+½
    }

    // stage tile k+1 into the other buffer set, fetch tile k+2 (past the chunk: its last
    // plane again, staged into the idle set and never read)
    stage_tile.template operator()<SBN>(rp[sl(1)], rm[sl(1)], ru[sl(1)]);
    fetch_tile(min(k + 2, klast));
    __syncthreads();  // y faces of k and tile k+1 visible

    const V fyl = lds_ld<V>(lb + fyb, SB + OFY - TX * E);
    const V fxl = wave_shr1(fx);  // face i-½ from lane l-1 (column 0: unused)
    // explicit fma, no contraction left to the compiler: the packed (f32x2) and the
    // scalar instances must round alike (fast contraction fused this sum differently in
    // the two, 1 ulp apart: round-5 test_burgers3d_fp32_packed_pairs)
    V L;
    {
#pragma clang fp contract(off)
      L = -fma(fz[sl(0)] - fz[sl(-1)], rdz6, fma(fx - fxl, rdx3, (fy - fyl) * rdy3));
      if constexpr (VISC) L = fma(vx, d2x, fma(vy, d2y, fma(vz, d2z, L)));
    }
    V dnew = V(0);
    const V v = stage_value<V, MODE>(axk, ctr, L, V(dt), V(a), V(b), dnew);
    if (active) {
      gs(out, k, v);
      if constexpr (PUT) halo_put2<V>(put, k, szb, goff, v);
      if constexpr (MODE == kLs1 || MODE == kLs) gs(aux, k, dnew);
    }
    rp[sl(3)] = pn;  // f+(k+3), u(k+3) replace f+(k-2), u(k-2)
    ru[sl(3)] = unew;
  };
  for (int kb = kc0; kb < kce; kb += 2 * NR) {
    [&]<int... P>(std::integer_sequence<int, P...>) {
      (void)((kb + P < kce ? (body.template operator()<P>(kb + P), true) : false) && ...);
    }(std::make_integer_sequence<int, 2 * NR>{});
  }
  // every peer store of this wave acknowledged before the wave (and the dispatch) ends
  if constexpr (PUT) __builtin_amdgcn_s_waitcnt(0);
}

template <typename T, int W, bool WZ, bool VISC, int MODE, int TX>
__global__ __launch_bounds__(TX) void burgers2d_stage_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int64_t sy, int j0, int j1, int ychunk,
    int border, T rdx, T rdy, T vx, T vy, T dt, T a, T b, const double* __restrict__ dtp) {
  using Rc = Recon<T, W, WZ>;
  constexpr int R = Rc::R, NP = 2 * R - 1, LX = TX + 2 * R;
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
  if (dtp != nullptr && !device_dt(dtp, dt)) {  // adaptive run at t_end: out = in
    if (active)
      for (int jj = jc0; jj < jc1; ++jj) out[(int64_t)jj * sy + i] = in[(int64_t)jj * sy + i];
    return;
  }
  const int g0 = clampi(i0 - R + tx, 0, nx - 1);
  const int g1 = clampi(i0 - R + TX + tx, 0, nx - 1);

  T pre0, pre1 = T(0);
  auto fetch_row = [&](int jj) {
    const T* src = in + (int64_t)jj * sy;
    pre0 = src[g0];
    if (tx < 2 * R) pre1 = src[g1];
  };
  auto lds_face = [&](int c) {
    T pv[NP], mv[NP];
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      pv[d] = s_p[c + d - R + 1];
      mv[d] = s_m[c + d - R + 2];
    }
    return Rc::face(pv, mv);
  };

  T P[NP], M[NP], U[NP];
  T fy_lo;
  {
    T uy[2 * R], fp[2 * R], fm[2 * R];
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) {
      uy[q] = in[(int64_t)(jc0 - R + q) * sy + ic];
      lf_split(uy[q], fp[q], fm[q]);
    }
    fy_lo = Rc::face(fp, fm + 1);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      P[q] = fp[q + 1];
      U[q] = uy[q + 1];
    }
#pragma unroll
    for (int q = 0; q < NP - 1; ++q) M[q] = fm[q + 2];
  }
  fetch_row(jc0);
  T unext = in[(int64_t)(jc0 + R) * sy + ic];

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
    M[NP - 1] = mn;
    const T un = unext;
    if (jj + 1 < jc1) {
      fetch_row(jj + 1);
      unext = in[(int64_t)(jj + 1 + R) * sy + ic];
    }
    __syncthreads();
    s_fx[tx + 1] = lds_face(lc);
    if (tx == TX - 1) s_fx[0] = lds_face(R - 1);  // left face i0-½ (last wave, one lane)
    const T fy_hi = Rc::face(P, M);
    __syncthreads();
    const T ctr = s_u[lc];
    T L = -((s_fx[tx + 1] - s_fx[tx]) * rdx + (fy_hi - fy_lo) * rdy);
    if constexpr (VISC) {
      L += vx * FD<4>::d2(s_u[lc - 2], s_u[lc - 1], ctr, s_u[lc + 1], s_u[lc + 2]) +
           vy * FD<4>::d2(U[R - 3], U[R - 2], ctr, U[R], U[R + 1]);
    }
    if (active) {
      const int64_t o = (int64_t)jj * sy + i;
      T ax = T(0);
      if constexpr (reads_aux<MODE>()) ax = aux[o];
      stage_store<T, MODE>(out, aux, o, ax, ctr, L, dt, a, b);
    }
    fy_lo = fy_hi;
#pragma unroll
    for (int q = 0; q < NP - 1; ++q) {
      P[q] = P[q + 1];
      M[q] = M[q + 1];
      U[q] = U[q + 1];
    }
    P[NP - 1] = pn;
    U[NP - 1] = un;
  }
}

// ------------------------------------------------------------------------------
// WENO5 2-D stage, v2 (default for WENO5-JS/Z in 2-D): every wave is independent — no
// __syncthreads at all.  A wave owns a 64-column strip (lane 0 supplies the left face of
// the strip only, lanes 1..63 are output cells: 63-cell strips anchored at the active
// region, as the 3-D v9 x tiles) and marches along y:
//   * y faces from the lane's own register column (rings of f+, f-, u and the scaled
//     curvatures, two of three curvatures per side carried from the previous row; the
//     march is unrolled by the ring length, so the rings rotate by renaming);
//   * x faces: the row's split fluxes (and u for the viscous term) go to a WAVE-PRIVATE
//     LDS row of 64 + 5 halo cells (5 lanes also stage one halo column each); a lane reads
//     f+(x-2..x+2) / f-(x-1..x+3) and computes the face to the right of its cell with the
//     v9 x-face form (w5_side_h, 37 fp64 ops per side, one reciprocal per face); the face
//     to its left arrives from lane l-1 by one DPP shift (the old kernel: 3 barriers per
//     row, the left face of the 256-lane tile computed by a single lane, two full
//     divisions per face);
//   * LDS writes and reads of one wave are executed in order, and a compiler fence keeps
//     them in program order, so the row needs no barrier (and, written after the previous
//     row's reads were issued, no second buffer);
//   * global loads: u(j+3) of the own column and the halo lane's column of row j+1, one
//     row ahead; plane-free 32-bit byte offsets through a buffer descriptor per launch.
// Per interior cell and stage ~170 fp64 lane-ops inviscid: the 3-D v9 stage's cost per
// direction (tests: bitwise P-rank == 1-rank, fp64 reference to rounding).
// ------------------------------------------------------------------------------
template <typename T, bool WZ, bool VISC, int MODE>
__global__ __launch_bounds__(256) void burgers2d_w5_kernel(
    const T* __restrict__ in, T* aux, T* out, int nx, int64_t sy, int j0, int j1, int ychunk,
    int border, T rdx3, T rdy6, T vx, T vy, T dt, T a, T b, const double* __restrict__ dtp) {
  constexpr int R = 3, NR = 5, TXO = 63, NW = 4;
  constexpr int LW = 64 + 5;  // x = ib-2 .. ib+66
  constexpr int NARR = VISC ? 3 : 2;
  __shared__ T lds[NW][NARR][LW];
  const W5Sgpr<T> kk;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int ib = border - 1 + ((int)blockIdx.x * NW + w) * TXO;  // x of lane 0
  if (ib + 1 >= nx - border) return;  // a strip past the active region: wave-uniform exit
  const int jc0 = j0 + (int)blockIdx.y * ychunk;
  const int jc1 = min(jc0 + ychunk, j1);
  const int jlast = jc1 - 1;
  const int i = ib + lane;
  const bool active = lane >= 1 && i < nx - border;
  const int E = (int)sizeof(T);
  const uint32_t goff = (uint32_t)min(i, nx - 1) * (uint32_t)E;
  // halo lanes 0..4 also stage x = ib-2, ib-1, ib+64, ib+65, ib+66
  const bool hl = lane < 5;
  const int hx = lane < 2 ? ib - 2 + lane : ib + 62 + lane;
  const int hslot = lane < 2 ? lane : 64 + lane;
  const uint32_t hoff = (uint32_t)clampi(hx, 0, nx - 1) * (uint32_t)E;
  const int64_t syb = sy * E;
  auto row = [&](const T* base, int j) { return plane_rsrc((const char*)base + (int64_t)j * syb); };
  if (dtp != nullptr && !device_dt(dtp, dt)) {  // adaptive run at t_end: out = in
    if (active)
      for (int j = jc0; j < jc1; ++j) gst<T>(row(out, j), goff, gld<T>(row(in, j), goff));
    return;
  }
  T* sp = lds[w][0];
  T* sm = lds[w][1];
  T* su = VISC ? lds[w][NARR - 1] : nullptr;

  // ---- rings: row p lives in slot (p - jc0 + 2 NR) % NR ----
  T rp[NR], rm[NR], ru[NR], cp[NR], cm[NR], fy[NR];  // f+, f-, u, C(f+), C(f-), 6 x y face
  {
    T uy[2 * R], fp[2 * R], fm[2 * R];  // rows jc0-3 .. jc0+2
#pragma unroll
    for (int q = 0; q < 2 * R; ++q) {
      uy[q] = gld<T>(row(in, jc0 - R + q), goff);
      lf_split(uy[q], fp[q], fm[q]);
    }
    auto sl = [](int p) { return (p + 2 * NR) % NR; };
    {  // face jc0-½: the march's y-face arithmetic (bit-identical to it)
      T n1, S1, n2, S2;
      w5_side<T, WZ>(fp[0], fp[1], fp[2], fp[3], fp[4], w5_curv(fp[0], fp[1], fp[2], kk),
                     w5_curv(fp[1], fp[2], fp[3], kk), w5_curv(fp[2], fp[3], fp[4], kk), n1, S1, kk);
      w5_side<T, WZ>(fm[5], fm[4], fm[3], fm[2], fm[1], w5_curv(fm[5], fm[4], fm[3], kk),
                     w5_curv(fm[4], fm[3], fm[2], kk), w5_curv(fm[3], fm[2], fm[1], kk), n2, S2, kk);
      fy[sl(-1)] = w5_combine6(n1, S1, n2, S2);
    }
    cp[sl(-1)] = w5_curv(fp[1], fp[2], fp[3], kk);
    cp[sl(0)] = w5_curv(fp[2], fp[3], fp[4], kk);
    cm[sl(0)] = w5_curv(fm[2], fm[3], fm[4], kk);
    cm[sl(1)] = w5_curv(fm[3], fm[4], fm[5], kk);
#pragma unroll
    for (int q = 1; q < 2 * R; ++q) {  // rows jc0-2 .. jc0+2
      rp[sl(q - R)] = fp[q];
      ru[sl(q - R)] = uy[q];
    }
#pragma unroll
    for (int q = 2; q < 2 * R; ++q) rm[sl(q - R)] = fm[q];  // jc0-1 .. jc0+2
  }
  T un = gld<T>(row(in, jc0 + R), goff);  // u(j+3) of the current row
  T hv = gld<T>(row(in, jc0), hoff);       // the halo column of the current row
  T ax = T(0);
  if constexpr (reads_aux<MODE>()) ax = gld<T>(row(aux, jc0), goff);

  auto body = [&]<int PH>(int j) {
    auto sl = [](int d) { return (PH + d + 2 * NR) % NR; };  // slot of row j + d
    // new row j+3 of the own column: f-(j+3) now; f+(j+3) and u(j+3) after their use
    T pn, mn;
    lf_split(un, pn, mn);
    rm[sl(3)] = mn;
    const T unew = un;
    const T hcur = hv;
    const int jn = min(j + 1, jlast);
    un = gld<T>(row(in, jn + R), goff);
    hv = gld<T>(row(in, jn), hoff);
    T axk = ax;
    if constexpr (reads_aux<MODE>()) ax = gld<T>(row(aux, jn), goff);

    // the row j into the wave's LDS row (own cell + one halo cell on lanes 0..4)
    const T ctr = ru[sl(0)];
    sp[lane + 2] = rp[sl(0)];
    sm[lane + 2] = rm[sl(0)];
    if constexpr (VISC) su[lane + 2] = ctr;
    if (hl) {
      T hp, hm;
      lf_split(hcur, hp, hm);
      sp[hslot] = hp;
      sm[hslot] = hm;
      if constexpr (VISC) su[hslot] = hcur;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // stores before the reads
    T pv[5], mv[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      pv[d] = sp[lane + d];      // f+(x-2 .. x+2)
      mv[d] = sm[lane + 1 + d];  // f-(x-1 .. x+3)
    }
    T d2x = T(0), d2y = T(0);
    if constexpr (VISC) {
      d2x = fd4_d2k(su[lane], su[lane + 1], ctr, su[lane + 3], su[lane + 4], kk);
      d2y = fd4_d2k(ru[sl(-2)], ru[sl(-1)], ctr, ru[sl(1)], ru[sl(2)], kk);
    }
    T fx;
    {
      T n1, S1, n2, S2;
      w5_face3_sides<T, WZ>(pv, mv, n1, S1, n2, S2, kk);
      fx = w5_combine6(n1, S1, n2, S2);  // 3 x flux at x+½
    }
    cp[sl(1)] = w5_curv(rp[sl(0)], rp[sl(1)], rp[sl(2)], kk);
    cm[sl(2)] = w5_curv(rm[sl(1)], rm[sl(2)], rm[sl(3)], kk);
    {
      T n1, S1, n2, S2;
      w5_side<T, WZ>(rp[sl(-2)], rp[sl(-1)], rp[sl(0)], rp[sl(1)], rp[sl(2)], cp[sl(-1)],
                     cp[sl(0)], cp[sl(1)], n1, S1, kk);
      w5_side<T, WZ>(rm[sl(3)], rm[sl(2)], rm[sl(1)], rm[sl(0)], rm[sl(-1)], cm[sl(2)],
                     cm[sl(1)], cm[sl(0)], n2, S2, kk);
      fy[sl(0)] = w5_combine6(n1, S1, n2, S2);  // 6 x flux at j+½
    }
    const T fxl = wave_shr1(fx);  // face x-½ from lane l-1 (lane 0: unused)
    T L = -((fx - fxl) * rdx3 + (fy[sl(0)] - fy[sl(-1)]) * rdy6);
    if constexpr (VISC) L += vx * d2x + vy * d2y;
    T dnew = T(0);
    const T v = stage_value<T, MODE>(axk, ctr, L, dt, a, b, dnew);
    if (active) {
      gst<T>(row(out, j), goff, v);
      if constexpr (MODE == kLs1 || MODE == kLs) gst<T>(row(aux, j), goff, dnew);
    }
    rp[sl(3)] = pn;  // f+(j+3), u(j+3) replace f+(j-2), u(j-2)
    ru[sl(3)] = unew;
  };
  for (int jb = jc0; jb < jc1; jb += NR) {
    [&]<int... P>(std::integer_sequence<int, P...>) {
      (void)((jb + P < jc1 ? (body.template operator()<P>(jb + P), true) : false) && ...);
    }(std::make_integer_sequence<int, NR>{});
  }
}

// ------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------
constexpr int kBTX3 = 64, kBTY3 = 8;
constexpr int kBTX2 = 256;

struct BArgs {
  const void* in;
  void* aux;
  void* out;
  int nx, ny;
  int64_t sy, sz;
  int lo, hi, border;  // marched-axis range [lo, hi)
  double rdx, rdy, rdz, vx, vy, vz, dt, a, b;
  hipStream_t st;
  const double* dtp;  // device dt (adaptive CFL) or nullptr: use dt
  int lo2 = 0, hi2 = 0;  // optional second marched-axis range (3-D: v9 in the same launch)
};

// generic scheme kernel (WENO7; 64 x 8 tiles)
template <typename T, int W, bool WZ, bool VISC, int MODE>
static hipError_t launch_b3_generic(const BArgs& p) {
  const int gx = div_up(p.nx, kBTX3), gy = div_up(p.ny, kBTY3);
  const int zc = pick_chunk(p.hi - p.lo, (long long)gx * gy, 8, 256);
  const int gz = div_up(p.hi - p.lo, zc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers3d_stage_kernel<T, W, WZ, VISC, MODE, kBTX3, kBTY3>),
                     dim3(gx, gy, gz), dim3(kBTX3, kBTY3, 1), 0, p.st, (const T*)p.in,
                     (T*)p.aux, (T*)p.out, p.nx, p.ny, p.sy, p.sz, p.lo, p.hi, zc, p.border,
                     T(p.rdx), T(p.rdy), T(p.rdz), T(p.vx * s), T(p.vy * s), T(p.vz * s),
                     T(p.dt), T(p.a), T(p.b), p.dtp);
  return hipGetLastError();
}

// v3: 63-cell x tiles, double-buffered LDS tile, 64-bit addressing (planes of any size)
template <typename T, bool WZ, bool VISC, int MODE>
static hipError_t launch_b3_v3(const BArgs& p) {
  const int gx = div_up(std::max(p.nx - 2 * p.border, 1), 63);
  const int gy = div_up(std::max(p.ny - 2 * p.border, 1), kBTY3);
  const int zc = pick_chunk(p.hi - p.lo, (long long)gx * gy, 8, 256);
  const int gz = div_up(p.hi - p.lo, zc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers3d_w5_kernel<T, WZ, VISC, MODE, kBTY3, true, 4>), dim3(gx, gy, gz),
                     dim3(64, kBTY3, 1), 0, p.st, (const T*)p.in, (T*)p.aux, (T*)p.out, p.nx,
                     p.ny, p.sy, p.sz, p.lo, p.hi, zc, p.border, T(p.rdx), T(p.rdy), T(p.rdz),
                     T(p.vx * s), T(p.vy * s), T(p.vz * s), T(p.dt), T(p.a), T(p.b), p.dtp);
  return hipGetLastError();
}

// busy share of the lanes of a tiling: `act` active cells in tiles of `per` outputs of
// `lanes` lanes each
static double lane_share(int act, int per, int lanes) {
  act = std::max(act, 1);
  return (double)act / ((double)div_up(act, per) * lanes);
}

// v9 tile row width for an nx x ny plane (ADVDIFF_B3_TX / advdiff_set_b3_tx = 64 / 32
// forces one, 0 = auto): the shape with the larger share of busy lanes over x and y, the
// 64-wide one on a tie
static int g_b3_tx = -1;
static int b3_tx() {
  if (g_b3_tx < 0) g_b3_tx = knob("B3_TX", 0);
  return g_b3_tx;
}
static int b3_tile_row(int nx, int ny, int border) {
  const int forced = b3_tx();
  if (forced == 64 || forced == 32) return forced;
  const int ax = nx - 2 * border, ay = ny - 2 * border;
  const double s64 = lane_share(ax, 63, 64) * lane_share(ay, 8, 8);
  const double s32 = lane_share(ax, 31, 32) * lane_share(ay, 16, 16);
  return s32 > s64 * 1.01 ? 32 : 64;
}

// forced z-chunk length of the v9 stage (advdiff_set_b3_zchunk; 0 = the rounds model):
// the bit-reproducibility tests move the chunk boundaries with it
static int g_b3_zchunk = 0;

template <typename T, bool WZ, bool VISC, int MODE, int TXL, bool PK = false, bool PUT = false>
static hipError_t launch_b3_v9_tx(const BArgs& p, const HaloPut2& put = HaloPut2{}) {
  // XCD-contiguous tile order (always, its switch removed in round 6): 256^3 WENO5-Z +
  // viscous step 0.584 -> 0.564 ms (+3.7 %, 3 interleaved rounds, bitwise identical;
  // profiles/archive/burgers3d_xcd_r2.log)
  constexpr int xcdmap = 1;
  constexpr int TY = 8 * (64 / TXL);
  const int gx = div_up(std::max(p.nx - 2 * p.border, 1), TXL - 1);
  const int gy = div_up(std::max(p.ny - 2 * p.border, 1), TY);
  const int na = std::max(p.hi - p.lo, 0), nb = std::max(p.hi2 - p.lo2, 0);
  // z chunks by the rounds model of the fused heat step (launch.hpp pick_chunk_rounds:
  // resident workgroups = CUs x occupancy, cost = rounds x (chunk + warm-up)).  The old
  // target-count rule (removed in round 6) gave 512^3 two chunks of 253 planes = 1088
  // workgroups for 512 resident slots: a third round with 64 workgroups alone on the chip.
  const int per_cu =
      occupancy_per_cu((const void*)burgers3d_w5s_kernel<T, WZ, VISC, MODE, TXL, PK, PUT>, 512);
  // PK: a workgroup marches two half chunks side by side — choose the half length
  const int nm = PK ? div_up(na + nb, 2) : na + nb;
  const int zm = g_b3_zchunk > 0 ? std::max(1, PK ? div_up(g_b3_zchunk, 2) : g_b3_zchunk)
                                 : pick_chunk_rounds(nm, (long long)gx * gy,
                                                     (long long)device_cus() * per_cu, 4, 8);
  const int zc = PK ? 2 * zm : zm;
  const int gza = div_up(na, zc);
  const int gz = gza + div_up(nb, zc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers3d_w5s_kernel<T, WZ, VISC, MODE, TXL, PK, PUT>), dim3(gx, gy, gz),
                     dim3(64, 8, 1), 0, p.st, (const T*)p.in, (T*)p.aux, (T*)p.out, p.nx, p.ny,
                     p.sy, p.sz, p.lo, p.hi, p.lo2, p.hi2, gza, zc, p.border, T(p.rdx / 3.0),
                     T(p.rdy / 3.0), T(p.rdz / 6.0), T(p.vx * s), T(p.vy * s), T(p.vz * s),
                     T(p.dt), T(p.a), T(p.b), p.dtp, xcdmap, put);
  return hipGetLastError();
}

// the stage with fused halo puts: fp64, WENO5 (JS / Z), SSP-RK3 epilogues, one range
template <bool WZ, bool VISC, int MODE>
static hipError_t launch_b3_put(const BArgs& p, const HaloPut2& put) {
  if (b3_tile_row(p.nx, p.ny, p.border) == 32)
    return launch_b3_v9_tx<double, WZ, VISC, MODE, 32, false, true>(p, put);
  return launch_b3_v9_tx<double, WZ, VISC, MODE, 64, false, true>(p, put);
}

// fp32: packed pairs (two z half chunks per lane, v_pk_* arithmetic) by default;
// ADVDIFF_B3_PACK=0 / advdiff_set_b3_pack(0) runs one cell per lane.  Both give the same
// bits (the pair elements take the scalar operation sequence; tests/test_kernels_gpu.py).
static int g_b3_pack = -1;
static int b3_pack() {
  if (g_b3_pack < 0) g_b3_pack = knob("B3_PACK", 1);
  return g_b3_pack;
}

template <typename T, bool WZ, bool VISC, int MODE>
static hipError_t launch_b3_v9(const BArgs& p) {
  const bool tx32 = b3_tile_row(p.nx, p.ny, p.border) == 32;
  if constexpr (std::is_same_v<T, float>) {
    if (b3_pack()) {
      if (tx32) return launch_b3_v9_tx<T, WZ, VISC, MODE, 32, true>(p);
      return launch_b3_v9_tx<T, WZ, VISC, MODE, 64, true>(p);
    }
  }
  if (tx32) return launch_b3_v9_tx<T, WZ, VISC, MODE, 32>(p);
  return launch_b3_v9_tx<T, WZ, VISC, MODE, 64>(p);
}

// (Round-3 A/B, rejected: the wave computing a plane's extra bottom faces raising its
// s_setprio for that plane — 233.9 vs 217.2 us per 256^3 stage, profiles/burgers_ab_r3.log.)

// v9 addresses a plane with 32-bit byte offsets
template <typename T>
static bool v9_fits(const BArgs& p) {
  return (int64_t)p.sy * p.ny * (int64_t)sizeof(T) < (int64_t(1) << 31);
}

// 3-D WENO5 kernel version (ADVDIFF_B3_VER / advdiff_set_b3_ver): 9 (default) = the v9
// kernel (ring renaming, compile-time LDS sets, unconditional prefetches, SGPR constants,
// w5_side_h x/y faces: 256^3 WENO5-Z + viscous stage 195 us, 290 lane-ops per cell,
// profiles/archive/burgers_v9_r2.md); 3 = v3 (double-buffered tile, one barrier per plane, 242
// us), also the fallback for planes of 2 GiB and more.  The round-1/2 variants v1, v2,
// v4-v8 and the 16-row tiles were removed after their A/Bs (profiles/archive/burgers_variants_r2.log,
// profiles/archive/burgers_v6_r2.md, docs/DESIGN.md); WENO7 runs the generic scheme kernel.
static int g_b3_ver = -1;
static int b3_ver() {
  if (g_b3_ver < 0) g_b3_ver = knob("B3_VER", 9);
  return g_b3_ver;
}

template <typename T, int W, bool WZ, bool VISC, int MODE>
static hipError_t launch_b3(const BArgs& p) {
  if constexpr (W == 5) {
    if (b3_ver() == 9 && v9_fits<T>(p)) return launch_b3_v9<T, WZ, VISC, MODE>(p);
    return launch_b3_v3<T, WZ, VISC, MODE>(p);
  } else {
    return launch_b3_generic<T, W, WZ, VISC, MODE>(p);
  }
}

// 2-D WENO5 kernel version (ADVDIFF_B2_VER / advdiff_set_b2_ver): 2 (default) = the
// barrier-free wave-strip kernel (burgers2d_w5_kernel), 1 = the generic row-tile kernel
// (three barriers per row; WENO7 always runs it).
static int g_b2_ver = -1;
static int b2_ver() {
  if (g_b2_ver < 0) g_b2_ver = knob("B2_VER", 2);
  return g_b2_ver;
}

template <typename T, bool WZ, bool VISC, int MODE>
static hipError_t launch_b2_w5(const BArgs& p) {
  const int strips = div_up(std::max(p.nx - 2 * p.border, 1), 63);
  const int gx = div_up(strips, 4);
  const int yc = pick_chunk(p.hi - p.lo, gx, 1, 256);
  const int gy = div_up(p.hi - p.lo, yc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers2d_w5_kernel<T, WZ, VISC, MODE>), dim3(gx, gy, 1), dim3(256, 1, 1),
                     0, p.st, (const T*)p.in, (T*)p.aux, (T*)p.out, p.nx, p.sy, p.lo, p.hi, yc,
                     p.border, T(p.rdx / 3.0), T(p.rdy / 6.0), T(p.vx * s), T(p.vy * s), T(p.dt),
                     T(p.a), T(p.b), p.dtp);
  return hipGetLastError();
}

template <typename T, int W, bool WZ, bool VISC, int MODE>
static hipError_t launch_b2(const BArgs& p) {
  if constexpr (W == 5) {
    // rows are addressed with 32-bit byte offsets inside a row (sy elements)
    if (b2_ver() == 2 && (int64_t)p.sy * (int64_t)sizeof(T) < (int64_t(1) << 31))
      return launch_b2_w5<T, WZ, VISC, MODE>(p);
  }
  const int gx = div_up(p.nx, kBTX2);
  // fewest rows per y chunk: 1 — small grids (the reference's 400x406 rows) are latency-
  // bound, and a wave walking fewer rows in sequence wins there (400x406 WENO5-JS step
  // 23.4 -> 20.4 us with 4 -> 1, profiles/archive/small2d_r2.log); from ~1000^2 up the chunk
  // comes from the block target and this floor is inactive
  const int yc = pick_chunk(p.hi - p.lo, gx, 1, 256);
  const int gy = div_up(p.hi - p.lo, yc);
  const double s = 1.0 / 12.0;
  hipLaunchKernelGGL((burgers2d_stage_kernel<T, W, WZ, VISC, MODE, kBTX2>), dim3(gx, gy, 1),
                     dim3(kBTX2, 1, 1), 0, p.st, (const T*)p.in, (T*)p.aux, (T*)p.out, p.nx,
                     p.sy, p.lo, p.hi, yc, p.border, T(p.rdx), T(p.rdy), T(p.vx * s),
                     T(p.vy * s), T(p.dt), T(p.a), T(p.b), p.dtp);
  return hipGetLastError();
}

// runtime (scheme, viscous, mode) -> template instance
template <typename T, bool THREE_D, int W, bool WZ, bool VISC>
static hipError_t by_mode(int mode, const BArgs& p) {
#define BM(M) return THREE_D ? launch_b3<T, W, WZ, VISC, M>(p) : launch_b2<T, W, WZ, VISC, M>(p)
  switch (mode) {
    case kSsp1: BM(kSsp1);
    case kSsp: BM(kSsp);
    case kLs1: BM(kLs1);
    default: BM(kLs);
  }
#undef BM
}

template <typename T, bool THREE_D, int W, bool WZ>
static hipError_t by_visc(bool visc, int mode, const BArgs& p) {
  return visc ? by_mode<T, THREE_D, W, WZ, true>(mode, p)
              : by_mode<T, THREE_D, W, WZ, false>(mode, p);
}

template <typename T, bool THREE_D>
static hipError_t dispatch_b(int scheme, bool visc, int mode, const BArgs& p) {
  switch (scheme) {
    case 0: return by_visc<T, THREE_D, 5, false>(visc, mode, p);
    case 1: return by_visc<T, THREE_D, 5, true>(visc, mode, p);
    case 2: return by_visc<T, THREE_D, 7, false>(visc, mode, p);
    default: return hipErrorInvalidValue;
  }
}

static int scheme_radius(int scheme) { return scheme == 2 ? 4 : 3; }

static hipError_t run_b(int dtype, bool three_d, int scheme, bool ls, const BArgs& p) {
  const bool two = p.hi2 > p.lo2;
  if (p.hi <= p.lo) {
    if (!two) return hipSuccess;
    BArgs q = p;  // only the second range: it becomes the first
    q.lo = p.lo2, q.hi = p.hi2, q.lo2 = q.hi2 = 0;
    return run_b(dtype, three_d, scheme, ls, q);
  }
  const int R = scheme_radius(scheme);
  if (scheme < 0 || scheme > 2 || p.lo < R || p.nx <= 0 || (three_d && p.ny <= 0) ||
      p.border < R || p.in == p.out || (ls && (p.in == p.aux || p.out == p.aux)) ||
      (two && p.lo2 < R))
    return hipErrorInvalidValue;
  // two plane ranges in one launch: the 3-D WENO5 v9 kernel; everything else launches
  // the ranges one after the other
  if (two && !(three_d && scheme != 2 && b3_ver() == 9 &&
               (dtype == ADVDIFF_F64 ? v9_fits<double>(p) : v9_fits<float>(p)))) {
    BArgs p1 = p, p2 = p;
    p1.lo2 = p1.hi2 = 0;
    p2.lo = p.lo2, p2.hi = p.hi2, p2.lo2 = p2.hi2 = 0;
    const hipError_t e = run_b(dtype, three_d, scheme, ls, p1);
    return e != hipSuccess ? e : run_b(dtype, three_d, scheme, ls, p2);
  }
  const bool visc = p.vx != 0.0 || p.vy != 0.0 || (three_d && p.vz != 0.0);
  const int mode = ls ? (p.a != 0.0 ? kLs : kLs1) : (p.a != 0.0 ? kSsp : kSsp1);
  if (dtype == ADVDIFF_F64)
    return three_d ? dispatch_b<double, true>(scheme, visc, mode, p)
                   : dispatch_b<double, false>(scheme, visc, mode, p);
  if (dtype == ADVDIFF_F32)
    return three_d ? dispatch_b<float, true>(scheme, visc, mode, p)
                   : dispatch_b<float, false>(scheme, visc, mode, p);
  return hipErrorInvalidValue;
}

}  // namespace advdiff

extern "C" int advdiff_set_b2_ver(int v) {
  const int old = advdiff::b2_ver();
  advdiff::g_b2_ver = v;
  return old;
}

extern "C" int advdiff_set_b3_pack(int on) {
  const int old = advdiff::b3_pack();
  advdiff::g_b3_pack = on ? 1 : 0;
  return old;
}

extern "C" int advdiff_set_b3_tx(int v) {
  const int old = advdiff::b3_tx();
  advdiff::g_b3_tx = v;
  return old;
}

extern "C" int advdiff_set_b3_zchunk(int zc) {
  const int old = advdiff::g_b3_zchunk;
  advdiff::g_b3_zchunk = zc > 0 ? zc : 0;
  return old;
}

extern "C" int advdiff_set_b3_ver(int v) {
  const int old = advdiff::b3_ver();
  advdiff::g_b3_ver = v;
  return old;
}

// dt_dev: device scalar with the step's dt (adaptive CFL, computed on the device by
// advdiff_adaptive_dt) or nullptr (use dt).  A device dt of exactly 0 marks a step past
// t_end: the stage becomes out = in on the active cells (aux untouched), so surplus steps
// issued ahead of the host's next look at t are exact no-ops.
extern "C" int advdiff_burgers3d_stage_dt(int dtype, const void* in, void* aux, void* out,
                                          int nx, int ny, int64_t sy, int64_t sz, int k0,
                                          int k1, int border, int weno, double rdx, double rdy,
                                          double rdz, double vx, double vy, double vz,
                                          double dt, double a, double b, int ls,
                                          const double* dt_dev, void* stream) {
  using namespace advdiff;
  const BArgs p{in, aux, out, nx, ny, sy, sz, k0, k1, border, rdx, rdy, rdz,
                vx, vy, vz, dt, a, b, (hipStream_t)stream, dt_dev};
  return run_b(dtype, true, weno, ls != 0, p);
}

// The same stage on two marched-axis ranges [k0, k1) and [k0b, k1b) (a slab rank's two
// boundary slabs after the halo wait): one launch with the default 3-D WENO5 kernel (v9),
// two launches otherwise.  Either range may be empty.
extern "C" int advdiff_burgers3d_stage2_dt(int dtype, const void* in, void* aux, void* out,
                                           int nx, int ny, int64_t sy, int64_t sz, int k0,
                                           int k1, int k0b, int k1b, int border, int weno,
                                           double rdx, double rdy, double rdz, double vx,
                                           double vy, double vz, double dt, double a, double b,
                                           int ls, const double* dt_dev, void* stream) {
  using namespace advdiff;
  BArgs p{in, aux, out, nx, ny, sy, sz, k0, k1, border, rdx, rdy, rdz,
          vx, vy, vz, dt, a, b, (hipStream_t)stream, dt_dev};
  p.lo2 = k0b;
  p.hi2 = k1b;
  return run_b(dtype, true, weno, ls != 0, p);
}

// One full-range stage of a slab rank whose output planes [lo_k0, lo_k1) / [hi_k0, hi_k1)
// are also stored, system scope, into the peer planes at dst_lo / dst_hi (IPC mappings of
// the neighbours' output fields: the peer plane of local plane lo_k0 / hi_k0; same row pitch
// and plane stride; null / empty: no peer that side).  fp64, WENO5-JS / -Z (weno 0 / 1),
// SSP-RK3 epilogues (a == 0: first stage), the v9 kernel (planes below 2 GiB).
extern "C" int advdiff_burgers3d_stage_put(int dtype, const void* in, void* aux, void* out,
                                           int nx, int ny, int64_t sy, int64_t sz, int k0,
                                           int k1, int border, int weno, double rdx, double rdy,
                                           double rdz, double vx, double vy, double vz,
                                           double dt, double a, double b, const double* dt_dev,
                                           void* dst_lo, int lo_k0, int lo_k1, void* dst_hi,
                                           int hi_k0, int hi_k1, void* stream) {
  using namespace advdiff;
  const BArgs p{in, aux, out, nx, ny, sy, sz, k0, k1, border, rdx, rdy, rdz,
                vx, vy, vz, dt, a, b, (hipStream_t)stream, dt_dev};
  if (k1 <= k0) return hipSuccess;
  if (dtype != ADVDIFF_F64 || (weno != 0 && weno != 1) || k0 < 3 || border < 3 || nx <= 0 ||
      ny <= 0 || in == out || b3_ver() != 9 || !v9_fits<double>(p))
    return hipErrorInvalidValue;
  HaloPut2 put{};
  void* dsts[2] = {dst_lo, dst_hi};
  const int pk0[2] = {lo_k0, hi_k0}, pk1[2] = {lo_k1, hi_k1};
  for (int s = 0; s < 2; ++s) {
    const bool on = dsts[s] != nullptr && pk1[s] > pk0[s];
    put.dst[s] = on ? (char*)dsts[s] : nullptr;
    put.k0[s] = on ? pk0[s] : 0;
    put.k1[s] = on ? pk1[s] : 0;
  }
  const bool visc = vx != 0.0 || vy != 0.0 || vz != 0.0;
  const int mode = a != 0.0 ? kSsp : kSsp1;
#define BP(WZ, V) \
  return mode == kSsp ? launch_b3_put<WZ, V, kSsp>(p, put) : launch_b3_put<WZ, V, kSsp1>(p, put)
  if (weno == 1) {
    if (visc) BP(true, true);
    BP(true, false);
  }
  if (visc) BP(false, true);
  BP(false, false);
#undef BP
}

extern "C" int advdiff_burgers2d_stage_dt(int dtype, const void* in, void* aux, void* out,
                                          int nx, int64_t sy, int j0, int j1, int border,
                                          int weno, double rdx, double rdy, double vx,
                                          double vy, double dt, double a, double b, int ls,
                                          const double* dt_dev, void* stream) {
  using namespace advdiff;
  const BArgs p{in, aux, out, nx, 0, sy, 0, j0, j1, border, rdx, rdy, 0.0,
                vx, vy, 0.0, dt, a, b, (hipStream_t)stream, dt_dev};
  return run_b(dtype, false, weno, ls != 0, p);
}

extern "C" int advdiff_burgers3d_stage(int dtype, const void* in, const void* u0, void* out,
                                       int nx, int ny, int64_t sy, int64_t sz, int k0, int k1,
                                       int border, int weno, double rdx, double rdy,
                                       double rdz, double vx, double vy, double vz, double dt,
                                       double a, double b, void* stream) {
  return advdiff_burgers3d_stage_dt(dtype, in, const_cast<void*>(u0), out, nx, ny, sy, sz, k0,
                                    k1, border, weno, rdx, rdy, rdz, vx, vy, vz, dt, a, b, 0,
                                    nullptr, stream);
}

extern "C" int advdiff_burgers3d_stage_ls(int dtype, const void* in, void* du, void* out,
                                          int nx, int ny, int64_t sy, int64_t sz, int k0,
                                          int k1, int border, int weno, double rdx, double rdy,
                                          double rdz, double vx, double vy, double vz,
                                          double dt, double A, double B, void* stream) {
  return advdiff_burgers3d_stage_dt(dtype, in, du, out, nx, ny, sy, sz, k0, k1, border, weno,
                                    rdx, rdy, rdz, vx, vy, vz, dt, A, B, 1, nullptr, stream);
}

extern "C" int advdiff_burgers2d_stage(int dtype, const void* in, const void* u0, void* out,
                                       int nx, int64_t sy, int j0, int j1, int border,
                                       int weno, double rdx, double rdy, double vx, double vy,
                                       double dt, double a, double b, void* stream) {
  return advdiff_burgers2d_stage_dt(dtype, in, const_cast<void*>(u0), out, nx, sy, j0, j1,
                                    border, weno, rdx, rdy, vx, vy, dt, a, b, 0, nullptr,
                                    stream);
}

extern "C" int advdiff_burgers2d_stage_ls(int dtype, const void* in, void* du, void* out,
                                          int nx, int64_t sy, int j0, int j1, int border,
                                          int weno, double rdx, double rdy, double vx,
                                          double vy, double dt, double A, double B,
                                          void* stream) {
  return advdiff_burgers2d_stage_dt(dtype, in, du, out, nx, sy, j0, j1, border, weno, rdx, rdy,
                                    vx, vy, dt, A, B, 1, nullptr, stream);
}

namespace advdiff {
template <typename T, bool PK>
static void preload_w5s_occupancies() {
  [&]<int... I>(std::integer_sequence<int, I...>) {
    // I = WZ | VISC << 1 | MODE << 2 | (TXL == 32) << 4
    ((void)occupancy_per_cu(
         (const void*)burgers3d_w5s_kernel<T, (I & 1) != 0, (I & 2) != 0, (I >> 2) & 3,
                                           (I & 16) ? 32 : 64, PK>,
         512),
     ...);
  }(std::make_integer_sequence<int, 32>{});
}
// the fused-put instances: fp64, SSP-RK3 epilogues (MODE 0 / 1), I as above
static void preload_w5s_put_occupancies() {
  [&]<int... I>(std::integer_sequence<int, I...>) {
    ((void)occupancy_per_cu(
         (const void*)burgers3d_w5s_kernel<double, (I & 1) != 0, (I & 2) != 0, (I >> 2) & 1,
                                           (I & 8) ? 32 : 64, false, true>,
         512),
     ...);
  }(std::make_integer_sequence<int, 16>{});
}
}  // namespace advdiff

// Code-object preload (see advdiff_preload in aux.hip): the attributes query makes the
// runtime load this translation unit's code object now instead of at the first launch.
extern "C" int advdiff_preload_burgers(void) {
  using namespace advdiff;
  hipFuncAttributes a;
  const hipError_t e =
      hipFuncGetAttributes(&a, (const void*)burgers3d_w5s_kernel<double, true, true, 1>);
  // occupancies of every 3-D stage instance the default dispatch can select (launch.hpp
  // occupancy_per_cu caches them), so no first launch — possibly inside a hipGraph capture
  // — queries the runtime: fp64 and fp32 (one cell or packed pairs per lane), WENO5-JS
  // and -Z, inviscid and viscous, every stage epilogue, both tile rows
  preload_w5s_occupancies<double, false>();
  preload_w5s_occupancies<float, false>();
  preload_w5s_occupancies<float, true>();
  preload_w5s_put_occupancies();
  return e;
}
