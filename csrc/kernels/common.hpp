// Shared device-side building blocks for the gfx950 stencil kernels.
//
// Numerics follow the reference's specification:
//   * FD4 second derivative  (-u[-2] + 16u[-1] - 30u[0] + 16u[+1] - u[+2]) / 12dx²
//     (reference: MultiGPU/Diffusion3d_Baseline/Kernels.cu:207-261,
//      SingleGPU/Diffusion3d_baselineCode/kernels.cu:66-99)
//   * FD2 second derivative  (u[-1] - 2u[0] + u[+1]) / dx²
//     (reference: SingleGPU/Diffusion3d_baselineCode/kernels.cu:37-64)
//   * WENO5-JS / WENO5-Z reconstruction with local Lax-Friedrichs flux splitting
//     (reference: MultiGPU/Burgers3d_Baseline/Kernels.cu:112-220,
//      SingleGPU/Burgers3d_WENO5/kernels.cu:92-192)
//
// Design notes (MI355X-first, not a translation):
//   * The nonlinear weights are evaluated with ONE division per reconstruction side:
//     w_k = alpha_k / sum(alpha) is rewritten over a common denominator
//     (alpha_k ∝ d_k * prod_{j!=k} s_j), removing 3 of the 4 fp64 divisions of the
//     textbook form. fp64 divisions are ~10 VALU instructions on CDNA4, so this is
//     the single largest instruction-count lever for the ALU-bound WENO kernels.
//   * Everything is templated on the scalar type (float/double) so the reference's
//     USE_FLOAT compile switch becomes a runtime dtype choice.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace advdiff {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// Packed fp32 pair: two cells per lane in one 64-bit register pair, so the templated
// helpers below (explicit fma, contraction off) compile to v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32 — CDNA4's 2x fp32 VALU rate (the fp64 and scalar-fp32 rates are equal).
// Each element goes through exactly the scalar operation sequence, so a packed kernel's
// results are the scalar-fp32 kernel's, cell by cell.  The using-declarations keep the
// float / double overloads visible next to the pair ones.
typedef float f32x2 __attribute__((ext_vector_type(2)));
using ::fabs;
using ::fma;
__device__ __forceinline__ f32x2 fma(f32x2 a, f32x2 b, f32x2 c) {
  return __builtin_elementwise_fma(a, b, c);
}
__device__ __forceinline__ f32x2 fabs(f32x2 a) { return __builtin_elementwise_abs(a); }
template <typename T>
inline constexpr bool is_pair_v = false;
template <>
inline constexpr bool is_pair_v<f32x2> = true;

template <typename T>
__device__ __forceinline__ T clampi(T v, T lo, T hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

// XCD-aware workgroup placement (cdna_hip_programming.md §5.5 T1): the dispatcher deals
// workgroups round-robin over the 8 XCDs (blocks b, b+8, ... share one L2), so
// consecutive logical tiles — which overlap in their halos — would land on 8 different
// L2s.  This bijective remap gives each XCD a CONTIGUOUS range of logical tiles (x
// fastest, then y, then z), so the tiles running together on one XCD are neighbours and
// their halo re-reads hit that XCD's L2.  Placement only affects speed, never results.
struct Tile3 {
  int x, y, z;
};
__device__ __forceinline__ Tile3 xcd_tile() {
  const int nbx = gridDim.x, nby = gridDim.y;
  const int total = nbx * nby * (int)gridDim.z;
  const int b = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
  const int q = total >> 3, r = total & 7;
  const int xcd = b & 7, slot = b >> 3;
  const int t = xcd * q + min(xcd, r) + slot;
  Tile3 o;
  o.x = t % nbx;
  const int yz = t / nbx;
  o.y = yz % nby;
  o.z = yz / nby;
  return o;
}

// The same placement for a 1-D grid of `bands` x C tiles dispatched band by band (the
// banded z schedule of the fused heat step): block b is band b / C; within its band every
// XCD gets a CONTIGUOUS run of the band's C logical tiles (x fastest), so each XCD holds
// its share of every band and neighbouring tiles share its L2.
__device__ __forceinline__ Tile3 xcd_tile_banded(int C, int gx) {
  const int b = blockIdx.x;
  const int band = b / C;
  const int off = band * C;
  const int x = b & 7;
  int start = 0;
  for (int xp = 0; xp < x; ++xp) {  // tiles of this band on the XCDs before x
    const int r = (xp - off) & 7;     // first k in [0, C) with (off + k) % 8 == xp
    start += r < C ? (C - r + 7) >> 3 : 0;
  }
  const int r = (x - off) & 7;
  Tile3 o;
  const int t = start + ((b - off - r) >> 3);
  o.x = t % gx;
  o.y = t / gx;
  o.z = band;
  return o;
}

// Second-derivative stencils. `d2` returns the UNSCALED combination; the caller folds
// 1/(12 dx²) (FD4) or 1/dx² (FD2) into a per-axis coefficient.  Written with explicit
// fma() and contraction off, so every kernel that evaluates a Laplacian (per-stage,
// fused-step, Burgers viscous term) produces bit-identical values.
template <int ORDER>
struct FD;

template <>
struct FD<4> {
  static constexpr int R = 2;
  template <typename T>
  __device__ __forceinline__ static T d2(T m2, T m1, T c, T p1, T p2) {
#pragma clang fp contract(off)
    return fma(T(-30), c, fma(T(16), m1 + p1, -(m2 + p2)));
  }
};

template <>
struct FD<2> {
  static constexpr int R = 1;
  template <typename T>
  __device__ __forceinline__ static T d2(T m1, T c, T p1) {
#pragma clang fp contract(off)
    return fma(T(-2), c, m1 + p1);
  }
};

// cx*d2x + cy*d2y + cz*d2z with a fixed evaluation order.
template <typename T>
__device__ __forceinline__ T lap3(T cx, T dxx, T cy, T dyy, T cz, T dzz) {
#pragma clang fp contract(off)
  return fma(cz, dzz, fma(cy, dyy, cx * dxx));
}
template <typename T>
__device__ __forceinline__ T lap2(T cx, T dxx, T cy, T dyy) {
#pragma clang fp contract(off)
  return fma(cy, dyy, cx * dxx);
}

// SSP-RK3 stage value  a*u0 + b*(c + dt*L)  (a = 0: no u0 term), fixed evaluation order.
template <typename T, bool USE_U0>
__device__ __forceinline__ T rk_stage(T uo, T c, T L, T dt, T a, T b) {
#pragma clang fp contract(off)
  T v = b * fma(dt, L, c);
  if constexpr (USE_U0) v = fma(a, uo, v);
  return v;
}

// ---------------------------------------------------------------------------------
// Folded heat-equation stage update (every diffusion kernel: per-stage, fused step,
// 2-D and 3-D).  An SSP stage  out = a u0 + b (c + dt Σ_d k_d d2_d(c))  with the FD4
// d2 = 16 (m1+p1) - (m2+p2) - 30 c is evaluated as
//     out = a u0 + KC c + Σ_d K_d [16 (m1+p1)_d - (m2+p2)_d]
//     K_d = b dt k_d,  KC = b (1 - 30 dt Σ_d k_d)
// (FD2: d2 = (m1+p1) - 2c, KC = b (1 - 2 dt Σ k_d)): per point 13-14 fp64 VALU ops
// (FD4) instead of 16-18 for d2 -> Laplacian -> RK combination, with 4 coefficients per
// stage (16 is an inline constant).  A low-storage stage uses the same chain with b = 1
// and no c term (it yields d = a du + dt L).  The coefficients come from one host helper
// (fd_coef) and the chain has a fixed evaluation order (centre, z, x, y; 2-D: centre,
// y, x), so the per-stage and fused kernels stay bit-identical.
// ---------------------------------------------------------------------------------
template <typename T>
struct FdCoef {
  T kc;    // centre
  T k[3];  // per axis (x, y, z)
};

// s: the stage's b (SSP) or 1 (low-storage); with_c: the "+ s c" term (SSP only).
// kx, ky, kz: K/dx², K/dy², K/dz² (unscaled; kz = 0 in 2-D).
template <typename T>
inline FdCoef<T> fd_coef(int order, double kx, double ky, double kz, double dt, double s,
                         bool with_c) {
  const double f = order == 4 ? 1.0 / 12.0 : 1.0, ctr = order == 4 ? 30.0 : 2.0;
  const double k[3] = {kx * f, ky * f, kz * f};
  FdCoef<T> c;
  c.kc = T(s * ((with_c ? 1.0 : 0.0) - ctr * dt * ((k[0] + k[1]) + k[2])));
  for (int d = 0; d < 3; ++d) c.k[d] = T(s * dt * k[d]);
  return c;
}

// centre term: base + KC c (base = a u0 / a du) or KC c
template <typename T>
__device__ __forceinline__ T fd_ctr(T kc, T c) {
  return kc * c;
}
template <typename T>
__device__ __forceinline__ T fd_ctr(T kc, T c, T base) {
#pragma clang fp contract(off)
  return fma(kc, c, base);
}
// one FD4 axis: acc + K (16 (m1+p1) - (m2+p2))
template <typename T>
__device__ __forceinline__ T fd4_axis(T acc, T k, T m2, T m1, T p1, T p2) {
#pragma clang fp contract(off)
  return fma(k, fma(T(16), m1 + p1, -(m2 + p2)), acc);
}
// the same split in two: the axis sum S = 16 (m1+p1) - (m2+p2) (FD4) / m1+p1 (FD2), then
// acc + K S — fd4_axis(acc, k, ...) == fd_apply(acc, k, fd4_sum(...)) bit for bit
template <typename T>
__device__ __forceinline__ T fd4_sum(T m2, T m1, T p1, T p2) {
#pragma clang fp contract(off)
  return fma(T(16), m1 + p1, -(m2 + p2));
}
template <typename T>
__device__ __forceinline__ T fd2_sum(T m1, T p1) {
#pragma clang fp contract(off)
  return m1 + p1;
}
template <typename T>
__device__ __forceinline__ T fd_apply(T acc, T k, T s) {
#pragma clang fp contract(off)
  return fma(k, s, acc);
}
// one FD2 axis: acc + K (m1+p1)
template <typename T>
__device__ __forceinline__ T fd2_axis(T acc, T k, T m1, T p1) {
#pragma clang fp contract(off)
  return fma(k, m1 + p1, acc);
}

// Burgers flux f(u) = u²/2, local Lax-Friedrichs split  f± = ½(f(u) ± |u|·u).
// (reference: MultiGPU/Burgers3d_Baseline/Kernels.cu:256-264)
//
// Determinism: the split and the WENO reconstruction are written with explicit fma()
// and FP contraction disabled inside, so a face flux is bit-identical wherever it is
// evaluated (the z-face of a chunk's prologue vs. the same face inside the march).
// That makes a P-rank run bitwise equal to the 1-rank run whatever the chunking.
template <typename T>
__device__ __forceinline__ void lf_split(T u, T& fp, T& fm) {
#pragma clang fp contract(off)
  // h = u/2: h·h = u²/4 exactly as (u/4)·u, |h|·u = (|u|/2)·u — 4 ops instead of 5
  const T h = T(0.5) * u;
  const T s = fabs(h) * u;
  fp = fma(h, h, s);
  fm = fma(h, h, -s);
}

// Division without the IEEE div_scale/div_fmas/div_fixup sequence: hardware reciprocal
// + two Newton steps + one residual correction (fp64: 7 VALU ops instead of ~10; error
// <= 1 ulp).  Written with explicit fma, so it is bit-reproducible in every context.
template <typename T>
__device__ __forceinline__ T fast_div(T n, T d) {
#pragma clang fp contract(off)
  if constexpr (sizeof(T) == 8) {
    T r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, T(1)), r, r);
    r = fma(fma(-d, r, T(1)), r, r);
    const T q = n * r;
    return fma(fma(-d, q, n), r, q);
  } else {
    return n / d;
  }
}

// Left-biased WENO5 reconstruction of the value at the right face of v2 from the
// five point values v0..v4 (= f at i-2..i+2), returned as numerator/denominator
// (value = num / den) so a face can combine its two sides with ONE division.
// The right-biased (f⁻) reconstruction at face i+½ is this function applied to the
// mirrored stencil f⁻(i+3..i-1).
// ZVARIANT=false: Jiang–Shu weights  alpha_k = d_k / (eps + beta_k)²
// ZVARIANT=true : Borges WENO-Z      alpha_k = d_k (1 + tau5 / (beta_k + eps)),
//                 tau5 = |beta_0 - beta_2|
// alpha_k is rewritten over a common denominator (alpha_k ∝ d_k · prod_{j≠k} s_j), so
// w_k = alpha_k / Σalpha needs no division of its own.
// Curvature part of a WENO5 smoothness indicator, 13/12 (a - 2b + c)²: the same for
// every sub-stencil centred on b, so a z-marching lane reuses two of three per side.
template <typename T>
__device__ __forceinline__ T weno5_curv(T a, T b, T c) {
#pragma clang fp contract(off)
  const T t = fma(T(-2), b, a + c);
  return (T(13.0 / 12.0) * t) * t;
}

// weno5_nd with the curvature terms K0 = curv(v0,v1,v2), K1 = curv(v1,v2,v3),
// K2 = curv(v2,v3,v4) supplied by the caller.
template <typename T, bool ZVARIANT>
__device__ __forceinline__ void weno5_nd_k(T v0, T v1, T v2, T v3, T v4, T K0, T K1, T K2,
                                           T& num, T& den) {
#pragma clang fp contract(off)
  constexpr T eps = T(1e-6);
  const T t0b = fma(T(3), v2, fma(T(-4), v1, v0));
  const T t1b = v1 - v3;
  const T t2b = fma(T(3), v2, fma(T(-4), v3, v4));
  const T b0 = fma(T(0.25) * t0b, t0b, K0);
  const T b1 = fma(T(0.25) * t1b, t1b, K1);
  const T b2 = fma(T(0.25) * t2b, t2b, K2);
  // candidate polynomials (times 6)
  const T q0 = fma(T(11), v2, fma(T(-7), v1, T(2) * v0));
  const T q1 = fma(T(5), v2, fma(T(2), v3, -v1));
  const T q2 = fma(T(5), v3, fma(T(2), v2, -v4));
  T w0, w1, w2;
  if constexpr (ZVARIANT) {
    const T tau = fabs(b0 - b2);
    const T e0 = b0 + eps, e1 = b1 + eps, e2 = b2 + eps;
    // alpha_k ∝ d_k (e_k + tau) * e_j * e_l
    w0 = (T(0.1) * (e0 + tau)) * (e1 * e2);
    w1 = (T(0.6) * (e1 + tau)) * (e0 * e2);
    w2 = (T(0.3) * (e2 + tau)) * (e0 * e1);
  } else {
    const T e0 = eps + b0, e1 = eps + b1, e2 = eps + b2;
    const T s0 = e0 * e0, s1 = e1 * e1, s2 = e2 * e2;
    // alpha_k ∝ d_k * s_j * s_l
    w0 = T(0.1) * (s1 * s2);
    w1 = T(0.6) * (s0 * s2);
    w2 = T(0.3) * (s0 * s1);
  }
  num = fma(w0, q0, fma(w1, q1, w2 * q2));
  den = T(6) * ((w0 + w1) + w2);
}

template <typename T, bool ZVARIANT>
__device__ __forceinline__ void weno5_nd(T v0, T v1, T v2, T v3, T v4, T& num, T& den) {
  weno5_nd_k<T, ZVARIANT>(v0, v1, v2, v3, v4, weno5_curv(v0, v1, v2), weno5_curv(v1, v2, v3),
                          weno5_curv(v2, v3, v4), num, den);
}

template <typename T, bool ZVARIANT>
__device__ __forceinline__ T weno5(T v0, T v1, T v2, T v3, T v4) {
  T n, d;
  weno5_nd<T, ZVARIANT>(v0, v1, v2, v3, v4, n, d);
  return fast_div(n, d);
}

// Numerical flux at face i+½ from split fluxes fp(i-2..i+2), fm(i-1..i+3).
// fp64: both sides over one denominator, n1/d1 + n2/d2 = (n1 d2 + n2 d1)/(d1 d2) —
// one division per face (d1·d2 >= ~1e-50 with eps = 1e-6: safe in fp64, not in fp32,
// which keeps two divisions).
template <typename T, bool ZVARIANT>
__device__ __forceinline__ T weno5_face(T p0, T p1, T p2, T p3, T p4,   // fp i-2..i+2
                                        T m0, T m1, T m2, T m3, T m4) {  // fm i-1..i+3
#pragma clang fp contract(off)
  T n1, d1, n2, d2;
  weno5_nd<T, ZVARIANT>(p0, p1, p2, p3, p4, n1, d1);
  weno5_nd<T, ZVARIANT>(m4, m3, m2, m1, m0, n2, d2);
  if constexpr (sizeof(T) == 8) {
    return fast_div(fma(n1, d2, n2 * d1), d1 * d2);
  } else {
    return fast_div(n1, d1) + fast_div(n2, d2);
  }
}

// weno5_face with precomputed curvatures: kp = curv of f+ centred on p1, p2, p3 and
// km = curv of f- centred on m1, m2, m3 (bit-identical to weno5_face).
template <typename T, bool ZVARIANT>
__device__ __forceinline__ T weno5_face_k(const T* p, const T* m, const T* kp, const T* km) {
#pragma clang fp contract(off)
  T n1, d1, n2, d2;
  weno5_nd_k<T, ZVARIANT>(p[0], p[1], p[2], p[3], p[4], kp[0], kp[1], kp[2], n1, d1);
  weno5_nd_k<T, ZVARIANT>(m[4], m[3], m[2], m[1], m[0], km[2], km[1], km[0], n2, d2);
  if constexpr (sizeof(T) == 8) {
    return fast_div(fma(n1, d2, n2 * d1), d1 * d2);
  } else {
    return fast_div(n1, d1) + fast_div(n2, d2);
  }
}

// ---------------------------------------------------------------------------------
// Non-inline fp64 constants of the WENO5 / FD4 helpers.  gfx9 VOP3 (v_fma_f64) cannot
// encode a literal, so fma(3.0, x, y) becomes the 2-address v_fmac_f64_e32 with the
// literal — plus a v_mov_b64 whenever the accumulator is still live.  W5Lit (default)
// keeps the literals; W5Sgpr holds the same values in SGPRs (laundered once per kernel),
// which VOP3 takes as an operand, so no copy is needed.  The values are identical, so
// both give bit-identical results.
// ---------------------------------------------------------------------------------
template <typename T>
struct W5Lit {
  static constexpr T k3 = T(3), k5 = T(5), k6 = T(6), k1_5 = T(1.5), k13_3 = T(13.0 / 3.0),
                     k4em6 = T(4e-6), k16 = T(16), km30 = T(-30);
};
template <typename T>
__device__ __forceinline__ T sgpr_const(T v) {
  asm volatile("" : "+s"(v));
  return v;
}
template <typename T>
struct W5Sgpr {
  T k3, k5, k6, k1_5, k13_3, k4em6, k16, km30;
  __device__ __forceinline__ W5Sgpr()
      : k3(sgpr_const(T(3))), k5(sgpr_const(T(5))), k6(sgpr_const(T(6))),
        k1_5(sgpr_const(T(1.5))), k13_3(sgpr_const(T(13.0 / 3.0))),
        k4em6(sgpr_const(T(4e-6))), k16(sgpr_const(T(16))), km30(sgpr_const(T(-30))) {}
};

// FD<4>::d2 with the constants from K (bit-identical)
template <typename T, class K>
__device__ __forceinline__ T fd4_d2k(T m2, T m1, T c, T p1, T p2, const K& kk) {
#pragma clang fp contract(off)
  return fma(kk.km30, c, fma(kk.k16, m1 + p1, -(m2 + p2)));
}

// ---------------------------------------------------------------------------------
// WENO5 with SCALED smoothness indicators (the 3-D stage kernel's reconstruction).
// Every indicator is carried as e_k = 4 (beta_k + eps) = t_k² + C_k, where t_k is the
// first-derivative term (v0 - 4v1 + 3v2 etc.) and C_k = 13/3 c_k² + 4 eps folds the
// curvature term and eps into one value per stencil centre (w5_curv: a z-marching lane
// reuses two of three per side).  The common factor 4 leaves both weight families
// unchanged (JS: alpha ∝ 1/e², a common 1/16; Z: tau/(beta+eps) is a ratio), and the
// linear weights (0.1, 0.6, 0.3) become (1, 6, 3) — the 1/10 cancels in num/den.  Per
// side this is 32 fp64 ops (Z) instead of 40, with the same results to rounding
// (tests/test_kernels_gpu.py compares against the textbook fp64 form).
// ---------------------------------------------------------------------------------
template <typename T, class K = W5Lit<T>>
__device__ __forceinline__ T w5_curv(T a, T b, T c, const K& kk = K{}) {
#pragma clang fp contract(off)
  const T t = fma(T(-2), b, a + c);
  return fma(kk.k13_3 * t, t, kk.k4em6);
}

// One side: numerator num = Σ w_k q_k (q_k = 6 x candidate) and S = Σ w_k, so the side's
// value is num / (6 S).  C0..C2 = w5_curv centred on v1, v2, v3.
template <typename T, bool ZVARIANT, class K = W5Lit<T>>
__device__ __forceinline__ void w5_side(T v0, T v1, T v2, T v3, T v4, T C0, T C1, T C2,
                                        T& num, T& S, const K& kk = K{}) {
#pragma clang fp contract(off)
  const T t0 = fma(kk.k3, v2, fma(T(-4), v1, v0));
  const T t1 = v1 - v3;
  const T t2 = fma(kk.k3, v2, fma(T(-4), v3, v4));
  const T e0 = fma(t0, t0, C0), e1 = fma(t1, t1, C1), e2 = fma(t2, t2, C2);
  // 2 v0 - 7 v1 + 11 v2 = 2 t0 + v1 + 5 v2: one op fewer than the direct form
  const T q0 = fma(T(2), t0, fma(kk.k5, v2, v1));
  const T q1 = fma(kk.k5, v2, fma(T(2), v3, -v1));
  const T q2 = fma(kk.k5, v3, fma(T(2), v2, -v4));
  T w0, w1, w2;
  if constexpr (ZVARIANT) {
    // (e_k + tau) * prod_{j!=k} e_j = P + tau * prod_{j!=k} e_j with P = e0 e1 e2:
    // 4 products + 3 fma instead of 3 products, 3 adds and 3 more products
    const T tau = fabs(e0 - e2);
    const T e12 = e1 * e2, e02 = e0 * e2, e01 = e0 * e1, P = e0 * e12;
    w0 = fma(tau, e12, P);
    w1 = kk.k6 * fma(tau, e02, P);
    w2 = kk.k3 * fma(tau, e01, P);
  } else {
    const T s0 = e0 * e0, s1 = e1 * e1, s2 = e2 * e2;
    w0 = s1 * s2;
    w1 = kk.k6 * (s0 * s2);
    w2 = kk.k3 * (s0 * s1);
  }
  num = fma(w0, q0, fma(w1, q1, w2 * q2));
  S = (w0 + w1) + w2;
}

// Face flux from both sides: n1/(6 S1) + n2/(6 S2) = (n1 S2 + n2 S1) / (6 S1 S2) with one
// division (fp64; S1 S2 >= ~1e-43 at eps = 1e-6 for the JS form); fp32 keeps two.
template <typename T>
__device__ __forceinline__ T w5_combine(T n1, T S1, T n2, T S2) {
#pragma clang fp contract(off)
  if constexpr (sizeof(T) == 8) {
    return fast_div(fma(n1, S2, n2 * S1), (T(6) * S1) * S2);
  } else {
    return fast_div(n1, T(6) * S1) + fast_div(n2, T(6) * S2);
  }
}

// Face i+½ from p = f⁺(i-2..i+2), m = f⁻(i-1..i+3), all curvatures computed here.
template <typename T, bool ZVARIANT>
__device__ __forceinline__ T w5_face(const T* p, const T* m) {
  T n1, S1, n2, S2;
  w5_side<T, ZVARIANT>(p[0], p[1], p[2], p[3], p[4], w5_curv(p[0], p[1], p[2]),
                       w5_curv(p[1], p[2], p[3]), w5_curv(p[2], p[3], p[4]), n1, S1);
  w5_side<T, ZVARIANT>(m[4], m[3], m[2], m[1], m[0], w5_curv(m[4], m[3], m[2]),
                       w5_curv(m[3], m[2], m[1]), w5_curv(m[2], m[1], m[0]), n2, S2);
  return w5_combine(n1, S1, n2, S2);
}

// The same face with the curvatures supplied: kp = C of f⁺ centred on p1, p2, p3 and
// km = C of f⁻ centred on m1, m2, m3 (bit-identical to w5_face).
template <typename T, bool ZVARIANT>
__device__ __forceinline__ T w5_face_k(const T* p, const T* m, const T* kp, const T* km) {
  T n1, S1, n2, S2;
  w5_side<T, ZVARIANT>(p[0], p[1], p[2], p[3], p[4], kp[0], kp[1], kp[2], n1, S1);
  w5_side<T, ZVARIANT>(m[4], m[3], m[2], m[1], m[0], km[2], km[1], km[0], n2, S2);
  return w5_combine(n1, S1, n2, S2);
}

// ---------------------------------------------------------------------------------
// One side of an x/y face of the v9 3-D stage, curvatures included, around the
// differences a = v2 - v1, b = v2 - v3 and the raw curvatures c_k (centred on v1, v2,
// v3):   t0 = c0 + 2a,  t2 = c2 + 2b,  t1 = b - a,  c1 = -(a + b);
//        Σ w_k q_k = S q1 + w0 (q0 - q1) + w2 (q2 - q1)   with
//        q0 - q1 = 2 (c0 - c1),  q2 - q1 = c1 - c2,  q1 / 2 = 3 v2 - b + a / 2,
// and (w0, w1, w2) = (g0, 6 g1, 3 g2) folded into S = g0 + 6 g1 + 3 g2.  The numerator
// is returned HALVED (numh = Σ w_k q_k / 2), so w5_combine6 of two such sides is 3 x
// the face flux.  37 fp64 ops per side (w5_side + its three w5_curv: 41).
// ---------------------------------------------------------------------------------
template <typename T, bool ZVARIANT, class K = W5Lit<T>>
__device__ __forceinline__ void w5_side_h(T v0, T v1, T v2, T v3, T v4, T& numh, T& S,
                                          const K& kk = K{}) {
#pragma clang fp contract(off)
  const T a = v2 - v1, b = v2 - v3;
  const T c0 = fma(T(-2), v1, v0 + v2);
  const T c2 = fma(T(-2), v3, v2 + v4);
  const T c1n = a + b;  // = -c1
  const T t0 = fma(T(2), a, c0), t1 = b - a, t2 = fma(T(2), b, c2);
  const T e0 = fma(t0, t0, fma(kk.k13_3 * c0, c0, kk.k4em6));
  const T e1 = fma(t1, t1, fma(kk.k13_3 * c1n, c1n, kk.k4em6));
  const T e2 = fma(t2, t2, fma(kk.k13_3 * c2, c2, kk.k4em6));
  const T q1h = fma(T(0.5), a, fma(kk.k3, v2, -b));
  const T d01 = c0 + c1n;     // c0 - c1
  const T d21n = c1n + c2;    // -(c1 - c2)
  T g0, g1, g2;
  if constexpr (ZVARIANT) {
    const T tau = fabs(e0 - e2);
    const T e12 = e1 * e2, P = e0 * e12;
    g0 = fma(tau, e12, P);
    g1 = fma(tau, e0 * e2, P);
    g2 = fma(tau, e0 * e1, P);
  } else {
    const T s0 = e0 * e0, s1 = e1 * e1, s2 = e2 * e2;
    g0 = s1 * s2;
    g1 = s0 * s2;
    g2 = s0 * s1;
  }
  S = fma(kk.k6, g1, fma(kk.k3, g2, g0));
  numh = fma(S, q1h, fma(g0, d01, -((kk.k1_5 * g2) * d21n)));
}

// Both sides of x/y face i+½ from p = f⁺(i-2..i+2), m = f⁻(i-1..i+3); w5_combine6 of
// them is 3 x the face flux.
template <typename T, bool ZVARIANT, class K = W5Lit<T>>
__device__ __forceinline__ void w5_face3_sides(const T* p, const T* m, T& n1, T& S1, T& n2,
                                               T& S2, const K& kk = K{}) {
  w5_side_h<T, ZVARIANT>(p[0], p[1], p[2], p[3], p[4], n1, S1, kk);
  w5_side_h<T, ZVARIANT>(m[4], m[3], m[2], m[1], m[0], n2, S2, kk);
}

// Left-biased WENO7 (Jiang–Shu weights) at the right face of v3 from v0..v6 (= f at
// i-3..i+3), as numerator/denominator.  Smoothness indicators and candidate stencils
// exactly as the MATLAB prototype (Matlab_Prototipes/InviscidBurgersNd/WENO7resAdv1d.m;
// CPU port: models/prototypes.py::weno7_res), linear weights (1, 12, 18, 4)/35 and
// eps = 1e-6; alpha_k = g_k/(eps+beta_k)² over the common denominator Π_k (eps+beta_k)²
// (the /35 cancels).  The beta_k are symmetric under stencil reversal, so the f⁻ side
// is this function on the mirrored stencil.
template <typename T>
__device__ __forceinline__ void weno7_nd(T m3, T m2, T m1, T o, T p1, T p2, T p3, T& num,
                                         T& den) {
#pragma clang fp contract(off)
  constexpr T eps = T(1e-6);
  const T b0 = fma(m1, fma(T(134241), m1, T(-114894) * o),
               fma(m3, fma(T(56694), m1, fma(T(-47214), m2, fma(T(6649), m3, T(-22778) * o))),
               fma(T(25729) * o, o, m2 * fma(T(-210282), m1, fma(T(85641), m2, T(86214) * o)))));
  const T b1 = fma(o, fma(T(41001), o, T(-30414) * p1),
               fma(m2, fma(T(-19374), m1, fma(T(3169), m2, fma(T(19014), o, T(-5978) * p1))),
               fma(T(6649) * p1, p1, m1 * fma(T(33441), m1, fma(T(-70602), o, T(23094) * p1)))));
  const T b2 = fma(p1, fma(T(33441), p1, T(-19374) * p2),
               fma(m1, fma(T(6649), m1, fma(T(-30414), o, fma(T(23094), p1, T(-5978) * p2))),
               fma(T(3169) * p2, p2, o * fma(T(41001), o, fma(T(-70602), p1, T(19014) * p2)))));
  const T b3 = fma(p2, fma(T(85641), p2, T(-47214) * p3),
               fma(o, fma(T(25729), o, fma(T(-114894), p1, fma(T(86214), p2, T(-22778) * p3))),
               fma(T(6649) * p3, p3, p1 * fma(T(134241), p1, fma(T(-210282), p2, T(56694) * p3)))));
  // candidate polynomials (times 12)
  const T q0 = fma(T(25), o, fma(T(-23), m1, fma(T(13), m2, T(-3) * m3)));
  const T q1 = fma(T(3), p1, fma(T(13), o, fma(T(-5), m1, m2)));
  const T q2 = fma(T(7), p1, fma(T(7), o, -(m1 + p2)));
  const T q3 = fma(T(13), p1, fma(T(-5), p2, fma(T(3), o, p3)));
  const T e0 = eps + b0, e1 = eps + b1, e2 = eps + b2, e3 = eps + b3;
  const T s0 = e0 * e0, s1 = e1 * e1, s2 = e2 * e2, s3 = e3 * e3;
  const T s01 = s0 * s1, s23 = s2 * s3;
  // alpha_k ∝ g_k Π_{j≠k} s_j
  const T w0 = s23 * s1, w1 = T(12) * (s23 * s0), w2 = T(18) * (s01 * s3), w3 = T(4) * (s01 * s2);
  num = fma(w0, q0, fma(w1, q1, fma(w2, q2, w3 * q3)));
  den = T(12) * (((w0 + w1) + w2) + w3);
}

// WENO7 numerical flux at face i+½ from fp(i-3..i+3) and fm(i-2..i+4).
template <typename T>
__device__ __forceinline__ T weno7_face(const T* p, const T* m) {
#pragma clang fp contract(off)
  T n1, d1, n2, d2;
  weno7_nd<T>(p[0], p[1], p[2], p[3], p[4], p[5], p[6], n1, d1);
  weno7_nd<T>(m[6], m[5], m[4], m[3], m[2], m[1], m[0], n2, d2);
  if constexpr (sizeof(T) == 8) {
    return fast_div(fma(n1, d2, n2 * d1), d1 * d2);
  } else {
    return fast_div(n1, d1) + fast_div(n2, d2);
  }
}

// Face-flux reconstruction by scheme: W = 5 (WZ: Jiang–Shu / Borges-Z) or 7 (Jiang–Shu).
// face(p, m): flux at c+½ from p = f⁺(c-R+1 .. c+R-1), m = f⁻(c-R+2 .. c+R).
template <typename T, int W, bool WZ>
struct Recon;

template <typename T, bool WZ>
struct Recon<T, 5, WZ> {
  static constexpr int R = 3;
  __device__ __forceinline__ static T face(const T* p, const T* m) {
    return weno5_face<T, WZ>(p[0], p[1], p[2], p[3], p[4], m[0], m[1], m[2], m[3], m[4]);
  }
};

template <typename T>
struct Recon<T, 7, false> {
  static constexpr int R = 4;
  __device__ __forceinline__ static T face(const T* p, const T* m) { return weno7_face<T>(p, m); }
};

// ---------------------------------------------------------------------------------
// Cross-lane shifts inside a 64-wide wave (DPP wave_shr:1 / wave_shl:1, pure VALU, no
// LDS traffic): lane i receives lane i-1 (shr) / i+1 (shl); lanes without a source get 0.
// Every lane of the wave must execute them (call only under wave-uniform control flow).
// ---------------------------------------------------------------------------------
// bound_ctrl = 1: lanes without a source read 0 and no "old" value has to be
// materialised (update_dpp with old = 0 costs an extra v_mov per 32-bit half).
template <int CTRL>
__device__ __forceinline__ double dpp_move(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xf, 0xf, true);
  hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp_move(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ f32x2 dpp_move(f32x2 v) {
  return f32x2{dpp_move<CTRL>(v.x), dpp_move<CTRL>(v.y)};
}
template <typename T>
__device__ __forceinline__ T wave_shr1(T v) { return dpp_move<0x138>(v); }  // from lane i-1
template <typename T>
__device__ __forceinline__ T wave_shl1(T v) { return dpp_move<0x130>(v); }  // from lane i+1

// Adaptive-CFL step size read from device memory (advdiff_adaptive_dt): false when the
// run has reached t_end (dt == 0), i.e. the stage is a no-op.
template <typename T>
__device__ __forceinline__ bool device_dt(const double* dtp, T& dt) {
  const double d = *dtp;
  if (d == 0.0) return false;
  dt = T(d);
  return true;
}

// ---------------------------------------------------------------------------------
// Stage epilogues.  MODE selects the time integrator's per-stage update:
//   kSsp1 : out = b (c + dt L)                      (SSP-RK3 stage 1)
//   kSsp  : out = a aux + b (c + dt L)              (SSP-RK3, aux = u^n)
//   kLs1  : d = dt L;          aux = d; out = c + b d   (low-storage RK, first stage)
//   kLs   : d = a aux + dt L;  aux = d; out = c + b d   (Carpenter–Kennedy 2N storage)
// ---------------------------------------------------------------------------------
enum : int { kSsp1 = 0, kSsp = 1, kLs1 = 2, kLs = 3 };

template <int MODE>
constexpr bool reads_aux() { return MODE == kSsp || MODE == kLs; }

template <typename T, int MODE>
__device__ __forceinline__ T stage_value(T ax, T c, T L, T dt, T a, T b, T& dnew) {
#pragma clang fp contract(off)
  if constexpr (MODE == kSsp1 || MODE == kSsp) {
    return rk_stage<T, MODE == kSsp>(ax, c, L, dt, a, b);
  } else {
    T d = dt * L;
    if constexpr (MODE == kLs) d = fma(a, ax, d);
    dnew = d;
    return fma(b, d, c);
  }
}

// out[o] (and aux[o] for low-storage modes) of an active cell
template <typename T, int MODE>
__device__ __forceinline__ void stage_store(T* out, T* aux, int64_t o, T ax, T c, T L, T dt,
                                            T a, T b) {
  T d = T(0);
  out[o] = stage_value<T, MODE>(ax, c, L, dt, a, b, d);
  if constexpr (MODE == kLs1 || MODE == kLs) aux[o] = d;
}

// Folded heat stage (see FdCoef): base term of the chain for MODE, and the epilogue.
// SSP: chain = [a u0 +] KC c + Σ..., out = chain.  Low-storage: chain = [a du +] dt L = d,
// du = d, out = c + b d.
template <typename T, int MODE>
__device__ __forceinline__ T fd_start(T kc, T c, T ax, T a) {
  if constexpr (reads_aux<MODE>())
    return fd_ctr(kc, c, a * ax);
  else
    return fd_ctr(kc, c);
}
template <typename T, int MODE>
__device__ __forceinline__ void fd_store(T* out, T* aux, int64_t o, T c, T acc, T b) {
#pragma clang fp contract(off)
  if constexpr (MODE == kSsp1 || MODE == kSsp) {
    out[o] = acc;
  } else {
    aux[o] = acc;
    out[o] = fma(b, acc, c);
  }
}

// ---------------------------------------------------------------------------------
// Addressing helpers shared by the v3-shaped kernels (fused heat step, WENO5 v6):
// byte-offset LDS access (immediate ds offsets) and per-plane buffer resources.
// ---------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T lds_ld(const char* base, int byte_off) {
  return *(const T*)(base + byte_off);
}
template <typename T>
__device__ __forceinline__ void lds_st(char* base, int byte_off, T v) {
  *(T*)(base + byte_off) = v;
}
// Plane-relative global access through a raw buffer resource: the plane base lives in
// the (scalar) descriptor and the per-lane part is a 32-bit byte offset, so a load or
// store costs no VALU address arithmetic (gfx9 descriptor word 3 = 0x00020000; the range
// check is disabled by num_records = 2^32 - 1; offsets stay inside one plane < 2^31 B).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ T gld(__amdgpu_buffer_rsrc_t r, uint32_t boff) {
  if constexpr (sizeof(T) == 8)
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, (int)boff, 0, 0));
  else
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, (int)boff, 0, 0));
}
template <typename T>
__device__ __forceinline__ void gst(__amdgpu_buffer_rsrc_t r, uint32_t boff, T v) {
  if constexpr (sizeof(T) == 8)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)boff, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)boff, 0, 0);
}

// Fused halo puts of a slab rank (ipc transport, round 6): the output planes [k0, k1) of a
// launch, rows [y0, y1) of them, are ALSO stored into a peer — part p's cell (k, y, x)
// goes to dst[p] + (k - k0[p]) pb[p] + the own in-plane byte offset of (y, x): dst[p] is
// set up so that holds for the peer's receive box (the neighbour's ghost planes, or a
// relay helper's row buffer of a striped exchange: then dst is offset by -y0 rows and pb
// is the buffer's plane size; every receive box has this field's row pitch).  Up to
// kHaloParts parts: the direct faces (2) or the striped ones (direct + helper parts per
// face).  System-scope stores, as ipc.hip's put kernel; the signal kernel after the
// launch publishes them.
constexpr int kHaloParts = 6;
struct HaloPut {
  char* dst[kHaloParts];
  int64_t pb[kHaloParts];
  int k0[kHaloParts], k1[kHaloParts], y0[kHaloParts], y1[kHaloParts];
  int n;  // parts in use
};
// The store: a buffer store on a scalar base (no 64-bit per-lane address — as a flat
// pointer the loop-invariant part dst + off was hoisted into VGPRs and spilled) with
// cache policy sc0 sc1 (aux 1 | 16), the code gfx942's memory model gives a relaxed
// system-scope atomic store: written through this XCD's L2 to the peer.
constexpr int kSysScopeStore = 1 | 16;
template <typename T>
__device__ __forceinline__ void halo_put(const HaloPut& put, int k, int y, uint32_t off, T v) {
#pragma unroll
  for (int s = 0; s < kHaloParts; ++s)
    if (s < put.n && k >= put.k0[s] && k < put.k1[s] && y >= put.y0[s] && y < put.y1[s]) {
      const auto r = __builtin_amdgcn_make_buffer_rsrc(
          put.dst[s] + (int64_t)(k - put.k0[s]) * put.pb[s], (short)0, -1, 0x00020000);
      if constexpr (sizeof(T) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)off, 0,
                                              kSysScopeStore);
      else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0,
                                              kSysScopeStore);
    }
}
// The direct two-face form (the WENO5 stage: the kernel is at its SGPR limit, and the six
// row-ranged parts of HaloPut cost it VGPR spills): all rows, this field's plane stride.
struct HaloPut2 {
  char* dst[2];
  int k0[2], k1[2];
};
template <typename T>
__device__ __forceinline__ void halo_put2(const HaloPut2& put, int k, int64_t plane_bytes,
                                          uint32_t off, T v) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
    if (k >= put.k0[s] && k < put.k1[s]) {
      const auto r = __builtin_amdgcn_make_buffer_rsrc(
          put.dst[s] + (int64_t)(k - put.k0[s]) * plane_bytes, (short)0, -1, 0x00020000);
      if constexpr (sizeof(T) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)off, 0,
                                              kSysScopeStore);
      else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0,
                                              kSysScopeStore);
    }
}
// host: a HaloPut of up to kHaloParts parts from arrays (null dst or empty range: skipped)
inline bool make_halo_put(int n, void* const* dst, const int* k0, const int* k1, const int* y0,
                          const int* y1, const int64_t* pb, int nz_alloc, HaloPut& out) {
  out = HaloPut{};
  if (n < 0 || n > kHaloParts) return false;
  for (int s = 0; s < n; ++s) {
    if (dst[s] == nullptr || k1[s] <= k0[s] || y1[s] <= y0[s]) continue;
    if (k0[s] < 0 || k1[s] > nz_alloc || pb[s] <= 0) return false;
    const int q = out.n++;
    out.dst[q] = (char*)dst[s];
    out.pb[q] = pb[s];
    out.k0[q] = k0[s];
    out.k1[q] = k1[s];
    out.y0[q] = y0[s];
    out.y1[q] = y1[s];
  }
  return true;
}

// keep a value computed on every lane (no exec-masked skip of the computation): the
// frozen-cell choice below it must be a v_cndmask, not a branch around the stencil
template <typename T>
__device__ __forceinline__ T pin(T v) {
  asm volatile("" : "+v"(v));
  return v;
}

}  // namespace advdiff
