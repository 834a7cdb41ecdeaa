// Auxiliary device kernels: reductions (CFL max|u|, L1/L2/Linf error norms), device
// initial conditions, strided box copies (halo pack/unpack) and build info.
//
// Reference counterparts: host-side Init_domain / Call_Init3D (MultiGPU/*/Tools.c:124-175,
// SingleGPU/Diffusion3d_baselineCode/tools.cpp:92-143), CalcError (tools.cpp:156-180,
// with its `u[i]` indexing bug fixed), copy_br_to_gc / copy_gc_to_br
// (MultiGPU/Diffusion3d_Baseline/Kernels.cu:32-99) and the unbuilt max-reduction fragment
// SingleGPU/Burgers3d_WENO5/max.c.  Here every rank builds its own slab on the device
// (no host scatter of a global array) and reductions are deterministic two-pass trees.
#include "common.hpp"
#include "launch.hpp"
#include "advdiff/kernels.h"

#include <math.h>

namespace advdiff {

constexpr int kRedBlocks = 1024;
constexpr int kRedThreads = 256;

struct Norm3 {
  double s1, s2, mx;
};

__device__ __forceinline__ Norm3 combine(Norm3 a, Norm3 b) {
  return {a.s1 + b.s1, a.s2 + b.s2, fmax(a.mx, b.mx)};
}

__device__ __forceinline__ Norm3 wave_reduce(Norm3 v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    Norm3 o{__shfl_down(v.s1, off), __shfl_down(v.s2, off), __shfl_down(v.mx, off)};
    v = combine(v, o);
  }
  return v;
}

__device__ Norm3 block_reduce(Norm3 v) {
  __shared__ Norm3 part[kRedThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  v = wave_reduce(v);
  if (lane == 0) part[w] = v;
  __syncthreads();
  if (w == 0) {
    v = lane < kRedThreads / kWave ? part[lane] : Norm3{0.0, 0.0, 0.0};
    v = wave_reduce(v);
  }
  return v;
}

template <typename T>
__global__ __launch_bounds__(kRedThreads) void norms_partial(const T* __restrict__ x,
                                                             const T* __restrict__ y,
                                                             int64_t sy, int64_t sz, int i0,
                                                             int ni, int j0, int nj, int k0,
                                                             int nk, Norm3* __restrict__ part) {
  Norm3 acc{0.0, 0.0, 0.0};
  const int64_t nrows = (int64_t)nj * nk;
  // one row segment per (wave-strided) iteration: coalesced along x
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int jj = (int)(r % nj), kk = (int)(r / nj);
    const int64_t base = (int64_t)(k0 + kk) * sz + (int64_t)(j0 + jj) * sy + i0;
    for (int ii = threadIdx.x; ii < ni; ii += kRedThreads) {
      double d = (double)x[base + ii];
      if (y) d -= (double)y[base + ii];
      const double ad = fabs(d);
      acc.s1 += ad;
      acc.s2 += d * d;
      acc.mx = fmax(acc.mx, ad);
    }
  }
  acc = block_reduce(acc);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kRedThreads) void norms_final(const Norm3* __restrict__ part,
                                                           int n, double* __restrict__ out) {
  Norm3 acc{0.0, 0.0, 0.0};
  for (int q = threadIdx.x; q < n; q += kRedThreads) acc = combine(acc, part[q]);
  acc = block_reduce(acc);
  if (threadIdx.x == 0) {
    out[0] = acc.s1;
    out[1] = acc.s2;
    out[2] = acc.mx;
  }
}

// ------------------------------------------------------------------------------
// Initial conditions.  Coordinates are vertex-centred: x_i = i*dx on [0, L].
// ------------------------------------------------------------------------------
template <typename T>
__global__ void init_ic_kernel(int ic, T* u, int nx, int ny, int nzl, int64_t sy, int64_t sz,
                               int ig0, int jg0, int kg0, int NX, int NY, int NZ, double dx,
                               double dy, double dz, double p0, double p1, int twod) {
  const int il = blockIdx.x * blockDim.x + threadIdx.x;
  const int jl = blockIdx.y * blockDim.y + threadIdx.y;
  const int kl = blockIdx.z;
  if (il >= nx || jl >= ny || kl >= nzl) return;
  // global indices of the local box (ghost cells beyond the domain are zero)
  const int i = ig0 + il;
  const int jg = jg0 + jl;
  const int k = twod ? 0 : kg0 + kl;
  const double x = i * dx, y = jg * dy, z = k * dz;
  const double cx = 0.5 * (NX - 1) * dx, cy = 0.5 * (NY - 1) * dy, cz = 0.5 * (NZ - 1) * dz;
  const bool face = i == 0 || i == NX - 1 || jg == 0 || jg == NY - 1 ||
                    (!twod && (k == 0 || k == NZ - 1));
  const bool outside = jg < 0 || jg >= NY || i < 0 || i >= NX || (!twod && (k < 0 || k >= NZ));
  double v = 0.0;
  switch (ic) {
    case 1: {  // square jump: 1 inside the middle half of every axis
      const bool in = i >= NX / 4 && i < 3 * NX / 4 && jg >= NY / 4 && jg < 3 * NY / 4 &&
                      (twod || (k >= NZ / 4 && k < 3 * NZ / 4));
      v = in ? 1.0 : 0.0;
      break;
    }
    case 2: {  // sine: sin(pi x/Lx) sin(pi y/Ly) sin(pi z/Lz), zero faces
      const double Lx = (NX - 1) * dx, Ly = (NY - 1) * dy, Lz = (NZ - 1) * dz;
      v = sin(M_PI * x / Lx) * sin(M_PI * y / Ly) * (twod ? 1.0 : sin(M_PI * z / Lz));
      if (face) v = 0.0;
      break;
    }
    case 3: {  // heat kernel at time t0 = p1, diffusivity d = p0, centred; zero faces
      const double r2 = (x - cx) * (x - cx) + (y - cy) * (y - cy) + (twod ? 0.0 : (z - cz) * (z - cz));
      v = exp(-r2 / (4.0 * p0 * p1));
      if (face) v = 0.0;
      break;
    }
    case 4: {  // Burgers Gaussian exp(-r²/w), w = p0, centred
      const double r2 = (x - cx) * (x - cx) + (y - cy) * (y - cy) + (twod ? 0.0 : (z - cz) * (z - cz));
      v = exp(-r2 / p0);
      break;
    }
    case 5: {  // hot plates: two bottom / two top planes (rows in 2-D) at 1
      const int kk = twod ? jg : k, nn = twod ? NY : NZ;
      v = (kk < 2 || kk >= nn - 2) ? 1.0 : 0.0;
      break;
    }
    case 6: {  // disc of radius p0 (relative to the shorter side) at the centre
      const double r2 = (x - cx) * (x - cx) + (y - cy) * (y - cy);
      const double R = p0 * fmin((NX - 1) * dx, (NY - 1) * dy);
      v = r2 < R * R ? 1.0 : 0.0;
      break;
    }
    default:
      v = 0.0;
  }
  if (outside) v = 0.0;
  u[(int64_t)kl * sz + (int64_t)jl * sy + il] = (T)v;
}

template <typename T>
__global__ void copy_box_kernel(T* __restrict__ dst, int64_t dsy, int64_t dsz,
                                const T* __restrict__ src, int64_t ssy, int64_t ssz, int ni,
                                int nj) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  const int k = blockIdx.z;
  if (i >= ni || j >= nj) return;
  dst[(int64_t)k * dsz + (int64_t)j * dsy + i] = src[(int64_t)k * ssz + (int64_t)j * ssy + i];
}

template <typename T>
__global__ void scale_kernel(T* __restrict__ x, int64_t n, T s) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x)
    x[q] *= s;
}

// Adaptive-CFL step size on the device (one lane): the host loop of solver.py
// (Burgers.stable_dt + the t_end clamp) evaluated in the same order, so the step
// sequence is bit-identical to the host-driven path.  state = [t, dt, steps].
__global__ void adaptive_dt_kernel(const double* __restrict__ red, double* state, double cfl_h,
                                   double dt_visc, double t_end, int has_tend) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double t = state[0];
  double dt = 0.0;
  if (!(has_tend && t >= t_end * (1.0 - 1e-14))) {
    const double u = red[2] >= 1e-300 ? red[2] : 1e-300;  // max(umax, 1e-300)
    dt = cfl_h / u;
    if (dt_visc > 0.0 && dt_visc < dt) dt = dt_visc;
    if (has_tend && t + dt > t_end) dt = t_end - t;
  }
  state[1] = dt;
  if (dt != 0.0) {
    state[0] = t + dt;
    state[2] = state[2] + 1.0;
  }
}

}  // namespace advdiff

extern "C" int advdiff_adaptive_dt(const double* red, double* state, double cfl_h,
                                   double dt_visc, double t_end, int has_tend, void* stream) {
  hipLaunchKernelGGL(advdiff::adaptive_dt_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     red, state, cfl_h, dt_visc, t_end, has_tend);
  return hipGetLastError();
}

extern "C" int advdiff_scale(int dtype, void* x, int64_t n, double s, void* stream) {
  using namespace advdiff;
  if (n <= 0) return hipSuccess;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)std::min<int64_t>((n + 255) / 256, 4096);
  if (dtype == ADVDIFF_F64)
    hipLaunchKernelGGL(scale_kernel<double>, dim3(nb), dim3(256), 0, st, (double*)x, n, s);
  else if (dtype == ADVDIFF_F32)
    hipLaunchKernelGGL(scale_kernel<float>, dim3(nb), dim3(256), 0, st, (float*)x, n, (float)s);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" size_t advdiff_reduce_workspace_bytes(void) {
  return sizeof(advdiff::Norm3) * advdiff::kRedBlocks;
}

extern "C" int advdiff_reduce_norms(int dtype, const void* x, const void* y, int64_t sy,
                                    int64_t sz, int i0, int i1, int j0, int j1, int k0, int k1,
                                    void* workspace, double* result, void* stream) {
  using namespace advdiff;
  hipStream_t st = (hipStream_t)stream;
  const int ni = i1 - i0, nj = j1 - j0, nk = k1 - k0;
  if (ni <= 0 || nj <= 0 || nk <= 0) {
    return hipMemsetAsync(result, 0, 3 * sizeof(double), st);
  }
  const int64_t rows = (int64_t)nj * nk;
  const int nb = (int)std::min<int64_t>(rows, kRedBlocks);
  Norm3* part = (Norm3*)workspace;
  if (dtype == ADVDIFF_F64)
    hipLaunchKernelGGL(norms_partial<double>, dim3(nb), dim3(kRedThreads), 0, st,
                       (const double*)x, (const double*)y, sy, sz, i0, ni, j0, nj, k0, nk, part);
  else if (dtype == ADVDIFF_F32)
    hipLaunchKernelGGL(norms_partial<float>, dim3(nb), dim3(kRedThreads), 0, st,
                       (const float*)x, (const float*)y, sy, sz, i0, ni, j0, nj, k0, nk, part);
  else
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(norms_final, dim3(1), dim3(kRedThreads), 0, st, part, nb, result);
  return hipGetLastError();
}

extern "C" int advdiff_init_ic_box(int dtype, int ic, void* u, int nx, int ny, int nzl,
                                   int64_t sy, int64_t sz, int ig0, int jg0, int kg0, int NX,
                                   int NY, int NZ, double dx, double dy, double dz, double p0,
                                   double p1, void* stream) {
  using namespace advdiff;
  hipStream_t st = (hipStream_t)stream;
  const int twod = NZ <= 1 ? 1 : 0;
  dim3 block(64, 4, 1), grid(div_up(nx, 64), div_up(ny, 4), std::max(nzl, 1));
  if (dtype == ADVDIFF_F64)
    hipLaunchKernelGGL(init_ic_kernel<double>, grid, block, 0, st, ic, (double*)u, nx, ny,
                       std::max(nzl, 1), sy, sz, ig0, jg0, kg0, NX, NY, NZ, dx, dy, dz, p0, p1,
                       twod);
  else if (dtype == ADVDIFF_F32)
    hipLaunchKernelGGL(init_ic_kernel<float>, grid, block, 0, st, ic, (float*)u, nx, ny,
                       std::max(nzl, 1), sy, sz, ig0, jg0, kg0, NX, NY, NZ, dx, dy, dz, p0, p1,
                       twod);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" int advdiff_init_ic(int dtype, int ic, void* u, int nx, int ny, int nzl, int64_t sy,
                               int64_t sz, int kg0, int NX, int NY, int NZ, double dx, double dy,
                               double dz, double p0, double p1, void* stream) {
  // slabs: 3-D offset along z, 2-D offset along y (rows)
  const bool twod = NZ <= 1;
  return advdiff_init_ic_box(dtype, ic, u, nx, ny, nzl, sy, sz, 0, twod ? kg0 : 0,
                             twod ? 0 : kg0, NX, NY, NZ, dx, dy, dz, p0, p1, stream);
}

extern "C" int advdiff_copy_box(int dtype, void* dst, int64_t dsy, int64_t dsz, const void* src,
                                int64_t ssy, int64_t ssz, int ni, int nj, int nk, void* stream) {
  using namespace advdiff;
  if (ni <= 0 || nj <= 0 || nk <= 0) return hipSuccess;
  hipStream_t st = (hipStream_t)stream;
  dim3 block(256), grid(div_up(ni, 256), nj, nk);
  if (dtype == ADVDIFF_F64)
    hipLaunchKernelGGL(copy_box_kernel<double>, grid, block, 0, st, (double*)dst, dsy, dsz,
                       (const double*)src, ssy, ssz, ni, nj);
  else if (dtype == ADVDIFF_F32)
    hipLaunchKernelGGL(copy_box_kernel<float>, grid, block, 0, st, (float*)dst, dsy, dsz,
                       (const float*)src, ssy, ssz, ni, nj);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

namespace advdiff {
// Device-side dump of a small box (one thread, printf) — the reference's PrintGPUmemory
// debug kernels (MultiGPU/Diffusion3d_Baseline/Kernels.cu).
template <typename T>
__global__ void debug_print_kernel(const T* u, int64_t sy, int64_t sz, int i0, int i1, int j0,
                                   int j1, int k0, int k1) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int k = k0; k < k1; ++k) {
    printf("[k=%d]\n", k);
    for (int j = j0; j < j1; ++j) {
      for (int i = i0; i < i1; ++i) printf("%8.4f ", (double)u[(int64_t)k * sz + (int64_t)j * sy + i]);
      printf("\n");
    }
  }
}

}  // namespace advdiff

extern "C" int advdiff_debug_print(int dtype, const void* u, int64_t sy, int64_t sz, int i0,
                                   int i1, int j0, int j1, int k0, int k1, void* stream) {
  using namespace advdiff;
  hipStream_t st = (hipStream_t)stream;
  if ((int64_t)(i1 - i0) * (j1 - j0) * (k1 - k0) > 4096) return hipErrorInvalidValue;
  if (dtype == ADVDIFF_F64)
    hipLaunchKernelGGL(debug_print_kernel<double>, dim3(1), dim3(64), 0, st, (const double*)u,
                       sy, sz, i0, i1, j0, j1, k0, k1);
  else if (dtype == ADVDIFF_F32)
    hipLaunchKernelGGL(debug_print_kernel<float>, dim3(1), dim3(64), 0, st, (const float*)u, sy,
                       sz, i0, i1, j0, j1, k0, k1);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" int advdiff_device_info(int dev, int64_t* out, int n) {
  // [cu_count, ecc_enabled, l2_bytes, lds_per_block, clock_khz, mem_clock_khz,
  //  mem_bus_bits, warp_size]  (the reference's DeviceScan / ECCCheck, Util.cu:32-93)
  const hipDeviceAttribute_t attrs[] = {
      hipDeviceAttributeMultiprocessorCount, hipDeviceAttributeEccEnabled,
      hipDeviceAttributeL2CacheSize,         hipDeviceAttributeMaxSharedMemoryPerBlock,
      hipDeviceAttributeClockRate,           hipDeviceAttributeMemoryClockRate,
      hipDeviceAttributeMemoryBusWidth,      hipDeviceAttributeWarpSize};
  const int na = (int)(sizeof(attrs) / sizeof(attrs[0]));
  for (int i = 0; i < n && i < na; ++i) {
    int v = -1;
    const hipError_t e = hipDeviceGetAttribute(&v, attrs[i], dev);
    if (e != hipSuccess) return e;
    out[i] = v;
  }
  return hipSuccess;
}

extern "C" int advdiff_peer_info(int a, int b, int* can_access, int* link_type, int* hops) {
  // xGMI topology between two devices: peer access, HSA link type (4 = xGMI), hop count
  hipError_t e = hipDeviceCanAccessPeer(can_access, a, b);
  if (e != hipSuccess) return e;
  uint32_t lt = 0, hc = 0;
  e = hipExtGetLinkTypeAndHopCount(a, b, &lt, &hc);
  if (e != hipSuccess) return e;
  *link_type = (int)lt;
  *hops = (int)hc;
  return hipSuccess;
}

extern "C" const char* advdiff_build_info(void) {
  return "libadvdiff gfx950 (CDNA4) HIP kernels: diffusion{2,3}d FD2/FD4 fused SSP-RK3, "
         "burgers{2,3}d WENO5-JS/Z fused SSP-RK3, norms, init, copy_box";
}

// Load every kernel translation unit's code object now (outside any timed region).  With
// deferred loading (the HIP default) a code object is loaded at the first launch of one
// of its kernels — for the WENO5 file (many template instances) ~20-25 ms, which landed
// inside the first timed step of a run (profiles/archive/native_apps_r2.log).
extern "C" int advdiff_preload_burgers(void);
extern "C" int advdiff_preload_diffusion(void);
extern "C" int advdiff_preload_diffusion_fused(void);
extern "C" int advdiff_preload_diffusion2d_fused(void);
extern "C" int advdiff_preload(void) {
  hipFuncAttributes a;
  int e = hipFuncGetAttributes(&a, (const void*)advdiff::init_ic_kernel<double>);
  if (e == hipSuccess) e = advdiff_preload_diffusion();
  if (e == hipSuccess) e = advdiff_preload_diffusion_fused();
  if (e == hipSuccess) e = advdiff_preload_diffusion2d_fused();
  if (e == hipSuccess) e = advdiff_preload_burgers();
  return e;
}
