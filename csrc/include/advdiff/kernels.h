// C ABI of libadvdiff: hand-written gfx950 (CDNA4) HIP stencil kernels.
//
// Every entry point enqueues work on the given HIP stream (nullptr = legacy default
// stream), never synchronises, never allocates, and returns a hipError_t value
// (0 = success) so it can be captured into a hipGraph and called from Python
// (ctypes) or from the native C++ apps alike.
//
// Array layout (all kernels): x fastest.  Element (i, j, k) lives at
//     k*sz + j*sy + i
// where sy >= nx is the row pitch and sz >= ny*sy the plane pitch (elements).
// 2-D arrays use (i, j) -> j*sy + i.
//
// dtype codes: 0 = float32, 1 = float64.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum advdiff_dtype { ADVDIFF_F32 = 0, ADVDIFF_F64 = 1 };

// ---------------------------------------------------------------------------------
// Heat equation u_t = K ∇²u : ONE fused SSP-RK3 stage
//     out = a*u0 + b*(in + dt*L(in)),   L = FD4 (13-pt) or FD2 (7-pt) Laplacian
// on cells i in [border, nx-border), j in [border, ny-border), k in [k0, k1).
// cx = K/dx², cy = K/dy², cz = K/dz²  (the kernel applies the 1/12 of FD4).
// Reads planes k0-R .. k1-1+R of `in` (R = order/2), which must be allocated.
// a == 0 skips reading u0 (stage 1). `out` may alias `u0` (in-place stage 3),
// never `in`.
int advdiff_diffusion3d_stage(int dtype, const void* in, const void* u0, void* out,
                              int nx, int ny, int64_t sy, int64_t sz, int k0, int k1,
                              int border, int order, double cx, double cy, double cz,
                              double dt, double a, double b, void* stream);

// Heat equation: ONE FULL SSP-RK3 step in one launch (temporal blocking, 16 B/cell):
//     uout[k0:k1) = RK3(uin)  on i,j in [border, n-border).
// Intermediate stages are evaluated on planes [zlo, zhi) (cells outside are frozen:
// A = B = u there), so the launch reads uin planes k0-3R .. k1+3R-1 (clamped to
// [0, nz_alloc)).  Multi-GPU: ghost width 3R, one exchange per step.  uin != uout.
// Bit-identical to three advdiff_diffusion3d_stage launches.
int advdiff_diffusion3d_step(int dtype, const void* uin, void* uout, int nx, int ny,
                             int64_t sy, int64_t sz, int nz_alloc, int k0, int k1, int zlo,
                             int zhi, int border, int order, double cx, double cy, double cz,
                             double dt, void* stream);

// Low-storage RK stage (Carpenter–Kennedy 2N, e.g. LSRK4(5)) of the same operator:
//     d = A*du + dt*L(in);  du = d;  out = in + B*d      (A == 0: du is not read)
// `du` is read and written in place (pointwise); `out` must differ from `in`.
int advdiff_diffusion3d_stage_ls(int dtype, const void* in, void* du, void* out, int nx,
                                 int ny, int64_t sy, int64_t sz, int k0, int k1, int border,
                                 int order, double cx, double cy, double cz, double dt,
                                 double A, double B, void* stream);
// The same step on TWO plane ranges [k0,k1) and [k0b,k1b) in one launch (the two
// boundary slabs of a multi-GPU rank: one grid, better CU utilisation than two launches).
int advdiff_diffusion3d_step2(int dtype, const void* uin, void* uout, int nx, int ny,
                              int64_t sy, int64_t sz, int nz_alloc, int k0, int k1, int k0b,
                              int k1b, int zlo, int zhi, int border, int order, double cx,
                              double cy, double cz, double dt, void* stream);
// General form for blocks of a Cartesian decomposition, launched on a VIEW: box[8] =
// {xa0, xa1, ya0, ya1, xo0, xo1, yo0, yo1} (view coordinates): cells outside the active
// box [xa0,xa1) x [ya0,ya1) are frozen, u^{n+1} is written on active cells inside the
// output box [xo0,xo1) x [yo0,yo1) (which must lie >= 3R inside the view on split axes).
int advdiff_diffusion3d_step_box(int dtype, const void* uin, void* uout, int nx, int ny,
                                 int64_t sy, int64_t sz, int nz_alloc, int k0, int k1, int k0b,
                                 int k1b, int zlo, int zhi, const int* box, int order,
                                 double cx, double cy, double cz, double dt, void* stream);
// Launch-policy flags of the _ex entry (placement hints only, results are bit-identical).
//   ADVDIFF_EXCLUSIVE: the launch has the GPU to itself (single rank, or a full-range
//   launch after the halo wait).  Currently every launch uses the grid of z chunks (the
//   persistent schedule it used to select measured slower and was removed).
#define ADVDIFF_EXCLUSIVE 1
int advdiff_diffusion3d_step_box_ex(int dtype, const void* uin, void* uout, int nx, int ny,
                                    int64_t sy, int64_t sz, int nz_alloc, int k0, int k1,
                                    int k0b, int k1b, int zlo, int zhi, const int* box,
                                    int order, double cx, double cy, double cz, double dt,
                                    int flags, void* stream);
// A full-range slab step (planes [k0, k1), active box from `border`) whose output planes
// [lo_k0, lo_k1) / [hi_k0, hi_k1) are also stored, system scope, into the peer planes at
// dst_lo / dst_hi (IPC mappings of the neighbours' output fields: the peer plane of local
// plane lo_k0 / hi_k0; same row pitch and plane stride).  Null / empty: no peer that side.
// The general form (striped exchanges): part p's cells — planes [k0[p], k1[p]), rows
// [y0[p], y1[p]) — to dst[p] + (k - k0[p]) pb[p] + the own in-plane byte offset; up to 6
// parts, every receive box with this field's row pitch.
int advdiff_diffusion3d_step_putv(int dtype, const void* uin, void* uout, int nx, int ny,
                                  int64_t sy, int64_t sz, int nz_alloc, int k0, int k1, int zlo,
                                  int zhi, int border, int order, double cx, double cy,
                                  double cz, double dt, int nparts, void* const* dst,
                                  const int* k0s, const int* k1s, const int* y0s,
                                  const int* y1s, const int64_t* pb, void* stream);
int advdiff_diffusion3d_step_put(int dtype, const void* uin, void* uout, int nx, int ny,
                                 int64_t sy, int64_t sz, int nz_alloc, int k0, int k1, int zlo,
                                 int zhi, int border, int order, double cx, double cy,
                                 double cz, double dt, void* dst_lo, int lo_k0, int lo_k1,
                                 void* dst_hi, int hi_k0, int hi_k1, void* stream);
// 2-D heat: ONE FULL SSP-RK3 step per launch on rows [j0, j1) (intermediate stages on
// the active rows [ylo, yhi)); reads rows j0-3R .. j1+3R-1 (clamped to [0, ny_alloc)).
// Wave-independent y-march, no LDS; bit-identical to three advdiff_diffusion2d_stage.
int advdiff_diffusion2d_step(int dtype, const void* uin, void* uout, int nx, int64_t sy,
                             int ny_alloc, int j0, int j1, int ylo, int yhi, int border,
                             int order, double cx, double cy, double dt, void* stream);
// Cartesian-block form: box[4] = {xa0, xa1, xo0, xo1} (active / output columns, view coords).
int advdiff_diffusion2d_step_box(int dtype, const void* uin, void* uout, int nx, int64_t sy,
                                 int ny_alloc, int j0, int j1, int ylo, int yhi, const int* box,
                                 int order, double cx, double cy, double dt, void* stream);
// 2-D heat stage, rows j in [j0, j1), columns i in [border, nx-border).
int advdiff_diffusion2d_stage(int dtype, const void* in, const void* u0, void* out,
                              int nx, int64_t sy, int j0, int j1, int border, int order,
                              double cx, double cy, double dt, double a, double b,
                              void* stream);
int advdiff_diffusion2d_stage_ls(int dtype, const void* in, void* du, void* out, int nx,
                                 int64_t sy, int j0, int j1, int border, int order, double cx,
                                 double cy, double dt, double A, double B, void* stream);

// ---------------------------------------------------------------------------------
// Burgers u_t + Σ_d ∂_d(u²/2) = C ∇²u : ONE fused SSP-RK3 stage
//     L(u) = -Σ_d (F_{+½} - F_{-½}) * rd_d  +  C ∇²u (FD4)
// Reconstruction `weno`: 0 = WENO5-JS, 1 = WENO5-Z (Borges), 2 = WENO7-JS (the MATLAB
// prototype's LFWENO7), with local Lax-Friedrichs splitting.  Stencil radius R = 3
// (WENO5) / 4 (WENO7): reads planes k0-R .. k1+R-1 and needs border >= R.
// rdx = 1/dx ...; vx = C/dx² ... (all zero = inviscid, the viscous path is not
// compiled in).
// Burgers stages with the step size in device memory (adaptive CFL; nullptr: use dt).
// ls != 0: low-storage stage (aux = du).  A device dt of 0 makes the stage out = in.
int advdiff_burgers3d_stage_dt(int dtype, const void* in, void* aux, void* out, int nx, int ny,
                               int64_t sy, int64_t sz, int k0, int k1, int border, int weno,
                               double rdx, double rdy, double rdz, double vx, double vy,
                               double vz, double dt, double a, double b, int ls,
                               const double* dt_dev, void* stream);
// The 3-D stage on two plane ranges [k0, k1) and [k0b, k1b) (either may be empty): one
// launch with the default WENO5 kernel (a slab rank's two boundary slabs), else two.
int advdiff_burgers3d_stage2_dt(int dtype, const void* in, void* aux, void* out, int nx, int ny,
                                int64_t sy, int64_t sz, int k0, int k1, int k0b, int k1b,
                                int border, int weno, double rdx, double rdy, double rdz,
                                double vx, double vy, double vz, double dt, double a, double b,
                                int ls, const double* dt_dev, void* stream);
// One full-range stage of a slab rank whose output planes [lo_k0, lo_k1) / [hi_k0, hi_k1)
// also go, system scope, to the peer planes at dst_lo / dst_hi (fused halo puts; fp64,
// WENO5-JS / -Z, SSP-RK3 epilogues; see advdiff_diffusion3d_step_put).
int advdiff_burgers3d_stage_put(int dtype, const void* in, void* aux, void* out, int nx, int ny,
                                int64_t sy, int64_t sz, int k0, int k1, int border, int weno,
                                double rdx, double rdy, double rdz, double vx, double vy,
                                double vz, double dt, double a, double b, const double* dt_dev,
                                void* dst_lo, int lo_k0, int lo_k1, void* dst_hi, int hi_k0,
                                int hi_k1, void* stream);
int advdiff_burgers2d_stage_dt(int dtype, const void* in, void* aux, void* out, int nx,
                               int64_t sy, int j0, int j1, int border, int weno, double rdx,
                               double rdy, double vx, double vy, double dt, double a, double b,
                               int ls, const double* dt_dev, void* stream);
// Adaptive CFL step on the device: red = advdiff_reduce_norms result (max|u| at [2], after
// any cross-rank MAX), state = [t, dt, steps] (double[3], device): dt = min(cfl_h / max(
// umax, 1e-300), dt_visc if > 0), clamped to t_end (has_tend) and 0 once t >= t_end; t and
// steps advance with it.
int advdiff_adaptive_dt(const double* red, double* state, double cfl_h, double dt_visc,
                        double t_end, int has_tend, void* stream);

int advdiff_burgers3d_stage(int dtype, const void* in, const void* u0, void* out,
                            int nx, int ny, int64_t sy, int64_t sz, int k0, int k1,
                            int border, int weno, double rdx, double rdy, double rdz,
                            double vx, double vy, double vz, double dt, double a,
                            double b, void* stream);
// Low-storage RK stage of the Burgers operator (see advdiff_diffusion3d_stage_ls).
int advdiff_burgers3d_stage_ls(int dtype, const void* in, void* du, void* out, int nx, int ny,
                               int64_t sy, int64_t sz, int k0, int k1, int border, int weno,
                               double rdx, double rdy, double rdz, double vx, double vy,
                               double vz, double dt, double A, double B, void* stream);

int advdiff_burgers2d_stage(int dtype, const void* in, const void* u0, void* out,
                            int nx, int64_t sy, int j0, int j1, int border, int weno,
                            double rdx, double rdy, double vx, double vy, double dt,
                            double a, double b, void* stream);
int advdiff_burgers2d_stage_ls(int dtype, const void* in, void* du, void* out, int nx,
                               int64_t sy, int j0, int j1, int border, int weno, double rdx,
                               double rdy, double vx, double vy, double dt, double A, double B,
                               void* stream);

// ---------------------------------------------------------------------------------
// Reductions over the box [i0,i1)x[j0,j1)x[k0,k1):
//     result[0] = Σ|x - y|, result[1] = Σ(x - y)², result[2] = max|x - y|
// (y == nullptr means y = 0, i.e. norms / max|u| of x).  `result` is a DEVICE
// pointer to 3 doubles.  `workspace` must hold advdiff_reduce_workspace_bytes().
size_t advdiff_reduce_workspace_bytes(void);
int advdiff_reduce_norms(int dtype, const void* x, const void* y, int64_t sy, int64_t sz,
                         int i0, int i1, int j0, int j1, int k0, int k1, void* workspace,
                         double* result, void* stream);

// ---------------------------------------------------------------------------------
// Device-side initial conditions (no host staging, each rank builds its own slab).
// ic codes (see multigpu_advectiondiffusion_amd/utils/ics.py for the formulas):
//   0 zero, 1 square jump, 2 sine (zero faces), 3 heat kernel (zero faces),
//   4 Burgers Gaussian, 5 hot plates, 6 disc (2-D)
// The array holds global planes kg0 .. kg0+nzl-1; in 2-D (NZ <= 1) it holds the
// global rows kg0 .. kg0+ny-1 (nzl = 1).
// p0, p1: IC parameters (heat kernel: d, t0; Gaussian: width; others ignored).
int advdiff_init_ic(int dtype, int ic, void* u, int nx, int ny, int nzl, int64_t sy,
                    int64_t sz, int kg0, int NX, int NY, int NZ, double dx, double dy,
                    double dz, double p0, double p1, void* stream);

// Same for an arbitrary local box of a Cartesian decomposition: local (i, j, k) is global
// (ig0+i, jg0+j, kg0+k) (2-D: (ig0+i, jg0+j), nzl = 1); cells outside the domain are 0.
int advdiff_init_ic_box(int dtype, int ic, void* u, int nx, int ny, int nzl, int64_t sy,
                        int64_t sz, int ig0, int jg0, int kg0, int NX, int NY, int NZ,
                        double dx, double dy, double dz, double p0, double p1, void* stream);
// Copy planes (contiguous z-slabs) — a strided 3-D copy for halo staging and
// x/y-face pack/unpack of a Cartesian decomposition:
//   dst[(k)*dsz + j*dsy + i] = src[(k)*ssz + j*ssy + i], (i,j,k) in [0,ni)x[0,nj)x[0,nk)
int advdiff_copy_box(int dtype, void* dst, int64_t dsy, int64_t dsz, const void* src,
                     int64_t ssy, int64_t ssz, int ni, int nj, int nk, void* stream);

// x[0:n] *= s (contiguous), e.g. to scale a device-generated IC into an exact solution.
int advdiff_scale(int dtype, void* x, int64_t n, double s, void* stream);

// Debug dump (device printf) of the box [i0,i1)x[j0,j1)x[k0,k1) (at most 4096 values).
int advdiff_debug_print(int dtype, const void* u, int64_t sy, int64_t sz, int i0, int i1,
                        int j0, int j1, int k0, int k1, void* stream);
// Device scan: out[0..n) = CU count, ECC enabled, L2 bytes, LDS per workgroup, clock kHz,
// memory clock kHz, memory bus bits, wavefront size.
int advdiff_device_info(int dev, int64_t* out, int n);
// Peer topology: can_access (hipDeviceCanAccessPeer), HSA link type (4 = xGMI), hop count.
int advdiff_peer_info(int a, int b, int* can_access, int* link_type, int* hops);
// 3-D WENO5 stage kernel version (9 = default, 3 = the v3 fallback used for planes of
// 2 GiB and more); returns the previous value.  Results agree to rounding (tests).
int advdiff_set_b3_ver(int v);
// TWO fused SSP-RK3 steps of the 7-point heat equation in one launch (8 B of HBM traffic
// per cell and step): uout[k0:k1] = RK3(RK3(uin)) on the output box (the intermediate over
// the active box), bit-identical to two one-step launches
int advdiff_diffusion3d_step2x(int dtype, const void* uin, void* uout, int nx, int ny,
                               int64_t sy, int64_t sz, int nz_alloc, int k0, int k1, int zlo,
                               int zhi, const int* box, double cx, double cy, double cz,
                               double dt, void* stream);
// one FD2 step or two per launch for this shape (measured once per shape and process,
// uin untouched, uout used as scratch; ADVDIFF_STEP2=0/1 forces): *use2 = 1 for two
int advdiff_diffusion3d_step2_pick(int dtype, const void* uin, void* uout, int nx, int ny,
                                   int64_t sy, int64_t sz, int nz_alloc, int k0, int k1,
                                   int zlo, int zhi, const int* box, double cx, double cy,
                                   double cz, double dt, void* stream, int* use2);
// banded z schedule of the fused step: -1 (default) the measured choice per launch
// (advdiff_diffusion3d_step_sched_pick; uniform z chunks for an unmeasured launch), 0
// never, 1 always; returns the previous setting
int advdiff_set_step_banded(int on);
// host-only band model query: out[5] = {first band, later band, bands, makespan of that
// split, makespan of the best uniform chunking} (plane-times, one XCD's slots)
int advdiff_step_bands_plan(int n, long long tiles, long long slots, int warm, int minc,
                            long long* out);
// measure banded vs uniform z chunks for this fused-step launch (uin -> uout, uout is
// scratch; synchronous, outside graph capture), cache the faster, *banded = 1 if banded
int advdiff_diffusion3d_step_sched_pick(int dtype, const void* uin, void* uout, int nx, int ny,
                                        int64_t sy, int64_t sz, int nz_alloc, int k0, int k1,
                                        int zlo, int zhi, const int* box, int order, double cx,
                                        double cy, double cz, double dt, void* stream,
                                        int* banded);
// fp32 3-D WENO5 stage: packed pairs (1, default) or one cell per lane (0); returns the
// previous setting.  Bit-identical either way.
int advdiff_set_b3_pack(int on);
// v9 tile row width: 64, 32 or 0 = chosen per plane shape (returns the previous setting)
int advdiff_set_b3_tx(int v);
// v9 stage: forced z-chunk length (0 = the rounds model); returns the previous setting
int advdiff_set_b3_zchunk(int zc);
// 2-D WENO5 stage kernel version (2 = the barrier-free wave-strip kernel, default; 1 = the
// generic row-tile kernel); returns the previous value.
int advdiff_set_b2_ver(int v);

// ---------------------------------------------------------------------------------
// Peer transport of one node (ipc.hip): hipIpc-mapped device memory + device flags.  A
// rank puts boundary cells straight into a neighbour's ghost cells (advdiff_ipc_put: a box
// copy with system-scope stores into a mapped destination), raises the neighbour's flag (advdiff_ipc_signal) and makes its
// stream wait for its own flags (advdiff_ipc_wait).  All stream-ordered kernels: no host
// synchronisation, hipGraph-capturable.  Works across the GPUs of a node (xGMI) and
// between several processes on one GPU.
typedef struct advdiff_ipc advdiff_ipc;
typedef struct advdiff_ipc_addr {
  unsigned char handle[64];  // hipIpcMemHandle_t of the allocation
  uint64_t offset;           // byte offset of the address in it
  uint64_t bytes;            // allocation size
} advdiff_ipc_addr;
int advdiff_ipc_create(int world, int rank, advdiff_ipc** out);
int advdiff_ipc_destroy(advdiff_ipc* c);
int advdiff_ipc_describe(advdiff_ipc* c, const void* ptr, advdiff_ipc_addr* out);
int advdiff_ipc_flags_addr(advdiff_ipc* c, advdiff_ipc_addr* out);
int advdiff_ipc_map(advdiff_ipc* c, const advdiff_ipc_addr* a, void** ptr);
int advdiff_ipc_set_peer(advdiff_ipc* c, int peer, const advdiff_ipc_addr* peer_flags);
int advdiff_ipc_put(int dtype, void* dst, int64_t dsy, int64_t dsz, const void* src,
                    int64_t ssy, int64_t ssz, int ni, int nj, int nk, void* stream);
// channel ch (0..2) of the flag block: independent counters per (peer, channel)
int advdiff_ipc_signal_ch(advdiff_ipc* c, int ch, const int* peers, int n, void* stream);
int advdiff_ipc_wait_ch(advdiff_ipc* c, int ch, const int* peers, int n, void* stream);
int advdiff_ipc_signal(advdiff_ipc* c, const int* peers, int n, void* stream);
int advdiff_ipc_wait(advdiff_ipc* c, const int* peers, int n, void* stream);
// close every peer mapping except the flag blocks (collective, no put in flight): after
// fields were freed and reallocated
int advdiff_ipc_reset(advdiff_ipc* c);
int advdiff_ipc_errors(advdiff_ipc* c, long long* timeouts);

// Library identification (build flags, arch) for diagnostics.
const char* advdiff_build_info(void);
// sha256 (first 16 hex digits) of the kernel sources this library was built from
// (csrc/Makefile SRC_HASH); the Python loader refuses a library that does not match the tree
const char* advdiff_source_hash(void);

// Load the code objects of every kernel file now (the runtime otherwise loads each at its
// first launch, ~20 ms for the WENO5 file); call once after selecting the device.
int advdiff_preload(void);

#ifdef __cplusplus
}
#endif
