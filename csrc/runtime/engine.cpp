// Time-stepping engine of the native runtime (mirror of multigpu_advectiondiffusion_amd/solver.py).
//
// Per stage, on the compute stream:  interior(in->out)  -> wait(halo of in) ->
// boundary(in->out) -> event -> [comm stream] exchange of out's ghost planes, which
// overlaps the next stage's interior.  SSP-RK3 buffers u -> A -> B -> u (stage 3 in
// place), no Lu array, no uo copy.  Reference: MultiGPU/Diffusion3d_Baseline/main.c:189-303.
// 3-D heat: one temporally blocked launch per step (ghost width 3R, one exchange per
// step).  Low-storage RK4(5): u <-> A ping-pong, du in B.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "runtime.hpp"

namespace advdiff::rt {

Range Slab::compute_range(int border) const {
  const int lo = std::max(start(), border);
  const int hi = std::min(start() + count(), n - border);
  if (hi <= lo) return {ghost, ghost};
  return {to_local(lo), to_local(hi)};
}

void Slab::split(int border, int radius, Range& interior, Range& blo, Range& bhi) const {
  Range r = compute_range(border);
  const int o0 = ghost, o1 = ghost + count();
  if (r.empty()) {
    interior = blo = bhi = {r.lo, r.lo};
    return;
  }
  const int blo_end = lower() >= 0 ? std::min(r.hi, o0 + radius) : r.lo;
  const int bhi_start = upper() >= 0 ? std::max(r.lo, o1 - radius) : r.hi;
  blo = {r.lo, std::max(r.lo, blo_end)};
  if (bhi_start < blo.hi) {
    interior = {blo.hi, blo.hi};
    blo = r;
    bhi = {r.hi, r.hi};
    return;
  }
  bhi = {bhi_start, r.hi};
  interior = {blo.hi, bhi_start};
}

// Pitched allocation, the rule of solver.py _pitch_pads / pitch_default (4 fp64 / 16 fp32
// elements more per row and one more row per plane on 3-D fields past 128 MiB per rank:
// the fused heat step +3.8 % FD4 / +5.6 % FD2 at 512^3, profiles/r5/ab/pitch_solver_c_*.log).
// Global quantities only, so every slab rank gets the same plane layout.
void pitch_pads(const Problem& p, int world, int elem, int* px, int* py) {
  int x = p.pitch_px, y = p.pitch_py;
  if (x < 0 || y < 0) {
    const char* v = std::getenv("ADVDIFF_PITCH");
    int ex = 0, ey = 0;
    if (v && std::sscanf(v, "%d,%d", &ex, &ey) >= 1) {
      x = ex;
      y = ey;
    } else if (p.dims == 3 && p.cells() / std::max(world, 1) * elem > (int64_t)(128 << 20)) {
      x = elem == 8 ? 4 : 16;
      y = 1;
    } else {
      x = y = 0;
    }
  }
  *px = std::max(x, 0);
  *py = p.dims == 3 ? std::max(y, 0) : 0;
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

Engine::Engine(const Problem& p, Transport* tr, const ProcEnv& env) : p_(p), tr_(tr), env_(env) {
  // process grid (array order; default: slabs along the slowest axis) and ghost width
  cd_ = make_cart(p, env.rank, env.size, &fused_);
  cart_ = !cd_.is_slab();
  slab_ = cd_.axis(0);
  for (int a = 0; a < p.dims; ++a) alloc_[a] = cd_.axis(a).alloc();
  elem_ = p.dtype == ADVDIFF_F64 ? 8 : 4;
  const int per = 256 / (int)elem_;
  const int ax = alloc_[p.dims - 1];
  int px = 0, py = 0;
  pitch_pads(p, env.size, (int)elem_, &px, &py);
  const int sx = (ax + per - 1) / per * per + px;  // 256-B row pitch (+ the pitch pad)
  sy_ = sx;
  if (p.dims == 3) {
    sz_ = (int64_t)(alloc_[1] + py) * sx;
    plane_bytes_ = (size_t)sz_ * elem_;
  } else {
    sz_ = sx;
    plane_bytes_ = (size_t)sx * elem_;
  }
  field_bytes_ = plane_bytes_ * (size_t)alloc_[0];
  int lo_pri = 0, hi_pri = 0;
  HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
  HIP_CHECK(hipStreamCreateWithPriority(&compute_, hipStreamNonBlocking, lo_pri));
  HIP_CHECK(hipStreamCreateWithPriority(&comm_, hipStreamNonBlocking, hi_pri));
  HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&halo_done_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&cready_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&bdone_, hipEventDisableTiming));
  ls_ = compute_;
  // Field setup, timed like the reference's barrier-fenced HtD copy of the initial
  // subdomain (MultiGPU/Diffusion3d_Baseline/main.c:137-148): here the IC is generated
  // on the device, so this is the allocation + IC kernel + stage-buffer copies.
  HIP_CHECK(hipDeviceSynchronize());
  tr_->barrier();
  const double ts = now_s();
  // fields: u and its ping-pong partner A; B only where a step uses a third buffer (the
  // per-stage SSP-RK3 output, or the LSRK du) — the fused heat step ping-pongs u <-> A, so
  // its largest grid per GPU is what utils/sizing.py promises (2 fields, like solver.py)
  HIP_CHECK(hipMalloc(&u_, field_bytes_));
  HIP_CHECK(hipMalloc(&A_, field_bytes_));
  if (!fused_) HIP_CHECK(hipMalloc(&B_, field_bytes_));
  // Stream-ordered fill of the whole allocation (row padding included) BEFORE the IC.  A
  // synchronous hipMemset on the null stream is NOT ordered before work on the
  // non-blocking compute stream: it can land after the IC kernel and zero part of it
  // (bench/native/ipc_probe.hip: 20 of 20 trials, profiles/probe_memset_ipc_r3.log) —
  // the cause of the intermittent 8-rank 2x2x2 Cartesian mismatch of round 2.
  const int fill = poison_enabled() ? 0xFF : 0;
  HIP_CHECK(hipMemsetAsync(u_, fill, field_bytes_, compute_));
  // initial condition on the device, ghosts included (they equal the neighbours' cells)
  int off[3] = {0, 0, 0};
  for (int a = 0; a < p.dims; ++a) {
    const Slab s = cd_.axis(a);
    off[a] = s.start() - s.ghost;
  }
  if (!cart_ && p.dims == 3)
    KERNEL_CHECK(advdiff_init_ic(p.dtype, p.ic, u_, p.nx, p.ny, slab_.alloc(), sy_, sz_, off[0],
                                 p.nx, p.ny, p.nz, p.dx(), p.dy(), p.dz(), p.ic_p0, p.ic_p1,
                                 compute_));
  else if (!cart_)
    KERNEL_CHECK(advdiff_init_ic(p.dtype, p.ic, u_, p.nx, slab_.alloc(), 1, sy_, sz_, off[0], p.nx,
                                 p.ny, 1, p.dx(), p.dy(), 0.0, p.ic_p0, p.ic_p1, compute_));
  else if (p.dims == 3)
    KERNEL_CHECK(advdiff_init_ic_box(p.dtype, p.ic, u_, alloc_[2], alloc_[1], alloc_[0], sy_, sz_,
                                     off[2], off[1], off[0], p.nx, p.ny, p.nz, p.dx(), p.dy(),
                                     p.dz(), p.ic_p0, p.ic_p1, compute_));
  else
    KERNEL_CHECK(advdiff_init_ic_box(p.dtype, p.ic, u_, alloc_[1], alloc_[0], 1, sy_, sz_, off[1],
                                     off[0], 0, p.nx, p.ny, 1, p.dx(), p.dy(), 0.0, p.ic_p0,
                                     p.ic_p1, compute_));
  // A (and B) start as copies of u, padding included: cells a step never writes (frozen
  // boundary cells, unwritten ghost edges) carry the IC in every buffer
  HIP_CHECK(hipMemcpyAsync(A_, u_, field_bytes_, hipMemcpyDeviceToDevice, compute_));
  if (B_ && p.integrator == 1)
    HIP_CHECK(hipMemsetAsync(B_, 0, field_bytes_, compute_));  // du
  else if (B_)
    HIP_CHECK(hipMemcpyAsync(B_, u_, field_bytes_, hipMemcpyDeviceToDevice, compute_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  tr_->barrier();
  init_s_ = tr_->allreduce_max(now_s() - ts);
  full_ = slab_.compute_range(p.border());
  slab_.split(p.border(), slab_.ghost, interior_, blo_, bhi_);
  full_box_ = cd_.compute_box(p.border());
  cd_.split_boxes(p.border(), cd_.ghost, interior_box_, boundary_boxes_);
  if (cart_) plan_ = halo_plan(cd_, fused_);
  const int zoff = slab_.start() - slab_.ghost;
  zact_ = {std::max(0, p.border() - zoff), std::min(slab_.alloc(), slab_.n - p.border() - zoff)};
  t_ = p.t0;
  // hipGraph stepping: on by default where every exchange is stream-ordered device work
  const char* ge = std::getenv("ADVDIFF_GRAPH");
  const int want = ge ? std::atoi(ge) : p.graph;
  graph_ = want < 0 ? tr_->graph_safe() : want != 0;
  if (const char* f = std::getenv("ADVDIFF_FAULT")) {  // "RANK:STEP"
    if (std::sscanf(f, "%d:%d", &fault_rank_, &fault_step_) != 2) fault_rank_ = fault_step_ = -1;
  }
  if (const char* s2 = std::getenv("ADVDIFF_STEP2")) step2_env_ = std::atoi(s2) != 0;
  {
    int bc = p.bcomm;
    if (bc < 0) {  // default: on for ipc (profiles/r5/overlap.md) and rccl (stream-ordered
                   // ncclSend/Recv on comm_, the same two-stream order), off for socket
      const char* v = std::getenv("ADVDIFF_BCOMM");
      bc = v ? std::atoi(v) : std::string(tr_->name()) != "socket";
    }
    // the exchange must be stream-ordered device work on comm_ (a host-staged transport
    // blocks the host on comm_ inside start_halo: keep its boundary on compute_)
    bcomm_ = bc != 0 && env.size > 1 && p.overlap && std::string(tr_->name()) != "socket";
  }
  {
    // fused halo puts (solver.py _step_fused_put / _stage_put): ipc slabs, the 3-D fused
    // heat step or the fp64 WENO5 SSP-RK3 stage; every rank must address the peer planes
    // with its own row pitch and plane stride, so those must agree across the ranks
    int fp = p.fused_put;
    if (fp < 0) {
      const char* v = std::getenv("ADVDIFF_FUSED_PUT");
      fp = v ? std::atoi(v) : 0;
    }
    const bool stage_ok = p_.physics == Physics::Burgers && p_.dims == 3 &&
                          (p_.weno == 0 || p_.weno == 1) && p_.dtype == ADVDIFF_F64 &&
                          p_.integrator == 0;
    fput_ = fp != 0 && env.size > 1 && !cart_ && p_.dims == 3 &&
            std::string(tr_->name()) == "ipc" && (fused_ || stage_ok);
    if (fput_) {
      const double z1 = tr_->allreduce_max((double)sz_), z0 = -tr_->allreduce_max(-(double)sz_);
      const double y1 = tr_->allreduce_max((double)sy_), y0 = -tr_->allreduce_max(-(double)sy_);
      fput_ = z1 == z0 && y1 == y0;
      if (fput_) bcomm_ = false;  // no boundary launch left to move
    }
  }
  if (sync_debug_enabled() || p.check_every > 0 || fault_rank_ >= 0)
    graph_ = false;  // per-launch / per-step host checks
  if (graph_ && std::string(tr_->name()) == "socket")
    throw std::runtime_error("--graph: the socket transport synchronises the host inside a step");
  if (env.size > 1) wd_ = std::make_unique<Watchdog>(tr_, env.rank, Watchdog::timeout_from_env());
  // one FD2 step or two per launch: measured for this shape (kernels.h
  // advdiff_diffusion3d_step2_pick; ADVDIFF_STEP2=0/1 forces), before any capture
  if (step2_env_ && fused_ && env_.size == 1 && !cart_ && p_.dims == 3 && p_.order == 2 &&
      p_.physics == Physics::Diffusion) {
    const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
    const int B = p_.border();
    const int box[8] = {B, p_.nx - B, B, p_.ny - B, 0, p_.nx, 0, p_.ny};
    int use2 = 1;
    HIP_CHECK((hipError_t)advdiff_diffusion3d_step2_pick(
        p_.dtype, u_, A_, p_.nx, p_.ny, sy_, sz_, slab_.alloc(), full_.lo, full_.hi, zact_.lo,
        zact_.hi, box, p_.K / (dx * dx), p_.K / (dy * dy), p_.K / (dz * dz), stable_dt(),
        compute_, &use2));
    HIP_CHECK(hipStreamSynchronize(compute_));
    step2_env_ = use2 != 0;
  }
  // banded or uniform z chunks for the fused 3-D heat launch that carries most planes (one
  // rank, or slabs with fused puts: the full range; slabs: the interior launch): measured,
  // cached in the kernel library (kernels.h advdiff_diffusion3d_step_sched_pick), before
  // any capture
  if (fused_ && !cart_ && p_.dims == 3 && p_.physics == Physics::Diffusion) {
    const Range r = env_.size == 1 || fput_ ? full_ : interior_;
    if (!r.empty()) {
      const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
      const int B = p_.border();
      const int box[8] = {B, p_.nx - B, B, p_.ny - B, 0, p_.nx, 0, p_.ny};
      int banded = 0;
      HIP_CHECK((hipError_t)advdiff_diffusion3d_step_sched_pick(
          p_.dtype, u_, A_, p_.nx, p_.ny, sy_, sz_, slab_.alloc(), r.lo, r.hi, zact_.lo,
          zact_.hi, box, p_.order, p_.K / (dx * dx), p_.K / (dy * dy), p_.K / (dz * dz),
          stable_dt(), compute_, &banded));
      HIP_CHECK(hipStreamSynchronize(compute_));
    }
  }
}

Engine::~Engine() {
  wd_.reset();
  (void)hipStreamSynchronize(compute_);
  (void)hipStreamSynchronize(comm_);
  for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
  (void)hipEventDestroy(ready_);
  (void)hipEventDestroy(halo_done_);
  (void)hipEventDestroy(cready_);
  (void)hipEventDestroy(bdone_);
  (void)hipStreamDestroy(compute_);
  (void)hipStreamDestroy(comm_);
  (void)hipFree(u_);
  (void)hipFree(A_);
  (void)hipFree(B_);
  (void)hipFree(red_ws_);
  (void)hipFree(red_);
}

double Engine::stable_dt() const {
  // same operation order as models/*.stable_dt so Python and C++ runs are bitwise equal
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  auto coef_sum = [&](double c) {
    double s = c / (dx * dx) + c / (dy * dy);
    if (p_.dims == 3) s += c / (dz * dz);
    return s;
  };
  if (p_.physics == Physics::Diffusion) return p_.safety / (2.0 * coef_sum(p_.K));
  double h = std::min(dx, dy);
  if (p_.dims == 3) h = std::min(h, dz);
  double dt = p_.cfl * h / 1.0;  // reference: max|u| assumed 1 (main.cpp:130-133)
  if (p_.C > 0) dt = std::min(dt, 0.9 / (2.0 * coef_sum(p_.C)));
  return dt;
}

void Engine::launch(const void* in, void* aux, void* out, Range r, double dt, double a,
                    double b, bool ls) {
  launch_view(in, aux, out, p_.nx, p_.ny, r, p_.border(), dt, a, b, ls);
}

void Engine::launch_view(const void* in, void* aux, void* out, int nx, int ny, Range r, int B,
                         double dt, double a, double b, bool ls) {
  if (r.empty()) return;
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  if (p_.physics == Physics::Diffusion) {
    const double cx = p_.K / (dx * dx), cy = p_.K / (dy * dy), cz = p_.K / (dz * dz);
    if (p_.dims == 3) {
      if (ls)
        KERNEL_CHECK(advdiff_diffusion3d_stage_ls(p_.dtype, in, aux, out, nx, ny, sy_, sz_,
                                                  r.lo, r.hi, B, p_.order, cx, cy, cz, dt, a, b,
                                                  ls_));
      else
        KERNEL_CHECK(advdiff_diffusion3d_stage(p_.dtype, in, aux, out, nx, ny, sy_, sz_,
                                               r.lo, r.hi, B, p_.order, cx, cy, cz, dt, a, b,
                                               ls_));
    } else {
      if (ls)
        KERNEL_CHECK(advdiff_diffusion2d_stage_ls(p_.dtype, in, aux, out, nx, sy_, r.lo, r.hi,
                                                  B, p_.order, cx, cy, dt, a, b, ls_));
      else
        KERNEL_CHECK(advdiff_diffusion2d_stage(p_.dtype, in, aux, out, nx, sy_, r.lo, r.hi, B,
                                               p_.order, cx, cy, dt, a, b, ls_));
    }
  } else {
    const double vx = p_.C / (dx * dx), vy = p_.C / (dy * dy), vz = p_.C / (dz * dz);
    if (p_.dims == 3) {
      if (ls)
        KERNEL_CHECK(advdiff_burgers3d_stage_ls(p_.dtype, in, aux, out, nx, ny, sy_, sz_,
                                                r.lo, r.hi, B, p_.weno, 1.0 / dx, 1.0 / dy,
                                                1.0 / dz, vx, vy, vz, dt, a, b, ls_));
      else
        KERNEL_CHECK(advdiff_burgers3d_stage(p_.dtype, in, aux, out, nx, ny, sy_, sz_, r.lo,
                                             r.hi, B, p_.weno, 1.0 / dx, 1.0 / dy, 1.0 / dz, vx,
                                             vy, vz, dt, a, b, ls_));
    } else {
      if (ls)
        KERNEL_CHECK(advdiff_burgers2d_stage_ls(p_.dtype, in, aux, out, nx, sy_, r.lo, r.hi, B,
                                                p_.weno, 1.0 / dx, 1.0 / dy, vx, vy, dt, a, b,
                                                ls_));
      else
        KERNEL_CHECK(advdiff_burgers2d_stage(p_.dtype, in, aux, out, nx, sy_, r.lo, r.hi, B,
                                             p_.weno, 1.0 / dx, 1.0 / dy, vx, vy, dt, a, b,
                                             ls_));
    }
  }
}

void Engine::launch_fused(Range r, double dt, Range r2, bool exclusive) {
  if (r.empty() && r2.empty()) return;
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  if (p_.dims == 2) {
    for (const Range& q : {r, r2})
      if (!q.empty())
        KERNEL_CHECK(advdiff_diffusion2d_step(p_.dtype, u_, A_, p_.nx, sy_, slab_.alloc(), q.lo,
                                              q.hi, zact_.lo, zact_.hi, p_.border(), p_.order,
                                              p_.K / (dx * dx), p_.K / (dy * dy), dt,
                                              ls_));
    return;
  }
  const int B = p_.border();
  const int box[8] = {B, p_.nx - B, B, p_.ny - B, 0, p_.nx, 0, p_.ny};
  KERNEL_CHECK(advdiff_diffusion3d_step_box_ex(
      p_.dtype, u_, A_, p_.nx, p_.ny, sy_, sz_, slab_.alloc(), r.lo, r.hi, r2.lo, r2.hi,
      zact_.lo, zact_.hi, box, p_.order, p_.K / (dx * dx), p_.K / (dy * dy), p_.K / (dz * dz),
      dt, exclusive ? ADVDIFF_EXCLUSIVE : 0, ls_));
}

void Engine::put_targets(void* f, void** dlo, void** dhi) {
  const int G = slab_.ghost, c = slab_.count();
  if (!tr_->halo_targets(plane(f, G), plane(f, 0), plane(f, G + c - G), plane(f, G + c),
                         (size_t)G * plane_bytes_, slab_.lower(), slab_.upper(), dlo, dhi))
    throw std::runtime_error("fused halo puts: the transport has no peer addresses");
}

// the exchange of a field whose send planes the producing launch already stored into the
// peers: signal + wait on comm_, after the launch (start_halo without the puts)
void Engine::signal_halo(void* f) {
  const int G = slab_.ghost, c = slab_.count();
  HIP_CHECK(hipEventRecord(ready_, compute_));
  HIP_CHECK(hipStreamWaitEvent(comm_, ready_, 0));
  tr_->halo_signal(plane(f, G), plane(f, 0), plane(f, G + c - G), plane(f, G + c),
                   (size_t)G * plane_bytes_, slab_.lower(), slab_.upper(), comm_);
  HIP_CHECK(hipEventRecord(halo_done_, comm_));
  halo_pending_ = true;
}

void Engine::step_fused(double dt) {
  if (cart_) {
    step_fused_cart(dt);
    return;
  }
  if (fput_) {  // one launch; its boundary planes go straight into the neighbours' ghosts
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    void *dlo = nullptr, *dhi = nullptr;
    put_targets(A_, &dlo, &dhi);
    const int G = slab_.ghost, c = slab_.count();
    const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
    KERNEL_CHECK(advdiff_diffusion3d_step_put(
        p_.dtype, u_, A_, p_.nx, p_.ny, sy_, sz_, slab_.alloc(), full_.lo, full_.hi, zact_.lo,
        zact_.hi, p_.border(), p_.order, p_.K / (dx * dx), p_.K / (dy * dy), p_.K / (dz * dz),
        dt, dlo, G, 2 * G, dhi, c, c + G, compute_));
    halo_pending_ = false;
    std::swap(u_, A_);
    signal_halo(u_);
    return;
  }
  if (env_.size == 1) {
    launch_fused(full_, dt, Range{}, true);
  } else if (p_.overlap && bcomm_) {
    bcomm_begin();
    launch_fused(interior_, dt);  // compute_, beside the whole exchange
    ls_ = comm_;                  // after the halo of u in stream order
    launch_fused(blo_, dt, bhi_);
    bcomm_end();
    halo_pending_ = false;
    std::swap(u_, A_);
    start_halo(u_, true);
    return;
  } else if (p_.overlap) {
    launch_fused(interior_, dt);  // overlaps the RCCL exchange: grid schedule
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    launch_fused(blo_, dt, bhi_);  // both boundary slabs in one launch
  } else {
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    launch_fused(full_, dt, Range{}, true);
  }
  halo_pending_ = false;
  std::swap(u_, A_);
  start_halo(u_);
}

bool Engine::step2_ok() const {
  return step2_env_ && fused_ && env_.size == 1 && !cart_ && p_.dims == 3 && p_.order == 2 &&
         p_.physics == Physics::Diffusion;
}

void Engine::step2(double dt) {
  if (!step2_ok()) {
    step(dt);
    step(dt);
    return;
  }
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  const int B = p_.border();
  const int box[8] = {B, p_.nx - B, B, p_.ny - B, 0, p_.nx, 0, p_.ny};
  KERNEL_CHECK(advdiff_diffusion3d_step2x(p_.dtype, u_, A_, p_.nx, p_.ny, sy_, sz_,
                                          slab_.alloc(), full_.lo, full_.hi, zact_.lo,
                                          zact_.hi, box, p_.K / (dx * dx), p_.K / (dy * dy),
                                          p_.K / (dz * dz), dt, compute_));
  std::swap(u_, A_);
  for (int q = 0; q < 2; ++q) {  // the same additions as two steps
    t_ += dt;
    ++it_;
  }
}

// Boundary launch on the comm stream (bcomm_): before it, comm_ joins compute_ (the
// previous interior launch read / wrote what the boundary launch overwrites); after it,
// compute_ joins comm_ at bdone_ — recorded BEFORE the puts and the wait for the peers, so
// a spinning device wait never holds a compute launch.  Every cross-stream wait forks from
// or joins into compute_ (a hipGraph capture's origin): no event is waited on by the
// stream that recorded it (profiles/r5/diag_bstream.md).
void Engine::bcomm_begin() {
  HIP_CHECK(hipEventRecord(cready_, compute_));
  HIP_CHECK(hipStreamWaitEvent(comm_, cready_, 0));
}

void Engine::bcomm_end() {
  ls_ = compute_;
  HIP_CHECK(hipEventRecord(bdone_, comm_));
  HIP_CHECK(hipStreamWaitEvent(compute_, bdone_, 0));
}

void Engine::start_halo(void* field, bool on_comm) {
  if (env_.size == 1) return;
  const int G = slab_.ghost, c = slab_.count();
  if (!on_comm) {  // on_comm: the producer ran on comm_ (stream order)
    HIP_CHECK(hipEventRecord(ready_, compute_));
    HIP_CHECK(hipStreamWaitEvent(comm_, ready_, 0));
  }
  tr_->halo(plane(field, G), plane(field, 0), plane(field, G + c - G), plane(field, G + c),
            (size_t)G * plane_bytes_, slab_.lower(), slab_.upper(), comm_);
  HIP_CHECK(hipEventRecord(halo_done_, comm_));
  halo_pending_ = true;
}

void Engine::stage(void* in, void* aux, void* out, double a, double b, double dt, bool ls) {
  if (cart_) {
    stage_cart(in, aux, out, a, b, dt, ls);
    return;
  }
  if (env_.size == 1) {
    launch(in, aux, out, full_, dt, a, b, ls);
    return;
  }
  if (fput_ && !ls) {  // the fp64 WENO5 stage with its halo puts inside (_stage_put)
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    void *dlo = nullptr, *dhi = nullptr;
    put_targets(out, &dlo, &dhi);
    const int G = slab_.ghost, c = slab_.count();
    const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
    KERNEL_CHECK(advdiff_burgers3d_stage_put(
        p_.dtype, in, aux, out, p_.nx, p_.ny, sy_, sz_, full_.lo, full_.hi, p_.border(),
        p_.weno, 1.0 / dx, 1.0 / dy, 1.0 / dz, p_.C / (dx * dx), p_.C / (dy * dy),
        p_.C / (dz * dz), dt, a, b, nullptr, dlo, G, 2 * G, dhi, c, c + G, compute_));
    halo_pending_ = false;
    signal_halo(out);
    return;
  }
  if (p_.overlap) {
    if (bcomm_) bcomm_begin();
    launch(in, aux, out, interior_, dt, a, b, ls);
    if (bcomm_)
      ls_ = comm_;  // after the halo of `in` in stream order
    else if (halo_pending_)
      HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    if (p_.physics == Physics::Burgers && p_.dims == 3) {  // both boundary slabs, one launch
      const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
      KERNEL_CHECK(advdiff_burgers3d_stage2_dt(
          p_.dtype, in, aux, out, p_.nx, p_.ny, sy_, sz_, blo_.lo, blo_.hi, bhi_.lo, bhi_.hi,
          p_.border(), p_.weno, 1.0 / dx, 1.0 / dy, 1.0 / dz, p_.C / (dx * dx),
          p_.C / (dy * dy), p_.C / (dz * dz), dt, a, b, ls ? 1 : 0, nullptr, ls_));
    } else {
      launch(in, aux, out, blo_, dt, a, b, ls);
      launch(in, aux, out, bhi_, dt, a, b, ls);
    }
    if (bcomm_) {
      bcomm_end();
      halo_pending_ = false;
      start_halo(out, true);
      return;
    }
  } else {
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    launch(in, aux, out, full_, dt, a, b, ls);
  }
  halo_pending_ = false;
  start_halo(out);
}

// Carpenter–Kennedy LSRK4(5) (Matlab_Prototipes/InviscidBurgersNd/LFWENO7FDM1d.m)
static const double kLsA[5] = {0.0, -567301805773.0 / 1357537059087.0,
                               -2404267990393.0 / 2016746695238.0,
                               -3550918686646.0 / 2091501179385.0,
                               -1275806237668.0 / 842570457699.0};
static const double kLsB[5] = {1432997174477.0 / 9575080441755.0,
                               5161836677717.0 / 13612068292357.0,
                               1720146321549.0 / 2090206949498.0,
                               3134564353537.0 / 4481467310338.0,
                               2277821191437.0 / 14882151754819.0};

void Engine::step(double dt) {
  if (fused_) {
    step_fused(dt);
  } else if (p_.integrator == 1) {
    for (int s = 0; s < 5; ++s) {
      stage(u_, B_, A_, kLsA[s], kLsB[s], dt, true);
      std::swap(u_, A_);
    }
  } else {
    stage(u_, nullptr, A_, 0.0, 1.0, dt);
    stage(A_, u_, B_, 0.75, 0.25, dt);
    stage(B_, u_, u_, 1.0 / 3.0, 2.0 / 3.0, dt);
  }
  t_ += dt;
  ++it_;
}

// Capture kGraphSteps steps of `dt` from the current state (u_ parity) into an executable
// graph.  The comm stream joins the capture through the ready_ event of the first halo
// start; the last exchange is joined back into compute_ before the capture ends, so a
// replay leaves no exchange pending.  Capturing runs no work: the host state the steps
// advance (t_, it_, buffer roles) is restored afterwards.
hipGraphExec_t Engine::graph_for(double dt) {
  const GraphKey key{dt, u_};
  auto it = graphs_.find(key);
  if (it != graphs_.end()) return it->second;
  const double t = t_;
  const int itn = it_;
  void *u = u_, *a = A_, *b = B_;
  HIP_CHECK(hipStreamBeginCapture(compute_, hipStreamCaptureModeThreadLocal));
  for (int q = 0; q < kGraphSteps;) {
    if (step2_ok()) {
      step2(dt);
      q += 2;
    } else {
      step(dt);
      ++q;
    }
  }
  if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
  halo_pending_ = false;
  hipGraph_t g = nullptr;
  HIP_CHECK(hipStreamEndCapture(compute_, &g));
  hipGraphExec_t ex = nullptr;
  HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(g));
  if (u_ != u || A_ != a || B_ != b)
    throw std::runtime_error("graph capture: buffer roles did not return to their start");
  t_ = t;
  it_ = itn;
  graphs_.emplace(key, ex);
  return ex;
}

void Engine::prepare_graphs(double dt) {
  if (!graph_) return;
  if (warm_ < 2) {
    // Dry exchanges of every buffer a step may exchange (fused / LSRK ping-pong u <-> A,
    // SSP-RK3 stage outputs A, B, u): the same message patterns the steps will use, with
    // no device work — the transport's one-time handshakes (ipc) and its staging buffers
    // (strided Cartesian boxes, any transport) are settled here, outside the capture.
    const bool pending = halo_pending_;
    tr_->set_dry(true);
    for (void* f : {u_, A_, B_}) {
      if (f == nullptr) continue;
      if (cart_)
        start_halo_cart(f);
      else
        start_halo(f);
    }
    tr_->set_dry(false);
    halo_pending_ = pending;  // halo_done_ now marks a later point of comm_: still covers it
  }
  warm_ = 2;
  if (halo_pending_) {
    HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    halo_pending_ = false;
  }
  (void)graph_for(dt);
}

void Engine::steps(int n, double dt) {
  // pairs of steps in one launch where nothing runs between steps (per-step host checks
  // and fault injection keep single steps)
  const bool pairs = step2_ok() && fault_rank_ < 0 && p_.check_every <= 0;
  if (!graph_) {
    for (; pairs && n >= 2; n -= 2) {
      step2(dt);
      beat();
    }
    for (int q = 0; q < n; ++q) {
      step(dt);
      beat();
      watchdog();
    }
    return;
  }
  // eager steps first: the transport's one-time handshakes (host communication) must not
  // fall inside a capture, and the u/A ping-pong visits both parities in two steps
  for (; warm_ < 2 && n > 0; ++warm_, --n) {
    step(dt);
    beat();
  }
  if (n >= kGraphSteps && halo_pending_) {  // an event recorded outside a capture cannot
    HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));  // be waited on inside it
    halo_pending_ = false;
  }
  for (; n >= kGraphSteps; n -= kGraphSteps) {
    HIP_CHECK(hipGraphLaunch(graph_for(dt), compute_));
    beat();
    for (int q = 0; q < kGraphSteps; ++q) {  // the same additions as kGraphSteps eager steps
      t_ += dt;
      ++it_;
    }
  }
  for (; pairs && n >= 2; n -= 2) {
    step2(dt);
    beat();
  }
  for (; n > 0; --n) {
    step(dt);
    beat();
  }
}

Stats Engine::run_iters(int iters) {
  const double dt = stable_dt();
  if (iters >= kGraphSteps) prepare_graphs(dt);
  HIP_CHECK(hipDeviceSynchronize());
  tr_->barrier();
  Armed armed(wd_.get());
  const double t0 = now_s();
  steps(iters, dt);
  HIP_CHECK(hipStreamSynchronize(compute_));
  HIP_CHECK(hipStreamSynchronize(comm_));
  tr_->barrier();
  Stats s;
  s.seconds = tr_->allreduce_max(now_s() - t0);
  s.steps = iters;
  s.t = t_;
  s.htod = init_s_;
  check_transport();
  return s;
}

void Engine::warmup(int n) {
  if (n <= 0) return;
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  void* const roles[3] = {u_, A_, B_};
  void* saved[3] = {nullptr, nullptr, nullptr};
  for (int q = 0; q < 3; ++q) {
    if (roles[q] == nullptr) continue;
    HIP_CHECK(hipMalloc(&saved[q], field_bytes_));
    HIP_CHECK(hipMemcpyAsync(saved[q], roles[q], field_bytes_, hipMemcpyDeviceToDevice, compute_));
  }
  const double t = t_;
  const int it = it_;
  const double dt = stable_dt();
  if (n >= kGraphSteps) prepare_graphs(dt);
  {
    Armed armed(wd_.get());
    steps(n, dt);
    HIP_CHECK(hipStreamSynchronize(compute_));
  }
  if (halo_pending_) {
    HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    halo_pending_ = false;
  }
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  tr_->barrier();  // no peer still puts into a ghost box being restored
  u_ = roles[0];
  A_ = roles[1];
  B_ = roles[2];
  for (int q = 0; q < 3; ++q) {
    if (roles[q] == nullptr) continue;
    HIP_CHECK(hipMemcpyAsync(roles[q], saved[q], field_bytes_, hipMemcpyDeviceToDevice, compute_));
  }
  HIP_CHECK(hipStreamSynchronize(compute_));
  for (void* b : saved)
    if (b) HIP_CHECK(hipFree(b));
  t_ = t;
  it_ = it;
  tr_->barrier();
}

Stats Engine::run_until(double t_end) {
  const double dt0 = stable_dt();
  prepare_graphs(dt0);
  HIP_CHECK(hipDeviceSynchronize());
  tr_->barrier();
  Armed armed(wd_.get());
  const double t0 = now_s();
  // the steps of the full dt0 (graph-replayable), counted with the loop's own arithmetic
  int n = 0;
  {
    double t = t_;
    while (t < t_end * (1 - 1e-14) && !(t + dt0 > t_end)) {
      t += dt0;
      ++n;
    }
  }
  steps(n, dt0);
  while (t_ < t_end * (1 - 1e-14)) {
    double dt = dt0;
    if (t_ + dt > t_end) dt = t_end - t_;
    step(dt);
    beat();
    watchdog();
    ++n;
  }
  HIP_CHECK(hipStreamSynchronize(compute_));
  HIP_CHECK(hipStreamSynchronize(comm_));
  tr_->barrier();
  Stats s;
  s.seconds = tr_->allreduce_max(now_s() - t0);
  s.steps = n;
  s.t = t_;
  s.htod = init_s_;
  check_transport();
  return s;
}

bool sync_debug_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("ADVDIFF_SYNC_DEBUG");
    return v != nullptr && *v != '\0' && std::string(v) != "0";
  }();
  return on;
}

double Engine::check_finite() {
  if (red_ws_ == nullptr) {
    HIP_CHECK(hipMalloc(&red_ws_, advdiff_reduce_workspace_bytes()));
    HIP_CHECK(hipMalloc((void**)&red_, 3 * sizeof(double)));
  }
  int lo[3], g0[3], n[3];
  own_box(lo, g0, n);
  const int64_t pz = p_.dims == 3 ? sz_ : sz_ * alloc_[0];
  KERNEL_CHECK(advdiff_reduce_norms(p_.dtype, u_, nullptr, sy_, pz, lo[2], lo[2] + n[2], lo[1],
                                    lo[1] + n[1], lo[0], lo[0] + n[0], red_ws_, red_, compute_));
  double h[3] = {0, 0, 0};
  HIP_CHECK(hipMemcpyAsync(h, red_, sizeof h, hipMemcpyDeviceToHost, compute_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  // a NaN can hide from a max (fmax drops it) but not from the sum; agree on a flag, since
  // NaN comparisons inside a MAX allreduce are not reliable either
  const bool bad = !std::isfinite(h[0]) || !std::isfinite(h[2]);
  if (tr_->allreduce_max(bad ? 1.0 : 0.0) > 0.0) {
    char msg[128];
    std::snprintf(msg, sizeof msg, "non-finite solution at step %d, t=%g", it_, t_);
    throw std::runtime_error(msg);
  }
  return tr_->allreduce_max(h[2]);
}

void Engine::error_norms(double& l1, double& l2, double& linf) {
  if (cart_) {
    error_norms_cart(l1, l2, linf);
    return;
  }
  const int G = slab_.ghost, c = slab_.count();
  void* ex = nullptr;
  HIP_CHECK(hipMalloc(&ex, plane_bytes_ * c));
  const double scale = exact_scale();
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  const double p0 = p_.ic == 3 ? p_.K : p_.ic_p0, p1 = p_.ic == 3 ? t_ : p_.ic_p1;
  if (p_.dims == 3)
    KERNEL_CHECK(advdiff_init_ic(p_.dtype, p_.ic, ex, p_.nx, p_.ny, c, sy_, sz_, slab_.start(),
                                 p_.nx, p_.ny, p_.nz, dx, dy, dz, p0, p1, compute_));
  else
    KERNEL_CHECK(advdiff_init_ic(p_.dtype, p_.ic, ex, p_.nx, c, 1, sy_, sz_, slab_.start(), p_.nx,
                                 p_.ny, 1, dx, dy, 0.0, p0, p1, compute_));
  KERNEL_CHECK(advdiff_scale(p_.dtype, ex, (int64_t)(plane_bytes_ / elem_) * c, scale, compute_));
  void* ws = nullptr;
  double* res = nullptr;
  HIP_CHECK(hipMalloc(&ws, advdiff_reduce_workspace_bytes()));
  HIP_CHECK(hipMalloc(&res, 3 * sizeof(double)));
  if (p_.dims == 3)
    KERNEL_CHECK(advdiff_reduce_norms(p_.dtype, plane(u_, G), ex, sy_, sz_, 0, p_.nx, 0, p_.ny,
                                      0, c, ws, res, compute_));
  else
    KERNEL_CHECK(advdiff_reduce_norms(p_.dtype, plane(u_, G), ex, sy_, sz_ * c, 0, p_.nx, 0, c,
                                      0, 1, ws, res, compute_));
  double h[3];
  HIP_CHECK(hipMemcpyAsync(h, res, sizeof(h), hipMemcpyDeviceToHost, compute_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  (void)hipFree(ws);
  (void)hipFree(res);
  (void)hipFree(ex);
  const double vol = dx * dy * (p_.dims == 3 ? dz : 1.0);
  l1 = vol * tr_->allreduce_sum(h[0]);
  l2 = std::sqrt(vol * tr_->allreduce_sum(h[1]));
  linf = tr_->allreduce_max(h[2]);
}

double Engine::exact_scale() const {
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  if (p_.ic == 2) {  // sine: separable decay
    const double Lx = (p_.nx - 1) * dx, Ly = (p_.ny - 1) * dy;
    double lam = 1.0 / (Lx * Lx) + 1.0 / (Ly * Ly);
    if (p_.dims == 3) lam += 1.0 / std::pow((p_.nz - 1) * dz, 2);
    return std::exp(-p_.K * M_PI * M_PI * lam * t_);
  }
  if (p_.ic == 3) return std::pow(p_.ic_p1 / t_, p_.dims / 2.0);  // heat kernel from t0
  return 1.0;
}

template <typename V>
std::vector<V> Engine::gather_as() {
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  if (cart_) return gather_cart<V>();
  const int G = slab_.ghost, c = slab_.count();
  std::vector<char> raw(plane_bytes_ * c);
  HIP_CHECK(hipMemcpy(raw.data(), plane(u_, G), raw.size(), hipMemcpyDeviceToHost));
  const int rows = p_.dims == 3 ? c * p_.ny : c;
  std::vector<char> packed((size_t)rows * p_.nx * sizeof(V));
  V* dst = (V*)packed.data();
  for (int r = 0; r < rows; ++r)
    for (int i = 0; i < p_.nx; ++i) {
      const size_t src = row_offset(r) + i;
      dst[(size_t)r * p_.nx + i] = elem_ == 8 ? (V)((const double*)raw.data())[src]
                                              : (V)((const float*)raw.data())[src];
    }
  std::vector<char> all = tr_->gather(packed);
  std::vector<V> out(all.size() / sizeof(V));
  if (!all.empty()) std::memcpy(out.data(), all.data(), all.size());
  return out;
}
template std::vector<float> Engine::gather_as<float>();
template std::vector<double> Engine::gather_as<double>();

// every rank's planes with their ghost planes (slabs), concatenated in rank order
void Engine::dtoh_local() {
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  int lo[3], g0[3], n[3];
  own_box(lo, g0, n);
  // 3-D: planes of n[1] rows of n[2] cells; 2-D (axis 0 a unit axis): one plane of rows
  const size_t row = (size_t)n[2] * elem_;
  const size_t plane = row * n[1];
  const int per = (int)std::max<size_t>(1, ((size_t)64 << 20) / std::max<size_t>(plane, 1));
  void* host = nullptr;
  HIP_CHECK(hipHostMalloc(&host, plane * std::min(per, n[0])));
  const int64_t pz = p_.dims == 3 ? sz_ : sz_ * alloc_[0];
  for (int k0 = 0; k0 < n[0]; k0 += per) {
    const int nk = std::min(per, n[0] - k0);
    for (int k = 0; k < nk; ++k) {
      const char* src = (const char*)u_ +
                        ((int64_t)(lo[0] + k0 + k) * pz + (int64_t)lo[1] * sy_ + lo[2]) * elem_;
      HIP_CHECK(hipMemcpy2DAsync((char*)host + (size_t)k * plane, row, src, (size_t)sy_ * elem_,
                                 row, n[1], hipMemcpyDeviceToHost, compute_));
    }
    HIP_CHECK(hipStreamSynchronize(compute_));
  }
  HIP_CHECK(hipHostFree(host));
}

std::vector<float> Engine::gather_float32_ghosts() {
  HIP_CHECK(hipStreamSynchronize(comm_));
  HIP_CHECK(hipStreamSynchronize(compute_));
  if (cart_) throw std::runtime_error("--write-ghosts: slab decompositions only");
  std::vector<char> raw(field_bytes_);
  HIP_CHECK(hipMemcpy(raw.data(), u_, raw.size(), hipMemcpyDeviceToHost));
  const int rows = p_.dims == 3 ? slab_.alloc() * p_.ny : slab_.alloc();
  std::vector<char> packed((size_t)rows * p_.nx * sizeof(float));
  float* dst = (float*)packed.data();
  for (int r = 0; r < rows; ++r)
    for (int i = 0; i < p_.nx; ++i) {
      const size_t src = row_offset(r) + i;
      dst[(size_t)r * p_.nx + i] = elem_ == 8 ? (float)((const double*)raw.data())[src]
                                              : ((const float*)raw.data())[src];
    }
  std::vector<char> all = tr_->gather(packed);
  std::vector<float> out(all.size() / sizeof(float));
  if (!all.empty()) std::memcpy(out.data(), all.data(), all.size());
  return out;
}

void Engine::check_transport() {
  const long long e = tr_->allreduce_max((double)tr_->errors());
  if (e > 0) {
    std::fprintf(stderr, "transport %s: %lld halo wait timeout(s): a peer stopped\n", tr_->name(), e);
    std::exit(5);
  }
}

static std::string fmt(const char* f, double v) {
  char b[128];
  std::snprintf(b, sizeof(b), f, v);
  return b;
}

std::string summary_multigpu(const std::string& title, const std::string& opt, const Stats& s,
                             const Problem& p, int nprocs) {
  const std::string sep(67, '=');
  const double gflops = s.seconds > 0 ? 3.0 * s.steps * p.cells() * 1e-9 * 8.0 / s.seconds : 0;
  const double mlups = s.seconds > 0 ? p.cells() * (double)s.steps / s.seconds / 1e6 : 0;
  std::ostringstream o;
  o << "=======================" << title << "=====================\n";
  o << "Optimization                                 :  " << opt << "\n";
  o << "Kernel time ex. data transfers               :  " << fmt("%lf", s.seconds) << " seconds\n";
  o << "Data transfer(s) HtD                         :  " << fmt("%lf", s.htod) << " seconds\n";
  o << "Data transfer(s) DtH                         :  " << fmt("%lf", s.dtoh) << " seconds\n";
  o << sep << "\n";
  o << "Total effective GFLOPs                       :  " << fmt("%lf", gflops) << "\n";
  o << sep << "\n";
  if (p.dims == 3)
    o << "3D Grid Size                                 :  " << p.nx << " x " << p.ny << " x "
      << p.nz << "\n";
  else
    o << "2D Grid Size                                 :  " << p.nx << " x " << p.ny << "\n";
  o << "Iterations                                   :  " << s.steps << " x 3 RK steps\n";
  o << sep << "\n";
  o << "MLUPS (cells x RK3 steps / s)                :  " << fmt("%.1f", mlups) << "\n";
  o << "Stage-MLUPS                                  :  " << fmt("%.1f", 3 * mlups) << "\n";
  o << "Processes / devices                          :  " << nprocs << " x gfx950\n";
  o << sep << "\n";
  return o.str();
}

// The single-GPU apps' block (SingleGPU/*/tools.cpp PrintSummary; the labels and layout of
// utils/metrics.py summary_singlegpu): GFLOPs without the x3 for diffusion (quirk of the
// reference's SG heat apps), with it for Burgers.
std::string summary_singlegpu(const std::string& title, const std::string& opt, const Stats& s,
                              const Problem& p, const std::vector<std::pair<std::string, std::string>>& extra) {
  const std::string sep(67, '=');
  const double k = p.physics == Physics::Burgers ? 3.0 : 1.0;
  const double gflops = s.seconds > 0 ? k * s.steps * p.cells() * 1e-9 * 8.0 / s.seconds : 0;
  std::ostringstream o;
  o << "=========================== " << title << " =======================\n";
  o << "Optimization                                 :  " << opt << "\n";
  o << "Kernel time ex. data transfers               :  " << fmt("%f", s.seconds) << " seconds\n";
  o << sep << "\n";
  o << "Total effective GFLOPs                       :  " << fmt("%f", gflops) << "\n";
  o << sep << "\n";
  if (p.dims == 3)
    o << "3D Grid Size                                 :  " << p.nx << " x " << p.ny << " x "
      << p.nz << " \n";
  else
    o << "2D Grid Size                                 :  " << p.nx << " x " << p.ny << " \n";
  o << "Iterations                                   :  " << s.steps << "\n";
  o << "Final Time                                   :  " << fmt("%g", s.t) << "\n";
  o << sep << "\n";
  for (const auto& kv : extra) {
    std::string key = kv.first;
    if (key.size() < 45) key.resize(45, ' ');
    o << key << ":  " << kv.second << "\n";
  }
  if (!extra.empty()) o << sep << "\n";
  return o.str();
}

void write_binary(const std::string& path, const std::vector<float>& data) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::perror(path.c_str());
    return;
  }
  std::fwrite(data.data(), sizeof(float), data.size(), f);
  std::fclose(f);
}

}  // namespace advdiff::rt
