// Cartesian block decomposition of the native runtime (mirror of
// multigpu_advectiondiffusion_amd/parallel/decomposition.py CartesianDecomposition and
// parallel/halo.py CartesianHalo, and of the Cartesian branches of solver.py):
//   * a block per rank over a 2-D/3-D process grid, ghosts on axis 0 and on split axes;
//   * stage kernels launched on VIEWS widened by R (border R), the fused heat step on
//     views with explicit active / output bounds — exactly the Python solver's launch
//     geometry, so native and Python Cartesian runs are bitwise equal (and equal to the
//     1-rank run: the kernels are decomposition-invariant);
//   * halo exchange: per-stage models send face blocks only (one phase); the fused step
//     needs edge/corner ghosts, exchanged axis by axis, fastest first, each phase carrying
//     the ghosts of the axes before it; strided faces are packed / unpacked with
//     advdiff_copy_box on the comm stream around one grouped transport call per phase.
// The reference has no counterpart (its only split is z-slabs).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <sstream>

#include "runtime.hpp"

namespace advdiff::rt {

void Cart::coords_of(int r, int* c) const {
  for (int a = dims - 1; a >= 0; --a) {
    c[a] = r % pgrid[a];
    r /= pgrid[a];
  }
}

int Cart::rank_of(const int* c) const {
  int r = 0;
  for (int a = 0; a < dims; ++a) r = r * pgrid[a] + c[a];
  return r;
}

Slab Cart::axis(int a, int r) const {
  int c[3] = {0, 0, 0};
  coords_of(r < 0 ? rank : r, c);
  Slab s;
  s.n = shape[a];
  s.size = pgrid[a];
  s.rank = c[a];
  s.ghost = ghost_of_axis(a);
  return s;
}

int Cart::neighbor(int a, int side) const {
  int c[3] = {0, 0, 0};
  coords_of(rank, c);
  c[a] += side;
  if (c[a] < 0 || c[a] >= pgrid[a]) return -1;
  return rank_of(c);
}

Box Cart::compute_box(int border) const {
  Box b;
  for (int a = 0; a < dims; ++a) b.r[a] = axis(a).compute_range(border);
  return b;
}

void Cart::split_boxes(int border, int width, Box& interior, std::vector<Box>& boundary) const {
  Range full[3], inner[3], lo[3], hi[3];
  for (int a = 0; a < dims; ++a) {
    const Slab s = axis(a);
    full[a] = s.compute_range(border);
    s.split(border, width, inner[a], lo[a], hi[a]);
  }
  boundary.clear();
  for (int a = 0; a < dims; ++a)
    for (const Range& rg : {lo[a], hi[a]}) {
      Box b;
      for (int q = 0; q < dims; ++q) b.r[q] = q < a ? inner[q] : (q == a ? rg : full[q]);
      if (!b.empty(dims)) boundary.push_back(b);
    }
  for (int a = 0; a < dims; ++a) interior.r[a] = inner[a];
}

void parse_pgrid(const std::string& spec, int dims, int world, int* pgrid) {
  std::vector<int> v;
  std::stringstream ss(spec);
  std::string tok;
  while (std::getline(ss, tok, 'x')) v.push_back(std::stoi(tok));
  int prod = 1;
  for (int x : v) prod *= x;
  if ((int)v.size() != dims || prod != world)
    throw std::runtime_error("--decomp " + spec + " does not match a " + std::to_string(dims) +
                             "-D grid of " + std::to_string(world) + " ranks");
  for (int a = 0; a < 3; ++a) pgrid[a] = a < dims ? v[a] : 1;
}

// ------------------------------------------------------------------------------------
// Host-only geometry (shared by the Engine and the geometry dump)
// ------------------------------------------------------------------------------------
Cart make_cart(const Problem& p, int rank, int size, bool* fused) {
  const int R = p.radius();
  Cart cd;
  cd.dims = p.dims;
  cd.rank = rank;
  if (p.dims == 3) {
    cd.shape[0] = p.nz;
    cd.shape[1] = p.ny;
    cd.shape[2] = p.nx;
  } else {
    cd.shape[0] = p.ny;
    cd.shape[1] = p.nx;
  }
  if (p.pgrid[0] > 0) {
    for (int a = 0; a < 3; ++a) cd.pgrid[a] = a < p.dims ? p.pgrid[a] : 1;
  } else {
    cd.pgrid[0] = size;
  }
  if (cd.size() != size) throw std::runtime_error("process grid does not match WORLD_SIZE");
  // fused: blocks at least 3R thick on every split axis (else per-stage, solver.py)
  bool thick = true;
  for (int a = 0; a < p.dims; ++a)
    if (cd.pgrid[a] > 1 && cd.shape[a] / cd.pgrid[a] < 3 * R) thick = false;
  const bool f = p.fused && p.physics == Physics::Diffusion && p.integrator == 0 && thick;
  cd.ghost = f ? 3 * R : R;
  for (int a = 0; a < p.dims; ++a)
    if (cd.shape[a] < cd.pgrid[a] * std::max(cd.ghost_of_axis(a), 1))
      throw std::runtime_error("block thinner than the ghost width: use fewer ranks");
  if (fused) *fused = f;
  return cd;
}

void fused_view(const Cart& cd, int radius, int border, int a, int lo, int hi, Range& view,
                Range& act, Range& outr) {
  const int R3 = 3 * radius;
  const Slab ax = cd.axis(a);
  view = {std::max(0, lo - R3), std::min(ax.alloc(), hi + R3)};
  const int origin = ax.start() - ax.ghost + view.lo;
  const int N = cd.shape[a];
  act = {std::max(0, border - origin), std::min(view.hi - view.lo, N - border - origin)};
  outr = {lo - view.lo, hi - view.lo};
}

bool halo_direct_default() {
  const char* v = std::getenv("ADVDIFF_CORNERS");
  return !(v && std::string(v) == "phased");
}

static void check_distinct(const std::vector<HaloPlanMsg>& ph) {
  for (size_t i = 0; i < ph.size(); ++i)  // distinct peers per phase (one message each)
    for (size_t j = i + 1; j < ph.size(); ++j)
      if (ph[i].peer == ph[j].peer)
        throw std::runtime_error("halo phase with two messages to one peer");
}

std::vector<std::vector<HaloPlanMsg>> halo_plan(const Cart& cd, bool corners, bool direct) {
  const int dims = cd.dims, G = cd.ghost;
  std::vector<int> split;
  for (int a = dims - 1; a >= 0; --a)
    if (cd.pgrid[a] > 1) split.push_back(a);
  std::vector<std::vector<HaloPlanMsg>> out;
  if (split.empty()) return out;
  Range own[3], alloc[3];
  for (int a = 0; a < dims; ++a) {
    const Slab s = cd.axis(a);
    own[a] = {s.ghost, s.ghost + s.count()};
    alloc[a] = {0, s.alloc()};
  }
  if (corners && direct) {
    // every offset d in {-1,0,1}^dims \ {0} (0 on unsplit axes), last axis fastest
    int c[3] = {0, 0, 0};
    cd.coords_of(cd.rank, c);
    std::vector<HaloPlanMsg> ph;
    int lim[3];
    for (int a = 0; a < 3; ++a) lim[a] = (a < dims && cd.pgrid[a] > 1) ? 1 : 0;
    for (int d0 = -lim[0]; d0 <= lim[0]; ++d0)
      for (int d1 = -lim[1]; d1 <= lim[1]; ++d1)
        for (int d2 = -lim[2]; d2 <= lim[2]; ++d2) {
          const int d[3] = {d0, d1, d2};
          if (!d0 && !d1 && !d2) continue;
          int nc[3] = {0, 0, 0};
          bool inside = true;
          for (int a = 0; a < dims; ++a) {
            nc[a] = c[a] + d[a];
            if (nc[a] < 0 || nc[a] >= cd.pgrid[a]) inside = false;
          }
          if (!inside) continue;
          HaloPlanMsg m;
          m.peer = cd.rank_of(nc);
          for (int a = 0; a < dims; ++a) {
            m.off[a] = d[a];
            if (d[a] < 0) {
              m.send.r[a] = {own[a].lo, own[a].lo + G};
              m.recv.r[a] = {0, G};
            } else if (d[a] > 0) {
              m.send.r[a] = {own[a].hi - G, own[a].hi};
              m.recv.r[a] = {own[a].hi, own[a].hi + G};
            } else {
              m.send.r[a] = m.recv.r[a] = own[a];
            }
          }
          ph.push_back(m);
        }
    check_distinct(ph);
    out.push_back(ph);
    return out;
  }
  std::vector<std::vector<int>> phases;
  if (corners)
    for (int a : split) phases.push_back({a});
  else
    phases.push_back(split);
  for (const auto& axes : phases) {
    std::vector<HaloPlanMsg> ph;
    for (int a : axes)
      for (int side : {-1, 1}) {
        const int peer = cd.neighbor(a, side);
        if (peer < 0) continue;
        HaloPlanMsg m;
        m.peer = peer;
        m.off[a] = side;
        for (int q = 0; q < dims; ++q) {
          const bool carried = corners && q > a;  // exchanged in an earlier phase
          m.send.r[q] = m.recv.r[q] = carried ? alloc[q] : own[q];
        }
        m.send.r[a] = side < 0 ? Range{own[a].lo, own[a].lo + G} : Range{own[a].hi - G, own[a].hi};
        m.recv.r[a] = side < 0 ? Range{0, G} : Range{own[a].hi, own[a].hi + G};
        ph.push_back(m);
      }
    check_distinct(ph);
    out.push_back(ph);
  }
  return out;
}

static std::string jrange(const Range& r) {
  return "[" + std::to_string(r.lo) + "," + std::to_string(r.hi) + "]";
}
static std::string jbox(const Box& b, int dims) {
  std::string s = "[";
  for (int a = 0; a < dims; ++a) s += (a ? "," : "") + jrange(b.r[a]);
  return s + "]";
}

std::string geometry_json(const Problem& p, int rank, int size) {
  bool fused = false;
  Cart cd = make_cart(p, rank, size, &fused);
  const int dims = p.dims, R = p.radius(), B = p.border();
  Box full = cd.compute_box(B), interior;
  std::vector<Box> bnd;
  cd.split_boxes(B, cd.ghost, interior, bnd);
  std::ostringstream o;
  int c[3] = {0, 0, 0};
  cd.coords_of(rank, c);
  o << "{\"rank\":" << rank << ",\"coords\":[";
  for (int a = 0; a < dims; ++a) o << (a ? "," : "") << c[a];
  o << "],\"ghost\":" << cd.ghost << ",\"fused\":" << (fused ? "true" : "false") << ",\"alloc\":[";
  for (int a = 0; a < dims; ++a) o << (a ? "," : "") << cd.axis(a).alloc();
  o << "],\"own\":[";
  for (int a = 0; a < dims; ++a) {
    const Slab s = cd.axis(a);
    o << (a ? "," : "") << jrange(Range{s.ghost, s.ghost + s.count()});
  }
  o << "],\"full\":" << jbox(full, dims) << ",\"interior\":" << jbox(interior, dims)
    << ",\"boundary\":[";
  for (size_t q = 0; q < bnd.size(); ++q) o << (q ? "," : "") << jbox(bnd[q], dims);
  o << "],\"views\":[";
  if (fused) {  // fused launches: (box, per x/y axis: view, active, output)
    std::vector<Box> boxes{full, interior};
    boxes.insert(boxes.end(), bnd.begin(), bnd.end());
    bool first = true;
    for (const Box& bx : boxes) {
      if (bx.empty(dims)) continue;
      o << (first ? "" : ",") << "{\"box\":" << jbox(bx, dims) << ",\"axes\":[";
      first = false;
      for (int a = 1; a < dims; ++a) {
        Range v, act, outr;
        fused_view(cd, R, B, a, bx.r[a].lo, bx.r[a].hi, v, act, outr);
        o << (a > 1 ? "," : "") << "[" << jrange(v) << "," << jrange(act) << "," << jrange(outr)
          << "]";
      }
      o << "]}";
    }
  }
  o << "],\"halo\":[";
  const auto plan = halo_plan(cd, fused);
  for (size_t ph = 0; ph < plan.size(); ++ph) {
    o << (ph ? "," : "") << "[";
    for (size_t q = 0; q < plan[ph].size(); ++q) {
      const HaloPlanMsg& m = plan[ph][q];
      o << (q ? "," : "") << "{\"peer\":" << m.peer << ",\"off\":[";
      for (int a = 0; a < dims; ++a) o << (a ? "," : "") << m.off[a];
      o << "],\"send\":" << jbox(m.send, dims)
        << ",\"recv\":" << jbox(m.recv, dims) << "}";
    }
    o << "]";
  }
  o << "]}";
  return o.str();
}

// ------------------------------------------------------------------------------------
// Engine: Cartesian launches and exchange
// ------------------------------------------------------------------------------------
void Engine::launch_box(void* in, void* aux, void* out, const Box& bx, double dt, double a,
                        double b, bool ls) {
  if (bx.empty(p_.dims)) return;
  const int R = p_.radius();
  if (p_.dims == 3) {
    const Range& y = bx.r[1];
    const Range& x = bx.r[2];
    auto v = [&](void* f) -> void* { return f ? at(f, 0, y.lo - R, x.lo - R) : nullptr; };
    launch_view(v(in), v(aux), v(out), x.hi - x.lo + 2 * R, y.hi - y.lo + 2 * R, bx.r[0], R, dt,
                a, b, ls);
  } else {
    const Range& x = bx.r[1];
    auto v = [&](void* f) -> void* { return f ? at(f, 0, 0, x.lo - R) : nullptr; };
    launch_view(v(in), v(aux), v(out), x.hi - x.lo + 2 * R, 0, bx.r[0], R, dt, a, b, ls);
  }
}

void Engine::fused_view(int a, int lo, int hi, Range& view, Range& act, Range& outr) const {
  rt::fused_view(cd_, p_.radius(), p_.border(), a, lo, hi, view, act, outr);
}

void Engine::launch_fused_box(const Box& bx, double dt, bool exclusive) {
  if (bx.empty(p_.dims)) return;
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  if (p_.dims == 3) {
    Range vy, ya, yo, vx, xa, xo;
    fused_view(1, bx.r[1].lo, bx.r[1].hi, vy, ya, yo);
    fused_view(2, bx.r[2].lo, bx.r[2].hi, vx, xa, xo);
    const int box[8] = {xa.lo, xa.hi, ya.lo, ya.hi, xo.lo, xo.hi, yo.lo, yo.hi};
    KERNEL_CHECK(advdiff_diffusion3d_step_box_ex(
        p_.dtype, at(u_, 0, vy.lo, vx.lo), at(A_, 0, vy.lo, vx.lo), vx.hi - vx.lo, vy.hi - vy.lo,
        sy_, sz_, alloc_[0], bx.r[0].lo, bx.r[0].hi, 0, 0, zact_.lo, zact_.hi, box, p_.order,
        p_.K / (dx * dx), p_.K / (dy * dy), p_.K / (dz * dz), dt,
        exclusive ? ADVDIFF_EXCLUSIVE : 0, ls_));
  } else {
    Range vx, xa, xo;
    fused_view(1, bx.r[1].lo, bx.r[1].hi, vx, xa, xo);
    const int box[4] = {xa.lo, xa.hi, xo.lo, xo.hi};
    KERNEL_CHECK(advdiff_diffusion2d_step_box(
        p_.dtype, at(u_, 0, 0, vx.lo), at(A_, 0, 0, vx.lo), vx.hi - vx.lo, sy_, alloc_[0],
        bx.r[0].lo, bx.r[0].hi, zact_.lo, zact_.hi, box, p_.order, p_.K / (dx * dx),
        p_.K / (dy * dy), dt, ls_));
  }
}

void Engine::stage_cart(void* in, void* aux, void* out, double a, double b, double dt, bool ls) {
  if (p_.overlap && bcomm_) {  // boundary boxes on the comm stream (engine.cpp bcomm_begin)
    bcomm_begin();
    launch_box(in, aux, out, interior_box_, dt, a, b, ls);
    ls_ = comm_;
    for (const Box& bx : boundary_boxes_) launch_box(in, aux, out, bx, dt, a, b, ls);
    bcomm_end();
    halo_pending_ = false;
    start_halo_cart(out, true);
    return;
  }
  if (p_.overlap) {
    launch_box(in, aux, out, interior_box_, dt, a, b, ls);
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    for (const Box& bx : boundary_boxes_) launch_box(in, aux, out, bx, dt, a, b, ls);
  } else {
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    launch_box(in, aux, out, full_box_, dt, a, b, ls);
  }
  halo_pending_ = false;
  start_halo_cart(out);
}

void Engine::step_fused_cart(double dt) {
  if (p_.overlap && bcomm_) {
    bcomm_begin();
    launch_fused_box(interior_box_, dt, false);
    ls_ = comm_;
    for (const Box& bx : boundary_boxes_) launch_fused_box(bx, dt, false);
    bcomm_end();
    halo_pending_ = false;
    std::swap(u_, A_);
    start_halo_cart(u_, true);
    return;
  }
  if (p_.overlap) {
    launch_fused_box(interior_box_, dt, false);
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    for (const Box& bx : boundary_boxes_) launch_fused_box(bx, dt, false);
  } else {
    if (halo_pending_) HIP_CHECK(hipStreamWaitEvent(compute_, halo_done_, 0));
    launch_fused_box(full_box_, dt, true);
  }
  halo_pending_ = false;
  std::swap(u_, A_);
  start_halo_cart(u_);
}

void Engine::start_halo_cart(void* field, bool on_comm) {
  if (!on_comm) {  // on_comm: the producer ran on comm_ (stream order)
    HIP_CHECK(hipEventRecord(ready_, compute_));
    HIP_CHECK(hipStreamWaitEvent(comm_, ready_, 0));
  }
  const int dims = p_.dims;
  auto origin = [&](const Box& b) {
    return dims == 3 ? at(field, b.r[0].lo, b.r[1].lo, b.r[2].lo)
                     : at(field, 0, b.r[0].lo, b.r[1].lo);
  };
  // phases are stream-ordered on comm_: a phase's sends carry the ghosts that the phases
  // before it received
  for (const auto& phase : plan_) {
    std::vector<BoxMsg> msgs;
    for (const HaloPlanMsg& m : phase) {
      BoxMsg b;
      b.peer = m.peer;
      b.dtype = p_.dtype;
      b.send = origin(m.send);
      b.recv = origin(m.recv);
      b.ssy = b.rsy = sy_;
      b.ssz = b.rsz = dims == 3 ? sz_ : 0;
      // extents as (ni, nj, nk) = (x, y, z); 2-D: one "plane" of rows
      b.nk = dims == 3 ? m.send.r[0].hi - m.send.r[0].lo : 1;
      b.nj = m.send.r[dims - 2].hi - m.send.r[dims - 2].lo;
      b.ni = m.send.r[dims - 1].hi - m.send.r[dims - 1].lo;
      msgs.push_back(b);
    }
    tr_->exchange_boxes(msgs, comm_);
  }
  HIP_CHECK(hipEventRecord(halo_done_, comm_));
  halo_pending_ = true;
}

// exact solution on the whole local block (same layout as u), reduced over the owned box
void Engine::error_norms_cart(double& l1, double& l2, double& linf) {
  void* ex = nullptr;
  HIP_CHECK(hipMalloc(&ex, field_bytes_));
  const double dx = p_.dx(), dy = p_.dy(), dz = p_.dz();
  const double p0 = p_.ic == 3 ? p_.K : p_.ic_p0, p1 = p_.ic == 3 ? t_ : p_.ic_p1;
  int off[3] = {0, 0, 0};
  Range own[3];
  for (int a = 0; a < p_.dims; ++a) {
    const Slab s = cd_.axis(a);
    off[a] = s.start() - s.ghost;
    own[a] = {s.ghost, s.ghost + s.count()};
  }
  if (p_.dims == 3)
    KERNEL_CHECK(advdiff_init_ic_box(p_.dtype, p_.ic, ex, alloc_[2], alloc_[1], alloc_[0], sy_,
                                     sz_, off[2], off[1], off[0], p_.nx, p_.ny, p_.nz, dx, dy, dz,
                                     p0, p1, compute_));
  else
    KERNEL_CHECK(advdiff_init_ic_box(p_.dtype, p_.ic, ex, alloc_[1], alloc_[0], 1, sy_, sz_,
                                     off[1], off[0], 0, p_.nx, p_.ny, 1, dx, dy, 0.0, p0, p1,
                                     compute_));
  KERNEL_CHECK(advdiff_scale(p_.dtype, ex, (int64_t)(field_bytes_ / elem_), exact_scale(),
                             compute_));
  void* ws = nullptr;
  double* res = nullptr;
  HIP_CHECK(hipMalloc(&ws, advdiff_reduce_workspace_bytes()));
  HIP_CHECK(hipMalloc(&res, 3 * sizeof(double)));
  if (p_.dims == 3)
    KERNEL_CHECK(advdiff_reduce_norms(p_.dtype, u_, ex, sy_, sz_, own[2].lo, own[2].hi, own[1].lo,
                                      own[1].hi, own[0].lo, own[0].hi, ws, res, compute_));
  else
    KERNEL_CHECK(advdiff_reduce_norms(p_.dtype, u_, ex, sy_, sz_ * alloc_[0], own[1].lo, own[1].hi,
                                      own[0].lo, own[0].hi, 0, 1, ws, res, compute_));
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

// owned block of every rank as float32 [z][y][x], assembled on rank 0
template <typename V>
std::vector<V> Engine::gather_cart() {
  const int dims = p_.dims;
  std::vector<char> raw(field_bytes_);
  HIP_CHECK(hipMemcpy(raw.data(), u_, raw.size(), hipMemcpyDeviceToHost));
  Range own[3] = {{0, 1}, {0, 1}, {0, 1}};
  for (int a = 0; a < dims; ++a) {
    const Slab s = cd_.axis(a);
    own[a] = {s.ghost, s.ghost + s.count()};
  }
  const Range z = dims == 3 ? own[0] : Range{0, 1};
  const Range y = own[dims - 2], x = own[dims - 1];
  std::vector<char> packed((size_t)(z.hi - z.lo) * (y.hi - y.lo) * (x.hi - x.lo) * sizeof(V));
  V* dst = (V*)packed.data();
  size_t q = 0;
  for (int k = z.lo; k < z.hi; ++k)
    for (int j = y.lo; j < y.hi; ++j)
      for (int i = x.lo; i < x.hi; ++i) {
        const size_t src = (size_t)k * (dims == 3 ? sz_ : 0) + (size_t)j * sy_ + i;
        dst[q++] = elem_ == 8 ? (V)((const double*)raw.data())[src]
                              : (V)((const float*)raw.data())[src];
      }
  std::vector<char> all = tr_->gather(packed);
  if (all.empty()) return {};
  const int NZ = dims == 3 ? cd_.shape[0] : 1, NY = cd_.shape[dims - 2], NX = cd_.shape[dims - 1];
  std::vector<V> out((size_t)NZ * NY * NX);
  const V* src = (const V*)all.data();
  for (int r = 0; r < cd_.size(); ++r) {
    int st[3] = {0, 0, 0}, ct[3] = {1, 1, 1};
    for (int a = 0; a < dims; ++a) {
      const Slab s = cd_.axis(a, r);
      st[3 - dims + a] = s.start();
      ct[3 - dims + a] = s.count();
    }
    for (int k = 0; k < ct[0]; ++k)
      for (int j = 0; j < ct[1]; ++j) {
        V* row = out.data() + ((size_t)(st[0] + k) * NY + st[1] + j) * NX + st[2];
        std::copy(src, src + ct[2], row);
        src += ct[2];
      }
  }
  return out;
}
template std::vector<float> Engine::gather_cart<float>();
template std::vector<double> Engine::gather_cart<double>();

}  // namespace advdiff::rt
