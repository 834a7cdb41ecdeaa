// Native C++ runtime of the MI355X framework: process bootstrap, transports (RCCL over
// xGMI, or host-staged TCP for single-GPU multi-rank testing), slab decomposition and the
// SSP-RK3 engine that drives the libadvdiff kernels with halo/compute overlap.
//
// It is the native counterpart of the reference's L3/L4 layers
// (MultiGPU/Diffusion3d_Baseline/main.c, Tools.c, Util.cu): no MPI, no host-side global
// arrays, device-resident slabs, one grouped RCCL send/recv per stage on a high-priority
// comm stream.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "advdiff/kernels.h"

// sha256 prefix of the runtime + app sources the executable was built from
// (csrc/Makefile RT_HASH; tests compare it with the tree)
extern "C" const char* advdiff_runtime_hash(void);

#define HIP_CHECK(expr)                                                                    \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, \
                   __LINE__, #expr);                                                       \
      std::exit(2);                                                                        \
    }                                                                                      \
  } while (0)

// ADVDIFF_SYNC_DEBUG=1: synchronise the device after every launch and report the first
// failing one by its call site (the reference's CUDA_ERROR_CHECK,
// MultiGPU/Diffusion2d_Baseline/Kernels.cu:12,34-57; hipGraph stepping is off then)
#define KERNEL_CHECK(expr)                                                                \
  do {                                                                                    \
    int e_ = (expr);                                                                      \
    if (e_ == 0 && advdiff::rt::sync_debug_enabled()) {                                   \
      e_ = (int)hipDeviceSynchronize();                                                   \
      if (e_ == 0) e_ = (int)hipGetLastError();                                           \
    }                                                                                     \
    if (e_ != 0) {                                                                        \
      std::fprintf(stderr, "kernel launch failed (%d) at %s:%d: %s\n", e_, __FILE__,      \
                   __LINE__, #expr);                                                      \
      std::exit(2);                                                                       \
    }                                                                                     \
  } while (0)

namespace advdiff::rt {

bool sync_debug_enabled();  // ADVDIFF_SYNC_DEBUG (see KERNEL_CHECK)

// ------------------------------------------------------------------------------------
// Process environment (torchrun-compatible: RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*)
// ------------------------------------------------------------------------------------
struct ProcEnv {
  int rank = 0, size = 1, local_rank = 0;
  std::string master_addr = "127.0.0.1";
  int master_port = 29500;
  static ProcEnv from_env();
};

// ------------------------------------------------------------------------------------
// Transport: how ghost planes and scalars move between ranks.
// ------------------------------------------------------------------------------------
// One point-to-point message of an exchange: `bytes` from `send` to rank `peer`, and
// `bytes` from `peer` into `recv` (neighbour pairs exchange equal-sized blocks).
struct Msg {
  int peer = -1;
  const void* send = nullptr;
  void* recv = nullptr;
  size_t bytes = 0;
};

// A strided box message: the ni x nj x nk box of elements at `send` (pitches ssy, ssz,
// elements) goes to `peer`, and the peer's matching box arrives in the box at `recv`
// (pitches rsy, rsz).  Both boxes live in the caller's fields.
struct BoxMsg {
  int peer = -1;
  int dtype = ADVDIFF_F64;
  const void* send = nullptr;
  int64_t ssy = 0, ssz = 0;
  void* recv = nullptr;
  int64_t rsy = 0, rsz = 0;
  int ni = 0, nj = 0, nk = 0;
  size_t elem() const { return dtype == ADVDIFF_F64 ? 8 : 4; }
  size_t bytes() const { return (size_t)ni * nj * nk * elem(); }
  bool send_contiguous() const { return (nj == 1 || ssy == ni) && (nk == 1 || ssz == (int64_t)ni * nj); }
  bool recv_contiguous() const { return (nj == 1 || rsy == ni) && (nk == 1 || rsz == (int64_t)ni * nj); }
};

class Transport {
 public:
  virtual ~Transport();
  virtual const char* name() const = 0;
  // Enqueue a set of messages to distinct peers on `stream` (one grouped RCCL call).
  virtual void exchange(const std::vector<Msg>& msgs, hipStream_t stream) = 0;
  // Enqueue a set of box messages to distinct peers on `stream`.  Default: strided boxes
  // are packed into / unpacked from device staging buffers with advdiff_copy_box around
  // one exchange() (contiguous boxes go zero-copy); the IPC transport overrides it with
  // direct puts into the peer's field.
  virtual void exchange_boxes(const std::vector<BoxMsg>& msgs, hipStream_t stream);
  // Enqueue the exchange of G-plane slabs (bytes each) with the lower/upper neighbour
  // (-1 = none) on `stream`: send_lo -> lower's recv_hi, send_hi -> upper's recv_lo.
  virtual void halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
                    size_t bytes, int lower, int upper, hipStream_t stream) = 0;
  // Fused halo puts (ipc): the peer address of the receive slab matching each send slab
  // of halo() — the same handshake and cache — so a step kernel can store the send planes
  // itself (dst_lo / dst_hi: nullptr where there is no neighbour); halo_signal() then
  // enqueues only the signal + wait of that halo.  false: the transport cannot.
  virtual bool halo_targets(const void* /*send_lo*/, void* /*recv_lo*/, const void* /*send_hi*/,
                            void* /*recv_hi*/, size_t /*bytes*/, int /*lower*/, int /*upper*/,
                            void** /*dst_lo*/, void** /*dst_hi*/) {
    return false;
  }
  virtual void halo_signal(const void* /*send_lo*/, void* /*recv_lo*/, const void* /*send_hi*/,
                           void* /*recv_hi*/, size_t /*bytes*/, int /*lower*/, int /*upper*/,
                           hipStream_t /*stream*/) {}
  virtual double allreduce_max(double v) = 0;
  virtual double allreduce_sum(double v) = 0;
  virtual void barrier() = 0;
  // Gather per-rank host byte blocks to rank 0 (returns the concatenation on rank 0).
  virtual std::vector<char> gather(const std::vector<char>& local) = 0;
  // Wait timeouts or other deferred transport errors seen so far (call at a sync point).
  virtual long long errors() { return 0; }
  // every exchange step is stream-ordered device work with no host synchronisation, so a
  // step can be captured into a hipGraph (local, ipc: yes; socket: host-staged, no; rccl:
  // capturable, but never run multi-rank on the 1-GPU test box -> opt-in with --graph)
  virtual bool graph_safe() const { return false; }
  // one-time host handshakes per message pattern (ipc)
  virtual bool needs_handshake() const { return false; }
  // Dry mode: an exchange runs only its host-side setup — the one-time handshakes (ipc)
  // and the sizing of device staging buffers (strided boxes) — and enqueues no device
  // work, so an engine settles both before it captures a graph (hipMalloc / hipFree /
  // stream syncs are not allowed inside a stream capture).
  virtual void set_dry(bool on) { dry_ = on; }
  // Watchdog hooks (SURVEY §5 failure detection): a deferred asynchronous error of the
  // transport (RCCL: ncclCommGetAsyncError), 0 if none; abort() tears the transport down
  // so blocked device work of a dead peer's exchange cannot hold the process (RCCL:
  // ncclCommAbort).  Both are called from the watchdog thread.
  virtual int poll_error() { return 0; }
  virtual void abort() {}

 protected:
  void* staging(size_t slot, size_t bytes, hipStream_t stream);  // device staging buffer
  bool dry_ = false;

 private:
  std::vector<void*> stage_;
  std::vector<size_t> stage_cap_;
};

// Comm watchdog (watchdog.cpp): while armed, ends the process (exit 6, after
// Transport::abort) when the transport reports an asynchronous error or the main thread
// has not beaten for `timeout_s` seconds.  on_fail replaces that action (tests).
class Watchdog {
 public:
  using FailFn = std::function<void(const std::string&)>;
  Watchdog(Transport* tr, int rank, double timeout_s, FailFn on_fail = nullptr,
           double poll_s = 0.1);
  ~Watchdog();
  Watchdog(const Watchdog&) = delete;
  Watchdog& operator=(const Watchdog&) = delete;
  void arm();
  void disarm();
  void beat();
  bool fired() const { return fired_; }
  static double timeout_from_env();  // ADVDIFF_COMM_TIMEOUT, default 600 s (<= 0: off)

 private:
  void loop();
  Transport* tr_;
  int rank_;
  double timeout_, poll_;
  FailFn on_fail_;
  std::atomic<double> last_{0.0};
  std::atomic<bool> armed_{false};
  std::atomic<bool> fired_{false};
  bool stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
};

// Debug: ADVDIFF_POISON=1 fills every device allocation of the runtime (fields incl. row
// padding and ghost shells, staging buffers) and the host staging buffers with 0xFF bytes
// (a NaN in fp32 and fp64) instead of zeros, so a read of a cell nobody wrote shows up.
bool poison_enabled();

// rank 0 <-> all TCP star used for bootstrap, scalars and gathers by every transport.
class Star;

std::unique_ptr<Transport> make_transport(const ProcEnv& env, const std::string& kind);

// ------------------------------------------------------------------------------------
// Slab decomposition along the slowest axis (mirror of parallel/decomposition.py).
// ------------------------------------------------------------------------------------
struct Range {
  int lo = 0, hi = 0;
  bool empty() const { return hi <= lo; }
};

struct Slab {
  int n = 0, size = 1, rank = 0, ghost = 0;
  int count_of(int r) const { return n / size + (r < n % size ? 1 : 0); }
  int start_of(int r) const { return r * (n / size) + std::min(r, n % size); }
  int count() const { return count_of(rank); }
  int start() const { return start_of(rank); }
  int alloc() const { return count() + 2 * ghost; }
  int lower() const { return rank > 0 ? rank - 1 : -1; }
  int upper() const { return rank < size - 1 ? rank + 1 : -1; }
  int to_local(int g) const { return g - start() + ghost; }
  Range compute_range(int border) const;
  void split(int border, int radius, Range& interior, Range& blo, Range& bhi) const;
};

// ------------------------------------------------------------------------------------
// Cartesian block decomposition (mirror of parallel/decomposition.py
// CartesianDecomposition): array axis order (z, y, x) in 3-D, (y, x) in 2-D; ranks are
// row-major over the process grid.  Axis 0 always carries G ghost layers, the other
// axes only when split.  pgrid = (P, 1, 1) is exactly the slab layout.
// ------------------------------------------------------------------------------------
struct Box {
  Range r[3];
  bool empty(int dims) const {
    for (int a = 0; a < dims; ++a)
      if (r[a].empty()) return true;
    return false;
  }
};

struct Cart {
  int dims = 3;
  int shape[3] = {1, 1, 1};  // global extents, array order
  int pgrid[3] = {1, 1, 1};
  int rank = 0, ghost = 0;
  int size() const { return pgrid[0] * pgrid[1] * (dims == 3 ? pgrid[2] : 1); }
  void coords_of(int r, int* c) const;
  int rank_of(const int* c) const;
  int ghost_of_axis(int a) const { return (a == 0 || pgrid[a] > 1) ? ghost : 0; }
  Slab axis(int a, int r = -1) const;
  int neighbor(int a, int side) const;  // -1 at the domain edge
  bool is_slab() const { return pgrid[1] == 1 && (dims == 2 || pgrid[2] == 1); }
  Box compute_box(int border) const;
  // interior (computable while the halo is in flight) + at most 2*dims boundary boxes
  void split_boxes(int border, int width, Box& interior, std::vector<Box>& boundary) const;
};

// "PZxPYxPX" / "PYxPX" -> pgrid (array order); throws on a mismatch with dims / world
void parse_pgrid(const std::string& spec, int dims, int world, int* pgrid);

// One message of a halo phase, in local (array-order) boxes of the block incl. ghosts;
// off = the peer's process-grid offset (array order).
struct HaloPlanMsg {
  int peer = -1;
  int off[3] = {0, 0, 0};
  Box send, recv;
};
// Halo phases of a Cartesian block (mirror of parallel/halo.py CartesianHalo): corners =
// false (per-stage star stencils): ONE phase with the faces of every split axis over the
// owned extent of the other axes.  corners = true (the fused step), direct (default,
// ADVDIFF_CORNERS != "phased"): ONE phase with a message to every neighbour offset in
// {-1,0,1}^dims (faces, edges and corners from the neighbours that own them — one xGMI
// hop each on a fully connected node); phased: one phase per split axis, fastest first,
// each message spanning the FULL allocated extent of the axes exchanged before it.
bool halo_direct_default();
std::vector<std::vector<HaloPlanMsg>> halo_plan(const Cart& cd, bool corners,
                                               bool direct = halo_direct_default());

// ------------------------------------------------------------------------------------
// Problem + engine
// ------------------------------------------------------------------------------------
enum class Physics { Diffusion, Burgers };

// ------------------------------------------------------------------------------------
// Checkpoint shards (checkpoint.cpp; the format of utils/io.py): host-only helpers
// ------------------------------------------------------------------------------------
struct ShardInfo {
  std::vector<int64_t> shape, box0, grid;  // shard box (array order), global grid (x first)
  std::string dtype;                       // "float64" (both writers) or "float32"
  double t = 0;
  long long it = 0;
  size_t offset = 0;  // byte offset of the payload
};
std::string shard_path(const std::string& prefix, int rank);  // PREFIX.rankNNNNN.ckpt
std::vector<std::string> list_shards(const std::string& prefix);
ShardInfo read_shard_info(const std::string& path);
// raw text of a top-level key of a JSON object (nested objects skipped)
bool json_top_value(const std::string& js, const std::string& key, std::string& raw);

struct Problem {
  Physics physics = Physics::Diffusion;
  int pgrid[3] = {0, 0, 0};        // process grid (array order); 0 = slab (P, 1, 1)
  int dims = 3;
  int nx = 0, ny = 0, nz = 1;     // global grid
  double L = 1, W = 1, H = 1;     // domain lengths
  int dtype = ADVDIFF_F64;
  // diffusion
  double K = 1.0;
  int order = 4;
  double safety = 0.9;
  // burgers
  double C = 1e-5;
  int weno = 1;                    // 0 WENO5-JS, 1 WENO5-Z, 2 WENO7-JS (kernels.h codes)
  double cfl = 0.3;
  // common
  int ic = 3;                      // kernels.h IC codes
  double ic_p0 = 1.0, ic_p1 = 0.1;
  double t0 = 0.0;
  bool overlap = true;
  // overlap: the boundary launch on the comm stream, between the wait for its input's
  // halo and the puts of its output (-1 = ADVDIFF_BCOMM, default on for the ipc transport;
  // --boundary-on-comm / --no-boundary-on-comm)
  int bcomm = -1;
  // fused halo puts (ipc slabs, 3-D fused heat step or fp64 WENO5 SSP-RK3 stages): the
  // step / stage launch stores its boundary planes into the neighbours' ghost planes
  // itself, then signal + wait (-1 = ADVDIFF_FUSED_PUT; --fused-put)
  int fused_put = -1;
  // pitched fields (solver.py pitch_default): extra elements per row after the 256-B
  // alignment and extra rows per 3-D plane, never read or written (-1 = ADVDIFF_PITCH,
  // else 4 fp64 / 16 fp32 elements and one row on 3-D fields past 128 MiB per rank;
  // --pitch PX,PY)
  int pitch_px = -1, pitch_py = -1;
  int integrator = 0;              // 0 SSP-RK3, 1 low-storage RK4(5)
  bool fused = true;               // 3-D heat + SSP-RK3: one launch per step (3R ghosts)
  int graph = -1;                  // hipGraph stepping: -1 auto (graph-safe transports), 0, 1
  int check_every = 0;             // NaN/Inf watchdog every N steps (0: off; eager stepping)
  // (ADVDIFF_FAULT="RANK:STEP" makes RANK throw after STEP, like the Python solver's fault
  // injection: the launcher must then stop every other rank; eager stepping)
  int radius() const {
    return physics == Physics::Diffusion ? order / 2 : (weno == 2 ? 4 : 3);
  }
  int border() const { return radius(); }
  double dx() const { return L / (nx - 1); }
  double dy() const { return W / (ny - 1); }
  double dz() const { return dims == 3 ? H / (nz - 1) : 0.0; }
  int n_decomposed() const { return dims == 3 ? nz : ny; }
  int64_t cells() const { return (int64_t)nx * ny * (dims == 3 ? nz : 1); }
};

// extra elements per row / rows per 3-D plane of this problem's device fields (engine.cpp)
void pitch_pads(const Problem& p, int world, int elem, int* px, int* py);

struct Stats {
  int steps = 0;
  double seconds = 0, htod = 0, dtoh = 0, t = 0;
};

// The block decomposition an Engine builds for a problem on `size` ranks (process grid,
// ghost width; fused = the one-launch-per-step heat path is used).  Host-only.
Cart make_cart(const Problem& p, int rank, int size, bool* fused);
// View window, active and output bounds (view coordinates) along array axis a of a fused
// launch on local cells [lo, hi) (solver.py _fused_view).  Host-only.
void fused_view(const Cart& cd, int radius, int border, int a, int lo, int hi, Range& view,
                Range& act, Range& outr);
// Every launch box, fused-step view and halo message of `rank` as one JSON object
// (geometry checks against the Python decomposition: tests/test_native_geometry.py).
std::string geometry_json(const Problem& p, int rank, int size);

class Engine {
 public:
  Engine(const Problem& p, Transport* tr, const ProcEnv& env);
  ~Engine();
  double stable_dt() const;
  void step(double dt);
  // two steps of dt in ONE launch where the step has it (single-rank 3-D FD2 heat:
  // advdiff_diffusion3d_step2x, bit-identical to two steps), else two steps
  void step2(double dt);
  bool step2_ok() const;
  // n steps of constant dt: through hipGraphs of kGraphSteps steps when enabled (after two
  // eager steps that run the transport's one-time handshakes for both buffer parities)
  void steps(int n, double dt);
  // settle the transport's handshakes (dry exchanges of every field) and capture the
  // graph of the current buffer parity, OUTSIDE the timed loop (captures run no work)
  void prepare_graphs(double dt);
  bool graphs() const { return graph_; }
  bool fused_puts() const { return fput_; }
  static constexpr int kGraphSteps = 8;  // even: the u/A ping-pong returns to its start
  Stats run_iters(int iters);
  // n untimed steps, then the state exactly as before them (fields, buffer roles, t, it):
  // clocks, code objects, graphs and transport handshakes are warm (cli.py --warmup)
  void warmup(int n);
  Stats run_until(double t_end);
  // Σ|u-e|, Σ(u-e)², max|u-e| over the owned slab vs the exact solution (sine/heat ICs)
  void error_norms(double& l1, double& l2, double& linf);
  // rank 0: global array (no ghosts), as float (result.bin) or double (--ascii, --print);
  // others empty
  std::vector<float> gather_float32() { return gather_as<float>(); }
  std::vector<double> gather_float64() { return gather_as<double>(); }
  template <typename V>
  std::vector<V> gather_as();
  // rank 0: every rank's planes INCLUDING its ghost planes, concatenated in rank order —
  // the reference's multi-GPU result.bin layout (each rank's Nx x Ny x (_Nz + 6) slab,
  // SaveBinary3D(h_u, Nx, Ny, NZ), MultiGPU/Diffusion3d_Baseline/main.c:341).  Slabs only.
  std::vector<float> gather_float32_ghosts();
  // per-rank device-to-host copy of the owned block through one reused pinned buffer of a
  // few planes (the reference's timed DtH without the rank-0 merge; host memory O(planes))
  void dtoh_local();
  // device bytes of the resident fields (u, A and, if a step uses it, B)
  size_t memory_bytes() const { return field_bytes_ * ((u_ ? 1 : 0) + (A_ ? 1 : 0) + (B_ ? 1 : 0)); }
  // fp64 shard of the owned cells (utils/io.py format; collective: returns when every
  // rank's shard is written) / restart from the shards of ANY layout (owned + in-domain
  // ghost cells, then the stage buffers as after the IC; sets t and it)
  void save_checkpoint(const std::string& prefix, const std::string& ic_name);
  void load_checkpoint(const std::string& prefix);
  // NaN/Inf watchdog: Σ|u| and max|u| of the owned cells on every rank; throws
  // "non-finite solution at step N" on every rank if any rank's are not finite
  double check_finite();
  double init_seconds() const { return init_s_; }  // barrier-fenced field setup (HtD line)
  double time() const { return t_; }
  int iteration() const { return it_; }
  const Slab& slab() const { return slab_; }
  bool fused() const { return fused_; }
  bool cartesian() const { return cart_; }
  const Cart& cart() const { return cd_; }

 private:
  void launch(const void* in, void* aux, void* out, Range r, double dt, double a, double b,
              bool ls);
  // stage kernel on a view of nx (x ny) cells with frozen border `border`, planes r
  void launch_view(const void* in, void* aux, void* out, int nx, int ny, Range r, int border,
                   double dt, double a, double b, bool ls);
  void stage(void* in, void* aux, void* out, double a, double b, double dt, bool ls = false);
  // exclusive: nothing runs beside the launch (single rank / full range after the halo
  // wait) -> persistent schedule of the 3-D step kernel (ADVDIFF_EXCLUSIVE)
  void launch_fused(Range r, double dt, Range r2 = Range{}, bool exclusive = false);
  void step_fused(double dt);
  void start_halo(void* field, bool on_comm = false);
  // fused halo puts: the peer planes of `field`'s send slabs / the signal + wait after
  void put_targets(void* field, void** dlo, void** dhi);
  void signal_halo(void* field);
  void* plane(void* base, int l) const { return (char*)base + (size_t)l * plane_bytes_; }
  // checkpoint views: array order padded to three axes (2-D: axis 0 is a unit axis whose
  // one "plane" is the whole field)
  void own_box(int lo[3], int g0[3], int n[3]) const;
  size_t plane_span() const { return p_.dims == 3 ? plane_bytes_ : field_bytes_; }
  void* plane3(void* base, int k) const { return p_.dims == 3 ? plane(base, k) : base; }
  // ---- Cartesian blocks (cart_): kernels on views, phased / face halo exchange ----
  void* at(void* base, int z, int y, int x) const {
    return (char*)base + ((size_t)z * sz_ + (size_t)y * sy_ + (size_t)x) * elem_;
  }
  void launch_box(void* in, void* aux, void* out, const Box& b, double dt, double a, double b_,
                  bool ls);
  void launch_fused_box(const Box& b, double dt, bool exclusive);
  void fused_view(int a, int lo, int hi, Range& view, Range& act, Range& outr) const;
  void stage_cart(void* in, void* aux, void* out, double a, double b, double dt, bool ls);
  void step_fused_cart(double dt);
  void start_halo_cart(void* field, bool on_comm = false);
  void error_norms_cart(double& l1, double& l2, double& linf);
  template <typename V>
  std::vector<V> gather_cart();
  double exact_scale() const;  // decay factor of the exact solution at t_ (sine / heat ICs)
  void check_transport();      // exits if the transport reported deferred errors

  Problem p_;
  Transport* tr_;
  ProcEnv env_;
  Slab slab_;
  int64_t sy_ = 0, sz_ = 0;  // element pitches (2-D: sz_ = row pitch of the decomposed axis)
  // element offset of the r-th row of a slab field counted over whole planes of p_.ny rows
  // (3-D planes may carry padding rows: sz_ >= ny sy_)
  size_t row_offset(int r) const {
    return p_.dims == 3 ? (size_t)(r / p_.ny) * sz_ + (size_t)(r % p_.ny) * sy_
                        : (size_t)r * sy_;
  }
  size_t elem_ = 8, plane_bytes_ = 0, field_bytes_ = 0;
  // SSP-RK3: u -> A -> B -> u.  Fused step / LSRK: u <-> A ping-pong (B = du for LSRK).
  void *u_ = nullptr, *A_ = nullptr, *B_ = nullptr;
  std::unique_ptr<Watchdog> wd_;  // multi-rank runs: comm watchdog while stepping
  void beat() {
    if (wd_) wd_->beat();
  }
  struct Armed {  // the watchdog watches the stepping phase of a run
    Watchdog* w;
    explicit Armed(Watchdog* w_) : w(w_) {
      if (w) w->arm();
    }
    ~Armed() {
      if (w) w->disarm();
    }
  };
  bool fused_ = false;
  Range zact_;  // fused: local planes whose intermediate stages are updated
  bool cart_ = false;
  Cart cd_;
  int alloc_[3] = {1, 1, 1};  // local extents incl. ghosts (array order)
  Box full_box_, interior_box_;
  std::vector<Box> boundary_boxes_;
  std::vector<std::vector<HaloPlanMsg>> plan_;  // Cartesian halo phases
  double init_s_ = 0;                          // barrier-fenced field setup time
  hipStream_t compute_ = nullptr, comm_ = nullptr;
  hipStream_t ls_ = nullptr;  // stream of the stencil launches (compute_, or comm_ for the
                              // boundary launch of the bcomm_ schedule)
  hipEvent_t ready_ = nullptr, halo_done_ = nullptr;
  hipEvent_t cready_ = nullptr, bdone_ = nullptr;  // bcomm_: compute_ -> comm_, comm_ -> compute_
  bool bcomm_ = false;
  bool fput_ = false;  // fused halo puts (engine.cpp step_fused / stage)
  void bcomm_begin();
  void bcomm_end();
  bool halo_pending_ = false;
  Range full_, interior_, blo_, bhi_;
  double t_ = 0;
  int it_ = 0;
  void* red_ws_ = nullptr;  // watchdog reduction workspace / device result (lazy)
  double* red_ = nullptr;
  int fault_rank_ = -1, fault_step_ = -1;  // ADVDIFF_FAULT="RANK:STEP" (failure tests)
  void watchdog() {
    if (p_.check_every > 0 && it_ % p_.check_every == 0) check_finite();
    if (fault_rank_ == env_.rank && fault_step_ == it_)
      throw std::runtime_error("injected fault on rank " + std::to_string(env_.rank) +
                               " at step " + std::to_string(it_));
  }
  // hipGraph stepping: one executable graph per (dt, u_ parity) of kGraphSteps steps
  bool graph_ = false;
  bool step2_env_ = true;  // ADVDIFF_STEP2=0: one step per launch
  int warm_ = 0;  // eager steps run so far (handshakes)
  struct GraphKey {
    double dt;
    void* u;
    bool operator<(const GraphKey& o) const { return dt < o.dt || (dt == o.dt && u < o.u); }
  };
  std::map<GraphKey, hipGraphExec_t> graphs_;
  hipGraphExec_t graph_for(double dt);
};

// Reference summary blocks (MultiGPU/Diffusion3d_Baseline/Tools.c:255-270)
std::string summary_multigpu(const std::string& title, const std::string& opt, const Stats& s,
                             const Problem& p, int nprocs);
// the single-GPU apps' summary block (utils/metrics.py summary_singlegpu)
std::string summary_singlegpu(const std::string& title, const std::string& opt, const Stats& s,
                              const Problem& p,
                              const std::vector<std::pair<std::string, std::string>>& extra);
void write_binary(const std::string& path, const std::vector<float>& data);

}  // namespace advdiff::rt
