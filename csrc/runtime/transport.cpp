// Transports of the native runtime.
//
//  * Star: TCP star around rank 0 (bootstrap of the RCCL unique id, scalar reductions,
//    barrier, result gather) — replaces MPI_Init / MPI_Barrier / the hand-rolled
//    Isend/Recv gather of the reference (MultiGPU/Diffusion3d_Baseline/Tools.c:228-242,
//    main.c:327-335).  Port: ADVDIFF_PORT, else MASTER_PORT+17 (MASTER_PORT itself may
//    be held by a torchrun agent's store).
//  * RcclTransport: grouped ncclSend/ncclRecv of the ghost slabs straight from/into the
//    device fields on the caller's stream (RCCL over xGMI, zero copy).
//  * SocketTransport: host-staged exchange over a TCP full mesh.  It lets several ranks
//    share ONE GPU (RCCL refuses that), so the native multi-rank path is testable on a
//    single-GPU box; it is also the reference's own transport pattern (D2H -> send ->
//    recv -> H2D, main.c:209-288).
//  * IpcTransport: peer-mapped puts (kernels/ipc.hip): a rank's
//    copy kernel writes its boundary box straight into the neighbour's ghost box (field
//    mapped with hipIpcOpenMemHandle), then raises the neighbour's device flag; the
//    receiving stream waits on its own flags.  No host synchronisation, no staging, no
//    pack/unpack; across GPUs over xGMI, and between ranks sharing one GPU (tests).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <map>
#include <thread>
#include <tuple>

#include "runtime.hpp"

namespace advdiff::rt {

static int env_int(const char* k, int def) {
  const char* v = std::getenv(k);
  return v ? std::atoi(v) : def;
}

bool poison_enabled() {
  static const bool on = env_int("ADVDIFF_POISON", 0) != 0;
  return on;
}

Transport::~Transport() {
  for (void* b : stage_)
    if (b) (void)hipFree(b);
}

void* Transport::staging(size_t slot, size_t bytes, hipStream_t stream) {
  if (stage_.size() <= slot) {
    stage_.resize(slot + 1, nullptr);
    stage_cap_.resize(slot + 1, 0);
  }
  if (stage_cap_[slot] < bytes) {
    if (stage_[slot]) {
      HIP_CHECK(hipStreamSynchronize(stream));  // the old buffer may still be in use
      HIP_CHECK(hipFree(stage_[slot]));
    }
    HIP_CHECK(hipMalloc(&stage_[slot], bytes));
    if (poison_enabled()) HIP_CHECK(hipMemsetAsync(stage_[slot], 0xFF, bytes, stream));
    stage_cap_[slot] = bytes;
  }
  return stage_[slot];
}

// pack strided send boxes, one exchange(), unpack strided receive boxes (stream-ordered)
void Transport::exchange_boxes(const std::vector<BoxMsg>& msgs, hipStream_t s) {
  std::vector<Msg> flat;
  struct Unpack {
    const BoxMsg* m;
    void* buf;
  };
  std::vector<Unpack> unpack;
  size_t slot = 0;
  for (const BoxMsg& m : msgs) {
    Msg f;
    f.peer = m.peer;
    f.bytes = m.bytes();
    if (m.send_contiguous()) {
      f.send = m.send;
    } else {
      void* b = staging(slot++, f.bytes, s);
      if (!dry_)
        KERNEL_CHECK(advdiff_copy_box(m.dtype, b, m.ni, (int64_t)m.ni * m.nj, m.send, m.ssy,
                                      m.ssz, m.ni, m.nj, m.nk, s));
      f.send = b;
    }
    if (m.recv_contiguous()) {
      f.recv = m.recv;
    } else {
      f.recv = staging(slot++, f.bytes, s);
      unpack.push_back(Unpack{&m, f.recv});
    }
    flat.push_back(f);
  }
  if (dry_) return;  // staging sized (outside any capture); nothing enqueued
  exchange(flat, s);
  for (const Unpack& u : unpack) {
    const BoxMsg& m = *u.m;
    KERNEL_CHECK(advdiff_copy_box(m.dtype, m.recv, m.rsy, m.rsz, u.buf, m.ni, (int64_t)m.ni * m.nj,
                                  m.ni, m.nj, m.nk, s));
  }
}

static void check_distinct_peers(const std::vector<int>& peers) {
  for (size_t i = 0; i < peers.size(); ++i)
    for (size_t j = i + 1; j < peers.size(); ++j)
      if (peers[i] == peers[j])
        throw std::runtime_error("transport: two messages to one peer in one exchange");
}

ProcEnv ProcEnv::from_env() {
  ProcEnv e;
  e.size = env_int("WORLD_SIZE", 1);
  e.rank = env_int("RANK", 0);
  e.local_rank = env_int("LOCAL_RANK", e.rank);
  if (const char* a = std::getenv("MASTER_ADDR")) e.master_addr = a;
  const int mp = env_int("MASTER_PORT", 29500);
  e.master_port = env_int("ADVDIFF_PORT", mp + 17);
  return e;
}

// ---------------------------------------------------------------- socket helpers
static void die(const char* what) {
  std::perror(what);
  std::exit(3);
}

static void send_all(int fd, const void* buf, size_t n) {
  const char* p = (const char*)buf;
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) die("send");
    p += k;
    n -= (size_t)k;
  }
}

static void recv_all(int fd, void* buf, size_t n) {
  char* p = (char*)buf;
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) die("recv");
    p += k;
    n -= (size_t)k;
  }
}

static int listen_on(int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)port);
  if (::bind(fd, (sockaddr*)&a, sizeof(a)) != 0) die("bind");
  if (::listen(fd, 256) != 0) die("listen");
  return fd;
}

static int connect_to(const std::string& host, int port, double timeout_s = 120.0) {
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    std::string ps = std::to_string(port);
    if (::getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) == 0) {
      int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        ::freeaddrinfo(res);
        int one = 1;
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        return fd;
      }
      ::close(fd);
      ::freeaddrinfo(res);
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      die("connect timeout");
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

// ---------------------------------------------------------------- star
class Star {
 public:
  explicit Star(const ProcEnv& e) : env_(e) {
    if (e.size == 1) return;
    if (e.rank == 0) {
      int lfd = listen_on(e.master_port);
      fds_.assign(e.size, -1);
      for (int q = 1; q < e.size; ++q) {
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) die("accept");
        int r = -1;
        recv_all(fd, &r, sizeof(r));
        fds_[r] = fd;
      }
      ::close(lfd);
    } else {
      hub_ = connect_to(e.master_addr, e.master_port);
      send_all(hub_, &e.rank, sizeof(int));
    }
  }
  ~Star() {
    for (int fd : fds_)
      if (fd >= 0) ::close(fd);
    if (hub_ >= 0) ::close(hub_);
  }
  void bcast(void* buf, size_t n) {
    if (env_.size == 1) return;
    if (env_.rank == 0)
      for (int q = 1; q < env_.size; ++q) send_all(fds_[q], buf, n);
    else
      recv_all(hub_, buf, n);
  }
  double reduce(double v, bool is_max) {
    if (env_.size == 1) return v;
    if (env_.rank == 0) {
      double acc = v;
      for (int q = 1; q < env_.size; ++q) {
        double x;
        recv_all(fds_[q], &x, sizeof(x));
        acc = is_max ? std::max(acc, x) : acc + x;
      }
      bcast(&acc, sizeof(acc));
      return acc;
    }
    send_all(hub_, &v, sizeof(v));
    double r;
    recv_all(hub_, &r, sizeof(r));
    return r;
  }
  std::vector<char> gather(const std::vector<char>& local) {
    if (env_.size == 1) return local;
    if (env_.rank == 0) {
      std::vector<char> out(local);
      for (int q = 1; q < env_.size; ++q) {
        uint64_t n = 0;
        recv_all(fds_[q], &n, sizeof(n));
        size_t off = out.size();
        out.resize(off + n);
        recv_all(fds_[q], out.data() + off, n);
      }
      return out;
    }
    uint64_t n = local.size();
    send_all(hub_, &n, sizeof(n));
    send_all(hub_, local.data(), n);
    return {};
  }

 private:
  ProcEnv env_;
  std::vector<int> fds_;
  int hub_ = -1;
};

// the two messages of a slab exchange (lower / upper neighbour; -1 = none)
static std::vector<Msg> neighbour_msgs(const void* send_lo, void* recv_lo, const void* send_hi,
                                       void* recv_hi, size_t bytes, int lower, int upper) {
  std::vector<Msg> m;
  if (lower >= 0) m.push_back(Msg{lower, send_lo, recv_lo, bytes});
  if (upper >= 0) m.push_back(Msg{upper, send_hi, recv_hi, bytes});
  return m;
}

// ---------------------------------------------------------------- RCCL
#define NCCL_CHECK(expr)                                                              \
  do {                                                                                \
    ncclResult_t r_ = (expr);                                                         \
    if (r_ != ncclSuccess) {                                                          \
      std::fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, \
                   __LINE__);                                                         \
      std::exit(4);                                                                   \
    }                                                                                 \
  } while (0)

class RcclTransport final : public Transport {
 public:
  explicit RcclTransport(const ProcEnv& e) : star_(e), env_(e) {
    ncclUniqueId id;
    if (e.rank == 0) NCCL_CHECK(ncclGetUniqueId(&id));
    star_.bcast(&id, sizeof(id));
    NCCL_CHECK(ncclCommInitRank(&comm_, e.size, id, e.rank));
  }
  ~RcclTransport() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  const char* name() const override { return "rccl"; }
  int poll_error() override {
    if (comm_ == nullptr) return 0;
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return 1;
    return r == ncclSuccess || r == ncclInProgress ? 0 : (int)r;
  }
  void abort() override {
    if (comm_ == nullptr) return;
    ncclComm_t c = comm_;
    comm_ = nullptr;  // the destructor must not destroy an aborted communicator
    (void)ncclCommAbort(c);
  }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty() || dry_) return;
    NCCL_CHECK(ncclGroupStart());
    for (const Msg& m : msgs) {
      NCCL_CHECK(ncclSend(m.send, m.bytes, ncclChar, m.peer, comm_, s));
      NCCL_CHECK(ncclRecv(m.recv, m.bytes, ncclChar, m.peer, comm_, s));
    }
    NCCL_CHECK(ncclGroupEnd());
  }
  void halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
            size_t bytes, int lower, int upper, hipStream_t s) override {
    exchange(neighbour_msgs(send_lo, recv_lo, send_hi, recv_hi, bytes, lower, upper), s);
  }
  double allreduce_max(double v) override { return star_.reduce(v, true); }
  double allreduce_sum(double v) override { return star_.reduce(v, false); }
  void barrier() override { star_.reduce(0.0, false); }
  std::vector<char> gather(const std::vector<char>& local) override { return star_.gather(local); }

 private:
  Star star_;
  ProcEnv env_;
  ncclComm_t comm_ = nullptr;
};

// ---------------------------------------------------------------- TCP full mesh
// rank j > i connects to rank i's listener (port MASTER_PORT+1+i), so any pair of ranks
// (slab neighbours, Cartesian faces) has its own socket
class Mesh {
 public:
  Mesh(const ProcEnv& e, Star& star) {
    if (e.size == 1) return;
    fds_.assign(e.size, -1);
    const int base = e.master_port + 1;
    int lfd = -1;
    if (e.rank < e.size - 1) lfd = listen_on(base + e.rank);
    star.reduce(0.0, false);  // every listener is up
    for (int q = 0; q < e.rank; ++q) {
      fds_[q] = connect_to("127.0.0.1", base + q);
      send_all(fds_[q], &e.rank, sizeof(int));
    }
    for (int n = e.rank + 1; n < e.size; ++n) {
      int fd = ::accept(lfd, nullptr, nullptr);
      if (fd < 0) die("accept");
      int r = -1;
      recv_all(fd, &r, sizeof(r));
      if (r <= e.rank || r >= e.size) die("bad peer rank");
      fds_[r] = fd;
    }
    if (lfd >= 0) ::close(lfd);
  }
  ~Mesh() {
    for (int fd : fds_)
      if (fd >= 0) ::close(fd);
  }
  int fd(int peer) const { return fds_[peer]; }
  // send out[q] to peers[q] and receive in[q] from peers[q] (distinct peers): one sender
  // thread per message, so a send that blocks on a full socket never stalls the receives
  void swap(const std::vector<int>& peers, const std::vector<const void*>& out,
            const std::vector<void*>& in, const std::vector<size_t>& bytes) {
    check_distinct_peers(peers);
    std::vector<std::thread> tx;
    for (size_t q = 0; q < peers.size(); ++q)
      tx.emplace_back([&, q] { send_all(fds_[peers[q]], out[q], bytes[q]); });
    for (size_t q = 0; q < peers.size(); ++q) recv_all(fds_[peers[q]], in[q], bytes[q]);
    for (auto& t : tx) t.join();
  }

 private:
  std::vector<int> fds_;
};

// ---------------------------------------------------------------- host-staged TCP
class SocketTransport final : public Transport {
 public:
  explicit SocketTransport(const ProcEnv& e) : star_(e), mesh_(e, star_), env_(e) {}
  ~SocketTransport() override {
    if (h_send_) (void)hipHostFree(h_send_);
    if (h_recv_) (void)hipHostFree(h_recv_);
  }
  const char* name() const override { return "socket"; }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty() || dry_) return;
    size_t total = 0;
    for (const Msg& m : msgs) total += m.bytes;
    if (total > cap_) {
      if (h_send_) (void)hipHostFree(h_send_);
      if (h_recv_) (void)hipHostFree(h_recv_);
      HIP_CHECK(hipHostMalloc(&h_send_, total));
      HIP_CHECK(hipHostMalloc(&h_recv_, total));
      if (poison_enabled()) {
        std::memset(h_send_, 0xFF, total);
        std::memset(h_recv_, 0xFF, total);
      }
      cap_ = total;
    }
    std::vector<int> peers;
    std::vector<const void*> out;
    std::vector<void*> in;
    std::vector<size_t> bytes;
    size_t o = 0;
    for (const Msg& m : msgs) {
      HIP_CHECK(hipMemcpyAsync((char*)h_send_ + o, m.send, m.bytes, hipMemcpyDeviceToHost, s));
      peers.push_back(m.peer);
      out.push_back((char*)h_send_ + o);
      in.push_back((char*)h_recv_ + o);
      bytes.push_back(m.bytes);
      o += m.bytes;
    }
    HIP_CHECK(hipStreamSynchronize(s));
    mesh_.swap(peers, out, in, bytes);
    for (size_t q = 0; q < msgs.size(); ++q)
      HIP_CHECK(hipMemcpyAsync(msgs[q].recv, in[q], msgs[q].bytes, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));  // staging buffers are reused next call
  }
  void halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
            size_t bytes, int lower, int upper, hipStream_t s) override {
    exchange(neighbour_msgs(send_lo, recv_lo, send_hi, recv_hi, bytes, lower, upper), s);
  }
  double allreduce_max(double v) override { return star_.reduce(v, true); }
  double allreduce_sum(double v) override { return star_.reduce(v, false); }
  void barrier() override { star_.reduce(0.0, false); }
  std::vector<char> gather(const std::vector<char>& local) override { return star_.gather(local); }

 private:
  Star star_;
  Mesh mesh_;
  ProcEnv env_;
  void *h_send_ = nullptr, *h_recv_ = nullptr;
  size_t cap_ = 0;
};

// ---------------------------------------------------------------- IPC peer puts
class IpcTransport final : public Transport {
 public:
  explicit IpcTransport(const ProcEnv& e) : star_(e), mesh_(e, star_), env_(e) {
    ipc_check(advdiff_ipc_create(e.size, e.rank, &ctx_), "advdiff_ipc_create");
    advdiff_ipc_addr mine;
    ipc_check(advdiff_ipc_flags_addr(ctx_, &mine), "advdiff_ipc_flags_addr");
    // every rank maps every other rank's flag block (small; any pair may be neighbours)
    std::vector<int> peers;
    for (int q = 0; q < e.size; ++q)
      if (q != e.rank) peers.push_back(q);
    std::vector<advdiff_ipc_addr> theirs(peers.size());
    std::vector<const void*> out(peers.size(), &mine);
    std::vector<void*> in;
    for (auto& t : theirs) in.push_back(&t);
    mesh_.swap(peers, out, in, std::vector<size_t>(peers.size(), sizeof(advdiff_ipc_addr)));
    for (size_t q = 0; q < peers.size(); ++q)
      ipc_check(advdiff_ipc_set_peer(ctx_, peers[q], &theirs[q]), "advdiff_ipc_set_peer");
    star_.reduce(0.0, false);  // all mapped before anyone signals
    if (env_int("ADVDIFF_IPC_PREFLIGHT", 1)) preflight(peers);
  }
  // Validated round trips between every pair of ranks before a run relies on the
  // transport (the Python counterpart: parallel/ipc.py IpcPeers.preflight): peer access
  // between the devices, then rounds of a distinct 32-bit pattern per (sender, receiver,
  // round), each receiver first reading its buffers through its caches (a reduction
  // kernel) so a put that the flag overtakes or a stale cache line shows up as a mismatch.
  void preflight(const std::vector<int>& peers) {
    if (peers.empty()) return;
    int mydev = 0;
    HIP_CHECK(hipGetDevice(&mydev));
    std::vector<int> devs(peers.size(), -1);
    {
      std::vector<const void*> o(peers.size(), &mydev);
      std::vector<void*> in;
      for (int& d : devs) in.push_back(&d);
      mesh_.swap(peers, o, in, std::vector<size_t>(peers.size(), sizeof(int)));
    }
    double bad = 0;
    for (size_t q = 0; q < peers.size(); ++q) {
      if (devs[q] == mydev) continue;
      int ok = 0;
      HIP_CHECK(hipDeviceCanAccessPeer(&ok, mydev, devs[q]));
      if (!ok) {
        std::fprintf(stderr, "ipc preflight: rank %d (device %d) has no peer access to rank %d "
                     "(device %d)\n", env_.rank, mydev, peers[q], devs[q]);
        bad = 1;
      }
    }
    if (star_.reduce(bad, true) > 0) std::exit(2);
    const size_t words = 3 * 24 * 200, bytes = words * 4;
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<void*> snd(peers.size()), rcv(peers.size());
    for (size_t q = 0; q < peers.size(); ++q) {
      HIP_CHECK(hipMalloc(&snd[q], bytes));
      HIP_CHECK(hipMalloc(&rcv[q], bytes));
      // stream-ordered fill (a null-stream hipMemset is not ordered before `st`)
      HIP_CHECK(hipMemsetAsync(rcv[q], 0, bytes, st));
    }
    HIP_CHECK(hipStreamSynchronize(st));
    void* ws = nullptr;
    double* red = nullptr;
    HIP_CHECK(hipMalloc(&ws, advdiff_reduce_workspace_bytes()));
    HIP_CHECK(hipMalloc((void**)&red, 3 * sizeof(double)));
    std::vector<uint32_t> host(words);
    long long mism = 0;
    for (uint32_t round = 1; round <= 3; ++round) {
      std::vector<Msg> msgs;
      for (size_t q = 0; q < peers.size(); ++q) {
        const uint32_t v = 0x10000u * (uint32_t)env_.rank + 0x100u * (uint32_t)peers[q] + round;
        HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)snd[q], v, words, st));
        // the (stale) receive buffer passes through this GPU's caches first
        KERNEL_CHECK(advdiff_reduce_norms(ADVDIFF_F32, rcv[q], nullptr, 200, 200 * 24, 0, 200, 0,
                                          24, 0, 3, ws, red, st));
        msgs.push_back(Msg{peers[q], snd[q], rcv[q], bytes});
      }
      HIP_CHECK(hipStreamSynchronize(st));
      star_.reduce(0.0, false);
      exchange(msgs, st);
      HIP_CHECK(hipStreamSynchronize(st));
      for (size_t q = 0; q < peers.size(); ++q) {
        const uint32_t want = 0x10000u * (uint32_t)peers[q] + 0x100u * (uint32_t)env_.rank + round;
        HIP_CHECK(hipMemcpy(host.data(), rcv[q], bytes, hipMemcpyDeviceToHost));
        for (uint32_t w : host) mism += w != want;
      }
      star_.reduce(0.0, false);  // nobody starts the next round's puts before all compared
    }
    const long long to = errors();
    const double worst = star_.reduce((double)(mism + to), true);
    HIP_CHECK(hipDeviceSynchronize());
    ipc_check(advdiff_ipc_reset(ctx_), "advdiff_ipc_reset");  // unmap the preflight buffers
    dest_.clear();
    calls_.clear();
    star_.reduce(0.0, false);
    for (size_t q = 0; q < peers.size(); ++q) {
      (void)hipFree(snd[q]);
      (void)hipFree(rcv[q]);
    }
    (void)hipFree(ws);
    (void)hipFree(red);
    (void)hipStreamDestroy(st);
    if (worst > 0) {
      std::fprintf(stderr, "ipc preflight failed on rank %d: %lld mismatching words, %lld wait "
                   "timeouts (worst rank: %.0f)\n", env_.rank, mism, to, worst);
      std::exit(2);
    }
  }
  ~IpcTransport() override {
    (void)hipDeviceSynchronize();
    star_.reduce(0.0, false);  // nobody unmaps while a peer may still put into it
    advdiff_ipc_destroy(ctx_);
  }
  const char* name() const override { return "ipc"; }
  bool graph_safe() const override { return true; }
  bool needs_handshake() const override { return true; }

  void exchange_boxes(const std::vector<BoxMsg>& msgs, hipStream_t s) override {
    if (msgs.empty()) return;
    std::vector<int> peers;
    for (const BoxMsg& m : msgs) peers.push_back(m.peer);
    check_distinct_peers(peers);
    const std::vector<Dest> dst = resolve(msgs);
    if (dry_) return;  // handshake only
    for (size_t q = 0; q < msgs.size(); ++q) {  // the put: my box -> the peer's ghost box
      const BoxMsg& m = msgs[q];
      KERNEL_CHECK(advdiff_ipc_put(m.dtype, dst[q].ptr, dst[q].sy, dst[q].sz, m.send, m.ssy,
                                   m.ssz, m.ni, m.nj, m.nk, s));
    }
    ipc_check(advdiff_ipc_signal(ctx_, peers.data(), (int)peers.size(), s), "advdiff_ipc_signal");
    ipc_check(advdiff_ipc_wait(ctx_, peers.data(), (int)peers.size(), s), "advdiff_ipc_wait");
  }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    std::vector<BoxMsg> b;
    for (const Msg& m : msgs) b.push_back(flat_box(m.peer, m.send, m.recv, m.bytes));
    exchange_boxes(b, s);
  }
  void halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
            size_t bytes, int lower, int upper, hipStream_t s) override {
    exchange(neighbour_msgs(send_lo, recv_lo, send_hi, recv_hi, bytes, lower, upper), s);
  }
  bool halo_targets(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
                    size_t bytes, int lower, int upper, void** dst_lo, void** dst_hi) override {
    const std::vector<BoxMsg> b = halo_boxes(send_lo, recv_lo, send_hi, recv_hi, bytes, lower,
                                             upper);
    const std::vector<Dest> d = resolve(b);
    *dst_lo = *dst_hi = nullptr;
    for (size_t q = 0; q < b.size(); ++q) (b[q].peer == lower ? *dst_lo : *dst_hi) = d[q].ptr;
    return true;
  }
  void halo_signal(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
                   size_t bytes, int lower, int upper, hipStream_t s) override {
    const std::vector<BoxMsg> b = halo_boxes(send_lo, recv_lo, send_hi, recv_hi, bytes, lower,
                                             upper);
    if (b.empty()) return;
    (void)resolve(b);  // the same handshake bookkeeping as a halo() with puts
    if (dry_) return;
    std::vector<int> peers;
    for (const BoxMsg& m : b) peers.push_back(m.peer);
    ipc_check(advdiff_ipc_signal(ctx_, peers.data(), (int)peers.size(), s), "advdiff_ipc_signal");
    ipc_check(advdiff_ipc_wait(ctx_, peers.data(), (int)peers.size(), s), "advdiff_ipc_wait");
  }
  double allreduce_max(double v) override { return star_.reduce(v, true); }
  double allreduce_sum(double v) override { return star_.reduce(v, false); }
  void barrier() override { star_.reduce(0.0, false); }
  std::vector<char> gather(const std::vector<char>& local) override { return star_.gather(local); }
  long long errors() override {
    long long n = 0;
    ipc_check(advdiff_ipc_errors(ctx_, &n), "advdiff_ipc_errors");
    return n;
  }

 private:
  struct Dest {
    void* ptr = nullptr;
    int64_t sy = 0, sz = 0;
  };
  // what a rank tells its peer about the box it receives from it
  struct Announce {
    advdiff_ipc_addr addr;
    int64_t rsy, rsz;
    int ni, nj, nk, dtype;
    uint64_t call;  // per-pair exchange counter: both sides must be at the same call
  };
  static void ipc_check(int e, const char* what) {
    if (e != 0) {
      std::fprintf(stderr, "%s failed: %s\n", what, hipGetErrorString((hipError_t)e));
      std::exit(2);
    }
  }
  // a contiguous byte message as a box of 32-bit words (bit-exact for any dtype)
  static BoxMsg flat_box(int peer, const void* send, void* recv, size_t bytes) {
    if (bytes % 4) throw std::runtime_error("ipc: message size not a multiple of 4 bytes");
    BoxMsg b;
    b.peer = peer;
    b.dtype = ADVDIFF_F32;
    b.send = send;
    b.recv = recv;
    b.ni = (int)(bytes / 4);
    b.nj = b.nk = 1;
    b.ssy = b.rsy = b.ni;
    b.ssz = b.rsz = b.ni;
    return b;
  }
  std::vector<BoxMsg> halo_boxes(const void* send_lo, void* recv_lo, const void* send_hi,
                                 void* recv_hi, size_t bytes, int lower, int upper) {
    std::vector<BoxMsg> b;
    for (const Msg& m : neighbour_msgs(send_lo, recv_lo, send_hi, recv_hi, bytes, lower, upper))
      b.push_back(flat_box(m.peer, m.send, m.recv, m.bytes));
    return b;
  }
  // The peer's receive address of every message.  First use of a (peer, send, recv,
  // shape) pattern: the two ranks of each pair swap Announces over the mesh (both sides
  // hit the pattern at the same call: every rank runs the same step schedule).  Later
  // calls are table lookups: no host communication inside the time loop.
  std::vector<Dest> resolve(const std::vector<BoxMsg>& msgs) {
    std::vector<Dest> out(msgs.size());
    std::vector<size_t> miss;
    for (size_t q = 0; q < msgs.size(); ++q) {
      const BoxMsg& m = msgs[q];
      ++calls_[m.peer];
      auto it = dest_.find(key(m));
      if (it == dest_.end())
        miss.push_back(q);
      else
        out[q] = it->second;
    }
    if (miss.empty()) return out;
    std::vector<int> peers;
    std::vector<Announce> mine(miss.size()), theirs(miss.size());
    std::vector<const void*> o;
    std::vector<void*> in;
    for (size_t q = 0; q < miss.size(); ++q) {
      const BoxMsg& m = msgs[miss[q]];
      Announce& a = mine[q];
      std::memset(&a, 0, sizeof(a));
      ipc_check(advdiff_ipc_describe(ctx_, m.recv, &a.addr), "advdiff_ipc_describe");
      a.rsy = m.rsy;
      a.rsz = m.rsz;
      a.ni = m.ni;
      a.nj = m.nj;
      a.nk = m.nk;
      a.dtype = m.dtype;
      a.call = calls_[m.peer];
      peers.push_back(m.peer);
      o.push_back(&mine[q]);
      in.push_back(&theirs[q]);
    }
    mesh_.swap(peers, o, in, std::vector<size_t>(miss.size(), sizeof(Announce)));
    for (size_t q = 0; q < miss.size(); ++q) {
      const BoxMsg& m = msgs[miss[q]];
      const Announce& t = theirs[q];
      if (t.ni != m.ni || t.nj != m.nj || t.nk != m.nk || t.dtype != m.dtype || t.call != mine[q].call)
        throw std::runtime_error("ipc: rank " + std::to_string(env_.rank) + " and peer " +
                                 std::to_string(m.peer) + " disagree on a halo message");
      Dest d;
      ipc_check(advdiff_ipc_map(ctx_, &t.addr, &d.ptr), "advdiff_ipc_map");
      d.sy = t.rsy;
      d.sz = t.rsz;
      dest_[key(m)] = d;
      out[miss[q]] = d;
    }
    return out;
  }
  using Key = std::tuple<int, const void*, const void*, int, int, int>;
  static Key key(const BoxMsg& m) { return Key{m.peer, m.send, m.recv, m.ni, m.nj, m.nk}; }

  Star star_;
  Mesh mesh_;
  ProcEnv env_;
  advdiff_ipc* ctx_ = nullptr;
  std::map<Key, Dest> dest_;
  std::map<int, uint64_t> calls_;
};

// Single process: no communication at all.
class LocalTransport final : public Transport {
 public:
  const char* name() const override { return "local"; }
  bool graph_safe() const override { return true; }
  void exchange(const std::vector<Msg>&, hipStream_t) override {}
  void halo(const void*, void*, const void*, void*, size_t, int, int, hipStream_t) override {}
  double allreduce_max(double v) override { return v; }
  double allreduce_sum(double v) override { return v; }
  void barrier() override {}
  std::vector<char> gather(const std::vector<char>& local) override { return local; }
};

std::unique_ptr<Transport> make_transport(const ProcEnv& env, const std::string& kind) {
  if (env.size == 1) return std::make_unique<LocalTransport>();
  if (kind == "socket") return std::make_unique<SocketTransport>(env);
  if (kind == "ipc") return std::make_unique<IpcTransport>(env);
  if (kind == "rccl" || kind.empty()) return std::make_unique<RcclTransport>(env);
  throw std::runtime_error("unknown transport " + kind);
}

}  // namespace advdiff::rt
