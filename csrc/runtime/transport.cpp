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
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <thread>

#include "runtime.hpp"

namespace advdiff::rt {

static int env_int(const char* k, int def) {
  const char* v = std::getenv(k);
  return v ? std::atoi(v) : def;
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
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty()) return;
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

// ---------------------------------------------------------------- host-staged TCP
class SocketTransport final : public Transport {
 public:
  // full mesh: rank j > i connects to rank i's listener (port MASTER_PORT+1+i), so any
  // pair of ranks (slab neighbours, Cartesian faces) has its own socket
  explicit SocketTransport(const ProcEnv& e) : star_(e), env_(e) {
    if (e.size == 1) return;
    fds_.assign(e.size, -1);
    const int base = e.master_port + 1;
    int lfd = -1;
    if (e.rank < e.size - 1) lfd = listen_on(base + e.rank);
    star_.reduce(0.0, false);  // every listener is up
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
  ~SocketTransport() override {
    for (int fd : fds_)
      if (fd >= 0) ::close(fd);
    if (h_send_) (void)hipHostFree(h_send_);
    if (h_recv_) (void)hipHostFree(h_recv_);
  }
  const char* name() const override { return "socket"; }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty()) return;
    size_t total = 0;
    for (const Msg& m : msgs) total += m.bytes;
    if (total > cap_) {
      if (h_send_) (void)hipHostFree(h_send_);
      if (h_recv_) (void)hipHostFree(h_recv_);
      HIP_CHECK(hipHostMalloc(&h_send_, total));
      HIP_CHECK(hipHostMalloc(&h_recv_, total));
      cap_ = total;
    }
    std::vector<size_t> off(msgs.size());
    size_t o = 0;
    for (size_t q = 0; q < msgs.size(); ++q) {
      off[q] = o;
      HIP_CHECK(hipMemcpyAsync((char*)h_send_ + o, msgs[q].send, msgs[q].bytes,
                               hipMemcpyDeviceToHost, s));
      o += msgs[q].bytes;
    }
    HIP_CHECK(hipStreamSynchronize(s));
    // one sender thread per message: a send that blocks on a full socket never stalls
    // the receives below, whatever order the peers read in
    std::vector<std::thread> tx;
    for (size_t q = 0; q < msgs.size(); ++q)
      tx.emplace_back([&, q] { send_all(fds_[msgs[q].peer], (char*)h_send_ + off[q], msgs[q].bytes); });
    for (size_t q = 0; q < msgs.size(); ++q)
      recv_all(fds_[msgs[q].peer], (char*)h_recv_ + off[q], msgs[q].bytes);
    for (auto& t : tx) t.join();
    for (size_t q = 0; q < msgs.size(); ++q)
      HIP_CHECK(hipMemcpyAsync(msgs[q].recv, (char*)h_recv_ + off[q], msgs[q].bytes,
                               hipMemcpyHostToDevice, s));
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
  ProcEnv env_;
  std::vector<int> fds_;
  void *h_send_ = nullptr, *h_recv_ = nullptr;
  size_t cap_ = 0;
};

// Single process: no communication at all.
class LocalTransport final : public Transport {
 public:
  const char* name() const override { return "local"; }
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
  if (kind == "rccl" || kind.empty()) return std::make_unique<RcclTransport>(env);
  throw std::runtime_error("unknown transport " + kind);
}

}  // namespace advdiff::rt
