// Peer-to-peer transport primitives of one node: hipIpc-mapped device memory + device-side
// flags.  This is the P2PComm of SURVEY.md §7.1 ("peer-mapped xGMI puts"): a rank writes
// its boundary cells STRAIGHT INTO the neighbour's ghost cells (a put kernel whose
// destination is the neighbour's field, mapped into this process with
// hipIpcOpenMemHandle), then raises the neighbour's flag with a release store; the
// neighbour's stream waits on its own flag with an acquire spin.  Every step of an
// exchange is a kernel on a stream: no host synchronisation, no staging buffer, no pack or
// unpack, and the whole exchange can be captured into a hipGraph (the counters live in
// device memory, so replays keep counting).
//
// It replaces the reference's host-staged choreography (MultiGPU/Diffusion3d_Baseline/
// main.c:209-288: pack kernel -> D2H -> host-blocking stream sync -> MPI_Isend/Irecv ->
// MPI_Wait -> H2D -> unpack kernel).  Across GPUs the puts travel over xGMI (the mapping is
// a peer mapping); with several ranks on ONE GPU (the test configuration of a 1-GPU box,
// where RCCL refuses two ranks per device) the same code runs as same-device IPC.
//
// Memory ordering of one message (producer P -> consumer C), each link explicit:
//  1. put (ipc_put_kernel, P's comm stream): every remote store is a SYSTEM-scope store
//     (global_store ... sc0 sc1: written through P's L2 to C's memory, never parked as a
//     dirty non-coherent line in the L2 of whichever XCD ran the wave), and each wave
//     ends with s_waitcnt vmcnt(0), so the dispatch completes
//     only after its stores are acknowledged.  Nothing depends on the scope of the
//     dispatch's end-of-kernel cache action, nor on which XCD runs the signal.
//  2. signal (ipc_signal_kernel, same stream => after the put dispatch completed): a
//     system-scope RELEASE store of the message counter into C's flag block (uncached
//     memory, coherent across devices while kernels run).
//  3. wait (ipc_wait_kernel, C's comm stream): kIpcWaitWgs workgroups, dispatched
//     round-robin over the 8 XCDs (>= 2 per XCD), each spin until the counter arrives with
//     system-scope ACQUIRE loads and then issue a system-scope acquire fence
//     (buffer_inv sc0 sc1) — so EVERY XCD's L2 drops lines of the ghost box it may hold
//     from the previous step before any consumer reads them.  (A single-lane wait would
//     invalidate only its own XCD's L2.)
//  4. consume: C's compute stream waits for the comm stream's event; the consumer kernel
//     starts after the wait dispatch completed, with fresh L1s.
// Ranks that share one GPU share one L2/MALL, so tests on a 1-GPU box cannot expose a
// missing link; the bench's ipc preflight (IpcPeers.preflight: stale-cache pattern round
// trips between every pair of ranks) and its bitwise N-rank-vs-1-GPU check can.
//
// Flags block of a rank (device memory, exported): kIpcChannels independent channels of
// { recv[world] (written by the peers: the number of messages peer q has delivered on this
// channel), sent[world] (messages delivered to q, local), expect[world][kIpcWaitWgs]
// (messages consumed from q, per wait workgroup) }, then err (wait timeouts).  Channel 0
// carries the symmetric neighbour exchanges; the striped (relayed) slab exchange uses 1
// for source -> helper and 2 for helper -> destination, so a pair of ranks that meets in
// several roles of one exchange never mixes its counts.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "advdiff/kernels.h"
#include "launch.hpp"

namespace advdiff {
constexpr int kIpcWaitWgs = 16;   // wait workgroups: >= 2 per XCD (8 XCDs, round-robin)
constexpr int kIpcChannels = 3;
}  // namespace advdiff

struct advdiff_ipc {
  int world = 1, rank = 0;
  uint64_t* block = nullptr;          // kIpcChannels x (recv | sent | expect), err
  std::vector<uint64_t*> peer_block;  // peer q's flag block (mapped), or nullptr
  std::map<std::string, void*> opened;  // IPC handle bytes -> mapped base
  std::map<uintptr_t, hipIpcMemHandle_t> exported;  // allocation base -> handle
  std::mutex mu;
  size_t block_bytes = 0;
  size_t chan_stride() const { return (2 + (size_t)advdiff::kIpcWaitWgs) * world; }
  uint64_t* recv(int ch = 0) const { return block + ch * chan_stride(); }
  uint64_t* sent(int ch = 0) const { return recv(ch) + world; }
  uint64_t* expect(int ch = 0) const { return recv(ch) + 2 * world; }  // [world][kIpcWaitWgs]
  // peer q's recv[rank] of channel ch (its block has our layout: same world)
  uint64_t* peer_cell(int q, int ch) const {
    return peer_block[q] ? peer_block[q] + ch * chan_stride() + rank : nullptr;
  }
  unsigned long long* err() const;
};

namespace advdiff {

constexpr int kIpcMaxPeers = 32;  // 3^3 - 1 = 26 neighbours of a direct exchange

struct IpcSignalArgs {
  uint64_t* remote[kIpcMaxPeers];  // peer's recv[rank]
  uint64_t* sent[kIpcMaxPeers];    // own sent[peer]
  int n;
};

struct IpcWaitArgs {
  const uint64_t* flag[kIpcMaxPeers];  // own recv[peer]
  uint64_t* expect[kIpcMaxPeers];      // own expect[peer][0..kIpcWaitWgs)
  int n;
  unsigned long long* err;
  uint64_t timeout_ticks;  // s_memrealtime runs at 100 MHz
};

// The put (link 1 above): dst box (peer memory) <- src box (own field), one row of ni
// elements per (blockIdx.y, blockIdx.z), every store system-scope.  Elements move as
// 32/64-bit words (bit-exact for any dtype).
template <typename W>
__global__ void ipc_put_kernel(W* __restrict__ dst, int64_t dsy, int64_t dsz,
                               const W* __restrict__ src, int64_t ssy, int64_t ssz, int ni,
                               int nj) {
  const int j = blockIdx.y;
  const int k = blockIdx.z;
  if (j < nj) {
    const W* s = src + (int64_t)k * ssz + (int64_t)j * ssy;
    W* d = dst + (int64_t)k * dsz + (int64_t)j * dsy;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ni; i += gridDim.x * blockDim.x)
      __hip_atomic_store(d + i, s[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // every store of this wave acknowledged before the wave (and so the dispatch) ends
  __builtin_amdgcn_s_waitcnt(0);
}

// lane q: sent[q] += 1, then publish it to the peer with a system-scope release store
// (link 2: the put dispatch before it on this stream has completed)
__global__ void ipc_signal_kernel(IpcSignalArgs a) {
  const int q = threadIdx.x;
  if (q >= a.n) return;
  // the counters are touched by one lane of one kernel at a time (stream order), but the
  // kernels may run on different XCDs: device-scope atomics, never a stale L2 line
  const uint64_t v = __hip_atomic_load(a.sent[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __hip_atomic_store(a.sent[q], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(a.remote[q], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Link 3.  Workgroup w, lane q: expect[q][w] += 1 (each workgroup its own counter, so no
// workgroup can see another's increment), spin (acquire loads, s_sleep) until recv[q]
// reaches it, then a system-scope acquire fence invalidates this XCD's caches.
// Bounded: after timeout_ticks the lane records a timeout and leaves, so the grid always
// drains even if a peer died (the host checks advdiff_ipc_errors at its sync points).
// Ranks SHARING one GPU (tests) need every queue of every rank mapped by the hardware
// scheduler: a spinning wait on a mapped queue can starve a producer whose queue is not.
// The tests and scripts run them with GPU_MAX_HW_QUEUES=2: 1 serialises a rank's own
// compute and comm streams onto one queue (the Python path then deadlocks: the comm
// stream's spin blocks the compute kernels queued behind it), and the default 4 per
// process oversubscribes the scheduler with 4+ ranks (a spinning queue starves a peer).
__global__ void ipc_wait_kernel(IpcWaitArgs a) {
  const int q = threadIdx.x;
  const int w = blockIdx.x;
  if (q < a.n) {
    uint64_t* ex = a.expect[q] + w;
    const uint64_t e = __hip_atomic_load(ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(ex, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(a.flag[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(4);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        atomicAdd(a.err, 1ull);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: buffer_inv sc0 sc1
}

static uint64_t wait_timeout_ticks() {
  static const uint64_t t = [] {
    const char* v = std::getenv("ADVDIFF_IPC_TIMEOUT_S");
    const double s = v ? std::atof(v) : 120.0;
    return (uint64_t)(s * 1e8);
  }();
  return t;
}

}  // namespace advdiff

unsigned long long* advdiff_ipc::err() const {
  return (unsigned long long*)(block + advdiff::kIpcChannels * chan_stride());
}

extern "C" int advdiff_ipc_create(int world, int rank, advdiff_ipc** out) {
  if (world < 1 || rank < 0 || rank >= world || out == nullptr) return hipErrorInvalidValue;
  auto* c = new advdiff_ipc;
  c->world = world;
  c->rank = rank;
  c->peer_block.assign(world, nullptr);
  const size_t bytes =
      (advdiff::kIpcChannels * (2 + (size_t)advdiff::kIpcWaitWgs) * world + 1) * sizeof(uint64_t);
  c->block_bytes = bytes < 4096 ? 4096 : bytes;
  // Uncached device memory: a peer GPU's release store lands in this block WHILE the wait
  // kernel spins on it, and only fine-grained / uncached memory promises cross-device
  // coherence inside a dispatch (coarse-grained memory only at dispatch boundaries).
  hipError_t e = hipExtMallocWithFlags((void**)&c->block, c->block_bytes,
                                       hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c->block, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();  // setup only: zeroed before any peer maps it
  if (e != hipSuccess) {
    delete c;
    return e;
  }
  *out = c;
  return hipSuccess;
}

extern "C" int advdiff_ipc_destroy(advdiff_ipc* c) {
  if (c == nullptr) return hipSuccess;
  (void)hipDeviceSynchronize();
  for (auto& kv : c->opened) (void)hipIpcCloseMemHandle(kv.second);
  (void)hipFree(c->block);
  delete c;
  return hipSuccess;
}

// address of `ptr` as (IPC handle of its allocation, byte offset)
extern "C" int advdiff_ipc_describe(advdiff_ipc* c, const void* ptr, advdiff_ipc_addr* out) {
  if (c == nullptr || ptr == nullptr || out == nullptr) return hipErrorInvalidValue;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr);
  if (e != hipSuccess) {
    std::fprintf(stderr, "advdiff_ipc_describe: hipMemGetAddressRange(%p): %s\n", ptr,
                 hipGetErrorString(e));
    return e;
  }
  std::lock_guard<std::mutex> g(c->mu);
  // Export first: it succeeds for an allocation not exported yet (new, or one reallocated
  // at a freed base — whose cached handle is stale) and fails for a live allocation
  // exported before, whose cached handle is then still the right one.
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, base);
  auto it = c->exported.find((uintptr_t)base);
  if (e == hipSuccess) {
    if (it == c->exported.end())
      it = c->exported.emplace((uintptr_t)base, h).first;
    else
      it->second = h;
  } else {
    (void)hipGetLastError();  // not a launch error: keep KERNEL_CHECK's last-error clean
    if (it == c->exported.end()) {
      std::fprintf(stderr, "advdiff_ipc_describe: hipIpcGetMemHandle(base %p, %zu B, ptr %p): %s\n",
                   (void*)base, size, ptr, hipGetErrorString(e));
      return e;
    }
  }
  static_assert(sizeof(hipIpcMemHandle_t) <= sizeof(out->handle), "IPC handle size");
  std::memset(out, 0, sizeof(*out));
  std::memcpy(out->handle, &it->second, sizeof(hipIpcMemHandle_t));
  out->offset = (uint64_t)((const char*)ptr - (const char*)base);
  out->bytes = (uint64_t)size;
  return hipSuccess;
}

extern "C" int advdiff_ipc_flags_addr(advdiff_ipc* c, advdiff_ipc_addr* out) {
  return advdiff_ipc_describe(c, c ? c->recv() : nullptr, out);
}

// map a peer's address into this process (handles are opened once and cached)
extern "C" int advdiff_ipc_map(advdiff_ipc* c, const advdiff_ipc_addr* a, void** ptr) {
  if (c == nullptr || a == nullptr || ptr == nullptr) return hipErrorInvalidValue;
  const std::string key((const char*)a->handle, sizeof(hipIpcMemHandle_t));
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->opened.find(key);
  if (it == c->opened.end()) {
    hipIpcMemHandle_t h;
    std::memcpy(&h, a->handle, sizeof(h));
    void* base = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return e;
    it = c->opened.emplace(key, base).first;
  }
  *ptr = (char*)it->second + a->offset;
  return hipSuccess;
}

extern "C" int advdiff_ipc_set_peer(advdiff_ipc* c, int peer, const advdiff_ipc_addr* flags) {
  if (c == nullptr || peer < 0 || peer >= c->world || peer == c->rank) return hipErrorInvalidValue;
  void* base = nullptr;
  const int e = advdiff_ipc_map(c, flags, &base);
  if (e != hipSuccess) return e;
  c->peer_block[peer] = (uint64_t*)base;
  return hipSuccess;
}

// the put of link 1: like advdiff_copy_box, but every store is system-scope (dst is a peer
// mapping).  Elements are moved as 64-bit words when the element size, both bases and all
// strides allow it, else as 32-bit words.
extern "C" int advdiff_ipc_put(int dtype, void* dst, int64_t dsy, int64_t dsz, const void* src,
                               int64_t ssy, int64_t ssz, int ni, int nj, int nk, void* stream) {
  using namespace advdiff;
  if (ni <= 0 || nj <= 0 || nk <= 0) return hipSuccess;
  if (dtype != ADVDIFF_F64 && dtype != ADVDIFF_F32) return hipErrorInvalidValue;
  if (nj > 65535 || nk > 65535) return hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int esz = dtype == ADVDIFF_F64 ? 8 : 4;
  const bool w64 = esz == 8 || (((uintptr_t)dst | (uintptr_t)src) % 8 == 0 && ni % 2 == 0 &&
                                dsy % 2 == 0 && dsz % 2 == 0 && ssy % 2 == 0 && ssz % 2 == 0);
  const int f = w64 ? 8 / esz : 1;  // elements per word
  const int wi = ni / f;
  dim3 block(256), grid(std::min(div_up(wi, 256), 8), nj, nk);
  if (w64)
    hipLaunchKernelGGL(ipc_put_kernel<uint64_t>, grid, block, 0, st, (uint64_t*)dst, dsy / f,
                       dsz / f, (const uint64_t*)src, ssy / f, ssz / f, wi, nj);
  else
    hipLaunchKernelGGL(ipc_put_kernel<uint32_t>, grid, block, 0, st, (uint32_t*)dst, dsy, dsz,
                       (const uint32_t*)src, ssy, ssz, wi, nj);
  return hipGetLastError();
}

extern "C" int advdiff_ipc_signal_ch(advdiff_ipc* c, int ch, const int* peers, int n,
                                     void* stream) {
  using namespace advdiff;
  if (n <= 0) return hipSuccess;
  if (c == nullptr || peers == nullptr || n > kIpcMaxPeers || ch < 0 || ch >= kIpcChannels)
    return hipErrorInvalidValue;
  IpcSignalArgs a{};
  a.n = n;
  for (int q = 0; q < n; ++q) {
    const int p = peers[q];
    if (p < 0 || p >= c->world || c->peer_cell(p, ch) == nullptr) return hipErrorInvalidValue;
    a.remote[q] = c->peer_cell(p, ch);
    a.sent[q] = c->sent(ch) + p;
  }
  hipLaunchKernelGGL(ipc_signal_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
  return hipGetLastError();
}

extern "C" int advdiff_ipc_wait_ch(advdiff_ipc* c, int ch, const int* peers, int n,
                                   void* stream) {
  using namespace advdiff;
  if (n <= 0) return hipSuccess;
  if (c == nullptr || peers == nullptr || n > kIpcMaxPeers || ch < 0 || ch >= kIpcChannels)
    return hipErrorInvalidValue;
  IpcWaitArgs a{};
  a.n = n;
  a.err = c->err();
  a.timeout_ticks = wait_timeout_ticks();
  for (int q = 0; q < n; ++q) {
    const int p = peers[q];
    if (p < 0 || p >= c->world || p == c->rank) return hipErrorInvalidValue;
    a.flag[q] = c->recv(ch) + p;
    a.expect[q] = c->expect(ch) + (size_t)p * kIpcWaitWgs;
  }
  hipLaunchKernelGGL(ipc_wait_kernel, dim3(kIpcWaitWgs), dim3(64), 0, (hipStream_t)stream, a);
  return hipGetLastError();
}

extern "C" int advdiff_ipc_signal(advdiff_ipc* c, const int* peers, int n, void* stream) {
  return advdiff_ipc_signal_ch(c, 0, peers, n, stream);
}

extern "C" int advdiff_ipc_wait(advdiff_ipc* c, const int* peers, int n, void* stream) {
  return advdiff_ipc_wait_ch(c, 0, peers, n, stream);
}

// Close every peer mapping except the flag blocks (call with no put in flight,
// collectively): a peer's field freed and reallocated may come back under a handle whose
// cached mapping still names the old allocation.
extern "C" int advdiff_ipc_reset(advdiff_ipc* c) {
  if (c == nullptr) return hipErrorInvalidValue;
  hipError_t e = hipDeviceSynchronize();
  std::lock_guard<std::mutex> g(c->mu);
  for (auto it = c->opened.begin(); it != c->opened.end();) {
    bool flags = false;  // a peer's flag block: keep it (the counters live there)
    // (a peer's block is as large as ours: same world size)
    for (uint64_t* blk : c->peer_block)
      if (blk && (char*)blk >= (char*)it->second &&
          (char*)blk < (char*)it->second + c->block_bytes)
        flags = true;
    if (flags) {
      ++it;
      continue;
    }
    const hipError_t ec = hipIpcCloseMemHandle(it->second);
    if (e == hipSuccess) e = ec;
    it = c->opened.erase(it);
  }
  // (the exported handles stay: a live allocation cannot be exported twice, and
  // advdiff_ipc_describe replaces the handle of a reallocated one)
  return e;
}

// wait timeouts so far (synchronous read: call at a sync point)
extern "C" int advdiff_ipc_errors(advdiff_ipc* c, long long* timeouts) {
  if (c == nullptr || timeouts == nullptr) return hipErrorInvalidValue;
  unsigned long long h = 0;
  const hipError_t e = hipMemcpy(&h, c->err(), sizeof(h), hipMemcpyDeviceToHost);
  *timeouts = (long long)h;
  return e;
}
