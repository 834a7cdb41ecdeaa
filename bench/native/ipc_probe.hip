// Standalone probes for the multi-rank device path (run on the GPU box):
//
//   ipc_probe memset <trials>
//       Is a synchronous hipMemset on the null stream ordered before work that is then
//       launched on a hipStreamNonBlocking stream?  (The native engine used to zero its
//       fields that way and then write the initial condition on such a stream.)  Each
//       trial: fill a 512 MiB buffer with 2, hipMemset(0) on the null stream, at once a
//       kernel on the non-blocking stream writes 1 everywhere, sync, count cells != 1.
//       Control: the same with hipMemsetAsync on the non-blocking stream.
//
//   ipc_probe ipc <rank 0|1> <dir> <iters> <put: 0 memcpy | 1 kernel>
//       Two processes on ONE GPU: each exports a data buffer and a flag block with
//       hipIpcGetMemHandle, opens the peer's, and per iteration puts a block into the
//       peer's buffer (hipMemcpyAsync D2D or a copy kernel), raises the peer's flag with a
//       release store (signal kernel), waits for its own flag with an acquire spin (wait
//       kernel, bounded), verifies the received block on the device and acknowledges it.
//       Everything is stream ordered: the host never waits inside the loop.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x,              \
                   hipGetErrorString(e_));                                           \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

__global__ void fill(double* p, size_t n, double v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void count_ne(const double* p, size_t n, double v, unsigned long long* c) {
  unsigned long long k = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    k += p[i] != v;
  if (k) atomicAdd(c, k);
}

__global__ void copyk(double* __restrict__ d, const double* __restrict__ s, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

// release store of v into a (possibly peer-process) flag
__global__ void signal_k(uint64_t* flag, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// acquire spin until *flag >= v; bounded (every wave exits): a timeout counts in err
__global__ void wait_k(const uint64_t* flag, uint64_t v, unsigned long long* err) {
  if (threadIdx.x == 0) {
    uint64_t n = 0;
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
      __builtin_amdgcn_s_sleep(8);
      if (++n > (1ull << 25)) {
        atomicAdd(err, 1ull);
        break;
      }
    }
  }
}

static int memset_probe(int trials) {
  const size_t n = (512ull << 20) / 8;
  double* buf = nullptr;
  unsigned long long* cnt = nullptr;
  CK(hipMalloc(&buf, n * 8));
  CK(hipMalloc(&cnt, 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int variant = 0; variant < 2; ++variant) {
    int bad = 0;
    double call_us = 0, max_call_us = 0;
    unsigned long long worst = 0;
    for (int t = 0; t < trials; ++t) {
      fill<<<4096, 256, 0, s>>>(buf, n, 2.0);
      CK(hipStreamSynchronize(s));
      CK(hipDeviceSynchronize());
      const double t0 = now();
      if (variant == 0)
        CK(hipMemset(buf, 0, n * 8));
      else
        CK(hipMemsetAsync(buf, 0, n * 8, s));
      const double dt = (now() - t0) * 1e6;
      call_us += dt;
      if (dt > max_call_us) max_call_us = dt;
      fill<<<4096, 256, 0, s>>>(buf, n, 1.0);
      CK(hipStreamSynchronize(s));
      CK(hipDeviceSynchronize());
      CK(hipMemsetAsync(cnt, 0, 8, s));
      count_ne<<<4096, 256, 0, s>>>(buf, n, 1.0, cnt);
      unsigned long long h = 0;
      CK(hipMemcpyAsync(&h, cnt, 8, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      if (h) ++bad;
      if (h > worst) worst = h;
    }
    std::printf("memset probe [%s]: %d of %d trials left cells != 1 (worst %llu of %zu); "
                "host call %.1f us mean, %.1f us max\n",
                variant == 0 ? "hipMemset on the null stream, kernel on a non-blocking stream"
                             : "hipMemsetAsync on the kernel's stream (control)",
                bad, trials, worst, n, call_us / trials, max_call_us);
  }
  return 0;
}

static void write_file(const std::string& path, const void* p, size_t n) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) std::exit(3);
  std::fwrite(p, 1, n, f);
  std::fclose(f);
  std::rename(tmp.c_str(), path.c_str());
}

static bool read_file(const std::string& path, void* p, size_t n) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  const size_t k = std::fread(p, 1, n, f);
  std::fclose(f);
  return k == n;
}

static void wait_file(const std::string& path, void* p, size_t n) {
  const double t0 = now();
  while (!read_file(path, p, n)) {
    if (now() - t0 > 60) {
      std::fprintf(stderr, "timeout waiting for %s\n", path.c_str());
      std::exit(4);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

static int ipc_probe(int rank, const std::string& dir, int iters, int put_kernel) {
  const int peer = 1 - rank;
  const size_t n = (16ull << 20) / 8;  // 16 MiB block
  double *data, *src;
  uint64_t* flags;  // [0..1]: data arrived from rank q; [2..3]: rank q consumed ours
  unsigned long long* err;
  CK(hipMalloc(&data, n * 8));
  CK(hipMalloc(&src, n * 8));
  CK(hipMalloc(&flags, 4096));
  CK(hipMalloc(&err, 16));
  CK(hipMemset(flags, 0, 4096));
  CK(hipMemset(err, 0, 16));
  CK(hipMemset(data, 0, n * 8));
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t h[2];
  CK(hipIpcGetMemHandle(&h[0], data));
  CK(hipIpcGetMemHandle(&h[1], flags));
  write_file(dir + "/h" + std::to_string(rank), h, sizeof(h));
  hipIpcMemHandle_t ph[2];
  wait_file(dir + "/h" + std::to_string(peer), ph, sizeof(ph));
  void *pdata_v = nullptr, *pflags_v = nullptr;
  const hipError_t e1 = hipIpcOpenMemHandle(&pdata_v, ph[0], hipIpcMemLazyEnablePeerAccess);
  const hipError_t e2 = hipIpcOpenMemHandle(&pflags_v, ph[1], hipIpcMemLazyEnablePeerAccess);
  std::printf("rank %d: hipIpcOpenMemHandle data -> %s, flags -> %s\n", rank,
              hipGetErrorString(e1), hipGetErrorString(e2));
  if (e1 != hipSuccess || e2 != hipSuccess) return 5;
  double* pdata = (double*)pdata_v;
  uint64_t* pflags = (uint64_t*)pflags_v;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const double t0 = now();
  for (int it = 1; it <= iters; ++it) {
    const double v = rank * 100000.0 + it;
    fill<<<1024, 256, 0, s>>>(src, n, v);
    if (it > 1) wait_k<<<1, 64, 0, s>>>(flags + 2 + peer, it - 1, err + 1);  // peer consumed
    if (put_kernel)
      copyk<<<1024, 256, 0, s>>>(pdata, src, n);
    else
      CK(hipMemcpyAsync(pdata, src, n * 8, hipMemcpyDeviceToDevice, s));
    signal_k<<<1, 64, 0, s>>>(pflags + rank, it);
    wait_k<<<1, 64, 0, s>>>(flags + peer, it, err + 1);
    count_ne<<<1024, 256, 0, s>>>(data, n, peer * 100000.0 + it, err);
    signal_k<<<1, 64, 0, s>>>(pflags + 2 + rank, it);
  }
  CK(hipStreamSynchronize(s));
  const double dt = now() - t0;
  unsigned long long he[2];
  CK(hipMemcpy(he, err, 16, hipMemcpyDeviceToHost));
  std::printf("rank %d: %d iterations (%s put of %zu MiB): %llu wrong cells, %llu wait "
              "timeouts, %.1f us per iteration\n",
              rank, iters, put_kernel ? "kernel" : "hipMemcpyAsync", n * 8 >> 20, he[0], he[1],
              dt / iters * 1e6);
  // both done before anyone unmaps / frees
  int one = 1;
  write_file(dir + "/done" + std::to_string(rank), &one, sizeof(one));
  wait_file(dir + "/done" + std::to_string(peer), &one, sizeof(one));
  CK(hipIpcCloseMemHandle(pdata_v));
  CK(hipIpcCloseMemHandle(pflags_v));
  CK(hipDeviceSynchronize());
  return (he[0] || he[1]) ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && !std::strcmp(argv[1], "memset"))
    return memset_probe(argc > 2 ? std::atoi(argv[2]) : 20);
  if (argc >= 6 && !std::strcmp(argv[1], "ipc"))
    return ipc_probe(std::atoi(argv[2]), argv[3], std::atoi(argv[4]), std::atoi(argv[5]));
  std::fprintf(stderr, "usage: ipc_probe memset [trials] | ipc <rank> <dir> <iters> <put>\n");
  return 1;
}
