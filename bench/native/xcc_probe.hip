// Which XCD runs which workgroup?  Launches grids shaped like the fused heat step's
// (1024 threads, ~105 KB LDS -> one workgroup per CU; and 768 threads / ~80 KB -> two) and
// records HW_REG_XCC_ID per block (one lane, vector store).  Prints how often
// xcc == (b + c) % 8 for the best constant c, i.e. whether blocks are dealt round-robin
// over the XCDs as xcd_tile (csrc/kernels/common.hpp) assumes.
//   hipcc --offload-arch=gfx950 -O2 bench/native/xcc_probe.hip -o bench/native/xcc_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void probe(int* out, int spin) {
  extern __shared__ double lds[];
  const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  lds[threadIdx.x] = (double)b;  // touch the LDS allocation
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    // HW_REG_XCC_ID (id 20), bits [3:0]
    const int xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    out[b] = xcc + (int)lds[1] * 0;
  }
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(8);  // keep the CU busy
}

static int run(int gx, int gy, int gz, int threads_y, size_t lds_bytes) {
  const int n = gx * gy * gz;
  int* d = nullptr;
  CHECK(hipMalloc(&d, n * sizeof(int)));
  CHECK(hipMemset(d, 0xff, n * sizeof(int)));
  CHECK(hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_bytes));
  hipLaunchKernelGGL(probe, dim3(gx, gy, gz), dim3(64, threads_y, 1), lds_bytes, 0, d, 2000);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::vector<int> h(n);
  CHECK(hipMemcpy(h.data(), d, n * sizeof(int), hipMemcpyDeviceToHost));
  CHECK(hipFree(d));
  int best = 0, bestc = 0;
  for (int c = 0; c < 8; ++c) {
    int m = 0;
    for (int b = 0; b < n; ++b) m += h[b] == (b + c) % 8;
    if (m > best) best = m, bestc = c;
  }
  int per[8] = {0};
  for (int b = 0; b < n; ++b)
    if (h[b] >= 0 && h[b] < 8) per[h[b]]++;
  std::printf("grid %dx%dx%d, %d threads, %zu B LDS: %d of %d blocks on XCC (b + %d) %% 8;"
              " per XCC:", gx, gy, gz, 64 * threads_y, lds_bytes, best, n, bestc);
  for (int i = 0; i < 8; ++i) std::printf(" %d", per[i]);
  std::printf("\n  first 32:");
  for (int b = 0; b < 32 && b < n; ++b) std::printf(" %d", h[b]);
  std::printf("\n");
  return 0;
}

int main() {
  if (run(10, 22, 1, 16, 105 * 1024)) return 1;  // FD4 step shape, one block per CU
  if (run(9, 16, 3, 12, 78 * 1024)) return 1;    // FD2 step shape, two per CU
  if (run(5, 32, 5, 8, 40 * 1024)) return 1;     // a Burgers-like launch
  if (run(64, 64, 1, 4, 0)) return 1;            // many small blocks
  return 0;
}
