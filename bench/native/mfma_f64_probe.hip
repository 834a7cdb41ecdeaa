// Probe: fp64 throughput of the matrix pipe (v_mfma_f64_16x16x4_f64) vs the vector pipe
// (v_fma_f64) on one MI355X — the number behind "stencils stay on the VALU"
// (docs/DESIGN.md §"Why no MFMA").  Each wave runs independent accumulator chains so the
// pipes, not the dependency latency, bound the rate.  Prints TFLOP/s for both.
//   hipcc --offload-arch=gfx950 -O3 mfma_f64_probe.hip -o mfma_f64_probe && ./mfma_f64_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void mfma_kernel(double* out, double a0, double b0) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = a0 + threadIdx.x * 1e-9, b = b0;
  for (int i = 0; i < kIters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  const d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + s.z + s.w;
}

__global__ __launch_bounds__(256) void fma_kernel(double* out, double a0, double b0) {
  double c[8];
  for (int j = 0; j < 8; ++j) c[j] = j;
  const double a = a0 + threadIdx.x * 1e-9, b = b0;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(a, c[j], b);
  double s = 0;
  for (int j = 0; j < 8; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8, threads = 256;
  double* out = nullptr;
  (void)hipMalloc(&out, sizeof(double) * blocks * threads);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    float ms_m = 0, ms_v = 0;
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_kernel, dim3(blocks), dim3(threads), 0, 0, out, 1.0, 1e-3);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms_m, e0, e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(fma_kernel, dim3(blocks), dim3(threads), 0, 0, out, 0.999, 1e-3);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms_v, e0, e1);
    // one 16x16x4 f64 MFMA = 16*16*4 MACs per wave; 4 per iteration per wave
    const double waves = blocks * (threads / 64.0);
    const double mflop = waves * kIters * 4 * (16.0 * 16 * 4) * 2;
    const double vflop = blocks * (double)threads * kIters * 8 * 2;
    std::printf("{\"cus\": %d, \"mfma_f64_tflops\": %.1f, \"valu_fma_f64_tflops\": %.1f, "
                "\"mfma_ms\": %.3f, \"valu_ms\": %.3f}\n",
                p.multiProcessorCount, mflop / (ms_m * 1e-3) / 1e12, vflop / (ms_v * 1e-3) / 1e12,
                ms_m, ms_v);
  }
  (void)hipFree(out);
  return 0;
}
