// Diagnostics: issue rate of v_mfma_f32_16x16x4_f32 vs v_mfma_f32_16x16x32_bf16
// in a loop shaped like the persistent kernels' inner loop (4 accumulators,
// B fragments from LDS), on every CU.  Prints ticks (s_memtime) per MFMA and
// the in-kernel clock (s_memtime / s_memrealtime x 100 MHz).
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_mfma.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(256) void kern(float* out, unsigned long long* t, int iters) {
  __shared__ f4 lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = f4{0.001f * i, 1.f, 2.f, 3.f};
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f4 acc[4] = {};
  f4 a = {1.f * lane, 2.f, 3.f, 4.f};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    f4 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = lds[(it * 4 + j) % 64 * 64 + lane];
    if (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[j][s], acc[j], 0, 0, 0);
    } else {
      bf8 av, bv[4];
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = (__bf16)a[e & 3];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[j][e] = (__bf16)b[j][e & 3];
      // 6 products per (chunk of 32 K, subtile): the bf16x6 split-fp32 form
#pragma unroll
      for (int s = 0; s < 6; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[j], acc[j], 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    t[blockIdx.x * 2] = t1 - t0;
    t[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int MODE>
void run(const char* name, int mfma_per_iter, double flop_per_mfma) {
  const int grid = 256, iters = 4096;
  float* out;
  unsigned long long* t;
  hipMalloc(&out, grid * 256 * 4);
  hipMalloc(&t, grid * 16);
  kern<MODE><<<grid, 256>>>(out, t, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  kern<MODE><<<grid, 256>>>(out, t, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(grid * 2);
  hipMemcpy(h.data(), t, grid * 16, hipMemcpyDeviceToHost);
  double ticks = 0, real = 0;
  for (int b = 0; b < grid; ++b) { ticks += h[2 * b]; real += h[2 * b + 1]; }
  ticks /= grid;
  real /= grid;
  const double n = (double)iters * mfma_per_iter;
  const double flops = n * flop_per_mfma * 4 /*waves*/ * grid;
  printf("%s: %.1f ticks/MFMA, clock %.2f GHz, %.1f TFLOP/s (event %.3f ms)\n", name, ticks / n,
         ticks / real * 0.1, flops / (ms * 1e-3) / 1e12, ms);
  hipFree(out);
  hipFree(t);
}

int main() {
  run<0>("f32 16x16x4 ", 16, 2.0 * 16 * 16 * 4);
  run<1>("bf16 16x16x32 (x6)", 24, 2.0 * 16 * 16 * 32);
  return 0;
}
