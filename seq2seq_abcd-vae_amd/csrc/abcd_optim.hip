// abcd_optim.hip -- clip_grad_norm_ + SGD over the flat fp32 parameter buffer
// (ABCD-VAE/learning.py:161-163,256), the step loss (learning.py:155-157) and
// the Philox noise generator used when noise is not supplied by the host.
//
// The whole model's parameters (1.95 M fp32 at the north-star config) live in
// ONE flat buffer, gradients in a second one: the global norm is a single
// deterministic two-pass reduction and the update is one streaming pass
// (read g, p[, buf]; write g, p[, buf]) -- HBM-bound, ~24-40 B per parameter.
#include "abcd_common.h"
#include "abcd_internal.h"

namespace abcd {

// global norm in one launch: each block's partial sum of squares (fp64) is
// stored write-through and the last block to finish (last_workgroup) sums
// them in a fixed order (thread-strided, shuffle tree, waves): deterministic.
// state[0] = norm, state[1] = clip coefficient
__device__ unsigned g_norm_ticket;
__global__ void sq_norm(const float* g, long n, double* part, float max_norm, float* state, float* out_norm) {
  __shared__ double sh[16];
  __shared__ int last;
  double v = 0.0;
  const long n4 = n / 4;
  const f4* g4 = reinterpret_cast<const f4*>(g);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f4 x = g4[i];
    v += (double)x[0] * x[0] + (double)x[1] * x[1] + (double)x[2] * x[2] + (double)x[3] * x[3];
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    v += (double)g[i] * g[i];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    st_agent(&part[blockIdx.x], t);
  }
  if (!last_workgroup(&g_norm_ticket, &last)) return;
  v = 0.0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) v += ld_agent(&part[i]);
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    const float norm = (float)sqrt(t);
    state[0] = norm;
    state[1] = fminf(max_norm / (norm + 1e-6f), 1.0f);
    if (out_norm) *out_norm = norm;
  }
}
__global__ void sgd_update(float* p, float* g, float* buf, long n, const float* state, float lr, float momentum,
                           int init) {
  const float coef = state[1];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gi = g[i] * coef;
    g[i] = gi;
    if (buf) {
      const float b = init ? gi : momentum * buf[i] + gi;
      buf[i] = b;
      gi = b;
    }
    p[i] -= lr * gi;
  }
}

__global__ void total_loss_kernel(const float* losses, const float* kl, int B, float* loss) {
  if (threadIdx.x == 0) *loss = (losses[0] + losses[1] + kl[0]) / (float)B;
}

__global__ void fill_normal_kernel(float* out, long n, uint64_t seed, uint64_t offset) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = philox_normal(seed, offset + (uint64_t)i);
}

}  // namespace abcd

using namespace abcd;

// partial slots; sq_norm runs kSqBlocks of them (its hand-over ticket is one
// word: ~12 ns per serialized add, so 1024 blocks cost ~12 us, 256 ~3 us)
static const int kNormBlocks = 1024;
static const int kSqBlocks = 256;

extern "C" size_t abcd_optim_workspace_bytes(long n) {
  (void)n;
  return kNormBlocks * sizeof(double) + 256;
}

extern "C" int abcd_grad_norm(const float* g, long n, float* out_norm, void* ws, size_t ws_bytes, void* stream) {
  if (!g || n <= 0 || !out_norm || !ws || ws_bytes < abcd_optim_workspace_bytes(n)) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)ws;
  float* state = (float*)(part + kNormBlocks);
  sq_norm<<<kSqBlocks, 256, 0, s>>>(g, n, part, 1.f, state, out_norm);
  ABCD_CHECK_LAUNCH();
  return 0;
}

extern "C" int abcd_clip_sgd(float* p, float* g, float* momentum_buf, long n, float max_norm, float lr,
                             float momentum, int momentum_init, float* out_norm, void* ws, size_t ws_bytes,
                             void* stream) {
  if (!p || !g || n <= 0 || !ws || ws_bytes < abcd_optim_workspace_bytes(n)) return ABCD_EINVAL;
  if (momentum != 0.f && !momentum_buf) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)ws;
  float* state = (float*)(part + kNormBlocks);
  sq_norm<<<kSqBlocks, 256, 0, s>>>(g, n, part, max_norm, state, out_norm);
  ABCD_CHECK_LAUNCH();
  const int nb = (int)std::min<long>(4096, (n + 255) / 256);
  sgd_update<<<nb, 256, 0, s>>>(p, g, momentum != 0.f ? momentum_buf : nullptr, n, state, lr, momentum,
                                momentum_init);
  ABCD_CHECK_LAUNCH();
  return 0;
}

extern "C" int abcd_total_loss(const float* losses, const float* kl, int B, float* loss, void* stream) {
  if (!losses || !kl || !loss || B <= 0) return ABCD_EINVAL;
  total_loss_kernel<<<1, 64, 0, (hipStream_t)stream>>>(losses, kl, B, loss);
  ABCD_CHECK_LAUNCH();
  return 0;
}

extern "C" int abcd_fill_normal(float* out, long n, uint64_t seed, uint64_t offset, void* stream) {
  if (!out || n < 0) return ABCD_EINVAL;
  if (n == 0) return 0;
  fill_normal_kernel<<<(int)std::min<long>(4096, (n + 255) / 256), 256, 0, (hipStream_t)stream>>>(out, n, seed,
                                                                                                 offset);
  ABCD_CHECK_LAUNCH();
  return 0;
}

#include "abcd_srchash.h"
// fp32 arithmetic: split-fp32 "x6" products on the bf16 matrix cores
// (v_mfma_f32_16x16x32_bf16, abcd_x6.h) for the recurrences and the big GEMMs,
// exact-fp32 v_mfma_f32_16x16x4_f32 elsewhere; src = ABCD_SRC_HASH (Makefile)
extern "C" const char* abcd_version(void) {
  return "abcd_hip 0.4 gfx950 fp32 (split-bf16x6 mfma_16x16x32_bf16 + mfma_16x16x4_f32) src " ABCD_SRC_HASH;
}

// ---------------------------------------------------------------------------
// live kernel timing (bench.py): event pairs around recurrent-kernel launches
// ---------------------------------------------------------------------------
#include <cstdarg>
#include <cstdio>
#include <vector>
namespace abcd {
struct TimingState {
  bool on = false;
  std::vector<hipEvent_t> ev;  // begin, end, begin, end, ...
  std::vector<int> kid;        // kernel id of each event
  size_t used = 0;
};
static TimingState g_timing;
bool timing_on() { return g_timing.on; }
void timing_mark(hipStream_t s, int k) {
  if (g_timing.used == g_timing.ev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) { g_timing.on = false; return; }
    g_timing.ev.push_back(e);
    g_timing.kid.push_back(0);
  }
  g_timing.kid[g_timing.used] = k;
  (void)hipEventRecord(g_timing.ev[g_timing.used++], s);
}
static int timing_sum(int want, double* out) {
  double tot = 0.0, n = 0.0;
  const size_t pairs = g_timing.used / 2;
  if (pairs) ABCD_TRY(hipEventSynchronize(g_timing.ev[2 * pairs - 1]));
  for (size_t i = 0; i < pairs; ++i) {
    if (want >= 0 && g_timing.kid[2 * i] != want) continue;
    float ms = 0.f;
    ABCD_TRY(hipEventElapsedTime(&ms, g_timing.ev[2 * i], g_timing.ev[2 * i + 1]));
    tot += ms;
    n += 1.0;
  }
  out[0] = tot;
  out[1] = n;
  out[2] = out[3] = 0.0;
  return 0;
}
}  // namespace abcd

namespace abcd {
static char g_dispatch[TK_N][128];
static long g_dispatch_n[TK_N];
void note_dispatch(int kid, const char* fmt, ...) {
  if (kid < 0 || kid >= TK_N) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_dispatch[kid], sizeof(g_dispatch[kid]), fmt, ap);
  va_end(ap);
  ++g_dispatch_n[kid];
}
}  // namespace abcd

extern "C" const char* abcd_dispatch_name(int kid) {
  return (kid < 0 || kid >= abcd::TK_N) ? "" : abcd::g_dispatch[kid];
}
extern "C" long abcd_dispatch_count(int kid) { return (kid < 0 || kid >= abcd::TK_N) ? -1 : abcd::g_dispatch_n[kid]; }
extern "C" void abcd_dispatch_reset(void) {
  for (int k = 0; k < abcd::TK_N; ++k) {
    abcd::g_dispatch[k][0] = 0;
    abcd::g_dispatch_n[k] = 0;
  }
}

extern "C" void abcd_timing_enable(int on) { abcd::g_timing.on = on != 0; }
extern "C" void abcd_timing_reset(void) { abcd::g_timing.used = 0; }
/* out[0] = total device ms inside the timed launches, out[1] = launches */
extern "C" int abcd_timing_read(double* out) { return abcd::timing_sum(-1, out); }
/* the same restricted to one kernel id (0 per-step kernels, 1 encoder forward,
 * 2 encoder backward, 3 decoder forward, 4 decoder backward) */
extern "C" int abcd_timing_read_kernel(int kid, double* out) { return abcd::timing_sum(kid, out); }
