// abcd_feat.hip -- GPU featurisation straight into the packed layout.
//
// Reference data path (per item, on the host, every epoch):
//   Dataset.__getitem__  (data_utils.py:88-103): int16 samples -> float32, no scaling
//   STFT.__call__        (data_utils.py:124-139): torch.stft(n_fft = frame_length,
//                        hop, window, center) -> |.| -> (time, freq)
//   log_and_normalize    (learning.py:466-470):  log(x + eps) / norm
//   DataLoader.__next__  (data_utils.py:165-182): sort by length (desc),
//                        pack_sequence, is_offset = 1 at each last frame
// Here one launch does all of it for a whole batch on the device: a
// workgroup owns 16 frames of one segment, stages their (reflect-padded)
// samples x window in LDS, evaluates the one-sided DFT bins with a twiddle
// table (angle index (f*k) mod n_fft kept incrementally, any n_fft), and
// writes log(|X| + eps) / norm to row off_t + b of the packed output (b = the
// segment's rank in the length-sorted batch), plus is_offset.  HBM-bound
// work apart from the DFT's n_fft MACs per bin; no GEMM reshaping.
#include <cmath>
#include <mutex>
#include <vector>

#include "abcd_common.h"
#include "abcd_internal.h"
#include "abcd_persist.h"

namespace abcd {

constexpr int FT_FRAMES = 16;  // frames per workgroup

struct FeatArgs {
  const float* wave;        // concatenated samples
  const int* seg;           // device: [B][3] = sample offset (lo, hi), length (packed order)
  const int* nfr;           // device: frames per segment
  const int* off;           // device: packed step offsets off[0..T]
  const float* window;      // n_fft
  const double* tw;         // twiddles: cos(2 pi j / n), sin(2 pi j / n), j < n  (2n doubles)
  int n, hop, center, F, tiles;
  float eps, inv_norm;
  float* out;               // L x F
  float* is_offset;         // L, or null
};

__global__ __launch_bounds__(256) void featurize_packed(FeatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int n = a.n, F = a.F;
  const int b = blockIdx.y, f0 = blockIdx.x * FT_FRAMES;
  const int nf = a.nfr[b];
  if (f0 >= nf) return;
  const int nfb = min(FT_FRAMES, nf - f0);
  const long long s0 = (long long)(unsigned)a.seg[3 * b] | ((long long)a.seg[3 * b + 1] << 32);
  const long long len = a.seg[3 * b + 2];
  double* cs = reinterpret_cast<double*>(fsm);  // [n] cos
  double* sn = cs + n;                           // [n] sin
  double* xw = sn + n;                           // [FT_FRAMES][n] windowed frames (exact products)
  for (int j = threadIdx.x; j < n; j += 256) {
    cs[j] = a.tw[j];
    sn[j] = a.tw[n + j];
  }
  const int pad = a.center ? n / 2 : 0;
  for (int e = threadIdx.x; e < nfb * n; e += 256) {
    const int fr = e / n, k = e - fr * n;
    long long idx = (long long)(f0 + fr) * a.hop + k - pad;  // torch.stft reflect padding
    if (idx < 0) idx = -idx;
    if (idx >= len) idx = 2 * (len - 1) - idx;
    xw[fr * n + k] = (double)a.wave[s0 + idx] * (double)a.window[k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nfb * F; e += 256) {
    const int fr = e / F, f = e - fr * F;
    const double* x = xw + fr * n;
    // fp64 throughout: the exact DFT of the fp32 samples x fp32 window, rounded
    // once -- at or below torch's own fp32-FFT error
    double re = 0.0, im = 0.0;
    int j = 0;  // (f * k) mod n
    for (int k = 0; k < n; ++k) {
      re = fma(x[k], cs[j], re);
      im = fma(x[k], sn[j], im);
      j += f;
      if (j >= n) j -= n;
    }
    const float mag = (float)sqrt(re * re + im * im);
    const int t = f0 + fr;
    const long row = (long)a.off[t] + b;
    a.out[row * F + f] = logf(mag + a.eps) * a.inv_norm;
    if (f == 0 && a.is_offset) a.is_offset[row] = t == nf - 1 ? 1.f : 0.f;
  }
}

// n_fft-point twiddle table per (device, n), built once on the host in double
static int twiddles(hipStream_t s, int n, const double** out) {
  static std::mutex mu;
  static std::vector<std::pair<long, double*>> cache;  // key: device * 2^20 + n
  int dev = 0;
  ABCD_TRY(hipGetDevice(&dev));
  const long key = (long)dev * (1L << 20) + n;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& kv : cache)
    if (kv.first == key) {
      *out = kv.second;
      return 0;
    }
  std::vector<double> h(2 * (size_t)n);
  for (int j = 0; j < n; ++j) {
    const double ang = 2.0 * M_PI * (double)j / (double)n;
    h[j] = std::cos(ang);
    h[n + j] = std::sin(ang);
  }
  double* d = nullptr;
  ABCD_TRY(hipMalloc((void**)&d, h.size() * sizeof(double)));
  ABCD_TRY(hipMemcpy(d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  cache.push_back({key, d});
  *out = d;
  (void)s;
  return 0;
}

}  // namespace abcd

using namespace abcd;

extern "C" int abcd_stft_frames(long long length, int n_fft, int hop, int center) {
  if (n_fft <= 0 || hop <= 0 || length <= 0) return 0;
  const long long padded = center ? length + 2 * (n_fft / 2) : length;
  if (padded < n_fft) return 0;
  return (int)(1 + (padded - n_fft) / hop);
}

extern "C" size_t abcd_featurize_workspace_bytes(int B, int T) { return ((size_t)T + 1 + 4 * (size_t)B) * 4 + 256; }

extern "C" int abcd_featurize_packed(const float* wave, const long long* seg_off, const long long* seg_len, int B,
                                     int n_fft, int hop, int center, const float* window, float eps, float norm,
                                     const int64_t* batch_sizes, int T, int L, float* out, float* is_offset, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (!wave || !seg_off || !seg_len || B <= 0 || n_fft <= 1 || hop <= 0 || !window || !batch_sizes || T <= 0 ||
      !out || !ws || norm == 0.f)
    return ABCD_EINVAL;
  if (ws_bytes < abcd_featurize_workspace_bytes(B, T)) return ABCD_EINVAL;
  const int F = n_fft / 2 + 1;
  const size_t lds = ((size_t)FT_FRAMES + 2) * n_fft * sizeof(double);
  if (lds > 160 * 1024) return ABCD_EINVAL;
  ABCD_REQUIRE(validate_batch(batch_sizes, T, L, B) == 0);
  // host-side layout, one int table uploaded through the pinned ring:
  // off[0..T] | frames per segment [B] | (offset lo, offset hi, length) [B]
  // frames must be non-increasing in packed order and agree with batch_sizes
  std::vector<int> tab((size_t)T + 1 + 4 * (size_t)B, 0);
  int* off = tab.data();
  int* nfr = off + T + 1;
  int* seg = nfr + B;
  for (int b = 0; b < B; ++b) {
    if (seg_len[b] <= (center ? n_fft / 2 : 0) || seg_len[b] >= (1LL << 31) || seg_off[b] < 0) return ABCD_EINVAL;
    seg[3 * b] = (int)(uint32_t)(seg_off[b] & 0xffffffffLL);
    seg[3 * b + 1] = (int)(seg_off[b] >> 32);
    seg[3 * b + 2] = (int)seg_len[b];
    nfr[b] = abcd_stft_frames(seg_len[b], n_fft, hop, center);
    if (nfr[b] <= 0 || nfr[b] > T || (b > 0 && nfr[b] > nfr[b - 1])) return ABCD_EINVAL;
  }
  if (nfr[0] != T) return ABCD_EINVAL;
  for (int t = 0; t < T; ++t) {
    int cnt = 0;
    for (int b = 0; b < B; ++b) cnt += nfr[b] > t;
    if (cnt != (int)batch_sizes[t]) return ABCD_EINVAL;
    off[t + 1] = off[t] + cnt;
  }
  hipStream_t s = (hipStream_t)stream;
  int* dtab = (int*)ws;
  ABCD_TRY((hipError_t)upload_offsets(s, tab, dtab));
  const double* tw = nullptr;
  ABCD_TRY((hipError_t)twiddles(s, n_fft, &tw));
  FeatArgs a{wave, dtab + T + 1 + B, dtab + T + 1, dtab, window, tw, n_fft, hop, center, F, 0, eps, 1.0f / norm, out,
             is_offset};
  ABCD_TRY(hipFuncSetAttribute((const void*)featurize_packed, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024));
  featurize_packed<<<dim3(cdiv(T, FT_FRAMES), B), 256, lds, s>>>(a);
  ABCD_CHECK_LAUNCH();
  return 0;
}
