// abcd_internal.h -- host-side helpers shared by the .hip translation units
// (not part of the C ABI; see include/abcd_hip.h for that).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <algorithm>

#include "abcd_hip.h"

namespace abcd {

#define ABCD_TRY(expr)                                   \
  do {                                                   \
    hipError_t e__ = (expr);                             \
    if (e__ != hipSuccess) return (int)e__;              \
  } while (0)
#define ABCD_CHECK_LAUNCH() ABCD_TRY(hipGetLastError())
#define ABCD_REQUIRE(cond)                               \
  do {                                                   \
    if (!(cond)) return ABCD_EINVAL;                     \
  } while (0)

enum Act { ACT_NONE = 0, ACT_TANH = 1 };

struct Operand {
  const float* p;
  long ld;
  int nrows;    // rows beyond this read as zero
  bool kmajor;  // false: (row,k) at p[row*ld+k] (K must be a multiple of 16); true: at p[k*ld+row]
};

inline Operand opKC(const float* p, long ld, int nrows) { return Operand{p, ld, nrows, false}; }
inline Operand opKM(const float* p, long ld, int nrows) { return Operand{p, ld, nrows, true}; }

// C[m][n] = alpha * sum_k A(m,k) B(n,k) + beta * C[m][n] + bias[n], then act.
// Stores rows < M, cols < N.  `scratch` (may be null) enables split-K slabs.
// One launch for up to GEMM_BATCH_MAX small GEMMs whose operands are both
// K-major (the batch-reduction weight gradients, K = the batch's rows):
// C_j = alpha_j A_j^T B_j + beta_j C_j, A_j element (m, k) at A[k * lda + m],
// B_j element (n, k) at B[k * ldb + n]; no split-K slabs, no second pass.
constexpr int GEMM_BATCH_MAX = 8;
struct GemmJob {
  const float* A; long lda;
  const float* B; long ldb;
  float* C; long ldc;
  int M, N, K;
  float alpha, beta;
};
int gemm_tn_batch(hipStream_t s, const GemmJob* jobs, int n);

int gemm(hipStream_t s, int M, int N, int K, Operand A, Operand B, float* C, long ldc, float alpha,
         float beta, const float* bias, int act, float* scratch, size_t scratch_floats);

// The decoder's offset head (model.py:121-122,191,195) folded into its two
// frame-parallel GEMMs (gemm_x6r8, 64-column slices):
//   forward:  Zo = tanh(Hs W1o^T + b1o) (M x N, K = H) and part[m * nsl + slice]
//             = the slice's share of Zo . w2 (nsl = offset_head_slices(N));
//   backward: DHO = dZo W1o with dZo = s dlog_raw (1 - Zo^2) w2 formed from Zo
//             while its fragments load (M x N, K = Hm); dZo (ld = K) and
//             dlog_s = s dlog_raw are stored on the way.
// Both return 0 with *done = false where the fused form does not apply (the
// caller then runs the separate kernels).
int offset_head_slices(int N);
int gemm_offset_fwd(hipStream_t s, int M, int N, int K, const float* Hs, long ldh, const float* W1o,
                    const float* b1o, float* Zo, const float* w2, float* part, bool* done);
int gemm_offset_bwd(hipStream_t s, int M, int N, int K, const float* Zo, const float* W1oT, float* DHO,
                    const float* w2, const float* dlog_raw, const float* s_off, float* dZo, float* dlog_s,
                    bool* done);

// A B^T (both K-contiguous) as raw split-K slabs slab[z][m*N + n], z < *zout.
int gemm_slabs(hipStream_t s, int M, int N, int K, Operand A, Operand B, float* slab, size_t slab_floats, int* zout);

// out[j] (+)= sum_r w[r] * Z[r*ldz + j]  (w == null -> 1), j < ncols, r < nrows; deterministic.
// out2 (optional) receives the same sum with the same beta (e.g. b_ih and b_hh of an LSTM).
// several colsum() jobs in one pass-1 + one pass-2 launch (each job sliced
// exactly as colsum() slices it: the same sums); scratch holds every job's
// partials (at most 256 x ncols each)
constexpr int COLSUM_BATCH_MAX = 8;
struct ColsumJob {
  const float* Z; long ldz; int nrows, ncols;
  const float* w;     // row weights, or null
  float* out; float beta;
  float* out2;        // a second destination, or null
};
int colsum_batch(hipStream_t s, const ColsumJob* jobs, int n, float* scratch, size_t scratch_floats);
int colsum(hipStream_t s, const float* Z, long ldz, int nrows, int ncols, const float* w, float* out,
           float beta, float* scratch, size_t scratch_floats, float* out2 = nullptr);

// dst[r*ldd + c] = (r < sr && c < sc) ? src(r, c) : 0 for r < dr, c < dc;
// src(r,c) = trans ? src[c*lds + r] : src[r*lds + c]
int pack2d(hipStream_t s, const float* src, long lds, int sr, int sc, bool trans, float* dst, long ldd,
           int dr, int dc);

// y = a + b elementwise (n floats)
int add_vec(hipStream_t s, const float* a, const float* b, float* y, int n);
// y = a * b elementwise (n floats; y may alias a)
int mul_vec(hipStream_t s, const float* a, const float* b, float* y, long n);

// A queue of pack2d jobs (optionally dst = src + src2, same layout) issued as
// one launch by flush() -- or earlier, when the queue is full.  ones: column sc
// of rows < sr is 1 instead of 0 (the encoder's [X | 1] frame copy).
constexpr int ABCD_PACK_MAX = 24;
struct PackJob {
  const float *src, *src2;
  long lds;
  float* dst;
  long ldd;
  int sr, sc, dr, dc, trans, ones;
};
struct PackList {
  PackJob j[ABCD_PACK_MAX];
  int n;
};
struct Packs {
  hipStream_t s;
  PackList pl;
  long maxn;
  explicit Packs(hipStream_t st) : s(st), pl{}, maxn(0) {}
  int add(const float* src, long lds, int sr, int sc, bool trans, float* dst, long ldd, int dr, int dc,
          const float* src2 = nullptr, bool ones = false);
  int flush();
};

// Sum of n doubles/floats -> out (device), deterministic two-pass.
int reduce_sum(hipStream_t s, const float* x, long n, double* partials, float* out, double* out64);

size_t gemm_scratch_floats_hint(int M, int N, int K);

// The layer-0 LSTM encoder weight gradients of nd <= 2 directions in one
// launch (gemm_wg2 + one slab reduction): direction d gets
// w_ih = dG^T X[:, :F], b_ih (and b_hh when set) = dG^T X[:, F] (X's column F
// holds 1), w_hh = dG^T Hprev; dG: K x M (ld M), X: K x Fp (ld Fp), Hprev: K x H
// (ld H).  Returns -1 when the shape has no instance (the caller falls back to
// gemm()), 0 on success, else a hipError_t.
struct WgDir {
  const float *dG, *X, *Hprev;
  float *w_ih, *b_ih, *b_hh, *w_hh;
};
struct WgArgs {
  const float* A[2];
  const float* B1[2];
  const float* B2[2];
  long lda, ldb1, ldb2;
  int M, K, kps, Z;
  float* slab;
};
struct WgOut {
  float* w_ih[2];
  float* b_ih[2];
  float* b_hh[2];
  float* w_hh[2];
};
bool wg3_on();  // gemm_wg3 (default) or gemm_wg2 for the layer-0 LSTM weight gradients
const char* wg_dispatch_fmt();  // "gemm_wg3b<%d,%d> x%d" etc.: the form wgrad_lstm_l0 runs
int wgrad_lstm_l0(hipStream_t s, int nd, const WgDir* dirs, int M, int K, int F, int Fp, int H, float* scratch,
                  size_t scratch_floats);

// While alive (on this host thread), GEMMs use the co-residency-friendly
// "side stream" tiling: see abcd_gemm.hip.
// diagnostics (abcd_debug_persist_prof): the stamp buffer when `bit` is set in its mask, else null
unsigned long long* debug_prof_buf(int bit);

struct GemmSideScope {
  int prev;
  explicit GemmSideScope(bool on);
  ~GemmSideScope();
};

// `to` waits for everything queued on `from` so far (a reusable per-device
// event per slot, re-recorded each call).  No-op when from == to.
int stream_fork(hipStream_t from, hipStream_t to, int slot);

}  // namespace abcd

namespace abcd {
// Bump allocator used to carve a caller-provided workspace.  The same carve
// sequence runs with base == nullptr to size the workspace.
struct Arena {
  char* base;
  size_t off, cap;
  bool ok;
  explicit Arena(void* b, size_t c) : base((char*)b), off(0), cap(c), ok(true) {}
  float* f(size_t n) {
    off = (off + 255) & ~(size_t)255;
    char* p = base ? base + off : nullptr;
    off += n * sizeof(float);
    if (base && off > cap) ok = false;
    return (float*)p;
  }
  double* d(size_t n) { return (double*)f(2 * n); }
};

// checks PackedSequence.batch_sizes (host): non-increasing, sum L, first B
int validate_batch(const int64_t* bs, int T, int L, int B);
}  // namespace abcd

namespace abcd {
// Optional live timing of the recurrent kernel family (bench.py roofline):
// when enabled, a HIP event pair brackets every launch inside TimedScope,
// tagged with the kernel id (TK_*) so one kernel can be read back alone.
enum TimedKernel {
  TK_STEP = 0, TK_ENC_FWD = 1, TK_ENC_BWD = 2, TK_DEC_FWD = 3, TK_DEC_BWD = 4,
  TK_SAMP_FWD = 5, TK_SAMP_BWD = 6,  // dispatch records only (no live timing)
  TK_ENC_WGRAD = 7,                  // the encoder's layer-0 weight-gradient route (dispatch record)
  TK_N = 8
};
bool timing_on();
void timing_mark(hipStream_t s, int kid);
// records which kernel (template instance) a role's last launch ran, so the
// tests can assert that the production-shape dispatch is the one checked
// against the reference (abcd_dispatch_name / abcd_dispatch_count)
void note_dispatch(int kid, const char* fmt, ...);
struct TimedScope {
  hipStream_t s;
  bool on;
  int kid;
  explicit TimedScope(hipStream_t st, int k = TK_STEP) : s(st), on(timing_on()), kid(k) { if (on) timing_mark(s, kid); }
  ~TimedScope() { if (on) timing_mark(s, kid); }
};
}  // namespace abcd
