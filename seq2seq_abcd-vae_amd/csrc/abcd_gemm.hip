// abcd_gemm.hip -- fp32 MFMA GEMM and small reduction / layout kernels.
//
// Two GEMM shapes share the wave core of abcd_common.h:
//   gemm_big : 4 waves as 2x2, each wave 64x64 (4x4 subtiles), WG tile 128x128.
//              For the frame-parallel GEMMs (encoder input projection over all
//              L packed frames, batched offset MLP, decoder-input GEMMs).
//   gemm_ks  : 4 waves split K of one 32x64 tile, reduced through LDS.  For
//              small-M GEMMs (B = 512 rows) and for the weight-gradient GEMMs
//              whose reduction runs over the packed frames (K = L ~ 65k), where
//              the grid is also split along K into fp32 slabs that a second
//              pass reduces deterministically.
#include <numeric>
#include <cstdlib>
#include <cstdio>

#include "abcd_common.h"
#include <mutex>

#include "abcd_internal.h"
#include "abcd_x6.h"


namespace abcd {

// Side-stream mode (GemmSideScope): weight-gradient GEMMs that run beside a
// persistent recurrent kernel keep each workgroup small enough (LDS <= 34 KiB,
// <= 112 VGPRs) to co-reside with it, and their grids to <= one workgroup per
// CU, so they fill the SIMDs the latency-bound recurrence leaves idle instead
// of displacing its workgroups.
static thread_local int tl_side = 0;
GemmSideScope::GemmSideScope(bool on) : prev(tl_side) { tl_side = on ? 1 : prev; }  // off: keep the caller's mode
GemmSideScope::~GemmSideScope() { tl_side = prev; }

int stream_fork(hipStream_t from, hipStream_t to, int slot) {
  if (from == to) return 0;
  static std::mutex mu;
  static hipEvent_t evs[64][8] = {};
  int dev = 0;
  ABCD_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64 || slot < 0 || slot >= 8) return (int)hipErrorInvalidValue;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (!evs[dev][slot]) ABCD_TRY(hipEventCreateWithFlags(&evs[dev][slot], hipEventDisableTiming));
    ev = evs[dev][slot];
  }
  ABCD_TRY(hipEventRecord(ev, from));
  return (int)hipStreamWaitEvent(to, ev, 0);
}

struct EpiArgs {
  float* C; long ldc; int M, N; float alpha, beta; const float* bias; int act;
  float* slab;  // non-null when gridDim.z > 1: raw partials, slab[z][m*N + n]
};

DEV float apply_epi(const EpiArgs& e, int row, int col, float acc) {
  float v = e.alpha * acc;
  if (e.beta != 0.f) v += e.beta * e.C[(long)row * e.ldc + col];
  if (e.bias) v += e.bias[col];
  if (e.act == ACT_TANH) v = tanhf(v);
  return v;
}

template <int MR, int NR, class OA, class OB>
__global__ __launch_bounds__(256) void gemm_big_kernel(OA A, OB B, int nch, int cps, EpiArgs e) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * (32 * MR) + wm * 16 * MR;
  const int n0 = blockIdx.x * (32 * NR) + wn * 16 * NR;
  int ar[MR], br[NR];
#pragma unroll
  for (int i = 0; i < MR; ++i) ar[i] = m0 + 16 * i + r;
#pragma unroll
  for (int j = 0; j < NR; ++j) br[j] = n0 + 16 * j + r;
  f4 acc[MR][NR];
  acc_zero(acc);
  const int c0 = blockIdx.z * cps, c1 = min(nch, c0 + cps);
  wave_mma<MR, NR>(acc, A, ar, B, br, c0, c1, 1, q);
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = m0 + 16 * i + 4 * q + g, col = n0 + 16 * j + r;
        if (row < e.M && col < e.N) {
          if (e.slab)
            e.slab[(long)blockIdx.z * e.M * e.N + (long)row * e.N + col] = acc[i][j][g];
          else
            e.C[(long)row * e.ldc + col] = apply_epi(e, row, col, acc[i][j][g]);
        }
      }
}

template <int MR, int NR, class OA, class OB>
__global__ __launch_bounds__(256) void gemm_ks_kernel(OA A, OB B, int nch, int cps, EpiArgs e) {
  constexpr int TM = 16 * MR, TN = 16 * NR, LD = TN + 4;
  __shared__ __attribute__((aligned(16))) float lds[4 * TM * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  int ar[MR], br[NR];
#pragma unroll
  for (int i = 0; i < MR; ++i) ar[i] = m0 + 16 * i + r;
#pragma unroll
  for (int j = 0; j < NR; ++j) br[j] = n0 + 16 * j + r;
  f4 acc[MR][NR];
  acc_zero(acc);
  const int c0 = blockIdx.z * cps, c1 = min(nch, c0 + cps);
  wave_mma<MR, NR>(acc, A, ar, B, br, c0 + w, c1, 4, q);
  reduce_waves_to_lds<MR, NR>(acc, lds, w, lane);
  for (int t = threadIdx.x; t < TM * TN; t += 256) {
    const int lr = t / TN, lc = t % TN;
    const int row = m0 + lr, col = n0 + lc;
    if (row < e.M && col < e.N) {
      const float v = lds[lr * LD + lc];
      if (e.slab)
        e.slab[(long)blockIdx.z * e.M * e.N + (long)row * e.N + col] = v;
      else
        e.C[(long)row * e.ldc + col] = apply_epi(e, row, col, v);
    }
  }
}

// Sum of the Z raw split-K slabs + the epilogue.  A thread owns 4 consecutive
// outputs (one 16-B load per slab when the slabs are 16-B aligned) and keeps
// SR_DEPTH slabs' loads in flight, adding them in slab order (the same sum as
// a sequential loop): ~Z / SR_DEPTH memory round trips per thread instead of
// Z.  The one-output, one-load-at-a-time loop took 157 us for the 64-slab
// encoder dW_ih reduction at c2 (34 MB read at ~0.2 TB/s).
constexpr int SR_DEPTH = 8;
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* slab, int Z, EpiArgs e) {
  const long n = (long)e.M * e.N;
  const bool vec = (n % 4 == 0) && (((uintptr_t)slab & 15) == 0);
  const long nq = vec ? n / 4 : n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nq; i += (long)gridDim.x * blockDim.x) {
    f4 s = f4zero();
    for (int z0 = 0; z0 < Z; z0 += SR_DEPTH) {
      f4 v[SR_DEPTH];
#pragma unroll
      for (int k = 0; k < SR_DEPTH; ++k) {
        const long base = (long)(z0 + k) * n;
        if (z0 + k >= Z) v[k] = f4zero();
        else if (vec) v[k] = *reinterpret_cast<const f4*>(slab + base + 4 * i);
        else v[k] = f4{slab[base + i], 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int k = 0; k < SR_DEPTH; ++k) s += v[k];
    }
    const int cnt = vec ? 4 : 1;
    for (int t = 0; t < cnt; ++t) {
      const long j = vec ? 4 * i + t : i;
      const int row = (int)(j / e.N), col = (int)(j % e.N);
      e.C[(long)row * e.ldc + col] = apply_epi(e, row, col, s[t]);
    }
  }
}
// The same sum with the slabs split over ZG thread groups: a workgroup owns
// 256 / ZG output quads, group g adds the contiguous slab range g of each in
// slab order, and the ZG partials are added in group order through LDS
// (deterministic).  For many slabs over a small output (the emission MLPs'
// dW2: 129 x 256 outputs, 125 slabs) the one-group form ran 33 workgroups,
// each thread ~16 dependent round trips: 50-55 us for 16.5 MB.
template <int ZG>
__global__ __launch_bounds__(256) void slab_reduce_zg_kernel(const float* slab, int Z, EpiArgs e) {
  constexpr int QB = 256 / ZG;
  __shared__ f4 part[256];
  const long n = (long)e.M * e.N, nq = n / 4;
  const int g = threadIdx.x / QB, ql = threadIdx.x % QB;
  const long i = (long)blockIdx.x * QB + ql;
  const int zper = (Z + ZG - 1) / ZG, zb = g * zper, ze = min(Z, zb + zper);
  f4 s = f4zero();
  if (i < nq) {
    for (int z0 = zb; z0 < ze; z0 += SR_DEPTH) {
      f4 v[SR_DEPTH];
#pragma unroll
      for (int k = 0; k < SR_DEPTH; ++k)
        v[k] = z0 + k < ze ? *reinterpret_cast<const f4*>(slab + (long)(z0 + k) * n + 4 * i) : f4zero();
#pragma unroll
      for (int k = 0; k < SR_DEPTH; ++k) s += v[k];
    }
  }
  part[threadIdx.x] = s;
  __syncthreads();
  if (g == 0 && i < nq) {
#pragma unroll
    for (int gg = 1; gg < ZG; ++gg) s += part[gg * QB + ql];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const long j = 4 * i + t;
      const int row = (int)(j / e.N), col = (int)(j % e.N);
      e.C[(long)row * e.ldc + col] = apply_epi(e, row, col, s[t]);
    }
  }
}
static int slab_reduce(hipStream_t s, const float* slab, int Z, const EpiArgs& e) {
  const long n = (long)e.M * e.N, nq = n / 4;
  if (n % 4 == 0 && ((uintptr_t)slab & 15) == 0 && Z >= 4) {
    // the fewest thread groups per quad that give >= 512 workgroups (2 per CU)
    if (nq >= 512 * 64 || Z < 16) {
      slab_reduce_zg_kernel<4><<<(int)cdiv(nq, 64), 256, 0, s>>>(slab, Z, e);
    } else {
      slab_reduce_zg_kernel<16><<<(int)cdiv(nq, 16), 256, 0, s>>>(slab, Z, e);
    }
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  slab_reduce_kernel<<<(int)std::max<long>(1, std::min<long>(2048, cdiv(n / 4 + 1, 256))), 256, 0, s>>>(slab, Z, e);
  ABCD_CHECK_LAUNCH();
  return 0;
}

template <class OA, class OB>
static int gemm_launch(hipStream_t s, int M, int N, int K, OA A, OB B, EpiArgs e, float* scratch,
                       size_t scratch_floats) {
  const int nch = cdiv(K, 16);
  const int tiles_big = cdiv(M, 128) * cdiv(N, 128);
  if (tiles_big >= 240) {
    dim3 grid(cdiv(N, 128), cdiv(M, 128), 1);
    gemm_big_kernel<4, 4, OA, OB><<<grid, 256, 0, s>>>(A, B, nch, nch, e);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  const int tiles = cdiv(M, 32) * cdiv(N, 64);
  int Z = 1;
  if (tiles < 768 && nch >= 16 && scratch) {
    Z = cdiv(tl_side ? 256 : 1024, tiles);
    Z = std::min(Z, std::max(1, nch / 8));
    const long per = (long)M * N;
    Z = std::min<long>(Z, (long)(scratch_floats / (size_t)per));
    if (Z < 2) Z = 1;
  }
  const int cps = cdiv(nch, Z);
  Z = cdiv(nch, cps);
  dim3 grid(cdiv(N, 64), cdiv(M, 32), Z);
  EpiArgs ek = e;
  if (Z > 1) ek.slab = scratch;
  gemm_ks_kernel<2, 4, OA, OB><<<grid, 256, 0, s>>>(A, B, nch, cps, ek);
  ABCD_CHECK_LAUNCH();
  if (Z > 1) {
    ABCD_TRY((hipError_t)slab_reduce(s, scratch, Z, e));
  }
  return 0;
}


// ---------------------------------------------------------------------------
// gemm_tn: C[m][n] = sum_k A[k*lda + m] * B[k*ldb + n] -- both operands
// K-major, the weight-gradient shape (dW = dG^T X with K = all packed frames).
// A 16-deep K slab of each operand is staged into LDS with coalesced 16-B row
// loads (double-buffered; the next slab's global loads are in flight while the
// current one feeds the MFMAs); fragments are read back with conflict-free
// 4-B LDS reads (row pitch BM+4 / BN+4).  WG tile (32 MR) x (32 NR), 4 waves
// as 2 x 2, each (16 MR) x (16 NR): at 256 x 256 one K slab is 32 KB of loads
// for 8192 MFMA cycles per SIMD, so the kernel stays MFMA-bound with HBM
// traffic ~2.5 TB/s (only MR = 4 is instantiated: larger accumulator arrays
// are demoted to scratch by the compiler).  The grid splits K into fp32 slabs
// (slab_reduce_kernel).
// ---------------------------------------------------------------------------
// AKC / BKC: the operand is K-contiguous instead (element (row, k) at
// p[row*ld + k], e.g. frames x features): a thread loads 4 consecutive k of
// one row and stores them transposed into the same [k][row] LDS slab (4
// conflict-free 4-B writes), so the MFMA loop is shared.  This is the
// frame-parallel GEMM path (input projection, offset head).
// XCD-aware tile order: the hardware deals workgroup ids round-robin over
// the 8 XCDs (id % 8), so tiles that share an operand slab (the M tiles of
// one K split, the N tiles of one row block) would sit on 8 different L2s and
// each fetch the slab from HBM.  Remapped, XCD x runs the contiguous logical
// range [x n/8, (x+1) n/8): neighbours in (x fastest, y, z) order share its L2.
DEV dim3 xcd_tile(bool remap) {
  const unsigned gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  unsigned i = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if (remap && n % 8 == 0) i = (i % 8) * (n / 8) + i / 8;
  return dim3(i % gx, (i / gx) % gy, i / (gx * gy));
}

template <int MR, int NR, int BK = 16>
constexpr int tn_lds_floats() { return 2 * BK * (32 * MR + 4) + 2 * BK * (32 * NR + 4); }
// one (32 MR) x (32 NR) output tile at (m0, n0) over K range [kb, ke); the
// result goes to `dst` (ldd) through the epilogue, or raw when `raw` (a split-K slab).
// BK: the K depth of one LDS slab (16; 64 for a long K chain on few
// workgroups: four times the loads in flight per barrier, K-major operands only)
template <int MR, int NR, bool AKC = false, bool BKC = false, int BK = 16>
DEV void gemm_tn_tile(float* smab, const float* __restrict__ A, long lda, const float* __restrict__ B, long ldb,
                      int kb, int ke, int m0, int n0, const EpiArgs& e, float* dst, long ldd, bool raw) {
  static_assert(BK == 16 || (!AKC && !BKC), "deep slabs for K-major operands only");
  constexpr int BM = 32 * MR, BN = 32 * NR, LA = BM + 4, LB = BN + 4;
  constexpr int AVT = BK * BM / 4, BVT = BK * BN / 4;   // f4 per slab
  constexpr int AV = (AVT + 255) / 256, BV = (BVT + 255) / 256;
  float* const As = smab;                  // [2][BK * LA]
  float* const Bs = smab + 2 * BK * LA;    // [2][BK * LB]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int M = e.M, N = e.N;
  f4 ra[AV], rb[BV];
  // slab element -> (k, row) of f4 x: K-major: 4 rows at one k; K-contiguous: 4 k of one row
  auto gload1 = [&](const float* P, long ld, int R, int r0, int k0, int x, int BR, bool kc) -> f4 {
    if (kc) {
      const int row = x / 4, k = 4 * (x % 4);
      if (r0 + row < R && k0 + k + 4 <= ke) return *reinterpret_cast<const f4*>(P + (long)(r0 + row) * ld + k0 + k);
      f4 v = f4zero();
      if (r0 + row < R)
        for (int s = 0; s < 4; ++s) v[s] = k0 + k + s < ke ? P[(long)(r0 + row) * ld + k0 + k + s] : 0.f;
      return v;
    }
    const int k = x / (BR / 4), row = (x % (BR / 4)) * 4;
    return (k0 + k < ke && r0 + row < R) ? *reinterpret_cast<const f4*>(P + (long)(k0 + k) * ld + r0 + row) : f4zero();
  };
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int x = threadIdx.x + 256 * u;
      ra[u] = x < AVT ? gload1(A, lda, M, m0, k0, x, BM, AKC) : f4zero();
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      const int x = threadIdx.x + 256 * u;
      rb[u] = x < BVT ? gload1(B, ldb, N, n0, k0, x, BN, BKC) : f4zero();
    }
  };
  auto lstore1 = [&](float* S, int LD, int BR, int x, const f4& v, bool kc) {
    if (kc) {
      const int row = x / 4, k = 4 * (x % 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) S[(k + s) * LD + row] = v[s];
    } else {
      const int k = x / (BR / 4), row = (x % (BR / 4)) * 4;
      *reinterpret_cast<f4*>(&S[k * LD + row]) = v;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int x = threadIdx.x + 256 * u;
      if (x < AVT) lstore1(As + buf * BK * LA, LA, BM, x, ra[u], AKC);
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      const int x = threadIdx.x + 256 * u;
      if (x < BVT) lstore1(Bs + buf * BK * LB, LB, BN, x, rb[u], BKC);
    }
  };
  f4 acc[MR][NR];
  acc_zero(acc);
  gload(kb);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) gload(k0 + BK);
    const float* as = As + cur * BK * LA + wm * 16 * MR + r;
    const float* bs = Bs + cur * BK * LB + wn * 16 * NR + r;
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const int k = 16 * (s / 4) + 4 * q + (s % 4);
      float a[MR], b[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) a[i] = as[k * LA + 16 * i];
#pragma unroll
      for (int j = 0; j < NR; ++j) b[j] = bs[k * LB + 16 * j];
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = mfma4(a[i], b[j], acc[i][j]);
    }
    if (more) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  // epilogue through a wave-private LDS transpose (the operand slabs are free
  // after the loop's last barrier): each 16-row strip of the wave's tile goes
  // out as whole rows of 16-B stores (4 x NR lanes per row) instead of 64-B
  // row pieces from the accumulator layout
  constexpr int SW = 16 * NR, SP = SW + 4;  // strip width, pitch (16 x SW floats = 64 NR f4 per strip)
  float* stg = smab + w * 16 * SP;
  const bool vec = (ldd % 4 == 0) && (((uintptr_t)dst & 15) == 0);
#pragma unroll
  for (int i = 0; i < MR; ++i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) stg[(4 * q + g) * SP + 16 * j + r] = acc[i][j][g];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const int lr = (lane + 64 * p) / (4 * NR), c4 = (lane + 64 * p) % (4 * NR);
      const int gcol = n0 + wn * SW + 4 * c4;
      const int row = m0 + wm * 16 * MR + 16 * i + lr;
      f4 v = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * c4);
      if (row < M) {
        if (!raw) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) v[t] = apply_epi(e, row, gcol + t, v[t]);
        }
        float* d = dst + (long)row * ldd + gcol;
        if (vec && gcol + 4 <= N) *reinterpret_cast<f4*>(d) = v;
        else
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) d[t] = v[t];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int MR, int NR, bool AKC = false, bool BKC = false>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(const float* __restrict__ A, long lda,
                                                      const float* __restrict__ B, long ldb, int K, int kps,
                                                      EpiArgs e, int remap) {
  __shared__ __attribute__((aligned(16))) float smab[tn_lds_floats<MR, NR>()];
  const dim3 bid = xcd_tile(remap != 0);
  const int kb = bid.z * kps, ke = min(K, kb + kps);
  float* const dst = e.slab ? e.slab + (long)bid.z * e.M * e.N : e.C;
  gemm_tn_tile<MR, NR, AKC, BKC>(smab, A, lda, B, ldb, kb, ke, bid.y * 32 * MR, bid.x * 32 * NR, e, dst,
                                 e.slab ? (long)e.N : e.ldc, e.slab != nullptr);
}

// gemm_tn_batch: gemm_tn's LDS-staged tile (32 x 32, fp32 MFMA) over the
// whole K for every tile of every job of the batch, one launch (the sampler's and the decoder
// initial state's weight gradients: four GEMMs, each 8-128 tiles at K = 512 /
// 1024, were four split-K launches + four slab reductions).  The job table
// travels in the kernel arguments; blockIdx.x walks the jobs' tiles in order.
struct GemmBatchArgs {
  GemmJob j[GEMM_BATCH_MAX];
  int tile0[GEMM_BATCH_MAX + 1];  // first tile of each job; tile0[n] = total
  int n;
};
template <int MR, int NR, int BK>
__global__ __launch_bounds__(256) void gemm_tn_batch_kernel(GemmBatchArgs b) {
  __shared__ __attribute__((aligned(16))) float smab[tn_lds_floats<MR, NR, BK>()];
  int ji = 0;
  while (ji + 1 < b.n && (int)blockIdx.x >= b.tile0[ji + 1]) ++ji;
  const GemmJob J = b.j[ji];
  const int t = (int)blockIdx.x - b.tile0[ji], tn = (J.N + 32 * NR - 1) / (32 * NR);
  const EpiArgs e{J.C, J.ldc, J.M, J.N, J.alpha, J.beta, nullptr, ACT_NONE, nullptr};
  gemm_tn_tile<MR, NR, false, false, BK>(smab, J.A, J.lda, J.B, J.ldb, 0, J.K, (t / tn) * 32 * MR, (t % tn) * 32 * NR,
                                         e, J.C, J.ldc, false);
}
// 32 x 32 tiles on a quiet chip: four times the workgroups at the same K
// depth as 64 x 64 (the sampler's parameter gradients, 88 -> 352 workgroups;
// same-box A/B at c2: step 8.51 / 8.52 -> 8.47 / 8.48 ms)
int gemm_tn_batch(hipStream_t s, const GemmJob* jobs, int n) {
  if (n <= 0) return 0;
  if (n > GEMM_BATCH_MAX) return (int)hipErrorInvalidValue;
  const int tb = tl_side ? 64 : 32;
  GemmBatchArgs b{};
  int tiles = 0, k = 0;
  for (int i = 0; i < n; ++i) {
    if (jobs[i].M <= 0 || jobs[i].N <= 0) continue;
    // gemm_tn_tile's staging: 16-B loads of 4 rows at one k
    if (jobs[i].lda % 4 || jobs[i].ldb % 4 || jobs[i].M % 4 || jobs[i].N % 4 || ((uintptr_t)jobs[i].A & 15) ||
        ((uintptr_t)jobs[i].B & 15))
      return ABCD_EINVAL;
    b.j[k] = jobs[i];
    b.tile0[k] = tiles;
    tiles += cdiv(jobs[i].M, tb) * cdiv(jobs[i].N, tb);
    ++k;
  }
  b.n = k;
  b.tile0[k] = tiles;
  if (!tiles) return 0;
  // 64-deep LDS slabs (70 KB) on a quiet chip; 16-deep ones (17 KB) beside a
  // persistent kernel (side mode), whose LDS image leaves ~40 KB per CU
  if (tl_side) gemm_tn_batch_kernel<2, 2, 16><<<tiles, 256, 0, s>>>(b);
  else gemm_tn_batch_kernel<1, 1, 64><<<tiles, 256, 0, s>>>(b);
  ABCD_CHECK_LAUNCH();
  return 0;
}

template <int MR, int NR, bool AKC = false, bool BKC = false>
static int gemm_tn_launch(hipStream_t s, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                          EpiArgs e, float* scratch, size_t scratch_floats) {
  const int BM = 32 * MR, BN = 32 * NR;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int Z = std::max(1, std::min(cdiv(tl_side ? 256 : 512, tiles), cdiv(K, 16 * 32)));
  if (scratch) Z = (int)std::min<long>(Z, (long)(scratch_floats / ((size_t)M * N)));
  else Z = 1;
  Z = std::max(Z, 1);
  const int kps = rup16(cdiv(K, Z));
  Z = cdiv(K, kps);
  EpiArgs ek = e;
  if (Z > 1) ek.slab = scratch;
  gemm_tn_kernel<MR, NR, AKC, BKC><<<dim3(cdiv(N, BN), cdiv(M, BM), Z), 256, 0, s>>>(A, lda, B, ldb, K, kps, ek,
                                                                                   1);
  ABCD_CHECK_LAUNCH();
  if (Z > 1) {
    ABCD_TRY((hipError_t)slab_reduce(s, scratch, Z, e));
  }
  return 0;
}

// ---------------------------------------------------------------------------
// gemm_x6s: the gemm_tn structure (fp32 [k][row] LDS slabs, double-buffered,
// K-major or K-contiguous operands, split-K over the grid, XCD-aware order,
// LDS-transposed epilogue) with the contraction on the bf16 matrix cores in
// split-fp32 form (abcd_x6.h: six bf16 MFMAs per 16x16x32 block, fp32-exact
// to one rounding).  The operands stay fp32 in LDS (32 KB per stage at
// 128 x 128, so two workgroups share a CU and hide each other's staging);
// each wave splits its own fragments -- one split per fragment and chunk,
// reused across the NR (A) or MR (B) blocks it multiplies.  Per 32-deep chunk
// a wave issues 6 MR NR MFMAs of 16 cycles against 16 (MR + NR) plain VALU
// ops of the splits: the f32-MFMA form of the same chunk costs 8 MR NR
// MFMAs of 32 cycles.
// ---------------------------------------------------------------------------
// ONE: a single operand stage (34 KB at 128 x 128, so the workgroup fits
// beside a persistent kernel's LDS image): the next chunk's loads still go
// out before the MFMAs, their LDS stores wait for a barrier after them.
template <int MR, int NR, bool AKC, bool BKC, bool ONE = false>
__global__ __launch_bounds__(256, 2) void gemm_x6s_kernel(const float* __restrict__ A, long lda,
                                                       const float* __restrict__ B, long ldb, int K, int kps,
                                                       EpiArgs e, int remap) {
  const dim3 bid = xcd_tile(remap != 0);
  // slab row k at k * L + 16 (k / 8): the four 8-k groups a fragment read
  // spans land on different bank quarters (a plain pitch of BM + 4 maps
  // groups 0 / 2 and 1 / 3 onto the same banks)
  constexpr int BM = 32 * MR, BN = 32 * NR, BK = 32, LA = BM + 4, LB = BN + 4;
  constexpr int SA = BK * LA + 16 * (BK / 8), SB = BK * LB + 16 * (BK / 8);  // one stage
  constexpr int AVT = BK * BM / 4, BVT = BK * BN / 4;  // f4 per slab
  constexpr int AV = (AVT + 255) / 256, BV = (BVT + 255) / 256;
  constexpr int NS = ONE ? 1 : 2;  // operand stages
  __shared__ __attribute__((aligned(16))) float smab[NS * SA + NS * SB];
  float* const As = smab;
  float* const Bs = smab + NS * SA;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = bid.y * BM, n0 = bid.x * BN;
  const int kb = bid.z * kps, ke = min(K, kb + kps);
  const int M = e.M, N = e.N;
  // slab element x -> K-major: 4 rows at one k; K-contiguous: 4 k of one row (BK / 4 per row)
  auto gload1 = [&](const float* P, long ld, int R, int r0, int k0, int x, int BR, bool kc) -> f4 {
    if (kc) {
      const int row = x / (BK / 4), k = 4 * (x % (BK / 4));
      if (r0 + row < R && k0 + k + 4 <= ke) return *reinterpret_cast<const f4*>(P + (long)(r0 + row) * ld + k0 + k);
      f4 v = f4zero();
      if (r0 + row < R)
        for (int t = 0; t < 4; ++t) v[t] = k0 + k + t < ke ? P[(long)(r0 + row) * ld + k0 + k + t] : 0.f;
      return v;
    }
    const int k = x / (BR / 4), row = (x % (BR / 4)) * 4;
    return (k0 + k < ke && r0 + row < R) ? *reinterpret_cast<const f4*>(P + (long)(k0 + k) * ld + r0 + row) : f4zero();
  };
  auto lstore1 = [&](float* S, int LD, int BR, int x, const f4& v, bool kc) {
    if (kc) {
      const int row = x / (BK / 4), k = 4 * (x % (BK / 4));
#pragma unroll
      for (int t = 0; t < 4; ++t) S[(k + t) * LD + 16 * ((k + t) >> 3) + row] = v[t];
    } else {
      const int k = x / (BR / 4), row = (x % (BR / 4)) * 4;
      *reinterpret_cast<f4*>(&S[k * LD + 16 * (k >> 3) + row]) = v;
    }
  };
  auto gload = [&](int k0, f4 (&xa)[AV], f4 (&xb)[BV]) {
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int x = threadIdx.x + 256 * u;
      xa[u] = x < AVT ? gload1(A, lda, M, m0, k0, x, BM, AKC) : f4zero();
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      const int x = threadIdx.x + 256 * u;
      xb[u] = x < BVT ? gload1(B, ldb, N, n0, k0, x, BN, BKC) : f4zero();
    }
  };
  auto lstore = [&](int buf, const f4 (&xa)[AV], const f4 (&xb)[BV]) {
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int x = threadIdx.x + 256 * u;
      if (x < AVT) lstore1(As + buf * SA, LA, BM, x, xa[u], AKC);
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      const int x = threadIdx.x + 256 * u;
      if (x < BVT) lstore1(Bs + buf * SB, LB, BN, x, xb[u], BKC);
    }
  };
  f4 acc[MR][NR];
  acc_zero(acc);
  auto compute = [&](int cur) {
    // fragment of lane (r, q): row r of the block, k = 8q .. 8q+7 of the chunk
    const float* as = As + cur * SA + 8 * q * LA + 16 * q + wm * 16 * MR + r;
    const float* bs = Bs + cur * SB + 8 * q * LB + 16 * q + wn * 16 * NR + r;
    bf8 bp[3][NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      f4 x0, x1;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        x0[t] = bs[t * LB + 16 * j];
        x1[t] = bs[(4 + t) * LB + 16 * j];
      }
      split8(x0, x1, bp[0][j], bp[1][j], bp[2][j]);
    }
    // per A block: its split, then the six terms (smallest first), each over
    // the NR blocks -- consecutive MFMAs write different accumulators
    constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      f4 x0, x1;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        x0[t] = as[t * LA + 16 * i];
        x1[t] = as[(4 + t) * LA + 16 * i];
      }
      bf8 ap[3];
      split8(x0, x1, ap[0], ap[1], ap[2]);
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = mfma_bf(ap[TA[t]], bp[TB[t]][j], acc[i][j]);
    }
  };
  f4 ra[AV], rb[BV];
  gload(kb, ra, rb);
  lstore(0, ra, rb);
  __syncthreads();
  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) gload(k0 + BK, ra, rb);
    compute(cur);
    if constexpr (ONE) {
      if (more) {
        __syncthreads();
        lstore(0, ra, rb);
      }
    } else {
      if (more) lstore(cur ^ 1, ra, rb);
      cur ^= 1;
    }
    __syncthreads();
  }
  // epilogue: wave-private LDS transpose, whole-row 16-B stores (as gemm_tn_kernel)
  constexpr int SW = 16 * NR, SP = SW + 4;
  float* stg = smab + w * 16 * SP;
  float* const dst = e.slab ? e.slab + (long)bid.z * M * N : e.C;
  const long ldd = e.slab ? (long)N : e.ldc;
  const bool vec = (ldd % 4 == 0) && (((uintptr_t)dst & 15) == 0);
#pragma unroll
  for (int i = 0; i < MR; ++i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) stg[(4 * q + g) * SP + 16 * j + r] = acc[i][j][g];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const int lr = (lane + 64 * p) / (4 * NR), c4 = (lane + 64 * p) % (4 * NR);
      const int gcol = n0 + wn * SW + 4 * c4;
      const int row = m0 + wm * 16 * MR + 16 * i + lr;
      f4 v = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * c4);
      if (row < M) {
        if (!e.slab) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) v[t] = apply_epi(e, row, gcol + t, v[t]);
        }
        float* d = dst + (long)row * ldd + gcol;
        if (vec && gcol + 4 <= N) *reinterpret_cast<f4*>(d) = v;
        else
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) d[t] = v[t];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// gemm_x6f: split-fp32 GEMM for two K-contiguous operands (element (row, k)
// at P[row * ld + k]: the frame-parallel projections).  gemm_x6s keeps fp32
// slabs in LDS and every wave splits the fragments it reads (8 fragment
// splits per wave and chunk, each fragment split by two waves); here each
// 32-deep chunk of the A and B tiles is read from global once per workgroup
// (two f4 per 8 k), split once into the three bf16 planes and stored in
// fragment order ([subtile][plane][lane] x 16 B), so a wave reads each
// fragment plane with one conflict-free ds_read_b128 and issues only MFMAs.
// Per chunk and thread: 4 splits of 8 values (the tile's 2 x 128 x 32
// values over 256 threads), 12 16-B LDS writes; per wave 24 ds_read_b128 and
// 96 MFMAs.  Loads go through buffer resources (rows >= M / N and k >= K read
// 0), so the staging is branch-free.  Input projection at c2: 458 us
// against gemm_x6s's 515 us (VALU per MFMA 7.4 -> 4.4, PMC); offset head
// 100 vs 110 us.
// ---------------------------------------------------------------------------
template <int MR, int NR>
__global__ __launch_bounds__(256, 2) void gemm_x6f_kernel(const float* __restrict__ A, long lda,
                                                       const float* __restrict__ B, long ldb, int K, EpiArgs e,
                                                       int remap) {
  extern __shared__ __attribute__((aligned(16))) f4 fsm[];
  constexpr int BM = 32 * MR, BN = 32 * NR, SA = BM / 16, SB = BN / 16;
  constexpr int STAGE = (SA + SB) * 3 * 64;  // f4 per stage
  constexpr int GA = BM * 4, GT = (BM + BN) * 4;  // groups of 8 k per chunk: A, A + B
  constexpr int UPT = GT / 256;                   // groups per thread
  static_assert(GT % 256 == 0 && GA % 256 == 0, "whole groups per thread");
  const dim3 bid = xcd_tile(remap != 0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = bid.y * BM, n0 = bid.x * BN;
  const int M = e.M, N = e.N, nch = (K + 31) / 32;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A, (uint32_t)((size_t)M * lda * 4));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, (uint32_t)((size_t)N * ldb * 4));
  auto gload = [&](int c, f4 (&v)[UPT][2]) {
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int g = threadIdx.x + 256 * u;
      const bool isB = g >= GA;  // uniform per u
      // group gi -> fragment slot: lane ln = gi & 63 of subtile gi >> 6 (row 16 sub + (ln & 15), k 8 (ln >> 4))
      const int gi = isB ? g - GA : g, ln = gi & 63, row = ((gi >> 6) << 4) + (ln & 15), qq = ln >> 4;
      const int k = c * 32 + 8 * qq;
      const bool ok = (isB ? n0 + row < N : m0 + row < M) && k < K;
      const uint32_t o = ok ? (uint32_t)(((isB ? (long)(n0 + row) * ldb : (long)(m0 + row) * lda) + k) * 4)
                            : 0x80000000u;
      const __amdgpu_buffer_rsrc_t rs = isB ? rb : ra;
      v[u][0] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
      v[u][1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? o + 16u : o, 0, 0));
    }
  };
  auto lstore = [&](int buf, const f4 (&v)[UPT][2]) {
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int g = threadIdx.x + 256 * u;
      const bool isB = g >= GA;
      const int gi = isB ? g - GA : g, ln = gi & 63;
      const int sub = (isB ? SA : 0) + (gi >> 6);
      bf8 h, m, l;
      split8(v[u][0], v[u][1], h, m, l);
      f4* dst = fsm + buf * STAGE + sub * 3 * 64 + ln;  // consecutive lanes, consecutive 16-B slots
      dst[0] = __builtin_bit_cast(f4, h);
      dst[64] = __builtin_bit_cast(f4, m);
      dst[128] = __builtin_bit_cast(f4, l);
    }
  };
  f4 acc[MR][NR];
  acc_zero(acc);
  auto compute = [&](int buf) {
    const f4* st = fsm + buf * STAGE;
    bf8 bp[NR][3];
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bp[j][p] = __builtin_bit_cast(bf8, st[((SA + wn * NR + j) * 3 + p) * 64 + lane]);
    constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      bf8 ap[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) ap[p] = __builtin_bit_cast(bf8, st[((wm * MR + i) * 3 + p) * 64 + lane]);
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = mfma_bf(ap[TA[t]], bp[j][TB[t]], acc[i][j]);
    }
  };
  // one LDS stage (48 KiB: two workgroups per CU); the next chunk's global
  // loads are in flight during this chunk's MFMAs.  Measured at the input
  // projection shape: 458 us against 685 us for a double-buffered stage at
  // one workgroup per CU and 475 us with two chunks of loads in flight
  f4 v[UPT][2];
  gload(0, v);
  lstore(0, v);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (more) gload(c + 1, v);
    compute(0);
    __syncthreads();  // every wave is done reading the stage
    if (more) lstore(0, v);
    __syncthreads();
  }
  // epilogue: wave-private LDS transpose, whole-row 16-B stores (as gemm_x6s_kernel)
  const int r = lane & 15, q = lane >> 4;
  constexpr int SW = 16 * NR, SP = SW + 4;
  float* stg = reinterpret_cast<float*>(fsm) + w * 16 * SP;
  float* const dst = e.C;
  const long ldd = e.ldc;
  const bool vec = (ldd % 4 == 0) && (((uintptr_t)dst & 15) == 0);
#pragma unroll
  for (int i = 0; i < MR; ++i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) stg[(4 * q + g) * SP + 16 * j + r] = acc[i][j][g];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int pp = 0; pp < NR; ++pp) {
      const int lr = (lane + 64 * pp) / (4 * NR), c4 = (lane + 64 * pp) % (4 * NR);
      const int gcol = n0 + wn * SW + 4 * c4;
      const int row = m0 + wm * 16 * MR + 16 * i + lr;
      f4 val = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * c4);
      if (row < M) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (gcol + t < N) val[t] = apply_epi(e, row, gcol + t, val[t]);
        float* d = dst + (long)row * ldd + gcol;
        if (vec && gcol + 4 <= N) *reinterpret_cast<f4*>(d) = val;
        else
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) d[t] = val[t];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int MR, int NR>
static int gemm_x6f_launch(hipStream_t s, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                           EpiArgs e) {
  constexpr int BM = 32 * MR, BN = 32 * NR;
  const size_t lds = (size_t)(BM / 16 + BN / 16) * 3 * 64 * 16;
  gemm_x6f_kernel<MR, NR><<<dim3(cdiv(N, BN), cdiv(M, BM), 1), 256, lds, s>>>(A, lda, B, ldb, K, e, 1);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// gemm_x6r8: frame-streaming split-fp32 GEMM for short K (K <= 32 NC) and
// K-contiguous operands: C[M x N] = A B^T with M = packed frames (~65k) and
// N = a few hundred to 2048 weight rows (the encoder's input projection, the
// offset head).  A workgroup owns one BN-column slice of B for the whole
// launch (split ONCE into the three bf16 planes in fragment order, resident
// in LDS) and streams a contiguous range of frames: each wave takes 16 MR
// rows at a time, loads the A fragments straight into registers, splits each
// chunk once and issues 6 MR NR MFMAs per chunk; epilogue through a
// wave-private LDS transpose, whole 16-B row stores.  Workgroups of one XCD
// (blockIdx % 8) take the slices of the same frame ranges, so A rows are
// fetched from HBM once per XCD L2.  EIGHT waves (two per SIMD) share the
// resident slice: with one wave per SIMD (round-4 gemm_x6r, removed in
// round 6) every A-load wait, split, B-plane read and epilogue store sat
// between its MFMAs (36 % MFMA busy); the second wave issues its MFMAs in
// those gaps.  The register budget halves (256 per wave), so the look-ahead
// is a rolling one in the same registers: as soon as chunk c of a block is
// split, the next block's chunk c is loaded into the fragment registers it
// came from.  The epilogue stages HR rows per wave (HR = 8 where 16 rows of
// the slice width would not fit beside the B planes).  MI355X,
// scripts/gemm_bench.py, same box: input projection 64044 x 2048 x 144
// 268-279 us against the four-wave form's 304-311 (gemm_x6f: 450), offset
// head 64044 x 256 x 256 57-60 against 70-71 (PMC: MFMA busy 51 % at the
// ~1.7 GHz the chip holds under this load).  Measured slower: the epilogue
// straight from the accumulators (64-B row segments, no LDS transpose):
// 342-347 / 69-70 us; a three-slot register ring, MR = 1 / 3 / 4 and 64-column
// slices at two workgroups per CU (four-wave form, rounds 2-4).
// MODE 1 / 2: the offset head's forward / backward (abcd_internal.h,
// gemm_offset_fwd / gemm_offset_bwd; BN = 64)
struct OffArgs {
  const float* w2;        // K (mode 2) / N (mode 1) floats
  float* part;            // mode 1: partial logits [M][nslices]
  const float* dlog_raw;  // mode 2
  const float* s;         // mode 2: device scalar
  float* dZo;             // mode 2: M x K, ld = lda
  float* dlog_s;          // mode 2
};
// T16: the last chunk holds at most 16 valid k (K <= 32 (NC - 1) + 16) and
// runs 16-deep (mma_x6_16): its B planes and A fragments in that layout
template <int NC, int BN, int MR, int HR, int MODE = 0, bool T16 = false>
__global__ __launch_bounds__(512, 1) void gemm_x6r8_kernel(const float* __restrict__ A, long lda,
                                                        const float* __restrict__ B, long ldb, int K, EpiArgs e,
                                                        int nslices, int rows_per, OffArgs oa) {
  extern __shared__ __attribute__((aligned(16))) f4 rsm[];
  constexpr int NR = BN / 16, SP = BN + 4, NW = 8, NPP = HR * BN / 256;
  static_assert(HR == 8 || HR == 16, "staging rows");
  static_assert(MODE == 0 || BN == 64, "offset-head modes: 64-column slices");
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3;  // grid = 8 * per
  const int lin = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const int slice = lin % nslices, part = lin / nslices;
  const int n0 = slice * BN, M = e.M, N = e.N;
  {  // B slice -> LDS planes [j][c][plane][lane]; rows >= N and k >= K read 0 (K % 8 == 0)
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(B + (size_t)n0 * ldb, (uint32_t)(std::max(0, std::min(BN, N - n0)) * ldb * 4));
    for (int x = threadIdx.x; x < NR * NC * 64; x += 64 * NW) {
      const int j = x / (NC * 64), c = (x / 64) % NC, ln = x & 63;
      f4* d = rsm + ((j * NC + c) * 3) * 64 + ln;
      if (T16 && c == NC - 1) {  // k = 32c + 4 (ln >> 4) + 0..3
        const int row = 16 * j + (ln & 15), kk = 32 * c + 4 * (ln >> 4);
        const uint32_t o = kk < K ? (uint32_t)(row * ldb + kk) * 4u : 0x80000000u;
        const f4 v = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, o, 0, 0));
        s4 h, m, l;
        split4(v, h, m, l);
        typedef float f2v __attribute__((ext_vector_type(2)));
        const f2v hh = __builtin_bit_cast(f2v, h), mm = __builtin_bit_cast(f2v, m), ll = __builtin_bit_cast(f2v, l);
        d[0] = f4{hh[0], hh[1], 0.f, 0.f};
        d[64] = f4{mm[0], mm[1], 0.f, 0.f};
        d[128] = f4{ll[0], ll[1], 0.f, 0.f};
        continue;
      }
      const int row = 16 * j + (ln & 15), kk = 32 * c + 8 * (ln >> 4);
      const uint32_t o = kk < K ? (uint32_t)(row * ldb + kk) * 4u : 0x80000000u;
      const f4 lo = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, o, 0, 0));
      const f4 hi = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, kk < K ? o + 16u : o, 0, 0));
      bf8 h, m, l;
      split8(lo, hi, h, m, l);
      d[0] = __builtin_bit_cast(f4, h);
      d[64] = __builtin_bit_cast(f4, m);
      d[128] = __builtin_bit_cast(f4, l);
    }
  }
  float* stg = reinterpret_cast<float*>(rsm + NR * NC * 3 * 64) + w * HR * SP;
  const int r0 = part * rows_per, r1 = std::min(M, r0 + rows_per);
  // mode 2: w2 (zero past K) and the row range's s dlog_raw, after the staging tiles
  float* w2s = reinterpret_cast<float*>(rsm + NR * NC * 3 * 64) + NW * HR * SP;
  float* dls = w2s + 32 * NC;
  if constexpr (MODE == 2) {
    const float sc = *oa.s;
    for (int k = threadIdx.x; k < 32 * NC; k += 64 * NW) w2s[k] = k < K ? oa.w2[k] : 0.f;
    for (int x = threadIdx.x; x < rows_per; x += 64 * NW) {
      const int row = r0 + x;
      const float dl = row < r1 ? sc * oa.dlog_raw[row] : 0.f;
      dls[x] = dl;
      if (slice == 0 && row < r1) oa.dlog_s[row] = dl;
    }
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A, (uint32_t)((size_t)M * lda * 4));
  // the lane's A fragments of chunk c of the block at row b: rows b + 16 i + r, k = 32 c + 8 q + 0..7
  auto aload = [&](int b, int c, f4 (&v)[MR][NC][2]) {
    const bool t16 = T16 && c == NC - 1;
    const int kk = 32 * c + (t16 ? 4 : 8) * q;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const uint32_t o = kk < K ? (uint32_t)((b + 16 * i + r) * lda + kk) * 4u : 0x80000000u;
      v[i][c][0] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, 0));
      if (!t16) v[i][c][1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, kk < K ? o + 16u : o, 0, 0));
    }
  };
  constexpr int RB = 16 * MR;
  const int ec = n0 + 4 * (lane % (BN / 4));
  f4 bq = f4zero(), w2q = f4zero();
  if (e.bias) {
#pragma unroll
    for (int t = 0; t < 4; ++t) bq[t] = ec + t < N ? e.bias[ec + t] : 0.f;
  }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) w2q[t] = ec + t < N ? oa.w2[ec + t] : 0.f;
  }
  f4 va[MR][NC][2];
  int b = r0 + w * RB;
  if (b < r1) {
#pragma unroll
    for (int c = 0; c < NC; ++c) aload(b, c, va);
  }
  for (; b < r1; b += NW * RB) {
    const int bn = b + NW * RB;  // the next block (rows past M read 0; past r1 a wasted read)
    f4 acc[MR][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = f4zero();
    auto bread = [&](int c, int j, f4 (&bb)[3]) {
      const f4* bp = rsm + ((j * NC + c) * 3) * 64 + lane;
      bb[0] = bp[0], bb[1] = bp[64], bb[2] = bp[128];
    };
    f4 bcur[3];
    bread(0, 0, bcur);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (T16 && c == NC - 1) {  // the 16-deep last chunk (MODE 0 only)
        s4 at[MR][3];
#pragma unroll
        for (int i = 0; i < MR; ++i) split4(va[i][c][0], at[i][0], at[i][1], at[i][2]);
        aload(bn, c, va);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          f4 bnxt[3];
          const bool nx = j + 1 < NR;
          if (nx) bread(c, j + 1, bnxt);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < MR; ++i)
            acc[i][j] = mma_x6_16(acc[i][j], at[i][0], at[i][1], at[i][2], lo_s4(bcur[0]), lo_s4(bcur[1]), lo_s4(bcur[2]));
          __builtin_amdgcn_sched_barrier(0);
          if (nx) bcur[0] = bnxt[0], bcur[1] = bnxt[1], bcur[2] = bnxt[2];
        }
        continue;
      }
      bf8 as[MR][3];
      if constexpr (MODE == 2) {  // Zo -> dZo = s dlog (1 - Zo^2) w2; this slice stores chunks c = slice mod nslices
        const int kk = 32 * c + 8 * q;
        const f4 wl = *reinterpret_cast<const f4*>(w2s + kk), wh = *reinterpret_cast<const f4*>(w2s + kk + 4);
#pragma unroll
        for (int i = 0; i < MR; ++i) {
          const int rl = b + 16 * i + r - r0;
          const float dl = dls[rl < rows_per ? rl : 0];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float z0 = va[i][c][0][t], z1 = va[i][c][1][t];
            va[i][c][0][t] = dl * wl[t] * (1.f - z0 * z0);
            va[i][c][1][t] = dl * wh[t] * (1.f - z1 * z1);
          }
          if (c % nslices == slice && b + 16 * i + r < r1 && kk < K) {
            float* d = oa.dZo + (long)(b + 16 * i + r) * lda + kk;
            *reinterpret_cast<f4*>(d) = va[i][c][0];
            *reinterpret_cast<f4*>(d + 4) = va[i][c][1];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < MR; ++i) split8(va[i][c][0], va[i][c][1], as[i][0], as[i][1], as[i][2]);
      // the rolling look-ahead, unconditional: a conditional load makes the
      // compiler copy the fragments at the loop latch behind a vmcnt(0)
      aload(bn, c, va);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        f4 bnxt[3];
        const bool nx = j + 1 < NR || c + 1 < NC;
        if (nx) bread(j + 1 < NR ? c : c + 1, j + 1 < NR ? j + 1 : 0, bnxt);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MR; ++i)
          acc[i][j] = mma_x6(acc[i][j], as[i][0], as[i][1], as[i][2], __builtin_bit_cast(bf8, bcur[0]),
                             __builtin_bit_cast(bf8, bcur[1]), __builtin_bit_cast(bf8, bcur[2]));
        __builtin_amdgcn_sched_barrier(0);
        if (nx) bcur[0] = bnxt[0], bcur[1] = bnxt[1], bcur[2] = bnxt[2];
      }
    }
    // epilogue: HR rows x BN at a time through the wave's LDS tile
#pragma unroll
    for (int i = 0; i < MR; ++i) {
#pragma unroll
      for (int h = 0; h < 16 / HR; ++h) {
        __builtin_amdgcn_wave_barrier();
        if (HR == 16 || (q >> 1) == h) {
#pragma unroll
          for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) stg[(4 * q + g - HR * h) * SP + 16 * j + r] = acc[i][j][g];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int pp = 0; pp < NPP; ++pp) {
          const int lr = (lane + 64 * pp) / (BN / 4), col = ec;
          const int row = b + 16 * i + HR * h + lr;
          f4 val = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * (lane % (BN / 4)));
          float pl = 0.f;  // mode 1: this quad's share of the row's logit
          if (row < r1 && col < N) {
            float* d = e.C + (long)row * e.ldc + col;
            val = val * e.alpha + bq;
            if (e.beta != 0.f) {
#pragma unroll
              for (int t = 0; t < 4; ++t)
                if (col + t < N) val[t] += e.beta * d[t];
            }
            if (e.act == ACT_TANH) {
#pragma unroll
              for (int t = 0; t < 4; ++t) val[t] = tanhf(val[t]);
            }
            if constexpr (MODE == 1) pl = val[0] * w2q[0] + val[1] * w2q[1] + val[2] * w2q[2] + val[3] * w2q[3];
            if (col + 4 <= N) *reinterpret_cast<f4*>(d) = val;
            else
#pragma unroll
              for (int t = 0; t < 4; ++t)
                if (col + t < N) d[t] = val[t];
          }
          if constexpr (MODE == 1) {  // the 16 quads of a row: lanes 16 k .. 16 k + 15, fixed order
            pl += __shfl_xor(pl, 1, 64);
            pl += __shfl_xor(pl, 2, 64);
            pl += __shfl_xor(pl, 4, 64);
            pl += __shfl_xor(pl, 8, 64);
            if ((lane & 15) == 0 && row < r1) oa.part[(long)row * nslices + slice] = pl;
          }
        }
      }
    }
  }
}

template <int NC, int BN, int MR>
struct X6r8Grid {
  int nslices, grid, rows_per;
  X6r8Grid(int M, int N) {
    nslices = cdiv(N, BN);
    // one workgroup per CU: about 256 / nslices frame ranges, their count a
    // multiple of 8 / gcd(nslices, 8) so that the grid (every (slice, range)
    // pair once) is a multiple of 8 for the XCD grouping
    const int step = 8 / std::gcd(nslices, 8);
    const int nparts = std::max(step, (256 / nslices) / step * step);
    grid = nslices * nparts;
    rows_per = ((cdiv(M, nparts) + 16 * MR - 1) / (16 * MR)) * (16 * MR);
  }
};
template <int NC, int BN, int MR, int HR, int MODE = 0, bool T16 = false>
static int gemm_x6r8_launch(hipStream_t s, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                            EpiArgs e, OffArgs oa = OffArgs{}) {
  const X6r8Grid<NC, BN, MR> gr(M, N);
  size_t lds = (size_t)(BN / 16) * NC * 3 * 64 * 16 + (size_t)8 * HR * (BN + 4) * 4;
  if (MODE == 2) lds += (size_t)(32 * NC + gr.rows_per) * 4;
  static bool attr = false;
  if (!attr) {
    ABCD_TRY(hipFuncSetAttribute((const void*)gemm_x6r8_kernel<NC, BN, MR, HR, MODE, T16>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  gemm_x6r8_kernel<NC, BN, MR, HR, MODE, T16><<<gr.grid, 512, lds, s>>>(A, lda, B, ldb, K, e, gr.nslices, gr.rows_per, oa);
  ABCD_CHECK_LAUNCH();
  return 0;
}
// the offset head's GEMMs (abcd_internal.h); shapes they do not take
// (decoder hidden size > 256, unaligned operands) run the separate head
// kernels dec_offset_head / dec_offset_bwd beside plain GEMMs
static bool offset_fused_ok(int M, int N, int K, long lda, const void* A, const void* B, long ldb) {
  return M > 0 && N > 0 && K > 0 && K <= 256 && K % 8 == 0 && lda % 4 == 0 &&
         ldb % 4 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 &&
         (size_t)M * lda * 4 < (1ull << 31) && (size_t)N * ldb * 4 < (1ull << 31);
}
int offset_head_slices(int N) { return cdiv(N, 64); }
int gemm_offset_fwd(hipStream_t s, int M, int N, int K, const float* Hs, long ldh, const float* W1o,
                    const float* b1o, float* Zo, const float* w2, float* part, bool* done) {
  *done = false;
  if (!offset_fused_ok(M, N, K, ldh, Hs, W1o, K) || (N % 4) != 0 || ((uintptr_t)Zo % 16) != 0) return 0;
  EpiArgs e{Zo, N, M, N, 1.f, 0.f, b1o, ACT_TANH, nullptr};
  OffArgs oa{};
  oa.w2 = w2;
  oa.part = part;
  ABCD_TRY((hipError_t)(gemm_x6r8_launch<8, 64, 2, 16, 1>(s, M, N, K, Hs, ldh, W1o, K, e, oa)));
  *done = true;
  return 0;
}
int gemm_offset_bwd(hipStream_t s, int M, int N, int K, const float* Zo, const float* W1oT, float* DHO,
                    const float* w2, const float* dlog_raw, const float* s_off, float* dZo, float* dlog_s,
                    bool* done) {
  *done = false;
  if (!offset_fused_ok(M, N, K, K, Zo, W1oT, K) || (N % 4) != 0 || ((uintptr_t)DHO % 16) != 0 ||
      ((uintptr_t)dZo % 16) != 0)
    return 0;
  const X6r8Grid<8, 64, 2> gr(M, N);
  const size_t lds = (size_t)4 * 8 * 3 * 64 * 16 + (size_t)8 * 16 * 68 * 4 + (size_t)(256 + gr.rows_per) * 4;
  if (lds > 160 * 1024) return 0;
  EpiArgs e{DHO, N, M, N, 1.f, 0.f, nullptr, ACT_NONE, nullptr};
  OffArgs oa{};
  oa.w2 = w2;
  oa.dlog_raw = dlog_raw;
  oa.s = s_off;
  oa.dZo = dZo;
  oa.dlog_s = dlog_s;
  ABCD_TRY((hipError_t)(gemm_x6r8_launch<8, 64, 2, 16, 2>(s, M, N, K, Zo, K, W1oT, K, e, oa)));
  *done = true;
  return 0;
}

// ---------------------------------------------------------------------------
// gemm_x6t: gemm_x6f for two K-major operands (element (row, k) at
// P[k * ld + row]: the weight gradients dW = dG^T X over all packed frames).
// A thread stages one row quad x 8 k of one operand per chunk: eight 16-B
// loads (rows 4rq .. 4rq + 3 at k, k + 1, ..., k + 7; the 32 row quads of a
// k are one contiguous 512-B read), then four splits (one per row) into the
// fragment-ordered bf16 planes.  Split-K over the grid into fp32 slabs as
// gemm_x6s.  Rows in [M, roundup4(M)) (padding of the leading dimension) are
// zeroed after the load; k >= the slab's end reads 0 (buffer range).
// dW_hh at c2 (M = 4H = 1024, N = H = 256, K = 65.6k frames): 250 us against
// gemm_x6s's 311 us (PMC: VALU per MFMA 3.7; LDS bank-conflict cycles 37.9 M
// -> 12.7 M per launch with the padded subtile blocks).  Two chunks of loads
// in flight measured no faster than one (kept: it costs no occupancy).
// ---------------------------------------------------------------------------
template <int MR, int NR>
__global__ __launch_bounds__(256, 2) void gemm_x6t_kernel(const float* __restrict__ A, long lda,
                                                          const float* __restrict__ B, long ldb, int K, int kps,
                                                          EpiArgs e, int remap) {
  extern __shared__ __attribute__((aligned(16))) f4 fsm[];
  constexpr int BM = 32 * MR, BN = 32 * NR, SA = BM / 16;
  constexpr int QA = BM / 4 * 4, QT = (BM + BN) / 4 * 4;  // (row quad, k group) units: A, A + B
  static_assert(QT == 256, "one unit per thread");
  // the operand's buffer resource lives in SGPRs: each wave must stage one operand only
  static_assert(QA % 64 == 0, "A / B split on a wave boundary");
  // subtile blocks of three 1-KiB planes, 16 B of pad between blocks: the
  // eight row quads a wave writes per store land in eight different
  // subtiles, which without the pad share one bank set (8-way conflicts)
  constexpr int BLK = 3 * 64 + 1;
  const dim3 bid = xcd_tile(remap != 0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = bid.y * BM, n0 = bid.x * BN;
  const int M = e.M, N = e.N;
  const int kb = bid.z * kps, ke = min(K, kb + kps);
  const int nch = (ke - kb + 31) / 32;
  // this thread's unit: operand, row quad, k group
  const int tid = threadIdx.x;
  const bool isB = tid >= QA;
  const int ui = isB ? tid - QA : tid;
  const int nrq = (isB ? BN : BM) / 4;
  const int rq = ui % nrq, qg = ui / nrq;
  const int row = (isB ? n0 : m0) + 4 * rq, R = isB ? N : M;
  const long ld = isB ? ldb : lda;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(isB ? B : A, (uint32_t)((size_t)ke * ld * 4));
  const bool rowok = row < R;
  auto gload = [&](int c, f4 (&v)[8]) {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = kb + c * 32 + 8 * qg + kk;
      const uint32_t o = (rowok && k < ke) ? (uint32_t)(((long)k * ld + row) * 4) : 0x80000000u;
      v[kk] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
    }
  };
  auto lstore = [&](const f4 (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f4 x0, x1;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        x0[t] = row + i < R ? v[t][i] : 0.f;
        x1[t] = row + i < R ? v[4 + t][i] : 0.f;
      }
      bf8 h, m, l;
      split8(x0, x1, h, m, l);
      const int rr = 4 * rq + i;
      f4* dst = fsm + ((isB ? SA : 0) + (rr >> 4)) * BLK + qg * 16 + (rr & 15);
      dst[0] = __builtin_bit_cast(f4, h);
      dst[64] = __builtin_bit_cast(f4, m);
      dst[128] = __builtin_bit_cast(f4, l);
    }
  };
  f4 acc[MR][NR];
  acc_zero(acc);
  auto compute = [&]() {
    bf8 bp[NR][3];
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bp[j][p] = __builtin_bit_cast(bf8, fsm[(SA + wn * NR + j) * BLK + p * 64 + lane]);
    constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      bf8 ap[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) ap[p] = __builtin_bit_cast(bf8, fsm[(wm * MR + i) * BLK + p * 64 + lane]);
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = mfma_bf(ap[TA[t]], bp[j][TB[t]], acc[i][j]);
    }
  };
  // two chunks of global loads in flight (register sets v0 / v1 alternate):
  // with one, every chunk waited out most of an HBM round trip
  f4 v0[8], v1[8];
  gload(0, v0);
  if (nch > 1) gload(1, v1);
  lstore(v0);
  __syncthreads();
  for (int c = 0; c < nch; c += 2) {
    if (c + 2 < nch) gload(c + 2, v0);
    compute();
    __syncthreads();
    if (c + 1 < nch) {
      lstore(v1);
      __syncthreads();
      if (c + 3 < nch) gload(c + 3, v1);
      compute();
      __syncthreads();
      if (c + 2 < nch) {
        lstore(v0);
        __syncthreads();
      }
    }
  }
  // epilogue (gemm_x6s_kernel's): wave-private LDS transpose, 16-B row stores, slab or C
  const int r = lane & 15, q = lane >> 4;
  constexpr int SW = 16 * NR, SP = SW + 4;
  float* stg = reinterpret_cast<float*>(fsm) + w * 16 * SP;
  float* const dst = e.slab ? e.slab + (long)bid.z * M * N : e.C;
  const long ldd = e.slab ? (long)N : e.ldc;
  const bool vec = (ldd % 4 == 0) && (((uintptr_t)dst & 15) == 0);
#pragma unroll
  for (int i = 0; i < MR; ++i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) stg[(4 * q + g) * SP + 16 * j + r] = acc[i][j][g];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int pp = 0; pp < NR; ++pp) {
      const int lr = (lane + 64 * pp) / (4 * NR), c4 = (lane + 64 * pp) % (4 * NR);
      const int gcol = n0 + wn * SW + 4 * c4;
      const int grow = m0 + wm * 16 * MR + 16 * i + lr;
      f4 val = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * c4);
      if (grow < M) {
        if (!e.slab) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) val[t] = apply_epi(e, grow, gcol + t, val[t]);
        }
        float* d = dst + (long)grow * ldd + gcol;
        if (vec && gcol + 4 <= N) *reinterpret_cast<f4*>(d) = val;
        else
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (gcol + t < N) d[t] = val[t];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int MR, int NR>
static int gemm_x6t_launch(hipStream_t s, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                           EpiArgs e, float* scratch, size_t scratch_floats) {
  const int BM = 32 * MR, BN = 32 * NR;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int Z = std::max(1, std::min(cdiv(512, tiles), cdiv(K, 32 * 16)));
  if (scratch) Z = (int)std::min<long>(Z, (long)(scratch_floats / ((size_t)M * N)));
  else Z = 1;
  Z = std::max(Z, 1);
  const int kps = ((cdiv(K, Z) + 31) / 32) * 32;
  Z = cdiv(K, kps);
  EpiArgs ek = e;
  if (Z > 1) ek.slab = scratch;
  const size_t lds = (size_t)(BM / 16 + BN / 16) * (3 * 64 + 1) * 16;
  gemm_x6t_kernel<MR, NR><<<dim3(cdiv(N, BN), cdiv(M, BM), Z), 256, lds, s>>>(A, lda, B, ldb, K, kps, ek, 1);
  ABCD_CHECK_LAUNCH();
  if (Z > 1) {
    ABCD_TRY((hipError_t)slab_reduce(s, scratch, Z, e));
  }
  return 0;
}


// ---------------------------------------------------------------------------
// gemm_wg2: every weight gradient of a layer-0 LSTM encoder cell, all
// directions in ONE launch (model.py:60-66's autograd for w_ih, b_ih, b_hh,
// w_hh):
//     [dW_ih | db | 0 | dW_hh]_d = dG_d^T [Xp | Hprev_d]      (K = all L frames)
// Xp is the padded frame copy whose column F holds 1 (set_col_kernel), so its
// N1 = Fp columns give dW_ih and the bias gradient in one product; the N2 = H
// columns of Hprev give dW_hh.  The split GEMMs this replaces (x6s dW_ih +
// x6t dW_hh per direction, two streams, four slab reductions) read dG twice
// and split every dG fragment twice; here a workgroup owns 128 gate rows x
// ALL N1 + N2 columns, so dG is read and split once and the B chunk is shared
// by the 8 row tiles of one K range (XCD-grouped: they run on one L2).
//   Tile 128 x 16 NB (NB = 25 at Fp = 144, H = 256), 4 waves as 2 x 2: a wave
// owns 64 rows x 13 column blocks (208 accumulator registers).  Operands are
// staged fp32 in LDS ([k][col], double-buffered: 139 KiB, one workgroup per
// CU) and each wave splits its own fragments (4 A + 13 B splits per 32-deep
// chunk against 312 MFMAs).  Branch-free buffer loads (k >= the K range and
// rows >= M read 0); the grid's K ranges write fp32 slabs that
// wg2_reduce_kernel sums in slab order and scatters into the gradients.
// ---------------------------------------------------------------------------
template <int N1, int N2>
struct Wg2 {
  static constexpr int NT = N1 + N2, NB = (NT + 15) / 16, NBW = (NB + 1) / 2;
  static constexpr int BM = 128, BK = 32, LA = BM + 4, LB = 32 * NBW + 4;
  static constexpr int SA = BK * LA + 16 * (BK / 8), SB = BK * LB + 16 * (BK / 8);
  static constexpr int AVT = BK * BM / 4, V1T = BK * N1 / 4, V2T = BK * N2 / 4;  // f4 per chunk
  static constexpr int AV = AVT / 256, V1 = (V1T + 255) / 256, V2 = (V2T + 255) / 256;
  static constexpr size_t LDS = (size_t)2 * (SA + SB) * 4;
  static_assert(N1 % 4 == 0 && N2 % 4 == 0 && AVT % 256 == 0, "f4 staging");
};

template <int N1, int N2>
__global__ __launch_bounds__(256, 1) void gemm_wg2_kernel(WgArgs a) {
  using G = Wg2<N1, N2>;
  constexpr int NT = G::NT, NBW = G::NBW, BM = G::BM, BK = G::BK, LA = G::LA, LB = G::LB;
  constexpr int SA = G::SA, SB = G::SB, AV = G::AV, V1 = G::V1, V2 = G::V2;
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  float* const As = wsm;
  float* const Bs = wsm + 2 * SA;
  const dim3 bid = xcd_tile(true);  // the row tiles of one (direction, K range) on one XCD
  const int dz = bid.z, d = dz / a.Z, z = dz % a.Z;
  const int m0 = bid.x * BM, M = a.M;
  const int kb = z * a.kps, ke = min(a.K, kb + a.kps);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, q = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.A[d], (uint32_t)((size_t)ke * a.lda * 4));
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.B1[d], (uint32_t)((size_t)ke * a.ldb1 * 4));
  const __amdgpu_buffer_rsrc_t r2 = make_rsrc(a.B2[d], (uint32_t)((size_t)ke * a.ldb2 * 4));
  constexpr uint32_t OOB = 0x80000000u;
  auto ld4 = [](const __amdgpu_buffer_rsrc_t& rs, uint32_t o) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
  };
  auto gload = [&](int k0, f4 (&xa)[AV], f4 (&x1)[V1], f4 (&x2)[V2]) {
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int x = tid + 256 * u, k = k0 + x / (BM / 4), m = m0 + 4 * (x % (BM / 4));
      xa[u] = ld4(rA, m < M ? (uint32_t)(((long)k * a.lda + m) * 4) : OOB);
    }
#pragma unroll
    for (int u = 0; u < V1; ++u) {
      const int x = tid + 256 * u, k = k0 + x / (N1 / 4), c = 4 * (x % (N1 / 4));
      x1[u] = ld4(r1, x < G::V1T ? (uint32_t)(((long)k * a.ldb1 + c) * 4) : OOB);
    }
#pragma unroll
    for (int u = 0; u < V2; ++u) {
      const int x = tid + 256 * u, k = k0 + x / (N2 / 4), c = 4 * (x % (N2 / 4));
      x2[u] = ld4(r2, x < G::V2T ? (uint32_t)(((long)k * a.ldb2 + c) * 4) : OOB);
    }
  };
  // [k][col] slabs, row k at k * LD + 16 (k / 8) (the four 8-k groups of a
  // fragment read on different bank quarters, as gemm_x6s)
  auto lstore = [&](int buf, const f4 (&xa)[AV], const f4 (&x1)[V1], const f4 (&x2)[V2]) {
    float* as = As + buf * SA;
    float* bs = Bs + buf * SB;
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int x = tid + 256 * u, k = x / (BM / 4), c = 4 * (x % (BM / 4));
      *reinterpret_cast<f4*>(as + k * LA + 16 * (k >> 3) + c) = xa[u];
    }
#pragma unroll
    for (int u = 0; u < V1; ++u) {
      const int x = tid + 256 * u, k = x / (N1 / 4), c = 4 * (x % (N1 / 4));
      if (x < G::V1T) *reinterpret_cast<f4*>(bs + k * LB + 16 * (k >> 3) + c) = x1[u];
    }
#pragma unroll
    for (int u = 0; u < V2; ++u) {
      const int x = tid + 256 * u, k = x / (N2 / 4), c = 4 * (x % (N2 / 4));
      if (x < G::V2T) *reinterpret_cast<f4*>(bs + k * LB + 16 * (k >> 3) + N1 + c) = x2[u];
    }
  };
  f4 acc[4][NBW];
  acc_zero(acc);
  auto compute = [&](int cur) {
    // fragment of lane (r, q): row / column r of the block, k = 8q .. 8q + 7
    const float* as = As + cur * SA + 8 * q * LA + 16 * q + wm * 64 + r;
    const float* bs = Bs + cur * SB + 8 * q * LB + 16 * q + wn * 16 * NBW + r;
    bf8 ap[4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f4 x0, x1;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        x0[t] = as[t * LA + 16 * i];
        x1[t] = as[(4 + t) * LA + 16 * i];
      }
      split8(x0, x1, ap[i][0], ap[i][1], ap[i][2]);
    }
    constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
    // (an odd block count leaves the last half-wave one block past NB: it
    // multiplies the zeroed pad columns, never stored -- no branch, so the
    // block loop stays one basic block the scheduler can interleave)
    // software-pipelined: block j + 1's B reads and split are issued between
    // block j's 24 MFMAs, two VALU per MFMA (the wave is alone on its SIMD:
    // VALU placed after an MFMA run only issues once the run has; same-box
    // A/B at c2: 723 -> 668 us in the step, 770 -> 720 us alone; three VALU
    // per MFMA 700)
    auto bsplit = [&](int j, bf8 (&bp)[3]) {
      f4 x0, x1;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        x0[t] = bs[t * LB + 16 * j];
        x1[t] = bs[(4 + t) * LB + 16 * j];
      }
      split8(x0, x1, bp[0], bp[1], bp[2]);
    };
    bf8 bp[3];
    bsplit(0, bp);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      bf8 bq[3];
      if (j + 1 < NBW) bsplit(j + 1, bq);
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = mfma_bf(ap[i][TA[t]], bp[TB[t]], acc[i][j]);
      if (j + 1 < NBW) {
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // the next block's B reads
#pragma unroll
        for (int k = 0; k < 24; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (j + 1 < NBW) bp[0] = bq[0], bp[1] = bq[1], bp[2] = bq[2];
    }
  };
  // the pad columns NT .. 32 NBW of both B stages read as 0
  for (int e = tid; e < 2 * BK * (LB - 4 - NT); e += 256) {
    const int st = e / (BK * (LB - 4 - NT)), x = e % (BK * (LB - 4 - NT)), k = x / (LB - 4 - NT);
    Bs[st * SB + k * LB + 16 * (k >> 3) + NT + x % (LB - 4 - NT)] = 0.f;
  }
  f4 ra[AV], r1v[V1], r2v[V2];
  gload(kb, ra, r1v, r2v);
  lstore(0, ra, r1v, r2v);
  __syncthreads();
  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) gload(k0 + BK, ra, r1v, r2v);
    compute(cur);
    if (more) lstore(cur ^ 1, ra, r1v, r2v);
    __syncthreads();
    cur ^= 1;
  }
  // epilogue: per 16-row block, a wave-private LDS transpose, then whole-row
  // 16-B stores into this K range's slab [M][NT]
  constexpr int SW = 16 * NBW, SP = SW + 4;
  float* stg = wsm + w * 16 * SP;
  float* const dst = a.slab + (size_t)dz * M * NT;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) stg[(4 * q + g) * SP + 16 * j + r] = acc[i][j][g];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < NBW; ++p) {  // 16 rows x 4 NBW quads = 64 NBW lanes' worth
      const int e = lane + 64 * p, lr = e / (4 * NBW), c4 = e % (4 * NBW);
      const int gcol = wn * SW + 4 * c4, grow = m0 + wm * 64 + 16 * i + lr;
      if (grow < M && gcol < NT)
        *reinterpret_cast<f4*>(dst + (size_t)grow * NT + gcol) = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * c4);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// sum of the Z slabs of each direction (slab order, SR_DEPTH loads in
// flight) scattered into w_ih (cols < F), b_ih / b_hh (col F), w_hh (cols
// N1 .. N1 + H)
__global__ __launch_bounds__(256) void wg2_reduce_kernel(const float* slab, int nd, int Z, int M, int NT, int N1,
                                                         int F, int H, WgOut o) {
  const long per = (long)M * NT / 4;  // f4 per slab
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nd * per; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i / per);
    const long e = i % per;
    const f4* base = reinterpret_cast<const f4*>(slab) + (long)d * Z * per + e;
    f4 s = f4zero();
    for (int z0 = 0; z0 < Z; z0 += SR_DEPTH) {
      f4 v[SR_DEPTH];
#pragma unroll
      for (int k = 0; k < SR_DEPTH; ++k) v[k] = z0 + k < Z ? base[(long)(z0 + k) * per] : f4zero();
#pragma unroll
      for (int k = 0; k < SR_DEPTH; ++k) s += v[k];
    }
    const int m = (int)(4 * e / NT), n0 = (int)(4 * e % NT);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = n0 + t;
      if (n < F) o.w_ih[d][(long)m * F + n] = s[t];
      else if (n == F) {
        o.b_ih[d][m] = s[t];
        if (o.b_hh[d]) o.b_hh[d][m] = s[t];
      } else if (n >= N1 && n < N1 + H) o.w_hh[d][(long)m * H + n - N1] = s[t];
    }
  }
}

// ---------------------------------------------------------------------------
// gemm_wg3b: gemm_wg2's product with every operand split ONCE, in the
// staging pass, and no VALU in the MFMA loop.  gemm_wg2 (above) keeps fp32 in
// LDS and each wave splits the fragments it reads -- the A rows and the B
// columns twice per workgroup, ~800 VALU per 32-deep chunk per wave against
// 312 MFMAs whose issue gaps hide ~620 -- so its MFMA pipe idles about half
// the time (PMC r07).  Here each thread splits the f4s it loaded into three
// bf16 planes stored [plane][k][col] with a k-row pitch that is an odd
// multiple of 32 B, and the MFMA loop reads its operands with
// ds_read_b64_tr_b16 (4 k-rows x 16 columns per 16-lane group, delivered
// column-major).  The 16-lane group g of a fragment reads k-rows 4g .. 4g + 3
// and 16 + 4g .. 16 + 4g + 3 (one permutation of k for both operands, so the
// sum is unchanged), which puts the 8 rows of a 32-lane half on 8 distinct
// 32-B bank slots: conflict-free.  A tile covers one HALF of the NT = N1 + N2
// columns (13 blocks of 16; the two halves of a row tile are adjacent
// workgroups on one XCD, so the second read of the dG tile is an L2 hit).
// (Round 4 also ran this staging on 128-row tiles, `gemm_wg3`, with 4 or 8
// waves: 623-691 us alone against wg3b's 572-619; removed in round 5.)
// ---------------------------------------------------------------------------
typedef short s4v __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

// 4 fp32 -> the three bf16 planes' 8-byte pieces (split8's decomposition)
DEV void split4(const f4& x, u2v& h, u2v& m, u2v& l) {
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    const uint32_t hp = cvt_pk(a, b);
    const float ra = a - lo_f(hp), rb = b - hi_f(hp);
    const uint32_t mp = cvt_pk(ra, rb);
    h[e] = hp;
    m[e] = mp;
    l[e] = cvt_pk(ra - lo_f(mp), rb - hi_f(mp));
  }
}

// gemm_wg3b tile: 256 gate rows (half the B-operand bytes per MFMA of a
// 128-row tile: that loop is bound by its operand traffic).  Two A stages (52
// KiB each) but ONE B stage (39 KiB): the next chunk's B columns are split and
// stored between two barriers at the end of each chunk; the A rows inside the
// MFMA gaps (each loaded f4 split and stored into the other stage, reloaded
// with the chunk after next).  8 waves as 4 row groups (64 rows) x 2 column
// groups (7 / 6 blocks).  Same-box A/B at c2 against the 128-row 4 x 2 form:
// 507 vs ~579 us per launch, step 8.97 / 8.94 -> 8.85 / 8.86 ms.
template <int N1, int N2>
struct Wg3b {
  static constexpr int NT = N1 + N2, NB = (NT + 15) / 16, NBH = (NB + 1) / 2, NH = 16 * NBH;
  static constexpr int BM = 256, BK = 32, T = 512, WM = 4, RW = BM / WM, MI = RW / 16;
  static constexpr int NB0 = (NBH + 1) / 2, NBL = NBH - NB0;
  static constexpr int odd32(int bytes) { return (((bytes + 31) / 32) | 1) * 32; }
  static constexpr int RA = odd32(BM * 2), RB = odd32(NH * 2);
  static constexpr int PA = BK * RA, PB = BK * RB, SA = 3 * PA, OB = 2 * SA, DUMMY = OB + 3 * PB;
  static constexpr int QX = N1 / 4, QH0 = (NH - N1) / 4, QH1 = (NT - NH) / 4;
  static constexpr int VX = (BK * QX + T - 1) / T, V0 = VX + (BK * QH0 + T - 1) / T, V1 = (BK * QH1 + T - 1) / T;
  static constexpr int AV = BK * BM / 4 / T, BV = V0 > V1 ? V0 : V1;
  static constexpr int SP = 16 * NB0 + 4;
  static constexpr size_t LDS = (size_t)DUMMY + 512;
  static_assert(LDS <= 160 * 1024 && (size_t)8 * 16 * SP * 4 <= LDS && AV + 1 <= NBL, "wg3b layout");
};

template <int N1, int N2>
__global__ __launch_bounds__(512, 1) void gemm_wg3b_kernel(WgArgs a) {
  using G = Wg3b<N1, N2>;
  constexpr int NT = G::NT, NH = G::NH, BM = G::BM, BK = G::BK, T = G::T, RW = G::RW, MI = G::MI, WM = G::WM;
  constexpr int NB0 = G::NB0, NBL = G::NBL, RA = G::RA, RB = G::RB, PA = G::PA, PB = G::PB, SA = G::SA, OB = G::OB;
  constexpr int AV = G::AV, BV = G::BV, QX = G::QX, QH0 = G::QH0, QH1 = G::QH1, VX = G::VX;
  constexpr uint32_t OOB = 0x80000000u;
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  char* const lds = reinterpret_cast<char*>(wsm);
  const dim3 bid = xcd_tile(true);
  const int dz = bid.z, d = dz / a.Z, z = dz % a.Z;
  const int half = bid.x & 1, m0 = (bid.x >> 1) * BM, M = a.M, n0 = half * NH;
  const int kb = z * a.kps, ke = min(a.K, kb + a.kps);
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wu % WM, wn = wu / WM;
  const int nb = wn ? NBL : NB0;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.A[d], (uint32_t)((size_t)ke * a.lda * 4));
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.B1[d], (uint32_t)((size_t)ke * a.ldb1 * 4));
  const __amdgpu_buffer_rsrc_t r2 = make_rsrc(a.B2[d], (uint32_t)((size_t)ke * a.ldb2 * 4));
  auto ld4 = [](const __amdgpu_buffer_rsrc_t& rs, uint32_t o) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
  };
  // A f4s: byte offset at k0 = 0 (OOB past M) and in plane 0 of an A stage
  uint32_t goa[AV];
  int loa[AV];
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    const int x = tid + T * v, k = x / (BM / 4), m = m0 + 4 * (x % (BM / 4));
    goa[v] = m < M ? 4u * (uint32_t)(k * (int)a.lda + m) : OOB;
    loa[v] = k * RA + 8 * (x % (BM / 4));
  }
  // B f4s (per v one uniform source, as gemm_wg3)
  uint32_t gobv[BV], rowbv[BV];
  int lob[BV];
#pragma unroll
  for (int u = 0; u < BV; ++u) {
    int k, c, n;
    bool in;
    if (half == 0 && u < VX) {
      const int x = tid + T * u;
      in = x < BK * QX, k = x / QX, c = 4 * (x % QX), n = c;
    } else if (half == 0) {
      const int x = tid + T * (u - VX);
      in = x < BK * QH0, k = x / QH0, c = N1 + 4 * (x % QH0), n = c - N1;
    } else {
      const int x = tid + T * u;
      in = x < BK * QH1, k = x / QH1, c = 4 * (x % QH1), n = NH - N1 + c;
    }
    const bool x1 = half == 0 && u < VX;
    const int ld = (int)(x1 ? a.ldb1 : a.ldb2);
    rowbv[u] = 4u * (uint32_t)ld;
    gobv[u] = in ? 4u * (uint32_t)(k * ld + n) : OOB;
    lob[u] = in ? OB + k * RB + 2 * c : -1;
  }
  auto glA = [&](int k0, int v) { return ld4(rA, goa[v] + (uint32_t)k0 * 4u * (uint32_t)a.lda); };
  auto glB = [&](int k0, int u) {
    const bool x1 = half == 0 && u < VX;
    return ld4(x1 ? r1 : r2, gobv[u] + (uint32_t)k0 * rowbv[u]);
  };
  auto stA = [&](int stage, int v, const f4& x) {
    u2v h, m, l;
    split4(x, h, m, l);
    char* base = lds + stage * SA + loa[v];
    *reinterpret_cast<u2v*>(base) = h;
    *reinterpret_cast<u2v*>(base + PA) = m;
    *reinterpret_cast<u2v*>(base + 2 * PA) = l;
  };
  auto stB = [&](int u, const f4& x) {
    u2v h, m, l;
    split4(x, h, m, l);
    const bool ok = lob[u] >= 0;
    char* base = lds + (ok ? lob[u] : G::DUMMY + 8 * lane);
    const int pp = ok ? PB : 0;
    *reinterpret_cast<u2v*>(base) = h;
    *reinterpret_cast<u2v*>(base + pp) = m;
    *reinterpret_cast<u2v*>(base + 2 * pp) = l;
  };
  const int offA = (4 * q + (r >> 2)) * RA + 8 * (r & 3) + 2 * (RW * wm);
  const int offB = OB + (4 * q + (r >> 2)) * RB + 8 * (r & 3) + 2 * 16 * NB0 * wn;
  typedef __attribute__((address_space(3))) s4v lds_s4;
  auto trf = [&](int off, int pitch) -> bf8 {
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + off));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + off + 16 * pitch));
    return __builtin_bit_cast(bf8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f4 acc[MI][NB0];
  acc_zero(acc);
  constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
  // the pad columns NT - n0 .. NH of the B planes read as 0 (never stored)
  for (int e = tid; n0 + NH > NT && e < 3 * BK * (n0 + NH - NT); e += T) {
    const int np = n0 + NH - NT, p = e / (BK * np), x = e % (BK * np);
    *reinterpret_cast<short*>(lds + OB + p * PB + (x / np) * RB + 2 * (NT - n0 + x % np)) = 0;
  }
  f4 ra[AV], rb[BV];
#pragma unroll
  for (int v = 0; v < AV; ++v) stA(0, v, glA(kb, v));
#pragma unroll
  for (int u = 0; u < BV; ++u) stB(u, glB(kb, u));
#pragma unroll
  for (int v = 0; v < AV; ++v) ra[v] = glA(kb + BK, v);
#pragma unroll
  for (int u = 0; u < BV; ++u) rb[u] = glB(kb + BK, u);
  __syncthreads();
  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const int sa = cur * SA;
    bf8 ap[MI][3];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) ap[i][p] = trf(sa + p * PA + offA + 2 * 16 * i, RA);
    auto bload = [&](int j, bf8 (&bp)[3]) {
#pragma unroll
      for (int p = 0; p < 3; ++p) bp[p] = trf(p * PB + offB + 2 * 16 * j, RB);
    };
    bf8 bp[3];
    bload(0, bp);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NB0; ++j) {
      bf8 bq[3];
      if (j + 1 < NB0) bload(j + 1, bq);
      if (j < nb) {
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][j] = mfma_bf(ap[i][TA[t]], bp[TB[t]], acc[i][j]);
      }
      constexpr int J0 = 1;  // A f4 j - J0 split into the other A stage in block j
      const bool sj = j >= J0 && j - J0 < AV;
      if (sj) {
        stA(cur ^ 1, j - J0, ra[j - J0]);
        ra[j - J0] = glA(k0 + 2 * BK, j - J0);
      }
      if (j + 1 < NB0) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
      for (int k = 0; k < 6 * MI; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (sj) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      }
      if (sj) {
        __builtin_amdgcn_sched_group_barrier(0x200, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (j + 1 < NB0) bp[0] = bq[0], bp[1] = bq[1], bp[2] = bq[2];
    }
    __syncthreads();  // every wave is done with the B stage
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      stB(u, rb[u]);
      rb[u] = glB(k0 + 2 * BK, u);
    }
    __syncthreads();
    cur ^= 1;
  }
  constexpr int SP = G::SP;
  float* stg = wsm + wu * 16 * SP;
  float* const out = a.slab + (size_t)dz * M * NT;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int j = 0; j < NB0; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) stg[(4 * q + g) * SP + 16 * j + r] = acc[i][j][g];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < NB0; ++p) {
      const int e = lane + 64 * p, lr = e / (4 * NB0), c4 = e % (4 * NB0);
      const int lcol = 16 * NB0 * wn + 4 * c4, gcol = n0 + lcol, grow = m0 + RW * wm + 16 * i + lr;
      if (grow < M && lcol < NH && gcol < NT)
        *reinterpret_cast<f4*>(out + (size_t)grow * NT + gcol) = *reinterpret_cast<const f4*>(stg + lr * SP + 4 * c4);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int N1, int N2, bool W3>
static int wgrad_wg2_launch(hipStream_t s, int nd, const WgDir* dirs, int M, int K, int F, float* scratch,
                            size_t scratch_floats) {
  using G = Wg2<N1, N2>;  // slab geometry (gemm_wg3b writes the same [M][NT] slabs)
  static_assert(Wg3b<N1, N2>::NT == G::NT, "same slab geometry");
  const int tw = W3 ? 2 * cdiv(M, 256) : cdiv(M, G::BM);  // workgroups per (direction, K range)
  int Z = std::max(1, 256 / (nd * tw));
  while ((nd * tw * Z) % 8) ++Z;
  Z = (int)std::min<long>(Z, (long)(scratch_floats / ((size_t)nd * M * G::NT)));
  if (Z < 1) return -1;
  const int kq = W3 ? 64 : 32, kps = ((cdiv(K, Z) + kq - 1) / kq) * kq;
  Z = cdiv(K, kps);
  WgArgs a{};
  WgOut o{};
  for (int d = 0; d < nd; ++d) {
    a.A[d] = dirs[d].dG; a.B1[d] = dirs[d].X; a.B2[d] = dirs[d].Hprev;
    o.w_ih[d] = dirs[d].w_ih; o.b_ih[d] = dirs[d].b_ih; o.b_hh[d] = dirs[d].b_hh; o.w_hh[d] = dirs[d].w_hh;
  }
  a.lda = M; a.ldb1 = N1; a.ldb2 = N2; a.M = M; a.K = K; a.kps = kps; a.Z = Z; a.slab = scratch;
  if (W3) {
    static bool attr_b = false;
    if (!attr_b) {
      ABCD_TRY(hipFuncSetAttribute((const void*)gemm_wg3b_kernel<N1, N2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)Wg3b<N1, N2>::LDS));
      attr_b = true;
    }
    gemm_wg3b_kernel<N1, N2><<<dim3(tw, 1, nd * Z), 512, Wg3b<N1, N2>::LDS, s>>>(a);
  } else {
    static bool attr = false;
    if (!attr) {
      ABCD_TRY(hipFuncSetAttribute((const void*)gemm_wg2_kernel<N1, N2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)G::LDS));
      attr = true;
    }
    gemm_wg2_kernel<N1, N2><<<dim3(tw, 1, nd * Z), 256, G::LDS, s>>>(a);
  }
  ABCD_CHECK_LAUNCH();
  const long nq = (long)nd * M * G::NT / 4;
  wg2_reduce_kernel<<<(int)std::min<long>(2048, cdiv(nq, 256)), 256, 0, s>>>(scratch, nd, Z, M, G::NT, N1, F,
                                                                             N2, o);
  ABCD_CHECK_LAUNCH();
  return 0;
}

int wgrad_lstm_l0(hipStream_t s, int nd, const WgDir* dirs, int M, int K, int F, int Fp, int H, float* scratch,
                  size_t scratch_floats) {
  if (nd < 1 || nd > 2 || K <= 0 || F >= Fp || !scratch) return -1;
  const char* ev = getenv("ABCD_WG2");
  if (ev && ev[0] == '0') return -1;
  // 32-bit buffer offsets: every operand's K range below 2 GiB
  if ((size_t)K * M * 4 >= (1ull << 31) || (size_t)K * Fp * 4 >= (1ull << 31) || (size_t)K * H * 4 >= (1ull << 31))
    return -1;
  for (int d = 0; d < nd; ++d)
    if (((uintptr_t)dirs[d].dG | (uintptr_t)dirs[d].X | (uintptr_t)dirs[d].Hprev) & 15) return -1;
  if (M % 4) return -1;
  if (Fp == 144 && H == 256)
    return wg3_on() ? wgrad_wg2_launch<144, 256, true>(s, nd, dirs, M, K, F, scratch, scratch_floats)
                    : wgrad_wg2_launch<144, 256, false>(s, nd, dirs, M, K, F, scratch, scratch_floats);
  return -1;
}

// ABCD_WG3=0 selects gemm_wg2 (fragments split by every wave in the MFMA loop)
bool wg3_on() {
  const char* v = getenv("ABCD_WG3");
  return !(v && v[0] == '0');
}
// the dispatch record's name of the form wgrad_lstm_l0 runs (printf format, Fp, H, nd)
const char* wg_dispatch_fmt() { return wg3_on() ? "gemm_wg3b<%d,%d> x%d" : "gemm_wg2<%d,%d> x%d"; }

template <int MR, int NR, bool AKC, bool BKC, bool ONE = false>
static int gemm_x6s_launch(hipStream_t s, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                           EpiArgs e, float* scratch, size_t scratch_floats) {
  const int BM = 32 * MR, BN = 32 * NR;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int Z = std::max(1, std::min(cdiv(tl_side ? 256 : 512, tiles), cdiv(K, 32 * 16)));
  if (scratch) Z = (int)std::min<long>(Z, (long)(scratch_floats / ((size_t)M * N)));
  else Z = 1;
  Z = std::max(Z, 1);
  const int kps = ((cdiv(K, Z) + 31) / 32) * 32;
  Z = cdiv(K, kps);
  EpiArgs ek = e;
  if (Z > 1) ek.slab = scratch;
  gemm_x6s_kernel<MR, NR, AKC, BKC, ONE><<<dim3(cdiv(N, BN), cdiv(M, BM), Z), 256, 0, s>>>(A, lda, B, ldb, K, kps,
                                                                                          ek, 1);
  ABCD_CHECK_LAUNCH();
  if (Z > 1) {
    ABCD_TRY((hipError_t)slab_reduce(s, scratch, Z, e));
  }
  return 0;
}


static bool tn_ok(const Operand& o, int rows) {
  return o.kmajor && o.ld % 4 == 0 && ((uintptr_t)o.p % 16) == 0 && o.ld >= ((rows + 3) & ~3);
}


int gemm(hipStream_t s, int M, int N, int K, Operand A, Operand B, float* C, long ldc, float alpha,
         float beta, const float* bias, int act, float* scratch, size_t scratch_floats) {
  if (M <= 0 || N <= 0) return 0;
  EpiArgs e{C, ldc, M, N, alpha, beta, bias, act, nullptr};
  if (K <= 0) {  // C = beta*C + bias
    KC za{A.p, 16, 0};
    KC zb{B.p, 16, 0};
    return gemm_launch(s, M, N, 16, za, zb, e, nullptr, 0);
  }
  if (!A.kmajor) ABCD_REQUIRE(K % 16 == 0 && A.ld % 4 == 0 && ((uintptr_t)A.p % 16) == 0);
  if (!B.kmajor) ABCD_REQUIRE(K % 16 == 0 && B.ld % 4 == 0 && ((uintptr_t)B.p % 16) == 0);
  if (!A.kmajor && !B.kmajor) {
    // frame-parallel GEMMs (M = packed frames): LDS-staged tiles, 128 x 256 (measured
    // ~1.6x the direct-fragment gemm_big at the input-projection shape)
    if (cdiv(M, 128) * cdiv(N, 128) >= 240 && A.nrows >= M && B.nrows >= N && A.ld % 4 == 0 && B.ld % 4 == 0 &&
        ((uintptr_t)A.p % 16) == 0 && ((uintptr_t)B.p % 16) == 0) {
      if (!tl_side) {
        // fragment-staged form (one split per workgroup) when both operands fit a buffer resource
        if (K % 8 == 0 && (size_t)M * A.ld * 4 < (1ull << 31) && (size_t)N * B.ld * 4 < (1ull << 31)) {
          // short K: B slice resident, frames streamed (gemm_x6r8)
          // (K in (128, 144]: the half-empty last chunk on 16-deep MFMAs, T16;
          // zero-padded to 32-deep it ran 269-282 against 266-267 us)
          if (K <= 160)
            return (K > 128 && K <= 144) ? gemm_x6r8_launch<5, 128, 2, 8, 0, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e)
                                         : gemm_x6r8_launch<5, 128, 2, 8>(s, M, N, K, A.p, A.ld, B.p, B.ld, e);
          if (K <= 256) return gemm_x6r8_launch<8, 64, 2, 16>(s, M, N, K, A.p, A.ld, B.p, B.ld, e);
          return gemm_x6f_launch<4, 4>(s, M, N, K, A.p, A.ld, B.p, B.ld, e);
        }
        return gemm_x6s_launch<4, 4, true, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, nullptr, 0);
      }
      if (N >= 256) return gemm_tn_launch<4, 8, true, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, nullptr, 0);
      return gemm_tn_launch<4, 4, true, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, nullptr, 0);
    }
    return gemm_launch(s, M, N, K, KC{A.p, A.ld, std::min(A.nrows, M)}, KC{B.p, B.ld, std::min(B.nrows, N)}, e,
                       scratch, scratch_floats);
  }
  if (A.kmajor && !B.kmajor)
    return gemm_launch(s, M, N, K, KM{A.p, A.ld, std::min(A.nrows, M), K}, KC{B.p, B.ld, std::min(B.nrows, N)}, e,
                       scratch, scratch_floats);
  if (!A.kmajor && B.kmajor)
    return gemm_launch(s, M, N, K, KC{A.p, A.ld, std::min(A.nrows, M)}, KM{B.p, B.ld, std::min(B.nrows, N), K}, e,
                       scratch, scratch_floats);
  // gemm_tn for the frame-reduction shapes (K = packed frames); short K (the
  // batch-reduction weight gradients, K = B = 512) goes to gemm_ks, whose
  // 32 x 64 tiles and grid split-K fill the chip (gemm_tn's 128 x 256 tiles
  // leave ~16 workgroups: ~100-170 us per GEMM measured, vs ~10)
  if (K >= 4096 && A.nrows >= M && B.nrows >= N && tn_ok(A, M) && tn_ok(B, N)) {
    if (!tl_side) {  // 66-76 KB of LDS: not beside a persistent kernel
      if (N > 128 && N <= 160)  // one 160-wide tile (e.g. dW_ih, N = F = 129)
        return gemm_x6s_launch<4, 5, false, false>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, scratch, scratch_floats);
      if ((size_t)K * A.ld * 4 < (1ull << 31) && (size_t)K * B.ld * 4 < (1ull << 31))
        return gemm_x6t_launch<4, 4>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, scratch, scratch_floats);
      return gemm_x6s_launch<4, 4, false, false>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, scratch, scratch_floats);
    }
    // beside the encoder BPTT (side mode): split-fp32 on one operand stage
    // (34 KB, 204 VGPRs: fits beside enc_bwd_w8's 120 KB / 256 registers);
    // the fp32-MFMA gemm_tn tiles it replaced cost the BPTT 0.2 ms of matrix
    // pipe
    if (N > 128 && N <= 160)
      return gemm_x6s_launch<4, 5, false, false, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, scratch, scratch_floats);
    if (M > 128 && M <= 160)
      return gemm_x6s_launch<5, 4, false, false, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, scratch, scratch_floats);
    return gemm_x6s_launch<4, 4, false, false, true>(s, M, N, K, A.p, A.ld, B.p, B.ld, e, scratch, scratch_floats);
  }
  return gemm_launch(s, M, N, K, KM{A.p, A.ld, std::min(A.nrows, M), K}, KM{B.p, B.ld, std::min(B.nrows, N), K},
                     e, scratch, scratch_floats);
}

// A B^T as raw split-K partial slabs (no epilogue): slab[z][m*N + n] for
// z < *zout, K split the way gemm() splits a small-M product; the consumer
// sums the slabs (the sampler head fuses that reduce into its prologue).
int gemm_slabs(hipStream_t s, int M, int N, int K, Operand A, Operand B, float* slab, size_t slab_floats, int* zout) {
  ABCD_REQUIRE(M > 0 && N > 0 && K > 0 && K % 16 == 0 && !A.kmajor && !B.kmajor && slab && zout);
  ABCD_REQUIRE(A.ld % 4 == 0 && B.ld % 4 == 0 && ((uintptr_t)A.p % 16) == 0 && ((uintptr_t)B.p % 16) == 0);
  const long per = (long)M * N;
  ABCD_REQUIRE((long)slab_floats >= per);
  const int nch = K / 16, tiles = cdiv(M, 32) * cdiv(N, 64);
  int Z = std::min(cdiv(1024, tiles), std::max(1, nch / 8));
  Z = (int)std::max<long>(1, std::min<long>(Z, (long)slab_floats / per));
  const int cps = cdiv(nch, Z);
  Z = cdiv(nch, cps);
  EpiArgs e{nullptr, N, M, N, 1.f, 0.f, nullptr, ACT_NONE, slab};
  dim3 grid(cdiv(N, 64), cdiv(M, 32), Z);
  gemm_ks_kernel<2, 4, KC, KC><<<grid, 256, 0, s>>>(KC{A.p, A.ld, std::min(A.nrows, M)},
                                                    KC{B.p, B.ld, std::min(B.nrows, N)}, nch, cps, e);
  ABCD_CHECK_LAUNCH();
  *zout = Z;
  return 0;
}

size_t gemm_scratch_floats_hint(int M, int N, int K) { return (size_t)M * N * 16; }

// ---------------------------------------------------------------------------
// column sums (bias gradients, GEMV-T): out[j] = beta*out[j] + sum_r w[r] Z[r][j]
// pass 1: block = 64 columns x 4 row groups over one row slice (coalesced
// 256-B rows, 4 independent accumulators per thread); pass 2 sums the slices.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void colsum_pass1(const float* Z, long ldz, int nrows, int ncols, const float* w,
                                                    int rows_per, float* part) {
  __shared__ float sh[4][64];
  const int cg = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cg;
  const int r0 = blockIdx.y * rows_per, r1 = min(nrows, r0 + rows_per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < ncols) {
    int r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      s0 += (w ? w[r] : 1.f) * Z[(long)r * ldz + j];
      s1 += (w ? w[r + 4] : 1.f) * Z[(long)(r + 4) * ldz + j];
      s2 += (w ? w[r + 8] : 1.f) * Z[(long)(r + 8) * ldz + j];
      s3 += (w ? w[r + 12] : 1.f) * Z[(long)(r + 12) * ldz + j];
    }
    for (; r < r1; r += 4) s0 += (w ? w[r] : 1.f) * Z[(long)r * ldz + j];
  }
  sh[rg][cg] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (rg == 0 && j < ncols) part[(long)blockIdx.y * ncols + j] = (sh[0][cg] + sh[1][cg]) + (sh[2][cg] + sh[3][cg]);
}
// pass 2: 64 columns x 4 slice groups per block, 4 independent accumulators
// per thread (the slice count reaches 256: keep many loads in flight)
__global__ __launch_bounds__(256) void colsum_pass2(const float* part, int nslices, int ncols, float* out,
                                                    float beta, float* out2) {
  __shared__ float sh[4][64];
  const int cg = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cg;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < ncols) {
    int z = sg;
    for (; z + 12 < nslices; z += 16) {
      s0 += part[(long)z * ncols + j];
      s1 += part[(long)(z + 4) * ncols + j];
      s2 += part[(long)(z + 8) * ncols + j];
      s3 += part[(long)(z + 12) * ncols + j];
    }
    for (; z < nslices; z += 4) s0 += part[(long)z * ncols + j];
  }
  sh[sg][cg] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sg == 0 && j < ncols) {
    const float v = (sh[0][cg] + sh[1][cg]) + (sh[2][cg] + sh[3][cg]);
    out[j] = (beta != 0.f ? beta * out[j] : 0.f) + v;
    if (out2) out2[j] = (beta != 0.f ? beta * out2[j] : 0.f) + v;
  }
}

int colsum(hipStream_t s, const float* Z, long ldz, int nrows, int ncols, const float* w, float* out,
           float beta, float* scratch, size_t scratch_floats, float* out2) {
  if (ncols <= 0) return 0;
  const int cblocks = cdiv(ncols, 64);
  // slices of >= 16 rows (one 4-load round per thread) until ~1024 workgroups:
  // the short batch reductions (nrows = B = 512) take 32 slices instead of 2
  // slices of 256 rows (16 dependent load rounds, ~18 us); the frame
  // reductions (nrows = L) keep the 1024-workgroup cap
  int slices = std::max(1, std::min(cdiv(std::max(nrows, 1), 16), std::max(1, 1024 / cblocks)));
  slices = std::min(slices, 256);
  slices = (int)std::max<long>(1, std::min<long>(slices, (long)(scratch_floats / (size_t)ncols)));
  const int rows_per = cdiv(std::max(nrows, 1), slices);
  slices = std::max(1, cdiv(std::max(nrows, 1), rows_per));
  colsum_pass1<<<dim3(cblocks, slices), 256, 0, s>>>(Z, ldz, nrows, ncols, w, rows_per, scratch);
  ABCD_CHECK_LAUNCH();
  colsum_pass2<<<cdiv(ncols, 64), 256, 0, s>>>(scratch, slices, ncols, out, beta, out2);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// colsum_batch: up to COLSUM_BATCH_MAX column sums in one pass-1 and one
// pass-2 launch (the decoder backward's bias gradients: seven pairs of
// launches before).  Each job keeps colsum()'s slicing, so its sum is the
// same, bit for bit.
struct ColsumBatchArgs {
  ColsumJob j[COLSUM_BATCH_MAX];
  int slices[COLSUM_BATCH_MAX], rows_per[COLSUM_BATCH_MAX];
  long part0[COLSUM_BATCH_MAX];    // offset of the job's partials in `part`
  int b1[COLSUM_BATCH_MAX + 1];    // first pass-1 block of each job (blocks = column blocks x slices)
  int b2[COLSUM_BATCH_MAX + 1];    // first pass-2 block (column blocks)
  int n;
  float* part;
};
__global__ __launch_bounds__(256) void colsum_batch_pass1(ColsumBatchArgs a) {
  __shared__ float sh[4][64];
  int ji = 0;
  while (ji + 1 < a.n && (int)blockIdx.x >= a.b1[ji + 1]) ++ji;
  const ColsumJob J = a.j[ji];
  const int cb = (J.ncols + 63) / 64, t = (int)blockIdx.x - a.b1[ji];
  const int cg = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = (t % cb) * 64 + cg, sl = t / cb;
  const int r0 = sl * a.rows_per[ji], r1 = min(J.nrows, r0 + a.rows_per[ji]);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < J.ncols) {
    const float* w = J.w;
    const float* Z = J.Z;
    const long ldz = J.ldz;
    int r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      s0 += (w ? w[r] : 1.f) * Z[(long)r * ldz + j];
      s1 += (w ? w[r + 4] : 1.f) * Z[(long)(r + 4) * ldz + j];
      s2 += (w ? w[r + 8] : 1.f) * Z[(long)(r + 8) * ldz + j];
      s3 += (w ? w[r + 12] : 1.f) * Z[(long)(r + 12) * ldz + j];
    }
    for (; r < r1; r += 4) s0 += (w ? w[r] : 1.f) * Z[(long)r * ldz + j];
  }
  sh[rg][cg] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (rg == 0 && j < J.ncols)
    a.part[a.part0[ji] + (long)sl * J.ncols + j] = (sh[0][cg] + sh[1][cg]) + (sh[2][cg] + sh[3][cg]);
}
__global__ __launch_bounds__(256) void colsum_batch_pass2(ColsumBatchArgs a) {
  __shared__ float sh[4][64];
  int ji = 0;
  while (ji + 1 < a.n && (int)blockIdx.x >= a.b2[ji + 1]) ++ji;
  const ColsumJob J = a.j[ji];
  const int cg = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int j = ((int)blockIdx.x - a.b2[ji]) * 64 + cg, nsl = a.slices[ji];
  const float* part = a.part + a.part0[ji];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < J.ncols) {
    int z = sg;
    for (; z + 12 < nsl; z += 16) {
      s0 += part[(long)z * J.ncols + j];
      s1 += part[(long)(z + 4) * J.ncols + j];
      s2 += part[(long)(z + 8) * J.ncols + j];
      s3 += part[(long)(z + 12) * J.ncols + j];
    }
    for (; z < nsl; z += 4) s0 += part[(long)z * J.ncols + j];
  }
  sh[sg][cg] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sg == 0 && j < J.ncols) {
    const float v = (sh[0][cg] + sh[1][cg]) + (sh[2][cg] + sh[3][cg]);
    J.out[j] = (J.beta != 0.f ? J.beta * J.out[j] : 0.f) + v;
    if (J.out2) J.out2[j] = (J.beta != 0.f ? J.beta * J.out2[j] : 0.f) + v;
  }
}
int colsum_batch(hipStream_t s, const ColsumJob* jobs, int n, float* scratch, size_t scratch_floats) {
  if (n <= 0) return 0;
  if (n > COLSUM_BATCH_MAX) return (int)hipErrorInvalidValue;
  ColsumBatchArgs a{};
  long used = 0;
  int k = 0, nb1 = 0, nb2 = 0;
  for (int i = 0; i < n; ++i) {
    const ColsumJob& J = jobs[i];
    if (J.ncols <= 0) continue;
    const int cblocks = cdiv(J.ncols, 64);
    // colsum()'s slicing, with the scratch shared by the jobs
    int slices = std::max(1, std::min(cdiv(std::max(J.nrows, 1), 16), std::max(1, 1024 / cblocks)));
    slices = std::min(slices, 256);
    const long left = (long)scratch_floats - used;
    if (left < J.ncols) return (int)hipErrorInvalidValue;
    slices = (int)std::max<long>(1, std::min<long>(slices, left / J.ncols));
    const int rows_per = cdiv(std::max(J.nrows, 1), slices);
    slices = std::max(1, cdiv(std::max(J.nrows, 1), rows_per));
    a.j[k] = J;
    a.slices[k] = slices;
    a.rows_per[k] = rows_per;
    a.part0[k] = used;
    a.b1[k] = nb1;
    a.b2[k] = nb2;
    used += (long)slices * J.ncols;
    nb1 += cblocks * slices;
    nb2 += cblocks;
    ++k;
  }
  if (!k) return 0;
  a.n = k;
  a.b1[k] = nb1;
  a.b2[k] = nb2;
  a.part = scratch;
  colsum_batch_pass1<<<nb1, 256, 0, s>>>(a);
  ABCD_CHECK_LAUNCH();
  colsum_batch_pass2<<<nb2, 256, 0, s>>>(a);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// layout copies (padding / transposition of weight compute copies)
// ---------------------------------------------------------------------------
__global__ void pack2d_kernel(const float* src, long lds, int sr, int sc, int trans, float* dst, long ldd, int dr,
                              int dc) {
  const long n = (long)dr * dc;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / dc), c = (int)(i % dc);
    float v = 0.f;
    if (r < sr && c < sc) v = trans ? src[(long)c * lds + r] : src[(long)r * lds + c];
    dst[(long)r * ldd + c] = v;
  }
}
int pack2d(hipStream_t s, const float* src, long lds, int sr, int sc, bool trans, float* dst, long ldd, int dr,
           int dc) {
  const long n = (long)dr * dc;
  if (n <= 0) return 0;
  pack2d_kernel<<<(int)std::min<long>(4096, cdiv(n, 256)), 256, 0, s>>>(src, lds, sr, sc, trans, dst, ldd, dr, dc);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// several pack2d / add_vec jobs in ONE launch (blockIdx.y = job): the
// per-step weight re-layouts of a module are ~10 tiny kernels otherwise,
// each paying a ~5 us launch slot on the step's critical path
// One launch for a list of pad / transpose copies.  A thread owns 4 adjacent
// destination columns of a row (one 16-B store where the row is aligned: the
// frame pad writes L x Fp floats per step); 32-bit index arithmetic (the
// host checks dr * dc < 2^31).
__global__ void pack_many_kernel(PackList pl) {
  const PackJob& j = pl.j[blockIdx.y];
  const int cq = (j.dc + 3) >> 2;
  const int n = j.dr * cq;
  const bool vec = ((j.ldd & 3) == 0) && ((reinterpret_cast<uintptr_t>(j.dst) & 15) == 0);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / cq, c0 = (i - r * cq) * 4;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + k;
      v[k] = 0.f;
      if (r < j.sr && c < j.sc) {
        const long o = j.trans ? (long)c * j.lds + r : (long)r * j.lds + c;
        v[k] = j.src[o];
        if (j.src2) v[k] += j.src2[o];
      } else if (j.ones && r < j.sr && c == j.sc) {
        v[k] = 1.f;
      }
    }
    float* d = j.dst + (long)r * j.ldd + c0;
    if (vec && c0 + 4 <= j.dc) {
      *reinterpret_cast<f4*>(d) = f4{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c0 + k < j.dc) d[k] = v[k];
    }
  }
}
int Packs::add(const float* src, long lds, int sr, int sc, bool trans, float* dst, long ldd, int dr, int dc,
               const float* src2, bool ones) {
  if ((long)dr * dc <= 0) return 0;
  if ((long)dr * (dc + 3) >= (1L << 31)) return ABCD_EINVAL;  // the kernel's 32-bit indices
  if (pl.n == ABCD_PACK_MAX) ABCD_TRY((hipError_t)flush());
  pl.j[pl.n++] = PackJob{src, src2, lds, dst, ldd, sr, sc, dr, dc, trans ? 1 : 0, ones ? 1 : 0};
  maxn = std::max(maxn, (long)dr * ((dc + 3) / 4));
  return 0;
}
int Packs::flush() {
  if (pl.n == 0) return 0;
  const int gx = (int)std::min<long>(2048, cdiv(maxn, 256));
  pack_many_kernel<<<dim3(gx, pl.n), 256, 0, s>>>(pl);
  ABCD_CHECK_LAUNCH();
  pl.n = 0;
  maxn = 0;
  return 0;
}

__global__ void mul_vec_kernel(const float* a, const float* b, float* y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = a[i] * b[i];
}
int mul_vec(hipStream_t s, const float* a, const float* b, float* y, long n) {
  if (n <= 0) return 0;
  mul_vec_kernel<<<(int)std::min<long>(4096, cdiv(n, 256)), 256, 0, s>>>(a, b, y, n);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// training-mode dropout noise (nn.Dropout / torch.nn.LSTM(dropout)): bernoulli(1 - p) / (1 - p)
// from the Philox stream (seed, offset + i)
__global__ void fill_dropout_kernel(float* out, long n, float keep, float scale, uint64_t seed, uint64_t offset) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t o[4];
    philox4x32(seed, offset + (uint64_t)i, o);
    out[i] = u01(o[0]) <= keep ? scale : 0.f;
  }
}

__global__ void add_vec_kernel(const float* a, const float* b, float* y, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = a[i] + b[i];
}
int add_vec(hipStream_t s, const float* a, const float* b, float* y, int n) {
  if (n <= 0) return 0;
  add_vec_kernel<<<cdiv(n, 256), 256, 0, s>>>(a, b, y, n);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// deterministic sum of a float array -> float (and double) scalar
// ---------------------------------------------------------------------------
DEV double block_sum_d(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  __syncthreads();
  return t;
}
__global__ void reduce_pass1(const float* x, long n, double* part) {
  __shared__ double sh[16];
  double v = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) v += x[i];
  v = block_sum_d(v, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}
__global__ void reduce_pass2(const double* part, int np, float* out, double* out64) {
  __shared__ double sh[16];
  double v = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) v += part[i];
  v = block_sum_d(v, sh);
  if (threadIdx.x == 0) {
    if (out) *out = (float)v;
    if (out64) *out64 = v;
  }
}
int reduce_sum(hipStream_t s, const float* x, long n, double* partials, float* out, double* out64) {
  const int nb = (int)std::max<long>(1, std::min<long>(1024, cdiv(n, 256)));
  reduce_pass1<<<nb, 256, 0, s>>>(x, n, partials);
  ABCD_CHECK_LAUNCH();
  reduce_pass2<<<1, 256, 0, s>>>(partials, nb, out, out64);
  ABCD_CHECK_LAUNCH();
  return 0;
}

}  // namespace abcd

// ---------------------------------------------------------------------------
// C ABI: plain GEMM (used by tests to check the MFMA core against the oracle)
// ---------------------------------------------------------------------------
extern "C" int abcd_gemm_nt(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C,
                            long ldc, const float* bias, void* ws, size_t ws_bytes, void* stream) {
  using namespace abcd;
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (K % 16 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0)
    return gemm(s, M, N, K, opKC(A, lda, M), opKC(B, ldb, N), C, ldc, 1.f, 0.f, bias, ACT_NONE, (float*)ws,
                ws_bytes / 4);
  // arbitrary K: read both operands K-major-style (transposed view) -> KM path handles tails
  // (A(m,k) = A[m*lda+k] is a KM operand with ld=1 over rows of stride lda? no: use a padded copy)
  const int Kp = rup16(K);
  const size_t need = ((size_t)M + N) * Kp;
  if (ws_bytes / 4 < need) return ABCD_EINVAL;
  float* Ap = (float*)ws;
  float* Bp = Ap + (size_t)M * Kp;
  ABCD_TRY((hipError_t)pack2d(s, A, lda, M, K, false, Ap, Kp, M, Kp));
  ABCD_TRY((hipError_t)pack2d(s, B, ldb, N, K, false, Bp, Kp, N, Kp));
  float* rest = Bp + (size_t)N * Kp;
  const size_t rest_f = ws_bytes / 4 - need;
  return gemm(s, M, N, Kp, opKC(Ap, Kp, M), opKC(Bp, Kp, N), C, ldc, 1.f, 0.f, bias, ACT_NONE, rest, rest_f);
}

// C ABI: C = A^T @ B with A (K x M, lda) and B (K x N, ldb) row-major: the
// weight-gradient GEMM shape (reduction over rows); used by tests
extern "C" int abcd_gemm_tn(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C,
                            long ldc, void* ws, size_t ws_bytes, void* stream) {
  using namespace abcd;
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C || lda < M || ldb < N) return ABCD_EINVAL;
  return gemm((hipStream_t)stream, M, N, K, opKM(A, lda, M), opKM(B, ldb, N), C, ldc, 1.f, 0.f, nullptr, ACT_NONE,
              (float*)ws, ws_bytes / 4);
}

// C ABI: y = act(x @ W^T + b), act 0 = none, 1 = tanh (nn.Linear [+ Tanh]); any K
extern "C" int abcd_linear(int M, int N, int K, const float* x, long ldx, const float* W, long ldw, const float* b,
                           int act, float* y, long ldy, void* ws, size_t ws_bytes, void* stream) {
  using namespace abcd;
  if (M < 0 || N < 0 || K < 0 || !x || !W || !y || (act != ACT_NONE && act != ACT_TANH)) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (K % 16 == 0 && ldx % 4 == 0 && ldw % 4 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)W % 16) == 0)
    return gemm(s, M, N, K, opKC(x, ldx, M), opKC(W, ldw, N), y, ldy, 1.f, 0.f, b, act, (float*)ws, ws_bytes / 4);
  const int Kp = rup16(K);
  const size_t need = ((size_t)M + N) * Kp;
  if (ws_bytes / 4 < need) return ABCD_EINVAL;
  float* xp = (float*)ws;
  float* wp = xp + (size_t)M * Kp;
  ABCD_TRY((hipError_t)pack2d(s, x, ldx, M, K, false, xp, Kp, M, Kp));
  ABCD_TRY((hipError_t)pack2d(s, W, ldw, N, K, false, wp, Kp, N, Kp));
  return gemm(s, M, N, Kp, opKC(xp, Kp, M), opKC(wp, Kp, N), y, ldy, 1.f, 0.f, b, act, wp + (size_t)N * Kp,
              ws_bytes / 4 - need);
}

namespace abcd {
// dy' = dy (act none) or dy (1 - y^2) (tanh) into an M x Np buffer, zero in the padding columns
__global__ void linear_dact(const float* dy, long lddy, const float* y, long ldy, int act, int M, int N, int Np,
                            float* out) {
  const long n = (long)M * Np;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / Np), j = (int)(i - (long)m * Np);
    float v = 0.f;
    if (j < N) {
      v = dy[(long)m * lddy + j];
      if (act == ACT_TANH) {
        const float t = y[(long)m * ldy + j];
        v *= 1.f - t * t;
      }
    }
    out[i] = v;
  }
}
static size_t linear_bwd_floats(int M, int N, int K) {
  const size_t Np = rup16(N), K4 = (K + 3) & ~3;
  return (size_t)M * Np + Np * K4 + (size_t)M * K4 + ((size_t)1 << 20) + 3 * 64;
}
}  // namespace abcd

extern "C" size_t abcd_linear_backward_workspace_bytes(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 ? abcd::linear_bwd_floats(M, N, K) * 4 : 0;
}

// C ABI: backward of abcd_linear (y = act(x W^T + b)): dx = dy' W, dW = dy'^T x,
// db = sum_m dy' with dy' = dy (1 - y^2) for tanh; each output may be NULL
extern "C" int abcd_linear_backward(int M, int N, int K, const float* x, long ldx, const float* W, long ldw,
                                    const float* y, long ldy, int act, const float* dy, long lddy, float* dx,
                                    long lddx, float* dW, float* db, void* ws, size_t ws_bytes, void* stream) {
  using namespace abcd;
  if (M <= 0 || N <= 0 || K <= 0 || !dy || !ws || (act != ACT_NONE && act != ACT_TANH)) return ABCD_EINVAL;
  if ((act == ACT_TANH && !y) || (dx && !W) || (dW && !x)) return ABCD_EINVAL;
  if (ws_bytes / 4 < linear_bwd_floats(M, N, K)) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int Np = rup16(N), K4 = (K + 3) & ~3;
  Arena A(ws, ws_bytes);
  float* dyp = A.f((size_t)M * Np);
  float* Wp = A.f((size_t)Np * K4);
  float* xp = A.f((size_t)M * K4);
  float* sc = A.f((size_t)1 << 20);
  ABCD_REQUIRE(A.ok);
  linear_dact<<<(int)std::min<long>(4096, cdiv((long)M * Np, 256)), 256, 0, s>>>(dy, lddy, y, ldy, act, M, N, Np,
                                                                                  dyp);
  ABCD_CHECK_LAUNCH();
  if (dx) {  // dx(m, k) = sum_n dy'(m, n) W(n, k)
    ABCD_TRY((hipError_t)pack2d(s, W, ldw, N, K, false, Wp, K4, Np, K4));
    ABCD_TRY((hipError_t)gemm(s, M, K, Np, opKC(dyp, Np, M), opKM(Wp, K4, K), dx, lddx, 1.f, 0.f, nullptr, ACT_NONE,
                              nullptr, 0));
  }
  if (dW) {  // dW(n, k) = sum_m dy'(m, n) x(m, k)
    ABCD_TRY((hipError_t)pack2d(s, x, ldx, M, K, false, xp, K4, M, K4));
    ABCD_TRY((hipError_t)gemm(s, N, K, M, opKM(dyp, Np, N), opKM(xp, K4, K), dW, K, 1.f, 0.f, nullptr, ACT_NONE, sc,
                              (size_t)1 << 20));
  }
  if (db) ABCD_TRY((hipError_t)colsum(s, dyp, Np, M, N, nullptr, db, 0.f, sc, (size_t)1 << 20));
  return 0;
}

extern "C" int abcd_fill_dropout(float* out, long n, float p, uint64_t seed, uint64_t offset, void* stream) {
  if (!out || n < 0 || !(p >= 0.f && p < 1.f)) return ABCD_EINVAL;
  if (n == 0) return 0;
  const float keep = 1.0f - p;
  abcd::fill_dropout_kernel<<<(int)std::min<long>(4096, abcd::cdiv(n, 256)), 256, 0, (hipStream_t)stream>>>(
      out, n, keep, 1.0f / keep, seed, offset);
  return (int)hipGetLastError();
}
