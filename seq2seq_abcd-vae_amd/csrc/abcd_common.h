// abcd_common.h -- shared device building blocks for the ABCD-VAE CDNA4 kernels.
//
// Everything here is written for gfx950 (MI355X): 64-lane waves, the f32-input
// matrix core `v_mfma_f32_16x16x4_f32` (exact f32, 64 FLOP/clk/SIMD), per-CU LDS.
//
// GEMM convention used by every kernel in this library
// ----------------------------------------------------
//   C[m][n] = sum_k A(m, k) * B(n, k)
// Both operands are addressed as (row, k).  An operand is either
//   * KC ("K-contiguous"): element (row, k) at p[row*ld + k]  (row-major A, or
//     a weight matrix W[n][k] used as x @ W^T) -- loaded as float4 along k;
//   * KM ("K-major"):      element (row, k) at p[k*ld + row]  (e.g. dG^T when
//     the reduction runs over the packed-frame axis) -- loaded as 4 dwords,
//     16 lanes reading 16 consecutive rows (64-B segments).
// K is walked in chunks of 16.  Inside a chunk lane (r = lane&15, q = lane>>4)
// supplies k = 16*kc + 4*q + s to MFMA step s (s = 0..3): the float4 of a KC
// operand therefore feeds four consecutive MFMAs with no shuffles.  The same
// k assignment is used for A and B, so every k is summed exactly once.
// Accumulator subtile (16x16): lane holds rows 4*q + {0..3}, column r.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__
typedef float f4 __attribute__((ext_vector_type(4)));

namespace abcd {

DEV f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
DEV f4 f4zero() { f4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

DEV float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
DEV float tanhf_(float x) { return tanhf(x); }
// short-latency forms for the recurrent critical path (v_exp + v_rcp, ~1 ulp
// each; tanh via 1 - 2/(1 + e^{2x}): absolute error ~1e-7 near 0)
DEV float fsigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
DEV float ftanh(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

// ---------------------------------------------------------------------------
// operand views
// ---------------------------------------------------------------------------
struct KC {
  const float* p; long ld; int nrows;
  DEV f4 frag(int row, int kc, int q) const {
    if (row < nrows) return *reinterpret_cast<const f4*>(p + (long)row * ld + kc * 16 + 4 * q);
    return f4zero();
  }
};
struct KM {
  const float* p; long ld; int nrows; int nk;
  DEV f4 frag(int row, int kc, int q) const {
    f4 v = f4zero();
    if (row < nrows) {
      int k0 = kc * 16 + 4 * q;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (k0 + s < nk) v[s] = p[(long)(k0 + s) * ld + row];
    }
    return v;
  }
};

// One wave accumulates MR x NR 16x16 subtiles over chunks kc0, kc0+step, ... < kc1.
// ar[i] / br[j]: absolute operand row this lane supplies for subtile i / j.
// PD chunks of operand loads are kept in flight (register ring): the step
// kernels are latency-bound on L2/MALL hits, so memory-level parallelism, not
// MFMA issue, sets their speed (measured: PD=1 -> ~1.3 us per chunk).
template <int MR, int NR, int PD = 4, class OA, class OB>
DEV void wave_mma(f4 (&acc)[MR][NR], const OA& A, const int (&ar)[MR], const OB& B, const int (&br)[NR],
                  int kc0, int kc1, int step, int q) {
  if (kc0 >= kc1) return;
  f4 a[PD][MR], b[PD][NR];
#pragma unroll
  for (int p = 0; p < PD; ++p) {
    const int kc = kc0 + p * step;
    if (kc < kc1) {
#pragma unroll
      for (int i = 0; i < MR; ++i) a[p][i] = A.frag(ar[i], kc, q);
#pragma unroll
      for (int j = 0; j < NR; ++j) b[p][j] = B.frag(br[j], kc, q);
    }
  }
  for (int base = kc0; base < kc1; base += PD * step) {
#pragma unroll
    for (int p = 0; p < PD; ++p) {
      const int kc = base + p * step;
      if (kc < kc1) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < MR; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j) acc[i][j] = mfma4(a[p][i][s], b[p][j][s], acc[i][j]);
        const int kn = kc + PD * step;
        if (kn < kc1) {
#pragma unroll
          for (int i = 0; i < MR; ++i) a[p][i] = A.frag(ar[i], kn, q);
#pragma unroll
          for (int j = 0; j < NR; ++j) b[p][j] = B.frag(br[j], kn, q);
        }
      }
    }
  }
}

template <int MR, int NR>
DEV void acc_zero(f4 (&acc)[MR][NR]) {
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f4zero();
}

// Chunks of a K range are dealt round-robin to the 4 waves of a workgroup
// ("wave split-K"); a segment starting at global chunk g0 gives wave w the
// chunks kc with (g0 + kc) % 4 == w.
DEV int first_chunk(int w, int g0) { return ((w - g0) % 4 + 4) % 4; }

// Sum the 4 waves' partial MR x NR tiles in LDS.  After the call, `tile`
// (TM x (TN+4) floats, TM = 16*MR, TN = 16*NR) holds the reduced tile.
// `lds` must hold 4 * TM * (TN+4) floats.
template <int MR, int NR>
DEV void reduce_waves_to_lds(const f4 (&acc)[MR][NR], float* lds, int wave, int lane) {
  constexpr int TM = 16 * MR, TN = 16 * NR, LD = TN + 4;
  const int r = lane & 15, q = lane >> 4;
  float* mine = lds + wave * TM * LD;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) mine[(16 * i + 4 * q + g) * LD + 16 * j + r] = acc[i][j][g];
  __syncthreads();
  for (int e = threadIdx.x; e < TM * TN; e += blockDim.x) {
    const int row = e / TN, col = e % TN;
    const int o = row * LD + col;
    lds[o] = lds[o] + lds[TM * LD + o] + lds[2 * TM * LD + o] + lds[3 * TM * LD + o];
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Philox-4x32-10 (Salmon et al. 2011), counter = (offset lo, offset hi, 0, 0),
// key = seed.  One call -> 4 uniform 32-bit words.
// ---------------------------------------------------------------------------
DEV void philox4x32(uint64_t seed, uint64_t ctr, uint32_t (&out)[4]) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
// uniform in (0, 1]
DEV float u01(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }
// standard normal for element index i of stream (seed, offset): Box-Muller
DEV float philox_normal(uint64_t seed, uint64_t idx) {
  uint32_t o[4];
  philox4x32(seed, idx, o);
  const float u1 = u01(o[0]), u2 = u01(o[1]);
  return sqrtf(-2.0f * __logf(u1)) * __cosf(6.2831853071795864f * u2);
}
// Gumbel(0,1) = -log(E), E ~ Exp(1) = -log(U)
DEV float philox_gumbel(uint64_t seed, uint64_t idx) {
  uint32_t o[4];
  philox4x32(seed, idx, o);
  const float u = u01(o[0]);
  const float e = -__logf(u);
  return -__logf(fmaxf(e, 1e-30f));
}

// Buffer resource over [p, p + bytes): loads beyond it return 0.
// The descriptor must live in SGPRs: its inputs are wave-uniform, but when
// divergence analysis cannot prove it the compiler wraps every load in a
// readfirstlane "waterfall" loop -- so make the uniformity explicit.
DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)n, 0x00020000);
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
inline int rup16(int x) { return (x + 15) & ~15; }

// true in every thread of the last workgroup to call it.  The hand-over is
// write-through (MI355X_MICROARCH.md visibility table, R1): every partial the
// last workgroup reads was stored by st_agent (sc1) and drained by its wave
// (vmcnt(0)) before the barrier and the relaxed ticket add, and is read back
// with ld_agent (sc1) -- no L2 write-back / invalidate (__threadfence: ~3.5
// us per call, twice on the last workgroup's path)
DEV bool last_workgroup(unsigned* ticket, int* flag_sh) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = n == gridDim.x - 1;
    if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_sh = last;
  }
  __syncthreads();
  return *flag_sh != 0;
}
template <class T>
DEV T ld_agent(const T* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class T>
DEV void st_agent(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

}  // namespace abcd

namespace abcd {
// ---------------------------------------------------------------------------
// "row-block" step GEMM: a workgroup owns 64 rows x NR*16 columns; each of its
// 4 waves owns 16 rows over the FULL K (no wave split-K, so no LDS reduce and
// the epilogue runs from the accumulator registers).  The B slice (NR*16 rows
// of a weight matrix x K) is staged ONCE per workgroup into LDS in
// fragment-major order -- [subtile j][chunk kc][lane] float4 -- so every B
// fragment read is one conflict-free ds_read_b128 of 64 consecutive 16-B
// slots; A rows stream from L2/HBM through a PD-deep register ring.
// Two accumulator sets alternate by chunk parity so single-subtile tiles
// still have two independent MFMA chains (16x16x4 f32: 32-cycle issue,
// 40-cycle dependent latency).
// ---------------------------------------------------------------------------

// Fill LDS with the B rows rowfn(j, r) (subtile j < nsub, r < 16), chunks
// [0, nch), source element (row, k) at W[row*ldw + k].  Global reads are
// row-contiguous float4s (coalesced); LDS writes land in fragment order.
template <class RowFn>
DEV void stage_rows(f4* dst, const float* W, long ldw, int nsub, int nch, RowFn rowfn) {
  // UNR loads in flight per thread before any LDS write: one memory round
  // trip per UNR*256 float4s instead of one per 256 (the fill is latency-bound)
  constexpr int UNR = 16;
  const int total = nsub * 16 * nch * 4;  // float4s
  for (int base = 0; base < total; base += UNR * 256) {
    f4 v[UNR];
    int dsti[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int e = base + u * 256 + threadIdx.x;
      dsti[u] = -1;
      if (e < total) {
        const int q = e & 3;
        const int kc = (e >> 2) % nch;
        const int rowi = (e >> 2) / nch;  // 0 .. nsub*16-1
        const int j = rowi >> 4, r = rowi & 15;
        v[u] = *reinterpret_cast<const f4*>(W + (long)rowfn(j, r) * ldw + kc * 16 + 4 * q);
        dsti[u] = (j * nch + kc) * 64 + q * 16 + r;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (dsti[u] >= 0) dst[dsti[u]] = v[u];
  }
}
// rows brow(j) + 0..15
template <class RowFn>
DEV void stage_b_frag(f4* dst, const float* W, long ldw, int nsub, int nch, RowFn brow) {
  stage_rows(dst, W, ldw, nsub, nch, [&](int j, int r) { return brow(j) + r; });
}

// acc[p][j] += A(row, k) * B_j(k) over chunks [0, nch) of one segment.
// Bl: the segment's fragment-major LDS image ([j][kc][lane]).  The ring of PD
// A chunks is refilled unconditionally (the loop is branch-free, so the
// compiler waits with `s_waitcnt vmcnt(PD-1)` for the oldest chunk instead of
// draining every load).  TAIL = false requires nch % PD == 0; TAIL = true
// guards the MFMAs of a final partial block (uniform branches, which cost a
// full drain there), so A must be readable up to chunk roundup(nch, PD)
// (BufKC: range-checked).
// `pre` (optional) runs between the A ring's first loads and the first
// MFMA: work whose memory operations must not delay those loads (its stores
// are issued after them, so the ring's vmcnt waits do not cover them).
struct NoPre {
  DEV void operator()() const {}
};
template <int NR, int PD, bool TAIL = false, class OA, class Pre = NoPre>
DEV void wave_mma_lds(f4 (&acc)[2][NR], const OA& A, int arow, const f4* Bl, int nch, int lane, int q,
                      Pre pre = Pre()) {
  f4 a[PD], b[NR];
#pragma unroll
  for (int p = 0; p < PD; ++p) a[p] = A.frag(arow, p, q);
#pragma unroll
  for (int j = 0; j < NR; ++j) b[j] = Bl[j * nch * 64 + lane];
  if constexpr (!std::is_same_v<Pre, NoPre>) {
    __builtin_amdgcn_sched_barrier(0);
    pre();
    __builtin_amdgcn_sched_barrier(0);
  }
  // one chunk: LDS reads of the NEXT chunk's B fragments are issued before
  // this chunk's MFMAs (their latency hides behind them); the A slot is
  // refilled PD chunks ahead when `refill`
  auto chunk = [&](int kc, int p, bool refill) {
    const int kn = kc + 1 < nch ? kc + 1 : kc;
    f4 bn[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) bn[j] = Bl[(j * nch + kn) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[p & 1][j] = mfma4(a[p][s], b[j][s], acc[p & 1][j]);
    if (refill) a[p] = A.frag(arow, kc + PD, q);
#pragma unroll
    for (int j = 0; j < NR; ++j) b[j] = bn[j];
    // keep each refill right behind its chunk's MFMAs (the scheduler would
    // otherwise sink all refills to the end of the block)
    __builtin_amdgcn_sched_barrier(0);
  };
  int base = 0;
  for (; base + PD < nch; base += PD) {
#pragma unroll
    for (int p = 0; p < PD; ++p) chunk(base + p, p, true);
  }
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (!TAIL || base + p < nch) chunk(base + p, p, false);
}

template <int NR>
DEV void acc2_zero(f4 (&acc)[2][NR]) {
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[p][j] = f4zero();
}
template <int NR>
DEV void acc2_fold(f4 (&acc)[2][NR]) {
#pragma unroll
  for (int j = 0; j < NR; ++j) acc[0][j] += acc[1][j];
}
}  // namespace abcd
