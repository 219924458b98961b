// abcd_x6.h -- fp32 GEMM on the bf16 matrix cores ("split-fp32", bf16x6).
//
// gfx950 runs f32-input MFMA at 1/16 of the bf16 rate (MI355X_MICROARCH.md,
// Matrix cores).  An fp32 value splits EXACTLY into three bf16 pieces
//     x = x0 + x1 + x2,   x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (each residual is exact in fp32; 3 x 8 significand bits cover fp32's 24),
// so a*b = sum_{i,j} a_i b_j.  Keeping the six terms with i + j <= 2 drops
// a1 b2 + a2 b1 + a2 b2, each below 2^-24 |a||b| -- the size of one fp32
// rounding -- and every bf16 x bf16 product is exact in the fp32 accumulator.
// The result is an fp32-accurate GEMM (tests/test_gpu_x6.py bounds it
// against float64 next to the f32-MFMA path) at 6 bf16 MFMAs
// (16x16x32, ~16 cycles each) per 32-deep K slice instead of 8 f32 MFMAs
// (16x16x4, 32 cycles each).
//
// Fragment layout of v_mfma_f32_16x16x32_bf16: lane l supplies A[row l&15]
// [k = 8(l>>4) + 0..7] and B[k = 8(l>>4) + 0..7][col l&15]; the accumulator
// layout equals the f32 16x16x4 one (rows 4(l>>4) + g, column l&15), so
// epilogues are unchanged.
//
// B (weights) is split once and staged in LDS as three planes in fragment
// order: [subtile j][chunk c][plane p][lane] x 16 B (one conflict-free
// ds_read_b128 per plane).  A (the recurrent operand) is read as fp32 (two
// float4 per lane per 32-deep chunk) and split in registers.
#pragma once
#include "abcd_common.h"

namespace abcd {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

DEV f4 mfma_bf(const bf8& a, const bf8& b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

DEV float bf_to_f(__bf16 h) { return (float)h; }

// 8 fp32 -> three bf16x8 pieces (hi, mid, lo), exact decomposition.  Pairs
// go through v_cvt_pk_bf16_f32; a bf16 pair widens back to two floats with
// a shift and a mask.
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
DEV uint32_t cvt_pk(float a, float b) {
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf2));
}
DEV float lo_f(uint32_t u) { return __builtin_bit_cast(float, u << 16); }
DEV float hi_f(uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); }
DEV void split8(const f4& x0, const f4& x1, bf8& h, bf8& m, bf8& l) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  u4 H, M, L;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = e < 2 ? x0[2 * e] : x1[2 * e - 4];
    const float b = e < 2 ? x0[2 * e + 1] : x1[2 * e - 3];
    const uint32_t hp = cvt_pk(a, b);
    const float ra = a - lo_f(hp), rb = b - hi_f(hp);
    const uint32_t mp = cvt_pk(ra, rb);
    const float sa = ra - lo_f(mp), sb = rb - hi_f(mp);
    H[e] = hp;
    M[e] = mp;
    L[e] = cvt_pk(sa, sb);
  }
  h = __builtin_bit_cast(bf8, H);
  m = __builtin_bit_cast(bf8, M);
  l = __builtin_bit_cast(bf8, L);
}

// 16-deep form for a last chunk with at most 16 valid k (the K = 144 input
// projection's fifth chunk): v_mfma_f32_16x16x16_bf16, lane l supplies
// A[row l&15][k = 4(l>>4) + 0..3] and B[k = 4(l>>4) + 0..3][col l&15]
// (same accumulator layout), half the cycles of a zero-padded 32-deep slice
typedef short s4 __attribute__((ext_vector_type(4)));
DEV void split4(const f4& x, s4& h, s4& m, s4& l) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  u2 H, M, L;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    const uint32_t hp = cvt_pk(a, b);
    const float ra = a - lo_f(hp), rb = b - hi_f(hp);
    const uint32_t mp = cvt_pk(ra, rb);
    H[e] = hp;
    M[e] = mp;
    L[e] = cvt_pk(ra - lo_f(mp), rb - hi_f(mp));
  }
  h = __builtin_bit_cast(s4, H);
  m = __builtin_bit_cast(s4, M);
  l = __builtin_bit_cast(s4, L);
}
DEV f4 mfma_bf16k(const s4& a, const s4& b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }
DEV f4 mma_x6_16(f4 acc, const s4& a0, const s4& a1, const s4& a2, const s4& b0, const s4& b1, const s4& b2) {
  acc = mfma_bf16k(a2, b0, acc);
  acc = mfma_bf16k(a1, b1, acc);
  acc = mfma_bf16k(a0, b2, acc);
  acc = mfma_bf16k(a1, b0, acc);
  acc = mfma_bf16k(a0, b1, acc);
  acc = mfma_bf16k(a0, b0, acc);
  return acc;
}
// the low 8 bytes of an LDS slot as a bf16x4 fragment
DEV s4 lo_s4(const f4& v) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(s4, f2v{v[0], v[1]});
}

// acc += a * b over one 32-deep slice, six-term split product
DEV f4 mma_x6(f4 acc, const bf8& a0, const bf8& a1, const bf8& a2, const bf8& b0, const bf8& b1, const bf8& b2) {
  acc = mfma_bf(a2, b0, acc);
  acc = mfma_bf(a1, b1, acc);
  acc = mfma_bf(a0, b2, acc);
  acc = mfma_bf(a1, b0, acc);
  acc = mfma_bf(a0, b1, acc);
  acc = mfma_bf(a0, b0, acc);
  return acc;
}

// Stage rows rowfn(j, r) (subtile j < nsub, r < 16) of an fp32 matrix W
// (element (row, k) at W[row*ldw + k], k < kvalid; zero beyond) as the x6
// image: chunks [c0, c0 + nseg) of an image with nch 32-deep chunks per
// subtile.  Each thread converts 8 consecutive k of one row.
template <class RowFn>
DEV void stage_x6(f4* dst, const float* W, long ldw, int kvalid, int nsub, int nseg, int c0, int nch, RowFn rowfn) {
  constexpr int UNR = 8;
  const int total = nsub * 16 * nseg * 4;  // (row, chunk, q) units of 8 floats
  for (int base = 0; base < total; base += UNR * 256) {
    f4 v0[UNR], v1[UNR];
    int dsti[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int e = base + u * 256 + threadIdx.x;
      dsti[u] = -1;
      v0[u] = v1[u] = f4zero();
      if (e < total) {
        const int q = e & 3;
        const int c = (e >> 2) % nseg;
        const int rowi = (e >> 2) / nseg;
        const int j = rowi >> 4, r = rowi & 15;
        const int k = c * 32 + 8 * q;
        const int wr = rowfn(j, r);  // < 0: a zero row
        const float* src = W + (long)(wr < 0 ? 0 : wr) * ldw + k;
        if (wr < 0) {
        } else if (k + 4 <= kvalid) v0[u] = *reinterpret_cast<const f4*>(src);
        else
          for (int s = 0; s < 4; ++s) v0[u][s] = k + s < kvalid ? src[s] : 0.f;
        if (wr < 0) {
        } else if (k + 8 <= kvalid) v1[u] = *reinterpret_cast<const f4*>(src + 4);
        else
          for (int s = 0; s < 4; ++s) v1[u][s] = k + 4 + s < kvalid ? src[4 + s] : 0.f;
        dsti[u] = ((j * nch + c0 + c) * 3) * 64 + q * 16 + r;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (dsti[u] >= 0) {
        bf8 h, m, l;
        split8(v0[u], v1[u], h, m, l);
        dst[dsti[u]] = __builtin_bit_cast(f4, h);
        dst[dsti[u] + 64] = __builtin_bit_cast(f4, m);
        dst[dsti[u] + 128] = __builtin_bit_cast(f4, l);
      }
  }
}

// acc[j] += A(row, k) * B_j(k) over NCH 32-deep chunks (compile time: the
// whole loop unrolls, so the ring slots are fixed registers -- a runtime
// trip count made the compiler rotate the ring with moves that waited for
// every load).  A supplies frag8(row, c, q, lo, hi) (k = 32c + 8q + 0..7 as
// two float4).  PD chunks of raw fp32 stay in flight; each is split in
// registers during the previous chunk's 6 x NR MFMAs (the persistent kernels
// use PD = 4: same-box A/B at c2 against PD = 8, enc_fwd 1.35 -> 1.23 ms,
// dec_fwd 2.51 -> 2.36 ms, dec_bwd 4.22 -> 4.17 ms; PD = 2 no better).
// wave_mma_x6p: one image segment per output tile, chunk c of tile j at
// Bp[j] + c * 3 * 64 (tiles from different LDS images sharing one A operand);
// wave_mma_x6 (below): the chunk-major image Bl with `nch` chunks per subtile
// (nch >= NCH; a segment of a wider image starts at Bl + c0 * 3 * 64).
// NR >= 4 (the encoder forward's four gate tiles): software-pipelined by one
// chunk (round 6) -- chunk c + 1's split (~36 dependent VALU) and its
// B-fragment LDS reads are interleaved with chunk c's 6 NR MFMAs instead of
// sitting between two MFMA runs, where the matrix pipe idled ~150 cycles per
// chunk (enc_fwd: 8 x 150 of its ~3070 MFMA cycles per step).  Same products
// in the same order: bit-identical results.
template <int NR, int NCH, int PD, class OA>
DEV void wave_mma_x6p_pipe(f4 (&acc)[NR], const OA& A, int arow, const f4* const (&Bp)[NR], int lane, int q,
                           int rot) {
  constexpr int P = PD < NCH ? PD : NCH;
  auto cc = [&](int c) { const int x = c + rot; return x >= NCH ? x - NCH : x; };
  f4 ra[P], rb[P];
#pragma unroll
  for (int p = 0; p < P; ++p) A.frag8(arow, cc(p), q, ra[p], rb[p]);
  f4 bw[NR][3];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) bw[j][pl] = Bp[j][(cc(0) * 3 + pl) * 64 + lane];
  __builtin_amdgcn_sched_barrier(0);
  bf8 a0, a1, a2;
  split8(ra[0], rb[0], a0, a1, a2);
  if (P < NCH) A.frag8(arow, cc(P), q, ra[0], rb[0]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    f4 bn[NR][3];
    bf8 n0, n1, n2;
    if (c + 1 < NCH) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) bn[j][pl] = Bp[j][(cc(c + 1) * 3 + pl) * 64 + lane];
      const int p1 = (c + 1) % P;
      split8(ra[p1], rb[p1], n0, n1, n2);
      if (c + 1 + P < NCH) A.frag8(arow, cc(c + 1 + P), q, ra[p1], rb[p1]);
    }
#pragma unroll
    for (int j = 0; j < NR; ++j)
      acc[j] = mma_x6(acc[j], a0, a1, a2, __builtin_bit_cast(bf8, bw[j][0]), __builtin_bit_cast(bf8, bw[j][1]),
                      __builtin_bit_cast(bf8, bw[j][2]));
    if (c + 1 < NCH) {
      // the next chunk's B reads first, then MFMAs with the split's VALU between them
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * NR, 0);
#pragma unroll
      for (int k = 0; k < 6 * NR; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, (40 + 6 * NR - 1) / (6 * NR), 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NCH) {
      a0 = n0, a1 = n1, a2 = n2;
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) bw[j][pl] = bn[j][pl];
    }
  }
}

// the same with each chunk split right before its own MFMAs (NR < 4: with
// 6 or 12 MFMAs per chunk the split's dependent VALU chain outlasts them, and
// the interleaved form measured no faster in the decoder kernels)
template <int NR, int NCH, int PD, class OA>
DEV void wave_mma_x6p_serial(f4 (&acc)[NR], const OA& A, int arow, const f4* const (&Bp)[NR], int lane, int q,
                             int rot) {
  constexpr int P = PD < NCH ? PD : NCH;
  auto cc = [&](int c) { const int x = c + rot; return x >= NCH ? x - NCH : x; };
  f4 ra[P], rb[P];
#pragma unroll
  for (int p = 0; p < P; ++p) A.frag8(arow, cc(p), q, ra[p], rb[p]);
  // B fragments double-buffered: chunk c + 1's LDS reads are issued before
  // chunk c's MFMAs so their latency hides behind them
  f4 bw[NR][3];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) bw[j][pl] = Bp[j][(cc(0) * 3 + pl) * 64 + lane];
  // pin the whole ring's loads here (the scheduler would sink each next to
  // its use) and keep each chunk's split + refill ahead of its MFMAs
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int p = c % P;
    f4 bn[NR][3];
    if (c + 1 < NCH) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) bn[j][pl] = Bp[j][(cc(c + 1) * 3 + pl) * 64 + lane];
    }
    bf8 a0, a1, a2;
    split8(ra[p], rb[p], a0, a1, a2);
    if (c + P < NCH) A.frag8(arow, cc(c + P), q, ra[p], rb[p]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NR; ++j)
      acc[j] = mma_x6(acc[j], a0, a1, a2, __builtin_bit_cast(bf8, bw[j][0]), __builtin_bit_cast(bf8, bw[j][1]),
                      __builtin_bit_cast(bf8, bw[j][2]));
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NCH) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) bw[j][pl] = bn[j][pl];
    }
  }
}

template <int NR, int NCH, int PD, class OA>
DEV void wave_mma_x6p(f4 (&acc)[NR], const OA& A, int arow, const f4* const (&Bp)[NR], int lane, int q,
                      int rot = 0) {
  if constexpr (NR >= 4) wave_mma_x6p_pipe<NR, NCH, PD>(acc, A, arow, Bp, lane, q, rot);
  else wave_mma_x6p_serial<NR, NCH, PD>(acc, A, arow, Bp, lane, q, rot);
}

template <int NR, int NCH, int PD, class OA>
DEV void wave_mma_x6(f4 (&acc)[NR], const OA& A, int arow, const f4* Bl, int nch, int lane, int q, int rot = 0) {
  const f4* Bp[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) Bp[j] = Bl + (size_t)j * nch * 3 * 64;
  wave_mma_x6p<NR, NCH, PD>(acc, A, arow, Bp, lane, q, rot);
}

}  // namespace abcd
