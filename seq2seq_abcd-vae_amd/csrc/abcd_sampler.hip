// abcd_sampler.hip -- attention-based categorical sampler (ABCDSampler,
// ABCD-VAE/modules/model.py:538-639), its Dirichlet-categorical KL, and the
// plain Gaussian feature sampler (plain/modules/model.py:538-567).
//
// Everything here is B x {E, Hm, D, K}: the MLP and the two codebook products
// run through the MFMA GEMM (abcd_gemm.hip); the row-wise Gumbel-softmax /
// softmax, the KL terms (device digamma / trigamma / lgamma in fp64) and the
// softmax / KL backward are one-wave-per-row kernels.
#include "abcd_common.h"
#include "abcd_internal.h"

#include <mutex>
#include <vector>

namespace abcd {

// learning.py:171-178 perplexities of rows of `ld` floats (first K = categories)
int perplexities_ld(const float* logits, int B, int ld, int K, const float* psl, float* out, void* stream);

// ---- special functions (fp64, x > 0) --------------------------------------
DEV double digamma_d(double x) {
  double r = 0.0;
  while (x < 6.0) { r -= 1.0 / x; x += 1.0; }
  const double f = 1.0 / (x * x);
  return r + log(x) - 0.5 / x -
         f * (1.0 / 12 - f * (1.0 / 120 - f * (1.0 / 252 - f * (1.0 / 240 - f * (1.0 / 132)))));
}
DEV double trigamma_d(double x) {
  double r = 0.0;
  while (x < 6.0) { r += 1.0 / (x * x); x += 1.0; }
  const double f = 1.0 / (x * x);
  return r + 1.0 / x + 0.5 * f +
         (1.0 / x) * f * (1.0 / 6 - f * (1.0 / 30 - f * (1.0 / 42 - f * (1.0 / 30 - f * (5.0 / 66)))));
}

DEV float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
DEV double wave_sum_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// y = softmax((logits + g) / tau) per row (g = 0 for the plain softmax).
// Rows have K columns of which the first Kv are categories; the padding
// columns (a zero-padded model, modules/padding.py) get y = 0.
__global__ void sample_softmax_rows(const float* logits, int B, int K, int Kv, int gumbel, float tau,
                                    const float* noise, uint64_t seed, uint64_t offset, float* Y) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* l = logits + (long)b * K;
  float* y = Y + (long)b * K;
  const float it = 1.f / tau;
  for (int k = Kv + lane; k < K; k += 64) y[k] = 0.f;
  float m = -INFINITY;
  for (int k = lane; k < Kv; k += 64) {
    float v = l[k];
    if (gumbel) v = (v + (noise ? noise[(long)b * K + k] : philox_gumbel(seed, offset + (uint64_t)b * K + k))) * it;
    y[k] = v;
    m = fmaxf(m, v);
  }
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < Kv; k += 64) {
    const float e = __expf(y[k] - m);
    y[k] = e;
    s += e;
  }
  s = wave_sum(s);
  const float is = 1.f / s;
  for (int k = lane; k < Kv; k += 64) y[k] *= is;
}

// Block reductions (blockDim = 64 x nw, nw <= 16); `sh` holds 16 doubles.
// Every thread returns the block-wide value.
DEV double block_sum_dd(double v, double* sh) {
  const int nw = blockDim.x >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}
DEV double block_max_dd(double v, double* sh) {
  const int nw = blockDim.x >> 6;
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = sh[0];
  for (int i = 1; i < nw; ++i) t = fmax(t, sh[i]);
  return t;
}

// KL prior part (model.py:620-633), one block: p = softmax(psl),
// alpha = p N + a0, elog = psi(alpha) - psi(S).  alphaL / elogL: K floats of
// block-shared scratch receiving alpha and elog (as fp32, the values the row
// terms use).  stash: also p / alpha / elog / tri to global and
// kl_small = [Eq log q(pi) - Eq log p(pi), psi'(S), S].  Only the first Kv of
// the K entries are categories; the padding entries are written as 0 (so the
// row terms that read them multiply a zero probability by a finite value).
DEV void prior_block(const float* psl, int K, int Kv, double N, float a0, float* alphaL, float* elogL, double* sh,
                     bool stash, float* p_out, float* alpha_out, float* elog_out, float* tri_out,
                     double* kl_small) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int k = Kv + tid; k < K; k += nt) {
    alphaL[k] = 0.f;
    elogL[k] = 0.f;
    if (stash) { p_out[k] = 0.f; alpha_out[k] = 0.f; elog_out[k] = 0.f; tri_out[k] = 0.f; }
  }
  K = Kv;
  double m = -1e300;
  for (int k = tid; k < K; k += nt) m = fmax(m, (double)psl[k]);
  m = block_max_dd(m, sh);
  double se = 0.0;
  for (int k = tid; k < K; k += nt) se += exp((double)psl[k] - m);
  se = block_sum_dd(se, sh);
  double sa = 0.0;
  for (int k = tid; k < K; k += nt) {
    const double p = exp((double)psl[k] - m) / se;
    const double al = (double)(float)((float)p * (float)N) + (double)a0;  // the product in fp32 like the reference
    alphaL[k] = (float)al;
    if (stash) { p_out[k] = (float)p; alpha_out[k] = (float)al; }
    sa += al;
  }
  sa = block_sum_dd(sa, sh);
  const double S = sa, psiS = digamma_d(S);
  double acc = 0.0;  // -sum lgamma(alpha) + sum (alpha-1) elog - (a0-1) sum elog
  for (int k = tid; k < K; k += nt) {
    const double al = alphaL[k];
    const double el = digamma_d(al) - psiS;
    elogL[k] = (float)el;
    if (stash) {
      elog_out[k] = (float)el;
      tri_out[k] = (float)trigamma_d(al);
      acc += -lgamma(al) + (al - 1.0) * el - ((double)a0 - 1.0) * el;
    }
  }
  if (stash) {
    acc = block_sum_dd(acc, sh);
    if (tid == 0) {
      const double a0d = a0;
      // write-through: the forward head's last workgroup reads [0] in this launch
      __hip_atomic_store(kl_small, lgamma(S) + acc - (lgamma(a0d * K) - K * lgamma(a0d)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(kl_small + 1, trigamma_d(S), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(kl_small + 2, S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
}

// standalone form (abcd_sampler_kl, abcd_sampler_prior): alpha / elog land in
// the global stash
__global__ void kl_prior(const float* psl, int K, int Kv, double N, float a0, float* p_out, float* alpha_out,
                         float* elog_out, float* tri_out, double* kl_small) {
  __shared__ double sh[16];
  prior_block(psl, K, Kv, N, a0, alpha_out, elog_out, sh, true, p_out, alpha_out, elog_out, tri_out, kl_small);
}

// per row: Q = softmax(l); v_b = sum_k Q (log Q - elog)  (padding columns: Q = 0)
__global__ void kl_rows(const float* logits, int B, int K, int Kv, const float* elog, float* Q, float* v) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* l = logits + (long)b * K;
  for (int k = Kv + lane; k < K; k += 64) Q[(long)b * K + k] = 0.f;
  float m = -INFINITY;
  for (int k = lane; k < Kv; k += 64) m = fmaxf(m, l[k]);
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < Kv; k += 64) s += __expf(l[k] - m);
  s = wave_sum(s);
  const float ls = __logf(s);
  float acc = 0.f;
  for (int k = lane; k < Kv; k += 64) {
    const float lq = l[k] - m - ls;
    const float q = __expf(lq);
    Q[(long)b * K + k] = q;
    acc += q * (lq - elog[k]);
  }
  acc = wave_sum(acc);
  if (lane == 0) v[b] = acc;
}

__global__ void kl_final(const double* kl_small, const float* v, int B, double N, float* out) {
  __shared__ double sh[16];
  double acc = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) acc += v[b];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    *out = (float)(kl_small[0] * ((double)B / N) + t);
  }
}

// sample backward: dL = y (dY - sum y dY) / tau          (accumulate: dL +=)
__global__ void sample_softmax_bwd(const float* Y, const float* dY, int B, int K, float tau, int accumulate,
                                   float* dL) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const long o = (long)b * K;
  float sdy = 0.f;
  for (int k = lane; k < K; k += 64) sdy += Y[o + k] * dY[o + k];
  sdy = wave_sum(sdy);
  const float it = 1.f / tau;
  for (int k = lane; k < K; k += 64) {
    const float g = Y[o + k] * (dY[o + k] - sdy) * it;
    dL[o + k] = accumulate ? dL[o + k] + g : g;
  }
}
// KL row backward: dL (+)= s q ((log q - elog) - v_b)
__global__ void kl_rows_bwd(const float* Q, const float* elog, const float* v, int B, int K, const float* dkl,
                            int accumulate, float* dL) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const long o = (long)b * K;
  const float s = *dkl, vb = v[b];
  for (int k = lane; k < K; k += 64) {
    const float q = Q[o + k];
    const float g = s * q * ((__logf(fmaxf(q, 1e-38f)) - elog[k]) - vb);
    dL[o + k] = accumulate ? dL[o + k] + g : g;
  }
}

// d posterior_shape_logits (model.py:620-633 backward), one block; Qsum[k] =
// sum_b Q(b, k) (global or block-shared)
DEV void prior_bwd_block(const float* p, const float* alpha, const float* tri, const double* kl_small,
                         const float* Qsum, int K, int B, double N, float a0, float dkl, float* dpsl, double* sh) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const double s = dkl;
  const double r = (double)B / N;
  double sde = 0.0;
  for (int k = tid; k < K; k += nt) sde += r * ((double)alpha[k] - a0) - Qsum[k];
  sde = block_sum_dd(sde, sh);
  const double triS = kl_small[1];
  double spd = 0.0;
  for (int k = tid; k < K; k += nt) {
    const double de = r * ((double)alpha[k] - a0) - Qsum[k];
    const double da = s * (de * tri[k] - triS * sde);
    spd += (double)p[k] * da * N;
  }
  spd = block_sum_dd(spd, sh);
  for (int k = tid; k < K; k += nt) {
    const double de = r * ((double)alpha[k] - a0) - Qsum[k];
    const double da = s * (de * tri[k] - triS * sde);
    dpsl[k] = (float)((double)p[k] * (da * N - spd));
  }
}
__global__ void kl_prior_bwd(const float* p, const float* alpha, const float* tri, const double* kl_small,
                             const float* Qsum, int K, int B, double N, float a0, const float* dkl, float* dpsl) {
  __shared__ double sh[16];
  prior_bwd_block(p, alpha, tri, kl_small, Qsum, K, B, N, a0, *dkl, dpsl, sh);
}

__global__ void tanh_bwd_inplace(float* dz, const float* z, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dz[i] *= 1.f - z[i] * z[i];
}

// ---- plain Gaussian sampler helpers ----------------------------------------
// fv: the model's feature dim (a zero-padded twin's real f): columns j >= fv
// are padding, their noise is 0 and their sample mu + 0 = 0 (padding mu = 0)
__global__ void plain_sample(const float* MV, int B, int f, int fv, const float* noise, uint64_t seed,
                             uint64_t offset, float* feats, float* EPS) {
  const int n = B * f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / f, j = i % f;
    const float mu = MV[(long)b * 2 * f + j], lv = MV[(long)b * 2 * f + f + j];
    const float e = j >= fv ? 0.f : noise ? noise[i] : philox_normal(seed, offset + (uint64_t)i);
    EPS[i] = e;
    feats[i] = mu + __expf(0.5f * lv) * e;
  }
}
__global__ void plain_kl(const float* MV, int B, int f, float* out) {
  __shared__ double sh[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < B * f; i += blockDim.x) {
    const int b = i / f, j = i % f;
    const float mu = MV[(long)b * 2 * f + j], lv = MV[(long)b * 2 * f + f + j];
    acc += 1.0 + lv - (double)mu * mu - exp((double)lv);
  }
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    *out = (float)(-0.5 * t);
  }
}
// dMV = [dmu | dlv]
__global__ void plain_dparams(const float* MV, const float* EPS, int B, int f, const float* dfeat, const float* dkl,
                              float* dMV) {
  const int n = B * f;
  const float s = dkl ? *dkl : 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / f, j = i % f;
    const float mu = MV[(long)b * 2 * f + j], lv = MV[(long)b * 2 * f + f + j];
    const float df = dfeat ? dfeat[i] : 0.f;
    const float sd = __expf(0.5f * lv);
    dMV[(long)b * 2 * f + j] = df + s * mu;
    dMV[(long)b * 2 * f + f + j] = df * 0.5f * sd * EPS[i] + s * 0.5f * (__expf(lv) - 1.f);
  }
}

// ---------------------------------------------------------------------------
// Sampler head: the ABCD sampler's forward (model.py:581-606 + the KL row
// terms of 608-639) and its backward as ONE row-tiled kernel each.  A
// workgroup owns 16 rows of the batch; every intermediate of those rows
// (Z1 -> U -> logits -> Q, Y -> feats) stays in LDS between the four
// products, which run on the exact-fp32 16x16x4 MFMA with the weights /
// codebook streamed from L2 as B operands (4 waves split the output columns,
// a 4-chunk register ring per wave).  The only grid-wide results -- the KL
// scalar and (backward) the bias / Qsum column sums feeding the Dirichlet
// prior gradient -- are reduced by the last workgroup to finish, over the
// per-tile partials in tile order (deterministic, no float atomics).
// Forward = the split-K h W1^T GEMM (raw slabs) + samp_head_fwd; backward =
// samp_head_bwd + the d_h GEMM, with the parameter-gradient GEMMs on the
// side stream.
// ---------------------------------------------------------------------------
constexpr int HEAD_ROWS = 16;
// diagnostics: thread 0 of each tile stamps s_memrealtime (100 MHz, device-wide) at phase k
#define HSTAMP(k)                                                                              \
  do {                                                                                         \
    if (a.prof && threadIdx.x == 0) a.prof[(size_t)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// "last workgroup" tickets (self-resetting): [0] forward KL, [1] backward
// column sums.  Launches on one device are serialised on the engine's stream.
__device__ unsigned g_head_ticket[2];

struct LdsRows {  // A operand: 16 rows resident in LDS, row pitch ld floats
  const float* p; int ld;
  DEV f4 frag(int row, int kc, int q) const { return *reinterpret_cast<const f4*>(p + row * ld + kc * 16 + 4 * q); }
};

// B operands of the tile products, read through buffer resources so every
// load is unconditional (out-of-range lanes / chunks read 0): a load under a
// divergent or conditional branch leaves the wait-count pass unsure of the
// in-order count and it falls back to vmcnt(0) before every chunk, which
// serialises the register ring behind one memory round trip per chunk.
struct BKC {  // B(n, k) at p[n * ld + k] (16-B loads along k); rsrc covers ncols rows
  __amdgpu_buffer_rsrc_t rs; uint32_t ld4;
  DEV f4 frag(int n, int kc, int q, bool ok) const {
    const uint32_t o = ok ? (uint32_t)n * ld4 + (uint32_t)(kc * 16 + 4 * q) * 4u : 0x80000000u;
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
  }
};
struct BKM {  // B(n, k) at p[k * ld + n] (4-B loads, 16 lanes over 16 consecutive n)
  __amdgpu_buffer_rsrc_t rs; uint32_t ld4;
  DEV f4 frag(int n, int kc, int q, bool ok) const {
    f4 v;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t o = ok ? (uint32_t)(kc * 16 + 4 * q + t) * ld4 + (uint32_t)n * 4u : 0x80000000u;
      v[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
    }
    return v;
  }
};
DEV BKC bkc(const float* p, int ld, int nrows) { return BKC{make_rsrc(p, (uint32_t)nrows * ld * 4u), (uint32_t)ld * 4u}; }
DEV BKM bkm(const float* p, int ld, int nk) { return BKM{make_rsrc(p, (uint32_t)nk * ld * 4u), (uint32_t)ld * 4u}; }

// out(r, n) = sum_k A(r, k) B(n, k) for the tile's 16 rows, n < ncols
// (multiple of 16), k < nk (multiple of 16); A: the 16 rows in LDS (pitch
// lda floats).  Wave w takes the 16-column subtiles w*NR.., (w+4)*NR..;
// epi(c0, acc): lane (r, q) holds rows 4q+g of column c0 + r.  PD chunks of
// A and B fragments in flight per wave, branch-free.
template <int NR, int PD, int NW, class OB, class Epi>
DEV void tile_mma(const float* Al, int lda, int nk, const OB& B, int ncols, int w, int lane, Epi&& epi) {
  const int r = lane & 15, q = lane >> 4;
  const int nsub = ncols >> 4, nch = nk >> 4;
  for (int j0 = w * NR; j0 < nsub; j0 += NW * NR) {
    f4 acc[NR];
    int bn[NR];
    bool bok[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      acc[j] = f4zero();
      bn[j] = (j0 + j) * 16 + r;
      bok[j] = bn[j] < ncols;
    }
    f4 a[PD], b[PD][NR];
    auto fetch = [&](int p, int kc) {
      const bool ok = kc < nch;
      const f4 av = *reinterpret_cast<const f4*>(Al + r * lda + (ok ? kc : 0) * 16 + 4 * q);
      a[p] = ok ? av : f4zero();
#pragma unroll
      for (int j = 0; j < NR; ++j) b[p][j] = B.frag(bn[j], kc, q, ok && bok[j]);
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) fetch(p, p);
    for (int base = 0; base < nch; base += PD) {
#pragma unroll
      for (int p = 0; p < PD; ++p) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < NR; ++j) acc[j] = mfma4(a[p][t], b[p][j][t], acc[j]);
        fetch(p, base + p + PD);
      }
    }
#pragma unroll
    for (int j = 0; j < NR; ++j)
      if (j0 + j < nsub) epi((j0 + j) * 16, acc[j]);
  }
}
template <int NW, class OB, class Epi>
DEV void tile_mma_any(const float* Al, int lda, int nk, const OB& B, int ncols, int w, int lane, Epi&& epi) {
  tile_mma<2, 4, NW>(Al, lda, nk, B, ncols, w, lane, epi);
}
// sum over the 16 rows a lane group holds (rows 4q+g): every lane of the
// column gets the column's tile sum
DEV float tile_colsum(f4 v) {
  float c = (v[0] + v[1]) + (v[2] + v[3]);
  c += __shfl_xor(c, 16, 64);
  c += __shfl_xor(c, 32, 64);
  return c;
}
constexpr int HEAD_MAX_SLABS = 8;  // split-K slabs the forward head sums (gemm_slabs' cap)

struct HeadFwdArgs {
  int B, Hm, D, K, nslab;
  int Kv; float rsD;  // categories (the first Kv of K columns), 1 / sqrt(model feature dim)
  const float *slab, *b1, *W2, *b2, *C, *psl;  // slab: nslab x B x Hm raw partials of h W1^T
  double N; float a0;
  int gumbel; float tau; const float* noise; uint64_t seed, offset;
  int prior_ready;  // the prior stash (p, alpha, elog, tri, kl_small) filled by abcd_sampler_prior
  float *Z1, *U, *logits, *Y, *Q, *v, *feats;
  float *p, *alpha, *elog, *tri; double* kl_small;  // prior stash (written by workgroup 0)
  double* klpart;                                   // per-tile sum_b v_b
  float* kl_out;
  float *CT, *W2T;   // K x D and Hm x D transposed copies for the backward (each tile writes a slice)
  // learning.py:171-178 cluster / batch perplexities of this forward (null: skipped)
  float* ppl;        // [exp(mean row entropy of Q), exp(entropy of the batch-mean Q)]
  double* entpart;   // per-tile sum of row entropies
  float* qcolpart;   // tiles x K column sums of Q
  unsigned long long* prof;  // diagnostics: per-tile phase stamps (tiles x 8), or null
};
inline size_t head_fwd_lds(int Hm, int D, int K) {
  return ((size_t)HEAD_ROWS * (std::max(Hm, K) + 4) + (size_t)HEAD_ROWS * (std::max(D, K) + 4) + 2 * (size_t)K) * 4 +
         16 * sizeof(double) + 16;
}

// KPL: categories per lane, ceil(K / 64) rounded up to a power of two
template <int KPL, int NT>
__global__ __launch_bounds__(NT) void samp_head_fwd(HeadFwdArgs a) {
  constexpr int NW = NT / 64, RPW = HEAD_ROWS / NW;  // waves, softmax rows per wave
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  const int Hm = a.Hm, D = a.D, K = a.K;
  const int ld1 = max(Hm, K) + 4, ld2 = max(D, K) + 4;
  float* R1 = hsm;                   // Z1, then logits
  float* R2 = R1 + HEAD_ROWS * ld1;  // U, then Y
  float* alphaL = R2 + HEAD_ROWS * ld2;
  float* elogL = alphaL + K;
  double* sh = reinterpret_cast<double*>(elogL + K);
  int* flag = reinterpret_cast<int*>(sh + 16);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * HEAD_ROWS, nr = min(HEAD_ROWS, a.B - row0);
  HSTAMP(0);
  // Prologue, one memory round trip per iteration: (a) this tile's slice of
  // the transposed codebook / W2 (the backward's K-contiguous operands):
  // CT[k][d] = C[d][k], W2T[j][d] = W2[d][j]; (b) Z1 = tanh(sum of the
  // split-K slabs + b1) (the slab-reduce epilogue), every slab of two f4
  // columns in flight (slabs >= nslab lie beyond the buffer resource: 0).
  // All loads are unconditional buffer loads (out-of-range offsets read 0).
  {
    const int nC = K * D, nW = Hm * D, nT = nC + nW;
    const int per = (nT + gridDim.x - 1) / gridDim.x, t0 = blockIdx.x * per, t1 = min(nT, t0 + per);
    const __amdgpu_buffer_rsrc_t rC = make_rsrc(a.C, (uint32_t)nC * 4u), rW = make_rsrc(a.W2, (uint32_t)nW * 4u);
    const uint32_t BH4 = (uint32_t)a.B * Hm * 4u;
    const __amdgpu_buffer_rsrc_t rS = make_rsrc(a.slab, (uint32_t)a.nslab * BH4);
    const __amdgpu_buffer_rsrc_t rB = make_rsrc(a.b1, (uint32_t)Hm * 4u);
    const int h4 = Hm >> 2, nZ = HEAD_ROWS * h4;
    constexpr int UT = 8, UZ = 2;
    const int itT = (t1 - t0 + NT * UT - 1) / (NT * UT), itZ = (nZ + NT * UZ - 1) / (NT * UZ);
    for (int it = 0; it < max(itT, itZ); ++it) {
      float tv[UT];
#pragma unroll
      for (int u = 0; u < UT; ++u) {
        const int e = t0 + (it * UT + u) * NT + tid;
        const bool inC = e < nC;
        const int k = e / D, d = e - k * D, f = e - nC, jj = f / D, dd = f - jj * D;
        const uint32_t oc = (e < t1 && inC) ? ((uint32_t)d * K + k) * 4u : 0x80000000u;
        const uint32_t ow = (e < t1 && !inC) ? ((uint32_t)dd * Hm + jj) * 4u : 0x80000000u;
        tv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(inC ? rC : rW, inC ? oc : ow, 0, 0));
      }
      f4 v[UZ][HEAD_MAX_SLABS + 1];  // [.][HEAD_MAX_SLABS]: b1
#pragma unroll
      for (int u = 0; u < UZ; ++u) {
        const int e = (it * UZ + u) * NT + tid, rr = e / h4, c = (e - rr * h4) * 4;
        const bool ok = e < nZ && rr < nr;
        const uint32_t o = ok ? ((uint32_t)(row0 + rr) * Hm + c) * 4u : 0x80000000u;
#pragma unroll
        for (int k = 0; k < HEAD_MAX_SLABS; ++k)
          v[u][k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rS, o + k * BH4, 0, 0));
        v[u][HEAD_MAX_SLABS] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rB, ok ? (uint32_t)c * 4u : 0x80000000u, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < UT; ++u) {
        const int e = t0 + (it * UT + u) * NT + tid;
        if (e < t1) { if (e < nC) a.CT[e] = tv[u]; else a.W2T[e - nC] = tv[u]; }
      }
#pragma unroll
      for (int u = 0; u < UZ; ++u) {
        const int e = (it * UZ + u) * NT + tid, rr = e / h4, c = (e - rr * h4) * 4;
        if (e >= nZ) continue;
        f4 z = f4zero();
        if (rr < nr) {
          f4 sacc = f4zero();
#pragma unroll
          for (int k = 0; k < HEAD_MAX_SLABS; ++k) sacc += v[u][k];
#pragma unroll
          for (int i = 0; i < 4; ++i) z[i] = tanhf(sacc[i] + v[u][HEAD_MAX_SLABS][i]);
          *reinterpret_cast<f4*>(a.Z1 + (long)(row0 + rr) * Hm + c) = z;
        }
        *reinterpret_cast<f4*>(R1 + rr * ld1 + c) = z;
      }
    }
  }
  __syncthreads();
  HSTAMP(1);
  // U = Z1 W2^T + b2
  tile_mma_any<NW>(R1, ld1, Hm, bkc(a.W2, Hm, D), D, w, lane, [&](int c0, f4 acc) {
    const int col = c0 + r;
    const float bb = a.b2[col];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 4 * q + g;
      const float v = acc[g] + bb;
      R2[row * ld2 + col] = v;
      if (row < nr) a.U[(long)(row0 + row) * D + col] = v;
    }
  });
  __syncthreads();
  HSTAMP(2);
  // logits = U C / sqrt(D)   (C: D x K, the K-major operand; D the model's feature dim)
  const float rs = a.rsD;
  const int Kv = a.Kv;
  tile_mma_any<NW>(R2, ld2, D, bkm(a.C, K, D), K, w, lane, [&](int c0, f4 acc) {
    const int col = c0 + r;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 4 * q + g;
      const float v = rs * acc[g];
      R1[row * ld1 + col] = v;
      if (row < nr) a.logits[(long)(row0 + row) * K + col] = v;
    }
  });
  HSTAMP(3);
  // Dirichlet posterior: elog for the row terms (every tile), the stash once
  // -- or, with the stash filled ahead by abcd_sampler_prior, elog read from it
  if (a.prior_ready) {
    for (int k = tid; k < K; k += NT) elogL[k] = a.elog[k];
    __syncthreads();
  } else {
    prior_block(a.psl, K, Kv, a.N, a.a0, alphaL, elogL, sh, blockIdx.x == 0, a.p, a.alpha, a.elog, a.tri,
                a.kl_small);
  }
  HSTAMP(4);
  // rows: KL row term v_b = sum_k Q (log Q - elog) (kl_rows) and the sample
  // Y = softmax((logits + g) / tau) (sample_softmax_rows), one wave per row,
  // the row's KPL logits per lane in registers
  const float it = 1.f / a.tau;
  double klsum = 0.0, entsum = 0.0;
  float qcol[KPL];
#pragma unroll
  for (int u = 0; u < KPL; ++u) qcol[u] = 0.f;
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = w * RPW + rr;
    float* y = R2 + row * ld2;
    if (row >= nr) {
      for (int k = lane; k < K; k += 64) y[k] = 0.f;
      continue;
    }
    const float* l = R1 + row * ld1;
    const long g0 = (long)(row0 + row) * K;
    float lv[KPL], gv[KPL];
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const int k = lane + 64 * u;
      lv[u] = k < Kv ? l[k] : -INFINITY;
      gv[u] = (a.gumbel && a.noise && k < Kv) ? a.noise[g0 + k] : 0.f;
    }
    float m = -INFINITY;
#pragma unroll
    for (int u = 0; u < KPL; ++u) m = fmaxf(m, lv[u]);
    m = wave_max(m);
    float se = 0.f;
#pragma unroll
    for (int u = 0; u < KPL; ++u) se += lane + 64 * u < Kv ? __expf(lv[u] - m) : 0.f;
    se = wave_sum(se);
    const float ls = __logf(se);
    float acc = 0.f, ent = 0.f;
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const int k = lane + 64 * u;
      if (k < Kv) {
        const float lq = lv[u] - m - ls;
        const float qv = __expf(lq);
        a.Q[g0 + k] = qv;
        acc += qv * (lq - elogL[k]);
        ent += -qv * lq;
        qcol[u] += qv;
      } else if (k < K) {
        a.Q[g0 + k] = 0.f;  // padding column of a zero-padded model
      }
    }
    acc = wave_sum(acc);
    ent = wave_sum(ent);
    if (lane == 0) a.v[row0 + row] = acc;
    klsum += acc;
    entsum += ent;
    float m2 = -INFINITY;
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const int k = lane + 64 * u;
      if (k < Kv && a.gumbel) {
        const float g = a.noise ? gv[u] : philox_gumbel(a.seed, a.offset + (uint64_t)g0 + k);
        lv[u] = (lv[u] + g) * it;
      }
      m2 = fmaxf(m2, lv[u]);
    }
    m2 = wave_max(m2);
    float s2 = 0.f;
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      lv[u] = lane + 64 * u < Kv ? __expf(lv[u] - m2) : 0.f;
      s2 += lv[u];
    }
    s2 = wave_sum(s2);
    const float is = 1.f / s2;
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const int k = lane + 64 * u;
      if (k < K) {
        const float yv = lv[u] * is;
        y[k] = yv;
        a.Y[g0 + k] = yv;
      }
    }
  }
  if (lane == 0) {
    sh[w] = klsum;
    sh[NW + w] = entsum;
  }
  __syncthreads();
  if (a.ppl) {  // the waves' Q column sums into the (now free) logits region
#pragma unroll
    for (int u = 0; u < KPL; ++u)
      if (lane + 64 * u < K) R1[w * K + lane + 64 * u] = qcol[u];
  }
  HSTAMP(5);
  // feats = Y C^T
  tile_mma_any<NW>(R2, ld2, K, bkc(a.C, K, D), D, w, lane, [&](int c0, f4 acc) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 4 * q + g;
      if (row < nr) a.feats[(long)(row0 + row) * D + c0 + r] = acc[g];
    }
  });
  if (!a.kl_out && !a.ppl) return;
  if (a.ppl) {
    __syncthreads();
    for (int k = tid; k < K; k += NT) {
      float c = 0.f;  // wave order
#pragma unroll
      for (int v = 0; v < NW; ++v) c += R1[v * K + k];
      st_agent(a.qcolpart + (long)blockIdx.x * K + k, c);
    }
  }
  if (tid == 0) {
    double kls = 0.0, ens = 0.0;  // wave order
#pragma unroll
    for (int v = 0; v < NW; ++v) kls += sh[v], ens += sh[NW + v];
    st_agent(a.klpart + blockIdx.x, kls);
    st_agent(a.entpart + blockIdx.x, ens);
  }
  HSTAMP(6);
  if (!last_workgroup(&g_head_ticket[0], flag)) return;
  const int nt = gridDim.x;
  if (a.kl_out && w == 0) {
    double t = 0.0;  // lane-strided partial sums, then a fixed shuffle tree: deterministic
    for (int i = lane; i < nt; i += 64) t += ld_agent(a.klpart + i);
    t = wave_sum_d(t);
    if (lane == 0) *a.kl_out = (float)(ld_agent(a.kl_small) * ((double)a.B / a.N) + t);
  }
  if (!a.ppl) return;
  // perplexities (perplex_kernel's formulas): exp(sum of row entropies / B),
  // exp(entropy of the column sums normalised by their total)
  double te = 0.0;
  for (int i = tid; i < nt; i += NT) te += ld_agent(a.entpart + i);
  te = block_sum_dd(te, sh);
  double tot = 0.0;
  for (int k = tid; k < K; k += NT) {
    float c = 0.f;  // tile order, 32 tiles' loads in flight
    int i = 0;
    for (; i + 32 <= nt; i += 32) {
      float v8[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v8[u] = ld_agent(a.qcolpart + (long)(i + u) * K + k);
#pragma unroll
      for (int u = 0; u < 32; ++u) c += v8[u];
    }
    for (; i < nt; ++i) c += ld_agent(a.qcolpart + (long)i * K + k);
    R1[k] = c;
    tot += c;
  }
  tot = block_sum_dd(tot, sh);
  double be = 0.0;
  for (int k = tid; k < K; k += NT) {
    const double bm = R1[k] / tot;
    if (bm > 0) be += -bm * log(bm);
  }
  be = block_sum_dd(be, sh);
  if (tid == 0) {
    a.ppl[0] = (float)exp(te / a.B);
    a.ppl[1] = (float)exp(be);
  }
  HSTAMP(7);
}

struct HeadBwdArgs {
  int B, Hm, D, K; float it;                // it: 1 / tau (Gumbel mode), else 1
  int Kv; float rsD;                        // as HeadFwdArgs
  const float *dfeat, *dkl, *Y, *Q, *v, *elog, *Z1, *C, *W2;
  const float *p, *alpha, *tri; const double* kl_small; double N; float a0;
  float* dfeat_copy;                       // the stacked [d_feats; U] operand of dC (top half), or null
  float *dLs, *dU, *dZ1;                   // dLs = d_logits / sqrt(D)
  float* colpart;                          // tiles x (D + Hm + K)
  float *db2, *db1, *dpsl;                 // last workgroup's outputs (each may be null)
  const float *CT, *W2T;                   // transposed copies written by the forward head
  unsigned long long* prof;                // diagnostics: per-tile phase stamps (tiles x 8), or null
};
constexpr int HEAD_THREADS = 512;  // 8 waves per 16-row tile (4: the U / dZ1 products ran two column passes per wave)
inline size_t head_bwd_lds(int Hm, int D, int K) {
  return ((size_t)HEAD_ROWS * (K + 4) + (size_t)HEAD_ROWS * (D + 4) + (size_t)HEAD_ROWS * (Hm + 4) +
          (size_t)(HEAD_THREADS / 64 + 2) * K) *
             4 + 16 * sizeof(double) + 16;
}

template <int KPL>
struct HeadRow {  // one row's backward inputs, KPL per lane
  float y[KPL], q[KPL], vb;
};
template <int KPL>
DEV HeadRow<KPL> head_row_load(const HeadBwdArgs& a, int brow, bool valid, int lane) {
  HeadRow<KPL> h;
  const long g0 = (long)brow * a.K;
#pragma unroll
  for (int u = 0; u < KPL; ++u) {
    const int k = lane + 64 * u;
    const bool ok = valid && k < a.K;
    h.y[u] = ok ? a.Y[g0 + k] : 0.f;
    h.q[u] = ok ? a.Q[g0 + k] : 0.f;
  }
  h.vb = valid ? a.v[brow] : 0.f;
  return h;
}

template <int KPL, int NT>
__global__ __launch_bounds__(NT) void samp_head_bwd(HeadBwdArgs a) {
  constexpr int NW = NT / 64, RPW = HEAD_ROWS / NW;  // waves, rows per wave
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  const int Hm = a.Hm, D = a.D, K = a.K;
  const int ld1 = K + 4, ld2 = D + 4, ldz = Hm + 4;
  float* R1 = hsm;                    // dY, then dL
  float* R2 = R1 + HEAD_ROWS * ld1;   // d_feats, then dU
  float* ZL = R2 + HEAD_ROWS * ld2;   // Z1 tile
  float* QcL = ZL + HEAD_ROWS * ldz;  // per-wave Q column sums (NW x K); the last workgroup's Qsum
  float* elogL = QcL + NW * K;
  double* sh = reinterpret_cast<double*>(elogL + K);
  int* flag = reinterpret_cast<int*>(sh + 16);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * HEAD_ROWS, nr = min(HEAD_ROWS, a.B - row0);
  const int NC = D + Hm + K;
  float* part = a.colpart + (long)blockIdx.x * NC;
  HSTAMP(0);
  // stage d_feats, Z1 and elog; zero the Q column sums
  {  // one round trip per iteration: d_feats, Z1 and elog loads all in flight
    const __amdgpu_buffer_rsrc_t rF = make_rsrc(a.dfeat + (long)row0 * D, (uint32_t)nr * D * 4u);
    const __amdgpu_buffer_rsrc_t rZ = make_rsrc(a.Z1 + (long)row0 * Hm, (uint32_t)nr * Hm * 4u);
    const __amdgpu_buffer_rsrc_t rE = make_rsrc(a.elog, (uint32_t)K * 4u);
    const int nF = HEAD_ROWS * D / 4, nZ = HEAD_ROWS * Hm / 4, nE = K / 4;
    const int nAll = nF + nZ + nE;
    constexpr int U = 4;
    for (int e0 = tid; e0 < nAll; e0 += NT * U) {
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + NT * u;
        const int ez = e - nF, ee = ez - nZ;
        // rows >= nr lie beyond the d_feats / Z1 resources and read 0
        const uint32_t o = e < nF ? (uint32_t)e * 16u : ez < nZ ? (uint32_t)ez * 16u : ee < nE ? (uint32_t)ee * 16u : 0x80000000u;
        v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(e < nF ? rF : ez < nZ ? rZ : rE, o, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + NT * u;
        if (e < nF) {
          const int rr = e / (D / 4), c = (e - rr * (D / 4)) * 4;
          *reinterpret_cast<f4*>(R2 + rr * ld2 + c) = v[u];
        } else if (e < nF + nZ) {
          const int ez = e - nF, rr = ez / (Hm / 4), c = (ez - rr * (Hm / 4)) * 4;
          *reinterpret_cast<f4*>(ZL + rr * ldz + c) = v[u];
        } else if (e < nAll) {
          *reinterpret_cast<f4*>(elogL + (e - nF - nZ) * 4) = v[u];
        }
      }
    }
  }
  for (int k = tid; k < NW * K; k += NT) QcL[k] = 0.f;
  __syncthreads();
  if (a.dfeat_copy) {
    const int d4 = D >> 2;
    for (int e = tid; e < nr * d4; e += NT) {
      const int rr = e / d4, c = (e - rr * d4) * 4;
      *reinterpret_cast<f4*>(a.dfeat_copy + (long)(row0 + rr) * D + c) = *reinterpret_cast<const f4*>(R2 + rr * ld2 + c);
    }
  }
  HSTAMP(1);
  // dY = d_feats C
  tile_mma_any<NW>(R2, ld2, D, bkc(a.CT, D, K), K, w, lane, [&](int c0, f4 acc) {
#pragma unroll
    for (int g = 0; g < 4; ++g) R1[(4 * q + g) * ld1 + c0 + r] = acc[g];
  });
  __syncthreads();
  HSTAMP(2);
  // dL = Y (dY - sum Y dY) / tau  +  s Q ((log Q - elog) - v_b)
  // (sample_softmax_bwd + kl_rows_bwd), one wave per row; the next row's
  // Y / Q / v_b loads are in flight while this row is reduced
  const float s = *a.dkl, rs = a.rsD;
  {
    const int rbase = w * RPW;
    float* qc = QcL + w * K;
    HeadRow<KPL> cur = head_row_load<KPL>(a, row0 + rbase, rbase < nr, lane);
    for (int rr = 0; rr < RPW; ++rr) {
      const int row = rbase + rr;
      HeadRow<KPL> nxt = cur;
      if (rr + 1 < RPW) nxt = head_row_load<KPL>(a, row0 + row + 1, row + 1 < nr, lane);
      float* d = R1 + row * ld1;
      if (row < nr) {
        const long g0 = (long)(row0 + row) * K;
        float sdy = 0.f;
#pragma unroll
        for (int u = 0; u < KPL; ++u)
          if (lane + 64 * u < K) sdy += cur.y[u] * d[lane + 64 * u];
        sdy = wave_sum(sdy);
#pragma unroll
        for (int u = 0; u < KPL; ++u) {
          const int k = lane + 64 * u;
          if (k < K) {
            const float g1 = cur.y[u] * (d[k] - sdy) * a.it;
            const float qv = cur.q[u];
            const float g2 = s * qv * ((__logf(fmaxf(qv, 1e-38f)) - elogL[k]) - cur.vb);
            const float dl = g1 + g2;
            d[k] = dl;
            a.dLs[g0 + k] = dl * rs;
            qc[k] += qv;
          }
        }
      } else {
        for (int k = lane; k < K; k += 64) d[k] = 0.f;
      }
      cur = nxt;
    }
  }
  __syncthreads();
  // Qsum partial of this tile (the prior gradient's column sums)
  for (int k = tid; k < K; k += NT) {
    float c = 0.f;  // wave order
#pragma unroll
    for (int v = 0; v < NW; ++v) c += QcL[v * K + k];
    st_agent(part + D + Hm + k, c);
  }
  HSTAMP(3);
  // dU = dL C^T / sqrt(D)  (+ the db2 partial)
  tile_mma_any<NW>(R1, ld1, K, bkc(a.C, K, D), D, w, lane, [&](int c0, f4 acc) {
    const int col = c0 + r;
    f4 v;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 4 * q + g;
      v[g] = rs * acc[g];
      R2[row * ld2 + col] = v[g];
      if (row < nr) a.dU[(long)(row0 + row) * D + col] = v[g];
    }
    const float cs = tile_colsum(v);  // rows >= nr are zero (dL rows zeroed)
    if (q == 0) st_agent(part + col, cs);
  });
  __syncthreads();
  HSTAMP(4);
  // dZ1 = (dU W2) (1 - Z1^2)  (+ the db1 partial)
  tile_mma_any<NW>(R2, ld2, D, bkc(a.W2T, D, Hm), Hm, w, lane, [&](int c0, f4 acc) {
    const int col = c0 + r;
    f4 v;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 4 * q + g;
      const float z = ZL[row * ldz + col];
      v[g] = row < nr ? acc[g] * (1.f - z * z) : 0.f;
      if (row < nr) a.dZ1[(long)(row0 + row) * Hm + col] = v[g];
    }
    const float cs = tile_colsum(v);
    if (q == 0) st_agent(part + D + col, cs);
  });
  HSTAMP(5);
  if (!last_workgroup(&g_head_ticket[1], flag)) return;
  // last workgroup: column sums over the tiles (tile order) -> db2, db1,
  // Qsum; then the Dirichlet prior's gradient
  const int nt = gridDim.x;
  for (int c = tid; c < NC; c += NT) {
    float t = 0.f;  // tile order; 32 tiles' loads in flight (8: 12 us for 640 columns x 32 tiles)
    int i = 0;
    for (; i + 32 <= nt; i += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = ld_agent(a.colpart + (long)(i + u) * NC + c);
#pragma unroll
      for (int u = 0; u < 32; ++u) t += v[u];
    }
    for (; i < nt; ++i) t += ld_agent(a.colpart + (long)i * NC + c);
    if (c < D) { if (a.db2) a.db2[c] = t; }
    else if (c < D + Hm) { if (a.db1) a.db1[c - D] = t; }
    else QcL[c - D - Hm] = t;
  }
  __syncthreads();
  HSTAMP(6);
  if (a.dpsl) prior_bwd_block(a.p, a.alpha, a.tri, a.kl_small, QcL, a.Kv, a.B, a.N, a.a0, s, a.dpsl, sh);
  HSTAMP(7);
}

// KPL dispatch: K <= 64 * KPL
template <template <int> class F, class... Args>
static int head_dispatch(int K, Args&&... args) {
  if (K <= 64) return F<1>::run(args...);
  if (K <= 128) return F<2>::run(args...);
  if (K <= 256) return F<4>::run(args...);
  if (K <= 512) return F<8>::run(args...);
  if (K <= 1024) return F<16>::run(args...);
  return ABCD_EINVAL;
}
static std::mutex g_head_attr_mu;
static int head_lds_attr(const void* fn, size_t lds) {  // once per kernel instance needing > 64 KiB
  if (lds <= 64 * 1024) return 0;
  static const void* done[16];
  std::lock_guard<std::mutex> lk(g_head_attr_mu);
  int i = 0;
  for (; i < 16 && done[i]; ++i)
    if (done[i] == fn) return 0;
  ABCD_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  if (i < 16) done[i] = fn;
  return 0;
}
template <int KPL>
struct HeadFwdLaunch {
  static int run(const HeadFwdArgs& a, int grid, size_t lds, hipStream_t s) {
    ABCD_TRY((hipError_t)head_lds_attr((const void*)samp_head_fwd<KPL, HEAD_THREADS>, lds));
    samp_head_fwd<KPL, HEAD_THREADS><<<grid, HEAD_THREADS, lds, s>>>(a);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
};
template <int KPL>
struct HeadBwdLaunch {
  static int run(const HeadBwdArgs& a, int grid, size_t lds, hipStream_t s) {
    ABCD_TRY((hipError_t)head_lds_attr((const void*)samp_head_bwd<KPL, HEAD_THREADS>, lds));
    samp_head_bwd<KPL, HEAD_THREADS><<<grid, HEAD_THREADS, lds, s>>>(a);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
};

struct SampWS {
  float *W1T[2], *W2T[2], *CT;
  float *Z1[2], *U, *Y, *Q, *v, *p, *alpha, *elog, *tri, *Qsum, *MV, *EPS;
  double* kl_small;
  float *dY, *dL, *dU, *dZ1[2], *dMV, *dh2;
  float *FU, *YdL;     // stacked dC operands: [d_feats; U] (2B x D), [Y; dL / sqrt(D)] (2B x K)
  float* colpart;      // sampler head backward: per-tile column sums
  double* klpart;      // sampler head forward: per-tile KL row sums
  double* entpart;     // ... per-tile row-entropy sums (perplexities)
  float* qcolpart;     // ... per-tile Q column sums (perplexities)
  float* ppl3;         // per-method perplexities (fused entry's fallback)
  float* scratch;
  size_t scratch_floats;
};

static int samp_check(const abcd_sampler_cfg* c) {
  if (!c || c->input_size <= 0 || c->input_size % 16 || c->mlp_hidden <= 0 || c->mlp_hidden % 16 ||
      c->feature_dim <= 0 || c->feature_dim % 16)
    return ABCD_EINVAL;
  if (!c->plain && (c->num_categories <= 0 || c->num_categories % 16)) return ABCD_EINVAL;
  if (c->valid_categories < 0 || c->valid_categories > c->num_categories || c->valid_feature_dim < 0 ||
      c->valid_feature_dim > c->feature_dim)
    return ABCD_EINVAL;
  return 0;
}
// categories of a zero-padded model (modules/padding.py): the first Kv of the K columns
static int kvalid(const abcd_sampler_cfg* c) { return c->valid_categories ? c->valid_categories : c->num_categories; }
// the logits scale 1 / sqrt(D) of model.py:589 with the MODEL's feature dim
static float rs_dim(const abcd_sampler_cfg* c) {
  return 1.f / sqrtf((float)(c->valid_feature_dim ? c->valid_feature_dim : c->feature_dim));
}

static SampWS carve_sampler(Arena& A, const abcd_sampler_cfg* c, int B) {
  SampWS w{};
  const int E = c->input_size, Hm = c->mlp_hidden, D = c->feature_dim, K = c->plain ? 16 : c->num_categories;
  const int nm = c->plain ? 2 : 1;
  for (int k = 0; k < nm; ++k) {
    w.W1T[k] = A.f((size_t)E * Hm);
    w.W2T[k] = A.f((size_t)Hm * D);
    w.Z1[k] = A.f((size_t)B * Hm);
    w.dZ1[k] = A.f((size_t)B * Hm);
  }
  w.CT = A.f((size_t)K * D);
  w.FU = A.f((size_t)2 * B * D); w.YdL = A.f((size_t)2 * B * K);
  w.U = w.FU ? w.FU + (size_t)B * D : nullptr; w.Y = w.YdL;
  w.Q = A.f((size_t)B * K); w.v = A.f(B);
  const int ntile = cdiv(B, HEAD_ROWS);
  w.colpart = A.f((size_t)ntile * (D + Hm + K)); w.klpart = A.d(ntile);
  w.entpart = A.d(ntile); w.qcolpart = A.f((size_t)ntile * K); w.ppl3 = A.f(4);
  w.p = A.f(K); w.alpha = A.f(K); w.elog = A.f(K); w.tri = A.f(K); w.Qsum = A.f(K);
  w.MV = A.f((size_t)B * 2 * D); w.EPS = A.f((size_t)B * D);
  w.kl_small = A.d(8);
  w.dY = A.f((size_t)B * K); w.dL = A.f((size_t)B * std::max(K, 2 * D)); w.dU = A.f((size_t)B * D); w.dMV = A.f((size_t)B * 2 * D);
  w.dh2 = A.f((size_t)B * E);
  w.scratch_floats = std::max<size_t>((size_t)16 * std::max({(size_t)Hm * E, (size_t)D * K, (size_t)D * Hm}),
                                      (size_t)1 << 20);
  w.scratch = A.f(w.scratch_floats);
  return w;
}

}  // namespace abcd

using namespace abcd;

extern "C" size_t abcd_sampler_workspace_bytes(const abcd_sampler_cfg* c, int B) {
  if (samp_check(c) || B <= 0) return 0;
  Arena A(nullptr, 0);
  carve_sampler(A, c, B);
  return A.off + 256;
}

extern "C" int abcd_sampler_forward(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h, int B,
                                    float* logits, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && h && logits && ws && B > 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  SampWS w = carve_sampler(A, c, B);
  ABCD_REQUIRE(A.ok);
  const int E = c->input_size, Hm = c->mlp_hidden, D = c->feature_dim, K = c->num_categories;
  if (c->plain) {  // Sampler.forward: [mean | log_var] = [MLP0(h) | MLP1(h)]
    for (int k = 0; k < 2; ++k) {
      const abcd_mlp_w& m = p->mlp[k];
      ABCD_TRY((hipError_t)gemm(s, B, Hm, E, opKC(h, E, B), opKC(m.w1, E, Hm), w.Z1[k], Hm, 1.f, 0.f, m.b1, ACT_TANH,
                                nullptr, 0));
      ABCD_TRY((hipError_t)gemm(s, B, D, Hm, opKC(w.Z1[k], Hm, B), opKC(m.w2, Hm, D), w.MV + k * D, 2 * D, 1.f, 0.f,
                                m.b2, ACT_NONE, nullptr, 0));
    }
    ABCD_TRY(hipMemcpyAsync(logits, w.MV, (size_t)B * 2 * D * 4, hipMemcpyDeviceToDevice, s));
    return 0;
  }
  const abcd_mlp_w& m = p->mlp[0];
  // K = E = 1024 over 64 output tiles: split-K (8 slabs + reduce, tanh in the
  // reduce epilogue) fills the chip instead of 64 long workgroups
  ABCD_TRY((hipError_t)gemm(s, B, Hm, E, opKC(h, E, B), opKC(m.w1, E, Hm), w.Z1[0], Hm, 1.f, 0.f, m.b1, ACT_TANH,
                            w.scratch, w.scratch_floats));
  ABCD_TRY((hipError_t)gemm(s, B, D, Hm, opKC(w.Z1[0], Hm, B), opKC(m.w2, Hm, D), w.U, D, 1.f, 0.f, m.b2, ACT_NONE,
                            nullptr, 0));
  // logits = U @ codebook / sqrt(D)   (codebook D x K used as a K-major operand)
  ABCD_TRY((hipError_t)gemm(s, B, K, D, opKC(w.U, D, B), opKM(p->codebook, K, K), logits, K,
                            rs_dim(c), 0.f, nullptr, ACT_NONE, nullptr, 0));
  // the transposed codebook / W2 the fused backward reads (the fused forward writes them in-kernel)
  ABCD_TRY((hipError_t)pack2d(s, p->codebook, K, K, D, true, w.CT, D, K, D));
  return pack2d(s, m.w2, Hm, Hm, D, true, w.W2T[0], D, Hm, D);
}

extern "C" int abcd_sampler_sample(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* logits,
                                   int B, int mode, float temperature, const float* noise, uint64_t seed,
                                   uint64_t offset, float* feats, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && logits && feats && ws && B > 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  SampWS w = carve_sampler(A, c, B);
  ABCD_REQUIRE(A.ok);
  const int D = c->feature_dim, K = c->num_categories;
  if (c->plain) {  // logits = [mean | log_var] (B x 2f); keep the stash self-contained for the backward
    if (logits != w.MV) ABCD_TRY(hipMemcpyAsync(w.MV, logits, (size_t)B * 2 * D * 4, hipMemcpyDeviceToDevice, s));
    plain_sample<<<std::max(1, std::min(4096, cdiv((long)B * D, 256))), 256, 0, s>>>(
        w.MV, B, D, c->valid_feature_dim ? c->valid_feature_dim : D, noise, seed, offset, feats, w.EPS);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  ABCD_REQUIRE(mode == ABCD_SAMPLE_SOFTMAX || temperature > 0.f);
  sample_softmax_rows<<<cdiv(B, 4), 256, 0, s>>>(logits, B, K, kvalid(c), mode == ABCD_SAMPLE_GUMBEL,
                                                 mode == ABCD_SAMPLE_GUMBEL ? temperature : 1.f, noise, seed, offset,
                                                 w.Y);
  ABCD_CHECK_LAUNCH();
  // feats = Y @ codebook^T
  return gemm(s, B, D, K, opKC(w.Y, K, B), opKC(p->codebook, K, D), feats, D, 1.f, 0.f, nullptr, ACT_NONE, nullptr,
              0);
}

extern "C" int abcd_sampler_kl(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* logits, int B,
                               double N, float* kl_out, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && kl_out && ws && B > 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  SampWS w = carve_sampler(A, c, B);
  ABCD_REQUIRE(A.ok);
  if (c->plain) {
    ABCD_REQUIRE(logits);
    if (logits != w.MV)
      ABCD_TRY(hipMemcpyAsync(w.MV, logits, (size_t)B * 2 * c->feature_dim * 4, hipMemcpyDeviceToDevice, s));
    plain_kl<<<1, 1024, 0, s>>>(w.MV, B, c->feature_dim, kl_out);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  ABCD_REQUIRE(logits && N > 0);
  const int K = c->num_categories;
  kl_prior<<<1, 256, 0, s>>>(p->posterior_shape_logits, K, kvalid(c), N, p->prior_concentration, w.p, w.alpha,
                             w.elog, w.tri, w.kl_small);
  ABCD_CHECK_LAUNCH();
  kl_rows<<<cdiv(B, 4), 256, 0, s>>>(logits, B, K, kvalid(c), w.elog, w.Q, w.v);
  ABCD_CHECK_LAUNCH();
  kl_final<<<1, 256, 0, s>>>(w.kl_small, w.v, B, N, kl_out);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// ---- the fused training-step forward: forward + sample + kl in two launches ----
constexpr size_t HEAD_LDS_MAX = 160 * 1024;

extern "C" int abcd_sampler_prior(const abcd_sampler_cfg* c, const abcd_sampler_params* p, int B, double N,
                                  void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && ws && B > 0 && N > 0);
  if (c->plain) return 0;
  Arena A(ws, ws_bytes);
  SampWS w = carve_sampler(A, c, B);
  ABCD_REQUIRE(A.ok);
  kl_prior<<<1, 256, 0, (hipStream_t)stream>>>(p->posterior_shape_logits, c->num_categories, kvalid(c), N,
                                               p->prior_concentration, w.p, w.alpha, w.elog, w.tri, w.kl_small);
  ABCD_CHECK_LAUNCH();
  return 0;
}

extern "C" int abcd_sampler_forward_fused(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h,
                                          int B, int mode, float temperature, const float* noise, uint64_t seed,
                                          uint64_t offset, double N, float* logits, float* feats, float* kl_out,
                                          float* ppl_out, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && h && logits && feats && ws && B > 0);
  const bool prior_ready = (mode & ABCD_SAMPLE_PRIOR_READY) != 0;
  mode &= ~ABCD_SAMPLE_PRIOR_READY;
  const int E = c->input_size, Hm = c->mlp_hidden, D = c->feature_dim, K = c->num_categories;
  const size_t lds = c->plain ? 0 : head_fwd_lds(Hm, D, K);
  if (c->plain || lds > HEAD_LDS_MAX || K > 1024) {  // the three reference methods in turn
    ABCD_TRY((hipError_t)abcd_sampler_forward(c, p, h, B, logits, ws, ws_bytes, stream));
    ABCD_TRY((hipError_t)abcd_sampler_sample(c, p, logits, B, mode, temperature, noise, seed, offset, feats, ws,
                                             ws_bytes, stream));
    if (kl_out) ABCD_TRY((hipError_t)abcd_sampler_kl(c, p, logits, B, N, kl_out, ws, ws_bytes, stream));
    if (ppl_out && !c->plain) {  // the first two of abcd_perplexities' three values
      Arena A(ws, ws_bytes);
      SampWS w = carve_sampler(A, c, B);
      ABCD_REQUIRE(A.ok);
      ABCD_TRY((hipError_t)perplexities_ld(logits, B, K, kvalid(c), p->posterior_shape_logits, w.ppl3, stream));
      ABCD_TRY(hipMemcpyAsync(ppl_out, w.ppl3, 2 * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    }
    return 0;
  }
  ABCD_REQUIRE(mode == ABCD_SAMPLE_SOFTMAX || temperature > 0.f);
  ABCD_REQUIRE(!kl_out || N > 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  SampWS w = carve_sampler(A, c, B);
  ABCD_REQUIRE(A.ok);
  const abcd_mlp_w& m = p->mlp[0];
  int Z = 0;
  ABCD_TRY((hipError_t)gemm_slabs(s, B, Hm, E, opKC(h, E, B), opKC(m.w1, E, Hm), w.scratch,
                                        std::min(w.scratch_floats, (size_t)HEAD_MAX_SLABS * B * Hm), &Z));
  HeadFwdArgs a{};
  a.B = B; a.Hm = Hm; a.D = D; a.K = K; a.nslab = Z; a.Kv = kvalid(c); a.rsD = rs_dim(c);
  a.slab = w.scratch; a.b1 = m.b1; a.W2 = m.w2; a.b2 = m.b2; a.C = p->codebook; a.psl = p->posterior_shape_logits;
  a.N = N > 0 ? N : 1.0; a.a0 = p->prior_concentration;
  a.gumbel = mode == ABCD_SAMPLE_GUMBEL; a.tau = a.gumbel ? temperature : 1.f;
  a.noise = noise; a.seed = seed; a.offset = offset;
  a.prior_ready = prior_ready ? 1 : 0;
  a.Z1 = w.Z1[0]; a.U = w.U; a.logits = logits; a.Y = w.Y; a.Q = w.Q; a.v = w.v; a.feats = feats;
  a.p = w.p; a.alpha = w.alpha; a.elog = w.elog; a.tri = w.tri; a.kl_small = w.kl_small;
  a.klpart = w.klpart; a.kl_out = kl_out;
  a.CT = w.CT; a.W2T = w.W2T[0];
  a.ppl = ppl_out; a.entpart = w.entpart; a.qcolpart = w.qcolpart;
  a.prof = debug_prof_buf(16);
  const int grid = cdiv(B, HEAD_ROWS);
  ABCD_TRY((hipError_t)head_dispatch<HeadFwdLaunch>(K, a, grid, lds, s));
  note_dispatch(TK_SAMP_FWD, "gemm_slabs[%d] + samp_head_fwd grid %d", Z, grid);
  return 0;
}

// ---- backward, split the way autograd sees the reference (three Functions) ----
// Every piece takes two streams: `s` carries the data-gradient chain to d_h
// (the encoder backward waits on it), `sw` the parameter gradients, which
// nothing reads before the caller joins sw (clip + SGD).  With sw == s it is
// one in-order stream.  Only sw uses the workspace's split-K scratch, so the
// two never share a buffer that either writes.
namespace {
struct SideWork {  // parameter-gradient launches: side-stream tiling when sw != s
  GemmSideScope scope;
  explicit SideWork(hipStream_t s, hipStream_t sw) : scope(sw != s) {}
};
}  // namespace

// sample():  d_feats -> d_logits (write), d_codebook (write)
//   ABCD : feats = softmax((l+g)/tau) C^T        plain: feats = mu + e^{lv/2} eps
static int samp_sample_bwd(const abcd_sampler_cfg* c, const abcd_sampler_params* p, int B, int mode,
                           float temperature, const float* d_feats, float* d_logits, float* d_codebook,
                           const SampWS& w, hipStream_t s, hipStream_t sw) {
  const int D = c->feature_dim, K = c->num_categories;
  if (c->plain) {
    plain_dparams<<<std::max(1, std::min(4096, cdiv((long)B * D, 256))), 256, 0, s>>>(w.MV, w.EPS, B, D, d_feats,
                                                                                      nullptr, d_logits);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  ABCD_TRY((hipError_t)gemm(s, B, K, D, opKC(d_feats, D, B), opKM(p->codebook, K, K), w.dY, K, 1.f, 0.f, nullptr,
                            ACT_NONE, nullptr, 0));
  if (d_codebook) {
    SideWork side(s, sw);
    ABCD_TRY((hipError_t)gemm(sw, D, K, B, opKM(d_feats, D, D), opKM(w.Y, K, K), d_codebook, K, 1.f, 0.f, nullptr,
                              ACT_NONE, w.scratch, w.scratch_floats));
  }
  sample_softmax_bwd<<<cdiv(B, 4), 256, 0, s>>>(w.Y, w.dY, B, K, mode == ABCD_SAMPLE_GUMBEL ? temperature : 1.f, 0,
                                                d_logits);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// kl_divergence(): d_kl (device scalar) -> d_logits (write or accumulate), d_psl (write)
static int samp_kl_bwd(const abcd_sampler_cfg* c, const abcd_sampler_params* p, int B, double N, const float* d_kl,
                       int accumulate, float* d_logits, float* d_psl, const SampWS& w, hipStream_t s,
                       hipStream_t sw) {
  const int D = c->feature_dim, K = c->num_categories;
  if (c->plain) {
    if (accumulate) {
      plain_dparams<<<std::max(1, std::min(4096, cdiv((long)B * D, 256))), 256, 0, s>>>(w.MV, w.EPS, B, D, nullptr,
                                                                                        d_kl, w.dMV);
      ABCD_CHECK_LAUNCH();
      return add_vec(s, d_logits, w.dMV, d_logits, B * 2 * D);
    }
    plain_dparams<<<std::max(1, std::min(4096, cdiv((long)B * D, 256))), 256, 0, s>>>(w.MV, w.EPS, B, D, nullptr,
                                                                                      d_kl, d_logits);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  kl_rows_bwd<<<cdiv(B, 4), 256, 0, s>>>(w.Q, w.elog, w.v, B, K, d_kl, accumulate, d_logits);
  ABCD_CHECK_LAUNCH();
  if (d_psl) {  // forward products only: no wait on s beyond the caller's fork
    SideWork side(s, sw);
    ABCD_TRY((hipError_t)colsum(sw, w.Q, K, B, K, nullptr, w.Qsum, 0.f, w.scratch, w.scratch_floats));
    kl_prior_bwd<<<1, 256, 0, sw>>>(w.p, w.alpha, w.tri, w.kl_small, w.Qsum, kvalid(c), B, N,
                                    p->prior_concentration, d_kl, d_psl);
    ABCD_CHECK_LAUNCH();
  }
  return 0;
}

// forward(): d_logits (plain: d [mean|log_var]) -> MLP grads, codebook grad of
// logits = U C / sqrt(D) (written, or accumulated when accumulate_codebook), d_h
static int samp_fwd_bwd(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h, int B,
                        const float* d_logits, float* d_h, const abcd_sampler_grads* g, int accumulate_codebook,
                        const SampWS& w, hipStream_t s, hipStream_t sw) {
  const int E = c->input_size, Hm = c->mlp_hidden, D = c->feature_dim, K = c->num_categories;
  float* sc = w.scratch;
  const size_t scf = w.scratch_floats;
  const int nm = c->plain ? 2 : 1;
  const float* dOut[2];
  long ldOut;
  ABCD_TRY((hipError_t)stream_fork(s, sw, 1));  // d_logits final
  if (c->plain) {
    dOut[0] = d_logits; dOut[1] = d_logits + D; ldOut = 2 * D;
  } else {
    const float rs = rs_dim(c);
    if (g->codebook) {
      SideWork side(s, sw);
      ABCD_TRY((hipError_t)gemm(sw, D, K, B, opKM(w.U, D, D), opKM(d_logits, K, K), g->codebook, K, rs,
                                accumulate_codebook ? 1.f : 0.f, nullptr, ACT_NONE, sc, scf));
    }
    ABCD_TRY((hipError_t)gemm(s, B, D, K, opKC(d_logits, K, B), opKC(p->codebook, K, D), w.dU, D, rs, 0.f, nullptr,
                              ACT_NONE, nullptr, 0));
    ABCD_TRY((hipError_t)stream_fork(s, sw, 2));  // dU
    dOut[0] = w.dU; dOut[1] = nullptr; ldOut = D;
  }
  for (int k = 0; k < nm; ++k) {
    const abcd_mlp_w& m = p->mlp[k];
    const abcd_mlp_g& mg = g->mlp[k];
    {
      SideWork side(s, sw);
      if (mg.w2)
        ABCD_TRY((hipError_t)gemm(sw, D, Hm, B, opKM(dOut[k], ldOut, D), opKM(w.Z1[k], Hm, Hm), mg.w2, Hm, 1.f, 0.f,
                                  nullptr, ACT_NONE, sc, scf));
      if (mg.b2) ABCD_TRY((hipError_t)colsum(sw, dOut[k], ldOut, B, D, nullptr, mg.b2, 0.f, sc, scf));
    }
    ABCD_TRY((hipError_t)pack2d(s, m.w2, Hm, Hm, D, true, w.W2T[k], D, Hm, D));
    ABCD_TRY((hipError_t)gemm(s, B, Hm, D, opKC(dOut[k], ldOut, B), opKC(w.W2T[k], D, Hm), w.dZ1[k], Hm, 1.f, 0.f,
                              nullptr, ACT_NONE, nullptr, 0));
    tanh_bwd_inplace<<<std::max(1, std::min(2048, cdiv((long)B * Hm, 256))), 256, 0, s>>>(w.dZ1[k], w.Z1[k],
                                                                                          (long)B * Hm);
    ABCD_CHECK_LAUNCH();
    ABCD_TRY((hipError_t)stream_fork(s, sw, 3));  // dZ1[k]
    {
      SideWork side(s, sw);
      if (mg.w1)
        ABCD_TRY((hipError_t)gemm(sw, Hm, E, B, opKM(w.dZ1[k], Hm, Hm), opKM(h, E, E), mg.w1, E, 1.f, 0.f, nullptr,
                                  ACT_NONE, sc, scf));
      if (mg.b1) ABCD_TRY((hipError_t)colsum(sw, w.dZ1[k], Hm, B, Hm, nullptr, mg.b1, 0.f, sc, scf));
    }
    if (d_h) {
      ABCD_TRY((hipError_t)pack2d(s, m.w1, E, E, Hm, true, w.W1T[k], Hm, E, Hm));
      ABCD_TRY((hipError_t)gemm(s, B, E, Hm, opKC(w.dZ1[k], Hm, B), opKC(w.W1T[k], Hm, E), d_h, E, 1.f,
                                k == 0 ? 0.f : 1.f, nullptr, ACT_NONE, nullptr, 0));
    }
  }
  return 0;
}

// the codebook / W2 / W1 gradients of the fused path, from the workspace its
// head kernel filled: ONE batched launch (gemm_tn_batch; four split-K GEMM +
// slab-reduction pairs before, ~85 us at c2)
// dC = [d_feats; U]^T [Y; dL / sqrt(D)] (the sample and the logits products in one reduction),
// dW2 = dU^T Z1, dW1 = dZ1^T h
static int samp_fused_params(const abcd_sampler_cfg* c, const float* h, int B, const abcd_sampler_grads* g,
                             const SampWS& w, hipStream_t s) {
  const int E = c->input_size, Hm = c->mlp_hidden, D = c->feature_dim, K = c->num_categories;
  const abcd_mlp_g& mg = g->mlp[0];
  GemmJob jobs[3];
  int nj = 0;
  if (g->codebook) jobs[nj++] = GemmJob{w.FU, D, w.YdL, K, g->codebook, K, D, K, 2 * B, 1.f, 0.f};
  if (mg.w2) jobs[nj++] = GemmJob{w.dU, D, w.Z1[0], Hm, mg.w2, Hm, D, Hm, B, 1.f, 0.f};
  if (mg.w1) jobs[nj++] = GemmJob{w.dZ1[0], Hm, h, E, mg.w1, E, Hm, E, B, 1.f, 0.f};
  return gemm_tn_batch(s, jobs, nj);
}
static bool samp_fused_ok(const abcd_sampler_cfg* c, const float* d_feats, const float* d_kl) {
  return !c->plain && d_feats && d_kl && c->num_categories <= 1024 &&
         head_bwd_lds(c->mlp_hidden, c->feature_dim, c->num_categories) <= HEAD_LDS_MAX;
}

// the fused training-step backward (ABCD, d_feats and d_kl both present):
// samp_head_bwd + the d_h GEMM on `s`; codebook / W2 / W1 gradients on `sw`
static int samp_fused_bwd(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h, int B, int mode,
                          float temperature, double N, const float* d_feats, const float* d_kl, float* d_h,
                          const abcd_sampler_grads* g, const SampWS& w, hipStream_t s, hipStream_t sw) {
  const int E = c->input_size, Hm = c->mlp_hidden, D = c->feature_dim, K = c->num_categories;
  const abcd_mlp_w& m = p->mlp[0];
  const abcd_mlp_g& mg = g->mlp[0];
  HeadBwdArgs a{};
  a.B = B; a.Hm = Hm; a.D = D; a.K = K; a.Kv = kvalid(c); a.rsD = rs_dim(c);
  a.it = 1.f / (mode == ABCD_SAMPLE_GUMBEL ? temperature : 1.f);
  a.dfeat = d_feats; a.dkl = d_kl; a.Y = w.Y; a.Q = w.Q; a.v = w.v; a.elog = w.elog; a.Z1 = w.Z1[0];
  a.C = p->codebook; a.W2 = m.w2;
  a.p = w.p; a.alpha = w.alpha; a.tri = w.tri; a.kl_small = w.kl_small; a.N = N; a.a0 = p->prior_concentration;
  a.dfeat_copy = g->codebook ? w.FU : nullptr;
  a.dLs = w.YdL + (size_t)B * K; a.dU = w.dU; a.dZ1 = w.dZ1[0];
  a.colpart = w.colpart; a.db2 = mg.b2; a.db1 = mg.b1; a.dpsl = g->posterior_shape_logits;
  a.CT = w.CT; a.W2T = w.W2T[0];
  a.prof = debug_prof_buf(32);
  const size_t lds = head_bwd_lds(Hm, D, K);
  const int grid = cdiv(B, HEAD_ROWS);
  ABCD_TRY((hipError_t)head_dispatch<HeadBwdLaunch>(K, a, grid, lds, s));
  note_dispatch(TK_SAMP_BWD, "samp_head_bwd grid %d + d_h gemm", grid);
  if (sw != (hipStream_t)ABCD_DEFER_PARAMS) {
    ABCD_TRY((hipError_t)stream_fork(s, sw, 1));
    GemmSideScope side(sw != s);
    ABCD_TRY((hipError_t)samp_fused_params(c, h, B, g, w, sw));
  }
  if (d_h)
    ABCD_TRY((hipError_t)gemm(s, B, E, Hm, opKC(w.dZ1[0], Hm, B), opKM(m.w1, E, E), d_h, E, 1.f, 0.f, nullptr,
                              ACT_NONE, nullptr, 0));
  return 0;
}

static int samp_ws(const abcd_sampler_cfg* c, int B, void* ws, size_t ws_bytes, SampWS* w) {
  Arena A(ws, ws_bytes);
  *w = carve_sampler(A, c, B);
  return A.ok ? 0 : ABCD_EINVAL;
}

extern "C" int abcd_sampler_sample_backward(const abcd_sampler_cfg* c, const abcd_sampler_params* p, int B, int mode,
                                            float temperature, const float* d_feats, float* d_logits,
                                            float* d_codebook, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && d_feats && d_logits && ws && B > 0);
  SampWS w;
  ABCD_REQUIRE(samp_ws(c, B, ws, ws_bytes, &w) == 0);
  hipStream_t s = (hipStream_t)stream;
  return samp_sample_bwd(c, p, B, mode, temperature, d_feats, d_logits, d_codebook, w, s, s);
}

extern "C" int abcd_sampler_kl_backward(const abcd_sampler_cfg* c, const abcd_sampler_params* p, int B, double N,
                                        const float* d_kl, int accumulate, float* d_logits, float* d_psl, void* ws,
                                        size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && d_kl && d_logits && ws && B > 0);
  SampWS w;
  ABCD_REQUIRE(samp_ws(c, B, ws, ws_bytes, &w) == 0);
  hipStream_t s = (hipStream_t)stream;
  return samp_kl_bwd(c, p, B, N, d_kl, accumulate, d_logits, d_psl, w, s, s);
}

extern "C" int abcd_sampler_forward_backward(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h,
                                             int B, const float* d_logits, float* d_h, const abcd_sampler_grads* g,
                                             int accumulate_codebook, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && h && d_logits && g && ws && B > 0);
  SampWS w;
  ABCD_REQUIRE(samp_ws(c, B, ws, ws_bytes, &w) == 0);
  hipStream_t s = (hipStream_t)stream;
  return samp_fwd_bwd(c, p, h, B, d_logits, d_h, g, accumulate_codebook, w, s, s);
}

// Which workspaces hold a deferred parameter-gradient job: set by a split
// call that actually deferred (fused ABCD path), consumed by
// abcd_sampler_backward_params, which does nothing for a workspace without one
// (the split call then took the unfused path and wrote those gradients itself;
// the products backward_params multiplies were never filled).
static std::mutex g_defer_mu;
static std::vector<const void*> g_deferred;
static void defer_mark(const void* ws, bool on) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  for (size_t i = 0; i < g_deferred.size(); ++i)
    if (g_deferred[i] == ws) {
      if (!on) g_deferred.erase(g_deferred.begin() + (long)i);
      return;
    }
  if (on) g_deferred.push_back(ws);
}
static bool defer_take(const void* ws) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  for (size_t i = 0; i < g_deferred.size(); ++i)
    if (g_deferred[i] == ws) {
      g_deferred.erase(g_deferred.begin() + (long)i);
      return true;
    }
  return false;
}

// fused: sample + kl + forward backward in one call (the training step).
// wgrad_stream (may be NULL or == stream): where the parameter gradients go;
// the caller joins it before reading them.
extern "C" int abcd_sampler_backward_split(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h,
                                           int B, int mode, float temperature, double N, const float* d_feats,
                                           const float* d_kl, float* d_h, const abcd_sampler_grads* g, void* ws,
                                           size_t ws_bytes, void* stream, void* wgrad_stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && h && g && ws && B > 0);
  SampWS w;
  ABCD_REQUIRE(samp_ws(c, B, ws, ws_bytes, &w) == 0);
  hipStream_t s = (hipStream_t)stream;
  bool defer = wgrad_stream == ABCD_DEFER_PARAMS;
  if (defer && !samp_fused_ok(c, d_feats, d_kl)) wgrad_stream = nullptr, defer = false;  // only the fused path defers
  defer_mark(ws, defer);
  hipStream_t sw = wgrad_stream ? (hipStream_t)wgrad_stream : s;
  if (!defer) ABCD_TRY((hipError_t)stream_fork(s, sw, 0));  // d_feats and the forward products
  const int D = c->feature_dim, K = c->num_categories;
  float* dL = c->plain ? w.dMV + 0 : w.dL;
  int have = 0;
  if (c->plain) {
    // plain_dparams handles both terms in one pass
    plain_dparams<<<std::max(1, std::min(4096, cdiv((long)B * D, 256))), 256, 0, s>>>(w.MV, w.EPS, B, D, d_feats,
                                                                                      d_kl, w.dL);
    ABCD_CHECK_LAUNCH();
    dL = w.dL;
    have = 1;
  } else if (samp_fused_ok(c, d_feats, d_kl)) {
    return samp_fused_bwd(c, p, h, B, mode, temperature, N, d_feats, d_kl, d_h, g, w, s, sw);
  } else {
    if (d_feats) {
      ABCD_TRY((hipError_t)samp_sample_bwd(c, p, B, mode, temperature, d_feats, dL, g->codebook, w, s, sw));
      have = 1;
    }
    if (d_kl) {
      ABCD_TRY((hipError_t)samp_kl_bwd(c, p, B, N, d_kl, have, dL, g->posterior_shape_logits, w, s, sw));
      have = 1;
    } else if (g->posterior_shape_logits) {
      ABCD_TRY(hipMemsetAsync(g->posterior_shape_logits, 0, (size_t)K * 4, sw));
    }
    if (!have) {
      ABCD_TRY(hipMemsetAsync(dL, 0, (size_t)B * K * 4, s));
      if (g->codebook) ABCD_TRY(hipMemsetAsync(g->codebook, 0, (size_t)D * K * 4, sw));
    }
  }
  return samp_fwd_bwd(c, p, h, B, dL, d_h, g, c->plain ? 0 : (d_feats ? 1 : 0), w, s, sw);
}

extern "C" int abcd_sampler_backward_params(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h,
                                            int B, const abcd_sampler_grads* g, void* ws, size_t ws_bytes,
                                            void* stream, void* wgrad_stream) {
  ABCD_REQUIRE(samp_check(c) == 0 && p && h && g && ws && B > 0 && wgrad_stream != ABCD_DEFER_PARAMS);
  if (!defer_take(ws)) return 0;  // the split call ran the unfused path, parameter gradients included
  SampWS w;
  ABCD_REQUIRE(samp_ws(c, B, ws, ws_bytes, &w) == 0);
  hipStream_t s = (hipStream_t)stream;
  hipStream_t sw = wgrad_stream ? (hipStream_t)wgrad_stream : s;
  if (sw == s) return samp_fused_params(c, h, B, g, w, s);
  // on the caller's side stream, behind an event on `stream` (the head
  // kernel's stash), in the tiling that co-resides with a persistent kernel
  ABCD_TRY((hipError_t)stream_fork(s, sw, 1));
  GemmSideScope side(true);
  return samp_fused_params(c, h, B, g, w, sw);
}

extern "C" int abcd_sampler_backward(const abcd_sampler_cfg* c, const abcd_sampler_params* p, const float* h, int B,
                                     int mode, float temperature, double N, const float* d_feats, const float* d_kl,
                                     float* d_h, const abcd_sampler_grads* g, void* ws, size_t ws_bytes,
                                     void* stream) {
  return abcd_sampler_backward_split(c, p, h, B, mode, temperature, N, d_feats, d_kl, d_h, g, ws, ws_bytes, stream,
                                     nullptr);
}

// learning.py:171-178 perplexities (single workgroup; diagnostics only).
// One wave per row (rows dealt round-robin over the waves); each wave keeps
// its own column-sum row in LDS (no atomics, deterministic), summed over the
// waves at the end.
// rows of `ld` floats whose first K columns are the categories
template <int KPL>
__global__ __launch_bounds__(1024) void perplex_kernel(const float* logits, int B, int ld, int K, const float* psl,
                                                       float* out) {
  extern __shared__ __attribute__((aligned(16))) float colsum_sh[];  // nw x K floats
  __shared__ double sh[32];
  __shared__ double bc[2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  float* mine = colsum_sh + (long)wv * K;
  for (int k = lane; k < K; k += 64) mine[k] = 0.f;
  double ent = 0.0;
  // PR rows per wave in flight: every row's K values (KPL per lane) are loaded
  // before any is reduced, so the wave pays one memory latency per PR rows
  constexpr int PR = 4;
  for (int b0 = wv * PR; b0 < B; b0 += nw * PR) {
    float v[PR][KPL];
#pragma unroll
    for (int rr = 0; rr < PR; ++rr)
#pragma unroll
      for (int u = 0; u < KPL; ++u) {
        const int k = lane + 64 * u;
        v[rr][u] = (b0 + rr < B && k < K) ? logits[(long)(b0 + rr) * ld + k] : -INFINITY;
      }
#pragma unroll
    for (int rr = 0; rr < PR; ++rr) {
      if (b0 + rr >= B) break;
      float m = -INFINITY;
#pragma unroll
      for (int u = 0; u < KPL; ++u) m = fmaxf(m, v[rr][u]);
      m = wave_max(m);
      float sm = 0.f;
#pragma unroll
      for (int u = 0; u < KPL; ++u) sm += lane + 64 * u < K ? __expf(v[rr][u] - m) : 0.f;
      sm = wave_sum(sm);
      const float ls = __logf(sm), inv = 1.0f / sm;
      float e = 0.f;
#pragma unroll
      for (int u = 0; u < KPL; ++u) {
        const int k = lane + 64 * u;
        if (k < K) {
          const float z = v[rr][u] - m;
          const float qq = __expf(z) * inv;
          e += -qq * (z - ls);
          mine[k] += qq;
        }
      }
      e = wave_sum(e);
      ent += e;
    }
  }
  if (lane == 0) sh[wv] = ent;
  __syncthreads();
  if (tid == 0) { double t = 0; for (int i = 0; i < nw; ++i) t += sh[i]; bc[0] = t; }
  // column sums over the waves (into wave 0's row)
  for (int k = tid; k < K; k += blockDim.x) {
    float c = 0.f;
    for (int i = 0; i < nw; ++i) c += colsum_sh[(long)i * K + k];
    colsum_sh[k] = c;
  }
  __syncthreads();
  double tot = 0.0;
  for (int k = tid; k < K; k += blockDim.x) tot += colsum_sh[k];
  tot = wave_sum_d(tot);
  __syncthreads();
  if (lane == 0) sh[wv] = tot;
  __syncthreads();
  if (tid == 0) { double t = 0; for (int i = 0; i < nw; ++i) t += sh[i]; bc[1] = t; }
  __syncthreads();
  tot = bc[1];
  double be = 0.0, pe = 0.0;
  float pm = -INFINITY;
  for (int k = tid; k < K; k += blockDim.x) pm = fmaxf(pm, psl[k]);
  pm = wave_max(pm);
  __syncthreads();
  if (lane == 0) sh[wv] = pm;
  __syncthreads();
  if (tid == 0) { float t = -INFINITY; for (int i = 0; i < nw; ++i) t = fmaxf(t, (float)sh[i]); sh[31] = t; }
  __syncthreads();
  pm = (float)sh[31];
  double ps = 0.0;
  for (int k = tid; k < K; k += blockDim.x) ps += exp((double)psl[k] - pm);
  ps = wave_sum_d(ps);
  __syncthreads();
  if (lane == 0) sh[wv] = ps;
  __syncthreads();
  double psum = 0.0;
  for (int i = 0; i < nw; ++i) psum += sh[i];
  __syncthreads();
  for (int k = tid; k < K; k += blockDim.x) {
    const double bm = colsum_sh[k] / tot;
    if (bm > 0) be += -bm * log(bm);
    const double pp = exp((double)psl[k] - pm) / psum;
    if (pp > 0) pe += -pp * log(pp);
  }
  be = wave_sum_d(be);
  pe = wave_sum_d(pe);
  __syncthreads();
  if (lane == 0) { sh[wv] = be; sh[16 + wv] = pe; }
  __syncthreads();
  if (tid == 0) {
    double tb = 0, tp = 0;
    for (int i = 0; i < nw; ++i) { tb += sh[i]; tp += sh[16 + i]; }
    out[0] = (float)exp(bc[0] / B);
    out[1] = (float)exp(tb);
    out[2] = (float)exp(tp);
  }
}

// exp(entropy of softmax(posterior_shape_logits)) (learning.py:176-178), one block
__global__ void shape_ppl_kernel(const float* psl, int K, float* out) {
  __shared__ double sh[16];
  const int tid = threadIdx.x;
  double m = -1e300;
  for (int k = tid; k < K; k += blockDim.x) m = fmax(m, (double)psl[k]);
  m = block_max_dd(m, sh);
  double se = 0.0;
  for (int k = tid; k < K; k += blockDim.x) se += exp((double)psl[k] - m);
  se = block_sum_dd(se, sh);
  double pe = 0.0;
  for (int k = tid; k < K; k += blockDim.x) {
    const double pp = exp((double)psl[k] - m) / se;
    if (pp > 0) pe += -pp * log(pp);
  }
  pe = block_sum_dd(pe, sh);
  if (tid == 0) *out = (float)exp(pe);
}

extern "C" int abcd_shape_perplexity(const float* psl, int K, float* out, void* stream) {
  if (!psl || !out || K <= 0) return ABCD_EINVAL;
  shape_ppl_kernel<<<1, 256, 0, (hipStream_t)stream>>>(psl, K, out);
  ABCD_CHECK_LAUNCH();
  return 0;
}

namespace abcd {
int perplexities_ld(const float* logits, int B, int ld, int K, const float* psl, float* out, void* stream) {
  if (!logits || !psl || !out || B <= 0 || K <= 0 || ld < K) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  // as many waves (<= 16) as per-wave column-sum rows fit in 64 KiB of LDS
  int nw = 16;
  while (nw > 1 && (size_t)nw * K * sizeof(float) > 65536) nw >>= 1;
  if ((size_t)nw * K * sizeof(float) > 160 * 1024) return ABCD_EINVAL;
  const size_t lds = (size_t)nw * K * sizeof(float);
  if (K <= 64) perplex_kernel<1><<<1, 64 * nw, lds, s>>>(logits, B, ld, K, psl, out);
  else if (K <= 128) perplex_kernel<2><<<1, 64 * nw, lds, s>>>(logits, B, ld, K, psl, out);
  else if (K <= 256) perplex_kernel<4><<<1, 64 * nw, lds, s>>>(logits, B, ld, K, psl, out);
  else if (K <= 1024) perplex_kernel<16><<<1, 64 * nw, lds, s>>>(logits, B, ld, K, psl, out);
  else return ABCD_EINVAL;
  ABCD_CHECK_LAUNCH();
  return 0;
}
}  // namespace abcd

extern "C" int abcd_perplexities(const float* logits, int B, int K, const float* psl, float* out, void* stream) {
  return abcd::perplexities_ld(logits, B, K, K, psl, out, stream);
}
