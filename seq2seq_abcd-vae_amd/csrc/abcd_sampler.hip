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

namespace abcd {

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

// y = softmax((logits + g) / tau) per row (g = 0 for the plain softmax)
__global__ void sample_softmax_rows(const float* logits, int B, int K, int gumbel, float tau, const float* noise,
                                    uint64_t seed, uint64_t offset, float* Y) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* l = logits + (long)b * K;
  float* y = Y + (long)b * K;
  const float it = 1.f / tau;
  float m = -INFINITY;
  for (int k = lane; k < K; k += 64) {
    float v = l[k];
    if (gumbel) v = (v + (noise ? noise[(long)b * K + k] : philox_gumbel(seed, offset + (uint64_t)b * K + k))) * it;
    y[k] = v;
    m = fmaxf(m, v);
  }
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float e = __expf(y[k] - m);
    y[k] = e;
    s += e;
  }
  s = wave_sum(s);
  const float is = 1.f / s;
  for (int k = lane; k < K; k += 64) y[k] *= is;
}

// KL prior part (one block): p = softmax(psl), alpha = p N + a0, elog = psi(alpha) - psi(S)
// kl_small: [0] = (Eq log q(pi) - Eq log p(pi)), [1] = psi'(S), [2] = S
__global__ void kl_prior(const float* psl, int K, double N, float a0, float* p_out, float* alpha_out,
                         float* elog_out, float* tri_out, double* kl_small) {
  __shared__ double sh[16];
  __shared__ double bc[4];
  const int tid = threadIdx.x;
  // softmax(psl) in double
  double m = -1e300;
  for (int k = tid; k < K; k += blockDim.x) m = fmax(m, (double)psl[k]);
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if ((tid & 63) == 0) sh[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) { double t = sh[0]; for (int i = 1; i < (int)(blockDim.x >> 6); ++i) t = fmax(t, sh[i]); bc[0] = t; }
  __syncthreads();
  m = bc[0];
  double se = 0.0;
  for (int k = tid; k < K; k += blockDim.x) se += exp((double)psl[k] - m);
  se = wave_sum_d(se);
  __syncthreads();
  if ((tid & 63) == 0) sh[tid >> 6] = se;
  __syncthreads();
  if (tid == 0) { double t = 0; for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i]; bc[1] = t; }
  __syncthreads();
  se = bc[1];
  double sa = 0.0;
  for (int k = tid; k < K; k += blockDim.x) {
    const double p = exp((double)psl[k] - m) / se;
    const double al = (double)(float)((float)p * (float)N) + (double)a0;  // fp32 like the reference
    p_out[k] = (float)p;
    alpha_out[k] = (float)al;
    sa += al;
  }
  sa = wave_sum_d(sa);
  __syncthreads();
  if ((tid & 63) == 0) sh[tid >> 6] = sa;
  __syncthreads();
  if (tid == 0) { double t = 0; for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i]; bc[2] = t; }
  __syncthreads();
  const double S = bc[2];
  const double psiS = digamma_d(S);
  double acc = 0.0;  // -sum lgamma(alpha) + sum (alpha-1) elog - (a0-1) sum elog
  for (int k = tid; k < K; k += blockDim.x) {
    const double al = alpha_out[k];
    const double el = digamma_d(al) - psiS;
    elog_out[k] = (float)el;
    tri_out[k] = (float)trigamma_d(al);
    acc += -lgamma(al) + (al - 1.0) * el - ((double)a0 - 1.0) * el;
  }
  acc = wave_sum_d(acc);
  __syncthreads();
  if ((tid & 63) == 0) sh[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    double t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    const double a0d = a0;
    kl_small[0] = lgamma(S) + t - (lgamma(a0d * K) - K * lgamma(a0d));
    kl_small[1] = trigamma_d(S);
    kl_small[2] = S;
  }
}

// per row: Q = softmax(l); v_b = sum_k Q (log Q - elog)
__global__ void kl_rows(const float* logits, int B, int K, const float* elog, float* Q, float* v) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* l = logits + (long)b * K;
  float m = -INFINITY;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, l[k]);
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += __expf(l[k] - m);
  s = wave_sum(s);
  const float ls = __logf(s);
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) {
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

// d posterior_shape_logits (one block)
__global__ void kl_prior_bwd(const float* p, const float* alpha, const float* tri, const double* kl_small,
                             const float* Qsum, int K, int B, double N, float a0, const float* dkl, float* dpsl) {
  __shared__ double sh[16];
  __shared__ double bc[2];
  const int tid = threadIdx.x;
  const double s = *dkl;
  const double r = (double)B / N;
  double sde = 0.0;
  for (int k = tid; k < K; k += blockDim.x) sde += r * ((double)alpha[k] - a0) - Qsum[k];
  sde = wave_sum_d(sde);
  if ((tid & 63) == 0) sh[tid >> 6] = sde;
  __syncthreads();
  if (tid == 0) { double t = 0; for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i]; bc[0] = t; }
  __syncthreads();
  sde = bc[0];
  const double triS = kl_small[1];
  double spd = 0.0;
  for (int k = tid; k < K; k += blockDim.x) {
    const double de = r * ((double)alpha[k] - a0) - Qsum[k];
    const double da = s * (de * tri[k] - triS * sde);
    spd += (double)p[k] * da * N;
  }
  spd = wave_sum_d(spd);
  __syncthreads();
  if ((tid & 63) == 0) sh[tid >> 6] = spd;
  __syncthreads();
  if (tid == 0) { double t = 0; for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i]; bc[1] = t; }
  __syncthreads();
  spd = bc[1];
  for (int k = tid; k < K; k += blockDim.x) {
    const double de = r * ((double)alpha[k] - a0) - Qsum[k];
    const double da = s * (de * tri[k] - triS * sde);
    dpsl[k] = (float)((double)p[k] * (da * N - spd));
  }
}

__global__ void tanh_bwd_inplace(float* dz, const float* z, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dz[i] *= 1.f - z[i] * z[i];
}

// ---- plain Gaussian sampler helpers ----------------------------------------
__global__ void plain_sample(const float* MV, int B, int f, const float* noise, uint64_t seed, uint64_t offset,
                             float* feats, float* EPS) {
  const int n = B * f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / f, j = i % f;
    const float mu = MV[(long)b * 2 * f + j], lv = MV[(long)b * 2 * f + f + j];
    const float e = noise ? noise[i] : philox_normal(seed, offset + (uint64_t)i);
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

struct SampWS {
  float *W1T[2], *W2T[2], *CT;
  float *Z1[2], *U, *Y, *Q, *v, *p, *alpha, *elog, *tri, *Qsum, *MV, *EPS;
  double* kl_small;
  float *dY, *dL, *dU, *dZ1[2], *dMV, *dh2;
  float* scratch;
  size_t scratch_floats;
};

static int samp_check(const abcd_sampler_cfg* c) {
  if (!c || c->input_size <= 0 || c->input_size % 16 || c->mlp_hidden <= 0 || c->mlp_hidden % 16 ||
      c->feature_dim <= 0 || c->feature_dim % 16)
    return ABCD_EINVAL;
  if (!c->plain && (c->num_categories <= 0 || c->num_categories % 16)) return ABCD_EINVAL;
  return 0;
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
  w.U = A.f((size_t)B * D); w.Y = A.f((size_t)B * K); w.Q = A.f((size_t)B * K); w.v = A.f(B);
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
                            1.f / sqrtf((float)D), 0.f, nullptr, ACT_NONE, nullptr, 0));
  return 0;
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
    plain_sample<<<std::max(1, std::min(4096, cdiv((long)B * D, 256))), 256, 0, s>>>(w.MV, B, D, noise, seed, offset,
                                                                                     feats, w.EPS);
    ABCD_CHECK_LAUNCH();
    return 0;
  }
  ABCD_REQUIRE(mode == ABCD_SAMPLE_SOFTMAX || temperature > 0.f);
  sample_softmax_rows<<<cdiv(B, 4), 256, 0, s>>>(logits, B, K, mode == ABCD_SAMPLE_GUMBEL, mode == ABCD_SAMPLE_GUMBEL ? temperature : 1.f,
                                                 noise, seed, offset, w.Y);
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
  kl_prior<<<1, 256, 0, s>>>(p->posterior_shape_logits, K, N, p->prior_concentration, w.p, w.alpha, w.elog, w.tri,
                             w.kl_small);
  ABCD_CHECK_LAUNCH();
  kl_rows<<<cdiv(B, 4), 256, 0, s>>>(logits, B, K, w.elog, w.Q, w.v);
  ABCD_CHECK_LAUNCH();
  kl_final<<<1, 256, 0, s>>>(w.kl_small, w.v, B, N, kl_out);
  ABCD_CHECK_LAUNCH();
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
    kl_prior_bwd<<<1, 256, 0, sw>>>(w.p, w.alpha, w.tri, w.kl_small, w.Qsum, K, B, N, p->prior_concentration, d_kl,
                                    d_psl);
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
    const float rs = 1.f / sqrtf((float)D);
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
  hipStream_t sw = wgrad_stream ? (hipStream_t)wgrad_stream : s;
  ABCD_TRY((hipError_t)stream_fork(s, sw, 0));  // d_feats and the forward products
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
template <int KPL>
__global__ __launch_bounds__(1024) void perplex_kernel(const float* logits, int B, int K, const float* psl,
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
        v[rr][u] = (b0 + rr < B && k < K) ? logits[(long)(b0 + rr) * K + k] : -INFINITY;
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

extern "C" int abcd_perplexities(const float* logits, int B, int K, const float* psl, float* out, void* stream) {
  if (!logits || !psl || !out || B <= 0 || K <= 0) return ABCD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  // as many waves (<= 16) as per-wave column-sum rows fit in 64 KiB of LDS
  int nw = 16;
  while (nw > 1 && (size_t)nw * K * sizeof(float) > 65536) nw >>= 1;
  if ((size_t)nw * K * sizeof(float) > 160 * 1024) return ABCD_EINVAL;
  const size_t lds = (size_t)nw * K * sizeof(float);
  if (K <= 64) perplex_kernel<1><<<1, 64 * nw, lds, s>>>(logits, B, K, psl, out);
  else if (K <= 128) perplex_kernel<2><<<1, 64 * nw, lds, s>>>(logits, B, K, psl, out);
  else if (K <= 256) perplex_kernel<4><<<1, 64 * nw, lds, s>>>(logits, B, K, psl, out);
  else if (K <= 1024) perplex_kernel<16><<<1, 64 * nw, lds, s>>>(logits, B, K, psl, out);
  else return ABCD_EINVAL;
  ABCD_CHECK_LAUNCH();
  return 0;
}
