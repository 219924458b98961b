// abcd_rnn.hip -- packed-sequence RNN encoder and self-feedback decoder for CDNA4.
//
// Hot path of ABCD-VAE/learning.py:149,153 (+ their autograd backward):
//   encoder  model.py:40-66   torch.nn.LSTM/GRU over a PackedSequence (bi-dir)
//   decoder  model.py:147-196 LSTMCell/GRUCell loop with Gaussian self-feedback
//
// Data layout in HBM (all fp32, row-major, "rows" = packed frames, time-major
// exactly like PackedSequence.data; step t owns rows [off_t, off_t + bs_t)):
//   X (L x Fp)   input frames, F padded to Fp = roundup(F, 16) with zeros
//   GX (L x D*G*H) input projection of all frames, one MFMA GEMM per layer
//   Hprev/Cprev (L x H)  the recurrent state each row CONSUMES; written by the
//                predecessor step's epilogue, zeroed by the row's own step when
//                the sequence has no predecessor.  Because row r's operand is
//                row r of Hprev, the recurrent GEMM reads a contiguous block and
//                the weight-gradient GEMM dW_hh = dG^T Hprev is one K=L GEMM.
//   Gst (L x 4H) activated gates (LSTM i,f,g,o; GRU r,z,n,W_hn h+b_hn)
// One launch per time step (both encoder directions share it).  A workgroup
// (4 waves, wave split-K) owns 16 rows x 16 units x G gates, so the LSTM/GRU
// cell update runs in the GEMM epilogue out of LDS.
#include <mutex>
#include <vector>
#include <cstdlib>

#include "abcd_common.h"
#include "abcd_internal.h"
#include "abcd_persist.h"

namespace abcd {

int validate_batch(const int64_t* bs, int T, int L, int B) {
  if (!bs || T <= 0 || L <= 0 || B <= 0) return ABCD_EINVAL;
  if (bs[0] != B) return ABCD_EINVAL;
  long s = 0;
  for (int t = 0; t < T; ++t) {
    if (bs[t] <= 0 || (t && bs[t] > bs[t - 1])) return ABCD_EINVAL;
    s += bs[t];
  }
  return s == L ? 0 : ABCD_EINVAL;
}

static std::vector<int> step_offsets(const int64_t* bs, int T) {
  std::vector<int> off(T + 1, 0);
  for (int t = 0; t < T; ++t) off[t + 1] = off[t] + (int)bs[t];
  return off;
}

// ===========================================================================
// forward step: gates = [x-part] + Hprev_rows @ W_hh^T, cell update epilogue
// ===========================================================================
struct FwdDir {
  const float* Ah; int prev_valid;            // Hprev + off*H
  const float* Whh;                           // G*H x H
  const float* Ax; long ldx; int xrows;       // decoder input rows (Xin + off*ldx)
  const float* Wih; long ldwih; int nchx;     // decoder W_ih (G*H x Fp)
  const float* GX; long ldgx;                 // encoder input projection (bias folded in)
  const float* bih; const float* bhh;         // decoder b_ih(+b_hh for LSTM); GRU b_hh
  float* Gst; float* Cst; float* Y; long ldy; float* Hprev; float* Cprev;
  float* out; long ldo; int hcol, ccol;       // encoder final state (last_hidden)
  int off, bs, next_off, next_bs, tiles;
};
struct FwdArgs { FwdDir d[2]; int H; int nd; };

template <int G>
__global__ __launch_bounds__(256) void rnn_fwd_step(FwdArgs a) {
  constexpr int TN = 16 * G, LD = TN + 4, TSZ = 16 * LD;
  __shared__ __attribute__((aligned(16))) float lds[2 * 4 * TSZ];
  int blk = blockIdx.x;
  int sel = 0;
  if (a.nd == 2 && blk >= a.d[0].tiles) { blk -= a.d[0].tiles; sel = 1; }
  const FwdDir& D = a.d[sel];
  const int H = a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int nut = H / 16;
  const int ut = blk % nut, rt = blk / nut;
  // epilogue operands of this thread's (row, unit), fetched before the GEMM so
  // their HBM latency overlaps the K loop
  const int row = threadIdx.x >> 4, u = threadIdx.x & 15;
  const int b = rt * 16 + row;
  const bool live = b < D.bs;
  const int unit = ut * 16 + u;
  const long rr = D.off + (live ? b : 0);
  const bool haspred = live && b < D.prev_valid;
  float gxp[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    gxp[j] = 0.f;
    if (live && D.GX) gxp[j] = D.GX[rr * D.ldgx + j * H + unit];
    if (live && D.bih) gxp[j] += D.bih[j * H + unit];
  }
  const float cprev = (G == 4 && haspred) ? D.Cprev[rr * H + unit] : 0.f;
  const float hprev = (G == 3 && haspred) ? D.Hprev[rr * H + unit] : 0.f;
  f4 accH[1][G], accX[1][G];
  acc_zero(accH);
  acc_zero(accX);
  const int ar[1] = {rt * 16 + r};
  int br[G];
#pragma unroll
  for (int j = 0; j < G; ++j) br[j] = j * H + ut * 16 + r;
  const int nchh = H / 16;
  wave_mma<1, G>(accH, KC{D.Ah, H, D.prev_valid}, ar, KC{D.Whh, H, G * H}, br, w, nchh, 4, q);
  if (D.xrows > 0)
    wave_mma<1, G>(accX, KC{D.Ax, D.ldx, D.xrows}, ar, KC{D.Wih, D.ldwih, G * H}, br, first_chunk(w, nchh),
                   D.nchx, 4, q);
  {
    reduce_waves_to_lds<1, G>(accH, lds, w, lane);
    reduce_waves_to_lds<1, G>(accX, lds + 4 * TSZ, w, lane);
  }
  const float* tH = lds;
  const float* tX = lds + 4 * TSZ;
  if (!live) return;
  float gx[G], gh[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    gh[j] = tH[row * LD + j * 16 + u];
    gx[j] = tX[row * LD + j * 16 + u] + gxp[j];
  }
  float* Gr = D.Gst + rr * 4 * H;
  float h, c = 0.f;
  if (G == 4) {
    const float i_ = sigmoidf_(gx[0] + gh[0]);
    const float f_ = sigmoidf_(gx[1] + gh[1]);
    const float g_ = tanhf(gx[2] + gh[2]);
    const float o_ = sigmoidf_(gx[3] + gh[3]);
    c = f_ * cprev + i_ * g_;
    h = o_ * tanhf(c);
    Gr[unit] = i_; Gr[H + unit] = f_; Gr[2 * H + unit] = g_; Gr[3 * H + unit] = o_;
    D.Cst[rr * H + unit] = c;
    if (!haspred) { D.Cprev[rr * H + unit] = 0.f; D.Hprev[rr * H + unit] = 0.f; }
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j) gh[j] += D.bhh[j * H + unit];
    const float r_ = sigmoidf_(gx[0] + gh[0]);
    const float z_ = sigmoidf_(gx[1] + gh[1]);
    const float n_ = tanhf(gx[2] + r_ * gh[G - 1]);
    h = (1.f - z_) * n_ + z_ * hprev;
    Gr[unit] = r_; Gr[H + unit] = z_; Gr[2 * H + unit] = n_; Gr[3 * H + unit] = gh[G - 1];
    if (!haspred) D.Hprev[rr * H + unit] = 0.f;
  }
  if (D.Y) D.Y[rr * D.ldy + unit] = h;  // (null: the top encoder layer, whose output sequence nothing reads)
  if (b < D.next_bs) {
    D.Hprev[(long)(D.next_off + b) * H + unit] = h;
    if (G == 4) D.Cprev[(long)(D.next_off + b) * H + unit] = c;
  } else if (D.out) {
    D.out[(long)b * D.ldo + D.hcol + unit] = h;
    if (G == 4) D.out[(long)b * D.ldo + D.ccol + unit] = c;
  }
}

// ===========================================================================
// backward step: dh = dG_succ @ W_hh (+ dZ @ W1cat for the decoder) + extra,
// then the cell backward in the epilogue -> dG (for the next GEMM and for
// the weight gradients), carry (dc for LSTM, dh*z for GRU) to the predecessor
// ===========================================================================
struct BwdDir {
  const float* Ag; int succ_valid;            // dGH + succ_off*G*H
  const float* WhhT;                          // H x G*H
  const float* Az; int zrows; const float* W1T; long ldz; int nchz;  // decoder: dZ rows, W1cat^T (H x 2Hm)
  const float* DHX; long lddhx;               // extra dh rows (upper layer / offset head)
  const float* dlast; long ldl; int hcol, ccol;  // final-state grads (encoder)
  const float* Gst; const float* Cst; const float* Cprev; const float* Hprev;
  float* dGX; float* dGH;                     // row-major, ld G*H (LSTM: same buffer)
  float* DC;                                  // carry rows read at this step
  float* DCpred; int pred_off;                // carry destination for the predecessor
  int off, bs, prev_valid, next_bs, tiles;
};
struct BwdArgs { BwdDir d[2]; int H; int nd; };

template <int G, int NR>
__global__ __launch_bounds__(256) void rnn_bwd_step(BwdArgs a) {
  constexpr int TN = 16 * NR, LD = TN + 4;
  __shared__ __attribute__((aligned(16))) float lds[4 * 16 * LD];
  int blk = blockIdx.x;
  int sel = 0;
  if (a.nd == 2 && blk >= a.d[0].tiles) { blk -= a.d[0].tiles; sel = 1; }
  const BwdDir& D = a.d[sel];
  const int H = a.H, GH = G * H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int nut = H / TN;
  const int ut = blk % nut, rt = blk / nut;
  // epilogue operands (NR elements per thread), fetched before the GEMM
  constexpr int EPT = (16 * TN) / 256;  // elements per thread
  float pg[EPT][4], pc[EPT], pcp[EPT], pdc[EPT], pdh[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int row = e / TN, cu = e % TN;
    const int b = rt * 16 + row;
    const bool live = b < D.bs;
    const int unit = ut * TN + cu;
    const long rr = D.off + (live ? b : 0);
    const bool fin = b >= D.next_bs;
    const bool haspred = live && b < D.prev_valid;
    const float* Gr = D.Gst + rr * 4 * H;
#pragma unroll
    for (int j = 0; j < 4; ++j) pg[k][j] = live ? Gr[j * H + unit] : 0.f;
    pc[k] = (live && G == 4) ? D.Cst[rr * H + unit] : 0.f;
    pcp[k] = 0.f;
    if (haspred) pcp[k] = G == 4 ? D.Cprev[rr * H + unit] : D.Hprev[rr * H + unit];
    float dh = 0.f, dc = 0.f;
    if (live) {
      if (D.DHX) dh += D.DHX[rr * D.lddhx + unit];
      if (fin) {
        if (D.dlast) {
          dh += D.dlast[(long)b * D.ldl + D.hcol + unit];
          if (G == 4 && D.ccol >= 0) dc = D.dlast[(long)b * D.ldl + D.ccol + unit];
        }
      } else {
        if (G == 4) dc = D.DC[rr * H + unit];
        else dh += D.DC[rr * H + unit];
      }
    }
    pdh[k] = dh;
    pdc[k] = dc;
  }
  f4 acc[1][NR];
  acc_zero(acc);
  const int ar[1] = {rt * 16 + r};
  int br[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) br[j] = ut * TN + 16 * j + r;
  const int nchg = GH / 16;
  if (D.succ_valid > 0)
    wave_mma<1, NR>(acc, KC{D.Ag, GH, D.succ_valid}, ar, KC{D.WhhT, GH, H}, br, w, nchg, 4, q);
  if (D.zrows > 0)
    wave_mma<1, NR>(acc, KC{D.Az, D.ldz, D.zrows}, ar, KC{D.W1T, D.ldz, H}, br, first_chunk(w, nchg), D.nchz, 4,
                    q);
  reduce_waves_to_lds<1, NR>(acc, lds, w, lane);
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int row = e / TN, cu = e % TN;
    const int b = rt * 16 + row;
    if (b >= D.bs) continue;
    const int unit = ut * TN + cu;
    const long rr = D.off + b;
    const bool haspred = b < D.prev_valid;
    const float dh = lds[row * LD + cu] + pdh[k];
    if (G == 4) {
      const float i_ = pg[k][0], f_ = pg[k][1], g_ = pg[k][2], o_ = pg[k][3];
      const float tc = tanhf(pc[k]);
      const float dc = pdc[k] + dh * o_ * (1.f - tc * tc);
      float* dg = D.dGX + rr * GH;
      dg[unit] = dc * g_ * i_ * (1.f - i_);
      dg[H + unit] = dc * pcp[k] * f_ * (1.f - f_);
      dg[2 * H + unit] = dc * i_ * (1.f - g_ * g_);
      dg[3 * H + unit] = dh * tc * o_ * (1.f - o_);
      if (haspred) D.DCpred[(long)(D.pred_off + b) * H + unit] = dc * f_;
    } else {
      const float r_ = pg[k][0], z_ = pg[k][1], n_ = pg[k][2], ghn = pg[k][3];
      const float hp = pcp[k];
      const float dnp = dh * (1.f - z_) * (1.f - n_ * n_);
      const float dzp = dh * (hp - n_) * z_ * (1.f - z_);
      const float drp = dnp * ghn * r_ * (1.f - r_);
      float* dx = D.dGX + rr * GH;
      float* dhh = D.dGH + rr * GH;
      dx[unit] = drp; dx[H + unit] = dzp; dx[2 * H + unit] = dnp;
      dhh[unit] = drp; dhh[H + unit] = dzp; dhh[2 * H + unit] = dnp * r_;
      if (haspred) D.DCpred[(long)(D.pred_off + b) * H + unit] = dh * z_;
    }
  }
}

template <int G>
static int launch_bwd_step(hipStream_t s, const BwdArgs& a, int grid, int H) {
  if ((H / 16) % 4 == 0)
    rnn_bwd_step<G, 4><<<grid, 256, 0, s>>>(a);
  else if ((H / 16) % 2 == 0)
    rnn_bwd_step<G, 2><<<grid, 256, 0, s>>>(a);
  else
    rnn_bwd_step<G, 1><<<grid, 256, 0, s>>>(a);
  ABCD_CHECK_LAUNCH();
  return 0;
}
static int bwd_tn(int H) { return (H / 16) % 4 == 0 ? 64 : ((H / 16) % 2 == 0 ? 32 : 16); }

// ===========================================================================
// ENCODER
// ===========================================================================
// Bias gradients folded into the input weight-gradient GEMM (layer 0 with a
// padded input, Fp > F): column F of the padded frame copy Xp is 1 (written by
// the forward's pack; W_ih's packed pad columns are 0, so the input projection
// is unchanged), so the GEMM dG^T [X | 1] of width F + 1 yields
// dW_ih and, in its last column, sum_r dG[r] = the bias gradient -- one
// colsum pass over the L x G*H gate gradients fewer per direction.
__global__ __launch_bounds__(256) void set_col_kernel(float* X, long ld, long rows, int col, float v) {
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < rows; r += (long)gridDim.x * 256) X[r * ld + col] = v;
}
__global__ __launch_bounds__(256) void split_wb_kernel(const float* dWx, int rows, int F, float* w, float* b1,
                                                       float* b2) {
  const long n = (long)rows * (F + 1);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / (F + 1)), j = (int)(i % (F + 1));
    const float v = dWx[i];
    if (j < F) w[(long)r * F + j] = v;
    else {
      b1[r] = v;
      if (b2) b2[r] = v;
    }
  }
}

struct EncWS {
  float* Xp;
  float* Wihp[ABCD_MAX_LAYERS];
  float* bcat[ABCD_MAX_LAYERS];
  float* WhhT[ABCD_MAX_LAYERS][2];
  float* WihT[ABCD_MAX_LAYERS][2];
  float* GX;
  float* Y[ABCD_MAX_LAYERS];
  float* Gst[ABCD_MAX_LAYERS][2];
  float* Cst[ABCD_MAX_LAYERS][2];
  float* Hprev[ABCD_MAX_LAYERS][2];
  float* Cprev[ABCD_MAX_LAYERS][2];
  float* dGX[ABCD_MAX_LAYERS][2];
  float* dGH[ABCD_MAX_LAYERS][2];
  float* DC[ABCD_MAX_LAYERS][2];
  float* DHX[ABCD_MAX_LAYERS];
  float* Ydrop[ABCD_MAX_LAYERS];  // layer output x dropout noise (input of layer l + 1)
  float* dWb;                     // layer 0: [dW_ih | db] (bias column folded into the GEMM)
  int* off;          // device copy of the step offsets (persistent kernels)
  unsigned* sync;    // persistent-kernel group counters
  float* skp;        // dec_bwd_sk split-K partials
  float* part;       // split-K partials of the persistent backward
  float* scratch;
  size_t scratch_floats;
};

static int enc_check(const abcd_encoder_cfg* c) {
  if (!c || c->hidden_size <= 0 || c->hidden_size % 16 || c->layers < 1 || c->layers > ABCD_MAX_LAYERS ||
      c->input_size <= 0 || (c->rnn_type != ABCD_LSTM && c->rnn_type != ABCD_GRU))
    return ABCD_EINVAL;
  return 0;
}

static EncWS carve_encoder(Arena& A, const abcd_encoder_cfg* c, int T, int L, int B) {
  EncWS w{};
  const int H = c->hidden_size, D = c->bidirectional ? 2 : 1, G = c->rnn_type == ABCD_LSTM ? 4 : 3;
  const int F = c->input_size, Fp = rup16(F);
  w.Xp = A.f((size_t)L * Fp);
  size_t maxMN = 0;
  for (int l = 0; l < c->layers; ++l) {
    const int In = l == 0 ? F : D * H, Inp = l == 0 ? Fp : D * H;
    w.Wihp[l] = A.f((size_t)D * G * H * Inp);
    w.bcat[l] = A.f((size_t)D * G * H);
    for (int d = 0; d < D; ++d) {
      w.WhhT[l][d] = A.f((size_t)H * G * H);
      w.WihT[l][d] = l > 0 ? A.f((size_t)In * G * H) : nullptr;
      w.Gst[l][d] = A.f((size_t)L * 4 * H);
      w.Cst[l][d] = c->rnn_type == ABCD_LSTM ? A.f((size_t)L * H) : nullptr;
      w.Hprev[l][d] = A.f((size_t)L * H);
      w.Cprev[l][d] = c->rnn_type == ABCD_LSTM ? A.f((size_t)L * H) : nullptr;
      w.dGX[l][d] = A.f((size_t)L * G * H);
      w.dGH[l][d] = c->rnn_type == ABCD_LSTM ? w.dGX[l][d] : A.f((size_t)L * G * H);
      w.DC[l][d] = A.f((size_t)L * H);
    }
    w.Y[l] = l + 1 < c->layers ? A.f((size_t)L * D * H) : nullptr;  // the top layer's sequence is never read
    w.DHX[l] = l + 1 < c->layers ? A.f((size_t)L * D * H) : nullptr;
    w.Ydrop[l] = l + 1 < c->layers ? A.f((size_t)L * D * H) : nullptr;
    maxMN = std::max(maxMN, (size_t)G * H * std::max(In, H));
  }
  w.GX = A.f((size_t)L * D * G * H);
  w.dWb = A.f((size_t)D * G * H * (F + 1));  // one per direction (their reductions may run concurrently)
  w.off = (int*)A.f((size_t)T + 1);
  w.sync = (unsigned*)A.f(persist_sync_uints(D, B));
  w.part = A.f(persist_part_floats(D, B, H));
  w.scratch_floats = std::max(maxMN * 64, (size_t)1 << 20);  // split-K slabs of the wgrad GEMMs
  w.scratch = A.f(w.scratch_floats);
  return w;
}

}  // namespace abcd

using namespace abcd;

extern "C" int abcd_encoder_out_size(const abcd_encoder_cfg* c) {
  if (enc_check(c)) return -1;
  int e = c->layers * c->hidden_size * (c->bidirectional ? 2 : 1);
  return c->rnn_type == ABCD_LSTM ? 2 * e : e;
}

extern "C" size_t abcd_encoder_workspace_bytes(const abcd_encoder_cfg* c, int T, int L, int B) {
  if (enc_check(c)) return 0;
  Arena A(nullptr, 0);
  carve_encoder(A, c, T, L, B);
  return A.off + 256;
}

extern "C" int abcd_encoder_forward(const abcd_encoder_cfg* c, const abcd_encoder_params* p, const abcd_packed* x,
                                    float* last_hidden, void* ws, size_t ws_bytes, void* stream) {
  return abcd_encoder_forward_dropout(c, p, x, nullptr, last_hidden, ws, ws_bytes, stream);
}

extern "C" int abcd_encoder_forward_dropout(const abcd_encoder_cfg* c, const abcd_encoder_params* p,
                                            const abcd_packed* x, const float* const* noise, float* last_hidden,
                                            void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(enc_check(c) == 0 && p && x && x->data && last_hidden && ws);
  ABCD_REQUIRE(x->F == c->input_size);
  ABCD_REQUIRE(validate_batch(x->batch_sizes, x->T, x->L, x->B) == 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  EncWS w = carve_encoder(A, c, x->T, x->L, x->B);
  ABCD_REQUIRE(A.ok);
  const int H = c->hidden_size, D = c->bidirectional ? 2 : 1, G = c->rnn_type == ABCD_LSTM ? 4 : 3;
  const int F = c->input_size, Fp = rup16(F), T = x->T, L = x->L;
  const int E = abcd_encoder_out_size(c);
  const std::vector<int> off = step_offsets(x->batch_sizes, T);
  const int64_t* bs = x->batch_sizes;
  Packs pk(s);
  // [X | 1 | 0]: the ones column (F < Fp) feeds the backward's bias-gradient
  // column and meets W_ih's zero padding in the input projection
  ABCD_TRY((hipError_t)pk.add(x->data, F, L, F, false, w.Xp, Fp, L, Fp, nullptr, F < Fp));
  for (int l = 0; l < c->layers; ++l) {
    const int In = l == 0 ? F : D * H, Inp = l == 0 ? Fp : D * H;
    for (int d = 0; d < D; ++d) {
      const abcd_rnn_w& W = p->w[l][d];
      ABCD_REQUIRE(W.w_ih && W.w_hh && W.b_ih && W.b_hh);
      ABCD_TRY((hipError_t)pk.add(W.w_ih, In, G * H, In, false, w.Wihp[l] + (size_t)d * G * H * Inp, Inp, G * H,
                                  Inp));
      ABCD_TRY((hipError_t)pk.add(W.b_ih, G * H, 1, G * H, false, w.bcat[l] + d * G * H, G * H, 1, G * H,
                                  G == 4 ? W.b_hh : nullptr));
      // W_hh^T for the backward pass (read from this workspace by abcd_encoder_backward*),
      // packed here in the same launch instead of in front of the BPTT
      ABCD_TRY((hipError_t)pk.add(W.w_hh, H, H, G * H, true, w.WhhT[l][d], G * H, H, G * H));
    }
    ABCD_TRY((hipError_t)pk.flush());
    const float* X = l == 0 ? w.Xp : w.Y[l - 1];
    if (l > 0 && noise && noise[l - 1]) {  // nn.LSTM(dropout=p): the layer below's packed output x noise
      ABCD_TRY((hipError_t)mul_vec(s, w.Y[l - 1], noise[l - 1], w.Ydrop[l - 1], (long)L * D * H));
      X = w.Ydrop[l - 1];
    }
    bool done = false;
    {
      PFwdArgs pa{};
      pa.H = H; pa.nd = D; pa.T = T; pa.nrt = cdiv(x->B, PERSIST_ROWS); pa.off = w.off; pa.sync = w.sync;
      for (int d = 0; d < D; ++d) {
        const abcd_rnn_w& W = p->w[l][d];
        PFwdDir& f = pa.d[d];
        f.Whh = W.w_hh;
        f.GX = w.GX + (size_t)d * G * H; f.ldgx = (long)D * G * H;
        f.bhh = G == 3 ? W.b_hh : nullptr;
        f.Gst = w.Gst[l][d]; f.Cst = w.Cst[l][d];
        f.Y = l + 1 < c->layers ? w.Y[l] + (size_t)d * H : nullptr; f.ldy = (long)D * H;
        f.Hprev = w.Hprev[l][d]; f.Cprev = w.Cprev[l][d];
        f.out = last_hidden; f.ldo = E;
        const int base = (l * D + d) * (G == 4 ? 2 * H : H);
        f.hcol = base; f.ccol = G == 4 ? base + H : -1;
        f.rev = d == 1;
      }
      if (l == 0 && persist_enabled()) ABCD_TRY((hipError_t)stage_offsets(s, off, w.off));
      // the L x D*G*H input projection GEMM feeds the recurrence (fusing it into
      // the persistent kernel measured +0.68 ms on the launch for the 0.6 ms saved)
      ABCD_TRY((hipError_t)gemm(s, L, D * G * H, Inp, opKC(X, Inp, L), opKC(w.Wihp[l], Inp, D * G * H), w.GX,
                                (long)D * G * H, 1.f, 0.f, w.bcat[l], ACT_NONE, w.scratch, w.scratch_floats));
      ABCD_TRY((hipError_t)persist_encoder_fwd(s, G, pa, &done));
      ABCD_TRY((hipError_t)flush_offsets());
    }
    if (!done) note_dispatch(TK_ENC_FWD, "per-step rnn_fwd_step<%d>", G);
    for (int i = 0; i < T && !done; ++i) {
      FwdArgs a{};
      a.H = H;
      a.nd = D;
      for (int d = 0; d < D; ++d) {
        const bool rev = d == 1;
        const int t = rev ? T - 1 - i : i;
        FwdDir& f = a.d[d];
        const abcd_rnn_w& W = p->w[l][d];
        const int prev_valid = rev ? (t == T - 1 ? 0 : (int)bs[t + 1]) : (t == 0 ? 0 : (int)bs[t]);
        f.Ah = w.Hprev[l][d] + (size_t)off[t] * H;
        f.prev_valid = prev_valid;
        f.Whh = W.w_hh;
        f.Ax = nullptr; f.ldx = 0; f.xrows = 0; f.Wih = nullptr; f.ldwih = 0; f.nchx = 0;
        f.GX = w.GX + (size_t)d * G * H;
        f.ldgx = (long)D * G * H;
        f.bih = nullptr;
        f.bhh = G == 3 ? W.b_hh : nullptr;
        f.Gst = w.Gst[l][d]; f.Cst = w.Cst[l][d];
        f.Y = l + 1 < c->layers ? w.Y[l] + (size_t)d * H : nullptr; f.ldy = (long)D * H;
        f.Hprev = w.Hprev[l][d]; f.Cprev = w.Cprev[l][d];
        f.out = last_hidden; f.ldo = E;
        const int base = (l * D + d) * (G == 4 ? 2 * H : H);
        f.hcol = base; f.ccol = G == 4 ? base + H : -1;
        f.off = off[t]; f.bs = (int)bs[t];
        if (rev) { f.next_off = t >= 1 ? off[t - 1] : 0; f.next_bs = t >= 1 ? (int)bs[t] : 0; }
        else { f.next_off = off[t + 1]; f.next_bs = t + 1 < T ? (int)bs[t + 1] : 0; }
        f.tiles = cdiv(f.bs, 16) * (H / 16);
      }
      const int grid = a.d[0].tiles + (D == 2 ? a.d[1].tiles : 0);
      {
        TimedScope ts(s);
        if (G == 4) rnn_fwd_step<4><<<grid, 256, 0, s>>>(a);
        else rnn_fwd_step<3><<<grid, 256, 0, s>>>(a);
      }
      ABCD_CHECK_LAUNCH();
    }
  }
  return 0;
}

static int fork_event(hipEvent_t* ev, int slot);

extern "C" int abcd_encoder_backward(const abcd_encoder_cfg* c, const abcd_encoder_params* p, const abcd_packed* x,
                                     const float* d_last_hidden, const abcd_encoder_grads* g, void* ws,
                                     size_t ws_bytes, void* stream) {
  return abcd_encoder_backward_dropout(c, p, x, nullptr, d_last_hidden, g, ws, ws_bytes, stream, nullptr);
}

extern "C" int abcd_encoder_backward_overlap(const abcd_encoder_cfg* c, const abcd_encoder_params* p,
                                             const abcd_packed* x, const float* d_last_hidden,
                                             const abcd_encoder_grads* g, void* ws, size_t ws_bytes, void* stream,
                                             void* wgrad_stream) {
  return abcd_encoder_backward_dropout(c, p, x, nullptr, d_last_hidden, g, ws, ws_bytes, stream, wgrad_stream);
}

extern "C" int abcd_encoder_backward_dropout(const abcd_encoder_cfg* c, const abcd_encoder_params* p,
                                             const abcd_packed* x, const float* const* noise,
                                             const float* d_last_hidden, const abcd_encoder_grads* g, void* ws,
                                             size_t ws_bytes, void* stream, void* wgrad_stream) {
  ABCD_REQUIRE(enc_check(c) == 0 && p && x && x->data && g && ws && d_last_hidden);
  ABCD_REQUIRE(validate_batch(x->batch_sizes, x->T, x->L, x->B) == 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  EncWS w = carve_encoder(A, c, x->T, x->L, x->B);
  ABCD_REQUIRE(A.ok);
  const int H = c->hidden_size, D = c->bidirectional ? 2 : 1, G = c->rnn_type == ABCD_LSTM ? 4 : 3;
  const int F = c->input_size, Fp = rup16(F), T = x->T, L = x->L, GH = G * H;
  const int E = abcd_encoder_out_size(c);
  const std::vector<int> off = step_offsets(x->batch_sizes, T);
  const int64_t* bs = x->batch_sizes;
  const int TN = bwd_tn(H);
  // wgrad_stream: the last layer's backward-direction weight gradients run
  // there after the BPTT, beside the forward direction's on s (a side-stream
  // gate that started them DURING the BPTT measured no gain)
  for (int l = c->layers - 1; l >= 0; --l) {
    const int In = l == 0 ? F : D * H;
    // w.WhhT[l][d] = W_hh^T: packed by the forward pass into this workspace
    bool done = false;
    {
      PBwdArgs pa{};
      pa.H = H; pa.nd = D; pa.T = T; pa.nrt = cdiv(x->B, PERSIST_ROWS); pa.off = w.off; pa.sync = w.sync;
      pa.B = x->B;
      pa.part = w.part;
      for (int d = 0; d < D; ++d) {
        PBwdDir& b = pa.d[d];
        b.WhhT = w.WhhT[l][d];
        b.DHX = l + 1 < c->layers ? w.DHX[l] + (size_t)d * H : nullptr;
        b.lddhx = (long)D * H;
        b.dlast = d_last_hidden; b.ldl = E;
        const int base = (l * D + d) * (G == 4 ? 2 * H : H);
        b.hcol = base; b.ccol = G == 4 ? base + H : -1;
        b.Gst = w.Gst[l][d]; b.Cst = w.Cst[l][d]; b.Cprev = w.Cprev[l][d]; b.Hprev = w.Hprev[l][d];
        b.dGX = w.dGX[l][d]; b.dGH = w.dGH[l][d];
        b.rev = d == 1;
      }
      if (l == c->layers - 1 && persist_enabled()) ABCD_TRY((hipError_t)stage_offsets(s, off, w.off));
      ABCD_TRY((hipError_t)persist_encoder_bwd(s, G, pa, &done));
      ABCD_TRY((hipError_t)flush_offsets());
    }
    if (!done) note_dispatch(TK_ENC_BWD, "per-step launch_bwd_step<%d>", G);
    for (int i = 0; i < T && !done; ++i) {
      BwdArgs a{};
      a.H = H;
      a.nd = D;
      for (int d = 0; d < D; ++d) {
        const bool rev = d == 1;
        const int t = rev ? i : T - 1 - i;
        BwdDir& b = a.d[d];
        int succ_off, succ_valid, prev_valid, pred_off;
        if (!rev) {
          succ_off = off[t + 1]; succ_valid = t + 1 < T ? (int)bs[t + 1] : 0;
          prev_valid = t == 0 ? 0 : (int)bs[t]; pred_off = t >= 1 ? off[t - 1] : 0;
        } else {
          succ_off = t >= 1 ? off[t - 1] : 0; succ_valid = t >= 1 ? (int)bs[t] : 0;
          prev_valid = t == T - 1 ? 0 : (int)bs[t + 1]; pred_off = off[t + 1];
        }
        b.Ag = w.dGH[l][d] + (size_t)succ_off * GH;
        b.succ_valid = succ_valid;
        b.WhhT = w.WhhT[l][d];
        b.Az = nullptr; b.zrows = 0; b.W1T = nullptr; b.ldz = 0; b.nchz = 0;
        b.DHX = l + 1 < c->layers ? w.DHX[l] + (size_t)d * H : nullptr;
        b.lddhx = (long)D * H;
        b.dlast = d_last_hidden; b.ldl = E;
        const int base = (l * D + d) * (G == 4 ? 2 * H : H);
        b.hcol = base; b.ccol = G == 4 ? base + H : -1;
        b.Gst = w.Gst[l][d]; b.Cst = w.Cst[l][d]; b.Cprev = w.Cprev[l][d]; b.Hprev = w.Hprev[l][d];
        b.dGX = w.dGX[l][d]; b.dGH = w.dGH[l][d];
        b.DC = w.DC[l][d]; b.DCpred = w.DC[l][d]; b.pred_off = pred_off;
        b.off = off[t]; b.bs = (int)bs[t]; b.prev_valid = prev_valid; b.next_bs = succ_valid;
        b.tiles = cdiv(b.bs, 16) * (H / TN);
      }
      const int grid = a.d[0].tiles + (D == 2 ? a.d[1].tiles : 0);
      TimedScope ts(s);
      if (G == 4) ABCD_TRY((hipError_t)launch_bwd_step<4>(s, a, grid, H));
      else ABCD_TRY((hipError_t)launch_bwd_step<3>(s, a, grid, H));
    }
    // weight gradients: reductions over all L packed frames (K = L, K-major
    // operands), over the row range [r0, r1) into the gradient with weight beta
    const bool ones_col = l == 0 && F < Fp && true;
    auto wgrad = [&](hipStream_t st, int d, int r0, int r1, float beta, float* scratch, size_t scf) -> int {
      const abcd_rnn_g& gr = g->g[l][d];
      const float* X = l == 0 ? w.Xp : ((noise && noise[l - 1]) ? w.Ydrop[l - 1] : w.Y[l - 1]);  // Xp: padded copy
      const long ldxx = l == 0 ? rup16(F) : (long)D * H;
      const int K = r1 - r0;
      const float* dGX = w.dGX[l][d] + (size_t)r0 * GH;
      const float* dGH = w.dGH[l][d] + (size_t)r0 * GH;
      if (ones_col && r0 == 0 && r1 == L && beta == 0.f && gr.w_ih && gr.b_ih) {
        // [dW_ih | db] in one GEMM
        float* dWb = w.dWb + (size_t)d * GH * (In + 1);
        ABCD_TRY((hipError_t)gemm(st, GH, In + 1, K, opKM(dGX, GH, GH), opKM(X, ldxx, In + 1), dWb, In + 1, 1.f,
                                  0.f, nullptr, ACT_NONE, scratch, scf));
        const bool same = dGX == dGH;  // LSTM: b_hh receives the same sum
        split_wb_kernel<<<(int)std::min<long>(1024, cdiv((long)GH * (In + 1), 256)), 256, 0, st>>>(
            dWb, GH, In, gr.w_ih, gr.b_ih, same ? gr.b_hh : nullptr);
        ABCD_CHECK_LAUNCH();
        if (gr.w_hh)
          ABCD_TRY((hipError_t)gemm(st, GH, H, K, opKM(dGH, GH, GH), opKM(w.Hprev[l][d], H, H), gr.w_hh, H, 1.f,
                                    0.f, nullptr, ACT_NONE, scratch, scf));
        if (!same && gr.b_hh) ABCD_TRY((hipError_t)colsum(st, dGH, GH, K, GH, nullptr, gr.b_hh, 0.f, scratch, scf));
        return 0;
      }
      if (gr.w_ih)
        ABCD_TRY((hipError_t)gemm(st, GH, In, K, opKM(dGX, GH, GH), opKM(X + (size_t)r0 * ldxx, ldxx, In), gr.w_ih,
                                  In, 1.f, beta, nullptr, ACT_NONE, scratch, scf));
      if (gr.w_hh)
        ABCD_TRY((hipError_t)gemm(st, GH, H, K, opKM(dGH, GH, GH), opKM(w.Hprev[l][d] + (size_t)r0 * H, H, H),
                                  gr.w_hh, H, 1.f, beta, nullptr, ACT_NONE, scratch, scf));
      // LSTM: b_ih and b_hh receive the same sum over dG (one pass, two outputs)
      if (dGX == dGH && gr.b_ih) {
        ABCD_TRY((hipError_t)colsum(st, dGX, GH, K, GH, nullptr, gr.b_ih, beta, scratch, scf, gr.b_hh));
        return 0;
      }
      if (gr.b_ih) ABCD_TRY((hipError_t)colsum(st, dGX, GH, K, GH, nullptr, gr.b_ih, beta, scratch, scf));
      if (gr.b_hh) ABCD_TRY((hipError_t)colsum(st, dGH, GH, K, GH, nullptr, gr.b_hh, beta, scratch, scf));
      return 0;
    };
    // (the ones column of Xp was written by the forward's pack)
    int wg2 = -1;  // 0: gemm_wg2 produced every gradient of this layer
    if (ones_col && G == 4) {
      WgDir dirs[2] = {};
      bool all = true;
      for (int d = 0; d < D; ++d) {
        const abcd_rnn_g& gr = g->g[l][d];
        all = all && gr.w_ih && gr.b_ih && gr.w_hh;
        dirs[d] = WgDir{w.dGX[l][d], w.Xp, w.Hprev[l][d], gr.w_ih, gr.b_ih, gr.b_hh, gr.w_hh};
      }
      if (all) {
        wg2 = wgrad_lstm_l0(s, D, dirs, GH, L, F, Fp, H, w.scratch, w.scratch_floats);
        if (wg2 > 0) return wg2;
      }
    }
    if (l == 0) note_dispatch(TK_ENC_WGRAD, wg2 == 0 ? wg_dispatch_fmt()
                                                   : "gemm split (x6s/x6t)", Fp, H, D);
    if (wg2 == 0) {
    } else if (D == 2 && l == 0 && wgrad_stream && wgrad_stream != stream) {
      // the last layer's two directions reduce concurrently: the backward
      // direction on wgrad_stream (forked after the BPTT), the forward one on
      // s, each with half of the split-K scratch; s then waits for
      // wgrad_stream, so every gradient is complete in `stream` order
      hipStream_t sw = (hipStream_t)wgrad_stream;
      const size_t half = w.scratch_floats / 2;
      ABCD_TRY((hipError_t)stream_fork(s, sw, 6));
      ABCD_TRY((hipError_t)wgrad(sw, 1, 0, L, 0.f, w.scratch + half, half));
      ABCD_TRY((hipError_t)wgrad(s, 0, 0, L, 0.f, w.scratch, half));
      ABCD_TRY((hipError_t)stream_fork(sw, s, 7));
    } else {
      for (int d = 0; d < D; ++d) ABCD_TRY((hipError_t)wgrad(s, d, 0, L, 0.f, w.scratch, w.scratch_floats));
    }
    if (l > 0) {  // dX of this layer = dh of the layer below (both directions)
      for (int d = 0; d < D; ++d) {
        ABCD_TRY((hipError_t)pack2d(s, p->w[l][d].w_ih, In, In, GH, true, w.WihT[l][d], GH, In, GH));
        ABCD_TRY((hipError_t)gemm(s, L, In, GH, opKC(w.dGX[l][d], GH, L), opKC(w.WihT[l][d], GH, In), w.DHX[l - 1],
                                  In, 1.f, d == 0 ? 0.f : 1.f, nullptr, ACT_NONE, w.scratch, w.scratch_floats));
      }
      if (noise && noise[l - 1])  // through the dropout: d(y * noise)/dy = noise
        ABCD_TRY((hipError_t)mul_vec(s, w.DHX[l - 1], noise[l - 1], w.DHX[l - 1], (long)L * In));
    }
  }
  return 0;
}

// ===========================================================================
// DECODER (model.py:147-196): per step t
//   D1 rnn_fwd_step    gates = Xin_rows @ W_ih^T + Hprev_rows @ W_hh^T (+b), cell
//   D2 gemm (tanh)     Aact = tanh(h @ [W1_mu; W1_lv]^T + b1)        (bs x 2Hm)
//   D3 dec_emit_fwd    [mu | lv] = Aact_{mu|lv} @ W2^T + b2, x = mu + e^{lv/2} eps
//                      -> Xin rows of step t+1 (self-feedback)
// backward per step (t = T-1 .. 0)
//   E1 dec_emit_bwd_x  dx_{t+1} = dGX_{t+1} @ W_ih ; dmu, dlv (+ emission NLL grad)
//   E2 dec_mlp_bwd     dZ = ([dmu|dlv] @ W2) * (1 - Aact^2)
//   E3 rnn_bwd_step    dh = dZ @ W1cat + dG_{t+1} @ W_hh + dh_offset ; cell bwd
// ===========================================================================
namespace abcd {

struct EmitFwd {
  const float* Aact; long lda; int Hm, nch;
  const float *W2m, *W2l, *b2m, *b2l;  // padded Fp x Hm, Fp
  const float* eps; uint64_t seed, offset;
  const float* xmask;  // input dropout of step t+1's cell input (rows x F) or null
  float *MU, *LV, *OUT, *Xin; int F, Fp;
  int off, bs, next_off, next_bs, feedback;
};

__global__ __launch_bounds__(256) void dec_emit_fwd(EmitFwd a) {
  constexpr int LD = 20;
  __shared__ __attribute__((aligned(16))) float lds[2 * 4 * 16 * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int nct = a.Fp / 16;
  const int ct = blockIdx.x % nct, rt = blockIdx.x / nct;
  f4 am[1][1], al[1][1];
  acc_zero(am);
  acc_zero(al);
  const int ar[1] = {rt * 16 + r};
  const int br[1] = {ct * 16 + r};
  const float* Arows = a.Aact + (long)a.off * a.lda;
  wave_mma<1, 1>(am, KC{Arows, a.lda, a.bs}, ar, KC{a.W2m, a.Hm, a.Fp}, br, w, a.nch, 4, q);
  wave_mma<1, 1>(al, KC{Arows + a.Hm, a.lda, a.bs}, ar, KC{a.W2l, a.Hm, a.Fp}, br, w, a.nch, 4, q);
  reduce_waves_to_lds<1, 1>(am, lds, w, lane);
  reduce_waves_to_lds<1, 1>(al, lds + 4 * 16 * LD, w, lane);
  const int row = threadIdx.x >> 4, cc = threadIdx.x & 15;
  const int b = rt * 16 + row;
  if (b >= a.bs) return;
  const int j = ct * 16 + cc;
  const long rr = a.off + b;
  float mu = 0.f, lv = 0.f, x = 0.f;
  if (j < a.F) {
    mu = lds[row * LD + cc] + a.b2m[j];
    lv = lds[4 * 16 * LD + row * LD + cc] + a.b2l[j];
    const float e = a.eps ? a.eps[rr * a.F + j] : philox_normal(a.seed, a.offset + (uint64_t)rr * a.F + j);
    x = mu + __expf(0.5f * lv) * e;
  }
  a.MU[rr * a.Fp + j] = mu;
  a.LV[rr * a.Fp + j] = lv;
  a.OUT[rr * a.Fp + j] = x;
  if (a.feedback && b < a.next_bs) {
    const long nr = a.next_off + b;
    a.Xin[nr * a.Fp + j] = (a.xmask && j < a.F) ? x * a.xmask[nr * a.F + j] : x;
  }
}

struct EmitBwdX {
  const float* Ag; long ldg; int succ_valid; int nch;  // dGX rows of step t+1
  const float* WihT;                                  // Fp x G*H
  const float *MU, *LV, *OUT, *Y;                     // stash (ld Fp), gt (ld F)
  const float* s_em;                                  // device scalar
  const float* xmask; int succ_off;                   // input dropout of step t+1's rows (or null)
  float *dMU, *dLV; int F, Fp; int off, bs;
};

__global__ __launch_bounds__(256) void dec_emit_bwd_x(EmitBwdX a) {
  constexpr int LD = 20;
  __shared__ __attribute__((aligned(16))) float lds[4 * 16 * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int nct = a.Fp / 16;
  const int ct = blockIdx.x % nct, rt = blockIdx.x / nct;
  f4 acc[1][1];
  acc_zero(acc);
  const int ar[1] = {rt * 16 + r};
  const int br[1] = {ct * 16 + r};
  if (a.succ_valid > 0) wave_mma<1, 1>(acc, KC{a.Ag, a.ldg, a.succ_valid}, ar, KC{a.WihT, a.ldg, a.Fp}, br, w, a.nch, 4, q);
  reduce_waves_to_lds<1, 1>(acc, lds, w, lane);
  const int row = threadIdx.x >> 4, cc = threadIdx.x & 15;
  const int b = rt * 16 + row;
  if (b >= a.bs) return;
  const int j = ct * 16 + cc;
  const long rr = a.off + b;
  float dmu = 0.f, dlv = 0.f;
  if (j < a.F) {
    float dx = lds[row * LD + cc];
    if (a.xmask && b < a.succ_valid) dx *= a.xmask[(long)(a.succ_off + b) * a.F + j];
    const float mu = a.MU[rr * a.Fp + j], lv = a.LV[rr * a.Fp + j], o = a.OUT[rr * a.Fp + j];
    const float y = a.Y[rr * a.F + j];
    const float s = *a.s_em;
    const float iv = __expf(-lv), d = y - mu;
    dmu = dx + s * (-d) * iv;
    dlv = dx * 0.5f * (o - mu) + s * 0.5f * (1.f - d * d * iv);
  }
  a.dMU[rr * a.Fp + j] = dmu;
  a.dLV[rr * a.Fp + j] = dlv;
}

struct MlpBwd {
  const float *dMU, *dLV; int Fp, nch;   // rows (ld Fp)
  const float *W2mT, *W2lT;              // Hm x Fp
  const float* Aact; float* dZ; int Hm;  // ld 2Hm
  int off, bs;
};

template <int NR>
__global__ __launch_bounds__(256) void dec_mlp_bwd(MlpBwd a) {
  constexpr int TN = 16 * NR, LD = TN + 4;
  __shared__ __attribute__((aligned(16))) float lds[2 * 4 * 16 * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, q = lane >> 4;
  const int nct = a.Hm / TN;
  const int ct = blockIdx.x % nct, rt = blockIdx.x / nct;
  f4 am[1][NR], al[1][NR];
  acc_zero(am);
  acc_zero(al);
  const int ar[1] = {rt * 16 + r};
  int br[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) br[j] = ct * TN + 16 * j + r;
  const long o = (long)a.off * a.Fp;
  wave_mma<1, NR>(am, KC{a.dMU + o, a.Fp, a.bs}, ar, KC{a.W2mT, a.Fp, a.Hm}, br, w, a.nch, 4, q);
  wave_mma<1, NR>(al, KC{a.dLV + o, a.Fp, a.bs}, ar, KC{a.W2lT, a.Fp, a.Hm}, br, w, a.nch, 4, q);
  reduce_waves_to_lds<1, NR>(am, lds, w, lane);
  reduce_waves_to_lds<1, NR>(al, lds + 4 * 16 * LD, w, lane);
  const int H2 = 2 * a.Hm;
  for (int e = threadIdx.x; e < 16 * TN; e += 256) {
    const int row = e / TN, cc = e % TN;
    const int b = rt * 16 + row;
    if (b >= a.bs) continue;
    const int j = ct * TN + cc;
    const long rr = a.off + b;
    const float xm = a.Aact[rr * H2 + j], xl = a.Aact[rr * H2 + a.Hm + j];
    a.dZ[rr * H2 + j] = lds[row * LD + cc] * (1.f - xm * xm);
    a.dZ[rr * H2 + a.Hm + j] = lds[4 * 16 * LD + row * LD + cc] * (1.f - xl * xl);
  }
}

// ---- small decoder helpers ------------------------------------------------
// FS = [features | embed_speaker[speaker]]
__global__ void dec_feats(const float* feats, int D, const float* emb, const int64_t* spk, int S, int B, float* FS) {
  const int DS = D + S;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < B * DS; i += gridDim.x * 256) {
    const int b = i / DS, c = i % DS;
    FS[i] = c < D ? feats[(long)b * D + c] : emb[spk[b] * S + (c - D)];
  }
}
// rows [0,B) of Hprev/Cprev from feature2hidden (LSTM: interleaved h/c, model.py:100,262-263); Xin rows [0,B) = 0
__global__ void dec_init(const float* Hinit, int B, int H, int lstm, float* Hprev, float* Cprev, float* Xin, int Fp) {
  const int n = B * H;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / H, u = i % H;
    if (lstm) {
      Hprev[i] = Hinit[(long)b * 2 * H + 2 * u];
      Cprev[i] = Hinit[(long)b * 2 * H + 2 * u + 1];
    } else {
      Hprev[i] = Hinit[(long)b * H + u];
    }
  }
  for (int i = blockIdx.x * 256 + threadIdx.x; i < B * Fp; i += gridDim.x * 256) Xin[i] = 0.f;
}
// feature2hidden (model.py:100,262-263) computed straight into the initial
// state: dec_init's scatter with the B x Htot product formed in place (fp32
// FMAs, k ascending, + bias), one launch instead of a split-K GEMM + dec_init
// on the sampler -> decoder chain.  A workgroup owns a 32 x 32 output tile:
// its FS rows (32 x DS) and WT columns (WT = f2h_w^T, DS x Htot, the
// backward's packed transpose) are loaded with every 16-B load in flight at
// once (NV per thread and operand, DS <= 32 NV), staged in LDS, and each
// thread forms a 2 x 2 block over all of K.  (One column per thread straight
// from HBM / L2 ran 121 us at c2: a chain of dependent load latencies.)
template <int NV>
__global__ __launch_bounds__(256) void dec_init_f2h(const float* FS, int DS, const float* WT, const float* bias,
                                                    int B, int H, int lstm, float* Hprev, float* Cprev, float* Xin,
                                                    int Fp) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int P = DS + 4;  // FS row pitch: 16-B rows, consecutive rows 4 banks apart
  float* fs = sm;        // 32 x P
  float* wt = sm + 32 * P;  // DS x 32
  const int tid = threadIdx.x, Htot = lstm ? 2 * H : H, q = DS / 4;
  const int j0 = blockIdx.x * 32, b0 = blockIdx.y * 32;
  f4 a[NV], w[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = tid + 256 * v, r = e / q, c = e % q;
    a[v] = e < 32 * q && b0 + r < B ? *reinterpret_cast<const f4*>(FS + (long)(b0 + r) * DS + 4 * c) : f4zero();
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = tid + 256 * v, k = e >> 3, c = e & 7;
    w[v] = k < DS && j0 + 4 * c < Htot ? *reinterpret_cast<const f4*>(WT + (long)k * Htot + j0 + 4 * c) : f4zero();
  }
  if (blockIdx.x == 0)  // Xin rows [b0, b0 + 32) = 0
    for (int i = tid; i < 32 * Fp; i += 256)
      if (b0 + i / Fp < B) Xin[(long)b0 * Fp + i] = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = tid + 256 * v;
    if (e < 32 * q) *reinterpret_cast<f4*>(fs + (e / q) * P + 4 * (e % q)) = a[v];
    if ((e >> 3) < DS) *reinterpret_cast<f4*>(wt + (e >> 3) * 32 + 4 * (e & 7)) = w[v];
  }
  __syncthreads();
  const int r0 = (tid >> 4) * 2, c0 = (tid & 15) * 2;
  float acc00 = 0.f, acc01 = 0.f, acc10 = 0.f, acc11 = 0.f;
#pragma unroll 8
  for (int k = 0; k < DS; ++k) {
    const float x0 = fs[r0 * P + k], x1 = fs[(r0 + 1) * P + k];
    const float2 y = *reinterpret_cast<const float2*>(wt + k * 32 + c0);
    acc00 = fmaf(x0, y.x, acc00);
    acc01 = fmaf(x0, y.y, acc01);
    acc10 = fmaf(x1, y.x, acc10);
    acc11 = fmaf(x1, y.y, acc11);
  }
  const float acc[2][2] = {{acc00, acc01}, {acc10, acc11}};
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int j = j0 + c0 + jj;
    if (j >= Htot) continue;
    const float bj = bias ? bias[j] : 0.f;
    const int u = lstm ? j >> 1 : j;
    float* dst = lstm && (j & 1) ? Cprev : Hprev;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (b0 + r0 + i < B) dst[(long)(b0 + r0 + i) * H + u] = acc[i][jj] + bj;
  }
}
static int dec_init_f2h_launch(hipStream_t s, const float* FS, int DS, const float* WT, const float* bias, int B,
                               int H, int lstm, float* Hprev, float* Cprev, float* Xin, int Fp) {
  const int Htot = lstm ? 2 * H : H;
  if (DS % 4 || Htot % 4 || DS > 512 || (((uintptr_t)FS | (uintptr_t)WT) & 15)) return -1;
  const size_t lds = ((size_t)32 * (DS + 4) + (size_t)DS * 32) * 4;
  const dim3 grid(cdiv(Htot, 32), cdiv(B, 32));
#define ABCD_DEC_INIT(NV)                                                                                 \
  {                                                                                                       \
    static bool attr = false;                                                                             \
    if (!attr) {                                                                                          \
      ABCD_TRY(hipFuncSetAttribute((const void*)dec_init_f2h<NV>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                   160 * 1024));                                                          \
      attr = true;                                                                                        \
    }                                                                                                     \
    dec_init_f2h<NV><<<grid, 256, lds, s>>>(FS, DS, WT, bias, B, H, lstm, Hprev, Cprev, Xin, Fp);         \
  }
  if (DS <= 128) ABCD_DEC_INIT(4)
  else if (DS <= 256) ABCD_DEC_INIT(8)
  else ABCD_DEC_INIT(16)
#undef ABCD_DEC_INIT
  return (int)hipGetLastError();
}
// offset head (model.py:121-122,191,195): logit = Zo . w2 + b2 ; BCE-with-logits (sum)
__global__ void dec_offset_head(const float* Zo, int L, int Hm, const float* w2, const float* b2, const float* tgt,
                                float* logit, float* dlog_raw, float* bce) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= L) return;
  float s = 0.f;
#pragma unroll 4
  for (int j = lane; j < Hm; j += 64) s += Zo[(long)row * Hm + j] * w2[j];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if (lane == 0) {
    const float x = s + b2[0];
    logit[row] = x;
    if (tgt) {
      const float y = tgt[row];
      bce[row] = fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
      dlog_raw[row] = 1.f / (1.f + __expf(-x)) - y;
    }
  }
}
// the same from the fused forward GEMM's per-slice partial dot products
// (gemm_offset_fwd), summed in slice order
__global__ void dec_offset_logit(const float* part, int nsl, int L, const float* b2, const float* tgt, float* logit,
                                 float* dlog_raw, float* bce) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= L) return;
  float s = 0.f;
  for (int k = 0; k < nsl; ++k) s += part[(long)row * nsl + k];
  const float x = s + b2[0];
  logit[row] = x;
  if (tgt) {
    const float y = tgt[row];
    bce[row] = fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
    dlog_raw[row] = 1.f / (1.f + __expf(-x)) - y;
  }
}
// emission NLL partial sums: 0.5*(log 2pi + lv + (y-mu)^2 e^{-lv}) over L x F
constexpr int NLL_ROWS = 16;
__global__ __launch_bounds__(256) void dec_emission_nll(const float* MU, const float* LV, int Fp, const float* Y,
                                                        int F, long L, double* part) {
  // a workgroup owns NLL_ROWS consecutive rows (one wave per NLL_ROWS / 4 of
  // them: coalesced row reads, every load of a wave in flight together) and
  // writes one fp64 partial.  Short workgroups: the pass runs on the loss
  // stream beside the offset head's backward GEMM, and the decoder BPTT
  // launched behind that GEMM needs one workgroup slot per CU -- it finds them
  // within one short workgroup's time (1024 grid-striding 16-wave workgroups
  // held them to the pass's end: dec_bwd start skew 1.4 us median at c2, 17 us
  // at c5)
  __shared__ double sh[4];
  double acc = 0.0;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r0 = (long)blockIdx.x * NLL_ROWS + w * (NLL_ROWS / 4);
#pragma unroll
  for (int i = 0; i < NLL_ROWS / 4; ++i) {
    const long r = r0 + i;
    if (r < L)
#pragma unroll 3
      for (int j = lane; j < F; j += 64) {
        const float mu = MU[r * Fp + j], lv = LV[r * Fp + j], d = Y[r * F + j] - mu;
        acc += 0.5f * (1.8378770664093453f + lv + d * d * __expf(-lv));
      }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) sh[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
}
__global__ void sum_partials(const double* part, int np, float* out) {
  __shared__ double sh[4];
  double v = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) v += part[i];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
    *out = (float)t;
  }
}
// offset-head backward: dlog = s_off * (sigmoid(x) - y); dZo = dlog * w2 * (1 - Zo^2)
__global__ void dec_offset_bwd(const float* Zo, int L, int Hm, const float* w2, const float* dlog_raw,
                               const float* s_off, float* dZo, float* dlog_s) {
  const float s = *s_off;
  // one wave per row (grid-stride over rows), as dec_offset_head
  const int lane = threadIdx.x & 63, nwv = gridDim.x * (blockDim.x >> 6);
  for (long r = blockIdx.x * (long)(blockDim.x >> 6) + (threadIdx.x >> 6); r < L; r += nwv) {
    const float dl = s * dlog_raw[r];
#pragma unroll 4
    for (int j = lane; j < Hm; j += 64) {
      const float z = Zo[r * Hm + j];
      dZo[r * Hm + j] = dl * w2[j] * (1.f - z * z);
    }
    if (lane == 0) dlog_s[r] = dl;
  }
}
// gradient of feature2hidden output from the t=0 carries
__global__ void dec_hidden_init_bwd(const float* dH0, const float* DC0, int B, int H, int lstm, float* dhid) {
  const int n = B * H;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / H, u = i % H;
    if (lstm) {
      dhid[(long)b * 2 * H + 2 * u] = dH0[i];
      dhid[(long)b * 2 * H + 2 * u + 1] = DC0[i];
    } else {
      dhid[i] = dH0[i] + DC0[i];
    }
  }
}
// d_features = dFS[:, :D]; embedding grad rows (deterministic: one thread per (speaker, col))
__global__ void dec_feats_bwd(const float* dFS, int D, int S, int B, const int64_t* spk, int nspk, float* dfeat,
                              float* demb) {
  const int DS = D + S;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < B * D; i += gridDim.x * 256) {
    const int b = i / D, c = i % D;
    if (dfeat) dfeat[i] = dFS[(long)b * DS + c];
  }
  if (!demb) return;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nspk * S; i += gridDim.x * 256) {
    const int sp = i / S, c = i % S;
    float acc = 0.f;
    for (int b = 0; b < B; ++b)
      if (spk[b] == sp) acc += dFS[(long)b * DS + D + c];
    demb[i] = acc;
  }
}
// copy a padded (rows x Fp) stash into a user (rows x F) buffer
__global__ void unpad_rows(const float* src, int Fp, float* dst, int F, long rows) {
  const long n = rows * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = src[(i / F) * Fp + (i % F)];
}

struct DecWS {
  // derived weights
  float *Wihp, *bcomb, *bgru, *W1cat, *b1cat, *W2mp, *W2lp, *b2mp, *b2lp;
  float *WihTp, *WhhT, *W2mT, *W2lT, *W1catT, *W1oT, *Wf2hT;
  // forward stash
  float *FS, *Hinit, *Xin, *Hprev, *Cprev, *Gst, *Cst, *Hs, *Aact, *MU, *LV, *OUT, *Zo, *offlog, *dlog_raw, *bce;
  float* offpart;  // the fused offset head's partial logits (L x offset_head_slices(Hm))
  float* EPS;  // the Philox decoder noise, rows x F (philox_normal_fill)
  float* dWb;  // [dW_ih | db] of the cell (bias column folded into the GEMM)
  double* part;
  // backward
  float *dGX, *dGH, *DC, *DC0, *dH0, *dhid, *dFS, *DHO, *dMU, *dLV, *dZ, *dZo, *dlog_s;
  int* off;          // device step offsets (persistent kernels)
  unsigned* sync;    // persistent-kernel group counters
  float* skp;        // dec_bwd_sk split-K partials
  float* scratch;
  size_t scratch_floats;
};

static int dec_check(const abcd_decoder_cfg* c) {
  if (!c || c->hidden_size <= 0 || c->hidden_size % 16 || c->mlp_hidden <= 0 || c->mlp_hidden % 16 ||
      c->feature_size <= 0 || c->feature_size % 16 || c->output_size <= 0 ||
      (c->rnn_type != ABCD_LSTM && c->rnn_type != ABCD_GRU))
    return ABCD_EINVAL;
  if (c->num_speakers > 0 && (c->speaker_dim <= 0 || c->speaker_dim % 16)) return ABCD_EINVAL;
  return 0;
}

static DecWS carve_decoder(Arena& A, const abcd_decoder_cfg* c, int T, int L, int B) {
  DecWS w{};
  const int H = c->hidden_size, Hm = c->mlp_hidden, F = c->output_size, Fp = rup16(F);
  const int G = c->rnn_type == ABCD_LSTM ? 4 : 3, GH = G * H;
  const int Htot = c->rnn_type == ABCD_LSTM ? 2 * H : H;
  const int DS = c->feature_size + (c->num_speakers > 0 ? c->speaker_dim : 0);
  w.Wihp = A.f((size_t)GH * Fp); w.bcomb = A.f(GH); w.bgru = A.f((size_t)4 * H);
  w.W1cat = A.f((size_t)2 * Hm * H); w.b1cat = A.f(2 * Hm);
  w.W2mp = A.f((size_t)Fp * Hm); w.W2lp = A.f((size_t)Fp * Hm); w.b2mp = A.f(Fp); w.b2lp = A.f(Fp);
  w.WihTp = A.f((size_t)Fp * GH); w.WhhT = A.f((size_t)H * GH);
  w.W2mT = A.f((size_t)Hm * Fp); w.W2lT = A.f((size_t)Hm * Fp);
  w.W1catT = A.f((size_t)H * 2 * Hm); w.W1oT = A.f((size_t)H * Hm); w.Wf2hT = A.f((size_t)DS * Htot);
  w.FS = A.f((size_t)B * DS); w.Hinit = A.f((size_t)B * Htot);
  w.Xin = A.f((size_t)L * Fp); w.Hprev = A.f((size_t)L * H);
  w.Cprev = G == 4 ? A.f((size_t)L * H) : nullptr;
  w.Gst = A.f((size_t)L * 4 * H);
  w.Cst = G == 4 ? A.f((size_t)L * H) : nullptr;
  w.Hs = A.f((size_t)L * H); w.Aact = A.f((size_t)L * 2 * Hm);
  w.MU = A.f((size_t)L * Fp); w.LV = A.f((size_t)L * Fp); w.OUT = A.f((size_t)L * Fp);
  w.EPS = A.f((size_t)L * F);
  w.Zo = A.f((size_t)L * Hm); w.offlog = A.f(L); w.dlog_raw = A.f(L); w.bce = A.f(L);
  w.offpart = A.f((size_t)L * offset_head_slices(Hm));
  w.part = A.d(1024 + (size_t)std::max(1, cdiv(L, NLL_ROWS)));  // [0, 1024): bce reduction; then the NLL partials
  w.dGX = A.f((size_t)L * GH);
  w.dGH = G == 4 ? w.dGX : A.f((size_t)L * GH);
  w.DC = A.f((size_t)L * H); w.DC0 = A.f((size_t)B * H); w.dH0 = A.f((size_t)B * H);
  w.dhid = A.f((size_t)B * Htot); w.dFS = A.f((size_t)B * DS); w.DHO = A.f((size_t)L * H);
  w.dMU = A.f((size_t)L * Fp); w.dLV = A.f((size_t)L * Fp); w.dZ = A.f((size_t)L * 2 * Hm);
  w.dZo = A.f((size_t)L * Hm); w.dlog_s = A.f(L);
  w.dWb = A.f((size_t)GH * (F + 1));
  size_t maxMN = std::max<size_t>({(size_t)GH * std::max(Fp, H), (size_t)Fp * Hm, (size_t)Hm * H,
                                   (size_t)Htot * DS, (size_t)L});
  w.off = (int*)A.f((size_t)T + 1);
  w.sync = (unsigned*)A.f(persist_sync_uints(1, B));
  w.skp = A.f(dec_part_floats(B, H, Fp));
  w.scratch_floats = std::max(maxMN * 64, (size_t)1 << 20);  // split-K slabs of the wgrad GEMMs
  w.scratch = A.f(w.scratch_floats);
  return w;
}

static int launch_grid(long n) { return (int)std::max<long>(1, std::min<long>(4096, cdiv(n, 256))); }
// ABCD_DEC_INIT_F2H=0: feature2hidden as a GEMM + dec_init (same-box A/B)
static bool dec_init_fused() {
  const char* v = getenv("ABCD_DEC_INIT_F2H");
  return !(v && v[0] == '0');
}
static bool dec_eps_fill() {
  const char* v = getenv("ABCD_DEC_EPSFILL");
  return !(v && v[0] == '0');
}

}  // namespace abcd

static size_t lstm_wgrad_floats(int nd, int F, int H, int K, size_t* xp_floats) {
  const size_t xp = (((size_t)K * rup16(F + 1)) + 63) & ~(size_t)63;
  if (xp_floats) *xp_floats = xp;
  const size_t M = 4 * (size_t)H;
  return xp + std::max((size_t)16 * nd * M * (rup16(F + 1) + H), M * std::max(F, H) * 64);
}

extern "C" size_t abcd_lstm_wgrad_workspace_bytes(int nd, int F, int H, int K) {
  if (nd < 1 || nd > 2 || F <= 0 || H <= 0 || K < 0) return 0;
  return lstm_wgrad_floats(nd, F, H, K, nullptr) * 4 + 256;
}

// C ABI: the LSTM layer's weight gradients (gemm_wg2 when the shape has an
// instance, else the split GEMM route the encoder backward falls back to)
extern "C" int abcd_lstm_wgrad(int nd, int F, int H, int K, const float* const* dG, const float* X, long ldx,
                               const float* const* Hprev, float* const* w_ih, float* const* b_ih,
                               float* const* b_hh, float* const* w_hh, void* ws, size_t ws_bytes, void* stream) {
  ABCD_REQUIRE(nd >= 1 && nd <= 2 && F > 0 && H > 0 && H % 4 == 0 && K >= 0 && dG && X && ldx >= F && Hprev && w_ih &&
               b_ih && w_hh && ws);
  size_t xpf = 0;
  const size_t need = lstm_wgrad_floats(nd, F, H, K, &xpf);
  ABCD_REQUIRE(ws_bytes / 4 >= need && ((uintptr_t)ws % 16) == 0);
  for (int d = 0; d < nd; ++d) ABCD_REQUIRE(dG[d] && Hprev[d] && w_ih[d] && b_ih[d] && w_hh[d]);
  if (K == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int M = 4 * H, Fp = rup16(F + 1);
  float* Xp = (float*)ws;
  float* scratch = Xp + xpf;
  const size_t scf = need - xpf;
  // [X | 1 | 0] with the gemm_wg2 row pitch
  ABCD_TRY((hipError_t)pack2d(s, X, ldx, K, F, false, Xp, Fp, K, Fp));
  set_col_kernel<<<std::max(1, std::min(1024, cdiv(K, 256))), 256, 0, s>>>(Xp, Fp, K, F, 1.f);
  ABCD_CHECK_LAUNCH();
  WgDir dirs[2] = {};
  for (int d = 0; d < nd; ++d) dirs[d] = WgDir{dG[d], Xp, Hprev[d], w_ih[d], b_ih[d], b_hh ? b_hh[d] : nullptr, w_hh[d]};
  const int r = wgrad_lstm_l0(s, nd, dirs, M, K, F, Fp, H, scratch, scf);
  if (r == 0) {
    note_dispatch(TK_ENC_WGRAD, wg_dispatch_fmt(), Fp, H, nd);
    return 0;
  }
  if (r > 0) return r;
  note_dispatch(TK_ENC_WGRAD, "gemm split (x6s/x6t)");
  for (int d = 0; d < nd; ++d) {
    ABCD_TRY((hipError_t)gemm(s, M, F, K, opKM(dG[d], M, M), opKM(Xp, Fp, F), w_ih[d], F, 1.f, 0.f, nullptr, ACT_NONE,
                              scratch, scf));
    ABCD_TRY((hipError_t)gemm(s, M, H, K, opKM(dG[d], M, M), opKM(Hprev[d], H, H), w_hh[d], H, 1.f, 0.f, nullptr,
                              ACT_NONE, scratch, scf));
    ABCD_TRY((hipError_t)colsum(s, dG[d], M, K, M, nullptr, b_ih[d], 0.f, scratch, scf, b_hh ? b_hh[d] : nullptr));
  }
  return 0;
}

extern "C" size_t abcd_decoder_workspace_bytes(const abcd_decoder_cfg* c, int T, int L, int B) {
  if (dec_check(c)) return 0;
  Arena A(nullptr, 0);
  carve_decoder(A, c, T, L, B);
  return A.off + 256;
}

extern "C" int abcd_decoder_forward(const abcd_decoder_cfg* c, const abcd_decoder_params* p, const abcd_packed* x,
                                    const float* features, const int64_t* speakers, const float* gt_offset,
                                    const float* eps, uint64_t seed, uint64_t offset, float* flatten_out,
                                    float* mu_out, float* lv_out, float* offset_logits, float* losses, void* ws,
                                    size_t ws_bytes, void* stream) {
  return abcd_decoder_forward_dropout(c, p, x, features, speakers, gt_offset, eps, nullptr, seed, offset,
                                      flatten_out, mu_out, lv_out, offset_logits, losses, ws, ws_bytes, stream);
}

static int dec_forward_impl(const abcd_decoder_cfg* c, const abcd_decoder_params* p, const abcd_packed* x,
                            const float* features, const int64_t* speakers, const float* gt_offset, const float* eps,
                            const float* xmask, uint64_t seed, uint64_t offset, float* flatten_out, float* mu_out,
                            float* lv_out, float* offset_logits, float* losses, void* ws, size_t ws_bytes,
                            void* stream, hipStream_t sl);

extern "C" int abcd_decoder_forward_dropout(const abcd_decoder_cfg* c, const abcd_decoder_params* p,
                                            const abcd_packed* x, const float* features, const int64_t* speakers,
                                            const float* gt_offset, const float* eps, const float* xmask,
                                            uint64_t seed, uint64_t offset, float* flatten_out, float* mu_out,
                                            float* lv_out, float* offset_logits, float* losses, void* ws,
                                            size_t ws_bytes, void* stream) {
  return dec_forward_impl(c, p, x, features, speakers, gt_offset, eps, xmask, seed, offset, flatten_out, mu_out,
                          lv_out, offset_logits, losses, ws, ws_bytes, stream, (hipStream_t)stream);
}

extern "C" int abcd_decoder_forward_split(const abcd_decoder_cfg* c, const abcd_decoder_params* p,
                                          const abcd_packed* x, const float* features, const int64_t* speakers,
                                          const float* gt_offset, const float* eps, const float* xmask,
                                          uint64_t seed, uint64_t offset, float* flatten_out, float* mu_out,
                                          float* lv_out, float* offset_logits, float* losses, void* ws,
                                          size_t ws_bytes, void* stream, void* loss_stream) {
  return dec_forward_impl(c, p, x, features, speakers, gt_offset, eps, xmask, seed, offset, flatten_out, mu_out,
                          lv_out, offset_logits, losses, ws, ws_bytes, stream,
                          loss_stream ? (hipStream_t)loss_stream : (hipStream_t)stream);
}

static int dec_forward_impl(const abcd_decoder_cfg* c, const abcd_decoder_params* p, const abcd_packed* x,
                            const float* features, const int64_t* speakers, const float* gt_offset, const float* eps,
                            const float* xmask, uint64_t seed, uint64_t offset, float* flatten_out, float* mu_out,
                            float* lv_out, float* offset_logits, float* losses, void* ws, size_t ws_bytes,
                            void* stream, hipStream_t sl) {
  ABCD_REQUIRE(dec_check(c) == 0 && p && x && features && ws);
  ABCD_REQUIRE(!xmask || c->feedback);
  ABCD_REQUIRE(validate_batch(x->batch_sizes, x->T, x->L, x->B) == 0);
  ABCD_REQUIRE(c->num_speakers == 0 || (speakers && p->embed_speaker));
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  DecWS w = carve_decoder(A, c, x->T, x->L, x->B);
  ABCD_REQUIRE(A.ok);
  const int H = c->hidden_size, Hm = c->mlp_hidden, F = c->output_size, Fp = rup16(F);
  const int G = c->rnn_type == ABCD_LSTM ? 4 : 3, GH = G * H;
  const int Htot = G == 4 ? 2 * H : H;
  const int D = c->feature_size, S = c->num_speakers > 0 ? c->speaker_dim : 0, DS = D + S;
  const int T = x->T, L = x->L, B = x->B;
  const int64_t* bs = x->batch_sizes;
  const std::vector<int> off = step_offsets(bs, T);
  const abcd_rnn_w& cw = p->cell;
  // ---- derived (compute-layout) weights ----
  {
    Packs pk(s);
    ABCD_TRY((hipError_t)pk.add(cw.w_ih, F, GH, F, false, w.Wihp, Fp, GH, Fp));
    if (G == 4) ABCD_TRY((hipError_t)pk.add(cw.b_ih, GH, 1, GH, false, w.bcomb, GH, 1, GH, cw.b_hh));
    else {
      ABCD_TRY((hipError_t)pk.add(cw.b_ih, GH, 1, GH, false, w.bcomb, GH, 1, GH));
      // persistent GRU cell bias [b_r | b_z | b_in | b_hn] (r, z: b_ih + b_hh)
      ABCD_TRY((hipError_t)pk.add(cw.b_ih, 2 * H, 1, 2 * H, false, w.bgru, 2 * H, 1, 2 * H, cw.b_hh));
      ABCD_TRY((hipError_t)pk.add(cw.b_ih + 2 * H, H, 1, H, false, w.bgru + 2 * H, H, 1, H));
      ABCD_TRY((hipError_t)pk.add(cw.b_hh + 2 * H, H, 1, H, false, w.bgru + 3 * H, H, 1, H));
    }
    ABCD_TRY((hipError_t)pk.add(p->mu.w1, H, Hm, H, false, w.W1cat, H, Hm, H));
    ABCD_TRY((hipError_t)pk.add(p->lv.w1, H, Hm, H, false, w.W1cat + (size_t)Hm * H, H, Hm, H));
    ABCD_TRY((hipError_t)pk.add(p->mu.b1, Hm, 1, Hm, false, w.b1cat, Hm, 1, Hm));
    ABCD_TRY((hipError_t)pk.add(p->lv.b1, Hm, 1, Hm, false, w.b1cat + Hm, Hm, 1, Hm));
    ABCD_TRY((hipError_t)pk.add(p->mu.w2, Hm, F, Hm, false, w.W2mp, Hm, Fp, Hm));
    ABCD_TRY((hipError_t)pk.add(p->lv.w2, Hm, F, Hm, false, w.W2lp, Hm, Fp, Hm));
    ABCD_TRY((hipError_t)pk.add(p->mu.b2, F, 1, F, false, w.b2mp, Fp, 1, Fp));
    ABCD_TRY((hipError_t)pk.add(p->lv.b2, F, 1, F, false, w.b2lp, Fp, 1, Fp));
    // the backward's transposed weights, in the same launch (off the
    // decoder-forward -> decoder-backward chain)
    ABCD_TRY((hipError_t)pk.add(cw.w_ih, F, F, GH, true, w.WihTp, GH, Fp, GH));  // rows >= F zero
    ABCD_TRY((hipError_t)pk.add(cw.w_hh, H, H, GH, true, w.WhhT, GH, H, GH));
    ABCD_TRY((hipError_t)pk.add(p->mu.w2, Hm, Hm, F, true, w.W2mT, Fp, Hm, Fp));
    ABCD_TRY((hipError_t)pk.add(p->lv.w2, Hm, Hm, F, true, w.W2lT, Fp, Hm, Fp));
    ABCD_TRY((hipError_t)pk.add(p->mu.w1, H, H, Hm, true, w.W1catT, 2 * Hm, H, Hm));
    ABCD_TRY((hipError_t)pk.add(p->lv.w1, H, H, Hm, true, w.W1catT + Hm, 2 * Hm, H, Hm));
    ABCD_TRY((hipError_t)pk.add(p->offset.w1, H, H, Hm, true, w.W1oT, Hm, H, Hm));
    ABCD_TRY((hipError_t)pk.add(p->f2h_w, DS, DS, Htot, true, w.Wf2hT, Htot, DS, Htot));
    ABCD_TRY((hipError_t)pk.flush());
  }
  // ---- feature2hidden -> initial state ----
  const float* FS = features;
  if (S > 0) {
    dec_feats<<<launch_grid((long)B * DS), 256, 0, s>>>(features, D, p->embed_speaker, speakers, S, B, w.FS);
    ABCD_CHECK_LAUNCH();
    FS = w.FS;
  }
  int rc = -1;
  if (dec_init_fused())
    rc = dec_init_f2h_launch(s, FS, DS, w.Wf2hT, p->f2h_b, B, H, G == 4, w.Hprev, w.Cprev, w.Xin, Fp);
  if (rc > 0) return rc;
  if (rc < 0) {
    ABCD_TRY((hipError_t)gemm(s, B, Htot, DS, opKC(FS, DS, B), opKC(p->f2h_w, DS, Htot), w.Hinit, Htot, 1.f, 0.f,
                              p->f2h_b, ACT_NONE, nullptr, 0));
    dec_init<<<launch_grid((long)B * std::max(H, Fp)), 256, 0, s>>>(w.Hinit, B, H, G == 4, w.Hprev, w.Cprev, w.Xin,
                                                                   Fp);
  }
  ABCD_CHECK_LAUNCH();
  // ---- time loop: one persistent launch, or one launch per phase and step ----
  bool done = false;
  {
    PDecFwdArgs pa{};
    pa.H = H; pa.Hm = Hm; pa.F = F; pa.Fp = Fp; pa.T = T; pa.nrt = cdiv(B, PERSIST_ROWS);
    pa.feedback = c->feedback;
    pa.off = w.off; pa.sync = w.sync;
    pa.Wih = w.Wihp; pa.Whh = cw.w_hh; pa.bias = G == 4 ? w.bcomb : w.bgru;
    pa.W1 = w.W1cat; pa.b1 = w.b1cat;
    pa.W2m = w.W2mp; pa.W2l = w.W2lp; pa.b2m = w.b2mp; pa.b2l = w.b2lp;
    pa.eps = eps; pa.seed = seed; pa.offset = offset; pa.xmask = xmask;
    // Philox noise in a workspace block (the same philox_normal(seed, offset +
    // row * F + col) the kernel would draw), read with one load per element
    // instead of ~1 us of VALU per step on the emit phase's path (dec_fwd 2.31
    // -> 2.17 ms at c2); drawn by the persistent launch's idle members (or up
    // front for the forms without them: PDecFwdArgs::eps_fill).
    // ABCD_DEC_EPSFILL=0: drawn by the emit waves themselves.
    if (!eps && persist_enabled() && dec_eps_fill()) {
      pa.eps = w.EPS;
      pa.eps_fill = 1;
      pa.nfill = (long)L * F;
    }
    pa.Xin = w.Xin; pa.Hprev = w.Hprev; pa.Cprev = w.Cprev; pa.Gst = w.Gst; pa.Cst = w.Cst; pa.Hs = w.Hs;
    pa.Aact = w.Aact; pa.MU = w.MU; pa.LV = w.LV; pa.OUT = w.OUT;
    if (persist_enabled()) ABCD_TRY((hipError_t)stage_offsets(s, off, w.off));
    ABCD_TRY((hipError_t)persist_decoder_fwd(s, G, pa, &done));
    ABCD_TRY((hipError_t)flush_offsets());
  }
  if (!done) note_dispatch(TK_DEC_FWD, "per-step decoder forward<%d>", G);
  for (int t = 0; t < T && !done; ++t) {
    const int b_t = (int)bs[t];
    const int nb = t + 1 < T ? (int)bs[t + 1] : 0;
    FwdArgs a{};
    a.H = H;
    a.nd = 1;
    FwdDir& f = a.d[0];
    f.Ah = w.Hprev + (size_t)off[t] * H; f.prev_valid = b_t; f.Whh = cw.w_hh;
    f.Ax = w.Xin + (size_t)off[t] * Fp; f.ldx = Fp; f.xrows = (c->feedback && t > 0) ? b_t : 0;
    f.Wih = w.Wihp; f.ldwih = Fp; f.nchx = Fp / 16;
    f.GX = nullptr; f.ldgx = 0; f.bih = w.bcomb; f.bhh = G == 3 ? cw.b_hh : nullptr;
    f.Gst = w.Gst; f.Cst = w.Cst; f.Y = w.Hs; f.ldy = H; f.Hprev = w.Hprev; f.Cprev = w.Cprev;
    f.out = nullptr; f.ldo = 0; f.hcol = 0; f.ccol = 0;
    f.off = off[t]; f.bs = b_t; f.next_off = off[t + 1]; f.next_bs = nb;
    f.tiles = cdiv(b_t, 16) * (H / 16);
    {
      TimedScope ts(s);
      if (G == 4) rnn_fwd_step<4><<<f.tiles, 256, 0, s>>>(a);
      else rnn_fwd_step<3><<<f.tiles, 256, 0, s>>>(a);
    }
    ABCD_CHECK_LAUNCH();
    ABCD_TRY((hipError_t)gemm(s, b_t, 2 * Hm, H, opKC(w.Hs + (size_t)off[t] * H, H, b_t), opKC(w.W1cat, H, 2 * Hm),
                              w.Aact + (size_t)off[t] * 2 * Hm, 2 * Hm, 1.f, 0.f, w.b1cat, ACT_TANH, nullptr, 0));
    EmitFwd e{};
    e.Aact = w.Aact; e.lda = 2 * Hm; e.Hm = Hm; e.nch = Hm / 16;
    e.W2m = w.W2mp; e.W2l = w.W2lp; e.b2m = w.b2mp; e.b2l = w.b2lp;
    e.eps = eps; e.seed = seed; e.offset = offset; e.xmask = xmask;
    e.MU = w.MU; e.LV = w.LV; e.OUT = w.OUT; e.Xin = w.Xin; e.F = F; e.Fp = Fp;
    e.off = off[t]; e.bs = b_t; e.next_off = off[t + 1]; e.next_bs = nb; e.feedback = c->feedback;
    dec_emit_fwd<<<cdiv(b_t, 16) * (Fp / 16), 256, 0, s>>>(e);
    ABCD_CHECK_LAUNCH();
  }
  // ---- offset head over all frames (off the recurrent critical path): the
  // logit's dot product folded into the Zo GEMM's epilogue where it applies ----
  bool fused = false;
  ABCD_TRY((hipError_t)gemm_offset_fwd(s, L, Hm, H, w.Hs, H, p->offset.w1, p->offset.b1, w.Zo, p->offset.w2,
                                       w.offpart, &fused));
  if (fused) {
    dec_offset_logit<<<cdiv(L, 256), 256, 0, s>>>(w.offpart, offset_head_slices(Hm), L, p->offset.b2, gt_offset,
                                                  w.offlog, w.dlog_raw, w.bce);
  } else {
    ABCD_TRY((hipError_t)gemm(s, L, Hm, H, opKC(w.Hs, H, L), opKC(p->offset.w1, H, Hm), w.Zo, Hm, 1.f, 0.f,
                              p->offset.b1, ACT_TANH, w.scratch, w.scratch_floats));
    dec_offset_head<<<cdiv(L, 4), 256, 0, s>>>(w.Zo, L, Hm, p->offset.w2, p->offset.b2, gt_offset, w.offlog,
                                               w.dlog_raw, w.bce);
  }
  ABCD_CHECK_LAUNCH();
  // ---- loss reductions: only the loss scalars read them, so with a loss
  // stream sl they run there beside the offset head's backward GEMM, behind
  // ONE fork after the logit pass (MU, LV, bce; w.part is theirs alone).  A
  // second fork after dec_fwd for the emission NLL alone cost its 6-7 us
  // event packet on the main queue.
  const bool em_loss = losses && x->data, off_loss = losses && gt_offset;
  if (em_loss || off_loss) ABCD_TRY((hipError_t)stream_fork(s, sl, 4));
  if (em_loss) {
    const int nbk = std::max(1, cdiv(L, NLL_ROWS));
    dec_emission_nll<<<nbk, 256, 0, sl>>>(w.MU, w.LV, Fp, x->data, F, L, w.part + 1024);
    ABCD_CHECK_LAUNCH();
    sum_partials<<<1, 256, 0, sl>>>(w.part + 1024, nbk, losses);
    ABCD_CHECK_LAUNCH();
  }
  if (off_loss) ABCD_TRY((hipError_t)reduce_sum(sl, w.bce, L, w.part, losses + 1, nullptr));
  if (flatten_out) { unpad_rows<<<launch_grid((long)L * F), 256, 0, s>>>(w.OUT, Fp, flatten_out, F, L); ABCD_CHECK_LAUNCH(); }
  if (mu_out) { unpad_rows<<<launch_grid((long)L * F), 256, 0, s>>>(w.MU, Fp, mu_out, F, L); ABCD_CHECK_LAUNCH(); }
  if (lv_out) { unpad_rows<<<launch_grid((long)L * F), 256, 0, s>>>(w.LV, Fp, lv_out, F, L); ABCD_CHECK_LAUNCH(); }
  if (offset_logits) ABCD_TRY(hipMemcpyAsync(offset_logits, w.offlog, (size_t)L * 4, hipMemcpyDeviceToDevice, s));
  return 0;
}

// reusable cross-stream events per device and slot (re-recorded each call:
// hipStreamWaitEvent captures the record that precedes it).  Slot 0: decoder
// data-gradient path done; 1: encoder counters zeroed; 2: encoder chunk A done;
// 3: decoder data-gradient path done, weight gradients deferred (the record of
// abcd_decoder_backward_dropout(..., ABCD_DEFER_PARAMS), waited for by the
// abcd_decoder_backward_params call that follows it on this host thread).
static int fork_event(hipEvent_t* ev, int slot) {
  static std::mutex mu;
  static hipEvent_t evs[64][4] = {};
  int dev = 0;
  ABCD_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64 || slot < 0 || slot >= 4) return (int)hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(mu);
  if (!evs[dev][slot]) ABCD_TRY(hipEventCreateWithFlags(&evs[dev][slot], hipEventDisableTiming));
  *ev = evs[dev][slot];
  return 0;
}

extern "C" int abcd_decoder_backward(const abcd_decoder_cfg* c, const abcd_decoder_params* p, const abcd_packed* x,
                                     const float* features, const int64_t* speakers, const float* gt_offset,
                                     const float* d_em, const float* d_off, float* d_features,
                                     const abcd_decoder_grads* g, void* ws, size_t ws_bytes, void* stream) {
  return abcd_decoder_backward_dropout(c, p, x, features, speakers, gt_offset, nullptr, d_em, d_off, d_features, g,
                                       ws, ws_bytes, stream, nullptr);
}

extern "C" int abcd_decoder_backward_overlap(const abcd_decoder_cfg* c, const abcd_decoder_params* p,
                                             const abcd_packed* x, const float* features, const int64_t* speakers,
                                             const float* gt_offset, const float* d_em, const float* d_off,
                                             float* d_features, const abcd_decoder_grads* g, void* ws,
                                             size_t ws_bytes, void* stream, void* wgrad_stream) {
  return abcd_decoder_backward_dropout(c, p, x, features, speakers, gt_offset, nullptr, d_em, d_off, d_features, g,
                                       ws, ws_bytes, stream, wgrad_stream);
}

// the decoder backward in two parts: DEC_DATA = the offset head, the BPTT and
// the initial-state / feature gradients (everything the sampler and encoder
// backward need), DEC_WGRAD = the weight gradients over all frames
enum { DEC_DATA = 1, DEC_WGRAD = 2 };
static int dec_bwd_impl(const abcd_decoder_cfg* c, const abcd_decoder_params* p, const abcd_packed* x,
                        const float* features, const int64_t* speakers, const float* gt_offset, const float* xmask,
                        const float* d_em, const float* d_off, float* d_features, const abcd_decoder_grads* g,
                        void* ws, size_t ws_bytes, void* stream, void* wgrad_stream, int mode);

extern "C" int abcd_decoder_backward_dropout(const abcd_decoder_cfg* c, const abcd_decoder_params* p,
                                             const abcd_packed* x, const float* features, const int64_t* speakers,
                                             const float* gt_offset, const float* xmask, const float* d_em,
                                             const float* d_off, float* d_features, const abcd_decoder_grads* g,
                                             void* ws, size_t ws_bytes, void* stream, void* wgrad_stream) {
  if (wgrad_stream == ABCD_DEFER_PARAMS)
    return dec_bwd_impl(c, p, x, features, speakers, gt_offset, xmask, d_em, d_off, d_features, g, ws, ws_bytes,
                        stream, nullptr, DEC_DATA);
  return dec_bwd_impl(c, p, x, features, speakers, gt_offset, xmask, d_em, d_off, d_features, g, ws, ws_bytes, stream,
                      wgrad_stream, DEC_DATA | DEC_WGRAD);
}

extern "C" int abcd_decoder_backward_params(const abcd_decoder_cfg* c, const abcd_decoder_params* p,
                                            const abcd_packed* x, const float* features, const int64_t* speakers,
                                            const float* gt_offset, const float* xmask, const float* d_em,
                                            const float* d_off, float* d_features, const abcd_decoder_grads* g,
                                            void* ws, size_t ws_bytes, void* stream, void* wgrad_stream) {
  ABCD_REQUIRE(wgrad_stream != ABCD_DEFER_PARAMS);
  return dec_bwd_impl(c, p, x, features, speakers, gt_offset, xmask, d_em, d_off, d_features, g, ws, ws_bytes, stream,
                      wgrad_stream, DEC_WGRAD);
}

static int dec_bwd_impl(const abcd_decoder_cfg* c, const abcd_decoder_params* p, const abcd_packed* x,
                        const float* features, const int64_t* speakers, const float* gt_offset, const float* xmask,
                        const float* d_em, const float* d_off, float* d_features, const abcd_decoder_grads* g,
                        void* ws, size_t ws_bytes, void* stream, void* wgrad_stream, int mode) {
  ABCD_REQUIRE(dec_check(c) == 0 && p && x && x->data && features && g && ws && d_em && d_off && gt_offset);
  ABCD_REQUIRE(!xmask || c->feedback);
  ABCD_REQUIRE(validate_batch(x->batch_sizes, x->T, x->L, x->B) == 0);
  hipStream_t s = (hipStream_t)stream;
  Arena A(ws, ws_bytes);
  DecWS w = carve_decoder(A, c, x->T, x->L, x->B);
  ABCD_REQUIRE(A.ok);
  const int H = c->hidden_size, Hm = c->mlp_hidden, F = c->output_size, Fp = rup16(F);
  const int G = c->rnn_type == ABCD_LSTM ? 4 : 3, GH = G * H;
  const int Htot = G == 4 ? 2 * H : H;
  const int D = c->feature_size, S = c->num_speakers > 0 ? c->speaker_dim : 0, DS = D + S;
  const int T = x->T, L = x->L, B = x->B;
  const int64_t* bs = x->batch_sizes;
  const std::vector<int> off = step_offsets(bs, T);
  float* sc = w.scratch;
  const size_t scf = w.scratch_floats;
  // (the transposed weights of the backward GEMMs were packed by the forward
  // pass, in its one pack launch: the backward reads the forward's stashes
  // from the same workspace anyway)
  const float* FS = S > 0 ? w.FS : features;
  if (mode & DEC_DATA) {
  // ---- offset head backward (batched over all frames): dZo formed from Zo
  // inside the DHO GEMM where it applies ----
  bool fused = false;
  ABCD_TRY((hipError_t)gemm_offset_bwd(s, L, H, Hm, w.Zo, w.W1oT, w.DHO, p->offset.w2, w.dlog_raw, d_off, w.dZo,
                                       w.dlog_s, &fused));
  if (!fused) {
    dec_offset_bwd<<<launch_grid((long)L * Hm), 256, 0, s>>>(w.Zo, L, Hm, p->offset.w2, w.dlog_raw, d_off, w.dZo,
                                                             w.dlog_s);
    ABCD_CHECK_LAUNCH();
    ABCD_TRY((hipError_t)gemm(s, L, H, Hm, opKC(w.dZo, Hm, L), opKC(w.W1oT, Hm, H), w.DHO, H, 1.f, 0.f, nullptr,
                              ACT_NONE, sc, scf));
  }
  // ---- BPTT: one persistent launch, or three launches per step ----
  bool done = false, dhid_done = false;
  {
    PDecBwdArgs pa{};
    pa.H = H; pa.Hm = Hm; pa.F = F; pa.Fp = Fp; pa.T = T; pa.nrt = cdiv(B, PERSIST_ROWS); pa.B = B;
    pa.feedback = c->feedback;
    pa.off = w.off; pa.sync = w.sync;
    pa.WihT = w.WihTp; pa.WhhT = w.WhhT; pa.W2mT = w.W2mT; pa.W2lT = w.W2lT; pa.W1T = w.W1catT;
    pa.Gst = w.Gst; pa.Cst = w.Cst; pa.Cprev = w.Cprev; pa.MU = w.MU; pa.LV = w.LV; pa.OUT = w.OUT;
    pa.Aact = w.Aact; pa.DHO = w.DHO; pa.Y = x->data; pa.s_em = d_em; pa.xmask = xmask;
    pa.dG = w.dGX; pa.dMU = w.dMU; pa.dLV = w.dLV; pa.dZ = w.dZ; pa.DHR = w.DC; pa.DC0 = w.DC0;
    pa.Hprev = w.Hprev; pa.dGH = w.dGH;
    pa.part = w.skp;
    pa.dhid = w.dhid;  // dec_bwd_w16 forms it in-kernel (dec_bwd_dhid_done)
    if (persist_enabled()) ABCD_TRY((hipError_t)stage_offsets(s, off, w.off));
    ABCD_TRY((hipError_t)persist_decoder_bwd(s, G, pa, &done));
    dhid_done = done && dec_bwd_dhid_done();
    ABCD_TRY((hipError_t)flush_offsets());
  }
  const int TN = bwd_tn(H);
  if (!done) note_dispatch(TK_DEC_BWD, "per-step decoder backward<%d>", G);
  for (int t = T - 1; t >= 0 && !done; --t) {
    const int b_t = (int)bs[t];
    const int nb = t + 1 < T ? (int)bs[t + 1] : 0;
    EmitBwdX e{};
    e.Ag = w.dGX + (size_t)off[t + 1] * GH; e.ldg = GH; e.succ_valid = c->feedback ? nb : 0; e.nch = GH / 16;
    e.WihT = w.WihTp; e.MU = w.MU; e.LV = w.LV; e.OUT = w.OUT; e.Y = x->data; e.s_em = d_em;
    e.xmask = xmask; e.succ_off = t + 1 < T ? off[t + 1] : 0;
    e.dMU = w.dMU; e.dLV = w.dLV; e.F = F; e.Fp = Fp; e.off = off[t]; e.bs = b_t;
    dec_emit_bwd_x<<<cdiv(b_t, 16) * (Fp / 16), 256, 0, s>>>(e);
    ABCD_CHECK_LAUNCH();
    MlpBwd m{};
    m.dMU = w.dMU; m.dLV = w.dLV; m.Fp = Fp; m.nch = Fp / 16; m.W2mT = w.W2mT; m.W2lT = w.W2lT;
    m.Aact = w.Aact; m.dZ = w.dZ; m.Hm = Hm; m.off = off[t]; m.bs = b_t;
    const int nr = (Hm / 16) % 4 == 0 ? 4 : ((Hm / 16) % 2 == 0 ? 2 : 1);
    const int mgrid = cdiv(b_t, 16) * (Hm / (16 * nr));
    if (nr == 4) dec_mlp_bwd<4><<<mgrid, 256, 0, s>>>(m);
    else if (nr == 2) dec_mlp_bwd<2><<<mgrid, 256, 0, s>>>(m);
    else dec_mlp_bwd<1><<<mgrid, 256, 0, s>>>(m);
    ABCD_CHECK_LAUNCH();
    BwdArgs a{};
    a.H = H;
    a.nd = 1;
    BwdDir& bd = a.d[0];
    bd.Ag = w.dGH + (size_t)off[t + 1] * GH; bd.succ_valid = nb; bd.WhhT = w.WhhT;
    bd.Az = w.dZ + (size_t)off[t] * 2 * Hm; bd.zrows = b_t; bd.W1T = w.W1catT; bd.ldz = 2 * Hm; bd.nchz = 2 * Hm / 16;
    bd.DHX = w.DHO; bd.lddhx = H;
    bd.dlast = nullptr; bd.ldl = 0; bd.hcol = 0; bd.ccol = -1;
    bd.Gst = w.Gst; bd.Cst = w.Cst; bd.Cprev = w.Cprev; bd.Hprev = w.Hprev;
    bd.dGX = w.dGX; bd.dGH = w.dGH; bd.DC = w.DC;
    bd.DCpred = t > 0 ? w.DC : w.DC0; bd.pred_off = t > 0 ? off[t - 1] : 0;
    bd.off = off[t]; bd.bs = b_t; bd.prev_valid = b_t; bd.next_bs = nb;
    bd.tiles = cdiv(b_t, 16) * (H / TN);
    TimedScope ts(s);
    if (G == 4) ABCD_TRY((hipError_t)launch_bwd_step<4>(s, a, bd.tiles, H));
    else ABCD_TRY((hipError_t)launch_bwd_step<3>(s, a, bd.tiles, H));
  }
  // ---- initial state gradient -> feature2hidden -> features / speaker embedding ----
  if (!dhid_done) {
    ABCD_TRY((hipError_t)gemm(s, B, H, GH, opKC(w.dGH, GH, B), opKC(w.WhhT, GH, H), w.dH0, H, 1.f, 0.f, nullptr,
                              ACT_NONE, sc, scf));
    dec_hidden_init_bwd<<<launch_grid((long)B * H), 256, 0, s>>>(w.dH0, w.DC0, B, H, G == 4, w.dhid);
    ABCD_CHECK_LAUNCH();
  }
  if (S == 0) {  // no speaker columns: the GEMM writes d_features itself (the split kernel was a copy)
    if (d_features)
      ABCD_TRY((hipError_t)gemm(s, B, D, Htot, opKC(w.dhid, Htot, B), opKC(w.Wf2hT, Htot, DS), d_features, D, 1.f,
                                0.f, nullptr, ACT_NONE, sc, scf));
  } else {
    ABCD_TRY((hipError_t)gemm(s, B, DS, Htot, opKC(w.dhid, Htot, B), opKC(w.Wf2hT, Htot, DS), w.dFS, DS, 1.f, 0.f,
                              nullptr, ACT_NONE, sc, scf));
    dec_feats_bwd<<<launch_grid((long)B * std::max(D, 1)), 256, 0, s>>>(w.dFS, D, S, B, speakers, c->num_speakers,
                                                                       d_features, g->embed_speaker);
    ABCD_CHECK_LAUNCH();
  }
  }
  if (!(mode & DEC_WGRAD)) {  // deferred: mark the end of the data path for abcd_decoder_backward_params
    hipEvent_t ev;
    ABCD_TRY((hipError_t)fork_event(&ev, 3));
    ABCD_TRY(hipEventRecord(ev, s));
    side_gate_arm();  // the next encoder BPTT launch of this thread is the gate's target
    return 0;
  }
  // ---- weight gradients, K = L frames ----
  // With a separate wgrad stream they run there, behind the data-gradient
  // path above, beside whatever the caller queues next on `stream` (the
  // sampler and encoder backward); the caller joins before reading them.
  const bool side = wgrad_stream && wgrad_stream != stream;
  if (side) {
    hipEvent_t ev;
    ABCD_TRY((hipError_t)fork_event(&ev, (mode & DEC_DATA) ? 0 : 3));
    if (mode & DEC_DATA) ABCD_TRY(hipEventRecord(ev, s));
    s = (hipStream_t)wgrad_stream;
    ABCD_TRY(hipStreamWaitEvent(s, ev, 0));
    // deferred form with abcd_side_gate_enable: the side work waits, on the
    // device, until the encoder BPTT queued since the data part is resident
    // (its members would otherwise wait for CUs the side GEMMs took first: up
    // to 150 us of start skew measured).  Queued only AFTER that launch, so
    // even a side stream sharing the BPTT's hardware queue cannot hold it back.
    if (!(mode & DEC_DATA)) ABCD_TRY((hipError_t)side_gate(s));
  }
  if (!(mode & DEC_DATA) && !side) side_gate_disarm();
  GemmSideScope side_tiles(side);
  if (g->f2h_w)
    ABCD_TRY((hipError_t)gemm(s, Htot, DS, B, opKM(w.dhid, Htot, Htot), opKM(FS, DS, DS), g->f2h_w, DS, 1.f, 0.f,
                              nullptr, ACT_NONE, sc, scf));
  if (g->f2h_b) ABCD_TRY((hipError_t)colsum(s, w.dhid, Htot, B, Htot, nullptr, g->f2h_b, 0.f, sc, scf));
  const abcd_rnn_g& cg = g->cell;
  // bias gradients as the last column of dG^T [Xin | 1] (Xin's pad column F
  // set to 1 after the BPTT; the packed W_ih pads are 0, so a later forward
  // that keeps it is unaffected) -- the colsum pass over L x G*H is gone
  const bool same_b = w.dGX == w.dGH;
  const bool ones = c->feedback && F < Fp && cg.w_ih && cg.b_ih && true;
  if (ones) {
    set_col_kernel<<<std::max(1, std::min(1024, cdiv(L, 256))), 256, 0, s>>>(w.Xin, Fp, L, F, 1.f);
    ABCD_CHECK_LAUNCH();
    ABCD_TRY((hipError_t)gemm(s, GH, F + 1, L, opKM(w.dGX, GH, GH), opKM(w.Xin, Fp, F + 1), w.dWb, F + 1, 1.f, 0.f,
                              nullptr, ACT_NONE, sc, scf));
    split_wb_kernel<<<(int)std::min<long>(1024, cdiv((long)GH * (F + 1), 256)), 256, 0, s>>>(
        w.dWb, GH, F, cg.w_ih, cg.b_ih, same_b ? cg.b_hh : nullptr);
    ABCD_CHECK_LAUNCH();
  } else if (cg.w_ih) {
    if (c->feedback)
      ABCD_TRY((hipError_t)gemm(s, GH, F, L, opKM(w.dGX, GH, GH), opKM(w.Xin, Fp, F), cg.w_ih, F, 1.f, 0.f, nullptr,
                                ACT_NONE, sc, scf));
    else
      ABCD_TRY(hipMemsetAsync(cg.w_ih, 0, (size_t)GH * F * 4, s));
  }
  if (cg.w_hh)
    ABCD_TRY((hipError_t)gemm(s, GH, H, L, opKM(w.dGH, GH, GH), opKM(w.Hprev, H, H), cg.w_hh, H, 1.f, 0.f, nullptr,
                              ACT_NONE, sc, scf));
  if (ones) {
    if (!same_b && cg.b_hh) ABCD_TRY((hipError_t)colsum(s, w.dGH, GH, L, GH, nullptr, cg.b_hh, 0.f, sc, scf));
  } else if (same_b && cg.b_ih) {  // LSTM: one pass for both bias gradients
    ABCD_TRY((hipError_t)colsum(s, w.dGX, GH, L, GH, nullptr, cg.b_ih, 0.f, sc, scf, cg.b_hh));
  } else {
    if (cg.b_ih) ABCD_TRY((hipError_t)colsum(s, w.dGX, GH, L, GH, nullptr, cg.b_ih, 0.f, sc, scf));
    if (cg.b_hh) ABCD_TRY((hipError_t)colsum(s, w.dGH, GH, L, GH, nullptr, cg.b_hh, 0.f, sc, scf));
  }
  // the emission MLPs' and the offset head's bias gradients (and the offset
  // head's w2 = Zo^T dlog) as ONE batched column sum (seven pass-1 / pass-2
  // pairs before), queued in front of their weight GEMMs so that a GEMM, not a
  // string of small reductions, ends the side stream's work
  const abcd_mlp_g* em[2] = {&g->mu, &g->lv};
  const float* dout[2] = {w.dMU, w.dLV};
  const abcd_mlp_g& og = g->offset;
  {
    ColsumJob cj[COLSUM_BATCH_MAX];
    int ncj = 0;
    for (int k = 0; k < 2; ++k) {
      if (em[k]->b2) cj[ncj++] = ColsumJob{dout[k], Fp, L, F, nullptr, em[k]->b2, 0.f, nullptr};
      if (em[k]->b1) cj[ncj++] = ColsumJob{w.dZ + k * Hm, 2 * Hm, L, Hm, nullptr, em[k]->b1, 0.f, nullptr};
    }
    if (og.b1) cj[ncj++] = ColsumJob{w.dZo, Hm, L, Hm, nullptr, og.b1, 0.f, nullptr};
    if (og.w2) cj[ncj++] = ColsumJob{w.Zo, Hm, L, Hm, w.dlog_s, og.w2, 0.f, nullptr};
    if (og.b2) cj[ncj++] = ColsumJob{w.dlog_s, 1, L, 1, nullptr, og.b2, 0.f, nullptr};
    ABCD_TRY((hipError_t)colsum_batch(s, cj, ncj, sc, scf));
  }
  for (int k = 0; k < 2; ++k) {
    const abcd_mlp_g& mg = *em[k];
    if (mg.w2)
      ABCD_TRY((hipError_t)gemm(s, F, Hm, L, opKM(dout[k], Fp, F), opKM(w.Aact + k * Hm, 2 * Hm, Hm), mg.w2, Hm, 1.f,
                                0.f, nullptr, ACT_NONE, sc, scf));
    if (mg.w1)
      ABCD_TRY((hipError_t)gemm(s, Hm, H, L, opKM(w.dZ + k * Hm, 2 * Hm, Hm), opKM(w.Hs, H, H), mg.w1, H, 1.f, 0.f,
                                nullptr, ACT_NONE, sc, scf));
  }
  if (og.w1)
    ABCD_TRY((hipError_t)gemm(s, Hm, H, L, opKM(w.dZo, Hm, Hm), opKM(w.Hs, H, H), og.w1, H, 1.f, 0.f, nullptr,
                              ACT_NONE, sc, scf));
  return 0;
}
