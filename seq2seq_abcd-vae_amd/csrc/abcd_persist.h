// abcd_persist.h -- persistent ("whole time loop in one launch") recurrent
// kernels.  Host-internal interface between the encoder/decoder drivers in
// abcd_rnn.hip and the kernels in abcd_persist.hip (not part of the C ABI).
//
// Layout shared with the per-step kernels of abcd_rnn.hip: packed time-major
// rows (step t owns rows [off_t, off_t + bs_t)), and the Hprev/Cprev stashes
// hold a step's predecessor state AT THE CONSUMER'S ROW, so the persistent
// kernels write exactly the stashes the per-step kernels write and the
// weight-gradient GEMMs that follow are shared by both paths.
#pragma once
#include <vector>

#include "abcd_internal.h"

namespace abcd {

// One direction of an encoder layer, forward.
struct PFwdDir {
  const float* Whh;              // G*H x H (torch layout)
  const float* GX; long ldgx;    // x @ W_ih^T + b  (LSTM b_ih + b_hh, GRU b_ih), rows = frames
  const float* bhh;              // GRU b_hh (recurrent part), else null
  float *Gst, *Cst, *Y; long ldy;
  float *Hprev, *Cprev;          // stashes (Hprev is also the in-launch hand-off)
  float* out; long ldo; int hcol, ccol;  // final state (last_hidden), or null
  int rev;
};
struct PFwdArgs {
  PFwdDir d[2];
  int H, nd, T, nrt;
  const int* off;    // device: off[0..T]
  unsigned* sync;    // one 128-B counter line per group, zeroed before the launch
  unsigned long long* prof;  // diagnostics: per-step s_memtime stamps, or null
};

// One direction of an encoder layer, backward (BPTT).
struct PBwdDir {
  const float* WhhT;              // H x G*H
  const float* DHX; long lddhx;   // dh from the layer above, or null
  const float* dlast; long ldl; int hcol, ccol;  // d last_hidden
  const float *Gst, *Cst, *Cprev, *Hprev;
  float *dGX, *dGH;               // LSTM: the same buffer; dGH is the in-launch hand-off
  int rev;
};
struct PBwdArgs {
  PBwdDir d[2];
  int H, nd, T, nrt;
  int B;             // batch (rows of the first step): the 32-row groups of enc_bwd_w8
  const int* off;
  unsigned* sync;
  unsigned long long* prof;
  float* part;       // split-K partials: 2 parity slots x groups x H/16 consumers x 4 waves x H/16 producers x 256
  unsigned* started; // residency count (a zeroed registry line): the last workgroup to start bumps g_bptt_epoch
};

// Decoder forward (self-feedback LSTM, model.py:147-196): one launch for the
// whole time loop; per step three phases handed off inside a row-tile group:
//   cell : gates = Xin_t W_ih^T + Hprev_t W_hh^T + b  -> c, h (8 units / member)
//   mlp  : Aact = tanh(h W1cat^T + b1cat)              (16 columns / member)
//   emit : mu, lv = Aact W2^T + b2; x = mu + e^{lv/2} eps -> Xin_{t+1}
struct PDecFwdArgs {
  int H, Hm, F, Fp, T, nrt, feedback;
  int flags;                       // hand-off form: 1 per-member flags, 0 group counter
  const int* off;
  unsigned* sync;
  unsigned long long* prof;
  const float *Wih, *Whh, *bias;   // GH x Fp (padded), GH x H, GH (b_ih + b_hh)
  const float *W1, *b1;            // 2Hm x H, 2Hm  ([mu; lv] first layers)
  const float *W2m, *W2l, *b2m, *b2l;  // Fp x Hm (padded rows), Fp
  const float* eps; uint64_t seed, offset;  // explicit noise (rows x F) or Philox stream
  // eps_fill: eps is a workspace the launch fills itself with the Philox
  // stream (philox_normal(seed, offset + row F + col), nfill = L F values):
  // dec_fwd_x6's members without an emit tile draw step t + 1's rows in step
  // t's emit phase (step 0's before the loop); the other persistent forms get
  // it filled by abcd_fill_normal in front of their launch
  int eps_fill;
  long nfill;
  const float* xmask;              // input-dropout noise of the cell input (rows x F, 0 or 1/(1-p)); null: none
  float *Xin, *Hprev, *Cprev, *Gst, *Cst, *Hs, *Aact, *MU, *LV, *OUT;
};

// Decoder backward (BPTT of the same loop), per step t = T-1 .. 0, three phases:
//   P0: [dx_{t+1} | dh_rec] = dG_{t+1} [W_ih | W_hh]; dx -> dMU, dLV (+ emission NLL grads)
//   P1: dZ = [dMU W2m | dLV W2l] * (1 - Aact^2)
//   P2: dh = dZ W1cat + dh_rec + dh_offset -> LSTM cell backward -> dG_t
struct PDecBwdArgs {
  int H, Hm, F, Fp, T, nrt, feedback;
  int B;                           // batch (rows of step 0): the 32-row groups of dec_bwd_w16
  int flags;                       // hand-off form: 1 per-member flags, 0 group counter
  const int* off;
  unsigned* sync;
  unsigned long long* prof;
  const float *WihT, *WhhT;        // Fp x GH (rows >= F zero), H x GH
  const float *W2mT, *W2lT;        // Hm x Fp
  const float* W1T;                // H x 2Hm
  const float *Gst, *Cst, *Cprev, *MU, *LV, *OUT, *Aact, *DHO;
  const float* Hprev;              // GRU: h_{t-1} of every row (the cell backward's dz term)
  const float* Y;                  // target frames (rows x F)
  const float* s_em;               // device scalar: d loss / d emission NLL
  const float* xmask;              // input-dropout noise (rows x F) of the cell inputs; null: none
  float *dG, *dMU, *dLV, *dZ, *DHR, *DC0;
  float* dGH;                      // GRU: the recurrent-side gate gradients (dG holds the input side)
  float* part;  // split-K partials (dec_bwd_w16): 2 parity slots x 32-row groups x (Fp+H)/16 subtiles x 2 row blocks x 16 producers x 256
  // dhid (dec_bwd_w16; null: not formed): the gradient of feature2hidden's
  // output, [dh_{-1} | dc_{-1}] interleaved per unit (LSTM, B x 2H) or
  // dh_{-1} + the carry (GRU, B x H), with dh_{-1} = dG_0 W_hh summed over the
  // members by one more split-K hand-off after the time loop
  float* dhid;
};
inline size_t dec_part_floats(int B, int H, int Fp) {
  return 2 * (size_t)cdiv(B, 64) * (size_t)((Fp + H) / 16) * 4 * (size_t)(H / 8) * 256;
}

constexpr int PERSIST_ROWS = 64;        // rows per workgroup
constexpr int PERSIST_SYNC_STRIDE = 32;  // uints per counter (128 B)

inline int persist_groups(int nd, int B) { return nd * cdiv(B, PERSIST_ROWS); }
inline size_t persist_part_floats(int nd, int B, int H) {
  const size_t nut = (size_t)H / 16;
  return 2 * (size_t)persist_groups(nd, B) * nut * 4 * nut * 256;
}
// group counters + the role registry (abcd_persist.hip: 9 lines) + a second
// counter per group + 64 per-member flag lines per group (flag-form
// hand-offs), sized for 32-row groups (dec_bwd_w16, enc_bwd_w8), a superset
// of the 64-row layouts
inline size_t persist_sync_uints(int nd, int B) { return (size_t)(66 * nd * cdiv(B, 32) + 9) * PERSIST_SYNC_STRIDE; }

// Copy off[0..T] to device memory `dst` on stream s through a pinned ring
// (asynchronous, no host/device synchronisation).
int upload_offsets(hipStream_t s, const std::vector<int>& off, int* dst);
// The same copy left pending: the next persistent launch's counter reset on s
// performs it (one kernel); flush_offsets() issues it if no launch took it.
int stage_offsets(hipStream_t s, const std::vector<int>& off, int* dst);
int flush_offsets();

// Launch the persistent kernel if its grid can be co-resident on this device
// (*launched = true); otherwise leave *launched = false (caller runs the
// per-step kernels).  Returns 0 or a hipError_t.
int persist_encoder_fwd(hipStream_t s, int G, const PFwdArgs& a, bool* launched);
int persist_encoder_bwd(hipStream_t s, int G, const PBwdArgs& a, bool* launched);
int persist_decoder_fwd(hipStream_t s, int G, const PDecFwdArgs& a, bool* launched);
int persist_decoder_bwd(hipStream_t s, int G, const PDecBwdArgs& a, bool* launched);
// true if the last persist_decoder_bwd of this thread wrote a.dhid
bool dec_bwd_dhid_done();

// ABCD_PERSIST=0 disables the persistent path (parity/timing comparisons).
bool persist_enabled();

// Side-stream gate (abcd_side_gate_enable): a deferred decoder backward arms
// it (side_gate_arm), the first encoder BPTT launched after that on this host
// thread becomes its target, and abcd_decoder_backward_params queues, in front
// of the deferred side work, a one-wave kernel that waits (bounded) until that
// launch has every workgroup resident -- so the side GEMMs cannot take the
// launch's CUs first (two side GEMM workgroups on a CU leave no room for a
// BPTT member, which then starts only when one of them retires).  Queued after
// the launch, so it never holds back a BPTT that shares its hardware queue.
bool side_gate_enabled();
void side_gate_arm();
void side_gate_disarm();
int side_gate(hipStream_t sw);

}  // namespace abcd
