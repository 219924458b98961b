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
  const int* off;
  unsigned* sync;
  unsigned long long* prof;
};

constexpr int PERSIST_ROWS = 64;        // rows per workgroup
constexpr int PERSIST_SYNC_STRIDE = 32;  // uints per counter (128 B)

inline int persist_groups(int nd, int B) { return nd * cdiv(B, PERSIST_ROWS); }
inline size_t persist_sync_uints(int nd, int B) { return (size_t)persist_groups(nd, B) * PERSIST_SYNC_STRIDE; }

// Copy off[0..T] to device memory `dst` on stream s through a pinned ring
// (asynchronous, no host/device synchronisation).
int upload_offsets(hipStream_t s, const std::vector<int>& off, int* dst);

// Launch the persistent kernel if its grid can be co-resident on this device
// (*launched = true); otherwise leave *launched = false (caller runs the
// per-step kernels).  Returns 0 or a hipError_t.
int persist_encoder_fwd(hipStream_t s, int G, const PFwdArgs& a, bool* launched);
int persist_encoder_bwd(hipStream_t s, int G, const PBwdArgs& a, bool* launched);

// ABCD_PERSIST=0 disables the persistent path (parity/timing comparisons).
bool persist_enabled();

}  // namespace abcd
