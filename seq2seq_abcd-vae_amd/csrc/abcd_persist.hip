// abcd_persist.hip -- persistent recurrent kernels: the whole packed time loop
// of one encoder layer (both directions) in ONE launch.
//
// Why: the per-step design of abcd_rnn.hip pays, at every one of the T steps,
// a kernel boundary plus a re-staging of the recurrent weight slice and a
// cold round trip for every operand -- ~15-20 us per step for ~2 us of MFMA
// work at the ABCD-VAE sizes (H = 256, batch 512).  Here each workgroup owns a
// fixed tile for the whole sequence:
//   forward : 64 rows x 16 units x G gates.  W_hh's 16-unit slice (G*16 x H)
//             is staged into LDS once; the cell state of the lane's 4 cells
//             stays in registers across steps.
//   backward: 64 rows x 16 units.  W_hh^T's 16-row slice (16 x G*H) in LDS;
//             the carry (LSTM dc*f, GRU dh*z) stays in registers.
// The only cross-workgroup dependency is the recurrent operand: step t's
// 64-row block needs all H (forward) / G*H (backward) columns of the previous
// step, produced by the NUT = H/16 workgroups of the same "group" (direction,
// row tile).  Hand-off per step (MI355X_MICROARCH.md, visibility table row 1):
// the payload is stored write-through (`sc1`), every storing wave drains
// (`s_waitcnt vmcnt(0)`), a workgroup barrier, ONE lane adds 1 to the group's
// counter (agent-scope atomic); the consumer's lane 0 polls the counter with
// `sc1` loads, a workgroup barrier releases the other waves, and EVERY load
// of the payload is an `sc1` buffer load (L1 bypass).  Stash rows are
// distinct per step, so no buffer is ever rewritten inside a launch (no WAR).
//
// Residency: every workgroup of a group must be resident for the group to
// progress, so the launcher checks grid <= CUs x occupancy and otherwise
// declines (the caller runs the per-step kernels).  Spins are bounded; a
// timeout sets abcd_device_status() and lets the grid drain.
#include <atomic>
#include <mutex>
#include <vector>
#include <cstdlib>

#include "abcd_common.h"
#include "abcd_internal.h"
#include "abcd_persist.h"
#include "abcd_x6.h"

namespace abcd {

__device__ unsigned g_persist_status = 0;
__device__ unsigned g_persist_sticky = 0;       // OR of every status abcd_step_status folded (abcd_device_status)
__device__ unsigned g_persist_abort = 0;        // a wait of the CURRENT launch timed out (zeroed by persist_reset)
__device__ unsigned g_spin_limit = 1u << 22;    // polls before a hand-off wait gives up (ABCD_SPIN_LIMIT, tests)
__device__ unsigned g_bptt_epoch = 0;           // encoder BPTT launches whose every workgroup has started

// ---------------------------------------------------------------------------
// hand-off primitives
// ---------------------------------------------------------------------------
// K-contiguous operand read through a buffer resource with `sc1` (bypasses
// this CU's L1, so it sees other workgroups' write-through stores); rows at
// or beyond the resource's extent read as zero (hardware range check).
template <int AUX = 16>  // the loads' cache policy (16 = sc1)
struct BufKCt {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t ld_bytes;
  DEV f4 frag(int row, int kc, int q) const {
    const uint32_t o = (uint32_t)row * ld_bytes + (uint32_t)(kc * 16 + 4 * q) * 4u;
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, AUX));
  }
  // x6 layout: k = 32c + 8q + 0..7
  DEV void frag8(int row, int c, int q, f4& lo, f4& hi) const {
    const uint32_t o = (uint32_t)row * ld_bytes + (uint32_t)(c * 32 + 8 * q) * 4u;
    lo = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, AUX));
    hi = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16u, 0, AUX));
  }
};
using BufKC = BufKCt<16>;
// Two K segments back to back (e.g. [x | h] of a recurrent cell): chunks
// [0, n0) come from segment 0, [n0, ntot) from segment 1; chunks >= ntot read
// zero without touching memory (offset past the descriptor's extent).
struct BufKC2 {
  __amdgpu_buffer_rsrc_t r0, r1;
  uint32_t ld0, ld1;
  int n0, ntot;
  DEV f4 frag(int row, int kc, int q) const {
    const bool s0 = kc < n0;
    const int k = s0 ? kc : kc - n0;
    uint32_t o = (uint32_t)row * (s0 ? ld0 : ld1) + (uint32_t)(k * 16 + 4 * q) * 4u;
    if (kc >= ntot) o = 0x80000000u;
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(s0 ? r0 : r1, o, 0, 16));
  }
};
// x6 form of BufKC2: 32-deep chunks, segment 0 holds n0 chunks of which the
// first kv0 elements are real (the rest read zero without touching memory)
template <int AUX = 16>
struct BufKC2xt {
  __amdgpu_buffer_rsrc_t r0, r1;
  uint32_t ld0, ld1;
  int n0, kv0;
  DEV void frag8(int row, int c, int q, f4& lo, f4& hi) const {
    const bool s0 = c < n0;
    const int k = (s0 ? c : c - n0) * 32 + 8 * q;
    uint32_t o = (uint32_t)row * (s0 ? ld0 : ld1) + (uint32_t)k * 4u;
    if (s0 && k >= kv0) o = 0x80000000u;
    lo = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(s0 ? r0 : r1, o, 0, AUX));
    hi = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(s0 ? r0 : r1, o + 16u, 0, AUX));
  }
};
using BufKC2x = BufKC2xt<16>;
DEV void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Wave-private LDS transpose of a 16 x 16 accumulator-layout tile (lane
// (r, q) holds rows 4q + g, column r) into row quads (lane l: row l >> 2,
// columns 4(l & 3) .. +3), so the tile leaves in ONE 16-B store per lane
// instead of four 4-B ones: a 4-B write-through store costs ~6x a 16-B one
// per byte (MI355X_MICROARCH.md), and every publish drains the wave's stores.
constexpr int TP_PITCH = 20;                    // floats per row: 16-B aligned rows, conflict-free writes
constexpr int TP_FLOATS = 16 * TP_PITCH;        // per wave
DEV f4 tp_quad(float* tb, const float (&v)[4], int lane) {
  const int r = lane & 15, q = lane >> 4;
  __builtin_amdgcn_wave_barrier();  // the previous quad reads of this buffer are issued (LDS is in order per wave)
#pragma unroll
  for (int g = 0; g < 4; ++g) tb[(4 * q + g) * TP_PITCH + r] = v[g];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return *reinterpret_cast<const f4*>(tb + (lane >> 2) * TP_PITCH + 4 * (lane & 3));
}
// 16-B store at byte offset `off` of the buffer `rs` (rows beyond its extent
// are dropped by the range check); sc1: write-through (hand-off payloads)
DEV void st4(__amdgpu_buffer_rsrc_t rs, uint32_t off, f4 v, bool wt) {
  if (wt) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rs, off, 0, 16);
  else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rs, off, 0, 0);
}

// Operands a phase needs only after its hand-off wait are loaded before it,
// branch-free (buffer loads: rows past the resource's extent read 0), and
// pinned after it: the poll's `s_waitcnt vmcnt(0)` then covers them in ONE
// round trip.  Conditional loads let the compiler hoist their consumers
// (tanh of the cell state) into the load branches, each with its own
// vmcnt(0) -- four serialized round trips in front of the P2 poll.
DEV float bld(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
}
template <int N>
DEV void pin(float (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" : "+v"(v[k]));
}
// Once a wait of this launch has timed out the launch's results are invalid
// anyway, so a wait that is still unsatisfied after SPIN_PROBE_MASK + 1
// polls gives up at once instead of spinning to its own limit: a failed
// launch drains in ~one wait instead of one limit per wait.  The word is the
// launch's own (persist_reset zeroes it in front of every persistent launch),
// so a timeout never shortens the waits of a later, healthy launch whatever
// reads or does not read the status words in between.  Probed every 1024
// polls only, off the fast path of a healthy hand-off.
constexpr unsigned SPIN_PROBE_MASK = 1023;
DEV bool spin_abandoned() {
  return __hip_atomic_load(&g_persist_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
DEV void spin_timed_out() {
  __hip_atomic_store(&g_persist_status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&g_persist_abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0 of the workgroup polls until *cnt >= target (bounded), then the
// barrier releases every wave (two polls in flight -- a new load issued
// before the previous one is checked -- measured slower: c2 step 8.43-8.49 ->
// 8.51-8.54 ms, dec_fwd +50 us, same box)
DEV void group_wait(unsigned* cnt, unsigned target, int pw = 0) {
  if (threadIdx.x == 64 * pw) {
    unsigned spins = 0;
    const unsigned lim = g_spin_limit;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > lim) {
        spin_timed_out();
        break;
      }
      if ((spins & SPIN_PROBE_MASK) == 0 && spin_abandoned()) break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
}
// every wave drains its stores, barrier, one lane signals
DEV void group_publish(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-member flag form of the same hand-off (MI355X_MICROARCH.md visibility
// table row 1 with a sharded counter): member m stores its publish count to
// its own 128-B line (sc1 store by one lane after every wave's vmcnt(0) drain
// and a barrier); a waiter's wave 0 polls the group's M lines with one sc1
// load per lane.  Replaces the M serialized atomic adds on one counter line
// (~12 ns each at the memory side) by parallel plain write-through stores.
constexpr int PERSIST_FLAG_LINES = 64;  // flag lines per group (members <= 64)
DEV void flags_publish(unsigned* fl, int mem, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(fl + mem * PERSIST_SYNC_STRIDE, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// pw: the polling wave (one whose pre-wait work is done soonest)
DEV void flags_wait(const unsigned* fl, int M, unsigned epoch, int pw = 0) {
  if ((threadIdx.x >> 6) == pw) {
    const int lane = threadIdx.x & 63;
    unsigned spins = 0;
    const unsigned lim = g_spin_limit;
    for (;;) {
      bool ok = true;
      if (lane < M)
        ok = __hip_atomic_load(fl + lane * PERSIST_SYNC_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > lim) {
        if (lane == 0) spin_timed_out();
        break;
      }
      if ((spins & SPIN_PROBE_MASK) == 0 && spin_abandoned()) break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
}
// a group's hand-off in either form (the launchers pick the per-member flags)
struct GSync {
  unsigned *cnt, *fl;
  int M, mem, use_flags;
  unsigned ep;  // publishes so far by this member
  DEV void wait(unsigned publishes, int pw = 0) {
    if (use_flags) flags_wait(fl, M, publishes, pw);
    else group_wait(cnt, (unsigned)M * publishes, pw);
  }
  DEV void publish() {
    ++ep;
    if (use_flags) flags_publish(fl, mem, ep);
    else group_publish(cnt);
  }
};

// residency: each workgroup of an encoder BPTT launch counts itself in on
// start; the last one bumps the device epoch the side-stream gate waits for
DEV void bptt_resident(unsigned* started) {
  if (started && threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n + 1 == gridDim.x) __hip_atomic_fetch_add(&g_bptt_epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// the gate: one wave polls until the epoch reaches `target` (bounded: 2^17
// polls of ~0.2-0.5 us, i.e. tens of ms; a timeout just lets the side work
// go -- no error)
__global__ void side_gate_kernel(unsigned target) {
  if (threadIdx.x == 0) {
    for (unsigned spins = 0; spins < (1u << 17); ++spins) {
      if (__hip_atomic_load(&g_bptt_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      __builtin_amdgcn_s_sleep(8);
    }
  }
}

// diagnostics: thread 0 stamps s_memrealtime (100 MHz, one clock for the whole
// device, so stamps of different workgroups compare) at the phase boundaries of step i
#define PSTAMP(k)                                                                                   \
  do {                                                                                              \
    if (a.prof && threadIdx.x == 0) a.prof[((size_t)blockIdx.x * T + i) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
static unsigned long long* g_prof = nullptr;
static int g_prof_mask = 0;  // 1 enc fwd, 2 enc bwd, 4 dec fwd, 8 dec bwd

// Workgroup -> (group, member) by block index (fallback placement).  Members
// of a group get equal blockIdx % 8, i.e. one XCD under round-robin dispatch
// (L2 locality; speed only).
DEV void group_role(int bid, int ngroups, int nmem, int& grp, int& mem) {
  if (ngroups % 8 == 0) {
    const int s = bid & 7, k = bid >> 3;
    grp = s + 8 * (k / nmem);
    mem = k % nmem;
  } else {
    grp = bid / nmem;
    mem = bid % nmem;
  }
}

// Registry lines after the group counters (kept in the sync layout: 8 + 1
// lines, zeroed with the counters).  Groups formed INSIDE XCDs from per-XCD
// tickets, with plain (L2-resident) hand-off stores, measured slower than
// write-through hand-offs on MI355X (c2: dec_bwd 4.63 vs 4.45 ms, enc_fwd 1.51
// vs 1.47), so roles come from the block index (group_role) and every
// hand-off store is write-through (sc1).
constexpr int PERSIST_REG_LINES = 9;
struct Role {
  int grp, mem;
};
DEV Role assign_role(int ngroups, int nmem) {
  Role r;
  group_role(blockIdx.x, ngroups, nmem, r.grp, r.mem);
  return r;
}
// ---------------------------------------------------------------------------
// encoder forward: one launch per layer, both directions
// ---------------------------------------------------------------------------
// X6 > 0: split-fp32 recurrent MMA with X6 = H / 32 chunks (abcd_x6.h).
template <int G, int PD, int X6>
__global__ __launch_bounds__(256) void enc_fwd_persist(PFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  const int H = a.H, nut = H / 16, nch = H / 16, T = a.T;
  const Role role = assign_role(a.nd * a.nrt, nut);
  const int grp = role.grp, mem = role.mem;
  const int dir = grp / a.nrt, rt = grp % a.nrt;
  const PFwdDir& D = a.d[dir];
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int u0 = mem * 16, unit = u0 + r;
  const int row0 = rt * PERSIST_ROWS + w * 16;  // this wave's first row inside a step
  unsigned* cnt = a.sync + grp * PERSIST_SYNC_STRIDE;
  if (X6) stage_x6(smem, D.Whh, H, H, G, H / 32, 0, H / 32, [&](int j, int rr) { return j * H + u0 + rr; });
  else stage_b_frag(smem, D.Whh, H, G, nch, [&](int j) { return j * H + u0; });
  float bh[G];
#pragma unroll
  for (int j = 0; j < G; ++j) bh[j] = (G == 3) ? D.bhh[j * H + unit] : 0.f;
  // wave-private transpose tile after the weight image (16-B stores, tp_quad)
  float* tb = reinterpret_cast<float*>(smem) + (size_t)G * 16 * H * (X6 ? 6 : 4) / 4 + w * TP_FLOATS;
  const int trow = lane >> 2, tcol = 4 * (lane & 3);
  __syncthreads();
  float st[4] = {0.f, 0.f, 0.f, 0.f};  // c (LSTM) / h (GRU) of the lane's 4 cells
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = D.rev ? T - 1 - i : i;
    const int o = off[t], bs = off[t + 1] - o;
    int prev_valid, next_off, next_bs;
    if (D.rev) {
      prev_valid = t == T - 1 ? 0 : off[t + 2] - off[t + 1];
      next_off = t >= 1 ? off[t - 1] : 0;
      next_bs = t >= 1 ? bs : 0;
    } else {
      prev_valid = t == 0 ? 0 : bs;
      next_off = off[t + 1];
      next_bs = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
    }
    PSTAMP(0);
    // input projection of this step (independent of the recurrence: loaded
    // before the wait so its latency hides behind it)
    float gxp[4][G];
    {
      const __amdgpu_buffer_rsrc_t rgx = make_rsrc(D.GX + (size_t)o * D.ldgx, (uint32_t)bs * D.ldgx * 4u);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < G; ++j) gxp[g][j] = bld(rgx, ((uint32_t)(row0 + 4 * q + g) * D.ldgx + j * H + unit) * 4u);
    }
    if (i > 0) group_wait(cnt, (unsigned)(nut * i));
#pragma unroll
    for (int g = 0; g < 4; ++g) pin(gxp[g]);
    PSTAMP(1);
    f4 acc[2][G];
    acc2_zero(acc);
    if (row0 < bs && prev_valid > 0) {
      const BufKC A{make_rsrc(D.Hprev + (size_t)o * H, (uint32_t)prev_valid * H * 4u),
                    (uint32_t)H * 4u};
      if (X6) {
        wave_mma_x6<G, (X6 > 0 ? X6 : 1), 4>(acc[0], A, row0 + r, smem, X6, lane, q);
      } else {
        wave_mma_lds<G, PD>(acc, A, row0 + r, smem, nch, lane, q);
      }
    }
    acc2_fold(acc);
    PSTAMP(2);
    // pass 1: cell update and the hand-off store of h (write-through), then
    // signal the group before any stash store is issued
    float gv[4][4], hv[4], cv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = row0 + 4 * q + g;
      const bool haspred = b < prev_valid;
      if (G == 4) {
        gv[g][0] = fsigmoid(gxp[g][0] + acc[0][0][g]);
        gv[g][1] = fsigmoid(gxp[g][1] + acc[0][1][g]);
        gv[g][2] = ftanh(gxp[g][2] + acc[0][2][g]);
        gv[g][3] = fsigmoid(gxp[g][3] + acc[0][3][g]);
        cv[g] = gv[g][1] * (haspred ? st[g] : 0.f) + gv[g][0] * gv[g][2];
        hv[g] = gv[g][3] * ftanh(cv[g]);
        st[g] = cv[g];
      } else {
        const float ghr = acc[0][0][g] + bh[0], ghz = acc[0][1][g] + bh[1], ghn = acc[0][2][g] + bh[2];
        gv[g][0] = fsigmoid(gxp[g][0] + ghr);
        gv[g][1] = fsigmoid(gxp[g][1] + ghz);
        gv[g][2] = ftanh(gxp[g][2] + gv[g][0] * ghn);
        gv[g][3] = ghn;
        hv[g] = (1.f - gv[g][1]) * gv[g][2] + gv[g][1] * (haspred ? st[g] : 0.f);
        cv[g] = 0.f;
        st[g] = hv[g];
      }
    }
    // h -> the next step's operand rows (write-through, 16-B stores; rows
    // >= next_bs fall outside the buffer's extent)
    const uint32_t qh = (uint32_t)((row0 + trow) * H + u0 + tcol) * 4u;
    {
      const f4 hq = tp_quad(tb, hv, lane);
      if (row0 < next_bs) st4(make_rsrc(D.Hprev + (size_t)next_off * H, (uint32_t)next_bs * H * 4u), qh, hq, true);
    }
    PSTAMP(3);
    group_publish(cnt);
    // pass 2: stashes for the backward pass and the outputs (plain 16-B
    // stores, drained while the next step waits for its operand)
    if (row0 < bs) {
      const __amdgpu_buffer_rsrc_t rg = make_rsrc(D.Gst + (size_t)o * 4 * H, (uint32_t)bs * 4 * H * 4u);
      const uint32_t go = (uint32_t)((row0 + trow) * 4 * H + u0 + tcol) * 4u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v[4] = {gv[0][j], gv[1][j], gv[2][j], gv[3][j]};
        st4(rg, go + (uint32_t)(j * H) * 4u, tp_quad(tb, v, lane), false);
      }
      if (G == 4) st4(make_rsrc(D.Cst + (size_t)o * H, (uint32_t)bs * H * 4u), qh, tp_quad(tb, cv, lane), false);
      if (D.Y)  // (null: the top layer's output sequence, which nothing reads)
        st4(make_rsrc(D.Y + (size_t)o * D.ldy, (uint32_t)bs * D.ldy * 4u),
            (uint32_t)((row0 + trow) * D.ldy + u0 + tcol) * 4u, tp_quad(tb, hv, lane), false);
      if (G == 4 && row0 < next_bs)
        st4(make_rsrc(D.Cprev + (size_t)next_off * H, (uint32_t)next_bs * H * 4u), qh, tp_quad(tb, cv, lane), false);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // rows without a predecessor / whose sequence ends here (rare)
      const int b = row0 + 4 * q + g;
      if (b >= bs) continue;
      const long rr = o + b;
      if (b >= prev_valid) {
        if (G == 4) D.Cprev[rr * H + unit] = 0.f;
        D.Hprev[rr * H + unit] = 0.f;
      }
      if (b >= next_bs && D.out) {
        D.out[(long)b * D.ldo + D.hcol + unit] = hv[g];
        if (G == 4) D.out[(long)b * D.ldo + D.ccol + unit] = cv[g];
      }
    }
    PSTAMP(4);
  }
}

// ---------------------------------------------------------------------------
// encoder backward (BPTT): one launch per layer, both directions
// ---------------------------------------------------------------------------
// fp32 MFMA gather form, for the widths the split-K forms (enc_bwd_w8 at
// H = 256, enc_bwd_sk at 64 / 128) do not cover
template <int G, int PD>
__global__ __launch_bounds__(256) void enc_bwd_persist(PBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  bptt_resident(a.started);
  const int H = a.H, GH = G * H, nut = H / 16, nchg = GH / 16, T = a.T;
  const Role role = assign_role(a.nd * a.nrt, nut);
  const int grp = role.grp, mem = role.mem;
  const int dir = grp / a.nrt, rt = grp % a.nrt;
  const PBwdDir& D = a.d[dir];
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int u0 = mem * 16, unit = u0 + r;
  const int row0 = rt * PERSIST_ROWS + w * 16;
  unsigned* cnt = a.sync + grp * PERSIST_SYNC_STRIDE;
  stage_b_frag(smem, D.WhhT, GH, 1, nchg, [&](int) { return u0; });
  __syncthreads();
  float carry[4] = {0.f, 0.f, 0.f, 0.f};  // LSTM dc*f / GRU dh*z flowing to the predecessor
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = D.rev ? i : T - 1 - i;
    const int o = off[t], bs = off[t + 1] - o;
    int succ_off, succ_valid, prev_valid;
    if (!D.rev) {
      succ_off = t + 1 < T ? off[t + 1] : 0;
      succ_valid = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
      prev_valid = t == 0 ? 0 : bs;
    } else {
      succ_off = t >= 1 ? off[t - 1] : 0;
      succ_valid = t >= 1 ? bs : 0;
      prev_valid = t == T - 1 ? 0 : off[t + 2] - off[t + 1];
    }
    PSTAMP(0);
    // epilogue operands (forward stashes, upper-layer dh, final-state grads)
    float pg[4][4], pc[4], pcp[4], pdh[4], pdc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = row0 + 4 * q + g;
      const bool live = b < bs;
      const long rr = o + (live ? b : 0);
      const bool fin = b >= succ_valid;
      const bool haspred = live && b < prev_valid;
      const float* Gr = D.Gst + rr * 4 * H;
#pragma unroll
      for (int j = 0; j < 4; ++j) pg[g][j] = live ? Gr[j * H + unit] : 0.f;
      pc[g] = (live && G == 4) ? D.Cst[rr * H + unit] : 0.f;
      pcp[g] = 0.f;
      if (haspred) pcp[g] = G == 4 ? D.Cprev[rr * H + unit] : D.Hprev[rr * H + unit];
      float dh = 0.f, dc = 0.f;
      if (live) {
        if (D.DHX) dh += D.DHX[rr * D.lddhx + unit];
        if (fin && D.dlast) {
          dh += D.dlast[(long)b * D.ldl + D.hcol + unit];
          if (G == 4 && D.ccol >= 0) dc = D.dlast[(long)b * D.ldl + D.ccol + unit];
        }
      }
      pdh[g] = dh;
      pdc[g] = dc;
    }
    if (i > 0) group_wait(cnt, (unsigned)(nut * i));
    PSTAMP(1);
    f4 acc[2][1];
    acc2_zero(acc);
    if (row0 < bs && succ_valid > 0) {
      const BufKC A{make_rsrc(D.dGH + (size_t)succ_off * GH, (uint32_t)succ_valid * GH * 4u), (uint32_t)GH * 4u};
      wave_mma_lds<1, PD>(acc, A, row0 + r, smem, nchg, lane, q);
    }
    acc2_fold(acc);
    PSTAMP(2);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = row0 + 4 * q + g;
      if (b >= bs) continue;
      const long rr = o + b;
      const bool fin = b >= succ_valid;
      float dh = acc[0][0][g] + pdh[g];
      if (G == 4) {
        const float i_ = pg[g][0], f_ = pg[g][1], g_ = pg[g][2], o_ = pg[g][3];
        const float tc = ftanh(pc[g]);
        const float dc = (fin ? pdc[g] : carry[g]) + dh * o_ * (1.f - tc * tc);
        float* dg = D.dGX + rr * GH;
        st_sc1(dg + unit, dc * g_ * i_ * (1.f - i_));
        st_sc1(dg + H + unit, dc * pcp[g] * f_ * (1.f - f_));
        st_sc1(dg + 2 * H + unit, dc * i_ * (1.f - g_ * g_));
        st_sc1(dg + 3 * H + unit, dh * tc * o_ * (1.f - o_));
        carry[g] = dc * f_;
      } else {
        if (!fin) dh += carry[g];
        const float r_ = pg[g][0], z_ = pg[g][1], n_ = pg[g][2], ghn = pg[g][3];
        const float hp = pcp[g];  // h_{t-1} of this cell (forward stash; 0 without predecessor)
        const float dnp = dh * (1.f - z_) * (1.f - n_ * n_);
        const float dzp = dh * (hp - n_) * z_ * (1.f - z_);
        const float drp = dnp * ghn * r_ * (1.f - r_);
        float* dx = D.dGX + rr * GH;
        float* dhh = D.dGH + rr * GH;
        dx[unit] = drp; dx[H + unit] = dzp; dx[2 * H + unit] = dnp;
        st_sc1(dhh + unit, drp); st_sc1(dhh + H + unit, dzp); st_sc1(dhh + 2 * H + unit, dnp * r_);
        carry[g] = dh * z_;
      }
    }
    PSTAMP(3);
    group_publish(cnt);
    PSTAMP(4);
  }
}


// ---------------------------------------------------------------------------
// encoder backward, split-K form (x6).  The recurrent product of BPTT,
//     dh_rec[b, u] = sum_k dG_succ[b, k] W_hh[k, u]     (k < G*H, u < H),
// is split over k by OWNERSHIP: member m produced the 64 columns
// k = gate*H + 16m + j of dG itself, so right after its cell-backward
// epilogue it multiplies them (through a wave-private LDS transpose, no
// global load) with its 64 rows of W_hh and publishes a partial
//     P_m[b, u] = sum_{k in own(m)} dG[b, k] W_hh[k, u]   for all 256 u,
// already in each consumer's accumulator layout (1 KiB per consumer and
// wave: one dwordx4 per lane).  The next step's consumer m' sums the 16
// partials of its unit tile.  Per wave and step this moves 16 KiB out and
// 16 KiB in instead of loading the whole 64 KiB dG row block of the group
// (the loads, not the MFMAs, bounded the gather form: tests/profiles).
// Partials are double-buffered by step parity: a member writes slot
// (i+1)&1 only after the wait for step i, which every member passes only
// after all of them consumed step i-1's partials (slot (i-1)&1).
// G = 3 (GRU) pads the own-column block to 64 with a zero gate.
// ---------------------------------------------------------------------------
// Round 3: wave w forms the partials of consumers 4w..4w+3 (NSUB / 4 of
// them) for all 64 rows of the member's tile, so its quarter of the W_hh
// image (2 chunks x 3 planes per consumer) lives in registers for the whole
// launch instead of every wave re-reading the whole 96 KiB image from LDS
// each step; the A fragments come from the member's shared dG tile (one
// barrier) and each consumer's partial leaves as soon as its accumulator is
// done, under the remaining MFMAs.  Same operands, same accumulation order as
// the per-wave form it replaced: bit-identical partials (same-box A/B at c2:
// enc_bwd 1.99 -> 1.93-1.97 ms).
constexpr int SK_PITCH = 68;  // floats per row of the wave-private dG transpose (conflict-free b128 reads)
template <int G, int NSUB>
__global__ __launch_bounds__(256) void enc_bwd_sk(PBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  bptt_resident(a.started);
  constexpr int H = NSUB * 16, GH = G * H, nut = NSUB;
  const int T = a.T, ng = a.nd * a.nrt;
  const Role role = assign_role(ng, nut);
  const int grp = role.grp, mem = role.mem;
  const int dir = grp / a.nrt, rt = grp % a.nrt;
  const PBwdDir& D = a.d[dir];
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int u0 = mem * 16, unit = u0 + r;
  const int row0 = rt * PERSIST_ROWS + w * 16;
  unsigned* cnt = a.sync + grp * PERSIST_SYNC_STRIDE;
  f4* Bimg = smem;                                         // [NSUB][2][3][64]
  float* Ast = reinterpret_cast<float*>(smem + NSUB * 2 * 3 * 64) + w * 16 * SK_PITCH;
  float* tb = reinterpret_cast<float*>(smem + NSUB * 2 * 3 * 64) + 4 * 16 * SK_PITCH + w * TP_FLOATS;
  const int trow = lane >> 2, tcol = 4 * (lane & 3);
  // B image: subtile j = output units 16j..16j+15, chunk c, lane (r, q):
  // kappa = 32c + 8q + 0..7 -> gate kappa/16, own unit kappa%16
  for (int e = threadIdx.x; e < NSUB * 16 * 2 * 4; e += 256) {
    const int qq = e & 3, c = (e >> 2) & 1, u = e >> 3;
    const int kap = 32 * c + 8 * qq, gate = kap >> 4, ju = kap & 15;
    f4 v0 = f4zero(), v1 = f4zero();
    if (gate < G) {
      const float* src = D.WhhT + (long)u * GH + gate * H + u0 + ju;
      v0 = *reinterpret_cast<const f4*>(src);
      v1 = *reinterpret_cast<const f4*>(src + 4);
    }
    bf8 h, m, l;
    split8(v0, v1, h, m, l);
    const int j = u >> 4, rr = u & 15;
    const int d = ((j * 2 + c) * 3) * 64 + qq * 16 + rr;
    Bimg[d] = __builtin_bit_cast(f4, h);
    Bimg[d + 64] = __builtin_bit_cast(f4, m);
    Bimg[d + 128] = __builtin_bit_cast(f4, l);
  }
  __syncthreads();
  constexpr int JW = NSUB / 4;  // consumers per wave
  static_assert(NSUB % 4 == 0, "the consumers are dealt over the 4 waves");
  bf8 Br[JW][2][3];  // this wave's quarter of the image, resident for the launch
#pragma unroll
  for (int jj = 0; jj < JW; ++jj)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        Br[jj][c][p] = __builtin_bit_cast(bf8, Bimg[(((JW * w + jj) * 2 + c) * 3 + p) * 64 + lane]);
  const float* const At = reinterpret_cast<const float*>(smem + NSUB * 2 * 3 * 64);  // the member's 64-row dG tile
  const size_t slot_f = (size_t)ng * nut * 4 * nut * 256;  // floats per parity slot
  float carry[4] = {0.f, 0.f, 0.f, 0.f};
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = D.rev ? i : T - 1 - i;
    const int o = off[t], bs = off[t + 1] - o;
    int succ_valid, prev_valid;
    if (!D.rev) {
      succ_valid = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
      prev_valid = t == 0 ? 0 : bs;
    } else {
      succ_valid = t >= 1 ? bs : 0;
      prev_valid = t == T - 1 ? 0 : off[t + 2] - off[t + 1];
    }
    PSTAMP(0);
    // cell operands: branch-free loads before the wait, pinned after it (bld)
    float pg[4][4], pc[4], pcp[4], pdh[4], pdl[4], pdc[4];
    {
      const uint32_t eh = (uint32_t)bs * H * 4u;
      const __amdgpu_buffer_rsrc_t rgs = make_rsrc(D.Gst + (size_t)o * 4 * H, eh * 4u),
                                   rcs = make_rsrc(D.Cst + (size_t)o * H, G == 4 ? eh : 0u),
                                   rcp = make_rsrc((G == 4 ? D.Cprev : D.Hprev) + (size_t)o * H,
                                                   (uint32_t)prev_valid * H * 4u),
                                   rdx = make_rsrc(D.DHX ? D.DHX + (size_t)o * D.lddhx : D.Gst,
                                                   D.DHX ? (uint32_t)bs * D.lddhx * 4u : 0u),
                                   rdl = make_rsrc(D.dlast ? D.dlast : D.Gst, D.dlast ? (uint32_t)bs * D.ldl * 4u : 0u);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t b = (uint32_t)(row0 + 4 * q + g);
        const bool fin = (int)b >= succ_valid;
#pragma unroll
        for (int j = 0; j < 4; ++j) pg[g][j] = bld(rgs, (b * 4 * H + j * H + unit) * 4u);
        pc[g] = G == 4 ? bld(rcs, (b * H + unit) * 4u) : 0.f;
        pcp[g] = bld(rcp, (b * H + unit) * 4u);
        pdh[g] = bld(rdx, (b * D.lddhx + unit) * 4u);
        // the last step's gradient enters rows that have no successor (rows >= bs read 0)
        pdl[g] = bld(rdl, fin ? (b * D.ldl + D.hcol + unit) * 4u : 0x80000000u);
        pdc[g] = (G == 4 && D.ccol >= 0) ? bld(rdl, fin ? (b * D.ldl + D.ccol + unit) * 4u : 0x80000000u) : 0.f;
      }
    }
    f4 dhr = f4zero();
    if (i > 0) group_wait(cnt, (unsigned)(nut * i));
    pin(pg[0]), pin(pg[1]), pin(pg[2]), pin(pg[3]), pin(pc), pin(pcp), pin(pdh), pin(pdl), pin(pdc);
#pragma unroll
    for (int g = 0; g < 4; ++g) pdh[g] += pdl[g];
    if (i > 0) {
      if (row0 < succ_valid) {
        const __amdgpu_buffer_rsrc_t pr = make_rsrc(a.part + (size_t)(i & 1) * slot_f, (uint32_t)(slot_f * 4));
        const uint32_t base = (uint32_t)((((size_t)grp * nut + mem) * 4 + w) * nut * 256 + lane * 4) * 4u;
        f4 v[NSUB];
#pragma unroll
        for (int m = 0; m < NSUB; ++m)
          v[m] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(pr, base + m * 1024u, 0, 16));
#pragma unroll
        for (int m = 0; m < NSUB; ++m) dhr += v[m];
      }
    }
    PSTAMP(1);
    // cell backward -> dG (LSTM: dGX == dGH; GRU: dGH = [dr, dz, dn*r])
    float dgh[4][4], dgx[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = row0 + 4 * q + g;
#pragma unroll
      for (int j = 0; j < 4; ++j) dgh[g][j] = dgx[g][j] = 0.f;
      if (b >= bs) continue;
      const bool fin = b >= succ_valid;
      float dh = (fin ? 0.f : dhr[g]) + pdh[g];
      if (G == 4) {
        const float i_ = pg[g][0], f_ = pg[g][1], g_ = pg[g][2], o_ = pg[g][3];
        const float tc = ftanh(pc[g]);
        const float dc = (fin ? pdc[g] : carry[g]) + dh * o_ * (1.f - tc * tc);
        dgx[g][0] = dc * g_ * i_ * (1.f - i_);
        dgx[g][1] = dc * pcp[g] * f_ * (1.f - f_);
        dgx[g][2] = dc * i_ * (1.f - g_ * g_);
        dgx[g][3] = dh * tc * o_ * (1.f - o_);
#pragma unroll
        for (int j = 0; j < 4; ++j) dgh[g][j] = dgx[g][j];
        carry[g] = dc * f_;
      } else {
        if (!fin) dh += carry[g];
        const float r_ = pg[g][0], z_ = pg[g][1], n_ = pg[g][2], ghn = pg[g][3];
        const float hp = pcp[g];
        const float dnp = dh * (1.f - z_) * (1.f - n_ * n_);
        const float dzp = dh * (hp - n_) * z_ * (1.f - z_);
        const float drp = dnp * ghn * r_ * (1.f - r_);
        dgx[g][0] = drp; dgx[g][1] = dzp; dgx[g][2] = dnp;
        dgh[g][0] = drp; dgh[g][1] = dzp; dgh[g][2] = dnp * r_;
        carry[g] = dh * z_;
      }
    }
    PSTAMP(2);
    // the wave's dG tile rows x [gate j][own unit] in LDS: the split-K
    // operand below and the stash after the publish
    if (row0 < bs) {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) Ast[(4 * q + g) * SK_PITCH + j * 16 + r] = dgh[g][j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // partials for the next step from this step's own dG columns
    if (i + 1 < T) {
      __syncthreads();  // every wave's dG rows are in the member's tile
      const __amdgpu_buffer_rsrc_t pw = make_rsrc(a.part + (size_t)((i + 1) & 1) * slot_f, (uint32_t)(slot_f * 4));
      // row tile mt + 1's split is issued between row tile mt's MFMAs (the
      // wave is alone on its SIMD: VALU after an MFMA run waits for its issue;
      // same-box A/B at c2: enc_bwd 1971 -> 1908 us)
      auto asplit = [&](int mt, bf8 (&av)[2][3]) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const float* ar = At + (16 * mt + r) * SK_PITCH + 32 * c + 8 * q;
          split8(*reinterpret_cast<const f4*>(ar), *reinterpret_cast<const f4*>(ar + 4), av[c][0], av[c][1], av[c][2]);
        }
      };
      bf8 av[2][3];
      asplit(0, av);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if (rt * PERSIST_ROWS + 16 * mt >= bs) break;  // uniform: row tiles past the step's batch
        bf8 an[2][3];
        if (mt + 1 < 4) asplit(mt + 1, an);
#pragma unroll
        for (int jj = 0; jj < JW; ++jj) {
          f4 acc = f4zero();
#pragma unroll
          for (int c = 0; c < 2; ++c) acc = mma_x6(acc, av[c][0], av[c][1], av[c][2], Br[jj][c][0], Br[jj][c][1], Br[jj][c][2]);
          // consumer j = JW w + jj, its wave mt: (((grp*nut + j)*4 + mt)*nut + mem)*256, lane's 4 floats (sc1)
          const int j = JW * w + jj;
          const uint32_t o = (uint32_t)(((((size_t)grp * nut + j) * 4 + mt) * nut + mem) * 256 + lane * 4) * 4u;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc), pw, o, 0, 16);
        }
        if (mt + 1 < 4) {
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // the next tile's dG reads
#pragma unroll
          for (int k = 0; k < 12 * JW; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
        }
        if (mt + 1 < 4) {  // a use here keeps the split in this block (LLVM would sink it past the break)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) asm volatile("" ::"v"(__builtin_bit_cast(f4, an[c][p])));
        }
        __builtin_amdgcn_sched_barrier(0);
        if (mt + 1 < 4) {
#pragma unroll
          for (int c = 0; c < 2; ++c) av[c][0] = an[c][0], av[c][1] = an[c][1], av[c][2] = an[c][2];
        }
      }
    }
    PSTAMP(3);
    group_publish(cnt);
    // stashes for the weight-gradient GEMMs after the launch (plain 16-B
    // stores after the publish, read back from the dG tile: 16 rows x 4 gates
    // x 4 quads of own units = 4 quads per lane).  LSTM: dGX = dGH = dG.
    // GRU: dGH = (dr, dz, dn r) is the tile; dGX = (dr, dz, dn) takes gate 2
    // from a transpose of dn.
    if (row0 < bs) {
      const __amdgpu_buffer_rsrc_t rx = make_rsrc(D.dGX + (size_t)o * GH, (uint32_t)bs * GH * 4u);
      const __amdgpu_buffer_rsrc_t rh = make_rsrc(D.dGH + (size_t)o * GH, (uint32_t)bs * GH * 4u);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        const int k = lane + 64 * k2, row = k >> 4, gate = (k >> 2) & 3, qd = 4 * (k & 3);
        if (gate >= G) continue;
        const f4 v = *reinterpret_cast<const f4*>(Ast + row * SK_PITCH + gate * 16 + qd);
        const uint32_t so = (uint32_t)((row0 + row) * GH + gate * H + u0 + qd) * 4u;
        if (G == 3) {
          st4(rh, so, v, false);
          if (gate < 2) st4(rx, so, v, false);
        } else {
          st4(rx, so, v, false);
        }
      }
      if (G == 3) {
        const float dn[4] = {dgx[0][2], dgx[1][2], dgx[2][2], dgx[3][2]};
        st4(rx, (uint32_t)((row0 + trow) * GH + 2 * H + u0 + tcol) * 4u, tp_quad(tb, dn, lane), false);
      }
    }
    PSTAMP(4);
  }
}


// stage chunks [0, nseg) of W's rows into chunks [kc0, kc0 + nseg) of an
// image with nch chunks per subtile
template <class RowFn>
DEV void stage_rows_seg(f4* dst, const float* W, long ldw, int nsub, int nseg, int kc0, int nch, RowFn rowfn) {
  constexpr int UNR = 16;
  const int total = nsub * 16 * nseg * 4;
  for (int base = 0; base < total; base += UNR * 256) {
    f4 v[UNR];
    int dsti[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int e = base + u * 256 + threadIdx.x;
      dsti[u] = -1;
      if (e < total) {
        const int q = e & 3, kc = (e >> 2) % nseg, rowi = (e >> 2) / nseg;
        const int j = rowi >> 4, r = rowi & 15;
        v[u] = *reinterpret_cast<const f4*>(W + (long)rowfn(j, r) * ldw + kc * 16 + 4 * q);
        dsti[u] = (j * nch + kc0 + kc) * 64 + q * 16 + r;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (dsti[u] >= 0) dst[dsti[u]] = v[u];
  }
}

// ring of 16 chunks; exact (drain-free) when nch is a multiple of 16
template <int NR, class OA, class Pre = NoPre>
DEV void mma16(f4 (&acc)[2][NR], const OA& A, int arow, const f4* Bl, int nch, int lane, int q, Pre pre = Pre()) {
  if (nch % 16 == 0) wave_mma_lds<NR, 16, false>(acc, A, arow, Bl, nch, lane, q, pre);
  else wave_mma_lds<NR, 16, true>(acc, A, arow, Bl, nch, lane, q, pre);
}

// ---------------------------------------------------------------------------
// decoder forward (LSTM): one launch for the whole time loop
// ---------------------------------------------------------------------------
// Group = 64-row tile, M = H/8 members.  Cell phase: member m owns units
// [8m, 8m+8) x 4 gates as two 16-column subtiles [i|f] and [g|o]; lanes r and
// r^8 swap their halves (one shuffle) so both hold all four gates of unit
// 8m + (r&7) and run the cell update redundantly (identical results).
// MLP / emit phases: 16-column tiles dealt round-robin over the members.
// Phase hand-offs use the group counter: every member adds 1 after each of
// the three phases; phase p of step i waits for M * (3i + p).
__device__ __forceinline__ int dec_cell_row(int H, int u0, int j, int r) { return (2 * j + (r >> 3)) * H + u0 + (r & 7); }
// GRU cell columns of a member (the same 2 x 16 subtile shape): subtile 0 =
// [r | z] (x and h parts), subtile 1 = [n_x | n_h] -- the candidate's input
// and recurrent projections stay apart (n = tanh(n_x + b_in + r (n_h + b_hn)),
// torch GRUCell), so n_x has a zero h part and n_h a zero x part.
// Row of W_ih (xpart) or W_hh for column (j, r); -1 = zero row.
__device__ __forceinline__ int dec_gru_row(int H, int u0, int j, int r, bool xpart) {
  const int g = 2 * j + (r >> 3), u = u0 + (r & 7);
  if (g < 2) return g * H + u;
  if (g == 2) return xpart ? 2 * H + u : -1;
  return xpart ? -1 : 2 * H + u;
}

// NCC > 0: the cell GEMM in split-fp32 (abcd_x6.h) over NCC 32-deep chunks
// (cdiv(Fp, 32) for x when self-feeding, + H / 32 for h)
template <int NCC>
__global__ __launch_bounds__(256) void dec_fwd_persist(PDecFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  const int H = a.H, Hm = a.Hm, Fp = a.Fp, F = a.F, T = a.T;
  const int M = H / 8, nchx = a.feedback ? Fp / 16 : 0, nchh = H / 16, nchm = Hm / 16, nchc = nchx + nchh;
  const int nx32 = a.feedback ? (Fp + 31) / 32 : 0;  // x6: chunks of x
  const int n1t = 2 * Hm / 16, n2t = Fp / 16;
  const Role role = assign_role(a.nrt, M);
  const int grp = role.grp, mem = role.mem;
  const int rt = grp;
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = rt * PERSIST_ROWS + w * 16;
  const int u0 = mem * 8, unit = u0 + (r & 7);
  unsigned* cnt = a.sync + grp * PERSIST_SYNC_STRIDE;
  // LDS images
  f4* BC = smem;                       // cell [x | h]  [2][nchc][64]  (x6: [2][NCC][3][64])
  f4* B1 = BC + (NCC ? 2 * NCC * 3 : 2 * nchc) * 64;  // mlp tiles [k][nchh][64]
  const int n1 = mem < n1t ? (n1t - 1 - mem) / M + 1 : 0;
  f4* B2 = B1 + n1 * nchh * 64;         // emit tiles   [k][2][nchm][64]
  const int n2 = mem < n2t ? (n2t - 1 - mem) / M + 1 : 0;
  if (NCC) {
    if (nx32) stage_x6(BC, a.Wih, Fp, Fp, 2, nx32, 0, NCC, [&](int j, int rr) { return dec_cell_row(H, u0, j, rr); });
    stage_x6(BC, a.Whh, H, H, 2, H / 32, nx32, NCC, [&](int j, int rr) { return dec_cell_row(H, u0, j, rr); });
  } else {
    if (nchx) stage_rows_seg(BC, a.Wih, Fp, 2, nchx, 0, nchc, [&](int j, int rr) { return dec_cell_row(H, u0, j, rr); });
    stage_rows_seg(BC, a.Whh, H, 2, nchh, nchx, nchc, [&](int j, int rr) { return dec_cell_row(H, u0, j, rr); });
  }
  for (int k = 0; k < n1; ++k) {
    const int j1 = mem + k * M;
    stage_b_frag(B1 + k * nchh * 64, a.W1, H, 1, nchh, [&](int) { return 16 * j1; });
  }
  for (int k = 0; k < n2; ++k) {
    const int j2 = mem + k * M;
    stage_b_frag(B2 + (2 * k) * nchm * 64, a.W2m, Hm, 1, nchm, [&](int) { return 16 * j2; });
    stage_b_frag(B2 + (2 * k + 1) * nchm * 64, a.W2l, Hm, 1, nchm, [&](int) { return 16 * j2; });
  }
  const float bias0 = a.bias[dec_cell_row(H, u0, 0, r)], bias1 = a.bias[dec_cell_row(H, u0, 1, r)];
  const bool lo = r < 8;
  __syncthreads();
  float cst[4] = {0.f, 0.f, 0.f, 0.f};
  bool cinit = false;
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = i;
    const int o = off[t], bs = off[t + 1] - o;
    const int next_off = off[t + 1];
    const int next_bs = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
    // ---------------- cell ----------------
    if (!cinit) {  // c_0 from feature2hidden (dec_init wrote it to the stash rows of step 0)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        cst[g] = b < bs ? a.Cprev[(long)(o + b) * H + unit] : 0.f;
      }
      cinit = true;
    }
    if (i > 0) group_wait(cnt, (unsigned)(M * 3 * i));
    PSTAMP(0);
    f4 acc[2][2];
    acc2_zero(acc);
    if (row0 < bs) {
      // [x_t | h_{t-1}] in one ring (x is zero at t = 0: empty descriptor)
      const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.Xin + (size_t)o * Fp, t > 0 ? (uint32_t)bs * Fp * 4u : 0u);
      const __amdgpu_buffer_rsrc_t rh = make_rsrc(a.Hprev + (size_t)o * H, (uint32_t)bs * H * 4u);
      if (NCC) {
        const BufKC2x A{rx, rh, (uint32_t)Fp * 4u, (uint32_t)H * 4u, nx32, Fp};
        wave_mma_x6<2, (NCC > 0 ? NCC : 1), 8>(acc[0], A, row0 + r, BC, NCC, lane, q);
      } else {
        const BufKC2 A{rx, rh, (uint32_t)Fp * 4u, (uint32_t)H * 4u, nchx, nchc};
        mma16<2>(acc, A, row0 + r, BC, nchc, lane, q);
      }
    }
    acc2_fold(acc);
    PSTAMP(7);
    float gi[4], gf[4], gg[4], go[4], hv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float v0 = acc[0][0][g] + bias0, v1 = acc[0][1][g] + bias1;
      const float w0 = __shfl_xor(v0, 8, 64), w1 = __shfl_xor(v1, 8, 64);
      gi[g] = fsigmoid(lo ? v0 : w0);
      gf[g] = fsigmoid(lo ? w0 : v0);
      gg[g] = ftanh(lo ? v1 : w1);
      go[g] = fsigmoid(lo ? w1 : v1);
      cst[g] = gf[g] * cst[g] + gi[g] * gg[g];
      hv[g] = go[g] * ftanh(cst[g]);
      const int b = row0 + 4 * q + g;
      if (b < bs) {
        if (lo) st_sc1(a.Hs + (long)(o + b) * H + unit, hv[g]);                       // -> mlp
        else if (b < next_bs) st_sc1(a.Hprev + (long)(next_off + b) * H + unit, hv[g]);  // -> next cell
      }
    }
    group_publish(cnt);
    PSTAMP(1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = row0 + 4 * q + g;
      if (b >= bs) continue;
      const long rr = o + b;
      float* Gr = a.Gst + rr * 4 * H;
      if (lo) {
        Gr[unit] = gi[g]; Gr[H + unit] = gf[g];
        a.Cst[rr * H + unit] = cst[g];
      } else {
        Gr[2 * H + unit] = gg[g]; Gr[3 * H + unit] = go[g];
        if (b < next_bs) a.Cprev[(long)(next_off + b) * H + unit] = cst[g];
      }
    }
    // ---------------- mlp ----------------
    group_wait(cnt, (unsigned)(M * (3 * i + 1)));
    PSTAMP(2);
    for (int k = 0; k < n1; ++k) {
      const int j1 = mem + k * M;
      f4 acc1[2][1];
      acc2_zero(acc1);
      if (row0 < bs) {
        const BufKC Hs{make_rsrc(a.Hs + (size_t)o * H, (uint32_t)bs * H * 4u), (uint32_t)H * 4u};
        mma16<1>(acc1, Hs, row0 + r, B1 + k * nchh * 64, nchh, lane, q);
      }
      acc2_fold(acc1);
      PSTAMP(6);
      const int col = 16 * j1 + r;
      const float bb = a.b1[col];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b < bs) st_sc1(a.Aact + (long)(o + b) * 2 * Hm + col, ftanh(acc1[0][0][g] + bb));
      }
    }
    group_publish(cnt);
    PSTAMP(3);
    // ---------------- emit ----------------
    // noise of the first owned tile, drawn before the wait (independent of
    // the recurrence); its stash stores go out after the hand-off publish
    float epre[4] = {0.f, 0.f, 0.f, 0.f}, mpre[4] = {1.f, 1.f, 1.f, 1.f}, mu0[4], lv0[4], x0[4];
    if (n2 > 0) {
      const int col = 16 * mem + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b < bs && col < F) {
          const long rr = o + b;
          epre[g] = a.eps ? a.eps[rr * F + col] : philox_normal(a.seed, a.offset + (uint64_t)rr * F + col);
          if (a.xmask && b < next_bs) mpre[g] = a.xmask[(long)(next_off + b) * F + col];
        }
      }
    }
    group_wait(cnt, (unsigned)(M * (3 * i + 2)));
    PSTAMP(4);
    for (int k = 0; k < n2; ++k) {
      const int j2 = mem + k * M;
      f4 am[2][1], al[2][1];
      acc2_zero(am);
      acc2_zero(al);
      if (row0 < bs) {
        const BufKC Am{make_rsrc(a.Aact + (size_t)o * 2 * Hm, (uint32_t)bs * 2 * Hm * 4u), (uint32_t)2 * Hm * 4u};
        const BufKC Al{make_rsrc(a.Aact + (size_t)o * 2 * Hm + Hm, (uint32_t)(bs * 2 * Hm - Hm) * 4u),
                       (uint32_t)2 * Hm * 4u};
        mma16<1>(am, Am, row0 + r, B2 + (2 * k) * nchm * 64, nchm, lane, q);
        mma16<1>(al, Al, row0 + r, B2 + (2 * k + 1) * nchm * 64, nchm, lane, q);
      }
      acc2_fold(am);
      acc2_fold(al);
      const int col = 16 * j2 + r;
      const float bm = a.b2m[col], bl = a.b2l[col];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        const long rr = o + b;
        float mu = 0.f, lv = 0.f, x = 0.f;
        if (col < F) {
          mu = am[0][0][g] + bm;
          lv = al[0][0][g] + bl;
          const float e = k == 0 ? epre[g]
                                 : (a.eps ? a.eps[rr * F + col]
                                          : philox_normal(a.seed, a.offset + (uint64_t)rr * F + col));
          x = mu + __expf(0.5f * lv) * e;
        }
        if (b < bs && a.feedback && b < next_bs) {
          const float m = k == 0 ? mpre[g] : ((a.xmask && col < F) ? a.xmask[(long)(next_off + b) * F + col] : 1.f);
          st_sc1(a.Xin + (long)(next_off + b) * Fp + col, x * m);
        }
        if (k == 0) {
          mu0[g] = mu; lv0[g] = lv; x0[g] = x;
        } else if (b < bs) {
          a.MU[rr * Fp + col] = mu;
          a.LV[rr * Fp + col] = lv;
          a.OUT[rr * Fp + col] = x;
        }
      }
    }
    group_publish(cnt);
    if (n2 > 0) {
      const int col = 16 * mem + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b >= bs) continue;
        const long rr = o + b;
        a.MU[rr * Fp + col] = mu0[g];
        a.LV[rr * Fp + col] = lv0[g];
        a.OUT[rr * Fp + col] = x0[g];
      }
    }
    PSTAMP(5);
  }
}


// ---------------------------------------------------------------------------
// decoder forward, all-x6 form.  The three phases of dec_fwd_persist<NCC>
// (cell / mlp / emit) with every product on the bf16 matrix cores (x6):
//   cell: as dec_fwd_persist<NCC>;
//   mlp : the member's 16-column tile of Aact (K = H, NH32 chunks);
//   emit: 2 * Fp/16 members, each owning one 16-column tile of [mu | lv] for
//         32 of the group's 64 rows: waves 0-1 compute mu, waves 2-3 lv
//         (K = Hm, NM32 chunks), so each wave gathers only its half of the
//         Aact row (16 KiB instead of 32) and runs one tile instead of two;
//         the lv waves hand lv to the mu waves through LDS, and those draw the
//         noise and store the self-feedback sample.
// ---------------------------------------------------------------------------
// GRU: the cell columns are dec_gru_row's, a.bias is [b_r | b_z | b_in | b_hn]
// (4H, r and z with b_ih + b_hh), the lanes carry h_{t-1} of their unit instead
// of c, and the stash row is (r, z, n, n_h + b_hn) as the per-step kernels'.
// HPRE: the recurrent half of step t+1's cell product, h_t W_hh^T, is formed
// in step t's mlp phase -- h_t is that phase's A operand already (rows of Hs =
// the next step's Hprev rows) -- as two more tiles beside the mlp tile, and
// carried in registers; step t+1's cell then waits only for x_{t+1} and runs
// the NCC - 8 input chunks (H = 256: 8 recurrent chunks).
// (Multiplying those two tiles after the mlp publish instead, from the Hs
// chunks kept in registers, measured slower: dec_fwd 2.17 / 2.20 -> 2.29 /
// 2.33 ms, same box.)
template <int NCC, int NH32, int NM32, bool GRU = false, bool HPRE = true>
__global__ __launch_bounds__(256) void dec_fwd_x6(PDecFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  const int H = a.H, Hm = a.Hm, Fp = a.Fp, F = a.F, T = a.T;
  const int M = H / 8;
  const int nx32 = a.feedback ? (Fp + 31) / 32 : 0;
  const int n1t = 2 * Hm / 16, n2t = Fp / 16;
  const Role role = assign_role(a.nrt, M);
  const int grp = role.grp, mem = role.mem;
  const int rt = grp;
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = rt * PERSIST_ROWS + w * 16;
  const int u0 = mem * 8, unit = u0 + (r & 7);
  GSync gs{a.sync + grp * PERSIST_SYNC_STRIDE,
           a.sync + ((size_t)2 * a.nrt + PERSIST_REG_LINES + (size_t)grp * PERSIST_FLAG_LINES) * PERSIST_SYNC_STRIDE,
           M, mem, a.flags, 0u};
  // emit roles: tile j2 of [mu | lv] columns, row half `half`; wave part 0 = mu, 1 = lv
  const int j2 = mem >> 1, half = mem & 1, part = w >> 1;
  const int erow0 = rt * PERSIST_ROWS + 32 * half + 16 * (w & 1);
  const bool has1 = mem < n1t, has2 = j2 < n2t;
  // LDS images
  f4* BC = smem;                        // cell [x | h]: [2][NCC][3][64]
  f4* B1 = BC + 2 * NCC * 3 * 64;       // mlp tile: [NH32][3][64]
  f4* B2 = B1 + NH32 * 3 * 64;          // emit: mu tile, lv tile: [2][NM32][3][64]
  float* LVX = reinterpret_cast<float*>(B2 + 2 * NM32 * 3 * 64);  // lv hand-over: [2][16][16]
  float* tb = LVX + 2 * 16 * 16 + w * TP_FLOATS;                   // this wave's transpose tile
  if (nx32)
    stage_x6(BC, a.Wih, Fp, Fp, 2, nx32, 0, NCC,
             [&](int j, int rr) { return GRU ? dec_gru_row(H, u0, j, rr, true) : dec_cell_row(H, u0, j, rr); });
  stage_x6(BC, a.Whh, H, H, 2, H / 32, nx32, NCC,
           [&](int j, int rr) { return GRU ? dec_gru_row(H, u0, j, rr, false) : dec_cell_row(H, u0, j, rr); });
  if (has1) stage_x6(B1, a.W1, H, H, 1, NH32, 0, NH32, [&](int, int rr) { return 16 * mem + rr; });
  if (has2) {
    stage_x6(B2, a.W2m, Hm, Hm, 1, NM32, 0, NM32, [&](int, int rr) { return 16 * j2 + rr; });
    stage_x6(B2 + NM32 * 3 * 64, a.W2l, Hm, Hm, 1, NM32, 0, NM32, [&](int, int rr) { return 16 * j2 + rr; });
  }
  const float bias0 = a.bias[dec_cell_row(H, u0, 0, r)], bias1 = a.bias[dec_cell_row(H, u0, 1, r)];
  const float b1v = has1 ? a.b1[16 * mem + r] : 0.f;
  // members without an emit tile draw the Philox noise of the group's rows of
  // a step into the eps workspace (write-through; read by the emit members'
  // sc1 loads a step later, after at least one hand-off that drained these
  // stores): the same philox_normal values abcd_fill_normal writes, drawn in
  // the emit phase these members otherwise idle through -- a side-stream fill
  // ran beside the input projection and delayed it / the encoder's launch
  const int nidle = M - 2 * n2t;
  auto fill_eps = [&](int ts) {
    const int o1 = a.off[ts], bs1 = a.off[ts + 1] - o1, rows = min(PERSIST_ROWS, bs1 - rt * PERSIST_ROWS);
    float* ep = const_cast<float*>(a.eps);
    for (int e = (mem - 2 * n2t) * 256 + (int)threadIdx.x; e < rows * F; e += nidle * 256) {
      const long rr = o1 + rt * PERSIST_ROWS + e / F;
      const int col = e % F;
      st_sc1(ep + rr * F + col, philox_normal(a.seed, a.offset + (uint64_t)rr * F + col));
    }
  };
  if (a.eps_fill && !has2 && nidle > 0) fill_eps(0);
  const int col2 = 16 * j2 + r;
  const float b2v = has2 ? (part ? a.b2l[col2] : a.b2m[col2]) : 0.f;
  const bool lo = r < 8;
  __syncthreads();
  float cst[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int NXC = NCC - 8;  // input chunks of the cell product (H = 256)
  f4 acch[2] = {f4zero(), f4zero()};  // HPRE: h_{t-1} W_hh^T of this step, from the previous mlp phase
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = i;
    const int o = off[t], bs = off[t + 1] - o;
    const int next_off = off[t + 1];
    const int next_bs = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
    // ---------------- cell ----------------
    if (i == 0) {  // c_0 (GRU: h_0) from feature2hidden (dec_init wrote it to the stash rows of step 0)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        cst[g] = b < bs ? (GRU ? a.Hprev : a.Cprev)[(long)(o + b) * H + unit] : 0.f;
      }
    }
    if (i > 0) gs.wait(3u * i);
    PSTAMP(0);
    f4 acc[2];
    acc[0] = acc[1] = f4zero();
    if (row0 < bs) {
      // [x_t | h_{t-1}] in one ring (x is zero at t = 0: empty descriptor)
      const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.Xin + (size_t)o * Fp, t > 0 ? (uint32_t)bs * Fp * 4u : 0u);
      const __amdgpu_buffer_rsrc_t rh = make_rsrc(a.Hprev + (size_t)o * H, (uint32_t)bs * H * 4u);
      const BufKC2x A{rx, rh, (uint32_t)Fp * 4u, (uint32_t)H * 4u, nx32, Fp};
      if (HPRE && i > 0) {
        acc[0] = acch[0];
        acc[1] = acch[1];
        if constexpr (NXC > 0)
          wave_mma_x6<2, (NXC > 0 ? NXC : 1), 4>(acc, A, row0 + r, BC, NCC, lane, q, mem % NXC);
      } else {
        wave_mma_x6<2, NCC, 4>(acc, A, row0 + r, BC, NCC, lane, q, mem % NCC);
      }
    }
    PSTAMP(7);
    // LSTM: (gi, gf, gg, go) = (i, f, g, o); GRU: (r, z, n, n_h + b_hn)
    float gi[4], gf[4], gg[4], go[4], hv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float v0 = acc[0][g] + bias0, v1 = acc[1][g] + bias1;
      const float w0 = __shfl_xor(v0, 8, 64), w1 = __shfl_xor(v1, 8, 64);
      if constexpr (GRU) {
        gi[g] = fsigmoid(lo ? v0 : w0);
        gf[g] = fsigmoid(lo ? w0 : v0);
        go[g] = lo ? w1 : v1;
        gg[g] = ftanh((lo ? v1 : w1) + gi[g] * go[g]);
        hv[g] = (1.f - gf[g]) * gg[g] + gf[g] * cst[g];
        cst[g] = hv[g];
      } else {
        gi[g] = fsigmoid(lo ? v0 : w0);
        gf[g] = fsigmoid(lo ? w0 : v0);
        gg[g] = ftanh(lo ? v1 : w1);
        go[g] = fsigmoid(lo ? w1 : v1);
        cst[g] = gf[g] * cst[g] + gi[g] * gg[g];
        hv[g] = go[g] * ftanh(cst[g]);
      }
    }
    // row quads of this wave's 16 rows x 8 units: lane l holds row trow, units
    // u0 + tc .. +3 of the tile's lo half (tcol < 8) or hi half (tcol >= 8)
    const int trow = lane >> 2, tcol = 4 * (lane & 3), tc = tcol & 7;
    const bool thi = tcol >= 8;
    const uint32_t qoff = (uint32_t)((row0 + trow) * H + u0 + tc) * 4u;  // byte offset in an H-pitch step block
    {  // h -> mlp (lo half) and -> the next cell (hi half, rows < next_bs)
      const f4 hq = tp_quad(tb, hv, lane);
      if (row0 < bs) {
        if (!thi) st4(make_rsrc(a.Hs + (size_t)o * H, (uint32_t)bs * H * 4u), qoff, hq, true);
        else st4(make_rsrc(a.Hprev + (size_t)next_off * H, (uint32_t)next_bs * H * 4u), qoff, hq, true);
      }
    }
    gs.publish();
    PSTAMP(1);
    if (row0 < bs) {  // stashes for the backward pass (plain 16-B stores)
      const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.Gst + (size_t)o * 4 * H, (uint32_t)bs * 4 * H * 4u);
      const uint32_t goff = (uint32_t)((row0 + trow) * 4 * H + u0 + tc) * 4u;
      {
        const float v[4] = {lo ? gi[0] : gg[0], lo ? gi[1] : gg[1], lo ? gi[2] : gg[2], lo ? gi[3] : gg[3]};
        st4(rg, goff + (uint32_t)(thi ? 2 * H : 0) * 4u, tp_quad(tb, v, lane), false);  // i | g
      }
      {
        const float v[4] = {lo ? gf[0] : go[0], lo ? gf[1] : go[1], lo ? gf[2] : go[2], lo ? gf[3] : go[3]};
        st4(rg, goff + (uint32_t)(thi ? 3 * H : H) * 4u, tp_quad(tb, v, lane), false);  // f | o
      }
      if constexpr (!GRU) {  // c -> Cst (lo half), -> the next step's Cprev row (hi half)
        const f4 cq = tp_quad(tb, cst, lane);
        if (!thi) st4(make_rsrc(a.Cst + (size_t)o * H, (uint32_t)bs * H * 4u), qoff, cq, false);
        else st4(make_rsrc(a.Cprev + (size_t)next_off * H, (uint32_t)next_bs * H * 4u), qoff, cq, false);
      }
    }
    // ---------------- mlp ----------------
    gs.wait(3u * i + 1);
    PSTAMP(2);
    if (has1) {
      f4 a1[1] = {f4zero()};
      if (row0 < bs) {
        const BufKC Hs{make_rsrc(a.Hs + (size_t)o * H, (uint32_t)bs * H * 4u), (uint32_t)H * 4u};
        if (HPRE && i + 1 < T) {  // + the next cell's recurrent tiles (chunks NXC.. of both BC subtiles)
          f4 a3[3] = {f4zero(), f4zero(), f4zero()};
          const f4* const bp[3] = {B1, BC + NXC * 3 * 64, BC + (NCC + NXC) * 3 * 64};
          wave_mma_x6p<3, NH32, 4>(a3, Hs, row0 + r, bp, lane, q, mem % NH32);
          a1[0] = a3[0];
          acch[0] = a3[1];
          acch[1] = a3[2];
        } else {
          wave_mma_x6<1, NH32, 4>(a1, Hs, row0 + r, B1, NH32, lane, q, mem % NH32);
        }
      }
      PSTAMP(6);
      const float av[4] = {ftanh(a1[0][0] + b1v), ftanh(a1[0][1] + b1v), ftanh(a1[0][2] + b1v), ftanh(a1[0][3] + b1v)};
      const f4 aq = tp_quad(tb, av, lane);
      if (row0 < bs)
        st4(make_rsrc(a.Aact + (size_t)o * 2 * Hm, (uint32_t)bs * 2 * Hm * 4u),
            (uint32_t)((row0 + trow) * 2 * Hm + 16 * mem + tcol) * 4u, aq, true);
    }
    gs.publish();
    PSTAMP(3);
    // ---------------- emit ----------------
    if (a.eps_fill && !has2 && nidle > 0 && i + 1 < T) fill_eps(t + 1);
    // the mu waves' noise, drawn before the wait (independent of the recurrence)
    float epre[4] = {0.f, 0.f, 0.f, 0.f}, mpre[4] = {1.f, 1.f, 1.f, 1.f};
    if (has2 && part == 0 && col2 < F) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = erow0 + 4 * q + g;
        if (b < bs) {
          const long rr = o + b;
          epre[g] = a.eps_fill ? __hip_atomic_load(a.eps + rr * F + col2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : a.eps    ? a.eps[rr * F + col2]
                               : philox_normal(a.seed, a.offset + (uint64_t)rr * F + col2);
          if (a.xmask && b < next_bs) mpre[g] = a.xmask[(long)(next_off + b) * F + col2];
        }
      }
    }
    // polled by wave 3 (an lv wave): the mu waves' noise draw above is ~1 us
    // of VALU that would otherwise delay the poll
    gs.wait(3u * i + 2, 3);
    PSTAMP(4);
    float ev[4] = {0.f, 0.f, 0.f, 0.f};  // mu (part 0) / lv (part 1); sample x kept in epre
    if (has2) {
      f4 ae[1] = {f4zero()};
      if (erow0 < bs) {
        const BufKC Aa{make_rsrc(a.Aact + (size_t)o * 2 * Hm + part * Hm, (uint32_t)(bs * 2 * Hm - part * Hm) * 4u),
                       (uint32_t)2 * Hm * 4u};
        wave_mma_x6<1, NM32, 4>(ae, Aa, erow0 + r, B2 + part * NM32 * 3 * 64, NM32, lane, q,
                                mem % NM32);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) ev[g] = col2 < F ? ae[0][g] + b2v : 0.f;
      if (part == 1) {
#pragma unroll
        for (int g = 0; g < 4; ++g) LVX[((w & 1) * 16 + 4 * q + g) * 16 + r] = ev[g];
      }
    }
    __syncthreads();
    // this wave's emit rows erow0 + trow, columns 16 j2 + tcol .. +3 (Fp pitch)
    const uint32_t eoff = (uint32_t)((erow0 + trow) * Fp + 16 * j2 + tcol) * 4u;
    if (has2 && part == 0) {
      float xm[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float lv = LVX[((w & 1) * 16 + 4 * q + g) * 16 + r];
        const float x = col2 < F ? ev[g] + __expf(0.5f * lv) * epre[g] : 0.f;
        epre[g] = x;
        xm[g] = x * mpre[g];
      }
      const f4 xq = tp_quad(tb, xm, lane);
      if (a.feedback && erow0 < next_bs)
        st4(make_rsrc(a.Xin + (size_t)next_off * Fp, (uint32_t)next_bs * Fp * 4u), eoff, xq, true);
    }
    gs.publish();
    if (has2 && erow0 < bs) {
      const uint32_t ext = (uint32_t)bs * Fp * 4u;
      if (part == 0) {
        st4(make_rsrc(a.MU + (size_t)o * Fp, ext), eoff, tp_quad(tb, ev, lane), false);
        st4(make_rsrc(a.OUT + (size_t)o * Fp, ext), eoff, tp_quad(tb, epre, lane), false);
      } else {
        st4(make_rsrc(a.LV + (size_t)o * Fp, ext), eoff, tp_quad(tb, ev, lane), false);
      }
    }
    PSTAMP(5);
  }
}

// ---------------------------------------------------------------------------
// decoder backward (LSTM): one launch for the whole BPTT loop
// ---------------------------------------------------------------------------
// Group = 64-row tile, M = H/8 members (as the forward).  Tiles of 16 columns
// dealt round-robin: P0 over Fp/16 + H/16 tiles, P1 over 2Hm/16, P2 over H/16
// (member m < H/16 owns unit tile m for the whole loop, so the dc carry of its
// cells stays in registers).
__global__ __launch_bounds__(256) void dec_bwd_persist(PDecBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  const int H = a.H, Hm = a.Hm, Fp = a.Fp, F = a.F, T = a.T, GH = 4 * H;
  const int M = H / 8, nchg = GH / 16, nchx = Fp / 16, nchz = 2 * Hm / 16;
  const int nFt = Fp / 16, n0t = nFt + H / 16, n1t = 2 * Hm / 16, n2t = H / 16;
  const Role role = assign_role(a.nrt, M);
  const int grp = role.grp, mem = role.mem;
  const int rt = grp;
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = rt * PERSIST_ROWS + w * 16;
  unsigned* cnt = a.sync + grp * PERSIST_SYNC_STRIDE;
  const int n0 = mem < n0t ? (n0t - 1 - mem) / M + 1 : 0;
  const int n1 = mem < n1t ? (n1t - 1 - mem) / M + 1 : 0;
  const bool own2 = mem < n2t;
  f4* B0 = smem;                       // P0 tiles [k][nchg][64]
  f4* B1 = B0 + n0 * nchg * 64;        // P1 tiles [k][nchx][64]
  f4* B2 = B1 + n1 * nchx * 64;        // P2 tile  [nchz][64]
  for (int k = 0; k < n0; ++k) {
    const int j0 = mem + k * M;
    if (j0 < nFt) stage_b_frag(B0 + k * nchg * 64, a.WihT, GH, 1, nchg, [&](int) { return 16 * j0; });
    else stage_b_frag(B0 + k * nchg * 64, a.WhhT, GH, 1, nchg, [&](int) { return 16 * (j0 - nFt); });
  }
  for (int k = 0; k < n1; ++k) {
    const int j1 = mem + k * M;
    if (j1 < Hm / 16) stage_b_frag(B1 + k * nchx * 64, a.W2mT, Fp, 1, nchx, [&](int) { return 16 * j1; });
    else stage_b_frag(B1 + k * nchx * 64, a.W2lT, Fp, 1, nchx, [&](int) { return 16 * (j1 - Hm / 16); });
  }
  if (own2) stage_b_frag(B2, a.W1T, 2 * Hm, 1, nchz, [&](int) { return 16 * mem; });
  const float s_em = *a.s_em;
  __syncthreads();
  float carry[4] = {0.f, 0.f, 0.f, 0.f};
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = T - 1 - i;
    const int o = off[t], bs = off[t + 1] - o;
    const int succ_off = t + 1 < T ? off[t + 1] : 0;
    const int succ_valid = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
    // ---------------- P0: dG_{t+1} [W_ih | W_hh] ----------------
    if (i > 0) group_wait(cnt, (unsigned)(M * 3 * i));
    PSTAMP(0);
    for (int k = 0; k < n0; ++k) {
      const int j0 = mem + k * M;
      const bool isx = j0 < nFt;
      f4 acc[2][1];
      acc2_zero(acc);
      if (row0 < bs && succ_valid > 0 && (!isx || a.feedback)) {
        const BufKC A{make_rsrc(a.dG + (size_t)succ_off * GH, (uint32_t)succ_valid * GH * 4u), (uint32_t)GH * 4u};
        mma16<1>(acc, A, row0 + r, B0 + k * nchg * 64, nchg, lane, q);
      }
      acc2_fold(acc);
      PSTAMP(6);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b >= bs) continue;
        const long rr = o + b;
        if (isx) {
          const int col = 16 * j0 + r;
          float dmu = 0.f, dlv = 0.f;
          if (col < F) {
            float dx = acc[0][0][g];
            if (a.xmask && b < succ_valid) dx *= a.xmask[(long)(succ_off + b) * F + col];
            const float mu = a.MU[rr * Fp + col], lv = a.LV[rr * Fp + col], ox = a.OUT[rr * Fp + col];
            const float y = a.Y[rr * F + col];
            const float iv = __expf(-lv), d = y - mu;
            dmu = dx + s_em * (-d) * iv;
            dlv = dx * 0.5f * (ox - mu) + s_em * 0.5f * (1.f - d * d * iv);
          }
          st_sc1(a.dMU + rr * Fp + col, dmu);
          st_sc1(a.dLV + rr * Fp + col, dlv);
        } else {
          st_sc1(a.DHR + rr * H + 16 * (j0 - nFt) + r, acc[0][0][g]);
        }
      }
    }
    group_publish(cnt);
    PSTAMP(1);
    // ---------------- P1: dZ ----------------
    // tanh outputs of the first owned tile, loaded before the wait
    float zpre[4] = {0.f, 0.f, 0.f, 0.f};
    if (n1 > 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b < bs) zpre[g] = a.Aact[(long)(o + b) * 2 * Hm + 16 * mem + r];
      }
    }
    group_wait(cnt, (unsigned)(M * (3 * i + 1)));
    PSTAMP(2);
    for (int k = 0; k < n1; ++k) {
      const int j1 = mem + k * M;
      const bool ismu = j1 < Hm / 16;
      f4 acc[2][1];
      acc2_zero(acc);
      if (row0 < bs) {
        const BufKC A{make_rsrc((ismu ? a.dMU : a.dLV) + (size_t)o * Fp, (uint32_t)bs * Fp * 4u), (uint32_t)Fp * 4u};
        mma16<1>(acc, A, row0 + r, B1 + k * nchx * 64, nchx, lane, q);
      }
      acc2_fold(acc);
      PSTAMP(7);
      const int col = 16 * j1 + r;  // column of [mu | lv] (2Hm)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b >= bs) continue;
        const long rr = o + b;
        const float z = k == 0 ? zpre[g] : a.Aact[rr * 2 * Hm + col];
        st_sc1(a.dZ + rr * 2 * Hm + col, acc[0][0][g] * (1.f - z * z));
      }
    }
    group_publish(cnt);
    PSTAMP(3);
    // ---------------- P2: dh -> cell backward -> dG_t ----------------
    // epilogue operands of the owned cells (plain: written by earlier launches)
    const int unit = 16 * mem + r;
    float pg[4][4], pc[4], pcp[4], pdho[4];
    if (own2) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        const bool live = b < bs;
        const long rr = o + (live ? b : 0);
        const float* Gr = a.Gst + rr * 4 * H;
#pragma unroll
        for (int j = 0; j < 4; ++j) pg[g][j] = live ? Gr[j * H + unit] : 0.f;
        pc[g] = live ? a.Cst[rr * H + unit] : 0.f;
        pcp[g] = live ? a.Cprev[rr * H + unit] : 0.f;
        pdho[g] = live ? a.DHO[rr * H + unit] : 0.f;
      }
    }
    group_wait(cnt, (unsigned)(M * (3 * i + 2)));
    PSTAMP(4);
    if (own2) {
      f4 acc[2][1];
      acc2_zero(acc);
      if (row0 < bs) {
        const BufKC A{make_rsrc(a.dZ + (size_t)o * 2 * Hm, (uint32_t)bs * 2 * Hm * 4u), (uint32_t)2 * Hm * 4u};
        mma16<1>(acc, A, row0 + r, B2, nchz, lane, q);
      }
      acc2_fold(acc);
      const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.DHR + (size_t)o * H, (uint32_t)bs * H * 4u);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = row0 + 4 * q + g;
        if (b >= bs) continue;
        const long rr = o + b;
        const bool fin = b >= succ_valid;
        const float dhr = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rd, (uint32_t)(b * H + unit) * 4u, 0, 16));
        const float dh = acc[0][0][g] + dhr + pdho[g];
        const float i_ = pg[g][0], f_ = pg[g][1], g_ = pg[g][2], o_ = pg[g][3];
        const float tc = ftanh(pc[g]);
        const float dc = (fin ? 0.f : carry[g]) + dh * o_ * (1.f - tc * tc);
        float* dg = a.dG + rr * GH;
        st_sc1(dg + unit, dc * g_ * i_ * (1.f - i_));
        st_sc1(dg + H + unit, dc * pcp[g] * f_ * (1.f - f_));
        st_sc1(dg + 2 * H + unit, dc * i_ * (1.f - g_ * g_));
        st_sc1(dg + 3 * H + unit, dh * tc * o_ * (1.f - o_));
        carry[g] = dc * f_;
        if (t == 0) a.DC0[(long)b * H + unit] = dc * f_;
      }
    }
    group_publish(cnt);
    PSTAMP(5);
  }
}

// ---------------------------------------------------------------------------
// split-K BPTT building blocks.  The big product of a BPTT step (decoder:
// [dx_{t+1} | dh_rec] = dG_{t+1} [W_ih | W_hh]^T-rows, K = 4H) is split over
// K by OWNERSHIP: every member owns a block of hidden units (their gate
// columns of dG), multiplies those columns with its rows of the weights right
// after its cell backward, and publishes one partial of every output subtile
// in each consumer's accumulator layout; consumers sum the partials
// (sum_partials).  Partials are double-buffered by step parity (written at
// step i into slot i & 1, read at step i + 1; rewritten at step i + 2 only
// after every member has published the next phase, i.e. finished its reads).
// The 64-row forms of rounds 2-3 (dec_bwd_sk: the dZ gather in P2;
// dec_bwd_fold: dZ W1cat folded into the partials) were superseded by the
// 32-row dec_bwd_w16 below and removed.
// ---------------------------------------------------------------------------
// acc += sum of NP partial f4s at base + p * 1 KiB, NB loads in flight
template <int NP, int NB = NP>
DEV void sum_partials(__amdgpu_buffer_rsrc_t rs, uint32_t base, f4& acc, int rot = 0) {
  auto pp = [&](int p) { const int x = p + rot; return x >= NP ? x - NP : x; };
#pragma unroll
  for (int p0 = 0; p0 < NP; p0 += NB) {
    f4 v[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k)
      v[k] = p0 + k < NP ? __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (uint32_t)pp(p0 + k) * 1024u,
                                                                                        0, 16))
                         : f4zero();
#pragma unroll
    for (int k = 0; k < NB; ++k) acc += v[k];
  }
}
// ---------------------------------------------------------------------------
// dec_bwd_w16 (round 4): the split-K decoder BPTT in 32-row groups.
//
// Per step a split-K member writes one partial of every output column for
// every row of its group, so the bytes a step moves chip-wide are
//     (CUs) x (rows per group) x (H + Fp output columns) x 4 B
// -- 25 MiB at c2 with 64-row groups of 32 members (8 units each), the
// write-through volume that makes dec_bwd_fold store-bound and slows it by a
// third when all 8 groups exchange at once.  Here a group is
// a 32-ROW tile of 16 members that own 16 units each (K = 64 gate columns,
// two 32-deep x6 chunks): the same 256 CUs, half the rows per group, half the
// partial bytes (12.5 MiB per step; a member writes 32 KiB of dh partials and
// 18 KiB of dx partials per step instead of 64 + 36) and half the fan-in of
// every reduction (16 producers).  The doubled K per member would not fit
// dec_bwd_fold's LDS images (150 KiB of x6 W_hh / W_ih rows alone), so the
// waves split the OUTPUT columns instead of the rows: wave w forms the dh
// partials of units 64w .. 64w + 63 (four subtiles, both 16-row blocks) and
// keeps that quarter of the W_hh image in registers for the whole launch
// (96 VGPRs); the W_ih (dx) image, the W1cat fold image and the dZ tile's W2
// fragments stay in LDS (145 KiB).
//   P0  (18 units = 2 row blocks x 9 column tiles, one wave each): sum the 16
//       dx partials of the tile -> dMU, dLV (+ the emission NLL terms)
//   P1  wave (rb, jj): the member's dZ column tile 2 mem + jj of row block rb
//       (x6, K = Fp); then every wave: its 8 dh partial tiles
//       = dG_{t+1}[:, own 64] W_hh[own 64, its 64 units]   (x6, before the wait)
//       + dZ_t[:, own 32]   W1cat[own 32, its 64 units]   (x6)
//  P2  waves (rb, half) sum 8 of the 16 dh partials of the member's 16
//       units; waves 0 / 1 add the other half through LDS and run the cell
//       backward of row block 0 / 1; every wave splits the 32 x 64 dG tile
//       and forms its share of the 18 dx partial tiles (x6, K = 64)
// Partials are double-buffered by step parity as in dec_bwd_fold.  Reference:
// the decoder BPTT of model.py:174-183 (LSTMCell / GRUCell, the emission MLPs
// 303-314 and the Gaussian NLL 30-37).
// ---------------------------------------------------------------------------
constexpr int W16_ROWS = 32;    // rows per group
constexpr int W16_M = 16;       // members per group (16 units each)
constexpr int W16_DTP = 68;     // pitch (floats) of the group's 32 x 64 dG tile in LDS
constexpr int W16_ZTP = 36;     // pitch of the 32 x 32 dZ tile
// The P1 dZ product (x6 over K = Fp in ceil(Fp / 32) chunks) runs on all four
// waves, one (row block, dZ column tile) each: a row block's dMU / dLV rows
// are loaded by two waves (the second mostly from L2), for half the MFMAs per
// wave on the critical path.  Same-box A/B (round 6) against waves 0 / 1 each
// running both tiles of one row block: dec_bwd 2.29 vs 2.32 ms (3 pairs).
// GRU: the member's gate columns are dec_fwd_x6's [r | z | n_x | n_h]
// (dG = [dr, dz, dn, dn r] pre-activation gradients), the split-K images take
// the n_x column from W_ih only and n_h from W_hh only, the carry is dh z, and
// the stash is dGX = (dr, dz, dn), dGH = (dr, dz, dn r) with pitch 3H as the
// per-step kernels write it.
template <int NXS, bool GRU = false>
__global__ __launch_bounds__(256) void dec_bwd_w16(PDecBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  constexpr int H = 256, NHS = 16, GH = (GRU ? 3 : 4) * H, M = W16_M;
  const int Hm = a.Hm, Fp = a.Fp, F = a.F, T = a.T;
  const int nFt = Fp / 16;
  constexpr int NCZ = (NXS > 0 ? NXS : 9) / 2 + 1;  // x6 chunks of K = Fp (Fp = 16 NXS with feedback)
  const int ncz = (Fp + 31) / 32;
  const int ng = a.nrt;  // 32-row groups (the launcher's count)
  const Role role = assign_role(ng, M);
  const int grp = role.grp, mem = role.mem;
  const int rowg = grp * W16_ROWS;
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  GSync gs{a.sync + grp * PERSIST_SYNC_STRIDE,
           a.sync + ((size_t)2 * ng + PERSIST_REG_LINES + (size_t)grp * PERSIST_FLAG_LINES) * PERSIST_SYNC_STRIDE,
           M, mem, a.flags, 0u};
  const int u0 = mem * 16;
  // LDS: dx image [NXS][2][3][64] | fold image [NHS][3][64] | P1 W2 image [2][ncz][3][64]
  //      | dG tile [32][68] | dZ tile [32][36] | dh half-sums [2][64] | wave transposes [4][2 TP]
  f4* DXI = smem;
  f4* W1X = DXI + NXS * 2 * 3 * 64;
  f4* B1 = W1X + NHS * 3 * 64;
  float* DT = reinterpret_cast<float*>(B1 + 2 * ncz * 3 * 64);
  float* ZT = DT + W16_ROWS * W16_DTP;
  f4* DHX = reinterpret_cast<f4*>(ZT + W16_ROWS * W16_ZTP);
  float* tb = reinterpret_cast<float*>(DHX + 2 * 64) + w * 2 * TP_FLOATS;
  const int trow = lane >> 2, tcol = 4 * (lane & 3);
  // gate-slot column of W for K index kappa = 16 slot + ju of this member
  // (xs: the W_ih image, else W_hh); GRU slots (r, z, n_x, n_h): n_x has no
  // W_hh part, n_h no W_ih part (-1: a zero row)
  auto kcol = [&](int slot, bool xs) -> int {
    if (GRU && slot >= 2) return (slot == 2) == xs ? 2 * H + u0 : -1;
    return slot * H + u0;
  };
  // dx image: column tile s, chunk c, lane (rr, qq): kappa = 32c + 8qq + 0..7
  for (int e = threadIdx.x; e < NXS * 2 * 64; e += 256) {
    const int s = e >> 7, c = (e >> 6) & 1, ln = e & 63, rr = ln & 15, qq = ln >> 4;
    const int col = kcol(2 * c + (qq >> 1), true);
    const float* src = a.WihT + (long)(16 * s + rr) * GH + (col < 0 ? 0 : col + 8 * (qq & 1));
    bf8 h, m, l;
    split8(col < 0 ? f4zero() : *reinterpret_cast<const f4*>(src), col < 0 ? f4zero() : *reinterpret_cast<const f4*>(src + 4),
           h, m, l);
    f4* d = DXI + ((s * 2 + c) * 3) * 64 + ln;
    d[0] = __builtin_bit_cast(f4, h);
    d[64] = __builtin_bit_cast(f4, m);
    d[128] = __builtin_bit_cast(f4, l);
  }
  // fold image: unit subtile s, lane (rr, qq): W1cat[unit 16s + rr][dZ column 32 mem + 8qq + 0..7]
  for (int e = threadIdx.x; e < NHS * 64; e += 256) {
    const int s = e >> 6, ln = e & 63, rr = ln & 15, qq = ln >> 4;
    const float* src = a.W1T + (long)(16 * s + rr) * 2 * Hm + 32 * mem + 8 * qq;
    bf8 h, m, l;
    split8(*reinterpret_cast<const f4*>(src), *reinterpret_cast<const f4*>(src + 4), h, m, l);
    f4* d = W1X + (s * 3) * 64 + ln;
    d[0] = __builtin_bit_cast(f4, h);
    d[64] = __builtin_bit_cast(f4, m);
    d[128] = __builtin_bit_cast(f4, l);
  }
  // P1 dZ column tiles 2 mem, 2 mem + 1 (mu tiles for mem < Hm / 32, else lv)
  const bool ismu = 2 * mem < Hm / 16;
  stage_x6(B1, ismu ? a.W2mT : a.W2lT, Fp, Fp, 2, ncz, 0, ncz,
           [&](int j, int rr) { return 16 * (2 * mem + j) - (ismu ? 0 : Hm) + rr; });
  // this wave's quarter of the W_hh image (units 64w .. 64w + 63), resident in registers
  bf8 Bh[4][2][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int col = kcol(2 * c + (q >> 1), false);
      const float* src = a.WhhT + (long)(16 * (4 * w + j) + r) * GH + (col < 0 ? 0 : col + 8 * (q & 1));
      split8(col < 0 ? f4zero() : *reinterpret_cast<const f4*>(src), col < 0 ? f4zero() : *reinterpret_cast<const f4*>(src + 4),
             Bh[j][c][0], Bh[j][c][1], Bh[j][c][2]);
    }
  const float s_em = *a.s_em;
  __syncthreads();
  const size_t slot_f = (size_t)ng * (NXS + NHS) * 2 * M * 256;  // floats per parity slot
  const __amdgpu_buffer_rsrc_t pr0 = make_rsrc(a.part, (uint32_t)(slot_f * 4));
  const __amdgpu_buffer_rsrc_t pr1 = make_rsrc(a.part + slot_f, (uint32_t)(slot_f * 4));
  // 1-KiB block of (output tile, row block rb, producer p); dx tiles first, then dh
  auto xblk = [&](int jx, int rb) { return (uint32_t)((((size_t)grp * NXS + jx) * 2 + rb) * M) * 1024u; };
  auto hblk = [&](int s, int rb) {
    return (uint32_t)(((size_t)ng * NXS * 2 * M + (((size_t)grp * NHS + s) * 2 + rb) * M)) * 1024u;
  };
  // P0 unit of this wave: k = 16 w + mem < 2 nFt.  The 2 (nFt - 1) full
  // column tiles come first (k -> row block k / (nFt - 1), tile k % (nFt - 1)),
  // the last tile of each row block last: at F = 129 that tile holds ONE real
  // column, so its lanes with col >= F gather nothing (out-of-range offsets) and
  // the two members that carry a second unit (k = 16, 17 on wave 1) carry a
  // 1-KiB gather instead of a 16-KiB one
  const int pk = M * w + mem, nfull = nFt - 1;
  const bool p0 = pk < 2 * nFt;
  const int prb = !p0 ? 0 : pk < 2 * nfull ? pk / nfull : pk - 2 * nfull;
  const int jx = !p0 ? 0 : pk < 2 * nfull ? pk % nfull : nfull;
  const int prow0 = rowg + 16 * prb;
  // P1 dZ unit of this wave: row block w >> 1, column tile 2 mem + (w & 1)
  // P2: dh half-sum of row block w & 1 over producers 8 (w >> 1) .. + 7; waves 0 / 1 run the cell
  const int crb = w & 1;
  const int crow0 = rowg + 16 * crb;
  const bool cellw = w < 2;
  const int unit = u0 + r;
  float carry[4] = {0.f, 0.f, 0.f, 0.f};
  bool dgv = false;  // DT holds the previous step's dG tile (rows < its batch) for the HX half
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = T - 1 - i;
    const int o = off[t], bs = off[t + 1] - o;
    const int succ_valid = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
    const __amdgpu_buffer_rsrc_t prd = (i & 1) ? pr0 : pr1;  // step t+1's slot
    const __amdgpu_buffer_rsrc_t pw = (i & 1) ? pr1 : pr0;   // this step's slot
    // ---------------- P0: dx_{t+1} tile -> dMU, dLV ----------------
    const int col0 = 16 * jx + r;
    float emu[4], elv[4], eox[4], ey[4], emk[4];
    if (p0) {
      const uint32_t ef = (uint32_t)bs * Fp * 4u;
      const __amdgpu_buffer_rsrc_t rmu = make_rsrc(a.MU + (size_t)o * Fp, ef), rlv = make_rsrc(a.LV + (size_t)o * Fp, ef),
                                   rox = make_rsrc(a.OUT + (size_t)o * Fp, ef),
                                   ryy = make_rsrc(a.Y + (size_t)o * F, (uint32_t)bs * F * 4u);
      const __amdgpu_buffer_rsrc_t rmk =
          make_rsrc(a.xmask ? a.xmask + (size_t)(o + bs) * F : a.Y, a.xmask ? (uint32_t)succ_valid * F * 4u : 0u);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t b = (uint32_t)(prow0 + 4 * q + g);
        const uint32_t of = col0 < F ? (b * Fp + col0) * 4u : 0x80000000u;
        const uint32_t oy = col0 < F ? (b * F + col0) * 4u : 0x80000000u;
        emu[g] = bld(rmu, of);
        elv[g] = bld(rlv, of);
        eox[g] = bld(rox, of);
        ey[g] = bld(ryy, oy);
        emk[g] = a.xmask ? bld(rmk, oy) : 1.f;
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) emu[g] = elv[g] = eox[g] = ey[g] = 0.f, emk[g] = 1.f;
    }
    if (i > 0) gs.wait(3u * i);
    pin(emu), pin(elv), pin(eox), pin(ey), pin(emk);
    PSTAMP(0);
    if (p0) {
      f4 dx = f4zero();
      if (NXS > 0 && i > 0 && prow0 < succ_valid)  // (lanes of padding columns: out-of-range offsets, no traffic)
        sum_partials<M>(prd, col0 < F ? xblk(jx, prb) + (uint32_t)lane * 16u : 0x80000000u, dx, mem % M);
      float dmu[4], dlv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        dmu[g] = dlv[g] = 0.f;
        if (col0 < F) {
          const float dxv = dx[g] * emk[g], mu = emu[g], lv = elv[g];
          const float iv = __expf(-lv), d = ey[g] - mu;
          dmu[g] = dxv + s_em * (-d) * iv;
          dlv[g] = dxv * 0.5f * (eox[g] - mu) + s_em * 0.5f * (1.f - d * d * iv);
        }
      }
      const f4 mq = tp_quad(tb, dmu, lane), lq = tp_quad(tb + TP_FLOATS, dlv, lane);
      if (prow0 < bs) {
        const uint32_t qo = (uint32_t)((prow0 + trow) * Fp + 16 * jx + tcol) * 4u;
        st4(make_rsrc(a.dMU + (size_t)o * Fp, (uint32_t)bs * Fp * 4u), qo, mq, true);
        st4(make_rsrc(a.dLV + (size_t)o * Fp, (uint32_t)bs * Fp * 4u), qo, lq, true);
      }
    }
    gs.publish();
    PSTAMP(1);
    // HX: the dG_{t+1} W_hh half of this step's dh partials needs nothing of
    // this step -- formed in front of the P1 wait from the previous step's dG
    // tile (still in LDS)
    f4 hx[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) hx[j][0] = hx[j][1] = f4zero();
    // blocks k = (row block k >> 1, chunk k & 1) of rows with a successor
    // (rows without one have no dG_{t+1}); block k + 1's split runs between
    // block k's 24 MFMAs (as wave_mma_x6p)
    {
      const int nblk = !dgv ? 0 : rowg + 16 < succ_valid ? 4 : rowg < succ_valid ? 2 : 0;  // uniform
      auto dt_split = [&](int k, bf8 (&v)[3]) {
        const float* ar = DT + (16 * (k >> 1) + r) * W16_DTP + 32 * (k & 1) + 8 * q;
        split8(*reinterpret_cast<const f4*>(ar), *reinterpret_cast<const f4*>(ar + 4), v[0], v[1], v[2]);
      };
      bf8 av[3];
      if (nblk) dt_split(0, av);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k >= nblk) break;
        bf8 nv[3];
        if (k + 1 < 4) dt_split(k + 1, nv);  // (block 2 of a one-row-block step: unused)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          hx[j][k >> 1] = mma_x6(hx[j][k >> 1], av[0], av[1], av[2], Bh[j][k & 1][0], Bh[j][k & 1][1], Bh[j][k & 1][2]);
        if (k + 1 < 4) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
          for (int m = 0; m < 24; ++m) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (k + 1 < 4) av[0] = nv[0], av[1] = nv[1], av[2] = nv[2];
      }
    }
#ifndef ABCD_STAMP_DIAG
    PSTAMP(6);
#endif
    // ---------------- P1: dZ tile -> this member's dh partials ----------------
    // the dZ product on all four waves: wave w -> row block w & 1, the
    // member's dZ column tile w >> 1 (the two waves of a row block load the
    // same dMU / dLV rows; the second one's mostly from this XCD's L2)
    const int zrb = w & 1, zjj = w >> 1;
    float zpre[4];  // the activations of this wave's tile
    {
      const __amdgpu_buffer_rsrc_t rz = make_rsrc(a.Aact + (size_t)o * 2 * Hm, (uint32_t)bs * 2 * Hm * 4u);
      const int zr0 = rowg + 16 * zrb;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        zpre[g] = bld(rz, ((uint32_t)(zr0 + 4 * q + g) * 2 * Hm + 32 * mem + 16 * zjj + r) * 4u);
    }
    gs.wait(3u * i + 1);
    pin(zpre);
    PSTAMP(2);
    {
      const int zr0 = rowg + 16 * zrb;
      f4 acc[1] = {f4zero()};
      if (zr0 < bs) {
        const __amdgpu_buffer_rsrc_t ra = make_rsrc((ismu ? a.dMU : a.dLV) + (size_t)o * Fp, (uint32_t)bs * Fp * 4u);
        const BufKC2x A{ra, ra, (uint32_t)Fp * 4u, (uint32_t)Fp * 4u, ncz, Fp};  // k >= Fp reads 0
        wave_mma_x6<1, NCZ, 4>(acc, A, zr0 + r, B1 + zjj * ncz * 3 * 64, ncz, lane, q);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
        ZT[(16 * zrb + 4 * q + g) * W16_ZTP + 16 * zjj + r] = acc[0][g] * (1.f - zpre[g] * zpre[g]);
    }
#ifdef ABCD_STAMP_DIAG
    PSTAMP(6);  // diagnostics build: dZ tile done (before the barrier)
#endif
    __syncthreads();  // the member's 32 x 32 dZ tile is in LDS
    {  // row block 1's split between row block 0's 24 MFMAs
      const int nrb = rowg + 16 < bs ? 2 : rowg < bs ? 1 : 0;  // uniform
      auto zt_split = [&](int rb, bf8 (&v)[3]) {
        const float* ar = ZT + (16 * rb + r) * W16_ZTP + 8 * q;
        split8(*reinterpret_cast<const f4*>(ar), *reinterpret_cast<const f4*>(ar + 4), v[0], v[1], v[2]);
      };
      bf8 zv[3];
      if (nrb) zt_split(0, zv);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        if (rb >= nrb) break;
        bf8 nv[3];
        if (rb == 0) zt_split(1, nv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f4* bp = W1X + ((4 * w + j) * 3) * 64 + lane;
          const f4 v = mma_x6(hx[j][rb], zv[0], zv[1], zv[2], __builtin_bit_cast(bf8, bp[0]),
                              __builtin_bit_cast(bf8, bp[64]), __builtin_bit_cast(bf8, bp[128]));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), pw,
                                                 hblk(4 * w + j, rb) + (uint32_t)mem * 1024u + (uint32_t)lane * 16u, 0,
                                                 16);
        }
        if (rb == 0) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
          for (int m = 0; m < 24; ++m) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (rb == 0) zv[0] = nv[0], zv[1] = nv[1], zv[2] = nv[2];
      }
    }
#ifdef ABCD_STAMP_DIAG
    PSTAMP(7);  // diagnostics build: fold MFMAs and partial stores issued
#endif
    gs.publish();
    PSTAMP(3);
    // the dZ stash for the weight gradients (plain 16-B stores of the LDS tile,
    // 32 rows x 32 columns = 1 quad per thread) after the publish, so the
    // publish's drain does not wait for them
    {
      const int row = threadIdx.x >> 3, qd = 4 * (threadIdx.x & 7);
      if (rowg + row < bs)
        st4(make_rsrc(a.dZ + (size_t)o * 2 * Hm, (uint32_t)bs * 2 * Hm * 4u),
            (uint32_t)((rowg + row) * 2 * Hm + 32 * mem + qd) * 4u,
            *reinterpret_cast<const f4*>(ZT + row * W16_ZTP + qd), false);
    }
    // ---------------- P2: dh -> cell backward -> dG_t -> dx partials ----------------
    float pg[4][4], pc[4], pcp[4], pdho[4];
    {
      const uint32_t eh = cellw ? (uint32_t)bs * H * 4u : 0u;  // the summing-only waves load nothing
      const __amdgpu_buffer_rsrc_t rgs = make_rsrc(a.Gst + (size_t)o * 4 * H, eh * 4u),
                                   rcs = make_rsrc(a.Cst + (size_t)o * H, GRU ? 0u : eh),
                                   rcp = make_rsrc((GRU ? a.Hprev : a.Cprev) + (size_t)o * H, eh),
                                   rdo = make_rsrc(a.DHO + (size_t)o * H, eh);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t b = (uint32_t)(crow0 + 4 * q + g);
#pragma unroll
        for (int j = 0; j < 4; ++j) pg[g][j] = bld(rgs, (b * 4 * H + j * H + unit) * 4u);
        pc[g] = GRU ? 0.f : bld(rcs, (b * H + unit) * 4u);
        pcp[g] = bld(rcp, (b * H + unit) * 4u);
        pdho[g] = bld(rdo, (b * H + unit) * 4u);
      }
    }
    gs.wait(3u * i + 2);
    pin(pg[0]), pin(pg[1]), pin(pg[2]), pin(pg[3]), pin(pc), pin(pcp), pin(pdho);
    PSTAMP(4);
    // dh of the own 16 units, row block crb: half the producers per wave
    f4 dhr = f4zero();
    if (crow0 < bs)
      sum_partials<M / 2>(pw, hblk(mem, crb) + (uint32_t)(8 * (w >> 1)) * 1024u + (uint32_t)lane * 16u, dhr,
                          mem % (M / 2));
    if (!cellw) DHX[crb * 64 + lane] = dhr;
    __syncthreads();
    if (cellw) dhr += DHX[crb * 64 + lane];
#ifndef ABCD_STAMP_DIAG
    PSTAMP(7);
#endif
    float dgh[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = crow0 + 4 * q + g;
#pragma unroll
      for (int j = 0; j < 4; ++j) dgh[g][j] = 0.f;
      if (!cellw || b >= bs) continue;
      const bool fin = b >= succ_valid;
      if constexpr (GRU) {
        const float dh = dhr[g] + (fin ? 0.f : carry[g]) + pdho[g];
        const float r_ = pg[g][0], z_ = pg[g][1], n_ = pg[g][2], ghn = pg[g][3];
        const float dnp = dh * (1.f - z_) * (1.f - n_ * n_);
        dgh[g][0] = dnp * ghn * r_ * (1.f - r_);
        dgh[g][1] = dh * (pcp[g] - n_) * z_ * (1.f - z_);
        dgh[g][2] = dnp;
        dgh[g][3] = dnp * r_;
        carry[g] = dh * z_;
        if (t == 0) a.DC0[(long)b * H + unit] = dh * z_;
      } else {
        const float dh = dhr[g] + pdho[g];
        const float i_ = pg[g][0], f_ = pg[g][1], g_ = pg[g][2], o_ = pg[g][3];
        const float tc = ftanh(pc[g]);
        const float dc = (fin ? 0.f : carry[g]) + dh * o_ * (1.f - tc * tc);
        dgh[g][0] = dc * g_ * i_ * (1.f - i_);
        dgh[g][1] = dc * pcp[g] * f_ * (1.f - f_);
        dgh[g][2] = dc * i_ * (1.f - g_ * g_);
        dgh[g][3] = dh * tc * o_ * (1.f - o_);
        carry[g] = dc * f_;
        if (t == 0) a.DC0[(long)b * H + unit] = dc * f_;
      }
    }
    if (cellw) {  // the dG tile: rows 16 crb + .., columns [slot][own unit] (rows >= bs hold 0)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) DT[(16 * crb + 4 * q + g) * W16_DTP + 16 * j + r] = dgh[g][j];
    }
    __syncthreads();
    dgv = i + 1 < T;
    // dx partials of this step's dG columns: 2 x NXS tiles dealt over the waves
    if (NXS > 0 && i + 1 < T) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        if (rowg + 16 * rb >= bs) continue;  // uniform
        bf8 av[2][3];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const float* ar = DT + (16 * rb + r) * W16_DTP + 32 * c + 8 * q;
          split8(*reinterpret_cast<const f4*>(ar), *reinterpret_cast<const f4*>(ar + 4), av[c][0], av[c][1], av[c][2]);
        }
#pragma unroll
        for (int jj = 0; jj < (NXS + 3) / 4; ++jj) {
          const int k = 4 * jj + ((w + 2 * rb) & 3);  // tile of this wave (rotated by row block: 5,5,4,4 per wave)
          if (k >= NXS) continue;
          f4 v = f4zero();
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const f4* bp = DXI + ((k * 2 + c) * 3) * 64 + lane;
            v = mma_x6(v, av[c][0], av[c][1], av[c][2], __builtin_bit_cast(bf8, bp[0]), __builtin_bit_cast(bf8, bp[64]),
                       __builtin_bit_cast(bf8, bp[128]));
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), pw,
                                                 xblk(k, rb) + (uint32_t)mem * 1024u + (uint32_t)lane * 16u, 0, 16);
        }
      }
    }
    gs.publish();
    PSTAMP(5);
    // stash for the weight-gradient GEMMs (plain 16-B stores after the publish):
    // 32 rows x 4 slots x 4 quads of own units = 2 quads per thread
    {
      const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.dG + (size_t)o * GH, (uint32_t)bs * GH * 4u);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int k = threadIdx.x + 256 * k2, row = k >> 4, slot = (k >> 2) & 3, qd = 4 * (k & 3);
        if (rowg + row >= bs) continue;
        const f4 v = *reinterpret_cast<const f4*>(DT + row * W16_DTP + 16 * slot + qd);
        const uint32_t so = (uint32_t)((rowg + row) * GH + u0 + qd) * 4u;
        if constexpr (GRU) {  // dGX = (dr, dz, dn), dGH = (dr, dz, dn r)
          const __amdgpu_buffer_rsrc_t rh = make_rsrc(a.dGH + (size_t)o * GH, (uint32_t)bs * GH * 4u);
          if (slot < 3) st4(rg, so + (uint32_t)(slot * H) * 4u, v, false);
          if (slot != 2) st4(rh, so + (uint32_t)((slot == 3 ? 2 : slot) * H) * 4u, v, false);
        } else {
          st4(rg, so + (uint32_t)(slot * H) * 4u, v, false);
        }
      }
    }
  }
  // ---------------- dh_{-1} = dG_0 W_hh -> dhid (feature2hidden's output gradient) ----------------
  // one more split-K round after the loop: every member's partial of dG_0[:,
  // own 64] W_hh[own 64, all units] (DT still holds dG_0) into the next
  // parity slot (its last readers, step T - 1's P0, are all past), a hand-off,
  // and the member's 16 units summed over the 16 producers: the three launches
  // after the kernel (dH0 GEMM, its slab reduction, the dhid assembly) go away
  if (a.dhid) {
    const __amdgpu_buffer_rsrc_t pw = (T & 1) ? pr1 : pr0;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      if (rowg + 16 * rb >= a.B) continue;  // uniform
      f4 h0[4] = {f4zero(), f4zero(), f4zero(), f4zero()};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float* ar = DT + (16 * rb + r) * W16_DTP + 32 * c + 8 * q;
        bf8 a0, a1, a2;
        split8(*reinterpret_cast<const f4*>(ar), *reinterpret_cast<const f4*>(ar + 4), a0, a1, a2);
#pragma unroll
        for (int j = 0; j < 4; ++j) h0[j] = mma_x6(h0[j], a0, a1, a2, Bh[j][c][0], Bh[j][c][1], Bh[j][c][2]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, h0[j]), pw,
                                               hblk(4 * w + j, rb) + (uint32_t)mem * 1024u + (uint32_t)lane * 16u, 0, 16);
    }
    gs.publish();
    gs.wait(3u * T + 1);
    f4 dhr = f4zero();
    if (crow0 < a.B)
      sum_partials<M / 2>(pw, hblk(mem, crb) + (uint32_t)(8 * (w >> 1)) * 1024u + (uint32_t)lane * 16u, dhr,
                          mem % (M / 2));
    if (!cellw) DHX[crb * 64 + lane] = dhr;
    __syncthreads();
    if (cellw) {
      dhr += DHX[crb * 64 + lane];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b = crow0 + 4 * q + g;
        if (b >= a.B) continue;
        if constexpr (GRU) {
          a.dhid[(long)b * H + unit] = dhr[g] + carry[g];  // carry = dh_0 z at t = 0
        } else {
          a.dhid[(long)b * 2 * H + 2 * unit] = dhr[g];
          a.dhid[(long)b * 2 * H + 2 * unit + 1] = carry[g];  // carry = dc_0 f at t = 0
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// enc_bwd_w8 (round 4): enc_bwd_sk with HALF the exchange, as dec_bwd_w16
// does for the decoder.  A group is a 32-ROW tile of one direction with 8
// members owning 32 units each (K = G x 32 gate columns: one 32-deep chunk
// per gate, so a GRU member multiplies 3 chunks instead of 2 padded ones);
// per step a member writes its partial of dh_rec for all 256 units of its 32
// rows (32 KiB instead of 64) and a consumer sums 8 partials instead of 16.
// The waves split the output columns: wave w forms the partials of units
// 64w .. 64w + 63 (4 subtiles x both 16-row blocks x G chunks = 24 G MFMAs
// per subtile pair, 192 per wave for the LSTM as in enc_bwd_sk) and keeps
// the first two chunks of its quarter of the W_hh image in registers (96
// VGPRs), the rest in LDS.  Cell backward: wave (rb, uh) runs rows 16 rb ..
// of units 16 uh .. of the member's 32.  Reference: the BPTT of nn.LSTM /
// nn.GRU, model.py:53,60-66.
// ---------------------------------------------------------------------------
constexpr int W8_ROWS = 32;   // rows per group
constexpr int W8_M = 8;       // members per group (32 units each)
constexpr int W8_DTP = 132;   // pitch (floats) of the member's 32 x 4*32 dG tile in LDS
// The encoder BPTT shares its CUs with the decoder's weight-gradient GEMMs
// (side stream): its waves win the issue arbitration (s_setprio; the GEMM
// waves stay at 0).  Same-box A/B at c2: enc_bwd 1.70 -> 1.66 ms, step 8.676
// -> 8.652 ms (three alternating pairs, each faster).
#ifndef ABCD_BWD_PRIO
#define ABCD_BWD_PRIO 3
#endif
template <int G>
__global__ __launch_bounds__(256) void enc_bwd_w8(PBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) f4 smem[];
  bptt_resident(a.started);
  if (ABCD_BWD_PRIO) __builtin_amdgcn_s_setprio(ABCD_BWD_PRIO);
  constexpr int H = 256, GH = G * H, M = W8_M, NSUB = H / 16;
  constexpr int NC = G;                     // 32-deep chunks = gates
  constexpr int NCR = 2, NCL = NC - NCR;    // chunks of the image in registers / in LDS
  const int T = a.T, ng = a.nd * a.nrt;     // a.nrt: 32-row tiles per direction (the launcher's count)
  const Role role = assign_role(ng, M);
  const int grp = role.grp, mem = role.mem;
  const int dir = grp / a.nrt, rt = grp % a.nrt;
  const PBwdDir& D = a.d[dir];
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int u0 = mem * 32;
  const int rb = w & 1, uh = w >> 1;        // this wave's cell tile: rows 16 rb .., units u0 + 16 uh ..
  const int unit = u0 + 16 * uh + r;
  const int rowg = rt * W8_ROWS, row0 = rowg + 16 * rb;
  unsigned* cnt = a.sync + grp * PERSIST_SYNC_STRIDE;
  // LDS: [wave][subtile j][chunk c - NCR][plane][64] | dG tile [32][132] | wave transposes
  f4* BL = smem;
  float* DT = reinterpret_cast<float*>(BL + 4 * 4 * (NCL > 0 ? NCL : 1) * 3 * 64);
  float* tb = DT + W8_ROWS * W8_DTP + w * TP_FLOATS;
  const int trow = lane >> 2, tcol = 4 * (lane & 3);
  // image of output subtile s = 4w + j, chunk c (gate c), lane (rr = r, qq = q):
  // rows k = 32c + 8q + 0..7 = W_hh rows c H + u0 + 8q + 0..7, column unit 16 s + r
  bf8 Br[4][NCR][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float* src = D.WhhT + (long)(16 * (4 * w + j) + r) * GH + c * H + u0 + 8 * q;
      bf8 h, m, l;
      split8(*reinterpret_cast<const f4*>(src), *reinterpret_cast<const f4*>(src + 4), h, m, l);
      if (c < NCR) {
        Br[j][c][0] = h, Br[j][c][1] = m, Br[j][c][2] = l;
      } else {
        f4* d = BL + (((w * 4 + j) * NCL + (c - NCR)) * 3) * 64 + lane;
        d[0] = __builtin_bit_cast(f4, h);
        d[64] = __builtin_bit_cast(f4, m);
        d[128] = __builtin_bit_cast(f4, l);
      }
    }
  __syncthreads();
  const size_t slot_f = (size_t)ng * NSUB * 2 * M * 256;  // floats per parity slot
  // 1-KiB block of (group, consumer subtile s, row block b2, producer)
  auto pblk = [&](int s, int b2) { return (uint32_t)((((size_t)grp * NSUB + s) * 2 + b2) * M) * 1024u; };
  float carry[4] = {0.f, 0.f, 0.f, 0.f};
  const int* off = a.off;
  for (int i = 0; i < T; ++i) {
    const int t = D.rev ? i : T - 1 - i;
    const int o = off[t], bs = off[t + 1] - o;
    int succ_valid, prev_valid;
    if (!D.rev) {
      succ_valid = t + 1 < T ? off[t + 2] - off[t + 1] : 0;
      prev_valid = t == 0 ? 0 : bs;
    } else {
      succ_valid = t >= 1 ? bs : 0;
      prev_valid = t == T - 1 ? 0 : off[t + 2] - off[t + 1];
    }
    PSTAMP(0);
    // cell operands: branch-free loads before the wait, pinned after it (bld)
    float pg[4][4], pc[4], pcp[4], pdh[4], pdl[4], pdc[4];
    {
      const uint32_t eh = (uint32_t)bs * H * 4u;
      const __amdgpu_buffer_rsrc_t rgs = make_rsrc(D.Gst + (size_t)o * 4 * H, eh * 4u),
                                   rcs = make_rsrc(D.Cst + (size_t)o * H, G == 4 ? eh : 0u),
                                   rcp = make_rsrc((G == 4 ? D.Cprev : D.Hprev) + (size_t)o * H,
                                                   (uint32_t)prev_valid * H * 4u),
                                   rdx = make_rsrc(D.DHX ? D.DHX + (size_t)o * D.lddhx : D.Gst,
                                                   D.DHX ? (uint32_t)bs * D.lddhx * 4u : 0u),
                                   rdl = make_rsrc(D.dlast ? D.dlast : D.Gst, D.dlast ? (uint32_t)bs * D.ldl * 4u : 0u);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t b = (uint32_t)(row0 + 4 * q + g);
        const bool fin = (int)b >= succ_valid;
#pragma unroll
        for (int j = 0; j < 4; ++j) pg[g][j] = bld(rgs, (b * 4 * H + j * H + unit) * 4u);
        pc[g] = G == 4 ? bld(rcs, (b * H + unit) * 4u) : 0.f;
        pcp[g] = bld(rcp, (b * H + unit) * 4u);
        pdh[g] = bld(rdx, (b * D.lddhx + unit) * 4u);
        // the last step's gradient enters rows that have no successor (rows >= bs read 0)
        pdl[g] = bld(rdl, fin ? (b * D.ldl + D.hcol + unit) * 4u : 0x80000000u);
        pdc[g] = (G == 4 && D.ccol >= 0) ? bld(rdl, fin ? (b * D.ldl + D.ccol + unit) * 4u : 0x80000000u) : 0.f;
      }
    }
    f4 dhr = f4zero();
    if (i > 0) group_wait(cnt, (unsigned)(M * i));
    pin(pg[0]), pin(pg[1]), pin(pg[2]), pin(pg[3]), pin(pc), pin(pcp), pin(pdh), pin(pdl), pin(pdc);
#pragma unroll
    for (int g = 0; g < 4; ++g) pdh[g] += pdl[g];
    if (i > 0 && row0 < succ_valid) {
      const __amdgpu_buffer_rsrc_t pr = make_rsrc(a.part + (size_t)(i & 1) * slot_f, (uint32_t)(slot_f * 4));
      sum_partials<M>(pr, pblk(2 * mem + uh, rb) + (uint32_t)lane * 16u, dhr, mem);
    }
    PSTAMP(1);
    // cell backward -> dG (LSTM: dGX == dGH; GRU: dGH = [dr, dz, dn*r], dGX gate 2 = dn)
    float dgh[4][4], dgx[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = row0 + 4 * q + g;
#pragma unroll
      for (int j = 0; j < 4; ++j) dgh[g][j] = dgx[g][j] = 0.f;
      if (b >= bs) continue;
      const bool fin = b >= succ_valid;
      float dh = (fin ? 0.f : dhr[g]) + pdh[g];
      if (G == 4) {
        const float i_ = pg[g][0], f_ = pg[g][1], g_ = pg[g][2], o_ = pg[g][3];
        const float tc = ftanh(pc[g]);
        const float dc = (fin ? pdc[g] : carry[g]) + dh * o_ * (1.f - tc * tc);
        dgx[g][0] = dc * g_ * i_ * (1.f - i_);
        dgx[g][1] = dc * pcp[g] * f_ * (1.f - f_);
        dgx[g][2] = dc * i_ * (1.f - g_ * g_);
        dgx[g][3] = dh * tc * o_ * (1.f - o_);
#pragma unroll
        for (int j = 0; j < 4; ++j) dgh[g][j] = dgx[g][j];
        carry[g] = dc * f_;
      } else {
        if (!fin) dh += carry[g];
        const float r_ = pg[g][0], z_ = pg[g][1], n_ = pg[g][2], ghn = pg[g][3];
        const float hp = pcp[g];
        const float dnp = dh * (1.f - z_) * (1.f - n_ * n_);
        const float dzp = dh * (hp - n_) * z_ * (1.f - z_);
        const float drp = dnp * ghn * r_ * (1.f - r_);
        dgx[g][0] = drp; dgx[g][1] = dzp; dgx[g][2] = dnp;
        dgh[g][0] = drp; dgh[g][1] = dzp; dgh[g][2] = dnp * r_;
        carry[g] = dh * z_;
      }
    }
    PSTAMP(2);
    // the member's dG tile: rows 16 rb + .., columns [gate][32 own units] (rows >= bs hold 0)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < G; ++j) DT[(16 * rb + 4 * q + g) * W8_DTP + 32 * j + 16 * uh + r] = dgh[g][j];
    // partials for the next step from this step's own dG columns
    if (i + 1 < T) {
      __syncthreads();  // every wave's dG rows are in the member's tile
      const __amdgpu_buffer_rsrc_t pw = make_rsrc(a.part + (size_t)((i + 1) & 1) * slot_f, (uint32_t)(slot_f * 4));
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2) {
        if (rowg + 16 * b2 >= bs) break;  // uniform: row blocks past the step's batch
        bf8 av[NC][3];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const float* ar = DT + (16 * b2 + r) * W8_DTP + 32 * c + 8 * q;
          split8(*reinterpret_cast<const f4*>(ar), *reinterpret_cast<const f4*>(ar + 4), av[c][0], av[c][1], av[c][2]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f4 acc = f4zero();
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            if (c < NCR) {
              acc = mma_x6(acc, av[c][0], av[c][1], av[c][2], Br[j][c < NCR ? c : 0][0], Br[j][c < NCR ? c : 0][1],
                           Br[j][c < NCR ? c : 0][2]);
            } else {
              const f4* bp = BL + (((w * 4 + j) * NCL + (c - NCR)) * 3) * 64 + lane;
              acc = mma_x6(acc, av[c][0], av[c][1], av[c][2], __builtin_bit_cast(bf8, bp[0]),
                           __builtin_bit_cast(bf8, bp[64]), __builtin_bit_cast(bf8, bp[128]));
            }
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc), pw,
                                                 pblk(4 * w + j, b2) + (uint32_t)mem * 1024u + (uint32_t)lane * 16u,
                                                 0, 16);
        }
      }
    }
    PSTAMP(3);
    group_publish(cnt);
    // stashes for the weight-gradient GEMMs after the launch (plain 16-B
    // stores after the publish, read back from the dG tile: 32 rows x G gates
    // x 8 quads of own units).  LSTM: dGX = dGH = dG.  GRU: the tile is dGH =
    // (dr, dz, dn r); dGX = (dr, dz, dn) takes gate 2 from a transpose of dn.
    {
      const __amdgpu_buffer_rsrc_t rx = make_rsrc(D.dGX + (size_t)o * GH, (uint32_t)bs * GH * 4u);
      const __amdgpu_buffer_rsrc_t rh = make_rsrc(D.dGH + (size_t)o * GH, (uint32_t)bs * GH * 4u);
#pragma unroll
      for (int k2 = 0; k2 < G; ++k2) {
        const int k = threadIdx.x + 256 * k2, row = k / (8 * G), gate = (k >> 3) % G, qd = 4 * (k & 7);
        if (rowg + row >= bs) continue;
        const f4 v = *reinterpret_cast<const f4*>(DT + row * W8_DTP + 32 * gate + qd);
        const uint32_t so = (uint32_t)((rowg + row) * GH + gate * H + u0 + qd) * 4u;
        if (G == 3) {
          st4(rh, so, v, false);
          if (gate < 2) st4(rx, so, v, false);
        } else {
          st4(rx, so, v, false);
        }
      }
      if (G == 3) {
        const float dn[4] = {dgx[0][2], dgx[1][2], dgx[2][2], dgx[3][2]};
        const f4 nq = tp_quad(tb, dn, lane);
        if (row0 < bs) st4(rx, (uint32_t)((row0 + trow) * GH + 2 * H + u0 + 16 * uh + tcol) * 4u, nq, false);
      }
    }
    PSTAMP(4);
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool persist_enabled() {
  const char* v = getenv("ABCD_PERSIST");  // read per call: tests flip it in-process
  return !(v && v[0] == '0');
}

// Pinned ring of offset tables.  upload_offsets copies one to the device with
// hipMemcpyAsync.  stage_offsets only fills a slot and leaves the copy pending
// (per host thread): the next zero_sync on the same stream folds it into the
// counter-reset kernel (one launch instead of a copy and two fills before
// each persistent kernel); flush_offsets issues a pending copy that no reset
// took (the per-step fallback paths).
namespace {
// Slots are guarded in groups of OFF_GRP: an event is recorded on each stream
// that used a group only after the group's last use, and a slot is refilled
// only after its group's events completed.  An event per use put a barrier
// packet between every counter reset and its persistent kernel: 7-12 us of
// idle queue before each of the four launches of a step (rocprofv3 trace,
// same-box A/B: -42 us per c2 step without them).
constexpr int OFF_NSLOT = 32;
constexpr int OFF_GRP = 8;
constexpr int OFF_NGRP = OFF_NSLOT / OFF_GRP;
constexpr int OFF_GSTREAMS = 4;  // distinct streams tracked per group (more: record at once)
constexpr size_t OFF_SLOT = 64 * 1024;
constexpr int OFF_MAXDEV = 16;
std::mutex g_off_mu;
// one ring per device: a group's events are recorded on streams of that device only
struct OffGroup {
  hipStream_t st[OFF_GSTREAMS];
  hipEvent_t ev[OFF_GSTREAMS + 1];  // the last one: an early record (more streams than tracked)
  int nst = 0;
  bool early = false;      // ev[OFF_GSTREAMS] recorded on a stream beyond the tracked ones
  bool recorded = false;   // ev[0 .. nst) recorded after the group's last use
};
struct OffRing {
  char* ring = nullptr;
  OffGroup g[OFF_NGRP];
  int next = 0;
};
OffRing g_rings[OFF_MAXDEV];
struct PendingOff {
  hipStream_t s;
  int* dst;
  const int* src;  // pinned host slot
  int n, slot, dev;
  bool on;
};
thread_local PendingOff g_pend{};

int off_slot(const std::vector<int>& off, int* slot_out, const int** src, int* dev_out) {
  const size_t bytes = off.size() * sizeof(int);
  if (bytes > OFF_SLOT) return (int)hipErrorInvalidValue;
  int dev = 0;
  ABCD_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= OFF_MAXDEV) return (int)hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(g_off_mu);
  OffRing& R = g_rings[dev];
  if (!R.ring) {
    ABCD_TRY(hipHostMalloc((void**)&R.ring, OFF_SLOT * OFF_NSLOT, hipHostMallocDefault));
    for (auto& G : R.g)
      for (auto& e : G.ev) ABCD_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const int k = R.next;
  R.next = (R.next + 1) % OFF_NSLOT;
  OffGroup& G = R.g[k / OFF_GRP];
  if (k % OFF_GRP == 0) {  // entering a group: its previous round of reads is done
    if (G.recorded)
      for (int i = 0; i < G.nst; ++i) ABCD_TRY(hipEventSynchronize(G.ev[i]));
    if (G.early) ABCD_TRY(hipEventSynchronize(G.ev[OFF_GSTREAMS]));
    G.nst = 0;
    G.early = G.recorded = false;
  }
  std::copy(off.begin(), off.end(), (int*)(R.ring + k * OFF_SLOT));
  *slot_out = k;
  *dev_out = dev;
  *src = (const int*)(R.ring + k * OFF_SLOT);
  return 0;
}
int off_release(hipStream_t s, int dev, int k) {  // after the op that reads slot k is queued on s
  OffRing& R = g_rings[dev];
  std::lock_guard<std::mutex> lk(g_off_mu);
  OffGroup& G = R.g[k / OFF_GRP];
  int i = 0;
  while (i < G.nst && G.st[i] != s) ++i;
  if (i == G.nst) {
    if (G.nst < OFF_GSTREAMS) {
      G.st[G.nst++] = s;
    } else {  // untracked stream: guard this use at once (sync'ed with the group)
      if (G.early) ABCD_TRY(hipEventSynchronize(G.ev[OFF_GSTREAMS]));
      ABCD_TRY(hipEventRecord(G.ev[OFF_GSTREAMS], s));
      G.early = true;
    }
  }
  if (k % OFF_GRP == OFF_GRP - 1) {  // the group's last use: one event per stream that used it
    for (int j = 0; j < G.nst; ++j) ABCD_TRY(hipEventRecord(G.ev[j], G.st[j]));
    G.recorded = true;
  }
  return 0;
}
}  // namespace

int flush_offsets() {
  if (!g_pend.on) return 0;
  g_pend.on = false;
  ABCD_TRY(hipMemcpyAsync(g_pend.dst, g_pend.src, (size_t)g_pend.n * sizeof(int), hipMemcpyHostToDevice, g_pend.s));
  return off_release(g_pend.s, g_pend.dev, g_pend.slot);
}

// a table staged by a call that returned early (error path) is dropped, never
// copied: its destination workspace may be gone.  Its slot is still released,
// so a group whose last slot is dropped records its events like any other
// (otherwise the group's next lap would refill slots without waiting for the
// reads of the earlier ones still queued on the GPU)
static void drop_stale_offsets() {
  if (!g_pend.on) return;
  g_pend.on = false;
  (void)off_release(g_pend.s, g_pend.dev, g_pend.slot);
}

int upload_offsets(hipStream_t s, const std::vector<int>& off, int* dst) {
  drop_stale_offsets();
  int k, dev;
  const int* src;
  ABCD_TRY((hipError_t)off_slot(off, &k, &src, &dev));
  ABCD_TRY(hipMemcpyAsync(dst, src, off.size() * sizeof(int), hipMemcpyHostToDevice, s));
  return off_release(s, dev, k);
}

int stage_offsets(hipStream_t s, const std::vector<int>& off, int* dst) {
  drop_stale_offsets();
  int k, dev;
  const int* src;
  ABCD_TRY((hipError_t)off_slot(off, &k, &src, &dev));
  g_pend = PendingOff{s, dst, src, (int)off.size(), k, dev, true};
  return 0;
}

template <class K>
static int fits_resident(K kernel, int grid, size_t lds, bool* ok) {
  *ok = false;
  if (lds > 160 * 1024) return 0;
  // (kernel, LDS bytes, device) -> resident workgroups on the chip; the
  // attribute and occupancy queries run once per key, not once per launch
  struct Key {
    const void* k;
    size_t lds;
    int dev;
  };
  static std::mutex mu;
  static std::vector<std::pair<Key, long>> cache;
  int dev = 0;
  ABCD_TRY(hipGetDevice(&dev));
  long cap = -1;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (const auto& e : cache)
      if (e.first.k == (const void*)kernel && e.first.lds == lds && e.first.dev == dev) cap = e.second;
  }
  if (cap < 0) {
    int cus = 0, per = 0;
    ABCD_TRY(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    ABCD_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    ABCD_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kernel, 256, lds));
    cap = (long)cus * per;
    std::lock_guard<std::mutex> lk(mu);
    cache.push_back({Key{(const void*)kernel, lds, dev}, cap});
  }
  *ok = cap > 0 && (long)grid <= cap;
  return 0;
}

// One launch before each persistent kernel: every sync word zeroed and, when
// a staged offset table is pending on s, that table read from its pinned host
// slot into device memory.
__global__ __launch_bounds__(256) void persist_reset(unsigned* sync, long nwords, const int* off_src,
                                                     int* off_dst, int noff) {
  const long i0 = (long)blockIdx.x * 256 + threadIdx.x, stride = (long)gridDim.x * 256;
  if (i0 == 0) __hip_atomic_store(&g_persist_abort, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (long i = i0; i < nwords / 4; i += stride) {
    uint4 z = make_uint4(0u, 0u, 0u, 0u);
    reinterpret_cast<uint4*>(sync)[i] = z;
  }
  for (long i = i0; i < noff; i += stride) off_dst[i] = off_src[i];
}

// ABCD_SPIN_LIMIT=<polls> (debug/tests): shrink the hand-off spin bound so a
// wait times out at once; the device word is only rewritten when the value
// changes (never in a default run)
static int sync_spin_limit(hipStream_t s) {
  static unsigned cur = 1u << 22, staged;
  const char* v = getenv("ABCD_SPIN_LIMIT");
  const unsigned want = (v && v[0]) ? (unsigned)strtoul(v, nullptr, 10) : (1u << 22);
  if (want == cur) return 0;
  staged = want;
  ABCD_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_spin_limit), &staged, sizeof(staged), 0, hipMemcpyHostToDevice, s));
  ABCD_TRY(hipStreamSynchronize(s));
  cur = want;
  return 0;
}

static int zero_sync_impl(hipStream_t s, unsigned* sync, int ngroups) {
  ABCD_TRY((hipError_t)sync_spin_limit(s));
  const long nwords = (long)(2 * ngroups + PERSIST_REG_LINES + PERSIST_FLAG_LINES * ngroups) * PERSIST_SYNC_STRIDE;
  const bool take = g_pend.on && g_pend.s == s;
  const int* src = nullptr;
  if (take) ABCD_TRY(hipHostGetDevicePointer((void**)&src, (void*)g_pend.src, 0));
  const int blocks = (int)std::min<long>(64, std::max<long>(1, (nwords / 4 + 255) / 256));
  persist_reset<<<blocks, 256, 0, s>>>(sync, nwords, src, take ? g_pend.dst : nullptr, take ? g_pend.n : 0);
  ABCD_TRY(hipGetLastError());
  if (take) {
    g_pend.on = false;
    ABCD_TRY((hipError_t)off_release(s, g_pend.dev, g_pend.slot));
  }
  return 0;
}
static hipError_t zero_sync(hipStream_t s, unsigned* sync, int ngroups) {
  return (hipError_t)zero_sync_impl(s, sync, ngroups);
}

// the side-stream gate's bookkeeping: encoder BPTT launches per device (the
// device counts the same launches once all their workgroups have started) and
// the gate's target.  The switch and the target are per host thread: the
// training step turns the switch on around its own decoder backward, so
// another thread's calls never queue a gate they did not ask for.
static unsigned h_bptt_launches[64];
static thread_local bool g_side_gate = false;
static thread_local bool tl_gate_armed[64];     // a deferred decoder backward waits for the next BPTT launch
static thread_local unsigned tl_gate_target[64];  // that launch's count (0: none was launched)
static int cur_dev() {
  int dev = 0;
  return hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 ? dev : 0;
}
// an encoder BPTT launch: its residency line (the first registry line, zeroed
// by the reset in front of it) and the host launch count
static void bptt_launch(PBwdArgs& b, int ngroups) {
  b.started = b.sync + (size_t)2 * ngroups * PERSIST_SYNC_STRIDE;
  const int dev = cur_dev();
  const unsigned n = ++h_bptt_launches[dev];
  if (tl_gate_armed[dev]) {
    tl_gate_target[dev] = n;
    tl_gate_armed[dev] = false;
  }
}
// ABCD_SIDE_GATE=0 keeps it off whatever the switch says (same-box A/B)
bool side_gate_enabled() {
  const char* v = getenv("ABCD_SIDE_GATE");  // read per call (tests flip it in-process)
  const bool env_off = v && v[0] == '0';
  return g_side_gate && !env_off && persist_enabled();  // (no persistent BPTT: nothing to wait for)
}
void side_gate_arm() {
  const int dev = cur_dev();
  tl_gate_armed[dev] = side_gate_enabled();
  tl_gate_target[dev] = 0;
}
void side_gate_disarm() {
  const int dev = cur_dev();
  tl_gate_armed[dev] = false;
  tl_gate_target[dev] = 0;
}
// queued on the side stream AFTER the encoder backward: waits only if that
// backward launched a persistent BPTT since the arming decoder backward (a
// per-step encoder backward, or none, leaves nothing to wait for)
int side_gate(hipStream_t sw) {
  const int dev = cur_dev();
  const unsigned target = tl_gate_target[dev];
  side_gate_disarm();
  if (!target) return 0;
  side_gate_kernel<<<1, 64, 0, sw>>>(target);
  return (int)hipGetLastError();
}


// ring depth: the largest of 16 / 4 / 1 dividing the chunk count
static int ring_depth(int nch) { return nch % 16 == 0 ? 16 : (nch % 4 == 0 ? 4 : 1); }

// x6 (split-fp32 on the bf16 matrix cores) for the compiled chunk counts
static bool x6_enabled(int K) { return K == 64 || K == 128 || K == 256; }

template <int G, int PD, int X6>
static int launch_fwd(hipStream_t s, const PFwdArgs& a, bool* launched) {
  const int grid = a.nd * a.nrt * (a.H / 16);
  const size_t lds = (size_t)G * 16 * a.H * (X6 ? 6 : 4) + (size_t)4 * TP_FLOATS * 4;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(enc_fwd_persist<G, PD, X6>, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY(zero_sync(s, a.sync, a.nd * a.nrt));
  PFwdArgs b = a;
  b.prof = (g_prof_mask & 1) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_ENC_FWD);
    enc_fwd_persist<G, PD, X6><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_ENC_FWD, "enc_fwd_persist<%d,%d,%d> grid %d", G, PD, X6, grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}
template <int G, int PD>
static int launch_bwd(hipStream_t s, const PBwdArgs& a, bool* launched) {
  const int grid = a.nd * a.nrt * (a.H / 16);
  const size_t lds = (size_t)16 * G * a.H * 4;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(enc_bwd_persist<G, PD>, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY(zero_sync(s, a.sync, a.nd * a.nrt));
  PBwdArgs b = a;
  b.prof = (g_prof_mask & 2) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_ENC_BWD);
    bptt_launch(b, a.nd * a.nrt);
    enc_bwd_persist<G, PD><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_ENC_BWD, "enc_bwd_persist<%d,%d> grid %d", G, PD, grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}

template <int G>
static int launch_fwd_x6(hipStream_t s, const PFwdArgs& a, bool* launched) {
  if (a.H == 64) return launch_fwd<G, 16, 2>(s, a, launched);
  if (a.H == 128) return launch_fwd<G, 16, 4>(s, a, launched);
  return launch_fwd<G, 16, 8>(s, a, launched);
}

int persist_encoder_fwd(hipStream_t s, int G, const PFwdArgs& a, bool* launched) {
  *launched = false;
  if (!persist_enabled()) return 0;
  if (x6_enabled(a.H)) return G == 4 ? launch_fwd_x6<4>(s, a, launched) : launch_fwd_x6<3>(s, a, launched);
  const int pd = ring_depth(a.H / 16);
  if (G == 4) {
    if (pd == 16) return launch_fwd<4, 16, 0>(s, a, launched);
    if (pd == 4) return launch_fwd<4, 4, 0>(s, a, launched);
    return launch_fwd<4, 1, 0>(s, a, launched);
  }
  if (pd == 16) return launch_fwd<3, 16, 0>(s, a, launched);
  if (pd == 4) return launch_fwd<3, 4, 0>(s, a, launched);
  return launch_fwd<3, 1, 0>(s, a, launched);
}

template <int G, int NSUB>
static int launch_bwd_sk(hipStream_t s, const PBwdArgs& a, bool* launched) {
  const int grid = a.nd * a.nrt * NSUB;
  const size_t lds = (size_t)NSUB * 2 * 3 * 64 * 16 + (size_t)4 * 16 * SK_PITCH * 4 + (size_t)4 * TP_FLOATS * 4;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(enc_bwd_sk<G, NSUB>, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY(zero_sync(s, a.sync, a.nd * a.nrt));
  PBwdArgs b = a;
  b.prof = (g_prof_mask & 2) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_ENC_BWD);
    bptt_launch(b, a.nd * a.nrt);
    enc_bwd_sk<G, NSUB><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_ENC_BWD, "enc_bwd_sk<%d,%d> grid %d", G, NSUB, grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}


// enc_bwd_w8 at H = 256 (32-row groups of 8 members: half the split-K
// exchange of the 64-row enc_bwd_sk<G, 16>, which it replaced): same-box A/B
// at c2, enc_bwd 1.90 / 1.89 -> 1.60 / 1.59 ms per launch, step 9.51 / 9.53 ->
// 9.26 / 9.23 ms; c5gru 5.10 / 5.21 -> 3.98 / 4.02 ms
template <int G>
static int launch_bwd_w8(hipStream_t s, const PBwdArgs& a, bool* launched) {
  const int nrt = cdiv(a.B, W8_ROWS);
  const int grid = a.nd * nrt * W8_M;
  constexpr int NCL = G - 2;
  const size_t lds = (size_t)4 * 4 * NCL * 3 * 64 * 16 + (size_t)W8_ROWS * W8_DTP * 4 + (size_t)4 * TP_FLOATS * 4;
  if (a.B <= 0) return 0;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(enc_bwd_w8<G>, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY(zero_sync(s, a.sync, a.nd * nrt));
  PBwdArgs b = a;
  b.nrt = nrt;
  b.prof = (g_prof_mask & 2) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_ENC_BWD);
    bptt_launch(b, a.nd * nrt);
    enc_bwd_w8<G><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_ENC_BWD, "enc_bwd_w8<%d> grid %d", G, grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}

int persist_encoder_bwd(hipStream_t s, int G, const PBwdArgs& a, bool* launched) {
  *launched = false;
  if (!persist_enabled()) return 0;
  if (a.part && a.H == 256) {
    const int rc = G == 4 ? launch_bwd_w8<4>(s, a, launched) : launch_bwd_w8<3>(s, a, launched);
    if (rc || *launched) return rc;
  } else if (a.part && (a.H == 64 || a.H == 128)) {  // split-K in 64-row groups of H / 16 members
    if (G == 4) return a.H == 64 ? launch_bwd_sk<4, 4>(s, a, launched) : launch_bwd_sk<4, 8>(s, a, launched);
    return a.H == 64 ? launch_bwd_sk<3, 4>(s, a, launched) : launch_bwd_sk<3, 8>(s, a, launched);
  }
  if (x6_enabled(a.H)) return 0;  // H = 256 that enc_bwd_w8 cannot hold resident: the per-step kernels
  const int pd = ring_depth(G * a.H / 16);
  if (G == 4) {
    if (pd == 16) return launch_bwd<4, 16>(s, a, launched);
    if (pd == 4) return launch_bwd<4, 4>(s, a, launched);
    return launch_bwd<4, 1>(s, a, launched);
  }
  if (pd == 16) return launch_bwd<3, 16>(s, a, launched);
  if (pd == 4) return launch_bwd<3, 4>(s, a, launched);
  return launch_bwd<3, 1>(s, a, launched);
}


// eps_fill for a form that does not draw the noise itself: the whole block up
// front (abcd_fill_normal: the same philox_normal(seed, offset + i) values)
static int prefill_eps(hipStream_t s, const PDecFwdArgs& a) {
  if (!a.eps_fill) return 0;
  return abcd_fill_normal(const_cast<float*>(a.eps), a.nfill, a.seed, a.offset, s);
}
template <int NCC>
static int launch_dec_fwd(hipStream_t s, const PDecFwdArgs& a, bool* launched) {
  const int M = a.H / 8, nchx = a.feedback ? a.Fp / 16 : 0, nchh = a.H / 16, nchm = a.Hm / 16;
  const int n1 = cdiv(2 * a.Hm / 16, M), n2 = cdiv(a.Fp / 16, M);
  const size_t cell = NCC ? (size_t)2 * NCC * 3 : (size_t)2 * (nchx + nchh);
  const size_t lds = (size_t)64 * 16 * (cell + n1 * nchh + 2 * n2 * nchm);
  const int grid = a.nrt * M;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(dec_fwd_persist<NCC>, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY((hipError_t)prefill_eps(s, a));
  ABCD_TRY(zero_sync(s, a.sync, a.nrt));
  PDecFwdArgs b = a;
  b.eps_fill = 0;
  b.flags = 1;  // per-member flags (the group-counter form measured slower)
  b.prof = (g_prof_mask & 4) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_DEC_FWD);
    dec_fwd_persist<NCC><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_DEC_FWD, "dec_fwd_persist<%d> grid %d", NCC, grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}

template <int NCC, int NH32, int NM32, bool GRU, bool HPRE>
static int launch_dec_fwd_x6_k(hipStream_t s, const PDecFwdArgs& a, bool* launched) {
  const int M = a.H / 8;
  const size_t lds = (size_t)64 * 16 * 3 * (2 * NCC + NH32 + 2 * NM32) + 2 * 16 * 16 * 4 + 4 * TP_FLOATS * 4;
  const int grid = a.nrt * M;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(dec_fwd_x6<NCC, NH32, NM32, GRU, HPRE>, grid, lds, &ok));
  if (!ok) return 0;
  const bool inkernel = 2 * (a.Fp / 16) < M;  // members without an emit tile draw the noise
  if (!inkernel) ABCD_TRY((hipError_t)prefill_eps(s, a));
  ABCD_TRY(zero_sync(s, a.sync, a.nrt));
  PDecFwdArgs b = a;
  if (!inkernel) b.eps_fill = 0;
  b.flags = 1;  // per-member flags (the group-counter form measured slower)
  b.prof = (g_prof_mask & 4) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_DEC_FWD);
    dec_fwd_x6<NCC, NH32, NM32, GRU, HPRE><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_DEC_FWD, "dec_fwd_x6<%d,%d,%d,%s> grid %d", NCC, NH32, NM32, GRU ? "GRU" : "LSTM", grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}


template <int NCC, int NH32, int NM32, bool GRU = false>
static int launch_dec_fwd_x6(hipStream_t s, const PDecFwdArgs& a, bool* launched) {
  return launch_dec_fwd_x6_k<NCC, NH32, NM32, GRU, true>(s, a, launched);
}

int persist_decoder_fwd(hipStream_t s, int G, const PDecFwdArgs& a, bool* launched) {
  *launched = false;
  if (!persist_enabled() || a.H % 8) return 0;
  if (G == 3) {  // GRU: the all-x6 form only (a.bias = [b_r | b_z | b_in | b_hn])
    if (!(x6_enabled(a.H) && a.H == 256 && a.Hm == 256 && 2 * (a.Fp / 16) <= a.H / 8))
      return 0;
    const int ncc = (a.feedback ? cdiv(a.Fp, 32) : 0) + a.H / 32;
    if (ncc == 13) return launch_dec_fwd_x6<13, 8, 8, true>(s, a, launched);
    if (ncc == 11) return launch_dec_fwd_x6<11, 8, 8, true>(s, a, launched);
    if (ncc == 8) return launch_dec_fwd_x6<8, 8, 8, true>(s, a, launched);
    return 0;
  }
  if (G != 4) return 0;
  // all-x6 form: H = Hm = 256 (one mlp tile per member), 2 Fp/16 emit members
  if (x6_enabled(a.H) && a.H == 256 && a.Hm == 256 && 2 * (a.Fp / 16) <= a.H / 8) {
    const int ncc = (a.feedback ? cdiv(a.Fp, 32) : 0) + a.H / 32;
    if (ncc == 13) return launch_dec_fwd_x6<13, 8, 8>(s, a, launched);
    if (ncc == 11) return launch_dec_fwd_x6<11, 8, 8>(s, a, launched);
    if (ncc == 8) return launch_dec_fwd_x6<8, 8, 8>(s, a, launched);
  }
  if (x6_enabled(a.H) && a.H == 256) {
    const int ncc = (a.feedback ? cdiv(a.Fp, 32) : 0) + a.H / 32;
    if (ncc == 13) return launch_dec_fwd<13>(s, a, launched);
    if (ncc == 8) return launch_dec_fwd<8>(s, a, launched);
  }
  return launch_dec_fwd<0>(s, a, launched);
}


// whether the last persistent decoder BPTT of this thread wrote PDecBwdArgs::dhid
thread_local bool tl_dec_bwd_dhid = false;
bool dec_bwd_dhid_done() { return tl_dec_bwd_dhid; }
// dec_bwd_w16 (32-row groups of 16 members: half the split-K exchange of the
// 64-row dec_bwd_fold it replaced): same-box A/B at c2, dec_bwd 3.08 / 3.06 ->
// 2.55 / 2.55 ms per launch, step 9.99 / 9.99 -> 9.49 / 9.47 ms
template <int NXS, bool GRU>
static int launch_dec_bwd_w16(hipStream_t s, const PDecBwdArgs& a, bool* launched) {
  const int ng = cdiv(a.B, W16_ROWS), nchx = a.Fp / 16, ncz = (a.Fp + 31) / 32;
  const size_t lds = (size_t)NXS * 2 * 3 * 64 * 16 + (size_t)16 * 3 * 64 * 16 + (size_t)2 * ncz * 3 * 64 * 16 +
                     (size_t)W16_ROWS * (W16_DTP + W16_ZTP) * 4 + (size_t)2 * 64 * 16 + (size_t)4 * 2 * TP_FLOATS * 4;
  const int grid = ng * W16_M;
  if (a.B <= 0 || 2 * nchx > 4 * W16_M) return 0;
  if (ncz != (NXS > 0 ? NXS : 9) / 2 + 1) return 0;  // the kernel's compile-time chunk count
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(dec_bwd_w16<NXS, GRU>, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY(zero_sync(s, a.sync, ng));
  PDecBwdArgs b = a;
  b.nrt = ng;
  b.flags = 1;
  b.prof = (g_prof_mask & 8) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_DEC_BWD);
    dec_bwd_w16<NXS, GRU><<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_DEC_BWD, "dec_bwd_w16<%d,%s> grid %d", NXS, GRU ? "GRU" : "LSTM", grid);
  tl_dec_bwd_dhid = b.dhid != nullptr;
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}

int persist_decoder_bwd(hipStream_t s, int G, const PDecBwdArgs& a, bool* launched) {
  *launched = false;
  tl_dec_bwd_dhid = false;
  if (!persist_enabled() || a.H % 8) return 0;
  // the split-K form: H = Hm = 256, Fp / 16 <= 16 (the GRU has no other persistent form)
  if (a.part && x6_enabled(a.H) && a.H == 256 && a.Hm == a.H && a.Fp / 16 <= a.H / 8 &&
      (G == 4 || (a.Hprev && a.dGH))) {
    const int nxs = a.feedback ? a.Fp / 16 : 0;
    int rc = 0;
    if (nxs == 9) rc = G == 4 ? launch_dec_bwd_w16<9, false>(s, a, launched) : launch_dec_bwd_w16<9, true>(s, a, launched);
    else if (nxs == 5) rc = G == 4 ? launch_dec_bwd_w16<5, false>(s, a, launched) : launch_dec_bwd_w16<5, true>(s, a, launched);
    else if (nxs == 0) rc = G == 4 ? launch_dec_bwd_w16<0, false>(s, a, launched) : launch_dec_bwd_w16<0, true>(s, a, launched);
    if (rc || *launched) return rc;
  }
  if (G != 4) return 0;  // GRU: the per-step kernels
  const int M = a.H / 8, nchg = 4 * a.H / 16, nchx = a.Fp / 16, nchz = 2 * a.Hm / 16;
  const int n0 = cdiv(a.Fp / 16 + a.H / 16, M), n1 = cdiv(2 * a.Hm / 16, M);
  const size_t lds = (size_t)64 * 16 * (n0 * nchg + n1 * nchx + nchz);
  const int grid = a.nrt * M;
  bool ok = false;
  ABCD_TRY((hipError_t)fits_resident(dec_bwd_persist, grid, lds, &ok));
  if (!ok) return 0;
  ABCD_TRY(zero_sync(s, a.sync, a.nrt));
  PDecBwdArgs b = a;
  b.flags = 1;  // per-member flags (the group-counter form measured slower)
  b.prof = (g_prof_mask & 8) ? g_prof : nullptr;
  {
    TimedScope ts(s, TK_DEC_BWD);
    dec_bwd_persist<<<grid, 256, lds, s>>>(b);
  }
  note_dispatch(TK_DEC_BWD, "dec_bwd_persist grid %d", grid);
  ABCD_CHECK_LAUNCH();
  *launched = true;
  return 0;
}

}  // namespace abcd

// diagnostics (abcd_hip.h: abcd_debug_xcc_map): which XCD (HW_REG_XCC_ID) and
// which CU (HW_REG_HW_ID) each workgroup of a one-per-CU grid runs on, the
// placement the persistent kernels' group_role assumes (blocks b and b + 8
// share an XCD); out holds 2 u32 per block
namespace abcd {
__global__ __launch_bounds__(256) void xcc_map_kernel(unsigned* out) {
  extern __shared__ float pad_lds[];
  if (threadIdx.x == 0) {
    unsigned x, h;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
    pad_lds[0] = 0.f;
    out[2 * blockIdx.x] = x;
    out[2 * blockIdx.x + 1] = h;
  }
}
}  // namespace abcd
extern "C" int abcd_debug_xcc_map(unsigned* dev_out, int blocks, void* stream) {
  const size_t lds = 100 * 1024;  // one workgroup per CU, as the persistent kernels
  if (hipFuncSetAttribute((const void*)abcd::xcc_map_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return -1;
  abcd::xcc_map_kernel<<<blocks, 256, lds, (hipStream_t)stream>>>(dev_out);
  return (int)hipGetLastError();
}

// diagnostics (abcd_hip.h: abcd_debug_persist_prof): stamp buffer for the
// persistent kernels selected by mask, grid x T x 8 u64, or null to disable
extern "C" void abcd_side_gate_enable(int on) { abcd::g_side_gate = on != 0; }

extern "C" void abcd_debug_persist_prof(unsigned long long* dev_buf, int mask) {
  abcd::g_prof = dev_buf;
  abcd::g_prof_mask = mask;
}
namespace abcd {
unsigned long long* debug_prof_buf(int bit) { return (g_prof_mask & bit) ? g_prof : nullptr; }
}  // namespace abcd

namespace abcd {
// stream-ordered: out[0] = the timeout status raised since the last fold
// (0 ok, 1 hand-off wait, 2 side-stream gate), the word cleared and OR-ed
// into the sticky word
__global__ void step_status_kernel(float* out) {
  if (threadIdx.x == 0) {
    const unsigned v = __hip_atomic_exchange(&g_persist_status, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[0] = (float)v;
    if (v) __hip_atomic_fetch_or(&g_persist_sticky, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
}  // namespace abcd

extern "C" int abcd_step_status(float* out, void* stream) {
  if (!out) return ABCD_EINVAL;
  abcd::step_status_kernel<<<1, 64, 0, (hipStream_t)stream>>>(out);
  ABCD_CHECK_LAUNCH();
  return 0;
}

// 0 = no persistent-kernel spin has timed out since the last call (reads and
// clears the device words; synchronises the device)
extern "C" int abcd_device_status(void) {
  unsigned v = 0, w = 0, z = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(abcd::g_persist_status), sizeof(v)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&w, HIP_SYMBOL(abcd::g_persist_sticky), sizeof(w)) != hipSuccess) return -1;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(abcd::g_persist_status), &z, sizeof(z));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(abcd::g_persist_sticky), &z, sizeof(z));
  return (int)(v | w);
}

