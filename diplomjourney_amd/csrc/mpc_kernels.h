// mpc_kernels.h — the rollout / arg-min / selection / sampling kernels (gfx950).
//
//   k_rollout_argmin   one lane per CPL adjacent candidates (CPL = 2: every
//                      control load is 16 B per lane = 1 KiB per wave
//                      instruction); N-step rollout in registers with the
//                      controls of the next kPrefetch-1 steps in flight;
//                      terminal cost; lane -> wave (shuffle) -> block (LDS)
//                      lexicographic (cost, index) arg-min; one 16-B record
//                      per block.
//   k_finalize         arg-min over the block records; the winner re-rolled
//                      lane-parallel (bitwise the arithmetic the lane scored).
//   k_rollout_argmin_batched / k_finalize_batched   robot-segmented variant.
//   k_select_winner    lexicographic min over gathered per-rank results.
//   k_sample_controls  synthetic control sequences (splitmix64 -> grid entry).
//
// Template modes: INTEG (MPC_INTEG_QK21 | MPC_INTEG_RECT), ROT (heading
// rotation recurrence instead of a per-step sincos), STATES (write every
// candidate's per-step states: the CoordinateTree payload), KDEV (problem
// constants read from device memory: the device-resident episode).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mpc_rollout.h"
#include "mpc_device.h"

namespace mpc {

constexpr int kBlock = 256;  // 4 waves of 64
// Tuning constants (DESIGN.md §5 records the A/B measurements behind them).
constexpr int kCplWide = 2;    // candidates per lane on the aligned path (16-B control loads)
constexpr int kPrefetch = 2;   // register-ring depth in steps of the scalar / states path
constexpr int kWaves = kBlock / 64;
constexpr int64_t kMaxBlocks = 2048;   // rollout grid cap: 256 CUs x 8 resident blocks
constexpr int kFinBlock = 256;         // one-block selection kernels (A/B: 1024 -> 256 = -0.7 us)

struct Rec {
  uint64_t key;
  int64_t idx;
};

// Offset of candidate c's control at step s: step-major SoA (pitch = the row
// pitch ld) or TILED (MPC_LAYOUT_TILED, pitch = n_steps: tile c / 512 holds
// per step 512 v then 512 beta; the beta pointer is the v pointer + 512).
template <bool TILED>
__host__ __device__ __forceinline__ int64_t ctl_off(int64_t s, int64_t c, int64_t pitch) {
  if constexpr (TILED)
    return (c >> 9) * (pitch << 10) + (s << 10) + (c & 511);
  else
    return s * pitch + c;
}
static_assert(MPC_TILE == 512, "ctl_off's shifts");

// Block-level arg-min: wave shuffle, then the kWaves wave records via LDS.
// The block winner ends up in thread 0.
// IDX31: every index is below 2^31 (wave_argmin32).
template <bool IDX31 = false>
__device__ __forceinline__ void block_argmin(uint64_t& k, int64_t& i) {
  __shared__ uint64_t s_key[kWaves];
  __shared__ int64_t s_idx[kWaves];
  if constexpr (IDX31)
    wave_argmin32(k, i);
  else
    wave_argmin(k, i);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_key[wave] = k;
    s_idx[wave] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < kWaves; ++w)
      if (rec_less(s_key[w], s_idx[w], k, i)) {
        k = s_key[w];
        i = s_idx[w];
      }
  }
}

// Block-uniform constants computed on the VALU (consts_from_problem) moved to
// SGPRs: hipcc keeps VALU results in VGPRs even when every lane holds the same
// value, which costs the batched kernel its fifth wave (120 VGPRs -> spills).
__device__ __forceinline__ double uniform_d(double a) {
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(a));
  const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(u)));
  const uint64_t hi =
      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(u >> 32)));
  return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
}

__device__ __forceinline__ Consts uniform_consts(const Consts& k) {
  Consts K;
  K.x = uniform_d(k.x);
  K.y = uniform_d(k.y);
  K.phi = uniform_d(k.phi);
  K.x_t = uniform_d(k.x_t);
  K.y_t = uniform_d(k.y_t);
  K.x_0 = uniform_d(k.x_0);
  K.y_0 = uniform_d(k.y_0);
  K.A = uniform_d(k.A);
  K.B = uniform_d(k.B);
  K.C1 = uniform_d(k.C1);
  K.C2 = uniform_d(k.C2);
  K.inv_den = uniform_d(k.inv_den);
  K.L = uniform_d(k.L);
  K.inv_L = uniform_d(k.inv_L);
  K.h = uniform_d(k.h);
  K.hlgth = uniform_d(k.hlgth);
  K.s0 = uniform_d(k.s0);
  K.c0 = uniform_d(k.c0);
  K.L_pow2 = __builtin_amdgcn_readfirstlane(k.L_pow2);
  K.pad_ = 0;
  return K;
}

// Rollout of CPL adjacent candidates starting at column c0; costs in cst.
template <int CPL, int INTEG, int ROT, bool STATES, bool PL2>
__device__ __forceinline__ void rollout_lane_l(const Consts& K, const double* __restrict__ v,
                                             const double* __restrict__ b, int64_t ld, int64_t c0,
                                             int n_steps, double (&cst)[CPL],
                                             double* __restrict__ states, int64_t n_cand) {
  double x[CPL], y[CPL], ph[CPL], sn[CPL], cs[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) step_start<ROT>(K, x[j], y[j], ph[j], sn[j], cs[j]);
  // Controls of step sr for this lane's CPL candidates: 16 B per lane per
  // array on the wide path (one 1 KiB wave-instruction each).
  auto load = [&](int sr, double (&vv)[CPL], double (&bb)[CPL]) {
    if constexpr (CPL >= 2) {
#pragma unroll
      for (int h = 0; h < CPL; h += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(v + sr * ld + c0 + h);
        const double2 b2 = *reinterpret_cast<const double2*>(b + sr * ld + c0 + h);
        vv[h] = v2.x;
        vv[h + 1] = v2.y;
        bb[h] = b2.x;
        bb[h + 1] = b2.y;
      }
    } else {
      vv[0] = v[sr * ld + c0];
      bb[0] = b[sr * ld + c0];
    }
  };
  bool bad[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) bad[j] = false;
  auto body = [&](int sr, const double (&vv)[CPL], const double (&bb)[CPL]) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      step_core<INTEG, ROT, PL2>(x[j], y[j], ph[j], sn[j], cs[j], vv[j], bb[j], K, bad[j]);
      if constexpr (STATES) {
        double px = x[j], py = y[j];
        if constexpr (ROT == kRotCum) cum_pose<PL2>(K, x[j], y[j], px, py);
        states[(sr * 3 + 0) * n_cand + c0 + j] = px;
        states[(sr * 3 + 1) * n_cand + c0 + j] = py;
        states[(sr * 3 + 2) * n_cand + c0 + j] = ph[j];
      }
    }
  };
  // Software pipeline: the controls of the next kPrefetch-1 steps are in
  // flight while this step's trig chain runs (rotating register buffers,
  // kPrefetch steps per trip, static indices, no copies).  One step of VALU
  // work is far shorter than the loaded HBM latency, so one step of lookahead
  // leaves the loop waiting on memory.
  constexpr int D = kPrefetch;
  double vq[D][CPL], bq[D][CPL];
#pragma unroll
  for (int u = 0; u < D - 1; ++u)
    if (u < n_steps) load(u, vq[u], bq[u]);
#pragma unroll 1
  for (int s = 0; s < n_steps; s += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int st = s + u;
      if (st < n_steps) {
        if (st + D - 1 < n_steps) load(st + D - 1, vq[(u + D - 1) % D], bq[(u + D - 1) % D]);
        body(st, vq[u], bq[u]);
      }
    }
  }
  // Irregular candidates (argument outside the trig cores' range, or NaN):
  // recompute with the safe recurrence.  Never taken for the reference's
  // arguments; kept out of the loop so the loop carries no fallback code.
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    if constexpr (ROT == kRotCum) {
      if (!bad[j]) cum_pose<PL2>(K, x[j], y[j], x[j], y[j]);
    }
    if (bad[j]) {
      x[j] = K.x;
      y[j] = K.y;
      ph[j] = K.phi;
      for (int sr = 0; sr < n_steps; ++sr) {
        step_safe<INTEG>(x[j], y[j], ph[j], v[sr * ld + c0 + j], b[sr * ld + c0 + j], K);
        if constexpr (STATES) {
          states[(sr * 3 + 0) * n_cand + c0 + j] = x[j];
          states[(sr * 3 + 1) * n_cand + c0 + j] = y[j];
          states[(sr * 3 + 2) * n_cand + c0 + j] = ph[j];
        }
      }
    }
    cst[j] = cost(x[j], y[j], K);
  }
}

// ---------------------------------------------------------------------------
// Wide path with an LDS-DMA control ring.  Each wave streams its own 128
// candidates: per step one global_load_lds_dwordx4 for v and one for beta
// (1 KiB each, lane-linear: lane l's 16 B land at slot + 16*l) into a ring of
// kRing step slots per wave, kRing-1 steps ahead of the step being computed.
// The loads need no VGPRs while in flight (the register ring of rollout_lane_l
// holds 8 per step of lookahead), so the lookahead is deeper at a lower VGPR
// count.  The DMA is issued by inline asm, which hipcc neither counts nor
// orders against the LDS reads: the waits are explicit (vmcnt for "slot
// landed", lgkmcnt(0) before a slot is refilled) and every asm statement
// clobbers memory.
// The control DMA is streamed once: non-temporal (A/B: -1.5 us/step on config C).
#define MPC_GLDS_POLICY " nt"
constexpr int kRing = 3;   // LDS ring depth in steps (kRing-1 steps in flight)

// One ring for every instantiation (namespace scope: allocated once per kernel).
__shared__ double2 g_ring[kWaves][kRing][2][64];  // [wave][slot][v|beta][lane]

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}

// Inline asm whose VMEM instruction takes an SGPR operand (the `saddr` base)
// must itself provide the wait states the hardware needs between a VALU that
// writes that SGPR and the VMEM that reads it (5 on CDNA): hipcc's hazard
// recognizer does not look inside asm statements, and it reloads spilled SGPRs
// with v_readlane — measured: a v_readlane of the base right before the load,
// 0 wait states, faulted.  Hence the `s_nop 4` ahead of the first such VMEM in
// every statement below (the M0 write's own 1-wait-state need is covered too).
// Both control rows of one step into LDS (v at dst_v, beta at dst_b).  The
// addresses are SGPR base + 32-bit VGPR offset (the `saddr` form): the row
// bases gv / gb (step s's rows: wave-uniform) advance per step on the SALU,
// the lane's byte offset `voff` is fixed for the tile — no 64-bit per-lane
// address arithmetic on the VALU in the loop.  The statement writes only M0
// (saved and restored) and `keep`: no SCC-setting instruction (s_add etc.),
// since hipcc may hold a live SCC across it.
// Refilling a slot must not overtake the LDS reads of its previous contents:
// `read_v`/`read_b` are the registers those reads produced, taken as inputs
// so hipcc completes the reads (lgkmcnt) before the DMA is issued — without a
// blanket lgkmcnt(0), which would also wait for unrelated scalar loads.
__device__ __forceinline__ void glds_pair(const double* gv, const double* gb, uint32_t voff,
                                          uint32_t dst_v, uint32_t dst_b) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 4\n\t"
      "global_load_lds_dwordx4 %1, %2" MPC_GLDS_POLICY "\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3" MPC_GLDS_POLICY "\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gv), "s"(gb), "s"(dst_v), "s"(dst_b)
      : "memory");
}

__device__ __forceinline__ void glds_refill(const double* gv, const double* gb, uint32_t voff,
                                            uint32_t dst_v, uint32_t dst_b,
                                            const double2& read_v, const double2& read_b) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 4\n\t"
      "global_load_lds_dwordx4 %1, %2" MPC_GLDS_POLICY "\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3" MPC_GLDS_POLICY "\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gv), "s"(gb), "s"(dst_v), "s"(dst_b), "v"(read_v.x), "v"(read_v.y),
        "v"(read_b.x), "v"(read_b.y)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  if constexpr (N == 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10)
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
}

struct NoPre {
  __device__ void operator()() const {}
};

// pre(): called before K is first read (the chained episode step waits there
// for this step's constants): ROT 0 / 1 once the first ring slots are in
// flight; kRotCum only after the loop, which reads Kloop (the step size h and
// the wheelbase terms; = K except in the chained step, which speculates them
// in pre0(), called once the first ring slots are in flight).
// mid(): kRotCum, called right after the wait of step n_steps - 3: loads it
// issues complete with that step's last control DMA (the tail waits for both).
// PIN: the leading trig coefficients pinned in VGPRs (8 VGPRs for ~8 VALU per
// lane-step); off where the register budget is tighter than the VALU budget.
template <int INTEG, int ROT, bool PL2, class Pre = NoPre, class Pre0 = NoPre,
          class Mid = NoPre, bool PIN = true>
__device__ __forceinline__ void rollout_lane_glds_k(const Consts& K, const Consts& Kloop,
                                                    const double* __restrict__ v,
                                                    const double* __restrict__ b, int64_t ld,
                                                    int64_t c0, int n_steps, double (&cst)[2],
                                                    const Pre& pre = Pre{},
                                                    const Pre0& pre0 = Pre0{},
                                                    const Mid& mid = Mid{}) {
  constexpr int CPL = 2;
  constexpr int R = kRing;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_addr(&g_ring[wv][0][0][0]));
  constexpr uint32_t kSlot = 2 * 64 * sizeof(double2);  // 2 KiB
  auto dst = [&](int slot) { return ring0 + slot * kSlot; };
  // the lane's byte offset in every control row (< 2^31: the host checks
  // 8 * ld < 2^31 for the aligned path)
  const uint32_t voff = static_cast<uint32_t>(c0) * 8u;
  // leading trig coefficients pinned in VGPRs (opaque to the compiler, so not
  // re-materialised per step)
  trig::Leads lead = trig::const_leads();
  if constexpr (PIN)
    asm volatile("" : "+v"(lead.tp), "+v"(lead.rs), "+v"(lead.rc));
  // The loop constants: Kloop (read after pre0), or K when a speculated step
  // size turns out wrong (kRotCum with a real pre(): the chained step after an
  // episode restart) and the loop runs again from the controls with the final
  // constants — the same code, bitwise the lane's arithmetic, and no second
  // copy of the recurrence to hold registers for.
  Consts KL;
  double x[CPL], y[CPL], ph[CPL], sn[CPL], cs[CPL];
  bool bad[CPL];
  for (int pass = 0;; ++pass) {
#pragma unroll
    for (int u = 0; u < R - 1; ++u)
      if (u < n_steps) glds_pair(v + u * ld, b + u * ld, voff, dst(u), dst(u) + kSlot / 2);
    if (pass == 0) {
      if constexpr (ROT != kRotCum)
        pre();
      else
        pre0();   // kRotCum: the loop constants Kloop (the chained step reads them here)
      KL = Kloop;
    }
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      step_start<ROT>(KL, x[j], y[j], ph[j], sn[j], cs[j]);
      bad[j] = false;
    }
    double2 v2 = make_double2(0.0, 0.0), b2 = v2;   // the last slot's contents as read
#pragma unroll 1
    for (int s = 0; s < n_steps; s += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int st = s + u;
        if (st < n_steps) {
          if (st + R - 1 < n_steps) {
            const int sr = st + R - 1, slot = (u + R - 1) % R;   // = the slot read last step
            glds_refill(v + sr * ld, b + sr * ld, voff, dst(slot), dst(slot) + kSlot / 2, v2,
                        b2);
            wait_vm<2 * (R - 1)>();   // this step's pair has landed
          } else {
            wait_vm<0>();             // pipeline tail
          }
          if constexpr (!std::is_same_v<Mid, NoPre>) {
            if (st == n_steps - 3) mid();
          }
          v2 = g_ring[wv][u][0][lane];
          b2 = g_ring[wv][u][1][lane];
          // the heading itself is not needed here (rotation mode carries sin/cos;
          // an irregular candidate is recomputed from K.phi), so no phi chain
          double ph0 = ROT ? 0.0 : ph[0], ph1 = ROT ? 0.0 : ph[1];
          step_core<INTEG, ROT, PL2>(x[0], y[0], ph0, sn[0], cs[0], v2.x, b2.x, KL, bad[0],
                                     &lead);
          step_core<INTEG, ROT, PL2>(x[1], y[1], ph1, sn[1], cs[1], v2.y, b2.y, KL, bad[1],
                                     &lead);
          if (!ROT) {
            ph[0] = ph0;
            ph[1] = ph1;
          }
        }
      }
    }
    if constexpr (ROT == kRotCum) {
      // the start pose is first needed here (chained step: this step's
      // constants are waited for now; if the step size speculated for the loop
      // turns out different — an episode restart reset t — the loop runs again)
      if (pass == 0) pre();
      if constexpr (!std::is_same_v<Pre, NoPre>) {
        // (the chained step's K lives in LDS: its h and, on the rare rerun,
        // the loop's terms are moved to SGPRs; nothing else of K is)
        if (KL.h != uniform_d(K.h)) {   // rare (episode restart); uniform over the block
          KL = uniform_consts(K);
          continue;
        }
      }
#pragma unroll
      for (int j = 0; j < CPL; ++j)
        if (!bad[j]) cum_pose<PL2>(K, x[j], y[j], x[j], y[j]);
    }
    break;
  }
  // The criterion first (an irregular candidate's value is replaced below),
  // then the rare recompute: nothing of the criterion (the target and line
  // terms of K, which the chained step reads from LDS into VGPRs) is live
  // across the recompute's register-hungry trig.
#pragma unroll
  for (int j = 0; j < CPL; ++j) cst[j] = cost(x[j], y[j], K);
  if (bad[0] || bad[1]) {
    // (wave-uniform SGPR copies: the recompute's trig needs the VGPRs)
    const Consts Ks = uniform_consts(K);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      if (bad[j]) {
        x[j] = Ks.x;
        y[j] = Ks.y;
        ph[j] = Ks.phi;
        for (int sr = 0; sr < n_steps; ++sr)
          step_safe<INTEG>(x[j], y[j], ph[j], v[sr * ld + c0 + j], b[sr * ld + c0 + j], Ks);
        cst[j] = cost(x[j], y[j], Ks);
      }
    }
  }
}

// kRotCum keeps the start pose's terms live across the loop: with pinned
// leads it needs > 96 VGPRs and spills at 5 waves/SIMD (any scratch costs far
// more than the fifth wave gains), unpinned it fits.
template <int INTEG, int ROT, bool PL2>
__device__ __forceinline__ void rollout_lane_glds(const Consts& K, const double* __restrict__ v,
                                                  const double* __restrict__ b, int64_t ld,
                                                  int64_t c0, int n_steps, double (&cst)[2]) {
  rollout_lane_glds_k<INTEG, ROT, PL2, NoPre, NoPre, NoPre, ROT != kRotCum>(
      K, K, v, b, ld, c0, n_steps, cst);
}

// L a power of two or not: one loop body each (see step_core).
template <int CPL, int INTEG, int ROT, bool STATES>
__device__ __forceinline__ void rollout_lane(const Consts& K, const double* __restrict__ v,
                                             const double* __restrict__ b, int64_t ld, int64_t c0,
                                             int n_steps, double (&cst)[CPL],
                                             double* __restrict__ states, int64_t n_cand) {
  if constexpr (CPL == 2 && !STATES) {
    if (K.L_pow2)
      rollout_lane_glds<INTEG, ROT, true>(K, v, b, ld, c0, n_steps, cst);
    else
      rollout_lane_glds<INTEG, ROT, false>(K, v, b, ld, c0, n_steps, cst);
    return;
  }
  if (K.L_pow2)
    rollout_lane_l<CPL, INTEG, ROT, STATES, true>(K, v, b, ld, c0, n_steps, cst, states, n_cand);
  else
    rollout_lane_l<CPL, INTEG, ROT, STATES, false>(K, v, b, ld, c0, n_steps, cst, states, n_cand);
}

template <int CPL, int INTEG, int ROT, bool STATES, bool KDEV>
__device__ __forceinline__ void rollout_argmin_body(
    const Consts& Karg, const Consts* __restrict__ Kdev, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, Rec* __restrict__ part,
    double* __restrict__ states) {
  const Consts K = KDEV ? *Kdev : Karg;
  const int64_t n_tiles = (n_cand + kBlock * CPL - 1) / (kBlock * CPL);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t c0 = tile * (kBlock * CPL) + threadIdx.x * CPL;
    if (c0 < n_cand) {  // CPL > 1 requires n_cand % CPL == 0: the whole group is valid
      double cst[CPL];
      rollout_lane<CPL, INTEG, ROT, STATES>(K, v, b, n_cand, c0, n_steps, cst, states, n_cand);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const uint64_t kk = cost_key_nonneg(cst[j]);
        if (kk < best_k) {  // ascending index per lane: strict < keeps the first
          best_k = kk;
          best_i = c0 + j;
        }
      }
    }
  }
  block_argmin<CPL == kCplWide>(best_k, best_i);   // (wide path: rows < 2^28 candidates)
  if (threadIdx.x == 0) part[blockIdx.x] = Rec{best_k, best_i};
}

// Scalar (CPL = 1), CoordinateTree-states and register-ring paths.
template <int CPL, int INTEG, int ROT, bool STATES, bool KDEV>
__global__ __launch_bounds__(kBlock, 1) void k_rollout_argmin(
    Consts Karg, const Consts* __restrict__ Kdev, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, Rec* __restrict__ part,
    double* __restrict__ states) {
  rollout_argmin_body<CPL, INTEG, ROT, STATES, KDEV>(Karg, Kdev, v, b, n_cand, n_steps, part,
                                                      states);
}

// The streaming kernel of the aligned path (CPL = 2, LDS-DMA ring).  With the
// irregular-candidate recompute free of the device library's large-argument
// trig (mpc_trig.h reduce_pio2_large), its registers fit kStreamWaves waves
// per SIMD (5: <= 96 VGPRs; 6 spills).
constexpr int kStreamWaves = 5;
template <int INTEG, int ROT, bool KDEV>
__global__ __launch_bounds__(kBlock, kStreamWaves) void k_rollout_argmin_stream(
    Consts Karg, const Consts* __restrict__ Kdev, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, Rec* __restrict__ part) {
  rollout_argmin_body<kCplWide, INTEG, ROT, false, KDEV>(Karg, Kdev, v, b, n_cand, n_steps,
                                                          part, nullptr);
}

// Measurement probe (mpc_stream_probe): the streaming kernel's memory side
// alone — the same grid, tiles, lanes and LDS-DMA control ring (kRing slots,
// kRing-1 steps in flight, `nt`), each landed slot read back from LDS and
// folded into one word per lane, no rollout arithmetic.  Its duration is the
// read-only stream ceiling of the rollout's own access pattern at the
// launch's size (launch ramp and tail included), the denominator the
// streaming kernels' time is compared with.
// TILED: the same over MPC_LAYOUT_TILED controls (a tile's rows at tile base +
// s * 1024 doubles, the lane's offset within its tile).
template <bool TILED>
__global__ __launch_bounds__(kBlock, kStreamWaves) void k_stream_probe(
    const double* __restrict__ v, const double* __restrict__ b, int64_t n_cand, int n_steps,
    uint64_t* __restrict__ sink) {
  constexpr int R = kRing;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_addr(&g_ring[wv][0][0][0]));
  constexpr uint32_t kSlot = 2 * 64 * sizeof(double2);
  auto dst = [&](int slot) { return ring0 + slot * kSlot; };
  const int64_t n_tiles = (n_cand + kBlock * 2 - 1) / (kBlock * 2);
  uint64_t acc = 0;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t c0 = tile * (kBlock * 2) + threadIdx.x * 2;
    if (c0 >= n_cand) continue;   // n_cand even (host check): the pair is valid
    const int64_t ld = TILED ? 2 * MPC_TILE : n_cand;   // row pitch
    const double* tv = TILED ? v + tile * ld * n_steps : v;
    const double* tb = TILED ? b + tile * ld * n_steps : b;
    const uint32_t voff = static_cast<uint32_t>(TILED ? c0 - tile * MPC_TILE : c0) * 8u;
#pragma unroll
    for (int u = 0; u < R - 1; ++u)
      if (u < n_steps) glds_pair(tv + u * ld, tb + u * ld, voff, dst(u), dst(u) + kSlot / 2);
    double2 v2 = make_double2(0.0, 0.0), b2 = v2;
#pragma unroll 1
    for (int s = 0; s < n_steps; s += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int st = s + u;
        if (st < n_steps) {
          if (st + R - 1 < n_steps) {
            const int sr = st + R - 1, slot = (u + R - 1) % R;
            glds_refill(tv + sr * ld, tb + sr * ld, voff, dst(slot), dst(slot) + kSlot / 2, v2,
                        b2);
            wait_vm<2 * (R - 1)>();
          } else {
            wait_vm<0>();
          }
          v2 = g_ring[wv][u][0][lane];
          b2 = g_ring[wv][u][1][lane];
          acc ^= static_cast<uint64_t>(__double_as_longlong(v2.x)) ^
                 static_cast<uint64_t>(__double_as_longlong(b2.y));
        }
      }
    }
  }
  if (acc == 0x5eedull) sink[blockIdx.x * kBlock + threadIdx.x] = acc;   // keeps the reads live
}

// What the episode update needs of a winner (kept in registers by the
// finalize kernel instead of being re-read from the result record).
struct Winner {
  double cost;
  int64_t index;
  int32_t found, n_steps;
  double v, beta;
  double tr[3][3];     // states of steps 0..2 (clamped to the horizon)
};

// r.tr[k][q] for a runtime k in {0, 1, 2} by selects: a dynamically indexed
// local array would live in scratch memory (a ~µs round trip per access).
__device__ __forceinline__ double tr_at(const Winner& r, int k, int q) {
  const double a = r.tr[0][q], b = r.tr[1][q], c = r.tr[2][q];
  return k == 0 ? a : (k == 1 ? b : c);
}

// Re-roll the winner and fill the result record.  Called by ALL threads of
// the block once thread 0 holds the winner (key, col).  The N-step recurrence
// is split so that only cheap accumulations stay serial: lane s computes the
// state-free heading increment dphi_s = Q((v_s/L) tan(beta_s)); lane 0
// accumulates the headings; lane s evaluates sincos(phi_s) (direct mode) or
// the rotation factors of dphi_s (ROT); lane 0 rotates (ROT) and accumulates
// x and y.  The winner is regular or irregular exactly as in rollout_lane
// (same tests), and each branch repeats that path's operations in the same
// order, so the emitted states are bitwise those the arg-min scored.
// LDS of the winner's re-roll (emit_winner) and of the selection's staged
// controls (finalize_block), provided by the caller: a kernel that owns LDS
// it is not using at that point — the chained step's block 0 and the fused
// finalize have the control ring — lends that instead of adding 2.5 KiB to
// the kernel's LDS (which decides how many blocks fit on a CU).
struct EmitLds {
  double v[MPC_MAX_STEPS], dphi[MPC_MAX_STEPS], phi[MPC_MAX_STEPS];
  double a[MPC_MAX_STEPS], c[MPC_MAX_STEPS];
  double tr[MPC_MAX_STEPS * 3];
  double pv[MPC_MAX_STEPS], pb[MPC_MAX_STEPS];
  double tail[5];      // deferred re-roll: lane 0's state (x, y, sin, cos, phi) ...
  int tail_from;       // ... after this many steps (== n_steps: nothing deferred)
};

// The control ring's LDS lent to the re-roll (a block whose ring is idle).
__device__ __forceinline__ EmitLds* ring_lds() {
  static_assert(sizeof(EmitLds) <= sizeof(g_ring), "the re-roll's LDS fits in the ring");
  return reinterpret_cast<EmitLds*>(&g_ring[0][0][0][0]);
}

// Side work for the threads that have no part in a phase of the re-roll (every
// thread >= 64: n_steps <= 32): side_a() runs beside the per-step factors,
// side_b(fast) beside lane 0's serial pass; both are called by every thread
// and pick their own threads.
struct NoSide {
  __device__ void operator()() const {}
  __device__ void operator()(bool) const {}
  __device__ void operator()(int, double, double, double) const {}
};

// on_layer(st, x, y, phi): lane 0, in the serial pass, as each of the first
// three layer states is formed.
template <int INTEG, int ROT, class SideA = NoSide, class SideB = NoSide, class OnLayer = NoSide>
__device__ void emit_winner(const Consts& K, const double* __restrict__ v,
                            const double* __restrict__ b, int64_t ld, int n_steps, uint64_t key,
                            int64_t col, int64_t reported_index, double incumbent,
                            mpc_result_t* __restrict__ out, EmitLds* lds, Winner* win = nullptr,
                            const double* pre_v = nullptr, const double* pre_b = nullptr,
                            bool defer_tail = false, const SideA& side_a = SideA{},
                            const SideB& side_b = SideB{}, const OnLayer& on_layer = OnLayer{}) {
  double* s_v = lds->v;
  double* s_dphi = lds->dphi;
  double* s_phi = lds->phi;
  double* s_a = lds->a;
  double* s_c = lds->c;
  __shared__ double s_b0;
  __shared__ uint64_t s_key;
  __shared__ int64_t s_col, s_rep;
  __shared__ int s_bad;
  if (threadIdx.x == 0) {
    s_key = key;
    s_col = col;
    s_rep = reported_index;
    s_bad = 0;
  }
  __syncthreads();
  key = s_key;
  col = s_col;
  const int lane = threadIdx.x;
  const bool valid = key != ~0ull;
  // Regular pass (step_core's forms and range checks), then — if any step is
  // irregular — the safe pass (step_safe's forms) for the whole candidate,
  // exactly as rollout_candidate / the rollout kernels decide.
  double vs = 0.0, w = 0.0, bs = 0.0, d = 0.0, ra = 0.0, rc = 0.0;
  if (valid && lane < n_steps) {
    // pre_v / pre_b: the winner's controls already staged in LDS by the caller
    // (finalize_block prefetches each wave's best during the block reduction)
    vs = pre_v ? pre_v[lane] : v[lane * ld + col];
    bs = pre_b ? pre_b[lane] : b[lane * ld + col];
    s_v[lane] = vs;
    if (lane == 0) s_b0 = bs;
    w = K.L_pow2 ? vs * K.inv_L : vs / K.L;
    d = heading_incr<INTEG>(w, trig::tan_small(bs), K);
    s_dphi[lane] = d;
    const bool lane_bad =
        !(fabs(bs) <= trig::kTanMax) || (ROT && !(fabs(d) <= trig::kRotMax));
    if (lane_bad) s_bad = 1;
    // rotation mode: the factors depend on this step's increment only, so
    // they are formed here, in the same phase (no heading chain needed)
    if (ROT && !lane_bad) {
      trig::rotation_sc(d, ra, rc);
      s_a[lane] = ra;
      s_c[lane] = rc;
    }
  }
  side_a();
  __syncthreads();
  // Regular rotation-mode winner: ONE serial pass on lane 0 (heading, rotation,
  // position); every other case keeps the heading chain / sincos phases.
  const bool fast = ROT && s_bad == 0;
  if (!fast) {
    if (valid && lane == 0) {
      double ph = K.phi;
      for (int st = 0; st < n_steps; ++st) {
        ph = ph + s_dphi[st];
        s_phi[st] = ph;
        if (!ROT && !(fabs(ph) <= trig::kFastMax)) s_bad = 1;
      }
    }
    __syncthreads();
    if (s_bad) {
      if (valid && lane < n_steps)
        s_dphi[lane] = heading_incr<INTEG>(w, trig::tan_fast(bs), K);
      __syncthreads();
      if (valid && lane == 0) {
        double ph = K.phi;
        for (int st = 0; st < n_steps; ++st) {
          ph = ph + s_dphi[st];
          s_phi[st] = ph;
        }
      }
      __syncthreads();
    }
    if (valid && lane < n_steps)
      trig::sincos_fast(s_phi[lane], &s_a[lane], &s_c[lane]);  // == sincos_core if regular
    __syncthreads();
  }
  // Lane 0 runs the serial pass into LDS; the record's trajectory is then
  // stored by one lane per value (a single lane's ~30 stores would serialise
  // in the address path for ~1 us).
  // defer_tail (a regular rotation-mode winner): the pass stops after the
  // three layer states the episode update needs; emit_winner_tail() finishes
  // the record's trajectory once the update is out (same operations, same
  // order, continued from the saved state).
  double* s_tr = lds->tr;
  const int n_run = (defer_tail && fast && n_steps > 3) ? 3 : n_steps;
  if (lane == 0) {
    lds->tail_from = n_steps;
    out->n_steps = n_steps;
    if (win) win->n_steps = n_steps;
    if (!valid) {
      out->cost = __builtin_inf();
      out->index = -1;
      out->found = 0;
      out->v = 0.0;
      out->beta = 0.0;
      if (win) {
        win->cost = __builtin_inf();
        win->index = -1;
        win->found = 0;
      }
    } else {
      const double c = key_cost(key);
      const int found = c < incumbent ? 1 : 0;
      out->cost = c;
      out->index = s_rep;
      out->found = found;
      out->v = s_v[0];
      out->beta = s_b0;
      if (win) {
        win->cost = c;
        win->index = s_rep;
        win->found = found;
        win->v = s_v[0];
        win->beta = s_b0;
      }
      double x, y, sn, cs, ph;
      if (fast)
        step_start<ROT>(K, x, y, ph, sn, cs);    // kRotCum: identity rotation, empty sums
      else
        step_start<0>(K, x, y, ph, sn, cs);
      // the fast pass takes step st's values from lane st's registers
      // (v_readlane: no LDS round trip per step on the serial path)
      auto rl = [](double val, int src) {
        const uint64_t u = static_cast<uint64_t>(__double_as_longlong(val));
        const uint32_t lo = __builtin_amdgcn_readlane(static_cast<int>(u), src);
        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), src);
        return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
      };
      for (int st = 0; st < n_run; ++st) {
        double vst;
        if (fast) {
          ph = ph + rl(d, st);
          trig::rotate_sc(rl(ra, st), rl(rc, st), sn, cs);
          vst = rl(vs, st);
        } else {
          ph = s_phi[st];
          sn = s_a[st];
          cs = s_c[st];
          vst = s_v[st];
        }
        x = position_step<INTEG>(x, vst, cs, K);
        y = position_step<INTEG>(y, vst, sn, K);
        double px = x, py = y;
        if (ROT == kRotCum && fast) cum_pose<false>(K, x, y, px, py);
        s_tr[3 * st] = px;
        s_tr[3 * st + 1] = py;
        s_tr[3 * st + 2] = ph;
        if (win && st < 3) {
          win->tr[st][0] = px;
          win->tr[st][1] = py;
          win->tr[st][2] = ph;
        }
        if (st < 3) on_layer(st, px, py, ph);
      }
      if (n_run < n_steps) {
        lds->tail[0] = x;
        lds->tail[1] = y;
        lds->tail[2] = sn;
        lds->tail[3] = cs;
        lds->tail[4] = ph;
        lds->tail_from = n_run;
      }
    }
  }
  side_b(fast);
  __syncthreads();
  if (valid && lane < 3 * lds->tail_from) (&out->traj[0][0])[lane] = s_tr[lane];
}

// The rest of a deferred re-roll (emit_winner with defer_tail): every thread,
// after a barrier that follows emit_winner; K = the constants it was given.
template <int INTEG, int ROT>
__device__ void emit_winner_tail(const Consts& K, int n_steps, EmitLds* lds,
                                 mpc_result_t* __restrict__ out) {
  const int from = lds->tail_from;   // uniform
  if (from >= n_steps) return;
  double* s_tr = lds->tr;
  if (threadIdx.x == 0) {
    double x = lds->tail[0], y = lds->tail[1], sn = lds->tail[2], cs = lds->tail[3],
           ph = lds->tail[4];
    for (int st = from; st < n_steps; ++st) {
      ph = ph + lds->dphi[st];
      trig::rotate_sc(lds->a[st], lds->c[st], sn, cs);
      x = position_step<INTEG>(x, lds->v[st], cs, K);
      y = position_step<INTEG>(y, lds->v[st], sn, K);
      double px = x, py = y;
      if (ROT == kRotCum) cum_pose<false>(K, x, y, px, py);
      s_tr[3 * st] = px;
      s_tr[3 * st + 1] = py;
      s_tr[3 * st + 2] = ph;
    }
  }
  __syncthreads();
  const int q = threadIdx.x;
  if (q >= 3 * from && q < 3 * n_steps) (&out->traj[0][0])[q] = s_tr[q];
}

// The device-resident episode's scalars (mpc_episode.h: EpisodeState = this
// head + the sampler grids).
struct EpisodeHead {
  Consts K;            // this step's problem constants
  double incumbent;    // optimal_criterion at the start of this step
  double x, y, phi, v, beta;
  double x_t, y_t, x_0, y_0;
  double t;
  uint64_t seed;       // this step's sampler seed
  int64_t step;
  int32_t p, m, steps_for_slowing, episodes;
  int32_t nv, nb;
  // math_mpc's stuck detector (:559-563); x_previous / y_previous (:540-541,
  // :570-571) are always the pose the step starts from, (x, y) above
  int32_t recursive;
  int32_t has_traj;    // optimal_trajectory holds a winner (not the initial [[[0]]])
};

// The module globals optimal_trajectory[0] (layer states 0..2), result_v,
// result_beta: what a step in which no candidate beats the incumbent returns
// (stale: :351-359 not taken; the post-processing :366-429 as usual).  Stored
// right after the head in HBM and staged with it in LDS; the update reads and
// writes it there (a register copy of head + trajectory would not fit
// thread 0's registers and lands in scratch).
struct StaleTraj {
  double ot[3][3];
  double v, beta;
};

// What a chained step's early publication needs of the update it makes,
// formed when the previous step's update is done (episode_early_prepare):
// the finishing layer k when the step can only be a common one (no event,
// break or limit; -1 otherwise), the next step's t and step sizes, and the
// pose a step without winner returns (stale layer k, or the pose) and whether
// it passes the end-of-step checks.  `step`: the head's
// step count it was formed for (a step completed by another path leaves it
// stale, and the next chained step then publishes after its update).
// Stored right after StaleTraj, staged with the head.
struct EarlyPub {
  int64_t step;
  int32_t k, alt;
  double t, h, hl;
  double x, y, ph;   // (its sin / cos are evaluated when used: a step without winner is rare)
};

struct EpisodeHook {  // single-GPU episode: finalize also advances it
  EpisodeHead* H;     // nullptr: no hook
  mpc_episode_log_t* log;
  int cap;
  uint64_t* chain_pub = nullptr;   // cleared with the update (ends a chain of chained steps) ...
  int chain_pub_words = 0;
  uint32_t publish_epoch = 0;      // ... or, nonzero, the next step's constants published
  uint32_t* chain_error = nullptr; // (publish_epoch: the early publication's self-check, code 6)
};
constexpr int kHeadWords = static_cast<int>(sizeof(EpisodeHead) / 8);
constexpr int kStaleWords = static_cast<int>(sizeof(StaleTraj) / 8);
constexpr int kEarlyWords = static_cast<int>(sizeof(EarlyPub) / 8);
constexpr int kStoredWords = kHeadWords + kStaleWords;   // head + stale trajectory
constexpr int kStagedWords = kStoredWords + kEarlyWords; // ... + the early-publication inputs
static_assert(kStagedWords <= 64, "staged head: one word per lane");
constexpr int kLogWords = static_cast<int>(sizeof(mpc_episode_log_t) / 8);
static_assert(sizeof(EpisodeHead) % 8 == 0 && kHeadWords <= 64, "head: one word per lane");
static_assert(sizeof(mpc_episode_log_t) % 8 == 0 && kLogWords <= 64, "log: one word per lane");

__device__ __forceinline__ mpc_episode_log_t* log_slot(mpc_episode_log_t* log, int cap,
                                                       int64_t step) {
  return (log && cap > 0) ? &log[step % cap] : nullptr;
}

// The episode update's stores, one 8-B word per lane (called by every thread
// after a barrier; thread 0 staged the head and the log record in LDS): a
// single lane's ~40 stores serialise in the address path for ~0.7 us.
// epoch != 0 (a chained launch's block 0): instead of clearing the chain
// tags, publish the updated head's Consts and t as epoch-tagged words (the
// layout of EpisodeState::chain_pub: Consts' dwords, then t's two) straight
// from the LDS copy — not re-read from HBM after the head's stores, which
// would put a store drain and a load round trip in front of the publication.
// published: the head's Consts are the published words `pub` (the early
// publication's), not s_head's.
__device__ __forceinline__ void store_update(EpisodeHead* H, const uint64_t* s_head,
                                             mpc_episode_log_t* slot, const uint64_t* s_log,
                                             uint64_t* chain_pub, int chain_words,
                                             uint32_t epoch = 0, bool published = false,
                                             const uint32_t* pub = nullptr) {
  const int q = threadIdx.x;
  if (chain_pub && q < chain_words && !published) {
    if (epoch) {
      constexpr int kKWords = static_cast<int>(sizeof(Consts) / 4);
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(s_head);
      const uint32_t d =
          q < kKWords ? dw[q] : dw[offsetof(EpisodeHead, t) / 4 + (q - kKWords)];
      __hip_atomic_store(&chain_pub[q], (static_cast<uint64_t>(d) << 32) | epoch,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      chain_pub[q] = 0ull;
    }
  }
  constexpr int kKQ = static_cast<int>(sizeof(Consts) / 8);
  if (q < kStoredWords)   // head, then StaleTraj
    reinterpret_cast<uint64_t*>(H)[q] =
        (published && q < kKQ) ? reinterpret_cast<const uint64_t*>(pub)[q] : s_head[q];
  if (slot && q < kLogWords) reinterpret_cast<uint64_t*>(slot)[q] = s_log[q];
}

__device__ void episode_hook(const mpc_episode_config_t& c, const EpisodeHook& h,
                             const Winner& r, EpisodeHead& H, StaleTraj& st,
                             mpc_episode_log_t& L, mpc_episode_log_t*& slot,
                             const uint32_t* early = nullptr, bool* early_bad = nullptr);
__device__ inline void episode_early_prepare(const mpc_episode_config_t& c, const EpisodeHead& S,
                                             const StaleTraj& st, EarlyPub& E);

// Block-record reduction + winner re-roll (+ episode update), run by every
// thread of one block of NT threads.  SC1: the records were written by
// blocks of the SAME launch (fused path): they were stored `sc1` and are read
// `sc1` (L1 bypassed; the counter hand-off of rollout_episode).
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// Eight records, `sc1`, in ONE statement that also waits for them: an asm
// load's destination is written whenever the data arrives, so it must never
// leave the statement un-waited (hipcc may copy or reuse the register).
__device__ __forceinline__ void load8_rec_sc1(const Rec* const (&p)[8], u64x2 (&r)[8]) {
  asm volatile(
      "global_load_dwordx4 %0, %8, off sc1\n\t"
      "global_load_dwordx4 %1, %9, off sc1\n\t"
      "global_load_dwordx4 %2, %10, off sc1\n\t"
      "global_load_dwordx4 %3, %11, off sc1\n\t"
      "global_load_dwordx4 %4, %12, off sc1\n\t"
      "global_load_dwordx4 %5, %13, off sc1\n\t"
      "global_load_dwordx4 %6, %14, off sc1\n\t"
      "global_load_dwordx4 %7, %15, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
        "=&v"(r[6]), "=&v"(r[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}

// The same from a wave-uniform base (SGPR pair) and 32-bit byte offsets: one
// VGPR per address instead of two (block 0 of the chained exchange step polls
// its records with these, and its register peak is the kernel's).
__device__ __forceinline__ void load8_rec_sc1_sbase(const Rec* base, const uint32_t (&o)[8],
                                                    u64x2 (&r)[8]) {
  // (the base through readfirstlane: uniform for the compiler whatever loop
  // the call sits in, so the "s" operand is an SGPR pair)
  const uint64_t ab = reinterpret_cast<uint64_t>(base);
  base = reinterpret_cast<const Rec*>(
      (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
           static_cast<int>(ab >> 32)))) << 32) |
      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ab))));
  asm volatile(
      "s_nop 4\n\t"   // VALU-written SGPR -> VMEM: see glds_pair
      "global_load_dwordx4 %0, %8, %16 sc1\n\t"
      "global_load_dwordx4 %1, %9, %16 sc1\n\t"
      "global_load_dwordx4 %2, %10, %16 sc1\n\t"
      "global_load_dwordx4 %3, %11, %16 sc1\n\t"
      "global_load_dwordx4 %4, %12, %16 sc1\n\t"
      "global_load_dwordx4 %5, %13, %16 sc1\n\t"
      "global_load_dwordx4 %6, %14, %16 sc1\n\t"
      "global_load_dwordx4 %7, %15, %16 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
        "=&v"(r[6]), "=&v"(r[7])
      : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "v"(o[5]), "v"(o[6]), "v"(o[7]),
        "s"(base)
      : "memory");
}

// The end-of-step checks of a candidate next pose that episode_advance makes
// after the events (none in the early publication's steps): the
// run_math_model stuck break (:266-272) and the arrival (:542).
__device__ __forceinline__ bool early_pose_ok(const mpc_episode_config_t& c, const EpisodeHead& H,
                                              double x, double y) {
  if (c.stop_rule == 1 && x == H.x && y == H.y && H.recursive >= 1) return false;
  const double ex = H.x_t - x, ey = H.y_t - y;
  return !(ex * ex + ey * ey <= c.eps);
}

// GEN (generated controls, k_rollout_generated): v / b are [n_part][MPC_MAX_STEPS]
// — the controls of each rollout block's best candidate — instead of the
// [n_steps][n_cand] candidate arrays; the winner's are those of its block.
// Src: where the block records come from.  NoRecSrc: `part` / `n_part` as
// below; otherwise src(k, i) leaves in every thread the lexicographic minimum
// of its share of the records (the persistent run's selector, which polls the
// tagged records of the same launch: mpc_run.h).
struct NoRecSrc {};
template <int INTEG, int ROT, bool KDEV, int NT, bool SC1, bool GEN = false, bool TILED = false,
          class Src = NoRecSrc>
__device__ __forceinline__ void finalize_block(
    const Rec* __restrict__ part, int n_part, const Consts& K, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, int64_t index_base,
    double incumbent, mpc_result_t* __restrict__ out, const mpc_episode_config_t& ecfg,
    const EpisodeHook& hook, EmitLds* lds, const Src& src = Src{}) {
  // One-GPU episode: the episode scalars are staged in LDS by wave 1 (one
  // 8-B vector load per lane, issued after its record loads) and updated by
  // thread 0 once the winner is known.  (Loading them into thread 0's SGPRs
  // serialised three scalar round trips in front of wave 0's record loads.)
  static_assert(NT >= 128, "head staging by wave 1");
  static_assert(MPC_MAX_STEPS * 3 <= NT, "trajectory stored one value per lane");
  __shared__ uint64_t s_head[kStagedWords];
  __shared__ mpc_episode_log_t s_log;   // filled field by field by the update
  __shared__ mpc_episode_log_t* s_slot;
  __shared__ uint64_t s_key[NT / 64];
  __shared__ int64_t s_idx[NT / 64];
  // the early publication (chained step's block 0, below)
  constexpr int kKWords = static_cast<int>(sizeof(Consts) / 4);
  __shared__ __attribute__((aligned(8))) uint32_t s_pub[64];
  __shared__ double2 s_sc[3];
  __shared__ int s_early, s_pose, s_sc_ready;
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
  // wave 1's head words, loaded BEFORE its records so that both are in flight
  // together (the block barrier after the reduction waits for the staging)
  const bool stage = KDEV && hook.H && threadIdx.x >= 64 && threadIdx.x < 64 + kStagedWords;
  const uint64_t head_word =
      stage ? reinterpret_cast<const uint64_t*>(hook.H)[threadIdx.x - 64] : 0ull;
  if constexpr (!std::is_same_v<Src, NoRecSrc>) {
    src(k, i);
  } else if constexpr (SC1) {
    // n_part <= kMaxBlocks = 8 * NT: eight loads per thread, addresses of
    // out-of-range slots clamped to a valid record and their values ignored
    static_assert(kMaxBlocks <= 8 * NT, "load8_rec_sc1 covers 8 records per thread");
    const Rec* ptr[8];
    u64x2 r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int p = threadIdx.x + q * NT;
      ptr[q] = part + (p < n_part ? p : n_part - 1);
    }
    load8_rec_sc1(ptr, r);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (threadIdx.x + q * NT < n_part &&
          rec_less(r[q].x, static_cast<int64_t>(r[q].y), k, i)) {
        k = r[q].x;
        i = static_cast<int64_t>(r[q].y);
      }
  } else if (n_part <= NT) {
    // at most one record per thread (a small launch, config B's 196): no
    // compare chain over seven sentinel records on the selection's path
    if (static_cast<int>(threadIdx.x) < n_part) {
      const Rec r = part[threadIdx.x];
      k = r.key;
      i = r.idx;
    }
  } else {
    // all of this thread's records are loaded before any is compared, so
    // the loads overlap (one memory round trip)
    constexpr int kPer = (kMaxBlocks + NT - 1) / NT;
    Rec r[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int p = threadIdx.x + q * NT;
      r[q] = p < n_part ? part[p] : Rec{~0ull, INT64_MAX};
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q)
      if (rec_less(r[q].key, r[q].idx, k, i)) {
        k = r[q].key;
        i = r[q].idx;
      }
  }
  if (stage) s_head[threadIdx.x - 64] = head_word;
  // record indices are local candidate indices: below 2^31 for any row the
  // candidate arrays can hold in practice -> three 32-bit DPP minima
  if (!GEN && n_cand < (int64_t{1} << 31))
    wave_argmin32(k, i);
  else
    wave_argmin(k, i);
  // Each wave's best candidate's controls, loaded while the waves' minima are
  // combined: the block's winner is one of them, so its re-roll starts
  // without a dependent load of its own (one memory round trip fewer on the
  // selection's critical path; the same values, so the same arithmetic).
  double* s_pv = lds->pv;
  double* s_pb = lds->pb;
  double pv = 0.0, pb = 0.0;
  const int ln = threadIdx.x & 63;
  if constexpr (!GEN) {
    if (k != ~0ull && ln < n_steps) {
      const int64_t o = ctl_off<TILED>(ln, i, TILED ? n_steps : n_cand);
      pv = v[o];
      pb = b[o];
    }
  }
  if (ln == 0) {
    s_key[threadIdx.x >> 6] = k;
    s_idx[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  // every thread forms the block's winner (thread 0's result as before), so
  // the wave that holds it knows to stage its controls
  int wbest = 0;
  k = s_key[0];
  i = s_idx[0];
  for (int w = 1; w < NT / 64; ++w)
    if (rec_less(s_key[w], s_idx[w], k, i)) {
      k = s_key[w];
      i = s_idx[w];
      wbest = w;
    }
  if constexpr (!GEN) {
    if ((threadIdx.x >> 6) == wbest && ln < n_steps) {
      s_pv[ln] = pv;
      s_pb[ln] = pb;
    }
  }   // (emit_winner's first barrier orders these stores before its reads)
  Winner w;
  if constexpr (GEN) {
    // (thread 0 holds the winner; emit_winner takes its column from thread 0)
    // (k_rollout_generated: 2 candidates per lane, tiles dealt round-robin)
    const int64_t col = k == ~0ull ? 0 : ((i / (kBlock * 2)) % n_part) * MPC_MAX_STEPS;
    emit_winner<INTEG, ROT>(K, v, b, 1, n_steps, k, col, index_base + i, incumbent, out, lds, &w);
  } else {
    // A chained step's block 0: in the common step (no event, no end of the
    // episode) the next step's published words follow from the new pose
    // alone, so they go out before the rest of the update — the tile blocks
    // waiting for them do not also wait for the log record, the stale
    // trajectory, the event and restart logic and the head's stores.  What
    // does not need the winner was formed by the previous update (the head's
    // early_* fields); wave 3 lays out the words that carry over while wave 0
    // forms the per-step factors, and wave 1 evaluates sin / cos of the
    // winner's layer headings (the pass's own sums, in its order) during lane
    // 0's serial pass.
    const EpisodeHead& Hs = *reinterpret_cast<const EpisodeHead*>(s_head);
    const EarlyPub& Es = *reinterpret_cast<const EarlyPub*>(&s_head[kStoredWords]);
    const bool early_on = KDEV && hook.H && hook.publish_epoch;
    auto side_a = [&]() {
      const int q = threadIdx.x - 192;
      if (!early_on || q < 0 || q >= 64) return;
      constexpr int kH = static_cast<int>(offsetof(Consts, h) / 4);
      constexpr int kHl = static_cast<int>(offsetof(Consts, hlgth) / 4);
      static_assert(kHl == kH + 2, "h, hlgth adjacent");
      const uint32_t* kw = reinterpret_cast<const uint32_t*>(s_head);   // Hs.K's dwords
      const uint32_t* ew = reinterpret_cast<const uint32_t*>(&Es.t);   // t, h, hl
      if (q < kKWords)
        s_pub[q] = (q >= kH && q < kH + 4) ? ew[2 + (q - kH)] : kw[q];
      else if (q < kKWords + 2)
        s_pub[q] = ew[q - kKWords];
    };
    // The pick: the winner's layer jj = min(k, N-1) as lane 0 forms it in the
    // serial pass (on_layer: the end-of-step checks, the pose into s_pub,
    // s_pose = 1 publish / 2 not), or the no-winner pose (decided by wave 3
    // alone); wave 3 then adds sin / cos and publishes — while lane 0 goes on
    // with the remaining layers.
    const bool can_early =
        early_on && Es.step == Hs.step && Es.k >= 0;   // (uniform: LDS words, all threads)
    const bool valid_w = k != ~0ull;
    const bool found_w = valid_w && key_cost(k) < incumbent;   // emit_winner's `found`
    const int jj_w = can_early ? (Es.k < n_steps - 1 ? Es.k : n_steps - 1) : -1;
    if (threadIdx.x == 0) {   // (LDS starts undefined; read only after emit_winner's barriers)
      s_pose = 0;
      s_sc_ready = 0;
    }
    auto on_layer = [&](int st, double x, double y, double ph) {
      if (!can_early || !found_w || st != jj_w) return;
      const bool ok = early_pose_ok(ecfg, Hs, x, y);
      if (ok) {
        Consts& Kp = *reinterpret_cast<Consts*>(s_pub);
        Kp.x = x;
        Kp.y = y;
        Kp.phi = ph;
      }
      __hip_atomic_store(&s_pose, ok ? 1 : 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto side_b = [&](bool fast) {
      const int q = threadIdx.x;
      if (early_on && q >= 64 && q < 64 + 3) {
        const int last = n_steps - 1, jj = q - 64 < last ? q - 64 : last;
        double ph;
        if (fast) {   // emit_winner's fast pass: K.phi + dphi_0 + ... in step order
          ph = K.phi;
          for (int st = 0; st <= jj; ++st) ph = ph + lds->dphi[st];
        } else {
          ph = lds->phi[jj];
        }
        // sincos_fast's own core (the same bits) on its range; beyond it (a
        // heading of more than 2^19 pi / 2, never in practice) no early
        // publication — the large reduction's code would cost the kernel
        // scratch memory
        double sn = 0.0, cs = 0.0;
        const bool in = fabs(ph) <= trig::kFastMax;
        if (in) trig::sincos_core(ph, &sn, &cs);
        s_sc[q - 64] = make_double2(sn, cs);
        const bool all_in = __ballot(!in) == 0;
        if (q == 64)   // (the wave's three LDS stores are in order before it)
          __hip_atomic_store(&s_sc_ready, all_in ? 1 : 2, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (early_on && q >= 192 && q < 256) {   // wave 3: the pick's last part, the publication
        if (q == 192) {
          int pub = 0;
          if (can_early) {
            Consts& Kp = *reinterpret_cast<Consts*>(s_pub);
            if (!found_w) {   // the no-winner pose: the stale layer k, or the pose
              if (Es.alt && fabs(Es.ph) <= trig::kFastMax) {
                double sn, cs;
                trig::sincos_core(Es.ph, &sn, &cs);   // (= sincos_fast on its range)
                Kp.x = Es.x;
                Kp.y = Es.y;
                Kp.phi = Es.ph;
                Kp.s0 = sn;
                Kp.c0 = cs;
                pub = 1;
              }
            } else {
              // lane 0's pose and wave 1's sin / cos (bounded waits: an
              // unanswered one only forgoes the early publication)
              int pose = 0, sc = 0;
              for (uint32_t it = 0; it < (1u << 22) && (pose == 0 || sc == 0); ++it) {
                pose = __hip_atomic_load(&s_pose, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                sc = __hip_atomic_load(&s_sc_ready, __ATOMIC_ACQUIRE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                if (pose == 2 || sc == 2) break;
                if (pose == 0 || sc == 0) __builtin_amdgcn_s_sleep(1);
              }
              if (pose == 1 && sc == 1) {
                Kp.s0 = s_sc[jj_w].x;
                Kp.c0 = s_sc[jj_w].y;
                pub = 1;
              }
            }
          }
          s_early = pub;
        }
        // thread 192's LDS stores, then wave 3's reads (one wave)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int w3 = q - 192;
        if (s_early && w3 < hook.chain_pub_words)
          __hip_atomic_store(&hook.chain_pub[w3],
                             (static_cast<uint64_t>(s_pub[w3]) << 32) | hook.publish_epoch,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    emit_winner<INTEG, ROT>(K, v, b, n_cand, n_steps, k, i, index_base + i, incumbent, out, lds,
                            &w, s_pv, s_pb, KDEV && hook.H, side_a, side_b, on_layer);
  }
  if (KDEV && hook.H) {
    const bool early = hook.publish_epoch && s_early;   // (uniform)
    if (threadIdx.x == 0) {
      // on the LDS copy itself: the update touches a few of its words, and a
      // copy into registers and back costs more than it saves; after an early
      // publication the constants are left as published
      bool bad = false;
      episode_hook(ecfg, hook, w, *reinterpret_cast<EpisodeHead*>(s_head),
                   *reinterpret_cast<StaleTraj*>(&s_head[kHeadWords]), s_log, s_slot,
                   early ? s_pub : nullptr, &bad);
      if (bad && hook.chain_error) *hook.chain_error = 6u;
    }
    __syncthreads();
    if (hook.publish_epoch && threadIdx.x == 64) {
      // the next step's early-publication inputs, beside the head's stores
      // (an EarlyPub follows the stale trajectory in the state)
      EarlyPub E;
      episode_early_prepare(ecfg, *reinterpret_cast<const EpisodeHead*>(s_head),
                            *reinterpret_cast<const StaleTraj*>(&s_head[kHeadWords]), E);
      *reinterpret_cast<EarlyPub*>(reinterpret_cast<uint64_t*>(hook.H) + kStoredWords) = E;
    }
    // the head and the log record back to HBM, the chain tags cleared (or the
    // next step's constants published, unless they already are)
    store_update(hook.H, s_head, s_slot, reinterpret_cast<const uint64_t*>(&s_log),
                 hook.chain_pub, hook.chain_pub_words, hook.publish_epoch, early, s_pub);
    // the record's remaining trajectory, off the update's critical path
    emit_winner_tail<INTEG, ROT>(K, n_steps, lds, out);
  }
}

// The selection of a generated-controls step (GEN finalize_block).
template <int INTEG, int ROT>
__global__ __launch_bounds__(kFinBlock) void k_finalize_gen(
    const Rec* __restrict__ part, int n_part, const Consts* __restrict__ Kdev,
    const double* __restrict__ part_v, const double* __restrict__ part_b, int n_steps,
    int64_t index_base, const double* __restrict__ incumbent_dev,
    mpc_result_t* __restrict__ out, mpc_episode_config_t ecfg, EpisodeHook hook) {
  const Consts K = *Kdev;
  __shared__ EmitLds lds;
  finalize_block<INTEG, ROT, true, kFinBlock, false, true>(part, n_part, K, part_v, part_b, 0,
                                                           n_steps, index_base, *incumbent_dev,
                                                           out, ecfg, hook, &lds);
}

template <int INTEG, int ROT, bool KDEV, bool TILED = false>
__global__ __launch_bounds__(kFinBlock) void k_finalize(
    const Rec* __restrict__ part, int n_part, Consts Karg, const Consts* __restrict__ Kdev,
    const double* __restrict__ v, const double* __restrict__ b, int64_t n_cand, int n_steps,
    int64_t index_base, double incumbent_arg, const double* __restrict__ incumbent_dev,
    mpc_result_t* __restrict__ out, mpc_episode_config_t ecfg, EpisodeHook hook) {
  const Consts K = KDEV ? *Kdev : Karg;
  const double incumbent = KDEV ? *incumbent_dev : incumbent_arg;
  __shared__ EmitLds lds;
  finalize_block<INTEG, ROT, KDEV, kFinBlock, false, false, TILED>(
      part, n_part, K, v, b, n_cand, n_steps, index_base, incumbent, out, ecfg, hook, &lds);
}

// Device-resident episode, one launch per MPC step: the streaming rollout +
// block arg-min of k_rollout_argmin, then the LAST block to finish runs the
// finalize (record reduction, winner re-roll, and on one GPU the episode
// update).  Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): each
// block's thread 0 stores its record `sc1`, waits for it (vmcnt(0)), then adds
// to the launch counter (agent-scope atomic); the block whose add returns
// gridDim-1 is last, and its threads read every record `sc1` after a
// workgroup barrier.  The last block re-arms the counter for the next launch.
template <int CPL, int INTEG, int ROT>
__global__ __launch_bounds__(kBlock, 1) void k_rollout_episode(
    const Consts* __restrict__ Kdev, const double* __restrict__ v, const double* __restrict__ b,
    int64_t n_cand, int n_steps, int64_t index_base, Rec* __restrict__ part,
    uint32_t* __restrict__ done, const double* __restrict__ incumbent_dev,
    mpc_result_t* __restrict__ out, mpc_episode_config_t ecfg, EpisodeHook hook) {
  const Consts K = *Kdev;
  const int64_t n_tiles = (n_cand + kBlock * CPL - 1) / (kBlock * CPL);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t c0 = tile * (kBlock * CPL) + threadIdx.x * CPL;
    if (c0 < n_cand) {
      double cst[CPL];
      rollout_lane<CPL, INTEG, ROT, false>(K, v, b, n_cand, c0, n_steps, cst, nullptr, n_cand);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const uint64_t kk = cost_key_nonneg(cst[j]);
        if (kk < best_k) {
          best_k = kk;
          best_i = c0 + j;
        }
      }
    }
  }
  block_argmin(best_k, best_i);
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    Rec* dst = part + blockIdx.x;
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)"
                 :
                 : "v"(dst),
                   "v"(u64x2{best_k, static_cast<uint64_t>(best_i)})
                 : "memory");
    const uint32_t prev =
        __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // (the block's control ring is drained: its LDS holds the re-roll)
  finalize_block<INTEG, ROT, true, kBlock, true>(part, gridDim.x, K, v, b, n_cand, n_steps,
                                                 index_base, *incumbent_dev, out, ecfg, hook,
                                                 ring_lds());
  if (threadIdx.x == 0) *done = 0u;
}

// Problem constants derived on the device (batched robots, episode).  The
// squares are x*x (glibc pow(x, 2.0) differs by 1 ulp in ~0.1% of inputs);
// the single-problem host path derives them with libm pow.
__device__ __forceinline__ Consts consts_from_problem(const mpc_problem_t& p) {
  Consts K;
  K.x = p.x;
  K.y = p.y;
  K.phi = p.phi;
  K.x_t = p.x_t;
  K.y_t = p.y_t;
  K.x_0 = p.x_0;
  K.y_0 = p.y_0;
  K.A = p.y_t - p.y_0;
  K.B = p.x_t - p.x_0;
  K.C1 = p.x_t * p.y_0;
  K.C2 = p.y_t * p.x_0;
  K.inv_den = 1.0 / sqrt(K.A * K.A + K.B * K.B);
  K.L = p.L;
  int e;
  const double m = frexp(p.L, &e);
  K.L_pow2 = (m == 0.5) ? 1 : 0;
  K.inv_L = K.L_pow2 ? 1.0 / p.L : 0.0;
  K.h = p.t_b - p.t_a;
  K.hlgth = 0.5 * (p.t_b - p.t_a);
  trig::sincos_fast(p.phi, &K.s0, &K.c0);
  K.pad_ = 0;
  return K;
}

// --------------------------- batched robots --------------------------------
// The wide variant runs the streaming kernel's lane (LDS-DMA ring): the same
// 5 waves per SIMD (4 at the default bound: 120 VGPRs).
template <int CPL, int INTEG, int ROT>
__global__ __launch_bounds__(kBlock, CPL == kCplWide ? kStreamWaves : 1) void
k_rollout_argmin_batched(
    const mpc_problem_t* __restrict__ probs, const double* __restrict__ v,
    const double* __restrict__ b, int64_t cand, int n_steps, int64_t ld, Rec* __restrict__ part) {
  const int r = blockIdx.y;
  const Consts K = uniform_consts(consts_from_problem(probs[r]));
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  const int64_t tiles = (cand + kBlock * CPL - 1) / (kBlock * CPL);
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t cl = tile * (kBlock * CPL) + threadIdx.x * CPL;  // local index
    if (cl < cand) {
      double cst[CPL];
      rollout_lane<CPL, INTEG, ROT, false>(K, v, b, ld, r * cand + cl, n_steps, cst, nullptr, 0);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const uint64_t kk = cost_key_nonneg(cst[j]);
        if (kk < best_k) {
          best_k = kk;
          best_i = cl + j;
        }
      }
    }
  }
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0)
    part[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] = Rec{best_k, best_i};
}

template <int INTEG, int ROT>
__global__ __launch_bounds__(kBlock) void k_finalize_batched(
    const Rec* __restrict__ part, int n_part, const mpc_problem_t* __restrict__ probs,
    const double* __restrict__ incumbents, const double* __restrict__ v,
    const double* __restrict__ b, int64_t cand, int n_steps, int64_t ld,
    mpc_result_t* __restrict__ out) {
  const int r = blockIdx.x;
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
  for (int p = threadIdx.x; p < n_part; p += kBlock) {
    const Rec q = part[static_cast<int64_t>(r) * n_part + p];
    if (rec_less(q.key, q.idx, k, i)) {
      k = q.key;
      i = q.idx;
    }
  }
  block_argmin(k, i);
  const Consts K = consts_from_problem(probs[r]);
  const double inc = incumbents ? incumbents[r] : __builtin_inf();
  __shared__ EmitLds lds;
  emit_winner<INTEG, ROT>(K, v, b, ld, n_steps, k, r * cand + i, i, inc, &out[r], &lds);
}

// --------------------------- exchange ----------------------------------------
// Lexicographic (cost, global index) min over n gathered per-rank results.
__device__ int select_index(const mpc_result_t* __restrict__ res, int n, uint64_t& bk) {
  int best = 0;
  int64_t bi = INT64_MAX;
  bk = ~0ull;
  for (int r = 0; r < n; ++r) {
    const uint64_t k = res[r].index < 0 ? ~0ull : cost_key(res[r].cost);
    const int64_t i = res[r].index < 0 ? INT64_MAX : res[r].index;
    if (r == 0 || rec_less(k, i, bk, bi)) {
      best = r;
      bk = k;
      bi = i;
    }
  }
  return best;
}

__global__ void k_select_winner(const mpc_result_t* __restrict__ res, int n, double incumbent,
                                mpc_result_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t bk;
  const int best = select_index(res, n, bk);
  *out = res[best];
  out->found = (bk != ~0ull && out->cost < incumbent) ? 1 : 0;
}

// --------------------------- sampler -----------------------------------------
// Grid entry of one (step, candidate): candidate g < n_grid of the constant
// prefix is the reference's enumeration k = g; otherwise the top 32 bits of
// splitmix64(seed ^ s<<40 ^ g) are mapped onto [0, n_grid) by multiply-shift
// (Lemire's fastrange: no integer division on the VALU).
__device__ __forceinline__ uint32_t grid_entry(uint64_t seed, int s, uint64_t g, uint32_t n_grid,
                                               int cprefix) {
  if (cprefix && g < n_grid) return static_cast<uint32_t>(g);
  const uint64_t h = splitmix64(seed ^ (static_cast<uint64_t>(s) << 40) ^ g);
  return static_cast<uint32_t>(((h >> 32) * static_cast<uint64_t>(n_grid)) >> 32);
}

constexpr int kSampleLdsEntries = 2048;  // expanded (v, beta) grid staged in LDS

// One thread per candidate pair (16-B stores), looping over the steps.  The
// grid |V| x |B| (<= 451 entries for the reference's acceleration limits) is
// expanded once per block into LDS, so the per-element lookup is one
// ds_read_b128 instead of a division by |B| and two loads.
// cprefix 2 (the episode's enumeration mode): candidates past the grid are
// padding — NaN controls, a NaN cost, never chosen.
// tiled: v / b are the MPC_LAYOUT_TILED buffer's base and base + 512, ld its
// n_steps (ctl_off).
__device__ void sample_items(const double2* s_grid, uint32_t n_grid, int64_t n_cand, int n_steps,
                             uint64_t seed, int64_t base, int cprefix, double* __restrict__ v,
                             double* __restrict__ b, int64_t ld, int pairs, int tiled = 0) {
  const int cpt = pairs ? 2 : 1;
  const int64_t n_items = n_cand / cpt;
  for (int64_t it = blockIdx.x * static_cast<int64_t>(kBlock) + threadIdx.x; it < n_items;
       it += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t c = it * cpt;
    const uint64_t g = static_cast<uint64_t>(base + c);
    const double2 pad = make_double2(__builtin_nan(""), 0.0);
    for (int st = 0; st < n_steps; ++st) {
      const double2 e0 =
          (cprefix == 2 && g >= n_grid) ? pad : s_grid[grid_entry(seed, st, g, n_grid, cprefix)];
      if (pairs) {
        const double2 e1 = (cprefix == 2 && g + 1 >= n_grid)
                               ? pad
                               : s_grid[grid_entry(seed, st, g + 1, n_grid, cprefix)];
        const int64_t o = tiled ? ctl_off<true>(st, c, ld) : ctl_off<false>(st, c, ld);
        *reinterpret_cast<double2*>(v + o) = make_double2(e0.x, e1.x);
        *reinterpret_cast<double2*>(b + o) = make_double2(e0.y, e1.y);
      } else {   // one candidate per item: the same layout choice as the pairs
        const int64_t o = tiled ? ctl_off<true>(st, c, ld) : ctl_off<false>(st, c, ld);
        v[o] = e0.x;
        b[o] = e0.y;
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_sample_controls(
    const double* __restrict__ vg, int nv, const double* __restrict__ bg, int nb, int64_t n_cand,
    int n_steps, uint64_t seed, int64_t base, int cprefix, double* __restrict__ v,
    double* __restrict__ b, int64_t ld, int pairs, int tiled) {
  __shared__ double2 s_grid[kSampleLdsEntries];
  const uint32_t n_grid = static_cast<uint32_t>(nv) * static_cast<uint32_t>(nb);
  if (n_grid > kSampleLdsEntries) {
    // large grids: direct lookups (one division per element)
    const int cpt = pairs ? 2 : 1;
    for (int64_t it = blockIdx.x * static_cast<int64_t>(kBlock) + threadIdx.x; it < n_cand / cpt;
         it += static_cast<int64_t>(gridDim.x) * kBlock) {
      const int64_t c = it * cpt;
      for (int st = 0; st < n_steps; ++st)
        for (int j = 0; j < cpt; ++j) {
          const uint32_t k = grid_entry(seed, st, base + c + j, n_grid, cprefix);
          const int64_t o = tiled ? ctl_off<true>(st, c + j, ld) : ctl_off<false>(st, c + j, ld);
          v[o] = vg[k / nb];
          b[o] = bg[k % nb];
        }
    }
    return;
  }
  for (uint32_t k = threadIdx.x; k < n_grid; k += kBlock)
    s_grid[k] = make_double2(vg[k / nb], bg[k % nb]);
  __syncthreads();
  sample_items(s_grid, n_grid, n_cand, n_steps, seed, base, cprefix, v, b, ld, pairs, tiled);
}

}  // namespace mpc
