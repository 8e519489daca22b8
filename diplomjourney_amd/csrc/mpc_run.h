// mpc_run.h — persistent episode run: K MPC steps of the device-resident
// episode (math_model_tree.py:515-635, heading mode kRotCum) in ONE launch.
//
// Why: a step launched as its own kernel(s) pays, every step, the launch's
// fill and drain (first control loads in flight with nothing to compute, the
// last tiles finishing on a part-idle chip) and the one-block selection
// during which HBM idles.  In kRotCum mode a candidate's rollout needs no
// start pose (mpc_device.h step_start / cum_pose), so step j+1's candidates
// can stream while step j is still being selected; only the final pose
// transform and the criterion wait for the pose.  One launch streams the K
// steps' tiles back to back:
//
//   unit u = (step j, tile) = (u / T, u % T), T = tiles of 512 candidates per
//   step.  Blocks register in start order; the first one selects
//   (run_select_step, one step after the other), the others stream units
//   s, s + G, s + 2G, ... (streaming block s of G registered ones: every
//   block that owns units is running, whatever residency the occupancy API
//   promised).  A streaming block's 4 waves are independent (run_stream_wave):
//   - each wave streams its quarter (128 candidates) of the block's units with
//     an LDS-DMA control ring that runs ACROSS units (a unit's last steps
//     already issue the next unit's first rows), the step size h speculated
//     from the last head the wave knows (+ dt per step, as episode_prepare
//     forms it);
//   - at a unit's end it keeps the quarter's position sums in registers (up
//     to kRunPend quarters) and goes on; it polls the oldest one's head with
//     an LDS-DMA that lands behind its counted waits, then scores the quarter
//     (the final pose transform and criterion; a mis-speculated h — an
//     episode restart reset t — or an irregular candidate is re-rolled at the
//     unit's end) and counts it in LDS; the wave whose count completes the
//     unit writes its tagged record;
//   - the selector sweeps step j's T records, re-rolls the winner
//     (emit_winner), applies the episode update (episode_advance: finishing
//     logic, operator events, restart, log record, the next step's t and
//     constants) and publishes step j+1's head.
//
// Hand-offs (MI355X_MICROARCH.md "inter-workgroup visibility",
// cdna_hip_programming.md Guideline 16 R2): every handed-off word is an 8-byte
// {data32 << 32 | tag32} granule written by ONE relaxed agent-scope atomic
// store (sc1) and read by relaxed agent-scope loads (sc1); the tag is the
// step index within the call + 1, so a granule validates itself and no fence
// is needed.  The polled words (registration, abort word, head and record
// granules) are zeroed by a memset node before every launch
// (mpc_episode_run), so a tag from an earlier call (or graph replay) never
// matches.  Inside a block the waves meet only in LDS.  Every wait is bounded:
// on a timeout the waiter sets the abort word (every other wait then gives up
// at once) and chain error 3.
#pragma once

#include "mpc_episode.h"

namespace mpc {

constexpr int kHeadDwords = kHeadWords * 2;                       // 70
constexpr int kRunTDword = static_cast<int>(offsetof(EpisodeHead, t) / 4);   // 58
static_assert(kHeadDwords <= 2 * 64, "head granules: two waves");
static_assert(kConstsWords <= 64 && kRunTDword + 1 < 64, "loop words: one wave");
#ifdef MPC_RUN_STATS
// Debug builds only (tools/build_variant.sh NAME -DMPC_RUN_STATS): counters
// and 100-MHz tick sums of the run's phases, read by mpc_debug_run_stats.
__device__ unsigned long long g_run_stats[32];
#define RUN_STAT(i, v) atomicAdd(&g_run_stats[i], static_cast<unsigned long long>(v))
#define RUN_TICK() __builtin_amdgcn_s_memrealtime()
#define RUN_ACC(i, v) (st_acc[i] += static_cast<uint64_t>(v))
// per-unit timestamps (units < 1 << 20), by lane 0 of wave 0 of the
// streaming block: 0 stream start, 1 stream end, 2 kept (after a full-hand
// wait), 3 record written (by the completing wave), 7 the block (plain stores)
__device__ unsigned long long g_run_ut[1 << 20][8];
#define RUN_UT(u, f) \
  do { if ((u) < (1 << 20)) g_run_ut[(u)][(f)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define RUN_UTV(u, f, v) \
  do { if ((u) < (1 << 20)) g_run_ut[(u)][(f)] = (v); } while (0)
// per-step timeline (steps < 512): 0 first unit stream start (min), 1 last
// stream end (max), 2 last unit completion (max), 3 sweep done, 4 published
__device__ unsigned long long g_run_tl[512][5];
#define RUN_TL_MIN(j, f) \
  do { if ((j) < 512) atomicMin(&g_run_tl[(j)][(f)], __builtin_amdgcn_s_memrealtime()); } while (0)
#define RUN_TL_MAX(j, f) \
  do { if ((j) < 512) atomicMax(&g_run_tl[(j)][(f)], __builtin_amdgcn_s_memrealtime()); } while (0)
#else
#define RUN_TL_MIN(j, f) ((void)0)
#define RUN_TL_MAX(j, f) ((void)0)
#define RUN_UT(u, f) ((void)0)
#define RUN_UTV(u, f, v) ((void)0)
#define RUN_STAT(i, v) ((void)0)
#define RUN_TICK() 0ull
#define RUN_ACC(i, v) ((void)0)
#endif

constexpr int kRunRecWords = 4;       // granules per unit record: key hi, key lo, index, pad
constexpr uint32_t kRunSpinLimit = 1u << 18;   // x s_sleep(16) ~1 us: ~0.25 s

// The published head, in kRunPubCopies copies 4 KiB apart (block b polls copy
// b % kRunPubCopies) for A/B: 1, 16 and 64 copies ran at the same speed (the
// ~3000 polling waves do not make the head's lines a hot spot that matters).
#ifndef MPC_RUN_PUB_COPIES
#define MPC_RUN_PUB_COPIES 1
#endif
constexpr int kRunPubCopies = MPC_RUN_PUB_COPIES;
struct RunPubCopy {
  uint64_t pub[2][kHeadDwords];   // head of step j in pub[j & 1], tag j + 1
  uint8_t pad_[4096 - 2 * kHeadDwords * 8];
};
// The polled block at the start of the run workspace (zeroed every call).
struct RunCtl {
  uint32_t abort;        // a bounded wait timed out: every wait gives up
  uint32_t unused_;
  uint32_t role;         // blocks registered (in start order): the first one selects
  uint32_t nres;         // registered blocks when the selector closed the registration
  uint32_t pad_[1020];
  RunPubCopy copy[kRunPubCopies];
};
static_assert(sizeof(RunCtl) % 16 == 0, "memset block: multiple of 16 B");

__device__ __forceinline__ void granule_store(uint64_t* g, uint32_t tag, uint32_t val) {
  __hip_atomic_store(g, (static_cast<uint64_t>(val) << 32) | tag, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t granule_load(const uint64_t* g) {
  return __hip_atomic_load(const_cast<uint64_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool run_aborted(const RunCtl* rc) {
  return __hip_atomic_load(const_cast<uint32_t*>(&rc->abort), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// A wait ran out (or another one did): make every other wait give up.
// `where` (debug builds) says which wait: chain error 3 + 16 * where.
__device__ __forceinline__ void run_fail(RunCtl* rc, EpisodeState* S, uint32_t where = 0) {
  const bool first = __hip_atomic_exchange(&rc->abort, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) == 0u;
#ifdef MPC_RUN_STATS
  if (first) S->chain_error = 3u + 16u * where;
#else
  (void)where;
  if (first) S->chain_error = 3u;
#endif
}

// Loop-word lanes of wave 0: the Consts dwords and t (dwords kRunTDword, +1).
__device__ __forceinline__ bool run_loop_word(int q) {
  return q < kConstsWords || q == kRunTDword || q == kRunTDword + 1;
}

// One wave: the loop words of the head in `g` (granules, tag `tag`) into s_w if
// every one carries the tag.  Returns (wave-uniform) whether they did.
__device__ __forceinline__ bool run_read_words(const uint64_t* g, uint32_t tag, uint32_t* s_w) {
  const int q = threadIdx.x & 63;
  const uint64_t w = run_loop_word(q) ? granule_load(g + q) : 0ull;
  const bool ok = !run_loop_word(q) || static_cast<uint32_t>(w) == tag;
  const bool all = __ballot(!ok) == 0;
  if (all && run_loop_word(q)) s_w[q] = static_cast<uint32_t>(w >> 32);
  return all;
}

// The t of the loop words (s_w dwords kRunTDword, +1).
__device__ __forceinline__ double run_words_t(const uint32_t* s_w) {
  const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(s_w[kRunTDword]));
  const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(s_w[kRunTDword + 1]));
  return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
}

// Consts from head granules (data in the high 32 bits), field by field.
__device__ __forceinline__ Consts consts_from_granules(const uint64_t* g) {
  auto d = [&](size_t off) {
    const int q = static_cast<int>(off / 4);
    const uint64_t lo = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g[q] >> 32)));
    const uint64_t hi = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g[q + 1] >> 32)));
    return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
  };
  Consts K;
  K.x = d(offsetof(Consts, x));
  K.y = d(offsetof(Consts, y));
  K.phi = d(offsetof(Consts, phi));
  K.x_t = d(offsetof(Consts, x_t));
  K.y_t = d(offsetof(Consts, y_t));
  K.x_0 = d(offsetof(Consts, x_0));
  K.y_0 = d(offsetof(Consts, y_0));
  K.A = d(offsetof(Consts, A));
  K.B = d(offsetof(Consts, B));
  K.C1 = d(offsetof(Consts, C1));
  K.C2 = d(offsetof(Consts, C2));
  K.den = d(offsetof(Consts, den));
  K.L = d(offsetof(Consts, L));
  K.inv_L = d(offsetof(Consts, inv_L));
  K.h = d(offsetof(Consts, h));
  K.hlgth = d(offsetof(Consts, hlgth));
  K.s0 = d(offsetof(Consts, s0));
  K.c0 = d(offsetof(Consts, c0));
  K.L_pow2 = static_cast<int32_t>(__builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(g[offsetof(Consts, L_pow2) / 4] >> 32)));
  K.pad_ = 0;
  return K;
}

// Step j's T unit records (kRunRecWords granules each, tag j + 1) -> the
// lexicographic (cost key, local index) minimum, per thread (the caller
// reduces over the block).  Every thread sweeps its records kSw at a time, all
// loads of a sweep in flight together, until each carries the tag (bounded).
constexpr int kSw = 4;
// All of the selector's kWaves waves agree (the block's fifth wave has ended:
// an OCKL work-group reduction such as __syncthreads_and would count it).
__device__ __forceinline__ bool selector_all(bool p) {
  __shared__ int s_all[kWaves];
  const bool w = __ballot(!p) == 0;
  if ((threadIdx.x & 63) == 0) s_all[threadIdx.x >> 6] = w;
  __syncthreads();
  bool r = true;
#pragma unroll
  for (int q = 0; q < kWaves; ++q) r = r && s_all[q] != 0;
  __syncthreads();   // s_all reuse
  return r;
}
__device__ __forceinline__ void run_sweep_records(const uint64_t* rec, int64_t T, uint32_t tag,
                                                  RunCtl* rc, EpisodeState* S, uint64_t& k,
                                                  int64_t& i) {
  k = ~0ull;
  i = INT64_MAX;
  for (int64_t base = 0; base < T; base += kSw * kBlock) {
    uint64_t hi[kSw], lo[kSw], ix[kSw];
    bool need[kSw];
#pragma unroll
    for (int q = 0; q < kSw; ++q) need[q] = base + threadIdx.x + q * kBlock < T;
    for (uint32_t spins = 0;; ++spins) {
#pragma unroll
      for (int q = 0; q < kSw; ++q) {
        if (need[q]) {
          const uint64_t* r = rec + (base + threadIdx.x + q * kBlock) * kRunRecWords;
          hi[q] = granule_load(r);
          lo[q] = granule_load(r + 1);
          ix[q] = granule_load(r + 2);
        }
      }
      bool all = true;
#pragma unroll
      for (int q = 0; q < kSw; ++q) {
        if (need[q]) {
          if (static_cast<uint32_t>(hi[q]) == tag && static_cast<uint32_t>(lo[q]) == tag &&
              static_cast<uint32_t>(ix[q]) == tag) {
            const uint64_t kk = (hi[q] & 0xffffffff00000000ull) | (lo[q] >> 32);
            const int64_t ii = static_cast<int64_t>(ix[q] >> 32);
            if (rec_less(kk, ii, k, i)) {
              k = kk;
              i = ii;
            }
            need[q] = false;
          } else {
            all = false;
          }
        }
      }
      if (threadIdx.x == 0) RUN_STAT(11, 1);
      if (selector_all(all)) break;
      if (spins >= kRunSpinLimit || run_aborted(rc)) {
        if (threadIdx.x == 0) run_fail(rc, S, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
}


// Block 0 of the run: completes the K steps one after the other.  Step j:
// sweep its T unit records (tag j + 1), re-roll the winner, episode update,
// publish step j+1's head.  The head lives in LDS (s_head) from step to step.
// One step per (non-inlined) call: with the step body inlined into the loop
// over j, the re-roll's and the update's constants were hoisted out of it and
// the kernel spilled (128 VGPRs + scratch); a call keeps them per step.
__shared__ uint32_t g_run_head[kHeadDwords];
__shared__ mpc_episode_config_t g_run_cfg;

template <int INTEG>
__device__ __noinline__ void run_select_step(
    int j, EpisodeState* __restrict__ S, const double* __restrict__ v,
    const double* __restrict__ b, int k_steps, int64_t n_cand, int n_steps, int64_t index_base,
    RunCtl* __restrict__ rc, const uint64_t* __restrict__ rec, int64_t T,
    mpc_result_t* __restrict__ res, mpc_episode_log_t* __restrict__ log, int cap,
    uint64_t* __restrict__ clock) {
  __shared__ mpc_episode_log_t s_log;
  __shared__ mpc_episode_log_t* s_slot;
  uint32_t* s_head = g_run_head;
  const int q = threadIdx.x;
  const uint32_t tag = static_cast<uint32_t>(j + 1);
  const bool last = j + 1 == k_steps;
  uint64_t k;
  int64_t i;
  const uint64_t t0 = RUN_TICK();
  run_sweep_records(rec + (j & 1) * T * kRunRecWords, T, tag, rc, S, k, i);
  block_argmin(k, i);   // (its barrier also orders the head's LDS words)
  const uint64_t t1 = RUN_TICK();
  if (q == 0) RUN_TL_MAX(j, 3);
  Winner w;
  {
    const Consts Kj = consts_from_words(s_head);
    double inc;
    __builtin_memcpy(&inc, &s_head[offsetof(EpisodeHead, incumbent) / 4], sizeof(double));
    emit_winner<INTEG, kRotCum>(Kj, v, b, n_cand, n_steps, k, i, index_base + i, inc, res, &w);
  }
  const uint64_t t2 = RUN_TICK();
  if (q == 0) {   // emit_winner ended with a barrier
    EpisodeHead H;
    __builtin_memcpy(&H, s_head, sizeof(EpisodeHead));
    s_slot = log_slot(log, cap, H.step);
    episode_advance(g_run_cfg, H, w, s_log);
    __builtin_memcpy(s_head, &H, sizeof(EpisodeHead));
  }
  __syncthreads();
  // step j+1's head: the streaming blocks' final constants
  if (!last)
    for (int i = q; i < kRunPubCopies * kHeadDwords; i += kBlock)
      granule_store(rc->copy[i / kHeadDwords].pub[(j + 1) & 1] + i % kHeadDwords, tag + 1u,
                    s_head[i % kHeadDwords]);
  if (clock && q == 0) clock[j] = __builtin_amdgcn_s_memrealtime();
  if (q == 0) RUN_TL_MAX(j, 4);
  if (q == 0) {
    const uint64_t t3 = RUN_TICK();
    RUN_STAT(8, t1 - t0);
    RUN_STAT(9, t2 - t1);
    RUN_STAT(10, t3 - t2);
  }
  // the log record; after the last step the head itself (read after the launch)
  if (s_slot && q < kLogWords)
    reinterpret_cast<uint64_t*>(s_slot)[q] = reinterpret_cast<const uint64_t*>(&s_log)[q];
  if (last && q < kHeadWords)
    reinterpret_cast<uint64_t*>(&S->h)[q] = reinterpret_cast<const uint64_t*>(s_head)[q];
  __syncthreads();   // s_log / s_slot reuse
}

// Per streaming block: the quarter minima of its units (unit k in slot
// k % kRunSlots) and each wave's head-poll buffer.  LDS only; the four
// streaming waves order their accesses with lgkmcnt waits (LDS operations of
// a wave complete in order) and relaxed LDS atomics.  A wave keeps its own
// unscored quarters (position sums) in registers: no parking in LDS, which
// left room for 4 blocks a CU.
#ifndef MPC_RUN_SLOTS
#define MPC_RUN_SLOTS 4
#endif
constexpr int kRunSlots = MPC_RUN_SLOTS;   // minima slots per block (unit k in slot k % kRunSlots)
static_assert(kRunSlots >= 1 && kRunSlots <= 8, "MPC_RUN_SLOTS must be in [1, 8]");
// The run's own control ring (kRunRing - 1 steps in flight per wave).  (4
// slots: 54272 B of LDS a block, and only 2 blocks per CU became resident.)
#ifndef MPC_RUN_RING
#define MPC_RUN_RING 4
#endif
constexpr int kRunRing = MPC_RUN_RING;
static_assert(kRunRing >= 2 && kRunRing <= 4, "MPC_RUN_RING must be in [2, 4]");
__shared__ double2 g_run_ring[kWaves][kRunRing][2][64];  // [wave][slot][v|beta][lane]
struct RunLds {
  uint64_t qkey[kRunSlots][kWaves]; // each wave's quarter minimum
  int64_t qidx[kRunSlots][kWaves];
  int32_t cnt[kRunSlots];           // quarters of the slot's unit scored
  int32_t seq[kRunSlots];           // unit index (per block) the slot accepts next
  uint64_t poll[kWaves][64];        // each wave's head poll (LDS-DMA target)
};

__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// 16 bytes (two granules) of a published head into this lane's 16 bytes of
// the LDS buffer at dst (lanes 0-31: 64 granules), bypassing the non-coherent
// cache levels (sc1, as an agent-scope relaxed load).  Counted by vmcnt like
// the control rows; the caller orders earlier LDS reads of the buffer first.
__device__ __forceinline__ void glds_poll(const uint64_t* g, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off sc1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(dst)
      : "memory");
}

__device__ __forceinline__ int32_t lds_load(const int32_t* p) {
  return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One wave: the unit's four quarter minima (LDS) -> unit u's record (step j,
// tag j + 1); then the slot is free for the block's unit k + kRunSlots.
__device__ __forceinline__ void run_combine(RunLds& sh, uint64_t* __restrict__ rec, int64_t T,
                                            int sl, int32_t k, int64_t u, int64_t j) {
  const int lane = threadIdx.x & 63;
  uint64_t bk = ~0ull;
  int64_t bi = INT64_MAX;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    const uint64_t k2 = sh.qkey[sl][w];
    const int64_t i2 = sh.qidx[sl][w];
    if (rec_less(k2, i2, bk, bi)) {
      bk = k2;
      bi = i2;
    }
  }
  if (lane == 0) {
    const uint32_t tag = static_cast<uint32_t>(j + 1);
    uint64_t* r = rec + ((j & 1) * T + (u - j * T)) * kRunRecWords;
    granule_store(r, tag, static_cast<uint32_t>(bk >> 32));
    granule_store(r + 1, tag, static_cast<uint32_t>(bk));
    granule_store(r + 2, tag, static_cast<uint32_t>(bi));   // < 2^31 (host check)
    RUN_UT(u, 3);
    lds_store(&sh.cnt[sl], 0);
    lds_order();
    lds_store(&sh.seq[sl], k + kRunSlots);
  }
}

// The rare path of scoring a parked candidate (out of line: it must not cost
// the streaming loop registers): a mis-speculated step size (an episode
// restart reset t) re-rolls the candidate from its controls with the head's
// h; an irregular candidate re-runs the safe recurrence; otherwise the
// parked sums give the pose.  `head`: the step's head granules (LDS).
template <int INTEG, bool PL2>
__device__ __noinline__ uint64_t run_rescore(const uint64_t* head, double hq, const double* cv,
                                             const double* cb, int64_t n_cand, int n_steps,
                                             int64_t col, double a, double b, bool irregular) {
  const Consts K = consts_from_granules(head);
  double cst;
  if (hq != K.h) {
    cst = rollout_candidate_l<INTEG, kRotCum, PL2>(K, cv, cb, n_cand, col, n_steps, nullptr);
  } else if (irregular) {
    double xx = K.x, yy = K.y, ph = K.phi;
    for (int sr = 0; sr < n_steps; ++sr)
      step_safe<INTEG>(xx, yy, ph, cv[sr * n_cand + col], cb[sr * n_cand + col], K);
    cst = cost(xx, yy, K);
  } else {
    double xx, yy;
    cum_pose(K, a, b, xx, yy);
    cst = cost(xx, yy, K);
  }
  return cost_key(cst);
}

// A wave's unscored quarter: its lanes' position sums and irregular flags,
// the h its loop used, the block's unit index and the step.
struct RunPend {
  double2 a, b;   // (A0, A1), (B0, B1)
  uint32_t bad;   // bit c: candidate c irregular
  double h;
  int32_t k;
  int64_t j;
};
#ifndef MPC_RUN_PEND
#define MPC_RUN_PEND 2
#endif
constexpr int kRunPend = MPC_RUN_PEND;   // unscored quarters a wave holds (registers)
static_assert(kRunPend >= 1 && kRunPend <= 4, "MPC_RUN_PEND must be in [1, 4]");

// Streaming wave (waves 0-3 of a streaming block): rolls out its quarter (128
// candidates: lane l of wave w holds candidates tile*512 + (64w + l)*2 + {0,1})
// of each of the block's units (s, s + G, s + 2G, ... for streaming block s of
// G), keeps the sums in registers and goes on.  The control ring (kRing slots of one step's
// v and beta rows, kRing-1 steps in flight) continues across units.  The
// wave learns a parked quarter's head by polling it with an LDS-DMA into its
// own buffer (it lands behind the counted waits two steps later), scores the
// quarter and counts it; the wave whose count completes the unit combines the
// four minima into the unit's record and frees the slot.  The only blocking
// waits: its own control rows; at a unit's end, when the wave already holds
// kRunPend unscored quarters, the oldest one's head; and a minima slot still
// holding the unit kRunSlots before (another wave that far behind).
template <int INTEG, bool PL2>
__device__ __forceinline__ void run_stream_wave(RunLds& sh, const double* const* __restrict__ ctl,
                                                int64_t total, int64_t T, int64_t s, int64_t G,
                                                int64_t n_cand, int n_steps,
                                                RunCtl* __restrict__ rc,
                                                uint64_t* __restrict__ rec,
                                                EpisodeState* __restrict__ S, const Consts& Kc,
                                                double delta_t) {
  constexpr int CPL = 2;
  constexpr int R = kRunRing;
  constexpr uint32_t kSlot = 2 * 64 * sizeof(double2);   // 2 KiB: v and beta rows
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_addr(&g_run_ring[wv][0][0][0]));
  auto dst = [&](uint32_t slot) { return ring0 + slot * kSlot; };
  auto unit_of = [&](int32_t k) -> int64_t {   // the block's k-th unit
    const int64_t u = s + static_cast<int64_t>(k) * G;
    return u < total ? u : total;
  };
  auto lane_col = [&](int64_t tile) {
    const int64_t c0 = tile * (kBlock * CPL) + threadIdx.x * CPL;
    return c0 < n_cand ? c0 : n_cand - CPL;   // lanes past a partial tile repeat the last pair
  };
  int64_t u = unit_of(0);
  if (u >= total) return;
  // issue cursor: the block's ik-th unit iu = (step ij, tile itile), control row ist
  int32_t ik = 0;
  int64_t iu = u, ij = u / T, itile = u - (u / T) * T;
  int ist = 0;
  const double* iv = ctl[2 * ij];
  const double* ib = ctl[2 * ij + 1];
  int64_t icl = lane_col(itile);
  uint32_t gi = 0, gc = 0;              // control rows issued / consumed (ring slot = count % R)
  auto issue = [&](bool dep, const double2& rv, const double2& rb) -> bool {
    if (iu >= total) return false;
    const uint32_t sl = gi % R;
    if (dep)
      glds_refill(iv + ist * n_cand + icl, ib + ist * n_cand + icl, dst(sl), dst(sl) + kSlot / 2,
                  rv, rb);
    else
      glds_pair(iv + ist * n_cand + icl, ib + ist * n_cand + icl, dst(sl), dst(sl) + kSlot / 2);
    ++gi;
    if (++ist == n_steps) {
      ist = 0;
      iu = unit_of(++ik);
      if (iu < total) {
        ij = iu / T;
        itile = iu - ij * T;
        iv = ctl[2 * ij];
        ib = ctl[2 * ij + 1];
        icl = lane_col(itile);
      }
    }
    return true;
  };
  {
    const double2 z = make_double2(0.0, 0.0);
#pragma unroll
    for (int q = 0; q < R - 1; ++q) issue(false, z, z);
  }
  double2 rv = make_double2(0.0, 0.0), rb = rv;   // the slot read last (refill dependency)
  trig::Leads lead = trig::const_leads();
  Consts Kl = Kc;                        // wheelbase terms; h per unit
#ifdef MPC_RUN_STATS
  uint64_t st_acc[16] = {0};
#endif
  // This wave's unscored quarters, oldest first (e0, then e1).
  const uint32_t pollw = __builtin_amdgcn_readfirstlane(lds_addr(&sh.poll[wv][0]));
  const RunPubCopy& pubc = rc->copy[s % kRunPubCopies];
  int pend_n = 0;
  RunPend e0{}, e1{}, e2{}, e3{};   // (entries past kRunPend are never used)
  int64_t khj = 0;                       // latest step whose head this wave took (poll buffer)
  double kt = S->h.t;                    // that head's t (the speculation's base)
  int poll_age = 0;                      // 0: none in flight; else steps waited since issue
  int64_t poll_j = 0;
  {
    // the call's first head, as if polled (tag 1 = step 0)
    const int q = lane;
    const uint32_t w = run_loop_word(q) ? reinterpret_cast<const uint32_t*>(&S->h)[q] : 0u;
    sh.poll[wv][q] = (static_cast<uint64_t>(w) << 32) | 1u;
  }
  auto head_t = [&]() {
    const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(sh.poll[wv][kRunTDword] >> 32)));
    const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(sh.poll[wv][kRunTDword + 1] >> 32)));
    return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
  };
  // score the oldest pending quarter with the head in the poll buffer (step
  // e0.j).  Inside the streaming loop (slow = false) only the regular case:
  // the rescoring call there cost the loop its registers (5x slower steps);
  // it returns false and the quarter waits for the unit's end.
  auto resolve_oldest = [&](bool slow) -> bool {
    const int sl = e0.k % kRunSlots;
    const int64_t u0 = unit_of(e0.k);
    const int64_t pj0 = e0.j;
    const double ph0 = e0.h;
    const double tj = head_t();
    const bool hok = ((tj + delta_t) - tj) == ph0;
    const uint32_t bb = e0.bad;
    const double2 px = e0.a, py = e0.b;
    const int64_t c0 = (u0 - pj0 * T) * (kBlock * CPL) + threadIdx.x * CPL;
    uint64_t k0, k1;
    const bool regular = hok && __ballot(bb != 0u) == 0;
    if (!slow && !regular) return false;
    if (regular) {
      const Consts K = consts_from_granules(sh.poll[wv]);
      double xx, yy;
      cum_pose(K, px.x, py.x, xx, yy);
      k0 = cost_key(cost(xx, yy, K));
      cum_pose(K, px.y, py.y, xx, yy);
      k1 = cost_key(cost(xx, yy, K));
    } else {
      RUN_ACC(1, 1);
      const int64_t cl = c0 < n_cand ? c0 : n_cand - CPL;
      const double* cv = ctl[2 * pj0];
      const double* cb = ctl[2 * pj0 + 1];
      k0 = run_rescore<INTEG, PL2>(sh.poll[wv], ph0, cv, cb, n_cand, n_steps, cl, px.x, py.x,
                                   (bb & 1u) != 0u);
      k1 = run_rescore<INTEG, PL2>(sh.poll[wv], ph0, cv, cb, n_cand, n_steps, cl + 1, px.y, py.y,
                                   (bb & 2u) != 0u);
    }
    uint64_t dk = ~0ull;
    int64_t di = INT64_MAX;
    if (c0 < n_cand) {
      dk = k0;
      di = c0;
    }
    if (c0 + 1 < n_cand && k1 < dk) {
      dk = k1;
      di = c0 + 1;
    }
    wave_argmin(dk, di);
    // the slot still holds unit k - kRunSlots if another wave is that far behind
    for (uint32_t it = 0; lds_load(&sh.seq[sl]) != e0.k; ++it) {
      RUN_ACC(4, 1);
      if ((it & 1023) == 1023 && run_aborted(rc)) break;
      if (it >= kRunSpinLimit * 8u) {
        if (lane == 0) run_fail(rc, S, 4);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
      sh.qkey[sl][wv] = dk;
      sh.qidx[sl][wv] = di;
    }
    lds_order();   // the minimum is in LDS before the count says so
    int32_t prev = 0;
    if (lane == 0)
      prev = __hip_atomic_fetch_add(&sh.cnt[sl], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev == kWaves - 1) {
      lds_order();
      run_combine(sh, rec, T, sl, e0.k, u0, pj0);
    }
    --pend_n;
    e0 = e1;   // shift (static registers; entries past pend_n are don't-care)
    if constexpr (kRunPend > 2) e1 = e2;
    if constexpr (kRunPend > 3) e2 = e3;
    return true;
  };
  // after a poll has landed: take it if every loop word carries the tag
  auto take_poll = [&]() {
    const int q = lane;
    const uint64_t w = sh.poll[wv][q];
    const bool ok =
        !run_loop_word(q) || static_cast<uint32_t>(w) == static_cast<uint32_t>(poll_j + 1);
    if (__ballot(!ok) == 0) {
      khj = poll_j;
      kt = head_t();
    }
    poll_age = 0;
    while (pend_n > 0 && khj == e0.j && resolve_oldest(false)) {
    }
  };
  // blocking: the head of the oldest pending quarter (relaxed polls)
  auto wait_oldest = [&]() {
    const uint64_t* g = pubc.pub[e0.j & 1];
    const uint32_t tag = static_cast<uint32_t>(e0.j + 1);
    const uint64_t w0 = RUN_TICK();
    for (uint32_t it = 0;; ++it) {
      const uint64_t w = run_loop_word(lane) ? granule_load(g + lane) : 0ull;
      const bool ok = !run_loop_word(lane) || static_cast<uint32_t>(w) == tag;
      if (__ballot(!ok) == 0) {
        sh.poll[wv][lane] = w;
        break;
      }
      if (it >= kRunSpinLimit || run_aborted(rc)) {
        if (lane == 0) run_fail(rc, S, 2);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    lds_order();
    khj = e0.j;
    kt = head_t();
    poll_age = 0;
    RUN_ACC(5, 1);
    RUN_ACC(6, RUN_TICK() - w0);
    while (pend_n > 0 && khj == e0.j) resolve_oldest(true);
  };
  for (int32_t k = 0; u < total; ++k, u = unit_of(k)) {
    const int64_t j = u / T;
    // step size: from this wave's latest head, + dt per step since
    {
      double t = kt;
      for (int64_t q = khj; q < j; ++q) t = t + delta_t;
      Kl.h = (t + delta_t) - t;          // consts_from_problem: t_b - t_a
    }
    double x[CPL], y[CPL], sn[CPL], cs[CPL];
    bool bad[CPL];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      double ph;
      step_start<kRotCum>(Kl, x[q], y[q], ph, sn[q], cs[q]);
      bad[q] = false;
    }
    if (lane == 0 && wv == 0) {
      RUN_UT(u, 0);
      RUN_UTV(u, 7, blockIdx.x);
    }
#pragma unroll 1
    for (int st = 0; st < n_steps; ++st) {
      issue(true, rv, rb);
      const uint32_t ahead = gi - gc - 1;   // row pairs issued behind this one
      static_assert(R <= 4, "tail waits below cover up to 3 pairs behind");
      if (ahead >= R - 1)
        wait_vm<2 * (R - 1)>();
      else if (ahead == 2)
        wait_vm<4>();
      else if (ahead == 1)
        wait_vm<2>();
      else
        wait_vm<0>();
      const uint32_t sl = gc % R;
      rv = g_run_ring[wv][sl][0][lane];
      rb = g_run_ring[wv][sl][1][lane];
      ++gc;
      // (the heading itself is not carried: kRotCum rotates (sn, cs))
      double h0 = 0.0, h1 = 0.0;
      step_core<INTEG, kRotCum, PL2>(x[0], y[0], h0, sn[0], cs[0], rv.x, rb.x, Kl, bad[0], &lead);
      step_core<INTEG, kRotCum, PL2>(x[1], y[1], h1, sn[1], cs[1], rv.y, rb.y, Kl, bad[1], &lead);
      // the head poll of the oldest pending quarter: issued here, landed R-1
      // counted waits later (R-1 more row pairs issued behind it), then taken
      if (poll_age > 0 && ++poll_age >= R) take_poll();
      if (pend_n > 0 && poll_age == 0) {
        poll_j = e0.j;
        lds_order();   // this wave's reads of the previous poll are done
        if (lane < 32) glds_poll(pubc.pub[e0.j & 1] + 2 * lane, pollw);
        poll_age = 1;
      }
    }
    if (lane == 0 && wv == 0) RUN_UT(u, 1);
    // a full hand: the oldest quarter's head first
    if (pend_n == kRunPend) {
      if (poll_age > 0) wait_vm<0>();    // (an in-flight poll must land first)
      poll_age = 0;
      wait_oldest();
    }
    if (lane == 0 && wv == 0) RUN_UT(u, 2);
    {
      RunPend e;
      e.a = make_double2(x[0], x[1]);
      e.b = make_double2(y[0], y[1]);
      e.bad = (bad[0] ? 1u : 0u) | (bad[1] ? 2u : 0u);
      e.h = Kl.h;
      e.k = k;
      e.j = j;
      if (pend_n == 0)
        e0 = e;
      else if (kRunPend == 2 || pend_n == 1)
        e1 = e;
      else if (kRunPend == 3 || pend_n == 2)
        e2 = e;
      else
        e3 = e;
      ++pend_n;
    }
    // this wave already holds the head of its oldest pending step: score now
    while (pend_n > 0 && khj == e0.j) resolve_oldest(true);
  }
  if (poll_age > 0) wait_vm<0>();
  while (pend_n > 0) wait_oldest();   // the wave's last quarters
#ifdef MPC_RUN_STATS
  if (lane == 0)
    for (int q = 0; q < 16; ++q)
      if (st_acc[q]) RUN_STAT(q, st_acc[q]);
#endif
}

// Block-wise streaming (MPC_RUN_BLOCKWISE): a streaming block rolls out one
// unit after the other with the chained step's tile path (rollout_lane_glds_k,
// 96 VGPRs: 5 waves/SIMD) — h speculated from the last head the block knows,
// the unit's head polled three steps before its loop ends and waited for at
// its end (the loop reruns with the final constants if h was wrong), then
// the block's arg-min is the unit's record.  No quarters are held back: a
// block waits at a unit's end until that step's head is out.
template <int INTEG, bool PL2>
__device__ __forceinline__ void run_stream_block(const double* const* __restrict__ ctl,
                                                 int64_t total, int64_t T, int64_t s, int64_t G,
                                                 int64_t n_cand, int n_steps,
                                                 RunCtl* __restrict__ rc,
                                                 uint64_t* __restrict__ rec,
                                                 EpisodeState* __restrict__ S, double delta_t) {
  constexpr int CPL = 2;
  __shared__ uint32_t s_w[64];   // loop words of the head of step jk
  const int q = threadIdx.x;
  if (q < 64 && run_loop_word(q)) s_w[q] = reinterpret_cast<const uint32_t*>(&S->h)[q];
  __syncthreads();
  Consts K = consts_from_words(s_w);   // the head of step jk (the call's first: S->h)
  double tk = run_words_t(s_w);
  int64_t jk = 0;
  const RunPubCopy& pubc = rc->copy[s % kRunPubCopies];
  for (int64_t u = s; u < total; u += G) {
    const int64_t j = u / T;
    const int64_t tile = u - j * T;
    const double* v = ctl[2 * j];
    const double* b = ctl[2 * j + 1];
    const int64_t c0 = tile * (kBlock * CPL) + q * CPL;
    const int64_t cl = c0 < n_cand ? c0 : n_cand - CPL;
    const bool have = jk == j;
    Consts Kl, Kf;
    uint64_t w_pre = 0;
    bool pre_issued = false;
    auto pre0 = [&]() {
      Kl = K;
      if (have) return;
      double t = tk;   // + dt per step since, as episode_prepare forms it
      for (int64_t r = jk; r < j; ++r) t = t + delta_t;
      Kl.h = (t + delta_t) - t;
    };
    auto mid = [&]() {
      if (have || pre_issued) return;
      pre_issued = true;
      if (q < 64 && run_loop_word(q)) w_pre = granule_load(pubc.pub[j & 1] + q);
    };
    auto wait = [&]() {
      if (q == 0) RUN_UT(u, 1);
      if (!have) {
        __syncthreads();   // s_w reuse
        if (q < 64) {
          const uint32_t tag = static_cast<uint32_t>(j + 1);
          bool fin = false;
          if (pre_issued) {
            const bool ok = !run_loop_word(q) || static_cast<uint32_t>(w_pre) == tag;
            fin = __ballot(!ok) == 0;
            if (fin && run_loop_word(q)) s_w[q] = static_cast<uint32_t>(w_pre >> 32);
          }
          for (uint32_t it = 0; !fin; ++it) {
            fin = run_read_words(pubc.pub[j & 1], tag, s_w);
            if (fin) break;
            if (it >= kRunSpinLimit || run_aborted(rc)) {
              if (q == 0) run_fail(rc, S, 2);
              break;
            }
            __builtin_amdgcn_s_sleep(4);
          }
        }
        __syncthreads();
        K = consts_from_words(s_w);
        tk = run_words_t(s_w);
        jk = j;
      }
      if (q == 0) RUN_UT(u, 2);
      Kf = K;
    };
    if (q == 0) RUN_UT(u, 0);
    double cst[CPL];
    rollout_lane_glds_k<INTEG, kRotCum, PL2, decltype(wait), decltype(pre0), decltype(mid),
                        false>(Kf, Kl, v, b, n_cand, cl, n_steps, cst, wait, pre0, mid);
    uint64_t bk = ~0ull;
    int64_t bi = INT64_MAX;
    if (c0 < n_cand) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const uint64_t kk = cost_key(cst[c]);
        if (kk < bk) {
          bk = kk;
          bi = c0 + c;
        }
      }
    }
    block_argmin(bk, bi);
    if (q == 0) {
      const uint32_t tag = static_cast<uint32_t>(j + 1);
      uint64_t* r = rec + ((j & 1) * T + tile) * kRunRecWords;
      granule_store(r, tag, static_cast<uint32_t>(bk >> 32));
      granule_store(r + 1, tag, static_cast<uint32_t>(bk));
      granule_store(r + 2, tag, static_cast<uint32_t>(bi));   // < 2^31 (host check)
      RUN_UTV(u, 7, blockIdx.x);
      RUN_UT(u, 3);
    }
  }
}

constexpr int kRunThreads = kBlock;   // 4 waves: the selector's, or a streaming block's
// Launch bound: waves per SIMD (4 blocks of 4 waves per CU).  It must not ask
// for more than LDS allows: that makes the bound void for the out-of-line
// callees (run_rescore then took 180 VGPRs, 2 blocks per CU).
#ifndef MPC_RUN_BLOCKWISE
#define MPC_RUN_BLOCKWISE 1   // 0: run_stream_wave (wave-wise quarters kept in registers, 3 waves/SIMD)
#endif
#ifndef MPC_RUN_WAVES
#if MPC_RUN_BLOCKWISE
#define MPC_RUN_WAVES 5
#else
#define MPC_RUN_WAVES 3
#endif
#endif
constexpr uint32_t kRunRegisterTicks = 1000;   // s_memrealtime (100 MHz): 10 us without a new block

// ctl: device array [k_steps][2] of the steps' control SoA pointers (v, beta).
// rec: [2][T][kRunRecWords] record granules (step j in half j & 1).
// out: step k_steps-1's winner; every other step's re-roll goes to scratch.
// clock: optional [k_steps] s_memrealtime (100 MHz) when step j was completed.
//
// Roles: blocks register in start order (rc->role).  The first one selects;
// it closes the registration when every block of the grid is in, or when no
// block has come in for 10 us (at least one other in), and publishes the count
// N (rc->nres).  Blocks 1 .. N-1 stream units s, s + G, ... (s = role - 1,
// G = N - 1): every block with a unit is running, whatever the residency the
// occupancy API promised.  A block that registers later has no unit.
template <int INTEG, bool PL2>
__global__ __launch_bounds__(kRunThreads, MPC_RUN_WAVES) void k_episode_run(
    EpisodeState* __restrict__ S, const double* const* __restrict__ ctl, int k_steps,
    int64_t n_cand, int n_steps, int64_t index_base, RunCtl* __restrict__ rc,
    uint64_t* __restrict__ rec, mpc_result_t* __restrict__ out,
    mpc_result_t* __restrict__ scratch, mpc_episode_config_t ecfg,
    mpc_episode_log_t* __restrict__ log, int cap, uint64_t* __restrict__ clock) {
  constexpr int CPL = 2;
  const int64_t T = (n_cand + kBlock * CPL - 1) / (kBlock * CPL);
  const int64_t total = T * k_steps;
#if !MPC_RUN_BLOCKWISE
  __shared__ RunLds sh;
#endif
  __shared__ uint32_t s_role, s_nres;
  if (threadIdx.x == 0) {
    const uint32_t r =
        __hip_atomic_fetch_add(&rc->role, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t n = 0;
    if (r == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t tc = t0;   // when the count last grew
      uint32_t last = 0;
      for (;;) {
        n = __hip_atomic_load(&rc->role, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (n != last) {
          last = n;
          tc = now;
        }
        if (n >= gridDim.x || (n >= 2 && now - tc > kRunRegisterTicks) ||
            now - t0 > 1000 * kRunRegisterTicks)
          break;
        __builtin_amdgcn_s_sleep(8);
      }
      __hip_atomic_store(&rc->nres, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n < 2) run_fail(rc, S, 6);   // no streaming block in 20 ms
    } else {
      for (uint32_t it = 0;; ++it) {
        n = __hip_atomic_load(&rc->nres, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n != 0u || run_aborted(rc)) break;
        if (it >= kRunSpinLimit) {
          run_fail(rc, S, 7);
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    s_role = r;
    s_nres = n;
  }
#if !MPC_RUN_BLOCKWISE
  if (threadIdx.x < kRunSlots) {
    sh.cnt[threadIdx.x] = 0;
    sh.seq[threadIdx.x] = threadIdx.x;
  }
#endif
  __syncthreads();
  const uint32_t role = s_role, nres = s_nres;
  if (role == 0u) {
    if (nres < 2u) return;
    // The host picked PL2 from cfg; a state reset with another wheelbase form
    // would be rolled out with the wrong dphi form: flag it (as the chain does).
    if (threadIdx.x == 0 && (S->h.K.L_pow2 != 0) != PL2) S->chain_error = 2u;
    if (threadIdx.x == 0) g_run_cfg = ecfg;
    if (threadIdx.x == 0) RUN_STAT(31, nres);
    if (threadIdx.x < kHeadDwords)
      g_run_head[threadIdx.x] = reinterpret_cast<const uint32_t*>(&S->h)[threadIdx.x];
    __syncthreads();
    for (int j = 0; j < k_steps; ++j)
      run_select_step<INTEG>(j, S, ctl[2 * j], ctl[2 * j + 1], k_steps, n_cand, n_steps,
                             index_base, rc, rec, T, j + 1 == k_steps ? out : scratch, log, cap,
                             clock);
    return;
  }
  if (role >= nres) return;   // registered after the count was taken: no units
#if MPC_RUN_BLOCKWISE
  run_stream_block<INTEG, PL2>(ctl, total, T, static_cast<int64_t>(role) - 1,
                               static_cast<int64_t>(nres) - 1, n_cand, n_steps, rc, rec, S,
                               ecfg.delta_t);
#else
  const Consts Kc = S->h.K;   // wheelbase terms (h set per unit)
  run_stream_wave<INTEG, PL2>(sh, ctl, total, T, static_cast<int64_t>(role) - 1,
                              static_cast<int64_t>(nres) - 1, n_cand, n_steps, rc, rec, S, Kc,
                              ecfg.delta_t);
#endif
}

// Resident blocks of one run instantiation (occupancy x CUs), per device.
template <int I, bool P>
int64_t run_grid(int64_t total_units) {
  static int64_t cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cache[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&k_episode_run<I, P>), kRunThreads, 0) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
#ifdef MPC_RUN_PER_CU
    per_cu = MPC_RUN_PER_CU;   // A/B builds only
#endif
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    cache[dev] = static_cast<int64_t>(per_cu) * cus;
  }
  // one block selects; at least one streams
  return std::max<int64_t>(2, std::min(total_units + 1, cache[dev]));
}

}  // namespace mpc
