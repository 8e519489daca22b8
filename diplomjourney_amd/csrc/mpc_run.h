// mpc_run.h — persistent episode run: K MPC steps of the device-resident
// episode (math_model_tree.py:515-635, heading mode kRotCum) in ONE launch.
//
// Why: a step launched as its own kernel(s) pays, every step, the launch's
// fill and drain (first control loads in flight with nothing to compute, the
// last tiles finishing on a part-idle chip).  In kRotCum mode a candidate's
// rollout needs no start pose (mpc_device.h step_start / cum_pose), so step
// j+1's candidates can stream while step j is still being selected; only the
// final pose transform and the criterion wait for the pose.  One launch
// streams the K steps' tiles back to back:
//
//   unit u = (step j, tile) = (u / T, u % T), T = tiles of 512 candidates per
//   step.  Blocks register in start order; the first one selects
//   (run_select_step, one step after the other), the others stream units
//   s, s + G, s + 2G, ... (streaming block s of G registered ones: every
//   block that owns units is running, whatever residency the occupancy API
//   promised).  A streaming block (run_stream_block) rolls out one unit at a
//   time with the chained step's tile path (rollout_lane_glds_k, 5
//   waves/SIMD), the step size h speculated from the last head it knows (+ dt
//   per step, as episode_prepare forms it); it polls the unit's head three
//   steps before the loop ends, waits for it at the end (the loop reruns with
//   the final constants if h was wrong), and its arg-min is the unit's tagged
//   record.  The selector sweeps step j's T records, re-rolls the winner
//   (emit_winner), applies the episode update (episode_advance: finishing
//   logic, operator events, restart, log record, the next step's t and
//   constants) and publishes step j+1's head.
//   (Measured: level with the chained steps of mpc_episode_chain_step at 8e6
//   candidates per step, slower at 1e6 — DESIGN.md §6d.)
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
  [[maybe_unused]] const uint64_t t0 = RUN_TICK();
  run_sweep_records(rec + (j & 1) * T * kRunRecWords, T, tag, rc, S, k, i);
  block_argmin(k, i);   // (its barrier also orders the head's LDS words)
  [[maybe_unused]] const uint64_t t1 = RUN_TICK();
  if (q == 0) RUN_TL_MAX(j, 3);
  Winner w;
  {
    const Consts Kj = consts_from_words(s_head);
    double inc;
    __builtin_memcpy(&inc, &s_head[offsetof(EpisodeHead, incumbent) / 4], sizeof(double));
    emit_winner<INTEG, kRotCum>(Kj, v, b, n_cand, n_steps, k, i, index_base + i, inc, res, &w);
  }
  [[maybe_unused]] const uint64_t t2 = RUN_TICK();
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
    [[maybe_unused]] const uint64_t t3 = RUN_TICK();
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

// Block-wise streaming: a streaming block rolls out one
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
// Launch bound: waves per SIMD (5: the tile path's 96 VGPRs).  It must not ask
// for more than LDS allows (that makes the bound void for the out-of-line
// selector call).
#ifndef MPC_RUN_WAVES
#define MPC_RUN_WAVES 5
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
  run_stream_block<INTEG, PL2>(ctl, total, T, static_cast<int64_t>(role) - 1,
                               static_cast<int64_t>(nres) - 1, n_cand, n_steps, rc, rec, S,
                               ecfg.delta_t);
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
